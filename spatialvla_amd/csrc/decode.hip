// KV-cached decode attention for Gemma2 greedy generation on gfx950.
//
// Reference semantics: the HybridCache decode of SpatialVLAForConditionalGeneration.generate
// (model/modeling_spatialvla.py:440-492): each new token attends to the cached keys of the prompt
// (bidirectional prefix, :294) and to every earlier generated token, through eager_attention_forward
// (model/modeling_gemma2.py:169-195): S = QK^T*scale, S = cap*tanh(S/cap), additive mask, softmax in fp32,
// P -> bf16, O = PV.  Numerics follow svla_attn_fwd (fp32 scores, unnormalised P rounded to bf16 for the PV
// product, one division by the fp32 row sum at the end), so a cached step reproduces the full re-forward.
//
// Shape of the work: Lq (usually 1) new queries per sequence against Lk cached keys — a GEMV over the
// K/V cache, HBM-bound (Lk * Hkv * D * 2 * 2 bytes per sequence), far from MFMA territory.  One workgroup
// per (kv head, query, sequence): the Hq/Hkv query heads of a GQA group share every K/V row read.
//  * scores: wave w takes keys w, w+4, ...; a lane holds D/64 contiguous elements of the key row (8-byte
//    coalesced loads for D = 256) and the dot products finish with one butterfly per query head;
//  * softmax: scores live in LDS ([group][Lk] fp32), block-wide max / sum;
//  * PV: thread t owns output column d = t and walks the keys (a V row is one 512-byte coalesced read).
#include "svla_common.h"

namespace {

constexpr float MASKVAL = -3.3895313892515355e38f;  // torch.finfo(bfloat16).min, as the reference mask
constexpr float LOG2E = 1.4426950408889634f;
constexpr int NT = 256;
constexpr int MAXG = 4;

__device__ __forceinline__ bool visible(int c, int kj, int qi, int window) {
  bool v = (c == 0) || (c == 1 && kj <= qi);
  if (window > 0 && qi - kj >= window) v = false;
  return v;
}

template <int E, int G>
__global__ __launch_bounds__(NT) void attn_decode_kernel(svla_attn_decode_args a, bf16_t* __restrict__ out,
                                                         int64_t ldo) {
  extern __shared__ float sc[];  // [G][Lk] scores, then bf16-rounded probabilities
  __shared__ float red[2 * NT / 64 * G];
  const int hk = blockIdx.x, t = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int Lk = a.Lk, D = a.D;
  const int qi = Lk - a.Lq + t;  // absolute (0-based) position of this query
  const bf16_t* qrow = (const bf16_t*)a.q + ((int64_t)b * a.Lq + t) * a.ldq + (int64_t)hk * G * D;
  const bf16_t* kb = (const bf16_t*)a.k + (int64_t)b * a.bsk + (int64_t)hk * D;
  const bf16_t* vb = (const bf16_t*)a.v + (int64_t)b * a.bsv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * a.ldc : nullptr;

  float qf[G][E];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < E; ++e) qf[g][e] = bf2f(qrow[g * D + lane * E + e]);

  // scores
  for (int j = w; j < Lk; j += NT / 64) {
    const bf16_t* kr = kb + (int64_t)j * a.ldk + lane * E;
    float kf[E];
#pragma unroll
    for (int e = 0; e < E; ++e) kf[e] = bf2f(kr[e]);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < E; ++e) s = fmaf(qf[g][e], kf[e], s);
      s = wave_sum(s);
      if (lane == 0) {
        float v = s * a.scale;
        if (a.softcap > 0.f) v = a.softcap * fast_tanh(v / a.softcap);
        if (!visible(cls ? cls[j] : 0, j, qi, a.sliding_window)) v = MASKVAL;
        sc[g * Lk + j] = v;
      }
    }
  }
  __syncthreads();

  // softmax statistics per query head (block-wide)
  float mx[G], inv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = -INFINITY;
    for (int j = tid; j < Lk; j += NT) m = fmaxf(m, sc[g * Lk + j]);
    m = wave_max(m);
    if (lane == 0) red[g * (NT / 64) + w] = m;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = red[g * (NT / 64)];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red[g * (NT / 64) + i]);
    mx[g] = m;
    float l = 0.f;
    for (int j = tid; j < Lk; j += NT) {
      const float p = exp2f((sc[g * Lk + j] - m) * LOG2E);
      l += p;
      sc[g * Lk + j] = round_bf(p);  // P enters the PV product as bf16 (the MFMA operand of svla_attn_fwd)
    }
    l = wave_sum(l);
    if (lane == 0) red[(NT / 64) * G + g * (NT / 64) + w] = l;
  }
  __syncthreads();
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) l += red[(NT / 64) * G + g * (NT / 64) + i];
    inv[g] = 1.0f / l;
  }

  // O = P V, thread tid owns column d = tid
  if (tid < D) {
    float acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = 0.f;
    const bf16_t* vc = vb + tid;
    for (int j = 0; j < Lk; ++j) {
      const float vv = bf2f(vc[(int64_t)j * a.ldv]);
#pragma unroll
      for (int g = 0; g < G; ++g) acc[g] = fmaf(sc[g * Lk + j], vv, acc[g]);
    }
    bf16_t* orow = out + ((int64_t)b * a.Lq + t) * ldo + (int64_t)hk * G * D + tid;
#pragma unroll
    for (int g = 0; g < G; ++g) orow[g * D] = f2bf(acc[g] * inv[g]);
  }
  (void)mx;
}

template <int E, int G>
int launch(const svla_attn_decode_args& a, bf16_t* out, int64_t ldo, hipStream_t s) {
  const size_t lds = (size_t)G * a.Lk * sizeof(float);
  if (lds > 48 * 1024) {
    static bool done = false;  // one flag per instantiation
    if (!done) {
      (void)hipFuncSetAttribute((const void*)attn_decode_kernel<E, G>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          128 * 1024);
      done = true;
    }
  }
  hipLaunchKernelGGL((attn_decode_kernel<E, G>), dim3(a.Hkv, a.Lq, a.B), dim3(NT), lds, s, a, out, ldo);
  return svla::check_launch("attn_decode");
}

template <int E>
int launch_g(const svla_attn_decode_args& a, bf16_t* out, int64_t ldo, hipStream_t s) {
  switch (a.Hq / a.Hkv) {
    case 1: return launch<E, 1>(a, out, ldo, s);
    case 2: return launch<E, 2>(a, out, ldo, s);
    default: return launch<E, 4>(a, out, ldo, s);
  }
}

}  // namespace

extern "C" int svla_attn_decode(const svla_attn_decode_args* a, void* out, int64_t ldo, void* stream) {
  SVLA_CHECK_ARG(a && out, "attn_decode: NULL args/out");
  SVLA_CHECK_ARG(a->q && a->k && a->v, "attn_decode: NULL q/k/v");
  SVLA_CHECK_ARG(a->B > 0 && a->Lq > 0 && a->Lk >= a->Lq && a->Hkv > 0 && a->Hq % a->Hkv == 0,
                 "attn_decode: bad B/Lq/Lk/Hq/Hkv");
  const int G = a->Hq / a->Hkv;
  SVLA_CHECK_ARG(G == 1 || G == 2 || G == MAXG, "attn_decode: GQA group must be 1, 2 or 4");
  SVLA_CHECK_ARG(a->D % 64 == 0 && a->D >= 64 && a->D <= 256, "attn_decode: head_dim must be 64/128/192/256");
  SVLA_CHECK_ARG((int64_t)G * a->Lk * 4 <= 128 * 1024, "attn_decode: group * Lk too large for the LDS scores");
  SVLA_CHECK_ARG(a->ldq >= (int64_t)a->Hq * a->D && a->ldk >= (int64_t)a->Hkv * a->D &&
                     a->ldv >= (int64_t)a->Hkv * a->D && ldo >= (int64_t)a->Hq * a->D,
                 "attn_decode: row strides smaller than the head block");
  SVLA_CHECK_ARG(a->B == 1 || (a->bsk >= (int64_t)a->Lk * a->ldk && a->bsv >= (int64_t)a->Lk * a->ldv),
                 "attn_decode: batch strides overlap the cached rows");
  SVLA_CHECK_ARG(!a->kv_class || a->ldc >= a->Lk, "attn_decode: kv_class row stride < Lk");
  hipStream_t s = (hipStream_t)stream;
  bf16_t* o = (bf16_t*)out;
  switch (a->D / 64) {
    case 1: return launch_g<1>(*a, o, ldo, s);
    case 2: return launch_g<2>(*a, o, ldo, s);
    case 3: return launch_g<3>(*a, o, ldo, s);
    default: return launch_g<4>(*a, o, ldo, s);
  }
}
