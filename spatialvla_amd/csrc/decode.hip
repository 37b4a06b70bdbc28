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
// K/V cache, HBM-bound (Lk * Hkv * D * 2 * 2 bytes per sequence), far from MFMA territory.  At B = 1 one
// workgroup per head would leave the chip idle, so the keys are split ("flash decoding"):
//  * attn_decode_split_kernel, grid (ceil(Lk/64), Hkv, B*Lq): one workgroup per 64-key chunk and kv head;
//    the Hq/Hkv query heads of the GQA group share every K/V row it reads.  Scores: 4 lanes per key, each
//    with D/4 contiguous elements (16-B loads), q from LDS, two butterfly steps.  Chunk softmax: wave g owns
//    query head g (64 keys = 64 lanes).  PV: D/8 lanes cover a V row with 16-B loads, 256/(D/8) row groups
//    reduce through LDS.  Writes the chunk's (max, sum, unnormalised O) to the fp32 workspace;
//  * attn_decode_combine_kernel, grid (Hq, B*Lq): rescales the chunks to the global max and normalises.
#include "svla_common.h"

namespace {

constexpr float MASKVAL = -3.3895313892515355e38f;  // torch.finfo(bfloat16).min, as the reference mask
constexpr float LOG2E = 1.4426950408889634f;
constexpr int NT = 256;
constexpr int CH = 64;  // keys per chunk
constexpr int MAXG = 4;

__device__ __forceinline__ bool visible(int c, int kj, int qi, int window) {
  bool v = (c == 0) || (c == 1 && kj <= qi);
  if (window > 0 && qi - kj >= window) v = false;
  return v;
}

// workspace per (sequence-query bq, query head h, chunk c): [D] O partial, then {max, sum}
__host__ __device__ inline int64_t ws_index(int64_t bq, int h, int c, int Hq, int nch, int D) {
  return (((int64_t)bq * Hq + h) * nch + c) * (D + 2);
}

template <int D, int G>
__global__ __launch_bounds__(NT) void attn_decode_split_kernel(svla_attn_decode_args a, float* __restrict__ ws) {
  constexpr int QP = D / 4;       // elements per score lane
  constexpr int CPR = D / 8;      // 16-B chunks per V row
  constexpr int RG = NT / CPR;    // V row groups
  __shared__ float qs[G][D];
  __shared__ float sc[G][CH];
  __shared__ float red[RG][G][D];
  const int c = blockIdx.x, hk = blockIdx.y, bq = blockIdx.z;
  const int b = bq / a.Lq, t = bq % a.Lq;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nch = gridDim.x;
  const int Lk = a.Lk;
  const int qi = Lk - a.Lq + t;
  const bf16_t* qrow = (const bf16_t*)a.q + ((int64_t)b * a.Lq + t) * a.ldq + (int64_t)hk * G * D;
  const bf16_t* kb = (const bf16_t*)a.k + (int64_t)b * a.bsk + (int64_t)hk * D;
  const bf16_t* vb = (const bf16_t*)a.v + (int64_t)b * a.bsv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * a.ldc : nullptr;
  for (int i = tid; i < G * D; i += NT) qs[i / D][i % D] = bf2f(qrow[(i / D) * D + i % D]);
  __syncthreads();

  // scores: key jj = tid/4, quarter p = tid%4 of the head dim
  {
    const int jj = tid >> 2, p = tid & 3;
    const int j = c * CH + jj;
    const bool jv = j < Lk;
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    if (jv) {
      const bf16_t* kr = kb + (int64_t)j * a.ldk + p * QP;
#pragma unroll
      for (int e = 0; e < QP; e += 8) {
        float kf[8];
        unpack8(*reinterpret_cast<const u32x4*>(kr + e), kf);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int i = 0; i < 8; ++i) s[g] = fmaf(qs[g][p * QP + e + i], kf[i], s[g]);
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      s[g] += __shfl_xor(s[g], 1, 64);
      s[g] += __shfl_xor(s[g], 2, 64);
    }
    if (p == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float v = -INFINITY;
        if (jv) {
          v = s[g] * a.scale;
          if (a.softcap > 0.f) v = a.softcap * fast_tanh(v / a.softcap);
          if (!visible(cls ? cls[j] : 0, j, qi, a.sliding_window)) v = MASKVAL;
        }
        sc[g][jj] = v;
      }
    }
  }
  __syncthreads();

  // chunk softmax: wave g <-> query head g
  if (w < G) {
    const float v = sc[w][lane];
    const float m = wave_max(v);
    const float pr = exp2f((v - m) * LOG2E);
    const float l = wave_sum(pr);
    sc[w][lane] = round_bf(pr);  // P enters the PV product as bf16 (the MFMA operand of svla_attn_fwd)
    if (lane == 0) {
      float* o = ws + ws_index(bq, hk * G + w, c, a.Hq, nch, D);
      o[D] = m;
      o[D + 1] = l;
    }
  }
  __syncthreads();

  // PV over the chunk
  {
    const int cc = tid % CPR, rg = tid / CPR;
    float acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[g][i] = 0.f;
    for (int jj = rg; jj < CH; jj += RG) {
      const int j = c * CH + jj;
      if (j >= Lk) break;
      float vf[8];
      unpack8(*reinterpret_cast<const u32x4*>(vb + (int64_t)j * a.ldv + cc * 8), vf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float pj = sc[g][jj];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[g][i] = fmaf(pj, vf[i], acc[g][i]);
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[rg][g][cc * 8 + i] = acc[g][i];
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += NT) {
    const int g = i / D, d = i % D;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RG; ++r) v += red[r][g][d];
    ws[ws_index(bq, hk * G + g, c, a.Hq, nch, D) + d] = v;
  }
}

template <int D>
__global__ __launch_bounds__(D) void attn_decode_combine_kernel(int Hq, int nch, const float* __restrict__ ws,
                                                                 bf16_t* __restrict__ out, int64_t ldo) {
  const int h = blockIdx.x, bq = blockIdx.y, d = threadIdx.x;
  float M = -INFINITY;
  for (int c = 0; c < nch; ++c) M = fmaxf(M, ws[ws_index(bq, h, c, Hq, nch, D) + D]);
  float l = 0.f, acc = 0.f;
  for (int c = 0; c < nch; ++c) {
    const float* o = ws + ws_index(bq, h, c, Hq, nch, D);
    const float f = __expf(o[D] - M);  // chunks whose keys are all masked (max = bf16 min) drop out
    l = fmaf(o[D + 1], f, l);
    acc = fmaf(o[d], f, acc);
  }
  out[(int64_t)bq * ldo + (int64_t)h * D + d] = f2bf(acc / l);
}

template <int D, int G>
int launch(const svla_attn_decode_args& a, bf16_t* out, int64_t ldo, float* ws, hipStream_t s) {
  const int nch = (a.Lk + CH - 1) / CH;
  hipLaunchKernelGGL((attn_decode_split_kernel<D, G>), dim3(nch, a.Hkv, a.B * a.Lq), dim3(NT), 0, s, a, ws);
  if (int rc = svla::check_launch("attn_decode")) return rc;
  hipLaunchKernelGGL((attn_decode_combine_kernel<D>), dim3(a.Hq, a.B * a.Lq), dim3(D), 0, s, a.Hq, nch, ws, out,
                     ldo);
  return svla::check_launch("attn_decode combine");
}

template <int D>
int launch_g(const svla_attn_decode_args& a, bf16_t* out, int64_t ldo, float* ws, hipStream_t s) {
  switch (a.Hq / a.Hkv) {
    case 1: return launch<D, 1>(a, out, ldo, ws, s);
    case 2: return launch<D, 2>(a, out, ldo, ws, s);
    default: return launch<D, 4>(a, out, ldo, ws, s);
  }
}

// Decode-step epilogue of the q|k|v projection (one launch instead of RoPE pass + two cache copies): rotate_half
// RoPE on q (in place) and k, k written rotated and v copied into cache rows p0 + t.  Same rounding as the
// GEMM's ROPE epilogue: out = bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)) (modeling_gemma2.py:123-154).
// One thread owns 8 columns of the low half of a head and their partners D/2 away (q/k), or 16 v columns.
__global__ void qkv_rope_append_kernel(int B, int Lq, int Hq, int Hkv, int D, bf16_t* __restrict__ qkv, int64_t ld,
                                       const bf16_t* __restrict__ cos_t, const bf16_t* __restrict__ sin_t,
                                       int64_t rope_ld, bf16_t* __restrict__ kc, int64_t ldk, int64_t bsk,
                                       bf16_t* __restrict__ vc, int64_t ldv, int64_t bsv, int p0) {
  const int half = D >> 1, cph = half / 8;
  const int64_t rot_per_row = (int64_t)(Hq + Hkv) * cph, v_per_row = (int64_t)Hkv * D / 16;
  const int64_t per_row = rot_per_row + v_per_row;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)B * Lq * per_row) return;
  const int64_t m = idx / per_row;
  const int r = (int)(idx % per_row);
  const int b = (int)(m / Lq), t = (int)(m % Lq);
  bf16_t* row = qkv + m * ld;
  if (r < rot_per_row) {
    const int head = r / cph, dd = (r % cph) * 8;
    bf16_t* lo = row + (int64_t)head * D + dd;
    bf16_t* hi = lo + half;
    float xl[8], xh[8], cs[8], sn[8], ol[8], oh[8];
    unpack8(*reinterpret_cast<const u32x4*>(lo), xl);
    unpack8(*reinterpret_cast<const u32x4*>(hi), xh);
    unpack8(*reinterpret_cast<const u32x4*>(cos_t + (int64_t)t * rope_ld + dd), cs);
    unpack8(*reinterpret_cast<const u32x4*>(sin_t + (int64_t)t * rope_ld + dd), sn);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ol[j] = round_bf(xl[j] * cs[j]) + round_bf(-xh[j] * sn[j]);
      oh[j] = round_bf(xh[j] * cs[j]) + round_bf(xl[j] * sn[j]);
    }
    if (head < Hq) {  // q stays in the projection output for the attention kernel
      *reinterpret_cast<u32x4*>(lo) = pack8(ol);
      *reinterpret_cast<u32x4*>(hi) = pack8(oh);
    } else {
      bf16_t* kr = kc + (int64_t)b * bsk + (int64_t)(p0 + t) * ldk + (int64_t)(head - Hq) * D + dd;
      *reinterpret_cast<u32x4*>(kr) = pack8(ol);
      *reinterpret_cast<u32x4*>(kr + half) = pack8(oh);
    }
  } else {
    const int c = (r - (int)rot_per_row) * 16;
    const bf16_t* src = row + (int64_t)(Hq + Hkv) * D + c;
    bf16_t* dst = vc + (int64_t)b * bsv + (int64_t)(p0 + t) * ldv + c;
    *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
    *reinterpret_cast<u32x4*>(dst + 8) = *reinterpret_cast<const u32x4*>(src + 8);
  }
}

}  // namespace

extern "C" size_t svla_attn_decode_workspace_bytes(int32_t B, int32_t Lq, int32_t Hq, int32_t Lk, int32_t D) {
  const int64_t nch = ((int64_t)Lk + CH - 1) / CH;
  return (size_t)B * Lq * Hq * nch * (D + 2) * sizeof(float);
}

extern "C" int svla_attn_decode(const svla_attn_decode_args* a, void* out, int64_t ldo, float* workspace,
                                size_t ws_bytes, void* stream) {
  SVLA_CHECK_ARG(a && out, "attn_decode: NULL args/out");
  SVLA_CHECK_ARG(a->q && a->k && a->v, "attn_decode: NULL q/k/v");
  SVLA_CHECK_ARG(a->B > 0 && a->Lq > 0 && a->Lk >= a->Lq && a->Hkv > 0 && a->Hq % a->Hkv == 0,
                 "attn_decode: bad B/Lq/Lk/Hq/Hkv");
  const int G = a->Hq / a->Hkv;
  SVLA_CHECK_ARG(G == 1 || G == 2 || G == MAXG, "attn_decode: GQA group must be 1, 2 or 4");
  SVLA_CHECK_ARG(a->D == 64 || a->D == 128 || a->D == 256, "attn_decode: head_dim must be 64, 128 or 256");
  SVLA_CHECK_ARG(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0 && a->bsk % 8 == 0 && a->bsv % 8 == 0,
                 "attn_decode: strides must be multiples of 8");
  SVLA_CHECK_ARG(((uintptr_t)a->k & 15) == 0 && ((uintptr_t)a->v & 15) == 0, "attn_decode: k/v must be 16-B aligned");
  SVLA_CHECK_ARG(a->ldq >= (int64_t)a->Hq * a->D && a->ldk >= (int64_t)a->Hkv * a->D &&
                     a->ldv >= (int64_t)a->Hkv * a->D && ldo >= (int64_t)a->Hq * a->D,
                 "attn_decode: row strides smaller than the head block");
  SVLA_CHECK_ARG(a->B == 1 || (a->bsk >= (int64_t)a->Lk * a->ldk && a->bsv >= (int64_t)a->Lk * a->ldv),
                 "attn_decode: batch strides overlap the cached rows");
  SVLA_CHECK_ARG(!a->kv_class || a->ldc >= a->Lk, "attn_decode: kv_class row stride < Lk");
  SVLA_CHECK_ARG(workspace && ws_bytes >= svla_attn_decode_workspace_bytes(a->B, a->Lq, a->Hq, a->Lk, a->D),
                 "attn_decode: workspace smaller than svla_attn_decode_workspace_bytes()");
  hipStream_t s = (hipStream_t)stream;
  bf16_t* o = (bf16_t*)out;
  switch (a->D) {
    case 64: return launch_g<64>(*a, o, ldo, workspace, s);
    case 128: return launch_g<128>(*a, o, ldo, workspace, s);
    default: return launch_g<256>(*a, o, ldo, workspace, s);
  }
}

extern "C" int svla_qkv_rope_append(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                                    const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache,
                                    int64_t ldk, int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0,
                                    void* stream) {
  SVLA_CHECK_ARG(qkv && rope_cos && rope_sin && k_cache && v_cache, "qkv_rope_append: NULL pointer");
  SVLA_CHECK_ARG(B > 0 && Lq > 0 && Hq > 0 && Hkv > 0 && p0 >= 0, "qkv_rope_append: bad sizes");
  SVLA_CHECK_ARG(D % 16 == 0 && D <= 256, "qkv_rope_append: head_dim must be a multiple of 16, <= 256");
  SVLA_CHECK_ARG(ld % 8 == 0 && rope_ld % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && bsk % 8 == 0 && bsv % 8 == 0 &&
                     ld >= (int64_t)(Hq + 2 * Hkv) * D && ldk >= (int64_t)Hkv * D && ldv >= (int64_t)Hkv * D,
                 "qkv_rope_append: strides");
  SVLA_CHECK_ARG((((uintptr_t)qkv | (uintptr_t)k_cache | (uintptr_t)v_cache | (uintptr_t)rope_cos |
                   (uintptr_t)rope_sin) & 15) == 0, "qkv_rope_append: pointers must be 16-B aligned");
  const int64_t per_row = (int64_t)(Hq + Hkv) * (D / 16) + (int64_t)Hkv * D / 16;
  const int64_t work = (int64_t)B * Lq * per_row;
  hipLaunchKernelGGL(qkv_rope_append_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     B, Lq, Hq, Hkv, D, (bf16_t*)qkv, ld, (const bf16_t*)rope_cos, (const bf16_t*)rope_sin, rope_ld,
                     (bf16_t*)k_cache, ldk, bsk, (bf16_t*)v_cache, ldv, bsv, p0);
  return svla::check_launch("qkv_rope_append");
}
