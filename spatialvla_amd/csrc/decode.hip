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
// svla_attn_decode_rope runs the whole decode-step attention (RoPE + cache append + split + combine) in one
// launch of the split kernel (DecodeFuse below).
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

// Every global load of a workgroup is issued up front -- its K rows (score lanes), its V rows (PV lanes) and q --
// so a chunk costs one memory round trip instead of three dependent ones (q -> K -> V); the arithmetic and its
// order are unchanged.
//
// The fused decode step (svla_attn_decode_rope) adds three things, so one launch replaces qkv_rope_append +
// split + combine:
//  * q is read from the raw q|k|v projection row and rotated on load (qkv_rope_append's rounding);
//  * the Lq (<= DEC_MAXLQ) new keys / values (j >= p0 = Lk - Lq) come from the projection rows: the chunk's new
//    keys are rotated into LDS beside q, the new value rows are loaded from the projection directly; the t == 0
//    workgroup of a chunk appends them (rotated k, v) to the cache rows, which no workgroup of the launch reads;
//  * in-launch combine (cdna_hip_programming.md split-K counter recipe, write-through form): partials and
//    {max, sum} are stored sc1 (agent-scope relaxed atomic stores), every wave drains, one lane draws a ticket
//    from the (bq, kv head) counter; the workgroup that draws nch-1 reads every partial with sc1 loads, combines
//    the chunks in chunk order (attn_decode_combine_kernel's arithmetic: bitwise the unfused output) and
//    re-zeroes the counter.
constexpr int DEC_MAXLQ = 16;

struct DecodeFuse {
  const bf16_t* cos;
  const bf16_t* sin;
  int64_t rope_ld;
  bf16_t* out;
  int64_t ldo;
  int* cnt;  // [B*Lq, Hkv] arrival counters, zero between launches
};

// rotated bf16 value of element d (partner d -/+ D/2) of a rotate_half RoPE row: the qkv_rope_append rounding
__device__ __forceinline__ float rope_elem(float x, float xp, float c, float s, bool lo) {
  return lo ? round_bf(round_bf(x * c) + round_bf(-xp * s)) : round_bf(round_bf(x * c) + round_bf(xp * s));
}

template <bool SC1>
__device__ __forceinline__ void ws_store(float* p, float v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

__device__ __forceinline__ float ws_load_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ROPE: q / new keys from the projection rows, cache append; COMB: in-launch combine (else the combine kernel)
template <int D, int G, bool ROPE, bool COMB>
__global__ __launch_bounds__(NT) void attn_decode_split_kernel(svla_attn_decode_args a, float* __restrict__ ws,
                                                               DecodeFuse f) {
  constexpr int QP = D / 4;       // elements per score lane
  constexpr int KL = QP / 8;      // 16-B K loads per score lane
  constexpr int CPR = D / 8;      // 16-B chunks per V row
  constexpr int RG = NT / CPR;    // V row groups
  constexpr int VR = CH / RG;     // V rows per PV lane
  constexpr int HALF = D / 2;
  __shared__ float qs[G][D];
  __shared__ float sc[G][CH];
  __shared__ float red[RG][G][D];
  __shared__ float kn[ROPE ? DEC_MAXLQ : 1][D];  // ROPE: this chunk's new keys, rotated
  const int c = blockIdx.x, hk = blockIdx.y, bq = blockIdx.z;
  const int b = bq / a.Lq, t = bq % a.Lq;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nch = gridDim.x;
  const int Lk = a.Lk;
  const int qi = Lk - a.Lq + t;
  const int p0 = ROPE ? Lk - a.Lq : Lk;  // first key read from the projection rows (ROPE)
  const bf16_t* qrow = (const bf16_t*)a.q + ((int64_t)b * a.Lq + t) * a.ldq + (int64_t)hk * G * D;
  const bf16_t* kb = (const bf16_t*)a.k + (int64_t)b * a.bsk + (int64_t)hk * D;
  const bf16_t* vb = (const bf16_t*)a.v + (int64_t)b * a.bsv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * a.ldc : nullptr;
  // projection row of new token tt (ROPE): q heads, then Hkv k heads, then Hkv v heads
  auto new_row = [&](int tt) { return (const bf16_t*)a.q + ((int64_t)b * a.Lq + tt) * a.ldq; };

  // ---- stage 1: issue the workgroup's loads
  const int jj = tid >> 2, p = tid & 3;  // score lane: key jj of the chunk, quarter p of the head dim
  const int j = c * CH + jj;
  const bool jv = j < Lk;
  u32x4 kraw[KL];
  if (jv && j < p0) {
    const bf16_t* kr = kb + (int64_t)j * a.ldk + p * QP;
#pragma unroll
    for (int e = 0; e < KL; ++e) kraw[e] = *reinterpret_cast<const u32x4*>(kr + e * 8);
  }
  const int cc = tid % CPR, rg = tid / CPR;  // PV lane: 16-B column chunk cc of rows rg, rg + RG, ..
  u32x4 vraw[VR];
#pragma unroll
  for (int i = 0; i < VR; ++i) {
    const int jr = c * CH + rg + RG * i;
    if (jr < Lk) {
      if (ROPE && jr >= p0)
        vraw[i] = *reinterpret_cast<const u32x4*>(new_row(jr - p0) + (int64_t)(a.Hq + a.Hkv + hk) * D + cc * 8);
      else
        vraw[i] = *reinterpret_cast<const u32x4*>(vb + (int64_t)jr * a.ldv + cc * 8);
    }
  }
  const int n0 = c * CH > p0 ? c * CH : p0;  // ROPE: new keys n0 .. n1-1 sit in this chunk
  const int n1 = (c + 1) * CH < Lk ? (c + 1) * CH : Lk;
  if constexpr (ROPE) {
    for (int i = tid; i < G * D; i += NT) {
      const int g = i / D, d = i % D, dl = d % HALF;
      const bool lo = d < HALF;
      const float x = bf2f(qrow[g * D + d]), xp = bf2f(qrow[g * D + (lo ? d + HALF : d - HALF)]);
      qs[g][d] = rope_elem(x, xp, bf2f(f.cos[(int64_t)bq * f.rope_ld + dl]), bf2f(f.sin[(int64_t)bq * f.rope_ld + dl]), lo);
    }
    for (int i = tid; i < (n1 - n0) * D; i += NT) {
      const int kk = i / D, d = i % D, dl = d % HALF, tt = n0 + kk - p0;
      const bool lo = d < HALF;
      const bf16_t* kr = new_row(tt) + (int64_t)(a.Hq + hk) * D;
      const float r = rope_elem(bf2f(kr[d]), bf2f(kr[lo ? d + HALF : d - HALF]),
                                bf2f(f.cos[((int64_t)b * a.Lq + tt) * f.rope_ld + dl]),
                                bf2f(f.sin[((int64_t)b * a.Lq + tt) * f.rope_ld + dl]), lo);
      kn[kk][d] = r;
      if (t == 0) ((bf16_t*)a.k)[(int64_t)b * a.bsk + (int64_t)(n0 + kk) * a.ldk + (int64_t)hk * D + d] = f2bf(r);
    }
  } else {
    for (int i = tid; i < G * D; i += NT) qs[i / D][i % D] = bf2f(qrow[(i / D) * D + i % D]);
  }
  __syncthreads();
  if constexpr (ROPE) {  // append the new value rows (t == 0 workgroup)
    if (t == 0) {
#pragma unroll
      for (int i = 0; i < VR; ++i) {
        const int jr = c * CH + rg + RG * i;
        if (jr < Lk && jr >= p0)
          *reinterpret_cast<u32x4*>((bf16_t*)a.v + (int64_t)b * a.bsv + (int64_t)jr * a.ldv + (int64_t)hk * D +
                                    cc * 8) = vraw[i];
      }
    }
  }

  // ---- scores
  {
    float s[G];
#pragma unroll
    for (int g = 0; g < G; ++g) s[g] = 0.f;
    if (jv) {
#pragma unroll
      for (int e = 0; e < KL; ++e) {
        float kf[8];
        if (ROPE && j >= p0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) kf[i] = kn[j - n0][p * QP + e * 8 + i];
        } else {
          unpack8(kraw[e], kf);
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
          for (int i = 0; i < 8; ++i) s[g] = fmaf(qs[g][p * QP + e * 8 + i], kf[i], s[g]);
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

  // ---- chunk softmax: wave g <-> query head g
  if (w < G) {
    const float v = sc[w][lane];
    const float m = wave_max(v);
    const float pr = exp2f((v - m) * LOG2E);
    const float l = wave_sum(pr);
    sc[w][lane] = round_bf(pr);  // P enters the PV product as bf16 (the MFMA operand of svla_attn_fwd)
    if (lane == 0) {
      float* o = ws + ws_index(bq, hk * G + w, c, a.Hq, nch, D);
      ws_store<COMB>(o + D, m);
      ws_store<COMB>(o + D + 1, l);
    }
  }
  __syncthreads();

  // ---- PV over the chunk
  {
    float acc[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[g][i] = 0.f;
#pragma unroll
    for (int i = 0; i < VR; ++i) {
      const int jr = c * CH + rg + RG * i;
      if (jr < Lk) {
        float vf[8];
        unpack8(vraw[i], vf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float pj = sc[g][rg + RG * i];
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[g][e] = fmaf(pj, vf[e], acc[g][e]);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rg][g][cc * 8 + e] = acc[g][e];
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += NT) {
    const int g = i / D, d = i % D;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < RG; ++r) v += red[r][g][d];
    ws_store<COMB>(ws + ws_index(bq, hk * G + g, c, a.Hq, nch, D) + d, v);
  }
  if constexpr (COMB) {
    // publish (write-through stores): every wave drains, then one lane draws the ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      int* cnt = f.cnt + (int64_t)bq * a.Hkv + hk;
      // agent-scope release (the barrier above orders every wave's partial stores before it) / acquire pair:
      // the ordering the combine relies on is the memory model's, not only the sc1 ISA behaviour
      const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = old == nch - 1;
      if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sc[0][0] = last ? 1.f : 0.f;  // broadcast through the existing LDS array
    }
    __syncthreads();
    if (sc[0][0] == 0.f) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every thread: the partials of other XCDs are visible
    // combine (attn_decode_combine_kernel's arithmetic and order), chunks in batches of CB whose sc1 loads are all
    // issued before the first use
    constexpr int CB = 8;
    constexpr int PER = (G * D + NT - 1) / NT;  // outputs per thread
    if (nch <= CB) {
      // up to 8 chunks (Lk <= 512, the decode of every SpatialVLA prompt): every partial this thread needs -- both
      // of its outputs, max, sum and O of every chunk -- is loaded in one batch, so the combine is one memory round
      // trip instead of 2 * PER dependent ones; the same arithmetic in the same order as the loop below
      float mv[PER][CB], lv[PER][CB], ov[PER][CB];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + k * NT;
        const int g = i / D, d = i % D;
        const float* o0 = ws + ws_index(bq, hk * G + (i < G * D ? g : 0), 0, a.Hq, nch, D);
#pragma unroll
        for (int u = 0; u < CB; ++u) {
          mv[k][u] = -INFINITY;
          if (u < nch && i < G * D) {
            const float* o = o0 + (int64_t)u * (D + 2);
            mv[k][u] = ws_load_sc1(o + D);
            lv[k][u] = ws_load_sc1(o + D + 1);
            ov[k][u] = ws_load_sc1(o + d);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = tid + k * NT;
        if (i >= G * D) continue;
        const int g = i / D, d = i % D, h = hk * G + g;
        float M = -INFINITY;
#pragma unroll
        for (int u = 0; u < CB; ++u) M = fmaxf(M, mv[k][u]);
        float l = 0.f, acc = 0.f;
#pragma unroll
        for (int u = 0; u < CB; ++u) {
          if (u < nch) {
            const float fc = __expf(mv[k][u] - M);
            l = fmaf(lv[k][u], fc, l);
            acc = fmaf(ov[k][u], fc, acc);
          }
        }
        f.out[(int64_t)bq * f.ldo + (int64_t)h * D + d] = f2bf(acc / l);
      }
      return;
    }
    for (int i = tid; i < G * D; i += NT) {
      const int g = i / D, d = i % D, h = hk * G + g;
      const float* o0 = ws + ws_index(bq, h, 0, a.Hq, nch, D);
      float M = -INFINITY;
      for (int c0 = 0; c0 < nch; c0 += CB) {
        float mv[CB];
#pragma unroll
        for (int u = 0; u < CB; ++u) mv[u] = c0 + u < nch ? ws_load_sc1(o0 + (int64_t)(c0 + u) * (D + 2) + D) : -INFINITY;
#pragma unroll
        for (int u = 0; u < CB; ++u) M = fmaxf(M, mv[u]);
      }
      float l = 0.f, acc = 0.f;
      for (int c0 = 0; c0 < nch; c0 += CB) {
        float mv[CB], lv[CB], ov[CB];
#pragma unroll
        for (int u = 0; u < CB; ++u) {
          if (c0 + u < nch) {
            const float* o = o0 + (int64_t)(c0 + u) * (D + 2);
            mv[u] = ws_load_sc1(o + D);
            lv[u] = ws_load_sc1(o + D + 1);
            ov[u] = ws_load_sc1(o + d);
          }
        }
#pragma unroll
        for (int u = 0; u < CB; ++u) {
          if (c0 + u < nch) {
            const float fc = __expf(mv[u] - M);
            l = fmaf(lv[u], fc, l);
            acc = fmaf(ov[u], fc, acc);
          }
        }
      }
      f.out[(int64_t)bq * f.ldo + (int64_t)h * D + d] = f2bf(acc / l);
    }
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
  hipLaunchKernelGGL((attn_decode_split_kernel<D, G, false, false>), dim3(nch, a.Hkv, a.B * a.Lq), dim3(NT), 0, s, a,
                     ws, DecodeFuse{});
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

// SVLA_DEC_INLAUNCH: 1 = the chunk partials are combined inside the split launch (one launch per decode step),
// 0 = by the combine kernel (two launches)
#ifndef SVLA_DEC_INLAUNCH
#define SVLA_DEC_INLAUNCH 1
#endif

template <int D, int G>
int launch_fused(const svla_attn_decode_args& a, const DecodeFuse& f, float* ws, hipStream_t s) {
  const int nch = (a.Lk + CH - 1) / CH;
  if (SVLA_DEC_INLAUNCH) {
    hipLaunchKernelGGL((attn_decode_split_kernel<D, G, true, true>), dim3(nch, a.Hkv, a.B * a.Lq), dim3(NT), 0, s, a,
                       ws, f);
    return svla::check_launch("attn_decode_rope");
  }
  hipLaunchKernelGGL((attn_decode_split_kernel<D, G, true, false>), dim3(nch, a.Hkv, a.B * a.Lq), dim3(NT), 0, s, a,
                     ws, f);
  if (int rc = svla::check_launch("attn_decode_rope")) return rc;
  hipLaunchKernelGGL((attn_decode_combine_kernel<D>), dim3(a.Hq, a.B * a.Lq), dim3(D), 0, s, a.Hq, nch, ws, f.out,
                     f.ldo);
  return svla::check_launch("attn_decode_rope combine");
}

template <int D>
int launch_fused_g(const svla_attn_decode_args& a, const DecodeFuse& f, float* ws, hipStream_t s) {
  switch (a.Hq / a.Hkv) {
    case 1: return launch_fused<D, 1>(a, f, ws, s);
    case 2: return launch_fused<D, 2>(a, f, ws, s);
    default: return launch_fused<D, 4>(a, f, ws, s);
  }
}

// counters first (a fixed offset, so a workspace zeroed once stays valid for every Lk), then the partials
constexpr size_t FUSED_CNT_ALIGN = 256;
size_t fused_cnt_bytes(int64_t B, int64_t Lq, int64_t Hkv) {
  return (size_t)((B * Lq * Hkv * (int64_t)sizeof(int) + FUSED_CNT_ALIGN - 1) / FUSED_CNT_ALIGN * FUSED_CNT_ALIGN);
}

// Decode-step epilogue of the q|k|v projection (one launch instead of RoPE pass + two cache copies): rotate_half
// RoPE on q (in place) and k, k written rotated and v copied into cache rows p0 + t.  Same rounding as the
// GEMM's ROPE epilogue: out = bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)) (modeling_gemma2.py:123-154).
// One thread owns 8 columns of the low half of a head and their partners D/2 away (q/k), or 16 v columns.
// KBACK (the prefill, svla_qkv_rope_fill): the rotated k is also written back into the projection rows, where the
// prompt's flash attention reads it.
template <bool KBACK>
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
    unpack8(*reinterpret_cast<const u32x4*>(cos_t + m * rope_ld + dd), cs);  // table row = token row b*Lq+t
    unpack8(*reinterpret_cast<const u32x4*>(sin_t + m * rope_ld + dd), sn);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ol[j] = round_bf(xl[j] * cs[j]) + round_bf(-xh[j] * sn[j]);
      oh[j] = round_bf(xh[j] * cs[j]) + round_bf(xl[j] * sn[j]);
    }
    if (head < Hq || KBACK) {  // q stays in the projection output for the attention kernel
      *reinterpret_cast<u32x4*>(lo) = pack8(ol);
      *reinterpret_cast<u32x4*>(hi) = pack8(oh);
    }
    if (head >= Hq) {
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

extern "C" size_t svla_attn_decode_rope_workspace_bytes(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t Lk,
                                                         int32_t D) {
  return fused_cnt_bytes(B, Lq, Hkv) + svla_attn_decode_workspace_bytes(B, Lq, Hq, Lk, D);
}

extern "C" int svla_attn_decode_rope(const svla_attn_decode_args* a, const void* rope_cos, const void* rope_sin,
                                     int64_t rope_ld, void* out, int64_t ldo, void* workspace, size_t ws_bytes,
                                     void* stream) {
  SVLA_CHECK_ARG(a && out && rope_cos && rope_sin, "attn_decode_rope: NULL args/out/tables");
  SVLA_CHECK_ARG(a->q && a->k && a->v, "attn_decode_rope: NULL qkv/k/v");
  SVLA_CHECK_ARG(a->B > 0 && a->Lq > 0 && a->Lq <= DEC_MAXLQ && a->Lk > a->Lq && a->Hkv > 0 && a->Hq % a->Hkv == 0,
                 "attn_decode_rope: bad B/Lq/Lk/Hq/Hkv (Lq <= 16 new tokens after a cached prefix, Lk > Lq)");
  const int G = a->Hq / a->Hkv;
  SVLA_CHECK_ARG(G == 1 || G == 2 || G == MAXG, "attn_decode_rope: GQA group must be 1, 2 or 4");
  SVLA_CHECK_ARG(a->D == 64 || a->D == 128 || a->D == 256, "attn_decode_rope: head_dim must be 64, 128 or 256");
  SVLA_CHECK_ARG(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0 && a->bsk % 8 == 0 && a->bsv % 8 == 0 &&
                     rope_ld % 8 == 0,
                 "attn_decode_rope: strides must be multiples of 8");
  SVLA_CHECK_ARG((((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v | (uintptr_t)rope_cos | (uintptr_t)rope_sin) &
                  15) == 0,
                 "attn_decode_rope: qkv/k/v/tables must be 16-B aligned");
  SVLA_CHECK_ARG(a->ldq >= (int64_t)(a->Hq + 2 * a->Hkv) * a->D && a->ldk >= (int64_t)a->Hkv * a->D &&
                     a->ldv >= (int64_t)a->Hkv * a->D && ldo >= (int64_t)a->Hq * a->D && rope_ld >= a->D / 2,
                 "attn_decode_rope: row strides smaller than the head block");
  SVLA_CHECK_ARG(a->B == 1 || (a->bsk >= (int64_t)a->Lk * a->ldk && a->bsv >= (int64_t)a->Lk * a->ldv),
                 "attn_decode_rope: batch strides overlap the cached rows");
  SVLA_CHECK_ARG(!a->kv_class || a->ldc >= a->Lk, "attn_decode_rope: kv_class row stride < Lk");
  SVLA_CHECK_ARG(workspace && ((uintptr_t)workspace & 255) == 0 &&
                     ws_bytes >= svla_attn_decode_rope_workspace_bytes(a->B, a->Lq, a->Hq, a->Hkv, a->Lk, a->D),
                 "attn_decode_rope: workspace must be 256-B aligned and >= svla_attn_decode_rope_workspace_bytes()");
  DecodeFuse f;
  f.cos = (const bf16_t*)rope_cos;
  f.sin = (const bf16_t*)rope_sin;
  f.rope_ld = rope_ld;
  f.out = (bf16_t*)out;
  f.ldo = ldo;
  f.cnt = (int*)workspace;
  float* ws = (float*)((char*)workspace + fused_cnt_bytes(a->B, a->Lq, a->Hkv));
  hipStream_t s = (hipStream_t)stream;
  switch (a->D) {
    case 64: return launch_fused_g<64>(*a, f, ws, s);
    case 128: return launch_fused_g<128>(*a, f, ws, s);
    default: return launch_fused_g<256>(*a, f, ws, s);
  }
}

namespace {
template <bool KBACK>
int qkv_rope_append_impl(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                         const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache, int64_t ldk,
                         int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0, void* stream) {
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
  hipLaunchKernelGGL(qkv_rope_append_kernel<KBACK>, dim3((unsigned)((work + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, B, Lq, Hq, Hkv, D, (bf16_t*)qkv, ld, (const bf16_t*)rope_cos,
                     (const bf16_t*)rope_sin, rope_ld, (bf16_t*)k_cache, ldk, bsk, (bf16_t*)v_cache, ldv, bsv, p0);
  return svla::check_launch("qkv_rope_append");
}
}  // namespace

extern "C" int svla_qkv_rope_append(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                                    const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache,
                                    int64_t ldk, int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0,
                                    void* stream) {
  return qkv_rope_append_impl<false>(B, Lq, Hq, Hkv, D, qkv, ld, rope_cos, rope_sin, rope_ld, k_cache, ldk, bsk,
                                     v_cache, ldv, bsv, p0, stream);
}

extern "C" int svla_qkv_rope_fill(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                                  const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache,
                                  int64_t ldk, int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0,
                                  void* stream) {
  return qkv_rope_append_impl<true>(B, Lq, Hq, Hkv, D, qkv, ld, rope_cos, rope_sin, rope_ld, k_cache, ldk, bsk,
                                    v_cache, ldv, bsv, p0, stream);
}
