// Fused prefix-LM GQA attention with logit softcap and on-load RoPE (Gemma2, head_dim 256) and
// plain bidirectional MHA (SigLIP, head_dim 72), forward and backward, for gfx950.
//
// Reference semantics: eager_attention_forward (model/modeling_gemma2.py:169-195): S = QK^T*scale,
// S = cap*tanh(S/cap), S += additive mask, softmax in fp32, P->bf16, O = PV; mask from
// _update_causal_mask (model/modeling_spatialvla.py:258-306) given here as per-key classes.
//
// CDNA4 layout choices:
//  * "swapped" S^T = K Q^T (16x16x32 MFMA): the accumulator puts one query per lane column, so the
//    row max / row sum need only 2 cross-lane steps, and the fp32 accumulator registers ARE the
//    B operand of the next product (O^T = V^T P^T) after a bf16 pack — P never touches LDS.  The
//    k order inside each 32-key MFMA step is permuted identically on both operands.
//  * V (and Q / dO / K where they feed a product over the key or query index) is consumed through
//    ds_read_b64_tr_b16 transpose reads from row-major LDS tiles; all tiles use the XOR swizzle
//    chunk ^ 2*(row&7), conflict-free for both the ds_read_b128 row reads and the tr reads.
//  * RoPE (rotate_half, modeling_gemma2.py:123-154) is applied in registers while Q/K are
//    loaded (d and d+128 sit in the same lane), and its transpose is applied to dQ/dK in the
//    accumulators before the store — no separate RoPE pass over HBM.
//  * Backward is two deterministic kernels (dK/dV per key tile looping over the GQA query heads,
//    dQ per query tile) — no float atomics.
#include "svla_common.h"

namespace {

constexpr float MASKVAL = -3.3895313892515355e38f;  // torch.finfo(bfloat16).min

template <int D> struct Cfg;
template <> struct Cfg<256> { static constexpr int DP = 256, DV = 256, RS = 256; };
template <> struct Cfg<72>  { static constexpr int DP = 96,  DV = 80,  RS = 128; };

// byte offset of 16-B chunk `ch` of row `r` in a [64][RS] bf16 LDS tile
template <int RS>
__device__ __forceinline__ int toff(int r, int ch) {
  return r * RS * 2 + ((ch ^ ((r & 7) << 1)) << 4);
}

// fragment of 16 rows (r0..r0+15) x 8 consecutive columns (32ks + 8g ..) : ds_read_b128
template <int RS>
__device__ __forceinline__ bf16x8 frag_row(const char* lds, int r0, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + toff<RS>(r0 + (lane & 15), 4 * ks + (lane >> 4)));
}
// transposed fragment: rows (k index) {rb+4g+q} and {rb+16+4g+q}, columns c0..c0+15 ; lane gets column c0+(l&15)
template <int RS>
__device__ __forceinline__ bf16x8 frag_tr(const char* lds, int rb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int col = c0 + 4 * p;
  const int r1 = rb + 4 * g + q, r2 = r1 + 16;
  const char* a1 = lds + toff<RS>(r1, col >> 3) + (col & 7) * 2;
  const char* a2 = lds + toff<RS>(r2, col >> 3) + (col & 7) * 2;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a2));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ bf16x8 pack_frag(const float* v) {
  // v[0..7] -> bf16x8
  u32x4 u = pack8(v);
  return __builtin_bit_cast(bf16x8, u);
}

// rotate a pair of 8-element chunks (d, d+128) by RoPE: lo' = lo*c - hi*s, hi' = hi*c + lo*s
__device__ __forceinline__ void rope_pair(float* lo, float* hi, const bf16_t* cs, const bf16_t* sn) {
  float c[8], s[8];
  unpack8(*reinterpret_cast<const u32x4*>(cs), c);
  unpack8(*reinterpret_cast<const u32x4*>(sn), s);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = lo[j], b = hi[j];
    lo[j] = a * c[j] - b * s[j];
    hi[j] = b * c[j] + a * s[j];
  }
}
// transpose of rope_pair (gradient): dlo = dlo'*c + dhi'*s, dhi = dhi'*c - dlo'*s
__device__ __forceinline__ void rope_pair_t(float& lo, float& hi, float c, float s) {
  float a = lo, b = hi;
  lo = a * c + b * s;
  hi = b * c - a * s;
}

// Stage a [64 rows][D] tile (row r -> global row row0+r of a (b,·,h) head slice) into LDS, zero
// padding columns >= D and rows >= L.  With ROPE (D==256), chunk pairs (c, c+16) are rotated.
template <int D, bool ROPE>
__device__ __forceinline__ void stage_tile(char* lds, const bf16_t* base, int64_t ld, int row0, int L,
                                           const svla_attn_args& a, int t) {
  constexpr int RS = Cfg<D>::RS;
  if constexpr (ROPE) {
    static_assert(D == 256, "rope needs D=256");
    for (int idx = t; idx < 64 * 16; idx += 256) {
      const int r = idx >> 4, ch = idx & 15;
      const int row = row0 + r;
      u32x4 lo = {0u, 0u, 0u, 0u}, hi = {0u, 0u, 0u, 0u};
      if (row < L) {
        const bf16_t* p = base + (int64_t)row * ld + ch * 8;
        float fl[8], fh[8];
        unpack8(*reinterpret_cast<const u32x4*>(p), fl);
        unpack8(*reinterpret_cast<const u32x4*>(p + 128), fh);
        const bf16_t* cs = (const bf16_t*)a.rope_cos + (int64_t)row * a.rope_ld + ch * 8;
        const bf16_t* sn = (const bf16_t*)a.rope_sin + (int64_t)row * a.rope_ld + ch * 8;
        rope_pair(fl, fh, cs, sn);
        lo = pack8(fl);
        hi = pack8(fh);
      }
      *reinterpret_cast<u32x4*>(lds + toff<RS>(r, ch)) = lo;
      *reinterpret_cast<u32x4*>(lds + toff<RS>(r, ch + 16)) = hi;
    }
  } else {
    constexpr int NCH = RS / 8;
    for (int idx = t; idx < 64 * NCH; idx += 256) {
      const int r = idx / NCH, ch = idx % NCH;
      const int row = row0 + r;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (row < L && ch * 8 < D) v = *reinterpret_cast<const u32x4*>(base + (int64_t)row * ld + ch * 8);
      *reinterpret_cast<u32x4*>(lds + toff<RS>(r, ch)) = v;
    }
  }
}

// Per-lane register fragments of one row (the lane's query/key) for all k-steps over d:
// frag[ks][j] = X[row][32ks + 8g + j]; rotated by RoPE in registers when ROPE.
template <int D, bool ROPE>
__device__ __forceinline__ void load_row_frags(bf16x8 (&f)[Cfg<D>::DP / 32], const bf16_t* rowp, bool valid,
                                               const svla_attn_args& a, int row, int lane) {
  constexpr int NKS = Cfg<D>::DP / 32;
  const int g = lane >> 4;
  float v[NKS][8];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int d = 32 * ks + 8 * g;
    if (valid && d < D) unpack8(*reinterpret_cast<const u32x4*>(rowp + d), v[ks]);
    else
#pragma unroll
      for (int j = 0; j < 8; ++j) v[ks][j] = 0.f;
  }
  if constexpr (ROPE) {
    if (valid) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int d = 32 * ks + 8 * g;
        rope_pair(v[ks], v[ks + 4], (const bf16_t*)a.rope_cos + (int64_t)row * a.rope_ld + d,
                  (const bf16_t*)a.rope_sin + (int64_t)row * a.rope_ld + d);
      }
    }
  }
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) f[ks] = pack_frag(v[ks]);
}

__device__ __forceinline__ bool visible(const uint8_t* cls, int kj, int qi, int window) {
  const int c = cls ? cls[kj] : 0;
  bool v = (c == 0) || (c == 1 && kj <= qi);
  if (window > 0 && qi - kj >= window) v = false;
  return v;
}

__device__ __forceinline__ float softcap_f(float z, float cap) { return cap > 0.f ? cap * tanhf(z / cap) : z; }

// ================================================================== forward
template <int D, bool ROPE>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(svla_attn_args a, bf16_t* __restrict__ out, int64_t ldo,
                                                          float* __restrict__ lse) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + 64 * RS * 2;
  uint8_t* lcls = (uint8_t*)(smem + 2 * 64 * RS * 2);

  const int b = blockIdx.z, h = blockIdx.y, qt = blockIdx.x;
  const int grp = a.Hq / a.Hkv, hk = h / grp;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int L = a.L;
  const int qi = qt * 64 + 16 * w + c;
  const bool qvalid = qi < L;

  const bf16_t* qbase = (const bf16_t*)a.q + (int64_t)b * L * a.ldq + (int64_t)h * D;
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * L : nullptr;

  bf16x8 qf[NKS];
  load_row_frags<D, ROPE>(qf, qbase + (int64_t)qi * a.ldq, qvalid, a, qi, lane);

  f32x4 acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const float LOG2E = 1.4426950408889634f;

  const int nkt = (L + 63) / 64;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    stage_tile<D, ROPE>(ldsK, kbase, a.ldk, kt * 64, L, a, t);
    stage_tile<D, false>(ldsV, vbase, a.ldv, kt * 64, L, a, t);
    if (t < 64) lcls[t] = (cls && kt * 64 + t < L) ? cls[kt * 64 + t] : 0;
    __syncthreads();

    f32x4 s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row<RS>(ldsK, 16 * nt, ks, lane), qf[ks], s[nt], 0, 0, 0);
    }
    float x[4][4];
    float mt = -INFINITY;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kl = 16 * nt + 4 * g + j, kj = kt * 64 + kl;
        float v = softcap_f(s[nt][j] * a.scale, a.softcap);
        if (kj >= L) v = -INFINITY;
        else if (!visible(a.kv_class ? lcls : nullptr, kl, qi - kt * 64, a.sliding_window)) v = MASKVAL;
        x[nt][j] = v;
        mt = fmaxf(mt, v);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mnew = fmaxf(m, mt);
    const float alpha = __expf(m - mnew);  // m=-inf -> 0
    float ps = 0.f;
    float p[4][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        p[nt][j] = exp2f((x[nt][j] - mnew) * LOG2E);
        ps += p[nt][j];
      }
    l = l * alpha + ps;
    m = mnew;
#pragma unroll
    for (int i = 0; i < NDT; ++i) acc[i] *= alpha;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float pv[8] = {p[2 * ks][0], p[2 * ks][1], p[2 * ks][2], p[2 * ks][3],
                     p[2 * ks + 1][0], p[2 * ks + 1][1], p[2 * ks + 1][2], p[2 * ks + 1][3]};
      const bf16x8 pb = pack_frag(pv);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr<RS>(ldsV, 32 * ks, 16 * dt, lane), pb, acc[dt], 0, 0, 0);
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.0f / l;
  if (qvalid && g == 0) lse[((int64_t)b * a.Hq + h) * L + qi] = m + __logf(l);

  // O^T accumulators (d = 16dt + 4g + j, q = lane col) -> per-wave LDS image [16 q][DV] -> 16-B stores
  __syncthreads();
  bf16_t* img = (bf16_t*)(smem) + w * 16 * DV;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    uint32_t lo = pack2(acc[dt][0] * inv, acc[dt][1] * inv), hi = pack2(acc[dt][2] * inv, acc[dt][3] * inv);
    *reinterpret_cast<u32x2*>(img + c * DV + 16 * dt + 4 * g) = u32x2{lo, hi};
  }
  __syncthreads();
  constexpr int CPR = D / 8;  // 16-B chunks per output row
  for (int idx = lane; idx < 16 * CPR; idx += 64) {
    const int r = idx / CPR, ch = idx % CPR;
    const int q = qt * 64 + 16 * w + r;
    if (q < L)
      *reinterpret_cast<u32x4*>(out + ((int64_t)b * L + q) * ldo + (int64_t)h * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(img + r * DV + ch * 8);
  }
}

// ================================================================== backward: delta = rowsum(dO * O)
__global__ void attn_delta_kernel(int B, int L, int H, int D, const bf16_t* __restrict__ o, int64_t ldo,
                                  const bf16_t* __restrict__ dout, int64_t lddo, float* __restrict__ delta) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (b, q, h) rows
  const int lane = threadIdx.x & 63;
  if (row >= (int64_t)B * L * H) return;
  const int h = (int)(row % H);
  const int64_t bq = row / H;
  const int q = (int)(bq % L), b = (int)(bq / L);
  const bf16_t* po = o + bq * ldo + (int64_t)h * D;
  const bf16_t* pd = dout + bq * lddo + (int64_t)h * D;
  float s = 0.f;
  for (int d = lane * 8; d < D; d += 512) {
    float x[8], y[8];
    unpack8(*reinterpret_cast<const u32x4*>(po + d), x);
    unpack8(*reinterpret_cast<const u32x4*>(pd + d), y);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * y[j];
  }
  s = wave_sum(s);
  if (lane == 0) delta[((int64_t)b * H + h) * L + q] = s;
}

// ================================================================== backward: dK, dV
template <int D, bool ROPE>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkv_kernel(svla_attn_args a, const bf16_t* __restrict__ dout,
                                                              int64_t lddo, const float* __restrict__ lse,
                                                              const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                                              int64_t lddk, bf16_t* __restrict__ dv, int64_t lddv) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16;
  constexpr int TB = 64 * RS * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + TB;
  char* ldsQ = smem + 2 * TB;
  char* ldsO = smem + 3 * TB;
  float* llse = (float*)(smem + 4 * TB);
  float* ldel = llse + 64;
  uint8_t* lcls = (uint8_t*)(ldel + 64);

  const int b = blockIdx.z, hk = blockIdx.y, kt = blockIdx.x;
  const int grp = a.Hq / a.Hkv;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int L = a.L;
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * L : nullptr;

  stage_tile<D, ROPE>(ldsK, kbase, a.ldk, kt * 64, L, a, t);
  stage_tile<D, false>(ldsV, vbase, a.ldv, kt * 64, L, a, t);
  if (t < 64) lcls[t] = (cls && kt * 64 + t < L) ? cls[kt * 64 + t] : 0;

  const int kl = 16 * w + c;  // this lane's key (local)
  const int kj = kt * 64 + kl;
  f32x4 adk[NDT], adv[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) adk[i] = adv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float LOG2E = 1.4426950408889634f;
  const int nqt = (L + 63) / 64;

  for (int hh = 0; hh < grp; ++hh) {
    const int h = hk * grp + hh;
    const bf16_t* qbase = (const bf16_t*)a.q + (int64_t)b * L * a.ldq + (int64_t)h * D;
    const bf16_t* obase = dout + (int64_t)b * L * lddo + (int64_t)h * D;
    for (int qt = 0; qt < nqt; ++qt) {
      __syncthreads();
      stage_tile<D, ROPE>(ldsQ, qbase, a.ldq, qt * 64, L, a, t);
      stage_tile<D, false>(ldsO, obase, lddo, qt * 64, L, a, t);
      if (t < 64) {
        const int q = qt * 64 + t;
        llse[t] = q < L ? lse[((int64_t)b * a.Hq + h) * L + q] : 0.f;
        ldel[t] = q < L ? delta[((int64_t)b * a.Hq + h) * L + q] : 0.f;
      }
      __syncthreads();
      f32x4 s[4], dp[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        s[mt] = dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row<RS>(ldsQ, 16 * mt, ks, lane),
                                                          frag_row<RS>(ldsK, 16 * w, ks, lane), s[mt], 0, 0, 0);
          dp[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row<RS>(ldsO, 16 * mt, ks, lane),
                                                           frag_row<RS>(ldsV, 16 * w, ks, lane), dp[mt], 0, 0, 0);
        }
      }
      // element (mt, j): query ql = 16mt + 4g + j, key = lane col (kl)
      float pz[4][4], zz[4][4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ql = 16 * mt + 4 * g + j, qi = qt * 64 + ql;
          float p = 0.f, z = 0.f;
          if (qi < L && kj < L) {
            const float sc = softcap_f(s[mt][j] * a.scale, a.softcap);
            const float xv = visible(a.kv_class ? lcls : nullptr, kl, qi - kt * 64, a.sliding_window) ? sc : MASKVAL;
            p = exp2f((xv - llse[ql]) * LOG2E);
            const float ds = p * (dp[mt][j] - ldel[ql]);
            const float dcap = a.softcap > 0.f ? (1.0f - (sc / a.softcap) * (sc / a.softcap)) : 1.0f;
            z = ds * dcap * a.scale;
          }
          pz[mt][j] = p;
          zz[mt][j] = z;
        }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pv[8] = {pz[2 * ks][0], pz[2 * ks][1], pz[2 * ks][2], pz[2 * ks][3],
                       pz[2 * ks + 1][0], pz[2 * ks + 1][1], pz[2 * ks + 1][2], pz[2 * ks + 1][3]};
        float zv[8] = {zz[2 * ks][0], zz[2 * ks][1], zz[2 * ks][2], zz[2 * ks][3],
                       zz[2 * ks + 1][0], zz[2 * ks + 1][1], zz[2 * ks + 1][2], zz[2 * ks + 1][3]};
        const bf16x8 pa = pack_frag(pv), za = pack_frag(zv);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          adv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, frag_tr<RS>(ldsO, 32 * ks, 16 * dt, lane), adv[dt], 0, 0, 0);
          adk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(za, frag_tr<RS>(ldsQ, 32 * ks, 16 * dt, lane), adk[dt], 0, 0, 0);
        }
      }
    }
  }
  // accumulators: C[key = 16w + 4g + j][d = 16dt + c]
  if constexpr (ROPE) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int key = kt * 64 + 16 * w + 4 * g + j;
        if (key < L) {
          const int d = 16 * dt + c;
          const float cs = bf2f(((const bf16_t*)a.rope_cos)[(int64_t)key * a.rope_ld + d]);
          const float sn = bf2f(((const bf16_t*)a.rope_sin)[(int64_t)key * a.rope_ld + d]);
          float lo = adk[dt][j], hi = adk[dt + 8][j];
          rope_pair_t(lo, hi, cs, sn);
          adk[dt][j] = lo;
          adk[dt + 8][j] = hi;
        }
      }
  }
  __syncthreads();
  // stage both results as bf16 [64][DV] images, then 16-B row stores
  bf16_t* imgK = (bf16_t*)smem;
  bf16_t* imgV = imgK + 64 * DV;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 16 * w + 4 * g + j;
      imgK[r * DV + 16 * dt + c] = f2bf(adk[dt][j]);
      imgV[r * DV + 16 * dt + c] = f2bf(adv[dt][j]);
    }
  __syncthreads();
  constexpr int CPR = D / 8;
  for (int idx = t; idx < 64 * CPR; idx += 256) {
    const int r = idx / CPR, ch = idx % CPR;
    const int key = kt * 64 + r;
    if (key < L) {
      *reinterpret_cast<u32x4*>(dk + ((int64_t)b * L + key) * lddk + (int64_t)hk * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(imgK + r * DV + ch * 8);
      *reinterpret_cast<u32x4*>(dv + ((int64_t)b * L + key) * lddv + (int64_t)hk * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(imgV + r * DV + ch * 8);
    }
  }
}

// ================================================================== backward: dQ
template <int D, bool ROPE>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(svla_attn_args a, const bf16_t* __restrict__ dout,
                                                             int64_t lddo, const float* __restrict__ lse,
                                                             const float* __restrict__ delta, bf16_t* __restrict__ dq,
                                                             int64_t lddq) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16;
  constexpr int TB = 64 * RS * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + TB;
  uint8_t* lcls = (uint8_t*)(smem + 2 * TB);

  const int b = blockIdx.z, h = blockIdx.y, qt = blockIdx.x;
  const int grp = a.Hq / a.Hkv, hk = h / grp;
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int L = a.L;
  const int qi = qt * 64 + 16 * w + c;
  const bool qvalid = qi < L;
  const bf16_t* qbase = (const bf16_t*)a.q + (int64_t)b * L * a.ldq + (int64_t)h * D;
  const bf16_t* obase = dout + (int64_t)b * L * lddo + (int64_t)h * D;
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;
  const uint8_t* cls = a.kv_class ? a.kv_class + (int64_t)b * L : nullptr;

  bf16x8 qf[NKS], of[NKS];
  load_row_frags<D, ROPE>(qf, qbase + (int64_t)qi * a.ldq, qvalid, a, qi, lane);
  load_row_frags<D, false>(of, obase + (int64_t)qi * lddo, qvalid, a, qi, lane);
  const float lq = qvalid ? lse[((int64_t)b * a.Hq + h) * L + qi] : 0.f;
  const float dq_ = qvalid ? delta[((int64_t)b * a.Hq + h) * L + qi] : 0.f;

  f32x4 acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float LOG2E = 1.4426950408889634f;
  const int nkt = (L + 63) / 64;
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    stage_tile<D, ROPE>(ldsK, kbase, a.ldk, kt * 64, L, a, t);
    stage_tile<D, false>(ldsV, vbase, a.ldv, kt * 64, L, a, t);
    if (t < 64) lcls[t] = (cls && kt * 64 + t < L) ? cls[kt * 64 + t] : 0;
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = dp[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row<RS>(ldsK, 16 * nt, ks, lane), qf[ks], s[nt], 0, 0, 0);
        dp[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row<RS>(ldsV, 16 * nt, ks, lane), of[ks], dp[nt], 0, 0, 0);
      }
    }
    float zz[4][4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kl = 16 * nt + 4 * g + j, kj = kt * 64 + kl;
        float z = 0.f;
        if (qvalid && kj < L) {
          const float sc = softcap_f(s[nt][j] * a.scale, a.softcap);
          const float xv = visible(a.kv_class ? lcls : nullptr, kl, qi - kt * 64, a.sliding_window) ? sc : MASKVAL;
          const float p = exp2f((xv - lq) * LOG2E);
          const float ds = p * (dp[nt][j] - dq_);
          const float dcap = a.softcap > 0.f ? (1.0f - (sc / a.softcap) * (sc / a.softcap)) : 1.0f;
          z = ds * dcap * a.scale;
        }
        zz[nt][j] = z;
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float zv[8] = {zz[2 * ks][0], zz[2 * ks][1], zz[2 * ks][2], zz[2 * ks][3],
                     zz[2 * ks + 1][0], zz[2 * ks + 1][1], zz[2 * ks + 1][2], zz[2 * ks + 1][3]};
      const bf16x8 za = pack_frag(zv);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(za, frag_tr<RS>(ldsK, 32 * ks, 16 * dt, lane), acc[dt], 0, 0, 0);
    }
  }
  // acc: C[q = 16w + 4g + j][d = 16dt + c]
  if constexpr (ROPE) {
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = qt * 64 + 16 * w + 4 * g + j;
        if (q < L) {
          const int d = 16 * dt + c;
          const float cs = bf2f(((const bf16_t*)a.rope_cos)[(int64_t)q * a.rope_ld + d]);
          const float sn = bf2f(((const bf16_t*)a.rope_sin)[(int64_t)q * a.rope_ld + d]);
          float lo = acc[dt][j], hi = acc[dt + 8][j];
          rope_pair_t(lo, hi, cs, sn);
          acc[dt][j] = lo;
          acc[dt + 8][j] = hi;
        }
      }
  }
  __syncthreads();
  bf16_t* img = (bf16_t*)smem + w * 16 * DV;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int j = 0; j < 4; ++j) img[(4 * g + j) * DV + 16 * dt + c] = f2bf(acc[dt][j]);
  __syncthreads();
  constexpr int CPR = D / 8;
  for (int idx = lane; idx < 16 * CPR; idx += 64) {
    const int r = idx / CPR, ch = idx % CPR;
    const int q = qt * 64 + 16 * w + r;
    if (q < L)
      *reinterpret_cast<u32x4*>(dq + ((int64_t)b * L + q) * lddq + (int64_t)h * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(img + r * DV + ch * 8);
  }
}

template <auto KERN>
void set_lds_once(int bytes) {
  static bool done = false;  // one flag per kernel instantiation
  if (!done) {
    (void)hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done = true;
  }
}

int check_args(const svla_attn_args* a, bool rope) {
  SVLA_CHECK_ARG(a, "attn: args NULL");
  SVLA_CHECK_ARG(a->B > 0 && a->L > 0 && a->Hq > 0 && a->Hkv > 0 && a->Hq % a->Hkv == 0, "attn: bad B/L/H");
  SVLA_CHECK_ARG(a->D == 256 || a->D == 72, "attn: head_dim %d unsupported (256 or 72)", a->D);
  SVLA_CHECK_ARG(a->q && a->k && a->v, "attn: q/k/v NULL");
  SVLA_CHECK_ARG(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0, "attn: ld must be multiples of 8");
  SVLA_CHECK_ARG(((uintptr_t)a->q & 15) == 0 && ((uintptr_t)a->k & 15) == 0 && ((uintptr_t)a->v & 15) == 0,
                 "attn: q/k/v must be 16-B aligned");
  if (rope) SVLA_CHECK_ARG(a->D == 256 && a->rope_sin && a->rope_ld % 8 == 0, "attn: RoPE needs D=256, sin, ld%8");
  return 0;
}

}  // namespace

extern "C" int svla_attn_fwd(const svla_attn_args* a, void* out, int64_t ldo, float* lse, void* stream) {
  const bool rope = a && a->rope_cos;
  if (int rc = check_args(a, rope)) return rc;
  SVLA_CHECK_ARG(out && lse && ldo % 8 == 0, "attn_fwd: out/lse");
  dim3 grid((a->L + 63) / 64, a->Hq, a->B), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (a->D == 256) {
    const int lds = 2 * 64 * 256 * 2 + 64;
    if (rope) {
      set_lds_once<attn_fwd_kernel<256, true>>(lds);
      hipLaunchKernelGGL((attn_fwd_kernel<256, true>), grid, block, lds, s, *a, (bf16_t*)out, ldo, lse);
    } else {
      set_lds_once<attn_fwd_kernel<256, false>>(lds);
      hipLaunchKernelGGL((attn_fwd_kernel<256, false>), grid, block, lds, s, *a, (bf16_t*)out, ldo, lse);
    }
  } else {
    const int lds = 2 * 64 * 128 * 2 + 64;
    set_lds_once<attn_fwd_kernel<72, false>>(lds);
    hipLaunchKernelGGL((attn_fwd_kernel<72, false>), grid, block, lds, s, *a, (bf16_t*)out, ldo, lse);
  }
  return svla::check_launch("attn_fwd");
}

extern "C" int svla_attn_bwd(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                             const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                             float* workspace, void* stream) {
  const bool rope = a && a->rope_cos;
  if (int rc = check_args(a, rope)) return rc;
  SVLA_CHECK_ARG(out && dout && lse && dq && dk && dv && workspace, "attn_bwd: NULL buffer");
  SVLA_CHECK_ARG(ldo % 8 == 0 && lddo % 8 == 0 && lddq % 8 == 0 && lddk % 8 == 0 && lddv % 8 == 0,
                 "attn_bwd: ld must be multiples of 8");
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)a->B * a->L * a->Hq;
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, a->B, a->L, a->Hq, a->D,
                     (const bf16_t*)out, ldo, (const bf16_t*)dout, lddo, workspace);
  if (int rc = svla::check_launch("attn_delta")) return rc;
  const int nt = (a->L + 63) / 64;
  dim3 gkv(nt, a->Hkv, a->B), gq(nt, a->Hq, a->B), block(256);
  if (a->D == 256) {
    const int lds_kv = 4 * 64 * 256 * 2 + 64 * 8 + 64;
    const int lds_q = 2 * 64 * 256 * 2 + 64;
    if (rope) {
      set_lds_once<attn_bwd_dkv_kernel<256, true>>(lds_kv);
      set_lds_once<attn_bwd_dq_kernel<256, true>>(lds_q);
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<256, true>), gkv, block, lds_kv, s, *a, (const bf16_t*)dout, lddo, lse,
                         workspace, (bf16_t*)dk, lddk, (bf16_t*)dv, lddv);
      hipLaunchKernelGGL((attn_bwd_dq_kernel<256, true>), gq, block, lds_q, s, *a, (const bf16_t*)dout, lddo, lse,
                         workspace, (bf16_t*)dq, lddq);
    } else {
      set_lds_once<attn_bwd_dkv_kernel<256, false>>(lds_kv);
      set_lds_once<attn_bwd_dq_kernel<256, false>>(lds_q);
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<256, false>), gkv, block, lds_kv, s, *a, (const bf16_t*)dout, lddo, lse,
                         workspace, (bf16_t*)dk, lddk, (bf16_t*)dv, lddv);
      hipLaunchKernelGGL((attn_bwd_dq_kernel<256, false>), gq, block, lds_q, s, *a, (const bf16_t*)dout, lddo, lse,
                         workspace, (bf16_t*)dq, lddq);
    }
  } else {
    const int lds_kv = 4 * 64 * 128 * 2 + 64 * 8 + 64;
    const int lds_q = 2 * 64 * 128 * 2 + 64;
    set_lds_once<attn_bwd_dkv_kernel<72, false>>(lds_kv);
    set_lds_once<attn_bwd_dq_kernel<72, false>>(lds_q);
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<72, false>), gkv, block, lds_kv, s, *a, (const bf16_t*)dout, lddo, lse,
                       workspace, (bf16_t*)dk, lddk, (bf16_t*)dv, lddv);
    hipLaunchKernelGGL((attn_bwd_dq_kernel<72, false>), gq, block, lds_q, s, *a, (const bf16_t*)dout, lddo, lse,
                       workspace, (bf16_t*)dq, lddq);
  }
  return svla::check_launch("attn_bwd");
}
