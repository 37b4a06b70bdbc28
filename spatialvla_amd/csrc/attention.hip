// Fused prefix-LM GQA attention with logit softcap (Gemma2, head_dim 256; RoPE transpose in the backward) and
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
//  * RoPE (rotate_half, modeling_gemma2.py:123-154) is not applied here on the way in: q / k arrive rotated
//    (the QKV GEMM's SVLA_EPI_ROPE epilogue).  The backward applies its transpose to dQ / dK in the accumulators
//    before the store, so the gradients leave w.r.t. the pre-rotation q / k.
//  * Backward is two deterministic kernels (dQ per query tile, which also forms delta = rowsum(dO * O); then dK/dV
//    per key tile looping over the GQA query heads) — no float atomics.
#include <atomic>
#include <type_traits>

#include "svla_common.h"

#ifndef SVLA_ATT_QW
#define SVLA_ATT_QW 2  // query sub-tiles per wave of the forward at head_dim 64 / 72 (variant builds: 1)
#endif
#ifndef SVLA_ATT_RS64
#define SVLA_ATT_RS64 1  // head_dim 64 (BEiT) tiles with 128-B rows (16 KB K+V stages, 32 KB per block) instead of 256-B:
                         // BEiT B=32 forward 157.5 -> 137.6 us with bias, 123 -> 86 us without (bitwise equal outputs;
                         // tools/beit_attn_probe.py, profiles/r3o_beit_attn_ab.txt)
#endif
#ifndef SVLA_ATT_WPE64
#define SVLA_ATT_WPE64 2  // head_dim 64 forward with SVLA_ATT_RS64: waves per SIMD the registers are sized for (3: spills
                          // 12 VGPRs, 165 us)
#endif
#ifndef SVLA_ATT_BPF
#define SVLA_ATT_BPF 1  // key tiles of score bias (BEiT) in flight ahead of the tile being scored: 1 or 2 (2: 245-261 us)
#endif
#ifndef SVLA_ATT_SUBWAVE
#define SVLA_ATT_SUBWAVE 1  // sub-wave forward grids take the variant with twice the workgroups (svla_attn_fwd)
#endif
#ifndef SVLA_ATT_QW256
#define SVLA_ATT_QW256 1  // head_dim 256 forward: 1 = head pairs (NH 2), 16 queries per wave; 2 = one head, 32 per wave
#endif

namespace {

constexpr float MASKVAL = -3.3895313892515355e38f;  // torch.finfo(bfloat16).min

template <int D> struct Cfg;
template <> struct Cfg<256> { static constexpr int DP = 256, DV = 256, RS = 256; };
template <> struct Cfg<72>  { static constexpr int DP = 96,  DV = 80,  RS = 128; };
template <> struct Cfg<64>  { static constexpr int DP = 64,  DV = 64,  RS = SVLA_ATT_RS64 ? 64 : 128; };  // BEiT (ZoeDepth)

// chunk swizzle of row r: 2(r & 7) for 256-B and wider rows, r & 7 for the 128-B rows of head_dim 64 (8 chunks);
// both conflict-free for the ds_read_b128 row reads and the ds_read_b64_tr_b16 transposed reads, and periodic in 8
// rows (TrFrag reads rows r and r + 16 with one swizzle)
template <int RS>
__device__ __forceinline__ int swz(int r) {
  return RS == 64 ? (r & 7) : ((r & 7) << 1);
}
// byte offset of 16-B chunk `ch` of row `r` in a [64][RS] bf16 LDS tile
template <int RS>
__device__ __forceinline__ int toff(int r, int ch) {
  return r * RS * 2 + ((ch ^ swz<RS>(r)) << 4);
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

// transpose of rope_pair (gradient): dlo = dlo'*c + dhi'*s, dhi = dhi'*c - dlo'*s
__device__ __forceinline__ void rope_pair_t(float& lo, float& hi, float c, float s) {
  float a = lo, b = hi;
  lo = a * c + b * s;
  hi = b * c - a * s;
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA staging of a [ROWS][RS] tile (rows row0.. of a (b, ·, head) slice, D valid columns) into the
// swizzled image toff<RS>: wave-instruction j writes 1 KiB lane-linearly (RPI = 512/RS rows); lane l lands at
// row j*RPI + l/CPR, image chunk p = l%CPR, which holds global chunk p ^ swz<RS>(row).  Rows >= nrows and
// columns >= D read as zero (descriptor range check).
template <int RS, int ROWS, int NW>
__device__ __forceinline__ void glds_tile(char* lds, const bf16_t* base, int64_t ld, int nrows, int D, int w,
                                          int lane) {
  constexpr int CPR = RS / 8, RPI = 1024 / (2 * RS), NI = ROWS * RS * 2 / 1024;
  static_assert(NI % NW == 0, "tile instructions must split evenly over the waves");
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(base);
#pragma unroll
  for (int i = 0; i < NI / NW; ++i) {
    const int j = w + NW * i;
    const int r = j * RPI + lane / CPR;
    const int ch = (lane % CPR) ^ swz<RS>(r);
    const uint32_t voff = (r < nrows && ch * 8 < D) ? (uint32_t)(r * ld * 2 + ch * 16) : SVLA_OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(lds + j * 1024), 16, voff, 0, 0, 0);
  }
}

// transposed fragment via inline-asm ds_read_b64_tr_b16 (through the builtin, hipcc drains every LDS-DMA in
// flight before it, which would serialise the prefetch); same element map as frag_tr.  Issue a batch with
// load(), then tr_wait(), then get(): the pair is assembled only after the data landed.
struct TrFrag {
  u32x2 lo, hi;
  template <int RS>
  __device__ __forceinline__ void load(const char* lds, int rb, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = c0 + 4 * p;
    const int r1 = rb + 4 * g + q;  // r1 + 16 has the same swizzle ((r & 7) unchanged)
    const uint32_t a1 = (uint32_t)(uintptr_t)(const LDS_AS char*)(lds + toff<RS>(r1, col >> 3) + (col & 7) * 2);
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:%3"
                 : "=&v"(lo), "=v"(hi)
                 : "v"(a1), "i"(16 * RS * 2));
  }
  __device__ __forceinline__ bf16x8 get() const {
    const u32x4 r = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, r);
  }
};
__device__ __forceinline__ void tr_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// acc[dt] += A(dt) * B over NDT d-tiles, A read transposed from LDS in batches of 4 fragments, double-buffered:
// batch i+1's 8 transpose reads are issued before batch i's MFMAs (lgkmcnt(8) waits for batch i only), so the LDS
// latency of a batch hides behind the previous batch's MFMAs instead of stalling every batch.
// AT_A: the LDS operand is the MFMA A operand (else B)
template <int RS, int NDT, bool AT_A>
__device__ __forceinline__ void mfma_tr_sweep(f32x4 (&acc)[NDT], const char* lds, int rb, bf16x8 other, int lane) {
  constexpr int CH = 4, NB = (NDT + CH - 1) / CH;
  TrFrag f[2][CH];
#pragma unroll
  for (int i = 0; i < CH; ++i)
    if (i < NDT) f[0][i].template load<RS>(lds, rb, 16 * i, lane);
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    const int d0 = bi * CH;
    if (bi + 1 < NB) {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        if (d0 + CH + i < NDT) f[(bi + 1) & 1][i].template load<RS>(lds, rb, 16 * (d0 + CH + i), lane);
      if (NDT - (d0 + CH) >= CH) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      if (d0 + i < NDT) {
        if (AT_A) acc[d0 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[bi & 1][i].get(), other, acc[d0 + i], 0, 0, 0);
        else acc[d0 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(other, f[bi & 1][i].get(), acc[d0 + i], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Per-lane register fragments of one row (the lane's query): f[ks] = X[row][32ks + 8g + j]
template <int D>
__device__ __forceinline__ void load_row_frags(bf16x8 (&f)[Cfg<D>::DP / 32], const bf16_t* rowp, bool valid,
                                               int lane) {
  constexpr int NKS = Cfg<D>::DP / 32;
  const int g = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int d = 32 * ks + 8 * g;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (valid && d < D) v = *reinterpret_cast<const u32x4*>(rowp + d);
    f[ks] = __builtin_bit_cast(bf16x8, v);
  }
}

__device__ __forceinline__ bool visible(int c, int kj, int qi, int window) {
  bool v = (c == 0) || (c == 1 && kj <= qi);
  if (window > 0 && qi - kj >= window) v = false;
  return v;
}

__device__ __forceinline__ float softcap_f(float z, float cap) { return cap > 0.f ? cap * fast_tanh(z / cap) : z; }

// key classes of the whole sequence -> LDS (plain loads, before any LDS-DMA is in flight)
__device__ __forceinline__ void load_classes(uint8_t* lcls, const uint8_t* cls, int L, int t, int nth) {
  for (int i = t; i < L; i += nth) lcls[i] = cls ? cls[i] : 0;
}

template <int D>
constexpr int tile_bytes(int rows) { return rows * Cfg<D>::RS * 2; }

// Softcapped scores without a running max (CAP): t = cap*tanh(s*scale/cap) lies in (-cap, cap), so p = exp(t)
// stays a normal fp32 / bf16 number (Gemma2: cap 50, e^50 = 5e21) and the softmax needs neither the row max nor
// the rescale of the output accumulators.  With r = 1/(1 + 2^(s*c2)), tanh = 1 - 2r and
//   p = 2^(C0 + C1*r),  c2 = 2*scale*log2(e)/cap,  C0 = cap*log2(e),  C1 = -2*cap*log2(e)
// -- two v_exp_f32 and one v_rcp_f32 per score.  A masked key gets p = 2^-120 instead of 0: at least one visible
// key contributes >= e^-cap = 2e-22, so masked keys weigh < 1e-14 of a row, and a row with no visible key
// becomes uniform over all keys, as the reference's softmax over equal finfo.min logits does.
struct CapExp {
  float c2, C0, C1;
  __device__ __forceinline__ CapExp(float scale, float cap) {
    const float LOG2E = 1.4426950408889634f;
    c2 = 2.f * scale * LOG2E / cap;
    C0 = cap * LOG2E;
    C1 = -2.f * cap * LOG2E;
  }
  __device__ __forceinline__ float r(float s) const { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(s * c2)); }
  // log2 of p = exp(t), given r
  __device__ __forceinline__ float lg2p(float r) const { return fmaf(C1, r, C0); }
};
constexpr float MASKED_LG2P = -120.f;
constexpr float MASKED_P = 0x1p-120f;  // exp2(MASKED_LG2P)

// every key of the 64-key tile at k0 is in range and visible to every query (class 0, no effective window):
// the per-score mask test can be skipped (wave-uniform; one LDS byte per lane)
__device__ __forceinline__ bool tile_plain(const uint8_t* lcls, int k0, int L, bool window_free, int lane) {
  const int kj = k0 + lane;
  const bool ok = kj < L && lcls[kj] == 0;
  return window_free && __ballot(ok) == ~0ull;
}

// blocks of one (batch, head group) are consecutive logical ids; xcd_remap puts consecutive ids on one XCD so the
// query tiles sharing a K/V stream share that XCD's L2
__device__ __forceinline__ void block_coords(int nqt, int nhg, int& qt, int& hg, int& b) {
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  qt = id % nqt;
  hg = (id / nqt) % nhg;
  b = id / (nqt * nhg);
}

// ================================================================== forward
// Block = (query tile of 64*QW, NH query heads sharing one kv head, batch); 4 waves per head, each wave QW sub-tiles
// of 16 queries (sub-tile u: queries 64u + 16wq + c of the block's tile).  Every K / V fragment read from LDS feeds
// QW MFMAs (QW = 2 for the short head dims, where one fragment per MFMA left the kernel LDS-bound).
// K/V tiles stream through two LDS stages by LDS-DMA: tile kt+1 lands while tile kt is consumed.
// acc[u][dt] += V(dt)^T * P_u^T over NDT d-tiles: the V fragment (transpose read, batches of 4 double-buffered as
// mfma_tr_sweep) is loaded once and multiplied into every sub-tile.
template <int RS, int NDT, int QW>
__device__ __forceinline__ void mfma_tr_sweep_q(f32x4 (&acc)[QW][NDT], const char* lds, int rb, const bf16x8 (&pb)[QW],
                                                int lane) {
  constexpr int CH = 4, NB = (NDT + CH - 1) / CH;
  TrFrag f[2][CH];
#pragma unroll
  for (int i = 0; i < CH; ++i)
    if (i < NDT) f[0][i].template load<RS>(lds, rb, 16 * i, lane);
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    const int d0 = bi * CH;
    if (bi + 1 < NB) {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        if (d0 + CH + i < NDT) f[(bi + 1) & 1][i].template load<RS>(lds, rb, 16 * (d0 + CH + i), lane);
      if (NDT - (d0 + CH) >= CH) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < CH; ++i)
      if (d0 + i < NDT) {
        const bf16x8 v = f[bi & 1][i].get();
#pragma unroll
        for (int u = 0; u < QW; ++u)
          acc[u][d0 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(v, pb[u], acc[u][d0 + i], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int D, int NH, bool CAP, bool BIAS = false, int QW = 1>
__global__ __launch_bounds__(256 * NH, (D == 64 && SVLA_ATT_RS64) ? SVLA_ATT_WPE64 : 1) void attn_fwd_kernel(svla_attn_args a, bf16_t* __restrict__ out,
                                                               int64_t ldo, float* __restrict__ lse) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16, NW = 4 * NH, QT = 64 * QW;
  constexpr int TB = tile_bytes<D>(64), STAGE = 2 * TB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* lcls = (uint8_t*)(smem + 2 * STAGE);

  const int L = a.L;
  int qt, hg, b;
  block_coords((L + QT - 1) / QT, a.Hq / NH, qt, hg, b);
  const int t = threadIdx.x, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = hg * NH + (w >> 2), wq = w & 3;
  const int grp = a.Hq / a.Hkv, hk = h / grp;
  int qi[QW];
  bool qvalid[QW];
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    qi[u] = qt * QT + 64 * u + 16 * wq + c;
    qvalid[u] = qi[u] < L;
  }
  const bool window_free = a.sliding_window <= 0 || a.sliding_window >= L;

  const bf16_t* qbase = (const bf16_t*)a.q + (int64_t)b * L * a.ldq + (int64_t)h * D;
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;

  load_classes(lcls, a.kv_class ? a.kv_class + (int64_t)b * L : nullptr, L, t, 64 * NW);
  bf16x8 qf[QW][NKS];
#pragma unroll
  for (int u = 0; u < QW; ++u) load_row_frags<D>(qf[u], qbase + (int64_t)qi[u] * a.ldq, qvalid[u], lane);
  const int nkt = (L + 63) / 64;
  glds_tile<RS, 64, NW>(smem, kbase, a.ldk, L, D, w, lane);
  glds_tile<RS, 64, NW>(smem + TB, vbase, a.ldv, L, D, w, lane);
  // BIAS: this lane's bias rows (its queries) are read one key tile ahead into registers (keys 16nt + 4g .. +3 of
  // the tile; 8 B per nt, zero beyond the padded row): the loads of tile kt+1 are in flight during tile kt
  // (SVLA_ATT_BPF = 2: two tiles ahead, in a ring of two register sets)
  const bf16_t* brow[QW];
  u32x2 bnext[SVLA_ATT_BPF][QW][4];
  auto bias_fetch = [&](int kt_, auto bslot) {
    constexpr int BS = decltype(bslot)::value;
#pragma unroll
    for (int u = 0; u < QW; ++u)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int k = kt_ * 64 + 16 * nt + 4 * g;
        bnext[BS][u][nt] = k < a.bias_ld ? *reinterpret_cast<const u32x2*>(brow[u] + k) : u32x2{0u, 0u};
      }
  };
  if constexpr (BIAS) {
#pragma unroll
    for (int u = 0; u < QW; ++u)
      brow[u] = (const bf16_t*)a.bias + ((int64_t)h * L + (qvalid[u] ? qi[u] : 0)) * a.bias_ld;
    bias_fetch(0, std::integral_constant<int, 0>{});
    if constexpr (SVLA_ATT_BPF == 2) bias_fetch(1, std::integral_constant<int, 1>{});
  }

  f32x4 acc[QW][NDT];
  float m[QW], l[QW];
#pragma unroll
  for (int u = 0; u < QW; ++u) {
#pragma unroll
    for (int i = 0; i < NDT; ++i) acc[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[u] = -INFINITY;
    l[u] = 0.f;
  }
  const float LOG2E = 1.4426950408889634f;
  const CapExp ce(a.scale, CAP ? a.softcap : 1.f);

  // one key tile; SL = kt % SVLA_ATT_BPF as a constant (the bias register ring is indexed statically)
  auto tile = [&](const int kt, auto slot) {
    constexpr int SL = decltype(slot)::value;
    // tile kt landed (and, BIAS with BPF 2, the bias of tile kt: only the QW*4 loads of tile kt+1 may stay in flight)
    if (BIAS && SVLA_ATT_BPF == 2 && kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QW * 4) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile kt landed for every wave; every wave is done with the stage refilled below
    const char* ldsK = smem + (kt & 1) * STAGE;
    const char* ldsV = ldsK + TB;
    if (kt + 1 < nkt) {
      char* nx = smem + ((kt + 1) & 1) * STAGE;
      const int r0 = (kt + 1) * 64;
      glds_tile<RS, 64, NW>(nx, kbase + (int64_t)r0 * a.ldk, a.ldk, L - r0, D, w, lane);
      glds_tile<RS, 64, NW>(nx + TB, vbase + (int64_t)r0 * a.ldv, a.ldv, L - r0, D, w, lane);
    }
    const bool plain = tile_plain(lcls, kt * 64, L, window_free, lane);
    f32x4 s[QW][4];
    {  // K fragments of k-step ks+1 are read while k-step ks multiplies (double-buffered)
      bf16x8 kb[2][4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
        for (int u = 0; u < QW; ++u) s[u][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
        kb[0][nt] = frag_row<RS>(ldsK, 16 * nt, 0, lane);
      }
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks + 1 < NKS) {
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) kb[(ks + 1) & 1][nt] = frag_row<RS>(ldsK, 16 * nt, ks + 1, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int u = 0; u < QW; ++u)
            s[u][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb[ks & 1][nt], qf[u][ks], s[u][nt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float bb[QW][4][4];  // additive score bias (BEiT relative position bias), rows qi[u], keys 16nt + 4g + j
    if constexpr (BIAS) {
#pragma unroll
      for (int u = 0; u < QW; ++u)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const u32x2 w2 = bnext[SL][u][nt];
          bb[u][nt][0] = __uint_as_float(w2[0] << 16); bb[u][nt][1] = __uint_as_float(w2[0] & 0xffff0000u);
          bb[u][nt][2] = __uint_as_float(w2[1] << 16); bb[u][nt][3] = __uint_as_float(w2[1] & 0xffff0000u);
        }
      if (kt + SVLA_ATT_BPF < nkt) bias_fetch(kt + SVLA_ATT_BPF, slot);
    }
    bf16x8 pb[2][QW];  // P of key halves 0 / 1 (the B operands of the PV products)
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      float p[4][4];
      if constexpr (CAP) {
        float ps = 0.f;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float e = ce.lg2p(ce.r(s[u][nt][j]));
            if (!plain) {
              const int kj = kt * 64 + 16 * nt + 4 * g + j;
              if (!visible(lcls[kj], kj, qi[u], a.sliding_window)) e = MASKED_LG2P;
              if (kj >= L) e = -INFINITY;
            }
            p[nt][j] = __builtin_amdgcn_exp2f(e);
            ps += p[nt][j];
          }
        l[u] += ps;
      } else {
        float x[4][4];
        float mt = -INFINITY;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float v = s[u][nt][j] * (a.scale * LOG2E);  // log2 domain
            if constexpr (BIAS) v = fmaf(bb[u][nt][j], LOG2E, v);
            if (!plain) {
              const int kj = kt * 64 + 16 * nt + 4 * g + j;
              if (kj >= L) v = -INFINITY;
              else if (!visible(lcls[kj], kj, qi[u], a.sliding_window)) v = MASKVAL;
            }
            x[nt][j] = v;
            mt = fmaxf(mt, v);
          }
        mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
        mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
        const float mnew = fmaxf(m[u], mt);
        const float alpha = __builtin_amdgcn_exp2f(m[u] - mnew);  // m=-inf -> 0
        float ps = 0.f;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            p[nt][j] = __builtin_amdgcn_exp2f(x[nt][j] - mnew);
            ps += p[nt][j];
          }
        l[u] = l[u] * alpha + ps;
        m[u] = mnew;
#pragma unroll
        for (int i = 0; i < NDT; ++i) acc[u][i] *= alpha;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        float pv[8] = {p[2 * ks][0], p[2 * ks][1], p[2 * ks][2], p[2 * ks][3],
                       p[2 * ks + 1][0], p[2 * ks + 1][1], p[2 * ks + 1][2], p[2 * ks + 1][3]};
        pb[ks][u] = pack_frag(pv);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) mfma_tr_sweep_q<RS, NDT, QW>(acc, ldsV, 32 * ks, pb[ks], lane);
  };
  for (int kt = 0; kt < nkt; kt += SVLA_ATT_BPF) {
    tile(kt, std::integral_constant<int, 0>{});
    if constexpr (SVLA_ATT_BPF == 2)
      if (kt + 1 < nkt) tile(kt + 1, std::integral_constant<int, SVLA_ATT_BPF - 1>{});
  }
  // O^T accumulators (d = 16dt + 4g + j, q = lane col) -> per-wave LDS image [QW*16 q][DV + 16] -> 16-B stores.
  // The 16-element row pad puts the 16 query rows of one 8-B store 32 B apart (an unpadded DV = 256 row stride
  // maps all 16 onto the same two banks: a 16-way conflict on every store).
  constexpr int IS = DV + 16;
  __syncthreads();
  bf16_t* img = (bf16_t*)(smem) + w * QW * 16 * IS;
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    float lu = l[u];
    lu += __shfl_xor(lu, 16, 64);
    lu += __shfl_xor(lu, 32, 64);
    const float inv = 1.0f / lu;
    // natural-log lse of the scores (CAP: of p = exp(t) directly; else of the max-shifted log2-domain sum)
    if (qvalid[u] && g == 0) lse[((int64_t)b * a.Hq + h) * L + qi[u]] = CAP ? __logf(lu) : (m[u] + __log2f(lu)) / LOG2E;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      uint32_t lo = pack2(acc[u][dt][0] * inv, acc[u][dt][1] * inv), hi = pack2(acc[u][dt][2] * inv, acc[u][dt][3] * inv);
      *reinterpret_cast<u32x2*>(img + (16 * u + c) * IS + 16 * dt + 4 * g) = u32x2{lo, hi};
    }
  }
  __syncthreads();
  constexpr int CPR = D / 8;  // 16-B chunks per output row
  for (int idx = lane; idx < QW * 16 * CPR; idx += 64) {
    const int r = idx / CPR, ch = idx % CPR;
    const int q = qt * QT + 64 * (r >> 4) + 16 * wq + (r & 15);
    if (q < L)
      *reinterpret_cast<u32x4*>(out + ((int64_t)b * L + q) * ldo + (int64_t)h * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(img + r * IS + ch * 8);
  }
}

// transpose of rotate_half RoPE on a [rows x 16dt+c] accumulator layout (lo half dt < 8, hi half dt + 8)
template <int NDT>
__device__ __forceinline__ void rope_t_acc(f32x4 (&acc)[NDT], const svla_attn_args& a, int row0, int L, int g,
                                           int c) {
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = row0 + 4 * g + j;
      if (row < L) {
        const int d = 16 * dt + c;
        const float cs = bf2f(((const bf16_t*)a.rope_cos)[(int64_t)row * a.rope_ld + d]);
        const float sn = bf2f(((const bf16_t*)a.rope_sin)[(int64_t)row * a.rope_ld + d]);
        float lo = acc[dt][j], hi = acc[dt + 8][j];
        rope_pair_t(lo, hi, cs, sn);
        acc[dt][j] = lo;
        acc[dt + 8][j] = hi;
      }
    }
}

// Per-score backward factor z = dS * dt/ds * scale (the softcap chain rule), for the score s (raw dot product)
// of a query with log2-domain lse2 and delta, or 0 when out of range.  Same p as the forward (CapExp, masked keys
// at 2^-120 of the row scale).
template <bool CAP>
__device__ __forceinline__ float score_grad(float s, float dp, float lse2, float delta, bool masked, const CapExp& ce,
                                            float scale) {
  const float LOG2E = 1.4426950408889634f;
  if constexpr (CAP) {
    const float r = ce.r(s);
    const float p = __builtin_amdgcn_exp2f((masked ? MASKED_LG2P : ce.lg2p(r)) - lse2);
    return p * (dp - delta) * (4.f * r * (1.f - r)) * scale;  // d tanh = 1 - (1 - 2r)^2
  } else {
    const float p = __builtin_amdgcn_exp2f((masked ? MASKVAL : s * (scale * LOG2E)) - lse2);
    return p * (dp - delta) * scale;
  }
}

// ================================================================== backward: dK, dV
// Block = (key tile of 64, kv head, batch), 4 waves x 16 keys.  Each wave keeps the K rows of its keys in
// registers (the B operand of S for every query) and reads its V rows from the block's LDS V tile.  The query
// heads of the group and their 32-row Q / dO tiles stream through one LDS stage by LDS-DMA (a co-resident block
// covers the load); lse / delta of the group's heads and the key classes are preloaded to LDS.  ~70 KiB of LDS: two blocks per CU where registers allow
// (D=72; at D=256 the K-row registers plus both accumulators need more than 256 VGPRs).
template <int D, bool ROPE, bool CAP, bool DS = false>
__global__ __launch_bounds__(256, D == 256 ? 1 : 2) void attn_bwd_dkv_kernel(svla_attn_args a, const bf16_t* __restrict__ dout,
                                                              int64_t lddo, const float* __restrict__ lse,
                                                              const float* __restrict__ delta, bf16_t* __restrict__ dk,
                                                              int64_t lddk, bf16_t* __restrict__ dv, int64_t lddv,
                                                              bf16_t* __restrict__ dsT = nullptr) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16;
  constexpr int TB = tile_bytes<D>(64), QB = tile_bytes<D>(32);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsV = smem;
  char* const ldsQ2 = smem + TB;  // two stages of {Q [32][RS], dO [32][RS]}: step+1 lands while step is consumed
  const int L = a.L, LP = (L + 35) / 32 * 32;  // lse/delta row stride: every 32-query tile in range
  const int grp = a.Hq / a.Hkv;
  float* llse = (float*)(ldsQ2 + 4 * QB);  // [grp][LP], log2 domain
  float* ldel = llse + grp * LP;
  uint8_t* lcls = (uint8_t*)(ldel + grp * LP);

  int kt, hk, b;
  block_coords((L + 63) / 64, a.Hkv, kt, hk, b);
  const int t = threadIdx.x, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;
  const float LOG2E = 1.4426950408889634f;

  load_classes(lcls, a.kv_class ? a.kv_class + (int64_t)b * L : nullptr, L, t, 256);
  for (int i = t; i < grp * LP; i += 256) {
    const int hh = i / LP, q = i % LP;
    const int64_t o = ((int64_t)b * a.Hq + hk * grp + hh) * L + q;
    llse[i] = q < L ? lse[o] * LOG2E : 0.f;
    ldel[i] = q < L ? delta[o] : 0.f;
  }
  const int r0 = kt * 64;
  const int kl = 16 * w + c;  // this lane's key (local)
  const int kj = r0 + kl;
  bf16x8 kf[NKS];
  load_row_frags<D>(kf, kbase + (int64_t)kj * a.ldk, kj < L, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // classes visible to tile_plain
  const int kcls = kj < L ? lcls[kj] : 3;  // this lane's key class (3: beyond L)
  const bool window_free = a.sliding_window <= 0 || a.sliding_window >= L;
  const bool keys_plain = window_free && __ballot(kcls != 0) == 0ull;  // the wave's 16 keys: all in range, class 0
  glds_tile<RS, 64, 4>(ldsV, vbase + (int64_t)r0 * a.ldv, a.ldv, L - r0, D, w, lane);

  const int nqt = (L + 31) / 32, nsteps = grp * nqt;
  auto issue_q = [&](int step, char* dst) {
    const int hh = step / nqt, q0 = (step % nqt) * 32;
    const int h = hk * grp + hh;
    const bf16_t* qb = (const bf16_t*)a.q + ((int64_t)b * L + q0) * a.ldq + (int64_t)h * D;
    const bf16_t* ob = dout + ((int64_t)b * L + q0) * lddo + (int64_t)h * D;
    glds_tile<RS, 32, 4>(dst, qb, a.ldq, L - q0, D, w, lane);
    glds_tile<RS, 32, 4>(dst + QB, ob, lddo, L - q0, D, w, lane);
  };

  f32x4 adk[NDT], adv[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) adk[i] = adv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const CapExp ce(a.scale, CAP ? a.softcap : 1.f);

  issue_q(0, ldsQ2);
  for (int step = 0; step < nsteps; ++step) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage step&1 landed everywhere; every wave is done with step-1 (its stage is free)
    if (step + 1 < nsteps) issue_q(step + 1, ldsQ2 + ((step + 1) & 1) * 2 * QB);
    const char* const ldsQ = ldsQ2 + (step & 1) * 2 * QB;
    const char* const ldsO = ldsQ + QB;
    const int hh = step / nqt, q0 = (step % nqt) * 32;
    const float* sl = llse + hh * LP;
    const float* sd = ldel + hh * LP;
    f32x4 s[2], dp[2];
    {  // Q / dO / V fragments of k-step ks+1 are read while k-step ks multiplies (double-buffered)
      bf16x8 qb[2][2], ob[2][2], vb[2];
      auto ld = [&](int ks, int bf) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          qb[bf][mt] = frag_row<RS>(ldsQ, 16 * mt, ks, lane);
          ob[bf][mt] = frag_row<RS>(ldsO, 16 * mt, ks, lane);
        }
        vb[bf] = frag_row<RS>(ldsV, 16 * w, ks, lane);
      };
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) s[mt] = dp[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
      ld(0, 0);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks + 1 < NKS) ld(ks + 1, (ks + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          s[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qb[ks & 1][mt], kf[ks], s[mt], 0, 0, 0);
          dp[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ob[ks & 1][mt], vb[ks & 1], dp[mt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // element (mt, j): query q0 + 16mt + 4g + j, key = lane col (kl)
    float pv[8], zv[8];
    // wave-uniform fast path: every key of the wave visible to every query (class 0, no effective window) and all
    // 32 queries in range -- no per-score mask test (the prefix keys of the Gemma2 training mask, 299 of 312)
    const bool plain = keys_plain && q0 + 32 <= L;
    auto scores = [&](auto PLAIN) {
      constexpr bool PL = decltype(PLAIN)::value;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(sl + q0 + 16 * mt + 4 * g);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(sd + q0 + 16 * mt + 4 * g);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qi = q0 + 16 * mt + 4 * g + j;
          const bool live = PL || (qi < L && kcls != 3);
          const bool masked = !PL && !visible(kcls, kj, qi, a.sliding_window);
          float p, z;
          if constexpr (CAP) {
            const float r = ce.r(s[mt][j]);
            p = __builtin_amdgcn_exp2f((masked ? MASKED_LG2P : ce.lg2p(r)) - l4[j]);
            z = p * (dp[mt][j] - d4[j]) * (4.f * r * (1.f - r)) * a.scale;
          } else {
            p = __builtin_amdgcn_exp2f((masked ? MASKVAL : s[mt][j] * (a.scale * LOG2E)) - l4[j]);
            z = p * (dp[mt][j] - d4[j]) * a.scale;
          }
          pv[4 * mt + j] = live ? p : 0.f;
          zv[4 * mt + j] = live ? z : 0.f;
        }
      }
    };
    if (plain) scores(std::true_type{});
    else scores(std::false_type{});
    const bf16x8 pa = pack_frag(pv), za = pack_frag(zv);
    if constexpr (DS) {  // dS^T[b][h][key][q]: this lane's key, queries q0 + 16mt + 4g .. +3 (8 B each)
      const int LPK = (L + 63) / 64 * 64;
      const u32x4 zw = __builtin_bit_cast(u32x4, za);
      bf16_t* dst = dsT + (((int64_t)b * a.Hq + hk * grp + hh) * LPK + kj) * LPK + q0 + 4 * g;
      *reinterpret_cast<uint64_t*>(dst) = (uint64_t)zw[0] | ((uint64_t)zw[1] << 32);
      *reinterpret_cast<uint64_t*>(dst + 16) = (uint64_t)zw[2] | ((uint64_t)zw[3] << 32);
    }
    mfma_tr_sweep<RS, NDT, false>(adv, ldsO, 0, pa, lane);
    mfma_tr_sweep<RS, NDT, false>(adk, ldsQ, 0, za, lane);
  }
  // accumulators: C[key = 16w + 4g + j][d = 16dt + c]
  if constexpr (ROPE) rope_t_acc<NDT>(adk, a, r0 + 16 * w, L, g, c);
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
    const int key = r0 + r;
    if (key < L) {
      *reinterpret_cast<u32x4*>(dk + ((int64_t)b * L + key) * lddk + (int64_t)hk * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(imgK + r * DV + ch * 8);
      *reinterpret_cast<u32x4*>(dv + ((int64_t)b * L + key) * lddv + (int64_t)hk * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(imgV + r * DV + ch * 8);
    }
  }
}

// ================================================================== backward with stored dS (head_dim 256)
// delta = rowsum(dO * O) per (b, h, q) row, one wave a row (the dS path runs it before dK/dV, which needs it).
// head_dim 256: 32 lanes x 16 B a row, two rows a wave, eight a block.
__global__ __launch_bounds__(256) void attn_delta_kernel(int B, int L, int H, const bf16_t* __restrict__ o,
                                                         int64_t ldo, const bf16_t* __restrict__ dout, int64_t lddo,
                                                         float* __restrict__ delta) {
  constexpr int D = 256;
  const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);  // (b, q, h) rows
  const int l32 = threadIdx.x & 31;
  const bool ok = row < (int64_t)B * L * H;
  const int64_t rw = ok ? row : 0;
  const int h = (int)(rw % H);
  const int64_t bq = rw / H;
  const int q = (int)(bq % L), b = (int)(bq / L);
  float x[8], y[8];
  unpack8(*reinterpret_cast<const u32x4*>(o + bq * ldo + (int64_t)h * D + 8 * l32), x);
  unpack8(*reinterpret_cast<const u32x4*>(dout + bq * lddo + (int64_t)h * D + 8 * l32), y);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j] * y[j];
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);  // within the 32-lane half
  if (l32 == 0 && ok) delta[((int64_t)b * H + h) * L + q] = s;
}

// dQ = dS K from the dS^T tiles the dK/dV kernel stored ([b][h][key][query], bf16, rows and columns padded to 64):
// no second recompute of S, P and dP.  Block = (query tile of 64, query head, batch), 4 waves x 16 queries; per
// 64-key tile the K rows (LDS-DMA) and the dS^T tile go to LDS, and each wave multiplies its 16 queries' dS (the A
// operand, in the dQ kernel's key order) into the K rows by mfma_tr_sweep, as attn_bwd_dq_kernel does with dS it
// recomputes.  Epilogue: RoPE transpose, bf16 rows.
// Padded query columns: when L % 64 is 1..32 the dK/dV kernel writes dS^T only up to query round32(L), so columns
// round32(L)..round64(L)-1 of the workspace hold whatever the allocator left there (possibly NaN patterns).  Query
// column q of dS^T feeds only output row q of dQ (it is the A operand's row), and rows q >= L are never stored (the
// q < L test of the epilogue), so those columns cannot reach a result; no zero-fill is needed.
// LDS row pitch of the dS^T tile (bf16): the A-operand reads take keys 4g + j (g = lane >> 4) of 16 queries, i.e.
// rows 4 apart; at a 64-element (128-B) pitch those four rows share one 8-bank span (4-way conflicts, 21.7 % of the
// kernel's LDS cycles, profiles/r5b_block_pmc.txt); at 72 (144 B) rows 4g start 16g banks apart: conflict-free,
// and rows stay 16-B aligned for the tile's b128 writes
#ifndef SVLA_DQ_DS_PITCH
#define SVLA_DQ_DS_PITCH 72
#endif
template <bool ROPE>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_ds_kernel(svla_attn_args a, const bf16_t* __restrict__ dsT,
                                                                bf16_t* __restrict__ dq, int64_t lddq) {
  constexpr int D = 256, RS = Cfg<256>::RS, DV = Cfg<256>::DV, NDT = DV / 16;
  constexpr int TB = tile_bytes<D>(64), SB = 64 * 64 * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int L = a.L, LPK = (L + 63) / 64 * 64;
  int qt, h, b;
  block_coords(LPK / 64, a.Hq, qt, h, b);
  const int t = threadIdx.x, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int hk = h / (a.Hq / a.Hkv);
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* sbase = dsT + ((int64_t)b * a.Hq + h) * LPK * LPK + qt * 64;
  // one stage (40 KB, several blocks a CU): a double-buffered version (80 KB) ran 52 vs 46 us per layer
  const bf16_t* ls = (const bf16_t*)(smem + TB);
  f32x4 acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < LPK / 64; ++kt) {
    __syncthreads();  // the previous tile is consumed
    glds_tile<RS, 64, 4>(smem, kbase + (int64_t)kt * 64 * a.ldk, a.ldk, L - kt * 64, D, w, lane);
    u32x4 sv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + 256 * u, r = i >> 3, ch = i & 7;
      sv[u] = *reinterpret_cast<const u32x4*>(sbase + (int64_t)(kt * 64 + r) * LPK + ch * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + 256 * u, r = i >> 3, ch = i & 7;
      *reinterpret_cast<u32x4*>(smem + TB + (r * SVLA_DQ_DS_PITCH + ch * 8) * 2) = sv[u];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float zv[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // keys 32ks + 4g + j and 32ks + 16 + 4g + j of the wave's query 16w + c
        zv[j] = bf2f(ls[(32 * ks + 4 * g + j) * SVLA_DQ_DS_PITCH + 16 * w + c]);
        zv[4 + j] = bf2f(ls[(32 * ks + 16 + 4 * g + j) * SVLA_DQ_DS_PITCH + 16 * w + c]);
      }
      mfma_tr_sweep<RS, NDT, false>(acc, smem, 32 * ks, pack_frag(zv), lane);
    }
  }
  // acc: C[q = 16w + 4g + j][d = 16dt + c]
  if constexpr (ROPE) rope_t_acc<NDT>(acc, a, qt * 64 + 16 * w, L, g, c);
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

// ================================================================== backward: dQ
// Block = (query tile of 64, NH query heads sharing one kv head, batch), like the forward: K/V tiles stream
// through two LDS stages by LDS-DMA.
template <int D, int NH, bool ROPE, bool CAP>
__global__ __launch_bounds__(256 * NH, 1) void attn_bwd_dq_kernel(svla_attn_args a, const bf16_t* __restrict__ dout,
                                                                  int64_t lddo, const bf16_t* __restrict__ out,
                                                                  int64_t ldo, const float* __restrict__ lse,
                                                                  float* __restrict__ delta,
                                                                  bf16_t* __restrict__ dq, int64_t lddq) {
  constexpr int DP = Cfg<D>::DP, DV = Cfg<D>::DV, RS = Cfg<D>::RS;
  constexpr int NKS = DP / 32, NDT = DV / 16, NW = 4 * NH;
  constexpr int TB = tile_bytes<D>(64), STAGE = 2 * TB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  uint8_t* lcls = (uint8_t*)(smem + 2 * STAGE);

  const int L = a.L;
  int qt, hg, b;
  block_coords((L + 63) / 64, a.Hq / NH, qt, hg, b);
  const int t = threadIdx.x, lane = t & 63, g = lane >> 4, c = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = hg * NH + (w >> 2), wq = w & 3;
  const int grp = a.Hq / a.Hkv, hk = h / grp;
  const int qi = qt * 64 + 16 * wq + c;
  const bool qvalid = qi < L;
  const bool window_free = a.sliding_window <= 0 || a.sliding_window >= L;
  const bf16_t* qbase = (const bf16_t*)a.q + (int64_t)b * L * a.ldq + (int64_t)h * D;
  const bf16_t* obase = dout + (int64_t)b * L * lddo + (int64_t)h * D;
  const bf16_t* kbase = (const bf16_t*)a.k + (int64_t)b * L * a.ldk + (int64_t)hk * D;
  const bf16_t* vbase = (const bf16_t*)a.v + (int64_t)b * L * a.ldv + (int64_t)hk * D;
  const float LOG2E = 1.4426950408889634f;

  load_classes(lcls, a.kv_class ? a.kv_class + (int64_t)b * L : nullptr, L, t, 64 * NW);
  bf16x8 qf[NKS], of[NKS];
  load_row_frags<D>(qf, qbase + (int64_t)qi * a.ldq, qvalid, lane);
  load_row_frags<D>(of, obase + (int64_t)qi * lddo, qvalid, lane);
  const float lq = qvalid ? lse[((int64_t)b * a.Hq + h) * L + qi] * LOG2E : 0.f;
  // delta = rowsum(dO * O) of this lane's query, here instead of a separate pass: the four lanes holding the query's
  // row chunks (g = 0..3) sum their halves and combine by two shuffles; written out for the dK/dV kernel that follows
  float dq_ = 0.f;
  {
    bf16x8 orow[NKS];
    load_row_frags<D>(orow, out + ((int64_t)b * L + qi) * ldo + (int64_t)h * D, qvalid, lane);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float x[8], y[8];
      unpack8(__builtin_bit_cast(u32x4, of[ks]), x);
      unpack8(__builtin_bit_cast(u32x4, orow[ks]), y);
#pragma unroll
      for (int e = 0; e < 8; ++e) dq_ += x[e] * y[e];
    }
    dq_ += __shfl_xor(dq_, 16, 64);
    dq_ += __shfl_xor(dq_, 32, 64);
    if (g == 0 && qvalid) delta[((int64_t)b * a.Hq + h) * L + qi] = dq_;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nkt = (L + 63) / 64;
  glds_tile<RS, 64, NW>(smem, kbase, a.ldk, L, D, w, lane);
  glds_tile<RS, 64, NW>(smem + TB, vbase, a.ldv, L, D, w, lane);

  f32x4 acc[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const CapExp ce(a.scale, CAP ? a.softcap : 1.f);
  for (int kt = 0; kt < nkt; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* ldsK = smem + (kt & 1) * STAGE;
    const char* ldsV = ldsK + TB;
    if (kt + 1 < nkt) {
      char* nx = smem + ((kt + 1) & 1) * STAGE;
      const int r0 = (kt + 1) * 64;
      glds_tile<RS, 64, NW>(nx, kbase + (int64_t)r0 * a.ldk, a.ldk, L - r0, D, w, lane);
      glds_tile<RS, 64, NW>(nx + TB, vbase + (int64_t)r0 * a.ldv, a.ldv, L - r0, D, w, lane);
    }
    const bool plain = tile_plain(lcls, kt * 64, L, window_free, lane);
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
        const int kj = kt * 64 + 16 * nt + 4 * g + j;
        bool masked = false, live = qvalid;
        if (!plain) {
          live = live && kj < L;
          masked = !visible(lcls[kj < L ? kj : 0], kj, qi, a.sliding_window);
        }
        const float z = score_grad<CAP>(s[nt][j], dp[nt][j], lq, dq_, masked, ce, a.scale);
        zz[nt][j] = live ? z : 0.f;
      }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      float zv[8] = {zz[2 * ks][0], zz[2 * ks][1], zz[2 * ks][2], zz[2 * ks][3],
                     zz[2 * ks + 1][0], zz[2 * ks + 1][1], zz[2 * ks + 1][2], zz[2 * ks + 1][3]};
      const bf16x8 za = pack_frag(zv);
      mfma_tr_sweep<RS, NDT, false>(acc, ldsK, 32 * ks, za, lane);
    }
  }
  // acc: C[q = 16wq + 4g + j][d = 16dt + c]
  if constexpr (ROPE) rope_t_acc<NDT>(acc, a, qt * 64 + 16 * wq, L, g, c);
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
    const int q = qt * 64 + 16 * wq + r;
    if (q < L)
      *reinterpret_cast<u32x4*>(dq + ((int64_t)b * L + q) * lddq + (int64_t)h * D + ch * 8) =
          *reinterpret_cast<const u32x4*>(img + r * DV + ch * 8);
  }
}

// The dynamic-LDS limit of a kernel must cover the largest launch so far: the class array (and the bwd
// lse/delta slabs) grow with L, so the attribute is raised whenever a launch needs more than the last setting.
template <auto KERN>
void set_lds_once(int bytes) {
  static std::atomic<int> set_to{0};  // one high-water mark per kernel instantiation
  int cur = set_to.load(std::memory_order_relaxed);
  while (bytes > cur) {
    if (set_to.compare_exchange_weak(cur, bytes)) {
      (void)hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
      break;
    }
  }
}

int check_args(const svla_attn_args* a) {
  SVLA_CHECK_ARG(a, "attn: args NULL");
  SVLA_CHECK_ARG(a->B > 0 && a->L > 0 && a->L <= 8192 && a->Hq > 0 && a->Hkv > 0 && a->Hq % a->Hkv == 0,
                 "attn: bad B/L/H (L <= 8192)");
  SVLA_CHECK_ARG(a->D == 256 || a->D == 72 || a->D == 64, "attn: head_dim %d unsupported (256, 72 or 64)", a->D);
  SVLA_CHECK_ARG(a->q && a->k && a->v, "attn: q/k/v NULL");
  SVLA_CHECK_ARG(a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0, "attn: ld must be multiples of 8");
  SVLA_CHECK_ARG(((uintptr_t)a->q & 15) == 0 && ((uintptr_t)a->k & 15) == 0 && ((uintptr_t)a->v & 15) == 0,
                 "attn: q/k/v must be 16-B aligned");
  return 0;
}

int round16(int x) { return (x + 15) & ~15; }

template <int D, int NH, bool CAP, bool BIAS = false, int QW = 1>
int fwd_launch(const svla_attn_args& a, bf16_t* out, int64_t ldo, float* lse, hipStream_t s) {
  const int lds = 4 * tile_bytes<D>(64) + round16(a.L);
  static_assert(4 * NH * QW * 16 * (Cfg<D>::DV + 16) * 2 <= 4 * tile_bytes<D>(64), "output image must fit");
  SVLA_CHECK_ARG(lds <= 160 * 1024, "attn_fwd: L too large for the LDS-resident key classes");
  const int64_t nblk = (int64_t)((a.L + 64 * QW - 1) / (64 * QW)) * (a.Hq / NH) * a.B;
  SVLA_CHECK_ARG(nblk < (1LL << 31), "attn_fwd: grid too large");
  set_lds_once<attn_fwd_kernel<D, NH, CAP, BIAS, QW>>(lds);
  hipLaunchKernelGGL((attn_fwd_kernel<D, NH, CAP, BIAS, QW>), dim3((unsigned)nblk), dim3(256 * NH), lds, s, a, out, ldo,
                     lse);
  return svla::check_launch("attn_fwd");
}

template <int D, int NH, bool ROPE, bool CAP>
int bwd_launch(const svla_attn_args& a, const bf16_t* out, int64_t ldo, const bf16_t* dout, int64_t lddo,
               const float* lse, float* delta, bf16_t* dq, int64_t lddq, bf16_t* dk, int64_t lddk, bf16_t* dv,
               int64_t lddv, hipStream_t s, bf16_t* dsT = nullptr) {
  const int grp = a.Hq / a.Hkv;
  const int LP = (a.L + 35) / 32 * 32;
  const int nt = (a.L + 63) / 64;
  if constexpr (D == 256) {
    if (dsT) {  // delta -> dK/dV (storing dS^T) -> dQ = dS K
      const int64_t rows = (int64_t)a.B * a.L * a.Hq;
      hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows + 7) / 8)), dim3(256), 0, s, a.B, a.L, a.Hq, out,
                         ldo, dout, lddo, delta);
      if (int rc = svla::check_launch("attn_delta")) return rc;
      const int lds_kv = tile_bytes<D>(64) + 4 * tile_bytes<D>(32) + 8 * grp * LP + round16(a.L);
      SVLA_CHECK_ARG(lds_kv <= 160 * 1024, "attn_bwd: L*group too large for the LDS-resident lse/delta");
      set_lds_once<attn_bwd_dkv_kernel<D, ROPE, CAP, true>>(lds_kv);
      hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, ROPE, CAP, true>), dim3((unsigned)(nt * a.Hkv * a.B)), dim3(256),
                         lds_kv, s, a, dout, lddo, lse, delta, dk, lddk, dv, lddv, dsT);
      if (int rc = svla::check_launch("attn_bwd_dkv")) return rc;
      const int lds_q = tile_bytes<D>(64) + 64 * SVLA_DQ_DS_PITCH * 2;
      set_lds_once<attn_bwd_dq_ds_kernel<ROPE>>(lds_q);
      hipLaunchKernelGGL((attn_bwd_dq_ds_kernel<ROPE>), dim3((unsigned)(nt * a.Hq * a.B)), dim3(256), lds_q, s, a,
                         dsT, dq, lddq);
      return svla::check_launch("attn_bwd_dq_ds");
    }
  }
  // dQ first: it forms delta = rowsum(dO * O) for its queries (no separate pass) and leaves it for dK/dV
  const int lds_q = 4 * tile_bytes<D>(64) + round16(a.L);
  set_lds_once<attn_bwd_dq_kernel<D, NH, ROPE, CAP>>(lds_q);
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, NH, ROPE, CAP>), dim3((unsigned)(nt * (a.Hq / NH) * a.B)), dim3(256 * NH),
                     lds_q, s, a, dout, lddo, out, ldo, lse, delta, dq, lddq);
  if (int rc = svla::check_launch("attn_bwd_dq")) return rc;
  const int lds_kv = tile_bytes<D>(64) + 4 * tile_bytes<D>(32) + 8 * grp * LP + round16(a.L);
  SVLA_CHECK_ARG(lds_kv <= 160 * 1024, "attn_bwd: L*group too large for the LDS-resident lse/delta");
  set_lds_once<attn_bwd_dkv_kernel<D, ROPE, CAP>>(lds_kv);
  hipLaunchKernelGGL((attn_bwd_dkv_kernel<D, ROPE, CAP>), dim3((unsigned)(nt * a.Hkv * a.B)), dim3(256), lds_kv, s, a,
                     dout, lddo, lse, delta, dk, lddk, dv, lddv);
  return svla::check_launch("attn_bwd");
}

}  // namespace

extern "C" int svla_attn_fwd(const svla_attn_args* a, void* out, int64_t ldo, float* lse, void* stream) {
  if (int rc = check_args(a)) return rc;
  SVLA_CHECK_ARG(out && lse && ldo % 8 == 0, "attn_fwd: out/lse");
  SVLA_CHECK_ARG(!a->rope_cos && !a->rope_sin, "attn_fwd: q/k must arrive rotated (RoPE is a GEMM epilogue)");
  hipStream_t s = (hipStream_t)stream;
  const bool pair = (a->Hq / a->Hkv) % 2 == 0;  // two query heads of a GQA group share the K/V stream
  const bool cap = a->softcap > 0.f;
  bf16_t* o = (bf16_t*)out;
  SVLA_CHECK_ARG(!a->bias || a->D == 64, "attn_fwd: an additive bias is only supported with head_dim 64");
  // sub-wave grids (the B = 1 prefill: Gemma2 at 299 prompt tokens, BEiT at 577, SigLIP at 256 patches): the
  // variant with twice the workgroups (one head per workgroup / one 16-query sub-tile per wave) when the default
  // one would leave most CUs idle
  const int64_t qt2 = (a->L + 127) / 128, qt1 = (a->L + 63) / 64;
  const bool subwave = SVLA_ATT_SUBWAVE && qt1 * (a->Hq / 2) * a->B < svla::num_cus();
  if (a->D == 256) {
    if (SVLA_ATT_QW256 == 2)
      return cap ? fwd_launch<256, 1, true, false, 2>(*a, o, ldo, lse, s)
                 : fwd_launch<256, 1, false, false, 2>(*a, o, ldo, lse, s);
    if (pair && !subwave)
      return cap ? fwd_launch<256, 2, true>(*a, o, ldo, lse, s) : fwd_launch<256, 2, false>(*a, o, ldo, lse, s);
    return cap ? fwd_launch<256, 1, true>(*a, o, ldo, lse, s) : fwd_launch<256, 1, false>(*a, o, ldo, lse, s);
  }
  if (a->D == 64) {  // BEiT: plain MHA with the additive relative position bias, nothing else
    SVLA_CHECK_ARG(!cap && !a->kv_class && a->sliding_window <= 0 && a->Hq == a->Hkv,
                   "attn_fwd: head_dim 64 is the BEiT path (MHA, no softcap, kv_class or window)");
    if (a->bias) {
      SVLA_CHECK_ARG(a->bias_ld >= (a->L + 7) / 8 * 8 && a->bias_ld % 8 == 0 && ((uintptr_t)a->bias & 15) == 0,
                     "attn_fwd: bias rows must hold round8(L) keys (ld a multiple of 8), 16-B aligned");
      if (qt2 * a->Hq * a->B < svla::num_cus() && SVLA_ATT_SUBWAVE) return fwd_launch<64, 1, false, true, 1>(*a, o, ldo, lse, s);
      return fwd_launch<64, 1, false, true, SVLA_ATT_QW>(*a, o, ldo, lse, s);
    }
    return fwd_launch<64, 1, false, false, SVLA_ATT_QW>(*a, o, ldo, lse, s);
  }
  if (qt2 * a->Hq * a->B < svla::num_cus() && SVLA_ATT_SUBWAVE && !cap)
    return fwd_launch<72, 1, false, false, 1>(*a, o, ldo, lse, s);
  return cap ? fwd_launch<72, 1, true, false, SVLA_ATT_QW>(*a, o, ldo, lse, s)
             : fwd_launch<72, 1, false, false, SVLA_ATT_QW>(*a, o, ldo, lse, s);
}

template <int D, int NH>
static int bwd_dispatch(const svla_attn_args& a, bool rope, bool cap, const bf16_t* o, int64_t ldo, const bf16_t* d_o,
                        int64_t lddo, const float* lse, float* delta, void* dq, int64_t lddq, void* dk, int64_t lddk,
                        void* dv, int64_t lddv, hipStream_t s, bf16_t* ds = nullptr) {
  bf16_t *q = (bf16_t*)dq, *k = (bf16_t*)dk, *v = (bf16_t*)dv;
  if (rope) return cap ? bwd_launch<D, NH, true, true>(a, o, ldo, d_o, lddo, lse, delta, q, lddq, k, lddk, v, lddv, s, ds)
                       : bwd_launch<D, NH, true, false>(a, o, ldo, d_o, lddo, lse, delta, q, lddq, k, lddk, v, lddv, s, ds);
  return cap ? bwd_launch<D, NH, false, true>(a, o, ldo, d_o, lddo, lse, delta, q, lddq, k, lddk, v, lddv, s, ds)
             : bwd_launch<D, NH, false, false>(a, o, ldo, d_o, lddo, lse, delta, q, lddq, k, lddk, v, lddv, s, ds);
}

static int attn_bwd_impl(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                         const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                         float* workspace, bf16_t* ds, void* stream) {
  if (int rc = check_args(a)) return rc;
  SVLA_CHECK_ARG(a->D != 64 && !a->bias, "attn_bwd: head_dim 64 / additive bias are forward-only (frozen BEiT)");
  const bool rope = a->rope_cos != nullptr;
  if (rope) SVLA_CHECK_ARG(a->D == 256 && a->rope_sin && a->rope_ld % 8 == 0, "attn_bwd: RoPE needs D=256, sin, ld%8");
  SVLA_CHECK_ARG(out && dout && lse && dq && dk && dv && workspace, "attn_bwd: NULL buffer");
  SVLA_CHECK_ARG(ldo % 8 == 0 && lddo % 8 == 0 && lddq % 8 == 0 && lddk % 8 == 0 && lddv % 8 == 0,
                 "attn_bwd: ld must be multiples of 8");
  hipStream_t s = (hipStream_t)stream;
  const bool pair = (a->Hq / a->Hkv) % 2 == 0;
  const bool cap = a->softcap > 0.f;
  const bf16_t *o = (const bf16_t*)out, *d_o = (const bf16_t*)dout;
  if (a->D == 256)
    return pair ? bwd_dispatch<256, 2>(*a, rope, cap, o, ldo, d_o, lddo, lse, workspace, dq, lddq, dk, lddk, dv, lddv, s, ds)
                : bwd_dispatch<256, 1>(*a, rope, cap, o, ldo, d_o, lddo, lse, workspace, dq, lddq, dk, lddk, dv, lddv, s, ds);
  SVLA_CHECK_ARG(!rope && !ds, "attn_bwd: RoPE and the stored-dS path only with D=256");
  return bwd_dispatch<72, 1>(*a, false, cap, o, ldo, d_o, lddo, lse, workspace, dq, lddq, dk, lddk, dv, lddv, s);
}

extern "C" int svla_attn_bwd(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                             const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                             float* workspace, void* stream) {
  return attn_bwd_impl(a, out, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, workspace, nullptr, stream);
}

static size_t delta_bytes(int32_t B, int32_t L, int32_t Hq) { return ((size_t)B * Hq * L * 4 + 255) / 256 * 256; }

extern "C" size_t svla_attn_bwd_ds_workspace_bytes(int32_t B, int32_t L, int32_t Hq) {
  const size_t lpk = ((size_t)L + 63) / 64 * 64;
  return delta_bytes(B, L, Hq) + (size_t)B * Hq * lpk * lpk * 2;
}

extern "C" int svla_attn_bwd_ds(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout,
                                int64_t lddo, const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk,
                                void* dv, int64_t lddv, void* workspace, size_t ws_bytes, void* stream) {
  if (int rc = check_args(a)) return rc;
  SVLA_CHECK_ARG(a->D == 256, "attn_bwd_ds: head_dim 256 only");
  SVLA_CHECK_ARG(workspace && ((uintptr_t)workspace & 255) == 0 &&
                     ws_bytes >= svla_attn_bwd_ds_workspace_bytes(a->B, a->L, a->Hq),
                 "attn_bwd_ds: workspace must be 256-B aligned and svla_attn_bwd_ds_workspace_bytes long");
  bf16_t* ds = reinterpret_cast<bf16_t*>(reinterpret_cast<char*>(workspace) + delta_bytes(a->B, a->L, a->Hq));
  return attn_bwd_impl(a, out, ldo, dout, lddo, lse, dq, lddq, dk, lddk, dv, lddv, (float*)workspace, ds, stream);
}
