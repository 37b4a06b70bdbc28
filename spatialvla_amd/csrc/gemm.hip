// bf16 GEMM with fused epilogues for gfx950 (MI355X).
//
// C[M,N] = epi( sum_k A(m,k) B(n,k) )  — one kernel family serves every projection of the
// SpatialVLA hot path, forward and backward (see include/svla.h for the reference call sites).
//
// Design (CDNA4-first):
//  * Block tiles BM x BN x 64 with 4 or 8 waves; each wave owns a WTM x WTN sub-tile of
//    v_mfma_f32_16x16x32_bf16 accumulators (64-lane operand maps).  Three instantiations:
//    256x256 (8 waves, 128x64 per wave), 256x128 (8 waves, 64x64), 128x128 (4 waves, 64x64); the
//    host picks the largest that still gives >= 2 waves of blocks on the 256 CUs.  Large tiles halve
//    the L2->LDS operand traffic per FLOP (a 128^2 tile needs ~39 TB/s of operand bandwidth at the
//    MFMA peak, more than the L2 delivers).
//  * Operands go global->LDS directly (buffer_load_dwordx4 ... lds, wave-uniform descriptors), out-of-
//    range chunks are zero-filled by the descriptor range check.  Each operand is KC (reduction dim
//    contiguous: Linear weights, activations) or RC (outer dim contiguous: activations read transposed
//    for dW, weights read for dX); RC tiles are read with the gfx950 transpose read ds_read_b64_tr_b16,
//    so no operand is ever transposed in HBM.  XOR swizzles live in the per-lane source address.
//  * Two LDS stages, k-tiles k+1 and k+2 in flight behind a counted s_waitcnt vmcnt(N) and raw
//    s_barrier (no vmcnt(0) inside the k-loop).
//  * Epilogue through LDS in 64-row passes (fp32, padded rows): every global store is a 16-B vector
//    along N, every epilogue input (bias, residual, saved activations) a 16-B vector load.
//  * Block ids are remapped XCD-aware (consecutive tiles share an XCD L2) and grouped along M.
#include "svla_common.h"
#include "agpr.h"
typedef int i32x8 __attribute__((ext_vector_type(8)));
#include "agpr_f8.h"
#include "softcap_tab.h"

#include <type_traits>

namespace {

// The GeGLU kernel's LDS copy of the gelu table (gelu_bf16_lut, svla_common.h): the direct epilogue looks up 128
// elements per lane per 256 x 256 tile, where gelu_tanh's ~30 VALU and two transcendentals made it VALU-bound (one
// wave per SIMD).
constexpr int GELU_TAB_BYTES = sizeof(svla_gelu_bf16_tab);
static_assert(GELU_TAB_BYTES % 16 == 0, "table copied in 16-B pieces");
__device__ __forceinline__ void gelu_tab_to_lds(char* dst) {
  for (int t = threadIdx.x; t < GELU_TAB_BYTES / 16; t += blockDim.x)
    *(LDS_AS u32x4*)(dst + 16 * t) = reinterpret_cast<const u32x4*>(svla_gelu_bf16_tab)[t];
}

#ifndef G4_STAMPS
#define G4_STAMPS 0
#endif
#ifndef G4_GELU_LUT
#define G4_GELU_LUT 1
#endif
constexpr int BK = 64;
constexpr int GROUP_M = 8;
constexpr uint32_t OOB = 0x80000000u;  // voffset beyond num_records -> returns zeros

// NST_: LDS stages of the k-loop.  2 = double buffering (one k-tile in flight while the other is read); more stages
// keep NST-1 k-tiles in flight, for grids whose blocks are few and whose k-loops are latency-bound (the B = 1
// prefill: a 64x64 tile's k-tile is ~64 MFMA cycles per wave against a ~1.3k-cycle load round trip).
template <int BM_, int BN_, int WGM_, int WGN_, int NST_ = 2>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_, NST = NST_;
  static constexpr int NW = WGM * WGN, NTH = 64 * NW;
  static constexpr int WTM = BM / WGM, WTN = BN / WGN;
  static constexpr int TM = WTM / 16, TN = WTN / 16;
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int IA = BM / (8 * NW), IB = BN / (8 * NW);  // LDS-DMA instructions per wave per k-tile
  static constexpr int EPI_ROWS = 64, EPI_LD = BN + 4;
  static constexpr int EPI_BYTES = EPI_ROWS * EPI_LD * 4;
  static constexpr int LDS = (NST * STAGE > EPI_BYTES) ? NST * STAGE : EPI_BYTES;
  static_assert(NST >= 2 && LDS <= 160 * 1024, "stages must fit the 160 KiB of LDS");
  static_assert(EPI_BYTES + TANH_TAB_BYTES <= LDS, "epilogue image + tanh table must fit");
  static_assert(IA >= 1 && IB >= 1, "tile too small for the wave count");
};
using CfgBig = Cfg<256, 256, 2, 4>;
using CfgMid = Cfg<256, 128, 4, 2>;
using CfgSmall = Cfg<128, 128, 2, 2>;
using CfgTiny = Cfg<64, 64, 2, 2>;  // sub-wave grids of the B = 1 prefill (4x the blocks of 128x128)
// deep-pipelined small tiles for the short-M GEMMs of the B = 1 prefill (launch_deep)
// stages: 4 x 16 KiB (64x64) and 3 x 24 KiB (64x128) leave room for two workgroups per CU, which keep twice the
// LDS-DMA in flight per CU -- 8 / 6 stages at one workgroup per CU measured slower (q|k|v 28.1 -> 24.5 us, o 18.5 ->
// 16.4, down 39.4 -> 31.1 at 299 rows; profiles/r9j_deep_two_per_cu_ab.txt); 128x128 keeps 4 stages (one per CU)
#ifndef TINY_NST
#define TINY_NST 4
#endif
#ifndef NARROW_NST
#define NARROW_NST 3
#endif
#ifndef SMALL_NST
#define SMALL_NST 4
#endif
using CfgTinyD = Cfg<64, 64, 2, 2, TINY_NST>;
using CfgNarrowD = Cfg<64, 128, 2, 2, NARROW_NST>;
using CfgSmallD = Cfg<128, 128, 2, 2, SMALL_NST>;
using CfgWideD = Cfg<128, 256, 2, 2, 3>;
// workgroups of a deep-pipelined instance one CU holds (LDS-bound; the register counts allow two)
template <typename C>
constexpr int deep_bpc() { return C::LDS <= 78 * 1024 ? 2 : 1; }

// RC image swizzle (even values 0..14, distinct over the 8 k-rows one tr-read half touches)
__device__ __forceinline__ int rc_swz(int k) { return ((k & 3) | ((k & 8) >> 1)) << 1; }

// segment pointer for outer tile start / k-tile start (scalar selects, no dynamic indexing)
__device__ __forceinline__ const bf16_t* seg_ptr(const svla_operand& op, int64_t idx, int64_t& base_idx) {
  const bf16_t* p = (const bf16_t*)op.ptr[0];
  base_idx = 0;
  if (op.nseg > 1 && idx >= op.seg_start[1]) { p = (const bf16_t*)op.ptr[1]; base_idx = op.seg_start[1]; }
  if (op.nseg > 2 && idx >= op.seg_start[2]) { p = (const bf16_t*)op.ptr[2]; base_idx = op.seg_start[2]; }
  if (op.nseg > 3 && idx >= op.seg_start[3]) { p = (const bf16_t*)op.ptr[3]; base_idx = op.seg_start[3]; }
  return p;
}

// ---------------------------------------------------------------------------------------------
// Operand staging.  A tile of TR outer rows x 64 k is TR*8 16-B chunks; wave-instruction j writes 1 KiB
// lane-linearly:
//   KC image [TR][64 k] (128-B rows): instruction j -> rows 8j..8j+7, lane l -> row 8j+(l>>3), LDS chunk
//      p = l&7 holding global chunk p ^ (row&7)
//   RC image [64 k][TR] (2*TR-B rows, CPR = TR/8 chunks): instruction j -> k-rows j*(64/CPR).., lane l ->
//      k-row j*(64/CPR) + l/CPR, LDS chunk p = l%CPR holding global chunk p ^ rc_swz(k-row)
// ---------------------------------------------------------------------------------------------
template <int LAYOUT, int TR, int NI>
struct OpState {
  uint32_t voff[NI];  // per-lane byte offset of each DMA chunk; OOB for rows beyond the valid extent
  int kq;             // KC: k offset (elements) of this lane's chunk; RC: k-row of instruction 0
};

template <int LAYOUT, int TR, int NI>
__device__ __forceinline__ void op_setup(const svla_operand& op, int64_t r0, int64_t rv, int w, int lane,
                                         OpState<LAYOUT, TR, NI>& st) {
  const int64_t ldb = op.ld * 2;
  if (LAYOUT == SVLA_LAYOUT_KC) {
    const int gc = (lane & 7) ^ (lane >> 3);  // row & 7 == lane >> 3 for every instruction
    st.kq = gc * 8;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int row = 8 * (w * NI + i) + (lane >> 3);
      int64_t grow = r0 + row;
      int rowoff = row;
      if (op.seg_dim == SVLA_SEG_GEGLU) {  // gate rows 0..TR/2-1, up rows TR/2..TR-1 of the tile
        grow = (r0 >> 1) + (row & (TR / 2 - 1));
        rowoff = row & (TR / 2 - 1);
      }
      st.voff[i] = grow < rv ? (uint32_t)(rowoff * ldb + gc * 16) : OOB;
    }
  } else {
    constexpr int CPR = TR / 8, RPI = 64 / CPR;
    st.kq = RPI * w * NI + lane / CPR;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int kr = st.kq + RPI * i;
      const int gc = (lane % CPR) ^ rc_swz(kr);
      st.voff[i] = (r0 + gc * 8 < rv) ? (uint32_t)(kr * ldb + gc * 16) : OOB;
    }
  }
}

template <int LAYOUT, int TR, int NI>
__device__ __forceinline__ void op_issue(const svla_operand& op, const OpState<LAYOUT, TR, NI>& st, int64_t r0,
                                         int64_t k0, int64_t kv, char* lds, int w) {
  const bf16_t* p;
  const char* base;
  if (LAYOUT == SVLA_LAYOUT_KC && op.seg_dim == SVLA_SEG_GEGLU) {
    // the wave's rows [8*w*NI, 8*w*NI + 8*NI) lie in one half of the tile: gate or up
    p = (const bf16_t*)(((8 * w * NI) >= TR / 2) ? op.ptr[1] : op.ptr[0]);
    base = (const char*)(p + (r0 >> 1) * op.ld + k0);
  } else {
    int64_t rb = 0, kb = 0;
    if (op.seg_dim == SVLA_SEG_K) p = seg_ptr(op, k0, kb);
    else p = seg_ptr(op, r0, rb);
    base = (LAYOUT == SVLA_LAYOUT_KC) ? (const char*)(p + (r0 - rb) * op.ld + (k0 - kb))
                                      : (const char*)(p + (k0 - kb) * op.ld + (r0 - rb));
  }
  __amdgpu_buffer_rsrc_t rs = make_rsrc(base);
  constexpr int RPI = (LAYOUT == SVLA_LAYOUT_KC) ? 0 : 64 / (TR / 8);
  const int64_t krem = kv - k0;  // valid k extent left in this k-tile
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const bool ok = (LAYOUT == SVLA_LAYOUT_KC) ? (st.kq < krem) : (st.kq + RPI * i < krem);
    const uint32_t voff = ok ? st.voff[i] : OOB;
    LDS_AS void* dst = (LDS_AS void*)(lds + (w * NI + i) * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, voff, 0, 0, 0);
  }
}

// ---- LDS -> MFMA operand fragment (16 rows starting at rb, k-step ks of 32)
template <int LAYOUT, int TR>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rb, int ks, int lane) {
  if (LAYOUT == SVLA_LAYOUT_KC) {
    int row = rb + (lane & 15);
    int chunk = 4 * ks + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int rc = rb + 4 * p;
    const int chunk = rc >> 3, off = (rc & 7) * 2;
    const int k1 = 32 * ks + 8 * g + q, k2 = k1 + 4;
    const LDS_AS s16x4* a1 = (const LDS_AS s16x4*)(lds + k1 * (2 * TR) + ((chunk ^ rc_swz(k1)) << 4) + off);
    const LDS_AS s16x4* a2 = (const LDS_AS s16x4*)(lds + k2 * (2 * TR) + ((chunk ^ rc_swz(k2)) << 4) + off);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)a1);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)a2);
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  }
}

struct CDesc {
  bf16_t* ptr[4];
  int64_t start[5];
  int n;
  int64_t ld;
};

#ifndef G_EPI_STORE
#define G_EPI_STORE 0  // diagnostic builds: 1 = no output store (timing ablation, wrong results), 2 = nontemporal stores
#endif
__device__ __forceinline__ void store8(bf16_t* p, const float* v, int64_t n_valid) {
  if (n_valid >= 8) {
    if constexpr (G_EPI_STORE == 1) {
      const u32x4 x = pack8(v);
      asm volatile("" ::"v"(x));
    } else if constexpr (G_EPI_STORE == 2) {
      __builtin_nontemporal_store(pack8(v), reinterpret_cast<u32x4*>(p));
    } else {
      *reinterpret_cast<u32x4*>(p) = pack8(v);
    }
  } else {
    for (int j = 0; j < n_valid; ++j) p[j] = f2bf(v[j]);
  }
}
__device__ __forceinline__ void load8f(const bf16_t* p, float* v, int64_t n_valid) {
  if (n_valid >= 8) {
    unpack8(*reinterpret_cast<const u32x4*>(p), v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (j < n_valid) ? bf2f(p[j]) : 0.f;
  }
}

// epilogue for one row/8-column chunk (all kinds except GEGLU, SOFTCAP_CE handled by the caller)
__device__ __forceinline__ void epi_chunk(const svla_epilogue& E, int kind, bf16_t* cp, int64_t m, int64_t n,
                                          int64_t nv, float* v) {
  switch (kind) {
    case SVLA_EPI_STORE: {
      if (E.accumulate) {
        float o[8];
        load8f(cp, o, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = E.alpha * v[j] + o[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= E.alpha;
      }
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_BIAS: {
      float b[8];
      load8f((const bf16_t*)E.bias + n, b, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + b[j]) * E.alpha;
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_BIAS_GELU: {
      float b[8], pre[8];
      load8f((const bf16_t*)E.bias + n, b, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pre[j] = round_bf(v[j] + b[j]);
        v[j] = gelu_bf16(pre[j]);
      }
      store8((bf16_t*)E.out1 + m * E.ld_out1 + n, pre, nv);
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_BIAS_GELU_ERF: {
      float b[8];
      load8f((const bf16_t*)E.bias + n, b, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = gelu_erf(round_bf(v[j] + b[j]));
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_BIAS_SCALE_RESID: {
      float b[8], sc[8], r[8];
      if (E.bias) load8f((const bf16_t*)E.bias + n, b, nv);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
      load8f((const bf16_t*)E.colscale + n, sc, nv);
      load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, r, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = round_bf(sc[j] * round_bf(v[j] + b[j])) + r[j];
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_BIAS_RESID: {
      float b[8], r[8];
      if (E.bias) load8f((const bf16_t*)E.bias + n, b, nv);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
      load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, r, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + b[j]) + r[j];
      store8(cp, v, nv);
    } break;
    case SVLA_EPI_GEGLU_BWD: {
      float g[8], u[8], dg[8], du[8];
      load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, g, nv);
      load8f((const bf16_t*)E.in1 + m * E.ld_in1 + n, u, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dh = round_bf(v[j]);
        float act = gelu_bf16(g[j]);
        float dact = round_bf(dh * u[j]);
        du[j] = dh * act;
        dg[j] = dact * gelu_tanh_grad(g[j]);
      }
      store8((bf16_t*)E.out1 + m * E.ld_out1 + n, dg, nv);
      store8((bf16_t*)E.out2 + m * E.ld_out2 + n, du, nv);
    } break;
    case SVLA_EPI_GELU_BWD: {
      float pre[8];
      load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, pre, nv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]) * gelu_tanh_grad(pre[j]);
      store8(cp, v, nv);
    } break;
    default:
      break;
  }
}

// One 64-row pass of a row-local epilogue (STORE, BIAS, BIAS_GELU, BIAS_RESID, GELU_BWD, GEGLU_BWD, GEGLU) with the
// kind fixed at compile time: every LDS read of the thread's chunks is issued before the first store, so the pass
// costs one LDS round trip instead of one per chunk (the runtime-switched per-chunk loop took ~8k cycles per
// 64-row pass of a 256-wide tile at 256 threads).
#ifndef G8_EPI_IT
#define G8_EPI_IT 1
#endif
#ifndef G2_EPI_IT
#define G2_EPI_IT 1
#endif
template <int KIND, int BN, int NTH, int ITMAX>
__device__ __forceinline__ void epi_pass_fast(const float* Ei, int64_t M, int64_t N, int64_t m0p, int64_t n0,
                                              bf16_t* cbase, int64_t cm0, int64_t ldc, const svla_epilogue& E,
                                              int t) {
  constexpr int EPI_LD = BN + 4;
  if constexpr (KIND == SVLA_EPI_GEGLU) {
    constexpr int HC = BN / 16;                 // 8-column chunks per half row (gate | up)
    constexpr int ITT = 64 * HC / NTH;          // chunks per thread
    constexpr int IC = ITMAX < 2 ? ITMAX : 2;
    constexpr int IT = ITT < IC ? ITT : IC;     // chunks in flight (register budget beside live accumulators)
    const int64_t I = N >> 1;
#pragma unroll 1
    for (int ib = 0; ib < ITT; ib += IT) {
    float g[IT][8], u[IT][8];
#pragma unroll
    for (int it0 = 0; it0 < IT; ++it0) {
      const int it = ib + it0;
      const int idx = t + it * NTH, row = idx / HC, c2 = idx % HC;
      const float* pg = Ei + row * EPI_LD + 8 * c2;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(pg), a1 = *reinterpret_cast<const f32x4*>(pg + 4);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(pg + BN / 2), b1 = *reinterpret_cast<const f32x4*>(pg + BN / 2 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { g[it0][j] = a0[j]; g[it0][4 + j] = a1[j]; u[it0][j] = b0[j]; u[it0][4 + j] = b1[j]; }
    }
#pragma unroll
    for (int it0 = 0; it0 < IT; ++it0) {
      const int idx = t + (ib + it0) * NTH, row = idx / HC, c2 = idx % HC;
      const int64_t m = m0p + row, n = (n0 >> 1) + 8 * c2;
      if (m < M && n < I) {
        float h[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g[it0][j] = round_bf(g[it0][j]);
          u[it0][j] = round_bf(u[it0][j]);
          h[j] = gelu_bf16(g[it0][j]) * u[it0][j];
        }
        store8(cbase + (m - cm0) * ldc + n, h, I - n);
        store8((bf16_t*)E.out1 + m * E.ld_out1 + n, g[it0], I - n);
        store8((bf16_t*)E.out2 + m * E.ld_out2 + n, u[it0], I - n);
        if constexpr (HC == 16) {  // the MX copy of h (fp8 down operand): 16 threads = one row's 128-column k-tile
          if (E.mx_q != nullptr) {
#pragma unroll
            for (int j = 0; j < 8; ++j) h[j] = round_bf(h[j]);
            mx_store8(h, true, (uint8_t*)E.mx_q + m * E.mx_ldq + n,
                      (uint8_t*)E.mx_scales + (n / 128) * E.mx_sld + m * 4);
          }
        }
      }
    }
    }
  } else {
    constexpr int CPR = BN / 8;
    constexpr int RPP = NTH / CPR;
    constexpr int ITT = 64 / RPP;
    constexpr int IT = ITT < ITMAX ? ITT : ITMAX;  // chunks in flight (register budget beside live accumulators)
    const int cc = t % CPR;
    const int64_t n = n0 + 8 * cc;
    const int64_t nv = N - n;
    float b[8];
    if constexpr (KIND == SVLA_EPI_BIAS || KIND == SVLA_EPI_BIAS_GELU || KIND == SVLA_EPI_BIAS_RESID ||
                  KIND == SVLA_EPI_BIAS_GELU_ERF || KIND == SVLA_EPI_BIAS_SCALE_RESID) {
      if (E.bias && nv > 0) load8f((const bf16_t*)E.bias + n, b, nv);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = 0.f;
    }
    float sc[8];
    if constexpr (KIND == SVLA_EPI_BIAS_SCALE_RESID) {
      if (nv > 0) load8f((const bf16_t*)E.colscale + n, sc, nv);
    }
    if (nv <= 0) return;
    if constexpr (KIND == SVLA_EPI_ROPE) {
      // q/k columns: x = bf16(acc), partner chunk D/2 away in the same head (same tile image), reference rounding
      // bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)); the cos/sin rows of the next row are loaded while this row
      // is processed (the generic path waited one L2 round trip per row)
      const bool rot = n < E.rope_cols;
      const int hd = E.rope_D, half = hd >> 1;
      const int d = (int)(n % hd);
      const bool lo = d < half;
      const int dd = lo ? d : d - half;
      const int poff = lo ? half : -half;
      const bf16_t* ctab = (const bf16_t*)E.rope_cos + dd;
      const bf16_t* stab = (const bf16_t*)E.rope_sin + dd;
      auto tab = [&](int it, u32x4& c4, u32x4& s4) {
        const int64_t m = m0p + t / CPR + it * RPP;
        const int64_t pos = (m < M ? m : m0p) % E.rope_L;
        c4 = *reinterpret_cast<const u32x4*>(ctab + pos * E.rope_ld);
        s4 = *reinterpret_cast<const u32x4*>(stab + pos * E.rope_ld);
      };
      u32x4 cn = {0u, 0u, 0u, 0u}, sn = {0u, 0u, 0u, 0u};
      if (rot) tab(0, cn, sn);
#pragma unroll 1
      for (int it = 0; it < ITT; ++it) {
        const u32x4 cc4 = cn, sc4 = sn;
        if (rot && it + 1 < ITT) tab(it + 1, cn, sn);
        const int row = t / CPR + it * RPP;
        const int64_t m = m0p + row;
        const float* pe = Ei + row * EPI_LD + 8 * cc;
        float x[8];
        {
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(pe), x1 = *reinterpret_cast<const f32x4*>(pe + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { x[j] = x0[j]; x[4 + j] = x1[j]; }
        }
        if (rot) {
          const f32x4 y0 = *reinterpret_cast<const f32x4*>(pe + poff), y1 = *reinterpret_cast<const f32x4*>(pe + poff + 4);
          float cf[8], sf[8];
          unpack8(cc4, cf);
          unpack8(sc4, sf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xv = round_bf(x[j]), yv = round_bf(j < 4 ? y0[j] : y1[j - 4]);
            const float rv = lo ? -yv : yv;
            x[j] = round_bf(xv * cf[j]) + round_bf(rv * sf[j]);
          }
        }
        if (m < M) store8(cbase + (m - cm0) * ldc + n, x, nv);
      }
      return;
    }
#pragma unroll 1
    for (int ib = 0; ib < ITT; ib += IT) {
    float v[IT][8];
#pragma unroll
    for (int it0 = 0; it0 < IT; ++it0) {
      const float* pe = Ei + (t / CPR + (ib + it0) * RPP) * EPI_LD + 8 * cc;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(pe), x1 = *reinterpret_cast<const f32x4*>(pe + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { v[it0][j] = x0[j]; v[it0][4 + j] = x1[j]; }
    }
#pragma unroll
    for (int it0 = 0; it0 < IT; ++it0) {
      const int64_t m = m0p + t / CPR + (ib + it0) * RPP;
      if (m >= M) continue;
      bf16_t* cp = cbase + (m - cm0) * ldc + n;
      float* x = v[it0];
      if constexpr (KIND == SVLA_EPI_STORE) {
        if (E.accumulate) {
          float o[8];
          load8f(cp, o, nv);
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = E.alpha * x[j] + o[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] *= E.alpha;
        }
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_BIAS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = round_bf(x[j] + b[j]) * E.alpha;
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_BIAS_GELU) {
        float pre[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pre[j] = round_bf(x[j] + b[j]);
          x[j] = gelu_bf16(pre[j]);
        }
        store8((bf16_t*)E.out1 + m * E.ld_out1 + n, pre, nv);
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_BIAS_RESID) {
        float r[8];
        load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, r, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = round_bf(x[j] + b[j]) + r[j];
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_BIAS_GELU_ERF) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = gelu_erf(round_bf(x[j] + b[j]));
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_BIAS_SCALE_RESID) {
        float r[8];
        load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, r, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = round_bf(sc[j] * round_bf(x[j] + b[j])) + r[j];
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_GELU_BWD) {
        float pre[8];
        load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, pre, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = round_bf(x[j]) * gelu_tanh_grad(pre[j]);
        store8(cp, x, nv);
      } else if constexpr (KIND == SVLA_EPI_GEGLU_BWD) {
        float g[8], u[8], dg[8], du[8];
        load8f((const bf16_t*)E.in0 + m * E.ld_in0 + n, g, nv);
        load8f((const bf16_t*)E.in1 + m * E.ld_in1 + n, u, nv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float dh = round_bf(x[j]);
          const float act = gelu_bf16(g[j]);
          const float dact = round_bf(dh * u[j]);
          du[j] = dh * act;
          dg[j] = dact * gelu_tanh_grad(g[j]);
        }
        store8((bf16_t*)E.out1 + m * E.ld_out1 + n, dg, nv);
        store8((bf16_t*)E.out2 + m * E.ld_out2 + n, du, nv);
      }
    }
    }
  }
}

// ---------------- epilogue: 64-row passes through an fp32 LDS image [64][BN+4]; write_pass(pass, Ei) stores
// the accumulators of rows [64*pass, 64*pass+64) into the image
// Workgroup barrier for the epilogue's LDS image only: waits for this wave's LDS accesses (lgkmcnt), not for its
// global stores -- __syncthreads() would drain vmcnt(0) as well, exposing every pass's output-store latency (the
// 4-wave kernel spent ~40k cycles per 256x256 tile in its epilogue, ~30 % of a K = 2304 tile; stamps, r2).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM, int BN, int NTH, typename WritePass, bool FAST = false, int ITMAX = 4>
__device__ __forceinline__ void tile_epilogue(int64_t M, int64_t N, int64_t m0, int64_t n0, const CDesc& Cd,
                                              const svla_epilogue& E, char* smem, int t, WritePass write_pass,
                                              unsigned long long* ep_stamps = nullptr) {
  constexpr int EPI_LD = BN + 4;
  float* Ei = reinterpret_cast<float*>(smem);
  int cs = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < Cd.n && m0 >= Cd.start[i]) cs = i;
  bf16_t* cbase = Cd.ptr[cs];
  const int64_t cm0 = Cd.start[cs];
  const int kind = E.kind;
  constexpr int CPR = BN / 8;     // 16-B chunks per row
  constexpr int RPP = NTH / CPR;  // rows per thread-pass
  const int cc = t % CPR;
  // SOFTCAP_CE: the bf16 tanh table goes to LDS right after the image (every kernel's LDS has >= 2.5 KiB spare
  // there); the first pass's barrier publishes it
  const LDS_AS unsigned short* ltab = (const LDS_AS unsigned short*)(smem + 64 * EPI_LD * 4);
  if (kind == SVLA_EPI_SOFTCAP_CE && t < TANH_TAB_BYTES / 16)
    *(LDS_AS u32x4*)(smem + 64 * EPI_LD * 4 + 16 * t) = reinterpret_cast<const u32x4*>(svla_tanh_bf16_tab)[t];
#pragma unroll 1
  for (int pass = 0; pass < BM / 64; ++pass) {
#if G4_STAMPS
    const unsigned long long e0 = __builtin_amdgcn_s_memtime();
#endif
    write_pass(pass, Ei);
    lds_barrier();
#if G4_STAMPS
    const unsigned long long e1 = __builtin_amdgcn_s_memtime();
    if (ep_stamps) ep_stamps[0] += e1 - e0;
#endif
    const int64_t m0p = m0 + 64 * pass;
    bool fast = FAST;
    if (FAST) switch (kind) {
      case SVLA_EPI_STORE: epi_pass_fast<SVLA_EPI_STORE, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t); break;
      case SVLA_EPI_BIAS: epi_pass_fast<SVLA_EPI_BIAS, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t); break;
      case SVLA_EPI_BIAS_GELU:
        epi_pass_fast<SVLA_EPI_BIAS_GELU, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      case SVLA_EPI_BIAS_RESID:
        epi_pass_fast<SVLA_EPI_BIAS_RESID, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      case SVLA_EPI_GELU_BWD:
        epi_pass_fast<SVLA_EPI_GELU_BWD, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      case SVLA_EPI_GEGLU_BWD:
        epi_pass_fast<SVLA_EPI_GEGLU_BWD, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      case SVLA_EPI_GEGLU: epi_pass_fast<SVLA_EPI_GEGLU, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t); break;
      case SVLA_EPI_ROPE: epi_pass_fast<SVLA_EPI_ROPE, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t); break;
      case SVLA_EPI_BIAS_GELU_ERF:
        epi_pass_fast<SVLA_EPI_BIAS_GELU_ERF, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      case SVLA_EPI_BIAS_SCALE_RESID:
        epi_pass_fast<SVLA_EPI_BIAS_SCALE_RESID, BN, NTH, ITMAX>(Ei, M, N, m0p, n0, cbase, cm0, Cd.ld, E, t);
        break;
      default: fast = false;
    }
    if (fast) {
    } else if (kind == SVLA_EPI_GEGLU) {
      // columns [0, BN/2) gate, [BN/2, BN) up of output columns n0/2 ..
      constexpr int HC = CPR / 2;
      const int64_t I = N >> 1;
      for (int idx = t; idx < 64 * HC; idx += NTH) {
        const int row = idx / HC, c2 = idx % HC;
        const int64_t m = m0 + 64 * pass + row;
        const int64_t n = (n0 >> 1) + 8 * c2;
        if (m < M && n < I) {
          float g[8], u[8], h[8];
          const float* pg = Ei + row * EPI_LD + 8 * c2;
          const float* pu = pg + BN / 2;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            g[j] = round_bf(pg[j]);
            u[j] = round_bf(pu[j]);
            h[j] = gelu_bf16(g[j]) * u[j];
          }
          store8(cbase + (m - cm0) * Cd.ld + n, h, I - n);
          store8((bf16_t*)E.out1 + m * E.ld_out1 + n, g, I - n);
          store8((bf16_t*)E.out2 + m * E.ld_out2 + n, u, I - n);
          if constexpr (HC == 16) {  // the MX copy of h, as epi_pass_fast<GEGLU>
            if (E.mx_q != nullptr) {
#pragma unroll
              for (int j = 0; j < 8; ++j) h[j] = round_bf(h[j]);
              mx_store8(h, true, (uint8_t*)E.mx_q + m * E.mx_ldq + n,
                        (uint8_t*)E.mx_scales + (n / 128) * E.mx_sld + m * 4);
            }
          }
        }
      }
    } else {
#pragma unroll 1
      for (int rr = t / CPR; rr < 64; rr += RPP) {
        const int64_t m = m0 + 64 * pass + rr;
        const int64_t n = n0 + 8 * cc;
        const int64_t nv = N - n;
        float v[8];
        {
          const float* pe = Ei + rr * EPI_LD + 8 * cc;
          f32x4 x0 = *reinterpret_cast<const f32x4*>(pe);
          f32x4 x1 = *reinterpret_cast<const f32x4*>(pe + 4);
          v[0] = x0[0]; v[1] = x0[1]; v[2] = x0[2]; v[3] = x0[3];
          v[4] = x1[0]; v[5] = x1[1]; v[6] = x1[2]; v[7] = x1[3];
        }
        if (kind == SVLA_EPI_SOFTCAP_CE) {
          // softcap, round to bf16, per-(row, 128-column group) online-softmax partials (16 lanes share one)
          float mx = -INFINITY, se = 0.f;
          int am = 0x7fffffff;
          const float cap = E.cap, icap = 1.0f / E.cap;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v[j] = softcap_bf16_tab(v[j], cap, icap, ltab);
            if (j < nv && v[j] > mx) { mx = v[j]; am = (int)(n + j); }
          }
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < nv) se += __expf(v[j] - mx);
          if (mx == -INFINITY) se = 0.f;
          // combine the 16 lanes of the group: the group max first, then each lane's sum rescaled to it (one exp
          // per lane instead of two per butterfly step) and the lowest column index among the lanes at the max
          float gm = mx;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) gm = fmaxf(gm, __shfl_xor(gm, o, 64));
          se = (mx == -INFINITY) ? 0.f : se * __expf(mx - gm);
          am = (mx == gm) ? am : 0x7fffffff;
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            se += __shfl_xor(se, o, 64);
            am = min(am, __shfl_xor(am, o, 64));
          }
          mx = gm;
          if (m < M) {
            if ((cc & 15) == 0 && n < N) {  // a 128-column group that starts beyond N has no stats slot
              const int64_t ntn = (N + 127) / 128;
              float* rs = E.row_stats + (m * ntn + (n0 + 8 * cc) / 128) * 3;
              rs[0] = mx; rs[1] = se; rs[2] = __int_as_float(am);
            }
            if (nv > 0) store8(cbase + (m - cm0) * Cd.ld + n, v, nv);
          }
          continue;
        }
        if (m >= M || nv <= 0) continue;
        if (kind == SVLA_EPI_ROPE) {
          // q/k columns: rotate with the partner chunk D/2 away inside the same head (same tile); reference
          // rounding: x = bf16(acc); out = bf16(bf16(x*cos) + bf16(rotate_half(x)*sin))
          if (n < E.rope_cols) {
            const int hd = E.rope_D, half = hd >> 1;
            const int d = (int)(n % hd);
            const bool lo = d < half;
            const float* pp = Ei + rr * EPI_LD + 8 * cc + (lo ? half : -half);
            const int64_t pos = m % E.rope_L;
            float cs[8], sn[8];
            const int dd = lo ? d : d - half;
            unpack8(*reinterpret_cast<const u32x4*>((const bf16_t*)E.rope_cos + pos * E.rope_ld + dd), cs);
            unpack8(*reinterpret_cast<const u32x4*>((const bf16_t*)E.rope_sin + pos * E.rope_ld + dd), sn);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float x = round_bf(v[j]), y = round_bf(pp[j]);
              const float rot = lo ? -y : y;
              v[j] = round_bf(x * cs[j]) + round_bf(rot * sn[j]);
            }
          }
          store8(cbase + (m - cm0) * Cd.ld + n, v, nv);
          continue;
        }
        epi_chunk(E, kind, cbase + (m - cm0) * Cd.ld + n, m, n, nv, v);
      }
    }
#if G4_STAMPS
    const unsigned long long e2 = __builtin_amdgcn_s_memtime();
#endif
    lds_barrier();
#if G4_STAMPS
    if (ep_stamps) {
      const unsigned long long e3 = __builtin_amdgcn_s_memtime();
      ep_stamps[1] += e2 - e1;
      ep_stamps[2] += e3 - e2;
    }
#endif
  }
}


// s_waitcnt vmcnt(NLD * later) for a wave-uniform later in [0, KMAX] (the count is an immediate)
template <int NLD, int KMAX>
__device__ __forceinline__ void vm_wait_upto(int later) {
  if constexpr (KMAX == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    static_assert(NLD * KMAX <= 63, "vmcnt field");
    if (later >= KMAX) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD * KMAX) : "memory");
    else vm_wait_upto<NLD, KMAX - 1>(later);
  }
}

// Split-K of the deep-pipelined instances (S > 1): block (tile, split) runs k-tiles [split*nk/S, (split+1)*nk/S) of
// its tile, stores its fp32 accumulators to slab tile*S + split and adds one to the tile's arrival counter; the
// block whose add completes the count sums the S slabs in split order (the same order whichever block is last)
// and runs the epilogue.  No block waits for another.  slabs / counters: the caller's stream-K workspace
// (counters zero between launches: the reducer resets its tile's).
struct SplitArgs {
  int S;
  float* slabs;
  int* counters;
};

template <typename C, int LA, int LB>
__global__ __launch_bounds__(C::NTH, 1) void gemm_kernel(int64_t M, int64_t N, int64_t K, svla_operand A,
                                                          svla_operand B, CDesc Cd, svla_epilogue E, SplitArgs sp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int sflag;
  constexpr int BM = C::BM, BN = C::BN, NTH = C::NTH, TM = C::TM, TN = C::TN;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  const int total = tiles_m * tiles_n;
  int tm, tn, split = 0;
  if (C::NST > 2 && sp.S > 1) {
    // the M tiles of one (split, column tile) are consecutive ids, so they share an XCD and its L2 copy of the weight
    // slice
    const int L = xcd_remap(blockIdx.x, total * sp.S);
    split = L / total;
    const int tile = L % total;
    tm = tile % tiles_m;
    tn = tile / tiles_m;
  } else {
    const int pid = xcd_remap(blockIdx.x, total);
    const int group = GROUP_M * tiles_n;
    const int first_m = (pid / group) * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    tm = first_m + (pid % group) % gsz;
    tn = (pid % group) / gsz;
  }
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;

  const int wr = w / C::WGN, wc = w % C::WGN;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int64_t rvA = A.r_valid > 0 ? A.r_valid : M;
  const int64_t kvA = A.k_valid > 0 ? A.k_valid : K;
  const int64_t rvB = B.r_valid > 0 ? B.r_valid : (B.seg_dim == SVLA_SEG_GEGLU ? B.seg_start[1] : N);
  const int64_t kvB = B.k_valid > 0 ? B.k_valid : K;
  OpState<LA, BM, C::IA> sa;
  OpState<LB, BN, C::IB> sb;
  op_setup<LA, BM, C::IA>(A, m0, rvA, w, lane, sa);
  op_setup<LB, BN, C::IB>(B, n0, rvB, w, lane, sb);

  constexpr int NLD = C::IA + C::IB;  // LDS-DMA instructions per lane per k-tile
  const int nk_all = (int)((K + BK - 1) / BK);
  const int kb = (C::NST > 2 && sp.S > 1) ? (int)((int64_t)split * nk_all / sp.S) : 0;
  const int nk = (C::NST > 2 && sp.S > 1) ? (int)((int64_t)(split + 1) * nk_all / sp.S) - kb : nk_all;
  auto mfma_stage = [&](const char* la) {
    const char* lb = la + C::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = read_frag<LA, BM>(la, C::WTM * wr + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_frag<LB, BN>(lb, C::WTN * wc + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (C::NST > 2) {
    // ring of NST stages, NST-1 k-tiles in flight: k-tile kt waits only for itself (vmcnt counts the later stages'
    // DMAs still allowed outstanding), one barrier a k-tile publishes every wave's DMA of kt and retires every
    // wave's reads of kt-1, whose slot then takes k-tile kt+NST-1
    constexpr int NST = C::NST;
#pragma unroll
    for (int st = 0; st < NST - 1; ++st)
      if (st < nk) {
        op_issue<LA, BM, C::IA>(A, sa, m0, (int64_t)(kb + st) * BK, kvA, smem + st * C::STAGE, w);
        op_issue<LB, BN, C::IB>(B, sb, n0, (int64_t)(kb + st) * BK, kvB, smem + st * C::STAGE + C::A_BYTES, w);
      }
#pragma unroll 1
    for (int kt = 0; kt < nk; ++kt) {
      vm_wait_upto<NLD, NST - 2>(min(NST - 2, nk - 1 - kt));
      __builtin_amdgcn_s_barrier();
      const int kn = kt + NST - 1;
      if (kn < nk) {
        char* dst = smem + (kn % NST) * C::STAGE;
        op_issue<LA, BM, C::IA>(A, sa, m0, (int64_t)(kb + kn) * BK, kvA, dst, w);
        op_issue<LB, BN, C::IB>(B, sb, n0, (int64_t)(kb + kn) * BK, kvB, dst + C::A_BYTES, w);
      }
      mfma_stage(smem + (kt % NST) * C::STAGE);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the epilogue image reuses the stage memory
    if (sp.S > 1) {
      // hand-off as the stream-K kernels': slabs stored / loaded sc1 (write-through, L1 bypass), every wave drains
      // vmcnt before the barrier, one lane counts the arrival (cdna_hip_programming.md G16 R1)
      const int tile = tm + tn * tiles_m;
      constexpr int SLAB = TM * TN * NTH * 16;  // bytes
      const char* base = reinterpret_cast<const char*>(sp.slabs) + (int64_t)tile * sp.S * SLAB;
      {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(base + (int64_t)split * SLAB);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                   (uint32_t)((t + (i * TN + j) * NTH) * 16), 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        int* cnt = sp.counters + tile;
        const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sflag = (old == sp.S - 1);
        if (old == sp.S - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (!sflag) return;  // block-uniform: another block reduces this tile
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: the loads stay below
#pragma unroll 1
      for (int sg = 0; sg < sp.S; ++sg) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(base + (int64_t)sg * SLAB);
        f32x4 x[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            x[i][j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((t + (i * TN + j) * NTH) * 16), 0, 16));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = sg == 0 ? x[i][j] : acc[i][j] + x[i][j];
      }
    }
  } else {
  op_issue<LA, BM, C::IA>(A, sa, m0, 0, kvA, smem, w);
  op_issue<LB, BN, C::IB>(B, sb, n0, 0, kvB, smem + C::A_BYTES, w);
  if (nk > 1) {
    op_issue<LA, BM, C::IA>(A, sa, m0, BK, kvA, smem + C::STAGE, w);
    op_issue<LB, BN, C::IB>(B, sb, n0, BK, kvB, smem + C::STAGE + C::A_BYTES, w);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    mfma_stage(smem + cur * C::STAGE);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) {
      op_issue<LA, BM, C::IA>(A, sa, m0, (int64_t)(kt + 2) * BK, kvA, smem + cur * C::STAGE, w);
      op_issue<LB, BN, C::IB>(B, sb, n0, (int64_t)(kt + 2) * BK, kvB, smem + cur * C::STAGE + C::A_BYTES, w);
    }
  }
  }

  auto wp = [&](int pass, float* Ei) {
    // waves whose accumulator rows fall in [64*pass, 64*pass+64) write them
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rbase = C::WTM * wr + 16 * i;
      if (rbase >= 64 * pass && rbase < 64 * pass + 64) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = C::WTN * wc + 16 * j + (lane & 15);
          const int r = rbase - 64 * pass + 4 * (lane >> 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) Ei[(r + q) * (BN + 4) + col] = acc[i][j][q];
        }
      }
    }
  };
  // the 256x256 instance has no registers to spare for the specialised passes (12-20 B of scratch)
  tile_epilogue<BM, BN, NTH, decltype(wp), !(BM == 256 && BN == 256), G2_EPI_IT>(M, N, m0, n0, Cd, E, smem, t, wp);
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 8-phase ping-pong main loop (the structure that keeps the MFMA pipe fed at 1 block/CU).
//
//  * 8 waves = two groups of 4 (G0 = waves 0-3, G1 = waves 4-7; partners on a SIMD are w and w+4).  G1 runs
//    one s_barrier behind G0, so on every SIMD one wave is in its MFMA section while its partner issues
//    LDS reads and LDS-DMA: the matrix pipe never waits for a fragment read.
//  * The tile is four 128-row half-tiles per K-step of 64: A_h0, A_h1 (rows 0-127, 128-255) and B_h0, B_h1.
//    Wave (wr = w>>2, wc = w&3) owns rows {64wr..64wr+63} of each A half and columns {32wc..32wc+31} of each
//    B half: four 64x32 quadrants, one per phase, 16 MFMAs each.
//  * Phases of K-tile t (buffer t&1):  p1 read A_h0+B_h0 -> (0,0);  p2 read B_h1 -> (0,1);
//    p3 read A_h1 -> (1,1);  p4 -> (1,0).  Every phase: [LDS-DMA one half-tile] reads, lgkmcnt(0), barrier,
//    MFMAs, barrier.  A half-tile is restaged one or more phases after its last read (A_h0 of t+2 in p2,
//    B_h0 in p3, B_h1 in p4, A_h1 of t+1 in p1), so two LDS buffers suffice; the only vmcnt wait is in p4
//    (vmcnt(6): the three half-tiles of t+2 stay in flight across the barriers).
// ---------------------------------------------------------------------------------------------
namespace p8 {
constexpr int BM = 256, BN = 256, HALF = 128, NTH = 512;
constexpr int HB = HALF * BK * 2;  // bytes per half-tile image (16 KiB)
constexpr int STAGE = 4 * HB;      // A_h0 | A_h1 | B_h0 | B_h1
constexpr int LDS = 2 * STAGE;     // 128 KiB (the 66.5 KiB epilogue image reuses it)
static_assert(64 * (BN + 4) * 4 + TANH_TAB_BYTES <= LDS, "epilogue image + tanh table must fit");
}  // namespace p8

template <int LAYOUT>
struct HalfOp {
  uint32_t voff[2][2];  // [half][instruction]: per-lane byte offset of the DMA chunk, OOB beyond the valid rows
  int kq;               // KC: k offset of this lane's chunk; RC: k-row of instruction 0
};

// instruction (w, i) of a half-tile: KC rows 8(2w+i)..+7; RC k-rows 4(2w+i)..+3 (see OpState for the images)
template <int LAYOUT>
__device__ __forceinline__ void half_setup(const svla_operand& op, int64_t r0, int64_t rv, int w, int lane,
                                           HalfOp<LAYOUT>& st) {
  const int64_t ldb = op.ld * 2;
  if (LAYOUT == SVLA_LAYOUT_KC) {
    const int gc = (lane & 7) ^ (lane >> 3);
    st.kq = gc * 8;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 8 * (2 * w + i) + (lane >> 3);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // GeGLU: half 0 = gate rows n0/2.., half 1 = up rows n0/2.. (same row index, different tensor)
        const int64_t grow = (op.seg_dim == SVLA_SEG_GEGLU) ? (r0 >> 1) + row : r0 + p8::HALF * h + row;
        st.voff[h][i] = grow < rv ? (uint32_t)(row * ldb + gc * 16) : OOB;
      }
    }
  } else {
    st.kq = 8 * w + lane / 16;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kr = st.kq + 4 * i;
      const int gc = (lane % 16) ^ rc_swz(kr);
#pragma unroll
      for (int h = 0; h < 2; ++h)
        st.voff[h][i] = (r0 + p8::HALF * h + gc * 8 < rv) ? (uint32_t)(kr * ldb + gc * 16) : OOB;
    }
  }
}

// base address of half H of an operand at k = 0 (segment resolved once per tile: the 8-phase kernel is only
// dispatched when no operand is segmented along k)
template <int LAYOUT>
__device__ __forceinline__ const char* half_base(const svla_operand& op, int64_t r0, int H) {
  if (LAYOUT == SVLA_LAYOUT_KC && op.seg_dim == SVLA_SEG_GEGLU)
    return (const char*)((const bf16_t*)op.ptr[H] + (r0 >> 1) * op.ld);
  const int64_t rh = r0 + p8::HALF * H;
  int64_t rb = 0;
  const bf16_t* p = seg_ptr(op, rh, rb);
  return (const char*)(p + (rh - rb) * (LAYOUT == SVLA_LAYOUT_KC ? op.ld : 1));
}

template <int LAYOUT, int H>
__device__ __forceinline__ void half_issue(const char* base, int64_t kstride, const HalfOp<LAYOUT>& st, int64_t k0,
                                           int64_t kv, char* lds, int w) {
  __amdgpu_buffer_rsrc_t rs = make_rsrc(base + k0 * kstride);
  const int64_t krem = kv - k0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool ok = (LAYOUT == SVLA_LAYOUT_KC) ? (st.kq < krem) : (st.kq + 4 * i < krem);
    const uint32_t voff = ok ? st.voff[H][i] : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(lds + (2 * w + i) * 1024), 16, voff, 0, 0, 0);
  }
}

// MFMA operand fragment of a 128-row half-tile image.  RC fragments are read with inline-asm
// ds_read_b64_tr_b16: through the builtin, hipcc treats the transpose read as aliasing every LDS-DMA in flight
// and drains vmcnt(0) before it, which would serialise the ping-pong pipeline.  The pair is only combined into
// the MFMA operand after the phase's lgkmcnt(0) + barrier (any register copy happens after the data landed).
template <int LAYOUT>
struct Frag;
template <>
struct Frag<SVLA_LAYOUT_KC> {
  bf16x8 v;
  __device__ __forceinline__ void load(const char* lds, int rb, int ks, int lane) {
    v = read_frag<SVLA_LAYOUT_KC, p8::HALF>(lds, rb, ks, lane);
  }
  __device__ __forceinline__ bf16x8 get() const { return v; }
};
template <>
struct Frag<SVLA_LAYOUT_RC> {
  u32x2 lo, hi;
  __device__ __forceinline__ void load(const char* lds, int rb, int ks, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int rc = rb + 4 * p;
    const int chunk = rc >> 3, off = (rc & 7) * 2;
    const int k1 = 32 * ks + 8 * g + q;  // k-row k1 + 4 has the same swizzle: offset 4 rows = 1 KiB
    const uint32_t a = (uint32_t)(uintptr_t)(const LDS_AS char*)(lds + k1 * (2 * p8::HALF) +
                                                                  ((chunk ^ rc_swz(k1)) << 4) + off);
    asm volatile("ds_read_b64_tr_b16 %0, %2\n\tds_read_b64_tr_b16 %1, %2 offset:1024"
                 : "=&v"(lo), "=v"(hi)
                 : "v"(a));
  }
  __device__ __forceinline__ bf16x8 get() const {
    const u32x4 r = {lo[0], lo[1], hi[0], hi[1]};
    return __builtin_bit_cast(bf16x8, r);
  }
};

#define P8_BARRIER()                      \
  __builtin_amdgcn_sched_barrier(0);      \
  __builtin_amdgcn_s_barrier();           \
  __builtin_amdgcn_sched_barrier(0)
#define P8_LGKM0()                                         \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       \
  __builtin_amdgcn_sched_barrier(0)

// Stream-K schedule of the 8-phase kernel.  Output tiles [0, dp_tiles) run whole, round-robin over the grid;
// the k-iterations of tiles [dp_tiles, tiles) are split evenly over the grid (block L owns iterations
// [L*I/G, (L+1)*I/G)).  A block that ends with a partial tile writes its fp32 accumulators to a slab; the last
// block to arrive at a tile (arrival counter, write-through slabs) sums the slabs in k order and runs
// the epilogue — no block ever waits for another.
struct SKArgs {
  int dp_tiles;
  int nk;
  int grid;
  int sk_first;      // 4-wave kernel: stream-K pieces before the data-parallel tiles, last piece first (gemm4_body)
  int64_t sk_iters;  // (tiles - dp_tiles) * nk, >= grid when nonzero
  float* slabs;      // [2 * grid][32 f32x4 x 512 threads]
  int* counters;     // [tiles - dp_tiles] (< 2 * grid), zero between launches
};

#define P8_FOR_ACC(BODY)                         \
  _Pragma("unroll") for (int a_ = 0; a_ < 2; ++a_)   \
  _Pragma("unroll") for (int i_ = 0; i_ < 4; ++i_)   \
  _Pragma("unroll") for (int b_ = 0; b_ < 2; ++b_)   \
  _Pragma("unroll") for (int j_ = 0; j_ < 2; ++j_) { \
    const int r_ = ((a_ * 4 + i_) * 2 + b_) * 2 + j_; \
    (void)r_;                                    \
    BODY;                                        \
  }

template <int LA, int LB>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(int64_t M, int64_t N, int64_t K, svla_operand A,
                                                        svla_operand B, CDesc Cd, svla_epilogue E, SKArgs sk) {
  using namespace p8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t_in = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(t_in >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int tiles_n = (int)((N + BN - 1) / BN), tiles_m = (int)((M + BM - 1) / BM);
  const int L = xcd_remap(blockIdx.x, sk.grid);  // consecutive L share an XCD (and its L2)
  const int nk = sk.nk;
  const int64_t rvA = A.r_valid > 0 ? A.r_valid : M;
  const int64_t kvA = A.k_valid > 0 ? A.k_valid : K;
  const int64_t rvB = B.r_valid > 0 ? B.r_valid : (B.seg_dim == SVLA_SEG_GEGLU ? B.seg_start[1] : N);
  const int64_t kvB = B.k_valid > 0 ? B.k_valid : K;
  const int64_t ksa = LA == SVLA_LAYOUT_KC ? 2 : A.ld * 2, ksb = LB == SVLA_LAYOUT_KC ? 2 : B.ld * 2;
  const int ra = 64 * wr, cb = 32 * wc;
  f32x4 acc[2][4][2][2];  // [A half][16-row frag][B half][16-col frag]

  auto coords = [&](int tile, int64_t& m0, int64_t& n0) {
    const int group = GROUP_M * tiles_n;
    const int first_m = (tile / group) * GROUP_M;
    const int gsz = min(tiles_m - first_m, GROUP_M);
    m0 = (int64_t)(first_m + (tile % group) % gsz) * BM;
    n0 = (int64_t)((tile % group) / gsz) * BN;
  };

  // acc = sum over k-tiles [kb, ke) of the (m0, n0) tile
  auto mainloop = [&](int64_t m0, int64_t n0, int kb, int ke, const int lane) {
    P8_FOR_ACC(acc[a_][i_][b_][j_] = (f32x4{0.f, 0.f, 0.f, 0.f}));
    HalfOp<LA> sa;
    HalfOp<LB> sb;
    half_setup<LA>(A, m0, rvA, w, lane, sa);
    half_setup<LB>(B, n0, rvB, w, lane, sb);
    const char* const a0p = half_base<LA>(A, m0, 0);
    const char* const a1p = half_base<LA>(A, m0, 1);
    const char* const b0p = half_base<LB>(B, n0, 0);
    const char* const b1p = half_base<LB>(B, n0, 1);
    const int64_t kb0 = (int64_t)kb * BK;
    // prologue: k-tile kb whole, k-tile kb+1 except A_h1 (issued in phase 1 of k-tile kb)
    half_issue<LA, 0>(a0p, ksa, sa, kb0, kvA, smem, w);
    half_issue<LA, 1>(a1p, ksa, sa, kb0, kvA, smem + HB, w);
    half_issue<LB, 0>(b0p, ksb, sb, kb0, kvB, smem + 2 * HB, w);
    half_issue<LB, 1>(b1p, ksb, sb, kb0, kvB, smem + 3 * HB, w);
    if (kb + 1 < ke) {
      half_issue<LA, 0>(a0p, ksa, sa, kb0 + BK, kvA, smem + STAGE, w);
      half_issue<LB, 0>(b0p, ksb, sb, kb0 + BK, kvB, smem + STAGE + 2 * HB, w);
      half_issue<LB, 1>(b1p, ksb, sb, kb0 + BK, kvB, smem + STAGE + 3 * HB, w);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    P8_BARRIER();
    if (wr) { P8_BARRIER(); }  // G1 runs one barrier behind G0

#pragma unroll 1
    for (int kt = kb; kt < ke; ++kt) {
      char* cur = smem + ((kt - kb) & 1) * STAGE;
      char* nxt = smem + (((kt - kb) & 1) ^ 1) * STAGE;
      const bool more1 = kt + 1 < ke, more2 = kt + 2 < ke;
      const int64_t k1 = (int64_t)(kt + 1) * BK, k2 = (int64_t)(kt + 2) * BK;
      Frag<LA> a0[2][4], a1[2][4];
      Frag<LB> b0[2][2], b1[2][2];

      // ---- phase 1: (A_h0, B_h0)
      if (more1) half_issue<LA, 1>(a1p, ksa, sa, k1, kvA, nxt + HB, w);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < 2; ++j) b0[ks][j].load(cur + 2 * HB, cb + 16 * j, ks, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) a0[ks][i].load(cur, ra + 16 * i, ks, lane);
      }
      P8_LGKM0();
      P8_BARRIER();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[0][i][0][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[ks][i].get(), b0[ks][j].get(), acc[0][i][0][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      P8_BARRIER();

      // ---- phase 2: (A_h0, B_h1)
      if (more2) half_issue<LA, 0>(a0p, ksa, sa, k2, kvA, cur, w);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) b1[ks][j].load(cur + 3 * HB, cb + 16 * j, ks, lane);
      P8_LGKM0();
      P8_BARRIER();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[0][i][1][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[ks][i].get(), b1[ks][j].get(), acc[0][i][1][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      P8_BARRIER();

      // ---- phase 3: (A_h1, B_h1)
      if (more2) half_issue<LB, 0>(b0p, ksb, sb, k2, kvB, cur + 2 * HB, w);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) a1[ks][i].load(cur + HB, ra + 16 * i, ks, lane);
      P8_LGKM0();
      P8_BARRIER();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[1][i][1][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ks][i].get(), b1[ks][j].get(), acc[1][i][1][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      P8_BARRIER();

      // ---- phase 4: (A_h1, B_h0); k-tile kt+1 must have landed before the next phase 1 reads it
      if (more2) {
        half_issue<LB, 1>(b1p, ksb, sb, k2, kvB, cur + 3 * HB, w);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      P8_BARRIER();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[1][i][0][j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[ks][i].get(), b0[ks][j].get(), acc[1][i][0][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      P8_BARRIER();
    }
    if (!wr) { P8_BARRIER(); }  // re-align the groups
    __syncthreads();
  };

  auto epilogue = [&](int64_t m0, int64_t n0, const int t) {
    const int lane = t & 63;
    auto wp = [&](int pass, float* Ei) {
      // pass p holds rows [64p, 64p+64) = A half (p>>1), group (p&1)
      if ((pass & 1) == wr) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if ((pass >> 1) != a) continue;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const int col = HALF * b + cb + 16 * j + (lane & 15);
                const int r = 16 * i + 4 * (lane >> 4);
#pragma unroll
                for (int q = 0; q < 4; ++q) Ei[(r + q) * (BN + 4) + col] = acc[a][i][b][j][q];
              }
        }
      }
    };
    tile_epilogue<BM, BN, NTH, decltype(wp), true, G8_EPI_IT>(M, N, m0, n0, Cd, E, smem, t, wp);
  };

  // one work unit per iteration: whole tiles L, L+G, .. < dp_tiles, then this block's stream-K segments
  const int64_t I = sk.sk_iters, G = sk.grid;
  const int64_t it1 = ((int64_t)L + 1) * I / G;
  int* sflag = reinterpret_cast<int*>(smem);
  int dp_tile = L;
  int64_t it = (int64_t)L * I / G;
#pragma unroll 1
  while (true) {
    int tile, kb, ke, st = 0;
    if (dp_tile < sk.dp_tiles) {
      tile = dp_tile;
      dp_tile += sk.grid;
      kb = 0;
      ke = nk;
    } else {
      if (it >= it1) break;
      st = (int)(it / nk);
      kb = (int)(it - (int64_t)st * nk);
      ke = (int)min((int64_t)nk, kb + (it1 - it));
      it += ke - kb;
      tile = sk.dp_tiles + st;
    }
    // an opaque copy of the thread id per work unit: keeps hipcc from hoisting the epilogue's per-thread
    // address arithmetic out of the unit loop, where it would stay live across the main loop and spill
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t_in));
    int64_t m0, n0;
    coords(tile, m0, n0);
    mainloop(m0, n0, kb, ke, t & 63);
    if (kb != 0 || ke != nk) {
      // ---- partial tile: segments are owned by blocks Lh..Ll (start(L) = floor(L*I/G) is strictly increasing)
      const int64_t T0 = (int64_t)st * nk, T1 = T0 + nk;
      const int Lh = (int)(((T0 + 1) * G + I - 1) / I - 1);
      const int Ll = (int)min(G - 1, (T1 * G + I - 1) / I - 1);
      const int nseg = Ll - Lh + 1, j = L - Lh;
      auto slab = [&](int seg) {  // the head segment is its block's last segment (slot 1), the others their first
        return make_rsrc(reinterpret_cast<const f32x4*>(sk.slabs) +
                         (int64_t)(2 * (Lh + seg) + (seg == 0 ? 1 : 0)) * (32 * NTH));
      };
      // Hand-off form (cdna_hip_programming.md G16 R1, MI355X_MICROARCH.md visibility table row 1): slabs are
      // stored and loaded sc1 (write-through / L1-bypass), every storing wave drains vmcnt before the barrier,
      // one lane adds to the tile's counter; the block whose add returns nseg-1 reduces.  No agent-scope fence:
      // a release would write back the XCD L2's dirty output lines (tens of us), an acquire is replaced by the
      // sc1 loads.
      int* cnt = sk.counters + st;
      bool last = false;
      if (j == 0) {  // the head usually finishes last: if every other segment is in, skip the slab round trip
        if (t == 0) {
          const int c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sflag[0] = (c == nseg - 1);
          if (c == nseg - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        last = sflag[0] != 0;
        __syncthreads();
      }
      if (!last) {
        const __amdgpu_buffer_rsrc_t rs = slab(j);
        uint32_t vo = t * 16;
        P8_FOR_ACC({
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[a_][i_][b_][j_]), rs, vo, 0, 16);
          vo += NTH * 16;
          asm volatile("" : "+v"(vo));
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
          const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sflag[0] = (old == nseg - 1);
          if (old == nseg - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        last = sflag[0] != 0;
        __syncthreads();
      }
      if (!last) continue;  // another block finishes this tile
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only: loads stay below
      // reducer: sum the segments in k order.  Every segment but a polled head is in its slab (this block's own
      // included), so the order ((s0 + s1) + s2) + .. is the same whichever block reduces.  The offset is
      // stepped opaquely: precomputed per-accumulator addresses would take VGPRs beside the 128 of acc.
      for (int sg = (j != 0) ? 0 : 1; sg < nseg; ++sg) {
        const __amdgpu_buffer_rsrc_t rs = slab(sg);
        const bool first = sg == 0;
        uint32_t vo = t * 16;
#pragma unroll
        for (int a = 0; a < 2; ++a) {  // 16 accumulators (256 B per lane) in flight per step
          f32x4 x[4][2][2];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
              for (int jj = 0; jj < 2; ++jj)
                x[i][b][jj] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, ((i * 2 + b) * 2 + jj) * NTH * 16, 16));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
              for (int jj = 0; jj < 2; ++jj)
                acc[a][i][b][jj] = first ? x[i][b][jj] : acc[a][i][b][jj] + x[i][b][jj];
          vo += 16 * NTH * 16;
          asm volatile("" : "+v"(vo));
        }
      }
    }
    epilogue(m0, n0, t);
  }
}

// ---------------------------------------------------------------------------------------------
// 256x256 tile, 4 waves (one per SIMD), 128x128 outputs per wave, two 64-k LDS buffers.
//
//  * Each wave keeps 64 16x16 accumulators (256 registers, AGPR-resident) and two fragment sets in VGPRs:
//    F0 = k 0..31 and F1 = k 32..63 of the current k-tile (8 A + 8 B ds_read_b128 each), half the LDS reads per
//    MFMA of the 8-wave tile.  Buffers are the KC images of the 8-wave kernel ([256][64], 128-B rows, chunk
//    p of row r holding global chunk p ^ (r & 7)), filled by LDS-DMA (8 rows per 1 KiB wave instruction).
//  * One k-tile = 128 MFMAs per wave with everything else issued in their gaps:
//      MFMA 0..15          read F1 (this tile, buffer b)
//      after MFMA RB1      lgkmcnt(0) + barrier: every wave holds the whole tile, buffer b is free
//      from MFMA DA0/DB0   LDS-DMA of k-tile kt+2 into buffer b (A then B, one piece every DST MFMAs)
//      after MFMA RB2      vmcnt(16) + barrier: k-tile kt+1 (buffer b^1) has landed everywhere
//      next 16 MFMAs       read F0 of kt+1
//    so every DMA has ~1.6 k-tiles to land and the matrix pipe never waits for a fragment.
// ---------------------------------------------------------------------------------------------
#ifndef G4_RB1
#define G4_RB1 23
#endif
#ifndef G4_DA0
#define G4_DA0 26
#endif
#ifndef G4_DB0
#define G4_DB0 62
#endif
#ifndef G4_DST
#define G4_DST 4
#endif
#ifndef G4_RB2
#define G4_RB2 95
#endif
#ifndef G4_PRIO
#define G4_PRIO 0
#endif
#ifndef G4_RS
#define G4_RS 1  // fragment reads: one per G4_RS MFMAs
#endif
#ifndef G4_SKFIRST_MIN
#define G4_SKFIRST_MIN 40  // stream-K k-tiles per block from which launch4 orders the stream-K pieces first
#endif
#ifndef G4_STAMPS
#define G4_STAMPS 0  // diagnostic build: per-wave cycles spent in each wait of the k-loop (tools/gemm_stamps.py)
#endif
#if G4_STAMPS
__device__ unsigned long long g4_stamps[16384][4][14];  // [block][wave][top lgkm, RB1, RB2, k-loop, prologue, epilogue, tiles, total]
#endif
#ifndef G4_GROUP_M
#define G4_GROUP_M GROUP_M
#endif
namespace p4 {
constexpr int BM = 256, BN = 256, NTH = 256;
constexpr int OPB = BM * BK * 2;  // bytes per operand image per buffer (32 KiB)
constexpr int STAGE = 2 * OPB;    // A | B
constexpr int LDS = 2 * STAGE;    // 128 KiB (the 66.5 KiB epilogue image reuses it)
constexpr int LDS_GELU = LDS + GELU_TAB_BYTES;  // the GeGLU kernel: the gelu table behind the operand stages
static_assert(64 * (BN + 4) * 4 + TANH_TAB_BYTES <= LDS, "epilogue image + tanh table must fit");
static_assert(G4_RB1 >= 15 * G4_RS && G4_DA0 > G4_RB1 && G4_DB0 >= G4_DA0 + 8 * G4_DST &&
                  G4_RB2 >= G4_DB0 + 8 * G4_DST - 1 && G4_RB2 + 1 + 15 * G4_RS < 128,
              "gemm4 schedule knobs out of order");
}  // namespace p4

template <int X, int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  if constexpr (X < N) {
    f(std::integral_constant<int, X>{});
    static_for<X + 1, N>(f);
  }
}

template <int LAYOUT>
struct Op4 {
  uint32_t v0, v1;  // per-lane byte offsets of piece 0 (RC: pieces with n & 2 use v1, KC fp8: odd pieces use v1);
                    // piece n adds n * rs via soffset
  int kq, kq1;      // KC: k offset (elements) of this lane's chunk (kq1: odd pieces); RC: k-row of this lane in piece 0
  int nvalid;       // KC: pieces whose row of this lane is inside the valid extent
  bool ok0, ok1;    // RC: this lane's outer chunk (v0 / v1 variant) starts inside the valid extent
  uint32_t rs;      // wave-uniform byte step per piece: KC 8 rows, RC 4 k-rows
};

// Staging of a 256-outer x 64-k operand tile: waves 0,1 stage outer half 0, waves 2,3 half 1, 8 pieces (1 KiB
// LDS-DMA wave instructions) each; offsets are relative to the base of the wave's half (op4_base).
//  KC: image [256][64] (128-B rows, chunk p of row r = global chunk p ^ (r & 7)); piece n of wave w = rows
//      64w + 8n .. +7.  GEGLU: rows 0..127 are gate rows r0/2.., 128..255 the up rows of the second tensor.
//  RC: two half images [64 k][128 outer] (256-B rows, chunk p of k-row k = global chunk p ^ rc_swz(k)); piece n
//      of wave w = k-rows 4j .. 4j+3 of its half, j = 8 (w & 1) + n.  rc_swz depends on n only through n & 2.
//  KC, fp8 (FSW): chunk p of row r holds global chunk p ^ ((r >> 1) & 7).  The 32x32x64 fp8 fragment puts rows
//      r = 0..31 on lanes 0..31 (and again on 32..63); a ds_read_b128 lane group ({0-3, 12-15, 20-27}, ...) then
//      holds rows r and r + 8, which the r & 7 swizzle puts on one 16-B slot of the bank row (2-way: 45 % of the
//      fp8 kernel's LDS cycles were conflict cycles, r5d PMC); (r >> 1) & 7 spreads the group over all 16 slots.
//      (r >> 1) & 7 of piece n's rows is (4 n + (lane >> 4)) & 7: two voffset variants, even and odd pieces.
template <int LAYOUT, bool FSW = false, int BMX = 256>
__device__ __forceinline__ void op4_setup(const svla_operand& op, int64_t r0, int64_t rv, int w, int lane,
                                          Op4<LAYOUT>& st) {
  static_assert(BMX == 256 || (LAYOUT == SVLA_LAYOUT_KC && !FSW), "192-row tiles: bf16 KC operands only");
  constexpr int PPW = BMX / 32, HALF = BMX / 2;  // pieces per wave, rows per wave pair
  const int64_t ldb = op.ld * 2;
  if (LAYOUT == SVLA_LAYOUT_KC) {
    const int gc = FSW ? (lane & 7) ^ (lane >> 4) : (lane & 7) ^ (lane >> 3);  // row & 7 == lane >> 3
    const int gc1 = FSW ? (lane & 7) ^ (4 + (lane >> 4)) : gc;
    st.kq = gc * 8;
    st.kq1 = gc1 * 8;
    const int row = 8 * PPW * w + (lane >> 3);
    const int rh = row - HALF * (w >> 1);  // row inside the wave pair's half (op4_base)
    const int64_t grow = (op.seg_dim == SVLA_SEG_GEGLU) ? (r0 >> 1) + rh : r0 + row;
    const int64_t nv = (rv - grow + 7) / 8;
    st.nvalid = grow >= rv ? 0 : (int)min<int64_t>(nv, PPW);
    st.v0 = (uint32_t)(rh * ldb + gc * 16);
    st.v1 = (uint32_t)(rh * ldb + gc1 * 16);
    st.ok0 = st.ok1 = true;
    st.rs = __builtin_amdgcn_readfirstlane((uint32_t)(8 * ldb));
  } else {
    const int kr = 32 * (w & 1) + (lane >> 4);  // k-row of piece 0 (piece n: + 4n)
    st.kq = st.kq1 = kr;
    st.nvalid = 8;
    const int64_t o = r0 + 128 * (w >> 1);
    const int gc0 = (lane & 15) ^ rc_swz(kr), gc1 = (lane & 15) ^ rc_swz(kr + 8);
    st.ok0 = o + gc0 * 8 < rv;
    st.ok1 = o + gc1 * 8 < rv;
    st.v0 = (uint32_t)(kr * ldb + gc0 * 16);
    st.v1 = (uint32_t)(kr * ldb + gc1 * 16);
    st.rs = __builtin_amdgcn_readfirstlane((uint32_t)(4 * ldb));
  }
}

// voffset of piece n of the wave at krem = valid k extent left in the k-tile (OOB -> zero-fill).  Plain overloads,
// not templates: the lambdas of gemm4_body are also analysed for the host, where a device-only function template
// called from them fails to substitute.
__device__ __forceinline__ uint32_t op4_voff(const Op4<SVLA_LAYOUT_KC>& st, int n, int64_t krem) {
  return (n & 1) ? ((st.kq1 < krem && n < st.nvalid) ? st.v1 : OOB) : ((st.kq < krem && n < st.nvalid) ? st.v0 : OOB);
}
__device__ __forceinline__ uint32_t op4_voff(const Op4<SVLA_LAYOUT_RC>& st, int n, int64_t krem) {
  return (st.kq + 4 * n < krem && ((n & 2) ? st.ok1 : st.ok0)) ? ((n & 2) ? st.v1 : st.v0) : OOB;
}

// piece n of the wave for the k-tile whose half-tile base address is kbase
#ifndef G4_ABL
#define G4_ABL 0  // timing ablations (wrong results): 1 no k-loop LDS-DMA, 2 no k-loop fragment reads, 4 no k-loop barriers
#endif
#ifndef G4_AUX
#define G4_AUX 0  // cache-policy bits of the operand LDS-DMA (1 sc0, 2 nt, 16 sc1)
#endif
__device__ __forceinline__ void op4_piece(const char* kbase, uint32_t voff, uint32_t soff, int n, char* img, int w,
                                          int ppw = 8) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(kbase), (LDS_AS void*)(img + (ppw * w + n) * 1024), 16, voff,
                                           soff, 0, G4_AUX);
}

// base address of the wave's 128-outer half of the operand tile at k = 0 (GEGLU: half 0 = gate, 1 = up tensor)
template <int LAYOUT, int BMX = 256>
__device__ __forceinline__ const char* op4_base(const svla_operand& op, int64_t r0, int half) {
  if (LAYOUT == SVLA_LAYOUT_KC && op.seg_dim == SVLA_SEG_GEGLU)
    return (const char*)((const bf16_t*)op.ptr[half] + (r0 >> 1) * op.ld);
  int64_t rb = 0;
  const int64_t rh = r0 + (BMX / 2) * half;
  const bf16_t* p = seg_ptr(op, rh, rb);
  return (const char*)(p + (rh - rb) * (LAYOUT == SVLA_LAYOUT_KC ? op.ld : 1));
}

// MFMA fragment of rows 16i of the wave's 128-outer block ob (= 128 wr or 128 wc) of an operand image
template <int LAYOUT>
__device__ __forceinline__ void frag4_load(Frag<LAYOUT>& f, const char* img, int ob, int i, int ks, int lane) {
  if (LAYOUT == SVLA_LAYOUT_KC) f.load(img, ob + 16 * i, ks, lane);
  else f.load(img + (ob >> 7) * (128 * BK * 2), 16 * i, ks, lane);
}

// The 64 accumulator quads of a wave live in fixed AGPRs (quad q = 8 * A-fragment + B-fragment in a[4q:4q+3]) and
// are touched only by the inline asm below (agpr.h): with compiler-allocated accumulators hipcc renames them between
// the MFMAs of a k-tile and pays ~250 v_accvgpr moves per k-tile at the loop back edge.
// Each MFMA statement names exactly the four AGPRs it writes (a[4Q:4Q+3]) as clobbers: with the whole file listed,
// the hazard recognizer pads every MFMA -> MFMA issue with an s_nop (it sees a write of every AGPR followed by a
// read of every AGPR), 77 nops per k-tile; with the exact quad it sees independent accumulators, as they are.
template <int Q>
__device__ __forceinline__ void agpr_mfma(const bf16x8& a, const bf16x8& b);
#define SVLA_AGPR_MFMA_Q(Q, A0, A1, A2, A3)                                                                     \
  template <>                                                                                                   \
  __device__ __forceinline__ void agpr_mfma<Q>(const bf16x8& a, const bf16x8& b) {                              \
    asm volatile("v_mfma_f32_16x16x32_bf16 a[" #A0 ":" #A3 "], %0, %1, a[" #A0 ":" #A3 "]" ::"v"(a), "v"(b)     \
                 : "a" #A0, "a" #A1, "a" #A2, "a" #A3);                                                         \
  }
SVLA_AGPR_MFMA_Q(0, 0, 1, 2, 3)
SVLA_AGPR_MFMA_Q(1, 4, 5, 6, 7)
SVLA_AGPR_MFMA_Q(2, 8, 9, 10, 11)
SVLA_AGPR_MFMA_Q(3, 12, 13, 14, 15)
SVLA_AGPR_MFMA_Q(4, 16, 17, 18, 19)
SVLA_AGPR_MFMA_Q(5, 20, 21, 22, 23)
SVLA_AGPR_MFMA_Q(6, 24, 25, 26, 27)
SVLA_AGPR_MFMA_Q(7, 28, 29, 30, 31)
SVLA_AGPR_MFMA_Q(8, 32, 33, 34, 35)
SVLA_AGPR_MFMA_Q(9, 36, 37, 38, 39)
SVLA_AGPR_MFMA_Q(10, 40, 41, 42, 43)
SVLA_AGPR_MFMA_Q(11, 44, 45, 46, 47)
SVLA_AGPR_MFMA_Q(12, 48, 49, 50, 51)
SVLA_AGPR_MFMA_Q(13, 52, 53, 54, 55)
SVLA_AGPR_MFMA_Q(14, 56, 57, 58, 59)
SVLA_AGPR_MFMA_Q(15, 60, 61, 62, 63)
SVLA_AGPR_MFMA_Q(16, 64, 65, 66, 67)
SVLA_AGPR_MFMA_Q(17, 68, 69, 70, 71)
SVLA_AGPR_MFMA_Q(18, 72, 73, 74, 75)
SVLA_AGPR_MFMA_Q(19, 76, 77, 78, 79)
SVLA_AGPR_MFMA_Q(20, 80, 81, 82, 83)
SVLA_AGPR_MFMA_Q(21, 84, 85, 86, 87)
SVLA_AGPR_MFMA_Q(22, 88, 89, 90, 91)
SVLA_AGPR_MFMA_Q(23, 92, 93, 94, 95)
SVLA_AGPR_MFMA_Q(24, 96, 97, 98, 99)
SVLA_AGPR_MFMA_Q(25, 100, 101, 102, 103)
SVLA_AGPR_MFMA_Q(26, 104, 105, 106, 107)
SVLA_AGPR_MFMA_Q(27, 108, 109, 110, 111)
SVLA_AGPR_MFMA_Q(28, 112, 113, 114, 115)
SVLA_AGPR_MFMA_Q(29, 116, 117, 118, 119)
SVLA_AGPR_MFMA_Q(30, 120, 121, 122, 123)
SVLA_AGPR_MFMA_Q(31, 124, 125, 126, 127)
SVLA_AGPR_MFMA_Q(32, 128, 129, 130, 131)
SVLA_AGPR_MFMA_Q(33, 132, 133, 134, 135)
SVLA_AGPR_MFMA_Q(34, 136, 137, 138, 139)
SVLA_AGPR_MFMA_Q(35, 140, 141, 142, 143)
SVLA_AGPR_MFMA_Q(36, 144, 145, 146, 147)
SVLA_AGPR_MFMA_Q(37, 148, 149, 150, 151)
SVLA_AGPR_MFMA_Q(38, 152, 153, 154, 155)
SVLA_AGPR_MFMA_Q(39, 156, 157, 158, 159)
SVLA_AGPR_MFMA_Q(40, 160, 161, 162, 163)
SVLA_AGPR_MFMA_Q(41, 164, 165, 166, 167)
SVLA_AGPR_MFMA_Q(42, 168, 169, 170, 171)
SVLA_AGPR_MFMA_Q(43, 172, 173, 174, 175)
SVLA_AGPR_MFMA_Q(44, 176, 177, 178, 179)
SVLA_AGPR_MFMA_Q(45, 180, 181, 182, 183)
SVLA_AGPR_MFMA_Q(46, 184, 185, 186, 187)
SVLA_AGPR_MFMA_Q(47, 188, 189, 190, 191)
SVLA_AGPR_MFMA_Q(48, 192, 193, 194, 195)
SVLA_AGPR_MFMA_Q(49, 196, 197, 198, 199)
SVLA_AGPR_MFMA_Q(50, 200, 201, 202, 203)
SVLA_AGPR_MFMA_Q(51, 204, 205, 206, 207)
SVLA_AGPR_MFMA_Q(52, 208, 209, 210, 211)
SVLA_AGPR_MFMA_Q(53, 212, 213, 214, 215)
SVLA_AGPR_MFMA_Q(54, 216, 217, 218, 219)
SVLA_AGPR_MFMA_Q(55, 220, 221, 222, 223)
SVLA_AGPR_MFMA_Q(56, 224, 225, 226, 227)
SVLA_AGPR_MFMA_Q(57, 228, 229, 230, 231)
SVLA_AGPR_MFMA_Q(58, 232, 233, 234, 235)
SVLA_AGPR_MFMA_Q(59, 236, 237, 238, 239)
SVLA_AGPR_MFMA_Q(60, 240, 241, 242, 243)
SVLA_AGPR_MFMA_Q(61, 244, 245, 246, 247)
SVLA_AGPR_MFMA_Q(62, 248, 249, 250, 251)
SVLA_AGPR_MFMA_Q(63, 252, 253, 254, 255)
#undef SVLA_AGPR_MFMA_Q
__device__ __forceinline__ void agpr_zero() { asm volatile(SVLA_AGPR_ZERO_ASM ::: SVLA_AGPR_CLOBBERS); }
// MFMA results -> v_accvgpr_read: 12 wait states (8-pass XDL)
__device__ __forceinline__ void agpr_fence() { asm volatile("s_nop 7\n\ts_nop 4" ::: SVLA_AGPR_CLOBBERS); }
template <int Q>
__device__ __forceinline__ f32x4 agpr_get() {
  float r0, r1, r2, r3;
  asm volatile(
      "v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\tv_accvgpr_read_b32 %2, a%c6\n\t"
      "v_accvgpr_read_b32 %3, a%c7"
      : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
      : "i"(4 * Q), "i"(4 * Q + 1), "i"(4 * Q + 2), "i"(4 * Q + 3));
  return f32x4{r0, r1, r2, r3};
}
template <int Q>
__device__ __forceinline__ void agpr_set(const f32x4& v) {
  asm volatile(
      "v_accvgpr_write_b32 a%c4, %0\n\tv_accvgpr_write_b32 a%c5, %1\n\tv_accvgpr_write_b32 a%c6, %2\n\t"
      "v_accvgpr_write_b32 a%c7, %3\n\ts_nop 1" ::"v"(v[0]),
      "v"(v[1]), "v"(v[2]), "v"(v[3]), "i"(4 * Q), "i"(4 * Q + 1), "i"(4 * Q + 2), "i"(4 * Q + 3)
      : SVLA_AGPR_CLOBBERS);
}

// ---- fp8 (OCP e4m3) operands of the 4-wave kernel (svla_gemm_fp8).  An fp8 KC operand tile of 256 rows x 128 k is
// byte-for-byte the bf16 KC tile of 256 x 64 (128-B rows), so staging, swizzles, zero-fill and stream-K run unchanged
// on "k units" of two fp8 values; only the fragments, the MFMA and the epilogue's read-out differ:
//  * v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate), unit block scales; a wave's 128x128 = 4x4 blocks of
//    32x32 in the same 256 AGPRs; a k-tile (128 fp8 k) = 2 k-halves x 16 MFMAs, each 4x a 16x16x32 bf16 MFMA, so the
//    k-tile takes the time of the bf16 k-tile (64 k) and every gap holds 4x the issue slots.
//  * fragment (32 rows at rb, k-half h): lane l holds row rb + (l & 31), 16-B chunks 4h + (l >> 5) and
//    4h + 2 + (l >> 5) of the row: the instruction's two 32-k blocks are bytes 0-15 and 16-31 of every lane, so an
//    MX block of 32 consecutive k of the row is one block of the instruction (FragF8, tools/mx_probe.py).
//  * epilogue: C = acc * sa[m] * sb[n] (per-row scales of A and of B = the output column), then the usual epilogue.
struct F8Scales {
  const float* sa;   // [M] row scales of A (activation rows)
  const float* sb;   // [N] (GEGLU: [2 I], gate rows then up rows) row scales of B (weight rows)
  int64_t na, nb;    // readable entries of sa / sb
  int64_t geglu_I;   // GEGLU: rows per weight half (tile column c < 128 -> gate row, else up row I + ..), else 0
  // MX mode (gemm4mx_kernel): OCP MX E8M0 block scales, one per 32 k of a row, tile-major: the 4 scale bytes of row r
  // in 128-k tile t at [t * m?_ld + 4 r] (svla_quant_mx_rows' layout); GEGLU B: the gate rows then the up rows of one
  // [2 I] scale matrix.  m?_bytes bounds the buffer (rows past it read scale byte 0 over zero-filled data).
  const uint8_t* ma;
  const uint8_t* mb;
  int64_t ma_ld, mb_ld, ma_bytes, mb_bytes;
};

struct FragF8 {
  i32x8 v;
  __device__ __forceinline__ void load(const char* img, int rb, int h, int lane) {
    // The MFMA reads bytes 0-15 of every lane as k of its first 32-k block (lane half g: k = 16 g + e) and bytes
    // 16-31 as its second block (k = 32 + 16 g + e), each block scaled by the E8M0 byte of lane half 0 / 1
    // respectively (measured, tools/mx_probe.py).  So lane half g takes chunk g of each 32-byte MX block of the
    // k-half: the first block (tile chunks 4h, 4h + 1) and the second (4h + 2, 4h + 3), and an MX block of the data
    // is a hardware block of the instruction.
    const int row = rb + (lane & 31);
    const int g = lane >> 5;
    const char* base = img + row * 128;
    const int sw = (row >> 1) & 7;  // the fp8 image swizzle (op4_setup, FSW)
    const u32x4 lo = *reinterpret_cast<const u32x4*>(base + (((4 * h + g) ^ sw) << 4));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(base + (((4 * h + 2 + g) ^ sw) << 4));
    v = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, int64_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* pb = (void*)(((uint64_t)hi << 32) | lo);
  const int n = (int)__builtin_amdgcn_readfirstlane((uint32_t)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0, n, 0x00020000);
}

// fp8 k-tile schedule (32 MFMA slots of 64 cycles): F1 reads at 0..7, RB1 after slot 9, then ONE LDS-DMA piece a
// slot -- A pieces 0..7 at slots 10..17, B pieces at slots 18..22 and 24..26 (a piece costs ~60 issue cycles: two a
// slot, as in rounds 2-4, held each slot past its 64-cycle MFMA) -- the MX scale pieces at slot 27, RB2 after slot
// 23 (vmcnt(13): the 13 pieces of k-tile kt+2 issued so far may stay in flight), then the 8 F0 reads of the next
// k-tile.
#define F8_RB1 9
#define F8_RB2 23
#define F8_P0 10    // first piece slot
#define F8_NPRE 13  // pieces issued before RB2 (slots F8_P0 .. F8_RB2 - 1)
__host__ __device__ constexpr int f8_piece(int x) {  // piece index issued in slot x, or -1
  return (x >= F8_P0 && x < F8_RB2) ? x - F8_P0 : (x > F8_RB2 && x <= F8_RB2 + 16 - F8_NPRE) ? x - F8_RB2 - 1 + F8_NPRE : -1;
}
static_assert(F8_RB2 - F8_P0 == F8_NPRE && f8_piece(F8_RB2 + 3) == 15 && F8_RB2 + 4 < 31, "fp8 schedule");

#define P4_FOR_ACC(BODY)                           \
  _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) \
  _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) { BODY; }

// The kernel body is a __device__ function template wrapped by four plain kernels: the lambdas of a __global__
// template are also instantiated for the host, where the device-only helpers they call fail to substitute and
// the kernel stub silently disappears.
// BMX: tile rows, 256 or 192 (RA = BMX / 32 A fragments and LDS-DMA pieces a wave; 192: bf16, KC A, data-parallel,
// direct-epilogue kinds on whole tiles only -- launch4's choice for grids that 256-row tiles quantise badly)
template <int LA, int LB, bool F8 = false, bool GG = false, bool MX = false, int BMX = 256>
__device__ __forceinline__ void gemm4_body(int64_t M, int64_t N, int64_t K, const svla_operand& A,
                                           const svla_operand& B, const CDesc& Cd, const svla_epilogue& E,
                                           const SKArgs& sk, const F8Scales& fs) {
  using namespace p4;
  static_assert(BMX == 256 || (BMX == 192 && !F8 && !GG && LA == SVLA_LAYOUT_KC), "192-row tiles: bf16, KC A");
  constexpr int RA = BMX / 32, HALF = BMX / 2;  // A fragments (and A pieces) a wave; rows of a wave row
  constexpr int NS = 16 * RA;                   // MFMA slots of a k-tile (two k-halves of RA x 8)
  // k-tile schedule (slots): F1 reads 0 .. RA + 7, RB1, A pieces from DA0, B pieces from DB0 (every G4_DST), RB2,
  // then the RA + 8 F0 reads of the next k-tile; the 256-row values are the tuned G4_* knobs
  constexpr int S_RB1 = BMX == 256 ? G4_RB1 : 19, S_DA0 = BMX == 256 ? G4_DA0 : 21;
  constexpr int S_DB0 = BMX == 256 ? G4_DB0 : S_DA0 + RA * G4_DST;
  constexpr int S_RB2 = BMX == 256 ? G4_RB2 : S_DB0 + 8 * G4_DST - 1;
  static_assert(S_RB1 >= (RA + 7) * G4_RS && S_DA0 > S_RB1 && S_DB0 >= S_DA0 + RA * G4_DST &&
                    S_RB2 >= S_DB0 + 8 * G4_DST - 1 && S_RB2 + 1 + (RA + 7) * G4_RS < NS,
                "gemm4 k-tile schedule out of order");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t_in = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(t_in >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int tiles_n = (int)((N + BN - 1) / BN), tiles_m = (int)((M + BMX - 1) / BMX);
  const int L = xcd_remap(blockIdx.x, sk.grid);
  const int nk = sk.nk;
  const int64_t rvA = A.r_valid > 0 ? A.r_valid : M;
  const int64_t kvA = A.k_valid > 0 ? A.k_valid : K;
  const int64_t rvB = B.r_valid > 0 ? B.r_valid : (B.seg_dim == SVLA_SEG_GEGLU ? B.seg_start[1] : N);
  const int64_t kvB = B.k_valid > 0 ? B.k_valid : K;

  auto coords = [&](int tile, int64_t& m0, int64_t& n0) {
    const int group = G4_GROUP_M * tiles_n;
    const int first_m = (tile / group) * G4_GROUP_M;
    const int gsz = min(tiles_m - first_m, G4_GROUP_M);
    m0 = (int64_t)(first_m + (tile % group) % gsz) * BMX;
    n0 = (int64_t)((tile % group) / gsz) * BN;
  };

  const int64_t ksa = LA == SVLA_LAYOUT_KC ? 2 : A.ld * 2, ksb = LB == SVLA_LAYOUT_KC ? 2 : B.ld * 2;
#if G4_STAMPS
  // [11..13]: stream-K mainloop ticks and k-tiles, data-parallel k-tiles (this block); [8..10] LDS-epilogue parts
  unsigned long long stmp[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long tk0 = __builtin_amdgcn_s_memtime();
#endif

  // Operand staging state of the tile being (or about to be) computed.  stage_first() sets it up and issues the
  // LDS-DMA of the tile's first two k-tiles; the tile loop calls it for the NEXT tile right before a direct
  // epilogue (which needs no LDS), so the next tile's prologue loads fly while this tile's outputs are stored.
  Op4<LA> sa;
  Op4<LB> sb;
  const char* abase = nullptr;
  const char* bbase = nullptr;
  // voffsets of every piece for a k-tile that lies wholly inside both reduction extents (all but the last when
  // K % 64 != 0): the per-piece range selects (v_cmp / s_and / v_cndmask per piece) leave the main loop
  uint32_t vfa[8], vfb[8];
  // piece n of the wave for the k-tile at krem = valid k extent left (KC: per-lane chunk check, RC: k-row check)
  // (the LDS-DMA itself lives in a __device__ function: lambdas of a kernel template are instantiated for the
  // host too, where the address-space cast would be a substitution failure and the kernel stub would vanish)
  auto pieceA = [&](const char* ka, int64_t krem, int n, char* img) { op4_piece(ka, op4_voff(sa, n, krem), n * sa.rs, n, img, w, RA); };
  auto pieceB = [&](const char* kb_, int64_t krem, int n, char* img) { op4_piece(kb_, op4_voff(sb, n, krem), n * sb.rs, n, img, w); };
  auto pieceA_full = [&](const char* ka, int n, char* img) { op4_piece(ka, vfa[n], n * sa.rs, n, img, w, RA); };
  auto pieceB_full = [&](const char* kb_, int n, char* img) { op4_piece(kb_, vfb[n], n * sb.rs, n, img, w); };
  // MX: each wave stages the E8M0 scales of its 64 image rows of A and of B for a k-tile (two 4-B-per-lane LDS-DMA
  // instructions of 256 B) into the k-tile's 2 KiB scale region behind the two operand stages (row i of an image at
  // byte 4 i: A at 0, B at 1024).  k units here are pairs of fp8 values, so a k-tile of 64 units is one 128-k MX tile.
  uint32_t vma = 0, vmb = 0;  // per-lane byte offsets of this wave's scale rows (the tile's rows 64 w + lane)
  auto mx_pieces = [&](int kt, int stage_idx) {
    if constexpr (MX) {
      char* const reg = smem + 2 * STAGE + stage_idx * 2048 + 256 * w;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc_n(fs.ma, fs.ma_bytes), (LDS_AS void*)reg, 4, vma,
                                               (uint32_t)(kt * fs.ma_ld), 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc_n(fs.mb, fs.mb_bytes), (LDS_AS void*)(reg + 1024), 4, vmb,
                                               (uint32_t)(kt * fs.mb_ld), 0, 0);
    }
  };
  auto issue_all = [&](int kt, char* stage) {
    const int64_t k0 = (int64_t)kt * BK;
    const char* const ka = abase + k0 * ksa;
    const char* const kbb = bbase + k0 * ksb;
#pragma unroll
    for (int n = 0; n < RA; ++n) pieceA(ka, kvA - k0, n, stage);
#pragma unroll
    for (int n = 0; n < 8; ++n) pieceB(kbb, kvB - k0, n, stage + OPB);
    if constexpr (MX) mx_pieces(kt, stage == smem ? 0 : 1);
  };
  auto stage_first = [&](int64_t m0, int64_t n0, int kb, int ke, const int lane) {
    op4_setup<LA, F8, BMX>(A, m0, rvA, w, lane, sa);
    op4_setup<LB, F8>(B, n0, rvB, w, lane, sb);
    abase = op4_base<LA, BMX>(A, m0, w >> 1);
    bbase = op4_base<LB>(B, n0, w >> 1);
    if constexpr (MX) {
      const int i = 64 * w + lane;  // image row staged by this lane
      vma = (uint32_t)((m0 + i) * 4);
      vmb = (uint32_t)(4 * (fs.geglu_I ? (i < 128 ? (n0 >> 1) + i : fs.geglu_I + (n0 >> 1) + (i - 128)) : n0 + i));
    }
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      vfa[n] = op4_voff(sa, n, (int64_t)1 << 40);
      vfb[n] = op4_voff(sb, n, (int64_t)1 << 40);
    }
    issue_all(kb, smem);
    if (ke - kb > 1) issue_all(kb + 1, smem + STAGE);
  };

  // pre: stage_first() already ran for this tile (during the previous tile's epilogue); its loads and that
  // epilogue's stores are then all drained here (vmcnt(0)): they have had a whole epilogue to land
  auto mainloop = [&](int64_t m0, int64_t n0, int kb, int ke, const int lane, bool pre) {
#if G4_STAMPS
    const unsigned long long tm0 = __builtin_amdgcn_s_memtime();
#endif
    agpr_zero();
    const int nq = ke - kb;
    if (pre) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      stage_first(m0, n0, kb, ke, lane);
      if (nq > 1) {
        if constexpr (MX) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");  // 16 operand + 2 scale pieces a k-tile
        else if constexpr (BMX == 192) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");  // 6 + 8 pieces a k-tile
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    P8_BARRIER();
    using T = std::true_type;
    using F = std::false_type;
    auto run_loop = [&](auto&& ktile) {
    int kt = kb;
#if G4_STAMPS
    const unsigned long long tl = __builtin_amdgcn_s_memtime();
#endif
    const int kfull = (int)(min(kvA, kvB) / BK);  // k-tiles [0, kfull) lie wholly inside both extents
#pragma unroll 1
    for (; kt + 2 < ke && kt + 3 <= kfull; ++kt) ktile(kt, T{}, T{}, T{});
#pragma unroll 1
    for (; kt + 2 < ke; ++kt) ktile(kt, T{}, T{}, F{});
    if (kt + 1 < ke) {
      ktile(kt, F{}, T{}, F{});
      ++kt;
    }
    ktile(kt, F{}, F{}, F{});
#if G4_STAMPS
    stmp[3] += __builtin_amdgcn_s_memtime() - tl;
    stmp[4] += tl - tm0;
#endif
    };
    if constexpr (F8) {
    const int s127 = 127;  // E8M0 unit block scale
    FragF8 f0a[4], f1a[4], f0b[4], f1b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) f0a[i].load(smem, 128 * wr + 32 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) f0b[j].load(smem + OPB, 128 * wc + 32 * j, 0, lane);
    // MX: the MFMA of k-half h scales its two k-blocks (MX blocks 2 h and 2 h + 1 of the k-tile, FragF8) by the
    // bytes that lane halves 0 and 1 pass: lane l passes byte 2 h + (l >> 5) of its row's scale dword.  tA / tB: the dwords of the lane's rows (read once per k-tile, after the barrier that makes the
    // tile visible); sA0 / sB0 (k-half 0) and sA1 / sB1 (k-half 1): the scale byte shifted to byte 0, the operand the
    // MFMA reads.  sA0 of the next tile is formed after the current tile's last k-half-0 MFMA, sA1 at the next tile's
    // first MFMA (after the current tile's last k-half-1 MFMA).
    uint32_t tA[4], tB[4];
    int sA0[4], sB0[4], sA1[4], sB1[4];
    const int sh0 = 8 * (lane >> 5), sh1 = 8 * (2 + (lane >> 5));
    auto read_sc = [&](int stage_idx) {
      if constexpr (MX) {
        const LDS_AS uint32_t* r = (const LDS_AS uint32_t*)(smem + 2 * STAGE + stage_idx * 2048);
#pragma unroll
        for (int i = 0; i < 4; ++i) tA[i] = r[128 * wr + 32 * i + (lane & 31)];
#pragma unroll
        for (int j = 0; j < 4; ++j) tB[j] = r[256 + 128 * wc + 32 * j + (lane & 31)];
      }
    };
    auto form0 = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i) { sA0[i] = (int)(tA[i] >> sh0); sB0[i] = (int)(tB[i] >> sh0); }
    };
    auto form1 = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i) { sA1[i] = (int)(tA[i] >> sh1); sB1[i] = (int)(tB[i] >> sh1); }
    };
    if constexpr (MX) {
      read_sc(0);
      form0();
    }
    auto ktile8 = [&](int kt, auto DMA, auto NEXT, auto FULLK) {
      char* const cur = smem + ((kt - kb) & 1) * STAGE;
      char* const nxt = smem + (((kt - kb) & 1) ^ 1) * STAGE;
      const int64_t k2 = (int64_t)(kt + 2) * BK;
      const char* const rsa = abase + k2 * ksa;
      const char* const rsb = bbase + k2 * ksb;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, 32>([&](auto XC) {
        constexpr int x = decltype(XC)::value;
        constexpr int y = x & 15, ii = y >> 2, jj = y & 3;
        if constexpr (MX) {
          if constexpr (x < 16) agpr_mfma_mx<ii * 4 + jj>(f0a[ii].v, f0b[jj].v, sA0[ii], sB0[jj]);
          else agpr_mfma_mx<ii * 4 + jj>(f1a[ii].v, f1b[jj].v, sA1[ii], sB1[jj]);
          if constexpr (x == 0) form1();  // this tile's k-half-1 scales (tA still holds this tile's dwords)
        } else {
          if constexpr (x < 16) agpr_mfma_f8<ii * 4 + jj>(f0a[ii].v, f0b[jj].v, s127);
          else agpr_mfma_f8<ii * 4 + jj>(f1a[ii].v, f1b[jj].v, s127);
        }
        if constexpr (x < 4) f1a[x].load(cur, 128 * wr + 32 * x, 1, lane);
        else if constexpr (x < 8) f1b[x - 4].load(cur + OPB, 128 * wc + 32 * (x - 4), 1, lane);
        if constexpr (x == F8_RB1) {
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): every F1 read of the tile landed, buffer free
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (decltype(DMA)::value) {
          constexpr int pc = f8_piece(x);
          if constexpr (pc >= 0 && pc < 8) {
            if constexpr (decltype(FULLK)::value) pieceA_full(rsa, pc, cur);
            else pieceA(rsa, kvA - k2, pc, cur);
          } else if constexpr (pc >= 8) {
            if constexpr (decltype(FULLK)::value) pieceB_full(rsb, pc - 8, cur + OPB);
            else pieceB(rsb, kvB - k2, pc - 8, cur + OPB);
          }
          if constexpr (MX && x == F8_RB2 + 4) mx_pieces(kt + 2, (kt - kb) & 1);  // after the 16 operand pieces
        }
        if constexpr (decltype(NEXT)::value) {
          if constexpr (x == F8_RB2) {
            // k-tile kt+1 (pieces and, MX, its scale pieces, all issued in the previous k-tile) has landed once only
            // the F8_NPRE pieces of k-tile kt+2 issued in this k-tile may be outstanding
            if constexpr (decltype(DMA)::value) asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
          }
          constexpr int r = x - F8_RB2 - 1;
          if constexpr (r >= 0 && r < 4) f0a[r].load(nxt, 128 * wr + 32 * r, 0, lane);
          else if constexpr (r >= 4 && r < 8) f0b[r - 4].load(nxt + OPB, 128 * wc + 32 * (r - 4), 0, lane);
          if constexpr (MX && r == 0) read_sc(((kt - kb) & 1) ^ 1);  // the next tile's scale dwords
          if constexpr (MX && x == 31) form0();                      // after this tile's last k-half-0 MFMA
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    run_loop(ktile8);
    } else {
    Frag<LA> f0a[8], f1a[8];
    Frag<LB> f0b[8], f1b[8];
    // B fragment j of the wave: rows 128 wc + 16 j of the B image; GG (GeGLU): the gate block j/2 (j even) or the up
    // block j/2 (j odd) of the wave's 64 output columns, so a lane's quads (i, 2p) and (i, 2p+1) hold the gate and the
    // up value of the same outputs
    auto loadB = [&](Frag<LB>& f, const char* img, int j, int ks) {
      if constexpr (GG) f.load(img, (j & 1) * 128 + 64 * wc + 16 * (j >> 1), ks, lane);
      else frag4_load<LB>(f, img, 128 * wc, j, ks, lane);
    };
#pragma unroll
    for (int i = 0; i < RA; ++i) frag4_load<LA>(f0a[i], smem, HALF * wr, i, 0, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) loadB(f0b[j], smem + OPB, j, 0);

    // one k-tile; DMA: stage k-tile kt+2 into this buffer; NEXT: k-tile kt+1 exists (wait for it, read its F0).
    // RC fragments come from asm transpose reads (hipcc would drain every LDS-DMA before a builtin one), which
    // the waitcnt pass cannot see: the fragments of a set are combined into MFMA operands only after an
    // explicit lgkmcnt(0) (set 0: at the top of the k-tile, set 1: at RB1).
    auto ktile = [&](int kt, auto DMA, auto NEXT, auto FULLK) {
      char* const cur = smem + ((kt - kb) & 1) * STAGE;
      char* const nxt = smem + (((kt - kb) & 1) ^ 1) * STAGE;
      const int64_t k2 = (int64_t)(kt + 2) * BK;
      const char* const rsa = abase + k2 * ksa;
      const char* const rsb = bbase + k2 * ksb;
#if G4_STAMPS
      unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#if G4_STAMPS
      stmp[0] += __builtin_amdgcn_s_memtime() - t0;
#endif
      __builtin_amdgcn_sched_barrier(0);
      if (G4_PRIO) __builtin_amdgcn_s_setprio(3);
      static_for<0, NS>([&](auto XC) {
        constexpr int x = decltype(XC)::value;
        constexpr int y = x % (NS / 2), ii = y >> 3, jj = y & 7;
        // swapped operands: quad (ii, jj) accumulates C^T, so a lane holds 4 consecutive columns of one row
        if constexpr (x < NS / 2) agpr_mfma<ii * 8 + jj>(f0b[jj].get(), f0a[ii].get());
        else agpr_mfma<ii * 8 + jj>(f1b[jj].get(), f1a[ii].get());
        if constexpr (G4_ABL & 2) {
        } else if constexpr (x % G4_RS == 0 && x / G4_RS < RA) frag4_load<LA>(f1a[x / G4_RS], cur, HALF * wr, x / G4_RS, 1, lane);
        else if constexpr (x % G4_RS == 0 && x / G4_RS < RA + 8)
          loadB(f1b[x / G4_RS - RA], cur + OPB, x / G4_RS - RA, 1);
        if constexpr (x == S_RB1) {
#if G4_STAMPS
          unsigned long long t1 = __builtin_amdgcn_s_memtime();
#endif
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), visible to the waitcnt pass
          if constexpr (!(G4_ABL & 4)) __builtin_amdgcn_s_barrier();
#if G4_STAMPS
          stmp[1] += __builtin_amdgcn_s_memtime() - t1;
#endif
        }
        if constexpr (decltype(DMA)::value && !(G4_ABL & 1)) {
          if constexpr (x >= S_DA0 && x < S_DA0 + RA * G4_DST && (x - S_DA0) % G4_DST == 0) {
            if constexpr (decltype(FULLK)::value) pieceA_full(rsa, (x - S_DA0) / G4_DST, cur);
            else pieceA(rsa, kvA - k2, (x - S_DA0) / G4_DST, cur);
          }
          if constexpr (x >= S_DB0 && x < S_DB0 + 8 * G4_DST && (x - S_DB0) % G4_DST == 0) {
            if constexpr (decltype(FULLK)::value) pieceB_full(rsb, (x - S_DB0) / G4_DST, cur + OPB);
            else pieceB(rsb, kvB - k2, (x - S_DB0) / G4_DST, cur + OPB);
          }
        }
        if constexpr (decltype(NEXT)::value) {
          if constexpr (x == S_RB2) {
#if G4_STAMPS
            unsigned long long t2 = __builtin_amdgcn_s_memtime();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
            if constexpr (decltype(DMA)::value && !(G4_ABL & 1)) {
              if constexpr (BMX == 192) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            } else {
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if constexpr (!(G4_ABL & 4)) __builtin_amdgcn_s_barrier();
#if G4_STAMPS
            stmp[2] += __builtin_amdgcn_s_memtime() - t2;
#endif
          }
          constexpr int r0 = x - S_RB2 - 1;
          constexpr int r = (r0 >= 0 && r0 % G4_RS == 0 && !(G4_ABL & 2)) ? r0 / G4_RS : -1;
          if constexpr (r >= 0 && r < RA) frag4_load<LA>(f0a[r], nxt, HALF * wr, r, 0, lane);
          else if constexpr (r >= RA && r < RA + 8) loadB(f0b[r - RA], nxt + OPB, r - RA, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if (G4_PRIO) __builtin_amdgcn_s_setprio(0);
    };
    run_loop(ktile);
    }
    if constexpr (F8) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: SVLA_AGPR_CLOBBERS);  // 16-pass XDL -> reads
    agpr_fence();  // MFMA results -> epilogue / slab readers
    __syncthreads();
  };

  // Direct epilogue (bf16 path, whole interior tiles).  The MFMAs accumulate C^T, so the quad (i, j) gives lane l 4
  // consecutive columns of one row; v_permlane16_swap of quads (i, j) and (i, j + 1) (16-lane halves: lanes 16-31 of
  // the first with lanes 0-15 of the second, 48-63 with 32-47) leaves each lane 8 consecutive columns, so every output
  // row chunk goes out as one 16-B store straight from the accumulators: no LDS image and no barrier (the LDS path
  // spent ~27k cycles per 256x256 tile, 22 % of a K = 2304 tile; tools/gemm_stamps.py).  After the swap lane g = l >> 4
  // holds columns 16 (j + (g & 1)) + 8 (g >> 1) .. +7.  STORE (alpha, accumulate) and GEGLU; every other kind, edge
  // tiles and fp8 take the LDS path.
  auto swap4 = [](f32x4& a, f32x4& b) {  // whole-vector bit casts, constant element indices
    // a and b come from v_accvgpr_read inside inline asm, which the hazard recognizer does not see: the 2 wait states
    // a VALU write owes a following v_permlane read (cdna_hip_programming.md T21) are padded here
    asm volatile("s_nop 1" ::"v"(a), "v"(b));
    const u32x4 ua = __builtin_bit_cast(u32x4, a), ub = __builtin_bit_cast(u32x4, b);
    const auto r0 = __builtin_amdgcn_permlane16_swap(ua[0], ub[0], false, false);
    const auto r1 = __builtin_amdgcn_permlane16_swap(ua[1], ub[1], false, false);
    const auto r2 = __builtin_amdgcn_permlane16_swap(ua[2], ub[2], false, false);
    const auto r3 = __builtin_amdgcn_permlane16_swap(ua[3], ub[3], false, false);
    a = __builtin_bit_cast(f32x4, u32x4{(uint32_t)r0[0], (uint32_t)r1[0], (uint32_t)r2[0], (uint32_t)r3[0]});
    b = __builtin_bit_cast(f32x4, u32x4{(uint32_t)r0[1], (uint32_t)r1[1], (uint32_t)r2[1], (uint32_t)r3[1]});
  };
  auto direct_epilogue = [&](int64_t m0, int64_t n0, int lane) -> bool {
    const int kind = E.kind;
    if (!(kind == SVLA_EPI_STORE || (GG && (kind == SVLA_EPI_GEGLU || kind == SVLA_EPI_ROPE)))) return false;
    if (GG && kind == SVLA_EPI_STORE) return false;  // the paired kernel runs GEGLU and head-256 ROPE only
    if (m0 + BMX > M || n0 + BN > N) return false;
    int cs = 0;
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (i < Cd.n && m0 >= Cd.start[i]) cs = i;
    bf16_t* const cbase = Cd.ptr[cs];
    const int64_t cm0 = Cd.start[cs];
    const int g = lane >> 4, r = lane & 15;
    const int cofs = 16 * (g & 1) + 8 * (g >> 1);
    if (kind == SVLA_EPI_SOFTCAP_CE) {  // the bf16 tanh table to LDS (the staging buffers are free)
      if ((int)threadIdx.x < TANH_TAB_BYTES / 16)
        *(LDS_AS u32x4*)(smem + 16 * threadIdx.x) = reinterpret_cast<const u32x4*>(svla_tanh_bf16_tab)[threadIdx.x];
      lds_barrier();
    }
    if constexpr (GG) {
     if (kind == SVLA_EPI_ROPE) {
      // head_dim 256, one head per tile: quads (i, 2p) hold the low half (d < 128) and (i, 2p + 1) the high half of
      // the same d, so rotate_half pairs meet in one lane.  epi_pass_fast<ROPE>'s rounding: x = bf16(acc),
      // out = bf16(bf16(x cos) + bf16(rotate_half(x) sin)); columns beyond rope_cols (v) are stored as they are.
      const bool rot = n0 < E.rope_cols;
      const int dl0 = 64 * wc + cofs;  // d of the lane's low-half chunk (pair P adds 32)
      const bf16_t* const ctab = (const bf16_t*)E.rope_cos + dl0;
      const bf16_t* const stab = (const bf16_t*)E.rope_sin + dl0;
      static_for<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int64_t m = m0 + 128 * wr + 16 * i + r;
        const int64_t pos = m % E.rope_L;
        u32x4 c4[2], s4[2];
        if (rot) {
#pragma unroll
          for (int P_ = 0; P_ < 2; ++P_) {
            c4[P_] = *reinterpret_cast<const u32x4*>(ctab + pos * E.rope_ld + 32 * P_);
            s4[P_] = *reinterpret_cast<const u32x4*>(stab + pos * E.rope_ld + 32 * P_);
          }
        }
        static_for<0, 2>([&](auto P) {
          constexpr int P_ = decltype(P)::value;
          f32x4 la = agpr_get<i * 8 + 4 * P_>(), ha = agpr_get<i * 8 + 4 * P_ + 1>();
          f32x4 lb = agpr_get<i * 8 + 4 * P_ + 2>(), hb = agpr_get<i * 8 + 4 * P_ + 3>();
          swap4(la, lb);
          swap4(ha, hb);
          float lo[8] = {la[0], la[1], la[2], la[3], lb[0], lb[1], lb[2], lb[3]};
          float hi[8] = {ha[0], ha[1], ha[2], ha[3], hb[0], hb[1], hb[2], hb[3]};
          if (rot) {
            float cf[8], sf[8];
            unpack8(c4[P_], cf);
            unpack8(s4[P_], sf);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const float xl = round_bf(lo[q]), xh = round_bf(hi[q]);
              lo[q] = round_bf(xl * cf[q]) + round_bf(-xh * sf[q]);
              hi[q] = round_bf(xh * cf[q]) + round_bf(xl * sf[q]);
            }
          }
          bf16_t* const p = cbase + (m - cm0) * Cd.ld + n0 + dl0 + 32 * P_;
          *reinterpret_cast<u32x4*>(p) = pack8(lo);
          *reinterpret_cast<u32x4*>(p + 128) = pack8(hi);
        });
      });
     } else {
      const int64_t ncol = (n0 >> 1) + 64 * wc + cofs;
      const LDS_AS unsigned short* const gtab = (const LDS_AS unsigned short*)(smem + LDS);  // gelu_tab_to_lds
      static_for<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        const int64_t m = m0 + 128 * wr + 16 * i + r;
        static_for<0, 2>([&](auto P) {
          constexpr int P_ = decltype(P)::value;
          f32x4 ga = agpr_get<i * 8 + 4 * P_>(), ua = agpr_get<i * 8 + 4 * P_ + 1>();
          f32x4 gb = agpr_get<i * 8 + 4 * P_ + 2>(), ub = agpr_get<i * 8 + 4 * P_ + 3>();
          swap4(ga, gb);
          swap4(ua, ub);
          // g and u rounded to bf16 once, in their stored packed form; h = bf16(bf16(gelu(g)) u) (gelu_bf16_lut)
          const u32x4 gp = {pack2(ga[0], ga[1]), pack2(ga[2], ga[3]), pack2(gb[0], gb[1]), pack2(gb[2], gb[3])};
          const u32x4 up = {pack2(ua[0], ua[1]), pack2(ua[2], ua[3]), pack2(ub[0], ub[1]), pack2(ub[2], ub[3])};
          u32x4 hp;
#if !G4_GELU_LUT  // diagnostic A/B: the fp32 formula
#pragma unroll
          for (int q = 0; q < 4; ++q)
            hp[q] = pack2(round_bf(gelu_tanh(__uint_as_float(gp[q] << 16))) * __uint_as_float(up[q] << 16),
                          round_bf(gelu_tanh(__uint_as_float(gp[q] & 0xffff0000u))) * __uint_as_float(up[q] & 0xffff0000u));
#else
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float h0 = gelu_bf16_lut(gp[q] & 0xffffu, __uint_as_float(gp[q] << 16), gtab) *
                             __uint_as_float(up[q] << 16);
            const float h1 = gelu_bf16_lut(gp[q] >> 16, __uint_as_float(gp[q] & 0xffff0000u), gtab) *
                             __uint_as_float(up[q] & 0xffff0000u);
            hp[q] = pack2(h0, h1);
          }
#endif
          const int64_t n = ncol + 32 * P_;
          *reinterpret_cast<u32x4*>(cbase + (m - cm0) * Cd.ld + n) = hp;
          *reinterpret_cast<u32x4*>((bf16_t*)E.out1 + m * E.ld_out1 + n) = gp;
          *reinterpret_cast<u32x4*>((bf16_t*)E.out2 + m * E.ld_out2 + n) = up;
        });
      });
     }
    } else {
      // one row chunk: v = 8 consecutive fp32 columns n .. n+7 of row m (reference rounding points of epi_pass_fast)
      const float alpha = E.alpha;
      const bool acc = E.accumulate != 0;
      const int64_t nb = n0 + 128 * wc + cofs;  // column of chunk p: nb + 32 p
      auto run = [&](auto KC) {
        constexpr int KIND = decltype(KC)::value;
        constexpr bool HAS_B = KIND == SVLA_EPI_BIAS || KIND == SVLA_EPI_BIAS_GELU || KIND == SVLA_EPI_BIAS_RESID ||
                               KIND == SVLA_EPI_BIAS_GELU_ERF || KIND == SVLA_EPI_BIAS_SCALE_RESID;
        constexpr bool HAS_IN0 = KIND == SVLA_EPI_BIAS_RESID || KIND == SVLA_EPI_BIAS_SCALE_RESID ||
                                 KIND == SVLA_EPI_GELU_BWD;
        u32x4 bq[4], sq[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          bq[p] = sq[p] = u32x4{0u, 0u, 0u, 0u};
          if (HAS_B && E.bias) bq[p] = *reinterpret_cast<const u32x4*>((const bf16_t*)E.bias + nb + 32 * p);
          if (KIND == SVLA_EPI_BIAS_SCALE_RESID) sq[p] = *reinterpret_cast<const u32x4*>((const bf16_t*)E.colscale + nb + 32 * p);
        }
        const LDS_AS unsigned short* ltab = (const LDS_AS unsigned short*)smem;
        const float cap = E.cap, icap = 1.0f / E.cap;
        static_for<0, RA>([&](auto I) {
          constexpr int i = decltype(I)::value;
          const int64_t m = m0 + HALF * wr + 16 * i + r;
          bf16_t* const rowp = cbase + (m - cm0) * Cd.ld + nb;
          u32x4 old[4];
          if (HAS_IN0 || (KIND == SVLA_EPI_STORE && acc)) {  // the row block's four chunks in flight at once
            const bf16_t* src = HAS_IN0 ? (const bf16_t*)E.in0 + m * E.ld_in0 + nb : rowp;
#pragma unroll
            for (int p = 0; p < 4; ++p) old[p] = *reinterpret_cast<const u32x4*>(src + 32 * p);
          }
          float mx = -INFINITY, se = 0.f, mold = -INFINITY;
          int am = 0x7fffffff;
          static_for<0, 4>([&](auto P) {
            constexpr int p = decltype(P)::value;
            f32x4 a = agpr_get<i * 8 + 2 * p>(), b = agpr_get<i * 8 + 2 * p + 1>();
            swap4(a, b);
            float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
            float bb[8], o[8];
            if constexpr (HAS_B) unpack8(bq[p], bb);
            if constexpr (HAS_IN0) unpack8(old[p], o);
            if constexpr (KIND == SVLA_EPI_STORE) {
              if (acc) {
                unpack8(old[p], o);
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = alpha * v[q] + o[q];
              } else if (alpha != 1.f) {
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] *= alpha;
              }
            } else if constexpr (KIND == SVLA_EPI_BIAS) {
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] = round_bf(v[q] + bb[q]) * alpha;
            } else if constexpr (KIND == SVLA_EPI_BIAS_GELU) {
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                bb[q] = round_bf(v[q] + bb[q]);  // pre-activation, saved for backward
                v[q] = gelu_bf16(bb[q]);
              }
              *reinterpret_cast<u32x4*>((bf16_t*)E.out1 + m * E.ld_out1 + nb + 32 * p) = pack8(bb);
            } else if constexpr (KIND == SVLA_EPI_BIAS_RESID) {
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] = round_bf(v[q] + bb[q]) + o[q];
            } else if constexpr (KIND == SVLA_EPI_BIAS_GELU_ERF) {
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] = gelu_erf(round_bf(v[q] + bb[q]));
            } else if constexpr (KIND == SVLA_EPI_BIAS_SCALE_RESID) {
              float sc[8];
              unpack8(sq[p], sc);
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] = round_bf(sc[q] * round_bf(v[q] + bb[q])) + o[q];
            } else if constexpr (KIND == SVLA_EPI_GELU_BWD) {
#pragma unroll
              for (int q = 0; q < 8; ++q) v[q] = round_bf(v[q]) * gelu_tanh_grad(o[q]);
            } else if constexpr (KIND == SVLA_EPI_SOFTCAP_CE) {
              // columns in increasing order across p: a strict > keeps the lowest index at the maximum
              mold = mx;
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                v[q] = softcap_bf16_tab(v[q], cap, icap, ltab);
                if (v[q] > mx) { mx = v[q]; am = (int)(nb + 32 * p + q); }
              }
            }
            *reinterpret_cast<u32x4*>(rowp + 32 * p) = pack8(v);
            if constexpr (KIND == SVLA_EPI_SOFTCAP_CE) {
              // online sum of exp against the lane's running max (the previous sum rescaled when the max grew)
              float s8 = 0.f;
#pragma unroll
              for (int q = 0; q < 8; ++q) s8 += __expf(v[q] - mx);
              se = (mold == -INFINITY) ? s8 : se * __expf(mold - mx) + s8;
            }
          });
          if constexpr (KIND == SVLA_EPI_SOFTCAP_CE) {
            // the 128-column group of the row is this wave's half tile: lanes r, r+16, r+32, r+48
            float gm = fmaxf(mx, __shfl_xor(mx, 16, 64));
            gm = fmaxf(gm, __shfl_xor(gm, 32, 64));
            float sg = (mx == -INFINITY) ? 0.f : se * __expf(mx - gm);
            int ag = (mx == gm) ? am : 0x7fffffff;
            sg += __shfl_xor(sg, 16, 64);
            ag = min(ag, __shfl_xor(ag, 16, 64));
            sg += __shfl_xor(sg, 32, 64);
            ag = min(ag, __shfl_xor(ag, 32, 64));
            if (g == 0) {
              const int64_t ntn = (N + 127) / 128;
              float* rs = E.row_stats + (m * ntn + (n0 + 128 * wc) / 128) * 3;
              rs[0] = gm;
              rs[1] = sg;
              rs[2] = __int_as_float(ag);
            }
          }
        });
      };
      switch (kind) {
        case SVLA_EPI_STORE: run(std::integral_constant<int, SVLA_EPI_STORE>{}); break;
        case SVLA_EPI_BIAS: run(std::integral_constant<int, SVLA_EPI_BIAS>{}); break;
        case SVLA_EPI_BIAS_GELU: run(std::integral_constant<int, SVLA_EPI_BIAS_GELU>{}); break;
        case SVLA_EPI_BIAS_RESID: run(std::integral_constant<int, SVLA_EPI_BIAS_RESID>{}); break;
        case SVLA_EPI_BIAS_GELU_ERF: run(std::integral_constant<int, SVLA_EPI_BIAS_GELU_ERF>{}); break;
        case SVLA_EPI_BIAS_SCALE_RESID: run(std::integral_constant<int, SVLA_EPI_BIAS_SCALE_RESID>{}); break;
        case SVLA_EPI_GELU_BWD: run(std::integral_constant<int, SVLA_EPI_GELU_BWD>{}); break;
        case SVLA_EPI_SOFTCAP_CE: run(std::integral_constant<int, SVLA_EPI_SOFTCAP_CE>{}); break;
        default: return false;
      }
    }
    return true;
  };

  auto epilogue = [&](int64_t m0, int64_t n0, const int t) {
    const int lane = t & 63;
    // tile column of B fragment j of the wave (GG: gate columns [0, 128), up columns [128, 256) of the image)
    auto colb = [&](int j) { return GG ? (j & 1) * 128 + 64 * wc + 16 * (j >> 1) : 128 * wc + 16 * j; };
    auto wp = [&](int pass, float* Ei) {
      // pass p holds rows [64p, 64p+64): wave row wr = p >> 1, fragments 4(p&1)..4(p&1)+3.  Quad (i, j) (C^T
      // accumulation): lane l holds row 16 i + (l & 15), columns colb(j) + 4 (l >> 4) .. +3 -> one 16-B LDS store
      if ((pass >> 1) == wr) {
        auto rows = [&](auto H) {
          static_for<0, 32>([&](auto IJ) {
            constexpr int i = decltype(IJ)::value >> 3, j = decltype(IJ)::value & 7;
            const f32x4 v = agpr_get<(4 * decltype(H)::value + i) * 8 + j>();
            const int col = colb(j) + 4 * (lane >> 4);
            const int r = 16 * i + (lane & 15);
            *reinterpret_cast<f32x4*>(Ei + r * (BN + 4) + col) = v;
          });
        };
        if (pass & 1) rows(std::integral_constant<int, 1>{});
        else rows(std::integral_constant<int, 0>{});
      }
    };
    if constexpr (BMX != 256) {  // whole tiles of direct-epilogue kinds only (launch4 checks)
      direct_epilogue(m0, n0, lane);
      return;
    }
    if constexpr (!F8) {
      if (direct_epilogue(m0, n0, lane)) return;
    }
    // fp8: 32x32 blocks (block q = 4i + j in a[16q:16q+15]; register r of a block: row (r&3) + 8(r>>2) + 4(l>>5),
    // column l&31), scaled by the row scales of A and B on the way into the image
    auto wp8 = [&](int pass, float* Ei) {
      if ((pass >> 1) == wr) {
        float csc[4];
        f32x4 rsc[2][4];
        if constexpr (MX) {  // the block scales were applied by the MFMA
#pragma unroll
          for (int j = 0; j < 4; ++j) csc[j] = 1.f;
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int q = 0; q < 4; ++q) rsc[ii][q] = f32x4{1.f, 1.f, 1.f, 1.f};
        } else {
        const __amdgpu_buffer_rsrc_t ra = make_rsrc_n(fs.sa, fs.na * 4), rb = make_rsrc_n(fs.sb, fs.nb * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 128 * wc + 32 * j + (lane & 31);
          const int64_t n = fs.geglu_I ? ((c < 128) ? (n0 >> 1) + c : fs.geglu_I + (n0 >> 1) + (c - 128)) : n0 + c;
          csc[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, (uint32_t)(n * 4), 0, 0));
        }
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int64_t m = m0 + 64 * pass + 32 * ii + 8 * q + 4 * (lane >> 5);
            rsc[ii][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, (uint32_t)(m * 4), 0, 0));
          }
        }
        auto rows = [&](auto H) {
          static_for<0, 32>([&](auto IJ) {
            constexpr int ii = decltype(IJ)::value >> 4, j = (decltype(IJ)::value >> 2) & 3, q4 = decltype(IJ)::value & 3;
            constexpr int i = 2 * decltype(H)::value + ii;
            const f32x4 v = agpr_get<(4 * i + j) * 4 + q4>();
            const int col = 128 * wc + 32 * j + (lane & 31);
            const int r = 32 * ii + 8 * q4 + 4 * (lane >> 5);
#pragma unroll
            for (int q = 0; q < 4; ++q) Ei[(r + q) * (BN + 4) + col] = v[q] * rsc[ii][q4][q] * csc[j];
          });
        };
        if (pass & 1) rows(std::integral_constant<int, 1>{});
        else rows(std::integral_constant<int, 0>{});
      }
    };
    if constexpr (F8) {
      tile_epilogue<BM, BN, NTH, decltype(wp8), true>(M, N, m0, n0, Cd, E, smem, t, wp8);
    } else {
#if G4_STAMPS
    tile_epilogue<BM, BN, NTH, decltype(wp), true>(M, N, m0, n0, Cd, E, smem, t, wp, stmp + 8);
#else
    tile_epilogue<BM, BN, NTH, decltype(wp), true>(M, N, m0, n0, Cd, E, smem, t, wp);
#endif
    }
  };

  const int64_t I = sk.sk_iters, G = sk.grid;
  const int64_t it1 = ((int64_t)L + 1) * I / G;
  int* sflag = reinterpret_cast<int*>(smem);
  int dp_tile = L;
  int64_t it = (int64_t)L * I / G;
  int64_t ithi = it1;
  // The block's work items.  sk.sk_first 0: its data-parallel tiles, then its stream-K k-range from the low end (the
  // tail of one tile, then the head of the next).  1: the stream-K pieces first, last piece first -- every block
  // opens with the head (k = 0) of a tile at the same moment, so the blocks of an XCD that share an operand panel
  // stream the same k-slices together (the low-end order left every block at its own k offset: 2x the L2->fabric
  // fetch of hipBLASLt's stream-K on the q|k|v weight gradient, r4j), and the data-parallel tiles that follow start
  // together too.  Pieces, slabs and the reduction order are the same, so the results are bitwise those of order 0.
  auto next_dp = [&](int& tile, int& kb, int& ke) -> bool {
    if (dp_tile >= sk.dp_tiles) return false;
    tile = dp_tile;
    dp_tile += sk.grid;
    kb = 0;
    ke = nk;
    return true;
  };
  auto next_sk_low = [&](int& tile, int& kb, int& ke, int& st) -> bool {
    if (it >= it1) return false;
    st = (int)(it / nk);
    kb = (int)(it - (int64_t)st * nk);
    ke = (int)min((int64_t)nk, kb + (it1 - it));
    it += ke - kb;
    tile = sk.dp_tiles + st;
    return true;
  };
  auto next_sk_high = [&](int& tile, int& kb, int& ke, int& st) -> bool {
    if (ithi <= it) return false;
    st = (int)((ithi - 1) / nk);
    const int64_t t0 = (int64_t)st * nk, pb = max(it, t0);
    kb = (int)(pb - t0);
    ke = (int)(ithi - t0);
    ithi = pb;
    tile = sk.dp_tiles + st;
    return true;
  };
  auto next_item = [&](int& tile, int& kb, int& ke, int& st) -> bool {
    st = 0;
    if (sk.sk_first) {
      if (next_sk_high(tile, kb, ke, st)) return true;
      st = 0;
      return next_dp(tile, kb, ke);
    } else {
      if (next_dp(tile, kb, ke)) return true;
      return next_sk_low(tile, kb, ke, st);
    }
  };
  // the direct epilogue (below) stores from the accumulators and leaves LDS untouched
  auto direct_ok = [&](int64_t m0, int64_t n0) {
    if constexpr (F8) return false;
    const int kind = E.kind;
    const bool k_ok = GG ? (kind == SVLA_EPI_GEGLU || kind == SVLA_EPI_ROPE) : kind == SVLA_EPI_STORE;
    return k_ok && m0 + BMX <= M && n0 + BN <= N;
  };
  int tile, kb, ke, st;
  bool have = next_item(tile, kb, ke, st), pre = false;
  if constexpr (GG) {  // read by the direct GeGLU epilogue, after the first mainloop's barriers
    if (E.kind == SVLA_EPI_GEGLU) gelu_tab_to_lds(smem + LDS);
  }
#pragma unroll 1
  while (have) {
    int t;
    asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(t_in));
    int64_t m0, n0;
    coords(tile, m0, n0);
#if G4_STAMPS
    const unsigned long long tml = __builtin_amdgcn_s_memtime();
#endif
    mainloop(m0, n0, kb, ke, t & 63, pre);
#if G4_STAMPS
    if (kb != 0 || ke != nk) {
      stmp[11] += __builtin_amdgcn_s_memtime() - tml;
      stmp[12] += ke - kb;
    } else {
      stmp[13] += ke - kb;
    }
#endif
    pre = false;
    if (kb != 0 || ke != nk) {
      // partial tile: the stream-K hand-off of gemm8_kernel (slab per segment, last arriver reduces in k order)
      const int64_t T0 = (int64_t)st * nk, T1 = T0 + nk;
      const int Lh = (int)(((T0 + 1) * G + I - 1) / I - 1);
      const int Ll = (int)min(G - 1, (T1 * G + I - 1) / I - 1);
      const int nseg = Ll - Lh + 1, j = L - Lh;
      auto slab = [&](int seg) {
        return make_rsrc(reinterpret_cast<const f32x4*>(sk.slabs) +
                         (int64_t)(2 * (Lh + seg) + (seg == 0 ? 1 : 0)) * (64 * NTH));
      };
      int* cnt = sk.counters + st;
      bool last = false;
      if (j == 0) {
        if (t == 0) {
          const int c = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sflag[0] = (c == nseg - 1);
          if (c == nseg - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        last = sflag[0] != 0;
        __syncthreads();
      }
      if (!last) {
        const __amdgpu_buffer_rsrc_t rs = slab(j);
        uint32_t vo = t * 16;
        static_for<0, 64>([&](auto Q) {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, agpr_get<decltype(Q)::value>()), rs, vo, 0,
                                                 16);
          vo += NTH * 16;
          asm volatile("" : "+v"(vo));
        });
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
          const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sflag[0] = (old == nseg - 1);
          if (old == nseg - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        last = sflag[0] != 0;
        __syncthreads();
      }
      if (!last) {
        have = next_item(tile, kb, ke, st);
        continue;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int sg = (j != 0) ? 0 : 1; sg < nseg; ++sg) {
        const __amdgpu_buffer_rsrc_t rs = slab(sg);
        const bool first = sg == 0;
        uint32_t vo = t * 16;
        static_for<0, 4>([&](auto A4) {  // 16 accumulator quads in flight per step
          constexpr int a = decltype(A4)::value;
          f32x4 x[16];
#pragma unroll
          for (int u = 0; u < 16; ++u)
            x[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, u * NTH * 16, 16));
          static_for<0, 16>([&](auto U) {
            constexpr int u = decltype(U)::value;
            agpr_set<16 * a + u>(first ? x[u] : agpr_get<16 * a + u>() + x[u]);
          });
          vo += 16 * NTH * 16;
          asm volatile("" : "+v"(vo));
        });
      }
    }
    have = next_item(tile, kb, ke, st);
    if (have && direct_ok(m0, n0)) {  // LDS is free (every wave is past mainloop's closing barrier)
      int64_t m1, n1;
      coords(tile, m1, n1);
      stage_first(m1, n1, kb, ke, t & 63);
      pre = true;
    }
#if G4_STAMPS
    const unsigned long long te0 = __builtin_amdgcn_s_memtime();
#endif
    epilogue(m0, n0, t);
#if G4_STAMPS
    stmp[5] += __builtin_amdgcn_s_memtime() - te0;
    stmp[6] += 1;
#endif
  }
#if G4_STAMPS
  stmp[7] = __builtin_amdgcn_s_memtime() - tk0;
  if ((t_in & 63) == 0)
    for (int i = 0; i < 14; ++i) g4_stamps[blockIdx.x % 16384][w][i] = stmp[i];
#endif
}

#define SVLA_GEMM4_KERNEL(LA_, LB_)                                                                      \
  __global__ __launch_bounds__(256, 1) void gemm4_kernel_##LA_##LB_(                                     \
      int64_t M, int64_t N, int64_t K, svla_operand A, svla_operand B, CDesc Cd, svla_epilogue E, SKArgs sk) { \
    gemm4_body<LA_, LB_>(M, N, K, A, B, Cd, E, sk, F8Scales{});                                          \
  }
SVLA_GEMM4_KERNEL(0, 0)
SVLA_GEMM4_KERNEL(0, 1)
SVLA_GEMM4_KERNEL(1, 0)
SVLA_GEMM4_KERNEL(1, 1)
#undef SVLA_GEMM4_KERNEL
// 192-row tiles (KC A and B): the o and down projections, whose 256-row grids leave most of a last round idle
// (9984 rows: 39 x 9 = 351 tiles on 256 CUs -> 52 x 9 = 468)
#define SVLA_GEMM4_KERNEL192(LB_)                                                                           \
  __global__ __launch_bounds__(256, 1) void gemm4_kernel_0##LB_##_192(                                       \
      int64_t M, int64_t N, int64_t K, svla_operand A, svla_operand B, CDesc Cd, svla_epilogue E, SKArgs sk) { \
    gemm4_body<SVLA_LAYOUT_KC, LB_, false, false, false, 192>(M, N, K, A, B, Cd, E, sk, F8Scales{});        \
  }
SVLA_GEMM4_KERNEL192(0)
#undef SVLA_GEMM4_KERNEL192
// Gemma2 gate|up: B fragments paired gate/up per output block, GeGLU straight from the accumulators
__global__ __launch_bounds__(256, 1) void gemm4_kernel_00g(int64_t M, int64_t N, int64_t K, svla_operand A,
                                                           svla_operand B, CDesc Cd, svla_epilogue E, SKArgs sk) {
  gemm4_body<SVLA_LAYOUT_KC, SVLA_LAYOUT_KC, false, true>(M, N, K, A, B, Cd, E, sk, F8Scales{});
}
__global__ __launch_bounds__(256, 1) void gemm4f8_kernel(int64_t M, int64_t N, int64_t K, svla_operand A, svla_operand B,
                                                         CDesc Cd, svla_epilogue E, SKArgs sk, F8Scales fs) {
  gemm4_body<SVLA_LAYOUT_KC, SVLA_LAYOUT_KC, true>(M, N, K, A, B, Cd, E, sk, fs);
}
// MX: per-32-k E8M0 block scales of both operands fed to the MFMA (staged by LDS-DMA beside the operand tiles)
__global__ __launch_bounds__(256, 1) void gemm4mx_kernel(int64_t M, int64_t N, int64_t K, svla_operand A, svla_operand B,
                                                         CDesc Cd, svla_epilogue E, SKArgs sk, F8Scales fs) {
  gemm4_body<SVLA_LAYOUT_KC, SVLA_LAYOUT_KC, true, false, true>(M, N, K, A, B, Cd, E, sk, fs);
}

template <auto KERN>
void set_lds_once(int bytes) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done = true;
  }
}

template <typename C>
int launch(int64_t M, int64_t N, int64_t K, const svla_operand& A, const svla_operand& B, const CDesc& Cd,
           const svla_epilogue& E, hipStream_t s, SplitArgs sp = SplitArgs{1, nullptr, nullptr}) {
  const int64_t tiles = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
  SVLA_CHECK_ARG(sp.S == 1 || (C::NST > 2 && sp.slabs && sp.counters), "gemm: split-K needs a deep-pipelined tile");
  dim3 grid((unsigned)(tiles * sp.S)), block(C::NTH);
  const int la = A.layout, lb = B.layout;
#define SVLA_LAUNCH(LA_, LB_)                                                                      \
  {                                                                                                \
    set_lds_once<gemm_kernel<C, LA_, LB_>>(C::LDS);                                                \
    hipLaunchKernelGGL((gemm_kernel<C, LA_, LB_>), grid, block, C::LDS, s, M, N, K, A, B, Cd, E, sp);  \
  }
  if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH(0, 0)
  else if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_RC) SVLA_LAUNCH(0, 1)
  else if (la == SVLA_LAYOUT_RC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH(1, 0)
  else SVLA_LAUNCH(1, 1)
#undef SVLA_LAUNCH
  return svla::check_launch("gemm");
}

__global__ void rope_inplace_kernel(int64_t M, bf16_t* __restrict__ c, int64_t ldc, svla_epilogue E);

// The deep-pipelined small-tile instances.  A head-wide RoPE (the partner column D/2 away in another tile) runs as
// the plain product followed by rope_inplace_kernel, which rounds as the epilogue does (bitwise).
template <typename C>
int launch_deep(int64_t M, int64_t N, int64_t K, const svla_operand& A, const svla_operand& B, const CDesc& Cd,
                const svla_epilogue& E, hipStream_t s, SplitArgs sp = SplitArgs{1, nullptr, nullptr}) {
  if (E.kind == SVLA_EPI_ROPE && E.rope_D > C::BN) {
    svla_epilogue E0 = E;
    E0.kind = SVLA_EPI_STORE;
    const int rc = launch<C>(M, N, K, A, B, Cd, E0, s, sp);
    if (rc != 0) return rc;
    const int64_t work = M * (E.rope_cols / E.rope_D) * (E.rope_D / 16);
    hipLaunchKernelGGL(rope_inplace_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, M, Cd.ptr[0], Cd.ld,
                       E);
    return svla::check_launch("gemm (rope pass)");
  }
  return launch<C>(M, N, K, A, B, Cd, E, s, sp);
}

// In-place rotate_half RoPE over the first rope_cols columns of a bf16 [M][ldc] matrix (heads of rope_D
// columns), row m at position m % rope_L: the ROPE epilogue as a separate pass, for the small-M GEMV path.  Same rounding as the epilogue: out = bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)).
// One thread owns 8 columns of the low half of a head and their partners D/2 away, so it reads both before
// writing either.
__global__ void rope_inplace_kernel(int64_t M, bf16_t* __restrict__ c, int64_t ldc, svla_epilogue E) {
  const int hd = E.rope_D, half = hd >> 1, cph = half / 8;  // 8-column chunks per half head
  const int64_t per_row = (int64_t)(E.rope_cols / hd) * cph;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * per_row) return;
  const int64_t m = idx / per_row;
  const int r = (int)(idx % per_row);
  const int head = r / cph, dd = (r % cph) * 8;
  bf16_t* lo = c + m * ldc + (int64_t)head * hd + dd;
  bf16_t* hi = lo + half;
  const int64_t pos = m % E.rope_L;
  float xl[8], xh[8], cs[8], sn[8], ol[8], oh[8];
  unpack8(*reinterpret_cast<const u32x4*>(lo), xl);
  unpack8(*reinterpret_cast<const u32x4*>(hi), xh);
  unpack8(*reinterpret_cast<const u32x4*>((const bf16_t*)E.rope_cos + pos * E.rope_ld + dd), cs);
  unpack8(*reinterpret_cast<const u32x4*>((const bf16_t*)E.rope_sin + pos * E.rope_ld + dd), sn);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ol[j] = round_bf(xl[j] * cs[j]) + round_bf(-xh[j] * sn[j]);
    oh[j] = round_bf(xh[j] * cs[j]) + round_bf(xl[j] * sn[j]);
  }
  *reinterpret_cast<u32x4*>(lo) = pack8(ol);
  *reinterpret_cast<u32x4*>(hi) = pack8(oh);
}

// Small-M GEMM (M <= 8: the decode step of greedy generation, one or a few token rows): y = x W^T streams
// every weight row once from HBM, so it is a GEMV — MFMA tiles of 256 rows would run at M/256 occupancy and
// a 256x256 grid over N leaves most CUs idle.  One wave owns RW output rows (or RW gate/up row pairs for
// GEGLU): each lane reads 16-B chunks of the weight rows (a 1 KiB coalesced sweep per row per step), the M
// activation rows come through L1/L2 (a few KiB, shared by every wave), fp32 dot products finish with a
// butterfly.  Epilogues: STORE, GEGLU (the fused epilogue's rounding: g, u, gelu(g) rounded to bf16), and
// ROPE by the in-place pass after the store.
constexpr int GEMV_MAXM = 8;

// weight row n of a B operand with up to 4 SEG_OUTER segments (q|k|v or gate|up kept in separate tensors)
__device__ __forceinline__ const bf16_t* gemv_row(const svla_operand& B, int64_t n) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < B.nseg && n >= B.seg_start[i]) s = i;
  return (const bf16_t*)B.ptr[s] + (n - B.seg_start[s]) * B.ld;
}

template <int RW, bool GEGLU>
__global__ __launch_bounds__(256) void gemv_kernel(int M, int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                   int64_t ldx, svla_operand B, bf16_t* __restrict__ c,
                                                   int64_t ldc, svla_epilogue E) {
  constexpr int NW = GEGLU ? 2 : 1;  // weight rows per output row
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = wave * RW;
  if (r0 >= rows) return;
  float acc[RW][NW][GEMV_MAXM];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) acc[r][q][m] = 0.f;
#pragma unroll 4
  for (int64_t k = (int64_t)lane * 8; k < K; k += 512) {
    float wf[RW][NW][8];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int64_t n = r0 + r < rows ? r0 + r : rows - 1;
      if constexpr (GEGLU) {  // gate row n in ptr[0], up row n in ptr[1]
        unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>((const bf16_t*)B.ptr[0] + n * B.ld + k)), wf[r][0]);
        unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>((const bf16_t*)B.ptr[1] + n * B.ld + k)), wf[r][NW - 1]);
      } else {
        unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(gemv_row(B, n) + k)), wf[r][0]);
      }
    }
#pragma unroll
    for (int m = 0; m < GEMV_MAXM; ++m) {
      if (m < M) {
        float xf[8];
        unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf);
#pragma unroll
        for (int r = 0; r < RW; ++r)
#pragma unroll
          for (int q = 0; q < NW; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[r][q][m] = fmaf(wf[r][q][j], xf[j], acc[r][q][m]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < GEMV_MAXM; ++m) {
    if (m < M) {
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        float v[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) v[q] = wave_sum(acc[r][q][m]);
        const int64_t n = r0 + r;
        if (lane == 0 && n < rows) {
          if constexpr (GEGLU) {
            const float g = round_bf(v[0]), u = round_bf(v[1]);
            c[m * ldc + n] = f2bf(gelu_bf16(g) * u);
            ((bf16_t*)E.out1)[m * E.ld_out1 + n] = f2bf(g);
            ((bf16_t*)E.out2)[m * E.ld_out2 + n] = f2bf(u);
          } else {
            c[m * ldc + n] = f2bf(v[0]);
          }
        }
      }
    }
  }
}

// SOFTCAP_CE at small M (the lm_head of a decode step): one workgroup per 128-column tile of the vocab, each of
// its four waves walks 32 of the tile's rows four at a time and keeps online-softmax partials {max, sumexp,
// argmax} per activation row in registers (logits rounded to bf16, softcapped, rounded again); the four partials
// merge through LDS in wave order into the row_stats record of the MFMA epilogue's layout.  Four waves per tile
// (2073 tiles -> 8292 waves) keep ~4x the weight loads in flight of one wave per tile.
__device__ __forceinline__ void gemv_ce_merge(float& mx, float& se, int& am, float m2, float s2, int a2) {
  if (m2 == -INFINITY) return;
  const float mn = fmaxf(mx, m2);
  se = (mx == -INFINITY ? 0.f : se * __expf(mx - mn)) + s2 * __expf(m2 - mn);
  if (m2 > mx || (m2 == mx && a2 < am)) am = a2;
  mx = mn;
}

__global__ __launch_bounds__(256) void gemv_softcap_kernel(int M, int64_t N, int64_t K, const bf16_t* __restrict__ x,
                                                           int64_t ldx, const bf16_t* __restrict__ w, int64_t ldw,
                                                           bf16_t* __restrict__ c, int64_t ldc, svla_epilogue E) {
#ifndef SVLA_LMHEAD_RW
#define SVLA_LMHEAD_RW 4  // 8: 272.7 us vs 259.9 us per lm_head launch (profiles/r2q_dec*)
#endif
  constexpr int RW = SVLA_LMHEAD_RW;  // vocab rows per step of a wave (32 % RW == 0)
  static_assert(32 % RW == 0, "a wave's 32 rows split into steps of RW");
  __shared__ float part[4][GEMV_MAXM][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  const int64_t ntn = (N + 127) / 128;
  const float cap = E.cap;
  float mx[GEMV_MAXM], se[GEMV_MAXM];
  int am[GEMV_MAXM];
#pragma unroll
  for (int m = 0; m < GEMV_MAXM; ++m) { mx[m] = -INFINITY; se[m] = 0.f; am[m] = 0x7fffffff; }
  const int64_t tend = (tile + 1) * 128 < N ? (tile + 1) * 128 : N;
  const int64_t wbeg = tile * 128 + wv * 32;
  const int64_t nend = wbeg + 32 < tend ? wbeg + 32 : tend;
  for (int64_t r0 = wbeg; r0 < nend; r0 += RW) {
    float acc[RW][GEMV_MAXM];
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) acc[r][m] = 0.f;
  #pragma unroll 4
  for (int64_t k = (int64_t)lane * 8; k < K; k += 512) {
      float wf[RW][8];
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        const int64_t n = r0 + r < nend ? r0 + r : nend - 1;
        unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w + n * ldw + k)), wf[r]);
      }
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) {
        if (m < M) {
          float xf[8];
          unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf);
#pragma unroll
          for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[r][m] = fmaf(wf[r][j], xf[j], acc[r][m]);
        }
      }
    }
#pragma unroll
    for (int m = 0; m < GEMV_MAXM; ++m) {
      if (m < M) {
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const int64_t n = r0 + r;
          const float v = softcap_bf16_tab(wave_sum(acc[r][m]), cap, 1.0f / cap, svla_tanh_bf16_tab);
          if (n < nend) {
            if (lane == 0) c[m * ldc + n] = f2bf(v);
            if (v > mx[m]) {
              se[m] = se[m] * __expf(mx[m] - v) + 1.0f;
              mx[m] = v;
              am[m] = (int)n;
            } else {
              se[m] += __expf(v - mx[m]);
            }
          }
        }
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < GEMV_MAXM; ++m) {
      part[wv][m][0] = mx[m];
      part[wv][m][1] = se[m];
      part[wv][m][2] = __int_as_float(am[m]);
    }
  }
  __syncthreads();
  if (threadIdx.x < M) {
    const int m = threadIdx.x;
    float tm = -INFINITY, ts = 0.f;
    int ta = 0x7fffffff;
    for (int q = 0; q < 4; ++q) gemv_ce_merge(tm, ts, ta, part[q][m][0], part[q][m][1], __float_as_int(part[q][m][2]));
    float* rs = E.row_stats + (m * ntn + tile) * 3;
    rs[0] = tm;
    rs[1] = ts;
    rs[2] = __int_as_float(ta);
  }
}

// Long-K STORE GEMV (the down projection, K = 9216): the four waves of a workgroup split one row's K range, so
// a row is streamed by 256 lanes instead of 64 (4x the loads in flight per row), and the partial dots are
// summed through LDS in wave order (deterministic).
__global__ __launch_bounds__(256) void gemv_splitk_kernel(int M, int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                          int64_t ldx, svla_operand B, bf16_t* __restrict__ c,
                                                          int64_t ldc) {
  __shared__ float part[4][GEMV_MAXM];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t n = blockIdx.x;
  const bf16_t* wr = gemv_row(B, n);
  float acc[GEMV_MAXM];
#pragma unroll
  for (int m = 0; m < GEMV_MAXM; ++m) acc[m] = 0.f;
  if (K <= 5 * 2048) {  // the down projection (K = 9216): every chunk of the lane's K range in flight at once
    constexpr int KCH = 5;
    u32x4 wv[KCH];
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int64_t k = (int64_t)threadIdx.x * 8 + i * 2048;
      if (k < K) wv[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr + k));
    }
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int64_t k = (int64_t)threadIdx.x * 8 + i * 2048;
      if (k < K) {
        float wf[8];
        unpack8(wv[i], wf);
#pragma unroll
        for (int m = 0; m < GEMV_MAXM; ++m) {
          if (m < M) {
            float xf[8];
            unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[m] = fmaf(wf[j], xf[j], acc[m]);
          }
        }
      }
    }
  } else {
#pragma unroll 4
    for (int64_t k = (int64_t)threadIdx.x * 8; k < K; k += 2048) {
      float wf[8];
      unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr + k)), wf);
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) {
        if (m < M) {
          float xf[8];
          unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[m] = fmaf(wf[j], xf[j], acc[m]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < GEMV_MAXM; ++m) {
    if (m < M) {
      const float v = wave_sum(acc[m]);
      if (lane == 0) part[w][m] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < M) {
    const int m = threadIdx.x;
    c[m * ldc + n] = f2bf(((part[0][m] + part[1][m]) + part[2][m]) + part[3][m]);
  }
}

// Prefetching GEMV: a lane's whole K range (KCH 16-B chunks per weight row, K <= KCH*512) is loaded before the
// first FMA, so a wave has RW*NW*KCH loads in flight instead of the runtime loop's unroll-bounded few -- the
// decode GEMVs are HBM-latency bound (a few MB per launch).  Same products and summation order per lane as
// gemv_kernel, so the results are bitwise equal.
template <int KCH, int RW, bool GEGLU>
__global__ __launch_bounds__(256) void gemv_pf_kernel(int M, int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                      int64_t ldx, svla_operand B, bf16_t* __restrict__ c,
                                                      int64_t ldc, svla_epilogue E) {
  constexpr int NW = GEGLU ? 2 : 1;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t r0 = wave * RW;
  if (r0 >= rows) return;
  u32x4 wv[RW][NW][KCH];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int64_t n = r0 + r < rows ? r0 + r : rows - 1;
    const bf16_t* wr[NW];
    if constexpr (GEGLU) {
      wr[0] = (const bf16_t*)B.ptr[0] + n * B.ld;
      wr[NW - 1] = (const bf16_t*)B.ptr[1] + n * B.ld;
    } else {
      wr[0] = gemv_row(B, n);
    }
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int i = 0; i < KCH; ++i) {
        const int64_t k = (int64_t)lane * 8 + i * 512;
        wv[r][q][i] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr[q] + k)) : u32x4{0, 0, 0, 0};
      }
  }
  float acc[RW][NW][GEMV_MAXM];
#pragma unroll
  for (int r = 0; r < RW; ++r)
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) acc[r][q][m] = 0.f;
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int64_t k = (int64_t)lane * 8 + i * 512;
    if (k < K) {
      float wf[RW][NW][8];
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int q = 0; q < NW; ++q) unpack8(wv[r][q][i], wf[r][q]);
#pragma unroll
      for (int m = 0; m < GEMV_MAXM; ++m) {
        if (m < M) {
          float xf[8];
          unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf);
#pragma unroll
          for (int r = 0; r < RW; ++r)
#pragma unroll
            for (int q = 0; q < NW; ++q)
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[r][q][m] = fmaf(wf[r][q][j], xf[j], acc[r][q][m]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < GEMV_MAXM; ++m) {
    if (m < M) {
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        float v[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) v[q] = wave_sum(acc[r][q][m]);
        const int64_t n = r0 + r;
        if (lane == 0 && n < rows) {
          if constexpr (GEGLU) {
            const float g = round_bf(v[0]), u = round_bf(v[1]);
            c[m * ldc + n] = f2bf(gelu_bf16(g) * u);
            ((bf16_t*)E.out1)[m * E.ld_out1 + n] = f2bf(g);
            ((bf16_t*)E.out2)[m * E.ld_out2 + n] = f2bf(u);
          } else {
            c[m * ldc + n] = f2bf(v[0]);
          }
        }
      }
    }
  }
}

template <int KCH, int RW, bool GEGLU>
void launch_gemv_pf(int M, int64_t rows, int64_t K, const svla_operand& A, const svla_operand& B, bf16_t* c,
                    int64_t ldc, const svla_epilogue& E, hipStream_t s) {
  const int64_t waves = (rows + RW - 1) / RW;
  hipLaunchKernelGGL((gemv_pf_kernel<KCH, RW, GEGLU>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, M, rows,
                     K, (const bf16_t*)A.ptr[0], A.ld, B, c, ldc, E);
}

// K chunk count of the prefetching GEMV for this K (0 = no instance: the runtime-loop kernels)
inline int gemv_pf_kch(int64_t K) {
  const int64_t kch = (K + 511) / 512;
  return (kch == 4 || kch == 5) ? (int)kch : 0;  // K = 9216 (down): the split-K kernel stays ahead (11.7 vs 13.2 us)
}

template <bool GEGLU>
bool try_gemv_pf(int variant, int M, int64_t rows, int64_t K, const svla_operand& A, const svla_operand& B,
                 bf16_t* c, int64_t ldc, const svla_epilogue& E, hipStream_t s) {
  const int kch = gemv_pf_kch(K);
  if (kch == 0 || variant == 6) return false;
  const bool rw2 = variant == 7;
#define SVLA_GEMV_PF(KC)                                                                   \
  if (kch == KC) {                                                                         \
    if (rw2) launch_gemv_pf<KC, 2, GEGLU>(M, rows, K, A, B, c, ldc, E, s);                 \
    else launch_gemv_pf<KC, 1, GEGLU>(M, rows, K, A, B, c, ldc, E, s);                     \
    return true;                                                                           \
  }
  SVLA_GEMV_PF(4)
  SVLA_GEMV_PF(5)
#undef SVLA_GEMV_PF
  return false;
}

// Decode GEMV with the two preceding Gemma2 norms in its prologue (svla_gemv_rmsnorm2): x = bf16(rms(h; w2)),
// h = bf16(res + bf16(rms(y; w1))) -- rms_add_norm2_kernel's chunk map and reduction order, so h and x are bitwise
// its outputs -- computed per block into LDS, h also stored by block 0; then the prefetching GEMV of gemv_pf_kernel
// on x.  Every thread issues its norm-input loads before its weight loads (vmcnt retires in order: the norm waits
// for its own inputs only), and the norm's block reductions use raw barriers (no vmcnt drain), so the weight stream
// is in flight while the norms run -- one launch and one HBM round trip fewer per fused norm.
constexpr int GN_MAXC = 2;  // norm chunks per thread: K <= 256 * 8 * 2
template <int KCH, bool GEGLU, int MR>
__global__ __launch_bounds__(256) void gemv_norm2_kernel(int M, int64_t rows, int64_t K, const bf16_t* __restrict__ res,
                                                         const bf16_t* __restrict__ y, int64_t ldx,
                                                         const bf16_t* __restrict__ w1, const bf16_t* __restrict__ w2,
                                                         float eps1, float eps2, bf16_t* __restrict__ h_out,
                                                         svla_operand B, bf16_t* __restrict__ c, int64_t ldc,
                                                         svla_epilogue E) {
  constexpr int NW = GEGLU ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) char gn_smem[];  // [M][K] bf16 x, then the reduction slots
  bf16_t* const xs = reinterpret_cast<bf16_t*>(gn_smem);
  float (*red)[4] = reinterpret_cast<float (*)[4]>(gn_smem + (size_t)M * K * 2);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int nch = (int)(K >> 3);
  // norm inputs first (older in vmcnt order than the weight stream)
  u32x4 yv[MR][GN_MAXC], rv[MR][GN_MAXC], w1v[GN_MAXC], w2v[GN_MAXC];
#pragma unroll
  for (int cI = 0; cI < GN_MAXC; ++cI) {
    const int ch = t + cI * 256;
    w1v[cI] = w2v[cI] = u32x4{0u, 0u, 0u, 0u};
    if (ch < nch) {
      w1v[cI] = *reinterpret_cast<const u32x4*>(w1 + ch * 8);
      w2v[cI] = *reinterpret_cast<const u32x4*>(w2 + ch * 8);
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      yv[m][cI] = rv[m][cI] = u32x4{0u, 0u, 0u, 0u};
      if (m < M && ch < nch) {
        yv[m][cI] = *reinterpret_cast<const u32x4*>(y + m * ldx + ch * 8);
        rv[m][cI] = *reinterpret_cast<const u32x4*>(res + m * ldx + ch * 8);
      }
    }
  }
  // weight stream (as gemv_pf_kernel, one row -- or gate|up row pair -- per wave)
  const int64_t r0 = (int64_t)blockIdx.x * 4 + wv;
  const int64_t n = r0 < rows ? r0 : rows - 1;
  u32x4 wt[NW][KCH];
  {
    const bf16_t* wr[NW];
    if constexpr (GEGLU) {
      wr[0] = (const bf16_t*)B.ptr[0] + n * B.ld;
      wr[NW - 1] = (const bf16_t*)B.ptr[1] + n * B.ld;
    } else {
      wr[0] = gemv_row(B, n);
    }
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int i = 0; i < KCH; ++i) {
        const int64_t k = (int64_t)lane * 8 + i * 512;
        wt[q][i] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr[q] + k)) : u32x4{0, 0, 0, 0};
      }
  }
  // the norms, one row at a time (block_sum's order: wave butterfly, then the four waves in order)
  auto bsum = [&](float v, int slot) {
    v = wave_sum(v);
    if (lane == 0) red[slot][wv] = v;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    return ((red[slot][0] + red[slot][1]) + red[slot][2]) + red[slot][3];
  };
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    if (m < M) {
      float v[GN_MAXC][8];
      float ss = 0.f;
#pragma unroll
      for (int cI = 0; cI < GN_MAXC; ++cI)
        if (t + cI * 256 < nch) {
          unpack8(yv[m][cI], v[cI]);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += v[cI][j] * v[cI][j];
        }
      const float rstd1 = rsqrtf(bsum(ss, 0) / (float)K + eps1);
      float ss2 = 0.f;
#pragma unroll
      for (int cI = 0; cI < GN_MAXC; ++cI) {
        const int ch = t + cI * 256;
        if (ch < nch) {
          float wf[8], r[8];
          unpack8(w1v[cI], wf);
          unpack8(rv[m][cI], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v[cI][j] = round_bf(r[j] + round_bf((v[cI][j] * rstd1) * (1.0f + wf[j])));
            ss2 += v[cI][j] * v[cI][j];
          }
          if (blockIdx.x == 0) *reinterpret_cast<u32x4*>(h_out + m * ldx + ch * 8) = pack8(v[cI]);
        }
      }
      const float rstd2 = rsqrtf(bsum(ss2, 1) / (float)K + eps2);
#pragma unroll
      for (int cI = 0; cI < GN_MAXC; ++cI) {
        const int ch = t + cI * 256;
        if (ch < nch) {
          float wf[8], o[8];
          unpack8(w2v[cI], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (v[cI][j] * rstd2) * (1.0f + wf[j]);
          *reinterpret_cast<u32x4*>(xs + m * K + ch * 8) = pack8(o);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (r0 >= rows) return;
  float acc[NW][MR];
#pragma unroll
  for (int q = 0; q < NW; ++q)
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[q][m] = 0.f;
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int64_t k = (int64_t)lane * 8 + i * 512;
    if (k < K) {
      float wf[NW][8];
#pragma unroll
      for (int q = 0; q < NW; ++q) unpack8(wt[q][i], wf[q]);
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        if (m < M) {
          float xf[8];
          unpack8(*reinterpret_cast<const u32x4*>(xs + m * K + k), xf);
#pragma unroll
          for (int q = 0; q < NW; ++q)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[q][m] = fmaf(wf[q][j], xf[j], acc[q][m]);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    if (m < M) {
      float v[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) v[q] = wave_sum(acc[q][m]);
      if (lane == 0) {
        if constexpr (GEGLU) {
          const float g = round_bf(v[0]), u = round_bf(v[1]);
          c[m * ldc + r0] = f2bf(gelu_bf16(g) * u);
          ((bf16_t*)E.out1)[m * E.ld_out1 + r0] = f2bf(g);
          ((bf16_t*)E.out2)[m * E.ld_out2 + r0] = f2bf(u);
        } else {
          c[m * ldc + r0] = f2bf(v[0]);
        }
      }
    }
  }
}

template <int RW, bool GEGLU>
int launch_gemv(int M, int64_t rows, int64_t K, const svla_operand& A, const svla_operand& B, bf16_t* c,
                int64_t ldc, const svla_epilogue& E, hipStream_t s) {
  const int64_t waves = (rows + RW - 1) / RW;
  hipLaunchKernelGGL((gemv_kernel<RW, GEGLU>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, M, rows, K,
                     (const bf16_t*)A.ptr[0], A.ld, B, c, ldc, E);
  return 0;
}

// Per-call dispatch context (no process state: the library is re-entrant across threads and streams).
// variant (tests / tools only, svla_gemm_bf16_ex): 0 = auto (the 4-wave kernel for long-K GEMMs with more than a
// wave of tiles, else 8-phase + stream-K, else the 2-barrier tiles), 1 = 2-barrier kernel, 2 = 8-phase without
// stream-K, 3 = 4-wave kernel for every 256x256 case, 4 = never the 4-wave kernel, 5 = no small-M GEMV path,
// 6 = small-M GEMVs without the prefetching kernel, 7 = the prefetching kernel with two rows per wave,
// 8 = 8-phase + stream-K for every sub-wave grid (tools/prefill_gemm_bench.py).
struct GemmCtx {
  void* ws;          // caller-owned stream-K workspace (slabs + arrival counters), NULL = no stream-K
  size_t ws_bytes;
  int variant;
};

using svla::num_cus;

// Persistent-grid cap of this host thread's GEMM launches (svla_gemm_set_cu_cap; 0 = every CU): the stream-K
// schedules of launch4 / launch8 size their persistent grid by it, so a GEMM queued on a side stream (the weight
// gradients beside the input-gradient chain, functional._SideWork) leaves CUs free for the main stream's kernels
// instead of holding every CU until it is done.
thread_local int g_cu_cap = 0;
int grid_cus() {
  const int g = num_cus();
  return g_cu_cap > 0 && g_cu_cap < g ? g_cu_cap : g;
}

#ifndef G4_SKMIN
// fewest k-tiles per block of the 4-wave kernel's stream-K share before a full wave of tiles is folded in as well:
// 4, not 8 -- the o-projection dgrad (312 tiles, K = 2304) ran all-stream-K at 8 (every tile split, a 256 KB slab
// per block) and 256 whole tiles + 56 split ones at 4: 132 -> 109 us (tools/gemm_ab.py, profiles/r4f_gemm_ab.txt)
#define G4_SKMIN 4
#endif

#ifndef G4_NOSK
#define G4_NOSK 0  // diagnostic builds: 1 = the 4-wave kernel never splits tiles (data-parallel rounds only)
#endif
#ifndef G4_SKMIN_NK
#define G4_SKMIN_NK 64  // fewest k-tiles per tile for the 4-wave kernel's stream-K schedule (launch4)
#endif
#ifndef G4_SKMIN_NK_SUB
#define G4_SKMIN_NK_SUB 64  // the same floor for grids under 3/4 of a wave of tiles (diagnostic A/B)
#endif
#ifndef G8_SKMIN_NK
#define G8_SKMIN_NK 0  // the same for the 8-phase kernel (launch8); 0 = no floor
#endif
// 2 slabs per block + one arrival counter per stream-K tile (at most 2G - 1 of them)
size_t sk_workspace_bytes(int G) { return (size_t)2 * G * 32 * p8::NTH * 16 + (size_t)2 * G * sizeof(int); }

#ifndef WIDE_DEEP
// the 128 x 256 deep tiles (3 stages) among the short-M candidates: measured no faster than the 4-wave kernel on the
// one shape the estimate gives them (gate|up GeGLU at 299 rows: 55.0 vs 53.4 us) and far slower where forced
// elsewhere (profiles/r8z_prefill_split_ab.txt), so off; variants 16 / 17 keep them for A/B
#define WIDE_DEEP 0
#endif

// Split-K factor of a deep-pipelined small-tile GEMM: as many splits as keep the grid within one wave of blocks
// (G / tiles), at least 4 k-tiles a split, at most 16; the slabs and the per-tile counters must fit the stream-K
// workspace's layout (slab region of 2G 256 KiB slabs, 2G counters behind it).  S = 1: no split.
template <typename C>
SplitArgs split_args(int64_t M, int64_t N, int64_t K, const GemmCtx& ctx) {
  const int G = grid_cus() * deep_bpc<C>();
  const int64_t tiles = ((M + C::BM - 1) / C::BM) * ((N + C::BN - 1) / C::BN);
  const int64_t nk = (K + BK - 1) / BK;
  int64_t S = tiles < G ? G / tiles : 1;
  S = std::min<int64_t>(S, std::min<int64_t>(nk / 4, 16));
  constexpr int64_t SLAB = (int64_t)C::TM * C::TN * C::NTH * 16;
  const int64_t slab_region = (int64_t)2 * num_cus() * 32 * p8::NTH * 16;
  if (S < 2 || !ctx.ws || ctx.ws_bytes < sk_workspace_bytes(num_cus()) || tiles > 2 * num_cus() ||
      tiles * S * SLAB > slab_region)
    return SplitArgs{1, nullptr, nullptr};
  return SplitArgs{(int)S, reinterpret_cast<float*>(ctx.ws),
                   reinterpret_cast<int*>(reinterpret_cast<char*>(ctx.ws) + slab_region)};
}

int launch8(int64_t M, int64_t N, int64_t K, const svla_operand& A, const svla_operand& B, const CDesc& Cd,
            const svla_epilogue& E, const GemmCtx& ctx, hipStream_t s) {
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  SKArgs sk;
  memset(&sk, 0, sizeof(sk));
  sk.nk = (int)((K + BK - 1) / BK);
  sk.dp_tiles = (int)tiles;
  sk.grid = (int)tiles;
  // stream-K over the tiles of the last, partial wave of the grid (persistent grid = one block per CU)
  const int G = grid_cus();
  const int64_t rem = tiles % G;
  int64_t sk_tiles = tiles < G ? tiles : rem;
  // fewer than 8 k-tiles per block would split a tile over too many slabs: fold one more full wave into SK
  if (sk_tiles * sk.nk < 8 * G && tiles >= rem + G) sk_tiles = rem + G;
  if (tiles > G && rem * 4 >= 3 * G) sk_tiles = 0;  // last wave nearly full: nothing to balance
  const size_t need = sk_workspace_bytes(num_cus());  // the chip-wide layout (counters behind num_cus() slabs)
  if (ctx.variant != 2 && sk.nk >= G8_SKMIN_NK && ctx.ws && ctx.ws_bytes >= need && sk_tiles > 0 &&
      sk_tiles < 2 * G && sk_tiles * sk.nk >= 8 * G) {
    sk.dp_tiles = (int)(tiles - sk_tiles);
    sk.grid = G;
    sk.sk_iters = sk_tiles * sk.nk;
    sk.slabs = reinterpret_cast<float*>(ctx.ws);
    // the workspace layout is that of the whole chip (svla_gemm_workspace_bytes): the arrival counters sit behind the
    // slabs of num_cus() blocks whatever grid this launch uses (a capped grid must not move them onto slab memory)
    sk.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(ctx.ws) + (size_t)2 * num_cus() * 32 * p8::NTH * 16);
  }
  dim3 grid((unsigned)sk.grid), block(p8::NTH);
  const int la = A.layout, lb = B.layout;
#define SVLA_LAUNCH8(LA_, LB_)                                                                         \
  {                                                                                                    \
    set_lds_once<gemm8_kernel<LA_, LB_>>(p8::LDS);                                                     \
    hipLaunchKernelGGL((gemm8_kernel<LA_, LB_>), grid, block, p8::LDS, s, M, N, K, A, B, Cd, E, sk);    \
  }
  if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH8(0, 0)
  else if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_RC) SVLA_LAUNCH8(0, 1)
  else if (la == SVLA_LAYOUT_RC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH8(1, 0)
  else SVLA_LAUNCH8(1, 1)
#undef SVLA_LAUNCH8
  return svla::check_launch("gemm8");
}

#ifndef G4_192
#define G4_192 1  // diagnostic builds: 0 = never the 192-row tiles
#endif
// fraction of the CU-rounds a data-parallel grid of t tiles keeps busy
static double dp_fill(int64_t t, int G) { return (double)t / (double)(((t + G - 1) / G) * G); }

int launch4(int64_t M, int64_t N, int64_t K, const svla_operand& A, const svla_operand& B, const CDesc& Cd,
            const svla_epilogue& E, const GemmCtx& ctx, hipStream_t s, const F8Scales* fs = nullptr) {
  // 192-row tiles, data-parallel: whole tiles (M % 192, N % 256), KC A without row segments, one C segment, a direct
  // epilogue kind, and a grid the 256-row tiles fill badly -- 9984 x 2304 (o fwd, q|k|v dgrad): 351 tiles on 256
  // CUs keep 69 % of two rounds busy, 468 tiles of 3/4 the work 91 %
  // Epilogue STORE (the direct epilogue's kind on plain tiles); up to 192 k-tiles: longer k-loops amortise the
  // stream-K hand-off of the 256-row grid better (gate/up dgrad, 288 k-tiles: 0.670 ms stream-K vs 0.723 ms here;
  // down fwd, 144: 0.345 vs 0.303; o fwd 0.100 -> 0.084 ms; profiles/r5q_gemm_ab_192.txt).  B KC only, i.e. the
  // forward projections x W^T: the input-gradient GEMMs (B = W read RC) were 12-16 % faster alone too, but in the
  // layer backward their weight-gradient partner runs beside them on the side stream (functional._SideWork) and
  // already fills the CUs the 256-row grid leaves idle -- there the 192-row grid took them away from it (block A/B:
  // forward -20 us, backward +20 us, profiles/r5r_*).
  if (G4_192 && !fs && A.layout == SVLA_LAYOUT_KC && B.layout == SVLA_LAYOUT_KC && E.kind == SVLA_EPI_STORE &&
      M % 192 == 0 && N % 256 == 0 && Cd.n == 1 && A.nseg <= 1 && B.seg_dim != SVLA_SEG_GEGLU &&
      (K + BK - 1) / BK <= 192) {
    const int G = num_cus();
    const int64_t t256 = ((M + 255) / 256) * (N / 256), t192 = (M / 192) * (N / 256);
    if (t192 >= G && dp_fill(t192, G) >= dp_fill(t256, G) + 0.15) {
      SKArgs sk;
      memset(&sk, 0, sizeof(sk));
      sk.nk = (int)((K + BK - 1) / BK);
      sk.dp_tiles = (int)t192;
      sk.grid = (int)t192;
      dim3 grid((unsigned)sk.grid), block(p4::NTH);
#define SVLA_LAUNCH4_192(LB_)                                                                                \
  {                                                                                                          \
    static bool lds_set = false;                                                                             \
    if (!lds_set) {                                                                                          \
      (void)hipFuncSetAttribute((const void*)gemm4_kernel_0##LB_##_192, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                p4::LDS);                                                                    \
      lds_set = true;                                                                                        \
    }                                                                                                        \
    hipLaunchKernelGGL(gemm4_kernel_0##LB_##_192, grid, block, p4::LDS, s, M, N, K, A, B, Cd, E, sk);         \
  }
      SVLA_LAUNCH4_192(0)
#undef SVLA_LAUNCH4_192
      return svla::check_launch("gemm4 (192-row tiles)");
    }
  }
  const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
  SKArgs sk;
  memset(&sk, 0, sizeof(sk));
  sk.nk = (int)((K + BK - 1) / BK);
  sk.dp_tiles = (int)tiles;
  sk.grid = (int)tiles;
  const int G = grid_cus();
  const int64_t rem = tiles % G;
  int64_t sk_tiles = tiles < G ? tiles : rem;
  if (sk_tiles * sk.nk < G4_SKMIN * G && tiles >= rem + G) sk_tiles = rem + G;
  if (tiles > G && rem * 4 >= 3 * G) sk_tiles = 0;
  const size_t need = sk_workspace_bytes(num_cus());  // the chip-wide layout (counters behind num_cus() slabs)
  // stream-K only from 64 k-tiles a tile: below that the slab hand-off costs more than the data-parallel tail round
  // it replaces (tools/gemm_ab.py, profiles/r5e_gemm_ab_nosk.txt, same box, interleaved: data-parallel rounds were
  // 3-7 % faster for q|k|v fwd, o fwd / dgrad and down dgrad at 32-36 k-tiles and 34-37 % faster for sub-wave grids
  // (252 tiles at K = 2048, SigLIP o fwd); stream-K stays 3-19 % ahead from 64 k-tiles up: q|k|v dgrad, down fwd,
  // gate/up dgrad / wgrad, every weight gradient)
  const int skmin_nk = tiles * 4 < 3 * G ? G4_SKMIN_NK_SUB : G4_SKMIN_NK;
  if (!G4_NOSK && sk.nk >= skmin_nk && ctx.ws && ctx.ws_bytes >= need && sk_tiles > 0 && sk_tiles < 2 * G &&
      sk_tiles * sk.nk >= G4_SKMIN * G) {
    sk.dp_tiles = (int)(tiles - sk_tiles);
    sk.grid = G;
    sk.sk_iters = sk_tiles * sk.nk;
    // long stream-K shares run first (tools/gemm_ab.py, profiles/r4k_skorder.txt: q|k|v wgrad 237 -> 175 us, gate/up
    // dgrad 705 -> 666, wgrad 697 -> 659, down fwd 366 -> 347); short ones (the o projection, SigLIP at K = 1152) were
    // 5-12 % slower that way
    sk.sk_first = sk.sk_iters >= (int64_t)G4_SKFIRST_MIN * G ? 1 : 0;
    sk.slabs = reinterpret_cast<float*>(ctx.ws);
    // the workspace layout is that of the whole chip (svla_gemm_workspace_bytes): the arrival counters sit behind the
    // slabs of num_cus() blocks whatever grid this launch uses (a capped grid must not move them onto slab memory)
    sk.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(ctx.ws) + (size_t)2 * num_cus() * 32 * p8::NTH * 16);
  }
  dim3 grid((unsigned)sk.grid), block(p4::NTH);
#define SVLA_LAUNCH4(LA_, LB_)                                                                       \
  {                                                                                                  \
    static bool lds_set = false;                                                                     \
    if (!lds_set) {                                                                                  \
      (void)hipFuncSetAttribute((const void*)gemm4_kernel_##LA_##LB_, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                p4::LDS);                                                            \
      lds_set = true;                                                                                \
    }                                                                                                \
    hipLaunchKernelGGL(gemm4_kernel_##LA_##LB_, grid, block, p4::LDS, s, M, N, K, A, B, Cd, E, sk);   \
  }
  if (fs && fs->ma) {  // MX block scales: 2 KiB of scale rows per operand stage behind the operand images
    static bool lds_set = false;
    constexpr int lds = p4::LDS + 2 * 2048;
    if (!lds_set) {
      (void)hipFuncSetAttribute((const void*)gemm4mx_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      lds_set = true;
    }
    hipLaunchKernelGGL(gemm4mx_kernel, grid, block, lds, s, M, N, K, A, B, Cd, E, sk, *fs);
    return svla::check_launch("gemm4 mxfp8");
  }
  if (fs) {
    static bool lds_set = false;
    if (!lds_set) {
      (void)hipFuncSetAttribute((const void*)gemm4f8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, p4::LDS);
      lds_set = true;
    }
    hipLaunchKernelGGL(gemm4f8_kernel, grid, block, p4::LDS, s, M, N, K, A, B, Cd, E, sk, *fs);
    return svla::check_launch("gemm4 fp8");
  }
  const int la = A.layout, lb = B.layout;
  // GeGLU (B: two KC GEGLU segments, checked by the dispatcher) and head_dim-256 RoPE (q|k|v): the paired kernel
  if (E.kind == SVLA_EPI_GEGLU ||
      (E.kind == SVLA_EPI_ROPE && E.rope_D == 256 && la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_KC)) {
    static bool lds_set = false;
    if (!lds_set) {
      (void)hipFuncSetAttribute((const void*)gemm4_kernel_00g, hipFuncAttributeMaxDynamicSharedMemorySize,
                                p4::LDS_GELU);
      lds_set = true;
    }
    hipLaunchKernelGGL(gemm4_kernel_00g, grid, block, p4::LDS_GELU, s, M, N, K, A, B, Cd, E, sk);
    return svla::check_launch("gemm4 geglu");
  }
  if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH4(0, 0)
  else if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_RC) SVLA_LAUNCH4(0, 1)
  else if (la == SVLA_LAYOUT_RC && lb == SVLA_LAYOUT_KC) SVLA_LAUNCH4(1, 0)
  else SVLA_LAUNCH4(1, 1)
#undef SVLA_LAUNCH4
  return svla::check_launch("gemm4");
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }


int check_operand(const svla_operand* op, const char* name, int64_t R, int64_t K) {
  SVLA_CHECK_ARG(op != nullptr, "gemm: operand %s is NULL", name);
  SVLA_CHECK_ARG(op->layout == SVLA_LAYOUT_KC || op->layout == SVLA_LAYOUT_RC, "gemm: %s bad layout", name);
  SVLA_CHECK_ARG(op->nseg >= 1 && op->nseg <= 4, "gemm: %s nseg=%d", name, op->nseg);
  SVLA_CHECK_ARG(op->ld % 8 == 0 && op->ld > 0, "gemm: %s ld=%lld must be a positive multiple of 8", name,
                 (long long)op->ld);
  for (int i = 0; i < op->nseg; ++i) {
    SVLA_CHECK_ARG(op->ptr[i] != nullptr && aligned16(op->ptr[i]), "gemm: %s ptr[%d] null or not 16-B aligned",
                   name, i);
  }
  if (op->seg_dim == SVLA_SEG_GEGLU) {
    SVLA_CHECK_ARG(op->nseg == 2 && op->layout == SVLA_LAYOUT_KC, "gemm: GEGLU operand needs 2 KC segments");
    SVLA_CHECK_ARG(op->seg_start[1] * 2 == R && op->seg_start[1] % 64 == 0,
                   "gemm: GEGLU rows per weight must be N/2 and a multiple of 64");
  } else if (op->nseg > 1) {
    const int64_t tile = op->seg_dim == SVLA_SEG_OUTER ? 128 : BK;
    SVLA_CHECK_ARG(op->seg_start[0] == 0, "gemm: %s seg_start[0] must be 0", name);
    for (int i = 1; i < op->nseg; ++i)
      SVLA_CHECK_ARG(op->seg_start[i] % tile == 0 && op->seg_start[i] > op->seg_start[i - 1],
                     "gemm: %s segment %d start %lld not tile aligned (%lld)", name, i, (long long)op->seg_start[i],
                     (long long)tile);
  }
  const int64_t kv = op->k_valid > 0 ? op->k_valid : K;
  // KC: a 16-B chunk straddling the reduction extent would multiply garbage into every output -> the
  // extent must be a multiple of 8 (zero-pad).  RC: a straddling chunk only feeds outputs beyond R,
  // which are never stored (the row of a [K][ld] matrix is readable up to ld >= round8(R)).
  if (op->layout == SVLA_LAYOUT_KC)
    SVLA_CHECK_ARG(kv % 8 == 0, "gemm: %s (KC) reduction extent %lld must be a multiple of 8 (zero-pad)", name,
                   (long long)kv);
  return 0;
}

}  // namespace

extern "C" size_t svla_gemm_workspace_bytes(void) { return sk_workspace_bytes(num_cus()); }

extern "C" void svla_gemm_set_cu_cap(int cap) { g_cu_cap = cap > 0 ? cap : 0; }

#if G4_STAMPS
extern "C" int svla_diag_g4_stamps(void* host, size_t bytes) {  // diagnostic builds only (not in svla.h)
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g4_stamps), bytes < sizeof(g4_stamps) ? bytes : sizeof(g4_stamps)) ==
                 hipSuccess ? 0 : 2;
}
extern "C" int svla_diag_g4_stamps_clear(void) {  // zero the stamp table (blocks of an earlier, larger grid)
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g4_stamps)) != hipSuccess) return 2;
  return hipMemset(p, 0, sizeof(g4_stamps)) == hipSuccess ? 0 : 2;
}
#endif

namespace {
int gemm_dispatch(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                  void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                  const svla_epilogue* epi, const GemmCtx& ctx, void* stream);
}  // namespace

extern "C" int svla_gemm_bf16(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                              void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                              const svla_epilogue* epi, void* workspace, size_t ws_bytes, void* stream) {
  return svla_gemm_bf16_ex(M, N, K, A, B, c_ptr, c_seg_start, c_nseg, ldc, epi, workspace, ws_bytes, 0, stream);
}

extern "C" int svla_gemm_bf16_ex(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                                 void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                                 const svla_epilogue* epi, void* workspace, size_t ws_bytes, int32_t variant,
                                 void* stream) {
  SVLA_CHECK_ARG(variant >= 0 && variant <= 17, "gemm: variant %d", variant);
  SVLA_CHECK_ARG(workspace == nullptr || ((uintptr_t)workspace & 255) == 0, "gemm workspace must be 256-B aligned");
  SVLA_CHECK_ARG(!epi || !epi->mx_q, "gemm: the MX copy of C (epi->mx_q) is an fp8-GEMM output only");
  GemmCtx ctx;
  ctx.ws = workspace;
  ctx.ws_bytes = workspace ? ws_bytes : 0;
  ctx.variant = variant;
  return gemm_dispatch(M, N, K, A, B, c_ptr, c_seg_start, c_nseg, ldc, epi, ctx, stream);
}

extern "C" int svla_gemv_rmsnorm2(int64_t M, int64_t N, int64_t K, const void* res, const void* y, int64_t ldx,
                                  const void* w1, const void* w2, float eps1, float eps2, void* h_out,
                                  const svla_operand* B, void* c, int64_t ldc, const svla_epilogue* epi, void* stream) {
  SVLA_CHECK_ARG(M >= 1 && M <= GEMV_MAXM && N > 0 && K > 0 && K % 8 == 0 && K <= 2560 && K <= 256 * 8 * GN_MAXC,
                 "gemv_rmsnorm2: M in [1, %d], K a multiple of 8 <= 2560", GEMV_MAXM);
  SVLA_CHECK_ARG(res && y && w1 && w2 && h_out && B && c && epi, "gemv_rmsnorm2: NULL argument");
  SVLA_CHECK_ARG(!epi->mx_q, "gemv_rmsnorm2: the MX copy of C (epi->mx_q) is an fp8-GEMM output only");
  SVLA_CHECK_ARG(ldx % 8 == 0 && ldx >= K && ldc % 8 == 0, "gemv_rmsnorm2: ldx >= K and ldc multiples of 8");
  SVLA_CHECK_ARG(B->layout == SVLA_LAYOUT_KC && B->ld % 8 == 0, "gemv_rmsnorm2: B must be KC with ld % 8 == 0");
  const bool geglu = epi->kind == SVLA_EPI_GEGLU;
  SVLA_CHECK_ARG(geglu || (epi->kind == SVLA_EPI_STORE && !epi->accumulate && epi->alpha == 1.0f),
                 "gemv_rmsnorm2: epilogue STORE (plain) or GEGLU");
  if (geglu)
    SVLA_CHECK_ARG(B->nseg == 2 && B->seg_dim == SVLA_SEG_GEGLU && B->seg_start[1] * 2 == N && epi->out1 && epi->out2,
                   "gemv_rmsnorm2: GEGLU needs two B segments of N/2 rows and out1/out2");
  const int64_t rows = geglu ? N / 2 : N;
  const int kch = (int)((K + 511) / 512);
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  const size_t lds = (size_t)M * K * 2 + 2 * 4 * sizeof(float);  // x rows + reduction slots: occupancy as the GEMV's
  hipStream_t s = (hipStream_t)stream;
#define SVLA_GN1(KC, GG, MR)                                                                                       \
  hipLaunchKernelGGL((gemv_norm2_kernel<KC, GG, MR>), grid, block, lds, s, (int)M, rows, K, (const bf16_t*)res,     \
                     (const bf16_t*)y, ldx, (const bf16_t*)w1, (const bf16_t*)w2, eps1, eps2, (bf16_t*)h_out, *B,     \
                     (bf16_t*)c, ldc, *epi)
  // MR: rows held in registers (the norm inputs of every row are loaded up front; M = 1 is the batch-1 decode step)
#define SVLA_GN(KC, GG) \
  if (M == 1) SVLA_GN1(KC, GG, 1); else SVLA_GN1(KC, GG, GEMV_MAXM);
  if (geglu) {
    if (kch <= 4) { SVLA_GN(4, true) } else { SVLA_GN(5, true) }
  } else {
    if (kch <= 4) { SVLA_GN(4, false) } else { SVLA_GN(5, false) }
  }
#undef SVLA_GN
#undef SVLA_GN1
  return svla::check_launch("gemv_rmsnorm2");
}

namespace {
int gemm_dispatch(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                  void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                  const svla_epilogue* epi, const GemmCtx& ctx, void* stream) {
  const int variant = ctx.variant;
  SVLA_CHECK_ARG(M > 0 && N > 0 && K > 0, "gemm: bad sizes M=%lld N=%lld K=%lld", (long long)M, (long long)N,
                 (long long)K);
  SVLA_CHECK_ARG(epi != nullptr, "gemm: epilogue is NULL");
  if (int rc = check_operand(A, "A", M, K)) return rc;
  if (int rc = check_operand(B, "B", N, K)) return rc;
  SVLA_CHECK_ARG(A->seg_dim != SVLA_SEG_GEGLU, "gemm: GEGLU segmentation is for B only");
  SVLA_CHECK_ARG((epi->kind == SVLA_EPI_GEGLU) == (B->seg_dim == SVLA_SEG_GEGLU && B->nseg == 2),
                 "gemm: EPI_GEGLU requires B with SVLA_SEG_GEGLU and vice versa");
  SVLA_CHECK_ARG(ldc % 8 == 0, "gemm: ldc must be a multiple of 8");
  SVLA_CHECK_ARG(c_nseg >= 1 && c_nseg <= 4, "gemm: c_nseg");
  CDesc C;
  C.n = c_nseg;
  C.ld = ldc;
  for (int i = 0; i < 4; ++i) C.ptr[i] = nullptr;
  for (int i = 0; i < 5; ++i) C.start[i] = 0;
  const bool needs_c = !(epi->kind == SVLA_EPI_GEGLU_BWD);
  for (int i = 0; i < c_nseg; ++i) {
    C.ptr[i] = (bf16_t*)c_ptr[i];
    C.start[i] = c_seg_start ? c_seg_start[i] : 0;
    SVLA_CHECK_ARG(!needs_c || (C.ptr[i] && aligned16(C.ptr[i])), "gemm: C ptr[%d] null or misaligned", i);
    if (i > 0) SVLA_CHECK_ARG(C.start[i] % 128 == 0, "gemm: C segment start must be a multiple of 128");
  }
  switch (epi->kind) {
    case SVLA_EPI_STORE: break;
    case SVLA_EPI_BIAS: SVLA_CHECK_ARG(epi->bias && aligned16(epi->bias), "gemm: bias"); break;
    case SVLA_EPI_BIAS_GELU:
      SVLA_CHECK_ARG(epi->bias && epi->out1 && epi->ld_out1 % 8 == 0, "gemm: BIAS_GELU needs bias,out1");
      break;
    case SVLA_EPI_BIAS_RESID: SVLA_CHECK_ARG(epi->in0 && epi->ld_in0 % 8 == 0, "gemm: BIAS_RESID needs in0"); break;
    case SVLA_EPI_GEGLU:
      SVLA_CHECK_ARG(epi->out1 && epi->out2 && epi->ld_out1 % 8 == 0 && epi->ld_out2 % 8 == 0,
                     "gemm: GEGLU needs out1,out2");
      break;
    case SVLA_EPI_GEGLU_BWD:
      SVLA_CHECK_ARG(epi->in0 && epi->in1 && epi->out1 && epi->out2, "gemm: GEGLU_BWD needs in0,in1,out1,out2");
      SVLA_CHECK_ARG(aligned16(epi->in0) && aligned16(epi->in1) && aligned16(epi->out1) && aligned16(epi->out2) &&
                         epi->ld_in0 % 8 == 0 && epi->ld_in1 % 8 == 0 && epi->ld_out1 % 8 == 0 &&
                         epi->ld_out2 % 8 == 0,
                     "gemm: GEGLU_BWD operands must be 16-B aligned rows");
      break;
    case SVLA_EPI_GELU_BWD: SVLA_CHECK_ARG(epi->in0, "gemm: GELU_BWD needs in0"); break;
    case SVLA_EPI_BIAS_GELU_ERF: SVLA_CHECK_ARG(epi->bias && aligned16(epi->bias), "gemm: BIAS_GELU_ERF needs bias"); break;
    case SVLA_EPI_BIAS_SCALE_RESID:
      SVLA_CHECK_ARG(epi->colscale && epi->in0 && epi->ld_in0 % 8 == 0 && (!epi->bias || aligned16(epi->bias)),
                     "gemm: BIAS_SCALE_RESID needs colscale, in0");
      break;
    case SVLA_EPI_SOFTCAP_CE: SVLA_CHECK_ARG(epi->row_stats && epi->cap > 0.f, "gemm: SOFTCAP_CE needs row_stats, cap"); break;
    case SVLA_EPI_ROPE:
      SVLA_CHECK_ARG(epi->rope_cos && epi->rope_sin && epi->rope_L > 0 && epi->rope_D >= 16 &&
                         epi->rope_D % 16 == 0 && epi->rope_D <= 256 && (256 % epi->rope_D) == 0 &&
                         epi->rope_ld % 8 == 0 && epi->rope_cols % epi->rope_D == 0 && epi->rope_cols <= N,
                     "gemm: ROPE needs cos/sin tables, rope_L, rope_D in {16,32,64,128,256}, rope_cols a multiple of D");
      SVLA_CHECK_ARG(c_nseg == 1, "gemm: ROPE writes one C matrix");
      break;
    default: SVLA_CHECK_ARG(false, "gemm: unknown epilogue %d", epi->kind);
  }
  if (epi->accumulate) SVLA_CHECK_ARG(epi->kind == SVLA_EPI_STORE, "gemm: accumulate only with EPI_STORE");
  hipStream_t s = (hipStream_t)stream;
  // tile choice: the largest tile that still gives >= ~2 waves of blocks on the 256 CUs (1 block/CU);
  // segment boundaries (outer segments, output segments, GeGLU halves) must not split a tile
  auto tiles = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  auto seg_ok = [&](int bm, int bn) {
    if (B->seg_dim == SVLA_SEG_GEGLU && (B->seg_start[1] % (bn / 2)) != 0) return false;
    bool ok = true;
    if (B->nseg > 1 && B->seg_dim == SVLA_SEG_OUTER)
      for (int i = 1; i < B->nseg; ++i) ok = ok && (B->seg_start[i] % bn == 0);
    if (A->nseg > 1 && A->seg_dim == SVLA_SEG_OUTER)
      for (int i = 1; i < A->nseg; ++i) ok = ok && (A->seg_start[i] % bm == 0);
    for (int i = 1; i < c_nseg; ++i) ok = ok && (C.start[i] % bm == 0);
    return ok;
  };
  const bool kseg = (A->nseg > 1 && A->seg_dim == SVLA_SEG_K) || (B->nseg > 1 && B->seg_dim == SVLA_SEG_K);
  const int64_t nk = (K + BK - 1) / BK;
  const bool sk_ok = variant != 2 && ctx.ws && ctx.ws_bytes >= sk_workspace_bytes(num_cus());
  // 4-wave kernel: ahead of the 8-phase one in the training step (tools/ab_prof.sh: kernel traces of bench.py
  // paired per call) once the k-loop is long enough to amortise its tile prologue/epilogue, the grid has more
  // than a wave of tiles and the epilogue is light -- it runs the epilogue on half the waves, so GEGLU-backward
  // (+31%), softcap-CE (+9%) and RoPE (+2%) stay on the 8-wave kernel, as do short-K / sub-wave shapes
  // decode-sized M: the GEMV path (STORE / GEGLU / ROPE, both operands K-contiguous, plain C)
  {
    const bool ek_ok = epi->kind == SVLA_EPI_STORE || epi->kind == SVLA_EPI_GEGLU ||
                       epi->kind == SVLA_EPI_SOFTCAP_CE || (epi->kind == SVLA_EPI_ROPE && epi->rope_D % 16 == 0);
    bool b_ok = epi->kind == SVLA_EPI_GEGLU ? (B->nseg == 2 && B->seg_start[1] == N / 2)
                                            : (B->nseg == 1 || (B->seg_dim == SVLA_SEG_OUTER &&
                                                                epi->kind != SVLA_EPI_SOFTCAP_CE));
    for (int i = 0; i < B->nseg; ++i) b_ok = b_ok && aligned16(B->ptr[i]);
    if (M <= GEMV_MAXM && ek_ok && b_ok && variant != 5 && !epi->accumulate && epi->alpha == 1.0f &&
        A->layout == SVLA_LAYOUT_KC && B->layout == SVLA_LAYOUT_KC && A->nseg == 1 && K % 8 == 0 &&
        A->ld % 8 == 0 && B->ld % 8 == 0 && (A->r_valid == 0 || A->r_valid >= M) &&
        (A->k_valid == 0 || A->k_valid >= K) && (B->r_valid == 0 || B->r_valid >= N) &&
        (B->k_valid == 0 || B->k_valid >= K) && c_nseg == 1 && C.start[0] == 0 && aligned16(A->ptr[0]) &&
        aligned16(B->ptr[0])) {
      bf16_t* c0 = C.ptr[0];
      if (epi->kind == SVLA_EPI_SOFTCAP_CE) {
        const int64_t ntn = (N + 127) / 128;
        hipLaunchKernelGGL(gemv_softcap_kernel, dim3((unsigned)ntn), dim3(256), 0, s, (int)M, N, K,
                           (const bf16_t*)A->ptr[0], A->ld, (const bf16_t*)B->ptr[0], B->ld, c0, ldc, *epi);
      } else if (epi->kind == SVLA_EPI_GEGLU) {
        if (!try_gemv_pf<true>(variant, (int)M, N / 2, K, *A, *B, c0, ldc, *epi, s))
          launch_gemv<1, true>((int)M, N / 2, K, *A, *B, c0, ldc, *epi, s);
      } else if (try_gemv_pf<false>(variant, (int)M, N, K, *A, *B, c0, ldc, *epi, s)) {
      } else if (K > 4096) {
        hipLaunchKernelGGL(gemv_splitk_kernel, dim3((unsigned)N), dim3(256), 0, s, (int)M, N, K,
                           (const bf16_t*)A->ptr[0], A->ld, *B, c0, ldc);
      } else if (N < 8192) {
        launch_gemv<1, false>((int)M, N, K, *A, *B, c0, ldc, *epi, s);
      } else {
        launch_gemv<2, false>((int)M, N, K, *A, *B, c0, ldc, *epi, s);
      }
      if (epi->kind == SVLA_EPI_ROPE) {
        const int64_t work = M * (epi->rope_cols / epi->rope_D) * (epi->rope_D / 16);
        hipLaunchKernelGGL(rope_inplace_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, M, c0, ldc,
                           *epi);
      }
      return svla::check_launch("gemm (small-M GEMV)");
    }
  }
  const int64_t t256 = tiles(256, 256);
  // The 4-wave kernel's direct epilogue (stores straight from the accumulators, gemm4_body) made it the faster kernel
  // for the light epilogues from one k-tile loop of 512 up and from a quarter wave of tiles (tools/gemm_bench.py:
  // o fwd 129 -> 106 us, down dgrad 422 -> 354 us, SigLIP qkv BIAS 89 -> 82 us; head_dim-256 ROPE
  // rotates in registers on the paired-fragment kernel, bitwise the 8-phase kernel's).  VALU-heavy or load-carrying epilogues stay on the 8-phase kernel, whose
  // two waves per SIMD run them faster than one wave does from registers (tools/epi_ab.py, tools/gemm_epi_bench.py:
  // SOFTCAP_CE 13.4 vs 16.4 ms, BIAS_GELU_ERF 270 vs 312 us, GELU_BWD 178 vs 224 us, BIAS_RESID 127 vs 138 us).
  // The k-loop floor is 384: the lm_head weight gradient (265344 x 2304 x 416) runs 0.70 ms here vs 0.85 ms on the
  // 8-phase kernel (tools/gemm_probe.py); head_dim-256 RoPE stores from the paired accumulators (qkv 0.23 -> 0.19 ms).
  const int ek = epi->kind;
  // (GEGLU_BWD measured in the direct epilogue of its own 4-wave instance, loads one row block ahead, r4: block
  // fwd+bwd 5.00 -> 5.11 ms against plain dgrad + svla_geglu_bwd; the pass stays separate)
  const bool light_epi = ek == SVLA_EPI_STORE || ek == SVLA_EPI_BIAS || ek == SVLA_EPI_GEGLU || ek == SVLA_EPI_ROPE;
  const bool use4 = !kseg && seg_ok(256, 256) &&
                    (variant == 3 || ((variant == 0 || variant >= 5) && light_epi && K >= 384 && 4 * t256 >= num_cus()));
  // forced deep-pipelined small tiles (tools/gemma_prefill_gemm_bench.py A/B): KC x KC, no k segments, whole
  // 64-column GeGLU halves
  if (variant >= 10 && A->layout == SVLA_LAYOUT_KC && B->layout == SVLA_LAYOUT_KC && !kseg &&
      ek != SVLA_EPI_SOFTCAP_CE && !(ek == SVLA_EPI_GEGLU && epi->mx_q)) {
    const int cv = variant == 17 ? 16 : (variant >= 13 && variant <= 15 ? variant - 3 : variant);
    const bool split = variant >= 13 && variant != 16;
    if (cv == 16 && seg_ok(128, 256))
      return launch_deep<CfgWideD>(M, N, K, *A, *B, C, *epi, s, split ? split_args<CfgWideD>(M, N, K, ctx) : SplitArgs{1, nullptr, nullptr});
    if (cv == 10 && seg_ok(64, 64))
      return launch_deep<CfgTinyD>(M, N, K, *A, *B, C, *epi, s, split ? split_args<CfgTinyD>(M, N, K, ctx) : SplitArgs{1, nullptr, nullptr});
    if (cv == 11 && seg_ok(64, 128))
      return launch_deep<CfgNarrowD>(M, N, K, *A, *B, C, *epi, s, split ? split_args<CfgNarrowD>(M, N, K, ctx) : SplitArgs{1, nullptr, nullptr});
    if (cv == 12 && seg_ok(128, 128))
      return launch_deep<CfgSmallD>(M, N, K, *A, *B, C, *epi, s, split ? split_args<CfgSmallD>(M, N, K, ctx) : SplitArgs{1, nullptr, nullptr});
  }
  // Short-M grids (the B = 1 prefill: Gemma2 at 299 prompt tokens, SigLIP at 256, BEiT at 577 patches): a block's
  // k-loop there is bound by what one CU can pull into LDS (~50-70 GB/s a CU, MI355X_MICROARCH.md ldsdma-fill /
  // ring-gemm), so the tile and split-K factor are the ones with the fewest bytes per block per wave of blocks:
  // operand fill (BM + BN) x k per k-tile, plus for a split tile its slab store and the reducer's S slab reads
  // (weighted 2x: latency-bound single-block reads).  The 256 x 256 data-parallel estimate stands for the 4-wave /
  // 8-phase path, which keeps ties (gate|up GeGLU at 299 rows: 55.7 vs 62.3 us).  Measured per shape in
  // profiles/r8z_prefill_split_ab.txt: Gemma2 q|k|v+RoPE 68.6 -> 26.9 us, down 68.6 -> 38.5, SigLIP fc2 34.1 ->
  // 18.2, BEiT fc2 33.2 -> 22.0.
  if (variant == 0 && M <= 1024 && A->layout == SVLA_LAYOUT_KC && B->layout == SVLA_LAYOUT_KC && !kseg &&
      ek != SVLA_EPI_SOFTCAP_CE && !(ek == SVLA_EPI_GEGLU && epi->mx_q)) {
    auto est = [&](int bm, int bn, int S, int bpc) {
      const int G = grid_cus() * bpc;
      const double waves = (double)((tiles(bm, bn) * S + G - 1) / G);
      const double fill = (double)nk / S * BK * (bm + bn) * 2;
      return waves * (fill + (S > 1 ? (double)bm * bn * 4 * (1 + 2 * S) : 0.0));
    };
    const SplitArgs s64 = split_args<CfgTinyD>(M, N, K, ctx), s64n = split_args<CfgNarrowD>(M, N, K, ctx),
                    s128 = split_args<CfgSmallD>(M, N, K, ctx), s128w = split_args<CfgWideD>(M, N, K, ctx);
    const double e64 = seg_ok(64, 64) ? est(64, 64, s64.S, deep_bpc<CfgTinyD>()) : 1e30;
    const double e64n = seg_ok(64, 128) ? est(64, 128, s64n.S, deep_bpc<CfgNarrowD>()) : 1e30;
    const double e128 = seg_ok(128, 128) ? est(128, 128, s128.S, deep_bpc<CfgSmallD>()) : 1e30;
    const double e128w = (WIDE_DEEP && seg_ok(128, 256)) ? est(128, 256, s128w.S, deep_bpc<CfgWideD>()) : 1e30;
    const double ebig = seg_ok(256, 256) ? est(256, 256, 1, 1) : 1e30;
    const double best = std::min(std::min(e64, e64n), std::min(e128, e128w));
    if (best < ebig) {
      if (best == e64n) return launch_deep<CfgNarrowD>(M, N, K, *A, *B, C, *epi, s, s64n);
      if (best == e64) return launch_deep<CfgTinyD>(M, N, K, *A, *B, C, *epi, s, s64);
      if (best == e128) return launch_deep<CfgSmallD>(M, N, K, *A, *B, C, *epi, s, s128);
      return launch_deep<CfgWideD>(M, N, K, *A, *B, C, *epi, s, s128w);
    }
  }
  if (epi->kind == SVLA_EPI_ROPE && epi->rope_D > 128) {  // a head must fit one 256-wide tile
    SVLA_CHECK_ARG(seg_ok(256, 256), "gemm: ROPE with head_dim > 128 needs 256-aligned segments");
    if (use4) return launch4(M, N, K, *A, *B, C, *epi, ctx, s);
    if (variant != 1 && !kseg) return launch8(M, N, K, *A, *B, C, *epi, ctx, s);
    return launch<CfgBig>(M, N, K, *A, *B, C, *epi, s);
  }
  if (use4) return launch4(M, N, K, *A, *B, C, *epi, ctx, s);
  // Sub-wave grids (the B = 1 prefill: SigLIP / BEiT at 256 / 577 tokens): 128x128 tiles leave most CUs idle and a
  // launch costs one tile's k-loop latency; 64x64 tiles put 4x the blocks on the chip.  Epilogues whose partials or
  // halves assume a 128-column group (softcap-CE, GeGLU) and the head-wide ROPE keep the larger tiles.
  // (both operands KC: the projections x @ W^T of the prefill; the RC staging of this kernel needs 128-wide tiles).
  // 19.7 -> 14.9 us (BEiT q|k|v), 18.4 -> 11.4 (BEiT o), 52 -> 34 (BEiT fc2), 19.7 -> 12.5 (SigLIP q|k|v), bitwise
  // the 128x128 result (tools/prefill_gemm_bench.py, profiles/r3n_prefill_gemm_ab.txt).
  if ((variant == 0 || variant == 9) && tiles(128, 128) < num_cus() && seg_ok(64, 64) &&
      A->layout == SVLA_LAYOUT_KC && B->layout == SVLA_LAYOUT_KC && ek != SVLA_EPI_SOFTCAP_CE &&
      ek != SVLA_EPI_GEGLU && ek != SVLA_EPI_ROPE)
    return launch<CfgTiny>(M, N, K, *A, *B, C, *epi, s);
  if (variant != 1 && !kseg && seg_ok(256, 256) &&
      (tiles(256, 256) >= 512 || (sk_ok && tiles(256, 256) * nk >= 8 * num_cus()) || (variant == 8 && sk_ok)))
    return launch8(M, N, K, *A, *B, C, *epi, ctx, s);
  if (tiles(256, 256) >= 512 && seg_ok(256, 256)) return launch<CfgBig>(M, N, K, *A, *B, C, *epi, s);
  if (tiles(256, 128) >= 256 && seg_ok(256, 128)) return launch<CfgMid>(M, N, K, *A, *B, C, *epi, s);
  SVLA_CHECK_ARG(seg_ok(128, 128), "gemm: segment starts must be multiples of 128");
  return launch<CfgSmall>(M, N, K, *A, *B, C, *epi, s);
}

}  // namespace


// ------------------------------------------------------------------------------------------------------------
// fp8 e4m3 GEMM (BASELINE configs[4]): both operands KC fp8 with per-row fp32 scales, the 4-wave kernel in fp8 mode.
// ------------------------------------------------------------------------------------------------------------
namespace {
int gemm_fp8_common(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B, F8Scales fs,
                    void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                    const svla_epilogue* epi, void* workspace, size_t ws_bytes, void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && K > 0 && K % 16 == 0, "gemm_fp8: sizes M=%lld N=%lld K=%lld (K multiple of 16)",
                 (long long)M, (long long)N, (long long)K);
  SVLA_CHECK_ARG(A && B && epi, "gemm_fp8: NULL argument");
  SVLA_CHECK_ARG(workspace == nullptr || ((uintptr_t)workspace & 255) == 0, "gemm workspace must be 256-B aligned");
  for (const svla_operand* op : {A, B}) {
    SVLA_CHECK_ARG(op->layout == SVLA_LAYOUT_KC, "gemm_fp8: operands must be KC (reduction dim contiguous)");
    SVLA_CHECK_ARG(op->ld > 0 && op->ld % 16 == 0, "gemm_fp8: ld %lld must be a positive multiple of 16",
                   (long long)op->ld);
    SVLA_CHECK_ARG((op->k_valid > 0 ? op->k_valid : K) % 16 == 0, "gemm_fp8: k_valid must be a multiple of 16");
    for (int i = 0; i < op->nseg; ++i) SVLA_CHECK_ARG(op->ptr[i] && aligned16(op->ptr[i]), "gemm_fp8: operand ptr");
  }
  SVLA_CHECK_ARG(A->nseg == 1, "gemm_fp8: A has one segment");
  const bool geglu = epi->kind == SVLA_EPI_GEGLU;
  SVLA_CHECK_ARG(geglu ? (B->nseg == 2 && B->seg_dim == SVLA_SEG_GEGLU && B->seg_start[1] * 2 == N &&
                          B->seg_start[1] % 128 == 0)
                       : B->nseg == 1,
                 "gemm_fp8: B is one segment, or two GEGLU segments of N/2 rows (multiple of 128) with EPI_GEGLU");
  SVLA_CHECK_ARG(!epi->accumulate, "gemm_fp8: accumulate unsupported");
  SVLA_CHECK_ARG(!epi->mx_q || epi->kind == SVLA_EPI_GEGLU, "gemm_fp8: the MX copy of C is a GEGLU output");
  switch (epi->kind) {
    case SVLA_EPI_STORE: break;
    case SVLA_EPI_BIAS: SVLA_CHECK_ARG(epi->bias && aligned16(epi->bias), "gemm_fp8: bias"); break;
    case SVLA_EPI_BIAS_RESID: SVLA_CHECK_ARG(epi->in0 && epi->ld_in0 % 8 == 0, "gemm_fp8: BIAS_RESID needs in0"); break;
    case SVLA_EPI_GEGLU:
      SVLA_CHECK_ARG(epi->out1 && epi->out2 && epi->ld_out1 % 8 == 0 && epi->ld_out2 % 8 == 0,
                     "gemm_fp8: GEGLU needs out1,out2");
      SVLA_CHECK_ARG(!epi->mx_q || (epi->mx_scales && (N / 2) % 128 == 0 && epi->mx_ldq >= N / 2 &&
                                    epi->mx_ldq % 8 == 0 && ((uintptr_t)epi->mx_q & 7) == 0 &&
                                    ((uintptr_t)epi->mx_scales & 3) == 0 && epi->mx_sld >= 4 * M &&
                                    epi->mx_sld % 4 == 0),
                     "gemm_fp8: GEGLU MX copy of h: N/2 % 128 == 0, mx_ldq >= N/2 (8-B rows), mx_sld >= 4 M");
      break;
    case SVLA_EPI_ROPE:
      SVLA_CHECK_ARG(epi->rope_cos && epi->rope_sin && epi->rope_L > 0 && epi->rope_D >= 16 && epi->rope_D % 16 == 0 &&
                         epi->rope_D <= 256 && (256 % epi->rope_D) == 0 && epi->rope_ld % 8 == 0 &&
                         epi->rope_cols % epi->rope_D == 0 && epi->rope_cols <= N,
                     "gemm_fp8: ROPE tables / sizes");
      SVLA_CHECK_ARG(c_nseg == 1, "gemm_fp8: ROPE writes one C matrix");
      break;
    default: SVLA_CHECK_ARG(false, "gemm_fp8: epilogue %d unsupported (STORE, BIAS, BIAS_RESID, GEGLU, ROPE)", epi->kind);
  }
  SVLA_CHECK_ARG(ldc % 8 == 0 && c_nseg >= 1 && c_nseg <= 4, "gemm_fp8: ldc / c_nseg");
  CDesc C;
  C.n = c_nseg;
  C.ld = ldc;
  for (int i = 0; i < 4; ++i) C.ptr[i] = nullptr;
  for (int i = 0; i < 5; ++i) C.start[i] = 0;
  for (int i = 0; i < c_nseg; ++i) {
    C.ptr[i] = (bf16_t*)c_ptr[i];
    C.start[i] = c_seg_start ? c_seg_start[i] : 0;
    SVLA_CHECK_ARG(C.ptr[i] && aligned16(C.ptr[i]), "gemm_fp8: C ptr[%d] null or misaligned", i);
    if (i > 0) SVLA_CHECK_ARG(C.start[i] % 256 == 0, "gemm_fp8: C segment start must be a multiple of 256");
  }
  // k units of two fp8 values: the bf16 staging machinery runs unchanged on them
  svla_operand A2 = *A, B2 = *B;
  A2.ld /= 2;
  B2.ld /= 2;
  A2.k_valid /= 2;
  B2.k_valid /= 2;
  fs.na = A->r_valid > 0 ? A->r_valid : M;
  fs.nb = geglu ? 2 * B->seg_start[1] : (B->r_valid > 0 ? B->r_valid : N);
  fs.geglu_I = geglu ? B->seg_start[1] : 0;
  GemmCtx ctx;
  ctx.ws = workspace;
  ctx.ws_bytes = workspace ? ws_bytes : 0;
  ctx.variant = 0;
  return launch4(M, N, K / 2, A2, B2, C, *epi, ctx, (hipStream_t)stream, &fs);
}
}  // namespace

extern "C" int svla_gemm_fp8(int64_t M, int64_t N, int64_t K, const svla_operand* A, const float* a_scale,
                             const svla_operand* B, const float* b_scale, void* const* c_ptr,
                             const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc, const svla_epilogue* epi,
                             void* workspace, size_t ws_bytes, void* stream) {
  SVLA_CHECK_ARG(a_scale && b_scale && aligned16(a_scale) && aligned16(b_scale),
                 "gemm_fp8: row scales must be non-NULL and 16-B aligned");
  F8Scales fs;
  memset(&fs, 0, sizeof(fs));
  fs.sa = a_scale;
  fs.sb = b_scale;
  return gemm_fp8_common(M, N, K, A, B, fs, c_ptr, c_seg_start, c_nseg, ldc, epi, workspace, ws_bytes, stream);
}

extern "C" int svla_gemm_mxfp8(int64_t M, int64_t N, int64_t K, const svla_operand* A, const void* a_mx,
                               int64_t a_mx_ld, int64_t a_mx_bytes, const svla_operand* B, const void* b_mx,
                               int64_t b_mx_ld, int64_t b_mx_bytes, void* const* c_ptr, const int64_t* c_seg_start,
                               int32_t c_nseg, int64_t ldc, const svla_epilogue* epi, void* workspace,
                               size_t ws_bytes, void* stream) {
  SVLA_CHECK_ARG(a_mx && b_mx && ((uintptr_t)a_mx & 3) == 0 && ((uintptr_t)b_mx & 3) == 0,
                 "gemm_mxfp8: block scales must be non-NULL and 4-B aligned");
  SVLA_CHECK_ARG(K % 128 == 0 && (A->k_valid == 0 || A->k_valid % 128 == 0) && (B->k_valid == 0 || B->k_valid % 128 == 0),
                 "gemm_mxfp8: K and k_valid must be multiples of 128 (whole MX k-tiles)");
  const int64_t ra = A->r_valid > 0 ? A->r_valid : M;
  const int64_t rb = epi->kind == SVLA_EPI_GEGLU ? N : (B->r_valid > 0 ? B->r_valid : N);
  SVLA_CHECK_ARG(a_mx_ld >= 4 * ra && b_mx_ld >= 4 * rb && a_mx_ld % 4 == 0 && b_mx_ld % 4 == 0,
                 "gemm_mxfp8: scale tile strides must cover 4 bytes per row");
  SVLA_CHECK_ARG(a_mx_bytes >= (K / 128 - 1) * a_mx_ld + 4 * ra && b_mx_bytes >= (K / 128 - 1) * b_mx_ld + 4 * rb &&
                     a_mx_bytes < ((int64_t)1 << 31) && b_mx_bytes < ((int64_t)1 << 31),
                 "gemm_mxfp8: scale buffers too small (or >= 2 GiB)");
  F8Scales fs;
  memset(&fs, 0, sizeof(fs));
  fs.ma = (const uint8_t*)a_mx;
  fs.mb = (const uint8_t*)b_mx;
  fs.ma_ld = a_mx_ld;
  fs.mb_ld = b_mx_ld;
  fs.ma_bytes = a_mx_bytes;
  fs.mb_bytes = b_mx_bytes;
  return gemm_fp8_common(M, N, K, A, B, fs, c_ptr, c_seg_start, c_nseg, ldc, epi, workspace, ws_bytes, stream);
}
