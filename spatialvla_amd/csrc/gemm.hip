// bf16 GEMM with fused epilogues for gfx950 (MI355X).
//
// C[M,N] = epi( sum_k A(m,k) B(n,k) )  — one kernel family serves every projection of the
// SpatialVLA hot path, forward and backward (see include/svla.h for the reference call sites).
//
// Design (CDNA4-first):
//  * 128x128x64 block tile, 256 threads = 4 waves in a 2x2 grid, each wave a 64x64 sub-tile of
//    4x4 v_mfma_f32_16x16x32_bf16 accumulators (64-lane operand maps, not 32-lane warp tiles).
//  * Each operand may be KC (reduction dim contiguous: nn.Linear weights, activations) or RC
//    (outer dim contiguous: activations read transposed for dW, weights read for dX). KC tiles
//    are read with ds_read_b128 from an XOR-swizzled [128][64] LDS image; RC tiles are stored
//    [64][128] (swizzled) and read with the gfx950 transpose read ds_read_b64_tr_b16, so no
//    operand is ever transposed in HBM.
//  * Register-staged double buffer: tile k+1 is loaded global->VGPR while tile k feeds the MFMAs,
//    then written to the other LDS buffer; one barrier per K-tile.
//  * Epilogue goes through LDS (fp32, padded rows) so every global store is a 16-B vector along N
//    and every epilogue input (bias, residual, saved activations) is a 16-B vector load.
//  * Block ids are remapped XCD-aware (consecutive tiles share an XCD L2) and grouped along M.
#include "svla_common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NTH = 256;
constexpr int TILE_BYTES = BM * BK * 2;                 // 16 KiB per operand per buffer
constexpr int EPI_LD = 132;                             // fp32 row stride of the epilogue image
constexpr int STAGE_BYTES = 4 * TILE_BYTES;             // A,B x 2 buffers
constexpr int EPI_BYTES = BM * EPI_LD * 4;
constexpr int LDS_BYTES = STAGE_BYTES > EPI_BYTES ? STAGE_BYTES : EPI_BYTES;
constexpr int GROUP_M = 8;

struct SegSel {
  const bf16_t* base;
  int64_t rbase, kbase;  // indices to subtract
};

__device__ __forceinline__ int find_seg(const svla_operand& op, int64_t idx) {
  int s = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < op.nseg && idx >= op.seg_start[i]) s = i;
  return s;
}

__device__ __forceinline__ SegSel select(const svla_operand& op, int64_t r0, int64_t k0) {
  SegSel s;
  if (op.nseg <= 1 || op.seg_dim == SVLA_SEG_GEGLU) {
    s.base = (const bf16_t*)op.ptr[0];
    s.rbase = 0;
    s.kbase = 0;
  } else if (op.seg_dim == SVLA_SEG_OUTER) {
    int i = find_seg(op, r0);
    s.base = (const bf16_t*)op.ptr[i];
    s.rbase = op.seg_start[i];
    s.kbase = 0;
  } else {
    int i = find_seg(op, k0);
    s.base = (const bf16_t*)op.ptr[i];
    s.rbase = 0;
    s.kbase = op.seg_start[i];
  }
  return s;
}

__device__ __forceinline__ u32x4 load8_guard(const bf16_t* p, int64_t n_valid) {
  // n_valid = number of valid elements starting at p (<= 0: none)
  if (n_valid >= 8) return *reinterpret_cast<const u32x4*>(p);
  u32x4 v = {0u, 0u, 0u, 0u};
  if (n_valid > 0) {
    uint16_t tmp[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) tmp[j] = (j < n_valid) ? p[j] : (uint16_t)0;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (uint32_t)tmp[2 * j] | ((uint32_t)tmp[2 * j + 1] << 16);
  }
  return v;
}

// swizzle of the RC image [64 k][16 chunks of 16 B]
__device__ __forceinline__ int rc_swz(int k) { return ((k & 3) | ((k & 8) >> 1)) << 1; }

// ---- global -> registers (4 x 16 B per thread per operand)
template <int LAYOUT>
__device__ __forceinline__ void load_tile(const svla_operand& op, int64_t R, int64_t K, int64_t r0, int64_t k0,
                                          int t, u32x4 (&st)[4]) {
  if (op.seg_dim == SVLA_SEG_GEGLU && op.nseg == 2) {
    // B only, KC: rows 0..63 of the tile from ptr[0] (gate), 64..127 from ptr[1] (up)
    const int64_t I = op.seg_start[1];
    const int c = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int lr = (t >> 3) + 32 * i;
      int64_t n = (r0 >> 1) + (lr & 63);
      const bf16_t* base = (const bf16_t*)op.ptr[lr >> 6];
      int64_t kk = k0 + 8 * c;
      st[i] = (n < I) ? load8_guard(base + n * op.ld + kk, K - kk) : u32x4{0u, 0u, 0u, 0u};
    }
    return;
  }
  SegSel s = select(op, r0, k0);
  if (LAYOUT == SVLA_LAYOUT_KC) {
    const int c = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t r = r0 + (t >> 3) + 32 * i;
      int64_t kk = k0 + 8 * c;
      st[i] = (r < R) ? load8_guard(s.base + (r - s.rbase) * op.ld + (kk - s.kbase), K - kk)
                      : u32x4{0u, 0u, 0u, 0u};
    }
  } else {
    const int c = t & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int64_t k = k0 + (t >> 4) + 16 * i;
      int64_t rr = r0 + 8 * c;
      st[i] = (k < K) ? load8_guard(s.base + (k - s.kbase) * op.ld + (rr - s.rbase), R - rr)
                      : u32x4{0u, 0u, 0u, 0u};
    }
  }
}

// ---- registers -> LDS image
template <int LAYOUT>
__device__ __forceinline__ void store_tile(char* lds, int t, const u32x4 (&st)[4]) {
  if (LAYOUT == SVLA_LAYOUT_KC) {
    const int c = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int row = (t >> 3) + 32 * i;
      *reinterpret_cast<u32x4*>(lds + row * 128 + ((c ^ (row & 7)) << 4)) = st[i];
    }
  } else {
    const int c = t & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int k = (t >> 4) + 16 * i;
      *reinterpret_cast<u32x4*>(lds + k * 256 + ((c ^ rc_swz(k)) << 4)) = st[i];
    }
  }
}

// ---- LDS -> MFMA operand fragment (16 rows starting at rb, k-step ks of 32)
template <int LAYOUT>
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
    const LDS_AS s16x4* a1 = (const LDS_AS s16x4*)(lds + k1 * 256 + ((chunk ^ rc_swz(k1)) << 4) + off);
    const LDS_AS s16x4* a2 = (const LDS_AS s16x4*)(lds + k2 * 256 + ((chunk ^ rc_swz(k2)) << 4) + off);
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

__device__ __forceinline__ void store8(bf16_t* p, const float* v, int64_t n_valid) {
  if (n_valid >= 8) {
    *reinterpret_cast<u32x4*>(p) = pack8(v);
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

template <int LA, int LB>
__global__ __launch_bounds__(NTH, 2) void gemm_kernel(int64_t M, int64_t N, int64_t K, svla_operand A,
                                                       svla_operand B, CDesc C, svla_epilogue E) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  const int total = tiles_m * tiles_n;
  int pid = xcd_remap(blockIdx.x, total);
  const int group = GROUP_M * tiles_n;
  const int first_m = (pid / group) * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (pid % group) % gsz;
  const int tn = (pid % group) / gsz;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;


  const int wr = w >> 1, wc = w & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BK - 1) / BK);
  u32x4 sa[4], sb[4];
  load_tile<LA>(A, M, K, m0, 0, t, sa);
  load_tile<LB>(B, N, K, n0, 0, t, sb);
  store_tile<LA>(smem, t, sa);
  store_tile<LB>(smem + 2 * TILE_BYTES, t, sb);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<LA>(A, M, K, m0, (int64_t)(kt + 1) * BK, t, sa);
      load_tile<LB>(B, N, K, n0, (int64_t)(kt + 1) * BK, t, sb);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = read_frag<LA>(smem + cur * TILE_BYTES, 64 * wr + 16 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = read_frag<LB>(smem + (2 + cur) * TILE_BYTES, 64 * wc + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<LA>(smem + (cur ^ 1) * TILE_BYTES, t, sa);
      store_tile<LB>(smem + (2 + (cur ^ 1)) * TILE_BYTES, t, sb);
    }
    __syncthreads();
  }

  // ---------------- epilogue: accumulators -> LDS fp32 image [128][EPI_LD]
  float* Ei = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = 64 * wc + 16 * j + (lane & 15);
      const int rowb = 64 * wr + 16 * i + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) Ei[(rowb + r) * EPI_LD + col] = acc[i][j][r];
    }
  __syncthreads();

  // output segment (tile aligned along M)
  int cs = 0;
#pragma unroll
  for (int i = 1; i < 4; ++i)
    if (i < C.n && m0 >= C.start[i]) cs = i;
  bf16_t* cbase = C.ptr[cs];
  const int64_t cm0 = C.start[cs];
  const int kind = E.kind;

  if (kind == SVLA_EPI_GEGLU) {
    const int64_t I = N >> 1;
    const int64_t nout0 = n0 >> 1;
    const int cc = t & 7;
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
      const int row = (t >> 3) + 32 * i;
      const int64_t m = m0 + row;
      const int64_t n = nout0 + 8 * cc;
      if (m >= M || n >= I) continue;
      float g[8], u[8], h[8];
      const float* pg = Ei + row * EPI_LD + 8 * cc;
      const float* pu = pg + 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[j] = round_bf(pg[j]);
        u[j] = round_bf(pu[j]);
        h[j] = round_bf(gelu_tanh(g[j])) * u[j];
      }
      store8(cbase + (m - cm0) * C.ld + n, h, I - n);
      store8((bf16_t*)E.out1 + m * E.ld_out1 + n, g, I - n);
      store8((bf16_t*)E.out2 + m * E.ld_out2 + n, u, I - n);
    }
    return;
  }

  const int cc = t & 15;
  const int ntn = tiles_n;
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    const int row = (t >> 4) + 16 * i;
    const int64_t m = m0 + row;
    const int64_t n = n0 + 8 * cc;
    const int64_t nv = N - n;
    float v[8];
    {
      const float* pe = Ei + row * EPI_LD + 8 * cc;
      f32x4 x0 = *reinterpret_cast<const f32x4*>(pe);
      f32x4 x1 = *reinterpret_cast<const f32x4*>(pe + 4);
      v[0] = x0[0]; v[1] = x0[1]; v[2] = x0[2]; v[3] = x0[3];
      v[4] = x1[0]; v[5] = x1[1]; v[6] = x1[2]; v[7] = x1[3];
    }
    if (kind == SVLA_EPI_SOFTCAP_CE) {
      // softcap, round to bf16, per-(row, tile) online-softmax partials over the valid columns
      float mx = -INFINITY, se = 0.f;
      int am = 0x7fffffff;
      const float cap = E.cap, icap = 1.0f / E.cap;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = round_bf(cap * tanhf(v[j] * icap));
        if (j < nv && v[j] > mx) { mx = v[j]; am = (int)(n + j); }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nv) se += __expf(v[j] - mx);
      if (mx == -INFINITY) se = 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        float mx2 = __shfl_xor(mx, o, 64), se2 = __shfl_xor(se, o, 64);
        int am2 = __shfl_xor(am, o, 64);
        float mn = fmaxf(mx, mx2);
        float s1 = (mx == -INFINITY) ? 0.f : se * __expf(mx - mn);
        float s2 = (mx2 == -INFINITY) ? 0.f : se2 * __expf(mx2 - mn);
        int a = (mx > mx2 || (mx == mx2 && am < am2)) ? am : am2;
        mx = mn; se = s1 + s2; am = a;
      }
      if (m < M) {
        if (cc == 0) {
          float* rs = E.row_stats + (m * ntn + tn) * 3;
          rs[0] = mx; rs[1] = se; rs[2] = __int_as_float(am);
        }
        if (nv > 0) store8(cbase + (m - cm0) * C.ld + n, v, nv);
      }
      continue;
    }
    if (m >= M || nv <= 0) continue;
    bf16_t* cp = cbase + (m - cm0) * C.ld + n;
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
          v[j] = gelu_tanh(pre[j]);
        }
        store8((bf16_t*)E.out1 + m * E.ld_out1 + n, pre, nv);
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
          float act = round_bf(gelu_tanh(g[j]));
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
}

template <auto KERN>
void set_lds_once(int bytes) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    done = true;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

int check_operand(const svla_operand* op, const char* name, int64_t R, int64_t K, int64_t tileR) {
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
    int64_t tile = op->seg_dim == SVLA_SEG_OUTER ? tileR : BK;
    SVLA_CHECK_ARG(op->seg_start[0] == 0, "gemm: %s seg_start[0] must be 0", name);
    for (int i = 1; i < op->nseg; ++i)
      SVLA_CHECK_ARG(op->seg_start[i] % tile == 0 && op->seg_start[i] > op->seg_start[i - 1],
                     "gemm: %s segment %d start %lld not tile aligned", name, i, (long long)op->seg_start[i]);
  }
  (void)K;
  return 0;
}

}  // namespace

extern "C" int svla_gemm_bf16(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                              void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                              const svla_epilogue* epi, void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && K > 0, "gemm: bad sizes M=%lld N=%lld K=%lld", (long long)M, (long long)N,
                 (long long)K);
  SVLA_CHECK_ARG(epi != nullptr, "gemm: epilogue is NULL");
  if (int rc = check_operand(A, "A", M, K, BM)) return rc;
  if (int rc = check_operand(B, "B", N, K, BN)) return rc;
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
    if (i > 0) SVLA_CHECK_ARG(C.start[i] % BM == 0, "gemm: C segment start must be a multiple of 128");
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
      break;
    case SVLA_EPI_GELU_BWD: SVLA_CHECK_ARG(epi->in0, "gemm: GELU_BWD needs in0"); break;
    case SVLA_EPI_SOFTCAP_CE: SVLA_CHECK_ARG(epi->row_stats && epi->cap > 0.f, "gemm: SOFTCAP_CE needs row_stats, cap"); break;
    default: SVLA_CHECK_ARG(false, "gemm: unknown epilogue %d", epi->kind);
  }
  if (epi->accumulate) SVLA_CHECK_ARG(epi->kind == SVLA_EPI_STORE, "gemm: accumulate only with EPI_STORE");
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  SVLA_CHECK_ARG(tiles < (1ll << 31), "gemm: too many tiles");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)tiles), block(NTH);
  const int la = A->layout, lb = B->layout;
  if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_KC)
  { set_lds_once<gemm_kernel<0, 0>>(LDS_BYTES);
    hipLaunchKernelGGL((gemm_kernel<0, 0>), grid, block, LDS_BYTES, s, M, N, K, *A, *B, C, *epi); }
  else if (la == SVLA_LAYOUT_KC && lb == SVLA_LAYOUT_RC)
  { set_lds_once<gemm_kernel<0, 1>>(LDS_BYTES);
    hipLaunchKernelGGL((gemm_kernel<0, 1>), grid, block, LDS_BYTES, s, M, N, K, *A, *B, C, *epi); }
  else if (la == SVLA_LAYOUT_RC && lb == SVLA_LAYOUT_KC)
  { set_lds_once<gemm_kernel<1, 0>>(LDS_BYTES);
    hipLaunchKernelGGL((gemm_kernel<1, 0>), grid, block, LDS_BYTES, s, M, N, K, *A, *B, C, *epi); }
  else
  { set_lds_once<gemm_kernel<1, 1>>(LDS_BYTES);
    hipLaunchKernelGGL((gemm_kernel<1, 1>), grid, block, LDS_BYTES, s, M, N, K, *A, *B, C, *epi); }
  return svla::check_launch("gemm");
}
