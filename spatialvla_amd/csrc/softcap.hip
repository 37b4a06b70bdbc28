// Softcap + softmax statistics of raw lm_head logits, in place (svla_softcap_ce_rows; the training step's lm_head
// runs as a plain-store GEMM and this pass follows it -- reference: modeling_gemma2.py final_logit_softcapping and
// the cross-entropy of modeling_spatialvla.py).  A wave covers 512 columns of a row (8 per lane, 16-B loads/stores),
// 16 lanes = one 128-column group: per lane {max, first argmax, sum exp} of its 8 values, then the group combine of
// SOFTCAP_CE's LDS epilogue (same chunk partition, same butterfly), so the statistics are bitwise the fused
// epilogue's.  Persistent blocks.
//
// Two LDS tables per block.  The full-range table ft[b] = softcap(bf16 value with bits b) for every |v| below 511
// (34 KB, built once per block from softcap_bf16_tab, so it is that function by construction) turns the softcap of a
// packed pair into an and, a packed min, two LDS reads and an and-or; every |v| >= 511 (inf included) saturates to
// ft[FT_N - 1] for the caps the launcher admits.  The 1280-entry tanh table serves the generic per-element path,
// which a lane takes for a NaN in its chunk, a ragged row end, or a zero maximum (where the sign of the max depends
// on the scan order).  The per-lane maximum is a v_max3 tree, the first argmax a reverse select chain, the exp
// arguments packed fp32 ops (each op is the scalar op's IEEE result), and the 16-lane butterfly DPP moves.
#include "softcap_tab.h"

#include <algorithm>
#include <cmath>

namespace {
#ifndef SCR_U
#define SCR_U 2  // units per wave group (A/B at the 4B shape, profiles/r6g_softcap_ab.txt: 2 adjacent + pipelined best)
#endif
#ifndef SCR_WPB
#define SCR_WPB 4  // waves per block (four blocks per CU fit the LDS tables)
#endif
#ifndef SCR_BPC
#define SCR_BPC 4  // resident blocks per CU the persistent grid asks for
#endif
#ifndef SCR_ADJ
#define SCR_ADJ 1  // 1: a wave's SU units are adjacent chunks (0: one per wave round)
#endif
#ifndef SCR_PIPE
#define SCR_PIPE 1  // the next group's loads issued before this group's arithmetic
#endif
#ifndef SCR_FT
#define SCR_FT 1  // diagnostic builds: 0 = the generic per-element path only
#endif
constexpr uint32_t TAB_LO = (uint32_t)SVLA_TANH_TAB_E0 << 7, TAB_N = ((uint32_t)SVLA_TANH_TAB_E1 << 7) - TAB_LO;
static_assert(TAB_N * 2 == TANH_TAB_BYTES, "table covers [E0, E1) exactly");
constexpr int FT_N = 0x4400;  // bf16 bits of |v| in [0, 512.0)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// softcap_bf16_tab on a packed bf16 pair, returning the packed bf16 results: the two roundings are one
// v_cvt_pk_bf16_f32 each, and the range tests fold into one unsigned offset d = |a| - lo: d < NTAB indexes the table,
// NTAB <= d <= 0x7f80 - lo (|a| >= 4, inf included) reads the sentinel entry tab[NTAB] = 1.0, and d beyond that (|a|
// below the table: tanh(a) = a in bf16; NaN) keeps |a|.  Bitwise softcap_bf16_tab<_, true> of each element.
template <typename Tab>
__device__ __forceinline__ uint32_t softcap_pair_tab(uint32_t w, float cap, float icap, const Tab& tab) {
  const uint32_t a = pack2(__uint_as_float(w << 16) * icap, __uint_as_float(w & 0xffff0000u) * icap);
  uint32_t t[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t ab = (a >> (16 * h)) & 0x7fffu;
    const uint32_t d = ab - TAB_LO;
    const uint32_t tb = tab[min(d, TAB_N)];
    const uint32_t rb = d > 0x7f80u - TAB_LO ? ab : tb;
    t[h] = (((a >> (16 * h)) & 0x8000u) | rb) << 16;
  }
  return pack2(__uint_as_float(t[0]) * cap, __uint_as_float(t[1]) * cap);
}

// The generic per-element unit: softcap of the lane's nv (<= 8) values, stored, and its {max, first argmax, sum exp}
// by an in-order scan.
typedef const unsigned short* Tab;
__device__ __forceinline__ void unit_generic(const u32x4& w, int64_t nv, int64_t n, bf16_t* p, float cap, float icap,
                                             Tab tab, float& mx, float& se, int& am) {
  float v[8];
  mx = -INFINITY;
  se = 0.f;
  am = 0x7fffffff;
  if (nv >= 8) {  // whole 16-B chunk: packed pairs
    u32x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = softcap_pair_tab(w[i], cap, icap, tab);
    *reinterpret_cast<u32x4*>(p) = o;
    unpack8(o, v);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (v[j] > mx) { mx = v[j]; am = (int)(n + j); }
#pragma unroll
    for (int j = 0; j < 8; ++j) se += __expf(v[j] - mx);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = j < nv ? bf2f(p[j]) : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = softcap_bf16_tab<Tab, true>(v[j], cap, icap, tab);  // v unpacked from bf16 logits
      if (j < nv && v[j] > mx) { mx = v[j]; am = (int)(n + j); }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (j < nv) se += __expf(v[j] - mx);
    for (int j = 0; j < nv; ++j) p[j] = f2bf(v[j]);
  }
  if (mx == -INFINITY) se = 0.f;
}

__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// lane value from the DPP partner: quad_perm [1,0,3,2] / [2,3,0,1] are xor 1 / xor 2; within the 16-lane group the
// half-row and row mirrors (7 - i, 15 - i) land in the other quad / other 8 lanes, which hold the same partial as
// xor 4 / xor 8 once the earlier steps have made the quads and 8-lane halves uniform -- the xor butterfly's result,
// operand for operand.
template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(dpp<CTRL>(__float_as_int(x)));
}
constexpr int DPP_X1 = 0xb1, DPP_X2 = 0x4e, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;

__global__ __launch_bounds__(64 * SCR_WPB) void softcap_rows_kernel(int64_t M, int64_t N, bf16_t* __restrict__ lg, int64_t ld,
                                                           float cap, float* __restrict__ row_stats, int full_tab) {
  __shared__ __attribute__((aligned(16))) unsigned short tab[TANH_TAB_BYTES / 2 + 8];  // + the 1.0 sentinel
  __shared__ __attribute__((aligned(16))) unsigned short ft[FT_N];
  if ((int)threadIdx.x < TANH_TAB_BYTES / 16)
    reinterpret_cast<u32x4*>(tab)[threadIdx.x] = reinterpret_cast<const u32x4*>(svla_tanh_bf16_tab)[threadIdx.x];
  if (threadIdx.x == 0) tab[TAB_N] = 0x3f80;
  __syncthreads();
  const float icap = 1.0f / cap;
  const bool use_ft = SCR_FT && full_tab;
  if (use_ft) {
    for (int b = threadIdx.x; b < FT_N; b += 64 * SCR_WPB)
      ft[b] = f2bf(softcap_bf16_tab<decltype(tab), true>(__uint_as_float((uint32_t)b << 16), cap, icap, tab));
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int64_t cpr = (N + 511) / 512;  // 512-column chunks per row
  const int64_t ntn = (N + 127) / 128;
  const int64_t total = M * cpr;
  // the wave's units walk as (row m, chunk c) pairs, stepped without a per-unit 64-bit division; all of it is
  // wave-uniform (scalar registers).  A group is SU units, KS apart (SCR_ADJ: adjacent chunks, else one per wave
  // round); groups are GS = nw * SU apart.
  const int64_t wid = (int64_t)blockIdx.x * SCR_WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * SCR_WPB;
  constexpr int SU = SCR_U;
  const int64_t KS = SCR_ADJ ? 1 : nw, GS = nw * SU;
  const int64_t qk = KS / cpr, rk = KS - qk * cpr, qg = GS / cpr, rg = GS - qg * cpr;
  const int64_t ustart = SCR_ADJ ? wid * SU : wid;
  int64_t mg = ustart / cpr, cg = ustart - mg * cpr;  // first unit of the current group
  auto units = [&](int64_t m, int64_t c, int64_t (&mk)[SU], int64_t (&ck)[SU]) {
#pragma unroll
    for (int k = 0; k < SU; ++k) {
      mk[k] = m;
      ck[k] = c;
      m += qk;
      c += rk;
      if (c >= cpr) { c -= cpr; ++m; }
    }
  };
  auto load_group = [&](int64_t u0, const int64_t (&mk)[SU], const int64_t (&ck)[SU], u32x4 (&w)[SU]) {
#pragma unroll
    for (int k = 0; k < SU; ++k) {
      const int64_t n = ck[k] * 512 + 8 * lane;
      if (u0 + k * KS < total && N - n >= 8) w[k] = *reinterpret_cast<const u32x4*>(lg + mk[k] * ld + n);
    }
  };
  u32x4 wpre[SU], wnext[SU];
  int64_t mk[SU], ck[SU], mn[SU], cn[SU];
  units(mg, cg, mk, ck);
  if (SCR_PIPE) load_group(ustart, mk, ck, wpre);
  for (int64_t u0 = ustart; u0 < total; u0 += GS) {
    // software pipeline (SCR_PIPE): the next group's chunk loads are in flight while this group is computed and stored
    mg += qg;
    cg += rg;
    if (cg >= cpr) { cg -= cpr; ++mg; }
    units(mg, cg, mn, cn);
    if (SCR_PIPE) {
      if (u0 + GS < total) load_group(u0 + GS, mn, cn, wnext);
    } else {
      load_group(u0, mk, ck, wpre);
    }
#pragma unroll
    for (int k = 0; k < SU; ++k) {
      const int64_t u = u0 + k * KS;
      if (u >= total) break;
      const int64_t m = mk[k];
      const int64_t n = ck[k] * 512 + 8 * lane;
      const int64_t nv = N - n;
      bf16_t* p = lg + m * ld + n;
      float mx = -INFINITY, se = 0.f;
      int am = 0x7fffffff;
      bool generic = nv > 0;
      if (use_ft && nv >= 8) {
        const u32x4 w = wpre[k];
        u32x4 o;
        u16x2 hi = {0, 0};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u16x2 a = __builtin_bit_cast(u16x2, w[i] & 0x7fff7fffu);
          hi = __builtin_elementwise_max(hi, a);
          const u16x2 idx = __builtin_elementwise_min(a, (u16x2){FT_N - 1, FT_N - 1});
          o[i] = (w[i] & 0x80008000u) | (uint32_t)ft[idx.x] | ((uint32_t)ft[idx.y] << 16);
        }
        if (max(hi.x, hi.y) <= 0x7f80) {  // no NaN in the chunk
          *reinterpret_cast<u32x4*>(p) = o;
          float v[8];
          unpack8(o, v);
          mx = max3f(max3f(max3f(v[0], v[1], v[2]), v[3], v[4]), v[5], max3f(v[6], v[7], v[7]));
          if (mx != 0.f) {  // finite (softcap bounds |v| by cap); nonzero, so its bits are unique
            int j = 7;
#pragma unroll
            for (int t = 6; t >= 0; --t) j = v[t] == mx ? t : j;
            am = (int)n + j;
            const f32x2 m2 = {mx, mx}, l2 = {1.44269502f, 1.44269502f};  // __expf(x) = exp2(x * log2e)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const f32x2 d = ((f32x2){v[2 * i], v[2 * i + 1]} - m2) * l2;
              se += __builtin_amdgcn_exp2f(d.x);
              se += __builtin_amdgcn_exp2f(d.y);
            }
            generic = false;
          }
        }
      }
      if (generic) unit_generic(wpre[k], nv, n, p, cap, icap, tab, mx, se, am);
      float gm = mx;
      gm = fmaxf(gm, dppf<DPP_X1>(gm));
      gm = fmaxf(gm, dppf<DPP_X2>(gm));
      gm = fmaxf(gm, dppf<DPP_HALF_MIRROR>(gm));
      gm = fmaxf(gm, dppf<DPP_MIRROR>(gm));
      se = (mx == -INFINITY) ? 0.f : se * __expf(mx - gm);
      am = (mx == gm) ? am : 0x7fffffff;
      se += dppf<DPP_X1>(se);
      am = min(am, dpp<DPP_X1>(am));
      se += dppf<DPP_X2>(se);
      am = min(am, dpp<DPP_X2>(am));
      se += dppf<DPP_HALF_MIRROR>(se);
      am = min(am, dpp<DPP_HALF_MIRROR>(am));
      se += dppf<DPP_MIRROR>(se);
      am = min(am, dpp<DPP_MIRROR>(am));
      if ((lane & 15) == 0 && nv > 0) {
        float* rs = row_stats + (m * ntn + n / 128) * 3;
        rs[0] = gm;
        rs[1] = se;
        rs[2] = __int_as_float(am);
      }
    }
#pragma unroll
    for (int k = 0; k < SU; ++k) {
      if (SCR_PIPE) wpre[k] = wnext[k];
      mk[k] = mn[k];
      ck[k] = cn[k];
    }
  }
}

// host: RNE to bf16 bits, as v_cvt_pk_bf16_f32 (finite inputs)
uint32_t bf16_bits_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
}  // namespace

extern "C" int svla_softcap_ce_rows(int64_t M, int64_t N, void* logits, int64_t ld, float cap, float* row_stats,
                                    void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && ld >= N && ld % 8 == 0 && cap > 0.f, "softcap_ce_rows: M, N, ld (multiple of 8 "
                 ">= N), cap > 0");
  SVLA_CHECK_ARG(logits && row_stats && ((uintptr_t)logits & 15) == 0, "softcap_ce_rows: logits 16-B aligned");
  // the full-range table needs every |v| >= 511 (the last entry) to saturate: bf16(511 * RN(1/cap)) >= 4.0, where
  // the tanh table returns 1.0 (softcap_bf16_tab) -- any cap up to ~127
  const float icap = 1.0f / cap;
  uint32_t last;
  {
    const uint32_t b = FT_N - 1;
    float v;
    const uint32_t vb = b << 16;
    memcpy(&v, &vb, 4);
    last = bf16_bits_rne(v * icap);
  }
  const int full_tab = std::isfinite(icap) && last >= ((uint32_t)SVLA_TANH_TAB_E1 << 7) && last < 0x7f80u;
  const int64_t units = M * ((N + 511) / 512);
  const int64_t blocks = std::min<int64_t>((units + SCR_WPB - 1) / SCR_WPB, (int64_t)svla::num_cus() * SCR_BPC);
  hipLaunchKernelGGL(softcap_rows_kernel, dim3((unsigned)blocks), dim3(64 * SCR_WPB), 0, (hipStream_t)stream, M, N,
                     (bf16_t*)logits, ld, cap, row_stats, full_tab);
  return svla::check_launch("softcap_ce_rows");
}
