// Row normalisations (HBM-bound): Gemma2 RMSNorm (+ residual), LayerNorm, and deterministic
// column reductions for their weight gradients and for bias gradients.
//
// One 256-thread block per row; each thread owns up to MAXC 16-B chunks (8 bf16) of the row in
// registers, so x is read from HBM exactly once per pass.  Weight-gradient partial sums are
// written per block (RPB rows) in fp32 and reduced in a fixed order by svla_colsum_f32 / svla_colsum2_f32
// (one launch) — no atomics, bitwise reproducible.
#include "svla_common.h"

#include <algorithm>

namespace {
constexpr int NTH = 256;
constexpr int MAXC = 4;  // rows up to 256*4*8 = 8192 elements
// Rows per block in the backward kernels (kernels.py mirrors both to size the weight-gradient partial planes).  The
// norm-pair backward walks each row through two dependent block reductions: at 16 rows a block the 4B shape gave 624
// blocks for 256 CUs (2.4 each) and 80.6 us, at 8 rows 70.5 us; the single-norm kernel is faster at 16 (35.1 vs
// 38.5 us: half the partial rows) -- tools/norm_ab.py, profiles/r4o_norm_ab.txt.
constexpr int RPB = 16;
constexpr int RPB2 = 8;

__device__ __forceinline__ void ld8(const bf16_t* p, float* f) { unpack8(*reinterpret_cast<const u32x4*>(p), f); }
__device__ __forceinline__ void st8(bf16_t* p, const float* f) { *reinterpret_cast<u32x4*>(p) = pack8(f); }

// ------------------------------------------------------------------ RMSNorm forward
// RES = false: y = rms(x; w)                 (Gemma2RMSNorm.forward, modeling_gemma2.py:69-74)
// RES = true : h = bf16(res + bf16(rms(x; w)))  (decoder residual, :489-490 / :495-496)
// q != NULL (RES = false): also the OCP MX e4m3 copy of y (the fp8 projection operand; bitwise svla_quant_mx_rows of
// the stored bf16 y; N % 128 == 0 so every 16-lane group holds one whole 128-column k-tile)
template <bool RES>
__global__ __launch_bounds__(NTH) void rms_fwd_kernel(int64_t N, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ res, const bf16_t* __restrict__ w,
                                                      float eps, bf16_t* __restrict__ y, float* __restrict__ rstd_out,
                                                      uint8_t* __restrict__ q = nullptr, int64_t ldq = 0,
                                                      uint8_t* __restrict__ sc = nullptr, int64_t sld = 0) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nch = (int)(N >> 3);
  const bf16_t* xr = x + row * N;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      ld8(xr + ch * 8, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = block_sum(ss, red);
  const float rstd = rsqrtf(ss / (float)N + eps);
  if (threadIdx.x == 0 && rstd_out) rstd_out[row] = rstd;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float wf[8], o[8];
      ld8(w + ch * 8, wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] * rstd) * (1.0f + wf[j]);
      if (RES) {
        float r[8];
        ld8(res + row * N + ch * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r[j] + round_bf(o[j]);
      }
      st8(y + row * N + ch * 8, o);
      if (!RES && q != nullptr) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]);
        mx_store8(o, true, q + row * ldq + ch * 8, sc + (ch / 16) * sld + row * 4);
      }
    }
  }
}

// Two chained Gemma2 norms in one pass (inference: the decode step): h = bf16(res + bf16(rms(y; w1))) as
// rms_fwd_kernel<true>, then x = bf16(rms(h; w2)) as rms_fwd_kernel<false> over the bf16 h -- the same chunk
// mapping and summation order as the two separate launches, so both outputs are bitwise theirs.
// post_attention_layernorm + pre_feedforward_layernorm, and post_feedforward_layernorm + the next layer's
// input_layernorm (modeling_gemma2.py:487-496).
__global__ __launch_bounds__(NTH) void rms_add_norm2_kernel(int64_t N, const bf16_t* __restrict__ y,
                                                            const bf16_t* __restrict__ res,
                                                            const bf16_t* __restrict__ w1,
                                                            const bf16_t* __restrict__ w2, float eps1, float eps2,
                                                            bf16_t* __restrict__ h, bf16_t* __restrict__ x,
                                                            float* __restrict__ rstd1_out, float* __restrict__ rstd2_out,
                                                            uint8_t* __restrict__ q = nullptr, int64_t ldq = 0,
                                                            uint8_t* __restrict__ sc = nullptr, int64_t sld = 0) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nch = (int)(N >> 3);
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      ld8(y + row * N + ch * 8, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = block_sum(ss, red);
  const float rstd1 = rsqrtf(ss / (float)N + eps1);
  if (threadIdx.x == 0 && rstd1_out) rstd1_out[row] = rstd1;
  float ss2 = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float wf[8], r[8];
      ld8(w1 + ch * 8, wf);
      ld8(res + row * N + ch * 8, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = round_bf(r[j] + round_bf((v[c][j] * rstd1) * (1.0f + wf[j])));
        ss2 += v[c][j] * v[c][j];
      }
      st8(h + row * N + ch * 8, v[c]);
    }
  }
  __syncthreads();  // red[] is reused by the second reduction
  ss2 = block_sum(ss2, red);
  const float rstd2 = rsqrtf(ss2 / (float)N + eps2);
  if (threadIdx.x == 0 && rstd2_out) rstd2_out[row] = rstd2;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float wf[8], o[8];
      ld8(w2 + ch * 8, wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] * rstd2) * (1.0f + wf[j]);
      st8(x + row * N + ch * 8, o);
      if (q != nullptr) {  // the MX copy of x (as rms_fwd_kernel's)
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]);
        mx_store8(o, true, q + row * ldq + ch * 8, sc + (ch / 16) * sld + row * 4);
      }
    }
  }
}

// ------------------------------------------------------------------ RMSNorm backward
// dx = rstd*(g - xhat*mean(g*xhat)) + dres,  g = dy*(1+w), xhat = x*rstd;  dw += sum_rows dy*xhat
// A block walks RPB rows; the next row's x / dy / dres (raw 16-B chunks) are loaded before the current row's
// reduction barriers, so every row after the first finds its operands in registers (the row-serial version paid a
// full HBM round trip per row: 40-63 us at [9984, 2304], ~3 TB/s).  MC = 16-B chunks per thread (N <= 256*8*MC).
template <int MC>
__global__ __launch_bounds__(NTH) void rms_bwd_kernel(int64_t rows, int64_t N, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w, const float* __restrict__ rstd,
                                                      const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dres,
                                                      bf16_t* __restrict__ dx, float* __restrict__ dw_partial,
                                                      uint8_t* __restrict__ q = nullptr, int64_t ldq = 0,
                                                      uint8_t* __restrict__ sc = nullptr, int64_t sld = 0) {
  __shared__ float red[16];
  const int nch = (int)(N >> 3);
  float wf[MC][8], dwacc[MC][8];
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    int ch = threadIdx.x + c * NTH;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[c][j] = 0.f;
    if (ch < nch) ld8(w + ch * 8, wf[c]);
  }
  const int64_t r0 = (int64_t)blockIdx.x * RPB;
  const int nr = (int)min<int64_t>(RPB, rows - r0);
  u32x4 px[MC], pd[MC], pr[MC];
  float prs = 0.f;
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      const int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        px[c] = *reinterpret_cast<const u32x4*>(x + row * N + ch * 8);
        pd[c] = *reinterpret_cast<const u32x4*>(dy + row * N + ch * 8);
        if (dres) pr[c] = *reinterpret_cast<const u32x4*>(dres + row * N + ch * 8);
      }
    }
    prs = rstd[row];
  };
  fetch(r0);
  for (int rr = 0; rr < nr; ++rr) {
    const int64_t row = r0 + rr;
    const float rs = prs;
    u32x4 cx[MC], cd[MC], cr[MC];
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      cx[c] = px[c];
      cd[c] = pd[c];
      cr[c] = pr[c];
    }
    if (rr + 1 < nr) fetch(row + 1);
    float xv[MC][8], gv[MC][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float d[8];
        unpack8(cx[c], xv[c]);
        unpack8(cd[c], d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xh = xv[c][j] * rs;
          xv[c][j] = xh;
          gv[c][j] = d[j] * (1.0f + wf[c][j]);
          dot += gv[c][j] * xh;
          dwacc[c][j] += d[j] * xh;
        }
      }
    }
    dot = block_sum(dot, red) / (float)N;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gv[c][j] - xv[c][j] * dot);
        if (dres) {
          float r[8];
          unpack8(cr[c], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]) + r[j];
        }
        st8(dx + row * N + ch * 8, o);
        if (q != nullptr) {  // the MX copy of dx (an fp8 dgrad operand; N % 128 == 0: whole k-tiles per 16 lanes)
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]);
          mx_store8(o, true, q + row * ldq + ch * 8, sc + (ch / 16) * sld + row * 4);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float* p = dw_partial + (int64_t)blockIdx.x * N + ch * 8;
      *reinterpret_cast<f32x4*>(p) = f32x4{dwacc[c][0], dwacc[c][1], dwacc[c][2], dwacc[c][3]};
      *reinterpret_cast<f32x4*>(p + 4) = f32x4{dwacc[c][4], dwacc[c][5], dwacc[c][6], dwacc[c][7]};
    }
  }
}

// ------------------------------------------------------------------ RMSNorm pair backward
// The backward of h = res + rms(y; w1), x = rms(h; w2) (decoder-layer post-attention norm + residual and the
// pre-feedforward norm, modeling_gemma2.py:487-490) in one pass over the rows:
//   dh = bf16(bf16(rms_bwd(h; dx)) + dres)    (stored: the residual-stream gradient of res)
//   dy = bf16(rms_bwd(y; dh))
// with the weight-gradient partials of both norms as two planes [2][blocks][N] (w2 first).  The per-row arithmetic and
// reduction order are rms_bwd_kernel's, so dh / dy are bitwise those of two svla_rmsnorm_bwd calls; the weight
// partials cover RPB2 = 8 rows a block (RPB = 16 there), the same sums reassociated.  One launch and one read of dh
// fewer.
template <int MC>
__global__ __launch_bounds__(NTH) void rms_bwd2_kernel(int64_t rows, int64_t N, const bf16_t* __restrict__ h,
                                                       const bf16_t* __restrict__ w2, const float* __restrict__ rstd2,
                                                       const bf16_t* __restrict__ dx, const bf16_t* __restrict__ dres,
                                                       const bf16_t* __restrict__ y, const bf16_t* __restrict__ w1,
                                                       const float* __restrict__ rstd1, bf16_t* __restrict__ dh_out,
                                                       bf16_t* __restrict__ dy_out, float* __restrict__ partial,
                                                       uint8_t* __restrict__ q = nullptr, int64_t ldq = 0,
                                                       uint8_t* __restrict__ sc = nullptr, int64_t sld = 0) {
  __shared__ float red[16];
  const int nch = (int)(N >> 3);
  float wf2[MC][8], wf1[MC][8], acc2[MC][8], acc1[MC][8];
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    int ch = threadIdx.x + c * NTH;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc2[c][j] = acc1[c][j] = 0.f;
    if (ch < nch) {
      ld8(w2 + ch * 8, wf2[c]);
      ld8(w1 + ch * 8, wf1[c]);
    }
  }
  const int64_t r0 = (int64_t)blockIdx.x * RPB2;
  const int nr = (int)min<int64_t>(RPB2, rows - r0);
  u32x4 ph[MC], pd[MC], pr[MC], py[MC];
  float prs2 = 0.f, prs1 = 0.f;
  auto fetch = [&](int64_t row) {
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      const int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        ph[c] = *reinterpret_cast<const u32x4*>(h + row * N + ch * 8);
        pd[c] = *reinterpret_cast<const u32x4*>(dx + row * N + ch * 8);
        if (dres) pr[c] = *reinterpret_cast<const u32x4*>(dres + row * N + ch * 8);
        py[c] = *reinterpret_cast<const u32x4*>(y + row * N + ch * 8);
      }
    }
    prs2 = rstd2[row];
    prs1 = rstd1[row];
  };
  fetch(r0);
  for (int rr = 0; rr < nr; ++rr) {
    const int64_t row = r0 + rr;
    const float rs2 = prs2, rs1 = prs1;
    u32x4 ch_[MC], cd[MC], cr[MC], cy[MC];
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      ch_[c] = ph[c];
      cd[c] = pd[c];
      cr[c] = pr[c];
      cy[c] = py[c];
    }
    if (rr + 1 < nr) fetch(row + 1);
    // norm 2 (x = rms(h; w2)): dh
    float xv[MC][8], gv[MC][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float d[8];
        unpack8(ch_[c], xv[c]);
        unpack8(cd[c], d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xh = xv[c][j] * rs2;
          xv[c][j] = xh;
          gv[c][j] = d[j] * (1.0f + wf2[c][j]);
          dot += gv[c][j] * xh;
          acc2[c][j] += d[j] * xh;
        }
      }
    }
    dot = block_sum(dot, red) / (float)N;
    float dh[MC][8];
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) dh[c][j] = rs2 * (gv[c][j] - xv[c][j] * dot);
        if (dres) {
          float r[8];
          unpack8(cr[c], r);
#pragma unroll
          for (int j = 0; j < 8; ++j) dh[c][j] = round_bf(dh[c][j]) + r[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) dh[c][j] = round_bf(dh[c][j]);  // the bf16 dh both consumers read
        st8(dh_out + row * N + ch * 8, dh[c]);
      }
    }
    // norm 1 (h = res + rms(y; w1)): dy from the bf16 dh
    float dot1 = 0.f;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        unpack8(cy[c], xv[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xh = xv[c][j] * rs1;
          xv[c][j] = xh;
          gv[c][j] = dh[c][j] * (1.0f + wf1[c][j]);
          dot1 += gv[c][j] * xh;
          acc1[c][j] += dh[c][j] * xh;
        }
      }
    }
    __syncthreads();  // red[] is reused by the second reduction
    dot1 = block_sum(dot1, red) / (float)N;
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs1 * (gv[c][j] - xv[c][j] * dot1);
        st8(dy_out + row * N + ch * 8, o);
        if (q != nullptr) {  // the MX copy of dy (the fp8 o-projection dgrad operand)
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]);
          mx_store8(o, true, q + row * ldq + ch * 8, sc + (ch / 16) * sld + row * 4);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float* p2 = partial + (int64_t)blockIdx.x * N + ch * 8;
      float* p1 = p2 + (int64_t)gridDim.x * N;
      *reinterpret_cast<f32x4*>(p2) = f32x4{acc2[c][0], acc2[c][1], acc2[c][2], acc2[c][3]};
      *reinterpret_cast<f32x4*>(p2 + 4) = f32x4{acc2[c][4], acc2[c][5], acc2[c][6], acc2[c][7]};
      *reinterpret_cast<f32x4*>(p1) = f32x4{acc1[c][0], acc1[c][1], acc1[c][2], acc1[c][3]};
      *reinterpret_cast<f32x4*>(p1 + 4) = f32x4{acc1[c][4], acc1[c][5], acc1[c][6], acc1[c][7]};
    }
  }
}

// ------------------------------------------------------------------ wave-per-row backward (N <= 1536 / 2048)
// One wave per row (lane l owns 16-B chunks l, l+64, ..): the row reductions are wave shuffles, so the four waves
// of a block work on four rows at once with no barrier; each block still covers RPB rows and writes one weight-
// gradient partial row (its four waves' sums combined through LDS in a fixed order).  Per-element arithmetic is
// that of the block-per-row kernels above.
constexpr int WCH = 5;  // chunks per lane: rows up to 64*5*8 = 2560 elements

template <bool LN>
__global__ __launch_bounds__(256) void norm_bwd_wave_kernel(int64_t rows, int64_t N, const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ w, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const bf16_t* __restrict__ dy,
                                                            const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                            float* __restrict__ partial) {
  extern __shared__ float sred[];  // [4][N] (LN: [4][2N])
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nch = (int)(N >> 3);
  float dwacc[WCH][8], dbacc[LN ? WCH : 1][8];
#pragma unroll
  for (int c = 0; c < WCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dwacc[c][j] = 0.f;
      if (LN) dbacc[LN ? c : 0][j] = 0.f;
    }
  const int64_t r0 = (int64_t)blockIdx.x * RPB;
  for (int rr = wv; rr < RPB; rr += 4) {
    const int64_t row = r0 + rr;
    if (row >= rows) break;
    const float rs = rstd[row];
    const float mu = LN ? mean[row] : 0.f;
    float xh[WCH][8], gv[WCH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < WCH; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float d[8], wf[8];
        ld8(x + row * N + ch * 8, xh[c]);
        ld8(dy + row * N + ch * 8, d);
        ld8(w + ch * 8, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (LN) {
            xh[c][j] = (xh[c][j] - mu) * rs;
            gv[c][j] = d[j] * wf[j];
            s1 += gv[c][j];
            s2 += gv[c][j] * xh[c][j];
            dbacc[LN ? c : 0][j] += d[j];
          } else {
            xh[c][j] = xh[c][j] * rs;
            gv[c][j] = d[j] * (1.0f + wf[j]);
            s2 += gv[c][j] * xh[c][j];
          }
          dwacc[c][j] += d[j] * xh[c][j];
        }
      }
    }
    s2 = wave_sum(s2) / (float)N;
    if (LN) s1 = wave_sum(s1) / (float)N;
#pragma unroll
    for (int c = 0; c < WCH; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = LN ? rs * (gv[c][j] - s1 - xh[c][j] * s2) : rs * (gv[c][j] - xh[c][j] * s2);
        if (dres) {
          float r[8];
          ld8(dres + row * N + ch * 8, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]) + r[j];
        }
        st8(dx + row * N + ch * 8, o);
      }
    }
  }
  // combine the four waves' weight-gradient sums in wave order, one partial row per block
  const int nv = LN ? 2 : 1;
#pragma unroll
  for (int c = 0; c < WCH; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sred[(wv * nv) * N + ch * 8 + j] = dwacc[c][j];
        if (LN) sred[(wv * nv + 1) * N + ch * 8 + j] = dbacc[LN ? c : 0][j];
      }
  }
  __syncthreads();
  for (int64_t i = threadIdx.x; i < nv * N; i += 256) {
    const int v = (int)(i / N);
    const int64_t k = i % N;
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc += sred[(q * nv + v) * N + k];
    partial[((int64_t)v * gridDim.x + blockIdx.x) * N + k] = acc;  // plane v (LN: dw, db) of [nv][blocks][N]
  }
}

// ------------------------------------------------------------------ LayerNorm
// Wave-per-row forward for rows up to 64*8*WC elements (SigLIP 1152, BEiT 1024): four rows per block, the mean and
// variance are wave reductions (no block barrier); the block-per-row kernel below left 112 of 256 threads idle at
// N = 1152 and paid four barriers per row (19.9 us for [8192, 1152], 1.9 TB/s).
template <int WC>
__global__ __launch_bounds__(256) void ln_fwd_wave_kernel(int64_t rows, int64_t N, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                          float eps, bf16_t* __restrict__ y, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nch = (int)(N >> 3);
  float v[WC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      ld8(x + row * N + ch * 8, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float mean = wave_sum(s) / (float)N;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mean;
        s2 += d * d;
      }
  }
  const float rstd = rsqrtf(wave_sum(s2) / (float)N + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < WC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float wf[8], bf[8], o[8];
      ld8(w + ch * 8, wf);
      ld8(b + ch * 8, bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wf[j] + bf[j];
      st8(y + row * N + ch * 8, o);
    }
  }
}

__global__ __launch_bounds__(NTH) void ln_fwd_kernel(int64_t N, const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                     float eps, bf16_t* __restrict__ y, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int nch = (int)(N >> 3);
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      ld8(x + row * N + ch * 8, v[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  const float mean = block_sum(s, red) / (float)N;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = v[c][j] - mean;
        s2 += d * d;
      }
  }
  const float var = block_sum(s2, red) / (float)N;
  const float rstd = rsqrtf(var + eps);
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float wf[8], bf[8], o[8];
      ld8(w + ch * 8, wf);
      ld8(b + ch * 8, bf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[c][j] - mean) * rstd * wf[j] + bf[j];
      st8(y + row * N + ch * 8, o);
    }
  }
}

// dx = rstd*(g - mean(g) - xhat*mean(g*xhat)) + dres, g = dy*w ; dw += dy*xhat ; db += dy
__global__ __launch_bounds__(NTH) void ln_bwd_kernel(int64_t rows, int64_t N, const bf16_t* __restrict__ x,
                                                     const bf16_t* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const bf16_t* __restrict__ dy,
                                                     const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                     float* __restrict__ dwb_partial) {
  __shared__ float red[16];
  const int nch = (int)(N >> 3);
  float wf[MAXC][8], dwacc[MAXC][8], dbacc[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[c][j] = dbacc[c][j] = 0.f;
    if (ch < nch) ld8(w + ch * 8, wf[c]);
  }
  const int64_t r0 = (int64_t)blockIdx.x * RPB;
  for (int rr = 0; rr < RPB; ++rr) {
    const int64_t row = r0 + rr;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXC][8], gv[MAXC][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float d[8];
        ld8(x + row * N + ch * 8, xh[c]);
        ld8(dy + row * N + ch * 8, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] = (xh[c][j] - mu) * rs;
          gv[c][j] = d[j] * wf[c][j];
          sg += gv[c][j];
          sgx += gv[c][j] * xh[c][j];
          dwacc[c][j] += d[j] * xh[c][j];
          dbacc[c][j] += d[j];
        }
      }
    }
    sg = block_sum(sg, red) / (float)N;
    sgx = block_sum(sgx, red) / (float)N;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      int ch = threadIdx.x + c * NTH;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (gv[c][j] - sg - xh[c][j] * sgx);
        if (dres) {
          float r[8];
          ld8(dres + row * N + ch * 8, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = round_bf(o[j]) + r[j];
        }
        st8(dx + row * N + ch * 8, o);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    int ch = threadIdx.x + c * NTH;
    if (ch < nch) {
      float* p = dwb_partial + (int64_t)blockIdx.x * N + ch * 8;  // planes [2][blocks][N]: dw, then db
      float* pb = p + (int64_t)gridDim.x * N;
      *reinterpret_cast<f32x4*>(p) = f32x4{dwacc[c][0], dwacc[c][1], dwacc[c][2], dwacc[c][3]};
      *reinterpret_cast<f32x4*>(p + 4) = f32x4{dwacc[c][4], dwacc[c][5], dwacc[c][6], dwacc[c][7]};
      *reinterpret_cast<f32x4*>(pb) = f32x4{dbacc[c][0], dbacc[c][1], dbacc[c][2], dbacc[c][3]};
      *reinterpret_cast<f32x4*>(pb + 4) = f32x4{dbacc[c][4], dbacc[c][5], dbacc[c][6], dbacc[c][7]};
    }
  }
}

// ------------------------------------------------------------------ column reductions
// Single-pass deterministic column sums (round 4: replaces the two colsum_kernel passes, 768 launches a step).  A
// block owns CB columns of every one of the P rows: its 256 threads are CB/8 column lanes (8 consecutive columns,
// one 16-B bf16 or two 16-B fp32 loads per row) x RG = 2048/CB row groups; group g sums rows g, g+RG, .. in
// increasing order in fp32 registers, four rows in flight, then one thread per column adds the RG group sums in
// group order from LDS.  grid.y = planes (plane y reads in + y * plane_stride, writes out_y), so the dw and db
// planes of the LayerNorm backward reduce in one launch.  Fixed assignment and order: bitwise reproducible.
template <typename T, int CB>
__global__ __launch_bounds__(256) void colsum1_kernel(int64_t P, int64_t N, const T* __restrict__ in, int64_t ld,
                                                      int64_t plane_stride, bf16_t* __restrict__ out0,
                                                      bf16_t* __restrict__ out1, int acc) {
  constexpr int CL = CB / 8, RG = 256 / CL;
  __shared__ float red[RG][CB + 1];
  const int cl = threadIdx.x % CL, rg = threadIdx.x / CL;
  const int64_t n0 = (int64_t)blockIdx.x * CB + cl * 8;
  const T* src = in + (int64_t)blockIdx.y * plane_stride + n0;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  auto add_row = [&](int64_t p) {
    float v[8];
    if constexpr (sizeof(T) == 2) {
      unpack8(*reinterpret_cast<const u32x4*>(src + p * ld), v);
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>(src + p * ld);
      const f32x4 b = *reinterpret_cast<const f32x4*>(src + p * ld + 4);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
      v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v[j];
  };
  if (n0 < N) {
    int64_t p = rg;
    for (; p + 3 * RG < P; p += 4 * RG) {  // four independent row loads in flight, summed in row order
      add_row(p);
      add_row(p + RG);
      add_row(p + 2 * RG);
      add_row(p + 3 * RG);
    }
    for (; p < P; p += RG) add_row(p);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cl * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < CB) {
    const int64_t n = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (n < N) {
      float t = 0.f;
      for (int q = 0; q < RG; ++q) t += red[q][threadIdx.x];
      bf16_t* o = blockIdx.y ? out1 : out0;
      if (acc) t += bf2f(o[n]);
      o[n] = f2bf(t);
    }
  }
}

template <typename T>
int launch_colsum1(int64_t P, int64_t N, const T* in, int64_t ld, int64_t plane_stride, int planes, bf16_t* out0,
                   bf16_t* out1, int acc, hipStream_t s) {
  // 32 columns a block when that still gives >= 64 blocks, else 16 (more blocks, shorter row segments); chosen by N
  // alone, so a plane reduced by svla_colsum2_f32 sums in the order svla_colsum_f32 uses
  (void)planes;
  if ((N + 31) / 32 >= 64)
    hipLaunchKernelGGL((colsum1_kernel<T, 32>), dim3((unsigned)((N + 31) / 32), (unsigned)planes), dim3(256), 0, s, P,
                       N, in, ld, plane_stride, out0, out1, acc);
  else
    hipLaunchKernelGGL((colsum1_kernel<T, 16>), dim3((unsigned)((N + 15) / 16), (unsigned)planes), dim3(256), 0, s, P,
                       N, in, ld, plane_stride, out0, out1, acc);
  return svla::check_launch("colsum");
}

// Row-split bf16 column sums (bias gradients of SigLIP's nn.Linear layers): a single pass gives one block per 32
// columns -- 36 to 135 blocks for N = 1152 .. 4304, most CUs idle.  Slice s of S sums rows [s*RS, (s+1)*RS) per
// column exactly as colsum1_kernel does over its rows (row groups, fixed order) into fp32 partial row s of the
// workspace; a second colsum1 launch reduces the S partial rows in slice order.
template <int CB>
__global__ __launch_bounds__(256) void colsum_slice_kernel(int64_t M, int64_t N, const bf16_t* __restrict__ in,
                                                           int64_t ld, int64_t rows_per_slice,
                                                           float* __restrict__ part) {
  constexpr int CL = CB / 8, RG = 256 / CL;
  __shared__ float red[RG][CB + 1];
  const int cl = threadIdx.x % CL, rg = threadIdx.x / CL;
  const int64_t n0 = (int64_t)blockIdx.x * CB + cl * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_slice, r1 = min(M, r0 + rows_per_slice);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (n0 < N) {
    const bf16_t* src = in + n0;
    int64_t p = r0 + rg;
    auto add_row = [&](int64_t q) {
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(src + q * ld), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    };
    for (; p + 3 * RG < r1; p += 4 * RG) {
      add_row(p);
      add_row(p + RG);
      add_row(p + 2 * RG);
      add_row(p + 3 * RG);
    }
    for (; p < r1; p += RG) add_row(p);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][cl * 8 + j] = s[j];
  __syncthreads();
  if (threadIdx.x < CB) {
    const int64_t n = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (n < N) {
      float t = 0.f;
      for (int q = 0; q < RG; ++q) t += red[q][threadIdx.x];
      part[(int64_t)blockIdx.y * N + n] = t;
    }
  }
}

// slices for an M x N bf16 column sum: about 1024 blocks of CS_CB = 64 columns (a whole 128-B line of every row per
// block: at 32 columns two blocks on different XCDs each fetched half of every line), slices of at least 512 rows.
// tools/colsum_ab.py, profiles/r4u_colsum_cb64_ab.txt: 8192 x 4304 25.1 -> 21.8 us, x 3456 17.9 -> 12.5, x 1152
// 14.8 -> 6.5 (32-column slices: 28.6 / 20.2 / 9.5, so they were kept to N < 2048 before)
constexpr int CS_CB = 64;
int64_t colsum_slices(int64_t M, int64_t N) {
  const int64_t cb = (N + CS_CB - 1) / CS_CB;
  int64_t S = (1024 + cb - 1) / cb;
  S = std::min<int64_t>(S, M / 512);
  return S < 2 ? 1 : S;
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
}  // namespace

extern "C" size_t svla_colsum_bf16_workspace_bytes(int64_t M, int64_t N) {
  const int64_t S = colsum_slices(M, N);
  return S > 1 ? (size_t)S * (size_t)N * sizeof(float) : 0;
}

extern "C" int svla_rmsnorm_fwd(int64_t rows, int64_t N, const void* x, const void* w, float eps, void* y,
                                float* rstd, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "rmsnorm: bad N=%lld", (long long)N);
  SVLA_CHECK_ARG(x && w && y && al16(x) && al16(w) && al16(y), "rmsnorm: null/misaligned pointer");
  hipLaunchKernelGGL((rms_fwd_kernel<false>), dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)x, (const bf16_t*)nullptr, (const bf16_t*)w, eps, (bf16_t*)y, rstd);
  return svla::check_launch("rmsnorm_fwd");
}

extern "C" int svla_add_rmsnorm_fwd(int64_t rows, int64_t N, const void* res, const void* yin, const void* w,
                                    float eps, void* h, float* rstd, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "add_rmsnorm: bad N");
  SVLA_CHECK_ARG(res && yin && w && h && al16(res) && al16(yin) && al16(h), "add_rmsnorm: null/misaligned");
  hipLaunchKernelGGL((rms_fwd_kernel<true>), dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)yin, (const bf16_t*)res, (const bf16_t*)w, eps, (bf16_t*)h, rstd);
  return svla::check_launch("add_rmsnorm_fwd");
}

extern "C" int svla_rmsnorm_bwd(int64_t rows, int64_t N, const void* x, const void* w, const float* rstd,
                                const void* dy, const void* dres, void* dx, float* dw_partial, int64_t* n_partial,
                                void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "rmsnorm_bwd: bad N");
  SVLA_CHECK_ARG(x && w && rstd && dy && dx && dw_partial, "rmsnorm_bwd: null pointer");
  const int64_t nb = (rows + RPB - 1) / RPB;
  if (n_partial) *n_partial = nb;
  if (N <= 1536) {  // measured: at N = 2304 (5 chunks a lane) the block-per-row kernel is faster (43 vs 58 us)
    const size_t lds = (size_t)4 * N * sizeof(float);
    hipLaunchKernelGGL(norm_bwd_wave_kernel<false>, dim3((unsigned)nb), dim3(256), lds, (hipStream_t)stream, rows, N,
                       (const bf16_t*)x, (const bf16_t*)w, (const float*)nullptr, rstd, (const bf16_t*)dy,
                       (const bf16_t*)dres, (bf16_t*)dx, dw_partial);
  } else {
    if (N <= NTH * 8 * 2)
      hipLaunchKernelGGL(rms_bwd_kernel<2>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                         (const bf16_t*)x, (const bf16_t*)w, rstd, (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx,
                         dw_partial);
    else
      hipLaunchKernelGGL(rms_bwd_kernel<MAXC>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                         (const bf16_t*)x, (const bf16_t*)w, rstd, (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx,
                         dw_partial);
  }
  return svla::check_launch("rmsnorm_bwd");
}

extern "C" int svla_rmsnorm2_bwd(int64_t rows, int64_t N, const void* h, const void* w2, const float* rstd2,
                                 const void* dx, const void* dres, const void* y, const void* w1, const float* rstd1,
                                 void* dh_out, void* dy_out, float* dw_partial, int64_t* n_partial, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * 8 * 4, "rmsnorm2_bwd: bad N");
  SVLA_CHECK_ARG(h && w2 && rstd2 && dx && y && w1 && rstd1 && dh_out && dy_out && dw_partial,
                 "rmsnorm2_bwd: null pointer");
  SVLA_CHECK_ARG(al16(h) && al16(w2) && al16(dx) && (!dres || al16(dres)) && al16(y) && al16(w1) && al16(dh_out) &&
                     al16(dy_out) && al16(dw_partial), "rmsnorm2_bwd: misaligned pointer");
  const int64_t nb = (rows + RPB2 - 1) / RPB2;
  if (n_partial) *n_partial = nb;
  if (N <= NTH * 8 * 2)
    hipLaunchKernelGGL(rms_bwd2_kernel<2>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)h, (const bf16_t*)w2, rstd2, (const bf16_t*)dx, (const bf16_t*)dres,
                       (const bf16_t*)y, (const bf16_t*)w1, rstd1, (bf16_t*)dh_out, (bf16_t*)dy_out, dw_partial);
  else
    hipLaunchKernelGGL(rms_bwd2_kernel<4>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)h, (const bf16_t*)w2, rstd2, (const bf16_t*)dx, (const bf16_t*)dres,
                       (const bf16_t*)y, (const bf16_t*)w1, rstd1, (bf16_t*)dh_out, (bf16_t*)dy_out, dw_partial);
  return svla::check_launch("rmsnorm2_bwd");
}

extern "C" int svla_layernorm_fwd(int64_t rows, int64_t N, const void* x, const void* w, const void* b, float eps,
                                  void* y, float* mean, float* rstd, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "layernorm: bad N");
  SVLA_CHECK_ARG(x && w && b && y && mean && rstd, "layernorm: null pointer");
  if (N <= 64 * 8 * 3)
    hipLaunchKernelGGL(ln_fwd_wave_kernel<3>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, rows,
                       N, (const bf16_t*)x, (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)y, mean, rstd);
  else
    hipLaunchKernelGGL(ln_fwd_kernel, dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N, (const bf16_t*)x,
                       (const bf16_t*)w, (const bf16_t*)b, eps, (bf16_t*)y, mean, rstd);
  return svla::check_launch("layernorm_fwd");
}

extern "C" int svla_layernorm_bwd(int64_t rows, int64_t N, const void* x, const void* w, const float* mean,
                                  const float* rstd, const void* dy, const void* dres, void* dx, float* dwb_partial,
                                  int64_t* n_partial, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "layernorm_bwd: bad N");
  SVLA_CHECK_ARG(x && w && mean && rstd && dy && dx && dwb_partial, "layernorm_bwd: null pointer");
  const int64_t nb = (rows + RPB - 1) / RPB;
  if (n_partial) *n_partial = nb;
  if (N <= 2048) {  // 8N fp32 of LDS must stay within the default 64 KiB dynamic limit
    const size_t lds = (size_t)8 * N * sizeof(float);
    hipLaunchKernelGGL(norm_bwd_wave_kernel<true>, dim3((unsigned)nb), dim3(256), lds, (hipStream_t)stream, rows, N,
                       (const bf16_t*)x, (const bf16_t*)w, mean, rstd, (const bf16_t*)dy, (const bf16_t*)dres,
                       (bf16_t*)dx, dwb_partial);
  } else {
    hipLaunchKernelGGL(ln_bwd_kernel, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)x, (const bf16_t*)w, mean, rstd, (const bf16_t*)dy, (const bf16_t*)dres,
                       (bf16_t*)dx, dwb_partial);
  }
  return svla::check_launch("layernorm_bwd");
}

extern "C" int svla_colsum_f32(int64_t P, int64_t N, const float* in, void* out_bf16, int32_t accumulate,
                               float* workspace, void* stream) {
  (void)workspace;  // single pass since round 4; kept in the ABI
  SVLA_CHECK_ARG(P > 0 && N > 0 && N % 8 == 0 && in && out_bf16 && al16(in), "colsum_f32: bad args");
  return launch_colsum1<float>(P, N, in, N, 0, 1, (bf16_t*)out_bf16, nullptr, accumulate, (hipStream_t)stream);
}

extern "C" int svla_colsum2_f32(int64_t P, int64_t N, const float* in, void* out0_bf16, void* out1_bf16,
                                int32_t accumulate, void* stream) {
  SVLA_CHECK_ARG(P > 0 && N > 0 && N % 8 == 0 && in && out0_bf16 && out1_bf16 && al16(in), "colsum2_f32: bad args");
  return launch_colsum1<float>(P, N, in, N, P * N, 2, (bf16_t*)out0_bf16, (bf16_t*)out1_bf16, accumulate,
                               (hipStream_t)stream);
}

extern "C" int svla_colsum_bf16(int64_t M, int64_t N, const void* x, int64_t ldx, void* out_bf16,
                                int32_t accumulate, float* workspace, void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && N % 8 == 0 && x && out_bf16 && ldx >= N && ldx % 8 == 0 && al16(x),
                 "colsum_bf16: bad args");
  const int64_t S = colsum_slices(M, N);
  if (workspace && S > 1) {  // sized by svla_colsum_bf16_workspace_bytes(M, N)
    const int64_t rps = (M + S - 1) / S;
    hipLaunchKernelGGL(colsum_slice_kernel<CS_CB>, dim3((unsigned)((N + CS_CB - 1) / CS_CB), (unsigned)S), dim3(256), 0,
                       (hipStream_t)stream, M, N, (const bf16_t*)x, ldx, rps, workspace);
    if (int rc = svla::check_launch("colsum_bf16 slices")) return rc;
    return launch_colsum1<float>(S, N, workspace, N, 0, 1, (bf16_t*)out_bf16, nullptr, accumulate,
                                 (hipStream_t)stream);
  }
  return launch_colsum1<bf16_t>(M, N, (const bf16_t*)x, ldx, 0, 1, (bf16_t*)out_bf16, nullptr, accumulate,
                                (hipStream_t)stream);
}

extern "C" int svla_add_rmsnorm2_fwd(int64_t rows, int64_t N, const void* res, const void* yin, const void* w1,
                                     const void* w2, float eps1, float eps2, void* h, void* x, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "add_rmsnorm2: bad N");
  SVLA_CHECK_ARG(res && yin && w1 && w2 && h && x && al16(res) && al16(yin) && al16(w1) && al16(w2) && al16(h) &&
                     al16(x), "add_rmsnorm2: null/misaligned pointer");
  hipLaunchKernelGGL(rms_add_norm2_kernel, dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)yin, (const bf16_t*)res, (const bf16_t*)w1, (const bf16_t*)w2, eps1, eps2,
                     (bf16_t*)h, (bf16_t*)x, (float*)nullptr, (float*)nullptr);
  return svla::check_launch("add_rmsnorm2_fwd");
}

extern "C" int svla_add_rmsnorm2_fwd_train(int64_t rows, int64_t N, const void* res, const void* yin, const void* w1,
                                           const void* w2, float eps1, float eps2, void* h, void* x, float* rstd1,
                                           float* rstd2, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 8 == 0 && N <= NTH * MAXC * 8, "add_rmsnorm2_train: bad N");
  SVLA_CHECK_ARG(res && yin && w1 && w2 && h && x && rstd1 && rstd2 && al16(res) && al16(yin) && al16(w1) &&
                     al16(w2) && al16(h) && al16(x), "add_rmsnorm2_train: null/misaligned pointer");
  hipLaunchKernelGGL(rms_add_norm2_kernel, dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)yin, (const bf16_t*)res, (const bf16_t*)w1, (const bf16_t*)w2, eps1, eps2,
                     (bf16_t*)h, (bf16_t*)x, rstd1, rstd2);
  return svla::check_launch("add_rmsnorm2_fwd_train");
}

extern "C" int svla_rmsnorm_fwd_mx(int64_t rows, int64_t N, const void* x, const void* w, float eps, void* y,
                                   float* rstd, void* q, int64_t ldq, void* scales, int64_t sld, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 128 == 0 && N <= NTH * MAXC * 8, "rmsnorm_mx: bad N=%lld (a multiple of 128)",
                 (long long)N);
  SVLA_CHECK_ARG(x && w && y && q && scales && al16(x) && al16(w) && al16(y) && ldq >= N && ldq % 8 == 0 &&
                     ((uintptr_t)q & 7) == 0 && ((uintptr_t)scales & 3) == 0 && sld >= 4 * rows && sld % 4 == 0,
                 "rmsnorm_mx: null/misaligned pointer or bad q / scale strides");
  hipLaunchKernelGGL((rms_fwd_kernel<false>), dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)x, (const bf16_t*)nullptr, (const bf16_t*)w, eps, (bf16_t*)y, rstd, (uint8_t*)q,
                     ldq, (uint8_t*)scales, sld);
  return svla::check_launch("rmsnorm_fwd_mx");
}

extern "C" int svla_add_rmsnorm2_fwd_train_mx(int64_t rows, int64_t N, const void* res, const void* yin,
                                              const void* w1, const void* w2, float eps1, float eps2, void* h, void* x,
                                              float* rstd1, float* rstd2, void* q, int64_t ldq, void* scales,
                                              int64_t sld, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 128 == 0 && N <= NTH * MAXC * 8, "add_rmsnorm2_mx: bad N");
  SVLA_CHECK_ARG(res && yin && w1 && w2 && h && x && rstd1 && rstd2 && q && scales && al16(res) && al16(yin) &&
                     al16(w1) && al16(w2) && al16(h) && al16(x) && ldq >= N && ldq % 8 == 0 && ((uintptr_t)q & 7) == 0 &&
                     ((uintptr_t)scales & 3) == 0 && sld >= 4 * rows && sld % 4 == 0,
                 "add_rmsnorm2_mx: null/misaligned pointer or bad q / scale strides");
  hipLaunchKernelGGL(rms_add_norm2_kernel, dim3((unsigned)rows), dim3(NTH), 0, (hipStream_t)stream, N,
                     (const bf16_t*)yin, (const bf16_t*)res, (const bf16_t*)w1, (const bf16_t*)w2, eps1, eps2,
                     (bf16_t*)h, (bf16_t*)x, rstd1, rstd2, (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  return svla::check_launch("add_rmsnorm2_fwd_train_mx");
}

extern "C" int svla_rmsnorm_bwd_mx(int64_t rows, int64_t N, const void* x, const void* w, const float* rstd,
                                   const void* dy, const void* dres, void* dx, float* dw_partial, int64_t* n_partial,
                                   void* q, int64_t ldq, void* scales, int64_t sld, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 1536 && N % 128 == 0 && N <= NTH * MAXC * 8,
                 "rmsnorm_bwd_mx: N=%lld (a multiple of 128 in (1536, %d])", (long long)N, NTH * MAXC * 8);
  SVLA_CHECK_ARG(x && w && rstd && dy && dx && dw_partial && q && scales && ldq >= N && ldq % 8 == 0 &&
                     ((uintptr_t)q & 7) == 0 && ((uintptr_t)scales & 3) == 0 && sld >= 4 * rows && sld % 4 == 0,
                 "rmsnorm_bwd_mx: null pointer or bad q / scale strides");
  const int64_t nb = (rows + RPB - 1) / RPB;
  if (n_partial) *n_partial = nb;
  if (N <= NTH * 8 * 2)
    hipLaunchKernelGGL(rms_bwd_kernel<2>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)x, (const bf16_t*)w, rstd, (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx,
                       dw_partial, (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  else
    hipLaunchKernelGGL(rms_bwd_kernel<MAXC>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)x, (const bf16_t*)w, rstd, (const bf16_t*)dy, (const bf16_t*)dres, (bf16_t*)dx,
                       dw_partial, (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  return svla::check_launch("rmsnorm_bwd_mx");
}

extern "C" int svla_rmsnorm2_bwd_mx(int64_t rows, int64_t N, const void* h, const void* w2, const float* rstd2,
                                    const void* dx, const void* dres, const void* y, const void* w1, const float* rstd1,
                                    void* dh_out, void* dy_out, float* dw_partial, int64_t* n_partial, void* q,
                                    int64_t ldq, void* scales, int64_t sld, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && N > 0 && N % 128 == 0 && N <= NTH * 8 * 4, "rmsnorm2_bwd_mx: bad N (a multiple of 128)");
  SVLA_CHECK_ARG(h && w2 && rstd2 && dx && y && w1 && rstd1 && dh_out && dy_out && dw_partial && q && scales,
                 "rmsnorm2_bwd_mx: null pointer");
  SVLA_CHECK_ARG(al16(h) && al16(w2) && al16(dx) && (!dres || al16(dres)) && al16(y) && al16(w1) && al16(dh_out) &&
                     al16(dy_out) && al16(dw_partial) && ldq >= N && ldq % 8 == 0 && ((uintptr_t)q & 7) == 0 &&
                     ((uintptr_t)scales & 3) == 0 && sld >= 4 * rows && sld % 4 == 0,
                 "rmsnorm2_bwd_mx: misaligned pointer or bad q / scale strides");
  const int64_t nb = (rows + RPB2 - 1) / RPB2;
  if (n_partial) *n_partial = nb;
  if (N <= NTH * 8 * 2)
    hipLaunchKernelGGL(rms_bwd2_kernel<2>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)h, (const bf16_t*)w2, rstd2, (const bf16_t*)dx, (const bf16_t*)dres,
                       (const bf16_t*)y, (const bf16_t*)w1, rstd1, (bf16_t*)dh_out, (bf16_t*)dy_out, dw_partial,
                       (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  else
    hipLaunchKernelGGL(rms_bwd2_kernel<4>, dim3((unsigned)nb), dim3(NTH), 0, (hipStream_t)stream, rows, N,
                       (const bf16_t*)h, (const bf16_t*)w2, rstd2, (const bf16_t*)dx, (const bf16_t*)dres,
                       (const bf16_t*)y, (const bf16_t*)w1, rstd1, (bf16_t*)dh_out, (bf16_t*)dy_out, dw_partial,
                       (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  return svla::check_launch("rmsnorm2_bwd_mx");
}
