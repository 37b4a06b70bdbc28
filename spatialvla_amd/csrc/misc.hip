// HBM-bound glue kernels of the hot path: embedding merge, Ego3D back-projection + frequency
// encoding, SigLIP patchify, elementwise helpers, softcapped-CE finalize/backward, grad-norm and
// AdamW.  All vectorised 16 B per lane (8 bf16) where the layout allows.
#include "svla_common.h"

namespace {

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline unsigned nblk(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// ------------------------------------------------------------------ embedding merge
// modeling_spatialvla.py:361-387 + modeling_gemma2.py:741-742 (see svla.h)
__global__ void embed_merge_kernel(int64_t rows, int64_t H, const int64_t* __restrict__ ids,
                                   const int32_t* __restrict__ img_index, const bf16_t* __restrict__ embed,
                                   const bf16_t* __restrict__ spatial, int64_t a0, int64_t na,
                                   const bf16_t* __restrict__ img, float normalizer, bf16_t* __restrict__ out) {
  const int64_t row = blockIdx.x;
  const int64_t id = ids[row];
  const int ii = img_index ? img_index[row] : -1;
  const int64_t nch = H >> 3;
  for (int64_t ch = threadIdx.x; ch < nch; ch += blockDim.x) {
    float v[8];
    if (ii >= 0) {
      unpack8(*reinterpret_cast<const u32x4*>(img + (int64_t)ii * H + ch * 8), v);
    } else if (spatial && id >= a0 && id < a0 + na) {
      float e[8];
      unpack8(*reinterpret_cast<const u32x4*>(embed + id * H + ch * 8), e);
      unpack8(*reinterpret_cast<const u32x4*>(spatial + (id - a0) * H + ch * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = round_bf(e[j] * 0.0f) + v[j];  // x*0.0 + spatial
    } else {
      unpack8(*reinterpret_cast<const u32x4*>(embed + id * H + ch * 8), v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j]) * normalizer;
    *reinterpret_cast<u32x4*>(out + row * H + ch * 8) = pack8(v);
  }
}

// image-feature grad: dimg[img_index[row]] = bf16(dout[row]*normalizer)
__global__ void embed_img_bwd_kernel(int64_t rows, int64_t H, const int32_t* __restrict__ img_index,
                                     const bf16_t* __restrict__ dout, float normalizer, bf16_t* __restrict__ dimg) {
  const int64_t row = blockIdx.x;
  const int ii = img_index[row];
  if (ii < 0) return;
  for (int64_t ch = threadIdx.x; ch < (H >> 3); ch += blockDim.x) {
    float v[8];
    unpack8(*reinterpret_cast<const u32x4*>(dout + row * H + ch * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= normalizer;
    *reinterpret_cast<u32x4*>(dimg + (int64_t)ii * H + ch * 8) = pack8(v);
  }
}

// spatial-table grad: one block per table row, summing its occurrences in sorted (CSR) order
__global__ void embed_spatial_bwd_kernel(int64_t H, const int32_t* __restrict__ sorted_rows,
                                         const int32_t* __restrict__ offsets, const bf16_t* __restrict__ dout,
                                         float normalizer, bf16_t* __restrict__ dspatial) {
  const int64_t sid = blockIdx.x;
  const int b = offsets[sid], e = offsets[sid + 1];
  for (int64_t ch = threadIdx.x; ch < (H >> 3); ch += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = b; i < e; ++i) {
      float v[8];
      unpack8(*reinterpret_cast<const u32x4*>(dout + (int64_t)sorted_rows[i] * H + ch * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += round_bf(v[j] * normalizer);
    }
    *reinterpret_cast<u32x4*>(dspatial + sid * H + ch * 8) = pack8(acc);
  }
}

// ------------------------------------------------------------------ Ego3D
// one block per (b, patch); thread layout: 12 coords x 17 features
__global__ void ego3d_kernel(int B, int Hd, int Wd, const float* __restrict__ depth, const float* __restrict__ kinv,
                             const float* __restrict__ uvh, int patch, int reso, int n_freqs,
                             bf16_t* __restrict__ feat, int64_t ldf, float* __restrict__ xyz_out) {
  const int b = blockIdx.y, p = blockIdx.x;
  const int hp = Hd / patch, wp = Wd / patch;
  const int py = p / wp, px = p % wp;
  const int gw = wp * reso, gh = hp * reso;  // area-pooled grid
  const int ry = Hd / gh, rx = Wd / gw;      // exact pooling window (224/32 = 7)
  __shared__ float xyz[64];
  const int npts = reso * reso;
  if ((int)threadIdx.x < npts) {
    const int sy = threadIdx.x / reso, sx = threadIdx.x % reso;
    const int gy = py * reso + sy, gx = px * reso + sx;
    // F.interpolate(mode="area") == mean over the ry x rx window; ZoeDepth's metric head returns fp32
    // depth, so the reference pools and back-projects in fp32 (no rounding here)
    float s = 0.f;
    for (int yy = 0; yy < ry; ++yy)
      for (int xx = 0; xx < rx; ++xx) s += depth[((int64_t)b * Hd + gy * ry + yy) * Wd + gx * rx + xx];
    const float d = s / (float)(ry * rx);
    const int idx = gy * gw + gx;
    const float u = uvh[idx], v = uvh[gh * gw + idx], w1 = uvh[2 * gh * gw + idx];
    const float* K = kinv + b * 9;
    for (int c = 0; c < 3; ++c) {
      const float pc = (K[c * 3 + 0] * u + K[c * 3 + 1] * v + K[c * 3 + 2] * w1) * d;
      xyz[threadIdx.x * 3 + c] = pc;
    }
  }
  __syncthreads();
  const int ncoord = npts * 3, nf = 2 * n_freqs + 1;
  bf16_t* frow = feat + ((int64_t)b * hp * wp + p) * ldf;
  for (int i = threadIdx.x; i < ldf; i += blockDim.x) {
    float o = 0.f;
    if (i < ncoord * nf) {
      const int m = i / nf, f = i % nf;
      const float center = (m % 3 == 2) ? 2.0f : 0.0f;
      const float xn = round_bf((xyz[m] - center) / 2.0f);
      if (f == 0) o = xn;
      else if (f <= n_freqs) o = sinf(round_bf(xn * (float)(1 << (f - 1))));
      else o = cosf(round_bf(xn * (float)(1 << (f - 1 - n_freqs))));
    }
    frow[i] = f2bf(o);
  }
  if (xyz_out && (int)threadIdx.x < ncoord) xyz_out[((int64_t)b * hp * wp + p) * ncoord + threadIdx.x] = xyz[threadIdx.x];
}

// ------------------------------------------------------------------ closed-form 3x3 inverse (camera intrinsics)
// inv(K) = adj(K) / det(K) in fp32, one thread per matrix: replaces torch.linalg.inv(K.float())
// (modeling_spatialvla.py:221), whose LU path checks its info on the host -- no sync here, capturable in a graph.
__global__ void inv3x3_kernel(int B, const float* __restrict__ K, float* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* k = K + 9 * b;
  const float a = k[0], bb = k[1], c = k[2], d = k[3], e = k[4], f = k[5], g = k[6], h = k[7], i = k[8];
  const float c00 = e * i - f * h, c01 = f * g - d * i, c02 = d * h - e * g;
  const float det = a * c00 + bb * c01 + c * c02;
  const float r = 1.0f / det;
  float* o = out + 9 * b;
  o[0] = c00 * r; o[1] = (c * h - bb * i) * r; o[2] = (bb * f - c * e) * r;
  o[3] = c01 * r; o[4] = (a * i - c * g) * r;  o[5] = (c * d - a * f) * r;
  o[6] = c02 * r; o[7] = (bb * g - a * h) * r; o[8] = (a * e - bb * d) * r;
}

// ------------------------------------------------------------------ SigLIP patchify
__global__ void im2col_kernel(int B, int S, int P, const bf16_t* __restrict__ x, bf16_t* __restrict__ cols,
                              int64_t ldc) {
  const int64_t r = blockIdx.x;  // b*np + patch
  const int np1 = S / P, np = np1 * np1;
  const int b = (int)(r / np), pi = (int)(r % np);
  const int py = pi / np1, px = pi % np1;
  const int K = 3 * P * P;
  for (int i = threadIdx.x; i < ldc; i += blockDim.x) {
    bf16_t v = 0;
    if (i < K) {
      const int c = i / (P * P), rem = i % (P * P), ky = rem / P, kx = rem % P;
      v = x[(((int64_t)b * 3 + c) * S + py * P + ky) * S + px * P + kx];
    }
    cols[r * ldc + i] = v;
  }
}

__global__ void affine_kernel(int64_t n, const bf16_t* __restrict__ x, float scale, float offset,
                              bf16_t* __restrict__ y) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  if (i + 8 <= n) {
    float v[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + i), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + offset) * scale;
    *reinterpret_cast<u32x4*>(y + i) = pack8(v);
  } else {
    for (int64_t j = i; j < n; ++j) y[j] = f2bf(round_bf(bf2f(x[j]) + offset) * scale);
  }
}

__global__ void relu_fwd_kernel(int64_t n, const bf16_t* __restrict__ x, bf16_t* __restrict__ y) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  for (int64_t j = i; j < min(n, i + 8); ++j) {
    float v = bf2f(x[j]);
    y[j] = f2bf(v > 0.f ? v : 0.f);
  }
}
__global__ void relu_bwd_kernel(int64_t n, const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                bf16_t* __restrict__ dx) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  for (int64_t j = i; j < min(n, i + 8); ++j) dx[j] = bf2f(x[j]) > 0.f ? dy[j] : (bf16_t)0;
}
// GeGLU backward (Gemma2MLP, modeling_gemma2.py:91-92, autograd of gelu_tanh(g) * u): dg = bf16(dh*u) * gelu'(g),
// du = dh * bf16(gelu(g)) with the reference's bf16 rounding points (the GEGLU_BWD GEMM epilogue's arithmetic).
// 8 columns per thread; dh may alias dg (each element is read before it is written).
__global__ __launch_bounds__(256) void geglu_bwd_kernel(int64_t M, int64_t I, const bf16_t* dh, int64_t ldh,
                                                        const bf16_t* __restrict__ g, int64_t ldg,
                                                        const bf16_t* __restrict__ u, int64_t ldu, bf16_t* dg,
                                                        int64_t lddg, bf16_t* __restrict__ du, int64_t lddu,
                                                        uint8_t* __restrict__ q, int64_t ldq, uint8_t* __restrict__ sc,
                                                        int64_t sld) {
  const int64_t cpr = I / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * cpr) return;
  const int64_t m = idx / cpr, c = (idx % cpr) * 8;
  float d[8], gv[8], uv[8], og[8], ou[8];
  unpack8(*reinterpret_cast<const u32x4*>(dh + m * ldh + c), d);
  unpack8(*reinterpret_cast<const u32x4*>(g + m * ldg + c), gv);
  unpack8(*reinterpret_cast<const u32x4*>(u + m * ldu + c), uv);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float act = gelu_bf16(gv[j]);
    const float dact = round_bf(d[j] * uv[j]);
    ou[j] = d[j] * act;
    og[j] = dact * gelu_tanh_grad(gv[j]);
  }
  *reinterpret_cast<u32x4*>(dg + m * lddg + c) = pack8(og);
  *reinterpret_cast<u32x4*>(du + m * lddu + c) = pack8(ou);
  if (q != nullptr) {  // also the MX e4m3 copy of [dg | du] (the fp8 dgrad operand), from the bf16 values just stored
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      og[j] = round_bf(og[j]);
      ou[j] = round_bf(ou[j]);
    }
    mx_store8(og, true, q + m * ldq + c, sc + (c / 128) * sld + m * 4);
    mx_store8(ou, true, q + m * ldq + I + c, sc + ((I + c) / 128) * sld + m * 4);
  }
}

// GELU as an HBM pass after a plain-store / bias GEMM (svla_gelu_rows): the VALU-heavy GELU epilogues ran slower
// inside the GEMM than as a separate read-once / write-once pass.  The rounding points of the fused epilogues:
// mode 0 y = bf16(gelu_tanh(x)), 1 y = bf16(gelu_erf(x)), 2 y = bf16(x * gelu_tanh'(pre)) (x = bf16 dL/dy).
// Modes 0 and 1: persistent blocks, gr_u<MODE>() 16-B chunks per thread loaded before any arithmetic, dense rows
// (ld == N everywhere) indexed linearly; mode 0 reads the gelu table from an LDS copy made once per block (from
// global memory every lookup was a scattered 2-B load): SigLIP fc1 38.1 -> 23.5 us isolated (profiles/r6i_gelu_ab.txt).
// Mode 2 keeps one chunk per thread, non-persistent (measured faster for it).
#ifndef GR_OLD
#define GR_OLD 0  // diagnostic builds: 1 = every mode one chunk per thread, non-persistent, global-memory table
#endif
template <int MODE>
constexpr bool gr_simple() { return GR_OLD || MODE == 2; }
template <int MODE>
constexpr int gr_u() { return MODE == 0 ? 1 : 2; }
template <int MODE>
__global__ __launch_bounds__(256) void gelu_rows_kernel(int64_t M, int64_t N, const bf16_t* x, int64_t ldx,
                                                        const bf16_t* __restrict__ pre, int64_t ldp, bf16_t* y,
                                                        int64_t ldy) {
  const int64_t cpr = N / 8;
  if constexpr (gr_simple<MODE>()) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= M * cpr) return;
    const int64_t m = idx / cpr, c = (idx % cpr) * 8;
    float v[8], o[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + m * ldx + c), v);
    if constexpr (MODE == 2) {
      float p[8];
      unpack8(*reinterpret_cast<const u32x4*>(pre + m * ldp + c), p);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[j] * gelu_tanh_grad(p[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = MODE == 0 ? gelu_bf16(v[j]) : gelu_erf(v[j]);
    }
    *reinterpret_cast<u32x4*>(y + m * ldy + c) = pack8(o);
    return;
  } else {
    __shared__ __attribute__((aligned(16))) unsigned short ltab[MODE == 0 ? 2 * SVLA_GELU_TAB_N : 8];
    if constexpr (MODE == 0) {
      constexpr int NCH = (int)(sizeof(svla_gelu_bf16_tab) / 16);
      for (int t = threadIdx.x; t < NCH; t += 256)
        reinterpret_cast<u32x4*>(ltab)[t] = reinterpret_cast<const u32x4*>(svla_gelu_bf16_tab)[t];
      __syncthreads();
    }
    const int64_t total = M * cpr;
    const bool dense = ldx == N && ldy == N && (MODE != 2 || ldp == N);
    auto off = [&](int64_t idx, int64_t ld) -> int64_t {
      if (dense) return idx * 8;
      const int64_t m = idx / cpr;
      return m * ld + (idx - m * cpr) * 8;
    };
    constexpr int U = gr_u<MODE>();
    const int64_t step = (int64_t)gridDim.x * 256 * U;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < total; base += step) {
      u32x4 xv[U], pv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int64_t idx = base + k * 256;
        if (idx < total) {
          xv[k] = *reinterpret_cast<const u32x4*>(x + off(idx, ldx));
          if constexpr (MODE == 2) pv[k] = *reinterpret_cast<const u32x4*>(pre + off(idx, ldp));
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int64_t idx = base + k * 256;
        if (idx >= total) break;
        float v[8], o[8];
        unpack8(xv[k], v);
        if constexpr (MODE == 2) {
          float p[8];
          unpack8(pv[k], p);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[j] * gelu_tanh_grad(p[j]);
        } else if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = gelu_bf16_lut(__float_as_uint(v[j]) >> 16, v[j], ltab);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = gelu_erf(v[j]);
        }
        *reinterpret_cast<u32x4*>(y + off(idx, ldy)) = pack8(o);
      }
    }
  }
}

__global__ void add_kernel(int64_t n, const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                           bf16_t* __restrict__ y) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  if (i + 8 <= n) {
    float u[8], v[8];
    unpack8(*reinterpret_cast<const u32x4*>(a + i), u);
    unpack8(*reinterpret_cast<const u32x4*>(b + i), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) u[j] += v[j];
    *reinterpret_cast<u32x4*>(y + i) = pack8(u);
  } else {
    for (int64_t j = i; j < n; ++j) y[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
  }
}

// ------------------------------------------------------------------ softcapped CE
// merge two online-softmax partials (max, sum of exp, argmax; ties to the smaller column)
__device__ __forceinline__ void ce_merge(float& mx, float& se, int& am, float m2, float s2, int a2) {
  if (m2 == -INFINITY) return;
  const float mn = fmaxf(mx, m2);
  se = (mx == -INFINITY ? 0.f : se * __expf(mx - mn)) + s2 * __expf(m2 - mn);
  if (m2 > mx || (m2 == mx && a2 < am)) am = a2;
  mx = mn;
}

// one wave per row: lanes stride over the row's 128-column partials (coalesced 12-B records), then a fixed
// butterfly merge -- deterministic, and every CU busy (a thread per row left the GPU on 39 CUs)
__global__ __launch_bounds__(256) void ce_finalize_kernel(int64_t M, int64_t N, int64_t ntiles,
                                                          const float* __restrict__ rs,
                                                          const bf16_t* __restrict__ logits, int64_t ldl,
                                                          const int64_t* __restrict__ target, float* __restrict__ lse,
                                                          int64_t* __restrict__ argmax, float* __restrict__ loss_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  float mx = -INFINITY, se = 0.f;
  int am = 0x7fffffff;
  const float* row = rs + m * ntiles * 3;
  for (int64_t t = lane; t < ntiles; t += 64)
    ce_merge(mx, se, am, row[t * 3], row[t * 3 + 1], __float_as_int(row[t * 3 + 2]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float m2 = __shfl_xor(mx, o, 64), s2 = __shfl_xor(se, o, 64);
    const int a2 = __shfl_xor(am, o, 64);
    ce_merge(mx, se, am, m2, s2, a2);
  }
  if (lane != 0) return;
  const float l = mx + __logf(se);
  lse[m] = l;
  argmax[m] = am;
  const int64_t tg = target ? target[m] : -1;
  loss_rows[m] = (tg >= 0 && tg < N) ? l - bf2f(logits[m * ldl + tg]) : 0.f;
}

__global__ void ce_loss_kernel(int64_t M, const float* __restrict__ loss_rows, const int64_t* __restrict__ target,
                               float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f, c = 0.f;
  for (int64_t m = threadIdx.x; m < M; m += blockDim.x) {
    s += loss_rows[m];
    c += (target && target[m] >= 0) ? 1.f : 0.f;
  }
  s = block_sum(s, red);
  c = block_sum(c, red);
  if (threadIdx.x == 0) {
    out[0] = s / fmaxf(c, 1.f);
    out[1] = c;
  }
}

// grid: (ceil(ldd/2048), M); each thread 8 columns
__global__ void ce_bwd_kernel(int64_t M, int64_t N, const bf16_t* __restrict__ logits, int64_t ldl,
                              const float* __restrict__ lse, const int64_t* __restrict__ target, float cap,
                              const float* __restrict__ gscale, bf16_t* __restrict__ d, int64_t ldd) {
  const int64_t m = blockIdx.y;
  const int64_t n = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (n >= ldd) return;
  const int64_t tg = target[m];
  u32x4 outv = {0u, 0u, 0u, 0u};
  if (tg >= 0 && n < N) {
    const float l = lse[m], sc = gscale[0];
    float y[8], o[8];
    if (n + 8 <= N) unpack8(*reinterpret_cast<const u32x4*>(logits + m * ldl + n), y);
    else
      for (int j = 0; j < 8; ++j) y[j] = (n + j < N) ? bf2f(logits[m * ldl + n + j]) : 0.f;
    const float icap = cap > 0.f ? 1.0f / cap : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (n + j < N) {
        float g = __expf(y[j] - l) - ((n + j == tg) ? 1.f : 0.f);
        g *= sc;
        // reference rounds the fp32 CE grad to bf16 at logits.float() and then differentiates the bf16 softcap
        g = round_bf(g);
        const float th = y[j] * icap;
        o[j] = cap > 0.f ? g * (1.0f - th * th) : g;
      } else {
        o[j] = 0.f;
      }
    }
    outv = pack8(o);
  }
  if (n + 8 <= ldd) *reinterpret_cast<u32x4*>(d + m * ldd + n) = outv;
  else {
    uint16_t tmp[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tmp[2 * j] = outv[j] & 0xffff;
      tmp[2 * j + 1] = outv[j] >> 16;
    }
    for (int j = 0; n + j < ldd; ++j) d[m * ldd + n + j] = tmp[j];
  }
}

// ------------------------------------------------------------------ norm + AdamW
__global__ void sumsq_stage1(int64_t n, const bf16_t* __restrict__ x, float* __restrict__ partial) {
  __shared__ float red[16];
  const int64_t per = (((n + gridDim.x - 1) / gridDim.x) + 7) & ~(int64_t)7;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  float s = 0.f;
  int64_t i = b0 + (int64_t)threadIdx.x * 8;
  // aligned vector body (b0 multiple of 8 when per is)
  for (; i + 8 <= b1; i += (int64_t)blockDim.x * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const u32x4*>(x + i), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  for (; i < b1; ++i) {
    float v = bf2f(x[i]);
    s += v * v;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}
__global__ void sumsq_stage2(int64_t np, const float* __restrict__ partial, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < np; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

__global__ void clip_kernel(const float* sumsq, float max_norm, float* clip, float* norm_out) {
  const float nrm = sqrtf(sumsq[0]);
  if (norm_out) norm_out[0] = nrm;
  clip[0] = (max_norm > 0.f) ? fminf(1.0f, max_norm / (nrm + 1e-6f)) : 1.0f;
}

#ifndef ADAMW_NT
#define ADAMW_NT 0
#endif
// 86 GB touched once per step; ADAMW_NT=1 (non-temporal loads/stores) measured 8.37 vs 7.66 ms at 1.5 G params
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (ADAMW_NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
__device__ __forceinline__ void st_stream(T* p, T v) {
  if constexpr (ADAMW_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

#ifndef ADAMW_U
#define ADAMW_U 1  // 8-element groups per thread per iteration (diagnostic A/B)
#endif
#ifndef ADAMW_NTS
#define ADAMW_NTS 0  // non-temporal stores only (diagnostic A/B)
#endif
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v) {
  if constexpr (ADAMW_NT || ADAMW_NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ void adamw_scalar(int64_t k, float* __restrict__ master, bf16_t* __restrict__ param,
                                             const bf16_t* __restrict__ grad, float* __restrict__ m,
                                             float* __restrict__ v, float lr, float b1, float b2, float eps, float wd,
                                             float bc1, float bc2, float cs) {
  const float gg = bf2f(grad[k]) * cs;
  m[k] = b1 * m[k] + (1.f - b1) * gg;
  v[k] = b2 * v[k] + (1.f - b2) * gg * gg;
  const float upd = (m[k] / bc1) / (sqrtf(v[k] / bc2) + eps);
  master[k] = master[k] - lr * (upd + wd * master[k]);
  param[k] = f2bf(master[k]);
}

__global__ void adamw_kernel(int64_t n, float* __restrict__ master, bf16_t* __restrict__ param,
                             const bf16_t* __restrict__ grad, float* __restrict__ m, float* __restrict__ v, float lr,
                             float b1, float b2, float eps, float wd, float bc1, float bc2,
                             const float* __restrict__ clip) {
  const float cs = clip ? clip[0] : 1.0f;
  // the two divides and the square root as 1-ulp hardware reciprocal / sqrt: the correctly rounded forms cost ~30
  // VALU instructions per element (the update agrees with torch.optim.AdamW to ~1e-7 relative)
  const float ibc1 = 1.0f / bc1, ibc2 = 1.0f / bc2;
  constexpr int U = ADAMW_U;
  const int64_t gs = (int64_t)blockDim.x * 8;  // elements a block covers per group
  const int64_t stride = (int64_t)gridDim.x * gs * U;
  for (int64_t base = (int64_t)blockIdx.x * gs * U + threadIdx.x * 8; base < n; base += stride) {
    if (base + (U - 1) * gs + 8 <= n) {
      float g[U][8], pp[U][8], mm[U][8], vv[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // every load of the U groups in flight before any arithmetic
        const int64_t i = base + u * gs;
        unpack8(ld_stream(reinterpret_cast<const u32x4*>(grad + i)), g[u]);
        const f32x4 p0 = ld_stream(reinterpret_cast<const f32x4*>(master + i)),
                    p1 = ld_stream(reinterpret_cast<const f32x4*>(master + i + 4));
        const f32x4 m0 = ld_stream(reinterpret_cast<const f32x4*>(m + i)),
                    m1 = ld_stream(reinterpret_cast<const f32x4*>(m + i + 4));
        const f32x4 v0 = ld_stream(reinterpret_cast<const f32x4*>(v + i)),
                    v1 = ld_stream(reinterpret_cast<const f32x4*>(v + i + 4));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          pp[u][q] = p0[q]; pp[u][4 + q] = p1[q];
          mm[u][q] = m0[q]; mm[u][4 + q] = m1[q];
          vv[u][q] = v0[q]; vv[u][4 + q] = v1[q];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * gs;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gg = g[u][j] * cs;
          mm[u][j] = b1 * mm[u][j] + (1.f - b1) * gg;
          vv[u][j] = b2 * vv[u][j] + (1.f - b2) * gg * gg;
          const float upd = (mm[u][j] * ibc1) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv[u][j] * ibc2) + eps);
          pp[u][j] = pp[u][j] - lr * (upd + wd * pp[u][j]);
        }
        st_out(reinterpret_cast<f32x4*>(master + i), f32x4{pp[u][0], pp[u][1], pp[u][2], pp[u][3]});
        st_out(reinterpret_cast<f32x4*>(master + i + 4), f32x4{pp[u][4], pp[u][5], pp[u][6], pp[u][7]});
        st_out(reinterpret_cast<f32x4*>(m + i), f32x4{mm[u][0], mm[u][1], mm[u][2], mm[u][3]});
        st_out(reinterpret_cast<f32x4*>(m + i + 4), f32x4{mm[u][4], mm[u][5], mm[u][6], mm[u][7]});
        st_out(reinterpret_cast<f32x4*>(v + i), f32x4{vv[u][0], vv[u][1], vv[u][2], vv[u][3]});
        st_out(reinterpret_cast<f32x4*>(v + i + 4), f32x4{vv[u][4], vv[u][5], vv[u][6], vv[u][7]});
        st_out(reinterpret_cast<u32x4*>(param + i), pack8(pp[u]));
      }
    } else {
      for (int u = 0; u < U; ++u) {
        const int64_t i = base + u * gs;
        if (i >= n) break;
        if (i + 8 <= n) {  // a whole group: the vector path's arithmetic
          float g[8], pp[8], mm[8], vv[8];
          unpack8(ld_stream(reinterpret_cast<const u32x4*>(grad + i)), g);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            pp[j] = master[i + j];
            mm[j] = m[i + j];
            vv[j] = v[i + j];
            const float gg = g[j] * cs;
            mm[j] = b1 * mm[j] + (1.f - b1) * gg;
            vv[j] = b2 * vv[j] + (1.f - b2) * gg * gg;
            const float upd = (mm[j] * ibc1) * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vv[j] * ibc2) + eps);
            pp[j] = pp[j] - lr * (upd + wd * pp[j]);
            master[i + j] = pp[j];
            m[i + j] = mm[j];
            v[i + j] = vv[j];
          }
          *reinterpret_cast<u32x4*>(param + i) = pack8(pp);
        } else {
          for (int64_t k = i; k < n; ++k) adamw_scalar(k, master, param, grad, m, v, lr, b1, b2, eps, wd, bc1, bc2, cs);
        }
      }
    }
  }
}

}  // namespace

extern "C" int svla_embed_merge(int64_t rows, int64_t H, const int64_t* ids, const int32_t* img_index,
                                const void* embed, const void* spatial, int64_t a0, int64_t na, const void* img,
                                float normalizer, void* out, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && H % 8 == 0 && ids && embed && out, "embed_merge: bad args");
  SVLA_CHECK_ARG(!img_index || img, "embed_merge: img_index without img");
  hipLaunchKernelGGL(embed_merge_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, rows, H, ids,
                     img_index, (const bf16_t*)embed, (const bf16_t*)spatial, a0, na, (const bf16_t*)img, normalizer,
                     (bf16_t*)out);
  return svla::check_launch("embed_merge");
}

extern "C" int svla_embed_merge_bwd(int64_t rows, int64_t H, const int64_t* ids, const int32_t* img_index,
                                    const int32_t* spatial_sorted_rows, const int32_t* spatial_offsets, int64_t na,
                                    const void* dout, float normalizer, void* dspatial, void* dimg, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && H % 8 == 0 && dout, "embed_merge_bwd: bad args");
  (void)ids;
  hipStream_t s = (hipStream_t)stream;
  if (dimg) {
    SVLA_CHECK_ARG(img_index != nullptr, "embed_merge_bwd: dimg needs img_index");
    hipLaunchKernelGGL(embed_img_bwd_kernel, dim3((unsigned)rows), dim3(256), 0, s, rows, H, img_index,
                       (const bf16_t*)dout, normalizer, (bf16_t*)dimg);
    if (int rc = svla::check_launch("embed_img_bwd")) return rc;
  }
  if (dspatial) {
    SVLA_CHECK_ARG(spatial_sorted_rows && spatial_offsets && na > 0, "embed_merge_bwd: spatial CSR missing");
    hipLaunchKernelGGL(embed_spatial_bwd_kernel, dim3((unsigned)na), dim3(256), 0, s, H, spatial_sorted_rows,
                       spatial_offsets, (const bf16_t*)dout, normalizer, (bf16_t*)dspatial);
    if (int rc = svla::check_launch("embed_spatial_bwd")) return rc;
  }
  return 0;
}

extern "C" int svla_ego3d_encode(int32_t B, int32_t Hd, int32_t Wd, const void* depth, const float* kinv,
                                 const float* uv_h, int32_t patch, int32_t reso, int32_t n_freqs, void* feat,
                                 int64_t ldf, float* xyz_out, void* stream) {
  SVLA_CHECK_ARG(B > 0 && depth && kinv && uv_h && feat, "ego3d: null");
  SVLA_CHECK_ARG(Hd % patch == 0 && Wd % patch == 0 && (Hd / patch * reso) > 0 && Hd % (Hd / patch * reso) == 0 &&
                     Wd % (Wd / patch * reso) == 0,
                 "ego3d: area pooling must be an exact integer window");
  SVLA_CHECK_ARG(reso * reso * 3 <= 64 && n_freqs <= 16 && ldf >= reso * reso * 3 * (2 * n_freqs + 1),
                 "ego3d: reso/n_freqs/ldf");
  dim3 grid((Hd / patch) * (Wd / patch), B);
  hipLaunchKernelGGL(ego3d_kernel, grid, dim3(256), 0, (hipStream_t)stream, B, Hd, Wd, (const float*)depth, kinv,
                     uv_h, patch, reso, n_freqs, (bf16_t*)feat, ldf, xyz_out);
  return svla::check_launch("ego3d");
}

extern "C" int svla_inv3x3_f32(int32_t B, const float* K, float* kinv, void* stream) {
  SVLA_CHECK_ARG(B > 0 && K && kinv, "inv3x3: bad args");
  hipLaunchKernelGGL(inv3x3_kernel, dim3((B + 63) / 64), dim3(64), 0, (hipStream_t)stream, B, K, kinv);
  return svla::check_launch("inv3x3");
}

extern "C" int svla_im2col_patch(int32_t B, int32_t S, int32_t patch, const void* x, void* cols, int64_t ldc,
                                 void* stream) {
  SVLA_CHECK_ARG(B > 0 && S % patch == 0 && x && cols && ldc >= 3 * patch * patch, "im2col: bad args");
  const int64_t rows = (int64_t)B * (S / patch) * (S / patch);
  hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, B, S, patch,
                     (const bf16_t*)x, (bf16_t*)cols, ldc);
  return svla::check_launch("im2col");
}

extern "C" int svla_affine_bf16(int64_t n, const void* x, float scale, float offset, void* out, void* stream) {
  SVLA_CHECK_ARG(n > 0 && x && out && al16(x) && al16(out), "affine: bad args");
  hipLaunchKernelGGL(affine_kernel, dim3(nblk(n, 256 * 8)), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)x,
                     scale, offset, (bf16_t*)out);
  return svla::check_launch("affine");
}
extern "C" int svla_relu_fwd(int64_t n, const void* x, void* y, void* stream) {
  SVLA_CHECK_ARG(n > 0 && x && y, "relu: bad args");
  hipLaunchKernelGGL(relu_fwd_kernel, dim3(nblk(n, 256 * 8)), dim3(256), 0, (hipStream_t)stream, n,
                     (const bf16_t*)x, (bf16_t*)y);
  return svla::check_launch("relu_fwd");
}
extern "C" int svla_relu_bwd(int64_t n, const void* x, const void* dy, void* dx, void* stream) {
  SVLA_CHECK_ARG(n > 0 && x && dy && dx, "relu_bwd: bad args");
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(nblk(n, 256 * 8)), dim3(256), 0, (hipStream_t)stream, n,
                     (const bf16_t*)x, (const bf16_t*)dy, (bf16_t*)dx);
  return svla::check_launch("relu_bwd");
}
extern "C" int svla_add_bf16(int64_t n, const void* a, const void* b, void* out, void* stream) {
  SVLA_CHECK_ARG(n > 0 && a && b && out && al16(a) && al16(b) && al16(out), "add: bad args");
  hipLaunchKernelGGL(add_kernel, dim3(nblk(n, 256 * 8)), dim3(256), 0, (hipStream_t)stream, n, (const bf16_t*)a,
                     (const bf16_t*)b, (bf16_t*)out);
  return svla::check_launch("add");
}

extern "C" int svla_ce_finalize(int64_t M, int64_t N, int64_t ntiles, const float* row_stats, const void* logits,
                                int64_t ldl, const int64_t* target, float* lse, int64_t* argmax, float* loss_rows,
                                float* loss_out, void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && row_stats && logits && lse && argmax && loss_rows && loss_out, "ce_finalize: args");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(nblk(M, 4)), dim3(256), 0, s, M, N, ntiles, row_stats,
                     (const bf16_t*)logits, ldl, target, lse, argmax, loss_rows);
  if (int rc = svla::check_launch("ce_finalize")) return rc;
  hipLaunchKernelGGL(ce_loss_kernel, dim3(1), dim3(1024), 0, s, M, loss_rows, target, loss_out);
  return svla::check_launch("ce_loss");
}

extern "C" int svla_ce_bwd(int64_t M, int64_t N, const void* logits, int64_t ldl, const float* lse,
                           const int64_t* target, float cap, const float* grad_scale, void* dlogits, int64_t ldd,
                           void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && logits && lse && target && grad_scale && dlogits, "ce_bwd: args");
  SVLA_CHECK_ARG(ldl % 8 == 0 && ldd % 8 == 0 && ldd >= N, "ce_bwd: ld");
  dim3 grid(nblk(ldd, 256 * 8), (unsigned)M);
  hipLaunchKernelGGL(ce_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, M, N, (const bf16_t*)logits, ldl, lse,
                     target, cap, grad_scale, (bf16_t*)dlogits, ldd);
  return svla::check_launch("ce_bwd");
}

extern "C" int svla_sumsq_bf16(int64_t n, const void* x, float* partial, int64_t n_partial, float* out,
                               void* stream) {
  SVLA_CHECK_ARG(n > 0 && x && partial && out && n_partial > 0 && n_partial <= 65535 && al16(x), "sumsq: args");
  hipStream_t s = (hipStream_t)stream;
  // per-block chunk must stay 8-aligned for the vector body
  hipLaunchKernelGGL(sumsq_stage1, dim3((unsigned)n_partial), dim3(256), 0, s, n, (const bf16_t*)x, partial);
  if (int rc = svla::check_launch("sumsq1")) return rc;
  hipLaunchKernelGGL(sumsq_stage2, dim3(1), dim3(1024), 0, s, n_partial, partial, out);
  return svla::check_launch("sumsq2");
}

extern "C" int svla_clip_scale(const float* sumsq, float max_norm, float* clip_scale, float* norm_out, void* stream) {
  SVLA_CHECK_ARG(sumsq && clip_scale, "clip: args");
  hipLaunchKernelGGL(clip_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, sumsq, max_norm, clip_scale, norm_out);
  return svla::check_launch("clip");
}

extern "C" int svla_adamw(int64_t n, float* master, void* param_bf16, const void* grad_bf16, float* m, float* v,
                          float lr, float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2,
                          const float* clip_scale, void* stream) {
  SVLA_CHECK_ARG(n > 0 && master && param_bf16 && grad_bf16 && m && v, "adamw: args");
  SVLA_CHECK_ARG(al16(master) && al16(param_bf16) && al16(grad_bf16) && al16(m) && al16(v), "adamw: alignment");
#ifndef ADAMW_GRID
#define ADAMW_GRID (256 * 64)  // block cap (diagnostic A/B)
#endif
  unsigned g = nblk(n, 256 * 8 * ADAMW_U);
  if (g > ADAMW_GRID) g = ADAMW_GRID;
  hipLaunchKernelGGL(adamw_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, n, master, (bf16_t*)param_bf16,
                     (const bf16_t*)grad_bf16, m, v, lr, beta1, beta2, eps, weight_decay, bc1, bc2, clip_scale);
  return svla::check_launch("adamw");
}

extern "C" int svla_geglu_bwd(int64_t M, int64_t I, const void* dh, int64_t ldh, const void* g, int64_t ldg,
                              const void* u, int64_t ldu, void* dg, int64_t lddg, void* du, int64_t lddu,
                              void* stream) {
  SVLA_CHECK_ARG(M > 0 && I > 0 && I % 8 == 0 && dh && g && u && dg && du, "geglu_bwd: bad args");
  SVLA_CHECK_ARG(ldh % 8 == 0 && ldg % 8 == 0 && ldu % 8 == 0 && lddg % 8 == 0 && lddu % 8 == 0 && al16(dh) &&
                     al16(g) && al16(u) && al16(dg) && al16(du),
                 "geglu_bwd: rows must be 16-B aligned");
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(nblk(M * (I / 8), 256)), dim3(256), 0, (hipStream_t)stream, M, I,
                     (const bf16_t*)dh, ldh, (const bf16_t*)g, ldg, (const bf16_t*)u, ldu, (bf16_t*)dg, lddg,
                     (bf16_t*)du, lddu, (uint8_t*)nullptr, (int64_t)0, (uint8_t*)nullptr, (int64_t)0);
  return svla::check_launch("geglu_bwd");
}

extern "C" int svla_geglu_bwd_mx(int64_t M, int64_t I, const void* dh, int64_t ldh, const void* g, int64_t ldg,
                                 const void* u, int64_t ldu, void* dg, int64_t lddg, void* du, int64_t lddu, void* q,
                                 int64_t ldq, void* scales, int64_t sld, void* stream) {
  SVLA_CHECK_ARG(M > 0 && I > 0 && I % 128 == 0 && dh && g && u && dg && du && q && scales,
                 "geglu_bwd_mx: bad args (I a multiple of 128)");
  SVLA_CHECK_ARG(ldh % 8 == 0 && ldg % 8 == 0 && ldu % 8 == 0 && lddg % 8 == 0 && lddu % 8 == 0 && al16(dh) &&
                     al16(g) && al16(u) && al16(dg) && al16(du),
                 "geglu_bwd_mx: rows must be 16-B aligned");
  SVLA_CHECK_ARG(ldq >= 2 * I && ldq % 8 == 0 && ((uintptr_t)q & 7) == 0 && ((uintptr_t)scales & 3) == 0 &&
                     sld >= 4 * M && sld % 4 == 0,
                 "geglu_bwd_mx: q [M][ldq >= 2I] 8-B rows, scale tile stride >= 4 M");
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(nblk(M * (I / 8), 256)), dim3(256), 0, (hipStream_t)stream, M, I,
                     (const bf16_t*)dh, ldh, (const bf16_t*)g, ldg, (const bf16_t*)u, ldu, (bf16_t*)dg, lddg,
                     (bf16_t*)du, lddu, (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  return svla::check_launch("geglu_bwd_mx");
}

extern "C" int svla_gelu_rows(int64_t M, int64_t N, int32_t mode, const void* x, int64_t ldx, const void* pre,
                              int64_t ldp, void* y, int64_t ldy, void* stream) {
  SVLA_CHECK_ARG(M > 0 && N > 0 && N % 8 == 0 && mode >= 0 && mode <= 2 && x && y && (mode != 2 || pre),
                 "gelu_rows: M, N (multiple of 8), mode 0..2, pointers");
  SVLA_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0 && (mode != 2 || ldp % 8 == 0) && al16(x) && al16(y) &&
                     (mode != 2 || al16(pre)), "gelu_rows: rows must be 16-B aligned");
  const int64_t chunks = M * (N / 8);
  auto grid = [&](bool simple, int u) {
    return dim3(simple ? nblk(chunks, 256)
                       : (unsigned)std::min<int64_t>(nblk(chunks, 256 * u), (int64_t)svla::num_cus() * 8));
  };
  const dim3 b(256);
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0)
    hipLaunchKernelGGL(gelu_rows_kernel<0>, grid(gr_simple<0>(), gr_u<0>()), b, 0, s, M, N, (const bf16_t*)x, ldx,
                       (const bf16_t*)pre, ldp, (bf16_t*)y, ldy);
  else if (mode == 1)
    hipLaunchKernelGGL(gelu_rows_kernel<1>, grid(gr_simple<1>(), gr_u<1>()), b, 0, s, M, N, (const bf16_t*)x, ldx,
                       (const bf16_t*)pre, ldp, (bf16_t*)y, ldy);
  else
    hipLaunchKernelGGL(gelu_rows_kernel<2>, grid(gr_simple<2>(), gr_u<2>()), b, 0, s, M, N, (const bf16_t*)x, ldx,
                       (const bf16_t*)pre, ldp, (bf16_t*)y, ldy);
  return svla::check_launch("gelu_rows");
}

// ---------------------------------------------------------------- action-token accuracy (integer, bit-exact)
// train/monkey_patch.py:267-309: pred[b,t] = argmax over V of logits[b,t] (t < L-1), gt[b,t] = labels[b,t+1];
// rows with gt in [trans_lo, grip_hi] count; correct = gt == pred, split by the translation / rotation / gripper id
// ranges.  One workgroup (a step has ~10^4 rows); integer sums, so the result is order-independent.
__global__ __launch_bounds__(1024) void action_accuracy_kernel(int64_t B, int64_t L, const int64_t* pred,
                                                               int64_t ldp, const int64_t* labels, int64_t ldl,
                                                               int64_t t_lo, int64_t t_hi, int64_t r_lo,
                                                               int64_t r_hi, int64_t g_lo, int64_t g_hi,
                                                               int64_t* counts, float* acc) {
  __shared__ int64_t red[8][1024 / 64];
  int64_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // {n, ok} x {all, translation, rotation, gripper}
  const int64_t rows = B * (L - 1);
  for (int64_t i = threadIdx.x; i < rows; i += blockDim.x) {
    const int64_t b = i / (L - 1), t = i % (L - 1);
    const int64_t gt = labels[b * ldl + t + 1];
    if (gt < t_lo || gt > g_hi) continue;
    const int64_t ok = pred[b * ldp + t] == gt ? 1 : 0;
    c[0] += 1;
    c[1] += ok;
    const int k = (gt >= t_lo && gt <= t_hi) ? 1 : (gt >= r_lo && gt <= r_hi) ? 2 : (gt >= g_lo && gt <= g_hi) ? 3 : 0;
    if (k) {
      c[2 * k] += 1;
      c[2 * k + 1] += ok;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int64_t v = c[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[j][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    int64_t v = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[threadIdx.x][k];
    counts[threadIdx.x] = v;
    red[threadIdx.x][0] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4)  // torch: correct.sum().float() / mask.sum().float() (0/0 -> nan)
    acc[threadIdx.x] = (float)red[2 * threadIdx.x + 1][0] / (float)red[2 * threadIdx.x][0];
}

extern "C" int svla_action_accuracy(int64_t B, int64_t L, const int64_t* pred, int64_t ldp, const int64_t* labels,
                                    int64_t ldl, const int64_t* ranges, int64_t* counts, float* acc, void* stream) {
  SVLA_CHECK_ARG(B > 0 && L > 1 && pred && labels && ranges && counts && acc && ldp >= L - 1 && ldl >= L,
                 "action_accuracy: bad args");
  SVLA_CHECK_ARG(ranges[0] <= ranges[1] && ranges[1] < ranges[2] && ranges[2] <= ranges[3] && ranges[3] < ranges[4] &&
                     ranges[4] <= ranges[5],
                 "action_accuracy: token ranges must be ordered translation < rotation < gripper");
  hipLaunchKernelGGL(action_accuracy_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, L, pred, ldp, labels,
                     ldl, ranges[0], ranges[1], ranges[2], ranges[3], ranges[4], ranges[5], counts, acc);
  return svla::check_launch("action_accuracy");
}
