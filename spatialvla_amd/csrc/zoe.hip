// ZoeDepth metric head tail, fused (frozen depth estimator, reference model/modeling_spatialvla.py:314-323 ->
// transformers ZoeDepthMetricDepthEstimationHead.forward [3p]).  Per output pixel (b, i, j):
//
//   last   = cat(outconv_activation[b, :, i, j] (C_F channels), relative_depth[b, i, j])
//   cond   = bilinear_align_corners(bin_embedding_lowres)[b, :, i, j]            (C_E channels)
//   h      = GELU(conv1x1_W1(cat(last, cond)) + b1)                               (HID = (C_F+1+C_E)/2)
//   s      = softplus(conv1x1_W2(h) + b2)                                          (4 channels)
//   p      = (s0+eps)/((s0+eps)+(s1+eps)),  t = (max_t-min_t)*(s2+eps)/((s2+eps)+(s3+eps)) + min_t
//   y_k    = logbinom(NB-1, k) + k*log(clamp(p)) + (NB-1-k)*log(clamp(1-p)),   x = softmax_k(y / t)
//   depth  = sum_k x_k * bilinear_align_corners(bin_centers_lowres)[b, k, i, j]
//
// The stock path materialises [B,161,H,W] bf16, [B,64,H,W] fp32 probabilities and two upsampled
// copies (several GB at B=32, 384x384); here every intermediate stays in registers.  Every bf16 rounding
// point of the eager reference (interpolation outputs, conv outputs, GELU, softplus, the elementwise bf16
// ops on p and t, k*log(p)) is reproduced; accumulation orders of the 1x1 convs and the final sum are
// fp32 but not bit-identical to MIOpen / torch.sum.
#include "svla_common.h"

namespace {

struct ZoeTailArgs {
  int B, H, W, h, w;            // output and low-resolution sizes
  int CF;                       // outconv_activation channels (main feature without the relative depth)
  int CE;                       // bin-embedding channels
  const bf16_t* feat; int64_t fs[4];   // [B, CF, H, W] element strides (b, c, y, x)
  const bf16_t* rel;  int64_t rs[3];   // [B, H, W]
  const bf16_t* emb;  int64_t es[4];   // [B, CE, h, w]
  const bf16_t* ctr;  int64_t cs[4];   // [B, NB, h, w]
  float p_eps, max_t, min_t, clamp_eps;
  float* out;                   // [B, H, W] fp32
};

constexpr int HID = 80, NB = 64, CIN_MAX = 192;

// branch-free erfc (Numerical Recipes erfcc, Chebyshev fit; fractional error < 1.2e-7 everywhere): libm's erff
// branches per argument range, which diverges across a wave and dominated this kernel.  The GELU output is
// rounded to bf16, far coarser than the fit error.
__device__ __forceinline__ float erfc_pos(float z) {  // z >= 0
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);  // 1-ulp reciprocal: the fit's own error is 1.2e-7
  const float p = -1.26551223f + t * (1.00002368f + t * (0.37409196f + t * (0.09678418f + t * (-0.18628806f +
                  t * (0.27886807f + t * (-1.13520398f + t * (1.48851587f + t * (-0.82215223f + t * 0.17087277f))))))));
  return t * __expf(-z * z + p);
}
// nn.GELU() (erf form): 0.5*x*(1+erf(x/sqrt2)); 1+erf(u) = erfc(-u) keeps negative arguments exact
__device__ __forceinline__ float gelu_erf(float x) {
  const float u = x * 0.70710678118654752f;
  const float one_plus_erf = u >= 0.f ? 2.0f - erfc_pos(u) : erfc_pos(-u);
  return 0.5f * x * one_plus_erf;
}
__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(__expf(x)); }

// align_corners=True bilinear source coordinate (ATen area_pixel_compute_source_index, fp32)
struct Tap {
  int i0, i1;
  float l0, l1;
};
__device__ __forceinline__ Tap tap(int dst, int in, int out) {
  const float scale = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
  const float src = scale * (float)dst;
  Tap t;
  t.i0 = (int)src;
  t.i1 = t.i0 + ((t.i0 < in - 1) ? 1 : 0);
  t.l1 = src - (float)t.i0;
  t.l0 = 1.f - t.l1;
  return t;
}
struct Taps2 {  // the four source offsets (elements) and weights of one output pixel
  int64_t o00, o01, o10, o11;
  float ly0, ly1, lx0, lx1;
};
__device__ __forceinline__ Taps2 taps2(const int64_t* s, const Tap& ty, const Tap& tx) {
  Taps2 t;
  t.o00 = ty.i0 * s[2] + tx.i0 * s[3];
  t.o01 = ty.i0 * s[2] + tx.i1 * s[3];
  t.o10 = ty.i1 * s[2] + tx.i0 * s[3];
  t.o11 = ty.i1 * s[2] + tx.i1 * s[3];
  t.ly0 = ty.l0; t.ly1 = ty.l1; t.lx0 = tx.l0; t.lx1 = tx.l1;
  return t;
}
// ATen upsample_bilinear2d (align_corners) value in fp32, rounded to the bf16 output
__device__ __forceinline__ float bilerp(const bf16_t* p, const Taps2& t) {
  const float a = bf2f(p[t.o00]), b = bf2f(p[t.o01]), c = bf2f(p[t.o10]), d = bf2f(p[t.o11]);
  return round_bf(t.ly0 * (t.lx0 * a + t.lx1 * b) + t.ly1 * (t.lx0 * c + t.lx1 * d));
}

// Parameters, fp32, one buffer (prepared once per module by the host): W1^T [CIN][HID], W2 [4][HID], b1 [HID],
// b2 [4], logbinom [NB].  Every read is at a wave-uniform address, so hipcc keeps them in SGPRs (s_load):
// the 1x1-conv FMAs take their weight as a scalar operand, no LDS traffic.
__device__ __forceinline__ void load8(const bf16_t* p, int64_t stride, bool vec, float* v) {
  if (vec) {
    unpack8(*reinterpret_cast<const u32x4*>(p), v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(p[j * stride]);
  }
}

// The hidden layer (CF+1+CE -> 80 1x1 conv, 98 % of the tail's FLOPs) runs on MFMA: a block owns 256 output pixels,
// each wave 64 of them as 4 groups of 16; the conv's input channels are permuted (feat 0..CF-1, emb CF.., rel last,
// zero pad to 192 = 6 k-steps of 32) on both operands, the weights are staged once per block in LDS in fragment
// order (bf16, exact: the module's weights are bf16), and every lane gathers the 8 channels of its (pixel, k-step)
// A fragment straight from the inputs (16-B loads, the bin embedding bilinearly interpolated and rounded to bf16 as
// the reference's upsampled tensor).  bf16(h + b1) goes through LDS back to one thread per pixel for the rest.
constexpr int KP = 192, KS = KP / 32, NT = HID / 16, HS_LD = HID + 8;
constexpr int ZT_LDS = KS * NT * 64 * 16 + 256 * HS_LD * 2;

__global__ __launch_bounds__(256, 2) void zoe_tail_kernel(ZoeTailArgs a, const float* __restrict__ prm) {
  extern __shared__ __attribute__((aligned(16))) char zsm[];
  bf16_t* wl = (bf16_t*)zsm;                              // [KS][NT][64 lanes][8] B fragments
  bf16_t* hs = (bf16_t*)(zsm + KS * NT * 64 * 16);         // [256 pixels][HS_LD] bf16(h + b1)
  const int CIN = a.CF + 1 + a.CE;
  const float* __restrict__ pw1 = prm;
  const float* __restrict__ pw2 = pw1 + CIN * HID;
  const float* __restrict__ pb1 = pw2 + 4 * HID;
  const float* __restrict__ pb2 = pb1 + HID;
  const float* __restrict__ plb = pb2 + 4;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t npix = (int64_t)a.B * a.H * a.W;
  const int64_t pix0 = (int64_t)blockIdx.x * 256;

  // permuted channel kk -> row of W1^T (-1: zero pad)
  auto wrow = [&](int kk) {
    if (kk < a.CF) return kk;
    if (kk < a.CF + a.CE) return kk + 1;
    if (kk == a.CF + a.CE) return a.CF;
    return -1;
  };
  for (int i = t; i < KS * NT * 64; i += 256) {  // fragment (ks, nt, lane): B[k = 32ks + 8(l>>4) + j][o = 16nt + (l&15)]
    const int l = i & 63, nt = (i >> 6) % NT, ks = (i >> 6) / NT;
    const int o = 16 * nt + (l & 15);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = wrow(32 * ks + 8 * (l >> 4) + j);
      v[j] = r >= 0 ? pw1[r * HID + o] : 0.f;
    }
    *reinterpret_cast<u32x4*>(wl + i * 8) = pack8(v);
  }
  __syncthreads();

  // one 16-pixel group at a time: its NT accumulators go to LDS as soon as its k-steps are done (20 live accumulator
  // registers instead of 80; with every group live the kernel ran at one wave per SIMD)
  const int g4 = lane >> 4;
#pragma unroll 1
  for (int pg = 0; pg < 4; ++pg) {
    f32x4 hacc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) hacc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    int64_t pix = pix0 + 64 * w + 16 * pg + (lane & 15);
    const bool pv = pix < npix;
    if (!pv) pix = npix - 1;
    const int x = (int)(pix % a.W), y = (int)((pix / a.W) % a.H), b = (int)(pix / ((int64_t)a.W * a.H));
    const Tap ty = tap(y, a.h, a.H), tx = tap(x, a.w, a.W);
    const Taps2 te = taps2(a.es, ty, tx);
    const bf16_t* fp = a.feat + (int64_t)b * a.fs[0] + y * a.fs[2] + x * a.fs[3];
    const bf16_t* eb = a.emb + (int64_t)b * a.es[0];
    const bool vf = a.fs[1] == 1, ve = a.es[1] == 1;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kk = 32 * ks + 8 * g4;  // first permuted channel of this lane's 8
      float v[8];
      if (kk < a.CF) {
        load8(fp + kk * a.fs[1], a.fs[1], vf, v);
      } else if (kk < a.CF + a.CE) {
        float q00[8], q01[8], q10[8], q11[8];
        const bf16_t* pc = eb + (kk - a.CF) * a.es[1];
        load8(pc + te.o00, a.es[1], ve, q00);
        load8(pc + te.o01, a.es[1], ve, q01);
        load8(pc + te.o10, a.es[1], ve, q10);
        load8(pc + te.o11, a.es[1], ve, q11);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = round_bf(te.ly0 * (te.lx0 * q00[j] + te.lx1 * q01[j]) + te.ly1 * (te.lx0 * q10[j] + te.lx1 * q11[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = 0.f;
        if (kk == a.CF + a.CE) v[0] = bf2f(a.rel[(int64_t)b * a.rs[0] + y * a.rs[1] + x * a.rs[2]]);
      }
      const bf16x8 af = __builtin_bit_cast(bf16x8, pack8(v));
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wl + ((ks * NT + nt) * 64 + lane) * 8);
        hacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, hacc[nt], 0, 0, 0);
      }
    }
    // C[pixel row 4(l>>4)+i][output 16nt + (l&15)] -> hs[pixel][o] = bf16(h + b1)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int o = 16 * nt + (lane & 15);
      const float bias = pb1[o];
#pragma unroll
      for (int i = 0; i < 4; ++i) hs[(64 * w + 16 * pg + 4 * g4 + i) * HS_LD + o] = f2bf(hacc[nt][i] + bias);
    }
  }
  __syncthreads();

  const int64_t pix = pix0 + t;
  if (pix >= npix) return;
  const int x = (int)(pix % a.W);
  const int y = (int)((pix / a.W) % a.H);
  const int b = (int)(pix / ((int64_t)a.W * a.H));
  const Tap ty = tap(y, a.h, a.H), tx = tap(x, a.w, a.W);
  float s4[4] = {pb2[0], pb2[1], pb2[2], pb2[3]};
#pragma unroll 2
  for (int o8 = 0; o8 < HID / 8; ++o8) {  // the hidden row in 8-channel pieces (not 80 registers at once)
    float h[8];
    unpack8(*reinterpret_cast<const u32x4*>(hs + t * HS_LD + 8 * o8), h);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = 8 * o8 + j;
      const float g = round_bf(gelu_erf(round_bf(h[j])));
#pragma unroll
      for (int q = 0; q < 4; ++q) s4[q] += pw2[q * HID + o] * g;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) s4[q] = round_bf(softplus_f(round_bf(s4[q])));
  // probabilities / temperature with the reference's bf16 elementwise ops
  const float p0 = round_bf(s4[0] + a.p_eps), p1 = round_bf(s4[1] + a.p_eps);
  float p = round_bf(p0 / round_bf(p0 + p1));
  const float t0 = round_bf(s4[2] + a.p_eps), t1 = round_bf(s4[3] + a.p_eps);
  const float tq = round_bf(t0 / round_bf(t0 + t1));
  const float temp = round_bf(round_bf((a.max_t - a.min_t) * tq) + a.min_t);
  // LogBinomialSoftmax: om = clamp(1 - p), p = clamp(p); y_k = lb_k + bf16(k*log p) + bf16((NB-1-k)*log om)
  const float om = round_bf(fminf(fmaxf(round_bf(1.f - p), a.clamp_eps), 1.f));
  p = round_bf(fminf(fmaxf(p, a.clamp_eps), 1.f));
  const float lp = round_bf(__logf(p)), lom = round_bf(__logf(om));
  const float itemp = __builtin_amdgcn_rcpf(temp);
  auto zk = [&](int k) { return (plb[k] + round_bf((float)k * lp) + round_bf((float)(NB - 1 - k) * lom)) * itemp; };
  float zmax = -INFINITY;
#pragma unroll 8
  for (int k = 0; k < NB; ++k) zmax = fmaxf(zmax, zk(k));
  float se = 0.f, acc = 0.f;
  const Taps2 tc = taps2(a.cs, ty, tx);
  const bf16_t* cb = a.ctr + (int64_t)b * a.cs[0];
  const bool cvec = a.cs[1] == 1;
#pragma unroll 1
  for (int k0 = 0; k0 < NB; k0 += 8) {
    float q00[8], q01[8], q10[8], q11[8];
    const bf16_t* pc = cb + k0 * a.cs[1];
    load8(pc + tc.o00, a.cs[1], cvec, q00);
    load8(pc + tc.o01, a.cs[1], cvec, q01);
    load8(pc + tc.o10, a.cs[1], cvec, q10);
    load8(pc + tc.o11, a.cs[1], cvec, q11);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float bc =
          round_bf(tc.ly0 * (tc.lx0 * q00[j] + tc.lx1 * q01[j]) + tc.ly1 * (tc.lx0 * q10[j] + tc.lx1 * q11[j]));
      const float e = __expf(zk(k0 + j) - zmax);
      se += e;
      acc += e * bc;
    }
  }
  a.out[pix] = acc / se;
}

// ---------------------------------------------------------------------------------------------
// Bilinear resize of a channels-last bf16 map (torch upsample_bilinear2d_nhwc_out_frame semantics, used by the
// ZoeDepth DPT neck: ZoeDepthFeatureFusionLayer's interpolate(scale_factor=2, align_corners=True) and the
// relative head's nn.Upsample).  One thread = one output pixel x 8 channels (four 16-B loads, one 16-B store)
// instead of torch's one element per thread; source index, lambdas and the blend in fp32 in torch's order.
struct UpsArgs {
  int B, C, H1, W1, H2, W2, align;
  float rh, rw;
  const bf16_t* in;
  bf16_t* out;
};

__device__ __forceinline__ float ups_src(float scale, int dst, int align) {
  if (align) return scale * (float)dst;
  const float src = scale * ((float)dst + 0.5f) - 0.5f;
  return src < 0.f ? 0.f : src;
}

__global__ __launch_bounds__(256) void upsample_bilinear_nhwc_kernel(UpsArgs a) {
  const int cg = a.C >> 3;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.H2 * a.W2 * cg;
  if (idx >= total) return;
  const int c8 = (int)(idx % cg);
  int64_t r = idx / cg;
  const int w2 = (int)(r % a.W2);
  r /= a.W2;
  const int h2 = (int)(r % a.H2);
  const int n = (int)(r / a.H2);
  const float h1r = ups_src(a.rh, h2, a.align);
  const int h1 = (int)h1r;
  const int h1p = (h1 < a.H1 - 1) ? 1 : 0;
  const float h1lambda = h1r - (float)h1;
  const float h0lambda = 1.f - h1lambda;
  const float w1r = ups_src(a.rw, w2, a.align);
  const int w1 = (int)w1r;
  const int w1p = (w1 < a.W1 - 1) ? 1 : 0;
  const float w1lambda = w1r - (float)w1;
  const float w0lambda = 1.f - w1lambda;
  const int64_t rowb = (int64_t)n * a.H1;
  auto at = [&](int y, int x) {
    return *reinterpret_cast<const u32x4*>(a.in + ((rowb + y) * a.W1 + x) * a.C + 8 * c8);
  };
  float p00[8], p01[8], p10[8], p11[8], o[8];
  unpack8(at(h1, w1), p00);
  unpack8(at(h1, w1 + w1p), p01);
  unpack8(at(h1 + h1p, w1), p10);
  unpack8(at(h1 + h1p, w1 + w1p), p11);
  // torch's expression as hipcc contracts it (the one ordering found bitwise-equal to the stock NHWC kernel
  // on MI355X, tools/ups_variants.py): fma over the w-pairs, then over the h-pair
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float t0 = fmaf(w0lambda, p00[j], w1lambda * p01[j]), t1 = fmaf(w0lambda, p10[j], w1lambda * p11[j]);
    o[j] = fmaf(h0lambda, t0, h1lambda * t1);
  }
  *reinterpret_cast<u32x4*>(a.out + (((int64_t)n * a.H2 + h2) * a.W2 + w2) * a.C + 8 * c8) = pack8(o);
}

// ---------------------------------------------------------------------------------------------
// ZoeDepthAttractorLayerUnnormed's bin update (transformers zoedepth [3p], the nyu-kitti head's four attractor
// layers, memory_efficient, "mean"/"sum"): for every (b, bin k, y, x) with c = bin_centers[b, k, y, x]
//   delta = 0;  for i < n_att: delta = bf16(delta + inv_attractor(bf16(A[b, i, y, x] - c)))
//   delta = bf16(delta / n_att) (mean);  out = bf16(c + delta)
// inv_attractor(dx) = dx / (1 + alpha dx^gamma) (the TorchScript-fused kernel: fp32 from the bf16 dx, one rounding),
// the bf16 rounding of each eager op between -- the 3 n_att + 2 launches and the bf16 traffic of the stock loop in
// one pass.  One thread = 8 consecutive bins of one pixel (channels-last maps: one 16-B load / store).
struct AttrArgs {
  int B, H, W, NA, NB, mean;
  float alpha;
  int gamma;
  const bf16_t* A; int64_t as[4];     // attractors [B, NA, H, W], element strides (b, c, y, x)
  const bf16_t* C; int64_t cs[4];     // bin centres [B, NB, H, W]
  bf16_t* out; int64_t os[4];         // new bin centres [B, NB, H, W]
};

__global__ __launch_bounds__(256) void zoe_attractor_kernel(AttrArgs a) {
  const int ng = a.NB / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.H * a.W * ng;
  if (idx >= total) return;
  const int kg = (int)(idx % ng);
  int64_t r = idx / ng;
  const int x = (int)(r % a.W);
  r /= a.W;
  const int y = (int)(r % a.H);
  const int b = (int)(r / a.H);
  const int k0 = 8 * kg;
  float c[8], d[8];
  const bf16_t* cp = a.C + (int64_t)b * a.cs[0] + y * a.cs[2] + x * a.cs[3] + k0 * a.cs[1];
  if (a.cs[1] == 1) {
    unpack8(*reinterpret_cast<const u32x4*>(cp), c);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = bf2f(cp[j * a.cs[1]]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
  const bf16_t* ap = a.A + (int64_t)b * a.as[0] + y * a.as[2] + x * a.as[3];
  for (int i = 0; i < a.NA; ++i) {
    const float ai = bf2f(ap[i * a.as[1]]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float dx = round_bf(ai - c[j]);
      float p = dx;
      for (int q = 1; q < a.gamma; ++q) p = p * dx;
      d[j] = round_bf(d[j] + round_bf(dx / (a.alpha * p + 1.0f)));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (a.mean) d[j] = round_bf(d[j] * (1.0f / (float)a.NA));
    d[j] = c[j] + d[j];
  }
  bf16_t* op = a.out + (int64_t)b * a.os[0] + y * a.os[2] + x * a.os[3] + k0 * a.os[1];
  if (a.os[1] == 1) {
    *reinterpret_cast<u32x4*>(op) = pack8(d);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) op[j * a.os[1]] = f2bf(d[j]);
  }
}

// DPT readout "project" input (transformers ZoeDepthReassembleStage.forward [3p]): row r = (b, t) of the
// [B*T, 2C] output is [hidden(b, 1 + t, :), hidden(b, 0, :)] -- the stacking cat, the NCHW round trip and the
// readout cat of the stock module as one 16-B copy per chunk.
__global__ __launch_bounds__(256) void zoe_readout_cat_kernel(int64_t B, int64_t T, int64_t C,
                                                              const bf16_t* __restrict__ hs, bf16_t* __restrict__ out) {
  const int64_t cpr = C >> 3;  // 16-B chunks per half row
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * T * 2 * cpr) return;
  const int64_t r = idx / (2 * cpr), j = idx - r * 2 * cpr;
  const int64_t b = r / T, t = r - b * T;
  const bf16_t* src = j < cpr ? hs + (b * (T + 1) + 1 + t) * C + 8 * j : hs + b * (T + 1) * C + 8 * (j - cpr);
  *reinterpret_cast<u32x4*>(out + r * 2 * C + 8 * j) = *reinterpret_cast<const u32x4*>(src);
}

}  // namespace

extern "C" int svla_zoe_readout_cat(int64_t B, int64_t T, int64_t C, const void* hidden, void* out, void* stream) {
  SVLA_CHECK_ARG(B > 0 && T > 0 && C > 0 && C % 8 == 0 && hidden && out, "zoe_readout_cat: bad args");
  SVLA_CHECK_ARG(((uintptr_t)hidden & 15) == 0 && ((uintptr_t)out & 15) == 0, "zoe_readout_cat: 16-B alignment");
  const int64_t total = B * T * (C / 4);
  hipLaunchKernelGGL(zoe_readout_cat_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     B, T, C, (const bf16_t*)hidden, (bf16_t*)out);
  return svla::check_launch("zoe_readout_cat");
}

extern "C" int svla_zoe_attractor(int B, int H, int W, int n_att, int n_bins, const void* attractors,
                                  const int64_t* a_strides, const void* centres, const int64_t* c_strides, float alpha,
                                  int gamma, int mean, void* out, const int64_t* out_strides, void* stream) {
  SVLA_CHECK_ARG(B > 0 && H > 0 && W > 0 && n_att > 0 && n_bins > 0 && n_bins % 8 == 0 && gamma >= 1,
                 "zoe_attractor: bad sizes (bins a multiple of 8, gamma >= 1)");
  SVLA_CHECK_ARG(attractors && centres && out && a_strides && c_strides && out_strides, "zoe_attractor: NULL");
  SVLA_CHECK_ARG((c_strides[1] != 1 || ((uintptr_t)centres & 15) == 0) && (out_strides[1] != 1 || ((uintptr_t)out & 15) == 0),
                 "zoe_attractor: channels-last maps must be 16-B aligned");
  AttrArgs a;
  a.B = B; a.H = H; a.W = W; a.NA = n_att; a.NB = n_bins; a.mean = mean ? 1 : 0; a.alpha = alpha; a.gamma = gamma;
  a.A = (const bf16_t*)attractors; a.C = (const bf16_t*)centres; a.out = (bf16_t*)out;
  for (int i = 0; i < 4; ++i) { a.as[i] = a_strides[i]; a.cs[i] = c_strides[i]; a.os[i] = out_strides[i]; }
  const int64_t total = (int64_t)B * H * W * (n_bins / 8);
  hipLaunchKernelGGL(zoe_attractor_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
  return svla::check_launch("zoe_attractor");
}

extern "C" int svla_zoe_metric_tail(int B, int H, int W, int h, int w, int CF, int CE, int NBins, int Hid,
                                    const void* feat, const int64_t* feat_strides, const void* rel,
                                    const int64_t* rel_strides, const void* emb, const int64_t* emb_strides,
                                    const void* ctr, const int64_t* ctr_strides, const float* params, float p_eps,
                                    float max_t, float min_t, float clamp_eps, float* out, void* stream) {
  SVLA_CHECK_ARG(B > 0 && H > 1 && W > 1 && h > 1 && w > 1 && CF > 0 && CE > 0, "zoe_tail: bad sizes");
  SVLA_CHECK_ARG(NBins == NB && Hid == HID && (CF + 1 + CE) / 2 == HID && CF % 8 == 0 && CE % 8 == 0,
                 "zoe_tail: built for %d bins, %d hidden channels, channel counts multiples of 8 (got %d, %d, %d, %d)",
                 NB, HID, NBins, Hid, CF, CE);
  SVLA_CHECK_ARG(feat && rel && emb && ctr && params && out, "zoe_tail: NULL pointer");
  const bool vf = feat_strides[1] == 1, ve = emb_strides[1] == 1, vc = ctr_strides[1] == 1;
  SVLA_CHECK_ARG((!vf || ((uintptr_t)feat & 15) == 0) && (!ve || ((uintptr_t)emb & 15) == 0) &&
                     (!vc || ((uintptr_t)ctr & 15) == 0),
                 "zoe_tail: channels-last inputs must be 16-B aligned");
  ZoeTailArgs a;
  a.B = B; a.H = H; a.W = W; a.h = h; a.w = w; a.CF = CF; a.CE = CE;
  a.feat = (const bf16_t*)feat; a.rel = (const bf16_t*)rel; a.emb = (const bf16_t*)emb; a.ctr = (const bf16_t*)ctr;
  for (int i = 0; i < 4; ++i) { a.fs[i] = feat_strides[i]; a.es[i] = emb_strides[i]; a.cs[i] = ctr_strides[i]; }
  for (int i = 0; i < 3; ++i) a.rs[i] = rel_strides[i];
  a.p_eps = p_eps; a.max_t = max_t; a.min_t = min_t; a.clamp_eps = clamp_eps; a.out = out;
  const int64_t npix = (int64_t)B * H * W;
  SVLA_CHECK_ARG(CF + 1 + CE <= KP, "zoe_tail: at most %d input channels", KP);
  static bool lds_set = false;
  if (!lds_set) {
    (void)hipFuncSetAttribute((const void*)zoe_tail_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, ZT_LDS);
    lds_set = true;
  }
  hipLaunchKernelGGL(zoe_tail_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), ZT_LDS, (hipStream_t)stream,
                     a, params);
  return svla::check_launch("zoe_metric_tail");
}

extern "C" int svla_upsample_bilinear_nhwc(int B, int C, int H1, int W1, int H2, int W2, int align_corners,
                                           float rh, float rw, const void* in, void* out, void* stream) {
  SVLA_CHECK_ARG(B > 0 && C > 0 && H1 > 0 && W1 > 0 && H2 > 0 && W2 > 0, "upsample: bad sizes");
  SVLA_CHECK_ARG(C % 8 == 0, "upsample: channel count must be a multiple of 8 (got %d)", C);
  SVLA_CHECK_ARG(in && out && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0,
                 "upsample: NULL or misaligned pointer");
  UpsArgs a;
  a.B = B; a.C = C; a.H1 = H1; a.W1 = W1; a.H2 = H2; a.W2 = W2; a.align = align_corners ? 1 : 0;
  a.rh = rh; a.rw = rw; a.in = (const bf16_t*)in; a.out = (bf16_t*)out;
  const int64_t total = (int64_t)B * H2 * W2 * (C / 8);
  hipLaunchKernelGGL(upsample_bilinear_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return svla::check_launch("upsample_bilinear_nhwc");
}

// ---------------------------------------------------------------------------------------------
// process_zoe (reference model/modeling_spatialvla.py:99-110) and the depth resize after the estimator (:318-323)
// as one pass each, instead of pad + upsample_bicubic2d + sub + div (and upsample_bicubic2d + crop + copy) on ATen.
//  * zoe_preprocess: out[b,c,oy,ox] = bf16(bf16(bicubic(reflect_pad(x, P))[oy,ox] - mean_c) / std_c): the padded
//    (H+2P)x(W+2P) image is never formed (a tap at padded coordinate p reads x at reflect(p - P)); bicubic as torch's
//    upsample_bicubic2d (align_corners=True: source = scale * dst, scale = (in - 1) / (out - 1); A = -0.75; taps
//    clamped to the padded image's border), fp32, rounded to bf16 once; TF.normalize's sub and div each rounded to
//    bf16 as torch's bf16 elementwise kernels do.
//  * zoe_depth_resize: out[b,y,x] = bf16(bicubic(depth[b], size (H+2P)x(W+2P))[y+P, x+P]): only the rows and
//    columns the crop [..., P:-P, P:-P] keeps are computed.
// Two contraction forms of torch's expressions (V): 0 = as hipcc contracts them under -ffp-contract=fast, 1 = every
// product and sum rounded separately; tests/test_model_gpu.py compares both with the stock ops.
// ---------------------------------------------------------------------------------------------
namespace {
struct ZoePre {
  int B, C, H, W, P, OH, OW;
  float scale_h, scale_w;
  float mean[4], stdv[4];
  const bf16_t* x;
  bf16_t* out;
};

template <int V>
__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  constexpr float A = -0.75f;
  if constexpr (V == 0) {
    auto cc1 = [](float x) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; };
    auto cc2 = [](float x) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; };
    c[0] = cc2(t + 1.f);
    c[1] = cc1(t);
    c[2] = cc1(1.f - t);
    c[3] = cc2((1.f - t) + 1.f);
  } else {
    auto cc1 = [](float x) {
      return __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(__fmul_rn(A + 2.f, x), A + 3.f), x), x), 1.f);
    };
    auto cc2 = [](float x) {
      return __fsub_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fsub_rn(__fmul_rn(A, x), 5.f * A), x), 8.f * A), x), 4.f * A);
    };
    c[0] = cc2(__fadd_rn(t, 1.f));
    c[1] = cc1(t);
    const float x2 = __fsub_rn(1.f, t);
    c[2] = cc1(x2);
    c[3] = cc2(__fadd_rn(x2, 1.f));
  }
}

template <int V>
__device__ __forceinline__ float cubic_1d(float x0, float x1, float x2, float x3, const float c[4]) {
  if constexpr (V == 0) return x0 * c[0] + x1 * c[1] + x2 * c[2] + x3 * c[3];
  else return __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(x0, c[0]), __fmul_rn(x1, c[1])), __fmul_rn(x2, c[2])),
                        __fmul_rn(x3, c[3]));
}

__device__ __forceinline__ int reflect_idx(int p, int n) {  // F.pad reflect for one overhang (p in (-n, 2n - 1))
  return p < 0 ? -p : (p >= n ? 2 * (n - 1) - p : p);
}

// bicubic sample of a (virtually padded) image at output (oy, ox): fetch(yy, xx) reads the unpadded source
template <int V, typename Fetch>
__device__ __forceinline__ float bicubic_at(int oy, int ox, float sh, float sw, int IH, int IW, Fetch fetch) {
  const float ry = sh * (float)oy, rx = sw * (float)ox;
  const int iy = (int)floorf(ry), ix = (int)floorf(rx);
  const float ty = ry - (float)iy, tx = rx - (float)ix;
  float cx[4], cy[4], rows[4];
  cubic_coeffs<V>(tx, cx);
  cubic_coeffs<V>(ty, cy);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int yy = min(max(iy - 1 + k, 0), IH - 1);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = fetch(yy, min(max(ix - 1 + j, 0), IW - 1));
    rows[k] = cubic_1d<V>(v[0], v[1], v[2], v[3], cx);
  }
  return cubic_1d<V>(rows[0], rows[1], rows[2], rows[3], cy);
}

template <int V>
__global__ __launch_bounds__(256) void zoe_preprocess_kernel(ZoePre a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.C * a.OH * a.OW;
  if (idx >= total) return;
  const int ox = (int)(idx % a.OW);
  int64_t r = idx / a.OW;
  const int oy = (int)(r % a.OH);
  r /= a.OH;
  const int c = (int)(r % a.C);
  const int b = (int)(r / a.C);
  const bf16_t* src = a.x + ((int64_t)b * a.C + c) * a.H * a.W;
  const int PH = a.H + 2 * a.P, PW = a.W + 2 * a.P;
  auto fetch = [&](int py, int px) {
    return bf2f(src[(int64_t)reflect_idx(py - a.P, a.H) * a.W + reflect_idx(px - a.P, a.W)]);
  };
  const float v = round_bf(bicubic_at<V>(oy, ox, a.scale_h, a.scale_w, PH, PW, fetch));
  const float y = round_bf(v - a.mean[c]);
  a.out[idx] = f2bf(__fdiv_rn(y, a.stdv[c]));
}

struct ZoeDepthRs {
  int B, IH, IW, P, OH, OW;  // OH x OW: the cropped output; the resize target is (OH + 2P) x (OW + 2P)
  float scale_h, scale_w;
  const bf16_t* depth;
  bf16_t* out;
};

template <int V>
__global__ __launch_bounds__(256) void zoe_depth_resize_kernel(ZoeDepthRs a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)a.B * a.OH * a.OW;
  if (idx >= total) return;
  const int x = (int)(idx % a.OW);
  int64_t r = idx / a.OW;
  const int y = (int)(r % a.OH);
  const int b = (int)(r / a.OH);
  const bf16_t* src = a.depth + (int64_t)b * a.IH * a.IW;
  auto fetch = [&](int yy, int xx) { return bf2f(src[(int64_t)yy * a.IW + xx]); };
  a.out[idx] = f2bf(bicubic_at<V>(y + a.P, x + a.P, a.scale_h, a.scale_w, a.IH, a.IW, fetch));
}

int g_zoe_bicubic_variant = 0;  // diagnostic switch (svla_diag_zoe_bicubic_variant), 0 in the product
}  // namespace

extern "C" int svla_diag_zoe_bicubic_variant(int v) {  // diagnostics only (not in svla.h)
  SVLA_CHECK_ARG(v == 0 || v == 1, "zoe bicubic variant %d", v);
  g_zoe_bicubic_variant = v;
  return 0;
}

extern "C" int svla_zoe_preprocess(int B, int C, int H, int W, int pad, int OH, int OW, const void* x,
                                   const float* mean, const float* stdv, void* out, void* stream) {
  SVLA_CHECK_ARG(B > 0 && C > 0 && C <= 4 && H > 1 && W > 1 && pad >= 0 && pad < H && pad < W && OH > 1 && OW > 1,
                 "zoe_preprocess: bad sizes (C <= 4, reflect pad < H, W)");
  SVLA_CHECK_ARG(x && mean && stdv && out, "zoe_preprocess: NULL pointer");
  ZoePre a;
  a.B = B; a.C = C; a.H = H; a.W = W; a.P = pad; a.OH = OH; a.OW = OW;
  a.scale_h = (float)(H + 2 * pad - 1) / (float)(OH - 1);
  a.scale_w = (float)(W + 2 * pad - 1) / (float)(OW - 1);
  for (int i = 0; i < 4; ++i) {
    a.mean[i] = i < C ? mean[i] : 0.f;
    a.stdv[i] = i < C ? stdv[i] : 1.f;
  }
  a.x = (const bf16_t*)x;
  a.out = (bf16_t*)out;
  const int64_t total = (int64_t)B * C * OH * OW;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (g_zoe_bicubic_variant) hipLaunchKernelGGL(zoe_preprocess_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(zoe_preprocess_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, a);
  return svla::check_launch("zoe_preprocess");
}

extern "C" int svla_zoe_depth_resize(int B, int IH, int IW, int pad, int OH, int OW, const void* depth, void* out,
                                     void* stream) {
  SVLA_CHECK_ARG(B > 0 && IH > 1 && IW > 1 && pad >= 0 && OH > 0 && OW > 0, "zoe_depth_resize: bad sizes");
  SVLA_CHECK_ARG(depth && out, "zoe_depth_resize: NULL pointer");
  ZoeDepthRs a;
  a.B = B; a.IH = IH; a.IW = IW; a.P = pad; a.OH = OH; a.OW = OW;
  a.scale_h = (float)(IH - 1) / (float)(OH + 2 * pad - 1);
  a.scale_w = (float)(IW - 1) / (float)(OW + 2 * pad - 1);
  a.depth = (const bf16_t*)depth;
  a.out = (bf16_t*)out;
  const int64_t total = (int64_t)B * OH * OW;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (g_zoe_bicubic_variant) hipLaunchKernelGGL(zoe_depth_resize_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(zoe_depth_resize_kernel<0>, grid, dim3(256), 0, (hipStream_t)stream, a);
  return svla::check_launch("zoe_depth_resize");
}
