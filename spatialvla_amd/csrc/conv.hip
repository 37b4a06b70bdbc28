// Implicit-GEMM NHWC convolutions for gfx950 (MI355X): the frozen ZoeDepth DPT neck and depth heads
// (transformers zoedepth [3p], called by the reference at model/modeling_spatialvla.py:314-323).
//
//   out[b, oy, ox, co] = epi( sum_{ky, kx, ci} act(x[b, oy*s + ky - p, ox*s + kx - p, ci]) * w[co, ky, kx, ci] )
//
// as a GEMM with M = B*OH*OW output pixels, N = Cout, K = KH*KW*Cin, never materialising the im2col matrix:
//  * A (the shifted input pixels) streams global -> LDS by buffer_load_dwordx4 ... lds with a per-lane source
//    address recomputed per 64-deep k-tile: each lane owns a few tile rows (pixels) and one 8-channel chunk, whose
//    (tap, channel) advances incrementally; zero padding, ragged rows and the K tail read as zeros through the
//    buffer descriptor's range check (OOB offset), so no branch guards a load.
//  * B (weights, [Cout][KH][KW][Cin] = K-contiguous rows) is an ordinary KC operand.
//  * v_mfma_f32_16x16x32_bf16, two LDS stages, k-tiles t+1 and t+2 in flight behind a counted vmcnt.
//  * Pre-activation ReLU (DPT's PreActResidualLayer: relu -> conv) is applied to the A fragments in registers
//    (v_pk_max_i16 against 0 is relu on bf16 bit patterns), so the relu'd input is never written to HBM.
//  * Epilogue through an fp32 LDS image in 64-row passes: bf16(acc + bias), optional relu, up to two residual
//    adds each rounded to bf16 (the eager module order), 16-B stores along the channels.  The transposed
//    convolution with kernel == stride (the reassemble resize) is the 1x1 GEMM N = f*f*Cout whose epilogue scatters
//    each 8-channel chunk to its output pixel (pixel shuffle), so no output is written twice.
#include "svla_common.h"

namespace {

#ifndef CONV_SPLIT_MAX
#define CONV_SPLIT_MAX 8  // split-K factor cap of the sub-wave 64x64 grids (diagnostic A/B: 1 = no split)
#endif
#ifndef CONV_SMALL
#define CONV_SMALL 1  // 64 x 64 tiles for sub-wave grids (diagnostic A/B: 0 = always 128 x 128)
#endif

constexpr int CBK = 64;
constexpr uint32_t COOB = 0x80000000u;

struct ConvK {
  const bf16_t* x;
  const bf16_t* w;
  const bf16_t* bias;
  const bf16_t* res1;
  const bf16_t* res2;
  bf16_t* out;
  int B, H, W, Cin, OH, OW, Cout, KH, KW, stride, pad, flags, factor;
  int RH, RW;  // the GEMM rows are B x RH x RW pixels: the output pixels, or the input pixels (transposed form)
  int N, K;
  int64_t M;
  int S;           // split-K factor (1 = none): slabs / counters in the caller's GEMM workspace
  float* slabs;
  int* counters;
};

template <int BM_, int BN_, int WGM_, int WGN_>
struct CCfg {
  static constexpr int BM = BM_, BN = BN_, WGM = WGM_, WGN = WGN_;
  static constexpr int NW = WGM * WGN, NTH = 64 * NW;
  static constexpr int WTM = BM / WGM, WTN = BN / WGN, TM = WTM / 16, TN = WTN / 16;
  static constexpr int A_BYTES = BM * CBK * 2, B_BYTES = BN * CBK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int IA = BM / (8 * NW), IB = BN / (8 * NW);
  static constexpr int EPI_LD = BN + 4;
  static constexpr int EPI_BYTES = 64 * EPI_LD * 4;
  static constexpr int LDS = 2 * STAGE > EPI_BYTES ? 2 * STAGE : EPI_BYTES;
  static_assert(IA >= 1 && IB >= 1, "tile too small for the wave count");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile must be a multiple of 16");
};
using ConvBig = CCfg<256, 128, 4, 2>;   // Cout >= 128: 8 waves, 64x64 per wave
using ConvMid = CCfg<128, 128, 2, 2>;   // 4 waves, 64x64 per wave
using ConvNarrow = CCfg<256, 32, 4, 1>; // Cout 32: 4 waves, 64x32 per wave
using ConvSmall = CCfg<64, 64, 2, 2>;   // sub-wave grids (the B = 1 DPT neck): 4 waves, 32x32 per wave

__device__ __forceinline__ bf16x8 relu8(bf16x8 v) {
  // relu on bf16 bit patterns: a negative bf16 is a negative int16, so max(x, 0) as packed int16 is relu
  u32x4 u = __builtin_bit_cast(u32x4, v);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t r;
    asm volatile("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(u[i]));
    u[i] = r;
  }
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ bf16x8 read_kc(const char* lds, int rb, int ks, int lane) {
  const int row = rb + (lane & 15);
  const int chunk = 4 * ks + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
}

template <typename C, bool PRE_RELU>
__global__ __launch_bounds__(C::NTH, 2) void conv_kernel(ConvK p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = C::BM, BN = C::BN, NTH = C::NTH, TM = C::TM, TN = C::TN, IA = C::IA, IB = C::IB;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  __shared__ int sflag;
  const int tiles_m = (int)((p.M + BM - 1) / BM), tiles_n = (p.N + BN - 1) / BN;
  const int total = tiles_m * tiles_n;
  int tm, tn, split = 0;
  if (p.S > 1) {  // gemm.hip's split-K hand-off: block (tile, split), the M tiles of a (split, column tile) adjacent
    const int L = xcd_remap(blockIdx.x, total * p.S);
    split = L / total;
    const int tile = L % total;
    tm = tile % tiles_m;
    tn = tile / tiles_m;
  } else {
    const int pid = xcd_remap(blockIdx.x, total);
    constexpr int GM = 8;
    const int group = GM * tiles_n;
    const int first_m = (pid / group) * GM;
    const int gsz = min(tiles_m - first_m, GM);
    tm = first_m + (pid % group) % gsz;
    tn = (pid % group) / gsz;
  }
  const int nk_all = (p.K + CBK - 1) / CBK;
  const int kb = (int)((int64_t)split * nk_all / p.S);
  const int nk = (int)((int64_t)(split + 1) * nk_all / p.S) - kb;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const int wr = w / C::WGN, wc = w % C::WGN;

  // ---- A: this lane's pixel rows and its k chunk (tap, channel), advanced by 64 per k-tile
  const int gc = (lane & 7) ^ (lane >> 3);
  int iy0[IA], ix0[IA], pb[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int64_t m = m0 + 8 * (w * IA + i) + (lane >> 3);
    if (m < p.M) {
      const int64_t ohw = (int64_t)p.RH * p.RW;
      const int b = (int)(m / ohw);
      const int r = (int)(m - (int64_t)b * ohw);
      const int oy = r / p.RW, ox = r - oy * p.RW;
      iy0[i] = oy * p.stride - p.pad;
      ix0[i] = ox * p.stride - p.pad;
      pb[i] = b * p.H * p.W;
    } else {
      iy0[i] = -(1 << 28);  // fails the range check for every tap
      ix0[i] = 0;
      pb[i] = 0;
    }
  }
  int kk = kb * CBK + gc * 8;    // this lane's k within the current k-tile's stream
  int tap = kk / p.Cin, ci = kk - tap * p.Cin;
  int ky = tap / p.KW, kx = tap - ky * p.KW;
  const int ntap = p.KH * p.KW;
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.x);
  auto issue_a = [&](char* dst) {
    const bool kok = tap < ntap;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int iy = iy0[i] + ky, ix = ix0[i] + kx;
      const bool ok = kok && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const uint32_t voff = ok ? (uint32_t)(((pb[i] + iy * p.W + ix) * p.Cin + ci) * 2) : COOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (LDS_AS void*)(dst + (w * IA + i) * 1024), 16, voff, 0, 0, 0);
    }
    // advance to the next k-tile: 64 channels further along the (tap, channel) order
    ci += CBK;
    while (ci >= p.Cin) {
      ci -= p.Cin;
      ++tap;
      if (++kx == p.KW) { kx = 0; ++ky; }
    }
  };
  // ---- B: weight rows n0 .. (K-contiguous)
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.w);
  uint32_t wv[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int n = n0 + 8 * (w * IB + i) + (lane >> 3);
    wv[i] = n < p.N ? (uint32_t)(((int64_t)n * p.K + gc * 8) * 2) : COOB;
  }
  auto issue_b = [&](char* dst, int k0) {
    const bool kok = k0 + gc * 8 < p.K;
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const uint32_t voff = (kok && wv[i] != COOB) ? wv[i] + (uint32_t)(k0 * 2) : COOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (LDS_AS void*)(dst + (w * IB + i) * 1024), 16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int NLD = IA + IB;
  issue_a(smem);
  issue_b(smem + C::A_BYTES, kb * CBK);
  if (nk > 1) {
    issue_a(smem + C::STAGE);
    issue_b(smem + C::STAGE + C::A_BYTES, (kb + 1) * CBK);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLD) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* la = smem + cur * C::STAGE;
    const char* lb = la + C::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        af[i] = read_kc(la, C::WTM * wr + 16 * i, ks, lane);
        if (PRE_RELU) af[i] = relu8(af[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = read_kc(lb, C::WTN * wc + 16 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) {
      issue_a(smem + cur * C::STAGE);
      issue_b(smem + cur * C::STAGE + C::A_BYTES, (kb + kt + 2) * CBK);
    }
  }
  if (p.S > 1) {
    // slab per (tile, split) stored write-through, arrival counter, the last arriver sums the slabs in split order
    // (gemm.hip gemm_kernel's hand-off; deterministic whichever block is last) and runs the epilogue
    const int tile = tm + tn * tiles_m;
    constexpr int SLAB = TM * TN * NTH * 16;
    const char* base = reinterpret_cast<const char*>(p.slabs) + (int64_t)tile * p.S * SLAB;
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
      int* cnt = p.counters + tile;
      const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sflag = (old == p.S - 1);
      if (old == p.S - 1) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!sflag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll 1
    for (int sg = 0; sg < p.S; ++sg) {
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

  // ---- epilogue: 64-row passes through the fp32 image
  constexpr int EPI_LD = C::EPI_LD;
  constexpr int CPR = BN / 8, RPP = NTH / CPR;
  float* Ei = reinterpret_cast<float*>(smem);
  const int cc = t % CPR;
  const int n = n0 + 8 * cc;
  const bool transposed = (p.flags & SVLA_CONV_TRANSPOSED) != 0;
  const int co = transposed ? n % p.Cout : n;
  float bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = 0.f;
  if (p.bias && n < p.N) unpack8(*reinterpret_cast<const u32x4*>(p.bias + co), bias);
#pragma unroll 1
  for (int pass = 0; pass < BM / 64; ++pass) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rbase = C::WTM * wr + 16 * i;
      if (rbase >= 64 * pass && rbase < 64 * pass + 64) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = C::WTN * wc + 16 * j + (lane & 15);
          const int r = rbase - 64 * pass + 4 * (lane >> 4);
#pragma unroll
          for (int q = 0; q < 4; ++q) Ei[(r + q) * EPI_LD + col] = acc[i][j][q];
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (n < p.N) {
#pragma unroll 1
      for (int rr = t / CPR; rr < 64; rr += RPP) {
        const int64_t m = m0 + 64 * pass + rr;
        if (m >= p.M) break;
        const float* pe = Ei + rr * EPI_LD + 8 * cc;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(pe), x1 = *reinterpret_cast<const f32x4*>(pe + 4);
        float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        int64_t o;
        if (transposed) {  // pixel shuffle: input pixel m, tap (dy, dx) of the f x f kernel
          const int64_t hw = (int64_t)p.H * p.W;
          const int b = (int)(m / hw);
          const int r = (int)(m - (int64_t)b * hw);
          const int iy = r / p.W, ix = r - iy * p.W;
          const int dd = n / p.Cout, dy = dd / p.factor, dx = dd - dy * p.factor;
          o = (((int64_t)b * p.OH + iy * p.factor + dy) * p.OW + ix * p.factor + dx) * p.Cout + co;
        } else {
          o = m * p.Cout + n;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = round_bf(v[j] + bias[j]);
          if (p.flags & SVLA_CONV_POST_RELU) v[j] = fmaxf(v[j], 0.f);
        }
        if (p.res1) {
          float r[8];
          unpack8(*reinterpret_cast<const u32x4*>(p.res1 + o), r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + r[j]);
        }
        if (p.res2) {
          float r[8];
          unpack8(*reinterpret_cast<const u32x4*>(p.res2 + o), r);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = round_bf(v[j] + r[j]);
        }
        *reinterpret_cast<u32x4*>(p.out + o) = pack8(v);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

template <typename C>
int launch_conv(const ConvK& k, bool pre_relu, hipStream_t s) {
  const int64_t tiles = ((k.M + C::BM - 1) / C::BM) * ((k.N + C::BN - 1) / C::BN) * k.S;
  if (tiles > 0x7fffffff) return SVLA_ERR_ARG;
  static bool set0 = false, set1 = false;
  if (pre_relu) {
    if (!set1) {
      (void)hipFuncSetAttribute((const void*)conv_kernel<C, true>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
      set1 = true;
    }
    hipLaunchKernelGGL((conv_kernel<C, true>), dim3((unsigned)tiles), dim3(C::NTH), C::LDS, s, k);
  } else {
    if (!set0) {
      (void)hipFuncSetAttribute((const void*)conv_kernel<C, false>, hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
      set0 = true;
    }
    hipLaunchKernelGGL((conv_kernel<C, false>), dim3((unsigned)tiles), dim3(C::NTH), C::LDS, s, k);
  }
  return svla::check_launch("conv2d_nhwc");
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

}  // namespace

extern "C" int svla_conv2d_nhwc(const svla_conv_args* a, void* stream) {
  SVLA_CHECK_ARG(a && a->x && a->w && a->out, "conv2d_nhwc: NULL args");
  SVLA_CHECK_ARG(a->B > 0 && a->H > 0 && a->W > 0 && a->Cin > 0 && a->Cout > 0 && a->OH > 0 && a->OW > 0,
                 "conv2d_nhwc: bad sizes");
  SVLA_CHECK_ARG(a->Cin % 8 == 0 && a->Cout % 8 == 0, "conv2d_nhwc: Cin (%d) and Cout (%d) must be multiples of 8",
                 a->Cin, a->Cout);
  SVLA_CHECK_ARG(al16(a->x) && al16(a->w) && al16(a->out) && (!a->bias || al16(a->bias)) &&
                     (!a->res1 || al16(a->res1)) && (!a->res2 || al16(a->res2)),
                 "conv2d_nhwc: pointers must be 16-B aligned");
  SVLA_CHECK_ARG((int64_t)a->B * a->H * a->W * a->Cin * 2 < (1ll << 31),
                 "conv2d_nhwc: input over 2 GiB (split the batch)");
  ConvK k;
  k.S = 1;
  k.slabs = nullptr;
  k.counters = nullptr;
  k.x = (const bf16_t*)a->x;
  k.w = (const bf16_t*)a->w;
  k.bias = (const bf16_t*)a->bias;
  k.res1 = (const bf16_t*)a->res1;
  k.res2 = (const bf16_t*)a->res2;
  k.out = (bf16_t*)a->out;
  k.B = a->B; k.H = a->H; k.W = a->W; k.Cin = a->Cin; k.OH = a->OH; k.OW = a->OW; k.Cout = a->Cout;
  k.flags = a->flags;
  k.factor = a->factor;
  if (a->flags & SVLA_CONV_TRANSPOSED) {
    SVLA_CHECK_ARG(a->factor >= 1 && a->OH == a->H * a->factor && a->OW == a->W * a->factor,
                   "conv2d_nhwc: transposed conv needs kernel == stride == factor and OH = H * factor");
    SVLA_CHECK_ARG(!a->res1 && !a->res2, "conv2d_nhwc: residuals are not supported with the transposed form");
    SVLA_CHECK_ARG(!(a->flags & SVLA_CONV_PRE_RELU), "conv2d_nhwc: no pre-activation with the transposed form");
    // GEMM over the input pixels (1x1 window), N = (dy, dx, co); the epilogue scatters each chunk to its pixel
    k.KH = k.KW = 1; k.stride = 1; k.pad = 0;
    k.RH = a->H; k.RW = a->W;
    k.N = a->factor * a->factor * a->Cout;
    k.K = a->Cin;
    k.M = (int64_t)a->B * a->H * a->W;
  } else {
    SVLA_CHECK_ARG(a->KH >= 1 && a->KW >= 1 && a->stride >= 1 && a->pad >= 0, "conv2d_nhwc: bad kernel geometry");
    SVLA_CHECK_ARG(a->OH == (a->H + 2 * a->pad - a->KH) / a->stride + 1 &&
                       a->OW == (a->W + 2 * a->pad - a->KW) / a->stride + 1,
                   "conv2d_nhwc: OH/OW do not match H/W, kernel, stride and padding");
    k.KH = a->KH; k.KW = a->KW; k.stride = a->stride; k.pad = a->pad;
    k.RH = a->OH; k.RW = a->OW;
    k.N = a->Cout;
    k.K = a->KH * a->KW * a->Cin;
    k.M = (int64_t)a->B * a->OH * a->OW;
  }
  hipStream_t s = (hipStream_t)stream;
  const bool pre = (a->flags & SVLA_CONV_PRE_RELU) != 0;
  if (k.N <= 32) return launch_conv<ConvNarrow>(k, pre, s);
  if (k.M >= (int64_t)256 * 256 && k.N >= 128) return launch_conv<ConvBig>(k, pre, s);
  // a grid of 128 x 128 tiles under one wave of CUs (B = 1 prefill: the 12x12 .. 48x48 maps of the DPT neck): 4x the
  // workgroups on 64 x 64 tiles, each k-tile half the bytes (a small block's k-loop is bound by its CU's intake)
  const int64_t t128 = ((k.M + 127) / 128) * ((k.N + 127) / 128);
  if (CONV_SMALL && t128 < svla::num_cus()) {
    // split-K while the 64x64 grid stays under one wave: S = G / tiles, >= 4 k-tiles a split, at most CONV_SPLIT_MAX
    // (the reducer reads S 16 KiB slabs); slabs and counters in the caller's GEMM workspace (its chip-wide layout:
    // counters behind 2 x CUs slabs of 256 KiB)
    const int G = svla::num_cus();
    const int64_t t64 = ((k.M + 63) / 64) * ((k.N + 63) / 64);
    const int64_t nk = (k.K + CBK - 1) / CBK;
    int64_t S = t64 < G ? G / t64 : 1;
    S = std::min<int64_t>(S, std::min<int64_t>(nk / 4, CONV_SPLIT_MAX));
    const size_t slab_region = (size_t)2 * G * 32 * 512 * 16;
    constexpr int64_t SLAB = (int64_t)ConvSmall::TM * ConvSmall::TN * ConvSmall::NTH * 16;
    if (S >= 2 && a->workspace && a->ws_bytes >= slab_region + (size_t)2 * G * sizeof(int) && t64 <= 2 * G &&
        t64 * S * SLAB <= (int64_t)slab_region && (((uintptr_t)a->workspace) & 255) == 0) {
      k.S = (int)S;
      k.slabs = reinterpret_cast<float*>(a->workspace);
      k.counters = reinterpret_cast<int*>(reinterpret_cast<char*>(a->workspace) + slab_region);
    }
    return launch_conv<ConvSmall>(k, pre, s);
  }
  return launch_conv<ConvMid>(k, pre, s);
}
