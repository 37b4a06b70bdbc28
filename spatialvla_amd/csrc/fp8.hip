// Row-wise OCP e4m3 quantisation for the fp8 projections (BASELINE configs[4]; the bf16 nn.Linear inputs and weights
// of model/modeling_gemma2.py:86-92, 351-354 feed svla_gemm_fp8 in this form).
//   scale[r] = amax_r / 448,  q[r, k] = e4m3(clamp(x[r, k] * (448 / amax_r), -448, 448))   (RNE; amax_r = 0 -> q = 0)
// One wave per row; the row stays in registers between the max and the convert pass (K <= 64 * 8 * NCH), so HBM
// sees one bf16 read and one fp8 write per element.
#include "svla_common.h"

#include <cstdlib>

namespace {


template <int NCH>
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                             int64_t ldx, const float* __restrict__ colscale,
                                                             uint8_t* __restrict__ q, int64_t ldq,
                                                             float* __restrict__ scale) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + row * ldx;
  uint8_t* qr = q + row * ldq;
  u32x4 v[NCH];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int64_t k = (int64_t)(c * 64 + lane) * 8;
    v[c] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xr + k)) : u32x4{0, 0, 0, 0};
    float f[8];
    unpack8(v[c], f);
    if (colscale && k < K) {
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(colscale + k), s1 = *reinterpret_cast<const f32x4*>(colscale + k + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) { f[j] *= s0[j]; f[4 + j] *= s1[j]; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? __fdiv_rn(448.f, amax) : 0.f;  // correctly rounded (the torch reference's division)
  if (lane == 0) scale[row] = __fdiv_rn(amax, 448.f);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int64_t k = (int64_t)(c * 64 + lane) * 8;
    if (k < K) {
      float f[8];
      unpack8(v[c], f);
      if (colscale) {
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(colscale + k), s1 = *reinterpret_cast<const f32x4*>(colscale + k + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { f[j] *= s0[j]; f[4 + j] *= s1[j]; }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -448.f), 448.f);
      const u32x2 o = {cvt4(f[0], f[1], f[2], f[3]), cvt4(f[4], f[5], f[6], f[7])};
      *reinterpret_cast<u32x2*>(qr + k) = o;
    }
  }
}

// Long rows (K > 64 * 8 * 8): two streaming passes over the row instead of holding it in registers (36 chunks a
// lane spilled: 730 us at [9984, 18432]); the second pass re-reads the row, mostly from L2.
__device__ __forceinline__ void load_scaled8(const bf16_t* xr, const float* colscale, int64_t k, float* f) {
  unpack8(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(xr + k)), f);
  if (colscale) {
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(colscale + k), s1 = *reinterpret_cast<const f32x4*>(colscale + k + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) { f[j] *= s0[j]; f[4 + j] *= s1[j]; }
  }
}

__global__ __launch_bounds__(256) void quant_fp8_rows_stream_kernel(int64_t rows, int64_t K,
                                                                    const bf16_t* __restrict__ x, int64_t ldx,
                                                                    const float* __restrict__ colscale,
                                                                    uint8_t* __restrict__ q, int64_t ldq,
                                                                    float* __restrict__ scale) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const bf16_t* xr = x + row * ldx;
  uint8_t* qr = q + row * ldq;
  float amax = 0.f;
#pragma unroll 4
  for (int64_t k = (int64_t)lane * 8; k < K; k += 512) {
    float f[8];
    load_scaled8(xr, colscale, k, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(f[j]));
  }
  amax = wave_max(amax);
  const float inv = amax > 0.f ? __fdiv_rn(448.f, amax) : 0.f;
  if (lane == 0) scale[row] = __fdiv_rn(amax, 448.f);
#pragma unroll 4
  for (int64_t k = (int64_t)lane * 8; k < K; k += 512) {
    float f[8];
    load_scaled8(xr, colscale, k, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -448.f), 448.f);
    const u32x2 o = {cvt4(f[0], f[1], f[2], f[3]), cvt4(f[4], f[5], f[6], f[7])};
    *reinterpret_cast<u32x2*>(qr + k) = o;
  }
}

// Byte transpose out[c][r] = in[r][c] through a 64x64 LDS tile (fp8 weight copies for the dgrad GEMMs): 16-B
// row-chunk loads, 4-B column-chunk stores; the tile's LDS rows are padded by 4 B against bank conflicts.
__global__ __launch_bounds__(256) void transpose_u8_kernel(int64_t R, int64_t C, const uint8_t* __restrict__ in,
                                                           int64_t ldi, uint8_t* __restrict__ out, int64_t ldo) {
  __shared__ uint8_t tile[64][68];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int t = threadIdx.x;
  {  // 64 rows x 4 chunks of 16 B
    const int r = t >> 2, ch = t & 3;
    const int64_t gr = r0 + r, gc = c0 + 16 * ch;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (gr < R && gc + 16 <= C) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(in + gr * ldi + gc);
      w[0] = v[0]; w[1] = v[1]; w[2] = v[2]; w[3] = v[3];
    } else if (gr < R) {
      for (int j = 0; j < 16; ++j)
        if (gc + j < C) w[j >> 2] |= (uint32_t)in[gr * ldi + gc + j] << (8 * (j & 3));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<uint32_t*>(&tile[r][16 * ch + 4 * j]) = w[j];
  }
  __syncthreads();
  {  // 64 output rows (input columns) x 16 chunks of 4 B (input rows)
    const int c = t >> 2;
#pragma unroll
    for (int part = 0; part < 4; ++part) {
      const int rq = (t & 3) * 4 + part;  // 4-row group 0..15
      const int64_t oc = c0 + c, orr = r0 + 4 * rq;
      if (oc < C) {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) w |= (uint32_t)tile[4 * rq + j][c] << (8 * j);
        if (orr + 4 <= R) *reinterpret_cast<uint32_t*>(out + oc * ldo + orr) = w;
        else
          for (int j = 0; j < 4; ++j)
            if (orr + j < R) out[oc * ldo + orr + j] = (uint8_t)(w >> (8 * j));
      }
    }
  }
}

// OCP MX quantisation of rows (e4m3 elements, one E8M0 scale per 32 consecutive k; OCP Microscaling Formats spec
// v1.0 §5.3): for block b of row r, X = ceil(log2(amax / 448)), clamped to E8M0's [-127, 127] -- the smallest power
// of two that maps the block maximum into e4m3's range, so nothing saturates (the spec's reference conversion
// §6.3 takes X = floor(log2(amax)) - 8 and clips block maxima in (448, 512): a 12.5 % error on ~19 % of the block
// maxima, measured as 4.1e-2 vs 3.75e-2 GEMM error on Gaussian operands); q = e4m3(x * 2^-X) (RNE); scale byte
// 127 + X.  Scales are stored tile-major, sc[(k / 128) * sld + r * 4 + (k % 128) / 32]:
// one 128-k tile's scales of 256 consecutive rows are 1 KiB contiguous (one LDS-DMA piece per operand and k-tile in
// the MX GEMM).  Lane layout: 8 elements a lane (one 16-B load), 4 lanes a block (amax by two xor shuffles), 16
// lanes a k-tile (the 4 scale bytes gathered into one dword store), a wave 512 k of one row.

// one (row, 512-k chunk) item of quant_mx_rows: the wave's 8 elements a lane already loaded into v
__device__ __forceinline__ void mx_item(const u32x4 v, bool ok, int64_t r, int64_t k, uint8_t* __restrict__ q,
                                        int64_t ldq, uint8_t* __restrict__ sc, int64_t sld) {
  float f[8];
  if (ok) unpack8(v, f);
  else
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
  mx_store8(f, ok, q + r * ldq + k, sc + (k / 128) * sld + r * 4);
}

// U consecutive items a wave, every item's 16-B load issued before the first is converted (one item a wave left a
// single 1 KiB load in flight per wave and ran at ~1.2 TB/s in the fp8 training step, profiles/r8b)
template <int U>
__global__ __launch_bounds__(256) void quant_mx_rows_kernel(int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                            int64_t ldx, uint8_t* __restrict__ q, int64_t ldq,
                                                            uint8_t* __restrict__ sc, int64_t sld) {
  const int lane = threadIdx.x & 63;
  const int64_t chunks = (K + 511) / 512;
  const int64_t items = rows * chunks;
  const int64_t base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * U;  // (row, 512-k chunk) items
  if (base >= items) return;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t it = base + u < items ? base + u : items - 1;
    const int64_t r = it / chunks, k = (it % chunks) * 512 + 8 * lane;
    v[u] = k < K ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(x + r * ldx + k)) : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t it = base + u;
    if (it >= items) break;
    const int64_t r = it / chunks, k = (it % chunks) * 512 + 8 * lane;
    mx_item(v[u], k < K, r, k, q, ldq, sc, sld);  // K % 128 == 0: whole 16-lane k-tiles are in or out together
  }
}

// MX quantisation of the columns of W [N][K] into the rows of W^T: q[k][n] = e4m3 of W[n][k] with one E8M0 scale per
// 32 consecutive n of column k, the layout quant_mx_rows gives for W^T (rows = K, reduction dim = N), bit for bit --
// without materialising the bf16 W^T.  A 256-thread block owns a 128 (n) x 64 (k) tile: each lane loads 16-B row
// pieces (8 consecutive k of one n), writes them transposed into LDS, then thread (k, b) reads the 32 n of block b of
// column k as four 16-B LDS reads, forms the block's scale in registers and stores 32 e4m3 bytes; the 4 scale bytes of
// a 128-n tile (threads b = 0..3 of one k) leave as one dword.
constexpr int QC_N = 128, QC_K = 64, QC_P = QC_N + 8;  // LDS row pitch (bf16): 16-B aligned rows
__global__ __launch_bounds__(256) void quant_mx_cols_kernel(int64_t N, int64_t K, const bf16_t* __restrict__ w,
                                                            int64_t ldw, uint8_t* __restrict__ q, int64_t ldq,
                                                            uint8_t* __restrict__ sc, int64_t sld) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[QC_K][QC_P];
  const int t = threadIdx.x;
  const int64_t n0 = (int64_t)blockIdx.x * QC_N, k0 = (int64_t)blockIdx.y * QC_K;
  u32x4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nl = (t >> 3) + 32 * i, kc = (t & 7) * 8;
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w + (n0 + nl) * ldw + k0 + kc));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nl = (t >> 3) + 32 * i, kc = (t & 7) * 8;
    const uint32_t e[4] = {v[i][0], v[i][1], v[i][2], v[i][3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[kc + 2 * j][nl] = (bf16_t)(e[j] & 0xffffu);
      tile[kc + 2 * j + 1][nl] = (bf16_t)(e[j] >> 16);
    }
  }
  __syncthreads();
  const int kl = t >> 2, b = t & 3;
  float f[32];
#pragma unroll
  for (int c = 0; c < 4; ++c) unpack8(*reinterpret_cast<const u32x4*>(&tile[kl][32 * b + 8 * c]), f + 8 * c);
  float amax = 0.f;
  int nonfinite = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    amax = fmaxf(amax, fabsf(f[j]));
    nonfinite |= (__float_as_uint(f[j]) & 0x7f800000u) == 0x7f800000u;
  }
  const int X = mx_exponent(amax);
  const float inv = __uint_as_float((uint32_t)(127 - X) << 23);
  u32x4 o[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t wd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float g[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = fminf(fmaxf(f[16 * h + 4 * j + e] * inv, -448.f), 448.f);
      wd[j] = nonfinite ? 0x7f7f7f7fu : cvt4(g[0], g[1], g[2], g[3]);
    }
    o[h] = u32x4{wd[0], wd[1], wd[2], wd[3]};
  }
  uint8_t* qr = q + (k0 + kl) * ldq + n0 + 32 * b;
  *reinterpret_cast<u32x4*>(qr) = o[0];
  *reinterpret_cast<u32x4*>(qr + 16) = o[1];
  const uint32_t byte = nonfinite ? 0xffu : (uint32_t)(127 + X);
  uint32_t wsc = byte;
  wsc |= (uint32_t)__shfl_down((int)byte, 1, 4) << 8;
  wsc |= (uint32_t)__shfl_down((int)byte, 2, 4) << 16;
  wsc |= (uint32_t)__shfl_down((int)byte, 3, 4) << 24;
  if (b == 0) *reinterpret_cast<uint32_t*>(sc + (n0 / 128) * sld + (k0 + kl) * 4) = wsc;
}

// Both MX layouts of one bf16 matrix W [R][C] from a single read (the fp8 weight copies: the forward operand W with
// blocks along C and the dgrad operand W^T with blocks along R; bitwise quant_mx_rows(W) and quant_mx_rows(W^T)).
// A 256-thread block owns a 128 x 128 tile: lane t loads 8 row pieces (row (t >> 4) + 16 i, columns (t & 15) * 8 ..
// + 8), quantises them in place for the row layout (16 lanes = one row's 128-column k-tile, mx_store8), and writes
// them transposed into LDS; then each thread quantises two 32-row blocks of a column for the W^T layout.
constexpr int QB_T = 128, QB_P = QB_T + 8;
__global__ __launch_bounds__(256) void quant_mx_both_kernel(int64_t R, int64_t C, const bf16_t* __restrict__ w,
                                                            int64_t ldw, uint8_t* __restrict__ qr, int64_t ldqr,
                                                            uint8_t* __restrict__ scr, int64_t sldr,
                                                            uint8_t* __restrict__ qc, int64_t ldqc,
                                                            uint8_t* __restrict__ scc, int64_t sldc) {
  __shared__ __attribute__((aligned(16))) bf16_t tile[QB_T][QB_P];
  const int t = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * QB_T, c0 = (int64_t)blockIdx.y * QB_T;
  const int kc = (t & 15) * 8;
  u32x4 v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w + (r0 + (t >> 4) + 16 * i) * ldw + c0 + kc));
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int rl = (t >> 4) + 16 * i;
    const uint32_t e[4] = {v[i][0], v[i][1], v[i][2], v[i][3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[kc + 2 * j][rl] = (bf16_t)(e[j] & 0xffffu);
      tile[kc + 2 * j + 1][rl] = (bf16_t)(e[j] >> 16);
    }
    float f[8];
    unpack8(v[i], f);
    mx_store8(f, true, qr + (r0 + rl) * ldqr + c0 + kc, scr + ((c0 + kc) / 128) * sldr + (r0 + rl) * 4);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int cl = (t >> 2) + 64 * p, b = t & 3;
    float f[32];
#pragma unroll
    for (int c = 0; c < 4; ++c) unpack8(*reinterpret_cast<const u32x4*>(&tile[cl][32 * b + 8 * c]), f + 8 * c);
    float amax = 0.f;
    int nonfinite = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      amax = fmaxf(amax, fabsf(f[j]));
      nonfinite |= (__float_as_uint(f[j]) & 0x7f800000u) == 0x7f800000u;
    }
    const int X = mx_exponent(amax);
    const float inv = __uint_as_float((uint32_t)(127 - X) << 23);
    u32x4 o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t wd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float g[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = fminf(fmaxf(f[16 * h + 4 * j + e] * inv, -448.f), 448.f);
        wd[j] = nonfinite ? 0x7f7f7f7fu : cvt4(g[0], g[1], g[2], g[3]);
      }
      o[h] = u32x4{wd[0], wd[1], wd[2], wd[3]};
    }
    uint8_t* q = qc + (c0 + cl) * ldqc + r0 + 32 * b;
    *reinterpret_cast<u32x4*>(q) = o[0];
    *reinterpret_cast<u32x4*>(q + 16) = o[1];
    const uint32_t byte = nonfinite ? 0xffu : (uint32_t)(127 + X);
    uint32_t wsc = byte;
    wsc |= (uint32_t)__shfl_down((int)byte, 1, 4) << 8;
    wsc |= (uint32_t)__shfl_down((int)byte, 2, 4) << 16;
    wsc |= (uint32_t)__shfl_down((int)byte, 3, 4) << 24;
    if (b == 0) *reinterpret_cast<uint32_t*>(scc + (r0 / 128) * sldc + (c0 + cl) * 4) = wsc;
  }
}

}  // namespace

extern "C" int svla_quant_mx_rows(int64_t rows, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                                  void* scales, int64_t sld, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && K > 0 && K % 128 == 0, "quant_mx_rows: K=%lld (a positive multiple of 128)",
                 (long long)K);
  SVLA_CHECK_ARG(x && q && scales && ldx >= K && ldq >= K && ldx % 8 == 0 && ldq % 8 == 0 &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0 && ((uintptr_t)scales & 3) == 0,
                 "quant_mx_rows: pointers / leading dimensions");
  SVLA_CHECK_ARG(sld >= 4 * rows && sld % 4 == 0, "quant_mx_rows: scale tile stride %lld < 4 * rows", (long long)sld);
  const int64_t items = rows * ((K + 511) / 512);
  static int U = -1;  // SVLA_QUANT_MX_ITEMS: items a wave (1, 2, 4 or 8; default 4)
  if (U < 0) {
    const char* e = getenv("SVLA_QUANT_MX_ITEMS");
    U = e ? atoi(e) : 4;
    if (U != 1 && U != 2 && U != 8) U = 4;
  }
  const dim3 grid((unsigned)((items + 4 * U - 1) / (4 * U)));
  hipStream_t s = (hipStream_t)stream;
#define SVLA_QMX(UU)                                                                                              \
  hipLaunchKernelGGL(quant_mx_rows_kernel<UU>, grid, dim3(256), 0, s, rows, K, (const bf16_t*)x, ldx, (uint8_t*)q, \
                     ldq, (uint8_t*)scales, sld)
  if (U == 1) SVLA_QMX(1);
  else if (U == 2) SVLA_QMX(2);
  else if (U == 8) SVLA_QMX(8);
  else SVLA_QMX(4);
#undef SVLA_QMX
  return svla::check_launch("quant_mx_rows");
}

extern "C" int svla_quant_mx_cols(int64_t N, int64_t K, const void* w, int64_t ldw, void* q, int64_t ldq, void* scales,
                                  int64_t sld, void* stream) {
  SVLA_CHECK_ARG(N > 0 && K > 0 && N % QC_N == 0 && K % QC_K == 0,
                 "quant_mx_cols: N=%lld (a multiple of 128), K=%lld (a multiple of 64)", (long long)N, (long long)K);
  SVLA_CHECK_ARG(w && q && scales && ldw >= K && ldq >= N && ldw % 8 == 0 && ldq % 16 == 0 &&
                     ((uintptr_t)w & 15) == 0 && ((uintptr_t)q & 15) == 0 && ((uintptr_t)scales & 3) == 0,
                 "quant_mx_cols: pointers / leading dimensions");
  SVLA_CHECK_ARG(sld >= 4 * K && sld % 4 == 0, "quant_mx_cols: scale tile stride %lld < 4 * K", (long long)sld);
  hipLaunchKernelGGL(quant_mx_cols_kernel, dim3((unsigned)(N / QC_N), (unsigned)(K / QC_K)), dim3(256), 0,
                     (hipStream_t)stream, N, K, (const bf16_t*)w, ldw, (uint8_t*)q, ldq, (uint8_t*)scales, sld);
  return svla::check_launch("quant_mx_cols");
}

extern "C" int svla_transpose_u8(int64_t R, int64_t C, const void* in, int64_t ldi, void* out, int64_t ldo,
                                 void* stream) {
  SVLA_CHECK_ARG(R > 0 && C > 0 && in && out && ldi >= C && ldo >= R && ldi % 16 == 0 && ldo % 4 == 0 &&
                     ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 3) == 0,
                 "transpose_u8: sizes / pointers (ldi % 16, ldo % 4, 16-B aligned input)");
  const dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64)), block(256);
  hipLaunchKernelGGL(transpose_u8_kernel, grid, block, 0, (hipStream_t)stream, R, C, (const uint8_t*)in, ldi,
                     (uint8_t*)out, ldo);
  return svla::check_launch("transpose_u8");
}

extern "C" int svla_quant_fp8_rows(int64_t rows, int64_t K, const void* x, int64_t ldx, const float* colscale,
                                   void* q, int64_t ldq, float* scale, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && K > 0 && K % 8 == 0, "quant_fp8_rows: K=%lld (a positive multiple of 8)",
                 (long long)K);
  SVLA_CHECK_ARG(x && q && scale && ldx >= K && ldq >= K && ldx % 8 == 0 && ldq % 8 == 0 &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0,
                 "quant_fp8_rows: pointers / leading dimensions");
  SVLA_CHECK_ARG(!colscale || ((uintptr_t)colscale & 15) == 0, "quant_fp8_rows: colscale must be 16-B aligned");
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (K <= 64 * 8 * 5)
    hipLaunchKernelGGL(quant_fp8_rows_kernel<5>, grid, block, 0, s, rows, K, (const bf16_t*)x, ldx, colscale,
                       (uint8_t*)q, ldq, scale);
  else if (K <= 64 * 8 * 8)
    hipLaunchKernelGGL(quant_fp8_rows_kernel<8>, grid, block, 0, s, rows, K, (const bf16_t*)x, ldx, colscale,
                       (uint8_t*)q, ldq, scale);
  else
    hipLaunchKernelGGL(quant_fp8_rows_stream_kernel, grid, block, 0, s, rows, K, (const bf16_t*)x, ldx, colscale,
                       (uint8_t*)q, ldq, scale);
  return svla::check_launch("quant_fp8_rows");
}

extern "C" int svla_quant_mx_both(int64_t R, int64_t C, const void* w, int64_t ldw, void* q_rows, int64_t ldq_rows,
                                  void* sc_rows, int64_t sld_rows, void* q_cols, int64_t ldq_cols, void* sc_cols,
                                  int64_t sld_cols, void* stream) {
  SVLA_CHECK_ARG(R > 0 && C > 0 && R % QB_T == 0 && C % QB_T == 0, "quant_mx_both: R=%lld, C=%lld (multiples of 128)",
                 (long long)R, (long long)C);
  SVLA_CHECK_ARG(w && q_rows && sc_rows && q_cols && sc_cols && ldw >= C && ldw % 8 == 0 && ((uintptr_t)w & 15) == 0,
                 "quant_mx_both: W pointer / leading dimension");
  SVLA_CHECK_ARG(ldq_rows >= C && ldq_rows % 8 == 0 && ((uintptr_t)q_rows & 7) == 0 && sld_rows >= 4 * R &&
                     sld_rows % 4 == 0 && ((uintptr_t)sc_rows & 3) == 0,
                 "quant_mx_both: row-layout output");
  SVLA_CHECK_ARG(ldq_cols >= R && ldq_cols % 16 == 0 && ((uintptr_t)q_cols & 15) == 0 && sld_cols >= 4 * C &&
                     sld_cols % 4 == 0 && ((uintptr_t)sc_cols & 3) == 0,
                 "quant_mx_both: column-layout output");
  hipLaunchKernelGGL(quant_mx_both_kernel, dim3((unsigned)(R / QB_T), (unsigned)(C / QB_T)), dim3(256), 0,
                     (hipStream_t)stream, R, C, (const bf16_t*)w, ldw, (uint8_t*)q_rows, ldq_rows, (uint8_t*)sc_rows,
                     sld_rows, (uint8_t*)q_cols, ldq_cols, (uint8_t*)sc_cols, sld_cols);
  return svla::check_launch("quant_mx_both");
}
