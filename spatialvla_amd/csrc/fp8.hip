// Row-wise OCP e4m3 quantisation for the fp8 projections (BASELINE configs[4]; the bf16 nn.Linear inputs and weights
// of model/modeling_gemma2.py:86-92, 351-354 feed svla_gemm_fp8 in this form).
//   scale[r] = amax_r / 448,  q[r, k] = e4m3(clamp(x[r, k] * (448 / amax_r), -448, 448))   (RNE; amax_r = 0 -> q = 0)
// One wave per row; the row stays in registers between the max and the convert pass (K <= 64 * 8 * NCH), so HBM
// sees one bf16 read and one fp8 write per element.
#include "svla_common.h"

namespace {

__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

template <int NCH>
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(int64_t rows, int64_t K, const bf16_t* __restrict__ x,
                                                             int64_t ldx, uint8_t* __restrict__ q, int64_t ldq,
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
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -448.f), 448.f);
      const u32x2 o = {cvt4(f[0], f[1], f[2], f[3]), cvt4(f[4], f[5], f[6], f[7])};
      *reinterpret_cast<u32x2*>(qr + k) = o;
    }
  }
}

}  // namespace

extern "C" int svla_quant_fp8_rows(int64_t rows, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                                   float* scale, void* stream) {
  SVLA_CHECK_ARG(rows > 0 && K > 0 && K % 8 == 0 && K <= 64 * 8 * 18, "quant_fp8_rows: K=%lld (multiple of 8, <= 9216)",
                 (long long)K);
  SVLA_CHECK_ARG(x && q && scale && ldx >= K && ldq >= K && ldx % 8 == 0 && ldq % 8 == 0 &&
                     ((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 7) == 0,
                 "quant_fp8_rows: pointers / leading dimensions");
  const dim3 grid((unsigned)((rows + 3) / 4)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (K <= 64 * 8 * 5)
    hipLaunchKernelGGL(quant_fp8_rows_kernel<5>, grid, block, 0, s, rows, K, (const bf16_t*)x, ldx, (uint8_t*)q, ldq,
                       scale);
  else
    hipLaunchKernelGGL(quant_fp8_rows_kernel<18>, grid, block, 0, s, rows, K, (const bf16_t*)x, ldx, (uint8_t*)q, ldq,
                       scale);
  return svla::check_launch("quant_fp8_rows");
}
