// Shared device/host helpers for the SpatialVLA gfx950 kernels.
// CDNA4 only: 64-lane waves, bf16 MFMA (v_mfma_f32_16x16x32_bf16), ds_read_b64_tr_b16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "../../include/svla.h"
#include "gelu_bf16_table.h"

typedef uint16_t bf16_t;  // raw bf16 bits in global memory
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define LDS_AS __attribute__((address_space(3)))

// ---------------------------------------------------------------- bf16 <-> f32
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  // round-to-nearest-even; NaN stays NaN (hipcc lowers this to v_cvt_pk_bf16_f32 on gfx950)
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (RNE) in ONE v_cvt_pk_bf16_f32 (the scalar form f2bf(a) | f2bf(b) << 16 costs
// two converts plus a shift and an or)
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ void unpack8(const u32x4 v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2(f[2 * i], f[2 * i + 1]);
  return r;
}

// ---------------------------------------------------------------- math
// Branch-free tanh, max relative error ~4e-7 (libm's tanhf branches per argument range and diverges across a
// wave; it dominated the GEMM epilogues, the attention softcap and the lm_head softcap).  |x| < 0.55: odd
// Taylor series to x^15; beyond: 1 - 2/(exp(2|x|)+1) (no cancellation there), sign restored; saturates to +-1.
__device__ __forceinline__ float fast_tanh(float x) {
  const float ax = fabsf(x), x2 = x * x;
  float p = 929569.f / 638512875.f;
  p = p * x2 - 21844.f / 6081075.f;
  p = p * x2 + 1382.f / 155925.f;
  p = p * x2 - 62.f / 2835.f;
  p = p * x2 + 17.f / 315.f;
  p = p * x2 - 2.f / 15.f;
  p = p * x2 + 1.f / 3.f;
  const float small = x - x * x2 * p;
  // v_rcp_f32 (1 ulp) instead of the correctly rounded divide (~10 instructions): tanh's absolute error stays ~1e-7
  const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * ax) + 1.0f);
  return ax < 0.55f ? small : copysignf(big, x);
}
// transformers "gelu_pytorch_tanh" == torch.nn.functional.gelu(approximate="tanh")
// Gemma2 final logit softcap on a bf16 tensor, op by op as the reference (modeling_gemma2.py:994-997):
// logits / cap, tanh, * cap, each rounded to bf16 (fast_tanh's 4e-7 error only matters at a bf16 rounding tie of
// tanh, which the argmax margin gate of the tests covers).  The division is a multiply by RN(1/cap): for every
// finite bf16 input, bf16(x * RN(1/cap)) == bf16(x / cap) at cap 30 and 50 (checked exhaustively over all 65536
// bf16 values, tools/check_softcap_recip.py), and it saves the ~10-instruction correctly rounded divide per logit.
__device__ __forceinline__ float softcap_bf16(float v, float cap, float icap) {
  const float a = round_bf(round_bf(v) * icap);
  return round_bf(round_bf(fast_tanh(a)) * cap);
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.0f + fast_tanh(u));
}
// bf16(gelu_tanh(g)) of a bf16 g (bits b in the low 16 bits, value gf): 2^-9 <= |g| < 8 from the table of
// tools/gen_gelu_table.py (in LDS for the GeGLU GEMM's direct epilogue, in global memory elsewhere), |g| < 2^-9 ->
// g / 2 (exact), g >= 8 -> g, g <= -8 -> -0, -inf / negative NaN -> NaN.  Bitwise the reference's fp32 op sequence
// (gelu_pytorch_tanh on a bf16 tensor: fp32 0.5 g (1 + tanh(k0 (g + k1 g^3))), correctly rounded tanh, cast to
// bf16) on all 65536 bf16 inputs, which the generator checks exhaustively; ~12 VALU and one 2-B load instead of
// gelu_tanh's ~30 VALU and two transcendentals.  Every bf16-input GELU(tanh) of the library goes through it, so the
// forward activation and the one the backward passes recompute are the same bits.
template <typename TabPtr>
__device__ __forceinline__ float gelu_bf16_lut(uint32_t b, float gf, TabPtr tab) {
  const uint32_t a = b & 0x7fffu, s = b >> 15;
  const uint32_t idx = a - (uint32_t)SVLA_GELU_TAB_LO;
  const float tv =
      __uint_as_float((uint32_t)tab[min(idx, (uint32_t)SVLA_GELU_TAB_N - 1u) + s * SVLA_GELU_TAB_N] << 16);
  const float hi = s ? (a < 0x7f80u ? -0.0f : __uint_as_float(0x7fc00000u)) : gf;
  return idx < (uint32_t)SVLA_GELU_TAB_N ? tv : (a < (uint32_t)SVLA_GELU_TAB_LO ? gf * 0.5f : hi);
}
// the same for a float holding a bf16 value, from the global-memory table
__device__ __forceinline__ float gelu_bf16(float g) {
  return gelu_bf16_lut(__float_as_uint(g) >> 16, g, svla_gelu_bf16_tab);
}
// torch GELU(approximate="none") in fp32: x/2 * (1 + erf(x / sqrt(2)))
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f)); }
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = fast_tanh(u);
  return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * k1 * x2);
}

// ---------------------------------------------------------------- wave reductions (64 lanes)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// block (<=1024 threads) sum through LDS; `red` must hold >= 16 floats
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---------------------------------------------------------------- error plumbing
namespace svla {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
int num_cus();
}  // namespace svla

#define SVLA_CHECK_ARG(cond, ...)            \
  do {                                       \
    if (!(cond)) {                           \
      svla::set_error(__VA_ARGS__);          \
      return SVLA_ERR_ARG;                   \
    }                                        \
  } while (0)

// bijective XCD-aware remap of a 1-D block id (MI355X: 8 XCDs, round-robin dispatch).
// Consecutive logical ids land on the same XCD so neighbouring tiles share its L2.
__device__ __forceinline__ int xcd_remap(int pid, int nwg) {
  const int nx = 8;
  int q = nwg / nx, r = nwg % nx;
  int xcd = pid % nx, idx = pid / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// wave-uniform buffer descriptor over [base, base + 2 GiB): loads beyond num_records return zeros (the OOB
// voffset 0x80000000 is how the kernels zero-fill ragged tile edges).  readfirstlane makes the base provably
// uniform, else hipcc wraps every buffer op in a waterfall loop (cdna_hip_programming.md T20).
constexpr uint32_t SVLA_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* pb = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0, (int)SVLA_OOB, 0x00020000);
}

// ---- e4m3 / OCP MX helpers (fp8.hip's quantisers and the producers that emit MX operands: misc.hip geglu_bwd)
// four fp32 -> four e4m3 bytes (RNE), packed in one dword
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}
// E8M0 exponent of an MX block: X = ceil(log2(amax / 448)) (the smallest power of two that maps the block maximum
// into e4m3's range), clamped to [-127, 127]; zero or subnormal amax -> -127 (fp8.hip quant_mx_rows documents it)
__device__ __forceinline__ int mx_exponent(float amax) {
  const uint32_t u = __float_as_uint(amax);
  const int e = (int)((u >> 23) & 0xff);            // floor(log2(amax)) + 127 for normal amax; 0: zero / subnormal
  const int up = (u & 0x7fffffu) > 0x600000u;       // amax * 2^-(floor(log2 amax) - 8) > 448: one more power of two
  return max(-127, min(127, e - 127 - 8 + up));     // subnormal or zero amax: clamps to -127 (byte 0)
}
// MX quantisation of 8 consecutive elements a lane (OCP MX: 4 lanes = one 32-element block, 16 lanes = one 128-element
// k-tile; lane groups aligned to both): block amax by two xor shuffles, e4m3(x * 2^-X) (RNE, clamped to +-448) to q8
// (8 bytes), and the 4 E8M0 bytes of the 16-lane group gathered into the dword the group's first lane stores at sc4.
// A NaN / +-Inf element makes its block NaN (scale 0xFF and e4m3 NaN elements).  Every lane of the 16-lane group must
// call it (the shuffles); `ok` false: the lane stores nothing (its f must then be finite, e.g. zeros).
__device__ __forceinline__ void mx_store8(float* f, bool ok, uint8_t* q8, uint8_t* sc4) {
  const int lane = threadIdx.x & 63;
  float amax = 0.f;
  int nonfinite = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    amax = fmaxf(amax, fabsf(f[j]));
    nonfinite |= (__float_as_uint(f[j]) & 0x7f800000u) == 0x7f800000u;
  }
  amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
  nonfinite |= __shfl_xor(nonfinite, 1, 64);
  nonfinite |= __shfl_xor(nonfinite, 2, 64);
  const int X = mx_exponent(amax);
  const float inv = __uint_as_float((uint32_t)(127 - X) << 23);  // 2^-X exactly (X >= -127 -> exponent <= 254)
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(f[j] * inv, -448.f), 448.f);
  u32x2 qv = u32x2{cvt4(f[0], f[1], f[2], f[3]), cvt4(f[4], f[5], f[6], f[7])};
  if (nonfinite) qv = u32x2{0x7f7f7f7fu, 0x7f7f7f7fu};
  if (ok) *reinterpret_cast<u32x2*>(q8) = qv;
  const uint32_t byte = nonfinite ? 0xffu : (uint32_t)(127 + X);
  uint32_t w = byte;
  w |= (uint32_t)__shfl_down((int)byte, 4, 16) << 8;
  w |= (uint32_t)__shfl_down((int)byte, 8, 16) << 16;
  w |= (uint32_t)__shfl_down((int)byte, 12, 16) << 24;
  if (ok && (lane & 15) == 0) *reinterpret_cast<uint32_t*>(sc4) = w;
}
