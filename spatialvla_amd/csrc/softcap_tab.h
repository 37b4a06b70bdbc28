// Gemma2 logit softcap with tanh from the bf16 table: shared by the GEMM epilogues (gemm.hip) and the
// standalone lm_head softcap pass (softcap.hip).
#pragma once
#include "svla_common.h"
#include "tanh_bf16_table.h"

namespace {

// Gemma2 final logit softcap (softcap_bf16 of svla_common.h) with tanh taken from a table: a = bf16(bf16(v) / cap) is
// a bf16 value, and bf16(tanh(a)) is a for |a| < 2^-8, 1 for |a| >= 4, and a 1280-entry table in between
// (tools/gen_tanh_table.py; a correctly rounded fp32 tanh cast to bf16, as the reference's bf16 tanh).  Replaces
// the branch-free polynomial/exp tanh (~17 VALU ops and two transcendentals) of the lm_head epilogue.
template <typename Tab, bool V_IS_BF16 = false>
__device__ __forceinline__ float softcap_bf16_tab(float v, float cap, float icap, Tab tab) {
  const float a = round_bf((V_IS_BF16 ? v : round_bf(v)) * icap);  // V_IS_BF16: v already a bf16 value
  const uint32_t u = __float_as_uint(a);
  const uint32_t ab = (u >> 16) & 0x7fffu;
  const uint32_t lo = (uint32_t)SVLA_TANH_TAB_E0 << 7, hi = (uint32_t)SVLA_TANH_TAB_E1 << 7;
  const uint32_t idx = ab < lo ? 0u : (ab >= hi ? 0u : ab - lo);
  const uint32_t tb = tab[idx];
  uint32_t rb = ab < lo ? ab : (ab >= hi ? 0x3f80u : tb);
  if (ab > 0x7f80u) rb = ab;  // NaN stays NaN
  const float t = __uint_as_float((((u >> 16) & 0x8000u) | rb) << 16);
  return round_bf(t * cap);
}
constexpr int TANH_TAB_BYTES = sizeof(svla_tanh_bf16_tab);
static_assert(TANH_TAB_BYTES % 16 == 0, "table copied in 16-B pieces");

}  // namespace
