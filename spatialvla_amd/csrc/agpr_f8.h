// Generated: one specialisation per 32x32 accumulator block Q (AGPRs a[16Q:16Q+15]) of the fp8 4-wave GEMM.
// v_mfma_scale_f32_32x32x64_f8f6f4 with e4m3 operands (cbsz/blgp 0) and unit E8M0 block scales (127 = 2^0):
// the per-row scales of both operands are applied in the epilogue.  Exact clobbers, as agpr_mfma (gemm.hip).
#pragma once
template <int Q>
__device__ __forceinline__ void agpr_mfma_f8(const i32x8& a, const i32x8& b, int s);
template <>
__device__ __forceinline__ void agpr_mfma_f8<0>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[0:15], %0, %1, a[0:15], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<1>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[16:31], %0, %1, a[16:31], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<2>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[32:47], %0, %1, a[32:47], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<3>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[48:63], %0, %1, a[48:63], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<4>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[64:79], %0, %1, a[64:79], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<5>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[80:95], %0, %1, a[80:95], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<6>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[96:111], %0, %1, a[96:111], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<7>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[112:127], %0, %1, a[112:127], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<8>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[128:143], %0, %1, a[128:143], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<9>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[144:159], %0, %1, a[144:159], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<10>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[160:175], %0, %1, a[160:175], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<11>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[176:191], %0, %1, a[176:191], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<12>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[192:207], %0, %1, a[192:207], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<13>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[208:223], %0, %1, a[208:223], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<14>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[224:239], %0, %1, a[224:239], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239");
}
template <>
__device__ __forceinline__ void agpr_mfma_f8<15>(const i32x8& a, const i32x8& b, int s) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[240:255], %0, %1, a[240:255], %2, %2 op_sel_hi:[0,0,0]"
               :: "v"(a), "v"(b), "v"(s) : "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255");
}
