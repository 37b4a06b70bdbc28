// Persistent decode-step Gemma2 MLP (svla_decode_mlp): the gate|up GEMV with the post-attention + pre-feedforward
// norm pair in its prologue and the down GEMV in ONE launch, the weights of both streamed without a kernel
// boundary (reference: Gemma2MLP.forward and the decoder layer's sandwich norms, modeling_gemma2.py:91-92,
// :487-490).  Bitwise the two-launch path (svla_gemv_rmsnorm2 with the GEGLU epilogue, then the long-K split GEMV
// of the down projection):
//  * phase A (gemv_norm2_kernel's arithmetic): every block forms h = bf16(res + rms(y; w1)) and x = rms(h; w2) in
//    LDS (block 0 stores h); each wave then walks gate|up row pairs r = wave, wave + waves, ... with the next
//    DM_DEPTH - 1 pairs' weights in flight while a pair's dot products run, and stores act[m][r] =
//    bf16(gelu(g) * u);
//  * a grid barrier: act is stored write-through, each wave drains its stores, thread 0 of each block arrives on a
//    counter and waits for the last arrival's generation bump, then one acquire fence per block;
//  * phase C (gemv_splitk_kernel's arithmetic): each block walks down-projection rows n = block, block + blocks, ...
//    (four waves split the row's K range, partial dots summed through LDS in wave order), next row prefetched.
// The grid is DM_BPC blocks per CU, sized so every block is resident; the barrier wait is bounded (a missed
// barrier would give wrong numbers, never a hung GPU) and the sync words return to {0, generation} after every
// launch, so a zeroed buffer serves every later call and graph replay.
#include "svla_common.h"

#include <algorithm>

namespace {

#ifndef DM_BPC
#define DM_BPC 2  // blocks per CU (all resident: registers and LDS allow it), i.e. the loads in flight per CU
#endif
constexpr int DM_MAXM = 8;
constexpr int DM_KCH = 5;   // 16-B chunks per lane of a gate / up row: H <= 2560
constexpr int DM_NC = 2;    // norm chunks per thread: H <= 4096
constexpr int DM_DCH = 5;   // 16-B chunks per thread of a down row: I <= 10240
constexpr int DM_OCH = 4;
#ifndef DM_DPRE
// down rows a block loads before the grid barrier at batch 1; 1 = only the first.  Loading all of a block's rows (5)
// measured slower, 1.90 vs 1.85 ms per token, and 2 or 3 the same as 1 (profiles/r8j_decode_mlp_down_prefetch_ab.txt):
// phase C is not where the launch waits
#define DM_DPRE 1
#endif
#ifndef DM_DEPTH
#define DM_DEPTH 2  // gate|up row pairs a wave has in flight in phase A (2 or 3; 3 measured slower, r7g)
#endif   // 16-B chunks per lane of an o-projection row: KO <= 2048

// act is stored write-through (agent-scope relaxed atomic stores, sc1), so a wave only drains its own stores before
// the block arrives; the arrival and the generation are relaxed agent-scope atomics, and one agent-scope acquire
// fence per block after the wait (an L1 / L2 invalidate, not one per thread) keeps phase C from reading a stale act.
// Two-level arrival: blocks count on one of DM_GROUPS group counters (separate 256-B lines, so the same-address
// atomics of a group serialise only among that group's blocks), the last arriver of a group counts on the top
// counter, and the last of those bumps the generation word sync[0]; every counter is back at zero after the launch.
#ifndef DM_GROUPS
#define DM_GROUPS 8
#endif
constexpr int DM_SET = 64 * (DM_GROUPS + 1);   // one barrier's counters (groups + top), 256-B apart
constexpr int DM_SYNC_WORDS = 64 + 2 * DM_SET;  // generation word, then the counter sets of barriers 0 and 1
// PEND: vector-memory ops issued after the stores this barrier publishes (they retire in issue order); SET: which
// counter set (a launch with two barriers never reuses a set, so a reset can not race a fast block's next arrival)
template <int PEND, int SET>
__device__ __forceinline__ bool grid_barrier(unsigned* sync, unsigned nblocks, int* flag, long long spin_ticks) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PEND) : "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = blockIdx.x % DM_GROUPS;
    const unsigned gsize = nblocks / DM_GROUPS + (g < nblocks % DM_GROUPS ? 1u : 0u);
    const unsigned ngroups = nblocks < DM_GROUPS ? nblocks : DM_GROUPS;
    unsigned* const gcnt = sync + 64 + SET * DM_SET + 64 * g;
    unsigned* const top = sync + 64 + SET * DM_SET + 64 * DM_GROUPS;
    const unsigned gen = __hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the generation must be read before this block's arrival is counted: the two requests target different lines
    // and could otherwise be serviced out of order, a late read then seeing the bump this arrival completes
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool last = false, timed_out = false;
    if (__hip_atomic_fetch_add(gcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(gcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1) {
        __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&sync[0], gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        last = true;
      }
    }
    if (!last) {
      // bounded by the constant-rate wall clock (1 s by default): a block that never sees the release (its grid was
      // not co-resident) counts a timeout in sync[32] and poisons what it writes next with NaN (the caller raises on
      // the counter); it never hangs the GPU
      const long long t0 = wall_clock64();
      while (__hip_atomic_load(&sync[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (wall_clock64() - t0 > spin_ticks) {
          __hip_atomic_fetch_add(&sync[32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // agent scope (the default for this builtin on the device)
    *flag = timed_out ? 1 : 0;
  }
  __syncthreads();
  return *flag != 0;
}

template <int MR>
__global__ __launch_bounds__(256, DM_BPC) void decode_mlp_kernel(int M, int H, int I, const bf16_t* __restrict__ res,
                                                            bf16_t* y, int64_t ldx,
                                                            const bf16_t* __restrict__ w1,
                                                            const bf16_t* __restrict__ w2, float eps1, float eps2,
                                                            bf16_t* __restrict__ h_out, const bf16_t* __restrict__ wg,
                                                            const bf16_t* __restrict__ wu, int64_t ldw,
                                                            const bf16_t* __restrict__ wd, int64_t ldd,
                                                            bf16_t* act, int64_t ldact, bf16_t* __restrict__ out,
                                                            int64_t ldo, const bf16_t* __restrict__ attn,
                                                            int64_t ld_attn, int KO, const bf16_t* __restrict__ wo,
                                                            int64_t ldwo, unsigned* sync, long long spin_ticks) {
  constexpr int DEPTH = MR == 1 ? DM_DEPTH : 2;  // the 8-row instance keeps two (registers)
  extern __shared__ __attribute__((aligned(16))) char dm_smem[];  // [M][H] bf16 x, reduction slots, down partials
  bf16_t* const xs = reinterpret_cast<bf16_t*>(dm_smem);
  float (*red)[4] = reinterpret_cast<float (*)[4]>(dm_smem + (size_t)M * H * 2);
  float (*part)[DM_MAXM] = reinterpret_cast<float (*)[DM_MAXM]>(dm_smem + (size_t)M * H * 2 + 2 * 4 * sizeof(float));
  int* const bflag = reinterpret_cast<int*>(dm_smem + (size_t)M * H * 2 + 2 * 4 * sizeof(float) +
                                            4 * DM_MAXM * sizeof(float));
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int nch = H >> 3;
  const int64_t K = H;

  const int64_t wstep = (int64_t)gridDim.x * 4;
  int64_t r = (int64_t)blockIdx.x * 4 + wv;
  u32x4 wa[2][DM_KCH], wb[2][DM_KCH], wc[2][DM_KCH];  // buffers of [gate, up][chunk] (static indices)
  auto load_pair = [&](int64_t row, u32x4 (&dst)[2][DM_KCH]) {
    const int64_t n = row < I ? row : I - 1;
    const bf16_t* wr[2] = {wg + n * ldw, wu + n * ldw};
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < DM_KCH; ++i) {
        const int64_t k = (int64_t)lane * 8 + i * 512;
        // branch-free (a chunk past K re-reads the last one; the dot products skip it), so the waits are exact
        dst[q][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr[q] + (k < K ? k : K - 8)));
      }
  };
  bool poison = false;
  // ---------------- phase O (attn != NULL): y = attn @ wo^T, the o projection (gemv_pf_kernel<4, 1>'s arithmetic,
  // one wave a row), stored write-through; the first gate|up pair is then issued and a grid barrier publishes y
  if (attn != nullptr) {
    // every o row of this wave (H <= 2 * waves: at most two) has its weight loads in flight before any dot product
    const int64_t ro[2] = {r, r + wstep};
    u32x4 ov[2][DM_OCH];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16_t* wr = wo + (ro[u] < H ? ro[u] : H - 1) * ldwo;
#pragma unroll
      for (int i = 0; i < DM_OCH; ++i) {
        const int64_t k = (int64_t)lane * 8 + i * 512;
        ov[u][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr + (k < KO ? k : KO - 8)));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (ro[u] >= H) break;
      float acc[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) acc[m] = 0.f;
#pragma unroll
      for (int i = 0; i < DM_OCH; ++i) {
        const int64_t k = (int64_t)lane * 8 + i * 512;
        if (k < KO) {
          float wf[8];
          unpack8(ov[u][i], wf);
#pragma unroll
          for (int m = 0; m < MR; ++m) {
            if (m < M) {
              float xf[8];
              unpack8(*reinterpret_cast<const u32x4*>(attn + m * ld_attn + k), xf);
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[m] = fmaf(wf[j], xf[j], acc[m]);
            }
          }
        }
      }
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        if (m < M) {
          const float v = wave_sum(acc[m]);
          if (lane == 0)
            __hip_atomic_store(reinterpret_cast<unsigned short*>(y + m * ldx + ro[u]), (unsigned short)f2bf(v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    asm volatile("" ::: "memory");
    load_pair(r, wa);
    if (DEPTH == 3) load_pair(r + wstep, wb);
    // a block that missed this barrier read a partial y: its act rows (and block 0's h) become NaN, and every
    // down row sums all of act, so the whole output is NaN
    poison = grid_barrier<2 * DM_KCH * (DEPTH == 3 ? 2 : 1), 0>(sync, gridDim.x, bflag, spin_ticks);
  }

  // ---------------- phase A prologue: norm inputs, then the first gate|up row pair (gemv_norm2_kernel's order)
  u32x4 yv[MR][DM_NC], rv[MR][DM_NC], w1v[DM_NC], w2v[DM_NC];
#pragma unroll
  for (int cI = 0; cI < DM_NC; ++cI) {
    const int ch = t + cI * 256;
    w1v[cI] = w2v[cI] = u32x4{0u, 0u, 0u, 0u};
    if (ch < nch) {
      w1v[cI] = *reinterpret_cast<const u32x4*>(w1 + ch * 8);
      w2v[cI] = *reinterpret_cast<const u32x4*>(w2 + ch * 8);
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      yv[m][cI] = rv[m][cI] = u32x4{0u, 0u, 0u, 0u};
      if (m < M && ch < nch) {
        yv[m][cI] = *reinterpret_cast<const u32x4*>(y + m * ldx + ch * 8);
        rv[m][cI] = *reinterpret_cast<const u32x4*>(res + m * ldx + ch * 8);
      }
    }
  }
  if (attn == nullptr) {
    load_pair(r, wa);
    if (DEPTH == 3) load_pair(r + wstep, wb);
  }

  // ---------------- the norm pair (block_sum's order: wave butterfly, then the four waves in order)
  auto bsum = [&](float v, int slot) {
    v = wave_sum(v);
    if (lane == 0) red[slot][wv] = v;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    return ((red[slot][0] + red[slot][1]) + red[slot][2]) + red[slot][3];
  };
#pragma unroll
  for (int m = 0; m < MR; ++m) {
    if (m < M) {
      float v[DM_NC][8];
      float ss = 0.f;
#pragma unroll
      for (int cI = 0; cI < DM_NC; ++cI)
        if (t + cI * 256 < nch) {
          unpack8(yv[m][cI], v[cI]);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += v[cI][j] * v[cI][j];
        }
      const float rstd1 = rsqrtf(bsum(ss, 0) / (float)K + eps1);
      float ss2 = 0.f;
#pragma unroll
      for (int cI = 0; cI < DM_NC; ++cI) {
        const int ch = t + cI * 256;
        if (ch < nch) {
          float wf[8], rr[8];
          unpack8(w1v[cI], wf);
          unpack8(rv[m][cI], rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            v[cI][j] = round_bf(rr[j] + round_bf((v[cI][j] * rstd1) * (1.0f + wf[j])));
            ss2 += v[cI][j] * v[cI][j];
          }
          if (blockIdx.x == 0)
            *reinterpret_cast<u32x4*>(h_out + m * ldx + ch * 8) =
                poison ? u32x4{0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u} : pack8(v[cI]);
        }
      }
      const float rstd2 = rsqrtf(bsum(ss2, 1) / (float)K + eps2);
#pragma unroll
      for (int cI = 0; cI < DM_NC; ++cI) {
        const int ch = t + cI * 256;
        if (ch < nch) {
          float wf[8], o[8];
          unpack8(w2v[cI], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (v[cI][j] * rstd2) * (1.0f + wf[j]);
          *reinterpret_cast<u32x4*>(xs + m * H + ch * 8) = pack8(o);
        }
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ---------------- phase A: gate|up row pairs of this wave, the next pair's weights in flight
  auto pair = [&](const u32x4 (&wcur)[2][DM_KCH], u32x4 (&wnext)[2][DM_KCH]) {
    // unconditional (clamped row): the compiler can then wait for the current pair only
    load_pair(r + (DEPTH - 1) * wstep, wnext);
    float acc[2][MR];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int m = 0; m < MR; ++m) acc[q][m] = 0.f;
#pragma unroll
    for (int i = 0; i < DM_KCH; ++i) {
      const int64_t k = (int64_t)lane * 8 + i * 512;
      if (k < K) {
        float wf[2][8];
#pragma unroll
        for (int q = 0; q < 2; ++q) unpack8(wcur[q][i], wf[q]);
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (m < M) {
            float xf[8];
            unpack8(*reinterpret_cast<const u32x4*>(xs + m * H + k), xf);
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[q][m] = fmaf(wf[q][j], xf[j], acc[q][m]);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if (m < M) {
        const float g = round_bf(wave_sum(acc[0][m])), u = round_bf(wave_sum(acc[1][m]));
        if (lane == 0)  // write-through: read by other CUs / XCDs after the grid barrier
          __hip_atomic_store(reinterpret_cast<unsigned short*>(act + m * ldact + r),
                             poison ? (unsigned short)0x7fc0 : (unsigned short)f2bf(gelu_bf16(g) * u),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    r += wstep;
  };
  if constexpr (DEPTH == 3) {
    while (r < I) {
      pair(wa, wc);
      if (r >= I) break;
      pair(wb, wa);
      if (r >= I) break;
      pair(wc, wb);
    }
  } else {
    while (r < I) {
      pair(wa, wb);
      if (r >= I) break;
      pair(wb, wa);
    }
  }

  // the block's down rows are independent of act: their weights stream in while phase A drains and the grid barrier
  // waits -- the first one, or at batch 1 the first DM_DPRE (all of them when H <= DM_DPRE x blocks)
  u32x4 da[DM_DCH], db[DM_DCH];
  auto load_down = [&](int64_t row, u32x4 (&dst)[DM_DCH]) {
    const bf16_t* wr = wd + row * ldd;
#pragma unroll
    for (int i = 0; i < DM_DCH; ++i) {
      const int64_t k = (int64_t)t * 8 + i * 2048;
      dst[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr + (k < I ? k : I - 8)));
    }
  };
  int64_t n = blockIdx.x;
  constexpr bool PRE_OK = MR == 1 && DM_DPRE > 1;
  const bool pre = PRE_OK && H <= (int64_t)DM_DPRE * gridDim.x;  // grid-uniform
  u32x4 dpre[PRE_OK ? DM_DPRE : 1][DM_DCH];
  bool late;
  if constexpr (PRE_OK) {
    if (pre) {
#pragma unroll
      for (int q = 0; q < DM_DPRE; ++q) {
        const int64_t rq = n + (int64_t)q * gridDim.x;
        load_down(rq < H ? rq : H - 1, dpre[q]);
      }
      // a block that missed this barrier would read a partial act: it writes NaN rows instead
      late = grid_barrier<DM_DPRE * DM_DCH, 1>(sync, gridDim.x, bflag, spin_ticks);
    }
  }
  if (!pre) {
    load_down(n < H ? n : H - 1, da);
    late = grid_barrier<DM_DCH, 1>(sync, gridDim.x, bflag, spin_ticks);
  }

  // ---------------- phase C: down rows of this block, four waves split each row's K range
  // one token row (the batch-1 decode step): the thread's act chunks, the same for every down row, in registers
  u32x4 av[DM_DCH];
  if constexpr (MR == 1) {
#pragma unroll
    for (int i = 0; i < DM_DCH; ++i) {
      const int64_t k = (int64_t)t * 8 + i * 2048;
      av[i] = k < I ? *reinterpret_cast<const u32x4*>(act + k) : u32x4{0u, 0u, 0u, 0u};
    }
  }
  auto dot_row = [&](const u32x4 (&dcur)[DM_DCH]) {
    float acc[MR];
#pragma unroll
    for (int m = 0; m < MR; ++m) acc[m] = 0.f;
#pragma unroll
    for (int i = 0; i < DM_DCH; ++i) {
      const int64_t k = (int64_t)t * 8 + i * 2048;
      if (k < I) {
        float wf[8];
        unpack8(dcur[i], wf);
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          if (m < M) {
            float xf[8];
            if constexpr (MR == 1) unpack8(av[i], xf);
            else unpack8(*reinterpret_cast<const u32x4*>(act + m * ldact + k), xf);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[m] = fmaf(wf[j], xf[j], acc[m]);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      if (m < M) {
        const float v = wave_sum(acc[m]);
        if (lane == 0) part[wv][m] = v;
      }
    }
    __syncthreads();
    if (t < M) out[t * ldo + n] = late ? (bf16_t)0x7fc0 : f2bf(((part[0][t] + part[1][t]) + part[2][t]) + part[3][t]);
    __syncthreads();  // part is rewritten by the next row
    n += gridDim.x;
  };
  if constexpr (PRE_OK) {
    if (pre) {
#pragma unroll
      for (int q = 0; q < DM_DPRE; ++q)
        if (n < H) dot_row(dpre[q]);
      return;
    }
  }
  auto row = [&](const u32x4 (&dcur)[DM_DCH], u32x4 (&dnext)[DM_DCH]) {
    load_down(n + gridDim.x < H ? n + gridDim.x : H - 1, dnext);  // unconditional: see phase A
    dot_row(dcur);
  };
  while (n < H) {
    row(da, db);
    if (n >= H) break;
    row(db, da);
  }
}

}  // namespace

namespace {
size_t dm_lds(int64_t M, int64_t H) {
  return (size_t)M * H * 2 + 2 * 4 * sizeof(float) + 4 * DM_MAXM * sizeof(float) + 16;
}

// blocks of the persistent grid: DM_BPC per CU, capped by what the occupancy calculator says can be resident at once
// for this instance and LDS size (so a grid barrier can complete), and by the rows there are; 0 = cannot run
int dm_blocks(int64_t M, int64_t H, int64_t I) {
  int per_cu = 0;
  const size_t lds = dm_lds(M, H);
  const hipError_t e =
      M == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_mlp_kernel<1>, 256, lds)
             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_mlp_kernel<DM_MAXM>, 256, lds);
  if (e != hipSuccess || per_cu <= 0) {
    (void)hipGetLastError();
    return 0;
  }
  const int64_t resident = (int64_t)svla::num_cus() * std::min(per_cu, DM_BPC);
  return (int)std::min<int64_t>(resident, std::max<int64_t>(I / 4, 1));
}

// SVLA_DECODE_MLP_COOP=1 launches with the cooperative attribute.  Not the default: measured 2.40-2.47 ms per
// decode token against 1.84 with the plain launch (profiles/r8a_decode_mlp_coop_ab.txt: ~21 us more per launch, 26
// launches a token).  The plain launch's grid is occupancy-capped (dm_blocks), and a block that still misses a
// barrier (another process holding CUs) writes NaN and counts a timeout the callers raise on.
bool dm_coop() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SVLA_DECODE_MLP_COOP");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

// test hooks (svla_decode_mlp_debug): a grid override, the launch mode and the barrier wait bound
int g_dm_grid_override = 0;
int g_dm_coop_override = -1;
int g_dm_timeout_ms = 1000;

long long dm_spin_ticks() {
  static int rate_khz = 0;  // the wall clock's rate (100 MHz on MI3xx)
  if (rate_khz <= 0) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess || v <= 0) v = 100000;
    rate_khz = v;
  }
  return (long long)rate_khz * g_dm_timeout_ms;
}
}  // namespace

extern "C" size_t svla_decode_mlp_sync_bytes(void) { return DM_SYNC_WORDS * sizeof(unsigned); }

extern "C" void svla_decode_mlp_debug(int grid_override, int cooperative, int timeout_ms) {
  g_dm_grid_override = grid_override > 0 ? grid_override : 0;
  g_dm_coop_override = cooperative;
  g_dm_timeout_ms = timeout_ms > 0 ? timeout_ms : 1000;
}

extern "C" int svla_decode_mlp_grid(int64_t M, int64_t H, int64_t I) {
  if (M < 1 || M > DM_MAXM || H <= 0 || I <= 0) return 0;
  return dm_blocks(M, H, I);
}

extern "C" int svla_decode_mlp(int64_t M, int64_t H, int64_t I, const void* res, void* y, int64_t ldx, const void* w1,
                               const void* w2, float eps1, float eps2, void* h_out, const void* w_gate,
                               const void* w_up, int64_t ldw, const void* w_down, int64_t ldd, void* act,
                               int64_t ldact, void* out, int64_t ldo, const void* attn, int64_t ld_attn, int64_t KO,
                               const void* w_o, int64_t ldwo, unsigned* sync, void* stream) {
  SVLA_CHECK_ARG(M >= 1 && M <= DM_MAXM && H > 0 && H % 8 == 0 && H <= 512 * DM_KCH && H <= 256 * 8 * DM_NC &&
                     I > 0 && I % 8 == 0 && I <= 2048 * DM_DCH,
                 "decode_mlp: M in [1, %d], H a multiple of 8 <= %d, I a multiple of 8 <= %d", DM_MAXM, 512 * DM_KCH,
                 2048 * DM_DCH);
  SVLA_CHECK_ARG(res && y && w1 && w2 && h_out && w_gate && w_up && w_down && act && out && sync,
                 "decode_mlp: NULL argument");
  SVLA_CHECK_ARG(ldx % 8 == 0 && ldx >= H && ldw % 8 == 0 && ldw >= H && ldd % 8 == 0 && ldd >= I &&
                     ldact % 8 == 0 && ldact >= I && ldo >= H,
                 "decode_mlp: leading dimensions");
  SVLA_CHECK_ARG(!attn || (w_o && KO > 0 && KO % 8 == 0 && KO <= 512 * DM_OCH && ld_attn % 8 == 0 && ld_attn >= KO &&
                           ldwo % 8 == 0 && ldwo >= KO),
                 "decode_mlp: the o projection needs w_o, KO a multiple of 8 <= %d and 16-B rows", 512 * DM_OCH);
  const int blocks = g_dm_grid_override > 0 ? g_dm_grid_override : dm_blocks(M, H, I);
  const bool coop = g_dm_coop_override >= 0 ? g_dm_coop_override == 1 : dm_coop();
  long long spin_ticks = dm_spin_ticks();
  SVLA_CHECK_ARG(blocks > 0, "decode_mlp: no block of this instance fits on a CU (LDS %zu B); use the two-launch path",
                 dm_lds(M, H));
  SVLA_CHECK_ARG(!attn || H <= 2 * 4 * (int64_t)blocks, "decode_mlp: the o phase covers at most two rows a wave");
  const size_t lds = dm_lds(M, H);
  hipStream_t s = (hipStream_t)stream;
  // plain launch of the occupancy-capped grid (default), or cooperative (SVLA_DECODE_MLP_COOP=1: the runtime then
  // dispatches the grid only when every block can be resident together, or fails the launch)
  int Mi = (int)M, Hi = (int)H, Ii = (int)I, KOi = (int)KO;
  const bf16_t *res_ = (const bf16_t*)res, *w1_ = (const bf16_t*)w1, *w2_ = (const bf16_t*)w2,
               *wg_ = (const bf16_t*)w_gate, *wu_ = (const bf16_t*)w_up, *wd_ = (const bf16_t*)w_down,
               *attn_ = (const bf16_t*)attn, *wo_ = (const bf16_t*)w_o;
  bf16_t *y_ = (bf16_t*)y, *h_ = (bf16_t*)h_out, *act_ = (bf16_t*)act, *out_ = (bf16_t*)out;
  void* args[] = {&Mi,  &Hi,    &Ii,   &res_,  &y_,      &ldx, &w1_,  &w2_,    &eps1, &eps2, &h_,   &wg_, &wu_,  &ldw,
                  &wd_, &ldd,   &act_, &ldact, &out_,    &ldo, &attn_, &ld_attn, &KOi, &wo_,  &ldwo, &sync,
                  &spin_ticks};
  hipLaunchAttribute attr[1];
  attr[0].id = hipLaunchAttributeCooperative;
  attr[0].val.cooperative = 1;
  hipLaunchConfig_t cfg{};
  cfg.gridDim = dim3((unsigned)blocks);
  cfg.blockDim = dim3(256);
  cfg.dynamicSmemBytes = lds;
  cfg.stream = s;
  cfg.attrs = attr;
  cfg.numAttrs = coop ? 1 : 0;
  const void* fn = M == 1 ? reinterpret_cast<const void*>(&decode_mlp_kernel<1>)
                          : reinterpret_cast<const void*>(&decode_mlp_kernel<DM_MAXM>);
  const hipError_t e = hipLaunchKernelExC(&cfg, fn, args);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    svla::set_error("decode_mlp: %s launch of %d blocks failed: %s", coop ? "cooperative" : "plain", blocks,
                    hipGetErrorString(e));
    return SVLA_ERR_HIP;
  }
  return svla::check_launch("decode_mlp");
}
