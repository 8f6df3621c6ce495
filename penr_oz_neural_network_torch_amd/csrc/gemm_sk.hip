// N1b — persistent stream-K bf16 GEMM for gfx950 (engine 2 of pz::gemm / pz::gemm_pair).
//
// Replaces the reference's per-layer matmuls (neural_net_model.py:117 forward `x @ W`, and the two
// autograd `mm` of cost.backward(), :495) with the fused stage epilogues around them (bias :119,
// activation :172-184, dropout :393-395, bias-gradient column sums).
//
// Where it runs: NOT the default step engine (gemm_mfma.hip's tiled kernels are; at the full CU
// budget both reach the same main-loop rate and the tiled epilogues are lighter). The trainer uses
// it for ONE launch: under data parallelism with PZ_COMM_BUDGET=k, the paired weight-gradient
// GEMMs issued while a gradient bucket is on the wire run as one stream-K schedule on the CUs the
// collective leaves (a one-round tiled grid would leave a straggler round behind the held CUs).
// PZ_GEMM_SK=1 routes every eligible GEMM here (A/B). The 4-wave 128x128-wave-tile loop measured
// in round 5 (0.70-0.75x the ping-pong, profiles/r5_pmc_sk4_vs_pingpong.txt) lives in
// tools/gemm_w4_lab.hip, not in the library.
//
// Design (MI355X-first; /opt/skills/guides/cdna_hip_programming.md §5, MI355X_MICROARCH.md):
//  * 256x256 macro tile on EIGHT waves (two per SIMD, 128x64 wave tiles of 16x16x32 bf16 MFMAs) in
//    the ping-pong schedule of gemm_mfma.hip VAR 30: a 2-slot ring of 64-deep K steps filled by
//    buffer-addressed LDS-DMA (`buffer_load_dwordx4 ... lds`, swizzle on the per-lane SOURCE
//    offset), the staging lane offsets precomputed once per piece class.
//  * PERSISTENT: the grid is the CU budget (GemmArgs::cus, at most the device's CUs, one
//    workgroup per CU). Every workgroup walks a static schedule: a stream-K region — the tiles
//    that do not fill whole rounds of workgroups, their K iterations split evenly over ALL
//    workgroups ("two-tile" stream-K: the remainder plus one full round) — then whole data-
//    parallel tiles. A CU budget below the device (RCCL channels resident beside the GEMMs)
//    shrinks the grid instead of leaving a straggler round of tiles.
//  * Stream-K partial tiles: each contributor stores its fp32 accumulators write-through (sc1)
//    into a slab, drains, joins a barrier and takes a relaxed agent-scope ticket (MI355X_MICROARCH
//    hand-off table, row 1); the LAST arriver folds the slabs in K order with sc1 loads and runs
//    the epilogue. The sum order never depends on which workgroup arrives last: deterministic.
//  * Epilogues: gemm_epilogue.h's LDS-staged kinds on 64-column wave tiles; fp32 outputs (weight
//    gradients) store straight from the accumulators.
//  * Two problems of one layout / epilogue kind / K may share a launch (the two skinny weight-
//    gradient GEMMs of a 3-layer MLP): their tiles form one schedule.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "pz_common.h"
#include "pz_launch.h"

namespace pz {
namespace {

#include "gemm_common.h"
#include "gemm_epilogue.h"

// tools/sk_stamps.hip (diagnostic build only): s_memrealtime stamps per workgroup and unit at
// unit start / main loop done / slab handed off / fold done / epilogue done, plus the unit's tile
// and K range, into g.p[0].dbg ([grid][kSkStampUnits][8] u64)
constexpr int kSkStampUnits = 6;
#ifdef PZ_GEMM_STAMPS
#define PZ_SK_STAMP(u, i)                                                                            \
  do {                                                                                               \
    if (threadIdx.x == 0 && (u) < kSkStampUnits)                                                     \
      g.p[0].dbg[(static_cast<int64_t>(w) * kSkStampUnits + (u)) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define PZ_SK_NOTE(u, v)                                                                             \
  do {                                                                                               \
    if (threadIdx.x == 0 && (u) < kSkStampUnits)                                                     \
      g.p[0].dbg[(static_cast<int64_t>(w) * kSkStampUnits + (u)) * 8 + 7] = (v);                     \
  } while (0)
#else
#define PZ_SK_STAMP(u, i) do {} while (0)
#define PZ_SK_NOTE(u, v) do {} while (0)
#endif

constexpr int kSkB = 256;                    // macro tile BM = BN
constexpr int kSkSlab = kSkB * kSkB;         // fp32 floats of one partial tile
constexpr int kSkF32 = 100;                  // epilogue code of the fp32-output store path
constexpr int kSkLds = 128 * 1024;           // both main loops' rings = the epilogue's C image

// Main-loop geometry (W = 8 waves): two waves per SIMD, 128x64 wave tiles, the ping-pong over a
// 2-slot 64-deep ring of the tiled kernels (gemm_mfma.hip VAR 30)
template <int W> struct SkGeo {
  static_assert(W == 8, "the library's stream-K engine runs the 8-wave ping-pong loop");
  static constexpr int NT = W * 64;
  static constexpr int WN = W / 2;           // wave grid 2 x WN
  static constexpr int TN = 16 / WN;         // 16x16 accumulator tiles across a wave tile
  static constexpr int WTN = kSkB / WN;
  static constexpr int BK = 64;              // K depth of one schedule step
  static constexpr int CH = 8 * TN;          // f32x4 accumulator chunks per lane
};

struct SkSched {
  int nprob;
  int tiles0;           // tiles of problem 0 (problem 1's tiles follow)
  int tiles;            // all tiles
  int iters;            // K steps per tile
  int grid;             // workgroups
  int sk_tiles;         // tiles [0, sk_tiles) are stream-K'd over every workgroup
  long long sk_iters;   // sk_tiles * iters
};

struct SkArgs {
  GemmArgs p[2];
  SkSched s;
  float* ws;      // [2 * grid][256 * 256] partial slabs: slab 2w = workgroup w's first unit, 2w+1 its last
  int* counters;  // [sk_tiles] tickets, zero between launches (the last arriver resets its tile's)
};

// first stream-K iteration of workgroup w (w = grid: the end)
PZ_DEV long long sk_start(const SkSched& s, int w) { return static_cast<long long>(w) * s.sk_iters / s.grid; }

// the workgroup whose stream-K range holds iteration `it`
PZ_DEV int sk_owner(const SkSched& s, long long it) {
  int w = static_cast<int>(it * s.grid / s.sk_iters);
  while (w + 1 < s.grid && sk_start(s, w + 1) <= it) ++w;
  while (w > 0 && sk_start(s, w) > it) --w;
  return w;
}

PZ_DEV void sk_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------------ W = 8: the ping-pong loop
// Waves 0-3 (group 0) and 4-7 (group 1) share the four SIMDs and run one barrier interval apart:
// while one wave of a SIMD issues its 64-MFMA block (setprio 1), its partner issues the next
// step's LDS-DMA and fragment reads into the gaps (hazard argument: gemm_mfma.hip gemm_body, BK 64
// branch). Group 0 stages step t+1 in its read interval of step t; every wave waits for it
// (vmcnt(0)) before the barrier that opens the next read interval.
// One operand's LDS-DMA of a 64-deep step by the four staging waves (team index tw): piece i of
// 8 per wave = 1 KiB at LDS byte tw * 8 KiB + i KiB of the operand image. The per-lane offsets
// carry the read-side swizzle and depend on the piece only through (i & 1) (K-contiguous) or
// (i & 1, i >> 2 & 1) (M/N-contiguous), so they are computed ONCE per kernel; everything that
// moves with the unit or the K step is wave-uniform (soffset). (gemm_mfma.hip's stage_mn
// recomputes row clamps and offsets per call: in the persistent kernel hipcc spilled them and
// reloaded each from scratch behind an `s_waitcnt vmcnt(0)` that drained the ring.)
struct PpOperand {
  uint32_t voff[4];  // per-lane byte offsets by piece class
  uint32_t base;     // uniform byte offset of this wave's piece 0 at the unit's first step
  uint32_t pstep;    // bytes between consecutive pieces
  uint32_t kstep;    // bytes per 64-deep K step
};

template <bool KC>
PZ_DEV void pp_lane_offsets(uint32_t (&voff)[4], uint32_t ld, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int par = q & 1, hi = q >> 1;
    int chunk;
    uint32_t row;
    if constexpr (KC) {  // 8 rows x 8 chunks of 16 B; swz_kc<64>(r) = (r >> 1) & 7
      row = static_cast<uint32_t>(lane >> 3);
      chunk = (lane & 7) ^ ((par * 4 + (lane >> 4)) & 7);
      (void)hi;
    } else {  // 2 k-rows x 32 chunks; swz_mn(kr) from kr & 3 and kr bit 3
      row = static_cast<uint32_t>(lane >> 5);
      chunk = (lane & 31) ^ ((((2 * par + (lane >> 5)) & 3) | (hi << 2)) << 1);
    }
    voff[q] = (row * ld + static_cast<uint32_t>(chunk) * 8u) * 2u;
  }
}

template <bool KC>
PZ_DEV PpOperand pp_operand(const uint32_t (&voff)[4], uint32_t ld, int row0, int kt0, int tw) {
  PpOperand o;
#pragma unroll
  for (int q = 0; q < 4; ++q) o.voff[q] = voff[q];
  if constexpr (KC) {
    o.base = __builtin_amdgcn_readfirstlane((static_cast<uint32_t>(row0 + tw * 64) * ld + static_cast<uint32_t>(kt0) * 64u) * 2u);
    o.pstep = __builtin_amdgcn_readfirstlane(8u * ld * 2u);
    o.kstep = 128u;
  } else {
    o.base = __builtin_amdgcn_readfirstlane((static_cast<uint32_t>(kt0 * 64 + tw * 16) * ld + static_cast<uint32_t>(row0)) * 2u);
    o.pstep = __builtin_amdgcn_readfirstlane(2u * ld * 2u);
    o.kstep = __builtin_amdgcn_readfirstlane(64u * ld * 2u);
  }
  return o;
}

template <bool KC>
PZ_DEV void pp_dma(const PpOperand& o, i32x4_t rs, int kt, uint32_t lds) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = KC ? (i & 1) : ((i & 1) | (((i >> 2) & 1) << 1));
    blds16<0>(rs, o.voff[q], o.base + static_cast<uint32_t>(i) * o.pstep + static_cast<uint32_t>(kt) * o.kstep,
              lds + static_cast<uint32_t>(i) * 1024u);
  }
}

// ------------------------------------------------------------------ W = 8: the ping-pong loop
// Waves 0-3 (group 0) and 4-7 (group 1) share the four SIMDs and run one barrier interval apart:
// while one wave of a SIMD issues its 64-MFMA block (setprio 1), its partner issues the next
// step's LDS-DMA and fragment reads into the gaps (hazard argument: gemm_mfma.hip gemm_body, BK 64
// branch). Group 0 stages step t+1 in its read interval of step t; every wave waits for it
// (vmcnt(0)) before the barrier that opens the next read interval.
template <bool A_KC, bool B_KC>
PZ_DEV void pp_mainloop(f32x4_t (&acc)[8][4], PZ_LDS char* smem, const PpOperand& oa, const PpOperand& ob,
                        i32x4_t rs_a, i32x4_t rs_b, int nk, int wave, int lane) {
  constexpr int BK = 64, A_BYTES = kSkB * BK * 2, SLOT = 2 * A_BYTES;
  const int grp = wave >> 2, tw = wave & 3;
  const int wm = wave >> 2, wn = wave & 3;
  const uint32_t lds0 = lds_addr(smem) + static_cast<uint32_t>(tw) * 8u * 1024u;
  auto stage = [&](int kt) __attribute__((always_inline)) {
    const uint32_t lds = lds0 + static_cast<uint32_t>(kt & 1) * SLOT;
    pp_dma<A_KC>(oa, rs_a, kt, lds);
    pp_dma<B_KC>(ob, rs_b, kt, lds + A_BYTES);
  };
  struct Frags { i16x8_t a[2][8]; i16x8_t b[2][4]; };
  auto read = [&](int slot, Frags& f) __attribute__((always_inline)) {
    const PZ_LDS char* ta = smem + slot * SLOT;
    const PZ_LDS char* tb = ta + A_BYTES;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (B_KC) f.b[kb][j] = frag_kc<BK>(tb, wn * 64 + j * 16 + (lane & 15), (lane >> 4) + 4 * kb);
        else f.b[kb][j] = frag_mn<kSkB>(tb, wn * 64 + j * 16, 8 * (lane >> 4) + 32 * kb, lane);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (A_KC) f.a[kb][i] = frag_kc<BK>(ta, wm * 128 + i * 16 + (lane & 15), (lane >> 4) + 4 * kb);
        else f.a[kb][i] = frag_mn<kSkB>(ta, wm * 128 + i * 16, 8 * (lane >> 4) + 32 * kb, lane);
      }
    }
  };
  // the previous unit's epilogue stores share the VM counter with the DMAs; and every wave is done
  // with the LDS image before slot 0 is refilled
  wait_vm<0>();
  sk_barrier();
  if (grp == 0) stage(0);
  wait_vm<0>();
  sk_barrier();
  if (grp == 1) sk_barrier();
  for (int t = 0; t < nk; ++t) {
    if (grp == 0 && t + 1 < nk) stage(t + 1);
    Frags f;
    read(t & 1, f);
    if (grp == 1) wait_vm<0>();  // step t+1 (issued by group 0 one interval ago) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sk_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, f.b[kb][j]),
                                                              __builtin_bit_cast(bf16x8_t, f.a[kb][i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (grp == 0) wait_vm<0>();
    sk_barrier();
  }
  if (grp == 0) sk_barrier();
}

// fp32-output epilogue (weight gradients): alpha, bias, accumulate; 16-B stores
template <int W>
PZ_DEV void sk_store_f32(const GemmArgs& p, f32x4_t (&acc)[8][SkGeo<W>::TN], int m0, int n0, int wm, int wn, int lane) {
  using G = SkGeo<W>;
  float* __restrict__ Cp = static_cast<float*>(p.C);
  const int g4 = 4 * (lane >> 4);
  static_for<G::TN>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int n = n0 + wn * G::WTN + j * 16 + g4;
    const f32x4_t bias4 = p.bias != nullptr ? *reinterpret_cast<const f32x4_t*>(p.bias + n) : f32x4_t{0.f, 0.f, 0.f, 0.f};
    static_for<8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int m = m0 + wm * 128 + i * 16 + (lane & 15);
      f32x4_t v = acc[i][j] * p.alpha + bias4;
      f32x4_t* dst = reinterpret_cast<f32x4_t*>(Cp + static_cast<int64_t>(m) * p.ldc + n);
      if (p.accumulate) v += *dst;
      *dst = v;
    });
  });
}

template <bool A_KC, bool B_KC, typename OutT, int EK, int W>
__global__ void __launch_bounds__(SkGeo<W>::NT) __attribute__((amdgpu_waves_per_eu(W / 4, W / 4)))
gemm_sk_kernel(const SkArgs g) {
  using G = SkGeo<W>;
  constexpr int NT = G::NT, CH = G::CH;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const SkSched& s = g.s;
  const int w = xcd_remap(blockIdx.x, gridDim.x);  // consecutive ids share an XCD's L2
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int tid = threadIdx.x;
  const int wm = wave / G::WN, wn = wave % G::WN;

  // Work units in schedule order: the stream-K range [s0, s1) cut at tile boundaries, then the
  // data-parallel tiles w, w + grid, ... ONE loop, so the unit body is inlined once.
  const long long s0 = s.sk_iters > 0 ? sk_start(s, w) : 0, s1 = s.sk_iters > 0 ? sk_start(s, w + 1) : 0;
  long long it = s0;
  int dp_t = s.sk_tiles + w;
  int unit = 0;  // (diagnostic stamps only)
  (void)unit;
  for (;;) {
    // this unit: K steps [kb, ke) of tile t; slab >= 0: a stream-K partial tile
    int t, kb, ke, slab;
    if (it < s1) {
      t = static_cast<int>(it / s.iters);
      kb = static_cast<int>(it - static_cast<long long>(t) * s.iters);
      const long long left = s1 - it;
      ke = left < static_cast<long long>(s.iters - kb) ? kb + static_cast<int>(left) : s.iters;
      slab = (kb == 0 && ke == s.iters) ? -1 : 2 * w + (it == s0 ? 0 : 1);
      it += ke - kb;
    } else if (dp_t < s.tiles) {
      t = dp_t;
      kb = 0;
      ke = s.iters;
      slab = -1;
      dp_t += s.grid;
    } else {
      break;
    }
    // (64-bit divisions run on the VALU: pin the unit's scalars to SGPRs, or every buffer
    // descriptor / soffset built from them becomes a waterfall loop)
    t = __builtin_amdgcn_readfirstlane(t);
    kb = __builtin_amdgcn_readfirstlane(kb);
    ke = __builtin_amdgcn_readfirstlane(ke);
    slab = __builtin_amdgcn_readfirstlane(slab);
    PZ_SK_STAMP(unit, 0);
    PZ_SK_NOTE(unit, (static_cast<uint64_t>(t) << 40) | (static_cast<uint64_t>(kb) << 20) | static_cast<uint64_t>(ke) |
                         (slab >= 0 ? (uint64_t(1) << 63) : 0));
    const int prob = (s.nprob > 1 && t >= s.tiles0) ? 1 : 0;
    const GemmArgs& p = g.p[prob];
    const int tl = t - prob * s.tiles0;
    int tm, tn, tile_, slice_;
    tile_coords(tl, p.M / kSkB, p.N / kSkB, 1, tm, tn, tile_, slice_);
    const int m0 = tm * kSkB, n0 = tn * kSkB;
    f32x4_t acc[8][G::TN];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < G::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    {
      const int tw = wave & 3;
      // (the staging lane offsets: recomputed per unit, ~20 VALU ops, rather than held live
      // through the fold and the epilogue)
      uint32_t va[4], vb[4];
      pp_lane_offsets<A_KC>(va, static_cast<uint32_t>(p.lda), lane);
      pp_lane_offsets<B_KC>(vb, static_cast<uint32_t>(p.ldb), lane);
      const PpOperand oa = pp_operand<A_KC>(va, static_cast<uint32_t>(p.lda), m0, kb, tw);
      const PpOperand ob = pp_operand<B_KC>(vb, static_cast<uint32_t>(p.ldb), n0, kb, tw);
      pp_mainloop<A_KC, B_KC>(acc, smem, oa, ob, buf_rsrc(p.A), buf_rsrc(p.B), ke - kb, wave, lane);
    }

    PZ_SK_STAMP(unit, 1);
    if (slab >= 0) {
      // ---- stream-K hand-off (write-through slabs, one ticket per contributor: MI355X_MICROARCH
      // hand-off table, row 1)
      constexpr int kSc1 = 16;
      const auto rs_own = __builtin_amdgcn_make_buffer_rsrc(g.ws + static_cast<int64_t>(slab) * kSkSlab, 0, kSkSlab * 4,
                                                            0x00020000);
      static_for<CH>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, acc[c / G::TN][c % G::TN]), rs_own,
                                               tid * 16, c * NT * 16, kSc1);
      });
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const long long t0 = static_cast<long long>(t) * s.iters;
      const int wlo = __builtin_amdgcn_readfirstlane(sk_owner(s, t0));
      const int whi = __builtin_amdgcn_readfirstlane(sk_owner(s, t0 + s.iters - 1));
      PZ_LDS int* flag = (PZ_LDS int*)(smem);
      if (tid == 0) {
        const int prev = __hip_atomic_fetch_add(g.counters + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = prev == whi - wlo;
        *flag = last;
        if (last) g.counters[t] = 0;  // ready for the next launch
      }
      __syncthreads();
      PZ_SK_STAMP(unit, 2);
      if (__builtin_amdgcn_readfirstlane(*flag) == 0) {  // (uniform) another contributor finishes it
        ++unit;
        continue;
      }
      auto slab_of = [&](int c) { return __builtin_amdgcn_readfirstlane(2 * c + (sk_start(s, c) < t0 ? 1 : 0)); };
      auto rs_of = [&](int c) {
        return __builtin_amdgcn_make_buffer_rsrc(g.ws + static_cast<int64_t>(slab_of(c)) * kSkSlab, 0, kSkSlab * 4,
                                                 0x00020000);
      };
      // in groups of 16 chunks (64 VGPRs of loads in flight): an unbounded unrolled fold let
      // hipcc hoist every load and spill
      auto fold = [&](const auto& rs) __attribute__((always_inline)) {
        static_for<CH / 16>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          f32x4_t ld[16];
          static_for<16>([&](auto cc) {
            constexpr int c = 16 * q + decltype(cc)::value;
            ld[c - 16 * q] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, c * NT * 16, kSc1));
          });
          static_for<16>([&](auto cc) {
            constexpr int c = 16 * q + decltype(cc)::value;
            acc[c / G::TN][c % G::TN] = acc[c / G::TN][c % G::TN] + ld[c - 16 * q];
          });
          __builtin_amdgcn_sched_barrier(0);
        });
      };
      // sk_plan gives every tile at most two contributors: own + other == the K-ordered sum
      // (addition commutes), one 256 KiB slab read. (Measured, not kept: tiles split over 3-4
      // contributors — the last arriver's fold of 0.75-1 MiB took 36-41 us, profiles/r5_sk_stamps.txt)
      fold(rs_of(w == wlo ? whi : wlo));
    }

    PZ_SK_STAMP(unit, 3);
    // ---- epilogue
    if constexpr (EK == kSkF32) {
      sk_store_f32<W>(p, acc, m0, n0, wm, wn, lane);
    } else {
      epilogue_lds<kSkB, kSkB, 2, G::WN, Lay16<8, G::TN>, false, EK>(p, acc, smem, m0, n0, wm, wn, lane, p.alpha);
    }
#ifdef PZ_GEMM_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's stores have left this CU
#endif
    PZ_SK_STAMP(unit, 4);
    ++unit;
  }
}

int device_cus() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return cus > 0 ? cus : 256;
  }();
  return n;
}

// which epilogue covers these arguments (-1: none on this engine)
int sk_epi_kind(const GemmArgs& p) {
  if (p.out_dtype == DT_F32) {
    if (p.epi_mode != EPI_STORE || p.mask != nullptr || p.out8 != nullptr || p.colsum != nullptr) return -1;
    return kSkF32;
  }
  if (p.out_dtype != DT_BF16 || p.accumulate) return -1;
  if (p.epi_mode == EPI_STORE) {
    if (p.out8 != nullptr) return -1;
    return (p.bias == nullptr && p.colsum == nullptr && p.mask == nullptr) ? EK_STORE : EK_ANY;
  }
  if (p.epi_mode == EPI_FWD) {
    const EpiSpec& e = p.epi;
    if ((e.act == ACT_NONE || e.act == ACT_RELU) && p.colsum == nullptr) {
      const bool relu = e.act == ACT_RELU;
      if (!e.drop_all) {
        if (relu && !e.drop_pre && e.drop_post) return EK_F_RELU_POST;
        if (relu && e.drop_pre && e.drop_post) return EK_F_RELU_PREPOST;
        if (!relu && e.drop_pre && !e.drop_post) return EK_F_PRE;
      }
      return EK_RELU;
    }
    return EK_ANY;
  }
  if (p.epi_mode == EPI_BWD) {
    if (p.mask != nullptr) return p.epi.act == ACT_RELU ? EK_BWD_MASK : -1;
    if (p.aux == nullptr || p.aux_dtype != DT_BF16 || p.ldaux % 8 != 0 || (reinterpret_cast<uintptr_t>(p.aux) & 15))
      return -1;
    return EK_ANY;
  }
  return -1;
}

SkSched sk_plan(const GemmArgs* probs, int n) {
  SkSched s{};
  s.nprob = n;
  s.tiles0 = (probs[0].M / kSkB) * (probs[0].N / kSkB);
  s.tiles = s.tiles0 + (n > 1 ? (probs[1].M / kSkB) * (probs[1].N / kSkB) : 0);
  constexpr int bk = SkGeo<8>::BK;
  s.iters = probs[0].K / bk;
  const int cus = device_cus();
  int grid = probs[0].cus > 0 ? std::min(probs[0].cus, cus) : cus;
  const int T = s.tiles;
  // At most TWO contributors per tile. Fewer tiles than workgroups: each tile in two K halves on
  // 2T workgroups when the budget holds them and the halves are >= 256 deep, else one workgroup
  // per tile (data-parallel; the other CUs idle but the survivors run faster per step). At least
  // as many tiles: the "two-tile" region gives every workgroup >= one tile of K steps, so a tile
  // meets at most two workgroups' ranges.
  if (T < grid) grid = (2 * T <= grid && s.iters * bk >= 512) ? 2 * T : T;
  int sk = 0;
  if (T % grid != 0) sk = T < grid ? T : T % grid + grid;
  s.grid = grid;
  s.sk_tiles = sk;
  s.sk_iters = static_cast<long long>(sk) * s.iters;
  return s;
}

template <bool AKC, bool BKC, typename OutT, int EK, int W>
hipError_t sk_launch(const SkArgs& a, hipStream_t st) {
  auto kern = gemm_sk_kernel<AKC, BKC, OutT, EK, W>;
  static bool attr_set = false;
  if (!attr_set) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, kSkLds);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.s.grid), dim3(SkGeo<W>::NT), kSkLds, st, a);
  return hipGetLastError();
}

hipError_t sk_dispatch(const SkArgs& a, int ek, hipStream_t st) {
  const GemmArgs& p = a.p[0];
  if (p.a_kc && !p.b_kc) {  // forward X · W[in, out]
    switch (ek) {
      case EK_STORE: return sk_launch<true, false, uint16_t, EK_STORE, 8>(a, st);
      case EK_RELU: return sk_launch<true, false, uint16_t, EK_RELU, 8>(a, st);
      case EK_F_RELU_POST: return sk_launch<true, false, uint16_t, EK_F_RELU_POST, 8>(a, st);
      case EK_F_RELU_PREPOST: return sk_launch<true, false, uint16_t, EK_F_RELU_PREPOST, 8>(a, st);
      case EK_F_PRE: return sk_launch<true, false, uint16_t, EK_F_PRE, 8>(a, st);
      case EK_ANY: return sk_launch<true, false, uint16_t, EK_ANY, 8>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if (p.a_kc && p.b_kc) {  // dX = dZ · Wᵀ
    switch (ek) {
      case EK_STORE: return sk_launch<true, true, uint16_t, EK_STORE, 8>(a, st);
      case EK_BWD_MASK: return sk_launch<true, true, uint16_t, EK_BWD_MASK, 8>(a, st);
      case EK_ANY: return sk_launch<true, true, uint16_t, EK_ANY, 8>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  if (!p.a_kc && !p.b_kc) {  // dW = Xᵀ · dZ
    switch (ek) {
      case EK_STORE: return sk_launch<false, false, uint16_t, EK_STORE, 8>(a, st);
      case kSkF32: return sk_launch<false, false, float, kSkF32, 8>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace

bool sk_default() {
  static const bool on = [] {
    const char* e = getenv("PZ_GEMM_SK");
    return e != nullptr && atoi(e) != 0;
  }();
  return on;
}

bool deterministic() {
  static const bool on = [] {
    const char* e = getenv("PZ_DETERMINISTIC");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

bool sk_eligible(const GemmArgs& p) {
  if (p.force_generic || p.in_dtype != DT_BF16 || (p.out_dtype != DT_BF16 && p.out_dtype != DT_F32)) return false;
  if (p.bias64 != nullptr || p.colsum64 != nullptr) return false;
  constexpr int bk = SkGeo<8>::BK;
  if (p.engine == 3) return false;  // (round-5 lab loop: tools/gemm_w4_lab.hip)
  if (p.M <= 0 || p.N <= 0 || p.M % kSkB != 0 || p.N % kSkB != 0 || p.K % bk != 0 || p.K < 2 * bk) return false;
  if (!p.a_kc && p.b_kc) return false;  // (no MLP GEMM has this layout)
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(p.A) || !al16(p.B) || (p.C != nullptr && !al16(p.C))) return false;
  if (p.lda % 8 != 0 || p.ldb % 8 != 0 || p.ldc % 8 != 0 || p.idx_ld % 2 != 0) return false;
  if (p.bias != nullptr && !al16(p.bias)) return false;
  constexpr int64_t kLim = int64_t(1) << 32;  // buffer-addressed staging: 32-bit byte offsets
  if ((p.a_kc ? static_cast<int64_t>(p.M) : static_cast<int64_t>(p.K)) * p.lda * 2 >= kLim) return false;
  if ((p.b_kc ? static_cast<int64_t>(p.N) : static_cast<int64_t>(p.K)) * p.ldb * 2 >= kLim) return false;
  if (p.mask != nullptr && (p.ldmask % 32 != 0 || (reinterpret_cast<uintptr_t>(p.mask) & 15) != 0)) return false;
  if (p.out8 != nullptr && (p.out8_fmt != (p.epi_mode == EPI_BWD ? 1 : 0) || p.ldout8 % 8 != 0 ||
                            (reinterpret_cast<uintptr_t>(p.out8) & 7) != 0 || p.out8_qscale == nullptr))
    return false;
  const int ek = sk_epi_kind(p);
  return ek >= 0;
}

int sk_tickets(const GemmArgs* probs, int n) { return sk_plan(probs, n).sk_tiles; }

int64_t sk_ws_floats(const GemmArgs* probs, int n) {
  const SkSched s = sk_plan(probs, n);
  return s.sk_tiles > 0 ? static_cast<int64_t>(2) * s.grid * kSkSlab : 0;
}

hipError_t gemm_sk(const GemmArgs* probs, int n, float* ws, int* counters, hipStream_t st) {
  if (n < 1 || n > 2) return hipErrorInvalidValue;
  for (int i = 0; i < n; ++i)
    if (!sk_eligible(probs[i])) return hipErrorInvalidValue;
  const int ek = sk_epi_kind(probs[0]);
  if (n == 2 && (probs[1].K != probs[0].K || probs[1].a_kc != probs[0].a_kc || probs[1].b_kc != probs[0].b_kc ||
                 sk_epi_kind(probs[1]) != ek || probs[1].out_dtype != probs[0].out_dtype))
    return hipErrorInvalidValue;
  SkArgs a{};
  for (int i = 0; i < n; ++i) {
    a.p[i] = probs[i];
    a.p[i].store_wt = 1;
  }
  a.s = sk_plan(probs, n);
  if (a.s.sk_tiles > 0 && (ws == nullptr || counters == nullptr)) return hipErrorInvalidValue;
  a.ws = ws;
  a.counters = counters;
  return sk_dispatch(a, ek, st);
}

}  // namespace pz
