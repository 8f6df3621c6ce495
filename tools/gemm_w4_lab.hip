// Feasibility probe: a 4-wave 256x256x64 bf16 GEMM main loop (one wave per SIMD, 128x128 wave
// tiles, accumulators in AGPRs, operands staged global -> VGPR -> ds_write_b128 two K steps ahead)
// against the library's 8-wave ping-pong (VAR 30). K-contiguous x K-contiguous (dX layout),
// plain bf16 store epilogue. Same harness conventions as tools/gemm_lab.hip.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I penr_oz_neural_network_torch_amd/csrc \
//         tools/gemm_w4_lab.hip -o tools/gemm_w4_lab && tools/gemm_w4_lab
#define PZ_GEMM_LAB 1
#include "../penr_oz_neural_network_torch_amd/csrc/gemm_mfma.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace pz;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);            \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

namespace w4 {
constexpr int BM = 256, BN = 256, BK = 64, NT = 256;
constexpr int A_BYTES = BM * BK * 2, SLOT = 2 * A_BYTES;  // A + B, 64 KiB
constexpr int PIECES = A_BYTES / 1024 / 4;                 // 1-KiB pieces per wave per operand (8)

PZ_DEV int swz(int row) { return (row >> 1) & 7; }  // BK 64: 128-B rows, 8 chunks

template <int SCHED>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) kern(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  int tm, tn, tile_id, slice;
  tile_coords(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
  const int m0 = tm * BM, n0 = tn * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), 0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.B), 0, -1, 0x00020000);
  // piece i of this wave: rows (wave*PIECES + i)*8 + lane/8, natural chunk lane%8 (global side),
  // swizzled chunk on the LDS side
  const int prow = lane >> 3, pch = lane & 7;
  const uint32_t va = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.lda) + pch * 8) * 2u;
  const uint32_t vb = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.ldb) + pch * 8) * 2u;
  // LDS byte offset of piece i: row r = (wave*PIECES+i)*8 + prow -> r*128 + ((pch ^ swz(r)) << 4);
  // swz(r) = ((wave*PIECES+i)*4 + prow/2) & 7 depends on i only through its parity
  uint32_t lo[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int r = (wave * PIECES + par) * 8 + prow;
    lo[par] = static_cast<uint32_t>(r * 128 + ((pch ^ swz(r)) << 4));
  }
  i32x4_t qa[PIECES], qb[PIECES];
  auto gload = [&](int kt) {
    const uint32_t k2 = static_cast<uint32_t>(kt * BK) * 2u;
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const uint32_t rowb = static_cast<uint32_t>(m0 + (wave * PIECES + i) * 8);
      qa[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                              ra, va, rowb * static_cast<uint32_t>(p.lda) * 2u + k2, 0));
    }
#pragma unroll
    for (int i = 0; i < PIECES; ++i) {
      const uint32_t rowb = static_cast<uint32_t>(n0 + (wave * PIECES + i) * 8);
      qb[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                              rb, vb, rowb * static_cast<uint32_t>(p.ldb) * 2u + k2, 0));
    }
  };
  auto lwrite = [&](int kt) {
    PZ_LDS char* base = smem + (kt & 1) * SLOT;
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      *reinterpret_cast<PZ_LDS i32x4_t*>(base + lo[i & 1] + (i & ~1) * 1024) = qa[i];
#pragma unroll
    for (int i = 0; i < PIECES; ++i)
      *reinterpret_cast<PZ_LDS i32x4_t*>(base + A_BYTES + lo[i & 1] + (i & ~1) * 1024) = qb[i];
  };
  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int nk = p.K / BK;
  if constexpr (SCHED >= 2) {
    // software-pipelined: phase 0 of step t issues the MFMAs of fragments F0 (t, k 0-31) while
    // reading F1 (t, k 32-63) and writing stage t+1 to the other slot; barrier; phase 1 issues
    // the MFMAs of F1 while reading F0 of step t+1 and loading stage t+2 into the staging
    // registers. Out-of-range stages are clamped (harmless extra traffic, no branches).
    auto rd = [&](int slot, int ks, i16x8_t (&fa)[8], i16x8_t (&fb)[8]) {
      const PZ_LDS char* ta = smem + slot * SLOT;
      const PZ_LDS char* tb = ta + A_BYTES;
#pragma unroll
      for (int j = 0; j < 8; ++j) fb[j] = frag_kc<64>(tb, wn * 128 + j * 16 + (lane & 15), (lane >> 4) + 4 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = frag_kc<64>(ta, wm * 128 + i * 16 + (lane & 15), (lane >> 4) + 4 * ks);
    };
    auto mm = [&](const i16x8_t (&fa)[8], const i16x8_t (&fb)[8]) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fb[j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[i]), acc[i][j], 0, 0, 0);
    };
    i16x8_t a0[8], b0[8], a1[8], b1[8];
    // hand-placed streams: 16 groups of {4 MFMAs, 1 fragment read, 1 staging op}, each group
    // fenced by sched_barrier so the compiler keeps the interleave
    auto frag = [&](int slot, int ks, int f) -> i16x8_t {
      const PZ_LDS char* ta = smem + slot * SLOT;
      if (f < 8) return frag_kc<64>(ta + A_BYTES, wn * 128 + f * 16 + (lane & 15), (lane >> 4) + 4 * ks);
      return frag_kc<64>(ta, wm * 128 + (f - 8) * 16 + (lane & 15), (lane >> 4) + 4 * ks);
    };
    auto mfma4 = [&](const i16x8_t (&fa)[8], const i16x8_t (&fb)[8], int g) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = g * 4 + q, i = idx >> 3, j = idx & 7;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fb[j]),
                                                            __builtin_bit_cast(bf16x8_t, fa[i]), acc[i][j], 0, 0, 0);
      }
    };
    auto wpiece = [&](int kt, int f) {
      PZ_LDS char* base = smem + (kt & 1) * SLOT + (f < 8 ? 0 : A_BYTES);
      const int i = f & 7;
      *reinterpret_cast<PZ_LDS i32x4_t*>(base + lo[i & 1] + (i & ~1) * 1024) = f < 8 ? qa[i] : qb[i];
    };
    auto gpiece = [&](int kt, int f) {
      const uint32_t k2 = static_cast<uint32_t>(kt * BK) * 2u;
      const int i = f & 7;
      if (f < 8) {
        const uint32_t rowb = static_cast<uint32_t>(m0 + (wave * PIECES + i) * 8);
        qa[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                ra, va, rowb * static_cast<uint32_t>(p.lda) * 2u + k2, 0));
      } else {
        const uint32_t rowb = static_cast<uint32_t>(n0 + (wave * PIECES + i) * 8);
        qb[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                rb, vb, rowb * static_cast<uint32_t>(p.ldb) * 2u + k2, 0));
      }
    };
    gload(0);
    lwrite(0);
    gload(min(1, nk - 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int f = 0; f < 16; ++f) (f < 8 ? b0[f] : a0[f - 8]) = frag(0, 0, f);
    auto mfma2 = [&](const i16x8_t (&fa)[8], const i16x8_t (&fb)[8], int h) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int idx = h * 2 + q, i = idx >> 3, j = idx & 7;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fb[j]),
                                                            __builtin_bit_cast(bf16x8_t, fa[i]), acc[i][j], 0, 0, 0);
      }
    };
    if constexpr (SCHED == 5) {  // stage t+2 loaded right behind the write of stage t+1 (a full step of latency)
      for (int t = 0; t < nk; ++t) {
        const int s = t & 1;
        const int kn = min(t + 2, nk - 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          mfma4(a0, b0, g);
          (g < 8 ? b1[g] : a1[g - 8]) = frag(s, 1, g);
          wpiece(t + 1, g);
          gpiece(kn, g);
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          mfma4(a1, b1, g);
          (g < 8 ? b0[g] : a0[g - 8]) = frag(s ^ 1, 0, g);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if constexpr (SCHED == 4) {  // finer: {2 MFMAs, 1 op} x 32 per phase, reads and staging alternating
      for (int t = 0; t < nk; ++t) {
        const int s = t & 1;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int h = 0; h < 32; ++h) {
          mfma2(a0, b0, h);
          if (h & 1) wpiece(t + 1, h >> 1);
          else (h < 16 ? b1[h >> 1] : a1[(h >> 1) - 8]) = frag(s, 1, h >> 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int kn = min(t + 2, nk - 1);
#pragma unroll
        for (int h = 0; h < 32; ++h) {
          mfma2(a1, b1, h);
          if (h & 1) gpiece(kn, h >> 1);
          else (h < 16 ? b0[h >> 1] : a0[(h >> 1) - 8]) = frag(s ^ 1, 0, h >> 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else
    for (int t = 0; t < nk; ++t) {
      const int s = t & 1;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        mfma4(a0, b0, g);
        (g < 8 ? b1[g] : a1[g - 8]) = frag(s, 1, g);
        if constexpr (SCHED == 3) {  // staging front-loaded: two pieces per group, first 8 groups
          if (g < 8) { wpiece(t + 1, 2 * g); wpiece(t + 1, 2 * g + 1); }
        } else {
          wpiece(t + 1, g);  // slot s^1 (at the last step: a harmless copy of the clamped stage)
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const int kn = min(t + 2, nk - 1);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        mfma4(a1, b1, g);
        (g < 8 ? b0[g] : a0[g - 8]) = frag(s ^ 1, 0, g);
        if constexpr (SCHED == 3) {
          if (g < 8) { gpiece(kn, 2 * g); gpiece(kn, 2 * g + 1); }
        } else {
          gpiece(kn, g);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
  gload(0);
  lwrite(0);
  if (nk > 1) gload(1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int t = 0; t < nk; ++t) {
    const PZ_LDS char* ta = smem + (t & 1) * SLOT;
    const PZ_LDS char* tb = ta + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      i16x8_t fa[8], fb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) fb[j] = frag_kc<64>(tb, wn * 128 + j * 16 + (lane & 15), (lane >> 4) + 4 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) fa[i] = frag_kc<64>(ta, wm * 128 + i * 16 + (lane & 15), (lane >> 4) + 4 * ks);
      if (ks == 1 && t + 1 < nk) lwrite(t + 1);  // slot (t+1)&1 was last read in step t-1
      if (ks == 1 && t + 2 < nk) gload(t + 2);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, fb[j]),
                                                              __builtin_bit_cast(bf16x8_t, fa[i]), acc[i][j], 0, 0, 0);
      if constexpr (SCHED == 1) {
        // interleave: 16 ds_read_b128 (next half's fragments are read up front, so only the
        // staging writes/loads remain to spread) among the 64 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  }
  uint16_t* C = static_cast<uint16_t*>(p.C);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wm * 128 + i * 16 + (lane & 15), n = n0 + wn * 128 + j * 16 + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha, acc[i][j][2] * p.alpha, acc[i][j][3] * p.alpha};
      store4<uint16_t>(C + static_cast<int64_t>(m) * p.ldc + n, v);
    }
}

template <int SCHED>
hipError_t launch(const GemmArgs& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern<SCHED>), hipFuncAttributeMaxDynamicSharedMemorySize,
                           2 * SLOT));
    set = true;
  }
  hipLaunchKernelGGL(kern<SCHED>, dim3((p.M / BM) * (p.N / BN)), dim3(NT), 2 * SLOT, s, p);
  return hipGetLastError();
}
// 32x32x16 form of the hand-placed pipe: half the MFMA instructions per FLOP (32-cycle MFMAs
// leave 24 free issue cycles each), groups of {2 MFMAs, 1 fragment read, 1 staging op}
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) kern32(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  int tm, tn, tile_id, slice;
  tile_coords(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
  const int m0 = tm * BM, n0 = tn * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), 0, -1, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.B), 0, -1, 0x00020000);
  const int prow = lane >> 3, pch = lane & 7;
  const uint32_t va = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.lda) + pch * 8) * 2u;
  const uint32_t vb = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.ldb) + pch * 8) * 2u;
  uint32_t lo[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int r = (wave * PIECES + par) * 8 + prow;
    lo[par] = static_cast<uint32_t>(r * 128 + ((pch ^ swz(r)) << 4));
  }
  i32x4_t qa[PIECES], qb[PIECES];
  auto wpiece = [&](int kt, int f) {
    PZ_LDS char* base = smem + (kt & 1) * SLOT + (f < 8 ? 0 : A_BYTES);
    const int i = f & 7;
    *reinterpret_cast<PZ_LDS i32x4_t*>(base + lo[i & 1] + (i & ~1) * 1024) = f < 8 ? qa[i] : qb[i];
  };
  auto gpiece = [&](int kt, int f) {
    const uint32_t k2 = static_cast<uint32_t>(kt * BK) * 2u;
    const int i = f & 7;
    if (f < 8) {
      const uint32_t rowb = static_cast<uint32_t>(m0 + (wave * PIECES + i) * 8);
      qa[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                              ra, va, rowb * static_cast<uint32_t>(p.lda) * 2u + k2, 0));
    } else {
      const uint32_t rowb = static_cast<uint32_t>(n0 + (wave * PIECES + i) * 8);
      qb[i] = __builtin_bit_cast(i32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                              rb, vb, rowb * static_cast<uint32_t>(p.ldb) * 2u + k2, 0));
    }
  };
  // fragment f of half ks: sub-step u = f >> 3 (k16 within the 32-deep half), tile q = f & 7
  // (q < 4: B tile q, else A tile q-4); lane: row l&31, k chunk (l>>5) + 2u + 4ks
  auto frag = [&](int slot, int ks, int f) -> i16x8_t {
    const PZ_LDS char* ta = smem + slot * SLOT;
    const int u = f >> 3, q = f & 7, ch = (lane >> 5) + 2 * u + 4 * ks;
    if (q < 4) return frag_kc<64>(ta + A_BYTES, wn * 128 + q * 32 + (lane & 31), ch);
    return frag_kc<64>(ta, wm * 128 + (q - 4) * 32 + (lane & 31), ch);
  };
  f32x16_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16_t{};
  // F[f]: 16 fragments per half
  auto mfma2 = [&](const i16x8_t (&F)[16], int h) {  // h in [0,16): sub-step h>>3, pair (h&7)
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int u = h >> 3, idx = (h & 7) * 2 + q, i = idx >> 2, j = idx & 3;
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, F[8 * u + j]),
                                                          __builtin_bit_cast(bf16x8_t, F[8 * u + 4 + i]), acc[i][j], 0, 0, 0);
    }
  };
  const int nk = p.K / BK;
  i16x8_t F0[16], F1[16];
#pragma unroll
  for (int f = 0; f < 16; ++f) gpiece(0, f);
#pragma unroll
  for (int f = 0; f < 16; ++f) wpiece(0, f);
#pragma unroll
  for (int f = 0; f < 16; ++f) gpiece(min(1, nk - 1), f);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) F0[f] = frag(0, 0, f);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    const int kn = min(t + 2, nk - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      mfma2(F0, h);
      F1[h] = frag(s, 1, h);
      wpiece(t + 1, h);
      gpiece(kn, h);
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      mfma2(F1, h);
      F0[h] = frag(s ^ 1, 0, h);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  uint16_t* C = static_cast<uint16_t*>(p.C);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // register quad g: columns 8g + 4(l>>5) + 0..3 of row l&31
        const int m = m0 + wm * 128 + i * 32 + (lane & 31), n = n0 + wn * 128 + j * 32 + 8 * g + 4 * (lane >> 5);
        float v[4] = {acc[i][j][4 * g] * p.alpha, acc[i][j][4 * g + 1] * p.alpha, acc[i][j][4 * g + 2] * p.alpha,
                      acc[i][j][4 * g + 3] * p.alpha};
        store4<uint16_t>(C + static_cast<int64_t>(m) * p.ldc + n, v);
      }
}

hipError_t launch32(const GemmArgs& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern32), hipFuncAttributeMaxDynamicSharedMemorySize, 2 * SLOT));
    set = true;
  }
  hipLaunchKernelGGL(kern32, dim3((p.M / BM) * (p.N / BN)), dim3(NT), 2 * SLOT, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// kdma<B0>: the schedule of hipBLASLt's gfx950 dX kernel (Custom_Cijk_Alik_Bljk_..._MT256x256x64,
// disassembled in round 6: profiles/r6_hipblaslt_kernels.txt) in HIP. 4 waves, 128x128 wave tiles
// (8x8 16x16x32 accumulators = 256 AGPRs), TWO LDS buffers of one 64-deep tile each, every
// operand k-half its own [256][32] slot (swz_kc<32>), filled by LDS-DMA. Fragments of BOTH
// k-halves of tile t are in registers before its second k-half's MFMAs start (sets S0 / S1), so
// buffer t&1 is free for tile t+2's DMAs half-way through iteration t — a prefetch distance of
// about one iteration with two buffers:
//   [B0: barrier, B0 = true]  phase 1: MFMAs S0 rows 0-3  + reads of S1        (+ k-half-0 DMAs)
//   B1: lgkmcnt(0) + barrier  phase 2: MFMAs S0 rows 4-7  + DMAs of tile t+2
//                             phase 3: MFMAs S1 rows 0-3  + DMAs of tile t+2
//   B2: vmcnt(tile t+1 landed) + barrier   phase 4: MFMAs S1 rows 4-7 + reads of S0 (tile t+1)
// B0 = true: a barrier at the top of the iteration certifies every wave's tile-t S0 reads done,
// so the k-half-0 slots take their DMAs already in phase 1 (16 DMAs over 96 MFMAs, not 64).
constexpr int HS = BM * 32 * 2;       // one operand k-half slot: 16 KiB
constexpr int TB = 4 * HS;            // one tile buffer: A kh0, A kh1, B kh0, B kh1 = 64 KiB

// D4: DMA pieces issued in phase 4 (the rest, 16 - D4, spread over phases 2-3); the loop body is
// branch-free — past the last tile the DMAs re-load tile nk-1 into the free buffer and the reads
// re-read the other buffer (harmless) — and every per-piece source offset is a precomputed scalar
template <int D4>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) kdma(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  int tm, tn, tile_id, slice;
  tile_coords(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
  const int m0 = tm * BM, n0 = tn * BN;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const i32x4_t rs_a = buf_rsrc(p.A), rs_b = buf_rsrc(p.B);
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz_kc<32>(prow);
  const uint32_t va = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.lda) + pch * 8) * 2u;
  const uint32_t vb = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.ldb) + pch * 8) * 2u;
  const uint32_t lds0 = lds_addr(smem);
  // per piece d: wave-uniform source byte offset at k = 0 and LDS destination in buffer 0
  uint32_t sbase[16], dbase[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const int sl = d >> 2, i = d & 3;
    const bool isb = sl >= 2;
    const uint32_t rbase = static_cast<uint32_t>((wave * 4 + i) * 16);
    const uint32_t ld = static_cast<uint32_t>(isb ? p.ldb : p.lda);
    sbase[d] = __builtin_amdgcn_readfirstlane(((static_cast<uint32_t>(isb ? n0 : m0) + rbase) * ld + (sl & 1) * 32) * 2u);
    dbase[d] = __builtin_amdgcn_readfirstlane(lds0 + static_cast<uint32_t>(sl * HS) + rbase * 64u);
  }
  const int nk = p.K / BK;
  auto dma = [&](int kt, int d) __attribute__((always_inline)) {
    kt = kt < nk ? kt : nk - 1;
    blds16<0>(d >= 8 ? rs_b : rs_a, d >= 8 ? vb : va, sbase[d] + static_cast<uint32_t>(kt) * (BK * 2),
              dbase[d] + static_cast<uint32_t>((kt & 1) * TB));
  };
  auto frag = [&](int buf, int kh, int f) __attribute__((always_inline)) -> i16x8_t {
    const PZ_LDS char* base = smem + buf * TB + (f < 8 ? 2 + kh : kh) * HS;
    const int row = (f < 8 ? wn : wm) * 128 + (f & 7) * 16 + (lane & 15);
    return frag_kc<32>(base, row, lane >> 4);
  };
  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mm = [&](const i16x8_t (&F)[16], int i, int j) __attribute__((always_inline)) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, F[j]),
                                                        __builtin_bit_cast(bf16x8_t, F[8 + i]), acc[i][j], 0, 0, 0);
  };
  i16x8_t S0[16], S1[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(0, d);
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(1, d);
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) S0[f] = frag(0, 0, f);
  constexpr int D23 = 16 - D4;  // pieces over phases 2-3 (64 MFMAs)
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    __builtin_amdgcn_sched_barrier(0);
    // phase 1: S0 rows 0-3 (32 MFMAs), the 16 S1 reads (1 per 2 MFMAs)
    static_for<16>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      mm(S0, g >> 2, 2 * (g & 3));
      mm(S0, g >> 2, 2 * (g & 3) + 1);
      S1[g] = frag(buf, 1, g);
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // phases 2-3: S0 rows 4-7, S1 rows 0-3 (64 MFMAs) + D23 DMA pieces of tile t+2 into buffer buf
    static_for<64>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if constexpr (c < 32) mm(S0, 4 + (c >> 3), c & 7);
      else mm(S1, (c - 32) >> 3, c & 7);
      constexpr int every = 64 / (D23 > 0 ? D23 : 1);
      if constexpr (D23 > 0 && c % every == every - 1 && c / every < D23) {
        dma(t + 2, c / every);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    // tile t+1 landed (the D23 pieces of tile t+2 just issued stay in flight)
    wait_vm<D23>();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // phase 4: S1 rows 4-7 (32 MFMAs) + the 16 S0 reads of tile t+1 (+ D4 DMA pieces)
    static_for<16>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      mm(S1, 4 + (g >> 2), 2 * (g & 3));
      mm(S1, 4 + (g >> 2), 2 * (g & 3) + 1);
      S0[g] = frag(buf ^ 1, 0, g);
      constexpr int every4 = 16 / (D4 > 0 ? D4 : 1);
      if constexpr (D4 > 0 && g % every4 == every4 - 1 && g / every4 < D4) dma(t + 2, D23 + g / every4);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  wait_vm<0>();  // no LDS-DMA may outlive the workgroup
  uint16_t* C = static_cast<uint16_t*>(p.C);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wm * 128 + i * 16 + (lane & 15), n = n0 + wn * 128 + j * 16 + 4 * (lane >> 4);
      float v[4] = {acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha, acc[i][j][2] * p.alpha, acc[i][j][3] * p.alpha};
      store4<uint16_t>(C + static_cast<int64_t>(m) * p.ldc + n, v);
    }
}

template <int D4>
hipError_t launch_dma(const GemmArgs& p, hipStream_t s) {
  static bool set = false;
  if (!set) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kdma<D4>), hipFuncAttributeMaxDynamicSharedMemorySize, 2 * TB));
    set = true;
  }
  if (p.M % BM || p.N % BN || p.K % BK || p.K < BK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kdma<D4>, dim3((p.M / BM) * (p.N / BN)), dim3(NT), 2 * TB, s, p);
  return hipGetLastError();
}

// kdmap<D4>: kdma made persistent — min(tiles, CUs) workgroups, workgroup r owns tiles r, r+G, ...
// and runs ONE k pipeline over all of them (global k step g = tile_i * nk + kt): the DMAs of the
// next tile's first two k steps go out during the current tile's last two, so only the epilogue
// (64 stores straight from the accumulators) separates two tiles — no prologue, no relaunch
// MODE (diagnostics): 0 = the GEMM, 1 = every tile reads tile (0, 0)'s operands (L2-resident loads),
// 2 = no DMAs at all (MFMA + LDS-read issue only; results are garbage); 3 = the GEMM with full
// 64-deep rows per slot ([256][64], swz_kc<64>: one DMA = 8 rows x 128 B, whole cache lines,
// instead of 16 rows x 64 B half-lines of the [256][32] k-half slots); diagnostics of the full
// layout: 4 = no swizzle at all (bank-conflicted reads), 5 = nt loads, 6 = natural-order global
// addresses with swizzled reads (timing only: the data lands permuted)
template <int D4, int MODE = 0>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(1, 1))) kdmap(const GemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / BM, tiles_n = p.N / BN, tiles = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int r = xcd_remap(blockIdx.x, G);
  const int T = (tiles - r + G - 1) / G;  // this workgroup's tile count (>= 1: G <= tiles)
  const int nk = p.K / BK;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const i32x4_t rs_a = buf_rsrc(p.A), rs_b = buf_rsrc(p.B);
  constexpr bool FULL = MODE >= 3, NOSWZ = MODE == 4, GNAT = MODE == 4 || MODE == 6;
  constexpr int POL = MODE == 5 ? 1 : 0;
  constexpr int RPD = FULL ? 8 : 16, CPR = FULL ? 8 : 4;  // rows per DMA, 16-B chunks per slot row
  const int prow = lane / CPR;
  // the chunk swizzle of row r (absolute in the slot) — for FULL it differs between even and odd
  // 8-row pieces ((r >> 1) & 4), hence two lane offsets per operand
  const int pch0 = (lane % CPR) ^ (GNAT ? 0 : FULL ? swz_kc<64>(prow) : swz_kc<32>(prow));
  const int pch1 = (lane % CPR) ^ (GNAT ? 0 : FULL ? swz_kc<64>(prow + 8) : swz_kc<32>(prow));
  const uint32_t va0 = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.lda) + pch0 * 8) * 2u;
  const uint32_t vb0 = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.ldb) + pch0 * 8) * 2u;
  const uint32_t va1 = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.lda) + pch1 * 8) * 2u;
  const uint32_t vb1 = (static_cast<uint32_t>(prow) * static_cast<uint32_t>(p.ldb) + pch1 * 8) * 2u;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t pofs[16], dbase[16];  // per piece: source byte offset within a tile at k = 0, LDS slot
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    if constexpr (FULL) {
      const int op = d >> 3, i = d & 7;
      const uint32_t rbase = static_cast<uint32_t>((wave * 8 + i) * RPD);
      const uint32_t ld = static_cast<uint32_t>(op ? p.ldb : p.lda);
      pofs[d] = __builtin_amdgcn_readfirstlane(rbase * ld * 2u);
      dbase[d] = __builtin_amdgcn_readfirstlane(lds0 + static_cast<uint32_t>(op * (TB / 2)) + rbase * 128u);
    } else {
      const int sl = d >> 2, i = d & 3;
      const uint32_t rbase = static_cast<uint32_t>((wave * 4 + i) * RPD);
      const uint32_t ld = static_cast<uint32_t>(sl >= 2 ? p.ldb : p.lda);
      pofs[d] = __builtin_amdgcn_readfirstlane((rbase * ld + (sl & 1) * 32) * 2u);
      dbase[d] = __builtin_amdgcn_readfirstlane(lds0 + static_cast<uint32_t>(sl * HS) + rbase * 64u);
    }
  }
  auto origin = [&](int i, int& m0, int& n0) __attribute__((always_inline)) {
    int tm, tn, tile_id, slice;
    tile_coords(r + i * G, tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // DMA cursor (k step dk of tile di; stays on the last step once there — re-loads are harmless)
  int dk = 0, di = 0;
  uint32_t abase, bbase;
  auto set_bases = [&]() __attribute__((always_inline)) {
    int m0, n0;
    origin(di, m0, n0);
    if constexpr (MODE == 1) m0 = n0 = 0;
    abase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m0) * static_cast<uint32_t>(p.lda) * 2u);
    bbase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(n0) * static_cast<uint32_t>(p.ldb) * 2u);
  };
  set_bases();
  auto dma = [&](int g, int d) __attribute__((always_inline)) {
    if constexpr (MODE == 2) return;
    const bool odd = FULL && (d & 1);
    blds16<POL>(d >= 8 ? rs_b : rs_a, d >= 8 ? (odd ? vb1 : vb0) : (odd ? va1 : va0),
              (d >= 8 ? bbase : abase) + pofs[d] + static_cast<uint32_t>(dk) * (BK * 2),
              dbase[d] + static_cast<uint32_t>((g & 1) * TB));
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (dk + 1 < nk) {
      ++dk;
    } else if (di + 1 < T) {
      dk = 0;
      ++di;
      set_bases();
    }
  };
  auto frag = [&](int buf, int kh, int f) __attribute__((always_inline)) -> i16x8_t {
    const int row = (f < 8 ? wn : wm) * 128 + (f & 7) * 16 + (lane & 15);
    if constexpr (NOSWZ)
      return *reinterpret_cast<const PZ_LDS i16x8_t*>(smem + buf * TB + (f < 8 ? TB / 2 : 0) + row * 128 +
                                                      (kh * 4 + (lane >> 4)) * 16);
    if constexpr (FULL) return frag_kc<64>(smem + buf * TB + (f < 8 ? TB / 2 : 0), row, kh * 4 + (lane >> 4));
    const PZ_LDS char* base = smem + buf * TB + (f < 8 ? 2 + kh : kh) * HS;
    return frag_kc<32>(base, row, lane >> 4);
  };
  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto mm = [&](const i16x8_t (&F)[16], int i, int j) __attribute__((always_inline)) {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, F[j]),
                                                        __builtin_bit_cast(bf16x8_t, F[8 + i]), acc[i][j], 0, 0, 0);
  };
  i16x8_t S0[16], S1[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(0, d);
  advance();
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(1, d);
  advance();
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) S0[f] = frag(0, 0, f);
  constexpr int D23 = 16 - D4;
  uint16_t* C = static_cast<uint16_t*>(p.C);
  int g = 0;  // global k step: buffer parity
  for (int ci = 0; ci < T; ++ci) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const int buf = g & 1;
      __builtin_amdgcn_sched_barrier(0);
      static_for<16>([&](auto gc) {
        constexpr int q = decltype(gc)::value;
        mm(S0, q >> 2, 2 * (q & 3));
        mm(S0, q >> 2, 2 * (q & 3) + 1);
        S1[q] = frag(buf, 1, q);
        __builtin_amdgcn_sched_barrier(0);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      static_for<64>([&](auto cc) {
        constexpr int c = decltype(cc)::value;
        if constexpr (c < 32) mm(S0, 4 + (c >> 3), c & 7);
        else mm(S1, (c - 32) >> 3, c & 7);
        constexpr int every = 64 / (D23 > 0 ? D23 : 1);
        if constexpr (D23 > 0 && c % every == every - 1 && c / every < D23) {
          dma(g, c / every);
          __builtin_amdgcn_sched_barrier(0);
        }
      });
      wait_vm<D23>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      static_for<16>([&](auto gc) {
        constexpr int q = decltype(gc)::value;
        mm(S1, 4 + (q >> 2), 2 * (q & 3));
        mm(S1, 4 + (q >> 2), 2 * (q & 3) + 1);
        S0[q] = frag(buf ^ 1, 0, q);
        constexpr int every4 = 16 / (D4 > 0 ? D4 : 1);
        if constexpr (D4 > 0 && q % every4 == every4 - 1 && q / every4 < D4) dma(g, D23 + q / every4);
        __builtin_amdgcn_sched_barrier(0);
      });
      advance();
    }
    // tile ci complete: store it straight from the accumulators
    int m0, n0;
    origin(ci, m0, n0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int m = m0 + wm * 128 + i * 16 + (lane & 15), n = n0 + wn * 128 + j * 16 + 4 * (lane >> 4);
        float v[4] = {acc[i][j][0] * p.alpha, acc[i][j][1] * p.alpha, acc[i][j][2] * p.alpha,
                      acc[i][j][3] * p.alpha};
        store4<uint16_t>(C + static_cast<int64_t>(m) * p.ldc + n, v);
      }
  }
  wait_vm<0>();  // no LDS-DMA may outlive the workgroup
}

template <int D4, int MODE = 0>
hipError_t launch_dmap(const GemmArgs& p, hipStream_t s) {
  static bool set = false;
  static int cus = 0;
  if (!set) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kdmap<D4, MODE>), hipFuncAttributeMaxDynamicSharedMemorySize, 2 * TB));
    int dev = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    set = true;
  }
  if (p.M % BM || p.N % BN || p.K % BK || p.K < BK) return hipErrorInvalidValue;
  const int tiles = (p.M / BM) * (p.N / BN);
  hipLaunchKernelGGL((kdmap<D4, MODE>), dim3(std::min(tiles, cus)), dim3(NT), 2 * TB, s, p);
  return hipGetLastError();
}
}  // namespace w4


__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(mix32(static_cast<uint32_t>(i) ^ seed) + static_cast<uint32_t>(i >> 32));
    p[i] = f2bf(static_cast<float>(h >> 8) * (2.f / 16777216.f) - 1.f);
  }
}

__global__ void ref_rows(const uint16_t* A, const uint16_t* B, float* R, int N, int K, int64_t lda, int64_t ldb,
                         int stride, int b_kc) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = static_cast<int64_t>(blockIdx.y) * stride;
  if (n >= N) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k)
    acc += bf2f(A[m * lda + k]) * bf2f(b_kc ? B[static_cast<int64_t>(n) * ldb + k] : B[static_cast<int64_t>(k) * ldb + n]);
  R[static_cast<int64_t>(blockIdx.y) * N + n] = acc;
}

typedef hipError_t (*LaunchFn)(const GemmArgs&, hipStream_t);

int main(int argc, char** argv) {
  struct V { const char* name; LaunchFn fn; };
  struct Case { const char* name; int M, N, K; bool b_kc; std::vector<V> vs; };
  // dX_*: B [N][K] (K-contiguous); fwd_*: B [K][N] (N-contiguous, the forward's weights). Earlier
  // variants (w4::launch_dma<D4>, launch_dmap<D4, MODE> diagnostics) stay instantiable here.
  const std::vector<V> dx = {{"lib_var30", launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 30>},
                             {"var40", launch_w4<EK_STORE, true>}, {"dmap4_full", w4::launch_dmap<4, 3>},
                             {"dmap8_nodma", w4::launch_dmap<8, 2>}};
  const std::vector<V> fw = {{"lib_var30", launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30>},
                             {"var41", launch_w4<EK_STORE, false>}};
  std::vector<Case> cases = {{"dX_L2", 8192, 4096, 4096, true, dx}, {"dX_L3", 8192, 4096, 1024, true, dx},
                             {"fwd_L2", 8192, 4096, 4096, false, fw}, {"fwd_L1", 8192, 4096, 1024, false, fw}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Case& c : cases) {
    const std::vector<V>& vs = c.vs;
    const int64_t na = int64_t(c.M) * c.K, nb = int64_t(c.N) * c.K, nc = int64_t(c.M) * c.N;
    uint16_t *A, *B, *C;
    float* R;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&B, nb * 2));
    CK(hipMalloc(&C, nc * 2));
    const int stride = 61, nref = (c.M + stride - 1) / stride;
    CK(hipMalloc(&R, int64_t(nref) * c.N * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, A, na, 12345u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, B, nb, 777u);
    const int64_t ldb = c.b_kc ? c.K : c.N;
    hipLaunchKernelGGL(ref_rows, dim3((c.N + 255) / 256, nref), dim3(256), 0, st, A, B, R, c.N, c.K, int64_t(c.K),
                       ldb, stride, int(c.b_kc));
    std::vector<float> ref(size_t(nref) * c.N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    GemmArgs p{};
    p.A = A; p.B = B; p.C = C;
    p.M = c.M; p.N = c.N; p.K = c.K;
    p.lda = c.K; p.ldb = ldb; p.ldc = c.N;
    p.a_kc = 1; p.b_kc = c.b_kc;
    p.in_dtype = DT_BF16; p.out_dtype = DT_BF16;
    p.alpha = 1.f; p.epi_mode = EPI_STORE; p.idx_ld = c.N; p.split_k = 1;
    const double flop = 2.0 * c.M * c.N * c.K;
    std::vector<std::vector<double>> tf(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipMemsetAsync(C, 0, nc * 2, st));
      CK(vs[v].fn(p, st));
      CK(hipStreamSynchronize(st));
      std::vector<uint16_t> out(nc);
      CK(hipMemcpy(out.data(), C, nc * 2, hipMemcpyDeviceToHost));
      double worst = 0.0;
      for (int r = 0; r < nref; ++r)
        for (int n = 0; n < c.N; ++n) {
          uint32_t u = uint32_t(out[size_t(r) * stride * c.N + n]) << 16;
          float got;
          memcpy(&got, &u, 4);
          const double want = ref[size_t(r) * c.N + n];
          worst = std::max(worst, fabs(got - want) / (fabs(want) * 0.01 + 0.05));
        }
      printf("%s %-10s check %s (worst err/tol %.3f)\n", c.name, vs[v].name, worst <= 1.0 ? "OK" : "FAIL", worst);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 5; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        for (int w = 0; w < 3; ++w) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 20; ++i) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tf[v].push_back(flop * 20 / (ms * 1e-3) / 1e12);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      auto t = tf[v];
      std::sort(t.begin(), t.end());
      printf("%s %-10s TF/s best %.1f median %.1f\n", c.name, vs[v].name, t.back(), t[t.size() / 2]);
    }
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R));
  }
  return 0;
}
