// VAR 40 — the dX GEMM (both operands K-contiguous) on 4-wave workgroups: the schedule of
// hipBLASLt's gfx950 dX kernel (Custom_Cijk_Alik_Bljk_..._MT256x256x64, disassembled in round 6:
// profiles/r6_hipblaslt_kernels.txt), written for this library's LDS-DMA and epilogues.
// Included by gemm_mfma.hip inside namespace pz::(anonymous).
//
//   * 256 x 256 tiles, 4 waves (one per SIMD), 128 x 128 per wave: 8 x 8 16x16x32 accumulators
//     = 256 AGPRs, mfma(B, A) so the Lay16 epilogue layout applies (gemm_epilogue.h).
//   * TWO 64-KiB LDS buffers, one 64-deep K step each ([256][64] A then [256][64] B, 128-B rows,
//     swz_kc<64>), filled by buffer_load ... lds: one DMA = 8 rows x 128 B (whole cache lines).
//   * Fragments of BOTH k-halves of step t are in registers before its second half's MFMAs (sets
//     S0 / S1), so buffer t&1 is free for step t+2's DMAs from the middle of iteration t on:
//       phase 1: MFMAs S0 rows 0-3 + the 16 S1 reads (step t)       B1: lgkmcnt(0) + barrier
//       phase 2-3: MFMAs S0 rows 4-7, S1 rows 0-3 + 12 DMAs (step t+2)
//       B2: vmcnt(12) (step t+1 landed) + barrier
//       phase 4: MFMAs S1 rows 4-7 + the 16 S0 reads (step t+1) + 4 DMAs (step t+2)
//     The last two iterations are compile-time copies without DMAs (no wasted loads, no per-DMA
//     branches: a per-piece guard inside the unrolled phases cost 11% in the lab).
//   * The 128 KiB of LDS then hold the epilogue's tile image (epilogue_lds: bias-free backward
//     kinds EK_BWD_MASK / EK_STORE, column sums, e5m2 copy — the library's own epilogue code).
// tools/gemm_w4_lab.hip (same box, plain store): dX [8192,4096] K=4096 1436 vs 1387 TF/s (VAR 30),
// K=1024 1095 vs 1040; the diagnostics there put the remaining gap to hipBLASLt (1569) in the
// DMA issue itself (no-DMA build 1690 TF/s; L2-resident operands: no change).
namespace w4cfg {
constexpr int kW4M = 256, kW4N = 256, kW4K = 64, kW4T = 256;
constexpr int kTB = kW4M * kW4K * 2 * 2;  // one K-step buffer: A + B, 64 KiB
constexpr int kD4 = 4;                  // DMA pieces issued in phase 4 (the other 12 in phases 2-3)
constexpr int kD23 = 16 - kD4;
}  // namespace w4cfg

// B_KC = false (instantiated by tools/gemm_w4_lab.hip only): B M/N-contiguous ([K][N], the
// forward's weights): its K-step slot is [64 k][256 n] (512-B rows, swz_mn), one DMA = 2 k-rows,
// fragments by transposing ds_read_b64_tr_b16 reads (frag_mn). Measured, not dispatched: fwd_L2
// 1,278 vs 1,286 TF/s (VAR 30), fwd_L1 926 vs 944, same box (profiles/r6_gemm_w4.txt)
template <int EK, bool B_KC = true>
__global__ void __launch_bounds__(w4cfg::kW4T) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_w4_kernel(const GemmArgs p) {
  using namespace w4cfg;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / kW4M, tiles_n = p.N / kW4N;
  int tm, tn, tile_id, slice;
  tile_coords(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
  const int m0 = tm * kW4M, n0 = tn * kW4N;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const i32x4_t rs_a = buf_rsrc(p.A), rs_b = buf_rsrc(p.B);
  // DMA lanes: row lane/8 of an 8-row piece, 16-B chunk lane%8; the chunk swizzle of slot row r is
  // (r >> 1) & 7, which for the piece's base row (a multiple of 8) differs between even and odd
  // pieces by 4 — hence two lane offsets per operand
  const int prow = lane >> 3;
  const int pch0 = (lane & 7) ^ swz_kc<64>(prow), pch1 = (lane & 7) ^ swz_kc<64>(prow + 8);
  const uint32_t lda = static_cast<uint32_t>(p.lda), ldb = static_cast<uint32_t>(p.ldb);
  const uint32_t va0 = (prow * lda + pch0 * 8) * 2u, va1 = (prow * lda + pch1 * 8) * 2u;
  // B lane offsets: K-contiguous as A; M/N-contiguous: k-row lane / 32 of a 2-row piece, 16-B column
  // chunk lane % 32 XOR swz_mn(k-row), whose bits 0-1 and 3 vary with the piece (4 classes)
  uint32_t vb[4];
  if constexpr (B_KC) {
    vb[0] = vb[2] = (prow * ldb + pch0 * 8) * 2u;
    vb[1] = vb[3] = (prow * ldb + pch1 * 8) * 2u;
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int kr = 2 * ((c & 1) + 4 * (c >> 1)) + (lane >> 5);  // a k-row of piece i = (c & 1) + 4 (c >> 1)
      vb[c] = ((lane >> 5) * ldb + (((lane & 31) ^ swz_mn(kr)) * 8)) * 2u;
    }
  }
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t abase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m0) * lda * 2u);
  const uint32_t bbase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(n0) * (B_KC ? ldb : 1u) * 2u);
  // K-step advance of a piece's source: 64 elements of a K-contiguous row, 64 rows of an
  // M/N-contiguous operand
  const uint32_t bstep = __builtin_amdgcn_readfirstlane(B_KC ? kW4K * 2u : kW4K * ldb * 2u);
  // piece d (16 per wave and K step): operand d / 8, 1 KiB at (wave * 8 + d % 8) KiB of the slot
  // (K-contiguous: rows 8 (wave * 8 + d % 8) .. + 8; M/N-contiguous B: k-rows 2 (wave * 8 + d % 8) .. + 2)
  uint32_t soff[16], dst[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const int op = d >> 3;
    const uint32_t piece = static_cast<uint32_t>(wave * 8 + (d & 7));
    if (op == 0 || B_KC)
      soff[d] = __builtin_amdgcn_readfirstlane((op ? bbase : abase) + piece * 8u * (op ? ldb : lda) * 2u);
    else
      soff[d] = __builtin_amdgcn_readfirstlane(bbase + piece * 2u * ldb * 2u);
    dst[d] = __builtin_amdgcn_readfirstlane(lds0 + static_cast<uint32_t>(op * (kTB / 2)) + piece * 1024u);
  }
  auto dma = [&](int kt, int d) __attribute__((always_inline)) {
    const int i = d & 7;
    if (d < 8)
      blds16<0>(rs_a, (i & 1) ? va1 : va0, soff[d] + static_cast<uint32_t>(kt) * (kW4K * 2),
                dst[d] + static_cast<uint32_t>((kt & 1) * kTB));
    else
      blds16<0>(rs_b, vb[(i & 1) + 2 * (i >> 2)], soff[d] + static_cast<uint32_t>(kt) * bstep,
                dst[d] + static_cast<uint32_t>((kt & 1) * kTB));
  };
  // fragment f of k-half kh: f < 8 -> B (output columns), else A (output rows)
  auto frag = [&](int buf, int kh, int f) __attribute__((always_inline)) -> i16x8_t {
    if constexpr (!B_KC) {
      if (f < 8) return frag_mn<kW4N>(smem + buf * kTB + kTB / 2, wn * 128 + f * 16, 8 * (lane >> 4) + 32 * kh, lane);
    }
    const int row = (f < 8 ? wn : wm) * 128 + (f & 7) * 16 + (lane & 15);
    return frag_kc<64>(smem + buf * kTB + (f < 8 ? kTB / 2 : 0), row, kh * 4 + (lane >> 4));
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
  const int nk = p.K / kW4K;  // >= 2 (w4_eligible)
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(0, d);
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(1, d);
  wait_vm<16>();
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 16; ++f) S0[f] = frag(0, 0, f);

  // one K step; DMA: step kt+2 goes out (kt + 2 < nk); NEXT: step kt+1's S0 is read in phase 4
  auto step = [&](int kt, auto dmac, auto nextc) __attribute__((always_inline)) {
    constexpr bool DMA = decltype(dmac)::value, NEXT = decltype(nextc)::value;
    const int buf = kt & 1;
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
    __builtin_amdgcn_s_barrier();  // every wave has both k-halves of step kt: buffer buf is free
    __builtin_amdgcn_sched_barrier(0);
    static_for<64>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if constexpr (c < 32) mm(S0, 4 + (c >> 3), c & 7);
      else mm(S1, (c - 32) >> 3, c & 7);
      constexpr int every = 64 / kD23;
      if constexpr (DMA && c % every == every - 1 && c / every < kD23) {
        dma(kt + 2, c / every);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    if constexpr (NEXT) {
      if constexpr (DMA) wait_vm<kD23>();  // step kt+1 landed; step kt+2's pieces stay in flight
      else wait_vm<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    static_for<16>([&](auto gc) {
      constexpr int q = decltype(gc)::value;
      mm(S1, 4 + (q >> 2), 2 * (q & 3));
      mm(S1, 4 + (q >> 2), 2 * (q & 3) + 1);
      if constexpr (NEXT) S0[q] = frag(buf ^ 1, 0, q);
      constexpr int every4 = 16 / kD4;
      if constexpr (DMA && q % every4 == every4 - 1) dma(kt + 2, kD23 + q / every4);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int kt = 0;
  for (; kt < nk - 2; ++kt) step(kt, T_{}, T_{});
  step(kt, F_{}, T_{});
  step(kt + 1, F_{}, F_{});
  PZ_STAMP(3);
  // (epilogue_lds opens with a barrier: every wave is done with the operand buffers)
  epilogue_lds<kW4M, kW4N, 2, 2, Lay16<8, 8>, false, EK>(p, acc, smem, m0, n0, wm, wn, lane, p.alpha);
}

// dX-layout bf16 GEMMs VAR 40 takes: whole 256 x 256 tiles that fill the CUs, >= 2 K steps, no
// split-K, buffer-addressable operands, a backward-mask or plain-store epilogue
inline bool w4_eligible(const GemmArgs& p, int ek) {
  if (!p.a_kc || !p.b_kc || p.in_dtype != DT_BF16 || p.out_dtype != DT_BF16 || p.accumulate) return false;
  if (p.split_k > 1 || p.M % 256 || p.N % 256 || p.K % 64 || p.K < 128) return false;
  if (ek != EK_BWD_MASK && ek != EK_STORE) return false;
  if ((p.M / 256) * (p.N / 256) < 240) return false;
  constexpr int64_t kLim = int64_t(1) << 32;
  return static_cast<int64_t>(p.M) * p.lda * 2 < kLim && static_cast<int64_t>(p.N) * p.ldb * 2 < kLim;
}

template <int EK, bool B_KC = true>
hipError_t launch_w4(const GemmArgs& p, hipStream_t s) {
  auto kern = gemm_w4_kernel<EK, B_KC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       2 * w4cfg::kTB);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((p.M / w4cfg::kW4M) * (p.N / w4cfg::kW4N)), dim3(w4cfg::kW4T), 2 * w4cfg::kTB, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// VAR 42 / 43 — the same schedule for the fp8 policy's dX / forward GEMMs. Lab (tools/gemm_w4f8_lab.hip,
// plain store, same box, TF/s median): dX [8192,8192] K=1024 1,584 vs 1,341 (VAR 17), [8192,4096]
// K=4096 2,479 vs 1,743; forward [8192,4096] K=4096 2,464 vs 2,262 (VAR 15), [8192,8192] K=1024
// 1,602 vs 1,598 (VAR 16). VAR 42 = the dX GEMM (e5m2 dZ x e4m3 W, both K-contiguous) on
// v_mfma_scale_f32_32x32x64_f8f6f4 (unit E8M0 block scales; the per-tensor dequant scales go into
// the epilogue's alpha). A 128-byte K step of fp8 is the bf16 kernel's slot geometry ([256][128 B],
// swz_kc<64>, the same DMA pieces); each 64-byte k-half is ONE 32x32x64 MFMA per 32x32 tile:
// 4 x 4 tiles per wave (f32x16 accumulators = 256 AGPRs), 16 MFMAs per k-half of 64 cycles each —
// the bf16 kernel's 64 x 16 cycles — so the phases, DMA spread and barriers carry over unchanged.
// B_KC = false (VAR 43): the fp8 forward X8 (e4m3, K-contiguous) x W8 (e4m3 [in, out], N-contiguous):
// B's K-step slot is [128 k][256 B] (one DMA = 4 k-rows, swz_mn8<256>), read per 64-k half with the
// transposing ds_read_b64_tr_b8 (frag_mn8) — the same natural-layout weight copy VAR 15 / 16 read
template <int EK, bool B_KC = true>
__global__ void __launch_bounds__(w4cfg::kW4T) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm_w4f8_kernel(const GemmArgs p) {
  using namespace w4cfg;
  constexpr int kStep = 128;  // K bytes (= fp8 elements) per K step
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);
  const int tiles_m = p.M / kW4M, tiles_n = p.N / kW4N;
  int tm, tn, tile_id, slice;
  tile_coords(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, 1, tm, tn, tile_id, slice);
  const int m0 = tm * kW4M, n0 = tn * kW4N;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const i32x4_t rs_a = buf_rsrc(p.A), rs_b = buf_rsrc(p.B);
  const int prow = lane >> 3;
  const int pch0 = (lane & 7) ^ swz_kc<64>(prow), pch1 = (lane & 7) ^ swz_kc<64>(prow + 8);
  const uint32_t lda = static_cast<uint32_t>(p.lda), ldb = static_cast<uint32_t>(p.ldb);  // bytes
  const uint32_t va0 = prow * lda + pch0 * 16, va1 = prow * lda + pch1 * 16;
  // B lane offsets: K-contiguous as A; N-contiguous: k-row lane / 16 of a 4-row piece, 16-B chunk
  // lane % 16 XOR ((k-row & 7) << 1), whose k-row bits vary with the piece's parity
  uint32_t vb0, vb1;
  if constexpr (B_KC) {
    vb0 = prow * ldb + pch0 * 16;
    vb1 = prow * ldb + pch1 * 16;
  } else {
    const int kq = lane >> 4;
    vb0 = kq * ldb + ((lane & 15) ^ (((0 + kq) & 7) << 1)) * 16;
    vb1 = kq * ldb + ((lane & 15) ^ (((4 + kq) & 7) << 1)) * 16;
  }
  const uint32_t lds0 = lds_addr(smem);
  const uint32_t abase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m0) * lda);
  const uint32_t bbase = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(n0) * (B_KC ? ldb : 1u));
  const uint32_t bstep = __builtin_amdgcn_readfirstlane(B_KC ? static_cast<uint32_t>(kStep) : kStep * ldb);
  uint32_t soff[16], dst[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) {
    const int op = d >> 3;
    const uint32_t piece = static_cast<uint32_t>(wave * 8 + (d & 7));
    if (op == 0 || B_KC)
      soff[d] = __builtin_amdgcn_readfirstlane((op ? bbase : abase) + piece * 8u * (op ? ldb : lda));
    else
      soff[d] = __builtin_amdgcn_readfirstlane(bbase + piece * 4u * ldb);
    dst[d] = __builtin_amdgcn_readfirstlane(lds0 + static_cast<uint32_t>(op * (kTB / 2)) + piece * 1024u);
  }
  auto dma = [&](int kt, int d) __attribute__((always_inline)) {
    const bool odd = d & 1;
    if (d < 8)
      blds16<0>(rs_a, odd ? va1 : va0, soff[d] + static_cast<uint32_t>(kt) * kStep,
                dst[d] + static_cast<uint32_t>((kt & 1) * kTB));
    else
      blds16<0>(rs_b, odd ? vb1 : vb0, soff[d] + static_cast<uint32_t>(kt) * bstep,
                dst[d] + static_cast<uint32_t>((kt & 1) * kTB));
  };
  // fragment f of k-half kh: f < 4 -> B (32 output columns each), else A (32 output rows); lane l
  // holds row l & 31, k bytes [32 (l >> 5), +32) of the half = 16-B chunks 4 kh + 2 (l >> 5) + {0, 1}
  auto frag = [&](int buf, int kh, int f) __attribute__((always_inline)) -> i32x8_t {
    const PZ_LDS char* t = smem + buf * kTB + (f < 4 ? kTB / 2 : 0);
    if constexpr (!B_KC) {  // the half's [64 k][256 B] image, transposing 8-bit reads
      if (f < 4) return frag_mn8<kW4N>(t + kh * 64 * kW4N, wn * 128 + f * 32, lane);
    }
    const int row = (f < 4 ? wn : wm) * 128 + (f & 3) * 32 + (lane & 31);
    const int c = 4 * kh + 2 * (lane >> 5);
    return cat_frag(frag_kc<64>(t, row, c), frag_kc<64>(t, row, c + 1));
  };
  f32x16_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16_t{};
  auto mm = [&](const i32x8_t (&F)[8], int i, int j) __attribute__((always_inline)) {
    // issued as mfma(B, A): cbsz = B's format (e4m3 = 0), blgp = A's (e5m2 = 1 in the backward,
    // e4m3 = 0 in the forward); E8M0 127 = 1.0
    acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(F[j], F[4 + i], acc[i][j], 0, B_KC ? 1 : 0, 0, 127,
                                                                 0, 127);
  };
  i32x8_t S0[8], S1[8];
  const int nk = p.K / kStep;  // >= 2 (w4f8_eligible)
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(0, d);
#pragma unroll
  for (int d = 0; d < 16; ++d) dma(1, d);
  wait_vm<16>();
  __syncthreads();
#pragma unroll
  for (int f = 0; f < 8; ++f) S0[f] = frag(0, 0, f);

  auto step = [&](int kt, auto dmac, auto nextc) __attribute__((always_inline)) {
    constexpr bool DMA = decltype(dmac)::value, NEXT = decltype(nextc)::value;
    const int buf = kt & 1;
    __builtin_amdgcn_sched_barrier(0);
    // phase 1: S0 rows 0-1 (8 MFMAs) + the 8 S1 reads (step kt, second k-half)
    static_for<8>([&](auto gc) {
      constexpr int q = decltype(gc)::value;
      mm(S0, q >> 2, q & 3);
      S1[q] = frag(buf, 1, q);
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // every wave has both k-halves of step kt: buffer buf is free
    __builtin_amdgcn_sched_barrier(0);
    // phases 2-3: S0 rows 2-3, S1 rows 0-1 (16 MFMAs) + 12 DMAs of step kt+2
    static_for<16>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if constexpr (c < 8) mm(S0, 2 + (c >> 2), c & 3);
      else mm(S1, (c - 8) >> 2, c & 3);
      if constexpr (DMA && c < kD23) {
        dma(kt + 2, c);
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    if constexpr (NEXT) {
      if constexpr (DMA) wait_vm<kD23>();
      else wait_vm<0>();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    // phase 4: S1 rows 2-3 (8 MFMAs) + the 8 S0 reads of step kt+1 + 4 DMAs
    static_for<8>([&](auto gc) {
      constexpr int q = decltype(gc)::value;
      mm(S1, 2 + (q >> 2), q & 3);
      if constexpr (NEXT) S0[q] = frag(buf ^ 1, 0, q);
      if constexpr (DMA && (q & 1)) dma(kt + 2, kD23 + (q >> 1));
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int kt = 0;
  for (; kt < nk - 2; ++kt) step(kt, T_{}, T_{});
  step(kt, F_{}, T_{});
  step(kt + 1, F_{}, F_{});
  const float alpha = p.alpha * (p.scale_a != nullptr ? *p.scale_a : 1.f) * (p.scale_b != nullptr ? *p.scale_b : 1.f);
  epilogue_lds<kW4M, kW4N, 2, 2, Lay32<4, 4>, !B_KC, EK>(p, acc, smem, m0, n0, wm, wn, lane, alpha);
}

// the fp8 policy's dX GEMMs VAR 42 takes (e5m2 x e4m3, both K-contiguous): whole 256 x 256 tiles
// that fill the CUs, >= 2 K steps of 128 bytes, no split-K, buffer-addressable operands
inline bool w4f8_eligible(const GemmArgs& p, int ek) {
  if (!p.a_kc || !p.b_kc || p.in_dtype != DT_FP8 || p.a_fmt != 1 || p.b_fmt != 0 || p.out_dtype != DT_BF16 ||
      p.accumulate)
    return false;
  if (p.split_k > 1 || p.M % 256 || p.N % 256 || p.K % 128 || p.K < 256) return false;
  if (ek != EK_BWD_MASK && ek != EK_ANY && ek != EK_STORE) return false;
  if ((p.M / 256) * (p.N / 256) < 240) return false;
  constexpr int64_t kLim = int64_t(1) << 32;
  return static_cast<int64_t>(p.M) * p.lda < kLim && static_cast<int64_t>(p.N) * p.ldb < kLim;
}

// the fp8 forward GEMMs VAR 43 takes (e4m3 x e4m3 [in, out] weights): same shape conditions
inline bool w4f8_fwd_eligible(const GemmArgs& p, int ek) {
  if (!p.a_kc || p.b_kc || p.in_dtype != DT_FP8 || p.a_fmt != 0 || p.b_fmt != 0 || p.out_dtype != DT_BF16 ||
      p.accumulate || p.epi_mode == EPI_BWD)
    return false;
  if (p.split_k > 1 || p.M % 256 || p.N % 256 || p.K % 128 || p.K < 256) return false;
  if (!ek_fixed(ek) && ek != EK_RELU && ek != EK_STORE) return false;
  if ((p.M / 256) * (p.N / 256) < 240) return false;
  constexpr int64_t kLim = int64_t(1) << 32;
  return static_cast<int64_t>(p.M) * p.lda < kLim && static_cast<int64_t>(p.K) * p.ldb < kLim;
}

template <int EK, bool B_KC = true>
hipError_t launch_w4f8(const GemmArgs& p, hipStream_t s) {
  auto kern = gemm_w4f8_kernel<EK, B_KC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       2 * w4cfg::kTB);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((p.M / w4cfg::kW4M) * (p.N / w4cfg::kW4N)), dim3(w4cfg::kW4T), 2 * w4cfg::kTB, s, p);
  return hipGetLastError();
}
