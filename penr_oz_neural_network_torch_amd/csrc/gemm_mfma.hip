// N1 — bf16 MFMA GEMM for gfx950 with fused MLP epilogues.
//
// Replaces the reference's three per-layer matmuls (neural_net_model.py:117 forward `x @ W`, and
// autograd's two `mm` for dX / dW) plus the bias add (:119), activation (:172-184), dropout (:395)
// and bias-gradient column sum that surround them.
//
// Design (CDNA4-first, /opt/skills/guides/cdna_hip_programming.md §5):
//  * 16x16x32 bf16 MFMA (v_mfma_f32_16x16x32_bf16), fp32 accumulation. Operands are issued
//    SWAPPED (mfma(B, A)) so each lane owns 4 consecutive output COLUMNS of one row: the epilogue
//    loads bias / aux and stores C with 8-16 B per lane.
//  * Both operand layouts are first-class. A K-contiguous operand is staged as [rows][32 k]
//    (64-B rows, 16-B chunks XOR-swizzled per 4-row group, read with ds_read_b128); an
//    M/N-contiguous operand (the reference's [in,out] weights in the forward, activations in
//    dW = XᵀdZ) is staged as [32 k][rows] and read with the gfx950 transposing
//    ds_read_b64_tr_b16 — no transpose kernels, no second weight copy.
//  * global->LDS by global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction; swizzle on the
//    per-lane SOURCE address + the read, rule 21).
//  * Pipeline: a ring of NS = 4 LDS slots, each one 32-deep K step. Loads run NS-1 steps
//    ahead; each step waits with a COUNTED `s_waitcnt vmcnt((NS-2)G)` (G = LDS-DMA instructions per
//    wave per step) so the NS-2 younger steps stay in flight across the raw `s_barrier` — never a
//    vmcnt(0) drain in the loop (guide "Pipelining across barriers", T3/T4). One barrier per step
//    covers both hazards: RAW (every wave's DMA for slot t landed) and WAR (every wave's reads of
//    slot t-1, which the step re-fills, completed: lgkmcnt(0) before the barrier).
//  * MFMA clusters bracketed by s_setprio(1)/(0) (T5).
//  * XCD-aware bijective block remap (T1) + grouped tile order for L2 reuse.
//  * Tile configs 256x256 (8 waves), 256x128 (8 waves), 128x128 (4 waves, 2 blocks/CU), chosen
//    per shape so the grid covers the 256 CUs.
#include <cstdlib>
#include <type_traits>

#include "pz_common.h"
#include "pz_launch.h"

namespace pz {
namespace {

constexpr int kBK = 32;  // K depth of one ring slot (BK64 variants: two of these per slot)

#include "gemm_common.h"  // LDS-DMA, swizzles, fragment reads, tile order (shared with gemm_sk.hip)

// Main-loop variants (template VAR). The library instantiates 0 (flat DMA, ragged > 4 GiB
// operands), 6 (buffer DMA, 32-deep ring), 30 (buffer DMA, 64-deep 2-slot ring, the default),
// 8 / 9 (fp8 e4m3 / e5m2 x e4m3), 10 / 11 (their buffer-DMA forms, PZ_GEMM_F8BUF=1) and 12 / 13
// (fp8 on the 64-deep buffer-DMA ring: 128 K-bytes per slot, two MFMA K-steps). The
// rest are tools/gemm_lab probes whose measurements are in profiles/: 1 / 2 / 3 (no MFMA / no
// DMA / no fragment reads), 4 (no deferred wait), 5 / 23 (3- / 5-slot rings), 20 / 21 / 31
// (64-deep ring with flat DMA / split staging), 24 (L2 prefetch), 25 (buffer DMA for M/N-
// contiguous operands only), 27-29 (cache policies), 41 (32x32x16 MFMA).
// Per-variant ring geometry: VAR 20/21/30/31 stage 64-deep K steps into two 64 KiB slots (one
// MFMA interval = 64 MFMAs per wave, half the barriers per FLOP of the 32-deep ring)
template <int VAR> constexpr int var_bk() {
  return (VAR == 20 || VAR == 21 || VAR == 30 || VAR == 31 || VAR == 32 || VAR == 33 || VAR == 12 || VAR == 13) ? 64 : 32;
}
template <int VAR> constexpr int var_ns() {
  return (VAR == 5 || VAR == 7 || VAR == 16 || VAR == 17) ? 3 : VAR == 23 ? 5 : (var_bk<VAR>() == 64 ? 2 : 4);
}
// VAR 7: buffer DMA on a 3-slot 32-deep ring, for 4-wave 256x128 tiles that run TWO workgroups
// per CU (72 KiB of LDS and <= 256 VGPRs each): one workgroup's epilogue overlaps the other's
// main loop (the hardware interleaves the two instead of a barrier-phased ping-pong)
// VAR 16 / 17: the fp8 forward (VAR 15) / e5m2 x e4m3 dX (VAR 9) the same way — 4-wave 256x128
// tiles, 3-slot ring (72 KiB), two workgroups per CU: at K = 1024 an fp8 tile's epilogue (the
// stage math, the e4m3 / e5m2 copies, the bitmask) costs about what its main loop does, and the
// other workgroup's MFMAs run through it
template <int VAR> constexpr int var_waves_per_eu() { return (VAR == 7 || VAR == 16 || VAR == 17) ? 2 : 1; }


template <int BM, int BN, int WM, int WN, int NS_ = 4, int BK_ = 32>
struct Cfg {
  static constexpr int BK = BK_;
  // ring depth in 32-deep K slots. Measured on the step's GEMMs: 5 slots for 256x256 (160 KiB)
  // and 6 for 256x128 are 2-4% SLOWER than 4 (the DMA stream is throughput-, not latency-bound),
  // and 5 slots for 128x128 drop it to one workgroup per CU (-20%).
  static constexpr int NS = NS_;
  static constexpr int NW = WM * WN;
  static constexpr int NT = NW * 64;
  static constexpr int WTM = BM / WM;
  static constexpr int WTN = BN / WN;
  static constexpr int TM = WTM / 16;
  static constexpr int TN = WTN / 16;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int SLOT_BYTES = A_BYTES + B_BYTES;
  static constexpr int LDS_BYTES = NS * SLOT_BYTES + 256;  // + L2-prefetch sink (VAR 24)
  static constexpr int GA = A_BYTES / 1024 / NW;  // LDS-DMA instructions per wave per slot
  static constexpr int GB = B_BYTES / 1024 / NW;
  static constexpr int G = GA + GB;
  static_assert(TM >= 1 && TN >= 1, "wave tile must hold at least one 16x16 MFMA tile");
  static_assert(GA >= 1 && GB >= 1 && GA * 1024 * NW == A_BYTES && GB * 1024 * NW == B_BYTES, "stage split");
  static_assert(LDS_BYTES <= 160 * 1024 + 256, "LDS budget");
};


template <int RB, int NW, int KROWS>
PZ_DEV void stage_mn8(int64_t ld16, int col0, int k0, PZ_LDS char* tile, int wave, int lane, i32x4_t rs) {
  constexpr int CHUNKS = RB / 16;
  constexpr int ROWS_PER = 1024 / RB;
  constexpr int INSTR = (KROWS * RB) / (1024 * NW);
  static_assert(INSTR >= 1 && INSTR * 1024 * NW == KROWS * RB, "fp8 M/N-contiguous stage split");
#pragma unroll
  for (int i = 0; i < INSTR; ++i) {
    const int kbase = (wave * INSTR + i) * ROWS_PER;
    const int kr = kbase + lane / CHUNKS;
    const int chunk = (lane % CHUNKS) ^ swz_mn8<RB>(kr);
    const uint32_t voff = (static_cast<uint32_t>(kr) * static_cast<uint32_t>(ld16)) * 2u +
                          static_cast<uint32_t>(col0 + chunk * 16);
    blds16<0>(rs, voff, __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(k0) * static_cast<uint32_t>(ld16) * 2u),
              lds_addr(tile + kbase * RB));
  }
}


// fp32-output store epilogue (dW / plain GEMMs): alpha, bias, optional accumulate, 16-B stores.
// The fused stage epilogues only exist for bf16 outputs (epilogue_lds); mfma_eligible routes
// anything else to the generic kernel.
template <typename OutT, typename AuxT>
PZ_DEV f32x4_t epi_apply(const GemmArgs& p, f32x4_t a, f32x4_t bias4, int m, int n, OutT* __restrict__ Cp,
                         const AuxT* __restrict__ aux) {
  (void)aux;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = a[r] * p.alpha + bias4[r];
  OutT* dst = Cp + static_cast<int64_t>(m) * p.ldc + n;
  if (p.accumulate) {
    float old[4];
    load4<OutT>(dst, old);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += old[r];
  }
  store4<OutT>(dst, v);
  return f32x4_t{v[0], v[1], v[2], v[3]};
}


#include "gemm_epilogue.h"

// EPI_OPT: the tile's accumulators are a block of the weight gradient g = alpha*AB; instead of
// storing it (and a separate optimizer pass reading it back), apply the optimizer update of the
// weight right here (GemmOpt). Each lane owns 4 consecutive columns of one row per fragment
// (acc[i][j]: m = lane & 15, n = 4*(lane >> 4)), so p / m / v move as 16-B vectors like the fp32
// C store they replace. The per-tile statistics (update-ratio sums, sum(w^2), amax) are reduced
// in LDS and leave as one atomic per accumulator.
template <class C, class Acc>
PZ_DEV void epilogue_opt(const GemmArgs& p, Acc& acc, PZ_LDS char* smem, int m0, int n0, int wm, int wn, int lane) {
  const GemmOpt& o = p.opt;
  float lr = o.lr, bc1 = o.bias_c1, bc2s = o.bias_c2_sqrt;
  int epoch = -1;
  if (o.epoch_ptr != nullptr) epoch = *o.epoch_ptr;
  if (o.hp != nullptr) {  // graph-replayed step: this epoch's hyper-parameters
    const double* h = o.hp + 4 * static_cast<int64_t>(epoch);
    lr = static_cast<float>(h[0]);
    bc1 = static_cast<float>(h[1]);
    bc2s = static_cast<float>(h[2]);
  }
  const bool full = o.stats_every == 1 || (o.stats_every > 1 && (epoch < 0 || epoch % o.stats_every == 0));
  const float step_size = lr / bc1;
  const bool adam = o.adam != 0;
  const int g4 = 4 * (lane >> 4);
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  float am = 0.f;
  static_for<C::TN>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int n = n0 + wn * C::WTN + j * 16 + g4;
    static_for<C::TM>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int m = m0 + wm * C::WTM + i * 16 + (lane & 15);
      if (n < p.N && m < p.M) {
        const int64_t gi = static_cast<int64_t>(m) * p.ldc + n;
        const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(o.params + gi);
        f32x4_t mm = {0.f, 0.f, 0.f, 0.f}, vv = mm, p1;
        if (adam) {
          mm = *reinterpret_cast<const f32x4_t*>(o.exp_avg + gi);
          vv = *reinterpret_cast<const f32x4_t*>(o.exp_avg_sq + gi);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float graw = acc[i][j][r] * p.alpha;
          float mr = mm[r], vr = vv[r];
          p1[r] = adam ? opt_update<true>(p0[r], graw, o.grad_scale, o.l2x2, lr, step_size, o.beta1, o.beta2, bc2s,
                                          o.eps, mr, vr)
                       : opt_update<false>(p0[r], graw, o.grad_scale, o.l2x2, lr, step_size, 0.f, 0.f, 1.f, 0.f, mr,
                                           vr);
          mm[r] = mr;
          vv[r] = vr;
        }
        if (adam) {
          *reinterpret_cast<f32x4_t*>(o.exp_avg + gi) = mm;
          *reinterpret_cast<f32x4_t*>(o.exp_avg_sq + gi) = vv;
        }
        *reinterpret_cast<f32x4_t*>(o.params + gi) = p1;
        if (o.shadow != nullptr) {
          if (o.shadow_dtype == DT_BF16)
            *reinterpret_cast<u32x2_t*>(static_cast<uint16_t*>(o.shadow) + gi) =
                u32x2_t{pack_bf2(p1[0], p1[1]), pack_bf2(p1[2], p1[3])};
          else
            *reinterpret_cast<f32x4_t*>(static_cast<float*>(o.shadow) + gi) = p1;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st[3] += static_cast<double>(p1[r]) * p1[r];
          if (full) {
            const double d = static_cast<double>(p1[r] - p0[r]);
            st[0] += d;
            st[1] += d * d;
            st[2] += p1[r];
          }
          am = fmaxf(am, fabsf(p1[r]));
        }
      }
    });
  });
  const bool want_st = o.stats != nullptr, want_am = o.amax != nullptr;
  if (!want_st && !want_am) return;
  constexpr int NW = C::NT / 64;
#pragma unroll
  for (int k = 0; k < 4; ++k) st[k] = wave_sum_d(st[k]);
  am = wave_max(am);
  __syncthreads();  // every wave is past its last ring read: the LDS is free
  PZ_LDS double* part = (PZ_LDS double*)(smem);  // [NW][5]
  const int w = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) part[w * 5 + k] = st[k];
    part[w * 5 + 4] = am;
  }
  __syncthreads();
  const int k = threadIdx.x;
  if (k < 5) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) s = k == 4 ? fmax(s, part[q * 5 + 4]) : s + part[q * 5 + k];
    if (k < 4 && want_st && (full || k == 3)) atomicAdd(o.stats + k, s);
    if (k == 4 && want_am)  // non-negative floats order like their bits
      atomicMax(reinterpret_cast<unsigned int*>(o.amax), __float_as_uint(static_cast<float>(s)));
  }
}


// The body of one workgroup: the GEMM `p`, workgroup `wgid` of its (XCD-remapped) grid
template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, typename OutT, typename AuxT, int VAR, int EK = EK_ANY>
PZ_DEV void gemm_body(const GemmArgs& p, int wgid) {
  static_assert(EK == EK_ANY || std::is_same<OutT, uint16_t>::value, "specialised epilogues: bf16 output");
  PZ_STAMP(0);
  constexpr int BK = var_bk<VAR>();
  constexpr int KB = BK / 32;  // 32-deep MFMA K blocks per ring slot
  using C = Cfg<BM, BN, WM, WN, var_ns<VAR>(), BK>;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PZ_LDS char* smem = (PZ_LDS char*)(smem_raw);

  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int split = p.split_k > 1 ? p.split_k : 1;
  int tm, tn, tile_id, slice;
  tile_coords(wgid, tiles_m, tiles_n, split, tm, tn, tile_id, slice);
  const int m0 = tm * BM, n0 = tn * BN;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const uint16_t* __restrict__ A = static_cast<const uint16_t*>(p.A);
  const uint16_t* __restrict__ B = static_cast<const uint16_t*>(p.B);

  // VAR 8: e4m3 operands (both K-contiguous), v_mfma_scale_f32_32x32x64_f8f6f4 with unit block
  // scales: a ring slot holds 64 K-bytes per row (the bf16 slot geometry), one MFMA K-step
  // VAR 9: A in e5m2 (bf8: gradients, wide range), B in e4m3 — the backward dX GEMM
  // dZ8 · W8ᵀ of the fp8 policy, with the backward (EPI_BWD) epilogues
  // VAR 10 / 11: VAR 8 / 9 with buffer-addressed staging DMA
  // VAR 14: the fp8 weight-gradient GEMM dW = X8ᵀ · dZ8 — e4m3 activations (A) x e5m2 output
  // gradients (B), BOTH M/N-contiguous ([K][M] / [K][N] bytes, K = batch rows), staged as k-row
  // images and read with the transposing ds_read_b64_tr_b8 (no transposed copies), bf16 output
  constexpr bool F8_MN = VAR == 14;
  // VAR 15: the fp8 forward X8 · W8 with the e4m3 weights in their natural [in, out] layout
  // (B N-contiguous, transposing 8-bit reads) — the same copy the backward dX GEMM reads as its
  // K-contiguous B, so one e4m3 weight copy serves both and no transposed copy is made
  constexpr bool F8_MNB = VAR == 15 || VAR == 16;
  constexpr bool F8 = VAR == 8 || VAR == 9 || VAR == 10 || VAR == 11 || VAR == 12 || VAR == 13 || VAR == 17 || F8_MN ||
                      F8_MNB;
  constexpr bool F8_BWD = VAR == 9 || VAR == 11 || VAR == 13 || VAR == 17;
  constexpr int F8_FMT_A = F8_BWD ? 1 : 0;  // MFMA format codes: 0 = fp8 e4m3, 1 = bf8 e5m2
  constexpr int F8_FMT_B = F8_MN ? 1 : 0;
  static_assert(!F8 || ((F8_MN ? (!A_KC && !B_KC) : F8_MNB ? (A_KC && !B_KC) : (A_KC && B_KC)) &&
                         std::is_same<OutT, uint16_t>::value),
                "fp8: K-contiguous in (M/N-contiguous for VAR 14), bf16 out");
  // VAR 41 (lab A/B): bf16 on v_mfma_f32_32x32x16_bf16 (32x32 accumulator tiles, the fp8 layout)
  constexpr bool M32 = VAR == 41;
  static_assert(!M32 || (A_KC && B_KC && std::is_same<OutT, uint16_t>::value), "M32: K-contiguous in, bf16 out");
  constexpr bool ACC32 = F8 || M32;  // 32x32 accumulator tiles
  constexpr int TM8 = C::WTM / 32, TN8 = C::WTN / 32;
  struct Frags16 { i16x8_t a[KB][C::TM]; i16x8_t b[KB][C::TN]; };
  struct Frags8 { i32x8_t a[KB][TM8]; i32x8_t b[KB][TN8]; };  // KB MFMA K-steps of 64 bytes
  struct Frags32 { i16x8_t a[2][TM8]; i16x8_t b[2][TN8]; };
  using Frags = std::conditional_t<F8, Frags8, std::conditional_t<M32, Frags32, Frags16>>;
  using AccT = std::conditional_t<ACC32, f32x16_t[TM8][TN8], f32x4_t[C::TM][C::TN]>;
  AccT acc;
  if constexpr (ACC32) {
#pragma unroll
    for (int i = 0; i < TM8; ++i)
#pragma unroll
      for (int j = 0; j < TN8; ++j) acc[i][j] = f32x16_t{};
  } else {
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
      for (int j = 0; j < C::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  // VAR 33 (lab A/B): VAR 30 without the s_setprio bracket around the MFMA block; GemmArgs::prio = 0
  // (PZ_GEMM_PRIO=0) drops it at run time (a uniform scalar branch per MFMA block)
  constexpr bool PRIO = VAR != 33;
  const bool prio = PRIO && p.prio != 0;
  auto mfma_step = [&](const Frags& f) {
    if (prio) __builtin_amdgcn_s_setprio(1);
    if constexpr (M32) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TM8; ++i)
#pragma unroll
          for (int j = 0; j < TN8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, f.b[ks][j]),
                                                                __builtin_bit_cast(bf16x8_t, f.a[ks][i]), acc[i][j], 0, 0, 0);
    } else if constexpr (F8) {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < TM8; ++i)
#pragma unroll
          for (int j = 0; j < TN8; ++j)  // issued as mfma(B, A): cbsz = B's format, blgp = A's;
                                         // E8M0 block scales 127 = 1.0
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(f.b[kb][j], f.a[kb][i], acc[i][j], F8_FMT_B,
                                                                         F8_FMT_A, 0, 127, 0, 127);
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int i = 0; i < C::TM; ++i)
#pragma unroll
          for (int j = 0; j < C::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, f.b[kb][j]),
                                                                __builtin_bit_cast(bf16x8_t, f.a[kb][i]), acc[i][j], 0, 0, 0);
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
  };
  auto read_frags = [&](int slot, Frags& f) {
    const PZ_LDS char* ta = smem + slot * C::SLOT_BYTES;
    const PZ_LDS char* tb = ta + C::A_BYTES;
    if constexpr (M32) {  // lane l: row l&31, k [8*(l>>5) + 16*ks, +8) = 16-B chunk (l>>5) + 2ks
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < TN8; ++j) f.b[ks][j] = frag_kc(tb, wn * C::WTN + j * 32 + (lane & 31), (lane >> 5) + 2 * ks);
#pragma unroll
        for (int i = 0; i < TM8; ++i) f.a[ks][i] = frag_kc(ta, wm * C::WTM + i * 32 + (lane & 31), (lane >> 5) + 2 * ks);
      }
    } else if constexpr (F8_MNB) {  // A: 16-B chunks of K-contiguous rows; B: transposing 8-bit reads
      const int h2 = 2 * (lane >> 5);
#pragma unroll
      for (int j = 0; j < TN8; ++j) f.b[0][j] = frag_mn8<BN>(tb, wn * C::WTN + j * 32, lane);
#pragma unroll
      for (int i = 0; i < TM8; ++i) {
        const int row = wm * C::WTM + i * 32 + (lane & 31);
        f.a[0][i] = cat_frag(frag_kc<BK>(ta, row, h2), frag_kc<BK>(ta, row, h2 + 1));
      }
    } else if constexpr (F8_MN) {  // transposing 8-bit reads of the [64 k][256 B] images (KB == 1)
#pragma unroll
      for (int j = 0; j < TN8; ++j) f.b[0][j] = frag_mn8<BN>(tb, wn * C::WTN + j * 32, lane);
#pragma unroll
      for (int i = 0; i < TM8; ++i) f.a[0][i] = frag_mn8<BM>(ta, wm * C::WTM + i * 32, lane);
    } else if constexpr (F8) {  // lane l: row l&31, K bytes [32*(l>>5), +32) of K-step kb = 16-B chunks
                                // 4kb + 2h, 4kb + 2h + 1
      const int h2 = 2 * (lane >> 5);
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int j = 0; j < TN8; ++j) {
          const int row = wn * C::WTN + j * 32 + (lane & 31);
          f.b[kb][j] = cat_frag(frag_kc<BK>(tb, row, 4 * kb + h2), frag_kc<BK>(tb, row, 4 * kb + h2 + 1));
        }
#pragma unroll
        for (int i = 0; i < TM8; ++i) {
          const int row = wm * C::WTM + i * 32 + (lane & 31);
          f.a[kb][i] = cat_frag(frag_kc<BK>(ta, row, 4 * kb + h2), frag_kc<BK>(ta, row, 4 * kb + h2 + 1));
        }
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
        for (int j = 0; j < C::TN; ++j) {
          if constexpr (B_KC) f.b[kb][j] = frag_kc<BK>(tb, wn * C::WTN + j * 16 + (lane & 15), (lane >> 4) + 4 * kb);
          else f.b[kb][j] = frag_mn<BN>(tb, wn * C::WTN + j * 16, 8 * (lane >> 4) + 32 * kb, lane);
        }
#pragma unroll
        for (int i = 0; i < C::TM; ++i) {
          if constexpr (A_KC) f.a[kb][i] = frag_kc<BK>(ta, wm * C::WTM + i * 16 + (lane & 15), (lane >> 4) + 4 * kb);
          else f.a[kb][i] = frag_mn<BM>(ta, wm * C::WTM + i * 16, 8 * (lane >> 4) + 32 * kb, lane);
        }
      }
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  const int nk = p.K / (F8 ? 2 * BK : BK) / split;  // K steps of this slice (fp8: 2 bytes per 16-bit unit)
  const int kt0 = slice * nk;
  // LDS-DMA addressing per operand: buffer (MUBUF, 32-bit per-lane offsets from one descriptor)
  // or flat (64-bit pointers). Measured (tools/gemm_lab, same box): buffer is +6..10% on the
  // M/N-contiguous operands, whose k-row addresses otherwise cost 64-bit multiplies every step,
  // and 1.5..5% slower on K-contiguous ones (VAR 25 = buffer for M/N-contiguous only)
  constexpr bool BUF_A = VAR == 6 || VAR == 7 || (VAR >= 10 && VAR <= 13) || VAR == 41 || (VAR == 25 && !A_KC) || (VAR >= 27 && VAR <= 33);
  constexpr bool BUF_B = VAR == 6 || VAR == 7 || (VAR >= 10 && VAR <= 13) || VAR == 41 || (VAR == 25 && !B_KC) || (VAR >= 27 && VAR <= 33);
  constexpr int POL = VAR >= 27 && VAR <= 29 ? VAR - 26 : 0;
  // VAR 30/31: full row tiles of the K-contiguous operands (use_bk64 checks M % BM, N % BN)
  constexpr bool FULL_KC = VAR == 30 || VAR == 31 || VAR == 32 || VAR == 33 || VAR == 12 || VAR == 13;
  const i32x4_t rs_a = buf_rsrc(A), rs_b = buf_rsrc(B);
  // staging works in 16-bit units: an e4m3 row of 64 K-bytes is the same 64-B piece
  const int64_t lda = F8 ? p.lda / 2 : p.lda, ldb = F8 ? p.ldb / 2 : p.ldb;
  // (measured, not kept: DMA issued by waves 0-3 only, twice the instructions each: -2..4%)
  constexpr int NWD = C::NW;
  constexpr bool PF = VAR == 24;      // L2 prefetch kPfAhead steps beyond the staged one
  constexpr int kPfAhead = 3;
  constexpr int GD = C::G + (PF ? 1 : 0);
  // TEAM waves (team-local index tw) issue one operand's DMA of a step
  auto stage_a_t = [&](int kt, auto team, int tw) {
    constexpr int TEAM = decltype(team)::value;
    PZ_LDS char* base = smem + (kt % C::NS) * C::SLOT_BYTES;
    if constexpr (F8_MN) stage_mn8<BM, TEAM, 64>(lda, m0, (kt0 + kt) * 64, base, tw, lane, rs_a);
    else if constexpr (A_KC) stage_kc<BM, TEAM, BK, BUF_A, POL, FULL_KC>(A, lda, m0, p.M, (kt0 + kt) * BK, base, tw, lane, rs_a);
    else stage_mn<BM, TEAM, BK, BUF_A, POL>(A, lda, m0, p.M, (kt0 + kt) * BK, base, tw, lane, rs_a);
  };
  auto stage_b_t = [&](int kt, auto team, int tw) {
    constexpr int TEAM = decltype(team)::value;
    PZ_LDS char* base = smem + (kt % C::NS) * C::SLOT_BYTES + C::A_BYTES;
    if constexpr (F8_MN || F8_MNB) stage_mn8<BN, TEAM, 64>(ldb, n0, (kt0 + kt) * 64, base, tw, lane, rs_b);
    else if constexpr (B_KC) stage_kc<BN, TEAM, BK, BUF_B, POL, FULL_KC>(B, ldb, n0, p.N, (kt0 + kt) * BK, base, tw, lane, rs_b);
    else stage_mn<BN, TEAM, BK, BUF_B, POL>(B, ldb, n0, p.N, (kt0 + kt) * BK, base, tw, lane, rs_b);
  };
  auto stage_a = [&](int kt) { stage_a_t(kt, std::integral_constant<int, NWD>{}, wave); };
  auto stage_b = [&](int kt) { stage_b_t(kt, std::integral_constant<int, NWD>{}, wave); };
  auto prefetch = [&](int kt) {  // one dword per 128-B line of step kt's A and B tiles
    kt = min(kt, nk - 1);
    const int k0 = (kt0 + kt) * BK;
    uint32_t sink = lds_addr(smem + C::NS * C::SLOT_BYTES);
    const int tid = wave * 64 + lane;  // 512 lanes: A lines first, then B lines
    auto line = [&](const uint16_t* g, int64_t ld, bool kc, int R, int r0, int valid, int idx) -> const void* {
      if (kc) {  // idx = row
        int gr = min(r0 + idx, valid - 1);
        return g + static_cast<int64_t>(gr) * ld + k0;
      }
      const int per = (R * 2) / 128;  // lines per k row
      const int kr = idx / per, c = (idx % per) * 64;
      return g + static_cast<int64_t>(k0 + kr) * ld + min(r0 + c, valid - 8);
    };
    const int na = A_KC ? BM : BK * (BM * 2 / 128);
    const int nb = B_KC ? BN : BK * (BN * 2 / 128);
    if (tid < na) glds4(line(A, lda, A_KC, BM, m0, p.M, tid), sink);
    else if (tid < na + nb) glds4(line(B, ldb, B_KC, BN, n0, p.N, tid - na), sink);
    else glds4(A, sink);
  };
  auto stage = [&](int kt, int slot) {  // slot == kt % NS
    (void)slot;
    stage_a(kt);
    stage_b(kt);
    if constexpr (PF) prefetch(kt + kPfAhead);
  };

  constexpr int NS = C::NS;
  // Measured, not kept: staging K-contiguous operands in PAIRS of steps so both 64-B halves of
  // every 128-B line are requested back to back (halved L1->L2 requests, matched hipBLASLt's
  // request count) ran 2-4% SLOWER than the plain ring with DEFER below.
  constexpr bool DEFER = VAR != 4;  // group 0 waits for step t+1 at the END of M_t (+2..6%)
  if constexpr (BK == 64) {
    // Ping-pong over 64-deep steps in a 2-slot ring (VAR 20: waves 0-3 issue every DMA in their
    // read interval; VAR 21: waves 0-3 stage A in their read interval R_t while waves 4-7 stage
    // B of the same step t+1 at the head of their MFMA interval M_{t-1} — the same barrier
    // interval). Interval 2t: G0 R_t | G1 M_{t-1}; interval 2t+1: G0 M_t | G1 R_t. Slot (t+1)%2
    // was last read by G1 in interval 2t-1, so step t+1 is issued in interval 2t and awaited
    // (vmcnt(0)) at the end of interval 2t+1 by every wave, before G0 reads it in 2t+2.
    static_assert(C::NW == 8, "BK64 ping-pong needs 8 waves");
    const int grp = wave >> 2, tw = wave & 3;
    using T4 = std::integral_constant<int, 4>;
    auto stage_g0 = [&](int kt) {
      stage_a_t(kt, T4{}, tw);
      if constexpr (!(VAR == 21 || VAR == 31)) stage_b_t(kt, T4{}, tw);  // 21 / 31: group 1 stages B
    };
    stage(0, 0);
    wait_vm<0>();
    barrier();
    PZ_STAMP(1);
    if (grp == 1) {
      if ((VAR == 21 || VAR == 31) && nk > 1) stage_b_t(1, T4{}, tw);
      barrier();
    }
    for (int t = 0; t < nk; ++t) {
      if (grp == 0 && t + 1 < nk) stage_g0(t + 1);
      Frags f;
      read_frags(t % 2, f);
      if (grp == 1) wait_vm<0>();  // step t+1 (issued in M_{t-1}) landed before interval 2t+2
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
      if ((VAR == 21 || VAR == 31) && grp == 1 && t + 2 < nk) stage_b_t(t + 2, T4{}, tw);
      mfma_step(f);
      if (grp == 0) wait_vm<0>();
      barrier();
    }
    if (grp == 0) barrier();
    PZ_STAMP(2);
  } else {
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) stage(s, s);

  if constexpr (C::NW == 8) {
    // Ping-pong (8 waves = 2 per SIMD). Waves 0-3 and 4-7 sit on the same four SIMDs and run one
    // barrier interval apart: while one wave of a SIMD issues its MFMA block (setprio 1) its
    // partner issues the next step's LDS-DMA + fragment reads into the MFMA gaps. Per wave and
    // step t: R_t = {stage t+NS-1, [group 1: wait until step t+1 landed], read slot t,
    // lgkmcnt(0)} | barrier | M_t = {MFMAs, [group 0: wait until step t+1 landed]} | barrier.
    // Group 0 runs one interval AHEAD, so its wait can sit at the end of its MFMA block (one
    // interval more of DMA latency hidden) and still precede the barrier that opens R_{t+1} for
    // both groups. Hazards: slot t+1 is waited for by every wave before that barrier; slot
    // (t+NS-1)%NS = (t-1)%NS was last read in R_{t-1} and every wave retired those reads
    // (lgkmcnt(0)) before the barrier that precedes R_t of either group.
    const int grp = wave >> 2;
    auto wait_step = [&](int n) {
      if constexpr (PF) wait_newer_pf<GD, NS - 2>(n);
      else wait_newer<GD, NS - 2>(n);
    };
    wait_step(min(nk, NS - 1) - 1);  // step 0 landed
    barrier();
    PZ_STAMP(1);
    if (grp == 1) barrier();
    for (int t = 0; t < nk; ++t) {
      if (VAR != 2 && t + NS - 1 < nk) stage(t + NS - 1, (t + NS - 1) % NS);
      if (!DEFER || grp == 1) wait_step(min(nk - 1, t + NS - 1) - (t + 1));  // step t+1 landed
      Frags f;
      if constexpr (VAR == 3) {  // perf probe: no fragment reads
#pragma unroll
        for (int i = 0; i < C::TM; ++i) f.a[0][i] = i16x8_t{(short)i, 1, 2, 3, 4, 5, 6, (short)t};
#pragma unroll
        for (int j = 0; j < C::TN; ++j) f.b[0][j] = i16x8_t{(short)j, 1, 2, 3, 4, 5, 6, (short)t};
      } else {
        read_frags(t % NS, f);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      barrier();
      if constexpr (VAR != 1) {
        mfma_step(f);
      } else {  // perf probe: no MFMAs (keep the fragments live)
#pragma unroll
        for (int i = 0; i < C::TM; ++i) acc[i][0][0] += static_cast<float>(f.a[0][i][0] + f.b[0][i % C::TN][1]);
      }
      if (DEFER && grp == 0) wait_step(min(nk - 1, t + NS - 1) - (t + 1));
      barrier();
    }
    if (grp == 0) barrier();
    PZ_STAMP(2);
    if constexpr (PF) wait_vm<0>();  // no prefetch DMA may outlive the workgroup's LDS
  } else {
  PZ_STAMP(1);  // (4-wave tiles: before the first wait)
  for (int t = 0; t < nk; ++t) {
    // slot t landed: everything newer than step t (at most NS-2 steps) may stay in flight
    wait_newer<C::G, NS - 2>(min(nk - 1, t + NS - 2) - t);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nk) stage(t + NS - 1, (t + NS - 1) % NS);
    Frags f;
    read_frags(t % NS, f);
    mfma_step(f);
  }
  PZ_STAMP(2);
  }
  }  // BK

  // ---------------------------------------------------------------- split-K reduction
  // Write-through hand-off (MI355X_MICROARCH "publish-large" / "splitk-seam", hand-off table row
  // 1): every slice stores its fp32 slab with `sc1` (write-through) 16-B buffer stores, drains
  // them (vmcnt(0)), joins a barrier, and ONE lane takes a relaxed agent-scope ticket; the slice
  // whose add returned split-1 sums the other slabs with `sc1` loads (after a barrier its waves
  // join) and runs the epilogue. No release fence (its L2 write-back of every dirty line of the
  // XCD cost ~2.7x the publish, measured 19-23 us of a split-K GEMM's 85-95 us) and no acquire.
  // (measured, not kept: plain stores + agent release / acquire fences, VAR 32)
  if (split > 1) {
    constexpr int CH = ACC32 ? TM8 * TN8 * 4 : C::TM * C::TN;  // f32x4 chunks per lane
    const int tid = threadIdx.x;
    auto get_chunk = [&](auto cc) -> f32x4_t {
      constexpr int c = decltype(cc)::value;
      if constexpr (ACC32) {
        constexpr int i = (c / 4) / TN8, j = (c / 4) % TN8, q = 4 * (c % 4);
        return f32x4_t{acc[i][j][q], acc[i][j][q + 1], acc[i][j][q + 2], acc[i][j][q + 3]};
      } else {
        return acc[c / C::TN][c % C::TN];
      }
    };
    static_assert(CH % 8 == 0, "the fold runs 8 chunks at a time");
    constexpr int kSlabBytes = BM * BN * 4;
    // one descriptor per tile's slab group (split x 256 KiB: 32-bit offsets always suffice)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.ws + static_cast<int64_t>(tile_id) * split * (BM * BN), 0,
                                                      split * kSlabBytes, 0x00020000);
    constexpr int kSc1 = 16;  // cache-policy bit sc1
    static_for<CH>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, get_chunk(cc)), rs,
                                             slice * kSlabBytes + (c * C::NT + tid) * 16, 0, kSc1);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    PZ_LDS int* flag = (PZ_LDS int*)(smem);
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(p.counters + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = prev == split - 1;
      if (prev == split - 1) p.counters[tile_id] = 0;  // ready for the next launch
    }
    __syncthreads();
    if (*flag == 0) return;  // block-uniform: another slice finishes this tile
    // The sum order must not depend on which slice arrived last (deterministic results): a fixed
    // pairwise tree ((s0 + s1) + (s2 + s3)) + ((s4 + s5) + (s6 + s7)) whose leaf pairs and subtree
    // pairs are each added in either order — float addition commutes exactly — so the last
    // arriver starts from its own slice in registers and loads only the split - 1 others.
    auto ld = [&](int sl, int c) {
      return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, sl * kSlabBytes + (c * C::NT + tid) * 16, 0, kSc1));
    };
    const int mate = slice ^ 1, pair2 = (slice ^ 2) & ~1, quad4 = (slice ^ 4) & ~3;
    static_for<CH / 8>([&](auto gc) {  // 8 chunks at a time: bounded temporaries
      static_for<8>([&](auto qc) {
        constexpr int c = 8 * decltype(gc)::value + decltype(qc)::value;
        f32x4_t v = get_chunk(std::integral_constant<int, c>{}) + ld(mate, c);
        if (split >= 4) v = v + (ld(pair2, c) + ld(pair2 + 1, c));
        if (split >= 8) v = v + ((ld(quad4, c) + ld(quad4 + 1, c)) + (ld(quad4 + 2, c) + ld(quad4 + 3, c)));
        if constexpr (ACC32) {
          constexpr int i = (c / 4) / TN8, j = (c / 4) % TN8, q = 4 * (c % 4);
          acc[i][j][q] = v[0]; acc[i][j][q + 1] = v[1]; acc[i][j][q + 2] = v[2]; acc[i][j][q + 3] = v[3];
        } else {
          acc[c / C::TN][c % C::TN] = v;
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  }

  // ---------------------------------------------------------------- epilogue
  // static_for (not #pragma unroll): the acc array must only ever be indexed by compile-time
  // constants or it is demoted to scratch (guide §5.4 rule 20)
  PZ_STAMP(3);
  OutT* __restrict__ Cp = static_cast<OutT*>(p.C);
  const AuxT* __restrict__ aux = static_cast<const AuxT*>(p.aux);
  const int g4 = 4 * (lane >> 4);
  if constexpr (ACC32) {
    const float alpha = p.alpha * (p.scale_a != nullptr ? *p.scale_a : 1.f) * (p.scale_b != nullptr ? *p.scale_b : 1.f);
    if constexpr (F8_BWD || M32) epilogue_lds<BM, BN, WM, WN, Lay32<TM8, TN8>, false, EK>(p, acc, smem, m0, n0, wm, wn, lane, alpha);
    else epilogue_lds<BM, BN, WM, WN, Lay32<TM8, TN8>, true, EK>(p, acc, smem, m0, n0, wm, wn, lane, alpha);
  } else if constexpr (std::is_same<OutT, uint16_t>::value) {
    epilogue_lds<BM, BN, WM, WN, Lay16<C::TM, C::TN>, false, EK>(p, acc, smem, m0, n0, wm, wn, lane, p.alpha);
  } else if (p.epi_mode == EPI_OPT) {
    epilogue_opt<C>(p, acc, smem, m0, n0, wm, wn, lane);
  } else {
  static_for<C::TN>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int n = n0 + wn * C::WTN + j * 16 + g4;
    const bool n_ok = n < p.N;
    f32x4_t bias4 = {0.f, 0.f, 0.f, 0.f};
    if (p.bias != nullptr && n_ok) bias4 = *reinterpret_cast<const f32x4_t*>(p.bias + n);
    f32x4_t cs = {0.f, 0.f, 0.f, 0.f};
    static_for<C::TM>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const int m = m0 + wm * C::WTM + i * 16 + (lane & 15);
      if (n_ok && m < p.M) cs += epi_apply<OutT, AuxT>(p, acc[i][j], bias4, m, n, Cp, aux);
    });
    if (p.colsum != nullptr) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = group_sum<16>(cs[r]);
        if ((lane & 15) == 0 && n + r < p.N) atomicAdd(p.colsum + n + r, s);
      }
    }
  });
  }
#ifdef PZ_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tile's stores have left this CU
  __syncthreads();
  PZ_STAMP(4);
#endif
}

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, typename OutT, typename AuxT, int VAR, int EK = EK_ANY>
__global__ void __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(var_waves_per_eu<VAR>())))
gemm_mfma_kernel(const GemmArgs p) {
  gemm_body<BM, BN, WM, WN, A_KC, B_KC, OutT, AuxT, VAR, EK>(p, xcd_remap(blockIdx.x, gridDim.x));
}

#include "gemm_w4.h"  // VAR 40: the dX layout on 4-wave workgroups (hipBLASLt's schedule)

// Two independent GEMMs of one layout / epilogue kind in ONE launch (gemm_pair): the first nwg0
// remapped workgroup ids run GEMM 0, the rest GEMM 1 — e.g. the two skinny weight-gradient GEMMs
// of a 3-layer MLP (64 tiles each at batch 8192) that alone would each need a 4-way split-K to
// fill the CUs: together they fill them with a 2-way split (or none), half (or none) of the slab
// hand-offs, and one launch instead of two
struct GemmPairArgs {
  GemmArgs p[2];
  int nwg0;
};

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, typename OutT, typename AuxT, int VAR, int EK = EK_ANY>
__global__ void __launch_bounds__(WM * WN * 64) __attribute__((amdgpu_waves_per_eu(var_waves_per_eu<VAR>())))
gemm_mfma_pair_kernel(const GemmPairArgs g) {
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int second = w >= g.nwg0 ? 1 : 0;  // workgroup-uniform
  gemm_body<BM, BN, WM, WN, A_KC, B_KC, OutT, AuxT, VAR, EK>(g.p[second], w - second * g.nwg0);
}

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, typename OutT, typename AuxT, int VAR, int EK = EK_ANY>
hipError_t launch_cfg(const GemmArgs& p, hipStream_t s) {
  using C = Cfg<BM, BN, WM, WN, var_ns<VAR>(), var_bk<VAR>()>;
  auto kern = gemm_mfma_kernel<BM, BN, WM, WN, A_KC, B_KC, OutT, AuxT, VAR, EK>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nwg = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN) * (p.split_k > 1 ? p.split_k : 1);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(C::NT), C::LDS_BYTES, s, p);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, typename OutT, typename AuxT, int VAR = 0>
hipError_t launch_layout(const GemmArgs& p, hipStream_t s) {
  if (p.a_kc && p.b_kc) return launch_cfg<BM, BN, WM, WN, true, true, OutT, AuxT, VAR>(p, s);
  if (p.a_kc && !p.b_kc) return launch_cfg<BM, BN, WM, WN, true, false, OutT, AuxT, VAR>(p, s);
  if (!p.a_kc && p.b_kc) return launch_cfg<BM, BN, WM, WN, false, true, OutT, AuxT, VAR>(p, s);
  return launch_cfg<BM, BN, WM, WN, false, false, OutT, AuxT, VAR>(p, s);
}

#ifndef PZ_GEMM_LAB  // tools/gemm_lab.hip instantiates only the variants it measures
// buffer-addressed DMA (VAR 6) needs every staged byte within 4 GiB of the operand's base
bool buffer_ok(const GemmArgs& p) {
  constexpr int64_t kLim = int64_t(1) << 32;
  const int64_t ea = (p.a_kc ? static_cast<int64_t>(p.M) : static_cast<int64_t>(p.K)) * p.lda * 2;
  const int64_t eb = (p.b_kc ? static_cast<int64_t>(p.N) : static_cast<int64_t>(p.K)) * p.ldb * 2;
  return ea < kLim && eb < kLim;
}

// (measured, not kept: 128x128 tiles, two workgroups per CU, instead of split-K 256x256 for
// skinny shapes — fwd [8192,1024] K=4096 950 vs 855 TFLOP/s alone, the mlp4 step 0.9% slower)
// 64-deep ring steps (VAR 30: 2 x 64 KiB slots, one MFMA interval = 64 MFMAs per wave, the
// staging waves fetch whole 128-B lines of K-contiguous rows) for layouts with an M/N-contiguous
// operand: fwd [8192,4096]x[4096,4096] +6%, dW +4%, fwd K=1024 +4% (tools/gemm_lab, same box).
// Both operands K-contiguous (dX) stay on the 32-deep ring: the BK64 form spills there (-11%).
bool use_bk64(const GemmArgs& p, bool buf) {
  const int split = p.split_k > 1 ? p.split_k : 1;
  // VAR 30 stages K-contiguous operands without a row clamp: full 256-row tiles only (which
  // also frees the K-contiguous x K-contiguous dX GEMMs from a scratch spill: +5..6%, lab)
  const bool full = (!p.a_kc || p.M % 256 == 0) && (!p.b_kc || p.N % 256 == 0);
  return buf && full && p.K % 64 == 0 && (p.K / 64) % split == 0;
}

// VAR 40 / 42 for the bf16 / fp8 dX layout (gemm_w4.h); PZ_GEMM_W4=0 keeps those GEMMs on VAR 30 /
// VAR 9, 17 (A/B)
bool w4_default() {
  static const bool on = [] {
    const char* e = getenv("PZ_GEMM_W4");
    return e == nullptr || atoi(e) != 0;
  }();
  return on;
}

// which specialised epilogue (gemm_epilogue.h: EK_*) covers these arguments
int epi_kind(const GemmArgs& p) {
  if (p.out_dtype != DT_BF16 || p.accumulate) return EK_ANY;
  if (p.epi_mode == EPI_STORE && p.bias == nullptr && p.colsum == nullptr && p.mask == nullptr && p.out8 == nullptr)
    return EK_STORE;
  if (p.epi_mode == EPI_FWD && (p.epi.act == ACT_NONE || p.epi.act == ACT_RELU) && p.colsum == nullptr) {
    const EpiSpec& e = p.epi;
    const bool relu = e.act == ACT_RELU;
    if (!e.drop_all) {
      if (relu && !e.drop_pre && e.drop_post) return EK_F_RELU_POST;
      if (relu && e.drop_pre && e.drop_post) return EK_F_RELU_PREPOST;
      if (!relu && e.drop_pre && !e.drop_post) return EK_F_PRE;
    }
    return EK_RELU;
  }
  if (p.epi_mode == EPI_BWD && p.mask != nullptr && p.epi.act == ACT_RELU) return EK_BWD_MASK;
  return EK_ANY;
}

// the MLP's three GEMM layouts on the 64-deep ring, each with its stage's specialised epilogue:
// forward X·W (K-contiguous x N-contiguous), dX = dZ·Wᵀ (both K-contiguous), dW = Xᵀ·dZ (both
// M/N-contiguous); anything else takes the generic epilogue
template <typename OutT, typename AuxT, int VAR>
hipError_t launch_bk64_256(const GemmArgs& p, hipStream_t s) {
  if constexpr (std::is_same<OutT, uint16_t>::value) {
    const int ek = epi_kind(p);
    if (p.a_kc && !p.b_kc) {
      if (ek == EK_RELU) return launch_cfg<256, 256, 2, 4, true, false, OutT, AuxT, VAR, EK_RELU>(p, s);
      if (ek == EK_F_RELU_POST) return launch_cfg<256, 256, 2, 4, true, false, OutT, AuxT, VAR, EK_F_RELU_POST>(p, s);
      if (ek == EK_F_RELU_PREPOST)
        return launch_cfg<256, 256, 2, 4, true, false, OutT, AuxT, VAR, EK_F_RELU_PREPOST>(p, s);
      if (ek == EK_F_PRE) return launch_cfg<256, 256, 2, 4, true, false, OutT, AuxT, VAR, EK_F_PRE>(p, s);
    }
    if (p.a_kc && p.b_kc && ek == EK_BWD_MASK)
      return launch_cfg<256, 256, 2, 4, true, true, OutT, AuxT, VAR, EK_BWD_MASK>(p, s);
    if (!p.a_kc && !p.b_kc && ek == EK_STORE) return launch_cfg<256, 256, 2, 4, false, false, OutT, AuxT, VAR, EK_STORE>(p, s);
  }
  return launch_layout<256, 256, 2, 4, OutT, AuxT, VAR>(p, s);
}

// Fixed-kind bf16 forward GEMMs with too few 256x256 tiles to fill the CUs (the logits GEMM,
// [8192, 1024] at K = 4096) run as 256x128 tiles on the 64-deep ring WITHOUT split-K: the
// deterministic split-K fold's slab round trip and the split tile's heavier epilogue cost more
// than the narrower tile's extra LDS traffic. r5 same box: fused fwd_L3 885-949 vs 830-841 TF/s,
// mlp4 step 1.111-1.113 vs 1.130-1.138 ms (profiles/r5_ab_w128_fixed.txt). (r2, before the
// fixed epilogue kinds and the deterministic fold: the generic-epilogue 256x128 form lost in-step.)
bool w128_fixed(const GemmArgs& p) {
  if (p.in_dtype != DT_BF16 || p.out_dtype != DT_BF16 || !p.a_kc || p.b_kc || p.accumulate) return false;
  if (p.M % 256 || p.N % 128 || !ek_fixed(epi_kind(p))) return false;
  return ((p.M / 256) * ((p.N + 255) / 256)) < 240 && (p.M / 256) * (p.N / 128) >= 240;
}

template <typename OutT, typename AuxT>
hipError_t launch_tiles(const GemmArgs& p, hipStream_t s) {
  auto tiles = [&](int bm, int bn) { return ((p.M + bm - 1) / bm) * ((p.N + bn - 1) / bn); };
  const bool buf = buffer_ok(p);
  const bool bk64 = use_bk64(p, buf);
  constexpr int kFill = 240;  // ~ CU count: a config below this leaves CUs idle
  if (p.split_k > 1) {  // slabs sized for 256x256
    if (bk64) return launch_bk64_256<OutT, AuxT, 30>(p, s);
    if (buf) return launch_layout<256, 256, 2, 4, OutT, AuxT, 6>(p, s);
    return launch_layout<256, 256, 2, 4, OutT, AuxT>(p, s);
  }
  if constexpr (std::is_same<OutT, uint16_t>::value) {
    const int ek = epi_kind(p);
    if (w4_default() && w4_eligible(p, ek))
      return ek == EK_BWD_MASK ? launch_w4<EK_BWD_MASK>(p, s) : launch_w4<EK_STORE>(p, s);
  }
  // buffer-addressed LDS-DMA (VAR 6; +2..12% on the step's shapes, tools/gemm_lab)
  if (tiles(256, 256) >= kFill) {
    if (bk64) return launch_bk64_256<OutT, AuxT, 30>(p, s);
    return buf ? launch_layout<256, 256, 2, 4, OutT, AuxT, 6>(p, s) : launch_layout<256, 256, 2, 4, OutT, AuxT>(p, s);
  }
  if (tiles(256, 128) >= kFill) {
    if constexpr (std::is_same<OutT, uint16_t>::value) {
      if (bk64 && w128_fixed(p)) {
        const int ek = epi_kind(p);
        if (ek == EK_F_RELU_POST) return launch_cfg<256, 128, 4, 2, true, false, OutT, AuxT, 30, EK_F_RELU_POST>(p, s);
        if (ek == EK_F_RELU_PREPOST) return launch_cfg<256, 128, 4, 2, true, false, OutT, AuxT, 30, EK_F_RELU_PREPOST>(p, s);
        if (ek == EK_F_PRE) return launch_cfg<256, 128, 4, 2, true, false, OutT, AuxT, 30, EK_F_PRE>(p, s);
      }
    }
    if (bk64) return launch_layout<256, 128, 4, 2, OutT, AuxT, 30>(p, s);
    return buf ? launch_layout<256, 128, 4, 2, OutT, AuxT, 6>(p, s) : launch_layout<256, 128, 4, 2, OutT, AuxT>(p, s);
  }
  return buf ? launch_layout<128, 128, 2, 2, OutT, AuxT, 6>(p, s) : launch_layout<128, 128, 2, 2, OutT, AuxT>(p, s);
}

// fp8 GEMMs with at least two 256x256 tiles per CU and no split-K run as 256x128 tiles on 4-wave
// workgroups, two per CU (VAR 16 / 17): one workgroup's epilogue beside the other's main loop
bool f8_two_wg(const GemmArgs& p) {
  const int t256 = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  return p.split_k <= 1 && t256 >= 480 && p.N % 128 == 0;
}

hipError_t launch_fp8(const GemmArgs& p, hipStream_t s) {
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  if (!p.a_kc && !p.b_kc)  // e4m3 x e5m2 weight gradient (fp8_eligible: full 256-tiles, buffer-addressable,
                          // plain store)
    return launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 14, EK_STORE>(p, s);
  int ek = epi_kind(p);
  // VAR 43: the fp8 forward on the 4-wave LDS-DMA schedule, plain stores at K >= 2048 (at K = 1,024 it
  // ties VAR 16). With the fused stage epilogues the 32x32 accumulator layout's 128-column wave rows
  // (16 four-column groups per lane: values, column sums, bias) spill 66-213 VGPRs — the fused fp8 dX
  // (VAR 42, tools/gemm_w4f8_lab.hip) ran 144 vs 106 us in the mlp8192 step (profiles/r6_gemm_w4.txt) —
  // so the trainer's fused fp8 GEMMs stay on VAR 9 / 15-17
  if (w4_default() && ek == EK_STORE && p.K >= 2048 && w4f8_fwd_eligible(p, ek)) return launch_w4f8<EK_STORE, false>(p, s);
  if (f8_two_wg(p)) {
    if (p.a_kc && !p.b_kc) {
      if (ek == EK_RELU) return launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16, EK_RELU>(p, s);
      if (ek == EK_F_RELU_POST) return launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16, EK_F_RELU_POST>(p, s);
      if (ek == EK_F_RELU_PREPOST)
        return launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16, EK_F_RELU_PREPOST>(p, s);
      if (ek == EK_F_PRE) return launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16, EK_F_PRE>(p, s);
      return launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16>(p, s);
    }
    if (p.a_kc && p.b_kc && p.a_fmt == 1) {
      if (ek == EK_BWD_MASK) return launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 17, EK_BWD_MASK>(p, s);
      return launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 17>(p, s);
    }
  }
  if (p.a_kc && !p.b_kc) {  // e4m3 X x e4m3 W[in, out] (fp8_eligible: N % 256 — B's transposed image
                           // rows are whole 256-B tiles, swz_mn8 — buffer-addressable B; split-K
                           // when the tiles do not fill the CUs, gemm_split)
    if (ek == EK_RELU) return launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, EK_RELU>(p, s);
    if (ek == EK_F_RELU_POST) return launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, EK_F_RELU_POST>(p, s);
    if (ek == EK_F_RELU_PREPOST)
      return launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, EK_F_RELU_PREPOST>(p, s);
    if (ek == EK_F_PRE) return launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, EK_F_PRE>(p, s);
    return launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15>(p, s);
  }
  // (measured, not kept: buffer-addressed staging, VAR 10 / 11; the 64-deep ring, VAR 12 / 13,
  // within noise of the 32-deep one, profiles/r2_ab_fp8_bk64.txt)
  if (ek_fixed(ek)) ek = EK_RELU;  // (VAR 8 forms: the generic ReLU-stage kind)
  const bool big = tiles >= 240 || p.split_k > 1;
  if (p.a_fmt == 1) {  // e5m2 x e4m3 (backward dX)
    if (ek == EK_BWD_MASK)
      return big ? launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 9, EK_BWD_MASK>(p, s)
                 : launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 9, EK_BWD_MASK>(p, s);
    return big ? launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 9>(p, s)
               : launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 9>(p, s);
  }
  if (ek == EK_RELU)
    return big ? launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 8, EK_RELU>(p, s)
               : launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 8, EK_RELU>(p, s);
  return big ? launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 8>(p, s)
             : launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 8>(p, s);
}

template <typename OutT, int VAR, int EK>
hipError_t launch_pair_cfg(const GemmPairArgs& g, int nwg, hipStream_t s) {
  using C = Cfg<256, 256, 2, 4, var_ns<VAR>(), var_bk<VAR>()>;
  auto kern = gemm_mfma_pair_kernel<256, 256, 2, 4, false, false, OutT, uint16_t, VAR, EK>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS_BYTES);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(C::NT), C::LDS_BYTES, s, g);
  return hipGetLastError();
}

#endif  // PZ_GEMM_LAB
}  // namespace

#ifndef PZ_GEMM_LAB
bool fp8_dw_eligible(const GemmArgs& p) {  // VAR 14: X8ᵀ (e4m3) · dZ8 (e5m2), both M/N-contiguous
  if (p.a_fmt != 0 || p.b_fmt != 1 || p.epi_mode != EPI_STORE || p.accumulate) return false;
  if (p.bias != nullptr || p.colsum != nullptr || p.mask != nullptr || p.out8 != nullptr || p.aux != nullptr) return false;
  if (p.M % 256 != 0 || p.N % 256 != 0 || p.K % 64 != 0 || p.K < 64) return false;
  if (p.lda % 16 != 0 || p.ldb % 16 != 0 || p.ldc % 8 != 0) return false;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(p.A) || !al16(p.B) || !al16(p.C)) return false;
  constexpr int64_t kLim = int64_t(1) << 32;  // buffer-addressed staging
  return static_cast<int64_t>(p.K) * p.lda < kLim && static_cast<int64_t>(p.K) * p.ldb < kLim;
}

bool fp8_eligible(const GemmArgs& p) {
  if (p.force_generic || p.in_dtype != DT_FP8 || p.out_dtype != DT_BF16) return false;
  if (p.bias64 != nullptr || p.colsum64 != nullptr) return false;
  if (!p.a_kc && !p.b_kc) return fp8_dw_eligible(p);
  if (p.b_fmt != 0) return false;
  if (p.a_kc && !p.b_kc) {  // VAR 15: forward on the [in, out] e4m3 weights
    if (p.a_fmt != 0 || p.epi_mode == EPI_BWD || p.accumulate || p.N % 256 != 0) return false;
    if (static_cast<int64_t>(p.K) * p.ldb >= (int64_t(1) << 32)) return false;  // buffer-addressed B
  } else if (!p.a_kc || p.accumulate) {
    return false;
  }
  if (p.M < 64 || p.N < 64 || p.K < 64 || p.K % 64 != 0) return false;
  if (p.N % 8 != 0 || p.ldc % 8 != 0 || p.lda % 16 != 0 || p.ldb % 16 != 0) return false;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(p.A) || !al16(p.B) || !al16(p.C)) return false;
  if (p.idx_ld % 2 != 0) return false;
  if (p.bias != nullptr && !al16(p.bias)) return false;
  // e4m3 x e4m3: forward stages; e5m2 (A, gradients) x e4m3 (B): backward dX stages only
  if ((p.a_fmt == 1) != (p.epi_mode == EPI_BWD)) return false;
  if (p.out8 != nullptr && p.out8_fmt != (p.epi_mode == EPI_BWD ? 1 : 0)) return false;
  if (p.epi_mode == EPI_BWD && p.mask == nullptr &&
      (p.aux == nullptr || p.aux_dtype != DT_BF16 || p.ldaux % 8 != 0 || (reinterpret_cast<uintptr_t>(p.aux) & 15)))
    return false;
  if (p.mask != nullptr && (p.ldmask % 32 != 0 || (reinterpret_cast<uintptr_t>(p.mask) & 7) != 0)) return false;
  if (p.out8 != nullptr && (p.ldout8 % 8 != 0 || (reinterpret_cast<uintptr_t>(p.out8) & 7) != 0 ||
                            p.out8_qscale == nullptr))
    return false;
  return true;
}

bool mfma_eligible(const GemmArgs& p) {
  if (p.in_dtype == DT_FP8) return fp8_eligible(p);
  if (p.force_generic || p.in_dtype != DT_BF16) return false;
  if (p.bias64 != nullptr || p.colsum64 != nullptr) return false;  // fp64 models: wide / generic paths
  if (p.out_dtype != DT_BF16 && p.out_dtype != DT_F32) return false;
  if (p.M < 64 || p.N < 64 || p.K < kBK || p.K % kBK != 0) return false;
  if (p.N % 8 != 0 || p.ldc % 8 != 0) return false;
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  if (!al16(p.A) || !al16(p.B) || !al16(p.C)) return false;
  if (p.lda % 8 != 0 || p.ldb % 8 != 0) return false;
  if (!p.a_kc && p.M % 8 != 0) return false;
  if (p.idx_ld % 2 != 0) return false;  // 4-element epilogue groups start at even element indices
  // fused stage epilogues: bf16 output only; accumulate: fp32 output only
  if (p.out_dtype == DT_F32 && p.epi_mode != EPI_STORE && p.epi_mode != EPI_OPT) return false;
  if (p.epi_mode == EPI_OPT) {  // fused optimizer update: plain gradient tiles, 16-B state vectors
    if (p.out_dtype != DT_F32 || p.bias != nullptr || p.colsum != nullptr || p.accumulate || p.mask != nullptr ||
        p.out8 != nullptr || p.ldc % 4 != 0 || p.opt.params == nullptr || !al16(p.opt.params))
      return false;
    if (p.opt.adam && (!al16(p.opt.exp_avg) || !al16(p.opt.exp_avg_sq))) return false;
    if (p.opt.shadow != nullptr &&
        (reinterpret_cast<uintptr_t>(p.opt.shadow) & (p.opt.shadow_dtype == DT_BF16 ? 7 : 15)) != 0)
      return false;
  }
  if (p.out_dtype == DT_BF16 && p.accumulate) return false;
  if (p.bias != nullptr && !al16(p.bias)) return false;
  if (p.out8 != nullptr && (p.out_dtype != DT_BF16 || p.out8_fmt != (p.epi_mode == EPI_BWD ? 1 : 0) ||
                            (p.epi_mode != EPI_BWD && p.epi_mode != EPI_FWD) || p.ldout8 % 8 != 0 ||
                            (reinterpret_cast<uintptr_t>(p.out8) & 7) != 0 || p.out8_qscale == nullptr))
    return false;
  if (p.mask != nullptr) {
    if (p.out_dtype != DT_BF16 || p.ldmask % 32 != 0 || (reinterpret_cast<uintptr_t>(p.mask) & 7) != 0) return false;
    if (p.epi_mode == EPI_BWD ? p.epi.act != ACT_RELU : p.epi_mode != EPI_FWD) return false;
    return true;
  }
  if (p.epi_mode == EPI_BWD) {
    if (p.aux == nullptr || p.ldaux % 8 != 0 || !al16(p.aux)) return false;
    if (p.aux_dtype != DT_BF16) return false;
  }
  return true;
}

int gemm_split(const GemmArgs& p) {
  // fp8 skinny shapes run better as 128x128 tiles (measured: split-K 256x256 -4%); the fp8
  // weight-gradient GEMM (both operands M/N-contiguous, 256-tiles only) splits like bf16
  // (and the N-contiguous-weight fp8 forward, VAR 15: 256x256 tiles only)
  const bool f8_dw = p.in_dtype == DT_FP8 && !p.b_kc;
  if ((p.in_dtype == DT_FP8 && !f8_dw) || !mfma_eligible(p)) return 1;
  if (w128_fixed(p)) return 1;
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  constexpr int kFill = 240;
  if (tiles >= kFill) return 1;
  // (fixed-kind forwards: 256x128 tiles instead, w128_fixed above; the generic-epilogue kinds
  // keep the split — r2: 1008 vs 881 TF/s alone but the mlp4 step slower,
  // profiles/r2_lab_skinny_fwd.txt)
  const int nk = p.K / (p.in_dtype == DT_FP8 ? 64 : kBK);
  for (int sp : {2, 4, 8})
    if (tiles * sp >= kFill && nk % sp == 0 && nk / sp >= 16) return sp;
  return 1;
}

int64_t gemm_split_ws_floats(const GemmArgs& p) {
  const int sp = gemm_split(p);
  if (sp <= 1) return 0;
  return static_cast<int64_t>((p.M + 255) / 256) * ((p.N + 255) / 256) * sp * 256 * 256;
}

// whole-tile epilogue stores write through (sc1) instead of leaving dirty L2 lines for the kernel
// boundary's write-back (GemmArgs::store_wt); on by default, PZ_GEMM_WT=0 turns it off. r4 A/B,
// mlp4 step: 1.1112 ms off, 1.1081 on; with PZ_OPT_NT on 1.1023 -> 1.0975
int store_wt_default() {
  static const int on = [] {
    const char* e = getenv("PZ_GEMM_WT");
    return e != nullptr ? atoi(e) : 1;
  }();
  return on;
}

// gemm_pair: both GEMMs in the weight-gradient layout (A and B M/N-contiguous), plain stores of
// whole 256 x 256 tiles, one K; returns the split-K factor of the pair, or 0 if it cannot be paired
int gemm_pair_split(const GemmArgs& a, const GemmArgs& b) {
  for (const GemmArgs* q : {&a, &b}) {
    const GemmArgs& p = *q;
    if (p.a_kc || p.b_kc || p.epi_mode != EPI_STORE || p.accumulate || p.force_generic) return 0;
    if (p.bias || p.colsum || p.mask || p.out8 || p.aux || p.bias64 || p.colsum64) return 0;
    if (p.M % 256 || p.N % 256 || p.K % 64 || !mfma_eligible(p)) return 0;
    if (p.in_dtype != DT_FP8 && (!buffer_ok(p) || epi_kind(p) != (p.out_dtype == DT_BF16 ? EK_STORE : EK_ANY)))
      return 0;
  }
  if (a.K != b.K || a.in_dtype != b.in_dtype || a.out_dtype != b.out_dtype || a.a_fmt != b.a_fmt ||
      a.b_fmt != b.b_fmt)
    return 0;
  if (a.in_dtype == DT_FP8 && a.out_dtype != DT_BF16) return 0;
  const int tiles = (a.M / 256) * (a.N / 256) + (b.M / 256) * (b.N / 256);
  const int nk = a.K / 64;
  constexpr int kFill = 240;
  for (int sp : {1, 2, 4, 8})
    if (tiles * sp >= kFill && nk % sp == 0 && nk / sp >= 16) return sp;
  return nk % 8 == 0 && nk / 8 >= 16 ? 8 : 1;
}

hipError_t gemm_pair(const GemmArgs& a, const GemmArgs& b, hipStream_t s) {
  const int split = gemm_pair_split(a, b);
  if (split == 0 || a.split_k != split || b.split_k != split) return hipErrorInvalidValue;
  if (split > 1 && (a.ws == nullptr || a.counters == nullptr || b.ws == nullptr || b.counters == nullptr))
    return hipErrorInvalidValue;
  GemmPairArgs g;
  g.p[0] = a;
  g.p[1] = b;
  g.p[0].store_wt = g.p[1].store_wt = store_wt_default();
  g.p[0].prio = g.p[1].prio = 1;
  g.nwg0 = (a.M / 256) * (a.N / 256) * split;
  const int nwg = g.nwg0 + (b.M / 256) * (b.N / 256) * split;
  if (a.in_dtype == DT_FP8) return launch_pair_cfg<uint16_t, 14, EK_STORE>(g, nwg, s);
  if (a.out_dtype == DT_BF16) return launch_pair_cfg<uint16_t, 30, EK_STORE>(g, nwg, s);
  return launch_pair_cfg<float, 30, EK_ANY>(g, nwg, s);
}

hipError_t gemm_mfma(const GemmArgs& in, hipStream_t s) {
  GemmArgs p = in;
  p.store_wt = store_wt_default();
  p.prio = 1;
  if (p.split_k > 1 && (p.ws == nullptr || p.counters == nullptr)) return hipErrorInvalidValue;
  if (p.in_dtype == DT_FP8) return launch_fp8(p, s);
  if (p.out_dtype == DT_BF16) return launch_tiles<uint16_t, uint16_t>(p, s);
  return launch_tiles<float, uint16_t>(p, s);
}
#endif  // PZ_GEMM_LAB

}  // namespace pz
