// Fused GEMM epilogue for bf16 outputs, staged through LDS (included by gemm_mfma.hip).
//
//   1. (EPI_BWD) the aux tile (stored stage output y) is read with coalesced 16-B row loads into
//      an LDS image of the C tile — instead of one dependent 8-B load per 4-element fragment;
//   2. the fused stage math runs as a few PASSES over the register accumulator tile — one pass
//      per enabled transform (bias, dropout-pre, activation, dropout-post or their derivatives).
//      Branches sit outside the unrolled fragment loops, so the code is the SUM of the passes,
//      not their product (a per-fragment switch produced ~5k basic blocks and I-cache stalls);
//   3. results go to the LDS image as bf16 and leave it as full 16-B-per-lane row segments;
//   4. ReLU stages: the forward also writes a 1-bit-per-element mask of y > 0 (tile-blocked, see
//      GemmArgs::mask), and the backward
//      reads 8 mask bytes per accumulator row instead of the 512-B aux row segment (dX GEMMs
//      with K = 1024 spent a third of their time streaming the bf16 aux tile);
//   5. fp8 consumers: the forward can also emit an e4m3 copy of y (scaled by a device-side
//      quantisation factor) and the tile's amax (delayed scaling for the next step).
// Image layout: row r holds BN bf16; 16-B chunk c of row r lives at chunk c ^ (r & 15).
//
// The accumulator layout is abstracted by a fragment LAYOUT: every lane owns, per accumulator
// ROW i, COLS groups of 4 consecutive output columns of ONE output row:
//   m = wave_m0 + MSTEP*i + m_lane(lane),  n = wave_n0 + n_off(j) + n_lane(lane) + r  (r < 4).
#pragma once

template <int BN>
PZ_DEV uint32_t cimg_off(int r, int col) {  // byte offset of element (r, col), col % 4 == 0
  const int c = col >> 3;
  return static_cast<uint32_t>(r * (BN * 2) + ((c ^ (r & 15)) << 4) + ((col & 4) << 1));
}

// 16x16x32 bf16 MFMA issued as mfma(B, A): acc[TM][TN] f32x4, lane -> m = lane&15, n = 4*(lane>>4)
template <int TM_, int TN_>
struct Lay16 {
  static constexpr int ROWS = TM_, COLS = TN_, MSTEP = 16, RED = 16;
  PZ_DEV static int m_lane(int lane) { return lane & 15; }
  PZ_DEV static int n_lane(int lane) { return 4 * (lane >> 4); }
  static constexpr int n_off(int j) { return 16 * j; }
  template <class Acc>
  PZ_DEV static f32x4_t get(const Acc& acc, int i, int j) { return acc[i][j]; }
};

// 32x32x64 f8 MFMA issued as mfma(B, A): acc[TM][TN] f32x16, lane -> m = lane&31,
// n = 8*(reg>>2) + 4*(lane>>5) + (reg&3): column group j = (block j>>2, register quad j&3)
template <int TM_, int TN_>
struct Lay32 {
  static constexpr int ROWS = TM_, COLS = 4 * TN_, MSTEP = 32, RED = 32;
  PZ_DEV static int m_lane(int lane) { return lane & 31; }
  PZ_DEV static int n_lane(int lane) { return 4 * (lane >> 5); }
  static constexpr int n_off(int j) { return 32 * (j >> 2) + 8 * (j & 3); }
  template <class Acc>
  PZ_DEV static f32x4_t get(const Acc& acc, int i, int j) {
    const int q = 4 * (j & 3);
    return f32x4_t{acc[i][j >> 2][q], acc[i][j >> 2][q + 1], acc[i][j >> 2][q + 2], acc[i][j >> 2][q + 3]};
  }
};

// The passes below work on ONE accumulator row (its COLS 4-element groups); the epilogue walks
// the rows so only one row's temporaries are live at a time.

// dropout: v[j][r] *= mask (scale or 0); pr_row = element-pair index of column group 0
template <class L>
PZ_DEV void dropout_row(f32x4_t (&v)[L::COLS], const EpiSpec& e, uint32_t key, uint32_t pr_row) {
  if (e.drop_all) {
#pragma unroll
    for (int j = 0; j < L::COLS; ++j) v[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const uint32_t th = e.thresh16;
  const float sc = e.scale;
#pragma unroll
  for (int j = 0; j < L::COLS; ++j) {
    const uint32_t pr = pr_row + static_cast<uint32_t>(L::n_off(j) / 2);
    const uint32_t b0 = mix32(pr ^ key), b1 = mix32((pr + 1u) ^ key);
    v[j][0] *= (b0 & 0xFFFFu) >= th ? sc : 0.f;
    v[j][1] *= (b0 >> 16) >= th ? sc : 0.f;
    v[j][2] *= (b1 & 0xFFFFu) >= th ? sc : 0.f;
    v[j][3] *= (b1 >> 16) >= th ? sc : 0.f;
  }
}

// dropout -> ReLU -> dropout (every hidden ReLU stage of the reference MLPs): the scale is
// positive, so relu(z * m1 * s) * m2 * s = (m1 & m2) ? relu(z) * s^2 : 0 — both keep decisions are
// combined before ONE select and multiply per element (the backward applies the same s^2)
template <class L>
PZ_DEV void dropout_relu_dropout_row(f32x4_t (&v)[L::COLS], const EpiSpec& e, uint32_t pr_row) {
  const uint32_t th = e.thresh16;
  const float s2 = e.scale * e.scale;
#pragma unroll
  for (int j = 0; j < L::COLS; ++j) {
    const uint32_t pr = pr_row + static_cast<uint32_t>(L::n_off(j) / 2);
    const uint32_t a0 = mix32(pr ^ e.key_pre), a1 = mix32((pr + 1u) ^ e.key_pre);
    const uint32_t c0 = mix32(pr ^ e.key_post), c1 = mix32((pr + 1u) ^ e.key_post);
    const bool k[4] = {(a0 & 0xFFFFu) >= th && (c0 & 0xFFFFu) >= th, (a0 >> 16) >= th && (c0 >> 16) >= th,
                       (a1 & 0xFFFFu) >= th && (c1 & 0xFFFFu) >= th, (a1 >> 16) >= th && (c1 >> 16) >= th};
#pragma unroll
    for (int r = 0; r < 4; ++r) v[j][r] = k[r] ? fmaxf(v[j][r], 0.f) * s2 : 0.f;
  }
}

// EK_RELU's single pass: keep = (drop_pre ? pre bit : 1) & (drop_post ? post bit : 1), then
// y = keep ? (act(z) * m1) * m2 : 0. With a positive scale, act(z * m1) == act(z) * m1 for act in
// {NONE, ReLU}, so this equals the separate passes bit for bit when the host passes (m1, m2) =
// (scale^2, 1) for ReLU with both dropouts (the combined form above) and (pre scale or 1, post
// scale or 1) otherwise (multiplying by 1 is exact)
template <class L>
PZ_DEV void relu_dropout_row(f32x4_t (&v)[L::COLS], const EpiSpec& e, uint32_t pr_row, bool relu, float m1, float m2) {
  const uint32_t th = e.thresh16;
#pragma unroll
  for (int j = 0; j < L::COLS; ++j) {
    const uint32_t pr = pr_row + static_cast<uint32_t>(L::n_off(j) / 2);
    // keep decisions as lane masks (compares -> SGPR pairs, ANDed on the scalar unit)
    bool k[4] = {!e.drop_all, !e.drop_all, !e.drop_all, !e.drop_all};
    if (e.drop_pre) {
      const uint32_t a0 = mix32(pr ^ e.key_pre), a1 = mix32((pr + 1u) ^ e.key_pre);
      k[0] = k[0] && (a0 & 0xFFFFu) >= th;
      k[1] = k[1] && (a0 >> 16) >= th;
      k[2] = k[2] && (a1 & 0xFFFFu) >= th;
      k[3] = k[3] && (a1 >> 16) >= th;
    }
    if (e.drop_post) {
      const uint32_t c0 = mix32(pr ^ e.key_post), c1 = mix32((pr + 1u) ^ e.key_post);
      k[0] = k[0] && (c0 & 0xFFFFu) >= th;
      k[1] = k[1] && (c0 >> 16) >= th;
      k[2] = k[2] && (c1 & 0xFFFFu) >= th;
      k[3] = k[3] && (c1 >> 16) >= th;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = relu ? fmaxf(v[j][r], 0.f) : v[j][r];
      v[j][r] = k[r] ? (x * m1) * m2 : 0.f;
    }
  }
}

template <int COLS>
PZ_DEV void act_fwd_row(f32x4_t (&v)[COLS], int act) {
#define PZ_ACT_LOOP(expr)                                                       \
  _Pragma("unroll") for (int j = 0; j < COLS; ++j) _Pragma("unroll") for (int r = 0; r < 4; ++r) { \
    const float x = v[j][r]; v[j][r] = (expr); }
  // branch-free fast forms (the result is rounded to bf16): sigmoid = 1/(1+e^-x),
  // tanh = 1 - 2/(e^{2x}+1) (saturates correctly for |x| large, e^{2x} -> inf or 0)
  if (act == ACT_RELU) { PZ_ACT_LOOP(x > 0.f ? x : 0.f) }
  else if (act == ACT_SIGMOID) { PZ_ACT_LOOP(__frcp_rn(1.f + __expf(-x))) }
  else if (act == ACT_TANH) { PZ_ACT_LOOP(1.f - 2.f * __frcp_rn(__expf(2.f * x) + 1.f)) }
#undef PZ_ACT_LOOP
}

// v *= act'(a) with a = y * yscale; y (stored stage output) read per group from the LDS image;
// ml = tile row, nl = tile column of group 0
template <int BN, class L>
PZ_DEV void act_bwd_row(f32x4_t (&v)[L::COLS], const PZ_LDS char* img, int ml, int nl, int act, float yscale) {
#define PZ_ACTB_LOOP(expr)                                                                                 \
  _Pragma("unroll") for (int j = 0; j < L::COLS; ++j) {                                                    \
    const u32x2_t y = *reinterpret_cast<const PZ_LDS u32x2_t*>(img + cimg_off<BN>(ml, nl + L::n_off(j)));  \
    const float ys[4] = {bf2f(y[0] & 0xFFFF), bf2f(y[0] >> 16), bf2f(y[1] & 0xFFFF), bf2f(y[1] >> 16)};     \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) { const float a = ys[r] * yscale; v[j][r] *= (expr); }    \
  }
  if (act == ACT_RELU) { PZ_ACTB_LOOP(a > 0.f ? 1.f : 0.f) }
  else if (act == ACT_SIGMOID) { PZ_ACTB_LOOP(a * (1.f - a)) }
  else if (act == ACT_TANH) { PZ_ACTB_LOOP(1.f - a * a) }
#undef PZ_ACTB_LOOP
}

// v *= relu'(.) from the stage's ReLU bitmask: `bits` = the mask bits of the wave's 64 or 128
// columns of this row; group j element r is bit n_off(j) + n_lane + r (never straddles a word)
template <class L, int NWORD>
PZ_DEV void act_bwd_mask_row(f32x4_t (&v)[L::COLS], const uint32_t (&bits)[NWORD], int nlane) {
#pragma unroll
  for (int j = 0; j < L::COLS; ++j) {
    const uint32_t w = bits[L::n_off(j) >> 5] >> ((L::n_off(j) & 31) + nlane);
    // bit r -> an all-ones / all-zeros word (v_bfe_i32) ANDed onto the float: 2 VALU per element
    // instead of and + compare + select
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[j][r] = __uint_as_float(__float_as_uint(v[j][r]) &
                                static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(w), r, 1)));
  }
}

// ReLU bitmask byte of 8 packed bf16 (bit b = element b > 0). A bf16 is > 0 iff its sign is clear
// and it is nonzero: per packed pair, ((w & 0x7FFF7FFF) + 0x7FFF7FFF) carries into bit 15 / 31
// exactly for a nonzero magnitude (no carry crosses the halves) and ~w clears the negative ones —
// 3 VALU per pair instead of 6 (positive NaN payloads count as > 0, as the compare form did)
PZ_DEV uint32_t relu_bits8(const u32x4_t& v) {
  uint32_t byte = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t pos = ((v[q] & 0x7FFF7FFFu) + 0x7FFF7FFFu) & ~v[q] & 0x80008000u;
    byte |= ((pos >> 15) & 1u) << (2 * q);
    byte |= (pos >> 31) << (2 * q + 1);
  }
  return byte;
}

// Compile-time epilogue kinds. The generic epilogue (EK_ANY) carries every transform — sigmoid /
// tanh with IEEE reciprocals, both dropout forms, aux-tile derivatives — unrolled over the tile's
// rows: ~20k instructions, and it measured ~5 us per tile of instruction-fetch stalls with EVERY
// transform switched off (tools/gemm_stamps.hip: stage-math phase 8.6 us in EPI_FWD with nothing
// enabled vs 3.3 us in EPI_STORE). The MLP's stages use three shapes, each specialised to only the
// code it runs (host: epi_kind()):
//   EK_STORE    alpha * acc -> bf16 (weight gradients)
//   EK_RELU     EPI_FWD with act NONE / RELU: bias, dropout pre / post, ReLU bitmask, fp8 copy
//   EK_BWD_MASK EPI_BWD through a ReLU stage from its bitmask: dropout scales, column sums, e5m2 copy
constexpr int EK_ANY = 0, EK_STORE = 1, EK_RELU = 2, EK_BWD_MASK = 3;
// Fixed forward stages (EPI_FWD, no colsum, not drop_all): the activation and both dropout flags
// are compile-time, so a row is ONE straight-line pass — no per-row flag branches, no untaken hash
// copies. EK_RELU with every transform switched off still ran ~1,400 more VALU instructions per
// wave and tile than the plain store (its 6.3k-instruction stage-math section: 3.6k I-cache
// misses per launch vs 0.6k; profiles/r3_epilogue_fixed_kinds.txt). The MLP's three stage
// shapes: linear -> ReLU -> dropout (first hidden stage), linear -> dropout -> ReLU -> dropout
// (later hidden stages), linear -> dropout (the logits).
constexpr int EK_F_RELU_POST = 4, EK_F_RELU_PREPOST = 5, EK_F_PRE = 6;
constexpr bool ek_fixed(int ek) { return ek >= EK_F_RELU_POST && ek <= EK_F_PRE; }
constexpr bool ek_relu(int ek) { return ek == EK_F_RELU_POST || ek == EK_F_RELU_PREPOST; }
constexpr bool ek_pre(int ek) { return ek == EK_F_RELU_PREPOST || ek == EK_F_PRE; }
constexpr bool ek_post(int ek) { return ek == EK_F_RELU_POST || ek == EK_F_RELU_PREPOST; }

// one row of a fixed forward stage: y = keep ? act(z) * sc : 0 with keep = pre bit & post bit and
// sc = the product of the enabled dropouts' scales (both: act(z * m1 * s) * m2 * s with s > 0 and
// act in {identity, ReLU} equals (m1 & m2) ? act(z) * s^2 : 0 — the EK_RELU forms bit for bit)
template <class L, int EK>
PZ_DEV void fixed_fwd_row(f32x4_t (&v)[L::COLS], const EpiSpec& e, uint32_t pr_row, float sc) {
  const uint32_t th = e.thresh16;
#pragma unroll
  for (int j = 0; j < L::COLS; ++j) {
    const uint32_t pr = pr_row + static_cast<uint32_t>(L::n_off(j) / 2);
    bool k0 = true, k1 = true, k2 = true, k3 = true;
    if constexpr (ek_pre(EK)) {
      const uint32_t a0 = mix32(pr ^ e.key_pre), a1 = mix32((pr + 1u) ^ e.key_pre);
      k0 = (a0 & 0xFFFFu) >= th; k1 = (a0 >> 16) >= th; k2 = (a1 & 0xFFFFu) >= th; k3 = (a1 >> 16) >= th;
    }
    if constexpr (ek_post(EK)) {
      const uint32_t c0 = mix32(pr ^ e.key_post), c1 = mix32((pr + 1u) ^ e.key_post);
      k0 = k0 && (c0 & 0xFFFFu) >= th; k1 = k1 && (c0 >> 16) >= th;
      k2 = k2 && (c1 & 0xFFFFu) >= th; k3 = k3 && (c1 >> 16) >= th;
    }
    const bool k[4] = {k0, k1, k2, k3};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float x = ek_relu(EK) ? fmaxf(v[j][r], 0.f) : v[j][r];
      v[j][r] = k[r] ? x * sc : 0.f;
    }
  }
}

// byte of the tile-blocked ReLU bitmask holding element (m, n) (GemmArgs::mask)
PZ_DEV int64_t mask_off(int64_t m, int n, int64_t ldmask) {
  return (m >> 8) * 256 * ldmask + static_cast<int64_t>(n >> 8) * 8192 + (m & 255) * 32 + ((n & 255) >> 3);
}

template <int BM, int BN, int WM, int WN, class L, bool FWD_ONLY = false, int EK = EK_ANY, class Acc>
PZ_DEV void epilogue_lds(const GemmArgs& p, Acc& acc, PZ_LDS char* smem, int m0, int n0, int wm, int wn, int lane,
                         float alpha) {
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int ROWS = L::ROWS, COLS = L::COLS;
  constexpr int CHUNKS_PER_ROW = BN / 8;
  constexpr int ROWS_PER_PASS = NT / CHUNKS_PER_ROW;
  constexpr int PASSES = BM / ROWS_PER_PASS;
  static_assert(WTN == 64 || WTN == 128, "the ReLU bitmask epilogue reads 64- or 128-column wave rows");
  constexpr int MWORDS = WTN / 32;  // bitmask words per accumulator row
  const int tid = threadIdx.x;
  const int my_row = tid / CHUNKS_PER_ROW, my_chunk = tid % CHUNKS_PER_ROW;
  // FWD_ONLY: no colsum / backward code
  const bool bwd = EK == EK_BWD_MASK || (EK == EK_ANY && !FWD_ONLY && p.epi_mode == EPI_BWD);
  const EpiSpec e = epi_resolve(p.epi);  // graph-replayed steps: epoch from the device counter
  const int ml0 = wm * WTM + L::m_lane(lane);  // + MSTEP*i
  const int nlane = L::n_lane(lane);
  const int nl0 = wn * WTN + nlane;            // + n_off(j)
  const bool use_mask = EK == EK_BWD_MASK || (EK != EK_STORE && p.mask != nullptr);
  constexpr bool kColsum = !FWD_ONLY && (EK == EK_ANY || EK == EK_BWD_MASK);

  // ReLU bitmask (EPI_BWD): 8 (16) bytes per accumulator row of a 64 (128)-column wave tile,
  // issued before the barrier so the loads fly while the slower waves finish their last MFMAs
  uint32_t mbits[ROWS][MWORDS];
  if (bwd && use_mask) {
    // (the tile's rows lie in one 256-row block: 32-B row pitch, wave-column aligned reads)
    const uint8_t* mrow = p.mask + mask_off(m0, n0 + wn * WTN, p.ldmask);
#pragma unroll
    for (int i = 0; i < ROWS; ++i) {
      const int m = m0 + ml0 + L::MSTEP * i;
      const uint8_t* src = mrow + (ml0 + L::MSTEP * i) * 32;
      if constexpr (MWORDS == 2) {
        const u32x2_t b = m < p.M ? *reinterpret_cast<const u32x2_t*>(src) : u32x2_t{0u, 0u};
        mbits[i][0] = b[0];
        mbits[i][1] = b[1];
      } else {
        const u32x4_t b = m < p.M ? *reinterpret_cast<const u32x4_t*>(src) : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
        for (int q = 0; q < 4; ++q) mbits[i][q] = b[q];
      }
    }
  }

  __syncthreads();  // every wave is done reading the ring
  if (EK == EK_ANY && bwd && !use_mask) {
    const uint16_t* __restrict__ aux = static_cast<const uint16_t*>(p.aux);
    u32x4_t v[PASSES];
#pragma unroll
    for (int s = 0; s < PASSES; ++s) {
      const int r = s * ROWS_PER_PASS + my_row;
      const int gm = m0 + r, gn = n0 + my_chunk * 8;
      v[s] = (gm < p.M && gn < p.N) ? *reinterpret_cast<const u32x4_t*>(aux + static_cast<int64_t>(gm) * p.ldaux + gn)
                                    : u32x4_t{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int s = 0; s < PASSES; ++s)
      *reinterpret_cast<PZ_LDS u32x4_t*>(smem + cimg_off<BN>(s * ROWS_PER_PASS + my_row, my_chunk * 8)) = v[s];
    __syncthreads();
  }

  // ---- the stage math: per accumulator row, one pass per enabled transform, then bf16 into the
  // LDS image. Each lane only rewrites the cells whose y it read itself (no barrier needed).
  f32x4_t bias4[COLS];
#pragma unroll
  for (int j = 0; j < COLS; ++j) {
    const int n = n0 + nl0 + L::n_off(j);
    bias4[j] = ((EK == EK_ANY || EK == EK_RELU || ek_fixed(EK)) && !bwd && p.bias != nullptr && n < p.N)
                   ? *reinterpret_cast<const f32x4_t*>(p.bias + n)
                   : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  f32x4_t cs[COLS];
#pragma unroll
  for (int j = 0; j < COLS; ++j) cs[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const uint64_t col0 = static_cast<uint64_t>(n0 + nl0);
  const float bwd_scale = (e.drop_post ? e.scale : 1.f) * (e.drop_pre ? e.scale : 1.f);
  const bool relu_on = e.act == ACT_RELU;
  const bool both = e.drop_pre && e.drop_post;
  const float rd_m1 = relu_on && both ? e.scale * e.scale : (e.drop_pre ? e.scale : 1.f);
  const float rd_m2 = relu_on && both ? 1.f : (e.drop_post ? e.scale : 1.f);
  const float fixed_sc = (ek_pre(EK) ? e.scale : 1.f) * (ek_post(EK) ? e.scale : 1.f);
  static_for<ROWS>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int ml = ml0 + L::MSTEP * i;
    const uint32_t pr_row =
        static_cast<uint32_t>((static_cast<uint64_t>(m0 + ml) * static_cast<uint64_t>(p.idx_ld) + col0) >> 1);
    f32x4_t v[COLS];
#pragma unroll
    for (int j = 0; j < COLS; ++j) v[j] = L::get(acc, i, j) * alpha + bias4[j];
    if constexpr (EK == EK_STORE) {
    } else if constexpr (ek_fixed(EK)) {
      fixed_fwd_row<L, EK>(v, e, pr_row, fixed_sc);
    } else if constexpr (EK == EK_RELU) {  // (dispatcher: EPI_FWD, act NONE or RELU)
      if (relu_on && both && !e.drop_all) dropout_relu_dropout_row<L>(v, e, pr_row);  // hidden ReLU stages
      else relu_dropout_row<L>(v, e, pr_row, relu_on, rd_m1, rd_m2);
    } else if (!bwd) {
      if (p.epi_mode == EPI_FWD) {
        if (e.drop_pre && e.drop_post && e.act == ACT_RELU && !e.drop_all) {
          dropout_relu_dropout_row<L>(v, e, pr_row);
        } else {
          if (e.drop_pre) dropout_row<L>(v, e, e.key_pre, pr_row);
          if (e.act != ACT_NONE) act_fwd_row<COLS>(v, e.act);
          if (e.drop_post) dropout_row<L>(v, e, e.key_post, pr_row);
        }
      }
    } else if (EK == EK_BWD_MASK || use_mask) {
      // ReLU stage: y > 0  <=>  kept by drop_post AND kept by drop_pre AND z > 0, so the whole
      // derivative chain is one bit times the dropout scales — no hashes in the backward
      act_bwd_mask_row<L, MWORDS>(v, mbits[i], nlane);
#pragma unroll
      for (int j = 0; j < COLS; ++j) v[j] *= bwd_scale;
    } else if constexpr (EK == EK_ANY) {
      if (e.drop_post) dropout_row<L>(v, e, e.key_post, pr_row);
      if (e.act != ACT_NONE) act_bwd_row<BN, L>(v, smem, ml, nl0, e.act, e.drop_post ? e.inv_scale : 1.f);
      if (e.drop_pre) dropout_row<L>(v, e, e.key_pre, pr_row);
    }
#pragma unroll
    for (int j = 0; j < COLS; ++j)
      *reinterpret_cast<PZ_LDS u32x2_t*>(smem + cimg_off<BN>(ml, nl0 + L::n_off(j))) =
          u32x2_t{pack_bf2(v[j][0], v[j][1]), pack_bf2(v[j][2], v[j][3])};
    if (kColsum && p.colsum != nullptr && m0 + ml < p.M) {
#pragma unroll
      for (int j = 0; j < COLS; ++j) cs[j] += v[j];
    }
    __builtin_amdgcn_sched_barrier(0);  // keep rows apart: bounds the live temporaries
  });
  // column sums: reduce across the lanes now, issue the atomics after the tile is stored — the
  // barrier below would otherwise wait (vmcnt(0)) for every contended atomic to come back
  if (kColsum && p.colsum != nullptr) {
#pragma unroll
    for (int j = 0; j < COLS; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        cs[j][r] = group_sum<L::RED>(cs[j][r]);
  }
  PZ_STAMP(5);  // (diagnostic builds: stage math + LDS image writes done, wave 0)
  __syncthreads();
  uint16_t* __restrict__ Cp = static_cast<uint16_t*>(p.C);
  // fp8 copy of the stored bf16 tile: e4m3 activations (forward) / e5m2 dZ (backward)
  const bool want8 = EK != EK_STORE && p.out8 != nullptr && (bwd ? p.out8_fmt == 1 : p.out8_fmt == 0);
  const float qs = want8 ? *p.out8_qscale : 1.f;
  float amax = 0.f;
  // Full tiles of the specialised kinds: every pass's image chunk is read up front (the
  // accumulators are dead: 64 VGPRs of 16-B chunks fit), then the stores go out back to back
  // from one base address advanced by a constant stride. The generic per-pass loop below waited
  // on each ds_read before its store and recomputed a 64-bit row address (two quarter-rate
  // multiplies) per pass behind per-pass range branches.
  const bool full_tile = EK != EK_ANY && m0 + BM <= p.M && n0 + BN <= p.N;
  if (full_tile) {
    u32x4_t vv[PASSES];
#pragma unroll
    for (int s = 0; s < PASSES; ++s)
      vv[s] = *reinterpret_cast<const PZ_LDS u32x4_t*>(smem + cimg_off<BN>(s * ROWS_PER_PASS + my_row, my_chunk * 8));
    const int gn = n0 + my_chunk * 8;
    const int64_t row0 = static_cast<int64_t>(m0 + my_row);
    // p.store_wt: write-through (sc1) buffer stores from the tile's base (32-bit byte offsets within
    // the tile's rows), so the kernel leaves no dirty lines behind in the L2s
    constexpr int kSc1 = 16;
    const bool wt = p.store_wt != 0;
    if (Cp != nullptr) {  // (fp8 policy: a bf16 output nobody reads is not written — only its copies)
      uint16_t* dst = Cp + row0 * p.ldc + gn;
      const int64_t step = static_cast<int64_t>(ROWS_PER_PASS) * p.ldc;
      if (wt) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(Cp + static_cast<int64_t>(m0) * p.ldc, 0, 0x7FFFFFFF, 0x00020000);
        const uint32_t off0 = static_cast<uint32_t>((my_row * p.ldc + gn) * 2);
#pragma unroll
        for (int s = 0; s < PASSES; ++s)
          __builtin_amdgcn_raw_buffer_store_b128(vv[s], rs, off0 + static_cast<uint32_t>(s * step * 2), 0, kSc1);
      } else {
#pragma unroll
        for (int s = 0; s < PASSES; ++s) *reinterpret_cast<u32x4_t*>(dst + s * step) = vv[s];
      }
    }
    if (!bwd && use_mask) {
      // tile-blocked mask: row r of the tile at +32 r, chunk c at +c — with BN = 256 the pass's
      // 512 bytes are contiguous (offset s * 512 + tid), written as 4-B words by the quad leaders
      uint8_t* mtile = p.mask + mask_off(m0, n0, p.ldmask);
      uint8_t* mdst = mtile + my_row * 32 + my_chunk;
      constexpr int mstep = ROWS_PER_PASS * 32;
      const auto rsm = __builtin_amdgcn_make_buffer_rsrc(mtile, 0, 0x7FFFFFFF, 0x00020000);
      const uint32_t moff0 = static_cast<uint32_t>(my_row * 32 + my_chunk);
#pragma unroll
      for (int s = 0; s < PASSES; ++s) {
        const uint32_t byte = relu_bits8(vv[s]);  // bit b = element gn+b > 0
        const uint32_t b1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0x55, 0xF, 0xF, false));
        const uint32_t b2 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0xAA, 0xF, 0xF, false));
        const uint32_t b3 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0xFF, 0xF, 0xF, false));
        const uint32_t word = byte | (b1 << 8) | (b2 << 16) | (b3 << 24);
        if ((my_chunk & 3) == 0) {
          if (wt) __builtin_amdgcn_raw_buffer_store_b32(word, rsm, moff0 + static_cast<uint32_t>(s * mstep), 0, kSc1);
          else *reinterpret_cast<uint32_t*>(mdst + s * mstep) = word;
        }
      }
    }
    if (want8) {  // fp8 copy of the stored bf16 values + running |y| max
      uint8_t* d8 = p.out8 + row0 * p.ldout8 + gn;
      const int64_t step8 = static_cast<int64_t>(ROWS_PER_PASS) * p.ldout8;
      const auto rs8 = __builtin_amdgcn_make_buffer_rsrc(p.out8 + static_cast<int64_t>(m0) * p.ldout8, 0, 0x7FFFFFFF,
                                                         0x00020000);
      const uint32_t off8 = static_cast<uint32_t>(my_row * p.ldout8 + gn);
#pragma unroll
      for (int s = 0; s < PASSES; ++s) {
        float x[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x[2 * q] = bf2f(vv[s][q] & 0xFFFFu);
          x[2 * q + 1] = bf2f(vv[s][q] >> 16);
          amax = fmaxf(amax, fmaxf(fabsf(x[2 * q]), fabsf(x[2 * q + 1])));
        }
        const u32x2_t q8 = bwd ? to_e5m2x8(x, qs) : to_e4m3x8(x, qs);
        if (wt) __builtin_amdgcn_raw_buffer_store_b64(q8, rs8, off8 + static_cast<uint32_t>(s * step8), 0, kSc1);
        else *reinterpret_cast<u32x2_t*>(d8 + s * step8) = q8;
      }
    }
  }
  // ragged tiles (and the generic kind): one pass at a time with range checks; the fixed forward
  // kinds keep it rolled by 4 (it indexes no accumulator)
  constexpr int kStoreUnroll = ek_fixed(EK) ? 4 : PASSES;
  if (!full_tile) {
#pragma unroll kStoreUnroll
  for (int s = 0; s < PASSES; ++s) {
    const int r = s * ROWS_PER_PASS + my_row;
    const int gm = m0 + r, gn = n0 + my_chunk * 8;
    const u32x4_t v = *reinterpret_cast<const PZ_LDS u32x4_t*>(smem + cimg_off<BN>(r, my_chunk * 8));
    const bool in_range = gm < p.M && gn < p.N;
    uint32_t byte = 0;  // ReLU bitmask of this 8-column chunk: bit b = element gn+b > 0
    if (in_range) {
      if (Cp != nullptr)  // (fp8 policy: a bf16 output nobody reads is not written — only its copies)
        *reinterpret_cast<u32x4_t*>(Cp + static_cast<int64_t>(gm) * p.ldc + gn) = v;
      if (!bwd && use_mask) byte = relu_bits8(v);
      if (want8) {  // e4m3 copy of the bf16 values + running |y| max
        float x[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x[2 * q] = bf2f(v[q] & 0xFFFFu);
          x[2 * q + 1] = bf2f(v[q] >> 16);
          amax = fmaxf(amax, fmaxf(fabsf(x[2 * q]), fabsf(x[2 * q + 1])));
        }
        *reinterpret_cast<u32x2_t*>(p.out8 + static_cast<int64_t>(gm) * p.ldout8 + gn) =
            bwd ? to_e5m2x8(x, qs) : to_e4m3x8(x, qs);
      }
    }
    if (!bwd && use_mask) {  // 4 neighbouring chunks of a row -> one 4-byte store (not 4 byte stores)
      // the 4 chunks are one DPP quad (lane % 4 == chunk % 4): quad_perm broadcasts of lanes 1..3
      // (full-rate VALU) instead of ds_bpermute round trips through the LDS the image reads use
      const uint32_t b1 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0x55, 0xF, 0xF, false));
      const uint32_t b2 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0xAA, 0xF, 0xF, false));
      const uint32_t b3 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(byte), 0xFF, 0xF, 0xF, false));
      if (in_range && (my_chunk & 3) == 0)
        *reinterpret_cast<uint32_t*>(p.mask + mask_off(gm, gn, p.ldmask)) = byte | (b1 << 8) | (b2 << 16) | (b3 << 24);
    }
  }
  }  // !full_tile
  PZ_STAMP(6);  // (stores issued)
  if (want8 && p.amax != nullptr) {  // one atomic per workgroup (same-address atomics serialise)
    amax = wave_max(amax);
    constexpr int NW = WM * WN;
    __syncthreads();  // the LDS image has been read out
    PZ_LDS float* part = (PZ_LDS float*)(smem);
    if (lane == 0) part[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0) {
      float m = part[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) m = fmaxf(m, part[w]);
      atomicMax(reinterpret_cast<unsigned int*>(p.amax), __float_as_uint(m));
    }
  }
  if (kColsum && p.colsum != nullptr) {
    // the WM waves that share a column range meet in LDS (the image has been read out), then ONE
    // atomic per tile column, 64 consecutive columns per wave instruction: the full-rate atomic
    // shape (256 contiguous bytes), instead of 4-lane instructions from every wave (measured:
    // the column sums cost 11% of the K = 1024 dX GEMM that way)
    PZ_LDS float* part = (PZ_LDS float*)(smem);  // [WM][BN]
    __syncthreads();
    if ((lane & (L::RED - 1)) == 0) {
#pragma unroll
      for (int j = 0; j < COLS; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[wm * BN + nl0 + L::n_off(j) + r] = cs[j][r];
    }
    __syncthreads();
    if (p.cs_ws != nullptr) {  // deterministic: this tile's partial row, then the ordered folds
      const int tiles_m = (p.M + BM - 1) / BM, tm = m0 / BM;
      const int cols = min(BN, p.N - n0);
      for (int c = tid; c < cols; c += NT) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) s += part[w * BN + c];
        st_wt(p.cs_ws + static_cast<int64_t>(tm) * p.N + n0 + c, s);
      }
      constexpr int kGroup = 64;
      det_colsum<NT>(p.cs_ws + n0, p.cs_tickets + (n0 / BN) * ((tiles_m + kGroup - 1) / kGroup + 1), tiles_m, kGroup, tm,
                     cols, p.N, p.colsum + n0, reinterpret_cast<PZ_LDS int*>(smem + WM * BN * 4));
    } else {
      for (int c = tid; c < BN; c += NT) {  // fire-and-forget: nothing waits for them in this kernel
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) s += part[w * BN + c];
        if (n0 + c < p.N) atomicAdd(p.colsum + n0 + c, s);
      }
    }
  }
}
