// Fused GEMM epilogue for bf16 outputs, staged through LDS (included by gemm_mfma.hip).
//
//   1. (EPI_BWD) the aux tile (stored stage output y) is read with coalesced 16-B row loads into
//      an LDS image of the C tile — instead of one dependent 8-B load per 4-element fragment;
//   2. the fused stage math runs as a few PASSES over the register accumulator tile — one pass
//      per enabled transform (bias, dropout-pre, activation, dropout-post or their derivatives).
//      Branches sit outside the unrolled fragment loops, so the code is the SUM of the passes,
//      not their product (a per-fragment switch produced ~5k basic blocks and I-cache stalls);
//   3. results go to the LDS image as bf16 and leave it as full 16-B-per-lane row segments;
//   4. ReLU stages: the forward also writes a 1-bit-per-element mask of y > 0, and the backward
//      reads 8 mask bytes per accumulator row instead of the 512-B aux row segment (dX GEMMs
//      with K = 1024 spent a third of their time streaming the bf16 aux tile).
// Image layout: row r holds BN bf16; 16-B chunk c of row r lives at chunk c ^ (r & 15).
#pragma once

template <int BN>
PZ_DEV uint32_t cimg_off(int r, int col) {  // byte offset of element (r, col), col % 4 == 0
  const int c = col >> 3;
  return static_cast<uint32_t>(r * (BN * 2) + ((c ^ (r & 15)) << 4) + ((col & 4) << 1));
}

// The passes below work on ONE fragment row (the TN 4-element fragments of accumulator row i);
// the epilogue walks the rows so only one row's temporaries are live at a time.

// dropout: v[j][r] *= mask (scale or 0); pr0 = element-pair index of fragment (i, 0)
template <int TN>
PZ_DEV void dropout_row(f32x4_t (&v)[TN], const EpiSpec& e, uint32_t key, uint32_t pr0) {
  if (e.drop_all) {
#pragma unroll
    for (int j = 0; j < TN; ++j) v[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const uint32_t th = e.thresh16;
  const float sc = e.scale;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const uint32_t pr = pr0 + static_cast<uint32_t>(j) * 8u;
    const uint32_t b0 = mix32(pr ^ key), b1 = mix32((pr + 1u) ^ key);
    v[j][0] *= (b0 & 0xFFFFu) >= th ? sc : 0.f;
    v[j][1] *= (b0 >> 16) >= th ? sc : 0.f;
    v[j][2] *= (b1 & 0xFFFFu) >= th ? sc : 0.f;
    v[j][3] *= (b1 >> 16) >= th ? sc : 0.f;
  }
}

template <int TN>
PZ_DEV void act_fwd_row(f32x4_t (&v)[TN], int act) {
#define PZ_ACT_LOOP(expr)                                                       \
  _Pragma("unroll") for (int j = 0; j < TN; ++j) _Pragma("unroll") for (int r = 0; r < 4; ++r) { \
    const float x = v[j][r]; v[j][r] = (expr); }
  // branch-free fast forms (the result is rounded to bf16): sigmoid = 1/(1+e^-x),
  // tanh = 1 - 2/(e^{2x}+1) (saturates correctly for |x| large, e^{2x} -> inf or 0)
  if (act == ACT_RELU) { PZ_ACT_LOOP(x > 0.f ? x : 0.f) }
  else if (act == ACT_SIGMOID) { PZ_ACT_LOOP(__frcp_rn(1.f + __expf(-x))) }
  else if (act == ACT_TANH) { PZ_ACT_LOOP(1.f - 2.f * __frcp_rn(__expf(2.f * x) + 1.f)) }
#undef PZ_ACT_LOOP
}

// v *= act'(a) with a = y * yscale; y (stored stage output) read per fragment from the LDS image
template <int BN, int TN>
PZ_DEV void act_bwd_row(f32x4_t (&v)[TN], const PZ_LDS char* img, int ml, int nl0, int act, float yscale) {
#define PZ_ACTB_LOOP(expr)                                                                           \
  _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                                   \
    const u32x2_t y = *reinterpret_cast<const PZ_LDS u32x2_t*>(img + cimg_off<BN>(ml, nl0 + 16 * j)); \
    const float ys[4] = {bf2f(y[0] & 0xFFFF), bf2f(y[0] >> 16), bf2f(y[1] & 0xFFFF), bf2f(y[1] >> 16)};  \
    _Pragma("unroll") for (int r = 0; r < 4; ++r) { const float a = ys[r] * yscale; v[j][r] *= (expr); } \
  }
  if (act == ACT_RELU) { PZ_ACTB_LOOP(a > 0.f ? 1.f : 0.f) }
  else if (act == ACT_SIGMOID) { PZ_ACTB_LOOP(a * (1.f - a)) }
  else if (act == ACT_TANH) { PZ_ACTB_LOOP(1.f - a * a) }
#undef PZ_ACTB_LOOP
}

// v *= relu'(.) from the stage's ReLU bitmask: `bits` = the 64 mask bits of the wave's 64 columns
// of this row (bit c = column c of the wave tile); fragment j, element r sits at 16j + g4 + r
template <int TN>
PZ_DEV void act_bwd_mask_row(f32x4_t (&v)[TN], u32x2_t bits, int g4) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const uint32_t w = bits[j >> 1] >> (16 * (j & 1) + g4);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[j][r] = ((w >> r) & 1u) ? v[j][r] : 0.f;
  }
}

template <int BM, int BN, int WM, int WN>
PZ_DEV void epilogue_lds(const GemmArgs& p, f32x4_t (&acc)[BM / WM / 16][BN / WN / 16], PZ_LDS char* smem, int m0,
                         int n0, int wm, int wn, int lane) {
  using C = Cfg<BM, BN, WM, WN>;
  constexpr int TM = C::TM, TN = C::TN;
  static_assert(BM * BN * 2 <= C::LDS_BYTES, "C tile must fit the ring's LDS");
  constexpr int CHUNKS_PER_ROW = BN / 8;
  constexpr int ROWS_PER_PASS = C::NT / CHUNKS_PER_ROW;
  constexpr int PASSES = BM / ROWS_PER_PASS;
  const int tid = threadIdx.x;
  const int my_row = tid / CHUNKS_PER_ROW, my_chunk = tid % CHUNKS_PER_ROW;
  const bool bwd = p.epi_mode == EPI_BWD;
  const EpiSpec& e = p.epi;
  const int g4 = 4 * (lane >> 4);
  const int ml0 = wm * C::WTM + (lane & 15);  // + i*16
  const int nl0 = wn * C::WTN + g4;           // + j*16
  // element index of fragment (i, j) = (m0+ml0+16i) * idx_ld + n0+nl0+16j; pairs = idx / 2
  const uint32_t pair0 =
      static_cast<uint32_t>((static_cast<uint64_t>(m0 + ml0) * static_cast<uint64_t>(p.idx_ld) + n0 + nl0) >> 1);
  const uint32_t row_pairs = static_cast<uint32_t>(p.idx_ld) * 8u;  // 16 rows down, in pairs
  static_assert(C::WTN == 64, "the ReLU bitmask epilogue assumes 64-column wave tiles");
  const bool use_mask = p.mask != nullptr;

  // ReLU bitmask (EPI_BWD): 8 bytes per accumulator row, issued before the barrier so the
  // loads fly while the slower waves finish their last MFMAs
  u32x2_t mbits[TM];
  if (bwd && use_mask) {
    const uint8_t* mrow = p.mask + (n0 + wn * C::WTN) / 8;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + ml0 + 16 * i;
      mbits[i] = m < p.M ? *reinterpret_cast<const u32x2_t*>(mrow + static_cast<int64_t>(m) * p.ldmask)
                         : u32x2_t{0u, 0u};
    }
  }

  __syncthreads();  // every wave is done reading the ring
  if (bwd && !use_mask) {
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
  f32x4_t bias4[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + nl0 + 16 * j;
    bias4[j] = (!bwd && p.bias != nullptr && n < p.N) ? *reinterpret_cast<const f32x4_t*>(p.bias + n)
                                                       : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  static_for<TM>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    f32x4_t (&v)[TN] = acc[i];
    const uint32_t pr0 = pair0 + static_cast<uint32_t>(i) * row_pairs;
    const int ml = ml0 + 16 * i;
#pragma unroll
    for (int j = 0; j < TN; ++j) v[j] = v[j] * p.alpha + bias4[j];
    if (!bwd) {
      if (p.epi_mode == EPI_FWD) {
        if (e.drop_pre) dropout_row(v, e, e.key_pre, pr0);
        if (e.act != ACT_NONE) act_fwd_row(v, e.act);
        if (e.drop_post) dropout_row(v, e, e.key_post, pr0);
      }
    } else {
      if (e.drop_post) dropout_row(v, e, e.key_post, pr0);
      if (use_mask) act_bwd_mask_row(v, mbits[i], g4);
      else if (e.act != ACT_NONE) act_bwd_row<BN>(v, smem, ml, nl0, e.act, e.drop_post ? e.inv_scale : 1.f);
      if (e.drop_pre) dropout_row(v, e, e.key_pre, pr0);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
      *reinterpret_cast<PZ_LDS u32x2_t*>(smem + cimg_off<BN>(ml, nl0 + 16 * j)) =
          u32x2_t{pack_bf2(v[j][0], v[j][1]), pack_bf2(v[j][2], v[j][3])};
    __builtin_amdgcn_sched_barrier(0);  // keep rows apart: bounds the live temporaries
  });
  if (p.colsum != nullptr) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4_t cs = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < TM; ++i)
        if (m0 + ml0 + 16 * i < p.M) cs += acc[i][j];
      const int n = n0 + nl0 + 16 * j;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = cs[r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        if ((lane & 15) == 0 && n + r < p.N) atomicAdd(p.colsum + n + r, s);
      }
    }
  }
  __syncthreads();
  uint16_t* __restrict__ Cp = static_cast<uint16_t*>(p.C);
#pragma unroll
  for (int s = 0; s < PASSES; ++s) {
    const int r = s * ROWS_PER_PASS + my_row;
    const int gm = m0 + r, gn = n0 + my_chunk * 8;
    const u32x4_t v = *reinterpret_cast<const PZ_LDS u32x4_t*>(smem + cimg_off<BN>(r, my_chunk * 8));
    if (gm < p.M && gn < p.N) {
      *reinterpret_cast<u32x4_t*>(Cp + static_cast<int64_t>(gm) * p.ldc + gn) = v;
      if (!bwd && use_mask) {  // bit b = element gn+b > 0 (bf16: sign clear, magnitude nonzero)
        uint32_t byte = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t lo = v[q] & 0xFFFFu, hi = v[q] >> 16;
          byte |= ((lo - 1u) < 0x7FFFu ? 1u : 0u) << (2 * q);
          byte |= ((hi - 1u) < 0x7FFFu ? 1u : 0u) << (2 * q + 1);
        }
        p.mask[static_cast<int64_t>(gm) * p.ldmask + gn / 8] = static_cast<uint8_t>(byte);
      }
    }
  }
}
