// Device helpers shared by the bf16/fp8 MFMA GEMMs (gemm_mfma.hip, gemm_sk.hip): LDS-DMA staging
// primitives, LDS swizzles, MFMA fragment reads, counted waits, the XCD-aware tile order.
// Included INSIDE `namespace pz { namespace {` by each kernel translation unit (like
// gemm_epilogue.h): every TU keeps its own internal copies.
#pragma once

// K-contiguous slot [rows][BK]. BK 32: 64-B rows = 4 chunks; chunk XOR for conflict-free
// ds_read_b128 under the gfx950 b128 lane grouping (row groups of 4 rows map to permutation
// {0,2,3,1}). BK 64: 128-B rows = 8 chunks, chunk ^= (row >> 1) & 7: every b128 lane group (16
// rows x one chunk column, two rows per 256-B bank row) hits 16 distinct 16-B bank slots, and an
// LDS-DMA instruction's 8 lanes per row still fetch one whole 128-B line.
template <int BK = 32>
PZ_DEV int swz_kc(int row) {
  if constexpr (BK == 64) return (row >> 1) & 7;
  else return (120 >> (2 * ((row >> 2) & 3))) & 3;
}
// M/N-contiguous slot [32][R]: chunk XOR so a half-wave's transposed reads hit 16 distinct slots
PZ_DEV int swz_mn(int krow) { return ((krow & 3) | (((krow >> 3) & 1) << 2)) << 1; }

// LDS-DMA of 16 B per lane into wave-uniform LDS byte address `lds` (+ lane*16).
// Inline asm ON PURPOSE: with the builtin, hipcc tracks the DMA as a pending LDS write and puts
// an `s_waitcnt vmcnt(0)` in front of the next ds_read — draining the whole ring every step.
// Hidden in asm, the DMA is counted only by our own `s_waitcnt vmcnt(N)` (guide §5.7 item 1).
PZ_DEV void glds16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

// Same DMA through the buffer (MUBUF) path: `rs` = raw buffer resource of the operand, `voff`
// = per-lane byte offset (loop-invariant: row / column position), `soff` = wave-uniform byte
// offset of the K step (an SGPR: no per-step vector address math). The operand must span
// < 4 GiB from its base (checked by the dispatcher).
typedef int i32x4_t __attribute__((ext_vector_type(4)));
// POL: cache policy of the request (0 default, 1 nt, 2 sc1, 3 sc0 sc1) — experiments
template <int POL = 0>
PZ_DEV void blds16(i32x4_t rs, uint32_t voff, uint32_t soff, uint32_t lds) {
  uint32_t keep;
#define PZ_BLDS(POLICY)                                          \
  asm volatile(                                                 \
      "s_mov_b32 %0, m0\n\t"                                    \
      "s_mov_b32 m0, %3\n\t"                                    \
      "s_nop 0\n\t"                                             \
      "buffer_load_dwordx4 %1, %2, %4 offen" POLICY " lds\n\t"  \
      "s_mov_b32 m0, %0"                                        \
      : "=&s"(keep)                                             \
      : "v"(voff), "s"(rs), "s"(lds), "s"(soff)                 \
      : "memory")
  if constexpr (POL == 1) PZ_BLDS(" nt");
  else if constexpr (POL == 2) PZ_BLDS(" sc1");
  else if constexpr (POL == 3) PZ_BLDS(" sc0 sc1");
  else PZ_BLDS("");
#undef PZ_BLDS
}

// 4-byte LDS-DMA used as an L2 PREFETCH: touching one dword of a 128-B line brings the line into
// the XCD's L2 several ring steps before the real staging DMA asks for it; the bytes land in a
// 256-B dummy LDS area nobody reads (no VGPR is written, so nothing can be clobbered)
PZ_DEV void glds4(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

PZ_DEV i32x4_t buf_rsrc(const void* base) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r[0] = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b)));
  r[1] = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(b >> 32)));
  r[2] = -1;           // num_records: whole 4 GiB window
  r[3] = 0x00020000;   // gfx9 raw buffer
  return r;
}

PZ_DEV uint32_t lds_addr(const PZ_LDS char* p) {
  return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p)));
}

// M/N-contiguous fp8 operand ([K][rows] bytes in memory; the weight-gradient GEMM's activations
// and output gradients): k rows [k0, k0+KROWS) x bytes [col0, col0+RB) -> slot [KROWS][RB]. The
// 16-B chunk of k-row kr is XOR-ed with (kr & 7) << 1, so the transposing 8-bit reads below
// (8 k-rows x 16 bytes per 16-lane group, two groups per 32-lane bank half) are conflict-free.
// 128-B rows (256x128 tiles' B, VAR 16): two k-rows share a 256-B bank row, so the XOR takes
// k-row bits 1-2 and the row parity selects the half — the same 16 distinct 16-B slots per
// 8 k-rows x 2 chunks of a 32-lane read
template <int RB>
PZ_DEV int swz_mn8(int krow) {
  if constexpr (RB >= 256) return (krow & 7) << 1;
  else return ((krow >> 1) & 3) << 1;
}

typedef int i32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x8_t __attribute__((ext_vector_type(8)));
// 32x32x64 f8 MFMA operand from an [64 k][RB] fp8 slot: lane l holds column col32 + (l & 31),
// k bytes [32 (l >> 5), +32) — four ds_read_b64_tr_b8 (per 16-lane group: 8 k-rows x 16 columns,
// lane 2q+p addresses k-row q, bytes 8p..8p+7 of the group's 16; lane i receives column i)
template <int RB>
PZ_DEV i32x8_t frag_mn8(const PZ_LDS char* tile, int col32, int lane) {
  const int q = (lane & 15) >> 1;
  const int col = col32 + 16 * ((lane >> 4) & 1) + 8 * (lane & 1);
  const int chunk = col >> 4, within = col & 15;
  i32x8_t out;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 32 * (lane >> 5) + 8 * i + q;
    const PZ_LDS char* a = tile + k * RB + ((chunk ^ swz_mn8<RB>(k)) << 4) + within;
    const i32x2_t r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((PZ_LDS i32x2_t*)(a));
    out[2 * i] = r[0];
    out[2 * i + 1] = r[1];
  }
  return out;
}

template <int BK = 32>
PZ_DEV i16x8_t frag_kc(const PZ_LDS char* tile, int row, int chunk) {
  const int slot = chunk ^ swz_kc<BK>(row);
  return *reinterpret_cast<const PZ_LDS i16x8_t*>(tile + row * (BK * 2) + slot * 16);
}

PZ_DEV i32x8_t cat_frag(i16x8_t lo, i16x8_t hi) {
  const i32x4_t a = __builtin_bit_cast(i32x4_t, lo), b = __builtin_bit_cast(i32x4_t, hi);
  return i32x8_t{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

template <int R>
PZ_DEV i16x8_t frag_mn(const PZ_LDS char* tile, int col16, int kbase, int lane) {
  const int q = (lane >> 2) & 3;
  const int p = lane & 3;
  const int col = col16 + 4 * p;
  const int chunk = col >> 3;
  const int within = (col & 7) * 2;
  const int k0 = kbase + q;
  const int k1 = k0 + 4;
  const PZ_LDS char* a0 = tile + k0 * (R * 2) + ((chunk ^ swz_mn(k0)) << 4) + within;
  const PZ_LDS char* a1 = tile + k1 * (R * 2) + ((chunk ^ swz_mn(k1)) << 4) + within;
  i16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((PZ_LDS i16x4_t*)(a0));
  i16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((PZ_LDS i16x4_t*)(a1));
  return i16x8_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// K-contiguous operand rows [row0, row0+R) x k [k0, k0+BK) -> slot [R][BK]; NW waves share it
// FULL (buffer path, dispatcher-guaranteed full row tiles): no row clamp, so the piece's row
// offset is wave-uniform and rides in soffset — one (BK 32) or two (BK 64: the swizzle flips
// with the piece's parity) per-lane offsets stay live instead of one per piece (the 16 of a
// BK 64 K-contiguous pair of operands spilled to scratch inside the loop)
template <int R, int NW, int BK = 32, bool BUF = false, int POL = 0, bool FULL = false>
PZ_DEV void stage_kc(const uint16_t* __restrict__ g, int64_t ld, int row0, int rows_valid, int k0,
                     PZ_LDS char* tile, int wave, int lane, i32x4_t rs = {}) {
  constexpr int CPR = BK / 8;             // 16-B chunks per row
  constexpr int RPI = 64 / CPR;           // rows per 1-KiB instruction
  constexpr int INSTR = R / (RPI * NW);
  static_assert(INSTR >= 1 && INSTR * RPI * NW == R, "K-contiguous stage split");
#pragma unroll
  for (int i = 0; i < INSTR; ++i) {
    const int rbase = (wave * INSTR + i) * RPI;
    const int r = rbase + lane / CPR;
    const int chunk = (lane % CPR) ^ swz_kc<BK>(r);
    if constexpr (BUF && FULL) {
      const uint32_t voff = (static_cast<uint32_t>(lane / CPR) * static_cast<uint32_t>(ld) + chunk * 8) * 2u;
      const uint32_t soff = (static_cast<uint32_t>(row0 + rbase) * static_cast<uint32_t>(ld) + static_cast<uint32_t>(k0)) * 2u;
      blds16<POL>(rs, voff, __builtin_amdgcn_readfirstlane(soff), lds_addr(tile + rbase * BK * 2));
      continue;
    }
    int gr = row0 + r;
    gr = gr < rows_valid ? gr : rows_valid - 1;
    if constexpr (BUF) {
      const uint32_t voff = (static_cast<uint32_t>(gr) * static_cast<uint32_t>(ld) + chunk * 8) * 2u;
      blds16<POL>(rs, voff, __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(k0) * 2u), lds_addr(tile + rbase * BK * 2));
    } else {
      const uint16_t* src = g + static_cast<int64_t>(gr) * ld + k0 + chunk * 8;
      glds16(src, lds_addr(tile + rbase * BK * 2));
    }
  }
}

// M/N-contiguous operand: k rows [k0, k0+BK) x cols [col0, col0+R) -> slot [BK][R]
template <int R, int NW, int BK = 32, bool BUF = false, int POL = 0>
PZ_DEV void stage_mn(const uint16_t* __restrict__ g, int64_t ld, int col0, int cols_valid, int k0,
                     PZ_LDS char* tile, int wave, int lane, i32x4_t rs = {}) {
  constexpr int ROW_BYTES = R * 2;
  constexpr int CHUNKS = R / 8;
  constexpr int ROWS_PER = 1024 / ROW_BYTES;
  constexpr int INSTR = (BK * ROW_BYTES) / (1024 * NW);
  static_assert(INSTR >= 1 && INSTR * 1024 * NW == BK * ROW_BYTES, "M/N-contiguous stage split");
#pragma unroll
  for (int i = 0; i < INSTR; ++i) {
    const int kbase = (wave * INSTR + i) * ROWS_PER;
    const int kr = kbase + lane / CHUNKS;
    const int chunk = (lane % CHUNKS) ^ swz_mn(kr);
    int gc = col0 + chunk * 8;
    gc = gc < cols_valid ? gc : cols_valid - 8;
    if constexpr (BUF) {
      const uint32_t voff = (static_cast<uint32_t>(kr) * static_cast<uint32_t>(ld) + gc) * 2u;
      blds16<POL>(rs, voff, __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(k0) * static_cast<uint32_t>(ld) * 2u),
             lds_addr(tile + kbase * ROW_BYTES));
    } else {
      const uint16_t* src = g + static_cast<int64_t>(k0 + kr) * ld + gc;
      glds16(src, lds_addr(tile + kbase * ROW_BYTES));
    }
  }
}

template <int N>
PZ_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// as wait_newer, with ONE extra (prefetch) operation issued after each step's G stage DMAs
template <int G, int MAXN>
PZ_DEV void wait_newer_pf(int n) {
  if constexpr (MAXN == 0) {
    wait_vm<1>();
  } else {
    if (n >= MAXN) wait_vm<MAXN * G + 1>();
    else wait_newer_pf<G, MAXN - 1>(n);
  }
}

// wait until at most n (<= MAXN) younger ring steps of G LDS-DMA instructions each are in flight
template <int G, int MAXN>
PZ_DEV void wait_newer(int n) {
  if constexpr (MAXN == 0) {
    wait_vm<0>();
  } else {
    if (n >= MAXN) wait_vm<MAXN * G>();
    else wait_newer<G, MAXN - 1>(n);
  }
}


template <typename OutT>
PZ_DEV void load4(const OutT* p, float v[4]);
template <>
PZ_DEV void load4<uint16_t>(const uint16_t* p, float v[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = bf2f(u.x & 0xFFFF); v[1] = bf2f(u.x >> 16); v[2] = bf2f(u.y & 0xFFFF); v[3] = bf2f(u.y >> 16);
}
template <>
PZ_DEV void load4<float>(const float* p, float v[4]) {
  const float4 u = *reinterpret_cast<const float4*>(p);
  v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
}
template <typename OutT>
PZ_DEV void store4(OutT* p, const float v[4]);
template <>
PZ_DEV void store4<uint16_t>(uint16_t* p, const float v[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
}
template <>
PZ_DEV void store4<float>(float* p, const float v[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

template <int N, typename F, int I = 0>
PZ_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

// XCD-aware bijective remap of the launch order: consecutive ids share an XCD's L2 (blocks are
// dealt round-robin over the 8 XCDs; speed only, never correctness)
PZ_DEV int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// remapped id -> tile = id / split, slice = id % split (a tile's K slices stay on one XCD), then
// grouped tile order for L2 reuse.
PZ_DEV void tile_coords(int wgid, int tiles_m, int tiles_n, int split, int& tm, int& tn, int& tile, int& slice) {
  tile = wgid / split;
  slice = wgid - tile * split;
  wgid = tile;
  constexpr int GROUP = 8;
  const int per_group = GROUP * tiles_n;
  const int g = wgid / per_group;
  const int first = g * GROUP;
  const int gsz = min(tiles_m - first, GROUP);
  const int in_group = wgid - g * per_group;
  tm = first + in_group % gsz;
  tn = in_group / gsz;
}

// tools/gemm_stamps.hip (diagnostic build only): per-workgroup s_memrealtime stamps at the phase
// boundaries (entry, first K step landed, main loop done, epilogue start, end) + XCC id into the
// lab's debug buffer p.dbg — where a tile's time goes (guide §7, in-kernel stamps)
#ifdef PZ_GEMM_STAMPS
#define PZ_STAMP(i)                                                                                        \
  do {                                                                                                     \
    if (threadIdx.x == 0) {                                                                                \
      uint64_t* st_ = p.dbg + 8 * static_cast<int64_t>(blockIdx.x);                                       \
      st_[i] = __builtin_amdgcn_s_memrealtime();                                                           \
      if ((i) == 0) st_[7] = static_cast<uint64_t>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11))); \
    }                                                                                                      \
  } while (0)
#else
#define PZ_STAMP(i) do {} while (0)
#endif
