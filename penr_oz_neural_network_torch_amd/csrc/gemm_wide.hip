// N1c — fp64 / fp32 GEMM on the gfx950 matrix cores (the reference's default precision is fp64,
// neural_net_model.py:43-45, 104-108; its forward is `x @ W`, :117, and autograd's two `mm`s).
//
//  * fp64: v_mfma_f64_16x16x4_f64 (exact fp64 FMA chains), fp32: v_mfma_f32_16x16x4_f32
//    (exact f32, the same rate as the f32 VALU but one VGPR per operand and the VALU left free
//    for the epilogue — guide §3 'FP32-input MFMA'). No reduced-precision shortcut: results are
//    k-ordered fma chains of the input precision.
//  * 128x128 tile, 4 waves (2x2), 64x64 per wave = 4x4 MFMA tiles; K in 32-deep tiles, staged
//    by 16-B vector loads; the fragments of k-step g+1 are read while the MFMAs of k-step g run.
//  * Operands staged through LDS in their own orientation (padded images, see Img), 16-B loads
//    coalesced along the contiguous dimension and one ds_write_b128 per vector, with the next tile
//    prefetched into registers while the MFMAs run on the current one (one register set, the
//    write placed after the barrier: guide T14). At 64 (fp64) / 32 (fp32) cycles per MFMA the
//    loop is matrix-bound; staging and fragment reads hide under it.
//  * Any M / N / K (zero-filled edges, masked stores) and the generic kernel's epilogue contract
//    (alpha, bias, EPI_FWD / EPI_BWD stage math, accumulate, fp32 column sums).
#include "pz_common.h"
#include "pz_launch.h"

namespace pz {
namespace {

constexpr int WT = 128;  // output tile
constexpr int WK = 32;   // K depth per LDS tile (8 MFMA k-steps: 8192 matrix cycles per wave at fp64)

template <typename T> struct Wide;
template <> struct Wide<float> {
  using Acc = f32x4_t;
  static PZ_DEV Acc mma(float a, float b, Acc c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  static PZ_DEV int row(int lane, int r) { return 4 * (lane >> 4) + r; }  // C/D: col = lane & 15
};
template <> struct Wide<double> {
  using Acc = f64x4_t;
  static PZ_DEV Acc mma(double a, double b, Acc c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
  static PZ_DEV int row(int lane, int r) { return (lane >> 4) + 4 * r; }  // f64 map (guide §3)
};

template <typename T> PZ_DEV double wld(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double wld<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> PZ_DEV void wst(T* p, int64_t i, double v) { p[i] = static_cast<T>(v); }
template <> PZ_DEV void wst<uint16_t>(uint16_t* p, int64_t i, double v) { p[i] = f2bf(static_cast<float>(v)); }

// LDS image of one operand tile (WT rows x WK k), kept in the operand's own orientation so the
// 16-B staging vectors land as ONE ds_write_b128 each:
//  * K-contiguous operand: [row][k], pitch WK + 2 elements — a fragment read (lanes 0-15: 16
//    rows at k, lanes 16-31: the same rows at k + 1) hits 32 distinct banks;
//  * M/N-contiguous: [k][row], pitch WT + 16 — rows k and k + 1 on opposite bank halves.
template <typename T, bool KC>
struct Img {
  static constexpr int PITCH = KC ? WK + 2 : WT + 16;
  static constexpr int ELEMS = KC ? WT * PITCH : WK * PITCH;
  PZ_DEV static int at(int r, int k) { return KC ? r * PITCH + k : k * PITCH + r; }
};

// One operand tile per 256 threads as 16-B vectors of V elements along the contiguous dimension:
// vector e = tid + 256 * i covers V consecutive k (K-contiguous) or V consecutive rows.
template <typename T, bool KC>
struct Stage {
  static constexpr int V = 16 / sizeof(T);
  static constexpr int NV = WK * WT / V / 256;  // vectors per thread
  T v[NV][V];
  PZ_DEV static void coords(int e, int& k, int& r) {
    if (KC) { k = (e % (WK / V)) * V; r = e / (WK / V); }
    else { k = e / (WT / V); r = (e % (WT / V)) * V; }
  }
  PZ_DEV void load(const T* __restrict__ g, int64_t ld, int r0, int rows, int k0, int K, bool vec_ok, int tid) {
    // interior tile (the common case, decided once per tile): straight 16-B loads with no
    // per-vector branch — a per-load "vector or element" branch makes hipcc wait vmcnt(0) after
    // every load (guide §5 'Projection GEMM' trap (c)) and serialises the prefetch
    if (vec_ok && r0 + WT <= rows && k0 + WK <= K) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int k, r;
        coords(tid + 256 * i, k, r);
        const int64_t off = KC ? int64_t(r0 + r) * ld + (k0 + k) : int64_t(k0 + k) * ld + (r0 + r);
        const f32x4_t q = *reinterpret_cast<const f32x4_t*>(g + off);
        __builtin_memcpy(v[i], &q, 16);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int k, r;
      coords(tid + 256 * i, k, r);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int rr = r0 + r + (KC ? 0 : j), kk = k0 + k + (KC ? j : 0);
        v[i][j] = (rr < rows && kk < K) ? g[KC ? int64_t(rr) * ld + kk : int64_t(kk) * ld + rr] : T(0);
      }
    }
  }
  PZ_DEV void store(T* img, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int k, r;
      coords(tid + 256 * i, k, r);
      f32x4_t q;
      __builtin_memcpy(&q, v[i], 16);
      *reinterpret_cast<f32x4_t*>(img + Img<T, KC>::at(r, k)) = q;
    }
  }
};

template <typename T, bool A_KC, bool B_KC, typename OutT>
__global__ void __launch_bounds__(256) gemm_wide_kernel(const GemmArgs p) {
  using W = Wide<T>;
  using Acc = typename W::Acc;
  using IA = Img<T, A_KC>;
  using IB = Img<T, B_KC>;
  extern __shared__ __attribute__((aligned(16))) char wide_smem[];
  T* As = reinterpret_cast<T*>(wide_smem);
  T* Bs = As + IA::ELEMS;
  const T* __restrict__ A = static_cast<const T*>(p.A);
  const T* __restrict__ B = static_cast<const T*>(p.B);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware bijective remap (consecutive tiles share an XCD's L2), column-major tile order
  const int tiles_m = (p.M + WT - 1) / WT, tiles_n = (p.N + WT - 1) / WT, nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
  const int m0 = (wg % tiles_m) * WT, n0 = (wg / tiles_m) * WT;

  Acc acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = Acc{0, 0, 0, 0};

  Stage<T, A_KC> sa;
  Stage<T, B_KC> sb;
  auto aligned = [](const void* ptr, int64_t ld) {
    return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0 && (ld * static_cast<int64_t>(sizeof(T))) % 16 == 0;
  };
  const bool va = aligned(A, p.lda), vb = aligned(B, p.ldb);
  sa.load(A, p.lda, m0, p.M, 0, p.K, va, tid);
  sb.load(B, p.ldb, n0, p.N, 0, p.K, vb, tid);
  const int ml = wm * 64 + (lane & 15), nl = wn * 64 + (lane & 15), kl = lane >> 4;
  for (int k0 = 0; k0 < p.K; k0 += WK) {
    __syncthreads();  // every wave is done reading the previous tile
    sa.store(As, tid);
    sb.store(Bs, tid);
    __syncthreads();
    if (k0 + WK < p.K) {  // next tile into registers while this one is multiplied
      sa.load(A, p.lda, m0, p.M, k0 + WK, p.K, va, tid);
      sb.load(B, p.ldb, n0, p.N, k0 + WK, p.K, vb, tid);
    }
    // fragments of k-step g+1 are read while the 16 MFMAs of k-step g run
    T a[2][4], b[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[0][i] = As[IA::at(ml + 16 * i, kl)];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[0][j] = Bs[IB::at(nl + 16 * j, kl)];
#pragma unroll
    for (int g = 0; g < WK / 4; ++g) {
      const int cur = g & 1, nxt = cur ^ 1;
      if (g + 1 < WK / 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[nxt][i] = As[IA::at(ml + 16 * i, 4 * (g + 1) + kl)];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[nxt][j] = Bs[IB::at(nl + 16 * j, 4 * (g + 1) + kl)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = W::mma(a[cur][i], b[cur][j], acc[i][j]);
    }
  }

  // ---- epilogue (the generic kernel's contract, element by element)
  const EpiSpec epi = epi_resolve(p.epi);
  OutT* __restrict__ Cp = static_cast<OutT*>(p.C);
  auto aux_at = [&](int64_t i) -> T {
    if (p.aux_dtype == DT_F64) return static_cast<T>(static_cast<const double*>(p.aux)[i]);
    if (p.aux_dtype == DT_F32) return static_cast<T>(static_cast<const float*>(p.aux)[i]);
    return static_cast<T>(bf2f(static_cast<const uint16_t*>(p.aux)[i]));
  };
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + 16 * j + (lane & 15);
    double cs = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + 16 * i + W::row(lane, r);
        if (m >= p.M || n >= p.N) continue;
        T v = static_cast<T>(acc[i][j][r]) * static_cast<T>(p.alpha);
        const uint64_t idx = static_cast<uint64_t>(m) * static_cast<uint64_t>(p.idx_ld) + n;
        if (p.epi_mode == EPI_BWD) {
          v = epi_bwd<T>(v, aux_at(int64_t(m) * p.ldaux + n), idx, epi);
        } else {
          if (p.bias64 != nullptr) v += static_cast<T>(p.bias64[n]);
          else if (p.bias != nullptr) v += static_cast<T>(p.bias[n]);
          if (p.epi_mode == EPI_FWD) v = epi_fwd<T>(v, idx, epi);
        }
        const int64_t off = int64_t(m) * p.ldc + n;
        if (p.accumulate) v += static_cast<T>(wld<OutT>(Cp, off));
        wst<OutT>(Cp, off, static_cast<double>(v));
        cs += static_cast<double>(v);
      }
    if (p.colsum != nullptr || p.colsum64 != nullptr) {  // lanes l, l+16, l+32, l+48 share column n
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (lane < 16 && n < p.N) {
        if (p.colsum64 != nullptr) atomicAdd(p.colsum64 + n, cs);
        else atomicAdd(p.colsum + n, static_cast<float>(cs));
      }
    }
  }
}

template <typename T, bool A_KC, bool B_KC, typename OutT>
hipError_t launch_wide_k(const GemmArgs& p, hipStream_t s) {
  constexpr int lds = sizeof(T) * (Img<T, A_KC>::ELEMS + Img<T, B_KC>::ELEMS);
  auto kern = gemm_wide_kernel<T, A_KC, B_KC, OutT>;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nwg = ((p.M + WT - 1) / WT) * ((p.N + WT - 1) / WT);
  hipLaunchKernelGGL(kern, dim3(nwg), dim3(256), lds, s, p);
  return hipGetLastError();
}

template <typename T, typename OutT>
hipError_t launch_wide_out(const GemmArgs& p, hipStream_t s) {
  if (p.a_kc && p.b_kc) return launch_wide_k<T, true, true, OutT>(p, s);
  if (p.a_kc) return launch_wide_k<T, true, false, OutT>(p, s);
  if (p.b_kc) return launch_wide_k<T, false, true, OutT>(p, s);
  return launch_wide_k<T, false, false, OutT>(p, s);
}

template <typename T>
hipError_t launch_wide_in(const GemmArgs& p, hipStream_t s) {
  switch (p.out_dtype) {
    case DT_BF16: return launch_wide_out<T, uint16_t>(p, s);
    case DT_F32: return launch_wide_out<T, float>(p, s);
    case DT_F64: return launch_wide_out<T, double>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

// fp32 / fp64 operands on the matrix cores; tiny problems (one partial tile, e.g. the
// reference's 9x9 tic-tac-toe layers) stay on the generic VALU tile, which wastes fewer lanes
bool wide_eligible(const GemmArgs& p) {
  if (p.force_generic || (p.in_dtype != DT_F32 && p.in_dtype != DT_F64)) return false;
  if (p.mask != nullptr || p.out8 != nullptr || p.split_k > 1 || p.epi_mode == EPI_OPT) return false;
  return static_cast<int64_t>(p.M) * p.N >= 64 * 64 && p.K >= 16;
}

hipError_t gemm_wide(const GemmArgs& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.in_dtype == DT_F64) return launch_wide_in<double>(p, s);
  return launch_wide_in<float>(p, s);
}

}  // namespace pz
