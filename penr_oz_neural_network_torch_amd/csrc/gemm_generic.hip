// N1b — shape-agnostic GEMM for gfx950: any M/N/K, any operand layout, bf16 / fp32 / fp64.
//
// Covers everything the matrix-core paths do not: tiny layers (the reference's [4,8,2]-style
// models, vocab 27 embeddings) and ragged bf16 shapes; fp32 / fp64 GEMMs of any real size run on
// the f32 / f64 MFMA kernel (gemm_wide.hip). Same fused epilogue contract as the MFMA kernels.
//
// 64x64 output tile, BK = 16, 256 threads (4 waves), 4x4 outputs per thread, operands staged
// through padded LDS ([k][m+1]) so both K-major and M-major global reads coalesce.
#include "pz_common.h"
#include "pz_launch.h"

namespace pz {
namespace {

template <typename T> PZ_DEV double load_elem(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double load_elem<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }

template <typename T, typename Acc> PZ_DEV Acc ld(const T* p, int64_t i) { return static_cast<Acc>(load_elem<T>(p, i)); }

template <typename T> PZ_DEV void store_elem(T* p, int64_t i, double v) { p[i] = static_cast<T>(v); }
template <> PZ_DEV void store_elem<uint16_t>(uint16_t* p, int64_t i, double v) { p[i] = f2bf(static_cast<float>(v)); }

constexpr int GT = 64;
constexpr int GK = 16;

template <typename T, typename Acc, typename OutT, typename AuxT>
__global__ void __launch_bounds__(256) gemm_generic_kernel(const GemmArgs p) {
  const EpiSpec epi = epi_resolve(p.epi);
  __shared__ Acc As[GK][GT + 1];
  __shared__ Acc Bs[GK][GT + 1];
  const T* __restrict__ A = static_cast<const T*>(p.A);
  const T* __restrict__ B = static_cast<const T*>(p.B);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * GT, n0 = blockIdx.x * GT;

  Acc acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = Acc(0);

  for (int k0 = 0; k0 < p.K; k0 += GK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int lin = threadIdx.x + e * 256;
      int mm, kk;
      if (p.a_kc) { kk = lin & (GK - 1); mm = lin / GK; } else { mm = lin & (GT - 1); kk = lin / GT; }
      const int gm = m0 + mm, gk = k0 + kk;
      Acc v = Acc(0);
      if (gm < p.M && gk < p.K) v = ld<T, Acc>(A, p.a_kc ? int64_t(gm) * p.lda + gk : int64_t(gk) * p.lda + gm);
      As[kk][mm] = v;
      int nn;
      if (p.b_kc) { kk = lin & (GK - 1); nn = lin / GK; } else { nn = lin & (GT - 1); kk = lin / GT; }
      const int gn = n0 + nn, gk2 = k0 + kk;
      Acc w = Acc(0);
      if (gn < p.N && gk2 < p.K) w = ld<T, Acc>(B, p.b_kc ? int64_t(gn) * p.ldb + gk2 : int64_t(gk2) * p.ldb + gn);
      Bs[kk][nn] = w;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; ++kk) {
      Acc a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a[i] * b[j];
    }
    __syncthreads();
  }

  OutT* __restrict__ Cp = static_cast<OutT*>(p.C);
  const AuxT* __restrict__ aux = static_cast<const AuxT*>(p.aux);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + tx + 16 * j;
    Acc colsum = Acc(0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + ty + 16 * i;
      if (m >= p.M || n >= p.N) continue;
      Acc v = acc[i][j] * static_cast<Acc>(p.alpha);
      const uint64_t idx = static_cast<uint64_t>(m) * static_cast<uint64_t>(p.idx_ld) + n;
      if (p.epi_mode == EPI_BWD) {
        const Acc y = ld<AuxT, Acc>(aux, int64_t(m) * p.ldaux + n);
        v = epi_bwd<Acc>(v, y, idx, epi);
      } else {
        if (p.bias64 != nullptr) v += static_cast<Acc>(p.bias64[n]);
        else if (p.bias != nullptr) v += static_cast<Acc>(p.bias[n]);
        if (p.epi_mode == EPI_FWD) v = epi_fwd<Acc>(v, idx, epi);
      }
      const int64_t off = int64_t(m) * p.ldc + n;
      if (p.accumulate) v += ld<OutT, Acc>(Cp, off);
      store_elem<OutT>(Cp, off, static_cast<double>(v));
      colsum += v;
    }
    if (p.colsum64 != nullptr && n < p.N) atomicAdd(p.colsum64 + n, static_cast<double>(colsum));
    else if (p.colsum != nullptr && n < p.N) atomicAdd(p.colsum + n, static_cast<float>(colsum));
  }
}

template <typename T, typename Acc, typename OutT>
hipError_t launch_generic_out(const GemmArgs& p, hipStream_t s) {
  dim3 grid((p.N + GT - 1) / GT, (p.M + GT - 1) / GT);
  if (p.aux_dtype == DT_F64)
    hipLaunchKernelGGL((gemm_generic_kernel<T, Acc, OutT, double>), grid, dim3(256), 0, s, p);
  else if (p.aux_dtype == DT_F32)
    hipLaunchKernelGGL((gemm_generic_kernel<T, Acc, OutT, float>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((gemm_generic_kernel<T, Acc, OutT, uint16_t>), grid, dim3(256), 0, s, p);
  return hipGetLastError();
}

template <typename T, typename Acc>
hipError_t launch_generic_in(const GemmArgs& p, hipStream_t s) {
  switch (p.out_dtype) {
    case DT_BF16: return launch_generic_out<T, Acc, uint16_t>(p, s);
    case DT_F32: return launch_generic_out<T, Acc, float>(p, s);
    case DT_F64: return launch_generic_out<T, Acc, double>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

bool mfma_eligible(const GemmArgs& p);
hipError_t gemm_mfma(const GemmArgs& p, hipStream_t s);
bool wide_eligible(const GemmArgs& p);
hipError_t gemm_wide(const GemmArgs& p, hipStream_t s);

hipError_t gemm_generic(const GemmArgs& p, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  switch (p.in_dtype) {
    case DT_BF16: return launch_generic_in<uint16_t, float>(p, s);
    case DT_F32: return launch_generic_in<float, float>(p, s);
    case DT_F64: return launch_generic_in<double, double>(p, s);
    default: return hipErrorInvalidValue;
  }
}

int gemm_path(const GemmArgs& p) { return mfma_eligible(p) ? 1 : (wide_eligible(p) ? 2 : 0); }

hipError_t gemm(const GemmArgs& p, hipStream_t s) {
  if (mfma_eligible(p)) return gemm_mfma(p, s);
  if (p.epi_mode == EPI_OPT) return hipErrorInvalidValue;  // the fused update: bf16 MFMA path only
  if (wide_eligible(p)) return gemm_wide(p, s);
  // bitmask / e4m3 epilogues and e4m3 operands exist on the MFMA path only
  if (p.mask != nullptr || p.out8 != nullptr || p.in_dtype == DT_FP8) return hipErrorInvalidValue;
  return gemm_generic(p, s);
}

}  // namespace pz
