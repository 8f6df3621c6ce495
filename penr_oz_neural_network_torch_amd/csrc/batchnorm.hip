// N4 — batch normalisation over all leading dims (reference neural_net_model.py:158-170),
// with the following stage epilogue (dropout / activation / dropout) fused into the normalise
// pass and its derivative fused into the backward reductions.
//
// Semantics kept from the reference: batch statistics in training mode with the UNBIASED
// variance, EMA update of the running estimates `(1-m)·old + m·new`, eval mode on the running
// estimates, y = gain·(x-mean)/sqrt(var+eps) + bias. Padded rows (rows >= rows_valid) are
// excluded from the statistics and get zero gradient.
//
// Column reductions: a 2-D grid of (64-column strip, row chunk) blocks accumulates fp64 partial
// sums (coalesced 64-wide reads per wave), then a per-column finalize, then an elementwise pass.
#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

template <typename T> PZ_DEV double lb(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double lb<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> PZ_DEV void sb(T* p, int64_t i, double v) { p[i] = static_cast<T>(v); }
template <> PZ_DEV void sb<uint16_t>(uint16_t* p, int64_t i, double v) { p[i] = f2bf(static_cast<float>(v)); }

constexpr int kRowsPerChunk = 256;

template <typename T>
__global__ void __launch_bounds__(256) bn_col_sums_kernel(const T* __restrict__ x, int rows_valid, int cols,
                                                          double* partial) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * kRowsPerChunk;
  const int r1 = min(rows_valid, r0 + kRowsPerChunk);
  double s = 0.0, ss = 0.0;
  if (c < cols)
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) {
      const double v = lb<T>(x, static_cast<int64_t>(r) * cols + c);
      s += v; ss += v * v;
    }
  __shared__ double red[2][4][64];
  red[0][threadIdx.x >> 6][threadIdx.x & 63] = s;
  red[1][threadIdx.x >> 6][threadIdx.x & 63] = ss;
  __syncthreads();
  if (threadIdx.x < 64 && c < cols) {
    const int l = threadIdx.x;
    atomicAdd(partial + c, red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l]);
    atomicAdd(partial + cols + c, red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l]);
  }
}

template <typename P>
__global__ void bn_finalize_kernel(const double* partial, int n, int cols, P* running_mean, P* running_var, double eps,
                                   double momentum, int training, double* save_mean, double* save_invstd) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  double mean, var;
  if (training) {
    mean = partial[c] / n;
    var = n > 1 ? (partial[cols + c] - n * mean * mean) / (n - 1) : NAN;
    if (var < 0) var = 0;
    running_mean[c] = static_cast<P>((1.0 - momentum) * static_cast<double>(running_mean[c]) + momentum * mean);
    running_var[c] = static_cast<P>((1.0 - momentum) * static_cast<double>(running_var[c]) + momentum * var);
  } else {
    mean = static_cast<double>(running_mean[c]);
    var = static_cast<double>(running_var[c]);
  }
  save_mean[c] = mean;
  save_invstd[c] = 1.0 / sqrt(var + static_cast<double>(eps));
}

template <typename T, typename P>
__global__ void __launch_bounds__(256) bn_normalize_kernel(BnArgs a) {
  a.epi = epi_resolve(a.epi);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  T* __restrict__ y = static_cast<T*>(a.y);
  const P* gain = static_cast<const P*>(a.gain);
  const P* bias = static_cast<const P*>(a.bias);
  const int64_t n = static_cast<int64_t>(a.rows) * a.cols;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const int64_t r = i / a.cols;
    const int c = static_cast<int>(i - r * a.cols);
    double v = 0.0;
    if (r < a.rows_valid) {
      const double xh = (lb<T>(x, i) - a.save_mean[c]) * a.save_invstd[c];
      v = static_cast<double>(gain[c]) * xh + static_cast<double>(bias[c]);
      v = epi_fwd<double>(v, static_cast<uint64_t>(r * a.idx_ld + c), a.epi);
    }
    sb<T>(y, i, v);
  }
}

// backward reductions: sum(dyn), sum(dyn * xhat) with dyn = epi_bwd(g, y)
template <typename T>
__global__ void __launch_bounds__(256) bn_bwd_sums_kernel(BnBwdArgs a) {
  a.epi = epi_resolve(a.epi);
  const T* __restrict__ g = static_cast<const T*>(a.g);
  const T* __restrict__ y = static_cast<const T*>(a.y);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * kRowsPerChunk;
  const int r1 = min(a.rows_valid, r0 + kRowsPerChunk);
  double s = 0.0, sx = 0.0;
  if (c < a.cols) {
    const double mean = a.save_mean[c], inv = a.save_invstd[c];
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) {
      const int64_t i = static_cast<int64_t>(r) * a.cols + c;
      const double dyn = epi_bwd<double>(lb<T>(g, i), lb<T>(y, i), static_cast<uint64_t>(r * a.idx_ld + c), a.epi);
      s += dyn;
      sx += dyn * (lb<T>(x, i) - mean) * inv;
    }
  }
  __shared__ double red[2][4][64];
  red[0][threadIdx.x >> 6][threadIdx.x & 63] = s;
  red[1][threadIdx.x >> 6][threadIdx.x & 63] = sx;
  __syncthreads();
  if (threadIdx.x < 64 && c < a.cols) {
    const int l = threadIdx.x;
    atomicAdd(a.partial + c, red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l]);
    atomicAdd(a.partial + a.cols + c, red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l]);
  }
}

template <typename P>
__global__ void bn_param_grads_kernel(const double* partial, int cols, P* dgain, P* dbias) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  if (dbias != nullptr) dbias[c] = static_cast<P>(static_cast<double>(dbias[c]) + partial[c]);
  if (dgain != nullptr) dgain[c] = static_cast<P>(static_cast<double>(dgain[c]) + partial[cols + c]);
}

template <typename T, typename P>
__global__ void __launch_bounds__(256) bn_dx_kernel(BnBwdArgs a) {
  a.epi = epi_resolve(a.epi);
  const T* __restrict__ g = static_cast<const T*>(a.g);
  const T* __restrict__ y = static_cast<const T*>(a.y);
  const T* __restrict__ x = static_cast<const T*>(a.x);
  T* __restrict__ dx = static_cast<T*>(a.dx);
  const P* gain = static_cast<const P*>(a.gain);
  const int64_t n = static_cast<int64_t>(a.rows) * a.cols;
  const double B = a.n_total > 0 ? static_cast<double>(a.n_total) : static_cast<double>(a.rows_valid);
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const int64_t r = i / a.cols;
    const int c = static_cast<int>(i - r * a.cols);
    double v = 0.0;
    if (r < a.rows_valid) {
      const double inv = a.save_invstd[c];
      const double xh = (lb<T>(x, i) - a.save_mean[c]) * inv;
      const double dyn = epi_bwd<double>(lb<T>(g, i), lb<T>(y, i), static_cast<uint64_t>(r * a.idx_ld + c), a.epi);
      const double sdy = a.partial[c], sdyx = a.partial[a.cols + c];
      v = static_cast<double>(gain[c]) * inv / B * (B * dyn - sdy - B / (B - 1.0) * xh * sdyx);
    }
    sb<T>(dx, i, v);
  }
}

int blocks_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<int>(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

}  // namespace

#define PZ_BN_DISPATCH(dt, pdt, T, P, ...)                                                   \
  do {                                                                                       \
    if (pdt == DT_F64) {                                                                     \
      using P = double;                                                                      \
      switch (dt) {                                                                          \
        case DT_BF16: { using T = uint16_t; __VA_ARGS__; break; }                            \
        case DT_F32: { using T = float; __VA_ARGS__; break; }                                \
        case DT_F64: { using T = double; __VA_ARGS__; break; }                               \
        default: return hipErrorInvalidValue;                                                \
      }                                                                                      \
    } else {                                                                                 \
      using P = float;                                                                       \
      switch (dt) {                                                                          \
        case DT_BF16: { using T = uint16_t; __VA_ARGS__; break; }                            \
        case DT_F32: { using T = float; __VA_ARGS__; break; }                                \
        case DT_F64: { using T = double; __VA_ARGS__; break; }                               \
        default: return hipErrorInvalidValue;                                                \
      }                                                                                      \
    }                                                                                        \
  } while (0)

hipError_t batchnorm_fwd(const BnArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
  const int n = a.n_total > 0 ? static_cast<int>(a.n_total) : a.rows_valid;
  PZ_BN_DISPATCH(a.dtype, a.param_dtype, T, P, {
    if (a.training && a.phase != 2) {
      hipMemsetAsync(a.partial, 0, sizeof(double) * 2 * a.cols, s);
      dim3 grid((a.cols + 63) / 64, (a.rows_valid + kRowsPerChunk - 1) / kRowsPerChunk);
      hipLaunchKernelGGL((bn_col_sums_kernel<T>), grid, dim3(256), 0, s, static_cast<const T*>(a.x), a.rows_valid,
                         a.cols, a.partial);
    }
    if (a.phase != 1) {
      hipLaunchKernelGGL((bn_finalize_kernel<P>), dim3((a.cols + 255) / 256), dim3(256), 0, s, a.partial, n, a.cols,
                         static_cast<P*>(a.running_mean), static_cast<P*>(a.running_var), a.eps, a.momentum,
                         a.training, a.save_mean, a.save_invstd);
      hipLaunchKernelGGL((bn_normalize_kernel<T, P>), dim3(blocks_for(int64_t(a.rows) * a.cols)), dim3(256), 0, s, a);
    }
  });
  return hipGetLastError();
}

hipError_t batchnorm_bwd(const BnBwdArgs& a, hipStream_t s) {
  if (a.rows <= 0 || a.cols <= 0) return hipSuccess;
  PZ_BN_DISPATCH(a.dtype, a.param_dtype, T, P, {
    if (a.phase != 2) {
      hipMemsetAsync(a.partial, 0, sizeof(double) * 2 * a.cols, s);
      dim3 grid((a.cols + 63) / 64, (a.rows_valid + kRowsPerChunk - 1) / kRowsPerChunk);
      hipLaunchKernelGGL((bn_bwd_sums_kernel<T>), grid, dim3(256), 0, s, a);
      hipLaunchKernelGGL((bn_param_grads_kernel<P>), dim3((a.cols + 255) / 256), dim3(256), 0, s, a.partial, a.cols,
                         static_cast<P*>(a.dgain), static_cast<P*>(a.dbias));
    }
    if (a.dx != nullptr && a.phase != 1)
      hipLaunchKernelGGL((bn_dx_kernel<T, P>), dim3(blocks_for(int64_t(a.rows) * a.cols)), dim3(256), 0, s, a);
  });
  return hipGetLastError();
}

}  // namespace pz
