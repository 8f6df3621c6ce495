// N7 — training diagnostics on the GPU (reference neural_net_model.py:542-583).
//
// torch.histogram has no GPU kernel (aten::histogram.bin_ct is CPU-only), so the reference's
// stats would force a full device->host copy of every activation, gradient and weight gradient.
// Here one moments pass (min/max/sum/sum^2/saturation count, exact orderable-key atomics for
// min/max) and one 100-bin LDS histogram pass run on the device; only ~1 KB per tensor crosses
// to the host.
#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

template <typename T> PZ_DEV double lds_(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double lds_<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }

PZ_DEV unsigned long long order_key(double x) {
  const unsigned long long b = __double_as_longlong(x);
  return (b >> 63) ? ~b : (b | (1ULL << 63));
}
PZ_DEV double key_value(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & ~(1ULL << 63)) : ~k;
  return __longlong_as_double(b);
}

// out layout: [0] min key, [1] max key, [2] sum, [3] sumsq, [4] saturated count (elementwise rules)
template <typename T>
__global__ void __launch_bounds__(256) moments_kernel(const T* __restrict__ x, int64_t n, int rule, float thr,
                                                      double* out) {
  double mn = INFINITY, mx = -INFINITY, s = 0.0, ss = 0.0, sat = 0.0;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const double v = lds_<T>(x, i);
    mn = fmin(mn, v); mx = fmax(mx, v); s += v; ss += v * v;
    if (rule == SAT_ABS_GT) sat += fabs(v) > thr ? 1.0 : 0.0;
    else if (rule == SAT_LE) sat += v <= thr ? 1.0 : 0.0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mn = fmin(mn, __shfl_xor(mn, o, 64));
    mx = fmax(mx, __shfl_xor(mx, o, 64));
    s += __shfl_xor(s, o, 64);
    ss += __shfl_xor(ss, o, 64);
    sat += __shfl_xor(sat, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
    atomicMin(keys + 0, order_key(mn));
    atomicMax(keys + 1, order_key(mx));
    atomicAdd(out + 2, s);
    atomicAdd(out + 3, ss);
    if (rule == SAT_ABS_GT || rule == SAT_LE) atomicAdd(out + 4, sat);
  }
}

// row rules: one wave per row of length row_len
template <typename T>
__global__ void __launch_bounds__(256) row_rule_kernel(const T* __restrict__ x, int64_t rows, int64_t row_len, int rule,
                                                       float thr, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * int64_t(4) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * row_len;
  double acc = rule == SAT_ROW_MAX_GT ? -INFINITY : 0.0;
  for (int64_t c = lane; c < row_len; c += 64) {
    const double v = lds_<T>(xr, c);
    if (rule == SAT_ROW_MAX_GT) acc = fmax(acc, v); else acc += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double other = __shfl_xor(acc, o, 64);
    acc = rule == SAT_ROW_MAX_GT ? fmax(acc, other) : acc + other;
  }
  const double metric = rule == SAT_ROW_MAX_GT ? acc : sqrt(acc);
  if (lane == 0 && metric > thr) atomicAdd(out + 4, 1.0);
}

__global__ void init_moments_kernel(double* out) {
  if (threadIdx.x < 8) {
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
    if (threadIdx.x == 0) keys[0] = ~0ULL;
    else if (threadIdx.x == 1) keys[1] = 0ULL;
    else out[threadIdx.x] = 0.0;
  }
}

__global__ void decode_moments_kernel(double* out) {
  if (threadIdx.x == 0) {
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
    const double lo = key_value(keys[0]);
    const double hi = key_value(keys[1]);
    out[0] = lo;
    out[1] = hi;
  }
}

// Exact integer counts: u32 per block in LDS, u64 device totals (an fp32 count stops being exact
// past 2^24, which the ReLU-zero bin of one [8192, 8192] activation already exceeds)
template <typename T>
__global__ void __launch_bounds__(256) histogram_kernel(const T* __restrict__ x, int64_t n, const double* range, int bins,
                                                        unsigned long long* counts) {
  extern __shared__ unsigned int hist_lds[];
  for (int b = threadIdx.x; b < bins; b += 256) hist_lds[b] = 0u;
  __syncthreads();
  double lo = range[0], hi = range[1];
  if (lo == hi) { lo -= 0.5; hi += 0.5; }  // torch.histogram widens a degenerate range
  const double scale = bins / (hi - lo);
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const double v = lds_<T>(x, i);
    if (!(v >= lo && v <= hi)) continue;
    int b = static_cast<int>((v - lo) * scale);
    b = b >= bins ? bins - 1 : (b < 0 ? 0 : b);
    atomicAdd(&hist_lds[b], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < bins; b += 256)
    if (hist_lds[b]) atomicAdd(counts + b, static_cast<unsigned long long>(hist_lds[b]));
}

int grid_stride_blocks(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return static_cast<int>(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

}  // namespace

#define PZ_STATS_DISPATCH(dt, T, ...)                         \
  switch (dt) {                                               \
    case DT_BF16: { using T = uint16_t; __VA_ARGS__; break; } \
    case DT_F32: { using T = float; __VA_ARGS__; break; }     \
    case DT_F64: { using T = double; __VA_ARGS__; break; }    \
    default: return hipErrorInvalidValue;                     \
  }

hipError_t tensor_moments(const void* x, int dtype, int64_t n, int64_t row_len, int sat_rule, float sat_thr,
                          double* out, hipStream_t s) {
  hipLaunchKernelGGL(init_moments_kernel, dim3(1), dim3(64), 0, s, out);
  if (n > 0) {
    PZ_STATS_DISPATCH(dtype, T, {
      hipLaunchKernelGGL((moments_kernel<T>), dim3(grid_stride_blocks(n)), dim3(256), 0, s, static_cast<const T*>(x), n,
                         sat_rule, sat_thr, out);
      if ((sat_rule == SAT_ROW_NORM_GT || sat_rule == SAT_ROW_MAX_GT) && row_len > 0) {
        const int64_t rows = n / row_len;
        hipLaunchKernelGGL((row_rule_kernel<T>), dim3(static_cast<unsigned>((rows + 3) / 4)), dim3(256), 0, s,
                           static_cast<const T*>(x), rows, row_len, sat_rule, sat_thr, out);
      }
    });
  }
  hipLaunchKernelGGL(decode_moments_kernel, dim3(1), dim3(64), 0, s, out);
  return hipGetLastError();
}

hipError_t histogram(const void* x, int dtype, int64_t n, const double* range, int bins, int64_t* counts, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  PZ_STATS_DISPATCH(dtype, T, {
    hipLaunchKernelGGL((histogram_kernel<T>), dim3(grid_stride_blocks(n)), dim3(256), bins * sizeof(unsigned int), s,
                       static_cast<const T*>(x), n, range, bins, reinterpret_cast<unsigned long long*>(counts));
  });
  return hipGetLastError();
}

}  // namespace pz
