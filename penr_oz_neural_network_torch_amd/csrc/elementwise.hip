// N2 / N3 — standalone stage epilogues, loss heads, row softmax, column sums, minibatch gather.
//
//  * stage_fwd / stage_bwd: y = drop_post(act(drop_pre(x))) and its derivative for tensors that
//    are not produced by a GEMM (batchnorm outputs, the autograd path's standalone relu/sigmoid/
//    tanh/dropout layers: reference neural_net_model.py:172-184, 393-395). Vectorised 4 per lane.
//  * xent_head: softmax + log-softmax + NLL (mean) AND the backward (p - onehot)/B pushed through
//    the logits' dropout, with the bias-gradient column sum fused (reference :400-403 and
//    autograd's nll_loss_backward / _log_softmax_backward_data). One wave per row.
//  * mse_head: mean squared error and its gradient through the last stage's epilogue (:404-406).
//  * softmax_rows: the final layer's probabilities (:186-188).
//  * gather_rows: on-device minibatch sampling with replacement (:460-472): indices come from the
//    counter hash, rows are gathered and cast to the compute dtype in one pass; padded rows are 0.
#include "pz_common.h"
#include "pz_launch.h"
#include "pz_kernels.h"

namespace pz {
namespace {

template <typename T> PZ_DEV double ldd(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double ldd<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> PZ_DEV void std_(T* p, int64_t i, double v) { p[i] = static_cast<T>(v); }
template <> PZ_DEV void std_<uint16_t>(uint16_t* p, int64_t i, double v) { p[i] = f2bf(static_cast<float>(v)); }

template <typename Tin, typename Tout, typename F>
__global__ void __launch_bounds__(256) stage_fwd_kernel(const Tin* __restrict__ x, Tout* __restrict__ y,
                                                        int64_t n, EpiSpec e) {
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const F v = static_cast<F>(ldd<Tin>(x, i));
    std_<Tout>(y, i, static_cast<double>(epi_fwd<F>(v, static_cast<uint64_t>(i), e)));
  }
}

// dx = epi_bwd(g, y); optional column sums over the last dim of width `cols`
template <typename T, typename F>
__global__ void __launch_bounds__(256) stage_bwd_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                        T* __restrict__ dx, int64_t n, EpiSpec e) {
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const F gv = static_cast<F>(ldd<T>(g, i));
    const F yv = static_cast<F>(ldd<T>(y, i));
    std_<T>(dx, i, static_cast<double>(epi_bwd<F>(gv, yv, static_cast<uint64_t>(i), e)));
  }
}

int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return static_cast<int>(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

// ---------------------------------------------------------------------------------------------
// cross-entropy head: one wave per row
// ---------------------------------------------------------------------------------------------
template <typename T, typename F>
__global__ void __launch_bounds__(256) xent_head_kernel(XentArgs a) {
  const T* __restrict__ logits = static_cast<const T*>(a.logits);
  T* __restrict__ dh = static_cast<T*>(a.dh);
  T* __restrict__ probs = static_cast<T*>(a.probs);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  __shared__ float loss_part[4];
  float row_loss = 0.f;
  if (row < a.rows) {
    const T* lr = logits + static_cast<int64_t>(row) * a.ld;
    if (row < a.rows_valid) {
      F mx = -INFINITY;
      for (int c = lane; c < a.cols; c += 64) mx = fmax(mx, static_cast<F>(ldd<T>(lr, c)));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
      F se = F(0);
      for (int c = lane; c < a.cols; c += 64) se += fexp(static_cast<F>(ldd<T>(lr, c)) - mx);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
      const int64_t label = a.labels[row];
      const F lse = mx + log(se);
      const F inv = F(1) / se;
      if (lane == 0) row_loss = static_cast<float>((lse - static_cast<F>(ldd<T>(lr, label))) * static_cast<F>(a.loss_scale));
      for (int c = lane; c < a.cols; c += 64) {
        const F pr = fexp(static_cast<F>(ldd<T>(lr, c)) - mx) * inv;
        if (probs != nullptr) std_<T>(probs, static_cast<int64_t>(row) * a.ld_probs + c, static_cast<double>(pr));
        if (dh != nullptr) {
          F g = (pr - (c == label ? F(1) : F(0))) * static_cast<F>(a.grad_scale);
          const uint64_t idx = static_cast<uint64_t>(row) * static_cast<uint64_t>(a.idx_ld) + c;
          g = epi_bwd<F>(g, F(0), idx, a.epi);
          std_<T>(dh, static_cast<int64_t>(row) * a.ld_dh + c, static_cast<double>(g));
          if (a.colsum != nullptr) atomicAdd(a.colsum + c, static_cast<float>(g));
        }
      }
    } else if (dh != nullptr) {
      for (int c = lane; c < a.cols; c += 64) std_<T>(dh, static_cast<int64_t>(row) * a.ld_dh + c, 0.0);
    }
  }
  if (a.loss != nullptr) {
    if (lane == 0) loss_part[threadIdx.x >> 6] = row_loss;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(a.loss, loss_part[0] + loss_part[1] + loss_part[2] + loss_part[3]);
  }
}

// ---------------------------------------------------------------------------------------------
// MSE head: loss = mean((y - t)^2); dx = epi_bwd(2 (y - t) / numel, y)
// ---------------------------------------------------------------------------------------------
template <typename T, typename F>
__global__ void __launch_bounds__(256) mse_head_kernel(MseArgs a) {
  const T* __restrict__ y = static_cast<const T*>(a.y);
  const T* __restrict__ t = static_cast<const T*>(a.target);
  T* __restrict__ dh = static_cast<T*>(a.dh);
  __shared__ float part[4];
  float acc = 0.f;
  const int64_t n = static_cast<int64_t>(a.rows) * a.cols;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const int64_t r = i / a.cols, c = i - r * a.cols;
    F g = F(0);
    if (r < a.rows_valid) {
      const F yv = static_cast<F>(ldd<T>(y, r * a.ld_y + c));
      const F d = yv - static_cast<F>(ldd<T>(t, r * a.ld_t + c));
      acc += static_cast<float>(d * d * static_cast<F>(a.loss_scale));
      g = epi_bwd<F>(F(2) * d * static_cast<F>(a.grad_scale), yv, static_cast<uint64_t>(r * a.idx_ld + c), a.epi);
    }
    if (dh != nullptr) {
      std_<T>(dh, r * a.ld_dh + c, static_cast<double>(g));
      if (a.colsum != nullptr && g != F(0)) atomicAdd(a.colsum + c, static_cast<float>(g));
    }
  }
  if (a.loss != nullptr) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(a.loss, part[0] + part[1] + part[2] + part[3]);
  }
}

// ---------------------------------------------------------------------------------------------
// row softmax (one wave per row)
// ---------------------------------------------------------------------------------------------
template <typename T, typename F>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const T* __restrict__ x, T* __restrict__ y, int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + static_cast<int64_t>(row) * cols;
  T* yr = y + static_cast<int64_t>(row) * cols;
  F mx = -INFINITY;
  for (int c = lane; c < cols; c += 64) mx = fmax(mx, static_cast<F>(ldd<T>(xr, c)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o, 64));
  F se = F(0);
  for (int c = lane; c < cols; c += 64) se += fexp(static_cast<F>(ldd<T>(xr, c)) - mx);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  const F inv = F(1) / se;
  for (int c = lane; c < cols; c += 64) std_<T>(yr, c, static_cast<double>(fexp(static_cast<F>(ldd<T>(xr, c)) - mx) * inv));
}

// softmax backward: dx = y * (g - sum(g*y))
template <typename T, typename F>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                          T* __restrict__ dx, int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t base = static_cast<int64_t>(row) * cols;
  F dot = F(0);
  for (int c = lane; c < cols; c += 64) dot += static_cast<F>(ldd<T>(g, base + c)) * static_cast<F>(ldd<T>(y, base + c));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) dot += __shfl_xor(dot, o, 64);
  for (int c = lane; c < cols; c += 64) {
    const F yv = static_cast<F>(ldd<T>(y, base + c));
    std_<T>(dx, base + c, static_cast<double>(yv * (static_cast<F>(ldd<T>(g, base + c)) - dot)));
  }
}

// column sums of a [rows][cols] matrix into fp32 (atomic per 64-column strip per block)
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ x, float* __restrict__ out, int rows,
                                                     int cols, int rows_per_block) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float s = 0.f;
  if (c < cols)
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) s += static_cast<float>(ldd<T>(x, static_cast<int64_t>(r) * cols + c));
  __shared__ float part[4][64];
  part[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  if (threadIdx.x < 64 && c < cols) atomicAdd(out + c, part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x]);
}

// ---------------------------------------------------------------------------------------------
// minibatch gather: out[i] = cast(data[idx_i]), idx_i = hash(seed, i) mod n_data (or given)
// ---------------------------------------------------------------------------------------------
template <typename Tin, typename Tout>
__global__ void __launch_bounds__(256) gather_rows_kernel(GatherArgs a) {
  const Tin* __restrict__ src = static_cast<const Tin*>(a.data);
  Tout* __restrict__ dst = static_cast<Tout*>(a.out);
  const int row = blockIdx.x;
  int64_t pick = 0;
  if (row < a.rows_valid) {
    if (a.indices != nullptr) {
      pick = a.indices[row];
    } else {
      const uint32_t h = mix32(mix32(static_cast<uint32_t>(row) ^ a.seed_lo) ^ a.seed_hi);
      pick = static_cast<int64_t>((static_cast<uint64_t>(h) * static_cast<uint64_t>(a.n_data)) >> 32);
    }
    if (threadIdx.x == 0) {
      if (a.picked != nullptr) a.picked[row] = pick;
      if (a.labels_out != nullptr) a.labels_out[row] = a.labels_in[pick];
    }
  } else if (threadIdx.x == 0 && a.labels_out != nullptr) {
    a.labels_out[row] = 0;
  }
  const int64_t so = pick * a.ld_data;
  const int64_t dof = static_cast<int64_t>(row) * a.ld_out;
  for (int c = threadIdx.x; c < a.cols; c += 256) {
    const double v = row < a.rows_valid ? ldd<Tin>(src, so + c) : 0.0;
    std_<Tout>(dst, dof + c, v);
  }
}

}  // namespace

#define PZ_DISPATCH_FLOAT(dt, T, ...)                       \
  switch (dt) {                                             \
    case DT_BF16: { using T = uint16_t; __VA_ARGS__; break; } \
    case DT_F32: { using T = float; __VA_ARGS__; break; }     \
    case DT_F64: { using T = double; __VA_ARGS__; break; }    \
    default: return hipErrorInvalidValue;                     \
  }

template <typename T> struct MathOf { using type = float; };
template <> struct MathOf<double> { using type = double; };

hipError_t stage_fwd(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, const EpiSpec& e, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(x_dtype, Tin, PZ_DISPATCH_FLOAT(y_dtype, Tout, {
    using F = typename MathOf<Tout>::type;
    hipLaunchKernelGGL((stage_fwd_kernel<Tin, Tout, F>), dim3(grid_for(n)), dim3(256), 0, s,
                       static_cast<const Tin*>(x), static_cast<Tout*>(y), n, e);
  }));
  return hipGetLastError();
}

hipError_t stage_bwd(const void* g, const void* y, void* dx, int dtype, int64_t n, const EpiSpec& e, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((stage_bwd_kernel<T, F>), dim3(grid_for(n)), dim3(256), 0, s, static_cast<const T*>(g),
                       static_cast<const T*>(y), static_cast<T*>(dx), n, e);
  });
  return hipGetLastError();
}

hipError_t xent_head(const XentArgs& a, hipStream_t s) {
  if (a.rows <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(a.dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((xent_head_kernel<T, F>), dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
  });
  return hipGetLastError();
}

hipError_t mse_head(const MseArgs& a, hipStream_t s) {
  const int64_t n = static_cast<int64_t>(a.rows) * a.cols;
  if (n <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(a.dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((mse_head_kernel<T, F>), dim3(grid_for(n)), dim3(256), 0, s, a);
  });
  return hipGetLastError();
}

hipError_t softmax_rows(const void* x, void* y, int dtype, int rows, int cols, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((softmax_rows_kernel<T, F>), dim3((rows + 3) / 4), dim3(256), 0, s, static_cast<const T*>(x),
                       static_cast<T*>(y), rows, cols);
  });
  return hipGetLastError();
}

hipError_t softmax_bwd(const void* g, const void* y, void* dx, int dtype, int rows, int cols, hipStream_t s) {
  if (rows <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((softmax_bwd_kernel<T, F>), dim3((rows + 3) / 4), dim3(256), 0, s, static_cast<const T*>(g),
                       static_cast<const T*>(y), static_cast<T*>(dx), rows, cols);
  });
  return hipGetLastError();
}

hipError_t colsum(const void* x, int dtype, float* out, int rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  const int rpb = 256;
  dim3 grid((cols + 63) / 64, (rows + rpb - 1) / rpb);
  PZ_DISPATCH_FLOAT(dtype, T, {
    hipLaunchKernelGGL((colsum_kernel<T>), grid, dim3(256), 0, s, static_cast<const T*>(x), out, rows, cols, rpb);
  });
  return hipGetLastError();
}

hipError_t gather_rows(const GatherArgs& a, hipStream_t s) {
  if (a.rows <= 0) return hipSuccess;
  PZ_DISPATCH_FLOAT(a.data_dtype, Tin, PZ_DISPATCH_FLOAT(a.out_dtype, Tout, {
    hipLaunchKernelGGL((gather_rows_kernel<Tin, Tout>), dim3(a.rows), dim3(256), 0, s, a);
  }));
  return hipGetLastError();
}

}  // namespace pz
