// N6 — fused multi-tensor optimizer step over the flat fp32 master-parameter buffer.
//
// Replaces, per parameter, the reference's chain (neural_net_model.py:482-506):
//   L2 term gradient (autograd of `cost += l2 * sum(w**2)`, weights only)  -> folded into g
//   1/world gradient scaling (data parallel mean)                          -> folded into g
//   torch.optim.Adam single-tensor step (lerp_, mul_/addcmul_, sqrt/div/add_, addcdiv_)
//     or manual SGD `p.data -= lr * p.grad`
//   prev_weights clone + (w - pw).std() / (w.std() + 1e-8) for the progress points
//                                                                         -> partial sums
//   bf16 shadow refresh for the next step's MFMA GEMMs                    -> fused store
// in ONE pass over (p, g, m, v): 16 B/param read + 12 B/param written (+2 B shadow) instead of
// the reference's ~10 passes. Numerics follow torch.optim.Adam (foreach=False, capturable=False).
#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = kOptElemsPerBlock / kThreads;  // 16

PZ_DEV int find_segment(const int64_t* block_seg, int nseg, int block) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {  // last segment whose first block <= block
    const int mid = (lo + hi + 1) >> 1;
    if (block_seg[mid] <= block) lo = mid; else hi = mid - 1;
  }
  return lo;
}

PZ_DEV void block_reduce_add(double v[4], double* dst) {
  __shared__ double red[4][kThreads / 64];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = wave_sum_d(v[k]);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) red[k][w] = v[k];
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kThreads / 64; ++i) s += red[threadIdx.x][i];
    atomicAdd(dst + threadIdx.x, s);
  }
}

template <bool ADAM>
__global__ void __launch_bounds__(kThreads) optimizer_kernel(OptArgs a) {
  if (a.hp != nullptr) {
    const float* h = a.hp + 4 * static_cast<int64_t>(*a.epoch_ptr);
    a.lr = h[0];
    a.bias_c1 = h[1];
    a.bias_c2_sqrt = h[2];
  }
  const int seg_id = find_segment(a.block_seg, a.num_segments, blockIdx.x);
  const OptSegment seg = a.segments[seg_id];
  const int64_t local0 = (static_cast<int64_t>(blockIdx.x) - a.block_seg[seg_id]) * kOptElemsPerBlock;
  const bool weight = seg.is_weight != 0;
  const float l2x2 = weight ? 2.f * a.l2_lambda : 0.f;
  const float step_size = a.lr / a.bias_c1;
  double st[4] = {0.0, 0.0, 0.0, 0.0};

#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    const int64_t li = local0 + static_cast<int64_t>(u) * kThreads + threadIdx.x;
    if (li >= seg.numel) break;
    const int64_t gi = seg.offset + li;
    const float p0 = a.params[gi];
    const float graw = seg.grad16 != nullptr ? bf2f(seg.grad16[li]) : a.grads[gi];
    const float g = graw * a.grad_scale + l2x2 * p0;
    float p1;
    if constexpr (ADAM) {
      float m = a.exp_avg[gi];
      float v = a.exp_avg_sq[gi];
      m = m + (1.f - a.beta1) * (g - m);
      v = v * a.beta2 + (1.f - a.beta2) * g * g;
      const float denom = sqrtf(v) / a.bias_c2_sqrt + a.eps;
      p1 = p0 - step_size * (m / denom);
      a.exp_avg[gi] = m;
      a.exp_avg_sq[gi] = v;
    } else {
      p1 = p0 - a.lr * g;
    }
    a.params[gi] = p1;
    if (seg.shadow != nullptr) {
      if (seg.shadow_dtype == DT_BF16) static_cast<uint16_t*>(seg.shadow)[li] = f2bf(p1);
      else static_cast<float*>(seg.shadow)[li] = p1;
    }
    if (seg.stat_slot >= 0) {
      const double d = static_cast<double>(p1 - p0);
      st[0] += d; st[1] += d * d; st[2] += p1; st[3] += static_cast<double>(p1) * p1;
    }
  }
  if (seg.stat_slot >= 0 && a.stats != nullptr) block_reduce_add(st, a.stats + 4 * seg.stat_slot);
}

__global__ void __launch_bounds__(kThreads) segment_stats_kernel(const float* __restrict__ params,
                                                                 const OptSegment* segments, const int64_t* block_seg,
                                                                 int nseg, double* stats) {
  const int seg_id = find_segment(block_seg, nseg, blockIdx.x);
  const OptSegment seg = segments[seg_id];
  if (seg.stat_slot < 0) return;
  const int64_t local0 = (static_cast<int64_t>(blockIdx.x) - block_seg[seg_id]) * kOptElemsPerBlock;
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  for (int u = 0; u < kPerThread; ++u) {
    const int64_t li = local0 + static_cast<int64_t>(u) * kThreads + threadIdx.x;
    if (li >= seg.numel) break;
    const double w = params[seg.offset + li];
    st[2] += w; st[3] += w * w;
  }
  block_reduce_add(st, stats + 4 * seg.stat_slot);
}

PZ_DEV double std_from_sums(double s, double ss, double n) {
  if (n < 2) return NAN;
  const double var = (ss - s * s / n) / (n - 1.0);
  return sqrt(var > 0.0 ? var : 0.0);
}

// cost[e] = loss / world + l2 * sum_w ||w||^2 (weights in use during the step)
// ratios[row][slot] = std(w_new - w_old) / (std(w_new) + 1e-8)       (progress points only)
__global__ void step_finalize_kernel(FinalizeArgs a) {
  __shared__ double l2sum;
  if (a.epoch < 0) a.epoch = *a.epoch_ptr;
  if (a.ratio_row == -2) a.ratio_row = a.epoch % a.every == 0 ? a.epoch / a.every : -1;
  if (a.ratio_row >= a.n_ratio_rows) a.ratio_row = -1;
  __syncthreads();  // every thread has read the counter before thread 0 advances it below
  if (threadIdx.x == 0) l2sum = 0.0;
  __syncthreads();
  for (int k = threadIdx.x; k < a.nslots; k += blockDim.x) {
    atomicAdd(&l2sum, a.stats_prev[4 * k + 3]);
    if (a.ratio_row >= 0) {
      const double n = a.slot_numel[k];
      const double* c = a.stats_cur + 4 * k;
      const double sd = std_from_sums(c[0], c[1], n);
      const double sw = std_from_sums(c[2], c[3], n);
      a.ratios[static_cast<int64_t>(a.ratio_row) * a.nslots + k] = static_cast<float>(sd / (sw + 1e-8));
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double loss = 0.0;
    if (a.loss != nullptr) {
      for (int k = 0; k < a.loss_slots; ++k) loss += static_cast<double>(a.loss[k]);
      loss /= a.loss_div;
    }
    if (a.epoch < a.n_costs) a.costs[a.epoch] = static_cast<float>(loss + static_cast<double>(a.l2) * l2sum);
    if (a.epoch_ptr != nullptr) *a.epoch_ptr = a.epoch + 1;
  }
  __syncthreads();
  // the previous stats buffer becomes the next step's accumulation target
  for (int k = threadIdx.x; k < 4 * a.nslots; k += blockDim.x) a.stats_prev[k] = 0.0;
}

}  // namespace

hipError_t step_finalize(const FinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(step_finalize_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t optimizer_step(const OptArgs& a, hipStream_t s) {
  if (a.total_blocks <= 0) return hipSuccess;
  if (a.adam) hipLaunchKernelGGL(optimizer_kernel<true>, dim3(a.total_blocks), dim3(kThreads), 0, s, a);
  else hipLaunchKernelGGL(optimizer_kernel<false>, dim3(a.total_blocks), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t segment_stats(const float* params, const OptSegment* segments, const int64_t* block_seg, int num_segments,
                         int total_blocks, double* stats, hipStream_t s) {
  if (total_blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(segment_stats_kernel, dim3(total_blocks), dim3(kThreads), 0, s, params, segments, block_seg,
                     num_segments, stats);
  return hipGetLastError();
}

}  // namespace pz
