// N6 — fused multi-tensor optimizer step over the flat master-parameter buffer (fp32, or fp64
// for fp64 models: the reference's own precision, updated in fp64 like torch.optim.Adam does).
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
#include <cstdlib>

#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = kOptElemsPerBlock / kThreads;  // 16
constexpr float kE4m3Max = 448.f;

// four floats -> four OCP e4m3 bytes (saturated to +-448, round to nearest even)
PZ_DEV uint32_t e4m3x4(float a, float b, float c, float d) {
  auto sat = [](float x) { return fminf(fmaxf(x, -kE4m3Max), kE4m3Max); };
  uint32_t w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(a), sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(sat(c), sat(d), w, true);
  return w;
}

PZ_DEV int find_segment(const int64_t* block_seg, int nseg, int block) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {  // last segment whose first block <= block
    const int mid = (lo + hi + 1) >> 1;
    if (block_seg[mid] <= block) lo = mid; else hi = mid - 1;
  }
  return lo;
}

PZ_DEV void block_reduce_add(double v[4], double* dst, bool full = true) {
  __shared__ double red[4][kThreads / 64];
  if (!full) {  // only sum(w^2): one wave reduction, one atomic
    const double s = wave_sum_d(v[3]);
    if ((threadIdx.x & 63) == 0) red[3][threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
#pragma unroll
      for (int i = 0; i < kThreads / 64; ++i) t += red[3][i];
      atomicAdd(dst + 3, t);
    }
    return;
  }
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

// the optimizer's view of OptArgs in master precision R (hyper-parameters rounded once)
template <typename R>
struct OptView {
  R* params;
  R* grads;
  R* exp_avg;
  R* exp_avg_sq;
  R lr, beta1, beta2, eps, bias_c1, bias_c2_sqrt, grad_scale, l2_lambda;
  PZ_DEV explicit OptView(const OptArgs& a)
      : params(static_cast<R*>(a.params)), grads(static_cast<R*>(a.grads)), exp_avg(static_cast<R*>(a.exp_avg)),
        exp_avg_sq(static_cast<R*>(a.exp_avg_sq)), lr(static_cast<R>(a.lr)), beta1(static_cast<R>(a.beta1)),
        beta2(static_cast<R>(a.beta2)), eps(static_cast<R>(a.eps)), bias_c1(static_cast<R>(a.bias_c1)),
        bias_c2_sqrt(static_cast<R>(a.bias_c2_sqrt)), grad_scale(static_cast<R>(a.grad_scale)),
        l2_lambda(static_cast<R>(a.l2_lambda)) {}
};

// one parameter's update: returns the new value; m / v are Adam's moments (in and out)
template <bool ADAM, typename R>
PZ_DEV R update_one(const OptView<R>& a, R p0, R graw, R l2x2, R step_size, R& m, R& v) {
  return opt_update<ADAM, R>(p0, graw, a.grad_scale, l2x2, a.lr, step_size, a.beta1, a.beta2, a.bias_c2_sqrt, a.eps, m,
                             v);
}

// max |w_new| of the block -> one atomic per block (non-negative floats order like their bits)
PZ_DEV void block_amax_commit(float m, float* amax) {
  __shared__ float part[kThreads / 64];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kThreads / 64; ++i) m = fmaxf(m, part[i]);
    atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
  }
}

// full: the update-ratio sums too (progress epochs only); otherwise just sum(w^2), which the
// next step's cost needs for its L2 term
template <typename R>
PZ_DEV void add_stats(double st[4], R p0, R p1, bool full) {
  st[3] += static_cast<double>(p1) * p1;
  if (full) {
    const double d = static_cast<double>(p1 - p0);
    st[0] += d; st[1] += d * d; st[2] += p1;
  }
}

// 16-B vectors of R (float4 / double2) for the vectorised segments
template <typename R> struct Vec;
template <> struct Vec<float> { using T = float4; static constexpr int N = 4; };
template <> struct Vec<double> { using T = double2; static constexpr int N = 2; };
// NT: non-temporal (streaming) access for the once-per-step state streams (PZ_OPT_NT): the update
// moves ~28 B per parameter that nothing re-reads before the next step, and default-policy
// accesses let it evict the GEMMs' operands from the L2s and the Infinity Cache
template <typename R, bool NT = false>
PZ_DEV void vld(const R* p, R (&x)[Vec<R>::N]) {
  if constexpr (NT && Vec<R>::N == 4) {
    const f32x4_t q = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p));
    x[0] = q[0]; x[1] = q[1]; x[2] = q[2]; x[3] = q[3];
    return;
  }
  const typename Vec<R>::T q = *reinterpret_cast<const typename Vec<R>::T*>(p);
  if constexpr (Vec<R>::N == 4) { x[0] = q.x; x[1] = q.y; x[2] = q.z; x[3] = q.w; }
  else { x[0] = q.x; x[1] = q.y; }
}
template <typename R, bool NT = false>
PZ_DEV void vst(R* p, const R (&x)[Vec<R>::N]) {
  if constexpr (NT && Vec<R>::N == 4) {
    __builtin_nontemporal_store(f32x4_t{x[0], x[1], x[2], x[3]}, reinterpret_cast<f32x4_t*>(p));
    return;
  }
  typename Vec<R>::T q;
  if constexpr (Vec<R>::N == 4) { q.x = x[0]; q.y = x[1]; q.z = x[2]; q.w = x[3]; }
  else { q.x = x[0]; q.y = x[1]; }
  *reinterpret_cast<typename Vec<R>::T*>(p) = q;
}

// Segments whose offset and length are multiples of 4 (every dense weight: ParamStore aligns
// offsets to 64) move 16 B per lane per stream — p, g, m, v in and p, m, v, shadow out — so a
// wave instruction covers 1 KiB; other segments (odd-sized biases) take the scalar loop.
//
// Grid: min(total_blocks, kOptMaxResident) workgroups loop over the 4096-element work blocks, so
// a launch that overlaps the MFMA-bound GEMMs (side stream) gets all its workgroups resident
// beside the GEMM's instead of queueing behind the GEMM's pending ones.
template <bool ADAM, typename R, int PRE, bool NT = false>
PZ_DEV void optimizer_block(const OptArgs& args, const OptView<R>& a, int block, bool full) {
  constexpr int VN = Vec<R>::N;
  const int seg_id = find_segment(args.block_seg, args.num_segments, block);
  const OptSegment seg = args.segments[seg_id];
  const int64_t local0 = (static_cast<int64_t>(block) - args.block_seg[seg_id]) * kOptElemsPerBlock;
  const bool weight = seg.is_weight != 0;
  const R l2x2 = weight ? R(2) * a.l2_lambda : R(0);
  const R step_size = a.lr / a.bias_c1;
  const bool stats = seg.stat_slot >= 0;
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  float am = 0.f;  // max |w_new| (fp8 weight scaling, seg.amax)
  float q8 = 1.f;  // e4m3 copy scale (delayed: from the previous update's amax)
  if (seg.w8 != nullptr) {
    const float ap = *seg.w8_amax_prev;
    q8 = ap > 0.f ? kE4m3Max / ap : seg.w8_qs[0];
    if (local0 == 0 && threadIdx.x == 0) {  // the segment's first block publishes the record
      seg.w8_qs[0] = q8;
      seg.w8_qs[1] = 1.f / q8;
    }
  }

  if (((seg.offset | seg.numel) & 3) == 0) {
    // the loads of PRE consecutive vectors of the thread are issued before their first store (the
    // streams are distinct buffers, __restrict__): PRE x 4 x 16 B in flight per lane instead of one
    // vector's worth behind each store — the update is HBM-bound
    constexpr int UN = kPerThread / VN;
    static_assert(UN % PRE == 0, "preload groups");
#pragma unroll
    for (int u0 = 0; u0 < UN; u0 += PRE) {
    const R* __restrict__ P = a.params;
    const R* __restrict__ Gr = a.grads;
    const R* __restrict__ Mm = a.exp_avg;
    const R* __restrict__ Vv = a.exp_avg_sq;
    const uint16_t* __restrict__ G16 = seg.grad16;
    R p0[PRE][VN], g[PRE][VN], m[PRE][VN], v[PRE][VN];
    bool ok[PRE];
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      const int64_t li = local0 + (static_cast<int64_t>(u0 + u) * kThreads + threadIdx.x) * VN;
      ok[u] = li < seg.numel;
      const int64_t gi = seg.offset + (ok[u] ? li : 0);
      const int64_t lc = ok[u] ? li : 0;
#pragma unroll
      for (int k = 0; k < VN; ++k) m[u][k] = v[u][k] = R(0);
      if (!ok[u]) continue;
      vld<R, NT>(P + gi, p0[u]);
      if constexpr (VN == 4) {
        if (G16 != nullptr) {
          const uint2 q = *reinterpret_cast<const uint2*>(G16 + lc);
          g[u][0] = bf2f(q.x & 0xFFFF); g[u][1] = bf2f(q.x >> 16); g[u][2] = bf2f(q.y & 0xFFFF); g[u][3] = bf2f(q.y >> 16);
        } else {
          vld<R>(Gr + gi, g[u]);
        }
      } else {
        vld<R>(Gr + gi, g[u]);
      }
      if constexpr (ADAM) {
        vld<R, NT>(Mm + gi, m[u]);
        vld<R, NT>(Vv + gi, v[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < PRE; ++u) {
      if (!ok[u]) continue;
      const int64_t li = local0 + (static_cast<int64_t>(u0 + u) * kThreads + threadIdx.x) * VN;
      const int64_t gi = seg.offset + li;
      if (seg.zero_grad && seg.grad16 == nullptr) {
        const R z[VN] = {};
        vst<R>(a.grads + gi, z);
      }
      R p1[VN];
#pragma unroll
      for (int k = 0; k < VN; ++k) p1[k] = update_one<ADAM, R>(a, p0[u][k], g[u][k], l2x2, step_size, m[u][k], v[u][k]);
      if constexpr (ADAM) {
        vst<R, NT>(a.exp_avg + gi, m[u]);
        vst<R, NT>(a.exp_avg_sq + gi, v[u]);
      }
      vst<R, NT>(a.params + gi, p1);
      if constexpr (VN == 4) {
        if (seg.w8 != nullptr)
          *reinterpret_cast<uint32_t*>(seg.w8 + li) = e4m3x4(p1[0] * q8, p1[1] * q8, p1[2] * q8, p1[3] * q8);
        if (seg.shadow != nullptr) {
          if (seg.shadow_dtype == DT_BF16)
            *reinterpret_cast<uint2*>(static_cast<uint16_t*>(seg.shadow) + li) =
                make_uint2(pack_bf2(p1[0], p1[1]), pack_bf2(p1[2], p1[3]));
          else
            *reinterpret_cast<float4*>(static_cast<float*>(seg.shadow) + li) = make_float4(p1[0], p1[1], p1[2], p1[3]);
        }
      }
#pragma unroll
      for (int k = 0; k < VN; ++k) {
        if (stats) add_stats<R>(st, p0[u][k], p1[k], full);
        am = fmaxf(am, fabsf(static_cast<float>(p1[k])));
      }
    }
    }
  } else {
#pragma unroll
    for (int u = 0; u < kPerThread; ++u) {
      const int64_t li = local0 + static_cast<int64_t>(u) * kThreads + threadIdx.x;
      if (li >= seg.numel) break;
      const int64_t gi = seg.offset + li;
      const R p0 = a.params[gi];
      R graw;
      if constexpr (VN == 4) graw = seg.grad16 != nullptr ? bf2f(seg.grad16[li]) : a.grads[gi];
      else graw = a.grads[gi];
      if (seg.zero_grad) a.grads[gi] = R(0);
      R m = R(0), v = R(0);
      if constexpr (ADAM) {
        m = a.exp_avg[gi];
        v = a.exp_avg_sq[gi];
      }
      const R p1 = update_one<ADAM, R>(a, p0, graw, l2x2, step_size, m, v);
      if constexpr (ADAM) {
        a.exp_avg[gi] = m;
        a.exp_avg_sq[gi] = v;
      }
      a.params[gi] = p1;
      if (seg.w8 != nullptr) {
        const float x = static_cast<float>(p1) * q8;
        seg.w8[li] = static_cast<uint8_t>(e4m3x4(x, 0.f, 0.f, 0.f) & 0xFFu);
      }
      if (seg.shadow != nullptr) {
        if (seg.shadow_dtype == DT_BF16) static_cast<uint16_t*>(seg.shadow)[li] = f2bf(static_cast<float>(p1));
        else static_cast<float*>(seg.shadow)[li] = static_cast<float>(p1);
      }
      if (stats) add_stats<R>(st, p0, p1, full);
      am = fmaxf(am, fabsf(static_cast<float>(p1)));
    }
  }
  if (stats && args.stats != nullptr) block_reduce_add(st, args.stats + 4 * seg.stat_slot, full);
  if (seg.amax != nullptr) block_amax_commit(am, seg.amax);
}

template <bool ADAM, typename R, int PRE, bool NT = false>
__global__ void __launch_bounds__(kThreads) optimizer_kernel(OptArgs a) {
  int epoch = -1;
  if (a.epoch_ptr != nullptr) epoch = *a.epoch_ptr;
  if (a.hp != nullptr) {
    const double* h = a.hp + 4 * static_cast<int64_t>(epoch);
    a.lr = h[0];
    a.bias_c1 = h[1];
    a.bias_c2_sqrt = h[2];
  }
  const OptView<R> view(a);
  const bool full = a.stats_every == 1 || (a.stats_every > 1 && (epoch < 0 || epoch % a.stats_every == 0));
  for (int b = blockIdx.x; b < a.total_blocks; b += gridDim.x) {
    optimizer_block<ADAM, R, PRE, NT>(a, view, b, full);
    __syncthreads();  // the block reductions reuse their LDS slots
  }
}

template <typename R>
__global__ void __launch_bounds__(kThreads) segment_stats_kernel(const R* __restrict__ params,
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
    if (a.loss64 != nullptr) {
      for (int k = 0; k < a.loss_slots; ++k) {
        loss += a.loss64[k];
        a.loss64[k] = 0.0;  // ready for the next step's head
      }
      loss /= a.loss_div;
    } else if (a.loss != nullptr) {
      for (int k = 0; k < a.loss_slots; ++k) {
        loss += static_cast<double>(a.loss[k]);
        a.loss[k] = 0.f;  // ready for the next step's head
      }
      loss /= a.loss_div;
    }
    if (a.epoch < a.n_costs) a.costs[a.epoch] = loss + static_cast<double>(a.l2) * l2sum;
    if (a.epoch_ptr != nullptr) *a.epoch_ptr = a.epoch + 1;
  }
  __syncthreads();
  // the previous stats buffer becomes the next step's accumulation target
  for (int k = threadIdx.x; k < 4 * a.nslots; k += blockDim.x) a.stats_prev[k] = 0.0;
  for (int k = threadIdx.x; k < a.nclear; k += blockDim.x) a.clear[k] = 0.f;
}

}  // namespace

hipError_t step_finalize(const FinalizeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(step_finalize_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t optimizer_step(const OptArgs& a, hipStream_t s) {
  if (a.total_blocks <= 0) return hipSuccess;
  const int cap = a.max_grid;  // resident workgroups (0 = one per work block)
  const int grid = cap > 0 && cap < a.total_blocks ? cap : a.total_blocks;
  // one 16-B vector of each stream per load group (PRE = 1): measured 5.7 TB/s for the whole-model
  // Adam update in isolation vs 5.2 with all four of a thread's vectors loaded up front (PRE = 4:
  // more VGPRs, fewer resident waves), tools/opt_bw.py, profiles/r3_opt_preload.txt
  if (a.real == DT_F64) {
    if (a.adam) hipLaunchKernelGGL((optimizer_kernel<true, double, 1>), dim3(grid), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((optimizer_kernel<false, double, 1>), dim3(grid), dim3(kThreads), 0, s, a);
  } else {
    // non-temporal state streams (r4 A/B: mlp4 1.1081 -> 1.1023 ms)
    // (measured r6, not kept: 2 / 4 preloaded vector groups for the one-round launches — step-end
    // first layer, head weight — mlp4 1.101-1.112 vs 1.088-1.094 ms, profiles/r6_ab_opt_pre_small.txt)
    if (a.adam) hipLaunchKernelGGL((optimizer_kernel<true, float, 1, true>), dim3(grid), dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((optimizer_kernel<false, float, 1, true>), dim3(grid), dim3(kThreads), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t segment_stats(const void* params, int real, const OptSegment* segments, const int64_t* block_seg,
                         int num_segments, int total_blocks, double* stats, hipStream_t s) {
  if (total_blocks <= 0) return hipSuccess;
  if (real == DT_F64)
    hipLaunchKernelGGL(segment_stats_kernel<double>, dim3(total_blocks), dim3(kThreads), 0, s,
                       static_cast<const double*>(params), segments, block_seg, num_segments, stats);
  else
    hipLaunchKernelGGL(segment_stats_kernel<float>, dim3(total_blocks), dim3(kThreads), 0, s,
                       static_cast<const float*>(params), segments, block_seg, num_segments, stats);
  return hipGetLastError();
}

}  // namespace pz
