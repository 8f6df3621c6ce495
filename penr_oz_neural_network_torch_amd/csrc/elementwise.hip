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
  e = epi_resolve(e);
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    const F v = static_cast<F>(ldd<Tin>(x, i));
    std_<Tout>(y, i, static_cast<double>(epi_fwd<F>(v, static_cast<uint64_t>(i), e)));
  }
}

// dx = epi_bwd(g, y); optional column sums over the last dim of width `cols`
template <typename T, typename F>
__global__ void __launch_bounds__(256) stage_bwd_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                        T* __restrict__ dx, int64_t n, EpiSpec e) {
  e = epi_resolve(e);
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
// Row blocks: a 256-thread block owns kHeadRows rows (4 waves x kHeadRows/4 rows each). The
// bias-gradient column sums are accumulated in LDS (ds_add_f32) and flushed with ONE global
// atomic per column per block — per-element global atomics made this kernel 20x slower.
constexpr int kHeadRows = 16;
// bf16 CE head: rows per 16-wave block (2 per wave): halves the blocks adding into the same
// bias-gradient columns, whose contended atomics were half the kernel's time at 16
constexpr int kBf16HeadRows = 32;

// block loss -> one of `slots` accumulators (the consumer sums them): hundreds of blocks adding
// to ONE address serialise at L2 (measured: 512 blocks cost the CE head ~10 us)
PZ_DEV void block_loss_flush(float* loss, float v, float* red, int slots) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss + (slots > 1 ? blockIdx.x % slots : 0), red[0] + red[1] + red[2] + red[3]);
}
// fp64 models: the loss accumulates in double (the reference reports an fp64 cost)
PZ_DEV void block_loss_flush(double* loss, double v, double* red, int slots) {
  v = wave_sum_d(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss + (slots > 1 ? blockIdx.x % slots : 0), red[0] + red[1] + red[2] + red[3]);
}

template <typename A>
PZ_DEV void block_colsum_flush(A* colsum, const A* cs, int cols) {
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256)
    if (cs[c] != A(0)) atomicAdd(colsum + c, cs[c]);
}

// the bf16 heads' bias-gradient column sums: the block's wave partials (LDS [WAVES][cols]) summed in
// wave order, then float atomics, or (a.cs_ws: deterministic) the block's partial row and the
// ordered folds of pz_common.h det_colsum over groups of 16 blocks
template <int WAVES>
PZ_DEV void head_colsum_flush(const XentArgs& a, const float* cs_lds) {
  __shared__ int det_flag;
  for (int c = threadIdx.x; c < a.cols; c += WAVES * 64) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) t += cs_lds[w * a.cols + c];
    if (a.cs_ws != nullptr) st_wt(a.cs_ws + static_cast<int64_t>(blockIdx.x) * a.cols + c, t);
    else if (t != 0.f) atomicAdd(a.colsum + c, t);
  }
  if (a.cs_ws != nullptr)
    det_colsum<WAVES * 64>(a.cs_ws, a.cs_tickets, gridDim.x, 16, blockIdx.x, a.cols, a.cols, a.colsum,
                           (PZ_LDS int*)(&det_flag));
}

// accumulator pointers of a head: double for fp64 logits (loss64 / colsum64), float otherwise
template <typename F> PZ_DEV F* head_loss(void* f32, void* f64);
template <> PZ_DEV float* head_loss<float>(void* f32, void*) { return static_cast<float*>(f32); }
template <> PZ_DEV double* head_loss<double>(void*, void* f64) { return static_cast<double*>(f64); }

template <typename T, typename F>
__global__ void __launch_bounds__(256) xent_head_kernel(XentArgs a) {
  apply_scale_update(a.su);
  a.epi = epi_resolve(a.epi);
  extern __shared__ __attribute__((aligned(16))) char cs_raw[];
  F* cs_lds = reinterpret_cast<F*>(cs_raw);  // [cols] when a.colsum (LDS column partials)
  __shared__ F red[4];
  F* const loss = head_loss<F>(a.loss, a.loss64);
  F* const colsum = head_loss<F>(a.colsum, a.colsum64);
  const T* __restrict__ logits = static_cast<const T*>(a.logits);
  T* __restrict__ dh = static_cast<T*>(a.dh);
  T* __restrict__ probs = static_cast<T*>(a.probs);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool cs_on = colsum != nullptr && dh != nullptr;
  if (cs_on) {
    for (int c = threadIdx.x; c < a.cols; c += 256) cs_lds[c] = F(0);
    __syncthreads();
  }
  F loss_acc = F(0);
  for (int rr = 0; rr < kHeadRows / 4; ++rr) {
    const int row = blockIdx.x * kHeadRows + wave * (kHeadRows / 4) + rr;
    if (row >= a.rows) break;
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
      // the host rejects labels outside [0, cols) (IndexError); a bad one only ever yields a NaN
      // loss here, never an out-of-row read
      const bool lab_ok = label >= 0 && label < a.cols;
      const F xlab = lab_ok ? static_cast<F>(ldd<T>(lr, label)) : static_cast<F>(NAN);
      if (lane == 0) loss_acc += (lse - xlab) * static_cast<F>(a.loss_scale);
      for (int c = lane; c < a.cols; c += 64) {
        const F pr = fexp(static_cast<F>(ldd<T>(lr, c)) - mx) * inv;
        if (probs != nullptr) std_<T>(probs, static_cast<int64_t>(row) * a.ld_probs + c, static_cast<double>(pr));
        if (dh != nullptr) {
          F g = (pr - (c == label ? F(1) : F(0))) * static_cast<F>(a.grad_scale);
          const uint64_t idx = static_cast<uint64_t>(row) * static_cast<uint64_t>(a.idx_ld) + c;
          g = epi_bwd<F>(g, F(0), idx, a.epi);
          std_<T>(dh, static_cast<int64_t>(row) * a.ld_dh + c, static_cast<double>(g));
          if (cs_on) atomicAdd(&cs_lds[c], g);
        }
      }
    } else if (dh != nullptr) {
      for (int c = lane; c < a.cols; c += 64) std_<T>(dh, static_cast<int64_t>(row) * a.ld_dh + c, 0.0);
    }
  }
  if (loss != nullptr) block_loss_flush(loss, loss_acc, red, a.loss_slots);
  if (cs_on) block_colsum_flush(colsum, cs_lds, a.cols);
}

// bf16 fast path: every lane holds NCH chunks of 8 logits in registers (one read of the row),
// 16-B loads / stores, dropout masks two hashes per 4 elements. A wave's RPW rows are loaded up
// front (memory-level parallelism), bias-gradient column partials stay in registers and are
// reduced across the block's waves through LDS once (no LDS atomics: they made this 60 us).
// WAVES = 16 (one row per wave, 1024-thread blocks): the row's reductions are serial shuffle
// chains, so the kernel is latency-bound and wants many resident waves; the block still owns
// kBf16HeadRows rows, which keeps the bias-gradient atomics at one per column per 32 rows.
template <int NCH, int WAVES, int RPB = kBf16HeadRows>
__global__ void __launch_bounds__(WAVES * 64) xent_head_bf16_kernel(XentArgs a) {
  apply_scale_update(a.su);
  a.epi = epi_resolve(a.epi);
  extern __shared__ float cs_lds[];  // [WAVES][cols] wave partials (when colsum)
  __shared__ float red[WAVES];
  constexpr int RPW = RPB / WAVES;
  static_assert(RPW * WAVES == RPB, "rows per block split over the waves");
  const uint16_t* __restrict__ logits = static_cast<const uint16_t*>(a.logits);
  uint16_t* __restrict__ dh = static_cast<uint16_t*>(a.dh);
  uint16_t* __restrict__ probs = static_cast<uint16_t*>(a.probs);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool cs_on = a.colsum != nullptr && dh != nullptr;
  float cs[NCH][8];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[j][e] = 0.f;
  bool ok[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) ok[j] = (lane + 64 * j) * 8 < a.cols;
  const int row0 = blockIdx.x * RPB + wave * RPW;
  uint4 raw[RPW][NCH];
  int64_t labels[RPW];  // fetched with the logits: no dependent load inside the row loop
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    labels[rr] = row < a.rows_valid ? a.labels[row] : -1;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
      raw[rr][j] = (row < a.rows && ok[j])
                       ? *reinterpret_cast<const uint4*>(logits + static_cast<int64_t>(row) * a.ld + (lane + 64 * j) * 8)
                       : make_uint4(0, 0, 0, 0);
  }
  float loss_acc = 0.f;
  float amax8 = 0.f;
  const float qs8 = a.out8 != nullptr ? *a.out8_qscale : 1.f;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    if (row >= a.rows) break;
    float v[NCH][8];
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const uint32_t w[4] = {raw[rr][j].x, raw[rr][j].y, raw[rr][j].z, raw[rr][j].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[j][2 * e] = bf2f(w[e] & 0xFFFF); v[j][2 * e + 1] = bf2f(w[e] >> 16); }
    }
    if (row < a.rows_valid) {
      const int64_t label = labels[rr];
      float mx = -INFINITY, xl = 0.f;  // xl: the label's logit, taken from registers
#pragma unroll
      for (int j = 0; j < NCH; ++j)
        if (ok[j])
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            mx = fmaxf(mx, v[j][e]);
            xl += (lane + 64 * j) * 8 + e == label ? v[j][e] : 0.f;
          }
      mx = wave_max(mx);
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[j][e] = ok[j] ? __expf(v[j][e] - mx) : 0.f;
          se += v[j][e];
        }
      se = wave_sum(se);
      xl = wave_sum(xl);
      const float inv = 1.f / se;
      if (lane == 0) loss_acc += (mx + __logf(se) - xl) * static_cast<float>(a.loss_scale);
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        if (!ok[j]) continue;
        const int c0 = (lane + 64 * j) * 8;
        float pr[8], g[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pr[e] = v[j][e] * inv;
          g[e] = (pr[e] - (c0 + e == label ? 1.f : 0.f)) * static_cast<float>(a.grad_scale);
        }
        if (probs != nullptr)
          *reinterpret_cast<uint4*>(probs + static_cast<int64_t>(row) * a.ld_probs + c0) =
              make_uint4(pack_bf2(pr[0], pr[1]), pack_bf2(pr[2], pr[3]), pack_bf2(pr[4], pr[5]), pack_bf2(pr[6], pr[7]));
        if (dh != nullptr) {
          const uint64_t idx = static_cast<uint64_t>(row) * static_cast<uint64_t>(a.idx_ld) + c0;
          const float zero4[4] = {0.f, 0.f, 0.f, 0.f};
          epi_bwd4(g, zero4, idx, a.epi);
          epi_bwd4(g + 4, zero4, idx + 4, a.epi);
          const uint4 gb = make_uint4(pack_bf2(g[0], g[1]), pack_bf2(g[2], g[3]), pack_bf2(g[4], g[5]), pack_bf2(g[6], g[7]));
          if (!a.skip_dh) *reinterpret_cast<uint4*>(dh + static_cast<int64_t>(row) * a.ld_dh + c0) = gb;
          if (a.out8 != nullptr) {  // e5m2 copy of the stored bf16 values (as quantize_rows would)
            const uint32_t w[4] = {gb.x, gb.y, gb.z, gb.w};
            float x[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              x[2 * e] = bf2f(w[e] & 0xFFFFu);
              x[2 * e + 1] = bf2f(w[e] >> 16);
              amax8 = fmaxf(amax8, fmaxf(fabsf(x[2 * e]), fabsf(x[2 * e + 1])));
            }
            *reinterpret_cast<u32x2_t*>(a.out8 + static_cast<int64_t>(row) * a.ld_out8 + c0) = to_e5m2x8(x, qs8);
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[j][e] += g[e];
        }
      }
    } else if (dh != nullptr) {
#pragma unroll
      for (int j = 0; j < NCH; ++j)
        if (ok[j]) {
          if (!a.skip_dh)
            *reinterpret_cast<uint4*>(dh + static_cast<int64_t>(row) * a.ld_dh + (lane + 64 * j) * 8) =
                make_uint4(0, 0, 0, 0);
          if (a.out8 != nullptr)
            *reinterpret_cast<u32x2_t*>(a.out8 + static_cast<int64_t>(row) * a.ld_out8 + (lane + 64 * j) * 8) =
                u32x2_t{0u, 0u};
        }
    }
  }
  if (a.out8 != nullptr && a.amax != nullptr) {  // one atomic per block
    __shared__ float red8[WAVES];
    const float m = wave_max(amax8);
    if (lane == 0) red8[wave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = red8[0];
#pragma unroll
      for (int w = 1; w < WAVES; ++w) t = fmaxf(t, red8[w]);
      atomicMax(reinterpret_cast<unsigned int*>(a.amax), __float_as_uint(t));
    }
  }
  if (a.loss != nullptr) {
    const float v = wave_sum(loss_acc);
    if (lane == 0) red[wave] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) t += red[w];
      atomicAdd(a.loss + (a.loss_slots > 1 ? blockIdx.x % a.loss_slots : 0), t);
    }
  }
  if (cs_on) {
    float* mine = cs_lds + wave * a.cols;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
      if (ok[j])
#pragma unroll
        for (int e = 0; e < 8; ++e) mine[(lane + 64 * j) * 8 + e] = cs[j][e];
    __syncthreads();
    head_colsum_flush<WAVES>(a, cs_lds);
  }
}

// ---------------------------------------------------------------------------------------------
// MSE head: loss = mean((y - t)^2); dx = epi_bwd(2 (y - t) / numel, y)
// ---------------------------------------------------------------------------------------------
template <typename T, typename F>
__global__ void __launch_bounds__(256) mse_head_kernel(MseArgs a) {
  a.epi = epi_resolve(a.epi);
  extern __shared__ __attribute__((aligned(16))) char cs_raw[];
  F* cs_lds = reinterpret_cast<F*>(cs_raw);
  __shared__ F red[4];
  F* const loss = head_loss<F>(a.loss, a.loss64);
  F* const colsum = head_loss<F>(a.colsum, a.colsum64);
  const T* __restrict__ y = static_cast<const T*>(a.y);
  const T* __restrict__ t = static_cast<const T*>(a.target);
  T* __restrict__ dh = static_cast<T*>(a.dh);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool cs_on = colsum != nullptr && dh != nullptr;
  if (cs_on) {
    for (int c = threadIdx.x; c < a.cols; c += 256) cs_lds[c] = F(0);
    __syncthreads();
  }
  F acc = F(0);
  for (int rr = 0; rr < kHeadRows / 4; ++rr) {
    const int64_t r = static_cast<int64_t>(blockIdx.x) * kHeadRows + wave * (kHeadRows / 4) + rr;
    if (r >= a.rows) break;
    for (int c = lane; c < a.cols; c += 64) {
      F g = F(0);
      if (r < a.rows_valid) {
        const F yv = static_cast<F>(ldd<T>(y, r * a.ld_y + c));
        const F d = yv - static_cast<F>(ldd<T>(t, r * a.ld_t + c));
        acc += d * d * static_cast<F>(a.loss_scale);
        g = epi_bwd<F>(F(2) * d * static_cast<F>(a.grad_scale), yv, static_cast<uint64_t>(r * a.idx_ld + c), a.epi);
      }
      if (dh != nullptr) {
        std_<T>(dh, r * a.ld_dh + c, static_cast<double>(g));
        if (cs_on) atomicAdd(&cs_lds[c], g);
      }
    }
  }
  if (loss != nullptr) block_loss_flush(loss, acc, red, a.loss_slots);
  if (cs_on) block_colsum_flush(colsum, cs_lds, a.cols);
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

// column sums of a [rows][cols] matrix into fp32 (fp64 for fp64 data). ws == nullptr: atomic per
// 64-column strip per block; otherwise each block stores its partial row ws[blockIdx.y][c] and
// colsum_fold_kernel adds the rows to out in block order — the sum order never depends on which
// block finished first (deterministic training, PZ_DETERMINISTIC)
template <typename T, typename A>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ x, A* __restrict__ out, int rows,
                                                     int cols, int rows_per_block, A* __restrict__ ws) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  A s = A(0);
  if (c < cols)
    for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) s += static_cast<A>(ldd<T>(x, static_cast<int64_t>(r) * cols + c));
  __shared__ A part[4][64];
  part[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  if (threadIdx.x < 64 && c < cols) {
    const A v = part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] + part[3][threadIdx.x];
    if (ws != nullptr) ws[static_cast<int64_t>(blockIdx.y) * cols + c] = v;
    else atomicAdd(out + c, v);
  }
}

template <typename A>
__global__ void __launch_bounds__(256) colsum_fold_kernel(const A* __restrict__ ws, A* __restrict__ out, int parts,
                                                          int cols) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  A s = A(0);
  for (int y = 0; y < parts; ++y) s += ws[static_cast<int64_t>(y) * cols + c];
  out[c] += s;
}

// Lean bf16 CE head for the trainer's logits stage: no probabilities, dZ always stored, the
// logits' dropout (if any) applied BEFORE the head only (the reference's linear -> dropout ->
// softmax), and the optional bias-gradient sums / e5m2 copy selected at COMPILE time. The general
// kernel above carries every option as runtime branches: ~4.4k instructions, 13.4 us for the
// [8192, 1024] head with no dropout and no column sums against a 4.1 us copy of the same bytes
// (tools/head_bench.py). One row per wave-iteration, every load issued up front.
template <int NCH, int WAVES, bool COLSUM, bool OUT8, bool DROP>
__global__ void __launch_bounds__(WAVES * 64) xent_head_lean_kernel(XentArgs a) {
  apply_scale_update(a.su);
  const EpiSpec e = epi_resolve(a.epi);
  extern __shared__ float cs_lds[];  // [WAVES][cols] wave partials (COLSUM)
  __shared__ float red[WAVES];
  constexpr int RPW = kBf16HeadRows / WAVES;
  const uint16_t* __restrict__ logits = static_cast<const uint16_t*>(a.logits);
  uint16_t* __restrict__ dh = static_cast<uint16_t*>(a.dh);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float cs[NCH][8];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
#pragma unroll
    for (int q = 0; q < 8; ++q) cs[j][q] = 0.f;
  const int row0 = blockIdx.x * kBf16HeadRows + wave * RPW;
  uint4 raw[RPW][NCH];
  int labels[RPW];
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    labels[rr] = row < a.rows_valid ? static_cast<int>(a.labels[row]) : -1;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
      raw[rr][j] = row < a.rows ? *reinterpret_cast<const uint4*>(logits + static_cast<int64_t>(row) * a.ld + (lane + 64 * j) * 8)
                                : make_uint4(0, 0, 0, 0);
  }
  const float gs = static_cast<float>(a.grad_scale);
  const float qs8 = OUT8 ? *a.out8_qscale : 1.f;
  float loss_acc = 0.f, amax8 = 0.f;
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    if (row >= a.rows) break;
    const bool valid = row < a.rows_valid;  // (wave-uniform) padding rows: zero gradient
    const int label = labels[rr];
    float v[NCH][8];
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const uint32_t w[4] = {raw[rr][j].x, raw[rr][j].y, raw[rr][j].z, raw[rr][j].w};
#pragma unroll
      for (int q = 0; q < 4; ++q) { v[j][2 * q] = bf2f(w[q] & 0xFFFF); v[j][2 * q + 1] = bf2f(w[q] >> 16); }
    }
    float mx = -INFINITY, xl = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        mx = fmaxf(mx, v[j][q]);
        xl += (lane + 64 * j) * 8 + q == label ? v[j][q] : 0.f;
      }
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        v[j][q] = __expf(v[j][q] - mx);
        se += v[j][q];
      }
    se = wave_sum(se);
    xl = wave_sum(xl);
    if (valid && lane == 0) loss_acc += (mx + __logf(se) - xl) * static_cast<float>(a.loss_scale);
    const float inv = valid ? gs / se : 0.f;  // padding rows: every gradient 0
    const uint64_t row_idx = static_cast<uint64_t>(row) * static_cast<uint64_t>(a.idx_ld);
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c0 = (lane + 64 * j) * 8;
      float g[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) g[q] = v[j][q] * inv - (c0 + q == label && valid ? gs : 0.f);
      if constexpr (DROP) {  // d(dropout_pre): keep ? g * scale : 0 (pairs 2p, 2p+1 share a hash)
        const uint32_t p0 = static_cast<uint32_t>((row_idx + c0) >> 1);
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t b = mix32((p0 + h) ^ e.key_pre);
          g[2 * h] = (b & 0xFFFFu) >= e.thresh16 ? g[2 * h] * e.scale : 0.f;
          g[2 * h + 1] = (b >> 16) >= e.thresh16 ? g[2 * h + 1] * e.scale : 0.f;
        }
      }
      const uint4 gb = make_uint4(pack_bf2(g[0], g[1]), pack_bf2(g[2], g[3]), pack_bf2(g[4], g[5]), pack_bf2(g[6], g[7]));
      if (!a.skip_dh) *reinterpret_cast<uint4*>(dh + static_cast<int64_t>(row) * a.ld_dh + c0) = gb;
      if constexpr (OUT8) {  // e5m2 copy of the stored bf16 values (as quantize_rows would)
        const uint32_t w[4] = {gb.x, gb.y, gb.z, gb.w};
        float x[8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x[2 * q] = bf2f(w[q] & 0xFFFFu);
          x[2 * q + 1] = bf2f(w[q] >> 16);
          amax8 = fmaxf(amax8, fmaxf(fabsf(x[2 * q]), fabsf(x[2 * q + 1])));
        }
        *reinterpret_cast<u32x2_t*>(a.out8 + static_cast<int64_t>(row) * a.ld_out8 + c0) = to_e5m2x8(x, qs8);
      }
      if constexpr (COLSUM) {
#pragma unroll
        for (int q = 0; q < 8; ++q) cs[j][q] += g[q];
      }
    }
  }
  if constexpr (OUT8) {
    if (a.amax != nullptr) {  // one atomic per block
      __shared__ float red8[WAVES];
      const float m = wave_max(amax8);
      if (lane == 0) red8[wave] = m;
      __syncthreads();
      if (threadIdx.x == 0) {
        float t = red8[0];
#pragma unroll
        for (int w = 1; w < WAVES; ++w) t = fmaxf(t, red8[w]);
        atomicMax(reinterpret_cast<unsigned int*>(a.amax), __float_as_uint(t));
      }
    }
  }
  if (a.loss != nullptr) {
    const float t = wave_sum(loss_acc);
    if (lane == 0) red[wave] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) s += red[w];
      atomicAdd(a.loss + (a.loss_slots > 1 ? blockIdx.x % a.loss_slots : 0), s);
    }
  }
  if constexpr (COLSUM) {
    float* mine = cs_lds + wave * a.cols;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
      for (int q = 0; q < 8; ++q) mine[(lane + 64 * j) * 8 + q] = cs[j][q];
    __syncthreads();
    head_colsum_flush<WAVES>(a, cs_lds);
  }
}

// ---------------------------------------------------------------------------------------------
// minibatch gather: out[i] = cast(data[idx_i]), idx_i = hash(seed, i) mod n_data (or given)
// ---------------------------------------------------------------------------------------------
template <typename Tin, typename Tout>
__global__ void __launch_bounds__(256) gather_rows_kernel(GatherArgs a) {
  apply_scale_update(a.su);
  if (a.epoch_ptr != nullptr) gather_seed(a.seed_lo, a.seed_hi, static_cast<uint32_t>(*a.epoch_ptr));
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
  if (a.out8 != nullptr)
    for (int c = threadIdx.x; c < a.cols; c += 256)
      a.out8[static_cast<int64_t>(row) * a.ld_out8 + c] = row < a.rows_valid ? a.data8[pick * a.ld_data8 + c] : 0;
}

// vectorised bf16-output gather (fp32 or bf16 table): one wave per row, 8 elements (one 16-B
// store) per lane-iteration; the sampled index is hashed once per row by lane 0
template <typename Tin>
__global__ void __launch_bounds__(256) gather_rows_vec_kernel(GatherArgs a) {
  apply_scale_update(a.su);
  if (a.epoch_ptr != nullptr) gather_seed(a.seed_lo, a.seed_hi, static_cast<uint32_t>(*a.epoch_ptr));
  const Tin* __restrict__ src = static_cast<const Tin*>(a.data);
  uint16_t* __restrict__ dst = static_cast<uint16_t*>(a.out);
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= a.rows) return;
  int64_t pick = 0;
  const bool valid = row < a.rows_valid;
  if (valid) {
    if (a.indices != nullptr) {
      pick = a.indices[row];
    } else {
      const uint32_t h = mix32(mix32(static_cast<uint32_t>(row) ^ a.seed_lo) ^ a.seed_hi);
      pick = static_cast<int64_t>((static_cast<uint64_t>(h) * static_cast<uint64_t>(a.n_data)) >> 32);
    }
    if (lane == 0) {
      if (a.picked != nullptr) a.picked[row] = pick;
      if (a.labels_out != nullptr) a.labels_out[row] = a.labels_in[pick];
    }
  } else if (lane == 0 && a.labels_out != nullptr) {
    a.labels_out[row] = 0;
  }
  const Tin* s = src + pick * a.ld_data;
  uint16_t* d = dst + static_cast<int64_t>(row) * a.ld_out;
  for (int c = lane * 8; c < a.cols; c += 64 * 8) {
    uint4 o = make_uint4(0, 0, 0, 0);
    if (valid) {
      if constexpr (sizeof(Tin) == 4) {
        const float4 x0 = *reinterpret_cast<const float4*>(s + c);
        const float4 x1 = *reinterpret_cast<const float4*>(s + c + 4);
        o = make_uint4(pack_bf2(x0.x, x0.y), pack_bf2(x0.z, x0.w), pack_bf2(x1.x, x1.y), pack_bf2(x1.z, x1.w));
      } else {
        o = *reinterpret_cast<const uint4*>(s + c);
      }
    }
    *reinterpret_cast<uint4*>(d + c) = o;
    if (a.out8 != nullptr) {  // the same 8 columns of the e4m3 table: one 8-B load / store
      const uint2 q = valid ? *reinterpret_cast<const uint2*>(a.data8 + pick * a.ld_data8 + c) : make_uint2(0, 0);
      *reinterpret_cast<uint2*>(a.out8 + static_cast<int64_t>(row) * a.ld_out8 + c) = q;
    }
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

template <int NCH, int W, int RPB = kBf16HeadRows>
hipError_t launch_xent_bf16(const XentArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  static bool attr = false;  // > 64 KiB of dynamic LDS (W partial rows of up to 2048 columns)
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(xent_head_bf16_kernel<NCH, W, RPB>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, W * 512 * NCH * 4);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((xent_head_bf16_kernel<NCH, W, RPB>), grid, dim3(W * 64), lds, s, a);
  return hipGetLastError();
}

template <int NCH, bool CS, bool O8, bool DR>
hipError_t launch_xent_lean1(const XentArgs& a, dim3 grid, size_t lds, hipStream_t s) {
  constexpr int W = 16;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(xent_head_lean_kernel<NCH, W, CS, O8, DR>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, W * 512 * NCH * 4);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((xent_head_lean_kernel<NCH, W, CS, O8, DR>), grid, dim3(W * 64), lds, s, a);
  return hipGetLastError();
}
template <int NCH>
hipError_t launch_xent_lean_n(const XentArgs& a, bool cs, bool o8, bool dr, dim3 grid, size_t lds, hipStream_t s) {
  if (cs) {
    if (o8) return dr ? launch_xent_lean1<NCH, true, true, true>(a, grid, lds, s) : launch_xent_lean1<NCH, true, true, false>(a, grid, lds, s);
    return dr ? launch_xent_lean1<NCH, true, false, true>(a, grid, lds, s) : launch_xent_lean1<NCH, true, false, false>(a, grid, lds, s);
  }
  if (o8) return dr ? launch_xent_lean1<NCH, false, true, true>(a, grid, lds, s) : launch_xent_lean1<NCH, false, true, false>(a, grid, lds, s);
  return dr ? launch_xent_lean1<NCH, false, false, true>(a, grid, lds, s) : launch_xent_lean1<NCH, false, false, false>(a, grid, lds, s);
}
hipError_t launch_xent_lean(const XentArgs& a, int nch, bool cs, bool o8, bool dr, dim3 grid, size_t lds, hipStream_t s) {
  if (nch == 1) return launch_xent_lean_n<1>(a, cs, o8, dr, grid, lds, s);
  if (nch == 2) return launch_xent_lean_n<2>(a, cs, o8, dr, grid, lds, s);
  return launch_xent_lean_n<4>(a, cs, o8, dr, grid, lds, s);
}

constexpr int kMaxLdsCols = 16384;  // 64 KiB of fp32 column partials

// the bf16 fast path (the only one with the e5m2 copy / skip_dh)
bool xent_head_out8_ok(const XentArgs& a) {
  return a.dtype == DT_BF16 && a.cols % 8 == 0 && a.cols <= 2048 && a.ld % 8 == 0 && a.dh != nullptr &&
         a.ld_dh % 8 == 0 && (a.probs == nullptr || a.ld_probs % 8 == 0) && a.idx_ld % 2 == 0 &&
         (reinterpret_cast<uintptr_t>(a.logits) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.dh) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(a.probs) & 15) == 0 && (a.out8 == nullptr || (a.ld_out8 % 8 == 0 &&
         (reinterpret_cast<uintptr_t>(a.out8) & 7) == 0 && a.out8_qscale != nullptr));
}

hipError_t xent_head(const XentArgs& in, hipStream_t s) {
  if (in.rows <= 0) return hipSuccess;
  XentArgs a = in;
  if ((a.out8 != nullptr || a.skip_dh) && !xent_head_out8_ok(a)) return hipErrorInvalidValue;
  void* colsum_direct = nullptr;
  const bool acc64 = a.dtype == DT_F64;
  if ((a.colsum != nullptr || a.colsum64 != nullptr) && a.cols > kMaxLdsCols / (acc64 ? 2 : 1)) {
    colsum_direct = acc64 ? static_cast<void*>(a.colsum64) : static_cast<void*>(a.colsum);  // separate pass
    a.colsum = nullptr;
    a.colsum64 = nullptr;
  }
  const size_t lds = (acc64 ? a.colsum64 != nullptr : a.colsum != nullptr) ? (acc64 ? 8 : 4) * a.cols : 0;
  const dim3 grid((a.rows + kHeadRows - 1) / kHeadRows);
  const bool vec = a.dtype == DT_BF16 && a.cols % 8 == 0 && a.ld % 8 == 0 && (a.dh == nullptr || a.ld_dh % 8 == 0) &&
                   (a.probs == nullptr || a.ld_probs % 8 == 0) && a.idx_ld % 2 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.logits) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.dh) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.probs) & 15) == 0;
  const dim3 grid16((a.rows + kBf16HeadRows - 1) / kBf16HeadRows);
  constexpr int kW = 16;         // waves per bf16 block: one row each
  const size_t ldsw = kW * lds;  // the bf16 kernel keeps one partial row per wave (up to 128 KiB)
  hipError_t le = hipSuccess;
  if (!vec || a.cols > 2048) a.cs_ws = nullptr;  // (the general kernel: float atomics)
  // the lean kernel: the trainer's logits stage (no probabilities, dZ stored, at most the logits'
  // pre-head dropout), row width a multiple of 512
  const EpiSpec& ep = a.epi;
  const int nch = a.cols / 512;
  if (vec && a.probs == nullptr && a.dh != nullptr && a.cols % 512 == 0 && nch >= 1 && nch <= 4 &&
      nch != 3 && ep.act == ACT_NONE && !ep.drop_post && !ep.drop_all && a.labels != nullptr &&
      (a.out8 == nullptr || xent_head_out8_ok(a))) {
    const bool cs = a.colsum != nullptr, o8 = a.out8 != nullptr, dr = ep.drop_pre != 0;
    return launch_xent_lean(a, nch, cs, o8, dr, grid16, cs ? ldsw : 0, s);
  }
  if (vec && a.cols <= 512) le = launch_xent_bf16<1, kW>(a, grid16, ldsw, s);
  else if (vec && a.cols <= 1024) le = launch_xent_bf16<2, kW>(a, grid16, ldsw, s);
  else if (vec && a.cols <= 2048) le = launch_xent_bf16<4, kW>(a, grid16, ldsw, s);
  else {
    PZ_DISPATCH_FLOAT(a.dtype, T, {
      using F = typename MathOf<T>::type;
      hipLaunchKernelGGL((xent_head_kernel<T, F>), grid, dim3(256), lds, s, a);
    });
  }
  if (le != hipSuccess) return le;
  if (colsum_direct != nullptr && a.dh != nullptr) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return colsum(a.dh, a.dtype, colsum_direct, acc64 ? DT_F64 : DT_F32, a.rows, a.cols, s);  // ld_dh == cols
  }
  return hipGetLastError();
}

hipError_t mse_head(const MseArgs& in, hipStream_t s) {
  if (in.rows <= 0 || in.cols <= 0) return hipSuccess;
  MseArgs a = in;
  void* colsum_direct = nullptr;
  const bool acc64 = a.dtype == DT_F64;
  if ((a.colsum != nullptr || a.colsum64 != nullptr) && a.cols > kMaxLdsCols / (acc64 ? 2 : 1)) {
    colsum_direct = acc64 ? static_cast<void*>(a.colsum64) : static_cast<void*>(a.colsum);
    a.colsum = nullptr;
    a.colsum64 = nullptr;
  }
  const size_t lds = (acc64 ? a.colsum64 != nullptr : a.colsum != nullptr) ? (acc64 ? 8 : 4) * a.cols : 0;
  PZ_DISPATCH_FLOAT(a.dtype, T, {
    using F = typename MathOf<T>::type;
    hipLaunchKernelGGL((mse_head_kernel<T, F>), dim3((a.rows + kHeadRows - 1) / kHeadRows), dim3(256), lds, s, a);
  });
  if (colsum_direct != nullptr && a.dh != nullptr) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return colsum(a.dh, a.dtype, colsum_direct, acc64 ? DT_F64 : DT_F32, a.rows, a.cols, s);
  }
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

int colsum_parts(int rows) { return (rows + kColsumRows - 1) / kColsumRows; }

hipError_t colsum(const void* x, int dtype, void* out, int out_dtype, int rows, int cols, hipStream_t s, void* ws) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  const int rpb = kColsumRows;
  const int parts = colsum_parts(rows);
  dim3 grid((cols + 63) / 64, parts);
  PZ_DISPATCH_FLOAT(dtype, T, {
    if (out_dtype == DT_F64) {
      hipLaunchKernelGGL((colsum_kernel<T, double>), grid, dim3(256), 0, s, static_cast<const T*>(x),
                         static_cast<double*>(out), rows, cols, rpb, static_cast<double*>(ws));
      if (ws != nullptr)
        hipLaunchKernelGGL(colsum_fold_kernel<double>, dim3((cols + 255) / 256), dim3(256), 0, s,
                           static_cast<const double*>(ws), static_cast<double*>(out), parts, cols);
    } else {
      hipLaunchKernelGGL((colsum_kernel<T, float>), grid, dim3(256), 0, s, static_cast<const T*>(x),
                         static_cast<float*>(out), rows, cols, rpb, static_cast<float*>(ws));
      if (ws != nullptr)
        hipLaunchKernelGGL(colsum_fold_kernel<float>, dim3((cols + 255) / 256), dim3(256), 0, s,
                           static_cast<const float*>(ws), static_cast<float*>(out), parts, cols);
    }
  });
  return hipGetLastError();
}

hipError_t gather_rows(const GatherArgs& a, hipStream_t s) {
  if (a.rows <= 0) return hipSuccess;
  const bool vec = a.out_dtype == DT_BF16 && (a.data_dtype == DT_F32 || a.data_dtype == DT_BF16) && a.cols % 8 == 0 &&
                   a.ld_data % 8 == 0 && a.ld_out % 8 == 0 && (reinterpret_cast<uintptr_t>(a.data) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.out) & 15) == 0 &&
                   (a.out8 == nullptr || ((a.ld_data8 | a.ld_out8) % 8 == 0 &&
                                          ((reinterpret_cast<uintptr_t>(a.data8) | reinterpret_cast<uintptr_t>(a.out8)) & 7) == 0));
  if (vec) {
    if (a.data_dtype == DT_F32)
      hipLaunchKernelGGL(gather_rows_vec_kernel<float>, dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(gather_rows_vec_kernel<uint16_t>, dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  PZ_DISPATCH_FLOAT(a.data_dtype, Tin, PZ_DISPATCH_FLOAT(a.out_dtype, Tout, {
    hipLaunchKernelGGL((gather_rows_kernel<Tin, Tout>), dim3(a.rows), dim3(256), 0, s, a);
  }));
  return hipGetLastError();
}

}  // namespace pz
