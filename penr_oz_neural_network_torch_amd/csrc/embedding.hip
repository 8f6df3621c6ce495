// N5 — embedding lookup (reference neural_net_model.py:67-68, `weights[input.long()]`) and its
// backward (autograd's index_put_ with accumulate=True, i.e. a scatter-add into the table).
//
// Token ids may arrive as int64 or as floats (the reference feeds ids as float tensors and
// calls .long(); the engine keeps gathered minibatches in fp32) — truncation toward zero like
// `.long()` happens in-kernel, so no separate cast pass.
// Forward: one wave per looked-up row, gathered and cast to the compute dtype in one pass.
// Backward: f32 atomics, one contiguous row segment per wave instruction (the shape the
// MI355X atomic unit serves at full rate, MI355X_MICROARCH § Global float atomics); tables are
// small (vocab x emb) so the atomic byte budget is tiny next to the GEMMs.
#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

template <typename T> PZ_DEV double le(const T* p, int64_t i) { return static_cast<double>(p[i]); }
template <> PZ_DEV double le<uint16_t>(const uint16_t* p, int64_t i) { return bf2f(p[i]); }
template <typename T> PZ_DEV void se(T* p, int64_t i, double v) { p[i] = static_cast<T>(v); }
template <> PZ_DEV void se<uint16_t>(uint16_t* p, int64_t i, double v) { p[i] = f2bf(static_cast<float>(v)); }
template <typename I> PZ_DEV int64_t id_of(const I* p, int64_t i) { return static_cast<int64_t>(p[i]); }

// Python indexing semantics of `weights[ids]`: negative ids count from the end. The host
// (ops/functional.py, engine) rejects ids outside [-vocab, vocab) with IndexError before a launch;
// this guard only guarantees that a bad id can never address memory outside the table (the row
// reads as zeros / its gradient is dropped).
PZ_DEV int64_t wrap_id(int64_t id, int64_t vocab) { return id < 0 ? id + vocab : id; }

template <typename Tt, typename To, typename I>
__global__ void __launch_bounds__(256) embedding_fwd_kernel(const Tt* __restrict__ table, const I* __restrict__ idx,
                                                            int64_t n_idx, int dim, int64_t vocab, To* __restrict__ out) {
  const int64_t row = blockIdx.x * int64_t(4) + (threadIdx.x >> 6);
  if (row >= n_idx) return;
  const int64_t id = wrap_id(id_of<I>(idx, row), vocab);
  const bool ok = id >= 0 && id < vocab;
  const int64_t src = (ok ? id : 0) * dim;
  for (int c = threadIdx.x & 63; c < dim; c += 64) se<To>(out, row * dim + c, ok ? le<Tt>(table, src + c) : 0.0);
}

template <typename Tg, typename Tt, typename I>
__global__ void __launch_bounds__(256) embedding_bwd_kernel(const Tg* __restrict__ dout, const I* __restrict__ idx,
                                                            int64_t n_idx, int dim, int64_t vocab, Tt* __restrict__ dtable) {
  const int64_t row = blockIdx.x * int64_t(4) + (threadIdx.x >> 6);
  if (row >= n_idx) return;
  const int64_t id = wrap_id(id_of<I>(idx, row), vocab);
  if (id < 0 || id >= vocab) return;
  const int64_t dst = id * dim;
  for (int c = threadIdx.x & 63; c < dim; c += 64)
    atomicAdd(dtable + dst + c, static_cast<Tt>(le<Tg>(dout, row * dim + c)));
}

}  // namespace

#define PZ_EMB_DISPATCH(dt, T, ...)                           \
  switch (dt) {                                               \
    case DT_BF16: { using T = uint16_t; __VA_ARGS__; break; } \
    case DT_F32: { using T = float; __VA_ARGS__; break; }     \
    case DT_F64: { using T = double; __VA_ARGS__; break; }    \
    default: return hipErrorInvalidValue;                     \
  }
#define PZ_IDX_DISPATCH(dt, I, ...)                           \
  switch (dt) {                                               \
    case IDX_I64: { using I = int64_t; __VA_ARGS__; break; }  \
    case IDX_F32: { using I = float; __VA_ARGS__; break; }    \
    case IDX_F64: { using I = double; __VA_ARGS__; break; }   \
    default: return hipErrorInvalidValue;                     \
  }

hipError_t embedding_fwd(const void* table, int table_dtype, int64_t vocab, const void* idx, int idx_dtype, int64_t n_idx,
                         int dim, void* out, int out_dtype, hipStream_t s) {
  if (n_idx <= 0) return hipSuccess;
  const dim3 grid(static_cast<unsigned>((n_idx + 3) / 4));
  PZ_IDX_DISPATCH(idx_dtype, I, PZ_EMB_DISPATCH(table_dtype, Tt, PZ_EMB_DISPATCH(out_dtype, To, {
    hipLaunchKernelGGL((embedding_fwd_kernel<Tt, To, I>), grid, dim3(256), 0, s, static_cast<const Tt*>(table),
                       static_cast<const I*>(idx), n_idx, dim, vocab, static_cast<To*>(out));
  })));
  return hipGetLastError();
}

hipError_t embedding_bwd(const void* dout, int dout_dtype, const void* idx, int idx_dtype, int64_t n_idx, int dim,
                         int64_t vocab, void* dtable, int dtable_dtype, hipStream_t s) {
  if (n_idx <= 0) return hipSuccess;
  const dim3 grid(static_cast<unsigned>((n_idx + 3) / 4));
  PZ_IDX_DISPATCH(idx_dtype, I, PZ_EMB_DISPATCH(dout_dtype, Tg, {
    if (dtable_dtype == DT_F64)
      hipLaunchKernelGGL((embedding_bwd_kernel<Tg, double, I>), grid, dim3(256), 0, s, static_cast<const Tg*>(dout),
                         static_cast<const I*>(idx), n_idx, dim, vocab, static_cast<double*>(dtable));
    else if (dtable_dtype == DT_F32)
      hipLaunchKernelGGL((embedding_bwd_kernel<Tg, float, I>), grid, dim3(256), 0, s, static_cast<const Tg*>(dout),
                         static_cast<const I*>(idx), n_idx, dim, vocab, static_cast<float*>(dtable));
    else
      return hipErrorInvalidValue;
  }));
  return hipGetLastError();
}

}  // namespace pz
