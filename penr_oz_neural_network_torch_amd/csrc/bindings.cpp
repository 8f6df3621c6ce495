// torch.ops.pz — registers every native kernel of the framework as a PyTorch operator.
//
// Device ops are registered for the CUDA dispatch key (which is the HIP device on ROCm builds of
// PyTorch) and launch on PyTorch's current HIP stream, so they order correctly with the caching
// allocator, RCCL collectives issued through torch.distributed, and hipGraph capture.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <map>
#include <mutex>

#include <torch/library.h>

#include <cstdio>
#include <cstring>
#include <tuple>
#include <vector>

#include "json_format.h"
#include "pz_kernels.h"

namespace {

using at::Tensor;
using c10::optional;

#define PZ_HIP_CHECK(expr)                                                                   \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    TORCH_CHECK(_e == hipSuccess, "pz: HIP error ", hipGetErrorString(_e), " in " #expr);    \
  } while (0)

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

int dt_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return pz::DT_BF16;
    case at::kFloat: return pz::DT_F32;
    case at::kDouble: return pz::DT_F64;
    case at::kFloat8_e4m3fn: return pz::DT_FP8;
    case at::kFloat8_e5m2: return pz::DT_FP8;  // gradient operands (GemmArgs::a_fmt = 1)
    default: TORCH_CHECK(false, "pz: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void check_dev(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "pz: ", name, " must be a GPU tensor");
}

template <typename T = void>
T* ptr_or_null(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? static_cast<T*>(t->data_ptr()) : nullptr;
}

// device epoch counter of graph-replayed steps: one int32 on the GPU
const int* epoch_counter(const optional<Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "pz: epoch counter must be a GPU int32");
  return t->data_ptr<int>();
}

pz::EpiSpec make_epi(at::IntArrayRef ei, at::ArrayRef<double> ef) {
  pz::EpiSpec e{};
  e.act = pz::ACT_NONE;
  e.scale = 1.f;
  e.inv_scale = 1.f;
  e.scale64 = 1.0;
  e.inv_scale64 = 1.0;
  if (ei.size() >= 7) {  // [act, drop_pre, drop_post, key_pre, key_post, thresh16, drop_all]
    e.act = static_cast<int>(ei[0]);
    e.drop_pre = ei[1] != 0;
    e.drop_post = ei[2] != 0;
    e.key_pre = static_cast<uint32_t>(ei[3]);
    e.key_post = static_cast<uint32_t>(ei[4]);
    e.thresh16 = static_cast<uint32_t>(ei[5]);
    e.drop_all = static_cast<int>(ei[6]);
  }
  // [7]: device address of an int32 epoch counter (graph-captured steps), 0 = keys are final.
  // Internal API: the trainer passes counter.data_ptr() of a tensor it owns for the graph's life.
  if (ei.size() >= 8 && ei[7] != 0) e.epoch_ptr = reinterpret_cast<const int*>(static_cast<uintptr_t>(ei[7]));
  if (ef.size() >= 2) {
    e.scale = static_cast<float>(ef[0]);
    e.inv_scale = static_cast<float>(ef[1]);
    e.scale64 = ef[0];
    e.inv_scale64 = ef[1];
  }
  return e;
}


// head accumulators (loss slots, bias-gradient column sums): fp32, or fp64 for fp64 models
template <typename Args>
void head_accumulators(Args& a, const optional<Tensor>& loss, const optional<Tensor>& colsum, bool f64,
                       const char* what) {
  for (const optional<Tensor>* t : {&loss, &colsum})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->scalar_type() == (f64 ? at::kDouble : at::kFloat), what,
                  ": loss / colsum accumulators must be ", f64 ? "fp64 for fp64 data" : "fp32");
  if (f64) {
    a.loss64 = ptr_or_null<double>(loss);
    a.colsum64 = ptr_or_null<double>(colsum);
  } else {
    a.loss = ptr_or_null<float>(loss);
    a.colsum = ptr_or_null<float>(colsum);
  }
  a.loss_slots = (loss.has_value() && loss->defined()) ? static_cast<int>(loss->numel()) : 1;
}

// ------------------------------------------------------------------------------------ GEMM
pz::GemmArgs gemm_args(const Tensor& A, bool a_kc, const Tensor& B, bool b_kc, const Tensor& C,
                       const optional<Tensor>& bias, const optional<Tensor>& aux, const optional<Tensor>& colsum,
                       int64_t epi_mode, at::IntArrayRef epi_i, at::ArrayRef<double> epi_f, double alpha,
                       bool accumulate, int64_t M, int64_t N, int64_t K, int64_t idx_ld, bool force_generic,
                       const optional<Tensor>& mask = c10::nullopt) {
  // (fp8 extras are attached by gemm_fp8_extras below)
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "pz::gemm: 2-D operands expected");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && C.stride(1) == 1, "pz::gemm: unit inner stride expected");
  TORCH_CHECK(A.scalar_type() == B.scalar_type() ||
                  (A.scalar_type() == at::kFloat8_e5m2 && B.scalar_type() == at::kFloat8_e4m3fn) ||
                  (A.scalar_type() == at::kFloat8_e4m3fn && B.scalar_type() == at::kFloat8_e5m2 && !a_kc && !b_kc),
              "pz::gemm: A/B dtype mismatch (mixed fp8: e5m2 A x e4m3 B, or the [K][M] e4m3 x [K][N] e5m2 "
              "weight gradient)");
  TORCH_CHECK(a_kc ? (A.size(0) >= M && A.size(1) >= K) : (A.size(0) >= K && A.size(1) >= M), "pz::gemm: A shape");
  TORCH_CHECK(b_kc ? (B.size(0) >= N && B.size(1) >= K) : (B.size(0) >= K && B.size(1) >= N), "pz::gemm: B shape");
  TORCH_CHECK(C.size(0) >= M && C.size(1) >= N, "pz::gemm: C shape");
  pz::GemmArgs p{};
  p.A = A.data_ptr();
  p.B = B.data_ptr();
  p.C = C.data_ptr();
  p.M = static_cast<int>(M);
  p.N = static_cast<int>(N);
  p.K = static_cast<int>(K);
  p.lda = A.stride(0);
  p.ldb = B.stride(0);
  p.ldc = C.stride(0);
  p.a_kc = a_kc;
  p.b_kc = b_kc;
  p.in_dtype = dt_of(A);
  p.out_dtype = dt_of(C);
  p.a_fmt = A.scalar_type() == at::kFloat8_e5m2 ? 1 : 0;  // fp8 operand formats (gemm_path sees them too)
  p.b_fmt = B.scalar_type() == at::kFloat8_e5m2 ? 1 : 0;
  p.alpha = static_cast<float>(alpha);
  p.accumulate = accumulate;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK((bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kDouble) && bias->is_contiguous() &&
                    bias->numel() >= N, "pz::gemm: bias must be fp32 or fp64 [N]");
    if (bias->scalar_type() == at::kDouble) p.bias64 = bias->data_ptr<double>();
    else p.bias = bias->data_ptr<float>();
  }
  if (aux.has_value() && aux->defined()) {
    TORCH_CHECK(aux->dim() == 2 && aux->stride(1) == 1 && aux->size(0) >= M && aux->size(1) >= N, "pz::gemm: aux");
    p.aux = aux->data_ptr();
    p.ldaux = aux->stride(0);
    p.aux_dtype = dt_of(*aux);
  }
  if (colsum.has_value() && colsum->defined()) {
    TORCH_CHECK((colsum->scalar_type() == at::kFloat || colsum->scalar_type() == at::kDouble) && colsum->numel() >= N,
                "pz::gemm: colsum must be fp32 or fp64 [N]");
    if (colsum->scalar_type() == at::kDouble) p.colsum64 = colsum->data_ptr<double>();
    else p.colsum = colsum->data_ptr<float>();
  }
  p.epi_mode = static_cast<int>(epi_mode);
  p.epi = make_epi(epi_i, epi_f);
  p.idx_ld = idx_ld > 0 ? idx_ld : N;
  p.force_generic = force_generic;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->dim() == 2 && mask->is_contiguous() &&
                    mask->size(0) >= (M + 255) / 256 * 256 && mask->size(1) == (N + 255) / 256 * 32,
                "pz::gemm: mask must be a contiguous uint8 [roundup(M, 256), ceil(N/256)*32] (tile-blocked)");
    p.mask = mask->data_ptr<uint8_t>();
    p.ldmask = mask->stride(0);
  }
  return p;
}

// per-tile split-K tickets: one zeroed device ring per GPU, handed out in chunks (the kernel's
// last arriver resets its tiles' counters, so a chunk is clean again when its launch retires)
int* split_counters(int tiles, const c10::Device& dev) {
  static std::mutex mu;
  static std::map<int, std::pair<at::Tensor, int64_t>> rings;
  constexpr int64_t kCap = 1 << 16;
  std::lock_guard<std::mutex> lock(mu);
  auto& ring = rings[dev.index()];
  if (!ring.first.defined()) ring.first = at::zeros({kCap}, at::TensorOptions().dtype(at::kInt).device(dev));
  TORCH_CHECK(tiles <= kCap, "pz::gemm: too many split-K tiles");
  if (ring.second + tiles > kCap) ring.second = 0;
  int* ptr = ring.first.data_ptr<int>() + ring.second;
  ring.second += tiles;
  return ptr;
}

const float* f32_scalar_ptr(const optional<Tensor>& t, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() >= 1, "pz::gemm: ", what, " must be an fp32 device scalar");
  return t->data_ptr<float>();
}

// a folded fp8 scale update (pz_kernels.h ScaleUpd) riding on another launch
pz::ScaleUpd scale_upd(const optional<Tensor>& amax, const optional<Tensor>& qs, double headroom, double maxval) {
  pz::ScaleUpd su{};
  if (!amax.has_value() || !amax->defined()) return su;
  TORCH_CHECK(qs.has_value() && qs->defined(), "scale update: su_amax needs su_qs");
  TORCH_CHECK(amax->scalar_type() == at::kFloat && qs->scalar_type() == at::kFloat && amax->is_contiguous() &&
                  qs->is_contiguous() && qs->numel() >= 2 * amax->numel() && amax->numel() <= 64,
              "scale update: fp32 amax[n <= 64], qs[2n]");
  su.amax = amax->data_ptr<float>();
  su.qs = qs->data_ptr<float>();
  su.n = static_cast<int>(amax->numel());
  su.headroom = static_cast<float>(headroom);
  su.maxval = static_cast<float>(maxval);
  su.qs_prev = nullptr;
  return su;
}

void gemm_op(const Tensor& A, bool a_kc, const Tensor& B, bool b_kc, const Tensor& C, const optional<Tensor>& bias,
             const optional<Tensor>& aux, const optional<Tensor>& colsum, int64_t epi_mode, at::IntArrayRef epi_i,
             at::ArrayRef<double> epi_f, double alpha, bool accumulate, int64_t M, int64_t N, int64_t K, int64_t idx_ld,
             bool force_generic, const optional<Tensor>& mask, const optional<Tensor>& scale_a,
             const optional<Tensor>& scale_b, const optional<Tensor>& out8, const optional<Tensor>& out8_qscale,
             const optional<Tensor>& amax, int64_t flags) {
  check_dev(A, "A");
  auto p = gemm_args(A, a_kc, B, b_kc, C, bias, aux, colsum, epi_mode, epi_i, epi_f, alpha, accumulate, M, N, K, idx_ld,
                     force_generic, mask);
  p.scale_a = f32_scalar_ptr(scale_a, "scale_a");
  p.scale_b = f32_scalar_ptr(scale_b, "scale_b");
  TORCH_CHECK(p.b_fmt == 0 || (!a_kc && !b_kc), "pz::gemm: an e5m2 B operand needs the M/N-contiguous dW layout");
  if (out8.has_value() && out8->defined()) {
    TORCH_CHECK((out8->scalar_type() == at::kFloat8_e4m3fn || out8->scalar_type() == at::kFloat8_e5m2) &&
                    out8->dim() == 2 && out8->stride(1) == 1 && out8->size(0) >= M && out8->size(1) >= N,
                "pz::gemm: out8 must be float8_e4m3fn (forward) or float8_e5m2 (backward) [M, N]");
    p.out8_fmt = out8->scalar_type() == at::kFloat8_e5m2 ? 1 : 0;
    TORCH_CHECK(p.out8_fmt == (epi_mode == 2 ? 1 : 0), "pz::gemm: out8 is e4m3 for EPI_FWD, e5m2 for EPI_BWD");
    p.out8 = static_cast<uint8_t*>(out8->data_ptr());
    p.ldout8 = out8->stride(0);
    p.out8_qscale = f32_scalar_ptr(out8_qscale, "out8_qscale");
    TORCH_CHECK(p.out8_qscale != nullptr, "pz::gemm: out8 needs out8_qscale");
  }
  if (amax.has_value() && amax->defined()) {
    TORCH_CHECK(amax->scalar_type() == at::kFloat, "pz::gemm: amax must be fp32");
    p.amax = amax->data_ptr<float>();
  }
  TORCH_CHECK((p.out8 == nullptr && p.in_dtype != pz::DT_FP8) || pz::gemm_path(p) == 1,
              "pz::gemm: fp8 operands / outputs need an MFMA-eligible shape");
  // flags bit 1: C is not stored — only the epilogue's side outputs (fp8 copy, ReLU bitmask, bias-
  // gradient column sums) are; the MFMA path's bf16 epilogue implements it
  if (flags & 2) {
    TORCH_CHECK(p.out_dtype == pz::DT_BF16 && pz::gemm_path(p) == 1 && (p.out8 != nullptr || p.mask != nullptr ||
                                                                         p.colsum != nullptr),
                "pz::gemm: store_c=False needs the MFMA path with a bf16 C and a side output");
    p.C = nullptr;
  }
  at::Tensor cs_ws;  // deterministic bias-gradient sums: per-tile partial rows (BM >= 128) + group rows
  if (p.colsum != nullptr && p.out_dtype == pz::DT_BF16 && pz::deterministic()) {
    const int parts = (p.M + 127) / 128, groups = (parts + 63) / 64;
    cs_ws = at::empty({static_cast<int64_t>(parts + groups) * p.N}, A.options().dtype(at::kFloat));
    p.cs_ws = cs_ws.data_ptr<float>();
    p.cs_tickets = split_counters(((p.N + 127) / 128) * (groups + 1), A.device());
  }
  at::Tensor ws;  // split-K / stream-K slabs: from the caching allocator, stream-ordered reuse is safe
  // flags bits 2-3: engine (0 default, 1 tiled gemm_mfma, 2 persistent stream-K; 3, the round-5
  // 4-wave lab loop, is refused: tools/gemm_w4_lab.hip); bits 16-31: the CU budget of the persistent engine (0 = every CU)
  p.engine = static_cast<int>((flags >> 2) & 3);
  p.cus = static_cast<int>((flags >> 16) & 0xFFFF);
  // (engine 0 with a CU budget: the persistent engine wherever it is eligible)
  if ((p.engine >= 2 || (p.engine == 0 && (pz::sk_default() || p.cus > 0))) && pz::sk_eligible(p)) {
    const int64_t sk_floats = pz::sk_ws_floats(&p, 1);
    int* tickets = nullptr;
    if (sk_floats > 0) {
      ws = at::empty({sk_floats}, A.options().dtype(at::kFloat));
      tickets = split_counters(pz::sk_tickets(&p, 1), A.device());
    }
    PZ_HIP_CHECK(pz::gemm_sk(&p, 1, sk_floats > 0 ? ws.data_ptr<float>() : nullptr, tickets, cur_stream(A)));
    return;
  }
  TORCH_CHECK(p.engine < 2, "pz::gemm: the stream-K engine cannot run this GEMM (pz::sk_eligible)");
  // flags bit 0: no split-K (a GEMM that runs concurrently with others: its tile count need not
  // fill the CUs on its own, and it skips the in-launch reduction)
  const int64_t ws_floats = (flags & 1) ? 0 : pz::gemm_split_ws_floats(p);
  if (ws_floats > 0) {
    ws = at::empty({ws_floats}, A.options().dtype(at::kFloat));
    p.split_k = pz::gemm_split(p);
    p.ws = ws.data_ptr<float>();
    p.counters = split_counters(static_cast<int>(((M + 255) / 256) * ((N + 255) / 256)), A.device());
  }
  TORCH_CHECK(p.mask == nullptr || pz::gemm_path(p) == 1, "pz::gemm: a mask epilogue needs an MFMA-eligible shape");
  PZ_HIP_CHECK(pz::gemm(p, cur_stream(A)));
}

// dW GEMM with the optimizer update fused into its epilogue (EPI_OPT): `grad` is the weight's
// gradient view (shape / leading dimension only — it is NOT written); params / exp_avg /
// exp_avg_sq / shadow are views of the same [in, out] shape; stats = this weight's 4 doubles
pz::GemmArgs update_args(const Tensor& A, bool a_kc, const Tensor& B, bool b_kc, const Tensor& grad, int64_t M, int64_t N,
                         int64_t K, double alpha, const Tensor& params, const optional<Tensor>& exp_avg,
                         const optional<Tensor>& exp_avg_sq, const optional<Tensor>& shadow,
                         const optional<Tensor>& stats, const optional<Tensor>& amax, bool adam, double lr, double beta1,
                         double beta2, double eps, double bias_c1, double bias_c2_sqrt, double grad_scale, double l2,
                         const optional<Tensor>& hp, const optional<Tensor>& epoch, int64_t stats_every) {
  check_dev(A, "A");
  auto p = gemm_args(A, a_kc, B, b_kc, grad, c10::nullopt, c10::nullopt, c10::nullopt, pz::EPI_OPT, {}, {}, alpha, false,
                     M, N, K, 0, false, c10::nullopt);
  TORCH_CHECK(grad.scalar_type() == at::kFloat, "pz::gemm_update: the gradient view must be fp32");
  auto same = [&](const Tensor& t, at::ScalarType dt, const char* what) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.dim() == 2 && t.size(0) >= M && t.size(1) >= N &&
                    t.stride(1) == 1 && t.stride(0) == grad.stride(0),
                "pz::gemm_update: ", what, " must match the gradient view's layout");
  };
  same(params, at::kFloat, "params");
  pz::GemmOpt& o = p.opt;
  o.params = params.data_ptr<float>();
  o.adam = adam;
  if (adam) {
    TORCH_CHECK(exp_avg.has_value() && exp_avg_sq.has_value(), "pz::gemm_update: Adam needs moment buffers");
    same(*exp_avg, at::kFloat, "exp_avg");
    same(*exp_avg_sq, at::kFloat, "exp_avg_sq");
    o.exp_avg = exp_avg->data_ptr<float>();
    o.exp_avg_sq = exp_avg_sq->data_ptr<float>();
  }
  if (shadow.has_value() && shadow->defined()) {
    same(*shadow, shadow->scalar_type(), "shadow");
    TORCH_CHECK(shadow->scalar_type() == at::kBFloat16 || shadow->scalar_type() == at::kFloat,
                "pz::gemm_update: bf16 or fp32 shadow");
    o.shadow = shadow->data_ptr();
    o.shadow_dtype = dt_of(*shadow);
  }
  if (stats.has_value() && stats->defined()) {
    TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->numel() >= 4 && stats->is_contiguous(),
                "pz::gemm_update: stats must be 4 contiguous doubles");
    o.stats = stats->data_ptr<double>();
  }
  if (amax.has_value() && amax->defined()) {
    TORCH_CHECK(amax->scalar_type() == at::kFloat, "pz::gemm_update: amax must be fp32");
    o.amax = amax->data_ptr<float>();
  }
  o.lr = static_cast<float>(lr);
  o.beta1 = static_cast<float>(beta1);
  o.beta2 = static_cast<float>(beta2);
  o.eps = static_cast<float>(eps);
  o.bias_c1 = static_cast<float>(bias_c1);
  o.bias_c2_sqrt = static_cast<float>(bias_c2_sqrt);
  o.grad_scale = static_cast<float>(grad_scale);
  o.l2x2 = static_cast<float>(2.0 * l2);
  o.stats_every = static_cast<int>(stats_every);
  if (epoch.has_value() && epoch->defined()) o.epoch_ptr = epoch_counter(epoch);
  if (stats_every > 1) TORCH_CHECK(o.epoch_ptr != nullptr, "pz::gemm_update: stats_every > 1 needs the epoch counter");
  if (hp.has_value() && hp->defined()) {
    TORCH_CHECK(hp->scalar_type() == at::kDouble && hp->is_contiguous() && hp->is_cuda(),
                "pz::gemm_update: hp table (fp64)");
    TORCH_CHECK(o.epoch_ptr != nullptr, "pz::gemm_update: an hp table needs the epoch counter");
    o.hp = hp->data_ptr<double>();
  }
  TORCH_CHECK(pz::gemm_path(p) == 1, "pz::gemm_update: needs an MFMA-eligible bf16 shape (16-B aligned state)");
  return p;
}

void gemm_update_op(const Tensor& A, bool a_kc, const Tensor& B, bool b_kc, const Tensor& grad, int64_t M, int64_t N,
                    int64_t K, double alpha, const Tensor& params, const optional<Tensor>& exp_avg,
                    const optional<Tensor>& exp_avg_sq, const optional<Tensor>& shadow, const optional<Tensor>& stats,
                    const optional<Tensor>& amax, bool adam, double lr, double beta1, double beta2, double eps,
                    double bias_c1, double bias_c2_sqrt, double grad_scale, double l2, const optional<Tensor>& hp,
                    const optional<Tensor>& epoch, int64_t stats_every) {
  auto p = update_args(A, a_kc, B, b_kc, grad, M, N, K, alpha, params, exp_avg, exp_avg_sq, shadow, stats, amax, adam, lr,
                       beta1, beta2, eps, bias_c1, bias_c2_sqrt, grad_scale, l2, hp, epoch, stats_every);
  at::Tensor ws;
  const int64_t ws_floats = pz::gemm_split_ws_floats(p);
  if (ws_floats > 0) {
    ws = at::empty({ws_floats}, A.options().dtype(at::kFloat));
    p.split_k = pz::gemm_split(p);
    p.ws = ws.data_ptr<float>();
    p.counters = split_counters(static_cast<int>(((M + 255) / 256) * ((N + 255) / 256)), A.device());
  }
  PZ_HIP_CHECK(pz::gemm(p, cur_stream(A)));
}

// two weight-gradient GEMMs C0 = op(A0)·op(B0), C1 = op(A1)·op(B1) (A, B M/N-contiguous, plain
// stores, one K) in ONE launch (pz::gemm_pair); fp8 operands take their dequantisation scalars
pz::GemmArgs pair_args(const Tensor& A, const Tensor& B, const Tensor& C, int64_t M, int64_t N, int64_t K,
                       const optional<Tensor>& scale_a, const optional<Tensor>& scale_b) {
  auto p = gemm_args(A, false, B, false, C, c10::nullopt, c10::nullopt, c10::nullopt, 0, {}, {}, 1.0, false, M, N, K,
                     0, false);
  p.scale_a = f32_scalar_ptr(scale_a, "scale_a");
  p.scale_b = f32_scalar_ptr(scale_b, "scale_b");
  return p;
}

// engine 2: also 0 unless the persistent stream-K engine takes BOTH problems (pz::sk_eligible:
// e.g. K >= two 64-deep steps) — the trainer's budgeted pair checks this before it asks for it
int64_t gemm_pair_split_op(const Tensor& A0, const Tensor& B0, const Tensor& C0, const Tensor& A1, const Tensor& B1,
                           const Tensor& C1, int64_t M0, int64_t N0, int64_t M1, int64_t N1, int64_t K, int64_t engine) {
  const auto a = pair_args(A0, B0, C0, M0, N0, K, c10::nullopt, c10::nullopt);
  const auto b = pair_args(A1, B1, C1, M1, N1, K, c10::nullopt, c10::nullopt);
  const int split = pz::gemm_pair_split(a, b);
  if (engine >= 2 && !(pz::sk_eligible(a) && pz::sk_eligible(b))) return 0;
  return split;
}

void launch_pair(pz::GemmArgs& a, pz::GemmArgs& b, const Tensor& A0) {
  const int M0 = a.M, N0 = a.N, M1 = b.M, N1 = b.N;
  const int split = pz::gemm_pair_split(a, b);
  TORCH_CHECK(split > 0, "pz::gemm_pair: the two GEMMs cannot share a launch (check gemm_pair_split first)");
  at::Tensor ws0, ws1;  // split-K slabs, one set per GEMM
  a.split_k = b.split_k = split;
  if (split > 1) {
    ws0 = at::empty({(M0 / 256) * (N0 / 256) * split * 65536}, A0.options().dtype(at::kFloat));
    ws1 = at::empty({(M1 / 256) * (N1 / 256) * split * 65536}, A0.options().dtype(at::kFloat));
    a.ws = ws0.data_ptr<float>();
    b.ws = ws1.data_ptr<float>();
    a.counters = split_counters(static_cast<int>((M0 / 256) * (N0 / 256)), A0.device());
    b.counters = split_counters(static_cast<int>((M1 / 256) * (N1 / 256)), A0.device());
  }
  PZ_HIP_CHECK(pz::gemm_pair(a, b, cur_stream(A0)));
}

void gemm_pair_op(const Tensor& A0, const Tensor& B0, const Tensor& C0, const Tensor& A1, const Tensor& B1,
                  const Tensor& C1, int64_t M0, int64_t N0, int64_t M1, int64_t N1, int64_t K,
                  const optional<Tensor>& scale_a0, const optional<Tensor>& scale_b0,
                  const optional<Tensor>& scale_a1, const optional<Tensor>& scale_b1, int64_t flags) {
  check_dev(A0, "A0");
  auto a = pair_args(A0, B0, C0, M0, N0, K, scale_a0, scale_b0);
  auto b = pair_args(A1, B1, C1, M1, N1, K, scale_a1, scale_b1);
  // flags as pz::gemm's: bits 2-3 engine (2 / 3: the two problems as ONE persistent stream-K
  // schedule), bits 16-31 its CU budget
  a.engine = b.engine = static_cast<int>((flags >> 2) & 3);
  a.cus = b.cus = static_cast<int>((flags >> 16) & 0xFFFF);
  if (a.engine >= 2) {
    TORCH_CHECK(pz::sk_eligible(a) && pz::sk_eligible(b), "pz::gemm_pair: the stream-K engine cannot run this pair");
    pz::GemmArgs probs[2] = {a, b};
    const int64_t sk_floats = pz::sk_ws_floats(probs, 2);
    at::Tensor ws;
    int* tickets = nullptr;
    if (sk_floats > 0) {
      ws = at::empty({sk_floats}, A0.options().dtype(at::kFloat));
      tickets = split_counters(pz::sk_tickets(probs, 2), A0.device());
    }
    PZ_HIP_CHECK(pz::gemm_sk(probs, 2, sk_floats > 0 ? ws.data_ptr<float>() : nullptr, tickets, cur_stream(A0)));
    return;
  }
  launch_pair(a, b, A0);
}

int64_t gemm_path_op(const Tensor& A, bool a_kc, const Tensor& B, bool b_kc, const Tensor& C, int64_t M, int64_t N,
                     int64_t K) {
  auto p = gemm_args(A, a_kc, B, b_kc, C, c10::nullopt, c10::nullopt, c10::nullopt, 0, {}, {}, 1.0, false, M, N, K, 0,
                     false, c10::nullopt);
  return pz::gemm_path(p);
}

// ------------------------------------------------------------------------------ elementwise
void stage_fwd_op(const Tensor& x, const Tensor& y, at::IntArrayRef ei, at::ArrayRef<double> ef) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "pz::stage_fwd: contiguous x/y");
  PZ_HIP_CHECK(pz::stage_fwd(x.data_ptr(), dt_of(x), y.data_ptr(), dt_of(y), x.numel(), make_epi(ei, ef), cur_stream(x)));
}

void stage_bwd_op(const Tensor& g, const Tensor& y, const Tensor& dx, at::IntArrayRef ei, at::ArrayRef<double> ef) {
  check_dev(g, "g");
  TORCH_CHECK(g.is_contiguous() && y.is_contiguous() && dx.is_contiguous(), "pz::stage_bwd: contiguous tensors");
  TORCH_CHECK(g.scalar_type() == y.scalar_type() && g.scalar_type() == dx.scalar_type(), "pz::stage_bwd: dtypes");
  PZ_HIP_CHECK(pz::stage_bwd(g.data_ptr(), y.data_ptr(), dx.data_ptr(), dt_of(g), g.numel(), make_epi(ei, ef),
                             cur_stream(g)));
}

void xent_head_op(const Tensor& logits, const Tensor& labels, int64_t rows_valid, const optional<Tensor>& loss,
                  double loss_scale, const optional<Tensor>& dh, double grad_scale, const optional<Tensor>& colsum,
                  const optional<Tensor>& probs, at::IntArrayRef ei, at::ArrayRef<double> ef, int64_t idx_ld,
                  const optional<Tensor>& out8, const optional<Tensor>& out8_qscale, const optional<Tensor>& amax,
                  bool store_dh, const optional<Tensor>& su_amax, const optional<Tensor>& su_qs, double su_headroom,
                  double su_maxval, const optional<Tensor>& su_qs_prev) {
  check_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "pz::xent_head: 2-D logits");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous(), "pz::xent_head: int64 labels");
  pz::XentArgs a{};
  a.logits = logits.data_ptr();
  a.ld = logits.stride(0);
  a.labels = labels.data_ptr<int64_t>();
  a.rows = static_cast<int>(logits.size(0));
  a.rows_valid = static_cast<int>(rows_valid);
  a.cols = static_cast<int>(logits.size(1));
  a.dtype = dt_of(logits);
  head_accumulators(a, loss, colsum, a.dtype == pz::DT_F64, "pz::xent_head");
  at::Tensor cs_ws;  // deterministic bias-gradient sums: 32-row blocks' partial rows + group rows
  if (a.colsum != nullptr && a.dtype == pz::DT_BF16 && pz::deterministic()) {
    const int blocks = (a.rows + 31) / 32, groups = (blocks + 15) / 16;
    cs_ws = at::empty({static_cast<int64_t>(blocks + groups) * a.cols}, logits.options().dtype(at::kFloat));
    a.cs_ws = cs_ws.data_ptr<float>();
    a.cs_tickets = split_counters(groups + 1, logits.device());
  }
  a.loss_scale = loss_scale;
  if (dh.has_value() && dh->defined()) {
    TORCH_CHECK(dh->scalar_type() == logits.scalar_type() && dh->stride(1) == 1, "pz::xent_head: dh");
    a.dh = dh->data_ptr();
    a.ld_dh = dh->stride(0);
  }
  a.grad_scale = grad_scale;
  if (probs.has_value() && probs->defined()) {
    TORCH_CHECK(probs->scalar_type() == logits.scalar_type() && probs->stride(1) == 1, "pz::xent_head: probs");
    a.probs = probs->data_ptr();
    a.ld_probs = probs->stride(0);
  }
  a.epi = make_epi(ei, ef);
  a.idx_ld = idx_ld > 0 ? idx_ld : a.cols;
  if (out8.has_value() && out8->defined()) {
    TORCH_CHECK(out8->scalar_type() == at::kFloat8_e5m2 && out8->dim() == 2 && out8->stride(1) == 1 &&
                    out8->size(0) >= a.rows && out8->size(1) >= a.cols,
                "pz::xent_head: out8 must be float8_e5m2 [rows, cols]");
    a.out8 = static_cast<uint8_t*>(out8->data_ptr());
    a.ld_out8 = out8->stride(0);
    a.out8_qscale = f32_scalar_ptr(out8_qscale, "out8_qscale");
    TORCH_CHECK(a.out8_qscale != nullptr, "pz::xent_head: out8 needs out8_qscale");
    if (amax.has_value() && amax->defined()) {
      TORCH_CHECK(amax->scalar_type() == at::kFloat, "pz::xent_head: amax must be fp32");
      a.amax = amax->data_ptr<float>();
    }
  }
  a.skip_dh = store_dh ? 0 : 1;
  a.su = scale_upd(su_amax, su_qs, su_headroom, su_maxval);
  if (su_qs_prev.has_value() && su_qs_prev->defined()) {
    TORCH_CHECK(a.su.n > 0 && su_qs_prev->scalar_type() == at::kFloat && su_qs_prev->is_contiguous() &&
                    su_qs_prev->numel() >= 2 * a.su.n && su_qs_prev->data_ptr<float>() != a.su.qs,
                "pz::xent_head: su_qs_prev: fp32 qs[2n] of the current step, not su_qs itself");
    a.su.qs_prev = su_qs_prev->data_ptr<float>();
  }
  TORCH_CHECK((a.out8 == nullptr && !a.skip_dh) || pz::xent_head_out8_ok(a),
              "pz::xent_head: out8 / store_dh=False need the bf16 fast path (bf16, cols % 8 == 0, <= 2048, aligned)");
  PZ_HIP_CHECK(pz::xent_head(a, cur_stream(logits)));
}

void mse_head_op(const Tensor& y, const Tensor& target, int64_t rows_valid, const optional<Tensor>& loss,
                 double loss_scale, const optional<Tensor>& dh, double grad_scale, const optional<Tensor>& colsum,
                 at::IntArrayRef ei, at::ArrayRef<double> ef, int64_t idx_ld) {
  check_dev(y, "y");
  TORCH_CHECK(y.dim() == 2 && target.dim() == 2 && y.stride(1) == 1 && target.stride(1) == 1, "pz::mse_head: 2-D");
  TORCH_CHECK(y.scalar_type() == target.scalar_type(), "pz::mse_head: dtype mismatch");
  pz::MseArgs a{};
  a.y = y.data_ptr();
  a.ld_y = y.stride(0);
  a.target = target.data_ptr();
  a.ld_t = target.stride(0);
  a.rows = static_cast<int>(y.size(0));
  a.rows_valid = static_cast<int>(rows_valid);
  a.cols = static_cast<int>(y.size(1));
  a.dtype = dt_of(y);
  head_accumulators(a, loss, colsum, a.dtype == pz::DT_F64, "pz::mse_head");
  a.loss_scale = loss_scale;
  if (dh.has_value() && dh->defined()) {
    a.dh = dh->data_ptr();
    a.ld_dh = dh->stride(0);
  }
  a.grad_scale = grad_scale;
  a.epi = make_epi(ei, ef);
  a.idx_ld = idx_ld > 0 ? idx_ld : a.cols;
  PZ_HIP_CHECK(pz::mse_head(a, cur_stream(y)));
}

void softmax_rows_op(const Tensor& x, const Tensor& y) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.scalar_type() == y.scalar_type(), "pz::softmax_rows");
  const int cols = static_cast<int>(x.size(-1));
  const int rows = static_cast<int>(x.numel() / std::max<int64_t>(cols, 1));
  PZ_HIP_CHECK(pz::softmax_rows(x.data_ptr(), y.data_ptr(), dt_of(x), rows, cols, cur_stream(x)));
}

void softmax_bwd_op(const Tensor& g, const Tensor& y, const Tensor& dx) {
  check_dev(g, "g");
  TORCH_CHECK(g.is_contiguous() && y.is_contiguous() && dx.is_contiguous(), "pz::softmax_bwd");
  const int cols = static_cast<int>(y.size(-1));
  const int rows = static_cast<int>(y.numel() / std::max<int64_t>(cols, 1));
  PZ_HIP_CHECK(pz::softmax_bwd(g.data_ptr(), y.data_ptr(), dx.data_ptr(), dt_of(y), rows, cols, cur_stream(g)));
}

void colsum_op(const Tensor& x, const Tensor& out) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && (out.scalar_type() == at::kFloat || out.scalar_type() == at::kDouble),
              "pz::colsum: fp32 or fp64 output");
  const int cols = static_cast<int>(x.size(-1));
  const int rows = static_cast<int>(x.numel() / std::max<int64_t>(cols, 1));
  at::Tensor ws;  // deterministic: per-block partial rows folded in block order (no float atomics)
  if (pz::deterministic() && rows > 0 && cols > 0)
    ws = at::empty({static_cast<int64_t>(pz::colsum_parts(rows)) * cols}, out.options());
  PZ_HIP_CHECK(pz::colsum(x.data_ptr(), dt_of(x), out.data_ptr(), dt_of(out), rows, cols, cur_stream(x),
                          ws.defined() ? ws.data_ptr() : nullptr));
}

void gather_rows_op(const Tensor& data, const optional<Tensor>& indices, int64_t seed_lo, int64_t seed_hi,
                    const Tensor& out, int64_t rows_valid, const optional<Tensor>& labels_in,
                    const optional<Tensor>& labels_out, const optional<Tensor>& picked,
                    const optional<Tensor>& epoch, const optional<Tensor>& data8, const optional<Tensor>& out8,
                    const optional<Tensor>& su_amax, const optional<Tensor>& su_qs, double su_headroom,
                    double su_maxval) {
  check_dev(data, "data");
  TORCH_CHECK(data.dim() == 2 && out.dim() == 2 && data.stride(1) == 1 && out.stride(1) == 1, "pz::gather_rows: 2-D");
  TORCH_CHECK(out.size(1) == data.size(1), "pz::gather_rows: width mismatch");
  pz::GatherArgs a{};
  a.data = data.data_ptr();
  a.ld_data = data.stride(0);
  a.data_dtype = dt_of(data);
  a.n_data = data.size(0);
  a.indices = ptr_or_null<const int64_t>(indices);
  a.seed_lo = static_cast<uint32_t>(seed_lo);
  a.seed_hi = static_cast<uint32_t>(seed_hi);
  a.out = out.data_ptr();
  a.ld_out = out.stride(0);
  a.out_dtype = dt_of(out);
  a.rows = static_cast<int>(out.size(0));
  a.rows_valid = static_cast<int>(rows_valid);
  a.cols = static_cast<int>(out.size(1));
  a.labels_in = ptr_or_null<const int64_t>(labels_in);
  a.labels_out = ptr_or_null<int64_t>(labels_out);
  a.picked = ptr_or_null<int64_t>(picked);
  a.epoch_ptr = epoch_counter(epoch);
  if (out8.has_value() && out8->defined()) {
    TORCH_CHECK(data8.has_value() && data8->defined(), "pz::gather_rows: out8 needs data8");
    const Tensor& d8 = *data8;
    const Tensor& o8 = *out8;
    TORCH_CHECK(d8.element_size() == 1 && o8.element_size() == 1 && d8.dim() == 2 && o8.dim() == 2 &&
                    d8.stride(1) == 1 && o8.stride(1) == 1 && d8.size(0) == data.size(0) &&
                    d8.size(1) == data.size(1) && o8.size(0) == out.size(0) && o8.size(1) == out.size(1),
                "pz::gather_rows: data8 [n_data, cols] / out8 [rows, cols] 1-byte tables");
    a.data8 = static_cast<const uint8_t*>(d8.data_ptr());
    a.ld_data8 = d8.stride(0);
    a.out8 = static_cast<uint8_t*>(o8.data_ptr());
    a.ld_out8 = o8.stride(0);
  }
  a.su = scale_upd(su_amax, su_qs, su_headroom, su_maxval);
  TORCH_CHECK(a.su.n == 0 || a.rows > 0, "pz::gather_rows: a folded scale update needs a launch");
  PZ_HIP_CHECK(pz::gather_rows(a, cur_stream(data)));
}

// ------------------------------------------------------------------------------- optimizer
Tensor pack_segments_op(at::IntArrayRef offsets, at::IntArrayRef numels, at::IntArrayRef is_weight,
                        at::IntArrayRef stat_slot, at::ArrayRef<optional<Tensor>> shadows,
                        at::ArrayRef<optional<Tensor>> grads16, at::IntArrayRef zero_grad,
                        at::ArrayRef<optional<Tensor>> amax, at::ArrayRef<optional<Tensor>> w8,
                        at::ArrayRef<optional<Tensor>> w8_amax_prev, at::ArrayRef<optional<Tensor>> w8_qs) {
  const size_t n = offsets.size();
  TORCH_CHECK(numels.size() == n && is_weight.size() == n && stat_slot.size() == n && shadows.size() == n &&
                  (grads16.empty() || grads16.size() == n) && (zero_grad.empty() || zero_grad.size() == n) &&
                  (amax.empty() || amax.size() == n) && (w8.empty() || w8.size() == n) &&
                  w8_amax_prev.size() == w8.size() && w8_qs.size() == w8.size(),
              "pz::pack_segments: length mismatch");
  Tensor out = at::empty({static_cast<int64_t>(n * sizeof(pz::OptSegment))}, at::TensorOptions().dtype(at::kByte));
  auto* segs = reinterpret_cast<pz::OptSegment*>(out.data_ptr<uint8_t>());
  for (size_t i = 0; i < n; ++i) {
    pz::OptSegment s{};
    s.offset = offsets[i];
    s.numel = numels[i];
    s.is_weight = static_cast<int>(is_weight[i]);
    s.stat_slot = static_cast<int>(stat_slot[i]);
    s.zero_grad = zero_grad.empty() ? 0 : static_cast<int>(zero_grad[i]);
    const auto& sh = shadows[i];
    if (sh.has_value() && sh->defined()) {
      TORCH_CHECK(sh->is_contiguous() && sh->numel() == numels[i], "pz::pack_segments: shadow shape");
      s.shadow = sh->data_ptr();
      s.shadow_dtype = dt_of(*sh);
    }
    if (!grads16.empty() && grads16[i].has_value() && grads16[i]->defined()) {
      const Tensor& g = *grads16[i];
      TORCH_CHECK(g.is_contiguous() && g.numel() == numels[i] && g.scalar_type() == at::kBFloat16,
                  "pz::pack_segments: bf16 gradient shape");
      s.grad16 = reinterpret_cast<const uint16_t*>(g.data_ptr());
    }
    if (!amax.empty() && amax[i].has_value() && amax[i]->defined()) {
      TORCH_CHECK(amax[i]->scalar_type() == at::kFloat && amax[i]->numel() >= 1, "pz::pack_segments: fp32 amax");
      s.amax = amax[i]->data_ptr<float>();
    }
    if (!w8.empty() && w8[i].has_value() && w8[i]->defined()) {
      const Tensor& q = *w8[i];
      TORCH_CHECK(q.is_contiguous() && q.numel() == numels[i] && q.element_size() == 1 &&
                      q.scalar_type() == at::kFloat8_e4m3fn,
                  "pz::pack_segments: e4m3 weight copy shape");
      TORCH_CHECK(w8_amax_prev[i].has_value() && w8_amax_prev[i]->scalar_type() == at::kFloat &&
                      w8_qs[i].has_value() && w8_qs[i]->scalar_type() == at::kFloat && w8_qs[i]->numel() >= 2,
                  "pz::pack_segments: e4m3 copy needs fp32 amax_prev and {q, 1/q}");
      s.w8 = reinterpret_cast<uint8_t*>(q.data_ptr());
      s.w8_amax_prev = w8_amax_prev[i]->data_ptr<float>();
      s.w8_qs = w8_qs[i]->data_ptr<float>();
    }
    std::memcpy(segs + i, &s, sizeof(s));
  }
  return out;
}

void optimizer_step_op(const Tensor& params, const Tensor& grads, const optional<Tensor>& exp_avg,
                       const optional<Tensor>& exp_avg_sq, const Tensor& segments, const Tensor& block_seg,
                       int64_t num_segments, int64_t total_blocks, bool adam, double lr, double beta1, double beta2,
                       double eps, double bias_c1, double bias_c2_sqrt, double grad_scale, double l2,
                       const optional<Tensor>& stats, const optional<Tensor>& hp, const optional<Tensor>& epoch,
                       int64_t stats_every, int64_t max_grid) {
  check_dev(params, "params");
  const auto rt = params.scalar_type();
  TORCH_CHECK((rt == at::kFloat || rt == at::kDouble) && grads.scalar_type() == rt,
              "pz::optimizer_step: fp32 or fp64 master with gradients of the same dtype");
  for (const optional<Tensor>* t : {&exp_avg, &exp_avg_sq})
    if (t->has_value() && (*t)->defined())
      TORCH_CHECK((*t)->scalar_type() == rt, "pz::optimizer_step: Adam moments must match the master dtype");
  pz::OptArgs a{};
  a.real = rt == at::kDouble ? pz::DT_F64 : pz::DT_F32;
  a.params = params.data_ptr();
  a.grads = grads.data_ptr();
  a.exp_avg = ptr_or_null<void>(exp_avg);
  a.exp_avg_sq = ptr_or_null<void>(exp_avg_sq);
  TORCH_CHECK(!adam || (a.exp_avg && a.exp_avg_sq), "pz::optimizer_step: Adam needs moment buffers");
  a.segments = reinterpret_cast<const pz::OptSegment*>(segments.data_ptr());
  a.num_segments = static_cast<int>(num_segments);
  a.block_seg = block_seg.data_ptr<int64_t>();
  a.total_blocks = static_cast<int>(total_blocks);
  a.adam = adam;
  a.lr = lr;
  a.beta1 = beta1;
  a.beta2 = beta2;
  a.eps = eps;
  a.bias_c1 = bias_c1;
  a.bias_c2_sqrt = bias_c2_sqrt;
  a.grad_scale = grad_scale;
  a.l2_lambda = l2;
  a.stats = ptr_or_null<double>(stats);
  a.stats_every = static_cast<int>(stats_every);
  a.max_grid = static_cast<int>(max_grid);
  if (stats_every > 1) TORCH_CHECK(epoch.has_value() && epoch->defined(), "pz::optimizer_step: stats_every > 1 needs the epoch counter");
  if (epoch.has_value() && epoch->defined()) a.epoch_ptr = epoch_counter(epoch);
  if (hp.has_value() && hp->defined()) {
    TORCH_CHECK(hp->scalar_type() == at::kDouble && hp->is_contiguous() && hp->is_cuda(),
                "pz::optimizer_step: hp table (fp64)");
    TORCH_CHECK(epoch.has_value(), "pz::optimizer_step: an hp table needs the epoch counter");
    a.hp = hp->data_ptr<double>();
    a.epoch_ptr = epoch_counter(epoch);
  }
  PZ_HIP_CHECK(pz::optimizer_step(a, cur_stream(params)));
}

void segment_stats_op(const Tensor& params, const Tensor& segments, const Tensor& block_seg, int64_t num_segments,
                      int64_t total_blocks, const Tensor& stats) {
  check_dev(params, "params");
  TORCH_CHECK(params.scalar_type() == at::kFloat || params.scalar_type() == at::kDouble, "pz::segment_stats: dtype");
  PZ_HIP_CHECK(pz::segment_stats(params.data_ptr(), params.scalar_type() == at::kDouble ? pz::DT_F64 : pz::DT_F32,
                                 reinterpret_cast<const pz::OptSegment*>(segments.data_ptr()),
                                 block_seg.data_ptr<int64_t>(), static_cast<int>(num_segments),
                                 static_cast<int>(total_blocks), stats.data_ptr<double>(), cur_stream(params)));
}

// ----------------------------------------------------------------------------------- stats
void tensor_moments_op(const Tensor& x, int64_t row_len, int64_t rule, double thr, const Tensor& out) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.scalar_type() == at::kDouble && out.numel() >= 8, "pz::tensor_moments");
  PZ_HIP_CHECK(pz::tensor_moments(x.data_ptr(), dt_of(x), x.numel(), row_len, static_cast<int>(rule),
                                  static_cast<float>(thr), out.data_ptr<double>(), cur_stream(x)));
}

void histogram_op(const Tensor& x, const Tensor& range, int64_t bins, const Tensor& counts) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && range.scalar_type() == at::kDouble && counts.scalar_type() == at::kLong &&
                  counts.is_contiguous() && counts.numel() >= bins,
              "pz::histogram: counts must be a contiguous int64 tensor of >= bins elements");
  PZ_HIP_CHECK(pz::histogram(x.data_ptr(), dt_of(x), x.numel(), range.data_ptr<double>(), static_cast<int>(bins),
                             counts.data_ptr<int64_t>(), cur_stream(x)));
}

// ------------------------------------------------------------------------------- batchnorm
void batchnorm_fwd_op(const Tensor& x, const Tensor& y, const Tensor& gain, const Tensor& bias,
                      const Tensor& running_mean, const Tensor& running_var, double eps, double momentum, bool training,
                      int64_t rows_valid, const Tensor& save_mean, const Tensor& save_invstd, const Tensor& partial,
                      at::IntArrayRef ei, at::ArrayRef<double> ef, int64_t idx_ld, int64_t phase, int64_t n_total) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous(), "pz::batchnorm_fwd: contiguous");
  TORCH_CHECK(gain.scalar_type() == bias.scalar_type() && gain.scalar_type() == running_mean.scalar_type() &&
                  running_mean.is_contiguous() && running_var.is_contiguous(),
              "pz::batchnorm_fwd: parameter dtypes");
  pz::BnArgs a{};
  a.x = x.data_ptr();
  a.y = y.data_ptr();
  a.dtype = dt_of(x);
  a.cols = static_cast<int>(x.size(-1));
  a.rows = static_cast<int>(x.numel() / std::max<int64_t>(a.cols, 1));
  a.rows_valid = static_cast<int>(rows_valid);
  a.gain = gain.data_ptr();
  a.bias = bias.data_ptr();
  a.param_dtype = dt_of(gain);
  a.running_mean = running_mean.data_ptr();
  a.running_var = running_var.data_ptr();
  a.eps = eps;
  a.momentum = momentum;
  a.training = training;
  a.save_mean = save_mean.data_ptr<double>();
  a.save_invstd = save_invstd.data_ptr<double>();
  a.partial = partial.data_ptr<double>();
  a.epi = make_epi(ei, ef);
  a.idx_ld = idx_ld > 0 ? idx_ld : a.cols;
  a.phase = static_cast<int>(phase);
  a.n_total = n_total;
  PZ_HIP_CHECK(pz::batchnorm_fwd(a, cur_stream(x)));
}

void batchnorm_bwd_op(const Tensor& g, const Tensor& y, const Tensor& x, const optional<Tensor>& dx, const Tensor& gain,
                      const Tensor& bias, const Tensor& save_mean, const Tensor& save_invstd,
                      const optional<Tensor>& dgain, const optional<Tensor>& dbias, const Tensor& partial,
                      int64_t rows_valid, at::IntArrayRef ei, at::ArrayRef<double> ef, int64_t idx_ld, int64_t phase, int64_t n_total) {
  check_dev(g, "g");
  TORCH_CHECK(g.is_contiguous() && y.is_contiguous() && x.is_contiguous(), "pz::batchnorm_bwd: contiguous");
  pz::BnBwdArgs a{};
  a.g = g.data_ptr();
  a.y = y.data_ptr();
  a.x = x.data_ptr();
  a.dx = ptr_or_null(dx);
  a.dtype = dt_of(x);
  a.cols = static_cast<int>(x.size(-1));
  a.rows = static_cast<int>(x.numel() / std::max<int64_t>(a.cols, 1));
  a.rows_valid = static_cast<int>(rows_valid);
  a.gain = gain.data_ptr();
  a.bias = bias.data_ptr();
  a.param_dtype = dt_of(gain);
  a.save_mean = save_mean.data_ptr<double>();
  a.save_invstd = save_invstd.data_ptr<double>();
  a.dgain = ptr_or_null(dgain);
  a.dbias = ptr_or_null(dbias);
  a.partial = partial.data_ptr<double>();
  a.epi = make_epi(ei, ef);
  a.idx_ld = idx_ld > 0 ? idx_ld : a.cols;
  a.phase = static_cast<int>(phase);
  a.n_total = n_total;
  PZ_HIP_CHECK(pz::batchnorm_bwd(a, cur_stream(g)));
}

// ------------------------------------------------------------------------------- embedding
int idx_type(const Tensor& idx) {
  switch (idx.scalar_type()) {
    case at::kLong: return pz::IDX_I64;
    case at::kFloat: return pz::IDX_F32;
    case at::kDouble: return pz::IDX_F64;
    default: TORCH_CHECK(false, "pz: embedding ids must be int64, float32 or float64");
  }
  return -1;
}

void embedding_fwd_op(const Tensor& table, const Tensor& idx, const Tensor& out) {
  check_dev(table, "table");
  TORCH_CHECK(idx.is_contiguous() && out.is_contiguous() && table.is_contiguous(), "pz::embedding_fwd: contiguous");
  const int dim = static_cast<int>(table.size(1));
  TORCH_CHECK(out.numel() == idx.numel() * dim, "pz::embedding_fwd: out shape");
  PZ_HIP_CHECK(pz::embedding_fwd(table.data_ptr(), dt_of(table), table.size(0), idx.data_ptr(), idx_type(idx),
                                 idx.numel(), dim, out.data_ptr(), dt_of(out), cur_stream(table)));
}

void embedding_bwd_op(const Tensor& dout, const Tensor& idx, const Tensor& dtable) {
  check_dev(dout, "dout");
  TORCH_CHECK(idx.is_contiguous() && dout.is_contiguous() && dtable.is_contiguous(), "pz::embedding_bwd: contiguous");
  const int dim = static_cast<int>(dtable.size(1));
  PZ_HIP_CHECK(pz::embedding_bwd(dout.data_ptr(), dt_of(dout), idx.data_ptr(), idx_type(idx), idx.numel(), dim,
                                 dtable.size(0), dtable.data_ptr(), dt_of(dtable), cur_stream(dout)));
}

// ------------------------------------------------------------------------------------ fp8
void amax_abs_op(const Tensor& x, const Tensor& amax) {
  check_dev(x, "x");
  TORCH_CHECK(x.is_contiguous() && amax.scalar_type() == at::kFloat, "pz::amax_abs: contiguous x, fp32 amax");
  PZ_HIP_CHECK(pz::amax_abs(x.data_ptr(), dt_of(x), x.numel(), amax.data_ptr<float>(), cur_stream(x)));
}

void scale_update_op(const Tensor& amax, const Tensor& qs, double headroom, bool reset, double maxval) {
  check_dev(amax, "amax");
  TORCH_CHECK(amax.scalar_type() == at::kFloat && qs.scalar_type() == at::kFloat && qs.numel() >= 2 * amax.numel(),
              "pz::scale_update: fp32 amax[n], qs[2n]");
  PZ_HIP_CHECK(pz::scale_update(amax.data_ptr<float>(), qs.data_ptr<float>(), static_cast<int>(amax.numel()),
                                static_cast<float>(headroom), reset, cur_stream(amax), static_cast<float>(maxval)));
}

void quant_transpose_op(const Tensor& w, const Tensor& out, const Tensor& qs, const optional<Tensor>& amax,
                        const optional<Tensor>& amax_clear) {
  check_dev(w, "w");
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.dim() == 2 && w.stride(1) == 1, "pz::quant_transpose: fp32 [K,N] w");
  TORCH_CHECK(out.scalar_type() == at::kFloat8_e4m3fn && out.dim() == 2 && out.stride(1) == 1 &&
                  out.size(0) == w.size(1) && out.size(1) == w.size(0) && out.stride(0) % 4 == 0,
              "pz::quant_transpose: out must be e4m3 [N,K]");
  TORCH_CHECK(qs.scalar_type() == at::kFloat && qs.numel() >= 2, "pz::quant_transpose: fp32 qs[2]");
  const bool fused = amax.has_value() && amax->defined();
  TORCH_CHECK(!fused || (amax_clear.has_value() && amax_clear->defined() && amax->scalar_type() == at::kFloat &&
                         amax_clear->scalar_type() == at::kFloat && amax->numel() >= 1 && amax_clear->numel() >= 1),
              "pz::quant_transpose: fp32 amax and amax_clear go together");
  PZ_HIP_CHECK(pz::quant_transpose(w.data_ptr<float>(), w.stride(0), static_cast<int>(w.size(0)),
                                   static_cast<int>(w.size(1)), static_cast<uint8_t*>(out.data_ptr()), out.stride(0),
                                   qs.data_ptr<float>(), fused ? amax->data_ptr<float>() : nullptr,
                                   fused ? amax_clear->data_ptr<float>() : nullptr, cur_stream(w)));
}

void quantize_rows_op(const Tensor& x, const Tensor& out, const Tensor& qs, const optional<Tensor>& amax,
                      const optional<Tensor>& amax_in, const optional<Tensor>& amax_clear) {
  check_dev(x, "x");
  const bool e5m2 = out.scalar_type() == at::kFloat8_e5m2;
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && out.dim() == 2 && out.stride(1) == 1 &&
                  (out.scalar_type() == at::kFloat8_e4m3fn || e5m2) && out.size(0) >= x.size(0) &&
                  out.size(1) >= x.size(1) && out.stride(0) % 4 == 0 && x.size(1) % 4 == 0,
              "pz::quantize_rows: x [rows, cols % 4 == 0], out e4m3 / e5m2 [rows, cols]");
  PZ_HIP_CHECK(pz::quantize_rows(x.data_ptr(), dt_of(x), x.stride(0), static_cast<int>(x.size(0)),
                                 static_cast<int>(x.size(1)), static_cast<uint8_t*>(out.data_ptr()), out.stride(0),
                                 qs.data_ptr<float>(), amax.has_value() ? amax->data_ptr<float>() : nullptr,
                                 cur_stream(x), e5m2 ? 1 : 0, f32_scalar_ptr(amax_in, "amax_in"),
                                 amax_clear.has_value() ? amax_clear->data_ptr<float>() : nullptr));
}

void step_finalize_op(const optional<Tensor>& loss, double loss_div, const Tensor& stats_prev, const Tensor& stats_cur,
                      const Tensor& slot_numel, int64_t nslots, double l2, const Tensor& costs, int64_t epoch,
                      const Tensor& ratios, int64_t ratio_row, const optional<Tensor>& epoch_ctr, int64_t every,
                      const optional<Tensor>& clear) {
  check_dev(costs, "costs");
  const bool dev_epoch = epoch < 0;  // read from the counter (graph-replayed step)
  TORCH_CHECK(!dev_epoch || epoch_ctr.has_value(), "pz::step_finalize: epoch < 0 needs the epoch counter");
  TORCH_CHECK(dev_epoch || epoch < costs.numel(), "pz::step_finalize: epoch out of range");
  TORCH_CHECK(ratio_row < 0 || (ratio_row + 1) * nslots <= ratios.numel(), "pz::step_finalize: ratio row out of range");
  TORCH_CHECK(ratio_row != -2 || every >= 1, "pz::step_finalize: ratio rule needs every >= 1");
  TORCH_CHECK(costs.scalar_type() == at::kDouble, "pz::step_finalize: costs must be fp64");
  pz::FinalizeArgs a{};
  if (loss.has_value() && loss->defined()) {
    TORCH_CHECK(loss->scalar_type() == at::kFloat || loss->scalar_type() == at::kDouble, "pz::step_finalize: loss dtype");
    if (loss->scalar_type() == at::kDouble) a.loss64 = loss->data_ptr<double>();
    else a.loss = loss->data_ptr<float>();
    a.loss_slots = static_cast<int>(loss->numel());
  } else {
    a.loss_slots = 1;
  }
  a.loss_div = static_cast<float>(loss_div);
  a.stats_prev = stats_prev.data_ptr<double>();
  a.stats_cur = stats_cur.data_ptr<double>();
  a.slot_numel = slot_numel.data_ptr<double>();
  a.nslots = static_cast<int>(nslots);
  a.l2 = l2;
  a.costs = costs.data_ptr<double>();
  a.epoch = static_cast<int>(epoch);
  a.ratios = ratios.data_ptr<float>();
  a.ratio_row = static_cast<int>(ratio_row);
  a.every = static_cast<int>(every);
  a.n_costs = static_cast<int>(costs.numel());
  a.n_ratio_rows = static_cast<int>(ratios.numel() / (nslots > 0 ? nslots : 1));
  a.epoch_ptr = const_cast<int*>(epoch_counter(epoch_ctr));
  if (clear.has_value() && clear->defined()) {
    TORCH_CHECK(clear->scalar_type() == at::kFloat && clear->is_contiguous(), "pz::step_finalize: fp32 clear");
    a.clear = clear->data_ptr<float>();
    a.nclear = static_cast<int>(clear->numel());
  }
  PZ_HIP_CHECK(pz::step_finalize(a, cur_stream(costs)));
}

// ----------------------------------------------------------------------------- host (N9)
std::string format_json_array_op(const Tensor& t, int64_t level) {
  TORCH_CHECK(!t.is_cuda() && t.scalar_type() == at::kDouble, "pz::format_json_array: CPU float64 tensor expected");
  std::vector<int64_t> shape(t.sizes().begin(), t.sizes().end());
  std::vector<int64_t> strides(t.strides().begin(), t.strides().end());
  return pz::format_json_array(t.data_ptr<double>(), shape.data(), strides.data(), static_cast<int>(t.dim()), level);
}

std::string repr_double_op(double x) { return pz::repr_double(x); }

// checkpoint reader (N9): -> (skeleton JSON text, float64 values, int64 [ndim, dims...] records)
std::tuple<std::string, Tensor, Tensor> scan_json_arrays_op(const std::string& path, const std::string& key) {
  std::string text;
  {
    FILE* f = std::fopen(path.c_str(), "rb");
    TORCH_CHECK(f != nullptr, "pz::scan_json_arrays: cannot open ", path);
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    text.resize(n > 0 ? static_cast<size_t>(n) : 0);
    const size_t got = n > 0 ? std::fread(&text[0], 1, static_cast<size_t>(n), f) : 0;
    std::fclose(f);
    TORCH_CHECK(got == text.size(), "pz::scan_json_arrays: short read of ", path);
  }
  std::string skeleton;
  std::vector<double> values;
  std::vector<int64_t> shapes;
  try {
    pz::scan_json_arrays(text, key, skeleton, values, shapes);
  } catch (const std::exception& e) {
    TORCH_CHECK(false, e.what());
  }
  Tensor v = at::empty({static_cast<int64_t>(values.size())}, at::TensorOptions().dtype(at::kDouble));
  if (!values.empty()) std::memcpy(v.data_ptr<double>(), values.data(), values.size() * sizeof(double));
  Tensor s = at::empty({static_cast<int64_t>(shapes.size())}, at::TensorOptions().dtype(at::kLong));
  if (!shapes.empty()) std::memcpy(s.data_ptr<int64_t>(), shapes.data(), shapes.size() * sizeof(int64_t));
  return {std::move(skeleton), v, s};
}

// metadata reader: top-level JSON object of `path` with the named members' values nulled (mmap'd,
// skipped structurally: the REST progress / stats polls never parse parameter arrays)
std::string json_skip_keys_op(const std::string& path, const std::vector<std::string>& keys) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  TORCH_CHECK(fd >= 0, "pz::json_skip_keys: cannot open ", path);
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    TORCH_CHECK(false, "pz::json_skip_keys: cannot stat ", path);
  }
  const size_t n = static_cast<size_t>(st.st_size);
  if (n == 0) {
    ::close(fd);
    TORCH_CHECK(false, "pz::json_skip_keys: empty file ", path);
  }
  void* m = ::mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  TORCH_CHECK(m != MAP_FAILED, "pz::json_skip_keys: mmap failed for ", path);
  ::madvise(m, n, MADV_SEQUENTIAL);
  std::string out;
  try {
    out = pz::json_null_keys(static_cast<const char*>(m), n, keys);
  } catch (const std::exception& e) {
    ::munmap(m, n);
    TORCH_CHECK(false, e.what());
  }
  ::munmap(m, n);
  return out;
}

}  // namespace

TORCH_LIBRARY(pz, m) {
  m.def("gemm(Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor(a!) C, Tensor? bias, Tensor? aux, Tensor(b!)? colsum, "
        "int epi_mode, int[] epi_i, float[] epi_f, float alpha, bool accumulate, int M, int N, int K, int idx_ld, "
        "bool force_generic, Tensor(c!)? mask=None, Tensor? scale_a=None, Tensor? scale_b=None, "
        "Tensor(d!)? out8=None, Tensor? out8_qscale=None, Tensor(e!)? amax=None, int flags=0) -> ()");
  m.def("gemm_update(Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor grad, int M, int N, int K, float alpha, "
        "Tensor(a!) params, Tensor(b!)? exp_avg, Tensor(c!)? exp_avg_sq, Tensor(d!)? shadow, Tensor(e!)? stats, "
        "Tensor(f!)? amax, bool adam, float lr, float beta1, float beta2, float eps, float bias_c1, "
        "float bias_c2_sqrt, float grad_scale, float l2, Tensor? hp=None, Tensor? epoch=None, int stats_every=1) -> ()");
  m.def("gemm_path(Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor C, int M, int N, int K) -> int");
  m.def("gemm_pair_split(Tensor A0, Tensor B0, Tensor C0, Tensor A1, Tensor B1, Tensor C1, int M0, int N0, int M1, "
        "int N1, int K, int engine=0) -> int");
  m.def("gemm_pair(Tensor A0, Tensor B0, Tensor(a!) C0, Tensor A1, Tensor B1, Tensor(b!) C1, int M0, int N0, int M1, "
        "int N1, int K, Tensor? scale_a0=None, Tensor? scale_b0=None, Tensor? scale_a1=None, "
        "Tensor? scale_b1=None, int flags=0) -> ()");
  m.def("stage_fwd(Tensor x, Tensor(a!) y, int[] epi_i, float[] epi_f) -> ()");
  m.def("stage_bwd(Tensor g, Tensor y, Tensor(a!) dx, int[] epi_i, float[] epi_f) -> ()");
  m.def("xent_head(Tensor logits, Tensor labels, int rows_valid, Tensor(a!)? loss, float loss_scale, Tensor(b!)? dh, "
        "float grad_scale, Tensor(c!)? colsum, Tensor(d!)? probs, int[] epi_i, float[] epi_f, int idx_ld, "
        "Tensor(e!)? out8=None, Tensor? out8_qscale=None, Tensor(f!)? amax=None, bool store_dh=True, "
        "Tensor(s!)? su_amax=None, Tensor(t!)? su_qs=None, float su_headroom=1.0, float su_maxval=448.0, "
        "Tensor? su_qs_prev=None) -> ()");
  m.def("mse_head(Tensor y, Tensor target, int rows_valid, Tensor(a!)? loss, float loss_scale, Tensor(b!)? dh, "
        "float grad_scale, Tensor(c!)? colsum, int[] epi_i, float[] epi_f, int idx_ld) -> ()");
  m.def("softmax_rows(Tensor x, Tensor(a!) y) -> ()");
  m.def("softmax_bwd(Tensor g, Tensor y, Tensor(a!) dx) -> ()");
  m.def("colsum(Tensor x, Tensor(a!) out) -> ()");
  m.def("gather_rows(Tensor data, Tensor? indices, int seed_lo, int seed_hi, Tensor(a!) out, int rows_valid, "
        "Tensor? labels_in, Tensor(b!)? labels_out, Tensor(c!)? picked, Tensor? epoch=None, Tensor? data8=None, "
        "Tensor(d!)? out8=None, Tensor(s!)? su_amax=None, Tensor(t!)? su_qs=None, float su_headroom=1.0, "
        "float su_maxval=448.0) -> ()");
  m.def("pack_segments(int[] offsets, int[] numels, int[] is_weight, int[] stat_slot, Tensor?[] shadows, "
        "Tensor?[] grads16, int[] zero_grad, Tensor?[] amax, Tensor?[] w8, Tensor?[] w8_amax_prev, "
        "Tensor?[] w8_qs) -> Tensor");
  m.def("optimizer_step(Tensor(a!) params, Tensor(e!) grads, Tensor(b!)? exp_avg, Tensor(c!)? exp_avg_sq, Tensor segments, "
        "Tensor block_seg, int num_segments, int total_blocks, bool adam, float lr, float beta1, float beta2, float eps, "
        "float bias_c1, float bias_c2_sqrt, float grad_scale, float l2, Tensor(d!)? stats, Tensor? hp=None, "
        "Tensor? epoch=None, int stats_every=1, int max_grid=0) -> ()");
  m.def("segment_stats(Tensor params, Tensor segments, Tensor block_seg, int num_segments, int total_blocks, "
        "Tensor(a!) stats) -> ()");
  m.def("tensor_moments(Tensor x, int row_len, int rule, float thr, Tensor(a!) out) -> ()");
  m.def("histogram(Tensor x, Tensor range, int bins, Tensor(a!) counts) -> ()");
  m.def("batchnorm_fwd(Tensor x, Tensor(a!) y, Tensor gain, Tensor bias, Tensor(b!) running_mean, "
        "Tensor(c!) running_var, float eps, float momentum, bool training, int rows_valid, Tensor(d!) save_mean, "
        "Tensor(e!) save_invstd, Tensor(f!) partial, int[] epi_i, float[] epi_f, int idx_ld, int phase=0, int n_total=0) -> ()");
  m.def("batchnorm_bwd(Tensor g, Tensor y, Tensor x, Tensor(a!)? dx, Tensor gain, Tensor bias, Tensor save_mean, "
        "Tensor save_invstd, Tensor(b!)? dgain, Tensor(c!)? dbias, Tensor(d!) partial, int rows_valid, int[] epi_i, "
        "float[] epi_f, int idx_ld, int phase=0, int n_total=0) -> ()");
  m.def("embedding_fwd(Tensor table, Tensor idx, Tensor(a!) out) -> ()");
  m.def("embedding_bwd(Tensor dout, Tensor idx, Tensor(a!) dtable) -> ()");
  m.def("step_finalize(Tensor(e!)? loss, float loss_div, Tensor(a!) stats_prev, Tensor stats_cur, Tensor slot_numel, "
        "int nslots, float l2, Tensor(b!) costs, int epoch, Tensor(c!) ratios, int ratio_row, "
        "Tensor(d!)? epoch_ctr=None, int every=1, Tensor(f!)? clear=None) -> ()");
  m.def("amax_abs(Tensor x, Tensor(a!) amax) -> ()");
  m.def("scale_update(Tensor(a!) amax, Tensor(b!) qs, float headroom, bool reset, float maxval=448.0) -> ()");
  m.def("quant_transpose(Tensor w, Tensor(a!) out, Tensor(b!) qs, Tensor? amax=None, Tensor(c!)? amax_clear=None) -> ()");
  m.def("quantize_rows(Tensor x, Tensor(a!) out, Tensor(c!) qs, Tensor(b!)? amax, Tensor? amax_in=None, "
        "Tensor(d!)? amax_clear=None) -> ()");
  m.def("format_json_array(Tensor t, int level) -> str");
  m.def("repr_double(float x) -> str");
  m.def("scan_json_arrays(str path, str key) -> (str, Tensor, Tensor)");
  m.def("json_skip_keys(str path, str[] keys) -> str");
}

TORCH_LIBRARY_IMPL(pz, CUDA, m) {
  m.impl("gemm", TORCH_FN(gemm_op));
  m.impl("gemm_path", TORCH_FN(gemm_path_op));
  m.impl("gemm_pair_split", TORCH_FN(gemm_pair_split_op));
  m.impl("gemm_pair", TORCH_FN(gemm_pair_op));
  m.impl("gemm_update", TORCH_FN(gemm_update_op));
  m.impl("stage_fwd", TORCH_FN(stage_fwd_op));
  m.impl("stage_bwd", TORCH_FN(stage_bwd_op));
  m.impl("xent_head", TORCH_FN(xent_head_op));

  m.impl("mse_head", TORCH_FN(mse_head_op));
  m.impl("softmax_rows", TORCH_FN(softmax_rows_op));
  m.impl("softmax_bwd", TORCH_FN(softmax_bwd_op));
  m.impl("colsum", TORCH_FN(colsum_op));
  m.impl("gather_rows", TORCH_FN(gather_rows_op));
  m.impl("optimizer_step", TORCH_FN(optimizer_step_op));
  m.impl("segment_stats", TORCH_FN(segment_stats_op));
  m.impl("tensor_moments", TORCH_FN(tensor_moments_op));
  m.impl("histogram", TORCH_FN(histogram_op));
  m.impl("batchnorm_fwd", TORCH_FN(batchnorm_fwd_op));
  m.impl("batchnorm_bwd", TORCH_FN(batchnorm_bwd_op));
  m.impl("embedding_fwd", TORCH_FN(embedding_fwd_op));
  m.impl("embedding_bwd", TORCH_FN(embedding_bwd_op));
  m.impl("step_finalize", TORCH_FN(step_finalize_op));
  m.impl("amax_abs", TORCH_FN(amax_abs_op));
  m.impl("scale_update", TORCH_FN(scale_update_op));
  m.impl("quant_transpose", TORCH_FN(quant_transpose_op));
  m.impl("quantize_rows", TORCH_FN(quantize_rows_op));
}

TORCH_LIBRARY_IMPL(pz, CPU, m) {
  m.impl("format_json_array", TORCH_FN(format_json_array_op));
}

TORCH_LIBRARY_IMPL(pz, CompositeExplicitAutograd, m) {
  m.impl("pack_segments", TORCH_FN(pack_segments_op));
  m.impl("repr_double", TORCH_FN(repr_double_op));
  m.impl("scan_json_arrays", TORCH_FN(scan_json_arrays_op));
  m.impl("json_skip_keys", TORCH_FN(json_skip_keys_op));
}
