// Host launch API for the non-GEMM kernels (elementwise, heads, optimizer, stats, batchnorm,
// embedding). Plain C++; bindings.cpp adapts torch tensors to these structs.
#pragma once

#include "pz_launch.h"

namespace pz {

// ------------------------------------------------------------------ elementwise / heads
// A folded fp8 delayed-scale update (the scale_update op inside another launch): block 0 turns
// amax[i] into qs[2i] = q = maxval / (amax[i] * headroom), qs[2i+1] = 1/q and clears amax[i]
// (i < n). Only for launches in which nothing reads qs or writes amax. qs_prev (optional): the
// records in use this step when qs is the NEXT step's copy (double-buffered scales): an entry
// with no amax this step carries its current (q, 1/q) over instead of keeping qs's stale one.
struct ScaleUpd {
  float* amax;
  float* qs;
  int n;
  float headroom, maxval;
  const float* qs_prev;
};

struct XentArgs {
  const void* logits;   // [rows][ld]
  int64_t ld;
  const int64_t* labels;  // [rows]
  int rows, rows_valid, cols;
  int dtype;
  float* loss;          // += sum_rows (lse - x_label) * loss_scale   (may be null)
  double* loss64;       // fp64 logits: the loss accumulates here instead (double)
  int loss_slots;       // > 1: block b adds into loss[b % loss_slots] (the consumer sums them)
  double loss_scale;    // doubles: exact for fp64 models (fp32 kernels round them once)
  void* dh;             // [rows][ld_dh] gradient wrt the pre-dropout logits (may be null)
  int64_t ld_dh;
  double grad_scale;    // usually 1/global_batch
  float* colsum;        // += column sums of dh (bias gradient), may be null
  double* colsum64;     // fp64 logits: column sums in double instead
  // bf16 heads, deterministic column sums (pz_common.h det_colsum): [blocks + groups][cols] partial
  // rows and tickets; null = float atomics
  float* cs_ws;
  int* cs_tickets;
  void* probs;          // optional softmax output [rows][ld_probs]
  int64_t ld_probs;
  EpiSpec epi;          // logits' dropout (drop_pre); act must be NONE
  int64_t idx_ld;
  // fp8 policy (bf16 fast path only): e5m2 copy sat(bf16(dh) * *out8_qscale) of the gradient for
  // the stage's fp8 dX / dW GEMMs, its running max |bf16(dh)| into *amax (delayed scaling), and
  // skip_dh: the bf16 dh itself is not stored (nobody reads it; colsum is still reduced)
  uint8_t* out8;
  int64_t ld_out8;
  const float* out8_qscale;
  float* amax;
  int skip_dh;
  ScaleUpd su;  // e.g. this step's activation amax -> the next step's scales (fp8 policy)
};
bool xent_head_out8_ok(const XentArgs& a);

struct MseArgs {
  const void* y;        // final stage output [rows][ld_y]
  int64_t ld_y;
  const void* target;   // [rows][ld_t]
  int64_t ld_t;
  int rows, rows_valid, cols;
  int dtype;
  float* loss;
  double* loss64;       // fp64 outputs: double accumulators (loss64 / colsum64) instead
  int loss_slots;       // > 1: block b adds into loss[b % loss_slots]
  double loss_scale;    // 1 / numel
  void* dh;
  int64_t ld_dh;
  double grad_scale;    // 1 / numel
  float* colsum;
  double* colsum64;
  EpiSpec epi;          // last stage's epilogue (derivative from y)
  int64_t idx_ld;
};

struct GatherArgs {
  const void* data;     // [n_data][ld_data]
  int64_t ld_data;
  int data_dtype;
  int64_t n_data;
  const int64_t* indices;   // optional explicit indices [rows_valid]
  uint32_t seed_lo, seed_hi;
  void* out;            // [rows][ld_out]
  int64_t ld_out;
  int out_dtype;
  int rows, rows_valid, cols;
  const int64_t* labels_in;  // optional [n_data]
  int64_t* labels_out;       // optional [rows]
  int64_t* picked;           // optional [rows]: chosen data index per row
  const int* epoch_ptr;      // graph-replayed steps: seeds += epoch (gather_seed), read on device
  // optional second table gathered with the same picks: the dataset pre-quantised to e4m3 once
  // (fp8 policy, static scale) -> the first GEMM's fp8 operand, no per-step quantisation pass
  const uint8_t* data8;      // [n_data][ld_data8]
  int64_t ld_data8;
  uint8_t* out8;             // [rows][ld_out8]
  int64_t ld_out8;
  ScaleUpd su;               // e.g. the previous step's gradient amax -> this step's e5m2 scales
};


hipError_t stage_fwd(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, const EpiSpec& e, hipStream_t s);
hipError_t stage_bwd(const void* g, const void* y, void* dx, int dtype, int64_t n, const EpiSpec& e, hipStream_t s);
hipError_t xent_head(const XentArgs& a, hipStream_t s);
hipError_t mse_head(const MseArgs& a, hipStream_t s);
hipError_t softmax_rows(const void* x, void* y, int dtype, int rows, int cols, hipStream_t s);
hipError_t softmax_bwd(const void* g, const void* y, void* dx, int dtype, int rows, int cols, hipStream_t s);
// column sums, out[c] += sum_r x[r][c]; ws (colsum_parts(rows) x cols accumulators of out's dtype):
// deterministic ordered fold instead of float atomics
constexpr int kColsumRows = 256;
int colsum_parts(int rows);
hipError_t colsum(const void* x, int dtype, void* out, int out_dtype, int rows, int cols, hipStream_t s,
                  void* ws = nullptr);
hipError_t gather_rows(const GatherArgs& a, hipStream_t s);

// ------------------------------------------------------------------ optimizer (N6)
// One launch updates every parameter segment of a flat fp32 buffer.
struct OptSegment {
  int64_t offset;       // into params / grads / m / v (elements)
  int64_t numel;
  int is_weight;        // L2 + update-ratio statistics apply (reference: weights only)
  int stat_slot;        // index into stats (4 doubles per slot), -1 = none
  void* shadow;         // optional low-precision copy written after the update
  int shadow_dtype;
  int zero_grad;        // accumulated gradient (atomics / colsums): reset to 0 once read, so
                        // the next step needs no separate zeroing pass
  const uint16_t* grad16;  // optional bf16 gradient of this segment (data parallel: the GEMM
                           // writes it and RCCL reduces it in bf16); replaces grads[offset..]
  float* amax;             // optional: max |w_new| of the segment is atomically max-ed into *amax
                           // (fp8 policy: the weight's current-scaling amax, no separate pass)
  // optional fp8 policy e4m3 weight copy written by the update itself (natural [in, out] layout,
  // same element order as the segment): w8 = e4m3(w_new * q) with DELAYED weight scaling,
  // q = 448 / *w8_amax_prev (the amax the previous update of this weight reduced); the segment's
  // first work block publishes {q, 1/q} into w8_qs for the GEMMs of the next step
  uint8_t* w8;
  const float* w8_amax_prev;
  float* w8_qs;
};

struct OptArgs {
  // flat master buffers in the master precision `real` (DT_F32, or DT_F64 for fp64 models)
  void* params;
  void* grads;                 // read; zero_grad segments are reset to 0
  void* exp_avg;
  void* exp_avg_sq;
  int real;
  const OptSegment* segments;  // device array
  int num_segments;
  const int64_t* block_seg;    // device array: first block index of each segment (+ total)
  int total_blocks;
  int adam;                    // 1 Adam, 0 SGD
  // hyper-parameters as the host's doubles (fp64 models update in fp64, like torch.optim.Adam on
  // fp64 tensors; fp32 masters round them to float)
  double lr;
  double beta1, beta2, eps;
  double bias_c1, bias_c2_sqrt; // 1 - beta1^t, sqrt(1 - beta2^t)
  double grad_scale;           // e.g. 1 / world_size
  double l2_lambda;            // grad += 2*l2*w for weight segments
  double* stats;               // per slot: sum(dw), sum(dw^2), sum(w), sum(w^2)  (accumulated)
  // graph-replayed steps: {lr, bias_c1, bias_c2_sqrt, -} of epoch *epoch_ptr from this table
  // (filled on the host for the whole run, so eager and replayed steps use identical values)
  const double* hp;
  const int* epoch_ptr;
  // update-ratio sums (sum dw, sum dw^2, sum w): 1 = this launch, 0 = not (only sum w^2, which the
  // next step's L2 cost term needs), k > 1 = when the device epoch (*epoch_ptr) % k == 0
  int stats_every;
  int max_grid;                // > 0: at most this many workgroups (they loop over the work blocks)
};

constexpr int kOptElemsPerBlock = 4096;
hipError_t optimizer_step(const OptArgs& a, hipStream_t s);
// sum of squares of each weight segment (for the L2 term before the first update); params of dtype `real`
hipError_t segment_stats(const void* params, int real, const OptSegment* segments, const int64_t* block_seg, int num_segments,
                         int total_blocks, double* stats, hipStream_t s);

struct FinalizeArgs {
  float* loss;              // accumulated loss (summed over ranks when data parallel); reset to 0
  double* loss64;           // fp64 models: the double accumulators instead
  int loss_slots;           // loss[0..loss_slots) are summed (the heads spread their block adds)
  float loss_div;           // world size
  double* stats_prev;       // [nslots][4] stats of the weights used by this step (zeroed afterwards)
  const double* stats_cur;  // [nslots][4] stats of the update just applied
  const double* slot_numel; // [nslots]
  int nslots;
  double l2;
  double* costs;            // costs[epoch]
  int epoch;
  float* ratios;            // [rows][nslots]
  int ratio_row;            // -1: no progress point this epoch; -2: epoch % every == 0 ? epoch / every : -1
  int every;
  int n_costs;              // costs[] length (device-read epochs are bounds-checked)
  int n_ratio_rows;
  int* epoch_ptr;           // device epoch counter: read when epoch < 0, always advanced to epoch + 1
  float* clear;             // optional [nclear] fp32 accumulators reset to 0 (fp8: the weight-amax
  int nclear;               // slots the step's updates read, ready for the next step's updates)
};
hipError_t step_finalize(const FinalizeArgs& a, hipStream_t s);

// ------------------------------------------------------------------ statistics (N7)
enum SatRule : int { SAT_NONE = 0, SAT_ABS_GT = 1, SAT_LE = 2, SAT_ROW_NORM_GT = 3, SAT_ROW_MAX_GT = 4 };
// out (double[8]): min, max, sum, sumsq, saturated_count, count, row_count, -
hipError_t tensor_moments(const void* x, int dtype, int64_t n, int64_t row_len, int sat_rule, float sat_thr,
                          double* out, hipStream_t s);
// counts[bins] (int64, exact) of x over [lo, hi] read from range (double[2] on device: lo, hi)
hipError_t histogram(const void* x, int dtype, int64_t n, const double* range, int bins, int64_t* counts, hipStream_t s);

// ------------------------------------------------------------------ batchnorm (N4)
struct BnArgs {
  const void* x;          // [rows][cols] (rows = all leading dims)
  void* y;
  int dtype;
  int rows, rows_valid, cols;
  const void* gain;       // [cols] master params, dtype param_dtype
  const void* bias;
  int param_dtype;        // DT_F32 or DT_F64 for gain/bias/running stats
  void* running_mean;     // [cols] updated in training mode
  void* running_var;
  double eps, momentum;   // doubles: fp64 models keep the reference's exact EMA / eps
  int training;
  double* save_mean;      // [cols] workspace: statistics used by this pass
  double* save_invstd;    // [cols]
  double* partial;        // workspace [2][cols] (sum, sumsq)
  EpiSpec epi;            // fused stage epilogue after the affine transform
  int64_t idx_ld;
  // Synchronised batchnorm under data parallelism: phase 1 = column sums into `partial` only;
  // the caller all-reduces partial; phase 2 = statistics from the reduced partial over n_total
  // rows (the global batch) + normalise. phase 0 = both (single process).
  int phase;
  int64_t n_total;        // rows behind `partial` (0: rows_valid)
};
hipError_t batchnorm_fwd(const BnArgs& a, hipStream_t s);
struct BnBwdArgs {
  const void* g;          // dLoss/d(stage output)
  const void* y;          // stage output (after epilogue)
  const void* x;          // batchnorm input
  void* dx;
  int dtype;
  int rows, rows_valid, cols;
  const void* gain;
  const void* bias;
  int param_dtype;
  const double* save_mean;
  const double* save_invstd;
  void* dgain;            // [cols] accumulate (param dtype)
  void* dbias;
  double* partial;        // workspace [2][cols]
  void* dxhat_buf;        // optional workspace [rows][cols] (same dtype as x) for the epilogue grads
  EpiSpec epi;
  int64_t idx_ld;
  // phase 1 = sum(dy), sum(dy*xhat) into `partial` + the LOCAL parameter gradients (the data-
  // parallel gradient all-reduce sums those); the caller all-reduces partial; phase 2 = dx from
  // the reduced partial over n_total rows. phase 0 = both.
  int phase;
  int64_t n_total;
};
hipError_t batchnorm_bwd(const BnBwdArgs& a, hipStream_t s);

// ------------------------------------------------------------------ embedding (N5)
enum IdxType : int { IDX_I64 = 0, IDX_F32 = 1, IDX_F64 = 2 };
// ids follow Python indexing (negative = from the end); ids outside [-vocab, vocab) read zeros /
// drop their gradient (the host raises IndexError before launching with such ids)
hipError_t embedding_fwd(const void* table, int table_dtype, int64_t vocab, const void* idx, int idx_dtype, int64_t n_idx,
                         int dim, void* out, int out_dtype, hipStream_t s);
hipError_t embedding_bwd(const void* dout, int dout_dtype, const void* idx, int idx_dtype, int64_t n_idx, int dim,
                         int64_t vocab, void* dtable, int dtable_dtype, hipStream_t s);

// ------------------------------------------------------------------ fp8 quantisation
// qs records are {q, s}: T8 = sat(T * q), T ~= T8 * s
hipError_t amax_abs(const void* x, int dtype, int64_t n, float* amax, hipStream_t s);
// q = maxval / (amax * headroom): maxval 448 for e4m3 records, 57344 for e5m2 (gradients)
hipError_t scale_update(float* amax, float* qs, int n, float headroom, bool reset, hipStream_t s,
                        float maxval = 448.f);
// amax != nullptr: q = 448 / *amax is derived in-kernel (the optimizer reduced it), {q, 1/q} are
// written to qs, and *amax_clear (the other parity's accumulator) is reset for the next update
hipError_t quant_transpose(const float* w, int64_t ldw, int K, int N, uint8_t* out, int64_t ldo, float* qs,
                           const float* amax, float* amax_clear,
                           hipStream_t s);
// fmt 0: e4m3 (sat 448), 1: e5m2 (sat 57344). amax_in != nullptr (e4m3 only): q = 448 / *amax_in is
// derived in-kernel and {q, 1/q} written to qs, *amax_clear reset (weights: the optimizer's amax)
hipError_t quantize_rows(const void* x, int dtype, int64_t ldx, int rows, int cols, uint8_t* out, int64_t ldo,
                         float* qs, float* amax, hipStream_t s, int fmt = 0, const float* amax_in = nullptr,
                         float* amax_clear = nullptr);

// ------------------------------------------------------------------ collective footprint proxy
// `wgs` resident workgroups for `us` microseconds, moving `chunk_bytes`-long scratch slices at one
// 4 KiB chunk per `step_us` each (comm_proxy.hip: one-GPU model of a ring all-reduce's kernels)
hipError_t comm_proxy(void* scratch, int wgs, int chunk_bytes, double us, double step_us, hipStream_t s);

}  // namespace pz
