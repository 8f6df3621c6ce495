// Host-side launch API of the pz HIP kernels. Plain C++ (no torch headers) so the kernel
// translation units compile fast; bindings.cpp adapts torch tensors to these calls.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pz_types.h"

namespace pz {

enum DType : int { DT_BF16 = 0, DT_F32 = 1, DT_F64 = 2, DT_FP8 = 3 };

enum EpiMode : int {
  EPI_STORE = 0,  // C = alpha*AB (+bias)                      [+ optional colsum of C]
  EPI_FWD = 1,    // C = epi_fwd(alpha*AB + bias)               (fused dropout/act/dropout)
  EPI_BWD = 2,    // C = epi_bwd(alpha*AB, aux)                 [+ optional colsum of C]
  EPI_OPT = 3,    // C is NOT stored: g = alpha*AB is the gradient of the fp32 weight p[M][N] and the
                  // optimizer update of p (GemmOpt) runs in the epilogue (fp32 output, MFMA path)
};

// EPI_OPT: the weight-gradient GEMM applies the update of the weight whose gradient it produces
// (single process: nothing has to be reduced first) — the fp32 gradient is never written to
// memory nor read back by a separate optimizer pass (8 B/param of HBM traffic and one launch per
// weight saved), and the update leaves the step's tail. Numerics are those of optimizer_step
// (torch.optim.Adam single-tensor / the reference's SGD). Element (m, n) of every array below is
// at m * ldc + n (the weight's own [in, out] layout, the dW GEMM's C).
struct GemmOpt {
  float* params;          // fp32 master weight
  float* exp_avg;         // Adam moments (nullptr: SGD)
  float* exp_avg_sq;
  void* shadow;           // low-precision GEMM copy written after the update (nullptr: none)
  int shadow_dtype;       // DT_BF16 or DT_F32
  int adam;
  double* stats;          // this weight's 4 accumulators: sum(dw), sum(dw^2), sum(w), sum(w^2)
  float* amax;            // optional: max |w_new| (fp8 weight scaling)
  const double* hp;       // graph-replayed steps: {lr, bias_c1, bias_c2_sqrt, -} of epoch *epoch_ptr
  const int* epoch_ptr;
  int stats_every;        // as OptArgs::stats_every
  float lr, beta1, beta2, eps, bias_c1, bias_c2_sqrt;
  float grad_scale;       // 1 / world
  float l2x2;             // 2 * l2 (the L2 term's gradient, weights only)
};

// C[M][N] = op(A) · op(B); row-major C with leading dim ldc.
//  a_kc: A stored [M][K] (K contiguous) if true, else [K][M]
//  b_kc: B stored [N][K] (K contiguous) if true, else [K][N]
struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  int M, N, K;
  int64_t lda, ldb, ldc;
  int a_kc, b_kc;
  int in_dtype;   // DType of A and B
  int out_dtype;  // DType of C
  float alpha;
  int accumulate;  // C += result (beta = 1)
  const float* bias;  // [N] fp32 or null (EPI_STORE / EPI_FWD)
  const void* aux;    // EPI_BWD: stored stage output y, [M][ldaux], dtype aux_dtype
  int64_t ldaux;
  int aux_dtype;
  float* colsum;      // [N] fp32: atomically accumulates column sums of the final C values
  // fp64 models (generic / wide paths only): the bias and the column sums in the master precision
  // (used instead of bias / colsum when set) — the fp64 fused engine stays exact to fp64 rounding
  const double* bias64;
  double* colsum64;
  // deterministic column sums (pz_common.h det_colsum; bf16 LDS-staged epilogues): per-tile partial
  // rows [ceil(M / BM) + groups][N] and per-column-strip tickets; null = float atomics
  float* cs_ws;
  int* cs_tickets;
  int epi_mode;
  EpiSpec epi;
  int64_t idx_ld;     // logical row stride used for dropout element indices (usually N)
  int force_generic;  // testing: bypass the MFMA path
  // ReLU bitmask, bit (n & 7) of byte mask_off(m, n) = (y[m][n] > 0), tile-blocked: 256 x 256
  // element blocks of 8 KiB (256 rows of 32 B), block (m / 256, n / 256) at byte
  // ((m / 256) * ldmask / 32 + n / 256) * 8192 — a [roundup(M, 256), ldmask] uint8 tensor with
  // ldmask = 32 * ceil(N / 256). One 256 x 256 tile's bits are one contiguous 8 KiB run: the
  // forward epilogue writes it as 512-B runs per store pass (a row-major [M][N/8] mask scattered
  // them as 32-B row segments over 256 rows), and the dX epilogue's 8-B reads stay inside it.
  // EPI_FWD writes it (from the final stage output); EPI_BWD with act == RELU reads it INSTEAD of
  // aux: 1/16 of the bytes of re-reading the stored bf16 activation. MFMA path only.
  uint8_t* mask;
  int64_t ldmask;
  // fp8 (e4m3) operands: A/B hold e4m3 bytes; the products are dequantised by the device-side
  // per-tensor factors *scale_a * *scale_b (nullptr = 1) on top of alpha
  const float* scale_a;
  const float* scale_b;
  int a_fmt;  // fp8 A operand format: 0 = e4m3, 1 = e5m2 (gradients of the dX GEMM)
  int b_fmt;  // fp8 B operand format: 1 = e5m2 only for the weight-gradient GEMM X8ᵀ · dZ8
  // EPI_FWD extra output: e4m3 copy of C, out8[m*ldout8 + n] = sat(C * *out8_qscale), and the
  // running max |C| (atomicMax into *amax, which the caller zeroes) for delayed scaling
  uint8_t* out8;
  int64_t ldout8;
  int out8_fmt;  // 0: e4m3 (EPI_FWD activations), 1: e5m2 (EPI_BWD: dZ for the next fp8 dW GEMM)
  const float* out8_qscale;
  float* amax;
  // split-K (set by the launcher, gemm_split()): K is cut into split_k slices computed by
  // separate workgroups; every slice stores its fp32 partial tile into ws, and the LAST slice to
  // arrive at a tile (per-tile counter) sums the others and runs the epilogue
  int split_k;
  float* ws;       // [tiles * split_k][BM * BN] fp32
  int* counters;   // [tiles], zero; reset by the last arriver
  GemmOpt opt;     // EPI_OPT only
  uint64_t* dbg;   // diagnostic phase stamps (tools/gemm_stamps.hip builds only); nullptr otherwise
  // epilogue stores of whole tiles (C, the ReLU bitmask, the fp8 copy) as write-through `sc1`
  // buffer stores (set by the launcher, PZ_GEMM_WT): a kernel boundary writes back every line a
  // kernel left dirty in the XCD L2s (~B / 6 TB/s for B dirty bytes, MI355X_MICROARCH "boundary"),
  // and a GEMM that stores 64 MB of output leaves the L2s full of them
  int store_wt;
  int prio;  // s_setprio(1) around the ping-pong MFMA blocks (set by the launcher, PZ_GEMM_PRIO)
  // persistent stream-K engine (gemm_sk.hip): workgroups = CUs it may occupy (0 = every CU; the
  // trainer lowers it while RCCL channels hold CUs), engine 0 = default choice, 1 = the tiled
  // kernels of gemm_mfma.hip, 2 = stream-K (8-wave ping-pong loop), 3 = stream-K on the 4-wave lab loop
  int cus;
  int engine;
};

// persistent stream-K engine: eligibility, workspace (fp32 floats for the partial-tile slabs of a
// `cus`-workgroup launch; 0 = none needed) and launch over one or two problems of one layout and
// epilogue kind (the second one's tiles follow the first's; equal K)
bool sk_eligible(const GemmArgs& p);
int64_t sk_ws_floats(const GemmArgs* probs, int n);
int sk_tickets(const GemmArgs* probs, int n);  // per-tile ticket counters needed
hipError_t gemm_sk(const GemmArgs* probs, int n, float* ws, int* counters, hipStream_t stream);
bool sk_default();  // PZ_GEMM_SK: the engine gemm() picks for eligible shapes
// PZ_DETERMINISTIC (default 1): bias-gradient column sums of the bf16 GEMM epilogues and heads are
// folded in a fixed order (pz_common.h det_colsum) instead of float atomics
bool deterministic();

// split-K plan for the MFMA path: 1 = none. Workspace floats needed: gemm_split_ws_floats().
int gemm_split(const GemmArgs& args);
int64_t gemm_split_ws_floats(const GemmArgs& args);

// returns hipSuccess or an error; chooses the MFMA path when the shape allows
hipError_t gemm(const GemmArgs& args, hipStream_t stream);
// two weight-gradient-layout GEMMs (A, B M/N-contiguous; plain stores; equal K; whole 256-tiles)
// in one launch. gemm_pair_split: the pair's split-K factor (set it as split_k of both, with
// gemm_split_ws_floats-sized workspaces for that factor), 0 = the pair is not eligible
int gemm_pair_split(const GemmArgs& a, const GemmArgs& b);
hipError_t gemm_pair(const GemmArgs& a, const GemmArgs& b, hipStream_t stream);
// exposed for tests / benchmarks: which path gemm() would take
int gemm_path(const GemmArgs& args);  // 0 = generic VALU, 1 = MFMA bf16 / fp8, 2 = MFMA fp32 / fp64

}  // namespace pz
