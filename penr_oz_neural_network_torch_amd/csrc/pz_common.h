// Shared device helpers for the pz kernels (gfx950 / CDNA4 only).
//
//  * bf16 <-> f32 conversions and the MFMA operand vector types
//  * the counter-based dropout hash: a mask is a pure function of (seed, layer id, element
//    index), so backward kernels REGENERATE masks instead of storing them
//  * the fused "stage epilogue": y = drop_post(act(drop_pre(x))) forward, and its derivative
//    computed from the stored stage output y backward. This is the one place that encodes the
//    reference's layer semantics (dropout on every hidden layer output, neural_net_model.py:393-395;
//    relu/sigmoid/tanh, :172-184) for the GEMM, head and elementwise kernels alike.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pz_types.h"

#define PZ_LDS __attribute__((address_space(3)))
#define PZ_DEV __device__ __forceinline__

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x8_t __attribute__((ext_vector_type(8)));
typedef short i16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef double f64x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));  // LDS-friendly (HIP uint2/uint4 are not)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

namespace pz {

constexpr int kWave = 64;

// ------------------------------------------------------------------------------------------
// conversions
// ------------------------------------------------------------------------------------------
PZ_DEV float bf2f(uint16_t v) { return __uint_as_float(static_cast<uint32_t>(v) << 16); }
PZ_DEV uint16_t f2bf(float f) {  // RNE; hipcc lowers the cast to v_cvt_pk_bf16_f32 (NaN-safe)
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}
// two floats -> one packed bf16 pair as ONE v_cvt_pk_bf16_f32 (RNE, NaN-safe): the scalar form
// (two casts + shift + or) cost 4 VALU instructions per pair in every epilogue
typedef float pz_f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 pz_bf16x2_t __attribute__((ext_vector_type(2)));
PZ_DEV uint32_t pack_bf2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(pz_f32x2_t{lo, hi}, pz_bf16x2_t));
}

template <typename T> PZ_DEV float to_f(T v) { return static_cast<float>(v); }
template <> PZ_DEV float to_f<uint16_t>(uint16_t v) { return bf2f(v); }
template <typename T> PZ_DEV T from_f(float v) { return static_cast<T>(v); }
template <> PZ_DEV uint16_t from_f<uint16_t>(float v) { return f2bf(v); }

// 8 fp32 -> 8 e5m2 bytes (OCP bf8, saturating at +-57344): the backward's dZ copy
PZ_DEV u32x2_t to_e5m2x8(const float (&x)[8], float qs) {
  u32x2_t out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = fminf(fmaxf(x[4 * h + q] * qs, -57344.f), 57344.f);
    int w = __builtin_amdgcn_cvt_pk_bf8_f32(c[0], c[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_bf8_f32(c[2], c[3], w, true);
    out[h] = static_cast<uint32_t>(w);
  }
  return out;
}

// 8 fp32 -> 8 e4m3 bytes (OCP, saturating at +-448)
PZ_DEV u32x2_t to_e4m3x8(const float (&x)[8], float qs) {
  u32x2_t out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) c[q] = fminf(fmaxf(x[4 * h + q] * qs, -448.f), 448.f);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w, true);
    out[h] = static_cast<uint32_t>(w);
  }
  return out;
}

// a folded scale update (pz_kernels.h ScaleUpd): call from every thread; block 0 applies it
template <class SU>
PZ_DEV void apply_scale_update(const SU& su) {
  if (su.n <= 0 || blockIdx.x != 0 || blockIdx.y != 0 || static_cast<int>(threadIdx.x) >= su.n) return;
  const int i = threadIdx.x;
  const float a = su.amax[i];
  if (a > 0.f) {  // no amax this step (nothing quantised that tensor): keep the previous scale
    const float q = su.maxval / (a * su.headroom);
    su.qs[2 * i] = q;
    su.qs[2 * i + 1] = 1.f / q;
  } else if (su.qs_prev != nullptr) {
    su.qs[2 * i] = su.qs_prev[2 * i];
    su.qs[2 * i + 1] = su.qs_prev[2 * i + 1];
  }
  su.amax[i] = 0.f;
}

// ------------------------------------------------------------------------------------------
// counter-based dropout RNG
// ------------------------------------------------------------------------------------------
PZ_DEV uint32_t mix32(uint32_t x) {  // "lowbias32" integer finaliser
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// per-epoch key of a (seed, layer) key; mirrored on the host by ops/functional.py: epoch_key
PZ_DEV uint32_t epoch_key(uint32_t key, uint32_t epoch) { return mix32(key ^ mix32(epoch * 0x9E3779B1u + 0x7F4A7C15u)); }
// per-epoch minibatch seeds; mirrored on the host by engine/trainer.py: FusedTrainer._gather_seed
PZ_DEV void gather_seed(uint32_t& lo, uint32_t& hi, uint32_t epoch) {
  lo += epoch * 0x632BE5ABu;
  hi ^= epoch;
}
// 32 random bits shared by the element pair (2j, 2j+1); each element uses 16 of them
PZ_DEV uint32_t pair_bits(uint32_t pair, uint32_t key) { return mix32(pair ^ key); }
PZ_DEV bool keep_elem(uint64_t idx, uint32_t key, uint32_t thresh16) {
  const uint32_t bits = pair_bits(static_cast<uint32_t>(idx >> 1), key);
  const uint32_t r = (idx & 1) ? (bits >> 16) : (bits & 0xFFFFu);
  return r >= thresh16;
}

// ------------------------------------------------------------------------------------------
// stage epilogue math (EpiSpec lives in pz_types.h)
// ------------------------------------------------------------------------------------------
PZ_DEV float fexp(float x) { return __expf(x); }
PZ_DEV double fexp(double x) { return exp(x); }
PZ_DEV float ftanh(float x) { return tanhf(x); }
PZ_DEV double ftanh(double x) { return tanh(x); }

template <typename F>
PZ_DEV F act_fwd(F x, int act) {
  switch (act) {
    case ACT_RELU: return x > F(0) ? x : F(0);
    case ACT_SIGMOID: return F(1) / (F(1) + fexp(-x));
    case ACT_TANH: return ftanh(x);
    default: return x;
  }
}
// derivative expressed through the activation OUTPUT a
template <typename F>
PZ_DEV F act_grad_from_out(F a, int act) {
  switch (act) {
    case ACT_RELU: return a > F(0) ? F(1) : F(0);
    case ACT_SIGMOID: return a * (F(1) - a);
    case ACT_TANH: return F(1) - a * a;
    default: return F(1);
  }
}

// make a (possibly graph-replayed) spec concrete: mix the device epoch counter into the keys
PZ_DEV EpiSpec epi_resolve(EpiSpec e) {
  if (e.epoch_ptr != nullptr) {
    const uint32_t ep = static_cast<uint32_t>(*e.epoch_ptr);
    e.key_pre = epoch_key(e.key_pre, ep);
    e.key_post = epoch_key(e.key_post, ep);
    e.epoch_ptr = nullptr;
  }
  return e;
}

PZ_DEV bool epi_keep(const EpiSpec& e, uint32_t key, uint64_t idx) {
  if (e.drop_all) return false;
  return keep_elem(idx, key, e.thresh16);
}

// forward: x = producing-op output (bias already added), idx = logical element index
// dropout scale in the math precision F: the fp64 kernels use the exact double (F.dropout's
// 1/(1-p) in fp64), the fp32 ones the float
template <typename F> PZ_DEV F epi_scale(const EpiSpec& e) { return F(e.scale); }
template <> PZ_DEV double epi_scale<double>(const EpiSpec& e) { return e.scale64; }
template <typename F> PZ_DEV F epi_inv_scale(const EpiSpec& e) { return F(e.inv_scale); }
template <> PZ_DEV double epi_inv_scale<double>(const EpiSpec& e) { return e.inv_scale64; }

template <typename F>
PZ_DEV F epi_fwd(F x, uint64_t idx, const EpiSpec& e) {
  const F sc = epi_scale<F>(e);
  if (e.drop_pre) x = epi_keep(e, e.key_pre, idx) ? x * sc : F(0);
  x = act_fwd(x, e.act);
  if (e.drop_post) x = epi_keep(e, e.key_post, idx) ? x * sc : F(0);
  return x;
}

// backward: g = dLoss/dy, y = stored stage output; returns dLoss/dx (x as in epi_fwd)
template <typename F>
PZ_DEV F epi_bwd(F g, F y, uint64_t idx, const EpiSpec& e) {
  const F sc = epi_scale<F>(e);
  if (e.drop_post) {
    if (!epi_keep(e, e.key_post, idx)) return F(0);
    g *= sc;
    y *= epi_inv_scale<F>(e);
  }
  if (e.act != ACT_NONE) g *= act_grad_from_out(y, e.act);
  if (e.drop_pre) {
    if (!epi_keep(e, e.key_pre, idx)) return F(0);
    g *= sc;
  }
  return g;
}

// 4 consecutive elements starting at an EVEN index: two hashes per dropout layer
PZ_DEV void keep4(const EpiSpec& e, uint32_t key, uint64_t idx, float m[4]) {
  if (e.drop_all) { m[0] = m[1] = m[2] = m[3] = 0.f; return; }
  const uint32_t p0 = static_cast<uint32_t>(idx >> 1);
  const uint32_t b0 = mix32(p0 ^ key), b1 = mix32((p0 + 1) ^ key);
  m[0] = (b0 & 0xFFFFu) >= e.thresh16 ? e.scale : 0.f;
  m[1] = (b0 >> 16) >= e.thresh16 ? e.scale : 0.f;
  m[2] = (b1 & 0xFFFFu) >= e.thresh16 ? e.scale : 0.f;
  m[3] = (b1 >> 16) >= e.thresh16 ? e.scale : 0.f;
}

PZ_DEV void epi_fwd4(float v[4], uint64_t idx, const EpiSpec& e) {
  if (e.drop_pre) {
    float m[4];
    keep4(e, e.key_pre, idx, m);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= m[r];
  }
  if (e.act != ACT_NONE) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = act_fwd(v[r], e.act);
  }
  if (e.drop_post) {
    float m[4];
    keep4(e, e.key_post, idx, m);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= m[r];
  }
}

PZ_DEV void epi_bwd4(float g[4], const float y_in[4], uint64_t idx, const EpiSpec& e) {
  float y[4] = {y_in[0], y_in[1], y_in[2], y_in[3]};
  if (e.drop_post) {
    float m[4];
    keep4(e, e.key_post, idx, m);
#pragma unroll
    for (int r = 0; r < 4; ++r) { g[r] *= m[r]; y[r] *= e.inv_scale; }
  }
  if (e.act != ACT_NONE) {
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] *= act_grad_from_out(y[r], e.act);
  }
  if (e.drop_pre) {
    float m[4];
    keep4(e, e.key_pre, idx, m);
#pragma unroll
    for (int r = 0; r < 4; ++r) g[r] *= m[r];
  }
}

// ------------------------------------------------------------------------------------------
// wave / block reductions (wave64)
// ------------------------------------------------------------------------------------------
// Reductions over DPP rows (16 lanes) with in-row DPP moves — quad_perm xor 1, xor 2, then
// row_half_mirror and row_mirror (each lane then holds its row's total) — instead of ds_bpermute
// shuffles (an LDS round trip of ~100 cycles per step on a serial chain); the four row totals are
// combined through v_readlane. Every lane returns the same value.
template <typename Op>
PZ_DEV float row16_reduce(float v, Op op) {
  // (the dpp control must be a literal: one builtin call per pattern)
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));   // xor 1
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));   // xor 2
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));  // half mirror
  v = op(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));  // mirror
  return v;
}
template <typename Op>
PZ_DEV float wave_reduce(float v, Op op) {
  v = row16_reduce(v, op);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return op(op(r0, r1), op(r2, r3));
}
struct OpAdd { PZ_DEV float operator()(float a, float b) const { return a + b; } };
struct OpMax { PZ_DEV float operator()(float a, float b) const { return fmaxf(a, b); } };
struct OpMin { PZ_DEV float operator()(float a, float b) const { return fminf(a, b); } };
PZ_DEV float wave_sum(float v) { return wave_reduce(v, OpAdd{}); }
PZ_DEV float wave_max(float v) { return wave_reduce(v, OpMax{}); }
PZ_DEV float wave_min(float v) { return wave_reduce(v, OpMin{}); }
// sum over the RED consecutive lanes sharing a 16- or 32-lane group (GEMM epilogue column sums)
template <int RED>
PZ_DEV float group_sum(float v) {
  static_assert(RED == 16 || RED == 32, "16- or 32-lane groups");
  v = row16_reduce(v, OpAdd{});
  if constexpr (RED == 32) v += __shfl_xor(v, 16, 64);
  return v;
}
PZ_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------------------
// Deterministic column sums across workgroups (bias gradients): instead of one float atomic per
// column and workgroup (a sum whose order is the arrival order), producer `idx` stores its partial
// row [nparts][ld] write-through (4-B sc1 stores), then the last arriver of its group of `group`
// producers folds that group's rows IN ROW ORDER into a group row (written after the partials, at
// row nparts + g), and the last group folder folds the group rows in order into colsum[c] (+=).
// Hand-off: MI355X_MICROARCH table row 1 (sc1 stores, every wave's vmcnt(0), barrier, one relaxed
// agent-scope ticket per producer; sc1 loads). Tickets: [ceil(nparts / group) + 1], zero between
// launches (each last arriver resets the one it completed).
PZ_DEV void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
PZ_DEV float ld_wt(const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// every wave's stores drained, then one ticket: true (block-uniform) in the expect-th arriver
PZ_DEV bool det_ticket(int* ticket, int expect, PZ_LDS int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == expect - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*flag) != 0;
}

// rows [r0, r1) of column c, summed in row order (loads issued 8 at a time)
PZ_DEV float det_fold(const float* ws, int64_t ld, int r0, int r1, int c) {
  float s = 0.f;
  int r = r0;
  for (; r + 8 <= r1; r += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld_wt(ws + static_cast<int64_t>(r + k) * ld + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  for (; r < r1; ++r) s += ld_wt(ws + static_cast<int64_t>(r) * ld + c);
  return s;
}

// after this block stored its row idx (columns [0, cols) of ws + idx * ld): the fold levels
template <int NT>
PZ_DEV void det_colsum(float* ws, int* tickets, int nparts, int group, int idx, int cols, int64_t ld, float* colsum,
                       PZ_LDS int* flag) {
  const int ngroups = (nparts + group - 1) / group;
  const int g = idx / group, gr0 = g * group, gr1 = min(nparts, gr0 + group);
  if (!det_ticket(tickets + g, gr1 - gr0, flag)) return;
  if (ngroups == 1) {
    for (int c = threadIdx.x; c < cols; c += NT) colsum[c] += det_fold(ws, ld, 0, nparts, c);
    return;
  }
  for (int c = threadIdx.x; c < cols; c += NT) st_wt(ws + static_cast<int64_t>(nparts + g) * ld + c, det_fold(ws, ld, gr0, gr1, c));
  if (!det_ticket(tickets + ngroups, ngroups, flag)) return;
  for (int c = threadIdx.x; c < cols; c += NT) colsum[c] += det_fold(ws, ld, nparts, nparts + ngroups, c);
}

// ------------------------------------------------------------------------------------------
// one parameter's optimizer update, shared by optimizer_step (optim.hip) and the dW-GEMM-fused
// update (EPI_OPT, gemm_mfma.hip) so both round identically. Adam = torch.optim.Adam's single-
// tensor step (lerp_, mul_/addcmul_, sqrt/div/add_, addcdiv_); SGD = the reference's
// `p -= lr * grad` (neural_net_model.py:496-507). g = graw * grad_scale + 2*l2*p0 (L2 term).
// ------------------------------------------------------------------------------------------
// R = float (fp32 masters) or double (fp64 models: torch.optim.Adam on fp64 tensors computes in
// fp64; the hyper-parameters arrive as the host's doubles rounded to R)
template <bool ADAM, typename R>
PZ_DEV R opt_update(R p0, R graw, R grad_scale, R l2x2, R lr, R step_size, R beta1, R beta2, R bias_c2_sqrt, R eps,
                    R& m, R& v) {
  const R g = graw * grad_scale + l2x2 * p0;
  if constexpr (ADAM) {
    m = m + (R(1) - beta1) * (g - m);
    v = v * beta2 + (R(1) - beta2) * g * g;
    const R denom = sqrt(v) / bias_c2_sqrt + eps;
    return p0 - step_size * (m / denom);
  } else {
    return p0 - lr * g;
  }
}

}  // namespace pz
