// fp8 (OCP e4m3) quantisation kernels for the fp8 precision policy.
//
// Per-tensor scaling: a tensor T is stored as T8 = sat(T * q) with q = 448 / (amax * headroom)
// and multiplied back by s = 1/q inside the GEMM epilogue. Weights use CURRENT scaling: the
// optimizer update reduces max |w_new| as it writes the weights (optim.hip, seg.amax) and the
// transpose-quantise that follows derives q from it; activations use DELAYED scaling: the
// producing GEMM epilogue records this step's amax and scale_update() turns it into the (q, s)
// pair of the next step; the first layer's input uses one STATIC scale per dataset (the dataset
// is quantised once, quantize_rows, and the minibatch gather copies its e4m3 rows).
//
// Scale records are fp32 device arrays {q, s} so no host sync is ever needed.
#include <cstdlib>

#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

constexpr float kE4m3Max = 448.f;

PZ_DEV uint8_t to_e4m3(float x) {
  x = fminf(fmaxf(x, -kE4m3Max), kE4m3Max);
  return static_cast<uint8_t>(__builtin_amdgcn_cvt_pk_fp8_f32(x, 0.f, 0, false) & 0xFF);
}
constexpr float kE5m2Max = 57344.f;
PZ_DEV uint8_t to_e5m2(float x) {
  x = fminf(fmaxf(x, -kE5m2Max), kE5m2Max);
  return static_cast<uint8_t>(__builtin_amdgcn_cvt_pk_bf8_f32(x, 0.f, 0, false) & 0xFF);
}

// one atomic per BLOCK (same-address atomics serialise: one per wave over a 4096-block grid
// cost 190 us for 8 M elements)
PZ_DEV void block_amax_commit(float m, float* amax) {
  __shared__ float part[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(part[0], part[1]), fmaxf(part[2], part[3]));
    atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
  }
}

template <typename T>
__global__ void __launch_bounds__(256) amax_kernel(const T* __restrict__ x, int64_t n, float* amax) {
  float m = 0.f;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    float v[4];
    if constexpr (sizeof(T) == 4) {
      const float4 q = reinterpret_cast<const float4*>(x)[i];
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      const uint2 q = reinterpret_cast<const uint2*>(x)[i];
      v[0] = bf2f(q.x & 0xFFFF); v[1] = bf2f(q.x >> 16); v[2] = bf2f(q.y & 0xFFFF); v[3] = bf2f(q.y >> 16);
    }
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256LL + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    m = fmaxf(m, fabsf(to_f(x[i])));
  block_amax_commit(m, amax);
}

// amax -> {q, s}; optionally clears amax for the next accumulation window
__global__ void scale_update_kernel(float* amax, float* qs, int n, float headroom, int reset, float maxval) {
  const int i = threadIdx.x + blockIdx.x * blockDim.x;
  if (i >= n) return;
  const float a = amax[i];
  // no amax recorded (a tensor nothing quantised this step: a record-mode step, a stage with no
  // e5m2 copy) carries no information: keep the previous scale instead of resetting it to 1
  if (a > 0.f) {
    const float q = maxval / (a * headroom);
    qs[2 * i] = q;
    qs[2 * i + 1] = 1.f / q;
  }
  if (reset) amax[i] = 0.f;
}

// W [K][N] (fp32, row stride ldw) -> W8 [N][K] e4m3 (row stride ldo): 64x64 tiles through LDS.
// The scale comes from qs[0] (q, already derived from the amax) or, when `amax` is given, from the
// amax the optimizer reduced while writing W: every block derives q itself, block 0 publishes
// {q, 1/q} for the GEMM and clears the other parity's accumulator (its last reader, the previous
// transpose of this weight, finished before this launch in stream order).
// FULL = every 64 x 64 tile in range with 16-B aligned rows (w: ldw % 4, out: ldo % 16): 16-B
// loads (4 instead of 16 per lane) and one 16-B store of 16 consecutive k per lane
template <bool FULL>
__global__ void __launch_bounds__(256) quant_transpose_kernel(const float* __restrict__ w, int64_t ldw, int K, int N,
                                                              uint8_t* __restrict__ out, int64_t ldo, float* qs,
                                                              const float* amax, float* amax_clear) {
  __shared__ float tile[64][65];
  const int k0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  float q;
  if (amax != nullptr) {
    const float am = *amax;
    q = am > 0.f ? kE4m3Max / am : 1.f;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
      qs[0] = q;
      qs[1] = 1.f / q;
      *amax_clear = 0.f;
    }
  } else {
    q = qs[0];
  }
  if constexpr (FULL) {
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
      const int r = (threadIdx.x >> 4) + 16 * pass, c = (threadIdx.x & 15) * 4;
      const float4 v = *reinterpret_cast<const float4*>(w + static_cast<int64_t>(k0 + r) * ldw + n0 + c);
      tile[r][c] = v.x;
      tile[r][c + 1] = v.y;
      tile[r][c + 2] = v.z;
      tile[r][c + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int r = ty; r < 64; r += 4) {
      const int k = k0 + r, n = n0 + tx;
      tile[r][tx] = (k < K && n < N) ? w[static_cast<int64_t>(k) * ldw + n] : 0.f;
    }
  }
  __syncthreads();
  // each thread writes 16 consecutive k of one output row n: 64 rows x 4 sixteen-byte runs
  const int n_local = threadIdx.x >> 2, kq = (threadIdx.x & 3) * 16;
  const int n = n0 + n_local;
  if constexpr (FULL) {
    uint32_t words[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t packed = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) packed |= static_cast<uint32_t>(to_e4m3(tile[kq + 4 * c + e][n_local] * q)) << (8 * e);
      words[c] = packed;
    }
    *reinterpret_cast<uint4*>(out + static_cast<int64_t>(n) * ldo + k0 + kq) =
        make_uint4(words[0], words[1], words[2], words[3]);
    return;
  }
  if (n >= N) return;
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const int k = k0 + kq + c;
    if (k + 3 < K) {
      uint32_t packed = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) packed |= static_cast<uint32_t>(to_e4m3(tile[kq + c + e][n_local] * q)) << (8 * e);
      *reinterpret_cast<uint32_t*>(out + static_cast<int64_t>(n) * ldo + k) = packed;
    } else {
      for (int e = 0; e < 4 && k + e < K; ++e) out[static_cast<int64_t>(n) * ldo + k + e] = to_e4m3(tile[kq + c + e][n_local] * q);
    }
  }
}

// x [rows][cols] (bf16 or fp32, row stride ldx) -> x8 [rows][ldo] (e4m3, or e5m2 when E5M2)
// with quantisation factor qs[0]
template <typename T, bool E5M2>
__global__ void __launch_bounds__(256) quantize_rows_kernel(const T* __restrict__ x, int64_t ldx, int rows, int cols,
                                                            uint8_t* __restrict__ out, int64_t ldo,
                                                            const float* __restrict__ qs, float* amax) {
  const float q = qs[0];
  float m = 0.f;
  const int per_row = cols / 4;
  const int64_t total = static_cast<int64_t>(rows) * per_row;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int r = static_cast<int>(i / per_row), c = static_cast<int>(i % per_row) * 4;
    uint32_t packed = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = to_f(x[static_cast<int64_t>(r) * ldx + c + e]);
      m = fmaxf(m, fabsf(v));
      packed |= static_cast<uint32_t>(E5M2 ? to_e5m2(v * q) : to_e4m3(v * q)) << (8 * e);
    }
    *reinterpret_cast<uint32_t*>(out + static_cast<int64_t>(r) * ldo + c) = packed;
  }
  if (amax != nullptr) block_amax_commit(m, amax);
}

// 8 elements per lane: one 16-B (bf16) or two 16-B (fp32) loads, four packed conversions and one
// 8-B store, one 32-bit row division per 8 elements (the scalar kernel above spends a 64-bit
// division and four 2-B loads per 4 elements: 18 us for the [8192, 1024] dX operand of mlp8192).
// Same clamp + conversion per value as to_e4m3 / to_e5m2, so the bytes are identical.
// amax_in != nullptr (weights, current scaling): q = 448 / *amax_in — the max the optimizer reduced
// while writing x — derived by every block, block 0 publishes {q, 1/q} into qs and clears
// *amax_clear (the other shadow parity's accumulator), as the transpose-quantise does
template <typename T, bool E5M2>
__global__ void __launch_bounds__(256) quantize_rows8_kernel(const T* __restrict__ x, int64_t ldx, int rows, int cols,
                                                             uint8_t* __restrict__ out, int64_t ldo, float* qs,
                                                             float* amax, const float* amax_in, float* amax_clear) {
  float q;
  if (amax_in != nullptr) {
    const float am = *amax_in;
    q = am > 0.f ? kE4m3Max / am : 1.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      qs[0] = q;
      qs[1] = 1.f / q;
      *amax_clear = 0.f;
    }
  } else {
    q = qs[0];
  }
  const float lim = E5M2 ? kE5m2Max : kE4m3Max;
  float m = 0.f;
  const uint32_t per_row = static_cast<uint32_t>(cols / 8);
  const uint32_t total = static_cast<uint32_t>(rows) * per_row;
#pragma unroll 4
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t r = i / per_row, c = (i - r * per_row) * 8u;
    float v[8];
    if constexpr (sizeof(T) == 2) {
      const uint4 w = *reinterpret_cast<const uint4*>(x + static_cast<int64_t>(r) * ldx + c);
      const uint32_t u[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[2 * e] = bf2f(u[e] & 0xFFFF); v[2 * e + 1] = bf2f(u[e] >> 16); }
    } else {
      const float4 a0 = *reinterpret_cast<const float4*>(x + static_cast<int64_t>(r) * ldx + c);
      const float4 a1 = *reinterpret_cast<const float4*>(x + static_cast<int64_t>(r) * ldx + c + 4);
      v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; v[4] = a1.x; v[5] = a1.y; v[6] = a1.z; v[7] = a1.w;
    }
    uint32_t w2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float cl[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        m = fmaxf(m, fabsf(v[4 * h + e]));
        cl[e] = fminf(fmaxf(v[4 * h + e] * q, -lim), lim);
      }
      int pk;
      if constexpr (E5M2) {
        pk = __builtin_amdgcn_cvt_pk_bf8_f32(cl[0], cl[1], 0, false);
        pk = __builtin_amdgcn_cvt_pk_bf8_f32(cl[2], cl[3], pk, true);
      } else {
        pk = __builtin_amdgcn_cvt_pk_fp8_f32(cl[0], cl[1], 0, false);
        pk = __builtin_amdgcn_cvt_pk_fp8_f32(cl[2], cl[3], pk, true);
      }
      w2[h] = static_cast<uint32_t>(pk);
    }
    *reinterpret_cast<uint2*>(out + static_cast<int64_t>(r) * ldo + c) = make_uint2(w2[0], w2[1]);
  }
  if (amax != nullptr) block_amax_commit(m, amax);
}

int grid_for(int64_t work, int per_block = 256, int cap = 4096) {
  const int64_t g = (work + per_block - 1) / per_block;
  return static_cast<int>(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

hipError_t amax_abs(const void* x, int dtype, int64_t n, float* amax, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(x) & 15) != 0) return hipErrorInvalidValue;
  const int g = grid_for(n / 4 + 1, 256 * 16, 512);  // 16 float4 per thread, <= 2 blocks per CU
  if (dtype == DT_F32) hipLaunchKernelGGL(amax_kernel<float>, dim3(g), dim3(256), 0, s, static_cast<const float*>(x), n, amax);
  else if (dtype == DT_BF16)
    hipLaunchKernelGGL(amax_kernel<uint16_t>, dim3(g), dim3(256), 0, s, static_cast<const uint16_t*>(x), n, amax);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t scale_update(float* amax, float* qs, int n, float headroom, bool reset, hipStream_t s, float maxval) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(scale_update_kernel, dim3((n + 63) / 64), dim3(64), 0, s, amax, qs, n, headroom, reset ? 1 : 0,
                     maxval);
  return hipGetLastError();
}

hipError_t quant_transpose(const float* w, int64_t ldw, int K, int N, uint8_t* out, int64_t ldo, float* qs,
                           const float* amax, float* amax_clear, hipStream_t s) {
  if (K <= 0 || N <= 0) return hipSuccess;
  if (amax != nullptr && amax_clear == nullptr) return hipErrorInvalidValue;
  const bool full = K % 64 == 0 && N % 64 == 0 && ldw % 4 == 0 && ldo % 16 == 0 &&
                    (reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (full)
    hipLaunchKernelGGL(quant_transpose_kernel<true>, dim3(N / 64, K / 64), dim3(256), 0, s, w, ldw, K, N, out, ldo, qs,
                       amax, amax_clear);
  else
    hipLaunchKernelGGL(quant_transpose_kernel<false>, dim3((N + 63) / 64, (K + 63) / 64), dim3(256), 0, s, w, ldw, K, N,
                       out, ldo, qs, amax, amax_clear);
  return hipGetLastError();
}

template <bool E5M2>
hipError_t quantize_rows_fmt(const void* x, int dtype, int64_t ldx, int rows, int cols, uint8_t* out, int64_t ldo,
                             float* qs, float* amax, hipStream_t s, const float* amax_in, float* amax_clear) {
  const int esz = dtype == DT_BF16 ? 2 : 4;
  const bool vec8 = (dtype == DT_BF16 || dtype == DT_F32) && cols % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0 &&
                    static_cast<int64_t>(rows) * (cols / 8) < (int64_t(1) << 31) && esz > 0;
  if (vec8) {
    // block cap 256: the per-block amax atomics hit one address and serialise, so fewer,
    // longer-lived blocks (profiles/r2_ab_quant_grid.txt); no amax output: 4 blocks per CU
    const int g8 = grid_for(static_cast<int64_t>(rows) * (cols / 8), 256 * 4, amax == nullptr ? 1024 : 256);
    if (dtype == DT_BF16)
      hipLaunchKernelGGL((quantize_rows8_kernel<uint16_t, E5M2>), dim3(g8), dim3(256), 0, s,
                         static_cast<const uint16_t*>(x), ldx, rows, cols, out, ldo, qs, amax, amax_in, amax_clear);
    else
      hipLaunchKernelGGL((quantize_rows8_kernel<float, E5M2>), dim3(g8), dim3(256), 0, s, static_cast<const float*>(x),
                         ldx, rows, cols, out, ldo, qs, amax, amax_in, amax_clear);
    return hipGetLastError();
  }
  if (amax_in != nullptr) return hipErrorInvalidValue;  // (the derived scale: 8-wide path only)
  const int g = grid_for(static_cast<int64_t>(rows) * (cols / 4), 256 * 8, 1024);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL((quantize_rows_kernel<uint16_t, E5M2>), dim3(g), dim3(256), 0, s,
                       static_cast<const uint16_t*>(x), ldx, rows, cols, out, ldo, qs, amax);
  else if (dtype == DT_F32)
    hipLaunchKernelGGL((quantize_rows_kernel<float, E5M2>), dim3(g), dim3(256), 0, s, static_cast<const float*>(x),
                       ldx, rows, cols, out, ldo, qs, amax);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t quantize_rows(const void* x, int dtype, int64_t ldx, int rows, int cols, uint8_t* out, int64_t ldo,
                         float* qs, float* amax, hipStream_t s, int fmt, const float* amax_in, float* amax_clear) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (cols % 4 != 0 || (amax_in != nullptr && (amax_clear == nullptr || fmt != 0))) return hipErrorInvalidValue;
  if (fmt == 1) return quantize_rows_fmt<true>(x, dtype, ldx, rows, cols, out, ldo, qs, amax, s, amax_in, amax_clear);
  return quantize_rows_fmt<false>(x, dtype, ldx, rows, cols, out, ldo, qs, amax, s, amax_in, amax_clear);
}

}  // namespace pz
