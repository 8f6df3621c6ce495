// Throughput of integer-hash building blocks on gfx950 (dropout mask generation cost):
// lowbias32 (2 x v_mul_lo_u32) vs a 24-bit-multiply mixer. Each thread chains 256 hashes.
//   hipcc --offload-arch=gfx950 -O3 tools/hash_rate_lab.hip -o tools/hash_rate_lab
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t mix24(uint32_t x) {  // two full-rate 24x24 multiplies
  x ^= x >> 16; x = __umul24(x, 0x2d352bU) ^ (x >> 24);
  x ^= x >> 15; x = __umul24(x, 0x6ca68bU) ^ (x >> 24);
  x ^= x >> 16;
  return x;
}
template <int K>
__global__ void k(uint32_t* out, uint32_t seed) {
  uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, acc = 0;
#pragma unroll 16
  for (int i = 0; i < 256; ++i) {
    const uint32_t h = K == 0 ? mix32(x ^ (seed + i)) : mix24(x ^ (seed + i));
    acc += h >> 16;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
int main() {
  const int n = 1 << 24;
  uint32_t* out;
  hipMalloc(&out, n * 4);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    for (int v = 0; v < 2; ++v) {
      auto f = v == 0 ? k<0> : k<1>;
      hipLaunchKernelGGL(f, dim3(n / 256), dim3(256), 0, 0, out, 1u);
      hipEventRecord(a);
      for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(f, dim3(n / 256), dim3(256), 0, 0, out, it + 2u);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      const double hashes = 5.0 * n * 256;
      printf("%s: %.2f Ghash/s\n", v == 0 ? "lowbias32 (mul_lo_u32)" : "mix24 (mul_u32_u24)", hashes / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
