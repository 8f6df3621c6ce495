// Lab: VAR 42 / 43 (csrc/gemm_w4.h: the 4-wave LDS-DMA schedule on the fp8 scale MFMA) against the
// library's fp8 kernels on the fp8 policy's shapes, bf16 out, plain store: dX = e5m2 dZ [M][K] x e4m3
// W [N][K] (both K-contiguous) vs VAR 17; forward = e4m3 X [M][K] x e4m3 W [K][N] vs VAR 15 / 16.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I penr_oz_neural_network_torch_amd/csrc \
//         tools/gemm_w4f8_lab.hip -o tools/gemm_w4f8_lab && tools/gemm_w4f8_lab
#define PZ_GEMM_LAB 1
#include "../penr_oz_neural_network_torch_amd/csrc/gemm_mfma.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace pz;

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);            \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

// random finite fp8 bytes of moderate magnitude: e5m2 exponent field 12..17, e4m3 4..9
__global__ void fill_f8(uint8_t* p, int64_t n, uint32_t seed, int e5m2) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(mix32(static_cast<uint32_t>(i) ^ seed) + static_cast<uint32_t>(i >> 32));
    const uint32_t s = (h >> 31) & 1;
    p[i] = e5m2 ? static_cast<uint8_t>((s << 7) | ((12 + (h >> 4) % 6) << 2) | (h & 3))
                : static_cast<uint8_t>((s << 7) | ((4 + (h >> 4) % 6) << 3) | (h & 7));
  }
}

__device__ float dec_f8(uint8_t b, int e5m2) {
  const float s = (b & 0x80) ? -1.f : 1.f;
  if (e5m2) {
    const int e = (b >> 2) & 31, m = b & 3;
    return e == 0 ? s * ldexpf(m / 4.f, -14) : s * ldexpf(1.f + m / 4.f, e - 15);
  }
  const int e = (b >> 3) & 15, m = b & 7;
  return e == 0 ? s * ldexpf(m / 8.f, -6) : s * ldexpf(1.f + m / 8.f, e - 7);
}

__global__ void ref_rows(const uint8_t* A, const uint8_t* B, float* R, int N, int K, int stride, int fwd) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = static_cast<int64_t>(blockIdx.y) * stride;
  if (n >= N) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k)
    acc += dec_f8(A[m * K + k], fwd ? 0 : 1) *
           dec_f8(fwd ? B[static_cast<int64_t>(k) * N + n] : B[static_cast<int64_t>(n) * K + k], 0);
  R[static_cast<int64_t>(blockIdx.y) * N + n] = acc;
}

typedef hipError_t (*LaunchFn)(const GemmArgs&, hipStream_t);

int main() {
  struct V { const char* name; LaunchFn fn; };
  struct Case { const char* name; int M, N, K; bool fwd; std::vector<V> vs; };
  // dX: e5m2 dZ [M][K] x e4m3 W [N][K]; fwd: e4m3 X [M][K] x e4m3 W [K][N] (the natural [in, out] copy)
  const std::vector<V> dx = {{"var17", launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 17>},
                             {"var42", launch_w4f8<EK_STORE, true>}};
  const std::vector<V> fw = {{"var16", launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16>},
                             {"var15", launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15>},
                             {"var43", launch_w4f8<EK_STORE, false>}};
  std::vector<Case> cases = {{"f8_dX_8k", 8192, 8192, 1024, false, dx}, {"f8_dX_L2", 8192, 4096, 4096, false, dx},
                             {"f8_fwd_8k", 8192, 8192, 1024, true, fw}, {"f8_fwd_L2", 8192, 4096, 4096, true, fw}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Case& c : cases) {
    const std::vector<V>& vs = c.vs;
    const int64_t na = int64_t(c.M) * c.K, nb = int64_t(c.N) * c.K, nc = int64_t(c.M) * c.N;
    uint8_t *A, *B;
    uint16_t* C;
    float* R;
    CK(hipMalloc(&A, na));
    CK(hipMalloc(&B, nb));
    CK(hipMalloc(&C, nc * 2));
    const int stride = 61, nref = (c.M + stride - 1) / stride;
    CK(hipMalloc(&R, int64_t(nref) * c.N * 4));
    hipLaunchKernelGGL(fill_f8, dim3(4096), dim3(256), 0, st, A, na, 12345u, c.fwd ? 0 : 1);
    hipLaunchKernelGGL(fill_f8, dim3(4096), dim3(256), 0, st, B, nb, 777u, 0);
    hipLaunchKernelGGL(ref_rows, dim3((c.N + 255) / 256, nref), dim3(256), 0, st, A, B, R, c.N, c.K, stride,
                       int(c.fwd));
    std::vector<float> ref(size_t(nref) * c.N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    double rmax = 0.0;
    for (float v : ref) rmax = std::max(rmax, double(fabsf(v)));
    GemmArgs p{};
    p.A = A; p.B = B; p.C = C;
    p.M = c.M; p.N = c.N; p.K = c.K;
    p.lda = c.K; p.ldb = c.fwd ? c.N : c.K; p.ldc = c.N;
    p.a_kc = 1; p.b_kc = c.fwd ? 0 : 1;
    p.in_dtype = DT_FP8; p.a_fmt = c.fwd ? 0 : 1; p.b_fmt = 0; p.out_dtype = DT_BF16;
    p.alpha = 1.f; p.epi_mode = EPI_STORE; p.idx_ld = c.N; p.split_k = 1;
    const double flop = 2.0 * c.M * c.N * c.K;
    std::vector<std::vector<double>> tf(vs.size());
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipMemsetAsync(C, 0, nc * 2, st));
      CK(vs[v].fn(p, st));
      CK(hipStreamSynchronize(st));
      std::vector<uint16_t> out(nc);
      CK(hipMemcpy(out.data(), C, nc * 2, hipMemcpyDeviceToHost));
      double worst = 0.0;
      for (int r = 0; r < nref; ++r)
        for (int n = 0; n < c.N; ++n) {
          uint32_t u = uint32_t(out[size_t(r) * stride * c.N + n]) << 16;
          float got;
          memcpy(&got, &u, 4);
          const double want = ref[size_t(r) * c.N + n];
          worst = std::max(worst, fabs(got - want) / (fabs(want) * 0.01 + 1e-3 * rmax));
        }
      printf("%s %-6s check %s (worst err/tol %.3f)\n", c.name, vs[v].name, worst <= 1.0 ? "OK" : "FAIL", worst);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < 5; ++r)
      for (size_t v = 0; v < vs.size(); ++v) {
        for (int w = 0; w < 3; ++w) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 20; ++i) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tf[v].push_back(flop * 20 / (ms * 1e-3) / 1e12);
      }
    for (size_t v = 0; v < vs.size(); ++v) {
      auto t = tf[v];
      std::sort(t.begin(), t.end());
      printf("%s %-6s TF/s best %.1f median %.1f\n", c.name, vs[v].name, t.back(), t[t.size() / 2]);
    }
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  return 0;
}
