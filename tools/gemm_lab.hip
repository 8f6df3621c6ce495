// Stand-alone GEMM main-loop laboratory: compiles ONLY the gemm_mfma variants listed below
// (seconds instead of the library's minutes), checks each against a naive fp32 reference on
// sampled rows, and times them in interleaved rounds on uniform [-1, 1) bf16 operands
// (guide §5.4 rules 24/25). Plain-store epilogue (EPI_STORE), the step's shapes.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I penr_oz_neural_network_torch_amd/csrc \
//         tools/gemm_lab.hip -o tools/gemm_lab && tools/gemm_lab [case ...]
#define PZ_GEMM_LAB 1
#include "../penr_oz_neural_network_torch_amd/csrc/gemm_mfma.hip"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
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

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(mix32(static_cast<uint32_t>(i) ^ seed) + static_cast<uint32_t>(i >> 32));
    p[i] = f2bf(static_cast<float>(h >> 8) * (2.f / 16777216.f) - 1.f);
  }
}

// reference rows m = r * stride: C[r][n] = sum_k A(m, k) B(k, n)
__global__ void ref_rows(const uint16_t* A, const uint16_t* B, float* R, int N, int K, int64_t lda, int64_t ldb,
                         int akc, int bkc, int stride) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = static_cast<int64_t>(blockIdx.y) * stride;
  if (n >= N) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) {
    const float a = bf2f(akc ? A[m * lda + k] : A[static_cast<int64_t>(k) * lda + m]);
    const float b = bf2f(bkc ? B[static_cast<int64_t>(n) * ldb + k] : B[static_cast<int64_t>(k) * ldb + n]);
    acc += a * b;
  }
  R[static_cast<int64_t>(blockIdx.y) * N + n] = acc;
}

typedef hipError_t (*LaunchFn)(const GemmArgs&, hipStream_t);
struct Variant {
  const char* name;
  LaunchFn fn;
  int split = 1;
};

#define PZ_VARIANTS(AKC, BKC, OUT)                                                   \
  {                                                                                  \
    {"buf", launch_cfg<256, 256, 2, 4, AKC, BKC, OUT, uint16_t, 6>},                 \
        {"bk64g0buf", launch_cfg<256, 256, 2, 4, AKC, BKC, OUT, uint16_t, 30>},      \
  }

struct Case {
  const char* name;
  int M, N, K;
  bool akc, bkc, f32out;
};

static std::vector<Variant> variants_for(const Case& c) {
  if (c.akc && !c.bkc && !c.f32out) {
    std::vector<Variant> v = PZ_VARIANTS(true, false, uint16_t);
    if (c.N <= 1024) {  // skinny forward (fwd_L3): split-K 2 (library) vs 256x128 tiles
      v.push_back({"bk64_s2", launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30>, 2});
      v.push_back({"t256x128", launch_cfg<256, 128, 4, 2, true, false, uint16_t, uint16_t, 6>});
      v.push_back({"t256x128bk64", launch_cfg<256, 128, 4, 2, true, false, uint16_t, uint16_t, 30>});
    }
    return v;
  }
  if (c.akc && c.bkc && !c.f32out) {
    std::vector<Variant> v = PZ_VARIANTS(true, true, uint16_t);
    v.push_back({"m32x32", launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 41>});
    return v;
  }
  if (!c.akc && !c.bkc && c.f32out) {
    std::vector<Variant> v = PZ_VARIANTS(false, false, float);
    if (c.N <= 1024 || c.M <= 1024) {  // skinny dW: the library's split-K 4 plan (VAR 30)
      v.push_back({"bk64_s4", launch_cfg<256, 256, 2, 4, false, false, float, uint16_t, 30>, 4});
      v.push_back({"bk64_s2", launch_cfg<256, 256, 2, 4, false, false, float, uint16_t, 30>, 2});
    }
    return v;
  }
  printf("no variants for layout\n");
  exit(1);
}

int main(int argc, char** argv) {
  const int B = 8192;
  std::vector<Case> cases = {
      {"fwd_L2", B, 4096, 4096, true, false, false}, {"dX_L2", B, 4096, 4096, true, true, false},
      {"dW_L2", 4096, 4096, B, false, false, true},  {"fwd_L1", B, 4096, 1024, true, false, false},
      {"dX_L3", B, 4096, 1024, true, true, false},   {"fwd_L3", B, 1024, 4096, true, false, false},
      {"dW_L3", 4096, 1024, B, false, false, true},  {"dW_L1", 1024, 4096, B, false, false, true},
      // same per-workgroup work as dW_L3 split 4 (256 tiles x K 2048), no reduction
      {"dW_sq2k", 4096, 4096, 2048, false, false, true},
  };
  const int rounds = getenv("LAB_ROUNDS") ? atoi(getenv("LAB_ROUNDS")) : 5, iters = 20;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Case& c : cases) {
    if (argc > 1) {
      bool want = false;
      for (int i = 1; i < argc; ++i) want |= strcmp(argv[i], c.name) == 0;
      if (!want) continue;
    }
    const int64_t na = static_cast<int64_t>(c.M) * c.K, nb = static_cast<int64_t>(c.N) * c.K;
    const int64_t nc = static_cast<int64_t>(c.M) * c.N;
    uint16_t *A, *Bm;
    void* C;
    float* R;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&Bm, nb * 2));
    CK(hipMalloc(&C, nc * (c.f32out ? 4 : 2)));
    const int stride = 61, nref = (c.M + stride - 1) / stride;
    CK(hipMalloc(&R, static_cast<int64_t>(nref) * c.N * 4));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, A, na, 12345u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, Bm, nb, 777u);
    const int64_t lda = c.akc ? c.K : c.M, ldb = c.bkc ? c.K : c.N;
    hipLaunchKernelGGL(ref_rows, dim3((c.N + 255) / 256, nref), dim3(256), 0, st, A, Bm, R, c.N, c.K, lda, ldb,
                       c.akc, c.bkc, stride);
    std::vector<float> ref(static_cast<size_t>(nref) * c.N);
    CK(hipMemcpyAsync(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));

    GemmArgs p{};
    p.A = A; p.B = Bm; p.C = C;
    p.M = c.M; p.N = c.N; p.K = c.K;
    p.lda = lda; p.ldb = ldb; p.ldc = c.N;
    p.a_kc = c.akc; p.b_kc = c.bkc;
    p.in_dtype = DT_BF16;
    p.out_dtype = c.f32out ? DT_F32 : DT_BF16;
    p.alpha = 1.f;
    p.epi_mode = EPI_STORE;
    p.idx_ld = c.N;
    p.split_k = 1;
    float* ws;
    int* counters;
    CK(hipMalloc(&ws, nc * 4 * 4 + (1 << 20)));
    CK(hipMalloc(&counters, 1 << 16));
    CK(hipMemset(counters, 0, 1 << 16));
    p.ws = ws;
    p.counters = counters;

    auto vs = variants_for(c);
    std::vector<std::vector<double>> tf(vs.size());
    const double flop = 2.0 * c.M * c.N * c.K;
    // correctness first
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(hipMemsetAsync(C, 0, nc * (c.f32out ? 4 : 2), st));
      p.split_k = vs[v].split;
      CK(vs[v].fn(p, st));
      CK(hipStreamSynchronize(st));
      std::vector<char> out(nc * (c.f32out ? 4 : 2));
      CK(hipMemcpy(out.data(), C, out.size(), hipMemcpyDeviceToHost));
      double worst = 0.0;
      for (int r = 0; r < nref; ++r) {
        const int64_t m = static_cast<int64_t>(r) * stride;
        for (int n = 0; n < c.N; ++n) {
          float got;
          if (c.f32out) {
            memcpy(&got, out.data() + (m * c.N + n) * 4, 4);
          } else {
            uint16_t h;
            memcpy(&h, out.data() + (m * c.N + n) * 2, 2);
            uint32_t u = static_cast<uint32_t>(h) << 16;
            memcpy(&got, &u, 4);
          }
          const double want = ref[static_cast<size_t>(r) * c.N + n];
          const double err = fabs(got - want) / (fabs(want) * 0.01 + 0.05);
          worst = std::max(worst, err);
        }
      }
      if (v == 0 || worst > 1.0) printf("%s %-10s check %s (worst err/tol %.3f)\n", c.name, vs[v].name, worst <= 1.0 ? "OK" : "FAIL", worst);
      fflush(stdout);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
      for (size_t v = 0; v < vs.size(); ++v) {
        p.split_k = vs[v].split;
        for (int w = 0; w < 3; ++w) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < iters; ++i) CK(vs[v].fn(p, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tf[v].push_back(flop * iters / (ms * 1e-3) / 1e12);
      }
    }
    for (size_t v = 0; v < vs.size(); ++v) {
      auto t = tf[v];
      std::sort(t.begin(), t.end());
      printf("%s %-10s TF/s best %.1f median %.1f\n", c.name, vs[v].name, t.back(), t[t.size() / 2]);
    }
    fflush(stdout);
    CK(hipFree(A));
    CK(hipFree(Bm));
    CK(hipFree(C));
    CK(hipFree(R));
    CK(hipFree(ws));
    CK(hipFree(counters));
  }
  return 0;
}
