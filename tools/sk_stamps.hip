// Where the persistent stream-K GEMM's time goes (csrc/gemm_sk.hip built with PZ_GEMM_STAMPS):
// per workgroup and work unit, s_memrealtime stamps (100 MHz) at unit start / main loop done /
// slab handed off / fold done / epilogue done. Prints per CU budget: the makespan, the spread of
// the workgroups' end times, and medians per unit kind (data-parallel tile, stream-K partial that
// hands off, stream-K partial that folds): main-loop time per 64-deep K step, hand-off, fold and
// epilogue. Diagnostic build only; the library never compiles the stamps.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I penr_oz_neural_network_torch_amd/csrc \
//         tools/sk_stamps.hip -o tools/sk_stamps && tools/sk_stamps [cus ...]
#define PZ_GEMM_STAMPS 1
#include "../penr_oz_neural_network_torch_amd/csrc/gemm_sk.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace pz;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(mix32(static_cast<uint32_t>(i) ^ seed) + static_cast<uint32_t>(i >> 32));
    p[i] = f2bf(static_cast<float>(h >> 8) * (2.f / 16777216.f) - 1.f);
  }
}

static double med(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct Shape {
  const char* name;
  int M, N, K;
  bool akc, bkc;
};

int main(int argc, char** argv) {
  std::vector<int> budgets;
  for (int i = 1; i < argc; ++i) budgets.push_back(atoi(argv[i]));
  if (budgets.empty()) budgets = {256, 240, 224, 128};
  const Shape shapes[] = {{"dX_L2", 8192, 4096, 4096, true, true}, {"dW_L2", 4096, 4096, 8192, false, false},
                          {"fwd_L1", 8192, 4096, 1024, true, false}, {"dW_L1", 1024, 4096, 8192, false, false}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (const Shape& sh : shapes) {
    const int64_t na = static_cast<int64_t>(sh.M) * sh.K, nb = static_cast<int64_t>(sh.N) * sh.K;
    uint16_t *A, *B, *C;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&B, nb * 2));
    CK(hipMalloc(&C, static_cast<int64_t>(sh.M) * sh.N * 2));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, A, na, 12345u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, B, nb, 777u);
    for (int cus : budgets) {
      GemmArgs p{};
      p.A = A; p.B = B; p.C = C;
      p.M = sh.M; p.N = sh.N; p.K = sh.K;
      p.lda = sh.akc ? sh.K : sh.M;
      p.ldb = sh.bkc ? sh.K : sh.N;
      p.ldc = sh.N;
      p.a_kc = sh.akc; p.b_kc = sh.bkc;
      p.in_dtype = DT_BF16; p.out_dtype = DT_BF16;
      p.alpha = 1.f; p.idx_ld = sh.N; p.epi_mode = EPI_STORE;
      p.engine = 2; p.cus = cus;
      const SkSched sched = sk_plan(&p, 1);
      const int64_t nd = static_cast<int64_t>(sched.grid) * kSkStampUnits * 8;
      uint64_t* dbg;
      CK(hipMalloc(&dbg, nd * 8));
      p.dbg = dbg;
      float* ws = nullptr;
      int* tickets = nullptr;
      const int64_t wsf = sk_ws_floats(&p, 1);
      if (wsf > 0) CK(hipMalloc(&ws, wsf * 4));
      const int nt = std::max(1, sk_tickets(&p, 1));
      CK(hipMalloc(&tickets, nt * 4));
      CK(hipMemset(tickets, 0, nt * 4));
      for (int r = 0; r < 3; ++r) CK(gemm_sk(&p, 1, ws, tickets, st));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0, st));
      const int reps = 10;
      for (int r = 0; r < reps; ++r) CK(gemm_sk(&p, 1, ws, tickets, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double tflops = 2.0 * sh.M * sh.N * sh.K / (ms / reps * 1e-3) / 1e12;
      CK(hipMemset(dbg, 0, nd * 8));
      CK(gemm_sk(&p, 1, ws, tickets, st));
      CK(hipStreamSynchronize(st));
      std::vector<uint64_t> h(nd);
      CK(hipMemcpy(h.data(), dbg, nd * 8, hipMemcpyDeviceToHost));
      uint64_t t0 = ~0ull, tend = 0;
      for (int w = 0; w < sched.grid; ++w) {
        const uint64_t s = h[(static_cast<int64_t>(w) * kSkStampUnits) * 8];
        if (s) t0 = std::min(t0, s);
      }
      std::vector<double> ends, dp_step, dp_epi, skh_step, skh_hand, skf_step, skf_hand, skf_fold, skf_epi, gaps;
      int units = 0;
      for (int w = 0; w < sched.grid; ++w) {
        uint64_t last_end = 0, wend = 0;
        for (int u = 0; u < kSkStampUnits; ++u) {
          const uint64_t* q = &h[(static_cast<int64_t>(w) * kSkStampUnits + u) * 8];
          if (q[0] == 0) break;
          ++units;
          const uint64_t note = q[7];
          const bool partial = (note >> 63) & 1;
          const int kb = static_cast<int>((note >> 20) & 0xFFFFF), ke = static_cast<int>(note & 0xFFFFF);
          const double steps = std::max(1, ke - kb);
          const double main_us = (q[1] - q[0]) * 0.01;  // 100 MHz
          if (last_end) gaps.push_back((q[0] - last_end) * 0.01);
          if (!partial) {
            dp_step.push_back(main_us / steps);
            dp_epi.push_back((q[4] - q[3]) * 0.01);
            last_end = q[4];
          } else if (q[3] == 0) {  // handed its slab to another contributor
            skh_step.push_back(main_us / steps);
            skh_hand.push_back((q[2] - q[1]) * 0.01);
            last_end = q[2];
          } else {
            skf_step.push_back(main_us / steps);
            skf_hand.push_back((q[2] - q[1]) * 0.01);
            skf_fold.push_back((q[3] - q[2]) * 0.01);
            skf_epi.push_back((q[4] - q[3]) * 0.01);
            last_end = q[4];
          }
          wend = last_end;
        }
        if (wend) {
          ends.push_back((wend - t0) * 0.01);
          tend = std::max(tend, wend);
        }
      }
      std::sort(ends.begin(), ends.end());
      printf("%s cus %d: grid %d sk_tiles %d iters %d units %d | %.1f TF/s, launch %.1f us | stamped makespan %.1f us, "
             "WG end p10/p50/p90 %.1f/%.1f/%.1f\n",
             sh.name, cus, sched.grid, sched.sk_tiles, sched.iters, units, tflops, ms / reps * 1e3, (tend - t0) * 0.01,
             ends.empty() ? 0 : ends[ends.size() / 10], med(ends), ends.empty() ? 0 : ends[ends.size() * 9 / 10]);
      printf("   DP tile    n=%4zu  us/step %.3f  epilogue %.2f\n", dp_step.size(), med(dp_step), med(dp_epi));
      printf("   SK handoff n=%4zu  us/step %.3f  slab+ticket %.2f\n", skh_step.size(), med(skh_step), med(skh_hand));
      printf("   SK fold    n=%4zu  us/step %.3f  slab+ticket %.2f  fold %.2f  epilogue %.2f\n", skf_step.size(),
             med(skf_step), med(skf_hand), med(skf_fold), med(skf_epi));
      printf("   gap between units (prologue not counted in main) median %.2f us\n", med(gaps));
      CK(hipFree(dbg));
      if (ws) CK(hipFree(ws));
      CK(hipFree(tickets));
    }
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
  }
  return 0;
}
