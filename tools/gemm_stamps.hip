// Where a GEMM tile's time goes: builds the library's gemm_mfma kernel with PZ_GEMM_STAMPS (per
// workgroup s_memrealtime stamps at entry / first K step landed / main loop done / epilogue start /
// end, 10 ns resolution) and prints, for the mlp4 step's shapes with the trainer's REAL epilogues,
// the median per-phase time of a workgroup and how the workgroups were spread over time
// (dispatch waves). Diagnostic build only; the library never compiles the stamps.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I penr_oz_neural_network_torch_amd/csrc \
//         tools/gemm_stamps.hip -o scratch/gemm_stamps && scratch/gemm_stamps [case ...]
#define PZ_GEMM_LAB 1
#define PZ_GEMM_STAMPS 1
#include "../penr_oz_neural_network_torch_amd/csrc/gemm_mfma.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace pz;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const uint32_t h = mix32(mix32(static_cast<uint32_t>(i) ^ seed) + static_cast<uint32_t>(i >> 32));
    p[i] = f2bf(static_cast<float>(h >> 8) * (2.f / 16777216.f) - 1.f);
  }
}

typedef hipError_t (*LaunchFn)(const GemmArgs&, hipStream_t);

struct Case {
  const char* name;
  int M, N, K;
  bool akc, bkc, f32out;
  int mode;  // 0 plain store, 1 stage-0 forward (bias, ReLU, dropout, bitmask), 2 drop-ReLU-drop forward,
             // 3 backward (bitmask ReLU derivative, dropout scales, bias-grad column sums), 4-6 see below
  int split;
  LaunchFn fn;
  int f8 = 0;  // 0 bf16, 1 e4m3 x e4m3 (forward), 2 e5m2 x e4m3 (backward dX), 3 e4m3 x e5m2 (dW)
  int tile_m = 0, tile_n = 0;  // 0: 256x256 (128x128 for the small fp8 config)
  int wt = 0;                  // write-through (sc1) epilogue stores (GemmArgs::store_wt)
};

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int B = 8192;
  using F = LaunchFn;
  // the library's dispatch (gemm_mfma.hip: launch_bk64_256 / launch_fp8): each stage's GEMM with its
  // specialised epilogue (EK_*); *_gen = the same GEMM on the generic epilogue (A/B)
  constexpr int R = EK_RELU, S = EK_STORE, M = EK_BWD_MASK, G = EK_ANY;
  constexpr int F1 = EK_F_RELU_POST, F2 = EK_F_RELU_PREPOST, F3 = EK_F_PRE;  // fixed forward kinds
  std::vector<Case> cases = {
      {"fwd_L1", B, 4096, 1024, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      // stage-0 epilogue decomposition (EK_RELU kernel): 9 nothing, 8 bias, 7 ReLU, 4 bias+ReLU+bitmask, 5 bias+ReLU+dropout (no bitmask)
      {"fwdL1_m9", B, 4096, 1024, true, false, false, 9, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwdL1_m8", B, 4096, 1024, true, false, false, 8, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwdL1_m7", B, 4096, 1024, true, false, false, 7, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwdL1_m4", B, 4096, 1024, true, false, false, 4, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwdL1_m5", B, 4096, 1024, true, false, false, 5, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwdL1_st", B, 4096, 1024, true, false, false, 0, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, S>},
      // the trainer's three forward stages on EK_RELU vs their fixed kinds (same arguments)
      {"fwd_L1_s0_fx", B, 4096, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, F1>},
      {"fwd_L2_fx", B, 4096, 4096, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, F2>},
      {"fwd_L3_fx", B, 1024, 4096, true, false, false, 11, 2, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, F3>},
      {"f8n_fwd_L1", B, 8192, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, R>, 1},
      {"f8n_fwd_L1_fx", B, 8192, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, F1>, 1},
      {"f8n_fwd_L2", B, 1024, 8192, true, false, false, 11, 2, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, R>, 1},
      {"f8n_fwd_L2_fx", B, 1024, 8192, true, false, false, 11, 2, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, F3>, 1},
      {"fwd_L1_s0", B, 4096, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      // two co-resident 4-wave workgroups per CU on 256x128 tiles (VAR 7: 3-slot 32-deep buffer ring)
      {"fwd_L1_s0_2wg", B, 4096, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 7, R>, 0, 256, 128},
      {"fwd_L2_2wg", B, 4096, 4096, true, false, false, 2, 1, (F)launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 7, R>, 0, 256, 128},
      {"fwd_L3_2wg", B, 1024, 4096, true, false, false, 11, 1, (F)launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 7, R>, 0, 256, 128},
      {"dX_L3_2wg", B, 4096, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 7, M>, 0, 256, 128},
      {"dX_L2_2wg", B, 4096, 4096, true, true, false, 3, 1, (F)launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 7, M>, 0, 256, 128},
      {"dW_L3_2wg", 4096, 1024, B, false, false, false, 0, 1, (F)launch_cfg<256, 128, 2, 2, false, false, uint16_t, uint16_t, 7, S>, 0, 256, 128},
      {"dW_L1_2wg", 1024, 4096, B, false, false, false, 0, 1, (F)launch_cfg<256, 128, 2, 2, false, false, uint16_t, uint16_t, 7, S>, 0, 256, 128},
      {"dW_L2_2wg", 4096, 4096, B, false, false, false, 0, 1, (F)launch_cfg<256, 128, 2, 2, false, false, uint16_t, uint16_t, 7, S>, 0, 256, 128},
      {"fwd_L1_gen", B, 4096, 1024, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, G>},
      {"fwd_L2", B, 4096, 4096, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"fwd_L3", B, 1024, 4096, true, false, false, 11, 2, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, R>},
      {"dX_L3", B, 4096, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 30, M>},
      {"dX_L3_gen", B, 4096, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 30, G>},
      {"dX_L2", B, 4096, 4096, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 30, M>},
      {"dW_L3", 4096, 1024, B, false, false, false, 0, 4, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 30, S>},
      {"dW_L1", 1024, 4096, B, false, false, false, 0, 4, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 30, S>},
      {"dW_L2", 4096, 4096, B, false, false, false, 0, 1, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 30, S>},
      // VAR 33: VAR 30 without the s_setprio bracket around the MFMA block (lab A/B)
      {"dX_L2_np", B, 4096, 4096, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 33, M>},
      {"fwd_L2_np", B, 4096, 4096, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 33, R>},
      {"dW_L2_np", 4096, 4096, B, false, false, false, 0, 1, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 33, S>},
      {"dW_L2_gen", 4096, 4096, B, false, false, false, 0, 1, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 30, G>},
      // the fp8 policy's GEMMs (mlp8192 [1024, 8192, 1024], batch 8192); operand bytes are
      // arbitrary (timing only)
      {"f8_fwd_L1", B, 8192, 1024, true, true, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 8, R>, 1},
      {"f8_fwd_L1_gen", B, 8192, 1024, true, true, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 8, G>, 1},
      {"f8_fwd_L2", B, 1024, 8192, true, true, false, 11, 1, (F)launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 8, R>, 1},
      {"f8_dX_L2", B, 8192, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 9, M>, 2},
      {"f8_dX_L2_gen", B, 8192, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 9, G>, 2},
      {"f8_dW_L2", 8192, 1024, B, false, false, false, 0, 2, (F)launch_cfg<256, 256, 2, 4, false, false, uint16_t, uint16_t, 14, S>, 3},
      // r4: the fp8 GEMMs on two 4-wave 256x128 workgroups per CU (VAR 16 / 17)
      {"f8n_fwd_L1_2wg", B, 8192, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 128, 2, 2, true, false, uint16_t, uint16_t, 16, F1>, 1, 256, 128},
      {"f8_dX_L2_2wg", B, 8192, 1024, true, true, false, 3, 1, (F)launch_cfg<256, 128, 2, 2, true, true, uint16_t, uint16_t, 17, M>, 2, 256, 128},
      // r4: write-through (sc1) epilogue stores
      {"fwd_L2_wt", B, 4096, 4096, true, false, false, 2, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 30, F2>, 0, 0, 0, 1},
      {"dX_L2_wt", B, 4096, 4096, true, true, false, 3, 1, (F)launch_cfg<256, 256, 2, 4, true, true, uint16_t, uint16_t, 30, M>, 0, 0, 0, 1},
      {"f8n_fwd_L1_fx_wt", B, 8192, 1024, true, false, false, 1, 1, (F)launch_cfg<256, 256, 2, 4, true, false, uint16_t, uint16_t, 15, F1>, 1, 0, 0, 1},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // cases run in command-line order (repeats allowed: interleave A/B pairs against clock drift);
  // no arguments: the whole table
  std::vector<const Case*> order;
  if (argc > 1) {
    for (int i = 1; i < argc; ++i)
      for (const Case& c : cases)
        if (strcmp(argv[i], c.name) == 0) order.push_back(&c);
  } else {
    for (const Case& c : cases) order.push_back(&c);
  }
  for (const Case* cp : order) {
    const Case& c = *cp;
    const int64_t na = static_cast<int64_t>(c.M) * c.K, nb = static_cast<int64_t>(c.N) * c.K;
    const int64_t nc = static_cast<int64_t>(c.M) * c.N;
    uint16_t *A, *Bm, *C;
    float *bias, *colsum;
    uint8_t* mask;
    CK(hipMalloc(&A, na * 2));
    CK(hipMalloc(&Bm, nb * 2));
    CK(hipMalloc(&C, nc * 2));
    CK(hipMalloc(&bias, c.N * 4));
    CK(hipMalloc(&colsum, c.N * 4));
    const int64_t ldmask = (c.N + 255) / 256 * 32;  // tile-blocked (GemmArgs::mask)
    const int64_t mrows = (c.M + 255) / 256 * 256;
    CK(hipMalloc(&mask, mrows * ldmask));
    CK(hipMemset(bias, 0, c.N * 4));
    CK(hipMemset(colsum, 0, c.N * 4));
    CK(hipMemset(mask, 0x5A, mrows * ldmask));
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, A, na, 12345u);
    hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, st, Bm, nb, 777u);
    GemmArgs p{};
    p.A = A; p.B = Bm; p.C = C;
    p.M = c.M; p.N = c.N; p.K = c.K;
    p.lda = c.akc ? c.K : c.M;
    p.ldb = c.bkc ? c.K : c.N;
    p.ldc = c.N;
    p.a_kc = c.akc; p.b_kc = c.bkc;
    p.in_dtype = c.f8 ? DT_FP8 : DT_BF16;
    p.a_fmt = c.f8 == 2 ? 1 : 0;
    p.b_fmt = c.f8 == 3 ? 1 : 0;
    p.out_dtype = DT_BF16;
    p.alpha = 1.f;
    p.idx_ld = c.N;
    p.epi_mode = EPI_STORE;
    EpiSpec e{};
    e.act = ACT_NONE;
    e.scale = e.scale64 = 1.25f;
    e.inv_scale = e.inv_scale64 = 0.8f;
    e.thresh16 = 13107;  // p = 0.2
    e.key_pre = 0x1234567u;
    e.key_post = 0x89abcdefu;
    if (c.mode == 1) {  // stage 0: bias, ReLU, dropout after the ReLU, bitmask for the dX GEMM
      p.epi_mode = EPI_FWD; p.bias = bias; e.act = ACT_RELU; e.drop_post = 1; p.mask = mask; p.ldmask = ldmask;
    } else if (c.mode == 2) {  // hidden ReLU stage: dropout, ReLU, dropout (+ bitmask)
      p.epi_mode = EPI_FWD; p.bias = bias; e.act = ACT_RELU; e.drop_pre = 1; e.drop_post = 1; p.mask = mask;
      p.ldmask = ldmask;
    } else if (c.mode == 4) {
      p.epi_mode = EPI_FWD; p.bias = bias; e.act = ACT_RELU; p.mask = mask; p.ldmask = ldmask;
    } else if (c.mode == 5) {
      p.epi_mode = EPI_FWD; p.bias = bias; e.act = ACT_RELU; e.drop_post = 1;
    } else if (c.mode == 6) {
      p.epi_mode = EPI_FWD; p.bias = bias; e.act = ACT_RELU; e.drop_pre = 1; e.drop_post = 1;
    } else if (c.mode == 11) {  // logits stage: bias + dropout of the linear output, no activation
      p.epi_mode = EPI_FWD; p.bias = bias; e.drop_pre = 1;
    } else if (c.mode == 7) {
      p.epi_mode = EPI_FWD; e.act = ACT_RELU;
    } else if (c.mode == 8) {
      p.epi_mode = EPI_FWD; p.bias = bias;
    } else if (c.mode == 9) {
      p.epi_mode = EPI_FWD;
    } else if (c.mode == 3) {  // backward through a ReLU stage read from its bitmask + bias grad
      p.epi_mode = EPI_BWD; e.act = ACT_RELU; e.drop_pre = 1; e.drop_post = 1; p.mask = mask; p.ldmask = ldmask;
      p.colsum = colsum;
    }
    p.epi = e;
    p.store_wt = c.wt;
    p.prio = 1;
    int bm = c.fn == (F)launch_cfg<128, 128, 2, 2, true, true, uint16_t, uint16_t, 8, R> ? 128 : 256, bn = bm;
    if (c.tile_m) bm = c.tile_m, bn = c.tile_n;
    const int tiles = ((c.M + bm - 1) / bm) * ((c.N + bn - 1) / bn);
    const int nwg = tiles * c.split;
    p.split_k = c.split;
    float* ws = nullptr;
    const int64_t slab_floats = c.split > 1 ? static_cast<int64_t>(tiles) * c.split * 65536 : 0;
    if (slab_floats) CK(hipMalloc(&ws, slab_floats * 4));
    int* counters;
    CK(hipMalloc(&counters, tiles * 4));
    CK(hipMemset(counters, 0, tiles * 4));
    uint64_t* stamps;
    CK(hipMalloc(&stamps, static_cast<int64_t>(nwg) * 64));
    CK(hipMemset(stamps, 0, static_cast<int64_t>(nwg) * 64));
    p.ws = ws;
    p.counters = counters;
    p.dbg = stamps;
    for (int w = 0; w < 5; ++w) CK(c.fn(p, st));  // warm-up (clocks, caches)
    CK(hipMemsetAsync(stamps, 0, static_cast<int64_t>(nwg) * 64, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    CK(c.fn(p, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint64_t> h(static_cast<size_t>(nwg) * 8);
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull, t1 = 0;
    for (int w = 0; w < nwg; ++w) {
      t0 = std::min(t0, h[8 * w + 0]);
      t1 = std::max(t1, std::max(h[8 * w + 4], h[8 * w + 2]));
    }
    std::vector<double> pro, loop, red, epi, tot, start, emath, eissue, edrain;
    for (int w = 0; w < nwg; ++w) {
      const uint64_t* s = &h[8 * w];
      const bool finished = s[4] != 0;  // non-last split-K slices return before stamp 4
      pro.push_back((s[1] - s[0]) * 0.01);
      loop.push_back((s[2] - s[1]) * 0.01);
      start.push_back((s[0] - t0) * 0.01);
      if (finished) {
        red.push_back((s[3] - s[2]) * 0.01);
        epi.push_back((s[4] - s[3]) * 0.01);
        if (s[5] && s[6]) {
          emath.push_back((s[5] - s[3]) * 0.01);
          eissue.push_back((s[6] - s[5]) * 0.01);
          edrain.push_back((s[4] - s[6]) * 0.01);
        }
        tot.push_back((s[4] - s[0]) * 0.01);
      }
    }
    std::vector<double> st_sorted = start;
    std::sort(st_sorted.begin(), st_sorted.end());
    const double flop = 2.0 * c.M * c.N * c.K;
    printf("%-13s %5d WGs  kernel %.1f us (%.0f TF/s)  span %.1f us | per WG median: prologue %.2f  main loop %.2f "
           "(%.3f us/K-step)  split-K %.2f  epilogue %.2f  total %.2f | start p50 %.1f p90 %.1f max %.1f us\n",
           c.name, nwg, ms * 1e3, flop / (ms * 1e-3) / 1e12, (t1 - t0) * 0.01, med(pro), med(loop),
           med(loop) / (c.K / 64 / c.split), med(red), med(epi), med(tot), st_sorted[st_sorted.size() / 2],
           st_sorted[st_sorted.size() * 9 / 10], st_sorted.back());
    if (!emath.empty()) printf("    epilogue (wave 0): stage math + LDS image %.2f  image read + stores issued %.2f  store drain %.2f\n", med(emath), med(eissue), med(edrain));
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(Bm)); CK(hipFree(C)); CK(hipFree(bias)); CK(hipFree(colsum)); CK(hipFree(mask));
    if (ws) CK(hipFree(ws));
    CK(hipFree(counters)); CK(hipFree(stamps));
  }
  return 0;
}
