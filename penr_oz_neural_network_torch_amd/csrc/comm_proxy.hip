// Collective-footprint proxy for one-GPU measurements of the data-parallel step (VERDICT r3
// missing #1). A ring all-reduce over xGMI runs as one persistent workgroup per channel on the
// communicator's stream, holding its CU for the whole collective while it moves the bucket at
// link speed and polls flags in between. On one GPU there is no second rank to talk to (RCCL
// refuses two ranks on one device and a 1-rank all-reduce launches nothing), so this kernel
// reproduces that FOOTPRINT instead: `wgs` workgroups (256 threads, few VGPRs — no GEMM tile can
// share their CU, as with the real channel kernels) stay resident for the modelled duration of the
// collective, streaming a scratch buffer at the modelled per-channel rate and sleeping between
// chunks. The trainer's bucket schedule, events and waits run unchanged on top (PZ_COMM=proxy).
#include <cstdint>

#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

__global__ void __launch_bounds__(256) comm_proxy_kernel(f32x4_t* __restrict__ scratch, int chunk4, uint64_t ticks,
                                                         uint64_t step_ticks) {
  // s_memrealtime: the 100 MHz constant clock (10 ns ticks), read by every wave for itself — the
  // waves of a workgroup exit independently (no barrier), within a few ticks of each other
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  f32x4_t* p = scratch + static_cast<int64_t>(blockIdx.x) * chunk4;
  uint64_t next = t0;
  int i = static_cast<int>(threadIdx.x);
  for (;;) {
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (now - t0 >= ticks) break;
    if (now >= next) {  // one 4 KiB chunk per step: read, modify, write back (vector memory only)
      f32x4_t v = __builtin_nontemporal_load(p + i);
      v += 1.0f;
      __builtin_nontemporal_store(v, p + i);
      i += 256;
      if (i >= chunk4) i = static_cast<int>(threadIdx.x);
      next += step_ticks;
    } else {
      __builtin_amdgcn_s_sleep(4);
    }
  }
}

}  // namespace

hipError_t comm_proxy(void* scratch, int wgs, int chunk_bytes, double us, double step_us, hipStream_t s) {
  if (wgs <= 0 || us <= 0.0) return hipSuccess;
  const int chunk4 = chunk_bytes / 16;
  if (chunk4 < 256) return hipErrorInvalidValue;
  const uint64_t ticks = static_cast<uint64_t>(us * 100.0);
  const uint64_t step = static_cast<uint64_t>(step_us * 100.0 > 1.0 ? step_us * 100.0 : 1.0);
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(wgs), dim3(256), 0, s, static_cast<f32x4_t*>(scratch), chunk4, ticks, step);
  return hipGetLastError();
}

}  // namespace pz
