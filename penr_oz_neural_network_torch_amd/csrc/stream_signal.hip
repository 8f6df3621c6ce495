// Device-side ordering between the trainer's compute stream and its optimizer stream.
//
// An event record on the compute stream that another stream waits on leaves the compute stream
// idle for ~7 us (tools/packet_gap.hip, profiles/r4_packet_gap.txt: a record alone ~3 us, a
// record with a cross-stream waiter ~7 us) — a marker packet for the command processor to retire
// and signal between two kernels. A one-wave kernel that bumps a counter costs the producer stream
// ~1.5 us instead; the consumer stream runs a one-wave kernel that polls the counter (vector
// atomic loads, s_sleep between polls) before its next kernel. Memory ordering: the kernels before
// the signal have completed (in-order stream) and the release increment at agent scope follows
// them; the waiter's acquire load and the next kernel's start-of-kernel acquire make their results
// visible to the consumer. Every poll loop is bounded by a wall-clock limit so the grid always
// drains; a timeout is recorded in the slot's second word for the host to check.
//
// Measured, not kept (PZ_DEV_SIG=1, off by default): mlp4 1.49-1.51 ms vs 1.09 with events
// (profiles/r4_step_timeline_devsig.txt). The waiter wave is resident for the whole forward and
// backward and holds one CU, so every 256x256-tile GEMM (tile counts multiples of 256 CUs) needs a
// whole extra round of workgroups: L2 fwd 286 vs 198 us, dW2 331 vs 190, dX2 267 vs 193. The poll
// rate does not matter (s_sleep 8 and 64 alike); the CU does. The same quantisation applies to any
// resident kernel beside the GEMMs (the collective-footprint proxy, RCCL channel kernels).
#include <cstdint>

#include "pz_common.h"
#include "pz_kernels.h"

namespace pz {
namespace {

constexpr int kSlotWords = 32;  // one 128-byte line per counter

__global__ void __launch_bounds__(64) signal_set_kernel(unsigned* __restrict__ ctr) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) signal_wait_kernel(unsigned* __restrict__ ctr, unsigned target, uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  // relaxed polls (a coherent load, nothing else): an acquire load would invalidate this XCD's L2
  // on every poll and starve the GEMMs running beside the waiter (r4: mlp4 step 1.53 vs 1.11 ms);
  // one acquire fence once the count is reached
  for (;;) {
    const unsigned v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (static_cast<int>(v - target) >= 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) {
      __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

}  // namespace

hipError_t signal_set(unsigned* ctr, int slot, hipStream_t s) {
  hipLaunchKernelGGL(signal_set_kernel, dim3(1), dim3(64), 0, s, ctr + static_cast<int64_t>(slot) * kSlotWords);
  return hipGetLastError();
}

hipError_t signal_wait(unsigned* ctr, int slot, unsigned target, double timeout_us, hipStream_t s) {
  const uint64_t ticks = static_cast<uint64_t>(timeout_us * 100.0);
  hipLaunchKernelGGL(signal_wait_kernel, dim3(1), dim3(64), 0, s, ctr + static_cast<int64_t>(slot) * kSlotWords,
                     target, ticks);
  return hipGetLastError();
}

}  // namespace pz
