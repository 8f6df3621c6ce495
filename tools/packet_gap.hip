// Inter-kernel gap on one stream for the ways the trainer can order its two streams
// (r4 step trace: ~7 us of idle compute stream around each cross-stream event).
//
//   plain    work; work                                      (kernel-to-kernel baseline)
//   rec_dev  work; record(ReleaseToDevice event); work
//   rec_sys  work; record(default event); work
//   wait_ok  work; wait(event already complete, other stream); work
//   spin     work; 1-wave kernel that reads an already-set counter; work
//   sig      work that bumps a counter from every workgroup at its end (vector atomic); work
//   xrec     rec_dev, and the other stream waits on that record then runs a short kernel
//   xwait    work; wait(event the other stream records after a short kernel, complete by then but
//            not when enqueued); work
//   xspin    sig, and the other stream runs spin_wait on the counter then a short kernel
//   xsig     work; one-wave kernel that bumps the counter once (csrc/stream_signal.hip's scheme);
//            the other stream runs spin_wait on it then a short kernel
//
// Each case runs REPS pairs back to back; reported: (case time - plain time) / REPS per pair.
// Build: hipcc --offload-arch=gfx950 -O3 tools/packet_gap.hip -o tools/packet_gap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

// ~40 us of ALU work over 2048 workgroups (enough to fill the chip several times)
__global__ void __launch_bounds__(256) work(float* out, int iters, unsigned* cnt) {
  float a = threadIdx.x * 1e-3f, b = blockIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
    a = __builtin_fmaf(a, 0.999f, b);
    b = __builtin_fmaf(b, 0.999f, a);
  }
  if (a == 12345.f) out[blockIdx.x] = b;  // keep the loop
  if (cnt != nullptr) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one wave: wait (bounded: 10 ms) until *cnt >= target
__global__ void __launch_bounds__(64) bump(unsigned* cnt) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) spin_wait(const unsigned* cnt, unsigned target) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000ull) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 4000;
  const int grid = 2048;
  float* out;
  unsigned* cnt;
  CK(hipMalloc(&out, grid * sizeof(float)));
  CK(hipMalloc(&cnt, sizeof(unsigned)));
  CK(hipMemset(cnt, 0, sizeof(unsigned)));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t t_a, t_b, e_dev, e_sys, e_done;
  CK(hipEventCreate(&t_a));
  CK(hipEventCreate(&t_b));
  CK(hipEventCreateWithFlags(&e_dev, hipEventDisableTiming | hipEventReleaseToDevice));
  CK(hipEventCreateWithFlags(&e_sys, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e_done, hipEventDisableTiming));
  CK(hipEventRecord(e_done, s1));
  CK(hipDeviceSynchronize());

  const char* names[] = {"plain", "rec_dev", "rec_sys", "wait_ok", "spin", "sig", "xrec", "xwait", "xspin", "xsig"};
  constexpr int NC = 10;
  double ms[NC] = {0};
  for (int round = 0; round < 3; ++round) {
    for (int c = 0; c < NC; ++c) {
      CK(hipMemset(cnt, 0, sizeof(unsigned)));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t_a, s0));
      for (int r = 0; r < reps; ++r) {
        if (c == 7) {
          work<<<64, 256, 0, s1>>>(out, 16, nullptr);
          CK(hipEventRecord(e_dev, s1));
        }
        work<<<grid, 256, 0, s0>>>(out, iters, (c == 5 || c == 8) ? cnt : nullptr);
        if (c == 1 || c == 6) CK(hipEventRecord(e_dev, s0));
        if (c == 6) {
          CK(hipStreamWaitEvent(s1, e_dev, 0));
          work<<<64, 256, 0, s1>>>(out, 16, nullptr);
        }
        if (c == 7) CK(hipStreamWaitEvent(s0, e_dev, 0));
        if (c == 8) {
          spin_wait<<<1, 64, 0, s1>>>(cnt, (unsigned)((r + 1) * grid));
          work<<<64, 256, 0, s1>>>(out, 16, nullptr);
        }
        if (c == 9) {
          bump<<<1, 64, 0, s0>>>(cnt);
          spin_wait<<<1, 64, 0, s1>>>(cnt, (unsigned)(r + 1));
          work<<<64, 256, 0, s1>>>(out, 16, nullptr);
        }
        if (c == 2) CK(hipEventRecord(e_sys, s0));
        if (c == 3) CK(hipStreamWaitEvent(s0, e_done, 0));
        if (c == 4) spin_wait<<<1, 64, 0, s0>>>(cnt, 0u);
        work<<<grid, 256, 0, s0>>>(out, iters, nullptr);
      }
      CK(hipEventRecord(t_b, s0));
      CK(hipEventSynchronize(t_b));
      CK(hipDeviceSynchronize());
      float t = 0.f;
      CK(hipEventElapsedTime(&t, t_a, t_b));
      if (round > 0) ms[c] += t;  // round 0 warms up
    }
  }
  unsigned h = 0;
  CK(hipMemcpy(&h, cnt, sizeof(unsigned), hipMemcpyDeviceToHost));
  std::printf("# packet_gap: reps %d, work %.1f us/kernel (plain pair / 2), last counter %u (expect %d)\n", reps,
              ms[0] / 2 / reps * 1000.0 / 2, h, reps);
  for (int c = 0; c < NC; ++c)
    std::printf("%-8s pair %.2f us   extra vs plain %+.2f us\n", names[c], ms[c] / 2 / reps * 1000.0,
                (ms[c] - ms[0]) / 2 / reps * 1000.0);
  return 0;
}
