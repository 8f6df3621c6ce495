// What a cross-stream dependency costs the stream that PRODUCES it, and what the alternatives cost.
// The trainer orders its side-stream optimizer launches behind compute-stream kernels with event
// record / stream-wait pairs; the r5 step trace shows ~7-9 us of compute-stream idle at each record
// and at each wait, although consecutive kernels on one stream start back to back.
//
// Each case launches  busy1 -> busy2  on the main stream, plus a small kernel on a side stream
// that must run after busy1. Every workgroup stamps its start / end (s_memrealtime, 100 MHz); the
// printed gap is busy2's first start minus busy1's last end (main-stream idle), and the side
// kernel's start minus busy1's end.
//   none     no dependency (baseline gap)
//   event    hipEventRecord(main) after busy1 + hipStreamWaitEvent(side) (the trainer's ordering)
//   flag     busy1's last workgroup stores a flag (release, system scope); the side stream waits
//            with hipStreamWaitValue32 — nothing extra is enqueued on the main stream
//   mwait    main waits (hipStreamWaitEvent) on an event the side stream recorded long before
//   tiny     a one-workgroup kernel on the main stream stores the flag after busy1; the side
//            stream waits with hipStreamWaitValue32
//   write    hipStreamWriteValue32 on the main stream after busy1; hipStreamWaitValue32 on the side
//   vwait    main waits with hipStreamWaitValue32 on a flag a side-stream kernel stored long before
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_sig_lab.hip -o tools/stream_sig_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ inline uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }

// stamps[2*blockIdx] = start, [2*blockIdx+1] = end; flag != nullptr: the last workgroup to finish
// (ticket) stores `val` into *flag after every workgroup's stores are visible
__global__ void __launch_bounds__(256) busy(float* out, int iters, uint64_t* stamps, int* ctr, uint32_t* flag,
                                            uint32_t val) {
  const uint64_t t0 = rt();
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = __builtin_fmaf(a, b, 1e-7f);
  out[blockIdx.x * 256 + threadIdx.x] = a;
  __shared__ int last;
  if (flag != nullptr) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      const int prev = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      last = prev == static_cast<int>(gridDim.x) - 1;
      if (last) {
        __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = rt();
  }
}

__global__ void set_flag(uint32_t* flag, uint32_t val) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Span {
  uint64_t s, e;
};
static Span span(const std::vector<uint64_t>& h, int off, int n) {
  Span r{~0ull, 0};
  for (int i = 0; i < n; ++i) {
    r.s = std::min(r.s, h[2 * (off + i)]);
    r.e = std::max(r.e, h[2 * (off + i) + 1]);
  }
  return r;
}

int main() {
  int can = 0;
  CK(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, 0));
  printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", can);
  const int G = 1024, GS = 64, IT = 20000;  // busy: ~60-100 us on 256 CUs
  float* out;
  uint64_t* st;
  int* ctr;
  uint32_t* flag;
  CK(hipMalloc(&out, (2 * G + GS) * 256 * 4));
  CK(hipMalloc(&st, (2 * G + GS) * 2 * 8));
  CK(hipMalloc(&ctr, 4));
  CK(hipMemset(ctr, 0, 4));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&flag), 8, hipMallocSignalMemory));
  CK(hipMemset(flag, 0, 8));
  hipStream_t m, s;
  CK(hipStreamCreateWithFlags(&m, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev, evs;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
  CK(hipEventCreateWithFlags(&evs, hipEventDisableTiming | hipEventReleaseToDevice));
  const char* names[] = {"none", "event", "flag", "mwait", "tiny", "write", "vwait"};
  uint32_t val = 0;
  for (int rep = 0; rep < 4; ++rep) {
    for (int mode = 0; mode < 7; ++mode) {
      ++val;
      CK(hipDeviceSynchronize());
      if (mode == 3) {  // the side event is long complete when main reaches the wait
        hipLaunchKernelGGL(busy, dim3(GS), dim3(256), 0, s, out + 2 * G * 256, 10, st + 2 * 2 * G, nullptr, nullptr, 0u);
        CK(hipEventRecord(evs, s));
      }
      if (mode == 6) hipLaunchKernelGGL(set_flag, dim3(1), dim3(64), 0, s, flag, val);
      hipLaunchKernelGGL(busy, dim3(G), dim3(256), 0, m, out, IT, st, ctr, mode == 2 ? flag : nullptr, val);
      if (mode == 1) {
        CK(hipEventRecord(ev, m));
        CK(hipStreamWaitEvent(s, ev, 0));
      } else if (mode == 2) {
        CK(hipStreamWaitValue32(s, flag, val, hipStreamWaitValueGte, 0xFFFFFFFFu));
      } else if (mode == 3) {
        CK(hipStreamWaitEvent(m, evs, 0));
      } else if (mode == 4) {
        hipLaunchKernelGGL(set_flag, dim3(1), dim3(64), 0, m, flag, val);
        CK(hipStreamWaitValue32(s, flag, val, hipStreamWaitValueGte, 0xFFFFFFFFu));
      } else if (mode == 6) {
        CK(hipStreamWaitValue32(m, flag, val, hipStreamWaitValueGte, 0xFFFFFFFFu));
      } else if (mode == 5) {
        CK(hipStreamWriteValue32(m, flag, val, 0));
        CK(hipStreamWaitValue32(s, flag, val, hipStreamWaitValueGte, 0xFFFFFFFFu));
      }
      hipLaunchKernelGGL(busy, dim3(G), dim3(256), 0, m, out + G * 256, IT, st + 2 * G, nullptr, nullptr, 0u);
      if (mode == 1 || mode == 2 || mode == 4 || mode == 5)
        hipLaunchKernelGGL(busy, dim3(GS), dim3(256), 0, s, out + 2 * G * 256, 10, st + 2 * 2 * G, nullptr, nullptr, 0u);
      CK(hipDeviceSynchronize());
      std::vector<uint64_t> h((2 * G + GS) * 2);
      CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
      const Span b1 = span(h, 0, G), b2 = span(h, G, G), sd = span(h, 2 * G, GS);
      printf("%-6s rep %d: busy1 %.1f us, main gap busy1 end -> busy2 start %.2f us", names[mode], rep,
             (b1.e - b1.s) * 0.01, (static_cast<double>(b2.s) - static_cast<double>(b1.e)) * 0.01);
      if (mode == 1 || mode == 2 || mode == 4 || mode == 5)
        printf(", side kernel start - busy1 end %.2f us", (static_cast<double>(sd.s) - static_cast<double>(b1.e)) * 0.01);
      printf("\n");
    }
  }
  return 0;
}
