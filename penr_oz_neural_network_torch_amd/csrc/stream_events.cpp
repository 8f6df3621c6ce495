// Device-scope cross-stream events for the trainer's step schedule.
//
// The fused step orders its side-stream optimizer launches behind the compute stream (and the
// next step's forward behind them) with event record / stream-wait pairs. A default HIP event
// (torch.cuda.Event) performs a SYSTEM-scope sequentially consistent fence when it transitions
// to recorded: every XCD's L2 is written back and invalidated, which the r4 step trace shows as
// ~7 us of idle compute stream around each record / wait and colder caches for the kernel after.
// Ordering two streams of ONE device needs only a device-scope release (kernel completion has
// already written the producer's results back to memory), so these events are created with
// hipEventDisableTiming | hipEventReleaseToDevice; the per-step timestamps the trainer reads after
// a synchronize are hipEventDisableSystemFence events. Handles are plain integers; a trainer keeps
// a ring of ordering events (re-recording an event after the waits on its previous record were
// enqueued is well defined).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <cstdint>

#include "pz_kernels.h"

namespace {

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "pz events: ", what, ": ", hipGetErrorString(e));
}

hipStream_t current(int64_t device) {
  return c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
}

// kind 0: an ordering event with a device-scope release; 1: a timestamp-only event
// (hipEventDisableSystemFence: the step-end stamps the trainer reads back after a device
// synchronize); 2: a default timing event (system-scope fence, what torch.cuda.Event(enable_timing)
// creates: the A/B baseline)
int64_t event_create_op(int64_t device, int64_t kind) {
  TORCH_CHECK(kind >= 0 && kind <= 2, "pz events: kind 0 (order), 1 (stamp) or 2 (default timing)");
  int prev = 0;
  check(hipGetDevice(&prev), "hipGetDevice");
  check(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
  hipEvent_t e = nullptr;
  const unsigned flags = kind == 0 ? (hipEventDisableTiming | hipEventReleaseToDevice)
                         : kind == 1 ? hipEventDisableSystemFence
                                     : hipEventDefault;
  const hipError_t err = hipEventCreateWithFlags(&e, flags);
  hipSetDevice(prev);
  check(err, "hipEventCreateWithFlags");
  return reinterpret_cast<int64_t>(e);
}

void event_record_op(int64_t ev, int64_t device) {
  check(hipEventRecord(reinterpret_cast<hipEvent_t>(ev), current(device)), "hipEventRecord");
}

void event_wait_op(int64_t ev, int64_t device) {
  check(hipStreamWaitEvent(current(device), reinterpret_cast<hipEvent_t>(ev), 0), "hipStreamWaitEvent");
}

bool event_query_op(int64_t ev) {
  const hipError_t e = hipEventQuery(reinterpret_cast<hipEvent_t>(ev));
  if (e == hipErrorNotReady) return false;
  check(e, "hipEventQuery");
  return true;
}

void event_destroy_op(int64_t ev) { hipEventDestroy(reinterpret_cast<hipEvent_t>(ev)); }

double event_elapsed_op(int64_t start, int64_t end) {
  float ms = 0.f;
  check(hipEventElapsedTime(&ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(end)),
        "hipEventElapsedTime");
  return ms;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(pz, m) {
  m.def("event_create(int device, int kind=0) -> int");
  m.def("event_record(int ev, int device) -> ()");
  m.def("event_wait(int ev, int device) -> ()");
  m.def("event_query(int ev) -> bool");
  m.def("event_destroy(int ev) -> ()");
  m.def("event_elapsed(int start, int end) -> float");
}

TORCH_LIBRARY_IMPL(pz, CompositeExplicitAutograd, m) {
  m.impl("event_create", TORCH_FN(event_create_op));
  m.impl("event_record", TORCH_FN(event_record_op));
  m.impl("event_wait", TORCH_FN(event_wait_op));
  m.impl("event_query", TORCH_FN(event_query_op));
  m.impl("event_destroy", TORCH_FN(event_destroy_op));
  m.impl("event_elapsed", TORCH_FN(event_elapsed_op));
}
