// N8 — the data-parallel communicator: RCCL driven directly from this extension (SURVEY §2.5,
// §5.8). One communicator per process/GPU (one rank per GPU), its collectives on a comm stream
// owned here (normal priority by default: a high-priority stream measured 1.7x slower steps),
// fenced to the compute stream with HIP events:
//
//   rccl_all_reduce(h, t)  current stream --event--> comm stream: ncclAllReduce(t, SUM, in place)
//                          --event[ticket]-->  (returns the ticket)
//   rccl_wait(h, ticket)   the CURRENT stream waits for that bucket (no host blocking) — the
//                          optimizer side stream waits for exactly the buckets it updates
//   rccl_reduce_scatter(h, full, shard) / rccl_all_gather(h, shard, full)
//                          the sharded optimizer (ZeRO-1, engine/zero.py): each rank receives the
//                          SUM of its 1/W slice of a gradient bucket, updates only that slice of
//                          the fp32 master / Adam moments, and the updated bf16 weight slices are
//                          gathered back into every rank's GEMM copy — the same ring bytes as one
//                          all-reduce, 1/W of the optimizer's HBM traffic per rank
//
// so a layer's gradient bucket crosses xGMI while the following layers' backward GEMMs run, and
// nothing but stream waits orders the update behind it (the ordering ProcessGroupNCCL's
// Work::wait() only implies). The RCCL entry points are resolved from the librccl that
// torch already mapped (same SONAME), so one RCCL runtime serves both.
#include <ATen/ATen.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <torch/library.h>

#include <array>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "pz_kernels.h"

namespace {

struct Api {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*destroy)(ncclComm_t);
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*);
  const char* (*error_string)(ncclResult_t);
};

template <typename F>
void resolve(void* lib, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(lib, name));
  TORCH_CHECK(fn != nullptr, "pz rccl: ", name, " not found in librccl");
}

const Api& api() {
  static const Api a = [] {
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, already mapped
    if (lib == nullptr) lib = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (lib == nullptr) lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    TORCH_CHECK(lib != nullptr, "pz rccl: cannot load librccl: ", dlerror());
    Api x{};
    resolve(lib, "ncclGetUniqueId", x.get_unique_id);
    resolve(lib, "ncclCommInitRank", x.init_rank);
    resolve(lib, "ncclAllReduce", x.all_reduce);
    resolve(lib, "ncclReduceScatter", x.reduce_scatter);
    resolve(lib, "ncclAllGather", x.all_gather);
    resolve(lib, "ncclCommDestroy", x.destroy);
    resolve(lib, "ncclCommGetAsyncError", x.async_error);
    resolve(lib, "ncclGetErrorString", x.error_string);
    return x;
  }();
  return a;
}

#define PZ_NCCL_CHECK(expr)                                                                 \
  do {                                                                                      \
    const ncclResult_t r_ = (expr);                                                         \
    TORCH_CHECK(r_ == ncclSuccess, "pz rccl: ", #expr, " failed: ", api().error_string(r_)); \
  } while (0)
#define PZ_HIP_OK(expr)                                                                      \
  do {                                                                                       \
    const hipError_t e_ = (expr);                                                            \
    TORCH_CHECK(e_ == hipSuccess, "pz rccl: ", #expr, " failed: ", hipGetErrorString(e_));   \
  } while (0)

// a bucket's completion event is reused after kRing later buckets: the trainer waits for every
// bucket within the step that issued it (at most a few per layer)
constexpr int kRing = 256;

struct Comm {
  ncclComm_t comm = nullptr;
  int device = 0;
  int nranks = 1;
  // proxy communicator (PZ_COMM=proxy, one GPU): no RCCL; every "all-reduce" launches the
  // collective-footprint kernel (comm_proxy.hip) for the time a ring all-reduce of that bucket
  // over `proxy_world` ranks at `proxy_gbps` bus bandwidth would take, on `proxy_wgs` channels
  bool proxy = false;
  int proxy_wgs = 0;
  double proxy_gbps = 0.0;
  int proxy_world = 1;
  at::Tensor scratch;
  c10::hip::HIPStream stream;
  hipEvent_t ready = nullptr;
  std::array<hipEvent_t, kRing> done{};
  int64_t next = 0;
  bool closed = false;
  // serialises all_reduce / wait / destroy on ONE communicator: ticket numbering and the event
  // ring are shared state, and destroy must not free the comm under a running op
  std::mutex mu;
  explicit Comm(c10::hip::HIPStream s) : stream(s) {}
};

std::mutex g_mu;
std::vector<std::shared_ptr<Comm>> g_comms;

// shared ownership: a concurrent destroy drops the table's reference, the op in flight keeps its own
std::shared_ptr<Comm> get(int64_t h) {
  std::lock_guard<std::mutex> lock(g_mu);
  TORCH_CHECK(h >= 0 && h < static_cast<int64_t>(g_comms.size()) && g_comms[h], "pz rccl: bad communicator handle");
  return g_comms[h];
}

ncclDataType_t nccl_type(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    default: TORCH_CHECK(false, "pz rccl: unsupported dtype ", t.scalar_type());
  }
}

at::Tensor unique_id_op() {
  ncclUniqueId id;
  PZ_NCCL_CHECK(api().get_unique_id(&id));
  at::Tensor out = at::empty({static_cast<int64_t>(sizeof(id))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &id, sizeof(id));
  return out;
}

// The communicator's stream. cu_count > 0: a stream whose kernels may only run on that many CUs
// (hipExtStreamCreateWithCUMask, bits spread evenly over the device's CUs so every XCD / shader
// engine gives up a few): the collective's channel kernels then never take a CU outside the mask,
// whatever the GEMMs on the compute stream leave free.
c10::hip::HIPStream make_stream(int dev, bool high_priority, int64_t cu_count) {
  if (cu_count <= 0) return c10::hip::getStreamFromPool(high_priority, static_cast<c10::DeviceIndex>(dev));
  hipDeviceProp_t prop;
  PZ_HIP_OK(hipGetDeviceProperties(&prop, dev));
  const int n = prop.multiProcessorCount;
  TORCH_CHECK(cu_count < n, "pz rccl: a CU mask of ", cu_count, " of ", n, " CUs");
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int64_t j = 0; j < cu_count; ++j) {
    const int64_t bit = j * n / cu_count;
    mask[bit / 32] |= 1u << (bit % 32);
  }
  hipStream_t s = nullptr;
  PZ_HIP_OK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
  // (never destroyed: one per communicator, for the process lifetime)
  return c10::hip::getStreamFromExternal(s, static_cast<c10::DeviceIndex>(dev));
}

int64_t add_comm(std::shared_ptr<Comm> c) {
  PZ_HIP_OK(hipEventCreateWithFlags(&c->ready, hipEventDisableTiming));
  for (auto& e : c->done) PZ_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::lock_guard<std::mutex> lock(g_mu);
  g_comms.push_back(std::move(c));
  return static_cast<int64_t>(g_comms.size()) - 1;
}

int64_t proxy_init_op(int64_t world, int64_t wgs, double gbps, int64_t cu_count, bool high_priority) {
  TORCH_CHECK(world >= 2 && wgs >= 1 && gbps > 0.0, "pz rccl: proxy needs world >= 2, wgs >= 1, gbps > 0");
  int dev = 0;
  PZ_HIP_OK(hipGetDevice(&dev));
  auto c = std::make_shared<Comm>(make_stream(dev, high_priority, cu_count));
  c->device = dev;
  c->proxy = true;
  c->proxy_wgs = static_cast<int>(wgs);
  c->proxy_gbps = gbps;
  c->proxy_world = static_cast<int>(world);
  c->scratch = at::zeros({wgs * (64 << 10) / 4}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
  return add_comm(std::move(c));
}

int64_t init_op(const at::Tensor& id, int64_t nranks, int64_t rank, bool high_priority, int64_t cu_count) {
  TORCH_CHECK(id.device().is_cpu() && id.scalar_type() == at::kByte && id.numel() == sizeof(ncclUniqueId),
              "pz rccl: the unique id is ", sizeof(ncclUniqueId), " CPU bytes");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "pz rccl: rank ", rank, " of ", nranks);
  ncclUniqueId uid;
  std::memcpy(&uid, id.contiguous().data_ptr(), sizeof(uid));
  int dev = 0;
  PZ_HIP_OK(hipGetDevice(&dev));
  auto c = std::make_shared<Comm>(make_stream(dev, high_priority, cu_count));
  c->device = dev;
  c->nranks = static_cast<int>(nranks);
  PZ_NCCL_CHECK(api().init_rank(&c->comm, static_cast<int>(nranks), uid, static_cast<int>(rank)));
  return add_comm(std::move(c));
}

enum class Coll { AllReduce, ReduceScatter, AllGather };

// One collective on the comm stream, fenced to the current stream by events. `send` / `recv`:
// all-reduce in place (send == recv); reduce-scatter full [W * n] -> shard [n]; all-gather shard
// [n] -> full [W * n] (in place when the shard is the rank's slice of the full buffer). Proxy
// communicators hold the collective's workgroups for the ring time instead: all-reduce 2 (W-1)/W
// x bytes, reduce-scatter / all-gather (W-1)/W x the FULL buffer's bytes, at the bus bandwidth.
int64_t collective(int64_t h, Coll kind, const at::Tensor& send, const at::Tensor& recv) {
  const std::shared_ptr<Comm> cp = get(h);
  Comm& c = *cp;
  std::lock_guard<std::mutex> lock(c.mu);
  TORCH_CHECK(!c.closed, "pz rccl: communicator destroyed");
  for (const at::Tensor* t : {&send, &recv}) {
    TORCH_CHECK(t->is_cuda() && t->device().index() == c.device, "pz rccl: tensor must live on the communicator's GPU");
    TORCH_CHECK(t->is_contiguous(), "pz rccl: contiguous buckets only");
  }
  TORCH_CHECK(send.scalar_type() == recv.scalar_type(), "pz rccl: send / recv dtypes differ");
  const at::Tensor& full = kind == Coll::AllGather ? recv : send;
  const at::Tensor& part = kind == Coll::AllGather ? send : recv;
  // (a proxy communicator models `proxy_world` ranks on one GPU: the caller shards for that world
  // as virtual rank 0, so any whole number of shards per buffer)
  if (kind != Coll::AllReduce)
    TORCH_CHECK(c.proxy ? (part.numel() > 0 && full.numel() % part.numel() == 0) : full.numel() == part.numel() * c.nranks,
                "pz rccl: the full buffer must hold ", c.proxy ? c.proxy_world : c.nranks, " shards of ", part.numel(),
                " elements (got ", full.numel(), ")");
  const int64_t ticket = c.next++;
  if (full.numel() == 0) {
    PZ_HIP_OK(hipEventRecord(c.done[ticket % kRing], c10::hip::getCurrentHIPStream(c.device).stream()));
    return ticket;
  }
  const hipStream_t cur = c10::hip::getCurrentHIPStream(c.device).stream();
  PZ_HIP_OK(hipEventRecord(c.ready, cur));
  PZ_HIP_OK(hipStreamWaitEvent(c.stream.stream(), c.ready, 0));
  if (c.proxy) {
    const double bytes = static_cast<double>(full.numel()) * full.element_size();
    const double f = (kind == Coll::AllReduce ? 2.0 : 1.0) * (c.proxy_world - 1) / c.proxy_world;
    const double us = f * bytes / (c.proxy_gbps * 1e3);
    const double step_us = 4096.0 * c.proxy_wgs / (c.proxy_gbps * 1e3);
    PZ_HIP_OK(pz::comm_proxy(c.scratch.data_ptr(), c.proxy_wgs, 64 << 10, us, step_us, c.stream.stream()));
    // virtual rank 0's slice moves (its sum over one real rank is itself)
    if (send.data_ptr() != recv.data_ptr() && kind != Coll::AllReduce)
      PZ_HIP_OK(hipMemcpyAsync(recv.data_ptr(), send.data_ptr(), part.numel() * part.element_size(),
                               hipMemcpyDeviceToDevice, c.stream.stream()));
  } else if (kind == Coll::AllReduce) {
    PZ_NCCL_CHECK(api().all_reduce(send.data_ptr(), recv.data_ptr(), static_cast<size_t>(recv.numel()), nccl_type(recv),
                                   ncclSum, c.comm, c.stream.stream()));
  } else if (kind == Coll::ReduceScatter) {
    PZ_NCCL_CHECK(api().reduce_scatter(send.data_ptr(), recv.data_ptr(), static_cast<size_t>(recv.numel()),
                                       nccl_type(recv), ncclSum, c.comm, c.stream.stream()));
  } else {
    PZ_NCCL_CHECK(api().all_gather(send.data_ptr(), recv.data_ptr(), static_cast<size_t>(send.numel()), nccl_type(send),
                                   c.comm, c.stream.stream()));
  }
  // the caching allocator must not hand the buffers' memory out again before the comm stream is done
  c10::hip::HIPCachingAllocator::recordStream(send.storage().data_ptr(), c.stream);
  if (recv.data_ptr() != send.data_ptr())
    c10::hip::HIPCachingAllocator::recordStream(recv.storage().data_ptr(), c.stream);
  PZ_HIP_OK(hipEventRecord(c.done[ticket % kRing], c.stream.stream()));
  return ticket;
}

int64_t all_reduce_op(int64_t h, const at::Tensor& t) { return collective(h, Coll::AllReduce, t, t); }

int64_t reduce_scatter_op(int64_t h, const at::Tensor& full, const at::Tensor& shard) {
  return collective(h, Coll::ReduceScatter, full, shard);
}

int64_t all_gather_op(int64_t h, const at::Tensor& shard, const at::Tensor& full) {
  return collective(h, Coll::AllGather, shard, full);
}

void wait_op(int64_t h, int64_t ticket) {
  const std::shared_ptr<Comm> cp = get(h);
  Comm& c = *cp;
  std::lock_guard<std::mutex> lock(c.mu);
  TORCH_CHECK(!c.closed, "pz rccl: communicator destroyed");
  TORCH_CHECK(ticket >= 0 && ticket < c.next && c.next - ticket <= kRing, "pz rccl: stale or unknown bucket ticket");
  if (!c.proxy) {
    ncclResult_t async = ncclSuccess;
    PZ_NCCL_CHECK(api().async_error(c.comm, &async));
    TORCH_CHECK(async == ncclSuccess || async == ncclInProgress, "pz rccl: communicator failed: ",
                api().error_string(async));
  }
  PZ_HIP_OK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(c.device).stream(), c.done[ticket % kRing], 0));
}

void destroy_op(int64_t h) {
  std::shared_ptr<Comm> c;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    TORCH_CHECK(h >= 0 && h < static_cast<int64_t>(g_comms.size()) && g_comms[h], "pz rccl: bad communicator handle");
    c = std::move(g_comms[h]);
  }
  std::lock_guard<std::mutex> lock(c->mu);  // waits for an op in flight on another thread
  c->closed = true;
  PZ_HIP_OK(hipStreamSynchronize(c->stream.stream()));
  if (!c->proxy) PZ_NCCL_CHECK(api().destroy(c->comm));
  hipEventDestroy(c->ready);
  for (auto& e : c->done) hipEventDestroy(e);
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(pz, m) {
  m.def("rccl_unique_id() -> Tensor");
  m.def("rccl_init(Tensor uid, int nranks, int rank, bool high_priority, int cu_count=0) -> int");
  m.def("rccl_proxy_init(int world, int wgs, float gbps, int cu_count=0, bool high_priority=False) -> int");
  m.def("rccl_all_reduce(int comm, Tensor(a!) t) -> int");
  m.def("rccl_reduce_scatter(int comm, Tensor full, Tensor(a!) shard) -> int");
  m.def("rccl_all_gather(int comm, Tensor shard, Tensor(a!) full) -> int");
  m.def("rccl_wait(int comm, int ticket) -> ()");
  m.def("rccl_destroy(int comm) -> ()");
}

TORCH_LIBRARY_IMPL(pz, CompositeExplicitAutograd, m) {
  m.impl("rccl_unique_id", TORCH_FN(unique_id_op));
  m.impl("rccl_init", TORCH_FN(init_op));
  m.impl("rccl_proxy_init", TORCH_FN(proxy_init_op));
  m.impl("rccl_all_reduce", TORCH_FN(all_reduce_op));
  m.impl("rccl_reduce_scatter", TORCH_FN(reduce_scatter_op));
  m.impl("rccl_all_gather", TORCH_FN(all_gather_op));
  m.impl("rccl_wait", TORCH_FN(wait_op));
  m.impl("rccl_destroy", TORCH_FN(destroy_op));
}
