"""Data parallelism over RCCL / xGMI (absent in the reference).

One process per GPU. ``torch.distributed`` (``nccl`` = RCCL on ROCm) brings the ranks up
(rendezvous, parameter broadcast, barriers) and, by default, carries the gradient buckets through
ProcessGroupNCCL; ``PZ_COMM=native`` moves the buckets to the extension's own RCCL communicator
(``csrc/rccl_comm.cpp``, N8).
Every rank holds a full parameter replica in one flat buffer (:mod:`..engine.params`); the global
minibatch is sharded over ranks; gradients are summed with bucketed all-reduces that are *issued
during backward*: the fused trainer calls :meth:`DataParallelContext.all_reduce_async` right after
each layer's dW GEMM is enqueued. The collective runs on the communicator's stream, fenced to the
compute stream by an event at issue time, so layer L's gradient travels over xGMI while layers
L-1 ... 0 are still computing; :meth:`wait_one` only makes the CURRENT stream (the optimizer's)
wait for that bucket's completion event (no host blocking), and the fused optimizer folds the
1/world mean into its update.

The same class runs on ``gloo`` for CPU tests (world_size > 1 without GPUs).

Bucketing policy for xGMI (7 links × ~153 GB/s per GPU, ring collectives per-link bound): one
bucket per layer weight (8-134 MB for the benchmark configs — large enough to saturate the rings,
and naturally ordered last-layer-first), plus one final bucket for all small parameters (biases,
batchnorm, embeddings) and the loss scalar.
"""
from __future__ import annotations

import os
from datetime import timedelta
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DataParallelContext:
    rank: int = 0
    world_size: int = 1
    group: object = None
    comm_dtype: torch.dtype | None = None   # e.g. bfloat16 to halve xGMI bytes (default: fp32)
    # PZ_FORCE_COMM=1: run every collective even at world size 1 (a 1-rank RCCL communicator), so
    # the comm-stream / wait ordering of the data-parallel step is exercised on a single GPU
    force: bool = False
    native: object = None  # _NativeComm: the extension's RCCL communicator (gradient buckets)
    # PZ_COMM_BUDGET=k (default 0 = off): CUs to leave to the gradient collectives while a bucket is
    # on the wire (RCCL holds one workgroup per channel). The fused trainer then runs the paired dW
    # launch that overlaps the largest bucket as one persistent stream-K schedule with a grid k CUs
    # smaller (csrc/gemm_sk.hip) instead of its one-round tiled grid, whose workgroups on the held
    # CUs would otherwise form a whole second round (profiles/r5_comm_pressure.txt).
    comm_cus: int = 0
    # second communicator (process group / native RCCL comm) for the sharded optimizer's all-gathers
    # and statistics sums: ONE communicator runs its collectives in issue order, and an all-gather
    # waits for its weight's update on the side stream — on the bucket communicator it would hold
    # every later reduce-scatter (the first layer's, on the step boundary) behind that update
    ag_group: object = None
    ag_native: object = None

    @property
    def enabled(self) -> bool:
        return self.world_size > 1 or self.force

    @property
    def backend(self) -> str | None:
        return dist.get_backend(self.group) if dist.is_initialized() else None

    def all_reduce_async(self, t: torch.Tensor, exact: bool = False):
        """Start a SUM all-reduce of ``t`` in place. ``exact``: never through ``comm_dtype``
        (buckets that carry the loss or small accumulated parameters)."""
        if not self.enabled or t.numel() == 0:
            return None
        low = None
        if not exact and self.comm_dtype is not None and t.dtype != self.comm_dtype:
            low = t.to(self.comm_dtype)
        buf = t if low is None else low
        if self.native is not None:
            work = self.native.all_reduce(buf)
        else:
            work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return (work, low, t if low is not None else None)

    # ---- sharded optimizer (ZeRO-1, engine/zero.py) ------------------------------------------
    @property
    def shard_world(self) -> int:
        """Ranks a sharded buffer is split over: the world, or the world a one-GPU collective
        proxy models (its caller then runs as that world's rank 0)."""
        return getattr(self.native, "model_world", None) or self.world_size

    @property
    def shard_rank(self) -> int:
        return 0 if getattr(self.native, "model_world", None) else self.rank

    def reduce_scatter_async(self, full: torch.Tensor, shard: torch.Tensor):
        """Start a SUM reduce-scatter: this rank's ``shard`` receives the sum over the ranks of its
        slice ``full[r*n:(r+1)*n]`` (``n = shard.numel()``). Same handle contract as
        :meth:`all_reduce_async` (:meth:`wait_one` makes the current stream wait)."""
        if not self.enabled:
            return None
        if self.native is not None:
            return (_Ticket(self.native.handle, torch.ops.pz.rccl_reduce_scatter(self.native.handle, full, shard)),
                    None, None)
        if full.is_cuda and self.backend == "gloo":
            # (gloo on device tensors: one all-reduce of a copy, then this rank's slice)
            n = shard.numel()
            tmp = full.clone()
            work = dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            return (work, tmp[self.rank * n:(self.rank + 1) * n], shard)
        work = dist.reduce_scatter_tensor(shard, full, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return (work, None, None)

    def open_side_comm(self) -> None:
        """Bring up the second communicator (collective: every rank calls it at the same point —
        the fused trainer's constructor when it shards the optimizer)."""
        if not self.enabled or self.ag_group is not None or self.ag_native is not None:
            return
        if isinstance(self.native, _ProxyComm):
            self.ag_native = _ProxyComm()
        elif self.native is not None:
            self.ag_native = _NativeComm(self.rank, self.world_size)
        elif dist.is_initialized():
            self.ag_group = dist.new_group(list(range(self.world_size)))

    def all_gather_async(self, shard: torch.Tensor, full: torch.Tensor, side: bool = False):
        """Start an all-gather of every rank's ``shard`` into ``full`` (rank r's at
        ``[r*n, (r+1)*n)``); ``shard`` may be this rank's slice of ``full`` (in place).
        ``side``: on the second communicator (:meth:`open_side_comm`) when there is one."""
        if not self.enabled:
            return None
        native = self.ag_native if side and self.ag_native is not None else self.native
        group = self.ag_group if side and self.ag_group is not None else self.group
        if native is not None:
            return (_Ticket(native.handle, torch.ops.pz.rccl_all_gather(native.handle, shard, full)), None, None)
        if full.is_cuda and self.backend == "gloo":
            # (gloo on device tensors: zeros elsewhere + one exact sum all-reduce)
            n = shard.numel()
            tmp = torch.zeros_like(full)
            tmp[self.rank * n:(self.rank + 1) * n].copy_(shard)
            work = dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group, async_op=True)
            return (work, tmp, full)
        work = dist.all_gather_into_tensor(full, shard, group=group, async_op=True)
        return (work, None, None)

    def side_all_reduce_async(self, t: torch.Tensor):
        """Exact SUM all-reduce on the second communicator (the sharded statistics)."""
        if not self.enabled:
            return None
        if self.ag_native is not None:
            return (_Ticket(self.ag_native.handle, torch.ops.pz.rccl_all_reduce(self.ag_native.handle, t)), None, None)
        if self.ag_group is not None:
            return (dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.ag_group, async_op=True), None, None)
        return self.all_reduce_async(t, exact=True)

    def all_reduce_(self, t: torch.Tensor) -> None:
        """Blocking exact SUM all-reduce in place (stream-ordered under RCCL): the synchronised
        batchnorm statistics, which the next kernel needs right away."""
        self.wait_one(self.all_reduce_async(t, exact=True))

    def wait_all(self, handles) -> None:
        for h in handles:
            self.wait_one(h)

    def wait_one(self, h) -> None:
        """Make the CURRENT stream wait for one bucket (and unpack a reduced-precision bucket)."""
        if h is None:
            return
        work, low, dst = h
        work.wait()
        if low is not None:
            if dst.is_cuda:
                low.record_stream(torch.cuda.current_stream(dst.device))
            dst.copy_(low)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> None:
        if self.enabled:
            dist.broadcast(t, src=src, group=self.group)

    def all_reduce_scalar(self, value: float, op=None) -> float:
        if not self.enabled:
            return value
        dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else "cpu"
        t = torch.tensor([value], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=self.group)
        return t.item()

    def all_reduce_scalar_max(self, value: float) -> float:
        return self.all_reduce_scalar(value, dist.ReduceOp.MAX) if self.enabled else value

    def barrier(self) -> None:
        if self.enabled:
            dist.barrier(group=self.group)


class _Ticket:
    """One bucket in flight on the native communicator: ``wait()`` makes the current stream wait."""
    __slots__ = ("comm", "ticket")

    def __init__(self, comm: int, ticket: int):
        self.comm, self.ticket = comm, ticket

    def wait(self) -> None:
        torch.ops.pz.rccl_wait(self.comm, self.ticket)


class _NativeComm:
    """The extension's RCCL communicator (``csrc/rccl_comm.cpp``): rank 0's unique id travels over
    the already initialised process group, then every rank joins with ncclCommInitRank on its GPU.
    A sum of ``rank + 1`` over the new communicator checks it before any gradient goes through."""

    def __init__(self, rank: int, world: int, group=None, device: torch.device | None = None):
        if device is None:
            from ..ops import native
            native.require()
        dev = device or torch.device("cuda", torch.cuda.current_device())
        uid = torch.ops.pz.rccl_unique_id() if rank == 0 else torch.zeros(128, dtype=torch.uint8)
        uid_dev = uid.to(dev)
        dist.broadcast(uid_dev, src=0, group=group)
        # comm stream at NORMAL priority (PZ_COMM_PRIO=1: high): a high-priority stream slowed every
        # compute kernel of the forced 1-rank step (2.44 vs 1.40 ms/step, profiles/r2_ab_native_comm.txt)
        # PZ_COMM_CUS=k: the communicator's stream is CU-masked to k CUs (evenly spread over the
        # XCDs): the channel kernels of every bucket all-reduce stay on those CUs
        self.handle = torch.ops.pz.rccl_init(uid_dev.cpu(), world, rank, os.environ.get("PZ_COMM_PRIO", "0") == "1",
                                             int(os.environ.get("PZ_COMM_CUS", "0")))
        probe = torch.full((1,), float(rank + 1), device=dev, dtype=torch.float64)
        self.all_reduce(probe).wait()
        got, want = probe.item(), world * (world + 1) / 2
        if got != want:
            raise RuntimeError(f"pz rccl communicator self-check failed: sum {got}, expected {want}")

    def all_reduce(self, t: torch.Tensor) -> _Ticket:
        return _Ticket(self.handle, torch.ops.pz.rccl_all_reduce(self.handle, t))

    def close(self) -> None:
        if self.handle is not None:
            torch.ops.pz.rccl_destroy(self.handle)
            self.handle = None


class _ProxyComm:
    """``PZ_COMM=proxy`` (one GPU, ``PZ_FORCE_COMM=1``): every bucket "all-reduce" launches the
    collective-footprint kernel of ``csrc/comm_proxy.hip`` on the communicator stream instead —
    ``PZ_COMM_PROXY_WGS`` resident channel workgroups (default 16) held for the time a ring
    all-reduce of that bucket over ``PZ_COMM_PROXY_WORLD`` ranks (default 8) at
    ``PZ_COMM_PROXY_GBPS`` bus bandwidth (default 150 GB/s) takes, optionally CU-masked
    (``PZ_COMM_CUS``). Buckets are left untouched (a 1-rank sum is the identity), so the step's
    results are the world-1 results; what changes is how the GEMMs share the GPU with the comm
    kernels — the data-parallel step's cost on one GPU (tools/comm_pressure.py)."""

    def __init__(self):
        from ..ops import native
        native.require()
        env = os.environ.get
        self.model_world = int(env("PZ_COMM_PROXY_WORLD", "8"))  # the sharded optimizer's modelled world
        self.handle = torch.ops.pz.rccl_proxy_init(int(env("PZ_COMM_PROXY_WORLD", "8")),
                                                   int(env("PZ_COMM_PROXY_WGS", "16")),
                                                   float(env("PZ_COMM_PROXY_GBPS", "150")),
                                                   int(env("PZ_COMM_CUS", "0")), False)

    def all_reduce(self, t: torch.Tensor) -> _Ticket:
        return _Ticket(self.handle, torch.ops.pz.rccl_all_reduce(self.handle, t))

    def close(self) -> None:
        if self.handle is not None:
            torch.ops.pz.rccl_destroy(self.handle)
            self.handle = None


_CONTEXT: DataParallelContext | None = None


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _default_backend(world: int) -> str:
    """RCCL unless this node has fewer visible GPUs than ranks. Only an explicit LOCAL_WORLD_SIZE
    (torchrun sets it) says how many ranks share this node; without one, WORLD_SIZE counts ranks on
    every node (srun / mpirun with 16 ranks on 8-GPU nodes) and is no reason to leave RCCL."""
    if not torch.cuda.is_available():
        return "gloo"
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    if lw is not None and int(lw) > torch.cuda.device_count():
        import logging
        logging.getLogger(__name__).warning(
            "LOCAL_WORLD_SIZE=%s ranks share %d visible GPU(s): falling back to the gloo backend "
            "(host collectives, much slower); set PZ_DIST_BACKEND to override", lw, torch.cuda.device_count())
        return "gloo"
    return "nccl"


def init_from_env(backend: str | None = None) -> DataParallelContext:
    """Initialise the process group from torchrun's env vars (RANK / WORLD_SIZE / MASTER_*).

    ``PZ_FORCE_COMM=1`` brings a group up even at world size 1 (rendezvous on 127.0.0.1) and
    marks the context ``force``: every bucket all-reduce then really runs through RCCL."""
    global _CONTEXT
    world = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("PZ_FORCE_COMM", "0") == "1"
    if force and world == 1 and not dist.is_initialized():
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    if (world > 1 or force) and not dist.is_initialized():
        if backend is None:
            # PZ_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU; so
            # does a launch with more ranks on this node than visible GPUs (RCCL needs one GPU per
            # rank: "invalid usage" otherwise), e.g. torchrun --nproc-per-node 4 on a 1-GPU box
            backend = os.environ.get("PZ_DIST_BACKEND") or _default_backend(world)
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())

            # failure detection: a rank that dies or a collective that hangs must abort the job
            # (RCCL async error handling + the collective watchdog timeout) instead of hanging the
            # node; the REST layer then persists status "Failed" 
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        timeout = timedelta(seconds=float(os.environ.get("PZ_DIST_TIMEOUT_S", "600")))
        rdv = os.environ.get("PZ_RENDEZVOUS_FILE")
        if rdv:  # a shared-file store: no TCP port to pick ahead of the ranks (and lose in a race)
            dist.init_process_group(backend=backend, init_method=f"file://{rdv}", timeout=timeout,
                                    rank=int(os.environ.get("RANK", "0")), world_size=world)
        else:
            dist.init_process_group(backend=backend, timeout=timeout)
    comm = os.environ.get("PZ_GRAD_COMM_DTYPE")
    comm_dtype = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": None, None: None}.get(comm)
    if dist.is_initialized():
        _CONTEXT = DataParallelContext(dist.get_rank(), dist.get_world_size(), None, comm_dtype, force=force)
        _CONTEXT.comm_cus = int(os.environ.get("PZ_COMM_BUDGET", "0"))
        # PZ_COMM=native: gradient buckets on the extension's own RCCL communicator instead of
        # ProcessGroupNCCL. Opt-in: with the same bucket schedule it measured 1.8% slower on the
        # forced 1-rank step (1.390-1.396 vs 1.366-1.373 ms, profiles/r2_ab_native_comm.txt), and
        # the multi-GPU node runs are the driver's, not ours to A/B
        mode = os.environ.get("PZ_COMM", "torch")
        if dist.get_backend() == "nccl" and mode == "native":
            _CONTEXT.native = _NativeComm(_CONTEXT.rank, _CONTEXT.world_size)
        elif mode == "proxy":
            if _CONTEXT.world_size != 1 or not torch.cuda.is_available():
                raise RuntimeError("PZ_COMM=proxy models the collectives of a multi-GPU step on ONE GPU "
                                   "(PZ_FORCE_COMM=1, world size 1)")
            _CONTEXT.native = _ProxyComm()
    else:
        _CONTEXT = DataParallelContext(0, 1, None, comm_dtype)
    return _CONTEXT


def get_context() -> DataParallelContext:
    global _CONTEXT
    if _CONTEXT is None:
        if dist.is_available() and dist.is_initialized():
            _CONTEXT = DataParallelContext(dist.get_rank(), dist.get_world_size())
        else:
            return DataParallelContext()
    return _CONTEXT


def set_context(ctx: DataParallelContext | None) -> None:
    global _CONTEXT
    _CONTEXT = ctx


def shutdown() -> None:
    global _CONTEXT
    if _CONTEXT is not None and (_CONTEXT.native is not None or _CONTEXT.ag_native is not None):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        for comm in (_CONTEXT.ag_native, _CONTEXT.native):
            if comm is not None:
                comm.close()
        _CONTEXT.native = _CONTEXT.ag_native = None
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _CONTEXT = None
