"""Multi-GPU data-parallel training behind the REST service (reference ``main.py:281-298``).

The reference trains in one worker thread of one process (``run_in_threadpool(model.train, ...)``).
Here the server process becomes **rank 0 of an N-rank group**: at startup it spawns N-1 worker
processes (one per further GPU, before this process touches the GPU) and joins them in one
``torch.distributed`` process group — RCCL over xGMI for GPU models (``gloo`` when rehearsing on
the CPU). A ``PUT /train/`` on a GPU model then runs on every rank:

    rank 0 (train thread)                       ranks 1..N-1 (parallel/worker.py)
    ─────────────────────                       ─────────────────────────────────
    send {"op": "load", model_id, data, hp} ──► deserialize model_<id> from the shared models/ dir
                                            ◄── "ok" | error text
    send "go" (or "abort" if any rank failed)──►
    model.train(data, **hp) ◄═══ RCCL ═══►      model.train(data, **hp)  (same data, own GPU)
    (writes the checkpoints: rank 0 only)   ◄── "done" | "failed: ..."

Inside ``train`` the fused engine shards every epoch's minibatch over the ranks and all-reduces
the gradient buckets during backward (:mod:`.dist`, :class:`..engine.trainer.FusedTrainer`); the
model writes its files on rank 0 only. Commands travel on a local authenticated socket, not on the
process group, so idle workers block on ``recv`` without a collective timeout. One group training
runs at a time (the group's lock); the process-wide default context stays world size 1, so CPU
models and inference in the server never issue collectives.

Failure handling: a watchdog thread polls the worker processes. A worker that dies
marks the group lost; if a training is in flight, the default process group is aborted so rank 0's
pending collectives fail instead of waiting out the collective timeout. A training whose workers
do not report back (lost worker, rank 0 failed while the others wait in a collective) tears the
group down (workers killed); the next ``train`` brings a fresh group up (new workers, new
rendezvous) before it runs. A failure every rank reports cleanly (e.g. a bad request) keeps the
group. ``status()`` exposes ``lost`` and ``restarts``.

Configuration: ``PZ_SERVICE_GPUS`` = unset / ``1`` (reference behaviour: no group), ``auto`` (every
visible GPU) or N. ``PZ_DIST_BACKEND`` overrides the backend (``gloo`` for CPU rehearsals).
"""
from __future__ import annotations

import logging
import os
import secrets
import subprocess
import sys
import threading
import time
from multiprocessing.connection import Listener

log = logging.getLogger("pz.service")

_GROUP: "TrainGroup | None" = None


def requested_world() -> int:
    raw = os.environ.get("PZ_SERVICE_GPUS", "1").strip().lower()
    if raw in ("", "0", "1", "none", "off"):
        return 1
    if raw == "auto":
        import torch
        return max(1, torch.cuda.device_count())  # does not initialise HIP on this build
    return max(1, int(raw))


class TrainGroup:
    """Rank 0's handle on the worker ranks (see module docstring)."""

    def __init__(self, world: int, backend: str | None = None, timeout_s: float = 600.0):
        import torch
        self.world = world
        self.backend = backend or os.environ.get("PZ_DIST_BACKEND") or (
            "nccl" if torch.cuda.device_count() >= world else "gloo")
        self.timeout_s = timeout_s
        self._lock = threading.Lock()
        self._ready = threading.Event()
        self._error: str | None = None
        self.ctx = None
        self.trainings = 0   # group trainings completed on every rank
        self.restarts = 0    # fresh groups brought up after a failure
        self.conns: list = []
        self.procs: list[subprocess.Popen] = []
        self._lost: str | None = None      # why the current group is unusable (worker exit, no reply)
        self._in_flight = False
        self._stopping = False
        self._start()
        threading.Thread(target=self._watch, name="pz-train-watchdog", daemon=True).start()

    # ---------------------------------------------------------------------------------------
    def _start(self) -> None:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            master_port = s.getsockname()[1]
        key = secrets.token_bytes(16)
        self._listener = Listener(("127.0.0.1", 0), authkey=key)
        models_dir = os.path.abspath(os.environ.get("PZ_MODELS_DIR", "models"))
        base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port), WORLD_SIZE=str(self.world),
                    LOCAL_WORLD_SIZE=str(self.world), PZ_DIST_BACKEND=self.backend, PZ_MODELS_DIR=models_dir,
                    PZ_CTRL_ADDR="%s:%d" % self._listener.address, PZ_CTRL_KEY=key.hex())
        base.pop("PZ_SERVICE_GPUS", None)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        base["PYTHONPATH"] = root + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
        # workers first: this process must not have initialised the GPU when they are started
        for r in range(1, self.world):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            self.procs.append(subprocess.Popen([sys.executable, "-m", "penr_oz_neural_network_torch_amd.parallel.worker"],
                                               env=env, cwd=os.getcwd()))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(master_port))
        threading.Thread(target=self._join, name="pz-train-group", daemon=True).start()

    def _join(self) -> None:
        """Rendezvous (blocks until every worker has imported torch and connected)."""
        try:
            from datetime import timedelta

            import torch
            import torch.distributed as dist

            from .dist import DataParallelContext, set_context
            conns: dict[int, object] = {}
            while len(conns) < self.world - 1:
                c = self._listener.accept()
                rank = c.recv()
                conns[int(rank)] = c
            self.conns = [conns[r] for r in sorted(conns)]
            set_context(DataParallelContext())  # everything else in this process stays single-rank
            if self.backend == "nccl":
                torch.cuda.set_device(0)
            dist.init_process_group(self.backend, rank=0, world_size=self.world,
                                    timeout=timedelta(seconds=self.timeout_s))
            comm = os.environ.get("PZ_GRAD_COMM_DTYPE")
            comm_dtype = torch.bfloat16 if comm in ("bf16", "bfloat16") else None
            self.ctx = DataParallelContext(0, self.world, None, comm_dtype)
            log.info(f"data-parallel train group up: {self.world} ranks over {self.backend}")
        except Exception as e:  # pragma: no cover - environment failures
            self._error = repr(e)
            log.exception("train group rendezvous failed")
        finally:
            self._ready.set()

    # ---------------------------------------------------------------------------------------
    @property
    def healthy(self) -> bool:
        return (self._ready.is_set() and self._error is None and self._lost is None
                and all(p.poll() is None for p in self.procs))

    def status(self) -> dict:
        return {"world_size": self.world, "backend": self.backend, "ready": self._ready.is_set(),
                "healthy": self.healthy, "error": self._error, "trainings": self.trainings,
                "lost": self._lost, "restarts": self.restarts}

    def _watch(self) -> None:
        """Worker-exit watchdog: mark the group lost; abort in-flight collectives on rank 0."""
        while not self._stopping:
            gen = self.procs  # the list object is replaced on restart: ignore exits of a torn-down group
            for r, p in enumerate(list(gen), 1):
                if p.poll() is not None and self._lost is None and not self._stopping and gen is self.procs:
                    self._lost = f"worker rank {r} exited with code {p.returncode}"
                    log.error("data-parallel group lost: %s", self._lost)
                    if self._in_flight:
                        self._abort_collectives()
            time.sleep(0.2)

    def _abort_collectives(self) -> None:
        try:
            import torch.distributed as dist
            from torch.distributed.distributed_c10d import _abort_process_group
            if dist.is_initialized():
                _abort_process_group()
        except Exception:  # gloo: the dead peer's sockets already fail the pending collectives
            log.debug("process group abort unavailable", exc_info=True)

    def _teardown(self) -> None:
        """Stop (or kill) the workers and drop the process group (failure path and shutdown)."""
        lost = self._lost is not None
        for c in self.conns:
            try:
                if not lost:
                    c.send({"op": "stop"})
                c.close()
            except OSError:
                pass
        for p in self.procs:
            try:
                if lost:
                    p.kill()
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:  # pragma: no cover
                p.kill()
        try:
            import torch.distributed as dist
            if self._ready.is_set() and self._error is None and dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # pragma: no cover - an aborted group may refuse a clean destroy
            log.debug("destroy_process_group after failure", exc_info=True)
        self._listener.close()

    def restart(self) -> None:
        """Replace a lost group: kill what is left of it, spawn fresh workers, rendezvous again."""
        log.warning("restarting the data-parallel train group (%s)", self._lost or self._error)
        self._lost = self._lost or "restart"
        self._teardown()
        self._ready.clear()
        self._error = None
        self.conns = []
        self.procs = []
        self._lost = None
        self.restarts += 1
        self._start()

    def wait_ready(self, timeout: float | None = None) -> bool:
        return self._ready.wait(timeout) and self._error is None

    def train(self, model, data, hp: dict) -> None:
        """Run ``model.train(data, **hp)`` on every rank (called from the service's train thread)."""
        with self._lock:
            if self._lost is not None or (self._ready.is_set() and not self.healthy):
                self.restart()
            if not self.wait_ready(self.timeout_s):
                raise RuntimeError(f"data-parallel train group unavailable: {self._error or 'rendezvous timeout'}")
            if not self.healthy:
                raise RuntimeError(f"data-parallel train group lost: {self._lost or 'a worker process has exited'}")
            cmd = {"op": "load", "model_id": model.model_id, "data": data, "hp": hp}
            for c in self.conns:
                c.send(cmd)
            replies = [c.recv() for c in self.conns]
            failed = [f"rank {r + 1}: {m}" for r, m in enumerate(replies) if m != "ok"]
            for c in self.conns:
                c.send("abort" if failed else "go")
            if failed:
                raise RuntimeError("data-parallel workers could not load the model: " + "; ".join(failed))
            model._context = self.ctx
            err = None
            self._in_flight = True
            try:
                model.train(data, **hp)
            except Exception as e:
                err = e
            finally:
                model._context = None
                self._in_flight = False
            # workers report "done" / "failed: ..."; no reply (dead worker, or workers stuck in a
            # collective rank 0 left) means the group is unusable: tear it down now
            results = []
            for c in self.conns:
                wait = self.timeout_s if err is None else 15.0
                try:
                    results.append(c.recv() if c.poll(wait) else None)
                except (EOFError, OSError):
                    results.append(None)
            if any(m is None for m in results) or self._lost is not None:
                self._lost = self._lost or "a worker did not report the end of the training"
                log.error("data-parallel training lost its group: %s", self._lost)
                self._teardown()
            bad = [f"rank {r + 1}: {m}" for r, m in enumerate(results) if m != "done"]
            if err is not None:
                raise err
            if bad:
                raise RuntimeError("data-parallel workers failed: " + "; ".join(bad))
            self.trainings += 1

    def shutdown(self) -> None:
        self._stopping = True
        self._teardown()


def start_from_env() -> "TrainGroup | None":
    """Bring the group up if ``PZ_SERVICE_GPUS`` asks for more than one rank (service startup)."""
    global _GROUP
    world = requested_world()
    if world <= 1 or _GROUP is not None:
        return _GROUP
    _GROUP = TrainGroup(world)
    return _GROUP


def get_group() -> "TrainGroup | None":
    return _GROUP


def stop() -> None:
    global _GROUP
    if _GROUP is not None:
        _GROUP.shutdown()
        _GROUP = None


def train(model, data, hp: dict) -> None:
    """The service's training entry: GPU models train on every rank of the group when one is
    up, everything else trains in this thread exactly like the reference."""
    group = _GROUP
    # RCCL groups carry GPU models; a gloo group (CPU rehearsal) carries every model
    if group is not None and (group.backend == "gloo" or getattr(model, "on_gpu", False)):
        group.train(model, data, hp)
    else:
        model.train(data, **hp)
