"""Multi-GPU data-parallel training behind the REST service (reference ``main.py:281-298``).

The reference trains in one worker thread of one process (``run_in_threadpool(model.train, ...)``).
Here the server process drives an **N-rank train group of its own child processes**: at startup
it spawns N rank processes (rank r on GPU r; before this process touches the GPU) that join one
``torch.distributed`` process group — RCCL over xGMI for GPU models (``gloo`` when rehearsing on
the CPU). The server itself never joins the group, so no collective state ever lives in the
process that serves HTTP. A ``PUT /train/`` on a GPU model then runs on every rank:

    server (train thread)                         ranks 0..N-1 (parallel/worker.py)
    ─────────────────────                         ─────────────────────────────────
    send {"op": "load", model_id, data, hp} ────► deserialize model_<id> from the shared models/ dir
                                              ◄── "ok" | error text
    send "go" (or "abort" if any rank failed) ──►
    wait, watching the processes                  model.train(data, **hp) ◄═ RCCL ═► (every rank)
                                              ◄── "done" | "failed: ..."   (rank 0 writes the files)

Inside ``train`` the fused engine shards every epoch's minibatch over the ranks and all-reduces
the gradient buckets during backward (:mod:`.dist`, :class:`..engine.trainer.FusedTrainer`); the
model writes its checkpoints on rank 0 only, and ``/progress/`` reads them as for any model.
Commands travel on a local authenticated socket, not on the process group, so idle ranks block
on ``recv`` without a collective timeout. One group training runs at a time (the group's lock).

Failure handling: a watchdog thread polls the rank processes. A rank that exits
marks the group lost; a training in flight then fails at once — the server stops waiting, kills
every rank of that group (the survivors may be stuck in a collective) and, since rank 0 may have
died with it, rewrites the checkpoint's status as ``"Failed"`` itself (no GPU involved). The next
``train`` brings a fresh group up: new processes, a new file rendezvous in a fresh directory,
a new process group — nothing is re-initialised inside a process whose group was aborted. Ranks
that do not answer a command within ``timeout_s`` count as lost too. A failure every rank reports
cleanly (e.g. a bad request) keeps the group. ``status()`` exposes ``lost`` and ``restarts``.

Configuration: ``PZ_SERVICE_GPUS`` = unset / ``1`` (reference behaviour: no group), ``auto`` (every
visible GPU) or N. ``PZ_DIST_BACKEND`` overrides the backend (``gloo`` for CPU rehearsals).
"""
from __future__ import annotations

import logging
import os
import secrets
import shutil
import subprocess
import sys
import tempfile
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
    """The server's handle on its rank processes (see module docstring)."""

    def __init__(self, world: int, backend: str | None = None, timeout_s: float = 600.0):
        import torch
        self.world = world
        self.backend = backend or os.environ.get("PZ_DIST_BACKEND") or (
            "nccl" if torch.cuda.device_count() >= world else "gloo")
        self.timeout_s = timeout_s
        self._lock = threading.Lock()
        self._ready = threading.Event()
        self._error: str | None = None
        self.trainings = 0   # group trainings completed on every rank
        self.restarts = 0    # fresh groups brought up after a failure
        self.conns: list = []
        self.procs: list[subprocess.Popen] = []
        self._lost: str | None = None      # why the current group is unusable (rank exit, no reply)
        self._in_flight = False
        self._stopping = False
        self._rdv_dir: str | None = None
        self._start()
        threading.Thread(target=self._watch, name="pz-train-watchdog", daemon=True).start()

    # ---------------------------------------------------------------------------------------
    def _start(self) -> None:
        # one generation of the group: its own control socket, its own rendezvous directory (a
        # file store: no TCP port picked here that someone else could take first)
        self._rdv_dir = tempfile.mkdtemp(prefix="pz_group_")
        key = secrets.token_bytes(16)
        self._listener = Listener(("127.0.0.1", 0), authkey=key)
        models_dir = os.path.abspath(os.environ.get("PZ_MODELS_DIR", "models"))
        base = dict(os.environ, MASTER_ADDR="127.0.0.1", WORLD_SIZE=str(self.world),
                    LOCAL_WORLD_SIZE=str(self.world), PZ_DIST_BACKEND=self.backend, PZ_MODELS_DIR=models_dir,
                    PZ_RENDEZVOUS_FILE=os.path.join(self._rdv_dir, "store"),
                    PZ_CTRL_ADDR="%s:%d" % self._listener.address, PZ_CTRL_KEY=key.hex())
        base.pop("PZ_SERVICE_GPUS", None)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        base["PYTHONPATH"] = root + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
        for r in range(self.world):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            self.procs.append(subprocess.Popen([sys.executable, "-m", "penr_oz_neural_network_torch_amd.parallel.worker"],
                                               env=env, cwd=os.getcwd()))
        threading.Thread(target=self._join, args=(self._listener, self.procs), name="pz-train-group",
                         daemon=True).start()

    def _join(self, listener, procs) -> None:
        """Rendezvous: every rank connects, then reports "ready" once its process group is up."""
        try:
            conns: dict[int, object] = {}
            while len(conns) < self.world:
                c = listener.accept()
                conns[int(c.recv())] = c
            ordered = [conns[r] for r in range(self.world)]
            for r, c in enumerate(ordered):
                if not c.poll(self.timeout_s):
                    raise RuntimeError(f"rank {r} did not join the process group")
                msg = c.recv()
                if msg != "ready":
                    raise RuntimeError(f"rank {r}: {msg}")
            if procs is self.procs:
                self.conns = ordered
                log.info(f"data-parallel train group up: {self.world} ranks over {self.backend}")
        except Exception as e:  # rendezvous failure, or the listener closed by a teardown
            if procs is self.procs:
                self._error = repr(e)
                log.exception("train group rendezvous failed")
        finally:
            if procs is self.procs:
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
        """Rank-exit watchdog: mark the group lost (an in-flight training notices at once)."""
        while not self._stopping:
            gen = self.procs  # the list object is replaced on restart: ignore exits of a torn-down group
            for r, p in enumerate(list(gen)):
                if p.poll() is not None and self._lost is None and not self._stopping and gen is self.procs:
                    self._lost = f"rank {r} exited with code {p.returncode}"
                    log.error("data-parallel group lost: %s", self._lost)
            time.sleep(0.2)

    def _teardown(self) -> None:
        """Stop the ranks (cleanly, or killed when the group is lost) and drop this generation."""
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
                p.wait()
        self._listener.close()
        if self._rdv_dir is not None:
            shutil.rmtree(self._rdv_dir, ignore_errors=True)
            self._rdv_dir = None

    def restart(self) -> None:
        """Replace a lost group by a fresh generation of rank processes."""
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

    def _collect(self, timeout: float | None, straggler_s: float | None = None, rank0_grace_s: float = 0.0) -> list:
        """One reply per rank; ``None`` for a rank that did not answer (closed, or ``timeout`` s
        passed). Stops early once the watchdog marks the group lost. ``straggler_s``: once ANY
        rank has answered, the others must answer within that many seconds — a training may run
        for hours, but its ranks finish together (every step ends in a collective), so a rank
        still silent long after a peer reported is hung (a kernel that never returns, a deadlock
        outside a collective) and must not hold the group lock forever. Rank 0 gets
        ``rank0_grace_s`` more: after the last collective it still drains progress and writes the
        final checkpoint (seconds to minutes for a large model), which no peer waits for."""
        out: list = [None] * len(self.conns)
        waiting = set(range(len(self.conns)))
        deadline = None if timeout is None else time.monotonic() + timeout
        first = None  # when the first reply arrived (arms the straggler windows)
        while waiting and self._lost is None:
            for r in sorted(waiting):
                c = self.conns[r]
                try:
                    if c.poll(0.05):
                        out[r] = c.recv()
                        waiting.discard(r)
                except (EOFError, OSError):
                    waiting.discard(r)
            now = time.monotonic()
            if straggler_s is not None and first is None and len(waiting) < len(self.conns):
                first = now
            if deadline is not None and now > deadline:
                break
            if first is not None:
                if any(r != 0 for r in waiting) and now > first + straggler_s:
                    break
                if 0 in waiting and now > first + straggler_s + rank0_grace_s:
                    break
        return out

    def _lose(self, why: str, model_id: str | None = None, rank0_done: bool = False) -> None:
        self._lost = self._lost or why
        log.error("data-parallel training lost its group: %s", self._lost)
        self._teardown()
        # rank 0 owned the files and may have died with the group: mark the model Failed, unless
        # rank 0 reported a completed training (its "Trained" checkpoint is final: a peer that
        # died afterwards does not undo it) or the persisted status is no longer "Training"
        if model_id is not None and not rank0_done:
            try:
                from ..utils import checkpoint as ckpt
                if ckpt.load_meta(model_id).get("status") == "Training":
                    ckpt.set_status(model_id, "Failed")
            except FileNotFoundError:  # no checkpoint at all: nothing to mark
                pass
            except Exception:  # pragma: no cover - keep the original failure
                log.exception(f"could not mark model {model_id} failed")

    def train(self, model, data, hp: dict) -> None:
        """Run ``model.train(data, **hp)`` on every rank (called from the service's train thread)."""
        with self._lock:
            if self._lost is not None or (self._ready.is_set() and not self.healthy):
                self.restart()
            if not self.wait_ready(self.timeout_s):
                raise RuntimeError(f"data-parallel train group unavailable: {self._error or 'rendezvous timeout'}")
            if not self.healthy:
                raise RuntimeError(f"data-parallel train group lost: {self._lost or 'a rank process has exited'}")
            cmd = {"op": "load", "model_id": model.model_id, "data": data, "hp": hp}
            for c in self.conns:
                c.send(cmd)
            replies = self._collect(self.timeout_s)  # a rank stuck in deserialize must not hang us
            if self._lost is not None or any(m is None for m in replies):
                self._lose("a rank did not answer the load command")
                raise RuntimeError(f"data-parallel train group lost: {self._lost}")
            failed = [f"rank {r}: {m}" for r, m in enumerate(replies) if m != "ok"]
            for c in self.conns:
                c.send("abort" if failed else "go")
            if failed:
                raise RuntimeError("data-parallel ranks could not load the model: " + "; ".join(failed))
            self._in_flight = True
            try:
                # until every rank reported, or the group is lost; once one rank reported, the
                # rest get the process-group timeout plus a margin, rank 0 also the time of its
                # final checkpoint write (~2 us per parameter, generously)
                grace = 120.0 + 2e-6 * float(getattr(model, "num_params", 0) or 0)
                results = self._collect(None, straggler_s=self.timeout_s + 60.0, rank0_grace_s=grace)
            finally:
                self._in_flight = False
            if self._lost is not None or any(m is None for m in results):
                self._lose("a rank did not report the end of the training", model.model_id,
                           rank0_done=bool(results) and results[0] == "done")
                raise RuntimeError(f"data-parallel training lost its group: {self._lost}")
            self._refresh(model)
            bad = [f"rank {r}: {m}" for r, m in enumerate(results) if m != "done"]
            if bad:
                raise RuntimeError("data-parallel training failed: " + "; ".join(bad))
            self.trainings += 1

    @staticmethod
    def _refresh(model) -> None:
        """The caller's model object mirrors what rank 0 persisted (status, progress, stats)."""
        try:
            from ..utils import checkpoint as ckpt
            meta = ckpt.load_meta(model.model_id)
        except Exception:  # pragma: no cover - informational only
            return
        model.progress = meta.get("progress", model.progress)
        model.avg_cost = meta.get("average_cost", model.avg_cost)
        model.avg_cost_history = meta.get("average_cost_history", model.avg_cost_history)
        model.stats = meta.get("stats", model.stats)
        model.status = meta.get("status", model.status)

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
