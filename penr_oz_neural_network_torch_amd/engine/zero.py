"""Sharded optimizer for data parallelism (ZeRO stage 1) — the fused trainer's DP update.

Replicated data parallelism (the round-1..5 design) all-reduces every dense weight gradient and
then runs the FULL Adam update on every rank: each rank streams all 25 M (mlp4) ... 1.07 B
(``[8192]x17``) parameters' fp32 master, gradient and both moments through HBM every step, the
same work N times over. Here each rank owns a contiguous 1/N slice of every dense GEMM weight:

    dW GEMM -> bf16 gradient [n, padded to N*s]
            -> reduce-scatter (RCCL over xGMI): rank r receives the SUM of slice r   [s]
            -> fused Adam / SGD on slice r only (fp32 master, m, v at seg.offset + r*s;
               writes the bf16 GEMM copy of slice r into the next step's shadow set)
            -> all-gather of the bf16 slices, in place, into every rank's shadow     [N*s]

A ring reduce-scatter plus a ring all-gather move exactly the bytes of one ring all-reduce, so the
xGMI traffic is unchanged while the optimizer's HBM traffic and kernel time per rank fall by N
(and the first-layer update on the step boundary with it). Small accumulated parameters (biases,
batchnorm, embeddings) and the loss stay in the exact replicated fp32 bucket. The per-weight
statistics (update-ratio sums, sum(w^2) for the L2 cost) are partial per rank and are summed by
one small exact all-reduce before ``step_finalize``.

Masters and Adam moments are only current on their owner between synchronisation points:
:meth:`ZeroShards.gather_state` all-gathers them (fp32) before anything reads whole tensors — a
record step (its weight gradients add ``2 l2 W``), ``drain()`` (checkpoints, the end of training).
The ``.pth`` checkpoint therefore stays a full ``torch.optim.Adam.state_dict()`` (reference
``neural_net_model.py:338-341, 351-354``).

Reference: ``neural_net_model.py:496-500`` (the optimizer step this distributes).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 64  # slice boundaries on 64 elements: 256-B aligned vector kernels and RCCL chunks


@dataclass
class Shard:
    seg: object              # the weight's params.Segment
    n: int                   # elements of the weight
    s: int                   # elements per rank's slice (padded)
    lo: int                  # this rank's first element
    cnt: int                 # this rank's real elements (<= s; 0 for a tiny weight's last ranks)
    g_full: torch.Tensor     # [world * s] bf16 gradient (the dW GEMM writes [:n]; the tail stays 0)
    g_shard: torch.Tensor    # [s] bf16: the reduce-scattered sum of this rank's slice
    sh_full: list            # per shadow parity: [world * s] bf16 storage of the GEMM weight copy


class ZeroShards:
    def __init__(self, ctx, dense_segments, shadow_parities: int, device: torch.device):
        self.ctx = ctx
        ctx.open_side_comm()  # all-gathers + statistics on a communicator of their own
        self.world = ctx.shard_world
        self.rank = ctx.shard_rank
        self.shards: dict[int, Shard] = {}
        for seg in dense_segments:
            n = seg.numel
            s = -(-(-(-n // self.world)) // ALIGN) * ALIGN  # ceil(ceil(n / world) / ALIGN) * ALIGN
            lo = self.rank * s
            cnt = max(0, min(s, n - lo))
            full = self.world * s
            self.shards[seg.offset] = Shard(
                seg, n, s, lo, cnt,
                g_full=torch.zeros(full, device=device, dtype=torch.bfloat16),
                g_shard=torch.zeros(s, device=device, dtype=torch.bfloat16),
                sh_full=[torch.zeros(full, device=device, dtype=torch.bfloat16) for _ in range(shadow_parities)])

    # ---- views the trainer / optimizer use ------------------------------------------------------
    def grad_view(self, off: int) -> torch.Tensor:
        sh = self.shards[off]
        return sh.g_full[:sh.n].view(sh.seg.shape)

    def shadow_view(self, off: int, parity: int) -> torch.Tensor:
        sh = self.shards[off]
        return sh.sh_full[parity][:sh.n].view(sh.seg.shape)

    def define_groups(self, opt) -> None:
        """One optimizer group per weight and gradient source: ("z", off, "rs") reads the
        reduce-scattered slice, ("z", off, "ar") this rank's slice of an all-reduced gradient
        (record steps, whose statistics need the whole reduced gradient)."""
        for off, sh in self.shards.items():
            if sh.cnt == 0:
                continue
            shadows = [f[sh.lo:sh.lo + sh.cnt] for f in sh.sh_full]
            opt.define_slice(("z", off, "rs"), sh.seg, sh.lo, sh.cnt, shadows, sh.g_shard[:sh.cnt])
            opt.define_slice(("z", off, "ar"), sh.seg, sh.lo, sh.cnt, shadows, sh.g_full[sh.lo:sh.lo + sh.cnt])

    # ---- collectives ----------------------------------------------------------------------------
    def reduce_scatter(self, off: int):
        sh = self.shards[off]
        return self.ctx.reduce_scatter_async(sh.g_full, sh.g_shard)

    def all_reduce(self, off: int):
        """Record steps: the whole summed gradient on every rank."""
        return self.ctx.all_reduce_async(self.shards[off].g_full)

    def update(self, opt, off: int, grads: torch.Tensor, l2: float, scale: float, parity: int, source: str = "rs",
               side: bool = True):
        """This rank's slice update into shadow set ``parity``, then the all-gather of that set
        (in place). Returns the all-gather's handle (the reader waits for it). ``side``: on the
        second communicator (updates on the side stream); the step-end update on the compute
        stream gathers on the bucket communicator, behind that step's last reduce-scatters, where
        no side-stream update can hold it."""
        sh = self.shards[off]
        if sh.cnt > 0:
            opt.step_group(("z", off, source), grads, l2, scale, parity)
        full = sh.sh_full[parity]
        return self.ctx.all_gather_async(full[sh.lo:sh.lo + sh.s], full, side=side)

    def all_reduce_stats(self, stats: torch.Tensor) -> None:
        """Sum the per-weight statistics partials over the ranks (stream-ordered on the current
        stream; exact fp64)."""
        self.ctx.wait_one(self.ctx.side_all_reduce_async(stats))

    def gather_state(self, flat: torch.Tensor, *moments: torch.Tensor | None) -> None:
        """All-gather every weight's fp32 master (and Adam moments) from the slice owners, so
        every rank holds whole, current tensors (checkpoints, record steps, inference)."""
        if getattr(self.ctx.native, "model_world", None):
            return  # (one-GPU collective proxy: there are no other slice owners to gather from)
        for sh in self.shards.values():
            for buf in (flat,) + moments:
                if buf is None:
                    continue
                part = torch.zeros(sh.s, device=buf.device, dtype=buf.dtype)
                part[:sh.cnt].copy_(buf[sh.seg.offset + sh.lo:sh.seg.offset + sh.lo + sh.cnt])
                full = torch.empty(self.world * sh.s, device=buf.device, dtype=buf.dtype)
                self.ctx.wait_one(self.ctx.all_gather_async(part, full))
                buf[sh.seg.offset:sh.seg.offset + sh.n].copy_(full[:sh.n])
