"""Fused optimizer bound to a genuine ``torch.optim.Adam`` (reference R24).

The reference persists ``torch.optim.Adam.state_dict()`` to ``optimizer_<id>.pth``
(``neural_net_model.py:338-341, 351-354``). A GPU model keeps that object — so checkpoints stay
interchangeable — but its ``exp_avg`` / ``exp_avg_sq`` state tensors are *views into flat device
buffers* that the single-launch fused kernel (``pz::optimizer_step``) updates in place, and its
per-parameter ``step`` counters are kept in sync. ``optimizer=None`` models get the reference's
manual SGD (``p -= lr * grad``) from the same kernel.

Also owned here: the per-step statistics the reference computes with clones and host syncs
(``weight_upd_ratio``, the L2 term's ``sum(w**2)``) — accumulated in-kernel into a double-buffered
device array and turned into ``costs[epoch]`` / ``ratios[row]`` by ``pz::step_finalize``.
"""
from __future__ import annotations

import math

import torch

from .params import ParamStore

ELEMS_PER_BLOCK = 4096  # keep in sync with kOptElemsPerBlock (csrc/pz_kernels.h)


class FusedOptimizer:
    def __init__(self, store: ParamStore, params: list[torch.Tensor], torch_opt: torch.optim.Optimizer | None,
                 shadows: dict[int, torch.Tensor] | list[dict[int, torch.Tensor]],
                 grads16: dict[int, torch.Tensor] | None = None):
        # shadows: low-precision weight copies the update writes; a LIST of dicts = ping-pong sets
        # selected per launch by `parity` (the trainer reads one set while the other is written)
        # grads16: segment offset -> bf16 gradient view that replaces the fp32 gradient of that
        # segment (data parallel: dense weight gradients are produced and all-reduced in bf16)
        shadow_sets = shadows if isinstance(shadows, list) else [shadows]
        self.grads16 = grads16 or {}
        self.store = store
        self.params = params
        self.torch_opt = torch_opt
        self.adam = torch_opt is not None
        dev = store.device
        n = store.numel
        dt = store.flat.dtype  # fp32 masters, or fp64 (fp64 models: torch.optim.Adam's fp64 state)
        self.exp_avg = torch.zeros(n, device=dev, dtype=dt) if self.adam else None
        self.exp_avg_sq = torch.zeros(n, device=dev, dtype=dt) if self.adam else None
        self.step_count = 0
        if self.adam:
            self._adopt_state()

        segs = sorted(store.segments, key=lambda s: s.offset)
        self.weight_slots = [s for s in store.segments if s.is_weight]
        self.weight_slots.sort(key=lambda s: s.param_index)
        slot_of = {id(s): i for i, s in enumerate(self.weight_slots)}
        blocks = [max(1, math.ceil(s.numel / ELEMS_PER_BLOCK)) for s in segs]
        starts, acc = [], 0
        for b in blocks:
            starts.append(acc)
            acc += b
        self.total_blocks = acc
        self.slot_of = slot_of
        self.shadow_sets = shadow_sets
        self.amax_sets: list[dict[int, torch.Tensor]] = [{} for _ in shadow_sets]
        # fp8 policy, per parity: segment offset -> (e4m3 copy, previous amax, {q, 1/q} record) that
        # the update writes itself (delayed weight scaling; set_w8)
        self.w8_sets: list[dict[int, tuple]] = [{} for _ in shadow_sets]
        self._segs = segs
        self._pack_all()
        self.block_seg = torch.tensor(starts, dtype=torch.int64, device=dev)
        self.num_segments = len(segs)
        self.nslots = len(self.weight_slots)
        self.slot_numel = torch.tensor([float(s.numel) for s in self.weight_slots] or [1.0], dtype=torch.float64,
                                       device=dev)
        # double-buffered per-slot stats: sum(dw), sum(dw^2), sum(w), sum(w^2)
        self.stats = [torch.zeros(max(1, self.nslots) * 4, device=dev, dtype=torch.float64) for _ in range(2)]
        self.cur = 0
        self.groups: dict = {}
        # (hp table, epoch counter) while a hipGraph is being captured: the kernels then read the
        # epoch's lr / bias corrections from the table instead of the baked-in scalars
        self.graph_tables = None

    def define_groups(self, keys: list[int], rest_stats: bool = True, replicated=()) -> None:
        """Split the update into launches: one per listed segment offset (a dense weight whose
        gradient bucket is ready early in the backward) plus one for every other segment. Each
        launch is the same fused kernel over its own packed segment table. ``rest_stats=False``:
        the rest group and the listed ``replicated`` keys add nothing to the per-weight statistics
        (sharded optimizer, ranks > 0: rank 0's replicated copy counts once in the all-reduced
        sums)."""
        dev = self.store.device
        by_off = {s.offset: s for s in self.store.segments}
        rest = sorted((s for s in self.store.segments if s.offset not in set(keys)), key=lambda s: s.offset)
        for key, segs in [(k, [by_off[k]]) for k in keys] + [("rest", rest)]:
            if not segs:
                continue
            blocks = [max(1, math.ceil(s.numel / ELEMS_PER_BLOCK)) for s in segs]
            starts, acc = [], 0
            for b in blocks:
                starts.append(acc)
                acc += b
            block_seg = torch.tensor(starts, dtype=torch.int64, device=dev)
            stats = rest_stats or (key != "rest" and key not in replicated)
            for parity in range(len(self.shadow_sets)):
                self.groups[(key, parity)] = (self._pack(segs, parity, stats), block_seg, len(segs), acc)

    def define_slice(self, key, seg, lo: int, numel: int, shadows: list[torch.Tensor | None],
                     grad16: torch.Tensor) -> None:
        """A group updating only elements ``[lo, lo + numel)`` of weight segment ``seg`` (the
        sharded optimizer's slice of this rank): masters / moments at ``seg.offset + lo``, the
        gradient from ``grad16`` (the reduce-scattered bf16 slice), per parity the shadow slice
        ``shadows[parity]`` it writes. Same statistics slot as the whole weight (its sums are
        all-reduced over the ranks before step_finalize)."""
        dev = self.store.device
        blocks = max(1, math.ceil(numel / ELEMS_PER_BLOCK))
        block_seg = torch.tensor([0], dtype=torch.int64, device=dev)
        for parity in range(len(self.shadow_sets)):
            pack = torch.ops.pz.pack_segments(
                [seg.offset + lo], [numel], [int(seg.is_weight)], [self.slot_of.get(id(seg), -1)],
                [shadows[parity]], [grad16], [0], [None], [None], [None], [None]).to(dev)
            self.groups[(key, parity)] = (pack, block_seg, 1, blocks)

    def _pack(self, segs, parity: int, stats: bool = True) -> torch.Tensor:
        sh, am, w8 = self.shadow_sets[parity], self.amax_sets[parity], self.w8_sets[parity]
        trip = [w8.get(s.offset, (None, None, None)) for s in segs]
        return torch.ops.pz.pack_segments(
            [s.offset for s in segs], [s.numel for s in segs], [int(s.is_weight) for s in segs],
            [self.slot_of.get(id(s), -1) if stats else -1 for s in segs], [sh.get(s.offset) for s in segs],
            [self.grads16.get(s.offset) for s in segs], self._zero_flags(segs),
            [am.get(s.offset) for s in segs], [t[0] for t in trip], [t[1] for t in trip],
            [t[2] for t in trip]).to(self.store.device)

    def _pack_all(self) -> None:
        self.segments_p = [self._pack(self._segs, p) for p in range(len(self.shadow_sets))]
        self.segments = self.segments_p[0]

    def set_amax(self, amax_sets: list[dict[int, torch.Tensor]]) -> None:
        """fp8 policy: per parity, segment offset -> fp32 scalar that the update max-es |w_new| into
        (the weight's current-scaling amax, consumed by the transpose-quantise that follows).
        Call before define_groups()."""
        assert len(amax_sets) == len(self.shadow_sets)
        self.amax_sets = amax_sets
        self._pack_all()

    def set_w8(self, w8_sets: list[dict[int, tuple]]) -> None:
        """fp8 policy: per parity, segment offset -> ``(w8, amax_prev, qs)``: the update writes the
        weight's e4m3 copy itself, scaled by q = 448 / amax_prev (the amax the previous update
        reduced: delayed weight scaling), and publishes {q, 1/q} into ``qs``. Call before
        define_groups()."""
        assert len(w8_sets) == len(self.shadow_sets)
        self.w8_sets = w8_sets
        self._pack_all()

    def _zero_flags(self, segs) -> list[int]:
        """Accumulated-gradient segments (biases, batchnorm, embeddings: filled by atomics and
        column sums) are reset to zero by the update kernel right after it reads them, which
        replaces a per-step zeroing pass; dense GEMM-written gradients are overwritten anyway."""
        return [int(s.offset >= self.store.accum_offset) for s in segs]

    # ------------------------------------------------------------------------------------
    def _adopt_state(self) -> None:
        """Move any existing Adam state into the flat buffers and re-point the state at views."""
        opt = self.torch_opt
        steps = []
        for seg in self.store.segments:
            p = self.params[seg.param_index]
            st = opt.state.get(p, {})
            m_view = self.store.view(seg, self.exp_avg)
            v_view = self.store.view(seg, self.exp_avg_sq)
            if "exp_avg" in st:
                m_view.copy_(st["exp_avg"].reshape(seg.shape))
                v_view.copy_(st["exp_avg_sq"].reshape(seg.shape))
                steps.append(float(st["step"]))
            step_t = st.get("step")
            if not isinstance(step_t, torch.Tensor):
                step_t = torch.tensor(0.0, dtype=torch.float32)
            opt.state[p] = {"step": step_t, "exp_avg": m_view, "exp_avg_sq": v_view}
        self.step_count = int(max(steps)) if steps else 0

    def sync_torch_state(self) -> None:
        """Publish the fused step counter into the torch optimizer's state (before saving)."""
        if not self.adam:
            return
        for p in self.params:
            st = self.torch_opt.state.get(p)
            if st is not None:
                st["step"].fill_(float(self.step_count))

    # ------------------------------------------------------------------------------------
    # update-ratio sums in the next launches: 1 = yes, 0 = no (sum(w^2) only), k > 1 = on device
    # epochs divisible by k (graph capture; needs graph_tables)
    stats_every = 1

    def init_stats(self) -> None:
        """sum(w^2) of the current weights into the 'previous' stats buffer (L2 term of step 0)."""
        prev = self.stats[1 - self.cur]
        prev.zero_()
        self.stats[self.cur].zero_()
        torch.ops.pz.segment_stats(self.store.flat, self.segments, self.block_seg, self.num_segments,
                                   self.total_blocks, prev)

    def step(self, grads: torch.Tensor, lr: float, l2: float, grad_scale: float, parity: int = 0) -> None:
        self.begin_step(lr)
        self._launch(grads, self.segments_p[parity], self.block_seg, self.num_segments, self.total_blocks, l2,
                     grad_scale)

    def step_group(self, key, grads: torch.Tensor, l2: float, grad_scale: float, parity: int = 0,
                   max_grid: int = 0) -> None:
        """Update one group (define_groups) with the hyper-parameters of the last begin_step().
        ``max_grid`` > 0 caps the workgroups (a background 'trickle' beside the GEMMs)."""
        g = self.groups.get((key, parity))
        if g is not None:
            self._launch(grads, *g, l2, grad_scale, max_grid)

    def gemm_update(self, a: torch.Tensor, a_kc: bool, b: torch.Tensor, b_kc: bool, seg, l2: float,
                    grad_scale: float, parity: int = 0) -> None:
        """The weight-gradient GEMM ``op(a) @ op(b)`` of segment ``seg`` with this weight's update
        fused into its epilogue (``pz::gemm_update``, EPI_OPT): the gradient is never stored. Same
        hyper-parameters, statistics and shadow / amax targets as :meth:`step_group` would use."""
        lr, b1, b2, eps, bc1, bc2s = self._hp
        hp, ctr = self.graph_tables or (None, None)
        every = self.stats_every
        if every > 1 and ctr is None:
            every = 1
        slot = self.slot_of.get(id(seg))
        stats = self.stats[self.cur][4 * slot:4 * slot + 4] if slot is not None else None
        view = self.store.view
        w = view(seg)  # also the layout of the (never stored) gradient
        M, N = w.shape
        K = a.shape[1] if a_kc else a.shape[0]
        torch.ops.pz.gemm_update(a, a_kc, b, b_kc, w, M, N, K, 1.0, w,
                                 view(seg, self.exp_avg) if self.adam else None,
                                 view(seg, self.exp_avg_sq) if self.adam else None,
                                 self.shadow_sets[parity].get(seg.offset), stats,
                                 self.amax_sets[parity].get(seg.offset), self.adam, lr, b1, b2, eps, bc1, bc2s,
                                 grad_scale, l2, hp, ctr, every)

    def begin_step(self, lr: float) -> None:
        if self.adam:
            group = self.torch_opt.param_groups[0]
            b1, b2 = group["betas"]
            eps = group["eps"]
            self.step_count += 1
            bc1 = 1.0 - b1 ** self.step_count
            bc2s = math.sqrt(1.0 - b2 ** self.step_count)
            group["lr"] = lr
        else:
            b1 = b2 = eps = 0.0
            bc1 = bc2s = 1.0
        self._hp = (lr, b1, b2, eps, bc1, bc2s)

    def _launch(self, grads, segments, block_seg, nseg, nblocks, l2: float, grad_scale: float,
                max_grid: int = 0) -> None:
        lr, b1, b2, eps, bc1, bc2s = self._hp
        hp, ctr = self.graph_tables or (None, None)
        every = self.stats_every
        if every > 1 and ctr is None:  # eager: the caller knows whether this is a progress epoch
            every = 1
        torch.ops.pz.optimizer_step(self.store.flat, grads, self.exp_avg, self.exp_avg_sq, segments, block_seg, nseg,
                                    nblocks, self.adam, lr, b1, b2, eps, bc1, bc2s, grad_scale, l2,
                                    self.stats[self.cur], hp, ctr, every, max_grid)

    def finalize(self, loss: torch.Tensor | None, world: int, l2: float, costs: torch.Tensor, epoch: int,
                 ratios: torch.Tensor, ratio_row: int, epoch_ctr: torch.Tensor | None = None, every: int = 1,
                 clear: torch.Tensor | None = None) -> None:
        """cost[epoch] and the update-ratio row; ``epoch=-1`` / ``ratio_row=-2``: taken from the
        device ``epoch_ctr`` (graph-replayed step), which is advanced to epoch + 1 either way.
        ``clear``: fp32 accumulators to reset (the weight-amax slots this step's updates read)."""
        prev = self.stats[1 - self.cur]
        torch.ops.pz.step_finalize(loss, float(world), prev, self.stats[self.cur], self.slot_numel, self.nslots, l2,
                                   costs, epoch, ratios, ratio_row, epoch_ctr, every, clear)
        self.cur = 1 - self.cur
