"""Device-resident fused trainer — the GPU implementation of the reference epoch loop.

Reference loop (``neural_net_model.py:459-522``) per epoch: sample with replacement, build an
input tensor from Python lists, clone all weights, forward with dropout on hidden outputs, add
the L2 term, backward through the autograd graph, Adam / SGD, ``.item()`` the cost and the
per-weight update ratios. Here the same math runs as an explicit schedule of ``torch.ops.pz``
HIP kernels with nothing on the host between epochs:

    gather_rows (on-device sampling + cast)  [+ embedding_fwd]
    per stage:  GEMM(+bias+dropout+act+dropout epilogue) | batchnorm(+epilogue) | flatten(+dropout)
    head:       xent_head / mse_head  (loss + dZ of the last stage + its bias-grad colsum)
    per stage, reversed:
                dW GEMM  (XᵀdZ straight into the gradient buffer, bf16; PZ_GRAD_DTYPE=fp32: fp32)
                -> async RCCL all-reduce of that bucket (data parallel)
                dX GEMM  (dZ Wᵀ with the previous stage's epilogue derivative + bias colsum fused)
                | batchnorm_bwd | embedding_bwd
    optimizer_step (one launch for all params, L2 folded in, bf16 shadows refreshed)
    step_finalize  (cost[e], weight_upd_ratio row -> device arrays)

Costs / ratios / progress timestamps are pulled off the device only in :meth:`drain` (end of
training, or the reference's 10 s checkpoint cadence). Epochs that feed the stats dashboard
(the last one, or a checkpoint epoch) run the *record* schedule instead: same kernels with
unfused epilogues so every layer output and its gradient exists for ``_record_training_overall_progress``.

A "stage" is a producing op plus the dropout / activation / dropout that follow it
(``linear [drop] [act [drop]]``, ``batchnorm [drop] [act [drop]]``, ``flatten [drop]``,
``embedding``); the algo normalisation of the reference guarantees every activation directly
follows a linear or batchnorm.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field
from datetime import datetime, timedelta

import torch

from ..ops import functional as PF
from ..ops import native
from ..parallel.dist import DataParallelContext, get_context
from .events import StreamEvents
from .fp8_policy import Fp8Policy
from .optim import FusedOptimizer
from .zero import ZeroShards

ROW_PAD = 64  # batch rows padded to the GEMM K-tile so dW = XᵀdZ stays on the MFMA path
_M32 = 0xFFFFFFFF
LOSS_SLOTS = 64
# Steps below this are launch-bound (measured on MI355X: [4,8,2] at batch 32 runs 0.093 ms/step
# replayed vs 0.172 eager; [256,1024,1024,64] at batch 1024 (8 GFLOP) is already GPU-bound and
# replays 5 % slower, as does the 1.2 TFLOP bench step: ROCm executes the captured side-stream
# branch with less overlap than eager streams)
GRAPH_MAX_FLOP = 4e9

# Tracing / debugging: PZ_TRACE=1 brackets every step phase in a roctx range
# (visible with `rocprofv3 --marker-trace`); PZ_DEBUG_SYNC=1 synchronises after every phase so an
# asynchronous kernel fault surfaces at the phase that caused it (combine with the runtime's
# AMD_SERIALIZE_KERNEL=3 for per-kernel attribution).
_TRACE = os.environ.get("PZ_TRACE", "0") == "1"
_DEBUG_SYNC = os.environ.get("PZ_DEBUG_SYNC", "0") == "1"




def _round_up(n: int, a: int) -> int:
    return (n + a - 1) // a * a


@dataclass
class Stage:
    kind: str                     # embed | flatten | gemm | bn
    first: int                    # first layer index covered
    layers: list[int]             # layer indices covered (for record mode)
    act: int = PF.ACT_NONE
    drop_pre: int = -1            # layer id of the dropout after the producing op
    act_layer: int = -1           # layer id of the activation (if any)
    drop_post: int = -1           # layer id of the dropout after the activation
    in_width: int = 0
    out_width: int = 0
    pos_in: int = 1               # positions per sample (rows = batch * pos)
    pos_out: int = 1
    seg_w: object = None
    seg_b: object = None
    layer: object = None
    buffers: dict = field(default_factory=dict)
    index: int = 0                # position in the stage list
    fp8: bool = False             # forward GEMM on e4m3 operands (fp8 policy)
    w8_index: int = -1            # row of the fp8 weight scale table

    @property
    def has_epi(self) -> bool:
        return self.act != PF.ACT_NONE or self.drop_pre >= 0 or self.drop_post >= 0


class UnsupportedModel(Exception):
    pass


def compile_stages(model) -> tuple[list[Stage], str]:
    """Group the model's layers into fused stages; returns (stages, head kind)."""
    layers, algos = model.layers, model.algos
    n = len(layers)
    stages: list[Stage] = []
    store = model._param_store
    head = "softmax" if algos[-1] == "softmax" else "mse"
    end = n - 1 if head == "softmax" else n
    pos, width = 1, None
    i = 0
    while i < end:
        a = algos[i]
        hid = layers[i].hidden
        if a == "embedding":
            if i != 0:
                raise UnsupportedModel("embedding must be the first layer")
            w = layers[i].weights
            st = Stage("embed", i, [i], seg_w=store.segment_for(i, "weights"), layer=layers[i],
                       in_width=0, out_width=w.shape[1])
            width = w.shape[1]
            st.pos_in = st.pos_out = -1  # resolved from the data (block size)
            stages.append(st)
            i += 1
            continue
        if a == "flatten":
            r = layers[i].ratio
            st = Stage("flatten", i, [i], drop_pre=i if hid else -1, layer=layers[i])
            st.in_width, st.out_width = width, width * r
            stages.append(st)
            width = width * r
            i += 1
            continue
        if a in ("linear", "batchnorm"):
            kind = "gemm" if a == "linear" else "bn"
            st = Stage(kind, i, [i], drop_pre=i if hid else -1, layer=layers[i])
            if kind == "gemm":
                st.seg_w = store.segment_for(i, "weights")
                st.seg_b = store.segment_for(i, "bias")
                st.in_width, st.out_width = layers[i].weights.shape
                if width is not None and width != st.in_width:
                    raise UnsupportedModel(f"width mismatch at layer {i}: {width} vs {st.in_width}")
            else:
                st.seg_w = store.segment_for(i, "gain")
                st.seg_b = store.segment_for(i, "bias")
                st.in_width = st.out_width = layers[i].gain.shape[0]
            width = st.out_width
            j = i + 1
            if j < end and algos[j] in ("relu", "sigmoid", "tanh"):
                st.act = PF.ACT_CODES[algos[j]]
                st.act_layer = j
                st.drop_post = j if layers[j].hidden else -1
                st.layers.append(j)
                j += 1
            stages.append(st)
            i = j
            continue
        raise UnsupportedModel(f"layer {i} ({a}) cannot start a fused stage")
    if not stages or stages[-1].kind not in ("gemm", "bn", "flatten"):
        raise UnsupportedModel("model must end in a linear/batchnorm stage before the head")
    if head == "softmax" and stages[-1].act != PF.ACT_NONE:
        raise UnsupportedModel("activation directly before softmax")
    return stages, head


class FusedTrainer(Fp8Policy):
    """Owns the device buffers of one GPU model's training run."""

    def __init__(self, model, context: DataParallelContext | None = None):
        native.require()
        if model._param_store is None or model._param_store.device.type != "cuda":
            raise UnsupportedModel("CPU models train under autograd (the reference's own runtime)")
        if model.precision.master not in (torch.float32, torch.float64):
            raise UnsupportedModel("fused engine needs fp32 or fp64 master parameters")
        self.model = model
        self.store = model._param_store
        self.dev = self.store.device
        # GEMM operand precision: bf16 (bf16 / fp8 policies, fp32 masters) or the master itself —
        # fp32 (f32 MFMA) or fp64 (f64 MFMA: the reference's own precision, a REST model created
        # with device="cuda" and no dtype); fp64 models also keep their gradients, Adam moments,
        # loss and bias-gradient accumulators and costs in fp64
        self.master = model.precision.master
        self.compute = torch.bfloat16 if model.precision.name in ("bfloat16", "fp8") else self.master
        self.ctx = context or get_context()
        self.stages, self.head = compile_stages(model)
        for i, st in enumerate(self.stages):
            st.index = i
        # LOSS_SLOTS loss accumulators after the parameters (inside the exact fp32 DP bucket): the
        # head's blocks spread their adds over them, step_finalize sums them
        self.grads = torch.zeros(self.store.numel + LOSS_SLOTS, device=self.dev, dtype=self.master)
        self.loss_slot = self.grads[self.store.numel:self.store.numel + LOSS_SLOTS]
        # low-precision GEMM copies of the weights, PING-PONG: step t's GEMMs read set `parity`
        # while its optimizer writes set 1-parity — so a weight can be updated as soon as its
        # gradient is reduced, even while the dX GEMM of the same layer still reads it
        self.shadow_sets: list[dict[int, torch.Tensor]] = [{}, {}]
        self.parity = 0
        # SHARDED OPTIMIZER under data parallelism (ZeRO-1, engine/zero.py; PZ_ZERO=0 replicates):
        # every dense weight's bf16 gradient is reduce-scattered, each rank updates its 1/N slice of
        # the fp32 master and Adam moments, and the bf16 GEMM copies are all-gathered in place —
        # the xGMI bytes of one all-reduce, 1/N of the optimizer's work per rank. bf16 GEMM copies
        # with bf16 gradient buckets and the overlapped update only (fp8 keeps replicated updates:
        # its e4m3 copies and weight amax are written by the update itself). PZ_ZERO=1 forces it
        # (e.g. a forced 1-rank RCCL group, or the one-GPU collective proxy's modelled world).
        # PZ_ZERO_SCOPE: "mid" (default) shards the weights whose gradient is complete while the
        # backward still runs (not the first layer, not its paired partner): their reduce-scatter ->
        # slice update -> all-gather chain overlaps the rest of the backward, while the two updates
        # that cross the step boundary stay one all-reduce hop each. "side" also shards the paired
        # partner, "all" every dense weight. Modelled 8-rank step (tools/comm_pressure.py, 16-WG
        # collective proxy, 3 interleaved rounds): mid +22.5%, replicated +26.4%, side +28.1%
        # (profiles/r6_comm_pressure.txt).
        zmode = os.environ.get("PZ_ZERO", "auto")
        self.zero: ZeroShards | None = None
        if ((zmode == "1" or (zmode == "auto" and self.ctx.world_size > 1)) and self.ctx.enabled
                and model.precision.name == "bfloat16" and self.master == torch.float32
                and os.environ.get("PZ_OPT_OVERLAP", "1") != "0"
                and os.environ.get("PZ_GRAD_COMM_DTYPE", "bf16").lower() in ("bf16", "bfloat16")):
            dense = [st.seg_w for st in self.stages if st.kind == "gemm"]
            scope = os.environ.get("PZ_ZERO_SCOPE", "mid")
            sharded = dense if scope == "all" else dense[1:]
            partner = self._pair_partner()
            if scope == "mid" and partner is not None:  # its update also crosses the boundary
                sharded = [sg for sg in sharded if sg is not partner.seg_w]
            if sharded:
                self.zero = ZeroShards(self.ctx, sharded, len(self.shadow_sets), self.dev)
        self._zero_ar = False  # record step: all-reduced dense gradients (the record needs them whole)
        for st in self.stages:
            if st.kind == "gemm" and self.compute != self.master:
                for par, sset in enumerate(self.shadow_sets):
                    sset[st.seg_w.offset] = (self.zero.shadow_view(st.seg_w.offset, par) if self._sharded(st.seg_w)
                                             else torch.empty(st.seg_w.shape, device=self.dev, dtype=self.compute))
        # Data parallel: dense weight gradients are written by the dW GEMMs straight in bf16 and
        # all-reduced in bf16 (half the xGMI bytes of fp32 — rings over xGMI are per-link bound,
        # SURVEY §5.8); the fused optimizer reads them back as fp32. Biases, BN, embeddings and
        # the loss stay in the exact fp32 bucket. PZ_GRAD_COMM_DTYPE=fp32 keeps fp32 gradients.
        # Why bf16 is the default (tests/test_dp_gpu.py, measured on MI355X against one rank on the
        # concatenated batch, 2 steps): the bf16 rounding of each rank's gradient plus the ring's
        # bf16 partial sums cost 5e-5 (2 ranks) / 1e-4 (8 ranks) relative cost error and SGD weight
        # deltas of 1.3e-5 / 1.8e-5 — a few bf16 ulps of the update, far below minibatch noise —
        # while the fp32 L2 bucket of the headline model (67 MB) would no longer hide behind the
        # remaining backward (dX L2 + dW L1, ~0.3 ms) at a ~300 GB/s ring over xGMI.
        # One process: the dense weight gradients are stored in bf16 as well (PZ_GRAD_DTYPE, default
        # bf16; fp32 keeps them exact): half the dW store and optimizer read traffic, the same
        # rounding the DP buckets already apply. Same-box A/B x3: mlp4 1.204-1.210 vs 1.212-1.221 ms,
        # fp8 mlp8192 0.801-0.809 vs 0.810-0.814 (profiles/r2_ab_opt_sched.txt).
        self.grads16: dict[int, torch.Tensor] = {}
        policy = os.environ.get("PZ_GRAD_COMM_DTYPE", "bf16").lower()
        local16 = os.environ.get("PZ_GRAD_DTYPE", "bf16").lower() in ("bf16", "bfloat16")
        if self.compute == torch.bfloat16 and (local16 if not self.ctx.enabled else policy in ("bf16", "bfloat16")):
            buf16 = None
            for st in self.stages:
                if st.kind == "gemm":
                    if self._sharded(st.seg_w):
                        self.grads16[st.seg_w.offset] = self.zero.grad_view(st.seg_w.offset)
                        continue
                    if buf16 is None:
                        buf16 = torch.zeros(max(1, self.store.accum_offset), device=self.dev, dtype=torch.bfloat16)
                    self.grads16[st.seg_w.offset] = self.store.view(st.seg_w, buf16)
        self.opt = FusedOptimizer(self.store, model.params, model.optimizer, self.shadow_sets, self.grads16)
        self.ctx.broadcast_(self.store.flat)  # identical replicas (rank 0 wins)
        for sset in self.shadow_sets:
            for sh_off, sh in sset.items():
                seg = next(s for s in self.store.segments if s.offset == sh_off)
                sh.copy_(self.store.view(seg))
        self.opt.init_stats()
        # fp8 policy: ONE e4m3 copy per GEMM weight in its natural [in, out] layout — the forward
        # reads it N-contiguous (transposing 8-bit LDS reads), the backward dX GEMM K-contiguous —
        # + per-tensor {q, s} records. Widths that are not multiples of 256 (the natural-layout
        # forward GEMM stages B as whole 256-byte rows) keep an [out, in] transposed forward copy.
        self.fp8 = model.precision.name == "fp8"
        self._w8_nat = all(st.seg_w.shape[1] % 256 == 0 for st in self.stages if st.kind == "gemm")
        self.w8_kc = not self._w8_nat  # the forward operand's layout (K-contiguous = transposed copy)
        self.w8: dict[int, torch.Tensor] = {}
        self._w8_fused = False
        if self.fp8:
            gemms = [st for st in self.stages if st.kind == "gemm"]
            self.wqs = torch.ones(len(gemms), 2, device=self.dev)
            self.wamax = torch.zeros(len(gemms), device=self.dev)
            # activations (delayed), double-buffered by step parity: step t's forward quantises
            # with, and its backward dequantises the same e4m3 copies with, _aqs_store[parity]; the
            # head folds this step's amax into the other parity's records for step t+1
            self._aqs_store = torch.ones(2, len(self.stages), 2, device=self.dev)
            self.aqs = self._aqs_store[0]
            self.aamax = torch.zeros(len(self.stages), device=self.dev)
            # backward dX GEMMs: e5m2 gradients (delayed scaling, q = 57344 / (2 amax of the previous
            # step; the first step calibrates on its own amax) x e4m3 weights [in, out] (current
            # scaling, the forward copy's scale)
            self.gqs = torch.ones(len(self.stages), 2, device=self.dev)
            self.gamax = torch.zeros(len(self.stages), device=self.dev)
            self._g8_calibrated = False
            self.w8n: dict[int, torch.Tensor] = {}
            self.xqs = torch.ones(2, device=self.dev)                       # first-layer input
            self.xamax = torch.zeros(1, device=self.dev)
            # weight amax accumulators per shadow parity: the optimizer update max-es |w_new| into
            # its parity's slot, the transpose-quantise right behind it consumes that slot and
            # clears the other parity's (no separate amax pass over the fp32 weights)
            # (every accumulator on a 256-B line of its own: the update's ~2k same-address atomic
            # max-es go to the memory side, and a plain read of a value sharing their line — the
            # previous amax the fused e4m3 copy scales by — queued behind them: the Adam update
            # ran 2x slower with the two parities packed into one line)
            self._wamax_store = torch.zeros(2, len(gemms), 64, device=self.dev)
            self.wamax2 = self._wamax_store[:, :, 0]
            for k, st in enumerate(gemms):
                st.w8_index = k
                if self._w8_nat:  # one copy: the forward's B and (layers 2..n) the dX GEMM's B
                    self.w8[st.seg_w.offset] = self.w8n[st.seg_w.offset] = torch.empty(
                        st.seg_w.shape, device=self.dev, dtype=torch.float8_e4m3fn)
                    continue
                self.w8[st.seg_w.offset] = torch.empty(st.seg_w.shape[1], st.seg_w.shape[0], device=self.dev,
                                                       dtype=torch.float8_e4m3fn)
                if k > 0:  # dX operand of layers 2..n
                    self.w8n[st.seg_w.offset] = torch.empty(st.seg_w.shape, device=self.dev,
                                                            dtype=torch.float8_e4m3fn)
            self._refresh_fp8_weights()
            self.opt.set_amax([{st.seg_w.offset: self.wamax2[p % 2, st.w8_index:st.w8_index + 1] for st in gemms}
                               for p in range(len(self.shadow_sets))])
            # natural layout: the optimizer writes the e4m3 copy itself with DELAYED weight scaling
            # (q from the amax the previous update reduced; the first update falls back to the
            # initial copies' current scale) — no quantisation pass re-reading the fp32 weights
            # behind every update.
            if self._w8_nat:
                self._w8_fused = True
                self.opt.set_w8([{st.seg_w.offset: (self.w8[st.seg_w.offset],
                                                    self.wamax2[1 - p % 2, st.w8_index:st.w8_index + 1],
                                                    self.wqs[st.w8_index]) for st in gemms}
                                 for p in range(len(self.shadow_sets))])
        # Optimizer overlap: each GEMM weight is updated on a side stream as soon as its gradient
        # bucket is complete (its dW GEMM on one GPU, its all-reduce under DP), while the rest of
        # the backward runs; the bandwidth-bound update hides behind the MFMA-bound GEMMs.
        # PZ_OPT_OVERLAP=0: every update on the compute stream, after the backward.
        self.overlap = os.environ.get("PZ_OPT_OVERLAP", "1") != "0"
        # (measured, not kept: the side stream at priority -1 under data parallelism, so the sharded
        # slice updates between a reduce-scatter and its all-gather dispatch ahead of the GEMMs —
        # every compute-stream kernel stretched, modelled 8-rank step +92 vs +29%,
        # profiles/r6_comm_pressure.txt)
        self.opt_stream = torch.cuda.Stream(device=self.dev) if self.overlap else None
        # One process: the steps run on a priority -1 stream of the trainer's own, so the compute
        # stream's workgroups dispatch ahead of the side stream's updates when both have work
        # queued — the step-end first-layer update 68 -> 50 us beside the side stream's L2 update,
        # mlp4 1.0894 vs 1.0947 ms (3 of 3 interleaved rounds, profiles/r6_ab_main_prio.txt).
        # Not under data parallelism: collectives issued from the caller's stream (_SaveAgreement)
        # and the trainer's must stay on one stream per communicator. PZ_MAIN_PRIO=0: off.
        self._main_stream = (torch.cuda.Stream(device=self.dev, priority=-1)
                             if self.overlap and not self.ctx.enabled and os.environ.get("PZ_MAIN_PRIO", "1") != "0"
                             else None)
        self._main_joined = False
        # (measured, not kept: the next batch's gather on the side stream during the step, double-
        # buffered; the step-end update on a high-priority stream — each saved its 12-20 us on the
        # boundary and paid it back in cross-stream event latency, profiles/r6_ab_boundary.txt)
        self._g8_done: dict = {}  # stage index -> the dZ tensor whose e5m2 copy is current this step
        self._g8_epi_ready: set = set()  # stages whose epilogue-written e5m2 dZ scale is calibrated
        self._y_dead_cache: dict = {}  # fp8 policy: which bf16 GEMM outputs go unwritten (_y_dead)
        self._grad_su_pending = False  # fp8: a gradient scale update waits for the next step's gather
        self._act_su = None            # fp8: this step's activation scale update (folded into the head)
        self._run_epoch = None
        # one launch per GEMM weight except the first layer's, which comes last anyway and
        # shares the final launch with the small accumulated parameters (biases, BN, embedding)
        gemm_w = [st.seg_w.offset for st in self.stages if st.kind == "gemm"]
        # PZ_OPT_FUSE (one process, bf16 policy): every dense weight is updated INSIDE its own dW
        # GEMM's epilogue (pz::gemm_update, EPI_OPT) — the fp32 gradient never makes the HBM round
        # trip and no weight update is left for the side stream or the step's tail; the last launch
        # only updates the biases / batchnorm / embedding parameters. Under data parallelism the
        # gradient must be all-reduced first, so the launches stay separate. The fused update's
        # traffic runs AFTER each CU's main loop instead of beside other GEMMs, so it pays only
        # where it removes most bytes: SGD (10 vs 18 B/param; deep16x8192 40.2 vs 40.6 ms), not
        # Adam (26 vs 34 B/param; mlp4 1.39 vs 1.25 ms, mlp8192 0.96 vs 0.87, mlp4x8192 11.2 vs
        # 10.8 — profiles/r2_ab_opt_fuse.txt). auto (default) = SGD only; 1 = always; 0 = never.
        mode = os.environ.get("PZ_OPT_FUSE", "auto")
        want = mode == "1" or (mode == "auto" and model.optimizer is None)
        self.fuse_opt = (want and self.overlap and not self.ctx.enabled and self.compute == torch.bfloat16
                         and not self.fp8)
        self._fuse_ok: dict = {}
        # PAIRED weight-gradient GEMMs (one process): the dW GEMM of the GEMM stage after the first
        # with the fewest output tiles is deferred to the end of the backward and launched
        # TOGETHER with the first layer's (pz::gemm_pair): two skinny GEMMs that alone each need a
        # 4-way split-K to fill the CUs (mlp4: 64 tiles each) share one launch with a 2-way split
        # (mlp8192: none) — half the slab hand-offs, one launch and one ramp fewer. Its update
        # then joins the side stream right behind the pair. PZ_DW_PAIR=0: one launch per dW.
        # (measured, not kept: both weights' updates in that launch's epilogue, EPI_OPT — the pair
        # ran 289 vs 119 us beside the side-stream update, mlp4 1.204 vs 1.111 ms, r5 same box)
        # Data parallel too: the partner's bucket then leaves with the first layer's at the end of
        # the backward (mlp4: 8 MB of bf16, ~14 MB of ring traffic per GPU at 8 ranks, ~50 us on
        # xGMI) while the pair saves ~60 us of GEMM time against two split-4 launches
        # (profiles/r5_step_timeline_dpnone.txt: 91 + 101 us vs 130 us paired).
        partner = self._pair_partner() if not self.fuse_opt and self.overlap else None
        self._pair_idx = partner.index if partner is not None else None
        self._early_keys = set() if self.fuse_opt else set(gemm_w[1:])
        if self.zero is not None:
            # the sharded weights by slices; the rest group (the replicated first layer under the
            # default scope, and the small parameters) reports its statistics from rank 0 only
            keys = [o for o in gemm_w if o in self.zero.shards or o in gemm_w[1:]]
            self._zero_repl = [o for o in keys if o not in self.zero.shards]  # replicated side-stream weights
            self.opt.define_groups(keys, rest_stats=self.zero.rank == 0, replicated=set(self._zero_repl))
            self.zero.define_groups(self.opt)
        else:
            self.opt.define_groups(gemm_w if self.fuse_opt else gemm_w[1:])
        # the side-stream updates of all layers but the first are queued together behind the last
        # of their gradients (one event instead of one per layer; mlp4 1.311-1.320 vs 1.321-1.326 ms)
        # (measured again in r6, not kept: the bf16 policy's side update queued right behind its dW
        # GEMM instead of behind the layer's dX — dX_L2 stretched 194 -> 286 us by the update beside
        # it, the boundary shrank 96 -> 48 us: mlp4 1.141 vs 1.099 ms, profiles/r6_ab_update_early.txt)
        self._flush_key = gemm_w[1] if len(gemm_w) > 1 else None
        self._side_pending: list = []

        self._pair_dw = None       # (stage, x_in, dZ) of the dW GEMM that waits for its partner
        self._pair_late = None     # (stage, gradient) of the paired partner, bucketed in the update phase
        # data parallel: the paired dW launch issued while a gradient bucket is on the wire runs as
        # one persistent stream-K schedule on the CUs the collective kernels leave
        # (parallel/dist.py comm_cus). Only the pair: a one-round grid is where a held CU costs a
        # whole extra round; the multi-round GEMMs absorb it (dX_L2 217 vs 194 us under the proxy)
        # better than the budgeted engine's split-tile hand-offs (profiles/r5_sk_stamps.txt)
        self._cus = 0
        self._cus_comm = 0
        if self.ctx.enabled and self.ctx.comm_cus != 0:
            n_cu = torch.cuda.get_device_properties(self.dev).multi_processor_count
            if not 0 < self.ctx.comm_cus < n_cu:
                raise ValueError(f"PZ_COMM_BUDGET={self.ctx.comm_cus}: the CUs left to the collectives must be "
                                 f"in 1..{n_cu - 1} on this device ({n_cu} CUs)")
            self._cus_comm = n_cu - self.ctx.comm_cus
        self._opt_done = None
        self._early_done = None  # previous step's side-stream updates (layers 2..n) + step_finalize done
        self._ov = None
        self._rows = None
        self._gbatch = 1           # global sample size of the current step (all ranks)
        # hipGraph replay of whole steps (single GPU) when a step is launch-bound: PZ_GRAPHS=auto
        # (default: steps under GRAPH_MAX_FLOP), 1 (always), 0 (never)
        mode = os.environ.get("PZ_GRAPHS", "auto")
        self.use_graphs = mode != "0"
        self._graphs_forced = mode == "1"
        self._dense_params = sum(st.seg_w.numel for st in self.stages if st.kind == "gemm")
        self.epoch_ctr = torch.zeros(1, device=self.dev, dtype=torch.int32)
        self._ctr_epoch = 0
        self._plan = None
        self._graphs: dict = {}
        self._warm: set = set()
        self._graph_pool = None
        self._last_event = None
        self._capturing = False
        self._pending: list = []   # (epoch, ratio_row or None, timestamp event)
        # device-scope ordering events + fence-free step timestamps (engine/events.py): a default
        # torch event's system-scope fence idled the compute stream ~7 us per record / wait
        self.events = StreamEvents(self.dev)
        self._drained = 0
        self._record = None
        self.data = None
        self.data8 = None  # fp8 policy: e4m3 copy of the dataset (first-layer operand)

    # ------------------------------------------------------------------------------------
    # data
    # ------------------------------------------------------------------------------------
    def _pair_partner(self) -> Stage | None:
        """The GEMM stage whose dW launch is deferred and paired with the first layer's: the later
        stage with the fewest weight elements (PZ_DW_PAIR=0: none)."""
        if os.environ.get("PZ_DW_PAIR", "1") != "1" or self.stages[0].kind != "gemm":
            return None
        cands = [st for st in self.stages if st.kind == "gemm" and st.index > 0]
        return min(cands, key=lambda st: (st.seg_w.numel, -st.index)) if cands else None

    def load_data(self, data) -> None:
        """Training pairs (python lists) -> device tensors, once per ``train()`` call."""
        inputs = [inp for inp, _ in data]
        targets = [tgt for _, tgt in data]
        first = self.stages[0]
        host = torch.float64 if self.master == torch.float64 else torch.float32  # fp64 models: exact inputs
        if first.kind == "embed":
            x = torch.tensor(inputs, dtype=torch.float32)
            if x.dim() == 1:
                x = x.unsqueeze(1)
            self.block = x.shape[1]
        else:
            x = torch.tensor(inputs, dtype=host).reshape(len(inputs), -1)
            self.block = 1
        lab = torch.tensor([int(t[0]) for t in targets], dtype=torch.int64) if self.head == "softmax" else None
        self._validate(x, lab)
        self.data = self._table(x)
        if self.head == "softmax":
            self.labels = lab.to(self.dev)
            self.targets = None
        else:
            self.targets = torch.tensor(targets, dtype=host).reshape(len(targets), -1).to(self.dev)
            self.labels = None
        seed = torch.randint(0, 2 ** 62, (1,)).item()
        self.base_seed = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
        self._rows = None
        self._invalidate_graphs()

    def _validate(self, x: torch.Tensor, labels: torch.Tensor | None) -> None:
        """Reject class labels / token ids the kernels cannot index, once per dataset (IndexError,
        as the reference's cross_entropy / `weights[ids]` raise), instead of per step."""
        if labels is not None:
            PF.check_index_range(labels, 0, self.stages[-1].out_width, "Target")
        if self.stages[0].kind == "embed":
            vocab = self.stages[0].seg_w.shape[0]
            PF.check_index_range(x.reshape(-1), -vocab, vocab, "index", vocab)

    def _table(self, x: torch.Tensor) -> torch.Tensor:
        """Device-resident dataset. Dense inputs are kept in the GEMM operand dtype (the gather
        would round them to it anyway): half the bytes per sampled row for bf16 models."""
        if self.stages[0].kind != "embed" and self.compute == torch.bfloat16:
            return x.to(device=self.dev, dtype=torch.bfloat16).contiguous()
        return x.to(self.dev).contiguous()

    def load_tensors(self, inputs: torch.Tensor, targets: torch.Tensor, seed: int | None = None) -> None:
        """Fast path for benchmarks / programmatic use: a dataset already held as tensors.

        ``inputs``: ``[N, in]`` (or ``[N, T]`` token ids); ``targets``: ``[N]`` class labels for a
        softmax head, ``[N, out]`` regression targets otherwise.
        """
        self._validate(inputs, targets.reshape(-1) if self.head == "softmax" else None)
        host = torch.float64 if self.master == torch.float64 and self.stages[0].kind != "embed" else torch.float32
        self.data = self._table(inputs.to(dtype=host))
        self.block = self.data.shape[1] if self.stages[0].kind == "embed" else 1
        if self.head == "softmax":
            self.labels = targets.reshape(-1).to(device=self.dev, dtype=torch.int64).contiguous()
            self.targets = None
        else:
            self.targets = targets.to(device=self.dev, dtype=self.master).reshape(len(targets), -1).contiguous()
            self.labels = None
        seed = torch.randint(0, 2 ** 62, (1,)).item() if seed is None else seed
        self.base_seed = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
        self._rows = None
        self._invalidate_graphs()

    def _ensure_buffers(self, batch: int) -> None:
        rows_b = _round_up(batch, ROW_PAD)
        if self._rows == (batch, rows_b):
            return
        self._rows = (batch, rows_b)
        self._invalidate_graphs()  # captured steps point at the old buffers
        dev, cd = self.dev, self.compute
        pos = self.block
        # sampled inputs / labels / picks
        self.x_in = torch.empty(rows_b, self.data.shape[1], device=dev,
                                dtype=torch.float32 if self.stages[0].kind == "embed" else cd)
        self.lab = torch.empty(rows_b, device=dev, dtype=torch.int64) if self.head == "softmax" else None
        self.picked = torch.empty(rows_b, device=dev, dtype=torch.int64)
        self.tgt = torch.empty(rows_b, self.targets.shape[1], device=dev, dtype=cd) if self.targets is not None \
            else None
        for st in self.stages:
            if st.kind == "embed":
                st.pos_in = st.pos_out = pos
                rows = rows_b * pos
                st.buffers["y"] = torch.empty(rows, st.out_width, device=dev, dtype=cd)
                st.buffers["g"] = torch.empty(rows, st.out_width, device=dev, dtype=cd)
                continue
            st.pos_in = pos
            if st.kind == "flatten":
                r = st.layer.ratio
                pos = pos // r
                st.pos_out = pos
            else:
                st.pos_out = pos
            rows = rows_b * st.pos_out
            st.buffers["y"] = torch.empty(rows, st.out_width, device=dev, dtype=cd)
            st.buffers["g"] = torch.empty(rows, st.out_width, device=dev, dtype=cd)
            if st.kind == "bn":
                c = st.out_width
                st.buffers["mean"] = torch.empty(c, device=dev, dtype=torch.float64)
                st.buffers["invstd"] = torch.empty(c, device=dev, dtype=torch.float64)
                st.buffers["partial"] = torch.empty(2 * c, device=dev, dtype=torch.float64)
                st.buffers["bn_in_grad"] = torch.empty(rows_b * st.pos_in, st.in_width, device=dev, dtype=cd)
        if pos != 1:
            raise UnsupportedModel(f"head input still has {pos} positions per sample")
        self._plan_relu_masks(rows_b)
        self._plan_fp8(rows_b)
        # record-mode scratch: one buffer per layer output / grad, allocated lazily

    def _gather(self, epoch, idx, batch, capture, su) -> None:
        ops = torch.ops.pz
        gseed = self._gather_seed(epoch)
        ops.gather_rows(self.data, idx, gseed[0], gseed[1], self.x_in, batch, self.labels, self.lab, self.picked,
                        self.epoch_ctr if capture else None, self.data8,
                        self.x8 if self.data8 is not None else None, *su)
        if self.tgt is not None:
            ops.gather_rows(self.targets, self.picked, 0, 0, self.tgt, batch, None, None, None)

    # ------------------------------------------------------------------------------------
    # epilogue specs
    def _opt_async(self, items: list, ready=None) -> None:
        """Queue the updates of optimizer groups ``[(key, handles, stages)]`` on the side stream
        behind their gradients: ONE event recorded on the compute stream for all of them (each
        record / cross-stream wait costs the compute stream a few microseconds of idle), or an
        already recorded ``ready`` event."""
        main, l2, scale = self._ov
        if ready is None:
            ready = self.events.sync(self._capturing)
            ready.record(main)
        with torch.cuda.stream(self.opt_stream):
            ready.wait(self.opt_stream)
            gathers = []
            for key, handles, stages in items:
                for h in handles:
                    self.ctx.wait_one(h)
                if self.zero is not None and key in self.zero.shards:  # slice, then all-gather of the bf16 copy
                    gathers.append(self.zero.update(self.opt, key, self.grads, l2, scale, 1 - self.parity))
                else:
                    self.opt.step_group(key, self.grads, l2, scale, 1 - self.parity)
                if self.fp8:
                    for st in stages:
                        self._refresh_fp8_weights(st, 1 - self.parity)
            for h in gathers:  # (the side stream's completion event then covers the gathered copies)
                self.ctx.wait_one(h)

    def _plan_relu_masks(self, rows_b: int) -> None:
        """ReLU GEMM stages feeding a GEMM stage keep a 1-bit mask of ``y > 0`` next to ``y``: the
        next stage's dX GEMM reads it (8 B per 64 columns) instead of re-reading ``y`` (128 B)."""
        for i, st in enumerate(self.stages):
            st.buffers.pop("mask", None)
            if st.kind != "gemm" or st.act != PF.ACT_RELU or i + 1 >= len(self.stages):
                continue
            nxt = self.stages[i + 1]
            x = self.stages[i - 1].buffers["y"] if i > 0 else self.x_in
            if nxt.kind != "gemm" or x.dtype != torch.bfloat16:
                continue
            if PF.gemm_path(x, True, self._w(st), False, st.buffers["y"]) != "mfma":
                continue
            if PF.gemm_path(nxt.buffers["g"], True, self._w(nxt), True, st.buffers["g"]) != "mfma":
                continue
            st.buffers["mask"] = PF.relu_mask_empty(rows_b * st.pos_out, st.out_width, device=self.dev)

    # ------------------------------------------------------------------------------------
    def _keys(self, epoch: int | None) -> tuple:
        """Dropout key context of one step: ``(seed_lo, seed_hi, epoch, epoch_ptr)``. Eager steps
        mix the epoch into the keys on the host; graph-captured steps (``epoch=None``) pass the
        device epoch counter and the kernels mix it in with the same function."""
        lo = self.base_seed[0] & _M32
        hi = (self.base_seed[1] + self.ctx.rank * 0xC2B2AE35) & _M32
        return (lo, hi, epoch, 0) if epoch is not None else (lo, hi, None, self.epoch_ctr.data_ptr())

    def _gather_seed(self, epoch: int | None) -> tuple[int, int]:
        """Minibatch sampler seeds (host mirror of the kernels' ``gather_seed``)."""
        lo = self.base_seed[0] & _M32
        hi = (self.base_seed[1] ^ (self.ctx.rank * 0x27D4EB2F)) & _M32
        if epoch is not None:
            lo = (lo + epoch * 0x632BE5AB) & _M32
            hi ^= epoch & _M32
        return lo, hi

    def _epi(self, st: Stage, p: float, keys, parts=("pre", "act", "post")):
        return PF.epi_spec(act=st.act if "act" in parts else PF.ACT_NONE,
                           drop_pre=st.drop_pre if "pre" in parts else -1,
                           drop_post=st.drop_post if "post" in parts else -1, p=p, seed=keys[:2], epoch=keys[2],
                           epoch_ptr=keys[3])

    def _w_grad(self, seg) -> torch.Tensor:
        """Gradient buffer of a weight segment: the bf16 DP view or the fp32 flat gradient."""
        g16 = self.grads16.get(seg.offset)
        return g16 if g16 is not None else self.store.view(seg, self.grads)

    def _w(self, st: Stage) -> torch.Tensor:
        """GEMM operand for the stage's weight: bf16 shadow or the fp32 master view, [in, out]."""
        sh = self.shadow_sets[self.parity].get(st.seg_w.offset)
        return sh if sh is not None else self.store.view(st.seg_w)

    # ------------------------------------------------------------------------------------
    # one epoch
    # ------------------------------------------------------------------------------------
    def begin(self, epochs: int, lr_schedule=None) -> None:
        """Size the device-side progress arrays for a ``train()`` call of ``epochs`` epochs.

        ``lr_schedule(epoch) -> lr`` (the learning rate :meth:`step` will be called with) enables
        hipGraph replay: the per-epoch optimizer hyper-parameters are tabulated on the device
        once, so a captured step needs nothing from the host but a replay."""
        self._alloc_progress(epochs)
        self._invalidate_graphs()
        self._plan = None
        if lr_schedule is None or not self._graphs_possible():
            return
        every = max(1, epochs // 100)
        t0 = self.opt.step_count
        lrs = [float(lr_schedule(e)) for e in range(epochs)]
        rows = []
        for e, lr in enumerate(lrs):
            if self.opt.adam:
                b1, b2 = self.opt.torch_opt.param_groups[0]["betas"]
                t = t0 + e + 1
                rows.append((lr, 1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t), 0.0))
            else:
                rows.append((lr, 1.0, 1.0, 0.0))
        self._plan = {"epochs": epochs, "every": every, "t0": t0, "lrs": lrs,
                      "hp": torch.tensor(rows or [(0.0, 1.0, 1.0, 0.0)], dtype=torch.float64, device=self.dev)}

    def _graphs_possible(self) -> bool:
        # single GPU only (collectives are not captured); no per-phase host syncs (PZ_DEBUG_SYNC)
        return self.use_graphs and self.overlap and not self.ctx.enabled and not _DEBUG_SYNC

    def _launch_bound(self, batch: int) -> bool:
        """Replay pays where the host's ~0.17 ms of per-step launches exceeds the GPU time."""
        return self._graphs_forced or 6.0 * self._dense_params * batch < GRAPH_MAX_FLOP

    def _invalidate_graphs(self) -> None:
        self._graphs = {}
        self._warm = set()

    def step(self, epoch: int, lr: float, sample_size: int, dropout: float, l2: float, want_ratios: bool,
              record: bool, indices: torch.Tensor | None = None) -> None:
        """One training epoch. ``indices`` (int64, this rank's ``batch`` rows) overrides the
        on-device sampler — used by the data-parallel equivalence tests.

        After :meth:`begin` with an ``lr_schedule``, plain (non-record) steps are captured once per
        weight-shadow parity into a hipGraph and replayed: the epoch-dependent values (dropout
        keys, sampler seeds, optimizer hyper-parameters, cost slot, ratio row) are then read from
        the device epoch counter, which every step advances in ``step_finalize``."""
        world, rank = self.ctx.world_size, self.ctx.rank
        if sample_size < world:
            raise ValueError(f"sample size {sample_size} is smaller than the {world} data-parallel ranks")
        # the global sample is split exactly (reference :441, 460 draw sample_size rows): rank r
        # draws rows [r*S//W, (r+1)*S//W): the S % W extra rows are spread by the floor division
        # (S=10, W=4: 2, 3, 2, 3 rows). Every rank scales its
        # loss and gradients by 1/S (the GLOBAL sample), so the all-reduced sum is the global mean
        # with no 1/world factor — unequal shards weigh exactly by their share
        batch = (rank + 1) * sample_size // world - rank * sample_size // world
        self._gbatch = sample_size
        self._ensure_buffers(batch)
        if not hasattr(self, "costs") or epoch >= self.costs.numel():
            self._alloc_progress(epoch + 1)
            self._invalidate_graphs()
            self._plan = None
        plan = self._plan
        row = None
        if want_ratios:
            if plan is not None:
                row = epoch // plan["every"]
            else:
                row = self._ratio_rows
                self._ratio_rows += 1
        graphable = (plan is not None and not record and indices is None and self._launch_bound(batch)
                     and epoch < plan["epochs"]
                     and want_ratios == (epoch % plan["every"] == 0) and lr == plan["lrs"][epoch]
                     and (not self.opt.adam or self.opt.step_count == plan["t0"] + epoch))
        gkey = (self.parity, batch, sample_size, float(dropout), float(l2))
        if self._main_stream is not None:
            if not self._main_joined:  # the caller's queued work (inputs, parameters) first
                self._main_stream.wait_stream(torch.cuda.current_stream(self.dev))
                self._main_joined = True
            with torch.cuda.stream(self._main_stream):
                self._step_on(gkey, graphable, epoch, lr, batch, dropout, l2, row, record, indices)
        else:
            self._step_on(gkey, graphable, epoch, lr, batch, dropout, l2, row, record, indices)
        self._ctr_epoch = epoch + 1

    def _step_on(self, gkey, graphable, epoch, lr, batch, dropout, l2, row, record, indices) -> None:
        if graphable and gkey in self._warm:
            self._replay(gkey, epoch, lr, batch, dropout, l2, row)
        else:
            self._run(epoch, lr, batch, dropout, l2, -1 if row is None else row, record, indices)
            self._pending.append((epoch, row, self._last_event))
            if graphable:
                self._warm.add(gkey)

    def _replay(self, gkey, epoch: int, lr: float, batch: int, dropout: float, l2: float, row) -> None:
        main = torch.cuda.current_stream(self.dev)
        if self._opt_done is not None:
            self._opt_done.wait(main)
            self._opt_done = None
        self._early_done = None
        if self._ctr_epoch != epoch:
            self.epoch_ctr.fill_(epoch)
        parity = self.parity
        graph = self._graphs.get(gkey)
        if graph is not None:
            self.opt.cur = 1 - self.opt.cur  # what the captured finalize did when it was recorded
        else:
            graph = torch.cuda.CUDAGraph()
            self.opt.graph_tables = (self._plan["hp"], self.epoch_ctr)
            try:
                with torch.cuda.graph(graph, pool=self._graph_pool, capture_error_mode="thread_local"):
                    self._run(None, lr, batch, dropout, l2, -2, False, None)
            finally:
                self.opt.graph_tables = None
            self._graph_pool = graph.pool()
            self._graphs[gkey] = graph
            self.parity = parity  # capture does not execute: the replay below runs this epoch
        self.opt.begin_step(lr)  # host bookkeeping only (step counter, param_group lr)
        graph.replay()
        self.parity = 1 - parity
        self._pending.append((epoch, row, self.events.stamp(main)))

    def _run(self, epoch: int | None, lr: float, batch: int, dropout: float, l2: float, row: int, record: bool,
             indices: torch.Tensor | None) -> None:
        """Enqueue one step. ``epoch=None``: hipGraph capture (epoch-dependent values from the
        device counter / tables; the side stream joins the capture stream at the end)."""
        capture = epoch is None
        self._capturing = capture  # (torch events inside a capture: engine/events.py)
        self._run_epoch = epoch  # None while a hipGraph is captured
        keys = self._keys(epoch)
        ops = torch.ops.pz
        main = torch.cuda.current_stream(self.dev)
        self._zero_ar = record and self.zero is not None
        if self._zero_ar:  # the record's weight gradients read whole fp32 masters (2 l2 W)
            if self._opt_done is not None:  # (the previous step's side-stream slice updates)
                self._opt_done.wait(main)
            self.zero.gather_state(self.store.flat)
        overlap = self.overlap and not record
        # update-ratio sums only on progress epochs (row >= 0; captured steps: decided on device)
        self.opt.stats_every = (self._plan["every"] if self._plan else 1) if row == -2 else (1 if row >= 0 else 0)
        if overlap:
            if not capture:
                self.opt.begin_step(lr)
            self._ov = (main, l2, 1.0)  # gradients arrive as the global mean (1/S-scaled heads)
            self._late_stages, self._late_handles = [], []
            self._side_pending = []
            self._pair_late = None

        # (no zeroing pass: the previous step's update kernel reset the accumulated-gradient region
        # as it read it, and its step_finalize the loss slots)

        # ---------------- sample + input
        self._phase("pz.sample")
        idx = None
        if indices is not None:
            idx = indices.to(device=self.dev, dtype=torch.int64).contiguous()
            if idx.numel() < batch:
                raise ValueError(f"need {batch} indices, got {idx.numel()}")
        if self.fp8:
            self.aqs = self._aqs_store[self.parity]
        # the previous step's gradient amax -> this step's e5m2 scales rides on the gather
        # (delayed scaling: nothing reads them before this step's backward)
        su = (self.gamax, self.gqs, 2.0, 57344.0) if self._grad_su_pending else (None, None, 1.0, 448.0)
        self._gather(epoch, idx, batch, capture, su)
        self._grad_su_pending = False

        rec = {} if record else None
        # the previous step's first-layer / bias update ran on this stream; its side-stream updates
        # (layers 2..n) and step_finalize (loss-slot / statistics reset) are awaited together
        # before the first stage that reads a side-updated weight (else before the head)
        self._phase("pz.forward")
        x = self.x_in
        prev = None
        for st in self.stages:
            if self._early_done is not None and st.kind == "gemm" and st.seg_w.offset in self._early_keys:
                self._early_done.wait(main)
                self._early_done = self._opt_done = None
            x = self._forward_stage(st, x, batch, dropout, keys, rec)
            prev = st
        last = prev
        # this step's activation amax -> next step's scales: folded into the softmax head's launch
        # (nothing reads them there), else its own launch
        # (into the other parity's records: this step's backward still dequantises the e4m3
        # copies its forward wrote, the weight-gradient GEMMs' X8, with this step's)
        self._act_su = (self.aamax, self._aqs_store[1 - self.parity], 1.25, 448.0) if (self.fp8 and not record) else None
        if self.fp8 and record:  # (no update folded: the next step keeps this step's records)
            self._aqs_store[1 - self.parity].copy_(self.aqs)

        # ---------------- head
        if self._opt_done is not None:
            self._opt_done.wait(main)
            self._opt_done = None
        self._early_done = None
        self._g8_done = {}  # this step's e5m2 dZ copies are produced anew (the head's included)
        self._phase("pz.head")
        g_pre = self._head(last, x, batch, dropout, keys, rec)
        if self._act_su is not None:  # (the head did not take it)
            self._act_su[1].copy_(self.aqs)
            ops.scale_update(self._act_su[0], self._act_su[1], self._act_su[2], True)
            self._act_su = None

        # ---------------- backward
        self._phase("pz.backward")
        self._cus = 0  # (full grid until the first bucket is on the wire)
        handles = []
        g = last.buffers["g"]
        for si in range(len(self.stages) - 1, -1, -1):
            st = self.stages[si]
            before = self.stages[si - 1] if si > 0 else None
            x_in = before.buffers["y"] if before is not None else self.x_in
            g, g_pre = self._backward_stage(st, before, x_in, g, g_pre, batch, dropout, keys, rec, handles)
        if self.fp8 and any(getattr(st, "fp8_bwd", False) or getattr(st, "g8_from_epi", False)
                            for st in self.stages):
            # this step's gradient amax -> next step's e5m2 scales (delayed scaling): applied by the
            # next step's first launch (the sample gather)
            self._grad_su_pending = True
            self._g8_calibrated = True

        # ---------------- reduce + update
        self._phase("pz.update")
        acc_h = self.ctx.all_reduce_async(self.grads[self.store.accum_offset:], exact=True)
        handles.append(acc_h)
        if self._pair_late is not None:
            sp, wp = self._pair_late
            self._pair_late = None
            hp = self._bucket_seg(sp.seg_w)
            handles.append(hp)
            self._side_pending.append((sp.seg_w.offset, [hp], [sp]))
        fin = dict(epoch_ctr=self.epoch_ctr, every=self._plan["every"] if self._plan else 1,
                   # fused e4m3 weight copies: this step's updates read the amax slot of the
                   # current parity; step_finalize clears it for the next step's updates
                   clear=self._wamax_store[self.parity] if self._w8_fused else None)
        if overlap:
            # the last update (first-layer weights, biases, batchnorm, embeddings) runs on THIS
            # stream right behind the last dW: the next step's first GEMM follows it in order (no
            # cross-stream wait), and it overlaps the side stream's still-running updates instead
            # of queueing behind them; step_finalize (side) waits for both
            pending, self._side_pending = self._side_pending, []
            gathers = []
            if self.zero is not None and any(self._sharded(st.seg_w) for st in self._late_stages):
                # the first layer's slice on this stream, its all-gather overlapping the small
                # replicated update behind it; the next forward (this stream) then reads it
                for h in self._late_handles:
                    self.ctx.wait_one(h)
                gathers = [self.zero.update(self.opt, st.seg_w.offset, self.grads, l2, 1.0, 1 - self.parity, side=False)
                           for st in self._late_stages]
                self.ctx.wait_one(acc_h)
            else:
                for h in list(self._late_handles) + [acc_h]:
                    self.ctx.wait_one(h)
            self.opt.step_group("rest", self.grads, l2, 1.0, 1 - self.parity)
            for h in gathers:
                self.ctx.wait_one(h)
            if self.fp8:
                for st in self._late_stages:
                    self._refresh_fp8_weights(st, 1 - self.parity)
            rest_ev = self.events.sync(capture)
            rest_ev.record(main)
            # side updates not flushed by their last layer (the paired partner's) join the side
            # stream behind the SAME event: one record on this stream fewer (~7 us of idle; the
            # side stream is still busy with the earlier layers' updates when it comes)
            # (measured, not kept: the partner's update on this stream behind the first layer's
            # instead of beside the next fwd_L1 — mlp4 1.097-1.102 vs 1.092-1.094 ms, fp8 mlp8192
            # 0.561-0.567 vs 0.536-0.539, profiles/r6_ab_partner_main.txt)
            if pending:
                self._opt_async(pending, ready=rest_ev)
            self._ov = None
            with torch.cuda.stream(self.opt_stream):
                if not pending:
                    rest_ev.wait(self.opt_stream)
                if self.zero is not None:  # every slice's statistics partials, summed (exact)
                    self.zero.all_reduce_stats(self.opt.stats[self.opt.cur])
                self.opt.finalize(self.loss_slot, 1, l2, self.costs, -1 if capture else epoch, self.ratios, row,
                                  **fin)
                ev = self.events.sync(capture)
                ev.record(self.opt_stream)
            if capture:  # join the side stream into the capture stream
                ev.wait(main)
            else:
                # ONE cross-stream wait in the next step, before the first GEMM that reads a
                # side-stream-updated weight: step_finalize (behind this stream's first-layer
                # update) finishes long before the next step's first GEMM does, and its loss-slot
                # and statistics resets are then ordered before the head and the updates
                self._opt_done = self._early_done = ev
                self._last_event = self.events.stamp(self.opt_stream)
            self.parity = 1 - self.parity
            self._phase(None)
            return
        self.ctx.wait_all(handles)
        if record:
            self._finish_record(rec, batch, l2)
        if self.zero is not None:  # (record step: this rank's slices of the all-reduced gradients)
            self.opt.begin_step(lr)
            gathers = [self.zero.update(self.opt, off, self.grads, l2, 1.0, 1 - self.parity, source="ar")
                       for off in self.zero.shards]
            for off in self._zero_repl + ["rest"]:
                self.opt.step_group(off, self.grads, l2, 1.0, 1 - self.parity)
            for h in gathers:
                self.ctx.wait_one(h)
            self.zero.all_reduce_stats(self.opt.stats[self.opt.cur])
        else:
            self.opt.step(self.grads, lr, l2, 1.0, 1 - self.parity)
        self.parity = 1 - self.parity
        if self.fp8:
            self._refresh_fp8_weights(parity=self.parity)
        self.opt.finalize(self.loss_slot, 1, l2, self.costs, epoch, self.ratios, row, **fin)
        self._last_event = self.events.stamp(torch.cuda.current_stream(self.dev))
        self._phase(None)

    _in_phase = False

    def _phase(self, name: str | None) -> None:
        """End the current step phase and start `name` (None: end only)."""
        if _TRACE:
            if self._in_phase:
                torch.cuda.nvtx.range_pop()
            if name is not None:
                torch.cuda.nvtx.range_push(name)
            self._in_phase = name is not None
        if _DEBUG_SYNC:
            torch.cuda.synchronize(self.dev)

    # ------------------------------------------------------------------------------------
    def _forward_stage(self, st: Stage, x, batch, p, keys, rec):
        ops = torch.ops.pz
        y = st.buffers["y"]
        rows_valid = batch * st.pos_out
        if st.kind == "embed":
            ids = x  # [rows_b, T] float32 ids
            ops.embedding_fwd(self.store.view(st.seg_w), ids, y)
            if rec is not None:
                rec[st.first] = y[:rows_valid]
            return y
        if st.kind == "flatten":
            src = x.view(y.shape)
            if st.drop_pre >= 0:
                ei, ef = self._epi(st, p, keys)
                ops.stage_fwd(src, y, ei, ef)
            else:
                y.copy_(src)
            if rec is not None:
                rec[st.first] = y[:rows_valid]
            return y
        if rec is None:
            ei, ef = self._epi(st, p, keys)
            if st.kind == "gemm":
                bias = self.store.view(st.seg_b) if st.seg_b is not None else None
                kw = {}
                if st.fp8:  # e4m3 x e4m3 with the per-tensor dequantisation factors
                    i = st.index
                    xa, sa = (self.x8, self.xqs[1:2]) if i == 0 else \
                        (self.stages[i - 1].buffers["y8"], self.aqs[i - 1, 1:2])
                    wa, wkc = self.w8[st.seg_w.offset], self.w8_kc
                    kw.update(scale_a=sa, scale_b=self.wqs[st.w8_index, 1:2])
                else:
                    xa, wa, wkc = x, self._w(st), False
                if "y8" in st.buffers:  # the next stage consumes an e4m3 copy (delayed scaling)
                    kw.update(out8=st.buffers["y8"], out8_qscale=self.aqs[st.index, 0:1],
                              amax=self.aamax[st.index:st.index + 1])
                    if self._y_dead(st):
                        kw["store_c"] = False
                PF.gemm(xa, True, wa, wkc, y, bias=bias, mode=PF.EPI_FWD, epi=(ei, ef),
                        mask=st.buffers.get("mask"), **kw)
            else:
                self._bn_fwd(st, x, y, batch, ei, ef)
            return y
        # record mode: producing op without epilogue, then one kernel per following layer
        z = self._scratch(("z", st.first), y)
        none = PF.epi_spec()
        if st.kind == "gemm":
            bias = self.store.view(st.seg_b) if st.seg_b is not None else None
            PF.gemm(x, True, self._w(st), False, z, bias=bias, mode=PF.EPI_STORE)
        else:
            self._bn_fwd(st, x, z, batch, *none)
        out_first = self._scratch(("o", st.first), y)
        ops.stage_fwd(z, out_first, *self._epi(st, p, keys, parts=("pre",)))
        rec[st.first] = out_first[:rows_valid]
        if st.act_layer >= 0:
            ops.stage_fwd(out_first, y, *self._epi(st, p, keys, parts=("act", "post")))
            rec[st.act_layer] = y[:rows_valid]
        else:
            y.copy_(out_first)
        rec[("z", st.first)] = z
        return y

    def _bn_fwd(self, st: Stage, x, y, batch, ei, ef):
        """Batchnorm forward. Under data parallelism the statistics are SYNCHRONISED: column
        sums (phase 1) -> all-reduce over the ranks -> mean / variance of the global batch and
        normalise (phase 2), so every rank normalises with, and keeps, the same running stats
        (one process training on the whole batch)."""
        layer = st.layer
        args = (x, y, self.store.view(st.seg_w), self.store.view(st.seg_b), layer.mean, layer.variance,
                float(layer.eps), float(layer.momentum), True, batch * st.pos_out, st.buffers["mean"],
                st.buffers["invstd"], st.buffers["partial"], ei, ef, 0)
        if not self.ctx.enabled:
            torch.ops.pz.batchnorm_fwd(*args)
            return
        torch.ops.pz.batchnorm_fwd(*args, 1, 0)
        self.ctx.all_reduce_(st.buffers["partial"])
        torch.ops.pz.batchnorm_fwd(*args, 2, self._gbatch * st.pos_out)  # rows of the global sample

    def _scratch(self, key, like):
        buf = getattr(self, "_scratch_bufs", None)
        if buf is None:
            buf = self._scratch_bufs = {}
        t = buf.get(key)
        if t is None or t.shape != like.shape:
            t = buf[key] = torch.empty_like(like)
        return t

    # ------------------------------------------------------------------------------------
    def _head(self, last: Stage, y, batch, p, keys, rec) -> bool:
        """Loss + gradient of the last stage. Returns True when the gradient is wrt the
        producing op (epilogue derivative already applied), False when wrt the stage output."""
        ops = torch.ops.pz
        g = last.buffers["g"]
        fuse = rec is None and last.kind == "gemm"
        bias_grad = self.store.view(last.seg_b, self.grads) if (last.seg_b is not None and last.kind == "gemm") else None
        ei, ef = self._epi(last, p, keys) if fuse else PF.epi_spec()
        n = self.model.layers
        if self.head == "softmax":
            probs = self._scratch(("probs",), y) if rec is not None else None
            gb = self._gbatch  # loss and gradient of the GLOBAL mean (this rank's share of it)
            kw8 = {}
            if fuse and self._head_g8_ok(last, y, g):
                # fp8 policy: the head writes dZ's e5m2 copy itself (no quantisation pass), and
                # not the bf16 dZ when the stage's dX and dW GEMMs both take the copy
                k = last.index
                kw8 = dict(out8=last.buffers["g8"], out8_qscale=self.gqs[k, 0:1], amax=self.gamax[k:k + 1],
                           store_dh=not self._fp8_dw_ready_cached(last))
                self._g8_done[k] = g
            if self._act_su is not None:
                kw8.update(su_amax=self._act_su[0], su_qs=self._act_su[1], su_headroom=self._act_su[2],
                           su_maxval=self._act_su[3], su_qs_prev=self.aqs)
                self._act_su = None
            ops.xent_head(y, self.lab, batch, self.loss_slot, 1.0 / gb, g, 1.0 / gb,
                          bias_grad if fuse else None, probs, ei, ef, 0, **kw8)
            if rec is not None:
                rec[len(n) - 1] = probs[:batch]
                rec[("grad", len(n) - 2)] = g[:batch]
        else:
            cols = y.shape[1]
            gn = self._gbatch * cols
            ops.mse_head(y, self.tgt, batch, self.loss_slot, 1.0 / gn, g, 1.0 / gn,
                         bias_grad if fuse else None, ei, ef, 0)
            if rec is not None:
                rec[("grad", len(n) - 1)] = g[:batch]
        return fuse

    def _backward_stage(self, st: Stage, before: Stage | None, x_in, g, g_pre: bool, batch, p, keys, rec, handles):
        """Consume the gradient of stage `st`; return (gradient for `before`, is_pre flag)."""
        ops = torch.ops.pz
        rows_valid = batch * st.pos_out
        if st.kind == "embed":
            gz = g if g_pre else g  # embedding has no epilogue
            ops.embedding_bwd(gz, x_in, self.store.view(st.seg_w, self.grads))
            return None, True
        # bring g to the producing op (dZ)
        if not g_pre:
            g = self._apply_epi_bwd(st, g, batch, p, keys, rec)
            if st.kind == "gemm" and st.seg_b is not None:
                ops.colsum(g[:rows_valid], self.store.view(st.seg_b, self.grads))
        if st.kind == "flatten":
            if before is None:
                return None, True
            gb = g.view(before.buffers["y"].shape)
            if rec is not None:
                rec[("grad", before.layers[-1])] = gb[:batch * before.pos_out]
            return gb, False
        if st.kind == "bn":
            dx = st.buffers["bn_in_grad"] if before is not None else None
            layer = st.layer
            none = PF.epi_spec()
            bargs = (g, st.buffers["y"] if rec is None else rec[("z", st.first)], x_in, dx,
                     self.store.view(st.seg_w), self.store.view(st.seg_b), st.buffers["mean"],
                     st.buffers["invstd"], self.store.view(st.seg_w, self.grads),
                     self.store.view(st.seg_b, self.grads), st.buffers["partial"], rows_valid, *none, 0)
            if not self.ctx.enabled:
                ops.batchnorm_bwd(*bargs)
            else:  # synchronised: local parameter grads, then dx from the global sums
                ops.batchnorm_bwd(*bargs, 1, 0)
                self.ctx.all_reduce_(st.buffers["partial"])
                ops.batchnorm_bwd(*bargs, 2, self._gbatch * st.pos_out)
            del layer
            if rec is not None and before is not None:
                rec[("grad", before.layers[-1])] = dx[:batch * st.pos_in]
            return dx, False
        # GEMM stage: dW = x_inᵀ · dZ
        if self.fuse_opt and self._ov is not None:
            self._dw_update(st, x_in, g)
            return self._backward_dx(st, before, g, batch, p, keys, rec)
        if st.index == self._pair_idx and rec is None and self._ov is not None:
            # paired backward: this weight's gradient GEMM shares the first layer's launch
            out = self._backward_dx(st, before, g, batch, p, keys, rec)
            self._pair_dw = (st, x_in, g)
            return out
        w_grad = self._w_grad(st.seg_w)
        # fp8 policy: e4m3 activations x e5m2 dZ — _fp8_dw_ready checked the shapes, so when the
        # bf16 dZ went unwritten (store_c=False) the e5m2 copy is always what the dW GEMM reads
        f8 = self._fp8_dw(st, g, w_grad)
        # (measured, not kept: these dW GEMMs on a stream of their own beside the dX chain, without
        # split-K: the concurrent GEMMs stretch each other, mlp4 1.26 vs 1.23 ms —
        # profiles/r3_ab_dw_stream.txt)
        paired = self._pair_dw if st.index == 0 else None
        self._pair_dw = None if st.index == 0 else self._pair_dw
        if paired is not None:
            mine = [self._run_pair(paired, st, x_in, g, w_grad, f8)]
        else:
            if f8 is not None:  # e4m3 activations x e5m2 dZ on the scaled fp8 MFMA
                x8, sx, g8, sg = f8
                PF.gemm(x8, False, g8, False, w_grad, scale_a=sx, scale_b=sg)
            else:
                PF.gemm(x_in, False, g, False, w_grad)
            mine = [self._bucket_seg(st.seg_w)]
        handles.extend(mine)
        # the update writes the OTHER shadow set, but it is queued after this layer's dX GEMM
        # (the fp8 dX operand and the float32 policy's GEMMs read the weight itself)
        own = st.seg_w.offset in self._early_keys
        if self._ov is not None and not own:  # updated by the final launch
            self._late_stages.append(st)
            self._late_handles.extend(mine)
        out = self._backward_dx(st, before, g, batch, p, keys, rec)
        if self._ov is not None and own:
            self._side_pending.append((st.seg_w.offset, mine, [st]))
            if st.seg_w.offset == self._flush_key and self._side_pending:
                self._opt_async(self._side_pending)
                self._side_pending = []
        return out

    def _run_pair(self, paired, st0: Stage, x0, g0, w0, f8_0):
        """The first layer's dW GEMM together with the deferred partner's (``_pair_idx``) in one
        launch when both take the same operand precision and the pair is eligible, else one
        after the other. The partner's bucket and update are queued in the update phase
        (``_pair_late``); returns the first layer's bucket handle."""
        sp, xp, gp = paired
        wp = self._w_grad(sp.seg_w)
        f8_p = self._fp8_dw(sp, gp, wp)
        ops0 = (f8_0[0], f8_0[2]) if f8_0 is not None else (x0, g0)
        opsp = (f8_p[0], f8_p[2]) if f8_p is not None else (xp, gp)
        key = ("pair", (f8_0 is None), (f8_p is None), ops0[0].shape, ops0[1].shape, opsp[0].shape, opsp[1].shape)
        ok = self._y_dead_cache.get(key)
        if ok is None:
            ok = self._y_dead_cache[key] = ((f8_0 is None) == (f8_p is None)
                                            and PF.gemm_pair_split(ops0[0], ops0[1], w0, opsp[0], opsp[1], wp) > 0)
        sk_ok = False
        if ok and self._cus and f8_0 is None:
            # the budgeted engine needs both problems stream-K eligible (a per-rank batch of 64 rows
            # is one 64-deep K step: below the engine's two); otherwise the tiled pair runs
            key_sk = key + ("sk",)
            sk_ok = self._y_dead_cache.get(key_sk)
            if sk_ok is None:
                sk_ok = self._y_dead_cache[key_sk] = PF.gemm_pair_split(ops0[0], ops0[1], w0, opsp[0], opsp[1], wp,
                                                                        engine=2) > 0
        if sk_ok:
            # a bucket is on the wire: the pair's 256-workgroup grid would leave a straggler round
            # behind the CUs the collective holds (239 vs 133 us under the 16-workgroup proxy,
            # profiles/r5_step_timeline_proxy16.txt): both GEMMs as one stream-K schedule on the
            # CUs left to it instead
            PF.gemm_pair(ops0[0], ops0[1], w0, opsp[0], opsp[1], wp, engine=2, cus=self._cus)
        elif ok:
            PF.gemm_pair(ops0[0], ops0[1], w0, opsp[0], opsp[1], wp,
                         scales0=(f8_0[1], f8_0[3]) if f8_0 is not None else (None, None),
                         scales1=(f8_p[1], f8_p[3]) if f8_p is not None else (None, None))
        else:
            for st, (a, b), f8, w in ((sp, opsp, f8_p, wp), (st0, ops0, f8_0, w0)):
                if f8 is not None:
                    PF.gemm(a, False, b, False, w, scale_a=f8[1], scale_b=f8[3])
                else:
                    PF.gemm(a, False, b, False, w)
        # the partner's bucket leaves in the update phase, after the first layer's and the
        # accumulated-gradient bucket: the first-layer update (the step boundary) waits for those
        # two only, and the partner's all-reduce overlaps it (its weight is next read by the next
        # step's later forward GEMMs)
        self._pair_late = (sp, wp)
        return self._bucket_seg(st0.seg_w)

    def _bucket_seg(self, seg):
        """Start a weight's gradient bucket: reduce-scatter (sharded optimizer) or all-reduce (the
        replicated update, and record steps); the GEMMs behind it get the comm CU budget."""
        self._cus = self._cus_comm
        if self._sharded(seg):
            return self.zero.all_reduce(seg.offset) if self._zero_ar else self.zero.reduce_scatter(seg.offset)
        return self.ctx.all_reduce_async(self._w_grad(seg))

    def _sharded(self, seg) -> bool:
        return self.zero is not None and seg.offset in self.zero.shards

    def _dw_update(self, st: Stage, x_in, g) -> None:
        """dW GEMM + the weight's optimizer update in one launch (fuse_opt). The update writes the
        OTHER shadow parity, so this layer's dX GEMM (next) still reads the weights of this step.
        Shapes the MFMA path does not take fall back to dW GEMM + a one-segment update launch."""
        _, l2, scale = self._ov
        parity = 1 - self.parity
        key = (st.seg_w.offset, x_in.shape[0], g.shape[0])
        ok = self._fuse_ok.get(key)
        if ok is None:
            ok = self._fuse_ok[key] = PF.gemm_path(x_in, False, g, False, self.store.view(st.seg_w)) == "mfma"
        if ok:
            self.opt.gemm_update(x_in, False, g, False, st.seg_w, l2, scale, parity)
        else:
            PF.gemm(x_in, False, g, False, self._w_grad(st.seg_w))
            self.opt.step_group(st.seg_w.offset, self.grads, l2, scale, parity)

    def _backward_dx(self, st: Stage, before: Stage | None, g, batch, p, keys, rec):
        if before is None:
            return None, True
        # dX = dZ · Wᵀ (+ previous stage's epilogue derivative and bias colsum when fusable)
        dx = before.buffers["g"]
        fuse_prev = rec is None and before.kind in ("gemm", "bn", "flatten") and before.has_epi
        if fuse_prev:
            ei, ef = self._epi(before, p, keys)
            colsum = self.store.view(before.seg_b, self.grads) if (before.kind == "gemm" and before.seg_b is not None) \
                else None
            mask = before.buffers.get("mask")
            # the receiving stage's fp8 dW wants dZ in e5m2: written by this epilogue once its
            # delayed scale is calibrated (first step: the amax of the bf16 dZ, below)
            b = before.index
            kw8 = {}
            if getattr(before, "g8_from_epi", False) and b in self._g8_epi_ready:
                kw8 = dict(out8=before.buffers["g8"], out8_qscale=self.gqs[b, 0:1], amax=self.gamax[b:b + 1])
                if b == 0 and self._fp8_dw_ready_cached(before):
                    # the first stage has no dX GEMM and its dW reads the e5m2 copy: the bf16 dZ
                    # is not written (mlp8192: 128 MB a step)
                    kw8["store_c"] = False
            if getattr(st, "fp8_bwd", False):  # e5m2 dZ x e4m3 W on the scaled fp8 MFMA
                k, g8 = st.index, self._quantize_g8(st, g)
                PF.gemm(g8, True, self.w8n[st.seg_w.offset], True, dx,
                        aux=None if mask is not None else before.buffers["y"], colsum=colsum, mode=PF.EPI_BWD,
                        epi=(ei, ef), mask=mask, scale_a=self.gqs[k, 1:2], scale_b=self.wqs[st.w8_index, 1:2],
                        **kw8)
            else:
                PF.gemm(g, True, self._w(st), True, dx, aux=None if mask is not None else before.buffers["y"],
                        colsum=colsum, mode=PF.EPI_BWD, epi=(ei, ef), mask=mask, **kw8)
            if kw8:
                self._g8_done[b] = dx
            elif getattr(before, "g8_from_epi", False) and rec is None and self._ov is not None \
                    and self._run_epoch is not None:  # eager step: calibrate the delayed scale
                torch.ops.pz.amax_abs(dx, self.gamax[b:b + 1])
                self._g8_epi_ready.add(b)
            return dx, True
        no_epi_prev = before.kind in ("gemm",) and not before.has_epi and rec is None
        colsum = None
        if no_epi_prev and before.seg_b is not None:
            colsum = self.store.view(before.seg_b, self.grads)
        PF.gemm(g, True, self._w(st), True, dx, colsum=colsum, mode=PF.EPI_STORE)
        if rec is not None:
            rec[("grad", before.layers[-1])] = dx[:batch * before.pos_out]
        if no_epi_prev or before.kind == "embed":
            return dx, True
        return dx, False

    def _apply_epi_bwd(self, st: Stage, g, batch, p, keys, rec):
        """dY (wrt stage output) -> dZ (wrt producing op); record mode keeps the per-layer grads."""
        ops = torch.ops.pz
        if not st.has_epi:
            return g
        if rec is None:
            dz = self._scratch(("dz", st.first), g)
            ops.stage_bwd(g, st.buffers["y"], dz, *self._epi(st, p, keys))
            return dz
        # record: y_act = stage output; out_first = output of the first layer of the stage
        out_first = self._scratch(("o", st.first), g)
        if st.act_layer >= 0:
            g_first = self._scratch(("go", st.first), g)
            ops.stage_bwd(g, st.buffers["y"], g_first, *self._epi(st, p, keys, parts=("act", "post")))
            rec[("grad", st.first)] = g_first[:batch * st.pos_out]
        else:
            g_first = g
        dz = self._scratch(("dz", st.first), g)
        ops.stage_bwd(g_first, out_first, dz, *self._epi(st, p, keys, parts=("pre",)))
        return dz

    # ------------------------------------------------------------------------------------
    # record / progress plumbing
    # ------------------------------------------------------------------------------------
    def _finish_record(self, rec, batch, l2):
        n = len(self.model.layers)
        acts, grads = [], []
        for i in range(n):
            a = rec.get(i)
            if a is None:
                raise RuntimeError(f"record mode missed layer {i}")
            acts.append(a.detach().clone())
            gi = rec.get(("grad", i))
            grads.append(gi.detach().clone() if gi is not None else None)
        wgrads = []
        for i, layer in enumerate(self.model.layers):
            seg = self.store.segment_for(i, "weights") if layer.weights is not None else None
            if seg is None:
                wgrads.append(None)
                continue
            gview = self._w_grad(seg).to(self.master)  # the all-reduced sum is the global mean already
            wgrads.append(gview + (2.0 * l2) * self.store.view(seg))
        self._record = {"activations": acts, "act_grads": grads, "weight_grads": wgrads}

    def _alloc_progress(self, epochs: int) -> None:
        points = math.ceil(epochs / max(1, epochs // 100)) + 1
        self.costs = torch.zeros(max(epochs, 1), device=self.dev, dtype=torch.float64)
        self.ratios = torch.zeros(points * max(1, self.opt.nslots), device=self.dev, dtype=torch.float32)
        self._ratio_rows = 0
        self._pending = []
        torch.cuda.synchronize(self.dev)  # (the previous run's stamps have completed)
        self.events.release()
        self._start_event = self.events.stamp(torch.cuda.current_stream(self.dev))
        self._last_ms = 0.0
        self.step_ms = {}
        torch.cuda.synchronize(self.dev)
        self._start_wall = datetime.now()

    def drain(self):
        """Yield ``(epoch, cost, ratios|None, iso_time)`` for every step since the last drain."""
        if not self._pending:
            return []
        torch.cuda.synchronize(self.dev)
        self._main_joined = False  # (device-synchronised: the next step re-joins the caller's stream)
        costs = self.costs.cpu().tolist()
        ratios = self.ratios.cpu().view(-1, max(1, self.opt.nslots)).tolist()
        out = []
        self.step_ms = {}  # epoch -> GPU time since the previous step ended (ms), for telemetry
        for epoch, row, ev in self._pending:
            ms = self.events.elapsed(self._start_event, ev)
            when = (self._start_wall + timedelta(milliseconds=ms)).isoformat()
            r = ratios[row][:self.opt.nslots] if row is not None else None
            out.append((epoch, costs[epoch], r, when))
            self.step_ms[epoch] = ms - self._last_ms
            self._last_ms = ms
        self._pending = []
        self.events.release(keep=self._start_event)  # (read: the step timestamps can go)
        if self.zero is not None:  # whole masters and Adam moments for the checkpoint / inference
            self.zero.gather_state(self.store.flat, self.opt.exp_avg, self.opt.exp_avg_sq)
        self.opt.sync_torch_state()
        return out

    def record(self):
        if self._record is None:
            raise RuntimeError("no record-mode step has run")
        return self._record

    def close(self, ok: bool = True) -> None:
        """Release the trainer's HIP events (after its last drain). ``ok=False`` (the run failed):
        no device synchronize — it could wait forever on a stuck collective or a faulted stream
        and replace the original error — the events are dropped, not destroyed."""
        if ok:
            torch.cuda.synchronize(self.dev)
            self.events.close()
        else:
            self.events.abandon()

    # convenience for benchmarks / tests --------------------------------------------------
    def synchronize(self) -> None:
        torch.cuda.synchronize(self.dev)


__all__ = ["FusedTrainer", "UnsupportedModel", "compile_stages", "time"]
