"""fp8 policy of the fused trainer (BASELINE config 5): which GEMM stages run on e4m3 / e5m2
operands, the per-tensor delayed-scaling records, and the weight copies — the methods of
:class:`..trainer.FusedTrainer` that only the fp8 precision uses (a mixin: they read the trainer's
stages, buffers and scale records). Forward: e4m3 activations (written by the producing GEMM's
epilogue) x e4m3 weights; backward: e5m2 dZ x e4m3 weights (dX) and e4m3 activations x e5m2 dZ
(dW), on the scaled fp8 MFMA (csrc/gemm_mfma.hip VAR 8-17)."""
from __future__ import annotations

from typing import TYPE_CHECKING

import torch

from ..ops import functional as PF

if TYPE_CHECKING:
    from .trainer import Stage


class Fp8Policy:
    def _refresh_fp8_weights(self, only: Stage | None = None, parity: int | None = None) -> None:
        """Current-scaled e4m3 weight copies, transposed to [out, in] (K-contiguous GEMM operand).
        ``parity``: the shadow parity of the optimizer update that just wrote the weights (its amax
        is already reduced); None: reduce the amax here (initial copies)."""
        ops = torch.ops.pz
        if parity is not None and self._w8_fused:
            return  # the optimizer update wrote the e4m3 copies and their scale records
        for st in self.stages if only is None else [only]:
            if st.kind != "gemm":
                continue
            k = st.w8_index
            w = self.store.view(st.seg_w)
            if self._w8_nat:
                w8 = self.w8[st.seg_w.offset]
                if parity is not None:  # q from the amax the update reduced; clear the other parity's
                    p = parity % 2
                    ops.quantize_rows(w, w8, self.wqs[k], None, self.wamax2[p, k:k + 1], self.wamax2[1 - p, k:k + 1])
                else:
                    ops.amax_abs(w, self.wamax[k:k + 1])
                    ops.scale_update(self.wamax[k:k + 1], self.wqs[k], 1.0, True)
                    ops.quantize_rows(w, w8, self.wqs[k], None)
                continue
            if parity is not None:
                p = parity % 2
                ops.quant_transpose(w, self.w8[st.seg_w.offset], self.wqs[k], self.wamax2[p, k:k + 1],
                                    self.wamax2[1 - p, k:k + 1])
            else:
                ops.amax_abs(w, self.wamax[k:k + 1])
                ops.scale_update(self.wamax[k:k + 1], self.wqs[k], 1.0, True)
                ops.quant_transpose(w, self.w8[st.seg_w.offset], self.wqs[k])
            w8n = self.w8n.get(st.seg_w.offset)
            if w8n is not None:  # [in, out] copy for the backward dX GEMM, same scale
                ops.quantize_rows(w, w8n, self.wqs[k], None)

    def _plan_fp8(self, rows_b: int) -> None:
        """Which GEMM stages run their forward on e4m3 operands (shape-eligible ones)."""
        for st in self.stages:
            st.fp8 = False
            st.buffers.pop("y8", None)
        if not self.fp8:
            return
        self.x8 = None
        for i, st in enumerate(self.stages):
            if st.kind != "gemm":
                continue
            prev = self.stages[i - 1] if i > 0 else None
            if prev is None:
                x = self.x_in
                if x.dtype != torch.bfloat16 or x.shape[1] % 64:
                    continue
                x8 = torch.empty(x.shape, device=self.dev, dtype=torch.float8_e4m3fn)
            else:
                # the producing GEMM writes the e4m3 copy from its epilogue: it must be on the MFMA path
                if prev.kind != "gemm" or prev.buffers["y"].shape[1] % 64:
                    continue
                px = self.x8 if prev.fp8 and prev.index == 0 else (
                    self.stages[prev.index - 1].buffers.get("y8") if prev.fp8 else
                    (self.stages[prev.index - 1].buffers["y"] if prev.index > 0 else self.x_in))
                pw = self.w8[prev.seg_w.offset] if prev.fp8 else self._w(prev)
                if px is None or PF.gemm_path(px, True, pw, prev.fp8 and self.w8_kc, prev.buffers["y"]) != "mfma":
                    continue
                x8 = torch.empty(prev.buffers["y"].shape, device=self.dev, dtype=torch.float8_e4m3fn)
            if PF.gemm_path(x8, True, self.w8[st.seg_w.offset], self.w8_kc, st.buffers["y"]) != "mfma":
                continue
            st.fp8 = True
            if prev is None:
                self.x8 = x8
            else:
                prev.buffers["y8"] = x8
        for i, st in enumerate(self.stages):  # backward: e5m2 dZ x e4m3 W for fused dX GEMMs
            st.fp8_bwd = False
            st.buffers.pop("g8", None)
            prev = self.stages[i - 1] if i > 0 else None
            # (the [in, out] e4m3 copy is single-buffered: the update of W must not run before this
            # step's dX GEMM has read it — true with the updates queued after the dX GEMMs)
            if (st.kind != "gemm" or not st.fp8 or prev is None or prev.kind != "gemm" or not prev.has_epi
                    or st.seg_w.offset not in self.w8n):
                continue
            if st.out_width % 64 or prev.out_width % 8 or rows_b < 64:
                continue
            st.fp8_bwd = True
            st.buffers["g8"] = torch.empty(st.buffers["g"].shape, device=self.dev, dtype=torch.float8_e5m2)
        # fp8 dW for fp8 stages whose dZ is NOT quantised for a dX GEMM (the first layer): the next
        # stage's fused dX GEMM writes dZ's e5m2 copy from its epilogue (delayed scaling), so the
        # weight-gradient GEMM runs on e4m3 x e5m2 without a separate quantisation pass
        for i, st in enumerate(self.stages):
            st.g8_from_epi = False
            nxt = self.stages[i + 1] if i + 1 < len(self.stages) else None
            if (st.kind != "gemm" or not st.fp8 or getattr(st, "fp8_bwd", False)
                    or nxt is None or nxt.kind != "gemm" or not st.has_epi or st.out_width % 256
                    or st.in_width % 256 or rows_b % 64):
                continue
            st.g8_from_epi = True
            st.buffers["g8"] = torch.empty(st.buffers["g"].shape, device=self.dev, dtype=torch.float8_e5m2)
        self._g8_epi_ready = set()
        self._y_dead_cache = {}
        self.data8 = None
        if self.x8 is not None:
            # first-layer input: the device-resident dataset is quantised to e4m3 ONCE with a static
            # dataset-wide scale (its amax bounds every minibatch's), and the per-step gather copies
            # the sampled e4m3 rows next to the bf16 ones: no per-step amax / quantise pass
            ops = torch.ops.pz
            self.data8 = torch.empty(self.data.shape, device=self.dev, dtype=torch.float8_e4m3fn)
            self.xamax.zero_()
            ops.amax_abs(self.data, self.xamax)
            ops.scale_update(self.xamax, self.xqs, 1.0, True)
            ops.quantize_rows(self.data, self.data8, self.xqs, None)

    def _quantize_g8(self, st: Stage, g):
        """dZ of an fp8 stage -> its e5m2 copy (delayed scaling; the first step calibrates on its
        own amax), once per step: the dW GEMM and the dX GEMM of the stage both consume it."""
        g8 = st.buffers["g8"]
        if self._g8_done.get(st.index) is g:
            return g8
        k, ops = st.index, torch.ops.pz
        if not self._g8_calibrated:  # first step: current scaling from this gradient
            ops.amax_abs(g, self.gamax[k:k + 1])
            ops.scale_update(self.gamax[k:k + 1], self.gqs[k], 2.0, True, 57344.0)
        ops.quantize_rows(g, g8, self.gqs[k], self.gamax[k:k + 1])
        self._g8_done[st.index] = g
        return g8

    def _head_g8_ok(self, last: Stage, y, g) -> bool:
        """The softmax head can write the last stage's e5m2 dZ (fp8 dX stage, delayed scale
        calibrated, the head kernel's bf16 fast path)."""
        if not (self.fp8 and getattr(last, "fp8_bwd", False) and self._g8_calibrated and "g8" in last.buffers):
            return False
        key = ("head", last.index)
        if key not in self._y_dead_cache:
            cols = y.shape[1]
            self._y_dead_cache[key] = (y.dtype == torch.bfloat16 and g.dtype == torch.bfloat16 and cols % 8 == 0
                                       and cols <= 2048 and y.stride(0) % 8 == 0 and g.stride(0) % 8 == 0)
        return self._y_dead_cache[key]

    def _fp8_dw_ready(self, st: Stage) -> bool:
        """This step's dW GEMM of ``st`` will run on fp8 operands (``_fp8_dw`` returns them)."""
        if not (self.fp8 and st.fp8 and st.kind == "gemm"):
            return False
        if getattr(st, "g8_from_epi", False):
            if st.index not in self._g8_epi_ready:
                return False
        elif not getattr(st, "fp8_bwd", False):
            return False
        x8 = self.x8 if st.index == 0 else self.stages[st.index - 1].buffers.get("y8")
        w_grad = self._w_grad(st.seg_w)
        return x8 is not None and w_grad.dtype == torch.bfloat16 and self._fp8_dw_shape_ok(st, x8, w_grad)

    def _fp8_dw_shape_ok(self, st: Stage, x8, w_grad) -> bool:
        """The fp8 dW GEMM (x8 x e5m2 dZ) takes the MFMA path."""
        key = ("dwshape", st.index)
        ok = self._y_dead_cache.get(key)
        if ok is None:
            ok = self._y_dead_cache[key] = PF.gemm_path(x8, False, st.buffers["g8"], False, w_grad) == "mfma"
        return ok

    def _fp8_dw_ready_cached(self, st: Stage) -> bool:
        key = ("dw", st.index, st.index in self._g8_epi_ready)
        if key not in self._y_dead_cache:
            self._y_dead_cache[key] = self._fp8_dw_ready(st)
        return self._y_dead_cache[key]

    def _y_dead(self, st: Stage) -> bool:
        """fp8 policy: nobody reads the bf16 output of ``st`` this step — the next stage's forward
        and weight-gradient GEMMs take its e4m3 copy, the next dX GEMM's ReLU derivative its
        bitmask — so the forward epilogue writes only those (mlp8192: 128 MB of writes a step)."""
        if "y8" not in st.buffers or st.buffers.get("mask") is None or st.index + 1 >= len(self.stages):
            return False
        return self._fp8_dw_ready_cached(self.stages[st.index + 1])

    def _fp8_dw(self, st: Stage, g, w_grad):
        """fp8 weight-gradient operands (BASELINE config 5): the stage input's e4m3 copy (written by
        the previous GEMM's epilogue, or the gathered e4m3 dataset rows) and dZ's e5m2 copy, both
        M/N-contiguous, with their dequantisation factors — or None (bf16 dW)."""
        if not (self.fp8 and st.fp8):
            return None
        if getattr(st, "g8_from_epi", False):  # dZ's e5m2 copy came from the dX epilogue this step
            if self._g8_done.get(st.index) is not g:
                return None
        elif not getattr(st, "fp8_bwd", False):
            return None
        i = st.index
        x8, sx = (self.x8, self.xqs[1:2]) if i == 0 else (self.stages[i - 1].buffers.get("y8"), self.aqs[i - 1, 1:2])
        if x8 is None or w_grad.dtype != torch.bfloat16:
            return None
        if not self._fp8_dw_shape_ok(st, x8, w_grad):
            return None
        return x8, sx, self._quantize_g8(st, g), self.gqs[i, 1:2]
