"""Flat device-resident parameter store (the GPU model's memory layout).

Every parameter of a GPU model lives in ONE contiguous master buffer; ``layer.weights`` /
``layer.bias`` / ``layer.gain`` are views into it. One buffer means one optimizer launch for all
parameters, one (or a few, bucketed) RCCL all-reduce(s) for all gradients, and one D2H copy per
checkpoint.

Layout (sized for 288 GB HBM: even the 1.07 B-parameter 16x8192 MLP is 4.3 GB of fp32 master):

    [ dense weights (GEMM-written grads) | accumulated params: embedding tables, biases, BN ]

Dense weight gradients are fully overwritten by the dW GEMMs each step; everything in the
second region receives atomically accumulated gradients, so only that (small) region is zeroed
per step. Each segment starts on a 64-element boundary so vector kernels stay 256-B aligned.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

ALIGN = 64


def _round_up(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


@dataclass
class Segment:
    layer_index: int
    attr: str            # "weights" | "bias" | "gain"
    offset: int
    numel: int
    shape: tuple
    is_weight: bool      # reference "weights" (linear/embedding W): L2 + update ratios apply
    dense: bool          # gradient written (not accumulated) by a GEMM
    param_index: int     # position in model.params (optimizer / checkpoint order)


class ParamStore:
    def __init__(self, flat: torch.Tensor, segments: list[Segment], accum_offset: int):
        self.flat = flat
        self.segments = segments
        self.accum_offset = accum_offset   # start of the zero-per-step gradient region

    @property
    def numel(self) -> int:
        return self.flat.numel()

    @property
    def device(self) -> torch.device:
        return self.flat.device

    def view(self, seg: Segment, buf: torch.Tensor | None = None) -> torch.Tensor:
        base = self.flat if buf is None else buf
        return base[seg.offset:seg.offset + seg.numel].view(seg.shape)

    def segment_for(self, layer_index: int, attr: str) -> Segment | None:
        for s in self.segments:
            if s.layer_index == layer_index and s.attr == attr:
                return s
        return None

    @classmethod
    def adopt(cls, layers, device: torch.device, dtype: torch.dtype) -> "ParamStore":
        """Copy every layer parameter into one flat buffer and re-point the layers at views."""
        entries = []  # (layer_index, attr, tensor, is_weight, dense, param_index)
        pidx = 0
        for li, layer in enumerate(layers):
            for attr in ("weights", "gain", "bias"):
                t = getattr(layer, attr, None)
                if t is None or (attr == "weights" and layer.algo == "batchnorm"):
                    continue
                is_weight = attr == "weights"
                dense = is_weight and layer.algo == "linear"
                entries.append((li, attr, t, is_weight, dense))
        # param order must match model.params: per layer [weights, bias] or BN [gain, bias]
        order = {}
        for li, layer in enumerate(layers):
            for p in layer.params:
                order[id(p)] = pidx
                pidx += 1
        dense_first = sorted(entries, key=lambda e: (not e[4], e[0]))
        offset = 0
        segments: list[Segment] = []
        accum_offset = None
        for li, attr, t, is_weight, dense in dense_first:
            if not dense and accum_offset is None:
                accum_offset = offset
            segments.append(Segment(li, attr, offset, t.numel(), tuple(t.shape), is_weight, dense, order[id(t)]))
            offset += _round_up(t.numel())
        if accum_offset is None:
            accum_offset = offset
        flat = torch.zeros(max(offset, 1), device=device, dtype=dtype)
        store = cls(flat, segments, accum_offset)
        for seg in segments:
            layer = layers[seg.layer_index]
            src = getattr(layer, seg.attr)
            view = store.view(seg)
            view.copy_(src.detach().to(device=device, dtype=dtype))
            setattr(layer, seg.attr, view)
        for layer in layers:
            layer.device, layer.dtype = torch.device(device), dtype
            if layer.algo == "batchnorm" and layer.mean is not None:
                layer.mean = layer.mean.detach().to(device=device, dtype=dtype).reshape(-1).clone()
                layer.variance = layer.variance.detach().to(device=device, dtype=dtype).reshape(-1).clone()
        return store
