"""Training diagnostics (reference R23, ``neural_net_model.py:532-585``).

Produces the exact ``stats`` schema the dashboard consumes::

    {"layers":  [{"algo", "activation": {"mean","std","saturated","histogram":{"x","y"}},
                  "gradient": {"mean","std","histogram"} | None}, ...],
     "weights": [{"shape", "data": {"mean","std"},
                  "gradient": {"mean","std","histogram"}} | None, ...]}

Histograms follow ``torch.histogram(t, density=True)`` semantics: 100 bins over
``[min, max]`` (widened by ±0.5 when ``min == max``), ``x`` = left bin edges, ``y`` = density.

CPU tensors use ATen (identical to the reference). GPU tensors use the fused ``pz`` stats
kernels (one pass for min/max/sum/sum²/saturation + one histogram pass; ``torch.histogram`` has
no GPU kernel) and a single device→host copy per tensor.
"""
from __future__ import annotations

import torch
from torch import Tensor

HIST_BINS = 100

# saturation rule per algo (reference neural_net_model.py:555-562)
_SAT_RULES = {
    "embedding": ("row_norm_gt", 5.0),
    "batchnorm": ("abs_gt", 3.0),
    "tanh": ("abs_gt", 0.97),
    "sigmoid": ("abs_gt", 0.97),
    "relu": ("le", 0.0),
    "softmax": ("row_max_gt", 0.97),
}


def saturation_rule(algo: str) -> tuple[str, float]:
    return _SAT_RULES.get(algo, ("abs_gt", 5.0))


def _cpu_saturation(a: Tensor, algo: str) -> float:
    kind, thr = saturation_rule(algo)
    if kind == "row_norm_gt":
        mask = torch.norm(a, dim=-1) > thr
    elif kind == "abs_gt":
        mask = a.abs() > thr
    elif kind == "le":
        mask = a <= thr
    else:
        mask = a.max(dim=-1).values > thr
    return mask.float().mean().item()


def _cpu_hist(t: Tensor) -> tuple[list, list]:
    h = torch.histogram(t, density=True)
    return h.bin_edges[:-1].tolist(), h.hist.tolist()


def summarize(t: Tensor, algo: str | None = None, hist: bool = True) -> dict:
    """mean / unbiased std / optional saturation / optional density histogram of ``t``."""
    t = t.detach()
    if t.is_cuda:
        from ..ops import functional as PF
        return PF.tensor_summary(t, algo, HIST_BINS if hist else 0)
    out = {"mean": t.mean().item(), "std": t.std().item()}
    if algo is not None:
        out["saturated"] = _cpu_saturation(t, algo)
    if hist:
        x, y = _cpu_hist(t)
        out["histogram"] = {"x": x, "y": y}
    return out


def build_stats(layers, activations: list[Tensor], act_grads: list[Tensor | None],
                weight_grads: list[Tensor | None]) -> dict:
    """Assemble the reference ``stats`` dict. ``weight_grads[i]`` pairs with ``layers[i]``."""
    layer_stats = []
    for layer, a, g in zip(layers, activations, act_grads):
        act = summarize(a, layer.algo)
        entry = {
            "algo": layer.algo,
            "activation": {"mean": act["mean"], "std": act["std"], "saturated": act["saturated"],
                           "histogram": act["histogram"]},
            "gradient": None,
        }
        if g is not None:
            gs = summarize(g)
            entry["gradient"] = {"mean": gs["mean"], "std": gs["std"], "histogram": gs["histogram"]}
        layer_stats.append(entry)
    weight_stats = []
    for layer, wg in zip(layers, weight_grads):
        if layer.weights is None:
            weight_stats.append(None)
            continue
        data = summarize(layer.weights, hist=False)
        gs = summarize(wg)
        weight_stats.append({
            "shape": str(tuple(layer.weights.shape)),
            "data": {"mean": data["mean"], "std": data["std"]},
            "gradient": {"mean": gs["mean"], "std": gs["std"], "histogram": gs["histogram"]},
        })
    return {"layers": layer_stats, "weights": weight_stats}
