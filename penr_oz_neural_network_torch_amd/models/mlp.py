"""Model builder (reference L3, ``neural_net_model.py:190-267``).

``normalize_algos`` is the reference's "linear sandwich" rule; ``MultiLayerPerceptron`` turns the
normalised algo list + ``layer_sizes`` into layers, applies the weight initialisation scheme and
marks hidden layers. Random draws happen in the reference's order, so ``torch.manual_seed(s)``
produces the reference's initial parameters exactly.
"""
from __future__ import annotations

import math

from torch import Tensor

from .layers import (ACTIVATIONS, BatchNormLayer, EmbeddingLayer, FlattenLayer, Layer, LinearLayer, ReluLayer,
                     SigmoidLayer, SoftmaxLayer, TanhLayer)

_PRODUCERS = ("batchnorm", "linear")   # what may directly precede an activation
_SIZE_CONSUMERS = ("embedding", "flatten", "linear")


def normalize_algos(algos: list[str]) -> list[str]:
    """Insert the implicit layers (``neural_net_model.py:202-212``).

    Walking the user's list right to left: an activation not preceded by ``linear`` or
    ``batchnorm`` gets a ``linear`` in front of it; an ``embedding`` not followed by ``flatten``
    gets one inserted at position ``i + 1`` of the list built so far (the reference's exact
    placement, which is "right after the embedding" whenever the embedding comes first).
    Normalised lists are fixed points, which is what lets checkpoints store them.
    """
    out: list[str] = []
    for i in range(len(algos) - 1, -1, -1):
        algo = algos[i]
        out.insert(0, algo)
        if algo in ACTIVATIONS:
            if i == 0 or algos[i - 1] not in _PRODUCERS:
                out.insert(0, "linear")
        elif algo == "embedding" and algos[i + 1] != "flatten":
            out.insert(i + 1, "flatten")
    return out


def _make_layer(algo: str, in_sz: int, out_sz: int, bias_algo, batchnorm) -> Layer:
    if algo == "embedding":
        return EmbeddingLayer(in_sz, out_sz)
    if algo == "flatten":
        return FlattenLayer(out_sz // max(1, in_sz))
    if algo == "linear":
        return LinearLayer(in_sz, out_sz, bias_algo)
    if algo == "batchnorm":
        return BatchNormLayer(in_sz, *batchnorm)
    simple = {"relu": ReluLayer, "sigmoid": SigmoidLayer, "softmax": SoftmaxLayer, "tanh": TanhLayer}.get(algo)
    if simple is None:
        raise ValueError(f"Unsupported activation algorithm: {algo}")
    return simple()


class MultiLayerPerceptron:
    def __init__(self, layer_sizes: list[int], weight_algo="xavier", bias_algo="zeros",
                 activation_algos: list[str] | None = None, batchnorm=(1e-5, 0.1)):
        self.algos = normalize_algos(activation_algos or ["relu"] * (len(layer_sizes) - 1))
        self.layers: list[Layer] = []
        n_sizes, n_algos = len(layer_sizes), len(self.algos)
        size_idx = 0
        gain_target: LinearLayer | None = None   # most recent linear layer under "he" init
        for i, algo in enumerate(self.algos):
            in_sz = layer_sizes[size_idx] if size_idx < n_sizes else 0
            out_sz = layer_sizes[size_idx + 1] if size_idx + 1 < n_sizes else 0
            layer = _make_layer(algo, in_sz, out_sz, bias_algo, batchnorm)
            if algo == "linear":
                # xavier / he: unit fan-in variance (embedding tables keep raw randn)
                if in_sz > 0 and weight_algo in ("xavier", "he") and layer.weights is not None:
                    layer.weights /= math.sqrt(in_sz)
                gain_target = layer if weight_algo == "he" else None
            if gain_target is not None and gain_target.weights is not None and algo in ("relu", "tanh"):
                gain_target.weights *= (ReluLayer if algo == "relu" else TanhLayer).weight_gain
            layer.hidden = 0 < i < n_algos - 1
            self.layers.append(layer)
            if algo in _SIZE_CONSUMERS:
                size_idx += 1

    @property
    def params(self) -> list[Tensor]:
        return [p for layer in self.layers for p in layer.params]


__all__ = ["MultiLayerPerceptron", "normalize_algos"]
