"""Layer library (reference L2, ``neural_net_model.py:16-188``).

Each layer keeps the reference's public surface — ``params``, ``state_dict`` (get/set), ``forward``,
``hidden``, ``training``, class attributes ``algo`` / ``weight_gain`` — and its math. The device
decides the implementation:

* **CPU tensors** run the reference's ATen expressions op for op (fp64 models stay bit-identical
  to the reference, which the reference's own 1e-17-tolerance backward tests rely on).
* **GPU tensors** run the hand-written HIP kernels through :mod:`..ops.functional` (MFMA GEMM,
  fused stage kernels, softmax, batchnorm, embedding) with autograd support. There is no ATen
  fallback on the GPU path: a missing native library is an error.

Weight layout stays ``[in, out]`` (``forward = x @ W``, reference ``neural_net_model.py:117``);
the GEMM kernels consume it directly (NN forward, TN dW, NT dX), nothing is transposed.
"""
from __future__ import annotations

import math

import torch
from torch import Tensor

_CPU = torch.device("cpu")


def _on_gpu(t: Tensor | None) -> bool:
    return t is not None and t.is_cuda


def set_bn_sync(layers, ctx) -> None:
    """Synchronised batchnorm for ONE model's layers: while ``ctx`` (a data-parallel context with
    world size > 1) is set on its BatchNormLayers, their training forward normalises the global
    batch (statistics all-reduced over the ranks). Per layer instance, never process-wide: the
    REST service trains other models in other threads at the same time."""
    sync = ctx if ctx is not None and ctx.enabled else None
    for layer in layers:
        if isinstance(layer, BatchNormLayer):
            layer.sync = sync


def _pf():
    from ..ops import functional as PF
    return PF


def _f64(values) -> Tensor:
    """Checkpoint values -> fp64 tensor: nested lists (reference loader) or tensors (native reader)."""
    if isinstance(values, Tensor):
        return values.detach().to(dtype=torch.float64, device=_CPU, copy=True)
    return torch.tensor(values, dtype=torch.float64)


def _randn_fp64(*shape: int) -> Tensor:
    """Initial values drawn exactly like the reference: fp32 ``randn`` widened to fp64
    (``neural_net_model.py:65,104,108``), so a seeded model equals the reference's bit for bit."""
    return torch.randn(*shape).double()


class Layer:
    """Identity layer with optional ``weights`` / ``bias`` (reference ``Layer``, ``:16-53``)."""

    algo = ""

    def __init__(self):
        self.hidden = False
        self.training = False
        self.weights: Tensor | None = None
        self.bias: Tensor | None = None
        # where the parameters live; GPU models re-point these at views of a flat device store
        self.device = _CPU
        self.dtype = torch.float64

    @property
    def params(self) -> list[Tensor]:
        return [t for t in (self.weights, self.bias) if t is not None]

    @property
    def state_dict(self) -> dict:
        return {"params": [p.tolist() for p in self.params]}

    @state_dict.setter
    def state_dict(self, new_state: dict):
        values = new_state["params"]
        if values:
            self.weights = _f64(values[0])
        if len(values) > 1:
            self.bias = _f64(values[1])

    def checkpoint_state(self, ref) -> dict:
        """``state_dict`` with parameter tensors wrapped by ``ref`` (rendered natively later)."""
        return {"params": [ref(p) for p in self.params]}

    def forward(self, input_tensor: Tensor) -> Tensor:
        return input_tensor


class EmbeddingLayer(Layer):
    """Token-id lookup ``W[ids]`` (``:55-68``); GPU: gather kernel fwd, atomic scatter-add bwd."""

    algo = "embedding"

    def __init__(self, vocab_size: int = 0, embedding_size: int = 0):
        super().__init__()
        if vocab_size > 0 and embedding_size > 0:
            self.weights = _randn_fp64(vocab_size, embedding_size)

    def forward(self, input_tensor: Tensor) -> Tensor:
        if _on_gpu(self.weights):
            return _pf().embedding(input_tensor, self.weights)
        return self.weights[input_tensor.long()]


class FlattenLayer(Layer):
    """Merge ``ratio`` adjacent positions: ``[..., T, C] -> [..., T/r, C*r]`` (``:70-91``).
    A pure view on every device."""

    algo = "flatten"

    def __init__(self, ratio: int):
        super().__init__()
        self.ratio = ratio

    @property
    def state_dict(self) -> dict:
        return {"ratio": self.ratio}

    @state_dict.setter
    def state_dict(self, new_state: dict):
        self.ratio = new_state["ratio"]

    def checkpoint_state(self, ref) -> dict:
        return {"ratio": self.ratio}

    def forward(self, input_tensor: Tensor) -> Tensor:
        if input_tensor.ndim <= 1:
            return input_tensor
        shape = list(input_tensor.shape)
        shape[-2] //= self.ratio
        shape[-1] *= self.ratio
        out = input_tensor.view(*shape)
        return out.squeeze(len(shape) - 2) if shape[-2] == 1 else out


class LinearLayer(Layer):
    """``x @ W + b`` with ``W`` stored ``[in, out]`` (``:93-120``)."""

    algo = "linear"

    def __init__(self, input_size: int = 0, output_size: int = 0, bias_algo="zeros"):
        super().__init__()
        if input_size > 0 and output_size > 0:
            self.weights = _randn_fp64(input_size, output_size)
            if bias_algo:
                self.bias = torch.zeros(output_size).double() if bias_algo == "zeros" else _randn_fp64(output_size)

    def forward(self, input_tensor: Tensor) -> Tensor:
        if _on_gpu(self.weights):
            return _pf().linear(input_tensor, self.weights, self.bias)
        out = input_tensor @ self.weights
        if self.bias is not None:
            out += self.bias
        return out


class BatchNormLayer(Layer):
    """Batch normalisation over every dim but the last (``:122-170``): unbiased batch variance,
    EMA running statistics updated in training, running statistics used in eval. Running stats
    are not persisted (the setter resets them, like the reference)."""

    algo = "batchnorm"

    def __init__(self, dim_size: int, eps=1e-5, momentum=0.1):
        super().__init__()
        self.eps = eps
        self.momentum = momentum
        have = dim_size > 0
        self.gain = torch.ones(dim_size, dtype=torch.float64) if have else None
        self.bias = torch.zeros(dim_size, dtype=torch.float64) if have else None
        self.variance = torch.ones(dim_size, dtype=torch.float64) if have else None
        self.mean = torch.zeros(dim_size, dtype=torch.float64) if have else None
        self.sync = None  # data-parallel context of a synchronised training run (set_bn_sync)

    @property
    def params(self) -> list[Tensor]:
        return [t for t in (self.gain, self.bias) if t is not None]

    @property
    def state_dict(self) -> dict:
        return {"params": [p.tolist() for p in self.params], "eps": self.eps, "momentum": self.momentum}

    @state_dict.setter
    def state_dict(self, new_state: dict):
        values = new_state["params"]
        if values:
            self.gain = _f64(values[0])
            self.variance = torch.ones_like(self.gain, dtype=torch.float64)
        if len(values) > 1:
            self.bias = _f64(values[1])
            self.mean = torch.zeros_like(self.bias, dtype=torch.float64)
        self.eps = new_state["eps"]
        self.momentum = new_state["momentum"]

    def checkpoint_state(self, ref) -> dict:
        return {"params": [ref(p) for p in self.params], "eps": self.eps, "momentum": self.momentum}

    def forward(self, input_tensor: Tensor) -> Tensor:
        sync = self.sync if self.training else None
        if _on_gpu(self.gain):
            y, rm, rv = _pf().batchnorm(input_tensor, self.gain, self.bias, self.mean, self.variance, self.eps,
                                        self.momentum, self.training, sync=sync)
            if self.training:
                self.mean, self.variance = rm, rv
            return y
        if sync is not None:  # global-batch statistics through a differentiable all-reduce
            from torch.distributed.nn.functional import all_reduce
            dims = tuple(range(input_tensor.ndim - 1))
            n = torch.tensor([float(input_tensor.numel() // input_tensor.shape[-1])], dtype=input_tensor.dtype)
            sums = all_reduce(torch.cat([input_tensor.sum(dims), (input_tensor * input_tensor).sum(dims), n]),
                              group=sync.group)
            c = input_tensor.shape[-1]
            total = sums[2 * c]
            keep = [1] * (input_tensor.ndim - 1) + [c]  # keepdim shape, as the reference's mean / var
            mean = (sums[:c] / total).view(keep)
            variance = ((sums[c:2 * c] - total * sums[:c] / total * sums[:c] / total) / (total - 1)).view(keep)
            with torch.no_grad():
                m = self.momentum
                self.mean = (1 - m) * self.mean + m * mean.detach()
                self.variance = (1 - m) * self.variance + m * variance.detach()
            return self.gain * (input_tensor - mean) / torch.sqrt(variance + self.eps) + self.bias
        if self.training:
            dims = tuple(range(input_tensor.ndim - 1))
            mean = input_tensor.mean(dims, keepdim=True)
            variance = input_tensor.var(dims, keepdim=True)
            with torch.no_grad():
                m = self.momentum
                self.mean = (1 - m) * self.mean + m * mean
                self.variance = (1 - m) * self.variance + m * variance
        else:
            mean, variance = self.mean, self.variance
        return self.gain * (input_tensor - mean) / torch.sqrt(variance + self.eps) + self.bias


class _Activation(Layer):
    def forward(self, pre_activation: Tensor) -> Tensor:
        if pre_activation.is_cuda:
            return _pf().activation(pre_activation, self.algo)
        return getattr(pre_activation, self.algo)()


class SigmoidLayer(_Activation):
    algo = "sigmoid"


class ReluLayer(_Activation):
    algo = "relu"
    weight_gain = math.sqrt(2.0)


class TanhLayer(_Activation):
    algo = "tanh"
    weight_gain = 5.0 / 3.0


class SoftmaxLayer(Layer):
    algo = "softmax"

    def forward(self, logits: Tensor) -> Tensor:
        if logits.is_cuda:
            return _pf().softmax(logits)
        return logits.softmax(dim=logits.ndim - 1)


LAYER_TYPES = {cls.algo: cls for cls in (EmbeddingLayer, FlattenLayer, LinearLayer, BatchNormLayer, SigmoidLayer,
                                         ReluLayer, TanhLayer, SoftmaxLayer)}
ACTIVATIONS = ("relu", "sigmoid", "softmax", "tanh")

__all__ = ["Layer", "EmbeddingLayer", "FlattenLayer", "LinearLayer", "BatchNormLayer", "SigmoidLayer", "ReluLayer",
           "TanhLayer", "SoftmaxLayer", "LAYER_TYPES", "ACTIVATIONS"]
