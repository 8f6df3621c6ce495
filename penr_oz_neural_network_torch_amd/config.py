"""Device / precision policy.

The reference runs everything on CPU in float64 (``neural_net_model.py:43,45,65,104`` of the
reference). Models created without ``device``/``dtype`` keep exactly that behaviour so the
reference test-suite passes unchanged. GPU models pick a *precision policy*:

============  ==================  =====================  ===========================
dtype         master params        GEMM operands          accumulation
============  ==================  =====================  ===========================
float64       fp64                 fp64 (f64 MFMA)        fp64
float32       fp32                 fp32 (f32 MFMA)        fp32
bfloat16      fp32                 bf16 shadows           fp32 (bf16 MFMA)
fp8           fp32                 e4m3 fwd, e5m2 x e4m3  fp32 (fp8 MFMA)
                                   dX, bf16 dW
============  ==================  =====================  ===========================

Master parameters are what ``params`` exposes and what the JSON checkpoint stores.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch

_ALIASES = {
    "float64": "float64", "fp64": "float64", "double": "float64",
    "float32": "float32", "fp32": "float32", "float": "float32",
    "bfloat16": "bfloat16", "bf16": "bfloat16",
    "fp8": "fp8", "float8": "fp8", "float8_e4m3fn": "fp8", "e4m3": "fp8",
}


@dataclass(frozen=True)
class Precision:
    name: str               # canonical policy name
    master: torch.dtype     # dtype of the parameters the user sees / checkpoints
    compute: torch.dtype    # dtype of GEMM operands / stored activations

    @property
    def mixed(self) -> bool:
        return self.master != self.compute


def resolve_precision(dtype) -> Precision:
    if isinstance(dtype, Precision):
        return dtype
    if isinstance(dtype, torch.dtype):
        dtype = str(dtype).replace("torch.", "")
    name = _ALIASES.get(str(dtype or "float64").lower())
    if name is None:
        raise ValueError(f"Unsupported dtype: {dtype}")
    if name == "float64":
        return Precision(name, torch.float64, torch.float64)
    if name == "float32":
        return Precision(name, torch.float32, torch.float32)
    if name == "bfloat16":
        return Precision(name, torch.float32, torch.bfloat16)
    return Precision(name, torch.float32, torch.float8_e4m3fn)


def resolve_device(device) -> torch.device:
    if device is None:
        device = os.environ.get("PZ_DEVICE", "cpu")
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        dev = torch.device("cuda", local)
    return dev
