"""penr-oz MLP training framework, MI355X-native.

Same capabilities as ``derinworks/penr-oz-neural-network-torch`` (REST microservice that
creates / trains / serves / persists / visualises multi-layer perceptrons), rebuilt around:

* hand-written CDNA4 (gfx950) HIP kernels for every hot op (``csrc/``, loaded as the
  ``torch.ops.pz`` library by :mod:`.ops`),
* a device-resident fused trainer (:mod:`.engine`) that schedules forward/backward/optimizer
  explicitly on HIP streams (no autograd graph, no per-step host syncs),
* data parallelism over RCCL/xGMI with ``torch.distributed`` (:mod:`.parallel`),
* a reference-compatible model facade (:mod:`.models`) and checkpoint format (:mod:`.utils`).
"""
from .config import Precision, resolve_device, resolve_precision  # noqa: F401

__version__ = "0.1.0"
