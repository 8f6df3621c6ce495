"""Independent (numpy) re-implementations used as references by the kernel tests."""
import numpy as np

from penr_oz_neural_network_torch_amd.ops.functional import epoch_key, layer_key

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def keep_mask(numel: int, seed_lo: int, seed_hi: int, lid: int, p: float, epoch: int | None = None) -> np.ndarray:
    """Dropout keep-mask of the pz kernels for logical element indices 0..numel-1 (``epoch``: the
    per-epoch key of a training step, as the fused trainer derives it)."""
    thresh = min(65536, int(round(p * 65536)))
    key = layer_key((seed_lo, seed_hi), lid)
    if epoch is not None:
        key = epoch_key(key, epoch)
    key = np.uint64(key)
    idx = np.arange(numel, dtype=np.uint64)
    bits = _mix32((idx >> np.uint64(1)) ^ key)
    r = np.where(idx & np.uint64(1), bits >> np.uint64(16), bits & np.uint64(0xFFFF))
    return r >= np.uint64(thresh)
