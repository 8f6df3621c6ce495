"""Independent (numpy) re-implementations used as references by the kernel tests."""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def keep_mask(numel: int, seed_lo: int, seed_hi: int, lid: int, p: float) -> np.ndarray:
    """Dropout keep-mask of the pz kernels for logical element indices 0..numel-1."""
    thresh = min(65536, int(round(p * 65536)))
    idx = np.arange(numel, dtype=np.uint64)
    pair = idx >> np.uint64(1)
    h = _mix32(pair ^ np.uint64(seed_lo))
    k = (np.uint64(seed_hi) + np.uint64(0x9E3779B9) * np.uint64(lid + 1)) & M32
    bits = _mix32(h ^ k)
    r = np.where(idx & np.uint64(1), bits >> np.uint64(16), bits & np.uint64(0xFFFF))
    return r >= np.uint64(thresh)
