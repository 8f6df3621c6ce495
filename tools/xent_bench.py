"""Micro-benchmark of the softmax-cross-entropy head (bench shape: 8192 x 1024 bf16 logits).

Variants: full (loss + dH + logit dropout + bias-gradient column sum), without the column sum,
without dropout. Interleaved rounds, best of 5, one process.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penr_oz_neural_network_torch_amd.ops import functional as PF, native  # noqa: E402


def timeit(fn, n=50, w=5):
    for _ in range(w):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    native.require()
    rows, cols = (int(v) for v in (sys.argv[1:3] if len(sys.argv) > 2 else (8192, 1024)))
    dev = "cuda"
    logits = torch.randn(rows, cols, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, cols, (rows,), device=dev)
    loss = torch.zeros(64, device=dev)  # the trainer spreads block adds over 64 slots
    dh = torch.empty_like(logits)
    colsum = torch.zeros(cols, device=dev)
    drop = PF.epi_spec(drop_pre=4, p=0.2, seed=(3, 4))
    ops = torch.ops.pz
    variants = {
        "full": lambda: ops.xent_head(logits, labels, rows, loss, 1.0 / rows, dh, 1.0 / rows, colsum, None, *drop, 0),
        "no_colsum": lambda: ops.xent_head(logits, labels, rows, loss, 1.0 / rows, dh, 1.0 / rows, None, None, *drop, 0),
        "no_dropout": lambda: ops.xent_head(logits, labels, rows, loss, 1.0 / rows, dh, 1.0 / rows, colsum, None,
                                            *PF.NO_EPI, 0),
    }
    best = {k: float("inf") for k in variants}
    for _ in range(5):
        for k, fn in variants.items():
            best[k] = min(best[k], timeit(fn))
    gb = 2 * rows * cols * 2 / 1e9
    for k, us in best.items():
        print(f"xent {rows}x{cols} {k:>10}: {us:7.2f} us  ({gb / (us * 1e-6):.0f} GB/s of logits+dH)")


if __name__ == "__main__":
    main()
