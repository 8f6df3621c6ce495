"""Isolated time of the softmax-cross-entropy head (pz::xent_head, bf16 fast path) on the headline
step's shape: logits [8192, 1024], loss + dZ + logit-dropout backward, with / without the
bias-gradient column sums (which every block adds into the same 1024 addresses).

    python tools/head_bench.py [--rows 8192] [--cols 1024] [--iters 200]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from penr_oz_neural_network_torch_amd.ops import functional as PF  # noqa: E402
from penr_oz_neural_network_torch_amd.ops import native  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--cols", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    native.require()
    R, C = args.rows, args.cols
    dev = "cuda"
    logits = torch.randn(R, C, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, C, (R,), device=dev)
    loss = torch.zeros(8, device=dev)
    dh = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
    colsum = torch.zeros(C, device=dev)
    epi_i, epi_f = PF.epi_spec(drop_pre=4, p=0.2, seed=(1, 2), epoch=0)
    no_i, no_f = PF.epi_spec()
    out = {}
    for name, cs, ei, ef in (("colsum", colsum, epi_i, epi_f), ("no_colsum", None, epi_i, epi_f),
                             ("no_colsum_no_dropout", None, no_i, no_f), ("copy_floor", None, None, None)):
        def run():
            if ei is None:  # the same bytes through a plain device copy (read 16 MB, write 16 MB)
                dh.copy_(logits)
                return
            torch.ops.pz.xent_head(logits, labels, R, loss, 1.0 / R, dh, 1.0 / R, cs, None, ei, ef, C)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / args.iters, 2)
    print(json.dumps({"rows": R, "cols": C, **out}))


if __name__ == "__main__":
    main()
