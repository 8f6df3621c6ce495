"""Isolated bandwidth of the fused optimizer launch (pz::optimizer_step) on the headline model.

Times the whole-model Adam / SGD update of the mlp4 bf16 policy (fp32 master, bf16 gradients,
bf16 shadow refresh) on its own, and reports the effective HBM rate from the bytes one update
moves per parameter. usage: python tools/opt_bw.py [--sizes 1024,4096,4096,1024] [--iters 50]
(profiles/r3_opt_preload.txt: the load-grouping A/B this measured.)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer  # noqa: E402
from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1024,4096,4096,1024")
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    sizes = [int(s) for s in args.sizes.split(",")]
    algos = ["relu"] * (len(sizes) - 2) + ["softmax"]
    model = NeuralNetworkModel("optbw", sizes, activation_algos=algos, optimizer_algo=args.optimizer,
                               dtype="bfloat16", device="cuda:0")
    tr = FusedTrainer(model)
    n = sum(p.numel() for p in model.params)
    grads = tr.grads
    grads.normal_()
    opt = tr.opt
    opt.stats_every = 0
    for _ in range(5):
        opt.step(grads, 1e-4, 1e-3, 1.0, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        opt.step(grads, 1e-4, 1e-3, 1.0, 0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / args.iters
    gb = 2 if grads.dtype == torch.bfloat16 else 4
    per = (4 + gb + 4 + 4) + (4 + 4 + 4 + 2) if opt.adam else (4 + gb) + (4 + 2)
    print(json.dumps({"params": n, "us_per_update": round(us, 2), "bytes_per_param": per,
                      "TB_per_s": round(n * per / us / 1e6, 3), "grad_dtype": str(grads.dtype)}))


if __name__ == "__main__":
    main()
