"""Training curves of two precision setups on the fused engine, same weights and minibatches.

Default: bf16 vs fp32 dense weight gradients (PZ_GRAD_DTYPE) on the headline
config. ``--fp8``: the fp8 policy vs bf16 on BASELINE config 5 ([1024,8192,1024] relu,softmax).

The headline config ([1024,4096,4096,1024] relu,relu,softmax, Adam, batch 8192, dropout 0.2,
L2 1e-3) trained for --steps steps on a LEARNABLE synthetic task (labels = argmax of a fixed random
linear map of the inputs, so the loss can fall well below ln 1024), once with PZ_GRAD_DTYPE=bf16
(the default) and once with fp32, from the same initial weights and the same minibatches. Each run is
a subprocess (the env knob is read at trainer construction); prints both cost curves and their gap.

    python tools/grad_dtype_convergence.py [--steps 300] [--lr 1e-3]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, torch
sys.path.insert(0, sys.argv[1])
from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
steps, lr, dtype = int(sys.argv[2]), float(sys.argv[3]), sys.argv[4]
sizes = [1024, 8192, 1024] if sys.argv[5] == "fp8cfg" else [1024, 4096, 4096, 1024]
g = torch.Generator().manual_seed(11)
n = 65536
x = torch.randn(n, sizes[0], generator=g)
proj = torch.randn(sizes[0], sizes[-1], generator=g)
y = (x @ proj).argmax(1)
torch.manual_seed(0)
algos = ["relu"] * (len(sizes) - 2) + ["softmax"]
m = NeuralNetworkModel("conv", sizes, "xavier", "zeros", algos, "adam", dtype=dtype, device="cuda")
tr = FusedTrainer(m)
tr.load_tensors(x, y, seed=5)
tr.begin(steps)
for e in range(steps):
    tr.step(e, lr, 8192, 0.2, 1e-3, want_ratios=False, record=False)
costs = [c for _, c, _, _ in tr.drain()]
print(json.dumps(costs))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--fp8", action="store_true", help="fp8 policy vs bf16 on [1024,8192,1024]")
    a = ap.parse_args()
    curves = {}
    runs = ((("bf16", "bfloat16", "bf16"), ("fp32", "bfloat16", "fp32")) if not a.fp8 else
            (("bf16", "bfloat16", "bf16"), ("fp32", "fp8", "bf16")))  # (curve key, model dtype, grad dtype)
    for key, mdt, gdt in runs:
        env = dict(os.environ, PZ_GRAD_DTYPE=gdt)
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(a.steps), str(a.lr), mdt,
                              "fp8cfg" if a.fp8 else "mlp4"], env=env, capture_output=True, text=True, timeout=900)
        if out.returncode != 0:
            print(out.stderr[-2000:], file=sys.stderr)
            raise SystemExit(out.returncode)
        curves[key] = json.loads(out.stdout.strip().splitlines()[-1])
    b, f = curves["bf16"], curves["fp32"]
    names = ("bf16", "fp8") if a.fp8 else ("bf16 grads", "fp32 grads")
    print(f"{'step':>6} {names[0]:>11} {names[1]:>11} {'gap':>8}")
    for i in list(range(0, len(b), max(1, len(b) // 15))) + [len(b) - 1]:
        print(f"{i:6d} {b[i]:11.4f} {f[i]:11.4f} {b[i] - f[i]:+8.4f}")
    tail = max(1, len(b) // 10)
    mb, mf = sum(b[-tail:]) / tail, sum(f[-tail:]) / tail
    print(f"mean cost over the last {tail} steps: {names[0]} {mb:.4f}, {names[1]} {mf:.4f} ({100 * (mf / mb - 1):+.2f}% "
          f"for the second)")


if __name__ == "__main__":
    main()
