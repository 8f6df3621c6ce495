"""Host-side cost of one fused training step (python + launch), vs the GPU time of the step.

Runs the bench model, then (1) times N steps enqueued back to back with one sync at the end
(GPU-bound wall time) and (2) times the host enqueue alone by keeping the GPU busy-waiting
behind a long dummy kernel... approximated here by measuring enqueue time of each step with
`time.perf_counter` (launches are asynchronous) and printing a cProfile of the step.
"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer  # noqa: E402
from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel  # noqa: E402


def main():
    sizes = [int(s) for s in (sys.argv[1] if len(sys.argv) > 1 else "1024,4096,4096,1024").split(",")]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    algos = ["relu"] * (len(sizes) - 2) + ["softmax"]
    torch.manual_seed(0)
    model = NeuralNetworkModel("h", sizes, "xavier", "zeros", algos, "adam", dtype="bfloat16", device="cuda")
    tr = FusedTrainer(model)
    x = torch.randn(2 * batch, sizes[0])
    y = torch.randint(0, sizes[-1], (2 * batch,))
    tr.load_tensors(x, y, seed=1)
    n = 60
    tr.begin(n + 20, lr_schedule=lambda e: 1e-3)  # enables hipGraph replay (PZ_GRAPHS=0: eager)
    every = max(1, (n + 20) // 100)
    for e in range(10):
        tr.step(e, 1e-3, batch, 0.2, 1e-3, want_ratios=e % every == 0, record=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    enq = []
    for e in range(10, 10 + n):
        a = time.perf_counter()
        tr.step(e, 1e-3, batch, 0.2, 1e-3, want_ratios=e % every == 0, record=False)
        enq.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n
    print(f"sizes={sizes} batch={batch}: wall {wall * 1e3:.3f} ms/step, host enqueue median "
          f"{sorted(enq)[n // 2] * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for e in range(10 + n, 20 + n):
        tr.step(e, 1e-3, batch, 0.2, 1e-3, want_ratios=e % every == 0, record=False)
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
