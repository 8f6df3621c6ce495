"""Error bound of the bf16 gradient buckets under a RING-ORDER reduction.

Data parallelism on bf16 models (``engine/trainer.py``): every rank's dW GEMM writes its dense
weight gradient in bf16 and RCCL sums the bucket in bf16. RCCL's ring all-reduce is a
reduce-scatter (chunk c starts at rank c+1 and travels the ring once; every hop adds the local
chunk to the incoming partial sum and the result is ROUNDED TO BF16 before it is sent on) followed
by an all-gather (exact copies). gloo's CPU sum — which the multi-rank CPU tests use — rounds
differently, so this file reduces in ring order explicitly, with a per-hop bf16 rounding (the
worst case: RCCL may keep wider partials inside one kernel, never narrower).

Bound (recursive summation, unit roundoff u = 2^-8: bf16 carries 8 significant bits): the reduced
element s_hat of the W rank gradients g_r (already rounded to bf16 once each) satisfies

    |s_hat - sum_r g_r| <= gamma_W * sum_r |g_r|,    gamma_W = W u / (1 - W u)

(W - 1 partial-sum roundings plus the rounding of each input). At W = 8 that is 3.2 % of the
absolute gradient mass of an element; relative to the L2 norm of the whole gradient the
measured error is several times smaller (independent rounding errors do not add coherently).
What it does to training is pinned below on a real MLP: one ring-reduced bf16 step vs the exact
fp64 step, against the tolerances ``tests/test_dp_gpu.py`` applies to the GPU runs.
"""
import math

import pytest
import torch

U_BF16 = 2.0 ** -8


def _bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16).to(torch.float64)


def ring_all_reduce_bf16(grads: list[torch.Tensor]) -> torch.Tensor:
    """Sum of the ranks' bf16 gradients in RCCL's ring order: the flat buffer is cut into W
    chunks; chunk c is reduced starting at rank (c + 1) % W around the ring, every partial sum
    rounded to bf16 when it leaves a rank; the all-gather copies the finished chunks."""
    world = len(grads)
    flat = [_bf16(g.reshape(-1).to(torch.float64)) for g in grads]
    n = flat[0].numel()
    bounds = [n * c // world for c in range(world + 1)]
    out = torch.empty(n, dtype=torch.float64)
    for c in range(world):
        lo, hi = bounds[c], bounds[c + 1]
        start = (c + 1) % world
        acc = flat[start][lo:hi].clone()
        for k in range(1, world):
            r = (start + k) % world
            acc = _bf16(acc + flat[r][lo:hi])  # the hop's bf16 partial sum
        out[lo:hi] = acc
    return out.view_as(grads[0])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ring_bf16_sum_within_recursive_summation_bound(world):
    g = torch.Generator().manual_seed(world)
    # gradient-like data: heavy-tailed magnitudes, mixed signs, a shared component across ranks
    common = torch.randn(4096, generator=g, dtype=torch.float64)
    grads = [(common + 0.5 * torch.randn(4096, generator=g, dtype=torch.float64))
             * torch.exp(torch.randn(4096, generator=g, dtype=torch.float64)) for _ in range(world)]
    exact = sum(grads)
    got = ring_all_reduce_bf16(grads)
    gamma = world * U_BF16 / (1 - world * U_BF16)
    mass = sum(g_.abs() for g_ in grads)
    err = (got - exact).abs()
    assert bool((err <= gamma * mass + 1e-300).all()), float((err / mass).max())
    rel_norm = float((got - exact).norm() / exact.norm())
    assert rel_norm < gamma / 2, (rel_norm, gamma)  # incoherent rounding errors: inside the bound


def _mlp(seed: int):
    from neural_net_model import NeuralNetworkModel
    torch.manual_seed(seed)
    return NeuralNetworkModel("ring", [64, 256, 256, 16], "he", "random", ["relu", "relu", "softmax"], "stochastic")


@pytest.mark.parametrize("world", [2, 8])
def test_ring_bf16_buckets_one_training_step(world):
    """One SGD step of a real MLP with data-parallel bf16 buckets reduced in ring order vs the
    exact fp64 step on the whole batch: the weight update differs by no more than the bf16
    tolerances the GPU equivalence tests use (tests/test_dp_gpu.py TOL, SGD max |dp| 2e-4 at
    lr 0.05), and the next step's cost by < 1e-4 relative."""
    torch.manual_seed(0)
    batch = 256
    x = torch.randn(batch, 64, dtype=torch.float64)
    y = torch.randint(0, 16, (batch,))
    lr = 0.05
    # exact: one process, whole batch
    ref = _mlp(1)
    _, cost = ref._forward(x, [[int(v)] for v in y], 0.0)
    for p in ref.params:
        p.requires_grad_()
    _, cost = ref._forward(x, [[int(v)] for v in y], 0.0)
    cost.backward()
    exact_grads = [p.grad.detach().clone() for p in ref.params]
    # data parallel: rank r's shard-mean gradient weighted by its share (what each rank's dW GEMM
    # produces after the 1/world folding), ring-reduced in bf16
    shard_grads = [[] for _ in ref.params]
    for r in range(world):
        lo, hi = r * batch // world, (r + 1) * batch // world
        m = _mlp(1)
        for p in m.params:
            p.requires_grad_()
        _, c = m._forward(x[lo:hi], [[int(v)] for v in y[lo:hi]], 0.0)
        (c * ((hi - lo) / batch)).backward()
        for i, p in enumerate(m.params):
            shard_grads[i].append(p.grad.detach().clone())
    ring = [ring_all_reduce_bf16(gs) for gs in shard_grads]
    for i, (gr, ge) in enumerate(zip(ring, exact_grads)):
        gamma = world * U_BF16 / (1 - world * U_BF16)
        mass = sum(s.abs() for s in shard_grads[i])
        assert bool(((gr - ge).abs() <= gamma * mass + 1e-15).all())
    # the SGD update each way
    d_ring = [lr * g for g in ring]
    d_exact = [lr * g for g in exact_grads]
    worst = max(float((a - b).abs().max()) for a, b in zip(d_ring, d_exact))
    assert worst < 2e-4, worst
    # cost after the step
    def cost_after(deltas):
        m = _mlp(1)
        with torch.no_grad():
            for p, d in zip(m.params, deltas):
                p -= d
        _, c = m._forward(x, [[int(v)] for v in y], 0.0)
        return float(c)
    c_ring, c_exact = cost_after(d_ring), cost_after(d_exact)
    assert abs(c_ring - c_exact) / abs(c_exact) < 1e-4, (c_ring, c_exact)
    assert math.isfinite(c_ring)
