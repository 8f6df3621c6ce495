"""The exact fast paths the benchmarks time, each against an independent reference (VERDICT r3
missing #2-#4).

* fp8 natural-layout weights (``_w8_nat``: every width a multiple of 256, as in BASELINE config 5
  ``[1024, 8192, 1024]``): the forward reads the ``[in, out]`` e4m3 copy through transposing 8-bit
  LDS reads (VAR 15), the dX GEMM the same copy K-contiguous, the first layer's fp8 dW GEMM the e5m2
  dZ the dX epilogue writes. Copies and scales are checked against torch casts, the loss curve
  against the bf16 run of the same batches.
* one bench-shape bf16 step (``[1024, 4096, 4096, 1024]``, batch 8192: 256x256 tiles, split-K,
  lean head, ReLU bitmask, bf16 gradients) against an fp32 torch step on the same picks.
* the reference's ``test_torch_backward.py`` scenario (embedding / flatten / linear / batchnorm /
  tanh / linear / softmax, fp64, batch = training_buffer_size) through the GPU autograd path
  against the CPU reference at rtol 1e-10.
* data parallel with an uneven split: 3 ranks, global sample 1000 (333 / 333 / 334 rows)
  equal to one rank on the concatenated batch.
"""
import math
import os
import random

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from neural_net_model import NeuralNetworkModel
from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer

pytestmark = pytest.mark.gpu


def _e4m3_ref(x: torch.Tensor, q: float) -> torch.Tensor:
    return (x.float() * q).clamp(-448.0, 448.0).to(torch.float8_e4m3fn)


def _close_fp8(got: torch.Tensor, ref: torch.Tensor) -> None:
    """Equal up to one rounding step of the 8-bit format on a vanishing fraction of elements
    (the kernels and torch may break exact ties differently)."""
    same = (got.view(torch.uint8) == ref.view(torch.uint8)).double().mean().item()
    assert same > 0.999, same
    g, r = got.float(), ref.float()
    assert torch.all((g - r).abs() <= r.abs() * 0.125 + 2 ** -9)


def test_fp8_natural_layout_engine_path():
    """BASELINE config 5 shape family at reduced size: [1024, 2048, 1024], batch 1024: the
    optimizer writes the e4m3 weight copies itself (delayed weight scaling)."""
    sizes = [1024, 2048, 1024]
    algos = ["relu", "softmax"]
    n, S, steps = 8192, 1024, 12
    g = torch.Generator().manual_seed(21)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    idx = torch.randint(0, n, (steps, S), generator=g)
    curves = {}
    for dtype in ("bfloat16", "fp8"):
        torch.manual_seed(0)
        model = NeuralNetworkModel("f8n", sizes, "xavier", "random", algos, "adam", dtype=dtype, device="cuda")
        tr = FusedTrainer(model)
        tr.load_tensors(inputs, labels, seed=9)
        tr.begin(steps)
        gqs_hist = []
        for e in range(steps):
            tr.step(e, 0.002, S, 0.1, 1e-4, want_ratios=False, record=False, indices=idx[e])
            if dtype == "fp8":
                gqs_hist.append(tr.gqs[0, 0].item())
        curves[dtype] = [c for _, c, _, _ in tr.drain()]
        if dtype != "fp8":
            continue
        # the natural-layout path really ran: one [in, out] e4m3 copy per weight, fp8 forward on
        # every stage, the dX GEMM of layer 2 on e5m2 x e4m3, the first
        # layer's dZ quantised by the dX epilogue and its dW GEMM on e4m3 x e5m2
        assert tr._w8_nat and not tr.w8_kc
        assert [st.fp8 for st in tr.stages] == [True, True]
        assert [st.fp8_bwd for st in tr.stages] == [False, True]
        assert tr.stages[0].g8_from_epi and 0 in tr._g8_epi_ready
        assert tr._fp8_dw_ready_cached(tr.stages[0])
        torch.cuda.synchronize()
        assert tr._w8_fused
        gemms = [st for st in tr.stages if st.kind == "gemm"]
        amax = torch.stack([tr.store.view(st.seg_w).abs().max() for st in gemms]).cpu()
        rows = tr.wamax2.cpu()  # the last update's amax slot holds max|w|, the other was cleared
        assert (rows == 0).all(dim=1).sum() == 1, rows
        assert torch.equal(rows.max(dim=0).values, amax), (rows, amax)
        for st in gemms:
            w = tr.store.view(st.seg_w)
            q = tr.wqs[st.w8_index, 0].item()
            # delayed scaling: q from the previous update's amax (a step of Adam moves max|w| by ~lr)
            assert math.isclose(q, 448.0 / w.abs().max().item(), rel_tol=0.05)
            assert math.isclose(tr.wqs[st.w8_index, 1].item(), 1.0 / q, rel_tol=1e-6)
            w8 = tr.w8[st.seg_w.offset]
            assert w8.shape == w.shape and w8 is tr.w8n[st.seg_w.offset]  # natural [in, out], one copy
            _close_fp8(w8, _e4m3_ref(w, q))
        # first-layer operand: the dataset quantised once at a static scale, gathered per step
        xq = tr.xqs[0].item()
        assert math.isclose(xq, 448.0 / inputs.to(torch.bfloat16).float().abs().max().item(), rel_tol=1e-6)
        _close_fp8(tr.data8, _e4m3_ref(tr.data, xq))
        picked = tr.picked[:S]
        assert torch.equal(tr.x8[:S].view(torch.uint8), tr.data8[picked].view(torch.uint8))
        # delayed e5m2 gradient scaling keeps moving after calibration
        assert all(math.isfinite(v) and v > 0 for v in gqs_hist)
        assert len(set(gqs_hist[2:])) > 1, gqs_hist
        assert gqs_hist[-1] != 1.0
        # the e5m2 dZ copy the first layer's dW GEMM read: dZ * q rounded to e5m2 (q = this step's)
        g8 = tr.stages[0].buffers["g8"][:S].float()
        assert torch.isfinite(g8).all() and g8.abs().max().item() > 1.0  # scaled into e5m2's range
    bf, f8 = curves["bfloat16"], curves["fp8"]
    assert all(math.isfinite(c) for c in f8)
    assert f8[-1] < f8[0] - 0.05, f8  # it learns
    # Adam's first steps move every weight by ~lr * sign(g): the gradient quantisation noise of
    # e5m2 dZ (2 mantissa bits) flips signs of small gradients and the early trajectories wander
    # apart by a few percent (in either direction); the SGD test below pins the gradients tightly
    for a, b in zip(bf, f8):
        assert abs(a - b) < 0.05 * abs(a) + 0.02, (bf, f8)


def test_fp8_natural_layout_gradients_and_sgd_curve():
    """The fp8 policy's gradients on the natural-layout path against the bf16 policy's, from the
    same weights and batches: per-layer weight-gradient relative error (one SGD step: delta =
    -lr * grad) within fp8 quantisation noise, and the SGD loss curve within 2 % + 0.01."""
    sizes = [1024, 2048, 1024]
    n, S, steps, lr = 8192, 1024, 12, 0.05
    g = torch.Generator().manual_seed(31)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    idx = torch.randint(0, n, (steps, S), generator=g)
    runs = {}
    for dtype in ("bfloat16", "fp8"):
        torch.manual_seed(0)
        model = NeuralNetworkModel("f8g", sizes, "xavier", "random", ["relu", "softmax"], "stochastic", dtype=dtype,
                                   device="cuda")
        tr = FusedTrainer(model)
        tr.load_tensors(inputs, labels, seed=9)
        tr.begin(steps)
        deltas = []
        for e in range(steps):
            before = [p.detach().float().clone() for p in model.params[0::2]]
            tr.step(e, lr, S, 0.0, 0.0, want_ratios=False, record=False, indices=idx[e])
            if e in (1, 2):  # step 0 calibrates the delayed scales on its own amax
                torch.cuda.synchronize()
                deltas.append([p.detach().float() - b for p, b in zip(model.params[0::2], before)])
        runs[dtype] = ([c for _, c, _, _ in tr.drain()], deltas)
        if dtype == "fp8":
            assert tr._w8_nat and [st.fp8 for st in tr.stages] == [True, True]
            assert tr._fp8_dw_ready_cached(tr.stages[0]) and tr._fp8_dw_ready_cached(tr.stages[1])
    (cb, db), (c8, d8) = runs["bfloat16"], runs["fp8"]
    # e4m3 forward, e5m2 x e4m3 dX, e4m3 x e5m2 dW. The first layer's dW = x^T dZ sums 1024 rows
    # of random inputs that carry no signal about the labels: the terms mostly cancel, so e5m2's
    # per-element rounding (2 mantissa bits) shows up amplified in the small sum (r4 GPU: 0.158);
    # the last layer's dW sums activations that do correlate with the head gradient
    bounds = (0.25, 0.08)
    rels = [[((a - b).norm() / a.norm()).item() for a, b in zip(step_b, step_8)] for step_b, step_8 in zip(db, d8)]
    for per_layer in rels:
        assert all(r < bd for r, bd in zip(per_layer, bounds)), rels
    assert c8[-1] < c8[0] - 0.05, c8
    for a, b in zip(cb, c8):
        assert abs(a - b) < 0.02 * abs(a) + 0.01, (cb, c8)


@pytest.mark.parametrize("optimizer", ["stochastic", "adam"])
def test_bench_shape_bf16_step_matches_fp32_torch(optimizer):
    """One step of the headline configuration (BASELINE config 2: [1024, 4096, 4096, 1024] relu,
    relu, softmax at batch 8192, dropout 0) on the fused engine — the shapes, tiles, split-K, lean
    head, ReLU bitmask and bf16 weight gradients the benchmark times — against an fp32 torch
    autograd step on the same picks, from the same fp32 master weights and the same bf16 inputs."""
    sizes = [1024, 4096, 4096, 1024]
    n, S, lr, l2 = 16384, 8192, 0.01, 1e-3
    torch.manual_seed(3)
    model = NeuralNetworkModel("mlp4", sizes, "xavier", "random", ["relu", "relu", "softmax"], optimizer,
                               dtype="bfloat16", device="cuda")
    g = torch.Generator().manual_seed(8)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    tr = FusedTrainer(model)
    tr.load_tensors(inputs, labels, seed=5)
    tr.begin(1)
    p0 = [p.detach().float().clone() for p in model.params]
    tr.step(0, lr, S, 0.0, l2, want_ratios=True, record=False)
    (_, cost, ratios, _), = tr.drain()
    picked = tr.picked[:S].clone()
    p1 = [p.detach().float().clone() for p in model.params]

    # independent fp32 reference (torch / hipBLASLt GEMMs, autograd)
    ref = [p.clone().requires_grad_() for p in p0]
    w1, b1, w2, b2, w3, b3 = ref
    x = tr.data[picked].float()  # the bf16 dataset rows the engine gathered
    y = labels.to(x.device)[picked]
    h = torch.relu(x @ w1 + b1)
    h = torch.relu(h @ w2 + b2)
    logits = h @ w3 + b3
    loss = F.cross_entropy(logits, y) + l2 * sum((w ** 2).sum() for w in (w1, w2, w3))
    loss.backward()
    assert abs(cost - loss.item()) < 2e-3 * abs(loss.item()), (cost, loss.item())
    # what bf16 storage alone costs: the same step in torch with bf16 weights, activations and
    # gradients (fp32-accumulating GEMMs, the engine's precision contract), l2 added in fp32.
    # The first layer's dW sums 8192 random input rows that carry no label signal, the terms
    # cancel and bf16 rounding of dZ shows amplified there (~3.7 %, any engine knob setting)
    emu = [p.to(torch.bfloat16).requires_grad_() for p in p0]
    e1, c1, e2, c2, e3, c3 = emu
    he = torch.relu(x.to(torch.bfloat16) @ e1 + c1)
    he = torch.relu(he @ e2 + c2)
    F.cross_entropy((he @ e3 + c3).float(), y).backward()
    g_emu = [e.grad.float() + (2 * l2 * p if i % 2 == 0 else 0) for i, (e, p) in enumerate(zip(emu, p0))]
    for i, (a, b, r) in enumerate(zip(p0, p1, ref)):
        gref = r.grad
        if optimizer == "stochastic":  # delta = -lr * grad: the gradient itself, relative error
            d_gpu, d_ref = b - a, -lr * gref
            rel = ((d_gpu - d_ref).norm() / d_ref.norm()).item()
            rel_emu = ((g_emu[i] - gref).norm() / gref.norm()).item()
            # no worse than bf16 storage itself by more than a quarter (+ slack for small tensors)
            assert rel < 1.25 * rel_emu + 5e-3, (i, rel, rel_emu)
        else:  # Adam's first step is lr * g / (|g| + eps): a sign test where the gradient is clear
            clear = gref.abs() > 0.1 * gref.pow(2).mean().sqrt()
            step = (a - b)[clear]
            agree = (torch.sign(step) == torch.sign(gref[clear])).double().mean().item()
            assert agree > 0.995, (i, agree)
            assert ((step.abs() - lr).abs() < 0.05 * lr).double().mean().item() > 0.95
    # update ratios std(dW) / (std(W) + 1e-8) against the reference's definition
    ws = [(a, b) for i, (a, b) in enumerate(zip(p0, p1)) if i % 2 == 0]
    want = [((b - a).std() / (b.std() + 1e-8)).item() for a, b in ws]
    assert len(ratios) == len(want)
    for r, w in zip(ratios, want):
        assert abs(r - w) < 1e-2 * w, (ratios, want)


def test_torch_backward_scenario_on_gpu_fp64():
    """The reference's manual-backprop scenario (reference test_torch_backward.py:14-119) on a
    ``device="cuda"`` fp64 model: the GPU autograd path (ops/functional.py _Linear / _Stage /
    batchnorm / embedding Functions) against the CPU fp64 reference — every activation, every
    activation gradient and every parameter gradient at rtol 1e-10."""
    block, emb, hidden, vocab = 3, 10, 64, 27
    sizes = [vocab, emb, emb * block, hidden, vocab]
    algos = ["embedding", "linear", "batchnorm", "tanh", "linear", "softmax"]
    torch.manual_seed(0)
    cpu = NeuralNetworkModel("tb_cpu", sizes, "xavier", "random", algos, None)
    torch.manual_seed(0)
    gpu = NeuralNetworkModel("tb_gpu", sizes, "xavier", "random", algos, None, device="cuda")
    assert gpu.on_gpu and gpu.precision.master == torch.float64
    batch = cpu.training_buffer_size
    g = torch.Generator().manual_seed(1)
    sample = torch.randint(0, vocab, (batch, block), generator=g)
    rnd = random.Random(2)
    target = [[rnd.randint(0, vocab - 1)] for _ in range(batch)]
    grads = {}
    for name, m in (("cpu", cpu), ("gpu", gpu)):
        for p in m.params:
            p.requires_grad_()
            p.grad = None
        acts, cost = m._forward(sample, target)
        for a in acts:
            a.retain_grad()
        cost.backward()
        grads[name] = (cost.detach().cpu(), [a.detach().cpu() for a in acts],
                       [a.grad.cpu() if a.grad is not None else None for a in acts],  # (probs: not in the loss)
                       [p.grad.detach().cpu() for p in m.params])
        for p in m.params:
            p.requires_grad_(False)
    (c0, a0, ag0, pg0), (c1, a1, ag1, pg1) = grads["cpu"], grads["gpu"]
    assert a1[0].dtype == torch.float64 and pg1[0].dtype == torch.float64
    torch.testing.assert_close(c1, c0, rtol=1e-12, atol=0)
    for i, (x, y) in enumerate(zip(a0, a1)):
        torch.testing.assert_close(y, x, rtol=1e-10, atol=1e-13, msg=f"activation {i}")
    assert [g is None for g in ag0] == [g is None for g in ag1]
    assert sum(g is not None for g in ag0) == len(ag0) - 1  # every activation but the softmax output
    for i, (x, y) in enumerate(zip(ag0, ag1)):
        if x is not None:
            torch.testing.assert_close(y, x, rtol=1e-10, atol=1e-15, msg=f"activation grad {i}")
    names = ["c", "w1", "b1", "bn_gain", "bn_bias", "w2", "b2"]
    for nm, x, y in zip(names, pg0, pg1):
        torch.testing.assert_close(y, x, rtol=1e-10, atol=1e-15, msg=nm)


# --------------------------------------------------------------------------------------------
# uneven data-parallel shards (reference neural_net_model.py:441, 460: sample_size rows drawn)
SIZES3 = [128, 256, 256, 64]
N3, S3, WORLD3 = 2048, 1000, 3


def _data3():
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N3, SIZES3[0], generator=g)
    y = torch.randint(0, SIZES3[-1], (N3,), generator=g)
    idx = torch.randint(0, N3, (S3,), generator=g)
    return x, y, idx


def _model3(optimizer, dtype="float32"):
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel as M
    torch.manual_seed(0)
    return M("dp3", SIZES3, "xavier", "random", ["relu", "tanh", "softmax"], optimizer, dtype=dtype,
             device="cuda:0")


def _rank3(rank, world, store, optimizer, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), PZ_GRAD_COMM_DTYPE="fp32")
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    model = _model3(optimizer)
    tr = FusedTrainer(model, DataParallelContext(rank, world))
    x, y, idx = _data3()
    tr.load_tensors(x, y, seed=3)
    tr.begin(2)
    lo, hi = rank * S3 // world, (rank + 1) * S3 // world  # the trainer's own split
    for e in range(2):
        tr.step(e, 0.01, S3, 0.0, 1e-3, want_ratios=True, record=False, indices=idx[lo:hi])
    out = tr.drain()
    torch.save({"flat": model._param_store.flat.cpu(), "costs": [c for _, c, _, _ in out],
                "ratios": [r for _, _, r, _ in out], "rows": hi - lo}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("optimizer", ["stochastic", "adam"])
def test_uneven_three_rank_step_equals_single_rank(tmp_path, monkeypatch, optimizer):
    """3 ranks, global sample 1000: shards of 333, 333 and 334 rows, each rank's loss and
    gradients scaled by 1/1000 so the all-reduced sum is the global mean — equal to one rank
    stepping on the 1000 concatenated rows."""
    out = str(tmp_path / "dp3.pt")
    mp.start_processes(_rank3, args=(WORLD3, str(tmp_path / "rdv"), optimizer, out), nprocs=WORLD3,
                       start_method="spawn")
    ranks = [torch.load(out + f".{r}", weights_only=True) for r in range(WORLD3)]
    assert [r["rows"] for r in ranks] == [333, 333, 334]
    monkeypatch.setenv("PZ_GRAD_DTYPE", "fp32")
    model = _model3(optimizer)
    tr = FusedTrainer(model)
    x, y, idx = _data3()
    tr.load_tensors(x, y, seed=3)
    tr.begin(2)
    for e in range(2):
        tr.step(e, 0.01, S3, 0.0, 1e-3, want_ratios=True, record=False, indices=idx)
    out1 = tr.drain()
    costs = [c for _, c, _, _ in out1]
    dp = ranks[0]
    for a, b in zip(dp["costs"], costs):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b)), (dp["costs"], costs)
    d = (dp["flat"] - model._param_store.flat.cpu()).abs()
    if optimizer == "adam":
        assert (d > 1e-3).double().mean().item() < 1e-3 and d.mean().item() < 1e-5
    else:
        assert d.max().item() < 1e-6, d.max().item()
    for a, b in zip(dp["ratios"], [r for _, _, r, _ in out1]):
        assert all(abs(u - v) < 1e-3 * abs(v) + 1e-7 for u, v in zip(a, b)), (a, b)
    for r in ranks:
        assert torch.equal(r["flat"], dp["flat"])


# --------------------------------------------------------------------------------------------
# fp8 policy under data parallelism: the first layer's dW GEMM runs in row
# chunks (its all-reduce travels chunk by chunk); once the dX epilogue writes only the e5m2 dZ
# (store_c=False) every chunk must read that copy, never the unwritten bf16 dZ
SIZES8 = [1024, 2048, 1024]
N8, B8, STEPS8 = 4096, 512, 4


def _data8(world):
    g = torch.Generator().manual_seed(23)
    x = torch.randn(N8, SIZES8[0], generator=g)
    y = torch.randint(0, SIZES8[-1], (N8,), generator=g)
    idx = torch.randint(0, N8, (STEPS8, world * B8), generator=g)
    return x, y, idx


def _model8():
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel as M
    torch.manual_seed(0)
    return M("dp8", SIZES8, "xavier", "random", ["relu", "softmax"], "stochastic", dtype="fp8", device="cuda:0")


def _rank8(rank, world, store, out_path):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method=f"file://{store}", rank=rank, world_size=world)
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    model = _model8()
    tr = FusedTrainer(model, DataParallelContext(rank, world))
    x, y, idx = _data8(world)
    tr.load_tensors(x, y, seed=3)
    tr.begin(STEPS8)
    for e in range(STEPS8):
        tr.step(e, 0.05, world * B8, 0.0, 0.0, want_ratios=False, record=False,
                indices=idx[e, rank * B8:(rank + 1) * B8])
    costs = [c for _, c, _, _ in tr.drain()]
    st0 = tr.stages[0]
    info = {"fp8_dw": tr._fp8_dw_ready_cached(st0),
            "calibrated": 0 in tr._g8_epi_ready}
    torch.save({"flat": model._param_store.flat.cpu(), "costs": costs, "info": info}, out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_fp8_data_parallel_dw_matches_single_rank(tmp_path):
    world = 2
    out = str(tmp_path / "dp8.pt")
    mp.start_processes(_rank8, args=(world, str(tmp_path / "rdv"), out), nprocs=world, start_method="spawn")
    ranks = [torch.load(out + f".{r}", weights_only=True) for r in range(world)]
    info = ranks[0]["info"]
    assert info == {"fp8_dw": True, "calibrated": True}, info
    model = _model8()
    w0 = model.params[0].detach().float().cpu().clone()
    tr = FusedTrainer(model)
    x, y, idx = _data8(world)
    tr.load_tensors(x, y, seed=3)
    tr.begin(STEPS8)
    for e in range(STEPS8):
        tr.step(e, 0.05, world * B8, 0.0, 0.0, want_ratios=False, record=False, indices=idx[e])
    costs = [c for _, c, _, _ in tr.drain()]
    # fp8 delayed scales are per rank (local amax), so the two runs differ at fp8 rounding level,
    # not bit for bit; an unwritten dZ would wreck the first layer's update outright
    for a, b in zip(ranks[0]["costs"], costs):
        assert abs(a - b) < 0.02 * abs(b) + 0.01, (ranks[0]["costs"], costs)
    n0 = model.params[0].numel()
    d_dp = ranks[0]["flat"][:n0].reshape(w0.shape) - w0
    d_1 = model.params[0].detach().float().cpu() - w0
    rel = ((d_dp - d_1).norm() / d_1.norm()).item()
    assert rel < 0.15, rel
    for r in ranks:
        assert torch.equal(r["flat"], ranks[0]["flat"])


@pytest.mark.parametrize("optimizer", ["adam", None])
def test_gpu_autograd_fallback_updates_through_fused_optimizer(optimizer):
    """A GPU model trained on the autograd path (models/network.py _autograd_epochs: the runtime of
    layer stacks the fused engine does not compile) takes its update from the fused optimizer kernel
    (csrc/optim.hip) over the flat parameter / gradient buffers: same trajectory as the reference's
    CPU fp64 torch.optim.Adam / SGD loop on the same picks, and a torch.optim.Adam state_dict whose
    moments and step counters match."""
    sizes, algos = [16, 32, 8], ["relu", "softmax"]
    g = torch.Generator().manual_seed(3)
    data = [(torch.randn(16, generator=g).tolist(), [int(torch.randint(0, 8, (1,), generator=g))]) for _ in range(64)]
    models = {}
    for dev in ("cpu", "cuda"):
        torch.manual_seed(0)
        m = NeuralNetworkModel(f"fb_{dev}", sizes, "xavier", "random", algos, optimizer, device=dev)
        torch.manual_seed(7)  # the reference's global-RNG picks
        m._train_autograd(data, epochs=5, learning_rate=0.01, sample_size=16, decay_rate=0.9, dropout_rate=0.0,
                          l2_lambda=0.001)
        models[dev] = m
    cpu, gpu = models["cpu"], models["cuda"]
    for pc, pg in zip(cpu.params, gpu.params):
        torch.testing.assert_close(pg.detach().cpu(), pc.detach(), rtol=1e-9, atol=1e-12)
    if optimizer is not None:
        sc, sg = cpu.optimizer.state_dict()["state"], gpu.optimizer.state_dict()["state"]
        for k in sc:
            assert float(sg[k]["step"]) == float(sc[k]["step"]) == 5
            torch.testing.assert_close(sg[k]["exp_avg"].cpu(), sc[k]["exp_avg"], rtol=1e-9, atol=1e-14)
            torch.testing.assert_close(sg[k]["exp_avg_sq"].cpu(), sc[k]["exp_avg_sq"], rtol=1e-9, atol=1e-16)
