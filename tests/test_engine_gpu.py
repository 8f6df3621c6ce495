"""Fused trainer (GPU) vs the reference algorithm on the CPU, one step at a time."""
import math

import pytest
import torch

from neural_net_model import NeuralNetworkModel
from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer

pytestmark = pytest.mark.gpu


def _pair(sizes, algos, optimizer, dtype, seed=0, bias_algo="random"):
    torch.manual_seed(seed)
    gpu = NeuralNetworkModel("g", sizes, "xavier", bias_algo, algos, optimizer, dtype=dtype, device="cuda")
    torch.manual_seed(seed)
    cpu = NeuralNetworkModel("c", sizes, "xavier", bias_algo, algos, optimizer)
    for pg, pc in zip(gpu.params, cpu.params):
        assert torch.equal(pg.double().cpu(), pc.float().double()) or torch.allclose(pg.double().cpu(), pc, atol=1e-7)
    return gpu, cpu


def _cpu_step(cpu, x, target, lr, l2):
    for p in cpu.params:
        p.requires_grad_()
    if cpu.optimizer is not None:
        for g in cpu.optimizer.param_groups:
            g["lr"] = lr
    acts, cost = cpu._forward(x, target, 0.0)
    cost = cost + l2 * sum((w ** 2).sum() for w in cpu.weights)
    for p in cpu.params:
        p.grad = None
    cost.backward()
    if cpu.optimizer is not None:
        cpu.optimizer.step()
    else:
        for p in cpu.params:
            p.data -= lr * p.grad
    return cost.item()


@pytest.mark.parametrize("optimizer", ["adam", "stochastic"])
@pytest.mark.parametrize("dtype,tol", [("float32", 2e-4), ("bfloat16", 3e-2)])
def test_dense_step_matches_reference(optimizer, dtype, tol):
    sizes = [256, 512, 256, 128]
    algos = ["relu", "tanh", "softmax"]
    gpu, cpu = _pair(sizes, algos, optimizer, dtype)
    n, S = 3000, 1024
    g = torch.Generator().manual_seed(1)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    data = [(inputs[i].tolist(), [int(labels[i])]) for i in range(n)]
    tr = FusedTrainer(gpu)
    tr.load_data(data)
    tr.begin(1)
    lr, l2 = 0.01, 0.001
    tr.step(0, lr, S, 0.0, l2, want_ratios=True, record=False)
    (epoch, cost, ratios, _), = tr.drain()
    picked = tr.picked[:S].cpu()
    x = inputs[picked].double()
    target = [[int(labels[i])] for i in picked]
    prev = [w.clone().detach() for w in cpu.weights]
    cpu_cost = _cpu_step(cpu, x, target, lr, l2)
    assert abs(cost - cpu_cost) < tol * max(1.0, abs(cpu_cost)), (cost, cpu_cost)
    for pg, pc in zip(gpu.params, cpu.params):
        d = (pg.detach().double().cpu() - pc.detach()).abs()
        if optimizer == "adam":
            # Adam's first step is ~lr * sign(g): elements whose gradient is at rounding-noise
            # level may flip sign, so compare in distribution (the optimizer itself is checked
            # bit-for-bit against torch.optim.Adam in test_kernels_gpu.py)
            bad = (d > 0.1 * lr).double().mean().item()
            assert bad < (0.002 if dtype == "float32" else 0.05), bad
            assert d.mean().item() < (1e-3 if dtype == "float32" else 1e-2) * lr * 10
        else:
            scale = pc.detach().abs().max().item()
            assert d.max().item() < tol * max(scale, 1e-3) + (1e-3 if dtype == "bfloat16" else 1e-6), d.max()
    ref_ratios = [((w - pw).std() / (w.std() + 1e-8)).item() for pw, w in zip(prev, cpu.weights)]
    for a, b in zip(ratios, ref_ratios):
        assert abs(a - b) < 0.05 * b + 1e-6 if dtype == "bfloat16" else abs(a - b) < 1e-3 * b + 1e-7


@pytest.mark.parametrize("optimizer", ["stochastic", "adam"])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_dropout_step_matches_fp64_reimplementation(optimizer, dtype):
    """Dropout semantics at the step level: one fused step at
    dropout_rate 0.3 vs an fp64 torch re-implementation of the reference epoch that applies the
    kernels' keep masks to EVERY hidden layer output (reference neural_net_model.py:393-395) —
    the ReLU output, the pre-tanh linear output, the tanh output and the logits that feed the
    softmax / cross-entropy head (:400-403) — each kept element scaled by 1/(1-p)."""
    from tests.helpers import keep_mask
    sizes = [128, 256, 192, 64]
    algos = ["relu", "tanh", "softmax"]  # -> linear relu linear tanh linear softmax
    gpu, cpu = _pair(sizes, algos, optimizer, dtype)
    assert cpu.algos == ["linear", "relu", "linear", "tanh", "linear", "softmax"]
    hidden = [i for i, layer in enumerate(cpu.layers) if layer.hidden]
    assert hidden == [1, 2, 3, 4]
    n, S, p = 2000, 512, 0.3
    g = torch.Generator().manual_seed(5)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    tr = FusedTrainer(gpu)
    tr.load_tensors(inputs, labels, seed=11)
    tr.begin(1)
    lr, l2 = 0.02, 0.001
    tr.step(0, lr, S, p, l2, want_ratios=False, record=False)
    (_, cost, _, _), = tr.drain()
    picked = tr.picked[:S].cpu()
    x = inputs[picked].double()
    y = labels[picked]
    lo, hi = tr.base_seed
    widths = {1: sizes[1], 2: sizes[2], 3: sizes[2], 4: sizes[3]}
    masks = {lid: torch.from_numpy(keep_mask(S * w, lo, hi, lid, p, epoch=0).reshape(S, w)).double()
             for lid, w in widths.items()}
    for m in masks.values():  # the masks really drop ~p of every hidden output
        assert abs(1.0 - m.mean().item() - p) < 0.02
    s = 1.0 / (1.0 - p)
    for q in cpu.params:
        q.requires_grad_()
    if cpu.optimizer is not None:
        for grp in cpu.optimizer.param_groups:
            grp["lr"] = lr
    L = cpu.layers
    z0 = x @ L[0].weights + L[0].bias
    a1 = torch.relu(z0) * masks[1] * s
    z2 = (a1 @ L[2].weights + L[2].bias) * masks[2] * s
    a3 = torch.tanh(z2) * masks[3] * s
    logits = (a3 @ L[4].weights + L[4].bias) * masks[4] * s
    ref = torch.nn.functional.cross_entropy(logits, y) + l2 * sum((w ** 2).sum() for w in cpu.weights)
    ref.backward()
    if cpu.optimizer is not None:
        cpu.optimizer.step()
    else:
        for q in cpu.params:
            q.data -= lr * q.grad
    ctol = 1e-4 if dtype == "float32" else 3e-2
    assert abs(cost - ref.item()) < ctol * max(1.0, abs(ref.item())), (cost, ref.item())
    for pg, pc in zip(gpu.params, cpu.params):
        d = (pg.detach().double().cpu() - pc.detach()).abs()
        if optimizer == "adam":  # first Adam step ~ lr*sign(g): compare in distribution
            assert (d > 0.1 * lr).double().mean().item() < (0.002 if dtype == "float32" else 0.05)
        else:
            tol = 2e-4 if dtype == "float32" else 3e-2
            scale = pc.detach().abs().max().item()
            assert d.max().item() < tol * max(scale, 1e-3) + (1e-3 if dtype == "bfloat16" else 1e-6), d.max()


@pytest.mark.parametrize("optimizer", ["adam", "stochastic"])
def test_fp64_fused_step_matches_reference(optimizer):
    """fp64 on the fused engine: the precision a REST model created with
    device="cuda" and no dtype gets. f64 MFMA GEMMs, fp64 heads / bias gradients / Adam: one step
    equals the CPU reference step to fp64 rounding (rtol 1e-10), the cost to 1e-12."""
    sizes = [256, 512, 256, 128]
    algos = ["relu", "tanh", "softmax"]
    gpu, cpu = _pair(sizes, algos, optimizer, "float64")
    tr = FusedTrainer(gpu)
    assert tr.compute == torch.float64 and tr.grads.dtype == torch.float64 and not tr.shadow_sets[0]
    n, S = 3000, 1024
    g = torch.Generator().manual_seed(1)
    inputs = torch.randn(n, sizes[0], generator=g, dtype=torch.float64)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    data = [(inputs[i].tolist(), [int(labels[i])]) for i in range(n)]
    tr.load_data(data)
    assert tr.data.dtype == torch.float64
    tr.begin(1)
    lr, l2 = 0.01, 0.001
    tr.step(0, lr, S, 0.0, l2, want_ratios=True, record=False)
    (_, cost, ratios, _), = tr.drain()
    picked = tr.picked[:S].cpu()
    prev = [w.clone().detach() for w in cpu.weights]
    cpu_cost = _cpu_step(cpu, inputs[picked], [[int(labels[i])] for i in picked], lr, l2)
    assert abs(cost - cpu_cost) <= 1e-12 * max(1.0, abs(cpu_cost)), (cost, cpu_cost)
    for pg, pc in zip(gpu.params, cpu.params):
        torch.testing.assert_close(pg.detach().cpu(), pc.detach(), rtol=1e-10, atol=1e-12)
    ref_ratios = [((w - pw).std() / (w.std() + 1e-8)).item() for pw, w in zip(prev, cpu.weights)]
    for a, b in zip(ratios, ref_ratios):
        assert abs(a - b) <= 1e-6 * b + 1e-9  # ratios leave the device as fp32


def test_fp64_model_train_uses_fused_engine(models_tmpdir):
    """A default-precision GPU model (fp64) trains through the fused engine, not autograd."""
    torch.manual_seed(0)
    model = NeuralNetworkModel("f64", [9, 18, 9], activation_algos=["relu", "softmax"], device="cuda")
    assert model.precision.name == "float64" and model._fused_trainer() is not None
    data = [([float((i + j) % 3 - 1) for j in range(9)], [i % 9]) for i in range(model.training_buffer_size)]
    model.train(data, epochs=3, learning_rate=0.01, batch_size=64)
    assert model.status == "Trained" and all(p.get("dtype") == "float64" for p in model.progress)


def test_embedding_batchnorm_step_matches_reference():
    sizes = [27, 10, 30, 64, 27]
    algos = ["embedding", "linear", "batchnorm", "tanh", "linear", "softmax"]
    gpu, cpu = _pair(sizes, algos, None, "float32")
    n, S = 2000, 512
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, 27, (n, 3), generator=g)
    labels = torch.randint(0, 27, (n,), generator=g)
    data = [(ids[i].tolist(), [int(labels[i])]) for i in range(n)]
    tr = FusedTrainer(gpu)
    tr.load_data(data)
    tr.begin(1)
    tr.step(0, 0.1, S, 0.0, 0.001, want_ratios=False, record=False)
    (_, cost, _, _), = tr.drain()
    picked = tr.picked[:S].cpu()
    cpu_cost = _cpu_step(cpu, ids[picked].double(), [[int(labels[i])] for i in picked], 0.1, 0.001)
    assert abs(cost - cpu_cost) < 1e-4 * max(1, abs(cpu_cost))
    for pg, pc in zip(gpu.params, cpu.params):
        assert (pg.detach().double().cpu() - pc.detach()).abs().max().item() < 1e-4


def test_mse_head_step_matches_reference():
    sizes = [64, 128, 32]
    algos = ["relu", "sigmoid"]
    gpu, cpu = _pair(sizes, algos, "adam", "float32")
    n, S = 500, 256
    g = torch.Generator().manual_seed(3)
    inputs = torch.randn(n, 64, generator=g)
    targets = torch.rand(n, 32, generator=g)
    data = [(inputs[i].tolist(), targets[i].tolist()) for i in range(n)]
    tr = FusedTrainer(gpu)
    tr.load_data(data)
    tr.begin(1)
    tr.step(0, 0.01, S, 0.0, 0.001, want_ratios=False, record=False)
    (_, cost, _, _), = tr.drain()
    picked = tr.picked[:S].cpu()
    cpu_cost = _cpu_step(cpu, inputs[picked].double(), targets[picked].double().tolist(), 0.01, 0.001)
    assert abs(cost - cpu_cost) < 1e-4 * max(1, abs(cpu_cost))
    for pg, pc in zip(gpu.params, cpu.params):
        assert (pg.detach().double().cpu() - pc.detach()).abs().max().item() < 2e-4


@pytest.mark.parametrize("dtype", ["bfloat16", "float32"])
def test_model_train_on_gpu_end_to_end(models_tmpdir, dtype):
    torch.manual_seed(0)
    model = NeuralNetworkModel("gpu_e2e", [9, 18, 9], activation_algos=["relu", "softmax"], dtype=dtype, device="cuda")
    data = [([float((i + j) % 3 - 1) for j in range(9)], [i % 9]) for i in range(model.training_buffer_size)]
    model.train(data, epochs=5, learning_rate=0.01, batch_size=64)
    assert model.status == "Trained"
    assert len(model.progress) == 5
    assert all(math.isfinite(p["cost"]) for p in model.progress)
    last = model.progress[-1]  # optional GPU telemetry beside the reference keys
    assert last["world_size"] == 1 and last["dtype"] == dtype and last["step_ms"] > 0 and last["samples_per_s"] > 0
    assert model.stats is not None and len(model.stats["layers"]) == len(model.layers)
    assert model.stats["layers"][-1]["gradient"] is None
    loaded = NeuralNetworkModel.deserialize("gpu_e2e")
    assert loaded.on_gpu and loaded.precision.name == dtype
    for a, b in zip(loaded.params, model.params):
        assert torch.equal(a, b)
    assert loaded.optimizer is not None
    out, cost = loaded.compute_output(data[0][0], data[0][1])
    assert len(out) == 9 and cost is not None


def test_record_mode_matches_fused_cost():
    sizes = [128, 256, 64]
    gpu, _ = _pair(sizes, ["relu", "softmax"], "adam", "float32")
    n = 400
    data = [(torch.randn(128).tolist(), [i % 64]) for i in range(n)]
    tr = FusedTrainer(gpu)
    tr.load_data(data)
    tr.begin(2)
    snap = gpu._param_store.flat.clone()
    tr.step(0, 0.01, 256, 0.2, 0.001, want_ratios=False, record=False)
    fused = tr.drain()[0][1]
    gpu._param_store.flat.copy_(snap)
    tr.opt.init_stats()
    tr.step(0, 0.01, 256, 0.2, 0.001, want_ratios=False, record=True)
    recorded = tr.drain()[0][1]
    assert abs(fused - recorded) < 1e-5 * max(1, abs(fused))
    rec = tr.record()
    assert len(rec["activations"]) == len(gpu.layers)


def test_fp8_training_tracks_bf16():
    """fp8 policy on the TRANSPOSED-copy path (a width of 128: not every width is a multiple of
    256, so the forward reads a [out, in] e4m3 copy; tests/test_fastpaths_gpu.py covers the
    natural-layout path the benchmark config takes): e4m3 forward GEMMs (current-scaled weights,
    delayed-scaled activations, e4m3 input at a static dataset scale), e5m2-gradient x e4m3-weight
    backward dX GEMMs (delayed gradient scaling), e4m3 x e5m2 dW where the shapes allow; the loss
    curve follows the bf16 run of the same model + batches within the Adam sign-noise band."""
    sizes = [256, 512, 512, 128]
    algos = ["relu", "relu", "softmax"]
    n, S, steps = 4096, 1024, 12
    g = torch.Generator().manual_seed(2)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    idx = torch.randint(0, n, (steps, S), generator=g)
    curves = {}
    for dtype in ("bfloat16", "fp8"):
        torch.manual_seed(0)
        model = NeuralNetworkModel("f8", sizes, "xavier", "random", algos, "adam", dtype=dtype, device="cuda")
        tr = FusedTrainer(model)
        tr.load_tensors(inputs, labels, seed=9)
        tr.begin(steps)
        for e in range(steps):
            tr.step(e, 0.002, S, 0.1, 1e-4, want_ratios=False, record=False, indices=idx[e])
        curves[dtype] = [c for _, c, _, _ in tr.drain()]
        if dtype == "fp8":
            assert [st.fp8 for st in tr.stages] == [True, True, True]
            # backward dX GEMMs of layers 2 and 3 on e5m2 gradients x e4m3 [in, out] weights
            assert [st.fp8_bwd for st in tr.stages] == [False, True, True]
            s_g = tr.gqs[1:, 1].cpu()
            assert torch.all(s_g > 0) and torch.all(torch.isfinite(s_g)) and tr._g8_calibrated
            assert "y8" in tr.stages[0].buffers and "y8" in tr.stages[1].buffers
            s_w = tr.wqs[:, 1].cpu()
            assert torch.all(s_w > 0) and torch.all(torch.isfinite(s_w))
            # weight scales: the amax the optimizer reduced equals max|w| of the current weights,
            # the other parity's accumulator was cleared, and the e4m3 copy is W^T * q
            torch.cuda.synchronize()
            gemms = [st for st in tr.stages if st.kind == "gemm"]
            amax = torch.stack([tr.store.view(st.seg_w).abs().max() for st in gemms])
            rows = tr.wamax2.cpu()
            assert (rows == 0).all(dim=1).sum() == 1, rows
            assert torch.equal(rows.max(dim=0).values, amax.cpu()), (rows, amax)
            for st in gemms:
                q = tr.wqs[st.w8_index, 0]
                assert torch.allclose(q, 448.0 / amax[st.w8_index], rtol=1e-6)
                ref = (tr.store.view(st.seg_w) * q).clamp(-448, 448).t()
                got = tr.w8[st.seg_w.offset].float()
                assert torch.all((got - ref).abs() <= ref.abs() * 0.0625 + 2 ** -9), st.index
            # first-layer input: the sampled rows of the once-quantised dataset
            assert torch.allclose(tr.xqs[0].cpu(), 448.0 / inputs.to(torch.bfloat16).float().abs().max(), rtol=1e-6)
            picked = tr.picked[:S]
            assert torch.equal(tr.x8[:S].view(torch.uint8), tr.data8[picked].view(torch.uint8))
            ref = (tr.x_in[:S].float() * tr.xqs[0]).clamp(-448, 448)
            assert torch.all((tr.x8[:S].float() - ref).abs() <= ref.abs() * 0.0625 + 2 ** -9)
    bf, f8 = curves["bfloat16"], curves["fp8"]
    assert all(math.isfinite(c) for c in f8)
    assert f8[-1] < f8[0] - 0.05  # it learns
    for a, b in zip(bf, f8):
        assert abs(a - b) < 0.05 * abs(a) + 0.02, (bf, f8)


@pytest.mark.parametrize("optimizer", ["adam", "stochastic"])
def test_fused_dw_update_matches_separate_launches(monkeypatch, optimizer):
    """PZ_OPT_FUSE: the weight updates applied in the dW GEMMs' epilogues reproduce the unfused
    schedule (dW GEMM -> fp32 gradient -> side-stream optimizer launches): costs, update ratios,
    parameters and Adam moments. Shapes cover the one-pass and the split-K dW GEMM."""
    sizes = [1024, 2048, 1024, 256]
    algos = ["relu", "relu", "softmax"]
    n, S, steps = 8192, 4096, 4
    g = torch.Generator().manual_seed(5)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    idx = torch.randint(0, n, (steps, S), generator=g)
    runs = {}
    for run in ("0", "0b", "1"):  # 0b: a second unfused run = the noise floor between two runs
        fuse = run[0]
        monkeypatch.setenv("PZ_OPT_FUSE", fuse)
        monkeypatch.setenv("PZ_GRAD_DTYPE", "fp32")  # the unfused schedule's gradients exact, as the fused ones
        gpu, _ = _pair(sizes, algos, optimizer, "bfloat16")
        tr = FusedTrainer(gpu)
        assert tr.fuse_opt == (fuse == "1")
        tr.load_tensors(inputs, labels, seed=3)
        tr.begin(steps)
        for e in range(steps):
            tr.step(e, 0.005, S, 0.1, 1e-3, want_ratios=e % 2 == 0, record=False, indices=idx[e])
        out = tr.drain()
        if fuse == "1":
            assert tr._fuse_ok and all(tr._fuse_ok.values())  # every dW GEMM took the fused path
        state = gpu.optimizer.state_dict() if gpu.optimizer is not None else None
        runs[run] = ([c for _, c, _, _ in out], [r for _, _, r, _ in out], gpu._param_store.flat.clone(), state,
                     tr.opt.exp_avg.clone() if tr.opt.adam else None)
    (c0, r0, p0, s0, m0), (c1, r1, p1, s1, m1) = runs["0"], runs["1"]
    cn = runs["0b"][0]
    for a, b, n in zip(c0, c1, cn):  # within the run-to-run noise of the unfused schedule itself
        # (the noise floor of ONE pair of runs can be tiny by chance: an absolute allowance of 5e-4
        # relative — a broken fused update moves the cost by O(1) — keeps this from flaking)
        assert abs(a - b) <= 3 * abs(a - n) + 5e-4 * max(1.0, abs(a)), (c0, c1, cn)
    for a, b in zip(r0, r1):
        assert (a is None) == (b is None)
        if a is not None:
            assert all(abs(x - y) < 1e-3 * abs(x) + 1e-7 for x, y in zip(a, b)), (a, b)
    # the schedules sum the dW tiles in different orders (split-K 4 beside the fused update, the
    # paired launch's split-K 2 in the unfused schedule), which bf16 activation rounding and Adam's
    # ~lr * sign(m) first steps amplify; two runs of the SAME schedule are bit-identical
    # (PZ_DETERMINISTIC), so the bounds are absolute
    pn = runs["0b"][2]
    assert torch.equal(p0, pn)
    d, dn = (p0 - p1).abs(), (p0 - pn).abs()
    mean, mean_n = d.mean().item(), dn.mean().item()
    frac, frac_n = (d > 1e-3).double().mean().item(), (dn > 1e-3).double().mean().item()
    assert mean <= 3 * mean_n + 2e-5 and frac <= 3 * frac_n + 1e-3, (mean, mean_n, frac, frac_n)
    if optimizer == "adam":
        assert mean < 1e-4, mean
        assert torch.equal(m0, runs["0b"][4])
        # (Adam's ~lr-sized sign flips on near-zero gradients feed the next steps' gradients, so
        # the moments drift by a few per cent where the parameters flipped; a broken fused update
        # moves them by O(1))
        rel = (m0 - m1).abs().mean().item() / m0.abs().mean().item()
        assert rel <= 0.05, rel
        for k in s0["state"]:
            assert float(s0["state"][k]["step"]) == float(s1["state"][k]["step"]) == steps
    else:
        assert d.max().item() < 1e-3 and mean < 1e-6, (d.max(), mean)


@pytest.mark.parametrize("optimizer", ["adam", "stochastic"])
def test_graph_replay_matches_eager_steps(optimizer):
    """hipGraph-replayed steps (epoch-dependent dropout keys, sampler seeds and optimizer
    hyper-parameters read from the device epoch counter / tables) reproduce eager launches."""
    sizes = [256, 512, 256, 128]
    algos = ["relu", "tanh", "softmax"]
    n, S, epochs = 2048, 512, 9
    g = torch.Generator().manual_seed(4)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    runs = {}
    for graphs in (False, True):
        gpu, _ = _pair(sizes, algos, optimizer, "bfloat16")
        tr = FusedTrainer(gpu)
        tr.use_graphs = graphs
        tr.load_tensors(inputs, labels, seed=11)
        sched = lambda e: 0.01 * 0.9 ** e  # noqa: E731
        tr.begin(epochs, lr_schedule=sched)
        every = max(1, epochs // 100)
        for e in range(epochs):
            tr.step(e, 0.01 * 0.9 ** e, S, 0.2, 1e-3, want_ratios=e % every == 0, record=e == epochs - 1)
        out = tr.drain()
        assert bool(tr._graphs) == graphs  # the graph run really replayed captured steps
        runs[graphs] = ([c for _, c, _, _ in out], [r for _, _, r, _ in out], gpu._param_store.flat.clone(),
                        gpu.optimizer.state_dict() if gpu.optimizer is not None else None)
    # same masks, seeds and hyper-parameters; only the float-atomic bias-gradient sums may round
    # in a different order (as between two eager runs)
    (c0, r0, p0, s0), (c1, r1, p1, s1) = runs[False], runs[True]
    assert all(math.isfinite(c) for c in c1)
    for a, b in zip(c0, c1):
        assert abs(a - b) < 1e-4 * max(1.0, abs(a)), (c0, c1)
    for a, b in zip(r0, r1):
        assert (a is None) == (b is None)
        if a is not None:
            assert all(abs(x - y) < 1e-3 * abs(x) + 1e-7 for x, y in zip(a, b)), (a, b)
    d = (p0 - p1).abs()
    assert (d > 1e-3).double().mean().item() < 1e-3 and d.mean().item() < 1e-5
    if s0 is not None:
        for k in s0["state"]:
            assert float(s0["state"][k]["step"]) == float(s1["state"][k]["step"]) == epochs


def test_paired_dw_gemm_matches_separate_launches():
    """pz::gemm_pair (the first layer's and a later layer's weight-gradient GEMMs in ONE launch)
    against one launch per GEMM, compared on the dW buffers themselves (fp32 outputs): both within
    fp32 summation-order rounding of the fp64 product."""
    from penr_oz_neural_network_torch_amd.ops import functional as PF
    K = 8192
    g = torch.Generator(device="cpu").manual_seed(7)
    x0 = torch.randn(K, 1024, generator=g).to("cuda", torch.bfloat16)   # [K, M0]: layer-1 input
    z0 = torch.randn(K, 4096, generator=g).to("cuda", torch.bfloat16)   # [K, N0]
    x1 = torch.randn(K, 4096, generator=g).to("cuda", torch.bfloat16)   # [K, M1]: last layer's input
    z1 = torch.randn(K, 1024, generator=g).to("cuda", torch.bfloat16)   # [K, N1]
    pair = [torch.empty(1024, 4096, device="cuda"), torch.empty(4096, 1024, device="cuda")]
    sep = [torch.empty_like(pair[0]), torch.empty_like(pair[1])]
    assert PF.gemm_pair_split(x0, z0, pair[0], x1, z1, pair[1]) > 0
    PF.gemm_pair(x0, z0, pair[0], x1, z1, pair[1])
    PF.gemm(x0, False, z0, False, sep[0])
    PF.gemm(x1, False, z1, False, sep[1])
    for (a, b), p_, s_ in zip(((x0, z0), (x1, z1)), pair, sep):
        ref = a.double().t() @ b.double()
        scale = ref.abs().max().item()
        assert (p_.double() - ref).abs().max().item() <= 2e-6 * scale
        assert (s_.double() - ref).abs().max().item() <= 2e-6 * scale
        assert (p_ - s_).abs().max().item() <= 2e-6 * scale


@pytest.mark.parametrize("dtype", ["bfloat16", "fp8"])
def test_paired_dw_step_tracks_separate_launches(monkeypatch, dtype):
    """PZ_DW_PAIR in the trainer: costs track the unpaired schedule and no weight moves further
    than Adam's per-step bound allows (the dW buffers themselves: the test above)."""
    sizes = [1024, 2048, 1024, 512]
    algos = ["relu", "relu", "softmax"]
    n, S, steps = 8192, 4096, 4
    g = torch.Generator().manual_seed(12)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    idx = torch.randint(0, n, (steps, S), generator=g)
    runs = {}
    for run in ("0", "1"):
        monkeypatch.setenv("PZ_DW_PAIR", run)
        torch.manual_seed(0)
        model = NeuralNetworkModel("pr", sizes, "xavier", "random", algos, "adam", dtype=dtype, device="cuda")
        tr = FusedTrainer(model)
        assert (tr._pair_idx is not None) == (run == "1")
        tr.load_tensors(inputs, labels, seed=3)
        tr.begin(steps)
        for e in range(steps):
            tr.step(e, 0.003, S, 0.1, 1e-3, want_ratios=True, record=False, indices=idx[e])
        out = tr.drain()
        if run == "1":
            assert tr._pair_idx == 2 and any(k[0] == "pair" and v for k, v in tr._y_dead_cache.items())
        runs[run] = ([c for _, c, _, _ in out], model._param_store.flat.clone())
    (c0, p0), (c1, p1) = runs["0"], runs["1"]
    for a, b in zip(c0, c1):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(a)), (c0, c1)
    assert (p0 - p1).abs().max().item() <= 2 * 0.003 * steps + 1e-6


def test_bf16_training_is_bit_reproducible():
    """PZ_DETERMINISTIC (default): the same model, data and seeds trained twice give bit-identical
    weights and optimizer moments — split-K / stream-K partial tiles and the bias-gradient column
    sums are folded in a fixed order, never in arrival order."""
    sizes = [1024, 4096, 4096, 1024]
    algos = ["relu", "relu", "softmax"]
    n, S, steps = 8192, 8192, 3
    g = torch.Generator().manual_seed(5)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    flats = []
    for _ in range(2):
        torch.manual_seed(0)
        model = NeuralNetworkModel("det", sizes, "xavier", "random", algos, "adam", dtype="bfloat16", device="cuda")
        tr = FusedTrainer(model)
        tr.load_tensors(inputs, labels, seed=9)
        tr.begin(steps)
        for e in range(steps):
            tr.step(e, 1e-3, S, 0.1, 0.0, want_ratios=False, record=False)
        tr.drain()
        st = model.optimizer.state_dict()["state"]
        flats.append((model._param_store.flat.clone(), [v["exp_avg"].clone() for v in st.values()]))
    assert torch.equal(flats[0][0], flats[1][0])
    assert all(torch.equal(a, b) for a, b in zip(flats[0][1], flats[1][1]))


def test_training_with_record_steps_is_bit_reproducible():
    """PZ_DETERMINISTIC across a batch-size change and a RECORD step (the stats epochs: unfused
    epilogues, per-layer outputs kept, bias gradients from pz::colsum's ordered fold instead of
    float atomics): two runs give bit-identical weights and Adam moments; the costs (float-atomic
    loss slots) agree to rounding."""
    sizes = [1024, 2048, 2048, 512]
    algos = ["relu", "relu", "softmax"]
    n, steps = 8192, 5
    g = torch.Generator().manual_seed(6)
    inputs = torch.randn(n, sizes[0], generator=g)
    labels = torch.randint(0, sizes[-1], (n,), generator=g)
    outs = []
    for _ in range(2):
        torch.manual_seed(0)
        model = NeuralNetworkModel("bnd", sizes, "xavier", "random", algos, "adam", dtype="bfloat16", device="cuda")
        tr = FusedTrainer(model)
        tr.load_tensors(inputs, labels, seed=4)
        tr.begin(steps)
        for e in range(steps):
            tr.step(e, 1e-3, 4096 if e != 3 else 2048, 0.2, 1e-3, want_ratios=True, record=e == 2)
        costs = [c for _, c, _, _ in tr.drain()]
        st = model.optimizer.state_dict()["state"]
        outs.append((model._param_store.flat.clone(), [v["exp_avg"].clone() for v in st.values()], costs))
        tr.close()
    assert torch.equal(outs[0][0], outs[1][0])
    assert all(torch.equal(a, b) for a, b in zip(outs[0][1], outs[1][1]))
    assert all(abs(a - b) <= 1e-12 * abs(b) for a, b in zip(outs[0][2], outs[1][2]))
