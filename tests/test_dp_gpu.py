"""Data-parallel equivalence: a 2-rank step == a 1-rank step on the concatenated batch.

Both ranks share the box's single GPU and talk over ``gloo`` (RCCL refuses two ranks on one
device); the code path under test — bucketed async all-reduce issued during backward, 1/world
folded into the optimizer, loss averaged through the gradient buffer — is the one that runs
over RCCL/xGMI on a full node.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [128, 256, 256, 64]
ALGOS = ["relu", "tanh", "softmax"]
N, B = 1024, 256  # dataset rows, per-rank batch


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


ALGOS_BN = ["linear", "batchnorm", "relu", "tanh", "softmax"]  # + linear before tanh / softmax


def _data(world=2):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, SIZES[0], generator=g)
    y = torch.randint(0, SIZES[-1], (N,), generator=g)
    idx = torch.randint(0, N, (world * B,), generator=g)
    return x, y, idx


def _build(optimizer, comm, bn=False):
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
    torch.manual_seed(0)
    dtype = "float32" if comm == "fp32" else "bfloat16"  # bf16 gradient buckets need a bf16-compute model
    return NeuralNetworkModel("dp", SIZES, "xavier", "random", ALGOS_BN if bn else ALGOS, optimizer, dtype=dtype,
                              device="cuda:0")


def _bn_stats(model):
    return [(l.mean.detach().float().cpu().reshape(-1), l.variance.detach().float().cpu().reshape(-1))
            for l in model.layers if l.algo == "batchnorm"]


def _zero_env(zero, on="auto"):
    """zero: "auto" / "1" (the default scope: weights complete mid-backward), "side" (+ the paired
    partner), "all" (every dense weight), "0" (replicated)"""
    os.environ.pop("PZ_ZERO_SCOPE", None)
    os.environ["PZ_ZERO"] = on if zero in ("side", "all") else zero
    if zero in ("side", "all"):
        os.environ["PZ_ZERO_SCOPE"] = zero


def _rank_main(rank, world, port, optimizer, comm, out_path, bn=False, zero="auto"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), PZ_GRAD_COMM_DTYPE=comm)
    _zero_env(zero)
    torch.set_num_threads(2)
    # file rendezvous (port = the store path): no TCP port picked ahead of the spawned ranks
    dist.init_process_group("gloo", init_method=f"file://{port}", rank=rank, world_size=world)
    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    model = _build(optimizer, comm, bn)
    tr = FusedTrainer(model, DataParallelContext(rank, world))
    assert bool(tr.grads16) == (comm == "bf16")
    # the sharded optimizer (engine/zero.py) is the default for bf16 buckets
    assert (tr.zero is not None) == (comm == "bf16" and zero != "0"), (comm, zero)
    x, y, idx = _data(world)
    tr.load_tensors(x, y, seed=3)
    tr.begin(2)
    for e in range(2):
        tr.step(e, 0.01, world * B, 0.0, 1e-3, want_ratios=True, record=False, indices=idx[rank * B:(rank + 1) * B])
    costs = [c for _, c, _, _ in tr.drain()]
    m = tr.opt.exp_avg.cpu() if tr.opt.exp_avg is not None else None
    torch.save({"flat": model._param_store.flat.cpu(), "costs": costs, "bn": _bn_stats(model), "m": m,
                "pth": model.optimizer.state_dict() if model.optimizer is not None else None},
               out_path + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


# Tolerances of the data-parallel step against ONE rank on the concatenated batch, per gradient
# bucket dtype and world size (measured on MI355X, with ~2x headroom): fp32 buckets differ only by
# the summation order; bf16 buckets (the default for bf16 models: dW GEMMs write bf16, the
# all-reduce sums bf16) add one bf16 rounding of each rank's gradient plus the ring's bf16 partial
# sums, which grow with the number of ranks (trainer.py, PZ_GRAD_COMM_DTYPE).
TOL = {  # (comm, world): (cost rel, adam mean |dp|, adam frac |dp| > 1e-3, sgd max |dp|)
    ("fp32", 2): (1e-5, 1e-5, 1e-3, 1e-6), ("bf16", 2): (2e-3, 2e-4, 2e-2, 1e-4),
    ("fp32", 8): (1e-5, 1e-5, 1e-3, 1e-6), ("bf16", 8): (4e-3, 4e-4, 4e-2, 2e-4),
    ("bf16", 3): (4e-3, 4e-4, 4e-2, 2e-4),
}


@pytest.mark.parametrize("world,optimizer,comm,bn,zero", [
    (2, "adam", "fp32", False, "auto"), (2, "adam", "bf16", False, "auto"), (2, "stochastic", "fp32", False, "auto"),
    (2, "stochastic", "bf16", False, "auto"), (2, "adam", "fp32", True, "auto"), (2, "adam", "bf16", True, "auto"),
    (2, "adam", "bf16", False, "0"), (3, "adam", "bf16", False, "auto"), (3, "stochastic", "bf16", False, "auto"),
    (3, "adam", "bf16", False, "all"), (8, "adam", "bf16", False, "auto"), (8, "adam", "bf16", False, "0"),
    (8, "adam", "bf16", False, "all"), (2, "adam", "bf16", False, "side"), (8, "adam", "bf16", False, "side"),
    (8, "stochastic", "fp32", False, "auto"),
    (8, "stochastic", "bf16", False, "auto")])
def test_multi_rank_step_equals_single_rank(tmp_path, monkeypatch, world, optimizer, comm, bn, zero):
    """A W-rank data-parallel fused step == one rank on the concatenated batch (W ranks share the
    box's GPU over gloo; the code path is the RCCL one). Batchnorm statistics are synchronised:
    every rank ends with the single rank's running mean / variance. bf16 buckets run the sharded
    optimizer (reduce-scatter, 1/W slice updates, all-gathered bf16 copies; 3 ranks: uneven
    slices) unless PZ_ZERO=0; its masters and Adam moments are gathered whole at drain(), so every
    rank's parameters AND the .pth Adam state equal the single rank's."""
    out = str(tmp_path / "dp.pt")
    mp.start_processes(_rank_main, args=(world, str(tmp_path / "rdv"), optimizer, comm, out, bn, zero), nprocs=world,
                       start_method="spawn")
    ranks = [torch.load(out + f".{r}", weights_only=True) for r in range(world)]
    dp = ranks[0]

    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    model = _build(optimizer, comm, bn)
    monkeypatch.setenv("PZ_GRAD_DTYPE", comm)  # the single process stores its gradients like the buckets
    tr = FusedTrainer(model)
    x, y, idx = _data(world)
    tr.load_tensors(x, y, seed=3)
    tr.begin(2)
    for e in range(2):
        tr.step(e, 0.01, world * B, 0.0, 1e-3, want_ratios=True, record=False, indices=idx)
    costs = [c for _, c, _, _ in tr.drain()]
    ctol, mtol, ftol, stol = TOL[(comm, world)]
    d = (dp["flat"] - model._param_store.flat.cpu()).abs()
    print(f"world {world} {comm} {optimizer} bn={bn}: cost rel "
          f"{max(abs(a - b) / max(1.0, abs(b)) for a, b in zip(dp['costs'], costs)):.2e}, |dp| mean "
          f"{d.mean().item():.2e} max {d.max().item():.2e} frac>1e-3 {(d > 1e-3).double().mean().item():.2e}")
    for a, b in zip(dp["costs"], costs):
        assert abs(a - b) < ctol * max(1.0, abs(b)), (dp["costs"], costs)
    if optimizer == "adam":  # sign-noise flips of ~lr on near-zero gradients are legitimate
        assert (d > 1e-3).double().mean().item() < ftol
        assert d.mean().item() < mtol
    else:
        assert d.max().item() < stol, d.max().item()
    for r in ranks:  # identical replicas (the sharded optimizer's gathered slices included)
        assert torch.equal(r["flat"], dp["flat"])
    if optimizer == "adam":  # the gathered Adam moments: whole, identical, and the single rank's
        dm = (dp["m"] - tr.opt.exp_avg.cpu()).abs()
        assert dm.mean().item() < 2e-2 * dp["m"].abs().mean().item() + 1e-8, dm.mean().item()
        for r in ranks:
            assert torch.equal(r["m"], dp["m"])
        st0, ref = dp["pth"]["state"], model.optimizer.state_dict()["state"]
        assert sorted(st0) == sorted(ref) and all(float(st0[k]["step"]) == 2.0 for k in st0)
        for k in st0:
            assert st0[k]["exp_avg"].shape == ref[k]["exp_avg"].shape
    if bn:
        want = _bn_stats(model)
        for r in ranks:
            # (bf16 buckets: step 2's batch statistics see step 1's bf16-rounded updates)
            rt, at = (1e-4, 1e-5) if comm == "fp32" else (2e-3, 1e-4)
            for (m, v), (wm, wv) in zip(r["bn"], want):
                torch.testing.assert_close(m, wm, rtol=rt, atol=at)
                torch.testing.assert_close(v, wv, rtol=rt, atol=at)


def _forced_main(rank, comm, out_path, impl="native", zero="auto"):
    """World size 1 with PZ_FORCE_COMM=1: every gradient bucket goes through a real 1-rank RCCL
    all-reduce (PZ_ZERO=1: reduce-scatter + slice update + all-gather) on its comm stream, waited
    for by the optimizer's stream."""
    os.environ.update(PZ_FORCE_COMM="1", PZ_GRAD_COMM_DTYPE=comm, PZ_COMM=impl, MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(_free_port()))
    _zero_env(zero, on="1")
    if impl == "proxy":  # (the proxy's 16 workgroups, and the GEMMs behind a bucket on 240 CUs)
        os.environ.update(PZ_COMM_PROXY_WGS="16", PZ_COMM_BUDGET="16")
    os.environ.pop("WORLD_SIZE", None)
    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    ctx = init_from_env()
    assert ctx.force and ctx.enabled and ctx.world_size == 1 and ctx.backend == "nccl", ctx
    # gradient buckets on the extension's RCCL communicator (csrc/rccl_comm.cpp), its collective-
    # footprint proxy (comm_proxy.hip: channel kernels held for a modelled 8-rank ring time, on a
    # CU-masked stream) or ProcessGroupNCCL
    assert (ctx.native is not None) == (impl in ("native", "proxy")), ctx
    model = _build("adam", "bf16")
    tr = FusedTrainer(model, ctx)
    assert bool(tr.grads16) == (comm == "bf16")
    assert (tr.zero is not None) == (zero in ("1", "side", "all")), zero
    if tr.zero is not None:  # one rank: one whole slice (the proxy shards for the world it models, as rank 0)
        assert tr.zero.world == (8 if impl == "proxy" else 1) and tr.zero.rank == 0
    # PZ_COMM_BUDGET: the backward GEMMs behind a bucket run on the persistent engine with the CUs
    # the collective kernels leave
    budget = 16 if impl == "proxy" else 0
    assert ctx.comm_cus == budget
    assert tr._cus_comm == (torch.cuda.get_device_properties(0).multi_processor_count - 16 if budget else 0)
    x, y, idx = _data()
    tr.load_tensors(x, y, seed=3)
    tr.begin(3)
    for e in range(3):
        # (epoch 2 is a record step: all-reduced buckets, whole-master gather, slice update)
        tr.step(e, 0.01, 2 * B, 0.2, 1e-3, want_ratios=True, record=e == 2, indices=idx)
    costs = [c for _, c, _, _ in tr.drain()]
    torch.save({"flat": model._param_store.flat.cpu(), "costs": costs}, out_path)
    shutdown()


@pytest.mark.parametrize("comm,impl,zero", [("fp32", "native", "auto"), ("bf16", "native", "auto"),
                                            ("fp32", "torch", "auto"), ("fp32", "proxy", "auto"),
                                            ("bf16", "native", "1"), ("bf16", "torch", "1"), ("bf16", "proxy", "1"),
                                            ("bf16", "native", "side"), ("bf16", "native", "all"),
                                            ("bf16", "proxy", "all")])
def test_forced_rccl_world1_matches_no_comm(tmp_path, monkeypatch, comm, impl, zero):
    out = str(tmp_path / "forced.pt")
    mp.start_processes(_forced_main, args=(comm, out, impl, zero), nprocs=1, start_method="spawn")
    got = torch.load(out, weights_only=True)
    if impl == "proxy" and zero in ("1", "side", "all"):
        # the proxy runs the sharded step of its modelled world as rank 0 (1/8 of every weight is
        # updated): a timing model, whose numbers need only be finite
        assert all(math.isfinite(c) for c in got["costs"]) and torch.isfinite(got["flat"]).all()
        return
    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    model = _build("adam", "bf16")
    monkeypatch.setenv("PZ_GRAD_DTYPE", comm)
    tr = FusedTrainer(model, DataParallelContext())
    x, y, idx = _data()
    tr.load_tensors(x, y, seed=3)
    tr.begin(3)
    for e in range(3):
        tr.step(e, 0.01, 2 * B, 0.2, 1e-3, want_ratios=True, record=e == 2, indices=idx)
    costs = [c for _, c, _, _ in tr.drain()]
    flat = model._param_store.flat.cpu()
    if comm == "fp32":
        # a 1-rank fp32 all-reduce is the identity; what remains is the schedule's summation order
        # (the single process pairs the first layer's dW with its partner's and runs the tiled
        # split-K engine; the DP step runs one dW per bucket on the budgeted stream-K engine),
        # which Adam turns into ~lr-sized flips only on near-zero gradients
        for a, b in zip(got["costs"], costs):
            assert abs(a - b) < 1e-5 * max(1.0, abs(b)), (got["costs"], costs)
        d = (got["flat"] - flat).abs()
        frac = (d > 0).double().mean().item()
        assert d.mean().item() < 1e-6 and (d > 1e-3).double().mean().item() < 1e-3, (d.max().item(), frac)
    else:  # bf16 gradient buckets: one rounding of each dense weight gradient
        for a, b in zip(got["costs"], costs):
            assert abs(a - b) < 2e-3 * max(1.0, abs(b))
        d = (got["flat"] - flat).abs()
        assert d.mean().item() < 2e-4 and (d > 1e-3).double().mean().item() < 2e-2


def test_bench_launches_its_own_ranks(tmp_path):
    """`bench.py --gpus 2` with no launcher starts 2 rank processes itself (on a 1-GPU box they
    rehearse over gloo, sharing the GPU) and reports the process group's real size."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--batch", "1024"], capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["config"]["dist_world_size"] == 2
    assert out["config"]["dist_backend"] in ("gloo", "nccl") and out["config"]["launcher"] == "self"
    assert out["config"]["global_batch"] == 2048 and out["value"] > 0
    # a process group that does not hold --gpus ranks is an error, not a relabelled 1-GPU number
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=dict(env, WORLD_SIZE="1"), cwd=str(tmp_path))
    assert r.returncode != 0 and "process group holds 1" in r.stderr


def test_native_rccl_communicator_world1(native_lib):
    """csrc/rccl_comm.cpp on one GPU: a 1-rank communicator sums in place (identity), a bucket's
    ticket orders ANOTHER stream behind the collective, stale tickets are refused."""
    uid = native_lib.rccl_unique_id()
    assert uid.dtype == torch.uint8 and uid.numel() == 128
    h = native_lib.rccl_init(uid, 1, 0, True)
    try:
        side = torch.cuda.Stream()
        for dt in (torch.float32, torch.bfloat16, torch.float64):
            x = torch.randn(1 << 20, device="cuda").to(dt)
            ref = x.clone()
            ticket = native_lib.rccl_all_reduce(h, x)
            with torch.cuda.stream(side):
                native_lib.rccl_wait(h, ticket)
                y = x * 2
            torch.cuda.synchronize()
            assert torch.equal(x, ref) and torch.equal(y, ref * 2)
        with pytest.raises(RuntimeError):
            native_lib.rccl_wait(h, 10 ** 6)
    finally:
        native_lib.rccl_destroy(h)
