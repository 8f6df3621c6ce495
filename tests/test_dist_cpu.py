"""CPU multi-process tests of the data-parallel communicator (gloo, world_size 2)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(PZ_RENDEZVOUS_FILE=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    ctx = init_from_env("gloo")
    assert ctx.rank == rank and ctx.world_size == world and ctx.enabled
    # bucketed async all-reduce, several buckets in flight, waited together (trainer pattern)
    flat = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    buckets = [flat[0:100], flat[100:600], flat[600:1000]]
    handles = [ctx.all_reduce_async(b) for b in reversed(buckets)]
    ctx.wait_all(handles)
    # broadcast: rank 0's replica wins
    rep = torch.full((7,), float(rank))
    ctx.broadcast_(rep)
    mx = ctx.all_reduce_scalar_max(float(rank) + 0.5)
    sm = ctx.all_reduce_scalar(1.0)
    # reduced-precision bucket path (PZ_GRAD_COMM_DTYPE=bf16)
    ctx.comm_dtype = torch.bfloat16
    g = torch.full((64,), 0.5 * (rank + 1))
    ctx.wait_all([ctx.all_reduce_async(g)])
    torch.save({"flat": flat, "rep": rep, "max": mx, "sum": sm, "bf16": g}, os.path.join(out_dir, f"r{rank}.pt"))
    ctx.barrier()
    shutdown()


def test_gloo_two_rank_communicator(tmp_path):
    mp.start_processes(_worker, args=(2, str(tmp_path / "rdv"), str(tmp_path)), nprocs=2, start_method="spawn")
    expect = torch.arange(1000, dtype=torch.float32) * 3
    for r in range(2):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.equal(got["flat"], expect)
        assert torch.equal(got["rep"], torch.zeros(7))
        assert got["max"] == 1.5 and got["sum"] == 2.0
        assert torch.allclose(got["bf16"], torch.full((64,), 1.5))


def _train_rank(rank, world, port, optimizer, out_dir, bn=False):
    os.environ.update(PZ_RENDEZVOUS_FILE=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    init_from_env("gloo")
    model, data = _dp_model(optimizer, bn)
    torch.manual_seed(100 + rank)  # ranks' own RNG streams differ; the shared sampler decides the data
    model._train_autograd(data, 4, 0.05, 32, 0.9, 0.0, 1e-3, sampler=torch.Generator().manual_seed(21))
    if rank == 0:
        torch.save({"params": [p.detach() for p in model.params], "costs": [p["cost"] for p in model.progress],
                    "bn": _bn_running(model)}, os.path.join(out_dir, "dp.pt"))
    else:
        torch.save({"bn": _bn_running(model)}, os.path.join(out_dir, f"bn{rank}.pt"))
    shutdown()


def _bn_running(model):
    return [(l.mean.detach().clone(), l.variance.detach().clone()) for l in model.layers if l.algo == "batchnorm"]


def _dp_model(optimizer, bn=False):
    from neural_net_model import NeuralNetworkModel
    torch.manual_seed(3)
    algos = ["linear", "batchnorm", "tanh", "softmax"] if bn else ["tanh", "softmax"]
    model = NeuralNetworkModel("dp", [6, 16, 4], "xavier", "random", algos, optimizer)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(200, 6, generator=g, dtype=torch.float64)
    y = torch.randint(0, 4, (200,), generator=g)
    return model, [(x[i].tolist(), [int(y[i])]) for i in range(200)]


import pytest  # noqa: E402


@pytest.mark.parametrize("world,optimizer,bn", [(2, "adam", False), (2, "stochastic", False), (2, "adam", True),
                                                (8, "adam", False), (8, "stochastic", True)])
def test_gloo_data_parallel_training_equals_single_process(tmp_path, world, optimizer, bn):
    """CPU data parallelism (reference fp64 path): W ranks x 32/W samples == 1 process x 32, to
    fp64 rounding — at world 8 too, and for batchnorm models, whose statistics are synchronised
    over the ranks (every rank ends with the single process's running mean / variance)."""
    mp.start_processes(_train_rank, args=(world, str(tmp_path / "rdv"), optimizer, str(tmp_path), bn), nprocs=world,
                       start_method="spawn")
    dp = torch.load(tmp_path / "dp.pt", weights_only=True)
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    model, data = _dp_model(optimizer, bn)
    model._train_autograd(data, 4, 0.05, 32, 0.9, 0.0, 1e-3, context=DataParallelContext(),
                          sampler=torch.Generator().manual_seed(21))
    # batchnorm: the ranks form the statistics from all-reduced sums / sums of squares where the
    # single process uses torch.var's two-pass form — equal up to fp64 cancellation (~1e-9)
    tol = 1e-7 if bn else 1e-10
    for a, b in zip(dp["params"], model.params):
        torch.testing.assert_close(a, b.detach(), rtol=tol, atol=tol * 1e-2)
    for a, b in zip(dp["costs"], [p["cost"] for p in model.progress]):
        assert abs(a - b) < tol * max(1.0, abs(b))
    want = _bn_running(model)
    for r in range(1, world):
        dp[f"r{r}"] = torch.load(tmp_path / f"bn{r}.pt", weights_only=True)["bn"]
    for stats in [dp["bn"]] + [dp[f"r{r}"] for r in range(1, world)]:
        for (m, v), (wm, wv) in zip(stats, want):
            torch.testing.assert_close(m, wm, rtol=tol, atol=tol * 1e-2)
            torch.testing.assert_close(v, wv, rtol=tol, atol=tol * 1e-2)


def _concurrent_rank(rank, world, port, out_dir):
    """Rank 0 trains a LOCAL batchnorm model in a second thread while the group training (also
    batchnorm, synchronised over the ranks) is in flight: the local model must not pick up the
    group's synchronisation (it was a process-wide global)."""
    import threading
    os.environ.update(PZ_RENDEZVOUS_FILE=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    init_from_env("gloo")
    model, data = _dp_model("adam", True)
    local_out = {}
    started = threading.Event()

    def local():
        started.wait()
        lm, ldata = _dp_model("stochastic", True)
        lm._train_autograd(ldata, 30, 0.05, 16, 0.9, 0.0, 1e-3, context=DataParallelContext(),
                           sampler=torch.Generator().manual_seed(5))
        local_out["params"] = [p.detach().clone() for p in lm.params]
        local_out["sync"] = [getattr(l, "sync", None) for l in lm.layers if l.algo == "batchnorm"]

    t = threading.Thread(target=local) if rank == 0 else None
    if t is not None:
        t.start()
    started.set()
    model._train_autograd(data, 30, 0.05, 32, 0.9, 0.0, 1e-3, sampler=torch.Generator().manual_seed(21))
    if t is not None:
        t.join()
        torch.save({"local": local_out["params"], "sync_none": all(s is None for s in local_out["sync"]),
                    "group_cleared": all(getattr(l, "sync", None) is None for l in model.layers)},
                   os.path.join(out_dir, "conc.pt"))
    shutdown()


def test_batchnorm_sync_is_per_model_under_concurrent_training(tmp_path):
    mp.start_processes(_concurrent_rank, args=(2, str(tmp_path / "rdv"), str(tmp_path)), nprocs=2,
                       start_method="spawn")
    got = torch.load(tmp_path / "conc.pt", weights_only=True)
    assert got["sync_none"] and got["group_cleared"]
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext
    lm, ldata = _dp_model("stochastic", True)
    lm._train_autograd(ldata, 30, 0.05, 16, 0.9, 0.0, 1e-3, context=DataParallelContext(),
                       sampler=torch.Generator().manual_seed(5))
    for a, b in zip(got["local"], lm.params):  # exactly the standalone run: no foreign all-reduce
        assert torch.equal(a, b.detach())


def _native_rank(rank, world, port, out_dir):
    """The native-communicator plumbing of parallel/dist.py (unique-id broadcast from rank 0, init
    self-check, bucket tickets, reduced-precision buckets, shutdown) over gloo, with the RCCL ops of
    csrc/rccl_comm.cpp stood in by host all-reduces (the GPU tier runs the real ones)."""
    os.environ.update(PZ_RENDEZVOUS_FILE=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from penr_oz_neural_network_torch_amd.parallel import dist as pd
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    log = {"init": [], "reduced": 0, "waited": [], "closed": []}

    class FakeOps:
        @staticmethod
        def rccl_unique_id():
            return torch.arange(128, dtype=torch.uint8)

        @staticmethod
        def rccl_init(uid, nranks, r, high_priority, cu_count=0):
            log["init"].append((uid.tolist(), nranks, r, high_priority))
            return 7

        @staticmethod
        def rccl_all_reduce(h, t):
            dist.all_reduce(t)
            log["reduced"] += 1
            return log["reduced"] - 1

        @staticmethod
        def rccl_wait(h, ticket):
            log["waited"].append((h, ticket))

        @staticmethod
        def rccl_destroy(h):
            log["closed"].append(h)

    class FakeTorch:  # torch with the pz namespace swapped
        ops = type("ops", (), {"pz": FakeOps})

        def __getattr__(self, name):
            return getattr(torch, name)

    pd.torch = FakeTorch()
    ctx = init_from_env("gloo")
    ctx.native = pd._NativeComm(rank, world, device=torch.device("cpu"))
    flat = torch.arange(100, dtype=torch.float32) * (rank + 1)
    handles = [ctx.all_reduce_async(flat[50:]), ctx.all_reduce_async(flat[:50])]
    assert all(isinstance(h[0], pd._Ticket) for h in handles)
    ctx.wait_all(handles)
    ctx.comm_dtype = torch.bfloat16
    g = torch.full((8,), 0.5 * (rank + 1))
    ctx.all_reduce_(g)  # exact: stays fp32
    g2 = torch.full((8,), 0.25 * (rank + 1))
    ctx.wait_one(ctx.all_reduce_async(g2))  # through a bf16 copy
    shutdown()
    pd.torch = torch
    torch.save({"flat": flat, "g": g, "g2": g2, "log": log}, os.path.join(out_dir, f"n{rank}.pt"))


def test_native_communicator_plumbing_two_ranks(tmp_path):
    mp.start_processes(_native_rank, args=(2, str(tmp_path / "rdv"), str(tmp_path)), nprocs=2, start_method="spawn")
    for r in range(2):
        got = torch.load(tmp_path / f"n{r}.pt", weights_only=True)
        assert torch.equal(got["flat"], torch.arange(100, dtype=torch.float32) * 3)
        assert torch.equal(got["g"], torch.full((8,), 1.5)) and torch.equal(got["g2"], torch.full((8,), 0.75))
        log = got["log"]
        # rank 0's id reached both ranks; normal-priority comm stream; self-check + 4 buckets; closed
        assert log["init"] == [(list(range(128)), 2, r, False)]
        assert log["reduced"] == 5 and [t for _, t in log["waited"]] == [0, 1, 2, 3, 4]
        assert log["closed"] == [7]


def _zero_worker(rank, world, port, out_dir):
    """The sharded optimizer's collectives and slice geometry on gloo / CPU tensors: uneven
    weights over 3 ranks (a slice padded to 64 elements, a weight smaller than one slice)."""
    os.environ.update(PZ_RENDEZVOUS_FILE=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from penr_oz_neural_network_torch_amd.engine.params import Segment
    from penr_oz_neural_network_torch_amd.engine.zero import ZeroShards
    from penr_oz_neural_network_torch_amd.parallel import init_from_env, shutdown
    ctx = init_from_env("gloo")
    assert ctx.shard_world == world and ctx.shard_rank == rank
    segs = [Segment(0, "weights", 0, 1000, (40, 25), True, True, 0),
            Segment(2, "weights", 1024, 30, (5, 6), True, True, 2),
            Segment(4, "weights", 1088, 4096, (64, 64), True, True, 4)]
    z = ZeroShards(ctx, segs, 2, torch.device("cpu"))
    got = {}
    for seg in segs:
        sh = z.shards[seg.offset]
        assert sh.s % 64 == 0 and sh.s * world >= sh.n and sh.lo == rank * sh.s
        # reduce-scatter: rank r's gradient = (r + 1) * (i % 16) -> slice sum = 6 * (i % 16) (3 ranks)
        z.grad_view(seg.offset).copy_((torch.arange(sh.n, dtype=torch.float32) % 16 * (rank + 1)).view(seg.shape))
        ctx.wait_one(z.reduce_scatter(seg.offset))
        got[f"rs{seg.offset}"] = sh.g_shard[:sh.cnt].float().clone()
        # in-place all-gather of a shadow parity: every rank writes only its slice
        full = sh.sh_full[1]
        full.zero_()
        full[sh.lo:sh.lo + sh.cnt] = torch.arange(sh.lo, sh.lo + sh.cnt, dtype=torch.float32).to(full.dtype)
        ctx.wait_one(ctx.all_gather_async(full[sh.lo:sh.lo + sh.s], full))
        got[f"ag{seg.offset}"] = z.shadow_view(seg.offset, 1).float().clone()
    # gather_state: each rank's masters / moments are current on its own slices only
    flat = torch.full((1088 + 4096,), -1.0)
    m = torch.full_like(flat, -2.0)
    for seg in segs:
        sh = z.shards[seg.offset]
        flat[seg.offset + sh.lo:seg.offset + sh.lo + sh.cnt] = float(rank)
        m[seg.offset + sh.lo:seg.offset + sh.lo + sh.cnt] = float(10 + rank)
    z.gather_state(flat, m, None)
    got["flat"], got["m"] = flat, m
    got["cnt"] = [z.shards[s.offset].cnt for s in segs]
    torch.save(got, os.path.join(out_dir, f"z{rank}.pt"))
    ctx.barrier()
    shutdown()


def test_gloo_sharded_optimizer_collectives_three_ranks(tmp_path):
    world = 3
    mp.start_processes(_zero_worker, args=(world, str(tmp_path / "rdv"), str(tmp_path)), nprocs=world,
                       start_method="spawn")
    outs = [torch.load(tmp_path / f"z{r}.pt", weights_only=True) for r in range(world)]
    sizes = {0: 1000, 1024: 30, 1088: 4096}
    for off, n in sizes.items():
        s = -(-(-(-n // world)) // 64) * 64
        cov = sum(o["cnt"][list(sizes).index(off)] for o in outs)
        assert cov == n  # the slices tile the weight exactly
        for r, o in enumerate(outs):
            lo = r * s
            cnt = max(0, min(s, n - lo))
            want = torch.arange(lo, lo + cnt, dtype=torch.float32) % 16 * 6  # (1 + 2 + 3) x, exact in bf16
            assert torch.equal(o[f"rs{off}"], want)
            assert torch.equal(o[f"ag{off}"].reshape(-1), torch.arange(n, dtype=torch.float32).bfloat16().float())
            # the gathered master: each element holds its owner's rank
            owner = torch.arange(n) // s
            assert torch.equal(o["flat"][off:off + n], owner.float())
            assert torch.equal(o["m"][off:off + n], owner.float() + 10)
    for o in outs[1:]:
        assert torch.equal(o["flat"], outs[0]["flat"]) and torch.equal(o["m"], outs[0]["m"])
    # the padding between segments is untouched
    assert torch.equal(outs[0]["flat"][1000:1024], torch.full((24,), -1.0))
