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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
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
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, start_method="spawn")
    expect = torch.arange(1000, dtype=torch.float32) * 3
    for r in range(2):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.equal(got["flat"], expect)
        assert torch.equal(got["rep"], torch.zeros(7))
        assert got["max"] == 1.5 and got["sum"] == 2.0
        assert torch.allclose(got["bf16"], torch.full((64,), 1.5))
