"""Unit tests of the small policy / loader / communicator helpers on the CPU: precision and device
resolution (config.py), the native loader's failure reporting (ops/native.py) and the
data-parallel context's forced single-rank path over gloo (parallel/dist.py, run in a child
process so this pytest process never holds a process group)."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

from penr_oz_neural_network_torch_amd import config
from penr_oz_neural_network_torch_amd.ops import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("spec,master,compute", [
    (None, torch.float64, torch.float64), ("fp64", torch.float64, torch.float64),
    (torch.float32, torch.float32, torch.float32), ("float", torch.float32, torch.float32),
    ("BF16", torch.float32, torch.bfloat16), (torch.bfloat16, torch.float32, torch.bfloat16),
    ("e4m3", torch.float32, torch.float8_e4m3fn), ("fp8", torch.float32, torch.float8_e4m3fn)])
def test_resolve_precision(spec, master, compute):
    p = config.resolve_precision(spec)
    assert (p.master, p.compute) == (master, compute)
    assert p.mixed == (master != compute)
    assert config.resolve_precision(p) is p


def test_resolve_precision_rejects_unknown():
    with pytest.raises(ValueError, match="Unsupported dtype"):
        config.resolve_precision("int8")


def test_resolve_device(monkeypatch):
    monkeypatch.delenv("PZ_DEVICE", raising=False)
    assert config.resolve_device(None) == torch.device("cpu")
    monkeypatch.setenv("PZ_DEVICE", "cpu")
    assert config.resolve_device(None).type == "cpu"
    monkeypatch.setenv("LOCAL_RANK", "3")
    assert config.resolve_device("cuda") == torch.device("cuda", 3)  # one process per GPU
    assert config.resolve_device("cuda:1") == torch.device("cuda", 1)


def test_native_loader_reports_a_missing_library(monkeypatch, tmp_path):
    saved = dict(native._state)
    try:
        native._state.update(loaded=False, error=None, path=None)
        monkeypatch.setattr(native, "library_path", lambda: str(tmp_path / "missing.so"))
        assert native.load() is False and native.has_host_ops() is False
        assert "not built" in native.error()
        with pytest.raises(RuntimeError, match="not built"):
            native.require()
    finally:
        native._state.clear()
        native._state.update(saved)
        monkeypatch.undo()
    assert native.load() is True  # the real in-tree library
    assert native.built_sources_stale() is False  # content-hash manifest matches csrc/


def test_forced_single_rank_context_over_gloo():
    code = textwrap.dedent("""
        import os, torch
        os.environ.update(PZ_FORCE_COMM="1", PZ_DIST_BACKEND="gloo", PZ_GRAD_COMM_DTYPE="bf16")
        for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            os.environ.pop(k, None)
        from penr_oz_neural_network_torch_amd.parallel import dist as D
        ctx = D.init_from_env()
        assert ctx.force and ctx.enabled and ctx.world_size == 1 and ctx.backend == "gloo"
        assert D.get_context() is ctx and ctx.comm_dtype == torch.bfloat16
        t = torch.tensor([1.0, 2.5, -3.0])
        h = ctx.all_reduce_async(t)            # through the bf16 bucket, unpacked by wait_one
        assert h[1] is not None and h[1].dtype == torch.bfloat16
        ctx.wait_all([h, None])
        assert t.tolist() == [1.0, 2.5, -3.0]
        e = torch.tensor([0.1])
        ctx.all_reduce_(e)                     # exact path
        assert abs(e.item() - 0.1) < 1e-7
        assert ctx.all_reduce_async(torch.empty(0)) is None
        assert ctx.all_reduce_scalar(2.0) == 2.0 and ctx.all_reduce_scalar_max(5.0) == 5.0
        b = torch.tensor([7.0]); ctx.broadcast_(b); ctx.barrier()
        D.shutdown()
        assert not D.dist.is_initialized()
        off = D.DataParallelContext()
        assert not off.enabled and off.all_reduce_async(t) is None and off.all_reduce_scalar(3.0) == 3.0
        assert off.all_reduce_scalar_max(4.0) == 4.0 and off.backend is None
        off.broadcast_(t); off.barrier()
        print("dist ok")
    """)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0 and "dist ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("m,n", [(256, 256), (300, 264), (8192, 4096), (5, 1000)])
def test_relu_mask_tile_blocked_layout(m, n):
    """The tile-blocked ReLU bitmask helpers (ops/functional.py) agree with the kernels' byte
    address (csrc/gemm_epilogue.h mask_off): element (m, n) is bit n & 7 of byte
    (m >> 8) * 256 * ld + (n >> 8) * 8192 + (m & 255) * 32 + (n & 255) >> 3, and pack / unpack
    round-trip."""
    from penr_oz_neural_network_torch_amd.ops import functional as PF
    g = torch.Generator().manual_seed(m * 7 + n)
    pos = torch.rand(m, n, generator=g) > 0.5
    mask = PF.relu_mask_pack(pos)
    rows, ld = PF.relu_mask_shape(m, n)
    assert mask.shape == (rows, ld) and mask.is_contiguous() and rows % 256 == 0 and ld % 32 == 0
    assert torch.equal(PF.relu_mask_bits(mask, m, n), pos)
    flat = mask.reshape(-1)
    for _ in range(64):
        i, j = (int(torch.randint(0, m, (1,), generator=g)), int(torch.randint(0, n, (1,), generator=g)))
        off = (i >> 8) * 256 * ld + (j >> 8) * 8192 + (i & 255) * 32 + ((j & 255) >> 3)
        assert bool((int(flat[off]) >> (j & 7)) & 1) == bool(pos[i, j])


def test_collective_footprint_proxy_plumbing():
    """PZ_COMM=proxy (parallel/dist.py _ProxyComm over csrc/comm_proxy.hip): its knobs reach the
    proxy communicator, bucket all-reduces become tickets on it, shutdown closes it; and it refuses
    anything but a forced world-1 GPU run. The proxy kernel itself runs in the GPU tier
    (tests/test_dp_gpu.py forced[fp32-proxy])."""
    code = textwrap.dedent("""
        import os, torch
        from penr_oz_neural_network_torch_amd.parallel import dist as D
        log = {"init": None, "reduced": [], "closed": []}
        class FakeOps:
            @staticmethod
            def rccl_proxy_init(world, wgs, gbps, cus, hp):
                log["init"] = (world, wgs, gbps, cus, hp); return 3
            @staticmethod
            def rccl_all_reduce(h, t):
                log["reduced"].append((h, t.numel())); return len(log["reduced"]) - 1
            @staticmethod
            def rccl_wait(h, ticket):
                pass
            @staticmethod
            def rccl_destroy(h):
                log["closed"].append(h)
        class FakeTorch:
            ops = type("ops", (), {"pz": FakeOps})
            def __getattr__(self, name):
                return getattr(torch, name)
        os.environ.update(PZ_COMM_PROXY_WORLD="4", PZ_COMM_PROXY_WGS="8", PZ_COMM_PROXY_GBPS="200", PZ_COMM_CUS="8")
        D.torch = FakeTorch()
        comm = D._ProxyComm()
        assert log["init"] == (4, 8, 200.0, 8, False)
        tk = comm.all_reduce(torch.zeros(10))
        assert isinstance(tk, D._Ticket) and log["reduced"] == [(3, 10)]
        ctx = D.DataParallelContext()
        ctx.native = comm
        D.set_context(ctx)
        D.shutdown()
        assert log["closed"] == [3] and comm.handle is None
        comm.close()  # idempotent
        assert log["closed"] == [3]
        D.torch = torch
        # forced world 1 over gloo without a GPU: refused
        os.environ.update(PZ_FORCE_COMM="1", PZ_DIST_BACKEND="gloo", PZ_COMM="proxy")
        for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            os.environ.pop(k, None)
        try:
            D.init_from_env()
            raise SystemExit("proxy accepted without a GPU")
        except RuntimeError as e:
            assert "ONE GPU" in str(e)
        D.shutdown()
        print("proxy ok")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "proxy ok" in r.stdout, r.stderr[-3000:]
