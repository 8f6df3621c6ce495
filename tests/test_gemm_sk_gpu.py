"""The persistent stream-K GEMM engine (csrc/gemm_sk.hip) against fp64 torch references: every
layout and epilogue kind the trainer runs, at CU budgets that give pure data-parallel tiles
(256), a two-tile stream-K region (240, 200) and tiles far outnumbering the workgroups (37), plus
bit-for-bit determinism of the stream-K fold (run on MI355X)."""
import math

import pytest
import torch

from penr_oz_neural_network_torch_amd.ops import functional as PF
from tests.helpers import keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"
CUS = [256, 240, 200, 37]


def _ops(M, N, K, a_kc, b_kc, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    a = (torch.rand((M, K) if a_kc else (K, M), generator=g) * 2 - 1).to(DEV, torch.bfloat16)
    b = (torch.rand((N, K) if b_kc else (K, N), generator=g) * 2 - 1).to(DEV, torch.bfloat16)
    ref = (a.double() if a_kc else a.double().t()) @ (b.double().t() if b_kc else b.double())
    return a, b, ref


def _close(out, ref, K, rel=0.01):
    err = (out.double() - ref).abs().max().item()
    assert err <= rel * ref.abs().max().item() + 1e-3 * math.sqrt(K), err


@pytest.mark.parametrize("cus", CUS)
@pytest.mark.parametrize("layout", ["fwd", "dx", "dw"])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_sk_plain_store(native_lib, layout, cus, out_dtype):
    a_kc, b_kc = {"fwd": (True, False), "dx": (True, True), "dw": (False, False)}[layout]
    if out_dtype == torch.float32 and layout != "dw":
        pytest.skip("fp32 outputs: the weight-gradient layout")
    M, N, K = (2048, 2048, 512) if layout != "dw" else (1024, 2048, 1024)
    a, b, ref = _ops(M, N, K, a_kc, b_kc, cus + M)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=out_dtype)
    PF.gemm(a, a_kc, b, b_kc, out, engine=2, cus=cus)
    _close(out, ref, K, 0.01 if out_dtype == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("cus", CUS)
@pytest.mark.parametrize("kind", ["relu_post", "relu_prepost", "pre", "relu_nodrop", "tanh"])
def test_sk_forward_epilogues(native_lib, kind, cus):
    """bias + dropout / activation / dropout of the forward stage, the ReLU bitmask it writes."""
    M, N, K = 1536, 1024, 768
    p, seed = 0.2, (4321, 77)
    x, w, h = _ops(M, N, K, True, False, 17 + cus)
    bias = torch.randn(N, device=DEV)
    h = h + bias.double()
    act = {"relu_post": "relu", "relu_prepost": "relu", "pre": None, "relu_nodrop": "relu", "tanh": "tanh"}[kind]
    pre = kind in ("relu_prepost", "pre", "tanh")
    post = kind in ("relu_post", "relu_prepost", "tanh")
    epi = PF.epi_spec(act=PF.ACT_CODES[act], drop_pre=3 if pre else -1, drop_post=4 if post else -1, p=p, seed=seed)
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 3, p).reshape(M, N)).to(DEV).double() / (1 - p)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 4, p).reshape(M, N)).to(DEV).double() / (1 - p)
    z = h * m1 if pre else h
    z = {"relu": torch.relu, "tanh": torch.tanh, None: lambda t: t}[act](z)
    ref = z * m2 if post else z
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    mask = PF.relu_mask_empty(M, N, device=DEV) if act == "relu" else None
    PF.gemm(x, True, w, False, out, bias=bias, mode=PF.EPI_FWD, epi=epi, mask=mask, engine=2, cus=cus)
    _close(out, ref, K, 0.02)
    if mask is not None:
        assert torch.equal(PF.relu_mask_bits(mask, M, N), out > 0)


@pytest.mark.parametrize("cus", CUS)
@pytest.mark.parametrize("use_mask", [True, False])
def test_sk_backward_epilogues_and_colsum(native_lib, use_mask, cus):
    """dX = dZ · Wᵀ through the previous stage's dropout-ReLU-dropout derivative (from its bitmask,
    or from its stored output), with the bias-gradient column sums."""
    M, N, K = 2048, 1280, 512
    p, seed = 0.25, (99, 7)
    g, w, gx = _ops(M, N, K, True, True, 5 + cus)
    y = torch.randn(M, N, device=DEV).to(torch.bfloat16)  # stored stage output (its sign = the ReLU bit)
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 1, p).reshape(M, N)).to(DEV).double() / (1 - p)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 2, p).reshape(M, N)).to(DEV).double() / (1 - p)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=p, seed=seed)
    if use_mask:
        # bitmask epilogue: y > 0 already encodes both keep decisions; the derivative is bit * s^2
        mask = PF.relu_mask_empty(M, N, device=DEV)
        bits = torch.rand(M, N, device=DEV) < 0.6
        ymask = torch.where(bits, torch.ones_like(y), -torch.ones_like(y))
        PF.gemm(torch.eye(M, device=DEV, dtype=torch.bfloat16), True, ymask.t().contiguous(), True,
                torch.empty(M, N, device=DEV, dtype=torch.bfloat16), mode=PF.EPI_FWD,
                epi=PF.epi_spec(act=PF.ACT_RELU), mask=mask, engine=1)
        assert torch.equal(PF.relu_mask_bits(mask, M, N), bits)
        ref = gx * bits.double() / (1 - p) ** 2
        kw = dict(mask=mask)
    else:
        ref = gx * m2 * (y > 0).double() * m1  # drop_post' * relu'(y / s) * drop_pre'
        kw = dict(aux=y)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    colsum = torch.zeros(N, device=DEV)
    PF.gemm(g, True, w, True, out, colsum=colsum, mode=PF.EPI_BWD, epi=epi, engine=2, cus=cus, **kw)
    _close(out, ref, K, 0.02)
    # the sums of the fp32 epilogue values (before the bf16 store): against the fp64 reference
    cs_ref = ref.sum(0)
    assert (colsum.double() - cs_ref).abs().max().item() <= 1e-4 * ref.abs().sum(0).max().item()


@pytest.mark.parametrize("shape,cus", [((8192, 1024, 4096), 256), ((4096, 1024, 8192), 256), ((2048, 4096, 1024), 96)])
def test_sk_stream_k_fold_is_deterministic(native_lib, shape, cus):
    """Stream-K tiles split over two contributors (K halves on 2T workgroups, or the two-tile
    region): bit-identical across runs, whichever workgroup arrives last."""
    M, N, K = shape
    a, b, ref = _ops(M, N, K, True, False, 3)
    outs = []
    for _ in range(3):
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        PF.gemm(a, True, b, False, out, engine=2, cus=cus)
        outs.append(out)
    _close(outs[0], ref, K)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_sk_matches_tiled_engine_bitwise_on_whole_tiles(native_lib):
    """Pure data-parallel tiles (512 tiles on 256 workgroups) accumulate in the same K order as the
    tiled kernels: identical bits."""
    M, N, K = 8192, 4096, 1024
    a, b, _ = _ops(M, N, K, True, False, 11)
    o1 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    PF.gemm(a, True, b, False, o1, engine=1)
    PF.gemm(a, True, b, False, o2, engine=2, cus=256)
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("engine,cus", [(1, 0), (2, 256), (2, 200)])
def test_bias_gradient_colsums_are_deterministic(native_lib, engine, cus):
    """PZ_DETERMINISTIC (default): the backward epilogue's bias-gradient column sums are folded in
    tile-row order (pz_common.h det_colsum), not in atomic arrival order — bit-identical across runs,
    on the tiled and the stream-K engines, and equal to the fp64 column sums of the stored dX."""
    M, N, K = 8192, 4096, 1024
    g, w, _ = _ops(M, N, K, True, True, 21)
    mask = PF.relu_mask_empty(M, N, device=DEV)
    mask.random_(0, 256)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=0.1, seed=(3, 4))
    outs = []
    for _ in range(3):
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        colsum = torch.zeros(N, device=DEV)
        PF.gemm(g, True, w, True, out, colsum=colsum, mode=PF.EPI_BWD, epi=epi, mask=mask, engine=engine, cus=cus)
        outs.append((out, colsum))
    assert all(torch.equal(outs[0][1], o[1]) and torch.equal(outs[0][0], o[0]) for o in outs[1:])
    # (the bf16 store rounds each element: compare the fp32 sums with a bound on that rounding)
    ref = outs[0][0].double()
    err = (outs[0][1].double() - ref.sum(0)).abs().max().item()
    assert err <= 2 ** -8 * ref.abs().sum(0).max().item(), err


@pytest.mark.parametrize("B,C", [(8192, 1024), (4096, 2048)])
def test_head_colsums_are_deterministic(native_lib, B, C):
    """The lean bf16 cross-entropy head's bias-gradient sums: partial rows of 32-row blocks folded
    in block order over two ticketed levels — bit-identical across runs, close to fp64."""
    logits = (torch.randn(B, C, device=DEV) * 2).to(torch.bfloat16)
    labels = torch.randint(0, C, (B,), device=DEV)
    ei, ef = PF.epi_spec(drop_pre=4, p=0.1, seed=(1, 9))
    sums = []
    for _ in range(3):
        loss, colsum = torch.zeros(1, device=DEV), torch.zeros(C, device=DEV)
        dh = torch.empty(B, C, device=DEV, dtype=torch.bfloat16)
        torch.ops.pz.xent_head(logits, labels, B, loss, 1.0 / B, dh, 1.0 / B, colsum, None, ei, ef, C)
        sums.append((colsum, dh))
    assert all(torch.equal(sums[0][0], s[0]) for s in sums[1:])
    ref = (torch.softmax(logits.double(), 1) - torch.nn.functional.one_hot(labels, C)) / B
    ref = ref * torch.from_numpy(keep_mask(B * C, 1, 9, 4, 0.1).reshape(B, C)).to(DEV) / 0.9
    assert (sums[0][0].double() - ref.sum(0)).abs().max().item() <= 1e-3 * ref.abs().max().item() * math.sqrt(B)


def test_sk_lab_engine_is_not_in_the_library(native_lib):
    """engine 3 (the round-5 4-wave lab loop) moved to tools/gemm_w4_lab.hip: the library refuses
    it loudly instead of silently running another engine."""
    M, N, K = 512, 512, 256
    a, b, _ = _ops(M, N, K, True, False, 5)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="stream-K engine cannot run"):
        PF.gemm(a, True, b, False, out, engine=3)


@pytest.mark.parametrize("cus", [256, 240, 100])
def test_sk_two_problem_schedule(native_lib, cus):
    """Two weight-gradient GEMMs (the first layer's and the last layer's) as ONE persistent
    stream-K schedule: the second problem's tiles follow the first's; both against fp64."""
    K = 4096
    a0, b0, r0 = _ops(1024, 2048, K, False, False, 31)
    a1, b1, r1 = _ops(2048, 1024, K, False, False, 32)
    o0 = torch.full((1024, 2048), float("nan"), device=DEV)
    o1 = torch.full((2048, 1024), float("nan"), device=DEV)
    PF.gemm_pair(a0, b0, o0, a1, b1, o1, engine=2, cus=cus)
    _close(o0, r0, K, 1e-5)
    _close(o1, r1, K, 1e-5)
