"""fp64 / fp32 GEMMs on the gfx950 matrix cores (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32,
csrc/gemm_wide.hip) against fp64 host references, every operand layout, ragged shapes, and the
fused-epilogue contract against the generic VALU kernel."""
import pytest
import torch

from penr_oz_neural_network_torch_amd.ops import functional as PF
from tests.helpers import keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _operands(M, N, K, a_kc, b_kc, dtype, seed):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn((M, K) if a_kc else (K, M), generator=g, dtype=torch.float64)
    b = torch.randn((N, K) if b_kc else (K, N), generator=g, dtype=torch.float64)
    return a.to(DEV, dtype), b.to(DEV, dtype)


def _ref(a, a_kc, b, b_kc):
    A = a.double().cpu() if a_kc else a.double().cpu().t()
    B = b.double().cpu().t() if b_kc else b.double().cpu()
    return A @ B, A.abs() @ B.abs()


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("shape", [(512, 384, 256), (300, 264, 200), (1024, 96, 1000), (129, 131, 16)])
def test_gemm_fp64_matrix_cores_exact(native_lib, a_kc, b_kc, shape):
    """fp64 fma chains: within 1e-12 of an fp64 host GEMM, relative to sum |a||b|."""
    M, N, K = shape
    a, b = _operands(M, N, K, a_kc, b_kc, torch.float64, M * 7 + N + K)
    out = torch.empty(M, N, device=DEV, dtype=torch.float64)
    assert PF.gemm_path(a, a_kc, b, b_kc, out) == "mfma_wide"
    PF.gemm(a, a_kc, b, b_kc, out)
    ref, scale = _ref(a, a_kc, b, b_kc)
    rel = ((out.cpu() - ref).abs() / scale.clamp_min(1e-300)).max().item()
    assert rel < 1e-12, rel


@pytest.mark.parametrize("a_kc,b_kc", [(True, False), (False, False), (True, True)])
def test_gemm_fp32_matrix_cores(native_lib, a_kc, b_kc):
    M, N, K = 640, 320, 1024
    a, b = _operands(M, N, K, a_kc, b_kc, torch.float32, 11)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    assert PF.gemm_path(a, a_kc, b, b_kc, out) == "mfma_wide"
    PF.gemm(a, a_kc, b, b_kc, out)
    ref, scale = _ref(a, a_kc, b, b_kc)
    rel = ((out.double().cpu() - ref).abs() / scale).max().item()
    assert rel < 2e-6, rel


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_gemm_wide_epilogues_match_generic(native_lib, dtype):
    """bias + dropout + ReLU + dropout forward, derivative-from-output backward with column
    sums, and accumulate: the MFMA kernel and the generic VALU kernel agree element for element."""
    M, N, K = 384, 200, 96
    p, seed = 0.25, (321, 9)
    x, w = _operands(M, N, K, True, False, dtype, 5)
    bias = torch.randn(N, device=DEV)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=3, drop_post=4, p=p, seed=seed)
    outs = []
    for force in (False, True):
        out = torch.empty(M, N, device=DEV, dtype=dtype)
        PF.gemm(x, True, w, False, out, bias=bias, mode=PF.EPI_FWD, epi=epi, force_generic=force)
        outs.append(out)
    tol = 1e-12 if dtype == torch.float64 else 1e-4
    assert (outs[0] - outs[1]).abs().max().item() < tol * outs[1].abs().max().item()
    # reference semantics of the forward stage
    h = x.double() @ w.double() + bias.double()
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 3, p).reshape(M, N)).to(DEV)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 4, p).reshape(M, N)).to(DEV)
    ref = torch.relu(h * m1 / (1 - p)) * m2 / (1 - p)
    # (the stage's dropout scale 1/(1-p) is an fp32 constant of the epilogue spec: ~6e-8 relative)
    assert (outs[0].double() - ref).abs().max().item() < max(tol, 2e-7) * ref.abs().max().item()
    # backward stage: dZ = epi_bwd(g_a @ Wᵀ, y) with column sums
    ga, wt = _operands(M, K, N, True, True, dtype, 8)  # [M, N] and [K, N]: dX = ga @ wtᵀ -> [M, K]
    y = torch.tanh(torch.randn(M, K, device=DEV, dtype=dtype))
    bepi = PF.epi_spec(act=PF.ACT_TANH, drop_pre=1, drop_post=2, p=p, seed=seed)
    res = []
    for force in (False, True):
        out = torch.empty(M, K, device=DEV, dtype=dtype)
        cs = torch.zeros(K, device=DEV)
        PF.gemm(ga, True, wt, True, out, aux=y, colsum=cs, mode=PF.EPI_BWD, epi=bepi, force_generic=force)
        res.append((out, cs))
    assert (res[0][0] - res[1][0]).abs().max().item() < tol * res[1][0].abs().max().item() + 1e-300
    assert (res[0][1] - res[1][1]).abs().max().item() < 1e-3 * res[1][1].abs().max().item()
    # accumulate: C += A @ B
    c0 = torch.randn(M, N, device=DEV, dtype=dtype)
    c = c0.clone()
    PF.gemm(x, True, w, False, c, accumulate=True)
    ref = c0.double() + x.double() @ w.double()
    assert (c.double() - ref).abs().max().item() < tol * ref.abs().max().item() * 10
