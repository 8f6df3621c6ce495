"""Numerics of every HIP kernel against plain PyTorch fp32/fp64 references (run on MI355X)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from penr_oz_neural_network_torch_amd.ops import functional as PF
from tests.helpers import keep_mask

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_mm(a, a_kc, b, b_kc):
    A = a.double() if a_kc else a.double().t()
    B = b.double().t() if b_kc else b.double()
    return A @ B


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("shape", [(512, 384, 256), (1024, 512, 128), (300, 264, 192), (8192, 1024, 128)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm_mfma_layouts(native_lib, a_kc, b_kc, shape, out_dtype):
    M, N, K = shape
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn((M, K) if a_kc else (K, M), generator=g).to(DEV, torch.bfloat16)
    b = torch.randn((N, K) if b_kc else (K, N), generator=g).to(DEV, torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=out_dtype)
    if M % 8 == 0 or a_kc:
        assert PF.gemm_path(a, a_kc, b, b_kc, out) == "mfma"
    PF.gemm(a, a_kc, b, b_kc, out)
    ref = _ref_mm(a, a_kc, b, b_kc)
    err = (out.double() - ref).abs().max().item()
    tol = 1e-3 * math.sqrt(K) + (0.02 * ref.abs().max().item() if out_dtype == torch.bfloat16 else 0)
    assert err < tol, err


def test_gemm_identity_asymmetric(native_lib):
    # A = I with an asymmetric B catches a transposed C write (guide §3)
    n = 256
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n) % 97).to(torch.bfloat16)
    for b_kc in (True, False):
        out = torch.empty(n, n, device=DEV, dtype=torch.float32)
        PF.gemm(a, True, b, b_kc, out)
        ref = b.float().t() if b_kc else b.float()
        assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.bfloat16])
def test_gemm_generic_small(native_lib, dtype):
    M, N, K = 37, 19, 23
    a = torch.randn(M, K, device=DEV, dtype=dtype)
    b = torch.randn(K, N, device=DEV, dtype=dtype)
    bias = torch.randn(N, device=DEV, dtype=torch.float32)
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    assert PF.gemm_path(a, True, b, False, out) == "generic"
    PF.gemm(a, True, b, False, out, bias=bias)
    ref = a.double() @ b.double() + bias.double()
    tol = {torch.float64: 1e-12, torch.float32: 1e-4, torch.bfloat16: 0.15}[dtype]
    assert (out.double() - ref).abs().max().item() < tol


@pytest.mark.parametrize("force_generic", [False, True])
def test_gemm_fused_forward_epilogue(native_lib, force_generic):
    M, N, K = 512, 256, 128
    p = 0.3
    seed = (12345, 678)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, N, device=DEV) / 8).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=3, drop_post=4, p=p, seed=seed)
    PF.gemm(x, True, w, False, out, bias=bias, mode=PF.EPI_FWD, epi=epi, force_generic=force_generic)
    h = x.double() @ w.double() + bias.double()
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 3, p).reshape(M, N)).to(DEV)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 4, p).reshape(M, N)).to(DEV)
    ref = torch.relu(h * m1 / (1 - p)) * m2 / (1 - p)
    assert (out.double() - ref).abs().max().item() < 0.05 * ref.abs().max().item()
    assert abs(m1.float().mean().item() - (1 - p)) < 0.01


@pytest.mark.parametrize("act", ["relu", "sigmoid", "tanh"])
def test_gemm_backward_epilogue_and_colsum(native_lib, act):
    M, N, K = 256, 128, 192
    p = 0.25
    seed = (99, 7)
    code = PF.ACT_CODES[act]
    z = torch.randn(M, N, device=DEV, dtype=torch.float64)
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 1, p).reshape(M, N)).to(DEV)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 2, p).reshape(M, N)).to(DEV)
    fn = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}[act]
    z.requires_grad_()
    y = fn(z * m1 / (1 - p)) * m2 / (1 - p)
    gy_a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    gy = gy_a.double() @ w.double().t()  # dY = gA @ Wᵀ (W stored [N,K] = [out,in]ᵀ layout)
    y.backward(gy)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    colsum = torch.zeros(N, device=DEV)
    epi = PF.epi_spec(act=code, drop_pre=1, drop_post=2, p=p, seed=seed)
    PF.gemm(gy_a, True, w, True, out, aux=y.detach().float(), colsum=colsum, mode=PF.EPI_BWD, epi=epi)
    ref = z.grad
    assert (out.double() - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-4
    assert (colsum.double() - out.double().sum(0)).abs().max().item() < 1e-3
    # MFMA path: bf16 stage output as aux (derivatives then carry bf16 rounding of y)
    out16 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y16 = y.detach().to(torch.bfloat16)
    assert PF.gemm_path(gy_a, True, w, True, out16) == "mfma"
    PF.gemm(gy_a, True, w, True, out16, aux=y16, mode=PF.EPI_BWD, epi=epi)
    assert (out16.double() - ref).abs().max().item() < 0.03 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 128), (8192, 1024, 2048)])
@pytest.mark.parametrize("act,pre,post", [("relu", False, True), ("relu", True, True), ("none", True, False)])
def test_gemm_fixed_forward_kinds(native_lib, M, N, K, act, pre, post):
    """The compile-time forward epilogues (EK_F_*: the trainer's stage-0, hidden and logits stages)
    on shapes that take the 256x256 64-deep-ring kernel (the second one split-K) == fp64 torch with
    the kernels' keep masks; ReLU stages also write the bitmask of y > 0."""
    p, seed = 0.2, (21, 4)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, N, device=DEV) / 8).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    relu = act == "relu"
    mask = torch.zeros(PF.relu_mask_shape(M, N), device=DEV, dtype=torch.uint8) if relu else None
    epi = PF.epi_spec(act=PF.ACT_RELU if relu else PF.ACT_NONE, drop_pre=3 if pre else -1,
                      drop_post=4 if post else -1, p=p, seed=seed)
    assert PF.gemm_path(x, True, w, False, y) == "mfma"
    PF.gemm(x, True, w, False, y, bias=bias, mode=PF.EPI_FWD, epi=epi, mask=mask)
    ref = x.double() @ w.double() + bias.double()
    if pre:
        ref = ref * torch.from_numpy(keep_mask(M * N, *seed, 3, p).reshape(M, N)).to(DEV) / (1 - p)
    if relu:
        ref = torch.relu(ref)
    if post:
        ref = ref * torch.from_numpy(keep_mask(M * N, *seed, 4, p).reshape(M, N)).to(DEV) / (1 - p)
    err = (y.double() - ref).abs()
    assert err.max().item() < 1e-2 * ref.abs().max().item(), err.max().item()
    assert torch.equal(y == 0, ref == 0) or (y == 0).ne(ref == 0).double().mean().item() < 1e-5
    if relu:
        assert torch.equal(PF.relu_mask_bits(mask, M, N), y.float() > 0)


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (8192 + 64, 1024 + 64, 256), (256, 4096, 64)])
def test_gemm_relu_bitmask_forward_and_backward(native_lib, M, N, K):
    """EPI_FWD writes bit(y > 0); EPI_BWD reading those bits == EPI_BWD reading y."""
    p, seed = 0.2, (5, 11)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, N, device=DEV) / 8).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    mask = torch.full(PF.relu_mask_shape(M, N), 0xAB, device=DEV, dtype=torch.uint8)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=3, drop_post=4, p=p, seed=seed)
    PF.gemm(x, True, w, False, y, bias=bias, mode=PF.EPI_FWD, epi=epi, mask=mask)
    assert torch.equal(PF.relu_mask_bits(mask, M, N), y.float() > 0)
    # backward: dX = dZ @ Wᵀ with the ReLU derivative from the bits vs from y
    gz = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wt = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    out_aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out_bit = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    cs_aux = torch.zeros(N, device=DEV)
    cs_bit = torch.zeros(N, device=DEV)
    PF.gemm(gz, True, wt, True, out_aux, aux=y, colsum=cs_aux, mode=PF.EPI_BWD, epi=epi)
    PF.gemm(gz, True, wt, True, out_bit, colsum=cs_bit, mode=PF.EPI_BWD, epi=epi, mask=mask)
    # the bit path folds both dropout scales into one multiply: equal up to one bf16 rounding
    torch.testing.assert_close(out_bit.float(), out_aux.float(), rtol=8e-3, atol=1e-6)
    torch.testing.assert_close(cs_aux, cs_bit, rtol=1e-4, atol=1e-3)
    ref = (gz.double() @ wt.double().t()) * (y.double() > 0)
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 3, p).reshape(M, N)).to(DEV)
    ref = ref * m1 / (1 - p) * (torch.from_numpy(keep_mask(M * N, *seed, 4, p).reshape(M, N)).to(DEV) / (1 - p))
    assert (out_bit.double() - ref).abs().max().item() < 0.02 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 128), (4096, 4096, 320), (8192, 4096, 1024)])
def test_gemm_w4_dx_engine(native_lib, M, N, K):
    """VAR 40 (csrc/gemm_w4.h: 4-wave LDS-DMA kernel for the dX layout, whole 256-tiles that fill
    the CUs): plain store and the ReLU-bitmask backward epilogue with column sums == fp64 torch, at
    the minimum two K steps, an odd step count and the mlp4 dX_L3 shape."""
    p, seed = 0.2, (7, 9)
    g = torch.Generator(device="cpu").manual_seed(M + K)
    gz = torch.randn(M, K, generator=g).to(DEV, torch.bfloat16)
    wt = torch.randn(N, K, generator=g).to(DEV, torch.bfloat16)
    ref = gz.double() @ wt.double().t()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    PF.gemm(gz, True, wt, True, out)
    assert (out.double() - ref).abs().max().item() < 1e-3 * math.sqrt(K) + 0.01 * ref.abs().max().item()
    yb = torch.randn(M, N, generator=g).to(DEV) > 0
    mask = PF.relu_mask_pack(yb)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=p, seed=seed)
    cs = torch.zeros(N, device=DEV)
    PF.gemm(gz, True, wt, True, out, colsum=cs, mode=PF.EPI_BWD, epi=epi, mask=mask)
    refb = ref * yb.double() / (1 - p) ** 2
    assert (out.double() - refb).abs().max().item() < 0.01 * refb.abs().max().item()
    assert (cs.double() - out.double().sum(0)).abs().max().item() < 2e-3 * out.double().abs().sum(0).max().item()


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (8192, 8192, 1024), (300, 264, 192)])
def test_gemm_fp8_e5m2_backward(native_lib, M, N, K):
    """Backward dX of the fp8 policy: e5m2 gradient x e4m3 weight (v_mfma_scale_f32_32x32x64_f8f6f4
    with mixed formats) + dequant scales + the ReLU-bitmask derivative / dropout scales + bias-grad
    column sums, against an fp64 reference on the same e5m2 / e4m3 values; and the e5m2 quantiser."""
    p, seed = 0.2, (5, 6)
    g = torch.randn(M, K, device=DEV) * 1e-3                       # dZ (bf16 in the trainer)
    gb = g.to(torch.bfloat16)
    qs = torch.tensor([57344.0 / (2 * gb.float().abs().max().item()), 0.0], device=DEV)
    qs[1] = 1.0 / qs[0]
    g8 = torch.empty(M, K, device=DEV, dtype=torch.float8_e5m2)
    amax = torch.zeros(1, device=DEV)
    torch.ops.pz.quantize_rows(gb, g8, qs, amax)
    assert amax.item() == gb.float().abs().max().item()
    exp8 = (gb.float() * qs[0]).to(torch.float8_e5m2)
    assert (g8.view(torch.uint8) != exp8.view(torch.uint8)).float().mean().item() < 1e-4
    w8 = (torch.randn(N, K, device=DEV) * 8).to(torch.float8_e4m3fn)  # W stored [in, out] = B[n][k]
    sb = torch.tensor([1.0 / 16], device=DEV)
    y = torch.relu(torch.randn(M, N, device=DEV)).to(torch.bfloat16)
    yb = y.float() > 0 if N % 8 == 0 else None
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    colsum = torch.zeros(N, device=DEV)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=p, seed=seed)
    if yb is not None:  # the trainer's form: ReLU bitmask written by the forward
        mask = PF.relu_mask_pack(yb)
        assert torch.equal(PF.relu_mask_bits(mask, M, N), yb)
        PF.gemm(g8, True, w8, True, out, colsum=colsum, mode=PF.EPI_BWD, epi=epi, mask=mask, scale_a=qs[1:2],
                scale_b=sb)
    else:
        PF.gemm(g8, True, w8, True, out, aux=y, colsum=colsum, mode=PF.EPI_BWD, epi=epi, scale_a=qs[1:2], scale_b=sb)
    h = (g8.double() @ w8.double().t()) * (qs[1].double() / 16)
    scale = 1.0 / (1 - p) ** 2  # relu' x both dropout scales (y > 0 implies kept by both)
    ref = h * (y.double() > 0) * scale
    err = (out.double() - ref).abs().max().item()
    assert err < 0.01 * ref.abs().max().item(), err
    assert (colsum.double() - out.double().sum(0)).abs().max().item() < 2e-3 * out.double().abs().sum(0).max().item()
    # the fp8 product itself tracks the exact fp64 GEMM of the unquantised operands
    exact = (gb.double() @ (w8.double().t() / 16)) * (y.double() > 0) * scale
    assert (out.double() - exact).abs().max().item() < 0.15 * exact.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (8192, 1024, 8192), (1024, 8192, 8192)])
def test_gemm_fp8_weight_gradient(native_lib, M, N, K):
    """fp8 dW (BASELINE config 5): dW[in, out] = X8ᵀ dZ8 with e4m3 activations X8 [K=batch, M] and
    e5m2 output gradients dZ8 [K, N], BOTH M/N-contiguous (transposing 8-bit LDS reads, no
    transposed copies), dequant scales, bf16 output; the skinny shapes run split-K. Checked
    against fp64 on the same quantised values."""
    x8 = (torch.randn(K, M, device=DEV) * 4).to(torch.float8_e4m3fn)
    g8 = (torch.randn(K, N, device=DEV) * 1000).to(torch.float8_e5m2)
    sa = torch.tensor([0.25], device=DEV)
    sb = torch.tensor([1.0 / 4096], device=DEV)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    assert PF.gemm_path(x8, False, g8, False, out) == "mfma"
    PF.gemm(x8, False, g8, False, out, scale_a=sa, scale_b=sb)
    ref = (x8.double().t() @ g8.double()) * (0.25 / 4096)
    err = (out.double() - ref).abs()
    # bf16 output rounding (2^-8 relative) on top of the MFMA's accumulation error, which is
    # absolute, relative to Σ|x||g|: measured ~2^-16 of it on elements that cancel to ~0 (the
    # f8f6f4 dot product of 64 terms is not an fp32-exact sum); 2^-12 bounds it, while a layout
    # or scale bug errs by O(|ref|) ~ Σ|x||g| / sqrt(K)
    mag = (x8.double().abs().t() @ g8.double().abs()) * (0.25 / 4096)
    bound = 2.0 ** -8 * ref.abs() + 2.0 ** -12 * mag
    assert (err <= bound).all(), (err - bound).max().item()
    assert err.max().item() <= 2.0 ** -8 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (4096 + 64, 4096, 512), (256, 1024, 8192), (4096, 4096, 512)])
def test_gemm_fp8_forward(native_lib, M, N, K):
    """e4m3 x e4m3 (v_mfma_scale_f32_32x32x64_f8f6f4) + dequant scales + fused stage epilogue +
    e4m3 copy of the output + amax, against an fp32 reference on the same e4m3 values."""
    f8 = torch.float8_e4m3fn
    p, seed = 0.1, (3, 4)
    x8 = (torch.randn(M, K, device=DEV) * 4).to(f8)
    w8 = (torch.randn(N, K, device=DEV) * 2).to(f8)        # weights stored [out, in] (K-contiguous)
    sa = torch.tensor([0.125], device=DEV)
    sb = torch.tensor([1.0 / 64], device=DEV)
    bias = torch.randn(N, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y8 = torch.empty(M, N, device=DEV, dtype=f8)
    qs = torch.tensor([8.0], device=DEV)
    amax = torch.zeros(1, device=DEV)
    mask = PF.relu_mask_empty(M, N, device=DEV)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=p, seed=seed)
    assert PF.gemm_path(x8, True, w8, True, y) == "mfma"
    PF.gemm(x8, True, w8, True, y, bias=bias, mode=PF.EPI_FWD, epi=epi, scale_a=sa, scale_b=sb, out8=y8,
            out8_qscale=qs, amax=amax, mask=mask)
    h = (x8.double() @ w8.double().t()) * (0.125 / 64) + bias.double()
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 1, p).reshape(M, N)).to(DEV)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 2, p).reshape(M, N)).to(DEV)
    ref = torch.relu(h * m1 / (1 - p)) * m2 / (1 - p)
    err = (y.double() - ref).abs().max().item()
    assert err < 0.01 * ref.abs().max().item(), err
    yf = y.float()
    assert amax.item() == yf.abs().max().item()
    exp8 = (yf * 8.0).clamp(-448, 448).to(f8)
    assert (y8.view(torch.uint8) != exp8.view(torch.uint8)).float().mean().item() < 1e-4
    assert torch.equal(PF.relu_mask_bits(mask, M, N), yf > 0)
    # store_c=False (the fp8 policy's unread bf16 outputs): C untouched, side outputs identical
    y_skip = torch.full_like(y, 7.0)
    y8_skip, mask_skip, amax_skip = torch.empty_like(y8), torch.empty_like(mask), torch.zeros(1, device=DEV)
    PF.gemm(x8, True, w8, True, y_skip, bias=bias, mode=PF.EPI_FWD, epi=epi, scale_a=sa, scale_b=sb, out8=y8_skip,
            out8_qscale=qs, amax=amax_skip, mask=mask_skip, store_c=False)
    assert (y_skip == 7.0).all()
    assert torch.equal(y8_skip.view(torch.uint8), y8.view(torch.uint8))
    assert torch.equal(PF.relu_mask_bits(mask_skip, M, N), PF.relu_mask_bits(mask, M, N))
    assert amax_skip.item() == amax.item()


@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (4096 + 64, 1024, 512), (8192, 8192, 1024), (8192, 1024, 8192)])
def test_gemm_fp8_forward_natural_weights(native_lib, M, N, K):
    """fp8 forward on the [in, out] e4m3 weights (B N-contiguous, transposing 8-bit LDS reads;
    256x256 tiles, ragged M, split-K on the skinny shape) with the fused stage epilogue == the same
    GEMM on the transposed [out, in] copy."""
    f8 = torch.float8_e4m3fn
    p, seed = 0.1, (3, 4)
    x8 = (torch.randn(M, K, device=DEV) * 4).to(f8)
    w8n = (torch.randn(K, N, device=DEV) * 2).to(f8)            # [in, out]
    w8t = w8n.t().contiguous()                                   # [out, in]
    sa, sb = torch.tensor([0.125], device=DEV), torch.tensor([1.0 / 64], device=DEV)
    bias = torch.randn(N, device=DEV)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=p, seed=seed)
    outs = []
    for w, kc in ((w8n, False), (w8t, True)):
        y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        y8 = torch.empty(M, N, device=DEV, dtype=f8)
        mask = PF.relu_mask_empty(M, N, device=DEV)
        amax = torch.zeros(1, device=DEV)
        assert PF.gemm_path(x8, True, w, kc, y) == "mfma"
        PF.gemm(x8, True, w, kc, y, bias=bias, mode=PF.EPI_FWD, epi=epi, scale_a=sa, scale_b=sb, out8=y8,
                out8_qscale=torch.tensor([8.0], device=DEV), amax=amax, mask=mask)
        outs.append((y, y8, mask, amax))
    (y, y8, mask, amax), (yt, y8t, maskt, amaxt) = outs
    h = (x8.double() @ w8n.double()) * (0.125 / 64) + bias.double()
    m1 = torch.from_numpy(keep_mask(M * N, *seed, 1, p).reshape(M, N)).to(DEV)
    m2 = torch.from_numpy(keep_mask(M * N, *seed, 2, p).reshape(M, N)).to(DEV)
    ref = torch.relu(h * m1 / (1 - p)) * m2 / (1 - p)
    assert (y.double() - ref).abs().max().item() < 0.01 * ref.abs().max().item()
    torch.testing.assert_close(y.float(), yt.float(), rtol=2 ** -7, atol=1e-3 * ref.abs().max().item())
    assert (y8.view(torch.uint8) != y8t.view(torch.uint8)).float().mean().item() < 1e-3
    assert (PF.relu_mask_bits(mask, M, N) != PF.relu_mask_bits(maskt, M, N)).float().mean().item() < 1e-3
    assert abs(amax.item() - amaxt.item()) <= 2 ** -7 * amaxt.item()


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 2048), (8192, 4096, 4096)])
def test_gemm_w4_fp8_forward_plain(native_lib, M, N, K):
    """VAR 43 (csrc/gemm_w4.h, plain stores, K >= 2048): e4m3 activations x the [in, out] e4m3 weights
    == fp64 torch on the same fp8 values with the per-tensor scales applied."""
    g = torch.Generator(device="cpu").manual_seed(K)
    sa, sb = torch.tensor([0.25], device=DEV), torch.tensor([1.0 / 32], device=DEV)
    x4 = (torch.randn(M, K, generator=g) * 4).to(DEV).to(torch.float8_e4m3fn)
    w4n = (torch.randn(K, N, generator=g) * 2).to(DEV).to(torch.float8_e4m3fn)  # [in, out]
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    assert PF.gemm_path(x4, True, w4n, False, out) == "mfma"
    PF.gemm(x4, True, w4n, False, out, scale_a=sa, scale_b=sb)
    ref = (x4.double() @ w4n.double()) * (0.25 / 32)
    assert (out.double() - ref).abs().max().item() < 0.01 * ref.abs().max().item()


@pytest.mark.parametrize("M,N,K", [(512, 768, 1024), (8192, 8192, 1024)])
def test_gemm_fp8_backward_store_c_false(native_lib, M, N, K):
    """e5m2 x e4m3 dX GEMM with store_c=False: only the e5m2 dZ copy, its amax and the bias-gradient
    column sums are written — equal to the ones of the storing launch."""
    g8 = (torch.randn(M, K, device=DEV) * 100).to(torch.float8_e5m2)
    w8 = (torch.randn(N, K, device=DEV) * 8).to(torch.float8_e4m3fn)
    sa, sb = torch.tensor([1e-3], device=DEV), torch.tensor([1.0 / 16], device=DEV)
    mask = torch.randint(0, 256, PF.relu_mask_shape(M, N), device=DEV, dtype=torch.uint8)
    epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=0.2, seed=(5, 6))
    qs = torch.tensor([4.0], device=DEV)
    outs = []
    for store in (True, False):
        out = torch.full((M, N), 3.0, device=DEV, dtype=torch.bfloat16)
        o8 = torch.empty(M, N, device=DEV, dtype=torch.float8_e5m2)
        cs, am = torch.zeros(N, device=DEV), torch.zeros(1, device=DEV)
        PF.gemm(g8, True, w8, True, out, colsum=cs, mode=PF.EPI_BWD, epi=epi, mask=mask, scale_a=sa, scale_b=sb,
                out8=o8, out8_qscale=qs, amax=am, store_c=store)
        outs.append((out, o8, cs, am))
    (y, y8, cs, am), (y_s, y8_s, cs_s, am_s) = outs
    assert (y_s == 3.0).all() and not (y == 3.0).all()
    assert torch.equal(y8_s.view(torch.uint8), y8.view(torch.uint8)) and am_s.item() == am.item()
    torch.testing.assert_close(cs_s, cs, rtol=1e-5, atol=1e-5 * cs.abs().max().item())


def test_stage_kernels_match_torch(native_lib):
    x = torch.randn(1000, 33, device=DEV, dtype=torch.float64, requires_grad=True)
    for algo, fn in [("relu", torch.relu), ("sigmoid", torch.sigmoid), ("tanh", torch.tanh)]:
        y = PF.activation(x, algo)
        yr = fn(x)
        torch.testing.assert_close(y, yr, rtol=1e-12, atol=1e-12)
        g = torch.randn_like(y)
        (gx,) = torch.autograd.grad(y, x, g)
        (gr,) = torch.autograd.grad(yr, x, g)
        torch.testing.assert_close(gx, gr, rtol=1e-10, atol=1e-12)


def test_dropout_statistics(native_lib):
    x = torch.ones(4096, 256, device=DEV)
    y = PF.dropout(x, 0.2)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.8) < 0.005
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1.25))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_cross_entropy_matches_torch(native_lib, dtype):
    logits = torch.randn(300, 27, device=DEV, dtype=dtype, requires_grad=True)
    labels = torch.randint(0, 27, (300,), device=DEV)
    loss = PF.cross_entropy(logits, labels)
    ref = F.cross_entropy(logits, labels)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-6)
    (g,) = torch.autograd.grad(loss, logits)
    (gr,) = torch.autograd.grad(ref, logits)
    torch.testing.assert_close(g, gr, rtol=1e-5, atol=1e-7)


def test_xent_head_fused_dropout_colsum(native_lib):
    B, C = 256, 64
    p = 0.2
    seed = (5, 6)
    logits = torch.randn(B, C, device=DEV)
    labels = torch.randint(0, C, (B,), device=DEV)
    loss = torch.zeros(1, device=DEV)
    dh = torch.empty(B, C, device=DEV)
    colsum = torch.zeros(C, device=DEV)
    ei, ef = PF.epi_spec(drop_pre=9, p=p, seed=seed)
    torch.ops.pz.xent_head(logits, labels, B, loss, 1.0 / B, dh, 1.0 / B, colsum, None, ei, ef, 0)
    lref = F.cross_entropy(logits.double(), labels)
    assert abs(loss.item() - lref.item()) < 1e-5
    m = torch.from_numpy(keep_mask(B * C, *seed, 9, p).reshape(B, C)).to(DEV)
    dref = (torch.softmax(logits.double(), 1) - F.one_hot(labels, C)) / B * m / (1 - p)
    assert (dh.double() - dref).abs().max().item() < 1e-6
    assert (colsum.double() - dref.sum(0)).abs().max().item() < 1e-5


@pytest.mark.parametrize("B,C,p", [(8192, 1024, 0.2), (1000, 512, 0.0), (64, 2048, 0.3)])
def test_xent_head_bf16_lean_matches_fp64(native_lib, B, C, p):
    """The lean bf16 head (the trainer's logits stage: widths of 512 / 1024 / 2048, dropout before
    the head only, dZ + bias-gradient sums) == fp64 torch: loss, dZ = (softmax - onehot) / B
    through the logits' keep mask, and the column sums; rows past rows_valid get a zero gradient."""
    seed = (13, 2)
    rows_valid = B - 8
    logits = (torch.randn(B, C, device=DEV) * 2).to(torch.bfloat16)
    labels = torch.randint(0, C, (B,), device=DEV)
    loss = torch.zeros(4, device=DEV)
    dh = torch.full((B, C), 7.0, device=DEV, dtype=torch.bfloat16)
    colsum = torch.zeros(C, device=DEV)
    ei, ef = PF.epi_spec(drop_pre=6 if p > 0 else -1, p=p, seed=seed)
    torch.ops.pz.xent_head(logits, labels, rows_valid, loss, 1.0 / rows_valid, dh, 1.0 / rows_valid, colsum, None,
                           ei, ef, C)
    lg = logits[:rows_valid].double()
    lref = F.cross_entropy(lg, labels[:rows_valid])
    assert abs(loss.sum().item() - lref.item()) < 1e-4 * max(1.0, lref.item())
    dref = (torch.softmax(lg, 1) - F.one_hot(labels[:rows_valid], C)) / rows_valid
    if p > 0:
        dref = dref * torch.from_numpy(keep_mask(B * C, *seed, 6, p).reshape(B, C))[:rows_valid].to(DEV) / (1 - p)
    scale = dref.abs().max().item()
    assert (dh[:rows_valid].double() - dref).abs().max().item() < 1e-2 * scale
    assert (dh[rows_valid:] == 0).all()
    assert (colsum.double() - dref.sum(0)).abs().max().item() < 1e-3 * scale * math.sqrt(B)


@pytest.mark.parametrize("B,C", [(8192, 1024), (300, 520)])
def test_xent_head_e5m2_copy(native_lib, B, C):
    """fp8 policy head: the bf16 kernel's e5m2 dZ copy equals quantize_rows of its bf16 dZ (same
    bytes, same amax), rows past rows_valid are zero in both, and store_dh=False leaves dh untouched
    while the loss and the bias-gradient column sums are unchanged."""
    rows_valid = B - 44
    logits = (torch.randn(B, C, device=DEV) * 3).to(torch.bfloat16)
    labels = torch.randint(0, C, (B,), device=DEV)
    ei, ef = PF.epi_spec(drop_pre=3, p=0.2, seed=(7, 8))
    qs = torch.tensor([2.0 ** 20, 2.0 ** -20], device=DEV)
    res = []
    for store in (True, False):
        loss, colsum, amax = torch.zeros(1, device=DEV), torch.zeros(C, device=DEV), torch.zeros(1, device=DEV)
        dh = torch.full((B, C), 5.0, device=DEV, dtype=torch.bfloat16)
        g8 = torch.empty(B, C, device=DEV, dtype=torch.float8_e5m2)
        torch.ops.pz.xent_head(logits, labels, rows_valid, loss, 1.0 / rows_valid, dh, 1.0 / rows_valid, colsum, None,
                               ei, ef, 0, g8, qs[0:1], amax, store)
        res.append((dh, g8, loss, colsum, amax))
    (dh, g8, loss, colsum, amax), (dh_s, g8_s, loss_s, colsum_s, amax_s) = res
    ref8 = torch.empty_like(g8)
    ref_amax = torch.zeros(1, device=DEV)
    torch.ops.pz.quantize_rows(dh, ref8, qs, ref_amax)
    assert torch.equal(g8.view(torch.uint8), ref8.view(torch.uint8)) and amax.item() == ref_amax.item()
    assert (g8[rows_valid:].view(torch.uint8) == 0).all()
    assert (dh_s == 5.0).all()
    assert torch.equal(g8_s.view(torch.uint8), g8.view(torch.uint8)) and amax_s.item() == amax.item()
    # (float atomics across blocks: equal up to summation order)
    assert abs(loss_s.item() - loss.item()) <= 1e-6 * abs(loss.item())
    torch.testing.assert_close(colsum_s, colsum, rtol=1e-5, atol=1e-6 * colsum.abs().max().item())


def test_mse_and_softmax(native_lib):
    y = torch.randn(64, 10, device=DEV, dtype=torch.float64, requires_grad=True)
    t = torch.randn(64, 10, device=DEV, dtype=torch.float64)
    loss = PF.mse_loss(y, t)
    ref = F.mse_loss(y, t)
    torch.testing.assert_close(loss, ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(torch.autograd.grad(loss, y)[0], torch.autograd.grad(ref, y)[0], rtol=1e-6, atol=1e-9)
    s = PF.softmax(y)
    torch.testing.assert_close(s, torch.softmax(y, -1), rtol=1e-12, atol=1e-12)


def test_adam_matches_torch(native_lib):
    from penr_oz_neural_network_torch_amd.engine.optim import FusedOptimizer
    from penr_oz_neural_network_torch_amd.engine.params import ParamStore
    from penr_oz_neural_network_torch_amd.models.layers import LinearLayer
    torch.manual_seed(0)
    layers = [LinearLayer(33, 65, "random"), LinearLayer(65, 7, "random")]
    ref_params = [p.detach().float().clone().to(DEV).requires_grad_() for l in layers for p in l.params]
    store = ParamStore.adopt(layers, torch.device(DEV), torch.float32)
    params = [p for l in layers for p in l.params]
    opt = torch.optim.Adam(params, betas=(0.9, 0.99), eps=1e-7)
    fused = FusedOptimizer(store, params, opt, {})
    ref_opt = torch.optim.Adam(ref_params, lr=0.01, betas=(0.9, 0.99), eps=1e-7)
    grads = torch.zeros(store.numel, device=DEV)
    for it in range(5):
        for seg in store.segments:
            g = torch.randn(seg.shape, device=DEV)
            store.view(seg, grads).copy_(g)
            ref_params[seg.param_index].grad = g.clone()
        fused.step(grads, 0.01, 0.0, 1.0)
        ref_opt.step()
    for seg in store.segments:
        torch.testing.assert_close(store.view(seg), ref_params[seg.param_index].detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape", [(512, 4096, 512), (1024, 2048, 4096)])  # one pass / split-K (8 slices)
@pytest.mark.parametrize("adam", [True, False])
def test_gemm_update_matches_separate_update(native_lib, shape, adam):
    """dW GEMM with the optimizer update in its epilogue (EPI_OPT) vs the fp64 gradient GEMM followed
    by the same update formula in torch fp32 (torch.optim.Adam's single-tensor step / the reference's
    SGD), plus the statistics the update reduces (update-ratio sums, sum w^2, amax)."""
    M, N, K = shape
    g = torch.Generator(device="cpu").manual_seed(M + N + K + adam)
    a = (torch.randn(K, M, generator=g) * 0.1).to(DEV, torch.bfloat16)  # x_in [rows, in]
    b = (torch.randn(K, N, generator=g) * 0.1).to(DEV, torch.bfloat16)  # dZ [rows, out]
    p0 = torch.randn(M, N, generator=g).to(DEV)
    m0 = (torch.randn(M, N, generator=g) * 0.01).to(DEV)
    v0 = (torch.rand(M, N, generator=g) * 1e-3 + 1e-4).to(DEV)
    p, m, v = p0.clone(), m0.clone(), v0.clone()
    shadow = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    stats = torch.zeros(4, device=DEV, dtype=torch.float64)
    amax = torch.zeros(1, device=DEV)
    lr, b1, b2, eps, l2, t, scale = 0.01, 0.9, 0.99, 1e-7, 1e-3, 3, 0.5
    bc1, bc2s = 1 - b1 ** t, math.sqrt(1 - b2 ** t)
    assert PF.gemm_path(a, False, b, False, p) == "mfma"
    torch.ops.pz.gemm_update(a, False, b, False, p, M, N, K, 1.0, p, m if adam else None, v if adam else None,
                             shadow, stats, amax, adam, lr, b1, b2, eps, bc1, bc2s, scale, l2, None, None, 1)
    grad = (a.double().t() @ b.double()).float()
    gg = grad * scale + 2 * l2 * p0
    if adam:
        m_ref = m0 + (1 - b1) * (gg - m0)
        v_ref = v0 * b2 + (1 - b2) * gg * gg
        p_ref = p0 - (lr / bc1) * (m_ref / (v_ref.sqrt() / bc2s + eps))
        torch.testing.assert_close(m, m_ref, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(v, v_ref, rtol=1e-4, atol=1e-9)
    else:
        p_ref = p0 - lr * gg
        assert torch.equal(m, m0) and torch.equal(v, v0)  # SGD has no moments
    torch.testing.assert_close(p, p_ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(shadow, p.to(torch.bfloat16))
    d = (p - p0).double()
    ref_st = torch.stack([d.sum(), (d * d).sum(), p.double().sum(), (p.double() ** 2).sum()])
    torch.testing.assert_close(stats, ref_st, rtol=1e-9, atol=1e-9)
    assert amax.item() == p.abs().max().item()


def test_histogram_and_moments(native_lib):
    x = torch.randn(10000, 7, device=DEV, dtype=torch.float64) * 3 + 1
    s = PF.tensor_summary(x, "tanh", 100)
    h = torch.histogram(x.cpu(), density=True)
    assert abs(s["mean"] - x.mean().item()) < 1e-9
    assert abs(s["std"] - x.std().item()) < 1e-9
    assert abs(s["saturated"] - (x.abs() > 0.97).double().mean().item()) < 1e-12
    np.testing.assert_allclose(s["histogram"]["x"], h.bin_edges[:-1].tolist(), rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(s["histogram"]["y"], h.hist.tolist(), rtol=1e-6, atol=1e-9)
    e = torch.randn(50, 3, 10, device=DEV) * 2
    se = PF.tensor_summary(e, "embedding", 100)
    assert abs(se["saturated"] - (torch.norm(e, dim=-1) > 5.0).double().mean().item()) < 1e-12
    sm = PF.tensor_summary(torch.softmax(e, -1), "softmax", 0)
    assert abs(sm["saturated"] - (torch.softmax(e, -1).max(-1).values > 0.97).double().mean().item()) < 1e-12


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_batchnorm_matches_reference_formula(native_lib, dtype):
    x = torch.randn(500, 3, 16, device=DEV, dtype=dtype, requires_grad=True)
    gain = torch.rand(16, device=DEV, dtype=dtype, requires_grad=True)
    bias = torch.randn(16, device=DEV, dtype=dtype, requires_grad=True)
    rm = torch.zeros(16, device=DEV, dtype=dtype)
    rv = torch.ones(16, device=DEV, dtype=dtype)
    y, rm2, rv2 = PF.batchnorm(x, gain, bias, rm, rv, 1e-5, 0.1, True)
    mean = x.mean((0, 1), keepdim=True)
    var = x.var((0, 1), keepdim=True)
    yr = gain * (x - mean) / torch.sqrt(var + 1e-5) + bias
    tol = 1e-9 if dtype == torch.float64 else 1e-4
    torch.testing.assert_close(y, yr, rtol=tol, atol=tol)
    torch.testing.assert_close(rm2, (0.1 * mean).reshape(-1).detach(), rtol=tol, atol=tol)
    g = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, gain, bias), g)
    ref = torch.autograd.grad(yr, (x, gain, bias), g)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-4 if dtype == torch.float32 else 1e-7,
                                   atol=1e-4 if dtype == torch.float32 else 1e-9)


def test_embedding_forward_backward(native_lib):
    table = torch.randn(27, 10, device=DEV, dtype=torch.float64, requires_grad=True)
    ids = torch.randint(0, 27, (64, 3), device=DEV).double()
    out = PF.embedding(ids, table)
    ref = table[ids.long()]
    torch.testing.assert_close(out, ref)
    g = torch.randn_like(out)
    torch.testing.assert_close(torch.autograd.grad(out, table, g)[0], torch.autograd.grad(ref, table, g)[0],
                               rtol=1e-12, atol=1e-12)


def test_gather_rows_sampling(native_lib):
    data = torch.arange(1000 * 4, device=DEV, dtype=torch.float32).view(1000, 4)
    labels = torch.arange(1000, device=DEV)
    out = torch.empty(128, 4, device=DEV, dtype=torch.bfloat16)
    lab = torch.empty(128, device=DEV, dtype=torch.int64)
    picked = torch.empty(128, device=DEV, dtype=torch.int64)
    torch.ops.pz.gather_rows(data, None, 11, 22, out, 100, labels, lab, picked)
    assert torch.equal(lab[:100], picked[:100])
    assert (picked[:100] >= 0).all() and (picked[:100] < 1000).all()
    torch.testing.assert_close(out[:100].float(), data[picked[:100]].to(torch.bfloat16).float())
    assert (out[100:] == 0).all()


@pytest.mark.parametrize("M,N,K,a_kc,b_kc,out", [
    (4096, 1024, 8192, False, False, torch.float32),   # dW-like (split 4)
    (1024, 4096, 8192, False, False, torch.float32),
    (8192, 1024, 4096, True, False, torch.bfloat16),   # skinny forward (split 2) with a fused epilogue
    (8192 - 64, 1024 - 64, 4096, True, True, torch.bfloat16),  # partial tiles
])
def test_gemm_split_k_matches_reference(native_lib, M, N, K, a_kc, b_kc, out):
    """Skinny shapes run as 256x256 tiles with K split over several workgroups and an in-kernel
    last-arriver slab reduction; repeated launches reuse the tile counters."""
    a = torch.randn((M, K) if a_kc else (K, M), device=DEV).to(torch.bfloat16)
    b = torch.randn((N, K) if b_kc else (K, N), device=DEV).to(torch.bfloat16)
    A = a.double() if a_kc else a.double().t()
    B = b.double().t() if b_kc else b.double()
    bias = torch.randn(N, device=DEV) if out == torch.bfloat16 else None
    ref = A @ B + (bias.double() if bias is not None else 0)
    c = torch.empty(M, N, device=DEV, dtype=out)
    for _ in range(3):
        c.fill_(float("nan"))
        if out == torch.bfloat16:
            PF.gemm(a, a_kc, b, b_kc, c, bias=bias, mode=PF.EPI_FWD, epi=PF.epi_spec())
        else:
            PF.gemm(a, a_kc, b, b_kc, c)
        tol = 0.02 if out == torch.bfloat16 else 2e-3
        err = (c.double() - ref).abs().max().item()
        assert err < tol * ref.abs().max().item(), err


def test_gemm_fp8_split_k(native_lib):
    f8 = torch.float8_e4m3fn
    M, N, K = 8192, 1024, 8192
    x8 = torch.randn(M, K, device=DEV).to(f8)
    w8 = torch.randn(N, K, device=DEV).to(f8)
    one = torch.ones(1, device=DEV)
    y = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    PF.gemm(x8, True, w8, True, y, mode=PF.EPI_FWD, epi=PF.epi_spec(), scale_a=one, scale_b=one)
    ref = x8.double() @ w8.double().t()
    assert (y.double() - ref).abs().max().item() < 0.01 * ref.abs().max().item()


def test_quantize_rows_derived_weight_scale(native_lib):
    """Weights under the fp8 policy: q = 448 / amax (the optimizer's reduced max |w|) derived in the
    kernel, {q, 1/q} published, the other parity's accumulator cleared, bytes == torch's cast."""
    w = torch.randn(1024, 8192, device=DEV) * 0.02
    amax_in = w.abs().max().reshape(1)
    clear = torch.full((1,), 3.0, device=DEV)
    qs = torch.zeros(2, device=DEV)
    out = torch.empty(1024, 8192, device=DEV, dtype=torch.float8_e4m3fn)
    torch.ops.pz.quantize_rows(w, out, qs, None, amax_in, clear)
    q = 448.0 / amax_in.item()
    assert abs(qs[0].item() - q) <= 1e-6 * q and abs(qs[1].item() * q - 1) < 1e-6 and clear.item() == 0.0
    ref = (w * qs[0]).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (out.view(torch.uint8) != ref.view(torch.uint8)).float().mean().item() < 1e-4


@pytest.mark.parametrize("dtype,fmt,cols", [(torch.bfloat16, torch.float8_e4m3fn, 1024),
                                            (torch.float32, torch.float8_e5m2, 520),
                                            (torch.bfloat16, torch.float8_e4m3fn, 12)])  # 12: scalar path
def test_quantize_rows_matches_torch_cast(native_lib, dtype, fmt, cols):
    """e4m3 / e5m2 row quantiser (8-wide vector path and the scalar fallback): saturating
    sat(x * q) bytes as torch's float8 cast of the clamped values, exact amax."""
    x = (torch.randn(777, cols, device=DEV) * 3).to(dtype)
    lim = 448.0 if fmt == torch.float8_e4m3fn else 57344.0
    q = lim / (0.5 * x.float().abs().max().item())  # half the values saturate
    qs = torch.tensor([q, 1.0 / q], device=DEV)
    out = torch.empty(777, cols, device=DEV, dtype=fmt)
    amax = torch.zeros(1, device=DEV)
    native_lib.quantize_rows(x, out, qs, amax)
    ref = (x.float() * qs[0]).clamp(-lim, lim).to(fmt)
    assert (out.view(torch.uint8) != ref.view(torch.uint8)).float().mean().item() < 1e-4
    assert amax.item() == x.float().abs().max().item()


@pytest.mark.parametrize("K,N", [(192, 320), (100, 70)])  # full 64x64 tiles (16-B path) / ragged edges
def test_quant_transpose_matches_torch_cast(native_lib, K, N):
    """fp32 W [K, N] -> e4m3 W^T [N, K] at q = 448 / amax (taken from the optimizer's amax record)."""
    w = torch.randn(K, N, device=DEV) * 0.05
    out = torch.empty(N, K, device=DEV, dtype=torch.float8_e4m3fn)
    qs = torch.zeros(2, device=DEV)
    amax = w.abs().max().reshape(1)
    clear = torch.full((1,), 7.0, device=DEV)
    native_lib.quant_transpose(w, out, qs, amax, clear)
    q = 448.0 / amax.item()
    assert abs(qs[0].item() - q) <= 1e-6 * q and clear.item() == 0.0
    ref = (w.t() * qs[0]).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (out.view(torch.uint8) != ref.view(torch.uint8)).float().mean().item() < 1e-4


@pytest.mark.parametrize("shapes,out", [
    (((1024, 4096), (4096, 1024), 8192), torch.bfloat16),  # mlp4's dW_L1 + dW_L3: 128 tiles, split 2
    (((1024, 4096), (4096, 1024), 8192), torch.float32),
    (((1024, 8192), (8192, 1024), 8192), torch.bfloat16),  # mlp8192's two dW: 256 tiles, no split
    (((256, 512), (512, 256), 1024), torch.bfloat16),      # small: split 4
])
def test_gemm_pair_matches_two_launches(native_lib, shapes, out):
    """pz::gemm_pair: two weight-gradient GEMMs in one launch (first workgroups GEMM 0, the rest
    GEMM 1, each with its own split-K slabs and tickets) == each against fp64; repeated launches
    reuse the tile counters."""
    (m0, n0), (m1, n1), K = shapes
    a0 = torch.randn(K, m0, device=DEV).to(torch.bfloat16)
    b0 = torch.randn(K, n0, device=DEV).to(torch.bfloat16)
    a1 = torch.randn(K, m1, device=DEV).to(torch.bfloat16)
    b1 = torch.randn(K, n1, device=DEV).to(torch.bfloat16)
    c0 = torch.empty(m0, n0, device=DEV, dtype=out)
    c1 = torch.empty(m1, n1, device=DEV, dtype=out)
    assert PF.gemm_pair_split(a0, b0, c0, a1, b1, c1) > 0
    r0 = a0.double().t() @ b0.double()
    r1 = a1.double().t() @ b1.double()
    for _ in range(3):
        c0.fill_(float("nan"))
        c1.fill_(float("nan"))
        PF.gemm_pair(a0, b0, c0, a1, b1, c1)
        for c, r in ((c0, r0), (c1, r1)):
            tol = (2.0 ** -7 if out == torch.bfloat16 else 1e-5) * r.abs().max().item() + 1e-3 * math.sqrt(K)
            assert (c.double() - r).abs().max().item() < tol


def test_gemm_pair_fp8_and_ineligible(native_lib):
    """The fp8 weight-gradient pair (e4m3 activations x e5m2 gradients, per-GEMM dequant scales)
    against fp64 on the quantised values; mixed precisions or unequal K are not paired."""
    K, (m0, n0), (m1, n1) = 8192, (1024, 8192), (8192, 1024)
    x0 = (torch.randn(K, m0, device=DEV) * 4).to(torch.float8_e4m3fn)
    g0 = (torch.randn(K, n0, device=DEV) * 1000).to(torch.float8_e5m2)
    x1 = (torch.randn(K, m1, device=DEV) * 2).to(torch.float8_e4m3fn)
    g1 = (torch.randn(K, n1, device=DEV) * 500).to(torch.float8_e5m2)
    s = [torch.tensor([v], device=DEV) for v in (0.25, 1.0 / 4096, 0.5, 1.0 / 2048)]
    c0 = torch.empty(m0, n0, device=DEV, dtype=torch.bfloat16)
    c1 = torch.empty(m1, n1, device=DEV, dtype=torch.bfloat16)
    assert PF.gemm_pair_split(x0, g0, c0, x1, g1, c1) == 1
    PF.gemm_pair(x0, g0, c0, x1, g1, c1, scales0=(s[0], s[1]), scales1=(s[2], s[3]))
    for c, x, gg, f in ((c0, x0, g0, 0.25 / 4096), (c1, x1, g1, 0.5 / 2048)):
        ref = (x.double().t() @ gg.double()) * f
        assert (c.double() - ref).abs().max().item() <= 2.0 ** -8 * ref.abs().max().item()
    b16 = torch.randn(K, m1, device=DEV).to(torch.bfloat16)
    assert PF.gemm_pair_split(x0, g0, c0, b16, torch.randn(K, n1, device=DEV).to(torch.bfloat16), c1) == 0
    short = torch.randn(K // 2, m1, device=DEV).to(torch.bfloat16)
    bb = torch.randn(K, n0, device=DEV).to(torch.bfloat16)
    assert PF.gemm_pair_split(torch.randn(K, m0, device=DEV).to(torch.bfloat16), bb, c0, short,
                              torch.randn(K // 2, n1, device=DEV).to(torch.bfloat16), c1) == 0


def test_gemm_pair_stream_k_eligibility_at_one_k_step(native_lib):
    """a 64-row per-rank batch is ONE 64-deep K step — the tiled pair takes it, the
    stream-K engine (>= two steps) does not, and gemm_pair_split(engine=2) says so instead of the
    budgeted launch raising mid-step."""
    K, (m0, n0), (m1, n1) = 64, (1024, 4096), (4096, 1024)
    bf = torch.bfloat16
    x0, g0 = torch.randn(K, m0, device=DEV).to(bf), torch.randn(K, n0, device=DEV).to(bf)
    x1, g1 = torch.randn(K, m1, device=DEV).to(bf), torch.randn(K, n1, device=DEV).to(bf)
    c0 = torch.empty(m0, n0, device=DEV, dtype=bf)
    c1 = torch.empty(m1, n1, device=DEV, dtype=bf)
    assert PF.gemm_pair_split(x0, g0, c0, x1, g1, c1) > 0
    assert PF.gemm_pair_split(x0, g0, c0, x1, g1, c1, engine=2) == 0
    PF.gemm_pair(x0, g0, c0, x1, g1, c1)
    for c, x, g in ((c0, x0, g0), (c1, x1, g1)):
        ref = x.double().t() @ g.double()
        assert (c.double() - ref).abs().max().item() <= 2.0 ** -7 * ref.abs().max().item() + 1e-2


_WT_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[2])
from penr_oz_neural_network_torch_amd.ops import functional as PF
torch.manual_seed(0)
D = "cuda"
M, N, K = 8192, 4096, 1024
a = torch.randn(M, K, device=D).to(torch.bfloat16)
w = torch.randn(K, N, device=D).to(torch.bfloat16)
bias = torch.randn(N, device=D)
epi = PF.epi_spec(act=PF.ACT_RELU, drop_post=2, p=0.2, seed=(1, 2))
y = torch.empty(M, N, device=D, dtype=torch.bfloat16)
mask = PF.relu_mask_empty(M, N, device=D)
PF.gemm(a, True, w, False, y, bias=bias, mode=PF.EPI_FWD, epi=epi, mask=mask)
x8 = (torch.randn(M, K, device=D) * 4).to(torch.float8_e4m3fn)
w8 = (torch.randn(K, N, device=D) * 2).to(torch.float8_e4m3fn)
y8 = torch.empty(M, N, device=D, dtype=torch.float8_e4m3fn)
yf = torch.empty(M, N, device=D, dtype=torch.bfloat16)
one = torch.ones(1, device=D)
PF.gemm(x8, True, w8, False, yf, bias=bias, mode=PF.EPI_FWD, epi=epi, scale_a=one, scale_b=one, out8=y8,
        out8_qscale=one, amax=torch.zeros(1, device=D))
dw = torch.empty(K, N, device=D, dtype=torch.bfloat16)
PF.gemm(a, False, y, False, dw)  # [K=8192 rows] x: dW layout (M/N-contiguous), split-K
torch.save({"y": y.cpu(), "mask": mask.cpu(), "y8": y8.view(torch.uint8).cpu(), "yf": yf.cpu(), "dw": dw.cpu()},
           sys.argv[1])
"""


def test_write_through_epilogue_stores_are_bit_identical(tmp_path):
    """PZ_GEMM_WT=1 (whole-tile epilogue stores as write-through sc1 buffer stores: C, the ReLU
    bitmask, the fp8 copy; bf16 forward, fp8 forward, split-K dW) writes exactly the bytes the
    default stores write. The policy is read once per process: one subprocess per setting."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "wt.py"
    script.write_text(_WT_SCRIPT)
    outs = []
    for wt in ("0", "1"):
        out = tmp_path / f"wt{wt}.pt"
        env = dict(os.environ, PZ_GEMM_WT=wt)
        subprocess.run([sys.executable, str(script), str(out), root], env=env, check=True, timeout=240)
        outs.append(torch.load(out, weights_only=True))
    for k in outs[0]:
        if k == "dw":  # split-K: the last-arriving slice (run-dependent) sets the fp32 summation order
            torch.testing.assert_close(outs[0][k].float(), outs[1][k].float(), rtol=2 ** -7, atol=1e-2)
        else:
            assert torch.equal(outs[0][k], outs[1][k]), k


def test_colsum_is_deterministic_and_accumulates(native_lib):
    """pz::colsum (record-step bias gradients): out += column sums, against fp64, and two runs
    bit-identical — per-block partial rows folded in block order, no float atomics."""
    for dt, odt in ((torch.bfloat16, torch.float32), (torch.float32, torch.float32), (torch.float64, torch.float64)):
        x = torch.randn(3001, 700, device=DEV).to(dt)
        base = torch.randn(700, device=DEV, dtype=odt)
        outs = []
        for _ in range(2):
            out = base.clone()
            native_lib.colsum(x, out)
            outs.append(out)
        assert torch.equal(outs[0], outs[1])
        ref = base.double() + x.double().sum(0)
        tol = 1e-9 if odt == torch.float64 else 1e-3
        assert (outs[0].double() - ref).abs().max().item() < tol * math.sqrt(3001)
