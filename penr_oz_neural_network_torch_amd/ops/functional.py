"""GPU operators with autograd, built on the ``torch.ops.pz`` HIP kernels.

This is the *autograd path* used by :class:`..models.layers.Layer` ``forward`` on GPU tensors
(``compute_output``, ``_forward`` + ``backward`` exactly as the reference calls them). The
throughput path (:mod:`..engine`) calls the same kernels with its own explicit schedule.

Every function here requires the native library; a missing ``_pz_C.so`` raises instead of
falling back to ATen (see :mod:`.native`).
"""
from __future__ import annotations

import math

import torch
from torch import Tensor

from . import native

ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH = 0, 1, 2, 3
ACT_CODES = {"relu": ACT_RELU, "sigmoid": ACT_SIGMOID, "tanh": ACT_TANH, None: ACT_NONE, "none": ACT_NONE}
EPI_STORE, EPI_FWD, EPI_BWD = 0, 1, 2
SAT_CODES = {"abs_gt": 1, "le": 2, "row_norm_gt": 3, "row_max_gt": 4}


def _ops():
    native.require()
    return torch.ops.pz


# --------------------------------------------------------------------------------------------
# epilogue specs
# --------------------------------------------------------------------------------------------
_M32 = 0xFFFFFFFF


def mix32(x: int) -> int:
    """The kernels' 32-bit integer finaliser ("lowbias32"), host side."""
    x &= _M32
    x ^= x >> 16
    x = (x * 0x7FEB352D) & _M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & _M32
    x ^= x >> 16
    return x


def layer_key(seed: tuple[int, int], lid: int) -> int:
    """Per-(seed, layer) dropout key: the mask bit of element pair j is ``mix32(j ^ key)``."""
    return mix32((seed[0] & _M32) ^ mix32((seed[1] + 0x9E3779B9 * (lid + 1)) & _M32))


def epoch_key(key: int, epoch: int) -> int:
    """Per-epoch variant of a (seed, layer) key — the kernels' ``epoch_key`` (pz_common.h)."""
    return mix32((key & _M32) ^ mix32((epoch * 0x9E3779B1 + 0x7F4A7C15) & _M32))


def epi_spec(act: int = ACT_NONE, drop_pre: int = -1, drop_post: int = -1, p: float = 0.0,
             seed: tuple[int, int] = (0, 0), epoch: int | None = None,
             epoch_ptr: int = 0) -> tuple[list[int], list[float]]:
    """Pack a stage epilogue ``drop_post(act(drop_pre(x)))`` for the kernels.

    ``drop_pre`` / ``drop_post`` are the reference layer indices whose dropout is applied (-1 =
    none). Dropout keeps an element iff its 16-bit counter-hash draw is ``>= round(p * 65536)``;
    kept elements are scaled by ``1/(1-p)`` like ``torch.nn.functional.dropout``.

    Training steps vary the masks per epoch: eagerly launched steps pass ``epoch`` (mixed in
    here), graph-replayed steps pass ``epoch_ptr`` = the device address of the trainer's int32
    epoch counter, and the kernels mix ``*epoch_ptr`` in with the same function.
    """
    if p <= 0.0:
        drop_pre = drop_post = -1
    drop_all = 1 if p >= 1.0 else 0
    thresh = min(65536, int(round(p * 65536)))
    scale = 0.0 if drop_all else 1.0 / (1.0 - p)
    inv_scale = 1.0 - p
    kpre = layer_key(seed, drop_pre) if drop_pre >= 0 else 0
    kpost = layer_key(seed, drop_post) if drop_post >= 0 else 0
    if epoch is not None:
        kpre = epoch_key(kpre, epoch) if drop_pre >= 0 else 0
        kpost = epoch_key(kpost, epoch) if drop_post >= 0 else 0
    return ([act, int(drop_pre >= 0), int(drop_post >= 0), kpre, kpost, thresh, drop_all, int(epoch_ptr)],
            [scale, inv_scale])


def new_seed() -> tuple[int, int]:
    """Fresh dropout seed drawn from torch's CPU generator (so ``torch.manual_seed`` controls it)."""
    s = torch.randint(0, 2 ** 62, (1,)).item()
    return s & 0xFFFFFFFF, (s >> 32) & 0xFFFFFFFF


NO_EPI = epi_spec()


# --------------------------------------------------------------------------------------------
# GEMM front-end
# --------------------------------------------------------------------------------------------
def gemm(a: Tensor, a_kc: bool, b: Tensor, b_kc: bool, out: Tensor, *, bias: Tensor | None = None,
         aux: Tensor | None = None, colsum: Tensor | None = None, mode: int = EPI_STORE,
         epi: tuple[list[int], list[float]] = NO_EPI, alpha: float = 1.0, accumulate: bool = False,
         idx_ld: int = 0, force_generic: bool = False, mask: Tensor | None = None,
         scale_a: Tensor | None = None, scale_b: Tensor | None = None, out8: Tensor | None = None,
         out8_qscale: Tensor | None = None, amax: Tensor | None = None, no_split: bool = False,
         store_c: bool = True, engine: int = 0, cus: int = 0) -> Tensor:
    """``out[M,N] = op(a) @ op(b)`` with a fused epilogue.

    ``a_kc``: ``a`` is stored ``[M,K]`` (else ``[K,M]``); ``b_kc``: ``b`` is stored ``[N,K]`` (else ``[K,N]``).
    ``mask`` (uint8 :func:`relu_mask_shape` ``(M, N)``, tile-blocked, MFMA shapes only): EPI_FWD writes the bitmask
    ``y > 0`` of the final output; EPI_BWD with a ReLU stage reads it instead of ``aux``.
    fp8: ``a``/``b`` may be ``float8_e4m3fn`` (both K-contiguous); products are multiplied by the
    device scalars ``scale_a * scale_b``. ``out8`` (e4m3, EPI_FWD) receives ``sat(y * out8_qscale)``
    and ``amax`` (fp32 scalar, caller-zeroed) the running ``max |y|``. ``no_split`` turns the
    split-K plan of a skinny shape off (a GEMM running beside others on its own stream).
    ``store_c=False`` (MFMA path, bf16 ``out``): only the side outputs — ``out8``, ``mask``,
    ``colsum`` — are written, ``out`` is not (the fp8 policy's bf16 tensors nobody reads).
    ``engine``: 0 = the default choice, 1 = the tiled kernels (gemm_mfma.hip), 2 = the persistent
    stream-K engine (gemm_sk.hip; raises if the shape is not eligible), 3 = that engine on its
    4-wave lab main loop (plain stores only); ``cus`` = the CU budget of
    the persistent engine (0 = every CU).
    """
    M, N = out.shape
    K = a.shape[1] if a_kc else a.shape[0]
    _ops().gemm(a, a_kc, b, b_kc, out, bias, aux, colsum, mode, epi[0], epi[1], alpha, accumulate,
                M, N, K, idx_ld, force_generic, mask, scale_a, scale_b, out8, out8_qscale, amax,
                (1 if no_split else 0) | (0 if store_c else 2) | ((engine & 3) << 2) | ((cus & 0xFFFF) << 16))
    return out


def gemm_pair(a0: Tensor, b0: Tensor, out0: Tensor, a1: Tensor, b1: Tensor, out1: Tensor, *,
              scales0: tuple = (None, None), scales1: tuple = (None, None), engine: int = 0, cus: int = 0) -> None:
    """Two weight-gradient GEMMs ``out_i = a_iᵀ @ b_i`` (``a_i`` stored ``[K, M_i]``, ``b_i``
    ``[K, N_i]``, one K) in ONE launch (``pz::gemm_pair``); fp8 operands take their
    ``(scale_a, scale_b)`` dequantisation scalars. Check :func:`gemm_pair_split` first.
    ``engine=2`` (bf16): both problems' tiles as one persistent stream-K schedule on ``cus`` CUs."""
    K = a0.shape[0]
    _ops().gemm_pair(a0, b0, out0, a1, b1, out1, out0.shape[0], out0.shape[1], out1.shape[0], out1.shape[1], K,
                     scales0[0], scales0[1], scales1[0], scales1[1], ((engine & 3) << 2) | ((cus & 0xFFFF) << 16))


def gemm_pair_split(a0: Tensor, b0: Tensor, out0: Tensor, a1: Tensor, b1: Tensor, out1: Tensor, engine: int = 0) -> int:
    """Split-K factor the pair would run with, 0 when the two GEMMs cannot share a launch
    (``engine=2``: or when the persistent stream-K engine cannot run both)."""
    if a0.shape[0] != a1.shape[0]:
        return 0
    return int(_ops().gemm_pair_split(a0, b0, out0, a1, b1, out1, out0.shape[0], out0.shape[1], out1.shape[0],
                                      out1.shape[1], a0.shape[0], engine))


def relu_mask_shape(m: int, n: int) -> tuple[int, int]:
    """Shape of the tile-blocked ReLU bitmask of an ``[m, n]`` output (csrc/pz_launch.h
    GemmArgs::mask): 256 x 256 element blocks of 8 KiB (256 rows of 32 B) in block-row-major order,
    held as a uint8 ``[roundup(m, 256), 32 * ceil(n / 256)]`` tensor."""
    return (m + 255) // 256 * 256, (n + 255) // 256 * 32


def relu_mask_empty(m: int, n: int, device=None) -> Tensor:
    return torch.empty(relu_mask_shape(m, n), device=device, dtype=torch.uint8)


def relu_mask_bits(mask: Tensor, m: int, n: int) -> Tensor:
    """Unpack a tile-blocked ReLU bitmask into a bool ``[m, n]`` (bit ``n & 7`` of each byte)."""
    rows, ld = mask.shape
    tn = ld // 32
    rowmajor = mask.reshape(rows // 256, tn, 256, 32).permute(0, 2, 1, 3).reshape(rows, ld)
    bits = (rowmajor.unsqueeze(-1).int() >> torch.arange(8, device=mask.device, dtype=torch.int32)) & 1
    return bits.reshape(rows, ld * 8)[:m, :n].bool()


def relu_mask_pack(y_pos: Tensor) -> Tensor:
    """The tile-blocked bitmask of a bool ``[m, n]`` (inverse of :func:`relu_mask_bits`)."""
    m, n = y_pos.shape
    rows, ld = relu_mask_shape(m, n)
    full = torch.zeros(rows, ld * 8, device=y_pos.device, dtype=torch.int32)
    full[:m, :n] = y_pos.int()
    rowmajor = (full.reshape(rows, ld, 8) << torch.arange(8, device=y_pos.device, dtype=torch.int32)).sum(-1)
    blocked = rowmajor.to(torch.uint8).reshape(rows // 256, 256, ld // 32, 32).permute(0, 2, 1, 3)
    return blocked.contiguous().reshape(rows, ld)


def gemm_path(a: Tensor, a_kc: bool, b: Tensor, b_kc: bool, out: Tensor) -> str:
    M, N = out.shape
    K = a.shape[1] if a_kc else a.shape[0]
    path = _ops().gemm_path(a, a_kc, b, b_kc, out, M, N, K)
    return {1: "mfma", 2: "mfma_wide"}.get(path, "generic")  # mfma_wide: fp32 / fp64 matrix cores


def _as_2d(x: Tensor) -> tuple[Tensor, tuple]:
    lead = x.shape[:-1]
    return x.reshape(-1, x.shape[-1]).contiguous(), lead


# --------------------------------------------------------------------------------------------
# Linear
# --------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, w: Tensor, b: Tensor | None):
        squeeze = x.dim() == 1
        x2, lead = _as_2d(x.unsqueeze(0) if squeeze else x)
        wc = w if w.dtype == x2.dtype else w.to(x2.dtype)
        wc = wc.contiguous()
        out = torch.empty(x2.shape[0], wc.shape[1], device=x.device, dtype=x2.dtype)
        bias_k = None
        if b is not None:  # fp64 models add the fp64 bias (the kernels take fp32 or fp64)
            bias_k = b.detach().to(torch.float64 if x2.dtype == torch.float64 else torch.float32).contiguous()
        gemm(x2, True, wc, False, out, bias=bias_k)
        ctx.save_for_backward(x2, wc)
        ctx.has_bias = b is not None
        ctx.w_dtype = w.dtype
        ctx.b_dtype = b.dtype if b is not None else None
        out = out.view(*lead, wc.shape[1])
        return out.squeeze(0) if squeeze else out

    @staticmethod
    def backward(ctx, grad_out: Tensor):
        x2, wc = ctx.saved_tensors
        g2 = grad_out.reshape(-1, wc.shape[1]).to(x2.dtype).contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x2)
            gemm(g2, True, wc, True, gx)  # dX = dY @ W^T, W stored [in,out] = [N,K]
            gx = gx.view(*grad_out.shape[:-1], wc.shape[0])
        if ctx.needs_input_grad[1]:
            acc_dtype = torch.float64 if x2.dtype == torch.float64 else torch.float32
            gw = torch.empty(wc.shape, device=wc.device, dtype=acc_dtype)
            gemm(x2, False, g2, False, gw)  # dW = X^T @ dY (K = batch)
            gw = gw.to(ctx.w_dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            acc = torch.float64 if x2.dtype == torch.float64 else torch.float32  # fp64 models stay fp64
            gb = torch.zeros(wc.shape[1], device=wc.device, dtype=acc)
            _ops().colsum(g2, gb)
            gb = gb.to(ctx.b_dtype)
        return gx, gw, gb


def linear(x: Tensor, w: Tensor, b: Tensor | None) -> Tensor:
    return _Linear.apply(x, w, b)


# --------------------------------------------------------------------------------------------
# activations / dropout (stage epilogue kernels)
# --------------------------------------------------------------------------------------------
class _Stage(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, ei: list, ef: list):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _ops().stage_fwd(xc, y, ei, ef)
        ctx.save_for_backward(y)
        ctx.ei, ctx.ef = ei, ef
        return y

    @staticmethod
    def backward(ctx, g: Tensor):
        (y,) = ctx.saved_tensors
        gc = g.contiguous().to(y.dtype)
        dx = torch.empty_like(y)
        _ops().stage_bwd(gc, y, dx, ctx.ei, ctx.ef)
        return dx, None, None


def activation(x: Tensor, algo: str) -> Tensor:
    ei, ef = epi_spec(act=ACT_CODES[algo])
    return _Stage.apply(x, ei, ef)


def dropout(x: Tensor, p: float) -> Tensor:
    if p <= 0.0:
        return x
    ei, ef = epi_spec(drop_pre=0, p=p, seed=new_seed())
    return _Stage.apply(x, ei, ef)


# --------------------------------------------------------------------------------------------
# softmax / losses
# --------------------------------------------------------------------------------------------
class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _ops().softmax_rows(xc, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g: Tensor):
        (y,) = ctx.saved_tensors
        dx = torch.empty_like(y)
        _ops().softmax_bwd(g.contiguous().to(y.dtype), y, dx)
        return dx


def softmax(x: Tensor) -> Tensor:
    return _Softmax.apply(x)


def check_index_range(idx: Tensor, lo: int, hi: int, what: str, size: int | None = None) -> None:
    """Raise IndexError (as ATen / Python indexing do) unless every id is in ``[lo, hi)``.
    The HIP kernels never read outside their tables either way, but a bad id must surface as an
    error, not as a silently wrong loss. A GPU tensor costs one small reduction + sync."""
    if idx.numel() == 0:
        return
    v = idx if idx.dtype == torch.int64 else idx.long()
    mn, mx = (int(t) for t in torch.aminmax(v))
    if mn < lo or mx >= hi:
        bad = mn if mn < lo else mx
        raise IndexError(f"{what} {bad} is out of bounds for size {hi if size is None else size}")


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits: Tensor, labels: Tensor):
        squeeze = logits.dim() == 1
        l2 = (logits.unsqueeze(0) if squeeze else logits).contiguous()
        check_index_range(labels.reshape(-1), 0, l2.shape[-1], "Target")
        lab = labels.reshape(-1).to(device=l2.device, dtype=torch.int64).contiguous()
        rows = l2.shape[0]
        loss = torch.zeros(1, device=l2.device, dtype=torch.float64 if l2.dtype == torch.float64 else torch.float32)
        dh = torch.empty_like(l2)
        _ops().xent_head(l2, lab, rows, loss, 1.0 / rows, dh, 1.0 / rows, None, None, NO_EPI[0], NO_EPI[1], 0)
        ctx.save_for_backward(dh)
        ctx.squeeze = squeeze
        return loss.reshape(()).to(logits.dtype)

    @staticmethod
    def backward(ctx, g: Tensor):
        (dh,) = ctx.saved_tensors
        out = dh * g.to(dh.dtype)
        return (out.squeeze(0) if ctx.squeeze else out), None


def cross_entropy(logits: Tensor, labels: Tensor) -> Tensor:
    return _CrossEntropy.apply(logits, labels)


class _Mse(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y: Tensor, target: Tensor):
        shape = y.shape
        y2 = y.reshape(-1, shape[-1] if y.dim() > 0 else 1).contiguous()
        t2 = target.to(y.dtype).reshape(y2.shape).contiguous()
        n = y2.numel()
        loss = torch.zeros(1, device=y.device, dtype=torch.float64 if y2.dtype == torch.float64 else torch.float32)
        dh = torch.empty_like(y2)
        _ops().mse_head(y2, t2, y2.shape[0], loss, 1.0 / n, dh, 1.0 / n, None, NO_EPI[0], NO_EPI[1], 0)
        ctx.save_for_backward(dh)
        ctx.shape = shape
        return loss.reshape(()).to(y.dtype)

    @staticmethod
    def backward(ctx, g: Tensor):
        (dh,) = ctx.saved_tensors
        return (dh * g.to(dh.dtype)).reshape(ctx.shape), None


def mse_loss(y: Tensor, target: Tensor) -> Tensor:
    return _Mse.apply(y, target)


# --------------------------------------------------------------------------------------------
# batchnorm / embedding
# --------------------------------------------------------------------------------------------
class _BatchNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gain, bias, rmean, rvar, eps, momentum, training, sync):
        cols = x.shape[-1]
        xc = x.contiguous()
        y = torch.empty_like(xc)
        dev = x.device
        save_mean = torch.empty(cols, device=dev, dtype=torch.float64)
        save_inv = torch.empty(cols, device=dev, dtype=torch.float64)
        partial = torch.empty(2 * cols, device=dev, dtype=torch.float64)
        rows = xc.numel() // max(cols, 1)
        args = (xc, y, gain.detach().contiguous(), bias.detach().contiguous(), rmean, rvar, eps, momentum, training,
                rows, save_mean, save_inv, partial, NO_EPI[0], NO_EPI[1], 0)
        total = rows
        if sync is not None and training:  # synchronised statistics: sums -> all-reduce -> finalise
            _ops().batchnorm_fwd(*args, 1, 0)
            sync.all_reduce_(partial)
            total = int(sync.all_reduce_scalar(float(rows)))
            _ops().batchnorm_fwd(*args, 2, total)
        else:
            _ops().batchnorm_fwd(*args)
        ctx.save_for_backward(xc, y, gain, bias, save_mean, save_inv)
        ctx.rows = rows
        ctx.training = training
        ctx.sync = sync if training else None
        ctx.total = total
        return y

    @staticmethod
    def backward(ctx, g):
        xc, y, gain, bias, save_mean, save_inv = ctx.saved_tensors
        if not ctx.training:  # eval: y = gain * (x - mean) * invstd + bias
            gc = g.contiguous().to(xc.dtype)
            dx = gc * (gain.to(xc.dtype) * save_inv.to(xc.dtype))
            dgain = (gc * ((xc - save_mean.to(xc.dtype)) * save_inv.to(xc.dtype))).reshape(-1, xc.shape[-1]).sum(0)
            return dx, dgain.to(gain.dtype), gc.reshape(-1, xc.shape[-1]).sum(0).to(bias.dtype), None, None, None, \
                None, None
        dx = torch.empty_like(xc)
        dgain = torch.zeros_like(gain)
        dbias = torch.zeros_like(bias)
        partial = torch.empty(2 * xc.shape[-1], device=xc.device, dtype=torch.float64)
        args = (g.contiguous().to(xc.dtype), y, xc, dx, gain.detach().contiguous(), bias.detach().contiguous(),
                save_mean, save_inv, dgain, dbias, partial, ctx.rows, NO_EPI[0], NO_EPI[1], 0)
        if ctx.sync is not None:  # local parameter grads; dx from the global sums
            _ops().batchnorm_bwd(*args, 1, 0)
            ctx.sync.all_reduce_(partial)
            _ops().batchnorm_bwd(*args, 2, ctx.total)
        else:
            _ops().batchnorm_bwd(*args)
        return dx, dgain, dbias, None, None, None, None, None, None


def batchnorm(x: Tensor, gain: Tensor, bias: Tensor, rmean: Tensor, rvar: Tensor, eps: float, momentum: float,
              training: bool, sync=None) -> tuple[Tensor, Tensor, Tensor]:
    """Returns ``(y, running_mean, running_var)``; running stats are fresh tensors like the reference.
    ``sync``: a data-parallel context whose ranks share the batch statistics (synchronised BN)."""
    rm = rmean.detach().reshape(-1).to(gain.dtype).clone()
    rv = rvar.detach().reshape(-1).to(gain.dtype).clone()
    y = _BatchNorm.apply(x, gain, bias, rm, rv, float(eps), float(momentum), bool(training), sync)
    return y, rm, rv


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx: Tensor, table: Tensor):
        vocab = table.shape[0]
        check_index_range(idx.reshape(-1), -vocab, vocab, "index", vocab)  # negative ids wrap (Python indexing)
        ids = idx.to(device=table.device, dtype=torch.int64).contiguous()
        out = torch.empty(*ids.shape, table.shape[1], device=table.device, dtype=table.dtype)
        _ops().embedding_fwd(table.detach().contiguous(), ids, out)
        ctx.save_for_backward(ids)
        ctx.table_shape = table.shape
        ctx.table_dtype = table.dtype
        return out

    @staticmethod
    def backward(ctx, g: Tensor):
        (ids,) = ctx.saved_tensors
        acc = torch.float64 if ctx.table_dtype == torch.float64 else torch.float32
        dtable = torch.zeros(ctx.table_shape, device=g.device, dtype=acc)
        _ops().embedding_bwd(g.contiguous(), ids, dtable)
        return None, dtable.to(ctx.table_dtype)


def embedding(idx: Tensor, table: Tensor) -> Tensor:
    return _Embedding.apply(idx, table)


# --------------------------------------------------------------------------------------------
# statistics (N7)
# --------------------------------------------------------------------------------------------
def tensor_summary(t: Tensor, algo: str | None, bins: int) -> dict:
    """mean / unbiased std / saturation / density histogram of a GPU tensor, one D2H copy."""
    from ..utils.stats import saturation_rule
    x = t.detach().contiguous()
    if x.dtype not in (torch.float32, torch.float64, torch.bfloat16):
        x = x.float()
    dev = x.device
    rule, thr = saturation_rule(algo) if algo is not None else ("abs_gt", 0.0)
    moments = torch.empty(8, device=dev, dtype=torch.float64)
    row_len = x.shape[-1] if x.dim() > 0 else 1
    _ops().tensor_moments(x, row_len, SAT_CODES[rule] if algo is not None else 0, thr, moments)
    counts = None
    if bins > 0:
        counts = torch.zeros(bins, device=dev, dtype=torch.int64)  # exact counts (u64 atomics)
        _ops().histogram(x, moments[:2], bins, counts)
    host = torch.cat([moments, counts.double()]) if counts is not None else moments
    host = host.cpu().tolist()
    n = x.numel()
    mn, mx, s, ss, sat = host[0], host[1], host[2], host[3], host[4]
    mean = s / n if n else math.nan
    var = (ss - s * s / n) / (n - 1) if n > 1 else math.nan
    out = {"mean": mean, "std": math.sqrt(var) if var == var and var > 0 else (0.0 if var == var else math.nan)}
    if algo is not None:
        rows = n // max(row_len, 1) if rule in ("row_norm_gt", "row_max_gt") else n
        out["saturated"] = sat / rows if rows else math.nan
    if bins > 0:
        lo, hi = mn, mx
        if lo == hi:
            lo, hi = lo - 0.5, hi + 0.5
        width = (hi - lo) / bins
        c = host[8:8 + bins]
        total = sum(c)
        edges = [lo + i * width for i in range(bins)]
        dens = [v / (total * width) if total else 0.0 for v in c]
        out["histogram"] = {"x": edges, "y": dens}
    return out


__all__ = ["gemm", "gemm_path", "linear", "activation", "dropout", "softmax", "cross_entropy", "mse_loss",
           "batchnorm", "embedding", "tensor_summary", "epi_spec", "new_seed"]
