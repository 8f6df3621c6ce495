"""Micro-benchmark of the pz MFMA GEMM on the flagship step's shapes (+ hipBLASLt reference).

Each case runs 30 timed launches after 5 warm-ups on random bf16 data; prints TFLOP/s for the
fused-epilogue variant, the plain-store variant, and torch.matmul on the same operands.
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from penr_oz_neural_network_torch_amd.ops import functional as PF  # noqa: E402


def timeit(fn, n=30, w=5):
    for _ in range(w):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e-3


def main():
    dev = "cuda"
    B = 8192
    cases = [  # name, M, N, K, a_kc, b_kc, out dtype, mode — the default rows are the mlp4 step's
        # GEMMs with the epilogue kinds the trainer runs: forward stages writing the ReLU bitmask,
        # dX reading it (+ bias-gradient column sums), dW straight into the bf16 gradient buffer
        ("fwd_L1", B, 4096, 1024, True, False, torch.bfloat16, "fwd_mask"),
        ("fwd_L2", B, 4096, 4096, True, False, torch.bfloat16, "fwd_mask"),
        ("fwd_L3", B, 1024, 4096, True, False, torch.bfloat16, "fwd_nodrop"),
        ("dX_L3", B, 4096, 1024, True, True, torch.bfloat16, "bwd_mask"),
        ("dX_L2", B, 4096, 4096, True, True, torch.bfloat16, "bwd_mask"),
        ("dW_L3", 4096, 1024, B, False, False, torch.bfloat16, "store"),
        ("dW_L2", 4096, 4096, B, False, False, torch.bfloat16, "store"),
        ("dW_L1", 1024, 4096, B, False, False, torch.bfloat16, "store"),
        # the previous rows' generic kinds: aux-derivative dX, fp32 weight gradients
        ("dX_L2_aux", B, 4096, 4096, True, True, torch.bfloat16, "bwd"),
        ("dW_L2_f32", 4096, 4096, B, False, False, torch.float32, "store"),
        # epilogue probes (only run when named): fwd_L2 with parts of the stage math
        ("fwdL2_bias", B, 4096, 4096, True, False, torch.bfloat16, "fwd_bias"),
        ("fwdL2_relu", B, 4096, 4096, True, False, torch.bfloat16, "fwd_relu"),
        ("fwdL2_drop1", B, 4096, 4096, True, False, torch.bfloat16, "fwd_nodrop"),
        ("dXL3_nodrop", B, 4096, 1024, True, True, torch.bfloat16, "bwd_nodrop"),
        # the trainer's actual epilogues: ReLU bitmask written by the forward, read by dX
        ("fwdL1_mask", B, 4096, 1024, True, False, torch.bfloat16, "fwd_mask"),
        ("fwdL2_mask", B, 4096, 4096, True, False, torch.bfloat16, "fwd_mask"),
        ("dXL3_mask", B, 4096, 1024, True, True, torch.bfloat16, "bwd_mask"),
        # one dropout instead of two in front of the ReLU mask (the hashing's share of the epilogue)
        ("fwdL1_mask1", B, 4096, 1024, True, False, torch.bfloat16, "fwd_mask1"),
        ("fwdL1_mask0", B, 4096, 1024, True, False, torch.bfloat16, "fwd_mask0"),  # ReLU + mask, no dropout
        ("fwdL1_bias", B, 4096, 1024, True, False, torch.bfloat16, "fwd_bias"),
        ("fwdL1_relu", B, 4096, 1024, True, False, torch.bfloat16, "fwd_relu"),
        ("fwdL1_nobias", B, 4096, 1024, True, False, torch.bfloat16, "fwd_nobias"),  # EPI_FWD, nothing enabled
        ("storeL1_bias", B, 4096, 1024, True, False, torch.bfloat16, "store_bias"),  # EPI_STORE + bias
        ("fwdL2_mask1", B, 4096, 4096, True, False, torch.bfloat16, "fwd_mask1"),
        ("dXL3_mask_nocs", B, 4096, 1024, True, True, torch.bfloat16, "bwd_mask_nocs"),
        ("dXL2_mask", B, 4096, 4096, True, True, torch.bfloat16, "bwd_mask"),
        # e4m3 forward GEMMs (run when named): mlp8192 layers and the mlp4 middle layer
        ("f8_8k_L1", B, 8192, 1024, True, True, "fp8", "fwd"),
        ("f8_8k_L2", B, 1024, 8192, True, True, "fp8", "fwd_nodrop"),
        ("f8_fwd_L2", B, 4096, 4096, True, True, "fp8", "fwd"),
        # the trainer's fp8 fast paths: natural [in, out] e4m3 weights (VAR 15 / 16) with the ReLU
        # bitmask epilogue, and the e5m2 x e4m3 dX with the bitmask derivative (VAR 9 / 17)
        ("f8n_8k_L1", B, 8192, 1024, True, False, "fp8", "fwd_mask"),
        ("f8_8k_dX", B, 8192, 1024, True, True, "fp8bwd", "bwd_mask"),
        ("bf_8k_L1", B, 8192, 1024, True, False, torch.bfloat16, "fwd"),
        ("bf_8k_L2", B, 1024, 8192, True, False, torch.bfloat16, "fwd_nodrop"),
    ]
    only = sys.argv[1:] or None
    out = {}
    for name, M, N, K, akc, bkc, odt, mode in cases:
        if (only and name not in only) or (not only and "_" in name.split("L")[-1][1:]):
            continue
        fp8 = odt in ("fp8", "fp8bwd")
        idt = torch.float8_e4m3fn if fp8 else torch.bfloat16
        adt = torch.float8_e5m2 if odt == "fp8bwd" else idt
        odt = torch.bfloat16 if fp8 else odt
        a = torch.randn((M, K) if akc else (K, M), device=dev).to(adt)
        b = torch.randn((N, K) if bkc else (K, N), device=dev).to(idt)
        c = torch.empty(M, N, device=dev, dtype=odt)
        bias = torch.randn(N, device=dev)
        aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
        colsum = torch.zeros(N, device=dev)
        epi = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, drop_post=2, p=0.2, seed=(1, 2))
        mask = torch.randint(0, 256, PF.relu_mask_shape(M, N), device=dev, dtype=torch.uint8)
        if mode == "fwd":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=epi)
        elif mode == "fwd_nodrop":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD,
                                    epi=PF.epi_spec(drop_pre=3, p=0.2, seed=(1, 2)))
        elif mode == "fwd_bias":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=PF.epi_spec())
        elif mode == "fwd_nobias":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, mode=PF.EPI_FWD, epi=PF.epi_spec())
        elif mode == "store_bias":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias)
        elif mode == "fwd_relu":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=PF.epi_spec(act=PF.ACT_RELU))
        elif mode == "bwd_nodrop":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, aux=aux, colsum=colsum, mode=PF.EPI_BWD,
                                    epi=PF.epi_spec(act=PF.ACT_RELU))
        elif mode == "fwd_mask":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=epi, mask=mask)
        elif mode == "fwd_mask1":
            e1 = PF.epi_spec(act=PF.ACT_RELU, drop_pre=1, p=0.36, seed=(1, 2))
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=e1, mask=mask)
        elif mode == "fwd_mask0":
            e0 = PF.epi_spec(act=PF.ACT_RELU)
            fused = lambda: PF.gemm(a, akc, b, bkc, c, bias=bias, mode=PF.EPI_FWD, epi=e0, mask=mask)
        elif mode == "bwd_mask":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, colsum=colsum, mode=PF.EPI_BWD, epi=epi, mask=mask)
        elif mode == "bwd_mask_nocs":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, mode=PF.EPI_BWD, epi=epi, mask=mask)
        elif mode == "bwd":
            fused = lambda: PF.gemm(a, akc, b, bkc, c, aux=aux, colsum=colsum, mode=PF.EPI_BWD, epi=epi)
        else:
            fused = lambda: PF.gemm(a, akc, b, bkc, c)
        plain = lambda: PF.gemm(a, akc, b, bkc, c)
        A = a if akc else a.t()
        Bm = b.t() if bkc else b
        if fp8:  # hipBLASLt fp8 GEMM through torch._scaled_mm (row-major A, column-major B)
            one = torch.ones((), device=dev)
            bt = b if bkc else b.t().contiguous()  # [N, K]: column-major B
            ref = lambda: torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        else:
            ref = lambda: torch.matmul(A, Bm)
        fl = 2.0 * M * N * K
        best = {"fused_TF": 0.0, "plain_TF": 0.0, "hipblaslt_TF": 0.0}
        for _ in range(3):  # interleaved rounds, best of 3: the clock drifts between cases
            for key, fn in (("fused_TF", fused), ("plain_TF", plain), ("hipblaslt_TF", ref)):
                try:
                    best[key] = max(best[key], round(fl / timeit(fn) / 1e12, 1))
                except RuntimeError as exc:  # e.g. no hipBLASLt fp8 kernel for this shape
                    print(name, key, "unavailable:", str(exc)[:120], flush=True)
                    best[key] = None
                    ref = plain
        r = best
        out[name] = r
        print(name, r, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
