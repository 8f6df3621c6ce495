"""fp64 / fp32 GEMM throughput on the matrix cores (csrc/gemm_wide.hip) for the flagship MLP's
shapes, against the generic VALU tile and torch.matmul (rocBLAS) on the same data.

    python tools/gemm_wide_bench.py [fp64|fp32 ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from penr_oz_neural_network_torch_amd.ops import functional as PF  # noqa: E402


def timeit(fn, n=10, w=3):
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
    B = 8192
    cases = [("fwd_L1", B, 4096, 1024, True, False), ("fwd_L2", B, 4096, 4096, True, False),
             ("dX_L2", B, 4096, 4096, True, True), ("dW_L2", 4096, 4096, B, False, False)]
    dtypes = {"fp64": torch.float64, "fp32": torch.float32}
    want = sys.argv[1:] or list(dtypes)
    out = {}
    for dname in want:
        dt = dtypes[dname]
        for name, M, N, K, akc, bkc in cases:
            a = torch.rand((M, K) if akc else (K, M), device="cuda", dtype=dt) * 2 - 1
            b = torch.rand((N, K) if bkc else (K, N), device="cuda", dtype=dt) * 2 - 1
            c = torch.empty(M, N, device="cuda", dtype=dt)
            A = a if akc else a.t()
            Bm = b.t() if bkc else b
            fl = 2.0 * M * N * K
            r = {"path": PF.gemm_path(a, akc, b, bkc, c)}
            for key, fn in (("mfma_TF", lambda: PF.gemm(a, akc, b, bkc, c)),
                            ("generic_TF", lambda: PF.gemm(a, akc, b, bkc, c, force_generic=True)),
                            ("rocblas_TF", lambda: torch.matmul(A, Bm))):
                r[key] = round(fl / timeit(fn) / 1e12, 1)
            out[f"{dname}_{name}"] = r
            print(dname, name, r, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
