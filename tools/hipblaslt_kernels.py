"""Run hipBLASLt (torch.matmul / torch._scaled_mm) once per mlp4 / mlp8192 step GEMM shape, so that
`rocprofv3 --kernel-trace --stats` records the FULL names of the kernels hipBLASLt picks.

The names encode the Tensile solution parameters (macro tile MT, DepthU, wave grid, prefetch
depths, LDS layout ...) that tools/hipblaslt_disasm.py looks up in the on-box gfx950 code objects.
Usage: rocprofv3 --kernel-trace --stats -d gpurun_out/hbl -o hbl -- python tools/hipblaslt_kernels.py
"""
import torch

B = 8192
# name, M, N, K, A K-contiguous, B K-contiguous — the same operand layouts as tools/gemm_bench.py
CASES = [
    ("fwd_L1", B, 4096, 1024, True, False),
    ("fwd_L2", B, 4096, 4096, True, False),
    ("fwd_L3", B, 1024, 4096, True, False),
    ("dX_L3", B, 4096, 1024, True, True),
    ("dX_L2", B, 4096, 4096, True, True),
    ("dW_L3", 4096, 1024, B, False, False),
    ("dW_L2", 4096, 4096, B, False, False),
    ("dW_L1", 1024, 4096, B, False, False),
]
F8_CASES = [
    ("f8_8k_L1", B, 8192, 1024),
    ("f8_8k_L2", B, 1024, 8192),
    ("f8_fwd_L2", B, 4096, 4096),
]


def main():
    dev = "cuda"
    for name, M, N, K, akc, bkc in CASES:
        a = torch.randn((M, K) if akc else (K, M), device=dev).to(torch.bfloat16)
        b = torch.randn((N, K) if bkc else (K, N), device=dev).to(torch.bfloat16)
        A = a if akc else a.t()
        Bm = b.t() if bkc else b
        for _ in range(3):
            torch.matmul(A, Bm)
        torch.cuda.synchronize()
        print(name, "done", flush=True)
    one = torch.ones((), device=dev)
    for name, M, N, K in F8_CASES:
        a = torch.randn(M, K, device=dev).to(torch.float8_e4m3fn)
        b = torch.randn(N, K, device=dev).to(torch.float8_e4m3fn)
        try:
            for _ in range(3):
                torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            torch.cuda.synchronize()
            print(name, "done", flush=True)
        except RuntimeError as exc:
            print(name, "unavailable:", str(exc)[:160], flush=True)


if __name__ == "__main__":
    main()
