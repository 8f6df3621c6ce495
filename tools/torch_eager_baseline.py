"""Second baseline: plain PyTorch-ROCm eager (hipBLASLt GEMMs) on the bench config.

Measures (a) raw bf16 matmul throughput for the GEMM shapes of the flagship MLP and
(b) one full reference-semantics training step (dropout 0.2 on hidden outputs, CE on
pre-softmax logits, L2 on weights, Adam) written with stock torch ops in bf16 autocast.
"""
import json
import time
import torch
import torch.nn.functional as F


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    dev = "cuda"
    out = {"device": torch.cuda.get_device_name(0)}
    shapes = [(8192, 4096, 1024), (8192, 4096, 4096), (8192, 1024, 4096),
              (1024, 4096, 8192), (4096, 4096, 8192), (4096, 1024, 8192)]
    gemm = {}
    for m, n, k in shapes:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        b = torch.randn(k, n, device=dev, dtype=torch.bfloat16)
        t = bench(lambda: a @ b)
        gemm[f"{m}x{n}x{k}"] = round(2 * m * n * k / t / 1e12, 1)
    out["torch_matmul_bf16_TFLOPs"] = gemm

    sizes = [1024, 4096, 4096, 1024]
    B = 8192
    ws = [torch.nn.Parameter(torch.randn(i, o, device=dev) / i ** 0.5) for i, o in zip(sizes[:-1], sizes[1:])]
    bs = [torch.nn.Parameter(torch.zeros(o, device=dev)) for o in sizes[1:]]
    opt = torch.optim.Adam(ws + bs, lr=1e-3)
    x = torch.randn(B, sizes[0], device=dev)
    y = torch.randint(0, sizes[-1], (B,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            h = x @ ws[0] + bs[0]
            h = F.dropout(F.relu(h), 0.2)
            h = F.dropout(h @ ws[1] + bs[1], 0.2)
            h = F.dropout(F.relu(h), 0.2)
            logits = F.dropout(h @ ws[2] + bs[2], 0.2)
            loss = F.cross_entropy(logits.float(), y)
        loss = loss + 1e-3 * sum((w ** 2).sum() for w in ws)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()

    t = bench(step, iters=20, warm=5)
    out["eager_step_ms"] = round(t * 1e3, 3)
    out["eager_samples_per_s"] = round(B / t, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
