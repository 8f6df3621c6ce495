"""Headline benchmark: training samples/sec (whole node) of the flagship MLP on MI355X.

Metric / config from BASELINE.json: "training samples/sec (whole node), 4x8192 MLP bf16 at
1/2/4/8 MI355X" — the 4-size MLP [1024, 4096, 4096, 1024] (relu, relu, softmax; 25.2 M params)
at batch 8192 per GPU, bf16 compute with fp32 master weights, Adam. One timed step is exactly
the reference's per-epoch body (``neural_net_model.py:459-514``, BASELINE.md method C):
minibatch sampling, forward with dropout 0.2 on every hidden layer output, cross-entropy on the
logits, L2 (lambda 1e-3) on the weights, backward, Adam update, cost + weight-update-ratio
bookkeeping — run by the fused HIP engine, with the data-parallel gradient all-reduce (RCCL over
xGMI) overlapped with backward when launched with torchrun.

    python bench.py                                  # 1 GPU, defaults
    python bench.py --gpus 1 --steps 50 --warmup 10
    python bench.py --gpus 8 --steps 50 --warmup 10  # starts 8 rank processes itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

``--gpus N`` without a launcher (no ``WORLD_SIZE`` in the environment) makes this process a pure
launcher: it starts N fresh rank processes of this script (one per GPU, RCCL over xGMI) before
anything here touches the GPU, forwards their output and exits with the first failing rank's
code. With fewer visible GPUs than N the ranks rehearse over gloo, several per GPU (the JSON
says ``"backend": "gloo"``). A rank whose process group does not hold exactly N ranks exits
non-zero.

Scaling is WEAK: each GPU processes 8192 samples per step; ``value`` is the whole-job
samples/s. Data are synthetic (random inputs / labels of the config's shape), weights random.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REFERENCE_SAMPLES_PER_S = {  # BASELINE.md, reference on CPU fp64 (no published numbers exist)
    "mlp4": 2064.0,
    "mlp4_fp32": 2064.0,
    "mlp4_fp64": 1775.0,  # BASELINE.md method C via_lists (the per-epoch torch.tensor(list) build)
    "mlp4_fp64_autograd": 2064.0,
    "deep16x8192": 22.8,
    "mlp8192": 3095.0,
    "mlp8192_bf16": 3095.0,
}

CONFIGS = {
    "mlp4": dict(sizes=[1024, 4096, 4096, 1024], algos=["relu", "relu", "softmax"], batch=8192, dtype="bfloat16",
                 optimizer="adam", name="mlp[1024,4096,4096,1024] relu,relu,softmax (25.2M params)"),
    "deep16x8192": dict(sizes=[8192] * 17, algos=["relu"] * 15 + ["softmax"], batch=8192, dtype="bfloat16",
                        optimizer="stochastic", name="mlp[8192]x17 (16 hidden 8192-wide, 1.07B params)"),
    # BASELINE config 5: fp8 weights/activations on the e4m3 MFMA (forward GEMMs), bf16 backward
    "mlp8192": dict(sizes=[1024, 8192, 1024], algos=["relu", "softmax"], batch=8192, dtype="fp8",
                    optimizer="adam", name="mlp[1024,8192,1024] relu,softmax (16.8M params), fp8 e4m3 fwd GEMMs"),
    "mlp8192_bf16": dict(sizes=[1024, 8192, 1024], algos=["relu", "softmax"], batch=8192, dtype="bfloat16",
                         optimizer="adam", name="mlp[1024,8192,1024] relu,softmax (16.8M params)"),
    # the other reading of the metric name "4x8192 MLP": four 8192-wide layers, Adam (268M params)
    "mlp4x8192": dict(sizes=[8192] * 5, algos=["relu"] * 3 + ["softmax"], batch=8192, dtype="bfloat16",
                      optimizer="adam", name="mlp[8192]x5 (4 layers 8192-wide, 268M params)"),
    # the headline model at the reference's own precisions: fp32 on the fused engine (f32 MFMA
    # GEMMs); fp64 (f64 MFMA GEMMs, fp64 Adam) the way a REST user gets it — NeuralNetworkModel.train()
    # on Python lists (BASELINE.md method A), timed from the model's own progress timestamps; and
    # fp64 through the autograd engine (the reference epoch body, method C, on the GPU)
    "mlp4_fp32": dict(sizes=[1024, 4096, 4096, 1024], algos=["relu", "relu", "softmax"], batch=8192,
                      dtype="float32", optimizer="adam", name="mlp[1024,4096,4096,1024] relu,relu,softmax fp32"),
    "mlp4_fp64": dict(sizes=[1024, 4096, 4096, 1024], algos=["relu", "relu", "softmax"], batch=8192,
                      dtype="float64", optimizer="adam", engine="train",
                      name="mlp[1024,4096,4096,1024] relu,relu,softmax fp64 (NeuralNetworkModel.train, lists)"),
    "mlp4_fp64_autograd": dict(sizes=[1024, 4096, 4096, 1024], algos=["relu", "relu", "softmax"], batch=8192,
                               dtype="float64", optimizer="adam", engine="autograd",
                               name="mlp[1024,4096,4096,1024] relu,relu,softmax fp64 (autograd engine)"),
}
DTYPE_LABEL = {"bfloat16": "bf16", "fp8": "fp8", "float32": "fp32", "float64": "fp64"}


HEADLINE_METRIC = "training samples/sec (whole node), 4x8192 MLP bf16 at 1/2/4/8 MI355X"  # BASELINE.json


def _metric_label(key: str, cfg: dict) -> str:
    """BASELINE.json's metric string for the headline config; every other config names its own
    model and precision (same unit, same whole-node aggregation)."""
    if key == "mlp4":
        return HEADLINE_METRIC
    return f"training samples/sec (whole node), {cfg['name']}, {DTYPE_LABEL[cfg['dtype']]} on MI355X"


_JSON_FD = None  # the original stdout (main() points fd 1 at stderr)


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _launch_ranks(n: int, argv: list[str]) -> int:
    """Start ``n`` rank processes of this script and wait for them (this process never
    initialises the GPU: ``device_count`` does not, on this ROCm build)."""
    import signal
    import subprocess
    import tempfile

    # file rendezvous: a port picked here could be taken by someone else before rank 0 listens
    rdv_dir = tempfile.mkdtemp(prefix="pz_rdv_")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PZ_RENDEZVOUS_FILE=os.path.join(rdv_dir, "store"),
               WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), PZ_BENCH_LAUNCHER="self")
    visible = torch.cuda.device_count()
    if visible < n and "PZ_DIST_BACKEND" not in os.environ:
        log(f"{visible} GPU(s) visible for {n} ranks: rehearsing over gloo with ranks sharing GPUs")
        env["PZ_DIST_BACKEND"] = "gloo"
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r))))
    rc = 0
    alive = list(procs)
    while alive:
        for p in list(alive):
            code = p.poll()
            if code is None:
                continue
            alive.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log(f"rank process {p.pid} exited with {code}; stopping the others")
                for q in alive:  # our own children only, by exact pid
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    import shutil
    shutil.rmtree(rdv_dir, ignore_errors=True)
    return rc


def _emit(args, cfg, world, elapsed, costs, batch, ctx, trainer=None) -> None:
    finite = all(c == c and abs(c) != float("inf") for c in costs)
    ms = elapsed * 1e3 / args.steps
    global_batch = batch * world
    value = global_batch * args.steps / elapsed
    ref = REFERENCE_SAMPLES_PER_S.get(args.config)
    if ctx.rank != 0:
        return
    log(f"cost first/last = {costs[0]:.4f} / {costs[-1]:.4f}, finite={finite}")
    line = json.dumps({
        "metric": _metric_label(args.config, cfg),
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / ref, 2) if ref else None,
        "dtype": DTYPE_LABEL[cfg["dtype"]],
        "data": "synthetic (random inputs/labels, random-init weights)",
        "config": {"model": cfg["name"], "global_batch": global_batch, "per_gpu_batch": batch,
                   "seq_len": None, "parallelism": f"dp{world}", "optimizer": cfg["optimizer"],
                   "dist_backend": ctx.backend or "none", "dist_world_size": world,
                   "launcher": os.environ.get("PZ_BENCH_LAUNCHER", "torchrun" if world > 1 else "none"),
                   "dropout": args.dropout, "l2": args.l2, "config_key": args.config,
                   "engine": cfg.get("engine", "fused"),
                   # dense weight-gradient storage of the fused engine (PZ_GRAD_DTYPE: bf16 default,
                   # fp32 = exact fp32 gradients into the fp32-master Adam)
                   "grad_dtype": os.environ.get("PZ_GRAD_DTYPE", "bf16") if cfg["dtype"] in ("bfloat16", "fp8")
                   else DTYPE_LABEL[cfg["dtype"]],
                   # data parallel optimizer: "zero1" = reduce-scatter + 1/N slice updates + all-gather
                   # (engine/zero.py), "replicated" = all-reduce + full update on every rank
                   "optimizer_sharding": ("zero1" if getattr(trainer, "zero", None) is not None else "replicated")
                   if world > 1 or getattr(trainer, "zero", None) is not None else "none"},
    })
    if _JSON_FD is None:
        print(line, flush=True)
    else:
        os.write(_JSON_FD, (line + "\n").encode())


def _bench_autograd(args, cfg, model, ctx, batch, local) -> int:
    """The reference epoch body (BASELINE.md method C: forward with dropout, CE, L2, backward,
    optimizer step, update ratios on progress epochs) through the autograd engine on the GPU."""
    if ctx.world_size != 1:
        log("error: the autograd-engine bench runs on one GPU")
        return 2
    dev = torch.device("cuda", local)
    g = torch.Generator(device="cpu").manual_seed(99)
    n_data = args.n_data or 2 * batch
    data = torch.randn(n_data, cfg["sizes"][0], generator=g).to(dev, torch.float64)
    labels = torch.randint(0, cfg["sizes"][-1], (n_data,), generator=g).to(dev)
    total = args.warmup + args.steps
    every = max(1, total // 100)
    lr0, decay = args.lr, 0.999
    costs = []

    def run(epoch: int) -> None:
        picks = torch.randint(0, n_data, (batch,), device=dev)
        x, y = data[picks], labels[picks]
        for group in model.optimizer.param_groups:
            group["lr"] = lr0 * decay ** epoch
        prev = [w.detach().clone() for w in model.weights] if epoch % every == 0 else None
        for p in model.params:
            p.requires_grad_()
        _, cost = model._forward(x, y, args.dropout)
        cost = cost + args.l2 * sum((w ** 2).sum() for w in model.weights)
        for p in model.params:
            p.grad = None
        cost.backward()
        model.optimizer.step()
        if prev is not None:
            with torch.no_grad():
                [((w - pw).std() / (w.std() + 1e-8)) for pw, w in zip(prev, model.weights)]
        costs.append(cost.detach())

    for e in range(args.warmup):
        run(e)
    torch.cuda.synchronize()
    start = time.perf_counter()
    for e in range(args.warmup, total):
        run(e)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - start
    _emit(args, cfg, 1, elapsed, [float(c) for c in costs[args.warmup:]], batch, ctx)
    return 0


def _bench_train(args, cfg, model, ctx, batch) -> int:
    """The REST user's path: ``NeuralNetworkModel.train()`` on Python lists (the data a PUT /train/
    body carries), here on one GPU with the fused engine. ms/step comes from the model's own
    progress points (one per epoch; each carries the device-event time at which its step ended):
    the span from the end of the last warm-up epoch to the end of the last epoch, divided by
    --steps. The buffer gate (num_params samples, reference :429) is lowered to the data at hand."""
    import tempfile
    if ctx.world_size != 1:
        log("error: the train() bench runs on one GPU")
        return 2
    g = torch.Generator(device="cpu").manual_seed(99)
    n_data = args.n_data or batch
    x = torch.randn(n_data, cfg["sizes"][0], generator=g, dtype=torch.float64)
    y = torch.randint(0, cfg["sizes"][-1], (n_data,), generator=g)
    data = [(x[i].tolist(), [int(y[i])]) for i in range(n_data)]
    model.training_buffer_size = len(data)
    total = args.warmup + args.steps
    os.environ["PZ_MODELS_DIR"] = tempfile.mkdtemp(prefix="pz_bench_models_")
    t0 = time.time()
    model.train(data, epochs=total, learning_rate=args.lr, batch_size=batch, decay_rate=0.999,
                dropout_rate=args.dropout, l2_lambda=args.l2)
    log(f"train() of {total} epochs incl. checkpoints: {time.time() - t0:.1f}s, status {model.status}")
    from datetime import datetime
    pts = {p["epoch"]: p for p in model.progress}
    if len(pts) != total or args.warmup < 1:
        log(f"error: need one progress point per epoch and --warmup >= 1 (got {len(pts)} / {total})")
        return 2
    t_a = datetime.fromisoformat(pts[args.warmup]["dt"])
    t_b = datetime.fromisoformat(pts[total]["dt"])
    elapsed = (t_b - t_a).total_seconds()
    import shutil
    shutil.rmtree(os.environ["PZ_MODELS_DIR"], ignore_errors=True)
    _emit(args, cfg, 1, elapsed, [pts[e]["cost"] for e in range(args.warmup + 1, total + 1)], batch, ctx)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="mlp4", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: config)")
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--l2", type=float, default=1e-3)
    # learning checks (not the headline): --lr 0.05 --weight-algo he --n-data 8192 --dropout 0 --l2 0
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--weight-algo", default="xavier")
    ap.add_argument("--n-data", type=int, default=None, help="synthetic dataset rows (default 2 x batch)")
    raw = list(sys.argv[1:] if argv is None else argv)
    args = ap.parse_args(raw)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return _launch_ranks(args.gpus, raw)
    # stdout carries exactly ONE line, the JSON result: everything else written to fd 1 — RCCL's
    # version banner from its C library included — goes to stderr from here on
    global _JSON_FD
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
    from penr_oz_neural_network_torch_amd.parallel import init_from_env

    ctx = init_from_env()
    world, rank = ctx.world_size, ctx.rank
    if world != args.gpus:
        log(f"error: --gpus {args.gpus} but the process group holds {world} rank(s)")
        return 2
    # modulo: a gloo rehearsal (PZ_DIST_BACKEND=gloo) may put several ranks on one GPU
    local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(local)
    cfg = CONFIGS[args.config]
    batch = args.batch or cfg["batch"]

    torch.manual_seed(1234)
    model = NeuralNetworkModel("bench", cfg["sizes"], args.weight_algo, "zeros", cfg["algos"], cfg["optimizer"],
                               dtype=cfg["dtype"], device=f"cuda:{local}")
    if cfg.get("engine") == "autograd":
        return _bench_autograd(args, cfg, model, ctx, batch, local)
    if cfg.get("engine") == "train":
        return _bench_train(args, cfg, model, ctx, batch)
    trainer = FusedTrainer(model, ctx)
    n_data = args.n_data or 2 * batch
    g = torch.Generator(device="cpu").manual_seed(99 + rank)
    inputs = torch.randn(n_data, cfg["sizes"][0], generator=g)
    labels = torch.randint(0, cfg["sizes"][-1], (n_data,), generator=g)
    trainer.load_tensors(inputs, labels, seed=7 + rank)
    total = args.warmup + args.steps
    global_batch = batch * world
    lr0, decay = args.lr, 0.999
    # the schedule lets the trainer tabulate per-epoch hyper-parameters and replay captured
    # hipGraphs of the step (single GPU); steps are launched eagerly under data parallelism
    trainer.begin(total, lr_schedule=lambda e: lr0 * decay ** e)
    every = max(1, total // 100)

    def run(epoch: int) -> None:
        trainer.step(epoch, lr0 * decay ** epoch, global_batch, args.dropout, args.l2,
                     want_ratios=epoch % every == 0, record=False)

    t0 = time.time()
    for e in range(args.warmup):
        run(e)
    torch.cuda.synchronize()
    log(f"rank {rank}: warmup {args.warmup} steps done in {time.time() - t0:.2f}s")
    ctx.barrier()
    torch.cuda.synchronize()
    start = time.perf_counter()
    for e in range(args.warmup, total):
        run(e)
        if rank == 0 and (e - args.warmup) % 50 == 49:
            log(f"step {e - args.warmup + 1}/{args.steps}")
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - start
    elapsed = ctx.all_reduce_scalar_max(elapsed)

    costs = [c for _, c, _, _ in trainer.drain()]
    if os.environ.get("PZ_BENCH_SERIES") == "1" and rank == 0:  # per-step GPU periods (the trainer's events)
        log("step periods (ms): " + " ".join(f"{trainer.step_ms[e]:.3f}" for e in sorted(trainer.step_ms)))
    _emit(args, cfg, world, elapsed, costs, batch, ctx, trainer)
    from penr_oz_neural_network_torch_amd.parallel import shutdown
    shutdown()  # the native RCCL communicator, then the process group
    return 0


if __name__ == "__main__":
    sys.exit(main())
