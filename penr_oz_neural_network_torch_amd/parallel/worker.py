"""Worker rank of the REST service's data-parallel train group (see :mod:`.service`).

Started by the server process with RANK / WORLD_SIZE / PZ_RENDEZVOUS_FILE / PZ_CTRL_ADDR /
PZ_CTRL_KEY in its environment. It binds its GPU (``LOCAL_RANK``), connects the control socket,
joins the process group (file rendezvous in the group generation's own directory), reports
``ready`` and then serves ``load`` → (``go`` | ``abort``) → ``train`` commands until ``stop``. Every
rank reads the shared ``models/`` directory; only rank 0 writes it.
"""
from __future__ import annotations

import logging
import os
import sys
from datetime import timedelta
from multiprocessing.connection import Client

log = logging.getLogger("pz.worker")


def main() -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - rank%(rank)s - %(name)s - %(levelname)s - %(message)s"
                        .replace("%(rank)s", os.environ.get("RANK", "?")))
    import torch
    import torch.distributed as dist

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    backend = os.environ.get("PZ_DIST_BACKEND", "nccl")
    host, port = os.environ["PZ_CTRL_ADDR"].rsplit(":", 1)
    conn = Client((host, int(port)), authkey=bytes.fromhex(os.environ["PZ_CTRL_KEY"]))
    conn.send(rank)
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    try:
        dist.init_process_group(backend, init_method="file://" + os.environ["PZ_RENDEZVOUS_FILE"], rank=rank,
                                world_size=world,
                                timeout=timedelta(seconds=float(os.environ.get("PZ_DIST_TIMEOUT_S", "600"))))
    except Exception as e:
        conn.send(f"{type(e).__name__}: {e}")
        return 1
    conn.send("ready")
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
    from penr_oz_neural_network_torch_amd.parallel.dist import DataParallelContext, set_context
    comm = os.environ.get("PZ_GRAD_COMM_DTYPE")
    ctx = DataParallelContext(rank, world, None, torch.bfloat16 if comm in ("bf16", "bfloat16") else None)
    set_context(ctx)
    while True:
        try:
            cmd = conn.recv()
        except EOFError:
            break
        if not isinstance(cmd, dict) or cmd.get("op") == "stop":
            break
        try:
            model = NeuralNetworkModel.deserialize(cmd["model_id"])
            model._context = ctx
        except Exception as e:  # reported to rank 0, which aborts the whole group training
            conn.send(f"{type(e).__name__}: {e}")
            conn.recv()
            continue
        conn.send("ok")
        if conn.recv() != "go":
            continue
        try:
            model.train(cmd["data"], **cmd["hp"])
            conn.send("done")
        except Exception as e:
            log.exception("training failed on this rank")
            conn.send(f"failed: {type(e).__name__}: {e}")
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
