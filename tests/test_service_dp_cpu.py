"""The REST service's multi-rank train group (parallel/service.py) on the CPU: ``PUT /train/``
drives a 2-rank gloo data-parallel training (two rank processes started by the app's lifespan;
the server process never joins the group) — the code path an 8-GPU node runs over RCCL."""
import threading
import time

import pytest
from fastapi.testclient import TestClient

import main


def _wait(client, model_id, want, timeout=120.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        r = client.get("/progress/", params={"model_id": model_id})
        assert r.status_code == 200, r.text
        if r.json()["status"] in want:
            return r.json()
        time.sleep(0.05)
    raise AssertionError(f"{model_id} did not reach {want}")


def _group_ready(client, timeout=120.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        g = client.get("/health").json()["train_group"]
        assert g is not None
        if g["ready"]:
            assert g["healthy"], g
            return g
        time.sleep(0.1)
    raise AssertionError("train group did not come up")


def _wait_trainings(client, n, timeout=60.0):
    """The model reads "Trained" as soon as rank 0's train() returns; the group counts the training
    once every worker has reported back — poll for that."""
    t0 = time.time()
    while client.get("/health").json()["train_group"]["trainings"] < n:
        assert time.time() - t0 < timeout, client.get("/health").json()["train_group"]
        time.sleep(0.02)
    return client.get("/health").json()["train_group"]


def test_train_route_runs_on_two_ranks(models_tmpdir, monkeypatch):
    monkeypatch.setenv("PZ_SERVICE_GPUS", "2")
    monkeypatch.setenv("PZ_DIST_BACKEND", "gloo")
    with TestClient(main.app) as client:
        g = _group_ready(client)
        assert g["world_size"] == 2 and g["backend"] == "gloo"
        r = client.post("/model/", json={"model_id": "dp", "layer_sizes": [4, 8, 2], "optimizer": "adam",
                                         "activation_algos": ["tanh", "softmax"]})
        assert r.status_code == 200
        data = [{"activation_vector": [i % 3, 1, 0, -(i % 2)], "target_vector": [i % 2]} for i in range(64)]
        r = client.put("/train/", json={"model_id": "dp", "training_data": data, "epochs": 8, "batch_size": 17,
                                        "learning_rate": 0.05, "decay_rate": 1.0})
        assert r.status_code == 202
        prog = _wait(client, "dp", ("Trained", "Failed"))
        assert prog["status"] == "Trained"
        assert len(prog["progress"]) == 8 and all(p["world_size"] == 2 for p in prog["progress"])
        assert _wait_trainings(client, 1)["trainings"] == 1
        # a sample smaller than the group fails on every rank (no hang) and the group survives it
        r = client.put("/train/", json={"model_id": "dp", "training_data": data, "epochs": 2, "batch_size": 1})
        assert r.status_code == 202
        assert _wait(client, "dp", ("Failed",))["status"] == "Failed"
        g = client.get("/health").json()["train_group"]
        assert g["healthy"] and g["trainings"] == 1
        r = client.put("/train/", json={"model_id": "dp", "training_data": data, "epochs": 2, "batch_size": 8})
        assert r.status_code == 202
        assert _wait(client, "dp", ("Trained",))["status"] == "Trained"
        assert _wait_trainings(client, 2)["trainings"] == 2


def _health_group(client):
    return client.get("/health").json()["train_group"]


def test_group_recovers_from_lost_workers(models_tmpdir, monkeypatch):
    """a rank that dies (idle, or in the middle of a training) is detected by the
    watchdog; an in-flight training fails promptly instead of waiting out the collective timeout
    (the checkpoint reads "Failed" although the rank that writes it died), and the next
    ``PUT /train/`` brings a fresh group up (new processes, new rendezvous) and trains."""
    from penr_oz_neural_network_torch_amd.parallel import service
    monkeypatch.setenv("PZ_SERVICE_GPUS", "2")
    monkeypatch.setenv("PZ_DIST_BACKEND", "gloo")
    with TestClient(main.app) as client:
        _group_ready(client)
        r = client.post("/model/", json={"model_id": "ft", "layer_sizes": [4, 8, 2], "optimizer": "adam",
                                         "activation_algos": ["tanh", "softmax"]})
        assert r.status_code == 200
        data = [{"activation_vector": [i % 3, 1, 0, -(i % 2)], "target_vector": [i % 2]} for i in range(64)]
        short = {"model_id": "ft", "training_data": data, "epochs": 3, "batch_size": 8}
        group = service.get_group()

        # 1) idle rank 1 killed: the watchdog marks the group lost, the next training restarts it
        group.procs[1].kill()
        t0 = time.time()
        while _health_group(client)["lost"] is None:
            assert time.time() - t0 < 10, "watchdog did not notice the dead worker"
            time.sleep(0.05)
        assert not _health_group(client)["healthy"]
        assert client.put("/train/", json=short).status_code == 202
        assert _wait(client, "ft", ("Trained", "Failed"))["status"] == "Trained"
        g = _wait_trainings(client, 1)
        assert g["healthy"] and g["restarts"] == 1 and g["trainings"] == 1

        # 2) rank 0 (the checkpoint writer) killed in the middle of a training: prompt failure,
        #    status "Failed" written by the server, then a fresh group
        long = dict(short, epochs=200000)
        assert client.put("/train/", json=long).status_code == 202
        _wait(client, "ft", ("Training",))
        time.sleep(0.5)
        victim = group.procs[0]
        victim.kill()
        t0 = time.time()
        assert _wait(client, "ft", ("Failed", "Trained"), timeout=60)["status"] == "Failed"
        assert time.time() - t0 < 60
        assert client.put("/train/", json=short).status_code == 202
        t0 = time.time()  # (the status reads "Failed" until the new training starts)
        while _health_group(client)["trainings"] < 2:
            assert time.time() - t0 < 120, _health_group(client)
            time.sleep(0.05)
        assert _wait(client, "ft", ("Trained",))["status"] == "Trained"
        g = _health_group(client)
        assert g["healthy"] and g["restarts"] == 2 and g["trainings"] == 2
        assert group.procs[0] is not victim and all(p.poll() is None for p in group.procs)


def test_collect_straggler_deadline_and_lose_keeps_a_finished_model(models_tmpdir):
    """a rank still silent long after a peer reported the end of the training is hung
    and must not hold the group lock forever (straggler deadline); and losing the group after
    rank 0 persisted a finished ("Trained") checkpoint must not rewrite it as "Failed"."""
    from multiprocessing import Pipe

    from neural_net_model import NeuralNetworkModel
    from penr_oz_neural_network_torch_amd.parallel.service import TrainGroup
    from penr_oz_neural_network_torch_amd.utils import checkpoint as ckpt

    class _Listener:
        def close(self):
            pass

    g = TrainGroup.__new__(TrainGroup)
    (a0, b0), (a1, b1) = Pipe(), Pipe()
    g.conns, g.procs, g._lost, g._listener, g._rdv_dir = [a0, a1], [], None, _Listener(), None
    b0.send("done")  # rank 0 finished, rank 1 never answers
    t0 = time.time()
    assert g._collect(None, straggler_s=0.5) == ["done", None]
    assert time.time() - t0 < 10
    b1.send("done")
    g2 = TrainGroup.__new__(TrainGroup)
    g2.conns, g2._lost = [a1], None
    assert g2._collect(None, straggler_s=0.5) == ["done"]  # nobody late: no deadline hit

    # rank 0 answers last (its final checkpoint write) -- within its grace window it is
    # not a straggler; past it, it is
    (c0, d0), (c1, d1) = Pipe(), Pipe()
    g3 = TrainGroup.__new__(TrainGroup)
    g3.conns, g3._lost = [c0, c1], None
    d1.send("done")
    threading.Timer(0.8, lambda: d0.send("done")).start()  # after the 0.3 s peer window
    assert g3._collect(None, straggler_s=0.3, rank0_grace_s=5.0) == ["done", "done"]
    d1.send("done")
    t0 = time.time()
    assert g3._collect(None, straggler_s=0.2, rank0_grace_s=0.3) == [None, "done"]
    assert time.time() - t0 < 10

    for status, rank0_done, want in (("Trained", False, "Trained"), ("Training", True, "Training"),
                                     ("Training", False, "Failed")):
        m = NeuralNetworkModel("lose", [4, 8, 2], activation_algos=["tanh", "softmax"])
        m.status = status
        m.serialize()
        g._lost = None
        g._lose("test", "lose", rank0_done=rank0_done)
        assert ckpt.load_meta("lose")["status"] == want, (status, rank0_done)
    g._lose("test", "no_such_model")  # nothing persisted: nothing to mark, no error
