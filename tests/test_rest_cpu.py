"""REST service end-to-end on the CPU (real model, background training actually runs)."""
import os
import subprocess
import sys
import time

import pytest
from fastapi.testclient import TestClient

import main

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wait_trained(client, model_id, timeout=60.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        r = client.get("/progress/", params={"model_id": model_id})
        assert r.status_code == 200, r.text  # atomic checkpoint writes: never a torn read (400)
        if r.json()["status"] == "Trained":
            return r.json()
        time.sleep(0.05)
    raise AssertionError("training did not finish")


def test_full_lifecycle(models_tmpdir):
    with TestClient(main.app) as client:
        r = client.post("/model/", json={"model_id": "m", "layer_sizes": [4, 8, 2],
                                         "activation_algos": ["relu", "softmax"], "optimizer": "stochastic"})
        assert r.status_code == 200 and r.json() == {"message": "Model m created and saved successfully"}
        data = [{"activation_vector": [i % 3, 1, 0, -1], "target_vector": [i % 2]} for i in range(64)]
        r = client.put("/train/", json={"model_id": "m", "training_data": data, "epochs": 20, "batch_size": 16,
                                        "learning_rate": 0.1, "decay_rate": 1.0})
        assert r.status_code == 202
        prog = _wait_trained(client, "m")
        assert len(prog["progress"]) == 20 and prog["average_cost"] is not None
        stats = client.get("/stats/", params={"model_id": "m"}).json()
        assert [l["algo"] for l in stats["layers"]] == ["linear", "relu", "linear", "softmax"]
        assert stats["weights"][1] is None and stats["weights"][0]["shape"] == "(4, 8)"
        out = client.post("/output/", json={"model_id": "m", "input": {"activation_vector": [1, 1, 0, -1],
                                                                         "target_vector": [1]}}).json()
        assert len(out["output_vector"]) == 2 and out["cost"] is not None
        assert client.delete("/model/", params={"model_id": "m"}).status_code == 204
        assert client.get("/progress/", params={"model_id": "m"}).status_code == 404


def test_buffering_and_conflict(models_tmpdir):
    with TestClient(main.app) as client:
        client.post("/model/", json={"model_id": "b", "layer_sizes": [9, 9, 9], "activation_algos": ["relu"] * 2})
        r = client.put("/train/", json={"model_id": "b", "training_data": [
            {"activation_vector": [0] * 9, "target_vector": [0] * 9}], "epochs": 1})
        assert r.status_code == 202
        time.sleep(0.2)
        prog = client.get("/progress/", params={"model_id": "b"}).json()
        assert prog["status"] == "Created"  # buffered only: 1 sample < 180 required


def test_train_start_failure_does_not_leave_a_stale_409(models_tmpdir, monkeypatch):
    """An exception between the checkpoint load and the task start (here: create_task itself) must
    not leave the model marked as starting (every later PUT /train/ answered 409)."""
    client = TestClient(main.app, raise_server_exceptions=False)
    client.post("/model/", json={"model_id": "s", "layer_sizes": [9, 9, 9], "activation_algos": ["relu"] * 2})
    body = {"model_id": "s", "training_data": [{"activation_vector": [0] * 9, "target_vector": [0] * 9}],
            "epochs": 1}

    def boom(coro):
        coro.close()
        raise RuntimeError("no task for you")

    with monkeypatch.context() as m:
        m.setattr(main, "create_task", boom)
        assert client.put("/train/", json=body).status_code == 500
        assert "s" not in main._starting
    with TestClient(main.app) as c2:
        assert c2.put("/train/", json=body).status_code == 202


def test_dashboard_assets_and_health(models_tmpdir):
    client = TestClient(main.app)
    r = client.get("/")
    assert r.status_code == 200 and r.url.path == "/dashboard"
    assert "Neural Network Model Dashboard" in r.text
    for asset in ("dashboard.js", "plot.js", "dashboard.css", "favicon.svg"):
        assert client.get(f"/static/{asset}").status_code == 200
    h = client.get("/health").json()
    assert h["status"] == "ok"


def test_validation_errors(models_tmpdir):
    client = TestClient(main.app, raise_server_exceptions=False)
    assert client.post("/output/", json={"model_id": "x"}).status_code == 422
    r = client.post("/output/", json={"model_id": "nope", "input": {"activation_vector": [0]}})
    assert r.status_code == 404 and "not created yet" in r.json()["detail"]
    r = client.post("/model/", json={"model_id": "bad", "layer_sizes": [2, 2], "activation_algos": ["nope"]})
    assert r.status_code == 400 and "Unsupported activation algorithm: nope" in r.json()["detail"]


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference checkout not mounted")
def test_reference_test_suite_passes_against_this_framework(tmp_path):
    """Run the reference repo's own 65 tests against our modules (parameterized shim)."""
    for name in ("test_main.py", "test_neural_net_model.py", "test_torch_backward.py"):
        with open(os.path.join("/root/reference", name)) as src, open(tmp_path / name, "w") as dst:
            dst.write(src.read())
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([ROOT, os.path.join(ROOT, "tests", "_shims")]))
    res = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider", "."], cwd=tmp_path,
                         env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]
    assert "65 passed" in res.stdout
