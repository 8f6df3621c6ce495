"""REST additions and error paths beyond the reference's own suite: the optional ``dtype`` /
``device`` fields, the 409 while a model trains, the generic 500 handler and the uvicorn log
config (reference ``main.py:1-370`` behaviour contract)."""
import types

from fastapi.testclient import TestClient

import main
from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel


def test_create_with_dtype_and_device_fields(models_tmpdir):
    with TestClient(main.app) as client:
        r = client.post("/model/", json={"model_id": "f32", "layer_sizes": [3, 5, 2], "dtype": "float32",
                                         "device": "cpu", "activation_algos": ["relu", "softmax"]})
        assert r.status_code == 200, r.text
        m = NeuralNetworkModel.deserialize("f32")
        assert m.precision.name == "float32" and str(m.device) == "cpu"
        out = client.post("/output/", json={"model_id": "f32", "input": {"activation_vector": [1.0, 0.5, -1.0]}})
        assert out.status_code == 200 and len(out.json()["output_vector"]) == 2


def test_second_train_while_training_is_409(models_tmpdir, monkeypatch):
    """The per-model lock is checked before anything is loaded: a held lock answers 409."""
    with TestClient(main.app) as client:
        assert client.post("/model/", json={"model_id": "busy", "layer_sizes": [2, 4, 2],
                                            "activation_algos": ["tanh", "softmax"]}).status_code == 200
        data = [{"activation_vector": [i % 2, 1 - i % 2], "target_vector": [i % 2]} for i in range(40)]
        body = {"model_id": "busy", "training_data": data, "epochs": 2, "batch_size": 4}
        monkeypatch.setitem(main.model_locks, "busy", types.SimpleNamespace(locked=lambda: True))
        r = client.put("/train/", json=body)
        assert r.status_code == 409 and "already in progress" in r.json()["detail"]
        monkeypatch.delitem(main.model_locks, "busy")
        assert client.put("/train/", json=body).status_code == 202


def test_unexpected_errors_map_to_500(models_tmpdir, monkeypatch):
    def boom(*a, **k):
        raise RuntimeError("disk on fire")
    monkeypatch.setattr(NeuralNetworkModel, "deserialize", staticmethod(boom))
    with TestClient(main.app, raise_server_exceptions=False) as client:
        r = client.get("/progress/", params={"model_id": "x"})
        assert r.status_code == 500 and r.json() == {"detail": "Please refer to server logs"}


def test_uvicorn_log_config_routes_through_the_service_format():
    cfg = main._uvicorn_log_config()
    assert cfg["formatters"]["default"]["format"] == main.LOG_FORMAT
    assert set(cfg["loggers"]) == {"uvicorn", "uvicorn.error", "uvicorn.access"}
    assert all(not v["propagate"] for v in cfg["loggers"].values())


def test_progress_answers_while_train_loads_a_large_checkpoint(models_tmpdir, monkeypatch):
    """PUT /train/ parses the checkpoint off the event loop — a /progress/ poll is
    answered while a (slow, large) checkpoint loads, and a second PUT /train/ for the same model in
    that window is a 409, not a second training."""
    import threading
    import time

    with TestClient(main.app) as client:
        assert client.post("/model/", json={"model_id": "big", "layer_sizes": [2, 4, 2],
                                            "activation_algos": ["tanh", "softmax"]}).status_code == 200
        real = NeuralNetworkModel.deserialize.__func__
        loading = threading.Event()

        def slow(cls, model_id, meta_only=False):
            if not meta_only:  # the full parse of a large checkpoint
                loading.set()
                time.sleep(1.5)
            return real(cls, model_id, meta_only=meta_only)

        monkeypatch.setattr(NeuralNetworkModel, "deserialize", classmethod(slow))
        data = [{"activation_vector": [i % 2, 1 - i % 2], "target_vector": [i % 2]} for i in range(40)]
        body = {"model_id": "big", "training_data": data, "epochs": 2, "batch_size": 4}
        res = {}
        t = threading.Thread(target=lambda: res.setdefault("train", client.put("/train/", json=body)))
        t.start()
        assert loading.wait(10)
        t0 = time.perf_counter()
        r = client.get("/progress/", params={"model_id": "big"})
        dt = time.perf_counter() - t0
        assert r.status_code == 200 and dt < 0.5, dt  # (the loop is not parsing: well under the 1.5 s load)
        assert client.put("/train/", json=body).status_code == 409  # still loading: in progress
        t.join(30)
        assert res["train"].status_code == 202
