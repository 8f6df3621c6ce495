"""The model-side orchestration of the fused GPU engine (``NeuralNetworkModel._train_fused``,
``_drain_progress``, ``_record_fused``; reference epoch loop ``neural_net_model.py:457-522``) on the
CPU, against a recording stand-in for ``engine.trainer.FusedTrainer`` — the GPU tier runs the
real engine (tests/test_engine_gpu.py). Checks the step schedule (learning-rate decay, progress
epochs, record step), the progress points' telemetry fields, and the final stats / status."""
import types

import torch

from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
from penr_oz_neural_network_torch_amd.models import network as network_mod


class FakeTrainer:
    """Stand-in with FusedTrainer's interface; the record step computes real activations and
    gradients with the model's CPU forward so the stats code sees genuine tensors."""

    def __init__(self, model):
        self.model = model
        self.ctx = types.SimpleNamespace(world_size=1, enabled=False)
        self.dev = torch.device("cpu")
        self.steps, self._pending, self.step_ms, self._rec = [], [], {}, None

    def load_data(self, data):
        self.data = data

    def begin(self, epochs, lr_schedule=None):
        self.schedule = [lr_schedule(e) for e in range(epochs)]

    def step(self, epoch, lr, sample_size, dropout, l2, want_ratios, record):
        self.steps.append(dict(epoch=epoch, lr=lr, sample_size=sample_size, dropout=dropout, l2=l2,
                               want_ratios=want_ratios, record=record))
        self._pending.append((epoch, want_ratios))
        if record:
            m = self.model
            m._fake_gpu = False  # the stand-in's own forward takes the CPU path
            inputs = m._input_tensor([inp for inp, _ in self.data[:8]])
            target = [tgt for _, tgt in self.data[:8]]
            for p in m.params:
                p.requires_grad_()
                p.grad = None
            acts, cost = m._forward(inputs, target, 0.0)
            for a in acts:
                a.retain_grad()
            cost.backward()
            wg = [layer.weights.grad if layer.weights is not None else None for layer in m.layers]
            self._rec = {"activations": acts, "act_grads": [a.grad for a in acts], "weight_grads": wg}
            m._fake_gpu = True

    def drain(self):
        out = []
        self.step_ms = {}
        for epoch, want in self._pending:
            ratios = [0.01 * (i + 1) for i in range(len(self.model.weights))] if want else None
            out.append((epoch, 1.0 / (epoch + 1), ratios, f"2026-01-01T00:00:{epoch % 60:02d}"))
            self.step_ms[epoch] = 0.5
        self._pending = []
        return out

    def record(self):
        return self._rec

    def close(self, ok=True):
        self.closed = ok


def test_fused_orchestration_schedule_progress_and_stats(models_tmpdir, monkeypatch):
    fakes = []

    def make(self):
        fakes.append(FakeTrainer(self))
        return fakes[-1]

    # routes train() to the fused path; the layers themselves stay on their CPU path
    monkeypatch.setattr(NeuralNetworkModel, "on_gpu", property(lambda self: getattr(self, "_fake_gpu", False)))
    monkeypatch.setattr(NeuralNetworkModel, "_fused_trainer", make)
    monkeypatch.setattr(network_mod, "MAX_PROGRESS_POINTS", 4)
    m = NeuralNetworkModel("orch", [4, 8, 3], activation_algos=["relu", "softmax"], optimizer_algo="adam")
    data = [([float(i % 5), 1.0, -1.0, float(i % 2)], [i % 3]) for i in range(80)]  # > num_params: trains now
    m._fake_gpu = True
    m.train(data, epochs=12, learning_rate=0.1, decay_rate=0.5, dropout_rate=0.1, l2_lambda=0.01, batch_size=10)
    (t,) = fakes
    assert [s["epoch"] for s in t.steps] == list(range(12))
    assert t.schedule == [0.1 * 0.5 ** e for e in range(12)]
    assert all(abs(s["lr"] - 0.1 * 0.5 ** s["epoch"]) < 1e-15 for s in t.steps)
    assert [s["want_ratios"] for s in t.steps] == [e % 3 == 0 for e in range(12)]  # every epochs // 4
    assert [s["record"] for s in t.steps] == [e == 11 for e in range(12)]
    assert all(s["sample_size"] == 10 and s["dropout"] == 0.1 and s["l2"] == 0.01 for s in t.steps)
    assert m.status == "Trained"
    assert [p["epoch"] for p in m.progress] == [1, 4, 7, 10]  # 1-based, as the reference records
    p0 = m.progress[0]
    assert p0["cost"] == 1.0 and p0["world_size"] == 1 and p0["step_ms"] == 0.5
    assert p0["samples_per_s"] == round(10 / 0.5e-3, 1)
    assert p0["weight_upd_ratio"] == [0.01, None, 0.02, None]  # per layer; activations have none
    assert m.stats is not None and m.avg_cost is not None
    # the checkpoint written at the end carries the same progress
    again = NeuralNetworkModel.deserialize("orch")
    assert [p["epoch"] for p in again.progress] == [1, 4, 7, 10] and again.status == "Trained"


def test_long_trainings_checkpoint_in_the_background(models_tmpdir, monkeypatch):
    """CHECKPOINT_INTERVAL_S elapsed: the fused loop drains, records and writes a background
    checkpoint mid-training (reference ``neural_net_model.py:488-492``)."""
    fakes = []
    monkeypatch.setattr(NeuralNetworkModel, "on_gpu", property(lambda self: getattr(self, "_fake_gpu", False)))
    monkeypatch.setattr(NeuralNetworkModel, "_fused_trainer", lambda self: fakes.append(FakeTrainer(self)) or fakes[-1])
    monkeypatch.setattr(network_mod, "CHECKPOINT_INTERVAL_S", 0.0)
    saves = []
    real = NeuralNetworkModel.serialize_background
    monkeypatch.setattr(NeuralNetworkModel, "serialize_background", lambda self: saves.append(1) or real(self))
    m = NeuralNetworkModel("long", [4, 8, 3], activation_algos=["relu", "softmax"])
    m._fake_gpu = True
    m.train([([float(i % 5), 1.0, -1.0, 0.0], [i % 3]) for i in range(80)], epochs=3, batch_size=8)
    assert [s["record"] for s in fakes[0].steps] == [True, True, True]
    assert len(saves) == 3 and m.status == "Trained"


def test_fused_engine_declines_cpu_models_and_gpu_requests_fall_back(models_tmpdir):
    m = NeuralNetworkModel("cpu", [4, 8, 2], activation_algos=["relu", "softmax"])
    assert m._fused_trainer() is None  # CPU models train under autograd (reference semantics)
    g = NeuralNetworkModel("want_gpu", [4, 8, 2], activation_algos=["relu", "softmax"], device="cuda")
    assert g.device.type == ("cuda" if torch.cuda.is_available() else "cpu")


def test_data_parallel_save_agreement_lags_and_skips():
    """Data parallel fused training: each rank's 10 s flag is summed over the ranks and acted on
    LAG steps later (same decision everywhere); flags raised before an agreed save are dropped."""
    class Ctx:  # one rank; a "sum" over ranks is the flag itself
        def all_reduce_async(self, t, exact=False):
            assert exact
            return None

        def wait_one(self, h):
            pass

    agree = network_mod._SaveAgreement(Ctx(), torch.device("cpu"))
    flags = [False, True, True, True, False, False, False, True, False, False, False]
    got = [agree.decide(f) for f in flags]
    # step e acts on step e-2's flag; the two flags in flight at a save are skipped
    assert got == [False, False, False, True, False, False, False, False, False, True, False]
