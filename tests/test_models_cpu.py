"""Model API on the reference-compatible CPU/fp64 path (no GPU needed)."""
import importlib.util
import json
import math
import os

import pytest
import torch

from neural_net_model import (BatchNormLayer, EmbeddingLayer, FlattenLayer, LinearLayer, MultiLayerPerceptron,
                              NeuralNetworkModel, ReluLayer, SoftmaxLayer, TanhLayer)
from penr_oz_neural_network_torch_amd.models.mlp import normalize_algos
from penr_oz_neural_network_torch_amd.utils import checkpoint as ckpt

REF = "/root/reference/neural_net_model.py"


def _reference_module():
    if not os.path.exists(REF):
        pytest.skip("reference checkout not mounted")
    spec = importlib.util.spec_from_file_location("ref_neural_net_model", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("algos,sizes,expected", [
    (None, [9, 9, 9], ["linear", "relu", "linear", "relu"]),
    (["relu", "linear", "tanh", "softmax"], [3, 3, 3, 3], ["linear", "relu", "linear", "tanh", "linear", "softmax"]),
    (["embedding", "tanh", "linear", "softmax"], [1], ["embedding", "flatten", "linear", "tanh", "linear", "softmax"]),
    (["embedding", "linear", "batchnorm", "tanh", "flatten", "linear", "softmax"], [1],
     ["embedding", "flatten", "linear", "batchnorm", "tanh", "flatten", "linear", "softmax"]),
    (["batchnorm", "sigmoid"], [1], ["batchnorm", "sigmoid"]),
])
def test_algo_normalisation(algos, sizes, expected):
    got = normalize_algos(algos or ["relu"] * (len(sizes) - 1))
    assert got == expected
    assert normalize_algos(got) == got  # idempotent: checkpoints store normalised algos


@pytest.mark.parametrize("sizes,algos,n", [
    ([3, 3], None, 12), ([9, 9, 9], None, 180), ([18, 9, 3], ["sigmoid"] * 2, 201),
    ([10, 3, 6, 20, 10], ["embedding", "tanh", "softmax"], 380),
    ([10, 3, 6, 20, 10], ["embedding", "linear", "batchnorm", "tanh", "softmax"], 420),
])
def test_num_params_and_buffer(sizes, algos, n):
    m = NeuralNetworkModel("t", sizes, activation_algos=algos)
    assert m.num_params == n == m.training_buffer_size
    assert m.status == "Created" and m.stats is None and m.avg_cost is None


def test_layer_structure_and_flatten_ratios():
    mlp = MultiLayerPerceptron([18, 2, 6, 10, 20, 18], "he", "",
                               ["embedding", "linear", "batchnorm", "tanh", "flatten", "linear", "softmax"])
    kinds = [type(l) for l in mlp.layers]
    assert kinds == [EmbeddingLayer, FlattenLayer, LinearLayer, BatchNormLayer, TanhLayer, FlattenLayer, LinearLayer,
                     SoftmaxLayer]
    assert [l.ratio for l in mlp.layers if isinstance(l, FlattenLayer)] == [3, 2]
    assert [tuple(p.shape) for p in mlp.layers[2].params] == [(6, 10)]  # bias_algo "" -> no bias
    assert not mlp.layers[0].hidden and not mlp.layers[-1].hidden and all(l.hidden for l in mlp.layers[1:-1])


def test_he_gain_and_confidence():
    torch.manual_seed(0)
    a = NeuralNetworkModel("a", [16, 32, 8], "he", "zeros", ["relu", "softmax"], confidence=0.5)
    torch.manual_seed(0)
    b = NeuralNetworkModel("b", [16, 32, 8], "gaussian", "zeros", ["relu", "softmax"])
    torch.testing.assert_close(a.weights[0], b.weights[0] / math.sqrt(16) * math.sqrt(2.0))
    torch.testing.assert_close(a.weights[1], b.weights[1] / math.sqrt(32) * 0.5)


def test_forward_shapes_and_costs():
    m = NeuralNetworkModel("t", [9, 2, 4, 9, 18, 9], activation_algos=["embedding", "tanh", "flatten", "linear",
                                                                       "softmax"])
    out, cost = m.compute_output([[0, 5, 8, 2], [1, 3, 7, 4]], [[2], [4]])
    assert len(out) == 2 and len(out[0]) == 9 and cost is not None
    out1, c1 = m.compute_output([0, 5, 8, 2])
    assert len(out1) == 9 and c1 is None


def test_init_and_training_bit_identical_to_reference(models_tmpdir):
    ref = _reference_module()
    args = ([9, 18, 9], "xavier", "random", ["relu", "softmax"], "adam")
    torch.manual_seed(42)
    r = ref.NeuralNetworkModel("r", *args)
    torch.manual_seed(42)
    o = NeuralNetworkModel("o", *args)
    for a, b in zip(r.params, o.params):
        assert torch.equal(a, b)
    data = [([float((i * 7 + j) % 5 - 2) for j in range(9)], [i % 9]) for i in range(o.training_buffer_size)]
    torch.manual_seed(7)
    r.train(list(data), epochs=3, batch_size=32)
    torch.manual_seed(7)
    o.train(list(data), epochs=3, batch_size=32)
    for a, b in zip(r.params, o.params):
        assert torch.equal(a, b)
    assert [p["cost"] for p in r.progress] == [p["cost"] for p in o.progress]
    assert [p["weight_upd_ratio"] for p in r.progress] == [p["weight_upd_ratio"] for p in o.progress]
    assert r.avg_cost == o.avg_cost
    assert json.dumps(r.stats) == json.dumps(o.stats)


def test_checkpoint_text_identical_to_json_dumps(models_tmpdir):
    torch.manual_seed(1)
    m = NeuralNetworkModel("ck", [27, 10, 30, 16, 27], activation_algos=["embedding", "linear", "batchnorm",
                                                                          "tanh", "linear", "softmax"])
    m.progress = [{"dt": "x", "epoch": 1, "cost": 1e-05, "weight_upd_ratio": [0.1, None]}]
    text = ckpt.render_json(m._checkpoint_skeleton())
    assert text == json.dumps(m.get_model_data(), indent=4)
    m.serialize()
    with open(ckpt.model_path("ck")) as f:
        assert f.read() == text
    loaded = NeuralNetworkModel.deserialize("ck")
    for a, b in zip(loaded.params, m.params):
        assert torch.equal(a, b)


def test_reference_checkpoints_interoperate(models_tmpdir):
    ref = _reference_module()
    torch.manual_seed(3)
    r = ref.NeuralNetworkModel("x", [8, 16, 4], activation_algos=["tanh", "softmax"], optimizer_algo="adam")
    r.serialize()  # reference writes models/model_x.json + optimizer_x.pth (cwd = tmp)
    o = NeuralNetworkModel.deserialize("x")
    for a, b in zip(r.params, o.params):
        assert torch.equal(a, b)
    assert o.optimizer is not None
    o.status = "Trained"
    o.serialize()
    back = ref.NeuralNetworkModel.deserialize("x")
    assert back.status == "Trained"
    for a, b in zip(back.params, o.params):
        assert torch.equal(a, b)


def test_sample_size_zero_is_clamped(models_tmpdir):
    m = NeuralNetworkModel("z", [2, 2], activation_algos=["sigmoid"], optimizer_algo="stochastic")
    data = [([0.1, 0.2], [0.0, 1.0])] * m.training_buffer_size
    m.train(data, epochs=100)  # 6 samples over 100 epochs -> reference crashes in mm
    assert m.status == "Trained"


def test_batchnorm_eval_uses_running_stats():
    layer = BatchNormLayer(4)
    layer.training = True
    x = torch.randn(32, 4, dtype=torch.float64)
    layer.forward(x)
    layer.training = False
    y = layer.forward(x)
    torch.testing.assert_close(y, (x - layer.mean) / torch.sqrt(layer.variance + layer.eps))


def test_relu_layer_gain_constants():
    assert ReluLayer.weight_gain == math.sqrt(2.0)
    assert TanhLayer.weight_gain == 5.0 / 3.0


def test_background_checkpoint_matches_synchronous(models_tmpdir):
    torch.manual_seed(5)
    m = NeuralNetworkModel("bg", [6, 12, 3], activation_algos=["relu", "softmax"], optimizer_algo="adam")
    data = [([float((i + j) % 4) for j in range(6)], [i % 3]) for i in range(m.training_buffer_size)]
    m.train(data, epochs=2, batch_size=16)
    m.serialize()
    with open(ckpt.model_path("bg")) as f:
        sync_text = f.read()
    sync_opt = torch.load(ckpt.optimizer_path("bg"), weights_only=True)
    assert m.serialize_background()
    snap_params = [p.clone() for p in m.params]
    with torch.no_grad():  # training continues while the snapshot is being written
        for p in m.params:
            p.add_(1.0)
    ckpt.wait_pending("bg")
    with open(ckpt.model_path("bg")) as f:
        assert f.read() == sync_text
    bg_opt = torch.load(ckpt.optimizer_path("bg"), weights_only=True)
    for k, st in sync_opt["state"].items():
        assert torch.equal(st["exp_avg"], bg_opt["state"][k]["exp_avg"])
    loaded = NeuralNetworkModel.deserialize("bg")
    for a, b in zip(loaded.params, snap_params):
        assert torch.equal(a, b)


def test_native_checkpoint_reader_matches_json_load(models_tmpdir, monkeypatch):
    """N9 reader: layer parameters parsed natively into tensors equal json.load + torch.tensor
    bit for bit (incl. NaN / inf / -0.0 / subnormals); every other field is untouched."""
    from penr_oz_neural_network_torch_amd.ops import native
    if not native.has_host_ops():
        pytest.skip("native library not built")
    torch.manual_seed(9)
    m = NeuralNetworkModel("rd", [27, 10, 30, 16, 27], "he", "",
                           ["embedding", "linear", "batchnorm", "tanh", "linear", "softmax"])
    with torch.no_grad():
        w = m.layers[2].weights
        w[0, :4] = torch.tensor([float("nan"), float("inf"), -0.0, 5e-324], dtype=torch.float64)
    m.training_data_buffer = [([1.0, 2.0, 3.0], [4]), ([0.5, -1.0, 2.0], [1])]
    m.stats = {"layers": [{"histogram": {"x": [1.0, 2.0], "y": [0.5, 0.25]}}]}
    m.serialize()
    path = ckpt.model_path("rd")
    fast = ckpt.read_model_data(path)
    with open(path) as f:
        slow = json.load(f)
    assert [type(p) for l in fast["layers"] for p in l.get("params", [])] == \
        [torch.Tensor] * sum(len(l.get("params", [])) for l in slow["layers"])
    for lf, ls in zip(fast["layers"], slow["layers"]):
        assert {k: v for k, v in lf.items() if k != "params"} == {k: v for k, v in ls.items() if k != "params"}
        for a, b in zip(lf.get("params", []), ls.get("params", [])):
            ref = torch.tensor(b, dtype=torch.float64)
            assert a.shape == ref.shape
            assert torch.equal(a.view(torch.int64), ref.view(torch.int64))  # bitwise, NaN included
    for k in slow:
        if k != "layers":
            assert fast[k] == slow[k]
    loaded = NeuralNetworkModel.deserialize("rd")
    for a, b in zip(loaded.params, m.params):
        assert torch.equal(a.view(torch.int64), b.detach().view(torch.int64))
    monkeypatch.setenv("PZ_NATIVE_JSON", "0")
    again = NeuralNetworkModel.deserialize("rd")
    for a, b in zip(again.params, loaded.params):
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
