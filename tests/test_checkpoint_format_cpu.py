"""Checkpoint text writer details (utils/checkpoint.py): the pure-Python fallback formatter is
byte-identical to the native one and to ``json.dumps(indent=4)`` at every nesting level, ``render_json``
without tensors is plain ``json.dumps``, and a failed atomic write leaves no temp file behind."""
import json
import math
import os

import pytest
import torch

from penr_oz_neural_network_torch_amd.utils import checkpoint as ck


def _reference_text(values, level):
    text = json.dumps(values, indent=4)
    return text if level == 0 else text.replace("\n", "\n" + " " * (4 * level))


@pytest.mark.parametrize("shape", [(5,), (3, 4), (2, 3, 2), (1, 1)])
@pytest.mark.parametrize("level", [0, 1, 3])
def test_python_and_native_formatters_agree(shape, level):
    g = torch.Generator().manual_seed(sum(shape) * 10 + level)
    t = torch.randn(shape, generator=g, dtype=torch.float64) * torch.tensor(10.0) ** torch.randint(-12, 12, shape, generator=g)
    flat = t.view(-1)
    flat[0] = 0.1
    if flat.numel() > 2:
        flat[1], flat[2] = -0.0, 5e-324
    want = _reference_text(t.tolist(), level)
    assert ck._format_array_py(t, level) == want
    fmt = ck._native_formatter()
    assert fmt is not None and fmt(t.contiguous(), level) == want
    assert ck.format_array(t.t() if t.dim() == 2 else t, level) == _reference_text(
        (t.t() if t.dim() == 2 else t).tolist(), level)  # strided source, fp32 input below
    t32 = t.float()
    assert ck.format_array(t32, level) == _reference_text(t32.double().tolist(), level)


def test_special_values_spelled_like_python_json():
    t = torch.tensor([math.nan, math.inf, -math.inf, 1e16, 1e-7], dtype=torch.float64)
    assert ck.format_array(t, 0) == json.dumps(t.tolist(), indent=4)


def test_render_json_without_tensors_is_json_dumps():
    data = {"a": [1, 2.5, "x"], "b": {"c": None, "d": True}}
    assert ck.render_json(data) == json.dumps(data, indent=4)


def test_failed_atomic_write_leaves_no_temp_file(tmp_path, monkeypatch):
    target = str(tmp_path / "model_x.json")

    def fail(src, dst):
        raise OSError("simulated rename failure")
    monkeypatch.setattr(ck.os, "replace", fail)
    with pytest.raises(OSError, match="simulated"):
        ck._atomic_write_text(target, "{}")
    with pytest.raises(OSError, match="simulated"):
        ck._atomic_torch_save({"x": torch.zeros(2)}, str(tmp_path / "model_x_optimizer.pth"))
    assert os.listdir(tmp_path) == []
