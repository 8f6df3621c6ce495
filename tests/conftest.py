"""Shared pytest configuration.

* ``gpu`` marker: tests that need an MI355X (run by the driver with ``-m gpu`` on a GPU box).
  They never fall back: if the native library is missing they fail, by design.
* ``models_tmpdir`` fixture: run a test inside a fresh CWD so ``models/`` checkpoints written by
  the (reference-compatible, CWD-relative) persistence layer do not leak between tests.
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
SHIMS = os.path.join(ROOT, "tests", "_shims")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct GPU (MI355X / gfx950) and the built _pz_C.so")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def models_tmpdir(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("PZ_MODELS_DIR", raising=False)
    return tmp_path


@pytest.fixture(scope="session")
def native_lib():
    from penr_oz_neural_network_torch_amd.ops import native
    native.require()
    return torch.ops.pz
