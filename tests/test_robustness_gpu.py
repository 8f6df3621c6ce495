"""User-supplied indices never fault the GPU: out-of-range class labels and
token ids raise IndexError on the host like the reference (`cross_entropy`, `weights[ids]`),
negative token ids wrap like Python indexing, and the kernels themselves stay inside their
tables even when called directly with bad ids."""
import math

import pytest
import torch

from penr_oz_neural_network_torch_amd.ops import functional as PF

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_cross_entropy_rejects_bad_labels(native_lib):
    logits = torch.randn(8, 10, device=DEV)
    for bad in (10, -1, 1000):
        lab = torch.zeros(8, dtype=torch.int64)
        lab[3] = bad
        with pytest.raises(IndexError):
            PF.cross_entropy(logits, lab)
        with pytest.raises(IndexError):
            PF.cross_entropy(logits, lab.to(DEV))
    torch.cuda.synchronize()  # the device is still healthy
    ok = PF.cross_entropy(logits, torch.arange(8) % 10)
    assert math.isfinite(ok.item())


def test_xent_kernel_guard_bad_label_gives_nan_not_fault(native_lib):
    logits = torch.randn(4, 16, device=DEV)
    lab = torch.tensor([1, 2, 1 << 40, -5], device=DEV)
    loss = torch.zeros(1, device=DEV)
    dh = torch.empty_like(logits)
    no = PF.NO_EPI
    torch.ops.pz.xent_head(logits, lab, 4, loss, 1.0, dh, 1.0, None, None, no[0], no[1], 0)
    torch.cuda.synchronize()
    assert math.isnan(loss.item())


def test_embedding_negative_ids_wrap_and_bad_ids_raise(native_lib):
    table = torch.randn(12, 6, device=DEV, dtype=torch.float64)
    ids = torch.tensor([[0, -1, 5], [-12, 11, 3]])
    out = PF.embedding(ids, table)
    torch.testing.assert_close(out, table.cpu()[ids].to(DEV))
    for bad in (12, -13):
        with pytest.raises(IndexError):
            PF.embedding(torch.tensor([1, bad]), table)


def test_embedding_kernel_guard_out_of_range(native_lib):
    table = torch.randn(5, 64, device=DEV)
    ids = torch.tensor([2, 1 << 33, -7, 4], device=DEV)
    out = torch.full((4, 64), 7.0, device=DEV)
    torch.ops.pz.embedding_fwd(table, ids, out)
    dtable = torch.zeros(5, 64, device=DEV)
    torch.ops.pz.embedding_bwd(torch.ones(4, 64, device=DEV), ids, dtable)
    torch.cuda.synchronize()
    torch.testing.assert_close(out[0], table[2])
    assert out[1].abs().max().item() == 0 and out[2].abs().max().item() == 0
    assert dtable[2].eq(1).all() and dtable[4].eq(1).all() and dtable[[0, 1, 3]].abs().max().item() == 0


def test_fused_trainer_rejects_bad_labels_at_load(native_lib):
    from penr_oz_neural_network_torch_amd.engine.trainer import FusedTrainer
    from penr_oz_neural_network_torch_amd.models import NeuralNetworkModel
    model = NeuralNetworkModel("robust", [16, 32, 4], activation_algos=["relu", "softmax"], dtype="bfloat16",
                               device=DEV)
    tr = FusedTrainer(model)
    with pytest.raises(IndexError):
        tr.load_tensors(torch.randn(8, 16), torch.tensor([0, 1, 2, 3, 4, 0, 1, 2]))
    tr.load_tensors(torch.randn(8, 16), torch.tensor([0, 1, 2, 3, 3, 0, 1, 2]))


def test_histogram_counts_exact_beyond_fp32(native_lib):
    """A ReLU-zero bin holds more elements than fp32 counts can represent exactly (2^24)."""
    n_zero = (1 << 24) + 3
    x = torch.zeros(n_zero + 5, device=DEV)
    x[-5:] = torch.tensor([1.0, 2.0, 3.0, 4.0, 4.0], device=DEV)
    rng = torch.tensor([0.0, 4.0], device=DEV, dtype=torch.float64)
    counts = torch.zeros(4, device=DEV, dtype=torch.int64)
    torch.ops.pz.histogram(x, rng, 4, counts)
    assert counts.cpu().tolist() == [n_zero, 1, 1, 3]
