"""``NeuralNetworkModel`` — model lifecycle, training, persistence, diagnostics (reference L4/L5,
``neural_net_model.py:269-585``).

Public API, attributes, checkpoint format and training semantics are the reference's. What a
model runs on is chosen at construction (new optional ``dtype`` / ``device`` arguments):

* default (``float64`` on the CPU): the reference algorithm on ATen, op for op. Seeded runs are
  bit-identical to the reference (tested), which keeps its 65-case test suite green.
* ``device="cuda"`` (any precision): parameters move into one flat device buffer
  (:class:`..engine.params.ParamStore`; layers hold views). ``train`` runs the device-resident
  fused engine (:class:`..engine.trainer.FusedTrainer`: MFMA GEMMs with fused epilogues, fused
  optimizer, on-device sampling, no host syncs between epochs, data parallel over RCCL when a
  process group is up). ``compute_output`` / ``_forward`` run the HIP kernels under autograd.
  Architectures the fused engine cannot schedule train through the same HIP kernels under
  autograd instead.

Fixes of reference defects: a zero sample size is clamped to 1; a training that
raises persists ``status == "Failed"`` instead of staying ``"Training"`` forever; checkpoints are
replaced atomically; periodic checkpoints of long trainings are written by a background thread.
"""
from __future__ import annotations

import logging
import random
import time
from datetime import datetime
from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from ..config import Precision, resolve_device, resolve_precision
from ..utils import checkpoint as ckpt
from ..utils.stats import build_stats
from .mlp import MultiLayerPerceptron

log = logging.getLogger("neural_net_model")

CHECKPOINT_INTERVAL_S = 10.0   # reference neural_net_model.py:488
MAX_PROGRESS_POINTS = 100      # reference :504


class _SaveAgreement:
    """Data parallel fused training: every rank must take the SAME record / checkpoint steps — a
    record step issues its collectives in another order (no paired dW launch, all-reduced instead
    of reduce-scattered buckets, the sharded optimizer's state gathers), so ranks whose 10 s
    wall clocks disagree would pair mismatched collectives. Each rank's "10 s since the last save"
    flag is summed over the ranks asynchronously; the step ``LAG`` epochs later acts on that
    agreed value. The sum is read through pinned memory behind an event on a side stream: the
    host waits for a two-step-old collective, never for the compute stream."""
    LAG = 2

    def __init__(self, ctx, device: torch.device):
        self.ctx, self.device = ctx, device
        self.side = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.queue: list = []
        self.skip = 0

    def decide(self, flag: bool) -> bool:
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=self.device)
        h = self.ctx.all_reduce_async(t, exact=True)
        if self.side is not None:
            host = torch.empty(1, dtype=torch.float64, pin_memory=True)
            self.side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side):
                self.ctx.wait_one(h)
                host.copy_(t, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.side)
            t.record_stream(self.side)
            self.queue.append((ev, host))
        else:
            self.ctx.wait_one(h)
            self.queue.append((None, t))
        if len(self.queue) <= self.LAG:
            return False
        ev, host = self.queue.pop(0)
        if ev is not None:
            ev.synchronize()
        agreed = host.item() > 0.0
        if self.skip:  # (flags raised before the last agreed save)
            self.skip -= 1
            return False
        if agreed:
            self.skip = self.LAG
        return agreed
MAX_COST_HISTORY = 100         # reference :539


def _effective_device(device) -> torch.device:
    dev = resolve_device(device)
    if dev.type == "cuda" and not torch.cuda.is_available():
        log.warning(f"device {dev} requested but no GPU is available; keeping the model on the CPU")
        return torch.device("cpu")
    return dev


class ModelMeta:
    """Checkpoint metadata under the attribute names of :class:`NeuralNetworkModel`."""

    def __init__(self, model_id: str, meta: dict):
        self.model_id = model_id
        self.algos = meta.get("algos")
        self.progress = meta.get("progress", [])
        self.avg_cost = meta.get("average_cost")
        self.avg_cost_history = meta.get("average_cost_history", [])
        self.stats = meta.get("stats")
        self.status = meta.get("status")
        self.runtime = meta.get("runtime")


class NeuralNetworkModel(MultiLayerPerceptron):
    def __init__(self, model_id, layer_sizes: list[int] = None, weight_algo="xavier", bias_algo="zeros",
                 activation_algos=None, optimizer_algo="adam", batchnorm=(1e-5, 0.1), confidence=1.0,
                 dtype=None, device=None):
        super().__init__(layer_sizes or [], weight_algo, bias_algo, activation_algos, batchnorm)
        self.model_id = model_id
        self.precision: Precision = resolve_precision(dtype)
        self.device = _effective_device(device)
        self._param_store = None
        self.optimizer: torch.optim.Optimizer | None = None
        if self.params:
            if self.weights:
                self.weights[-1] *= confidence
            self._place()
            if optimizer_algo == "adam":
                self.optimizer = torch.optim.Adam(self.params)
        self.progress = []
        self.training_data_buffer: list = []
        self.training_buffer_size: int = self.num_params
        self.avg_cost = None
        self.avg_cost_history = []
        self.stats = None
        self.status = "Created"
        # data-parallel group this model trains in (None: the process-wide context); set by the
        # REST service's multi-GPU train group (parallel/service.py) around ``train``
        self._context = None

    # ------------------------------------------------------------------------------------
    # placement
    # ------------------------------------------------------------------------------------
    @property
    def is_reference_runtime(self) -> bool:
        """fp64 on the CPU: the reference's own runtime (and checkpoint without a runtime key)."""
        return self.device.type == "cpu" and self.precision.name == "float64"

    @property
    def on_gpu(self) -> bool:
        return self.device.type == "cuda"

    def _place(self) -> None:
        """Move the (fp64, CPU) parameters into one flat buffer on the model's device/precision."""
        if self.is_reference_runtime or not self.params:
            self._param_store = None
            return
        from ..engine.params import ParamStore
        self._param_store = ParamStore.adopt(self.layers, self.device, self.precision.master)

    @property
    def weights(self) -> list[Tensor]:
        return [layer.weights for layer in self.layers if layer.weights is not None]

    @property
    def num_params(self) -> int:
        return sum(p.numel() for p in self.params)

    # ------------------------------------------------------------------------------------
    # persistence (reference :306-369)
    # ------------------------------------------------------------------------------------
    def _runtime_entry(self) -> dict | None:
        if self.is_reference_runtime:
            return None
        return {"dtype": self.precision.name, "device": self.device.type}

    def _model_data(self, layer_states: list) -> dict:
        data = {
            "algos": self.algos,
            "layers": layer_states,
            "progress": self.progress,
            "training_data_buffer": self.training_data_buffer,
            "average_cost": self.avg_cost,
            "average_cost_history": self.avg_cost_history,
            "stats": self.stats,
            "status": self.status,
        }
        runtime = self._runtime_entry()
        if runtime is not None:  # optional key; the reference ignores unknown keys on load
            data["runtime"] = runtime
        return data

    def get_model_data(self) -> dict:
        return self._model_data([layer.state_dict for layer in self.layers])

    def _checkpoint_skeleton(self) -> dict:
        """``get_model_data`` with parameter tensors left as tensors (rendered natively)."""
        return self._model_data([layer.checkpoint_state(ckpt.TensorRef) for layer in self.layers])

    def set_model_data(self, model_data: dict):
        for layer, state in zip(self.layers, model_data["layers"]):
            layer.state_dict = state
        self._place()
        self.progress = model_data["progress"]
        self.training_data_buffer = model_data["training_data_buffer"]
        self.training_buffer_size = self.num_params
        self.avg_cost = model_data["average_cost"]
        self.avg_cost_history = model_data["average_cost_history"]
        self.stats = model_data["stats"]
        self.status = model_data["status"]

    def _optimizer_state(self) -> dict | None:
        return self.optimizer.state_dict() if self.optimizer is not None else None

    def _dp_context(self):
        from ..parallel.dist import get_context
        return self._context if self._context is not None else get_context()

    def _is_writer(self) -> bool:
        """Under data parallelism every rank holds the same model; rank 0 owns the files."""
        return self._dp_context().rank == 0

    def serialize(self):
        if not self._is_writer():
            return
        ckpt.wait_pending(self.model_id)  # a background snapshot must not land after this write
        ckpt.save(self.model_id, self._checkpoint_skeleton(), self._optimizer_state())

    def serialize_background(self) -> bool:
        """Snapshot now, write on a background thread; False if the previous write is still running."""
        if not self._is_writer() or ckpt.pending(self.model_id):
            return False
        skeleton, opt_state = ckpt.snapshot(self._checkpoint_skeleton(), self._optimizer_state())
        ckpt.save_async(self.model_id, skeleton, opt_state)
        return True

    @classmethod
    def deserialize(cls, model_id: str, meta_only: bool = False):
        """Load a model. ``meta_only=True`` (the REST ``/progress/`` / ``/stats/`` polls; the
        reference deserialises the whole model for each, ``main.py:303-318``): a :class:`ModelMeta`
        with the progress / cost / status / stats attributes only — no parameter is parsed and
        nothing is placed on a GPU."""
        if meta_only:
            try:
                return ModelMeta(model_id, ckpt.load_meta(model_id))
            except FileNotFoundError as e:
                log.error(f"File not found error occurred: {str(e)}")
                raise KeyError(f"Model {model_id} not created yet.")
        try:
            model_data, opt_state = ckpt.load(model_id)
        except FileNotFoundError as e:
            log.error(f"File not found error occurred: {str(e)}")
            raise KeyError(f"Model {model_id} not created yet.")
        runtime = model_data.get("runtime") or {}
        model = cls(model_id, activation_algos=model_data["algos"], dtype=runtime.get("dtype"),
                    device=runtime.get("device"))
        model.set_model_data(model_data)
        if opt_state is not None:
            model.optimizer = torch.optim.Adam(model.params)
            model.optimizer.load_state_dict(opt_state)
        return model

    @classmethod
    def delete(cls, model_id: str):
        try:
            ckpt.delete(model_id)
        except FileNotFoundError as e:
            log.warning(f"Failed to delete: {str(e)}")

    # ------------------------------------------------------------------------------------
    # inference / forward (reference :371-408)
    # ------------------------------------------------------------------------------------
    @property
    def _activation_dtype(self) -> torch.dtype:
        """dtype of activations on the GPU autograd path (GEMM operand precision)."""
        if self.precision.name in ("bfloat16", "fp8"):
            return torch.bfloat16
        return self.precision.master

    def _input_tensor(self, data) -> Tensor:
        if self.is_reference_runtime or not self.on_gpu:
            return torch.tensor(data, dtype=self.precision.master if not self.is_reference_runtime else torch.float64)
        return torch.tensor(data, dtype=self.precision.master).to(self.device)

    def compute_output(self, input_data: list, target: list = None) -> Tuple[list, float]:
        activations, cost = self._forward(self._input_tensor(input_data), target)
        out = activations[-1].detach()
        if out.dtype == torch.bfloat16:
            out = out.float()
        return out.tolist(), cost.item() if cost.numel() > 0 else None

    def _forward(self, input_tensor: Tensor, target: list, dropout_rate=0.0) -> Tuple[list[Tensor], Tensor]:
        target_specified = target is not None and (isinstance(target, Tensor) or all(t is not None for t in target))
        gpu = self.on_gpu
        if gpu:
            from ..ops import functional as PF
            input_tensor = input_tensor.to(self.device)
            if self.algos[0] != "embedding":
                input_tensor = input_tensor.to(self._activation_dtype)
        outputs: list[Tensor] = []
        x = logits = input_tensor
        for layer in self.layers:
            layer.training = target_specified
            logits = x
            x = layer.forward(logits)
            if layer.hidden and layer.training:  # dropout on every hidden output (reference :393-395)
                x = PF.dropout(x, dropout_rate) if gpu else F.dropout(x, p=dropout_rate)
            outputs.append(x)

        if not target_specified:
            cost = torch.empty(0)
        elif self.algos[-1] == "softmax":  # CE on the softmax layer's input (reference :400-403)
            if isinstance(target, Tensor):  # programmatic use: class ids already as a tensor
                label_tensor = target.reshape(-1).to(torch.int64)
            else:
                labels = target[0] if logits.ndim == 1 else [t[0] for t in target]
                label_tensor = torch.tensor(labels, dtype=torch.int64)
            if gpu:
                cost = PF.cross_entropy(logits.to(self._loss_dtype), label_tensor.to(self.device))
            else:
                cost = F.cross_entropy(logits, label_tensor)
        else:
            target_tensor = torch.tensor(target, dtype=torch.float64)
            if gpu:
                cost = PF.mse_loss(x.to(self._loss_dtype), target_tensor.to(self.device, self._loss_dtype))
            else:
                cost = F.mse_loss(x, target_tensor.to(x.dtype) if x.dtype != torch.float64 else target_tensor)
        return outputs, cost

    @property
    def _loss_dtype(self) -> torch.dtype:
        return torch.float64 if self.precision.master == torch.float64 else torch.float32

    # ------------------------------------------------------------------------------------
    # training (reference :410-530)
    # ------------------------------------------------------------------------------------
    def train(self, training_data: list, epochs=100, learning_rate=0.01, batch_size=None, decay_rate=0.9,
              dropout_rate=0.2, l2_lambda=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8):
        self.training_data_buffer.extend(training_data)
        if len(self.training_data_buffer) < self.training_buffer_size:
            log.info(f"Model {self.model_id}: Insufficient training data. "
                     f"Current buffer size: {len(self.training_data_buffer)}, "
                     f"required: {self.training_buffer_size}")
            self.serialize()  # keep the partial buffer for next time
            return

        data = self.training_data_buffer
        self.training_data_buffer = []
        epochs = max(0, int(epochs))
        # explicit, or an equal share per epoch; clamped (the reference crashes on 0 in mm)
        sample_size = max(1, batch_size or (int(len(data) / epochs) if epochs else len(data)))
        log.info(f"Training sample size: {sample_size}")

        if self.optimizer is not None:
            for group in self.optimizer.param_groups:
                group["betas"] = (beta1, beta2)
                group["eps"] = epsilon

        self.progress = []
        self.stats = None
        self.status = "Training"
        self.serialize()

        hp = dict(epochs=epochs, learning_rate=learning_rate, sample_size=sample_size, decay_rate=decay_rate,
                  dropout_rate=dropout_rate, l2_lambda=l2_lambda)
        try:
            trainer = self._fused_trainer() if self.on_gpu else None
            if trainer is not None:
                try:
                    self._train_fused(trainer, data, **hp)
                except BaseException:
                    trainer.close(ok=False)  # no device sync on the failure path (engine/events.py)
                    raise
                trainer.close()
            else:
                self._train_autograd(data, **hp)
        except Exception:
            log.exception(f"Model {self.model_id}: training failed")
            self.status = "Failed"
            try:
                self.serialize()
            except Exception:  # pragma: no cover - keep the original error
                log.exception(f"Model {self.model_id}: could not persist the failed status")
            raise

        self.status = "Trained"
        log.info(f"Model {self.model_id}: Done training for {epochs} epochs.")
        self.serialize()

    def _progress_point(self, when: str, epoch: int, cost: float, ratios: list[float] | None,
                        extra: dict | None = None) -> None:
        pending = list(ratios or [])
        point = {
            "dt": when,
            "epoch": epoch + 1,
            "cost": cost,
            "weight_upd_ratio": [pending.pop(0) if layer.weights is not None and pending else None
                                 for layer in self.layers],
        }
        if extra:  # optional telemetry of GPU runs; the dashboard ignores unknown keys
            point.update(extra)
        self.progress.append(point)

    def _train_autograd(self, data, epochs, learning_rate, sample_size, decay_rate, dropout_rate, l2_lambda,
                        context=None, sampler: torch.Generator | None = None):
        """The reference epoch loop (``neural_net_model.py:457-522``). On the CPU it is the
        reference's exact op / RNG sequence; GPU models run it on the HIP kernels.

        Data parallel (a process group is up, e.g. gloo for CPU models): replicas start from rank
        0's parameters, every rank draws the same global sample from a shared ``sampler`` seed and
        trains on its contiguous shard, and gradients are averaged with one all-reduce before the
        (identical) optimizer step — equivalent to one process training on the whole sample."""
        ctx = context or self._dp_context()
        world, rank = ctx.world_size, ctx.rank
        from . import layers as _layers
        _layers.set_bn_sync(self.layers, ctx if world > 1 else None)  # synchronised batchnorm statistics
        try:
            self._autograd_epochs(data, epochs, learning_rate, sample_size, decay_rate, dropout_rate, l2_lambda,
                                  ctx, sampler)
        finally:
            _layers.set_bn_sync(self.layers, None)

    def _autograd_epochs(self, data, epochs, learning_rate, sample_size, decay_rate, dropout_rate, l2_lambda, ctx,
                         sampler):
        world, rank = ctx.world_size, ctx.rank
        if world > 1:
            dev = self.params[0].device if self.params else torch.device("cpu")
            with torch.no_grad():
                for p in self.params:
                    ctx.broadcast_(p.data)
            if sampler is None:
                seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(dev)
                ctx.broadcast_(seed)
                sampler = torch.Generator().manual_seed(int(seed.item()))
        if sample_size < world:
            raise ValueError(f"sample size {sample_size} is smaller than the {world} data-parallel ranks")
        # contiguous shards of the global sample; the sample_size % world extra rows are spread by the
        # floor division (S=10, W=4: shards 2, 3, 2, 3)
        lo, hi = rank * sample_size // world, (rank + 1) * sample_size // world
        weight = (hi - lo) / sample_size  # this rank's share of the global mean loss
        activations = None
        every = max(1, epochs // MAX_PROGRESS_POINTS)
        last_saved = time.time()
        # GPU models: the parameters live in one flat device buffer (ParamStore); autograd
        # accumulates every gradient into views of one flat gradient buffer and the update is the
        # fused optimizer kernel (csrc/optim.hip, the trainer's), not torch.optim's per-tensor ops —
        # same math, and the torch.optim.Adam state stays the checkpointed object (its moments
        # become views of the kernel's flat buffers)
        fused, flat_grad, grad_views = None, None, None
        if self._param_store is not None and self._param_store.device.type == "cuda":
            from ..engine.optim import FusedOptimizer
            store = self._param_store
            fused = FusedOptimizer(store, self.params, self.optimizer, {})
            flat_grad = torch.zeros_like(store.flat)
            by_param = {seg.param_index: seg for seg in store.segments}
            grad_views = [store.view(by_param[i], flat_grad) for i in range(len(self.params))]
        for epoch in range(epochs):
            if sampler is None:  # the reference's draw from the global RNG
                picks = torch.randint(0, len(data), (sample_size,))
            else:
                picks = torch.randint(0, len(data), (sample_size,), generator=sampler)
            if world > 1:
                picks = picks[lo:hi]
            sample = [data[i] for i in picks]
            lr = learning_rate * (decay_rate ** epoch)
            if self.optimizer is not None:
                for group in self.optimizer.param_groups:
                    group["lr"] = lr
            inputs = self._input_tensor([inp for inp, _ in sample])
            target = [tgt for _, tgt in sample]
            prev_weights = [w.clone().detach() for w in self.weights]
            for p in self.params:
                p.requires_grad_()
            activations, cost = self._forward(inputs, target, dropout_rate)
            if l2_lambda > 0.0:
                cost = cost + l2_lambda * sum((w ** 2).sum() for w in self.weights)
            if fused is not None:  # backward accumulates into the zeroed flat buffer's views
                flat_grad.zero_()
                for p, gv in zip(self.params, grad_views):
                    p.grad = gv
            else:
                for p in self.params:
                    p.grad = None
            long_training = time.time() - last_saved >= CHECKPOINT_INTERVAL_S
            if epoch + 1 == epochs or long_training:
                for a in activations:
                    a.retain_grad()
            if world > 1:
                # the rank's share of the global objective: gradients then simply SUM over the ranks
                # (and a synchronised batchnorm's all-reduce backward combines the shares correctly)
                (cost * weight).backward()
                self._average_gradients(ctx, 1.0)
            else:
                cost.backward()
            if fused is not None:  # (the L2 term is already in the autograd gradient)
                fused.step(flat_grad, lr, 0.0, 1.0)
                fused.sync_torch_state()
            elif self.optimizer is not None:
                self.optimizer.step()
            else:
                for p in self.params:
                    p.data -= lr * p.grad
            when, value = datetime.now().isoformat(), cost.item()
            if world > 1:
                value = ctx.all_reduce_scalar(value * weight)
            if epoch % every == 0:
                with torch.no_grad():
                    ratios = [((w - pw).data.std() / (w.data.std() + 1e-8)).item()
                              for pw, w in zip(prev_weights, self.weights)]
                self._progress_point(when, epoch, value, ratios, {"world_size": world} if world > 1 else None)
            log.info(f"Model {self.model_id}: Epoch {epoch + 1}, Cost: {value:.4f}")
            if long_training:  # pragma: no cover - timing dependent
                self._record_training_overall_progress(activations)
                self.serialize_background()
                last_saved = time.time()
        if activations is not None:
            self._record_training_overall_progress(activations)

    def _average_gradients(self, ctx, weight: float) -> None:
        """Global-batch mean of every parameter gradient: each rank's shard-mean gradient weighted
        by its share of the sample, summed over the ranks in one flat all-reduce."""
        grads = [p.grad for p in self.params]
        flat = torch.cat([g.reshape(-1) for g in grads]) * weight
        ctx.wait_all([ctx.all_reduce_async(flat, exact=True)])
        off = 0
        for g in grads:
            g.copy_(flat[off:off + g.numel()].view_as(g))
            off += g.numel()

    def _fused_trainer(self):
        from ..engine.trainer import FusedTrainer, UnsupportedModel
        try:
            return FusedTrainer(self, self._dp_context())
        except UnsupportedModel as e:
            log.info(f"Model {self.model_id}: fused engine unavailable ({e}); training under autograd")
            return None

    def _drain_progress(self, trainer, sample_size: int) -> None:
        drained = trainer.drain()
        world = trainer.ctx.world_size
        for epoch, cost, ratios, when in drained:
            if ratios is not None:
                ms = trainer.step_ms.get(epoch)
                extra = {"device": str(self.device), "dtype": self.precision.name, "world_size": world}
                if ms:
                    extra["step_ms"] = round(ms, 4)
                    extra["samples_per_s"] = round(sample_size / (ms * 1e-3), 1)
                self._progress_point(when, epoch, cost, ratios, extra)
            log.info(f"Model {self.model_id}: Epoch {epoch + 1}, Cost: {cost:.4f}")

    def _record_fused(self, trainer) -> None:
        rec = trainer.record()
        self._record_training_overall_progress(rec["activations"], rec["act_grads"], rec["weight_grads"])

    def _train_fused(self, trainer, data, epochs, learning_rate, sample_size, decay_rate, dropout_rate, l2_lambda):
        """Same schedule as :meth:`_train_autograd`, enqueued on the GPU without host syncs;
        costs / ratios / timestamps come back in :meth:`FusedTrainer.drain`."""
        trainer.load_data(data)
        trainer.begin(epochs, lr_schedule=lambda e: learning_rate * decay_rate ** e)
        every = max(1, epochs // MAX_PROGRESS_POINTS)
        last_saved = time.time()
        agree = _SaveAgreement(trainer.ctx, trainer.dev) if trainer.ctx.enabled else None
        for epoch in range(epochs):
            long_training = time.time() - last_saved >= CHECKPOINT_INTERVAL_S
            if agree is not None:
                long_training = agree.decide(long_training)
            trainer.step(epoch, learning_rate * decay_rate ** epoch, sample_size, dropout_rate, l2_lambda,
                         want_ratios=epoch % every == 0, record=epoch + 1 == epochs or long_training)
            if long_training:
                self._drain_progress(trainer, sample_size)
                self._record_fused(trainer)
                self.serialize_background()
                last_saved = time.time()
        self._drain_progress(trainer, sample_size)
        if epochs:
            self._record_fused(trainer)

    # ------------------------------------------------------------------------------------
    # diagnostics (reference :532-585)
    # ------------------------------------------------------------------------------------
    def _record_training_overall_progress(self, activations, act_grads=None, weight_grads=None):
        costs = [p["cost"] for p in self.progress]
        if not costs:
            return
        avg = sum(costs) / len(costs)
        self.avg_cost = ((self.avg_cost or avg) + avg) / 2.0
        self.avg_cost_history.append(self.avg_cost)
        if len(self.avg_cost_history) > MAX_COST_HISTORY:
            self.avg_cost_history.pop(random.randint(1, 98))
        if act_grads is None:
            act_grads = [a.grad for a in activations]
        if weight_grads is None:
            weight_grads = [layer.weights.grad if layer.weights is not None else None for layer in self.layers]
        self.stats = build_stats(self.layers, activations, act_grads, weight_grads)
        log.info(f"Model {self.model_id} - Cost: {avg:.4f} Overall Cost: {self.avg_cost:.4f}")


__all__ = ["NeuralNetworkModel"]
