"""REST microservice (reference L6/L8, ``main.py:1-370``): create / train / serve / inspect MLPs.

Routes, request schemas, defaults, status codes and error mapping are those of the reference so
existing clients, its test-suite and the dashboard work unchanged:

    GET  /              -> 307 /dashboard            GET /dashboard      -> HTML page
    POST /model/        create + serialize            POST /output/       inference (+ cost)
    PUT  /train/        202, training in background   (409 while that model is training)
    GET  /progress/     progress / avg cost / status  GET /stats/         training diagnostics
    DELETE /model/      204

Additions (optional, defaults reproduce the reference): ``dtype`` and ``device`` on model
creation (``"bfloat16"`` + ``"cuda"`` trains on the MI355X fused engine), ``GET /health``, and
multi-GPU data-parallel training of GPU models (``PZ_SERVICE_GPUS=N|auto``: this process is rank 0
of an N-rank RCCL group whose workers it starts at startup — ``parallel/service.py``).
Fixes of reference races: the 409 check happens before the model is loaded,
checkpoint files are replaced atomically (no torn reads from ``/progress/``), and exceptions in a
background training task are logged instead of vanishing.
"""
from __future__ import annotations

import logging
import os
from asyncio import Lock, create_task
from contextlib import asynccontextmanager
from typing import Dict

from fastapi import Body, FastAPI, HTTPException, Request
from fastapi.concurrency import run_in_threadpool
from fastapi.params import Query
from fastapi.responses import HTMLResponse, JSONResponse, RedirectResponse, Response
from fastapi.staticfiles import StaticFiles
from fastapi.templating import Jinja2Templates
from pydantic import BaseModel, Field

from neural_net_model import NeuralNetworkModel
from penr_oz_neural_network_torch_amd.parallel import service

_HERE = os.path.dirname(os.path.abspath(__file__))


@asynccontextmanager
async def lifespan(_: FastAPI):
    # PZ_SERVICE_GPUS=N|auto: GPU models train data-parallel on N GPUs (rank 0 = this process);
    # the worker ranks are started here, before anything in this process touches the GPU
    service.start_from_env()
    try:
        yield
    finally:
        service.stop()


app = FastAPI(
    title="Neural Network Model API",
    description="API to create, serialize, compute output and diagnose of neural network models.",
    version="0.0.1",
    lifespan=lifespan,
)
app.mount("/static", StaticFiles(directory=os.path.join(_HERE, "static")), name="static")
templates = Jinja2Templates(directory=os.path.join(_HERE, "templates"))

LOG_FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"
DATE_FORMAT = "%Y-%m-%dT%H:%M:%S"
logging.basicConfig(datefmt=DATE_FORMAT, format=LOG_FORMAT)
log = logging.getLogger(__name__)

# tic-tac-toe style examples for the OpenAPI docs: 9-cell board in {-1,0,1} -> one-hot next move
_BOARDS = [
    ([0, 0, 0, 0, 0, 0, 0, 0, 0], 4), ([0, 0, 0, 0, -1, 0, 0, 0, 0], 0), ([1, 0, 0, 0, -1, 0, 0, 0, 0], 1),
    ([1, -1, 0, 0, -1, 0, 0, 0, 0], 7), ([1, -1, 0, 0, -1, 0, 0, 1, 0], 2), ([1, -1, -1, 0, -1, 0, 0, 1, 0], 6),
    ([1, -1, -1, 0, -1, 0, 1, 1, 0], 8), ([1, -1, -1, 0, -1, 0, 1, 1, -1], 3), ([1, -1, -1, 1, -1, 0, 1, 1, -1], 5),
]
EXAMPLES = [{"activation_vector": board, "target_vector": [1 if i == move else 0 for i in range(9)]}
            for board, move in _BOARDS]


class InputItem(BaseModel):
    activation_vector: list = Field(..., description="The input activation data. 1D or 2D supported.")
    target_vector: list | None = Field(None, description="The optional expected target data same size as input data.")


class TrainingItem(InputItem):
    target_vector: list[float] = Field(..., description="The expected output vector, required for training items.")


class ModelRequest(BaseModel):
    model_id: str = Field(..., examples=["test"], description="The unique identifier for the model.")


class CreateModelRequest(ModelRequest):
    layer_sizes: list[int] = Field(..., examples=[[9, 1, 9, 9]],
                                   description="A list of integers representing the sizes of each layer in the neural network.")
    weight_algo: str = Field("xavier", examples=["xavier", "he", "gaussian"], description="An initialization algorithm")
    bias_algo: str = Field("random", examples=["random", "zeros"], description="An initialization algorithm")
    activation_algos: list[str] = Field(..., examples=[["sigmoid"] * 3, ["relu"] * 2 + ["sigmoid"],
                                                       ["relu"] * 2 + ["softmax"], ["embedding", "tanh"]],
                                        description="The activation algorithms to apply")
    optimizer: str = Field("adam", examples=["adam", "stochastic"],
                           description="The optimizer to use for updating for gradient descent")
    batchnorm_eps: float = Field(1e-5, examples=[1e-5], description="Batch Normalization Epsilon")
    batchnorm_momentum: float = Field(0.1, examples=[0.1], description="Batch Normalization Momentum")
    confidence: float = Field(1.0, examples=[1.0], description="Confidence factor for the last layer with weights")
    dtype: str | None = Field(None, examples=["float64", "bfloat16"],
                              description="Compute precision (default float64 = reference behaviour)")
    device: str | None = Field(None, examples=["cpu", "cuda"], description="Device to keep the model on (default cpu)")


class ActivationRequest(ModelRequest):
    input: InputItem = Field(..., description="The input data, an InputItem.")


class TrainingRequest(ModelRequest):
    training_data: list[TrainingItem] = Field(..., examples=[EXAMPLES], description="A list of training data pairs.")
    epochs: int = Field(10, examples=[10], description="The number of training epochs.")
    learning_rate: float = Field(0.01, examples=[0.01], description="The learning rate for training.")
    batch_size: int | None = Field(None, examples=[32], description="The batch size for training sample each epoch. (Optional)")
    decay_rate: float = Field(0.9, examples=[0.9], description="The decay rate of learning rate during training.")
    dropout_rate: float = Field(0.2, examples=[0.2],
                                description="The drop out rate of activated neurons to improve generalization")
    l2_lambda: float = Field(0.001, examples=[0.001],
                             description="The L2 Lambda penalty reducing weight magnitude during backpropagation")
    adam_beta1: float = Field(0.9, examples=[0.9],
                              description="The Adam optimizer parameter for gradient mean optimization after backpropagation")
    adam_beta2: float = Field(0.999, examples=[0.999],
                              description="The Adam optimizer parameter for gradient variance optimization after backpropagation")
    adam_epsilon: float = Field(1e-8, examples=[1e-8],
                                description="The Adam optimizer parameter for smallest step for gradient optimization after backpropagation")


class ModelIdQuery(Query):
    description = "The unique identifier for the model."


@app.exception_handler(Exception)
async def generic_exception_handler(_: Request, e: Exception):
    log.error(f"An error occurred: {str(e)}")
    return JSONResponse(status_code=500, content={"detail": "Please refer to server logs"})


@app.exception_handler(KeyError)
async def key_error_handler(_: Request, e: KeyError):
    raise HTTPException(status_code=404, detail=f"Not found error occurred: {str(e)}")


@app.exception_handler(ValueError)
async def value_error_handler(_: Request, e: ValueError):
    raise HTTPException(status_code=400, detail=f"Value error occurred: {str(e)}")


@app.get("/", include_in_schema=False)
def redirect_to_dashboard():
    return RedirectResponse(url="/dashboard")


@app.get("/dashboard", response_class=HTMLResponse)
async def dashboard(request: Request):
    return templates.TemplateResponse(request, "dashboard.html")


@app.get("/health")
def health():
    import torch
    gpus = torch.cuda.device_count() if torch.cuda.is_available() else 0
    from penr_oz_neural_network_torch_amd.ops import native
    group = service.get_group()
    return {"status": "ok", "gpus": gpus, "native": native.has_host_ops(), "training": sorted(
        k for k, v in model_locks.items() if v.locked()), "train_group": group.status() if group else None}


@app.post("/model/")
def create_model(body: CreateModelRequest = Body(...)):
    model_id = body.model_id
    log.info(f"Requesting creation of model {model_id}")
    kwargs = {}
    if body.dtype is not None:
        kwargs["dtype"] = body.dtype
    if body.device is not None:
        kwargs["device"] = body.device
    model = NeuralNetworkModel(model_id, body.layer_sizes, body.weight_algo, body.bias_algo, body.activation_algos,
                               body.optimizer, (body.batchnorm_eps, body.batchnorm_momentum), body.confidence,
                               **kwargs)
    model.serialize()
    return {"message": f"Model {model_id} created and saved successfully"}


@app.post("/output/")
def compute_model_output(body: ActivationRequest = Body(..., openapi_examples={
        f"example_{i}": {"summary": f"Example {i + 1}", "description": f"Example input and training data for case {i + 1}",
                         "value": {"model_id": "test", "input": ex}} for i, ex in enumerate(EXAMPLES)})):
    model_id = body.model_id
    log.info(f"Requesting output for model {model_id}")
    model = NeuralNetworkModel.deserialize(model_id)
    output, cost = model.compute_output(body.input.activation_vector, body.input.target_vector)
    return {"output_vector": output, "cost": cost}


# active training sessions by model id (one event loop, so a plain dict is safe), and the ids
# whose PUT /train/ is still loading the checkpoint (between the 409 check and the task start)
model_locks: Dict[str, Lock] = {}
_starting: set = set()


def _log_task_failure(task) -> None:
    if not task.cancelled() and task.exception() is not None:
        log.error(f"Background training failed: {task.exception()!r}")


@app.put("/train/")
async def train_model(body: TrainingRequest = Body(...)):
    model_id = body.model_id
    log.info(f"Requesting training for model {model_id}")
    lock = model_locks.setdefault(model_id, Lock())
    if lock.locked() or model_id in _starting:
        raise HTTPException(status_code=409, detail=f"Training already in progress for model {model_id}.")
    # the checkpoint loads OFF the event loop (seconds for a 25 M-1 B parameter model; the
    # reference parses it on the loop, main.py:270, and every /progress/ poll stalls meanwhile)
    _starting.add(model_id)
    try:
        model = await run_in_threadpool(NeuralNetworkModel.deserialize, model_id)
        data = [(item.activation_vector, item.target_vector) for item in body.training_data]
        hp = dict(epochs=body.epochs, learning_rate=body.learning_rate, batch_size=body.batch_size,
                  decay_rate=body.decay_rate, dropout_rate=body.dropout_rate, l2_lambda=body.l2_lambda,
                  beta1=body.adam_beta1, beta2=body.adam_beta2, epsilon=body.adam_epsilon)

        async def train():
            try:
                async with lock:
                    _starting.discard(model_id)  # the lock now says "in progress"
                    # one thread trains; with a multi-GPU train group up, a GPU model trains on every rank
                    await run_in_threadpool(service.train, model, data, hp)
            finally:
                _starting.discard(model_id)

        def _done(task) -> None:
            if task.cancelled():  # cancelled before its first step: its body (and finally) never ran
                _starting.discard(model_id)
            _log_task_failure(task)

        create_task(train()).add_done_callback(_done)
    except BaseException:
        # anything before the task exists (load, request unpacking, task creation) must not leave
        # the id marked as starting: every later PUT /train/ would answer 409
        _starting.discard(model_id)
        raise
    return JSONResponse(content={"message": f"Training for model {model_id} started asynchronously."},
                        status_code=202)


@app.get("/progress/")
def model_progress(model_id: str = ModelIdQuery(...)):
    log.info(f"Requesting progress for model {model_id}")
    model = NeuralNetworkModel.deserialize(model_id, meta_only=True)  # no parameters, no GPU
    return {"progress": model.progress, "average_cost": model.avg_cost,
            "average_cost_history": model.avg_cost_history, "status": model.status}


@app.get("/stats/")
def model_stats(model_id: str = ModelIdQuery(...)):
    log.info(f"Requesting stats for model {model_id}")
    return NeuralNetworkModel.deserialize(model_id, meta_only=True).stats


@app.delete("/model/")
def delete_model(model_id: str = ModelIdQuery(...)):
    log.info(f"Requesting deletion of model {model_id}")
    NeuralNetworkModel.delete(model_id)
    return Response(status_code=204)


def _uvicorn_log_config() -> dict:
    handler = {"level": "INFO", "class": "logging.StreamHandler", "formatter": "default"}
    quiet = {"level": "INFO", "handlers": ["default"], "propagate": False}
    return {
        "version": 1,
        "disable_existing_loggers": False,
        "formatters": {"default": {"format": LOG_FORMAT, "datefmt": DATE_FORMAT}},
        "handlers": {"default": handler},
        "loggers": {"uvicorn": quiet, "uvicorn.error": dict(quiet), "uvicorn.access": dict(quiet)},
        "root": {"level": "INFO", "handlers": ["default"]},
    }


if __name__ == "__main__":  # pragma: no cover
    import uvicorn

    uvicorn.run(app, host=os.environ.get("PZ_HOST", "127.0.0.1"), port=int(os.environ.get("PZ_PORT", "8000")),
                log_config=_uvicorn_log_config())
