"""Data parallelism over RCCL (``torch.distributed`` nccl backend) / gloo on CPU."""
from .dist import DataParallelContext, get_context, init_from_env, set_context, shutdown  # noqa: F401
