"""Native operators (``torch.ops.pz``) and their autograd wrappers."""
from . import native  # noqa: F401
