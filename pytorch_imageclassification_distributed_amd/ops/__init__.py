from . import functional
from .functional import get_backend, set_backend, use_hip

__all__ = ["functional", "get_backend", "set_backend", "use_hip"]
