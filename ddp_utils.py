"""Reference-compatible facade for ``ddp_utils`` (reference ddp_utils.py).

``reduce_tensor(t)`` -> mean over ranks; ``all_gather(obj)`` -> list of every
rank's picklable object.  Implemented in
``pytorch_imageclassification_distributed_amd.parallel.comm``.
"""
from pytorch_imageclassification_distributed_amd.parallel.comm import all_gather, reduce_tensor

__all__ = ["all_gather", "reduce_tensor"]
