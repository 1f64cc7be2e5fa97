from . import comm_timer
from .comm import all_gather, all_gather_tensor, all_reduce_sum_, reduce_tensor
from .dist import DistContext, barrier, destroy, get_rank, get_world_size, init_distributed
from .peer import (PeerAllReduce, PeerTimeoutError, SyncBNMismatchError, check_peer_errors, check_syncbn_consistency,
                   peer_active, peer_errors, setup_peer_syncbn, teardown_peer_syncbn)
from .reducer import GradReducer, broadcast_module_state
from .syncbn import combine_stats, convert_sync_batchnorm, sync_batch_norm

__all__ = [
    "DistContext", "init_distributed", "barrier", "destroy", "get_rank", "get_world_size",
    "GradReducer", "broadcast_module_state",
    "PeerAllReduce", "setup_peer_syncbn", "teardown_peer_syncbn", "peer_active", "peer_errors",
    "check_peer_errors", "PeerTimeoutError", "check_syncbn_consistency", "SyncBNMismatchError",
    "convert_sync_batchnorm", "sync_batch_norm", "combine_stats",
    "all_gather", "all_gather_tensor", "all_reduce_sum_", "reduce_tensor",
]
