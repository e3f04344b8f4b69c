from .comm import *  # noqa: F401,F403
from .comm import (init_distributed, is_initialized, get_rank, get_world_size, get_local_rank, new_group,  # noqa: F401
                   all_reduce, reduce, reduce_scatter_tensor, all_gather_into_tensor, all_gather, broadcast,
                   all_to_all_single, send, recv, isend, irecv, barrier, ReduceOp, configure, log_summary,
                   verify_fingerprints, enable_fingerprint, reset_fingerprint, group_ranks, destroy_process_group)
