"""santa_hip — MI355X-native block-Hungarian optimiser for Kaggle Santa 2017.

A from-scratch gfx950 build of the hot path of bigzhao/MPI-Hungarian-method
(mpi_single.py / mpi_twins.py): block cost build + scipy-exact LSAP + swap
apply + score, behind the C-ABI in include/santa_hip.h (libsanta_hip.so).

Reference-surface entry points:
    init(child_data, gift_data)                 module set-up (tables -> HBM)
    avg_normalized_happiness(pred, child_pref, gift_pref)
    optimize_block(child_block, current_gift_ids)
    optimize_block_twins(child_block, subm)
    optimize_block_triplets(child_block, subm)   (extension: 3-slot triplet units)
    linear_sum_assignment(C)
    my_optimizer(subm, score_org, comm, rank, size, gift_data, child_data)
"""
from ._lib import LIB_PATH, SantaHipError, lib  # noqa: F401  (fails loudly if the .so is missing)
from .api import (avg_normalized_happiness, init, optimize_block,  # noqa: F401
                  optimize_block_triplets, optimize_block_twins, session)
from .context import SantaGPU, score_from_sums  # noqa: F401
from .driver import my_optimizer, run_rounds  # noqa: F401
from .lsap import linear_sum_assignment, solve_batched, solve_hash  # noqa: F401

lib()  # load the C-ABI at import: no silent CPU path

__all__ = [
    "init", "session", "avg_normalized_happiness", "optimize_block", "optimize_block_twins",
    "optimize_block_triplets",
    "linear_sum_assignment", "solve_batched", "solve_hash", "my_optimizer", "run_rounds",
    "SantaGPU", "score_from_sums", "SantaHipError",
]
