"""Exact-parity multi-GPU layout of one iteration ("exact-parity option").

Sharding the long reads (each rank indexes only its shard) is not bit-exact against a
single full index: occurrence caps (-c, -y) count over the whole index and -D compares
chains of one short read across all long reads.  The exact layout keeps the full
long-read index on every rank (a few GB even at configs[4]; 288 GB of HBM per GPU),
shards the *short reads* (contiguous ranges, so every rank seeds exactly what the
single run seeds for those reads), and routes each seed-extension task to the rank that
owns its long read with one all-to-all.  The owner then runs SW + hand-off + consensus
(pr_iter_*) for its long reads.

Order: the single run groups tasks by long read, stably, i.e. in read order within a
long read.  Rank r holds reads [s_r, e_r) with s_r increasing in r, and the all-to-all
delivers rank 0's tasks first, then rank 1's ... each in its own read order — so the
owner's stable grouping reproduces the single run's order exactly.

The exchange goes through comm.py: RCCL in libprgpu on GPUs, torch gloo in the CPU tests.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .seed import TASK_DTYPE

NFIELD = len(TASK_DTYPE.names)


def lr_bounds(lr_off: np.ndarray, world: int) -> np.ndarray:
    """[world+1] contiguous long-read ranges with about equal bases (rank r owns [b[r], b[r+1]))."""
    n = len(lr_off) - 1
    tot = int(lr_off[-1])
    b = np.zeros(world + 1, np.int64)
    for r in range(1, world):
        b[r] = int(np.searchsorted(lr_off[1:], tot * r / world, side="left"))
        b[r] = max(b[r], b[r - 1])
    b[world] = n
    return b


def sr_range(n_sr: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous short-read shard of a rank."""
    return n_sr * rank // world, n_sr * (rank + 1) // world


def owners(tasks: np.ndarray, bounds: np.ndarray) -> np.ndarray:
    return np.searchsorted(bounds, tasks["lr"].astype(np.int64), side="right") - 1


def exchange_tasks(tasks: np.ndarray, bounds: np.ndarray, comm) -> np.ndarray:
    """All-to-all of seed-extension tasks to the owners of their long reads.

    tasks: this rank's tasks (TASK_DTYPE, read order); comm: a comm.RcclComm (GPU ranks)
    or comm.TorchComm (gloo, CPU tests).  Returns the tasks of the long reads this rank
    owns, source-rank-major, each source's order kept."""
    own = owners(tasks, bounds)
    order = np.argsort(own, kind="stable")
    send = np.ascontiguousarray(tasks[order]).view(np.int32).reshape(-1, NFIELD)
    send_counts = np.bincount(own, minlength=comm.world).astype(np.int64)
    got = comm.alltoallv_rows(send, send_counts)
    return np.ascontiguousarray(got).view(TASK_DTYPE).reshape(-1)


def group_by_lr(tasks: np.ndarray) -> np.ndarray:
    """Stable grouping by long read (the iteration hand-off's layout)."""
    return tasks[np.argsort(tasks["lr"], kind="stable")]


def localize(tasks: np.ndarray, bounds: np.ndarray, rank: int) -> np.ndarray:
    """Long-read ids relative to the rank's shard (its pr_iter batch holds only its long reads)."""
    t = tasks.copy()
    t["lr"] -= int(bounds[rank])
    return t
