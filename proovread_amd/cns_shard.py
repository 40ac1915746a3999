"""Multi-GPU drop-in for proovread's consensus fan-out.

bin/proovread:1596-1637 writes one bam2cns command line per long-read chunk into
`TASK.cmds` and runs them with `cat TASK.cmds | xargs -P THREADS -L 1 bam2cns`.
This module runs the same command file on one or more GPUs:

    python -m proovread_amd.cns_shard TASK.cmds                      # one GPU
    python -m torch.distributed.run --nproc-per-node 8 \\
        --master-addr 127.0.0.1 -m proovread_amd.cns_shard TASK.cmds  # one rank per GPU

Chunks are independent (each has its own output prefix), so they are dealt to
ranks round-robin (`chunk % world_size == rank`) with no data-path collective;
each rank batches all of its chunks into one launch (bam2cns.execute) and writes
the usual per-chunk files, which proovread's merge step (bin/proovread:1640-1699)
reads unchanged.  The only collective is a final barrier so rank 0 returns after
every chunk file exists (RCCL in libprgpu on GPU ranks, comm.py).
"""
from __future__ import annotations

import ctypes as C
import os
import shlex
import sys
from typing import List, Sequence

from . import bam2cns


def read_cmds(path: str) -> List[List[str]]:
    """One bam2cns argument vector per non-empty line of the command file."""
    out = []
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if line:
                out.append(shlex.split(line))
    return out


def my_chunks(n_chunks: int, rank: int, world: int) -> List[int]:
    return list(range(rank, n_chunks, world))


def run(cmds: Sequence[Sequence[str]], rank: int = 0, world: int = 1) -> List[int]:
    mine = my_chunks(len(cmds), rank, world)
    jobs = [bam2cns.prepare(cmds[i]) for i in mine]
    bam2cns.execute(jobs)
    return mine


def _barrier_comm(rank: int, world: int):
    """The final barrier's communicator: RCCL inside libprgpu on GPU ranks (no torch in the
    process), gloo where no device is visible (the CPU multi-process test: chunks without
    --ref never reach the device)."""
    from . import _abi, comm
    n = C.c_int(0)
    _abi.lib().pr_device_count(C.byref(n))
    if n.value > 0:
        return comm.RcclComm(_abi.default_context(), rank, world)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    return comm.TorchComm()


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 1:
        print("usage: cns_shard TASK.cmds", file=sys.stderr)
        return 2
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    cm = _barrier_comm(rank, world) if world > 1 else None
    try:
        run(read_cmds(argv[0]), rank, world)
    finally:
        if cm is not None:
            cm.barrier()
            if hasattr(cm, "close"):
                cm.close()
            else:
                cm.dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
