"""Exact-parity multi-GPU layout: full long-read index on every rank,
contiguous short-read shards, one all-to-all of seed-extension tasks to the long-read
owners.  world_size-2 gloo run on CPU: every rank's task list equals the single-process
(full index, all reads) task list restricted to its long reads, in the same order."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    from proovread_amd import synth
    return synth.simulate(31, 80_000, 80, 4000, 30.0, sr_frac=0.5)


def _rank(rank, world, port, outdir):
    import torch.distributed as dist
    from proovread_amd import exact_shard as ex, seed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = _data()
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)            # full index on every rank
    s, e = ex.sr_range(d.n_sr, world, rank)
    tasks = ix.map(d.sr_seq, d.sr_off, threads=2)      # all reads, then keep this rank's shard
    mine = tasks[(tasks["sr"] >= s) & (tasks["sr"] < e)]
    # seeding the shard alone must give the same tasks (sr ids relative to the shard)
    sub = ix.map(d.sr_seq[d.sr_off[s]:d.sr_off[e]], d.sr_off[s:e + 1] - d.sr_off[s], threads=2)
    assert len(sub) == len(mine) and np.array_equal(sub["sr"] + s, mine["sr"])
    b = ex.lr_bounds(d.lr_off, world)
    from proovread_amd.comm import TorchComm
    got = ex.group_by_lr(ex.exchange_tasks(mine, b, TorchComm()))
    np.save(os.path.join(outdir, f"r{rank}.npy"), got)
    dist.barrier()
    dist.destroy_process_group()


def test_exact_layout_two_ranks(tmp_path):
    from proovread_amd import exact_shard as ex, seed
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d = _data()
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    full = ex.group_by_lr(ix.map(d.sr_seq, d.sr_off, threads=2))
    b = ex.lr_bounds(d.lr_off, world)
    assert 0 < b[1] < d.n_lr
    n = 0
    for r in range(world):
        got = np.load(tmp_path / f"r{r}.npy")
        want = full[(full["lr"] >= b[r]) & (full["lr"] < b[r + 1])]
        assert np.array_equal(got, want)
        n += len(got)
        loc = ex.localize(got, b, r)
        assert loc["lr"].min() >= 0 and loc["lr"].max() < b[r + 1] - b[r]
    assert n == len(full) > 1000


def test_lr_bounds_balance_bases():
    from proovread_amd import exact_shard as ex
    off = np.cumsum([0] + [1000] * 10 + [5000] * 2).astype(np.int64)
    b = ex.lr_bounds(off, 4)
    assert b[0] == 0 and b[-1] == 12 and np.all(np.diff(b) >= 0)
    assert ex.sr_range(10, 3, 2) == (6, 10)
