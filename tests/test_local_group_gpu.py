"""The multi-rank device paths on one GPU: an in-process group of ranks (include/prgpu.h
pr_comm_init_local: threads of this process, one context each, device copies in place of
RCCL) runs the same communicator calls the one-process-per-GPU launch makes over RCCL.

* the collectives themselves (all-reduce, all-gather, all-to-all of host and device blocks)
  at world 3 against their definitions;
* the whole sr-noccs loop on the device stages at world 2 and 3 (exact-parity layout:
  short-read shards seeded and aligned per rank, alignments exchanged to the long reads'
  owners with pr_aln_exchange, owned consensus and masking, the resident long-read sets
  all-gathered by pr_lrset_commit) equals the world-1 loop byte for byte: reads,
  qualities, chimera lines and every task's statistics."""
import dataclasses
import threading

import numpy as np
import pytest

from proovread_amd import correct


def _ranks(world, fn):
    """fn(rank, ctx, comm) on `world` threads of one group; -> results in rank order."""
    from proovread_amd import _abi, comm
    g = comm.LocalGroup(world)
    ctxs = [_abi.Context(0) for _ in range(world)]
    cms = [comm.LocalComm(ctxs[r], g, r) for r in range(world)]
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            out[r] = fn(r, ctxs[r], cms[r])
        except BaseException as e:   # noqa: BLE001 - reported below
            err[r] = e
            g.abort()   # the other ranks must not wait for this one in a collective

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank did not finish"
    for c in cms:
        c.close()
    g.close()
    for e in err:
        if e is not None:
            raise e
    return out


@pytest.mark.gpu
def test_local_group_collectives():
    from proovread_amd import _abi
    W = 3

    def fn(r, ctx, cm):
        red = cm.allreduce_ints([r + 1, 10 * r, -r])
        mx = cm.allreduce_ints([r, -r], op=1)
        gat = cm.allgather_bytes(bytes([65 + r]) * (r + 2))
        # rank r sends (r + 1) * (d + 1) bytes of value 16 r + d to rank d
        counts = np.array([(r + 1) * (d + 1) for d in range(W)], np.int64)
        send = b"".join(bytes([16 * r + d]) * int(counts[d]) for d in range(W))
        a2a = cm.alltoallv_bytes(send, counts)
        # device all-reduce in place
        buf = _abi.DevBuffer(ctx, 16)
        buf.upload(np.array([r, 2 * r], np.int64))
        cm.allreduce_dev(buf.ptr, 2)
        dv = buf.download(np.int64)
        buf.close()
        return red, mx, gat, a2a, [int(x) for x in dv[:2]]

    res = _ranks(W, fn)
    for r, (red, mx, gat, a2a, dv) in enumerate(res):
        assert red == [6, 30, -3]
        assert mx == [2, 0]
        assert gat == [bytes([65 + k]) * (k + 2) for k in range(W)]
        assert a2a == b"".join(bytes([16 * s + r]) * ((s + 1) * (r + 1)) for s in range(W))
        assert dv == [3, 6]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_local_group_loop_equals_world1(world):
    from test_correct_loop import _inputs
    _, lrs, srd = _inputs(seed=6)
    cfg = correct.LoopConfig(coverage=40.0)
    want = correct.run(lrs, srd, cfg)   # world 1, device stages

    def fn(r, ctx, cm):
        return correct.run(lrs, srd, cfg, stages=correct.GpuStages(ctx), comm=cm)

    got = _ranks(world, fn)
    n_tasks = [0] * len(want.log)
    for res in got:
        assert res.reads.ids == want.reads.ids
        assert res.reads.seqs == want.reads.seqs
        assert res.reads.quals == want.reads.quals
        assert res.chim == want.chim
        for k, (g, w) in enumerate(zip(res.log, want.log)):
            assert (g.task, g.n_sr, g.bpt, g.bpn, g.shortcut) == (w.task, w.n_sr, w.bpt, w.bpn, w.shortcut)
            n_tasks[k] += g.n_tasks
        assert len(res.log) == len(want.log)
    # the ranks' seed counts (each its short-read shard) add up to the single run's
    assert n_tasks == [w.n_tasks for w in want.log]


@pytest.mark.gpu
def test_local_group_exact_world1_with_comm_equals_plain():
    """World 1 with a communicator: the exchange and the commit go through the group's calls."""
    from test_correct_loop import _inputs
    _, lrs, srd = _inputs(seed=7)
    cfg = correct.LoopConfig(coverage=40.0)
    want = correct.run(lrs, srd, cfg)
    got = _ranks(1, lambda r, ctx, cm: correct.run(lrs, srd, dataclasses.replace(cfg, exact_layout=True),
                                                   stages=correct.GpuStages(ctx), comm=cm))[0]
    assert got.reads.seqs == want.reads.seqs and got.reads.quals == want.reads.quals
    assert got.chim == want.chim
