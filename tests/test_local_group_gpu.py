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


def _shared_task_inputs():
    """One genome, one long-read set and one short-read run in sequencer order (unsorted over
    the genome) -- what every rank holds in the exact layout."""
    from proovread_amd import correct, synth
    d = synth.simulate_reads(31, 400_000, 300, 5_000, 12_000, threads=8)
    pool = np.frombuffer(b"ACGTN", np.uint8)[d.lr_seq]
    reads = correct.LongReads([f"lr{i}" for i in range(d.n_lr)],
                              pools=(pool, d.lr_off, np.full(len(pool), ord("$"), np.uint8)))
    return d, reads


def _task(ctx, cm, d, reads, exact):
    from proovread_amd import cns, correct, iteration
    st = correct.GpuStages(ctx)
    st.load(reads)
    params = cns.CnsParams(coverage=11.25, use_ref_qual=True, max_ins_length=0)
    out = st.task("bwa-sr-1", d.sr_seq, d.sr_off, params, (20, 300.0), comm=cm, exact=exact,
                  mask_cfg=("20,41,80,130,60,0.7", 150))
    src = iteration.exchange_sources(ctx) if exact else None
    off, seq, qual, mp = st.lrs.download(seq=True, qual=True, mapping=True)
    return out, src, off, seq, qual, mp


@pytest.mark.gpu
def test_local_group_task_on_shared_genome_crosses_ranks():
    """World 3 on ONE shared dataset (short reads in sequencer order): most alignments a rank
    receives come from the other ranks' short-read shards (pr_aln_exchange moves them), and the
    task's corrected reads, qualities and masked reads equal the world-1 task's byte for byte."""
    d, reads = _shared_task_inputs()
    from proovread_amd import _abi
    want = _task(_abi.default_context(), None, d, reads, False)
    got = _ranks(3, lambda r, ctx, cm: _task(ctx, cm, d, reads, True))
    bpt = bpn = n_tasks = 0
    for r, (out, src, off, seq, qual, mp) in enumerate(got):
        assert np.array_equal(off, want[2])
        assert np.array_equal(seq, want[3]) and np.array_equal(qual, want[4]) and np.array_equal(mp, want[5])
        assert len(src) == 3 and sum(src) > 1000
        assert sum(src) - src[r] > 0.5 * sum(src), src   # received from the other ranks' shards
        bpt, bpn, n_tasks = bpt + out.bpt, bpn + out.bpn, n_tasks + out.n_tasks
    assert (bpt, bpn, n_tasks) == (want[0].bpt, want[0].bpn, want[0].n_tasks)


@pytest.mark.gpu
def test_local_group_error_on_one_rank_returns_on_every_rank():
    """a failure on one rank before the exchange's collectives (here rank 1's
    long-read bounds are not ascending, so its pack fails) makes pr_aln_exchange return an
    error on EVERY rank (pr_comm_agree) instead of leaving the others in the all-to-all."""
    from proovread_amd import _abi, correct, exact_shard as ex, iteration, seed, sw
    d, reads = _shared_task_inputs()

    def fn(r, ctx, cm):
        L = _abi.lib()
        st = correct.GpuStages(ctx)
        st.load(reads)
        st.lrs.index(st.lrs.MAP)
        s, e = ex.sr_range(d.n_sr, 2, r)
        a0, a1 = int(d.sr_off[s]), int(d.sr_off[e])
        seed._map_gpu(L, ctx, d.sr_seq[a0:a1], d.sr_off[s:e + 1] - a0, seed.default_opts(False), False,
                      keep_on_device=True)
        iteration.ShardSW(ctx, d.sr_seq, d.sr_off, s, e, None, d.lr_off, device_pools=True).launch(
            sw.default_opts(finish=False))
        bounds = ex.lr_bounds(d.lr_off, 2)
        if r == 1:
            bounds = np.array([0, d.n_lr, d.n_lr // 2], np.int64)   # not ascending
        with pytest.raises(RuntimeError) as ei:
            iteration.exchange(ctx, cm, s, bounds)
        return str(ei.value)

    msgs = _ranks(2, fn)
    assert "ascending" in msgs[1]
    assert "another rank failed" in msgs[0]
