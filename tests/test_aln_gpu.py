"""bwa mode on the device: pr_sw_run with pr_sw_batch.t_chain (the seeds of every kept chain,
aln_kernels.hip: mem_chain2aln over every seed with speculative first seeds and resumed walks,
mem_sort_dedup_patch, mem_mark_primary_se, mem_reg2sam's -T / -D filters and SAM order)
against the CPU restatement (oracle/aln_oracle.c over oracle/sw_oracle.c) read by read: the
same reported alignments in the same order with the same long read, strand, POS, CIGAR, AS,
FLAG and aligned intervals.  bwa-proovread itself is absent: parity with it is unpinned."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
pytestmark = pytest.mark.gpu


def _data(seed_, err, finish, n_lr=40, lr_len=2500, cov=15):
    from proovread_amd import seed, synth
    f = err / 0.15
    d = synth.simulate(seed_, 40000, n_lr, lr_len, cov, p_ins=0.09 * f, p_del=0.045 * f, p_sub=0.015 * f)
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    d = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(finish), threads=4))
    ix.close()
    return d


def _by_read(res, d):
    out = {}
    for i in range(res.n):
        t = int(res["task"][i])
        r = int(d.t_sr[t])
        assert res["status"][i] == 0
        out.setdefault(r, []).append((int(d.t_lr[t]), int(d.t_strand[t]), int(res["pos"][i]),
                                      [int(x) for x in res.cigar_ops(i)], int(res["score"][i]),
                                      int(res["flag"][i]), int(res["qb"][i]), int(res["qe"][i]),
                                      int(res["rb"][i]), int(res["re"][i]), int(res["truesc"][i]), t))
    return out


@pytest.mark.parametrize("finish,err", [(False, 0.15), (False, 0.05), (True, 0.05), (True, 0.02)])
def test_bwa_mode_matches_oracle(finish, err):
    import cpu_chain
    from proovread_amd import _abi, sw
    d = _data(41 + int(finish) + int(err * 100), err, finish)
    task = "bwa-sr-finish" if finish else "bwa-sr"
    ctx = _abi.default_context()
    res = sw.run(d.sw_input(), sw.default_opts(finish), ctx=ctx)
    rounds, n_ext, n_patch = sw.bwa_stats(ctx)
    print(f"rounds {rounds} extended {n_ext} patches {n_patch}")
    want = cpu_chain.bwa_alignments(d, task)
    got = _by_read(res, d)
    n = 0
    for r in range(d.n_sr):
        assert got.get(r, []) == want[r], r
        n += len(want[r])
    assert n == res.n and n > 5 * d.n_lr
    n_chain = len(np.unique(d.t_sr.astype(np.int64) * 65536 + d.t_chain))
    assert rounds >= 1 and n_ext >= n_chain > 0
    if finish:   # -D .75 drops low secondaries, -T 4 per base drops most 5 %-error alignments
        assert any(f & 0x100 for v in got.values() for (_, _, _, _, _, f, *_r) in v)


def test_bwa_mode_heads_lane_path(monkeypatch):
    """aln_heads_kernel's lane-0 path (reads with more chain heads than the wave's LDS list,
    forced here with a list of 3): the same alignments as the oracle"""
    import cpu_chain
    from proovread_amd import _abi, sw
    d = _data(43, 0.15, False)
    heads = np.unique(d.t_sr.astype(np.int64) * 65536 + d.t_chain) >> 16
    assert (np.bincount(heads) > 3).sum() > 100   # many reads take the lane path
    monkeypatch.setenv("PRGPU_HEADS_CAP", "3")
    res = sw.run(d.sw_input(), sw.default_opts(False), ctx=_abi.default_context())
    want = cpu_chain.bwa_alignments(d, "bwa-sr")
    got = _by_read(res, d)
    assert all(got.get(r, []) == want[r] for r in range(d.n_sr))
    assert res.n == sum(len(v) for v in want) > 0


def test_bwa_mode_seed_order_and_empty_reads():
    """reads without seeds, and a batch whose seeds are not grouped by read, fail loudly"""
    from proovread_amd import _abi, sw
    d = _data(77, 0.15, False, n_lr=12, lr_len=2000)
    inp = d.sw_input()
    bad = sw.SwInput(**{**inp.__dict__})
    perm = np.arange(len(inp.t_sr))[::-1].copy()
    for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen", "t_chain"):
        setattr(bad, k, np.ascontiguousarray(getattr(inp, k)[perm]))
    with pytest.raises(RuntimeError):
        sw.run(bad, sw.default_opts(False))
    keep = inp.t_sr >= d.n_sr // 2   # the first half of the reads have no seeds
    half = sw.SwInput(**{**inp.__dict__})
    for k in ("t_sr", "t_lr", "t_strand", "t_qbeg", "t_rbeg", "t_slen", "t_chain"):
        setattr(half, k, np.ascontiguousarray(getattr(inp, k)[keep]))
    res = sw.run(half, sw.default_opts(False), ctx=_abi.default_context())
    assert res.n > 0 and (half.t_sr[res["task"][:res.n]] >= d.n_sr // 2).all()


def test_iteration_from_device_seeds_equals_host_handed_seeds():
    """pr_iter_upload_gpu_seeds: the seeds pr_seed_gpu_map leaves in HBM feed the iteration
    without a host round trip; the corrected reads equal those of the same seeds handed over
    from the host (pr_iter_upload in bwa mode)."""
    from proovread_amd import _abi, cns, iteration, seed, sw, synth
    d = synth.simulate(53, 40000, 40, 2500, 15)
    ctx = _abi.default_context()
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    tasks, st = ix.map(d.sr_seq, d.sr_off, seed.default_opts(False))
    assert (st == 0).all() and len(tasks) > 10 * d.n_lr
    db = synth.with_seeds(d, tasks)
    cp = cns.CnsParams(coverage=11.25, use_ref_qual=True)
    it = iteration.Iteration(db, ctx=ctx)
    it.launch(sw.default_opts(False), cp)
    want = [(r.status, r.fastq, r.trace) for r in it.results()]
    ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), keep_on_device=True)
    it2 = iteration.Iteration(d, ctx=ctx, gpu_seeds=True)
    assert it2.n_task == len(tasks)
    it2.launch(sw.default_opts(False), cp)
    got = [(r.status, r.fastq, r.trace) for r in it2.results()]
    assert got == want and all(g[0] == 0 for g in got)


@pytest.mark.parametrize("task,sr_len", [("bwa-mr-1", 600), ("bwa-mr-finish", 950)])
def test_bwa_mode_mr_reads_match_oracle(task, sr_len):
    """mr mode (short reads > 150 bp, bin/proovread:637-641; up to 1000 bp, :457) with
    proovread.cfg:343-365's options: the seeds come through mem_flt_chained_seeds (reads
    >= 440 bp at -W 20, >= 880 bp at -W 40), GPU seeding = host seeding, and the device's
    bwa mode = the oracle read by read."""
    import cpu_chain
    from proovread_amd import _abi, seed, sw, synth, tasks
    so_, wo = tasks.options(task)
    finish = task.endswith("finish")
    f = 0.02 / 0.15 if finish else 1.0   # finish's -T 4 per base needs long reads corrected to ~2 % error
    d = synth.simulate(61 + sr_len, 60000, 30, 4000, 8, p_ins=0.09 * f, p_del=0.045 * f, p_sub=0.015 * f,
                       sr_len=sr_len)
    ctx = _abi.default_context()
    hx = seed.SeedIndex(d.lr_seq, d.lr_off)
    tk = hx.map(d.sr_seq, d.sr_off, so_, threads=4)
    hx.close()
    gx = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    gtk, st = gx.map(d.sr_seq, d.sr_off, so_)
    assert (st == 0).all() and np.array_equal(gtk, tk)
    d = synth.with_seeds(d, tk)
    res = sw.run(d.sw_input(), wo, ctx=ctx)
    swt = (wo.a, wo.b, wo.o_del, wo.o_ins, wo.e_del, wo.e_ins, wo.w, wo.pen_clip5, wo.pen_clip3, wo.zdrop,
           wo.min_score_per_base)
    want = cpu_chain.bwa_alignments(d, swt, drop_ratio=wo.drop_ratio)
    got = _by_read(res, d)
    n = 0
    for r in range(d.n_sr):
        assert got.get(r, []) == want[r], r
        n += len(want[r])
    assert n == res.n and n > 2 * d.n_lr


@pytest.mark.parametrize("err", [0.05, 0.15])
def test_bwa_mode_patches_match_oracle(err):
    """mem_patch_reg's global scores (aln_patch_wave_kernel, a wave per patch): long reads with
    N windows (a short read across one is extended up to it from each side: two colinear
    regions the final pass merges through a patch); the
    device = the oracle read by read, and patches were scored."""
    import cpu_chain
    from proovread_amd import _abi, seed, sw, synth
    f = err / 0.15
    d = synth.simulate(97 + int(err * 100), 40000, 40, 2500, 15, p_ins=0.09 * f, p_del=0.045 * f, p_sub=0.015 * f)
    rng = np.random.default_rng(5)
    lr = d.lr_seq.copy()
    for i in range(len(d.lr_off) - 1):   # a 10-110 bp N window every ~300 bp
        a, b = int(d.lr_off[i]), int(d.lr_off[i + 1])
        for x in range(a + 100, b - 200, 300):
            x += int(rng.integers(0, 100))
            lr[x:x + int(rng.integers(10, 111))] = 4
    d.lr_seq = lr
    ix = seed.SeedIndex(d.lr_seq, d.lr_off)
    d = synth.with_seeds(d, ix.map(d.sr_seq, d.sr_off, seed.default_opts(False), threads=4))
    ix.close()
    ctx = _abi.default_context()
    res = sw.run(d.sw_input(), sw.default_opts(False), ctx=ctx)
    rounds, n_ext, n_patch = sw.bwa_stats(ctx)
    print(f"rounds {rounds} extended {n_ext} patches {n_patch}")
    want = cpu_chain.bwa_alignments(d, "bwa-sr")
    got = _by_read(res, d)
    assert all(got.get(r, []) == want[r] for r in range(d.n_sr))
    assert res.n == sum(len(v) for v in want) > 0
    assert n_patch > 0
