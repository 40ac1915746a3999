"""BASELINE configs[2] and configs[3] at one rank's size, on one GPU, through the product's
multi-GPU layout (SURVEY.md §8d C3 / C4, §8e exact-parity option).

proovread maps every sampled short read against the whole long-read set (bin/proovread:1270
index, 1313 mem), so in the exact-parity layout every rank indexes ALL long reads and aligns
its share of the short reads; each reported alignment then goes to the owner of its long read.
One rank's share of a bwa-sr-1 task at N = 8:

  configs[2]  50 Mb genome, 100 k x 10 kb long reads (1 Gb indexed), 50x short reads sampled
              6 of 20 chunks (cov2seqchunker at --coverage 50, proovread:2085-2102) -> 1/8 of
              them: 625 k reads
  configs[3]  135 Mb genome, 270 k x 10 kb long reads (2.7 Gb, 5.4 G text positions), 80x
              short reads sampled 4 of 20 chunks -> 1/8: 1.8 M reads

The task runs exactly as correct.GpuStages runs it for a rank (pr_lrset_index over the
resident set, pr_seed_gpu_map of the shard, pr_sw_upload_gpu_seeds + pr_sw_launch,
pr_aln_exchange with PRGPU_XCHG_FORCE=1 so the owner pack and the exchange run at world 1,
pr_iter_upload_owned + pr_iter_launch, pr_iter_mask, pr_lrset_commit).  World 1 owns every
long read, so its consensus buffers are 8x a real rank's: the measured peak bounds a rank of
the N = 8 run from above.

Checked: every read's consensus status is 0; the masked fraction is in (0, 1); GPU seeds =
the host seeding path (seed_core.h on the CPU, over the same full index) on 20 k random short
reads plus every short read with a seed on the sampled long reads; the consensus of 6 long
reads spread over the set = the oracle chain (bwa mem per-read alignment + SW restatement,
-b/-l, coordinate order, the consensus restatement pinned to the Perl engine) byte for byte.
The library's peak device memory per buffer group is written to gpurun_out/ (DESIGN.md §6).
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))

pytestmark = pytest.mark.gpu

# (seed, genome bp, long reads, --coverage)
CONFIGS = {
    "configs2": (20261015 + 3, 50_000_000, 100_000, 50.0),
    "configs3": (20261015 + 4, 135_000_000, 270_000, 80.0),
}
RANKS = 8
TASK_COV = 15.0          # sr-coverage of bwa-sr-1 (proovread.cfg:188-192)


def rank_share(genome: int, cov: float) -> int:
    """Short reads of one rank's share of one bwa-sr iteration's sample."""
    per_step = int(20 * (TASK_COV / cov) + .5)           # cov2seqchunker (proovread:2085-2102)
    return int(round(cov * genome / 150 * per_step / 20 / RANKS))


def _log(cfg, rec):
    out = ROOT / "gpurun_out"
    if out.is_dir():
        (out / f"scale_{cfg}.json").write_text(json.dumps(rec, indent=1))


@pytest.mark.parametrize("cfg", ["configs2", "configs3"])
def test_one_rank_share_on_one_gpu(cfg, monkeypatch):
    import cpu_chain
    from proovread_amd import _abi, cns, correct, seed, synth
    monkeypatch.setenv("PRGPU_XCHG_FORCE", "1")
    sd, glen, n_lr, cov = CONFIGS[cfg]
    n_sr = rank_share(glen, cov)
    rec = {"config": cfg, "long_reads": n_lr, "short_reads": n_sr}
    t = time.perf_counter()
    d = synth.simulate_reads(sd, glen, n_lr, 10_000, n_sr, threads=16)
    rec["gen_s"] = round(time.perf_counter() - t, 1)
    rec["long_read_bases"] = int(d.lr_off[-1])
    # a context of its own, destroyed at the end: the next tests get the device memory back
    ctx = _abi.Context(int(os.environ.get("LOCAL_RANK", "-1")))
    try:
        _run(cfg, ctx, sd, glen, n_lr, cov, n_sr, d, rec, cpu_chain, _abi, cns, correct, seed, synth)
    finally:
        ctx.close()


def _run(cfg, ctx, sd, glen, n_lr, cov, n_sr, d, rec, cpu_chain, _abi, cns, correct, seed, synth):
    ascii_pool = np.frombuffer(b"ACGTN", np.uint8)[d.lr_seq]
    reads = correct.LongReads([f"lr{i}" for i in range(n_lr)],
                              pools=(ascii_pool, d.lr_off, np.full(len(ascii_pool), ord("$"), np.uint8)))
    _abi.mem_reset_peak()
    st = correct.GpuStages(ctx)
    t = time.perf_counter()
    st.load(reads)
    del ascii_pool, reads
    cap = min(cov, TASK_COV) * 0.75                          # proovread:1540-1541
    binf = (20, 20.0 * min(cov, TASK_COV))                   # -b/-l, proovread:1302-1313
    params = cns.CnsParams(coverage=cap, use_ref_qual=True, max_ins_length=0)
    out = st.task("bwa-sr-1", d.sr_seq, d.sr_off, params, binf, comm=None, exact=True,
                  mask_cfg=("20,41,80,130,60,0.7", 150))
    rec["task_s"] = round(time.perf_counter() - t, 1)
    rec["device_ms"] = round(st.device_ms, 1)
    mem = _abi.mem_stats()
    rec["peak_device_bytes"] = mem["peak"]
    rec["groups_at_peak"] = {k: v["at_total_peak"] for k, v in mem["groups"].items()}
    rec["group_peaks"] = {k: v["peak"] for k, v in mem["groups"].items()}
    rec["seeds"] = out.n_tasks
    it = st.last_iteration
    L0 = _abi.lib()
    rec["event_ms"] = {"index": round(seed._last_ms(L0.pr_seed_gpu_index_last_ms, ctx), 1),
                       "seeding": round(seed._last_ms(L0.pr_seed_gpu_last_ms, ctx), 1),
                       **{k: round(v, 1) for k, v in zip(("sw_extend", "sw_global_cigar", "exchange_handoff",
                                                          "consensus"), it.timing())}}
    rec["seeding_phases"] = seed._phase_ms(L0, ctx)
    rec["alignments"] = it.alignment_stats()[0]
    _log(cfg, rec)
    status = it.statuses()
    assert len(status) == n_lr
    assert (status == 0).all(), np.flatnonzero(status)[:10]
    frac = out.bpn / out.bpt
    rec["masked_frac"] = round(frac, 4)
    assert 0.0 < frac < 1.0
    assert rec["alignments"] > 10 * n_lr // RANKS

    # GPU seeds of every short read (same device index), then the host path on a sample
    L = _abi.lib()
    so = seed.default_opts(False)
    gpu_tasks, gst = seed._map_gpu(L, ctx, d.sr_seq, d.sr_off, so, False)
    assert (gst == 0).all()
    assert len(gpu_tasks) == out.n_tasks
    sample_lrs = [int(x) for x in np.linspace(0, n_lr - 1, 6).astype(np.int64)]
    on_sample = np.isin(gpu_tasks["lr"], sample_lrs)
    rng = np.random.default_rng(sd)
    picked = np.union1d(np.unique(gpu_tasks["sr"][on_sample]), rng.choice(n_sr, 20_000, replace=False))
    sub_off = np.zeros(len(picked) + 1, np.int64)
    sub_off[1:] = np.cumsum(np.full(len(picked), 150, np.int64))
    sub_seq = d.sr_seq.reshape(-1, 150)[picked].reshape(-1)
    t = time.perf_counter()
    hx = seed.SeedIndex(d.lr_seq, d.lr_off)
    rec["host_index_s"] = round(time.perf_counter() - t, 1)
    host = hx.map(sub_seq, sub_off, so, threads=16)
    hx.close()
    host["sr"] = picked[host["sr"]]
    want_gpu = gpu_tasks[np.isin(gpu_tasks["sr"], picked)]
    del gpu_tasks
    for f in host.dtype.names:
        assert np.array_equal(host[f], want_gpu[f]), f
    rec["seed_check_reads"] = int(len(picked))
    rec["seed_check_seeds"] = int(len(host))

    # consensus of the sampled long reads = the oracle chain over the same seeds
    dd = synth.with_seeds(d, host)
    o = ob.sw_opts("bwa-sr")
    swt = (o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w, o.pen_clip5, o.pen_clip3, o.zdrop, o.min_score_per_base)
    _, _, want, _ = cpu_chain.run_sample(dd, sample_lrs, task=swt, coverage=cap, use_ref_qual=True,
                                         detect_chimera=False, workers=16, full=True, bin_filter=binf, drop_ratio=0.0)
    got = it.results_of(sample_lrs)
    for i, g, (rc, fq, trace, ch) in zip(sample_lrs, got, want):
        assert rc == 0 and g.status == 0, (i, rc, g.status)
        assert g.fastq == fq, i
        assert g.trace == trace, i
        assert ch == "" and not g.chim, i
    rec["oracle_reads"] = sample_lrs
    _log(cfg, rec)


def test_configs2_loop_one_rank_share(monkeypatch):
    """configs[2] as BASELINE states it, an iterative loop, at one rank's
    share on one GPU: the index of ALL 100 k long reads every task, each task's SeqChunker sample
    cut to rank 0's 1/8 (correct.run_tasks sample_shard), bwa-sr-1 .. bwa-sr-6 with
    mask_shortcut_frac, then bwa-sr-finish (the lazy occurrence table at 1 Gb).  Checked: every
    task commits (every read's status 0), the masked fractions never fall, GPU seeds = the host
    path on finish-task reads, and 6 spread long reads' finish consensus and chimera lines = the
    oracle chain over the pre-finish reads.  A rank's consensus sees 1/8 of the coverage here, so
    the masked fractions stay far below a real run's (the shortcut fires on the 3 % gain rule)."""
    import cpu_chain
    from proovread_amd import _abi, correct, seed, synth
    from proovread_amd import tasks as T
    monkeypatch.setenv("PRGPU_XCHG_FORCE", "1")
    sd, glen, n_lr, cov = CONFIGS["configs2"]
    n_sr = int(round(cov * glen / 150))
    rec = {"config": "configs2-loop", "long_reads": n_lr, "short_reads_total": n_sr, "ranks": RANKS}
    t = time.perf_counter()
    d = synth.simulate_reads(sd, glen, n_lr, 10_000, n_sr, threads=16)
    rec["gen_s"] = round(time.perf_counter() - t, 1)
    ctx = _abi.Context(int(os.environ.get("LOCAL_RANK", "-1")))
    try:
        ascii_pool = np.frombuffer(b"ACGTN", np.uint8)[d.lr_seq[:int(d.lr_off[-1])]]
        reads = correct.LongReads([f"lr{i}" for i in range(n_lr)],
                                  pools=(ascii_pool, d.lr_off, np.full(len(ascii_pool), ord("$"), np.uint8)))
        _abi.mem_reset_peak()
        st = correct.GpuStages(ctx)
        st.load(reads)
        del ascii_pool, reads
        srs = correct.ShortReads.from_pool(d.sr_seq[:int(d.sr_off[-1])], d.sr_off)
        st.load_short_reads(srs)
        cfg = correct.LoopConfig(coverage=cov, exact_layout=True)
        pre_finish = {}
        peaks = []

        def on_task(task):
            m = _abi.mem_stats()
            peaks.append(m["peak"])
            _abi.mem_reset_peak()
            if task.endswith("finish"):
                off, seq, qual, _ = st.lrs.download(seq=True, qual=True)
                pre_finish.update(off=off, seq=seq, qual=qual)

        t = time.perf_counter()
        chim, _, log = correct.run_tasks(st, srs, list(T.MODE_TASKS["sr-noccs"][1:]), cfg, "sr-noccs", 150, True,
                                         None, sample_shard=(0, RANKS), on_task=on_task)
        rec["loop_s"] = round(time.perf_counter() - t, 1)
        peaks.append(_abi.mem_stats()["peak"])
        rec["tasks"] = [{"task": e.task, "short_reads": e.n_sr, "seeds": e.n_tasks, "wall_ms": e.wall_ms,
                         "masked_frac": e.masked_frac, "shortcut": e.shortcut, "stage_event_ms": e.stage_ms}
                        for e in log]
        rec["peak_device_bytes_per_task"] = peaks[1:]
        rec["chimera_lines"] = len(chim)
        _log("configs2_loop", rec)
        assert log[-1].task == "bwa-sr-finish" and len(log) >= 2
        fr = [e.masked_frac for e in log if e.masked_frac is not None]
        assert all(0.0 <= f < 1.0 for f in fr) and all(b >= a for a, b in zip(fr, fr[1:])), fr
        it = st.last_iteration
        status = it.statuses()
        assert len(status) == n_lr and (status == 0).all()
        sample_lrs = [int(x) for x in np.linspace(0, n_lr - 1, 6).astype(np.int64)]
        got = it.results_of(sample_lrs)   # (before the seed checks reuse the seeding buffers)

        # the finish task's seeds: GPU (the lazy occurrence table) = the host path, on a sample
        L = _abi.lib()
        fo = seed.default_opts(True)
        sampler = correct.control.Sampler()
        for e in log:   # replay the samples to the finish task's
            rg, off = srs.sample_ranges(sampler.cov2seqchunker(cov, T.sr_coverage(e.task)))
        from proovread_amd.exact_shard import sr_range
        s0, s1 = sr_range(len(off) - 1, RANKS, 0)
        rg = correct.sample_subranges(rg, s0, s1)
        f_seq = np.ascontiguousarray(srs.gather(rg), np.uint8)
        f_off = np.ascontiguousarray(off[s0:s1 + 1] - off[s0], np.int64)
        assert len(f_off) - 1 == log[-1].n_sr
        rng = np.random.default_rng(sd + 1)
        pick = np.sort(rng.choice(len(f_off) - 1, 20_000, replace=False))
        p_off = np.zeros(len(pick) + 1, np.int64)
        p_off[1:] = np.cumsum(f_off[pick + 1] - f_off[pick])
        p_seq = np.concatenate([f_seq[f_off[i]:f_off[i + 1]] for i in pick])
        gpu, gst = seed._map_gpu(L, ctx, p_seq, p_off, fo, False)   # the finish index (the pre-finish reads)
        nt4 = correct.NT4[pre_finish["seq"]]
        hx = seed.SeedIndex(nt4, pre_finish["off"])
        host = hx.map(p_seq, p_off, fo, threads=16)
        hx.close()
        assert (gst == 0).all() and np.array_equal(gpu, host) and len(host) > 20_000
        rec["finish_seed_check"] = {"reads": int(len(pick)), "seeds": int(len(host))}

        # 6 spread long reads: finish consensus + chimera lines = the oracle chain (over the GPU
        # seeds of the finish shard, which equal the host path's on the sample above)
        ft, fst = seed._map_gpu(L, ctx, f_seq, f_off, fo, False)
        assert (fst == 0).all()
        on = np.isin(ft["lr"], sample_lrs)
        keep_sr = np.zeros(len(f_off) - 1, bool)
        keep_sr[ft["sr"][on]] = True
        ft = ft[keep_sr[ft["sr"]]]
        dd = synth.with_seeds(dataclasses_replace(d, lr_seq=nt4, lr_off=pre_finish["off"], sr_seq=f_seq,
                                                  sr_off=f_off), ft)
        o = ob.sw_opts("bwa-sr-finish")
        swt = (o.a, o.b, o.o_del, o.o_ins, o.e_del, o.e_ins, o.w, o.pen_clip5, o.pen_clip3, o.zdrop,
               o.min_score_per_base)
        capf = min(cov, T.sr_coverage("bwa-sr-finish")) * 0.75
        _, _, want, _ = cpu_chain.run_sample(dd, sample_lrs, task=swt, coverage=capf, use_ref_qual=False,
                                             detect_chimera=True, workers=16, full=True,
                                             bin_filter=(20, 20.0 * min(cov, T.sr_coverage("bwa-sr-finish"))),
                                             drop_ratio=0.75, ref_seq=pre_finish["seq"], ref_qual=pre_finish["qual"])
        for i, g, (rc, fq, trace, ch) in zip(sample_lrs, got, want):
            assert rc == 0 and g.status == 0, (i, rc, g.status)
            assert g.fastq == fq, i
            assert g.trace == trace, i
            assert "".join(x + "\n" for x in g.chim_lines()) == ch, i
        rec["oracle_reads"] = sample_lrs
        _log("configs2_loop", rec)
    finally:
        ctx.close()


def dataclasses_replace(d, **kw):
    import dataclasses
    return dataclasses.replace(d, **kw)
