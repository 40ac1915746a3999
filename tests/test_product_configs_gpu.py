"""BASELINE.json's single-GPU configs through the path the product ships, against the oracle
chain, read by read.

The product path (what bench.py and correct.py run): the long-read index built in HBM
(pr_seed_gpu_index_build), GPU seeding that leaves the seeds in HBM
(pr_seed_gpu_map(keep_on_device)), one iteration on them (pr_iter_upload_gpu_seeds ->
pr_iter_launch: bwa mode over every seed of the kept chains, bwa-proovread's -b/-l bin
filter on the device, hand-off, consensus) and the masking of the corrected reads with the
{bpt, bpN} statistic (pr_iter_mask).

The oracle chain: the host seeding path (seed_core.h compiled for the host; it equals the
pure-Python oracle/seed_oracle.py on tests/test_seed.py's cases -- the Python oracle is too
slow for these sizes), then oracle/aln_oracle.c + sw_oracle.c per short read (bwa mode),
SAM records -> -b/-l -> coordinate order -> oracle/cns_oracle.c (pinned to the reference
Perl engine), then oracle/seqfilter_oracle.py's masking of the oracle's corrected reads.

configs[4]: 25 kb reads at 20 % error (5 % ins, 8 % del, 7 % sub), band
override -w 100, `--coverage 100` with sr-coverage 50: cap 0.75 * 50 = 37.5
(bin/proovread:1540-1541), -b 20 -l 20 * 50 (bin/proovread:1302-1313); bwa-sr-1 and
bwa-sr-finish (-D .75, chimera detection, no reference qualities).
configs[1] (C2) scaled to a tenth: the bench's own workload generator, options and path.
"""
import dataclasses
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_bind as ob

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))

pytestmark = pytest.mark.gpu


def _product_iteration(ctx, d, finish, w, cap, binf, use_ref_qual, detect_chimera, hcr_mask, min_sr_len):
    """-> (Iteration after launch + mask, GPU seeds downloaded, masked reads, (bpt, bpN))."""
    from proovread_amd import _abi, cns, iteration, mask, seed, sw, synth
    ix = seed.DeviceSeedIndex(ctx, d.lr_seq, d.lr_off)
    so = seed.default_opts(finish)
    so.w = w   # bwa's -w also bounds the chaining gap (cal_max_gap)
    tasks, st = ix.map(d.sr_seq, d.sr_off, so)            # a host copy, for the oracle's seed check
    assert (st == 0).all()
    ix.map(d.sr_seq, d.sr_off, so, keep_on_device=True)   # what the iteration consumes
    it = iteration.Iteration(synth.with_seeds(d, tasks), ctx=ctx, gpu_seeds=True)
    o = sw.default_opts(finish=finish)
    o.w = w
    o.bin_size, o.bin_length = binf
    it.launch(o, cns.CnsParams(coverage=cap, use_ref_qual=use_ref_qual, detect_chimera=detect_chimera))
    stats = _abi.DevBuffer(ctx, 16)
    it.mask_to(stats.ptr, mask.params(hcr_mask, min_sr_len))
    it.sync()
    return it, tasks, it.masked(), tuple(int(x) for x in stats.download(np.int64))


def _oracle_chain(d, finish, w, cap, binf, use_ref_qual, detect_chimera):
    import cpu_chain
    from proovread_amd import seed, synth
    hx = seed.SeedIndex(d.lr_seq, d.lr_off)
    sop = seed.default_opts(finish)
    sop.w = w
    want_tasks = hx.map(d.sr_seq, d.sr_off, sop, threads=8)
    hx.close()
    so = ob.sw_opts("bwa-sr-finish" if finish else "bwa-sr")
    so.w = w
    swt = (so.a, so.b, so.o_del, so.o_ins, so.e_del, so.e_ins, so.w, so.pen_clip5, so.pen_clip3, so.zdrop,
           so.min_score_per_base)
    _, _, want, _ = cpu_chain.run_sample(synth.with_seeds(d, want_tasks), range(d.n_lr), task=swt, coverage=cap,
                                         use_ref_qual=use_ref_qual, detect_chimera=detect_chimera, workers=16,
                                         full=True, bin_filter=binf, drop_ratio=0.75 if finish else 0.0)
    return want_tasks, want


def _check(d, finish, w, cap, binf, hcr_mask, min_sr_len):
    import seqfilter_oracle as SO
    from proovread_amd import _abi
    urq, chim = not finish, finish
    ctx = _abi.default_context()
    it, tasks, masked, (bpt, bpn) = _product_iteration(ctx, d, finish, w, cap, binf, urq, chim, hcr_mask, min_sr_len)
    want_tasks, want = _oracle_chain(d, finish, w, cap, binf, urq, chim)
    assert np.array_equal(tasks, want_tasks), "GPU seeding != host seeding path"
    got = it.results()
    assert len(got) == len(want) == d.n_lr
    seqs, quals = [], []
    n_chim = 0
    for i, (g, (rc, fq, trace, ch)) in enumerate(zip(got, want)):
        assert rc == 0 and g.status == 0, (i, rc, g.status)
        assert g.fastq == fq, i
        assert g.trace == trace, i
        assert "".join(l + "\n" for l in g.chim_lines()) == ch, i
        n_chim += len(g.chim)
        lines = fq.split("\n")
        seqs.append(lines[1].encode())
        quals.append(lines[3].encode())
    # SeqFilter --phred-mask of the corrected reads: masked bases and (bpt, bpN)
    P = SO.mask_params_from_cfg(hcr_mask, min_sr_len)
    wmasked, _, wst = SO.mask_reads(seqs, quals, P)
    assert masked == wmasked
    assert (bpt, bpn) == tuple(wst)
    n_aln = it.alignment_stats()[0]
    assert n_aln > 20 * d.n_lr
    return n_aln, n_chim, bpn / max(bpt, 1)


@pytest.mark.parametrize("finish", [False, True])
def test_configs4_product_path_matches_oracle_chain(finish):
    """configs[4]: 40 x 25 kb at 20 % error over a 200 kb genome (5x long reads), 50x short
    reads (so the 37.5x cap and the -l 1000 filter both bite), w = 100.  The finish task runs
    on reads the iterations have corrected (its -T 4 per base keeps next to nothing of a 20 %
    error read): there the long reads carry a tenth of the error."""
    from proovread_amd import synth
    f = 0.1 if finish else 1.0
    d = synth.simulate(20261015 + 4 + finish, 200_000, 40, 25_000, 50.0, p_ins=0.05 * f, p_del=0.08 * f,
                       p_sub=0.07 * f, sr_frac=1.0)
    cap = min(100.0, 50.0) * 0.75
    n_aln, _, frac = _check(d, finish, 100, cap, (20, 20.0 * 50.0), "20,41,80,130,60,0.7", 150)
    assert 0.0 <= frac <= 1.0


def test_configs1_scaled_shard_bench_path_matches_oracle_chain():
    """configs[1] at scale 0.1 through exactly bench.py's generator and options: 1,380 x 10 kb
    CLR reads (15 % error), 50x short reads sampled to 15x, bwa-sr-1 with -b 20 -l 300, cap
    11.25 with the reads' own qualities, hcr-mask 20,41,80,130,60,0.7."""
    import bench
    from proovread_amd import synth
    d = synth.simulate(20261015 + 2, int(4_600_000 * 0.1), int(13_800 * 0.1), 10_000, 50.0, sr_frac=0.3)
    n_aln, _, frac = _check(d, False, 40, 15.0 * 0.75, bench.BIN_FILTER, "20,41,80,130,60,0.7", 150)
    assert n_aln > 100_000
    assert 0.0 < frac < 1.0


def test_configs4_finish_on_iterated_full_error_reads():
    """configs[4] at full error through two tasks: a 1 Mb genome, 1,200 x 25 kb long reads at
    20 % error (30x long-read coverage), 50x short reads, w = 100.  bwa-sr-1 (cap 37.5, -l
    1000, the reads' own qualities) corrects every read on the device; bwa-sr-finish then maps
    to those corrected reads (-D .75, chimera detection, no reference qualities, cap
    0.75 * 30 = 22.5, -l 600): at 30x every 12-mer of a near-exact read hits ~30 copies, so
    seeding runs its later passes.  GPU seeding = host seeding over every read of both tasks;
    the consensus (sequence, quality, trace, chimera lines) = the oracle chain on a spread
    sample of long reads (the oracle chain is exact for the long reads it is asked about)."""
    import cpu_chain
    from proovread_amd import _abi, seed, synth
    NT4 = np.full(256, 4, np.uint8)
    for i, c in enumerate(b"ACGT"):
        NT4[c] = NT4[c + 32] = i
    d = synth.simulate(20261015 + 44, 1_000_000, 1_200, 25_000, 50.0, p_ins=0.05, p_del=0.08, p_sub=0.07,
                       sr_frac=1.0)
    ctx = _abi.default_context()
    sample = list(range(0, d.n_lr, d.n_lr // 6))[:6]

    def oracle(dd, finish, cap, binf):
        hx = seed.SeedIndex(dd.lr_seq, dd.lr_off)
        sop = seed.default_opts(finish)
        sop.w = 100
        want_tasks = hx.map(dd.sr_seq, dd.sr_off, sop, threads=16)
        hx.close()
        so = ob.sw_opts("bwa-sr-finish" if finish else "bwa-sr")
        so.w = 100
        swt = (so.a, so.b, so.o_del, so.o_ins, so.e_del, so.e_ins, so.w, so.pen_clip5, so.pen_clip3, so.zdrop,
               so.min_score_per_base)
        _, _, want, _ = cpu_chain.run_sample(synth.with_seeds(dd, want_tasks), sample, task=swt, coverage=cap,
                                             use_ref_qual=not finish, detect_chimera=finish, workers=16, full=True,
                                             bin_filter=binf, drop_ratio=0.75 if finish else 0.0)
        return want_tasks, want

    def check(dd, finish, cap, binf):
        it, tasks, _, _ = _product_iteration(ctx, dd, finish, 100, cap, binf, not finish, finish,
                                             "20,41,80,130,60,0.7", 150)
        want_tasks, want = oracle(dd, finish, cap, binf)
        assert np.array_equal(tasks, want_tasks), "GPU seeding != host seeding path"
        got = it.results()
        assert all(g.status == 0 for g in got)
        for k, i in enumerate(sample):
            rc, fq, trace, ch = want[k]
            assert rc == 0, i
            assert got[i].fastq == fq, i
            assert got[i].trace == trace, i
            assert "".join(l + "\n" for l in got[i].chim_lines()) == ch, i
        return got, len(tasks)

    got1, n1 = check(d, False, 37.5, (20, 1000.0))
    seqs = [np.frombuffer(g.seq.encode("latin-1"), np.uint8) for g in got1]
    off = np.zeros(d.n_lr + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    d2 = dataclasses.replace(d, lr_seq=NT4[np.concatenate(seqs)], lr_off=off)
    got2, n2 = check(d2, True, 22.5, (20, 600.0))
    # the finish task sees corrected reads: the per-read seed load grows with the near-exact matches
    assert n2 > 0 and n1 > 0
