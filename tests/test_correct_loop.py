"""The in-process sr-noccs loop (proovread_amd.correct; bin/proovread:705-905).

CPU: read-long preprocessing (stubby reads, IUPAC -> N, byfile order), SeqChunker
sampling equal to the SeqChunker drop-in's output, and the whole loop driven by
the oracle stages (tests/loop_oracle.py): the reads get corrected, the masked
fraction grows, mask_shortcut_frac decides like proovread.
GPU: the loop on the device stages (pr_iter_* with the previous .fq as consensus
reference, pr_mask_run) equals the oracle loop byte-for-byte at every task:
corrected reads, qualities, chimera lines, masked fractions and the task list."""
import io

import numpy as np
import pytest

from proovread_amd import correct, seqchunker, synth

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _inputs(seed=5, gl=24000, n_lr=10, lr_len=2400, sr_cov=40.0, sr_len=150):
    d = synth.simulate(seed, gl, n_lr, lr_len, sr_cov, sr_frac=1.0, sr_len=sr_len)
    lrs = [(f"lr_{i}", ACGT[np.minimum(d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]], 3)].tobytes(), None)
           for i in range(d.n_lr)]
    sr = io.BytesIO()
    for i in range(d.n_sr):
        s = ACGT[np.minimum(d.sr_seq[d.sr_off[i]:d.sr_off[i + 1]], 3)].tobytes()
        sr.write(b"@sr%d\n%s\n+\n%s\n" % (i, s, b"I" * len(s)))
    return d, lrs, sr.getvalue()


def _kmers(g, k=20):
    s = ACGT[g].tobytes()
    rc = s[::-1].translate(bytes.maketrans(b"ACGT", b"TGCA"))
    return {t[i:i + k] for t in (s, rc) for i in range(len(t) - k + 1)}


def _exact(s, km, k=20):
    n = len(s) - k + 1
    return sum(s[i:i + k] in km for i in range(n)) / max(n, 1)


def test_read_long_preprocessing():
    recs = [("r10", b"acgtRYacgt" * 30, None), ("r9", b"ACGT" * 80, b"#" * 320), ("r1", b"ACGT" * 10, None)]
    reads, ign = correct.read_long(recs, 300)
    assert reads.ids == ["r9", "r10"]                  # byfile: 9 < 10; r1 is stubby
    assert ign == ["r1\tstubby"]
    assert reads.seqs[1] == b"ACGTNNACGT" * 30 and reads.quals[1] == b"$" * 300
    assert reads.quals[0] == b"#" * 320
    with pytest.raises(ValueError):
        correct.read_long([("a", b"A" * 10, None), ("a", b"C" * 10, None)], 1)


def test_short_read_sampling_matches_seqchunker():
    _, _, data = _inputs()
    srs = correct.ShortReads(data)
    sc = {"--chunk-number": 1000, "--chunk-step": 20, "--chunks-per-step": 6, "--first-chunk": 3}
    pool, off = srs.sample(sc)
    out = io.BytesIO()
    import tempfile
    with tempfile.NamedTemporaryFile(suffix=".fq") as f:
        f.write(data)
        f.flush()
        args = [x for k, v in sc.items() for x in (k, str(v))] + [f.name]
        assert seqchunker.main(args, stdout=out) == 0
    recs = out.getvalue().split(b"\n")[1::4]
    assert len(recs) == len(off) - 1 and 0 < len(recs) < len(srs.lengths)
    got = [ACGT[np.minimum(pool[off[i]:off[i + 1]], 3)].tobytes() for i in range(len(off) - 1)]
    assert got == recs


def test_loop_on_oracle_stages():
    import loop_oracle
    d, lrs, srd = _inputs()
    res = correct.run(lrs, srd, correct.LoopConfig(coverage=40.0, seed_threads=2), stages=loop_oracle.OracleStages(4))
    tasks = [e.task for e in res.log]
    assert tasks[0] == "read-long" and tasks[-1] == "bwa-sr-finish"
    fr = [e.masked_frac for e in res.log[1:-1]]
    assert fr[0] > 0.05 and fr == sorted(fr)
    if len(tasks) < 8:                                 # shortcut taken: by proovread's rule
        assert res.log[len(tasks) - 2].shortcut == "skip"
    km = _kmers(d.genome)
    raw = np.mean([_exact(s, km) for _, s, _ in lrs])
    cor = np.mean([_exact(s, km) for s in res.reads.seqs])
    assert raw < 0.3 and cor > 0.85, (raw, cor)
    assert all(len(s) == len(q) for s, q in zip(res.reads.seqs, res.reads.quals))
    for ln in res.chim:
        assert ln.split("\t")[0] in res.reads.ids


def test_mr_loop_on_oracle_stages():
    """300 bp short reads: proovread picks the mr-noccs mode (bin/proovread:636-642), its
    bwa-mr-1 / bwa-mr / bwa-mr-finish option sets (proovread.cfg:343-365) and bin size 50
    (-b 50 -l 50*min(cov, task cov)); the reads get corrected."""
    import loop_oracle
    d, lrs, srd = _inputs(seed=9, sr_len=300, sr_cov=40.0)
    res = correct.run(lrs, srd, correct.LoopConfig(coverage=40.0, seed_threads=2), stages=loop_oracle.OracleStages(4))
    tasks = [e.task for e in res.log]
    assert tasks[0] == "read-long" and tasks[1] == "bwa-mr-1" and tasks[-1] == "bwa-mr-finish"
    km = _kmers(d.genome)
    raw = np.mean([_exact(s, km) for _, s, _ in lrs])
    cor = np.mean([_exact(s, km) for s in res.reads.seqs])
    assert raw < 0.3 and cor > 0.85, (raw, cor)


def test_task_options_follow_proovread_cfg():
    from proovread_amd import seed, sw, tasks as T
    for t, fin in [("bwa-sr-1", False), ("bwa-sr-4", False), ("bwa-sr-finish", True)]:
        so, wo = T.options(t)
        ds, dw = seed.default_opts(fin), sw.default_opts(fin)
        assert all(getattr(so, n) == getattr(ds, n) for n, _ in so._fields_), t
        assert all(getattr(wo, n) == getattr(dw, n) for n, _ in wo._fields_), t
    so, wo = T.options("bwa-mr-3")          # cfg('bwa-mr-3') -> bwa-mr (proovread:1991-1994)
    assert (so.min_seed_len, so.drop_ratio, wo.min_score_per_base) == (13, 0.5, 3.0)
    so, wo = T.options("bwa-mr-finish")     # bwa defaults for -r / -D
    assert (so.min_seed_len, so.min_chain_weight, so.split_factor, so.drop_ratio, wo.b, wo.w) == (19, 40, 1.5, 0.5, 13, 30)
    assert T.hcr_mask("bwa-mr-5").endswith(",0.3") and T.hcr_mask("bwa-mr-2").endswith(",0.7")
    assert (T.sr_coverage("bwa-mr-2"), T.sr_coverage("bwa-mr-finish")) == (15.0, 30.0)
    assert (T.bin_size("sr-noccs"), T.bin_size("mr-noccs")) == (20, 50)
    assert T.mode_for(150) == "sr-noccs" and T.mode_for(151) == "mr-noccs"


@pytest.mark.gpu
def test_gpu_mr_loop_matches_oracle_loop():
    import loop_oracle
    _, lrs, srd = _inputs(seed=10, sr_len=300, sr_cov=40.0)
    cfg = correct.LoopConfig(coverage=40.0, seed_threads=4)
    want = correct.run(lrs, srd, cfg, stages=loop_oracle.OracleStages(8))
    got = correct.run(lrs, srd, cfg)
    assert [e.task for e in got.log] == [e.task for e in want.log] and got.log[1].task == "bwa-mr-1"
    for g, w in zip(got.log, want.log):
        assert (g.n_sr, g.n_tasks, g.bpt, g.bpn, g.shortcut) == (w.n_sr, w.n_tasks, w.bpt, w.bpn, w.shortcut), g.task
    assert got.reads.seqs == want.reads.seqs
    assert got.reads.quals == want.reads.quals
    assert got.chim == want.chim


@pytest.mark.gpu
def test_gpu_loop_matches_oracle_loop():
    import loop_oracle
    _, lrs, srd = _inputs(seed=6)
    cfg = correct.LoopConfig(coverage=40.0, seed_threads=4)
    want = correct.run(lrs, srd, cfg, stages=loop_oracle.OracleStages(8))
    got = correct.run(lrs, srd, cfg)
    assert [e.task for e in got.log] == [e.task for e in want.log]
    for g, w in zip(got.log, want.log):
        assert (g.n_sr, g.n_tasks, g.bpt, g.bpn, g.shortcut) == (w.n_sr, w.n_tasks, w.bpt, w.bpn, w.shortcut), g.task
    assert got.reads.seqs == want.reads.seqs
    assert got.reads.quals == want.reads.quals
    assert got.chim == want.chim


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["none", "rccl"])
def test_gpu_exact_layout_loop_matches_oracle_loop(transport, monkeypatch, tmp_path):
    """The multi-GPU exact-parity layout of the loop at world 1 (GpuStages.owned_iteration:
    device seeding of the shard, SW, pr_aln_exchange -- through RCCL's self send/recv with a
    communicator --, owned consensus and masking on the device) = the oracle loop."""
    import dataclasses
    import loop_oracle
    from proovread_amd import _abi, comm
    _, lrs, srd = _inputs(seed=6)
    cfg = correct.LoopConfig(coverage=40.0, seed_threads=4)
    want = correct.run(lrs, srd, cfg, stages=loop_oracle.OracleStages(8))
    cm = None
    if transport == "rccl":   # the full exchange through RCCL (world 1 would pass the SW output through)
        monkeypatch.setenv("PRGPU_XCHG_FORCE", "1")
        monkeypatch.setenv("PRGPU_RDZV_DIR", str(tmp_path))
        cm = comm.RcclComm(_abi.default_context(), 0, 1, key="loopx")
    try:
        got = correct.run(lrs, srd, dataclasses.replace(cfg, exact_layout=True), comm=cm)
    finally:
        if cm is not None:
            cm.close()
    for g, w in zip(got.log, want.log):
        assert (g.n_sr, g.n_tasks, g.bpt, g.bpn, g.shortcut) == (w.n_sr, w.n_tasks, w.bpt, w.bpn, w.shortcut), g.task
    assert got.reads.seqs == want.reads.seqs
    assert got.reads.quals == want.reads.quals
    assert got.chim == want.chim


# ---------------------------------------------------------------- configs[0]: the bundled sample
def _sample_inputs():
    from test_fantasticus_chain import FX, simulate_sr
    from proovread_amd import bwa_proovread as bp, sw
    names, seqs, quals = bp.read_fastx(str(FX / "F.antasticus_long_error.fq"))
    _, gs, _ = bp.read_fastx(str(FX / "F.antasticus_genome.fa"))
    G = sw.NT4[np.frombuffer(gs[0], np.uint8)]
    sr, off = simulate_sr(G, 50)
    buf = io.BytesIO()
    for i in range(len(off) - 1):
        s = ACGT[sr[off[i]:off[i + 1]]].tobytes()
        buf.write(b"@sr%d\n%s\n+\n%s\n" % (i, s, b"I" * len(s)))
    return G, list(zip(names, seqs, quals)), buf.getvalue()


def test_loop_on_sample_oracle_stages():
    """configs[0] through the whole sr-noccs loop on the oracle stages: every genomic
    read ends >= 95 % genome-exact (20-mers), the contamination read does not."""
    import loop_oracle
    G, lrs, srd = _sample_inputs()
    res = correct.run(lrs, srd, correct.LoopConfig(coverage=50.0, seed_threads=4), stages=loop_oracle.OracleStages(4))
    assert res.log[-1].task == "bwa-sr-finish" and len(res.reads.ids) == len(lrs)
    km = _kmers(G)
    for rid, s in zip(res.reads.ids, res.reads.seqs):
        f = _exact(s, km)
        if rid.startswith("long_contamination"):
            assert f < 0.5, rid
        else:
            assert f >= 0.95, (rid, f)


@pytest.mark.gpu
def test_gpu_loop_on_sample_matches_oracle_loop():
    import loop_oracle
    _, lrs, srd = _sample_inputs()
    cfg = correct.LoopConfig(coverage=50.0, seed_threads=4)
    want = correct.run(lrs, srd, cfg, stages=loop_oracle.OracleStages(8))
    got = correct.run(lrs, srd, cfg)
    assert [(e.task, e.n_tasks, e.bpn) for e in got.log] == [(e.task, e.n_tasks, e.bpn) for e in want.log]
    assert got.reads.fastq() == want.reads.fastq()
    assert got.chim == want.chim


# ---------------------------------------------------------------- multi-rank (exact layout)
def _loop_rank(rank, world, port, outdir):
    import json
    import os
    import torch.distributed as dist
    import loop_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _, lrs, srd = _inputs(seed=7)
    res = correct.run(lrs, srd, correct.LoopConfig(coverage=40.0, seed_threads=2),
                      stages=loop_oracle.OracleStages(1), comm=correct.Comm())
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump({"fastq": res.reads.fastq(), "chim": res.chim, "n_tasks": [e.n_tasks for e in res.log],
                   "log": [(e.task, e.n_sr, e.bpt, e.bpn, e.shortcut) for e in res.log]}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_loop_two_ranks_equals_single_process(tmp_path):
    """world_size-2 gloo run of the loop (short-read shards, task all-to-all to the long-read
    owners, all-gather of corrected and masked reads, all-reduce of bpt/bpN) gives exactly
    the single-process loop's reads, chimera lines and task decisions on both ranks."""
    import json
    import torch.multiprocessing as tmp
    import loop_oracle
    from test_exact_shard import _free_port
    world = 2
    tmp.spawn(_loop_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    _, lrs, srd = _inputs(seed=7)
    want = correct.run(lrs, srd, correct.LoopConfig(coverage=40.0, seed_threads=2), stages=loop_oracle.OracleStages(2))
    got = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(world)]
    for g in got:
        assert g["fastq"] == want.reads.fastq()
        assert g["chim"] == want.chim
        assert [tuple(x) for x in g["log"]] == [(e.task, e.n_sr, e.bpt, e.bpn, e.shortcut) for e in want.log]
    assert [a + b for a, b in zip(got[0]["n_tasks"], got[1]["n_tasks"])] == [e.n_tasks for e in want.log]
    assert min(got[0]["n_tasks"][1:]) > 0 and min(got[1]["n_tasks"][1:]) > 0


def test_loop_outputs_on_sample(tmp_path):
    """write_outputs: untrimmed = the loop's reads; trimmed reads are >= 500 bp pieces of them
    cut at the chimera breakpoints and quality windows (SeqFilter drop-in), FASTA mirrors FASTQ."""
    import loop_oracle
    from proovread_amd.seqfilter import read_records
    G, lrs, srd = _sample_inputs()
    res = correct.run(lrs, srd, correct.LoopConfig(coverage=50.0, seed_threads=4), stages=loop_oracle.OracleStages(4))
    pre = str(tmp_path / "out")
    correct.write_outputs(res, pre)
    un = read_records(pre + ".untrimmed.fq")
    assert [r[2] for r in un] == res.reads.seqs
    tr = read_records(pre + ".trimmed.fq")
    fa = read_records(pre + ".trimmed.fa")
    assert len(tr) >= 100 and [r[2] for r in tr] == [r[2] for r in fa]
    full = dict(zip(res.reads.ids, res.reads.seqs))
    for r in tr:
        rid = r[0].split()[0]
        base = rid.rsplit(".", 1)[0] if rid not in full else rid
        assert len(r[2]) >= 500 and r[2] in full[base], rid
    assert (tmp_path / "out.chim.tsv").exists() and (tmp_path / "out.ignored.tsv").read_text() == ""
