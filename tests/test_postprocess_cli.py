"""Drop-ins around the iteration: SeqFilter (masking with the
oracle injected in place of the GPU kernel, trimming through libprgpu's host
pr_trim_windows), ChimeraToSeqFilter, SeqChunker, and proovread's iteration control
(cov2seqchunker, mask_shortcut_frac).  CPU only."""
import io
import random
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import seqfilter_oracle as O  # noqa: E402

from proovread_amd import chimera_filter, control, seqchunker, seqfilter  # noqa: E402


def _oracle_mask(seqs, quals, spec):
    return O.mask_reads(seqs, quals, O.mask_params_from_cfg(spec, 100))


def _fastq(rng, n, L=(300, 3000)):
    recs = []
    for i in range(n):
        ln = rng.randint(*L)
        seq = bytes(rng.choice(b"ACGT") for _ in range(ln))
        ph, hi = [], rng.random() < 0.6
        while len(ph) < ln:
            k = rng.randint(1, rng.choice([30, 300, 900]))
            ph += [rng.randint(20, 40) if hi else rng.randint(0, 15) for _ in range(k)]
            hi = not hi
        recs.append((f"r{i}", f"len={ln}" if i % 2 else "", seq, bytes(33 + p for p in ph[:ln])))
    return recs


def _write_fq(path, recs):
    path.write_bytes(b"".join(seqfilter.format_record(r, False, 0) for r in recs))


# ---------------------------------------------------------------- SeqFilter

def test_seqfilter_phred_mask_call_of_proovread(tmp_path):
    """proovread:1706: masked FASTA out, TSV on stdout with bpt and bpN at fields 1 and 6."""
    rng = random.Random(3)
    recs = _fastq(rng, 40)
    fq = tmp_path / "it.fq"
    _write_fq(fq, recs)
    spec = "20,41,120,195,60,0.7"   # cfg hcr-mask scaled to 150 bp by proovread
    out = io.BytesIO()
    rc = seqfilter.run([str(fq), "--line-width", "80", "--quiet", "--out", str(tmp_path / "it.masked.fa"),
                        "--phred-offset", "33", "--phred-mask", spec, "--fasta", "--base-content", "N", "--tsv", "-"],
                       stdout=out, mask_runner=_oracle_mask)
    assert rc == 0
    f = out.getvalue().decode().split()
    masked, _, (bpt, bpn) = _oracle_mask([r[2] for r in recs], [r[3] for r in recs], spec)
    assert (int(f[1]), int(f[6])) == (bpt, bpn) and bpn > 0
    fa = seqfilter.read_records(str(tmp_path / "it.masked.fa"))
    assert [r[2] for r in fa] == masked
    assert [r[0] for r in fa] == [r[0] for r in recs]
    lines = (tmp_path / "it.masked.fa").read_bytes().split(b"\n")
    assert max(len(x) for x in lines) == 80


def test_seqfilter_unmasked_fasta(tmp_path):
    rng = random.Random(4)
    recs = _fastq(rng, 5, (0, 200))
    fq = tmp_path / "a.fq"
    _write_fq(fq, recs)
    assert seqfilter.run(["--in", str(fq), "--out", str(tmp_path / "a.fa"), "--fasta", "--quiet",
                          "--phred-offset", "33"]) == 0
    fa = seqfilter.read_records(str(tmp_path / "a.fa"))
    assert [(r[0], r[1], r[2]) for r in fa] == [(r[0], r[1], r[2]) for r in recs]


def test_seqfilter_final_trim(tmp_path):
    """proovread:936-942: --trim-win 12,5 --min-length 500 --substr CHIM on the untrimmed reads."""
    rng = random.Random(5)
    recs = _fastq(rng, 30, (500, 6000))
    fq = tmp_path / "x.untrimmed.fq"
    _write_fq(fq, recs)
    chim = tmp_path / "x.chim.tsv"
    chim.write_text("r1\t0\t700\nr1\t800\t1600\nr1\t1700\nr4\t0\t100000\n")
    assert seqfilter.run(["--trim-win", "12,5", "--min-length", "500", "--substr", str(chim), "--in", str(fq),
                          "--out", str(tmp_path / "x.trimmed.fq"), "--phred-offset", "33"]) == 0
    got = seqfilter.read_records(str(tmp_path / "x.trimmed.fq"))
    want = []
    P = O.WinParams.trim_win("12,5")
    sub = {"r1": [(0, 700), (800, 800), (1700, None)], "r4": [(0, None)]}
    for rid, desc, s, q in recs:
        pieces = [(rid, desc, s, q)]
        if rid in sub:
            rs = [(a, (len(s) if b is None else min(len(s), a + b)) - a) for a, b in sub[rid]]
            pieces = seqfilter._split((rid, desc, s, q), rs)
        for pr in pieces:
            w = O.qual_window([c - 33 for c in pr[3]], P)
            want += [x for x in (seqfilter._split(pr, w) if w else []) if len(x[2]) >= 500]
    assert [(r[0], r[1], r[2], r[3]) for r in got] == want
    assert any(r[0].startswith("r1.") for r in got) and len(got) > 5


def test_seqfilter_errors(tmp_path):
    fa = tmp_path / "a.fa"
    fa.write_text(">a\nACGT\n")
    assert seqfilter.main(["--in", str(fa), "--phred-mask", "20,41,80,130,60,0.7", "--out", "-"]) == 1
    bad = tmp_path / "b.fq"
    bad.write_text("@a\nACGT\n+\nII\n")
    assert seqfilter.main(["--in", str(bad), "--out", str(tmp_path / "o")]) == 1


# ---------------------------------------------------------------- ChimeraToSeqFilter

def test_chimera_filter_known_answers():
    lines = ["id\tfrom\tto\tscore",
             "a\t100\t140\t0.9",      # first line of a: opens the read, never added
             "a\t500\t540\t0.5",
             "a\t900\t930\t0.005",    # below --min-score 0.01
             "a\t1200\t1260\t0.2",
             "b\t10\t20\t1",
             "c\t300\t340\t0.7",
             "c\t800\t820\t0.7",
             "d\t5\t6\t1",
             "d\t7\t8\t1"]            # d is the last read: never printed
    assert chimera_filter.convert(lines) == ["a\t0\t500", "a\t540\t1200", "a\t1260", "c\t0\t800", "c\t820"]
    assert chimera_filter.convert(lines, 0.6) == ["c\t0\t800", "c\t820"]
    assert chimera_filter.convert(["a\t1\t2\t1", "a\t3\t4\t1"]) == []   # header swallowed
    assert chimera_filter.convert([]) == []


def test_chimera_filter_cli(tmp_path):
    p = tmp_path / "c.tsv"
    p.write_text("id\tfrom\tto\tscore\nx\t1\t2\t1\nx\t10\t20\t0.3\ny\t5\t5\t1\n")
    out = tmp_path / "o.tsv"
    assert chimera_filter.main(["--in", str(p), "--out", str(out), "--min-score", "0.2", "--trim-length", "20",
                                "--verbose", "2"]) == 0
    assert out.read_text() == "x\t0\t10\nx\t20\n"


# ---------------------------------------------------------------- SeqChunker

def test_seqchunker_partition_and_sampling(tmp_path):
    rng = random.Random(6)
    recs = _fastq(rng, 400, (50, 200))
    recs[7] = ("r7", "", recs[7][2], b"@" * len(recs[7][2]))   # '@' quality line
    fq = tmp_path / "sr.fq"
    _write_fq(fq, recs)
    data = fq.read_bytes()
    n, chunks = seqchunker.chunk(data, 40)
    assert n == 40
    assert b"".join(data[s:e] for c in chunks for s, e in c) == data
    sel = seqchunker.select(40, 3, 10, 2)
    assert sel == [3, 4, 13, 14, 23, 24, 33, 34]
    out = io.BytesIO()
    assert seqchunker.main(["--chunk-number", "40", "--chunk-step", "10", "--chunks-per-step", "2",
                            "--first-chunk", "3", str(fq)], stdout=out) == 0
    got = seqfilter.read_records(_tmp(tmp_path, out.getvalue()))
    assert 0.1 < len(got) / len(recs) < 0.3
    ids = {r[0] for r in recs}
    assert all(r[0] in ids for r in got)


def _tmp(tmp_path, blob):
    p = tmp_path / "sel.fq"
    p.write_bytes(blob)
    return str(p)


def test_cov2seqchunker_rotation():
    s = control.Sampler()
    assert s.cov2seqchunker(50, 45) is None          # more than 80 % of the data
    got = [s.cov2seqchunker(50, 15) for _ in range(5)]
    assert [g["--chunks-per-step"] for g in got] == [6] * 5
    assert [g["--first-chunk"] for g in got] == [1, 7, 13, 19, 5]
    assert control.Sampler(sampling=False).cov2seqchunker(50, 15) is None


def test_mask_shortcut():
    tasks = ["read-long", "bwa-sr-1", "bwa-sr-2", "bwa-sr-3", "bwa-sr-finish"]
    fr = []
    assert control.mask_shortcut(tasks, 1, 0.60, fr) == "continue"
    assert control.mask_shortcut(tasks, 2, 0.61, fr) == "skip"          # gain < 3 %
    assert tasks == ["read-long", "bwa-sr-1", "bwa-sr-2", "bwa-sr-finish"]
    tasks = ["read-long", "bwa-sr-1", "bwa-sr-2", "bwa-sr-3", "bwa-sr-finish"]
    assert control.mask_shortcut(tasks, 1, 0.95, []) == "skip"          # > 92 % masked
    assert tasks == ["read-long", "bwa-sr-1", "bwa-sr-finish"]
    assert control.mask_shortcut(["a", "b", "c"], 1, 0.99, []) == ""    # second to last task
    assert control.masked_fraction(200, 50) == 0.25
