"""The bam2cns drop-in (proovread_amd/bam2cns.py): option handling, BAM/SAM
readers and natural read order on CPU; end-to-end output files against the
reference golden vectors (tests/golden/cns_expected.txt) on the GPU.

The end-to-end case mirrors how proovread calls bam2cns (bin/proovread:1596-1619):
a chunk FASTQ of long reads, a coordinate-sorted BAM, --ref-offset/--max-ref-seqs,
--coverage, --detect-chimera, --append; the .fq/.chim.tsv contents must equal
the per-read Perl outputs concatenated in `byfile` order (bam2cns:324).
"""
import functools
from pathlib import Path

import pytest

import bamio
import casefmt
from cns_case_util import case_inputs, params_key
from proovread_amd import bam2cns, cns

GOLD = Path(__file__).resolve().parent / "golden"
CASES = casefmt.read_cases(GOLD / "cns_cases.txt")
EXPECT = casefmt.read_expect(GOLD / "cns_expected.txt")


def test_byfile_natural_order():
    ids = ["r10", "r2", "r1", "a", "r1b", "r01", "10x", "9x", "r1_2", "r1_10"]
    got = sorted(ids, key=functools.cmp_to_key(bam2cns.byfile_cmp))
    assert got == ["9x", "10x", "a", "r1", "r01", "r1_2", "r1_10", "r1b", "r2", "r10"]


def _golden_group():
    """The largest group of golden cases sharing bam2cns parameters."""
    groups = {}
    for c in CASES:
        if EXPECT[c.name].error or c.p("noref") == "1" or c.p("qual_weighted") == "1":
            continue
        if c.ref_id == "hc_lr":
            continue  # handcrafted cases share one read id
        _, _, p = case_inputs(c)
        groups.setdefault(params_key(p), (p, []))[1].append(c)
    return max(groups.values(), key=lambda g: len(g[1]))


def _write_inputs(tmp_path, cases):
    fq = tmp_path / "lr.fq"
    fq.write_text("".join("\n".join(c.ref) + "\n" for c in cases))
    refs = [(c.ref_id, len(c.ref[1])) for c in cases]
    lines = [l for c in cases for l in c.sam]
    bamio.write_bam(str(tmp_path / "x.bam"), refs, lines)
    (tmp_path / "x.sam").write_text(
        "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in refs) + "".join(l + "\n" for l in lines))
    return fq


def test_bam_reader_matches_sam_text(tmp_path):
    p, cases = _golden_group()
    _write_inputs(tmp_path, cases[:6])
    hb, rb = bam2cns.bam_records(str(tmp_path / "x.bam"))
    hs, rs = bam2cns.sam_records(str(tmp_path / "x.sam"))
    assert hb == hs
    a, b = list(rb), list(rs)
    assert len(a) == len(b) == sum(len(c.sam) for c in cases[:6])
    for x, y in zip(a, b):
        assert (x.rname, x.pos, x.cigar, x.seq.upper(), x.qual, x.score) == \
               (y.rname, y.pos, y.cigar, y.seq.upper(), y.qual, y.score)


def test_reads_with_phred64_offset_rejected(tmp_path):
    fq = tmp_path / "lr.fq"
    fq.write_text("@r1\nACGT\n+\nhhhh\n")
    bamio.write_bam(str(tmp_path / "x.bam"), [("r1", 4)], [])
    with pytest.raises(SystemExit) as e:
        bam2cns.main(["--bam", str(tmp_path / "x.bam"), "--ref", str(fq), "--prefix", str(tmp_path / "o")])
    assert e.value.code == 255


@pytest.mark.parametrize("opt", [["--utg-mode"], ["--min-ncscore", "1"], ["--qual-weighted"],
                                 ["--haplo-coverage"], []])
def test_unsupported_modes_exit_255(tmp_path, opt):
    args = ["--prefix", str(tmp_path / "o")] + opt
    if opt:
        args += ["--bam", str(tmp_path / "none.bam")]
    with pytest.raises(SystemExit) as e:
        bam2cns.main(args)
    assert e.value.code == 255


def test_without_ref_processes_nothing(tmp_path):
    """bam2cns:313-320 never fills @LR_IDS from the header: empty outputs."""
    bamio.write_bam(str(tmp_path / "x.bam"), [("r1", 100)], [])
    assert bam2cns.main(["--bam", str(tmp_path / "x.bam"), "--prefix", str(tmp_path / "o")]) == 0
    for ext in (".fq", ".chim.tsv", ".ignored.tsv"):
        assert (tmp_path / ("o" + ext)).read_text() == ""


def _cli_args(p):
    a = ["--coverage", cns.perl_num(p.coverage), "--max-ins-length", str(p.max_ins_length)]
    a.append("--use-ref-qual" if p.use_ref_qual else "--no-use-ref-qual")
    if p.detect_chimera:
        a.append("--detect-chimera")
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["bam", "sam"])
def test_cli_matches_reference_golden(tmp_path, fmt):
    p, cases = _golden_group()
    if fmt == "bam":
        # BAM stores 4-bit bases: a lowercase base of the SAM text comes back uppercase,
        # which the consensus (like samtools view output for the reference) sees differently
        cases = [c for c in cases if not any(ch.islower() for l in c.sam for ch in l.split("\t")[9])]
    fq = _write_inputs(tmp_path, cases)
    pre = str(tmp_path / "out")
    # two chunks through --ref-offset/--max-ref-seqs and --append, as proovread fans them out
    half = len(cases) // 2
    off = sum(len("\n".join(c.ref)) + 1 for c in cases[:half])
    base = [f"--{fmt}", str(tmp_path / f"x.{fmt}"), "--ref", str(fq), "--prefix", pre, "--debug"] + _cli_args(p)
    assert bam2cns.main(base + ["--ref-offset", "0", "--max-ref-seqs", str(half)]) == 0
    assert bam2cns.main(base + ["--ref-offset", str(off), "--max-ref-seqs", "0", "--append"]) == 0
    order = lambda cs: sorted(cs, key=functools.cmp_to_key(lambda x, y: bam2cns.byfile_cmp(x.ref_id, y.ref_id)))
    want_fq, want_chim = [], []
    for chunk in (cases[:half], cases[half:]):
        for c in order(chunk):
            want_fq += EXPECT[c.name].fastq
            want_chim += EXPECT[c.name].chim
    assert Path(pre + ".fq").read_text().rstrip("\n").split("\n") == want_fq
    chim = Path(pre + ".chim.tsv").read_text()
    assert (chim.rstrip("\n").split("\n") if chim else []) == want_chim
    assert Path(pre + ".ignored.tsv").read_text() == ""
    trace = Path(pre + ".debug.trace").read_text().split("\n")
    assert trace[4] == EXPECT[order(cases[:half])[0].name].trace


def test_native_bam_columns_equal_python_reader(tmp_path):
    """bam2cns's native BAM path (pr_bgzf_decompress + pr_bam_decode_alns + pack_bam_chunk)
    hands pr_cns_run the same alignments, field for field, as the Python reader + pack_chunk
    (POS, AS, flags, SEQ, QUAL, CIGAR per read in file order), including a repeated read id."""
    import numpy as np
    from proovread_amd import cns
    p, cases = _golden_group()
    cases = [c for c in cases if not any(ch.islower() for l in c.sam for ch in l.split("\t")[9])]
    _write_inputs(tmp_path, cases)
    names, cols = bam2cns.bam_alns_native(str(tmp_path / "x.bam"))
    _, recs = bam2cns.bam_records(str(tmp_path / "x.bam"))
    recs = list(recs)
    ids = [c.ref_id for c in cases] + [cases[0].ref_id]
    lrs = [cns.LongRead(i, None, None, "", 100000) for i in ids]
    d = bam2cns.pack_bam_chunk(lrs, names, cols)
    want = cns.pack_chunk(lrs, [[r for r in recs if r.rname == i] for i in ids])

    def per_aln(d):
        out = []
        for k in range(int(d["aln_off"][-1])):
            so, ls = int(d["aln_seq_off"][k]), int(d["aln_lseq"][k])
            co, nc = int(d["aln_cig_off"][k]), int(d["aln_ncig"][k])
            out.append((int(d["aln_pos"][k]), float(d["aln_score"][k]), int(d["aln_flags"][k]),
                        d["seq_pool"][so:so + ls].tobytes(), d["qual_pool"][so:so + ls].tobytes(),
                        d["cig_pool"][co:co + nc].tolist()))
        return out
    assert np.array_equal(d["aln_off"], want["aln_off"]) and int(d["aln_off"][-1]) > 100
    assert per_aln(d) == per_aln(want)
