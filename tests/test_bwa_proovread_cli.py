"""`bwa-proovread` drop-in CLI (proovread_amd/bwa_proovread.py): option parsing as
proovread passes it (bin/proovread:1313 with proovread.cfg bwa-sr), FASTA/FASTQ
input, host seeding, SAM output.  The bwa-mode SW stage is injected here as the
CPU oracle (oracle/aln_oracle.c through oracle/cpu_chain.py) so the CLI logic is
checked without a GPU; on the GPU the same CLI calls pr_sw_run in bwa mode, whose
parity with the oracle is covered by test_aln_gpu.py."""
import io

import numpy as np

import oracle_bind as ob
from proovread_amd import bwa_proovread as bp
from proovread_amd import sw


class _OracleResult:
    """pr_sw_out of bwa mode from the CPU restatement (oracle/aln_oracle.c)."""

    def __init__(self, rows):
        n = len(rows)
        self.a = {k: np.zeros(max(n, 1), np.int32) for k in ("pos", "score", "status", "task", "flag")}
        self.a["pass"] = np.ones(max(n, 1), np.uint8)
        self.cig = []
        for i, x in enumerate(rows):
            self.a["pos"][i], self.a["score"][i], self.a["flag"][i], self.a["task"][i] = x[2], x[4], x[5], x[11]
            self.cig.append("".join(f"{c >> 4}{'MIDNSHP=X'[c & 15]}" for c in x[3]))
        self.n = n

    def __getitem__(self, k):
        return self.a[k][: self.n]

    def cigar_str(self, t):
        return self.cig[t]


def oracle_runner(task):
    import sys
    import types
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import cpu_chain

    def run(inp, opts):
        d = types.SimpleNamespace(sr_seq=inp.sr_seq, sr_off=inp.sr_off, lr_seq=inp.lr_seq, lr_off=inp.lr_off,
                                  t_sr=inp.t_sr, t_lr=inp.t_lr, t_strand=inp.t_strand, t_qbeg=inp.t_qbeg,
                                  t_rbeg=inp.t_rbeg, t_slen=inp.t_slen, t_chain=inp.t_chain,
                                  n_sr=len(inp.sr_off) - 1, n_lr=len(inp.lr_off) - 1)
        rows = [x for per in cpu_chain.bwa_alignments(d, task, drop_ratio=opts.drop_ratio) for x in per]
        return _OracleResult(rows)
    return run


def _write(tmp_path, rng):
    G = rng.integers(0, 4, 6000)
    lrs = []
    for i in range(5):
        s = int(rng.integers(0, 4000))
        g = G[s:s + 2000]
        out = []
        for c in g:
            u = rng.random()
            if u < 0.04:
                continue
            if u < 0.05:
                c = (c + 1) % 4
            out.append(int(c))
            if rng.random() < 0.08:
                out.append(int(rng.integers(0, 4)))
        lrs.append(out)
    with open(tmp_path / "lr.fa", "w") as fh:
        for i, x in enumerate(lrs):
            fh.write(f">lr{i} some description\n")
            s = "".join("ACGT"[c] for c in x)
            for k in range(0, len(s), 60):
                fh.write(s[k:k + 60] + "\n")
    srs = []
    with open(tmp_path / "sr.fq", "w") as fh:
        for i in range(60):
            s = int(rng.integers(0, 5850))
            r = "".join("ACGT"[c] for c in G[s:s + 150])
            if rng.random() < 0.5:
                r = r[::-1].translate(str.maketrans("ACGT", "TGCA"))
            q = "".join(chr(33 + int(x)) for x in rng.integers(30, 41, 150))
            fh.write(f"@sr{i}/1\n{r}\n+\n{q}\n")
            srs.append((r, q))
    return lrs, srs


ARGS = "-b 20 -l 225 -a -Y -A 5 -B 11 -O 2,1 -E 4,3 -T 2.5 -k 12 -W 20 -w 40 -r 1 -D 0 -y 20 -L 30,30 -t 2".split()


def test_cli_sam_output(tmp_path):
    lrs, srs = _write(tmp_path, np.random.default_rng(5))
    assert bp.index([str(tmp_path / "lr.fa"), str(tmp_path / "lr.fa")], log=io.StringIO()) == 0
    out = io.StringIO()
    rc = bp.mem(ARGS + [str(tmp_path / "lr.fa"), str(tmp_path / "sr.fq")], out=out, sw_runner=oracle_runner("bwa-sr"),
                log=io.StringIO())
    assert rc == 0
    lines = out.getvalue().splitlines()
    sq = [x for x in lines if x.startswith("@SQ")]
    assert sq == [f"@SQ\tSN:lr{i}\tLN:{len(x)}" for i, x in enumerate(lrs)]
    recs = [x.split("\t") for x in lines if not x.startswith("@")]
    assert len(recs) > 40
    prim = {}
    for f in recs:
        name, flag, rname, pos, mapq, cig = f[0], int(f[1]), f[2], int(f[3]), int(f[4]), f[5]
        r, q = srs[int(name[2:].split("/")[0])]
        # SEQ / QUAL printed for every hit, reverse complemented on the reverse strand
        if flag & 16:
            assert f[9] == r[::-1].translate(str.maketrans("ACGT", "TGCA")) and f[10] == q[::-1]
        else:
            assert f[9] == r and f[10] == q
        # the CIGAR consumes the whole read; the alignment lies on the long read
        import re
        ops = re.findall(r"(\d+)([MIDS])", cig)
        assert sum(int(n) for n, o in ops if o in "MIS") == 150
        ref_len = sum(int(n) for n, o in ops if o in "MD")
        assert 1 <= pos and pos - 1 + ref_len <= len(lrs[int(rname[2:])])
        assert f[11].startswith("AS:i:") and int(f[11][5:]) >= 2.5 * sum(int(n) for n, o in ops if o in "MI")
        if not flag & 0x900:   # the read's first record is its best (mem_mark_primary_se order)
            assert mapq == 60 and name not in prim
            prim[name] = int(f[11][5:])
        assert name in prim   # secondaries / supplementaries follow their read's first record
    for f in recs:
        assert int(f[11][5:]) <= prim[f[0]]


def test_cli_options_map_to_proovread_cfg():
    a = bp.parse_mem(ARGS + ["ref", "reads"])
    so, wo = bp.options(a)
    assert (so.min_seed_len, so.min_chain_weight, so.w, so.split_factor, so.drop_ratio, so.max_mem_intv) == \
        (12, 20, 40, 1.0, 0.0, 20)
    assert (wo.a, wo.b, wo.o_del, wo.o_ins, wo.e_del, wo.e_ins, wo.w, wo.pen_clip5, wo.pen_clip3) == \
        (5, 11, 2, 1, 4, 3, 40, 30, 30)
    assert abs(wo.min_score_per_base - 2.5) < 1e-12


def test_cli_rejects_unknown_option(capsys):
    assert bp.main(["mem", "--bogus", "ref", "reads"]) == 1


def test_bin_filter_reproduces_reference_binning():
    """-b/-l (row A4, semantics unpinned): the filter is restated as Sam::Seq's
    add_aln_by_score (Seq.pm:582-614).  On the consensus goldens (SAM records per
    long read, made by the reference Perl engine), BinFilter with -b 20 -l 20*coverage
    keeps exactly the alignments the reference keeps after binning."""
    import casefmt
    from pathlib import Path
    from proovread_amd.bwa_proovread import BinFilter, aln_length
    gold = Path(__file__).resolve().parent / "golden"
    cases = casefmt.read_cases(gold / "cns_cases.txt")
    exp = casefmt.read_expect(gold / "cns_expected.txt")
    n = 0
    for c in cases:
        e = exp[c.name]
        if e.error or not e.kept or c.p("noref") == "1":
            continue
        recs = [l.split("\t") for l in c.sam]
        if any(not any(x.startswith("AS:i:") for x in r[11:]) or r[9] == "*" for r in recs):
            continue
        f = BinFilter(20, 20 * float(c.p("coverage")))
        for r in recs:
            sc = float([x for x in r[11:] if x.startswith("AS:i:")][0][5:])
            f.add(0, int(r[3]), aln_length(r[5], len(r[9])), sc)
        assert "".join("1" if k else "0" for k in f.alive) == e.kept, c.name
        n += 1
    assert n > 10
