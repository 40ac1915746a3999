"""BAM I/O and the samtools drop-in (proovread_amd/bamio.py, proovread_amd/samtools.py)
for the commands proovread / bam2cns run: view -bS / -H / region, sort, index, merge,
--version.  Checked by round trips (SAM -> BAM -> SAM field-identical), the coordinate
order samtools sort defines ((ref id, POS, reverse flag), input order on ties,
unmapped last), region reads through the BAI index against a full scan, merge against
sort, and readability by the bam2cns drop-in's own BAM parser."""
import io
import random
import re

import pytest

from proovread_amd import bam2cns, bamio, samtools

REFS = [("lr0", 5000), ("lr1", 120000), ("lr2", 300)]


def _records(n, seed=3):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        r = rng.randrange(len(REFS) + 1)
        if r == len(REFS):
            out.append(f"u{i}\t4\t*\t0\t0\t*\t*\t0\t0\tACGTN\t*")
            continue
        name, L = REFS[r]
        ln = rng.randint(20, 150)
        pos = rng.randint(1, max(1, L - ln))
        d = rng.randint(0, 3)
        ins = rng.randint(0, 3)
        s5 = rng.randint(0, 5)
        cig = (f"{s5}S" if s5 else "") + f"{ln - d - ins - s5}M{d}D{ins}I" if ln - d - ins - s5 > 0 else f"{ln}M"
        cig = cig.replace("0D", "").replace("0I", "")
        seq = "".join(rng.choice("ACGT") for _ in range(ln))
        qual = "".join(chr(33 + rng.randint(0, 40)) for _ in range(ln)) if rng.random() < 0.7 else "*"
        flag = rng.choice([0, 16, 256, 272])
        tags = [f"AS:i:{rng.randint(-5, 700)}", "XA:Z:lr1,+5,10M,0", f"XF:f:{rng.random():g}", "XC:A:q"]
        out.append(f"r{i}\t{flag}\t{name}\t{pos}\t{rng.choice([0, 60])}\t{cig}\t*\t0\t0\t{seq}\t{qual}\t" + "\t".join(tags))
    return out


HEADER = "@HD\tVN:1.5\tSO:unsorted\n" + "".join(f"@SQ\tSN:{n}\tLN:{l}\n" for n, l in REFS)


def _sam_file(tmp_path, recs):
    p = tmp_path / "in.sam"
    p.write_text(HEADER + "\n".join(recs) + "\n")
    return p


def _norm(line):
    f = line.split("\t")
    return f[:11] + sorted(f[11:])


def test_view_bS_round_trip(tmp_path):
    recs = _records(3000)
    sam = _sam_file(tmp_path, recs)
    assert samtools.main(["view", "-@", "4", "-bS", str(sam), "-o", str(tmp_path / "a.bam")]) == 0
    out = io.StringIO()
    assert samtools.view([str(tmp_path / "a.bam")], out=out) == 0
    got = out.getvalue().splitlines()
    assert [_norm(x) for x in got] == [_norm(x) for x in recs]
    out = io.StringIO()
    samtools.view(["-H", str(tmp_path / "a.bam")], out=out)
    assert out.getvalue() == HEADER


def _key(line):
    f = line.split("\t")
    if f[2] == "*":
        return (len(REFS), 0, 0)
    return ([n for n, _ in REFS].index(f[2]), int(f[3]), (int(f[1]) >> 4) & 1)


def test_sort_index_region(tmp_path):
    recs = _records(4000, seed=5)
    sam = _sam_file(tmp_path, recs)
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "u.bam")])
    assert samtools.main(["sort", "-m", "2G", "-@", "3", "-T", str(tmp_path / "tmp"), "-o", str(tmp_path / "s.bam"),
                          str(tmp_path / "u.bam")]) == 0
    out = io.StringIO()
    samtools.view([str(tmp_path / "s.bam")], out=out)
    got = out.getvalue().splitlines()
    want = [r for _, r in sorted(((_key(r), i), r) for i, r in enumerate(recs))]
    assert [_norm(x) for x in got] == [_norm(x) for x in want]
    assert samtools.main(["index", str(tmp_path / "s.bam")]) == 0
    assert (tmp_path / "s.bam.bai").exists()
    # region reads through the index == a scan
    for ref, beg, end in [("lr0", None, None), ("lr1", None, None), ("lr2", None, None), ("lr1", 30000, 31000),
                          ("lr1", 1, 17000), ("lr0", 4990, 5000)]:
        region = f"{ref}:" if beg is None else f"{ref}:{beg}-{end}"
        out = io.StringIO()
        samtools.view([str(tmp_path / "s.bam"), region], out=out)
        b0 = 0 if beg is None else beg - 1
        e0 = 1 << 29 if end is None else end
        scan = []
        for r in want:
            f = r.split("\t")
            if f[2] != ref:
                continue
            p = int(f[3]) - 1
            span = bamio.ref_span(bamio.cigar_ops(f[5])) or 1
            if p < e0 and p + span > b0:
                scan.append(r)
        assert [_norm(x) for x in out.getvalue().splitlines()] == [_norm(x) for x in scan], region


def test_merge_equals_sort(tmp_path):
    recs = _records(2000, seed=9)
    parts = [recs[:700], recs[700:]]
    for k, p in enumerate(parts):
        s = tmp_path / f"p{k}.sam"
        s.write_text(HEADER + "\n".join(p) + "\n")
        samtools.main(["view", "-bS", str(s), "-o", str(tmp_path / f"p{k}u.bam")])
        samtools.main(["sort", "-o", str(tmp_path / f"p{k}.bam"), str(tmp_path / f"p{k}u.bam")])
    assert samtools.main(["merge", str(tmp_path / "m.bam"), str(tmp_path / "p0.bam"), str(tmp_path / "p1.bam")]) == 0
    out = io.StringIO()
    samtools.view([str(tmp_path / "m.bam")], out=out)
    want = [r for _, r in sorted(((_key(r), i), r) for i, r in enumerate(recs))]
    assert [_norm(x) for x in out.getvalue().splitlines()] == [_norm(x) for x in want]


def test_bam2cns_reader_reads_dropin_bam(tmp_path):
    recs = [r for r in _records(500, seed=11) if "\t*\t0\t0\t" not in r.split("\t", 2)[2][:10]]
    sam = _sam_file(tmp_path, recs)
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "c.bam")])
    hdr, it = bam2cns.bam_records(str(tmp_path / "c.bam"))
    assert hdr == dict(REFS)
    got = list(it)
    mapped = [r for r in recs if r.split("\t")[2] != "*"]
    assert len(got) == len(mapped)
    for g, r in zip(got, mapped):
        f = r.split("\t")
        assert (g.rname, g.pos, g.seq) == (f[2], int(f[3]), f[9])
        assert g.score == float(f[11][5:])


def test_version_satisfies_proovread_check():
    v = re.search(r"([0-9\.]+)", samtools.VERSION).group(1)
    assert tuple(int(x) for x in v.split(".")) >= (1, 1)


def test_native_sam_to_bam_is_byte_identical(tmp_path):
    """libprgpu's pr_sam_encode + pr_bgzf_compress (threads over lines / blocks) write the same
    bytes as the pure-Python encoder (sam_to_record + BgzfWriter), across block boundaries and
    for every tag type."""
    import random
    from proovread_amd import bamio
    rng = random.Random(4)
    refs = [f"lr{i}" for i in range(30)] + ["dup", "dup"]
    header = "@HD\tVN:1.5\tSO:unsorted\n" + "".join(f"@SQ\tSN:{r}\tLN:{rng.randint(500, 20000)}\n" for r in refs)
    lines = []
    for k in range(6000):
        L = rng.choice([0, 1, 33, 150, 301])
        seq = "".join(rng.choice("ACGTacgtNRY=") for _ in range(L)) or "*"
        qual = "*" if rng.random() < 0.3 or seq == "*" else "".join(chr(rng.randint(35, 73)) for _ in range(L))
        cig = "*" if seq == "*" or rng.random() < 0.1 else (f"{L}M" if rng.random() < 0.5 else f"3S{max(L - 6, 0)}M1I2S")
        rname = rng.choice(refs + ["*", "unknown"])
        tags = [f"AS:i:{rng.choice([0, 5, -5, 127, 128, 255, 256, -129, 40000, 70000, -70000, 3000000000])}"]
        if rng.random() < 0.3:
            tags += ["XZ:Z:hello world", "XA:A:x", "XF:f:1.5", "XB:B:c,1,-2,3", "XS:B:S,1,65535", "XG:B:f,0.5,2",
                     "XH:H:1AE3"]
        lines.append("\t".join([f"q{k}", str(rng.choice([0, 16, 256, 272, 4])), rname, str(rng.randint(0, 19000)),
                                str(rng.randint(0, 60)), cig, rng.choice(["*", "=", "lr3"]), str(rng.randint(0, 500)),
                                str(rng.randint(-300, 300)), seq, qual] + tags))
    a, b = tmp_path / "py.bam", tmp_path / "nat.bam"
    bamio.write_bam_from_sam([header] + [l + "\n" for l in lines], str(a), native=False)
    bamio.write_bam_from_sam([header] + [l + "\n" for l in lines], str(b), native=True, threads=4)
    assert a.read_bytes() == b.read_bytes()
    assert len(a.read_bytes()) > 3 * 65280 // 4


@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (30000, 11)])
def test_native_sort_is_byte_identical(tmp_path, n, seed):
    """sort_bam in libprgpu (pr_bgzf_decompress + pr_bam_sort_records + pr_bgzf_compress)
    writes the same bytes as the pure-Python path; many equal keys (POS drawn from a narrow
    range), unmapped records, both strands, records spanning BGZF blocks."""
    recs = _records(n, seed=seed)
    rng = random.Random(seed)
    recs = [r if r.startswith("u") else "\t".join(r.split("\t")[:3] + [str(rng.randint(1, 40))] + r.split("\t")[4:])
            for r in recs]
    sam = _sam_file(tmp_path, recs)
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "u.bam")])
    bamio.sort_bam(str(tmp_path / "u.bam"), str(tmp_path / "n.bam"), native=True, threads=4)
    bamio.sort_bam(str(tmp_path / "u.bam"), str(tmp_path / "p.bam"), native=False)
    assert (tmp_path / "n.bam").read_bytes() == (tmp_path / "p.bam").read_bytes()


def test_native_inflate_rejects_corrupt_input():
    with pytest.raises(RuntimeError, match="BGZF"):
        bamio._native_inflate(b"\x1f\x8b\x08\x00not bgzf at all")


@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (50000, 12)])
def test_native_index_is_byte_identical(tmp_path, n, seed):
    """pr_bam_index writes the BAI the pure-Python index_bam writes (bins, merged chunks,
    pseudo-bin, linear index across BGZF block boundaries, unmapped count)."""
    recs = _records(n, seed=seed)
    sam = _sam_file(tmp_path, recs)
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "u.bam")])
    bamio.sort_bam(str(tmp_path / "u.bam"), str(tmp_path / "s.bam"))
    bamio.index_bam(str(tmp_path / "s.bam"), str(tmp_path / "n.bai"), native=True, threads=4)
    bamio.index_bam(str(tmp_path / "s.bam"), str(tmp_path / "p.bai"), native=False)
    assert (tmp_path / "n.bai").read_bytes() == (tmp_path / "p.bai").read_bytes()


def test_native_index_rejects_unsorted(tmp_path):
    sam = _sam_file(tmp_path, _records(2000, seed=4))
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "u.bam")])
    with pytest.raises(ValueError, match="coordinate-sorted"):
        bamio.index_bam(str(tmp_path / "u.bam"))


def test_native_index_placed_record_without_position(tmp_path):
    """A placed record with POS 0 (BAM pos -1: RNAME set, unmapped mate-style placement) is
    indexed at 0 as hts_idx_push does (beg clamped to 0, end >= beg + 1); native and Python
    indexes agree and stay readable."""
    recs = [f"p{i}\t4\tlr0\t0\t0\t*\t*\t0\t0\tACGTA\t*" for i in range(3)] + _records(300, seed=21)
    sam = _sam_file(tmp_path, recs)
    samtools.main(["view", "-bS", str(sam), "-o", str(tmp_path / "u.bam")])
    bamio.sort_bam(str(tmp_path / "u.bam"), str(tmp_path / "s.bam"))
    bamio.index_bam(str(tmp_path / "s.bam"), str(tmp_path / "n.bai"), native=True, threads=2)
    bamio.index_bam(str(tmp_path / "s.bam"), str(tmp_path / "p.bai"), native=False)
    assert (tmp_path / "n.bai").read_bytes() == (tmp_path / "p.bai").read_bytes()
    bins, lin = bamio.read_bai(str(tmp_path / "n.bai"))[0]
    assert lin and lin[0] > 0
