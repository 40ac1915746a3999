"""`SeqFilter`-compatible CLI for the calls proovread makes.

SeqFilter is an absent submodule (.gitmodules:1-3).  proovread calls it for

  * masking after every iteration (bin/proovread:1706, ccseq tasks :882):
        SeqFilter FQ --line-width 80 --quiet --out FA --phred-offset 33
                  --phred-mask <hcr-mask> --fasta --base-content N --tsv -
    stdout is one TSV line whose whitespace fields 1 and 6 are bpt and bpN
    (proovread:1711);
  * unmasked FASTA for the finish pass (:766-772, :842-848):
        SeqFilter --in FQ --out FA --fasta --quiet --phred-offset 33
  * final trimming (:936-942) and FASTA conversion (:950-955):
        SeqFilter --trim-win 12,5 --min-length 500 --substr CHIM --in FQ --out FQ
                  --phred-offset 33

Masking runs on the GPU (pr_mask_run, mask_kernels.hip); trim windows are
Fastq::Seq::qual_window in libprgpu.so (pr_trim_windows, host).  The glue is
restated without a reference to pin it (parity unpinned): per read,
--substr pieces (one piece keeps the id, several become id.1, id.2 ... as
Fastq::Seq::substr_seq names clones, Seq.pm:813-876, descriptions gain
SUBSTR:offset,length), then the --trim-win windows of every piece (same naming),
then --min-length, then --phred-mask.  --substr lines are `id start end` or
`id start` (to the read end), the layout ChimeraToSeqFilter writes
(ChimeraToSeqFilter.pl:183-191).
"""
from __future__ import annotations

import argparse
import gzip
import sys
from typing import Callable, Dict, List, Optional, Sequence, Tuple

Record = Tuple[str, str, bytes, Optional[bytes]]   # id, description, seq, qual (None: FASTA)


def read_records(path: str) -> List[Record]:
    """FASTA / FASTQ (optionally gzipped, '-' = stdin) -> records with id and description."""
    if path in ("-", "/dev/stdin", "/dev/fd/0"):
        fh = sys.stdin.buffer
    elif path.endswith(".gz"):
        fh = gzip.open(path, "rb")
    else:
        fh = open(path, "rb")
    out: List[Record] = []
    try:
        data = fh.read()
    finally:
        if fh is not sys.stdin.buffer:
            fh.close()
    lines = data.split(b"\n")
    i = 0
    n = len(lines)
    while i < n and not lines[i].strip():
        i += 1
    if i == n:
        return out
    if lines[i].startswith(b">"):
        head, buf = None, []
        for ln in lines[i:]:
            ln = ln.rstrip(b"\r")
            if ln.startswith(b">"):
                if head is not None:
                    out.append(_rec(head, b"".join(buf), None))
                head, buf = ln[1:], []
            elif ln:
                buf.append(ln.strip())
        if head is not None:
            out.append(_rec(head, b"".join(buf), None))
    elif lines[i].startswith(b"@"):
        while i < n:
            if not lines[i].strip():
                i += 1
                continue
            if i + 3 >= n or not lines[i].startswith(b"@"):
                raise ValueError(f"{path}: truncated or malformed FASTQ record at line {i + 1}")
            head = lines[i].rstrip(b"\r")[1:]
            seq = lines[i + 1].strip()
            qual = lines[i + 3].strip()
            if len(qual) != len(seq):
                raise ValueError(f"{path}: record {head[:40]!r}: quality length != sequence length")
            out.append(_rec(head, seq, qual))
            i += 4
    else:
        raise ValueError(f"{path}: neither FASTA nor FASTQ")
    return out


def _rec(head: bytes, seq: bytes, qual: Optional[bytes]) -> Record:
    h = head.decode("latin-1")
    parts = h.split(None, 1)
    rid = parts[0] if parts else ""
    desc = parts[1] if len(parts) > 1 else ""
    return rid, desc, seq, qual


def format_record(r: Record, fasta: bool, line_width: int) -> bytes:
    rid, desc, seq, qual = r
    head = rid + (" " + desc if desc else "")
    if fasta:
        out = [(">" + head).encode("latin-1")]
        if line_width and line_width > 0:
            out += [seq[k:k + line_width] for k in range(0, len(seq), line_width)]
        elif seq:
            out.append(seq)
        return b"\n".join(out) + b"\n"
    if qual is None:
        raise ValueError(f"{rid}: FASTQ output needs qualities")
    return b"@" + head.encode("latin-1") + b"\n" + seq + b"\n+\n" + qual + b"\n"


def parse_substr(lines: Sequence[str]) -> Dict[str, List[Tuple[int, Optional[int]]]]:
    d: Dict[str, List[Tuple[int, Optional[int]]]] = {}
    for ln in lines:
        f = ln.rstrip("\n").split("\t")
        if len(f) < 2 or not f[0]:
            continue
        d.setdefault(f[0], []).append((int(f[1]), int(f[2]) if len(f) > 2 and f[2] != "" else None))
    return d


def _pieces(L: int, ranges) -> List[Tuple[int, int]]:
    out = []
    for s, e in ranges:
        e = L if e is None else min(e, L)
        s = max(0, min(s, L))
        out.append((s, max(0, e - s)))
    return out


def _split(r: Record, ranges) -> List[Record]:
    rid, desc, seq, qual = r
    many = len(ranges) > 1
    res = []
    for k, (o, l) in enumerate(ranges, 1):
        tag = f"SUBSTR:{o},{l}"
        res.append((f"{rid}.{k}" if many else rid, f"{desc} {tag}" if desc else tag, seq[o:o + l],
                    qual[o:o + l] if qual is not None else None))
    return res


MaskRunner = Callable[[List[bytes], List[bytes], str], Tuple[List[bytes], List, Tuple[int, int]]]


def _gpu_mask(seqs: List[bytes], quals: List[bytes], spec: str, phred_offset: int):
    from . import mask
    return mask.run(seqs, quals, mask.params(spec, 100, phred_offset))


def parse_args(argv: List[str]):
    ap = argparse.ArgumentParser(prog="SeqFilter", add_help=True)
    ap.add_argument("input", nargs="?")
    ap.add_argument("--in", dest="inp")
    ap.add_argument("--out", default="-")
    ap.add_argument("--fasta", action="store_true")
    ap.add_argument("--line-width", type=int, default=80)
    ap.add_argument("--phred-offset", type=int, default=33)
    ap.add_argument("--phred-mask")
    ap.add_argument("--base-content", action="append", default=[])
    ap.add_argument("--tsv")
    ap.add_argument("--trim-win")
    ap.add_argument("--min-length", type=int, default=0)
    ap.add_argument("--substr")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--threads", type=int, default=0)
    return ap.parse_args(argv)


def run(argv: List[str], stdout=None, mask_runner=None) -> int:
    a = parse_args(argv)
    stdout = stdout or sys.stdout.buffer
    path = a.inp or a.input or "-"
    recs = read_records(path)
    if a.substr:
        with open(a.substr) as fh:
            sub = parse_substr(fh.read().splitlines())
        nr: List[Record] = []
        for r in recs:
            nr += _split(r, _pieces(len(r[2]), sub[r[0]])) if r[0] in sub else [r]
        recs = nr
    if a.trim_win:
        from . import trim
        if any(r[3] is None for r in recs):
            raise ValueError("--trim-win needs FASTQ input")
        p = trim.params(a.trim_win, a.phred_offset)
        wins = trim.windows([r[3] for r in recs], p, threads=a.threads)
        nr = []
        for r, w in zip(recs, wins):
            if w:
                nr += _split(r, w)
        recs = nr
    if a.min_length:
        recs = [r for r in recs if len(r[2]) >= a.min_length]
    if a.phred_mask:
        if any(r[3] is None for r in recs):
            raise ValueError("--phred-mask needs FASTQ input")
        seqs = [r[2] for r in recs]
        quals = [r[3] for r in recs]
        if mask_runner is not None:
            masked, _, _ = mask_runner(seqs, quals, a.phred_mask)
        else:
            masked, _, _ = _gpu_mask(seqs, quals, a.phred_mask, a.phred_offset)
        recs = [(r[0], r[1], m, r[3]) for r, m in zip(recs, masked)]
    fasta = a.fasta or any(r[3] is None for r in recs)
    blob = b"".join(format_record(r, fasta, a.line_width) for r in recs)
    if a.out == "-":
        stdout.write(blob)
    else:
        with open(a.out, "wb") as fh:
            fh.write(blob)
    if a.tsv:
        lens = [len(r[2]) for r in recs]
        cols = [path, str(sum(lens)), str(len(recs)), str(min(lens) if lens else 0), str(max(lens) if lens else 0)]
        for pat in a.base_content:
            chars = pat.encode()
            cols += [pat, str(sum(sum(r[2].count(bytes([c])) for c in set(chars)) for r in recs))]
        line = ("\t".join(cols) + "\n").encode()
        if a.tsv == "-":
            stdout.write(line)
        else:
            with open(a.tsv, "wb") as fh:
                fh.write(line)
    if hasattr(stdout, "flush"):
        stdout.flush()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    try:
        return run(argv)
    except SystemExit as e:
        return int(e.code or 0)
    except Exception as e:   # proovread checks $? (proovread:1714)
        print(f"[SeqFilter] error: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
