"""`samtools`-compatible CLI for the commands proovread and bam2cns issue
(SURVEY.md §8f.3), on proovread_amd.bamio:

    samtools --version                                  (check_binary, bin/proovread:666)
    samtools view [-@ N] -bS FILE|/dev/fd/0 > out.bam   (bin/proovread:1313, 1015)
    samtools view -b - > out.bam                        (bin/bam2cns:289)
    samtools view -H in.bam                             (bin/bam2cns:224, 290)
    samtools view [-h] in.bam ["REF:"|"REF:BEG-END"]    (bin/bam2cns:336)
    samtools sort [-m M] [-@ N] [-T PFX] -o out.bam in.bam   (bin/proovread:1338)
    samtools index in.bam                               (bin/proovread:1348)
    samtools merge out.bam in1.bam ...                  (bin/proovread:1692)
"""
from __future__ import annotations

import argparse
import re
import sys
from typing import List, Optional

from . import bamio

VERSION = "samtools 1.10 (prgpu drop-in: proovread_amd.samtools)"


def _open_text(path: str):
    if path in ("-", "/dev/fd/0", "/dev/stdin"):
        return sys.stdin
    return open(path, "r", encoding="latin-1")


def view(argv: List[str], out=None) -> int:
    out = out or sys.stdout
    ap = argparse.ArgumentParser(prog="samtools view", add_help=False)
    ap.add_argument("-b", action="store_true")
    ap.add_argument("-S", action="store_true")
    ap.add_argument("-h", action="store_true")
    ap.add_argument("-H", action="store_true")
    ap.add_argument("-@", dest="threads", type=int, default=0)
    ap.add_argument("-o", dest="out", default=None)
    ap.add_argument("input")
    ap.add_argument("region", nargs="?")
    a = ap.parse_args(argv)
    is_bam = False
    if a.input not in ("-", "/dev/fd/0", "/dev/stdin"):
        with open(a.input, "rb") as fh:
            is_bam = fh.read(2) == b"\x1f\x8b"
    if a.b:   # SAM (or BAM) -> BAM
        target = a.out or sys.stdout.buffer
        if is_bam:
            rd = bamio.BamReader(a.input)
            w = bamio.BamWriter(target, rd.header)
            for _, r, _ in rd.records():
                w.write_record(len(r).to_bytes(4, "little", signed=True) + r)
            w.close()
            rd.close()
        else:
            fh = _open_text(a.input)
            bamio.write_bam_from_sam(fh, target)
            if fh is not sys.stdin:
                fh.close()
        return 0
    if not is_bam:
        raise ValueError("view: text output needs a BAM input")
    rd = bamio.BamReader(a.input)
    if a.H or a.h:
        out.write(rd.header.text if rd.header.text.endswith("\n") or not rd.header.text else rd.header.text + "\n")
    if a.H:
        rd.close()
        return 0
    if a.region:
        m = re.match(r"^(.*?):(?:(\d+)(?:-(\d+))?)?$", a.region)
        ref, beg, end = (m.group(1), m.group(2), m.group(3)) if m else (a.region, None, None)
        b0 = int(beg) - 1 if beg else 0
        e0 = int(end) if end else 1 << 29
        names = rd.names
        rd.close()
        for r in bamio.region_records(a.input, ref, b0, e0):
            out.write(bamio.record_to_sam(r, names) + "\n")
        return 0
    for _, r, _ in rd.records():
        out.write(bamio.record_to_sam(r, rd.names) + "\n")
    rd.close()
    return 0


def sort(argv: List[str]) -> int:
    ap = argparse.ArgumentParser(prog="samtools sort", add_help=False)
    ap.add_argument("-m", default=None)
    ap.add_argument("-@", dest="threads", type=int, default=0)
    ap.add_argument("-T", dest="tmp", default=None)
    ap.add_argument("-o", dest="out", required=True)
    ap.add_argument("input")
    a = ap.parse_args(argv)
    bamio.sort_bam(a.input, a.out)
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if not argv:
        print("usage: samtools <view|sort|index|merge|--version> ...", file=sys.stderr)
        return 1
    cmd, rest = argv[0], argv[1:]
    try:
        if cmd == "--version":
            print(VERSION)
            return 0
        if cmd == "view":
            return view(rest)
        if cmd == "sort":
            return sort(rest)
        if cmd == "index":
            bamio.index_bam(rest[0], rest[1] if len(rest) > 1 else None)
            return 0
        if cmd == "merge":
            args = [x for x in rest if not x.startswith("-")]
            bamio.merge_bams(args[0], args[1:])
            return 0
        print(f"samtools: unsupported command {cmd}", file=sys.stderr)
        return 1
    except SystemExit as e:
        return 1 if e.code else 0
    except Exception as e:
        print(f"samtools {cmd}: {e}", file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
