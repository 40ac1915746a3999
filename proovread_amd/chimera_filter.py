"""`ChimeraToSeqFilter.pl` drop-in: bam2cns chimera annotations ->
SeqFilter --substr coordinates, run once per job (bin/proovread:913-916, 1808-1822;
options proovread.cfg:145-149).

Restates bin/ChimeraToSeqFilter.pl:171-201 including its behaviour on real input:
  * the first line of the file is a header and is skipped (:176);
  * the first line of every read only opens the read; its breakpoint is never
    added (:182-194) — only later lines of the same id with score >= --min-score
    are (:196-198);
  * a read's pieces are printed when the next id starts: `id 0 from1`,
    `id to1 from2`, ..., `id toN` (:183-191); the last read of the file is never
    printed (there is no flush after the loop);
  * --trim-length is accepted and unused.
Coordinates are copied as text.  The script was not run here: the
known-answer tests follow this reading of the source.
"""
from __future__ import annotations

import argparse
import re
import sys
from typing import List, Optional, Sequence


def _perl_num(s: str) -> float:
    m = re.match(r"\s*([+-]?(?:\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?))", s or "")
    return float(m.group(1)) if m else 0.0


def convert(lines: Sequence[str], min_score: float = 0.01) -> List[str]:
    out: List[str] = []
    rid, coords = "", []
    for raw in list(lines)[1:]:
        f = raw.rstrip("\n").split("\t")
        while f and f[-1] == "":   # Perl split drops trailing empty fields
            f.pop()
        id_ = f[0] if f else ""
        fr = f[1] if len(f) > 1 else ""
        to = f[2] if len(f) > 2 else ""
        score = f[3] if len(f) > 3 else ""
        if id_ != rid:
            if coords:
                c = ["0"] + coords
                i = 0
                while i < len(c) - 1:
                    out.append(f"{rid}\t{c[i]}\t{c[i + 1]}")
                    i += 2
                out.append(f"{rid}\t{c[i]}")
            rid, coords = id_, []
        elif _perl_num(score) >= min_score:
            coords += [fr, to]
    return out


def main(argv: Optional[List[str]] = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser(prog="ChimeraToSeqFilter")
    ap.add_argument("input", nargs="?")
    ap.add_argument("--in", dest="inp")
    ap.add_argument("--out")
    ap.add_argument("--min-score", default="0.01")
    ap.add_argument("--trim-length", type=int, default=20)
    ap.add_argument("--verbose", type=int, default=2)
    ap.add_argument("--quiet", action="store_true")
    a = ap.parse_args(argv)
    path = a.inp or a.input
    if not path:
        print("Input file required", file=sys.stderr)
        return 1
    try:
        with open(path) as fh:
            lines = fh.read().splitlines()
    except OSError as e:
        print(str(e), file=sys.stderr)
        return 255
    res = convert(lines, _perl_num(a.min_score))
    text = "".join(x + "\n" for x in res)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)
    else:
        sys.stdout.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
