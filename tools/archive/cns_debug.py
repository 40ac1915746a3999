"""Debug helper: run the golden consensus cases on the GPU and print first diffs."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "tests" / "golden")]
import casefmt
from cns_case_util import case_inputs
from proovread_amd import cns

cases = casefmt.read_cases(ROOT / "tests/golden/cns_cases.txt")
exp = casefmt.read_expect(ROOT / "tests/golden/cns_expected.txt")
nbad = 0
for c in cases:
    lr, alns, p = case_inputs(c)
    if p.qual_weighted:
        continue
    r = cns.run_chunk([lr], [alns], p)[0]
    e = exp[c.name]
    if e.error:
        ok = r.status != 0
        if not ok:
            print(c.name, "expected error, got", r.status)
        continue
    if r.status != 0:
        print(c.name, "status", r.status); nbad += 1; continue
    fq = r.fastq.rstrip("\n").split("\n")
    msgs = []
    for nm, a, b in (("seq", fq[1], e.fastq[1]), ("qual", fq[3], e.fastq[3]), ("trace", r.trace, e.trace)):
        if a != b:
            i = next((k for k in range(min(len(a), len(b))) if a[k] != b[k]), min(len(a), len(b)))
            msgs.append(f"{nm}@{i} len {len(a)}/{len(b)} got {a[max(0,i-5):i+8]!r} exp {b[max(0,i-5):i+8]!r}")
    if r.chim_lines() != e.chim:
        msgs.append(f"chim got {r.chim_lines()} exp {e.chim}")
    kept = "".join(str(int(x)) for x in r.kept)
    if kept != e.kept:
        msgs.append("kept differs")
    if msgs:
        nbad += 1
        print(c.name, " | ".join(msgs))
print("bad", nbad, "of", len(cases))
