"""Consensus cases on the reference's bundled sample ("one fixture set
built on sample/F.antasticus_long_error.fq with SR alignments simulated from
F.antasticus_genome.fa").

Short reads are simulated from the genome at 15x (the sample's short-read file is not
in the checkout), seeded by the product's host front end (pr_seed_map) and extended
by the SW oracle (oracle/sw_oracle.c); each selected long read's passing alignments
become SAM records in samtools coordinate order, its FASTQ record (IUPAC codes and
all) the reference.  The expected outputs come from the reference Perl engine
(gen_cns_golden.pl, regen_fantasticus.sh).

    python make_fantasticus_cases.py OUT_CASES
"""
from __future__ import annotations

import ctypes as C
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import oracle_bind as ob  # noqa: E402
from casefmt import Case, write_cases  # noqa: E402

from proovread_amd import bwa_proovread as bp  # noqa: E402
from proovread_amd import seed, sw  # noqa: E402

FX = HERE / "fantasticus"
ASCII = np.frombuffer(b"ACGTN", np.uint8)


def simulate_sr(G, cov, seed_=20261015, L=150):
    rng = np.random.default_rng(seed_)
    n = int(cov * len(G) / L)
    st = rng.integers(0, len(G) - L, n)
    srs = G[st[:, None] + np.arange(L)[None, :]].copy()
    m = rng.random(n) < 0.15
    pos = rng.integers(0, L, int(m.sum()))
    srs[np.nonzero(m)[0], pos] = (srs[np.nonzero(m)[0], pos] + 1) % 4
    rev = rng.random(n) < 0.5
    srs[rev] = (3 - srs[rev])[:, ::-1]
    return srs.reshape(-1).astype(np.uint8), np.arange(n + 1, dtype=np.int64) * L


def read_fastq(path):
    lines = Path(path).read_text().splitlines()
    return [(lines[i][1:], lines[i + 1], lines[i + 3]) for i in range(0, len(lines) - 3, 4)]


def main():
    out = sys.argv[1]
    recs = read_fastq(FX / "F.antasticus_long_error.fq")
    names, seqs, _ = bp.read_fastx(str(FX / "F.antasticus_long_error.fq"))
    _, gs, _ = bp.read_fastx(str(FX / "F.antasticus_genome.fa"))
    G = sw.NT4[np.frombuffer(gs[0], np.uint8)]
    lr_seq, lr_off = bp._pool(seqs)
    sr_seq, sr_off = simulate_sr(G, 15)
    ix = seed.SeedIndex(lr_seq, lr_off)
    tasks = ix.map(sr_seq, sr_off, seed.default_opts(False), threads=4)
    ix.close()
    L = ob.sw_lib()
    opts = ob.sw_opts("bwa-sr")
    by_lr = {}
    r = ob.OswResult()
    for t in tasks:
        lr, sid = int(t["lr"]), int(t["sr"])
        so, lq = int(sr_off[sid]), int(sr_off[sid + 1] - sr_off[sid])
        Llen = int(lr_off[lr + 1] - lr_off[lr])
        rc = L.osw_task(C.byref(opts), C.cast(sr_seq.ctypes.data + so, C.POINTER(C.c_uint8)), lq,
                        C.cast(lr_seq.ctypes.data + int(lr_off[lr]), C.POINTER(C.c_uint8)), Llen, int(t["strand"]),
                        int(t["qbeg"]), int(t["rbeg"]), int(t["slen"]), C.byref(r))
        if rc or not getattr(r, "pass"):
            continue
        strand = int(t["strand"])
        q = sr_seq[so:so + lq]
        s = (ASCII[np.where(q < 4, 3 - q, 4)][::-1] if strand else ASCII[q]).tobytes().decode()
        cg = "".join(f"{x >> 4}{'MIDNSHP=X'[x & 15]}" for x in r.cigar[:r.n_cigar])
        by_lr.setdefault(lr, []).append((r.pos, strand, len(by_lr.get(lr, [])),
                                         f"sr{sid}\t{16 if strand else 0}\t{names[lr]}\t{r.pos + 1}\t60\t{cg}\t*\t0\t0\t"
                                         f"{s}\t{'I' * lq}\tAS:i:{r.score}"))
    # long reads with the most alignments (deep pileups, bin capping), plus the first IUPAC one
    ranked = sorted(by_lr, key=lambda k: -len(by_lr[k]))
    pick = ranked[:10]
    iupac = [i for i in by_lr if any(c not in "ACGTacgt" for c in recs[i][1])]
    for i in iupac[:2]:
        if i not in pick:
            pick.append(i)
    cases = []
    for k, lr in enumerate(pick):
        alns = sorted(by_lr[lr], key=lambda x: (x[0], x[1], x[2]))
        head, seq_, qual = recs[lr]
        params = {"coverage": "11.25", "use_ref_qual": "1"}
        if k % 3 == 2:
            params["detect_chimera"] = "1"
        if k % 4 == 3:
            params["use_ref_qual"] = "0"
        cases.append(Case(f"fant_{lr}", params, ["@" + head, seq_, "+", qual], [a[3] for a in alns]))
    write_cases(out, cases)
    print(f"{len(cases)} cases, {sum(len(c.sam) for c in cases)} alignments")


if __name__ == "__main__":
    main()
