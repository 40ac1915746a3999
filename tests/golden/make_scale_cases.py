"""Full-size consensus cases pinned to the reference Perl engine (VERDICT r03 "pin finish mode
at scale"): 10 kb long reads at 15 % CLR error with the bwa-mode alignments a real iteration
feeds bam2cns, in two task settings:

  bwa-sr-1      the raw long reads (qualities '$'), short reads sampled to 15x, bwa-sr
                options, -b 20 -l 300, coverage cap 11.25, --use-ref-qual
                (bin/proovread:1302-1313, 1541; proovread.cfg:188-192, 318-333)
  bwa-sr-finish the reads corrected by that bwa-sr-1 iteration (sequence and qualities of the
                consensus), short reads sampled to 30x, finish seeding/SW options with -D .75,
                -b 20 -l 600, cap 22.5, --no-use-ref-qual --detect-chimera, --max-ins-length 0
                (bin/proovread:1572-1579; lib/Sam/Seq.pm:774-889; bin/bam2cns:461-491)

Six of the 64 long reads are chimeric (first half of one read, second half of a read from
elsewhere in the genome), so the finish cases exercise chimera() / detect_chimera on real
breakpoints.  The alignments come from the oracle chain (host seeding, oracle/aln_oracle.c +
sw_oracle.c: bwa mem's per-read alignment restated) -- only the consensus half of this fixture
is pinned by the Perl run; its inputs are the ones the GPU's SW stage equals bit for bit.

    python make_scale_cases.py OUT_DIR        (writes bwa_sr1_cases.txt and finish_cases.txt)

regen_scale.sh runs this, then gen_cns_golden.pl over both files, and gzips everything.
"""
from __future__ import annotations

import dataclasses
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path[:0] = [str(HERE), str(ROOT / "tests"), str(ROOT), str(ROOT / "oracle")]
import cpu_chain  # noqa: E402
from casefmt import Case, write_cases  # noqa: E402

from proovread_amd import seed, synth  # noqa: E402

ASCII = np.frombuffer(b"ACGTN", np.uint8)
NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = _i
N_LR, N_CASES = 64, 32
CHIMERAS = {5: 37, 13: 50, 22: 2, 29: 61, 40: 18, 57: 9}   # read -> donor of its second half


def pool(seqs):
    off = np.zeros(len(seqs) + 1, np.int64)
    np.cumsum([len(s) for s in seqs], out=off[1:])
    return np.concatenate(seqs).astype(np.uint8), off


def main():
    out = Path(sys.argv[1])
    d = synth.simulate(20261104, 100_000, N_LR, 10_000, 50.0)
    lrs = [d.lr_seq[d.lr_off[i]:d.lr_off[i + 1]] for i in range(N_LR)]
    for i, j in CHIMERAS.items():
        a, b = lrs[i], d.lr_seq[d.lr_off[j]:d.lr_off[j + 1]]
        lrs[i] = np.concatenate([a[:len(a) // 2], b[len(b) // 2:]])
    lr_seq, lr_off = pool(lrs)
    k = np.arange(d.n_sr)
    sel1 = np.nonzero(k % 10 < 3)[0]            # 15x of the 50x set
    sel2 = np.nonzero(k % 10 >= 4)[0]           # 30x
    cases_pick = list(range(0, N_LR, 2))[:N_CASES - len(CHIMERAS)]
    cases_pick = sorted(set(cases_pick) | set(CHIMERAS))[:N_CASES]

    def sr_subset(sel):
        L = (d.sr_off[1:] - d.sr_off[:-1])[sel]
        off = np.zeros(len(sel) + 1, np.int64)
        np.cumsum(L, out=off[1:])
        idx = np.concatenate([np.arange(d.sr_off[s], d.sr_off[s + 1]) for s in sel])
        return d.sr_seq[idx], off

    def bwa_mode(lseq, loff, sseq, soff, finish):
        ix = seed.SeedIndex(lseq, loff)
        tk = ix.map(sseq, soff, seed.default_opts(finish), threads=8)
        ix.close()
        dd = dataclasses.replace(d, lr_seq=lseq, lr_off=loff, sr_seq=sseq, sr_off=soff)
        return synth.with_seeds(dd, tk)

    # bwa-sr-1 on the raw reads
    s1, o1 = sr_subset(sel1)
    db = bwa_mode(lr_seq, lr_off, s1, o1, False)
    _, _, sams1, _ = cpu_chain.run_sample(db, range(N_LR), task="bwa-sr", bin_filter=(20, 300), sam_only=True,
                                          workers=8)
    _, _, full1, _ = cpu_chain.run_sample(db, range(N_LR), task="bwa-sr", coverage=11.25, use_ref_qual=True,
                                          bin_filter=(20, 300), full=True, workers=8)
    cases1, cseq, cqual = [], [], []
    for i in range(N_LR):
        rc, fq, _, _ = full1[i]
        assert rc == 0, (i, rc)
        _, s, _, q = fq.rstrip("\n").split("\n")
        cseq.append(s)
        cqual.append(q)
    for i in cases_pick:
        ref = ASCII[lrs[i]].tobytes().decode()
        cases1.append(Case(f"sr1_lr{i}", {"coverage": "11.25", "use_ref_qual": "1"},
                           [f"@lr{i}", ref, "+", "$" * len(ref)], sams1[i]))
    write_cases(out / "bwa_sr1_cases.txt", cases1)

    # bwa-sr-finish on the corrected reads (mapping reference = unmasked .fq, proovread:838-850)
    c_seq, c_off = pool([NT4[np.frombuffer(s.encode(), np.uint8)] for s in cseq])
    s2, o2 = sr_subset(sel2)
    db2 = bwa_mode(c_seq, c_off, s2, o2, True)
    _, _, sams2, _ = cpu_chain.run_sample(db2, range(N_LR), task="bwa-sr-finish", bin_filter=(20, 600),
                                          sam_only=True, workers=8)
    cases2 = []
    for i in cases_pick:
        cases2.append(Case(f"fin_lr{i}", {"coverage": "22.5", "use_ref_qual": "0", "detect_chimera": "1"},
                           [f"@lr{i}", cseq[i], "+", cqual[i]], sams2[i]))
    write_cases(out / "finish_cases.txt", cases2)
    for name, cs in (("bwa-sr-1", cases1), ("finish", cases2)):
        print(f"{name}: {len(cs)} reads, {sum(len(c.ref[1]) for c in cs)} columns, "
              f"{sum(len(c.sam) for c in cs)} alignments")


if __name__ == "__main__":
    main()
