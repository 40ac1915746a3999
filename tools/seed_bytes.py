"""Algorithmic bytes per short read of the seeding stage on bench.py's dataset (configs[1]):
the compulsory reads of the index and writes of the output, not the scratch the lane-per-read
kernel moves.  Per read:
  150 B of bases
  16 B per start with a 12-mer (koff[code], koff[code + 1])
  32 B per occurrence-table hit: kpos (4) + kext (8) for the match length, cblk (4) + cstart (8)
      + lr_off (8) for its long read and coordinate
  40 B per output seed (pr_seed_task)
Hits per read: the 12-mer counts of the indexed text (both strands of every long read) summed
over a read's starts, averaged over a 20 k-read sample.  Prints the constants bench.py uses.

    python tools/seed_bytes.py
"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from proovread_amd import synth  # noqa: E402

SEED, GENOME, N_LR = 20261015 + 2, 4_600_000, 13_800
n_sr = int(round(50.0 * GENOME / 150 * 6 / 20))
d = synth.simulate_reads(SEED, GENOME, N_LR, 10_000, n_sr, threads=8)
K = 12


def kmer_codes(seq):
    s = seq.astype(np.int64)
    ok = s < 4
    n = len(s) - K + 1
    code = np.zeros(n, np.int64)
    good = np.ones(n, bool)
    for j in range(K):
        code = code * 4 + np.where(ok[j:j + n], s[j:j + n], 0)
        good &= ok[j:j + n]
    return code, good


lr = d.lr_seq
# text: forward reads and their reverse complement (12-mers never span two reads: count per read)
counts = np.zeros(4 ** K, np.int64)
off = d.lr_off
step = 2000
for i in range(0, N_LR, step):
    a, b = off[i], off[min(i + step, N_LR)]
    seg = lr[a:b]
    bounds = off[i:min(i + step, N_LR) + 1] - a
    for strand in (0, 1):
        s = seg if strand == 0 else np.where(seg[::-1] < 4, 3 - seg[::-1], 4).astype(np.uint8)
        code, good = kmer_codes(s)
        # drop k-mers that cross a read boundary
        pos = np.arange(len(code))
        bb = bounds if strand == 0 else (len(seg) - bounds)[::-1]
        rid_start = np.searchsorted(bb, pos, side="right")
        rid_end = np.searchsorted(bb, pos + K - 1, side="right")
        keep = good & (rid_start == rid_end)
        counts += np.bincount(code[keep], minlength=4 ** K)
rng = np.random.default_rng(1)
pick = rng.choice(n_sr, 20000, replace=False)
starts = hits = 0
for i in pick:
    r = d.sr_seq[d.sr_off[i]:d.sr_off[i + 1]]
    code, good = kmer_codes(r)
    starts += int(good.sum())
    hits += int(counts[code[good]].sum())
sp, hp = starts / len(pick), hits / len(pick)
print(f"starts with a 12-mer per read {sp:.1f}, occurrence-table hits per read {hp:.1f}")
print(f"bytes per read without the output: {150 + 16 * sp + 32 * hp:.0f} (+ 40 per output seed)")
