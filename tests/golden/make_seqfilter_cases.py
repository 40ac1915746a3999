"""Case generator for the masking / trim-window goldens (seeded, deterministic).

    python make_seqfilter_cases.py OUT_CASES

Case lines (tab separated):
    MASK  pmin pmax mask_min unmask_min reduce end_ratio qual
    WIN   size soft hard min_len qual          (qual: phred+33 chars)
"""
import random
import sys


def segs(rng, L, hi_lo, lo_hi, p_hi, hi_len, lo_len):
    out = []
    while len(out) < L:
        if rng.random() < p_hi:
            n = rng.randint(*hi_len)
            out += [rng.randint(*hi_lo) for _ in range(n)]
        else:
            n = rng.randint(*lo_len)
            out += [rng.randint(*lo_hi) for _ in range(n)]
    return out[:L]


def qs(ph):
    return "".join(chr(33 + max(0, min(41, p))) for p in ph)


MASK_PARAMS = [
    (20, 41, 80, 130, 60, 0.7),     # proovread.cfg:235 at 100 bp
    (20, 41, 120, 195, 60, 0.7),    # scaled to 150 bp (proovread:1703-1704)
    (20, 41, 120, 195, 60, 0.3),    # bwa-sr-4..6
    (20, 41, 10, 40, 5, 0.5),       # small values: many HCRs, iterative gap loop
    (20, 41, 5, 60, 2, 0.7),
    (25, 35, 20, 30, 0, 0.0),
    (20, 41, 1, 25, 3, 1.0),
]
WIN_PARAMS = [(10, 12, 5, 10), (10, 25, 3, 10), (10, 12, 5, 30), (5, 20, 8, 5), (3, 15, 2, 3)]


def main():
    out = sys.argv[1]
    rng = random.Random(20261016)
    lines = []
    for k, P in enumerate(MASK_PARAMS):
        for t in range(14):
            L = rng.choice([0, 1, 50, 199, 400, 1000, 2500, 6000])
            hi_len = rng.choice([(5, 60), (50, 400), (150, 1500), (1, 20)])
            lo_len = rng.choice([(1, 5), (5, 40), (30, 300), (100, 200)])
            ph = segs(rng, L, (20, 41), (0, 19), rng.choice([0.5, 0.7, 0.9]), hi_len, lo_len)
            if t == 0 and L:
                ph = [rng.randint(20, 41) for _ in range(L)]   # whole read high
            if t == 1 and L:
                ph = [rng.randint(0, 19) for _ in range(L)]    # nothing to mask
            lines.append("MASK\t" + "\t".join(map(str, P)) + "\t" + qs(ph))
    for k, P in enumerate(WIN_PARAMS):
        for t in range(16):
            L = rng.choice([0, 3, 9, 10, 11, 40, 300, 1200, 5000])
            ph = segs(rng, L, (rng.choice([10, 14, 20]), 41), (0, rng.choice([4, 12, 20])),
                      rng.choice([0.4, 0.6, 0.85]), rng.choice([(1, 8), (5, 50), (30, 400)]),
                      rng.choice([(1, 3), (1, 10), (5, 60)]))
            if t == 0 and L:
                ph = [40] * L
            if t == 1 and L:
                ph = [rng.choice([2, 30]) for _ in range(L)]
            lines.append("WIN\t" + "\t".join(map(str, P)) + "\t" + qs(ph))
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
