"""Helpers for SW parity tests: run the oracle over a synthetic task list."""
import numpy as np

import oracle_bind as ob


def oracle_results(d, opts, idx):
    out = []
    for t in idx:
        r, cg = ob.sw_task(opts, d.sr_str(d.t_sr[t]), d.lr_str(d.t_lr[t]), int(d.t_strand[t]),
                           int(d.t_qbeg[t]), int(d.t_rbeg[t]), int(d.t_slen[t]))
        out.append((r.qb, r.qe, r.rb, r.re, r.score, r.truesc, r.pos, cg, int(getattr(r, "pass"))))
    return out


def gpu_tuple(res, t):
    a = res.a
    return (int(a["qb"][t]), int(a["qe"][t]), int(a["rb"][t]), int(a["re"][t]), int(a["score"][t]),
            int(a["truesc"][t]), int(a["pos"][t]), res.cigar_str(t), int(a["pass"][t]))


def with_ns(d, rng, frac=0.002):
    """Sprinkle N (code 4) into the long reads (bwa maps ambiguous bases to 4)."""
    m = rng.random(len(d.lr_seq)) < frac
    d.lr_seq = d.lr_seq.copy()
    d.lr_seq[m] = 4
    return d
