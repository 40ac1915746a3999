"""CPU reference of one iteration (TEST INFRASTRUCTURE): SW oracle for every
task -> SAM records (bwa mem_aln2sam fields the consensus reads) -> sort per
long read in samtools coordinate order (POS, strand, input order) -> consensus
oracle per long read."""
import numpy as np

import oracle_bind as ob
from casefmt import Case


def rc(s):
    return s[::-1].translate(str.maketrans("ACGTN", "TGCAN"))


def sam_for_tasks(d, task="bwa-sr"):
    o = ob.sw_opts(task)
    per_lr = {}
    for t in range(len(d.t_sr)):
        sr, lr = int(d.t_sr[t]), int(d.t_lr[t])
        q = d.sr_str(sr)
        r, cg = ob.sw_task(o, q, d.lr_str(lr), int(d.t_strand[t]), int(d.t_qbeg[t]), int(d.t_rbeg[t]),
                           int(d.t_slen[t]))
        if not getattr(r, "pass"):
            continue
        strand = int(d.t_strand[t])
        seq = rc(q) if strand else q
        line = f"sr{sr}\t{16 if strand else 0}\tlr{lr}\t{r.pos + 1}\t60\t{cg}\t*\t0\t0\t{seq}\t{'I' * len(seq)}\tAS:i:{r.score}"
        per_lr.setdefault(lr, []).append((r.pos, strand, t, line))
    return {lr: [x[3] for x in sorted(v, key=lambda x: (x[0], x[1], x[2]))] for lr, v in per_lr.items()}


def consensus_cases(d, sams, params):
    cases = []
    for lr in range(d.n_lr):
        seq = d.lr_str(lr)
        c = Case(f"lr{lr}", dict(params), [f"@lr{lr}", seq, "+", "$" * len(seq)], sams.get(lr, []))
        cases.append(c)
    return cases
