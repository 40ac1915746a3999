"""CPU reference of one iteration (TEST INFRASTRUCTURE): SW oracle for every
task -> SAM records (bwa mem_aln2sam fields the consensus reads) -> sort per
long read in samtools coordinate order (POS, strand, input order) -> consensus
oracle per long read."""
import numpy as np

import oracle_bind as ob
from casefmt import Case


def rc(s):
    return s[::-1].translate(str.maketrans("ACGTN", "TGCAN"))


def sam_for_tasks(d, task="bwa-sr", bin_filter=None):
    """bin_filter: (BIN, LEN) of bwa-proovread -b/-l over each long read's records in task
    (= bwa output) order (oracle/cpu_chain.py restatement)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import cpu_chain
    o = ob.sw_opts(task) if isinstance(task, str) else task   # a task name or an OswOpts
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
        per_lr.setdefault(lr, []).append((r.pos, strand, t, line, float(r.score),
                                          cpu_chain._aln_length(list(r.cigar[:r.n_cigar]), len(q))))
    if bin_filter:
        for lr, v in per_lr.items():
            keep = cpu_chain._bin_filter([(x[0], x[4], x[5]) for x in v], *bin_filter)
            per_lr[lr] = [x for x, k in zip(v, keep) if k]
    return {lr: [x[3] for x in sorted(v, key=lambda x: (x[0], x[1], x[2]))] for lr, v in per_lr.items()}


def consensus_cases(d, sams, params):
    cases = []
    for lr in range(d.n_lr):
        seq = d.lr_str(lr)
        c = Case(f"lr{lr}", dict(params), [f"@lr{lr}", seq, "+", "$" * len(seq)], sams.get(lr, []))
        cases.append(c)
    return cases
