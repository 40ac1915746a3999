"""Deterministic generator of consensus-stage test cases (SAM alignments of
short reads against one long read + the long read as reference FASTQ).

The cases are built to exercise every branch of the reference consensus
engine: bin capping and eviction, soft/hard clips,
taboo head/tail trimming (including leading/trailing indels), D+I pairs,
leading insertions, ties between insertion states, empty columns, reference
quality injection, MCR ignore ranges, max-ins-length, qual-weighting,
missing AS tags, and chimera windows.

    python make_cns_cases.py out_cases.txt [n_random]
"""
from __future__ import annotations

import random
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from casefmt import Case, write_cases  # noqa: E402

BASES = "ACGT"


def rand_seq(rng, n, alphabet=BASES):
    return "".join(rng.choice(alphabet) for _ in range(n))


def mutate_read(rng, ref, start, rlen, p_sub, p_ins, p_del, ins_max=3, del_max=3):
    """Walk the reference from `start`, emitting a read and its CIGAR."""
    ops = []
    seq = []
    r = start
    while len(seq) < rlen and r < len(ref):
        x = rng.random()
        if x < p_ins and seq:
            k = rng.randint(1, ins_max)
            seq.extend(rand_seq(rng, k))
            ops.append(("I", k))
        elif x < p_ins + p_del and seq:
            k = rng.randint(1, del_max)
            k = min(k, len(ref) - r - 1)
            if k <= 0:
                continue
            r += k
            ops.append(("D", k))
        else:
            b = ref[r]
            if rng.random() < p_sub:
                b = rng.choice([c for c in BASES if c != b.upper()])
            seq.append(b)
            ops.append(("M", 1))
            r += 1
    # merge
    merged = []
    for op, k in ops:
        if merged and merged[-1][0] == op:
            merged[-1] = (op, merged[-1][1] + k)
        else:
            merged.append((op, k))
    # a trailing D would make the span end after the read; drop it
    while merged and merged[-1][0] == "D":
        merged.pop()
    return "".join(seq), merged


def cigar_str(ops):
    return "".join(f"{k}{op}" for op, k in ops)


def sam_line(qname, flag, rname, pos, cigar, seq, qual, score):
    opt = f"\tAS:i:{score}" if score is not None else ""
    return f"{qname}\t{flag}\t{rname}\t{pos}\t60\t{cigar}\t*\t0\t0\t{seq}\t{qual}{opt}"


def make_case(rng, name, L=None, cov=None, params=None, chimera=False, quirks=True):
    L = L or rng.randint(300, 1600)
    cov = cov or rng.choice([4, 8, 15, 25, 40])
    ref = rand_seq(rng, L)
    if quirks and rng.random() < 0.3:   # IUPAC / lowercase n in the reference
        ref = list(ref)
        for _ in range(rng.randint(1, 4)):
            ref[rng.randrange(L)] = rng.choice("NnRY")
        ref = "".join(ref)
    rid = f"lr_{name}"
    params = dict(params or {})
    desc = ""
    if params.pop("mcr", None):
        a = rng.randrange(0, L - 60)
        b = rng.randrange(0, L - 60)
        desc = f" MCR1:{a},{rng.randint(5, 50)} MCR2:{b},{rng.randint(5, 50)}"
    if params.get("use_ref_qual", "1") == "1" and rng.random() < 0.5:
        rq = "".join(chr(33 + rng.randint(0, 40)) for _ in range(L))
    else:
        rq = "$" * L
    if rng.random() < 0.15:
        rq = rq[: L - rng.randint(1, 30)] + "".join(chr(33 + rng.choice([0, 1, 2])) for _ in range(0))
        rq = rq + "$" * (L - len(rq))
    reads = []
    n_reads = max(1, int(cov * L / 120))
    src2 = rand_seq(rng, L) if chimera else None
    gap = None
    if chimera:
        g0 = rng.randint(L // 2 - 40, L // 2)
        gap = (g0, g0 + rng.randint(20, 70))
    for i in range(n_reads):
        rl = rng.choice([150, 150, 150, 120, 100, 60, 52, 45, 149])
        start = rng.randrange(0, max(1, L - 30))
        if chimera and gap[0] - 100 < start < gap[1]:
            # thin coverage around the breakpoint: few reads span it
            if rng.random() < 0.85:
                continue
        base = ref
        if chimera and start > gap[1] - 10 and rng.random() < 0.7:
            # right part of a chimera: the reads carry another haplotype in
            # the junction region so combined columns have higher entropy
            base = ref[: gap[0]] + src2[gap[0]: gap[1] + 40] + ref[gap[1] + 40:]
        er = rng.choice([0.0, 0.01, 0.03, 0.08])
        seq, ops = mutate_read(rng, base, start, rl, er, er / 2, er / 2)
        if not ops or not any(op == "M" for op, _ in ops):
            continue
        span = sum(k for op, k in ops if op in "MD")
        if start + span > L:
            continue
        # edge indels for the taboo trim
        if quirks and rng.random() < 0.08 and ops[0][0] == "M" and ops[0][1] > 6:
            k = rng.randint(1, 4)
            ops = [("M", 2), ("I", k)] + [("M", ops[0][1] - 2)] + ops[1:]
            seq = seq[:2] + rand_seq(rng, k) + seq[2:]
        if quirks and rng.random() < 0.04:
            # leading insertion (no M before): creates a state at the first column
            k = rng.randint(1, 3)
            ops = [("I", k)] + ops
            seq = rand_seq(rng, k) + seq
        if quirks and rng.random() < 0.05 and ops[-1][0] == "M" and ops[-1][1] > 6:
            k = rng.randint(1, 3)
            ops = ops[:-1] + [("M", ops[-1][1] - 3), ("D", k), ("M", 3)]
            seq = seq  # read bases unchanged; span grows by k
            if start + sum(x for o, x in ops if o in "MD") > L:
                continue
        if quirks and rng.random() < 0.05:
            # D immediately followed by I (bowtie2-style mismatch)
            mids = [j for j, (o, k) in enumerate(ops) if o == "M" and k > 10]
            if mids:
                j = rng.choice(mids)
                k = ops[j][1]
                qoff = sum(x for o, x in ops[:j] if o in "MI")
                ops = ops[:j] + [("M", k // 2), ("D", 1), ("I", 1), ("M", k - k // 2 - 1)] + ops[j + 1:]
                # read keeps its length: the I consumes the base that the M lost
                if start + sum(x for o, x in ops if o in "MD") > L:
                    continue
                _ = qoff
        # soft / hard clips
        if quirks and rng.random() < 0.15:
            k = rng.randint(1, 40)
            ops = [("S", k)] + ops
            seq = rand_seq(rng, k) + seq
        if quirks and rng.random() < 0.12:
            k = rng.randint(1, 40)
            ops = ops + [("S", k)]
            seq = seq + rand_seq(rng, k)
        if quirks and rng.random() < 0.03 and ops[0][0] != "S":
            ops = [("H", rng.randint(1, 20))] + ops
        qlen = sum(k for op, k in ops if op in "MIS")
        if qlen != len(seq):
            continue
        if rng.random() < 0.05:
            qual = "*"
        else:
            qual = "".join(chr(33 + rng.randint(2, 40)) for _ in range(len(seq)))
        aspan = sum(k for op, k in ops if op in "M")
        r = rng.random()
        if r < 0.04:
            score = None
        elif r < 0.3:
            score = rng.choice([aspan * 5 - 20, aspan * 5 - 20, aspan * 3, 100])  # ties
        else:
            score = rng.randint(-20, 5 * aspan)
        flag = rng.choice([0, 16, 256, 272])
        reads.append((start + 1, flag, cigar_str(ops), seq, qual, score, i))
    # BAM coordinate order: pos, then strand, then input order
    reads.sort(key=lambda t: (t[0], (t[1] & 16) >> 4, t[6]))
    sam = [sam_line(f"sr{t[6]}", t[1], rid, t[0], t[2], t[3], t[4], t[5]) for t in reads]
    return Case(name, params, [f"@{rid}{desc}", ref, "+", rq], sam)


def handcrafted():
    """Small cases checking single behaviours."""
    cases = []
    ref = "ACGTACGTTGCATGCAAACCCGGGTTTACGATCGATCGTAGCTAGCTAGGATCCATGCATGACGATGCAGCATGCATGCCCATGACGTTTACGGGACATGACGAGCATGCGGCATAAAAAACGACTAGCCCCCCA"
    L = len(ref)
    rid = "hc_lr"

    def mk(name, alns, params=None, refq=None, desc=""):
        sam = []
        for j, (pos, cig, seq, sc) in enumerate(alns):
            sam.append(sam_line(f"q{j}", 0, rid, pos, cig, seq, "I" * len(seq), sc))
        return Case(name, dict(params or {}), [f"@{rid}{desc}", ref, "+", refq or "$" * L], sam)

    r60 = ref[10:70]
    # ties between two insertion states at the same column
    a1 = r60[:30] + "T" + r60[30:]
    a2 = r60[:30] + "G" + r60[30:]
    cases.append(mk("ins_tie", [(11, "30M1I30M", a1, 300), (11, "30M1I30M", a2, 300),
                                (11, "30M1I30M", a2, 290), (11, "30M1I30M", a1, 280)],
                    {"use_ref_qual": "0"}))
    cases.append(mk("ins_tie_refq", [(11, "30M1I30M", a2, 300), (11, "30M1I30M", a1, 300)]))
    # D+I → mismatch
    cases.append(mk("del_ins", [(11, "30M1D1I29M", r60[:30] + "A" + r60[31:], 250)] * 3,
                    {"use_ref_qual": "0"}))
    # deletion majority → trace I
    d = r60[:25] + r60[27:]
    cases.append(mk("del_major", [(11, "25M2D33M", d, 250)] * 3 + [(11, "60M", r60, 240)]))
    # leading insertion (no trim: taboo not reachable) and trim off
    cases.append(mk("lead_ins", [(11, "2I60M", "TT" + r60, 260), (11, "60M", r60, 250)],
                    {"use_ref_qual": "0"}))
    # soft clips
    cases.append(mk("softclip", [(11, "5S60M", "GGGGG" + r60, 260),
                                 (11, "60M7S", r60 + "CCCCCCC", 250)]))
    # max-ins-length skip
    a3 = r60[:30] + "TTTT" + r60[30:]
    cases.append(mk("maxins", [(11, "30M4I30M", a3, 300)] * 3, {"max_ins_length": "3"}))
    # no AS tag
    cases.append(mk("noscore", [(11, "60M", r60, None), (11, "60M", r60, 200)]))
    # empty reference columns keep ref bases, and 'n' without ref
    cases.append(mk("noref", [(21, "60M", ref[20:80], 200)], {"noref": "1"}))
    # MCR ignore ranges
    cases.append(mk("mcr", [(11, "60M", r60, 200)] * 2, desc=" MCR1:20,10 MCR2:60,5"))
    # bin overflow: many alignments in one bin, eviction of the lowest
    many = [(11, "60M", r60, 200 + (k * 7) % 13) for k in range(12)]
    cases.append(mk("bin_evict", many, {"coverage": "5"}))
    # read beyond reference end -> reference dies (bin out of range)
    # hard clip in front of a soft clip: the reference dies (Unknown Cigar 'S')
    cases.append(mk("hclip_sclip", [(11, "5H3S60M", "GGG" + r60, 260)]))
    cases.append(mk("hclip", [(11, "5H60M4H", r60, 260), (11, "60M", r60, 250)]))
    cases.append(mk("beyond_end", [(L - 20, "60M", ref[L - 21:] + "A" * 39, 200)]))
    return cases


def main():
    out = sys.argv[1]
    n_random = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rng = random.Random(20261015)
    cases = handcrafted()
    for i in range(n_random):
        params = {}
        params["coverage"] = rng.choice(["11.25", "11.25", "22.5", "5", "37.5"])
        params["use_ref_qual"] = rng.choice(["1", "1", "0"])
        params["detect_chimera"] = rng.choice(["0", "1"])
        params["max_ins_length"] = rng.choice(["0", "0", "0", "2", "3"])
        params["qual_weighted"] = rng.choice(["0"] * 6 + ["1"])
        if rng.random() < 0.1:
            params["mcr"] = "1"
        chim = params["detect_chimera"] == "1" and rng.random() < 0.6
        L = rng.randint(450, 1800) if chim else None
        cases.append(make_case(rng, f"rnd{i:03d}", L=L, params=params, chimera=chim))
    write_cases(out, cases)


if __name__ == "__main__":
    main()
