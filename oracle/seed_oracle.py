"""ORACLE — TEST INFRASTRUCTURE ONLY.  Never imported by the product path.

Pure-Python restatement of the seeding / chaining front end of bwa mem as used
by proovread (`bwa-proovread mem`, bin/proovread:1313, options proovread.cfg:
318-333), for small inputs.  It checks the library's host implementation
(proovread_amd/csrc/seed.cpp) with an independent occurrence oracle: every
substring count is a plain string search over the long reads and their reverse
complements (no k-mer index, no count tables).

Restated from upstream bwa (absent here; bwa-proovread's pinned commit is
unknown, .gitmodules:4-6 — parity unpinned):
  bwamem.c  mem_collect_intv (three seeding rounds), mem_chain, test_and_merge,
            mem_chain_weight, mem_chain_flt, mem_flt_chained_seeds + mem_seed_sw (bwa >=
            0.7.13: reads with 1.1 W <= 0.05 length), mem_chain2aln's seed order (every
            seed of a kept chain, srt order) and window
  ksw.c     ksw_align2's best local score (mem_seed_sw), as a plain affine-gap local DP
  bwt.c     bwt_smem1a (max_intv = 0), bwt_seed_strategy1
over the same index definition as the library: forward long reads then the
reverse complement of their concatenation (bwa's forward-reverse coordinates),
contigs separated, N never matching, occurrences of a seed in text-position order.
"""
from __future__ import annotations

import bisect
import dataclasses
import math
import struct

COMP = {0: 3, 1: 2, 2: 1, 3: 0}


@dataclasses.dataclass
class Opts:
    min_seed_len: int = 12
    min_chain_weight: int = 20
    w: int = 40
    split_factor: float = 1.0
    split_width: int = 10
    max_mem_intv: int = 20
    max_occ: int = 500
    drop_ratio: float = 0.0
    max_chain_gap: int = 10000
    mask_level: float = 0.5
    a: int = 5
    o_del: int = 2
    e_del: int = 4
    o_ins: int = 1
    e_ins: int = 3
    b: int = 11

    @classmethod
    def finish(cls):
        return cls(min_seed_len=17, min_chain_weight=18, w=30, split_factor=1.5, drop_ratio=0.75,
                   o_del=15, e_del=3, o_ins=19, e_ins=3, b=13)


class Index:
    """Long reads (lists of codes 0-4) -> contig strings in bwa's forward-reverse order."""

    def __init__(self, lrs):
        self.lrs = [list(x) for x in lrs]
        self.n_lr = len(lrs)
        self.lr_off = [0]
        for x in self.lrs:
            self.lr_off.append(self.lr_off[-1] + len(x))
        self.l_pac = self.lr_off[-1]
        # text order: LR0..LRn-1 forward, then rc(LRn-1)..rc(LR0); chars 'ACGTN'
        self.contigs = ["".join("ACGTN"[c] for c in x) for x in self.lrs]
        self.contigs += ["".join("ACGTN"[COMP.get(c, 4)] for c in reversed(x)) for x in reversed(self.lrs)]

    def positions(self, s: str):
        """(contig, offset) of every occurrence of s (overlapping), contig-major."""
        out = []
        for ci, t in enumerate(self.contigs):
            p = t.find(s)
            while p >= 0:
                out.append((ci, p))
                p = t.find(s, p + 1)
        return out

    def occ(self, s: str) -> int:
        if "N" in s:
            return 0
        return len(self.positions(s))

    def fr(self, ci, off):
        """(forward-reverse coordinate, long read id) of a contig offset."""
        if ci < self.n_lr:
            return self.lr_off[ci] + off, ci
        rid = 2 * self.n_lr - 1 - ci
        return self.l_pac + (self.l_pac - self.lr_off[rid + 1]) + off, rid


def _qs(q, a, b):
    return "".join("ACGTN"[c] for c in q[a:b])


def smem1(I: Index, q, x, min_intv):
    """bwt_smem1a with max_intv = 0 -> (SMEMs [(start, end, occ)] sorted by start, next x)."""
    n = len(q)
    if q[x] > 3:
        return [], x + 1
    min_intv = max(min_intv, 1)
    occ = lambda a, b: I.occ(_qs(q, a, b))
    curr = []
    ik = (x, x + 1, occ(x, x + 1))
    i = x + 1
    broke = False
    while i < n:
        if q[i] < 4:
            o = occ(x, i + 1)
            if o != ik[2]:
                curr.append(ik)
                if o < min_intv:
                    broke = True
                    break
            ik = (x, i + 1, o)
        else:
            curr.append(ik)
            broke = True
            break
        i += 1
    if not broke:
        curr.append(ik)
    curr.reverse()
    ret = curr[0][1]
    prev = curr
    mem = []
    i = x - 1
    while i >= -1:
        c = -1 if i < 0 else (q[i] if q[i] < 4 else -1)
        curr = []
        for p in prev:
            o = occ(i, p[1]) if c >= 0 else 0
            if c < 0 or o < min_intv:
                if not curr and (not mem or i + 1 < mem[-1][0]):
                    mem.append((i + 1, p[1], p[2]))
            elif not curr or o != curr[-1][2]:
                curr.append((i, p[1], o))
        if not curr:
            break
        prev = curr
        i -= 1
    mem.reverse()
    return mem, ret


def seed_strategy1(I: Index, q, x, min_len, max_intv):
    n = len(q)
    if q[x] > 3:
        return None, x + 1
    for i in range(x + 1, n):
        if q[i] > 3:
            return None, i + 1
        if i - x >= min_len:
            o = I.occ(_qs(q, x, i + 1))
            if o < max_intv:
                return (x, i + 1, o), i + 1
    return None, n


def collect_intv(I: Index, O: Opts, q):
    n = len(q)
    mems = []
    x = 0
    while x < n:
        if q[x] < 4:
            m1, x = smem1(I, q, x, 1)
            mems += [m for m in m1 if m[1] - m[0] >= O.min_seed_len]
        else:
            x += 1
    split_len = int(O.min_seed_len * O.split_factor + .499)
    for p in list(mems):
        if p[1] - p[0] < split_len or p[2] > O.split_width:
            continue
        m1, _ = smem1(I, q, (p[0] + p[1]) >> 1, p[2] + 1)
        mems += [m for m in m1 if m[1] - m[0] >= O.min_seed_len]
    if O.max_mem_intv > 0:
        x = 0
        while x < n:
            if q[x] < 4:
                m, x = seed_strategy1(I, q, x, O.min_seed_len, O.max_mem_intv)
                if m is not None and m[2] > 0:
                    mems.append(m)
            else:
                x += 1
    mems.sort(key=lambda m: (m[0], m[1]))   # stable
    return mems


def _test_and_merge(O, l_pac, c, s, rid):
    last = c["seeds"][-1]
    qend, rend = last["qbeg"] + last["len"], last["rbeg"] + last["len"]
    if rid != c["rid"]:
        return False
    f = c["seeds"][0]
    if s["qbeg"] >= f["qbeg"] and s["qbeg"] + s["len"] <= qend and s["rbeg"] >= f["rbeg"] and s["rbeg"] + s["len"] <= rend:
        return True
    if (last["rbeg"] < l_pac or f["rbeg"] < l_pac) and s["rbeg"] >= l_pac:
        return False
    x, y = s["qbeg"] - last["qbeg"], s["rbeg"] - last["rbeg"]
    if y >= 0 and x - y <= O.w and y - x <= O.w and x - last["len"] < O.max_chain_gap and y - last["len"] < O.max_chain_gap:
        c["seeds"].append(s)
        return True
    return False


def _weight(c):
    def cov(key):
        end = w = 0
        for s in c["seeds"]:
            b = s[key]
            if b >= end:
                w += s["len"]
            elif b + s["len"] > end:
                w += b + s["len"] - end
            end = max(end, b + s["len"])
        return w
    return min(cov("qbeg"), cov("rbeg"), (1 << 30) - 1)


def _max_gap(O, qlen):
    l_del = int((qlen * O.a - O.o_del) / O.e_del + 1.)
    l_ins = int((qlen * O.a - O.o_ins) / O.e_ins + 1.)
    return min(max(l_del, l_ins, 1), O.w << 1)


def _f32(x: float) -> float:
    return struct.unpack("f", struct.pack("f", x))[0]


def flt_min_score(O: Opts, n: int):
    """mem_flt_chained_seeds' min_HSP_score for a read of n bases, or None when bwa skips the
    filter: min_l = MEM_HSP_COEF * W (1.1f, float arithmetic), skipped when min_l >
    MEM_SEEDSW_COEF * l_query (0.05f * n, float)."""
    if O.min_chain_weight:
        min_l = _f32(_f32(1.1) * O.min_chain_weight)
    else:
        min_l = _f32(5.5) * math.log(n)   # MEM_MINSC_COEF * log(l_query)
    if min_l > _f32(_f32(0.05) * n):
        return None
    return int(O.a * min_l + .499)


def _ref_base(I: Index, rid: int, p: int) -> int:
    """The base at forward-reverse coordinate p of long read rid (code 0-4)."""
    if p < I.l_pac:
        return "ACGTN".index(I.contigs[rid][p - I.lr_off[rid]])
    return "ACGTN".index(I.contigs[2 * I.n_lr - 1 - rid][p - (2 * I.l_pac - I.lr_off[rid + 1])])


def local_sw(O: Opts, q, t) -> int:
    """ksw_align2's score: best local alignment of query q against target t, a gap of k
    bases costing o + k e (deletions = target bases: o_del/e_del; insertions: o_ins/e_ins),
    match a, mismatch -b, N -1."""
    qn = len(q)
    H = [0] * qn
    E = [0] * qn
    best = 0
    for tb in t:
        hdiag = f = 0
        for j in range(qn):
            qb = q[j]
            sc = -1 if (tb > 3 or qb > 3) else (O.a if tb == qb else -O.b)
            e = E[j]
            h = max(hdiag + sc, e, f, 0)
            hdiag = H[j]
            H[j] = h
            best = max(best, h)
            E[j] = max(e - O.e_del, h - O.o_del - O.e_del, 0)
            f = max(f - O.e_ins, h - O.o_ins - O.e_ins, 0)
    return best


def seed_sw(I: Index, O: Opts, q, s, rid) -> int:
    """mem_seed_sw: the local score around seed s (+- MEM_SHORT_EXT = 50), or -1 when the seed
    or a window reaches MEM_SHORT_LEN = 200; the reference window is clamped to [0, 2 l_pac),
    the seed's strand half and (bns_fetch_seq) its long read."""
    n = len(q)
    if s["len"] >= 200:
        return -1
    qb, qe = max(s["qbeg"] - 50, 0), min(s["qbeg"] + s["len"] + 50, n)
    rb, re = s["rbeg"], s["rbeg"] + s["len"]
    mid = (rb + re) >> 1
    rb, re = max(rb - 50, 0), min(re + 50, 2 * I.l_pac)
    if rb < I.l_pac < re:
        if mid < I.l_pac:
            re = I.l_pac
        else:
            rb = I.l_pac
    if qe - qb >= 200 or re - rb >= 200:
        return -1
    if mid >= I.l_pac:
        fb, fe = 2 * I.l_pac - I.lr_off[rid + 1], 2 * I.l_pac - I.lr_off[rid]
    else:
        fb, fe = I.lr_off[rid], I.lr_off[rid + 1]
    rb, re = max(rb, fb), min(re, fe)
    return local_sw(O, q[qb:qe], [_ref_base(I, rid, p) for p in range(rb, re)])


def map_read(I: Index, O: Opts, q, sid=0):
    """Tasks of one read: dicts with the pr_seed_task fields."""
    n = len(q)
    chains = []   # sorted by pos (insertion after equal keys, like the library's multimap)
    keys = []
    for (a, b, _) in collect_intv(I, O, q):
        pos = I.positions(_qs(q, a, b))   # text order: contig-major, then offset
        npos = len(pos)
        step = npos // O.max_occ if npos > O.max_occ else 1
        k = count = 0
        while k < npos and count < O.max_occ:
            rbeg, rid = I.fr(*pos[k])
            s = {"rbeg": rbeg, "qbeg": a, "len": b - a}
            add = True
            j = bisect.bisect_right(keys, rbeg) - 1
            if j >= 0 and _test_and_merge(O, I.l_pac, chains[j], s, rid):
                add = False
            if add:
                j = bisect.bisect_right(keys, rbeg)
                keys.insert(j, rbeg)
                chains.insert(j, {"pos": rbeg, "rid": rid, "seeds": [s]})
            k += step
            count += 1
    for c in chains:
        c["w"] = _weight(c)
    chains = [c for c in chains if c["w"] >= O.min_chain_weight]
    chains.sort(key=lambda c: -c["w"])   # stable
    for c in chains:
        c["kept"], c["first"] = 0, -1
    if chains:
        beg = lambda c: c["seeds"][0]["qbeg"]
        end = lambda c: c["seeds"][-1]["qbeg"] + c["seeds"][-1]["len"]
        kept = [0]
        chains[0]["kept"] = 3
        for i in range(1, len(chains)):
            large = 0
            broke = False
            for j in kept:
                cj, ci = chains[j], chains[i]
                bmax, emin = max(beg(cj), beg(ci)), min(end(cj), end(ci))
                if emin > bmax:
                    minl = min(end(ci) - beg(ci), end(cj) - beg(cj))
                    if emin - bmax >= minl * O.mask_level and minl < O.max_chain_gap:
                        large = 1
                        if cj["first"] < 0:
                            cj["first"] = i
                        if ci["w"] < cj["w"] * O.drop_ratio and cj["w"] - ci["w"] >= O.min_seed_len << 1:
                            broke = True
                            break
            if not broke:
                kept.append(i)
                chains[i]["kept"] = 2 if large else 3
        for j in kept:
            if chains[j]["first"] >= 0:
                chains[chains[j]["first"]]["kept"] = 1
    out = []
    nk = 0
    flt = flt_min_score(O, n)
    for c in chains:
        if c["kept"] == 0:
            continue
        seeds = c["seeds"]
        scores = [t["len"] for t in seeds]
        if flt is not None:   # mem_flt_chained_seeds
            kept_s = []
            for t in seeds:
                x = seed_sw(I, O, q, t, c["rid"])
                if x < 0 or x >= flt:
                    kept_s.append((t, t["len"] * O.a if x < 0 else x))
            seeds = [x[0] for x in kept_s]
            scores = [x[1] for x in kept_s]
            if not seeds:   # mem_chain2aln returns on an empty chain
                continue
        rev = seeds[0]["rbeg"] >= I.l_pac
        rid = c["rid"]
        L = I.lr_off[rid + 1] - I.lr_off[rid]
        cs = I.l_pac + (I.l_pac - I.lr_off[rid + 1]) if rev else I.lr_off[rid]
        r0 = min(t["rbeg"] - (t["qbeg"] + _max_gap(O, t["qbeg"])) for t in seeds) - cs
        r1 = max(t["rbeg"] + t["len"] + ((n - t["qbeg"] - t["len"]) + _max_gap(O, n - t["qbeg"] - t["len"]))
                 for t in seeds) - cs
        # mem_chain2aln's srt order: (score, index) descending; score = length unless filtered
        order = sorted(range(len(seeds)), key=lambda i: (scores[i], i), reverse=True)
        for rank, i in enumerate(order):
            s = seeds[i]
            out.append(dict(sr=sid, lr=rid, strand=int(rev), qbeg=s["qbeg"], rbeg=s["rbeg"] - cs, slen=s["len"],
                            rmax0=max(r0, 0), rmax1=min(r1, L), chain=nk, rank=rank))
        nk += 1
    return out
