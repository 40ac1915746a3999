"""Synthetic proovread workloads generated with numpy.

A random genome (iid ACGT), long reads sampled from it with a PacBio-CLR-like
error process (insertions / deletions / substitutions), Illumina-like short
reads (150 bp, one substitution in ~15% of reads = 0.1%/base, random strand),
and the seed-extension task list.

The task list stands in for bwa-proovread's FM-index front end (SMEM seeding
and chaining, SURVEY.md §8f "next"): for every (short read, long read) pair
whose genome spans overlap, the seed is the longest exact match between them,
read off the simulation truth; pairs without an exact match of >= k bases get
no task (bwa would not seed them either).  Tasks are emitted grouped by long
read and, within a long read, by short-read genome position.
"""
from __future__ import annotations

import dataclasses

from typing import Optional

import numpy as np


@dataclasses.dataclass
class Dataset:
    genome: np.ndarray
    lr_seq: np.ndarray     # nt4 pool
    lr_off: np.ndarray     # int64 [n_lr+1]
    lr_start: np.ndarray   # genome start of each long read
    sr_seq: np.ndarray     # nt4 pool
    sr_off: np.ndarray
    sr_start: np.ndarray
    sr_strand: np.ndarray
    t_sr: np.ndarray
    t_lr: np.ndarray
    t_strand: np.ndarray
    t_qbeg: np.ndarray
    t_rbeg: np.ndarray
    t_slen: np.ndarray
    # bwa mode: tasks are every seed of the kept chains grouped by short read (pr_seed_map
    # order) and t_chain their chain; None: single-seed tasks grouped by long read
    t_chain: Optional[np.ndarray] = None

    @property
    def n_lr(self):
        return len(self.lr_off) - 1

    @property
    def n_sr(self):
        return len(self.sr_off) - 1

    def lr_str(self, i):
        return "".join("ACGTN"[x] for x in self.lr_seq[self.lr_off[i]:self.lr_off[i + 1]])

    def sr_str(self, i):
        return "".join("ACGTN"[x] for x in self.sr_seq[self.sr_off[i]:self.sr_off[i + 1]])

    def sw_input(self):
        from .sw import SwInput
        return SwInput(self.sr_off, self.sr_seq, self.lr_off, self.lr_seq, self.t_sr, self.t_lr, self.t_strand,
                       self.t_qbeg, self.t_rbeg, self.t_slen, self.t_chain)


def simulate(seed: int, genome_len: int, n_lr: int, lr_len: int, sr_cov: float,
             p_ins: float = 0.09, p_del: float = 0.045, p_sub: float = 0.015,
             sr_len: int = 150, k: int = 12, sr_frac: float = 1.0) -> Dataset:
    rng = np.random.default_rng(seed)
    genome = rng.integers(0, 4, genome_len, dtype=np.uint8)
    span = min(lr_len, genome_len)
    lr_start = np.sort(rng.integers(0, genome_len - span + 1, n_lr))
    lr_parts, lr_lens = [], []
    run_s, run_l, run_p, run_lr = [], [], [], []
    for i in range(n_lr):
        s = int(lr_start[i])
        g = genome[s:s + span]
        u = rng.random(span)
        deleted = u < p_del
        sub = (u >= p_del) & (u < p_del + p_sub)
        base = g.copy()
        ns = int(sub.sum())
        if ns:
            base[sub] = (g[sub] + rng.integers(1, 4, ns, dtype=np.uint8)) % 4
        ins = rng.geometric(1.0 - p_ins, span) - 1 if p_ins > 0 else np.zeros(span, np.int64)
        kept = ~deleted
        counts = kept.astype(np.int64) + ins
        starts = np.cumsum(counts) - counts
        out = rng.integers(0, 4, int(counts.sum()), dtype=np.uint8)
        out[starts[kept]] = base[kept]
        lr_parts.append(out)
        lr_lens.append(len(out))
        # maximal exact runs: ok bases linked without insertions in between
        ok = kept & ~sub
        link = np.zeros(span, bool)
        link[:-1] = ok[:-1] & ok[1:] & (ins[:-1] == 0)
        # run starts: ok[j] and not (link[j-1])
        prev_link = np.zeros(span, bool)
        prev_link[1:] = link[:-1]
        rstart = np.nonzero(ok & ~prev_link)[0]
        # run end: first j >= start with not link[j] -> length = j - start + 1
        brk = np.nonzero(~link)[0]
        rend = brk[np.searchsorted(brk, rstart)]
        rlen = rend - rstart + 1
        keep = rlen >= k
        run_s.append(rstart[keep] + s)
        run_l.append(rlen[keep])
        run_p.append(starts[rstart[keep]])
        run_lr.append(np.full(int(keep.sum()), i, np.int64))
    lr_off = np.zeros(n_lr + 1, np.int64)
    np.cumsum(lr_lens, out=lr_off[1:])
    lr_seq = np.concatenate(lr_parts) if lr_parts else np.zeros(0, np.uint8)
    run_s = np.concatenate(run_s)
    run_l = np.concatenate(run_l)
    run_p = np.concatenate(run_p)
    run_lr = np.concatenate(run_lr)
    lr_lens = np.asarray(lr_lens, np.int64)

    # short reads
    n_sr = int(round(sr_cov * genome_len / sr_len * sr_frac))
    sr_start = np.sort(rng.integers(0, genome_len - sr_len + 1, n_sr))
    sr_strand = rng.integers(0, 2, n_sr).astype(np.uint8)
    idx = sr_start[:, None] + np.arange(sr_len)[None, :]
    srs = genome[idx]
    has_sub = rng.random(n_sr) < (0.001 * sr_len)
    sub_pos = rng.integers(0, sr_len, n_sr)
    rows = np.nonzero(has_sub)[0]
    srs[rows, sub_pos[rows]] = (srs[rows, sub_pos[rows]] + rng.integers(1, 4, len(rows)).astype(np.uint8)) % 4
    rev = sr_strand == 1
    srs[rev] = (3 - srs[rev])[:, ::-1]
    sr_seq = srs.reshape(-1).astype(np.uint8)
    sr_off = np.arange(n_sr + 1, dtype=np.int64) * sr_len
    sub_g = np.where(has_sub, sr_start + sub_pos, -1)   # genome coordinate of the substitution

    # (SR, LR) pairs with overlapping genome spans; LRs sorted by start
    lo = np.searchsorted(lr_start, sr_start - span, side="right")
    hi = np.searchsorted(lr_start, sr_start + sr_len, side="left")
    cnt = np.maximum(hi - lo, 0)
    p_sr = np.repeat(np.arange(n_sr), cnt)
    p_lr = (np.repeat(lo, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))).astype(np.int64)
    a = sr_start[p_sr]
    b = a + sr_len
    # runs of each LR are contiguous and sorted; key = lr * BIG + genome pos
    BIG = np.int64(1) << 40
    rkey_end = run_lr * BIG + (run_s + run_l)
    rkey_start = run_lr * BIG + run_s
    r_lo = np.searchsorted(rkey_end, p_lr * BIG + a, side="right")
    r_hi = np.searchsorted(rkey_start, p_lr * BIG + b, side="left")
    best_len = np.zeros(len(p_sr), np.int64)
    best_g = np.zeros(len(p_sr), np.int64)
    best_r = np.full(len(p_sr), -1, np.int64)
    sg = sub_g[p_sr]
    for o in range(64):
        r = r_lo + o
        valid = r < r_hi
        if not valid.any():
            break
        rc = np.where(valid, r, 0)
        gs = np.maximum(run_s[rc], a)
        ge = np.minimum(run_s[rc] + run_l[rc], b)
        # a short-read substitution inside the overlap: keep the longer side
        inside = (sg >= gs) & (sg < ge)
        left_len = sg - gs
        right_len = ge - sg - 1
        use_right = inside & (right_len > left_len)
        gs2 = np.where(use_right, sg + 1, gs)
        ge2 = np.where(inside & ~use_right, sg, ge)
        ln = np.where(valid, ge2 - gs2, 0)
        better = ln > best_len
        best_len = np.where(better, ln, best_len)
        best_g = np.where(better, gs2, best_g)
        best_r = np.where(better, rc, best_r)
    ok = best_len >= k
    p_sr, p_lr, a, best_len, best_g, best_r = p_sr[ok], p_lr[ok], a[ok], best_len[ok], best_g[ok], best_r[ok]
    lrpos = run_p[best_r] + (best_g - run_s[best_r])
    strand = sr_strand[p_sr]
    L = lr_lens[p_lr]
    qbeg = np.where(strand == 1, (a + sr_len) - (best_g + best_len), best_g - a)
    rbeg = np.where(strand == 1, L - (lrpos + best_len), lrpos)
    # group tasks by long read, then by short-read position
    order = np.lexsort((a, p_lr))
    return Dataset(genome, lr_seq, lr_off, lr_start, sr_seq, sr_off, sr_start, sr_strand,
                   p_sr[order].astype(np.int32), p_lr[order].astype(np.int32), strand[order].astype(np.uint8),
                   qbeg[order].astype(np.int32), rbeg[order].astype(np.int32), best_len[order].astype(np.int32))


_SYNTH = None


def _synth_lib():
    """libprsynth.so (csrc/synth.c, built by build.py next to libprgpu.so): the host-thread
    generator behind simulate_reads."""
    global _SYNTH
    if _SYNTH is None:
        import ctypes as C
        from pathlib import Path
        p = Path(__file__).resolve().parent / "libprsynth.so"
        if not p.exists():
            raise RuntimeError(f"{p} not found: run __graft_entry__.build()")
        L = C.CDLL(str(p))
        P64, PU8 = C.POINTER(C.c_int64), C.POINTER(C.c_uint8)
        L.prs_genome.argtypes = [C.c_uint64, C.c_int64, PU8]
        L.prs_long_reads.argtypes = [PU8, P64, C.c_int64, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_uint64,
                                     C.c_int, P64, P64, PU8]
        L.prs_short_reads.argtypes = [PU8, P64, PU8, C.c_int64, C.c_int64, C.c_double, C.c_uint64, C.c_int, PU8]
        _SYNTH = L
    return _SYNTH


def simulate_reads(seed: int, genome_len: int, n_lr: int, lr_len: int, n_sr: int, p_ins: float = 0.09,
                   p_del: float = 0.045, p_sub: float = 0.015, sr_len: int = 150, threads: int = 16) -> Dataset:
    """The reads of simulate()'s model at BASELINE configs[2] / configs[3] scale (SURVEY.md §8d
    C3 / C4: 100 k / 270 k x 10 kb long reads), generated on host threads (libprsynth.so),
    without the simulation-truth task list (the product's seeding front end makes the tasks).
    n_sr short reads in sequencer order -- unsorted over the genome, as a FASTQ from a
    sequencing run is, so contiguous short-read shards hit every part of the long-read set.
    Deterministic for a seed whatever the thread count."""
    import ctypes as C
    L = _synth_lib()
    P64, PU8 = C.POINTER(C.c_int64), C.POINTER(C.c_uint8)
    seed = int(seed) & (2 ** 64 - 1)
    genome = np.empty(genome_len, np.uint8)
    L.prs_genome(seed, genome_len, genome.ctypes.data_as(PU8))
    span = min(lr_len, genome_len)
    rp = np.random.default_rng(seed)
    lr_start = np.ascontiguousarray(np.sort(rp.integers(0, genome_len - span + 1, n_lr)), np.int64)
    sr_start = np.ascontiguousarray(rp.integers(0, genome_len - sr_len + 1, n_sr), np.int64)
    sr_strand = np.ascontiguousarray(rp.integers(0, 2, n_sr), np.uint8)
    gp = genome.ctypes.data_as(PU8)
    lens = np.zeros(max(n_lr, 1), np.int64)
    if L.prs_long_reads(gp, lr_start.ctypes.data_as(P64), n_lr, span, p_ins, p_del, p_sub, seed, threads,
                        lens.ctypes.data_as(P64), None, None):
        raise RuntimeError("prs_long_reads failed")
    lr_off = np.zeros(n_lr + 1, np.int64)
    np.cumsum(lens[:n_lr], out=lr_off[1:])
    lr_seq = np.empty(int(lr_off[-1]) + 1, np.uint8)
    if L.prs_long_reads(gp, lr_start.ctypes.data_as(P64), n_lr, span, p_ins, p_del, p_sub, seed, threads,
                        lens.ctypes.data_as(P64), lr_off.ctypes.data_as(P64), lr_seq.ctypes.data_as(PU8)):
        raise RuntimeError("prs_long_reads failed")
    sr_seq = np.empty(n_sr * sr_len + 1, np.uint8)
    if L.prs_short_reads(gp, sr_start.ctypes.data_as(P64), sr_strand.ctypes.data_as(PU8), n_sr, sr_len,
                         0.001 * sr_len, seed, threads, sr_seq.ctypes.data_as(PU8)):
        raise RuntimeError("prs_short_reads failed")
    sr_off = np.arange(n_sr + 1, dtype=np.int64) * sr_len
    z32, z8 = np.zeros(0, np.int32), np.zeros(0, np.uint8)
    return Dataset(genome, lr_seq[:-1], lr_off, lr_start, sr_seq[:-1], sr_off, sr_start, sr_strand, z32, z32, z8, z32,
                   z32, z32)


def with_seeds(d: Dataset, tasks: np.ndarray) -> Dataset:
    """The same reads with the seeding front end's output (seed.TASK_DTYPE records of
    pr_seed_map / pr_seed_gpu_map: every seed of the kept chains, grouped by short read, then
    chain, in mem_chain2aln's order) as a bwa-mode task list."""
    t = tasks
    return dataclasses.replace(d, t_sr=t["sr"].astype(np.int32), t_lr=t["lr"].astype(np.int32),
                               t_strand=t["strand"].astype(np.uint8), t_qbeg=t["qbeg"].astype(np.int32),
                               t_rbeg=t["rbeg"].astype(np.int32), t_slen=t["slen"].astype(np.int32),
                               t_chain=t["chain"].astype(np.int32))


def with_seeded_tasks(d: Dataset, tasks: np.ndarray) -> Dataset:
    """The same reads with the task list of the seeding front end (seed.TASK_DTYPE records,
    pr_seed_map / pr_seed_gpu_map) in place of the simulation truth: grouped by long read
    (stable, so a long read's tasks stay in read order, then chain order) as the iteration
    hand-off expects."""
    order = np.argsort(tasks["lr"], kind="stable")
    t = tasks[order]
    return dataclasses.replace(d, t_sr=t["sr"].astype(np.int32), t_lr=t["lr"].astype(np.int32),
                               t_strand=t["strand"].astype(np.uint8), t_qbeg=t["qbeg"].astype(np.int32),
                               t_rbeg=t["rbeg"].astype(np.int32), t_slen=t["slen"].astype(np.int32))
