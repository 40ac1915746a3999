// bwa mode's per-read logic (mem_chain2aln's walk, mem_sort_dedup_patch .. mem_reg2sam,
// mem_patch_reg's global score): one implementation for the device kernels
// (aln_kernels.hip, one lane per read) and the host build of the CPU tests
// (tests/native/aln_host.cpp).  Restated from upstream bwa (>= 0.7.13) bwamem.c, klib
// ksort.h's ks_introsort and bwa.c bwa_gen_cigar2 / ksw.c ksw_global2; bwa-proovread is an
// absent submodule (.gitmodules:4-6), parity unpinned.
#pragma once
#include <stdint.h>

#include "aln_dev.h"

#if defined(__HIPCC__)
#define AL_HD __host__ __device__ inline
#else
#define AL_HD inline
#endif

namespace prgpu {
namespace alnc {

AL_HD int cal_max_gap_a(const AlnDev &A, int qlen) {
    int l_del = (int)((double)(qlen * A.a - A.o_del) / A.e_del + 1.);
    int l_ins = (int)((double)(qlen * A.a - A.o_ins) / A.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < A.w << 1 ? l : A.w << 1;
}

AL_HD int64_t fr_of(const AlnDev &A, int lr, int strand, int64_t x) {
    const int64_t l_pac = A.lr_off[A.n_lr];
    return strand ? l_pac + (l_pac - A.lr_off[lr + 1]) + x : A.lr_off[lr] + x;
}

AL_HD uint64_t hash_64(uint64_t key) {
    key += ~(key << 32);
    key ^= (key >> 22);
    key += ~(key << 13);
    key ^= (key >> 8);
    key += (key << 3);
    key ^= (key >> 15);
    key += ~(key << 27);
    key ^= (key >> 31);
    return key;
}

// ---------------------------------------------------------------- klib ks_introsort
// over an index array into the read's regions (the permutation klib's element moves make)
struct LtEnd {   // alnreg_slt2 (mem_ars2)
    template <class Reg>
    AL_HD bool operator()(const Reg &a, const Reg &b) const { return a.re < b.re; }
};
struct LtScore {   // alnreg_slt (mem_ars)
    template <class Reg>
    AL_HD bool operator()(const Reg &a, const Reg &b) const {
        return a.score > b.score || (a.score == b.score && (a.rb < b.rb || (a.rb == b.rb && a.qb < b.qb)));
    }
};
struct LtHash {   // alnreg_hlt (mem_ars_hash)
    template <class Reg>
    AL_HD bool operator()(const Reg &a, const Reg &b) const {
        return a.score > b.score || (a.score == b.score && a.hash < b.hash);
    }
};

// klib ks_introsort (ksort.h as vendored by bwa) over an index array into the read's
// regions, written with integer positions (the permutation klib's element moves make)
template <class Lt, class Reg>
AL_HD void insertsort(int32_t *a, int s, int t, const Reg *R, Lt lt) {   // [s, t)
    for (int i = s + 1; i < t; ++i)
        for (int j = i; j > s && lt(R[a[j]], R[a[j - 1]]); --j) {
            const int32_t x = a[j];
            a[j] = a[j - 1];
            a[j - 1] = x;
        }
}
template <class Lt, class Reg>
AL_HD void combsort(int32_t *a, int s, int n, const Reg *R, Lt lt) {   // [s, s + n)
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    int gap = n;
    do {
        if (gap > 2) {
            gap = (int)((double)gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (int i = s; i < s + n - gap; ++i) {
            const int j = i + gap;
            if (lt(R[a[j]], R[a[i]])) {
                const int32_t x = a[i];
                a[i] = a[j];
                a[j] = x;
                do_swap = 1;
            }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) insertsort(a, s, s + n, R, lt);
}
template <class Lt, class Reg>
AL_HD void introsort(int n, int32_t *a, const Reg *R, Lt lt) {
    int st_l[64], st_r[64], st_d[64];
    int top = 0, d;
    if (n < 1) return;
    if (n == 2) {
        if (lt(R[a[1]], R[a[0]])) {
            const int32_t x = a[0];
            a[0] = a[1];
            a[1] = x;
        }
        return;
    }
    for (d = 2; (1ll << d) < n; ++d) {}
    int s = 0, t = n - 1;
    d <<= 1;
    for (;;) {
        if (s < t) {
            if (--d == 0) {
                combsort(a, s, t - s + 1, R, lt);
                t = s;
                continue;
            }
            int i = s, j = t, k = i + ((j - i) >> 1) + 1;
            if (lt(R[a[k]], R[a[i]])) {
                if (lt(R[a[k]], R[a[j]])) k = j;
            } else {
                k = lt(R[a[j]], R[a[i]]) ? i : j;
            }
            const int32_t rp = a[k];
            if (k != t) {
                a[k] = a[t];
                a[t] = rp;
            }
            for (;;) {
                do ++i; while (lt(R[a[i]], R[rp]));
                do --j; while (i <= j && lt(R[rp], R[a[j]]));
                if (j <= i) break;
                const int32_t x = a[i];
                a[i] = a[j];
                a[j] = x;
            }
            {
                const int32_t x = a[i];
                a[i] = a[t];
                a[t] = x;
            }
            if (i - s > t - i) {
                if (i - s > 16) {
                    st_l[top] = s;
                    st_r[top] = i - 1;
                    st_d[top] = d;
                    ++top;
                }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) {
                    st_l[top] = i + 1;
                    st_r[top] = t;
                    st_d[top] = d;
                    ++top;
                }
                t = i - s > 16 ? s : i - 1;
            }
        } else {
            if (top == 0) {
                insertsort(a, 0, n, R, lt);
                return;
            }
            --top;
            s = st_l[top];
            t = st_r[top];
            d = st_d[top];
        }
    }
}

// round-0 state of task t: every chain's first seed is extended speculatively; cnext[t] of
// a chain's first seed = the next chain's first seed (chains are consecutive)
AL_HD bool aln_init_task(const AlnDev &A, int64_t t) {
    const bool first = t == 0 || A.t_sr[t] != A.t_sr[t - 1] || A.t_chain[t] != A.t_chain[t - 1];
    A.sel[t] = first ? SEL_EXT : 0;
    A.ext[t] = 0;
    A.dec[t] = 0;
    if (first && !A.cnext_ready) {
        int64_t e = t + 1;
        while (e < A.n_task && A.t_sr[e] == A.t_sr[t] && A.t_chain[e] == A.t_chain[t]) ++e;
        A.cnext[t] = (int32_t)e;
    }
    return first;
}

// hprev of every chain head of read r: the closest earlier head of the read on the same long
// read and strand (-1: none).  A short read's chains lie on ~one long read each, so the walk's
// containment test then visits the few chains that can contain a seed instead of every earlier
// chain head (a dependent cnext chase per head).  The heads met so far and their keys sit in
// the read's own ix / R scratch (contiguous per lane; the final pass rewrites both).
AL_HD void aln_heads_read(const AlnDev &A, int64_t r) {
    const int64_t s0 = A.seed_off[r], s1 = A.seed_off[r + 1];
    int32_t *hl = A.ix + s0;
    int32_t *hk = reinterpret_cast<int32_t *>(A.R + s0);   // 16 ints per task of room
    int nh = 0;
    for (int64_t h = s0; h < s1; h = A.cnext[h]) {
        const int32_t key = A.t_lr[h] * 2 + (A.t_strand[h] ? 1 : 0);
        int32_t p = -1;
        for (int j = nh - 1; j >= 0; --j)
            if (hk[j] == key) {
                p = hl[j];
                break;
            }
        A.hprev[h] = p;
        hl[nh] = (int32_t)h;
        hk[nh] = key;
        ++nh;
    }
}

// is a seed (srb, sqb, slen) "around" the region (pqb, pqe, prb, pre) extended from a seed of
// length pslen with band pw (mem_chain2aln's containment test)
AL_HD bool around_f(const AlnDev &A, int pqb, int pqe, int64_t prb, int64_t pre, int pslen, int pw, int64_t srb,
                    int sqb, int slen, int lq) {
    if (srb < prb || srb + slen > pre || sqb < pqb || sqb + slen > pqe) return false;   // not contained
    if ((double)(slen - pslen) > .1 * lq) return false;   // may give a better alignment
    int64_t qd = sqb - pqb, rd = srb - prb;
    int mg = cal_max_gap_a(A, (int)(qd < rd ? qd : rd));
    int w = mg < pw ? mg : pw;
    if (qd - rd < w && rd - qd < w) return true;
    qd = pqe - (sqb + slen);
    rd = pre - (srb + slen);
    mg = cal_max_gap_a(A, (int)(qd < rd ? qd : rd));
    w = mg < pw ? mg : pw;
    return qd - rd < w && rd - qd < w;
}

// is seed (slr, sst, srb, sqb, slen) "around" region i?
AL_HD bool aln_around(const AlnDev &A, int64_t i, int64_t srb, int sqb, int slen, int lq) {
    AlnBox bx;
    if (A.box) bx = A.box[i];
    else bx = AlnBox{A.o_qb[i], A.o_qe[i], A.o_rb[i], A.o_re[i], A.t_slen[i], A.o_w[i], 0, 0};
    return around_f(A, bx.qb, bx.qe, bx.rb, bx.re, bx.slen, bx.w, srb, sqb, slen, lq);
}

// mem_chain2aln's exception for a seed (srb, sqb, slen) inside a region: an earlier seed of its
// chain (tr, tq, tl), >= 95 % of its length, overlapping it on the query on another diagonal
AL_HD bool other_diag(int64_t srb, int sqb, int slen, int64_t tr, int tq, int tl) {
    if (tl < slen * .95) return false;
    if (sqb <= tq && sqb + slen - tq >= slen >> 2 && (int64_t)(tq - sqb) != tr - srb) return true;
    return tq <= sqb && tq + tl - sqb >= slen >> 2 && (int64_t)(sqb - tq) != srb - tr;
}

// any region made before seed k (dec == 1) that seed k is around?  Regions on another long
// read or strand never contain it (disjoint in bwa's coordinates), so after k's own chain
// [c0, k) only the earlier chains on k's long read and strand are looked at (their first
// seeds carry the chain's long read, strand and end).  "Exists" is order-free.
AL_HD bool aln_around_any(const AlnDev &A, int64_t s0, int64_t c0, int64_t k, int lq) {
    const int slr = A.t_lr[k], sst = A.t_strand[k];
    const int64_t srb = A.t_rbeg[k];
    const int sqb = A.t_qbeg[k], slen = A.t_slen[k];
    for (int64_t i = c0; i < k; ++i)
        if (A.dec[i] == 1 && aln_around(A, i, srb, sqb, slen, lq)) return true;
    if (A.hprev) {   // only the earlier chains on k's long read and strand (aln_heads_read's links)
        for (int64_t h = A.hprev[c0]; h >= 0; h = A.hprev[h])
            for (int64_t i = h; i < A.cnext[h]; ++i)
                if (A.dec[i] == 1 && aln_around(A, i, srb, sqb, slen, lq)) return true;
        return false;
    }
    for (int64_t h = s0; h < c0; h = A.cnext[h]) {
        if (A.t_lr[h] != slr || A.t_strand[h] != sst) continue;
        for (int64_t i = h; i < A.cnext[h]; ++i)
            if (A.dec[i] == 1 && aln_around(A, i, srb, sqb, slen, lq)) return true;
    }
    return false;
}

// could mem_chain2aln's "longer seed on another diagonal" exception apply to seed k later: a
// chain mate j in [c0, k) not skipped (dec != 2), >= 95 % of k's length, overlapping k on the
// query on another diagonal (the walk's own test, for mates whose region is not known yet)
AL_HD bool aln_maybe_other(const AlnDev &A, int64_t c0, int64_t k) {
    const int64_t srb = A.t_rbeg[k];
    const int sqb = A.t_qbeg[k], slen = A.t_slen[k];
    for (int64_t j = c0; j < k; ++j) {
        if (A.dec[j] == 2) continue;
        if (other_diag(srb, sqb, slen, A.t_rbeg[j], A.t_qbeg[j], A.t_slen[j])) return true;
    }
    return false;
}

// mem_chain2aln for read r, resumed at its first open seed.  A seed to extend whose result
// is not there stops the walk (decisions before it are final: they only depend on earlier
// seeds); the later open seeds that are around no region yet are requested with it
// (speculation: an extension result only ever replaces a kernel launch, the walk still
// decides).  push(t) lists a requested seed; -> the number requested.
template <class Push>
AL_HD int aln_walk_read(const AlnDev &A, int64_t r, Push push) {
    const int64_t s0 = A.seed_off[r], s1 = A.seed_off[r + 1];
    int64_t k = A.resume[r];
    if (k >= s1) return 0;
    // results of the last extension round (the flags read 8 at a time: independent loads)
    for (int64_t j0 = s0; j0 < s1; j0 += 8) {
        uint8_t f[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) f[u] = j0 + u < s1 ? A.sel[j0 + u] : (uint8_t)0;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t j = j0 + u;
            if (!(f[u] & SEL_EXT)) continue;
            A.ext[j] = 1;
            A.sel[j] = 0;
            if (A.box)
                A.box[j] = AlnBox{A.o_qb[j], A.o_qe[j], A.o_rb[j], A.o_re[j], A.t_slen[j], A.o_w[j], A.t_qbeg[j],
                                  A.t_rbeg[j]};
        }
    }
    const int lq = (int)(A.sr_off[r + 1] - A.sr_off[r]);
    int64_t c0 = k;   // first seed of k's chain
    while (c0 > s0 && A.t_chain[c0 - 1] == A.t_chain[k]) --c0;
    for (; k < s1; ++k) {
        if (k > s0 && A.t_chain[k] != A.t_chain[k - 1]) c0 = k;
        if (A.dec[k]) continue;
        const int64_t srb = A.t_rbeg[k];
        const int sqb = A.t_qbeg[k], slen = A.t_slen[k];
        if (aln_around_any(A, s0, c0, k, lq)) {
            bool other = false;   // a longer extended seed of the chain overlapping on another diagonal
            for (int64_t j = c0; j < k; ++j) {
                if (A.dec[j] != 1) continue;
                int tl, tq;
                int64_t tr;
                if (A.box) {
                    const AlnBox bj = A.box[j];
                    tl = bj.slen, tq = bj.tq, tr = bj.tr;
                } else {
                    tl = A.t_slen[j], tq = A.t_qbeg[j], tr = A.t_rbeg[j];
                }
                if (other_diag(srb, sqb, slen, tr, tq, tl)) { other = true; break; }
            }
            if (!other) {
                A.dec[k] = 2;
                continue;
            }
        }
        if (!A.ext[k]) {   // extension needed: request it (and the likely ones after it), resume here
            A.sel[k] = SEL_EXT;
            push(k);
            int n = 1;
            int64_t cc = c0;
            for (int64_t kk = k + 1; kk < s1; ++kk) {
                if (A.t_chain[kk] != A.t_chain[kk - 1]) cc = kk;
                if (A.dec[kk] || A.ext[kk] || (A.sel[kk] & SEL_EXT)) continue;
                // a seed inside a region is still extended when a longer (>= 95 %) seed of its
                // chain overlaps it on another diagonal; that seed's region may not exist yet,
                // so any such chain mate that is not skipped makes the seed speculated too
                // (saves the late rounds those seeds would each cost)
                if (aln_around_any(A, s0, cc, kk, lq) && !aln_maybe_other(A, cc, kk)) continue;
                A.sel[kk] = SEL_EXT;
                push(kk);
                ++n;
            }
            A.resume[r] = (int32_t)k;
            return n;
        }
        A.dec[k] = 1;
    }
    A.resume[r] = (int32_t)s1;
    return 0;
}

// mem_sort_dedup_patch's redundancy test and colinear merges (mem_patch_reg) over the regions
// sorted by end (ix): -> 1 when a patch's global score is not known yet (*req filled; the read
// is replayed once it is), 0 done
template <class Reg>
AL_HD int dedup_patch(const AlnDev &A, int64_t r, int64_t s0, Reg *R, const int32_t *ix, int n, AlnPatch *req) {
    const int64_t l_pac = A.lr_off[A.n_lr];
    int m_patch = 0;
    for (int i = 1; i < n; ++i) {
        Reg &p = R[ix[i]];
        const Reg &pv = R[ix[i - 1]];
        if (p.lr != pv.lr || p.rb >= pv.re + A.max_chain_gap) continue;
        for (int j = i - 1; j >= 0 && p.lr == R[ix[j]].lr && p.rb < R[ix[j]].re + A.max_chain_gap; --j) {
            Reg &q = R[ix[j]];
            if (q.qe == q.qb) continue;   // excluded
            const int64_t orr = q.re - p.rb;
            const int64_t oq = q.qb < p.qb ? q.qe - p.qb : p.qe - q.qb;
            const int64_t mr = q.re - q.rb < p.re - p.rb ? q.re - q.rb : p.re - p.rb;
            const int64_t mq = q.qe - q.qb < p.qe - p.qb ? q.qe - q.qb : p.qe - p.qb;
            if (orr > A.mask_level_redun * mr && oq > A.mask_level_redun * mq) {   // one is redundant
                if (p.score < q.score) {
                    p.qe = p.qb;
                    break;
                }
                q.qe = q.qb;
                continue;
            }
            if (!(q.rb < p.rb)) continue;
            // mem_patch_reg(q, p)
            if (q.rb < l_pac && p.rb >= l_pac) continue;   // different strands
            if (q.qb >= p.qb || q.qe >= p.qe || q.re >= p.re) continue;   // not colinear
            int w = (int)((q.re - p.rb) - (q.qe - p.qb));
            w = w > 0 ? w : -w;
            double rr = (double)(q.re - p.rb) / (double)(p.re - q.rb) - (double)(q.qe - p.qb) / (double)(p.qe - q.qb);
            rr = rr > 0. ? rr : -rr;
            if (q.re < p.rb || q.qe < p.qb) {
                if (w > A.w << 1 || rr >= 0.05) continue;
            } else if (w > A.w << 2 || rr >= 0.05 * 2) {
                continue;
            }
            w += q.w + p.w;
            w = w < A.w << 2 ? w : A.w << 2;
            int score;
            if (m_patch < A.npk[r]) {
                score = A.pscore[s0 + m_patch];
            } else {   // the global score is not known yet: request it, replay the read later
                const int64_t base = fr_of(A, q.lr, q.strand, 0);
                req->read = (int32_t)r;
                req->m = m_patch;
                req->lr = q.lr;
                req->strand = q.strand;
                req->qb = q.qb;
                req->qe = p.qe;
                req->rb = (int32_t)(q.rb - base);
                req->re = (int32_t)(p.re - base);
                req->w = w;
                req->pad = 0;
                return 1;
            }
            ++m_patch;
            const int q_s = (int)((double)(p.qe - q.qb) / ((p.qe - p.qb) + (q.qe - q.qb)) * (p.score + q.score) + .5);
            const int r_s = (int)((double)(p.re - q.rb) / (double)((p.re - p.rb) + (q.re - q.rb)) * (p.score + q.score) + .5);
            if (score <= 0 || (double)score / (q_s > r_s ? q_s : r_s) < 0.90) continue;
            p.qb = q.qb, p.rb = q.rb;
            p.truesc = p.score = score;
            p.w = w;
            p.patched = 1;
            q.qb = q.qe;
        }
    }
    return 0;
}

// the regions left (qe > qb), in place -> their count
template <class Reg>
AL_HD int compact_live(int n, int32_t *ix, const Reg *R) {
    int m = 0;
    for (int i = 0; i < n; ++i)
        if (R[ix[i]].qe > R[ix[i]].qb) ix[m++] = ix[i];
    return m;
}

// after the (score, rb, qb) sort: identical hits after the first removed -> the regions left
template <class Reg>
AL_HD int drop_identical(int n, int32_t *ix, Reg *R) {
    for (int i = 1; i < n; ++i) {
        Reg &a = R[ix[i]];
        const Reg &b = R[ix[i - 1]];
        if (a.score == b.score && a.rb == b.rb && a.qb == b.qb) a.qe = a.qb;
    }
    int m = n > 0 ? 1 : 0;
    for (int i = 1; i < n; ++i)
        if (R[ix[i]].qe > R[ix[i]].qb) ix[m++] = ix[i];
    return m;
}

// the final pass of read r -> 0 done, 1: the global score of patch *req is needed first
AL_HD int aln_final_read(const AlnDev &A, int64_t r, AlnPatch *req) {
    if (A.fdone[r]) return 0;
    const int64_t s0 = A.seed_off[r], s1 = A.seed_off[r + 1];
    AlnReg *R = A.R + s0;
    int32_t *ix = A.ix + s0;
    int n = 0;
    for (int64_t t0 = s0; t0 < s1; t0 += 8) {   // the decisions read 8 at a time (independent loads)
      uint8_t dv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) dv[u] = t0 + u < s1 ? A.dec[t0 + u] : (uint8_t)0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t t = t0 + u;
        if (dv[u] != 1) continue;
        AlnReg &g = R[n];
        const int lr = A.t_lr[t], st = A.t_strand[t];
        const int64_t base = fr_of(A, lr, st, 0);
        g.rb = base + A.o_rb[t];
        g.re = base + A.o_re[t];
        g.qb = A.o_qb[t];
        g.qe = A.o_qe[t];
        g.score = A.o_score[t];
        g.truesc = A.o_truesc[t];
        g.w = A.o_w[t];
        g.seedlen0 = A.t_slen[t];
        g.lr = lr;
        g.strand = st;
        g.task = (int32_t)t;
        g.secondary = -1;
        g.patched = 0;
        ix[n] = n;
        ++n;
      }
    }
    if (n > 1) {
        introsort(n, ix, R, LtEnd());
        if (dedup_patch(A, r, s0, R, ix, n, req)) return 1;
        n = compact_live(n, ix, R);
        introsort(n, ix, R, LtScore());
        n = drop_identical(n, ix, R);
    }
    // mem_mark_primary_se
    for (int i = 0; i < n; ++i) R[ix[i]].hash = hash_64((uint64_t)(A.read_id0 + r + i));
    introsort(n, ix, R, LtHash());
    // secondaries: a region overlapping an earlier primary (z of mem_mark_primary_se_core)
    for (int i = 0; i < n; ++i) R[ix[i]].secondary = -1;
    for (int i = 1; i < n; ++i) {
        AlnReg &ai = R[ix[i]];
        for (int j = 0; j < i; ++j) {   // the primaries before i, in order (z of mem_mark_primary_se_core)
            const AlnReg &aj = R[ix[j]];
            if (aj.secondary >= 0) continue;
            const int b_max = aj.qb > ai.qb ? aj.qb : ai.qb;
            const int e_min = aj.qe < ai.qe ? aj.qe : ai.qe;
            if (e_min > b_max) {
                const int min_l = ai.qe - ai.qb < aj.qe - aj.qb ? ai.qe - ai.qb : aj.qe - aj.qb;
                if (e_min - b_max >= min_l * A.mask_level) {
                    ai.secondary = j;
                    break;
                }
            }
        }
    }
    // mem_reg2sam: -T per aligned base, -D for secondaries; SAM order; mark for the CIGAR pass
    for (int64_t t = s0; t < s1; ++t) {
        A.sel[t] = 0;
        A.o_pass[t] = 0;
    }
    int no = 0;
    for (int k = 0; k < n; ++k) {
        const AlnReg &p = R[ix[k]];
        if (!((double)p.score >= A.min_score_per_base * (double)(p.qe - p.qb))) continue;
        if (p.secondary >= 0 && p.score < R[ix[p.secondary]].score * A.drop_ratio) continue;
        const int t = p.task;
        const int64_t base = fr_of(A, p.lr, p.strand, 0);
        A.o_qb[t] = p.qb;
        A.o_rb[t] = (int32_t)(p.rb - base);
        A.o_score[t] = p.score;
        A.o_truesc[t] = p.truesc;
        A.o_w[t] = p.w;
        A.o_pass[t] = 1;
        A.sel[t] = SEL_CIG;
        A.olist[s0 + no] = t;
        A.oflag[s0 + no] = (p.strand ? 0x10 : 0) | (p.secondary >= 0 ? 0x100 : (no > 0 ? 0x800 : 0));
        ++no;
    }
    A.nout[r] = no;
    A.fdone[r] = 1;
    return 0;
}

// bwa_gen_cigar2 (score only) of patch P with the H/E row in pool[0, 2 * stride)
AL_HD int aln_patch_score(const AlnDev &A, const AlnPatch &P, int32_t *pool, int64_t stride) {
    const int r = P.read;
    const uint8_t *Q = A.sr + A.sr_off[r] + P.qb;
    const int lq = P.qe - P.qb;
    const uint8_t *Lr = A.lr + A.lr_off[P.lr];
    const int L = (int)(A.lr_off[P.lr + 1] - A.lr_off[P.lr]);
    const int rlen = P.re - P.rb;
    int score = 0;
    auto qb_at = [&](int j) -> int {   // query, reversed on the reverse strand (indels leftmost)
        return P.strand ? Q[lq - 1 - j] : Q[j];
    };
    auto rf_at = [&](int i) -> int {   // strand reference [rb, re), reversed on the reverse strand
        const int x = P.strand ? P.re - 1 - i : P.rb + i;   // strand coordinate
        if (!P.strand) return Lr[x];
        const int c = Lr[L - 1 - x];
        return c < 4 ? 3 - c : c;
    };
    auto sc = [&](int tb, int qb) -> int { return (tb > 3 || qb > 3) ? -1 : (tb == qb ? A.a : -A.b); };
    if (lq > 0 && rlen > 0) {
        if (lq == rlen && P.w == 0) {
            for (int i = 0; i < lq; ++i) score += sc(rf_at(i), qb_at(i));
        } else {
            const int mn = lq < rlen ? lq : rlen;
            const int max_ins = (int)((double)(mn * A.a - A.o_ins) / A.e_ins + 1.);
            const int max_del = (int)((double)(mn * A.a - A.o_del) / A.e_del + 1.);
            int max_gap = max_ins > max_del ? max_ins : max_del;
            max_gap = max_gap > 1 ? max_gap : 1;
            const int dl = rlen > lq ? rlen - lq : lq - rlen;
            int w = (max_gap + dl + 1) >> 1;
            w = w < P.w ? w : P.w;
            w = w > dl + 3 ? w : dl + 3;
            // ksw_global2, score path
            constexpr int NEG = -0x40000000;
            int32_t *H = pool, *E = pool + (stride >> 1);
            const int oe_del = A.o_del + A.e_del, oe_ins = A.o_ins + A.e_ins;
            H[0] = 0;
            E[0] = NEG;
            int j;
            for (j = 1; j <= lq && j <= w; ++j) H[j] = -(A.o_ins + A.e_ins * j), E[j] = NEG;
            for (; j <= lq; ++j) H[j] = E[j] = NEG;
            for (int i = 0; i < rlen; ++i) {
                int f = NEG, h1;
                const int beg = i > w ? i - w : 0;
                const int end = i + w + 1 < lq ? i + w + 1 : lq;
                h1 = beg == 0 ? -(A.o_del + A.e_del * (i + 1)) : NEG;
                const int tb = rf_at(i);
                for (j = beg; j < end; ++j) {
                    int mm = H[j], e = E[j];
                    H[j] = h1;
                    mm += sc(tb, qb_at(j));
                    int h = mm >= e ? mm : e;
                    h = h >= f ? h : f;
                    h1 = h;
                    int tt = mm - oe_del;
                    e -= A.e_del;
                    e = e > tt ? e : tt;
                    E[j] = e;
                    tt = mm - oe_ins;
                    f -= A.e_ins;
                    f = f > tt ? f : tt;
                }
                H[end] = h1;
                E[end] = NEG;
            }
            score = H[lq];
        }
    }
    return score;
}

}  // namespace alnc
}  // namespace prgpu
