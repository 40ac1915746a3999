// ksw_extend2 with the DP row in a register ring (device code, also compiled
// for the host by tests/native/ring_host.cpp to check it against the oracle).
#pragma once
#include <stdint.h>

#include "sw_dev.h"

#ifndef SW_RING_HOST
#define SW_RING_FN __device__ __forceinline__
#define SW_RING_ANY(x) __any(x)
#else
#define SW_RING_FN inline
#define SW_RING_ANY(x) (x)
#endif

namespace prgpu {

SW_RING_FN int ring_max3(int a, int b, int c) {
    const int m = a > b ? a : b;
    return m > c ? m : c;
}
SW_RING_FN int ring_ctz(uint32_t x) { return __builtin_ctz(x); }
SW_RING_FN int ring_clz(uint32_t x) { return __builtin_clz(x); }

struct ExtIO {
    int qle, tle, gtle, gscore, max_off;
};

// ---------------------------------------------------------------------------
// ksw_extend2 with the DP row in registers.
//
// The band of row i covers query columns [i-w, i+w]; with WB >= w fixed at
// compile time, slot s of the register ring R holds query column i - WB + s
// (NS = 2*WB + 2 slots).  ksw_extend2's eh[j] after row i-1 (H(i-1, j-1) and
// E(i, j)) sits in R[s+1] when row i reaches slot s, and the row's new eh[j]
// goes to R[s]: one ascending sweep reads each word before overwriting it, and
// every column moves down one slot per row, carrying its query base with it.
// Word: q*5 [0,5) | H [5,18) | E [18,31).
//
// Cells outside the lane's band are computed as well but change nothing that
// is read later: a column left of `beg` is never read again (beg only grows),
// a column right of `end` keeps its word (ksw_extend2 reads such stale words
// when the pruned end grows by two), columns entering the ring carry their
// first-row H, and the row max / h1 / f only take in-band cells.  Slot chunks
// left of every lane's band or right of every lane's query end are skipped.
template <int WB>
SW_RING_FN int ext_ring(const uint8_t *Q, int qb, int qs, int qlen, const uint8_t *Lr, long tb, int ts,
                        bool comp, int tlen, const SwOptsDev &O, int w, int end_bonus, int h0, ExtIO &io) {
    constexpr int NS = 2 * WB + 2;
    constexpr int NM = (NS + 31) / 32;
    constexpr int CH = 8;
    constexpr int NCH = (NS + CH - 1) / CH;
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    int max_ins = (int)((double)(qlen * a + end_bonus - o_ins) / e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    int max_del = (int)((double)(qlen * a + end_bonus - o_del) / e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    // row -1: eh[j] = {max(h0 - oe_ins - e_ins*(j-1), 0) (h0 at j = 0), 0, q[j]}; R[s] = column s-WB-1
    uint32_t R[NS];
    const int hj1 = h0 > oe_ins ? h0 - oe_ins : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int j = s - WB - 1;
        uint32_t wd = 0u;
        if (j >= 0 && j <= qlen) {
            int h = j == 0 ? h0 : hj1 - e_ins * (j - 1);
            h = h > 0 ? h : 0;
            const uint32_t q5 = j < qlen ? 5u * (uint32_t)Q[qb + qs * j] : 0u;
            wd = q5 | ((uint32_t)h << 5);
        }
        R[s] = wd;
    }
    int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    // score field per query code (q = 0..4), biased by 16: 5 bits each
    const uint32_t mm5 = (uint32_t)(16 - b);
    const uint32_t tab_mis = mm5 | (mm5 << 5) | (mm5 << 10) | (mm5 << 15) | (15u << 20);
    const uint32_t tab_n = 15u | (15u << 5) | (15u << 10) | (15u << 15) | (15u << 20);
    // a column entering the ring at the top: its query base and first-row H
    auto entering = [&](int j) -> uint32_t {
        if (j > qlen) return 0u;
        int h = hj1 - e_ins * (j - 1);
        h = h > 0 ? h : 0;
        return (j < qlen ? 5u * (uint32_t)Q[qb + qs * j] : 0u) | ((uint32_t)h << 5);
    };
    int tc_next = tlen > 0 ? (int)Lr[tb] : 0;
    uint32_t qin_next = entering(WB + 1);
    for (int i = 0; i < tlen; ++i) {
        int tc = tc_next;
        if (comp && tc < 4) tc = 3 - tc;
        const uint32_t qin = qin_next;   // column i + WB + 1 enters at the top slot
        if (i + 1 < tlen) tc_next = (int)Lr[tb + (long)ts * (i + 1)];
        qin_next = entering(i + WB + 2);
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        int h1;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else
            h1 = 0;
        const uint32_t tab = tc > 3 ? tab_n : ((tab_mis & ~(31u << (5 * tc))) | ((uint32_t)(16 + a) << (5 * tc)));
        const int sb = beg - i + WB, se = end - i + WB;   // slots of [beg, end)
        const int stop = qlen - i + WB;                   // slot of column qlen
        const unsigned nb = (unsigned)(se - sb);
        int f = 0, hl = 0;
        uint32_t mp = 0u;
        uint32_t nz[NM];
#pragma unroll
        for (int k = 0; k < NM; ++k) nz[k] = 0u;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (!SW_RING_ANY(sb < (c + 1) * CH && stop >= c * CH)) continue;
#pragma unroll
            for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s) {
                const uint32_t wd = (s + 1 < NS) ? R[s + 1] : qin;
                const uint32_t q5 = wd & 31u;
                const int Mr = (int)((wd >> 5) & 0x1FFFu);
                const int e0 = (int)(wd >> 18);
                const int sc = (int)((tab >> q5) & 31u);
                const int M = Mr ? Mr + sc - 16 : 0;   // separating H and M (ksw_extend2)
                const int h = ring_max3(M, e0, f);
                const int en = ring_max3(e0 - e_del, M - oe_del, 0);
                const int fn = ring_max3(f - e_ins, M - oe_ins, 0);
                const unsigned rel = (unsigned)(s - sb);
                const bool inb = rel < nb;
                const bool isend = s == se;
                const uint32_t nw = q5 | ((uint32_t)h1 << 5) | ((uint32_t)(isend ? 0 : en) << 18);
                R[s] = s > se ? wd : nw;
                if (isend) hl = h1;
                if (inb) {
                    const uint32_t cand = ((uint32_t)h << 9) | (uint32_t)s;
                    mp = mp > cand ? mp : cand;
                }
                if (rel <= nb && nw > 31u) nz[s >> 5] |= 1u << (s & 31);
                const bool pre = s < sb;
                h1 = pre ? h1 : h;
                f = pre ? 0 : fn;
            }
        }
        const int jend = beg < end ? end : beg;
        if (jend == qlen) {
            max_ie = gscore > hl ? max_ie : i;
            gscore = gscore > hl ? gscore : hl;
        }
        const int m = (int)(mp >> 9);
        if (m == 0) break;
        const int mj = i - WB + (int)(mp & 511u);
        if (m > max) {
            max = m, max_i = i, max_j = mj;
            const int d = mj - i < 0 ? i - mj : mj - i;
            max_off = max_off > d ? max_off : d;
        } else if (O.zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - m - ((i - max_i) - (mj - max_j)) * e_del > O.zdrop) break;
            } else {
                if (max - m - ((mj - max_j) - (i - max_i)) * e_ins > O.zdrop) break;
            }
        }
        // band pruning: first non-zero eh in [beg, end), last in [beg', end]
        int fs = NS, ls = -1;
#pragma unroll
        for (int k = NM - 1; k >= 0; --k)
            if (nz[k]) fs = k * 32 + ring_ctz(nz[k]);
#pragma unroll
        for (int k = 0; k < NM; ++k)
            if (nz[k]) ls = k * 32 + 31 - ring_clz(nz[k]);
        const int bs = fs < se ? fs : se;
        const int js = ls >= bs ? ls : bs - 1;
        beg = i - WB + bs;
        end = i - WB + js + 2 < qlen ? i - WB + js + 2 : qlen;
    }
    io.qle = max_j + 1;
    io.tle = max_i + 1;
    io.gtle = max_ie + 1;
    io.gscore = gscore;
    io.max_off = max_off;
    return max;
}


// ---------------------------------------------------------------------------
// ksw_global2 with the DP row in a register ring (same slot scheme as ext_ring;
// no band pruning, so columns right of the band are never read before their
// end-cell write and need no protection).  Word: q [0,3) | E [3,17) | H [17,31),
// H and E 14-bit two's complement with G_NEG standing in for MINUS_INF (only
// ever compared with finite values: the host bounds |finite| < 7000).
// Direction nibbles (h source [0,2), E-continue bit 2, F-continue bit 3) of row
// i, slot s go to z[(i * NW + s / 8) * ZS] bits 4*(s%8); ZS is the lane stride.
constexpr int G_RNEG = -8192;
SW_RING_FN uint32_t gword(uint32_t q, int e, int h) {
    return q | (((uint32_t)e & 0x3FFFu) << 3) | ((uint32_t)h << 17);
}
SW_RING_FN int gw_e(uint32_t w) { return ((int)(w << 15)) >> 18; }
SW_RING_FN int gw_h(uint32_t w) { return ((int)(w << 1)) >> 18; }

template <int WB>
SW_RING_FN int glob_ring(const uint8_t *Q, int qb, int qs, int qlen, const uint8_t *Lr, long tb, int ts,
                         bool comp, int tlen, const SwOptsDev &O, int w, uint32_t *z, int ZS) {
    constexpr int NS = 2 * WB + 2;
    constexpr int NW = (NS + 7) / 8;
    constexpr int CH = 8;
    constexpr int NCH = (NS + CH - 1) / CH;
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    // row -1: eh[0] = {0, -inf}, eh[j] = {-(o_ins + e_ins*j), -inf} for j <= w, else {-inf, -inf}
    auto init_word = [&](int j) -> uint32_t {
        if (j < 0 || j > qlen) return 0u;
        const int h = j == 0 ? 0 : (j <= w ? -(o_ins + e_ins * j) : G_RNEG);
        const uint32_t q = j < qlen ? (uint32_t)Q[qb + qs * j] : 0u;
        return gword(q, G_RNEG, h);
    };
    uint32_t R[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) R[s] = init_word(s - WB - 1);
    const uint32_t mm5 = (uint32_t)(16 - b);
    const uint32_t tab_mis = mm5 | (mm5 << 5) | (mm5 << 10) | (mm5 << 15) | (15u << 20);
    const uint32_t tab_n = 15u | (15u << 5) | (15u << 10) | (15u << 15) | (15u << 20);
    int tc_next = tlen > 0 ? (int)Lr[tb] : 0;
    uint32_t qin_next = init_word(WB + 1);
    for (int i = 0; i < tlen; ++i) {
        int tc = tc_next;
        if (comp && tc < 4) tc = 3 - tc;
        const uint32_t qin = qin_next;
        if (i + 1 < tlen) tc_next = (int)Lr[tb + (long)ts * (i + 1)];
        qin_next = init_word(i + WB + 2);
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        const uint32_t tab = tc > 3 ? tab_n : ((tab_mis & ~(31u << (5 * tc))) | ((uint32_t)(16 + a) << (5 * tc)));
        const int sb = beg - i + WB, se = end - i + WB;
        const int stop = qlen - i + WB;   // slot of column qlen: columns beyond are dead
        int f = G_RNEG;
        int h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : G_RNEG;
        uint32_t *zi = z + (long)i * NW * ZS;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (!SW_RING_ANY(sb < (c + 1) * CH && stop >= c * CH)) continue;
            uint32_t dacc = 0u;
#pragma unroll
            for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s) {
                const uint32_t wd = (s + 1 < NS) ? R[s + 1] : qin;
                const uint32_t q = wd & 7u;
                const int e0 = gw_e(wd);
                const int m = gw_h(wd) + (int)((tab >> (5u * q)) & 31u) - 16;
                uint32_t d = m >= e0 ? 0u : 1u;
                int h = m >= e0 ? m : e0;
                d = h >= f ? d : 2u;
                h = h >= f ? h : f;
                const int t1 = m - oe_del;
                int e = e0 - e_del;
                d |= e > t1 ? 4u : 0u;
                e = e > t1 ? e : t1;
                const int t2 = m - oe_ins;
                int fn = f - e_ins;
                d |= fn > t2 ? 8u : 0u;
                fn = fn > t2 ? fn : t2;
                R[s] = gword(q, s == se ? G_RNEG : e, h1);
                dacc |= d << (4 * (s - c * CH));
                const bool pre = s < sb;
                h1 = pre ? h1 : h;
                f = pre ? G_RNEG : fn;
            }
            zi[c * ZS] = dacc;
        }
    }
    // eh[qlen].h: column qlen sits in slot qlen - (tlen - 1) + WB after the last row
    const int sq = qlen - (tlen - 1) + WB;
    int score = G_RNEG;
#pragma unroll
    for (int s = 0; s < NS; ++s)
        if (s == sq) score = gw_h(R[s]);
    if (tlen == 0) score = qlen <= w ? (qlen == 0 ? 0 : -(o_ins + e_ins * qlen)) : G_RNEG;
    return score;
}

// ksw_global2's backtrack over the ring's direction nibbles: ops (0 M, 1 I, 2 D)
// pushed in reverse order; returns the op count or -1 if more than maxcig.
template <int WB>
SW_RING_FN int glob_backtrack(const uint32_t *z, int ZS, int tlen, int qlen, int w, uint32_t *cg, int maxcig) {
    constexpr int NS = 2 * WB + 2;
    constexpr int NW = (NS + 7) / 8;
    int n = 0;
    auto push = [&](int op, int len) {
        if (n < 0) return;
        if (n > 0 && (int)(cg[n - 1] & 0xFu) == op) {
            cg[n - 1] += (uint32_t)len << 4;
            return;
        }
        if (n >= maxcig) { n = -1; return; }
        cg[n++] = ((uint32_t)len << 4) | (uint32_t)op;
    };
    int i = tlen - 1, k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1, which = 0;
    while (i >= 0 && k >= 0 && n >= 0) {
        const int s = k - i + WB;
        const uint32_t nib = (z[((long)i * NW + (s >> 3)) * ZS] >> (4 * (s & 7))) & 15u;
        which = which == 0 ? (int)(nib & 3u) : (which == 1 ? (int)((nib >> 2) & 1u) : (int)((nib >> 3) & 1u) * 2);
        if (which == 0) push(0, 1), --i, --k;
        else if (which == 1) push(2, 1), --i;
        else push(1, 1), --k;
    }
    if (n >= 0 && i >= 0) push(2, i + 1);
    if (n >= 0 && k >= 0) push(1, k + 1);
    return n;
}

}  // namespace prgpu
