// Seeding and chaining of one short read: the part of
// `bwa-proovread mem` that turns a read into seed-extension tasks.  One
// implementation for the host path (seed.cpp, scratch that grows on demand)
// and the device path (seed_kernels.hip, one lane per read, fixed scratch per
// lane; a read that outgrows it is flagged, never silently changed).
//
// Restates upstream bwa (absent submodule, .gitmodules:4-6; parity unpinned,
// DESIGN.md) over the index of seed.cpp:
//   mem_collect_intv  bwt_smem1a SMEMs >= -k, re-seeding of long SMEMs with
//                     <= split_width hits (-r), bwt_seed_strategy1 (-y)
//   mem_chain         occurrences (<= -c per SMEM, sampled in text order), each
//                     merged into the chain with the largest pos <= its rbeg by
//                     test_and_merge or opening a new chain after the chains of
//                     equal pos (the btree order; per-range lists here, see range_slot)
//   mem_chain_flt     chain weight, -W minimum, stable sort, -D / mask_level
//   mem_flt_chained_seeds (bwa >= 0.7.13; runs for reads with 1.1 W <= 0.05 len, i.e.
//                     >= 440 bp at proovread's mr -W 20): each seed's local SW score
//                     (ksw_align2 over the seed +- 50 bp when both windows stay < 200)
//                     drops seeds scoring below a*1.1*W and becomes the seed's score
//   mem_chain2aln     its input: every seed of every kept chain in the order it
//                     tries them (longest first, last on ties) with the chain's
//                     reference window (cal_max_gap over its seeds); the
//                     extension and the containment test run on the device
// Occurrence counts come from a per-read table: for every start a, the hits of
// the 12-mer q[a, a+12) with their exact match length ml = LCP(q[a..], T[p..]);
// occ(q[a, b)) = #{hits of a with ml >= b - a} (a per-start count table for
// ml < 12 + HB), j-mer count tables below 12.  Match lengths follow diagonals
// (p-1 a hit of a-1 with ml >= 13 -> p a hit of a with ml - 1); a new diagonal
// compares the KX bases the index stores after the hit (kext) and reads the
// text only after a full KX-base match.
#pragma once
#include <math.h>
#include <stdint.h>

#include "../../include/prgpu.h"

#if defined(__HIPCC__)
#define SC_HD __host__ __device__ inline
#else
#define SC_HD inline
#endif

// work counters of a host-only statistics build (tools/seed_stats.sh); compiled out otherwise
#if defined(PR_SEED_STATS) && !defined(__HIP_DEVICE_COMPILE__)
extern unsigned long long pr_seed_stat_g[24];
#define SC_STAT(k, v) __atomic_fetch_add(&pr_seed_stat_g[k], (unsigned long long)(v), __ATOMIC_RELAXED)
#else
#define SC_STAT(k, v) ((void)0)
#endif

namespace prgpu {
namespace seedc {

constexpr int KI = 12;                        // indexed k-mer length
constexpr uint32_t NK = 1u << (2 * KI);       // 4^12
constexpr int KX = 28;                        // bases stored after each hit
constexpr uint64_t KX_MASK = (1ull << (2 * KX)) - 1;
#ifndef SC_SCANGE   // count jumps past the per-start table (Occ::scan_ge) in smem1 / seed_strategy1
#define SC_SCANGE 1
#endif
constexpr int HB = 20;                        // per-start count table width
constexpr int CB_SHIFT = 12;                  // contig block table granularity
constexpr int RK = 11;                        // R_k tabulated per start for k <= RK (split_width + 1)

// Text positions: the text holds both strands of every long read, 2 l_pac + 2 n_lr bases, up to
// 2^33 (l_pac < 4.29 Gb: configs[3]'s 2.7 Gb read set).  Hit positions are
// stored as their low 32 bits; a k-mer's hits are in text order, so those at or beyond 2^32
// form the tail of its list, from ksplit[code] on (ksplit null: the text is below 2^32).
constexpr uint64_t POS_PAGE = 1ull << 32;
constexpr int64_t MAX_TEXT = (int64_t)1 << 33;

// Per 2^CB_SHIFT text block (device index only): the contig at the block's start (c0), the
// offsets in the block where contigs c0 + 1 and c0 + 2 start (2^CB_SHIFT: none), and the
// coordinate offsets of c0 and c0 + 1 (fr = text position + d): text_to_fr in one load.
struct BlkFr {
    int64_t d0, d1;
    int32_t c0, bnd, bnd2, pad;
};

// Device- or host-resident index, plain pointers (built by seed.cpp).
struct IndexView {
    const uint8_t *text;       // forward long reads, then rc of their concatenation, SEP (5) after each
    int64_t n_text;
    const int64_t *cstart;     // [n_contig] text offset of contig c
    int32_t n_contig;          // 2 * n_lr
    const int32_t *cblk;       // contig at the start of every 2^CB_SHIFT text block
    const int64_t *lr_off;     // [n_lr + 1] forward long-read offsets
    int32_t n_lr;
    int64_t l_pac;
    const uint64_t *koff;      // [NK + 1]
    const uint32_t *kpos;      // 12-mer hits (low 32 bits of the text position), text order within a k-mer
    const uint64_t *ksplit;    // [NK] first hit of k-mer `code` at or beyond POS_PAGE, or null
    const uint64_t *kext;      // per hit: KX bases after it (2 bits each) | count << 56
    const uint32_t *cnt[KI - 1];   // cnt[j-1][code]: occurrences of the j-mer `code`, j = 1..11
    const uint64_t *text4;     // device: the text 16 bases per word (4 bits each) + a padding word, or null
    const BlkFr *blkfr;        // device: [n_text >> CB_SHIFT + 1] block coordinate table, or null
    int32_t walk_nw = 4;       // device: the match-length walk's 16-base compares per text round trip
};

struct Iv {
    int32_t start, end;
    int64_t occ;
};
struct Seed {
    int64_t rbeg;   // forward-reverse coordinate (bwa): reverse strand >= l_pac
    int16_t qbeg, len;   // (reads <= 1000 bp: proovread:457)
    int32_t nx;     // the next seed of its chain (-1: the last)
};
// A (long read, strand) range of the chaining (map_chains): its chain list and, for the merges
// that nearly every occurrence makes, a copy of the list's last chain's merge state (its pos,
// first and last seed, seed count) -- one cache line per occurrence instead of the range table,
// the chain record and two seed records.  n / last / l_idx are authoritative while the chain is
// the range's tail and written back to it when another chain becomes the tail and at the end.
struct RangeRec {
    int32_t head, tail, n, l_idx;   // list head / tail (chain indices), the tail chain's seeds / last seed
    int64_t tpos;                   // the tail chain's pos
    int64_t f_rbeg, l_rbeg;         // its first and last seed
    int32_t f_ql, l_ql;             // qbeg | len << 16
    int32_t pad[4];                 // (64 bytes: one record per half cache line)
};
struct RangeEnt {
    int32_t key, r;   // rid * 2 + strand (-1: free), its RangeRec
};
struct Chain {
    int64_t pos;
    int32_t rid, head, tail, n;   // seeds: a linked list in the pool (only ever appended)
    int32_t w, kept, first;
};

enum {
    SC_OVER_LEN = 1, SC_OVER_HITS = 2, SC_OVER_IV = 4, SC_OVER_MEMS = 8, SC_OVER_SEEDS = 16,
    SC_OVER_CHAINS = 32, SC_OVER_OUT = 64
};

// Scratch of one read (host: vectors; device: a lane's slice of a global buffer).
struct Scratch {
    int32_t lmax;                              // longest read the per-start arrays hold
    int32_t *hoff;                             // [lmax + 1]
    uint64_t *qext;                            // [lmax + 1]
    int32_t *codes;                            // [lmax + 1]
    uint32_t *ge;                              // [lmax * HB]
    uint32_t *hpos;                            // [cap_hits] low 32 bits of the hit's text position
    uint8_t *hhi;                              // [cap_hits] bit 32 of it (null: the text is below 2^32)
    uint16_t *hml;                             // [cap_hits]
    int32_t cap_hits;
    Iv *mems;                                  // [cap_mems]
    int32_t cap_mems;
    Iv *m1, *curr, *prev;                      // [cap_iv] each
    int32_t cap_iv;
    Seed *seeds;                               // [cap_seeds]
    int32_t cap_seeds;
    Chain *cv, *ch;                            // [cap_chains] each
    int32_t *cnx, *kept;                       // [cap_chains] each; cnx: next chain of its range's list
    RangeEnt *htab;                            // [hsize] range table (open addressing)
    RangeRec *rg;                              // [cap_chains] the ranges, in creation order
    int32_t cap_chains, hsize;                 // hsize: power of two >= 2 * cap_chains
    uint16_t *rmax;                            // [(lmax + 1) * RK] R_k(a), k = 1..RK (rmax_k)
    uint64_t *hfr;                             // [cap_hits] pack_fr of the hit (the chaining's coordinates)
    // lazy occurrence table (Caps.lazy; null otherwise): a start's hits, count row and R_k are
    // computed the first time the SMEM search or the chaining asks for them (materialize), its hits
    // appended to a per-read pool: hits of start a at [hoff[a], hend[a])
    int32_t *hend;                             // [lmax + 1]
    uint8_t *ready;                            // [lmax + 1] start materialized
    uint64_t *q4w;                             // [lmax / 16 + 4] the read 16 bases per word (4 bits each), or null
    int32_t *lz;                               // [4] pool fill, SC_OVER_* flags, hits the read would need
};

SC_HD uint64_t pack_ext(const uint8_t *s, int n) {
    uint64_t v = 0;
    int k = 0;
    for (; k < n && s[k] < 4; ++k) v |= (uint64_t)s[k] << (2 * k);
    return v | ((uint64_t)k << 56);
}

SC_HD int ctz64(uint64_t x) { return __builtin_ctzll(x); }

// a long-read byte as a base code: nt4 codes (0-3, else N) or ASCII (ACGT in either case, else N)
SC_HD uint8_t base_code(uint8_t c) {
    if (c < 4) return c;
    switch (c | 0x20) {
        case 'a': return 0;
        case 'c': return 1;
        case 'g': return 2;
        case 't': return 3;
        default: return 4;
    }
}

// text position of hit r of k-mer `code`
SC_HD uint64_t hit_pos(const IndexView &I, uint32_t code, uint64_t r) {
    uint64_t p = I.kpos[r];
    if (I.ksplit && r >= I.ksplit[code]) p += POS_PAGE;
    return p;
}
// the per-read hit table's positions
SC_HD uint64_t get_hpos(const Scratch &S, int64_t k) {
    return (uint64_t)S.hpos[k] | (S.hhi ? (uint64_t)S.hhi[k] << 32 : 0ull);
}
SC_HD void set_hpos(const Scratch &S, int64_t k, uint64_t p) {
    if (!S.hpos) return;
    S.hpos[k] = (uint32_t)p;
    if (S.hhi) S.hhi[k] = (uint8_t)(p >> 32);
}

// ---------------------------------------------------------------- text -> bwa coordinates
SC_HD int contig_of(const IndexView &I, int64_t p) {
    int c = I.cblk[p >> CB_SHIFT];
    while (c + 1 < I.n_contig && I.cstart[c + 1] <= p) ++c;
    return c;
}

SC_HD void text_to_fr(const IndexView &I, uint64_t p, int64_t &fr, int &rid) {
    const int c = contig_of(I, p);
    const int64_t o = (int64_t)p - I.cstart[c];
    if (c < I.n_lr) {
        rid = c;
        fr = I.lr_off[c] + o;
    } else {
        rid = 2 * I.n_lr - 1 - c;   // the reverse half holds the long reads in reverse order
        fr = I.l_pac + (I.l_pac - I.lr_off[rid + 1]) + o;
    }
}

// pack_fr through the device's block coordinate table when the hit's block has at most two
// contig starts after its first contig (one load), else the cblk -> cstart walk
SC_HD uint64_t pack_fr_blk(const IndexView &I, uint64_t p);

// a hit's forward-reverse coordinate and long read, packed for the chaining (rid < 2^24)
constexpr int FR_RID_BITS = 24;
SC_HD uint64_t pack_fr(const IndexView &I, uint64_t p) {
    int64_t fr;
    int rid;
    text_to_fr(I, p, fr, rid);
    return ((uint64_t)fr << FR_RID_BITS) | (uint64_t)rid;
}

SC_HD uint64_t pack_fr_blk(const IndexView &I, uint64_t p) {
    if (I.blkfr) {
        const BlkFr bt = I.blkfr[p >> CB_SHIFT];
        const int o = (int)(p & ((1u << CB_SHIFT) - 1u));
        int c = -1;
        int64_t d = 0;
        if (o < bt.bnd) c = bt.c0, d = bt.d0;
        else if (o < bt.bnd2) c = bt.c0 + 1, d = bt.d1;
        if (c >= 0) {
            const int rid = c < I.n_lr ? c : 2 * I.n_lr - 1 - c;   // (reverse half: reads in reverse order)
            return ((uint64_t)((int64_t)p + d) << FR_RID_BITS) | (uint64_t)rid;
        }
    }
    return pack_fr(I, p);
}

// 16 bases from base x of a 4-bit packed sequence (a padding word after the last)
SC_HD uint64_t nib16c(const uint64_t *w4, uint64_t x) {
    const uint64_t w = x >> 4;
    const int sh = (int)(x & 15) * 4;
    const uint64_t lo = w4[w];
    return sh ? (lo >> sh) | (w4[w + 1] << (64 - sh)) : lo;
}

// ---------------------------------------------------------------- occurrence table
// the j-mer count tables j = 1..LC_MAX held on chip by the device kernels (5,460 entries):
// table j at LC_OFF(j) = (4^j - 4) / 3
constexpr int LC_MAX = 6;
SC_HD constexpr int lc_off(int j) { return ((1 << (2 * j)) - 4) / 3; }
constexpr int LC_N = lc_off(LC_MAX + 1);   // 4 + 16 + ... + 4^LC_MAX

template <bool LZ> struct OccB;
SC_HD void materialize(const OccB<true> &occ, int a);

// The occurrence counts of read q's substrings.  LZ: the lazy table (Scratch.hend), a start
// materialized on first use; the eager table's code (LZ = false) has no trace of it.
template <bool LZ>
struct OccB {
    const IndexView *I;
    const Scratch *S;
    const uint8_t *q;
    int len;
    const uint32_t *lc = nullptr;   // LDS copy of cnt[0 .. LC_MAX-1] (device) or null

    // the lazy table's start a on first use (a no-op for the eager table)
    SC_HD void need(int a) const {
        if constexpr (LZ) {
            if (a < len && !S->ready[a]) materialize(*this, a);
        }
    }
    // the end of start a's hits (the eager table: the next start's offset)
    SC_HD int32_t end_of(int a) const {
        if constexpr (LZ) return S->hend[a];
        else return S->hoff[a + 1];
    }

    // occ(a, b) for b - a < KI: the j-mer count tables (no occurrence-table access)
    SC_HD int64_t jmer(int a, int b) const {
        const int n = b - a;
        uint32_t code = 0;
        const int32_t c12 = a + KI <= len ? S->codes[a] : -1;
        if (c12 >= 0) code = (uint32_t)c12 >> (2 * (KI - n));   // the start's 12-mer code, truncated
        else
            for (int x = a; x < b; ++x) code = (code << 2) | q[x];
        if (lc && n <= LC_MAX) return lc[lc_off(n) + code];
        return I->cnt[n - 1][code];
    }

    SC_HD int64_t operator()(int a, int b) const {
        const int n = b - a;
        SC_STAT(8, 1);
        if (n < KI) return jmer(a, b);
        need(a);
        if (n - KI < HB) return S->ge[(int64_t)a * HB + (n - KI)];
        int64_t c = 0;
        SC_STAT(9, 1);
        const int32_t h1 = end_of(a);
        SC_STAT(10, h1 - S->hoff[a]);
        for (int32_t k = S->hoff[a]; k < h1; ++k) c += S->hml[k] >= n;
        return c;
    }
    // occ(a, a + n) for n >= KI + HB (a scan of the start's hits) and the smallest match length
    // >= n (mn; 0 when none): occ(a, a + n') is the same for every n' in [n, mn], so a forward
    // extension can step from n to mn at once (the finish task's near-exact reads: one scan per
    // distinct match length instead of one per base)
    SC_HD int64_t scan_ge(int a, int n, int &mn) const {
        int64_t c = 0;
        int m = 0x7fffffff;
        need(a);
        const int32_t h1 = end_of(a);
        SC_STAT(9, 1);
        SC_STAT(10, h1 - S->hoff[a]);
        for (int32_t k = S->hoff[a]; k < h1; ++k) {
            const int v = S->hml[k];
            if (v >= n) {
                ++c;
                m = v < m ? v : m;
            }
        }
        mn = c ? m : 0;
        return c;
    }
};
using Occ = OccB<false>;
using OccLazy = OccB<true>;

// The end of the longest match from start a that occurs >= k times in the text:
// R_k(a) = max{e : occ(a, e) >= k} (a when even q[a] occurs fewer than k times or is N).
// occ(a, e) never grows with e and never shrinks as a moves right (every occurrence of
// q[a, e) contains one of q[a + 1, e)), which is what makes smem1's backward extension a
// staircase over R_k (below).  Below 12 bases: the N-free j-mer counts.
SC_HD int short_limit(const uint8_t *q, int len, int a) {   // the N-free bases from a, <= KI - 1
    int e = a;
    while (e < len && e - a < KI - 1 && q[e] < 4) ++e;
    return e;
}
template <class OccT>
SC_HD int rmax_short(const OccT &occ, const uint8_t *q, int len, int a, int64_t k) {
    int e = short_limit(q, len, a);   // from the longest down: one lookup when it qualifies
    while (e > a && occ.jmer(a, e) < k) --e;
    return e;
}

// R_1 .. R_RK of start a into S.rmax[a * RK ..]: with >= k hits of its 12-mer, a + the k-th
// largest hit match length (occ(a, e) >= k exactly when k hits match >= e - a bases); with
// fewer, the longest N-free j-mer (j < 12) with >= k occurrences (R_k never grows with k)
// insert a hit's match length into a start's descending top-RK list
SC_HD void topk_insert(uint16_t (&top)[RK], uint16_t v) {
#pragma unroll
    for (int k = 0; k < RK; ++k) {
        const uint16_t t = top[k];
        const bool gt = v > t;
        top[k] = gt ? v : t;
        v = gt ? t : v;
    }
}
// R_1 .. R_RK of start a from its top list (the RK largest hit match lengths, 0-padded; all
// zero when the start has no 12-mer or q[a] is N)
template <class OccT>
SC_HD void fill_rk_top(const OccT &occ, const Scratch &S, const uint8_t *q, int len, int a, const uint16_t (&top)[RK]) {
    uint16_t *r = S.rmax + (int64_t)a * RK;
    int e = -1;   // the short part: j-mer counts never grow with k, so its end only falls
    int64_t ce = 0;
    for (int k = 1; k <= RK; ++k) {
        if (top[k - 1] > 0) {
            r[k - 1] = (uint16_t)(a + top[k - 1]);
            continue;
        }
        if (e < 0) {
            e = short_limit(q, len, a);
            ce = e > a ? occ.jmer(a, e) : 0;
        }
        while (e > a && ce < k) {
            --e;
            ce = e > a ? occ.jmer(a, e) : 0;
        }
        r[k - 1] = (uint16_t)e;
    }
}
template <class OccT>
SC_HD void fill_rk(const OccT &occ, const Scratch &S, const uint8_t *q, int len, int a) {
    uint16_t top[RK];
#pragma unroll
    for (int k = 0; k < RK; ++k) top[k] = 0;
    if (q[a] < 4 && a + KI <= len && S.codes[a] >= 0)
        for (int32_t h = S.hoff[a]; h < S.hoff[a + 1]; ++h) topk_insert(top, S.hml[h]);
    fill_rk_top(occ, S, q, len, a, top);
}

// R_k(a): tabulated for k <= RK; beyond (re-seeding with split_width >= RK), from the start's
// count row and its hits' lengths
template <class OccT>
SC_HD int rmax_k(const OccT &occ, const Scratch &S, const uint8_t *q, int len, int a, int64_t k) {
    if (k < 1) k = 1;
    occ.need(a);
    if (k <= RK) return S.rmax[(int64_t)a * RK + (k - 1)];
    if (q[a] > 3) return a;
    if (a + KI <= len && S.codes[a] >= 0) {
        const uint32_t *g = S.ge + (int64_t)a * HB;
        if ((int64_t)g[0] >= k) {
            if ((int64_t)g[HB - 1] < k) {   // the largest t with g[t] >= k (the row never grows with t)
                int lo = 0, hi = HB - 2;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if ((int64_t)g[mid] >= k) lo = mid; else hi = mid - 1;
                }
                return a + KI + lo;
            }
            // >= k hits match at least KI + HB - 1 bases: the k-th largest match length
            int lo = KI + HB - 1, hi = len - a;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                int64_t c = 0;
                const int32_t h1 = occ.end_of(a);
                for (int32_t h = S.hoff[a]; h < h1; ++h) c += S.hml[h] >= mid;
                if (c >= k) lo = mid; else hi = mid - 1;
            }
            return a + lo;
        }
    }
    return rmax_short(occ, q, len, a, k);
}

// the exact match length ml = LCP(q[a..], T[p..]) of a hit of start a: the KX bases stored after
// the hit (ex) against the read's (qe), then the text (16 bases a step from the 4-bit copies when
// the index and the read have them, else a base a step)
SC_HD int hit_ml(const IndexView &I, const Scratch &S, const uint8_t *q, int len, int a, uint64_t p, uint64_t ex,
                 uint64_t qe) {
    const int le = (int)(ex >> 56), lq = (int)(qe >> 56);
    const uint64_t x = (ex ^ qe) & KX_MASK;
    int m = x ? ctz64(x) >> 1 : KX;
    m = m < le ? m : le;
    m = m < lq ? m : lq;
    int ml = KI + m;
    if (m < KX) return ml;
    if (I.text4 && S.q4w) {   // 64 bases a round trip: 5 text words loaded together (8 padding words)
        bool go = a + ml < len;
        while (go) {
            const uint64_t tp = p + (uint64_t)ml;
            const uint64_t *tw4 = I.text4 + (tp >> 4);
            const int sh = (int)(tp & 15) * 4;
            uint64_t w5[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) w5[j] = tw4[j];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!go) break;
                const int xx = a + ml;
                const uint64_t tw = sh ? (w5[j] >> sh) | (w5[j + 1] << (64 - sh)) : w5[j];
                const uint64_t qw = nib16c(S.q4w, (uint64_t)xx);
                const uint64_t nq = (qw >> 2) & 0x1111111111111111ull;   // read N (code 4) or past the end (6)
                const uint64_t bad = (qw ^ tw) | (nq * 0xFull);
                const int lim = len - xx;
                if (bad) {
                    const int f = ctz64(bad) >> 2;
                    ml += f < lim ? f : lim;
                    go = false;
                } else if (lim <= 16) {
                    ml += lim;
                    go = false;
                } else {
                    ml += 16;
                }
            }
        }
    } else {
        while (a + ml < len && q[a + ml] < 4 && I.text[p + ml] == q[a + ml]) ++ml;
    }
    return ml;
}

// The lazy table's start a (Scratch.hend): its hits appended to the read's pool with their match
// lengths and coordinates, its count row and R_1 .. R_RK -- the values the eager table holds for
// it.  A pool that would overflow flags the read (lz[1]) and records the hits it needs (lz[2]).
#if defined(__HIPCC__)
__attribute__((noinline))   // (out of line: the eager table's kernels only test S.hend)
#endif
SC_HD void materialize(const OccLazy &occ, int a) {
    const IndexView &I = *occ.I;
    const Scratch &S = *occ.S;
    const uint8_t *q = occ.q;
    const int len = occ.len;
    S.ready[a] = 1;
    const int32_t beg = S.lz[0];
    uint32_t g[HB];
    uint16_t top[RK];
#pragma unroll
    for (int t = 0; t < HB; ++t) g[t] = 0u;
#pragma unroll
    for (int k = 0; k < RK; ++k) top[k] = 0;
    int32_t n = 0;
    const int32_t code = a + KI <= len ? S.codes[a] : -1;
    if (code >= 0) {
        const uint64_t r0 = I.koff[code], r1 = I.koff[code + 1];
        const int64_t need = (int64_t)beg + (int64_t)(r1 - r0);
        if (need > S.cap_hits) {
            S.lz[1] |= SC_OVER_HITS;
            S.lz[2] = (int32_t)(need < (int64_t)1 << 30 ? need : (int64_t)1 << 30);
        } else {
            n = (int32_t)(r1 - r0);
            const uint64_t qe = S.qext[a];
            const bool ranked = q[a] < 4;
            // 4 hits at a time: their position, extension and block-table loads are independent
            // (one latency per batch, not per hit), then each hit's match length and coordinate
            constexpr int MB = 4;
            for (uint64_t r = r0; r < r1; r += MB) {
                uint64_t pp[MB], ex[MB], fr[MB];
#pragma unroll
                for (int u = 0; u < MB; ++u) {
                    const bool ok = r + u < r1;
                    pp[u] = ok ? hit_pos(I, (uint32_t)code, r + u) : 0ull;
                    ex[u] = ok ? I.kext[r + u] : 0ull;
                }
#pragma unroll
                for (int u = 0; u < MB; ++u) fr[u] = r + u < r1 ? pack_fr_blk(I, pp[u]) : 0ull;
#pragma unroll
                for (int u = 0; u < MB; ++u) {
                    if (r + u >= r1) break;
                    const int ml = hit_ml(I, S, q, len, a, pp[u], ex[u], qe);
                    const int32_t k = beg + (int32_t)(r + u - r0);
                    const uint16_t v = (uint16_t)(ml < 65535 ? ml : 65535);
                    S.hml[k] = v;
                    S.hfr[k] = fr[u];
                    const int d = ml - KI;
#pragma unroll
                    for (int t = 0; t < HB; ++t) g[t] += d >= t ? 1u : 0u;
                    if (ranked) topk_insert(top, v);
                }
            }
        }
    }
    S.hoff[a] = beg;
    S.hend[a] = beg + n;
    S.lz[0] = beg + n;
    uint32_t *dst = S.ge + (int64_t)a * HB;
#pragma unroll
    for (int t = 0; t < HB; ++t) dst[t] = g[t];
    fill_rk_top(occ, S, q, len, a, top);
}

// The lazy table's per-start inputs of read q (the host's; the device builds them wave-parallel in
// seed_kernels.hip): 12-mer codes, the KX bases after each start, the 4-bit copy, no start ready
SC_HD int build_starts(const IndexView &I, Scratch &S, const uint8_t *q, int len) {
    if (len > S.lmax) return SC_OVER_LEN;
    for (int a = 0; a <= len; ++a) {
        S.codes[a] = -1;
        S.qext[a] = 0;
        S.hoff[a] = 0;
        S.hend[a] = 0;
        S.ready[a] = a == len ? 1 : 0;
    }
    for (int a = 0; a + KI <= len; ++a) {
        const int n = len - a - KI;
        S.qext[a] = pack_ext(q + a + KI, n < KX ? n : KX);
    }
    uint32_t code = 0;
    int run = 0;
    for (int e = 0; e < len; ++e) {
        if (q[e] > 3) {
            run = 0;
            code = 0;
        } else {
            code = ((code << 2) | q[e]) & (NK - 1);
            ++run;
        }
        if (e - KI + 1 >= 0 && run >= KI) S.codes[e - KI + 1] = (int32_t)code;
    }
    if (S.q4w) {
        for (int w = 0; w <= (len >> 4) + 3; ++w) {
            uint64_t v = 0;
            for (int k = 0; k < 16; ++k) {
                const int x = w * 16 + k;
                const uint64_t c = x < len ? (q[x] < 4 ? q[x] : 4u) : 6u;
                v |= c << (4 * k);
            }
            S.q4w[w] = v;
        }
    }
    S.lz[0] = S.lz[1] = S.lz[2] = 0;
    return 0;
}

// -> 0 or SC_OVER_*
SC_HD int build_occ(const IndexView &I, Scratch &S, const uint8_t *q, int len) {
    if (len > S.lmax) return SC_OVER_LEN;
    for (int a = 0; a <= len; ++a) {
        S.hoff[a] = 0;
        S.codes[a] = -1;
        S.qext[a] = 0;
    }
    for (int64_t k = 0; k < (int64_t)len * HB; ++k) S.ge[k] = 0;
    for (int a = 0; a + KI <= len; ++a) {
        const int n = len - a - KI;
        S.qext[a] = pack_ext(q + a + KI, n < KX ? n : KX);
    }
    {
        uint32_t code = 0;
        int run = 0;
        for (int e = 0; e < len; ++e) {
            if (q[e] > 3) {
                run = 0;
                code = 0;
            } else {
                code = ((code << 2) | q[e]) & (NK - 1);
                ++run;
            }
            if (e - KI + 1 >= 0 && run >= KI) S.codes[e - KI + 1] = (int32_t)code;
        }
    }
    const uint8_t *T = I.text;
    int32_t nh = 0, prev0 = 0, prev1 = 0;   // hits of start a-1: [prev0, prev1)
    for (int a = 0; a + KI <= len; ++a) {
#if !defined(__HIP_DEVICE_COMPILE__)
        constexpr int PF_OFF = 24, PF_POS = 12;   // latency-bound on the host: prefetch ahead
        if (a + PF_OFF < len && S.codes[a + PF_OFF] >= 0) __builtin_prefetch(&I.koff[S.codes[a + PF_OFF]]);
        if (a + PF_POS < len && S.codes[a + PF_POS] >= 0) {
            const uint64_t r0 = I.koff[S.codes[a + PF_POS]];
            __builtin_prefetch(&I.kpos[r0]);
            __builtin_prefetch(&I.kext[r0]);
            __builtin_prefetch(&I.kext[r0] + 8);
        }
#endif
        S.hoff[a] = nh;
        if (S.codes[a] >= 0) {
            const uint32_t code = (uint32_t)S.codes[a];
            const uint64_t r0 = I.koff[code], r1 = I.koff[code + 1];
            if ((int64_t)nh + (int64_t)(r1 - r0) > S.cap_hits) return SC_OVER_HITS;
            uint32_t *g = S.ge + (int64_t)a * HB;
            int32_t k = prev0;
            for (uint64_t r = r0; r < r1; ++r) {
                const uint64_t p = hit_pos(I, code, r);
                while (k < prev1 && get_hpos(S, k) + 1 < p) ++k;
                int ml;
                if (k < prev1 && get_hpos(S, k) + 1 == p && S.hml[k] > KI) {
                    ml = S.hml[k] - 1;
                } else {
                    const uint64_t ex = I.kext[r];
                    const uint64_t qe = S.qext[a];
                    const int le = (int)(ex >> 56), lq = (int)(qe >> 56);
                    const uint64_t x = (ex ^ qe) & KX_MASK;
                    int m = x ? ctz64(x) >> 1 : KX;
                    m = m < le ? m : le;
                    m = m < lq ? m : lq;
                    ml = KI + m;
                    if (m == KX)
                        while (a + ml < len && q[a + ml] < 4 && T[p + ml] == q[a + ml]) ++ml;
                }
                set_hpos(S, nh, p);
                S.hfr[nh] = pack_fr(I, p);
                S.hml[nh] = (uint16_t)(ml < 65535 ? ml : 65535);
                ++nh;
                ++g[ml - KI < HB - 1 ? ml - KI : HB - 1];
            }
            for (int t = HB - 2; t >= 0; --t) g[t] += g[t + 1];
        }
        prev0 = S.hoff[a];
        prev1 = nh;
    }
    for (int a = len - KI + 1 < 0 ? 0 : len - KI + 1; a <= len; ++a) S.hoff[a] = nh;
    const Occ occ{&I, &S, q, len, nullptr};
    for (int a = 0; a < len; ++a) fill_rk(occ, S, q, len, a);
    return 0;
}

// ---------------------------------------------------------------- SMEMs
SC_HD void iv_reverse(Iv *v, int n) {
    for (int i = 0, j = n - 1; i < j; ++i, --j) {
        const Iv t = v[i];
        v[i] = v[j];
        v[j] = t;
    }
}

// bwt_smem1a (max_intv = 0): SMEMs covering x with >= min_intv occurrences, sorted by
// start, into mem[0, *nmem); returns the end of the longest forward match from x.
template <class OccT>
SC_HD int smem1(const OccT &occ, const Scratch &S, const uint8_t *q, int len, int x, int64_t min_intv, Iv *mem,
                int &nmem, int &err) {
    nmem = 0;
    if (q[x] > 3) return x + 1;
    SC_STAT(16, 1);
    if (min_intv < 1) min_intv = 1;
    Iv *curr = S.curr, *prev = S.prev;
    const int cap = S.cap_iv;
    int nc = 0, np = 0;
    Iv ik{x, x + 1, occ(x, x + 1)};
    int i;
    // the forward extension's counts for lengths 7..15 do not depend on each other: when the
    // 12-mer at x is N-free they are loaded up front (9 independent loads instead of a
    // dependent chain of table and count-row lookups); the same values as occ()
    uint32_t pre[9];
    const bool have = S.codes != nullptr && x + KI <= len && S.codes[x] >= 0;
    if (have) {
        occ.need(x);
        const uint32_t c12 = (uint32_t)S.codes[x];
#pragma unroll
        for (int n = 7; n < KI; ++n) pre[n - 7] = occ.I->cnt[n - 1][c12 >> (2 * (KI - n))];
#pragma unroll
        for (int n = KI; n < 16; ++n) pre[n - 7] = S.ge[(int64_t)x * HB + (n - KI)];
    }
    uint32_t blk[8];   // lengths 16..31: the start's count row 8 entries at a time
    int blk0 = -1;
    for (i = x + 1; i < len; ++i) {
        if (q[i] < 4) {
            const int n = i + 1 - x;
            int64_t o;
            int skip = 0;   // lengths n + 1 .. n + skip have the same count (Occ::scan_ge)
            if (SC_SCANGE && have && n >= KI + HB) {
                int mn;
                o = occ.scan_ge(x, n, mn);
                skip = mn > n ? mn - n : 0;   // (no read N inside a hit's match: q[x, x + mn) is N-free)
            } else if (have && n >= 7 && n < 16) {
                uint32_t v = pre[0];
#pragma unroll
                for (int t = 1; t < 9; ++t) v = n - 7 == t ? pre[t] : v;
                o = v;
            } else if (have && n >= 16 && n < KI + HB) {
                const int b0 = n & ~7;
                if (b0 != blk0) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) blk[t] = S.ge[(int64_t)x * HB + (b0 - KI) + t];
                    blk0 = b0;
                }
                uint32_t v = blk[0];
#pragma unroll
                for (int t = 1; t < 8; ++t) v = (n & 7) == t ? blk[t] : v;
                o = v;
            } else {
                o = occ(x, i + 1);
            }
            if (o != ik.occ) {
                if (nc >= cap) { err |= SC_OVER_IV; return len; }
                curr[nc++] = ik;
                if (o < min_intv) break;
            }
            i += skip;
            ik = Iv{x, i + 1, o};
        } else {
            if (nc >= cap) { err |= SC_OVER_IV; return len; }
            curr[nc++] = ik;
            break;
        }
    }
    if (i == len) {
        if (nc >= cap) { err |= SC_OVER_IV; return len; }
        curr[nc++] = ik;
    }
    const int ret = curr[nc - 1].end;   // the longest forward match
    (void)prev;
    (void)np;
    // Backward extension.  bwa extends the forward intervals (longest end first) one column
    // to the left at a time; an interval stops at the first column i with occ(i, end) <
    // min_intv, and is reported as [i + 1, end) when no longer-end interval survived that
    // column (and none was reported there).  Since occ(a, e) >= k holds for every a from x
    // down to the stopping column (it never shrinks as a moves right), an interval's stopping
    // start is a(e) = the lowest a <= x with R_k(a') >= e for all a' in [a, x), found by one
    // downward sweep over R_k as the ends decrease; the reported intervals are those whose
    // a(e) is strictly below the previous (longer-end) interval's.  Intervals bwa drops for an
    // occurrence count equal to a longer neighbour's share that neighbour's a(e) and are never
    // reported either.  Same SMEMs, one R_k load per column instead of one count lookup per
    // live interval per column.
    int a = x, last = x + 1;
    for (int j = nc - 1; j >= 0; --j) {
        const Iv p = curr[j];
        SC_STAT(17, 1);
        while (a > 0 && rmax_k(occ, S, q, len, a - 1, min_intv) >= p.end) --a;
        if (a < last) {
            if (nmem >= cap) { err |= SC_OVER_IV; return len; }
            mem[nmem++] = Iv{a, p.end, a == x ? p.occ : occ(a, p.end)};
            last = a;
        }
    }
    iv_reverse(mem, nmem);
    return ret;
}

// bwt_seed_strategy1: the shortest match from x longer than min_len with < max_intv hits
template <class OccT>
SC_HD int seed_strategy1(const OccT &occ, const uint8_t *q, int len, int x, int min_len, int64_t max_intv, Iv &m) {
    m = Iv{0, 0, 0};
    if (q[x] > 3) return x + 1;
    for (int i = x + 1; i < len; ++i) {
        if (q[i] > 3) return i + 1;
        if (i - x >= min_len) {
            const int n = i + 1 - x;
            int mn = 0;
            const int64_t o = SC_SCANGE && n >= KI + HB ? occ.scan_ge(x, n, mn) : occ(x, i + 1);
            if (o < max_intv) {
                m = Iv{x, i + 1, o};
                return i + 1;
            }
            if (mn > n) i += mn - n;   // the count holds up to length mn (Occ::scan_ge; q[x, x + mn) is N-free)
        }
    }
    return len;
}

// wall-clock ticks per part of a read's lane work (device, optional): [SMEM pass, re-seeding,
// -y seeds + sort, chaining, mem_chain_flt, filter + output]
#if defined(__HIP_DEVICE_COMPILE__)
#define SC_TICK(k)                                          \
    do {                                                    \
        if (ticks) {                                        \
            const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();   \
            ticks[k] += t_ - t_last;                        \
            t_last = t_;                                    \
        }                                                   \
    } while (0)
#else
#define SC_TICK(k) do { (void)ticks; } while (0)
#endif

// mem_collect_intv -> S.mems[0, return) sorted by (start, end), stable
template <class OccT>
SC_HD int collect_intv(const OccT &occ, Scratch &S, const pr_seed_opts &O, const uint8_t *q, int len, int &err,
                       unsigned long long *ticks = nullptr) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned long long t_last = ticks ? __builtin_amdgcn_s_memrealtime() : 0ULL;
#endif
    int nm = 0, n1 = 0;
    auto push = [&](const Iv &v) {
        if (nm >= S.cap_mems) {
            err |= SC_OVER_MEMS;
            return;
        }
        S.mems[nm++] = v;
    };
    for (int x = 0; x < len && !err;) {
        if (q[x] < 4) {
            x = smem1(occ, S, q, len, x, 1, S.m1, n1, err);
            for (int k = 0; k < n1; ++k)
                if (S.m1[k].end - S.m1[k].start >= O.min_seed_len) push(S.m1[k]);
        } else {
            ++x;
        }
    }
    SC_TICK(0);
    const int split_len = (int)(O.min_seed_len * O.split_factor + .499);
    const int nfirst = nm;
    for (int k = 0; k < nfirst && !err; ++k) {
        const Iv p = S.mems[k];
        if (p.end - p.start < split_len || p.occ > O.split_width) continue;
        smem1(occ, S, q, len, (p.start + p.end) >> 1, p.occ + 1, S.m1, n1, err);
        for (int j = 0; j < n1; ++j)
            if (S.m1[j].end - S.m1[j].start >= O.min_seed_len) push(S.m1[j]);
    }
    SC_TICK(1);
    if (O.max_mem_intv > 0) {
        for (int x = 0; x < len && !err;) {
            if (q[x] < 4) {
                Iv m;
                x = seed_strategy1(occ, q, len, x, O.min_seed_len, O.max_mem_intv, m);
                if (m.occ > 0) push(m);
            } else {
                ++x;
            }
        }
    }
    // stable sort by (start, end).  The three rounds each come out sorted by start, so a
    // counting sort by start (into the seed pool, free until mem_chain; the counts in `codes`,
    // which nothing reads after the occurrence lookups) and an insertion sort by end inside each
    // start's run (a few intervals) replace one insertion sort over all ~150 (quadratic moves)
    if (nm > 1 && S.cap_seeds >= nm && !err && !S.hend) {   // (the lazy table still needs `codes`)
        static_assert(sizeof(Seed) == sizeof(Iv), "the seed pool holds the sorted intervals");
        int32_t *cnt = S.codes;
        Iv *tmp = reinterpret_cast<Iv *>(S.seeds);
        for (int x = 0; x <= len; ++x) cnt[x] = 0;
        for (int i = 0; i < nm; ++i) ++cnt[S.mems[i].start + 1];
        for (int x = 1; x <= len; ++x) cnt[x] += cnt[x - 1];
        for (int i = 0; i < nm; ++i) {
            const Iv v = S.mems[i];
            tmp[cnt[v.start]++] = v;
        }
        for (int i = 0; i < nm; ++i) {
            const Iv v = tmp[i];
            int j = i - 1;
            while (j >= 0 && S.mems[j].start == v.start && S.mems[j].end > v.end) {
                S.mems[j + 1] = S.mems[j];
                --j;
            }
            S.mems[j + 1] = v;
        }
    } else {
        for (int i = 1; i < nm; ++i) {
            const Iv v = S.mems[i];
            int j = i - 1;
            while (j >= 0 && (S.mems[j].start > v.start || (S.mems[j].start == v.start && S.mems[j].end > v.end))) {
                S.mems[j + 1] = S.mems[j];
                --j;
            }
            S.mems[j + 1] = v;
        }
    }
    SC_TICK(2);
    return nm;
}

// ---------------------------------------------------------------- chaining
// ---------------------------------------------------------------- chain order
// mem_chain keeps its chains in a btree by pos (ties: creation order) and tests every
// occurrence against the chain with the largest pos <= its rbeg (the predecessor).
// test_and_merge never merges across long reads or strands, and every (long read, strand)
// is one contiguous range of the forward-reverse coordinate, so the predecessor can merge
// only when it lies in the occurrence's own range -- and then it is the last chain of that
// range with pos <= rbeg.  So the chains sit in one list per range (sorted by pos, ties in
// creation order), found through a small open-addressing table keyed by rid * 2 + strand;
// an occurrence with no such chain opens a new one.  mem_chain_flt's stable weight sort of
// the pos-ordered chains becomes one sort by (weight desc, pos, creation).  Round 2 kept
// one sorted array (every insert shifted ~40 entries, the seeding kernel's largest cost).
SC_HD int range_slot(const Scratch &S, int32_t key) {
    uint32_t h = ((uint32_t)key * 0x9E3779B1u) & (uint32_t)(S.hsize - 1);
    while (S.htab[h].key != -1 && S.htab[h].key != key) h = (h + 1) & (uint32_t)(S.hsize - 1);
    return (int)h;
}
SC_HD int32_t pack_ql(const Seed &s) { return (int32_t)(uint16_t)s.qbeg | ((int32_t)s.len << 16); }

// -> 1 merged, 0 not, -1 pool full
SC_HD int test_and_merge(const pr_seed_opts &O, int64_t l_pac, Scratch &S, int32_t &ns, Chain &c, const Seed &p,
                         int rid) {
    const Seed &last = S.seeds[c.tail];
    const Seed &first = S.seeds[c.head];
    const int64_t qend = last.qbeg + last.len, rend = last.rbeg + last.len;
    if (rid != c.rid) return 0;
    if (p.qbeg >= first.qbeg && p.qbeg + p.len <= qend && p.rbeg >= first.rbeg && p.rbeg + p.len <= rend)
        return 1;   // contained seed
    if ((last.rbeg < l_pac || first.rbeg < l_pac) && p.rbeg >= l_pac) return 0;   // other strand
    const int64_t x = p.qbeg - last.qbeg, y = p.rbeg - last.rbeg;
    if (y >= 0 && x - y <= O.w && y - x <= O.w && x - last.len < O.max_chain_gap && y - last.len < O.max_chain_gap) {
        if (ns >= S.cap_seeds) return -1;
        S.seeds[ns] = p;
        S.seeds[ns].nx = -1;
        S.seeds[c.tail].nx = ns;
        c.tail = ns++;
        ++c.n;
        return 1;
    }
    return 0;
}

// test_and_merge against a range's tail chain through its RangeRec copy (same decisions)
SC_HD int merge_tail(const pr_seed_opts &O, int64_t l_pac, Scratch &S, int32_t &ns, RangeRec &R, const Seed &p) {
    const int64_t f_rbeg = R.f_rbeg, l_rbeg = R.l_rbeg;
    const int f_q = (int16_t)(R.f_ql & 0xFFFF), l_q = (int16_t)(R.l_ql & 0xFFFF), l_len = R.l_ql >> 16;
    const int64_t qend = l_q + l_len, rend = l_rbeg + l_len;
    if (p.qbeg >= f_q && p.qbeg + p.len <= qend && p.rbeg >= f_rbeg && p.rbeg + p.len <= rend)
        return 1;   // contained seed
    if ((l_rbeg < l_pac || f_rbeg < l_pac) && p.rbeg >= l_pac) return 0;   // other strand
    const int64_t x = p.qbeg - l_q, y = p.rbeg - l_rbeg;
    if (y >= 0 && x - y <= O.w && y - x <= O.w && x - l_len < O.max_chain_gap && y - l_len < O.max_chain_gap) {
        if (ns >= S.cap_seeds) return -1;
        S.seeds[ns] = p;
        S.seeds[ns].nx = -1;
        S.seeds[R.l_idx].nx = ns;
        R.l_idx = ns++;
        R.l_rbeg = p.rbeg;
        R.l_ql = pack_ql(p);
        ++R.n;
        return 1;
    }
    return 0;
}
// the tail chain's authoritative fields back into its chain record
SC_HD void flush_tail(Scratch &S, const RangeRec &R) {
    S.cv[R.tail].tail = R.l_idx;
    S.cv[R.tail].n = R.n;
}

SC_HD int chain_weight(const Scratch &S, const Chain &c) {
    int64_t end = 0;
    int w = 0;
    for (int32_t k = c.head; k >= 0; k = S.seeds[k].nx) {
        const Seed &s = S.seeds[k];
        if (s.qbeg >= end) w += s.len;
        else if (s.qbeg + s.len > end) w += (int)(s.qbeg + s.len - end);
        end = end > s.qbeg + s.len ? end : s.qbeg + s.len;
    }
    const int tmp = w;
    w = 0;
    end = 0;
    for (int32_t k = c.head; k >= 0; k = S.seeds[k].nx) {
        const Seed &s = S.seeds[k];
        if (s.rbeg >= end) w += s.len;
        else if (s.rbeg + s.len > end) w += (int)(s.rbeg + s.len - end);
        end = end > s.rbeg + s.len ? end : s.rbeg + s.len;
    }
    w = w < tmp ? w : tmp;
    return w < (1 << 30) ? w : (1 << 30) - 1;
}

SC_HD int cal_max_gap(const pr_seed_opts &O, int qlen) {
    int l_del = (int)((double)(qlen * O.a - O.o_del) / O.e_del + 1.);
    int l_ins = (int)((double)(qlen * O.a - O.o_ins) / O.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < O.w << 1 ? l : O.w << 1;
}

// ---------------------------------------------------------------- mem_flt_chained_seeds
// min_HSP_score of mem_flt_chained_seeds for a read of len bases, or -1 when bwa skips the
// filter ("don't run the following for short reads"): min_l = MEM_HSP_COEF (1.1f) * W in
// float arithmetic, compared with MEM_SEEDSW_COEF (0.05f) * len, as bwamem.c computes them
SC_HD int seed_flt_min_score(const pr_seed_opts &O, int len) {
    double min_l;
    if (O.min_chain_weight) min_l = (double)(1.1f * (float)O.min_chain_weight);
    else min_l = (double)5.5f * log((double)len);   // MEM_MINSC_COEF * log(l_query)
    if (min_l > (double)(0.05f * (float)len)) return -1;
    return (int)(O.a * min_l + .499);
}

// mem_seed_sw: the best local score (ksw_align2: affine gaps, a gap of k bases costs o + k e,
// deletions o_del/e_del, insertions o_ins/e_ins; match a, mismatch -b, N -1) of the read
// around seed s against the reference around it, or -1 when the seed or a window reaches
// MEM_SHORT_LEN (200) bases.  Windows: +- MEM_SHORT_EXT (50), clamped to [0, 2 l_pac) and to
// the seed's strand half, then (bns_fetch_seq) to its long read.  H / E: 2 x 201 ints.
// (H / E: rows of 201 values at a stride -- int32 on one thread, or int16 interleaved over
// the lanes of a wave; every value is <= 5 x 200)
template <class T>
SC_HD int seed_sw_score(const IndexView &I, const pr_seed_opts &O, const uint8_t *q, int len, const Seed &s, int rid,
                        T *H, T *E, int stride = 1) {
    if (s.len >= 200) return -1;
    int qb = s.qbeg - 50, qe = s.qbeg + s.len + 50;
    qb = qb > 0 ? qb : 0;
    qe = qe < len ? qe : len;
    int64_t rb = s.rbeg - 50, re = s.rbeg + s.len + 50;
    const int64_t mid = (s.rbeg + s.rbeg + s.len) >> 1;
    rb = rb > 0 ? rb : 0;
    re = re < (I.l_pac << 1) ? re : (I.l_pac << 1);
    if (rb < I.l_pac && I.l_pac < re) {
        if (mid < I.l_pac) re = I.l_pac;
        else rb = I.l_pac;
    }
    if (qe - qb >= 200 || re - rb >= 200) return -1;
    const bool rev = mid >= I.l_pac;
    const int64_t fb = rev ? (I.l_pac << 1) - I.lr_off[rid + 1] : I.lr_off[rid];
    const int64_t fe = rev ? (I.l_pac << 1) - I.lr_off[rid] : I.lr_off[rid + 1];
    rb = rb > fb ? rb : fb;
    re = re < fe ? re : fe;
    // the text: forward long reads, then the reverse complement of their concatenation
    const int64_t tc = rev ? I.cstart[2 * I.n_lr - 1 - rid] : I.cstart[rid];
    const uint8_t *t = I.text + tc + (rb - fb);
    const int qn = qe - qb, tn = (int)(re - rb);
    const int oe_del = O.o_del + O.e_del, oe_ins = O.o_ins + O.e_ins;
    for (int j = 0; j < qn; ++j) H[j * stride] = 0, E[j * stride] = 0;
    int best = 0;
    for (int i = 0; i < tn; ++i) {
        const int ti = t[i];
        int hdiag = 0, f = 0;
        for (int j = 0; j < qn; ++j) {
            const int qj = q[qb + j];
            const int sc = (ti > 3 || qj > 3) ? -1 : (ti == qj ? O.a : -O.b);
            int h = hdiag + sc;
            const int e = E[j * stride];
            h = h > e ? h : e;
            h = h > f ? h : f;
            h = h > 0 ? h : 0;
            hdiag = H[j * stride];
            H[j * stride] = (T)h;
            best = best > h ? best : h;
            int en = e - O.e_del, eo = h - oe_del;
            en = en > eo ? en : eo;
            E[j * stride] = (T)(en > 0 ? en : 0);
            int fn = f - O.e_ins, fo = h - oe_ins;
            fn = fn > fo ? fn : fo;
            f = fn > 0 ? fn : 0;
        }
    }
    return best;
}

SC_HD void chain_flt(const pr_seed_opts &O, Scratch &S, int ncv, int *n_chains);
template <bool LZ = false>
SC_HD int chain_seq(const IndexView &I, const pr_seed_opts &O, Scratch &S, int nm, int *n_cv);

// Everything after the occurrence table (S.hoff / hpos / hml / ge of the read, built by
// build_occ or by the device's wave-parallel equivalent): SMEMs, chaining, the chain
// filter and the tasks into out[0, *n_out) (chain order after mem_chain_flt).
// Returns 0 or an SC_OVER_* mask (then the read's output is not valid).
// ticks (device, optional): wall-clock ticks added per part [SMEMs, chaining, filter + output]
// Part 1: SMEMs, chaining and mem_chain_flt; *n_chains = the chains in S.ch (kept flags set).
template <bool LZ = false>
SC_HD int map_chains(const IndexView &I, const pr_seed_opts &O, Scratch &S, const uint8_t *q, int len, int *n_chains,
                     unsigned long long *ticks = nullptr, const uint32_t *lcnt = nullptr) {
    *n_chains = 0;
    int err = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned long long t_last = ticks ? __builtin_amdgcn_s_memrealtime() : 0ULL;
#endif
    const OccB<LZ> occ{&I, &S, q, len, lcnt};
    const int nm = collect_intv(occ, S, O, q, len, err, ticks);
    if (LZ) err |= S.lz[1];   // the lazy table's pool overflowed: the counts are not valid
    if (err) return err;
    SC_STAT(0, 1);
    SC_STAT(1, nm);
#if defined(__HIP_DEVICE_COMPILE__)
    if (ticks) t_last = __builtin_amdgcn_s_memrealtime();
#endif
    int ncv = 0;
    err = chain_seq<LZ>(I, O, S, nm, &ncv);
    if (LZ) err |= S.lz[1];
    if (err) return err;
    SC_TICK(3);
    SC_STAT(11, ncv);
    SC_STAT(12, (unsigned long long)ncv * ncv);
    chain_flt(O, S, ncv, n_chains);
    SC_TICK(4);
    return 0;
}

// mem_chain over the SMEMs S.mems[0, nm) -> the chains S.cv[0, *n_cv) in creation order
// (one thread); 0 or SC_OVER_SEEDS / SC_OVER_CHAINS
template <bool LZ>
SC_HD int chain_seq(const IndexView &I, const pr_seed_opts &O, Scratch &S, int nm, int *n_cv) {
    int32_t ns = 0, ncv = 0, nrg = 0;
    for (int k = 0; k < S.hsize; ++k) S.htab[k].key = -1;
    for (int mi = 0; mi < nm; ++mi) {
        const Iv p = S.mems[mi];
        const int slen = p.end - p.start;
        // (lazy table: every SMEM's start was counted by the SMEM search, so it is materialized)
        if (LZ && !S.ready[p.start]) return SC_OVER_HITS;
        const int32_t h0 = S.hoff[p.start], h1 = LZ ? S.hend[p.start] : S.hoff[p.start + 1];
        // the SMEM's occurrence count is the number of the start's hits with ml >= slen
        // (every interval's occ comes from the same per-start table, slen >= 12)
        const int64_t np = p.occ;
        const int64_t step = np > O.max_occ ? np / O.max_occ : 1;
        int64_t fidx = 0, take = 0, count = 0;
        // the selected occurrences in batches of CB: their forward-reverse coordinates and
        // range-table probes are independent loads, issued together (one latency per batch
        // instead of several dependent ones per occurrence); then each in order
        constexpr int CB = 8;
        int32_t k = h0;
        while (k < h1 && count < O.max_occ) {
            int32_t sel[CB];
            int nsel = 0;
            while (k < h1 && count < O.max_occ && nsel < CB) {
                // the start's match lengths 8 at a time (independent loads), then in order
                uint16_t ml[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) ml[u] = k + u < h1 ? S.hml[k + u] : (uint16_t)0;
                int u = 0;
                for (; u < 8 && k < h1 && count < O.max_occ && nsel < CB; ++u, ++k) {
                    if (ml[u] < slen) continue;   // text-position order: the 12-mer lists are sorted
                    const bool use = fidx == take;
                    ++fidx;
                    if (!use) continue;
                    take += step;
                    ++count;
                    sel[nsel++] = k;
                }
            }
            int64_t rb[CB];
            int rd[CB], hsl[CB];
            int32_t key[CB];
#pragma unroll
            for (int u = 0; u < CB; ++u) {
                const uint64_t v = u < nsel ? S.hfr[sel[u]] : 0ull;   // coordinates from the occurrence table
                rb[u] = (int64_t)(v >> FR_RID_BITS);
                rd[u] = (int)(v & ((1u << FR_RID_BITS) - 1u));
                key[u] = rd[u] * 2 + (rb[u] >= I.l_pac ? 1 : 0);
            }
#pragma unroll
            for (int u = 0; u < CB; ++u) hsl[u] = u < nsel ? range_slot(S, key[u]) : 0;
            bool opened = false;   // a range opened in this batch moves later probes: redo them
            for (int u = 0; u < nsel; ++u) {
                SC_STAT(3, 1);
                Seed s;
                s.rbeg = rb[u];
                s.qbeg = (int16_t)p.start;
                s.len = (int16_t)slen;
                s.nx = -1;
                const int rid = rd[u];
                // the predecessor that can merge: the last chain of the occurrence's range with
                // pos <= rbeg (`at`, also the insertion point); occurrences at one locus mostly
                // come in increasing rbeg, so the list's tail (its RangeRec copy) first
                const int hs = opened ? range_slot(S, key[u]) : hsl[u];
                const RangeEnt e = S.htab[hs];
                const bool found = e.key == key[u];
                int at = -1;
                bool at_tail = false;
                if (found) {
                    RangeRec &R = S.rg[e.r];
                    SC_STAT(4, 1);
                    if (R.tpos <= s.rbeg) {
                        at = R.tail;
                        at_tail = true;
                    } else {
                        for (int x = R.head; x >= 0 && S.cv[x].pos <= s.rbeg; x = S.cnx[x]) {
                            at = x;
                            SC_STAT(4, 1);
                        }
                    }
                    if (at >= 0) {
                        const int r = at_tail ? merge_tail(O, I.l_pac, S, ns, R, s)
                                              : test_and_merge(O, I.l_pac, S, ns, S.cv[at], s, rid);
                        if (r < 0) return SC_OVER_SEEDS;
                        if (r) { SC_STAT(5, 1); continue; }
                    }
                }
                SC_STAT(6, 1);
                if (ncv >= S.cap_chains) return SC_OVER_CHAINS;
                if (ns >= S.cap_seeds) return SC_OVER_SEEDS;
                S.seeds[ns] = s;
                Chain c;
                c.pos = s.rbeg;
                c.rid = rid;
                c.head = c.tail = ns;
                c.n = 1;
                c.w = c.kept = 0;
                c.first = -1;
                S.cv[ncv] = c;
                if (!found) {   // the range's first chain
                    RangeRec &R = S.rg[nrg];
                    R.head = R.tail = ncv;
                    R.n = 1;
                    R.l_idx = ns;
                    R.tpos = s.rbeg;
                    R.f_rbeg = R.l_rbeg = s.rbeg;
                    R.f_ql = R.l_ql = pack_ql(s);
                    S.htab[hs].key = key[u];
                    S.htab[hs].r = nrg++;
                    S.cnx[ncv] = -1;
                    opened = true;
                } else {
                    RangeRec &R = S.rg[e.r];
                    if (at < 0) {   // before every chain of the range
                        S.cnx[ncv] = R.head;
                        R.head = ncv;
                    } else {   // after `at` (and after every chain of equal pos)
                        const int nx = S.cnx[at];
                        S.cnx[ncv] = nx;
                        S.cnx[at] = ncv;
                        if (nx < 0) {   // the new tail: the old one's fields back into its record
                            flush_tail(S, R);
                            R.tail = ncv;
                            R.n = 1;
                            R.l_idx = ns;
                            R.tpos = s.rbeg;
                            R.f_rbeg = R.l_rbeg = s.rbeg;
                            R.f_ql = R.l_ql = pack_ql(s);
                        }
                    }
                }
                ++ns;
                ++ncv;
            }
        }
    }
    for (int r = 0; r < nrg; ++r) flush_tail(S, S.rg[r]);
    *n_cv = ncv;
    return 0;
}

// mem_chain_flt over the chains S.cv[0, ncv) in creation order -> S.ch[0, *n_chains) with their
// kept flags: the weight filter, then bwa's stable sort by weight (descending) of the
// pos-ordered chains = a sort by (weight desc, pos, creation order = first seed's index)
SC_HD void chain_flt(const pr_seed_opts &O, Scratch &S, int ncv, int *n_chains) {
    int nch = 0;
    for (int j = 0; j < ncv; ++j) {
        Chain c = S.cv[j];
        c.w = chain_weight(S, c);
        if (c.w >= O.min_chain_weight) S.ch[nch++] = c;
    }
    for (int i = 1; i < nch; ++i) {
        const Chain v = S.ch[i];
        int j = i - 1;
        while (j >= 0 && (S.ch[j].w < v.w || (S.ch[j].w == v.w && (S.ch[j].pos > v.pos ||
                                                                   (S.ch[j].pos == v.pos && S.ch[j].head > v.head))))) {
            S.ch[j + 1] = S.ch[j];
            --j;
            SC_STAT(13, 1);
        }
        S.ch[j + 1] = v;
    }
    if (nch > 0) {
        int nk = 1;
        S.kept[0] = 0;
        S.ch[0].kept = 3;
        for (int i = 1; i < nch; ++i) {
            int large = 0, k;
            const int bi = S.seeds[S.ch[i].head].qbeg;
            const int ei = S.seeds[S.ch[i].tail].qbeg + S.seeds[S.ch[i].tail].len;
            for (k = 0; k < nk; ++k) {
                Chain &cj = S.ch[S.kept[k]];
                const int bj = S.seeds[cj.head].qbeg;
                const int ej = S.seeds[cj.tail].qbeg + S.seeds[cj.tail].len;
                const int bmax = bj > bi ? bj : bi;
                const int emin = ej < ei ? ej : ei;
                if (emin > bmax) {
                    const int li = ei - bi, lj = ej - bj;
                    const int minl = li < lj ? li : lj;
                    if (emin - bmax >= minl * O.mask_level && minl < O.max_chain_gap) {
                        large = 1;
                        if (cj.first < 0) cj.first = i;
                        if (S.ch[i].w < cj.w * O.drop_ratio && cj.w - S.ch[i].w >= O.min_seed_len << 1) break;
                    }
                }
            }
            if (k == nk) {
                S.kept[nk++] = i;
                S.ch[i].kept = large ? 2 : 3;
            }
        }
        for (int k = 0; k < nk; ++k)
            if (S.ch[S.kept[k]].first >= 0) S.ch[S.ch[S.kept[k]].first].kept = 1;
    }
    *n_chains = nch;
}

// The seeds whose mem_flt_chained_seeds score part 2 needs (every seed of every kept chain,
// chain order) into list[0, return); -1 when they do not fit cap
SC_HD int flt_seed_list(const Scratch &S, int nch, int32_t *list, int cap) {
    int n = 0;
    for (int ci = 0; ci < nch; ++ci) {
        const Chain &c = S.ch[ci];
        if (c.kept == 0) continue;
        for (int32_t k = c.head; k >= 0; k = S.seeds[k].nx) {
            if (n >= cap) return -1;
            list[n++] = k;
        }
    }
    return n;
}

// Part 2: mem_flt_chained_seeds over the kept chains (long reads only) and the tasks into
// out[0, *n_out).  scores: the seeds' seed_sw_score by seed index when computed beforehand
// (the device's one-wave-per-read pass scores them over all lanes), else null.
// dp16 (device, lane per read): the SW rows as int16 interleaved over the wave's lanes (dp16 =
// the wave's area + lane, stride 64: the lanes' row accesses share cache lines), else the
// int32 rows in `ge`.
SC_HD int map_output(const IndexView &I, const pr_seed_opts &O, Scratch &S, const uint8_t *q, int len, int sid,
                     int nch, pr_seed_task *out, int cap_out, int *n_out, const int32_t *scores = nullptr,
                     unsigned long long *ticks = nullptr, int16_t *dp16 = nullptr) {
    *n_out = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned long long t_last = ticks ? __builtin_amdgcn_s_memrealtime() : 0ULL;
#endif
    // (the occurrence table's per-start array `ge` is dead by now and holds the SW rows)
    const int flt = seed_flt_min_score(O, len);
    int32_t *swH = (int32_t *)S.ge, *swE = swH + 201;
    // mem_chain2aln's input: every seed of every kept chain with the chain's reference window,
    // seeds in the order mem_chain2aln tries them (srt: score -- the length, or the seed SW
    // score after mem_flt_chained_seeds -- then the larger index first on ties); a chain the
    // filter empties is never extended (mem_chain2aln returns on c->n == 0)
    int no = 0, nkept = 0;
    for (int ci = 0; ci < nch; ++ci) {
        const Chain &c = S.ch[ci];
        if (c.kept == 0) continue;
        const bool rev = S.seeds[c.head].rbeg >= I.l_pac;
        const int64_t L = I.lr_off[c.rid + 1] - I.lr_off[c.rid];
        const int64_t cs = rev ? I.l_pac + (I.l_pac - I.lr_off[c.rid + 1]) : I.lr_off[c.rid];
        if (no + c.n > cap_out) return SC_OVER_OUT;
        const int first = no;
        int idx = 0;
        int64_t r0 = INT64_MAX, r1 = INT64_MIN;
        for (int32_t k = c.head; k >= 0; k = S.seeds[k].nx) {
            const Seed &s = S.seeds[k];
            int score = s.len;
            if (flt >= 0) {
                const int x = scores ? scores[k]
                                     : (dp16 ? seed_sw_score(I, O, q, len, s, c.rid, dp16, dp16 + 201 * 64, 64)
                                             : seed_sw_score(I, O, q, len, s, c.rid, swH, swE));
                if (x >= 0 && x < flt) continue;   // dropped
                score = x < 0 ? s.len * O.a : x;
            }
            // the chain's window over its (remaining) seeds
            const int64_t b = s.rbeg - (s.qbeg + cal_max_gap(O, s.qbeg));
            const int64_t e = s.rbeg + s.len + ((len - s.qbeg - s.len) + cal_max_gap(O, len - s.qbeg - s.len));
            r0 = r0 < b ? r0 : b;
            r1 = r1 > e ? r1 : e;
            pr_seed_task &t = out[no];
            t.sr = sid;
            t.lr = c.rid;
            t.strand = rev ? 1 : 0;
            t.qbeg = s.qbeg;
            t.rbeg = (int32_t)(s.rbeg - cs);
            t.slen = s.len;
            t.chain = nkept;
            t.rmax0 = score;   // the srt key (score, index) until the sort below: rmax0 / rank
            t.rank = idx++;
            // insertion sort by (score, index) descending
            int j = no - 1;
            while (j >= first && (out[j].rmax0 < t.rmax0 || (out[j].rmax0 == t.rmax0 && out[j].rank < t.rank))) --j;
            const pr_seed_task v = t;
            for (int m = no; m > j + 1; --m) out[m] = out[m - 1];
            out[j + 1] = v;
            ++no;
        }
        if (no == first) continue;
        r0 -= cs;
        r1 -= cs;
        for (int m = first; m < no; ++m) {
            out[m].rank = m - first;
            out[m].rmax0 = (int32_t)(r0 > 0 ? r0 : 0);
            out[m].rmax1 = (int32_t)(r1 < L ? r1 : L);
        }
        ++nkept;
    }
    *n_out = no;
    SC_STAT(14, nch);
    SC_STAT(15, no);
    SC_TICK(5);
    return 0;
}

// Everything after the occurrence table: parts 1 and 2 on one thread.
template <bool LZ = false>
SC_HD int map_after_occ(const IndexView &I, const pr_seed_opts &O, Scratch &S, const uint8_t *q, int len, int sid,
                        pr_seed_task *out, int cap_out, int *n_out, unsigned long long *ticks = nullptr,
                        const uint32_t *lcnt = nullptr, int16_t *dp16 = nullptr) {
    *n_out = 0;
    int nch = 0;
    const int err = map_chains<LZ>(I, O, S, q, len, &nch, ticks, lcnt);
    if (err) return err;
    return map_output(I, O, S, q, len, sid, nch, out, cap_out, n_out, nullptr, ticks, dp16);
}
#undef SC_TICK

// The whole read: occurrence table (the lazy one when S has it), then map_after_occ.
SC_HD int map_read(const IndexView &I, const pr_seed_opts &O, Scratch &S, const uint8_t *q, int len, int sid,
                   pr_seed_task *out, int cap_out, int *n_out) {
    *n_out = 0;
    if (S.hend) {
        const int err = build_starts(I, S, q, len);
        return err ? err : map_after_occ<true>(I, O, S, q, len, sid, out, cap_out, n_out);
    }
    const int err = build_occ(I, S, q, len);
    return err ? err : map_after_occ<false>(I, O, S, q, len, sid, out, cap_out, n_out);
}

// Whether the device path builds the lazy occurrence table for these options: the finish tasks'
// near-exact mapping (-k >= 17: bwa-sr-finish, bwa-mr-finish) consults a few starts per read
// (its SMEMs run to the read's end), the iterations' noisy mapping nearly every start.  Either
// table gives the same seeds; only the cost differs.
SC_HD bool lazy_occ(const pr_seed_opts &O) { return O.min_seed_len >= 17; }

}  // namespace seedc
}  // namespace prgpu

namespace prgpu {
namespace seedc {

// Fixed scratch capacities of the device path (one lane per read).  Reads that
// need more are flagged with the SC_OVER_* bit of the array that overflowed.
struct Caps {
    int32_t lmax, hits, iv, mems, seeds, chains, out;
    int32_t hi;      // the text reaches beyond 2^32: the hit table carries bit 32 of the positions (hhi)
    int32_t nopos;   // no hit positions (hpos / hhi): the device's tables keep only the chaining's
                     // coordinates (hfr); the host's build_occ follows diagonals through hpos
    int32_t lazy;    // the lazy occurrence table (Scratch.hend / ready / q4w / lz)
};
// output slots per read (the seeds of its kept chains): 384 for short reads, 2 per base for
// the mr modes' 300-1000 bp reads (~300 seeds per 600 bp read at 15x long-read coverage)
SC_HD int device_out_cap(int qmax) { return qmax > 192 ? 2 * ((qmax + 15) & ~15) : 384; }
SC_HD Caps device_caps(int qmax = 0) {
    Caps c{1024, 8192, 256, 1024, 8192, 4096, 384, 0};   // (seeds / chains: pass 2 chains reads of up to ~6.8 k occurrences over the wave)
    c.out = device_out_cap(qmax);
    if (qmax > 192) {   // pass 2 for mr reads: at least twice pass 1's room (device_caps_small)
        const int l = (qmax + 15) & ~15;
        c.hits = c.hits > 48 * l ? c.hits : 48 * l;
        c.iv = c.iv > l / 2 ? c.iv : l / 2;
        c.mems = c.mems > 2 * l ? c.mems : 2 * l;
        c.seeds = c.seeds > 4 * l ? c.seeds : 4 * l;
        c.chains = c.chains > 2 * l ? c.chains : 2 * l;
    }
    return c;
}
// pass 1 of the device path: 64 slices per wave, sized for reads of <= lmax bases.  Reads
// beyond 160 bases (mr modes) get hit / interval / seed / chain room in proportion to their
// length (a 600 bp read at 15x long-read coverage has ~9k hits), so they stay in the lane-per-read
// pass instead of the one-wave-per-read pass 2; configs[1]'s 150 bp slices are unchanged.
SC_HD Caps device_caps_small(int lmax) {
    const int l = lmax < 16 ? 16 : (lmax + 15) & ~15;
    Caps c{l, 4096, 64, 512, 512, 384, device_out_cap(lmax), 0};   // ~0.1 % of configs[1]'s reads outgrow it (mems)
    if (l > 160) {
        c.hits = c.hits > 24 * l ? c.hits : 24 * l;
        c.iv = c.iv > l / 4 ? c.iv : l / 4;
        c.mems = c.mems > 2 * l ? c.mems : 2 * l;
        c.seeds = c.seeds > 2 * l ? c.seeds : 2 * l;
        c.chains = c.chains > l ? c.chains : l;
    }
    return c;
}

SC_HD int64_t align8(int64_t x) { return (x + 7) & ~(int64_t)7; }
SC_HD int32_t range_table_size(int32_t chains) {
    int32_t h = 64;
    while (h < 2 * chains) h <<= 1;
    return h;
}

// bytes of one lane's scratch slice
SC_HD int64_t scratch_bytes(const Caps &c) {
    int64_t b = 0;
    b += align8(4 * (int64_t)(c.lmax + 1));              // hoff
    b += align8(8 * (int64_t)(c.lmax + 1));              // qext
    b += align8(4 * (int64_t)(c.lmax + 1));              // codes
    b += align8(4 * (int64_t)c.lmax * HB);               // ge
    if (!c.nopos) b += align8(4 * (int64_t)c.hits);      // hpos
    b += align8(2 * (int64_t)c.hits);                    // hml
    b += align8((int64_t)sizeof(Iv) * c.mems);           // mems
    b += 3 * align8((int64_t)sizeof(Iv) * c.iv);         // m1, curr, prev
    b += align8((int64_t)sizeof(Seed) * c.seeds);        // seeds
    b += 2 * align8((int64_t)sizeof(Chain) * c.chains);  // cv, ch
    b += 2 * align8(4 * (int64_t)c.chains);              // cnx, kept
    b += align8((int64_t)sizeof(RangeEnt) * range_table_size(c.chains));   // htab
    b = (b + 63) & ~(int64_t)63;                         // (rg 64-byte aligned)
    b += align8((int64_t)sizeof(RangeRec) * c.chains);   // rg
    b += align8(2 * (int64_t)(c.lmax + 1) * RK);         // rmax
    b += align8(8 * (int64_t)c.hits);                    // hfr
    if (c.hi && !c.nopos) b += align8((int64_t)c.hits);  // hhi
    if (c.lazy) {
        b += align8(4 * (int64_t)(c.lmax + 1));          // hend
        b += align8((int64_t)(c.lmax + 1));              // ready
        b += align8(8 * (int64_t)(c.lmax / 16 + 4));     // q4w
        b += align8(16);                                 // lz
    }
    return (b + 63) & ~(int64_t)63;                      // (slices 64-byte aligned)
}

// lay a Scratch over an 8-byte aligned slice of scratch_bytes(c) bytes
SC_HD Scratch carve(uint8_t *p, const Caps &c) {
    Scratch S{};
    auto take = [&p](int64_t bytes) {
        uint8_t *r = p;
        p += align8(bytes);
        return r;
    };
    S.lmax = c.lmax;
    S.hoff = (int32_t *)take(4 * (int64_t)(c.lmax + 1));
    S.qext = (uint64_t *)take(8 * (int64_t)(c.lmax + 1));
    S.codes = (int32_t *)take(4 * (int64_t)(c.lmax + 1));
    S.ge = (uint32_t *)take(4 * (int64_t)c.lmax * HB);
    S.hpos = c.nopos ? nullptr : (uint32_t *)take(4 * (int64_t)c.hits);
    S.hml = (uint16_t *)take(2 * (int64_t)c.hits);
    S.cap_hits = c.hits;
    S.mems = (Iv *)take((int64_t)sizeof(Iv) * c.mems);
    S.cap_mems = c.mems;
    S.m1 = (Iv *)take((int64_t)sizeof(Iv) * c.iv);
    S.curr = (Iv *)take((int64_t)sizeof(Iv) * c.iv);
    S.prev = (Iv *)take((int64_t)sizeof(Iv) * c.iv);
    S.cap_iv = c.iv;
    S.seeds = (Seed *)take((int64_t)sizeof(Seed) * c.seeds);
    S.cap_seeds = c.seeds;
    S.cv = (Chain *)take((int64_t)sizeof(Chain) * c.chains);
    S.ch = (Chain *)take((int64_t)sizeof(Chain) * c.chains);
    S.cnx = (int32_t *)take(4 * (int64_t)c.chains);
    S.kept = (int32_t *)take(4 * (int64_t)c.chains);
    S.hsize = range_table_size(c.chains);
    S.htab = (RangeEnt *)take((int64_t)sizeof(RangeEnt) * S.hsize);
    p = (uint8_t *)(((uintptr_t)p + 63) & ~(uintptr_t)63);   // (scratch_bytes' alignment of rg)
    S.rg = (RangeRec *)take((int64_t)sizeof(RangeRec) * c.chains);
    S.cap_chains = c.chains;
    S.rmax = (uint16_t *)take(2 * (int64_t)(c.lmax + 1) * RK);
    S.hfr = (uint64_t *)take(8 * (int64_t)c.hits);
    S.hhi = c.hi && !c.nopos ? (uint8_t *)take((int64_t)c.hits) : nullptr;
    if (c.lazy) {
        S.hend = (int32_t *)take(4 * (int64_t)(c.lmax + 1));
        S.ready = (uint8_t *)take((int64_t)(c.lmax + 1));
        S.q4w = (uint64_t *)take(8 * (int64_t)(c.lmax / 16 + 4));
        S.lz = (int32_t *)take(16);
    }
    return S;
}

}  // namespace seedc
}  // namespace prgpu
