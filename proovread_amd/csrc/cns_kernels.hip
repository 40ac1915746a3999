// Consensus (pileup) kernels for gfx950 — proovread's Sam::Seq engine as driven
// by bin/bam2cns, one long read per workgroup.
//
// One persistent launch; each 256-thread workgroup dequeues long reads and runs,
// with the read's data on chip:
//   1. alignment prep          Alignment.pm:417-431 length, 525-546 ncscore,
//                              Seq.pm:1354 bin, Seq.pm:270-385 clip/taboo trim
//   2. bin capping             Seq.pm:582-614 add_aln_by_score / 639 remove_aln_by_iid
//                              (stable counting sort by bin in LDS, one thread per bin)
//   3. insertion-state table   Seq.pm:446-448 first-seen state indices, as an LDS hash
//                              keyed by the state string with atomicMin first-seen order
//   4. windowed pileup         Seq.pm:438-461 scatter into per-column state counts
//                              (LDS atomics, 512-column windows) and
//                              Seq.pm:1568-1654 argmax / phred / trace, block scans
//   5. Trace2cigar             Seq.pm:206-225 run-length encoding
//   6. chimera                 Seq.pm:774-889 + bam2cns:461-491
//
// No MFMA: nothing here is a dense contraction.  The roofline is HBM (reads
// of SEQ/CIGAR/reference, writes of consensus), see DESIGN.md.
// Build flags include -ffp-contract=off: every double op of the Perl code is
// evaluated separately (bit-exact ncscore / Phreds2freqs / Freqs2phreds).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cns_dev.h"

namespace prgpu {

// ---------------------------------------------------------------------------
// numeric helpers (Seq.pm:136-156)
__device__ __forceinline__ double phred2freq(int p) {
    double x = __dadd_rn(__dmul_rn(__ddiv_rn(__dmul_rn((double)p, (double)p), 120.0), 100.0), 0.5);
    return __ddiv_rn((double)(long long)x, 100.0);
}
__device__ __forceinline__ int freq2phred(double f) {
    double x = __dadd_rn(__dsqrt_rn(__dmul_rn(f, 120.0)), 0.5);
    long long p = (long long)x;
    return p > 40 ? 40 : (int)p;
}
// Seq.pm:531-539 fixed states; unknown single chars look up undef -> index 0
__device__ __forceinline__ int fixed_idx(uint8_t c) {
    switch (c) {
        case 'A': return 0;
        case 'T': return 1;
        case 'G': return 2;
        case 'C': return 3;
        case '-': return 4;
        case 'N': return 5;
        default: return 0;
    }
}
__device__ __forceinline__ int code5(uint8_t c) {
    switch (c) {
        case 'A': return 1;
        case 'C': return 2;
        case 'G': return 3;
        case 'T': return 4;
        case 'N': return 5;
        default: return 0;
    }
}
// nt4 code (0-4) -> 'A','C','G','T','N' without a memory table
__device__ __forceinline__ uint8_t nt4_ascii(uint32_t c) { return (uint8_t)(0x4E54474341ULL >> (8 * c)); }
// injective key for insertion-state strings of <=19 chars over ACGTN, else a
// 63-bit FNV-1a hash with the top bit set (collision note)
// Read-only view of an alignment's SEQ as SAM prints it: the stored bytes are
// ASCII or nt4 codes (0-4, bwa's nst_nt4_table); `rc` means SEQ is the reverse
// complement of the stored read (GPU pipeline: bwa prints reverse-strand hits
// reverse-complemented, bwamem.c mem_aln2sam).
struct SeqV {
    const uint8_t *p;
    int n;
    bool rc, nt4;
    __device__ __forceinline__ uint8_t operator[](int s) const {
        uint8_t c = rc ? p[n - 1 - s] : p[s];
        if (nt4) {
            if (c > 4) c = 4;
            if (rc && c < 4) c = (uint8_t)(3 - c);
            return nt4_ascii(c);
        }
        if (rc) {
            switch (c) {
                case 'A': return 'T';
                case 'C': return 'G';
                case 'G': return 'C';
                case 'T': return 'A';
                default: return c;
            }
        }
        return c;
    }
};
__device__ __forceinline__ uint64_t state_key(const SeqV &v, int off, int n) {
    if (n <= 19) {
        uint64_t k = (uint64_t)n << 57;
        bool ok = true;
        for (int i = 0; i < n; ++i) {
            int c = code5(v[off + i]);
            ok &= (c != 0);
            k |= (uint64_t)c << (3 * i);
        }
        if (ok) return k;
    }
    uint64_t h = 1469598103934665603ULL;
    for (int i = 0; i < n; ++i) { h ^= v[off + i]; h *= 1099511628211ULL; }
    h ^= (uint64_t)n; h *= 1099511628211ULL;
    return h | (1ULL << 63);
}
// exemplar of a state-table entry: len<<48 | SEQ offset<<32 | alignment index
__device__ __forceinline__ int ex_len(uint64_t e) { return (int)(e >> 48); }
__device__ __forceinline__ int ex_off(uint64_t e) { return (int)((e >> 32) & 0xFFFFu); }
__device__ __forceinline__ int64_t ex_aln(uint64_t e) { return (int64_t)(e & 0xFFFFFFFFu); }
__device__ __forceinline__ SeqV seq_view(const CnsDev &D, int64_t g) {
    SeqV v;
    v.p = D.seq + D.seq_off[g];
    v.n = D.lseq[g];
    v.rc = (D.aflags[g] & 8) != 0;
    v.nt4 = D.seq_nt4 != 0;
    return v;
}
__device__ __forceinline__ uint8_t ref_base(const CnsDev &D, int64_t i) {
    const uint8_t c = D.ref_seq[i];
    return D.ref_nt4 ? nt4_ascii(c > 4 ? 4 : c) : c;
}
__device__ __forceinline__ uint32_t key_slot_hash(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return (uint32_t)k;
}

// ---------------------------------------------------------------------------
// block-wide exclusive scan of a 64-bit value (256 threads = 4 waves of 64)
__device__ __forceinline__ long long block_scan_excl(long long v, long long *scr, long long *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        long long y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) scr[w] = x;
    __syncthreads();
    long long base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < CNS_THREADS / 64; ++i) {
        long long s = scr[i];
        if (i < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}
__device__ __forceinline__ int block_or(int v, int *scr) {
    v = __any(v) ? 1 : 0;
    if ((threadIdx.x & 63) == 0) scr[threadIdx.x >> 6] = v;
    __syncthreads();
    int r = 0;
    for (int i = 0; i < CNS_THREADS / 64; ++i) r |= scr[i];
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------------------
// State walker (Seq.pm:390-461): visits every state of a prepared alignment
// in order.  kind 0 = sequence state (qoff,len; len>1 is an insertion state),
// kind 1 = '-' (deletion).  A state is final once the next op is not an I.
template <bool MULTI_ONLY, class F>
__device__ __forceinline__ void walk_states(const uint32_t *cg, int cb, int ce, int rpos0,
                                            int cmin, int cmax, F &&f) {
    int col = rpos0, sidx = 0, qpos = 0;
    int p_col = 0, p_sidx = 0, p_kind = -1, p_qoff = 0, p_len = 0;
    for (int k = cb; k < ce; ++k) {
        const uint32_t c = cg[k];
        const int n = (int)(c >> 4), op = (int)(c & 15u);
        if (op == 1) {  // I
            if (k > cb) {
                if (p_kind == 1) { p_kind = 0; p_qoff = qpos; p_len = n; }
                else p_len += n;
            } else {
                p_col = col; p_sidx = sidx; p_kind = 0; p_qoff = qpos; p_len = n;
                ++col; ++sidx;
            }
            qpos += n;
            continue;
        }
        if (n == 0) continue;   // split() of an empty run pushes nothing
        if (p_kind >= 0) {
            if ((!MULTI_ONLY || (p_kind == 0 && p_len > 1)) && p_col >= cmin && p_col < cmax)
                f(p_col, p_sidx, p_kind, p_qoff, p_len);
            p_kind = -1;
        }
        if (col > cmax) break;   // everything further right is outside [cmin,cmax)
        const int kind = (op == 0) ? 0 : 1;
        if (!MULTI_ONLY) {
            const int lo = col > cmin ? col : cmin;
            const int hi = (col + n - 1) < cmax ? (col + n - 1) : cmax;
            for (int x = lo; x < hi; ++x) f(x, sidx + (x - col), kind, qpos + (x - col), 1);
        }
        p_col = col + n - 1; p_sidx = sidx + n - 1; p_kind = kind;
        p_qoff = kind == 0 ? qpos + n - 1 : 0; p_len = 1;
        col += n; sidx += n;
        if (kind == 0) qpos += n;
    }
    if (p_kind >= 0 && (!MULTI_ONLY || (p_kind == 0 && p_len > 1)) && p_col >= cmin && p_col < cmax)
        f(p_col, p_sidx, p_kind, p_qoff, p_len);
}

// ---------------------------------------------------------------------------
// per-alignment prep (Alignment.pm:417-546, Seq.pm:270-432 up to the states)
__device__ void prep_alignment(const CnsDev &D, const CnsParamsDev &P, int64_t g, long L, long nbins) {
    const uint8_t fl = D.aflags[g];
    const int n = D.ncig[g];
    const uint32_t *cg = D.cig + D.cig_off[g];
    const int ls = D.lseq[g];
    const int pos = D.pos[g];
    uint32_t st = 0;
    if (fl & 4) st |= ST_NOSEQ;
    long qlen = 0, md = 0;
    for (int k = 0; k < n; ++k) {
        const int op = cg[k] & 15, m = (int)(cg[k] >> 4);
        if (op > 8) st |= ST_SAM;
        if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) qlen += m;
        if (op == 0 || op == 2) md += m;
        if (op == 1 && m == 0) st |= ST_SAM;
    }
    if (!(fl & 4) && n > 0 && qlen != ls) st |= ST_SAM;
    const bool clipped = n > 0 && (((cg[0] & 15) == 4) || ((cg[n - 1] & 15) == 4));
    const long len = ((fl & 4) || clipped) ? md : ls;
    D.a_len[g] = (int32_t)len;
    double nc = 0.0;
    int bin = -1;
    if (fl & 1) {
        st |= ST_SCORED;
        double sc = D.score[g];
        if (P.invert_scores) sc = __dmul_rn(sc, -1.0);
        if (len == 0) st |= ST_DIV0;
        else {
            const double ns = __ddiv_rn(sc, (double)len);
            nc = __dmul_rn(ns, __ddiv_rn((double)len, (double)(40 + len)));
        }
        const double c = __ddiv_rn(__dadd_rn((double)pos, __ddiv_rn((double)len, 2.0)), P.bin_size);
        const long b = (long)c;
        if (b < 0 || b >= nbins) st |= ST_BINRANGE;
        else bin = (int)b;
    }
    D.a_nc[g] = nc;
    D.a_bin[g] = bin;

    // ---- State_matrix per-alignment preparation (Seq.pm:275-385)
    int cb = 0, ce = n, sb = 0, se = ls;
    int rpos = pos - 1;
    const int orig = ls;
    if (!(orig > P.min_aln_length) || (st & (ST_SAM | ST_NOSEQ))) {
        st |= ST_SMSKIP;
    } else if (n == 0) {
        st |= ST_SMERR;   // "Empty Cigar" (Seq.pm:313)
    } else {
        if ((cg[cb] & 15) == 4) { const int k = (int)(cg[cb] >> 4); sb = k < orig ? k : orig; ++cb; }
        if (ce > cb && (cg[ce - 1] & 15) == 4) { const int k = (int)(cg[ce - 1] >> 4); se = (se - sb) > k ? se - k : sb; --ce; }
        if (ce > cb && (cg[cb] & 15) == 5) ++cb;
        if (ce > cb && (cg[ce - 1] & 15) == 5) --ce;
        if (ce <= cb) st |= ST_SMERR;
        if (!(st & ST_SMERR) && P.trim) {
            long mc = 0, dc = 0, ic = 0;
            const long taboo = P.indel_taboo_length ? P.indel_taboo_length
                                                    : (long)__dadd_rn(__dmul_rn((double)orig, P.indel_taboo), 0.5);
            for (int i = cb; i < ce; ++i) {
                const int op = cg[i] & 15;
                const long m = (long)(cg[i] >> 4);
                if (op == 0) {
                    if (mc + ic + m > taboo) {
                        if (i > cb) {
                            cb = i;
                            rpos += (int)(mc + dc);
                            const long cut = mc + ic;
                            sb = (se - sb) > cut ? sb + (int)cut : se;
                        }
                        break;
                    }
                    mc += m;
                } else if (op == 2) dc += m;
                else if (op == 1) ic += m;
                else { st |= ST_SMERR; break; }
            }
            if (!(st & ST_SMERR)) {
                const int kl = se - sb;
                if (kl < 50 || __ddiv_rn((double)kl, (double)orig) < 0.7) st |= ST_SMSKIP;
            }
            if (!(st & (ST_SMERR | ST_SMSKIP))) {
                long tail = 0;
                for (int i = ce - 1; i != cb; --i) {
                    const int op = cg[i] & 15;
                    const long m = (long)(cg[i] >> 4);
                    if (op == 0) {
                        tail += m;
                        if (tail > taboo) {
                            if (i < ce - 1) {
                                const long cut = tail - m;
                                ce = i + 1;
                                se = (long)(se - sb) > cut ? se - (int)cut : sb;
                            }
                            break;
                        }
                    } else if (op == 2) {
                    } else if (op == 1) tail += m;
                    else { st |= ST_SMERR; break; }
                }
                if (!(st & ST_SMERR)) {
                    const int kl = se - sb;
                    if (kl < P.min_aln_length || __ddiv_rn((double)kl, (double)orig) < 0.7) st |= ST_SMSKIP;
                }
            }
        }
        if (!(st & (ST_SMERR | ST_SMSKIP))) {
            // cigar -> states: count states, validate ops (Seq.pm:396-432)
            int ns = 0;
            for (int k = cb; k < ce; ++k) {
                const int op = cg[k] & 15, m = (int)(cg[k] >> 4);
                if (op == 0 || op == 2) ns += m;
                else if (op == 1) {
                    if (k > cb) { if (ns == 0) { st |= ST_SMERR; break; } }
                    else ++ns;
                } else { st |= ST_SMERR; break; }
            }
            if (rpos < 0) st |= ST_BEYOND;
            if ((long)rpos + ns > L) st |= ST_BEYOND;
            if (ns >= 4096) st |= ST_SMCAP;
            D.a_end[g] = rpos + ns;
        }
    }
    D.a_st[g] = st;
    D.a_cb[g] = cb;
    D.a_ce[g] = ce;
    D.a_sb[g] = sb;
    D.a_rpos[g] = rpos;
}

// ---------------------------------------------------------------------------
// LDS carve (bytes).  Everything lives in one dynamic array (G17 alignment).
constexpr int OFF_CTRL = 0;                       // 256 B control block
constexpr int OFF_SCAN = 256;                     // 256 x 8 B scan scratch
constexpr int OFF_A = OFF_SCAN + 2048;            // region A: bin arrays, then state table
constexpr int SZ_A = TCAP * 24;
constexpr int OFF_B = OFF_A + SZ_A;               // region B: window / chimera buffers
constexpr int B_CNT6 = 0;                                   // u32 [WCOLS*6] (scatter fallback)
constexpr int B_WL = B_CNT6;                                // int4 [2*WLCAP] (expanded path, aliases CNT6)
constexpr int B_WBEG = B_WL + WLCAP * 32;                   // i32 [WBCAP]    (expanded path)
static_assert(WLCAP * 32 + WBCAP * 4 <= WCOLS * 6 * 4, "window staging fits the CNT6 area");
static_assert(WCOLS == 2 * CNS_THREADS, "two pileup columns per thread");
constexpr int B_WKEY = B_CNT6 + WCOLS * 6 * 4;              // u32 [WCAP]
constexpr int B_WCNT = B_WKEY + WCAP * 4;                   // u32 [WCAP]
constexpr int B_COLCNT = B_WCNT + WCAP * 4;                 // i32 [WCOLS]
constexpr int B_COLST = B_COLCNT + WCOLS * 4;               // i32 [WCOLS]
constexpr int B_ELIST = B_COLST + WCOLS * 4;                // u16 [WCAP]
constexpr int B_CDESC = B_ELIST + WCAP * 2;                 // u32 [WCOLS]
constexpr int B_COUT = B_CDESC + WCOLS * 4;                 // u16 [WCOLS] out len
constexpr int B_CPHR = B_COUT + WCOLS * 2;                  // u8  [WCOLS] phred
constexpr int SZ_B = B_CPHR + WCOLS;
constexpr int CNS_LDS_BYTES = OFF_B + SZ_B;
static_assert(CNS_LDS_BYTES <= 81920, "two workgroups per CU");
constexpr int MAX_BINS_LDS = (SZ_A - CNS_THREADS * 4) / 8;

// per-column descriptor: flag bits above the 11-bit state-table slot
constexpr uint32_t DESC_FIXED = 1u << 16;
constexpr uint32_t DESC_INS = 1u << 17;
// expanded pileup codes (per alignment and column)
constexpr uint32_t E_INS = 0x80000000u;   // | state-table slot
constexpr uint32_t E_DEL = 0xFFFFFFFFu;

struct Ctrl {
    int lr;
    int err_code;
    unsigned long long err_first;   // atomicMin (index<<8 | code)
    int run_seq, run_trace;
    int cand_b0, cand_b1;
    int nchim;
    int flag;
    unsigned long long ne;          // expanded entries: total, then running offset
    int nk, maxspan, fast, pad;
};

__device__ __forceinline__ bool in_ign(const int32_t *ig, int nig, int col) {
    for (int r = 0; r < nig; ++r)
        if (col >= ig[2 * r] && col < ig[2 * r] + ig[2 * r + 1]) return true;
    return false;
}

// state table (region A after binning)
struct STab {
    unsigned long long *key;  // TCAP
    unsigned int *ord_cns;    // TCAP (min order of non-ignored occurrences)
    unsigned int *ord_all;    // TCAP (min order of all occurrences)
    unsigned long long *exem; // TCAP  len<<48 | SEQ offset<<32 | alignment index
};
__device__ __forceinline__ int stab_find(const STab &T, uint64_t k) {
    uint32_t h = key_slot_hash(k) & (TCAP - 1);
    for (int p = 0; p < TCAP; ++p) {
        const uint64_t x = T.key[h];
        if (x == k) return (int)h;
        if (x == 0) return -1;
        h = (h + 1) & (TCAP - 1);
    }
    return -1;
}
__device__ __forceinline__ int stab_insert(const STab &T, uint64_t k, uint64_t exem) {
    uint32_t h = key_slot_hash(k) & (TCAP - 1);
    for (int p = 0; p < TCAP; ++p) {
        const unsigned long long x = T.key[h];
        if (x == k) return (int)h;
        if (x == 0) {
            const unsigned long long old = atomicCAS(&T.key[h], 0ULL, (unsigned long long)k);
            if (old == 0ULL) { T.exem[h] = exem; return (int)h; }
            if (old == k) return (int)h;
        }
        h = (h + 1) & (TCAP - 1);
    }
    return -1;
}
// (column-in-window, slot) -> count, window table in region B
__device__ __forceinline__ int wtab_add(uint32_t *wkey, uint32_t *wcnt, uint32_t key) {
    uint32_t h = (key * 2654435761u) >> 22;   // 10 bits -> WCAP 1024
    for (int p = 0; p < WCAP; ++p) {
        const uint32_t x = wkey[h];
        if (x == key) { atomicAdd(&wcnt[h], 1u); return 0; }
        if (x == 0) {
            const uint32_t old = atomicCAS(&wkey[h], 0u, key);
            if (old == 0u || old == key) { atomicAdd(&wcnt[h], 1u); return 0; }
        }
        h = (h + 1) & (WCAP - 1);
    }
    return -1;
}

__device__ __forceinline__ void set_err(Ctrl *C, long idx, int code) {
    atomicMin(&C->err_first, ((unsigned long long)idx << 8) | (unsigned long long)(-code));
}

// chimera-table ordering key for a state-table slot: consensus indices first,
// then states first seen only in the no-ignore recompute (Seq.pm:777, 446)
__device__ __forceinline__ unsigned long long chim_order(const STab &T, int slot) {
    const unsigned int oc = T.ord_cns[slot];
    return oc != 0xFFFFFFFFu ? (unsigned long long)oc : (1ULL << 32) | T.ord_all[slot];
}

// count of (column c, slot) in a chimera side table (0 if absent)
__device__ __forceinline__ uint32_t chim_count(const uint32_t *tk, const uint32_t *tc, uint32_t key) {
    uint32_t h = (key * 2654435761u) >> 24;
    for (int p = 0; p < CHIM_TCAP; ++p) {
        const uint32_t x = tk[h];
        if (x == key) return tc[h];
        if (x == 0u) return 0u;
        h = (h + 1) & (CHIM_TCAP - 1);
    }
    return 0u;
}

// Hx (Seq.pm:188-197) of column c of the left matrix (side 0), the right matrix
// (side 1) or their element-wise sum (side 2, the combined column of
// Seq.pm:857-865).  Fixed states first, then insertion states in state-index
// order (selection over the LDS tables: no per-thread arrays).
__device__ double chim_hx(int side, int c, const uint32_t *f6l, const uint32_t *f6r, const uint32_t *tkl,
                          const uint32_t *tcl, const uint32_t *tkr, const uint32_t *tcr, const STab &T) {
    const double l2 = log(2.0);
    double total = 0.0;
    for (int s = 0; s < 6; ++s) {
        const uint32_t v = (side != 1 ? f6l[c * 6 + s] : 0u) + (side != 0 ? f6r[c * 6 + s] : 0u);
        if (v) total += (double)v;
    }
    // pass 0: total over insertion states; pass 1: entropy terms
    double h = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
            for (int s = 0; s < 6; ++s) {
                const uint32_t v = (side != 1 ? f6l[c * 6 + s] : 0u) + (side != 0 ? f6r[c * 6 + s] : 0u);
                if (!v) continue;
                const double p = (double)v / total;
                h -= p * (log(p) / l2);
            }
        }
        unsigned long long prev = 0;
        bool first = true;
        for (;;) {
            unsigned long long best = ~0ULL;
            int bslot = -1;
            for (int t = 0; t < 2; ++t) {
                if ((t == 0 && side == 1) || (t == 1 && side == 0)) continue;
                const uint32_t *tk = t == 0 ? tkl : tkr;
                for (int e = 0; e < CHIM_TCAP; ++e) {
                    const uint32_t k = tk[e];
                    if (!k || (int)(k >> 11) - 1 != c) continue;
                    const int slot = (int)(k & 2047u);
                    const unsigned long long o = chim_order(T, slot);
                    if ((first || o > prev) && o < best) { best = o; bslot = slot; }
                }
            }
            if (bslot < 0) break;
            const uint32_t key = ((uint32_t)(c + 1) << 11) | (uint32_t)bslot;
            const uint32_t v = (side != 1 ? chim_count(tkl, tcl, key) : 0u) + (side != 0 ? chim_count(tkr, tcr, key) : 0u);
            if (v) {
                if (pass == 0) total += (double)v;
                else {
                    const double p = (double)v / total;
                    h -= p * (log(p) / l2);
                }
            }
            prev = best;
            first = false;
        }
    }
    return h;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(CNS_THREADS, 2) cns_lr_kernel(CnsDev D, CnsParamsDev P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Ctrl *C = reinterpret_cast<Ctrl *>(smem + OFF_CTRL);
    long long *scan = reinterpret_cast<long long *>(smem + OFF_SCAN);
    uint8_t *A = smem + OFF_A;
    uint8_t *B = smem + OFF_B;
    const int tid = threadIdx.x;
    // phase clock (thread 0, 100 MHz wall clock): ticks per phase summed over workgroups
    unsigned long long pt[CNS_NPHASE] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tlast = wall_clock64();
#define CNS_TICK(ph)                                                      \
    do {                                                                  \
        if (D.prof && tid == 0) {                                         \
            const unsigned long long t_ = wall_clock64();                 \
            pt[ph] += t_ - tlast;                                         \
            tlast = t_;                                                   \
        }                                                                 \
    } while (0)

    for (;;) {
        if (tid == 0) {
            C->lr = atomicAdd(D.work, 1);
            C->err_first = ~0ULL;
            C->run_seq = 0;
            C->run_trace = 0;
            C->nchim = 0;
            C->flag = 0;
        }
        __syncthreads();
        const int lr = C->lr;
        CNS_TICK(7);
        if (lr >= D.n_lr) break;
        const int64_t a0 = D.aln_off[lr];
        const int na = (int)(D.aln_off[lr + 1] - a0);
        const long L = (long)(D.lr_off[lr + 1] - D.lr_off[lr]);
        const long nbins = (long)((double)L / P.bin_size) + 1;
        const int64_t r0 = D.lr_off[lr];
        const int nig = D.ign_off ? (int)(D.ign_off[lr + 1] - D.ign_off[lr]) : 0;
        const int32_t *ig = D.ign_off ? D.ign + 2 * D.ign_off[lr] : nullptr;
        const int64_t o0 = D.out_off[lr];

        // ---- 1. prep (and kept := 0)
        for (int i = tid; i < na; i += CNS_THREADS) {
            prep_alignment(D, P, a0 + i, L, nbins);
            D.kept[a0 + i] = 0;
            const uint32_t st = D.a_st[a0 + i];
            // first offending alignment in arrival order decides the error (bam2cns:345-353)
            if (st & ST_NOSEQ) set_err(C, i, PR_ERR_CODE_NOSEQ);
            else if (st & ST_SAM) set_err(C, i, PR_ERR_CODE_SAM);
            else if ((st & ST_SCORED) && (st & ST_DIV0)) set_err(C, i, PR_ERR_CODE_DIV0);
            else if ((st & ST_SCORED) && (st & ST_BINRANGE)) set_err(C, i, PR_ERR_CODE_BIN);
        }
        if (nbins > MAX_BINS_LDS && tid == 0) set_err(C, 0, PR_ERR_CODE_CAP);
        __syncthreads();
        CNS_TICK(0);
        if (C->err_first != ~0ULL) {
            if (tid == 0) {
                D.status[lr] = -(int)(C->err_first & 0xFF);
                D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0;
            }
            __syncthreads();
            continue;
        }

        // ---- 2. binning (Seq.pm:582-614)
        {
            int32_t *cnt = reinterpret_cast<int32_t *>(A);
            int32_t *start = cnt + nbins;
            int32_t *chunk = start + nbins;
            for (long b = tid; b < nbins; b += CNS_THREADS) cnt[b] = 0;
            __syncthreads();
            for (int i = tid; i < na; i += CNS_THREADS)
                if (D.a_st[a0 + i] & ST_SCORED) atomicAdd(&cnt[D.a_bin[a0 + i]], 1);
            __syncthreads();
            // exclusive scan of cnt -> start (each thread scans a contiguous chunk)
            const long per = (nbins + CNS_THREADS - 1) / CNS_THREADS;
            const long b0 = tid * per, b1 = (b0 + per) < nbins ? (b0 + per) : nbins;
            long long s = 0;
            for (long b = b0; b < b1; ++b) s += cnt[b];
            long long tot;
            long long base = block_scan_excl(s, scan, &tot);
            for (long b = b0; b < b1; ++b) { start[b] = (int32_t)base; base += cnt[b]; cnt[b] = 0; }
            __syncthreads();
            // stable scatter by bin, chunks of 256 in arrival order
            for (int c0 = 0; c0 < na; c0 += CNS_THREADS) {
                const int i = c0 + tid;
                const int b = (i < na && (D.a_st[a0 + i] & ST_SCORED)) ? D.a_bin[a0 + i] : -1;
                chunk[tid] = b;
                __syncthreads();
                int rank = 0;
                bool last = true;
                if (b >= 0) {
                    for (int j = 0; j < CNS_THREADS; ++j) {
                        const int bj = chunk[j];
                        if (bj == b) { if (j < tid) ++rank; else if (j > tid) last = false; }
                    }
                    D.sorted[a0 + start[b] + cnt[b] + rank] = i;
                }
                __syncthreads();
                if (b >= 0 && last) cnt[b] += rank + 1;
                __syncthreads();
            }
            // one thread per bin: sequential add_aln_by_score within the bin
            const double maxb = P.bin_max_bases;
            for (long b = tid; b < nbins; b += CNS_THREADS) {
                const int sidx = start[b], nb = cnt[b];
                double *ls = D.lst_score + a0 + sidx;
                int32_t *la = D.lst_aln + a0 + sidx;
                int ln = 0;
                long bases = 0;
                for (int k = 0; k < nb; ++k) {
                    const int i = D.sorted[a0 + sidx + k];
                    const double nc = D.a_nc[a0 + i];
                    if ((double)bases > maxb) {
                        if (nc <= ls[ln - 1]) continue;
                        bases -= D.a_len[a0 + la[ln - 1]];
                        --ln;
                    }
                    bases += D.a_len[a0 + i];
                    int j = ln - 1;
                    while (j >= 0 && nc > ls[j]) { ls[j + 1] = ls[j]; la[j + 1] = la[j]; --j; }
                    ls[j + 1] = nc; la[j + 1] = i;
                    ++ln;
                }
                for (int k = 0; k < ln; ++k) D.kept[a0 + la[k]] = 1;
                D.bin_bases[D.bin_off[lr] + b] = bases;
            }
            __syncthreads();
        }
        CNS_TICK(1);
        // kept alignments that State_matrix would die on (Seq.pm:313/348/430)
        for (int i = tid; i < na; i += CNS_THREADS) {
            if (!D.kept[a0 + i]) continue;
            const uint32_t st = D.a_st[a0 + i];
            if (st & ST_SMSKIP) continue;
            if (st & ST_SMERR) set_err(C, i, PR_ERR_CODE_CIGAR);
            else if (st & ST_BEYOND) set_err(C, i, PR_ERR_CODE_BEYOND);
            else if (st & ST_SMCAP) set_err(C, i, PR_ERR_CODE_CAP);
            else if (i >= (1 << 20)) set_err(C, i, PR_ERR_CODE_CAP);
        }
        __syncthreads();
        if (C->err_first != ~0ULL) {
            if (tid == 0) {
                D.status[lr] = -(int)(C->err_first & 0xFF);
                D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0;
            }
            __syncthreads();
            continue;
        }

        // ---- 3. insertion-state table: first-seen order (Seq.pm:446-448), and (expanded
        //         path) every kept alignment's states written once as one code per column
        STab T;
        T.key = reinterpret_cast<unsigned long long *>(A);
        T.exem = T.key + TCAP;
        T.ord_cns = reinterpret_cast<unsigned int *>(T.exem + TCAP);
        T.ord_all = T.ord_cns + TCAP;
        for (int h = tid; h < TCAP; h += CNS_THREADS) {
            T.key[h] = 0ULL; T.exem[h] = 0ULL; T.ord_cns[h] = 0xFFFFFFFFu; T.ord_all[h] = 0xFFFFFFFFu;
        }
        int4 *WL = reinterpret_cast<int4 *>(B + B_WL);
        int32_t *wbeg = reinterpret_cast<int32_t *>(B + B_WBEG);
        int32_t *wcur = reinterpret_cast<int32_t *>(B + B_COLCNT);   // colcnt+colst: WBCAP ints
        const int nwin = (int)((L + WCOLS - 1) / WCOLS);
        uint32_t *E = D.e_pool ? D.e_pool + (int64_t)blockIdx.x * D.e_cap : nullptr;
        int4 *K = D.k_pool ? D.k_pool + (int64_t)blockIdx.x * D.k_cap * 2 : nullptr;
        if (tid == 0) { C->ne = 0ULL; C->nk = 0; C->maxspan = 0; }
        for (int x = tid; x < WBCAP; x += CNS_THREADS) wcur[x] = 0;
        __syncthreads();
        for (int i = tid; i < na; i += CNS_THREADS) {
            const int64_t g = a0 + i;
            if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
            const int rp = D.a_rpos[g], span = D.a_end[g] - rp;
            atomicAdd(&C->ne, (unsigned long long)span);
            atomicAdd(&C->nk, 1);
            atomicMax(&C->maxspan, span);
            const int win = rp / WCOLS;
            if (win < WBCAP) atomicAdd(&wcur[win], 1);
        }
        __syncthreads();
        const bool fast = E && K && nwin + 1 <= WBCAP && C->nk <= D.k_cap && C->ne <= (unsigned long long)D.e_cap;
        if (fast) {
            // start-window buckets: wbeg = exclusive scan of counts (4 windows per thread)
            long long sc = 0;
            for (int k = 0; k < 4; ++k) { const int w = tid * 4 + k; if (w < nwin) sc += wcur[w]; }
            long long tot;
            long long base = block_scan_excl(sc, scan, &tot);
            for (int k = 0; k < 4; ++k) {
                const int w = tid * 4 + k;
                if (w < nwin) { wbeg[w] = (int32_t)base; base += wcur[w]; wcur[w] = 0; }
            }
            if (tid == 0) { wbeg[nwin] = (int32_t)tot; C->ne = 0ULL; }
            __syncthreads();
            for (int i = tid; i < na; i += CNS_THREADS) {
                const int64_t g = a0 + i;
                if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
                const int rp = D.a_rpos[g], en = D.a_end[g];
                const int win = rp / WCOLS;
                const int kpos = wbeg[win] + atomicAdd(&wcur[win], 1);
                const int eoff = (int)atomicAdd(&C->ne, (unsigned long long)(en - rp));
                const SeqV sv = seq_view(D, g);
                const int64_t so = D.seq_off[g];
                K[2 * kpos] = make_int4(rp, en, eoff, sv.n | (sv.rc ? (int)0x80000000 : 0));
                K[2 * kpos + 1] = make_int4((int)(so & 0xFFFFFFFF), (int)(so >> 32), 0, 0);
                uint32_t *Ea = E + eoff;
                const int sb = D.a_sb[g];
                const uint32_t *cg = D.cig + D.cig_off[g];
                // codes: SEQ position of a single-base state (the base is read later, in the
                // coalesced pileup), E_DEL for '-', E_INS|slot for an insertion state
                walk_states<false>(cg, D.a_cb[g], D.a_ce[g], rp, 0, 0x7fffffff,
                                   [&](int col, int sidx, int kind, int qoff, int qlen) {
                                       uint32_t code;
                                       if (kind == 1) code = E_DEL;
                                       else if (qlen == 1) code = (uint32_t)(sb + qoff);
                                       else {
                                           const uint64_t k = state_key(sv, sb + qoff, qlen);
                                           if (qlen > 0xFFFF || sb + qoff > 0xFFFF || g > 0xFFFFFFFFLL) { C->flag = 1; return; }
                                           const int h = stab_insert(T, k, ((uint64_t)qlen << 48) |
                                                                               ((uint64_t)(sb + qoff) << 32) | (uint64_t)g);
                                           if (h < 0) { C->flag = 1; return; }
                                           const unsigned int ord = ((unsigned int)i << 12) | (unsigned int)sidx;
                                           atomicMin(&T.ord_all[h], ord);
                                           if (!(nig && in_ign(ig, nig, col))) atomicMin(&T.ord_cns[h], ord);
                                           code = E_INS | (uint32_t)h;
                                       }
                                       Ea[sidx] = code;
                                   });
            }
        } else {
            for (int i = tid; i < na; i += CNS_THREADS) {
                const int64_t g = a0 + i;
                if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
                const SeqV sv = seq_view(D, g);
                const int sb = D.a_sb[g];
                const uint32_t *cg = D.cig + D.cig_off[g];
                walk_states<true>(cg, D.a_cb[g], D.a_ce[g], D.a_rpos[g], 0, 0x7fffffff,
                                  [&](int col, int sidx, int kind, int qoff, int qlen) {
                                      const uint64_t k = state_key(sv, sb + qoff, qlen);
                                      if (qlen > 0xFFFF || sb + qoff > 0xFFFF || g > 0xFFFFFFFFLL) { C->flag = 1; return; }
                                      const int h = stab_insert(T, k, ((uint64_t)qlen << 48) |
                                                                          ((uint64_t)(sb + qoff) << 32) | (uint64_t)g);
                                      if (h < 0) { C->flag = 1; return; }
                                      const unsigned int ord = ((unsigned int)i << 12) | (unsigned int)sidx;
                                      atomicMin(&T.ord_all[h], ord);
                                      if (!(nig && in_ign(ig, nig, col))) atomicMin(&T.ord_cns[h], ord);
                                  });
            }
        }
        __syncthreads();
        if (C->flag) {
            if (tid == 0) {
                D.status[lr] = PR_ERR_CODE_CAP;
                D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0;
            }
            __syncthreads();
            continue;
        }
        const int wback = (C->maxspan + WCOLS - 1) / WCOLS;   // windows an alignment can reach back

        CNS_TICK(2);
        // ---- 4. windowed pileup + argmax (Seq.pm:438-461, 1568-1654)
        uint32_t *cnt6 = reinterpret_cast<uint32_t *>(B + B_CNT6);
        uint32_t *wkey = reinterpret_cast<uint32_t *>(B + B_WKEY);
        uint32_t *wcnt = reinterpret_cast<uint32_t *>(B + B_WCNT);
        int32_t *colcnt = reinterpret_cast<int32_t *>(B + B_COLCNT);
        int32_t *colst = reinterpret_cast<int32_t *>(B + B_COLST);
        uint16_t *elist = reinterpret_cast<uint16_t *>(B + B_ELIST);
        uint32_t *cdesc = reinterpret_cast<uint32_t *>(B + B_CDESC);
        uint16_t *cout_ = reinterpret_cast<uint16_t *>(B + B_COUT);
        uint8_t *cphr = B + B_CPHR;
        const bool use_rq = P.use_ref_qual && D.ref_seq && D.ref_qual;
        for (long w0 = 0; w0 < L; w0 += WCOLS) {
            const int wn = (L - w0) < WCOLS ? (int)(L - w0) : WCOLS;
            uint32_t cnt0[6], cnt1[6];
#pragma unroll
            for (int s = 0; s < 6; ++s) { cnt0[s] = 0u; cnt1[s] = 0u; }
            if (!fast)
                for (int x = tid; x < WCOLS * 6; x += CNS_THREADS) cnt6[x] = 0u;
            for (int x = tid; x < WCAP; x += CNS_THREADS) { wkey[x] = 0u; wcnt[x] = 0u; }
            __syncthreads();
            if (fast) {
                // column-parallel: each thread owns columns tid and tid+256 and reads the
                // codes of every candidate alignment (consecutive columns -> coalesced)
                const int wi = (int)(w0 / WCOLS);
                const int kb = wbeg[wi - wback > 0 ? wi - wback : 0], ke = wbeg[wi + 1];
                for (int c0 = kb; c0 < ke; c0 += WLCAP) {
                    const int n = (ke - c0) < WLCAP ? (ke - c0) : WLCAP;
                    for (int x = tid; x < 2 * n; x += CNS_THREADS) WL[x] = K[2 * c0 + x];
                    __syncthreads();
                    auto accumulate = [&](const int c, uint32_t (&f6)[6]) {
                        const int col = (int)w0 + c;
                        if (c < wn && !(nig && in_ign(ig, nig, col))) {
                            unsigned long long acc = 0ULL;   // six 10-bit counters (n <= WLCAP)
#pragma unroll 4
                            for (int j = 0; j < n; ++j) {
                                const int4 e = WL[2 * j];
                                if (col >= e.x && col < e.y) {
                                    const uint32_t v = E[e.z + col - e.x];
                                    if (v < E_INS) {
                                        const int4 e2 = WL[2 * j + 1];
                                        SeqV sv;
                                        sv.p = D.seq + (((int64_t)e2.y << 32) | (uint32_t)e2.x);
                                        sv.n = e.w & 0x7FFFFFFF;
                                        sv.rc = e.w < 0;
                                        sv.nt4 = D.seq_nt4 != 0;
                                        acc += 1ULL << (10u * (uint32_t)fixed_idx(sv[(int)v]));
                                    } else if (v == E_DEL) {
                                        acc += 1ULL << 40;
                                    } else if (wtab_add(wkey, wcnt, ((uint32_t)(c + 1) << 11) | (v & 2047u)) < 0) {
                                        C->flag = 1;
                                    }
                                }
                            }
#pragma unroll
                            for (int s = 0; s < 6; ++s) f6[s] += (uint32_t)(acc >> (10 * s)) & 1023u;
                        }
                    };
                    accumulate(tid, cnt0);
                    accumulate(tid + CNS_THREADS, cnt1);
                    __syncthreads();
                }
            } else {
                for (int i = tid; i < na; i += CNS_THREADS) {
                    const int64_t g = a0 + i;
                    if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
                    const int rp = D.a_rpos[g];
                    if (rp >= w0 + wn || D.a_end[g] <= w0) continue;
                    const SeqV sv = seq_view(D, g);
                    const int sb = D.a_sb[g];
                    const uint32_t *cg = D.cig + D.cig_off[g];
                    walk_states<false>(cg, D.a_cb[g], D.a_ce[g], rp, (int)w0, (int)(w0 + wn),
                                       [&](int col, int sidx, int kind, int qoff, int qlen) {
                                           if (nig && in_ign(ig, nig, col)) return;
                                           const int c = col - (int)w0;
                                           if (kind == 1) { atomicAdd(&cnt6[c * 6 + 4], 1u); return; }
                                           if (qlen == 1) { atomicAdd(&cnt6[c * 6 + fixed_idx(sv[sb + qoff])], 1u); return; }
                                           const int h = stab_find(T, state_key(sv, sb + qoff, qlen));
                                           if (h < 0 || wtab_add(wkey, wcnt, ((uint32_t)(c + 1) << 11) | (uint32_t)h) < 0)
                                               C->flag = 1;
                                       });
                }
                __syncthreads();
#pragma unroll
                for (int s = 0; s < 6; ++s) {
                    cnt0[s] = cnt6[tid * 6 + s];
                    cnt1[s] = cnt6[(tid + CNS_THREADS) * 6 + s];
                }
            }
            for (int x = tid; x < WCOLS; x += CNS_THREADS) colcnt[x] = 0;
            __syncthreads();
            CNS_TICK(3);
            // per-column lists of insertion entries (counting sort)
            for (int e = tid; e < WCAP; e += CNS_THREADS)
                if (wkey[e]) atomicAdd(&colcnt[(wkey[e] >> 11) - 1], 1);
            __syncthreads();
            {
                const int per = WCOLS / CNS_THREADS;   // 2
                long long s = 0;
                for (int k = 0; k < per; ++k) s += colcnt[tid * per + k];
                long long tot;
                long long base = block_scan_excl(s, scan, &tot);
                for (int k = 0; k < per; ++k) { colst[tid * per + k] = (int32_t)base; base += colcnt[tid * per + k]; colcnt[tid * per + k] = 0; }
            }
            __syncthreads();
            for (int e = tid; e < WCAP; e += CNS_THREADS)
                if (wkey[e]) {
                    const int c = (int)(wkey[e] >> 11) - 1;
                    elist[colst[c] + atomicAdd(&colcnt[c], 1)] = (uint16_t)e;
                }
            __syncthreads();
            // argmax per column (the thread's two columns; counts stay in registers)
            auto argmax_col = [&](const int c, const uint32_t (&f6)[6]) {
                uint16_t olen = 0;
                uint32_t desc = 0;
                uint8_t ph = 0;
                if (c < wn) {
                    const long col = w0 + c;
                    double val[6];
                    bool def[6];
                    bool any = false;
                    int rs = -1;
                    double vref = 0.0;
                    if (use_rq) {
                        const double fr = phred2freq((int)D.ref_qual[r0 + col] - P.ref_phred_offset);
                        if (fr != 0.0) {
                            rs = fixed_idx(ref_base(D, r0 + col));
                            vref = fr;   // ref freq is added first, then +1 per alignment
                            uint32_t n = 0;
#pragma unroll
                            for (int s = 0; s < 6; ++s) n = s == rs ? f6[s] : n;
                            for (uint32_t kk = 0; kk < n; ++kk) vref = __dadd_rn(vref, 1.0);
                        }
                    }
#pragma unroll
                    for (int s = 0; s < 6; ++s) {
                        const uint32_t n = f6[s];
                        val[s] = s == rs ? vref : (double)n;
                        def[s] = (n != 0u) || (s == rs);
                        any |= def[s];
                    }
                    const int ne = colcnt[c];
                    any |= ne > 0;
                    double maxf = 0.0;
                    int idx = -1;
                    unsigned int best_ord = 0xFFFFFFFFu;
                    int best_slot = -1;
#pragma unroll
                    for (int s = 0; s < 6; ++s)
                        if (def[s] && val[s] > maxf) { maxf = val[s]; idx = s; }
                    for (int x = 0; x < ne; ++x) {
                        const int e = elist[colst[c] + x];
                        const int slot = (int)(wkey[e] & 2047u);
                        const int slen = ex_len(T.exem[slot]);
                        if (P.max_ins_length && slen > P.max_ins_length) continue;
                        const double v = (double)wcnt[e];
                        const unsigned int o = T.ord_cns[slot];
                        if (v > maxf || (v == maxf && idx >= 6 && o < best_ord)) {
                            maxf = v; idx = 6; best_ord = o; best_slot = slot;
                        }
                    }
                    if (!any || !(maxf != 0.0)) {
                        olen = 1; desc = DESC_FIXED | (D.ref_seq ? ref_base(D, r0 + col) : (uint8_t)'n'); ph = 0;
                    } else if (idx == 4) {
                        olen = 0; desc = 0; ph = 0;
                    } else if (idx < 6) {
                        olen = 1; desc = DESC_FIXED | (uint8_t)(0x4E2D43475441ULL >> (8 * idx)); ph = (uint8_t)freq2phred(maxf);
                    } else {
                        olen = (uint16_t)ex_len(T.exem[best_slot]); desc = DESC_INS | (uint32_t)best_slot;
                        ph = (uint8_t)freq2phred(maxf);
                    }
                }
                cout_[c] = olen;
                cdesc[c] = desc;
                cphr[c] = ph;
            };
            argmax_col(tid, cnt0);
            argmax_col(tid + CNS_THREADS, cnt1);
            __syncthreads();
            // block scan of (seq len, trace len) over the window's columns, then write
            {
                const int per = WCOLS / CNS_THREADS;
                long long s = 0;
                for (int k = 0; k < per; ++k) {
                    const int c = tid * per + k;
                    if (c < wn) {
                        const long long ol = cout_[c];
                        s += ol | ((long long)(ol ? ol : 1) << 32);
                    }
                }
                long long tot;
                long long base = block_scan_excl(s, scan, &tot);
                int so = C->run_seq + (int)(base & 0xffffffffLL);
                int to = C->run_trace + (int)(base >> 32);
                const uint8_t qch_off = (uint8_t)P.phred_offset;
                // output capacity of this read (always sufficient for pr_cns_run batches,
                // a guard for pipeline batches whose capacity is estimated)
                const long long cap = D.out_off[lr + 1] - o0;
                const bool fits = (long long)C->run_trace + (tot >> 32) <= cap;
                if (!fits && tid == 0) C->flag = 1;
                for (int k = 0; k < per && fits; ++k) {
                    const int c = tid * per + k;
                    if (c >= wn) break;
                    const int ol = cout_[c];
                    const uint32_t d = cdesc[c];
                    const uint8_t qc = (uint8_t)(cphr[c] + qch_off);
                    if (ol == 0) {
                        D.o_trace[o0 + to] = 'I';
                        to += 1;
                    } else if (d & DESC_FIXED) {
                        D.o_seq[o0 + so] = (uint8_t)(d & 0xFFu);
                        D.o_qual[o0 + so] = qc;
                        D.o_trace[o0 + to] = 'M';
                        so += 1; to += 1;
                    } else {
                        const int slot = (int)(d & 2047u);
                        const uint64_t ex = T.exem[slot];
                        const SeqV src = seq_view(D, ex_aln(ex));
                        const int eo = ex_off(ex);
                        for (int q = 0; q < ol; ++q) {
                            D.o_seq[o0 + so + q] = src[eo + q];
                            D.o_qual[o0 + so + q] = qc;
                            D.o_trace[o0 + to + q] = q ? 'D' : 'M';
                        }
                        so += ol; to += ol;
                    }
                }
                __syncthreads();
                if (tid == 0) {
                    C->run_seq += (int)(tot & 0xffffffffLL);
                    C->run_trace += (int)(tot >> 32);
                }
                __syncthreads();
            }
            CNS_TICK(4);
        }
        if (C->flag) {
            if (tid == 0) {
                D.status[lr] = PR_ERR_CODE_CAP;
                D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0;
            }
            __syncthreads();
            continue;
        }
        const int tlen = C->run_trace;

        // ---- 5. Trace2cigar (Seq.pm:206-225): run starts -> ops
        int nruns = 0;
        {
            int32_t *rstart = reinterpret_cast<int32_t *>(D.o_cig + o0);   // reuse cigar buffer
            for (int c0 = 0; c0 < tlen; c0 += CNS_THREADS) {
                const int i = c0 + tid;
                int f = 0;
                if (i < tlen) f = (i == 0 || D.o_trace[o0 + i] != D.o_trace[o0 + i - 1]) ? 1 : 0;
                long long tot;
                const long long r = block_scan_excl(f, scan, &tot);
                if (f) rstart[nruns + (int)r] = i;
                nruns += (int)tot;
            }
            __syncthreads();
            for (int r0_ = 0; r0_ < nruns; r0_ += CNS_THREADS) {
                const int r = r0_ + tid;
                int s0 = 0, s1 = 0;
                uint8_t opc = 0;
                if (r < nruns) {
                    s0 = rstart[r];
                    s1 = (r + 1 < nruns) ? rstart[r + 1] : tlen;
                    opc = D.o_trace[o0 + s0];
                }
                __syncthreads();
                if (r < nruns) {
                    const uint32_t op = opc == 'M' ? 0u : (opc == 'I' ? 1u : 2u);
                    D.o_cig[o0 + r] = ((uint32_t)(s1 - s0) << 4) | op;
                }
                __syncthreads();
            }
        }

        CNS_TICK(5);
        // ---- 6. chimera (Seq.pm:774-889) + detect_chimera (bam2cns:461-491)
        int nch = 0;
        if (P.detect_chimera && nbins > 20) {
            const int64_t bb = D.bin_off[lr];
            const double thr = P.bin_max_bases / 5.0 + 1.0;
            uint32_t *f6a = reinterpret_cast<uint32_t *>(B);              // all: nonempty flags
            uint32_t *f6l = f6a + CHIM_MAXCOLS;                           // left fixed counts
            uint32_t *f6r = f6l + CHIM_MAXCOLS * 6;                       // right fixed counts
            uint32_t *tkl = f6r + CHIM_MAXCOLS * 6;                       // left table keys
            uint32_t *tcl = tkl + CHIM_TCAP;
            uint32_t *tkr = tcl + CHIM_TCAP;
            uint32_t *tcr = tkr + CHIM_TCAP;
            int *ired = reinterpret_cast<int *>(tcr + CHIM_TCAP);          // reductions
            const int64_t c_off = D.chim_off[lr];
            long scan_i = 5;
            long cntlow = 0;
            for (;;) {
                // thread 0 finds the next candidate window (Seq.pm:790-799)
                if (tid == 0) {
                    C->cand_b0 = -1;
                    for (; scan_i < nbins - 5; ++scan_i) {
                        if ((double)D.bin_bases[bb + scan_i] <= thr) ++cntlow;
                        else if (cntlow) {
                            const long c = cntlow;
                            cntlow = 0;
                            if (c >= 1 && c < 5) {
                                C->cand_b0 = (int)(scan_i - c);
                                C->cand_b1 = (int)(scan_i - 1);
                                ++scan_i;
                                break;
                            }
                        }
                    }
                }
                __syncthreads();
                const int cb0 = C->cand_b0, cb1 = C->cand_b1;
                __syncthreads();
                if (cb0 < 0) break;
                const int bs = (int)P.bin_size;
                const int mf = (cb0 - 1) * bs, mt = (cb1 + 2) * bs - 1;
                const int ncol = mt - mf + 1;
                const int fl = cb0 - 4, tr = cb1 + 5;
                const int dlt = (tr - fl - 1) / 2;
                const int tl = fl + dlt, fr = tr - dlt;
                for (int x = tid; x < CHIM_MAXCOLS * 13; x += CNS_THREADS) f6a[x] = 0u;
                for (int x = tid; x < CHIM_TCAP * 4; x += CNS_THREADS) tkl[x] = 0u;
                __syncthreads();
                for (int i = tid; i < na; i += CNS_THREADS) {
                    const int64_t g = a0 + i;
                    if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
                    const int rp = D.a_rpos[g];
                    if (rp > mt || D.a_end[g] <= mf) continue;
                    const int bin = D.a_bin[g];
                    const bool inl = bin >= fl && bin <= tl, inr = bin >= fr && bin <= tr;
                    const SeqV sv = seq_view(D, g);
                    const int sb = D.a_sb[g];
                    const uint32_t *cg = D.cig + D.cig_off[g];
                    walk_states<false>(cg, D.a_cb[g], D.a_ce[g], rp, mf, mt + 1,
                                       [&](int col, int sidx, int kind, int qoff, int qlen) {
                                           const int c = col - mf;
                                           f6a[c] = 1u;
                                           int fi = -1, slot = -1;
                                           if (kind == 1) fi = 4;
                                           else if (qlen == 1) fi = fixed_idx(sv[sb + qoff]);
                                           else slot = stab_find(T, state_key(sv, sb + qoff, qlen));
                                           for (int side = 0; side < 2; ++side) {
                                               if (side == 0 ? !inl : !inr) continue;
                                               uint32_t *f6 = side == 0 ? f6l : f6r;
                                               uint32_t *tk = side == 0 ? tkl : tkr;
                                               uint32_t *tc = side == 0 ? tcl : tcr;
                                               if (fi >= 0) { atomicAdd(&f6[c * 6 + fi], 1u); continue; }
                                               if (slot < 0) { C->flag = 1; continue; }
                                               const uint32_t key = ((uint32_t)(c + 1) << 11) | (uint32_t)slot;
                                               uint32_t h = (key * 2654435761u) >> 24;
                                               int p = 0;
                                               for (; p < CHIM_TCAP; ++p) {
                                                   const uint32_t x = tk[h];
                                                   if (x == key) break;
                                                   if (x == 0u) {
                                                       const uint32_t o = atomicCAS(&tk[h], 0u, key);
                                                       if (o == 0u || o == key) break;
                                                   }
                                                   h = (h + 1) & (CHIM_TCAP - 1);
                                               }
                                               if (p == CHIM_TCAP) C->flag = 1;
                                               else atomicAdd(&tc[h], 1u);
                                           }
                                       });
                }
                __syncthreads();
                // skip if any column of [mf, mt] is empty in the full recompute (Seq.pm:808)
                int empty = 0;
                for (int c = tid; c < ncol; c += CNS_THREADS) if (!f6a[c]) empty = 1;
                empty = block_or(empty, ired);
                if (empty) continue;
                int npos = 0, ntot = 0;
                for (int c = tid; c < ncol; c += CNS_THREADS) {
                    bool nel = false, ner = false;
                    for (int s = 0; s < 6; ++s) { nel |= f6l[c * 6 + s] != 0u; ner |= f6r[c * 6 + s] != 0u; }
                    for (int e = 0; e < CHIM_TCAP; ++e) {
                        nel |= tkl[e] != 0u && (int)(tkl[e] >> 11) - 1 == c;
                        ner |= tkr[e] != 0u && (int)(tkr[e] >> 11) - 1 == c;
                    }
                    if (!nel || !ner) continue;
                    const double hr = chim_hx(1, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                    const double hl = chim_hx(0, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                    const double hc = chim_hx(2, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                    const double hgt = hr > hl ? hr : hl;
                    ++ntot;
                    if (hc - hgt > 0.7) ++npos;
                }
                long long tp, tt;
                block_scan_excl(npos, scan, &tp);
                block_scan_excl(ntot, scan, &tt);
                if (tid == 0 && tt > 0 && C->nchim >= (int)(D.chim_off[lr + 1] - c_off)) C->flag = 1;
                else if (tid == 0 && tt > 0) {
                    int32_t *rec = D.o_chim + 4 * (c_off + C->nchim);
                    rec[0] = mf + bs; rec[1] = mt - bs; rec[2] = (int32_t)tp; rec[3] = (int32_t)tt;
                    C->nchim += 1;
                }
                __syncthreads();
            }
            nch = C->nchim;
            // bam2cns:479-486 coordinate correction through the consensus CIGAR,
            // with the m//g position carried across records (and reset when exhausted)
            if (tid == 0 && nch) {
                long cM = 0, cI = 0, cD = 0;
                int rp = 0;
                for (int k = 0; k < nch; ++k) {
                    int32_t *rec = D.o_chim + 4 * (c_off + k);
                    const long from = rec[0];
                    for (;;) {
                        if (rp >= nruns) { rp = 0; break; }
                        const uint32_t op = D.o_cig[o0 + rp];
                        ++rp;
                        if (!(cM + cI < from)) break;
                        const long len = (long)(op >> 4);
                        const uint32_t o = op & 15u;
                        if (o == 0) cM += len; else if (o == 1) cI += len; else cD += len;
                    }
                    const long pc = cD - cI;
                    rec[0] = (int32_t)(rec[0] + pc);
                    rec[1] = (int32_t)(rec[1] + pc);
                }
            }
            __syncthreads();
            if (C->flag) {
                if (tid == 0) D.status[lr] = PR_ERR_CODE_CAP;
                __syncthreads();
            }
        }
        CNS_TICK(6);
        if (tid == 0) {
            if (!C->flag) D.status[lr] = 0;
            D.seq_len[lr] = C->run_seq;
            D.trace_len[lr] = tlen;
            D.ncigar[lr] = nruns;
            D.nchim[lr] = nch;
        }
        __syncthreads();
    }
    if (D.prof && tid == 0)
        for (int k = 0; k < CNS_NPHASE; ++k) atomicAdd(&D.prof[k], pt[k]);
#undef CNS_TICK
}

}  // namespace prgpu

namespace prgpu {
int cns_launch(const CnsDev &D, const CnsParamsDev &P, int grid, void *stream) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)cns_lr_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, CNS_LDS_BYTES);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipLaunchKernelGGL(cns_lr_kernel, dim3(grid), dim3(CNS_THREADS), CNS_LDS_BYTES,
                       (hipStream_t)stream, D, P);
    return (int)hipGetLastError();
}
int cns_lds_bytes() { return CNS_LDS_BYTES; }
int cns_max_bins() { return MAX_BINS_LDS; }
}  // namespace prgpu
