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

#include <cstdlib>
#include <stdint.h>

#include "cns_dev.h"

namespace prgpu {

// ---------------------------------------------------------------------------
// numeric helpers (Seq.pm:136-156)
__device__ __forceinline__ double phred2freq(int p) {
    double x = __dadd_rn(__dmul_rn(__ddiv_rn(__dmul_rn((double)p, (double)p), 120.0), 100.0), 0.5);
    return __ddiv_rn((double)(long long)x, 100.0);
}
// int(sqrt(120 f) + 0.5) capped at 40: 40 for every f >= 14 (sqrt(1680) + 0.5 > 41); integer
// counts below 14 from a table (their square roots are nowhere near a rounding boundary)
__device__ __forceinline__ int freq2phred(double f) {
    if (f >= 14.0) return 40;
    const int m = (int)f;
    if ((double)m == f && m >= 0) {   // 0 11 15 19 22 24 27 29 | 31 33 35 36 38 39
        const unsigned long long t = m < 8 ? 0x1D1B1816130F0B00ULL : 0x000027262423211FULL;
        return (int)((t >> (8 * (m & 7))) & 0xFFu);
    }
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
__device__ __forceinline__ uint8_t ascii_comp(uint8_t c) {
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        default: return c;
    }
}
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
// fixed-state index (A0 T1 G2 C3 -4 N5) of SEQ position s as SAM prints it, branchless for
// nt4 pools (A0 C1 G2 T3 N4; reverse complement through the second nibble table)
__device__ __forceinline__ int fixed_idx_at(const SeqV &v, int s) {
    if (v.nt4) {
        uint32_t c = v.rc ? v.p[v.n - 1 - s] : v.p[s];
        c = c > 4u ? 4u : c;
        return (int)(((v.rc ? 0x50321u : 0x51230u) >> (4u * c)) & 15u);
    }
    return fixed_idx(v[s]);
}
__device__ __forceinline__ uint64_t state_key(const SeqV &v, int off, int n) {
    if (v.nt4 && n <= 19) {   // every nt4 code is one of ACGTN: the injective key, no ASCII round trip
        uint64_t k = (uint64_t)n << 57;
        for (int i = 0; i < n; ++i) {
            const int s = off + i;
            uint32_t c = v.rc ? v.p[v.n - 1 - s] : v.p[s];
            c = c > 4u ? 4u : c;
            if (v.rc && c < 4u) c = 3u - c;
            // code5 of 'A','C','G','T','N' = 1..5 = nt4 code + 1
            k |= (uint64_t)(c + 1u) << (3 * i);
        }
        return k;
    }
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
    // a rolling window of the next 4 ops: each op is loaded 4 iterations before it is used
    // (4 loads in flight instead of one HBM latency per op; 8 measured no faster)
    constexpr int PF = 4;
    uint32_t w[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) w[u] = cb + u < ce ? cg[cb + u] : 0u;
    for (int k = cb; k < ce; ++k) {
        const uint32_t c = w[0];
#pragma unroll
        for (int u = 0; u + 1 < PF; ++u) w[u] = w[u + 1];
        w[PF - 1] = k + PF < ce ? cg[k + PF] : 0u;
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
    for (int k0 = 0; k0 < n; k0 += 8) {   // 8 independent loads in flight (the later passes hit cache)
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = k0 + u < n ? cg[k0 + u] : 0u;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (k0 + u >= n) break;
            const int op = v[u] & 15, m = (int)(v[u] >> 4);
            if (op > 8) st |= ST_SAM;
            if (op == 0 || op == 1 || op == 4 || op == 7 || op == 8) qlen += m;
            if (op == 0 || op == 2) md += m;
            if (op == 1 && m == 0) st |= ST_SAM;
        }
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
// LDS geometry.  One dynamic array per workgroup (16-byte aligned regions):
//   control block + scan scratch | region A: insertion-state table | region B: window
// buffers (fixed-state counts, (column, insertion state) counts, per-column best
// insertion, ignore bits, work-item prefix, argmax outputs) — chimera tables alias B;
// the binning arrays of phase 2 use A and B together.
// Three geometries: a small one (GeoM, 4 workgroups per CU; or GeoS, 2 per CU) takes every
// read first; a read whose tables overflow it is rerun with the large one (1 per CU).
constexpr int SLOT_SH = 12;                 // window / chimera keys: (column + 1) << 12 | state slot
constexpr uint32_t SLOT_MASK = (1u << SLOT_SH) - 1u;

// the pileup: kept alignments processed by groups of CNS_GW lanes, CNS_NG per wave
#ifndef CNS_GW_DEF
#define CNS_GW_DEF 16
#endif
constexpr int CNS_GW = CNS_GW_DEF;   // lanes per kept alignment in the pileup (16: four per wave)
constexpr int CNS_NG = 64 / CNS_GW;  // alignments per wave
#ifndef CNS_OPF_DEF
#define CNS_OPF_DEF 3
#endif
constexpr int CNS_OPF = CNS_GW == 16 ? CNS_OPF_DEF : 2;       // CIGAR ops per lane loaded ahead (16 x CNS_OPF_DEF / 64 ops)
constexpr int CNS_SEQ_DW = CNS_GW == 16 ? 40 : 64;            // SEQ dwords a group keeps in LDS (160 / 256 bytes)
constexpr int CNS_SEQ_PL = (CNS_SEQ_DW + CNS_GW - 1) / CNS_GW; // of them per lane

template <int TCAP_, int W_, int WCAP_, int WGCU_, bool RETRY_>
struct CnsGeo {
    static constexpr int TCAP = TCAP_;      // distinct insertion states per read
    static constexpr int W = W_;            // pileup window columns
    static constexpr int WCAP = WCAP_;      // (column, insertion state) pairs per window
    static constexpr int WGCU = WGCU_;      // workgroups per CU (launch bounds)
    static constexpr bool RETRY = RETRY_;   // capacity overflows go to the retry list
    static constexpr int OFF_CTRL = 0;
    static constexpr int OFF_SCAN = 256;
    static constexpr int OFF_A = OFF_SCAN + 2048;
    static constexpr int SZ_A = TCAP * 24;
    static constexpr int OFF_B = OFF_A + SZ_A;
    static constexpr int B_CNT = 0;                         // u32 [3W]: A|T<<16, G|C<<16, -|N<<16
    static constexpr int B_BEST = B_CNT + 12 * W;           // u64 [W] best insertion state per column
    static constexpr int B_WKEY = B_BEST + 8 * W;           // u32 [WCAP]
    static constexpr int B_WCNT = B_WKEY + 4 * WCAP;        // u32 [WCAP]
    static constexpr int B_IGN = B_WCNT + 4 * WCAP;         // u32 [W/32] ignored columns (MCR ranges)
    static constexpr int WAVE_BYTES = 64 * 16 + (64 / CNS_GW) * CNS_SEQ_DW * 4;   // per wave: op tables int4[NG][GW], SEQ dwords u32[NG][SEQ_DW]
    static constexpr int B_WAVE = (B_IGN + W / 8 + 15) & ~15;
    static constexpr int SZ_WIN = B_WAVE + (CNS_THREADS / 64) * WAVE_BYTES;
    static constexpr int SZ_CHIM = (CHIM_MAXCOLS * 13 + CHIM_TCAP * 4 + 16) * 4 +
                                   CHIM_MAXCOLS * (4 + CHIM_CL * 12);   // + the per-column entry lists
    static constexpr int SZ_B = ((SZ_WIN > SZ_CHIM ? SZ_WIN : SZ_CHIM) + 15) & ~15;
    static constexpr int LDS = OFF_B + SZ_B;
    static constexpr int MAX_BINS = (SZ_A + SZ_B - CNS_THREADS * 4) / 8;
    static_assert(LDS * WGCU <= 160 * 1024, "LDS per CU");
    static_assert(TCAP <= (1 << SLOT_SH), "slots fit the key");
    static_assert(W % CNS_THREADS == 0 && W % 32 == 0, "window shape");
    static_assert(B_BEST % 8 == 0 && B_WAVE % 16 == 0, "alignment");
};
// the first pass: 1024-column windows, 4 workgroups per CU (16 waves per CU: the per-alignment
// wave work is latency-bound, occupancy hides it); GeoS (more insertion states, 2 per CU)
// stays selectable with PRGPU_CNS_GEO=S; GeoL (1 per CU) reruns the reads that overflow
using GeoS = CnsGeo<512, 1024, 1024, 2, true>;
#ifndef CNS_M_WGCU
#define CNS_M_WGCU 4
#endif
using GeoM = CnsGeo<256, 1024, 512, CNS_M_WGCU, true>;
using GeoL = CnsGeo<2048, 1024, 8192, 1, false>;

// per-column descriptor: flag bits above the 12-bit state-table slot
constexpr uint32_t DESC_FIXED = 1u << 16;
constexpr uint32_t DESC_INS = 1u << 17;

struct Ctrl {
    int lr;
    int err_code;
    unsigned long long err_first;   // atomicMin (index<<8 | code)
    int run_seq, run_trace;
    int cand_b0, cand_b1;
    int nchim;
    int flag;
    int nk, maxspan, nrun, nins;
};

__device__ __forceinline__ bool in_ign(const int32_t *ig, int nig, int col) {
    for (int r = 0; r < nig; ++r)
        if (col >= ig[2 * r] && col < ig[2 * r] + ig[2 * r + 1]) return true;
    return false;
}

// state table (region A after binning)
template <int TCAP>
struct STab {
    unsigned long long *key;  // TCAP
    unsigned int *ord_cns;    // TCAP (min order of non-ignored occurrences)
    unsigned int *ord_all;    // TCAP (min order of all occurrences)
    unsigned long long *exem; // TCAP  len<<48 | SEQ offset<<32 | alignment index
    __device__ __forceinline__ int find(uint64_t k) const {
        uint32_t h = key_slot_hash(k) & (TCAP - 1);
        for (int p = 0; p < TCAP; ++p) {
            const uint64_t x = key[h];
            if (x == k) return (int)h;
            if (x == 0) return -1;
            h = (h + 1) & (TCAP - 1);
        }
        return -1;
    }
    __device__ __forceinline__ int insert(uint64_t k, uint64_t ex) const {
        uint32_t h = key_slot_hash(k) & (TCAP - 1);
        for (int p = 0; p < TCAP; ++p) {
            const unsigned long long x = key[h];
            if (x == k) return (int)h;
            if (x == 0) {
                const unsigned long long old = atomicCAS(&key[h], 0ULL, (unsigned long long)k);
                if (old == 0ULL) { exem[h] = ex; return (int)h; }
                if (old == k) return (int)h;
            }
            h = (h + 1) & (TCAP - 1);
        }
        return -1;
    }
    // chimera-table ordering key for a slot: consensus indices first, then states first
    // seen only in the no-ignore recompute (Seq.pm:777, 446)
    __device__ __forceinline__ unsigned long long chim_order(int slot) const {
        const unsigned int oc = ord_cns[slot];
        return oc != 0xFFFFFFFFu ? (unsigned long long)oc : (1ULL << 32) | ord_all[slot];
    }
};

// (column-in-window + 1) << SLOT_SH | slot -> count, open addressing in LDS
template <int WCAP>
__device__ __forceinline__ int wtab_add(uint32_t *wkey, uint32_t *wcnt, uint32_t key) {
    uint32_t h = (key * 2654435761u) >> (32 - __builtin_ctz(WCAP));
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
template <int TCAP>
__device__ double chim_hx(int side, int c, const uint32_t *f6l, const uint32_t *f6r, const uint32_t *tkl,
                          const uint32_t *tcl, const uint32_t *tkr, const uint32_t *tcr, const STab<TCAP> &T) {
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
                    if (!k || (int)(k >> SLOT_SH) - 1 != c) continue;
                    const int slot = (int)(k & SLOT_MASK);
                    const unsigned long long o = T.chim_order(slot);
                    if ((first || o > prev) && o < best) { best = o; bslot = slot; }
                }
            }
            if (bslot < 0) break;
            const uint32_t key = ((uint32_t)(c + 1) << SLOT_SH) | (uint32_t)bslot;
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

// chim_hx over a column's merged entry list (chim_cols): n insertion states sorted by their
// chimera-table order (ok: order << SLOT_SH | slot), each with its left / right counts (cnt: l | r
// << 16).  The same additions in the same order as chim_hx's selection over the whole tables (a
// state absent from a side has count 0 there and adds nothing), so the same doubles.
__device__ double chim_hx_list(int side, int c, const uint32_t *f6l, const uint32_t *f6r, const unsigned long long *ok,
                               const uint32_t *cnt, int n) {
    const double l2 = log(2.0);
    double total = 0.0;
    for (int s = 0; s < 6; ++s) {
        const uint32_t v = (side != 1 ? f6l[c * 6 + s] : 0u) + (side != 0 ? f6r[c * 6 + s] : 0u);
        if (v) total += (double)v;
    }
    auto ins = [&](int k) -> uint32_t {
        const uint32_t x = cnt[k];
        return side == 0 ? (x & 0xFFFFu) : side == 1 ? (x >> 16) : (x & 0xFFFFu) + (x >> 16);
    };
    for (int k = 0; k < n; ++k) {
        const uint32_t v = ins(k);
        if (v) total += (double)v;
    }
    double h = 0.0;
    for (int s = 0; s < 6; ++s) {
        const uint32_t v = (side != 1 ? f6l[c * 6 + s] : 0u) + (side != 0 ? f6r[c * 6 + s] : 0u);
        if (!v) continue;
        const double p = (double)v / total;
        h -= p * (log(p) / l2);
    }
    for (int k = 0; k < n; ++k) {
        const uint32_t v = ins(k);
        if (!v) continue;
        const double p = (double)v / total;
        h -= p * (log(p) / l2);
    }
    (void)ok;
    return h;
}

// ---------------------------------------------------------------------------
// Append slot in an LDS list for every active lane: one atomic per wave (the lanes that
// reach the call together), ranks by lane order.
__device__ __forceinline__ int wave_append(int *ctr) {
    const unsigned long long m = __ballot(1);
    const int lane = (int)__lane_id();
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr, __popcll(m));
    base = __shfl(base, leader, 64);
    return base + __popcll(m & ((1ULL << lane) - 1ULL));
}

// ---------------------------------------------------------------------------
// inclusive prefix sum over each GW-lane group of the wave (row shifts 1, 2, 4, 8 scan the
// rows of 16; for 32-lane groups row_bcast:15 carries row 0's total into row 1, row 2's into 3)
template <int GW>
__device__ __forceinline__ int group_incl_scan(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    if (GW == 32) v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    return v;
}

// Lane exchanges inside a 16-lane group as DPP row operations (VALU, no LDS round trip):
// lane l of the row gets lane l + D's value (D = 1, 2; the row's last lanes get 0), or lane F's.
template <int D>
__device__ __forceinline__ uint32_t row_down(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + D, 0xf, 0xf, true);   // row_shl:D
}
template <int F>
__device__ __forceinline__ int row_bcast(int v) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + F, 0xf, 0xf, false);   // row_newbcast:F
}

// the number of the row's lanes whose v <= x (x per lane), from 16 row broadcasts
template <int F = 0>
__device__ __forceinline__ int row_count_le(int v, int x) {
    if constexpr (F == 16) {
        return 0;
    } else {
        return (row_bcast<F>(v) <= x ? 1 : 0) + row_count_le<F + 1>(v, x);
    }
}

// a wave's LDS writes visible to its own later LDS reads (lanes exchange through LDS)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// field F of the K entry held in lanes 0..11 of each group, for every lane of the group
template <int F>
__device__ __forceinline__ int32_t kfld(int32_t kv, int g) {
    if constexpr (CNS_GW == 16) {
        return __builtin_amdgcn_update_dpp(0, kv, 0x150 + F, 0xf, 0xf, false);   // row_newbcast:F
    } else {
        const int32_t a0 = __builtin_amdgcn_readlane(kv, F), a1 = __builtin_amdgcn_readlane(kv, 32 + F);
        return g ? a1 : a0;
    }
}

// One kept alignment's states inside the window [cmin, cmax) (walk_states' semantics,
// Seq.pm:396-461) by one 32-lane half of a wave, op-parallel: lane k of the half takes CIGAR op
// k (chunks of 32 ops; c_first0 / c_first1: this lane's ops of the first two chunks, loaded
// ahead by the caller) and half-wave scans give every op its first column and SEQ position
// (q0 = the SEQ position of the first kept base).  An op that owns columns (M / D with n > 0,
// a leading I: one column) ends in a deferred state: when insertions follow it (zero-length
// ops skipped), or for a leading I, that last column holds a multi-character state -- base +
// inserted bases; after a D the inserted bases replace '-' (a single inserted base is then a
// one-character state) -- emitted by the op's own lane as special(column, SEQ position,
// length).  Every other column is a single-base or '-' state, visited as column(column, SEQ
// position or -1 for '-'): each lane takes a contiguous block of the chunk's columns, finds
// the first one's op by a binary search over the chunk's op starts (ops: the half's LDS
// table, 32 int4) and walks on from there.  The two halves of a wave run their own
// alignments (their loops may differ in length: every cross-lane step stays in the half).
template <bool COLS = true, class FS, class FC>
__device__ __forceinline__ void group_states(const uint32_t *cg, int nop, int rp, int q0, int cmin, int cmax, int4 *ops,
                                             const uint32_t (&c_first)[CNS_OPF], FS &&special, FC &&column) {
    constexpr int GW = CNS_GW;
    const int lane = (int)__lane_id();
    const int gl = lane & (GW - 1), glast = (lane & ~(GW - 1)) + GW - 1;
    int col0 = rp, qb = q0;
    for (int k0 = 0; k0 < nop && col0 < cmax; k0 += GW) {
        const int k = k0 + gl;
        const bool valid = k < nop;
        uint32_t c = valid && k0 >= CNS_OPF * GW ? cg[k] : 0u;
#pragma unroll
        for (int u = 0; u < CNS_OPF; ++u) c = k0 == u * GW ? c_first[u] : c;
        // this lane's op of the next chunk (its first two are the last lanes' look-ahead below:
        // from the caller's registers, not a dependent HBM load on every chunk)
        uint32_t cn = 0u;
        if (k0 + GW >= CNS_OPF * GW) {
            if (gl < 2 && k + GW < nop) cn = cg[k + GW];
        } else {
#pragma unroll
            for (int u = 0; u + 1 < CNS_OPF; ++u) cn = k0 == u * GW ? c_first[u + 1] : cn;
        }
        uint32_t n0, n1;
        if constexpr (GW == 16) {
            n0 = (uint32_t)row_bcast<0>((int)cn);
            n1 = (uint32_t)row_bcast<1>((int)cn);
        } else {
            n0 = __shfl(cn, 0, GW);
            n1 = __shfl(cn, 1, GW);
        }
        const int n = (int)(c >> 4), code = (int)(c & 15u);
        const bool lead = k == 0 && code == 1;
        const int ncol = !valid ? 0 : (code == 0 || code == 2) ? n : (lead ? 1 : 0);
        const int qadv = valid && (code == 0 || code == 1) ? n : 0;
        uint32_t nx1, nx2;
        if constexpr (GW == 16) {
            nx1 = row_down<1>(c);
            nx2 = row_down<2>(c);
        } else {
            nx1 = __shfl_down(c, 1, GW);
            nx2 = __shfl_down(c, 2, GW);
        }
        const int sc = group_incl_scan<GW>(ncol), sq = group_incl_scan<GW>(qadv);
        // inserted bases right after an op that owns columns (zero-length ops skipped)
        int tot = 0;
        if (ncol > 0 && k + 1 < nop) {
            const uint32_t x1 = gl <= GW - 2 ? nx1 : n0;
            if ((x1 & 15u) == 1u || (x1 >> 4) == 0u) {
                tot = (x1 & 15u) == 1u ? (int)(x1 >> 4) : 0;
                for (int j = k + 2; j < nop; ++j) {
                    const uint32_t x2 = j != k + 2 ? cg[j] : gl <= GW - 3 ? nx2 : gl == GW - 2 ? n0 : n1;
                    if ((x2 & 15u) == 1u) tot += (int)(x2 >> 4);
                    else if ((x2 >> 4) != 0u) break;
                }
            }
        }
        const int cs = col0 + sc - ncol, qs = qb + sq - qadv;
        int ctot, qtot;
        if constexpr (GW == 16) {
            ctot = row_bcast<15>(sc);
            qtot = row_bcast<15>(sq);
        } else {
            ctot = __shfl(sc, glast, 64);
            qtot = __shfl(sq, glast, 64);
        }
        int scol = -1;
        if (ncol > 0 && (tot > 0 || lead)) {
            int sqp, slen;
            if (lead) { scol = cs; sqp = qs; slen = n + tot; }
            else if (code == 0) { scol = cs + n - 1; sqp = qs + n - 1; slen = 1 + tot; }
            else { scol = cs + n - 1; sqp = qs; slen = tot; }   // D + I: the insertion replaces '-'
            if (scol >= cmin && scol < cmax) special(scol, sqp, slen);
        }
        if (!COLS) {   // the deferred (insertion) states only
            col0 += ctot;
            qb += qtot;
            continue;
        }
        ops[gl] = make_int4(valid ? cs : 0x7fffffff, qs, code == 2 ? 1 : 0, scol);
        wave_sync();
        const int cA = col0 > cmin ? col0 : cmin, cB = col0 + ctot < cmax ? col0 + ctot : cmax;
        const int nv = nop - k0 < GW ? nop - k0 : GW;
        const int per = cB > cA ? (cB - cA + GW - 1) / GW : 0;
        int cc = cA + gl * per;
        int lo_dpp = 0;
        if constexpr (GW == 16) {   // (every lane of the group active: DPP reads the row)
            lo_dpp = row_count_le(valid ? cs : 0x7fffffff, cc) - 1;
            lo_dpp = lo_dpp < 0 ? 0 : lo_dpp;
        }
        if (cB > cA) {
            const int ce_ = cc + per < cB ? cc + per : cB;
            if (cc < ce_) {
                int lo;   // the last op starting at or before cc owns it
                if constexpr (GW == 16) {
                    lo = lo_dpp;
                } else {
                    lo = 0;
                    int hi = nv - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (ops[mid].x <= cc) lo = mid; else hi = mid - 1;
                    }
                }
                int4 o = ops[lo];
                int nxs = lo + 1 < nv ? ops[lo + 1].x : 0x7fffffff;
                for (; cc < ce_; ++cc) {
                    while (nxs <= cc) {
                        ++lo;
                        o = ops[lo];
                        nxs = lo + 1 < nv ? ops[lo + 1].x : 0x7fffffff;
                    }
                    if (cc == o.w) continue;   // the deferred special state, emitted above
                    column(cc, o.z ? -1 : o.y + (cc - o.x));
                }
            }
        }
        wave_sync();
        col0 += ctot;
        qb += qtot;
    }
}

// ---------------------------------------------------------------------------
// One kept alignment as a 16-lane group sees it (its SEQ bytes in the group's LDS area when
// they fit: `fast`)
struct KeptView {
    int rp, i, sb, nop, ls;
    bool rc, fast;
    const uint8_t *sl;   // SEQ base 0 (fast: the group's LDS copy)
    SeqV sv;
    int64_t cgi;         // its first CIGAR op kept
};

// Every kept alignment of K[kb, ke) that overlaps the columns [cw0, cw1) -> body(view, ops,
// op table, first ops), by CNS_NG groups of CNS_GW lanes per wave: stream wv * CNS_NG + g takes
// the entries kb + stream + NSTREAM j, software-pipelined (the next entry's first CIGAR ops
// and SEQ dwords, and the K entry of the one after it, are in flight while the current one is
// processed).  A K entry (12 ints) is held spread over lanes 0..11 of its group in one register.
#ifndef CNS_PD_M
#define CNS_PD_M 1
#endif
#ifndef CNS_PD_S
#define CNS_PD_S 1
#endif
template <int PD, class Body>
__device__ __forceinline__ void stream_kept(const CnsDev &D, const int4 *K, int kb, int ke, int cw0, int cw1,
                                            int4 *wops, uint32_t *wseq, bool snt4, Body &&body) {
    constexpr int NWAVE = CNS_THREADS / 64;
    constexpr int NSTREAM = CNS_NG * NWAVE;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int g = lane / CNS_GW, gl = lane % CNS_GW;
    const int stream = wv * CNS_NG + g;
    int4 *gops = wops + g * CNS_GW;
    uint32_t *gseq = wseq + g * CNS_SEQ_DW;
    const int32_t *Ki = reinterpret_cast<const int32_t *>(K);
    const uint32_t *gdw = reinterpret_cast<const uint32_t *>(D.seq);
    auto ldK = [&](int kk) -> int32_t {
        return kk < ke ? (gl < 12 ? Ki[12 * (int64_t)kk + gl] : 0) : (gl == 0 ? 0x7fffffff : 0);
    };
    auto overl = [&](int32_t kv) { return kfld<0>(kv, g) < cw1 && kfld<1>(kv, g) > cw0; };
    auto ldD = [&](int32_t kv, uint32_t (&op)[CNS_OPF], uint32_t (&dw)[CNS_SEQ_PL]) {
#pragma unroll
        for (int u = 0; u < CNS_OPF; ++u) op[u] = 0u;
#pragma unroll
        for (int u = 0; u < CNS_SEQ_PL; ++u) dw[u] = 0u;
        if (!overl(kv)) return;
        const int64_t so = (int64_t)(uint32_t)kfld<6>(kv, g) | ((int64_t)kfld<7>(kv, g) << 32);
        const int64_t cgi = (int64_t)(uint32_t)kfld<8>(kv, g) | ((int64_t)kfld<9>(kv, g) << 32);
        const int nop = kfld<4>(kv, g);
#pragma unroll
        for (int u = 0; u < CNS_OPF; ++u)
            if (u * CNS_GW + gl < nop) op[u] = D.cig[cgi + u * CNS_GW + gl];
        const int ndw = ((int)(so & 3) + (kfld<2>(kv, g) & 0x7FFFFFFF) + 3) >> 2;
        if (ndw <= CNS_SEQ_DW) {
#pragma unroll
            for (int u = 0; u < CNS_SEQ_PL; ++u)
                if (u * CNS_GW + gl < ndw) dw[u] = gdw[(so >> 2) + u * CNS_GW + gl];
        }
    };
    // the K entries of this stream's candidates j .. j + PD and the data of j .. j + PD - 1
    int32_t kv[PD + 1];
    uint32_t op[PD][CNS_OPF], dw[PD][CNS_SEQ_PL];
#pragma unroll
    for (int d = 0; d <= PD; ++d) kv[d] = ldK(kb + stream + d * NSTREAM);
#pragma unroll
    for (int d = 0; d < PD; ++d) ldD(kv[d], op[d], dw[d]);
    for (int kk = kb + stream; kk < ke; kk += NSTREAM) {
        uint32_t opn[CNS_OPF], dwn[CNS_SEQ_PL];
        ldD(kv[PD], opn, dwn);
        const int32_t kn = ldK(kk + (PD + 1) * NSTREAM);
        const int32_t ckv = kv[0];
        if (overl(ckv)) {
            KeptView v;
            v.rp = kfld<0>(ckv, g);
            const int e0z = kfld<2>(ckv, g);
            v.sb = kfld<3>(ckv, g);
            v.nop = kfld<4>(ckv, g);
            v.i = kfld<5>(ckv, g);
            v.ls = e0z & 0x7FFFFFFF;
            v.rc = e0z < 0;
            const int64_t so = (int64_t)(uint32_t)kfld<6>(ckv, g) | ((int64_t)kfld<7>(ckv, g) << 32);
            v.cgi = (int64_t)(uint32_t)kfld<8>(ckv, g) | ((int64_t)kfld<9>(ckv, g) << 32);
            const int head = (int)(so & 3);
            const int ndw = (head + v.ls + 3) >> 2;
            v.fast = ndw <= CNS_SEQ_DW;
            if (v.fast) {
#pragma unroll
                for (int u = 0; u < CNS_SEQ_PL; ++u)
                    if (u * CNS_GW + gl < CNS_SEQ_DW) gseq[u * CNS_GW + gl] = dw[0][u];
            }
            v.sl = reinterpret_cast<const uint8_t *>(gseq) + head;
            v.sv.p = v.fast ? v.sl : D.seq + so;   // (the insertion states' keys; the slow path's bases)
            v.sv.n = v.ls;
            v.sv.rc = v.rc;
            v.sv.nt4 = snt4;
            wave_sync();
            body(v, gops, op[0]);
        }
#pragma unroll
        for (int d = 0; d < PD; ++d) kv[d] = kv[d + 1];
        kv[PD] = kn;
#pragma unroll
        for (int d = 0; d + 1 < PD; ++d) {
#pragma unroll
            for (int u = 0; u < CNS_OPF; ++u) op[d][u] = op[d + 1][u];
#pragma unroll
            for (int u = 0; u < CNS_SEQ_PL; ++u) dw[d][u] = dw[d + 1][u];
        }
#pragma unroll
        for (int u = 0; u < CNS_OPF; ++u) op[PD - 1][u] = opn[u];
#pragma unroll
        for (int u = 0; u < CNS_SEQ_PL; ++u) dw[PD - 1][u] = dwn[u];
    }
}

// ---------------------------------------------------------------------------
// One long read per workgroup (persistent: workgroups dequeue reads).  G: LDS geometry.

template <class G>
__global__ void __launch_bounds__(CNS_THREADS, G::WGCU) cns_lr_kernel(CnsDev D, CnsParamsDev P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Ctrl *C = reinterpret_cast<Ctrl *>(smem + G::OFF_CTRL);
    long long *scan = reinterpret_cast<long long *>(smem + G::OFF_SCAN);
    uint8_t *A = smem + G::OFF_A;
    uint8_t *B = smem + G::OFF_B;
    const int tid = threadIdx.x;
    // the reads this launch takes: all of them, or (large geometry) the retry list
    const int n_reads = G::RETRY ? D.n_lr : D.retry_n[0];
    int32_t *work = G::RETRY ? D.work : D.work + 1;
    // phase clock (thread 0, 100 MHz wall clock): ticks per phase summed over workgroups,
    // kept in LDS after the control block (not in every lane's registers)
    static_assert(sizeof(Ctrl) <= 64 && 64 + 8 * CNS_NPHASE <= G::OFF_SCAN, "phase clock slots");
    unsigned long long *pt = reinterpret_cast<unsigned long long *>(smem + 64);
    if (tid < CNS_NPHASE) pt[tid] = 0ULL;
    __syncthreads();
    unsigned long long tlast = wall_clock64();
#define CNS_TICK(ph)                                                      \
    do {                                                                  \
        if (D.prof && tid == 0) {                                         \
            const unsigned long long t_ = wall_clock64();                 \
            pt[ph] += t_ - tlast;                                         \
            tlast = t_;                                                   \
        }                                                                 \
    } while (0)
    // a read that overflowed the small geometry's tables goes to the retry list
#define CNS_CAP_FAIL()                                                    \
    do {                                                                  \
        if (tid == 0) {                                                   \
            D.status[lr] = PR_ERR_CODE_CAP;                               \
            D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0; \
            if (G::RETRY) D.retry[atomicAdd(D.retry_n, 1)] = lr;          \
        }                                                                 \
        __syncthreads();                                                  \
    } while (0)

    for (;;) {
        if (tid == 0) {
            const int q = atomicAdd(work, 1);
            C->lr = q < n_reads ? (G::RETRY ? q : D.retry[q]) : -1;
            C->err_first = ~0ULL;
            C->run_seq = 0;
            C->run_trace = 0;
            C->nchim = 0;
            C->flag = 0;
        }
        __syncthreads();
        const int lr = C->lr;
        CNS_TICK(7);
        if (lr < 0) break;
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
        if (nbins > G::MAX_BINS) {   // the binning arrays do not fit this geometry's LDS
            CNS_CAP_FAIL();
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

        // ---- 3. insertion-state table: first-seen order (Seq.pm:446-448) of every kept
        //         alignment's multi-character states (a thread per alignment: walk_states),
        //         and the kept alignments bucketed by the pileup window they start in (K pool
        //         of this workgroup, HBM)
        STab<G::TCAP> T;
        T.key = reinterpret_cast<unsigned long long *>(A);
        T.exem = T.key + G::TCAP;
        T.ord_cns = reinterpret_cast<unsigned int *>(T.exem + G::TCAP);
        T.ord_all = T.ord_cns + G::TCAP;
        for (int h = tid; h < G::TCAP; h += CNS_THREADS) {
            T.key[h] = 0ULL; T.exem[h] = 0ULL; T.ord_cns[h] = 0xFFFFFFFFu; T.ord_all[h] = 0xFFFFFFFFu;
        }
        const int nwin = (int)((L + G::W - 1) / G::W);
        int32_t *wcur = reinterpret_cast<int32_t *>(B + G::B_CNT);   // per-window counters (<= 3W)
        // K pool of this workgroup: Kh[0, nwin] window starts, Ks[0, nwin) the start of each
        // window's straddlers (alignments that run past the window's end: they sit last in their
        // window, so the candidates of window w are the contiguous K[Ks[w - wback], Kh[w + 1])),
        // then the entries
        int32_t *Kh = D.k_pool + (int64_t)blockIdx.x * D.k_cap;
        int32_t *Ks = Kh + nwin + 1;
        int4 *K = reinterpret_cast<int4 *>(Kh + ((2 * nwin + 4) & ~3));
        int32_t *wst = wcur + nwin + 1;   // per-window straddler counters
        const int wv = tid >> 6;
        int4 *wops = reinterpret_cast<int4 *>(B + G::B_WAVE + wv * G::WAVE_BYTES);   // this wave's op table
        uint32_t *wseq = reinterpret_cast<uint32_t *>(B + G::B_WAVE + wv * G::WAVE_BYTES + 64 * 16);   // its SEQ dwords
        const bool snt4 = D.seq_nt4 != 0;
        if (tid == 0) { C->nk = 0; C->maxspan = 0; }
        for (int x = tid; x < 2 * (nwin + 1) && x < 3 * G::W; x += CNS_THREADS) wcur[x] = 0;
        __syncthreads();
        if (2 * (nwin + 1) > 3 * G::W) C->flag = 1;
        for (int i = tid; i < na; i += CNS_THREADS) {   // a thread per kept alignment: the window counts
            const int64_t g = a0 + i;
            if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
            const int rp = D.a_rpos[g], span = D.a_end[g] - rp;
            atomicAdd(&C->nk, 1);
            atomicMax(&C->maxspan, span);
            const int win = rp / G::W;
            if (2 * (nwin + 1) <= 3 * G::W) {
                atomicAdd(&wcur[win], 1);
                if (D.a_end[g] > (win + 1) * G::W) atomicAdd(&wst[win], 1);
            }
        }
        __syncthreads();
        // 16-bit fixed-state counters: at most 65535 kept alignments per read
        if (C->flag || (int64_t)((2 * nwin + 4) & ~3) + 12 * (int64_t)C->nk > D.k_cap || C->nk > 65535) {
            CNS_CAP_FAIL();
            continue;
        }
        {   // window starts: exclusive scan of the per-window counts
            const int per = (nwin + 1 + CNS_THREADS - 1) / CNS_THREADS;
            const int b0 = tid * per, b1 = (b0 + per) < nwin + 1 ? (b0 + per) : nwin + 1;
            long long s = 0;
            for (int w = b0; w < b1; ++w) s += w < nwin ? wcur[w] : 0;
            long long tot;
            long long base = block_scan_excl(s, scan, &tot);
            for (int w = b0; w < b1; ++w) {
                Kh[w] = (int32_t)base;
                if (w < nwin) Ks[w] = (int32_t)base + wcur[w] - wst[w];
                base += w < nwin ? wcur[w] : 0;
            }
            __syncthreads();
            for (int w = tid; w < nwin; w += CNS_THREADS) { wcur[w] = 0; wst[w] = 0; }
            __syncthreads();
        }
        for (int i = tid; i < na; i += CNS_THREADS) {
            const int64_t g = a0 + i;
            if (!D.kept[g] || (D.a_st[g] & ST_SMSKIP)) continue;
            const int rp = D.a_rpos[g], win = rp / G::W;
            const int kpos = D.a_end[g] > (win + 1) * G::W ? Ks[win] + atomicAdd(&wst[win], 1)
                                                           : Kh[win] + atomicAdd(&wcur[win], 1);
            // the entry carries what a window's wave needs (one 48-byte record instead of seven
            // scattered per-alignment loads per window)
            const int cbk = D.a_cb[g];
            const int64_t so = D.seq_off[g], cgi = D.cig_off[g] + cbk;
            int4 *Ke = K + 3 * (int64_t)kpos;
            Ke[0] = make_int4(rp, D.a_end[g], D.lseq[g] | ((D.aflags[g] & 8) ? (int)0x80000000 : 0), D.a_sb[g]);
            Ke[1] = make_int4(D.a_ce[g] - cbk, i, (int)(uint32_t)(so & 0xFFFFFFFFLL), (int)(so >> 32));
            Ke[2] = make_int4((int)(uint32_t)(cgi & 0xFFFFFFFFLL), (int)(cgi >> 32), 0, 0);
            // its multi-character states (walk_states: the thread walks its own ops, a kept
            // alignment per thread -- every thread busy, ~700 independent walks in flight per
            // read, where a 16-lane group per alignment kept 16 in flight); the state index of
            // a column is column - rp
            const SeqV sv = seq_view(D, g);
            const int sbg = D.a_sb[g];
            walk_states<true>(D.cig + D.cig_off[g], cbk, D.a_ce[g], rp, 0, 0x7fffffff,
                              [&](int scol, int, int, int qoff, int slen) {
                                  const int sqp = sbg + qoff;
                                  if (slen > 0xFFFF || sqp > 0xFFFF || g > 0xFFFFFFFFLL) { C->flag = 1; return; }
                                  const uint64_t k = state_key(sv, sqp, slen);
                                  const int h = T.insert(k, ((uint64_t)slen << 48) | ((uint64_t)sqp << 32) | (uint64_t)g);
                                  if (h < 0) { C->flag = 1; return; }
                                  const unsigned int ord = ((unsigned int)i << 12) | (unsigned int)(scol - rp);
                                  atomicMin(&T.ord_all[h], ord);
                                  if (!(nig && in_ign(ig, nig, scol))) atomicMin(&T.ord_cns[h], ord);
                              });
        }
        __threadfence_block();
        __syncthreads();
        if (C->flag) {
            CNS_CAP_FAIL();
            continue;
        }
        const int wback = (C->maxspan + G::W - 1) / G::W;   // windows an alignment can reach back
        CNS_TICK(2);

        // ---- 4. windowed pileup (Seq.pm:438-461) + argmax (Seq.pm:1568-1654).  Per window of
        //   W columns: every kept alignment overlapping it is taken by one wave (wave_states:
        //   the Perl state semantics, op-parallel, columns lane-parallel, its SEQ bytes in the
        //   wave's LDS area); fixed states go to 16-bit LDS counters, insertion states to the
        //   window's (column, slot) table; then the best insertion state per column (count,
        //   then first-seen order), the argmax with the reference quality, a block scan of the
        //   output lengths and the coalesced write of seq / qual / trace.
        uint32_t *cnt = reinterpret_cast<uint32_t *>(B + G::B_CNT);
        uint32_t *wkey = reinterpret_cast<uint32_t *>(B + G::B_WKEY);
        uint32_t *wcnt = reinterpret_cast<uint32_t *>(B + G::B_WCNT);
        unsigned long long *best = reinterpret_cast<unsigned long long *>(B + G::B_BEST);
        uint32_t *ignb = reinterpret_cast<uint32_t *>(B + G::B_IGN);
        const bool use_rq = P.use_ref_qual && D.ref_seq && D.ref_qual;
        constexpr int CPT = G::W / CNS_THREADS;   // argmax columns per thread
        for (int wi = 0; wi < nwin; ++wi) {
            const long w0 = (long)wi * G::W;
            const int wn = (L - w0) < G::W ? (int)(L - w0) : G::W;
            for (int x = tid; x < 3 * G::W; x += CNS_THREADS) cnt[x] = 0u;
            for (int x = tid; x < G::WCAP; x += CNS_THREADS) { wkey[x] = 0u; wcnt[x] = 0u; }
            for (int x = tid; x < G::W; x += CNS_THREADS) best[x] = 0ULL;
            for (int x = tid; x < G::W / 32; x += CNS_THREADS) ignb[x] = 0u;
            __syncthreads();
            for (int r = tid; r < nig; r += CNS_THREADS) {   // MCR ranges -> ignore bits
                const long s0 = ig[2 * r], s1 = s0 + ig[2 * r + 1];
                const long lo = s0 > w0 ? s0 : w0, hi = s1 < w0 + wn ? s1 : w0 + wn;
                for (long col = lo; col < hi; ++col) atomicOr(&ignb[(col - w0) >> 5], 1u << ((col - w0) & 31));
            }
            const int wb0 = wi - wback;   // the earliest window whose straddlers can reach this one
            const int kb = wb0 < 0 ? 0 : (wb0 < wi ? Ks[wb0] : Kh[wi]), ke = Kh[wi + 1];
            __syncthreads();
            CNS_TICK(8);
            if (D.prof && tid == 0) pt[14] += 1;
            const int cw0 = (int)w0, cw1 = (int)w0 + wn;
            stream_kept<G::WGCU >= 4 ? CNS_PD_M : CNS_PD_S>(D, K, kb, ke, cw0, cw1, wops, wseq, snt4, [&](const KeptView &v, int4 *gops, const uint32_t (&cop)[CNS_OPF]) {
                const uint32_t lut = v.rc ? 0x50321u : 0x51230u;   // nt4 code -> fixed-state index
                auto fixed_at = [&](int s) -> int {
                    if (v.fast && snt4) {
                        uint32_t c8 = v.sl[v.rc ? v.ls - 1 - s : s];
                        c8 = c8 > 4u ? 4u : c8;
                        return (int)((lut >> (4u * c8)) & 15u);
                    }
                    return fixed_idx_at(v.sv, s);
                };
                auto add_fixed = [&](int cc, int fi) {
                    const int c = cc - cw0;
                    if (nig && ((ignb[c >> 5] >> (c & 31)) & 1u)) return;
                    atomicAdd(&cnt[3 * c + (fi >> 1)], 1u << (16 * (fi & 1)));
                };
                group_states(D.cig + v.cgi, v.nop, v.rp, v.sb, cw0, cw1, gops, cop,
                             [&](int scol, int sqp, int slen) {
                                 if (slen == 1) { add_fixed(scol, fixed_at(sqp)); return; }
                                 const int c = scol - cw0;
                                 if (nig && ((ignb[c >> 5] >> (c & 31)) & 1u)) return;
                                 const int h = T.find(state_key(v.sv, sqp, slen));
                                 if (h < 0 || wtab_add<G::WCAP>(wkey, wcnt, ((uint32_t)(c + 1) << SLOT_SH) | (uint32_t)h) < 0)
                                     C->flag = 1;
                             },
                             [&](int cc, int qp) { add_fixed(cc, qp < 0 ? 4 : fixed_at(qp)); });
            });
            __syncthreads();
            CNS_TICK(3);
            if (C->flag) break;
            // this thread's argmax columns' reference bases and qualities, loaded now (one
            // dword each for 4 columns) and used after the best-insertion pass and its barrier
            uint32_t rq4 = 0u, rb4 = 0u;
            {
                const int cth = tid * CPT;
                const int64_t at = r0 + w0 + cth;
                if (CPT == 4 && cth + 3 < wn) {
                    if (use_rq) __builtin_memcpy(&rq4, D.ref_qual + at, 4);
                    if (D.ref_seq) __builtin_memcpy(&rb4, D.ref_seq + at, 4);
                } else {
                    for (int k = 0; k < CPT && k < 4 && cth + k < wn; ++k) {
                        if (use_rq) rq4 |= (uint32_t)D.ref_qual[at + k] << (8 * k);
                        if (D.ref_seq) rb4 |= (uint32_t)D.ref_seq[at + k] << (8 * k);
                    }
                }
            }
            auto ref_at = [&](int k, long col) -> uint8_t {   // ref_base(D, r0 + col)
                if (CPT != 4) return ref_base(D, r0 + col);
                const uint8_t c = (uint8_t)(rb4 >> (8 * k));
                return D.ref_nt4 ? nt4_ascii(c > 4 ? 4 : c) : c;
            };
            auto qual_at = [&](int k, long col) -> int {
                return CPT != 4 ? (int)D.ref_qual[r0 + col] : (int)((rq4 >> (8 * k)) & 0xFFu);
            };
            // best insertion state per column: highest count, then lowest first-seen order
            for (int x = tid; x < G::WCAP; x += CNS_THREADS) {
                const uint32_t k = wkey[x];
                if (!k) continue;
                const int slot = (int)(k & SLOT_MASK), c = (int)(k >> SLOT_SH) - 1;
                if (P.max_ins_length && ex_len(T.exem[slot]) > P.max_ins_length) continue;
                const unsigned long long v = ((unsigned long long)wcnt[x] << 44) |
                                             ((unsigned long long)(0xFFFFFFFFu - T.ord_cns[slot]) << SLOT_SH) |
                                             (unsigned long long)slot;
                atomicMax(&best[c], v);
            }
            __syncthreads();
            // argmax per column (Seq.pm:1576-1636): first index with strictly greater freq
            uint16_t olen_r[CPT];
            uint32_t desc_r[CPT];
            uint8_t ph_r[CPT];
#pragma unroll
            for (int k = 0; k < CPT; ++k) {
                const int c = tid * CPT + k;
                uint16_t olen = 0;
                uint32_t desc = 0;
                uint8_t ph = 0;
                if (c < wn) {
                    const long col = w0 + c;
                    const uint32_t q0 = cnt[3 * c], q1 = cnt[3 * c + 1], q2 = cnt[3 * c + 2];
                    const uint32_t f6[6] = {q0 & 0xFFFFu, q0 >> 16, q1 & 0xFFFFu, q1 >> 16, q2 & 0xFFFFu, q2 >> 16};
                    int rs = -1;
                    double vref = 0.0;
                    if (use_rq) {
                        const double fr = phred2freq(qual_at(k, col) - P.ref_phred_offset);
                        if (fr != 0.0) {
                            rs = fixed_idx(ref_at(k, col));
                            vref = fr;   // ref freq is added first, then +1 per alignment
                            uint32_t n = 0;
#pragma unroll
                            for (int s = 0; s < 6; ++s) n = s == rs ? f6[s] : n;
                            for (uint32_t kk = 0; kk < n; ++kk) vref = __dadd_rn(vref, 1.0);
                        }
                    }
                    double maxf = 0.0;
                    int idx = -1;
#pragma unroll
                    for (int s = 0; s < 6; ++s) {
                        const double v = s == rs ? vref : (double)f6[s];
                        if ((f6[s] != 0u || s == rs) && v > maxf) { maxf = v; idx = s; }
                    }
                    const unsigned long long bi = best[c];
                    int bslot = -1;
                    if (bi && (double)(bi >> 44) > maxf) {
                        maxf = (double)(bi >> 44);
                        idx = 6;
                        bslot = (int)(bi & SLOT_MASK);
                    }
                    if (!(maxf != 0.0)) {
                        olen = 1; desc = DESC_FIXED | (D.ref_seq ? ref_at(k, col) : (uint8_t)'n'); ph = 0;
                    } else if (idx == 4) {
                        olen = 0; desc = 0; ph = 0;
                    } else if (idx < 6) {
                        olen = 1; desc = DESC_FIXED | (uint8_t)(0x4E2D43475441ULL >> (8 * idx)); ph = (uint8_t)freq2phred(maxf);
                    } else {
                        olen = (uint16_t)ex_len(T.exem[bslot]); desc = DESC_INS | (uint32_t)bslot;
                        ph = (uint8_t)freq2phred(maxf);
                    }
                }
                olen_r[k] = olen;
                desc_r[k] = desc;
                ph_r[k] = ph;
            }
            // block scan of (seq len, trace len) over the window's columns (each thread's own
            // columns, from registers), then the write
            {
                long long s = 0;
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    const int c = tid * CPT + k;
                    if (c < wn) {
                        const long long ol = olen_r[k];
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
                if (!fits && tid == 0) C->flag = 2;
#pragma unroll
                for (int k = 0; k < CPT; ++k) {
                    const int c = tid * CPT + k;
                    if (!fits || c >= wn) break;
                    const int ol = olen_r[k];
                    const uint32_t d = desc_r[k];
                    const uint8_t qc = (uint8_t)(ph_r[k] + qch_off);
                    if (ol == 0) {
                        D.o_trace[o0 + to] = 'I';
                        to += 1;
                    } else if (d & DESC_FIXED) {
                        D.o_seq[o0 + so] = (uint8_t)(d & 0xFFu);
                        D.o_qual[o0 + so] = qc;
                        D.o_trace[o0 + to] = 'M';
                        so += 1; to += 1;
                    } else {
                        const int slot = (int)(d & SLOT_MASK);
                        const uint64_t key = T.key[slot];
                        if (!(key >> 63)) {   // an injective key holds the string: no exemplar SEQ loads
                            for (int q = 0; q < ol; ++q) {
                                D.o_seq[o0 + so + q] = (uint8_t)(0x4E544743413FULL >> (8 * ((key >> (3 * q)) & 7u)));
                                D.o_qual[o0 + so + q] = qc;
                                D.o_trace[o0 + to + q] = q ? 'D' : 'M';
                            }
                        } else {
                            const uint64_t ex = T.exem[slot];
                            const SeqV src = seq_view(D, ex_aln(ex));
                            const int eo = ex_off(ex);
                            for (int q = 0; q < ol; ++q) {
                                D.o_seq[o0 + so + q] = src[eo + q];
                                D.o_qual[o0 + so + q] = qc;
                                D.o_trace[o0 + to + q] = q ? 'D' : 'M';
                            }
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
            if (C->flag == 2) {   // output capacity (pipeline estimate): no retry helps
                if (tid == 0) {
                    D.status[lr] = PR_ERR_CODE_CAP;
                    D.seq_len[lr] = 0; D.trace_len[lr] = 0; D.ncigar[lr] = 0; D.nchim[lr] = 0;
                }
                __syncthreads();
            } else {
                CNS_CAP_FAIL();
            }
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
                // the kept alignments that can overlap [mf, mt]: the pileup's K pool range of the
                // windows mf .. mt touch (those starting there, and the straddlers of the wback
                // windows before), not every alignment of the read
                const int kw0 = mf / G::W, kw1 = mt / G::W, kwb = kw0 - wback;
                const int kb = kwb < 0 ? 0 : (kwb < kw0 ? Ks[kwb] : Kh[kw0]), ke = Kh[kw1 + 1];
                // a kept alignment's states in [mf, mt] by a 16-lane group, op-parallel (the pileup's
                // stream_kept / group_states: its SEQ in the group's LDS area), not a thread walking
                // its CIGAR; each state counted into the side tables of the bins the alignment is in
                stream_kept<G::WGCU >= 4 ? CNS_PD_M : CNS_PD_S>(D, K, kb, ke, mf, mt + 1, wops, wseq, snt4, [&](const KeptView &v, int4 *gops, const uint32_t (&cop)[CNS_OPF]) {
                    const int bin = D.a_bin[a0 + v.i];
                    const bool inl = bin >= fl && bin <= tl, inr = bin >= fr && bin <= tr;
                    const uint32_t lut = v.rc ? 0x50321u : 0x51230u;   // nt4 code -> fixed-state index
                    auto fixed_at = [&](int sq) -> int {
                        if (v.fast && snt4) {
                            uint32_t c8 = v.sl[v.rc ? v.ls - 1 - sq : sq];
                            c8 = c8 > 4u ? 4u : c8;
                            return (int)((lut >> (4u * c8)) & 15u);
                        }
                        return fixed_idx_at(v.sv, sq);
                    };
                    auto add = [&](int col, int fi, int slot) {
                        const int c = col - mf;
                        f6a[c] = 1u;
                        for (int side = 0; side < 2; ++side) {
                            if (side == 0 ? !inl : !inr) continue;
                            uint32_t *f6 = side == 0 ? f6l : f6r;
                            uint32_t *tk = side == 0 ? tkl : tkr;
                            uint32_t *tc = side == 0 ? tcl : tcr;
                            if (fi >= 0) { atomicAdd(&f6[c * 6 + fi], 1u); continue; }
                            if (slot < 0) { C->flag = 1; continue; }
                            const uint32_t key = ((uint32_t)(c + 1) << SLOT_SH) | (uint32_t)slot;
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
                    };
                    group_states(D.cig + v.cgi, v.nop, v.rp, v.sb, mf, mt + 1, gops, cop,
                                 [&](int scol, int sqp, int slen) {
                                     if (slen == 1) add(scol, fixed_at(sqp), -1);
                                     else add(scol, -1, (inl || inr) ? T.find(state_key(v.sv, sqp, slen)) : -1);
                                 },
                                 [&](int cc, int qp) { add(cc, qp < 0 ? 4 : fixed_at(qp), -1); });
                });
                __syncthreads();
                CNS_TICK(9);   // (the candidate's side tables)
                // skip if any column of [mf, mt] is empty in the full recompute (Seq.pm:808)
                int empty = 0;
                for (int c = tid; c < ncol; c += CNS_THREADS) if (!f6a[c]) empty = 1;
                empty = block_or(empty, ired);
                if (empty) continue;
                // every column's insertion-state entries of both side tables, listed once (an entry a
                // thread) and merged per state in chimera-table order, so the three Hx of a column
                // visit its few states instead of selecting each from both whole tables (the
                // selection was ~2/3 of the finish task's consensus kernel); a column with more than
                // CHIM_CL states keeps the table selection
                uint32_t *cln = reinterpret_cast<uint32_t *>(ired + 16);            // [CHIM_MAXCOLS]
                unsigned long long *clk = reinterpret_cast<unsigned long long *>(cln + CHIM_MAXCOLS);   // [.. x CHIM_CL]
                uint32_t *clc = reinterpret_cast<uint32_t *>(clk + CHIM_MAXCOLS * CHIM_CL);             // [.. x CHIM_CL]
                for (int c = tid; c < CHIM_MAXCOLS; c += CNS_THREADS) cln[c] = 0u;
                __syncthreads();
                for (int e = tid; e < 2 * CHIM_TCAP; e += CNS_THREADS) {
                    const int side = e >= CHIM_TCAP ? 1 : 0, x = e - side * CHIM_TCAP;
                    const uint32_t k = side ? tkr[x] : tkl[x];
                    if (!k) continue;
                    const int c = (int)(k >> SLOT_SH) - 1;
                    if (c < 0 || c >= CHIM_MAXCOLS) continue;
                    const uint32_t at = atomicAdd(&cln[c], 1u);
                    // (raw entries first: the table index and its side)
                    if (at < (uint32_t)CHIM_CL) clc[c * CHIM_CL + (int)at] = (uint32_t)e;
                }
                __syncthreads();
                int npos = 0, ntot = 0;
                for (int c = tid; c < ncol; c += CNS_THREADS) {
                    bool nel = false, ner = false;
                    for (int s = 0; s < 6; ++s) { nel |= f6l[c * 6 + s] != 0u; ner |= f6r[c * 6 + s] != 0u; }
                    const int ne = (int)cln[c];
                    const bool listed = ne <= CHIM_CL;
                    int nm = 0;   // merged states of the column
                    unsigned long long *mk = clk + c * CHIM_CL;
                    uint32_t *mc = clc + c * CHIM_CL;
                    if (listed) {
                        // (in place: the merged list's writes stay at or below entry k, read first)
                        for (int k = 0; k < ne; ++k) {
                            const int e = (int)mc[k], side = e >= CHIM_TCAP ? 1 : 0, x = e - side * CHIM_TCAP;
                            const uint32_t key = side ? tkr[x] : tkl[x], v = side ? tcr[x] : tcl[x];
                            nel |= side == 0;
                            ner |= side == 1;
                            const int slot = (int)(key & SLOT_MASK);
                            const unsigned long long o = (T.chim_order(slot) << SLOT_SH) | (unsigned long long)slot;
                            int j = 0;
                            while (j < nm && mk[j] != o) ++j;
                            if (j == nm) {   // insert in order
                                int i = nm++;
                                while (i > 0 && mk[i - 1] > o) { mk[i] = mk[i - 1]; mc[i] = mc[i - 1]; --i; }
                                mk[i] = o;
                                mc[i] = side ? v << 16 : v;
                            } else {
                                mc[j] += side ? v << 16 : v;
                            }
                        }
                    } else {
                        for (int e = 0; e < CHIM_TCAP; ++e) {
                            nel |= tkl[e] != 0u && (int)(tkl[e] >> SLOT_SH) - 1 == c;
                            ner |= tkr[e] != 0u && (int)(tkr[e] >> SLOT_SH) - 1 == c;
                        }
                    }
                    if (!nel || !ner) continue;
                    double hr, hl, hc;
                    if (listed) {
                        hr = chim_hx_list(1, c, f6l, f6r, mk, mc, nm);
                        hl = chim_hx_list(0, c, f6l, f6r, mk, mc, nm);
                        hc = chim_hx_list(2, c, f6l, f6r, mk, mc, nm);
                    } else {
                        hr = chim_hx(1, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                        hl = chim_hx(0, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                        hc = chim_hx(2, c, f6l, f6r, tkl, tcl, tkr, tcr, T);
                    }
                    const double hgt = hr > hl ? hr : hl;
                    ++ntot;
                    if (hc - hgt > 0.7) ++npos;
                }
                long long tp, tt;
                block_scan_excl(npos, scan, &tp);
                block_scan_excl(ntot, scan, &tt);
                CNS_TICK(10);   // (its column entropies)
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
#undef CNS_CAP_FAIL
}

static bool cns_geo_m() {
    const char *g = getenv("PRGPU_CNS_GEO");
    return !(g && g[0] == 'S');
}
int cns_wg_per_cu() { return cns_geo_m() ? GeoM::WGCU : GeoS::WGCU; }

int cns_launch(const CnsDev &D, const CnsParamsDev &P, int grid, int grid_retry, void *stream) {
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void *)cns_lr_kernel<GeoS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           GeoS::LDS);
        if (e != hipSuccess) return (int)e;
        e = hipFuncSetAttribute((const void *)cns_lr_kernel<GeoM>, hipFuncAttributeMaxDynamicSharedMemorySize, GeoM::LDS);
        if (e != hipSuccess) return (int)e;
        e = hipFuncSetAttribute((const void *)cns_lr_kernel<GeoL>, hipFuncAttributeMaxDynamicSharedMemorySize, GeoL::LDS);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    hipStream_t s = (hipStream_t)stream;
    if (!D.force_large) {
        if (cns_geo_m()) hipLaunchKernelGGL(cns_lr_kernel<GeoM>, dim3(grid), dim3(CNS_THREADS), GeoM::LDS, s, D, P);
        else hipLaunchKernelGGL(cns_lr_kernel<GeoS>, dim3(grid), dim3(CNS_THREADS), GeoS::LDS, s, D, P);
    }
    // reads whose tables outgrew the small geometry (device-side list; usually empty)
    hipLaunchKernelGGL(cns_lr_kernel<GeoL>, dim3(grid_retry), dim3(CNS_THREADS), GeoL::LDS, s, D, P);
    return (int)hipGetLastError();
}
int cns_max_bins() { return GeoL::MAX_BINS; }
int cns_k_header() { return 1024; }

}  // namespace prgpu
