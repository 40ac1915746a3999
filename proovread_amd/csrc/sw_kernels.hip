// Seed extension + CIGAR kernels for gfx950 — the ksw stage of bwa-proovread mem
// (bin/proovread:1313) as a batched inter-task SW: one (short read, long-read
// window, seed) task per lane, rows of the banded DP walked in lock-step by the
// 64 lanes of a wave.
//
//   sw_extend_kernel : mem_chain2aln for a single-seed chain — left and right
//                      ksw_extend2 (band pruning, z-drop, to-end gscore) with
//                      MAX_BAND_TRY=2 band doubling and the -L clip decision.
//   sw_global_kernel : mem_reg2aln / bwa_gen_cigar2 — infer_bw, up to three
//                      ksw_global2 passes, backtrack, D-squeeze, soft clips.
//
// Layout: the DP row state (H, E and the query base) of every lane lives in LDS
// as one 32-bit word per query column, interleaved [column][lane] so that a
// wave's 64 accesses always hit 64 distinct banks whatever column each lane is
// at.  ksw_global2's direction bytes go to a per-block slab in HBM laid out
// [row][column][lane] (64 lanes write one contiguous 64-byte segment).
// Integer VALU is the roofline (no MFMA: no dense contraction here).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sw_dev.h"

namespace prgpu {

__device__ __forceinline__ int sw_score(int t, int q, int a, int b) {
    // bwa_fill_scmat: match a, mismatch -b, anything with N (4) -1
    return (t > 3 || q > 3) ? -1 : (t == q ? a : -b);
}

// ---- extension: packed LDS word = h[0,13) | e[13,26) | 8*q[26,32)
// (H and E of ksw_extend2 are >= 0 and bounded by a * read length < 8192;
// the query base is stored pre-multiplied by 8 to index the row score table)
__device__ __forceinline__ uint32_t pk(int h, int e, uint32_t q8) {
    return (uint32_t)h | ((uint32_t)e << 13) | (q8 << 26);
}
constexpr uint32_t PK_HE = (1u << 26) - 1u;
__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }
// bwa_fill_scmat row for target base tc as bytes q = 0..4 (N row / column = -1)
__device__ __forceinline__ uint64_t score_row(int tc, int a, int b) {
    uint32_t lo;
    if (tc > 3) {
        lo = 0xFFFFFFFFu;
    } else {
        const uint32_t mm = (uint32_t)(uint8_t)(int8_t)(-b);
        lo = mm * 0x01010101u;
        lo = (lo & ~(0xFFu << (8 * tc))) | ((uint32_t)(uint8_t)a << (8 * tc));
    }
    return ((uint64_t)0xFFu << 32) | lo;
}

struct ExtIO {
    int qle, tle, gtle, gscore, max_off;
};

// ksw_extend2 for one lane.  eh: this lane's column 0 in LDS (stride 64 words).
// Query column j is Q[qb + qs*j]; target row i is comp?(L[tb + ts*i]).
__device__ int ksw_extend_lane(uint32_t *eh, const uint8_t *Q, int qb, int qs, int qlen,
                               const uint8_t *Lr, long tb, int ts, bool comp, int tlen,
                               const SwOptsDev &O, int w, int end_bonus, int h0, ExtIO &io,
                               unsigned long long &cells) {
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    // first row + query bases
    {
        int hp = h0;
        bool alive = true;
        for (int j = 0; j <= qlen; ++j) {
            int h;
            if (j == 0) h = h0;
            else if (j == 1) h = h0 > oe_ins ? h0 - oe_ins : 0;
            else {
                alive = alive && hp > e_ins;
                h = alive ? hp - e_ins : 0;
            }
            hp = h;
            const uint32_t q = j < qlen ? (uint32_t)Q[qb + qs * j] : 0u;
            eh[j * SW_WAVE] = pk(h, 0, q << 3);
        }
    }
    int max_ins = (int)((double)(qlen * a + end_bonus - o_ins) / e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    int max_del = (int)((double)(qlen * a + end_bonus - o_del) / e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    // canonical unpruned band cell count
    {
        unsigned long long c = 0;
        for (int i = 0; i < tlen; ++i) {
            const int lo = i - w > 0 ? i - w : 0;
            const int hi = i + w + 1 < qlen ? i + w + 1 : qlen;
            if (hi > lo) c += (unsigned long long)(hi - lo);
        }
        cells += c;
    }
    int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    for (int i = 0; i < tlen; ++i) {
        int f = 0, h1, m = 0, mj = -1;
        int tc = (int)Lr[tb + (long)ts * i];
        if (comp && tc < 4) tc = 3 - tc;
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else
            h1 = 0;
        const uint64_t srow = score_row(tc, a, b);
        int j;
        uint32_t wd = eh[beg * SW_WAVE];
        for (j = beg; j < end; ++j) {
            const uint32_t wn = eh[(j + 1) * SW_WAVE];   // prefetch: column j+1 is not written at j
            const int Mr = (int)(wd & 0x1FFFu);
            const int e0 = (int)((wd >> 13) & 0x1FFFu);
            const uint32_t q8 = wd >> 26;
            const int sc = (int)(int8_t)(uint8_t)(srow >> q8);
            const int M = Mr ? Mr + sc : 0;   // separating H and M (ksw: no 100M3I3D20M)
            const int h = imax3(M, e0, f);
            mj = m > h ? mj : j;
            m = m > h ? m : h;
            const int e = imax3(e0 - e_del, M - oe_del, 0);
            f = imax3(f - e_ins, M - oe_ins, 0);
            eh[j * SW_WAVE] = pk(h1, e, q8);
            h1 = h;
            wd = wn;
        }
        {
            const uint32_t w2 = eh[end * SW_WAVE];
            eh[end * SW_WAVE] = pk(h1, 0, w2 >> 26);
        }
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (m == 0) break;
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
        for (j = beg; j < end && (eh[j * SW_WAVE] & PK_HE) == 0u; ++j);
        beg = j;
        for (j = end; j >= beg && (eh[j * SW_WAVE] & PK_HE) == 0u; --j);
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    io.qle = max_j + 1;
    io.tle = max_i + 1;
    io.gtle = max_ie + 1;
    io.gscore = gscore;
    io.max_off = max_off;
    return max;
}

__device__ __forceinline__ int cal_max_gap(const SwOptsDev &O, int qlen) {
    int l_del = (int)((double)(qlen * O.a - O.o_del) / O.e_del + 1.);
    int l_ins = (int)((double)(qlen * O.a - O.o_ins) / O.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < O.w << 1 ? l : O.w << 1;
}

__global__ void __launch_bounds__(SW_WAVE) sw_extend_kernel(SwDev D, SwOptsDev O) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_eh[];
    const int lane = threadIdx.x;
    const int64_t slot = (int64_t)blockIdx.x * SW_WAVE + lane;
    unsigned long long cells = 0;
    if (slot < D.n_task) {
        const int64_t t = D.perm[slot];
        uint32_t *eh = lds_eh + lane;
        const int sid = D.t_sr[t], lid = D.t_lr[t];
        const uint8_t *Q = D.sr + D.sr_off[sid];
        const int lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
        const uint8_t *Lr = D.lr + D.lr_off[lid];
        const int L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
        const bool rev = D.t_strand[t] != 0;
        const int qbeg = D.t_qbeg[t], rbeg = D.t_rbeg[t], slen = D.t_slen[t];
        // mem_chain2aln: max possible span
        long rmax0 = (long)rbeg - (qbeg + cal_max_gap(O, qbeg));
        long rmax1 = (long)rbeg + slen + ((lq - qbeg - slen) + cal_max_gap(O, lq - qbeg - slen));
        if (rmax0 < 0) rmax0 = 0;
        if (rmax1 > L) rmax1 = L;
        int aw0 = O.w, aw1 = O.w;
        int score = -1, truesc = -1, qb, qe, rb, re;
        ExtIO io;
        if (qbeg) {
            const int tlen = (int)(rbeg - rmax0);
            // left: query Q[qbeg-1-j], target strand position rbeg-1-i
            const long tb = rev ? (long)L - rbeg : (long)rbeg - 1;
            const int ts = rev ? 1 : -1;
            unsigned long long c = 0;
            for (int i = 0; i < 2; ++i) {
                const int prev = score;
                aw0 = O.w << i;
                c = 0;
                score = ksw_extend_lane(eh, Q, qbeg - 1, -1, qbeg, Lr, tb, ts, rev, tlen, O, aw0,
                                        O.pen_clip5, slen * O.a, io, c);
                if (score == prev || io.max_off < (aw0 >> 1) + (aw0 >> 2)) break;
            }
            cells += c;
            if (io.gscore <= 0 || io.gscore <= score - O.pen_clip5) {
                qb = qbeg - io.qle, rb = rbeg - io.tle;
                truesc = score;
            } else {
                qb = 0, rb = rbeg - io.gtle;
                truesc = io.gscore;
            }
        } else {
            score = truesc = slen * O.a, qb = 0, rb = rbeg;
        }
        if (qbeg + slen != lq) {
            const int sc0 = score;
            const int qe0 = qbeg + slen;
            const int re0 = (int)(rbeg + slen - rmax0);
            const int tlen = (int)(rmax1 - rmax0 - re0);
            const long tb = rev ? (long)L - 1 - rbeg - slen : (long)rbeg + slen;
            const int ts = rev ? -1 : 1;
            unsigned long long c = 0;
            for (int i = 0; i < 2; ++i) {
                const int prev = score;
                aw1 = O.w << i;
                c = 0;
                score = ksw_extend_lane(eh, Q, qe0, 1, lq - qe0, Lr, tb, ts, rev, tlen, O, aw1,
                                        O.pen_clip3, sc0, io, c);
                if (score == prev || io.max_off < (aw1 >> 1) + (aw1 >> 2)) break;
            }
            cells += c;
            if (io.gscore <= 0 || io.gscore <= score - O.pen_clip3) {
                qe = qe0 + io.qle, re = (int)(rmax0 + re0 + io.tle);
                truesc += score - sc0;
            } else {
                qe = lq, re = (int)(rmax0 + re0 + io.gtle);
                truesc += io.gscore - sc0;
            }
        } else {
            qe = lq, re = rbeg + slen;
        }
        D.o_qb[t] = qb;
        D.o_qe[t] = qe;
        D.o_rb[t] = rb;
        D.o_re[t] = re;
        D.o_score[t] = score;
        D.o_truesc[t] = truesc;
        D.o_w[t] = aw0 > aw1 ? aw0 : aw1;
        D.o_pass[t] = (double)score >= O.min_score_per_base * (double)(qe - qb) ? 1 : 0;
    }
    // one atomic per wave for the cell counter
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if (lane == 0 && cells) atomicAdd(&D.cells[0], cells);
}

// ---------------------------------------------------------------------------
// global alignment: packed word = h (int16) | e (int16) << 16; query bases lane-major
constexpr int G_NEG = -30000;   // MINUS_INF stand-in: only ever compared against finite values
__device__ __forceinline__ uint32_t gpk(int h, int e) {
    return ((uint32_t)(uint16_t)(int16_t)h) | ((uint32_t)(uint16_t)(int16_t)e << 16);
}
__device__ __forceinline__ int gh(uint32_t w) { return (int)(int16_t)(w & 0xFFFFu); }
__device__ __forceinline__ int ge(uint32_t w) { return (int)(int16_t)(w >> 16); }

__device__ __forceinline__ int infer_bw(int l1, int l2, int score, int a, int q, int r) {
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    int w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    const int d = l1 > l2 ? l1 - l2 : l2 - l1;
    if (w < d) w = d;
    return w;
}

// ksw_global2 for one lane.  Direction bytes (h-source | e-bit<<2 | f-bit<<5,
// exactly ksw_global2's) are packed four per dword into the block's slab:
// dword index ((row * nc4 + col/4) * 64 + lane), byte col%4.  qv holds 8*q.
__device__ int ksw_global_lane(uint32_t *eh, const uint8_t *qv /* lane query (8*q), LDS */, int qlen,
                               const uint8_t *Lr, long tb, int ts, bool comp, int tlen,
                               const SwOptsDev &O, int w, uint32_t *zl /* slab + lane */, int nc4,
                               unsigned long long &cells) {
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    eh[0] = gpk(0, G_NEG);
    int j;
    for (j = 1; j <= qlen && j <= w; ++j) eh[j * SW_WAVE] = gpk(-(o_ins + e_ins * j), G_NEG);
    for (; j <= qlen; ++j) eh[j * SW_WAVE] = gpk(G_NEG, G_NEG);
    for (int i = 0; i < tlen; ++i) {
        int tc = (int)Lr[tb + (long)ts * i];
        if (comp && tc < 4) tc = 3 - tc;
        const uint64_t srow = score_row(tc, a, b);
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        int f = G_NEG;
        int h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : G_NEG;
        uint32_t *zi = zl + (long)i * nc4 * SW_WAVE;
        cells += (unsigned long long)(end > beg ? end - beg : 0);
        uint32_t wd = eh[beg * SW_WAVE];
        uint32_t qn = qv[beg];
        uint32_t dacc = 0;
        for (j = beg; j < end; ++j) {
            const uint32_t wn = eh[(j + 1) * SW_WAVE];   // prefetch (column j+1 is not written at j)
            const uint32_t qc = qn;
            qn = qv[j + 1];
            int m = gh(wd), e = ge(wd);
            m += (int)(int8_t)(uint8_t)(srow >> qc);
            uint32_t d = m >= e ? 0u : 1u;
            int h = m >= e ? m : e;
            d = h >= f ? d : 2u;
            h = h >= f ? h : f;
            const int t1 = m - oe_del;
            e -= e_del;
            d |= e > t1 ? 4u : 0u;
            e = e > t1 ? e : t1;
            const int t2 = m - oe_ins;
            f -= e_ins;
            d |= f > t2 ? 32u : 0u;
            f = f > t2 ? f : t2;
            eh[j * SW_WAVE] = gpk(h1, e);
            h1 = h;
            wd = wn;
            const int jj = j - beg;
            dacc |= d << ((jj & 3) << 3);
            if ((jj & 3) == 3 || j + 1 == end) {
                if (!(O.debug & 2)) zi[(long)(jj >> 2) * SW_WAVE] = dacc;
                dacc = 0;
            }
        }
        eh[end * SW_WAVE] = gpk(h1, G_NEG);
    }
    return gh(eh[qlen * SW_WAVE]);
}

__device__ __forceinline__ int push_op(uint32_t *cg, int n, int op, int len) {
    if (n > 0 && (int)(cg[n - 1] & 0xFu) == op) {
        cg[n - 1] += (uint32_t)len << 4;
        return n;
    }
    if (n >= SW_MAXCIG) return -1;
    cg[n] = ((uint32_t)len << 4) | (uint32_t)op;
    return n + 1;
}

__global__ void __launch_bounds__(SW_WAVE) sw_global_kernel(SwDev D, SwOptsDev O) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_g[];
    __shared__ int s_task;
    const int lane = threadIdx.x;
    const int qpad = (D.qmax + 8) & ~3;
    uint32_t *eh = lds_g + lane;
    uint8_t *qv = reinterpret_cast<uint8_t *>(lds_g + (D.qmax + 1) * SW_WAVE) + lane * qpad;
    const int nc4 = (D.qmax + 3) >> 2;
    uint32_t *zl = reinterpret_cast<uint32_t *>(D.z + (int64_t)blockIdx.x * D.z_slab) + lane;
    unsigned long long cells = 0;
    for (;;) {
        if (lane == 0) s_task = atomicAdd(D.work, 1);
        __syncthreads();
        const int64_t t0 = (int64_t)s_task * SW_WAVE;
        __syncthreads();
        if (t0 >= D.n_task) break;
        const int64_t slot = t0 + lane;
        if (slot < D.n_task) {
            const int64_t t = D.perm[slot];
            const int sid = D.t_sr[t], lid = D.t_lr[t];
            const uint8_t *Q = D.sr + D.sr_off[sid];
            const int lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
            const uint8_t *Lr = D.lr + D.lr_off[lid];
            const int L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
            const bool rev = D.t_strand[t] != 0;
            const int qb = D.o_qb[t], qe = D.o_qe[t], rb = D.o_rb[t], re = D.o_re[t];
            const int truesc = D.o_truesc[t];
            const int lqq = qe - qb, rlen = re - rb;
            // query (reversed for the reverse strand: indels leftmost on the forward strand)
            for (int j = 0; j < lqq; ++j) qv[j] = (uint8_t)((rev ? Q[qe - 1 - j] : Q[qb + j]) << 3);
            qv[lqq] = 0;
            // reference rows: forward strand rb.., reverse strand comp(L[L-re+i])
            const long tb = rev ? (long)L - re : (long)rb;
            int tmpw = infer_bw(lqq, rlen, truesc, O.a, O.o_del, O.e_del);
            int w2 = infer_bw(lqq, rlen, truesc, O.a, O.o_ins, O.e_ins);
            w2 = w2 > tmpw ? w2 : tmpw;
            const int wreg = D.o_w[t];
            if (w2 > O.w) w2 = w2 < wreg ? w2 : wreg;
            int last_sc = -(1 << 30), gsc = 0, iter = 0, ww = 0;
            bool nogap = false;
            uint32_t *cg = D.o_cig + t * SW_MAXCIG;
            int status = 0;
            unsigned long long cpass = 0;
            do {
                w2 = w2 < O.w << 2 ? w2 : O.w << 2;
                if (lqq <= 0 || rlen <= 0) { gsc = 0; ww = -1; break; }
                if (lqq == rlen && w2 == 0) {
                    nogap = true;
                    gsc = 0;
                    for (int i = 0; i < lqq; ++i) {
                        int tc = (int)Lr[tb + i];
                        if (rev && tc < 4) tc = 3 - tc;
                        gsc += sw_score(tc, (int)(qv[i] >> 3), O.a, O.b);
                    }
                    ww = 0;
                } else {
                    nogap = false;
                    const int mn = lqq < rlen ? lqq : rlen;
                    const int max_ins = (int)((double)(mn * O.a - O.o_ins) / O.e_ins + 1.);
                    const int max_del = (int)((double)(mn * O.a - O.o_del) / O.e_del + 1.);
                    int max_gap = max_ins > max_del ? max_ins : max_del;
                    max_gap = max_gap > 1 ? max_gap : 1;
                    const int dl = rlen > lqq ? rlen - lqq : lqq - rlen;
                    ww = (max_gap + dl + 1) >> 1;
                    ww = ww < w2 ? ww : w2;
                    const int min_w = dl + 3;
                    ww = ww > min_w ? ww : min_w;
                    cpass = 0;
                    gsc = ksw_global_lane(eh, qv, lqq, Lr, tb, 1, rev, rlen, O, ww, zl, nc4, cpass);
                }
                if (gsc == last_sc || w2 == O.w << 2) break;
                last_sc = gsc;
                w2 <<= 1;
            } while (++iter < 3 && gsc < truesc - O.a);
            cells += cpass;
            // backtrack (ksw_global2) into ops in reverse order
            int n = 0;
            if (ww < 0) {
                n = 0;
            } else if (nogap || (O.debug & 1)) {
                cg[0] = ((uint32_t)lqq << 4);
                n = 1;
            } else {
                int i = rlen - 1, k = (i + ww + 1 < lqq ? i + ww + 1 : lqq) - 1, which = 0;
                while (i >= 0 && k >= 0 && n >= 0) {
                    const int jj = k - (i > ww ? i - ww : 0);
                    const uint32_t zw = zl[((long)i * nc4 + (jj >> 2)) * SW_WAVE];
                    which = ((zw >> ((jj & 3) << 3)) >> (which << 1)) & 3;
                    if (which == 0) n = push_op(cg, n, 0, 1), --i, --k;
                    else if (which == 1) n = push_op(cg, n, 2, 1), --i;
                    else n = push_op(cg, n, 1, 1), --k;
                }
                if (n >= 0 && i >= 0) n = push_op(cg, n, 2, i + 1);
                if (n >= 0 && k >= 0) n = push_op(cg, n, 1, k + 1);
                if (n < 0) { status = -9; n = 0; }
                for (int x = 0; x < n >> 1; ++x) {
                    const uint32_t tmp = cg[x];
                    cg[x] = cg[n - 1 - x];
                    cg[n - 1 - x] = tmp;
                }
            }
            // mem_reg2aln: position, D squeeze, clipping
            int pos = rev ? L - re : rb;
            if (n > 0) {
                if ((cg[0] & 0xFu) == 2u) {
                    pos += (int)(cg[0] >> 4);
                    for (int x = 0; x + 1 < n; ++x) cg[x] = cg[x + 1];
                    --n;
                } else if ((cg[n - 1] & 0xFu) == 2u) {
                    --n;
                }
            }
            if (qb != 0 || qe != lq) {
                const int clip5 = rev ? lq - qe : qb;
                const int clip3 = rev ? qb : lq - qe;
                if (n + (clip5 ? 1 : 0) + (clip3 ? 1 : 0) > SW_MAXCIG) {
                    status = -9;
                } else {
                    if (clip5) {
                        for (int x = n; x > 0; --x) cg[x] = cg[x - 1];
                        cg[0] = ((uint32_t)clip5 << 4) | 4u;
                        ++n;
                    }
                    if (clip3) cg[n++] = ((uint32_t)clip3 << 4) | 4u;
                }
            }
            D.o_gscore[t] = gsc;
            D.o_pos[t] = pos;
            D.o_ncig[t] = n;
            D.o_status[t] = status;
        }
    }
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if (lane == 0 && cells) atomicAdd(&D.cells[1], cells);
}

// ---------------------------------------------------------------------------
// Task ordering: lanes of a wave run in lock-step, so tasks are bucketed by
// (left extension length = qbeg, right extension length / 8) before the DP
// kernels (counting sort; the order inside a bucket does not affect results).
__device__ __forceinline__ int sw_task_key(const SwDev &D, int64_t t) {
    const int sid = D.t_sr[t];
    const int lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
    const int qbeg = D.t_qbeg[t];
    int right = (lq - qbeg - D.t_slen[t]) >> 3;
    right = right < 31 ? right : 31;
    const int left = qbeg < 1023 ? qbeg : 1023;
    return (left << 5) | right;
}
__global__ void sw_order_count(SwDev D) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < D.n_task; t += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&D.bucket[sw_task_key(D, t)], 1);
}
__global__ void __launch_bounds__(1024) sw_order_scan(int32_t *b) {
    __shared__ int part[1024];
    const int tid = threadIdx.x, per = SW_NBUCKET / 1024;
    int s = 0;
    for (int k = 0; k < per; ++k) s += b[tid * per + k];
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int base = part[tid] - s;
    for (int k = 0; k < per; ++k) {
        const int c = b[tid * per + k];
        b[tid * per + k] = base;
        base += c;
    }
}
__global__ void sw_order_scatter(SwDev D) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < D.n_task; t += (int64_t)gridDim.x * blockDim.x)
        D.perm[atomicAdd(&D.bucket[sw_task_key(D, t)], 1)] = (int32_t)t;
}

int sw_launch_order(const SwDev &D, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(D.bucket, 0, (SW_NBUCKET + 1) * sizeof(int32_t), s);
    if (e != hipSuccess) return (int)e;
    int grid = (int)((D.n_task + 255) / 256);
    grid = grid < 4096 ? (grid > 0 ? grid : 1) : 4096;
    hipLaunchKernelGGL(sw_order_count, dim3(grid), dim3(256), 0, s, D);
    hipLaunchKernelGGL(sw_order_scan, dim3(1), dim3(1024), 0, s, D.bucket);
    hipLaunchKernelGGL(sw_order_scatter, dim3(grid), dim3(256), 0, s, D);
    return (int)hipGetLastError();
}

int sw_launch_extend(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream) {
    hipError_t e = hipFuncSetAttribute((const void *)sw_extend_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(sw_extend_kernel, dim3(grid), dim3(SW_WAVE), lds, (hipStream_t)stream, D, O);
    return (int)hipGetLastError();
}
int sw_launch_global(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream) {
    hipError_t e = hipFuncSetAttribute((const void *)sw_global_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(sw_global_kernel, dim3(grid), dim3(SW_WAVE), lds, (hipStream_t)stream, D, O);
    return (int)hipGetLastError();
}

}  // namespace prgpu
