// Seed extension + CIGAR kernels for gfx950 — the ksw stage of bwa-proovread mem
// (bin/proovread:1313) as a batched inter-task SW: one (short read, long-read
// window, seed) task per lane, rows of the banded DP walked in lock-step by the
// 64 lanes of a wave.
//
//   sw_ext_phase_kernel<WB> : mem_chain2aln for a single-seed chain — left and
//                      right ksw_extend2 (band pruning, z-drop, to-end gscore),
//                      the DP row in registers; MAX_BAND_TRY=2 band doubling as
//                      separate compacted phases; sw_*_finish: the -L clip decision.
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
#include "sw_ring.h"
#include "sw_pk.h"

namespace prgpu {

__device__ __forceinline__ int sw_score(int t, int q, int a, int b) {
    // bwa_fill_scmat: match a, mismatch -b, anything with N (4) -1
    return (t > 3 || q > 3) ? -1 : (t == q ? a : -b);
}

// bwa_gen_cigar2's gap-free score (query length == reference length, no DP): the scores of query
// base qbase + qstep * i against reference row i (complemented on the reverse strand), 16 rows a
// step from two 16-byte windows -- the query read forward from its first base, the reference
// forward or, on the reverse strand, backwards from its last row (pk_tref16; the pools' 64 bytes
// of slack on both sides cover the windows' overhang) -- instead of two byte loads per row (the
// finish task's near-exact alignments are nearly all gap-free: ~16 ms of its CIGAR pass)
__device__ int nogap_score(const uint8_t *Q, int qbase, int qstep, const uint8_t *Lr, long tb, bool rev, int n,
                           const SwOptsDev &O) {
    const int q0 = qstep > 0 ? qbase : qbase - n + 1;   // the query's first base
    // pair u: query q0 + u with row i = (qstep > 0 ? u : n - 1 - u)
    const uint8_t *T = qstep > 0 ? Lr + tb : Lr + tb + n - 1;
    const int ts = qstep > 0 ? 1 : -1;
    int sc = 0;
    for (int u0 = 0; u0 < n; u0 += 16) {
        uint32_t qw[4], tw[4];
        __builtin_memcpy(qw, Q + q0 + u0, 16);
        pk_tref16(T, ts, u0, tw);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (u0 + k >= n) break;
            int tc = (int)((tw[k >> 2] >> (8 * (k & 3))) & 0xFFu);
            if (rev && tc < 4) tc = 3 - tc;
            const int qc = (int)((qw[k >> 2] >> (8 * (k & 3))) & 0xFFu);
            sc += sw_score(tc, qc, O.a, O.b);
        }
    }
    return sc;
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

// canonical unpruned band cells of one ksw_extend2 call
__device__ __forceinline__ unsigned long long band_cells(int tlen, int qlen, int w) {
    unsigned long long c = 0;
    for (int i = 0; i < tlen; ++i) {
        const int lo = i - w > 0 ? i - w : 0;
        const int hi = i + w + 1 < qlen ? i + w + 1 : qlen;
        if (hi > lo) c += (unsigned long long)(hi - lo);
    }
    return c;
}

__device__ __forceinline__ int cal_max_gap(const SwOptsDev &O, int qlen) {
    int l_del = (int)((double)(qlen * O.a - O.o_del) / O.e_del + 1.);
    int l_ins = (int)((double)(qlen * O.a - O.o_ins) / O.e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < O.w << 1 ? l : O.w << 1;
}

// mem_chain2aln geometry of a single-seed task
struct TaskGeo {
    const uint8_t *Q, *Lr;
    int lq, L, qbeg, rbeg, slen;
    bool rev;
    long rmax0, rmax1;
};
__device__ __forceinline__ TaskGeo task_geo(const SwDev &D, const SwOptsDev &O, int64_t t) {
    TaskGeo g;
    const int sid = D.t_sr[t], lid = D.t_lr[t];
    g.Q = D.sr + D.sr_off[sid];
    g.lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
    g.Lr = D.lr + D.lr_off[lid];
    g.L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
    g.rev = D.t_strand[t] != 0;
    g.qbeg = D.t_qbeg[t];
    g.rbeg = D.t_rbeg[t];
    g.slen = D.t_slen[t];
    g.rmax0 = (long)g.rbeg - (g.qbeg + cal_max_gap(O, g.qbeg));
    g.rmax1 = (long)g.rbeg + g.slen + ((g.lq - g.qbeg - g.slen) + cal_max_gap(O, g.lq - g.qbeg - g.slen));
    if (g.rmax0 < 0) g.rmax0 = 0;
    if (g.rmax1 > g.L) g.rmax1 = g.L;
    return g;
}

// packed extension key (mode 1 = left, 2 = right side, first band try): the side's
// query length, for tasks whose scores fit the kernel's int16 frame; -1 otherwise
__device__ __forceinline__ int pk_ext_key(const SwDev &D, const SwOptsDev &O, int64_t t, int side) {
    if (!O.pk || O.w > 40 || !sel_ext(D, t)) return -1;
    const int sid = D.t_sr[t];
    const int lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
    const int ql = side == 0 ? D.t_qbeg[t] : lq - D.t_qbeg[t] - D.t_slen[t];
    if (ql <= 0 || ql > PK_QMAX || O.a * lq > 2047) return -1;
    return ql;
}
// per-task extension scratch: field f of side s at x[(s * XF + f) * n_task + t]
enum { XF_SCORE, XF_QLE, XF_TLE, XF_GTLE, XF_GSCORE, XF_MAXOFF, XF };
__device__ __forceinline__ int32_t &xref(const SwDev &D, int side, int f, int64_t t) {
    return D.x[((int64_t)(side * XF + f)) * D.n_task + t];
}

// One extension phase: side 0 = left (query reversed from qbeg-1), 1 = right;
// band try `tryi` (w = O.w << tryi, mem_chain2aln's MAX_BAND_TRY loop).  Lanes
// take tasks from the phase's list (bucketed by query length).
template <int WB>
__global__ void __launch_bounds__(SW_WAVE) sw_ext_phase_kernel(SwDev D, SwOptsDev O, int side, int tryi) {
    const int lane = threadIdx.x;
    const int n = D.list_n[0];
    for (int64_t c0 = (int64_t)blockIdx.x * SW_WAVE; c0 < n; c0 += (int64_t)gridDim.x * SW_WAVE) {
        const int64_t slot = c0 + lane;
        int64_t t = -1;
        TaskGeo g;
        const uint8_t *Q = D.sr;
        const uint8_t *Lr = D.lr;
        int qb = 0, qs = 1, qlen = 0, tlen = 0, ts = 1, end_bonus = 0, h0 = 0;
        long tb = 0;
        bool comp = false;
        if (slot < n) {
            t = D.list[slot];
            g = task_geo(D, O, t);
            Q = g.Q;
            Lr = g.Lr;
            comp = g.rev;
            if (side == 0) {
                qb = g.qbeg - 1; qs = -1; qlen = g.qbeg;
                tlen = (int)(g.rbeg - g.rmax0);
                tb = g.rev ? (long)g.L - g.rbeg : (long)g.rbeg - 1;
                ts = g.rev ? 1 : -1;
                end_bonus = O.pen_clip5;
                h0 = g.slen * O.a;
            } else {
                const int qe0 = g.qbeg + g.slen;
                const int re0 = (int)(g.rbeg + g.slen - g.rmax0);
                qb = qe0; qs = 1; qlen = g.lq - qe0;
                tlen = (int)(g.rmax1 - g.rmax0 - re0);
                tb = g.rev ? (long)g.L - 1 - g.rbeg - g.slen : (long)g.rbeg + g.slen;
                ts = g.rev ? -1 : 1;
                end_bonus = O.pen_clip3;
                h0 = D.o_score[t];   // left result (sc0)
            }
        }
        ExtIO io;
        const int aw = O.w << tryi;
        const int score = ext_ring<WB>(Q, qb, qs, qlen, Lr, tb, ts, comp, tlen, O, aw, end_bonus, h0, io);
        if (t >= 0) {
            xref(D, side, XF_SCORE, t) = score;
            xref(D, side, XF_QLE, t) = io.qle;
            xref(D, side, XF_TLE, t) = io.tle;
            xref(D, side, XF_GTLE, t) = io.gtle;
            xref(D, side, XF_GSCORE, t) = io.gscore;
            xref(D, side, XF_MAXOFF, t) = io.max_off;
            if (tryi == 0) {
                const int prev = side == 0 ? -1 : h0;
                const bool stop = score == prev || io.max_off < (aw >> 1) + (aw >> 2);
                D.x_try[t] = (uint8_t)(D.x_try[t] | (stop ? 0 : (1 << side)));
            }
        }
    }
}

// ksw_extend2 (oracle/sw_oracle.c osw_extend) for ONE task per wave: the row's band
// [beg, end) -- at most XW_COLS * 64 columns, 2w+1 <= 192 -- spread over the lanes (column
// beg + lane + 64 r), the DP row eh in the wave's LDS area (h | e << 16 per column, as
// ext_row_lane).  ksw's horizontal recurrence f(j+1) = max(f(j) - e_ins, max(M(j) - oe_ins, 0))
// with f(beg) = 0 is F(j) = max_{beg <= k < j} (t(k) + k e_ins) - (j - 1) e_ins (t >= 0 makes the
// f(beg) term lose), an exclusive prefix max over the band; H(i, j-1) for eh[j].h is the left
// neighbour's h; the row maximum (last column on ties), the band pruning (first / last
// non-zero eh) and the z-drop are wave reductions / ballots.  The w = 80 band retries ran one
// task per LANE (sw_ext_phase_kernel<80>): ~300 rows x 161 cells in one dependent chain per
// lane, ~1.5 ms per launch whatever the number of retried tasks.
constexpr int XW_COLS = 3;

// one DPP step of a max scan: lanes without a source (outside the row / masked rows) keep INT_MIN
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_max_step(int v) {
    const int t = __builtin_amdgcn_update_dpp((int)INT32_MIN, v, CTRL, ROWS, 0xf, false);
    return t > v ? t : v;
}
// inclusive prefix max over the wave's lanes: row_shr 1, 2, 4, 8 scan the rows of 16, then
// row_bcast:15 carries rows 0 / 2 into 1 / 3 and row_bcast:31 the first half into the second
// (register-to-register DPP moves: no LDS round trip per step, unlike __shfl_up)
__device__ __forceinline__ int wave_scan_max_i32(int v) {
    v = dpp_max_step<0x111, 0xf>(v);
    v = dpp_max_step<0x112, 0xf>(v);
    v = dpp_max_step<0x114, 0xf>(v);
    v = dpp_max_step<0x118, 0xf>(v);
    v = dpp_max_step<0x142, 0xa>(v);
    v = dpp_max_step<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ int wave_max_i32(int v) { return __builtin_amdgcn_readlane(wave_scan_max_i32(v), 63); }
// lane l gets lane l - 1's value, lane 0 gets `first` (wave_shr:1)
__device__ __forceinline__ int wave_shr1(int v, int first) { return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false); }

__device__ int ext_wave(uint32_t *eh, uint8_t *qrow, const uint8_t *Q, int qb, int qs, int qlen, const uint8_t *Lr,
                        long tb, int ts, bool comp, int tlen, const SwOptsDev &O, int w, int end_bonus, int h0, int lane,
                        ExtIO &io) {
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    {   // row -1 (ksw's first row) and the band cap by the longest possible gap (max entry = a);
        // the query in extension order in the wave's LDS (one load per column per task, not per row)
        const int hj1 = h0 > oe_ins ? h0 - oe_ins : 0;
        for (int j = lane; j <= qlen + 1; j += 64) {
            int h = j == 0 ? h0 : (j <= qlen ? hj1 - e_ins * (j - 1) : 0);
            eh[j] = (uint32_t)(h > 0 ? h : 0);
            if (j < qlen) qrow[j] = Q[qb + qs * j];
        }
        int max_ins = (int)((double)(qlen * a + end_bonus - o_ins) / e_ins + 1.);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = (int)((double)(qlen * a + end_bonus - o_del) / e_del + 1.);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    __builtin_amdgcn_wave_barrier();
    int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    int tv = 0;   // target bases of rows i0 .. i0 + 63, one per lane (loaded every 64 rows)
    for (int i = 0; i < tlen; ++i) {
        if ((i & 63) == 0) {
            const int ii = i + lane;
            tv = ii < tlen ? (int)Lr[tb + (long)ts * ii] : 0;
            if (comp && tv < 4) tv = 3 - tv;
        }
        const int tc = __builtin_amdgcn_readlane(tv, i & 63);
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        int h1 = 0;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        }
        const int nr = end > beg ? (end - beg + 63) >> 6 : 0;   // lane blocks of the band (uniform)
        int M[XW_COLS], E[XW_COLS], H[XW_COLS];
        int carry = INT32_MIN;   // prefix max of A over the earlier blocks
        int key = 0;             // row maximum: h << 10 | (j - beg + 1), last column on ties
        int hprev_blk = h1;      // h of the column left of the block's lane 0 (h1 before the band)
        uint32_t nzb[XW_COLS];
#pragma unroll
        for (int r = 0; r < XW_COLS; ++r) {
            M[r] = E[r] = H[r] = 0;
            nzb[r] = 0u;
            if (r >= nr) continue;
            const int j = beg + lane + 64 * r;
            const bool in = j < end;
            int Mv = 0, e = 0, A = INT32_MIN;
            if (in) {
                const uint32_t p = eh[j];
                const int hp = (int)(p & 0xFFFFu);
                e = (int)(p >> 16);
                Mv = hp ? hp + sw_score(tc, (int)qrow[j], a, b) : 0;
                const int t = Mv - oe_ins > 0 ? Mv - oe_ins : 0;
                A = t + j * e_ins;
            }
            // F(j) = exclusive prefix max of A - (j - 1) e_ins, F(beg) = 0
            const int inc = wave_scan_max_i32(A);
            int exl = wave_shr1(inc, (int)INT32_MIN);
            exl = exl > carry ? exl : carry;
            const int top = __builtin_amdgcn_readlane(inc, 63);
            carry = top > carry ? top : carry;
            const int F = exl == INT32_MIN ? 0 : exl - (j - 1) * e_ins;
            int h = Mv > e ? Mv : e;
            h = h > F ? h : F;
            int tn = Mv - oe_del > 0 ? Mv - oe_del : 0;
            const int en = e - e_del > tn ? e - e_del : tn;
            M[r] = Mv;
            E[r] = in ? en : 0;
            H[r] = in ? h : 0;
            if (in) {
                const int kk = (h << 10) | (j - beg + 1);
                key = kk > key ? kk : key;
            }
        }
        // the new row: eh[j] = H(i, j-1) | E(i+1, j) << 16 for j in [beg, end), eh[end] = h1'
        int hlast = h1;   // H(i, end-1), or h1 when the band is empty
#pragma unroll
        for (int r = 0; r < XW_COLS; ++r) {
            if (r >= nr) continue;
            const int j = beg + lane + 64 * r;
            // lane 0: h1 before the band, else lane 63's h of the previous block
            const int left = wave_shr1(H[r], r == 0 ? h1 : __builtin_amdgcn_readlane(hprev_blk, 63));
            hprev_blk = H[r];
            if (j < end) {
                const uint32_t nw = (uint32_t)left | ((uint32_t)E[r] << 16);
                eh[j] = nw;
                nzb[r] = nw != 0u ? 1u : 0u;
            }
            const int jl = end - 1;   // the band's last column
            if (jl >= beg + 64 * r && jl < beg + 64 * (r + 1)) hlast = __builtin_amdgcn_readlane(H[r], jl - beg - 64 * r);
        }
        if (lane == 0) eh[end] = (uint32_t)hlast;   // e = 0
        __builtin_amdgcn_wave_barrier();
        const int jend = beg < end ? end : beg;
        if (jend == qlen) {
            max_ie = gscore > hlast ? max_ie : i;
            gscore = gscore > hlast ? gscore : hlast;
        }
        key = wave_max_i32(key);
        const int mm = key >> 10;
        if (mm == 0) break;
        const int mj = beg + (key & 1023) - 1;
        if (mm > max) {
            max = mm, max_i = i, max_j = mj;
            const int d = mj - i > 0 ? mj - i : i - mj;
            max_off = max_off > d ? max_off : d;
        } else if (O.zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - mm - ((i - max_i) - (mj - max_j)) * e_del > O.zdrop) break;
            } else {
                if (max - mm - ((mj - max_j) - (i - max_i)) * e_ins > O.zdrop) break;
            }
        }
        // band pruning: beg = first non-zero eh in [beg, end) (else end); end = last non-zero in
        // [beg', end] + 2 (capped), eh[end] = {hlast, 0} included
        int nb = end, ne = -1;
#pragma unroll
        for (int r = 0; r < XW_COLS; ++r) {
            if (r >= nr) continue;
            const uint64_t m = __ballot(nzb[r] != 0u);
            if (m) {
                const int f0 = beg + 64 * r + __builtin_ctzll(m);
                const int l0 = beg + 64 * r + 63 - __builtin_clzll(m);
                nb = nb < f0 ? nb : f0;
                ne = ne > l0 ? ne : l0;
            }
        }
        if (hlast != 0) ne = end;
        beg = nb;
        const int jj = ne >= beg ? ne : beg - 1;
        end = jj + 2 < qlen ? jj + 2 : qlen;
    }
    io.qle = max_j + 1;
    io.tle = max_i + 1;
    io.gtle = max_ie + 1;
    io.gscore = gscore;
    io.max_off = max_off;
    return max;
}

// One extension phase with one task per wave (ext_wave): the w = 80 band retries.  LDS: one
// DP row of qmax + 2 words per wave.
__global__ void __launch_bounds__(256) sw_ext_wave_kernel(SwDev D, SwOptsDev O, int side, int tryi) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_w[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const int per_wave = (D.qmax + 2) + (D.qmax + 3) / 4;   // DP row words + the query's bytes
    uint32_t *eh = lds_w + wv * per_wave;
    uint8_t *qrow = reinterpret_cast<uint8_t *>(eh + D.qmax + 2);
    const int n = D.list_n[0];
    for (int64_t k = (int64_t)blockIdx.x * nwv + wv; k < n; k += (int64_t)gridDim.x * nwv) {
        const int64_t t = D.list[k];
        const TaskGeo g = task_geo(D, O, t);
        int qb, qs, qlen, tlen, ts, end_bonus, h0;
        long tb;
        if (side == 0) {
            qb = g.qbeg - 1; qs = -1; qlen = g.qbeg;
            tlen = (int)(g.rbeg - g.rmax0);
            tb = g.rev ? (long)g.L - g.rbeg : (long)g.rbeg - 1;
            ts = g.rev ? 1 : -1;
            end_bonus = O.pen_clip5;
            h0 = g.slen * O.a;
        } else {
            const int qe0 = g.qbeg + g.slen;
            const int re0 = (int)(g.rbeg + g.slen - g.rmax0);
            qb = qe0; qs = 1; qlen = g.lq - qe0;
            tlen = (int)(g.rmax1 - g.rmax0 - re0);
            tb = g.rev ? (long)g.L - 1 - g.rbeg - g.slen : (long)g.rbeg + g.slen;
            ts = g.rev ? -1 : 1;
            end_bonus = O.pen_clip3;
            h0 = D.o_score[t];   // left result (sc0)
        }
        ExtIO io;
        const int aw = O.w << tryi;
        const int score = ext_wave(eh, qrow, g.Q, qb, qs, qlen, g.Lr, tb, ts, g.rev, tlen, O, aw, end_bonus, h0, lane, io);
        if (lane == 0) {
            xref(D, side, XF_SCORE, t) = score;
            xref(D, side, XF_QLE, t) = io.qle;
            xref(D, side, XF_TLE, t) = io.tle;
            xref(D, side, XF_GTLE, t) = io.gtle;
            xref(D, side, XF_GSCORE, t) = io.gscore;
            xref(D, side, XF_MAXOFF, t) = io.max_off;
            if (tryi == 0) {
                const int prev = side == 0 ? -1 : h0;
                const bool stop = score == prev || io.max_off < (aw >> 1) + (aw >> 2);
                D.x_try[t] = (uint8_t)(D.x_try[t] | (stop ? 0 : (1 << side)));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ksw_extend2 (oracle/sw_oracle.c osw_extend, upstream ksw.c) for one lane with the DP row
// in memory: eh[j * SW_WAVE] = H(i-1, j-1) | E(i, j) << 16 (both >= 0 and < 2^15 in an
// extension: a * query length + h0 <= 10000).  The band of any width; the wide-band
// extension kernel's core (bands beyond the register ring's 80 columns).
__device__ int ext_row_lane(uint32_t *eh, const uint8_t *Q, int qb, int qs, int qlen, const uint8_t *Lr, long tb,
                            int ts, bool comp, int tlen, const SwOptsDev &O, int w, int end_bonus, int h0, ExtIO &io) {
    const int a = O.a, b = O.b, o_del = O.o_del, e_del = O.e_del, o_ins = O.o_ins, e_ins = O.e_ins;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    io.qle = io.tle = io.gtle = 0;
    io.gscore = -1;
    io.max_off = 0;
    if (qlen <= 0 || tlen <= 0) {
        io.gscore = -1;
        return h0;
    }
    for (int j = 0; j <= qlen + 1; ++j) eh[j * SW_WAVE] = 0u;
    eh[0] = (uint32_t)h0;
    eh[SW_WAVE] = (uint32_t)(h0 > oe_ins ? h0 - oe_ins : 0);
    for (int j = 2; j <= qlen && (int)(eh[(j - 1) * SW_WAVE] & 0xFFFFu) > e_ins; ++j)
        eh[j * SW_WAVE] = (uint32_t)((int)(eh[(j - 1) * SW_WAVE] & 0xFFFFu) - e_ins);
    {   // cap the band by the longest possible gap (max matrix entry = a)
        int max_ins = (int)((double)(qlen * a + end_bonus - o_ins) / e_ins + 1.);
        max_ins = max_ins > 1 ? max_ins : 1;
        w = w < max_ins ? w : max_ins;
        int max_del = (int)((double)(qlen * a + end_bonus - o_del) / e_del + 1.);
        max_del = max_del > 1 ? max_del : 1;
        w = w < max_del ? w : max_del;
    }
    int max = h0, max_i = -1, max_j = -1, max_ie = -1, gscore = -1, max_off = 0;
    int beg = 0, end = qlen;
    for (int i = 0; i < tlen; ++i) {
        int tc = (int)Lr[tb + (long)ts * i];
        if (comp && tc < 4) tc = 3 - tc;
        int f = 0, h1, mm = 0, mj = -1;
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else {
            h1 = 0;
        }
        int j;
        for (j = beg; j < end; ++j) {
            const uint32_t p = eh[j * SW_WAVE];
            int M = (int)(p & 0xFFFFu), e = (int)(p >> 16);
            const int qc = (int)Q[qb + qs * j];
            M = M ? M + sw_score(tc, qc, a, b) : 0;
            int h = M > e ? M : e;
            h = h > f ? h : f;
            const int hp = h1;
            h1 = h;
            mj = mm > h ? mj : j;
            mm = mm > h ? mm : h;
            int t = M - oe_del;
            t = t > 0 ? t : 0;
            e -= e_del;
            e = e > t ? e : t;
            eh[j * SW_WAVE] = (uint32_t)hp | ((uint32_t)e << 16);
            t = M - oe_ins;
            t = t > 0 ? t : 0;
            f -= e_ins;
            f = f > t ? f : t;
        }
        eh[end * SW_WAVE] = (uint32_t)h1;   // h1, e = 0
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (mm == 0) break;
        if (mm > max) {
            max = mm, max_i = i, max_j = mj;
            const int d = mj - i > 0 ? mj - i : i - mj;
            max_off = max_off > d ? max_off : d;
        } else if (O.zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - mm - ((i - max_i) - (mj - max_j)) * e_del > O.zdrop) break;
            } else {
                if (max - mm - ((mj - max_j) - (i - max_i)) * e_ins > O.zdrop) break;
            }
        }
        for (j = beg; j < end && eh[j * SW_WAVE] == 0u; ++j) {}
        beg = j;
        for (j = end; j >= beg && eh[j * SW_WAVE] == 0u; --j) {}
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    io.qle = max_j + 1;
    io.tle = max_i + 1;
    io.gtle = max_ie + 1;
    io.gscore = gscore;
    io.max_off = max_off;
    return max;
}

// One extension phase for bands beyond the register ring (w > 80 at this try): the DP row
// per lane in LDS (queries <= LDSQ) or in a per-block HBM scratch; otherwise as
// sw_ext_phase_kernel.
template <bool HBM>
__global__ void __launch_bounds__(SW_WAVE) sw_ext_wide_kernel(SwDev D, SwOptsDev O, int side, int tryi) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_x[];
    const int lane = threadIdx.x;
    uint32_t *eh = (HBM ? D.eh_g + (int64_t)blockIdx.x * D.eh_g_stride : lds_x) + lane;
    const int n = D.list_n[0];
    for (int64_t c0 = (int64_t)blockIdx.x * SW_WAVE; c0 < n; c0 += (int64_t)gridDim.x * SW_WAVE) {
        const int64_t slot = c0 + lane;
        if (slot >= n) continue;
        const int64_t t = D.list[slot];
        const TaskGeo g = task_geo(D, O, t);
        int qb, qs, qlen, tlen, ts, end_bonus, h0;
        long tb;
        if (side == 0) {
            qb = g.qbeg - 1; qs = -1; qlen = g.qbeg;
            tlen = (int)(g.rbeg - g.rmax0);
            tb = g.rev ? (long)g.L - g.rbeg : (long)g.rbeg - 1;
            ts = g.rev ? 1 : -1;
            end_bonus = O.pen_clip5;
            h0 = g.slen * O.a;
        } else {
            const int qe0 = g.qbeg + g.slen;
            const int re0 = (int)(g.rbeg + g.slen - g.rmax0);
            qb = qe0; qs = 1; qlen = g.lq - qe0;
            tlen = (int)(g.rmax1 - g.rmax0 - re0);
            tb = g.rev ? (long)g.L - 1 - g.rbeg - g.slen : (long)g.rbeg + g.slen;
            ts = g.rev ? -1 : 1;
            end_bonus = O.pen_clip3;
            h0 = D.o_score[t];
        }
        ExtIO io;
        const int aw = O.w << tryi;
        const int score = ext_row_lane(eh, g.Q, qb, qs, qlen, g.Lr, tb, ts, g.rev, tlen, O, aw, end_bonus, h0, io);
        xref(D, side, XF_SCORE, t) = score;
        xref(D, side, XF_QLE, t) = io.qle;
        xref(D, side, XF_TLE, t) = io.tle;
        xref(D, side, XF_GTLE, t) = io.gtle;
        xref(D, side, XF_GSCORE, t) = io.gscore;
        xref(D, side, XF_MAXOFF, t) = io.max_off;
        if (tryi == 0) {
            const int prev = side == 0 ? -1 : h0;
            const bool stop = score == prev || io.max_off < (aw >> 1) + (aw >> 2);
            D.x_try[t] = (uint8_t)(D.x_try[t] | (stop ? 0 : (1 << side)));
        }
    }
}

__device__ __forceinline__ int band_w(const SwOptsDev &O, int w, int qlen, int end_bonus) {
    int max_ins = (int)((double)(qlen * O.a + end_bonus - O.o_ins) / O.e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    int max_del = (int)((double)(qlen * O.a + end_bonus - O.o_del) / O.e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    return w < max_del ? w : max_del;
}

// The next segment of a packed launch, longest first: segments sit in ascending key order (query
// length; band, then query length for the CIGAR pass), so the dequeue walks the list from its
// end, and the waves that finish early take the short segments (a static round robin left the
// longest segments for the last, partial round).  Counter `which` is zeroed by
// sw_launch_pk_order; -1 when the list is done.
__device__ __forceinline__ int pk_next_seg(const SwDev &D, int which, int nseg) {
    int s = 0;
    if (threadIdx.x == 0) s = atomicAdd(D.bucket + SW_NBUCKET + 8 + which, 1);
    s = __builtin_amdgcn_readfirstlane(s);
    return s < nseg ? nseg - 1 - s : -1;
}

// First band try of one extension side for two tasks per lane (sw_pk.h ext_pk):
// wave k takes the 128-task segment of one side query length (so qlen and the
// capped band are wave-uniform); lane l runs list[128k + l] and list[128k + 64 + l].
// Tasks that meet an N are flagged (x_try bit 3 + side) for sw_ext_phase_kernel.
template <int WB, bool SMALLH>
__global__ void __launch_bounds__(SW_WAVE, 2) sw_ext_pk_kernel(SwDev D, SwOptsDev O, int side) {
    __shared__ __attribute__((aligned(16))) uint32_t lm[2 * 2 * PK_NQW * SW_WAVE];
    const int lane = threadIdx.x;
    const int nseg = D.pk_bucket[PK_SCAN] / PK_SEG;
    const int end_bonus = side == 0 ? O.pen_clip5 : O.pen_clip3;
    for (;;) {
        const int seg = pk_next_seg(D, 0, nseg);
        if (seg < 0) break;
        const int64_t tt[2] = {D.list[(int64_t)seg * PK_SEG + lane], D.list[(int64_t)seg * PK_SEG + 64 + lane]};
        const int qlen = __builtin_amdgcn_readfirstlane(pk_ext_key(D, O, D.list[(int64_t)seg * PK_SEG], side));
        const int w = __builtin_amdgcn_readfirstlane(band_w(O, O.w, qlen, end_bonus));
        PkExtHalf H[2];
        int nrow = 0, nflag = 0;
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t t = tt[h];
            H[h] = PkExtHalf{D.lr, 1, false, 0, 0};
            const uint8_t *Q = D.sr;
            int qb = 0, qs = 1, ql = 0;
            if (t >= 0) {
                const TaskGeo g = task_geo(D, O, t);
                Q = g.Q;
                ql = qlen;
                if (side == 0) {
                    qb = g.qbeg - 1; qs = -1;
                    const long tb = g.rev ? (long)g.L - g.rbeg : (long)g.rbeg - 1;
                    H[h] = PkExtHalf{g.Lr + tb, g.rev ? 1 : -1, g.rev, (int)(g.rbeg - g.rmax0), g.slen * O.a};
                } else {
                    const int qe0 = g.qbeg + g.slen;
                    const int re0 = (int)(g.rbeg + g.slen - g.rmax0);
                    qb = qe0; qs = 1;
                    const long tb = g.rev ? (long)g.L - 1 - g.rbeg - g.slen : (long)g.rbeg + g.slen;
                    H[h] = PkExtHalf{g.Lr + tb, g.rev ? -1 : 1, g.rev, (int)(g.rmax1 - g.rmax0 - re0), D.o_score[t]};
                }
            }
            if (pk_build_mask(Q, qb, qs, ql, lm + (h * 2 * PK_NQW) * SW_WAVE + lane, SW_WAVE)) nflag |= 1 << h;
            nrow = nrow > H[h].tlen ? nrow : H[h].tlen;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const int v = __shfl_xor(nrow, o, 64);
            nrow = nrow > v ? nrow : v;
        }
        nrow = __builtin_amdgcn_readfirstlane(nrow);
        PkExtOut out[2];
        ext_pk<WB, SMALLH>(H[0], H[1], qlen, w, nrow, O, lm + lane, lm + 2 * PK_NQW * SW_WAVE + lane, SW_WAVE, out, nflag);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t t = tt[h];
            if (t < 0) continue;
            if ((nflag >> h) & 1) {
                D.x_try[t] = (uint8_t)(D.x_try[t] | (8 << side));
                continue;
            }
            xref(D, side, XF_SCORE, t) = out[h].score;
            xref(D, side, XF_QLE, t) = out[h].qle;
            xref(D, side, XF_TLE, t) = out[h].tle;
            xref(D, side, XF_GTLE, t) = out[h].gtle;
            xref(D, side, XF_GSCORE, t) = out[h].gscore;
            xref(D, side, XF_MAXOFF, t) = out[h].max_off;
            const int aw = O.w;
            const int prev = side == 0 ? -1 : H[h].h0;
            const bool stop = out[h].score == prev || out[h].max_off < (aw >> 1) + (aw >> 2);
            D.x_try[t] = (uint8_t)(D.x_try[t] | (stop ? 0 : (1 << side)));
        }
    }
}

// after the left phases: qb, rb, score, truesc (mem_chain2aln); o_w holds aw[0]
__global__ void sw_left_finish_kernel(SwDev D, SwOptsDev O) {
    unsigned long long cells = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < sel_count(D);
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = sel_task(D, k);
        if (!sel_ext(D, t)) continue;
        const TaskGeo g = task_geo(D, O, t);
        int score, truesc, qb, rb, aw0 = O.w;
        if (g.qbeg) {
            const int tr = (D.x_try[t] & 1) ? 1 : 0;
            aw0 = O.w << tr;
            score = xref(D, 0, XF_SCORE, t);
            const int gs = xref(D, 0, XF_GSCORE, t);
            if (gs <= 0 || gs <= score - O.pen_clip5) {
                qb = g.qbeg - xref(D, 0, XF_QLE, t), rb = g.rbeg - xref(D, 0, XF_TLE, t);
                truesc = score;
            } else {
                qb = 0, rb = g.rbeg - xref(D, 0, XF_GTLE, t);
                truesc = gs;
            }
            cells += band_cells((int)(g.rbeg - g.rmax0), g.qbeg, band_w(O, aw0, g.qbeg, O.pen_clip5));
        } else {
            score = truesc = g.slen * O.a, qb = 0, rb = g.rbeg;
        }
        D.o_qb[t] = qb;
        D.o_rb[t] = rb;
        D.o_score[t] = score;
        D.o_truesc[t] = truesc;
        D.o_w[t] = aw0;
    }
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if ((threadIdx.x & 63) == 0 && cells) atomicAdd(&D.cells[0], cells);
}

// after the right phases: qe, re, score, truesc, w, pass
__global__ void sw_right_finish_kernel(SwDev D, SwOptsDev O) {
    unsigned long long cells = 0;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < sel_count(D);
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = sel_task(D, k);
        if (!sel_ext(D, t)) continue;
        const TaskGeo g = task_geo(D, O, t);
        int score = D.o_score[t], truesc = D.o_truesc[t], qe, re, aw1 = O.w;
        const int qb = D.o_qb[t];
        if (g.qbeg + g.slen != g.lq) {
            const int sc0 = score;
            const int qe0 = g.qbeg + g.slen;
            const int re0 = (int)(g.rbeg + g.slen - g.rmax0);
            const int tr = (D.x_try[t] & 2) ? 1 : 0;
            aw1 = O.w << tr;
            score = xref(D, 1, XF_SCORE, t);
            const int gs = xref(D, 1, XF_GSCORE, t);
            if (gs <= 0 || gs <= score - O.pen_clip3) {
                qe = qe0 + xref(D, 1, XF_QLE, t), re = (int)(g.rmax0 + re0 + xref(D, 1, XF_TLE, t));
                truesc += score - sc0;
            } else {
                qe = g.lq, re = (int)(g.rmax0 + re0 + xref(D, 1, XF_GTLE, t));
                truesc += gs - sc0;
            }
            cells += band_cells((int)(g.rmax1 - g.rmax0 - re0), g.lq - qe0, band_w(O, aw1, g.lq - qe0, O.pen_clip3));
        } else {
            qe = g.lq, re = g.rbeg + g.slen;
        }
        const int aw0 = D.o_w[t];
        D.o_qe[t] = qe;
        D.o_re[t] = re;
        D.o_score[t] = score;
        D.o_truesc[t] = truesc;
        D.o_w[t] = aw0 > aw1 ? aw0 : aw1;
        D.o_pass[t] = (double)score >= O.min_score_per_base * (double)(qe - qb) ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if ((threadIdx.x & 63) == 0 && cells) atomicAdd(&D.cells[0], cells);
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

__device__ __forceinline__ int push_op(uint32_t *cg, int n, int op, int len, int cap) {
    if (n < 0) return n;
    if (n > 0 && (int)(cg[n - 1] & 0xFu) == op) {
        cg[n - 1] += (uint32_t)len << 4;
        return n;
    }
    if (n >= cap) return -1;
    cg[n] = ((uint32_t)len << 4) | (uint32_t)op;
    return n + 1;
}

// the task's CIGAR destination and capacity: its slot, or (overflow pass) its spill range
__device__ __forceinline__ uint32_t *cig_dest(const SwDev &D, int64_t t, int &cap) {
    if (D.rerun) {
        cap = cig_bound_ops(D.o_qe[t] - D.o_qb[t], D.o_re[t] - D.o_rb[t]);
        return D.o_cig + D.o_cig_at[t];
    }
    const int64_t a = D.cig_slot[t];
    cap = (int)(D.cig_slot[t + 1] - a);
    return D.o_cig + a;
}

// a CIGAR longer than its slot: the overflow pass recomputes the task into the spill area
__device__ __forceinline__ void cig_overflow(const SwDev &D, int64_t t) {
    if (D.rerun) {   // cannot happen: the spill range bounds every op sequence of the task
        D.o_status[t] = -9;
        D.o_ncig[t] = 0;
        return;
    }
    D.o_status[t] = SW_ST_OVERFLOW;
    D.x_try[t] = (uint8_t)(D.x_try[t] | 0x20);
    atomicAdd(&D.spill[0], 1ull);
    atomicAdd(&D.spill[1], (unsigned long long)cig_bound_ops(D.o_qe[t] - D.o_qb[t], D.o_re[t] - D.o_rb[t]));
}

// mem_reg2aln after ksw_global2: position, leading/trailing D squeeze, soft clips
// (n < 0: the backtrack outgrew cap)
__device__ __forceinline__ void glob_emit(const SwDev &D, int64_t t, uint32_t *cg, int n, int cap, int gsc,
                                          bool rev, int lq, int L, int qb, int qe, int rb, int re) {
    if (n < 0) {
        cig_overflow(D, t);
        return;
    }
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
        if (n + (clip5 ? 1 : 0) + (clip3 ? 1 : 0) > cap) {
            cig_overflow(D, t);
            return;
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
    D.o_status[t] = 0;
}

// band of one ksw_global2 pass (mem_reg2aln/bwa_gen_cigar2); -1: empty query or
// reference, 0 with nogap: equal lengths and w2 == 0 (no DP)
__device__ __forceinline__ int glob_pass_w(const SwOptsDev &O, int lqq, int rlen, int w2, bool &nogap) {
    nogap = false;
    if (lqq <= 0 || rlen <= 0) return -1;
    if (lqq == rlen && w2 == 0) { nogap = true; return 0; }
    const int mn = lqq < rlen ? lqq : rlen;
    const int max_ins = (int)((double)(mn * O.a - O.o_ins) / O.e_ins + 1.);
    const int max_del = (int)((double)(mn * O.a - O.o_del) / O.e_del + 1.);
    int max_gap = max_ins > max_del ? max_ins : max_del;
    max_gap = max_gap > 1 ? max_gap : 1;
    const int dl = rlen > lqq ? rlen - lqq : lqq - rlen;
    int ww = (max_gap + dl + 1) >> 1;
    ww = ww < w2 ? ww : w2;
    const int min_w = dl + 3;
    return ww > min_w ? ww : min_w;
}
// first-pass w2 of a task (after the extension)
__device__ __forceinline__ int glob_w2(const SwDev &D, const SwOptsDev &O, int64_t t, int lqq, int rlen) {
    const int truesc = D.o_truesc[t];
    int tmpw = infer_bw(lqq, rlen, truesc, O.a, O.o_del, O.e_del);
    int w2 = infer_bw(lqq, rlen, truesc, O.a, O.o_ins, O.e_ins);
    w2 = w2 > tmpw ? w2 : tmpw;
    const int wreg = D.o_w[t];
    if (w2 > O.w) w2 = w2 < wreg ? w2 : wreg;
    return w2 < O.w << 2 ? w2 : O.w << 2;
}
// band class of the first pass: 0 -> ring<40>, 1 -> ring<80>, 2 -> LDS kernel
__device__ __forceinline__ int glob_class(const SwDev &D, const SwOptsDev &O, int64_t t) {
    const int lqq = D.o_qe[t] - D.o_qb[t], rlen = D.o_re[t] - D.o_rb[t];
    bool nogap;
    const int ww = glob_pass_w(O, lqq, rlen, glob_w2(D, O, t, lqq, rlen), nogap);
    return ww <= 40 ? 0 : (ww <= 80 ? 1 : 2);
}
// packed-kernel key (band * 256 + query length) of a task whose first pass runs a
// DP with band <= 40 inside the kernel's int16 frame; -1 otherwise
__device__ __forceinline__ int pk_key(const SwDev &D, const SwOptsDev &O, int64_t t) {
    if (!O.pk || !sel_cig(D, t)) return -1;
    const int lqq = D.o_qe[t] - D.o_qb[t], rlen = D.o_re[t] - D.o_rb[t];
    if (lqq > PK_QMAX || rlen > PK_TMAX) return -1;
    bool nogap;
    const int ww = glob_pass_w(O, lqq, rlen, glob_w2(D, O, t, lqq, rlen), nogap);
    if (ww <= 0 || nogap || ww > 40) return -1;
    return ww * 256 + lqq;
}

// The general CIGAR pass (any band, N bases, the whole bwa_gen_cigar2 loop).  HBM = true:
// the DP row and query live in a per-block HBM scratch instead of LDS (queries too long for
// the 160 KB LDS; same [column][lane] layout, coalesced).
template <bool HBM>
__global__ void __launch_bounds__(SW_WAVE) sw_global_kernel(SwDev D, SwOptsDev O) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_g[];
    __shared__ int s_task;
    const int lane = threadIdx.x;
    const int qpad = (D.qmax + 8) & ~3;
    uint32_t *base = HBM ? D.eh_g + (int64_t)blockIdx.x * D.eh_g_stride : lds_g;
    uint32_t *eh = base + lane;
    uint8_t *qv = reinterpret_cast<uint8_t *>(base + (D.qmax + 1) * SW_WAVE) + lane * qpad;
    const int nc4 = (D.qmax + 3) >> 2;
    uint32_t *zl = reinterpret_cast<uint32_t *>(D.z + (int64_t)blockIdx.x * D.z_slab) + lane;
    unsigned long long cells = 0;
    for (;;) {
        if (lane == 0) s_task = atomicAdd(D.work, 1);
        __syncthreads();
        const int64_t t0 = (int64_t)s_task * SW_WAVE;
        __syncthreads();
        const int nl = D.list_n[0];
        if (t0 >= nl) break;
        const int64_t slot = t0 + lane;
        if (slot < nl) {
            const int64_t t = D.list[slot];
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
            int cap = 0;
            uint32_t *cg = cig_dest(D, t, cap);
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
                    if (which == 0) n = push_op(cg, n, 0, 1, cap), --i, --k;
                    else if (which == 1) n = push_op(cg, n, 2, 1, cap), --i;
                    else n = push_op(cg, n, 1, 1, cap), --k;
                }
                if (i >= 0) n = push_op(cg, n, 2, i + 1, cap);
                if (k >= 0) n = push_op(cg, n, 1, k + 1, cap);
                for (int x = 0; x < n >> 1; ++x) {
                    const uint32_t tmp = cg[x];
                    cg[x] = cg[n - 1 - x];
                    cg[n - 1 - x] = tmp;
                }
            }
            glob_emit(D, t, cg, n, cap, gsc, rev, lq, L, qb, qe, rb, re);
        }
    }
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if (lane == 0 && cells) atomicAdd(&D.cells[1], cells);
}


// ksw_global2 pass 1 with the DP row in registers (band class WB); a task whose
// loop would run a second pass is left to the LDS kernel (x_try bit 2).
template <int WB>
__global__ void __launch_bounds__(SW_WAVE) sw_global_ring_kernel(SwDev D, SwOptsDev O) {
    constexpr int NW = (2 * WB + 2 + 7) / 8;
    const int lane = threadIdx.x;
    uint32_t *zl = reinterpret_cast<uint32_t *>(D.z) + (int64_t)blockIdx.x * D.z_ring_slab + lane;
    unsigned long long cells = 0;
    const int n = D.list_n[0];
    for (int64_t c0 = (int64_t)blockIdx.x * SW_WAVE; c0 < n; c0 += (int64_t)gridDim.x * SW_WAVE) {
        const int64_t slot = c0 + lane;
        int64_t t = -1;
        const uint8_t *Q = D.sr, *Lr = D.lr;
        int lq = 0, L = 0, qb = 0, qe = 0, rb = 0, re = 0, lqq = 0, rlen = 0, w2 = 0, ww = -1, truesc = 0;
        bool rev = false, nogap = false;
        long tb = 0;
        if (slot < n) {
            t = D.list[slot];
            const int sid = D.t_sr[t], lid = D.t_lr[t];
            Q = D.sr + D.sr_off[sid];
            lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
            Lr = D.lr + D.lr_off[lid];
            L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
            rev = D.t_strand[t] != 0;
            qb = D.o_qb[t], qe = D.o_qe[t], rb = D.o_rb[t], re = D.o_re[t];
            truesc = D.o_truesc[t];
            lqq = qe - qb, rlen = re - rb;
            tb = rev ? (long)L - re : (long)rb;
            w2 = glob_w2(D, O, t, lqq, rlen);
            ww = glob_pass_w(O, lqq, rlen, w2, nogap);
        }
        const bool dp = t >= 0 && ww > 0 && !nogap;
        // query reversed on the reverse strand (indels leftmost on the forward strand)
        const int qbase = rev ? qe - 1 : qb, qstep = rev ? -1 : 1;
        int gsc = glob_ring<WB>(Q, qbase, qstep, dp ? lqq : 0, Lr, tb, 1, rev, dp ? rlen : 0, O, dp ? ww : 0, zl, SW_WAVE);
        if (t < 0) continue;
        if (ww < 0) gsc = 0;
        if (nogap) gsc = nogap_score(Q, qbase, qstep, Lr, tb, rev, lqq, O);
        // bwa_gen_cigar2's loop after pass 1: stop when w2 hit its cap or the score is close
        // enough; otherwise the LDS kernel reruns the whole loop for this task
        if (dp && w2 != O.w << 2 && gsc < truesc - O.a) {
            D.x_try[t] = (uint8_t)(D.x_try[t] | 4);
            continue;
        }
        int cap = 0;
        uint32_t *cg = cig_dest(D, t, cap);
        int nc = 0;
        if (ww < 0) {
            nc = 0;
        } else if (!dp || (O.debug & 1)) {
            cg[0] = ((uint32_t)lqq << 4);
            nc = 1;
        } else {
            cells += band_cells(rlen, lqq, ww);
            nc = glob_backtrack<WB>(zl, SW_WAVE, rlen, lqq, ww, cg, cap);
            for (int x = 0; x < nc >> 1; ++x) {
                const uint32_t tmp = cg[x];
                cg[x] = cg[nc - 1 - x];
                cg[nc - 1 - x] = tmp;
            }
        }
        glob_emit(D, t, cg, nc, cap, gsc, rev, lq, L, qb, qe, rb, re);
    }
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if (lane == 0 && cells) {
        atomicAdd(&D.cells[1], cells);
        if (WB == 40 && !O.pk) atomicAdd(&D.cells[2], cells);   // the dominant launch's own cells (bench roofline)
    }
}

// ---------------------------------------------------------------------------
// ksw_global2 pass 1 for two tasks per lane (sw_pk.h).  Wave k takes the 128-task
// segment list[128k, 128k + 128) of one (band, query length) key: lane l runs
// tasks list[128k + l] (low halves) and list[128k + 64 + l] (high halves).
// Tasks that meet an N, or whose loop would run a second pass, are left to the
// LDS kernel (x_try bit 2).
//
// split = 0 (the default): the fused kernel, one slab per resident wave, the walk right after
// the DP.  split = 1 (PRGPU_PK_SPLIT, sw_api.cpp pk_prepare): two kernels per chunk of
// segments [seg0, seg1): the DP writes every segment's direction words into its own slab of
// the chunk's slab array and the scores; the backtrack + emit (sw_global_pk_bt_kernel, fewer
// registers, more waves per SIMD) reads them back.  Measured equal in total.

// mem_reg2aln after ksw_global2 (glob_emit's rules) on the forward-ordered ops at the end of
// the task's slots: position, leading/trailing D squeeze, soft clips
__device__ __forceinline__ void pk_emit(const SwDev &D, int64_t t, uint32_t *cg, int cap, int nc, uint32_t fst,
                                        uint32_t lst, int gsc, bool rev) {
    const int sid = D.t_sr[t], lid = D.t_lr[t];
    const int lq = (int)(D.sr_off[sid + 1] - D.sr_off[sid]);
    const int L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
    const int qb = D.o_qb[t], qe = D.o_qe[t], rb = D.o_rb[t], re = D.o_re[t];
    int m = nc, src = cap - nc;
    int pos = rev ? L - re : rb;
    if (m < 0) {
        cig_overflow(D, t);
        return;
    }
    if (m > 0) {
        if ((fst & 0xFu) == 2u) {
            pos += (int)(fst >> 4);
            ++src, --m;
        } else if ((lst & 0xFu) == 2u) {
            --m;
        }
    }
    int clip5 = 0, clip3 = 0;
    if (qb != 0 || qe != lq) {
        clip5 = rev ? lq - qe : qb;
        clip3 = rev ? qb : lq - qe;
        if (m + (clip5 ? 1 : 0) + (clip3 ? 1 : 0) > cap) {
            cig_overflow(D, t);
            return;
        }
    }
    const int d0 = clip5 ? 1 : 0;
    pk_cig_move(cg, d0, src, m);
    if (clip5) cg[0] = ((uint32_t)clip5 << 4) | 4u;
    if (clip3) cg[d0 + m] = ((uint32_t)clip3 << 4) | 4u;
    D.o_gscore[t] = gsc;
    D.o_pos[t] = pos;
    D.o_ncig[t] = d0 + m + (clip3 ? 1 : 0);
    D.o_status[t] = 0;
}

template <int WB, int BTW>
__global__ void __launch_bounds__(SW_WAVE, 2) sw_global_pk_kernel(SwDev D, SwOptsDev O, int seg0, int seg1, int split) {
    // query masks ([half][bit][word][lane])
    __shared__ __attribute__((aligned(16))) uint32_t lsh[2 * 2 * PK_NQW * SW_WAVE];
    const int lane = threadIdx.x;
    uint32_t *lm = lsh;
    unsigned long long cells = 0;
    const int nseg_all = D.pk_bucket[PK_SCAN] / PK_SEG;
    const int nseg = seg1 < nseg_all ? seg1 : nseg_all;
    unsigned long long ph[4] = {0, 0, 0, 0};   // wave cycles: masks, DP, backtrack, emit
    for (int it = 0;; ++it) {   // fused: longest segments first from the dequeue; split: the chunk's round robin
        int seg;
        if (split) {
            seg = seg0 + blockIdx.x + it * gridDim.x;
            if (seg >= nseg) break;
        } else {
            seg = pk_next_seg(D, 1, nseg);
            if (seg < 0) break;
        }
        // split: the segment's slab in the chunk's array; fused: this wave's own slab
        PkDir *zl = reinterpret_cast<PkDir *>(D.z) + (int64_t)(split ? seg - seg0 : blockIdx.x) * D.z_pk_slab + lane;
        unsigned long long c0 = clock64();
        const int64_t tt[2] = {D.list[(int64_t)seg * PK_SEG + lane], D.list[(int64_t)seg * PK_SEG + 64 + lane]};
        // the segment's key (its first task is never padding)
        const int key = __builtin_amdgcn_readfirstlane(pk_key(D, O, D.list[(int64_t)seg * PK_SEG]));
        const int ww = key >> 8, lqq = key & 255;
        PkHalf H[2];
        int nrow = 0, qn = 0;
        __syncthreads();   // the previous segment is done with the masks
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t t = tt[h];
            H[h] = PkHalf{D.lr, 0, false};
            const uint8_t *Q = D.sr;
            int qbase = 0, qstep = 1, ql = 0;
            if (t >= 0) {
                const int sid = D.t_sr[t], lid = D.t_lr[t];
                const bool rev = D.t_strand[t] != 0;
                const int qb = D.o_qb[t], qe = D.o_qe[t], rb = D.o_rb[t], re = D.o_re[t];
                const int L = (int)(D.lr_off[lid + 1] - D.lr_off[lid]);
                H[h] = PkHalf{D.lr + D.lr_off[lid] + (rev ? (long)L - re : (long)rb), re - rb, rev};
                Q = D.sr + D.sr_off[sid];
                qbase = rev ? qe - 1 : qb;
                qstep = rev ? -1 : 1;
                ql = lqq;
            }
            if (pk_build_mask(Q, qbase, qstep, ql, lm + (h * 2 * PK_NQW) * SW_WAVE + lane, SW_WAVE)) qn |= 1 << h;
            nrow = nrow > H[h].tlen ? nrow : H[h].tlen;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const int v = __shfl_xor(nrow, o, 64);
            nrow = nrow > v ? nrow : v;
        }
        nrow = __builtin_amdgcn_readfirstlane(nrow);
        const int npair = pk_npair(ww);
        int sc[2] = {0, 0}, nflag = 0;
        unsigned long long c1 = clock64();
        ph[0] += c1 - c0;
        glob_pk<WB>(H[0], H[1], lqq, ww, nrow, O, lm + lane, lm + 2 * PK_NQW * SW_WAVE + lane, SW_WAVE, zl,
                    SW_WAVE, sc[0], sc[1], nflag);
        nflag |= qn;
        // (the masks are dead from here on)
        uint32_t *cg[2] = {nullptr, nullptr};
        int tl[2] = {0, 0}, cap[2] = {0, 0};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t t = tt[h];
            if (t < 0) continue;
            const int rlen = H[h].tlen;
            const int w2 = glob_w2(D, O, t, lqq, rlen);
            if ((nflag >> h) & 1 || (w2 != O.w << 2 && sc[h] < D.o_truesc[t] - O.a)) {
                D.x_try[t] = (uint8_t)(D.x_try[t] | 4);
                continue;
            }
            cells += band_cells(rlen, lqq, ww);
            if (split) {   // the score for the backtrack kernel's emit
                D.o_gscore[t] = sc[h];
                continue;
            }
            cg[h] = cig_dest(D, t, cap[h]);
            tl[h] = rlen;
        }
        unsigned long long c2 = clock64();
        ph[1] += c2 - c1;
        if (split) continue;
        int nc[2] = {0, 0};
        uint32_t fst[2] = {0u, 0u}, lst[2] = {0u, 0u};
        if (O.debug & 1) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (cg[h]) cg[h][cap[h] - 1] = fst[h] = lst[h] = ((uint32_t)lqq << 4), nc[h] = 1;
        } else {
            pk_backtrack2<BTW>(zl, SW_WAVE, npair, nrow, tl, lqq, ww, cg, nc, fst, lst, cap);
        }
        unsigned long long c3 = clock64();
        ph[2] += c3 - c2;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (cg[h]) pk_emit(D, tt[h], cg[h], cap[h], nc[h], fst[h], lst[h], sc[h], H[h].comp);
        ph[3] += clock64() - c3;
    }
    if (lane == 0)
        for (int q = 0; q < 4; ++q)
            if (ph[q]) atomicAdd(&D.cells[3 + q], ph[q]);
    for (int o = 32; o > 0; o >>= 1) cells += __shfl_down(cells, o, 64);
    if (lane == 0 && cells) {
        atomicAdd(&D.cells[1], cells);
        atomicAdd(&D.cells[2], cells);   // the dominant launch's own cells (bench roofline)
    }
}

// The backtrack + emit of the packed CIGAR pass over the slabs sw_global_pk_kernel(split = 1)
// wrote for the chunk [seg0, seg1): one wave per segment, the same lanes and halves as the DP;
// tasks the DP handed to the LDS kernel (x_try bit 2) are skipped.
template <int WIN>
__global__ void __launch_bounds__(SW_WAVE, WIN == 4 ? 6 : (WIN == 8 ? 4 : 3)) sw_global_pk_bt_kernel(SwDev D, SwOptsDev O, int seg0, int seg1) {
    const int lane = threadIdx.x;
    const int nseg_all = D.pk_bucket[PK_SCAN] / PK_SEG;
    const int nseg = seg1 < nseg_all ? seg1 : nseg_all;
    unsigned long long ph[2] = {0, 0};   // wave cycles: backtrack, emit
    unsigned st[2] = {0u, 0u};           // O.debug & 4: off-pair loads, walk steps
    for (int seg = seg0 + blockIdx.x; seg < nseg; seg += gridDim.x) {
        const unsigned long long c0 = clock64();
        const PkDir *zl = reinterpret_cast<const PkDir *>(D.z) + (int64_t)(seg - seg0) * D.z_pk_slab + lane;
        const int64_t tt[2] = {D.list[(int64_t)seg * PK_SEG + lane], D.list[(int64_t)seg * PK_SEG + 64 + lane]};
        const int key = __builtin_amdgcn_readfirstlane(pk_key(D, O, D.list[(int64_t)seg * PK_SEG]));
        const int ww = key >> 8, lqq = key & 255;
        uint32_t *cg[2] = {nullptr, nullptr};
        int tl[2] = {0, 0}, cap[2] = {0, 0}, nrow = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t t = tt[h];
            if (t < 0 || (D.x_try[t] & 4)) continue;
            tl[h] = D.o_re[t] - D.o_rb[t];
            cg[h] = cig_dest(D, t, cap[h]);
            nrow = nrow > tl[h] ? nrow : tl[h];
        }
        for (int o = 32; o > 0; o >>= 1) {
            const int v = __shfl_xor(nrow, o, 64);
            nrow = nrow > v ? nrow : v;
        }
        nrow = __builtin_amdgcn_readfirstlane(nrow);
        int nc[2] = {0, 0};
        uint32_t fst[2] = {0u, 0u}, lst[2] = {0u, 0u};
        if (O.debug & 1) {
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (cg[h]) cg[h][cap[h] - 1] = fst[h] = lst[h] = ((uint32_t)lqq << 4), nc[h] = 1;
        } else if (nrow > 0) {
            pk_backtrack2<WIN>(zl, SW_WAVE, pk_npair(ww), nrow, tl, lqq, ww, cg, nc, fst, lst, cap,
                               (O.debug & 4) ? st : nullptr);
        }
        const unsigned long long c1 = clock64();
        ph[0] += c1 - c0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (cg[h]) pk_emit(D, tt[h], cg[h], cap[h], nc[h], fst[h], lst[h], D.o_gscore[tt[h]], D.t_strand[tt[h]] != 0);
        ph[1] += clock64() - c1;
    }
    if (lane == 0) {
        if (ph[0]) atomicAdd(&D.cells[5], ph[0]);
        if (ph[1]) atomicAdd(&D.cells[6], ph[1]);
    }
    if (O.debug & 4) {
        unsigned long long a = st[0], b = st[1];
        for (int o = 32; o > 0; o >>= 1) a += __shfl_down(a, o, 64), b += __shfl_down(b, o, 64);
        if (lane == 0) atomicAdd(&D.cells[7], a), atomicAdd(&D.cells[9], b);
    }
}

// ordering of the packed kernel's tasks: counting sort by key, every key's run
// padded to a multiple of 128 (padding entries -1)
__device__ __forceinline__ int pk_mode_key(const SwDev &D, const SwOptsDev &O, int64_t t, int mode) {
    return mode == 0 ? pk_key(D, O, t) : pk_ext_key(D, O, t, mode - 1);
}
__global__ void __launch_bounds__(256) pk_order_count(SwDev D, SwOptsDev O, int mode) {
    __shared__ int hist[PK_NB];
    for (int k = threadIdx.x; k < PK_NB; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = sel_task(D, q);
        const int k = pk_mode_key(D, O, t, mode);
        D.perm[q] = k;   // the scatter pass reads the key back instead of recomputing it twice
        if (k >= 0) atomicAdd(&hist[k], 1);
        else if (mode == 0 && sel_cig(D, t)) {
            // the CIGAR pass's other kernels: their class as an x_try bit, so the three listing
            // passes after the packed kernel test one byte (0x40 ring<40>, 0x80 ring<80>, 4 LDS)
            const int c = glob_class(D, O, t);
            D.x_try[t] = (uint8_t)(D.x_try[t] | (c == 0 ? 0x40 : (c == 1 ? 0x80 : 4)));
        }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < PK_NB; k += blockDim.x)
        if (hist[k]) atomicAdd(&D.pk_bucket[k], hist[k]);
}
__global__ void __launch_bounds__(1024) pk_order_scan(int32_t *b) {
    __shared__ int part[1024];
    constexpr int per = PK_SCAN / 1024;
    const int tid = threadIdx.x;
    int s = 0;
    for (int k = 0; k < per; ++k) s += (b[tid * per + k] + PK_SEG - 1) / PK_SEG * PK_SEG;
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
        const int c = (b[tid * per + k] + PK_SEG - 1) / PK_SEG * PK_SEG;
        b[tid * per + k] = base;
        base += c;
    }
    if (tid == 1023) b[PK_SCAN] = part[1023];   // padded list length
}
__global__ void __launch_bounds__(256) pk_order_scatter(SwDev D, SwOptsDev O, int mode) {
    __shared__ int hist[PK_NB];
    for (int k = threadIdx.x; k < PK_NB; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int k = D.perm[q];   // (pk_order_count's key of selection entry q)
        if (k >= 0) atomicAdd(&hist[k], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < PK_NB; k += blockDim.x)
        if (hist[k]) hist[k] = atomicAdd(&D.pk_bucket[k], hist[k]);
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int k = D.perm[q];
        if (k >= 0) D.list[atomicAdd(&hist[k], 1)] = (int32_t)sel_task(D, q);
    }
}
// Fill of a large buffer with a byte-pattern word (0 / 0xFF..): 16-byte stores over a grid that
// spreads over the chip.  The runtime's fill kernel for tens of MB takes a few workgroups and,
// beside a kernel that holds most CUs (the chain-head links on the side stream), ran 2 ms for
// the 35 MB x_try of configs[1].
__global__ void __launch_bounds__(256) sw_fill_kernel(uint32_t *p, uint32_t v, int64_t n) {
    const int64_t n4 = n >> 2, stride = (int64_t)gridDim.x * blockDim.x;
    uint4 *q = reinterpret_cast<uint4 *>(p);
    const uint4 vv = make_uint4(v, v, v, v);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) q[i] = vv;
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}
static hipError_t sw_fill(void *p, uint32_t byte, size_t bytes, hipStream_t s) {
    if (((uintptr_t)p & 15u) || (bytes & 3u) || bytes < ((size_t)1 << 20))
        return hipMemsetAsync(p, (int)byte, bytes, s);
    const int64_t n = (int64_t)(bytes >> 2);
    int64_t grid = (n / 4 + 255) / 256;
    grid = grid < 2048 ? grid : 2048;
    hipLaunchKernelGGL(sw_fill_kernel, dim3((unsigned)grid), dim3(256), 0, s, (uint32_t *)p, byte * 0x01010101u, n);
    return hipGetLastError();
}

int sw_launch_pk_order(const SwDev &D, const SwOptsDev &O, int mode, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    // the key counts and (8 words before them) the packed kernels' segment dequeue counters
    hipError_t e = hipMemsetAsync(D.pk_bucket - 8, 0, (8 + PK_SCAN + 1) * sizeof(int32_t), s);
    if (e != hipSuccess) return (int)e;
    e = sw_fill(D.list, 0xFFu, (size_t)(sel_count(D) + (int64_t)PK_NB * PK_SEG + 1) * sizeof(int32_t), s);
    if (e != hipSuccess) return (int)e;
    int grid = (int)((sel_count(D) + 255) / 256);
    grid = grid < 2048 ? (grid > 0 ? grid : 1) : 2048;
    hipLaunchKernelGGL(pk_order_count, dim3(grid), dim3(256), 0, s, D, O, mode);
    hipLaunchKernelGGL(pk_order_scan, dim3(1), dim3(1024), 0, s, D.pk_bucket);
    hipLaunchKernelGGL(pk_order_scatter, dim3(grid), dim3(256), 0, s, D, O, mode);
    return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Task ordering: lanes of a wave run in lock-step, so every DP launch takes its
// tasks bucketed by query length (counting sort; the order inside a bucket does
// not affect results).  Phase keys: 0/1 left extension try 0/1 (qbeg), 2/3
// right extension try 0/1 (right length), 5/6 CIGAR pass 1 in the register
// ring (band <= 40 / <= 80), 7 CIGAR passes in the LDS kernel (query length).
__device__ __forceinline__ int sw_phase_key(const SwDev &D, const SwOptsDev &O, int64_t t, int phase) {
    // (the task's flags first: most tasks of a listing pass are decided by that one byte, and
    // their geometry loads are skipped)
    if (!(phase < 4 ? sel_ext(D, t) : sel_cig(D, t))) return -1;
    const uint8_t x = D.x_try[t];
    // every extension inside the packed kernel's frame went through it: only N-flagged tasks are left
    const bool pk_all = O.pk && O.w <= 40 && D.qmax <= PK_QMAX && O.a * D.qmax <= 2047;
    switch (phase) {
        case 0: case 1: case 2: case 3: {
            const int side = phase >> 1;
            if (phase & 1 ? !(x & (1 << side)) : (pk_all && !(x & (8 << side)))) return -1;
            const int qbeg = D.t_qbeg[t];
            if (side == 0) return phase == 1 ? qbeg : ((qbeg > 0 && (pk_ext_key(D, O, t, 0) < 0 || (x & 8))) ? qbeg : -1);
            const int sid = D.t_sr[t];
            const int right = (int)(D.sr_off[sid + 1] - D.sr_off[sid]) - qbeg - D.t_slen[t];
            return phase == 3 ? right : ((right > 0 && (pk_ext_key(D, O, t, 1) < 0 || (x & 16))) ? right : -1);
        }
        // with the packed kernel, its ordering pass left the class of every other task in x_try
        case 5: return (O.pk ? (x & 0x40) != 0 : glob_class(D, O, t) == 0) ? D.o_qe[t] - D.o_qb[t] : -1;
        case 6: return (O.pk ? (x & 0x80) != 0 : glob_class(D, O, t) == 1) ? D.o_qe[t] - D.o_qb[t] : -1;
        case 7: return ((x & 4) || (!O.pk && glob_class(D, O, t) == 2)) ? D.o_qe[t] - D.o_qb[t] : -1;
        case 8: return (x & 0x20) ? D.o_qe[t] - D.o_qb[t] : -1;   // CIGAR overflow pass
        default: return -1;
    }
}
// block-local histograms in LDS, one global atomic per (block, key)
__global__ void __launch_bounds__(256) sw_order_count(SwDev D, SwOptsDev O, int phase) {
    __shared__ int hist[SW_NBUCKET];
    for (int k = threadIdx.x; k < SW_NBUCKET; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = sel_task(D, q);
        const int k = sw_phase_key(D, O, t, phase);
        D.keyc[q] = k;   // read back by sw_order_scatter
        if (k >= 0) atomicAdd(&hist[k < SW_NBUCKET ? k : SW_NBUCKET - 1], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < SW_NBUCKET; k += blockDim.x)
        if (hist[k]) atomicAdd(&D.bucket[k], hist[k]);
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
    if (tid == 1023) b[SW_NBUCKET] = part[1023];   // list length
}
// same grid and task partition as sw_order_count: each block reserves its
// per-key ranges with one atomic each, then places its tasks
__global__ void __launch_bounds__(256) sw_order_scatter(SwDev D, SwOptsDev O, int phase, int32_t *out) {
    __shared__ int hist[SW_NBUCKET];
    for (int k = threadIdx.x; k < SW_NBUCKET; k += blockDim.x) hist[k] = 0;
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int k = D.keyc[q];   // (sw_order_count's key of selection entry q)
        if (k >= 0) atomicAdd(&hist[k < SW_NBUCKET ? k : SW_NBUCKET - 1], 1);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < SW_NBUCKET; k += blockDim.x)
        if (hist[k]) hist[k] = atomicAdd(&D.bucket[k], hist[k]);
    __syncthreads();
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < sel_count(D); q += (int64_t)gridDim.x * blockDim.x) {
        const int k = D.keyc[q];
        if (k >= 0) out[atomicAdd(&hist[k < SW_NBUCKET ? k : SW_NBUCKET - 1], 1)] = (int32_t)sel_task(D, q);
    }
}

int sw_launch_order(const SwDev &D, const SwOptsDev &O, int phase, int32_t *out, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(D.bucket, 0, (SW_NBUCKET + 1) * sizeof(int32_t), s);
    if (e != hipSuccess) return (int)e;
    int grid = (int)((sel_count(D) + 255) / 256);
    grid = grid < 2048 ? (grid > 0 ? grid : 1) : 2048;
    hipLaunchKernelGGL(sw_order_count, dim3(grid), dim3(256), 0, s, D, O, phase);
    hipLaunchKernelGGL(sw_order_scan, dim3(1), dim3(1024), 0, s, D.bucket);
    hipLaunchKernelGGL(sw_order_scatter, dim3(grid), dim3(256), 0, s, D, O, phase, out);
    return (int)hipGetLastError();
}

// resident waves per CU of the packed CIGAR backtrack kernel (window of win rows)
int sw_pk_bt_occupancy(int win) {
    int nb = 0;
    const hipError_t e = win == 4 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_global_pk_bt_kernel<4>, SW_WAVE, 0)
        : win == 8 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_global_pk_bt_kernel<8>, SW_WAVE, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sw_global_pk_bt_kernel<16>, SW_WAVE, 0);
    return e == hipSuccess && nb > 0 ? nb : 8;
}

// the four extension phases + the two finish passes (mem_chain2aln)
int sw_launch_extend(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, void *stream, SwEvPool *evp) {
    hipStream_t s = (hipStream_t)stream;
    auto mark = [&]() {   // an event before / after each DP launch (when the pool has room)
        if (evp && evp->n < SwEvPool::CAP && evp->ev[evp->n]) (void)hipEventRecord((hipEvent_t)evp->ev[evp->n++], s);
        else if (evp) ++evp->dropped;   // pool full: this launch goes untimed (reported by the caller)
    };
    int fgrid = (int)((sel_count(D) + 255) / 256);
    fgrid = fgrid < 8192 ? (fgrid > 0 ? fgrid : 1) : 8192;
    // (a whole number of dwords: a byte-sized fill takes the runtime's byte kernel, 2 ms for the
    // 35 MB of configs[1]; the buffer has 64 bytes of slack)
    hipError_t e = sw_fill(D.x_try, 0u, ((size_t)D.n_task + 1 + 15) & ~(size_t)15, s);
    if (e != hipSuccess) return (int)e;
    for (int side = 0; side < 2; ++side) {
        for (int tryi = 0; tryi < 2; ++tryi) {
            if (tryi == 0 && O.pk && O.w <= 40) {
                int rc = sw_launch_pk_order(D, O, 1 + side, stream);
                if (rc) return rc;
                mark();
                // every DP value <= a x read length: the one-accumulator row maximum when that fits 9 bits
                if ((long)O.a * D.qmax <= 511)
                    hipLaunchKernelGGL((sw_ext_pk_kernel<40, true>), dim3(grid_pk), dim3(SW_WAVE), 0, s, D, O, side);
                else
                    hipLaunchKernelGGL((sw_ext_pk_kernel<40, false>), dim3(grid_pk), dim3(SW_WAVE), 0, s, D, O, side);
                mark();
                if ((e = hipGetLastError()) != hipSuccess) return (int)e;
            }
            int rc = sw_launch_order(D, O, side * 2 + tryi, D.list, stream);
            if (rc) return rc;
            const int wb = O.w << tryi;
            mark();
            if (wb <= 32) hipLaunchKernelGGL(sw_ext_phase_kernel<32>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O, side, tryi);
            else if (wb <= 40) hipLaunchKernelGGL(sw_ext_phase_kernel<40>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O, side, tryi);
            else if (wb <= 64) hipLaunchKernelGGL(sw_ext_phase_kernel<64>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O, side, tryi);
            else if (wb <= 80 && (2 * wb + 1 > XW_COLS * 64 || getenv("PRGPU_EXT80_LANE")))   // one task per lane
                hipLaunchKernelGGL(sw_ext_phase_kernel<80>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O, side, tryi);
            else if (wb <= 80) {   // one task per wave (ext_wave)
                const int lds = 4 * ((D.qmax + 2) + (D.qmax + 3) / 4) * 4;
                hipLaunchKernelGGL(sw_ext_wave_kernel, dim3(grid_waves), dim3(256), lds, s, D, O, side, tryi);
            }
            else if (D.eh_g) hipLaunchKernelGGL(sw_ext_wide_kernel<true>, dim3(D.eh_g_blocks), dim3(SW_WAVE), 0, s, D, O, side, tryi);
            else {
                const int lds = (D.qmax + 2) * SW_WAVE * 4;
                e = hipFuncSetAttribute((const void *)sw_ext_wide_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
                if (e != hipSuccess) return (int)e;
                hipLaunchKernelGGL(sw_ext_wide_kernel<false>, dim3(grid_waves), dim3(SW_WAVE), lds, s, D, O, side, tryi);
            }
            mark();
            if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        }
        if (side == 0) hipLaunchKernelGGL(sw_left_finish_kernel, dim3(fgrid), dim3(256), 0, s, D, O);
        else hipLaunchKernelGGL(sw_right_finish_kernel, dim3(fgrid), dim3(256), 0, s, D, O);
    }
    return (int)hipGetLastError();
}
int sw_launch_global(const SwDev &D, const SwOptsDev &O, int grid_waves, int grid_pk, int grid_lds, int lds,
                     void *stream, void *ev_a, void *ev_b, bool pk_ordered, void *side, void *ev_fork, void *ev_join,
                     void *z_side, void *ev_mid) {
    hipStream_t s = (hipStream_t)stream;
    int rc;
    // band-80 tasks beside the packed kernel: their class is known from the packed ordering pass
    // (x_try 0x80), their list goes to D.perm and their direction slabs to z_side; the main stream
    // waits for them before its next listing pass (which reuses the bucket counts)
    // (the packed kernel is launched once the band-80 list is made, so that the dispatcher takes
    // the ring kernel's workgroups beside the packed kernel's instead of after them)
    const bool ring80_side = O.pk && D.pk_chunk <= 0 && side && ev_fork && ev_join && ev_mid && z_side && D.perm;
    if (O.pk) {
        if (!pk_ordered && (rc = sw_launch_pk_order(D, O, 0, stream))) return rc;
        if (ring80_side) {
            hipError_t e = hipEventRecord((hipEvent_t)ev_fork, s);
            if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)side, (hipEvent_t)ev_fork, 0);
            if (e != hipSuccess) return (int)e;
            SwDev D6 = D;
            D6.list = D.perm;
            D6.z = (uint8_t *)z_side;
            if ((rc = sw_launch_order(D6, O, 6, D6.list, side))) return rc;
            if ((e = hipEventRecord((hipEvent_t)ev_mid, (hipStream_t)side)) != hipSuccess) return (int)e;
            hipLaunchKernelGGL(sw_global_ring_kernel<80>, dim3(grid_waves), dim3(SW_WAVE), 0, (hipStream_t)side, D6, O);
            if ((e = hipEventRecord((hipEvent_t)ev_join, (hipStream_t)side)) != hipSuccess) return (int)e;
            if ((e = hipStreamWaitEvent(s, (hipEvent_t)ev_mid, 0)) != hipSuccess) return (int)e;
        }
        if (ev_a) (void)hipEventRecord((hipEvent_t)ev_a, s);
        if (D.pk_chunk <= 0) {   // fused: DP and backtrack in one kernel, a slab per resident wave
            // (backtrack window: 8 rows, or 16 with PRGPU_PK_WIN=16)
            if (D.pk_bt_win == 8)
                hipLaunchKernelGGL((sw_global_pk_kernel<40, 8>), dim3(grid_pk), dim3(SW_WAVE), 0, s, D, O, 0, INT32_MAX, 0);
            else
                hipLaunchKernelGGL((sw_global_pk_kernel<40, 16>), dim3(grid_pk), dim3(SW_WAVE), 0, s, D, O, 0, INT32_MAX, 0);
        } else {   // chunks of segments: the DP kernel, then the backtrack kernel over the chunk's slabs
            for (int64_t c0 = 0; c0 < D.pk_nseg_bound; c0 += D.pk_chunk) {
                const int c1 = (int)(c0 + D.pk_chunk < D.pk_nseg_bound ? c0 + D.pk_chunk : D.pk_nseg_bound);
                const int n = c1 - (int)c0;
                hipLaunchKernelGGL((sw_global_pk_kernel<40, 16>), dim3(n < grid_pk ? n : grid_pk), dim3(SW_WAVE), 0, s, D, O,
                                   (int)c0, c1, 1);
                if (D.pk_bt_win == 4)
                    hipLaunchKernelGGL(sw_global_pk_bt_kernel<4>, dim3(n < D.pk_bt_grid ? n : D.pk_bt_grid), dim3(SW_WAVE),
                                       0, s, D, O, (int)c0, c1);
                else if (D.pk_bt_win == 8)
                    hipLaunchKernelGGL(sw_global_pk_bt_kernel<8>, dim3(n < D.pk_bt_grid ? n : D.pk_bt_grid), dim3(SW_WAVE),
                                       0, s, D, O, (int)c0, c1);
                else
                    hipLaunchKernelGGL(sw_global_pk_bt_kernel<16>, dim3(n < D.pk_bt_grid ? n : D.pk_bt_grid), dim3(SW_WAVE),
                                       0, s, D, O, (int)c0, c1);
            }
        }
        if (ev_b) (void)hipEventRecord((hipEvent_t)ev_b, s);
        if (ring80_side) {
            hipError_t e = hipStreamWaitEvent(s, (hipEvent_t)ev_join, 0);
            if (e != hipSuccess) return (int)e;
        }
    }
    if ((rc = sw_launch_order(D, O, 5, D.list, stream))) return rc;
    if (!O.pk && ev_a) (void)hipEventRecord((hipEvent_t)ev_a, s);
    hipLaunchKernelGGL(sw_global_ring_kernel<40>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O);
    if (!O.pk && ev_b) (void)hipEventRecord((hipEvent_t)ev_b, s);
    if (!ring80_side) {
        if ((rc = sw_launch_order(D, O, 6, D.list, stream))) return rc;
        hipLaunchKernelGGL(sw_global_ring_kernel<80>, dim3(grid_waves), dim3(SW_WAVE), 0, s, D, O);
    }
    if ((rc = sw_launch_order(D, O, 7, D.list, stream))) return rc;
    return sw_launch_lds(D, O, grid_lds, lds, stream);
}

// the general CIGAR kernel over the current task list (LDS row, or HBM row when D.eh_g)
int sw_launch_lds(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (D.eh_g) {
        hipLaunchKernelGGL(sw_global_kernel<true>, dim3(grid), dim3(SW_WAVE), 0, s, D, O);
        return (int)hipGetLastError();
    }
    hipError_t e = hipFuncSetAttribute((const void *)sw_global_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(sw_global_kernel<false>, dim3(grid), dim3(SW_WAVE), lds, s, D, O);
    return (int)hipGetLastError();
}

// spill ranges of the overflowed tasks (bump allocation; placement order does not matter)
__global__ void __launch_bounds__(256) sw_spill_assign_kernel(SwDev D) {
    const int n = D.list_n[0];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = D.list[i];
        const unsigned long long b = (unsigned long long)cig_bound_ops(D.o_qe[t] - D.o_qb[t], D.o_re[t] - D.o_rb[t]);
        D.o_cig_at[t] = D.spill_base + (int64_t)atomicAdd(&D.spill[2], b);
    }
}

// compaction of the tasks' CIGARs into one pool in task order (pr_sw_download)
__global__ void __launch_bounds__(256) sw_cig_compact_kernel(const uint32_t *pool, const int64_t *at,
                                                             const int32_t *ncig, const int64_t *off, int64_t n,
                                                             uint32_t *out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t *src = pool + at[t];
        uint32_t *dst = out + off[t];
        const int m = (int)(off[t + 1] - off[t]);
        for (int k = 0; k < m; ++k) dst[k] = src[k];
    }
}
int sw_launch_cig_compact(const uint32_t *pool, const int64_t *at, const int32_t *ncig, const int64_t *off,
                          int64_t n, uint32_t *out, void *stream) {
    int grid = (int)((n + 255) / 256);
    grid = grid < 4096 ? (grid > 0 ? grid : 1) : 4096;
    hipLaunchKernelGGL(sw_cig_compact_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, pool, at, ncig, off, n, out);
    return (int)hipGetLastError();
}

// the overflow pass: list the overflowed tasks, give them spill ranges, rerun their CIGAR loop
int sw_launch_overflow(const SwDev &D, const SwOptsDev &O, int grid, int lds, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    int rc;
    if ((rc = sw_launch_order(D, O, 8, D.list, stream))) return rc;
    hipLaunchKernelGGL(sw_spill_assign_kernel, dim3(256), dim3(256), 0, s, D);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    SwDev R = D;
    R.rerun = 1;
    return sw_launch_lds(R, O, grid, lds, stream);
}


}  // namespace prgpu
