// ksw_global2 for TWO tasks per lane in packed 16-bit arithmetic (device code,
// also compiled for the host by tests/native/ring_host.cpp and checked against
// the oracle there).
//
// Every 32-bit register holds one DP value of task A (low half) and of task B
// (high half); one v_pk_* instruction advances both.  The two tasks of a lane,
// and all 64 lanes of a wave, share the band w and the query length (the
// ordering kernel groups tasks by (w, qlen) in 128-task segments), so the band
// geometry of every row is wave-uniform and only the sequences differ.
//
// Slot scheme.  Slot s of row i holds query column c = i - w + s (the band of
// row i starts at slot max(0, w - i)); NS = 2*WB + 2 slots.  The word read by
// slot s is ring word s+1 (ksw_global2's eh[c]: H(i-1, c-1), E(i, c)), the new
// eh[c] goes to ring word s: every column moves down one slot per row.
// Columns left of the band are not masked out: columns < 0 carry NEG words and
// column -1 carries E(i,-1) = -(o_del + e_del*(i+1)), so its cell yields
// ksw_global2's H(i,-1) boundary naturally and the left edge needs no select.
// Columns right of the band end are dead; the end column's E is set to NEG by
// a per-row fixup (ksw_global2's eh[end].e = KSW_NEG_INF).
//
// Biased frame.  Values of row i carry the bias beta_i = (i+1)*b, so the score
// step is M = Hdiag + (a+b)*[match] (no separate mismatch add); E is stored
// pre-biased for the next row (its constants absorb the +b), F lives within the
// row.  The final score is H - tlen*b.  All finite values stay within
// (-7000, 9000) for the routed tasks (qlen <= 255, tlen <= 320, penalties <= 32);
// NEG = -18000 (KSW_NEG_INF stand-in, only ever compared with finite values).
//
// Direction bits per cell (ksw_global2's): D1 = M < E, D2 = max(M,E) < F,
// D3 = E-continue, D4 = F-continue, from the sign bits of packed differences;
// v_perm_b32 turns the signs of two differences into four 0x00/0xFF bytes and
// one v_bfi_b32 drops the slot's bit into them.  Per 8-slot chunk a lane
// accumulates two dwords x = [A.D1, B.D1, A.D2, B.D2], y = [A.D3, B.D3, A.D4,
// B.D4] (byte per task and bit, bit k = slot 8c+k) and stores them per row as
// 16-byte pairs of chunks (one coalesced 1 KB store per wave).
//
// Match bits come from two bit masks per task (bit 0 / bit 1 of the 2-bit base
// code over the query positions, 64-bit left pad), windowed per row with
// v_alignbit_b32 and interleaved into 16-slot groups with v_perm_b32.  Tasks
// with an N in the query or the target window are flagged and recomputed by
// the general kernel (exact N scoring).
#pragma once
#include <stdint.h>

#include "sw_ring.h"

namespace prgpu {

constexpr int PK_NQW = 13;        // mask words per (task, bit): 64-bit pad + 255 bases + 96-bit window
constexpr int PK_QMAX = 255;      // routed query lengths
constexpr int PK_TMAX = 320;      // routed reference lengths
constexpr int PK_NEG = -18000;

#ifndef SW_RING_HOST
typedef short pk_v __attribute__((ext_vector_type(2)));
SW_RING_FN pk_v PV(uint32_t u) { return __builtin_bit_cast(pk_v, u); }
SW_RING_FN uint32_t PU(pk_v v) { return __builtin_bit_cast(uint32_t, v); }
SW_RING_FN uint32_t pk_add(uint32_t a, uint32_t b) { return PU(PV(a) + PV(b)); }
SW_RING_FN uint32_t pk_sub(uint32_t a, uint32_t b) { return PU(PV(a) - PV(b)); }
SW_RING_FN uint32_t pk_max(uint32_t a, uint32_t b) { return PU(__builtin_elementwise_max(PV(a), PV(b))); }
SW_RING_FN uint32_t pk_min(uint32_t a, uint32_t b) { return PU(__builtin_elementwise_min(PV(a), PV(b))); }
SW_RING_FN uint32_t pk_maxu(uint32_t a, uint32_t b) {
    typedef unsigned short pu_v __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(pu_v, a), __builtin_bit_cast(pu_v, b)));
}
SW_RING_FN uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c) { return PU(PV(a) * PV(b) + PV(c)); }
SW_RING_FN uint32_t pk_shl(uint32_t a, int k) { return PU(PV(a) << pk_v{(short)k, (short)k}); }
SW_RING_FN uint32_t pk_asr15(uint32_t a) { return PU(PV(a) >> pk_v{15, 15}); }
typedef unsigned short pku_v __attribute__((ext_vector_type(2)));
// unsigned saturating subtract: max(a - b, 0) per half for a, b in [0, 32767] (v_pk_sub_u16 clamp)
SW_RING_FN uint32_t pk_subs(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(pku_v, a), __builtin_bit_cast(pku_v, b)));
}
SW_RING_FN uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) { return __builtin_amdgcn_perm(s0, s1, sel); }
SW_RING_FN uint32_t align_b32(uint32_t hi, uint32_t lo, uint32_t sh) { return __builtin_amdgcn_alignbit(hi, lo, sh); }
#else
SW_RING_FN int16_t pk_lo(uint32_t a) { return (int16_t)(a & 0xFFFFu); }
SW_RING_FN int16_t pk_hi(uint32_t a) { return (int16_t)(a >> 16); }
SW_RING_FN uint32_t pk_mk(int lo, int hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); }
SW_RING_FN uint32_t pk_add(uint32_t a, uint32_t b) { return pk_mk(pk_lo(a) + pk_lo(b), pk_hi(a) + pk_hi(b)); }
SW_RING_FN uint32_t pk_sub(uint32_t a, uint32_t b) { return pk_mk(pk_lo(a) - pk_lo(b), pk_hi(a) - pk_hi(b)); }
SW_RING_FN uint32_t pk_max(uint32_t a, uint32_t b) {
    return pk_mk(pk_lo(a) > pk_lo(b) ? pk_lo(a) : pk_lo(b), pk_hi(a) > pk_hi(b) ? pk_hi(a) : pk_hi(b));
}
SW_RING_FN uint32_t pk_min(uint32_t a, uint32_t b) {
    return pk_mk(pk_lo(a) < pk_lo(b) ? pk_lo(a) : pk_lo(b), pk_hi(a) < pk_hi(b) ? pk_hi(a) : pk_hi(b));
}
SW_RING_FN uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c) {
    return pk_mk(pk_lo(a) * pk_lo(b) + pk_lo(c), pk_hi(a) * pk_hi(b) + pk_hi(c));
}
SW_RING_FN uint32_t pk_maxu(uint32_t a, uint32_t b) {
    const uint32_t al = a & 0xFFFFu, bl = b & 0xFFFFu, ah = a >> 16, bh = b >> 16;
    return (al > bl ? al : bl) | ((ah > bh ? ah : bh) << 16);
}
SW_RING_FN uint32_t pk_shl(uint32_t a, int k) { return pk_mk((uint16_t)(a << k), (uint16_t)((a >> 16) << k)); }
SW_RING_FN uint32_t pk_asr15(uint32_t a) { return pk_mk(pk_lo(a) >> 15, pk_hi(a) >> 15); }
SW_RING_FN uint32_t pk_subs(uint32_t a, uint32_t b) {
    const uint32_t al = a & 0xFFFFu, bl = b & 0xFFFFu, ah = a >> 16, bh = b >> 16;
    return (al > bl ? al - bl : 0u) | ((ah > bh ? ah - bh : 0u) << 16);
}
SW_RING_FN uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
    const uint64_t d = ((uint64_t)s0 << 32) | s1;
    uint32_t r = 0;
    for (int k = 0; k < 4; ++k) {
        const uint32_t v = (sel >> (8 * k)) & 0xFFu;
        uint32_t byte;
        if (v >= 13) byte = 0xFFu;
        else if (v == 12) byte = 0u;
        else if (v >= 8) byte = ((d >> (16 * (v - 8) + 15)) & 1u) ? 0xFFu : 0u;
        else byte = (uint32_t)(d >> (8 * v)) & 0xFFu;
        r |= byte << (8 * k);
    }
    return r;
}
SW_RING_FN uint32_t align_b32(uint32_t hi, uint32_t lo, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (sh & 31u));
}
#endif
SW_RING_FN uint32_t pk_dup(int v) { return (uint32_t)(uint16_t)v * 0x10001u; }
#ifdef SW_RING_HOST
// host test builds: every direction-word read is checked against the slab the test allocated
extern long pk_host_zlen;
#define PK_ZCHECK(idx) do { if ((idx) < 0 || (idx) >= pk_host_zlen) __builtin_trap(); } while (0)
#else
#define PK_ZCHECK(idx) ((void)0)
#endif

// One half (task) of a lane pair as glob_pk sees it.
struct PkHalf {
    const uint8_t *T;   // first reference base of the window in the forward long read (nt4)
    int tlen;           // rows; 0 = empty half
    bool comp;          // reverse strand: complement the reference bases
};

// The reference bases of rows r .. r + 15 of a task (step ts), byte k = row r + k (not yet complemented):
// one unaligned 16-byte load per 16 rows instead of a byte load per row.  (Per-row byte loads
// kept one 128-B line per task live for the whole extension: 128 tasks x 8 waves per CU filled
// each XCD's L2, so nearly every row missed it.)  The window may run up to 15 bytes past either
// end of the read: the pools keep 64 bytes of slack on both sides, and the bytes of rows >= tlen
// are never used.
SW_RING_FN void pk_tref16(const uint8_t *T, int ts, int r, uint32_t w[4]) {
    uint32_t x[4];
    __builtin_memcpy(x, ts > 0 ? T + r : T - r - 15, 16);
    if (ts > 0) {
        w[0] = x[0], w[1] = x[1], w[2] = x[2], w[3] = x[3];
    } else {
        w[0] = __builtin_bswap32(x[3]), w[1] = __builtin_bswap32(x[2]);
        w[2] = __builtin_bswap32(x[1]), w[3] = __builtin_bswap32(x[0]);
    }
}
// 8 bases (rows r .. r + 7), as pk_tref16
SW_RING_FN void pk_tref8(const uint8_t *T, int ts, int r, uint32_t w[2]) {
    uint32_t x[2];
    __builtin_memcpy(x, ts > 0 ? T + r : T - r - 7, 8);
    if (ts > 0) {
        w[0] = x[0], w[1] = x[1];
    } else {
        w[0] = __builtin_bswap32(x[1]), w[1] = __builtin_bswap32(x[0]);
    }
}
SW_RING_FN void pk_shr8_2(uint32_t w[2]) {
    w[0] = (w[0] >> 8) | (w[1] << 24);
    w[1] >>= 8;
}
// the window one row on
SW_RING_FN void pk_shr8(uint32_t w[4]) {
    w[0] = (w[0] >> 8) | (w[1] << 24);
    w[1] = (w[1] >> 8) | (w[2] << 24);
    w[2] = (w[2] >> 8) | (w[3] << 24);
    w[3] >>= 8;
}

// Query bit masks of one task: m[(bit * PK_NQW + k) * MS], bit 0 / 1 of the base code
// at bit 64 + j of the 416-bit string; returns true if the query holds an N.
// (The byte loads of a word are unrolled so that they are all in flight together.)
SW_RING_FN bool pk_build_mask(const uint8_t *Q, int qbase, int qstep, int qlen, uint32_t *m, int MS) {
    bool has_n = false;
    for (int k = 0; k < PK_NQW; ++k) {
        uint32_t b0 = 0u, b1 = 0u;
        const int j0 = 32 * k - 64;
        if (j0 + 32 > 0 && j0 < qlen) {
            uint32_t q[32];
#pragma unroll
            for (int x = 0; x < 32; ++x) {
                const int j = j0 + x;
                q[x] = (j >= 0 && j < qlen) ? (uint32_t)Q[qbase + qstep * j] : 0u;
            }
#pragma unroll
            for (int x = 0; x < 32; ++x) {
                has_n |= q[x] > 3u;
                b0 |= (q[x] & 1u) << x;
                b1 |= ((q[x] >> 1) & 1u) << x;
            }
        }
        m[k * MS] = b0;
        m[(PK_NQW + k) * MS] = b1;
    }
    return has_n;
}

// match bits of one task for the 96 columns from (p - 64): bit x of win[g] = column p - 64 + 32g + x
SW_RING_FN void pk_window(const uint32_t *m, int MS, int p, int t, uint32_t win[3]) {
    const int k = p >> 5;
    const uint32_t sh = (uint32_t)(p & 31);
    const uint32_t t0 = (t & 1) ? 0xFFFFFFFFu : 0u, t1 = (t & 2) ? 0xFFFFFFFFu : 0u;
    uint32_t a[4], c[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
        a[x] = m[(k + x) * MS];
        c[x] = m[(PK_NQW + k + x) * MS];
    }
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        const uint32_t q0 = align_b32(a[g + 1], a[g], sh), q1 = align_b32(c[g + 1], c[g], sh);
        win[g] = ~((q0 ^ t0) | (q1 ^ t1));
    }
}

// bitfield insert: bits of v where mask is set, of acc elsewhere (one v_bfi_b32)
#ifndef SW_RING_HOST
SW_RING_FN uint32_t bfi_b32(uint32_t mask, uint32_t v, uint32_t acc) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(mask), "v"(v), "v"(acc));
    return r;
}
// (a plain expression: the compiler emits v_bfi_b32 / v_bitop3_b32 and, unlike for an
// inline asm, knows its hazards)
// keeps a wave-uniform conditional block a real branch (a volatile asm cannot be
// speculated), so skipped chunks cost a scalar branch instead of per-slot selects
SW_RING_FN uint32_t bfi_b32v(uint32_t mask, uint32_t v, uint32_t acc) { return (mask & v) | (~mask & acc); }
#define PK_BRANCH_BARRIER() asm volatile("")
#else
SW_RING_FN uint32_t bfi_b32v(uint32_t mask, uint32_t v, uint32_t acc) { return (mask & v) | (~mask & acc); }
SW_RING_FN uint32_t bfi_b32(uint32_t mask, uint32_t v, uint32_t acc) { return (mask & v) | (~mask & acc); }
#define PK_BRANCH_BARRIER() ((void)0)
#endif

// Direction bits of one (row, 16-slot pair of chunks), 3 bit planes (12 bytes a lane; round 4's
// four planes D1..D4 were 16).  ksw_global2's backtrack reads at a cell either the h source
// (state M: F if D2, else E if D1, else M), or D3 (state E) or D4 (state F), and D1 => D3, D2 => D4
// (e0 > M => M - e0 < o_del; f > max(M, e0) => f > M - o_ins): 8 cases, 3 bits.  Planes: p3 = the
// source is not M; p1 = source F, or (source M and D3); p2 = D3 for source F, else D4.  Each plane
// word: byte 0 / 1 = half A / B of chunk 2p (a bit per slot), byte 2 / 3 = the same of chunk 2p+1.
struct PkDir {
    uint32_t p1, p2, p3;
};
// glob_pk's chunk words (bytes D1A, D1B, D2A, D2B and D3A, D3B, D4A, D4B) of chunks 2p / 2p+1 -> PkDir
SW_RING_FN PkDir pk_dir_enc(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    const uint32_t d1 = perm_b32(x1, x0, 0x05040100u), d2 = perm_b32(x1, x0, 0x07060302u);
    const uint32_t d3 = perm_b32(y1, y0, 0x05040100u), d4 = perm_b32(y1, y0, 0x07060302u);
    return PkDir{d2 | (d3 & ~d1), (d2 & d3) | (d4 & ~d2), d1 | d2};
}
// the planes back to D1 (D1 and not D2: the backtrack never reads D1 under D2) .. D4, words in
// the plane layout
SW_RING_FN void pk_dir_dec(const PkDir &v, uint32_t &d1, uint32_t &d2, uint32_t &d3, uint32_t &d4) {
    d1 = v.p3 & ~v.p1;
    d2 = v.p3 & v.p1;
    d3 = (v.p1 ^ v.p3) | (v.p1 & v.p2 & v.p3);
    d4 = v.p2 | (v.p3 & v.p1);
}
constexpr int pk_npair(int w) { return (2 * w + 2 + 15) >> 4; }

// The DP of both tasks.  mA/mB: their query masks; nrows = wave max of tlen;
// z: direction words of this lane, (row, pair) at z[(i * npair + p) * ZS];
// scA/scB: ksw_global2 scores (reference N rows scored as bwa does, -1 a cell; the caller flags
// queries with an N).  w and qlen must be wave-uniform.
template <int WB>
SW_RING_FN void glob_pk(const PkHalf &A, const PkHalf &B, int qlen, int w, int nrows, const SwOptsDev &O,
                        const uint32_t *mA, const uint32_t *mB, int MS, PkDir *z, int ZS, int &scA, int &scB,
                        int &nflag) {
    constexpr int NS = 2 * WB + 2;
    constexpr int CH = 8;
    constexpr int NCH = (NS + CH - 1) / CH;
    const int b = O.b;
    const int npair = pk_npair(w);
    const uint32_t NEG = pk_dup(PK_NEG);
    const uint32_t NAB = pk_dup(-(O.a + b));               // m = -1 on a match: M = Hd + (a + b)
    const uint32_t NB1 = pk_dup(-(b - 1));                 // a reference N row: M = Hd + (b - 1)
    const uint32_t cE = pk_dup(O.e_del - b);               // E' = e0 - e_del (+ b: next row's bias)
    const uint32_t cT1 = pk_dup(O.o_del + O.e_del - b);    // t1 = M - oe_del (+ b)
    const uint32_t cD3 = pk_dup(O.o_del);                  // t1 - E' = D1 - o_del
    const uint32_t cF = pk_dup(O.e_ins);
    const uint32_t cT2 = pk_dup(O.o_ins + O.e_ins);
    uint32_t RH[NS], RE[NS];
    // row -1 (bias 0 for H, b for the stored E): eh[c] for c = s - w - 1
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int c = s - w - 1;
        int h = PK_NEG, e = PK_NEG;
        if (c == -1) e = -(O.o_del + O.e_del) + b;
        else if (c == 0) h = 0;
        else if (c > 0 && c <= w && c <= qlen) h = -(O.o_ins + O.e_ins * c);
        RH[s] = pk_dup(h);
        RE[s] = pk_dup(e);
    }
    uint32_t twA[4] = {0u, 0u, 0u, 0u}, twB[4] = {0u, 0u, 0u, 0u};   // reference windows: byte 0 = row i
    if (A.tlen > 0) pk_tref16(A.T, 1, 0, twA);
    if (B.tlen > 0) pk_tref16(B.T, 1, 0, twB);
    int hlA = 0, hlB = 0;
    const int tmax = A.tlen > B.tlen ? A.tlen : B.tlen;
    for (int i = 0; i < nrows; ++i) {
        // reference bases of row i
        int ca = (int)(twA[0] & 0xFFu), cb = (int)(twB[0] & 0xFFu);
        if ((i & 15) == 15) {   // (wave-uniform)
            if (i + 1 < A.tlen) pk_tref16(A.T, 1, i + 1, twA);
            if (i + 1 < B.tlen) pk_tref16(B.T, 1, i + 1, twB);
        } else {
            pk_shr8(twA);
            pk_shr8(twB);
        }
        if (A.comp && ca < 4) ca = 3 - ca;
        if (B.comp && cb < 4) cb = 3 - cb;
        // match groups: slot s <-> bit s & 15 of G[s >> 4] (low half A, high half B)
        uint32_t wa[3], wb[3], G[6];
        pk_window(mA, MS, i - w + 64, ca & 3, wa);
        pk_window(mB, MS, i - w + 64, cb & 3, wb);
        // a reference N row scores -1 in every column (bwa_fill_scmat): with the row bias b that is
        // + (b - 1) on every slot -- all bits set and the row's step (b - 1) for that half
        const bool na = ca > 3, nb = cb > 3;
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            wa[g] = na ? 0xFFFFFFFFu : wa[g];
            wb[g] = nb ? 0xFFFFFFFFu : wb[g];
            G[2 * g] = perm_b32(wb[g], wa[g], 0x05040100u);
            G[2 * g + 1] = perm_b32(wb[g], wa[g], 0x07060302u);
        }
        const uint32_t NABr = (na || nb) ? ((na ? NB1 : NAB) & 0xFFFFu) | ((nb ? NB1 : NAB) & 0xFFFF0000u) : NAB;
        const int beta = (i + 1) * b;
        uint32_t h1 = i == w ? pk_dup(-(O.o_del + O.e_del * (i + 1)) + beta) : NEG;
        uint32_t f = NEG;
        const int se = (2 * w + 1 < qlen - i + w) ? 2 * w + 1 : qlen - i + w;   // slot of column end
        const int lo = w - i - 2;                                                 // slot of column -2
        const int cse = se >> 3;
        PkDir *zi = z + (long)i * npair * ZS;
        uint32_t hl = 0u, px = 0u, py = 0u;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c * CH > se || (c + 1) * CH - 1 < lo) continue;   // dead chunk (wave-uniform)
            PK_BRANCH_BARRIER();
            uint32_t ax = 0u, ay = 0u;
#pragma unroll
            for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s) {
                const uint32_t Hd = s + 1 < NS ? RH[s + 1] : NEG;
                const uint32_t e0 = s + 1 < NS ? RE[s + 1] : NEG;
                const uint32_t mm = pk_asr15(pk_shl(G[s >> 4], 15 - (s & 15)));
                const uint32_t M = pk_mad(mm, NABr, Hd);
                const uint32_t hme = pk_max(M, e0);
                const uint32_t h = pk_max(hme, f);
                const uint32_t D1 = pk_sub(M, e0);
                const uint32_t D2 = pk_sub(hme, f);
                const uint32_t Ep = pk_sub(e0, cE);
                const uint32_t t1 = pk_sub(M, cT1);
                RE[s] = pk_max(Ep, t1);
                const uint32_t D3 = pk_sub(D1, cD3);
                const uint32_t Fp = pk_sub(f, cF);
                const uint32_t t2 = pk_sub(M, cT2);
                f = pk_max(Fp, t2);
                const uint32_t D4 = pk_sub(t2, Fp);
                RH[s] = h1;
                h1 = h;
                const uint32_t bit = 0x01010101u << (s - c * CH);
                ax = bfi_b32(bit, perm_b32(D2, D1, 0x0B0A0908u), ax);
                ay = bfi_b32(bit, perm_b32(D4, D3, 0x0B0A0908u), ay);
            }
            // (rows past both of the lane's tasks are never walked: no store)
            if (c & 1) {
                if (!(O.debug & 2) && i < tmax) zi[(c >> 1) * ZS] = pk_dir_enc(px, py, ax, ay);
            } else if (c == cse || c + 1 == NCH) {
                if (!(O.debug & 2) && i < tmax) zi[(c >> 1) * ZS] = pk_dir_enc(ax, ay, 0u, 0u);
            } else {
                px = ax, py = ay;
            }
            // eh[end]: E = NEG; its H (= H(i, end-1)) is the score once end == qlen.  A real
            // (wave-uniform) branch: the 8 selects run in one chunk per row, not in all.
            if (c == cse) {
                PK_BRANCH_BARRIER();
#pragma unroll
                for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s)
                    if (s == se) {
                        RE[s] = NEG;
                        hl = RH[s];
                    }
            }
        }
        if (i == A.tlen - 1) hlA = (int)(int16_t)(hl & 0xFFFFu) - beta;
        if (i == B.tlen - 1) hlB = (int)(int16_t)(hl >> 16) - beta;
    }
    scA = hlA;
    scB = hlB;
}


// ---------------------------------------------------------------------------
// ksw_extend2 for two tasks per lane in packed 16-bit arithmetic.
//
// Same slot scheme as glob_pk (slot s of row i = query column i - w + s; the
// 64 lanes of a wave share qlen and w).  Left edge: negative columns and the
// columns that the band pruning drops on the left hold zero words, which the
// DP keeps at zero (no select, no effect on the row maximum); ksw_extend2's
// first-column H(i,-1) = max(h0 - oe_del - e_del*i, 0) only ever enters as the
// H part of column 0's word, written by a per-row fixup at the (wave-uniform)
// slot of column 0 while i <= w.  Right edge, per
// task: slot se = end - i + w.  Cells at s >= se are dead: the end word gets
// E = 0 (eh[end] = {h1, 0}) and words above it are carried down unchanged
// (ksw_extend2 reads such stale words when the pruned end grows again), with
// the masks GE_s = [s >= se] (per half, from a sign) and GT_s = GE_{s-1}.
// Row maximum and its last column: per 16-slot group the packed max of
// h * 16 + (s & 15) (h <= 2047 for the routed tasks).  Pruned end: the last
// word eh[j] != 0 is one past the last column with H > 0 (E(i+1,j) > 0 implies
// H(i,j) > 0), tracked as a packed max of [h > 0] * (s + 1).
// Reference N rows are scored as bwa does (-1 a cell); tasks whose query holds an N are flagged
// by the caller for the exact kernel.
struct PkExtHalf {
    const uint8_t *T;   // first reference base of the side's window
    int ts;             // +1 / -1: reference step
    bool comp;          // reverse strand: complement the reference bases
    int tlen;           // rows (0 = empty half)
    int h0;             // start score
};
struct PkExtOut {
    int score, qle, tle, gtle, gscore, max_off;
};


// SMALLH (every H <= 511: a x read length <= 511): the row maximum and its last slot as one
// packed unsigned max of h * 128 + s instead of one h * 16 + (s & 15) per 16-slot group (one
// accumulator, no per-row reduction over the groups)
template <int WB, bool SMALLH = false>
SW_RING_FN void ext_pk(const PkExtHalf &A, const PkExtHalf &B, int qlen, int w, int nrows, const SwOptsDev &O,
                       const uint32_t *mA, const uint32_t *mB, int MS, PkExtOut out[2], int &nflag) {
    constexpr int NS = 2 * WB + 2;
    constexpr int CH = 8;
    constexpr int NCH = (NS + CH - 1) / CH;
    constexpr int NG = SMALLH ? 1 : (NS + 15) / 16;
    static_assert(!SMALLH || NS <= 128, "slot index in 7 bits");
    const int b = O.b, oe_del = O.o_del + O.e_del, oe_ins = O.o_ins + O.e_ins;
    const uint32_t NAB = pk_dup(-(O.a + b)), BD = pk_dup(b);
    const uint32_t cOD = pk_dup(oe_del), cED = pk_dup(O.e_del), cOI = pk_dup(oe_ins), cEI = pk_dup(O.e_ins);
    const PkExtHalf *Hh[2] = {&A, &B};
    uint32_t RH[NS], RE[NS];
    {
        int h1v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int h0 = Hh[h]->h0;
            h1v[h] = h0 > oe_ins ? h0 - oe_ins : 0;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int c = s - w - 1;
            int hv[2] = {0, 0}, ev[2] = {0, 0};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (c == 0) hv[h] = Hh[h]->h0;
                else if (c > 0 && c <= qlen) {
                    const int v = h1v[h] - O.e_ins * (c - 1);
                    hv[h] = v > 0 ? v : 0;
                }
            }
            RH[s] = (uint32_t)(uint16_t)hv[0] | ((uint32_t)(uint16_t)hv[1] << 16);
            RE[s] = (uint32_t)(uint16_t)ev[0] | ((uint32_t)(uint16_t)ev[1] << 16);
        }
    }
    int end[2] = {qlen, qlen}, mx[2], max_i[2] = {-1, -1}, max_j[2] = {-1, -1}, max_ie[2] = {-1, -1};
    int gscore[2] = {-1, -1}, max_off[2] = {0, 0};
    bool live[2];
#ifndef PK_EXT_TW
#define PK_EXT_TW 4   // reference window of the extension: 4 dwords (16 rows) or 2 (8 rows)
#endif
    constexpr int TW = PK_EXT_TW, TROWS = 4 * TW;
    uint32_t tw[2][TW];   // reference window: byte 0 = row i
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        mx[h] = Hh[h]->h0;
        live[h] = Hh[h]->tlen > 0;
#pragma unroll
        for (int x = 0; x < TW; ++x) tw[h][x] = 0u;
        if (live[h]) {
            if constexpr (TW == 4) pk_tref16(Hh[h]->T, Hh[h]->ts, 0, tw[h]);
            else pk_tref8(Hh[h]->T, Hh[h]->ts, 0, tw[h]);
        }
    }
    for (int i = 0; i < nrows; ++i) {
        int cb[2];
        bool rn[2];
        uint32_t sev = 0u, bnd = 0u;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int c = (int)(tw[h][0] & 0xFFu);
            if ((i & (TROWS - 1)) == TROWS - 1) {   // (wave-uniform)
                if (i + 1 < Hh[h]->tlen) {
                    if constexpr (TW == 4) pk_tref16(Hh[h]->T, Hh[h]->ts, i + 1, tw[h]);
                    else pk_tref8(Hh[h]->T, Hh[h]->ts, i + 1, tw[h]);
                }
            } else {
                if constexpr (TW == 4) pk_shr8(tw[h]);
                else pk_shr8_2(tw[h]);
            }
            if (Hh[h]->comp && c < 4) c = 3 - c;
            if (live[h] && i >= Hh[h]->tlen) live[h] = false;
            rn[h] = c > 3;   // a reference N row: -1 in every column (below)
            cb[h] = c & 3;
            if (end[h] > i + w + 1) end[h] = i + w + 1;
            if (end[h] > qlen) end[h] = qlen;
            sev |= (uint32_t)(uint16_t)(end[h] - i + w - 1) << (16 * h);   // se - 1
            int bd = Hh[h]->h0 - (O.o_del + O.e_del * (i + 1));
            bnd |= (uint32_t)(uint16_t)(bd > 0 ? bd : 0) << (16 * h);
        }
        uint32_t wa[3], wb[3], G[6];
        pk_window(mA, MS, i - w + 64, cb[0], wa);
        pk_window(mB, MS, i - w + 64, cb[1], wb);
        // a reference N row (bwa_fill_scmat: -1 against every query base): no match bits and the
        // mismatch step 1 instead of b for that half -- M = max(Hd - 1, 0) where Hd > 0
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            wa[g] = rn[0] ? 0u : wa[g];
            wb[g] = rn[1] ? 0u : wb[g];
            G[2 * g] = perm_b32(wb[g], wa[g], 0x05040100u);
            G[2 * g + 1] = perm_b32(wb[g], wa[g], 0x07060302u);
        }
        const uint32_t BDr = (rn[0] || rn[1]) ? ((rn[0] ? 1u : BD & 0xFFFFu) | (rn[1] ? 0x10000u : BD & 0xFFFF0000u)) : BD;
        // the column entering at the top slot still holds its row -1 word (H only)
        uint32_t qin = 0u;
        {
            const int cin = i - w + NS;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int v = 0;
                if (cin == 0) v = Hh[h]->h0;
                else if (cin > 0 && cin <= qlen) {
                    const int h0 = Hh[h]->h0;
                    v = (h0 > oe_ins ? h0 - oe_ins : 0) - O.e_ins * (cin - 1);
                    v = v > 0 ? v : 0;
                }
                qin |= (uint32_t)(uint16_t)v << (16 * h);
            }
        }
        uint32_t h1 = 0u, f = 0u, gt = 0u, lp = 0u;
        uint32_t gm[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) gm[g] = 0u;
        const int stop = qlen - i + w;   // slot of column qlen (wave-uniform)
        const int sbl = w - i;           // slot of column 0 (wave-uniform)
        const int lo = w - i - 2;        // slot of column -2
        uint32_t hl = 0u;
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            if (c * CH > stop || (c + 1) * CH - 1 < lo) continue;   // dead chunk (wave-uniform)
            PK_BRANCH_BARRIER();
#pragma unroll
            for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s) {
                const uint32_t Hd = s + 1 < NS ? RH[s + 1] : qin;
                const uint32_t e0 = s + 1 < NS ? RE[s + 1] : 0u;
                const uint32_t mm = pk_asr15(pk_shl(G[s >> 4], 15 - (s & 15)));
                // M = H(i-1,j-1) ? H(i-1,j-1) + S : 0, clamped at 0 (a negative M acts as 0 in
                // every use: h = max(M, e, f) with e, f >= 0, and the gap openings max(M - oe, 0)),
                // so the unsigned saturating subtracts replace the max-with-0 steps
                const uint32_t M = pk_min(pk_shl(Hd, 4), pk_subs(pk_mad(mm, NAB, Hd), BDr));
                const uint32_t h = pk_max(pk_max(M, e0), f);
                const uint32_t en = pk_max(pk_subs(e0, cED), pk_subs(M, cOD));
                const uint32_t fn = pk_max(pk_subs(f, cEI), pk_subs(M, cOI));
                const uint32_t ge = perm_b32(0u, pk_sub(sev, pk_dup(s)), 0x09090808u);   // s >= se
                RH[s] = bfi_b32v(gt, Hd, h1);
                RE[s] = bfi_b32v(gt, e0, bfi_b32v(ge, 0u, en));
                const uint32_t hm = bfi_b32v(ge, 0u, h);
                if (SMALLH) gm[0] = pk_maxu(gm[0], pk_mad(hm, pk_dup(128), pk_dup(s)));
                else gm[s >> 4] = pk_max(gm[s >> 4], pk_mad(hm, pk_dup(16), pk_dup(s & 15)));
                lp = pk_max(lp, pk_mad(pk_min(hm, pk_dup(1)), pk_dup(s + 1), 0u));
                h1 = h;
                f = fn;
                gt = ge;
            }
            if (c == (sbl >> 3) && sbl >= 0) {   // column 0's word: H(i,-1), the first-column score
                PK_BRANCH_BARRIER();
#pragma unroll
                for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s)
                    if (s == sbl) RH[s] = bnd;
            }
            if (c == (stop >> 3)) {   // eh[qlen].h = H(i, qlen-1) when the band reaches the query end
                PK_BRANCH_BARRIER();
#pragma unroll
                for (int s = c * CH; s < (c + 1) * CH && s < NS; ++s)
                    if (s == stop) hl = RH[s];
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!live[h]) continue;
            if (end[h] == qlen) {
                const int v = (int)((hl >> (16 * h)) & 0xFFFFu);
                max_ie[h] = gscore[h] > v ? max_ie[h] : i;
                gscore[h] = gscore[h] > v ? gscore[h] : v;
            }
            int best = -1;
            if (SMALLH) {
                const int kv = (int)((gm[0] >> (16 * h)) & 0xFFFFu);
                best = ((kv >> 7) << 8) | (kv & 127);
            } else {
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const int kv = (int)((gm[g] >> (16 * h)) & 0xFFFFu);
                    const int cand = ((kv >> 4) << 8) | (g * 16 + (kv & 15));
                    best = best > cand ? best : cand;
                }
            }
            const int m = best >> 8;
            if (m == 0) {
                live[h] = false;
                continue;
            }
            const int mj = i - w + (best & 255);
            if (m > mx[h]) {
                mx[h] = m, max_i[h] = i, max_j[h] = mj;
                const int d = mj - i < 0 ? i - mj : mj - i;
                max_off[h] = max_off[h] > d ? max_off[h] : d;
            } else if (O.zdrop > 0) {
                if (i - max_i[h] > mj - max_j[h]) {
                    if (mx[h] - m - ((i - max_i[h]) - (mj - max_j[h])) * O.e_del > O.zdrop) { live[h] = false; continue; }
                } else {
                    if (mx[h] - m - ((mj - max_j[h]) - (i - max_i[h])) * O.e_ins > O.zdrop) { live[h] = false; continue; }
                }
            }
            const int jl = i - w + (int)((lp >> (16 * h)) & 0xFFFFu);   // last column whose word is non-zero
            end[h] = jl + 2 < qlen ? jl + 2 : qlen;
        }
        if (!SW_RING_ANY(live[0] || live[1])) break;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        out[h].score = mx[h];
        out[h].qle = max_j[h] + 1;
        out[h].tle = max_i[h] + 1;
        out[h].gtle = max_ie[h] + 1;
        out[h].gscore = gscore[h];
        out[h].max_off = max_off[h];
    }
}

// direction nibble (D1 | D2 << 1 | D3 << 2 | D4 << 3) of half hb at (row i, slot s)
SW_RING_FN int pk_nib(const PkDir &v, int s, int hb) {
    uint32_t d1, d2, d3, d4;
    pk_dir_dec(v, d1, d2, d3, d4);
    const int bt = (s & 7) + 8 * hb + ((s & 8) ? 16 : 0);
    return (int)(((d1 >> bt) & 1u) | (((d2 >> bt) & 1u) << 1) | (((d3 >> bt) & 1u) << 2) | (((d4 >> bt) & 1u) << 3));
}
// ksw_global2's state step: h source (M 0, E 1, F 2) from state 0, continue bits otherwise
SW_RING_FN int pk_which(int which, int nib) {
    if (which == 0) return (nib & 2) ? 2 : (nib & 1);
    if (which == 1) return (nib >> 2) & 1;
    return ((nib >> 3) & 1) * 2;
}

// ksw_global2's backtrack for half `hb` (0 = A, 1 = B) over glob_pk's direction
// words: ops (0 M, 1 I, 2 D) pushed in reverse order; returns the count or -1.
SW_RING_FN int glob_pk_backtrack(const PkDir *z, int ZS, int npair, int hb, int tlen, int qlen, int w, uint32_t *cg,
                                 int maxcig) {
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
        const int s = k - i + w;
        which = pk_which(which, pk_nib(z[((long)i * npair + (s >> 4)) * ZS], s, hb));
        if (which == 0) push(0, 1), --i, --k;
        else if (which == 1) push(2, 1), --i;
        else push(1, 1), --k;
    }
    if (n >= 0 && i >= 0) push(2, i + 1);
    if (n >= 0 && k >= 0) push(1, k + 1);
    return n;
}

// Backtrack of both halves of a lane (glob_pk_backtrack's walk; the plain
// version above is its reference), in row lockstep across the wave: every
// walk leaves a row only by an M or D step, so all lanes can sweep the rows
// together from the wave's last row down.  Windows of WIN rows (8 in the fused kernel) are loaded at
// each half's current 16-slot pair (the walks hug the band centre, so the 64
// lanes mostly read the same pair: the loads are coalesced rows of the
// [row][pair][lane] slab), the half's direction bytes are picked out with
// v_perm_b32 into registers (wave-uniform row index: static register
// indexing); a step whose slot left the loaded pair reads its word directly.
// The current op run stays in registers and every finished run is stored once,
// from the END of the task's CIGAR slots backwards: the ops land in final
// (forward) order at cg[h][maxcig[h] - n, maxcig[h]).  n[h] = op count or -1 (more
// than maxcig[h]); first[h] / last[h] = the first / last op of the forward CIGAR.
template <int WIN = 16>
SW_RING_FN void pk_backtrack2(const PkDir *zl, int ZS, int npair, int nrows, const int tl[2], int qlen, int w,
                              uint32_t *const cg[2], int n[2], uint32_t first[2], uint32_t last[2],
                              const int maxcig[2], unsigned *stat = nullptr) {
    int i[2], k[2], which[2] = {0, 0}, rop[2] = {-1, -1}, rln[2] = {0, 0};
    bool live[2];
    auto flush = [&](int h) {
        const uint32_t v = ((uint32_t)rln[h] << 4) | (uint32_t)rop[h];
        if (n[h] == 0) last[h] = v;
        first[h] = v;
        cg[h][maxcig[h] - 1 - n[h]++] = v;
    };
    // ksw's push with the last op kept in registers: false when the op count would exceed maxcig
    auto push = [&](int h, int op, int len) -> bool {
        if (op == rop[h]) {
            rln[h] += len;
            return true;
        }
        if (rop[h] >= 0) {
            if (n[h] + 1 >= maxcig[h]) return false;
            flush(h);
        }
        rop[h] = op;
        rln[h] = len;
        return true;
    };
    // the half's direction bytes of a (row, pair) word: x = D1|D2 of both chunks, y = D3|D4
    auto pick = [&](const PkDir &v, int h, uint32_t &x, uint32_t &y) {
        uint32_t d1, d2, d3, d4;
        pk_dir_dec(v, d1, d2, d3, d4);
        const uint32_t sel = h ? 0x07030501u : 0x06020400u;
        x = perm_b32(d2, d1, sel);
        y = perm_b32(d4, d3, sel);
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        i[h] = tl[h] - 1;
        k[h] = (i[h] + w + 1 < qlen ? i[h] + w + 1 : qlen) - 1;
        n[h] = 0;
        first[h] = last[h] = 0u;
        live[h] = cg[h] != nullptr && i[h] >= 0 && k[h] >= 0;
    }
    for (int R = nrows - 1; R >= 0 && SW_RING_ANY(live[0] || live[1]); R -= WIN) {
        uint32_t bx[2][WIN], by[2][WIN];
        int p[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            p[h] = (k[h] - i[h] + w) >> 4;
            PkDir v[WIN];
#pragma unroll
            for (int d = 0; d < WIN; ++d) {
                v[d] = PkDir{0u, 0u, 0u};
                if (live[h] && R - d >= 0 && R - d <= i[h]) {
                    const long ix = ((long)(R - d) * npair + p[h]) * ZS;
                    PK_ZCHECK(ix);
                    v[d] = zl[ix];
                }
            }
#pragma unroll
            for (int d = 0; d < WIN; ++d) pick(v[d], h, bx[h][d], by[h][d]);
        }
#pragma unroll
        for (int d = 0; d < WIN; ++d) {
            const int r = R - d;
            // one loop for both halves: an iteration steps every half still on row r
            for (;;) {
                const bool go[2] = {live[0] && i[0] == r, live[1] && i[1] == r};
                if (!SW_RING_ANY(go[0] || go[1])) break;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (!go[h]) continue;
                    const int sl = k[h] - r + w;
                    uint32_t X = bx[h][d], Y = by[h][d];
                    if ((sl >> 4) != p[h]) {
                        const long ix = ((long)r * npair + (sl >> 4)) * ZS;
                        PK_ZCHECK(ix);
                        pick(zl[ix], h, X, Y);
                        if (stat) ++stat[0];
                    }
                    if (stat) ++stat[1];
                    const int bt = ((sl >> 3) & 1) * 16 + (sl & 7);
                    // the step, branch-free apart from the stores (round 3: the nested push /
                    // move branches cost ~280 instructions per step, most of them exec-mask
                    // bookkeeping): pk_which on the slot's bits (a: D1 at bit 0, D2 at bit 8;
                    // b: D3, D4), then an I step takes the F-continuations below it in the
                    // loaded pair along (one per D4 bit set, ksw's F state); the first D4 = 0
                    // ends the run with the M step of ksw's F -> M transition, unless the query
                    // column runs out first
                    // which = 0 reads D1 (bit 0) / D2 (bit 8) of X, which = 1 D3 (bit 0) and
                    // which = 2 D4 (bit 8) of Y: D2 or D4 -> 2 (unless which = 1), else D1 or D3
                    // (unless which = 2)
                    const uint32_t u = (which[h] == 0 ? X : Y) >> bt;
                    const bool s2 = (u & 0x100u) != 0u && which[h] != 1;
                    const bool s1 = (u & 1u) != 0u && which[h] != 2;
                    const int wn = s2 ? 2 : (s1 ? 1 : 0);
                    const int j = sl & 15;
                    const uint32_t d4 = perm_b32(0u, Y, 0x0C0C0301u);   // D4 bytes of both chunks
                    const uint32_t zeros = ~d4 & ((1u << j) - 1u);
                    const int m = zeros ? j - 1 - (31 - __builtin_clz(zeros | 1u)) : j;   // ones below sl
                    const int mi = m < k[h] ? m : k[h];
                    const bool isI = wn == 2;
                    const int len = isI ? 1 + mi : 1;
                    const bool mstep = isI && zeros != 0u && mi == m && k[h] - len >= 0;
                    const int op = (int)((0x18u >> (2 * wn)) & 3u);   // M, D, I for which = 0, 1, 2
                    // push(op, len), then (mstep) push(M, 1), which always closes the I run
                    const bool same = op == rop[h];
                    const bool fl1 = !same && rop[h] >= 0;
                    const uint32_t v1 = ((uint32_t)rln[h] << 4) | (uint32_t)rop[h];
                    const int ra = same ? rln[h] + len : len;
                    const uint32_t v2 = ((uint32_t)ra << 4) | 1u;
                    const int n0 = n[h], n1 = n0 + (int)fl1, n2 = n1 + (int)mstep;
                    // a flush needs n + 1 < maxcig; n0 < maxcig always holds, so the pushes fail
                    // exactly when the count after them reaches maxcig
                    const bool fail = n2 >= maxcig[h];
                    if (fl1 && !fail) cg[h][(uint32_t)(maxcig[h] - 1 - n0)] = v1;   // (unsigned: no sign extension)
                    if (mstep && !fail) cg[h][(uint32_t)(maxcig[h] - 1 - n1)] = v2;
                    last[h] = (fl1 && n0 == 0) ? v1 : ((mstep && n1 == 0) ? v2 : last[h]);
                    first[h] = mstep ? v2 : (fl1 ? v1 : first[h]);
                    n[h] = fail ? -1 : n2;
                    rop[h] = mstep ? 0 : op;
                    rln[h] = mstep ? 1 : ra;
                    which[h] = mstep ? 0 : wn;
                    i[h] -= (int)!isI + (int)mstep;
                    k[h] -= (isI ? len : (int)(wn == 0)) + (int)mstep;
                    live[h] = !fail && i[h] >= 0 && k[h] >= 0;
                }
            }
        }
    }
    // leading D / I remainders (ksw's pushes after the walk), then the last run
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (cg[h] == nullptr || n[h] < 0) continue;
        bool ok = true;
        if (i[h] >= 0) ok = push(h, 2, i[h] + 1);
        if (ok && k[h] >= 0) ok = push(h, 1, k[h] + 1);
        if (!ok) n[h] = -1;
        else if (rop[h] >= 0) flush(h);
    }
}

// Forward copy of n ops from cg[src] to cg[dst] (dst <= src), 8 independent loads at a time.
SW_RING_FN void pk_cig_move(uint32_t *cg, int dst, int src, int n) {
    for (int x = 0; x < n; x += 8) {
        uint32_t v[8];
#pragma unroll
        for (int y = 0; y < 8; ++y) v[y] = x + y < n ? cg[src + x + y] : 0u;
#pragma unroll
        for (int y = 0; y < 8; ++y)
            if (x + y < n) cg[dst + x + y] = v[y];
    }
}

}  // namespace prgpu
