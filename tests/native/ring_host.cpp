// Host build of the register-ring ksw_extend2 (proovread_amd/csrc/sw_ring.h) for
// the CPU test suite: one lane of the GPU kernel, checked against the oracle
// (oracle/sw_oracle.c osw_extend) on random and edge-case inputs.
#define SW_RING_HOST 1
#include "../../proovread_amd/csrc/sw_ring.h"

using namespace prgpu;

extern "C" int ring_extend(int wb, int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop,
                           int qlen, const uint8_t *q, int tlen, const uint8_t *t, int w, int end_bonus,
                           int h0, int *out5) {
    SwOptsDev O{};
    O.a = a; O.b = b; O.o_del = o_del; O.e_del = e_del; O.o_ins = o_ins; O.e_ins = e_ins; O.zdrop = zdrop;
    ExtIO io{};
    int sc;
    switch (wb) {
        case 32: sc = ext_ring<32>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, end_bonus, h0, io); break;
        case 40: sc = ext_ring<40>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, end_bonus, h0, io); break;
        case 64: sc = ext_ring<64>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, end_bonus, h0, io); break;
        case 80: sc = ext_ring<80>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, end_bonus, h0, io); break;
        default: return -12345;
    }
    out5[0] = io.qle; out5[1] = io.tle; out5[2] = io.gtle; out5[3] = io.gscore; out5[4] = io.max_off;
    return sc;
}

// ksw_global2 + backtrack (register ring); cigar in bwa's order (reversed back)
extern "C" int ring_global(int wb, int a, int b, int o_del, int e_del, int o_ins, int e_ins, int qlen,
                           const uint8_t *q, int tlen, const uint8_t *t, int w, int *n_cigar, uint32_t *cigar,
                           int max_cigar) {
    SwOptsDev O{};
    O.a = a; O.b = b; O.o_del = o_del; O.e_del = e_del; O.o_ins = o_ins; O.e_ins = e_ins;
    const int NW = (2 * wb + 2 + 7) / 8;
    uint32_t *z = new uint32_t[(size_t)(tlen + 1) * NW + 1]();
    int sc = 0, n = 0;
    switch (wb) {
        case 40:
            sc = glob_ring<40>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, z, 1);
            n = glob_backtrack<40>(z, 1, tlen, qlen, w, cigar, max_cigar);
            break;
        case 80:
            sc = glob_ring<80>(q, 0, 1, qlen, t, 0, 1, false, tlen, O, w, z, 1);
            n = glob_backtrack<80>(z, 1, tlen, qlen, w, cigar, max_cigar);
            break;
        default: delete[] z; return -12345;
    }
    delete[] z;
    if (n > 0)
        for (int x = 0; x < n / 2; ++x) { uint32_t tmp = cigar[x]; cigar[x] = cigar[n - 1 - x]; cigar[n - 1 - x] = tmp; }
    *n_cigar = n;
    return sc;
}

// ksw_global2 + backtrack for a lane pair in the packed kernel's arithmetic
// (proovread_amd/csrc/sw_pk.h): two tasks with the same query length and band,
// their own queries/targets; scores to sc[2], CIGARs (bwa order) to cig[h * max_cigar ..].
#include <algorithm>
#include <vector>
#include "../../proovread_amd/csrc/sw_pk.h"
namespace prgpu { long pk_host_zlen = 0; }
extern "C" int pk_global(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int qlen, int w,
                         const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb, const uint8_t *tb,
                         int *sc, int *ncig, uint32_t *cig, int max_cigar, int nrow_min) {
    SwOptsDev O{};
    O.a = a; O.b = b; O.o_del = o_del; O.e_del = e_del; O.o_ins = o_ins; O.e_ins = e_ins;
    uint32_t m[2][2 * PK_NQW];
    int qn = 0;
    if (pk_build_mask(qa, 0, 1, tla >= 0 ? qlen : 0, m[0], 1)) qn |= 1;
    if (pk_build_mask(qb, 0, 1, tlb >= 0 ? qlen : 0, m[1], 1)) qn |= 2;
    // the kernel reads 16-byte reference windows past the window's end: padded copies
    std::vector<uint8_t> pa((tla > 0 ? tla : 0) + 64, 4), pb((tlb > 0 ? tlb : 0) + 64, 4);
    if (tla > 0) std::copy(ta, ta + tla, pa.begin());
    if (tlb > 0) std::copy(tb, tb + tlb, pb.begin());
    PkHalf A{pa.data(), tla > 0 ? tla : 0, false}, B{pb.data(), tlb > 0 ? tlb : 0, false};
    int nrow = A.tlen > B.tlen ? A.tlen : B.tlen;
    if (nrow < nrow_min) nrow = nrow_min;   // other lanes of the wave may run longer
    const int npair = pk_npair(w);
    PkDir *z = new PkDir[(size_t)(nrow + 1) * npair + 1]();
    pk_host_zlen = (long)nrow * npair;   // rows [0, nrow) x pairs
    int s2[2] = {0, 0}, nflag = 0;
    glob_pk<40>(A, B, qlen, w, nrow, O, m[0], m[1], 1, z, 1, s2[0], s2[1], nflag);
    // the kernel's windowed two-half backtrack, checked against the plain one
    const int tl2[2] = {A.tlen, B.tlen};
    uint32_t *cg2[2] = {A.tlen > 0 ? cig : nullptr, B.tlen > 0 ? cig + max_cigar : nullptr};
    int n2[2] = {0, 0};
    uint32_t fst[2], lst[2];
    const int caps[2] = {max_cigar, max_cigar};
    pk_backtrack2(z, 1, npair, nrow, tl2, qlen, w, cg2, n2, fst, lst, caps);
    for (int h = 0; h < 2; ++h)   // forward order at the slots' end -> reverse order at the start (plain walk's)
        if (cg2[h] && n2[h] > 0) {
            if (fst[h] != cg2[h][max_cigar - n2[h]] || lst[h] != cg2[h][max_cigar - 1]) { delete[] z; return -2000 - h; }
            pk_cig_move(cg2[h], 0, max_cigar - n2[h], n2[h]);
            std::reverse(cg2[h], cg2[h] + n2[h]);
        }
    for (int h = 0; h < 2; ++h) {
        const int tl = h ? B.tlen : A.tlen;
        uint32_t *cg = cig + (size_t)h * max_cigar;
        std::vector<uint32_t> ref(max_cigar + 1);
        int n = tl > 0 ? glob_pk_backtrack(z, 1, npair, h, tl, qlen, w, ref.data(), max_cigar) : 0;
        if (tl > 0 && (n != n2[h] || (n > 0 && !std::equal(ref.begin(), ref.begin() + n, cg)))) {
            delete[] z;
            return -1000 - h;   // windowed walk disagrees with the plain walk
        }
        if (n > 0)
            for (int x = 0; x < n / 2; ++x) { uint32_t t = cg[x]; cg[x] = cg[n - 1 - x]; cg[n - 1 - x] = t; }
        ncig[h] = n;
        sc[h] = s2[h];
    }
    delete[] z;
    return nflag | (qn << 2);
}

// ksw_extend2 for a lane pair in the packed kernel's arithmetic (sw_pk.h ext_pk):
// two tasks with the same query length and band; out[12] = (score, qle, tle, gtle,
// gscore, max_off) per half; returns the N flags.
template <bool SMALLH>
static int pk_extend_t(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop, int qlen, int w,
                       const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb,
                       const uint8_t *tb, int h0a, int h0b, int nrow_min, int *out) {
    SwOptsDev O{};
    O.a = a; O.b = b; O.o_del = o_del; O.e_del = e_del; O.o_ins = o_ins; O.e_ins = e_ins; O.zdrop = zdrop;
    uint32_t m[2][2 * PK_NQW];
    int nflag = 0;
    if (pk_build_mask(qa, 0, 1, qlen, m[0], 1)) nflag |= 4;
    if (pk_build_mask(qb, 0, 1, qlen, m[1], 1)) nflag |= 8;
    // the kernel reads 16-byte reference windows past the read's end: padded copies
    std::vector<uint8_t> pa(tla + 64, 4), pb(tlb + 64, 4);
    std::copy(ta, ta + tla, pa.begin());
    std::copy(tb, tb + tlb, pb.begin());
    PkExtHalf A{pa.data(), 1, false, tla, h0a}, B{pb.data(), 1, false, tlb, h0b};
    int nrow = tla > tlb ? tla : tlb;
    if (nrow < nrow_min) nrow = nrow_min;
    PkExtOut o[2];
    ext_pk<40, SMALLH>(A, B, qlen, w, nrow, O, m[0], m[1], 1, o, nflag);
    for (int h = 0; h < 2; ++h) {
        out[6 * h + 0] = o[h].score; out[6 * h + 1] = o[h].qle; out[6 * h + 2] = o[h].tle;
        out[6 * h + 3] = o[h].gtle; out[6 * h + 4] = o[h].gscore; out[6 * h + 5] = o[h].max_off;
    }
    return nflag;
}
// the same pair with both references walked backwards (ts = -1), as the kernel reads a reverse-strand
// window: each target stored reversed behind 64 bytes of front slack (SB_LR_FRONT), T at its last
// byte, so row r is T[-r] = the target's base r; the 16- / 8-byte windows load T - r - 15 (- 7)
static int pk_extend_rev_t(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop, int qlen, int w,
                           const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb,
                           const uint8_t *tb, int h0a, int h0b, int nrow_min, int *out) {
    SwOptsDev O{};
    O.a = a; O.b = b; O.o_del = o_del; O.e_del = e_del; O.o_ins = o_ins; O.e_ins = e_ins; O.zdrop = zdrop;
    uint32_t m[2][2 * PK_NQW];
    int nflag = 0;
    if (pk_build_mask(qa, 0, 1, qlen, m[0], 1)) nflag |= 4;
    if (pk_build_mask(qb, 0, 1, qlen, m[1], 1)) nflag |= 8;
    std::vector<uint8_t> pa(64 + tla + 64, 4), pb(64 + tlb + 64, 4);
    for (int r = 0; r < tla; ++r) pa[64 + tla - 1 - r] = ta[r];
    for (int r = 0; r < tlb; ++r) pb[64 + tlb - 1 - r] = tb[r];
    PkExtHalf A{pa.data() + 64 + tla - 1, -1, false, tla, h0a}, B{pb.data() + 64 + tlb - 1, -1, false, tlb, h0b};
    int nrow = tla > tlb ? tla : tlb;
    if (nrow < nrow_min) nrow = nrow_min;
    PkExtOut o[2];
    ext_pk<40, false>(A, B, qlen, w, nrow, O, m[0], m[1], 1, o, nflag);
    for (int h = 0; h < 2; ++h) {
        out[6 * h + 0] = o[h].score; out[6 * h + 1] = o[h].qle; out[6 * h + 2] = o[h].tle;
        out[6 * h + 3] = o[h].gtle; out[6 * h + 4] = o[h].gscore; out[6 * h + 5] = o[h].max_off;
    }
    return nflag;
}
extern "C" int pk_extend_rev(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop, int qlen, int w,
                             const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb,
                             const uint8_t *tb, int h0a, int h0b, int nrow_min, int *out) {
    return pk_extend_rev_t(a, b, o_del, e_del, o_ins, e_ins, zdrop, qlen, w, qa, qb, tla, ta, tlb, tb, h0a, h0b,
                           nrow_min, out);
}
extern "C" int pk_extend(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop, int qlen, int w,
                         const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb,
                         const uint8_t *tb, int h0a, int h0b, int nrow_min, int *out) {
    return pk_extend_t<false>(a, b, o_del, e_del, o_ins, e_ins, zdrop, qlen, w, qa, qb, tla, ta, tlb, tb, h0a, h0b,
                              nrow_min, out);
}
// the one-accumulator row maximum (every H <= 511)
extern "C" int pk_extend_small(int a, int b, int o_del, int e_del, int o_ins, int e_ins, int zdrop, int qlen, int w,
                               const uint8_t *qa, const uint8_t *qb, int tla, const uint8_t *ta, int tlb,
                               const uint8_t *tb, int h0a, int h0b, int nrow_min, int *out) {
    return pk_extend_t<true>(a, b, o_del, e_del, o_ins, e_ins, zdrop, qlen, w, qa, qb, tla, ta, tlb, tb, h0a, h0b,
                             nrow_min, out);
}
