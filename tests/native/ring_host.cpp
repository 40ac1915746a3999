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
