// Host build of the masking core (proovread_amd/csrc/mask_core.h) for the tests:
// the device kernel's flow with the wave ballot emulated (one 64-bit in-range
// bitmap per 64 columns), then the scalar resolve.
#include <stdint.h>
#include <vector>

#include "../../proovread_amd/csrc/mask_core.h"

using namespace prgpu;

extern "C" int mask_host(const uint8_t *qual, int64_t L, int lo, int hi, int lcs_min, int hcr_min, int lcr_min,
                         int sticky, double end_ratio, int32_t *found, int64_t *n_found, int32_t *mcr,
                         int64_t *n_mcr) {
    MaskCfg c{lo, hi, lcs_min, hcr_min, lcr_min, sticky, end_ratio};
    const int64_t cap = mask_run_cap(L, lcs_min);
    std::vector<MaskRun> h(cap), tmp(cap);
    int64_t n = 0, run = -1;
    for (int64_t base = 0; base < L; base += 64) {
        const int valid = (int)(L - base < 64 ? L - base : 64);
        uint64_t bits = 0;
        for (int l = 0; l < valid; ++l) {
            const int q = qual[base + l];
            if (q >= lo && q <= hi) bits |= 1ull << l;
        }
        mask_runs_feed(bits, base, valid, run, lcs_min, h.data(), n, cap);
    }
    mask_runs_close(L, run, lcs_min, h.data(), n, cap);
    if (n > cap) return -1;
    for (int64_t i = 0; i < n; ++i) {
        found[2 * i] = h[i].off;
        found[2 * i + 1] = h[i].len;
    }
    *n_found = n;
    const int64_t m = mask_resolve(h.data(), n, L, c, tmp.data());
    for (int64_t i = 0; i < m; ++i) {
        mcr[2 * i] = h[i].off;
        mcr[2 * i + 1] = h[i].len;
    }
    *n_mcr = m;
    return 0;
}
