// Device-side descriptor of the masking kernel (mask_kernels.hip).
#pragma once
#include <stdint.h>

#include "mask_core.h"

namespace prgpu {

struct MaskDev {
    int32_t n;                     // reads
    const int64_t *off;            // [n+1] read offsets into seq/qual/out (a capacity prefix is fine)
    const int32_t *len;            // [n] read lengths, or null: off[i+1] - off[i]
    const int32_t *status;         // [n] or null: reads with status != 0 are skipped (not counted)
    const uint8_t *seq, *qual;     // ASCII bases, phred+offset chars
    uint8_t *out;                  // masked bases (same layout as seq)
    const int64_t *run_off;        // [n+1] prefix of mask_run_cap(capacity, lcs_min)
    MaskRun *runs, *tmp;           // [run_off[n]] HCR lists (MCRs on return) and the resolve copy
    int32_t *n_runs;               // [n] MCR count, or null
    int32_t *err;                  // [1] set to 1 if a read's HCRs exceed its run capacity
    unsigned long long *stats;     // [2] bases, 'N' bases of the masked output (zeroed by the launch)
    MaskCfg cfg;
};

// Enqueue the masking of D.n reads on `stream` (hipStream_t).  Returns a hipError_t.
int mask_launch(const MaskDev &D, int n_cu, void *stream);

}  // namespace prgpu
