// Launch descriptor of the seeding kernel (seed_kernels.hip).
#pragma once
#include <stdint.h>

#include "seed_core.h"

namespace prgpu {

struct SeedDev {
    seedc::IndexView V;        // device pointers
    pr_seed_opts O;
    const uint8_t *sr_seq;     // nt4 codes (anything > 3 is N)
    const int64_t *sr_off;     // [n_sr + 1]
    int64_t n_sr;
    uint8_t *scratch;          // n_lanes * stride bytes
    int64_t stride;            // seedc::scratch_bytes(caps), 8-byte multiple
    int64_t n_lanes;
    seedc::Caps caps;
    pr_seed_task *out;         // [n_sr * caps.out]
    int32_t *n_out;            // [n_sr]
    int32_t *status;           // [n_sr] 0 or SC_OVER_* bits
};

int seed_launch(const SeedDev &D, void *stream);

// host-side view of a built index (seed.cpp)
seedc::IndexView seed_index_view(const pr_seed_index *h);
// sizes of the index arrays for the device copy
struct SeedIndexSizes {
    int64_t text, cstart, cblk, lr_off, koff, kpos, cnt[seedc::KI - 1];
};
SeedIndexSizes seed_index_sizes(const pr_seed_index *h);

}  // namespace prgpu
