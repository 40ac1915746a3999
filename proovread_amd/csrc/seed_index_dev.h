// Launch descriptor of the device seed-index build (seed_index.hip).  All pointers are
// device pointers; the host computes the small tables (contig starts, block table).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seed_core.h"

namespace prgpu {

struct SeedIndexBuild {
    const uint8_t *lr_seq;        // [l_pac] long-read codes (0-3 bases, anything else N)
    const int64_t *lr_off;        // [n_lr + 1] rebased to 0
    int n_lr;
    int64_t l_pac;
    const int64_t *cstart;        // [2 n_lr] text offset of every contig
    int64_t n_text;               // 2 l_pac + 2 n_lr
    uint8_t *text;                // [n_text]
    uint32_t *key0, *key1, *val0; // [n_text] sort scratch
    uint32_t *kc;                 // [NK + 1] 12-mer histogram (last entry 0)
    uint32_t *koff;               // [NK + 1]
    uint32_t *kpos;               // [n_text] sorted positions; the first koff[NK] are the hits
    uint64_t *kext;               // [n_text]; the first koff[NK] are written
    uint32_t *cnt[seedc::KI - 1]; // cnt[j-1]: [4^j] j-mer counts
    uint32_t *const *cnt_dev;     // the cnt pointers, in device memory
    void *temp;                   // rocPRIM temporary storage
    size_t temp_bytes;
};

// enqueue the whole build on stream s; 0 or a hipError_t
int seed_index_device_build(const SeedIndexBuild &B, hipStream_t s);
size_t seed_index_temp_bytes(int64_t n_text);

}  // namespace prgpu
