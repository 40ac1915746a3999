// Launch descriptor of the device seed-index build (seed_index.hip).  All pointers are
// device pointers; the host computes the small tables (contig starts, block table).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "seed_core.h"

namespace prgpu {

struct SeedIndexBuild {
    uint8_t *lr_seq;              // [l_pac] long-read codes (nt4 or ASCII), rewritten as nt4
    const int64_t *lr_off;        // [n_lr + 1] rebased to 0
    int n_lr;
    int64_t l_pac;
    const int64_t *cstart;        // [2 n_lr] text offset of every contig
    int64_t n_text;               // 2 l_pac + 2 n_lr (<= seedc::MAX_TEXT)
    uint8_t *text;                // [n_text]
    // the 12-mer lists are sorted in chunks of `chunk` text positions (a divisor of 2^32); one
    // chunk (the text fits): the sort writes kpos directly
    int64_t chunk;
    uint32_t *key0, *key1, *val0; // [chunk] sort scratch
    uint32_t *val1;               // [chunk] sorted positions (several chunks only)
    uint32_t *kc;                 // [NK + 1] 12-mer histogram (last entry 0)
    uint64_t *koff;               // [NK + 1]
    uint32_t *kcc, *koffc;        // [NK + 1] a chunk's histogram and its scan (several chunks)
    uint64_t *kcur;               // [NK] next slot of every k-mer (several chunks)
    uint32_t *kpos;               // [hits] sorted positions (low 32 bits)
    uint64_t *kext;               // [hits]
    uint64_t *ksplit;             // [NK] first hit at or beyond 2^32 (n_text > 2^32), else null
    uint32_t *cnt[seedc::KI - 1]; // cnt[j-1]: [4^j] j-mer counts
    uint32_t *const *cnt_dev;     // the cnt pointers, in device memory
    void *temp;                   // rocPRIM temporary storage
    size_t temp_bytes;
};

// enqueue the whole build on stream s; 0 or a hipError_t
int seed_index_device_build(const SeedIndexBuild &B, hipStream_t s);
// the 4-bit packed copy of a device text (IndexView.text4): words needed, launch
int64_t ix_pack4_words(int64_t n_text);
int ix_pack4_launch(const uint8_t *text, int64_t n_text, uint64_t *text4, hipStream_t s);
size_t seed_index_temp_bytes(int64_t chunk);

}  // namespace prgpu
