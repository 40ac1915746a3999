// Launch descriptor of the seeding kernel (seed_kernels.hip).
#pragma once
#include <stdint.h>

#include <vector>

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
    int64_t n_lanes;           // scratch slots = resident waves (one read per wave at a time)
    int32_t *next;             // read counter the waves dequeue from (zeroed before the launch)
    unsigned long long *prof;  // [8] wall-clock ticks summed over waves: occurrence tables, SMEMs
                               // (pass 1: the whole lane-per-read phase), chaining and filter +
                               // output of pass 2 (may be null)
    seedc::Caps caps;
    pr_seed_task *out;         // [(reads of the chunk) * caps.out]: read i's slots at (i - out0) * caps.out
    int64_t out0;              // first read of the chunk (pass 1 maps reads [*next, n_sr) at entry)
    int32_t *n_out;            // [n_sr]
    int32_t *status;           // [n_sr] 0 or SC_OVER_* bits
    int16_t *dp;               // pass 1: per wave 2 x 201 x 64 int16 (mem_flt_chained_seeds rows, lane-interleaved)
    const int32_t *rlist;      // pass 2: the reads to map (n_list of them); null: 0 .. n_list
    int64_t n_list;
};

int seed_launch(const SeedDev &D, void *stream);         // pass 2: one wave per read of rlist
int seed_batch_launch(const SeedDev &D, void *stream);   // pass 1: 64 reads per wave, lane per read
// pass 1's read order, costliest first: a per-read cost estimate (the summed occurrence counts of
// its 12-mers, every second start) sorted descending -> order[0 .. n) (reads r0 .. r0 + n).
// buf: seed_order_bytes(n) bytes of device scratch
size_t seed_order_bytes(int64_t n);
int seed_order_launch(const SeedDev &D, int64_t r0, int64_t n, void *buf, int32_t **order, void *stream);
// resident waves per CU of the seeding kernel (= scratch slots per CU)
int seed_slots_per_cu(int walk_nw);   // pass 2's resident waves per CU (seed_wave_kernel<walk_nw>)
// dense task list: out[pre[i] + j] = slots[i * cap + j] for j < n_out[i]
int seed_compact_launch(const pr_seed_task *slots, const int32_t *n_out, const int64_t *pre, int64_t n_sr, int cap,
                        pr_seed_task *out, void *stream);

// host-side view of a built index (seed.cpp)
seedc::IndexView seed_index_view(const pr_seed_index *h);
// sizes of the index arrays for the device copy
struct SeedIndexSizes {
    int64_t text, cstart, cblk, lr_off, koff, kpos, ksplit, cnt[seedc::KI - 1];
};
SeedIndexSizes seed_index_sizes(const pr_seed_index *h);
// pr_seed_index_digest's six values over tables copied to the host (device index test hook)
void seed_digest_tables(const std::vector<uint8_t> &text, const std::vector<uint64_t> &koff,
                        const std::vector<uint32_t> &kpos, const std::vector<uint64_t> &kext,
                        const std::vector<std::vector<uint32_t>> &cnt, const std::vector<int64_t> &cstart,
                        const std::vector<int32_t> &cblk, const std::vector<int64_t> &lr_off,
                        const std::vector<uint64_t> &ksplit, uint64_t *out6);

}  // namespace prgpu
