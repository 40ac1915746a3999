// Device side of the exact-parity multi-GPU layout's alignment exchange (xchg_kernels.hip,
// driven by pr_aln_exchange / pr_iter_launch on an owned batch in prgpu_api.cpp).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace prgpu {

// one reported alignment on the wire: what the owner's -b/-l filter, hand-off and consensus
// read (bin/proovread:1313 SAM fields: QNAME as the global short-read id, RNAME as the global
// long-read id, POS 0-based, AS:i, the strand bit of FLAG; the CIGAR ops travel separately)
struct XRec {
    int32_t sr, lr, pos, score, ncig, strand;
};

// sender: the reported alignments of the last bwa-mode pr_sw_launch, partitioned by the
// owner of their long read (stable: SAM order inside each owner's block)
struct XchgSend {
    int64_t n;                    // reported alignments
    const int32_t *alist;         // alignment -> task, SAM order
    const int32_t *t_sr, *t_lr, *status, *pos, *score, *ncig;
    const uint8_t *strand, *pass;
    const int64_t *cig_at;
    const uint32_t *cig;
    const int64_t *bounds;        // [world+1] long-read ranges of the ranks
    int world;
    int64_t sr0;                  // global id of the shard's short read 0
    int32_t *key0, *key1, *idx0, *idx1;   // [n] owner keys / alignment indices (sort in, out)
    unsigned long long *cnt;      // [2 * (world + 1)]: records, then CIGAR ops, per owner (world: dropped)
    int64_t *op_in, *op_at;       // [n + 1] CIGAR ops per sorted alignment, their exclusive prefix
    XRec *rec;                    // [n] wire records, owner blocks back to back
    uint32_t *wcig;               // wire CIGAR ops, owner blocks back to back
};

// receiver: the owner's alignments (source-rank-major = the single run's read order)
// regrouped by long read (stable) into the hand-off's per-alignment arrays
struct XchgRecv {
    int64_t n;                    // received records
    const XRec *rec;
    int32_t lr0, n_lr;            // owned long reads [lr0, lr0 + n_lr)
    int32_t *key0, *key1, *idx0, *idx1;   // [n]
    int32_t *cnt;                 // [n_lr + 1] alignments per owned long read
    int64_t *cnt64;               // [n_lr + 1] scan input
    int64_t *task_off;            // [n_lr + 1]
    int64_t *op_in, *rcig_at;     // [n + 1] ops per received record, their prefix (wire CIGAR pool)
    int32_t *err;                 // [1] a record outside the owned range (cannot happen: sender bounds)
    // grouped outputs (PipeDev inputs)
    int32_t *o_sr, *o_status, *o_pos, *o_score, *o_ncig;
    int64_t *o_cig_at;
    uint8_t *o_strand, *o_pass;
};

size_t xchg_temp_bytes(int64_t n, int32_t n_keys);
// owners, counts (X.cnt), the stable partition and the ops prefix; then, once the host has sized
// the wire CIGAR pool from the counts, the records and ops
int xchg_pack_launch(const XchgSend &X, void *temp, size_t temp_bytes, void *stream);
int xchg_write_launch(const XchgSend &X, void *stream);
int xchg_group_launch(const XchgRecv &X, void *temp, size_t temp_bytes, void *stream);

}  // namespace prgpu
