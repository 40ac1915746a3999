// Device-side structures of bwa mode: bwa mem's per-read alignment after seeding
// (mem_chain2aln over every seed of the kept chains, mem_sort_dedup_patch,
// mem_mark_primary_se, mem_reg2sam's filters and order) around the SW kernels.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/prgpu.h"
#include "sw_dev.h"

namespace prgpu {

// the largest read (seeds) the wave-per-read walk and final kernels take; larger reads go to
// the lane-per-read kernels
constexpr int ALN_WAVE_SEEDS = 128;

// one region of a read in the final pass (per-read scratch, in HBM)
struct AlnReg {
    int64_t rb, re;        // bwa's forward-reverse coordinates
    uint64_t hash;         // hash_64(read_id + i) (mem_mark_primary_se)
    int32_t qb, qe, score, truesc, w, seedlen0, lr, strand, task, secondary, patched, pad;
};

// an extended seed's region as the walk's containment tests read it, packed in one 32-byte
// record (one cache line per test instead of one per field array)
struct alignas(32) AlnBox {
    int32_t qb, qe, rb, re, slen, w, tq, tr;   // region (strand coordinates), seed length, seed qbeg / rbeg
};

// a patch (mem_patch_reg) whose global score the final pass needs
struct AlnPatch {
    int32_t read, m, lr, strand, qb, qe, rb, re, w, pad;   // query [qb,qe) x strand reference [rb,re)
};

struct AlnDev {
    int64_t n_task;
    int32_t n_sr, n_lr;
    int64_t read_id0;
    const int64_t *seed_off;   // [n_sr+1] seeds (tasks) of short read r
    const int32_t *t_sr, *t_lr, *t_qbeg, *t_rbeg, *t_slen, *t_chain;
    const uint8_t *t_strand;
    const int64_t *sr_off, *lr_off;
    const uint8_t *sr, *lr;
    // extension results per task (strand coordinates); the final pass writes merged regions back
    int32_t *o_qb, *o_qe, *o_rb, *o_re, *o_score, *o_truesc, *o_w;
    uint8_t *o_pass;
    uint8_t *sel;              // SEL_EXT: extend in the next round; SEL_CIG: reported alignment
    uint8_t *ext;              // 1: the task's extension result is available
    uint8_t *dec;              // mem_chain2aln's decision: 0 open, 1 extended (a region), 2 skipped
    int32_t *resume;           // [n_sr] first undecided seed of the read
    int32_t *counter;          // [0] extension requests (aln_list_kernel), [1] patch requests
    int32_t *tlist;            // [n_task] the seeds to extend in the next round (their count in counter)
    int32_t *cnext;            // [n_task] of a chain's first seed: the next chain's first seed
    int32_t cnext_ready;       // cnext already written (aln_unpack_kernel, from the seeds' ranks)
    int64_t n_big;             // reads of more than ALN_WAVE_SEEDS seeds (0: no lane-kernel launches)
    AlnBox *box;               // [n_task] the extended seeds' regions, packed by the walk (null: the field arrays)
    int32_t *hprev;            // [n_task] of a chain head: the read's previous head on the same long read and strand (or -1); null: scan every head
    AlnReg *R;                 // [n_task] region scratch (read r: from seed_off[r])
    int32_t *ix;               // [n_task] sort scratch
    int32_t *pscore;           // [n_task] known patch scores of read r (from seed_off[r])
    int32_t *npk;              // [n_sr] patch scores known
    uint8_t *fdone;            // [n_sr] final pass done
    AlnPatch *preq;            // patch requests of this round
    int32_t preq_cap;
    int32_t *nout;             // [n_sr] reported alignments
    int32_t *olist;            // [n_task] reported tasks of read r (from seed_off[r]), SAM order
    int32_t *oflag;            // [n_task] their SAM FLAG bits (0x10, 0x100, 0x800)
    // options
    int32_t a, b, o_del, e_del, o_ins, e_ins, w, max_chain_gap;
    double min_score_per_base, drop_ratio, mask_level, mask_level_redun;
};

int aln_launch_init(const AlnDev &A, void *stream);
int aln_launch_walk(const AlnDev &A, void *stream);
// hprev of every chain head (after the init kernel)
int aln_launch_heads(const AlnDev &A, void *stream);
// the seeds flagged SEL_EXT -> tlist, their count -> counter[0] (add to it)
int aln_launch_list(const AlnDev &A, void *stream);
// early: only reads whose walk has finished, patch requests not recorded (the late pass replays)
// complement (with early_snap): the reads the early pass skips, beside it
int aln_launch_final(const AlnDev &A, void *stream, const int32_t *early_snap, bool complement = false);
int aln_launch_patch(const AlnDev &A, int n_req, int32_t *pool, int64_t pool_stride, void *stream);
// CIGAR slots of the reported tasks: slot[t] = cig_slot_ops(lq) or 0 -> exclusive prefix (n+1)
int aln_launch_cig_slots(const AlnDev &A, int64_t *slot_prefix, int64_t *tmp_in, void *temp, size_t temp_bytes,
                         void *stream);
size_t aln_scan_temp_bytes(int64_t n);
// reported alignments in read order: aoff = prefix of nout, alist = their tasks, aflag
int aln_launch_compact(const AlnDev &A, int64_t *aoff, int64_t *tmp_in, int32_t *alist, int32_t *aflag, void *temp,
                       size_t temp_bytes, void *stream);
// stable regrouping of the reported alignments by long read: out_list, lr_off (n_lr+1)
int aln_launch_group_lr(const int32_t *alist, const int32_t *t_lr, int64_t n, int32_t n_lr, int32_t *key0, int32_t *key1,
                        int32_t *out_list, int32_t *cnt, int64_t *lr_off, int64_t *tmp_in, void *temp,
                        size_t temp_bytes, void *stream);
size_t aln_group_temp_bytes(int64_t n, int32_t n_lr);
// the dense seed list of pr_seed_gpu_map (pr_seed_task AoS) -> the SW task columns; n_first[0]
// += the seeds of rank 0 (every chain's first seed); cnext of every chain's first seed
// (a chain's seeds are consecutive with ranks 0, 1, ..: its first is t - rank)
int aln_launch_unpack_seeds(const pr_seed_task *src, int64_t n, int32_t *sr, int32_t *lr, uint8_t *strand,
                            int32_t *qbeg, int32_t *rbeg, int32_t *slen, int32_t *chain, int32_t *n_first,
                            int32_t *cnext, void *stream);

}  // namespace prgpu
