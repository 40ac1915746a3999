/* ORACLE — TEST INFRASTRUCTURE ONLY (see aln_oracle.c header). */
#ifndef PROOVREAD_ALN_ORACLE_H
#define PROOVREAD_ALN_ORACLE_H
#include <stdint.h>

#include "sw_oracle.h"
#ifdef __cplusplus
extern "C" {
#endif

/* one seed of a kept chain (pr_seed_task layout): seeds grouped by chain (chain order of
 * mem_chain_flt), inside a chain in mem_chain2aln's extension order (rank 0 first) */
typedef struct {
    int sr, lr, strand, qbeg, rbeg, slen, rmax0, rmax1, chain, rank;
} oaln_seed;

typedef struct {
    double drop_ratio;        /* -D: mem_reg2sam drops secondaries below drop_ratio x primary */
    double mask_level;        /* 0.5 (mem_mark_primary_se)                                     */
    double mask_level_redun;  /* 0.95 (mem_sort_dedup_patch)                                   */
    int max_chain_gap;        /* 10000                                                         */
} oaln_opts;

/* one reported region, in SAM output order */
typedef struct {
    int lr, strand;
    osw_region g;             /* strand coordinates; patched regions carry the merged span    */
    int secondary;            /* index (output order) of its primary; -1 primary or unreported */
    int flag;                 /* SAM FLAG bits 0x10 / 0x100 / 0x800                           */
    int seed;                 /* the seed (index into the read's seeds) that produced it       */
    int patched;
} oaln_reg;

/* One short read through bwa mem after seeding (bwamem.c mem_chain2aln over every seed,
 * mem_sort_dedup_patch, mem_mark_primary_se, mem_reg2sam's -T / -D filters and order).
 * lr_seq/lr_off: forward long reads (nt4); read_id: the read's index in the bwa input
 * (hash_64(read_id + i) orders equal scores).  out: capacity ns.  Returns 0 or < 0;
 * *n_ext: seeds extended. */
int oaln_read(const osw_opts *o, const oaln_opts *ao, const uint8_t *q, int lq, const uint8_t *lr_seq,
              const int64_t *lr_off, int n_lr, const oaln_seed *s, int ns, int64_t read_id, oaln_reg *out,
              int *n_out, int *n_ext);

#ifdef __cplusplus
}
#endif
#endif
