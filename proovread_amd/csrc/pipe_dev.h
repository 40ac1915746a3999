// SW -> consensus device hand-off (pipe_kernels.hip).
#pragma once
#include <stdint.h>

namespace prgpu {

struct PipeDev {
    int n_lr;
    int sort_cap;            // max alignments per long read the LDS sort holds
    const int64_t *task_off; // [n_lr+1] tasks grouped by long read
    const int32_t *t_sr;
    const uint8_t *strand;
    const uint8_t *pass;
    const int32_t *status, *pos, *score, *ncig;
    const int64_t *sr_off;
    const int64_t *cig_at;   // [n_task] first op of each task's CIGAR in the SW pool
    int32_t *cnt;            // [n_lr]
    int64_t *aln_off;        // [n_lr+1]
    int32_t *err;            // [n_lr]
    // consensus-stage alignment arrays (BAM coordinate order per read)
    int32_t *a_pos;
    double *a_score;
    uint8_t *a_flags;
    int64_t *a_seq_off;
    int32_t *a_lseq;
    int64_t *a_cig_off;
    int32_t *a_ncig;
};

int pipe_launch(const PipeDev &P, int grid, void *stream, int lds_sort);
int iter_stats_launch(const int64_t *out_off, const int32_t *status, const int32_t *seq_len, const uint8_t *qual,
                      int n_lr, int min_char, unsigned long long *out, void *stream);

}  // namespace prgpu
