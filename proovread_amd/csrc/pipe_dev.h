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
    const int64_t *lr_off;   // [n_lr+1] long-read offsets (bin count of the -b/-l filter)
    const uint32_t *cig;     // SW CIGAR pool (cig_at)
    uint8_t *keep;           // [n_task] survivors of the -b/-l filter, or null (filter off)
    int32_t *fsorted;        // [n_task] scratch: tasks of a long read grouped by bin
    int32_t *fbin;           // [n_task] scratch: bin of each task (-1: not reported)
    double *fnc;             // [n_task] scratch: ncscore
    int32_t *flen;           // [n_task] scratch: Sam::Alignment length
    double *flst;            // [n_task] scratch: per-bin score lists
    int32_t *flsti;          // [n_task] scratch: per-bin list members
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
// bwa-proovread -b/-l score binning (the filter runs before pipe_launch when P.keep is set)
int pipe_binfilter_launch(const PipeDev &P, int bin_size, double bin_length, int max_bins, int grid, void *stream);
// dense pools of the consensus (d0), its quality (d1) and masked copy (d2) from the capacity layout
int lr_compact_launch(const int64_t *src_off, const int32_t *len, const int64_t *dst_off, int n, const uint8_t *s0,
                      uint8_t *d0, const uint8_t *s1, uint8_t *d1, const uint8_t *s2, uint8_t *d2, void *stream);
// the consensus input (SEQ bytes, CIGAR ops) copied into pools in the hand-off's order
size_t cns_gather_temp_bytes(int64_t n);
int cns_gather_offsets(const int64_t *aln_total, int64_t n, const int32_t *lseq, const int32_t *ncig, int64_t *sz_seq,
                       int64_t *sz_cig, int64_t *nso, int64_t *nco, void *temp, size_t temp_bytes, void *stream);
int cns_gather_copy(const int64_t *aln_total, int64_t n, const uint8_t *seq, const uint32_t *cig, int64_t *seq_off,
                    const int32_t *lseq, int64_t *cig_off, const int32_t *ncig, const int64_t *nso, const int64_t *nco,
                    uint8_t *gseq, uint32_t *gcig, void *stream);
int iter_stats_launch(const int64_t *out_off, const int32_t *status, const int32_t *seq_len, const uint8_t *qual,
                      int n_lr, int min_char, unsigned long long *out, void *stream);

}  // namespace prgpu
