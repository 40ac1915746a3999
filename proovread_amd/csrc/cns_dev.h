// Device-side structures shared by the consensus kernels and the host API.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace prgpu {

// negative PR_ERR_* codes (include/prgpu.h) used inside kernels
constexpr int PR_ERR_CODE_SAM = -3;
constexpr int PR_ERR_CODE_NOSEQ = -4;
constexpr int PR_ERR_CODE_BIN = -5;
constexpr int PR_ERR_CODE_DIV0 = -6;
constexpr int PR_ERR_CODE_CIGAR = -7;
constexpr int PR_ERR_CODE_BEYOND = -8;
constexpr int PR_ERR_CODE_CAP = -9;

// per-alignment prep status bits (cns_prep)
enum : uint32_t {
    ST_NOSEQ = 1u,      // SEQ '*'                       -> LR error (bam2cns:347)
    ST_SAM = 2u,        // malformed record              -> LR error
    ST_DIV0 = 4u,       // scored, length 0              -> LR error (Alignment.pm:537)
    ST_BINRANGE = 8u,   // scored, bin beyond last bin   -> LR error (Seq.pm:606)
    ST_SCORED = 16u,    // has AS -> offered to add_aln_by_score
    ST_SMSKIP = 32u,    // skipped by State_matrix (length / trim filters)
    ST_SMERR = 64u,     // State_matrix would die (unknown / empty CIGAR)
    ST_BEYOND = 128u,   // states extend past the long read end
    ST_SMCAP = 256u,    // too many states for the 12-bit state index
};

struct CnsParamsDev {
    double max_coverage, bin_size, bin_max_bases, indel_taboo;
    int trim, indel_taboo_length, min_aln_length, max_ins_length;
    int fallback_phred, phred_offset, ref_phred_offset, use_ref_qual;
    int detect_chimera, invert_scores;
};

struct CnsDev {
    int32_t n_lr;
    int64_t n_aln;
    // inputs
    const int64_t *lr_off;
    const uint8_t *ref_seq;   // may be null
    const uint8_t *ref_qual;  // may be null
    const int64_t *ign_off;   // may be null
    const int32_t *ign;
    const int64_t *aln_off;
    const int32_t *pos;
    const double *score;
    const uint8_t *aflags;
    const int64_t *seq_off;
    const int32_t *lseq;
    const int64_t *cig_off;
    const int32_t *ncig;
    const uint8_t *seq;
    const uint32_t *cig;
    int seq_nt4;           // seq pool holds nt4 codes (GPU pipeline) instead of ASCII
    int ref_nt4;           // reference pool holds nt4 codes
    // prep outputs (per alignment)
    uint32_t *a_st;
    int32_t *a_len;
    double *a_nc;
    int32_t *a_bin;
    int32_t *a_cb, *a_ce, *a_sb, *a_rpos, *a_end;
    // scratch
    int32_t *sorted;     // per alignment: LR-local index, grouped by bin
    double *lst_score;   // per alignment slot: bin list scores
    int32_t *lst_aln;    // per alignment slot: bin list members
    uint8_t *kept;       // per alignment
    int64_t *bin_off;    // [n_lr+1] prefix of bins
    int64_t *bin_bases;  // per bin
    int32_t *work;       // [2] dequeue counters (small, large geometry)
    // kept alignments bucketed by start window (per resident workgroup, k_cap ints each):
    // window starts, then {rpos, end, alignment index, 0} per kept alignment
    int32_t *k_pool;
    int64_t k_cap;
    // reads whose tables outgrew the small LDS geometry, rerun with the large one
    int32_t *retry;      // [n_lr]
    int32_t *retry_n;    // [1]
    int force_large;     // diagnostics: every read through the large geometry (PRGPU_CNS_LARGE)
    int debug;           // timing ablations only (PRGPU_CNS_DEBUG; outputs invalid when set)
    unsigned long long *prof;  // [CNS_NPHASE] summed wall-clock ticks per phase (may be null)
    // outputs
    const int64_t *out_off;  // [n_lr+1]
    const int64_t *chim_off; // [n_lr+1]
    int32_t *status, *seq_len, *trace_len, *ncigar, *nchim;
    uint8_t *o_seq, *o_qual, *o_trace;
    uint32_t *o_cig;
    int32_t *o_chim;     // 4 ints per record
};

// host-side launcher (returns a hipError_t value); stream is a hipStream_t.  grid: small-
// geometry workgroups (2 per CU); grid_retry: large-geometry workgroups (1 per CU)
int cns_launch(const CnsDev &D, const CnsParamsDev &P, int grid, int grid_retry, void *stream);
int cns_max_bins();
int cns_wg_per_cu();   // workgroups per CU of the first-pass geometry
int cns_k_header();      // ints of window starts reserved at the head of a K pool slice

constexpr int CNS_THREADS = 256;
constexpr int CHIM_MAXCOLS = 128;
constexpr int CHIM_TCAP = 256;
constexpr int CHIM_CL = 8;   // insertion states a column's chimera entry list holds (more: the table scan)
// per-phase wall-clock ticks: prep, binning, state table, scatter, argmax+write, cigar, chimera,
// idle; scatter detail: zero+ignore, group select, staging, walks; counts: groups, items, windows
constexpr int CNS_NPHASE = 24;

}  // namespace prgpu
