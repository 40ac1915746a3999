/*
 * prgpu.h — C-ABI of libprgpu.so, the MI355X (gfx950) implementation of
 * proovread's hot path.  Plain pointers and sizes only; no torch / HIP types.
 *
 * Two stages of the reference become HIP kernels behind this ABI:
 *
 *  1. Consensus (pileup): what one `bam2cns` worker process does for a chunk
 *     of long reads (bin/bam2cns:332-365 per-read loop, 375-455
 *     generate_consensus, 461-491 detect_chimera) using the Sam::Seq engine
 *     (lib/Sam/Seq.pm: add_aln_by_score 582-614, State_matrix 232-467,
 *     state_matrix_consensus 1568-1654, chimera 774-889).
 *     REPLACES: the `xargs -P T perl bam2cns ...` fan-out of
 *     bin/proovread:1596-1619 (correct_sr_mt) — one pr_cns_run() call per
 *     chunk (or per GPU shard of chunks).  The class globals of Sam::Seq
 *     (Seq.pm:114-128, set at bam2cns:227-237) become pr_cns_params.
 *
 *  2. Seed extension + CIGAR (SW): the ksw_extend2 / ksw_global2 stage inside
 *     `bwa-proovread mem` (called from bin/proovread:1313 run_bwa) for a batch
 *     of (short read, long read, seed) tasks.  REPLACES: the extension and
 *     CIGAR-generation inner loops of the absent bwa-proovread binary
 *     (SURVEY.md §8a A2/A3), see pr_sw_run().
 *
 * Conventions: every function returns 0 (PR_OK) on success or a negative
 * PR_ERR_* code; pr_last_error() returns a thread-local message.  Callers own
 * all input buffers (copied before the call returns); output buffers are
 * owned by the caller too (sizes are given by the *_bounds helpers).
 * Handles are not thread-safe; use one pr_ctx per thread / device.
 */
#ifndef PRGPU_H
#define PRGPU_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum {
    PR_OK = 0,
    PR_ERR_ARG = -1,          /* bad argument / shape                                   */
    PR_ERR_HIP = -2,          /* HIP runtime failure (no device, OOM, launch failure)   */
    PR_ERR_SAM = -3,          /* malformed record (CIGAR query length != SEQ length ...) */
    PR_ERR_NOSEQ = -4,        /* SEQ '*' (bam2cns:347 "Cannot handle ... without seq")  */
    PR_ERR_BIN_RANGE = -5,    /* alignment centre beyond last bin (Perl dies, Seq.pm:606) */
    PR_ERR_DIV0 = -6,         /* zero-length scored alignment (Perl "Illegal division") */
    PR_ERR_CIGAR = -7,        /* unknown CIGAR op in a kept alignment (Seq.pm:348/378/430) */
    PR_ERR_BEYOND_REF = -8,   /* kept alignment extends past the long read end            */
    PR_ERR_CAPACITY = -9,     /* an on-chip table overflowed (see DESIGN.md limits)       */
    PR_ERR_UNSUPPORTED = -10, /* option not implemented on the GPU path                   */
};

const char *pr_last_error(void);
const char *pr_version(void);

/* ------------------------------------------------------------------ */
/* device context                                                      */
typedef struct pr_ctx pr_ctx;
/* device: HIP device ordinal (one process per GPU; -1 = current device) */
int pr_ctx_create(int device, pr_ctx **out);
void pr_ctx_destroy(pr_ctx *ctx);
int pr_device_count(int *n);
/* wait for everything enqueued on the context's stream */
int pr_ctx_sync(pr_ctx *ctx);
/* device memory of the context (plumbing for drivers: e.g. the int64[2] statistic that
 * pr_iter_stats / pr_iter_mask fill and pr_comm_allreduce_dev reduces across GPUs) */
int pr_dev_alloc(pr_ctx *ctx, int64_t bytes, void **dev);
int pr_dev_free(pr_ctx *ctx, void *dev);
/* copies on the context stream; both synchronise */
int pr_dev_download(pr_ctx *ctx, void *host, const void *dev, int64_t bytes);
int pr_dev_upload(pr_ctx *ctx, void *dev, const void *host, int64_t bytes);
/* Device memory the library's buffers hold (every context of the process; not the HIP
 * runtime's own): bytes now, the peak since the last pr_mem_reset_peak, and per buffer group
 * ("cns", "pipe", "mask", "seed", "xchg", "lrset", "sw") its bytes now, its own peak and its
 * bytes at the moment of the total peak.  No reference counterpart (sizing at configs[2] /
 * configs[3]). */
typedef struct {
    char name[16];
    int64_t cur, peak, at_total_peak;
} pr_mem_group;
int pr_mem_stats(int64_t *cur, int64_t *peak, pr_mem_group *groups, int cap, int *n_groups);
void pr_mem_reset_peak(void);

/* ------------------------------------------------------------------ */
/* multi-GPU collectives over RCCL (one process per GPU, xGMI).  The reference has no
 * distributed backend (processes on one host exchange files); what
 * crosses GPUs here is the per-iteration masked-fraction statistic {bpt, bpN}
 * (bin/proovread:1702-1720, consumed by mask_shortcut_frac 2026-2047) and, in the
 * exact-parity layout, seed-extension tasks and corrected reads.
 * Rank 0 creates the id and hands it to the other ranks out of band (a file or
 * socket rendezvous: proovread_amd/comm.py).  Host-buffer calls synchronise;
 * pr_comm_allreduce_dev is asynchronous on the context stream.                  */
#define PR_COMM_ID_BYTES 128
enum { PR_DT_I64 = 0, PR_DT_F64 = 1, PR_DT_I32 = 2, PR_DT_U8 = 3 };
enum { PR_RED_SUM = 0, PR_RED_MAX = 1, PR_RED_MIN = 2 };
typedef struct pr_comm pr_comm;
int pr_comm_unique_id(uint8_t *id);                        /* id[PR_COMM_ID_BYTES] */
int pr_comm_init(pr_ctx *ctx, int world, int rank, const uint8_t *id, pr_comm **out);
void pr_comm_destroy(pr_comm *c);
int pr_comm_rank(const pr_comm *c, int *rank, int *world);
/* every rank passes its local status (0 or a PR_ERR_*): 0 on all ranks only if all were 0;
 * a rank that failed gets its own code back, the others PR_ERR_ARG.  The multi-rank calls
 * (pr_aln_exchange, pr_lrset_commit) agree this way before their first data collective, so
 * an error on one GPU returns on every rank instead of leaving the others in a collective. */
int pr_comm_agree(pr_comm *c, int local_rc);
int pr_comm_allreduce_dev(pr_comm *c, const void *dev_in, void *dev_out, int64_t n, int dtype, int op);
int pr_comm_allreduce_host(pr_comm *c, void *buf, int64_t n, int dtype, int op);
int pr_comm_barrier(pr_comm *c);
/* every rank's nbytes block, back to back in rank order; counts[world] = block sizes.
 * recv NULL: only fills counts (size query). */
int pr_comm_allgatherv_host(pr_comm *c, const uint8_t *send, int64_t nbytes, uint8_t *recv, int64_t recv_cap,
                            int64_t *counts);
/* recv_counts[r] = bytes rank r sends to this rank */
int pr_comm_alltoall_counts(pr_comm *c, const int64_t *send_counts, int64_t *recv_counts);
int pr_comm_alltoallv_host(pr_comm *c, const uint8_t *send, const int64_t *send_counts, uint8_t *recv,
                           const int64_t *recv_counts);
/* the same on DEVICE buffers, asynchronous on the context stream (no host copy) */
int pr_comm_alltoallv_dev(pr_comm *c, const void *send, const int64_t *send_counts, void *recv,
                          const int64_t *recv_counts);
/* all-gather of DEVICE byte blocks: counts[world] (the same on every rank) = each rank's bytes;
 * rank r's block lands at recv + sum(counts[0..r)); asynchronous on the context stream */
int pr_comm_allgatherv_dev(pr_comm *c, const void *send, const int64_t *counts, void *recv);
/* An in-process group: `world` ranks as threads of one process, each with its own context
 * (on one GPU or several), collectives through device copies in place of RCCL; every call
 * above works on such a communicator (synchronously).  A single-GPU box runs the multi-rank
 * paths with it (tests/test_local_group_gpu.py).  The group outlives its communicators. */
typedef struct pr_comm_group pr_comm_group;
int pr_comm_group_create(int world, pr_comm_group **out);
void pr_comm_group_destroy(pr_comm_group *g);
/* a rank of the in-process group left its collective sequence (an exception in its thread):
 * the ranks waiting in a collective return PR_ERR_ARG, and so does every later collective */
void pr_comm_group_abort(pr_comm_group *g);
int pr_comm_init_local(pr_ctx *ctx, pr_comm_group *g, int rank, pr_comm **out);

/* ------------------------------------------------------------------ */
/* consensus stage                                                     */

/* Sam::Seq class globals (Seq.pm:114-128) + consensus() options.          */
typedef struct pr_cns_params {
    double max_coverage;      /* --coverage (bam2cns:230); proovread passes min(cov,task)*0.75 */
    double bin_size;          /* BinSize; bam2cns always uses 20 (bam2cns:186 quirk)     */
    int32_t trim;             /* Sam::Seq->Trim (cfg sr-trim)                            */
    int32_t indel_taboo_length; /* cfg sr-indel-taboo-length (7); 0 => use indel_taboo    */
    double indel_taboo;       /* cfg sr-indel-taboo (0.1)                                */
    int32_t min_aln_length;   /* StateMatrixMinAlnLength (50)                            */
    int32_t max_ins_length;   /* --max-ins-length                                        */
    int32_t fallback_phred;   /* FallbackPhred (1)                                       */
    int32_t phred_offset;     /* Sam::Seq PhredOffset (33) — consensus quality output    */
    int32_t ref_phred_offset; /* phred offset of the reference FASTQ (--qv-offset)       */
    int32_t use_ref_qual;     /* --[no-]use-ref-qual                                     */
    int32_t qual_weighted;    /* --qual-weighted (not on the GPU path: PR_ERR_UNSUPPORTED) */
    int32_t detect_chimera;   /* --detect-chimera                                        */
    int32_t invert_scores;    /* --invert-scores (Alignment.pm InvertScores)             */
} pr_cns_params;

void pr_cns_params_default(pr_cns_params *p);

/* A batch = a set of long reads (a bam2cns chunk or a GPU shard) with their
 * alignments in BAM order.  CIGAR ops are BAM-encoded: len<<4 | op with
 * op in {M=0,I=1,D=2,N=3,S=4,H=5,P=6,'='=7,X=8}.                          */
enum { PR_ALN_HAS_SCORE = 1, PR_ALN_NO_QUAL = 2, PR_ALN_NO_SEQ = 4 };

typedef struct pr_cns_batch {
    int32_t n_lr;
    const int64_t *lr_off;    /* [n_lr+1] prefix of long-read lengths                    */
    const uint8_t *ref_seq;   /* concatenated long-read sequences (lr_off) or NULL (no --ref) */
    const uint8_t *ref_qual;  /* concatenated qualities (lr_off) or NULL                 */
    const int64_t *ign_off;   /* [n_lr+1] prefix into ign, or NULL (no MCR ranges)       */
    const int32_t *ign;       /* (offset,length) pairs: MCRn:off,len tags (bam2cns:384)  */
    const int64_t *aln_off;   /* [n_lr+1] prefix of alignment counts                     */
    const int32_t *aln_pos;   /* 1-based POS                                             */
    const double *aln_score;  /* AS:i value (valid if PR_ALN_HAS_SCORE)                  */
    const uint8_t *aln_flags; /* PR_ALN_*                                                */
    const int64_t *aln_seq_off; /* offset of SEQ (and QUAL) in seq_pool / qual_pool      */
    const int32_t *aln_lseq;
    const int64_t *aln_cig_off;
    const int32_t *aln_ncig;
    const uint8_t *seq_pool;
    const uint8_t *qual_pool;
    const uint32_t *cig_pool;
    int64_t seq_pool_len, cig_pool_len;
} pr_cns_batch;

/* Output capacities for a batch (all in elements).                        */
typedef struct pr_cns_bounds {
    int64_t seq_cap;          /* bytes for consensus seq (and qual, and trace, cigar ops) */
    int64_t chim_cap;         /* chimera records                                         */
} pr_cns_bounds;
int pr_cns_bounds_of(const pr_cns_batch *b, pr_cns_bounds *out);

typedef struct pr_cns_out {
    /* per long read, offsets into the pools are out_off[i] (from the bounds) */
    int64_t *out_off;         /* [n_lr+1] capacity prefix (filled by the library)       */
    int32_t *status;          /* [n_lr] PR_OK or PR_ERR_* for that read                 */
    int32_t *seq_len;         /* [n_lr] consensus length (= qual length)                */
    int32_t *trace_len;       /* [n_lr]                                                  */
    int32_t *ncigar;          /* [n_lr] consensus CIGAR ops (Trace2cigar)                */
    int32_t *nchim;           /* [n_lr] chimera records                                  */
    uint8_t *seq;             /* [seq_cap]                                               */
    uint8_t *qual;            /* [seq_cap] phred+phred_offset chars                      */
    uint8_t *trace;           /* [seq_cap] M/D/I                                         */
    uint32_t *cigar;          /* [seq_cap] len<<4|op (M=0,I=1,D=2)                      */
    int64_t *chim_off;        /* [n_lr+1] capacity prefix of chim records                */
    int32_t *chim;            /* [chim_cap*4] (from, to, n_pos, n_cols) per record        */
    uint8_t *kept;            /* [n_alns] 1 if kept after binning (may be NULL)          */
    int64_t *bin_bases;       /* optional: per-read bin fill (Seq.pm _bin_bases), reads
                                 concatenated, int(L/bin_size)+1 bins each (may be NULL)  */
} pr_cns_out;

/* One-shot: upload, run, download (synchronous). */
int pr_cns_run(pr_ctx *ctx, const pr_cns_params *p, const pr_cns_batch *b, pr_cns_out *o);

/* Resident-batch API (bench / pipelined drivers): inputs stay in HBM. */
int pr_cns_upload(pr_ctx *ctx, const pr_cns_batch *b);
int pr_cns_launch(pr_ctx *ctx, const pr_cns_params *p);     /* async on ctx stream */
int pr_cns_download(pr_ctx *ctx, pr_cns_out *o);            /* syncs               */
/* milliseconds of the last launch's dominant (pileup) kernel, HIP events on ctx stream */
int pr_cns_last_timing(pr_ctx *ctx, double *ms_prep, double *ms_pileup);
/* number of columns (sum of long-read lengths) and algorithmic bytes of the resident batch
 * (SURVEY.md §8d pileup byte model) */
/* Diagnostics: wall-clock ticks (100 MHz) the consensus workgroups spent per phase in the
 * last launch, summed over workgroups: [prep, binning, state table, pileup scatter,
 * argmax+write, Trace2cigar, chimera, dequeue/idle], then (n >= 24) the scatter's parts
 * [zero + ignore bits, group select, staging copy, fixed-state runs], counts [candidate
 * groups, candidates, windows], [op pre-pass], [insertion states], 3 spare;
 * n must be >= 8 (the first min(n, 24) are filled). */
int pr_cns_phase_ticks(pr_ctx *ctx, uint64_t *ticks, int n);
int pr_cns_resident_stats(pr_ctx *ctx, int64_t *columns, int64_t *alg_bytes);


/* ------------------------------------------------------------------ */
/* seed-extension stage (ksw_extend2 / ksw_global2 of bwa-proovread mem) */

/* bwa mem scoring / band options (proovread.cfg:320-333, 343-365).        */
typedef struct pr_sw_opts {
    int32_t a, b;                  /* -A match, -B mismatch                        */
    int32_t o_del, e_del;          /* -O d / -E d                                   */
    int32_t o_ins, e_ins;          /* -O ,i / -E ,i                                 */
    int32_t w;                     /* -w band width                                 */
    int32_t pen_clip5, pen_clip3;  /* -L 5,3 clipping penalties                     */
    int32_t zdrop;                 /* -d (bwa default 100)                          */
    double min_score_per_base;     /* -T "per-base-score" (cfg:324; semantics unpinned) */
    /* -b BIN -l LEN: bwa-proovread's score binning of the reported alignments (its
     * proovread.[ch], README.org:228-236; called with BIN = cfg bin-size, LEN = BIN x
     * min(--coverage, task sr-coverage), bin/proovread:1302-1313).  Applied by pr_iter_launch
     * between the SW stage and the consensus hand-off; 0 = off (pr_sw_opts_default).   */
    int32_t bin_size;
    double bin_length;
    /* bwa mode only (pr_sw_batch.t_chain): -D of mem_reg2sam (a secondary scoring below
     * drop_ratio x its primary is not reported), mem_mark_primary_se's mask_level (0.5),
     * mem_sort_dedup_patch's mask_level_redun (0.95) and max_chain_gap (10000)           */
    double drop_ratio;
    double mask_level;
    double mask_level_redun;
    int32_t max_chain_gap;
} pr_sw_opts;
/* finish = 0: bwa-sr iterations (-A5 -B11 -O2,1 -E4,3 -w40 -T2.5 -L30,30);
 * finish = 1: bwa-sr-finish (-A5 -B13 -O15,19 -E3,3 -w30 -T4 -L30,30)            */
void pr_sw_opts_default(pr_sw_opts *o, int finish);

/* A batch of extension tasks.  Sequences are nt4-coded (A0 C1 G2 T3 N4, as
 * bwa's nst_nt4_table).  A task is one exact-match seed of short read t_sr
 * on long read t_lr: t_strand 1 = the short read aligns to the reverse
 * complement; t_rbeg is in that strand's coordinates (reverse: L-1-x). This
 * replaces bwa-proovread's mem_chain2aln/mem_reg2aln for single-seed chains
 * (bwamem.c), i.e. one alignment per (short read, long read, strand).      */
typedef struct pr_sw_batch {
    int32_t n_sr;
    const int64_t *sr_off;          /* [n_sr+1]                                      */
    const uint8_t *sr_seq;
    int32_t n_lr;
    const int64_t *lr_off;          /* [n_lr+1]                                      */
    const uint8_t *lr_seq;
    int64_t n_task;
    const int32_t *t_sr, *t_lr;
    const uint8_t *t_strand;
    const int32_t *t_qbeg, *t_rbeg, *t_slen;
    /* bwa mode (NULL: single-seed tasks as above).  The tasks are every seed of the kept
     * chains, as pr_seed_map returns them: grouped by short read (ascending), then chain
     * (t_chain, mem_chain_flt order), in mem_chain2aln's order inside a chain.  The stage
     * then runs bwa mem's per-read alignment (bwamem.c): mem_chain2aln's containment test
     * over every seed (a seed inside an earlier region is not extended), mem_sort_dedup_patch,
     * mem_mark_primary_se and mem_reg2sam's -T / -D filters, and its outputs are the reported
     * alignments in SAM order (pr_sw_aln_count of them), not one per task.                */
    const int32_t *t_chain;
    int64_t read_id0;               /* bwa's input index of short read 0 (hash_64 ties)       */
} pr_sw_batch;

typedef struct pr_sw_out {          /* per task (any pointer may be NULL)              */
    int32_t *qb, *qe;               /* aligned query interval                          */
    int32_t *rb, *re;               /* reference interval (strand coordinates)         */
    int32_t *score;                 /* AS:i (local extension score)                    */
    int32_t *truesc;                /* mem_alnreg_t truesc                             */
    int32_t *pos;                   /* 0-based leftmost forward position (SAM POS-1)   */
    int32_t *ncigar;
    uint8_t *pass;                  /* score >= T * (qe - qb)                          */
    int32_t *status;                /* 0 (PR_ERR_CAPACITY cannot occur: CIGARs have no
                                       length limit, bwa_gen_cigar2's own bound holds) */
    /* CIGARs, variable length, compacted in task order: task t's ops (BAM codes M0 I1 D2
     * S4) are cigar[cigar_off[t] .. cigar_off[t+1]).  cigar_off [n_task+1] is filled when
     * given; cigar (capacity cigar_cap ops) when given and large enough, otherwise the call
     * returns PR_ERR_CAPACITY after filling everything else (pr_sw_cigar_total gives the
     * size; the batch stays resident, so pr_sw_download can be repeated).              */
    int64_t *cigar_off;
    uint32_t *cigar;
    int64_t cigar_cap;
    /* bwa mode: per reported alignment (SAM order, read by read) the seed task that made it
     * (its sr / lr / strand) and the SAM FLAG bits 0x10 / 0x100 (secondary) / 0x800; all the
     * arrays above are then per alignment (pr_sw_aln_count entries)                       */
    int32_t *task;
    int32_t *flag;
} pr_sw_out;

int pr_sw_run(pr_ctx *ctx, const pr_sw_opts *o, const pr_sw_batch *b, pr_sw_out *out);
int pr_sw_upload(pr_ctx *ctx, const pr_sw_batch *b);
int pr_sw_launch(pr_ctx *ctx, const pr_sw_opts *o);   /* async on ctx stream */
int pr_sw_download(pr_ctx *ctx, pr_sw_out *out);      /* syncs               */
/* total CIGAR ops of the last launch (the pr_sw_out.cigar size) and the tasks whose CIGAR
 * outgrew its slot and was recomputed into the spill area (syncs) */
int pr_sw_cigar_total(pr_ctx *ctx, int64_t *total, int64_t *n_overflow);
/* bwa mode: reported alignments of the last launch (syncs) */
int pr_sw_aln_count(pr_ctx *ctx, int64_t *n_aln);
/* bwa-proovread mem's output stage on the last bwa-mode launch (the `mem` drop-in, replacing
 * bwa-proovread's mem_reg2sam printing and its proovread.[ch] bin filter, bin/proovread:1302-1313).
 * pr_sw_binfilter: the -b BIN -l LEN score binning on the device (pipe_binfilter_kernel, the
 * same filter as pr_iter_launch's) -> keep[pr_sw_aln_count] in SAM order (1 = printed).
 * pr_sw_sam: the SAM records (QNAME FLAG RNAME POS MAPQ CIGAR * 0 0 SEQ QUAL AS:i) of the
 * reported alignments that passed -T (and keep, when given), in SAM order, formatted on host
 * threads into one library-allocated text (pr_buffer_free).  SEQ: the read as given, upper
 * case, or its reverse complement (N for non-ACGT) on the reverse strand; QUAL reversed there,
 * '*' without qualities.  MAPQ 60 primary, 0 secondary (bwa's MAPQ model is not restated). */
typedef struct pr_sam_in {
    const int64_t *sr_off;        /* [n_sr+1] the batch's short reads (pr_sw_batch.sr_off)      */
    const uint8_t *sr_text;       /* the reads as given (ASCII, sr_off layout)                  */
    const uint8_t *sr_qual;       /* phred+33 (sr_off layout), or NULL                          */
    const char *sr_names;         /* names pool: read i at [sr_name_off[i], sr_name_off[i+1])   */
    const int64_t *sr_name_off;
    const char *lr_names;         /* long-read names pool (RNAME)                               */
    const int64_t *lr_name_off;
    const uint8_t *keep;          /* [pr_sw_aln_count] from pr_sw_binfilter, or NULL            */
    int32_t n_threads;            /* <= 0: all cores                                            */
} pr_sam_in;
int pr_sw_binfilter(pr_ctx *ctx, int32_t bin_size, double bin_length, uint8_t *keep);
int pr_sw_sam(pr_ctx *ctx, const pr_sam_in *in, char **text, int64_t *len, int64_t *n_records);
/* bwa mode diagnostics of the last launch: extension rounds, seeds extended, mem_patch_reg
 * global scores computed */
int pr_sw_bwa_stats(pr_ctx *ctx, int32_t *rounds, int64_t *n_extended, int64_t *n_patch);
/* bwa mode's bookkeeping kernels of the last launch (HIP events): the walks summed over the
 * extension rounds and the main-stream final passes (the complement and the late passes), both
 * on the critical path, and the early final pass on the side stream beside the later rounds */
int pr_sw_bwa_timing(pr_ctx *ctx, float *walk_ms, float *final_ms, float *early_final_ms);
/* kernel milliseconds of the last launch (HIP events on the ctx stream) */
int pr_sw_last_timing(pr_ctx *ctx, double *ms_extend, double *ms_global);
/* canonical DP cells of the last launch (unpruned band, final width) */
int pr_sw_last_cells(pr_ctx *ctx, int64_t *cells_extend, int64_t *cells_global);
/* Diagnostics for the roofline: duration (HIP events on the SW stream) of the last
 * launch's dominant kernel, the CIGAR pass's packed launch (the band <= 40 ring launch
 * when the packed kernel is off), and the DP cells it computed. */
int pr_sw_dominant_kernel(pr_ctx *ctx, double *ms, int64_t *cells);
/* Diagnostics for the extension stage's roofline: the summed durations (HIP events around
 * each launch on the SW stream) of every extension DP launch of the last pr_sw_launch
 * (ksw_extend2: packed, ring and wide kernels, both sides, both band tries, every bwa-mode
 * round), the DP cells they computed and the number of launches.  PR_ERR_CAPACITY when
 * there were more launches than the 64 timed ones. */
int pr_sw_extension_kernels(pr_ctx *ctx, double *ms, int64_t *cells, int32_t *launches);
/* Diagnostics: shader-clock cycles summed over waves of the packed CIGAR kernel's
 * phases in the last launch: [0] query masks, [1] DP, [2] backtrack, [3] CIGAR emit. */
int pr_sw_phase_cycles(pr_ctx *ctx, int64_t *out4);

/* ------------------------------------------------------------------ */
/* host seeding front end: `bwa-proovread index` + the seeding / chaining part
 * of `bwa-proovread mem` (bin/proovread:1270, 1313), producing the pr_sw_batch
 * task list.  Restates upstream bwa's mem_collect_intv (SMEMs, re-seeding, the
 * -y third round), mem_chain / test_and_merge, mem_chain_flt and the seed choice
 * of mem_chain2aln over an exact 12-mer index of the long reads (both strands).
 * Parity with the absent bwa-proovread is unpinned.              */
typedef struct pr_seed_opts {
    int min_seed_len;        /* -k (>= 12)                                    */
    int min_chain_weight;    /* -W                                            */
    int w;                   /* -w: chaining diagonal tolerance, window gaps  */
    double split_factor;     /* -r                                            */
    int split_width;         /* bwa default 10                                */
    int max_mem_intv;        /* -y                                            */
    int max_occ;             /* -c (bwa default 500)                          */
    double drop_ratio;       /* -D                                            */
    int max_chain_gap;       /* bwa default 10000                             */
    double mask_level;       /* bwa default 0.5                               */
    int a, o_del, e_del, o_ins, e_ins;   /* scoring, for the chain window (cal_max_gap) and
                                            mem_flt_chained_seeds' seed SW            */
    int b;                   /* -B mismatch penalty (mem_flt_chained_seeds' seed SW; that
                                filter runs for reads with 1.1 W <= 0.05 length only) */
} pr_seed_opts;
typedef struct pr_seed_task {
    int32_t sr, lr;          /* short read, long read                         */
    int32_t strand;          /* 1: the read aligns to the long read's reverse complement */
    int32_t qbeg, rbeg, slen;/* seed: read offset, long-read offset in strand coordinates, length */
    int32_t rmax0, rmax1;    /* the chain's reference window (strand coordinates) */
    int32_t chain;           /* the chain among the read's kept chains (mem_chain_flt order) */
    int32_t rank;            /* the seed's place in mem_chain2aln's extension order (0 first) */
} pr_seed_task;
typedef struct pr_seed_tasks {
    int64_t n;
    pr_seed_task *t;         /* library-owned; pr_seed_tasks_free              */
} pr_seed_tasks;
typedef struct pr_seed_index pr_seed_index;
void pr_seed_opts_default(pr_seed_opts *o, int finish);   /* bwa-sr / bwa-sr-finish (proovread.cfg:318-333) */
int pr_seed_index_build(const uint8_t *lr_seq, const int64_t *lr_off, int n_lr, pr_seed_index **out);
void pr_seed_index_free(pr_seed_index *h);
/* seeds of every read, in read order and chain order (n_threads <= 0: all cores) */
int pr_seed_map(const pr_seed_index *h, const pr_seed_opts *o, const uint8_t *sr_seq, const int64_t *sr_off,
                int n_sr, int n_threads, pr_seed_tasks *out);
void pr_seed_tasks_free(pr_seed_tasks *t);
/* diagnostics (tests): occurrences of a string (both strands), and bwt_smem1a's SMEMs at x */
int pr_seed_index_occ(const pr_seed_index *h, const uint8_t *s, int n, int64_t *count);
/* order-sensitive digests of the index tables (text, koff, kpos, kext, j-mer counts,
   contig tables): a test hook proving that build changes leave the tables identical */
int pr_seed_index_digest(const pr_seed_index *h, uint64_t *out6);
/* test hooks: the k-mer offsets koff[4^12 + 1] and, for texts beyond 2^32, the first hit of
 * every k-mer at or beyond 2^32 (ksplit[4^12], left untouched otherwise); host / device index */
int pr_seed_index_koff(const pr_seed_index *h, uint64_t *koff, uint64_t *ksplit);
int pr_seed_gpu_index_koff(pr_ctx *ctx, uint64_t *koff, uint64_t *ksplit);
int pr_seed_smem(const pr_seed_index *h, const uint8_t *q, int len, int x, int64_t min_intv, int32_t *start,
                 int32_t *end, int64_t *occ, int cap, int *n_out);
/* The GPU seeding path (seed_kernels.hip: the same per-read core; pass 1 64 reads per wave,
 * pass 2 one wave per read for the reads that outgrew pass 1's scratch, up to 4 more passes with
 * the overflowed arrays grown -- hits x4, the others x2 -- for the reads that outgrew pass 2's).  pr_seed_gpu_upload
 * copies a built index into the context's HBM; pr_seed_gpu_map seeds n_sr reads (nt4 codes)
 * into library-owned tasks in read order (out = NULL: the tasks stay in HBM for
 * pr_iter_upload_gpu_seeds); status[i] (may be NULL) is 0 or the overflow flags of a read
 * whose work outgrew the scratch (it then has no tasks, and the call returns
 * PR_ERR_CAPACITY after filling everything else). */
int pr_seed_gpu_upload(pr_ctx *ctx, const pr_seed_index *h);
int pr_seed_gpu_map(pr_ctx *ctx, const pr_seed_opts *o, const uint8_t *sr_seq, const int64_t *sr_off, int n_sr,
                    pr_seed_tasks *out, int32_t *status);
/* The seed index built in the context's HBM from the long reads (bwa-proovread index,
 * proovread:1270): the tables of pr_seed_index_build byte for byte (text, 12-mer lists
 * sorted by a stable device radix sort, the bases after every hit, j-mer counts); replaces
 * pr_seed_index_build + pr_seed_gpu_upload.  lr_seq: host codes (0-3 bases, else N). */
int pr_seed_gpu_index_build(pr_ctx *ctx, const uint8_t *lr_seq, const int64_t *lr_off, int n_lr);
/* pr_seed_index_digest's six values over the device-built index (test hook) */
int pr_seed_gpu_index_digest(pr_ctx *ctx, uint64_t *out6);
/* milliseconds of the last pr_seed_gpu_index_build (HIP events on the ctx stream) */
int pr_seed_gpu_index_last_ms(pr_ctx *ctx, double *ms);
/* seeds of the last pr_seed_gpu_map (those kept in HBM when out = NULL) */
int pr_seed_gpu_seed_count(pr_ctx *ctx, int64_t *n);
/* reads of the last pr_seed_gpu_map that outgrew pass 1's small scratch slices (64 reads per
 * wave, lane per read) and ran in pass 2 (one wave per read, the large slices) */
int pr_seed_gpu_pass2_reads(pr_ctx *ctx, int64_t *n);
/* milliseconds of the last pr_seed_gpu_map kernel (HIP events on the ctx stream) */
int pr_seed_gpu_last_ms(pr_ctx *ctx, double *ms);
/* Diagnostics: wall-clock ticks (100 MHz) of the last pr_seed_gpu_map summed over waves:
 * [occurrence table, SMEMs + re-seeding, chaining, chain filter + output] */
int pr_seed_gpu_phase_ticks(pr_ctx *ctx, uint64_t *ticks4);
/* Diagnostics: pass 1's lane work summed over lanes (100 MHz ticks): [SMEM pass, re-seeding,
 * -y seeds + sort, chaining, mem_chain_flt, filter + output] */
int pr_seed_gpu_lane_ticks(pr_ctx *ctx, uint64_t *ticks6);
/* pass 1's occurrence tables (profiling): 100 MHz wave-clock ticks summed over
   waves of the start pass, the hit pass and the count table */
int pr_seed_gpu_occ_ticks(pr_ctx *ctx, uint64_t *ticks3);
/* pass 2 (profiling): reads chained on one lane (occurrences beyond the wave's slots), then
   ticks summed over waves of the wave-parallel chaining, of the one-lane chaining and of the
   chain filter; then the largest ticks of one read's occurrence table, of its SMEMs and of the
   whole read (7 values) */
int pr_seed_gpu_pass2_ticks(pr_ctx *ctx, uint64_t *t7);
/* wall time of the last pr_seed_gpu_map's second pass (the reads that outgrew pass 1's slices), ms */
int pr_seed_gpu_pass2_ms(pr_ctx *ctx, double *ms);
/* diagnostics (tests): the device path's core and capacities (its passes included) run on the host */
int pr_seed_map_device_caps(const pr_seed_index *h, const pr_seed_opts *o, const uint8_t *sr_seq,
                            const int64_t *sr_off, int n_sr, int n_threads, pr_seed_tasks *out, int32_t *status);

/* ------------------------------------------------------------------ */
/* one correction iteration on the device: SW -> assemble -> consensus  */
/* (bin/proovread:835-869 for one task: run_bwa, create_sorted_bam and
 * correct_sr_mt without the SAM/BAM round trip; the hand-off sorts the
 * reported alignments of every long read into samtools coordinate order)   */
typedef struct pr_iter_batch {
    pr_sw_batch sw;               /* tasks grouped by long read                        */
    const int64_t *task_lr_off;   /* [sw.n_lr+1]: tasks of read i are [off[i],off[i+1]) */
    const uint8_t *lr_qual;       /* phred+33 qualities of the long reads (lr_off), or NULL */
    const uint8_t *ref_seq;       /* ASCII bases of the consensus reference (bam2cns --ref, the
                                   * previous iteration's .fq; lr_off layout), or NULL: the SW long
                                   * reads (sw.lr_seq, nt4) are the reference.  Differs from the
                                   * mapping reference after masking (proovread:848-858: bwa maps
                                   * to .masked.fa, bam2cns reads the unmasked .fq)             */
} pr_iter_batch;
int pr_iter_upload(pr_ctx *ctx, const pr_iter_batch *b);
/* bwa mode straight from the device seeding: the seeds of the last pr_seed_gpu_map called with
 * out = NULL (they stay in HBM, no host round trip) are the tasks; b->sw gives the reads (the
 * same short reads, sr pool + offsets) and the long reads, its task fields are ignored. */
int pr_iter_upload_gpu_seeds(pr_ctx *ctx, const pr_iter_batch *b);
int pr_iter_launch(pr_ctx *ctx, const pr_sw_opts *o, const pr_cns_params *p);   /* async */
int pr_iter_download(pr_ctx *ctx, pr_cns_out *out);   /* consensus outputs, syncs */
/* bam2cns's chimera lines (bam2cns:488: "ID\tFROM\tTO\tRATIO\n", RATIO = npos / ntot printed as
 * Perl prints a number, %.15g) of every read with nchim > 0, reads in order, each read's rows in
 * order -- from pr_iter_download's nchim / chim_off / chim rows ([from, to, npos, ntot] int32) and
 * the reads' names (pool + [n_lr+1] offsets).  Host only; one library-allocated text
 * (pr_buffer_free).  Replaces the finish task's per-line formatting in the host language. */
int pr_fmt_chim_lines(int32_t n_lr, const char *names, const int64_t *name_off, const int32_t *nchim,
                      const int64_t *chim_off, const int32_t *chim, char **text, int64_t *len, int64_t *n_lines);
/* the outputs of reads [first, first + n) only (one bam2cns chunk's FASTQ, bam2cns:332-365;
 * a sample of a configs[3]-size batch): per-read arrays of n entries, out_off / chim_off of
 * n + 1 counted from the range's first read, pools sized by them; kept / bin_bases NULL */
int pr_iter_download_range(pr_ctx *ctx, int32_t first, int32_t n, pr_cns_out *out);
int pr_iter_bounds(pr_ctx *ctx, int32_t *n_lr, int64_t *n_task, pr_cns_bounds *bd);
/* reported alignments of the last iteration: count, total CIGAR ops, total SEQ bytes (syncs) */
int pr_iter_alignment_stats(pr_ctx *ctx, int64_t *n_aln, int64_t *sum_ncig, int64_t *sum_lseq);
int pr_iter_last_timing(pr_ctx *ctx, double *ms_sw_extend, double *ms_sw_global, double *ms_assemble,
                        double *ms_consensus);
/* The exact-parity multi-GPU layout, device-resident.  proovread maps every
 * short read against ALL long reads (bin/proovread:1270, 1313) and then corrects the long
 * reads in chunks (xargs -P, 1596-1619); across GPUs every rank holds the index of all long
 * reads, seeds and aligns a contiguous shard of the short reads (bwa mode), and sends each
 * reported alignment to the owner of its long read (contiguous long-read ranges), which then
 * runs bwa-proovread's -b/-l filter, the hand-off and the consensus for the reads it owns.
 * Because the shards are contiguous and the blocks arrive source-rank-major, the owner sees
 * every long read's alignments in the single run's order: the outputs equal one GPU's.
 *
 * 1. pr_sw_upload_gpu_seeds: the SW batch of the rank's shard from the device seeds of the last
 *    pr_seed_gpu_map(out = NULL) (b: the shard's short reads -- sr 0 is global id read_id0 --
 *    and all long reads; task fields ignored; sr_seq / lr_seq NULL: the device copies of the
 *    last pr_seed_gpu_map / pr_seed_gpu_index_build, no second upload), then pr_sw_launch.
 * 2. pr_aln_exchange: the reported alignments -> 24-byte records + CIGAR ops packed by owner on
 *    the device, the counts exchanged, one RCCL all-to-all of device buffers (comm NULL: world
 *    1, no RCCL); lr_bounds[world+1] are the owners' long-read ranges, sr0 the global id of the
 *    shard's first short read.  n_recv: records this rank received.
 * 3. pr_iter_upload_owned: the owned long reads (consensus reference, qualities) and every
 *    short read of the task (the consensus reads SEQ from it by global id); once per task --
 *    steps 1's launch, 2 and 4 may be repeated on the resident batches.
 * 4. pr_iter_launch (its SW options give -b/-l) runs filter + hand-off + consensus over the
 *    alignments the last exchange received (no SW); pr_iter_download / pr_iter_mask /
 *    pr_iter_stats as usual; pr_iter_last_timing's hand-off includes the exchange. */
int pr_sw_upload_gpu_seeds(pr_ctx *ctx, const pr_sw_batch *b);
int pr_aln_exchange(pr_ctx *ctx, pr_comm *comm, int64_t sr0, const int64_t *lr_bounds, int64_t *n_recv);
/* the same exchange among `world` contexts of ONE process (several shards on one GPU, or one
 * process driving several GPUs): every context's pack, then device copies in source order in
 * place of RCCL; sr0[k] is context k's first short read, n_recv[world] (may be NULL) */
int pr_aln_exchange_local(pr_ctx *const *ctxs, int world, const int64_t *sr0, const int64_t *lr_bounds,
                          int64_t *n_recv);
/* the last exchange's received records by source rank (per_rank[cap]; world = ranks) */
int pr_aln_exchange_sources(pr_ctx *ctx, int64_t *per_rank, int cap, int *world);
typedef struct pr_own_batch {
    int32_t lr0, n_lr;            /* owned long reads: global ids [lr0, lr0 + n_lr)          */
    const int64_t *lr_off;        /* [n_lr+1] their offsets (from 0)                          */
    const uint8_t *ref_seq;       /* ASCII consensus reference (bam2cns --ref), or NULL: the
                                   * SW batch's long reads (mapping reference = reference)    */
    const uint8_t *lr_qual;       /* phred+33 qualities (lr_off), or NULL                     */
    int32_t n_sr;                 /* every short read of the task, global ids                 */
    const int64_t *sr_off;        /* [n_sr+1]                                                 */
    const uint8_t *sr_seq;        /* nt4, or NULL when the SW batch holds every short read    */
    int32_t from_set;             /* PR_OWN_FROM_SET: reference and qualities from the resident
                                   * long-read set (pr_lrset_*; ref_seq / lr_qual ignored);
                                   * | PR_OWN_RESIDENT_SR: the short reads are the resident ones
                                   * (pr_srset_load, or the task sample of pr_srset_sample;
                                   * sr_seq NULL; no upload per task)                          */
} pr_own_batch;
enum { PR_OWN_FROM_SET = 1, PR_OWN_RESIDENT_SR = 2 };
int pr_iter_upload_owned(pr_ctx *ctx, const pr_own_batch *b);

/* The resident long-read set: the correction loop's state between tasks -- the current reads
 * (proovread's LR.fq: sequence and qualities) and their mapping reference (LR.masked.fa,
 * bin/proovread:835-869, 1700-1720) -- kept in HBM, so a task moves only its short reads
 * across PCIe.  pr_lrset_load: the read-long output (ASCII bases, phred+33 qualities); the
 * mapping reference starts as the reads.  pr_lrset_index: the seed index over the mapping
 * reference (PR_LRSET_MAP) or the reads (PR_LRSET_READS: the finish task, proovread:838-850),
 * replacing pr_seed_gpu_index_build; its long-read pool then feeds the SW batch on the device.
 * pr_iter_upload_lrset: a world-1 iteration from the seeds of the last pr_seed_gpu_map (b: the
 * short reads -- sr_seq NULL: the seeding's copy -- and read_id0; its long-read fields are
 * ignored) with the set's reads and qualities as the consensus reference (bam2cns --ref).
 * pr_lrset_commit: after pr_iter_launch (+ pr_iter_mask with with_mask): every read's
 * consensus (and quality; with_mask its masked copy as the next mapping reference) replaces
 * the set's -- a read whose consensus failed makes the call fail with its status; an owned
 * batch (pr_iter_upload_owned) needs comm: the ranks' reads are all-gathered on the device.
 * pr_lrset_download: offsets [n+1] and pools (any may be NULL; map = the mapping reference). */
enum { PR_LRSET_MAP = 0, PR_LRSET_READS = 1 };
/* pr_lrset_commit flags: MASK = the masked copy becomes the next mapping reference (a regular
 * iteration); DRY = every step of the commit (checks, compaction, the ranks' all-gathers into
 * scratch pools) without replacing the set (bench.py repeats one task on the same input) */
enum { PR_LRSET_COMMIT_MASK = 1, PR_LRSET_COMMIT_DRY = 2 };
int pr_lrset_load(pr_ctx *ctx, int32_t n_lr, const int64_t *off, const uint8_t *seq, const uint8_t *qual);
int pr_lrset_info(pr_ctx *ctx, int32_t *n_lr, int64_t *bases);
int pr_lrset_index(pr_ctx *ctx, int which);
int pr_iter_upload_lrset(pr_ctx *ctx, const pr_sw_batch *b);
int pr_lrset_commit(pr_ctx *ctx, pr_comm *comm, int flags);
int pr_lrset_download(pr_ctx *ctx, int64_t *off, uint8_t *seq, uint8_t *qual, uint8_t *map);
/* pr_lrset_snapshot: a device copy of the set's current reads and qualities (the read-long
 * output); pr_lrset_restore: the set returns to it, the mapping reference to the reads -- a
 * correction run restarted on the same input without a host round trip (bench.py: every step
 * runs the whole loop, bin/proovread:705-905, from the raw long reads) */
int pr_lrset_snapshot(pr_ctx *ctx);
int pr_lrset_restore(pr_ctx *ctx);
/* The resident short reads: the whole short-read input (nt4, in stream order) once; a task's
 * sample -- SeqChunker's chunks are contiguous record ranges (bin/proovread:2085-2102) -- is then
 * gathered on the device from ranges[2k], ranges[2k+1] (records [r0, r1)) and seeded as
 * pr_seed_gpu_map with out = NULL (the seeds and the gathered reads stay in HBM;
 * pr_iter_upload_lrset with sr_seq NULL takes them). */
int pr_srset_load(pr_ctx *ctx, int64_t n_sr, const int64_t *off, const uint8_t *seq);
int pr_seed_gpu_map_sampled(pr_ctx *ctx, const pr_seed_opts *o, const int64_t *ranges, int n_ranges, int32_t *status);
/* The task's whole sample of the resident short reads (ranges as above), gathered on the device
 * for the consensus of an owned batch: with ranks each seeds only its shard of the sample
 * (pr_seed_gpu_map_sampled over the shard's ranges), while the alignments it receives name any
 * read of the sample.  PR_OWN_RESIDENT_SR then reads this sample (its sr_off must equal the
 * sample's offsets, checked element by element); without a sample, the whole resident set.
 * pr_srset_load clears the sample. */
int pr_srset_sample(pr_ctx *ctx, const int64_t *ranges, int n_ranges);

/* enqueue (ctx stream) the per-iteration statistic of the resident consensus:
 * dev_out[0] = corrected bases, dev_out[1] = bases with phred >= min_phred.
 * dev_out is DEVICE memory (e.g. a tensor gathered with RCCL all_reduce across
 * GPUs: the global masked-fraction input of mask_shortcut_frac, proovread:2026) */
int pr_iter_stats(pr_ctx *ctx, int32_t min_phred, int64_t *dev_out);

/* ------------------------------------------------------------------ */
/* masking: `SeqFilter --phred-mask <hcr-mask> --base-content N` after every
 * iteration (bin/proovread:1701-1716).  High-confidence regions of the
 * corrected reads (quality runs in [phred_min, phred_max]) become N, minus
 * sticky ends, with read-end and gap rules (sam2cns:806-951, the in-tree
 * predecessor of SeqFilter's masking; mapping of the hcr-mask fields in
 * DESIGN.md, parity with the absent SeqFilter unpinned).  The masked reads are
 * the next iteration's bwa reference (.masked.fa, proovread:850), bpN/bpt the
 * mask_shortcut_frac input (proovread:1711-1716, 2026-2047).                 */
typedef struct pr_mask_params {
    int32_t phred_min, phred_max;  /* hcr-mask fields 0-1                              */
    int32_t mask_min_len;          /* field 2 (scaled to the short-read length)     */
    int32_t unmask_min_len;        /* field 3 (scaled)                              */
    int32_t mask_reduce;           /* field 4: bases unmasked at each HCR end       */
    double end_ratio;              /* field 5                                       */
    int32_t phred_offset;          /* --phred-offset (33)                           */
} pr_mask_params;
void pr_mask_params_default(pr_mask_params *p);   /* proovread.cfg:235 at 100 bp   */
/* "20,41,80,130,60,0.7" scaled to min_sr_length as proovread:1702-1705 does */
int pr_mask_params_parse(const char *hcr_mask, int32_t min_sr_length, pr_mask_params *out);
/* MCR capacity (pairs) of a batch of reads with offsets off[n+1] */
int pr_mask_bound(const pr_mask_params *p, int32_t n, const int64_t *off, int64_t *mcr_cap);
/* One-shot masking of n reads (ASCII seq, phred+offset qual, offsets off[n+1]):
 * out_seq[off[n]] masked bases; mcr_off[n+1] (filled) capacity prefix into mcr;
 * mcr (offset, length) pairs of read i at mcr[2*mcr_off[i]], n_mcr[i] of them;
 * stats[0] = bases, stats[1] = N bases (bpt, bpN).  Output pointers may be NULL. */
int pr_mask_run(pr_ctx *ctx, const pr_mask_params *p, int32_t n, const int64_t *off, const uint8_t *seq,
                const uint8_t *qual, uint8_t *out_seq, int64_t *mcr_off, int32_t *mcr, int32_t *n_mcr,
                int64_t *stats);
/* Mask the resident consensus of the last pr_iter_launch / pr_cns_launch (async,
 * ctx stream).  dev_stats is DEVICE int64[2] = {bases, N bases} of the reads with
 * status 0 (RCCL-reducible, like pr_iter_stats). */
int pr_iter_mask(pr_ctx *ctx, const pr_mask_params *p, int64_t *dev_stats);
/* the masked consensus of the last pr_iter_mask: seq_cap bytes laid out like
 * pr_cns_out.seq (syncs; PR_ERR_CAPACITY if a run list overflowed) */
int pr_iter_mask_download(pr_ctx *ctx, uint8_t *masked);

/* ------------------------------------------------------------------ */
/* short-read input (bin/proovread:1293, the short-read files as one stream): a FASTQ stream of
   plain 4-line records ('@' first, '\n' last, no '\r', QUAL as long as SEQ) scanned natively;
   PR_ERR_ARG for anything else (the caller's record parser takes FASTA / multi-line input).
   scan: the record and base counts; fill: every record's start offset [n_rec], the sequence
   offsets [n_rec + 1] and the bases through table256 (e.g. ASCII -> nt4) [n_bases] */
int pr_fastq4_scan(const uint8_t *data, int64_t n, int64_t *n_rec, int64_t *n_bases);
int pr_fastq4_fill(const uint8_t *data, int64_t n, const uint8_t *table256, int64_t *starts, int64_t *off,
                   uint8_t *pool);

/* final quality trimming: the windows `SeqFilter --trim-win mean,min` keeps
 * (proovread.cfg:152-155; bin/proovread:919-943), i.e. Fastq::Seq::qual_window
 * (lib/Fastq/Seq.pm:1064-1160).  Host code (once per job), threads over reads. */
typedef struct pr_trim_params {
    int32_t size;          /* Qual_window_size (10)                               */
    int32_t soft;          /* Qual_window_min_score_soft: window mean (25; --trim-win field 0) */
    int32_t hard;          /* Qual_window_min_score_hard: any position (3; field 1) */
    int32_t min_len;       /* Qual_window_min_stretch_length (10)                 */
    int32_t phred_offset;  /* 33                                                   */
} pr_trim_params;
void pr_trim_params_default(pr_trim_params *p);
int pr_trim_params_parse(const char *trim_win, pr_trim_params *p);   /* "12,5" */
/* window capacity (pairs) of a batch */
int pr_trim_bound(const pr_trim_params *p, int32_t n, const int64_t *off, int64_t *win_cap);
/* windows of read i: (offset, length) pairs at win[2*win_off[i]], n_win[i] of them, in
 * read order; win_off[n+1] is filled (capacity prefix).  n_threads <= 0: all cores. */
int pr_trim_windows(const pr_trim_params *p, int32_t n, const int64_t *off, const uint8_t *qual, int64_t *win_off,
                    int32_t *win, int32_t *n_win, int n_threads);

/* ------------------------------------------------------------------ */
/* BAM I/O for the samtools drop-in (`samtools view -bS`, bin/proovread:1313): host code.
 * pr_sam_encode: SAM text (header lines skipped) -> concatenated BAM records (each with its
 * block_size prefix), reference ids from ref_names[n_ref]; PR_ERR_SAM on a malformed line.
 * pr_bgzf_compress: BGZF blocks of 0xFF00 input bytes (raw deflate at `level`, BC field,
 * CRC32, ISIZE), no EOF marker.  Outputs are library-allocated: pr_buffer_free.
 * n_threads <= 0: all cores.                                                     */
int pr_sam_encode(const char *text, int64_t len, const char *const *ref_names, int32_t n_ref, int n_threads,
                  uint8_t **out, int64_t *out_len, int64_t *n_records);
int pr_bgzf_compress(const uint8_t *data, int64_t len, int level, int n_threads, uint8_t **out, int64_t *out_len);
/* samtools sort (bin/proovread:1338) on the host.  pr_bgzf_decompress: BGZF bytes -> the
 * uncompressed stream (blocks inflated in parallel).  pr_bam_sort_records: a stream of
 * block_size-prefixed BAM records (what follows the BAM header) in samtools coordinate
 * order — (reference id, unmapped last; POS; reverse flag), stable on equal keys.      */
int pr_bgzf_decompress(const uint8_t *data, int64_t len, int n_threads, uint8_t **out, int64_t *out_len);
int pr_bam_sort_records(const uint8_t *recs, int64_t len, int n_threads, uint8_t **out, int64_t *out_len,
                        int64_t *n_records);
/* bam2cns's BAM reader (bam2cns:336 region reads, restated as one pass): every record of a
 * BAM record stream decoded into the pr_cns_batch alignment columns — rid (-1 unmapped),
 * POS (1-based), AS:i/f/Z value and PR_ALN_* flags, SEQ as SAM prints it, QUAL phred+33
 * ('!' x l_seq when absent), BAM CIGAR ops; pools and offsets library-owned.          */
typedef struct pr_bam_alns {
    int64_t n;
    int32_t *rid, *pos1;
    double *score;
    uint8_t *flags;
    int64_t *seq_off;
    int32_t *lseq;
    int64_t *cig_off;
    int32_t *ncig;
    uint8_t *seq, *qual;
    uint32_t *cig;
    int64_t seq_len, cig_len;
} pr_bam_alns;
int pr_bam_decode_alns(const uint8_t *recs, int64_t len, int n_threads, pr_bam_alns *out);
void pr_bam_alns_free(pr_bam_alns *a);
/* `samtools index` (bin/proovread:1343-1355): the BAI bytes of a coordinate-sorted BAM file
 * (bins + chunks, pseudo-bin 37450, 16 kb linear index, no-coordinate count);
 * PR_ERR_ARG if the file is not coordinate-sorted.                                     */
int pr_bam_index(const uint8_t *data, int64_t len, int n_threads, uint8_t **out, int64_t *out_len);
void pr_buffer_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
