/* ORACLE — TEST INFRASTRUCTURE ONLY (see sw_oracle.c header). */
#ifndef PROOVREAD_SW_ORACLE_H
#define PROOVREAD_SW_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* CIGAR capacity: >= query + reference span + clips for queries up to proovread's
 * 1000 bp limit (bin/proovread:457) */
#define OSW_MAXCIG 4096

/* bwa mem options used by proovread (proovread.cfg:320-333, 343-365) */
typedef struct {
    int a, b;                  /* -A, -B                      */
    int o_del, o_ins;          /* -O d,i                      */
    int e_del, e_ins;          /* -E d,i                      */
    int w;                     /* -w                          */
    int pen_clip5, pen_clip3;  /* -L 5,3                      */
    int zdrop;                 /* -d (bwa default 100)        */
    double min_score_per_base; /* -T (proovread: per-base score, parity unpinned) */
} osw_opts;

typedef struct {
    int qb, qe;                /* query interval [qb,qe)                   */
    int rb, re;                /* reference interval in strand coordinates */
    int score, truesc, w;      /* mem_alnreg_t fields                      */
    int global_score, w2;      /* ksw_global2 score and band used          */
    int pos;                   /* 0-based leftmost forward position        */
    int n_cigar;
    uint32_t cigar[OSW_MAXCIG]; /* len<<4|op, op M0 I1 D2 S4 (BAM codes)   */
    int pass;                  /* score >= T * aligned query length        */
} osw_result;

void osw_fill_scmat(int a, int b, int8_t mat[25]);
int osw_extend(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
               const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
               int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore,
               int *max_off);
int osw_global(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
               const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
               int *n_cigar, uint32_t *cigar, int max_cigar);
/* One seed-extension task: short read `q` (nt4, length lq) against long read
 * `ref` (forward strand, nt4, length L); strand 1 = the read aligns to the
 * reverse complement; (qbeg, rbeg, slen) is the exact-match seed with rbeg in
 * strand coordinates.  Returns 0 or <0 on error. */
/* mem_alnreg_t of one extended seed (strand coordinates) */
typedef struct {
    int qb, qe, rb, re, score, truesc, w, seedlen0;
} osw_region;
int osw_extend_seed(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
                    int qbeg, int rbeg, int slen, osw_region *g);
/* mem_reg2aln: CIGAR, POS and the -T flag of a region */
int osw_reg2aln(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
                const osw_region *g, osw_result *r);
/* bwa_gen_cigar2's global score of qseg[0,lqq) against strand reference [rb,re) at band w_ */
int osw_gen_score(const osw_opts *o, int w_, const uint8_t *qseg, int lqq, const uint8_t *ref, int L, int strand,
                  int rb, int re);
int osw_task(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
             int qbeg, int rbeg, int slen, osw_result *r);

#ifdef __cplusplus
}
#endif
#endif
