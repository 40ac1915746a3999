/* ORACLE — TEST INFRASTRUCTURE ONLY (see cns_oracle.c header). */
#ifndef PROOVREAD_CNS_ORACLE_H
#define PROOVREAD_CNS_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors the Sam::Seq class globals bam2cns sets (bam2cns:227-237) plus the
 * per-call consensus() options (bam2cns:434-438). */
typedef struct {
    double max_coverage;     /* Sam::Seq->MaxCoverage  (--coverage)            */
    double bin_size;         /* Sam::Seq->BinSize       (always 20, bam2cns:186) */
    int trim;                /* Sam::Seq->Trim          (cfg sr-trim = 1)       */
    int indel_taboo_length;  /* cfg sr-indel-taboo-length = 7 (0 => use frac)  */
    double indel_taboo;      /* cfg sr-indel-taboo = 0.1                        */
    int min_aln_length;      /* StateMatrixMinAlnLength = 50                    */
    int max_ins_length;      /* --max-ins-length                                */
    int fallback_phred;      /* FallbackPhred = 1                               */
    int phred_offset;        /* Sam::Seq->PhredOffset = 33 (consensus output)   */
    int ref_phred_offset;    /* phred offset of the reference FASTQ (--qv-offset) */
    int use_ref_qual;
    int qual_weighted;
    int detect_chimera;
    int invert_scores;
} ocns_params;

typedef struct {
    char *fastq;   /* "@id\nSEQ\n+\nQUAL\n" (bam2cns:453) */
    char *seq, *qual, *trace, *cigar;
    char *chim;    /* lines "id\tfrom\tto\tscore\n" (bam2cns:488) */
    int *kept;     /* per input SAM line: kept after binning */
    long *bin_bases;
    long nbins;
} ocns_result;

enum {
    OCNS_ERR_SAM = -2,
    OCNS_ERR_NOSEQ = -3,
    OCNS_ERR_BIN_RANGE = -4,
    OCNS_ERR_DIV0 = -5,
    OCNS_ERR_CIGAR = -6,
    OCNS_ERR_BEYOND_REF = -7,
};

double ocns_phred2freq(int p);
int ocns_freq2phred(double f);
/* ign: nign pairs (offset, length), Seq.pm:2063 _is_in_range ranges */
int ocns_run(const ocns_params *P, const char *id, const char *ref_seq, const char *ref_qual,
             long len, const char *const *sam, long nsam, const long *ign, int nign,
             ocns_result *R);
void ocns_free(ocns_result *R);

#ifdef __cplusplus
}
#endif
#endif
