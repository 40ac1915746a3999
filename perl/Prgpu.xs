/* Perl XS binding of libprgpu's consensus stage (include/prgpu.h).
 *
 * This is the in-process replacement a proovread maintainer binds where bin/proovread's
 * correct_sr_mt (bin/proovread:1528-1721) fans bam2cns out over `xargs -P`
 * (bin/proovread:1596-1619): one cns_run call processes a whole chunk of long reads
 * (bam2cns:332-365 for every read) on the GPU.  The Sam::Seq class globals that bam2cns
 * sets (bam2cns:227-237) arrive as a hash; the chunk arrives as the SoA buffers of
 * pr_cns_batch, packed on the Perl side (lib/Prgpu.pm) with pack().
 *
 * The seed-extension stage is bound the same way (seed_index_build / seed_map / sw_run):
 * what bin/proovread's run_bwa (bin/proovread:1254-1322) gets from a `bwa-proovread mem`
 * process, minus the SAM text round trip; lib/Prgpu.pm turns the results into the SAM
 * records bwa-proovread prints.
 *
 * The binding is thin on purpose: it checks that every packed buffer holds what the
 * batch's counts say it must (so the library never reads past a Perl string), calls
 * pr_cns_run, and hands the output pools back as packed strings.  Library errors croak
 * with pr_last_error(), as bam2cns dies through Verbose->exit (Verbose.pm:454).
 */
#define PERL_NO_GET_CONTEXT
#include "EXTERN.h"
#include "perl.h"
#include "XSUB.h"

#include <stdint.h>
#include <string.h>

#include "prgpu.h"

/* a packed batch field holding at least `need` bytes (NULL if optional and absent) */
static const char *field(pTHX_ HV *b, const char *key, size_t need, int optional, STRLEN *got) {
    SV **sv = hv_fetch(b, key, (I32)strlen(key), 0);
    STRLEN len = 0;
    const char *p;
    if (!sv || !SvOK(*sv)) {
        if (optional) {
            if (got) *got = 0;
            return NULL;
        }
        croak("Prgpu::cns_run: batch field '%s' missing", key);
    }
    p = SvPVbyte(*sv, len);
    if (len < need)
        croak("Prgpu::cns_run: batch field '%s' holds %lu bytes, %lu needed", key, (unsigned long)len,
              (unsigned long)need);
    if (got) *got = len;
    return p;
}

static double num(pTHX_ HV *h, const char *key, double dflt) {
    SV **sv = hv_fetch(h, key, (I32)strlen(key), 0);
    return (sv && SvOK(*sv)) ? SvNV(*sv) : dflt;
}

static int32_t inum(pTHX_ HV *h, const char *key, int32_t dflt) {
    SV **sv = hv_fetch(h, key, (I32)strlen(key), 0);
    return (sv && SvOK(*sv)) ? (int32_t)SvIV(*sv) : dflt;
}

/* an int64 element of a packed buffer (Perl strings are not 8-byte aligned in general) */
static int64_t i64_at(const char *p, int64_t i) {
    int64_t v;
    memcpy(&v, p + 8 * i, 8);
    return v;
}

/* a packed buffer argument holding at least `need` bytes */
static const char *arg_buf(pTHX_ SV *sv, const char *what, size_t need, STRLEN *got) {
    STRLEN len = 0;
    const char *p;
    if (!SvOK(sv)) croak("Prgpu: %s undefined", what);
    p = SvPVbyte(sv, len);
    if (len < need) croak("Prgpu: %s holds %lu bytes, %lu needed", what, (unsigned long)len, (unsigned long)need);
    if (got) *got = len;
    return p;
}

/* offsets packed as int64: n+1 entries from 0, monotone, ending within a pool of `pool` bytes */
static int64_t check_off(pTHX_ const char *off, STRLEN off_len, STRLEN pool, const char *what) {
    int64_t n, i;
    if (off_len < 8 || off_len % 8) croak("Prgpu: %s must hold n+1 int64 offsets", what);
    n = (int64_t)(off_len / 8) - 1;
    if (i64_at(off, 0) != 0) croak("Prgpu: %s must start at 0", what);
    for (i = 0; i < n; ++i)
        if (i64_at(off, i + 1) < i64_at(off, i)) croak("Prgpu: %s not monotone", what);
    if (i64_at(off, n) > (int64_t)pool) croak("Prgpu: %s ends past its sequence pool", what);
    return n;
}

/* Sam::Seq class globals (Seq.pm:114-128) as bam2cns sets them (bam2cns:227-237) */
static void fill_cns_params(pTHX_ HV *params, pr_cns_params *p) {
    pr_cns_params_default(p);
    p->max_coverage = num(aTHX_ params, "coverage", p->max_coverage);
    p->bin_size = num(aTHX_ params, "bin_size", p->bin_size);
    p->trim = inum(aTHX_ params, "trim", p->trim);
    p->indel_taboo_length = inum(aTHX_ params, "indel_taboo_length", p->indel_taboo_length);
    p->indel_taboo = num(aTHX_ params, "indel_taboo", p->indel_taboo);
    p->min_aln_length = inum(aTHX_ params, "min_aln_length", p->min_aln_length);
    p->max_ins_length = inum(aTHX_ params, "max_ins_length", p->max_ins_length);
    p->fallback_phred = inum(aTHX_ params, "fallback_phred", p->fallback_phred);
    p->phred_offset = inum(aTHX_ params, "phred_offset", p->phred_offset);
    p->ref_phred_offset = inum(aTHX_ params, "qv_offset", p->ref_phred_offset);
    p->use_ref_qual = inum(aTHX_ params, "use_ref_qual", p->use_ref_qual);
    p->qual_weighted = inum(aTHX_ params, "qual_weighted", p->qual_weighted);
    p->detect_chimera = inum(aTHX_ params, "detect_chimera", p->detect_chimera);
    p->invert_scores = inum(aTHX_ params, "invert_scores", p->invert_scores);
}

/* bwa mem scoring / band options (proovread.cfg:320-333) over the bwa-sr / finish defaults */
static void fill_sw_opts(pTHX_ HV *opts, pr_sw_opts *o) {
    pr_sw_opts_default(o, inum(aTHX_ opts, "finish", 0));
    o->a = inum(aTHX_ opts, "a", o->a);
    o->b = inum(aTHX_ opts, "b", o->b);
    o->o_del = inum(aTHX_ opts, "o_del", o->o_del);
    o->e_del = inum(aTHX_ opts, "e_del", o->e_del);
    o->o_ins = inum(aTHX_ opts, "o_ins", o->o_ins);
    o->e_ins = inum(aTHX_ opts, "e_ins", o->e_ins);
    o->w = inum(aTHX_ opts, "w", o->w);
    o->pen_clip5 = inum(aTHX_ opts, "pen_clip5", o->pen_clip5);
    o->pen_clip3 = inum(aTHX_ opts, "pen_clip3", o->pen_clip3);
    o->zdrop = inum(aTHX_ opts, "zdrop", o->zdrop);
    o->min_score_per_base = num(aTHX_ opts, "min_score_per_base", o->min_score_per_base);
    o->bin_size = inum(aTHX_ opts, "bin_size", o->bin_size);
    o->bin_length = num(aTHX_ opts, "bin_length", o->bin_length);
    o->drop_ratio = num(aTHX_ opts, "drop_ratio", o->drop_ratio);
    o->mask_level = num(aTHX_ opts, "mask_level", o->mask_level);
    o->mask_level_redun = num(aTHX_ opts, "mask_level_redun", o->mask_level_redun);
    o->max_chain_gap = inum(aTHX_ opts, "max_chain_gap", o->max_chain_gap);
}

/* consensus output pools as Perl strings (13 of them, returned as a hash of packed data) */
#define CNS_NOUT 13
static void cns_out_alloc(pTHX_ int64_t n, int64_t na, const pr_cns_bounds *bd, SV **all, pr_cns_out *o) {
    const STRLEN lens[CNS_NOUT] = {8 * (n + 1), 4 * n, 4 * n, 4 * n, 4 * n, 4 * n, bd->seq_cap, bd->seq_cap,
                                   bd->seq_cap, 4 * bd->seq_cap, 8 * (n + 1), 16 * bd->chim_cap, na};
    unsigned k;
    for (k = 0; k < CNS_NOUT; ++k) {
        all[k] = newSV(lens[k] + 1);
        SvPOK_on(all[k]);
        memset(SvPVX(all[k]), 0, lens[k] + 1);
        SvCUR_set(all[k], lens[k]);
    }
    memset(o, 0, sizeof *o);
    o->out_off = (int64_t *)SvPVX(all[0]);
    o->status = (int32_t *)SvPVX(all[1]);
    o->seq_len = (int32_t *)SvPVX(all[2]);
    o->trace_len = (int32_t *)SvPVX(all[3]);
    o->ncigar = (int32_t *)SvPVX(all[4]);
    o->nchim = (int32_t *)SvPVX(all[5]);
    o->seq = (uint8_t *)SvPVX(all[6]);
    o->qual = (uint8_t *)SvPVX(all[7]);
    o->trace = (uint8_t *)SvPVX(all[8]);
    o->cigar = (uint32_t *)SvPVX(all[9]);
    o->chim_off = (int64_t *)SvPVX(all[10]);
    o->chim = (int32_t *)SvPVX(all[11]);
    o->kept = (uint8_t *)SvPVX(all[12]);
}

static SV *cns_out_hash(pTHX_ SV **all) {
    static const char *keys[CNS_NOUT] = {"out_off", "status", "seq_len", "trace_len", "ncigar", "nchim", "seq",
                                         "qual", "trace", "cigar", "chim_off", "chim", "kept"};
    HV *res = newHV();
    unsigned k;
    for (k = 0; k < CNS_NOUT; ++k) hv_store(res, keys[k], (I32)strlen(keys[k]), all[k], 0);
    return newRV_noinc((SV *)res);
}

/* the SW batch fields of a batch hash (nt4 pools, offsets, task columns), checked */
static void fill_sw_batch(pTHX_ HV *batch, pr_sw_batch *b) {
    STRLEN lss = 0, lso = 0, lls = 0, llo = 0;
    const char *ss, *so, *ls_, *lo_;
    int64_t nt;
    memset(b, 0, sizeof *b);
    ss = field(aTHX_ batch, "sr_seq", 0, 0, &lss);
    so = field(aTHX_ batch, "sr_off", 8, 0, &lso);
    ls_ = field(aTHX_ batch, "lr_seq", 0, 0, &lls);
    lo_ = field(aTHX_ batch, "lr_off", 8, 0, &llo);
    b->n_sr = (int32_t)check_off(aTHX_ so, lso, lss, "sr_off");
    b->n_lr = (int32_t)check_off(aTHX_ lo_, llo, lls, "lr_off");
    b->sr_seq = (const uint8_t *)ss;
    b->sr_off = (const int64_t *)so;
    b->lr_seq = (const uint8_t *)ls_;
    b->lr_off = (const int64_t *)lo_;
    nt = (int64_t)num(aTHX_ batch, "n_task", -1);
    if (nt < 0) croak("Prgpu: batch field 'n_task' missing or negative");
    b->n_task = nt;
    b->t_sr = (const int32_t *)field(aTHX_ batch, "t_sr", 4 * (size_t)nt, 0, NULL);
    b->t_lr = (const int32_t *)field(aTHX_ batch, "t_lr", 4 * (size_t)nt, 0, NULL);
    b->t_strand = (const uint8_t *)field(aTHX_ batch, "t_strand", (size_t)nt, 0, NULL);
    b->t_qbeg = (const int32_t *)field(aTHX_ batch, "t_qbeg", 4 * (size_t)nt, 0, NULL);
    b->t_rbeg = (const int32_t *)field(aTHX_ batch, "t_rbeg", 4 * (size_t)nt, 0, NULL);
    b->t_slen = (const int32_t *)field(aTHX_ batch, "t_slen", 4 * (size_t)nt, 0, NULL);
    /* bwa mode: the seeds of every kept chain with their chain index (pr_seed_map order) */
    b->t_chain = (const int32_t *)field(aTHX_ batch, "t_chain", 4 * (size_t)nt, 1, NULL);
    b->read_id0 = (int64_t)num(aTHX_ batch, "read_id0", 0);
}

/* bwa mem seeding + chaining options (bin/proovread:1313, proovread.cfg:318-333) */
static void fill_seed_opts(pTHX_ HV *opts, pr_seed_opts *o) {
    pr_seed_opts_default(o, inum(aTHX_ opts, "finish", 0));
    o->min_seed_len = inum(aTHX_ opts, "min_seed_len", o->min_seed_len);
    o->min_chain_weight = inum(aTHX_ opts, "min_chain_weight", o->min_chain_weight);
    o->w = inum(aTHX_ opts, "w", o->w);
    o->split_factor = num(aTHX_ opts, "split_factor", o->split_factor);
    o->split_width = inum(aTHX_ opts, "split_width", o->split_width);
    o->max_mem_intv = inum(aTHX_ opts, "max_mem_intv", o->max_mem_intv);
    o->max_occ = inum(aTHX_ opts, "max_occ", o->max_occ);
    o->drop_ratio = num(aTHX_ opts, "drop_ratio", o->drop_ratio);
    o->a = inum(aTHX_ opts, "a", o->a);
    o->o_del = inum(aTHX_ opts, "o_del", o->o_del);
    o->e_del = inum(aTHX_ opts, "e_del", o->e_del);
    o->o_ins = inum(aTHX_ opts, "o_ins", o->o_ins);
    o->e_ins = inum(aTHX_ opts, "e_ins", o->e_ins);
    o->b = inum(aTHX_ opts, "b", o->b);
}

/* the seed index of the batch's long reads built in HBM and its short reads seeded there, the
   seeds left in HBM (pr_seed_gpu_index_build + pr_seed_gpu_map(out = NULL)): bwa-proovread
   index / mem's front end on the device */
static void gpu_seed(pTHX_ pr_ctx *cx, HV *seed_opts, const pr_sw_batch *b) {
    pr_seed_opts so;
    int rc;
    fill_seed_opts(aTHX_ seed_opts, &so);
    if ((rc = pr_seed_gpu_index_build(cx, b->lr_seq, b->lr_off, b->n_lr)) != 0)
        croak("Prgpu: pr_seed_gpu_index_build: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_seed_gpu_map(cx, &so, b->sr_seq, b->sr_off, b->n_sr, NULL, NULL)) != 0)
        croak("Prgpu: pr_seed_gpu_map: %s (%d)", pr_last_error(), rc);
}

static void pools_batch(pTHX_ HV *batch, pr_sw_batch *b) {
    STRLEN lss = 0, lso = 0, lls = 0, llo = 0;
    const char *ss = field(aTHX_ batch, "sr_seq", 0, 0, &lss), *so = field(aTHX_ batch, "sr_off", 8, 0, &lso);
    const char *ls_ = field(aTHX_ batch, "lr_seq", 0, 0, &lls), *lo_ = field(aTHX_ batch, "lr_off", 8, 0, &llo);
    memset(b, 0, sizeof *b);
    b->n_sr = (int32_t)check_off(aTHX_ so, lso, lss, "sr_off");
    b->n_lr = (int32_t)check_off(aTHX_ lo_, llo, lls, "lr_off");
    b->sr_seq = (const uint8_t *)ss;
    b->sr_off = (const int64_t *)so;
    b->lr_seq = (const uint8_t *)ls_;
    b->lr_off = (const int64_t *)lo_;
}

MODULE = Prgpu  PACKAGE = Prgpu

PROTOTYPES: DISABLE

const char *
version()
  CODE:
    RETVAL = pr_version();
  OUTPUT:
    RETVAL

const char *
last_error()
  CODE:
    RETVAL = pr_last_error();
  OUTPUT:
    RETVAL

int
device_count()
  CODE:
    int n = 0;
    if (pr_device_count(&n) != 0) n = 0;
    RETVAL = n;
  OUTPUT:
    RETVAL

IV
ctx_create(int device)
  CODE:
    pr_ctx *c = NULL;
    int rc = pr_ctx_create(device, &c);
    if (rc != 0) croak("Prgpu: pr_ctx_create: %s (%d)", pr_last_error(), rc);
    RETVAL = PTR2IV(c);
  OUTPUT:
    RETVAL

void
ctx_destroy(IV ctx)
  CODE:
    if (ctx) pr_ctx_destroy(INT2PTR(pr_ctx *, ctx));

SV *
cns_run(IV ctx, HV *params, HV *batch)
  CODE:
    pr_cns_params p;
    pr_cns_batch b;
    pr_cns_bounds bd;
    pr_cns_out o;
    const char *lr_off, *aln_off, *ign_off;
    STRLEN seq_len = 0, qual_len = 0, cig_len = 0;
    int64_t n, na, nbases, nign = 0, i;
    int rc;
    fill_cns_params(aTHX_ params, &p);

    /* the batch: every buffer checked against the counts before the library sees it */
    memset(&b, 0, sizeof b);
    n = (int64_t)inum(aTHX_ batch, "n_lr", -1);
    if (n < 0) croak("Prgpu::cns_run: batch field 'n_lr' missing or negative");
    b.n_lr = (int32_t)n;
    lr_off = field(aTHX_ batch, "lr_off", 8 * (size_t)(n + 1), 0, NULL);
    aln_off = field(aTHX_ batch, "aln_off", 8 * (size_t)(n + 1), 0, NULL);
    nbases = i64_at(lr_off, n);
    na = i64_at(aln_off, n);
    if (nbases < 0 || na < 0 || i64_at(lr_off, 0) != 0 || i64_at(aln_off, 0) != 0)
        croak("Prgpu::cns_run: lr_off / aln_off must start at 0 and end non-negative");
    b.lr_off = (const int64_t *)lr_off;
    b.aln_off = (const int64_t *)aln_off;
    b.ref_seq = (const uint8_t *)field(aTHX_ batch, "ref_seq", (size_t)nbases, 1, NULL);
    b.ref_qual = (const uint8_t *)field(aTHX_ batch, "ref_qual", (size_t)nbases, 1, NULL);
    ign_off = field(aTHX_ batch, "ign_off", 8 * (size_t)(n + 1), 1, NULL);
    if (ign_off) {
        nign = i64_at(ign_off, n);
        if (nign < 0 || i64_at(ign_off, 0) != 0) croak("Prgpu::cns_run: ign_off must start at 0");
        b.ign_off = (const int64_t *)ign_off;
        b.ign = (const int32_t *)field(aTHX_ batch, "ign", 8 * (size_t)nign, 0, NULL);
    }
    b.aln_pos = (const int32_t *)field(aTHX_ batch, "aln_pos", 4 * (size_t)na, na == 0, NULL);
    b.aln_score = (const double *)field(aTHX_ batch, "aln_score", 8 * (size_t)na, na == 0, NULL);
    b.aln_flags = (const uint8_t *)field(aTHX_ batch, "aln_flags", (size_t)na, na == 0, NULL);
    b.aln_seq_off = (const int64_t *)field(aTHX_ batch, "aln_seq_off", 8 * (size_t)na, na == 0, NULL);
    b.aln_lseq = (const int32_t *)field(aTHX_ batch, "aln_lseq", 4 * (size_t)na, na == 0, NULL);
    b.aln_cig_off = (const int64_t *)field(aTHX_ batch, "aln_cig_off", 8 * (size_t)na, na == 0, NULL);
    b.aln_ncig = (const int32_t *)field(aTHX_ batch, "aln_ncig", 4 * (size_t)na, na == 0, NULL);
    b.seq_pool = (const uint8_t *)field(aTHX_ batch, "seq_pool", 0, 1, &seq_len);
    b.qual_pool = (const uint8_t *)field(aTHX_ batch, "qual_pool", 0, 1, &qual_len);
    b.cig_pool = (const uint32_t *)field(aTHX_ batch, "cig_pool", 0, 1, &cig_len);
    if (qual_len < seq_len) croak("Prgpu::cns_run: qual_pool shorter than seq_pool");
    b.seq_pool_len = (int64_t)seq_len;
    b.cig_pool_len = (int64_t)(cig_len / 4);
    for (i = 0; i < n; ++i) {
        int64_t l0 = i64_at(lr_off, i), l1 = i64_at(lr_off, i + 1);
        int64_t a0 = i64_at(aln_off, i), a1 = i64_at(aln_off, i + 1);
        if (l1 < l0 || a1 < a0 || l1 > nbases || a1 > na) croak("Prgpu::cns_run: lr_off / aln_off not monotone");
        if (ign_off && (i64_at(ign_off, i + 1) < i64_at(ign_off, i) || i64_at(ign_off, i + 1) > nign))
            croak("Prgpu::cns_run: ign_off not monotone");
    }

    rc = pr_cns_bounds_of(&b, &bd);
    if (rc != 0) croak("Prgpu: pr_cns_bounds_of: %s (%d)", pr_last_error(), rc);
    {
        SV *all[CNS_NOUT];
        unsigned k;
        cns_out_alloc(aTHX_ n, na, &bd, all, &o);
        rc = pr_cns_run(INT2PTR(pr_ctx *, ctx), &p, &b, &o);
        if (rc != 0) {
            for (k = 0; k < CNS_NOUT; ++k) SvREFCNT_dec(all[k]);
            croak("Prgpu: pr_cns_run: %s (%d)", pr_last_error(), rc);
        }
        RETVAL = cns_out_hash(aTHX_ all);
    }
  OUTPUT:
    RETVAL

IV
seed_index_build(SV *lr_seq, SV *lr_off)
  CODE:
    STRLEN ls = 0, lo = 0;
    const char *seq = arg_buf(aTHX_ lr_seq, "lr_seq", 0, &ls);
    const char *off = arg_buf(aTHX_ lr_off, "lr_off", 8, &lo);
    const int64_t n = check_off(aTHX_ off, lo, ls, "lr_off");
    pr_seed_index *h = NULL;
    int rc = pr_seed_index_build((const uint8_t *)seq, (const int64_t *)off, (int)n, &h);
    if (rc != 0) croak("Prgpu: pr_seed_index_build: %s (%d)", pr_last_error(), rc);
    RETVAL = PTR2IV(h);
  OUTPUT:
    RETVAL

void
seed_index_free(IV ix)
  CODE:
    if (ix) pr_seed_index_free(INT2PTR(pr_seed_index *, ix));

SV *
seed_map(IV ix, HV *opts, SV *sr_seq, SV *sr_off, int threads)
  CODE:
    /* bwa mem seeding + chaining options (bin/proovread:1313, proovread.cfg:318-333) */
    pr_seed_opts o;
    pr_seed_tasks t;
    STRLEN ls = 0, lo = 0;
    const char *seq = arg_buf(aTHX_ sr_seq, "sr_seq", 0, &ls);
    const char *off = arg_buf(aTHX_ sr_off, "sr_off", 8, &lo);
    const int64_t n = check_off(aTHX_ off, lo, ls, "sr_off");
    int rc;
    if (!ix) croak("Prgpu::seed_map: no index");
    fill_seed_opts(aTHX_ opts, &o);
    rc = pr_seed_map(INT2PTR(const pr_seed_index *, ix), &o, (const uint8_t *)seq, (const int64_t *)off, (int)n,
                     threads, &t);
    if (rc != 0) croak("Prgpu: pr_seed_map: %s (%d)", pr_last_error(), rc);
    RETVAL = newSVpvn(t.n ? (const char *)t.t : "", (STRLEN)(t.n * sizeof(pr_seed_task)));
    pr_seed_tasks_free(&t);
  OUTPUT:
    RETVAL

SV *
sw_run(IV ctx, HV *opts, HV *batch)
  CODE:
    /* ksw_extend2 + ksw_global2 over the task list (bwa mem -A -B -O -E -w -L -d -T) */
    pr_sw_opts o;
    pr_sw_batch b;
    pr_sw_out out;
    int64_t nt;
    int rc;
    HV *res;
    fill_sw_opts(aTHX_ opts, &o);
    fill_sw_batch(aTHX_ batch, &b);
    {
        /* outputs, one Perl string each, per task (bwa mode: per reported alignment, SAM order,
           with the seed task and FLAG); CIGARs variable length (cigar_off prefix) */
        int64_t ctot = 0, nover = 0;
        pr_ctx *cx = INT2PTR(pr_ctx *, ctx);
        rc = pr_sw_upload(cx, &b);
        if (rc == 0) rc = pr_sw_launch(cx, &o);
        if (rc == 0) rc = pr_sw_aln_count(cx, &nt);
        if (rc == 0) rc = pr_sw_cigar_total(cx, &ctot, &nover);
        if (rc != 0) croak("Prgpu: pr_sw_run: %s (%d)", pr_last_error(), rc);
        SV *s_pos = newSV(4 * nt + 1), *s_sc = newSV(4 * nt + 1), *s_nc = newSV(4 * nt + 1),
           *s_cig = newSV(4 * (size_t)ctot + 1), *s_pass = newSV(nt + 1), *s_st = newSV(4 * nt + 1),
           *s_qb = newSV(4 * nt + 1), *s_qe = newSV(4 * nt + 1), *s_coff = newSV(8 * (size_t)(nt + 1) + 1),
           *s_task = newSV(4 * nt + 1), *s_flag = newSV(4 * nt + 1);
        SV *all[] = {s_pos, s_sc, s_nc, s_cig, s_pass, s_st, s_qb, s_qe, s_coff, s_task, s_flag};
        const STRLEN lens[] = {4 * nt, 4 * nt, 4 * nt, 4 * (size_t)ctot, nt, 4 * nt, 4 * nt, 4 * nt, 8 * (size_t)(nt + 1),
                               4 * nt, 4 * nt};
        const char *keys[] = {"pos", "score", "ncigar", "cigar", "pass", "status", "qb", "qe", "cigar_off", "task", "flag"};
        unsigned k;
        for (k = 0; k < sizeof all / sizeof all[0]; ++k) {
            SvPOK_on(all[k]);
            memset(SvPVX(all[k]), 0, lens[k] + 1);
            SvCUR_set(all[k], lens[k]);
        }
        memset(&out, 0, sizeof out);
        out.pos = (int32_t *)SvPVX(s_pos);
        out.score = (int32_t *)SvPVX(s_sc);
        out.ncigar = (int32_t *)SvPVX(s_nc);
        out.cigar = (uint32_t *)SvPVX(s_cig);
        out.cigar_cap = ctot;
        out.cigar_off = (int64_t *)SvPVX(s_coff);
        out.pass = (uint8_t *)SvPVX(s_pass);
        out.status = (int32_t *)SvPVX(s_st);
        out.qb = (int32_t *)SvPVX(s_qb);
        out.qe = (int32_t *)SvPVX(s_qe);
        out.task = (int32_t *)SvPVX(s_task);
        out.flag = (int32_t *)SvPVX(s_flag);
        rc = pr_sw_download(cx, &out);
        if (rc != 0) {
            for (k = 0; k < sizeof all / sizeof all[0]; ++k) SvREFCNT_dec(all[k]);
            croak("Prgpu: pr_sw_run: %s (%d)", pr_last_error(), rc);
        }
        res = newHV();
        for (k = 0; k < sizeof all / sizeof all[0]; ++k) hv_store(res, keys[k], (I32)strlen(keys[k]), all[k], 0);
        hv_store(res, "n", 1, newSViv((IV)nt), 0);
    }
    RETVAL = newRV_noinc((SV *)res);
  OUTPUT:
    RETVAL

SV *
mem_gpu(IV ctx, HV *seed_opts, HV *sw_opts, HV *in)
  CODE:
    /* bwa-proovread mem on the device end to end: the index and the seeds in HBM, bwa mode on
       them, the -b/-l filter on the device (pr_sw_binfilter), the SAM records formatted natively
       (pr_sw_sam) -> the record text.  in: the pools of pools_batch (nt4 codes) plus sr_text,
       sr_qual (optional), sr_names / sr_name_off, lr_names / lr_name_off, b, l, threads. */
    pr_ctx *cx = INT2PTR(pr_ctx *, ctx);
    pr_sw_batch b, ub;
    pr_sw_opts o;
    pr_sam_in si;
    STRLEN lt = 0, lq = 0, lsn = 0, lln = 0;
    const char *text, *qual;
    char *sam = NULL;
    int64_t len = 0, nrec = 0, n_aln = 0;
    int32_t bs;
    double bl;
    SV *keep = NULL;
    int rc;
    pools_batch(aTHX_ in, &b);
    fill_sw_opts(aTHX_ sw_opts, &o);
    text = field(aTHX_ in, "sr_text", (size_t)i64_at((const char *)b.sr_off, b.n_sr), 0, &lt);
    qual = field(aTHX_ in, "sr_qual", (size_t)i64_at((const char *)b.sr_off, b.n_sr), 1, &lq);
    memset(&si, 0, sizeof si);
    si.sr_off = b.sr_off;
    si.sr_text = (const uint8_t *)text;
    si.sr_qual = (const uint8_t *)qual;
    si.sr_names = field(aTHX_ in, "sr_names", 0, 0, &lsn);
    si.sr_name_off = (const int64_t *)field(aTHX_ in, "sr_name_off", 8 * ((size_t)b.n_sr + 1), 0, NULL);
    si.lr_names = field(aTHX_ in, "lr_names", 0, 0, &lln);
    si.lr_name_off = (const int64_t *)field(aTHX_ in, "lr_name_off", 8 * ((size_t)b.n_lr + 1), 0, NULL);
    if (i64_at((const char *)si.sr_name_off, b.n_sr) > (int64_t)lsn ||
        i64_at((const char *)si.lr_name_off, b.n_lr) > (int64_t)lln)
        croak("Prgpu::mem_gpu: name offsets beyond their pools");
    si.n_threads = inum(aTHX_ in, "threads", 0);
    bs = inum(aTHX_ in, "b", 0);
    bl = num(aTHX_ in, "l", 0);
    gpu_seed(aTHX_ cx, seed_opts, &b);
    ub = b;
    ub.sr_seq = NULL;   /* the seeding's device copies */
    ub.lr_seq = NULL;
    if ((rc = pr_sw_upload_gpu_seeds(cx, &ub)) != 0) croak("Prgpu: pr_sw_upload_gpu_seeds: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_sw_launch(cx, &o)) != 0) croak("Prgpu: pr_sw_launch: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_sw_aln_count(cx, &n_aln)) != 0) croak("Prgpu: pr_sw_aln_count: %s (%d)", pr_last_error(), rc);
    if (bs > 0 && bl > 0) {
        keep = newSV((STRLEN)n_aln + 1);
        SvPOK_on(keep);
        SvCUR_set(keep, (STRLEN)n_aln);
        if ((rc = pr_sw_binfilter(cx, bs, bl, (uint8_t *)SvPVX(keep))) != 0) {
            SvREFCNT_dec(keep);
            croak("Prgpu: pr_sw_binfilter: %s (%d)", pr_last_error(), rc);
        }
        si.keep = (const uint8_t *)SvPVX(keep);
    }
    rc = pr_sw_sam(cx, &si, &sam, &len, &nrec);
    if (keep) SvREFCNT_dec(keep);
    if (rc != 0) croak("Prgpu: pr_sw_sam: %s (%d)", pr_last_error(), rc);
    RETVAL = newSVpvn(len ? sam : "", (STRLEN)len);
    pr_buffer_free(sam);
  OUTPUT:
    RETVAL

SV *
iter_run_gpu(IV ctx, HV *seed_opts, HV *sw_opts, HV *params, HV *batch)
  CODE:
    /* one correction iteration with the seeding on the device too: the index and the bwa-mode
       seeds in HBM (gpu_seed), then pr_iter_upload_gpu_seeds + pr_iter_launch as iter_run */
    pr_ctx *cx = INT2PTR(pr_ctx *, ctx);
    pr_sw_opts o;
    pr_cns_params p;
    pr_iter_batch ib;
    pr_cns_bounds bd;
    pr_cns_out out;
    int32_t n_lr = 0;
    int64_t n_task = 0, nbases;
    int rc;
    fill_sw_opts(aTHX_ sw_opts, &o);
    fill_cns_params(aTHX_ params, &p);
    memset(&ib, 0, sizeof ib);
    pools_batch(aTHX_ batch, &ib.sw);
    nbases = i64_at((const char *)ib.sw.lr_off, ib.sw.n_lr);
    ib.lr_qual = (const uint8_t *)field(aTHX_ batch, "lr_qual", (size_t)nbases, 1, NULL);
    ib.ref_seq = (const uint8_t *)field(aTHX_ batch, "ref_seq", (size_t)nbases, 1, NULL);
    gpu_seed(aTHX_ cx, seed_opts, &ib.sw);
    if ((rc = pr_iter_upload_gpu_seeds(cx, &ib)) != 0)
        croak("Prgpu: pr_iter_upload_gpu_seeds: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_iter_bounds(cx, &n_lr, &n_task, &bd)) != 0) croak("Prgpu: pr_iter_bounds: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_iter_launch(cx, &o, &p)) != 0) croak("Prgpu: pr_iter_launch: %s (%d)", pr_last_error(), rc);
    {
        SV *all[CNS_NOUT];
        unsigned k;
        cns_out_alloc(aTHX_ n_lr, n_task, &bd, all, &out);
        rc = pr_iter_download(cx, &out);
        if (rc != 0) {
            for (k = 0; k < CNS_NOUT; ++k) SvREFCNT_dec(all[k]);
            croak("Prgpu: pr_iter_download: %s (%d)", pr_last_error(), rc);
        }
        RETVAL = cns_out_hash(aTHX_ all);
    }
  OUTPUT:
    RETVAL

SV *
mask_params(const char *hcr_mask, int min_sr_length)
  CODE:
    /* proovread.cfg:235 hcr-mask scaled to the short-read length (bin/proovread:1702-1705) */
    pr_mask_params p;
    HV *h = newHV();
    int rc = pr_mask_params_parse(hcr_mask, min_sr_length, &p);
    if (rc != 0) {
        SvREFCNT_dec((SV *)h);
        croak("Prgpu: pr_mask_params_parse: %s (%d)", pr_last_error(), rc);
    }
    hv_store(h, "phred_min", 9, newSViv(p.phred_min), 0);
    hv_store(h, "phred_max", 9, newSViv(p.phred_max), 0);
    hv_store(h, "mask_min_len", 12, newSViv(p.mask_min_len), 0);
    hv_store(h, "unmask_min_len", 14, newSViv(p.unmask_min_len), 0);
    hv_store(h, "mask_reduce", 11, newSViv(p.mask_reduce), 0);
    hv_store(h, "end_ratio", 9, newSVnv(p.end_ratio), 0);
    hv_store(h, "phred_offset", 12, newSViv(p.phred_offset), 0);
    RETVAL = newRV_noinc((SV *)h);
  OUTPUT:
    RETVAL

SV *
mask_run(IV ctx, HV *params, SV *seq, SV *qual, SV *off)
  CODE:
    /* SeqFilter --phred-mask on the GPU (bin/proovread:1706): masked bases, the MCRs and
       (bpt, bpN) of reads packed as ASCII seq / phred+offset qual pools with int64 offsets */
    pr_mask_params p;
    STRLEN ls = 0, lq = 0, lo = 0;
    const char *s = arg_buf(aTHX_ seq, "seq", 0, &ls);
    const char *q = arg_buf(aTHX_ qual, "qual", 0, &lq);
    const char *o = arg_buf(aTHX_ off, "off", 8, &lo);
    const int64_t n = check_off(aTHX_ o, lo, ls, "off");
    int64_t cap = 0;
    int rc;
    HV *res;
    if (lq < ls) croak("Prgpu::mask_run: qual shorter than seq");
    pr_mask_params_default(&p);
    p.phred_min = inum(aTHX_ params, "phred_min", p.phred_min);
    p.phred_max = inum(aTHX_ params, "phred_max", p.phred_max);
    p.mask_min_len = inum(aTHX_ params, "mask_min_len", p.mask_min_len);
    p.unmask_min_len = inum(aTHX_ params, "unmask_min_len", p.unmask_min_len);
    p.mask_reduce = inum(aTHX_ params, "mask_reduce", p.mask_reduce);
    p.end_ratio = num(aTHX_ params, "end_ratio", p.end_ratio);
    p.phred_offset = inum(aTHX_ params, "phred_offset", p.phred_offset);
    rc = pr_mask_bound(&p, (int32_t)n, (const int64_t *)o, &cap);
    if (rc != 0) croak("Prgpu: pr_mask_bound: %s (%d)", pr_last_error(), rc);
    {
        SV *s_out = newSV(ls + 1), *s_moff = newSV(8 * (n + 1) + 1), *s_mcr = newSV(8 * cap + 1),
           *s_nm = newSV(4 * n + 1), *s_st = newSV(16 + 1);
        SV *all[] = {s_out, s_moff, s_mcr, s_nm, s_st};
        const STRLEN lens[] = {ls, 8 * (n + 1), 8 * cap, 4 * n, 16};
        const char *keys[] = {"seq", "mcr_off", "mcr", "n_mcr", "stats"};
        unsigned k;
        for (k = 0; k < sizeof all / sizeof all[0]; ++k) {
            SvPOK_on(all[k]);
            memset(SvPVX(all[k]), 0, lens[k] + 1);
            SvCUR_set(all[k], lens[k]);
        }
        rc = pr_mask_run(INT2PTR(pr_ctx *, ctx), &p, (int32_t)n, (const int64_t *)o, (const uint8_t *)s,
                         (const uint8_t *)q, (uint8_t *)SvPVX(s_out), (int64_t *)SvPVX(s_moff),
                         (int32_t *)SvPVX(s_mcr), (int32_t *)SvPVX(s_nm), (int64_t *)SvPVX(s_st));
        if (rc != 0) {
            for (k = 0; k < sizeof all / sizeof all[0]; ++k) SvREFCNT_dec(all[k]);
            croak("Prgpu: pr_mask_run: %s (%d)", pr_last_error(), rc);
        }
        res = newHV();
        for (k = 0; k < sizeof all / sizeof all[0]; ++k) hv_store(res, keys[k], (I32)strlen(keys[k]), all[k], 0);
    }
    RETVAL = newRV_noinc((SV *)res);
  OUTPUT:
    RETVAL

SV *
iter_run(IV ctx, HV *sw_opts, HV *params, HV *batch)
  CODE:
    /* One correction iteration on the device (bin/proovread:835-869 for one task: run_bwa,
       create_sorted_bam and correct_sr_mt without the SAM/BAM files): seed extension + CIGAR
       of every task, the hand-off into samtools coordinate order, the consensus of every long
       read.  Tasks grouped by long read (task_lr_off), or bwa mode (t_chain: the seeds of every
       kept chain, grouped by short read); lr_qual / ref_seq optional. */
    pr_sw_opts o;
    pr_cns_params p;
    pr_iter_batch b;
    pr_cns_bounds bd;
    pr_cns_out out;
    int32_t n_lr = 0;
    int64_t n_task = 0, nbases, i;
    const char *tlo;
    int rc;
    fill_sw_opts(aTHX_ sw_opts, &o);
    fill_cns_params(aTHX_ params, &p);
    memset(&b, 0, sizeof b);
    fill_sw_batch(aTHX_ batch, &b.sw);
    nbases = i64_at((const char *)b.sw.lr_off, b.sw.n_lr);
    if (!b.sw.t_chain) {   /* single-seed tasks grouped by long read; bwa mode groups on the device */
        tlo = field(aTHX_ batch, "task_lr_off", 8 * (size_t)(b.sw.n_lr + 1), 0, NULL);
        if (i64_at(tlo, 0) != 0 || i64_at(tlo, b.sw.n_lr) != b.sw.n_task)
            croak("Prgpu::iter_run: task_lr_off must run from 0 to n_task");
        for (i = 0; i < b.sw.n_lr; ++i)
            if (i64_at(tlo, i + 1) < i64_at(tlo, i)) croak("Prgpu::iter_run: task_lr_off not monotone");
        b.task_lr_off = (const int64_t *)tlo;
    }
    b.lr_qual = (const uint8_t *)field(aTHX_ batch, "lr_qual", (size_t)nbases, 1, NULL);
    b.ref_seq = (const uint8_t *)field(aTHX_ batch, "ref_seq", (size_t)nbases, 1, NULL);
    if ((rc = pr_iter_upload(INT2PTR(pr_ctx *, ctx), &b)) != 0)
        croak("Prgpu: pr_iter_upload: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_iter_bounds(INT2PTR(pr_ctx *, ctx), &n_lr, &n_task, &bd)) != 0)
        croak("Prgpu: pr_iter_bounds: %s (%d)", pr_last_error(), rc);
    if ((rc = pr_iter_launch(INT2PTR(pr_ctx *, ctx), &o, &p)) != 0)
        croak("Prgpu: pr_iter_launch: %s (%d)", pr_last_error(), rc);
    {
        SV *all[CNS_NOUT];
        unsigned k;
        cns_out_alloc(aTHX_ n_lr, n_task, &bd, all, &out);
        rc = pr_iter_download(INT2PTR(pr_ctx *, ctx), &out);
        if (rc != 0) {
            for (k = 0; k < CNS_NOUT; ++k) SvREFCNT_dec(all[k]);
            croak("Prgpu: pr_iter_download: %s (%d)", pr_last_error(), rc);
        }
        RETVAL = cns_out_hash(aTHX_ all);
    }
  OUTPUT:
    RETVAL
