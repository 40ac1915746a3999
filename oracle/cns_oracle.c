/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called
 * from the product path (proovread_amd/libprgpu.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
 * as the checker / CPU baseline.
 *
 * Plain-C restatement of proovread's consensus stage for ONE long read, i.e.
 * what bin/bam2cns does per reference sequence (bam2cns:332-365, 375-491)
 * with the Sam::Seq engine (lib/Sam/Seq.pm) and Sam::Alignment scoring
 * (lib/Sam/Alignment.pm).  Every quirk of the Perl code is reproduced:
 *
 *   - Sam::Alignment::length   Alignment.pm:417-431  (M+D if soft-clipped, else length(SEQ))
 *   - score/nscore/ncscore     Alignment.pm:525-546  (same double op order)
 *   - Sam::Seq::bin            Seq.pm:1354-1357
 *   - add_aln_by_score         Seq.pm:582-614  (strict '>' cap test, one eviction, stable insert)
 *   - remove_aln_by_iid        Seq.pm:639-659
 *   - State_matrix             Seq.pm:232-467  (S/H clip, taboo head/tail trim incl. the
 *                              tail loop that never visits op 0, D+I => mismatch, leading I,
 *                              first-seen insertion-state indices)
 *   - Phreds2freqs/Freqs2phreds Seq.pm:136-156
 *   - state_matrix_consensus   Seq.pm:1568-1654 (first strictly-greater argmax)
 *   - Trace2cigar              Seq.pm:206-225
 *   - chimera + Hx             Seq.pm:774-889, 188-197
 *   - detect_chimera           bam2cns:461-491 (m//g pos() quirk: a token failing the
 *                              '< from' test is consumed; an exhausted regex restarts)
 *
 * Canonicalisation: the Perl engine iterates alignments in
 * hash order (Seq.pm:1278-1287); this restatement iterates them in ascending
 * internal id (= arrival) order, which is one of the outputs the reference
 * can produce and the one the golden fixtures were generated with
 * (tests/golden/gen_cns_golden.pl overrides Sam::Seq::alns the same way).
 *
 * Parity pinned: tests/test_oracle_cns.py checks this file against golden
 * vectors produced by running the reference Perl modules in this container.
 */
#include <ctype.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cns_oracle.h"

/* ------------------------------------------------------------------------ */
/* small growable string                                                     */
typedef struct { char *s; size_t n, cap; } ostr;
static void os_putn(ostr *o, const char *s, size_t n) {
    if (o->n + n + 1 > o->cap) {
        size_t c = o->cap ? o->cap : 64;
        while (c < o->n + n + 1) c *= 2;
        o->s = (char *)realloc(o->s, c);
        o->cap = c;
    }
    memcpy(o->s + o->n, s, n);
    o->n += n;
    o->s[o->n] = 0;
}
static void os_putc(ostr *o, char c) { os_putn(o, &c, 1); }
static void os_puts(ostr *o, const char *s) { os_putn(o, s, strlen(s)); }

/* ------------------------------------------------------------------------ */
/* Seq.pm:151-156  Phreds2freqs: int(((p**2/120)*100)+.5)/100                */
double ocns_phred2freq(int p) {
    double x = ((double)p * (double)p / 120.0) * 100.0 + 0.5;
    return (double)(long long)x / 100.0;   /* Perl int() truncates toward 0 */
}
/* Seq.pm:136-142  Freqs2phreds: min(40, int(sqrt(f*120)+.5))               */
int ocns_freq2phred(double f) {
    double x = sqrt(f * 120.0) + 0.5;
    long long p = (long long)x;
    return p > 40 ? 40 : (int)p;
}

/* ------------------------------------------------------------------------ */
/* parsed SAM record (Alignment.pm:87-110: split("\t", $line, 12))           */
typedef struct {
    long pos;
    char *cigar, *seq, *qual;
    int has_score;
    double score;
    long length;   /* Alignment.pm:417 cached length */
    long iid;
    int removed;
} oaln;

static char *dupn(const char *s, size_t n) {
    char *r = (char *)malloc(n + 1);
    memcpy(r, s, n);
    r[n] = 0;
    return r;
}

static int parse_sam(const char *line, oaln *a, int invert_scores) {
    const char *f[12];
    size_t fl[12];
    int nf = 0;
    size_t L = strlen(line);
    while (L && (line[L - 1] == '\n' || line[L - 1] == '\r')) {
        if (line[L - 1] == '\r') break;  /* chomp removes only \n */
        L--;
    }
    const char *p = line, *end = line + L;
    while (nf < 12) {
        const char *t = (nf == 11) ? end : memchr(p, '\t', (size_t)(end - p));
        if (!t) t = end;
        f[nf] = p;
        fl[nf] = (size_t)(t - p);
        nf++;
        if (t >= end) break;
        p = t + 1;
    }
    if (nf < 11) return -1;
    memset(a, 0, sizeof(*a));
    char tmp[32];
    size_t n = fl[3] < 31 ? fl[3] : 31;
    memcpy(tmp, f[3], n);
    tmp[n] = 0;
    a->pos = strtol(tmp, NULL, 10);
    a->cigar = dupn(f[5], fl[5]);
    a->seq = dupn(f[9], fl[9]);
    a->qual = dupn(f[10], fl[10]);
    a->has_score = 0;
    if (nf == 12) {
        /* Alignment.pm:341-382 opt(): split on \t, key = substr(0,2), value = substr(5) */
        const char *q = f[11], *qe = f[11] + fl[11];
        while (q < qe) {
            const char *t = memchr(q, '\t', (size_t)(qe - q));
            if (!t) t = qe;
            if (t - q >= 2 && q[0] == 'A' && q[1] == 'S') {
                if (t - q > 5) {
                    char *v = dupn(q + 5, (size_t)(t - q - 5));
                    a->score = strtod(v, NULL);
                    free(v);
                } else {
                    a->score = 0;
                }
                a->has_score = 1;   /* last AS wins like a hash assignment */
            }
            q = t + 1;
        }
    }
    if (a->has_score && invert_scores) a->score = a->score * -1;
    /* Alignment.pm:417-431 */
    size_t cl = strlen(a->cigar);
    int clipped = 0;
    {
        size_t i = 0;
        while (i < cl && isdigit((unsigned char)a->cigar[i])) i++;
        if (i > 0 && i < cl && a->cigar[i] == 'S') clipped = 1;
        if (cl && a->cigar[cl - 1] == 'S') clipped = 1;
    }
    if (strcmp(a->seq, "*") == 0 || clipped) {
        long l = 0;
        size_t i = 0;
        while (i < cl) {
            if (isdigit((unsigned char)a->cigar[i])) {
                size_t j = i;
                long v = 0;
                while (j < cl && isdigit((unsigned char)a->cigar[j])) v = v * 10 + (a->cigar[j++] - '0');
                if (j < cl && (a->cigar[j] == 'M' || a->cigar[j] == 'D')) l += v;
                i = j;
            } else i++;
        }
        a->length = l;
    } else {
        a->length = (long)strlen(a->seq);
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* state string -> index map (Seq.pm:531-539 fixed states + dynamic ones)    */
typedef struct { char **key; int *val; int cap, n; } smap;
static uint64_t shash(const char *s) {
    uint64_t h = 1469598103934665603ULL;
    while (*s) { h ^= (unsigned char)*s++; h *= 1099511628211ULL; }
    return h;
}
static void smap_init(smap *m) {
    m->cap = 64; m->n = 0;
    m->key = (char **)calloc((size_t)m->cap, sizeof(char *));
    m->val = (int *)calloc((size_t)m->cap, sizeof(int));
}
static void smap_free(smap *m) {
    for (int i = 0; i < m->cap; i++) free(m->key[i]);
    free(m->key); free(m->val);
}
static int *smap_find(smap *m, const char *k) {
    int i = (int)(shash(k) & (uint64_t)(m->cap - 1));
    while (m->key[i]) {
        if (strcmp(m->key[i], k) == 0) return &m->val[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}
static void smap_put(smap *m, const char *k, int v);
static void smap_grow(smap *m) {
    smap o = *m;
    m->cap *= 2; m->n = 0;
    m->key = (char **)calloc((size_t)m->cap, sizeof(char *));
    m->val = (int *)calloc((size_t)m->cap, sizeof(int));
    for (int i = 0; i < o.cap; i++) if (o.key[i]) { smap_put(m, o.key[i], o.val[i]); free(o.key[i]); }
    free(o.key); free(o.val);
}
static void smap_put(smap *m, const char *k, int v) {
    if ((m->n + 1) * 2 > m->cap) smap_grow(m);
    int i = (int)(shash(k) & (uint64_t)(m->cap - 1));
    while (m->key[i]) {
        if (strcmp(m->key[i], k) == 0) { m->val[i] = v; return; }
        i = (i + 1) & (m->cap - 1);
    }
    m->key[i] = strdup(k); m->val[i] = v; m->n++;
}
static void smap_copy(smap *dst, const smap *src) {
    smap_init(dst);
    for (int i = 0; i < src->cap; i++) if (src->key[i]) smap_put(dst, src->key[i], src->val[i]);
}

/* ------------------------------------------------------------------------ */
/* state matrix: columns of (possibly undef) doubles                          */
typedef struct { double *v; unsigned char *def; int n, cap; } ocol;
typedef struct { ocol *c; long n, cap; } omat;

static void mat_init(omat *m, long len) {
    m->cap = len > 16 ? len : 16;
    m->n = len;
    m->c = (ocol *)calloc((size_t)m->cap, sizeof(ocol));
}
static void mat_free(omat *m) {
    for (long i = 0; i < m->cap; i++) { free(m->c[i].v); free(m->c[i].def); }
    free(m->c);
}
static void mat_add(omat *m, long col, int idx, double x) {
    if (col >= m->cap) {
        long nc = m->cap;
        while (nc <= col) nc *= 2;
        m->c = (ocol *)realloc(m->c, (size_t)nc * sizeof(ocol));
        memset(m->c + m->cap, 0, (size_t)(nc - m->cap) * sizeof(ocol));
        m->cap = nc;
    }
    if (col >= m->n) m->n = col + 1;   /* Perl autovivification */
    ocol *c = &m->c[col];
    if (idx >= c->cap) {
        int nc = c->cap ? c->cap : 8;
        while (nc <= idx) nc *= 2;
        c->v = (double *)realloc(c->v, (size_t)nc * sizeof(double));
        c->def = (unsigned char *)realloc(c->def, (size_t)nc);
        memset(c->def + c->cap, 0, (size_t)(nc - c->cap));
        c->cap = nc;
    }
    if (idx >= c->n) c->n = idx + 1;
    if (!c->def[idx]) { c->def[idx] = 1; c->v[idx] = 0.0; }
    c->v[idx] += x;   /* ($S[$rpos][$idx]) += x */
}

/* ------------------------------------------------------------------------ */
typedef struct {
    const ocns_params *P;
    const char *id;
    const char *ref_seq;    /* may be NULL */
    const char *ref_qual;   /* may be NULL */
    long len;
    double bin_size, bin_max_bases;
    long nbins;
    /* per-bin sorted lists (Seq.pm:1437-1444) */
    double **bscore; long **bid; long **blen; int *bn, *bcap;
    long *bin_bases;
    oaln *alns; long nalns;   /* indexed by iid-1 */
    smap states;
    omat S;
} osseq;

static long bin_of(const osseq *s, const oaln *a) {
    double c = ((double)a->pos + ((double)a->length / 2.0)) / s->bin_size;
    return (long)c;   /* int() */
}

static void bin_insert(osseq *s, long b, int at, double sc, long id, long ln) {
    if (s->bn[b] + 1 > s->bcap[b]) {
        int nc = s->bcap[b] ? s->bcap[b] * 2 : 8;
        s->bscore[b] = (double *)realloc(s->bscore[b], (size_t)nc * sizeof(double));
        s->bid[b] = (long *)realloc(s->bid[b], (size_t)nc * sizeof(long));
        s->blen[b] = (long *)realloc(s->blen[b], (size_t)nc * sizeof(long));
        s->bcap[b] = nc;
    }
    int n = s->bn[b];
    memmove(s->bscore[b] + at + 1, s->bscore[b] + at, (size_t)(n - at) * sizeof(double));
    memmove(s->bid[b] + at + 1, s->bid[b] + at, (size_t)(n - at) * sizeof(long));
    memmove(s->blen[b] + at + 1, s->blen[b] + at, (size_t)(n - at) * sizeof(long));
    s->bscore[b][at] = sc; s->bid[b][at] = id; s->blen[b][at] = ln;
    s->bn[b] = n + 1;
}

/* Seq.pm:639-659 */
static void remove_aln_by_iid(osseq *s, long iid) {
    oaln *a = &s->alns[iid - 1];
    if (a->removed) return;
    a->removed = 1;
    long b = bin_of(s, a);
    int n = s->bn[b];
    for (int i = 0; i < n; i++) {
        if (s->bid[b][i] == iid) {
            long rm = s->blen[b][i];
            memmove(s->bscore[b] + i, s->bscore[b] + i + 1, (size_t)(n - i - 1) * sizeof(double));
            memmove(s->bid[b] + i, s->bid[b] + i + 1, (size_t)(n - i - 1) * sizeof(long));
            memmove(s->blen[b] + i, s->blen[b] + i + 1, (size_t)(n - i - 1) * sizeof(long));
            s->bn[b] = n - 1;
            s->bin_bases[b] -= rm;
            return;
        }
    }
}

/* Seq.pm:582-614. returns iid (>0), 0 rejected, -1 undef score, <-1 error */
static long add_aln_by_score(osseq *s, oaln *a) {
    long b = bin_of(s, a);
    if (!a->has_score) return -1;
    if (a->length == 0) return OCNS_ERR_DIV0;
    double ns = a->score / (double)a->length;
    double nc = ns * ((double)a->length / (double)(40 + a->length));
    if (b < 0 || b >= s->nbins) return OCNS_ERR_BIN_RANGE;  /* Perl dies (strict refs) */
    if ((double)s->bin_bases[b] > s->bin_max_bases) {
        if (nc <= s->bscore[b][s->bn[b] - 1]) return 0;
        remove_aln_by_iid(s, s->bid[b][s->bn[b] - 1]);
    }
    s->bin_bases[b] += a->length;
    long id = ++s->nalns;
    a->iid = id;
    s->alns[id - 1] = *a;
    int i = s->bn[b] - 1;
    while (i >= 0 && nc > s->bscore[b][i]) i--;
    bin_insert(s, b, i + 1, nc, id, a->length);
    return id;
}

static int in_ranges(long v, const long *rg, int nrg) {
    for (int i = 0; i < nrg; i++)
        if (v >= rg[2 * i] && v < rg[2 * i] + rg[2 * i + 1]) return 1;
    return 0;
}

/* cigar "10M2I" -> parallel arrays (split(/(\d+)/) semantics for well-formed cigars) */
typedef struct { long n; char op; } cop;
static int split_cigar(const char *c, cop **out) {
    int cap = 16, n = 0;
    cop *v = (cop *)malloc((size_t)cap * sizeof(cop));
    size_t i = 0, L = strlen(c);
    while (i < L) {
        long x = 0;
        size_t j = i;
        while (j < L && isdigit((unsigned char)c[j])) x = x * 10 + (c[j++] - '0');
        if (j == i || j >= L) { free(v); return -1; }
        if (n == cap) { cap *= 2; v = (cop *)realloc(v, (size_t)cap * sizeof(cop)); }
        v[n].n = x; v[n].op = c[j]; n++;
        i = j + 1;
    }
    *out = v;
    return n;
}

static double min_freq_of_qual(const char *q, size_t n, int po) {
    if (n == 0) return 0.0;   /* min() of empty list is undef -> += adds 0 */
    double m = 0;
    for (size_t i = 0; i < n; i++) {
        double f = ocns_phred2freq((int)(unsigned char)q[i] - po);
        if (i == 0 || f < m) m = f;
    }
    return m;
}

typedef struct { char *st; char *sq; } ostate;

/* Seq.pm:232-467 State_matrix. Adds into *S (already sized) using/extending *states. */
static int state_matrix(osseq *s, omat *S, smap *states, long *ids, long nids,
                        int use_ref_qual, const long *ign, int nign, int qual_weighted) {
    const ocns_params *P = s->P;
    if (use_ref_qual && s->ref_seq) {
        size_t rl = strlen(s->ref_seq);
        size_t ql = s->ref_qual ? strlen(s->ref_qual) : 0;
        for (size_t i = 0; i < rl; i++) {
            if (i >= ql) continue;
            double f = ocns_phred2freq((int)(unsigned char)s->ref_qual[i] - P->ref_phred_offset);
            if (!(f != 0.0)) continue;
            char k[2] = {s->ref_seq[i], 0};
            int *ix = smap_find(&s->states, k);   /* self->{_states} */
            mat_add(S, (long)i, ix ? *ix : 0, f);
        }
    }
    for (long ai = 0; ai < nids; ai++) {
        oaln *a = &s->alns[ids[ai] - 1];
        char *seq = a->seq;
        size_t orig = strlen(seq);
        if (!((long)orig > P->min_aln_length)) continue;
        char *qua;
        int qfree = 0;
        if (strcmp(a->qual, "*") == 0) {
            qua = (char *)malloc(orig + 1);
            memset(qua, (char)(P->fallback_phred + P->phred_offset), orig);
            qua[orig] = 0;
            qfree = 1;
        } else qua = a->qual;
        size_t qlen_all = strlen(qua);
        cop *cg;
        int nc = split_cigar(a->cigar, &cg);
        if (nc <= 0) { if (qfree) free(qua); return OCNS_ERR_CIGAR; }
        /* work on [sb, se) windows of seq/qua */
        size_t sb = 0, se = orig, qb = 0, qe = qlen_all;
        int cb = 0, ce = nc;   /* active cigar ops [cb, ce) */
        if (cg[cb].op == 'S') {
            size_t k = (size_t)cg[cb].n;
            sb = k < orig ? k : orig;      /* substr($seq, n) */
            qb = k < qlen_all ? k : qlen_all;
            cb++;
        }
        if (ce > cb && cg[ce - 1].op == 'S') {
            size_t k = (size_t)cg[ce - 1].n;
            se = (se - sb) > k ? se - k : sb;
            qe = (qe - qb) > k ? qe - k : qb;
            ce--;
        }
        if (ce > cb && cg[cb].op == 'H') cb++;
        if (ce > cb && cg[ce - 1].op == 'H') ce--;
        if (ce <= cb) { free(cg); if (qfree) free(qua); return OCNS_ERR_CIGAR; }
        long rpos = a->pos - 1;
        if (P->trim) {
            long mc = 0, dc = 0, ic = 0;
            long taboo = P->indel_taboo_length ? P->indel_taboo_length
                                               : (long)((double)orig * P->indel_taboo + 0.5);
            for (int i = cb; i < ce; i++) {
                char op = cg[i].op;
                if (op == 'M') {
                    if (mc + ic + cg[i].n > taboo) {
                        if (i > cb) {
                            cb = i;
                            rpos += mc + dc;
                            size_t cut = (size_t)(mc + ic);
                            sb = (se - sb) > cut ? sb + cut : se;
                            qb = (qe - qb) > cut ? qb + cut : qe;
                        }
                        break;
                    }
                    mc += cg[i].n;
                } else if (op == 'D') dc += cg[i].n;
                else if (op == 'I') ic += cg[i].n;
                else { free(cg); if (qfree) free(qua); return OCNS_ERR_CIGAR; }
            }
            if ((long)(se - sb) < 50 || ((double)(se - sb) / (double)orig) < 0.7) {
                free(cg); if (qfree) free(qua); continue;
            }
            long tail = 0;
            for (int i = ce - 1; i != cb; i--) {   /* for ($i=$#cigar-1; $i; $i-=2) */
                char op = cg[i].op;
                if (op == 'M') {
                    tail += cg[i].n;
                    if (tail > taboo) {
                        if (i < ce - 1) {
                            long cut = tail - cg[i].n;
                            ce = i + 1;
                            se = (long)(se - sb) > cut ? se - (size_t)cut : sb;
                            qe = (long)(qe - qb) > cut ? qe - (size_t)cut : qb;
                        }
                        break;
                    }
                } else if (op == 'D') {
                } else if (op == 'I') tail += cg[i].n;
                else { free(cg); if (qfree) free(qua); return OCNS_ERR_CIGAR; }
            }
            if ((long)(se - sb) < P->min_aln_length || ((double)(se - sb) / (double)orig) < 0.7) {
                free(cg); if (qfree) free(qua); continue;
            }
        }
        /* cigar -> states (Seq.pm:390-432) */
        long cap = 16, ns = 0;
        ostate *st = (ostate *)calloc((size_t)cap, sizeof(ostate));
        size_t qpos = 0;
        const char *sv = seq + sb;
        size_t svl = se - sb;
        const char *qv = qua + qb;
        size_t qvl = qe - qb;
#define SUBSTR(buf, bl, off, n, out) do { size_t _o = (off) < (bl) ? (off) : (bl); \
            size_t _n = (size_t)(n); if (_o + _n > (bl)) _n = (bl) - _o; out = dupn((buf) + _o, _n); } while (0)
#define PUSH_STATE(S_, Q_) do { if (ns == cap) { cap *= 2; st = (ostate *)realloc(st, (size_t)cap * sizeof(ostate)); } \
            st[ns].st = (S_); st[ns].sq = (Q_); ns++; } while (0)
        int err = 0;
        for (int i = cb; i < ce; i++) {
            char op = cg[i].op;
            long n = cg[i].n;
            if (op == 'M') {
                for (long k = 0; k < n; k++) {
                    size_t o = qpos + (size_t)k;
                    if (o >= svl) break;     /* split(//, substr(...)) of a short tail */
                    char *x = dupn(sv + o, 1);
                    char *y = NULL;
                    if (qual_weighted) y = (o < qvl) ? dupn(qv + o, 1) : dupn("", 0);
                    PUSH_STATE(x, y);
                }
                qpos += (size_t)n;
            } else if (op == 'D') {
                char *qd = NULL;
                if (qual_weighted) {
                    char qbf, qaf;
                    qbf = qpos > 1 ? (qpos - 1 < qvl ? qv[qpos - 1] : 0) : (qpos < qvl ? qv[qpos] : 0);
                    qaf = qpos < qvl ? qv[qpos] : (qpos >= 1 && qpos - 1 < qvl ? qv[qpos - 1] : 0);
                    char qq = (unsigned char)qbf < (unsigned char)qaf ? qbf : qaf;
                    qd = dupn(&qq, qq ? 1 : 0);
                }
                for (long k = 0; k < n; k++) PUSH_STATE(dupn("-", 1), qd ? dupn(qd, strlen(qd)) : NULL);
                free(qd);
            } else if (op == 'I') {
                char *ins, *iq = NULL;
                SUBSTR(sv, svl, qpos, n, ins);
                if (qual_weighted) SUBSTR(qv, qvl, qpos, n, iq);
                if (i > cb) {
                    if (ns == 0) { free(ins); free(iq); err = 1; break; }
                    ostate *l = &st[ns - 1];
                    if (strcmp(l->st, "-") == 0) {
                        free(l->st); l->st = ins;
                        if (qual_weighted) { free(l->sq); l->sq = iq; iq = NULL; }
                    } else {
                        size_t a1 = strlen(l->st), a2 = strlen(ins);
                        l->st = (char *)realloc(l->st, a1 + a2 + 1);
                        memcpy(l->st + a1, ins, a2 + 1);
                        free(ins);
                        if (qual_weighted) {
                            size_t b1 = l->sq ? strlen(l->sq) : 0, b2 = strlen(iq);
                            l->sq = (char *)realloc(l->sq, b1 + b2 + 1);
                            memcpy(l->sq + b1, iq, b2 + 1);
                        }
                    }
                    free(iq);
                } else {
                    if (ns == 0) PUSH_STATE(ins, iq);
                    else { free(st[0].st); free(st[0].sq); st[0].st = ins; st[0].sq = iq; }
                }
                qpos += (size_t)n;
            } else { err = 1; break; }
        }
        if (err) {
            for (long k = 0; k < ns; k++) { free(st[k].st); free(st[k].sq); }
            free(st); free(cg); if (qfree) free(qua);
            return OCNS_ERR_CIGAR;
        }
        /* states -> matrix (Seq.pm:438-461) */
        for (long k = 0; k < ns; k++) {
            if (nign && in_ranges(rpos, ign, nign)) { rpos++; continue; }
            const char *state = st[k].st;
            if (strlen(state) > 1 && !smap_find(states, state)) smap_put(states, state, states->n);
            int *ix = smap_find(states, state);
            double x = 1.0;
            if (qual_weighted) x = min_freq_of_qual(st[k].sq, st[k].sq ? strlen(st[k].sq) : 0, P->phred_offset);
            if (rpos < 0) { err = 1; break; }
            mat_add(S, rpos, ix ? *ix : 0, x);
            rpos++;
        }
        for (long k = 0; k < ns; k++) { free(st[k].st); free(st[k].sq); }
        free(st); free(cg); if (qfree) free(qua);
        if (err) return OCNS_ERR_CIGAR;
#undef SUBSTR
#undef PUSH_STATE
    }
    return 0;
}

/* canonical alignment iteration order: ascending iid */
static long kept_ids(osseq *s, long **out) {
    long *v = (long *)malloc((size_t)(s->nalns + 1) * sizeof(long));
    long n = 0;
    for (long i = 0; i < s->nalns; i++) if (!s->alns[i].removed) v[n++] = s->alns[i].iid;
    *out = v;
    return n;
}

/* Seq.pm:188-197 Hx over the values of a column (undef/0 omitted) */
static double Hx(const double *v, const unsigned char *def, int n) {
    double total = 0;
    for (int i = 0; i < n; i++) if (def[i] && v[i] != 0.0) total += v[i];
    double h = 0.0;
    for (int i = 0; i < n; i++) {
        if (!(def[i] && v[i] != 0.0)) continue;
        double p = v[i] / total;
        h -= p * (log(p) / log(2.0));
    }
    return h;
}

int ocns_run(const ocns_params *P, const char *id, const char *ref_seq, const char *ref_qual,
             long len, const char *const *sam, long nsam, const long *ign, int nign,
             ocns_result *R) {
    memset(R, 0, sizeof(*R));
    osseq s;
    memset(&s, 0, sizeof(s));
    s.P = P; s.id = id; s.ref_seq = ref_seq; s.ref_qual = ref_qual; s.len = len;
    s.bin_size = P->bin_size;
    s.bin_max_bases = P->bin_size * P->max_coverage;
    s.nbins = (long)((double)len / s.bin_size) + 1;
    s.bscore = (double **)calloc((size_t)s.nbins, sizeof(double *));
    s.bid = (long **)calloc((size_t)s.nbins, sizeof(long *));
    s.blen = (long **)calloc((size_t)s.nbins, sizeof(long *));
    s.bn = (int *)calloc((size_t)s.nbins, sizeof(int));
    s.bcap = (int *)calloc((size_t)s.nbins, sizeof(int));
    s.bin_bases = (long *)calloc((size_t)s.nbins, sizeof(long));
    s.alns = (oaln *)calloc((size_t)(nsam + 1), sizeof(oaln));
    smap_init(&s.states);
    const char *fixed[6] = {"A", "T", "G", "C", "-", "N"};
    for (int i = 0; i < 6; i++) smap_put(&s.states, fixed[i], i);
    int rc = 0;
    R->kept = (int *)calloc((size_t)(nsam + 1), sizeof(int));
    long *arrival_to_iid = (long *)calloc((size_t)(nsam + 1), sizeof(long));
    for (long i = 0; i < nsam; i++) {
        oaln a;
        if (parse_sam(sam[i], &a, P->invert_scores)) { rc = OCNS_ERR_SAM; goto done; }
        if (strcmp(a.seq, "*") == 0) {   /* bam2cns:347 */
            free(a.cigar); free(a.seq); free(a.qual);
            rc = OCNS_ERR_NOSEQ; goto done;
        }
        long r = add_aln_by_score(&s, &a);
        if (r < -1) { free(a.cigar); free(a.seq); free(a.qual); rc = (int)r; goto done; }
        if (r <= 0) { free(a.cigar); free(a.seq); free(a.qual); }
        arrival_to_iid[i] = r > 0 ? r : 0;
    }
    for (long i = 0; i < nsam; i++) {
        long iid = arrival_to_iid[i];
        R->kept[i] = (iid > 0 && !s.alns[iid - 1].removed) ? 1 : 0;
    }
    R->nbins = s.nbins;
    R->bin_bases = (long *)malloc((size_t)s.nbins * sizeof(long));
    memcpy(R->bin_bases, s.bin_bases, (size_t)s.nbins * sizeof(long));

    /* consensus (Seq.pm:714-734) */
    long *ids;
    long nk = kept_ids(&s, &ids);
    mat_init(&s.S, len);
    {
        smap st2;
        smap_copy(&st2, &s.states);
        rc = state_matrix(&s, &s.S, &st2, ids, nk, P->use_ref_qual, ign, nign, P->qual_weighted);
        smap_free(&s.states);
        s.states = st2;   /* _init_state_matrix stores the extended states */
    }
    if (rc) { free(ids); goto done; }
    if (s.S.n > len) { rc = OCNS_ERR_BEYOND_REF; free(ids); goto done; }

    /* state_matrix_consensus (Seq.pm:1568-1654) */
    ostr seq = {0}, trace = {0}, qual = {0};
    int nstates = s.states.n;
    const char **rev = (const char **)calloc((size_t)nstates + 1, sizeof(char *));
    for (int i = 0; i < s.states.cap; i++) if (s.states.key[i]) rev[s.states.val[i]] = s.states.key[i];
    for (long c = 0; c < s.S.n; c++) {
        ocol *col = &s.S.c[c];
        char refc = (ref_seq && c < (long)strlen(ref_seq)) ? ref_seq[c] : 'n';
        if (col->n == 0) {
            os_putc(&seq, ref_seq ? refc : 'n');
            os_putc(&qual, (char)(ocns_freq2phred(0.0) + P->phred_offset));
            os_putc(&trace, 'M');
            continue;
        }
        int idx = -1;
        double maxf = 0;
        for (int i = 0; i < col->n; i++) {
            if (!col->def[i]) continue;
            double f = col->v[i];
            if (f > maxf) {
                if (P->max_ins_length && i > 4 && (long)strlen(rev[i]) > P->max_ins_length) continue;
                maxf = f;
                idx = i;
            }
        }
        if (!(maxf != 0.0)) {
            os_putc(&seq, ref_seq ? refc : 'n');
            os_putc(&qual, (char)(ocns_freq2phred(0.0) + P->phred_offset));
            os_putc(&trace, 'M');
            continue;
        }
        if (idx == 4) { os_putc(&trace, 'I'); continue; }
        const char *con = rev[idx];
        size_t cl = strlen(con);
        os_puts(&seq, con);
        char qc = (char)(ocns_freq2phred(maxf) + P->phred_offset);
        for (size_t k = 0; k < cl; k++) os_putc(&qual, qc);
        os_putc(&trace, 'M');
        for (size_t k = 1; k < cl; k++) os_putc(&trace, 'D');
    }
    free(rev);
    /* Trace2cigar (Seq.pm:206-225) */
    ostr cig = {0};
    for (size_t i = 0; i < trace.n;) {
        size_t j = i;
        while (j < trace.n && trace.s[j] == trace.s[i]) j++;
        char b[32];
        snprintf(b, sizeof b, "%zu%c", j - i, trace.s[i]);
        os_puts(&cig, b);
        i = j;
    }
    ostr fq = {0};
    os_putc(&fq, '@'); os_puts(&fq, id); os_putc(&fq, '\n');
    os_putn(&fq, seq.s ? seq.s : "", seq.n); os_puts(&fq, "\n+\n");
    os_putn(&fq, qual.s ? qual.s : "", qual.n); os_putc(&fq, '\n');
    R->fastq = fq.s ? fq.s : strdup("");
    R->seq = seq.s ? seq.s : strdup("");
    R->qual = qual.s ? qual.s : strdup("");
    R->trace = trace.s ? trace.s : strdup("");
    R->cigar = cig.s ? cig.s : strdup("");

    /* chimera (Seq.pm:774-889) + detect_chimera (bam2cns:461-491) */
    ostr chim = {0};
    if (P->detect_chimera) {
        omat S2;
        mat_init(&S2, len);
        smap st3;
        smap_copy(&st3, &s.states);
        rc = state_matrix(&s, &S2, &st3, ids, nk, 0, NULL, 0, 0);
        smap_free(&s.states);
        s.states = st3;
        if (rc) { mat_free(&S2); free(ids); goto done; }
        long nb = s.nbins;
        if (nb > 20) {
            double thr = s.bin_max_bases / 5.0 + 1.0;
            long cnt = 0;
            long cap = 8, nwin = 0;
            long *win = (long *)malloc((size_t)cap * 2 * sizeof(long));
            for (long i = 5; i < nb - 5; i++) {
                if ((double)s.bin_bases[i] <= thr) cnt++;
                else if (cnt) {
                    if (cnt >= 1 && cnt < 5) {
                        if (nwin == cap) { cap *= 2; win = (long *)realloc(win, (size_t)cap * 2 * sizeof(long)); }
                        win[2 * nwin] = i - cnt; win[2 * nwin + 1] = i - 1; nwin++;
                    }
                    cnt = 0;
                }
            }
            /* the consensus cigar walk state lives across coordinates */
            long cM = 0, cI = 0, cD = 0;
            size_t rpos_re = 0;
            const char *cs = R->cigar;
            size_t csl = strlen(cs);
            for (long w = 0; w < nwin; w++) {
                long b0 = win[2 * w], b1 = win[2 * w + 1];
                long mf = (b0 - 1) * (long)s.bin_size, mt = (b1 + 2) * (long)s.bin_size - 1;
                int empty = 0;
                for (long c = mf; c <= mt; c++) if (c >= S2.n || S2.c[c].n == 0) { empty = 1; break; }
                if (empty) continue;
                long fl = b0 - 4, tr = b1 + 5;
                long delta = (tr - fl - 1) / 2;
                long tl = fl + delta, fr = tr - delta;
                /* alns_by_bins(fl..tl), (fr..tr) */
                long *il = (long *)malloc((size_t)(nk + 1) * sizeof(long)), nl = 0;
                long *ir = (long *)malloc((size_t)(nk + 1) * sizeof(long)), nr = 0;
                for (long b = fl; b <= tl; b++) for (int k = 0; k < s.bn[b]; k++) il[nl++] = s.bid[b][k];
                for (long b = fr; b <= tr; b++) for (int k = 0; k < s.bn[b]; k++) ir[nr++] = s.bid[b][k];
                omat ML, MR;
                mat_init(&ML, len); mat_init(&MR, len);
                smap sl, sr;
                smap_copy(&sl, &s.states); smap_copy(&sr, &s.states);
                rc = state_matrix(&s, &ML, &sl, il, nl, 0, NULL, 0, 0);
                if (!rc) rc = state_matrix(&s, &MR, &sr, ir, nr, 0, NULL, 0, 0);
                smap_free(&sl); smap_free(&sr);
                free(il); free(ir);
                if (rc) { mat_free(&ML); mat_free(&MR); break; }
                long npos = 0, ntot = 0;
                for (long c = mf; c <= mt; c++) {
                    ocol *cl_ = c < ML.n ? &ML.c[c] : NULL, *cr = c < MR.n ? &MR.c[c] : NULL;
                    if (!cl_ || !cr || cl_->n == 0 || cr->n == 0) continue;
                    double hr = Hx(cr->v, cr->def, cr->n), hl = Hx(cl_->v, cl_->def, cl_->n);
                    double hgt = hr > hl ? hr : hl;
                    int m = cl_->n > cr->n ? cl_->n : cr->n;
                    double *cv = (double *)calloc((size_t)m, sizeof(double));
                    unsigned char *cd = (unsigned char *)calloc((size_t)m, 1);
                    for (int j = 0; j < m; j++) {
                        int dl = j < cl_->n && cl_->def[j] && cl_->v[j] != 0.0;
                        int dr = j < cr->n && cr->def[j] && cr->v[j] != 0.0;
                        if (dl && dr) { cv[j] = cl_->v[j] + cr->v[j]; cd[j] = 1; }
                        else if (dl) { cv[j] = cl_->v[j]; cd[j] = 1; }
                        else if (j < cr->n && cr->def[j]) { cv[j] = cr->v[j]; cd[j] = 1; }
                    }
                    double d = Hx(cv, cd, m) - hgt;
                    free(cv); free(cd);
                    ntot++;
                    if (d > 0.7) npos++;
                }
                mat_free(&ML); mat_free(&MR);
                if (!ntot) continue;
                double score = (double)npos / (double)ntot;
                long from = mf + (long)s.bin_size, to = mt - (long)s.bin_size;
                /* bam2cns:479-481 */
                for (;;) {
                    /* m/(\d+)(\w)/g from rpos_re */
                    size_t p = rpos_re;
                    int found = 0;
                    long num = 0;
                    char op = 0;
                    while (p < csl) {
                        if (isdigit((unsigned char)cs[p])) {
                            size_t q = p;
                            while (q < csl && isdigit((unsigned char)cs[q])) q++;
                            /* greedy digits then \w; backtrack one digit if needed */
                            if (q < csl && (isalnum((unsigned char)cs[q]) || cs[q] == '_')) {
                                num = strtol(cs + p, NULL, 10);   /* digits p..q */
                                {
                                    char tmp[32];
                                    size_t k = q - p < 31 ? q - p : 31;
                                    memcpy(tmp, cs + p, k); tmp[k] = 0;
                                    num = strtol(tmp, NULL, 10);
                                }
                                op = cs[q];
                                rpos_re = q + 1;
                                found = 1;
                                break;
                            } else if (q - p >= 2) {
                                char tmp[32];
                                size_t k = q - p - 1 < 31 ? q - p - 1 : 31;
                                memcpy(tmp, cs + p, k); tmp[k] = 0;
                                num = strtol(tmp, NULL, 10);
                                op = cs[q - 1];
                                rpos_re = q;
                                found = 1;
                                break;
                            }
                            p = q;
                        } else p++;
                    }
                    if (!found) { rpos_re = 0; break; }
                    if (!(cM + cI < from)) break;
                    if (op == 'M') cM += num;
                    else if (op == 'I') cI += num;
                    else if (op == 'D') cD += num;
                }
                long pc = cD - cI;
                char line[512];
                char scs[64];
                snprintf(scs, sizeof scs, "%.15g", score);
                snprintf(line, sizeof line, "%s\t%ld\t%ld\t%s\n", id, from + pc, to + pc, scs);
                os_puts(&chim, line);
            }
            free(win);
        }
        mat_free(&S2);
    }
    R->chim = chim.s ? chim.s : strdup("");
    free(ids);
done:
    if (rc && !R->chim) {
        free(R->fastq); free(R->seq); free(R->qual); free(R->trace); free(R->cigar);
        R->fastq = R->seq = R->qual = R->trace = R->cigar = NULL;
    }
    free(arrival_to_iid);
    for (long b = 0; b < s.nbins; b++) { free(s.bscore[b]); free(s.bid[b]); free(s.blen[b]); }
    free(s.bscore); free(s.bid); free(s.blen); free(s.bn); free(s.bcap); free(s.bin_bases);
    for (long i = 0; i < s.nalns; i++) { free(s.alns[i].cigar); free(s.alns[i].seq); free(s.alns[i].qual); }
    free(s.alns);
    smap_free(&s.states);
    if (s.S.c) mat_free(&s.S);
    return rc;
}

void ocns_free(ocns_result *R) {
    free(R->fastq); free(R->seq); free(R->qual); free(R->trace); free(R->cigar); free(R->chim);
    free(R->kept); free(R->bin_bases);
    memset(R, 0, sizeof(*R));
}
