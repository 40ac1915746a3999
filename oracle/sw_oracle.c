/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called from the
 * product path (proovread_amd/libprgpu.so).
 *
 * Plain-C restatement of the seed-extension stage of `bwa-proovread mem`
 * (bin/proovread:1313, options proovread.cfg:320-333 / 343-365).
 *
 * bwa-proovread is an EMPTY submodule in the reference (.gitmodules:4-6,
 * url https://github.com/BioInf-Wuerzburg/bwa.git, pinned commit unknown; a
 * fork of upstream bwa >= 0.7.11 since it accepts -y).  No bwa source or
 * binary exists in this container, so this file restates the PUBLISHED
 * upstream bwa algorithms:
 *   - ksw.c  ksw_extend2  : banded local extension from a seed (h0), band
 *                           pruning of zero cells, z-drop, to-end gscore
 *   - ksw.c  ksw_global2  : banded global alignment with a direction matrix,
 *                           backtrack M/D/I, CIGAR
 *   - bwamem.c mem_chain2aln (single seed): rmax window via cal_max_gap,
 *                           left/right extension with MAX_BAND_TRY=2 band
 *                           doubling, local vs to-end decision with -L
 *   - bwamem.c mem_reg2aln / bwa.c bwa_gen_cigar2: infer_bw, up to 3 global
 *                           passes doubling w2, leading/trailing-D squeeze,
 *                           soft clips; AS:i = the extension (local) score
 *   - bwa.c bwa_fill_scmat: match a, mismatch -b, any N -1
 * proovread's own -T is a per-base minimum score (cfg:324 "per-base-score !!");
 * its exact bwa-proovread semantics are unpinned: here score >= T*(qe-qb).
 *
 * PARITY UNPINNED against the reference (no reference binary, no golden
 * vectors in the reference tree): tests pin this file with hand-derived
 * known-answer cases and self-consistency properties, and the GPU kernel is
 * held bit-exact to it.
 */
#include "sw_oracle.h"

#include <stdlib.h>
#include <string.h>

#define MINUS_INF (-0x40000000)

typedef struct { int32_t h, e; } eh_t;

void osw_fill_scmat(int a, int b, int8_t mat[25]) {
    int i, j, k;
    for (i = k = 0; i < 4; ++i) {
        for (j = 0; j < 4; ++j) mat[k++] = (int8_t)(i == j ? a : -b);
        mat[k++] = -1;
    }
    for (j = 0; j < 5; ++j) mat[k++] = -1;
}

int osw_extend(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
               const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
               int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle, int *_gscore,
               int *_max_off) {
    eh_t *eh;
    int8_t *qp;
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, beg, end, max, max_i, max_j,
                 max_ins, max_del, max_ie, gscore, max_off;
    qp = (int8_t *)malloc((size_t)(qlen * m) + 1);
    eh = (eh_t *)calloc((size_t)qlen + 1, sizeof(eh_t));
    /* query profile: qp[t*qlen + j] = mat[t][query[j]] */
    for (k = i = 0; k < m; ++k) {
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    /* first row */
    eh[0].h = h0;
    eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;   /* callers guarantee qlen >= 1 */
    for (j = 2; j <= qlen && eh[j - 1].h > e_ins; ++j) eh[j].h = eh[j - 1].h - e_ins;
    /* cap the band by the longest possible gap */
    k = m * m;
    for (i = 0, max = 0; i < k; ++i) max = max > mat[i] ? max : mat[i];
    max_ins = (int)((double)(qlen * max + end_bonus - o_ins) / e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    max_del = (int)((double)(qlen * max + end_bonus - o_del) / e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    /* DP */
    max = h0, max_i = max_j = -1;
    max_ie = -1, gscore = -1;
    max_off = 0;
    beg = 0, end = qlen;
    for (i = 0; i < tlen; ++i) {
        int t, f = 0, h1, mm = 0, mj = -1;
        const int8_t *q = &qp[target[i] * qlen];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else
            h1 = 0;
        for (j = beg; j < end; ++j) {
            /* eh[j] = {H(i-1,j-1), E(i,j)}, f = F(i,j), h1 = H(i,j-1) */
            eh_t *p = &eh[j];
            int h, M = p->h, e = p->e;
            p->h = h1;
            M = M ? M + q[j] : 0;
            h = M > e ? M : e;
            h = h > f ? h : f;
            h1 = h;
            mj = mm > h ? mj : j;
            mm = mm > h ? mm : h;
            t = M - oe_del;
            t = t > 0 ? t : 0;
            e -= e_del;
            e = e > t ? e : t;
            p->e = e;
            t = M - oe_ins;
            t = t > 0 ? t : 0;
            f -= e_ins;
            f = f > t ? f : t;
        }
        eh[end].h = h1;
        eh[end].e = 0;
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (mm == 0) break;
        if (mm > max) {
            max = mm, max_i = i, max_j = mj;
            max_off = max_off > abs(mj - i) ? max_off : abs(mj - i);
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - mm - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
            } else {
                if (max - mm - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
            }
        }
        for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j);
        beg = j;
        for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j);
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    free(eh);
    free(qp);
    if (_qle) *_qle = max_j + 1;
    if (_tle) *_tle = max_i + 1;
    if (_gtle) *_gtle = max_ie + 1;
    if (_gscore) *_gscore = gscore;
    if (_max_off) *_max_off = max_off;
    return max;
}

static int push_cigar(uint32_t *cig, int n, int max, int op, int len) {
    if (n && (int)(cig[n - 1] & 0xf) == op) {
        cig[n - 1] += (uint32_t)len << 4;
        return n;
    }
    if (n >= max) return -1;
    cig[n] = (uint32_t)len << 4 | (uint32_t)op;
    return n + 1;
}

/* ksw_global2: ops in bwa's encoding 0=M 1=I 2=D */
int osw_global(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
               const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
               int *n_cigar_, uint32_t *cigar, int max_cigar) {
    eh_t *eh;
    int8_t *qp;
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, score, n_col;
    uint8_t *z;
    *n_cigar_ = 0;
    n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    z = (uint8_t *)malloc((size_t)n_col * (size_t)tlen + 1);
    qp = (int8_t *)malloc((size_t)(qlen * m) + 1);
    eh = (eh_t *)calloc((size_t)qlen + 1, sizeof(eh_t));
    for (k = i = 0; k < m; ++k) {
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    eh[0].h = 0;
    eh[0].e = MINUS_INF;
    for (j = 1; j <= qlen && j <= w; ++j) eh[j].h = -(o_ins + e_ins * j), eh[j].e = MINUS_INF;
    for (; j <= qlen; ++j) eh[j].h = eh[j].e = MINUS_INF;
    for (i = 0; i < tlen; ++i) {
        int32_t f = MINUS_INF, h1, beg, end, t;
        const int8_t *q = &qp[target[i] * qlen];
        uint8_t *zi = &z[(long)i * n_col];
        beg = i > w ? i - w : 0;
        end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : MINUS_INF;
        for (j = beg; j < end; ++j) {
            eh_t *p = &eh[j];
            int32_t h, mm = p->h, e = p->e;
            uint8_t d;
            p->h = h1;
            mm += q[j];
            d = mm >= e ? 0 : 1;
            h = mm >= e ? mm : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            h1 = h;
            t = mm - oe_del;
            e -= e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            p->e = e;
            t = mm - oe_ins;
            f -= e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            zi[j - beg] = d;
        }
        eh[end].h = h1;
        eh[end].e = MINUS_INF;
    }
    score = eh[qlen].h;
    {
        int n = 0, which = 0;
        i = tlen - 1;
        k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        while (i >= 0 && k >= 0 && n >= 0) {
            which = z[(long)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0) n = push_cigar(cigar, n, max_cigar, 0, 1), --i, --k;
            else if (which == 1) n = push_cigar(cigar, n, max_cigar, 2, 1), --i;
            else n = push_cigar(cigar, n, max_cigar, 1, 1), --k;
        }
        if (n >= 0 && i >= 0) n = push_cigar(cigar, n, max_cigar, 2, i + 1);
        if (n >= 0 && k >= 0) n = push_cigar(cigar, n, max_cigar, 1, k + 1);
        if (n < 0) {
            free(eh); free(qp); free(z);
            return MINUS_INF;
        }
        for (i = 0; i < n >> 1; ++i) {
            uint32_t tmp = cigar[i];
            cigar[i] = cigar[n - 1 - i];
            cigar[n - 1 - i] = tmp;
        }
        *n_cigar_ = n;
    }
    free(eh);
    free(qp);
    free(z);
    return score;
}

static int cal_max_gap(const osw_opts *o, int qlen) {
    int l_del = (int)((double)(qlen * o->a - o->o_del) / o->e_del + 1.);
    int l_ins = (int)((double)(qlen * o->a - o->o_ins) / o->e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < o->w << 1 ? l : o->w << 1;
}

static int infer_bw(int l1, int l2, int score, int a, int q, int r) {
    int w;
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    if (w < abs(l1 - l2)) w = abs(l1 - l2);
    return w;
}

static inline uint8_t strand_base(const uint8_t *ref, int L, int strand, int x) {
    if (!strand) return ref[x];
    uint8_t c = ref[L - 1 - x];
    return c < 4 ? (uint8_t)(3 - c) : c;
}

/* one strand-coordinate base of long read `ref` (forward, length L) */
static void fetch_strand(const uint8_t *ref, int L, int strand, long b, long e, uint8_t *out) {
    for (long x = b; x < e; ++x) out[x - b] = strand_base(ref, L, strand, (int)x);
}

/* bwamem.c mem_chain2aln, the extension of one seed (the window of a single seed: a chain's
 * wider window adds only rows the band cannot reach with a gain, cal_max_gap's bound) */
int osw_extend_seed(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
                    int qbeg, int rbeg, int slen, osw_region *g) {
    int8_t mat[25];
    osw_fill_scmat(o->a, o->b, mat);
    memset(g, 0, sizeof(*g));
    if (lq <= 0 || slen <= 0 || qbeg < 0 || qbeg + slen > lq || rbeg < 0 || rbeg + slen > L) return -1;
    /* mem_chain2aln: max possible span */
    long rmax0 = (long)rbeg - (qbeg + cal_max_gap(o, qbeg));
    long rmax1 = (long)rbeg + slen + ((lq - qbeg - slen) + cal_max_gap(o, lq - qbeg - slen));
    if (rmax0 < 0) rmax0 = 0;
    if (rmax1 > L) rmax1 = L;
    const int rl = (int)(rmax1 - rmax0);
    uint8_t *rseq = (uint8_t *)malloc((size_t)rl + 1);
    fetch_strand(ref, L, strand, rmax0, rmax1, rseq);
    int aw0 = o->w, aw1 = o->w;
    int score = -1, truesc = -1, qb, qe, rb, re;
    if (qbeg) {
        int qle, tle, gtle, gscore, max_off;
        uint8_t *qs = (uint8_t *)malloc((size_t)qbeg);
        for (int i = 0; i < qbeg; ++i) qs[i] = q[qbeg - 1 - i];
        int tmp = (int)(rbeg - rmax0);
        uint8_t *rs = (uint8_t *)malloc((size_t)tmp + 1);
        for (int i = 0; i < tmp; ++i) rs[i] = rseq[tmp - 1 - i];
        for (int i = 0; i < 2; ++i) {
            int prev = score;
            aw0 = o->w << i;
            score = osw_extend(qbeg, qs, tmp, rs, 5, mat, o->o_del, o->e_del, o->o_ins, o->e_ins, aw0,
                               o->pen_clip5, o->zdrop, slen * o->a, &qle, &tle, &gtle, &gscore, &max_off);
            if (score == prev || max_off < (aw0 >> 1) + (aw0 >> 2)) break;
        }
        if (gscore <= 0 || gscore <= score - o->pen_clip5) {
            qb = qbeg - qle, rb = rbeg - tle;
            truesc = score;
        } else {
            qb = 0, rb = rbeg - gtle;
            truesc = gscore;
        }
        free(qs);
        free(rs);
    } else {
        score = truesc = slen * o->a, qb = 0, rb = rbeg;
    }
    if (qbeg + slen != lq) {
        int qle, tle, gtle, gscore, max_off, sc0 = score;
        int qe0 = qbeg + slen;
        int re0 = (int)(rbeg + slen - rmax0);
        for (int i = 0; i < 2; ++i) {
            int prev = score;
            aw1 = o->w << i;
            score = osw_extend(lq - qe0, q + qe0, rl - re0, rseq + re0, 5, mat, o->o_del, o->e_del,
                               o->o_ins, o->e_ins, aw1, o->pen_clip3, o->zdrop, sc0, &qle, &tle, &gtle,
                               &gscore, &max_off);
            if (score == prev || max_off < (aw1 >> 1) + (aw1 >> 2)) break;
        }
        if (gscore <= 0 || gscore <= score - o->pen_clip3) {
            qe = qe0 + qle, re = (int)(rmax0 + re0 + tle);
            truesc += score - sc0;
        } else {
            qe = lq, re = (int)(rmax0 + re0 + gtle);
            truesc += gscore - sc0;
        }
    } else {
        qe = lq, re = rbeg + slen;
    }
    free(rseq);
    g->qb = qb; g->qe = qe; g->rb = rb; g->re = re;
    g->score = score; g->truesc = truesc;
    g->w = aw0 > aw1 ? aw0 : aw1;
    g->seedlen0 = slen;
    return 0;
}

/* bwa.c bwa_gen_cigar2 over query q[0,lqq) and strand reference [rb, re): the global score,
 * and the CIGAR (bwa op codes, reversed-both placement on the reverse strand) when cig != 0 */
static int gen_cigar2(const osw_opts *o, const int8_t *mat, int w_, const uint8_t *qseg, int lqq, const uint8_t *ref,
                      int L, int strand, int rb, int re, uint32_t *cig, int *ncig, int *w_used) {
    const int rlen = re - rb;
    int gsc = 0;
    *ncig = 0;
    *w_used = 0;
    if (lqq <= 0 || rlen <= 0) return 0;
    uint8_t *qq = (uint8_t *)malloc((size_t)lqq + 1);
    uint8_t *rr = (uint8_t *)malloc((size_t)rlen + 1);
    memcpy(qq, qseg, (size_t)lqq);
    fetch_strand(ref, L, strand, rb, re, rr);
    if (strand) { /* reverse both so indels are placed leftmost on the forward strand */
        for (int i = 0; i < lqq >> 1; ++i) { uint8_t t = qq[i]; qq[i] = qq[lqq - 1 - i]; qq[lqq - 1 - i] = t; }
        for (int i = 0; i < rlen >> 1; ++i) { uint8_t t = rr[i]; rr[i] = rr[rlen - 1 - i]; rr[rlen - 1 - i] = t; }
    }
    if (lqq == rlen && w_ == 0) {
        if (cig) { cig[0] = (uint32_t)lqq << 4; *ncig = 1; }
        for (int i = 0; i < lqq; ++i) gsc += mat[rr[i] * 5 + qq[i]];
    } else {
        int mn = lqq < rlen ? lqq : rlen;
        int max_ins = (int)((double)(mn * mat[0] - o->o_ins) / o->e_ins + 1.);
        int max_del = (int)((double)(mn * mat[0] - o->o_del) / o->e_del + 1.);
        int max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        int ww = (max_gap + abs(rlen - lqq) + 1) >> 1;
        ww = ww < w_ ? ww : w_;
        int min_w = abs(rlen - lqq) + 3;
        ww = ww > min_w ? ww : min_w;
        int nc = 0;
        uint32_t *tmp = cig ? cig : (uint32_t *)malloc(sizeof(uint32_t) * OSW_MAXCIG);
        gsc = osw_global(lqq, qq, rlen, rr, 5, mat, o->o_del, o->e_del, o->o_ins, o->e_ins, ww, &nc, tmp,
                         OSW_MAXCIG - 4);
        if (cig) *ncig = nc; else free(tmp);
        *w_used = ww;
    }
    free(qq);
    free(rr);
    return gsc;
}

int osw_gen_score(const osw_opts *o, int w_, const uint8_t *qseg, int lqq, const uint8_t *ref, int L, int strand,
                  int rb, int re) {
    int8_t mat[25];
    osw_fill_scmat(o->a, o->b, mat);
    int nc, wu;
    return gen_cigar2(o, mat, w_, qseg, lqq, ref, L, strand, rb, re, 0, &nc, &wu);
}

/* bwamem.c mem_reg2aln: the CIGAR of region g (infer_bw, up to 3 global passes) */
int osw_reg2aln(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
                const osw_region *g, osw_result *r) {
    int8_t mat[25];
    osw_fill_scmat(o->a, o->b, mat);
    memset(r, 0, sizeof(*r));
    const int qb = g->qb, qe = g->qe, rb = g->rb, re = g->re, truesc = g->truesc;
    r->qb = qb; r->qe = qe; r->rb = rb; r->re = re;
    r->score = g->score; r->truesc = truesc; r->w = g->w;
    r->pass = (double)g->score >= o->min_score_per_base * (double)(qe - qb);
    int tmpw = infer_bw(qe - qb, re - rb, truesc, o->a, o->o_del, o->e_del);
    int w2 = infer_bw(qe - qb, re - rb, truesc, o->a, o->o_ins, o->e_ins);
    w2 = w2 > tmpw ? w2 : tmpw;
    if (w2 > o->w) w2 = w2 < g->w ? w2 : g->w;
    int last_sc = -(1 << 30), gsc = 0, ncig = 0, iter = 0;
    uint32_t cig[OSW_MAXCIG];
    int w_used = 0;
    do {
        w2 = w2 < o->w << 2 ? w2 : o->w << 2;
        gsc = gen_cigar2(o, mat, w2, q + qb, qe - qb, ref, L, strand, rb, re, cig, &ncig, &w_used);
        if (qe - qb <= 0 || re - rb <= 0) break;
        if (gsc == last_sc || w2 == o->w << 2) break;
        last_sc = gsc;
        w2 <<= 1;
    } while (++iter < 3 && gsc < truesc - o->a);
    r->global_score = gsc;
    r->w2 = w_used;
    /* forward position; convert bwa op codes (M0 I1 D2) to BAM (M0 I1 D2 S4) */
    int pos = strand ? L - re : rb;
    int n = 0;
    uint32_t out[OSW_MAXCIG];
    for (int i = 0; i < ncig; ++i) out[n++] = cig[i];
    if (n > 0) {
        if ((out[0] & 0xf) == 2) {
            pos += (int)(out[0] >> 4);
            memmove(out, out + 1, (size_t)(n - 1) * 4);
            --n;
        } else if ((out[n - 1] & 0xf) == 2) {
            --n;
        }
    }
    int clip5 = strand ? lq - qe : qb;
    int clip3 = strand ? qb : lq - qe;
    int m = 0;
    if (qb != 0 || qe != lq) {
        if (clip5) r->cigar[m++] = (uint32_t)clip5 << 4 | 4u;
    }
    for (int i = 0; i < n; ++i) r->cigar[m++] = out[i];
    if ((qb != 0 || qe != lq) && clip3) r->cigar[m++] = (uint32_t)clip3 << 4 | 4u;
    r->n_cigar = m;
    r->pos = pos;
    return 0;
}

/* one single-seed task: extension + CIGAR */
int osw_task(const osw_opts *o, const uint8_t *q, int lq, const uint8_t *ref, int L, int strand,
             int qbeg, int rbeg, int slen, osw_result *r) {
    osw_region g;
    memset(r, 0, sizeof(*r));
    if (osw_extend_seed(o, q, lq, ref, L, strand, qbeg, rbeg, slen, &g)) return -1;
    return osw_reg2aln(o, q, lq, ref, L, strand, &g, r);
}
