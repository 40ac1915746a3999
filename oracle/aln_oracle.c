/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called from the product path.
 *
 * Plain-C restatement of what `bwa-proovread mem` (bin/proovread:1313; an EMPTY submodule,
 * .gitmodules:4-6, pinned commit unknown — PARITY UNPINNED) does with one short read after
 * seeding, following the published upstream bwa (>= 0.7.13) bwamem.c:
 *   mem_chain2aln       every seed of every kept chain in srt order (seed score = length,
 *                       larger index first on ties); a seed contained in an earlier region
 *                       ("around" it within min(cal_max_gap, band)) is skipped unless a longer
 *                       (>= 95 %) already-extended seed of the chain overlaps it by >= 1/4 on
 *                       another diagonal; otherwise ksw_extend2 both sides (sw_oracle.c)
 *   mem_sort_dedup_patch sort by end (ks_introsort), redundant hits (overlap > 95 % on both
 *                       sequences: the lower score goes), colinear neighbours merged by
 *                       mem_patch_reg (global score >= 90 % of the predicted one), sort by
 *                       (score desc, rb, qb), identical hits removed
 *   mem_mark_primary_se sort by (score desc, hash_64(read_id + i)), secondaries = regions whose
 *                       query span overlaps an earlier primary's by >= mask_level
 *   mem_reg2sam         -T (proovread: per aligned base, cfg:324, unpinned) and -D: a
 *                       secondary scoring below drop_ratio x its primary is not reported
 * The sorts replay klib's ks_introsort (ksort.h, as vendored by bwa) so ties fall as bwa's do.
 * Coordinates: bwa's forward-reverse space (forward long reads, then the reverse complement
 * of their concatenation); regions keep strand coordinates and compare in that space.
 */
#include "aln_oracle.h"

#include <stdlib.h>
#include <string.h>

static int cal_max_gap(const osw_opts *o, int qlen) {
    int l_del = (int)((double)(qlen * o->a - o->o_del) / o->e_del + 1.);
    int l_ins = (int)((double)(qlen * o->a - o->o_ins) / o->e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < o->w << 1 ? l : o->w << 1;
}

static uint64_t hash_64(uint64_t key) {
    key += ~(key << 32);
    key ^= (key >> 22);
    key += ~(key << 13);
    key ^= (key >> 8);
    key += (key << 3);
    key ^= (key >> 15);
    key += ~(key << 27);
    key ^= (key >> 31);
    return key;
}

/* a region in bwa's terms */
typedef struct {
    int64_t rb, re;   /* forward-reverse coordinates */
    int qb, qe, rid, score, truesc, w, seedlen0, strand, seed, patched;
    int secondary;
    uint64_t hash;
} reg_t;

/* ---------------------------------------------------------------- klib ks_introsort */
typedef int (*lt_fn)(const reg_t *, const reg_t *);
static void swap_r(reg_t *a, reg_t *b) {
    reg_t t = *a;
    *a = *b;
    *b = t;
}
static void insertsort(reg_t *s, reg_t *t, lt_fn lt) {
    for (reg_t *i = s + 1; i < t; ++i)
        for (reg_t *j = i; j > s && lt(j, j - 1); --j) swap_r(j, j - 1);
}
static void combsort(size_t n, reg_t *a, lt_fn lt) {
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    size_t gap = n;
    do {
        if (gap > 2) {
            gap = (size_t)(gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (reg_t *i = a; i < a + n - gap; ++i) {
            reg_t *j = i + gap;
            if (lt(j, i)) {
                swap_r(i, j);
                do_swap = 1;
            }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) insertsort(a, a + n, lt);
}
typedef struct {
    reg_t *left, *right;
    int depth;
} isort_stack_t;
static void introsort(size_t n, reg_t *a, lt_fn lt) {
    int d;
    reg_t rp;
    reg_t *s, *t, *i, *j, *k;
    if (n < 1) return;
    if (n == 2) {
        if (lt(&a[1], &a[0])) swap_r(&a[0], &a[1]);
        return;
    }
    for (d = 2; 1ul << d < n; ++d) {}
    isort_stack_t *stack = (isort_stack_t *)malloc(sizeof(isort_stack_t) * ((sizeof(size_t) * d) + 2));
    isort_stack_t *top = stack;
    s = a;
    t = a + (n - 1);
    d <<= 1;
    for (;;) {
        if (s < t) {
            if (--d == 0) {
                combsort((size_t)(t - s + 1), s, lt);
                t = s;
                continue;
            }
            i = s;
            j = t;
            k = i + ((j - i) >> 1) + 1;
            if (lt(k, i)) {
                if (lt(k, j)) k = j;
            } else {
                k = lt(j, i) ? i : j;
            }
            rp = *k;
            if (k != t) swap_r(k, t);
            for (;;) {
                do ++i; while (lt(i, &rp));
                do --j; while (i <= j && lt(&rp, j));
                if (j <= i) break;
                swap_r(i, j);
            }
            swap_r(i, t);
            if (i - s > t - i) {
                if (i - s > 16) {
                    top->left = s;
                    top->right = i - 1;
                    top->depth = d;
                    ++top;
                }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) {
                    top->left = i + 1;
                    top->right = t;
                    top->depth = d;
                    ++top;
                }
                t = i - s > 16 ? s : i - 1;
            }
        } else {
            if (top == stack) {
                free(stack);
                insertsort(a, a + n, lt);
                return;
            }
            --top;
            s = top->left;
            t = top->right;
            d = top->depth;
        }
    }
}
/* bwamem.c alnreg_slt2 (mem_ars2), alnreg_slt (mem_ars), alnreg_hlt (mem_ars_hash) */
static int lt_end(const reg_t *a, const reg_t *b) { return a->re < b->re; }
static int lt_score(const reg_t *a, const reg_t *b) {
    return a->score > b->score || (a->score == b->score && (a->rb < b->rb || (a->rb == b->rb && a->qb < b->qb)));
}
static int lt_hash(const reg_t *a, const reg_t *b) {
    return a->score > b->score || (a->score == b->score && a->hash < b->hash);
}

/* ---------------------------------------------------------------- mem_patch_reg */
static int64_t fr_of(const int64_t *lr_off, int n_lr, int lr, int strand, int64_t x) {
    const int64_t l_pac = lr_off[n_lr];
    return strand ? l_pac + (l_pac - lr_off[lr + 1]) + x : lr_off[lr] + x;
}

static int patch_reg(const osw_opts *o, const uint8_t *q, const uint8_t *lr_seq, const int64_t *lr_off, int n_lr,
                     const reg_t *a, const reg_t *b, int *_w) {
    const int64_t l_pac = lr_off[n_lr];
    if (a->rb < l_pac && b->rb >= l_pac) return 0;   /* on different strands */
    if (a->qb >= b->qb || a->qe >= b->qe || a->re >= b->re) return 0;   /* not colinear */
    int w = (int)((a->re - b->rb) - (a->qe - b->qb));   /* required bandwidth */
    w = w > 0 ? w : -w;
    double r = (double)(a->re - b->rb) / (double)(b->re - a->rb) - (double)(a->qe - b->qb) / (double)(b->qe - a->qb);
    r = r > 0. ? r : -r;
    if (a->re < b->rb || a->qe < b->qb) {   /* no overlap on query or on ref */
        if (w > o->w << 1 || r >= 0.05) return 0;
    } else if (w > o->w << 2 || r >= 0.05 * 2) {
        return 0;
    }
    w += a->w + b->w;
    w = w < o->w << 2 ? w : o->w << 2;
    /* global alignment of query [a.qb, b.qe) against [a.rb, b.re) (strand coordinates) */
    const int lr = a->rid, strand = a->strand;
    const int64_t base = fr_of(lr_off, n_lr, lr, strand, 0);
    const int L = (int)(lr_off[lr + 1] - lr_off[lr]);
    const int score = osw_gen_score(o, w, q + a->qb, b->qe - a->qb, lr_seq + lr_off[lr], L, strand,
                                    (int)(a->rb - base), (int)(b->re - base));
    const int q_s = (int)((double)(b->qe - a->qb) / ((b->qe - b->qb) + (a->qe - a->qb)) * (b->score + a->score) + .5);
    const int r_s = (int)((double)(b->re - a->rb) / (double)((b->re - b->rb) + (a->re - a->rb)) * (b->score + a->score) + .5);
    if ((double)score / (q_s > r_s ? q_s : r_s) < 0.90) return 0;
    *_w = w;
    return score;
}

/* ---------------------------------------------------------------- one read */
int oaln_read(const osw_opts *o, const oaln_opts *ao, const uint8_t *q, int lq, const uint8_t *lr_seq,
              const int64_t *lr_off, int n_lr, const oaln_seed *s, int ns, int64_t read_id, oaln_reg *out,
              int *n_out, int *n_ext) {
    *n_out = 0;
    *n_ext = 0;
    if (ns <= 0) return 0;
    reg_t *av = (reg_t *)calloc((size_t)ns, sizeof(reg_t));
    char *done = (char *)calloc((size_t)ns, 1);   /* 1: extended (srt != 0), 2: skipped */
    int nav = 0;
    /* mem_chain2aln per chain; seeds of a chain are consecutive, in rank order */
    for (int c0 = 0; c0 < ns;) {
        int c1 = c0 + 1;
        while (c1 < ns && s[c1].chain == s[c0].chain) ++c1;
        for (int k = c0; k < c1; ++k) {
            const oaln_seed *sd = &s[k];
            const int64_t srb = fr_of(lr_off, n_lr, sd->lr, sd->strand, sd->rbeg);
            int i;
            for (i = 0; i < nav; ++i) {   /* test whether extension has been made before */
                const reg_t *p = &av[i];
                if (srb < p->rb || srb + sd->slen > p->re || sd->qbeg < p->qb || sd->qbeg + sd->slen > p->qe)
                    continue;   /* not fully contained */
                if (sd->slen - p->seedlen0 > .1 * lq) continue;   /* this seed may give a better alignment */
                int64_t qd = sd->qbeg - p->qb, rd = srb - p->rb;
                int max_gap = cal_max_gap(o, (int)(qd < rd ? qd : rd));
                int w = max_gap < p->w ? max_gap : p->w;
                if (qd - rd < w && rd - qd < w) break;   /* "around" a previous hit */
                qd = p->qe - (sd->qbeg + sd->slen);
                rd = p->re - (srb + sd->slen);
                max_gap = cal_max_gap(o, (int)(qd < rd ? qd : rd));
                w = max_gap < p->w ? max_gap : p->w;
                if (qd - rd < w && rd - qd < w) break;
            }
            if (i < nav) {   /* almost contained: extend only if a longer extended seed overlaps elsewhere */
                int j;
                for (j = k - 1; j >= c0; --j) {   /* the chain's seeds tried before this one */
                    if (done[j] != 1) continue;
                    const oaln_seed *t = &s[j];
                    if (t->slen < sd->slen * .95) continue;
                    const int64_t trb = fr_of(lr_off, n_lr, t->lr, t->strand, t->rbeg);
                    if (sd->qbeg <= t->qbeg && sd->qbeg + sd->slen - t->qbeg >= sd->slen >> 2 &&
                        t->qbeg - sd->qbeg != trb - srb)
                        break;
                    if (t->qbeg <= sd->qbeg && t->qbeg + t->slen - sd->qbeg >= sd->slen >> 2 &&
                        sd->qbeg - t->qbeg != srb - trb)
                        break;
                }
                if (j < c0) {
                    done[k] = 2;
                    continue;
                }
            }
            const int L = (int)(lr_off[sd->lr + 1] - lr_off[sd->lr]);
            osw_region g;
            if (osw_extend_seed(o, q, lq, lr_seq + lr_off[sd->lr], L, sd->strand, sd->qbeg, sd->rbeg, sd->slen, &g)) {
                free(av);
                free(done);
                return -1;
            }
            ++*n_ext;
            done[k] = 1;
            reg_t *a = &av[nav++];
            memset(a, 0, sizeof(*a));
            const int64_t base = fr_of(lr_off, n_lr, sd->lr, sd->strand, 0);
            a->rb = base + g.rb;
            a->re = base + g.re;
            a->qb = g.qb;
            a->qe = g.qe;
            a->rid = sd->lr;
            a->strand = sd->strand;
            a->score = g.score;
            a->truesc = g.truesc;
            a->w = g.w;
            a->seedlen0 = g.seedlen0;
            a->seed = k;
        }
        c0 = c1;
    }
    free(done);
    /* mem_sort_dedup_patch */
    int n = nav;
    if (n > 1) {
        introsort((size_t)n, av, lt_end);
        for (int i = 1; i < n; ++i) {
            reg_t *p = &av[i];
            if (p->rid != av[i - 1].rid || p->rb >= av[i - 1].re + ao->max_chain_gap) continue;
            for (int j = i - 1; j >= 0 && p->rid == av[j].rid && p->rb < av[j].re + ao->max_chain_gap; --j) {
                reg_t *qq = &av[j];
                int score, w;
                if (qq->qe == qq->qb) continue;   /* excluded */
                const int64_t orr = qq->re - p->rb;
                const int64_t oq = qq->qb < p->qb ? qq->qe - p->qb : p->qe - qq->qb;
                const int64_t mr = qq->re - qq->rb < p->re - p->rb ? qq->re - qq->rb : p->re - p->rb;
                const int64_t mq = qq->qe - qq->qb < p->qe - p->qb ? qq->qe - qq->qb : p->qe - p->qb;
                if (orr > ao->mask_level_redun * mr && oq > ao->mask_level_redun * mq) {   /* redundant */
                    if (p->score < qq->score) {
                        p->qe = p->qb;
                        break;
                    } else {
                        qq->qe = qq->qb;
                    }
                } else if (qq->rb < p->rb && (score = patch_reg(o, q, lr_seq, lr_off, n_lr, qq, p, &w)) > 0) {
                    p->qb = qq->qb, p->rb = qq->rb;
                    p->truesc = p->score = score;
                    p->w = w;
                    p->patched = 1;
                    qq->qb = qq->qe;
                }
            }
        }
        int m = 0;
        for (int i = 0; i < n; ++i)
            if (av[i].qe > av[i].qb) av[m++] = av[i];
        n = m;
        introsort((size_t)n, av, lt_score);
        for (int i = 1; i < n; ++i)
            if (av[i].score == av[i - 1].score && av[i].rb == av[i - 1].rb && av[i].qb == av[i - 1].qb)
                av[i].qe = av[i].qb;
        m = n > 0 ? 1 : 0;
        for (int i = 1; i < n; ++i)
            if (av[i].qe > av[i].qb) av[m++] = av[i];
        n = m;
    }
    /* mem_mark_primary_se */
    for (int i = 0; i < n; ++i) {
        av[i].secondary = -1;
        av[i].hash = hash_64((uint64_t)(read_id + i));
    }
    introsort((size_t)n, av, lt_hash);
    if (n > 0) {
        int *z = (int *)malloc(sizeof(int) * (size_t)n);
        int nz = 0;
        z[nz++] = 0;
        for (int i = 1; i < n; ++i) {
            int k;
            for (k = 0; k < nz; ++k) {
                const int j = z[k];
                const int b_max = av[j].qb > av[i].qb ? av[j].qb : av[i].qb;
                const int e_min = av[j].qe < av[i].qe ? av[j].qe : av[i].qe;
                if (e_min > b_max) {
                    const int min_l = av[i].qe - av[i].qb < av[j].qe - av[j].qb ? av[i].qe - av[i].qb : av[j].qe - av[j].qb;
                    if (e_min - b_max >= min_l * ao->mask_level) break;
                }
            }
            if (k == nz) z[nz++] = i;
            else av[i].secondary = z[k];
        }
        free(z);
    }
    /* mem_reg2sam: -T (per aligned base) and -D for secondaries */
    int no = 0;
    int *omap = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int k = 0; k < n; ++k) {
        const reg_t *p = &av[k];
        omap[k] = -1;
        if (!((double)p->score >= o->min_score_per_base * (double)(p->qe - p->qb))) continue;
        if (p->secondary >= 0 && p->score < av[p->secondary].score * ao->drop_ratio) continue;
        oaln_reg *r = &out[no];
        const int64_t base = fr_of(lr_off, n_lr, p->rid, p->strand, 0);
        r->lr = p->rid;
        r->strand = p->strand;
        r->g.qb = p->qb;
        r->g.qe = p->qe;
        r->g.rb = (int)(p->rb - base);
        r->g.re = (int)(p->re - base);
        r->g.score = p->score;
        r->g.truesc = p->truesc;
        r->g.w = p->w;
        r->g.seedlen0 = p->seedlen0;
        r->secondary = p->secondary;   /* remapped below */
        r->seed = p->seed;
        r->patched = p->patched;
        /* mem_reg2aln / mem_reg2sam flags: 0x100 secondary, 0x800 a later primary (supplementary) */
        r->flag = (p->strand ? 0x10 : 0) | (p->secondary >= 0 ? 0x100 : (no > 0 ? 0x800 : 0));
        omap[k] = no++;
    }
    for (int k = 0; k < no; ++k)
        if (out[k].secondary >= 0) out[k].secondary = omap[out[k].secondary];
    free(omap);
    free(av);
    *n_out = no;
    return 0;
}
