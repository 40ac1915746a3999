/* libprsynth.so: the synthetic workloads of SURVEY.md §8d at configs[2] / configs[3] scale
 * (1 - 2.7 Gb of long reads), generated on host threads.  Benchmark and test input only: not
 * part of the drop-in boundary (include/prgpu.h), never on the product path.
 *
 * The model is proovread_amd/synth.py simulate()'s: an iid ACGT genome; long reads sampled
 * at sorted uniform starts, every genome base deleted with p_del, else substituted with
 * p_sub (a different base), then followed by a geometric number of random inserted bases
 * (continue with p_ins); short reads of sr_len bases at uniform starts in sequencer order
 * (unsorted), one substitution in 0.1 % x sr_len of them, reverse-complemented on strand 1.
 * Every read draws from its own counter-based stream (splitmix64 of the seed and its index),
 * so the output does not depend on the thread count. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* xoshiro256** seeded from splitmix64 */
typedef struct { uint64_t s[4]; } rng_t;
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rnext(rng_t *r) {
    const uint64_t res = rotl(r->s[1] * 5, 7) * 9, t = r->s[1] << 17;
    r->s[2] ^= r->s[0];
    r->s[3] ^= r->s[1];
    r->s[1] ^= r->s[2];
    r->s[0] ^= r->s[3];
    r->s[2] ^= t;
    r->s[3] = rotl(r->s[3], 45);
    return res;
}
static void rseed(rng_t *r, uint64_t seed, uint64_t stream, uint64_t item) {
    uint64_t z = mix64(seed ^ mix64(stream * 0x100000001b3ull + 0x51ed27ull) ^ mix64(item + 0x632be5ab3ull));
    for (int i = 0; i < 4; ++i) r->s[i] = z = mix64(z + (uint64_t)i);
}
/* uniform in [0, 2^32): compared against p * 2^32 */
static inline uint32_t ru32(rng_t *r) { return (uint32_t)(rnext(r) >> 32); }
static inline uint64_t rbelow(rng_t *r, uint64_t n) { return (uint64_t)(((unsigned __int128)rnext(r) * n) >> 64); }

typedef struct {
    const uint8_t *genome;
    const int64_t *starts;
    int64_t n, span;
    uint32_t t_del, t_sub, t_ins;   /* thresholds of p_del, p_del + p_sub, p_ins on a u32 */
    uint64_t seed;
    int64_t *lens;
    const int64_t *off;
    uint8_t *out;
    int64_t i0, i1;
} lr_job;

/* one long read: pass out == NULL counts its bases */
static int64_t lr_one(const lr_job *J, int64_t i, uint8_t *out) {
    rng_t r;
    rseed(&r, J->seed, 1, (uint64_t)i);
    const uint8_t *g = J->genome + J->starts[i];
    int64_t k = 0;
    for (int64_t j = 0; j < J->span; ++j) {
        const uint32_t u = ru32(&r);
        if (u >= J->t_del) {
            uint8_t b = g[j];
            if (u < J->t_sub) b = (uint8_t)((b + 1 + rbelow(&r, 3)) & 3);
            if (out) out[k] = b;
            ++k;
        }
        while (ru32(&r) < J->t_ins) {
            const uint8_t b = (uint8_t)(rnext(&r) >> 62);
            if (out) out[k] = b;
            ++k;
        }
    }
    return k;
}

static void *lr_count(void *p) {
    lr_job *J = (lr_job *)p;
    for (int64_t i = J->i0; i < J->i1; ++i) J->lens[i] = lr_one(J, i, NULL);
    return NULL;
}
static void *lr_write(void *p) {
    lr_job *J = (lr_job *)p;
    for (int64_t i = J->i0; i < J->i1; ++i) lr_one(J, i, J->out + J->off[i]);
    return NULL;
}

static int run_jobs(void *(*fn)(void *), void *jobs, size_t job_size, int threads) {
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!th) return -1;
    int started = 0, rc = 0;
    for (int t = 0; t < threads; ++t) {
        if (pthread_create(&th[t], NULL, fn, (char *)jobs + (size_t)t * job_size)) {
            rc = -1;
            break;
        }
        ++started;
    }
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    free(th);
    return rc;
}

static uint32_t thresh(double p) {
    if (p <= 0) return 0;
    if (p >= 1) return 0xffffffffu;
    return (uint32_t)(p * 4294967296.0);
}

/* genome of n bases (nt4 0..3) */
int prs_genome(uint64_t seed, int64_t n, uint8_t *out) {
    rng_t r;
    rseed(&r, seed, 0, 0);
    int64_t i = 0;
    for (; i + 32 <= n; i += 32) {
        const uint64_t x = rnext(&r);
        for (int k = 0; k < 32; ++k) out[i + k] = (uint8_t)((x >> (2 * k)) & 3);
    }
    if (i < n) {
        const uint64_t x = rnext(&r);
        for (int k = 0; i < n; ++i, ++k) out[i] = (uint8_t)((x >> (2 * k)) & 3);
    }
    return 0;
}

/* long reads at `starts` (span bases of the genome each): out == NULL -> lens[n] only;
 * otherwise the bases at off[i] (off = exclusive prefix of lens) */
int prs_long_reads(const uint8_t *genome, const int64_t *starts, int64_t n, int64_t span, double p_ins, double p_del,
                   double p_sub, uint64_t seed, int threads, int64_t *lens, const int64_t *off, uint8_t *out) {
    if (threads < 1) threads = 1;
    if (n < 0 || span < 0) return -1;
    lr_job *J = (lr_job *)calloc((size_t)threads, sizeof(lr_job));
    if (!J) return -1;
    for (int t = 0; t < threads; ++t) {
        lr_job *j = &J[t];
        j->genome = genome;
        j->starts = starts;
        j->n = n;
        j->span = span;
        j->t_del = thresh(p_del);
        j->t_sub = thresh(p_del + p_sub);
        j->t_ins = thresh(p_ins);
        j->seed = seed;
        j->lens = lens;
        j->off = off;
        j->out = out;
        j->i0 = n * t / threads;
        j->i1 = n * (t + 1) / threads;
    }
    const int rc = run_jobs(out ? lr_write : lr_count, J, sizeof(lr_job), threads);
    free(J);
    return rc;
}

typedef struct {
    const uint8_t *genome;
    const int64_t *starts;
    const uint8_t *strand;
    int64_t sr_len;
    uint32_t t_sub;
    uint64_t seed;
    uint8_t *out;
    int64_t i0, i1;
} sr_job;

static void *sr_write(void *p) {
    sr_job *J = (sr_job *)p;
    for (int64_t i = J->i0; i < J->i1; ++i) {
        rng_t r;
        rseed(&r, J->seed, 2, (uint64_t)i);
        uint8_t *o = J->out + i * J->sr_len;
        memcpy(o, J->genome + J->starts[i], (size_t)J->sr_len);
        if (ru32(&r) < J->t_sub) {
            const int64_t k = (int64_t)rbelow(&r, (uint64_t)J->sr_len);
            o[k] = (uint8_t)((o[k] + 1 + rbelow(&r, 3)) & 3);
        }
        if (J->strand[i]) {
            for (int64_t a = 0, b = J->sr_len - 1; a <= b; ++a, --b) {
                const uint8_t x = (uint8_t)(3 - o[a]), y = (uint8_t)(3 - o[b]);
                o[a] = y;
                o[b] = x;
            }
        }
    }
    return NULL;
}

/* n short reads of sr_len bases at starts / strands into out[n * sr_len] */
int prs_short_reads(const uint8_t *genome, const int64_t *starts, const uint8_t *strand, int64_t n, int64_t sr_len,
                    double p_read_sub, uint64_t seed, int threads, uint8_t *out) {
    if (threads < 1) threads = 1;
    if (n < 0 || sr_len < 0) return -1;
    sr_job *J = (sr_job *)calloc((size_t)threads, sizeof(sr_job));
    if (!J) return -1;
    for (int t = 0; t < threads; ++t) {
        sr_job *j = &J[t];
        j->genome = genome;
        j->starts = starts;
        j->strand = strand;
        j->sr_len = sr_len;
        j->t_sub = thresh(p_read_sub);
        j->seed = seed;
        j->out = out;
        j->i0 = n * t / threads;
        j->i1 = n * (t + 1) / threads;
    }
    const int rc = run_jobs(sr_write, J, sizeof(sr_job), threads);
    free(J);
    return rc;
}
