// Final quality trimming: the windows `SeqFilter --trim-win
// mean,min` keeps of every corrected read (proovread.cfg:152-155, run once per
// job at bin/proovread:919-943).  SeqFilter is absent; the window search is
// Fastq::Seq::qual_window and its _qw_slide_init / _qw_slide_low /
// _qw_slide_high helpers (lib/Fastq/Seq.pm:1064-1160), restated with its
// quirks:
//   * the low-slide update subtracts X[I-W+1], an element still inside the
//     window (Seq.pm:1122), while the high slide subtracts X[I-W] (:1142);
//   * `WX < SW || X[I-W+1] > S && return 1` (:1113, :1124) ends the low stretch
//     only when WX >= SW and X[I-W+1] > S (&& binds tighter than ||);
//   * the high end rewinds to the last position >= S (:1153) and the window is
//     kept only when its length >= the minimum stretch length (:1159).
// Host code: it runs once per job over the final reads; reads are split over
// worker threads.
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/prgpu.h"

int pr_set_error(int code, const char *msg);

namespace {

struct QW {
    const uint8_t *x;   // phred + offset chars
    int64_t n;
    int off;
    int W, S, H;
    int64_t SW;
    int64_t I = -1, WX = 0;

    int X(int64_t i) const { return (int)x[i] - off; }

    bool init() {
        if (!(I + W < n)) return false;
        WX = 0;
        for (int k = 0; k < W; ++k) {
            ++I;
            if (X(I) < H) return false;
            WX += X(I);
        }
        return true;
    }
    bool low() {
        if (X(I) < H) return false;
        if (!(WX < SW) && X(I - W + 1) > S) return true;
        while (++I < n) {
            if (X(I) < H) return false;
            WX += X(I) - X(I - W + 1);
            if (!(WX < SW) && X(I - W + 1) > S) return true;
        }
        --I;
        return false;
    }
    // -> window length (0: not kept), offset in *o
    int64_t high(int64_t *o, int min_len) {
        *o = I - W + 1;
        while (++I < n) {
            WX += X(I) - X(I - W);
            if (WX < SW || X(I) < H) break;
        }
        --I;
        int64_t j = I;
        while (X(j) < S) --j;   // stops at *o: X(*o) > S when low() returned
        const int64_t l = j - *o + 1;
        return l >= min_len ? l : 0;
    }
};

int64_t windows_of(const uint8_t *q, int64_t n, const pr_trim_params &p, int32_t *out, int64_t cap) {
    QW s{q, n, p.phred_offset, p.size, p.soft, p.hard, (int64_t)p.soft * p.size};
    int64_t k = 0;
    while (s.I < n - s.W) {
        if (!s.init()) continue;
        if (!s.low()) continue;
        int64_t o = 0;
        const int64_t l = s.high(&o, p.min_len);
        if (l) {
            if (k < cap) {
                out[2 * k] = (int32_t)o;
                out[2 * k + 1] = (int32_t)l;
            }
            ++k;
        }
    }
    return k;
}

// windows are disjoint and at least min_len (and >= 1) long
int64_t cap_of(int64_t L, const pr_trim_params &p) { return L / std::max(1, p.min_len) + 1; }

}  // namespace

extern "C" void pr_trim_params_default(pr_trim_params *p) {
    p->size = 10;      // Qual_window_size (Seq.pm:235)
    p->soft = 25;      // Qual_window_min_score_soft (:236)
    p->hard = 3;       // Qual_window_min_score_hard (:237)
    p->min_len = 10;   // Qual_window_min_strecht_length (:238)
    p->phred_offset = 33;
}

extern "C" int pr_trim_params_parse(const char *trim_win, pr_trim_params *p) {
    if (!trim_win || !p) return pr_set_error(PR_ERR_ARG, "null argument");
    pr_trim_params_default(p);
    char *e = nullptr;
    const long a = std::strtol(trim_win, &e, 10);
    if (e == trim_win || *e != ',') return pr_set_error(PR_ERR_ARG, "--trim-win wants mean-min,abs-min");
    const char *b0 = e + 1;
    const long b = std::strtol(b0, &e, 10);
    if (e == b0 || (*e && *e != '\n')) return pr_set_error(PR_ERR_ARG, "--trim-win wants mean-min,abs-min");
    if (a) p->soft = (int32_t)a;   // the class setter ignores 0 (Seq.pm:418-421)
    p->hard = (int32_t)b;
    return 0;
}

static int check_params(const pr_trim_params *p) {
    if (!p || p->size < 1 || p->min_len < 0) return pr_set_error(PR_ERR_ARG, "trim params: size >= 1, min_len >= 0");
    return 0;
}

extern "C" int pr_trim_bound(const pr_trim_params *p, int32_t n, const int64_t *off, int64_t *win_cap) {
    int rc = check_params(p);
    if (rc) return rc;
    if (n < 0 || (n && !off) || !win_cap) return pr_set_error(PR_ERR_ARG, "bad batch");
    int64_t c = 0;
    for (int32_t i = 0; i < n; ++i) c += cap_of(off[i + 1] - off[i], *p);
    *win_cap = c;
    return 0;
}

extern "C" int pr_trim_windows(const pr_trim_params *p, int32_t n, const int64_t *off, const uint8_t *qual,
                               int64_t *win_off, int32_t *win, int32_t *n_win, int n_threads) {
    int rc = check_params(p);
    if (rc) return rc;
    if (n < 0 || (n && (!off || !qual || !win_off || !win || !n_win))) return pr_set_error(PR_ERR_ARG, "bad batch");
    if (n && off[0] != 0) return pr_set_error(PR_ERR_ARG, "offsets must start at 0");
    win_off[0] = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (off[i + 1] < off[i]) return pr_set_error(PR_ERR_ARG, "offsets not monotone");
        win_off[i + 1] = win_off[i] + cap_of(off[i + 1] - off[i], *p);
    }
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min(nt, 64));
    if ((int64_t)nt > n / 16 + 1) nt = (int)(n / 16 + 1);
    std::vector<int> over(nt, 0);
    auto work = [&](int t) {
        for (int32_t i = t; i < n; i += nt) {
            const int64_t cap = win_off[i + 1] - win_off[i];
            const int64_t k = windows_of(qual + off[i], off[i + 1] - off[i], *p, win + 2 * win_off[i], cap);
            if (k > cap) over[t] = 1;
            n_win[i] = (int32_t)std::min(k, cap);
        }
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
        for (auto &x : th) x.join();
    }
    for (int v : over)
        if (v) return pr_set_error(PR_ERR_CAPACITY, "trim windows exceeded their bound");
    return 0;
}
