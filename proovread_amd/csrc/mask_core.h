// Scalar core of the per-iteration masking, shared by the
// device kernel (mask_kernels.hip, executed wave-uniformly) and a host build
// used by the tests (tests/native/mask_host.cpp).
//
// proovread masks every corrected long read after each iteration with
// `SeqFilter --phred-mask <hcr-mask>` (bin/proovread:1701-1716, hcr-mask at
// proovread.cfg:230-242).  SeqFilter is an absent submodule; the procedure is
// its in-tree predecessor, sam2cns:806-951 (mask_hcrs):
//   1. HCRs = maximal runs of quality chars in [phred_min, phred_max] of length
//      >= mask_min + 2*reduce (Fastq::Seq::qual_lcs, Seq.pm:709-717;
//      sam2cns:432-434);
//   2. every HCR loses `reduce` bases at both ends (sticky ends, :824-827);
//   3. read start / end: a leading / trailing unmasked stretch shorter than
//      unmask_min is either grown to unmask_min (shortening the HCR, dropping
//      it when shorter than mask_min) or, if the shortfall is >= end_ratio *
//      unmask_min, masked completely (:829-871);
//   4. repeat: gaps shorter than unmask_min are widened by shrinking both
//      neighbours (floor half left, ceil half right) on a copy; HCRs that
//      become shorter than mask_min are collected, adjacent ones collapse to
//      the later one (:914 compares a length with an array reference, always
//      true); none -> the copy is the result, else drop those HCRs from the
//      unmodified list and repeat (:873-937).
// The remaining HCRs are the MCRs, masked with N (:942-946).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PR_HD __host__ __device__ inline
#else
#define PR_HD inline
#endif

namespace prgpu {

struct MaskCfg {
    int32_t lo_char, hi_char;   // phred_min/max + phred offset
    int32_t lcs_min;            // mask_min + 2 * reduce (>= 1)
    int32_t hcr_min;            // mask_min
    int32_t lcr_min;            // unmask_min
    int32_t sticky;             // reduce
    double end_ratio;
};

struct MaskRun {
    int32_t off, len;
};

// Upper bound of the HCR count of a read of length L: runs of >= lcs_min chars
// separated by >= 1 char.
PR_HD int64_t mask_run_cap(int64_t L, int32_t lcs_min) { return L / (int64_t)(lcs_min > 0 ? lcs_min : 1) + 2; }

PR_HD int mask_ctz64(uint64_t x) { return __builtin_ctzll(x); }

// Feed the in-range bitmap of columns [base, base+valid) (bit i = column base+i,
// bits >= valid are zero).  run_start is the open run's first column or -1.
// Closed runs of length >= lcs_min are appended to out[n] (n counts them even
// when out is null: the device kernel stores from lane 0 only).
PR_HD void mask_runs_feed(uint64_t bits, int64_t base, int valid, int64_t &run_start, int32_t lcs_min, MaskRun *out,
                          int64_t &n, int64_t cap) {
    int p = 0;
    while (p < valid) {
        const uint64_t rest = bits >> p;
        if (run_start < 0) {
            if (rest == 0) return;
            p += mask_ctz64(rest);
            if (p >= valid) return;
            run_start = base + p;
        } else {
            const uint64_t inv = ~rest;   // zeros of the word from p on (shifted-in bits are ones)
            p += inv ? mask_ctz64(inv) : 64;
            if (p >= valid) return;      // the run continues into the next word
            const int64_t end = base + p;
            if (end - run_start >= lcs_min) {
                if (out && n < cap) {
                    out[n].off = (int32_t)run_start;
                    out[n].len = (int32_t)(end - run_start);
                }
                ++n;
            }
            run_start = -1;
        }
    }
}

PR_HD void mask_runs_close(int64_t L, int64_t &run_start, int32_t lcs_min, MaskRun *out, int64_t &n, int64_t cap) {
    if (run_start >= 0 && L - run_start >= lcs_min) {
        if (out && n < cap) {
            out[n].off = (int32_t)run_start;
            out[n].len = (int32_t)(L - run_start);
        }
        ++n;
    }
    run_start = -1;
}

// Steps 2-4 on h[0..n) (in place); tmp has room for n runs.  Returns the MCR count.
PR_HD int64_t mask_resolve(MaskRun *h, int64_t n, int64_t L, const MaskCfg &c, MaskRun *tmp) {
    if (n <= 0) return 0;
    for (int64_t i = 0; i < n; ++i) {
        h[i].off += c.sticky;
        h[i].len -= 2 * c.sticky;
    }
    // head
    {
        const int64_t s = (int64_t)c.lcr_min - h[0].off;
        if (s > 0) {
            if ((double)s < c.end_ratio * (double)c.lcr_min) {
                h[0].len -= (int32_t)s;
                if (h[0].len < c.hcr_min) {
                    for (int64_t i = 1; i < n; ++i) h[i - 1] = h[i];
                    --n;
                } else {
                    h[0].off += (int32_t)s;
                }
            } else {
                h[0].len += h[0].off;
                h[0].off = 0;
            }
        }
    }
    // tail
    if (n > 0) {
        MaskRun &t = h[n - 1];
        const int64_t s = (int64_t)c.lcr_min - (L - ((int64_t)t.off + t.len));
        if (s > 0) {
            if ((double)s < c.end_ratio * (double)c.lcr_min) {
                t.len -= (int32_t)s;
                if (t.len < c.hcr_min) --n;
            } else {
                t.len += (int32_t)(c.lcr_min - s);
            }
        }
    }
    // gap rounds
    while (n > 0) {
        for (int64_t i = 0; i < n; ++i) tmp[i] = h[i];
        // The short HCRs to drop are marked in h[] itself (off -> -off-1; offsets are
        // >= 0): shorts arrive in increasing order and an adjacent later one replaces
        // the earlier, so only the last marked index can be unmarked.
        int64_t n_clean = 0, last_clean = -2;
        int64_t i = 0;
        for (; i < n - 1; ++i) {
            MaskRun &ha = tmp[i];
            MaskRun &hb = tmp[i + 1];
            const int64_t s = (int64_t)c.lcr_min - ((int64_t)hb.off - ((int64_t)ha.off + ha.len));
            if (s > 0) {
                const int64_t a = s / 2;
                const int64_t b = a + s % 2;
                ha.len -= (int32_t)a;
                if (ha.len < c.hcr_min) {
                    if (last_clean == i - 1) {   // replaces the previous short index
                        h[i - 1].off = -(h[i - 1].off) - 1;
                    } else {
                        ++n_clean;
                    }
                    h[i].off = -(h[i].off) - 1;   // mark
                    last_clean = i;
                }
                hb.off += (int32_t)b;
                hb.len -= (int32_t)b;
            }
        }
        if (tmp[i].len < c.hcr_min) {
            if (last_clean == i - 1) {
                h[i - 1].off = -(h[i - 1].off) - 1;
            } else {
                ++n_clean;
            }
            h[i].off = -(h[i].off) - 1;
            last_clean = i;
        }
        if (n_clean == 0) {
            for (int64_t k = 0; k < n; ++k) h[k] = tmp[k];
            break;
        }
        int64_t m = 0;
        for (int64_t k = 0; k < n; ++k)
            if (h[k].off >= 0) h[m++] = h[k];
        n = m;
    }
    return n;
}

}  // namespace prgpu
