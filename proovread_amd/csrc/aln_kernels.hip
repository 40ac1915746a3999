// bwa mode on the device: what `bwa-proovread mem` (bin/proovread:1313; absent submodule,
// restated from upstream bwa >= 0.7.13 bwamem.c, parity unpinned) does with a short read
// between seeding and SAM output, around the batched SW kernels (sw_kernels.hip):
//
//   aln_init_kernel   every chain's first seed (rank 0) is extended speculatively in the
//                     first round (a contained rank-0 seed is later skipped and its result
//                     dropped, so the speculation never changes an output)
//   aln_walk_kernel   mem_chain2aln's loop, one lane per read, resumed every round: seeds in
//                     chain order and srt order; a seed inside an earlier region ("around" it
//                     within min(cal_max_gap, band)) is skipped unless a longer (>= 95 %)
//                     extended seed of its chain overlaps it on another diagonal; a seed to
//                     extend whose result is not there yet is requested for the next round and
//                     the lane stops there (decisions before it are final: they only depend on
//                     earlier seeds)
//   aln_final_kernel  mem_sort_dedup_patch (klib introsort by end, redundant hits, colinear
//                     merges through mem_patch_reg whose global scores come from
//                     aln_patch_kernel in extra rounds), the (score, rb, qb) sort with identical
//                     hits removed, mem_mark_primary_se (score, hash_64(read_id + i)) and
//                     mem_reg2sam's -T (per aligned base, proovread cfg:324) and -D filters;
//                     writes the reported alignments in SAM order and marks them for the CIGAR
//                     pass (SEL_CIG)
// One lane per read: the per-read work is a few dozen sequential decisions over
// HBM-resident scratch (latency-bound bookkeeping, no roofline claim).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "aln_core.h"

namespace prgpu {

using namespace alnc;

constexpr int WAVE_SEEDS = ALN_WAVE_SEEDS;

// ---------------------------------------------------------------- round 0
__global__ void __launch_bounds__(256) aln_init_kernel(AlnDev A) {
    // (the round-0 list -- every chain's first seed, sel = SEL_EXT -- is made by aln_list_kernel)
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < A.n_task; t += (int64_t)gridDim.x * blockDim.x)
        (void)aln_init_task(A, t);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < A.n_sr; r += (int64_t)gridDim.x * blockDim.x) {
        A.resume[r] = (int32_t)A.seed_off[r];
        A.npk[r] = 0;
        A.fdone[r] = 0;
        A.nout[r] = 0;
    }
}

// hprev (aln_heads_read's links) with one wave per read: the read's chain heads (a seed whose
// chain differs from its predecessor's) and their (long read, strand) keys are gathered into the
// wave's LDS with a ballot per 64 seeds, then every head's closest earlier head with its key is
// found lane-parallel against the LDS list.  The lane-per-read version followed the heads one
// dependent cnext load at a time and searched its list in HBM scratch: 2.8 ms at configs[1],
// on the critical path in front of round 0's extension.  Reads with more heads than the LDS list
// holds take that path on lane 0.
constexpr int HEADS_CAP = 512;
__global__ void __launch_bounds__(256) aln_heads_kernel(AlnDev A, int cap) {
    __shared__ int32_t sh_key[4][HEADS_CAP];
    __shared__ int32_t sh_head[4][HEADS_CAP];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int32_t *hk = sh_key[wv], *hh = sh_head[wv];
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wv; r < A.n_sr; r += (int64_t)gridDim.x * 4) {
        const int64_t s0 = A.seed_off[r], s1 = A.seed_off[r + 1];
        int nh = 0;
        for (int64_t b = s0; b < s1; b += 64) {
            const int64_t t = b + lane;
            bool head = false;
            int key = 0;
            if (t < s1) {
                head = t == s0 || A.t_chain[t] != A.t_chain[t - 1];
                if (head) key = A.t_lr[t] * 2 + (A.t_strand[t] ? 1 : 0);
            }
            const unsigned long long m = __ballot(head);
            const int pos = nh + __popcll(m & below);
            if (head && pos < cap) {
                hk[pos] = key;
                hh[pos] = (int32_t)t;
            }
            nh += __popcll(m);
        }
        if (nh > cap) {
            if (lane == 0) aln_heads_read(A, r);
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int c = 0; c < nh; c += 64) {
            const int i = c + lane;
            const int key = i < nh ? hk[i] : -1;
            const int jend = (c + 64 < nh ? c + 64 : nh) - 1;   // heads below the chunk's last one
            int p = -1;
            for (int j = 0; j < jend; ++j) {
                const int kj = hk[j];
                if (j < i && kj == key) p = hh[j];
            }
            if (i < nh) A.hprev[hh[i]] = p;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();   // the list is read before the next read rewrites it
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ---------------------------------------------------------------- mem_chain2aln
__global__ void __launch_bounds__(256, 8) aln_walk_kernel(AlnDev A, int big_only) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= A.n_sr) return;
    if (big_only && A.seed_off[r + 1] - A.seed_off[r] <= WAVE_SEEDS) return;   // the wave kernel's
    // requested seeds carry SEL_EXT; aln_list_kernel lists them
    aln_walk_read(A, r, [](int64_t) {});
}

// The seeds flagged SEL_EXT -> tlist (any order: the extension kernels order their tasks
// themselves), their count -> counter[0].  A workgroup takes a contiguous range, counts it,
// reserves its part of the list with ONE device-scope atomic and writes it (a single counter
// word serialises ~88 atomics per us: per-wave or per-lane atomics on it cost 6-8 ms for the
// 10 M first seeds / 0.7 M requests of a configs[1] iteration).
__global__ void __launch_bounds__(256) aln_list_kernel(AlnDev A) {
    __shared__ int32_t ws[4];
    __shared__ int32_t base_s;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t per = ((A.n_task + gridDim.x - 1) / gridDim.x + 255) / 256 * 256;
    const int64_t b0 = (int64_t)blockIdx.x * per;
    const int64_t b1 = b0 + per < A.n_task ? b0 + per : A.n_task;
    int c = 0;
    for (int64_t t = b0 + threadIdx.x; t < b1; t += 256) c += (A.sel[t] & SEL_EXT) ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) ws[wv] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = ws[0] + ws[1] + ws[2] + ws[3];
        base_s = tot ? atomicAdd(&A.counter[0], tot) : 0;
    }
    __syncthreads();
    int base = base_s;
    for (int64_t t0 = b0; t0 < b1; t0 += 256) {
        const int64_t t = t0 + threadIdx.x;
        const bool f = t < b1 && (A.sel[t] & SEL_EXT);
        const unsigned long long m = __ballot(f);
        __syncthreads();   // the previous tile is done with ws
        if (lane == 0) ws[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int x = 0; x < wv; ++x) off += ws[x];
        if (f) A.tlist[off + __popcll(m & ((1ull << lane) - 1))] = (int32_t)t;
        base += ws[0] + ws[1] + ws[2] + ws[3];
    }
}

// early pass (snap != nullptr, on a side stream beside the later extension rounds): only the
// reads whose walk had finished when it was launched, read from a snapshot of `resume` taken on
// the main stream before the launch -- the live array (and the read's decisions / extension
// outputs) of a read still walking is written concurrently by the main stream's rounds
// Persistent: the grid holds the resident workgroups the residency cap allows, and each wave
// takes 64 consecutive reads at a time from a dequeue counter (`next`, zeroed before the launch).
// With one lane per read over the whole read set the cap left 2.34 rounds of workgroups at
// configs[1], the last one a third full.
// complement: the reads the early pass does NOT take (still walking at the snapshot), run on the
// main stream beside the early pass once every walk is done (disjoint reads); no patch requests
// are recorded there either (the late pass replays what is left)
__global__ void __launch_bounds__(256) aln_final_kernel(AlnDev A, const int32_t *snap, int32_t *next, int complement,
                                                        int big_only) {
    const int lane = threadIdx.x & 63;
    const bool early = snap != nullptr;
    for (;;) {
        int c = 0;
        if (lane == 0) c = atomicAdd(next, 1);
        c = __builtin_amdgcn_readfirstlane(c);
        if ((int64_t)c * 64 >= A.n_sr) break;
        const int64_t r = (int64_t)c * 64 + lane;
        if (r >= A.n_sr) continue;
        if (early && (snap[r] < A.seed_off[r + 1]) != (complement != 0)) continue;   // (not) walking at the snapshot
        if (big_only && A.seed_off[r + 1] - A.seed_off[r] <= WAVE_SEEDS) continue;   // the wave kernel's
        AlnPatch req;
        if (aln_final_read(A, r, &req) && !early) {   // a patch score is needed: the read is replayed later
            const int slot = atomicAdd(&A.counter[1], 1);
            if (slot < A.preq_cap) A.preq[slot] = req;
        }
    }
}

// ---------------------------------------------------------------- the wave-per-read paths
// A read of at most WAVE_SEEDS seeds (at configs[1]'s bwa-sr-1: 75 on average, 104 at the 99th
// percentile, 132 at most in a 20 k-read sample) is walked and finalised by ONE wave, its
// seeds / regions staged in LDS: every containment test of a seed against the read's regions,
// every rank of a sort and every secondary test runs lane-parallel over LDS, where the lane
// kernels above made each of them a chain of dependent HBM/L2 loads of one lane (measured
// waiting 94 % of their cycles).  The decisions are the lane path's, statement for statement:
// the sequential parts (mem_sort_dedup_patch's redundancy / patch loop, and a sort whose keys
// tie, where klib's introsort order decides) run on lane 0 through the same aln_core.h code.
// Larger reads keep the lane kernels (big_only), so mr-mode reads lose nothing.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WalkLds {   // one read's seeds (5.6 KB)
    int32_t key[WAVE_SEEDS], hk[WAVE_SEEDS], qbeg[WAVE_SEEDS], rbeg[WAVE_SEEDS], slen[WAVE_SEEDS];
    int32_t bqb[WAVE_SEEDS], bqe[WAVE_SEEDS], brb[WAVE_SEEDS], bre[WAVE_SEEDS], bw[WAVE_SEEDS];   // regions
    int16_t cst[WAVE_SEEDS];   // first seed of the seed's chain
    uint8_t dec[WAVE_SEEDS], ext[WAVE_SEEDS];
};

// aln_walk_read for read r (s0, ns seeds, resumed at local seed kl) by the calling wave.  The
// walk's per-seed test (around a region before it and no longer chain mate on another
// diagonal) only changes when a region is made, so every lane keeps the test's two parts for
// its two seeds (`around`, `other`) and updates them when one is: the next seed to decide is the
// first open seed whose test fails (a ballot), the open seeds before it are skipped (dec 2) --
// the order-by-order walk's decisions, at one round of LDS work per region instead of per seed.
__device__ void walk_wave_read(const AlnDev &A, WalkLds &L, int64_t r, int64_t s0, int ns, int kl, int lane) {
    const int lq = (int)(A.sr_off[r + 1] - A.sr_off[r]);
    for (int j = lane; j < ns; j += 64) {   // the last round's results, the seeds, the regions
        const int64_t t = s0 + j;
        uint8_t e = A.ext[t];
        if (A.sel[t] & SEL_EXT) {
            e = 1;
            A.ext[t] = 1;
            A.sel[t] = 0;
        }
        L.dec[j] = A.dec[t];
        L.ext[j] = e;
        L.key[j] = A.t_lr[t] * 2 + (A.t_strand[t] ? 1 : 0);
        L.qbeg[j] = A.t_qbeg[t];
        L.rbeg[j] = A.t_rbeg[t];
        L.slen[j] = A.t_slen[t];
        if (e) {
            L.bqb[j] = A.o_qb[t];
            L.bqe[j] = A.o_qe[t];
            L.brb[j] = A.o_rb[t];
            L.bre[j] = A.o_re[t];
            L.bw[j] = A.o_w[t];
        }
    }
    int carry = 0;   // chain starts: a ballot of the starts, the last one at or before each seed
    for (int b = 0; b < ns; b += 64) {
        const int j = b + lane;
        const bool st = j < ns && (j == 0 || A.t_chain[s0 + j] != A.t_chain[s0 + j - 1]);
        const uint64_t m = __ballot(st) & ((2ull << lane) - 1);
        const int c = m ? b + 63 - __builtin_clzll(m) : carry;
        if (j < ns) L.cst[j] = (int16_t)c;
        carry = __shfl(c, 63, 64);
    }
    wsync();
    for (int j = lane; j < ns; j += 64) L.hk[j] = L.key[L.cst[j]];
    wsync();
    // the lane's seeds j0 = lane, j1 = lane + 64
    const int j0 = lane, j1 = lane + 64;
    const bool v0 = j0 < ns, v1 = j1 < ns;
    int64_t rb0 = 0, rb1 = 0;
    int qb0 = 0, qb1 = 0, sl0 = 0, sl1 = 0, cs0 = 0, cs1 = 0, hk0 = 0, hk1 = 0;
    if (v0) rb0 = L.rbeg[j0], qb0 = L.qbeg[j0], sl0 = L.slen[j0], cs0 = L.cst[j0], hk0 = L.hk[j0];
    if (v1) rb1 = L.rbeg[j1], qb1 = L.qbeg[j1], sl1 = L.slen[j1], cs1 = L.cst[j1], hk1 = L.hk[j1];
    bool ar0 = false, ot0 = false, ar1 = false, ot1 = false;
    // region i (dec 1) against the lane's seeds after it: aln_around_any's set (the seed's chain
    // mates, and the earlier chains whose head has its chain head's long read and strand) and
    // the walk's "longer chain mate on another diagonal"
    auto add_region = [&](int i) {
        const int pqb = L.bqb[i], pqe = L.bqe[i], prb = L.brb[i], pre = L.bre[i], psl = L.slen[i], pw = L.bw[i];
        const int hki = L.hk[i], iq = L.qbeg[i];
        const int64_t ir = L.rbeg[i];
        if (v0 && i < j0) {
            if (!ar0 && (i >= cs0 || hki == hk0)) ar0 = around_f(A, pqb, pqe, prb, pre, psl, pw, rb0, qb0, sl0, lq);
            if (!ot0 && i >= cs0) ot0 = other_diag(rb0, qb0, sl0, ir, iq, psl);
        }
        if (v1 && i < j1) {
            if (!ar1 && (i >= cs1 || hki == hk1)) ar1 = around_f(A, pqb, pqe, prb, pre, psl, pw, rb1, qb1, sl1, lq);
            if (!ot1 && i >= cs1) ot1 = other_diag(rb1, qb1, sl1, ir, iq, psl);
        }
    };
    {   // the regions made in earlier rounds
        const uint64_t m0 = __ballot(v0 && L.dec[j0] == 1), m1 = __ballot(v1 && L.dec[j1] == 1);
        for (uint64_t m = m0; m; m &= m - 1) add_region(__builtin_ctzll(m));
        for (uint64_t m = m1; m; m &= m - 1) add_region(64 + __builtin_ctzll(m));
    }
    const int k_first = kl;
    for (;;) {
        // the next seed to decide: the first open one from kl whose test fails
        const bool c0f = v0 && j0 >= kl && L.dec[j0] == 0 && !(ar0 && !ot0);
        const bool c1f = v1 && j1 >= kl && L.dec[j1] == 0 && !(ar1 && !ot1);
        const uint64_t m0 = __ballot(c0f), m1 = __ballot(c1f);
        const int ks = m0 ? __builtin_ctzll(m0) : (m1 ? 64 + __builtin_ctzll(m1) : ns);
        if (v0 && j0 >= kl && j0 < ks && L.dec[j0] == 0) L.dec[j0] = 2;   // inside a region: skipped
        if (v1 && j1 >= kl && j1 < ks && L.dec[j1] == 0) L.dec[j1] = 2;
        wsync();
        if (ks >= ns) break;
        if (!L.ext[ks]) {   // extension needed: request it and the likely ones after it, resume here
            // a later open seed is requested with it unless it is inside a region and no chain
            // mate that is not skipped (>= 95 % of its length, another diagonal) could save it
            auto spec = [&](int kk, bool ar, int cs, int64_t rb, int qb, int sl) {
                if (kk <= ks || L.dec[kk] || L.ext[kk]) return;
                if (ar) {
                    bool mo = false;   // aln_maybe_other
                    for (int j = cs; j < kk && !mo; ++j)
                        mo = L.dec[j] != 2 && other_diag(rb, qb, sl, L.rbeg[j], L.qbeg[j], L.slen[j]);
                    if (!mo) return;
                }
                A.sel[s0 + kk] = SEL_EXT;
            };
            if (v0) spec(j0, ar0, cs0, rb0, qb0, sl0);
            if (v1) spec(j1, ar1, cs1, rb1, qb1, sl1);
            if (lane == 0) {
                A.sel[s0 + ks] = SEL_EXT;
                A.resume[r] = (int32_t)(s0 + ks);
            }
            for (int j = k_first + lane; j < ks; j += 64) A.dec[s0 + j] = L.dec[j];
            return;
        }
        if (lane == 0) L.dec[ks] = 1;
        add_region(ks);
        wsync();
        kl = ks + 1;
    }
    if (lane == 0) A.resume[r] = (int32_t)(s0 + ns);
    for (int j = k_first + lane; j < ns; j += 64) A.dec[s0 + j] = L.dec[j];
}

// a wave per 64 consecutive reads: the ones still walking (and small enough) one after another
__global__ void __launch_bounds__(256) aln_walk_wave_kernel(AlnDev A) {
    __shared__ WalkLds sh[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t base = ((int64_t)blockIdx.x * 4 + wv) * 64;
    if (base >= A.n_sr) return;
    const int64_t r = base + lane;
    long long s0 = 0;
    int ns = 0, kl = 0;
    bool act = false;
    if (r < A.n_sr) {
        s0 = A.seed_off[r];
        const int64_t s1 = A.seed_off[r + 1], k = A.resume[r];
        ns = (int)(s1 - s0);
        kl = (int)(k - s0);
        act = k < s1 && ns <= WAVE_SEEDS;
    }
    for (uint64_t m = __ballot(act); m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        walk_wave_read(A, sh[wv], base + l, (int64_t)__shfl(s0, l, 64), __shfl(ns, l, 64), __shfl(kl, l, 64), lane);
        wsync();   // the LDS is the next read's
    }
}

struct RegW {   // a region of the wave final pass (LDS)
    int64_t rb, re;
    uint64_t hash;
    int32_t qb, qe, score, truesc, w, lr;
    int16_t task, secondary;   // task: the seed's index in the read; secondary: an ix position or -1
    uint8_t strand, patched, pad[2];
};

struct FinalLds {   // one read's regions (7.7 KB)
    RegW R[WAVE_SEEDS];
    int32_t ix[WAVE_SEEDS];
    uint8_t pass[WAVE_SEEDS];
};

// ix[0, n) sorted by lt, lane-parallel: every element's rank is the number of elements before
// it; -> false (ix untouched) when two keys tie, where klib's order decides (the caller then
// runs introsort on lane 0)
template <class Lt>
__device__ bool rank_sort(FinalLds &L, int n, int lane, Lt lt) {
    const int e0 = lane < n ? L.ix[lane] : 0, e1 = lane + 64 < n ? L.ix[lane + 64] : 0;
    const RegW a0 = L.R[e0], a1 = L.R[e1];
    int r0 = 0, r1 = 0;
    bool tie = false;
    for (int j = 0; j < n; ++j) {
        const RegW &b = L.R[L.ix[j]];
        if (lt(b, a0)) ++r0;
        else if (j != lane && !lt(a0, b)) tie = true;
        if (lt(b, a1)) ++r1;
        else if (j != lane + 64 && !lt(a1, b) && lane + 64 < n) tie = true;
    }
    if (__ballot(tie && lane < n)) return false;
    wsync();   // every lane has read ix
    if (lane < n) L.ix[r0] = e0;
    if (lane + 64 < n) L.ix[r1] = e1;
    wsync();
    return true;
}

__device__ __forceinline__ int64_t rl64(int64_t v, int l) {   // lane l's 64-bit value (l uniform)
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// The final pass of a read with at most 64 regions (every read at configs[1]): lane i holds
// the region at position i in registers, a sort's ranks come from readlane broadcasts, the
// regions move to their ranks through LDS (L.R is kept in position order with L.ix the
// identity, so the lane-0 fallbacks -- a tie under a sort key, a region that may be redundant
// or merged -- run aln_core.h's code on it unchanged).
__device__ int final_wave_small(const AlnDev &A, FinalLds &L, int64_t r, int64_t s0, int ns, int n, int lane,
                                AlnPatch *req) {
    RegW e;
    bool v = lane < n;
    if (v) e = L.R[lane];
    auto place = [&](int rank) {   // every region to its rank
        wsync();
        if (v) L.R[rank] = e;
        wsync();
        if (v) e = L.R[lane];
    };
    auto adopt = [&](int m) {   // L.R in L.ix[0, m)'s order (after a lane-0 sort), L.ix the identity
        wsync();
        RegW t;
        if (lane < m) t = L.R[L.ix[lane]];
        wsync();
        if (lane < m) L.R[lane] = t;
        L.ix[lane] = lane;
        L.ix[lane + 64] = lane + 64;
        n = m;
        v = lane < n;
        if (v) e = t;
        wsync();
    };
    if (n > 1) {
        int rk = 0;   // alnreg_slt2: by end
        bool tie = false;
        for (int j = 0; j < n; ++j) {
            const int64_t re = rl64(e.re, j);
            rk += re < e.re;
            tie |= j != lane && re == e.re;
        }
        if (__ballot(v && tie)) {
            if (lane == 0) introsort(n, L.ix, L.R, LtEnd());
            adopt(n);
        } else {
            place(rk);
        }
        // redundant / colinear regions: only where a region starts within max_chain_gap of its
        // predecessor's end on the same long read does mem_sort_dedup_patch's loop do anything
        const int plr = __shfl(e.lr, lane > 0 ? lane - 1 : 0, 64);
        const int64_t pre = (int64_t)__shfl((long long)e.re, lane > 0 ? lane - 1 : 0, 64);
        if (__ballot(v && lane > 0 && e.lr == plr && e.rb < pre + A.max_chain_gap)) {
            int need = 0;
            if (lane == 0) need = dedup_patch(A, r, s0, L.R, L.ix, n, req);
            need = __shfl(need, 0, 64);
            wsync();
            if (need) return 1;
            if (v) e = L.R[lane];
        }
        const bool live = v && e.qe > e.qb;
        const uint64_t lm = __ballot(live);
        if (lm != __ballot(v)) {   // the regions left, in order
            wsync();
            if (live) L.R[__popcll(lm & ((1ull << lane) - 1))] = e;
            n = __popcll(lm);
            v = lane < n;
            wsync();
            if (v) e = L.R[lane];
        }
        rk = 0;   // alnreg_slt: score, then rb, then qb
        tie = false;
        for (int j = 0; j < n; ++j) {
            const int sc = __builtin_amdgcn_readlane(e.score, j), qb = __builtin_amdgcn_readlane(e.qb, j);
            const int64_t rb = rl64(e.rb, j);
            rk += sc > e.score || (sc == e.score && (rb < e.rb || (rb == e.rb && qb < e.qb)));
            tie |= j != lane && sc == e.score && rb == e.rb && qb == e.qb;
        }
        if (__ballot(v && tie)) {   // identical hits: klib's order decides which one stays
            int nn = 0;
            if (lane == 0) {
                introsort(n, L.ix, L.R, LtScore());
                nn = drop_identical(n, L.ix, L.R);
            }
            adopt(__shfl(nn, 0, 64));
        } else {
            place(rk);
        }
    }
    // mem_mark_primary_se: hash_64 is a bijection, so (score, hash) never ties
    if (v) e.hash = hash_64((uint64_t)(A.read_id0 + r + lane));
    if (n > 1) {
        int rk = 0;
        bool tie = false;
        for (int j = 0; j < n; ++j) {
            const int sc = __builtin_amdgcn_readlane(e.score, j);
            const uint64_t h = (uint64_t)rl64((int64_t)e.hash, j);
            rk += sc > e.score || (sc == e.score && h < e.hash);
            tie |= j != lane && sc == e.score && h == e.hash;
        }
        if (__ballot(v && tie)) {
            wsync();
            if (v) L.R[lane] = e;
            wsync();
            if (lane == 0) introsort(n, L.ix, L.R, LtHash());
            adopt(n);
        } else {
            place(rk);
        }
    }
    int sec = -1;   // the first earlier primary the region overlaps (mem_mark_primary_se_core)
    for (int i = 1; i < n; ++i) {
        const int aqb = __builtin_amdgcn_readlane(e.qb, i), aqe = __builtin_amdgcn_readlane(e.qe, i);
        bool c = false;
        if (lane < i && sec < 0) {
            const int b_max = e.qb > aqb ? e.qb : aqb;
            const int e_min = e.qe < aqe ? e.qe : aqe;
            if (e_min > b_max) {
                const int min_l = aqe - aqb < e.qe - e.qb ? aqe - aqb : e.qe - e.qb;
                c = e_min - b_max >= min_l * A.mask_level;
            }
        }
        const uint64_t mk = __ballot(c);
        if (mk && lane == i) sec = __builtin_ctzll(mk);
    }
    // mem_reg2sam: -T per aligned base, -D for secondaries; SAM order; mark for the CIGAR pass
    for (int j = lane; j < ns; j += 64) L.pass[j] = 0;
    wsync();
    const int sec_score = __shfl(e.score, sec >= 0 ? sec : lane, 64);
    bool ok = v && (double)e.score >= A.min_score_per_base * (double)(e.qe - e.qb);
    if (ok && sec >= 0 && e.score < sec_score * A.drop_ratio) ok = false;
    const uint64_t mk = __ballot(ok);
    if (ok) {
        const int o = __popcll(mk & ((1ull << lane) - 1));
        const int64_t t = s0 + e.task;
        const int64_t base = fr_of(A, e.lr, e.strand, 0);
        A.o_qb[t] = e.qb;
        A.o_rb[t] = (int32_t)(e.rb - base);
        A.o_score[t] = e.score;
        A.o_truesc[t] = e.truesc;
        A.o_w[t] = e.w;
        L.pass[e.task] = 1;
        A.olist[s0 + o] = (int32_t)t;
        A.oflag[s0 + o] = (e.strand ? 0x10 : 0) | (sec >= 0 ? 0x100 : (o > 0 ? 0x800 : 0));
    }
    wsync();
    for (int j = lane; j < ns; j += 64) {
        const uint8_t pm = L.pass[j];
        A.o_pass[s0 + j] = pm;
        A.sel[s0 + j] = pm ? SEL_CIG : 0;
    }
    if (lane == 0) {
        A.nout[r] = __popcll(mk);
        A.fdone[r] = 1;
    }
    return 0;
}

// aln_final_read for read r by the calling wave -> 1: the global score of patch *req (lane 0's)
// is needed first
__device__ int final_wave_read(const AlnDev &A, FinalLds &L, int64_t r, int64_t s0, int ns, int lane, AlnPatch *req) {
    int n = 0;
    for (int b = 0; b < ns; b += 64) {   // the regions, in seed order
        const int j = b + lane;
        const int64_t t = s0 + j;
        const bool reg = j < ns && A.dec[t] == 1;
        const uint64_t m = __ballot(reg);
        if (reg) {
            const int pos = n + __popcll(m & ((1ull << lane) - 1));
            RegW &g = L.R[pos];
            const int lr = A.t_lr[t], st = A.t_strand[t];
            const int64_t base = fr_of(A, lr, st, 0);
            g.rb = base + A.o_rb[t];
            g.re = base + A.o_re[t];
            g.qb = A.o_qb[t];
            g.qe = A.o_qe[t];
            g.score = A.o_score[t];
            g.truesc = A.o_truesc[t];
            g.w = A.o_w[t];
            g.lr = lr;
            g.strand = (uint8_t)st;
            g.task = (int16_t)j;
            g.secondary = -1;
            g.patched = 0;
            L.ix[pos] = pos;
        }
        n += __popcll(m);
    }
    wsync();
    if (n <= 64) return final_wave_small(A, L, r, s0, ns, n, lane, req);
    if (n > 1) {
        if (!rank_sort(L, n, lane, LtEnd())) {
            if (lane == 0) introsort(n, L.ix, L.R, LtEnd());
            wsync();
        }
        int need = 0;
        if (lane == 0) need = dedup_patch(A, r, s0, L.R, L.ix, n, req);
        need = __shfl(need, 0, 64);
        wsync();
        if (need) return 1;
        int m = 0;   // the regions left, in order
        for (int b = 0; b < n; b += 64) {
            const int i = b + lane;
            const int e = i < n ? L.ix[i] : 0;
            const bool live = i < n && L.R[e].qe > L.R[e].qb;
            const uint64_t mk = __ballot(live);
            wsync();
            if (live) L.ix[m + __popcll(mk & ((1ull << lane) - 1))] = e;
            m += __popcll(mk);
            wsync();
        }
        n = m;
        if (!rank_sort(L, n, lane, LtScore())) {   // a tie is an identical hit: klib's order keeps one
            int nn = 0;
            if (lane == 0) {
                introsort(n, L.ix, L.R, LtScore());
                nn = drop_identical(n, L.ix, L.R);
            }
            n = __shfl(nn, 0, 64);
            wsync();
        }
    }
    // mem_mark_primary_se: hash_64 is a bijection, so (score, hash) never ties
    for (int i = lane; i < n; i += 64) L.R[L.ix[i]].hash = hash_64((uint64_t)(A.read_id0 + r + i));
    wsync();
    if (n > 1 && !rank_sort(L, n, lane, LtHash())) {
        if (lane == 0) introsort(n, L.ix, L.R, LtHash());
        wsync();
    }
    for (int i = 1; i < n; ++i) {   // secondaries: the first earlier primary a region overlaps
        const RegW ai = L.R[L.ix[i]];
        int first = -1;
        for (int b = 0; b < i; b += 64) {
            const int j = b + lane;
            bool c = false;
            if (j < i) {
                const RegW &aj = L.R[L.ix[j]];
                if (aj.secondary < 0) {
                    const int b_max = aj.qb > ai.qb ? aj.qb : ai.qb;
                    const int e_min = aj.qe < ai.qe ? aj.qe : ai.qe;
                    if (e_min > b_max) {
                        const int min_l = ai.qe - ai.qb < aj.qe - aj.qb ? ai.qe - ai.qb : aj.qe - aj.qb;
                        c = e_min - b_max >= min_l * A.mask_level;
                    }
                }
            }
            const uint64_t mk = __ballot(c);
            if (mk) {
                first = b + __builtin_ctzll(mk);
                break;
            }
        }
        if (first >= 0) {
            if (lane == 0) L.R[L.ix[i]].secondary = (int16_t)first;
            wsync();
        }
    }
    // mem_reg2sam: -T per aligned base, -D for secondaries; SAM order; mark for the CIGAR pass
    for (int j = lane; j < ns; j += 64) L.pass[j] = 0;
    wsync();
    int no = 0;
    for (int b = 0; b < n; b += 64) {
        const int k = b + lane;
        bool ok = false;
        RegW p;
        if (k < n) {
            p = L.R[L.ix[k]];
            ok = (double)p.score >= A.min_score_per_base * (double)(p.qe - p.qb);
            if (ok && p.secondary >= 0 && p.score < L.R[L.ix[p.secondary]].score * A.drop_ratio) ok = false;
        }
        const uint64_t mk = __ballot(ok);
        if (ok) {
            const int o = no + __popcll(mk & ((1ull << lane) - 1));
            const int64_t t = s0 + p.task;
            const int64_t base = fr_of(A, p.lr, p.strand, 0);
            A.o_qb[t] = p.qb;
            A.o_rb[t] = (int32_t)(p.rb - base);
            A.o_score[t] = p.score;
            A.o_truesc[t] = p.truesc;
            A.o_w[t] = p.w;
            L.pass[p.task] = 1;
            A.olist[s0 + o] = (int32_t)t;
            A.oflag[s0 + o] = (p.strand ? 0x10 : 0) | (p.secondary >= 0 ? 0x100 : (o > 0 ? 0x800 : 0));
        }
        no += __popcll(mk);
    }
    wsync();
    for (int j = lane; j < ns; j += 64) {
        const uint8_t pm = L.pass[j];
        A.o_pass[s0 + j] = pm;
        A.sel[s0 + j] = pm ? SEL_CIG : 0;
    }
    if (lane == 0) {
        A.nout[r] = no;
        A.fdone[r] = 1;
    }
    return 0;
}

// a wave per 64 consecutive reads; snap / complement as aln_final_kernel's
__global__ void __launch_bounds__(128) aln_final_wave_kernel(AlnDev A, const int32_t *snap, int complement) {
    __shared__ FinalLds sh[2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool early = snap != nullptr;
    const int64_t base = ((int64_t)blockIdx.x * 2 + wv) * 64;
    if (base >= A.n_sr) return;
    const int64_t r = base + lane;
    long long s0 = 0;
    int ns = 0;
    bool act = false;
    if (r < A.n_sr) {
        s0 = A.seed_off[r];
        const int64_t s1 = A.seed_off[r + 1];
        ns = (int)(s1 - s0);
        act = ns <= WAVE_SEEDS && !A.fdone[r] && (!early || (snap[r] < s1) == (complement != 0));
    }
    for (uint64_t m = __ballot(act); m; m &= m - 1) {
        const int l = __builtin_ctzll(m);
        AlnPatch req;
        const int need = final_wave_read(A, sh[wv], base + l, (int64_t)__shfl(s0, l, 64), __shfl(ns, l, 64), lane, &req);
        if (need && !early && lane == 0) {   // replayed once the score is there
            const int slot = atomicAdd(&A.counter[1], 1);
            if (slot < A.preq_cap) A.preq[slot] = req;
        }
        wsync();
    }
}

// mem_patch_reg's global score (bwa_gen_cigar2's ksw_global2, score only) with one wave per
// patch: lane l owns CB consecutive query columns, row i runs on lane l at step i + l (an
// anti-diagonal wavefront), F(i, first column) and H(i-1, first column - 1) come from the lane
// to the left through shuffles, and the band's outside reads as the very negative values the
// row-by-row kernel leaves there.  aln_patch_kernel (one lane per patch, H/E rows in HBM) walked
// every cell with a dependent global load: 6.5 ms at configs[1] bwa-sr-2 for its longest patch.
constexpr int PATCH_REF_MAX = 2048;

template <int CB>
__device__ int patch_wave_score(const AlnDev &A, const AlnPatch &P, int lq, int rlen, int w, const uint8_t *sref,
                                int lane) {
    constexpr int NEG = -0x40000000;
    const uint8_t *Q = A.sr + A.sr_off[P.read] + P.qb;
    const int cb = (lq + 63) / 64, nl = (lq + cb - 1) / cb, c0 = lane * cb;
    const int oe_del = A.o_del + A.e_del, oe_ins = A.o_ins + A.e_ins;
    int8_t qv[CB];
    int hp[CB], ev[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) {
        const int j = c0 + c;
        const bool in = c < cb && j < lq;
        qv[c] = in ? (int8_t)(P.strand ? Q[lq - 1 - j] : Q[j]) : (int8_t)4;
        hp[c] = in && j + 1 <= w ? -(A.o_ins + A.e_ins * (j + 1)) : NEG;   // H(-1, j)
        ev[c] = NEG;
    }
    int pub_f = NEG, pub_hd = NEG, score = NEG;
    const int nsteps = rlen + nl - 1;
    for (int st = 0; st < nsteps; ++st) {
        const int fin = __shfl_up(pub_f, 1, 64), hdin = __shfl_up(pub_hd, 1, 64);
        const int i = st - lane;
        if (lane < nl && i >= 0 && i < rlen) {
            int f, dg;
            if (lane == 0) {
                f = NEG;
                dg = i == 0 ? 0 : (i - 1 <= w ? -(A.o_del + A.e_del * i) : NEG);   // H(i-1, -1)
            } else {
                f = fin;
                dg = hdin;
            }
            const int tb = sref[i];
            const int beg = i > w ? i - w : 0, end = i + w + 1 < lq ? i + w + 1 : lq;
            int hlast = NEG;   // H(i-1, last column), for the right lane
#pragma unroll
            for (int c = 0; c < CB; ++c)
                if (c == cb - 1) hlast = hp[c];
#pragma unroll
            for (int c = 0; c < CB; ++c) {
                if (c >= cb) break;
                const int j = c0 + c;
                const int old = hp[c];
                if (j >= beg && j < end) {
                    const int qb = qv[c];
                    const int m = dg + ((tb > 3 || qb > 3) ? -1 : (tb == qb ? A.a : -A.b));
                    int h = m >= ev[c] ? m : ev[c];
                    h = h >= f ? h : f;
                    hp[c] = h;
                    int t = m - oe_del;
                    const int e = ev[c] - A.e_del;
                    ev[c] = e > t ? e : t;
                    t = m - oe_ins;
                    f -= A.e_ins;
                    f = f > t ? f : t;
                } else {
                    hp[c] = NEG;
                    ev[c] = NEG;
                    f = NEG;
                }
                dg = old;
            }
            pub_f = f;
            pub_hd = hlast;
            if (i == rlen - 1 && lq - 1 >= c0 && lq - 1 < c0 + cb) {
#pragma unroll
                for (int c = 0; c < CB; ++c)
                    if (c0 + c == lq - 1) score = hp[c];
            }
        }
    }
    return __shfl(score, (lq - 1) / cb, 64);
}

__global__ void __launch_bounds__(256) aln_patch_wave_kernel(AlnDev A, int n_req, int32_t *pool, int64_t stride) {
    __shared__ uint8_t sref[4][PATCH_REF_MAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int k = blockIdx.x * 4 + wv;
    if (k >= n_req) return;
    const AlnPatch P = A.preq[k];
    const int lq = P.qe - P.qb, rlen = P.re - P.rb;
    int score;
    if (lq <= 0 || rlen <= 0 || (lq == rlen && P.w == 0) || lq > 64 * 16 || rlen > PATCH_REF_MAX) {
        if (lane == 0) score = aln_patch_score(A, P, pool + (int64_t)k * stride, stride);   // aln_patch_kernel's way
    } else {
        const uint8_t *Lr = A.lr + A.lr_off[P.lr];
        const int L = (int)(A.lr_off[P.lr + 1] - A.lr_off[P.lr]);
        for (int i = lane; i < rlen; i += 64) {   // the strand reference row, reversed on the reverse strand
            const int x = P.strand ? P.re - 1 - i : P.rb + i;
            int c = P.strand ? Lr[L - 1 - x] : Lr[x];
            if (P.strand && c < 4) c = 3 - c;
            sref[wv][i] = (uint8_t)c;
        }
        wsync();
        const int mn = lq < rlen ? lq : rlen;   // the band, as aln_patch_score's
        const int max_ins = (int)((double)(mn * A.a - A.o_ins) / A.e_ins + 1.);
        const int max_del = (int)((double)(mn * A.a - A.o_del) / A.e_del + 1.);
        int max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        const int dl = rlen > lq ? rlen - lq : lq - rlen;
        int w = (max_gap + dl + 1) >> 1;
        w = w < P.w ? w : P.w;
        w = w > dl + 3 ? w : dl + 3;
        score = lq <= 64 * 4 ? patch_wave_score<4>(A, P, lq, rlen, w, sref[wv], lane)
                             : patch_wave_score<16>(A, P, lq, rlen, w, sref[wv], lane);
    }
    if (lane == 0) {
        A.pscore[A.seed_off[P.read] + P.m] = score;
        A.npk[P.read] = P.m + 1;
    }
}

__global__ void __launch_bounds__(64) aln_patch_kernel(AlnDev A, int n_req, int32_t *pool, int64_t stride) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_req) return;
    const AlnPatch P = A.preq[k];
    A.pscore[A.seed_off[P.read] + P.m] = aln_patch_score(A, P, pool + (int64_t)k * stride, stride);
    A.npk[P.read] = P.m + 1;
}

// ---------------------------------------------------------------- outputs
__global__ void __launch_bounds__(256) aln_slot_kernel(AlnDev A, int64_t *slot) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < A.n_task; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t v = 0;
        if (A.sel[t] & SEL_CIG) {
            const int64_t r = A.t_sr[t];
            v = cig_slot_ops((int)(A.sr_off[r + 1] - A.sr_off[r]));
        }
        slot[t] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) slot[A.n_task] = 0;
}
__global__ void __launch_bounds__(256) aln_nout64_kernel(const int32_t *nout, int64_t n, int64_t *o) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= n; r += (int64_t)gridDim.x * blockDim.x)
        o[r] = r < n ? nout[r] : 0;
}
// 16 lanes per read (a read reports ~20 alignments at configs[1]: one lane per read copied them
// one dependent pair of loads at a time)
__global__ void __launch_bounds__(256) aln_compact_kernel(AlnDev A, const int64_t *aoff, int32_t *alist, int32_t *aflag) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int sub = (int)(gid & 15);
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 4;
    for (int64_t r = gid >> 4; r < A.n_sr; r += stride) {
        const int64_t s0 = A.seed_off[r], o = aoff[r];
        const int n = A.nout[r];
        for (int i = sub; i < n; i += 16) {
            alist[o + i] = A.olist[s0 + i];
            aflag[o + i] = A.oflag[s0 + i];
        }
    }
}
__global__ void __launch_bounds__(256) aln_key_kernel(const int32_t *alist, const int32_t *t_lr, int64_t n, int32_t *key,
                                                      int32_t *cnt) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t lr = t_lr[alist[i]];
        key[i] = lr;
        atomicAdd(&cnt[lr], 1);
    }
}
__global__ void __launch_bounds__(256) aln_cnt64_kernel(const int32_t *cnt, int32_t n, int64_t *o) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
        o[i] = i < n ? cnt[i] : 0;
}

__global__ void __launch_bounds__(256) sw_gather_kernel(SwGather G) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < G.n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t t = G.list[i];
        if (G.o_sr) G.o_sr[i] = G.t_sr[t];
        if (G.o_lr) G.o_lr[i] = G.t_lr[t];
        if (G.o_task) G.o_task[i] = t;
        if (G.o_status) G.o_status[i] = G.status[t];
        if (G.o_pos) G.o_pos[i] = G.pos[t];
        if (G.o_score) G.o_score[i] = G.score[t];
        if (G.o_ncig) G.o_ncig[i] = G.ncig[t];
        if (G.o_qb) G.o_qb[i] = G.qb[t];
        if (G.o_qe) G.o_qe[i] = G.qe[t];
        if (G.o_rb) G.o_rb[i] = G.rb[t];
        if (G.o_re) G.o_re[i] = G.re[t];
        if (G.o_truesc) G.o_truesc[i] = G.truesc[t];
        if (G.o_strand) G.o_strand[i] = G.strand[t];
        if (G.o_pass) G.o_pass[i] = G.pass[t];
        if (G.o_cig_at) G.o_cig_at[i] = G.cig_at[t];
    }
}

__global__ void __launch_bounds__(256) aln_unpack_kernel(const pr_seed_task *src, int64_t n, int32_t *sr, int32_t *lr,
                                                         uint8_t *strand, int32_t *qbeg, int32_t *rbeg, int32_t *slen,
                                                         int32_t *chain, int32_t *n_first, int32_t *cnext) {
    __shared__ int32_t nf;   // first seeds of this workgroup: one device-scope atomic per workgroup
    if (threadIdx.x == 0) nf = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n; t0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = t0 + threadIdx.x;
        bool first = false;
        if (t < n) {
            const pr_seed_task x = src[t];
            sr[t] = x.sr;
            lr[t] = x.lr;
            strand[t] = (uint8_t)x.strand;
            qbeg[t] = x.qbeg;
            rbeg[t] = x.rbeg;
            slen[t] = x.slen;
            chain[t] = x.chain;
            first = x.rank == 0;
            if (t + 1 == n || src[t + 1].rank == 0) cnext[t - x.rank] = (int32_t)(t + 1);   // the chain's last seed
        }
        const unsigned long long m = __ballot(first);
        if (lane == 0 && m) atomicAdd(&nf, __popcll(m));
    }
    __syncthreads();
    if (threadIdx.x == 0 && nf) atomicAdd(n_first, nf);
}

static int grid_of(int64_t n, int cap = 8192) {
    int64_t g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

// PRGPU_ALN_LANE=1: every read on the lane kernels (the wave kernels off)
static bool aln_lane_only() {
    static const int v = getenv("PRGPU_ALN_LANE") ? atoi(getenv("PRGPU_ALN_LANE")) : 0;
    return v != 0;
}
int aln_launch_init(const AlnDev &A, void *stream) {
    const int64_t n = A.n_task > A.n_sr ? A.n_task : A.n_sr;
    hipLaunchKernelGGL(aln_init_kernel, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}
int aln_launch_heads(const AlnDev &A, void *stream) {
    if (A.n_sr <= 0) return 0;
    if (!aln_lane_only() && A.n_big == 0) return 0;   // hprev only feeds the lane walk
    const int64_t blocks = (A.n_sr + 3) / 4;   // a wave per read (grid-stride beyond 16 k workgroups)
    // PRGPU_HEADS_CAP (tests): a smaller LDS list, so that reads take the lane-0 path sooner
    const int cap_env = getenv("PRGPU_HEADS_CAP") ? atoi(getenv("PRGPU_HEADS_CAP")) : HEADS_CAP;
    const int cap = cap_env > 0 && cap_env < HEADS_CAP ? cap_env : HEADS_CAP;
    hipLaunchKernelGGL(aln_heads_kernel, dim3((unsigned)(blocks < 16384 ? blocks : 16384)), dim3(256), 0,
                       (hipStream_t)stream, A, cap);
    return (int)hipGetLastError();
}
int aln_launch_list(const AlnDev &A, void *stream) {
    if (A.n_task <= 0) return 0;
    hipLaunchKernelGGL(aln_list_kernel, dim3((unsigned)grid_of(A.n_task, 2048)), dim3(256), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
}
int aln_launch_walk(const AlnDev &A, void *stream) {
    if (A.n_sr <= 0) return 0;
    static const int wgcu = getenv("PRGPU_ALN_WALK_WG") ? atoi(getenv("PRGPU_ALN_WALK_WG")) : 0;
    const unsigned lds = wgcu > 0 ? (unsigned)(160 * 1024 / wgcu) & ~255u : 0u;
    const bool wave = !aln_lane_only();
    if (wave) {
        hipLaunchKernelGGL(aln_walk_wave_kernel, dim3((unsigned)((A.n_sr + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    if (wave && A.n_big == 0) return 0;
    hipLaunchKernelGGL(aln_walk_kernel, dim3((unsigned)((A.n_sr + 255) / 256)), dim3(256), lds, (hipStream_t)stream, A,
                       wave ? 1 : 0);
    return (int)hipGetLastError();
}
int aln_launch_final(const AlnDev &A, void *stream, const int32_t *early_snap, bool complement) {
    if (A.n_sr <= 0) return 0;
    // tuning hook: PRGPU_ALN_FINAL_WG=k caps the resident workgroups per CU at k (dynamic LDS),
    // i.e. the reads whose region scratch is live at once
    // (default 3: 17.5 -> 13.6 ms at configs[1]; the per-lane region scratch of all resident reads
    // then stays on chip instead of thrashing L2; profiles/r02_alnwg_sweep.txt)
    static const int wgcu = getenv("PRGPU_ALN_FINAL_WG") ? atoi(getenv("PRGPU_ALN_FINAL_WG")) : 3;
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n_cu <= 0)
            n_cu = 256;
    }
    const unsigned lds = wgcu > 0 ? (unsigned)(160 * 1024 / wgcu) & ~255u : 0u;
    // the dequeue counter: its own word for the early (side stream) and the late passes
    int32_t *next = A.counter + (early_snap ? (complement ? 10 : 8) : 9);
    hipError_t e = hipMemsetAsync(next, 0, 4, (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
    const int64_t chunks = (A.n_sr + 63) / 64;
    int64_t grid = (int64_t)n_cu * (wgcu > 0 ? wgcu : 8);
    if (grid > (chunks + 3) / 4) grid = (chunks + 3) / 4;
    if (grid < 1) grid = 1;
    const bool wave = !aln_lane_only();
    if (wave) {
        hipLaunchKernelGGL(aln_final_wave_kernel, dim3((unsigned)((A.n_sr + 127) / 128)), dim3(128), 0,
                           (hipStream_t)stream, A, early_snap, complement ? 1 : 0);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        if (A.n_big == 0) return 0;
    }
    hipLaunchKernelGGL(aln_final_kernel, dim3((unsigned)grid), dim3(256), lds, (hipStream_t)stream, A, early_snap, next,
                       complement ? 1 : 0, wave ? 1 : 0);
    return (int)hipGetLastError();
}
int aln_launch_patch(const AlnDev &A, int n_req, int32_t *pool, int64_t stride, void *stream) {
    if (n_req <= 0) return 0;
    if (aln_lane_only())
        hipLaunchKernelGGL(aln_patch_kernel, dim3((unsigned)((n_req + 63) / 64)), dim3(64), 0, (hipStream_t)stream, A,
                           n_req, pool, stride);
    else
        hipLaunchKernelGGL(aln_patch_wave_kernel, dim3((unsigned)((n_req + 3) / 4)), dim3(256), 0, (hipStream_t)stream, A,
                           n_req, pool, stride);
    return (int)hipGetLastError();
}

int sw_launch_gather(const SwGather &G, void *stream) {
    if (G.n <= 0) return 0;
    hipLaunchKernelGGL(sw_gather_kernel, dim3(grid_of(G.n)), dim3(256), 0, (hipStream_t)stream, G);
    return (int)hipGetLastError();
}

int aln_launch_unpack_seeds(const pr_seed_task *src, int64_t n, int32_t *sr, int32_t *lr, uint8_t *strand,
                            int32_t *qbeg, int32_t *rbeg, int32_t *slen, int32_t *chain, int32_t *n_first,
                            int32_t *cnext, void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(aln_unpack_kernel, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, src, n, sr, lr, strand,
                       qbeg, rbeg, slen, chain, n_first, cnext);
    return (int)hipGetLastError();
}

size_t aln_scan_temp_bytes(int64_t n) {
    size_t a = 0;
    (void)rocprim::exclusive_scan(nullptr, a, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0, (size_t)n + 1,
                                  rocprim::plus<int64_t>(), (hipStream_t)0);
    return a;
}
int aln_launch_cig_slots(const AlnDev &A, int64_t *slot, int64_t *tmp_in, void *temp, size_t temp_bytes,
                         void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(aln_slot_kernel, dim3(grid_of(A.n_task + 1)), dim3(256), 0, s, A, tmp_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    e = rocprim::exclusive_scan(temp, tb, tmp_in, slot, (int64_t)0, (size_t)A.n_task + 1, rocprim::plus<int64_t>(), s);
    return (int)e;
}
int aln_launch_compact(const AlnDev &A, int64_t *aoff, int64_t *tmp_in, int32_t *alist, int32_t *aflag, void *temp,
                       size_t temp_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(aln_nout64_kernel, dim3(grid_of(A.n_sr + 1)), dim3(256), 0, s, A.nout, (int64_t)A.n_sr, tmp_in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    if ((e = rocprim::exclusive_scan(temp, tb, tmp_in, aoff, (int64_t)0, (size_t)A.n_sr + 1, rocprim::plus<int64_t>(),
                                     s)) != hipSuccess)
        return (int)e;
    if (A.n_sr > 0)
        hipLaunchKernelGGL(aln_compact_kernel, dim3(grid_of(16 * (int64_t)A.n_sr)), dim3(256), 0, s, A, aoff, alist, aflag);
    return (int)hipGetLastError();
}

size_t aln_group_temp_bytes(int64_t n, int32_t n_lr) {
    size_t a = 0, b = 0;
    (void)rocprim::radix_sort_pairs(nullptr, a, (int32_t *)nullptr, (int32_t *)nullptr, (int32_t *)nullptr,
                                    (int32_t *)nullptr, (size_t)(n > 0 ? n : 1), 0, 32, (hipStream_t)0);
    (void)rocprim::exclusive_scan(nullptr, b, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0, (size_t)n_lr + 1,
                                  rocprim::plus<int64_t>(), (hipStream_t)0);
    return a > b ? a : b;
}
int aln_launch_group_lr(const int32_t *alist, const int32_t *t_lr, int64_t n, int32_t n_lr, int32_t *key0, int32_t *key1,
                        int32_t *out_list, int32_t *cnt, int64_t *lr_off, int64_t *tmp_in, void *temp,
                        size_t temp_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(cnt, 0, (size_t)(n_lr + 1) * 4, s);
    if (e != hipSuccess) return (int)e;
    if (n > 0) {
        hipLaunchKernelGGL(aln_key_kernel, dim3(grid_of(n)), dim3(256), 0, s, alist, t_lr, n, key0, cnt);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
        int bits = 1;
        while (bits < 31 && (1 << bits) < n_lr) ++bits;
        size_t tb = temp_bytes;   // LSD radix sort: stable, so a long read's alignments stay in read order
        if ((e = rocprim::radix_sort_pairs(temp, tb, key0, key1, alist, out_list, (size_t)n, 0, bits, s)) != hipSuccess)
            return (int)e;
    }
    hipLaunchKernelGGL(aln_cnt64_kernel, dim3(grid_of((int64_t)n_lr + 1)), dim3(256), 0, s, cnt, n_lr, tmp_in);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    return (int)rocprim::exclusive_scan(temp, tb, tmp_in, lr_off, (int64_t)0, (size_t)n_lr + 1, rocprim::plus<int64_t>(), s);
}

}  // namespace prgpu
