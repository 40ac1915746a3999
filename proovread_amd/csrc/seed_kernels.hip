// Seeding and chaining on the GPU: seed_core.h's map_read with one
// 64-lane wave per short read.  The index (text, 12-mer hit lists with the 28 bases
// after every hit, count tables) is resident in HBM.
//
// Pass 1 (seed_batch_kernel, persistent waves dequeue 64 reads at a time):
//   1. the 64 occurrence tables, one after the other, each wave-parallel (build_occ_wave)
//   2. SMEMs, re-seeding, -y seeds, chaining, chain filter, task output: seed_core.h's
//      map_after_occ, one lane per read (sequential, latency-bound decisions; 64 reads'
//      loads in flight per wave).  Scratch slices are sized for the batch's reads; a read
//      that outgrows its slice is flagged.
// Pass 2 (seed_wave_kernel, the flagged reads): one wave per read with the large slice,
// map_after_occ on lane 0.  A read that still outgrows it is reported with its SC_OVER_*
// flags and no tasks.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "seed_core.h"
#include "seed_dev.h"

namespace prgpu {

#ifndef SEED_WAVES_DEF   // (tuning builds: tools/probe/build_variant.sh)
#define SEED_WAVES_DEF 4
#endif
#ifndef SEED_LMAX_DEF
#define SEED_LMAX_DEF 1024
#endif
constexpr int SEED_WAVES = SEED_WAVES_DEF;   // waves (reads in flight) per workgroup
constexpr int SEED_LMAX = SEED_LMAX_DEF;     // LDS start offsets per wave: reads <= 1024 bases
#ifndef SEED_MINB
#define SEED_MINB 4
#endif
#ifndef SEED_WAVE_MINB   // the by-wave kernel's workgroups per CU (register budget)
#define SEED_WAVE_MINB SEED_MINB
#endif
#ifndef OCC_U
#define OCC_U 2   // hits per lane per pass of the occurrence table's hit loop
#endif

// the short j-mer count tables (j <= LC_MAX) into the workgroup's LDS: the SMEM search's
// occurrence counts of short extensions are dependent lookups, on chip instead of L2/MALL
__device__ void load_lcnt(const seedc::IndexView &V, uint32_t *lc) {
    for (int j = 1; j <= seedc::LC_MAX; ++j) {
        const int o = seedc::lc_off(j), n = 1 << (2 * j);
        for (int k = threadIdx.x; k < n; k += blockDim.x) lc[o + k] = V.cnt[j - 1][k];
    }
    __syncthreads();
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The occurrence table of read q (len bases) in S, wave-parallel (all 64 lanes): lanes over the
// read's starts compute the 12-mer code, the packed bases after it and the start's hit count; a
// wave scan gives the start offsets (also kept in LDS `ho` for the lookup below); lanes over the
// read's hits (consecutive hits -> coalesced kpos / kext loads) compute each hit's exact match
// length (LCP with the packed bases, then the text past them) and count it into the start's
// match-length histogram; a per-start suffix sum makes the count table.  This is
// build_occ's table without its diagonal shortcut (same match lengths).  -> 0 or SC_OVER_HITS.
// 16 bases from base x of a 4-bit packed sequence (a padding word after the last)
__device__ __forceinline__ uint64_t nib16(const uint64_t *w4, uint64_t x) {
    const uint64_t w = x >> 4;
    const int sh = (int)(x & 15) * 4;
    const uint64_t lo = w4[w];
    return sh ? (lo >> sh) | (w4[w + 1] << (64 - sh)) : lo;
}

template <int NW>   // the match-length walk's 16-base compares per text round trip (1 or 4)
__device__ int build_occ_wave(const seedc::IndexView &V, seedc::Scratch &S, const uint8_t *q, int len, int32_t *ho,
                              int lane, uint64_t *q4, const uint32_t *lc, int *n_hits = nullptr,
                              unsigned long long *ot = nullptr, bool lazy = false) {
    // ot (optional): wall-clock ticks of the start pass, the hit pass and the count table
    unsigned long long t_occ = ot ? wall_clock64() : 0ULL;
#define OCC_TICK(k)                                        \
    do {                                                   \
        if (ot) {                                          \
            const unsigned long long t_ = wall_clock64();  \
            ot[k] += t_ - t_occ;                           \
            t_occ = t_;                                    \
        }                                                  \
    } while (0)
    using seedc::HB;
    using seedc::KI;
    using seedc::KX;
    int err = 0;
    int run = 0;
    // the read 16 bases per word in LDS (past the read: 6, never a text code) for the start
    // pass's codes and the match lengths below (words up to (len >> 4) + 3: a start's 12-mer and
    // the KX bases after it, read 16 at a time)
    if (V.text4) {
        for (int w = lane; w <= (len >> 4) + 3; w += 64) {
            const int x0 = w * 16;
            uint8_t b[16];
            if (x0 + 16 <= len) {
                __builtin_memcpy(b, q + x0, 16);
            } else {
#pragma unroll
                for (int k = 0; k < 16; ++k) b[k] = x0 + k < len ? q[x0 + k] : (uint8_t)6;
            }
            uint64_t v = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t c = x0 + k < len ? (b[k] < 4 ? b[k] : 4u) : 6u;
                v |= (uint64_t)c << (4 * k);
            }
            q4[w] = v;
        }
        wave_sync_lds();
    }
    // per-start side tables for the hit pass in the LDS area beyond the start offsets (reads of
    // up to 170 bases: ho [L1] | code [L1] | qext [L1] u64 | koff of the code [L1] u64, L1 = len + 1
    // rounded up to even); longer reads read S.codes / S.qext / koff from HBM
    const int L1 = (len + 2) & ~1;
    const bool side = 6 * L1 <= SEED_LMAX + 4;
    int32_t *lcode = ho + L1;
    uint64_t *lqext = reinterpret_cast<uint64_t *>(ho + 2 * L1);
    uint64_t *lr0 = reinterpret_cast<uint64_t *>(ho + 4 * L1);
    for (int a0 = 0; a0 <= len; a0 += 64) {
        const int a = a0 + lane;
        int ca = 0;
        uint64_t r0a = 0;
        if (a <= len) {
            int32_t code_a = -1;
            uint64_t qe = 0;
            if (a + KI <= len) {
                uint32_t code = 0;
                bool ok = true;
                const int n = len - a - KI;
                if (V.text4) {   // from the read's packed copy in LDS (4 bits a base, 6 past its end)
                    const uint64_t w0 = nib16(q4, (uint64_t)a), w1 = nib16(q4, (uint64_t)a + 16),
                                   w2 = nib16(q4, (uint64_t)a + 32);
#pragma unroll
                    for (int x = 0; x < KI; ++x) {
                        const uint32_t c = (uint32_t)(w0 >> (4 * x)) & 15u;
                        ok &= c < 4;
                        code = (code << 2) | (c & 3u);
                    }
                    // pack_ext of the KX bases after the 12-mer: 2 bits each up to the first N
                    const int nmax = n < KX ? n : KX;
                    uint64_t v = 0;
                    int k = 0;
#pragma unroll
                    for (int x = 0; x < KX; ++x) {
                        const int b = KI + x;   // base a + b: word b >> 4, nibble b & 15
                        const uint64_t wb = b < 16 ? w0 : b < 32 ? w1 : w2;
                        const uint32_t c = (uint32_t)(wb >> (4 * (b & 15))) & 15u;
                        const bool go = k == x && x < nmax && c < 4;
                        v |= go ? (uint64_t)c << (2 * x) : 0ull;
                        k += go ? 1 : 0;
                    }
                    qe = v | ((uint64_t)k << 56);
                } else {
                    for (int x = 0; x < KI; ++x) {
                        const uint8_t c = q[a + x];
                        ok &= c < 4;
                        code = (code << 2) | (c & 3u);
                    }
                    qe = seedc::pack_ext(q + a + KI, n < KX ? n : KX);
                }
                if (ok) {
                    code_a = (int32_t)code;
                    if (!lazy) {
                        r0a = V.koff[code];
                        ca = (int)(V.koff[code + 1] - r0a);
                    }
                }
            }
            S.codes[a] = code_a;
            S.qext[a] = qe;
            if (lazy) {   // the lazy table: no start ready, the hits come on first use (seed_core.h materialize)
                S.ready[a] = a == len ? 1 : 0;
                S.hoff[a] = 0;
                S.hend[a] = 0;
                ca = 0;
            }
            if (side) {   // the hit pass's per-start inputs on chip
                lcode[a] = code_a;
                lqext[a] = qe;
                lr0[a] = r0a;
            }
        }
        int x = ca;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        const int ex = run + x - ca;
        if (a <= len) {
            ho[a] = ex;
            S.hoff[a] = ex;
        }
        run += __shfl(x, 63, 64);
    }
    if (lazy) {   // the read's 4-bit copy for materialize's text walks, an empty pool
        if (S.q4w) {
            if (V.text4) {
                for (int w = lane; w <= (len >> 4) + 3; w += 64) S.q4w[w] = q4[w];
            } else {
                for (int w = lane; w <= (len >> 4) + 3; w += 64) {
                    uint64_t v = 0;
                    for (int k = 0; k < 16; ++k) {
                        const int x = w * 16 + k;
                        const uint64_t c = x < len ? (q[x] < 4 ? q[x] : 4u) : 6u;
                        v |= c << (4 * k);
                    }
                    S.q4w[w] = v;
                }
            }
        }
        if (lane == 0) S.lz[0] = S.lz[1] = S.lz[2] = 0;
        if (n_hits) *n_hits = 0;
        __threadfence_block();
        wave_sync_lds();
        OCC_TICK(0);
        return 0;
    }
    const int nh = run;
    if (n_hits) *n_hits = nh;
    if (nh > S.cap_hits) err = seedc::SC_OVER_HITS;
    wave_sync_lds();
    __threadfence_block();
    OCC_TICK(0);
    if (!err) {
        const int amax = len - KI;   // last start with a 12-mer
        // OCC_U hits per lane per pass, their dependent load chains (start lookup -> code ->
        // k-mer list -> position -> contig -> coordinates) interleaved: one chain's latency per
        // OCC_U hits instead of per hit
        constexpr int U = OCC_U;
        // the start of a pass's first hit (wave-uniform, non-decreasing): each lane walks from it
        // to the last start whose hits begin at or before its hit (a few steps over the LDS start
        // offsets instead of a binary search over all of them)
        int apos = 0;
        for (int k0 = lane; k0 < nh; k0 += 64 * U) {
            int aa[U];
            bool ok[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + 64 * u;
                ok[u] = k < nh;
                int a = apos;
                if (ok[u])
                    while (a < amax && ho[a + 1] <= k) ++a;
                aa[u] = a;
            }
            apos = __shfl(aa[U - 1], 63, 64);   // (the pass's last hit, or a start before nh's)
            uint32_t code[U];
            uint64_t qe[U], r[U], p[U], exb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int a = aa[u], k = k0 + 64 * u;
                if (side) {
                    code[u] = ok[u] ? (uint32_t)lcode[a] : 0u;
                    qe[u] = ok[u] ? lqext[a] : 0ull;
                    r[u] = ok[u] ? lr0[a] + (uint64_t)(k - ho[a]) : 0ull;
                } else {
                    code[u] = ok[u] ? (uint32_t)S.codes[a] : 0u;
                    qe[u] = ok[u] ? S.qext[a] : 0ull;
                    r[u] = V.koff[code[u]] + (uint64_t)(k - ho[a]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                p[u] = ok[u] ? seedc::hit_pos(V, code[u], r[u]) : 0ull;
                exb[u] = ok[u] ? V.kext[r[u]] : 0ull;
            }
            // the contigs (seed_core.h contig_of) and bwa coordinates (pack_fr): from the block
            // table when the hit's block has at most two contig starts after its first contig,
            // else the cblk -> cstart walk; interleaved over the pass's hits
            int c[U];
            int64_t dlt[U];
            bool walk[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                walk[u] = true;
                if (V.blkfr && ok[u]) {
                    const seedc::BlkFr bt = V.blkfr[p[u] >> seedc::CB_SHIFT];
                    const int o = (int)(p[u] & ((1u << seedc::CB_SHIFT) - 1u));
                    if (o < bt.bnd) { c[u] = bt.c0; dlt[u] = bt.d0; walk[u] = false; }
                    else if (o < bt.bnd2) { c[u] = bt.c0 + 1; dlt[u] = bt.d1; walk[u] = false; }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!walk[u]) continue;
                int cc = V.cblk[p[u] >> seedc::CB_SHIFT];
                int64_t nx = cc + 1 < V.n_contig ? V.cstart[cc + 1] : INT64_MAX;
                while (nx <= (int64_t)p[u]) {
                    ++cc;
                    nx = cc + 1 < V.n_contig ? V.cstart[cc + 1] : INT64_MAX;
                }
                c[u] = cc;
                const int64_t cst = V.cstart[cc];
                const int64_t lro = cc < V.n_lr ? V.lr_off[cc] : V.lr_off[2 * V.n_lr - cc];
                dlt[u] = cc < V.n_lr ? lro - cst : 2 * V.l_pac - lro - cst;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!ok[u]) continue;
                const int k = k0 + 64 * u, a = aa[u];
                const int le = (int)(exb[u] >> 56), lq = (int)(qe[u] >> 56);
                const uint64_t xd = (exb[u] ^ qe[u]) & seedc::KX_MASK;
                int m = xd ? seedc::ctz64(xd) >> 1 : KX;
                m = m < le ? m : le;
                m = m < lq ? m : lq;
                int ml = KI + m;
                if (m == KX) {
                    if (V.text4) {   // 16 bases at a time: the first differing nibble, or a read N, or the read's end
                        // the text words of up to 64 bases are loaded together (5 independent loads, the
                        // text has 8 padding words) and compared from registers: one memory round trip
                        // per 64 bases instead of one per 16 (the finish task's near-exact reads walk ~110)
                        bool go = a + ml < len;
                        // (NW compares per round trip: 1 for dense indexes' by-wave pass, where the
                        // 5-word buffers cost occupancy, V.walk_nw)
                        constexpr int nw = NW;
                        while (go) {
                            const uint64_t tp = p[u] + (uint64_t)ml;
                            const uint64_t* tw4 = V.text4 + (tp >> 4);
                            const int sh = (int)(tp & 15) * 4;
                            uint64_t w5[5];
#pragma unroll
                            for (int j = 0; j < 5; ++j) w5[j] = j <= nw ? tw4[j] : 0ull;
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                if (!go || j >= nw) break;
                                const int x = a + ml;
                                const uint64_t tw = sh ? (w5[j] >> sh) | (w5[j + 1] << (64 - sh)) : w5[j];
                                const uint64_t qw = nib16(q4, (uint64_t)x);
                                const uint64_t nq = (qw >> 2) & 0x1111111111111111ull;   // read N (code 4) or past the end (6)
                                const uint64_t bad = (qw ^ tw) | (nq * 0xFull);
                                const int lim = len - x;
                                if (bad) {
                                    const int f = __builtin_ctzll(bad) >> 2;
                                    ml += f < lim ? f : lim;
                                    go = false;
                                } else if (lim <= 16) {
                                    ml += lim;
                                    go = false;
                                } else {
                                    ml += 16;
                                }
                            }
                        }
                    } else {
                        while (a + ml < len && q[a + ml] < 4 && V.text[p[u] + ml] == q[a + ml]) ++ml;
                    }
                }
                seedc::set_hpos(S, k, p[u]);
                // pack_fr: the hit's forward-reverse coordinate and long read (text_to_fr: fr =
                // lr_off[c] + (p - cstart[c]) forward, l_pac + (l_pac - lr_off[rid + 1]) +
                // (p - cstart[c]) reverse, both p + dlt)
                const int64_t fr = (int64_t)p[u] + dlt[u];
                const int rid = c[u] < V.n_lr ? c[u] : 2 * V.n_lr - 1 - c[u];   // (reverse half: reads in reverse order)
                S.hfr[k] = ((uint64_t)fr << seedc::FR_RID_BITS) | (uint64_t)rid;
                S.hml[k] = (uint16_t)(ml < 65535 ? ml : 65535);
            }
        }
        __threadfence_block();
        wave_sync_lds();
        OCC_TICK(1);
        // the count table, a lane per start: ge[a][t] = #{hits of a with ml - KI >= t} summed
        // directly in registers (no zeroing, no atomics, no suffix pass over HBM)
        // and R_1 .. R_RK(a), the ends of the start's longest matches with >= k occurrences
        // (seed_core.h fill_rk: smem1's backward extension sweeps them), from the same hits, or
        // below 12 bases from the j-mer counts
        const seedc::Occ occ{&V, &S, q, len, lc};
        for (int a = lane; a < len; a += 64) {
            uint32_t g[HB];
            uint16_t top[seedc::RK];   // (fill_rk's top list, from the same pass over the hits)
#pragma unroll
            for (int t = 0; t < HB; ++t) g[t] = 0u;
#pragma unroll
            for (int k = 0; k < seedc::RK; ++k) top[k] = 0;
            const bool has = a + KI <= len && S.codes[a] >= 0;
            const bool ranked = has && q[a] < 4;
            if (has) {
                // the match lengths 4 at a time (one 8-byte load; the slice's hml array has room past
                // its last hit): the count row and the top list in one pass
                const int h0 = ho[a], h1 = ho[a + 1];
                for (int h = h0; h < h1; h += 4) {
                    uint64_t w4;
                    __builtin_memcpy(&w4, S.hml + h, 8);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (h + j >= h1) break;
                        const uint16_t ml = (uint16_t)(w4 >> (16 * j));
                        const int d = (int)ml - KI;
#pragma unroll
                        for (int t = 0; t < HB; ++t) g[t] += d >= t ? 1u : 0u;
                        if (ranked) seedc::topk_insert(top, ml);
                    }
                }
            }
            uint32_t *dst = S.ge + (int64_t)a * HB;
#pragma unroll
            for (int t = 0; t < HB; ++t) dst[t] = g[t];
            seedc::fill_rk_top(occ, S, q, len, a, top);
        }
        __threadfence_block();
    }
    wave_sync_lds();
    OCC_TICK(2);
#undef OCC_TICK
    return err;
}

// mem_chain of one read by the whole wave (pass 2's reads: their thousands of occurrences chained
// on one lane were pass 2's wall time).  Chains of different (long read, strand) ranges never
// interact (seed_core.h chain_seq), so the ranges are dealt to lanes by a hash of their key and
// every lane chains its ranges' occurrences in the sequential order.  A seed's slot, and a new
// chain's, is the occurrence's place in that order: creation order -- the chain sort's last
// tie-break -- is the sequential one and no slot counter is shared.  -> the number of chains,
// compacted into S.cv[0, n) in creation order; -1 when the occurrences do not fit the slice
// (the caller then chains on one lane); -2 when the chains or ranges exceed cap_chains (the
// sequential chaining's SC_OVER_CHAINS).  lds: 129 ints of the wave's LDS.
__device__ int chain_wave(const seedc::IndexView &I, const pr_seed_opts &O, seedc::Scratch &S, int nm, int lane,
                          int32_t *lds) {
    using namespace seedc;
    // 1. the selected occurrences in chaining order (chain_seq's selection) over the lanes: (hit, SMEM)
    int2 *ol = reinterpret_cast<int2 *>(S.ge);   // (the count table is dead after the SMEMs)
    const int cap_ge = (int)((int64_t)S.lmax * HB * 4 / 12);   // 8 bytes an entry + a 4-byte list index
    // chain slots run on into S.ch and S.cnx into S.kept (carve: cv|ch and cnx|kept adjacent,
    // both dead until the filter); more than cap_chains chains or ranges -> -2 (SC_OVER_CHAINS,
    // as the sequential chaining flags them)
    const int cap2 = 2 * S.cap_chains;
    const int cap = cap_ge < S.cap_seeds ? (cap_ge < cap2 ? cap_ge : cap2) : (S.cap_seeds < cap2 ? S.cap_seeds : cap2);
    // (the 64 hits of a step filtered by match length, then every step-th of them up to max_occ:
    // ranks from ballots keep the sequential order)
    const unsigned long long below = (1ull << lane) - 1ull;
    int n = 0;
    wave_sync_lds();   // (lane 0's SMEMs)
    for (int mi = 0; mi < nm && n >= 0; ++mi) {
        const Iv p = S.mems[mi];
        const int slen = p.end - p.start;
        const int32_t h0 = S.hoff[p.start], h1 = S.hoff[p.start + 1];
        const int step = p.occ > O.max_occ ? (int)(p.occ / O.max_occ) : 1;
        int fbase = 0, count = 0;
        for (int32_t kb = h0; kb < h1 && count < O.max_occ; kb += 64) {
            const int32_t k = kb + lane;
            const bool qual = k < h1 && S.hml[k] >= slen;   // text-position order: the 12-mer lists are sorted
            const unsigned long long qm = __ballot(qual);
            const int f = fbase + __popcll(qm & below);
            const bool use = qual && f % step == 0 && f / step < O.max_occ;
            const unsigned long long um = __ballot(use);
            const int nu = __popcll(um);
            if (n + nu > cap) {
                n = -1;
                break;
            }
            if (use) ol[n + __popcll(um & below)] = make_int2(k, mi);
            n += nu;
            count += nu;
            fbase += __popcll(qm);
        }
    }
    if (n < 0) return -1;
    int32_t *idx = reinterpret_cast<int32_t *>(ol + n);   // the lanes' lists of occurrence indices
    int32_t *cnt = lds, *cur = lds + 64;                 // per-lane counts / cursors (LDS)
    cnt[lane] = 0;
    for (int e = lane; e < n; e += 64) S.cv[e].n = 0;   // (chain slots: n > 0 marks a chain)
    for (int k = lane; k < S.hsize; k += 64) S.htab[k].key = -1;
    if (lane == 0) lds[128] = 0;                          // ranges so far
    __threadfence_block();
    wave_sync_lds();
    auto owner_of = [&](int e) -> int {
        const uint64_t v = S.hfr[ol[e].x];
        const int rid = (int)(v & ((1u << FR_RID_BITS) - 1u));
        const int key = rid * 2 + ((int64_t)(v >> FR_RID_BITS) >= I.l_pac ? 1 : 0);
        return (int)(((uint32_t)key * 0x9E3779B1u) >> 26);
    };
    // 2. every lane's share, 64 occurrences at a time: same-owner lanes by 6 ballots, ranks in
    // occurrence order; counts, then the stable scatter into the lanes' lists
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {   // list starts: exclusive prefix of the counts over lanes
            int x = cnt[lane];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const int y = __shfl_up(x, d, 64);
                if (lane >= d) x += y;
            }
            cur[lane] = x - cnt[lane];
            wave_sync_lds();
        }
        for (int e0 = 0; e0 < n; e0 += 64) {
            const int e = e0 + lane;
            const int own = e < n ? owner_of(e) : 64;
            unsigned long long m = __ballot(e < n);
#pragma unroll
            for (int b = 0; b < 7; ++b) {
                const bool bit = (own >> b) & 1;
                const unsigned long long w = __ballot(bit);
                m &= bit ? w : ~w;
            }
            const int rank = __popcll(m & below);
            const bool leader = e < n && rank == 0;
            if (pass == 0) {
                if (leader) atomicAdd(&cnt[own], __popcll(m));
            } else {
                if (e < n) idx[cur[own] + rank] = e;
                wave_sync_lds();
                if (leader) cur[own] += __popcll(m);
            }
            wave_sync_lds();
        }
        wave_sync_lds();
    }
    __threadfence_block();
    wave_sync_lds();
    // 3. each lane chains its occurrences in order (chain_seq's decisions; slots = occurrence index)
    const int mine = cnt[lane], first = cur[lane] - mine;
    for (int t = 0; t < mine; ++t) {
        const int e = idx[first + t];
        const int2 oe = ol[e];
        const Iv p = S.mems[oe.y];
        const uint64_t v = S.hfr[oe.x];
        Seed sd;
        sd.rbeg = (int64_t)(v >> FR_RID_BITS);
        sd.qbeg = (int16_t)p.start;
        sd.len = (int16_t)(p.end - p.start);
        sd.nx = -1;
        const int rid = (int)(v & ((1u << FR_RID_BITS) - 1u));
        const int32_t key = rid * 2 + (sd.rbeg >= I.l_pac ? 1 : 0);
        // the range: probe, claiming a free entry with a CAS (other lanes' keys may share a probe run)
        uint32_t h = ((uint32_t)key * 0x9E3779B1u) & (uint32_t)(S.hsize - 1);
        bool found = false;
        for (;;) {
            const int32_t kk = S.htab[h].key;
            if (kk == key) { found = true; break; }
            if (kk == -1) {
                const int32_t old = atomicCAS(&S.htab[h].key, -1, key);
                if (old == -1) break;   // claimed: a new range
                if (old == key) { found = true; break; }
            }
            h = (h + 1) & (uint32_t)(S.hsize - 1);
        }
        int at = -1;
        bool at_tail = false;
        int32_t ns = e;
        if (found && S.htab[h].r < 0) continue;   // (a range beyond cap_chains: the read is flagged)
        if (found) {
            RangeRec &R = S.rg[S.htab[h].r];
            if (R.tpos <= sd.rbeg) {
                at = R.tail;
                at_tail = true;
            } else {
                for (int x = R.head; x >= 0 && S.cv[x].pos <= sd.rbeg; x = S.cnx[x]) at = x;
            }
            if (at >= 0) {
                const int r = at_tail ? merge_tail(O, I.l_pac, S, ns, R, sd)
                                      : test_and_merge(O, I.l_pac, S, ns, S.cv[at], sd, rid);
                if (r) continue;   // merged or contained (slots < the capacities: r >= 0)
            }
        }
        S.seeds[e] = sd;
        Chain c;
        c.pos = sd.rbeg;
        c.rid = rid;
        c.head = c.tail = e;
        c.n = 1;
        c.w = c.kept = 0;
        c.first = -1;
        S.cv[e] = c;
        if (!found) {
            const int r = atomicAdd(&lds[128], 1);
            if (r >= S.cap_chains) {
                S.htab[h].r = -1;
                continue;
            }
            RangeRec &R = S.rg[r];
            R.head = R.tail = e;
            R.n = 1;
            R.l_idx = e;
            R.tpos = sd.rbeg;
            R.f_rbeg = R.l_rbeg = sd.rbeg;
            R.f_ql = R.l_ql = pack_ql(sd);
            S.htab[h].r = r;
            S.cnx[e] = -1;
        } else {
            RangeRec &R = S.rg[S.htab[h].r];
            if (at < 0) {
                S.cnx[e] = R.head;
                R.head = e;
            } else {
                const int nx = S.cnx[at];
                S.cnx[e] = nx;
                S.cnx[at] = e;
                if (nx < 0) {
                    flush_tail(S, R);
                    R.tail = e;
                    R.n = 1;
                    R.l_idx = e;
                    R.tpos = sd.rbeg;
                    R.f_rbeg = R.l_rbeg = sd.rbeg;
                    R.f_ql = R.l_ql = pack_ql(sd);
                }
            }
        }
    }
    __threadfence_block();
    wave_sync_lds();
    const int nrg = lds[128];
    if (nrg > S.cap_chains) return -2;
    for (int r = lane; r < nrg; r += 64) flush_tail(S, S.rg[r]);
    __threadfence_block();
    wave_sync_lds();
    // 4. the chains in creation order (slot order), compacted 64 slots a step (a chunk's chains
    // are all loaded before any is stored: destinations are at or below their sources)
    int ncv = 0;
    for (int e0 = 0; e0 < n; e0 += 64) {
        const int e = e0 + lane;
        Chain c{};
        if (e < n) c = S.cv[e];
        const bool live = e < n && c.n > 0;
        const unsigned long long lm = __ballot(live);
        wave_sync_lds();
        if (live) S.cv[ncv + __popcll(lm & below)] = c;
        ncv += __popcll(lm);
        __threadfence_block();
        wave_sync_lds();
    }
    return ncv > S.cap_chains ? -2 : ncv;
}

// mem_chain_flt (seed_core.h chain_flt) of one read by the whole wave: pass 2's reads carry up to
// 2,048 chains, and the sequential filter's kept-list scan (every chain against every kept one,
// three dependent loads a test) was ~90 ms per read at configs[3].  The weights a chain per lane;
// the stable sort as ranks (the keys (weight desc, pos, head) are distinct, so every chain's
// place is the number of smaller keys: the same order as the insertion sort); the kept scan in
// sorted order with the kept list dealt over the lanes, 64 entries a step, ended at the first
// entry that drops the chain (a ballot: the lowest lane is the sequential loop's break).  S.ge
// (dead after the chaining) holds the keys, then the chains' query intervals, the kept list and
// its `first` marks.  -> false when they do not fit (the caller filters on lane 0).
__device__ bool chain_flt_wave(const pr_seed_opts &O, seedc::Scratch &S, int ncv, int lane, int *n_chains) {
    using namespace seedc;
    const int64_t ge_bytes = (int64_t)S.lmax * HB * 4;
    if ((int64_t)ncv * 36 > ge_bytes) return false;
    struct Key { int32_t nw, head; int64_t pos; };   // nw = -weight (INT32_MAX: filtered out)
    Key *key = reinterpret_cast<Key *>(S.ge);
    for (int j = lane; j < ncv; j += 64) {
        Chain &c = S.cv[j];
        const int w = chain_weight(S, c);
        c.w = w;
        key[j] = Key{w >= O.min_chain_weight ? -w : INT32_MAX, c.head, c.pos};
    }
    __threadfence_block();
    wave_sync_lds();
    int nch = 0;
    for (int ib = 0; ib < ncv; ib += 64) {
        const int i = ib + lane;
        const Key ki = i < ncv ? key[i] : Key{INT32_MAX, 0, 0};
        const bool pass = ki.nw != INT32_MAX;
        nch += __popcll(__ballot(pass));
        int rank = 0;
        for (int jb = 0; jb < ncv; jb += 64) {   // 64 keys a step, one coalesced load, read out by lane
            // (a padding key -- INT32_MAX weight -- is never below a key that passes)
            const Key kj = jb + lane < ncv ? key[jb + lane] : Key{INT32_MAX, 0, 0};
            const int plo = (int)(uint32_t)kj.pos, phi = (int)(kj.pos >> 32);
#pragma unroll
            for (int t = 0; t < 64; ++t) {
                const int nw = __builtin_amdgcn_readlane(kj.nw, t), hd = __builtin_amdgcn_readlane(kj.head, t);
                const int64_t ps = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane(phi, t) << 32) |
                                             (uint32_t)__builtin_amdgcn_readlane(plo, t));
                rank += (nw < ki.nw || (nw == ki.nw && (ps < ki.pos || (ps == ki.pos && hd < ki.head)))) ? 1 : 0;
            }
        }
        if (pass) S.ch[rank] = S.cv[i];
    }
    __threadfence_block();
    wave_sync_lds();
    // the sorted chains' query intervals and weights; the kept list's (KV) and its first marks (F)
    int4 *iv = reinterpret_cast<int4 *>(S.ge);
    int4 *kv = iv + nch;
    int32_t *fm = reinterpret_cast<int32_t *>(kv + nch);
    for (int i = lane; i < nch; i += 64) {
        const Chain &c = S.ch[i];
        const Seed &h = S.seeds[c.head], &t = S.seeds[c.tail];
        iv[i] = make_int4(h.qbeg, t.qbeg + t.len, c.w, 0);
        fm[i] = -1;
    }
    __threadfence_block();
    wave_sync_lds();
    if (nch > 0) {
        int nk = 1;
        if (lane == 0) {
            kv[0] = iv[0];
            S.ch[0].kept = 3;
        }
        __threadfence_block();
        wave_sync_lds();
        for (int i = 1; i < nch; ++i) {
            const int4 ci = iv[i];
            const int bi = ci.x, ei = ci.y;
            bool large = false, drop = false;
            for (int kb = 0; kb < nk && !drop; kb += 64) {
                const int k = kb + lane;
                bool ov = false, br = false;
                if (k < nk) {
                    const int4 cj = kv[k];
                    const int bj = cj.x, ej = cj.y;
                    const int bmax = bj > bi ? bj : bi;
                    const int emin = ej < ei ? ej : ei;
                    if (emin > bmax) {
                        const int li = ei - bi, lj = ej - bj;
                        const int minl = li < lj ? li : lj;
                        if (emin - bmax >= minl * O.mask_level && minl < O.max_chain_gap) {
                            ov = true;
                            br = ci.z < cj.z * O.drop_ratio && cj.z - ci.z >= O.min_seed_len << 1;
                        }
                    }
                }
                const unsigned long long bm = __ballot(br);
                const int last = bm ? __ffsll((long long)bm) - 1 : 63;   // the lanes the sequential loop visits
                if (ov && lane <= last && fm[k] < 0) fm[k] = i;
                large = large || __ballot(ov && lane <= last) != 0ull;
                drop = bm != 0ull;
            }
            if (!drop) {
                if (lane == 0) {
                    kv[nk] = ci;
                    S.ch[i].kept = large ? 2 : 3;
                }
                ++nk;
                __threadfence_block();
                wave_sync_lds();
            }
        }
        __threadfence_block();
        wave_sync_lds();
        for (int k = lane; k < nk; k += 64)
            if (fm[k] >= 0) S.ch[fm[k]].kept = 1;
    }
    __threadfence_block();
    wave_sync_lds();
    *n_chains = nch;
    return true;
}

// Pass 2: one wave per read with the large scratch slice (the reads of D.rlist: those that
// outgrew pass 1's slices), the sequential part on lane 0.
template <int NW>
__global__ void __launch_bounds__(64 * SEED_WAVES, SEED_WAVE_MINB) seed_wave_kernel(SeedDev D) {
    __shared__ __attribute__((aligned(16))) int32_t hoff_lds[SEED_WAVES][SEED_LMAX + 4];
    __shared__ uint64_t q4_lds[SEED_WAVES][SEED_LMAX / 16 + 4];
    __shared__ uint32_t lcnt[seedc::LC_N];
    load_lcnt(D.V, lcnt);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t slot = (int64_t)blockIdx.x * SEED_WAVES + wv;
    if (slot >= D.n_lanes) return;
    seedc::Scratch S = seedc::carve(D.scratch + slot * D.stride, D.caps);
    int32_t *ho = hoff_lds[wv];
    unsigned long long pt[4] = {0ULL, 0ULL, 0ULL, 0ULL};   // lane 0: phase ticks of this wave
    unsigned long long pl[6] = {0ULL, 0ULL, 0ULL, 0ULL, 0ULL, 0ULL};   // lane 0: seed_core.h's parts
    for (;;) {
        int j = 0;
        if (lane == 0) j = atomicAdd(D.next, 1);
        j = __shfl(j, 0, 64);
        if (j >= D.n_list) {   // every wave reaches this: the grid drains
            if (D.prof && lane == 0) {
                pt[1] += pl[0] + pl[1] + pl[2];
                pt[2] += pl[3] + pl[4];
                pt[3] += pl[5];
                for (int k = 0; k < 4; ++k) atomicAdd(&D.prof[k], pt[k]);
            }
            break;
        }
        const int i = D.rlist ? D.rlist[j] : j;
        const int64_t o = D.sr_off[i];
        const int len = (int)(D.sr_off[i + 1] - o);
        const uint8_t *q = D.sr_seq + o;
        int err = 0;
        const unsigned long long t0 = D.prof && lane == 0 ? wall_clock64() : 0ULL;
        if (len > S.lmax || len > SEED_LMAX - 1) err = seedc::SC_OVER_LEN;
        if (len > 0 && !err) err = build_occ_wave<NW>(D.V, S, q, len, ho, lane, q4_lds[wv], lcnt);
        // SMEMs and chaining on lane 0; then, for reads where bwa runs mem_flt_chained_seeds
        // (>= 440 bp), the seeds' local SW scores over all 64 lanes (a seed per lane, the rows
        // int16 and lane-interleaved in the dead count table); the output on lane 0
        int nch = 0, nlist = -1, nm = 0;
        unsigned long long tm = 0ULL;   // (lane 0, profiling: the read's phase boundaries)
        if (lane == 0) {
            if (D.prof) {
                tm = wall_clock64();
                pt[0] += tm - t0;
                atomicMax(&D.prof[17], tm - t0);
            }
            if (len > 0 && !err) {
                const seedc::Occ occ{&D.V, &S, q, len, lcnt};
                nm = seedc::collect_intv(occ, S, D.O, q, len, err, D.prof ? pl : nullptr);
            }
            if (D.prof) atomicMax(&D.prof[18], wall_clock64() - tm);
        }
        err = __shfl(err, 0, 64);
        nm = __shfl(nm, 0, 64);
        if (len > 0 && !err) {
            // chaining over the wave's lanes (by range), on lane 0 when the occurrences do not fit
            const unsigned long long tc = D.prof && lane == 0 ? wall_clock64() : 0ULL;
            __threadfence_block();
            int ncv = chain_wave(D.V, D.O, S, nm, lane, ho);
            unsigned long long tf = D.prof && lane == 0 ? wall_clock64() : 0ULL;
            if (lane == 0 && D.prof) atomicAdd(&D.prof[14 + (ncv == -1 ? 1 : 0)], tf - tc);
            if (ncv == -2) {
                ncv = 0;
                err = seedc::SC_OVER_CHAINS;
            }
            if (lane == 0 && ncv == -1) {
                ncv = 0;
                err = seedc::chain_seq(D.V, D.O, S, nm, &ncv);
                if (D.prof) {
                    const unsigned long long t_ = wall_clock64();
                    atomicAdd(&D.prof[13], 1ULL);
                    atomicAdd(&D.prof[15], t_ - tf);
                    tf = t_;
                }
            }
            err = __shfl(err, 0, 64);
            ncv = __shfl(ncv, 0, 64);
            __threadfence_block();
            wave_sync_lds();
            bool flt = err != 0 || chain_flt_wave(D.O, S, ncv, lane, &nch);
            if (lane == 0) {
                if (!flt) seedc::chain_flt(D.O, S, ncv, &nch);
                if (D.prof) {
                    const unsigned long long t_ = wall_clock64();
                    pl[3] += t_ - tc;
                    atomicAdd(&D.prof[16], t_ - tf);
                }
                if (!err && seedc::seed_flt_min_score(D.O, len) >= 0 && 3 * S.cap_seeds <= 2 * S.cap_hits &&
                    2 * 201 * 64 * 2 <= 4 * S.lmax * seedc::HB)
                    nlist = seedc::flt_seed_list(S, nch, (int32_t *)S.hfr + S.cap_seeds, S.cap_seeds);
            }
        }
        err = __shfl(err, 0, 64);
        nlist = __shfl(nlist, 0, 64);
        if (nlist > 0) {
            __threadfence_block();
            const int32_t *list = (const int32_t *)S.hfr + S.cap_seeds;   // (the dead hit coordinates)
            int32_t *rid = (int32_t *)S.hfr + 2 * S.cap_seeds;
            if (lane == 0) {   // each listed seed's long read (its chain's)
                int x = 0;
                for (int ci = 0; ci < nch; ++ci) {
                    const seedc::Chain &c = S.ch[ci];
                    if (c.kept == 0) continue;
                    for (int32_t k = c.head; k >= 0; k = S.seeds[k].nx) rid[x++] = c.rid;
                }
            }
            __threadfence_block();
            int32_t *scores = (int32_t *)S.hfr;
            int16_t *H = (int16_t *)S.ge + lane, *E = H + 201 * 64;
            for (int x = lane; x < nlist; x += 64) {
                const int32_t k = list[x];
                scores[k] = seedc::seed_sw_score(D.V, D.O, q, len, S.seeds[k], rid[x], H, E, 64);
            }
            __threadfence_block();
        }
        if (lane == 0) {
            int n = 0;
            if (len > 0 && !err)
                err = seedc::map_output(D.V, D.O, S, q, len, i, nch, D.out + (int64_t)(i - D.out0) * D.caps.out,
                                        D.caps.out, &n, nlist >= 0 ? (const int32_t *)S.hfr : nullptr,
                                        D.prof ? pl : nullptr);
            D.n_out[i] = err ? 0 : n;
            D.status[i] = err;
            if (D.prof) atomicMax(&D.prof[19], wall_clock64() - t0);   // the slowest read
        }
        __threadfence_block();
    }
}

// Pass 1: a wave takes 64 reads at a time; their occurrence tables are built one after the
// other by the whole wave (build_occ_wave), then every lane runs its own read's SMEMs,
// chaining and chain filter (seed_core.h map_after_occ) -- the sequential, latency-bound part
// with 64 reads' loads in flight per wave instead of one.  Scratch: 64 small slices per wave
// (D.caps sized for the batch's read lengths); a read that outgrows its slice is flagged and
// goes to pass 2.
template <bool LZ>   // LZ: the lazy occurrence table (D.caps.lazy), a separate kernel so the eager one carries none of it
__global__ void __launch_bounds__(64 * SEED_WAVES, SEED_MINB) seed_batch_kernel(SeedDev D) {
    __shared__ __attribute__((aligned(16))) int32_t hoff_lds[SEED_WAVES][SEED_LMAX + 4];
    __shared__ uint64_t q4_lds[SEED_WAVES][SEED_LMAX / 16 + 4];
    __shared__ uint32_t lcnt[seedc::LC_N];
    load_lcnt(D.V, lcnt);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t slot = (int64_t)blockIdx.x * SEED_WAVES + wv;
    if (slot >= D.n_lanes) return;
    uint8_t *base = D.scratch + slot * 64 * D.stride;
    int32_t *ho = hoff_lds[wv];
    unsigned long long pt[2] = {0ULL, 0ULL};   // wave wall-clock: occurrence tables, lane work
    // per lane: SMEM pass, re-seeding, -y seeds + sort, chaining, mem_chain_flt, filter + output
    unsigned long long lt[6] = {0ULL, 0ULL, 0ULL, 0ULL, 0ULL, 0ULL};
    unsigned long long ot[3] = {0ULL, 0ULL, 0ULL};   // occurrence table: starts, hits, count table
    for (;;) {
        int b0 = 0;
        if (lane == 0) b0 = atomicAdd(D.next, 64);
        b0 = __shfl(b0, 0, 64);
        const int64_t nlim = D.rlist ? D.n_list : D.n_sr;   // rlist: the reads of a retry pass
        if (b0 >= nlim) {   // every wave reaches this: the grid drains
            if (D.prof) {
#pragma unroll
                for (int k = 0; k < 6; ++k)
                    for (int o = 32; o > 0; o >>= 1) lt[k] += __shfl_xor(lt[k], o, 64);
            }
            if (D.prof && lane == 0) {
                atomicAdd(&D.prof[0], pt[0]);
                atomicAdd(&D.prof[1], pt[1]);
                for (int k = 0; k < 6; ++k) atomicAdd(&D.prof[4 + k], lt[k]);   // lane-summed
                for (int k = 0; k < 3; ++k) atomicAdd(&D.prof[10 + k], ot[k]);
            }
            break;
        }
        const unsigned long long t0 = D.prof ? wall_clock64() : 0ULL;
        int my_err = 0, my_hits = 0;
        const int nb = (int)(nlim - b0 < 64 ? nlim - b0 : 64);
        for (int rd = 0; rd < nb; ++rd) {
            const int i = D.rlist ? D.rlist[b0 + rd] : b0 + rd;
            const int64_t o = D.sr_off[i];
            const int len = (int)(D.sr_off[i + 1] - o);
            seedc::Scratch S = seedc::carve(base + (int64_t)rd * D.stride, D.caps);
            int err = 0, nh = 0;
            if (len > S.lmax || len > SEED_LMAX - 1) err = seedc::SC_OVER_LEN;
            if (len > 0 && !err)
                err = build_occ_wave<4>(D.V, S, D.sr_seq + o, len, ho, lane, q4_lds[wv], lcnt, &nh, D.prof ? ot : nullptr,
                                     LZ);
            if (lane == rd) my_err = err, my_hits = nh;
        }
        const unsigned long long t1 = D.prof ? wall_clock64() : 0ULL;
        if (lane < nb) {
            const int i = D.rlist ? D.rlist[b0 + lane] : b0 + lane;
            const int64_t o = D.sr_off[i];
            const int len = (int)(D.sr_off[i + 1] - o);
            seedc::Scratch S = seedc::carve(base + (int64_t)lane * D.stride, D.caps);
            int n = 0, err = my_err;
            if (len > 0 && !err)
                err = seedc::map_after_occ<LZ>(D.V, D.O, S, D.sr_seq + o, len, i, D.out + (int64_t)(i - D.out0) * D.caps.out,
                                           D.caps.out, &n, D.prof ? lt : nullptr, lcnt,
                                           D.dp ? D.dp + slot * (2 * 201 * 64) + lane : nullptr);
            // a read whose hit table overflowed reports the hits it needs (the retry pass sizes
            // its slices from them: texts of 1 - 3 Gb give ~20-50 k hits per 150 bp read)
            D.n_out[i] = (my_err & seedc::SC_OVER_HITS) ? -my_hits
                         : (LZ && (err & seedc::SC_OVER_HITS)) ? -S.lz[2]   // (the lazy pool's need)
                                                                        : (err ? 0 : n);
            D.status[i] = err;
        }
        if (D.prof && lane == 0) {
            pt[0] += t1 - t0;
            pt[1] += wall_clock64() - t1;
        }
        __threadfence_block();
    }
}

// Pass 1's tail: a wave maps 64 reads in lock-step (its time is its slowest lane's read) and the
// ~7.2 k batches of configs[1] fill the 4,096 resident waves 1.75 times, so the last batches ran
// with a quarter of the waves idle and the waves' busy time averaged 73 % of the launch.  Mapping
// the reads costliest first (longest-processing-time order) puts similar reads in a batch and
// the cheap batches at the end.  The estimate: every second 12-mer start's occurrence count in
// the index (capped at 1024), summed; reads with N bases only lose those starts.  Measured slower
// at configs[1] (312.5 vs 306.2 ms): opt-in only (PRGPU_SEED_LPT=1, pr_seed_gpu_map).
__global__ void __launch_bounds__(256) seed_cost_kernel(seedc::IndexView V, const uint8_t *sr_seq, const int64_t *sr_off,
                                                        int64_t r0, int64_t n, uint32_t *key, int32_t *val) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = r0 + k;
        const int64_t o = sr_off[i];
        const int len = (int)(sr_off[i + 1] - o);
        uint32_t code = 0u, cost = 0u;
        int valid = 0;
        for (int p = 0; p < len; ++p) {
            const uint32_t c = sr_seq[o + p];
            if (c > 3u) {
                valid = 0;
                continue;
            }
            code = ((code << 2) | c) & (seedc::NK - 1u);
            if (++valid >= seedc::KI && (p & 1) == 0) {
                const uint64_t m = V.koff[code + 1] - V.koff[code];
                cost += m < 1024u ? (uint32_t)m : 1024u;
            }
        }
        key[k] = 0xFFFFFFFFu - cost;   // ascending sort = costliest first
        val[k] = (int32_t)i;
    }
}
size_t seed_order_bytes(int64_t n) {
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int32_t *)nullptr,
                                    (int32_t *)nullptr, (size_t)(n > 0 ? n : 1), 0u, 32u, (hipStream_t)0);
    return (size_t)(n > 0 ? n : 1) * 16 + ((tb + 255) & ~(size_t)255) + 256;
}
int seed_order_launch(const SeedDev &D, int64_t r0, int64_t n, void *buf, int32_t **order, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const size_t n1 = (size_t)(n > 0 ? n : 1);
    uint32_t *k0 = (uint32_t *)buf, *k1 = k0 + n1;
    int32_t *v0 = (int32_t *)(k1 + n1), *v1 = v0 + n1;
    void *temp = (void *)(((uintptr_t)(v1 + n1) + 255) & ~(uintptr_t)255);
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, n1, 0u, 32u, s);
    int64_t grid = (n + 255) / 256;
    grid = grid < 4096 ? (grid > 0 ? grid : 1) : 4096;
    hipLaunchKernelGGL(seed_cost_kernel, dim3((unsigned)grid), dim3(256), 0, s, D.V, D.sr_seq, D.sr_off, r0, n, k0, v0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    // (stable LSD sort: equal estimates keep read order)
    if ((e = rocprim::radix_sort_pairs(temp, tb, k0, k1, v0, v1, (size_t)n, 0u, 32u, s)) != hipSuccess) return (int)e;
    *order = v1;
    return 0;
}

int seed_slots_per_cu(int walk_nw) {
    int nb = 0;
    const hipError_t e = walk_nw == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, seed_wave_kernel<1>, 64 * SEED_WAVES, 0)
                                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, seed_wave_kernel<4>, 64 * SEED_WAVES, 0);
    if (e != hipSuccess || nb < 1)
        nb = 2;
    return nb * SEED_WAVES;
}

int seed_launch(const SeedDev &D, void *stream) {
    if (D.n_list <= 0) return 0;
    const int64_t blocks = (D.n_lanes + SEED_WAVES - 1) / SEED_WAVES;
    if (D.V.walk_nw == 1)
        hipLaunchKernelGGL(seed_wave_kernel<1>, dim3((unsigned)blocks), dim3(64 * SEED_WAVES), 0, (hipStream_t)stream, D);
    else
        hipLaunchKernelGGL(seed_wave_kernel<4>, dim3((unsigned)blocks), dim3(64 * SEED_WAVES), 0, (hipStream_t)stream, D);
    return (int)hipGetLastError();
}

int seed_batch_launch(const SeedDev &D, void *stream) {
    if (D.n_sr <= 0) return 0;
    const int64_t blocks = (D.n_lanes + SEED_WAVES - 1) / SEED_WAVES;
    if (D.caps.lazy)
        hipLaunchKernelGGL(seed_batch_kernel<true>, dim3((unsigned)blocks), dim3(64 * SEED_WAVES), 0, (hipStream_t)stream, D);
    else
        hipLaunchKernelGGL(seed_batch_kernel<false>, dim3((unsigned)blocks), dim3(64 * SEED_WAVES), 0, (hipStream_t)stream, D);
    return (int)hipGetLastError();
}

__global__ void seed_compact_kernel(const pr_seed_task *slots, const int32_t *n_out, const int64_t *pre, int64_t n_sr,
                                    int cap, pr_seed_task *out) {
    // one wave per read: lanes copy the read's tasks (10 dwords each) as dwords
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (i >= n_sr) return;
    const int n = n_out[i];
    constexpr int TW = (int)(sizeof(pr_seed_task) / 4);
    const uint32_t *src = reinterpret_cast<const uint32_t *>(slots + i * cap);
    uint32_t *dst = reinterpret_cast<uint32_t *>(out + pre[i]);
    for (int k = lane; k < n * TW; k += 64) dst[k] = src[k];
}

int seed_compact_launch(const pr_seed_task *slots, const int32_t *n_out, const int64_t *pre, int64_t n_sr, int cap,
                        pr_seed_task *out, void *stream) {
    if (n_sr <= 0) return 0;
    const int64_t blocks = (n_sr + 3) / 4;
    hipLaunchKernelGGL(seed_compact_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, slots, n_out, pre,
                       n_sr, cap, out);
    return (int)hipGetLastError();
}

}  // namespace prgpu
