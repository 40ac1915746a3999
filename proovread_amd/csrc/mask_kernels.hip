// Per-iteration masking of corrected long reads: the work of
// `SeqFilter --phred-mask <hcr-mask> --base-content N` at bin/proovread:1706,
// done on the consensus while it is still in HBM.  Algorithm: mask_core.h.
//
// One wave per read (grid-stride over reads, 4 waves per workgroup):
//   1. scan: each lane loads one quality char per 64-column step (coalesced),
//      the in-range test is ballot-ed into a 64-bit mask and the wave-uniform
//      run tracker (mask_runs_feed: ctz over the mask, scalar registers) closes
//      the HCRs; lane 0 stores them to the read's run slots;
//   2. resolve: lane 0 runs the sticky / end / gap rounds on its own stores
//      (mask_resolve); the MCR count is broadcast with readfirstlane;
//   3. write: per 64-column step every lane copies its base or writes 'N'; the
//      MCRs that intersect the step are read by lane 0 and broadcast, so no lane
//      reads another lane's global stores.  'N' bases and read lengths are
//      summed per lane, reduced per wave and added to stats[0..1].
// Bytes per column: quality in + base in + base out (3 B/column, HBM bound).
#include <hip/hip_runtime.h>

#include "mask_dev.h"

namespace prgpu {

__device__ __forceinline__ int32_t bcast_i32(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

__global__ void __launch_bounds__(256) mask_lr_kernel(MaskDev D) {
    const int lane = threadIdx.x & 63;
    const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nw = gridDim.x * 4;
    const int lo = D.cfg.lo_char, hi = D.cfg.hi_char;
    unsigned long long tot = 0, nn = 0;
    for (int r = wid; r < D.n; r += nw) {
        if (D.status && D.status[r] != 0) continue;
        const int64_t o = D.off[r];
        const int64_t room = D.off[r + 1] - o;
        int64_t L = D.len ? (int64_t)D.len[r] : room;
        L = L < 0 ? 0 : (L > room ? room : L);   // a length never exceeds the read's slot
        const uint8_t *q = D.qual + o;
        const uint8_t *s = D.seq + o;
        uint8_t *w = D.out + o;
        const int64_t r0 = D.run_off[r];
        const int64_t cap = D.run_off[r + 1] - r0;
        MaskRun *h = D.runs + r0;
        MaskRun *t = D.tmp + r0;
        MaskRun *hs = lane == 0 ? h : nullptr;

        // 1. HCR scan
        int64_t n = 0, run = -1;
        for (int64_t base = 0; base < L; base += 64) {
            const int64_t c = base + lane;
            const int qq = c < L ? (int)q[c] : 0;
            const uint64_t bits = __ballot(c < L && qq >= lo && qq <= hi);
            const int valid = (int)(L - base < 64 ? L - base : 64);
            mask_runs_feed(bits, base, valid, run, D.cfg.lcs_min, hs, n, cap);
        }
        mask_runs_close(L, run, D.cfg.lcs_min, hs, n, cap);

        // 2. resolve (lane 0 on its own stores)
        int32_t m = 0;
        if (n > cap) {
            if (lane == 0) *D.err = 1;
            n = 0;
        }
        if (lane == 0) m = (int32_t)mask_resolve(h, n, L, D.cfg, t);
        m = bcast_i32(m);
        if (lane == 0 && D.n_runs) D.n_runs[r] = m;

        // 3. write the masked read
        int32_t k = 0, ko = 0, ke = 0;   // first MCR not ending before the step, its [off, end)
        auto load = [&](int32_t j, int32_t &jo, int32_t &je) {
            int32_t a = 0, b = 0;
            if (lane == 0) {
                a = h[j].off;
                b = h[j].off + h[j].len;
            }
            jo = bcast_i32(a);
            je = bcast_i32(b);
        };
        if (m > 0) load(0, ko, ke);
        for (int64_t base = 0; base < L; base += 64) {
            while (k < m && ke <= base) {
                ++k;
                if (k < m) load(k, ko, ke);
            }
            const int64_t c = base + lane;
            bool masked = false;
            int32_t j = k, jo = ko, je = ke;
            while (j < m && jo < base + 64) {
                masked |= c >= jo && c < je;
                ++j;
                if (j < m) load(j, jo, je);
            }
            if (c < L) {
                const uint8_t b = masked ? (uint8_t)'N' : s[c];
                w[c] = b;
                nn += b == 'N';
            }
        }
        if (lane == 0) tot += (unsigned long long)L;
    }
    for (int sh = 32; sh > 0; sh >>= 1) {
        tot += __shfl_down(tot, sh, 64);
        nn += __shfl_down(nn, sh, 64);
    }
    if (lane == 0) {
        if (tot) atomicAdd(&D.stats[0], tot);
        if (nn) atomicAdd(&D.stats[1], nn);
    }
}

int mask_launch(const MaskDev &D, int n_cu, void *stream) {
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(D.stats, 0, 16, st);
    if (e != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(D.err, 0, 4, st)) != hipSuccess) return (int)e;
    if (D.n <= 0) return 0;
    int64_t blocks = ((int64_t)D.n + 3) / 4;
    const int64_t max_blocks = (int64_t)(n_cu > 0 ? n_cu : 256) * 16;
    if (blocks > max_blocks) blocks = max_blocks;
    hipLaunchKernelGGL(mask_lr_kernel, dim3((unsigned)blocks), dim3(256), 0, st, D);
    return (int)hipGetLastError();
}

}  // namespace prgpu
