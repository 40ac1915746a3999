// SW -> consensus hand-off on the device (one proovread iteration without the
// SAM/BAM round trip): what `bwa-proovread mem | samtools view -bS`,
// `samtools sort` and bam2cns's per-read `samtools view BAM id:` do between the
// two hot stages (bin/proovread:1313, 1330-1355; bin/bam2cns:336).
//
//   pipe_count_kernel : per long read, the reported alignments (score >= -T
//                       per-base threshold, CIGAR ok)
//   pipe_scan_kernel  : exclusive prefix -> first alignment of every read
//   pipe_sort_kernel  : per long read, bitonic sort in LDS of
//                       (POS, strand, task order) = samtools' coordinate order
//                       (stable for equal keys), then the consensus-stage
//                       alignment arrays are written in that order.  SEQ is not
//                       materialised: the consensus reads the short read (nt4)
//                       through the reverse-complement flag, and the CIGAR in
//                       place from the SW output.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pipe_dev.h"

namespace prgpu {

constexpr int PIPE_THREADS = 256;

__global__ void __launch_bounds__(PIPE_THREADS) pipe_count_kernel(PipeDev P) {
    __shared__ int red[PIPE_THREADS / 64];
    for (int lr = blockIdx.x; lr < P.n_lr; lr += gridDim.x) {
        const int64_t t0 = P.task_off[lr], t1 = P.task_off[lr + 1];
        int c = 0;
        for (int64_t t = t0 + threadIdx.x; t < t1; t += PIPE_THREADS) c += (P.pass[t] && P.status[t] == 0) ? 1 : 0;
        for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) {
            int s = 0;
            for (int i = 0; i < PIPE_THREADS / 64; ++i) s += red[i];
            P.cnt[lr] = s;
        }
        __syncthreads();
    }
}

// single-block exclusive scan of n counts into off[0..n]
__global__ void __launch_bounds__(1024) pipe_scan_kernel(const int32_t *cnt, int64_t *off, int n) {
    __shared__ long long part[1024];
    const int tid = threadIdx.x;
    const int per = (n + 1023) / 1024;
    const int b0 = tid * per, b1 = (b0 + per) < n ? (b0 + per) : n;
    long long s = 0;
    for (int i = b0; i < b1; ++i) s += cnt[i];
    part[tid] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        long long v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    long long base = part[tid] - s;
    for (int i = b0; i < b1; ++i) { off[i] = base; base += cnt[i]; }
    if (tid == 1023) off[n] = part[1023];
}

__global__ void __launch_bounds__(PIPE_THREADS) pipe_sort_kernel(PipeDev P) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];
    __shared__ int s_n;
    for (int lr = blockIdx.x; lr < P.n_lr; lr += gridDim.x) {
        const int64_t t0 = P.task_off[lr], t1 = P.task_off[lr + 1];
        const int nt = (int)(t1 - t0);
        const int cnt = P.cnt[lr];
        if (cnt > P.sort_cap) {   // cannot happen: sort_cap >= max tasks per read (host)
            if (threadIdx.x == 0) P.err[lr] = 1;
            continue;
        }
        int n2 = 1;
        while (n2 < cnt) n2 <<= 1;
        if (threadIdx.x == 0) s_n = 0;
        for (int i = threadIdx.x; i < n2; i += PIPE_THREADS) keys[i] = ~0ULL;
        __syncthreads();
        for (int i = threadIdx.x; i < nt; i += PIPE_THREADS) {
            const int64_t t = t0 + i;
            if (!(P.pass[t] && P.status[t] == 0)) continue;
            const int slot = atomicAdd(&s_n, 1);
            keys[slot] = ((unsigned long long)(uint32_t)P.pos[t] << 33) |
                         ((unsigned long long)(P.strand[t] & 1u) << 32) | (unsigned long long)(uint32_t)i;
        }
        __syncthreads();
        // bitonic sort ascending
        for (int k = 2; k <= n2; k <<= 1) {
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < n2; i += PIPE_THREADS) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const unsigned long long a = keys[i], b = keys[ixj];
                        const bool up = (i & k) == 0;
                        if ((a > b) == up) { keys[i] = b; keys[ixj] = a; }
                    }
                }
                __syncthreads();
            }
        }
        const int64_t a0 = P.aln_off[lr];
        for (int r = threadIdx.x; r < cnt; r += PIPE_THREADS) {
            const int64_t t = t0 + (int64_t)(keys[r] & 0xFFFFFFFFull);
            const int64_t g = a0 + r;
            const int sid = P.t_sr[t];
            P.a_pos[g] = P.pos[t] + 1;
            P.a_score[g] = (double)P.score[t];
            P.a_flags[g] = (uint8_t)(1u | (P.strand[t] ? 8u : 0u));   // HAS_SCORE | REVCOMP
            P.a_seq_off[g] = P.sr_off[sid];
            P.a_lseq[g] = (int32_t)(P.sr_off[sid + 1] - P.sr_off[sid]);
            P.a_cig_off[g] = P.cig_at[t];
            P.a_ncig[g] = P.ncig[t];
        }
        __syncthreads();
    }
}

// per-iteration statistic gathered across GPUs (proovread:1702-1720 computes
// bpN/bpt with SeqFilter --phred-mask; here: corrected bases and bases with
// phred >= min_phred, summed into out[0..1] on the device)
__global__ void __launch_bounds__(256) iter_stats_kernel(const int64_t *out_off, const int32_t *status,
                                                         const int32_t *seq_len, const uint8_t *qual, int n_lr,
                                                         int min_char, unsigned long long *out) {
    unsigned long long tot = 0, hq = 0;
    for (int lr = blockIdx.x; lr < n_lr; lr += gridDim.x) {
        if (status[lr] != 0) continue;
        const int64_t o = out_off[lr];
        const int n = seq_len[lr];
        if (threadIdx.x == 0) tot += (unsigned long long)n;
        for (int i = threadIdx.x; i < n; i += 256) hq += qual[o + i] >= min_char ? 1ull : 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) { tot += __shfl_down(tot, o, 64); hq += __shfl_down(hq, o, 64); }
    if ((threadIdx.x & 63) == 0) {
        if (tot) atomicAdd(&out[0], tot);
        if (hq) atomicAdd(&out[1], hq);
    }
}

int iter_stats_launch(const int64_t *out_off, const int32_t *status, const int32_t *seq_len, const uint8_t *qual,
                      int n_lr, int min_char, unsigned long long *out, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(out, 0, 16, s);
    if (e != hipSuccess) return (int)e;
    const int grid = n_lr < 2048 ? (n_lr > 0 ? n_lr : 1) : 2048;
    hipLaunchKernelGGL(iter_stats_kernel, dim3(grid), dim3(256), 0, s, out_off, status, seq_len, qual, n_lr,
                       min_char, out);
    return (int)hipGetLastError();
}

int pipe_launch(const PipeDev &P, int grid, void *stream, int lds_sort) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(pipe_count_kernel, dim3(grid), dim3(PIPE_THREADS), 0, s, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(pipe_scan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t *)P.cnt, P.aln_off, P.n_lr);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    e = hipFuncSetAttribute((const void *)pipe_sort_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_sort);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(pipe_sort_kernel, dim3(grid), dim3(PIPE_THREADS), lds_sort, s, P);
    return (int)hipGetLastError();
}

}  // namespace prgpu
