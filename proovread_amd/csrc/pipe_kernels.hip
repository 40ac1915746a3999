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

#include <rocprim/device/device_scan.hpp>

#include "pipe_dev.h"

namespace prgpu {

constexpr int PIPE_THREADS = 256;

__global__ void __launch_bounds__(PIPE_THREADS) pipe_count_kernel(PipeDev P) {
    __shared__ int red[PIPE_THREADS / 64];
    for (int lr = blockIdx.x; lr < P.n_lr; lr += gridDim.x) {
        const int64_t t0 = P.task_off[lr], t1 = P.task_off[lr + 1];
        int c = 0;
        for (int64_t t = t0 + threadIdx.x; t < t1; t += PIPE_THREADS)
            c += (P.pass[t] && P.status[t] == 0 && (!P.keep || P.keep[t])) ? 1 : 0;
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
            if (!(P.pass[t] && P.status[t] == 0 && (!P.keep || P.keep[t]))) continue;
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

// bwa-proovread's -b/-l filter (bin/proovread:1302-1313; its proovread.[ch] is absent, the
// filter is restated as proovread's own score binning, Sam::Seq add_aln_by_score,
// Seq.pm:582-614, as bwa_proovread.py's BinFilter does): per long read, the reported
// alignments in bwa's output order (the read order of the tasks) are binned by centre,
// bin = int((POS + length / 2) / BIN), length by Sam::Alignment::length
// (Alignment.pm:417-431: M+D when clipped, else the SEQ length), ncscore =
// AS/length * length/(40+length); a bin holding more than LEN bases admits an alignment
// only if it beats the bin's lowest ncscore, which it evicts.  One workgroup per long
// read: a stable counting sort by bin in LDS, then one thread per bin in task order.
__global__ void __launch_bounds__(PIPE_THREADS) pipe_binfilter_kernel(PipeDev P, int bin_size, double bin_length,
                                                                       int max_bins) {
    extern __shared__ __attribute__((aligned(16))) int fsm[];
    int *cnt = fsm, *start = fsm + max_bins, *chunk = fsm + 2 * max_bins;
    __shared__ long long red[PIPE_THREADS / 64];
    __shared__ int s_tot;
    for (int lr = blockIdx.x; lr < P.n_lr; lr += gridDim.x) {
        const int64_t t0 = P.task_off[lr], t1 = P.task_off[lr + 1];
        const int nt = (int)(t1 - t0);
        const long L = (long)(P.lr_off[lr + 1] - P.lr_off[lr]);
        const int nbins = (int)((double)(L + 1024) / bin_size) + 2;   // centres <= L + query / 2
        for (int b = threadIdx.x; b < nbins; b += PIPE_THREADS) cnt[b] = 0;
        __syncthreads();
        for (int i = threadIdx.x; i < nt; i += PIPE_THREADS) {
            const int64_t t = t0 + i;
            P.keep[t] = 0;
            int bin = -1;
            if (P.pass[t] && P.status[t] == 0) {
                const uint32_t *cg = P.cig + P.cig_at[t];
                const int n = P.ncig[t];
                const int sid = P.t_sr[t];
                const int ls = (int)(P.sr_off[sid + 1] - P.sr_off[sid]);
                long md = 0;
                uint32_t c_first = 0u, c_last = 0u;
                for (int k0 = 0; k0 < n; k0 += 8) {   // 8 independent loads in flight per step
                    uint32_t v[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) v[u] = k0 + u < n ? cg[k0 + u] : 0u;
                    if (k0 == 0) c_first = v[0];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t op = v[u] & 15u;
                        if (k0 + u < n && (op == 0u || op == 2u)) md += v[u] >> 4;
                        if (k0 + u == n - 1) c_last = v[u];
                    }
                }
                const bool clipped = n > 0 && ((c_first & 15u) == 4u || (c_last & 15u) == 4u);
                const long len = (ls == 0 || clipped) ? md : ls;
                P.flen[t] = (int32_t)len;
                if (len > 0) {
                    const double sc = (double)P.score[t];
                    P.fnc[t] = __dmul_rn(__ddiv_rn(sc, (double)len), __ddiv_rn((double)len, (double)(40 + len)));
                    const double c = __ddiv_rn(__dadd_rn((double)(P.pos[t] + 1), __ddiv_rn((double)len, 2.0)),
                                               (double)bin_size);
                    bin = (int)(long)c;
                    if (bin < 0 || bin >= nbins) bin = -2;   // cannot happen (nbins bound); reported as an error
                }
            }
            P.fbin[t] = bin;
            if (bin >= 0) atomicAdd(&cnt[bin], 1);
            if (bin == -2) P.err[lr] = 2;
        }
        __syncthreads();
        // exclusive scan of cnt -> start
        {
            const int per = (nbins + PIPE_THREADS - 1) / PIPE_THREADS;
            const int b0 = threadIdx.x * per, b1 = (b0 + per) < nbins ? (b0 + per) : nbins;
            long long s = 0;
            for (int b = b0; b < b1; ++b) s += cnt[b];
            long long x = s;
            const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
            for (int o = 1; o < 64; o <<= 1) {
                const long long y = __shfl_up(x, o, 64);
                if (lane >= o) x += y;
            }
            if (lane == 63) red[w] = x;
            __syncthreads();
            long long base = 0;
            for (int k = 0; k < w; ++k) base += red[k];
            base += x - s;
            for (int b = b0; b < b1; ++b) { start[b] = (int)base; base += cnt[b]; cnt[b] = 0; }
        }
        __syncthreads();
        // stable scatter by bin, chunks of 256 tasks in task order
        for (int c0 = 0; c0 < nt; c0 += PIPE_THREADS) {
            const int i = c0 + (int)threadIdx.x;
            const int b = i < nt ? P.fbin[t0 + i] : -1;
            chunk[threadIdx.x] = b;
            __syncthreads();
            int rank = 0;
            bool last = true;
            if (b >= 0) {
                for (int j = 0; j < PIPE_THREADS; ++j) {
                    const int bj = chunk[j];
                    if (bj == b) { if (j < (int)threadIdx.x) ++rank; else if (j > (int)threadIdx.x) last = false; }
                }
                P.fsorted[t0 + start[b] + cnt[b] + rank] = i;
            }
            __syncthreads();
            if (b >= 0 && last) cnt[b] += rank + 1;
            __syncthreads();
        }
        // one thread per bin: sequential admission in task order
        for (int b = threadIdx.x; b < nbins; b += PIPE_THREADS) {
            const int sidx = start[b], nb = cnt[b];
            double *ls = P.flst + t0 + sidx;
            int32_t *la = P.flsti + t0 + sidx;
            int ln = 0;
            long bases = 0;
            for (int k = 0; k < nb; ++k) {
                const int i = P.fsorted[t0 + sidx + k];
                const double nc = P.fnc[t0 + i];
                if ((double)bases > bin_length) {
                    if (nc <= ls[ln - 1]) continue;
                    bases -= P.flen[t0 + la[ln - 1]];
                    --ln;
                }
                bases += P.flen[t0 + i];
                int j = ln - 1;
                while (j >= 0 && nc > ls[j]) { ls[j + 1] = ls[j]; la[j + 1] = la[j]; --j; }
                ls[j + 1] = nc; la[j + 1] = i;
                ++ln;
            }
            for (int k = 0; k < ln; ++k) P.keep[t0 + la[k]] = 1;
        }
        __syncthreads();
    }
}

int pipe_binfilter_launch(const PipeDev &P, int bin_size, double bin_length, int max_bins, int grid, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const int lds = (2 * max_bins + PIPE_THREADS) * 4;
    hipError_t e = hipFuncSetAttribute((const void *)pipe_binfilter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(pipe_binfilter_kernel, dim3(grid), dim3(PIPE_THREADS), lds, s, P, bin_size, bin_length, max_bins);
    return (int)hipGetLastError();
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

// the resident long-read set after a consensus launch: every read's consensus (and its quality and
// masked copy) from the per-read capacity layout (out_off) into dense pools (dst_off); a
// workgroup per read, 16-byte stores where the destination allows
__global__ void __launch_bounds__(256) lr_compact_kernel(const int64_t *src_off, const int32_t *len,
                                                         const int64_t *dst_off, int n, const uint8_t *s0, uint8_t *d0,
                                                         const uint8_t *s1, uint8_t *d1, const uint8_t *s2, uint8_t *d2) {
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t so = src_off[i], dof = dst_off[i];
        const int L = len[i];
        for (int k = threadIdx.x; k < L; k += 256) {
            d0[dof + k] = s0[so + k];
            if (s1) d1[dof + k] = s1[so + k];
            if (s2) d2[dof + k] = s2[so + k];
        }
    }
}

int lr_compact_launch(const int64_t *src_off, const int32_t *len, const int64_t *dst_off, int n, const uint8_t *s0,
                      uint8_t *d0, const uint8_t *s1, uint8_t *d1, const uint8_t *s2, uint8_t *d2, void *stream) {
    if (n <= 0) return 0;
    const int grid = n < 4096 ? n : 4096;
    hipLaunchKernelGGL(lr_compact_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src_off, len, dst_off, n, s0, d0,
                       s1, d1, s2, d2);
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

// ---------------------------------------------------------------------------
// The consensus input in consensus order.  The hand-off lists each long read's alignments, but
// their SEQ bytes sit in the short-read pool (sequencer order: short reads from anywhere on the
// genome side by side) and their CIGAR ops in the SW output pool (task order); every consensus
// phase that reads them (prep, state table, pileup windows) then touches a line per alignment
// that holds other reads' bytes.  One pass copies them behind each other in the hand-off's order
// (SEQ padded to dwords), and the consensus reads its alignments' inputs sequentially.
__global__ void __launch_bounds__(256) cns_gather_sizes_kernel(const int64_t *aln_total, int64_t n, const int32_t *lseq,
                                                               const int32_t *ncig, int64_t *sz_seq, int64_t *sz_cig) {
    const int64_t m = *aln_total;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g <= n; g += (int64_t)gridDim.x * blockDim.x) {
        const bool in = g < m;
        sz_seq[g] = in ? (int64_t)((lseq[g] + 3) & ~3) : 0;
        sz_cig[g] = in ? (int64_t)ncig[g] : 0;
    }
}

__global__ void __launch_bounds__(256) cns_gather_kernel(const int64_t *aln_total, const uint8_t *seq, const uint32_t *cig,
                                                         int64_t *seq_off, const int32_t *lseq, int64_t *cig_off,
                                                         const int32_t *ncig, const int64_t *nso, const int64_t *nco,
                                                         uint8_t *gseq, uint32_t *gcig) {
    // a 16-lane group per alignment (four alignments in flight per wave: the copies are short
    // and latency-bound); a group's lanes copy dwords k, k + 16, ... of the SEQ, then the ops
    const int gl = threadIdx.x & 15;
    const int64_t m = *aln_total;
    const int64_t stride = ((int64_t)gridDim.x * blockDim.x) >> 4;
    for (int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; g < m; g += stride) {
        const int64_t so = seq_off[g], co = cig_off[g];
        const int ls = lseq[g], nc = ncig[g];
        const int64_t ds = nso[g], dc = nco[g];
        uint32_t *dst = reinterpret_cast<uint32_t *>(gseq + ds);
        const int nw = (ls + 3) >> 2;
        const uint32_t sh = (uint32_t)(so & 3);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(seq + (so & ~(int64_t)3));   // (64 bytes of slack)
        for (int k = gl; k < nw; k += 16) {
            const uint32_t lo = src[k], hi = src[k + 1];
            dst[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
        }
        for (int k = gl; k < nc; k += 16) gcig[dc + k] = cig[co + k];
        if (gl == 0) {   // (every lane of the group has read the old offsets: one instruction stream)
            seq_off[g] = ds;
            cig_off[g] = dc;
        }
    }
}

size_t cns_gather_temp_bytes(int64_t n) {
    size_t tb = 0;
    (void)rocprim::exclusive_scan(nullptr, tb, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0, (size_t)(n + 1),
                                  rocprim::plus<int64_t>());
    return tb + 256;
}

// offsets of the gathered pools: nso / nco [n + 1] (entry n: the totals)
int cns_gather_offsets(const int64_t *aln_total, int64_t n, const int32_t *lseq, const int32_t *ncig, int64_t *sz_seq,
                       int64_t *sz_cig, int64_t *nso, int64_t *nco, void *temp, size_t temp_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    int64_t blocks = (n + 256) / 256;
    blocks = blocks < 65536 ? blocks : 65536;
    hipLaunchKernelGGL(cns_gather_sizes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, aln_total, n, lseq, ncig, sz_seq,
                       sz_cig);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    if ((e = rocprim::exclusive_scan(temp, tb, sz_seq, nso, (int64_t)0, (size_t)(n + 1), rocprim::plus<int64_t>(), s)) !=
        hipSuccess)
        return (int)e;
    tb = temp_bytes;
    if ((e = rocprim::exclusive_scan(temp, tb, sz_cig, nco, (int64_t)0, (size_t)(n + 1), rocprim::plus<int64_t>(), s)) !=
        hipSuccess)
        return (int)e;
    return 0;
}

int cns_gather_copy(const int64_t *aln_total, int64_t n, const uint8_t *seq, const uint32_t *cig, int64_t *seq_off,
                    const int32_t *lseq, int64_t *cig_off, const int32_t *ncig, const int64_t *nso, const int64_t *nco,
                    uint8_t *gseq, uint32_t *gcig, void *stream) {
    int64_t blocks = (n + 15) / 16;   // 16 lanes per alignment
    blocks = blocks < 65536 ? (blocks > 0 ? blocks : 1) : 65536;
    hipLaunchKernelGGL(cns_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, aln_total, seq, cig,
                       seq_off, lseq, cig_off, ncig, nso, nco, gseq, gcig);
    return (int)hipGetLastError();
}

}  // namespace prgpu
