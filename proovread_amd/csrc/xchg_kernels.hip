// The exact-parity multi-GPU layout's alignment exchange on the device:
// what proovread does between `bwa-proovread mem` and bam2cns with files -- every long
// read's SAM records collected from wherever they were computed (bin/proovread:1313,
// 1330-1355, bam2cns:336) -- as two kernels around one RCCL all-to-all, with no SAM text.
//
//   sender   xchg_key_kernel    owner of every reported alignment's long read (binary
//                               search of the rank ranges), per-owner record / op counts
//                               (LDS histogram, one atomic per workgroup and owner)
//            radix sort         stable by owner: SAM order inside every owner's block
//            xchg_pack_kernel   24-byte wire records + the CIGAR ops at their prefix
//   receiver xchg_rkey_kernel   local long read of every received record, ops per record
//            radix sort         stable by long read: the single run's per-long-read order
//                               (the blocks arrive source-rank-major, the short-read shards
//                               are contiguous), which -b/-l and the hand-off sort rely on
//            xchg_gather_kernel the hand-off's per-alignment arrays in grouped order
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "xchg_dev.h"

namespace prgpu {

constexpr int XT = 256;
constexpr int XMAXW = 64;   // ranks the per-workgroup histogram holds

static unsigned grid_of(int64_t n) {
    const int64_t g = (n + XT - 1) / XT;
    return (unsigned)(g < 1 ? 1 : (g > 65535 * 16 ? 65535 * 16 : g));
}

__device__ inline bool x_ok(const XchgSend &X, int32_t t) { return X.pass[t] && X.status[t] == 0; }

__global__ void __launch_bounds__(XT) xchg_key_kernel(XchgSend X) {
    __shared__ unsigned long long h[2 * (XMAXW + 1)];
    for (int k = threadIdx.x; k < 2 * (X.world + 1); k += XT) h[k] = 0ull;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < X.n; i += (int64_t)gridDim.x * XT) {
        const int32_t t = X.alist[i];
        int o = X.world;
        if (x_ok(X, t)) {
            const int64_t lr = X.t_lr[t];
            int lo = 0, hi = X.world;   // last rank r with bounds[r] <= lr
            while (hi - lo > 1) {
                const int m = (lo + hi) >> 1;
                if (X.bounds[m] <= lr) lo = m;
                else hi = m;
            }
            o = lo;
            atomicAdd(&h[X.world + 1 + o], (unsigned long long)X.ncig[t]);
        }
        atomicAdd(&h[o], 1ull);
        X.key0[i] = o;
        X.idx0[i] = (int32_t)i;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * (X.world + 1); k += XT)
        if (h[k]) atomicAdd(&X.cnt[k], h[k]);
}

__global__ void __launch_bounds__(XT) xchg_ops_kernel(XchgSend X) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i <= X.n; i += (int64_t)gridDim.x * XT) {
        int64_t v = 0;
        if (i < X.n && X.key1[i] < X.world) v = X.ncig[X.alist[X.idx1[i]]];
        X.op_in[i] = v;
    }
}

__global__ void __launch_bounds__(XT) xchg_pack_kernel(XchgSend X) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < X.n; i += (int64_t)gridDim.x * XT) {
        if (X.key1[i] >= X.world) continue;   // not reported (sorted to the end)
        const int32_t t = X.alist[X.idx1[i]];
        XRec r;
        r.sr = (int32_t)(X.sr0 + X.t_sr[t]);
        r.lr = X.t_lr[t];
        r.pos = X.pos[t];
        r.score = X.score[t];
        r.ncig = X.ncig[t];
        r.strand = X.strand[t];
        X.rec[i] = r;
        const uint32_t *src = X.cig + X.cig_at[t];
        uint32_t *dst = X.wcig + X.op_at[i];
        for (int k = 0; k < r.ncig; ++k) dst[k] = src[k];
    }
}

__global__ void __launch_bounds__(XT) xchg_rkey_kernel(XchgRecv X) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i <= X.n; i += (int64_t)gridDim.x * XT) {
        if (i == X.n) {
            X.op_in[i] = 0;
            continue;
        }
        const XRec r = X.rec[i];
        int32_t l = r.lr - X.lr0;
        if (l < 0 || l >= X.n_lr) {
            X.err[0] = 1;
            l = 0;
        }
        X.key0[i] = l;
        X.idx0[i] = (int32_t)i;
        X.op_in[i] = r.ncig;
        atomicAdd(&X.cnt[l], 1);
    }
}

__global__ void __launch_bounds__(XT) xchg_cnt64_kernel(XchgRecv X) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i <= X.n_lr; i += (int64_t)gridDim.x * XT)
        X.cnt64[i] = i < X.n_lr ? X.cnt[i] : 0;
}

__global__ void __launch_bounds__(XT) xchg_gather_kernel(XchgRecv X) {
    for (int64_t i = (int64_t)blockIdx.x * XT + threadIdx.x; i < X.n; i += (int64_t)gridDim.x * XT) {
        const int32_t j = X.idx1[i];
        const XRec r = X.rec[j];
        X.o_sr[i] = r.sr;
        X.o_status[i] = 0;
        X.o_pos[i] = r.pos;
        X.o_score[i] = r.score;
        X.o_ncig[i] = r.ncig;
        X.o_cig_at[i] = X.rcig_at[j];
        X.o_strand[i] = (uint8_t)r.strand;
        X.o_pass[i] = 1;
    }
}

static int key_bits(int32_t n_keys) {
    int b = 1;
    while (b < 31 && (1 << b) < n_keys) ++b;
    return b;
}

size_t xchg_temp_bytes(int64_t n, int32_t n_keys) {
    size_t a = 0, b = 0, c = 0;
    (void)n_keys;
    (void)rocprim::radix_sort_pairs(nullptr, a, (int32_t *)nullptr, (int32_t *)nullptr, (int32_t *)nullptr,
                                    (int32_t *)nullptr, (size_t)(n > 0 ? n : 1), 0, 31, (hipStream_t)0);
    (void)rocprim::exclusive_scan(nullptr, b, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0, (size_t)n + 1,
                                  rocprim::plus<int64_t>(), (hipStream_t)0);
    (void)rocprim::exclusive_scan(nullptr, c, (int64_t *)nullptr, (int64_t *)nullptr, (int64_t)0,
                                  (size_t)(n_keys > 0 ? n_keys : 1) + 1, rocprim::plus<int64_t>(), (hipStream_t)0);
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

int xchg_pack_launch(const XchgSend &X, void *temp, size_t temp_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (X.world < 1 || X.world > XMAXW) return (int)hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(X.cnt, 0, (size_t)2 * (X.world + 1) * 8, s);
    if (e != hipSuccess || X.n <= 0) return (int)e;
    hipLaunchKernelGGL(xchg_key_kernel, dim3(grid_of(X.n) < 4096 ? grid_of(X.n) : 4096), dim3(XT), 0, s, X);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    if ((e = rocprim::radix_sort_pairs(temp, tb, X.key0, X.key1, X.idx0, X.idx1, (size_t)X.n, 0, key_bits(X.world + 1),
                                       s)) != hipSuccess)
        return (int)e;
    hipLaunchKernelGGL(xchg_ops_kernel, dim3(grid_of(X.n + 1)), dim3(XT), 0, s, X);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    tb = temp_bytes;
    if ((e = rocprim::exclusive_scan(temp, tb, X.op_in, X.op_at, (int64_t)0, (size_t)X.n + 1, rocprim::plus<int64_t>(),
                                     s)) != hipSuccess)
        return (int)e;
    return 0;
}

int xchg_write_launch(const XchgSend &X, void *stream) {
    if (X.n <= 0) return 0;
    hipLaunchKernelGGL(xchg_pack_kernel, dim3(grid_of(X.n)), dim3(XT), 0, (hipStream_t)stream, X);
    return (int)hipGetLastError();
}

int xchg_group_launch(const XchgRecv &X, void *temp, size_t temp_bytes, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(X.cnt, 0, (size_t)(X.n_lr + 1) * 4, s);
    if (e != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(X.err, 0, 4, s)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(xchg_rkey_kernel, dim3(grid_of(X.n + 1)), dim3(XT), 0, s, X);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    size_t tb = temp_bytes;
    if ((e = rocprim::exclusive_scan(temp, tb, X.op_in, X.rcig_at, (int64_t)0, (size_t)X.n + 1,
                                     rocprim::plus<int64_t>(), s)) != hipSuccess)
        return (int)e;
    if (X.n > 0) {
        tb = temp_bytes;
        if ((e = rocprim::radix_sort_pairs(temp, tb, X.key0, X.key1, X.idx0, X.idx1, (size_t)X.n, 0,
                                           key_bits(X.n_lr), s)) != hipSuccess)
            return (int)e;
        hipLaunchKernelGGL(xchg_gather_kernel, dim3(grid_of(X.n)), dim3(XT), 0, s, X);
        if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(xchg_cnt64_kernel, dim3(grid_of((int64_t)X.n_lr + 1)), dim3(XT), 0, s, X);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    tb = temp_bytes;
    return (int)rocprim::exclusive_scan(temp, tb, X.cnt64, X.task_off, (int64_t)0, (size_t)X.n_lr + 1,
                                        rocprim::plus<int64_t>(), s);
}

}  // namespace prgpu
