// Probe: does RCCL's point-to-point path deliver a multi-GB block that a
// rank sends to itself intact?  (pr_comm_alltoallv_dev sends the self block as a device copy and
// the others in 256 MB pieces since round 4, when a configs[1] exchange at world 1 over a
// communicator came back corrupted.)  For each size: a pattern block, ncclSend + ncclRecv to
// the same rank in one group, then a device count of the wrong bytes and the first wrong offset.
//   hipcc --offload-arch=gfx950 -O2 rccl_self_p2p.hip -lrccl -o rccl_self_p2p && ./rccl_self_p2p
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) { std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } \
    } while (0)
#define NK(x)                                                                                   \
    do {                                                                                        \
        ncclResult_t r_ = (x);                                                                  \
        if (r_ != ncclSuccess) { std::printf("RCCL %s at %d\n", ncclGetErrorString(r_), __LINE__); std::exit(1); } \
    } while (0)

__device__ __forceinline__ unsigned char pat(unsigned long long i) {
    return (unsigned char)((i * 2654435761ull) >> 13);
}
__global__ void fill(unsigned char *p, unsigned long long n) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        p[i] = pat(i);
}
__global__ void check(const unsigned char *p, unsigned long long n, unsigned long long *bad, unsigned long long *first) {
    unsigned long long b = 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        if (p[i] != pat(i)) {
            ++b;
            atomicMin(first, i);
        }
    if (b) atomicAdd(bad, b);
}

int main(int argc, char **argv) {
    const unsigned long long GiB = 1ull << 30;
    const unsigned long long sizes[] = {256ull << 20, GiB, 2 * GiB - 4096, 2 * GiB, 2 * GiB + 4096, 3 * GiB, 4 * GiB + 4096};
    ncclComm_t comm;
    int dev = 0;
    CK(hipSetDevice(0));
    NK(ncclCommInitAll(&comm, 1, &dev));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    unsigned long long *cnt;
    CK(hipMalloc(&cnt, 16));
    for (unsigned long long n : sizes) {
        unsigned char *a, *b;
        CK(hipMalloc(&a, n));
        CK(hipMalloc(&b, n));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, s, a, n);
        CK(hipMemsetAsync(b, 0, n, s));
        unsigned long long init[2] = {0ull, ~0ull};
        CK(hipMemcpyAsync(cnt, init, 16, hipMemcpyHostToDevice, s));
        NK(ncclGroupStart());
        NK(ncclSend(a, n, ncclUint8, 0, comm, s));
        NK(ncclRecv(b, n, ncclUint8, 0, comm, s));
        NK(ncclGroupEnd());
        hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, s, b, n, cnt, cnt + 1);
        unsigned long long r[2];
        CK(hipMemcpyAsync(r, cnt, 16, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        std::printf("{\"bytes\": %llu, \"wrong\": %llu, \"first_wrong\": %lld}\n", n, r[0], r[0] ? (long long)r[1] : -1ll);
        std::fflush(stdout);
        CK(hipFree(a));
        CK(hipFree(b));
    }
    NK(ncclCommDestroy(comm));
    return 0;
}
