// Calibration of rocprofv3's FETCH_SIZE on gfx950 for the access widths our kernels use
// (MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a 16-B-per-lane coalesced read; other
// widths are uncalibrated).  Each kernel reads a known number of distinct bytes from a
// 1 GiB buffer (well past the 256 MiB Infinity Cache) and writes one dword per workgroup:
//   k16   16 B per lane, coalesced (dwordx4)          -> 1 GiB
//   k4    4 B per lane, coalesced (dword)             -> 1 GiB
//   k1    1 B per lane, coalesced (ubyte)             -> 1 GiB
//   kline one 4-B load per 128-B line, line-strided   -> 1 GiB of lines touched (32 MiB used)
//   krand one 4-B load at a hashed line               -> 2^23 lines touched once (1 GiB)
// tools/fetch_calib.sh runs it under separate FETCH_SIZE passes; the ratios FETCH_SIZE /
// bytes are the corrections tools/pmc_summary.py applies per access class.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr size_t NB = size_t(1) << 30;

__global__ void k16(const uint4 *p, uint32_t *o) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NB / 16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) o[blockIdx.x] = acc;
}
__global__ void k4(const uint32_t *p, uint32_t *o) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NB / 4; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) o[blockIdx.x] = acc;
}
__global__ void k1(const uint8_t *p, uint32_t *o) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NB; i += (size_t)gridDim.x * blockDim.x)
        acc += p[i];
    if (acc == 0x12345678u) o[blockIdx.x] = acc;
}
__global__ void kline(const uint32_t *p, uint32_t *o) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < NB / 128; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i * 32];
    if (acc == 0x12345678u) o[blockIdx.x] = acc;
}
__global__ void krand(const uint32_t *p, uint32_t *o) {
    uint32_t acc = 0;
    const size_t nl = NB / 128;   // a permutation of the lines: odd multiplier mod 2^23
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[((i * 2654435761ull) & (nl - 1)) * 32];
    if (acc == 0x12345678u) o[blockIdx.x] = acc;
}

int main() {
    void *buf = nullptr, *out = nullptr;
    if (hipMalloc(&buf, NB) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    if (hipMemset(buf, 1, NB) != hipSuccess) return 1;
    const int grid = 256 * 8, blk = 256;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k16, dim3(grid), dim3(blk), 0, 0, (const uint4 *)buf, (uint32_t *)out);
        hipLaunchKernelGGL(k4, dim3(grid), dim3(blk), 0, 0, (const uint32_t *)buf, (uint32_t *)out);
        hipLaunchKernelGGL(k1, dim3(grid), dim3(blk), 0, 0, (const uint8_t *)buf, (uint32_t *)out);
        hipLaunchKernelGGL(kline, dim3(grid), dim3(blk), 0, 0, (const uint32_t *)buf, (uint32_t *)out);
        hipLaunchKernelGGL(krand, dim3(grid), dim3(blk), 0, 0, (const uint32_t *)buf, (uint32_t *)out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("fetch_calib: bytes k16=k4=k1=%zu, kline lines=%zu (x128 B), krand lines=%zu\n", NB, NB / 128, NB / 128);
    hipFree(buf);
    hipFree(out);
    return 0;
}
