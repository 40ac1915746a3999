// Seeding and chaining on the GPU: seed_core.h's map_read, one
// lane per short read, each lane working in its own slice of a global scratch
// buffer (seedc::carve, seedc::device_caps).  The index (text, 12-mer hit lists
// with the 28 bases after every hit, count tables) is resident in HBM.  A read
// whose work outgrows the lane's scratch is reported with its SC_OVER_* flags
// and no tasks; the host decides what to do with it.
//
// Per lane: the read's occurrence table (the 12-mer lists of its ~140 starts:
// contiguous kpos/kext segments), the SMEM / re-seeding / -y passes over that
// table, chaining into a sorted chain array with a seed pool, the chain filter
// and the task output.  Latency-bound, irregular integer work: the lanes of a
// wave follow different reads, so the kernel relies on many resident waves.
#include <hip/hip_runtime.h>

#include "seed_core.h"
#include "seed_dev.h"

namespace prgpu {

__global__ void __launch_bounds__(64) seed_map_kernel(SeedDev D) {
    const int64_t lane = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nl = (int64_t)gridDim.x * blockDim.x;
    if (lane >= D.n_lanes) return;
    seedc::Scratch S = seedc::carve(D.scratch + lane * D.stride, D.caps);
    for (int64_t i = lane; i < D.n_sr; i += nl) {
        const int64_t o = D.sr_off[i];
        const int len = (int)(D.sr_off[i + 1] - o);
        int n = 0, err = 0;
        if (len > 0)
            err = seedc::map_read(D.V, D.O, S, D.sr_seq + o, len, (int)i, D.out + i * D.caps.out, D.caps.out, &n);
        D.n_out[i] = err ? 0 : n;
        D.status[i] = err;
    }
}

int seed_launch(const SeedDev &D, void *stream) {
    if (D.n_sr <= 0) return 0;
    const int64_t blocks = (D.n_lanes + 63) / 64;
    hipLaunchKernelGGL(seed_map_kernel, dim3((unsigned)blocks), dim3(64), 0, (hipStream_t)stream, D);
    return (int)hipGetLastError();
}

}  // namespace prgpu
