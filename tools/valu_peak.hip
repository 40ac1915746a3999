// INT32 VALU peak microbenchmark (SURVEY.md §8d asks to confirm the SW roofline):
// every lane runs 16 independent chains of v_add_u32 / v_max_i32, enough waves to
// fill every SIMD; ops/s = lanes x chains x iterations x 2 / time.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) valu_kernel(int *out, int iters, int seed) {
    int a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = threadIdx.x * 7 + k * seed;
    const int c1 = seed + 3, c2 = seed - 5;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            a[k] = a[k] + c1;
            a[k] = max(a[k], c2 ^ k);
        }
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s ^= a[k];
    if (s == 0x7fffffff) out[0] = s;
}

typedef short short2_t __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(256) pk16_kernel(int *out, int iters, int seed) {
    short2_t a[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = short2_t{(short)(threadIdx.x + k), (short)(seed * k)};
    const short2_t c1 = short2_t{(short)(seed + 3), (short)(seed + 1)};
    const short2_t c2 = short2_t{(short)(seed - 5), (short)(seed - 7)};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            a[k] = a[k] + c1;                                          // v_pk_add_u16
            a[k] = __builtin_elementwise_max(a[k], c2);                // v_pk_max_i16
        }
    }
    int s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s ^= (int)a[k].x ^ ((int)a[k].y << 16);
    if (s == 0x7fffffff) out[0] = s;
}

int main() {
    int *out;
    (void)hipMalloc(&out, 4);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int blocks = p.multiProcessorCount * 8;   // 8 x 256 threads = 32 waves per CU
    const int iters = 20000;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(256), 0, 0, out, 100, 1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    const double ops = (double)blocks * 256 * iters * 16 * 2;
    hipLaunchKernelGGL(pk16_kernel, dim3(blocks), dim3(256), 0, 0, out, 100, 1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(pk16_kernel, dim3(blocks), dim3(256), 0, 0, out, iters, 1);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms16 = 0.f;
    (void)hipEventElapsedTime(&ms16, a, b);
    printf("{\"cus\": %d, \"int32\": {\"ms\": %.3f, \"ops\": %.4g, \"tops\": %.2f}, "
           "\"pk_i16\": {\"ms\": %.3f, \"instr\": %.4g, \"tops_16bit_lanes\": %.2f}}\n",
           p.multiProcessorCount, ms, ops, ops / (ms * 1e-3) / 1e12, ms16, ops, 2 * ops / (ms16 * 1e-3) / 1e12);
    return 0;
}
