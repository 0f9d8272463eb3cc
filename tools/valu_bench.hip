// valu_bench.hip -- issue rate of v_fma_f32 vs v_pk_fma_f32 (and v_exp_f32) on gfx950.
// Every thread runs 8 independent FMA chains for N iterations; each kernel reports
// G wave-instructions/s and fp32 FMA lanes/s.  Build: hipcc --offload-arch=gfx950 -O3 valu_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(256) void fma_scalar(float *out, int n, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < n; i++) {
        asm volatile(
            "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
            "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(a), "v"(b));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void fma_packed(float *out, int n, float a, float b) {
    f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6,
       x7 = x0 + 7;
    f2 A = {a, a}, B = {b, b};
    for (int i = 0; i < n; i++) {
        asm volatile(
            "v_pk_fma_f32 %0, %0, %8, %9\n v_pk_fma_f32 %1, %1, %8, %9\n v_pk_fma_f32 %2, %2, %8, %9\n v_pk_fma_f32 %3, %3, %8, %9\n"
            "v_pk_fma_f32 %4, %4, %8, %9\n v_pk_fma_f32 %5, %5, %8, %9\n v_pk_fma_f32 %6, %6, %8, %9\n v_pk_fma_f32 %7, %7, %8, %9\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(A), "v"(B));
    }
    f2 s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y;
}

__global__ __launch_bounds__(256) void exp_scalar(float *out, int n, float a, float b) {
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < n; i++) {
        asm volatile(
            "v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n"
            "v_exp_f32 %4, %4\n v_exp_f32 %5, %5\n v_exp_f32 %6, %6\n v_exp_f32 %7, %7\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + a + b;
}

// 4 fma + 1 exp per group of 5: interleaved with the transcendental
__global__ __launch_bounds__(256) void fma_exp_mix(float *out, int n, float a, float b) {
    float x0 = threadIdx.x * 1e-3f, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    float e0 = x0, e1 = x1;
    for (int i = 0; i < n; i++) {
        asm volatile(
            "v_fma_f32 %0, %0, %10, %11\n v_fma_f32 %1, %1, %10, %11\n v_fma_f32 %2, %2, %10, %11\n v_fma_f32 %3, %3, %10, %11\n"
            "v_exp_f32 %8, %8\n"
            "v_fma_f32 %4, %4, %10, %11\n v_fma_f32 %5, %5, %10, %11\n v_fma_f32 %6, %6, %10, %11\n v_fma_f32 %7, %7, %10, %11\n"
            "v_exp_f32 %9, %9\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7), "+v"(e0), "+v"(e1)
            : "v"(a), "v"(b));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + e0 + e1;
}

template <typename K>
int run(const char *name, K kern, float *d, int blocks, int n, int instr_per_iter, int lanes_per_instr) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, n, 0.999f, 0.001f);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, n, 0.999f, 0.001f);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const double waves = (double)blocks * 4 * 5;
    const double instr = waves * (double)n * instr_per_iter;
    printf("%-12s %8.3f ms  %8.1f G wave-instr/s  %8.2f T lane-ops/s\n", name, ms, instr / (ms * 1e-3) / 1e9,
           instr * 64 * lanes_per_instr / (ms * 1e-3) / 1e12);
    return 0;
}

int main() {
    const int blocks = 256 * 8 * 4;  // 8 waves per SIMD
    const int n = 4096;
    float *d;
    CHECK(hipMalloc(&d, sizeof(float) * blocks * 256));
    run("fma_f32", fma_scalar, d, blocks, n, 8, 1);
    run("pk_fma_f32", fma_packed, d, blocks, n, 8, 2);
    run("exp_f32", exp_scalar, d, blocks, n, 8, 1);
    run("fma+exp 8:2", fma_exp_mix, d, blocks, n, 10, 1);
    run("fma_f32", fma_scalar, d, blocks, n, 8, 1);
    run("pk_fma_f32", fma_packed, d, blocks, n, 8, 2);
    CHECK(hipFree(d));
    return 0;
}
