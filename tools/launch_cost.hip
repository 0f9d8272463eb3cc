// Host cost of the HIP calls a rasterizer frame issues (run ON the GPU box):
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o /tmp/launch_cost && /tmp/launch_cost
// Per call, averaged over 2000: an empty kernel launch with 1 / 24 arguments (64 / 256 / 1024
// threads per block, small / large grids), hipEventRecord, hipStreamWaitEvent across two streams,
// hipGetDevice, hipGetLastError, hipStreamQuery, and the same launches while the stream is busy.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k1(int *p) {
    if (p && threadIdx.x == 1000000) p[0] = 1;
}
__global__ void k24(int *a, int *b, int *c, int *d, int *e, int *f, int g, int h, int i, int j, float k, float l,
                    float m, float n, int *o, int *q, int *r, int *s, unsigned t, unsigned u, unsigned v, unsigned w,
                    int *x, int *y) {
    if (a && threadIdx.x == 1000000) a[0] = g + h + i + j + (int)(k + l + m + n) + (int)(t + u + v + w);
}
__global__ void spin(unsigned long long cycles) {
    const unsigned long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
}

template <class F>
double per_call_us(F f, int n = 2000) {
    for (int i = 0; i < 50; i++) f();
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) f();
    const auto t1 = std::chrono::steady_clock::now();
    (void)hipDeviceSynchronize();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

int main() {
    hipStream_t s, s2;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    int *p = nullptr;
    (void)hipMalloc(&p, 4096);
    printf("launch 1 arg, 1x64:        %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k1, dim3(1), dim3(64), 0, s, p); }));
    printf("launch 1 arg, 8160x256:    %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k1, dim3(8160), dim3(256), 0, s, p); }));
    printf("launch 24 args, 8160x256:  %.2f us\n", per_call_us([&] {
               hipLaunchKernelGGL(k24, dim3(8160), dim3(256), 0, s, p, p, p, p, p, p, 1, 2, 3, 4, 1.f, 2.f, 3.f, 4.f, p,
                                  p, p, p, 1u, 2u, 3u, 4u, p, p);
           }));
    printf("launch 1 arg, 123x1024:    %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k1, dim3(123), dim3(1024), 0, s, p); }));
    printf("hipEventRecord:            %.2f us\n", per_call_us([&] { (void)hipEventRecord(ev, s); }));
    printf("record + wait (2 streams): %.2f us\n", per_call_us([&] {
               (void)hipEventRecord(ev, s);
               (void)hipStreamWaitEvent(s2, ev, 0);
           }));
    int d;
    printf("hipGetDevice:              %.3f us\n", per_call_us([&] { (void)hipGetDevice(&d); }, 20000));
    printf("hipGetLastError:           %.3f us\n", per_call_us([&] { (void)hipGetLastError(); }, 20000));
    printf("hipStreamQuery:            %.3f us\n", per_call_us([&] { (void)hipStreamQuery(s); }, 2000));
    // the same launches behind a busy stream (the host runs ahead of the GPU in a training loop)
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 2400ull * 1000 * 200);  // ~200 ms
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 1000; i++) hipLaunchKernelGGL(k1, dim3(8160), dim3(256), 0, s, p);
    const auto t1 = std::chrono::steady_clock::now();
    printf("launch behind a busy stream: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 1000);
    (void)hipDeviceSynchronize();
    // device time per empty launch back to back (the GPU-side gap a launch costs)
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < 1000; i++) hipLaunchKernelGGL(k1, dim3(8160), dim3(256), 0, s, p);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("device time per empty 8160x256 launch: %.2f us\n", ms);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < 1000; i++) hipLaunchKernelGGL(k1, dim3(1), dim3(64), 0, s, p);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
    printf("device time per empty 1x64 launch: %.2f us\n", ms);
    return 0;
}
