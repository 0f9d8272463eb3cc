// dsort_bench.hip -- standalone measurement harness for the depth sort (csrc/dsort.hip), built
// as one translation unit with the kernels (diagnostic stamps on):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DGSR_DS_TRACE \
//         -I street-sparse-3dgs_amd/csrc -I include tools/dsort_bench.hip -o tools/dsort_bench
//   tools/dsort_bench [P] [iters]
// Synthetic keys: view depths z ~ U[2, 20] as float bits, 2% culled (0xFFFFFFFF); tile counts
// 1..32; 8-B tile rects (rect4 unset: pass 3 gathers them, no rect carry).  Checks the order against std::stable_sort, the record offsets and K, then prints the
// per-kernel HIP-event times and the per-workgroup phase stamps (median / max over workgroups,
// relative to the kernel's first workgroup start).
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#include "dsort.hip"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

using namespace gsr;

int main(int argc, char **argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 1000000;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> uz(2.f, 20.f);
    std::uniform_int_distribution<int> ut(1, 32);
    std::vector<uint32_t> key(P), tiles(P);
    std::vector<GRec> rec(P);
    for (int i = 0; i < P; i++) {
        const float z = uz(rng);
        const bool culled = (rng() % 50) == 0;
        key[i] = culled ? 0xFFFFFFFFu : __builtin_bit_cast(uint32_t, z);
        tiles[i] = culled ? 0u : (uint32_t)ut(rng);
        rec[i] = GRec{};
        rec[i].rect0 = (uint32_t)(i % 100) | ((uint32_t)(i % 60) << 16);
        rec[i].rectw = 1;
    }
    GeomState gs{};
    CK(hipMalloc(&gs.rec, sizeof(GRec) * P));
    CK(hipMalloc(&gs.tiles, 4 * (size_t)P));
    CK(hipMalloc(&gs.dkey, 4 * (size_t)P));
    CK(hipMalloc(&gs.dkey_sorted, 4 * (size_t)P));
    CK(hipMalloc(&gs.ids, 4 * (size_t)P));
    CK(hipMalloc(&gs.order, 4 * (size_t)P));
    CK(hipMalloc(&gs.offsets, 4 * (size_t)P));
    CK(hipMalloc(&gs.drect, 8 * (size_t)P));
    CK(hipMalloc(&gs.rect8, 8 * (size_t)P));
    const size_t ctrl_words = dsort_ctrl_words(P);
    gs.ctrl_zero = (uint32_t)dsort_ctrl_zero_words(P);
    CK(hipMalloc(&gs.ctrl, 4 * ctrl_words));
    uint64_t *trace = nullptr;
    CK(hipMalloc(&trace, 8ull * 5 * 4096 * 8));
#ifdef GSR_DS_TRACE
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ds_trace), &trace, sizeof(trace)));
#endif
    CK(hipMemcpy(gs.rec, rec.data(), sizeof(GRec) * P, hipMemcpyHostToDevice));
    CK(hipMemcpy(gs.tiles, tiles.data(), 4 * (size_t)P, hipMemcpyHostToDevice));
    std::vector<uint2> r8(P);
    for (int i = 0; i < P; i++) r8[i] = tiles[i] ? make_uint2(i % 100, i % 60) : make_uint2(0u, 0u);
    CK(hipMemcpy(gs.rect8, r8.data(), 8 * (size_t)P, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t ev[7];
    for (auto &e : ev) CK(hipEventCreate(&e));
    const int nb = dsort_blocks(P);
    double tk[6] = {0};
    for (int it = 0; it < iters + 2; it++) {
        CK(hipMemcpyAsync(gs.dkey, key.data(), 4 * (size_t)P, hipMemcpyHostToDevice, s));
        CK(hipMemsetAsync(gs.ctrl, 0, 4 * (size_t)gs.ctrl_zero, s));
        CK(hipMemsetAsync(trace, 0, 8ull * 5 * 4096 * 8, s));
        CK(hipEventRecord(ev[0], s));
        hipLaunchKernelGGL(dsort_upsweep_kernel, dim3(up_blocks(nb)), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.tiles, gs.ctrl,
                           (uint32_t *)nullptr);
        CK(hipEventRecord(ev[1], s));
        hipLaunchKernelGGL(dsort_pass_kernel<0>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted,
                           (const uint32_t *)nullptr, gs.ids, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, (const uint32_t *)nullptr, gs.drect,
                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
        CK(hipEventRecord(ev[2], s));
        hipLaunchKernelGGL(dsort_pass_kernel<1>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted, gs.dkey,
                           gs.ids, gs.order, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, (const uint32_t *)nullptr, gs.drect,
                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
        CK(hipEventRecord(ev[3], s));
        hipLaunchKernelGGL(dsort_pass_kernel<2>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted,
                           gs.order, gs.ids, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, (const uint32_t *)nullptr, gs.drect,
                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
        CK(hipEventRecord(ev[4], s));
        hipLaunchKernelGGL(dsort_pass_kernel<3>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted,
                           (uint32_t *)nullptr, gs.ids, gs.order, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, (const uint32_t *)nullptr, gs.drect,
                           (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
        CK(hipEventRecord(ev[5], s));
        CK(hipStreamSynchronize(s));
        if (it >= 2)
            for (int k = 0; k < 5; k++) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
                tk[k] += ms;
            }
    }
    // correctness
    std::vector<uint32_t> order(P), want(P);
    std::vector<uint32_t> offs(P);
    CK(hipMemcpy(order.data(), gs.order, 4 * (size_t)P, hipMemcpyDeviceToHost));
    CK(hipMemcpy(offs.data(), gs.offsets, 4 * (size_t)P, hipMemcpyDeviceToHost));
    std::iota(want.begin(), want.end(), 0u);
    std::stable_sort(want.begin(), want.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b]; });
    size_t bad = 0;
    for (int i = 0; i < P; i++) bad += order[i] != want[i];
    uint64_t run = 0, badoff = 0;
    for (int i = 0; i < P; i++)
        if (tiles[i]) {
            badoff += offs[i] != run;
            run += tiles[i];
        }
    uint32_t K = 0;
    CK(hipMemcpy(&K, dsort_K_word(gs), 4, hipMemcpyDeviceToHost));
    std::vector<uint2> dr(P);
    CK(hipMemcpy(dr.data(), gs.drect, 8 * (size_t)P, hipMemcpyDeviceToHost));
    for (int i = 0; i < P; i++) bad += dr[i].x != r8[want[i]].x || dr[i].y != r8[want[i]].y;
    printf("P=%d blocks=%d  order mismatches=%zu  offset mismatches=%llu  K=%u (want %llu)\n", P, nb, bad,
           (unsigned long long)badoff, K, (unsigned long long)run);
    const char *names[5] = {"upsweep", "pass0", "pass1", "pass2", "pass3"};
    for (int k = 0; k < 5; k++) printf("%-8s %8.2f us\n", names[k], 1e3 * tk[k] / iters);
    // phase stamps of the last iteration
    std::vector<uint64_t> tr(5 * 4096 * 8);
    CK(hipMemcpy(tr.data(), trace, 8 * tr.size(), hipMemcpyDeviceToHost));
    for (int k = 0; k < 5; k++) {
        const int nslot = k == 0 ? 3 : 8;
        uint64_t t0 = ~0ull;
        const int nbk = k == 0 ? (int)up_blocks(nb) : nb;
        for (int b = 0; b < nbk && b < 4096; b++) t0 = std::min(t0, tr[((size_t)k * 4096 + b) * 8]);
        printf("%-8s", names[k]);
        for (int sl = 0; sl < nslot; sl++) {
            std::vector<double> v;
            for (int b = 0; b < nbk && b < 4096; b++) v.push_back((tr[((size_t)k * 4096 + b) * 8 + sl] - t0) * 0.01);
            std::sort(v.begin(), v.end());
            printf("  s%d med %6.2f max %6.2f", sl, v[v.size() / 2], v.back());
        }
        printf("  (us)\n");
    }
    return bad || badoff || K != run;
}
