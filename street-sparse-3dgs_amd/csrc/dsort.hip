// dsort.hip -- the depth order of the P Gaussians: a stable LSD radix sort
// of the 32-bit depth keys with the tile-count scan and the depth-order gather fused in.
//
// Upstream sorts K (tile << 32 | depth bits) keys; this build sorts only the P depth keys
// (binning.hip derives every tile's (depth, id) list from this order) and does it with its own
// onesweep-style kernels instead of a library sort, because at P ~ 1M the library's per-pass
// launches, memsets and lookback resets cost more than the data movement (~0.17 ms vs ~8 MB
// per pass):
//
//   dsort_upsweep   one read of the keys and tile counts: the four 8-bit digit histograms
//                   (global, for every pass) and the exclusive scan of tiles_touched in Gaussian
//                   order (chained single-pass scan) -> rec[g].off, K = the total.  K is also
//                   stored straight into pinned host memory, so the host can size the binning
//                   buffer while the sort passes still run.
//   dsort_pass x4   per 8192-key tile (1024 threads, 8 keys each, wave-striped so that wave,
//                   item, lane order is the input order): match-mask ranking (8 ballots per key)
//                   into per-wave LDS counters, block digit scan, decoupled lookback per digit
//                   over the preceding tiles, the tile reordered through LDS by digit, coalesced
//                   stores.  Pass 0 takes the Gaussian index as the value (no id array); the last
//                   pass writes the order plus each slot's tile rect and count (the depth gather).
//
// Stability: every pass ranks equal digits in input order, so equal depth bits keep Gaussian-id
// order -- upstream's key (depth bits, then the stable sort's index order).  Culled Gaussians
// carry key 0xFFFFFFFF and end up behind every visible one.
//
// Control words (zeroed by the preprocess kernel, which runs first on the same stream):
// tickets (one per kernel: tiles are numbered in start order, so a tile only ever waits for
// tiles that are already running), the 4 x 256 histograms, K, the scan's per-tile status and
// the per-pass, per-tile, per-digit lookback status (count | flag << 30).
#include "gsr_launch.h"

namespace gsr {

namespace {

constexpr int kDsThreads = 1024;
constexpr int kDsWaves = kDsThreads / kWave;
constexpr int kDsItems = 8;
constexpr int kDsTile = kDsThreads * kDsItems;
constexpr int kRadix = 256;
constexpr int kPasses = 4;

// control word offsets
constexpr int kCtlTicket = 0;                  // [0] upsweep, [1 + p] pass p
constexpr int kCtlHist = 8;                    // [kPasses][kRadix]
constexpr int kCtlK = kCtlHist + kPasses * kRadix;
constexpr int kCtlErr = kCtlK + 1;             // set when a bounded spin gave up (never expected)
constexpr int kCtlScan = kCtlK + 8;            // [nb] u64 scan status (8-B aligned)
constexpr int kSpinLimit = 1 << 20;            // ~1 s of polling: a predecessor tile can never take that long
__host__ __device__ inline size_t ctl_pass(int nb, int p) { return kCtlScan + 2 * (size_t)nb + (size_t)p * nb * kRadix; }

// Diagnostic build only (tools/dsort_bench.hip): per-workgroup phase stamps of s_memrealtime
// (100 MHz) into g_ds_trace[(kernel * 4096 + block) * 8 + slot].
#ifdef GSR_DS_TRACE
__device__ uint64_t *g_ds_trace;
#define DS_STAMP(kern, slot)                                                                          \
    do {                                                                                              \
        if (threadIdx.x == 0) {                                                                       \
            const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                     \
            __builtin_amdgcn_s_waitcnt(0xC07F);                                                       \
            if (blockIdx.x < 4096) g_ds_trace[((size_t)(kern) * 4096 + blockIdx.x) * 8 + (slot)] = t_; \
        }                                                                                             \
    } while (0)
#else
#define DS_STAMP(kern, slot) \
    do {                     \
    } while (0)
#endif

constexpr uint32_t kFlagAgg = 1u << 30, kFlagInc = 2u << 30, kCountMask = (1u << 30) - 1u;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// lanes of `valid` whose 8-bit digit equals this lane's
__device__ __forceinline__ uint64_t match8(uint32_t d, uint64_t valid) {
    uint64_t m = valid;
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// Exclusive scan of 256 LDS counters in place by one wave (4 per lane); returns the total.
__device__ __forceinline__ uint32_t scan256_wave(uint32_t *a, int lane) {
    const uint32_t x0 = a[4 * lane], x1 = a[4 * lane + 1], x2 = a[4 * lane + 2], x3 = a[4 * lane + 3];
    const uint32_t s = x0 + x1 + x2 + x3;
    const uint32_t incl = wave_incl_scan(s, lane);
    const uint32_t e = incl - s;
    a[4 * lane] = e;
    a[4 * lane + 1] = e + x0;
    a[4 * lane + 2] = e + x0 + x1;
    a[4 * lane + 3] = e + x0 + x1 + x2;
    return (uint32_t)__shfl((int)incl, 63, 64);
}

__global__ __launch_bounds__(kDsThreads) void dsort_upsweep_kernel(int P, int nb, const uint32_t *__restrict__ keys,
                                                                    const uint32_t *__restrict__ tiles,
                                                                    GRec *__restrict__ rec, uint32_t *__restrict__ ctl,
                                                                    uint32_t *__restrict__ host_K) {
    __shared__ uint32_t s_hist[kPasses * kRadix];
    __shared__ uint32_t s_wsum[kDsWaves];
    __shared__ uint32_t s_v, s_prefix;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    DS_STAMP(0, 0);
    s_hist[t] = 0u;
    if (t == 0) s_v = atomicAdd(&ctl[kCtlTicket], 1u);
    __syncthreads();
    const uint32_t v = s_v;
    if (v >= (uint32_t)nb) return;  // control words not zeroed: never index past P
    const size_t base = (size_t)v * kDsTile + (size_t)w * kDsItems * kWave;
    uint32_t key[kDsItems], tl[kDsItems];
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const size_t e = base + (size_t)k * kWave + lane;
        key[k] = e < (size_t)P ? keys[e] : 0u;
        tl[k] = e < (size_t)P ? tiles[e] : 0u;
    }
    // digit histograms of all passes: one LDS add per (wave, distinct digit)
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const size_t e = base + (size_t)k * kWave + lane;
        const bool valid = e < (size_t)P;
        const uint64_t vm = __ballot(valid);
        if (vm == 0ull) break;
#pragma unroll
        for (int p = 0; p < kPasses; p++) {
            const uint32_t d = (key[k] >> (8 * p)) & 0xFFu;
            const uint64_t m = match8(d, vm);
            if (valid && below(m) == 0u) atomicAdd(&s_hist[p * kRadix + d], (uint32_t)__popcll(m));
        }
    }
    // tiles_touched: exclusive offsets inside the wave's 512 keys (wave-major, item, lane order)
    uint32_t off[kDsItems], run = 0;
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const uint32_t incl = wave_incl_scan(tl[k], lane);
        off[k] = run + incl - tl[k];
        run += (uint32_t)__shfl((int)incl, 63, 64);
    }
    if (lane == 0) s_wsum[w] = run;
    __syncthreads();
    DS_STAMP(0, 1);
    {
        const uint32_t c = s_hist[t];
        if (c) atomicAdd(&ctl[kCtlHist + t], c);
    }
    if (w == 0) {
        const uint32_t x = lane < kDsWaves ? s_wsum[lane] : 0u;
        const uint32_t incl = wave_incl_scan(x, lane);
        if (lane < kDsWaves) s_wsum[lane] = incl - x;
        const uint32_t total = (uint32_t)__shfl((int)incl, 63, 64);
        if (lane == 0) {
            // chained scan over tiles: publish the aggregate, walk back to an inclusive prefix
            uint64_t *st = reinterpret_cast<uint64_t *>(ctl + kCtlScan);
            uint32_t prefix = 0;
            if (v == 0) {
                st_agent64(&st[0], (2ull << 32) | total);
            } else {
                st_agent64(&st[v], (1ull << 32) | total);
                int spins = 0;
                for (int j = (int)v - 1; j >= 0;) {
                    const uint64_t s = ld_agent64(&st[j]);
                    const uint32_t f = (uint32_t)(s >> 32);
                    if (f == 0u) {
                        if (++spins > kSpinLimit) {
                            ctl[kCtlErr] = 1u;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    prefix += (uint32_t)s;
                    if (f == 2u) break;
                    j--;
                }
                st_agent64(&st[v], (2ull << 32) | (uint64_t)(prefix + total));
            }
            s_prefix = prefix;
            if (v == (uint32_t)nb - 1u) {
                ctl[kCtlK] = prefix + total;
                if (host_K) __hip_atomic_store(host_K, prefix + total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    __syncthreads();
    DS_STAMP(0, 2);
    const uint32_t pre = s_prefix + s_wsum[w];
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const size_t e = base + (size_t)k * kWave + lane;
        if (e < (size_t)P && tl[k] > 0u) rec[e].off = pre + off[k];
    }
    DS_STAMP(0, 3);
}

template <int kPass>
__global__ __launch_bounds__(kDsThreads) void dsort_pass_kernel(int P, int nb, const uint32_t *__restrict__ kin,
                                                                 uint32_t *__restrict__ kout,
                                                                 const uint32_t *__restrict__ vin,
                                                                 uint32_t *__restrict__ vout, uint32_t *__restrict__ ctl,
                                                                 const GRec *__restrict__ rec,
                                                                 const uint32_t *__restrict__ tiles,
                                                                 uint2 *__restrict__ drect, uint32_t *__restrict__ dtiles) {
    constexpr bool kLast = kPass == kPasses - 1;
    constexpr int kShift = 8 * kPass;
    __shared__ uint32_t s_key[kDsTile];
    __shared__ uint32_t s_val[kDsTile];
    __shared__ uint32_t s_wh[kDsWaves][kRadix];  // per-wave digit counts -> exclusive prefix over waves
    __shared__ uint32_t s_gb[kRadix];            // global digit base
    __shared__ uint32_t s_bex[kRadix];           // tile-local digit base
    __shared__ uint32_t s_dst[kRadix];           // global slot of tile-local position 0 of each digit
    __shared__ uint32_t s_v;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    DS_STAMP(1 + kPass, 0);
#pragma unroll
    for (int k = 0; k < kDsWaves * kRadix / kDsThreads; k++) (&s_wh[0][0])[t + k * kDsThreads] = 0u;
    if (t < kRadix) s_gb[t] = ctl[kCtlHist + kPass * kRadix + t];
    if (t == 0) s_v = atomicAdd(&ctl[kCtlTicket + 1 + kPass], 1u);
    __syncthreads();
    const uint32_t v = s_v;
    if (v >= (uint32_t)nb) return;  // control words not zeroed: never index past P
    const size_t tile0 = (size_t)v * kDsTile;
    const int n = (int)min((size_t)kDsTile, (size_t)P - tile0);
    const int wbase = w * kDsItems * kWave;
    uint32_t key[kDsItems], val[kDsItems];
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const int i = wbase + k * kWave + lane;
        const bool valid = i < n;
        key[k] = valid ? kin[tile0 + i] : 0xFFFFFFFFu;
        val[k] = kPass == 0 ? (uint32_t)(tile0 + i) : (valid ? vin[tile0 + i] : 0u);
    }
    if (w == 0) (void)scan256_wave(s_gb, lane);
    // ranks: within the wave, equal digits in (item, lane) order
    uint32_t rk[kDsItems];
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const int i = wbase + k * kWave + lane;
        const bool valid = i < n;
        const uint64_t vm = __ballot(valid);
        const uint32_t d = (key[k] >> kShift) & 0xFFu;
        const uint64_t m = match8(d, vm);
        const uint32_t b = below(m);
        const uint32_t old = s_wh[w][d];
        if (valid && b == 0u) s_wh[w][d] = old + (uint32_t)__popcll(m);
        rk[k] = old + b;
    }
    __syncthreads();
    DS_STAMP(1 + kPass, 1);
    uint32_t cnt = 0;
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < kDsWaves; ww++) {
            const uint32_t c = s_wh[ww][t];
            s_wh[ww][t] = cnt;
            cnt += c;
        }
        uint32_t *st = ctl + ctl_pass(nb, kPass);
        st_agent(&st[(size_t)v * kRadix + t], (v == 0 ? kFlagInc : kFlagAgg) | cnt);
        s_bex[t] = cnt;
    }
    __syncthreads();
    if (w == 0) (void)scan256_wave(s_bex, lane);
    __syncthreads();
    DS_STAMP(1 + kPass, 2);
    // the tile in digit order, through LDS
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const int i = wbase + k * kWave + lane;
        if (i < n) {
            const uint32_t d = (key[k] >> kShift) & 0xFFu;
            const uint32_t lp = s_bex[d] + s_wh[w][d] + rk[k];
            s_key[lp] = key[k];
            s_val[lp] = val[k];
        }
    }
    if (t < kRadix) {
        // decoupled lookback for digit t over the preceding tiles
        uint32_t *st = ctl + ctl_pass(nb, kPass);
        uint32_t excl = 0;
        if (v > 0) {
            int spins = 0;
            for (int j = (int)v - 1; j >= 0;) {
                const uint32_t s = ld_agent(&st[(size_t)j * kRadix + t]);
                if ((s & ~kCountMask) == 0u) {
                    if (++spins > kSpinLimit) {
                        ctl[kCtlErr] = 1u;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += s & kCountMask;
                if ((s & ~kCountMask) == kFlagInc) break;
                j--;
            }
            st_agent(&st[(size_t)v * kRadix + t], kFlagInc | (excl + cnt));
        }
        s_dst[t] = s_gb[t] + excl - s_bex[t];
    }
    __syncthreads();
    DS_STAMP(1 + kPass, 3);
    for (int i = t; i < n; i += kDsThreads) {
        const uint32_t k = s_key[i];
        const uint32_t j = s_dst[(k >> kShift) & 0xFFu] + (uint32_t)i;
        const uint32_t g = s_val[i];
        if (kLast) {
            vout[j] = g;
            const uint32_t area = tiles[g];
            uint2 r = make_uint2(0u, 0u);
            if (area > 0) {
                const uint4 q3 = reinterpret_cast<const uint4 *>(rec + g)[3];
                const uint32_t wd = q3.y, x0 = q3.x & 0xFFFFu, y0 = q3.x >> 16;
                r = make_uint2(q3.x, (x0 + wd) | ((y0 + area / wd) << 16));
            }
            drect[j] = r;
            dtiles[j] = area;
        } else {
            kout[j] = k;
            vout[j] = g;
        }
    }
    DS_STAMP(1 + kPass, 4);
}

}  // namespace

int dsort_blocks(int P) { return (P + kDsTile - 1) / kDsTile; }

size_t dsort_ctrl_words(int P) {
    const int nb = dsort_blocks(P) > 0 ? dsort_blocks(P) : 1;
    return ctl_pass(nb, kPasses);
}

void launch_depth_sort(int P, const GeomState &gs, uint32_t *host_K, hipStream_t s, hipEvent_t k_ready) {
    if (P == 0) return;
    const int nb = dsort_blocks(P);
    hipLaunchKernelGGL(dsort_upsweep_kernel, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.tiles, gs.rec, gs.ctrl,
                       host_K);
    if (k_ready) (void)hipEventRecord(k_ready, s);
    // keys: dkey -> dkey_sorted -> dkey -> dkey_sorted -> (none); values: (index) -> ids -> order -> ids -> order
    hipLaunchKernelGGL(dsort_pass_kernel<0>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted,
                       (const uint32_t *)nullptr, gs.ids, gs.ctrl, gs.rec, gs.tiles, gs.drect, gs.dtiles);
    hipLaunchKernelGGL(dsort_pass_kernel<1>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted, gs.dkey, gs.ids,
                       gs.order, gs.ctrl, gs.rec, gs.tiles, gs.drect, gs.dtiles);
    hipLaunchKernelGGL(dsort_pass_kernel<2>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted, gs.order,
                       gs.ids, gs.ctrl, gs.rec, gs.tiles, gs.drect, gs.dtiles);
    hipLaunchKernelGGL(dsort_pass_kernel<3>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted,
                       (uint32_t *)nullptr, gs.ids, gs.order, gs.ctrl, gs.rec, gs.tiles, gs.drect, gs.dtiles);
}

uint32_t *dsort_K_word(const GeomState &gs) { return gs.ctrl + kCtlK; }
uint32_t *dsort_err_word(const GeomState &gs) { return gs.ctrl + kCtlErr; }

}  // namespace gsr
