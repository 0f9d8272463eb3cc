// dsort.hip -- the depth order of the P Gaussians: a stable LSD radix sort
// of the 32-bit depth keys with the tile-count scan and the depth-order gather fused in.
//
// Upstream sorts K (tile << 32 | depth bits) keys; this build sorts only the P depth keys
// (binning.hip derives every tile's (depth, id) list from this order) and does it with its own
// onesweep-style kernels instead of a library sort: at P ~ 1M the library's per-pass launches,
// memsets and lookback resets cost ~0.17 ms for ~8 MB of data movement per pass.
//
//   dsort_upsweep   one read of the keys and tile counts by <= 128 workgroups: each one's four
//                   8-bit digit histograms (LDS, written out as one row -- no global atomics on a
//                   few hot lines) and tiles_touched sums; the last workgroup to finish adds up K
//                   and stores it straight into pinned host memory, so the host sizes the binning
//                   buffer while the sort passes still run.
//   dsort_pass x4   per 8192-key tile (1024 threads, 8 keys each, wave-striped so that wave, item,
//                   lane order is the input order): the pass's global digit bases from the per-tile
//                   histograms, match-mask ranking (8 ballots per key) into per-wave LDS counters,
//                   block digit scan, decoupled lookback per digit over the preceding tiles (16
//                   predecessors per round trip), the tile reordered through LDS by digit,
//                   coalesced stores.  Pass 0 takes the Gaussian index as the value (no id array)
//                   and writes the Gaussian-major record offsets (exclusive scan of tiles_touched
//                   in index order, gs.offsets); the last pass writes the order and each slot's
//                   tile rect gathered from the preprocess's compact rect array.
//
// Stability: every pass ranks equal digits in input order, so equal depth bits keep Gaussian-id
// order -- upstream's key (depth bits, then the stable sort's index order).  Culled Gaussians
// carry key 0xFFFFFFFF and end up behind every visible one.
//
// Control words: [0, kCtlHead) tickets / counters, then the lookback status of every pass
// (count | flag << 30) -- zeroed by the preprocess kernel, which runs first on the same stream --
// then the upsweep's tile offsets, workgroup totals and histogram rows (fully written by it).
#include "gsr_launch.h"

namespace gsr {

namespace {

constexpr int kDsThreads = 1024;
constexpr int kDsWaves = kDsThreads / kWave;
constexpr int kDsItems = 8;
constexpr int kDsTile = kDsThreads * kDsItems;
constexpr int kRadix = 256;
constexpr int kPasses = 4;
constexpr int kLookWin = 16;
constexpr int kMaxResident = 240;  // tiles numbered by blockIdx.x up to this many (< CUs)

// control word offsets
constexpr int kCtlTicket = 0;  // [p] pass p
constexpr int kCtlDone = 4;    // upsweep tiles finished
constexpr int kCtlK = 5;       // sum of tiles_touched
constexpr int kCtlErr = 6;     // set when a bounded spin gave up (never expected)
constexpr int kCtlAux = 7;     // per-frame counter lent to the binning (sb_colscan's last-workgroup count)
constexpr int kCtlMaxSB = 8;   // local-sort frames: the longest SB list (sb_colscan)
constexpr int kCtlFwdReady = 9;  // the forward split's queue released by tile_order (workers launched ahead)
constexpr int kCtlLongest = 10;  // [2]: the frame's longest tile list and superblock list (split gate hints)
constexpr int kCtlCulled = 12;   // culled Gaussians (key 0xFFFFFFFF): the depth order's last P - visible slots
constexpr int kCtlLive = 13;     // [2]: the backward's live-row list length and finished workgroups (backward.hip;
                                 // zeroed again by grad_live_kernel's last workgroup)
constexpr int kCtlHead = 16;
// The upsweep runs at most kUpMax workgroups, each over tpb consecutive tiles, so that a pass
// reduces at most kUpMax histogram rows (kUpMax / 4 loads per thread, all in flight at once).
constexpr int kUpMax = 128;
__host__ __device__ inline int up_tpb(int nb) { return (nb + kUpMax - 1) / kUpMax; }
__host__ __device__ inline int up_blocks(int nb) { return (nb + up_tpb(nb) - 1) / up_tpb(nb); }
__host__ __device__ inline size_t ctl_status(int nb, int p) { return kCtlHead + (size_t)p * nb * kRadix; }
__host__ __device__ inline size_t ctl_zero_words(int nb) { return ctl_status(nb, kPasses); }
__host__ __device__ inline size_t ctl_bex(int nb) { return ctl_zero_words(nb); }              // [nb]
__host__ __device__ inline size_t ctl_btot(int nb) { return ctl_bex(nb) + nb; }               // [kUpMax]
__host__ __device__ inline size_t ctl_blkhist(int nb) { return (ctl_btot(nb) + kUpMax + 63) / 64 * 64; }
__host__ __device__ inline size_t ctl_words(int nb) { return ctl_blkhist(nb) + (size_t)kUpMax * kPasses * kRadix; }
constexpr int kSpinLimit = 1 << 20;  // ~1 s of polling: a predecessor tile can never take that long

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
#ifdef GSR_DS_TRACE
#define DS_STAMP_AFTER(kern, slot, x)            \
    do {                                         \
        asm volatile("s_waitcnt vmcnt(0)" ::"v"(x)); \
        DS_STAMP(kern, slot);                    \
    } while (0)
#else
#define DS_STAMP_AFTER(kern, slot, x) DS_STAMP(kern, slot)
#endif

// GSR_DSORT_CARRY: with 4-B rects, the tile rect travels with the Gaussian id through the four
// passes (read coalesced by pass 0 in index order, ping-ponged through the idle rect8 array), so
// pass 3 stores it instead of gathering rect4[id] -- one random 64-B line per Gaussian.
#ifndef GSR_DSORT_CARRY
#define GSR_DSORT_CARRY 1
#endif

constexpr uint32_t kFlagAgg = 1u << 30, kFlagInc = 2u << 30, kCountMask = (1u << 30) - 1u;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint32_t *p, uint32_t v) {
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

// Per workgroup u: tiles [u tpb, (u + 1) tpb): the digit histograms of all passes over its tiles
// (one LDS add per key and pass; conflicts only where a wave's digits coincide) -> histogram row
// u; the tiles_touched sum of each tile -> its exclusive offset inside the workgroup (bex) and the
// workgroup total (btot); K = the sum of the totals, stored by the last workgroup to finish.
__global__ __launch_bounds__(kDsThreads) void dsort_upsweep_kernel(int P, int nb, const uint32_t *__restrict__ keys,
                                                                    const uint32_t *__restrict__ tiles,
                                                                    uint32_t *__restrict__ ctl,
                                                                    uint32_t *__restrict__ host_K) {
    GSR_KS(kKsUpsweep);
    // the top digit (sign + exponent + 1 mantissa bit) takes a handful of values: its counters are
    // replicated 16x (lane & 15 picks the copy) so a wave's LDS adds collide at most 4 ways
    constexpr int kTopCopies = 16;
    __shared__ uint32_t s_hist[kPasses * kRadix];
    __shared__ uint32_t s_top[kTopCopies][kRadix];
    // the third digit (exponent bit 0 + 7 mantissa bits) repeats inside a wave when neighbouring rows
    // have similar depths (rows in spatial order, gs_train.chunk.reorder_rows: 64-way conflicts,
    // config-3 upsweep 15.5 -> 25.0 us per call): replicated the same way
    __shared__ uint32_t s_mid[kTopCopies][kRadix];
    __shared__ uint32_t s_wsum[kDsWaves];
    __shared__ uint32_t s_cull;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int u = blockIdx.x, tpb = up_tpb(nb);
    DS_STAMP(0, 0);
    s_hist[t] = 0u;
    if (t == 0) s_cull = 0u;
#pragma unroll
    for (int k = 0; k < kTopCopies * kRadix / kDsThreads; k++) {
        (&s_top[0][0])[t + k * kDsThreads] = 0u;
        (&s_mid[0][0])[t + k * kDsThreads] = 0u;
    }
    __syncthreads();
    uint32_t run = 0;  // thread 0: tiles_touched of the workgroup's earlier tiles
    uint32_t culled = 0;  // this wave's culled keys (wave-uniform)
    const int v1 = min(nb, (u + 1) * tpb);
    for (int v = u * tpb; v < v1; v++) {
        const size_t base = (size_t)v * kDsTile + (size_t)w * kDsItems * kWave;
        uint32_t key[kDsItems], tl[kDsItems];
#pragma unroll
        for (int k = 0; k < kDsItems; k++) {
            const size_t e = base + (size_t)k * kWave + lane;
            key[k] = e < (size_t)P ? keys[e] : 0u;
            tl[k] = e < (size_t)P ? tiles[e] : 0u;
        }
        uint32_t sum = 0;
#pragma unroll
        for (int k = 0; k < kDsItems; k++) {
            const size_t e = base + (size_t)k * kWave + lane;
            // culled Gaussians (key 0xFFFFFFFF) are left out of the sort: counted by a ballot (LDS
            // atomics would all hit one word -- 70% of a street view's rows lie outside its 90-degree
            // frustum: config-3 upsweep 59 us per call at 3M rows, r05i), and dropped by pass 0
            const bool cull = e < (size_t)P && key[k] == 0xFFFFFFFFu;
            culled += (uint32_t)__popcll(__ballot(cull));
            if (e < (size_t)P && !cull) {
#pragma unroll
                for (int p = 0; p < kPasses - 2; p++) atomicAdd(&s_hist[p * kRadix + ((key[k] >> (8 * p)) & 0xFFu)], 1u);
                atomicAdd(&s_mid[lane & (kTopCopies - 1)][(key[k] >> 16) & 0xFFu], 1u);
                atomicAdd(&s_top[lane & (kTopCopies - 1)][key[k] >> 24], 1u);
            }
            sum += tl[k];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o, 64);
        if (lane == 0) s_wsum[w] = sum;
        __syncthreads();
        if (t == 0) {
            ctl[ctl_bex(nb) + v] = run;
#pragma unroll
            for (int k = 0; k < kDsWaves; k++) run += s_wsum[k];
        }
        __syncthreads();
    }
    if (lane == 0 && culled) atomicAdd(&s_cull, culled);
    __syncthreads();
    DS_STAMP(0, 1);
    uint32_t hv = s_hist[t];
    if (t >= (kPasses - 1) * kRadix) {
#pragma unroll
        for (int c = 0; c < kTopCopies; c++) hv += s_top[c][t - (kPasses - 1) * kRadix];
    } else if (t >= (kPasses - 2) * kRadix) {
#pragma unroll
        for (int c = 0; c < kTopCopies; c++) hv += s_mid[c][t - (kPasses - 2) * kRadix];
    }
    ctl[ctl_blkhist(nb) + (size_t)u * kPasses * kRadix + t] = hv;
    if (t == 0) {
        ctl[ctl_btot(nb) + u] = run;
        __hip_atomic_fetch_add(&ctl[kCtlK], run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (s_cull) __hip_atomic_fetch_add(&ctl[kCtlCulled], s_cull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t done = __hip_atomic_fetch_add(&ctl[kCtlDone], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (uint32_t)gridDim.x - 1u && host_K) {
            const uint32_t K = ld_agent(&ctl[kCtlK]);
            __hip_atomic_store(host_K, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    DS_STAMP(0, 2);
}

template <int kPass>
__global__ __launch_bounds__(kDsThreads) void dsort_pass_kernel(int P, int nb, const uint32_t *__restrict__ kin,
                                                                 uint32_t *__restrict__ kout,
                                                                 const uint32_t *__restrict__ vin,
                                                                 uint32_t *__restrict__ vout, uint32_t *__restrict__ ctl,
                                                                 uint32_t *__restrict__ offsets,
                                                                 const uint32_t *__restrict__ tiles,
                                                                 const uint2 *__restrict__ rect8,
                                                                 const uint32_t *__restrict__ rect4,
                                                                 uint2 *__restrict__ drect,
                                                                 const uint32_t *__restrict__ rin,
                                                                 uint32_t *__restrict__ rout,
                                                                 uint32_t *__restrict__ host_err) {
    GSR_KS(kKsPass0 + kPass);
    constexpr bool kFirst = kPass == 0, kLast = kPass == kPasses - 1;
    // rect carry (GSR_DSORT_CARRY): pass 0 reads rect4 itself, the others rin; pass 3 stores into
    // drect's 4-B form, the others into rout
    const bool carry = GSR_DSORT_CARRY && rect4 != nullptr;
    constexpr int kShift = 8 * kPass;
    __shared__ uint32_t s_key[kDsTile];
    __shared__ uint32_t s_val[kDsTile];
    __shared__ uint32_t s_rc[GSR_DSORT_CARRY ? kDsTile : 1];  // carried rects
    __shared__ uint32_t s_wh[kDsWaves][kRadix];  // per-wave digit counts -> exclusive prefix over waves
    __shared__ uint32_t s_gb[4][kRadix];         // global digit base (4 partial sums, then [0] scanned)
    __shared__ uint32_t s_bex[kRadix];           // tile-local digit base
    __shared__ uint32_t s_dst[kRadix];           // global slot of tile-local position 0 of each digit
    __shared__ uint32_t s_wsum[kDsWaves];
    __shared__ uint32_t s_v, s_pre, s_nsort;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    DS_STAMP(1 + kPass, 0);
#pragma unroll
    for (int k = 0; k < kDsWaves * kRadix / kDsThreads; k++) (&s_wh[0][0])[t + k * kDsThreads] = 0u;
    // Tile numbering: up to kMaxResident tiles every workgroup can be resident at once (one per CU;
    // nothing else this build runs holds a CU indefinitely), so a tile waiting on lower-numbered
    // ones can always be overtaken and blockIdx.x is the tile; above that, tiles are numbered in
    // start order by a ticket, so a tile only ever waits on tiles that are already running.
    // The histogram-row loads are issued first and summed after the ranking.
    const int nbu = up_blocks(nb);
    uint32_t h[kUpMax / 4];
    {
        const uint32_t *bh = ctl + ctl_blkhist(nb) + kPass * kRadix + (t & (kRadix - 1));
#pragma unroll
        for (int q = 0; q < kUpMax / 4; q++) {
            const int j = (t >> 8) + 4 * q;
            h[q] = j < nbu ? bh[(size_t)j * kPasses * kRadix] : 0u;
        }
    }
    uint32_t v = blockIdx.x;
    if (nb > kMaxResident) {
        if (t == 0) s_v = atomicAdd(&ctl[kCtlTicket + kPass], 1u);
        __syncthreads();
        v = s_v;
    } else {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // s_wh zeroed: LDS only (the row loads stay in flight)
        __builtin_amdgcn_s_barrier();
    }
    // Culled Gaussians (key 0xFFFFFFFF, no tiles) are not sorted: pass 0 reads every key in index
    // order and drops them, so passes 1-3 run over the Pv = P - culled visible keys only and the
    // depth order's slots [Pv, P) are never written (nothing reads them: the binning stops at Pv).
    const size_t Pn = kFirst ? (size_t)P : (size_t)P - min((size_t)ctl[kCtlCulled], (size_t)P);
    const uint32_t nbv = (uint32_t)((Pn + kDsTile - 1) / kDsTile);
    if (v >= nbv) return;  // control words not zeroed past nb; tiles past the visible keys: nothing to do
    DS_STAMP(1 + kPass, 5);
    const int wbase = w * kDsItems * kWave;
    const size_t tile0 = (size_t)v * kDsTile;
    const int n = (int)min((size_t)kDsTile, Pn - tile0);
    uint32_t key[kDsItems], val[kDsItems], tl[kDsItems], rc[kDsItems];
    const uint32_t *rsrc = kFirst ? rect4 : rin;
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const int i = wbase + k * kWave + lane;
        const bool valid = i < n;
        key[k] = valid ? kin[tile0 + i] : 0xFFFFFFFFu;
        val[k] = kFirst ? (uint32_t)(tile0 + i) : (valid ? vin[tile0 + i] : 0u);
        tl[k] = (kFirst && valid) ? tiles[tile0 + i] : 0u;
        // pass 0 loads its rects after the histogram rows are summed (register pressure)
        rc[k] = (!kFirst && carry && valid) ? rsrc[tile0 + i] : 0u;
    }
    DS_STAMP_AFTER(1 + kPass, 6, key[kDsItems - 1] + val[kDsItems - 1]);
    uint32_t toff[kDsItems];
    if (kFirst) {
        // record offsets: the totals of the earlier upsweep workgroups + this tile's offset inside
        // its workgroup, then the in-tile order
        if (w == 0) {
            const int u = (int)v / up_tpb(nb);
            uint32_t c = 0;
#pragma unroll
            for (int q = 0; q < kUpMax / kWave; q++) c += lane + q * kWave < u ? ctl[ctl_btot(nb) + lane + q * kWave] : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
            if (lane == 0) s_pre = c + ctl[ctl_bex(nb) + v];
        }
        uint32_t run = 0;
#pragma unroll
        for (int k = 0; k < kDsItems; k++) {
            const uint32_t incl = wave_incl_scan(tl[k], lane);
            toff[k] = run + incl - tl[k];  // exclusive offset inside the wave's 512 keys
            run += (uint32_t)__shfl((int)incl, 63, 64);
        }
        if (lane == 0) s_wsum[w] = run;
    }
    // ranks: within the wave, equal digits in (item, lane) order (8 ballots per key)
    uint32_t rk[kDsItems];
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const bool valid = wbase + k * kWave + lane < n && key[k] != 0xFFFFFFFFu;
        const uint32_t d = (key[k] >> kShift) & 0xFFu;
        const uint64_t m = match8(d, __ballot(valid));
        const uint32_t b = below(m);
        const uint32_t old = s_wh[w][d];
        if (valid && b == 0u) s_wh[w][d] = old + (uint32_t)__popcll(m);
        rk[k] = old + b;
    }
    {
        // global digit base: column kPass of the upsweep's histogram rows, 4 strided partial sums
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < kUpMax / 4; q++) c += h[q];
        s_gb[t >> 8][t & (kRadix - 1)] = c;
    }
    if (kFirst && carry) {
#pragma unroll
        for (int k = 0; k < kDsItems; k++) {
            const int i = wbase + k * kWave + lane;
            rc[k] = i < n ? rsrc[tile0 + i] : 0u;
        }
    }
    __syncthreads();
    DS_STAMP(1 + kPass, 1);
    if (kFirst) {
        uint32_t pre = s_pre;
        for (int k = 0; k < w; k++) pre += s_wsum[k];
#pragma unroll
        for (int k = 0; k < kDsItems; k++) {
            const int i = wbase + k * kWave + lane;
            if (i < n) offsets[tile0 + i] = pre + toff[k];
        }
    }
    uint32_t cnt = 0;
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < kDsWaves; ww++) {
            const uint32_t c = s_wh[ww][t];
            s_wh[ww][t] = cnt;
            cnt += c;
        }
        uint32_t *st = ctl + ctl_status(nb, kPass);
        st_agent(&st[(size_t)v * kRadix + t], (v == 0 ? kFlagInc : kFlagAgg) | cnt);
        s_bex[t] = cnt;
        s_gb[0][t] += s_gb[1][t] + s_gb[2][t] + s_gb[3][t];
    }
    __syncthreads();
    if (w == 0) {
        const uint32_t nv = scan256_wave(s_bex, lane);  // the tile's sorted (visible) keys
        if (lane == 0) s_nsort = nv;
    }
    if (w == 1) (void)scan256_wave(s_gb[0], lane);
    __syncthreads();
    const int nsort = (int)s_nsort;
    DS_STAMP(1 + kPass, 2);
    // the tile in digit order, through LDS
#pragma unroll
    for (int k = 0; k < kDsItems; k++) {
        const int i = wbase + k * kWave + lane;
        if (i < n && key[k] != 0xFFFFFFFFu) {
            const uint32_t d = (key[k] >> kShift) & 0xFFu;
            const uint32_t lp = s_bex[d] + s_wh[w][d] + rk[k];
            s_key[lp] = key[k];
            s_val[lp] = val[k];
            if (GSR_DSORT_CARRY && carry) s_rc[lp] = rc[k];
        }
    }
    DS_STAMP(1 + kPass, 7);
    if (t < kRadix) {
        // decoupled lookback for digit t over the preceding tiles, kLookWin status words per round
        // trip: add words from the nearest predecessor back until an inclusive one; a word not yet
        // published ends the round (re-polled next round)
        const uint32_t *st = ctl + ctl_status(nb, kPass);
        uint32_t excl = 0;
        int spins = 0;
        for (int j = (int)v - 1; j >= 0;) {
            uint32_t s[kLookWin];
#pragma unroll
            for (int q = 0; q < kLookWin; q++)
                s[q] = j - q >= 0 ? ld_agent(&st[(size_t)(j - q) * kRadix + t]) : kFlagInc;  // past tile 0: +0, stop
            int q = 0;
            bool inc = false;
#pragma unroll
            for (int qq = 0; qq < kLookWin; qq++) {
                const uint32_t f = s[qq] & ~kCountMask;
                if (q == qq && f != 0u && !inc) {
                    excl += s[qq] & kCountMask;
                    inc = f == kFlagInc;
                    q = qq + 1;
                }
            }
            if (inc) break;
            j -= q;
            if (q < kLookWin) {
                if (++spins > kSpinLimit) {
                    // never expected; made loud: render_fwd writes NaN pixels when this word is
                    // set, and the sticky host word fails the next library call on this thread
                    ctl[kCtlErr] = 1u;
                    if (host_err) __hip_atomic_store(host_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (v > 0) st_agent(&ctl[ctl_status(nb, kPass) + (size_t)v * kRadix + t], kFlagInc | (excl + cnt));
        s_dst[t] = s_gb[0][t] + excl - s_bex[t];
    }
    __syncthreads();
    DS_STAMP(1 + kPass, 3);
    for (int i = t; i < nsort; i += kDsThreads) {
        const uint32_t k = s_key[i];
        const uint32_t j = s_dst[(k >> kShift) & 0xFFu] + (uint32_t)i;
        const uint32_t g = s_val[i];
        if (kLast) {
            vout[j] = g;
            if (GSR_DSORT_CARRY && carry) {
                reinterpret_cast<uint32_t *>(drect)[j] = s_rc[i];  // drect4_of(gs), carried
            } else if (rect4) {
                reinterpret_cast<uint32_t *>(drect)[j] = rect4[g];  // drect4_of(gs)
            } else {
                drect[j] = rect8[g];
            }
        } else {
            kout[j] = k;
            vout[j] = g;
            if (GSR_DSORT_CARRY && carry) rout[j] = s_rc[i];
        }
    }
    DS_STAMP(1 + kPass, 4);
}

}  // namespace

int dsort_blocks(int P) { return (P + kDsTile - 1) / kDsTile; }

size_t dsort_ctrl_words(int P) { return ctl_words(dsort_blocks(P) > 0 ? dsort_blocks(P) : 1); }
size_t dsort_ctrl_zero_words(int P) { return ctl_zero_words(dsort_blocks(P) > 0 ? dsort_blocks(P) : 1); }

void launch_depth_sort(int P, const GeomState &gs, uint32_t *host_K, uint32_t *host_err, hipStream_t s,
                       hipEvent_t k_ready) {
    if (P == 0) return;
    const int nb = dsort_blocks(P);
    hipLaunchKernelGGL(dsort_upsweep_kernel, dim3(up_blocks(nb)), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.tiles,
                       gs.ctrl, host_K);
    if (k_ready) (void)hipEventRecord(k_ready, s);
    // keys: dkey -> dkey_sorted -> dkey -> dkey_sorted -> (none); values: (index) -> ids -> order -> ids -> order;
    // carried 4-B rects (rect4 set: rect8 is idle, two P-word halves): rect4 -> A -> B -> A -> drect
    uint32_t *ra = reinterpret_cast<uint32_t *>(gs.rect8), *rb = ra + P;
    hipLaunchKernelGGL(dsort_pass_kernel<0>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted,
                       (const uint32_t *)nullptr, gs.ids, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, gs.rect4, gs.drect,
                       (const uint32_t *)nullptr, ra, host_err);
    hipLaunchKernelGGL(dsort_pass_kernel<1>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted, gs.dkey, gs.ids,
                       gs.order, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, gs.rect4, gs.drect, ra, rb, host_err);
    hipLaunchKernelGGL(dsort_pass_kernel<2>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey, gs.dkey_sorted, gs.order,
                       gs.ids, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, gs.rect4, gs.drect, rb, ra, host_err);
    hipLaunchKernelGGL(dsort_pass_kernel<3>, dim3(nb), dim3(kDsThreads), 0, s, P, nb, gs.dkey_sorted,
                       (uint32_t *)nullptr, gs.ids, gs.order, gs.ctrl, gs.offsets, gs.tiles, gs.rect8, gs.rect4, gs.drect,
                       ra, (uint32_t *)nullptr, host_err);
}

uint32_t *dsort_K_word(const GeomState &gs) { return gs.ctrl + kCtlK; }
uint32_t *dsort_err_word(const GeomState &gs) { return gs.ctrl + kCtlErr; }
uint32_t *dsort_aux_word(const GeomState &gs) { return gs.ctrl + kCtlAux; }
uint32_t *dsort_maxsb_word(const GeomState &gs) { return gs.ctrl + kCtlMaxSB; }
uint32_t *dsort_fwdready_word(const GeomState &gs) { return gs.ctrl + kCtlFwdReady; }
uint32_t *dsort_longest_words(const GeomState &gs) { return gs.ctrl + kCtlLongest; }
uint32_t *dsort_culled_word(const GeomState &gs) { return gs.ctrl + kCtlCulled; }
uint32_t *dsort_live_words(const GeomState &gs) { return gs.ctrl + kCtlLive; }
int dsort_head_words() { return kCtlHead; }

GSR_KSTAMP_READER(kstamp_read_dsort)

}  // namespace gsr
