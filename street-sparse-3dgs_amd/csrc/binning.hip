// binning.hip -- tile lists without a K-element sort.
//
// Upstream emits K (tile << 32 | depth) keys and radix-sorts them (6 passes over 24-B pairs at
// 1080p), then scans the sorted keys for tile ranges.  Here the Gaussians are already in depth
// order (one 32-bit sort of P keys, dsort.hip), and the per-tile lists are built by two stable
// counting passes that exploit each splat's footprint being a rectangle of tiles:
//
//   level 1  Gaussian -> superblock (SB = 2^s x 2^s tiles, ~500 at 1080p).  Chunks of 1024 (more when P is large)
//            depth-ordered Gaussians count their SB footprints in LDS (sb_count), per-SB column
//            scans over chunks give every chunk its offsets (sb_colscan, sb_base), and a second
//            pass writes each SB's Gaussian list in depth order (sb_scatter): per batch of 64
//            Gaussians, each lane ORs its bit into an LDS lane mask per SB it covers, and its
//            rank in an SB's list is the popcount of the lower lanes of that mask.
//   level 2  SB -> tiles (tile_bin): one workgroup per SB counts its tiles' instances, writes the
//            tile ranges, and re-walks the SB list with the same lane-mask ranking per tile to
//            place every instance at its stable position.
//
// The result is the upstream order inside every tile -- (depth bits, Gaussian id) -- with tiles
// laid out SB-major instead of row-major; every consumer goes through `ranges`, so the layout of
// whole tiles in point_list is free.  Traffic ~ 8 B per SB instance + 4 B per tile instance written.
//
// Two ways to reach depth order (rasterizer.hip picks per frame):
//   local sort (default)  level 1 runs over the Gaussians in INDEX order (no global depth sort), so
//                         every SB list is in id order; sb_sort_bin then sorts each SB's list by
//                         depth inside LDS (stable LSD radix over the list's own key range: equal
//                         depths keep id order) and bins it into the SB's tiles from LDS.  The
//                         column scan publishes K and the longest SB list.
//   global sort           dsort.hip's depth order of all P Gaussians, level 1 over it, and
//                         tile_bin over the (already depth-ordered) SB lists: frames with an SB
//                         list longer than the LDS sort holds (kSortCap), and deterministic mode
//                         (whose backward needs dsort's Gaussian-major record offsets).
#include "gsr_launch.h"

namespace gsr {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

struct TileRect {
    int x0, y0, x1, y1;  // inclusive tile bounds; x1 < x0 when empty
};

__device__ __forceinline__ TileRect unpack_rect(uint2 d) {
    TileRect r;
    r.x0 = (int)(d.x & 0xFFFFu);
    r.y0 = (int)(d.x >> 16);
    r.x1 = (int)(d.y & 0xFFFFu) - 1;  // stored exclusive so that 0/0 means "no tiles"
    r.y1 = (int)(d.y >> 16) - 1;
    return r;
}

// A depth-ordered rect: 8-bit fields (gs.rect4 layout) when drect4 is set, else the uint2 form.
__device__ __forceinline__ uint2 load_drect(const uint2 *__restrict__ drect, const uint32_t *__restrict__ drect4, int j) {
    return drect4 ? unpack_rect4(drect4[j]) : drect[j];
}

// Depth-ordered rect / tile count of every Gaussian: the one random gather of the binning.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

#ifndef GSR_SCATTER_WAVES
#define GSR_SCATTER_WAVES 8
#endif
#ifndef GSR_SMALL_SB
#define GSR_SMALL_SB 16
#endif
constexpr int kScatterWaves = GSR_SCATTER_WAVES;
constexpr int kSmallSB = GSR_SMALL_SB;

struct SBFoot {
    int sx0, sy0, sw, n;
};

__device__ __forceinline__ SBFoot sb_foot(const TileRect &r, int shift) {
    SBFoot f{0, 0, 1, 0};
    if (r.x1 < r.x0) return f;
    f.sx0 = r.x0 >> shift;
    f.sy0 = r.y0 >> shift;
    f.sw = (r.x1 >> shift) - f.sx0 + 1;
    f.n = f.sw * ((r.y1 >> shift) - f.sy0 + 1);
    return f;
}

__device__ __forceinline__ uint32_t sb_key(const SBFoot &f, int k, int nsbx) {
    return (uint32_t)((f.sy0 + k / f.sw) * nsbx + f.sx0 + k % f.sw);
}

// footprint clipped to SB `key`, in SB-local tile coordinates (8 bits each)
__device__ __forceinline__ uint32_t sb_local(const TileRect &r, uint32_t key, const SBGrid &sg) {
    const int side = 1 << sg.shift;
    const int ox = (int)(key % (uint32_t)sg.nsbx) * side, oy = (int)(key / (uint32_t)sg.nsbx) * side;
    return (uint32_t)(max(r.x0, ox) - ox) | ((uint32_t)(max(r.y0, oy) - oy) << 8) |
           ((uint32_t)(min(r.x1, ox + side - 1) - ox) << 16) | ((uint32_t)(min(r.y1, oy + side - 1) - oy) << 24);
}

// lane b's value; b is wave-uniform, so v_readlane (no LDS round trip as with __shfl)
__device__ __forceinline__ int rl(int v, int b) { return __builtin_amdgcn_readlane(v, b); }

__device__ __forceinline__ TileRect lane_rect(const TileRect &r, int b) {
    return TileRect{rl(r.x0, b), rl(r.y0, b), rl(r.x1, b), rl(r.y1, b)};
}

__device__ __forceinline__ SBFoot lane_foot(const SBFoot &f, int b) {
    return SBFoot{rl(f.sx0, b), rl(f.sy0, b), rl(f.sw, b), rl(f.n, b)};
}

// Level 1, pass 1: per chunk and SB, the number of Gaussians and of tile instances.
// The depth order's last `*culled` slots hold the culled Gaussians (no tiles: key 0xFFFFFFFF sorts
// last), so chunks wholly past P - *culled have no footprint -- the level-1 kernels skip them and
// the column scan stops before them (a 90-degree street view culls ~70% of a chunk's rows).
__device__ __forceinline__ int visible_chunks(const SBGrid &sg, int P, const uint32_t *culled) {
    if (!culled) return sg.nchunks;
    const int pv = P - (int)min(*culled, (uint32_t)P);
    return min(sg.nchunks, (pv + sg.chunk - 1) / sg.chunk);
}

__global__ __launch_bounds__(1024) void sb_count_kernel(int P, SBGrid sg, const uint2 *__restrict__ drect, const uint32_t *__restrict__ drect4,
                                                       uint32_t *__restrict__ cnt_g, uint32_t *__restrict__ cnt_i,
                                                       const uint32_t *__restrict__ culled) {
    GSR_KS(kKsSbCount);
    extern __shared__ uint32_t lds[];
    uint32_t *cg = lds, *ci = lds + sg.nsb;
    const int chunk = chunk_of_block(blockIdx.x);
    if (chunk >= visible_chunks(sg, P, culled)) return;  // culled rows only, or the last XCD group's padding
    for (int i = threadIdx.x; i < 2 * sg.nsb; i += 1024) lds[i] = 0u;
    __syncthreads();
    // depth-ordered slots past the visible Gaussians were not written by the sort (dsort.hip)
    const int pv = culled ? P - (int)min(*culled, (uint32_t)P) : P;
    const int j0 = chunk * sg.chunk, j1 = min(pv, j0 + sg.chunk);
    const int side = 1 << sg.shift;
    // instances of Gaussian footprint r in SB `key`
    const auto count = [&](const TileRect &r, uint32_t key) {
        const int sx = (int)(key % (uint32_t)sg.nsbx), sy = (int)(key / (uint32_t)sg.nsbx);
        const int h = min(r.y1, sy * side + side - 1) - max(r.y0, sy * side) + 1;
        const int w = min(r.x1, sx * side + side - 1) - max(r.x0, sx * side) + 1;
        atomicAdd(&cg[key], 1u);
        atomicAdd(&ci[key], (uint32_t)(w * h));
    };
    for (int jb = j0; jb < j1; jb += 1024) {
        const int j = jb + (int)threadIdx.x;
        const TileRect r = j < j1 ? unpack_rect(load_drect(drect, drect4, j)) : TileRect{0, 0, -1, -1};
        const SBFoot f = sb_foot(r, sg.shift);
        // footprints over more than kSmallSB superblocks are counted by the whole wave, one SB per
        // lane (a single lane would hold its wave for hundreds of iterations)
        const bool small = f.n <= kSmallSB;
        for (int k = 0; small && k < f.n; k++) count(r, sb_key(f, k, sg.nsbx));
        for (uint64_t big = __ballot(!small); big; big &= big - 1) {
            const int b = __ffsll((unsigned long long)big) - 1;
            const SBFoot fb = lane_foot(f, b);
            const TileRect rb = lane_rect(r, b);
            for (int k = threadIdx.x & 63; k < fb.n; k += 64) count(rb, sb_key(fb, k, sg.nsbx));
        }
    }
    __syncthreads();
    for (int s = threadIdx.x; s < sg.nsb; s += 1024) {
        cnt_g[(size_t)s * sg.ccols + cnt_col(sg, chunk)] = cg[s];
        cnt_i[(size_t)s * sg.ccols + cnt_col(sg, chunk)] = ci[s];
    }
}

// Exclusive scan of NT values held one per thread; returns the exclusive prefix and the total.
template <int NT>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t *wsum, uint32_t &total) {
    constexpr int kW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
        if (lane >= o) incl += t;
    }
    __syncthreads();
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < kW; k++) {
        before += k < w ? wsum[k] : 0u;
        total += wsum[k];
    }
    return before + incl - v;
}

#ifndef GSR_SORT_CAP
#define GSR_SORT_CAP 8192
#endif
constexpr int kSBThreads = 1024;
constexpr int kSBWaves = kSBThreads / 64;
constexpr int kSortCap = GSR_SORT_CAP;            // longest SB list the local sort holds in LDS
constexpr int kSBItems = kSortCap / kSBThreads;   // keys per thread
static_assert(kSortCap % kSBThreads == 0 && kSortCap <= 65536, "kSortCap: a multiple of 1024, 16-bit positions");

// Level 1, pass 2: per SB, exclusive scan of the Gaussian counts over chunks (in place) and the
// SB totals of Gaussians and instances; the last workgroup to finish (a per-frame counter in the
// depth sort's zeroed control words) turns the totals into exclusive SB bases, base[nsb] = the
// total -- one launch instead of a column scan plus a single-workgroup base scan.
constexpr int kColThreads = 256;
__global__ __launch_bounds__(kColThreads) void sb_colscan_kernel(SBGrid sg, uint32_t *__restrict__ cnt_g,
                                                                 const uint32_t *__restrict__ cnt_i,
                                                                 uint32_t *__restrict__ base_g,
                                                                 uint32_t *__restrict__ base_i,
                                                                 uint32_t *__restrict__ done, FrameWords fw,
                                                                 uint32_t *__restrict__ sb_order,
                                                                 uint32_t *__restrict__ zero_classes,
                                                                 uint32_t *__restrict__ tb_flag,
                                                                 uint32_t *__restrict__ tb_items, uint32_t tb_len,
                                                                 uint32_t *__restrict__ host_sblist, int P,
                                                                 const uint32_t *__restrict__ culled) {
    GSR_KS(kKsSbColscan);
    __shared__ uint32_t wsum[kColThreads / 64];
    __shared__ uint32_t s_last, s_tb;
    __shared__ uint32_t s_ci[GSR_FWD_SB_ORDER ? kMaxSB : 1];  // last workgroup: SB instance totals
    __shared__ uint32_t s_hist[GSR_FWD_SB_ORDER ? 256 : 1];
    const int s = blockIdx.x;
    uint32_t *row = cnt_g + (size_t)s * sg.ccols;
    const uint32_t *rowi = cnt_i + (size_t)s * sg.ccols;
    uint32_t carry = 0, isum = 0;
    const int nch = visible_chunks(sg, P, culled);  // later chunks' counters were not written (all zero)
    for (int b = 0; b < nch; b += kColThreads) {
        const int c = b + (int)threadIdx.x;
        const uint32_t v = c < nch ? row[cnt_col(sg, c)] : 0u;
        isum += c < nch ? rowi[cnt_col(sg, c)] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan<kColThreads>(v, wsum, tot);
        if (c < nch) row[cnt_col(sg, c)] = carry + ex;
        carry += tot;
    }
    uint32_t itot;
    (void)block_exclusive_scan<kColThreads>(isum, wsum, itot);
    if (threadIdx.x == 0) {
        // publish the totals write-through (sc1), drain, then count this workgroup in; the last
        // one reads them back with sc1 loads (MI355X_MICROARCH.md hand-off rules: no L2 fences)
        __hip_atomic_store(&base_g[s], carry, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&base_i[s], itot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = prev == gridDim.x - 1u;
    }
    __syncthreads();
    if (!s_last) return;
    const int nsb = sg.nsb;
    if (threadIdx.x == 0) s_tb = 0u;
    __syncthreads();
    uint32_t cg = 0, ci = 0, mg = 0;
    for (int b = 0; b < nsb; b += kColThreads) {
        const int k = b + (int)threadIdx.x;
        const uint32_t vg = k < nsb ? __hip_atomic_load(&base_g[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        const uint32_t vi = k < nsb ? __hip_atomic_load(&base_i[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        mg = max(mg, vg);
        if (tb_flag && k < nsb) {
            // tile_bin split: a long list's slices (consecutive items); a full queue leaves it whole
            uint32_t nsl = tb_len && vg > tb_len ? min((vg + tb_len - 1u) / tb_len, kTBMaxSlices) : 0u;
            const uint32_t at = nsl ? atomicAdd(&s_tb, nsl) : 0u;
            const bool fits = nsl && at + nsl <= (uint32_t)kTBMaxItems;
            for (uint32_t j = 0; j < nsl && at + j < (uint32_t)kTBMaxItems; j++)
                tb_items[at + j] = fits ? ((uint32_t)k | j << 12 | nsl << 18) : kTBVoid;
            tb_flag[k] = fits ? 1u : 0u;
        }
        if (GSR_FWD_SB_ORDER && k < nsb) s_ci[k] = vi;
        uint32_t tg, ti;
        const uint32_t eg = block_exclusive_scan<kColThreads>(vg, wsum, tg);
        const uint32_t ei = block_exclusive_scan<kColThreads>(vi, wsum, ti);
        if (k < nsb) {
            base_g[k] = cg + eg;
            base_i[k] = ci + ei;
        }
        cg += tg;
        ci += ti;
    }
    if (threadIdx.x == 0) {
        base_g[nsb] = cg;
        base_i[nsb] = ci;
    }
    if (tb_flag) {
        __syncthreads();
        if (threadIdx.x == 0) tb_flag[nsb] = min(s_tb, (uint32_t)kTBMaxItems);
    }
    if (zero_classes && threadIdx.x < kBwdClasses) zero_classes[threadIdx.x] = 0u;
    if (zero_classes && threadIdx.x == 0) zero_classes[kBwdSegCount] = 0u;
    if (GSR_FWD_SB_ORDER && sb_order) {
        // the forward's launch order, heaviest first: SBs bucketed into 256 descending classes of
        // their mean tile list length (16 instances per class), in order of the bucket scan
        const int tshift = 2 * sg.shift;
        const auto cls = [&](int k) {
            const uint32_t c = (s_ci[k] >> tshift) >> 4;
            return 255u - (c < 255u ? c : 255u);
        };
        s_hist[threadIdx.x] = 0u;  // kColThreads == 256
        __syncthreads();
        for (int k = threadIdx.x; k < nsb; k += kColThreads) atomicAdd(&s_hist[cls(k)], 1u);
        __syncthreads();
        if (threadIdx.x < 64) {
            const int l = threadIdx.x;
            const uint32_t a = s_hist[4 * l], b = s_hist[4 * l + 1], c = s_hist[4 * l + 2], d = s_hist[4 * l + 3];
            const uint32_t sum = a + b + c + d;
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
                if (l >= o) incl += v;
            }
            const uint32_t ex = incl - sum;
            s_hist[4 * l] = ex;
            s_hist[4 * l + 1] = ex + a;
            s_hist[4 * l + 2] = ex + a + b;
            s_hist[4 * l + 3] = ex + a + b + c;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < nsb; k += kColThreads) sb_order[atomicAdd(&s_hist[cls(k)], 1u)] = (uint32_t)k;
    }
    if (fw.dev_K || host_sblist) {
        // the longest SB list: for the split gate's hint (host_sblist), and on local-sort frames K
        // (= the instance total) and that maximum for the kernels and the host.  The host's K word
        // is stored last (the host reads the others once it is set).
        mg = wave_max_u32(mg);  // DPP and row / half swaps: no LDS round trips
        __syncthreads();
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = mg;
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < kColThreads / 64; k++) mg = max(mg, wsum[k]);
            if (host_sblist) {
                if (GSR_HOST_WORDS == 2) *host_sblist = mg;  // a device word render_fwd forwards
                else __hip_atomic_store(host_sblist, mg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (fw.dev_K) {
        if (threadIdx.x == 0) {
            // an SB list too long for the local sort: the device K word reads "capacity short" to
            // every later kernel of the frame (they exit at once; the host re-runs the frame
            // through the global sort, which stores the real K there again)
            *fw.dev_K = mg > (uint32_t)kSortCap ? 0xFFFFFFFFu : ci;
            *fw.dev_maxsb = mg;
            if (fw.host) {
                __hip_atomic_store(&fw.host[kHostMaxSB], mg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&fw.host[kHostP1], cg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&fw.host[kHostK], ci, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

// The lane masks are only ever touched through workgroup-scope atomics: the ORs of step 1 and the
// reads of steps 2 and 3 address the same LDS words, and with a plain read after the atomic OR the
// compiler may serve the read from the atomic's own result (that lane's OR alone, without the other
// lanes' bits -- the hazard that once produced wrong ranks in the depth sort).  An atomic load
// cannot be forwarded that way; the hardware keeps one wave's LDS operations in order, so it
// costs no wait beyond the ds_read itself.
__device__ __forceinline__ void mask_or(uint64_t *m, uint64_t bit) {
    (void)__hip_atomic_fetch_or(m, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint64_t mask_load(uint64_t *m) {
    return __hip_atomic_load(m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void mask_clear(uint64_t *m) {
    __hip_atomic_store(m, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Level 1, pass 3: stable scatter of (chunk, wave, batch, lane)-ordered Gaussians into the SB
// lists.  Ranks come from LDS lane masks: every lane ORs its bit into the mask of each SB it
// covers, its rank in that SB's list is the popcount of the lower lanes, and the highest lane of
// each mask advances the SB's position and clears the mask.  Footprints of up to kSmallSB SBs
// are walked per lane; larger ones (rare, 3-sigma splats) by the whole wave, one at a time, so
// one outlier does not serialise its batch.
__global__ __launch_bounds__(64 * kScatterWaves) void sb_scatter_kernel(int P, SBGrid sg,
                                                                         const uint32_t *__restrict__ order,
                                                                         const uint2 *__restrict__ drect,
                                                                         const uint32_t *__restrict__ drect4,
                                                                         const uint32_t *__restrict__ col,
                                                                         const uint32_t *__restrict__ base_g,
                                                                         uint2 *__restrict__ sblist,
                                                                         uint4 *__restrict__ sblist4,
                                                                         const uint32_t *__restrict__ dkey,
                                                                         const uint32_t *__restrict__ kdev, uint32_t cap,
                                                                         const uint32_t *__restrict__ culled) {
    GSR_KS(kKsSbScatter);
    // the point-list capacity is short: the host re-runs at K (SB instances <= K, so K <= cap
    // bounds the level-1 lists too; the same test as every other binning / render kernel)
    if (*kdev > cap) return;
    const int chunk = chunk_of_block(blockIdx.x);
    if (chunk >= visible_chunks(sg, P, culled)) return;  // culled rows only, or the XCD group's padding
    extern __shared__ uint32_t wc[];  // [W][nsb] per-wave running positions, then [W][nsb] u64 masks
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nsb = sg.nsb;
    for (int i = threadIdx.x; i < 3 * kScatterWaves * nsb; i += 64 * kScatterWaves) wc[i] = 0u;
    __syncthreads();
    const int per_wave = sg.chunk / kScatterWaves;
    const int pv = culled ? P - (int)min(*culled, (uint32_t)P) : P;  // slots past pv: not written by the sort
    const int jw0 = chunk * sg.chunk + w * per_wave, jw1 = min(pv, jw0 + per_wave);
    uint32_t *run = wc + w * nsb;
    uint64_t *msk = reinterpret_cast<uint64_t *>(wc + kScatterWaves * nsb) + w * nsb;
    const uint64_t lt = (1ull << lane) - 1ull;
    // the SB bases of this chunk (read after the counting): loads issued now
    constexpr int kSBPerThread = (kMaxSB + 64 * kScatterWaves - 1) / (64 * kScatterWaves);
    uint32_t sbase[kSBPerThread];
#pragma unroll
    for (int q = 0; q < kSBPerThread; q++) {
        const int sq = (int)threadIdx.x + q * 64 * kScatterWaves;
        sbase[q] = sq < nsb ? base_g[sq] + col[(size_t)sq * sg.ccols + cnt_col(sg, chunk)] : 0u;
    }
    // list loads one batch ahead of their use
    const auto rect_at = [&](int j) { return j < jw1 ? load_drect(drect, drect4, j) : make_uint2(0u, 0u); };

    // per-wave SB counts
    uint2 rnext = rect_at(jw0 + lane);
    for (int jb = jw0; jb < jw1; jb += 64) {
        const TileRect r = unpack_rect(rnext);
        rnext = rect_at(jb + 64 + lane);
        const SBFoot f = sb_foot(r, sg.shift);
        const bool small = f.n <= kSmallSB;
#pragma unroll
        for (int k = 0; k < kSmallSB; k++)
            if (small && k < f.n) atomicAdd(&run[sb_key(f, k, sg.nsbx)], 1u);
        for (uint64_t big = __ballot(!small); big; big &= big - 1) {
            const int b = __ffsll((unsigned long long)big) - 1;
            const SBFoot fb = lane_foot(f, b);
            for (int k = lane; k < fb.n; k += 64) atomicAdd(&run[sb_key(fb, k, sg.nsbx)], 1u);
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSBPerThread; q++) {
        const int s = (int)threadIdx.x + q * 64 * kScatterWaves;
        if (s >= nsb) break;
        uint32_t b = sbase[q];
        for (int k = 0; k < kScatterWaves; k++) {
            const uint32_t c = wc[k * nsb + s];
            wc[k * nsb + s] = b;
            b += c;
        }
    }
    __syncthreads();

    // local sort (sblist4): index order, and each entry carries the Gaussian's depth key (read
    // here in index order, coalesced -- the sort kernel would otherwise gather it per entry)
    const auto id_at = [&](int j) { return j < jw1 ? (order ? order[j] : (uint32_t)j) : 0u; };
    const auto key_at = [&](int j) { return (sblist4 && j < jw1) ? dkey[j] : 0u; };
    uint32_t gnext = id_at(jw0 + lane), knext = key_at(jw0 + lane);
    rnext = rect_at(jw0 + lane);
    for (int jb = jw0; jb < jw1; jb += 64) {
        const uint32_t g = gnext, gk = knext;
        const TileRect r = unpack_rect(rnext);  // (0, 0) past the end: no tiles
        gnext = id_at(jb + 64 + lane);
        knext = key_at(jb + 64 + lane);
        rnext = rect_at(jb + 64 + lane);
        const SBFoot f = sb_foot(r, sg.shift);
        const bool small = f.n <= kSmallSB;
        const uint64_t bigs = __ballot(!small);
        // 1. masks
#pragma unroll
        for (int k = 0; k < kSmallSB; k++)
            if (small && k < f.n) mask_or(&msk[sb_key(f, k, sg.nsbx)], 1ull << lane);
        for (uint64_t big = bigs; big; big &= big - 1) {
            const int b = __ffsll((unsigned long long)big) - 1;
            const SBFoot fb = lane_foot(f, b);
            for (int k = lane; k < fb.n; k += 64)
                mask_or(&msk[sb_key(fb, k, sg.nsbx)], 1ull << b);
        }
        // 2. ranked writes
#pragma unroll
        for (int k = 0; k < kSmallSB; k++)
            if (small && k < f.n) {
                const uint32_t key = sb_key(f, k, sg.nsbx);
                const uint32_t at = run[key] + (uint32_t)__popcll(mask_load(&msk[key]) & lt);
                if (sblist4)
                    sblist4[at] = make_uint4(g, sb_local(r, key, sg), gk, 0u);
                else
                    sblist[at] = make_uint2(g, sb_local(r, key, sg));
            }
        for (uint64_t big = bigs; big; big &= big - 1) {
            const int b = __ffsll((unsigned long long)big) - 1;
            const SBFoot fb = lane_foot(f, b);
            const TileRect rb = lane_rect(r, b);
            const uint32_t gb = (uint32_t)rl((int)g, b), gkb = (uint32_t)rl((int)gk, b);
            for (int k = lane; k < fb.n; k += 64) {
                const uint32_t key = sb_key(fb, k, sg.nsbx);
                const uint32_t at = run[key] + (uint32_t)__popcll(mask_load(&msk[key]) & ((1ull << b) - 1ull));
                if (sblist4)
                    sblist4[at] = make_uint4(gb, sb_local(rb, key, sg), gkb, 0u);
                else
                    sblist[at] = make_uint2(gb, sb_local(rb, key, sg));
            }
        }
        // 3. the highest lane of every mask advances the SB position and clears the mask
#pragma unroll
        for (int k = 0; k < kSmallSB; k++)
            if (small && k < f.n) {
                const uint32_t key = sb_key(f, k, sg.nsbx);
                const uint64_t m = mask_load(&msk[key]);
                if (m != 0 && 63 - __clzll((long long)m) == lane) {
                    run[key] += (uint32_t)__popcll(m);
                    mask_clear(&msk[key]);
                }
            }
        for (uint64_t big = bigs; big; big &= big - 1) {
            const int b = __ffsll((unsigned long long)big) - 1;
            const SBFoot fb = lane_foot(f, b);
            for (int k = lane; k < fb.n; k += 64) {
                const uint32_t key = sb_key(fb, k, sg.nsbx);
                const uint64_t m = mask_load(&msk[key]);
                if (m != 0 && 63 - __clzll((long long)m) == b) {
                    run[key] += (uint32_t)__popcll(m);
                    mask_clear(&msk[key]);
                }
            }
        }
    }
}

// Level 2: one workgroup per SB; wave w owns a contiguous 1/kTBWaves of the SB's list (entries
// carry the footprint clipped to the SB, so the list is read sequentially).  For each batch of 64
// entries and each of the SB's tiles (16 at a time), a ballot of "footprint contains the tile"
// gives the tile's count (pass A) or, after the tile scan, the stable rank of every covering
// entry (pass B).  Counters and positions are wave-uniform registers: no LDS in the loops.
#ifndef GSR_TB_WAVES
#define GSR_TB_WAVES 8  // waves per superblock for short lists (1M Gaussians: 8 > 16 > 4)
#endif
#ifndef GSR_TB_WAVES_LONG
#define GSR_TB_WAVES_LONG 16  // ... and for long ones (more than GSR_TB_LONG Gaussians per SB on average)
#endif
#ifndef GSR_TB_LONG
#define GSR_TB_LONG 4096
#endif
constexpr int kTileGroup = 16;
constexpr int kTBSplitBlocks = 256;  // tb_split_kernel's grid (items dealt round-robin)

#ifndef GSR_TB_DEPTH
#define GSR_TB_DEPTH 2  // list batches in flight per wave (loads issued one group ahead)
#endif
constexpr int kTBDepth = GSR_TB_DEPTH;

// Footprint of SB-clipped rect r over tile group [tg, tg + 16) (SB-local row-major), one bit per
// tile: the column range as a bit run, replicated over the group's rows inside the row range.
__device__ __forceinline__ uint32_t group_mask(uint32_t r, int tg, int shift) {
    const int side = 1 << shift;
    const int x0 = (int)(r & 0xFFu), y0 = (int)((r >> 8) & 0xFFu), x1 = (int)((r >> 16) & 0xFFu),
              y1 = (int)(r >> 24);
    if (x1 < x0) return 0u;  // padding entry (0xFF) or empty
    const uint32_t cols = ((2u << x1) - 1u) & ~((1u << x0) - 1u);  // x1 <= 15
    const int row0 = tg >> shift, rows = kTileGroup >> shift;     // side <= 16: rows >= 1
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int ry = row0 + q;
        if (q < rows && ry >= y0 && ry <= y1) m |= cols << (q * side);
    }
    return m;
}

// tile_bin's two list walks over entries [a, b) of an SB list at L0, split over the workgroup's
// kTBWaves waves (wave w: a contiguous 1/kTBWaves): count = per-wave tile counts into tc[w][t];
// place = stable placement from per-wave tile starts tc[w][t].
template <int kTBWaves, bool kPlace>
__device__ __forceinline__ void tb_walk(const SBGrid &sg, uint32_t L0, uint32_t a, uint32_t b,
                                        const uint2 *__restrict__ sblist, uint32_t *__restrict__ point_list,
                                        uint32_t (*tc)[kMaxTilesPerSB]) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tps = 1 << (2 * sg.shift);
    const uint32_t n = b - a;
    const uint32_t seg0 = a + (uint32_t)(((uint64_t)n * w) / kTBWaves), seg1 = a + (uint32_t)(((uint64_t)n * (w + 1)) / kTBWaves);
    const uint64_t lt = (1ull << lane) - 1ull;
    // the wave's list segment in groups of kTBDepth batches: group n + 1's entries are loaded
    // while group n is ranked (one dependent load latency per group instead of one per batch)
    const auto load = [&](uint32_t gb, uint2 *e) {
#pragma unroll
        for (int d = 0; d < kTBDepth; d++) {
            const uint32_t i = gb + (uint32_t)(d * 64 + lane);
            e[d] = i < seg1 ? sblist[L0 + i] : make_uint2(0u, 0xFFu);
        }
    };
    constexpr uint32_t kGroup = 64 * kTBDepth;
    for (int tg = 0; tg < tps; tg += kTileGroup) {
        uint32_t acc[kTileGroup];
#pragma unroll
        for (int k = 0; k < kTileGroup; k++) acc[k] = kPlace ? (tg + k < tps ? tc[w][tg + k] : 0u) : 0u;
        uint2 cur[kTBDepth], nxt[kTBDepth];
        load(seg0, cur);
        for (uint32_t gb = seg0; gb < seg1; gb += kGroup) {
            load(gb + kGroup, nxt);
#pragma unroll
            for (int d = 0; d < kTBDepth; d++) {
                const uint32_t m = group_mask(cur[d].y, tg, sg.shift);
#pragma unroll
                for (int k = 0; k < kTileGroup; k++) {
                    const bool hit = (m >> k) & 1u;
                    const uint64_t bm = __ballot(hit);
                    if (kPlace && hit) point_list[acc[k] + (uint32_t)__popcll(bm & lt)] = cur[d].x;
                    acc[k] += (uint32_t)__popcll(bm);
                }
            }
#pragma unroll
            for (int d = 0; d < kTBDepth; d++) cur[d] = nxt[d];
        }
        if (!kPlace && lane == 0)
#pragma unroll
            for (int k = 0; k < kTileGroup; k++)
                if (tg + k < tps) tc[w][tg + k] = acc[k];
    }
}

// Per-wave tile counts tc[w][t] -> per-wave starts, tiles in SB-local row-major order from `base`
// plus extra[t] (the instances of tile t placed before this workgroup's entries, tb_place), waves
// in list order; wave 0 writes the ranges (tile totals tot[t] when given, else this workgroup's
// counts) when `ranges` is set.
template <int kTBWaves>
__device__ __forceinline__ void tb_bases(const SBGrid &sg, int gx, int gy, int s, uint32_t base,
                                         uint32_t (*tc)[kMaxTilesPerSB], const uint32_t *tot, const uint32_t *extra,
                                         uint2 *__restrict__ ranges) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int side = 1 << sg.shift, tps = side * side;
    const int ox = (s % sg.nsbx) * side, oy = (s / sg.nsbx) * side;
    if (w != 0) return;
    uint32_t carry = 0;
    for (int t0 = 0; t0 < tps; t0 += 64) {
        const int t = t0 + lane;
        uint32_t c = 0;
        if (t < tps) {
            if (tot) c = tot[t];
            else
                for (int k = 0; k < kTBWaves; k++) c += tc[k][t];
        }
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
            if (lane >= o) incl += v;
        }
        if (t < tps) {
            const uint32_t t_base = base + carry + incl - c;
            const int x = ox + (t & (side - 1)), y = oy + (t >> sg.shift);
            if (ranges && x < gx && y < gy) ranges[y * gx + x] = make_uint2(t_base, t_base + c);
            uint32_t b = t_base + (extra ? extra[t] : 0u);
            for (int k = 0; k < kTBWaves; k++) {
                const uint32_t ck = tc[k][t];
                tc[k][t] = b;
                b += ck;
            }
        }
        carry += (uint32_t)__shfl((int)incl, 63, 64);
    }
}

template <int kTBWaves>
__global__ __launch_bounds__(64 * kTBWaves) void tile_bin_kernel(SBGrid sg, int gx, int gy,
                                                                 const uint32_t *__restrict__ base_g,
                                                                 const uint32_t *__restrict__ base_i,
                                                                 const uint2 *__restrict__ sblist,
                                                                 uint32_t *__restrict__ point_list,
                                                                 uint2 *__restrict__ ranges,
                                                                 const uint32_t *__restrict__ kdev, uint32_t cap,
                                                                 const uint32_t *__restrict__ tb_flag) {
    GSR_KS(kKsTileBin);
    if (*kdev > cap) return;  // the point-list capacity is short: the host re-runs at K
    const int s = blockIdx.x;
    if (tb_flag && tb_flag[s]) return;  // a long list: binned in slices (tb_split_kernel)
    __shared__ uint32_t tc[kTBWaves][kMaxTilesPerSB];
    const uint32_t L0 = base_g[s], L = base_g[s + 1] - L0;
    tb_walk<kTBWaves, false>(sg, L0, 0u, L, sblist, point_list, tc);  // pass A: per-wave tile counts
    __syncthreads();
    // tile bases (SB-local row-major tile order, waves in list order) and the tile ranges
    tb_bases<kTBWaves>(sg, gx, gy, s, base_i[s], tc, nullptr, nullptr, ranges);
    __syncthreads();
    tb_walk<kTBWaves, true>(sg, L0, 0u, L, sblist, point_list, tc);  // pass B: stable placement
}

// Long SB lists (tile_bin split): the SB's list in nsl slices of ~L / nsl entries, one work item
// each, on the side stream beside tile_bin.  kPlace = false (first launch): the slice's tile counts
// into tb_cnt[item][t].  kPlace = true (second launch): the tile totals and the counts of the
// slices before this one from every slice's tb_cnt, then tile_bin's bases and placement for the
// slice -- the same stable order (slices in list order), so the point list is the one tile_bin
// would write.  Items are dealt round-robin (no waits between items).
template <int kTBWaves, bool kPlace>
__global__ __launch_bounds__(64 * kTBWaves) void tb_split_kernel(SBGrid sg, int gx, int gy,
                                                                 const uint32_t *__restrict__ base_g,
                                                                 const uint32_t *__restrict__ base_i,
                                                                 const uint2 *__restrict__ sblist,
                                                                 uint32_t *__restrict__ point_list,
                                                                 uint2 *__restrict__ ranges,
                                                                 const uint32_t *__restrict__ kdev, uint32_t cap,
                                                                 const uint32_t *__restrict__ tb_flag,
                                                                 const uint32_t *__restrict__ tb_items,
                                                                 uint32_t *__restrict__ tb_cnt) {
    if (*kdev > cap) return;
    __shared__ uint32_t tc[kTBWaves][kMaxTilesPerSB];
    __shared__ uint32_t s_tot[kMaxTilesPerSB], s_pre[kMaxTilesPerSB];
    const int tps = 1 << (2 * sg.shift);
    const uint32_t n = tb_flag[sg.nsb];
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t it = tb_items[i];
        if (it == kTBVoid) continue;
        const int s = (int)(it & 0xFFFu);
        const uint32_t j = (it >> 12) & 0x3Fu, nsl = it >> 18;
        const uint32_t L0 = base_g[s], L = base_g[s + 1] - L0;
        const uint32_t Ls = (L + nsl - 1u) / nsl;
        const uint32_t a = min(L, j * Ls), b = min(L, a + Ls);
        tb_walk<kTBWaves, false>(sg, L0, a, b, sblist, point_list, tc);
        __syncthreads();
        if (!kPlace) {
            for (int t = threadIdx.x; t < tps; t += 64 * kTBWaves) {
                uint32_t c = 0;
                for (int k = 0; k < kTBWaves; k++) c += tc[k][t];
                tb_cnt[(size_t)i * tps + t] = c;
            }
        } else {
            const uint32_t i0 = i - j;
            for (int t = threadIdx.x; t < tps; t += 64 * kTBWaves) {
                uint32_t tot = 0, pre = 0;
                for (uint32_t jj = 0; jj < nsl; jj++) {
                    const uint32_t c = tb_cnt[(size_t)(i0 + jj) * tps + t];
                    tot += c;
                    pre += jj < j ? c : 0u;
                }
                s_tot[t] = tot;
                s_pre[t] = pre;
            }
            __syncthreads();
            tb_bases<kTBWaves>(sg, gx, gy, s, base_i[s], tc, s_tot, s_pre, j == 0 ? ranges : nullptr);
            __syncthreads();
            tb_walk<kTBWaves, true>(sg, L0, a, b, sblist, point_list, tc);
        }
        __syncthreads();  // tc / s_tot reused by the next item
    }
}

// ---------------------------------------------------------------------------------------------
// Local sort: one workgroup per SB sorts its list (id order, from an index-order level 1) by depth
// in LDS and bins it into the SB's tiles -- the global depth sort's job, per SB and without a pass
// over global memory per digit.
//
// 1. Load: entry e's depth key (stored with the entry by the index-order scatter) into registers,
//    wave-striped so that (wave, item, lane) order is list order; the list's key range by a block
//    min / max.
// 2. Stable LSD radix over (key - min) in 8-bit digits, only as many passes as the range needs
//    (equal depths: none): match-mask ranking (8 ballots per key) into per-wave LDS counters, a
//    digit scan, the reorder through LDS (keys and 16-bit list positions ping-pong).  Stability
//    keeps id order among equal depths: the (depth bits, id) order of upstream's keys.
// 3. The sorted (id, footprint) pairs, gathered once from the SB list into LDS, then tile_bin's
//    two ballot passes (per-wave tile counts, tile bases and ranges, stable placement) over them.
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ uint64_t lanes_with_digit(uint32_t d, uint64_t valid) {
    uint64_t m = valid;
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

// Measurement builds only (GSR_SB_TRACE=1): per-workgroup phase stamps (s_memrealtime, 100 MHz)
// of sb_sort_bin, read back with gsr_debug_trace.
#ifndef GSR_SB_TRACE
#define GSR_SB_TRACE 0
#endif
__device__ unsigned long long g_sb_trace[2048 * 8];
#define SB_STAMP(slot)                                                                         \
    do {                                                                                       \
        if (GSR_SB_TRACE && threadIdx.x == 0 && blockIdx.x < 2048) {                           \
            __builtin_amdgcn_s_waitcnt(0);                                                     \
            g_sb_trace[blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();            \
        }                                                                                      \
    } while (0)

// __launch_bounds__(1024, 8): registers budgeted for 8 waves per SIMD -- two 1024-thread
// workgroups per CU (66 KiB of LDS each); at the compiler's default (7 waves per SIMD, 104 SGPRs)
// only one fit and the 510 superblocks of a 1080p frame ran in two rounds
__global__ __launch_bounds__(kSBThreads, 8) void sb_sort_bin_kernel(SBGrid sg, int gx, int gy,
                                                                const uint32_t *__restrict__ base_g,
                                                                const uint32_t *__restrict__ base_i,
                                                                const uint4 *__restrict__ sblist,
                                                                uint32_t *__restrict__ point_list,
                                                                uint2 *__restrict__ ranges,
                                                                const uint32_t *__restrict__ kdev, uint32_t cap,
                                                                const uint32_t *__restrict__ maxsb) {
    // capacity short (the host re-runs at K) or an SB list the LDS cannot hold (the host re-runs
    // the frame through the global depth sort): nothing is written
    if (*kdev > cap || *maxsb > (uint32_t)kSortCap) return;
    // one key / position buffer: each pass scatters into it after every thread has its elements in
    // registers (65 KiB of LDS in all: two workgroups per CU)
    __shared__ uint32_t s_key[kSortCap];
    __shared__ uint16_t s_pos[kSortCap];
    __shared__ uint32_t s_wh[kSBWaves][256];  // per-wave digit counts; later the per-wave tile counters
    __shared__ uint32_t s_bex[256];
    __shared__ uint32_t s_lo, s_hi;
    const int s = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int side = 1 << sg.shift, tps = side * side;
    const int ox = (s % sg.nsbx) * side, oy = (s / sg.nsbx) * side;
    const uint32_t L0 = base_g[s], n = base_g[s + 1] - L0;
    const uint64_t lt = (1ull << lane) - 1ull;
    const int wb = w * kSBItems * 64;  // the wave's first list position
    SB_STAMP(0);
    if (GSR_SB_TRACE && t == 0) g_sb_trace[min(blockIdx.x, 2047u) * 8 + 7] = n;

    // 1. keys and their range
    if (t == 0) {
        s_lo = 0xFFFFFFFFu;
        s_hi = 0u;
    }
    for (int i = t; i < kSBWaves * 256; i += kSBThreads) (&s_wh[0][0])[i] = 0u;
    uint32_t key[kSBItems];
    uint16_t pos[kSBItems];
    {
        uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
        for (int k = 0; k < kSBItems; k++) {
            const uint32_t e = (uint32_t)(wb + k * 64 + lane);
            key[k] = e < n ? sblist[L0 + e].z : 0u;  // the depth key the scatter stored with the entry
            pos[k] = (uint16_t)e;
            if (e < n) {
                lo = min(lo, key[k]);
                hi = max(hi, key[k]);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
        }
        __syncthreads();
        if (lane == 0 && lo <= hi) {
            atomicMin(&s_lo, lo);
            atomicMax(&s_hi, hi);
        }
    }
    __syncthreads();
    const uint32_t klo = s_lo, range = s_lo <= s_hi ? s_hi - s_lo : 0u;
    const int passes = range ? (32 - __clz((int)range) + 7) / 8 : 0;
    SB_STAMP(1);
#pragma unroll
    for (int k = 0; k < kSBItems; k++) key[k] -= klo;  // padding keys wrap: never ranked (valid mask)

    // 2. stable LSD passes; the sorted list positions end in s_pos (and in pos[] by striped slot)
    for (int p = 0; p < passes; p++) {
        const int shift = 8 * p;
        uint32_t rk[kSBItems];
#pragma unroll
        for (int k = 0; k < kSBItems; k++) {
            if (wb + k * 64 >= (int)n) {  // wave-uniform: nothing of this item in the list
                rk[k] = 0u;
                continue;
            }
            const bool valid = (uint32_t)(wb + k * 64 + lane) < n;
            const uint32_t d = (key[k] >> shift) & 0xFFu;
            const uint64_t m = lanes_with_digit(d, __ballot(valid));
            const uint32_t b = lanes_below(m);
            const uint32_t old = s_wh[w][d];
            if (valid && b == 0u) s_wh[w][d] = old + (uint32_t)__popcll(m);
            rk[k] = old + b;
        }
        __syncthreads();
        if (t < 256) {
            uint32_t c = 0;
#pragma unroll
            for (int ww = 0; ww < kSBWaves; ww++) {
                const uint32_t v = s_wh[ww][t];
                s_wh[ww][t] = c;
                c += v;
            }
            s_bex[t] = c;
        }
        __syncthreads();
        if (w == 0) {
            uint32_t *a = s_bex;
            const uint32_t x0 = a[4 * lane], x1 = a[4 * lane + 1], x2 = a[4 * lane + 2], x3 = a[4 * lane + 3];
            const uint32_t sum = x0 + x1 + x2 + x3;
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
                if (lane >= o) incl += v;
            }
            const uint32_t e = incl - sum;
            a[4 * lane] = e;
            a[4 * lane + 1] = e + x0;
            a[4 * lane + 2] = e + x0 + x1;
            a[4 * lane + 3] = e + x0 + x1 + x2;
        }
        __syncthreads();  // (every element of the last pass is back in registers: the buffer is free)
#pragma unroll
        for (int k = 0; k < kSBItems; k++) {
            if ((uint32_t)(wb + k * 64 + lane) < n) {
                const uint32_t d = (key[k] >> shift) & 0xFFu;
                const uint32_t dst = s_bex[d] + s_wh[w][d] + rk[k];
                s_key[dst] = key[k];
                s_pos[dst] = pos[k];
            }
        }
        __syncthreads();
        for (int i = t; i < kSBWaves * 256; i += kSBThreads) (&s_wh[0][0])[i] = 0u;
#pragma unroll
        for (int k = 0; k < kSBItems; k++) {
            const uint32_t e = (uint32_t)(wb + k * 64 + lane);
            if (e < n) {
                key[k] = s_key[e];
                pos[k] = s_pos[e];
            }
        }
        // s_wh cleared and this pass's reads done before the next pass ranks and scatters
        __syncthreads();
    }

    SB_STAMP(2);
    // 3. the sorted (id, footprint) pairs into registers: sorted position e = wb + 64 k + lane is
    // held by that lane as item k (pos[] after the last pass), so the wave's tile binning below runs
    // over its own 512 consecutive sorted positions with no LDS and no further gathers
    uint32_t gid[kSBItems], gfp[kSBItems];
#pragma unroll
    for (int k = 0; k < kSBItems; k++) {
        const uint32_t e = (uint32_t)(wb + k * 64 + lane);
        gid[k] = 0u;
        gfp[k] = 0xFFu;  // padding: an empty footprint (x1 < x0)
        if (e < n) {
            const uint2 v = reinterpret_cast<const uint2 *>(sblist + L0 + min((uint32_t)pos[k], n - 1u))[0];
            gid[k] = v.x;  // (pos: a permutation of [0, n))
            gfp[k] = v.y;
        }
    }
    SB_STAMP(3);
    // tile binning over the sorted list (tile_bin's two ballot passes): wave w owns sorted
    // positions [wb, wb + 512), batch k = its item k
    uint32_t(*tc)[256] = s_wh;
    const int kmax = wb >= (int)n ? 0 : min(kSBItems, ((int)n - wb + 63) / 64);  // the wave's non-empty items
    for (int tg = 0; tg < tps; tg += kTileGroup) {
        uint32_t cnt[kTileGroup];
#pragma unroll
        for (int k = 0; k < kTileGroup; k++) cnt[k] = 0u;
#pragma unroll
        for (int b = 0; b < kSBItems; b++) {
            if (b >= kmax) break;
            const uint32_t m = group_mask(gfp[b], tg, sg.shift);
#pragma unroll
            for (int k = 0; k < kTileGroup; k++) cnt[k] += (uint32_t)__popcll(__ballot((m >> k) & 1u));
        }
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < kTileGroup; k++)
                if (tg + k < tps) tc[w][tg + k] = cnt[k];
    }
    __syncthreads();
    if (w == 0) {
        uint32_t carry = 0;
        for (int t0 = 0; t0 < tps; t0 += 64) {
            const int tt = t0 + lane;
            uint32_t c = 0;
            if (tt < tps)
                for (int k = 0; k < kSBWaves; k++) c += tc[k][tt];
            uint32_t incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
                if (lane >= o) incl += v;
            }
            if (tt < tps) {
                uint32_t b = base_i[s] + carry + incl - c;
                const int x = ox + (tt & (side - 1)), y = oy + (tt >> sg.shift);
                if (x < gx && y < gy) ranges[y * gx + x] = make_uint2(b, b + c);
                for (int k = 0; k < kSBWaves; k++) {
                    const uint32_t ck = tc[k][tt];
                    tc[k][tt] = b;
                    b += ck;
                }
            }
            carry += (uint32_t)__shfl((int)incl, 63, 64);
        }
    }
    __syncthreads();
    SB_STAMP(4);
    for (int tg = 0; tg < tps; tg += kTileGroup) {
        uint32_t pk[kTileGroup];
#pragma unroll
        for (int k = 0; k < kTileGroup; k++) pk[k] = tg + k < tps ? tc[w][tg + k] : 0u;
#pragma unroll
        for (int b = 0; b < kSBItems; b++) {
            if (b >= kmax) break;
            const uint32_t m = group_mask(gfp[b], tg, sg.shift);
#pragma unroll
            for (int k = 0; k < kTileGroup; k++) {
                const bool hit = (m >> k) & 1u;
                const uint64_t bm = __ballot(hit);
                if (hit) point_list[pk[k] + (uint32_t)__popcll(bm & lt)] = gid[b];
                pk[k] += (uint32_t)__popcll(bm);
            }
        }
    }
    __syncthreads();
    SB_STAMP(5);
}

}  // namespace

int sort_cap() { return kSortCap; }

int debug_trace(int64_t *out, int n, int reset) {
    static unsigned long long v[2048 * 8];
    if (!out || n < 0) return -1;
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_sb_trace), sizeof(v)) != hipSuccess) return -3;
    if (reset) {
        static const unsigned long long z[2048 * 8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sb_trace), z, sizeof(z)) != hipSuccess) return -3;
    }
    int k = 0;
    for (; k < n && k < 2048 * 8; k++) out[k] = (int64_t)v[k];
    return k;
}

SBGrid sb_grid(int gx, int gy, int P) {
    SBGrid g;
    g.shift = 2;
    for (;;) {
        const int side = 1 << g.shift;
        g.nsbx = (gx + side - 1) / side;
        g.nsby = (gy + side - 1) / side;
        g.nsb = g.nsbx * g.nsby;
        if (g.nsb <= kMaxSB || (1 << (2 * (g.shift + 1))) > kMaxTilesPerSB) break;
        g.shift++;
    }
    // The per-(SB, chunk) counters are written column-major ([nsb][nchunks], one 4-B store per
    // SB and chunk): with too many chunks they outgrow the caches and every store becomes a partial
    // HBM line write (sb_count 282 us at 5.1M Gaussians and 1K-Gaussian chunks), so large P takes
    // bigger chunks (at most GSR_MAX_CHUNKS of them; too few, and sb_scatter's per-wave walks get
    // long).
    g.chunk = kSBChunk;
    while ((P + g.chunk - 1) / g.chunk > kMaxChunks) g.chunk *= 2;
    g.nchunks = (P + g.chunk - 1) / g.chunk;
    if (g.nchunks < 1) g.nchunks = 1;
    g.cper = sb_blocks(g) / 8 + (sb_blocks(g) % 8 != 0);
    g.ccols = GSR_CNT_XCD ? 8 * g.cper : g.nchunks;
    return g;
}

bool sb_grid_supported(const SBGrid &g) { return g.nsb <= kMaxSB; }

void launch_binning_count(int P, const Camera &cam, const GeomState &gs, bool index_order, const FrameWords &fw,
                          uint32_t *sb_order, uint32_t *zero_classes, hipStream_t s, uint32_t tb_split,
                          uint32_t *host_sblist) {
    const SBGrid &sg = gs.sb;
    if (P == 0 || cam.gx * cam.gy == 0) return;
    const size_t l1 = sizeof(uint32_t) * 2 * (size_t)sg.nsb;
    const uint2 *rects = index_order ? gs.rect8 : gs.drect;
    const uint32_t *rects4 = index_order ? gs.rect4 : drect4_of(gs);
    const uint32_t *culled = index_order ? nullptr : dsort_culled_word(gs);  // index order: culled rows anywhere
    hipLaunchKernelGGL(sb_count_kernel, dim3(sb_blocks(sg)), dim3(1024), l1, s, P, sg, rects, rects4, gs.sb_cnt_g,
                       gs.sb_cnt_i, culled);
    hipLaunchKernelGGL(sb_colscan_kernel, dim3(sg.nsb), dim3(kColThreads), 0, s, sg, gs.sb_cnt_g, gs.sb_cnt_i,
                       gs.sb_base_g, gs.sb_base_i, dsort_aux_word(gs), fw, sb_order, zero_classes,
                       index_order ? nullptr : gs.tb_flag, gs.tb_items, tb_split, host_sblist, P, culled);
}

void launch_binning_scatter(int P, const Camera &cam, const GeomState &gs, const BinningState &bs, bool index_order,
                            hipStream_t s) {
    const SBGrid &sg = gs.sb;
    if (P == 0 || cam.gx * cam.gy == 0) return;
    const size_t l3 = sizeof(uint32_t) * 3 * kScatterWaves * (size_t)sg.nsb;
    const uint2 *rects = index_order ? gs.rect8 : gs.drect;
    const uint32_t *rects4 = index_order ? gs.rect4 : drect4_of(gs);
    hipLaunchKernelGGL(sb_scatter_kernel, dim3(sb_blocks(sg)), dim3(64 * kScatterWaves), l3, s, P, sg,
                       index_order ? (const uint32_t *)nullptr : gs.order, rects, rects4, gs.sb_cnt_g, gs.sb_base_g,
                       bs.sblist, index_order ? bs.sblist4 : (uint4 *)nullptr, gs.dkey, bs.kdev, bs.cap,
                       index_order ? (const uint32_t *)nullptr : dsort_culled_word(gs));
}

void launch_binning_tiles(int P, const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                          bool local_sort, const uint32_t *maxsb, hipStream_t s, bool tb_split, hipStream_t split_stream) {
    const SBGrid &sg = gs.sb;
    const int T = cam.gx * cam.gy;
    if (T == 0) return;
    if (P == 0) {
        (void)hipMemsetAsync(is.ranges, 0, sizeof(uint2) * (size_t)T, s);
        return;
    }
    if (local_sort) {
        hipLaunchKernelGGL(sb_sort_bin_kernel, dim3(sg.nsb), dim3(kSBThreads), 0, s, sg, cam.gx, cam.gy, gs.sb_base_g,
                           gs.sb_base_i, bs.sblist4, bs.point_list, is.ranges, bs.kdev, bs.cap, maxsb);
        return;
    }
    const uint32_t *flag = tb_split ? gs.tb_flag : nullptr;
    if (tb_split) {
        // the long lists' slices beside tile_bin (the caller forked split_stream and joins it)
        const hipStream_t ss = split_stream ? split_stream : s;
        hipLaunchKernelGGL((tb_split_kernel<GSR_TB_WAVES_LONG, false>), dim3(kTBSplitBlocks), dim3(64 * GSR_TB_WAVES_LONG), 0,
                           ss, sg, cam.gx, cam.gy, gs.sb_base_g, gs.sb_base_i, bs.sblist, bs.point_list, is.ranges,
                           bs.kdev, bs.cap, gs.tb_flag, gs.tb_items, gs.tb_cnt);
        hipLaunchKernelGGL((tb_split_kernel<GSR_TB_WAVES_LONG, true>), dim3(kTBSplitBlocks), dim3(64 * GSR_TB_WAVES_LONG), 0,
                           ss, sg, cam.gx, cam.gy, gs.sb_base_g, gs.sb_base_i, bs.sblist, bs.point_list, is.ranges,
                           bs.kdev, bs.cap, gs.tb_flag, gs.tb_items, gs.tb_cnt);
    }
    // long superblock lists (large P): more waves per superblock, the 510-ish workgroups of a
    // 1080p frame are too few to hide the list walk's latency otherwise
    if ((int64_t)P > (int64_t)GSR_TB_LONG * sg.nsb)
        hipLaunchKernelGGL(tile_bin_kernel<GSR_TB_WAVES_LONG>, dim3(sg.nsb), dim3(64 * GSR_TB_WAVES_LONG), 0, s, sg, cam.gx, cam.gy, gs.sb_base_g,
                       gs.sb_base_i, bs.sblist, bs.point_list, is.ranges, bs.kdev, bs.cap, flag);
    else
        hipLaunchKernelGGL(tile_bin_kernel<GSR_TB_WAVES>, dim3(sg.nsb), dim3(64 * GSR_TB_WAVES), 0, s, sg, cam.gx, cam.gy, gs.sb_base_g,
                       gs.sb_base_i, bs.sblist, bs.point_list, is.ranges, bs.kdev, bs.cap, flag);
}

GSR_KSTAMP_READER(kstamp_read_binning)

}  // namespace gsr
