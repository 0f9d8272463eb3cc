// lod.hip -- the hierarchy LOD cut that feeds render_post:
// gaussian_hierarchy._C.expand_to_size and get_interpolation_weights, as the reference's callers
// use them (render_hierarchy.py:61-85, train_post.py:91-113, render_hierarchy_final.py:222-245).
//
// The gaussianhierarchy extension is not vendored in the reference, so this is a
// restatement of the published hierarchical-3DGS cut (Kerbl et al. 2024, "A Hierarchical 3D
// Gaussian Representation for Real-Time Rendering of Very Large Datasets", sec. 4) over the
// extension's in-memory layout:
//   node  (int32 x 7): depth, parent (-1 = root), start (first Gaussian), count_leafs,
//                      count_merged, start_children, count_children
//   box   (float  x 8): minn.xyz, size | maxx.xyz, (unused) -- minn.w holds the node's world size
// Projected size of a node seen from viewpoint v: +inf when v is inside the box, else
// size / |v - closest point of the box|.  A node is in the cut when it is small enough
// (size < target) and its parent is not (or it is a root): all its Gaussians are rendered; a node
// that is still too big renders only its leaf Gaussians (its children carry on).  The blend
// weight of a rendered node with its parent (sec. 4.3):
//   t = 1                                   root, or parent size > 2 target
//   t = max(1 - max(0, target - s0) / (sp - s0), 0),  s0 = max(sp / 2, s), when sp > s0
// and num_kids = the parent's child count.  Parity is pinned to the C restatement
// (oracle/gs_oracle.c gso_expand_to_size / gso_interpolation_weights), not to the unvendored
// extension ("parity unpinned" against gaussianhierarchy itself).
//
// MI355X mapping: expand_to_size is one launch (lod_cut_kernel): a workgroup per 1024 nodes stages
// the nodes through LDS (4 KiB per load instruction), reads each node's box (and its parent's box
// and first Gaussian where the decision needs them; parents of consecutive nodes are consecutive in
// a level-ordered hierarchy, so they stay in L2), scans the counts, takes its offset by a
// decoupled lookback over the preceding tiles and writes (render index, parent's first Gaussian,
// node) per rendered Gaussian.  The host reads the total once (the value expand_to_size returns).
#include <algorithm>
#include <cfloat>
#include <cstring>
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_hier.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

struct HNode {
    int depth, parent, start, count_leafs, count_merged, start_children, count_children;
};
static_assert(sizeof(HNode) == 28, "node layout: 7 int32");

struct HBox {
    float4 minn, maxx;
};

__device__ __forceinline__ HNode load_node(const int *__restrict__ nodes, int64_t i) {
    const int *p = nodes + 7 * i;
    return HNode{p[0], p[1], p[2], p[3], p[4], p[5], p[6]};
}

// size / distance of the box from the viewpoint (+FLT_MAX inside); the oracle restates this order
__device__ __forceinline__ float node_size(const HBox &b, float vx, float vy, float vz) {
    if (vx >= b.minn.x && vx <= b.maxx.x && vy >= b.minn.y && vy <= b.maxx.y && vz >= b.minn.z && vz <= b.maxx.z)
        return FLT_MAX;
    const float cx = fmaxf(b.minn.x, fminf(b.maxx.x, vx));
    const float cy = fmaxf(b.minn.y, fminf(b.maxx.y, vy));
    const float cz = fmaxf(b.minn.z, fminf(b.maxx.z, vz));
    const float dx = vx - cx, dy = vy - cy, dz = vz - cz;
    const float d = sqrtf(dx * dx + dy * dy + dz * dz);
    return b.minn.w / d;
}

__device__ __forceinline__ HBox load_box(const float *__restrict__ boxes, int64_t i) {
    const float4 *p = reinterpret_cast<const float4 *>(boxes) + 2 * i;
    return HBox{p[0], p[1]};
}

// expand_to_size in two launches over tiles of kCutTile nodes, with no wait between workgroups:
//   lod_cut_count_kernel  per tile: each node's cut count (the node's box; the parent's box and first
//                         Gaussian where the decision needs them), the counts' exclusive scan, and
//                         a 16-byte record {offset in the tile, first Gaussian, parent's first
//                         Gaussian, node in the tile} per rendered node, compacted in node order
//                         into the tile's slot; the tile's sum stored and added to its group's
//                         (groups of kCutGroup tiles, one no-return atomic per tile);
//   lod_cut_write_kernel  per tile: its offset (the earlier groups' sums plus the group's earlier
//                         tiles', one round of loads; past kCutDirectGroups groups the group sums
//                         are scanned by one workgroup in between) and its records' entries there.
// The nodes and boxes are read once; the records (16 B per rendered node) are written and read once.
// A count pass, a library scan and a write pass read the nodes twice and a 4-byte count per node
// three times (config 5's 50M nodes: 0.66 + 0.18 + 0.21 ms); one pass with a decoupled lookback
// (measured 0.92-0.97 ms) waits on the slowest predecessor tile of every tile.
#ifndef GSR_CUT_ITEMS
#define GSR_CUT_ITEMS 4
#endif
constexpr int kCutThreads = 256, kCutItems = GSR_CUT_ITEMS, kCutTile = kCutThreads * kCutItems;
constexpr int kCutWaves = kCutThreads / kWave;
constexpr int kCutTotal = 0, kCutHead = 4;  // control words (uint64)

constexpr int kCutGroup = 256;  // tiles per group: a tile adds its group's earlier tiles to the earlier groups' sum
// Up to this many groups (16M nodes) each write workgroup sums the earlier groups itself (one load
// per thread); past it a one-workgroup scan of the group sums runs between the two launches, so the
// write launch's work stays linear in the node count (config 5's 50M nodes take the scan).
constexpr int64_t kCutDirectGroups = 64;
struct CutScratch {
    uint64_t *ctl;         // [kCutHead + ngroups]: control words, then the group sums; zeroed per call
    uint32_t *tile_sum;    // [ntiles] entries per tile
    uint32_t *tile_nrec;   // [ntiles] rendered nodes per tile
    uint64_t *group_off;   // [ngroups] exclusive scan of the group sums (past kCutDirectGroups groups)
    uint4 *recs;           // [ntiles * kCutTile]
};
__host__ __device__ inline int64_t cut_groups(int64_t ntiles) { return (ntiles + kCutGroup - 1) / kCutGroup; }

__host__ __device__ inline size_t cut_scratch_bytes(int64_t ntiles, CutScratch *sc, char *base) {
    size_t at = 0;
    const auto take = [&](size_t bytes) {
        const size_t o = at;
        at = align_up(at + bytes, 256);
        return base ? base + o : nullptr;
    };
    char *ctl = take(sizeof(uint64_t) * (size_t)(kCutHead + cut_groups(ntiles)));
    char *sum = take(sizeof(uint32_t) * (size_t)ntiles);
    char *nrec = take(sizeof(uint32_t) * (size_t)ntiles);
    char *goff = take(sizeof(uint64_t) * (size_t)cut_groups(ntiles));
    char *recs = take(sizeof(uint4) * (size_t)ntiles * kCutTile);
    if (sc) *sc = CutScratch{reinterpret_cast<uint64_t *>(ctl), reinterpret_cast<uint32_t *>(sum),
                             reinterpret_cast<uint32_t *>(nrec), reinterpret_cast<uint64_t *>(goff),
                             reinterpret_cast<uint4 *>(recs)};
    return at;
}

__global__ __launch_bounds__(kCutThreads) void lod_cut_count_kernel(int64_t N, int64_t ntiles, const int *__restrict__ nodes,
                                                                    const float *__restrict__ boxes, float target,
                                                                    const float *__restrict__ viewpoint, CutScratch sc) {
    __shared__ uint32_t s_cnt[kCutTile];  // counts, then exclusive offsets in the tile
    __shared__ uint32_t s_wsum[kCutWaves];
    __shared__ uint32_t s_wc[kCutItems * kCutWaves];  // rendered nodes per (item, wave)
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const int64_t tile = blockIdx.x, t0 = tile * kCutTile;
    const int n = (int)min((int64_t)kCutTile, N - t0);
    const float vx = viewpoint[0], vy = viewpoint[1], vz = viewpoint[2];
    const int *src = nodes + 7 * t0;
    // node q = k * kCutThreads + tid: its box (2 KiB contiguous per wave and instruction pair) and
    // the four fields the cut reads
    HBox b[kCutItems];
    int f_par[kCutItems], f_cl[kCutItems], f_cm[kCutItems], start[kCutItems];
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        const int q = k * kCutThreads + tid;
        b[k] = q < n ? load_box(boxes, t0 + q) : HBox{};
        f_par[k] = q < n ? src[7 * q + 1] : -1;
        start[k] = q < n ? src[7 * q + 2] : 0;
        f_cl[k] = q < n ? src[7 * q + 3] : 0;
        f_cm[k] = q < n ? src[7 * q + 4] : 0;
    }
    // cut_count's decision (the parent's box only for a node that is small enough) and the parent's
    // first Gaussian for a node that may render, both loaded in one round
    int c[kCutItems], pg[kCutItems];
    bool ptest[kCutItems];
    HBox pb[kCutItems];
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        const int q = k * kCutThreads + tid;
        const bool big = q < n && node_size(b[k], vx, vy, vz) >= target;
        c[k] = q >= n ? 0 : big ? f_cl[k] : f_cl[k] + f_cm[k];  // small: cl + cm unless the parent is small too
        ptest[k] = q < n && !big && f_par[k] >= 0;
        pb[k] = ptest[k] ? load_box(boxes, f_par[k]) : HBox{};
        pg[k] = f_par[k] >= 0 && c[k] > 0 ? nodes[7 * (int64_t)f_par[k] + 2] : -1;
    }
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        if (ptest[k] && node_size(pb[k], vx, vy, vz) < target) c[k] = 0;  // its parent is in the cut or below
        s_cnt[k * kCutThreads + tid] = (uint32_t)c[k];                      // 0 past the tile's end
        const uint64_t m = __ballot(c[k] > 0);
        if (lane == 0) s_wc[k * kCutWaves + w] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    // exclusive scan of the counts in node order: thread tid holds nodes kCutItems tid .. + kCutItems - 1
    uint32_t cv[kCutItems], own = 0;
#pragma unroll
    for (int j = 0; j < kCutItems; j++) {
        cv[j] = s_cnt[kCutItems * tid + j];
        own += cv[j];
    }
    uint32_t incl = own;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o, kWave);
        if (lane >= o) incl += t;
    }
    if (lane == kWave - 1) s_wsum[w] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kCutWaves; k++) {
        before += k < w ? s_wsum[k] : 0u;
        total += s_wsum[k];
    }
    uint32_t ex = before + incl - own;
#pragma unroll
    for (int j = 0; j < kCutItems; j++) {
        s_cnt[kCutItems * tid + j] = ex;
        ex += cv[j];
    }
    __syncthreads();
    // the rendered nodes' records in node order: rank = rendered nodes of the earlier (item, wave)
    // groups + the lower lanes of this one
    uint4 *slot = sc.recs + (size_t)tile * kCutTile;
    uint32_t nrec = 0;
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        uint32_t rb = 0;
#pragma unroll
        for (int g = 0; g < kCutItems * kCutWaves; g++) {
            const uint32_t v = s_wc[g];
            rb += g < k * kCutWaves + w ? v : 0u;
            nrec += k == 0 ? v : 0u;
        }
        const uint64_t m = __ballot(c[k] > 0);
        const int q = k * kCutThreads + tid;
        if (c[k] > 0) {
            const uint32_t rank = rb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            slot[rank] = make_uint4(s_cnt[q], (uint32_t)start[k], (uint32_t)pg[k], (uint32_t)q);
        }
    }
    if (tid == 0) {
        // read by the write launch: the tile's sum and record count, and its group's sum (a
        // no-return agent-scope atomic; nothing here waits for it)
        sc.tile_sum[tile] = total;
        sc.tile_nrec[tile] = nrec;
        if (total) (void)__hip_atomic_fetch_add(&sc.ctl[kCutHead + tile / kCutGroup], (uint64_t)total, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Past kCutDirectGroups groups: the group offsets in one workgroup, kScanThreads groups at a time.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void lod_cut_scan_kernel(int64_t ngroups, CutScratch sc) {
    __shared__ uint64_t s_w[kScanThreads / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    uint64_t carry = 0;
    for (int64_t b0 = 0; b0 < ngroups; b0 += kScanThreads) {
        const int64_t gi = b0 + tid;
        const uint64_t v = gi < ngroups ? sc.ctl[kCutHead + gi] : 0ull;
        uint64_t inc = v;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const uint64_t u = __shfl_up(inc, o, kWave);
            if (lane >= o) inc += u;
        }
        __syncthreads();  // the previous round's reads of s_w are done
        if (lane == kWave - 1) s_w[w] = inc;
        __syncthreads();
        uint64_t before = 0, tot = 0;
        for (int k = 0; k < kScanThreads / kWave; k++) {
            before += k < w ? s_w[k] : 0ull;
            tot += s_w[k];
        }
        if (gi < ngroups) sc.group_off[gi] = carry + before + inc - v;
        carry += tot;
    }
}

__global__ __launch_bounds__(kCutThreads) void lod_cut_write_kernel(int64_t ntiles, CutScratch sc,
                                                                    int *__restrict__ render_indices,
                                                                    int *__restrict__ parent_indices,
                                                                    int *__restrict__ nodes_for_render, int64_t capacity) {
    __shared__ uint32_t s_off[kCutTile + 1];
    __shared__ uint64_t s_red[kCutWaves];
    const int64_t tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    // the tile's offset, in one round of loads: the sums of the earlier groups and of the group's
    // earlier tiles
    const int64_t g = tile / kCutGroup, g0 = g * kCutGroup;
    static_assert(kCutGroup == kCutThreads, "one earlier tile per thread");
    const int nrec = (int)sc.tile_nrec[tile];
    uint64_t acc = g0 + tid < tile ? sc.tile_sum[g0 + tid] : 0u;
    if (cut_groups(ntiles) > kCutDirectGroups) {
        if (tid == 0) acc += sc.group_off[g];
    } else {
        for (int64_t j = tid; j < g; j += kCutThreads) acc += sc.ctl[kCutHead + j];
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, kWave);
    if (lane == 0) s_red[w] = acc;
    __syncthreads();
    uint64_t base = 0;
#pragma unroll
    for (int k = 0; k < kCutWaves; k++) base += s_red[k];
    if (tile == ntiles - 1 && tid == 0) sc.ctl[kCutTotal] = base + sc.tile_sum[tile];  // read by the host
    if (nrec == 0) return;
    const uint4 *slot = sc.recs + (size_t)tile * kCutTile;
    uint4 r[kCutItems];
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        const int i = k * kCutThreads + tid;
        r[k] = i < nrec ? slot[i] : make_uint4(0u, 0u, 0u, 0u);
        if (i < nrec) s_off[i] = r[k].x;
    }
    if (tid == 0) s_off[nrec] = sc.tile_sum[tile];
    __syncthreads();
    // record i's entries: from its offset up to the next record's (the tile's sum after the last)
#pragma unroll
    for (int k = 0; k < kCutItems; k++) {
        const int i = k * kCutThreads + tid;
        if (i >= nrec) continue;
        const uint32_t c = s_off[i + 1] - r[k].x;
        const int64_t at0 = (int64_t)(base + r[k].x);
        const int node = (int)(tile * kCutTile + (int64_t)r[k].w);
        for (uint32_t e = 0; e < c; e++) {
            const int64_t at = at0 + (int64_t)e;
            if (at >= capacity) break;
            render_indices[at] = (int)r[k].y + (int)e;
            parent_indices[at] = (int)r[k].z;
            nodes_for_render[at] = node;
        }
    }
}

__global__ __launch_bounds__(256) void lod_weights_kernel(int64_t n, const int *__restrict__ node_indices,
                                                          float target, const int *__restrict__ nodes,
                                                          const float *__restrict__ boxes, float vx, float vy,
                                                          float vz, float *__restrict__ weights,
                                                          int *__restrict__ num_kids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int id = node_indices[i];
    const int parent = nodes[7 * (int64_t)id + 1];
    float t = 1.f;
    int kids = 1;
    if (parent >= 0) {
        kids = nodes[7 * (int64_t)parent + 6];
        const float sp = node_size(load_box(boxes, parent), vx, vy, vz);
        if (!(sp > 2.f * target)) {
            const float s = node_size(load_box(boxes, id), vx, vy, vz);
            const float s0 = fmaxf(0.5f * sp, s);
            const float diff = sp - s0;
            if (diff > 0.f) {
                const float tdiff = fmaxf(0.f, target - s0);
                t = fmaxf(1.f - tdiff / diff, 0.f);
            }
        }
    }
    weights[i] = t;
    num_kids[i] = kids;
}

int fail_lod(int code, const std::string &m) {
    set_last_error(m);
    return code;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_expand_to_size_scratch_bytes(int64_t N) {
    const int64_t ntiles = (std::max<int64_t>(N, 1) + kCutTile - 1) / kCutTile;
    return cut_scratch_bytes(ntiles, nullptr, nullptr) + 256;
}

int gsr_expand_to_size(int64_t N, const int *nodes, const float *boxes, float target_size, const float *viewpoint,
                       int *render_indices, int *parent_indices, int *nodes_for_render_indices, int64_t capacity,
                       void *scratch, size_t scratch_bytes, int64_t *to_render, void *stream) {
    if (to_render) *to_render = 0;
    if (N < 0 || N > INT32_MAX) return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_expand_to_size: N out of range");
    if (N == 0) return GSR_OK;
    if (!nodes || !boxes || !viewpoint || !render_indices || !parent_indices || !nodes_for_render_indices ||
        !scratch || !to_render)
        return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_expand_to_size: NULL pointer");
    if (scratch_bytes < gsr_expand_to_size_scratch_bytes(N))
        return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_expand_to_size: scratch too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t ntiles = (N + kCutTile - 1) / kCutTile;
    CutScratch sc;
    (void)cut_scratch_bytes(ntiles, &sc, reinterpret_cast<char *>(align_up(reinterpret_cast<uintptr_t>(scratch), 256)));
    // the done counter, the total and the group sums
    hipError_t e = hipMemsetAsync(sc.ctl, 0, sizeof(uint64_t) * (size_t)(kCutHead + cut_groups(ntiles)), s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(lod_cut_count_kernel, dim3((unsigned)ntiles), dim3(kCutThreads), 0, s, N, ntiles, nodes,
                           boxes, target_size, viewpoint, sc);
        if (cut_groups(ntiles) > kCutDirectGroups)
            hipLaunchKernelGGL(lod_cut_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, cut_groups(ntiles), sc);
        hipLaunchKernelGGL(lod_cut_write_kernel, dim3((unsigned)ntiles), dim3(kCutThreads), 0, s, ntiles, sc, render_indices,
                           parent_indices, nodes_for_render_indices, capacity < 0 ? (int64_t)0 : capacity);
        e = hipGetLastError();
    }
    uint64_t words[kCutHead] = {};
    if (e == hipSuccess) e = hipMemcpyAsync(words, sc.ctl, sizeof(words), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fail_lod(GSR_ERR_DEVICE, std::string("gsr_expand_to_size: ") + hipGetErrorString(e));
    const int64_t total = (int64_t)words[kCutTotal];
    *to_render = total;
    if (total > capacity)
        return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_expand_to_size: the cut needs " + std::to_string(total) +
                                                      " entries, the output arrays hold " + std::to_string(capacity));
    return GSR_OK;
}

int gsr_interpolation_weights(int64_t n, const int *node_indices, float target_size, const int *nodes,
                              const float *boxes, float vx, float vy, float vz, float *weights, int *num_kids,
                              void *stream) {
    if (n < 0) return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_interpolation_weights: n < 0");
    if (n == 0) return GSR_OK;
    if (!node_indices || !nodes || !boxes || !weights || !num_kids)
        return fail_lod(GSR_ERR_INVALID_ARGUMENT, "gsr_interpolation_weights: NULL pointer");
    hipLaunchKernelGGL(lod_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), n, node_indices, target_size, nodes, boxes, vx, vy, vz,
                       weights, num_kids);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail_lod(GSR_ERR_DEVICE, std::string("gsr_interpolation_weights: ") + hipGetErrorString(e));
    return GSR_OK;
}

}  // extern "C"
