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
// MI355X mapping: one lane per node; the count pass reads the node (28 B), its box and its
// parent's box (32 B each; parents of consecutive nodes are consecutive in a level-ordered
// hierarchy, so the parent boxes stay in L2), a rocPRIM decoupled-lookback scan turns the counts
// into output offsets, and the write pass emits (render index, parent's first Gaussian, node) per
// rendered Gaussian.  The host reads the total once (the value expand_to_size returns).
#include <cfloat>
#include <cstring>
#include <string>

#include <rocprim/rocprim.hpp>

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

__device__ __forceinline__ int cut_count(const int *__restrict__ nodes, const float *__restrict__ boxes, int64_t i,
                                         float target, float vx, float vy, float vz) {
    const HNode n = load_node(nodes, i);
    const float s = node_size(load_box(boxes, i), vx, vy, vz);
    if (s >= target) return n.count_leafs;  // still too big: its children are expanded
    if (n.parent < 0 || node_size(load_box(boxes, n.parent), vx, vy, vz) >= target)
        return n.count_leafs + n.count_merged;  // first small node on its path: the cut
    return 0;
}

__global__ __launch_bounds__(256) void lod_count_kernel(int64_t N, const int *__restrict__ nodes,
                                                        const float *__restrict__ boxes, float target,
                                                        const float *__restrict__ viewpoint,
                                                        int *__restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    counts[i] = cut_count(nodes, boxes, i, target, viewpoint[0], viewpoint[1], viewpoint[2]);
}

__global__ __launch_bounds__(256) void lod_put_kernel(int64_t N, const int *__restrict__ nodes,
                                                      const int *__restrict__ counts, const int *__restrict__ incl,
                                                      int *__restrict__ render_indices, int *__restrict__ parent_indices,
                                                      int *__restrict__ nodes_for_render, int64_t capacity) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    // a cut longer than the output arrays writes nothing (the host reports the length it needs)
    if ((int64_t)incl[N - 1] > capacity) return;
    // the count from the inclusive scan (its neighbour is in the same line): no second 4-B-per-node
    // array read (200 MB at 50M nodes)
    const int hi = incl[i], off = i > 0 ? incl[i - 1] : 0;
    const int c = hi - off;
    if (c == 0) return;
    (void)counts;
    const HNode n = load_node(nodes, i);
    const int pg = n.parent < 0 ? -1 : nodes[7 * (int64_t)n.parent + 2];  // the parent's first Gaussian
    for (int k = 0; k < c; k++) {
        render_indices[off + k] = n.start + k;
        parent_indices[off + k] = pg;
        nodes_for_render[off + k] = (int)i;
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
    size_t tmp = 0;
    (void)rocprim::inclusive_scan(nullptr, tmp, (const int *)nullptr, (int *)nullptr, (size_t)(N > 0 ? N : 1),
                            rocprim::plus<int>());
    return align_up(sizeof(int) * (size_t)(N > 0 ? N : 1), 256) * 2 + align_up(tmp, 256) + 256;
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
    char *base = static_cast<char *>(scratch);
    const size_t a = align_up(sizeof(int) * (size_t)N, 256);
    int *counts = reinterpret_cast<int *>(base);
    int *incl = reinterpret_cast<int *>(base + a);
    void *tmp = base + 2 * a;
    size_t tmp_bytes = scratch_bytes - 2 * a;
    const unsigned blocks = (unsigned)((N + 255) / 256);
    hipLaunchKernelGGL(lod_count_kernel, dim3(blocks), dim3(256), 0, s, N, nodes, boxes, target_size, viewpoint, counts);
    if (rocprim::inclusive_scan(tmp, tmp_bytes, counts, incl, (size_t)N, rocprim::plus<int>(), s) != hipSuccess)
        return fail_lod(GSR_ERR_DEVICE, "gsr_expand_to_size: scan failed");
    hipLaunchKernelGGL(lod_put_kernel, dim3(blocks), dim3(256), 0, s, N, nodes, counts, incl, render_indices,
                       parent_indices, nodes_for_render_indices, capacity < 0 ? (int64_t)0 : capacity);
    int total = 0;
    hipError_t e = hipMemcpyAsync(&total, incl + (N - 1), sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) return fail_lod(GSR_ERR_DEVICE, std::string("gsr_expand_to_size: ") + hipGetErrorString(e));
    *to_render = total;
    if ((int64_t)total > capacity)
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
