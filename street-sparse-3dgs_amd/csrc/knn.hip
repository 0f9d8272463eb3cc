// knn.hip -- mean squared distance to the 3 nearest neighbours of every point (include/gsr_knn.h),
// the initial-scale source of GaussianModel.create_from_pcd (scene/gaussian_model.py:207:
// dist2 = clamp_min(distCUDA2(points), 1e-7)).  The reference calls
// simple_knn._C.distCUDA2 (submodules/simple-knn, not vendored): an exact 3-NN over
// Morton-ordered boxes.  Same result here, organised for gfx950:
//
//   1. bounding box (block reduce + ordered-uint atomics), 30-bit Morton keys, rocPRIM pair sort
//   2. the sorted points as float4, one AABB per 64 consecutive points (a "box" = one wave's
//      worth) and one per 64 boxes (a "superbox")
//   3. one wave per box of 64 queries: its own box and the two neighbours in Morton order first
//      (a tight bound early), then every superbox / box whose AABB distance to the query box's
//      AABB does not exceed the wave's current worst 3rd-best distance.  A visited box is read
//      with one coalesced load and its 64 candidates are broadcast with v_readlane, so the
//      distance tests run on scalar operands.
//
// Exactness: the box-to-box gap g is computed with the point distance's own operation order on
// per-axis gaps that bound the point differences from below, and float rounding is monotone, so
// the AABB distance never exceeds a true candidate distance: pruning is conservative and the
// result is the exact 3 smallest squared distances (self excluded by index, duplicates count).
#include <cfloat>
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_knn.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

constexpr int kBox = 64;  // points per box = lanes per wave; boxes per superbox
constexpr int kKnnWaves = 4;

__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ float wave_minf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// simple-knn's updateKBest<3>: insertion into the ascending best list (strict >)
__device__ __forceinline__ void update3(float d, float &b0, float &b1, float &b2) {
    if (b0 > d) { const float t = b0; b0 = d; d = t; }
    if (b1 > d) { const float t = b1; b1 = d; d = t; }
    if (b2 > d) b2 = d;
}

// squared distance in a fixed order (the oracle's): fma(dz, dz, fma(dy, dy, dx * dx))
__device__ __forceinline__ float sqd(float dx, float dy, float dz) { return fmaf(dz, dz, fmaf(dy, dy, dx * dx)); }

__device__ __forceinline__ float gap(float amin, float amax, float bmin, float bmax) {
    return fmaxf(0.f, fmaxf(bmin - amax, amin - bmax));
}

__device__ __forceinline__ float box_dist(const float4 &amin, const float4 &amax, const float4 &bmin,
                                          const float4 &bmax) {
    return sqd(gap(amin.x, amax.x, bmin.x, bmax.x), gap(amin.y, amax.y, bmin.y, bmax.y),
               gap(amin.z, amax.z, bmin.z, bmax.z));
}

__global__ __launch_bounds__(256) void knn_bbox_kernel(int64_t N, const float *__restrict__ p, uint32_t *bb) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const float v = p[3 * i + k];
            mn[k] = fminf(mn[k], v);
            mx[k] = fmaxf(mx[k], v);
        }
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
        mn[k] = wave_minf(mn[k]);
        mx[k] = wave_maxf(mx[k]);
    }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 3; k++) {
            atomicMin(&bb[k], f2ord(mn[k]));
            atomicMax(&bb[3 + k], f2ord(mx[k]));
        }
    }
}

__global__ void knn_bbox_init_kernel(uint32_t *bb) {
    if (threadIdx.x < 3) {
        bb[threadIdx.x] = 0xffffffffu;
        bb[3 + threadIdx.x] = 0u;
    }
}

__device__ __forceinline__ uint32_t spread10(uint32_t x) {  // 10 bits -> every third bit
    x &= 0x3ffu;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

__device__ __forceinline__ uint32_t quant10(float v, float lo, float hi) {
    const float ext = hi - lo;
    if (!(ext > 0.f)) return 0u;
    const float t = (v - lo) / ext * 1023.f;
    return (uint32_t)fminf(fmaxf(t, 0.f), 1023.f);
}

__global__ __launch_bounds__(256) void knn_morton_kernel(int64_t N, const float *__restrict__ p,
                                                         const uint32_t *__restrict__ bb, uint32_t *__restrict__ key,
                                                         uint32_t *__restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float lo[3] = {ord2f(bb[0]), ord2f(bb[1]), ord2f(bb[2])};
    const float hi[3] = {ord2f(bb[3]), ord2f(bb[4]), ord2f(bb[5])};
    const uint32_t x = quant10(p[3 * i], lo[0], hi[0]), y = quant10(p[3 * i + 1], lo[1], hi[1]),
                   z = quant10(p[3 * i + 2], lo[2], hi[2]);
    key[i] = spread10(x) | (spread10(y) << 1) | (spread10(z) << 2);
    idx[i] = (uint32_t)i;
}

// sorted float4 points and one AABB per box (one wave per box)
__global__ __launch_bounds__(256) void knn_boxes_kernel(int64_t N, const float *__restrict__ p,
                                                        const uint32_t *__restrict__ sidx, float4 *__restrict__ pts,
                                                        float4 *__restrict__ boxes, int64_t nb) {
    const int64_t b = (int64_t)blockIdx.x * kKnnWaves + (threadIdx.x >> 6);
    if (b >= nb) return;
    const int64_t i = b * kBox + (threadIdx.x & 63);
    float4 v = make_float4(FLT_MAX, FLT_MAX, FLT_MAX, 0.f);
    float4 w = make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f);
    if (i < N) {
        const uint32_t s = sidx[i];
        const float4 q = make_float4(p[3 * (size_t)s], p[3 * (size_t)s + 1], p[3 * (size_t)s + 2], 0.f);
        pts[i] = q;
        v = q;
        w = q;
    }
    v = make_float4(wave_minf(v.x), wave_minf(v.y), wave_minf(v.z), 0.f);
    w = make_float4(wave_maxf(w.x), wave_maxf(w.y), wave_maxf(w.z), 0.f);
    if ((threadIdx.x & 63) == 0) {
        boxes[2 * b] = v;
        boxes[2 * b + 1] = w;
    }
}

// one AABB per 64 boxes (one wave per superbox)
__global__ __launch_bounds__(256) void knn_superboxes_kernel(const float4 *__restrict__ boxes, int64_t nb,
                                                             float4 *__restrict__ sboxes, int64_t nsb) {
    const int64_t sb = (int64_t)blockIdx.x * kKnnWaves + (threadIdx.x >> 6);
    if (sb >= nsb) return;
    const int64_t b = sb * kBox + (threadIdx.x & 63);
    float4 v = make_float4(FLT_MAX, FLT_MAX, FLT_MAX, 0.f), w = make_float4(-FLT_MAX, -FLT_MAX, -FLT_MAX, 0.f);
    if (b < nb) {
        v = boxes[2 * b];
        w = boxes[2 * b + 1];
    }
    v = make_float4(wave_minf(v.x), wave_minf(v.y), wave_minf(v.z), 0.f);
    w = make_float4(wave_maxf(w.x), wave_maxf(w.y), wave_maxf(w.z), 0.f);
    if ((threadIdx.x & 63) == 0) {
        sboxes[2 * sb] = v;
        sboxes[2 * sb + 1] = w;
    }
}

struct Best {
    float b0 = FLT_MAX, b1 = FLT_MAX, b2 = FLT_MAX;
};

// all 64 lanes test the (up to) 64 candidates of box cb against their own query
__device__ __forceinline__ void visit_box(int64_t N, const float4 *__restrict__ pts, int64_t cb, int64_t self,
                                          const float4 &q, Best &B) {
    const int64_t base = cb * kBox;
    const int lane = threadIdx.x & 63;
    const float4 c = base + lane < N ? pts[base + lane] : make_float4(0.f, 0.f, 0.f, 0.f);
    const int cnt = (int)(N - base < kBox ? N - base : kBox);
    for (int j = 0; j < cnt; j++) {
        const float px = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.x), j));
        const float py = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.y), j));
        const float pz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c.z), j));
        if (base + j == self) continue;
        update3(sqd(px - q.x, py - q.y, pz - q.z), B.b0, B.b1, B.b2);
    }
}

__global__ __launch_bounds__(64 * kKnnWaves) void knn_query_kernel(int64_t N, const float4 *__restrict__ pts,
                                                                   const float4 *__restrict__ boxes, int64_t nb,
                                                                   const float4 *__restrict__ sboxes, int64_t nsb,
                                                                   const uint32_t *__restrict__ sidx,
                                                                   float *__restrict__ out) {
    const int64_t b = (int64_t)blockIdx.x * kKnnWaves + (threadIdx.x >> 6);
    if (b >= nb) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t self = b * kBox + lane;
    const bool valid = self < N;
    const float4 q = valid ? pts[self] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 qmin = boxes[2 * b], qmax = boxes[2 * b + 1];
    Best B;
    // own box and its Morton neighbours first: a tight bound before the scan
    visit_box(N, pts, b, self, q, B);
    if (b > 0) visit_box(N, pts, b - 1, self, q, B);
    if (b + 1 < nb) visit_box(N, pts, b + 1, self, q, B);
    float bound = wave_maxf(valid ? B.b2 : 0.f);
    for (int64_t s0 = 0; s0 < nsb; s0 += kBox) {
        const int64_t s = s0 + lane;
        bool pass = false;
        if (s < nsb) pass = !(box_dist(qmin, qmax, sboxes[2 * s], sboxes[2 * s + 1]) > bound);
        uint64_t sm = __ballot(pass);
        while (sm) {
            const int64_t S = s0 + __builtin_ctzll(sm);
            sm &= sm - 1;
            const int64_t cb = S * kBox + lane;
            bool bp = false;
            if (cb < nb && (cb < b - 1 || cb > b + 1))
                bp = !(box_dist(qmin, qmax, boxes[2 * cb], boxes[2 * cb + 1]) > bound);
            uint64_t bm = __ballot(bp);
            while (bm) {
                const int64_t C = S * kBox + __builtin_ctzll(bm);
                bm &= bm - 1;
                if (box_dist(qmin, qmax, boxes[2 * C], boxes[2 * C + 1]) > bound) continue;  // bound tightened
                visit_box(N, pts, C, self, q, B);
                bound = wave_maxf(valid ? B.b2 : 0.f);
            }
        }
    }
    if (valid) out[sidx[self]] = (B.b0 + B.b1 + B.b2) / 3.0f;
}

struct KnnLayout {
    uint32_t *bb, *key, *key_s, *idx, *idx_s;
    float4 *pts, *boxes, *sboxes;
    void *tmp;
    size_t tmp_bytes, total;
};

KnnLayout knn_layout(char *base, int64_t N) {
    KnnLayout L{};
    const int64_t nb = (N + kBox - 1) / kBox, nsb = (nb + kBox - 1) / kBox;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off = align_up(off + bytes, 256);
        return p;
    };
    L.bb = reinterpret_cast<uint32_t *>(take(8 * sizeof(uint32_t)));
    L.key = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * N));
    L.key_s = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * N));
    L.idx = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * N));
    L.idx_s = reinterpret_cast<uint32_t *>(take(sizeof(uint32_t) * N));
    L.pts = reinterpret_cast<float4 *>(take(sizeof(float4) * N));
    L.boxes = reinterpret_cast<float4 *>(take(sizeof(float4) * 2 * nb));
    L.sboxes = reinterpret_cast<float4 *>(take(sizeof(float4) * 2 * nsb));
    L.tmp_bytes = sort_pairs_temp_bytes((size_t)N, 30);
    L.tmp = take(L.tmp_bytes);
    L.total = off;
    return L;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_knn_scratch_bytes(int64_t N) {
    if (N <= 0) return 0;
    return knn_layout(nullptr, N).total;
}

int gsr_knn_mean_dist2(int64_t N, const float *points, float *out, void *scratch, void *stream) {
    if (N < 0 || N > 0xffffffffLL || (N > 0 && (!points || !out || !scratch))) {
        set_last_error("gsr_knn_mean_dist2: bad size (0 <= N < 2^32) or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (N == 0) return GSR_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const KnnLayout L = knn_layout(static_cast<char *>(scratch), N);
    const int64_t nb = (N + kBox - 1) / kBox, nsb = (nb + kBox - 1) / kBox;
    hipLaunchKernelGGL(knn_bbox_init_kernel, dim3(1), dim3(64), 0, s, L.bb);
    const int64_t gb = (N + 255) / 256;
    hipLaunchKernelGGL(knn_bbox_kernel, dim3((unsigned)(gb < 2048 ? gb : 2048)), dim3(256), 0, s, N, points, L.bb);
    hipLaunchKernelGGL(knn_morton_kernel, dim3((unsigned)gb), dim3(256), 0, s, N, points, L.bb, L.key, L.idx);
    hipError_t e = sort_pairs(L.tmp, L.tmp_bytes, L.key, L.key_s, L.idx, L.idx_s, (size_t)N, 30, s);
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_knn_mean_dist2: sort: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    hipLaunchKernelGGL(knn_boxes_kernel, dim3((unsigned)((nb + kKnnWaves - 1) / kKnnWaves)), dim3(64 * kKnnWaves), 0,
                       s, N, points, L.idx_s, L.pts, L.boxes, nb);
    hipLaunchKernelGGL(knn_superboxes_kernel, dim3((unsigned)((nsb + kKnnWaves - 1) / kKnnWaves)),
                       dim3(64 * kKnnWaves), 0, s, L.boxes, nb, L.sboxes, nsb);
    hipLaunchKernelGGL(knn_query_kernel, dim3((unsigned)((nb + kKnnWaves - 1) / kKnnWaves)), dim3(64 * kKnnWaves), 0,
                       s, N, L.pts, L.boxes, nb, L.sboxes, nsb, L.idx_s, out);
    e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_knn_mean_dist2: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"
