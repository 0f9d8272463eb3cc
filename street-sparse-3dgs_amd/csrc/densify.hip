// densify.hip -- densify-and-prune as one planned gather (include/gsr_densify.h; SURVEY.md 8(f)
// row 4).  The reference rebuilds every parameter and both Adam moments three times per call
// (clone: cat; split: cat then boolean-index prune; opacity prune: boolean index), each through
// a nonzero() + gather per tensor.  Here:
//
//   plan:  one lane per old row evaluates the clone / split / prune predicates
//          (scene/gaussian_model.py:672-778 formulas, fp32 as torch evaluates them) into four 0/1
//          counters, rocPRIM scans them once (a 4-counter struct), and a scatter writes the output
//          row map: (source row, kind, normal-sample rank) per output row
//   apply: one launch over every (output row, element) of every group: copy, clone, or split
//          child (xyz = R(q) (z * exp(s)) + xyz, scaling = log(exp(s) / 1.6)); Adam moments
//          copied for old rows, zero for new ones
#include <cstring>
#include <string>

#include <rocprim/rocprim.hpp>

#include "../../include/gsr.h"
#include "../../include/gsr_densify.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

struct Cnt4 {
    uint32_t a, b, s, k;  // old rows kept, clones kept, split rows (all), split rows kept
};
__host__ __device__ inline Cnt4 operator+(const Cnt4 &x, const Cnt4 &y) {
    return Cnt4{x.a + y.a, x.b + y.b, x.s + y.s, x.k + y.k};
}
struct Cnt4Plus {
    __host__ __device__ inline Cnt4 operator()(const Cnt4 &x, const Cnt4 &y) const { return x + y; }
};

enum : uint32_t { kOld = 0, kClone = 1, kChild1 = 2, kChild2 = 3 };
constexpr int kMaxRowGroups = 8;

struct DensifyLayout {
    Cnt4 *flags, *pre, *tot;
    uint2 *map;
    void *tmp;
    size_t tmp_bytes, total;
};

DensifyLayout densify_layout(char *base, int64_t P0) {
    DensifyLayout L{};
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off = align_up(off + bytes, 256);
        return p;
    };
    const size_t n = (size_t)(P0 > 0 ? P0 : 1);
    L.flags = reinterpret_cast<Cnt4 *>(take(sizeof(Cnt4) * n));
    L.pre = reinterpret_cast<Cnt4 *>(take(sizeof(Cnt4) * n));
    L.tot = reinterpret_cast<Cnt4 *>(take(sizeof(Cnt4)));
    L.map = reinterpret_cast<uint2 *>(take(sizeof(uint2) * 3 * n));  // at most P0 + 2 * P0 rows
    size_t bytes = 0;
    rocprim::exclusive_scan(nullptr, bytes, (const Cnt4 *)nullptr, (Cnt4 *)nullptr, Cnt4{0, 0, 0, 0}, n, Cnt4Plus());
    L.tmp_bytes = bytes;
    L.tmp = take(bytes);
    L.total = off;
    return L;
}

__global__ __launch_bounds__(256) void densify_flags_kernel(int64_t P0, int64_t first, const float *__restrict__ g_acc,
                                                            const float *__restrict__ maxr,
                                                            const float *__restrict__ o_raw,
                                                            const float *__restrict__ s_raw, float max_grad,
                                                            float min_op, float max_scale, Cnt4 *__restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P0) return;
    float g = g_acc[i];
    if (isnan(g)) g = 0.f;  // grads[grads.isnan()] = 0.0
    const float op = 1.f / (1.f + expf(-o_raw[i]));  // torch.sigmoid
    const float pw = powf(op, 0.2f);                  // torch.pow(opacity, 1/5.0)
    const float smax = fmaxf(fmaxf(expf(s_raw[3 * i]), expf(s_raw[3 * i + 1])), expf(s_raw[3 * i + 2]));
    const bool eligible = i >= first && op > 0.15f;
    const float r = maxr[i];
    const bool clone = eligible && sqrtf(g * g) * r * pw >= max_grad && smax <= max_scale;  // torch.norm(dim=-1)
    const bool split = eligible && g * r * pw >= max_grad && smax > max_scale;
    const bool prune = i >= first && op < min_op;
    flags[i] = Cnt4{(!split && !prune) ? 1u : 0u, (clone && !prune) ? 1u : 0u, split ? 1u : 0u,
                    (split && !prune) ? 1u : 0u};
}

__global__ void densify_totals_kernel(int64_t P0, const Cnt4 *__restrict__ flags, const Cnt4 *__restrict__ pre,
                                      Cnt4 *__restrict__ tot, int64_t *__restrict__ counts) {
    if (threadIdx.x != 0) return;
    const Cnt4 t = P0 > 0 ? pre[P0 - 1] + flags[P0 - 1] : Cnt4{0, 0, 0, 0};
    *tot = t;
    counts[0] = t.a;
    counts[1] = t.b;
    counts[2] = t.s;
    counts[3] = (int64_t)t.a + t.b + 2 * (int64_t)t.k;
}

__global__ __launch_bounds__(256) void densify_map_kernel(int64_t P0, const Cnt4 *__restrict__ flags,
                                                          const Cnt4 *__restrict__ pre, const Cnt4 *__restrict__ tot,
                                                          uint2 *__restrict__ map) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P0) return;
    const Cnt4 f = flags[i], p = pre[i], t = *tot;
    const uint32_t src = (uint32_t)i;
    if (f.a) map[p.a] = make_uint2(src, kOld << 30);
    if (f.b) map[(size_t)t.a + p.b] = make_uint2(src, kClone << 30);
    if (f.k) {
        const size_t c1 = (size_t)t.a + t.b + p.k;
        map[c1] = make_uint2(src, (kChild1 << 30) | p.s);
        map[c1 + t.k] = make_uint2(src, (kChild2 << 30) | p.s);
    }
}

struct ApplyArgs {
    gsr_row_group src[kMaxRowGroups], dst[kMaxRowGroups];
    int64_t block_start[kMaxRowGroups + 1];
    int n, xyz, scaling, rotation;
};

// utils/general_utils.py:81-100 (build_rotation), row `row` of R, fp32 without contraction
__device__ inline void rotation_row(const float *q, int row, float &r0, float &r1, float &r2) {
    const float norm = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const float r = q[0] / norm, x = q[1] / norm, y = q[2] / norm, z = q[3] / norm;
    if (row == 0) {
        r0 = 1.f - 2.f * (y * y + z * z);
        r1 = 2.f * (x * y - r * z);
        r2 = 2.f * (x * z + r * y);
    } else if (row == 1) {
        r0 = 2.f * (x * y + r * z);
        r1 = 1.f - 2.f * (x * x + z * z);
        r2 = 2.f * (y * z - r * x);
    } else {
        r0 = 2.f * (x * z - r * y);
        r1 = 2.f * (y * z + r * x);
        r2 = 1.f - 2.f * (x * x + y * y);
    }
}

__global__ __launch_bounds__(256) void densify_apply_kernel(ApplyArgs a, const uint2 *__restrict__ map,
                                                            const float *__restrict__ normals, int64_t n_split,
                                                            int64_t rows) {
    int gi = 0;
    while (gi + 1 < a.n && (int64_t)blockIdx.x >= a.block_start[gi + 1]) gi++;
    const gsr_row_group &S = a.src[gi];
    const gsr_row_group &D = a.dst[gi];
    const int64_t w = S.width;
    const int64_t e = ((int64_t)blockIdx.x - a.block_start[gi]) * 256 + threadIdx.x;
    if (e >= rows * w) return;
    const int64_t o = e / w, col = e - o * w;
    const uint2 m = map[o];
    const int64_t src = m.x;
    const uint32_t kind = m.y >> 30, rank = m.y & 0x3fffffffu;
    const float *p = S.param + src * w;
    float v = p[col];
    if (kind >= kChild1) {
        const gsr_row_group &SS = a.src[a.scaling];
        const float *s = SS.param + src * 3;
        if (gi == a.xyz) {
            // new_xyz = bmm(build_rotation(q), normal(0, exp(s))) + xyz   (gaussian_model.py:688-690)
            const int64_t zr = (kind == kChild1 ? 0 : n_split) + rank;
            const float s0 = normals[3 * zr] * expf(s[0]) + 0.f, s1 = normals[3 * zr + 1] * expf(s[1]) + 0.f,
                        s2 = normals[3 * zr + 2] * expf(s[2]) + 0.f;
            float r0, r1, r2;
            rotation_row(a.src[a.rotation].param + src * 4, (int)col, r0, r1, r2);
            v = fmaf(r2, s2, fmaf(r1, s1, r0 * s0)) + v;
        } else if (gi == a.scaling) {
            // scaling_inverse_activation(get_scaling / (0.8 * N)), N = 2: torch divides a CUDA
            // tensor by a scalar as a multiply by the fp32 reciprocal of the fp32 scalar
            v = logf(expf(v) * (1.f / 1.6f));
        }
    }
    const int64_t d = o * w + col;
    D.param[d] = v;
    if (D.exp_avg && S.exp_avg) D.exp_avg[d] = kind == kOld ? S.exp_avg[src * w + col] : 0.f;
    if (D.exp_avg_sq && S.exp_avg_sq) D.exp_avg_sq[d] = kind == kOld ? S.exp_avg_sq[src * w + col] : 0.f;
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_densify_scratch_bytes(int64_t P0) {
    if (P0 < 0) return 0;
    return densify_layout(nullptr, P0).total;
}

int gsr_densify_plan(int64_t P0, int64_t first_row, const float *grad_accum, const float *max_radii2D,
                     const float *opacity_raw, const float *scaling_raw, float max_grad, float min_opacity,
                     float max_scale, void *scratch, int64_t *counts, void *stream) {
    if (P0 < 0 || P0 >= (1LL << 30) || first_row < 0 || !scratch || !counts ||
        (P0 > 0 && (!grad_accum || !max_radii2D || !opacity_raw || !scaling_raw))) {
        set_last_error("gsr_densify_plan: bad sizes (0 <= P0 < 2^30) or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const DensifyLayout L = densify_layout(static_cast<char *>(scratch), P0);
    const unsigned blocks = (unsigned)((P0 + 255) / 256);
    if (P0 > 0) {
        hipLaunchKernelGGL(densify_flags_kernel, dim3(blocks), dim3(256), 0, s, P0, first_row, grad_accum, max_radii2D,
                           opacity_raw, scaling_raw, max_grad, min_opacity, max_scale, L.flags);
        size_t tb = L.tmp_bytes;
        const hipError_t e = rocprim::exclusive_scan(L.tmp, tb, L.flags, L.pre, Cnt4{0, 0, 0, 0}, (size_t)P0,
                                                     Cnt4Plus(), s);
        if (e != hipSuccess) {
            set_last_error(std::string("gsr_densify_plan: scan: ") + hipGetErrorString(e));
            return GSR_ERR_DEVICE;
        }
    }
    hipLaunchKernelGGL(densify_totals_kernel, dim3(1), dim3(64), 0, s, P0, L.flags, L.pre, L.tot, counts);
    if (P0 > 0)
        hipLaunchKernelGGL(densify_map_kernel, dim3(blocks), dim3(256), 0, s, P0, L.flags, L.pre, L.tot, L.map);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_densify_plan: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_densify_apply(int64_t P0, int n_groups, const gsr_row_group *src, const gsr_row_group *dst, int xyz_group,
                      int scaling_group, int rotation_group, const float *normals, int64_t n_split,
                      const void *scratch, int64_t total_rows, void *stream) {
    if (P0 < 0 || n_groups <= 0 || n_groups > kMaxRowGroups || !src || !dst || !scratch || total_rows < 0 ||
        total_rows > 3 * P0 || xyz_group < 0 || xyz_group >= n_groups || scaling_group < 0 ||
        scaling_group >= n_groups || rotation_group < 0 || rotation_group >= n_groups || n_split < 0 ||
        (n_split > 0 && !normals)) {
        set_last_error("gsr_densify_apply: bad group layout, sizes or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (src[xyz_group].width != 3 || src[scaling_group].width != 3 || src[rotation_group].width != 4) {
        set_last_error("gsr_densify_apply: xyz / scaling / rotation groups must have widths 3 / 3 / 4");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (total_rows == 0) return GSR_OK;
    ApplyArgs a;
    std::memset(&a, 0, sizeof(a));
    a.n = n_groups;
    a.xyz = xyz_group;
    a.scaling = scaling_group;
    a.rotation = rotation_group;
    int64_t blocks = 0;
    for (int k = 0; k < n_groups; k++) {
        if (!src[k].param || !dst[k].param || src[k].width <= 0 || dst[k].width != src[k].width) {
            set_last_error("gsr_densify_apply: group with a NULL param or mismatched width");
            return GSR_ERR_INVALID_ARGUMENT;
        }
        a.src[k] = src[k];
        a.dst[k] = dst[k];
        a.block_start[k] = blocks;
        blocks += (total_rows * src[k].width + 255) / 256;
    }
    a.block_start[n_groups] = blocks;
    const DensifyLayout L = densify_layout(static_cast<char *>(const_cast<void *>(scratch)), P0);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(densify_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, L.map, normals, n_split,
                       total_rows);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_densify_apply: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"
