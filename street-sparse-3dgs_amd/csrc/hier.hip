// hier.hip -- fused hierarchy-cut interpolation of render_post (include/gsr_hier.h; SURVEY.md
// 8(a) A14, 8(f) row 3).  Thread per output row for the scalar fields; the 48-float SH rows are
// moved 16 lanes per row (one float4 per lane) when M = 16.  Backward scatters with float atomics into the N-row
// gradients: the same accumulate semantics as torch's index backward, which the reference relies
// on when several rendered nodes share a parent.
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_hier.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

struct CutRow {
    int64_t c, p;  // child (rendered) and parent rows; p == c for skybox copies
    float t;       // weight of the child
    bool copy;
};

__device__ __forceinline__ CutRow cut_row(int64_t r, int64_t N, int64_t R, int64_t S, const int *ri, const int *pi,
                                          const float *w) {
    CutRow o;
    if (r < R) {
        o.c = ri[r];
        o.p = pi[r];
        // expand_to_size gives root nodes the parent -1; torch's gather in render_post reads that
        // as the last row (weight 1 - t = 0 for a root), so do the same instead of reading before
        // the array
        if (o.p < 0) o.p += N;
        o.t = w[r];
        o.copy = false;
    } else {
        o.c = o.p = N - S + (r - R);
        o.t = 1.f;
        o.copy = true;
    }
    return o;
}

__device__ __forceinline__ float lerp_w(float t, float a, float b) { return t * a + (1.f - t) * b; }

// act (gsr_interpolate_cut_forward_act): the inputs are the pre-activation parameters and the
// getters of scene/gaussian_model.py:39-47 are applied to the rows the cut reads -- exp of the
// log-scales, normalize of the quaternions, the opacity activation (GSR_OPACITY_SIGMOID, or
// GSR_OPACITY_ABS: the hierarchy model's torch.abs, :411-412) -- so no N-row activated copy is
// written and re-read; the backward chains the activation derivatives into the scatter.
__device__ __forceinline__ float act_opac(int act, float o) {
    return act == GSR_OPACITY_ABS ? fabsf(o) : act == GSR_OPACITY_SIGMOID ? act_opacity(o) : o;
}
__device__ __forceinline__ float act_opac_grad(int act, float o, float g) {
    if (act == GSR_OPACITY_ABS) return o > 0.f ? g : (o < 0.f ? -g : 0.f);  // torch: g * sgn(o)
    if (act == GSR_OPACITY_SIGMOID) {
        const float y = act_opacity(o);
        return g * (1.f - y) * y;
    }
    return g;
}
// F.normalize's backward at the raw quaternion x for the upstream g (activate_bwd_kernel's form)
__device__ __forceinline__ float4 normalize_grad(float4 x, float4 g) {
    const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
    const float d = fmaxf(n, 1e-12f);
    const float gd = -(g.x * ((x.x / d) / d) + g.y * ((x.y / d) / d) + g.z * ((x.z / d) / d) + g.w * ((x.w / d) / d));
    const float gn = n >= 1e-12f && n != 0.f ? gd / n : 0.f;
    return make_float4(g.x / d + x.x * gn, g.y / d + x.y * gn, g.z / d + x.z * gn, g.w / d + x.w * gn);
}
__device__ __forceinline__ float4 ld_rot(const float *rots, int64_t i, int act) {
    const float4 q = reinterpret_cast<const float4 *>(rots)[i];
    return act ? act_rot(q) : q;
}

// Thread per output row for the 14 scalar fields.  The 192-B SH rows (M = 16, 16-B aligned) are
// moved by the wave as a whole: 16 lanes per row (12 active, one float4 each), four rows per
// instruction, so every load reads whole contiguous rows instead of one float4 from each of 64
// rows 192 B apart.  The row's (child, parent, weight) come from its owner lane by shuffle.
__global__ __launch_bounds__(256) void cut_fwd_kernel(int64_t N, int M, int64_t R, int64_t S, const int *ri,
                                                      const int *pi, const float *w, const float *__restrict__ means,
                                                      const float *__restrict__ scales, const float *__restrict__ rots,
                                                      const float *__restrict__ opac, const float *__restrict__ shs,
                                                      float *__restrict__ om, float *__restrict__ os,
                                                      float *__restrict__ orot, float *__restrict__ oop,
                                                      float *__restrict__ osh, bool vec, int act) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t rows = R + S;
    const bool valid = r < rows;
    const auto sc = [&](int64_t i) { return act ? act_scale(scales[i]) : scales[i]; };
    CutRow q{0, 0, 1.f, true};
    if (valid) q = cut_row(r, N, R, S, ri, pi, w);
    const float t = q.t;
    if (valid) {
        if (q.copy) {
            for (int k = 0; k < 3; k++) om[3 * r + k] = means[3 * q.c + k];
            for (int k = 0; k < 3; k++) os[3 * r + k] = sc(3 * q.c + k);
            reinterpret_cast<float4 *>(orot)[r] = ld_rot(rots, q.c, act);
            oop[r] = act_opac(act, opac[q.c]);
        } else {
            for (int k = 0; k < 3; k++) om[3 * r + k] = lerp_w(t, means[3 * q.c + k], means[3 * q.p + k]);
            for (int k = 0; k < 3; k++) os[3 * r + k] = lerp_w(t, sc(3 * q.c + k), sc(3 * q.p + k));
            const float4 qc = ld_rot(rots, q.c, act);
            float4 qp = ld_rot(rots, q.p, act);
            // torch.bmm(rots (1x4), parents (4x1)): the dot in float, left to right
            const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;
            if (dot < 0.f) qp = make_float4(-qp.x, -qp.y, -qp.z, -qp.w);
            reinterpret_cast<float4 *>(orot)[r] = make_float4(lerp_w(t, qc.x, qp.x), lerp_w(t, qc.y, qp.y),
                                                              lerp_w(t, qc.z, qp.z), lerp_w(t, qc.w, qp.w));
            oop[r] = lerp_w(t, act_opac(act, opac[q.c]), act_opac(act, opac[q.p]));
        }
    }
    if (vec) {
        const int lane = threadIdx.x & 63, col = lane & 15, sub = lane >> 4;
        const int64_t wrow0 = r - lane;
        if (wrow0 >= rows) return;  // wave-uniform
        const float4 *sh4 = reinterpret_cast<const float4 *>(shs);
        float4 *o4 = reinterpret_cast<float4 *>(osh);
#pragma unroll 4
        for (int k = 0; k < 16; k++) {
            const int src = 4 * k + sub;
            const int64_t rr = wrow0 + src;
            const int64_t cc = __shfl((long long)q.c, src, 64), pp = __shfl((long long)q.p, src, 64);
            const float tt = __shfl(t, src, 64);
            const bool cp = __shfl((int)q.copy, src, 64) != 0;
            if (rr < rows && col < 12) {
                const float4 x = sh4[12 * cc + col];
                float4 v = x;
                if (!cp) {
                    const float4 y = sh4[12 * pp + col];
                    v = make_float4(lerp_w(tt, x.x, y.x), lerp_w(tt, x.y, y.y), lerp_w(tt, x.z, y.z), lerp_w(tt, x.w, y.w));
                }
                o4[12 * rr + col] = v;
            }
        }
    } else if (valid) {
        if (q.copy)
            for (int k = 0; k < 3 * M; k++) osh[(size_t)r * 3 * M + k] = shs[(size_t)q.c * 3 * M + k];
        else
            for (int k = 0; k < 3 * M; k++)
                osh[(size_t)r * 3 * M + k] = lerp_w(t, shs[(size_t)q.c * 3 * M + k], shs[(size_t)q.p * 3 * M + k]);
    }
}

__global__ __launch_bounds__(256) void cut_bwd_kernel(int64_t N, int M, int64_t R, int64_t S, const int *ri,
                                                      const int *pi, const float *w, const float *__restrict__ rots,
                                                      const float *__restrict__ gm, const float *__restrict__ gs,
                                                      const float *__restrict__ grot, const float *__restrict__ gop,
                                                      const float *__restrict__ gsh, float *dm, float *ds, float *drot,
                                                      float *dop, float *dsh, bool vec, int act,
                                                      const float *__restrict__ s_raw,
                                                      const float *__restrict__ o_raw, bool uniq) {
    // d(act(x))/dx times the upstream, per input row (act == 0: the identity)
    const auto dsc = [&](int64_t i, float g) { return act ? g * act_scale(s_raw[i]) : g; };
    if (uniq) {
        // a cut: thread per row (coalesced), child rows written; the parent contributions of
        // consecutive rows with the same parent (siblings: expand_to_size emits a node's rendered
        // children consecutively) summed across the wave by a segmented scan, then one set of atomics
        // per sibling run (the activation derivatives are linear in the upstream: applied to the sum)
        const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int lane = threadIdx.x & 63;
        const bool valid = r < R + S;
        CutRow q{0, 0, 1.f, true};
        if (valid) q = cut_row(r, N, R, S, ri, pi, w);
        const float t = q.t, u = 1.f - q.t;
        float v[11];
        for (int k = 0; k < 11; k++) v[k] = 0.f;
        if (valid) {
            const float4 gr = make_float4(grot[4 * r + 0], grot[4 * r + 1], grot[4 * r + 2], grot[4 * r + 3]);
            const float4 qc = ld_rot(rots, q.c, act);
            for (int k = 0; k < 3; k++) {
                dm[3 * q.c + k] = t * gm[3 * r + k];
                ds[3 * q.c + k] = dsc(3 * q.c + k, t * gs[3 * r + k]);
            }
            float4 g = make_float4(t * gr.x, t * gr.y, t * gr.z, t * gr.w);
            if (act) g = normalize_grad(reinterpret_cast<const float4 *>(rots)[q.c], g);
            drot[4 * q.c + 0] = g.x;
            drot[4 * q.c + 1] = g.y;
            drot[4 * q.c + 2] = g.z;
            drot[4 * q.c + 3] = g.w;
            dop[q.c] = act_opac_grad(act, act ? o_raw[q.c] : 0.f, t * gop[r]);
            if (!vec)
                for (int k = 0; k < 3 * M; k++) dsh[(size_t)q.c * 3 * M + k] = t * gsh[(size_t)r * 3 * M + k];
            if (!q.copy) {
                const float4 qp = ld_rot(rots, q.p, act);
                const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;
                const float su = (dot < 0.f ? -1.f : 1.f) * u;
                for (int k = 0; k < 3; k++) {
                    v[k] = u * gm[3 * r + k];
                    v[3 + k] = u * gs[3 * r + k];
                }
                v[6] = su * gr.x;
                v[7] = su * gr.y;
                v[8] = su * gr.z;
                v[9] = su * gr.w;
                v[10] = u * gop[r];
                if (!vec)
                    for (int k = 0; k < 3 * M; k++) atomicAdd(&dsh[(size_t)q.p * 3 * M + k], u * gsh[(size_t)r * 3 * M + k]);
            }
        }
        const int par = valid && !q.copy ? (int)q.p : -1;
        const int prev = __shfl_up(par, 1, 64), next = __shfl_down(par, 1, 64);
        const uint64_t heads = __ballot(lane == 0 || par != prev);
        const int start = 63 - __clzll((long long)(heads & ((2ull << lane) - 1ull)));
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
            for (int k = 0; k < 11; k++) {
                const float up = __shfl_up(v[k], o, 64);
                if (lane - o >= start) v[k] += up;
            }
        }
        if (par >= 0 && (lane == 63 || next != par)) {  // the run's last lane holds its sums
            const int64_t cur = par;
            for (int k = 0; k < 3; k++) {
                atomicAdd(&dm[3 * cur + k], v[k]);
                atomicAdd(&ds[3 * cur + k], dsc(3 * cur + k, v[3 + k]));
            }
            float4 g = make_float4(v[6], v[7], v[8], v[9]);
            if (act) g = normalize_grad(reinterpret_cast<const float4 *>(rots)[cur], g);
            atomicAdd(&drot[4 * cur + 0], g.x);
            atomicAdd(&drot[4 * cur + 1], g.y);
            atomicAdd(&drot[4 * cur + 2], g.z);
            atomicAdd(&drot[4 * cur + 3], g.w);
            atomicAdd(&dop[cur], act_opac_grad(act, act ? o_raw[cur] : 0.f, v[10]));
        }
        return;
    }
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R + S) return;
    const CutRow q = cut_row(r, N, R, S, ri, pi, w);
    const float t = q.t, u = 1.f - q.t;
    const auto add_rot = [&](int64_t row, float4 g, bool store) {
        if (act) g = normalize_grad(reinterpret_cast<const float4 *>(rots)[row], g);
        if (store) {
            drot[4 * row + 0] = g.x;
            drot[4 * row + 1] = g.y;
            drot[4 * row + 2] = g.z;
            drot[4 * row + 3] = g.w;
            return;
        }
        atomicAdd(&drot[4 * row + 0], g.x);
        atomicAdd(&drot[4 * row + 1], g.y);
        atomicAdd(&drot[4 * row + 2], g.z);
        atomicAdd(&drot[4 * row + 3], g.w);
    };
    // a cut's child rows are unique (uniq): written; parent rows are shared by siblings: accumulated
    const auto put = [&](float *a, float v) {
        if (uniq) *a = v;
        else atomicAdd(a, v);
    };
    const float4 gr = make_float4(grot[4 * r + 0], grot[4 * r + 1], grot[4 * r + 2], grot[4 * r + 3]);
    if (q.copy) {
        for (int k = 0; k < 3; k++) put(&dm[3 * q.c + k], gm[3 * r + k]);
        for (int k = 0; k < 3; k++) put(&ds[3 * q.c + k], dsc(3 * q.c + k, gs[3 * r + k]));
        add_rot(q.c, gr, uniq);
        put(&dop[q.c], act_opac_grad(act, act ? o_raw[q.c] : 0.f, gop[r]));
        if (!vec)
            for (int k = 0; k < 3 * M; k++) put(&dsh[(size_t)q.c * 3 * M + k], gsh[(size_t)r * 3 * M + k]);
        return;
    }
    for (int k = 0; k < 3; k++) {
        put(&dm[3 * q.c + k], t * gm[3 * r + k]);
        atomicAdd(&dm[3 * q.p + k], u * gm[3 * r + k]);
        put(&ds[3 * q.c + k], dsc(3 * q.c + k, t * gs[3 * r + k]));
        atomicAdd(&ds[3 * q.p + k], dsc(3 * q.p + k, u * gs[3 * r + k]));
    }
    const float4 qc = ld_rot(rots, q.c, act);
    const float4 qp = ld_rot(rots, q.p, act);
    const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;
    const float sgn = dot < 0.f ? -1.f : 1.f;
    add_rot(q.c, make_float4(t * gr.x, t * gr.y, t * gr.z, t * gr.w), uniq);
    add_rot(q.p, make_float4(sgn * u * gr.x, sgn * u * gr.y, sgn * u * gr.z, sgn * u * gr.w), false);
    put(&dop[q.c], act_opac_grad(act, act ? o_raw[q.c] : 0.f, t * gop[r]));
    atomicAdd(&dop[q.p], act_opac_grad(act, act ? o_raw[q.p] : 0.f, u * gop[r]));
    if (vec) return;
    for (int k = 0; k < 3 * M; k++) {
        const float g = gsh[(size_t)r * 3 * M + k];
        put(&dsh[(size_t)q.c * 3 * M + k], t * g);
        atomicAdd(&dsh[(size_t)q.p * 3 * M + k], u * g);
    }
}

// SH part of the backward for M = 16: 16 lanes per row (12 active, 4 floats each).  uniq (a cut):
// lane group g walks the kShRun consecutive rows [g kShRun, (g + 1) kShRun), writes each child row
// with one 16-B store and adds the parent contributions of consecutive rows with the same parent
// (siblings: expand_to_size emits a node's rendered children consecutively) before one atomic per
// parent run.  Otherwise every row's child and parent contributions are atomics.
constexpr int kShRun = 16;
__global__ __launch_bounds__(256) void cut_bwd_sh_kernel(int64_t N, int64_t R, int64_t S, const int *ri, const int *pi,
                                                         const float *w, const float *__restrict__ gsh,
                                                         float *dsh, bool uniq) {
    const int64_t grp = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int col = threadIdx.x & 15;
    if (col >= 12) return;
    const auto add4 = [&](float *a, float4 v) {
        atomicAdd(a + 0, v.x);
        atomicAdd(a + 1, v.y);
        atomicAdd(a + 2, v.z);
        atomicAdd(a + 3, v.w);
    };
    if (!uniq) {
        const int64_t rr = grp;
        if (rr >= R + S) return;
        const CutRow q = cut_row(rr, N, R, S, ri, pi, w);
        const float4 g = reinterpret_cast<const float4 *>(gsh)[12 * rr + col];
        const float t = q.copy ? 1.f : q.t, u = 1.f - q.t;
        add4(dsh + 48 * q.c + 4 * col, make_float4(t * g.x, t * g.y, t * g.z, t * g.w));
        if (!q.copy) add4(dsh + 48 * q.p + 4 * col, make_float4(u * g.x, u * g.y, u * g.z, u * g.w));
        return;
    }
    const int64_t r0 = grp * kShRun, r1 = min(R + S, r0 + kShRun);
    int64_t cur = -1;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t rr = r0; rr < r1; rr++) {
        const CutRow q = cut_row(rr, N, R, S, ri, pi, w);
        const float4 g = reinterpret_cast<const float4 *>(gsh)[12 * rr + col];
        const float t = q.copy ? 1.f : q.t, u = 1.f - q.t;
        reinterpret_cast<float4 *>(dsh + 48 * q.c + 4 * col)[0] = make_float4(t * g.x, t * g.y, t * g.z, t * g.w);
        if (q.copy) continue;
        if (q.p != cur) {
            if (cur >= 0) add4(dsh + 48 * cur + 4 * col, acc);
            cur = q.p;
            acc = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        acc.x = fmaf(u, g.x, acc.x);
        acc.y = fmaf(u, g.y, acc.y);
        acc.z = fmaf(u, g.z, acc.z);
        acc.w = fmaf(u, g.w, acc.w);
    }
    if (cur >= 0) add4(dsh + 48 * cur + 4 * col, acc);
}

}  // namespace
}  // namespace gsr

using namespace gsr;

namespace {

int cut_forward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices, const int *parent_indices,
                const float *interpolation_weights, const float *means3D, const float *scales, const float *rotations,
                const float *opacities, const float *shs, int act, float *out_means3D, float *out_scales,
                float *out_rotations, float *out_opacities, float *out_shs, void *stream, const char *who) {
    if (N < 0 || R < 0 || S < 0 || S > N || M <= 0 || M > 16 || act < 0 || act > GSR_OPACITY_ABS) {
        set_last_error(std::string(who) + ": bad sizes or activation (need 0 <= S <= N, 1 <= M <= 16)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (R + S == 0) return GSR_OK;
    if (!means3D || !scales || !rotations || !opacities || !shs || !out_means3D || !out_scales || !out_rotations ||
        !out_opacities || !out_shs || (R > 0 && (!render_indices || !parent_indices || !interpolation_weights))) {
        set_last_error(std::string(who) + ": NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if ((reinterpret_cast<uintptr_t>(rotations) | reinterpret_cast<uintptr_t>(out_rotations)) % 16 != 0) {
        set_last_error(std::string(who) + ": rotations must be 16-byte aligned");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    const bool vec = M == 16 && reinterpret_cast<uintptr_t>(shs) % 16 == 0 && reinterpret_cast<uintptr_t>(out_shs) % 16 == 0;
    const int64_t rows = R + S;
    hipLaunchKernelGGL(cut_fwd_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, M, R, S, render_indices, parent_indices,
                       interpolation_weights, means3D, scales, rotations, opacities, shs, out_means3D, out_scales,
                       out_rotations, out_opacities, out_shs, vec, act);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string(who) + ": " + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int cut_backward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices, const int *parent_indices,
                 const float *interpolation_weights, const float *s_raw, const float *rotations, const float *o_raw,
                 int act, const float *dL_dout_means3D, const float *dL_dout_scales, const float *dL_dout_rotations,
                 const float *dL_dout_opacities, const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscales,
                 float *dL_drotations, float *dL_dopacities, float *dL_dshs, void *stream, const char *who) {
    const bool uniq = (act & GSR_CUT_UNIQUE_CHILDREN) != 0;
    act &= ~GSR_CUT_UNIQUE_CHILDREN;
    if (N < 0 || R < 0 || S < 0 || S > N || M <= 0 || M > 16 || act < 0 || act > GSR_OPACITY_ABS) {
        set_last_error(std::string(who) + ": bad sizes or activation (need 0 <= S <= N, 1 <= M <= 16)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (R + S == 0) return GSR_OK;
    if (!rotations || !dL_dout_means3D || !dL_dout_scales || !dL_dout_rotations || !dL_dout_opacities ||
        !dL_dout_shs || !dL_dmeans3D || !dL_dscales || !dL_drotations || !dL_dopacities || !dL_dshs ||
        (act && (!s_raw || !o_raw)) || (R > 0 && (!render_indices || !parent_indices || !interpolation_weights))) {
        set_last_error(std::string(who) + ": NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (reinterpret_cast<uintptr_t>(rotations) % 16 != 0) {
        set_last_error(std::string(who) + ": rotations must be 16-byte aligned");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    const int64_t rows = R + S;
    const bool vec = M == 16 && reinterpret_cast<uintptr_t>(dL_dout_shs) % 16 == 0 &&
                     reinterpret_cast<uintptr_t>(dL_dshs) % 16 == 0;
    hipLaunchKernelGGL(cut_bwd_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, M, R, S, render_indices, parent_indices,
                       interpolation_weights, rotations, dL_dout_means3D, dL_dout_scales, dL_dout_rotations,
                       dL_dout_opacities, dL_dout_shs, dL_dmeans3D, dL_dscales, dL_drotations, dL_dopacities,
                       dL_dshs, vec, act, s_raw, o_raw, uniq);
    if (vec)
        hipLaunchKernelGGL(cut_bwd_sh_kernel, dim3((unsigned)((16 * (uniq ? (rows + kShRun - 1) / kShRun : rows) + 255) / 256)),
                           dim3(256), 0,
                           static_cast<hipStream_t>(stream), N, R, S, render_indices, parent_indices,
                           interpolation_weights, dL_dout_shs, dL_dshs, uniq);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string(who) + ": " + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

constexpr int kZeroMax = 8;
struct ZeroArrays {
    float *p[kZeroMax];
    int64_t w[kZeroMax];
};

// one thread per (locked row, array): the last `tail` rows, then the listed rows
__global__ __launch_bounds__(256) void zero_rows_kernel(ZeroArrays z, int n, int64_t N, int64_t tail,
                                                        const int64_t *__restrict__ rows, int64_t n_rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int k = (int)blockIdx.y;
    if (i >= tail + n_rows || k >= n) return;
    const int64_t row = i < tail ? N - tail + i : rows[i - tail];
    if (row < 0 || row >= N) return;
    float *d = z.p[k] + row * z.w[k];
    for (int64_t c = 0; c < z.w[k]; c++) d[c] = 0.f;
}

}  // namespace

extern "C" {

int gsr_interpolate_cut_forward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                const int *parent_indices, const float *interpolation_weights, const float *means3D,
                                const float *scales, const float *rotations, const float *opacities, const float *shs,
                                float *out_means3D, float *out_scales, float *out_rotations, float *out_opacities,
                                float *out_shs, void *stream) {
    return cut_forward(N, M, R, S, render_indices, parent_indices, interpolation_weights, means3D, scales, rotations,
                       opacities, shs, 0, out_means3D, out_scales, out_rotations, out_opacities, out_shs, stream,
                       "gsr_interpolate_cut_forward");
}

int gsr_interpolate_cut_forward_act(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                    const int *parent_indices, const float *interpolation_weights,
                                    const float *means3D, const float *scaling_raw, const float *rotation_raw,
                                    const float *opacity_raw, const float *shs, int opacity_act, float *out_means3D,
                                    float *out_scales, float *out_rotations, float *out_opacities, float *out_shs,
                                    void *stream) {
    // act 0 is reserved for the activated inputs: the raw form always activates scales / rotations
    const int act = opacity_act == GSR_OPACITY_IDENTITY ? -1 : opacity_act;
    if (act < 0) {
        set_last_error("gsr_interpolate_cut_forward_act: opacity_act must be GSR_OPACITY_SIGMOID or GSR_OPACITY_ABS");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    return cut_forward(N, M, R, S, render_indices, parent_indices, interpolation_weights, means3D, scaling_raw,
                       rotation_raw, opacity_raw, shs, act, out_means3D, out_scales, out_rotations, out_opacities,
                       out_shs, stream, "gsr_interpolate_cut_forward_act");
}

int gsr_interpolate_cut_backward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                 const int *parent_indices, const float *interpolation_weights,
                                 const float *rotations, const float *dL_dout_means3D, const float *dL_dout_scales,
                                 const float *dL_dout_rotations, const float *dL_dout_opacities,
                                 const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscales,
                                 float *dL_drotations, float *dL_dopacities, float *dL_dshs, void *stream) {
    return cut_backward(N, M, R, S, render_indices, parent_indices, interpolation_weights, nullptr, rotations,
                        nullptr, 0, dL_dout_means3D, dL_dout_scales, dL_dout_rotations, dL_dout_opacities, dL_dout_shs,
                        dL_dmeans3D, dL_dscales, dL_drotations, dL_dopacities, dL_dshs, stream,
                        "gsr_interpolate_cut_backward");
}

int gsr_interpolate_cut_backward_act(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                     const int *parent_indices, const float *interpolation_weights,
                                     const float *scaling_raw, const float *rotation_raw, const float *opacity_raw,
                                     int opacity_act, const float *dL_dout_means3D, const float *dL_dout_scales,
                                     const float *dL_dout_rotations, const float *dL_dout_opacities,
                                     const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscaling_raw,
                                     float *dL_drotation_raw, float *dL_dopacity_raw, float *dL_dshs, void *stream) {
    const int oa = opacity_act & ~GSR_CUT_UNIQUE_CHILDREN;
    if (oa != GSR_OPACITY_SIGMOID && oa != GSR_OPACITY_ABS) {
        set_last_error("gsr_interpolate_cut_backward_act: opacity_act must be GSR_OPACITY_SIGMOID or GSR_OPACITY_ABS "
                       "(optionally | GSR_CUT_UNIQUE_CHILDREN)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    return cut_backward(N, M, R, S, render_indices, parent_indices, interpolation_weights, scaling_raw, rotation_raw,
                        opacity_raw, opacity_act, dL_dout_means3D, dL_dout_scales, dL_dout_rotations,
                        dL_dout_opacities, dL_dout_shs, dL_dmeans3D, dL_dscaling_raw, dL_drotation_raw,
                        dL_dopacity_raw, dL_dshs, stream, "gsr_interpolate_cut_backward_act");
}

int gsr_zero_grad_rows(int n, float *const *grads, const int64_t *widths, int64_t N, int64_t tail,
                       const int64_t *rows, int64_t n_rows, void *stream) {
    if (n < 0 || n > kZeroMax || N < 0 || tail < 0 || tail > N || n_rows < 0 || (n > 0 && (!grads || !widths)) ||
        (n_rows > 0 && !rows)) {
        set_last_error("gsr_zero_grad_rows: bad sizes or NULL pointer (at most 8 arrays)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    ZeroArrays z{};
    for (int k = 0; k < n; k++) {
        if (!grads[k] || widths[k] <= 0) {
            set_last_error("gsr_zero_grad_rows: NULL array or non-positive width");
            return GSR_ERR_INVALID_ARGUMENT;
        }
        z.p[k] = grads[k];
        z.w[k] = widths[k];
    }
    const int64_t m = tail + n_rows;
    if (m == 0 || n == 0) return GSR_OK;
    hipLaunchKernelGGL(zero_rows_kernel, dim3((unsigned)((m + 255) / 256), (unsigned)n), dim3(256), 0,
                       static_cast<hipStream_t>(stream), z, n, N, tail, rows, n_rows);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_zero_grad_rows: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"
