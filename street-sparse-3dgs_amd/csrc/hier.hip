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
                                                      float *__restrict__ osh, bool vec) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t rows = R + S;
    const bool valid = r < rows;
    CutRow q{0, 0, 1.f, true};
    if (valid) q = cut_row(r, N, R, S, ri, pi, w);
    const float t = q.t;
    if (valid) {
        if (q.copy) {
            for (int k = 0; k < 3; k++) om[3 * r + k] = means[3 * q.c + k];
            for (int k = 0; k < 3; k++) os[3 * r + k] = scales[3 * q.c + k];
            for (int k = 0; k < 4; k++) orot[4 * r + k] = rots[4 * q.c + k];
            oop[r] = opac[q.c];
        } else {
            for (int k = 0; k < 3; k++) om[3 * r + k] = lerp_w(t, means[3 * q.c + k], means[3 * q.p + k]);
            for (int k = 0; k < 3; k++) os[3 * r + k] = lerp_w(t, scales[3 * q.c + k], scales[3 * q.p + k]);
            const float4 qc = reinterpret_cast<const float4 *>(rots)[q.c];
            float4 qp = reinterpret_cast<const float4 *>(rots)[q.p];
            // torch.bmm(rots (1x4), parents (4x1)): the dot in float, left to right
            const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;
            if (dot < 0.f) qp = make_float4(-qp.x, -qp.y, -qp.z, -qp.w);
            reinterpret_cast<float4 *>(orot)[r] = make_float4(lerp_w(t, qc.x, qp.x), lerp_w(t, qc.y, qp.y),
                                                              lerp_w(t, qc.z, qp.z), lerp_w(t, qc.w, qp.w));
            oop[r] = lerp_w(t, opac[q.c], opac[q.p]);
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
                                                      float *dop, float *dsh, bool vec) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R + S) return;
    const CutRow q = cut_row(r, N, R, S, ri, pi, w);
    const float t = q.t, u = 1.f - q.t;
    if (q.copy) {
        for (int k = 0; k < 3; k++) atomicAdd(&dm[3 * q.c + k], gm[3 * r + k]);
        for (int k = 0; k < 3; k++) atomicAdd(&ds[3 * q.c + k], gs[3 * r + k]);
        for (int k = 0; k < 4; k++) atomicAdd(&drot[4 * q.c + k], grot[4 * r + k]);
        atomicAdd(&dop[q.c], gop[r]);
        if (!vec)
            for (int k = 0; k < 3 * M; k++) atomicAdd(&dsh[(size_t)q.c * 3 * M + k], gsh[(size_t)r * 3 * M + k]);
        return;
    }
    for (int k = 0; k < 3; k++) {
        atomicAdd(&dm[3 * q.c + k], t * gm[3 * r + k]);
        atomicAdd(&dm[3 * q.p + k], u * gm[3 * r + k]);
        atomicAdd(&ds[3 * q.c + k], t * gs[3 * r + k]);
        atomicAdd(&ds[3 * q.p + k], u * gs[3 * r + k]);
    }
    const float4 qc = reinterpret_cast<const float4 *>(rots)[q.c];
    const float4 qp = reinterpret_cast<const float4 *>(rots)[q.p];
    const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;
    const float sgn = dot < 0.f ? -1.f : 1.f;
    for (int k = 0; k < 4; k++) {
        atomicAdd(&drot[4 * q.c + k], t * grot[4 * r + k]);
        atomicAdd(&drot[4 * q.p + k], sgn * u * grot[4 * r + k]);
    }
    atomicAdd(&dop[q.c], t * gop[r]);
    atomicAdd(&dop[q.p], u * gop[r]);
    if (vec) return;
    for (int k = 0; k < 3 * M; k++) {
        const float g = gsh[(size_t)r * 3 * M + k];
        atomicAdd(&dsh[(size_t)q.c * 3 * M + k], t * g);
        atomicAdd(&dsh[(size_t)q.p * 3 * M + k], u * g);
    }
}

// SH part of the backward for M = 16: 16 lanes per row (12 active, 4 floats each), four rows per
// wave instruction, so the atomics of one row hit one or two cache lines together.
__global__ __launch_bounds__(256) void cut_bwd_sh_kernel(int64_t N, int64_t R, int64_t S, const int *ri, const int *pi,
                                                         const float *w, const float *__restrict__ gsh,
                                                         float *dsh) {
    const int64_t rr = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int col = threadIdx.x & 15;
    if (rr >= R + S || col >= 12) return;
    const CutRow q = cut_row(rr, N, R, S, ri, pi, w);
    const float4 g = reinterpret_cast<const float4 *>(gsh)[12 * rr + col];
    float *dc = dsh + 48 * q.c + 4 * col;
    if (q.copy) {
        atomicAdd(dc + 0, g.x);
        atomicAdd(dc + 1, g.y);
        atomicAdd(dc + 2, g.z);
        atomicAdd(dc + 3, g.w);
        return;
    }
    const float t = q.t, u = 1.f - q.t;
    float *dp = dsh + 48 * q.p + 4 * col;
    atomicAdd(dc + 0, t * g.x);
    atomicAdd(dc + 1, t * g.y);
    atomicAdd(dc + 2, t * g.z);
    atomicAdd(dc + 3, t * g.w);
    atomicAdd(dp + 0, u * g.x);
    atomicAdd(dp + 1, u * g.y);
    atomicAdd(dp + 2, u * g.z);
    atomicAdd(dp + 3, u * g.w);
}

}  // namespace
}  // namespace gsr

using namespace gsr;

extern "C" {

int gsr_interpolate_cut_forward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                const int *parent_indices, const float *interpolation_weights, const float *means3D,
                                const float *scales, const float *rotations, const float *opacities, const float *shs,
                                float *out_means3D, float *out_scales, float *out_rotations, float *out_opacities,
                                float *out_shs, void *stream) {
    if (N < 0 || R < 0 || S < 0 || S > N || M <= 0 || M > 16) {
        set_last_error("gsr_interpolate_cut_forward: bad sizes (need 0 <= S <= N, 1 <= M <= 16)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (R + S == 0) return GSR_OK;
    if (!means3D || !scales || !rotations || !opacities || !shs || !out_means3D || !out_scales || !out_rotations ||
        !out_opacities || !out_shs || (R > 0 && (!render_indices || !parent_indices || !interpolation_weights))) {
        set_last_error("gsr_interpolate_cut_forward: NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    const bool vec = M == 16 && reinterpret_cast<uintptr_t>(shs) % 16 == 0 && reinterpret_cast<uintptr_t>(out_shs) % 16 == 0;
    const int64_t rows = R + S;
    hipLaunchKernelGGL(cut_fwd_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, M, R, S, render_indices, parent_indices,
                       interpolation_weights, means3D, scales, rotations, opacities, shs, out_means3D, out_scales,
                       out_rotations, out_opacities, out_shs, vec);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_interpolate_cut_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_interpolate_cut_backward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                 const int *parent_indices, const float *interpolation_weights,
                                 const float *rotations, const float *dL_dout_means3D, const float *dL_dout_scales,
                                 const float *dL_dout_rotations, const float *dL_dout_opacities,
                                 const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscales,
                                 float *dL_drotations, float *dL_dopacities, float *dL_dshs, void *stream) {
    if (N < 0 || R < 0 || S < 0 || S > N || M <= 0 || M > 16) {
        set_last_error("gsr_interpolate_cut_backward: bad sizes (need 0 <= S <= N, 1 <= M <= 16)");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (R + S == 0) return GSR_OK;
    if (!rotations || !dL_dout_means3D || !dL_dout_scales || !dL_dout_rotations || !dL_dout_opacities ||
        !dL_dout_shs || !dL_dmeans3D || !dL_dscales || !dL_drotations || !dL_dopacities || !dL_dshs ||
        (R > 0 && (!render_indices || !parent_indices || !interpolation_weights))) {
        set_last_error("gsr_interpolate_cut_backward: NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    const int64_t rows = R + S;
    const bool vec = M == 16 && reinterpret_cast<uintptr_t>(dL_dout_shs) % 16 == 0;
    hipLaunchKernelGGL(cut_bwd_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), N, M, R, S, render_indices, parent_indices,
                       interpolation_weights, rotations, dL_dout_means3D, dL_dout_scales, dL_dout_rotations,
                       dL_dout_opacities, dL_dout_shs, dL_dmeans3D, dL_dscales, dL_drotations, dL_dopacities,
                       dL_dshs, vec);
    if (vec)
        hipLaunchKernelGGL(cut_bwd_sh_kernel, dim3((unsigned)((16 * rows + 255) / 256)), dim3(256), 0,
                           static_cast<hipStream_t>(stream), N, R, S, render_indices, parent_indices,
                           interpolation_weights, dL_dout_shs, dL_dshs);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_interpolate_cut_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"
