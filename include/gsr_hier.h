/*
 * gsr_hier.h -- C ABI of the fused hierarchy-cut interpolation that feeds the rasterizer in
 * render_post.  Exported by libgsr_hip.so.
 *
 *   gsr_interpolate_cut_forward / _backward  replace the Python LOD blend of
 *   gaussian_renderer/__init__.py:200-243 (interp_python=True, the default on every reference
 *   call path: train_post.py:119, render_hierarchy.py:88): for each rendered node r < R with
 *   child c = render_indices[r], parent p = parent_indices[r] and t = interpolation_weights[r],
 *
 *     means, scales, shs, opacities:  t * x[c] + (1 - t) * x[p]
 *     rotations:                      q_p is negated when dot(q_c, q_p) < 0, then
 *                                     t * q_c + (1 - t) * q_p   (not re-normalised)
 *
 *   followed by S unchanged "skybox" rows copied from the last S Gaussians.  One pass over the
 *   gathered rows instead of ~25 torch gather / lerp / cat kernels.
 *
 * Conventions as in gsr.h.  Indices are int32 device arrays; shs is (N, M, 3).
 */
#ifndef GSR_HIER_H
#define GSR_HIER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Outputs have R + S rows. */
int gsr_interpolate_cut_forward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                const int *parent_indices, const float *interpolation_weights, const float *means3D,
                                const float *scales, const float *rotations, const float *opacities, const float *shs,
                                float *out_means3D, float *out_scales, float *out_rotations, float *out_opacities,
                                float *out_shs, void *stream);

/* Accumulates (+=) the gradients of the R + S output rows into the N-row input gradients, which
 * the caller zero-initialises; rows shared by several rendered nodes receive the sum (float
 * atomics, as torch's index backward). */
int gsr_interpolate_cut_backward(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                 const int *parent_indices, const float *interpolation_weights,
                                 const float *rotations, const float *dL_dout_means3D, const float *dL_dout_scales,
                                 const float *dL_dout_rotations, const float *dL_dout_opacities,
                                 const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscales,
                                 float *dL_drotations, float *dL_dopacities, float *dL_dshs, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_HIER_H */
