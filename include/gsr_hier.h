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

/* The same blend over the PRE-activation parameters (ABI 3): scales are log-scales (exp applied),
 * rotations unnormalised quaternions (F.normalize applied before the dot test and the lerp) and
 * opacities the stored values with opacity_act applied -- the getters of
 * scene/gaussian_model.py:39-47,125-156 evaluated only on the rows the cut reads (train_post.py's
 * model: create_from_hier sets opacity_activation = torch.abs, :411-412).  The backward
 * accumulates the gradients of the raw parameters (activation derivatives chained per gathered
 * row); it reads the raw scales, rotations and opacities.  Means and SH have no activation. */
#define GSR_OPACITY_IDENTITY 0
#define GSR_OPACITY_SIGMOID 1
#define GSR_OPACITY_ABS 2
/* OR'ed into opacity_act of gsr_interpolate_cut_backward_act: render_indices name every row at most
 * once and none of them is also a parent row (a cut: expand_to_size's output), so the children's
 * gradient rows are written, not accumulated with atomics (the gradients must be zero on entry, as
 * for the accumulating form). */
#define GSR_CUT_UNIQUE_CHILDREN 0x100
int gsr_interpolate_cut_forward_act(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                    const int *parent_indices, const float *interpolation_weights,
                                    const float *means3D, const float *scaling_raw, const float *rotation_raw,
                                    const float *opacity_raw, const float *shs, int opacity_act, float *out_means3D,
                                    float *out_scales, float *out_rotations, float *out_opacities, float *out_shs,
                                    void *stream);
int gsr_interpolate_cut_backward_act(int64_t N, int M, int64_t R, int64_t S, const int *render_indices,
                                     const int *parent_indices, const float *interpolation_weights,
                                     const float *scaling_raw, const float *rotation_raw, const float *opacity_raw,
                                     int opacity_act, const float *dL_dout_means3D, const float *dL_dout_scales,
                                     const float *dL_dout_rotations, const float *dL_dout_opacities,
                                     const float *dL_dout_shs, float *dL_dmeans3D, float *dL_dscaling_raw,
                                     float *dL_drotation_raw, float *dL_dopacity_raw, float *dL_dshs, void *stream);

/* Zero the gradient rows train_post.py:167-181 locks: the last `tail` rows (the skybox) and the
 * rows listed in `rows` (the anchors, int64, may repeat), in each of n arrays of widths[k] floats
 * per row over N rows.  One launch. */
int gsr_zero_grad_rows(int n, float *const *grads, const int64_t *widths, int64_t N, int64_t tail,
                       const int64_t *rows, int64_t n_rows, void *stream);

/* ---- LOD cut (csrc/lod.hip) ------------------------------------------------------------
 * Replace gaussian_hierarchy._C.expand_to_size / get_interpolation_weights (the gaussianhierarchy
 * extension, un-vendored; called at render_hierarchy.py:63-85, train_post.py:91-113,
 * render_hierarchy_final.py:222-245, render_position.py:105-130 of the reference).
 *   nodes: (N, 7) int32 {depth, parent, start, count_leafs, count_merged, start_children,
 *          count_children};  boxes: (N, 2, 4) float {minn.xyz, size, maxx.xyz, -}.
 * expand_to_size writes the cut -- render_indices (Gaussian ids), parent_indices (the parent
 * node's first Gaussian, -1 for roots) and nodes_for_render_indices (node ids), in node order --
 * and returns its length in *to_render (the value the Python function returns; one host read, as
 * upstream).  viewpoint is a DEVICE float[3] (the caller's camera_center on the GPU).
 * `capacity` = the entries each output array holds: nothing is stored past it, and a cut longer
 * than it (possible when nodes hold several Gaussians: the cut can reach the sum of count_leafs +
 * count_merged, more than N) fails with GSR_ERR_INVALID_ARGUMENT, *to_render set to the length it
 * needs (the entries that fit may have been written: one pass counts and writes).  scratch: a device buffer of gsr_expand_to_size_scratch_bytes(N) bytes. */
size_t gsr_expand_to_size_scratch_bytes(int64_t N);
int gsr_expand_to_size(int64_t N, const int *nodes, const float *boxes, float target_size, const float *viewpoint,
                       int *render_indices, int *parent_indices, int *nodes_for_render_indices, int64_t capacity,
                       void *scratch, size_t scratch_bytes, int64_t *to_render, void *stream);

/* get_interpolation_weights: for the n rendered nodes node_indices[i], weights[i] = the blend
 * weight t of the node with its parent and num_kids[i] = the parent's child count (1 for roots).
 * The viewpoint is passed by value (the reference hands camera_center.cpu()). */
int gsr_interpolation_weights(int64_t n, const int *node_indices, float target_size, const int *nodes,
                              const float *boxes, float vx, float vy, float vz, float *weights, int *num_kids,
                              void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_HIER_H */
