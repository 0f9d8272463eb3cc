/*
 * gsr_densify.h -- C ABI of densify-and-prune as one device pass over the Gaussian rows
 * (SURVEY.md 8(f) row 4).  Exported by libgsr_hip.so.
 *
 * Replaces GaussianModel.densify_and_prune (scene/gaussian_model.py:733-778) with
 * densify_and_clone (:708-731), densify_and_split (:672-706), prune_points (:588-603),
 * cat_tensors_to_optimizer (:605-644) and densification_postfix (:646-670), as train_single.py:197
 * calls it (gt_point_cloud_constraints off).  With P0 rows, g = xyz_gradient_accum (NaN -> 0),
 * op = sigmoid(opacity_raw), smax = max_k exp(scaling_raw[k]), rows r >= first_row only:
 *
 *   clone  C_i = sqrt(g*g) * max_radii2D * op^0.2 >= max_grad  &&  op > 0.15  &&  smax <= max_scale
 *   split  S_i =        g  * max_radii2D * op^0.2 >= max_grad  &&  op > 0.15  &&  smax >  max_scale
 *   prune  Z_i = op < min_opacity   (clones and split children inherit their parent's opacity)
 *
 * The reference's sequence of cat / boolean-index operations leaves the rows, in order, as
 *   [old rows i with !S_i && !Z_i] [clones of C_i && !Z_i] [split children, set 1] [set 2]
 * (children of S_i && !Z_i; set k's child of the r-th split row uses normal sample row
 * (k-1)*n_split + r, where n_split counts every S_i).  A child's xyz is R(q) (z * exp(s)) + xyz,
 * its scaling_raw log(exp(s) * (1/1.6f)) (torch divides a tensor by a scalar through the fp32
 * reciprocal), every other array copied.
 * Optimizer moments: copied for old rows, zero for new rows.  Densification statistics are
 * all reset to zero by the reference and are not part of this ABI.
 *
 * Two calls: _plan (selection, ranks, output map, counts on the device; the host reads the
 * counts to allocate the new arrays and draw the 2 n_split x 3 standard normal samples exactly
 * as the reference's torch.normal does) and _apply (one launch writes every new array).
 */
#ifndef GSR_DENSIFY_H
#define GSR_DENSIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One per-Gaussian parameter group: (P, width) param and its two Adam moments (moments may be
 * NULL when the group has no optimizer state yet; destination moments are then not written). */
typedef struct {
    float *param;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t width;
} gsr_row_group;

/* Bytes of device scratch the pair of calls needs for P0 rows. */
size_t gsr_densify_scratch_bytes(int64_t P0);

/* counts (device, 4 x int64): {old rows kept, clones kept, n_split (all S rows), total output rows}. */
int gsr_densify_plan(int64_t P0, int64_t first_row, const float *grad_accum, const float *max_radii2D,
                     const float *opacity_raw, const float *scaling_raw, float max_grad, float min_opacity,
                     float max_scale, void *scratch, int64_t *counts, void *stream);

/* src[k] (P0 rows) -> dst[k] (counts[3] rows).  Group roles: xyz (width 3), scaling (width 3),
 * rotation (width 4) by index; normals: (2 * n_split, 3) standard normal samples (may be NULL
 * when n_split == 0).  Needs the scratch of the preceding _plan call. */
int gsr_densify_apply(int64_t P0, int n_groups, const gsr_row_group *src, const gsr_row_group *dst, int xyz_group,
                      int scaling_group, int rotation_group, const float *normals, int64_t n_split,
                      const void *scratch, int64_t total_rows, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_DENSIFY_H */
