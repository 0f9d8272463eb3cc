/*
 * gsr_train.h -- C ABI of the train-step kernels that sit either side of the rasterizer in one
 * Street-sparse-3DGS iteration.  Exported by the same
 * libgsr_hip.so as include/gsr.h.
 *
 *   gsr_l1_ssim_forward / _backward  replace  utils/loss_utils.py:17-18 (l1_loss) and :33-63
 *                                    (ssim: five 11x11 depthwise conv2d, sigma 1.5, zero pad),
 *                                    as combined at train_single.py:121-123
 *   gsr_sparse_adam_step             replaces scene/OurAdam.py:105-175 + _single_tensor_adam
 *                                    (:249-337) / _single_tensor_adam2 (:338-...) for the six
 *                                    Gaussian parameter groups (scene/gaussian_model.py:286-296),
 *                                    with `relevant = opacity.grad != 0` (train_single.py:224-230)
 *                                    evaluated on the device
 *   gsr_exposure_forward / _backward replace  the per-image exposure affine + clamp of render()
 *                                    (gaussian_renderer/__init__.py:115-120, use_trained_exp=True
 *                                    at train_single.py:111): a (H*W, 3) x (3, 3) GEMM, a
 *                                    broadcast add and a clamp in torch
 *   gsr_densify_stats                replaces train_single.py:193-194 +
 *                                    scene/gaussian_model.py:780-793 (add_densification_stats)
 *   gsr_activate_forward / _backward replace  the exp / normalize / sigmoid getters
 *                                    (scene/gaussian_model.py:39-47, 125-156) and their autograd
 *   gsr_shrink_scales                replaces train_single.py:235-241
 *
 * Conventions as in gsr.h: device pointers, fp32, contiguous, `stream` a hipStream_t.
 */
#ifndef GSR_TRAIN_H
#define GSR_TRAIN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes of device scratch gsr_l1_ssim_forward needs for C planes of H x W. */
size_t gsr_l1_ssim_scratch_bytes(int C, int H, int W);

/* out[0] = mean |img - gt|, out[1] = mean SSIM map (reference: l1_loss(img, gt), ssim(img, gt)).
 * img, gt: (C, H, W).  Deterministic (fixed-order reduction, no atomics). */
int gsr_l1_ssim_forward(const float *img, const float *gt, int C, int H, int W, void *scratch, float *out,
                        void *stream);

/* dL_dimg = dL_dout[0] * d(mean|img-gt|)/dimg + dL_dout[1] * d(mean SSIM)/dimg.
 * dL_dout is a 2-float DEVICE array (the autograd grad_outputs; no host sync). */
int gsr_l1_ssim_backward(const float *img, const float *gt, int C, int H, int W, const float *dL_dout,
                         float *dL_dimg, void *stream);

/* Training form of the pair above.  _forward_with_map computes out (as gsr_l1_ssim_forward, same
 * scratch) and, in the same pass, the per-pixel field G = d(sum of the SSIM map)/dimg into
 * ssim_grad_map (C, H, W); dL/dimg is linear in dL_dout, so _backward_from_map is then the
 * elementwise dL_dimg = (dL_dout[0] sign(img - gt) + dL_dout[1] G) / (C H W), equal to
 * gsr_l1_ssim_backward's result.  One halo recomputation per step instead of two. */
int gsr_l1_ssim_forward_with_map(const float *img, const float *gt, int C, int H, int W, void *scratch, float *out,
                                 float *ssim_grad_map, void *stream);
int gsr_l1_ssim_backward_from_map(const float *img, const float *gt, const float *ssim_grad_map, int C, int H, int W,
                                  const float *dL_dout, float *dL_dimg, void *stream);

/* The whole photometric loss of train_single.py:121-123,
 *   loss = (1 - lambda_dssim) * L1 + lambda_dssim * (1 - SSIM),
 * as one autograd node: _forward writes out3 = (L1, SSIM, loss) (the combination in torch's fp32
 * op order) and the SSIM gradient field; _backward takes the scalar dL/dloss (device pointer) and
 * forms the pair torch's backward of that expression would hand to gsr_l1_ssim_backward_from_map,
 * bit for bit.  Replaces the ~10 one-element torch launches of the composed expression and its
 * backward.  lambda_dssim in [0, 1]. */
int gsr_photo_loss_forward(const float *img, const float *gt, int C, int H, int W, double lambda_dssim, void *scratch,
                           float *out3, float *ssim_grad_map, void *stream);
int gsr_photo_loss_backward(const float *img, const float *gt, const float *ssim_grad_map, int C, int H, int W,
                            double lambda_dssim, const float *dL_dloss, float *dL_dimg, void *stream);

/* One parameter group of the sparse Adam step: a (P, width) row-major parameter with its grad
 * and moment buffers.  step_size = lr / (1 - beta1^step) and bias_correction2_sqrt =
 * sqrt(1 - beta2^step) are computed by the host in double, exactly as OurAdam does. */
typedef struct {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t width;
    float step_size;
    float bias_correction2_sqrt;
    /* Elements between consecutive rows of the four arrays (0 = width): a group may be a column
     * block of a wider array, e.g. the DC and rest SH coefficients of one (P, 16, 3) buffer,
     * each with its own learning rate, without splitting the buffer every step. */
    int64_t row_stride;
} gsr_adam_group;

/* Rows r with relevance[r] != 0 are updated in every group; if no row is relevant, every row
 * is updated (OurAdam's _single_tensor_adam2 branch).  flag_scratch: one device int.
 * relevance NULL: a dense step over every row (one launch; flag_scratch unused). */
int gsr_sparse_adam_step(int n_groups, const gsr_adam_group *groups, int64_t P, const float *relevance,
                         double beta1, double beta2, double eps, int *flag_scratch, void *stream);

/* out[c][p] = clamp(sum_k color[k][p] * E[k][c] + E[c][3], 0, 1) for the 3 planes of npix
 * pixels; E is the 3x4 exposure matrix (row-major, device). */
int gsr_exposure_forward(const float *color, const float *exposure, int64_t npix, float *out, void *stream);

/* Bytes of device scratch gsr_exposure_backward needs. */
size_t gsr_exposure_scratch_bytes(int64_t npix);

/* dL_dcolor (3, npix) and dL_dexposure (3x4) from dL_dout (3, npix); the clamp passes gradient
 * where 0 <= pre-clamp value <= 1 (torch.clamp).  dL_dexposure is overwritten (deterministic,
 * fixed-order reduction). */
int gsr_exposure_backward(const float *color, const float *exposure, int64_t npix, const float *dL_dout,
                          float *dL_dcolor, float *dL_dexposure, void *scratch, void *stream);

/* For rows with radii > 0: max_radii2D = max(max_radii2D, radii);
 * grad_accum = max(||dL_dmeans2D[:, :2]||, grad_accum); denom += 1. */
int gsr_densify_stats(int64_t P, const int *radii, const float *dL_dmeans2D, float *max_radii2D,
                      float *grad_accum, float *denom, void *stream);

/* scales = exp(scaling_raw) (P,3), rotations = normalize(rotation_raw) (P,4; 16-B aligned),
 * opacities = sigmoid(opacity_raw) (P,1): the getters of scene/gaussian_model.py:125-156 in one
 * pass. */
int gsr_activate_forward(int64_t P, const float *scaling_raw, const float *rotation_raw, const float *opacity_raw,
                         float *scales, float *rotations, float *opacities, void *stream);

/* Gradients of the raw parameters from those of the activated ones (torch autograd's formulas);
 * outputs are overwritten. */
int gsr_activate_backward(int64_t P, const float *rotation_raw, const float *scales, const float *opacities,
                          const float *dL_dscales, const float *dL_drotations, const float *dL_dopacities,
                          float *dL_dscaling_raw, float *dL_drotation_raw, float *dL_dopacity_raw, void *stream);

/* train_single.py:235-241: rows r >= first_row (the scaffold points come first) whose largest
 * exp(scaling_raw) exceeds max_scale get scaling_raw = log(exp(scaling_raw) * 0.8), in place. */
int gsr_shrink_scales(int64_t P, int64_t first_row, float *scaling_raw, float max_scale, void *stream);

/* Masked inverse-depth L1 of train_single.py:135-141 (the Street-sparse depth supervision):
 *   out2[0] = mean(|(invdepth - mono_invdepth) * mask|)   (Ll1depth_pure; mask NULL = all ones)
 *   out2[1] = weight * out2[0]                            (Ll1depth, weight = depth_l1_weight(it))
 * n = H * W elements, 16-byte aligned arrays; scratch of gsr_depth_l1_scratch_bytes(n).  The
 * backward writes dL/dinvdepth = ((dL/dout2[1] * weight) * (1/n)) * sgn(d) * mask, d = (invdepth -
 * mono) * mask: torch's autograd chain through the reference's expression, bit for bit. */
size_t gsr_depth_l1_scratch_bytes(int64_t n);
int gsr_depth_l1_forward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                         float weight, void *scratch, float *out2, void *stream);
int gsr_depth_l1_backward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                          float weight, const float *dL_dloss, float *dL_dinvdepth, void *stream);

/* The loss of a depth-only view (Street-sparse's additional depth maps, train_single.py:145-156):
 *   pure = mean(|(invdepth - mono_invdepth) * mask|)           (Ll1depth_pure; mask NULL = ones)
 *   dens = mean(clamp(mono_invdepth - invdepth, min=0))         (Ll1depth_dens, unmasked)
 *   loss = weight * (dens_weight * dens + (1 - dens_weight) * pure)
 * weight = depth_l1_weight(iteration), dens_weight = additional_depth_maps_weight (0.9 by
 * default, arguments/__init__.py:71).  _forward writes out3 = (pure, dens, loss) (the means in
 * fp64, the combination in torch's fp32 op order); _backward writes dL/dinvdepth for the scalar
 * dL/dloss (device pointer), torch's autograd chain through the reference's expression bit for
 * bit.  Scratch of gsr_depth_only_scratch_bytes(n); 16-byte aligned arrays. */
size_t gsr_depth_only_scratch_bytes(int64_t n);
int gsr_depth_only_loss_forward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                                float weight, double dens_weight, void *scratch, float *out3, void *stream);
int gsr_depth_only_loss_backward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                                 float weight, double dens_weight, const float *dL_dloss, float *dL_dinvdepth,
                                 void *stream);

/* ---- Native train-step executor ------------------------------------------------------------
 * gsr_train_step runs one whole Street-sparse iteration (train_single.py:65-247: render with
 * the exposure of the view, photometric loss + masked inverse-depth L1, backward, densification
 * statistics, exposure Adam, skybox lock, sparse Adam, scale shrink) as ONE host call, with the
 * arithmetic of the entry points above and gsr_rasterize_forward_ex / _backward in the order
 * gs_train/harness.py TrainStep.step issues them (several fused into one launch), so its results
 * are those of the Python step (bit for bit in the deterministic backward mode).  The context owns every per-step
 * intermediate (rasterizer buffers, images, activated values and their gradients) in grow-only
 * device allocations reused across steps; the caller owns the parameters, their gradients
 * (overwritten each step), the Adam moments and the densification statistics.
 * Replaces the Python-driven step; none of the reference's files has a native executor. */
typedef struct gsr_train_ctx gsr_train_ctx;
gsr_train_ctx *gsr_train_ctx_create(void);
/* Waits for the last step's stream, then frees the context's device buffers. */
void gsr_train_ctx_destroy(gsr_train_ctx *ctx);
/* The context's buffer statistics: out[0] = buffer growths since creation (each re-allocates one
 * grow-only buffer 1/4 larger than asked; stream-ordered, hipFreeAsync / hipMallocAsync from the
 * device's default pool, unless GSR_STEP_SYNC_ALLOC=1), out[1] = bytes held, out[2] = 1 when the
 * growth is stream-ordered.  Returns the number of values written (<= n).  ABI 5. */
int gsr_train_ctx_stats(const gsr_train_ctx *ctx, int64_t *out, int n);

typedef struct {
    int64_t P;   /* Gaussians */
    int D, M;    /* active SH degree, coefficients per Gaussian (features is (P, M, 3)) */
    int width, height;
    /* parameters (updated in place) and their gradients (overwritten) */
    float *xyz, *features, *opacity, *scaling, *rotation;           /* raw: (P,3) (P,M,3) (P,1) (P,3) (P,4) */
    float *xyz_grad, *features_grad, *opacity_grad, *scaling_grad, *rotation_grad;
    float *exposure, *exposure_grad; /* (n_images, 3, 4); the gradient is zero outside image_index */
    int n_images, image_index;
    /* the view */
    const float *viewmatrix, *projmatrix, *campos; /* device: 16, 16, 3 */
    float tan_fovx, tan_fovy;
    const float *background;                        /* device: 3 */
    const float *gt;                                /* (3, H, W) */
    const float *alpha_mask;                        /* (H, W) or NULL */
    const float *mono_invdepth, *depth_mask;        /* (H, W) or NULL (no depth term); mask NULL = ones */
    float depth_weight;                             /* depth_l1_weight(iteration); <= 0: no depth term */
    double lambda_dssim;
    /* densification statistics (P) */
    float *max_radii2D, *xyz_gradient_accum, *denom;
    /* optimizers: the Gaussian groups (their grad pointers are the gradients above) and the
     * exposure's one dense group (n_images rows of 12) */
    int n_groups;
    const gsr_adam_group *groups;
    double beta1, beta2, eps;
    const gsr_adam_group *exposure_group;
    double exposure_beta1, exposure_beta2, exposure_eps;
    int64_t skybox_rows;   /* the first rows: their opacity gradient is zeroed before the sparse step */
    int64_t scaffold_rows; /* the first rows: left alone by the scale shrink */
    float max_scale;       /* shrink rows whose largest scale exceeds this (extent * 0.02) */
    /* out (device, 6 floats): L1, SSIM, photometric loss, (depth term only) the unweighted and
     * weighted depth L1, then the step's loss ([2] + [4], or [2]); depth-only view: Ll1depth_dens,
     * 0, 0, Ll1depth_pure, Ll1depth, loss */
    float *losses;
    void *stream;
    /* A depth-only view (train_single.py:69-72,145-161,203-214; ABI 3): no target image; the loss
     * is gsr_depth_only_loss's (depth_weight > 0 and mono_invdepth required), the colour gradient
     * is zero, the exposure gradient is zeroed and no exposure Adam step runs (the caller does not
     * advance the exposure optimizer's step count).  gt may be NULL. */
    int depth_only;
    double depth_dens_weight; /* additional_depth_maps_weight */
    /* Nonzero: everything up to the optimizers only (forward, losses, backward, densification
     * statistics, exposure step) -- no Gaussian Adam step and no scale shrink.  An iteration of
     * train_single.py that densifies / resets the opacities replaces the parameters between the
     * statistics and the optimizers and then takes no Gaussian Adam step (:190-201, :217, :225);
     * the caller runs those and the shrink itself (gsr_shrink_scales).  ABI 3. */
    int skip_gaussian_step;
} gsr_train_step_args;

/* *num_rendered receives the frame's K. */
int gsr_train_step(gsr_train_ctx *ctx, const gsr_train_step_args *args, int64_t *num_rendered);

#ifdef __cplusplus
}
#endif
#endif /* GSR_TRAIN_H */
