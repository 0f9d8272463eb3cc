/*
 * gsr.h -- C ABI of the MI355X (gfx950) Gaussian-splat rasterizer library
 * (street-sparse-3dgs_amd/diff_gaussian_rasterization/libgsr_hip.so).
 *
 * This is the drop-in boundary for the hot path named in BASELINE.json: the entry points
 * are the ones the reference's torch extension binds (`diff_gaussian_rasterization._C`,
 * imported at gaussian_renderer/__init__.py:14,17 of Street-sparse-3DGS; the extension's
 * source lives in the un-vendored submodule submodules/hierarchy-rasterizer,
 * .gitmodules:5-7).  Plain pointers and sizes only: no torch types cross this line.
 *
 *   gsr_rasterize_forward   replaces  _C.rasterize_gaussians           (called from the
 *                                     autograd Function's forward)
 *   gsr_rasterize_backward  replaces  _C.rasterize_gaussians_backward  (autograd backward)
 *   gsr_mark_visible        replaces  _C.mark_visible                  (GaussianRasterizer.markVisible)
 *
 * Conventions:
 *   - every array pointer is DEVICE memory on the current HIP device, fp32 unless noted,
 *     row-major and contiguous; `stream` is a hipStream_t (NULL = default stream);
 *   - viewmatrix / projmatrix are the 4x4 torch row-major tensors W2C^T and (P W2C)^T,
 *     read column-major (scene/cameras.py:96-99 of the reference);
 *   - shs is (P, M, 3) coefficient-major / channel-minor; rotations are (r,x,y,z) used as
 *     given (the caller normalises, scene/gaussian_model.py:47); cov3D is the 6-float
 *     upper triangle xx,xy,xz,yy,yz,zz;
 *   - scratch ("geometry", "binning", "image", "backward") buffers are obtained through the
 *     caller's resize callback so they live in the caller's allocator (the torch caching
 *     allocator in the Python host) and are handed back to the backward call unchanged.
 *
 * Return value: GSR_OK (0) or a negative gsr_status; gsr_last_error() gives the message.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 6

typedef enum {
    GSR_OK = 0,
    GSR_ERR_INVALID_ARGUMENT = -1,
    GSR_ERR_ALLOCATION = -2,
    GSR_ERR_DEVICE = -3,
    GSR_ERR_UNSUPPORTED = -4
} gsr_status;

/* Resize callback: return a device pointer to at least `bytes` bytes that stays valid until
 * the caller releases it (after the backward call).  Called at most once per buffer per call.
 * Returning NULL aborts the call with GSR_ERR_ALLOCATION. */
typedef void *(*gsr_resize_fn)(void *ctx, size_t bytes);

/* Forward: preprocess -> depth sort + scan -> binning (per-tile lists + ranges) -> blend.
 * Mirrors CudaRasterizer::Rasterizer::forward as the reference's
 * _C.rasterize_gaussians(bg, means3D, colors, opacity, scales, rotations, scale_modifier,
 * cov3D_precomp, viewmatrix, projmatrix, tanfovx, tanfovy, H, W, sh, degree, campos,
 * prefiltered, debug, render_indices, parent_indices, interpolation_weights, num_node_kids,
 * do_depth) drives it.
 *   shs / colors_precomp: exactly one non-NULL.  scales+rotations / cov3D_precomp: exactly one.
 *   M = shs.shape[1] (coefficient stride), D = active SH degree (0..3, (D+1)^2 <= M).
 *   out_color (3,H,W); out_invdepth (1,H,W) or NULL when do_depth is false; radii (P) int32.
 *   render_indices/parent_indices/interpolation_weights/num_node_kids: the hierarchy-cut
 *   fields.  num_render == 0 (every reference call path: render_post blends in Python and
 *   passes empty ones) means plain 3DGS and the four pointers are never dereferenced (they may
 *   be host pointers).  num_render = R > 0: the P input rows are a hierarchy's Gaussians and the
 *   frame renders the R rows render_post's blend would produce (gaussian_renderer/__init__.py:
 *   200-220; row r = t * x[render_indices[r]] + (1 - t) * x[parent_indices[r]], parent
 *   quaternions sign-aligned, t = interpolation_weights[r], parent -1 = the last row); needs shs,
 *   scales and rotations; the three arrays are device int32 / int32 / float32 of >= R entries;
 *   radii then has R entries.  num_node_kids is accepted and not read (render_post ignores it).
 *   *num_rendered receives K, the number of tile instances. */
int gsr_rasterize_forward(gsr_resize_fn geom_buffer, gsr_resize_fn binning_buffer, gsr_resize_fn image_buffer,
                          void *resize_ctx, int P, int D, int M, const float *background, int width, int height,
                          const float *means3D, const float *shs, const float *colors_precomp,
                          const float *opacities, const float *scales, float scale_modifier,
                          const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                          const float *projmatrix, const float *cam_pos, float tan_fovx, float tan_fovy,
                          int prefiltered, float *out_color, float *out_invdepth, int *radii,
                          const int *render_indices, const int *parent_indices,
                          const float *interpolation_weights, const int *num_node_kids, int num_render,
                          int debug, void *stream, int64_t *num_rendered);

/* gsr_rasterize_forward with flags (same arguments, then `flags`; gsr_rasterize_forward passes 0).
 *   GSR_FWD_NO_BACKWARD: no backward will follow (the Python host sets it when autograd records
 *   no graph: torch.no_grad() frames such as render_hierarchy.py's evaluation loop, SURVEY.md
 *   3.3).  The frame skips clearing the backward's per-Gaussian accumulator rows (64 B per
 *   Gaussian) and building the backward's tile order; gsr_rasterize_backward on its buffers fails
 *   with GSR_ERR_INVALID_ARGUMENT. */
#define GSR_FWD_NO_BACKWARD 1u
int gsr_rasterize_forward_ex(gsr_resize_fn geom_buffer, gsr_resize_fn binning_buffer, gsr_resize_fn image_buffer,
                             void *resize_ctx, int P, int D, int M, const float *background, int width, int height,
                             const float *means3D, const float *shs, const float *colors_precomp,
                             const float *opacities, const float *scales, float scale_modifier,
                             const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                             const float *projmatrix, const float *cam_pos, float tan_fovx, float tan_fovy,
                             int prefiltered, float *out_color, float *out_invdepth, int *radii,
                             const int *render_indices, const int *parent_indices,
                             const float *interpolation_weights, const int *num_node_kids, int num_render,
                             int debug, void *stream, int64_t *num_rendered, unsigned flags);

/* Backward.  geom/binning/image are the pointers the forward's callbacks returned; R = K.
 * The hierarchy-cut fields must be the forward's; with num_render > 0 the gradients of the P
 * input rows are those of render_post's blend (shared parents summed) and dL_dmeans2D holds the
 * rendered rows' screen-space gradient in rows [0, num_render), zero below.
 * dL_dpix (3,H,W); dL_dinvdepth (1,H,W) or NULL (no depth gradient).  `scratch` provides
 * the per-tile-instance gradient workspace.  The call is repeatable: a second backward through
 * the same buffers (retain_graph) returns the same gradients.  Every output row is written (zeros where
 * radii == 0 and beyond the active SH degree), so outputs need no pre-zeroing:
 *   dL_dmeans2D (P,3)  dL_dcolors (P,3) [may be NULL when shs != NULL]  dL_dopacity (P,1)
 *   dL_dmeans3D (P,3)  dL_dcov3D (P,6) [may be NULL when cov3D_precomp == NULL]
 *   dL_dsh (P,M,3) [ignored if shs == NULL]
 *   dL_dscales (P,3)  dL_drotations (P,4) [ignored if scales == NULL]
 * (the optional ones are identically zero there: the caller need not allocate them) */
int gsr_rasterize_backward(gsr_resize_fn scratch, void *resize_ctx, int P, int D, int M, int64_t R,
                           const float *background, int width, int height, const float *means3D,
                           const float *shs, const float *colors_precomp, const float *scales,
                           float scale_modifier, const float *rotations, const float *cov3D_precomp,
                           const float *viewmatrix, const float *projmatrix, const float *cam_pos,
                           float tan_fovx, float tan_fovy, const int *radii, void *geom_buffer,
                           void *binning_buffer, void *image_buffer, const float *dL_dpix,
                           const float *dL_dinvdepth, float *dL_dmeans2D, float *dL_dcolors, float *dL_dopacity,
                           float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscales,
                           float *dL_drotations, const int *render_indices, const int *parent_indices,
                           const float *interpolation_weights, const int *num_node_kids, int num_render,
                           int debug, void *stream);

/* Frustum test (view-space z > 0.2), present[P] as bytes 0/1. */
int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream);

/* Per-stage device time of the last forward/backward on this thread, filled only when
 * gsr_set_profiling(1) was called (HIP events; for bench.py's roofline).  Stage order:
 * 0 preprocess, 1 depth sort + scan, 2 binning level 1 (superblocks), 3 binning level 2 (tiles and
 * ranges), 4 forward tile order, 5 render_fwd, 6 render_bwd, 7 preprocess_bwd, 8 SH colour (on an
 * internal side stream, overlapping stages 1-4; joined before stage 5), 9 backward tile order.
 * Returns the number of stages written. */
int gsr_set_profiling(int enable);
int gsr_stage_times_ms(float *out, int max_stages);

/* dL/dscales convention, process-wide.  0 (default): upstream's -- the gradient with respect to
 * the modified scale scale_modifier * s, reported as dL/ds.  1: the exact derivative dL/ds
 * (multiplied by scale_modifier; identical when scale_modifier == 1).  Returns the previous mode. */
int gsr_set_true_scale_gradient(int enable);

/* Backward accumulation mode, process-wide.  0 (default): render_bwd adds every tile instance's
 * ten per-Gaussian gradient sums into a per-Gaussian row with hardware float atomics (like
 * upstream's atomicAdd accumulation: results vary in the last bits from run to run).  1: each
 * instance writes a record and a second pass sums every Gaussian's records in a fixed order --
 * forward + backward bitwise reproducible, slower.  A frame's backward uses the mode that was in
 * force at its forward.  Returns the previous mode. */
int gsr_set_deterministic(int enable);

/* Backward work split, process-wide.  L = 0: render_bwd replays every tile in one workgroup.
 * L > 0 (a multiple of 64, >= 512; default 512): the forward checkpoints each pixel's transmittance
 * and accumulated colour every L list positions of its tile, and the backward replays a tile whose
 * last contributor lies past L as ceil(work / L) independent segments (the few very long tiles of a
 * street view no longer form the kernel's tail).  Gradients agree with the unsegmented replay to
 * fp32 rounding.  A frame's backward uses the length its forward was made with.  Returns the
 * previous length, or GSR_ERR_INVALID_ARGUMENT / GSR_ERR_UNSUPPORTED. */
int gsr_set_bwd_segment(int L);

/* Forward work split, process-wide.  L = 0: render_fwd blends every tile in one workgroup.  L > 0
 * (a multiple of 64, >= 1024; default 2048, behind the split gate): a tile whose list is longer than
 * 6 L (gsr_set_fwd_split_min) is blended as
 * ceil(len / L) work items by a pool of worker workgroups -- each item multiplies out the
 * transmittance through its positions, takes its predecessors' product (in segment order) and
 * blends its positions from there; the tile's last item adds the items' colours in order.  Colours
 * agree with the one-workgroup blend to fp32 summation order; the stop rule is the same up to an
 * ulp of the transmittance product.  Returns the previous length, or GSR_ERR_INVALID_ARGUMENT /
 * GSR_ERR_UNSUPPORTED. */
int gsr_set_fwd_segment(int L);

/* The shortest tile list the forward split takes, process-wide: 0 (default) = 6 segments
 * (GSR_FSEG_FACTOR); otherwise max(len, L).  Returns the previous setting. */
int gsr_set_fwd_split_min(int len);

/* The forward-split workers' bounded spins, process-wide (for tests; 0 = the default): `ready` loop
 * trips (~256 clocks each) waiting for tile_order's release of the queue, after which a worker
 * leaves (counted in gsr_forward_stats[4]; the pool's second launch blends its items), and `flag`
 * trips (~128 clocks) waiting for a predecessor segment's transmittance, after which that tile's
 * pixels are NaN and the next rasterizer call on the thread fails (GSR_ERR_DEVICE).  ready = -1 (fault
 * injection): the workers leave without waiting, as if the release never came.  ABI 5. */
int gsr_set_fwd_spin_limits(int64_t ready, int64_t flag);

/* The split gate, process-wide.  1 (default): the forward split (gsr_set_fwd_segment) and the
 * tile binning's split of long superblock lists are armed only for the 256 frames (per device and
 * calling thread) after one whose longest tile / superblock list called for them -- they cost a few
 * microseconds of launches and stream hand-offs per frame and pay only on such frames.  0: armed on
 * every frame (the outputs are the same either way, to fp32 summation order).  Returns the previous
 * setting. */
int gsr_set_split_gate(int enable);

/* How the backward walks the live rows (the Gaussians with a nonzero screen-space gradient),
 * process-wide.  0 (default): each 2048-row range's workgroup walks its own live rows -- one launch,
 * the better choice when the live rows are scattered over the model (rows in the order training
 * appends them).  1: the ranges append their live rows to one list that a grid of two workgroups
 * per CU walks -- one more launch, every thread the same share, the better choice when the rows are
 * in spatial order and a view's live rows come in runs (gs_train.chunk.reorder_rows).  The
 * gradients are the same bits either way.  Returns the previous setting (ABI 6). */
int gsr_set_live_list(int enable);

/* Diagnostic (host arithmetic only): the bytes the backward checkpoints and the forward items need
 * past the start of a binning buffer carved for K instances with segment lengths L / Lf (*need),
 * and the buffer's size (*have).  GSR_OK when they fit. */
int gsr_segment_layout_check(int64_t K, int L, int Lf, int64_t *need, int64_t *have);

/* Depth-order strategy of the binning, process-wide.  0: the local sort -- level 1 in Gaussian
 * index order, each superblock list sorted by depth in LDS -- except for frames forwarded in
 * deterministic mode and frames with a superblock list longer than the LDS sort holds, which take
 * the global sort.  1 (default): always the global depth sort of all P Gaussians (dsort.hip).  Both
 * give the same per-tile lists.  Returns the previous mode (or GSR_ERR_INVALID_ARGUMENT). */
int gsr_set_binning(int mode);

/* Forward statistics since load: out[0] = frames rasterized (P > 0), out[1] = frames whose
 * binning ran twice because the capacity hint from the previous frame was short of K,
 * out[2] = frames binned by the local sort, out[3] = local frames re-run through the global sort
 * (a superblock list too long for LDS), out[4] = frames whose forward-split workers gave up waiting
 * for tile_order's release of their queue (the side stream did not run beside the main one; the
 * pool's second launch completed those frames exactly -- ABI 5), out[5] = host nanoseconds spent waiting
 * for K (num_rendered) in forward calls, out[6] / out[7] = frames forwarded with the forward split /
 * the tile binning's superblock split armed (gsr_set_split_gate; ABI 5).  Returns the number of
 * values written (<= n). */
int gsr_forward_stats(int64_t *out, int n);

/* The forward-split worker pool's time since load (or the last reset), in s_memrealtime ticks of
 * 10 ns summed over its workgroups: out[0] waiting for tile_order's release of the queue, out[1]
 * waiting for predecessor segments' transmittance, out[2] the workgroups' lifetimes, out[3] the
 * workgroups.  The pool's busy fraction is 1 - (out[0] + out[1]) / out[2].  Synchronises the
 * device; reset != 0 zeroes the counters.  Returns the number of values written (<= n). */
int gsr_fwd_pool_stats(int64_t *out, int n, int reset);

/* Forget the calling thread's point-list capacity hint (the largest K of its last 256 frames per
 * device) and its split-gate history: the next frame reads K before binning, as the first one does,
 * and the gated splits wait for a long-list frame again.  For a caller that switches to a much
 * smaller workload (the buffers follow the hint) and for tests.  ABI 3. */
int gsr_reset_capacity_hint(void);

/* Statistics of one forward frame, read from its geometry buffer (synchronises the device):
 * out[0] = level-1 binning entries (Gaussian x superblock pairs, "P1" of DESIGN.md), out[1] = tile
 * instances (K), out[2] = tile_bin split items queued (global-sort frames), out[3] = the longest
 * superblock list.  P = the frame's rendered rows (num_render when non-zero).  Returns the number
 * of values written (<= n).  For bench.py's algorithmic-bytes model. */
int gsr_frame_stats(const void *geom_buffer, int P, int width, int height, int64_t *out, int n);

/* Measurement builds only (a variant library compiled with -DGSR_BLEND_STATS=1; zeros otherwise):
 * lane-liveness counters of the blend kernels since the last reset, out[0..13] = backward
 * {(instance, sub-block) pairs, live lanes, live 8x4 halves, live 16x1 rows, live 4x4 quads,
 * staged instances, batches}, forward {pairs, alpha-passing lanes, halves, rows, quads, accepted
 * lanes}, backward tiles.  reset != 0 zeroes them after the read.  Returns the count written. */
int gsr_blend_stats(int64_t *out, int n, int reset);

/* Measurement builds only (-DGSR_SB_TRACE=1; zeros otherwise): per-workgroup phase stamps of the
 * local sort kernel, 8 words per superblock (s_memrealtime at 100 MHz; word 7 = list length).
 * -DGSR_HOST_TRACE=1 builds instead: the host nanoseconds spent issuing each stage (out[0..9], the
 * gsr_stage_times_ms order), whole forward and backward calls (out[10], out[11]) and the matching
 * counts (out[12..23]).  reset != 0 zeroes them after the read.  Returns the count written. */
int gsr_debug_trace(int64_t *out, int n, int reset);

/* Measurement builds only (-DGSR_KSTAMP=1; GSR_ERR_UNSUPPORTED otherwise): the instrumented kernels'
 * last 4 launches on the GPU's clock, out[24 * 9]: per kernel id (gsr_device.h KsId) its launch
 * count, 4 starts and 4 ends (s_memrealtime ticks, 100 MHz).  tools/kstamp.py turns them into the
 * frame's timeline with the idle gaps between kernels. */
int gsr_kstamp_read(unsigned long long *out, int n);

/* Version / diagnostics. */
int gsr_abi_version(void);
const char *gsr_last_error(void);
const char *gsr_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
