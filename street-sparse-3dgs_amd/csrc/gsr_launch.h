// gsr_launch.h -- host-side launchers for the gfx950 kernels (one translation unit each).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "gsr_device.h"
#include "../../include/gsr_train.h"

namespace gsr {

// rasterizer.hip: message returned by gsr_last_error() for the calling thread.
void set_last_error(const std::string &msg);
// gsr_set_true_scale_gradient: dL/dscales including the scale_modifier factor (default off: upstream)
bool true_scale_gradient();

struct Camera {
    const float *view;  // device, 16
    const float *proj;  // device, 16
    const float *campos;  // device, 3
    float tanx, tany, fx, fy;
    int W, H, gx, gy;
};

// raw (the native train step, set_raw_params): scales / rotations / opacities are the
// pre-activation parameters (log-scales, unnormalised quaternions, logits), activated in the
// kernels that read them (gsr_device.h act_*), so no activated copy is written and re-read.
struct GaussianInputs {
    int P, D, M;
    const float *means3D, *shs, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp;
    float scale_modifier;
    int raw;
    // cut.ri != nullptr (render_post's blend fused, forwards without a backward): the P rows are
    // blended on the fly from the cut.N rows the pointers above address (gsr_device.h CutRef)
    CutRef cut{};
};
// the fused cut is supported for SH frames the colour pass takes (M = 16), scales + rotations
bool cut_fusable(const GaussianInputs &in);
// rasterizer.hip: gsr_rasterize_forward_ex / gsr_rasterize_backward on this thread take raw
// parameters (plain frames: no precomputed covariance, no hierarchy cut)
void set_raw_params(bool on);

// preprocess.hip
void launch_preprocess(const GaussianInputs &in, const Camera &cam, const GeomState &gs, int *radii,
                       hipStream_t s, bool split_color);
// SH colour of the visible Gaussians (rec.col, clamped) after a split_color preprocess
bool color_split_supported(const GaussianInputs &in);
// blocks > 0: a persistent grid of that many blocks (the pass held to part of the chip)
void launch_preprocess_color(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const int *radii,
                             hipStream_t s, int blocks = 0);
// render.hip: tiles ordered heaviest first by work[t] (or, with work == NULL, by list length).
// fctl != NULL and fseg_len != 0: also the forward segments' item queue (FwdSegLayout in the
// binning buffer at bin_base; fctl = bwd_cnt + kFwdItemsWord).
void launch_tile_order(const uint32_t *work, const uint2 *ranges, int T, int shift, uint32_t *order, hipStream_t s,
                       const uint32_t *kdev = nullptr, uint32_t cap = 0, uint32_t *zero_classes = nullptr,
                       uint32_t *fctl = nullptr, void *bin_base = nullptr, uint32_t seg_len = 0, uint32_t fseg_len = 0,
                       uint32_t *host_tilelist = nullptr, uint32_t *fwd_ready = nullptr, uint32_t fseg_min = 0);
void launch_mark_visible(int P, const float *means3D, const float *view, uint8_t *present, hipStream_t s);

// sort.hip (rocPRIM)
// Stable LSD sort of n (key, value) pairs over key bits [0, end_bit) (kNN Morton order).
size_t sort_pairs_temp_bytes(size_t n, int end_bit);
hipError_t sort_pairs(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                      uint32_t *vout, size_t n, int end_bit, hipStream_t s);
// dsort.hip: the stable (depth bits, id) order of the P Gaussians (gs.order), depth-ordered tile
// rects (gs.drect, from gs.rect8), the Gaussian-major record offsets (rec.off) and
// K = sum of tiles_touched, stored to *dsort_K_word and, when host_K != NULL, to that pinned
// host word; k_ready (optional) is recorded once K is final, before the sort passes run.
int dsort_blocks(int P);
size_t dsort_ctrl_words(int P);
size_t dsort_ctrl_zero_words(int P);
// host_err (optional, pinned): set with a system-scope store when a lookback spin gives up.
void launch_depth_sort(int P, const GeomState &gs, uint32_t *host_K, uint32_t *host_err, hipStream_t s,
                       hipEvent_t k_ready);
uint32_t *dsort_K_word(const GeomState &gs);
uint32_t *dsort_err_word(const GeomState &gs);
// a zeroed-per-frame control word the binning uses as a completion counter
uint32_t *dsort_aux_word(const GeomState &gs);
// local-sort frames: the longest SB list (sb_colscan); the head words (tickets, counters, K, ...)
// a frame re-run through the global sort must zero again
uint32_t *dsort_maxsb_word(const GeomState &gs);
// the forward split's queue-ready word (zeroed with the control words by every frame's preprocess)
uint32_t *dsort_fwdready_word(const GeomState &gs);
// the frame's longest tile list and superblock list, [2] (zeroed by the preprocess; render_fwd copies
// them to the pinned host words)
uint32_t *dsort_longest_words(const GeomState &gs);
int device_cus();  // compute units of the current device (rasterizer.hip, cached)
uint32_t *dsort_live_words(const GeomState &gs);
uint32_t *dsort_culled_word(const GeomState &gs);  // culled Gaussians of the frame (the upsweep's sum)
int dsort_head_words();
// binning.hip: per-tile lists (two stable counting levels).  index_order: level 1 over the
// Gaussians in index order (local sort: sb_sort_bin orders each SB list by depth in LDS); else over
// dsort's depth order (gs.order / gs.drect; tile_bin).
SBGrid sb_grid(int gx, int gy, int P);
bool sb_grid_supported(const SBGrid &g);
int sort_cap();  // the longest SB list the local sort holds
int debug_trace(int64_t *out, int n, int reset);  // GSR_SB_TRACE builds: sb_sort_bin phase stamps
// level-1 counts and SB bases; with fw.dev_K set (local sort) the column scan also stores K, the
// longest SB list and the level-1 total (FrameWords)
// sb_order != NULL: the SBs in forward launch order (GSR_FWD_SB_ORDER); zero_classes != NULL: the
// backward class counters render_fwd fills are zeroed (GSR_BWD_CLS)
void launch_binning_count(int P, const Camera &cam, const GeomState &gs, bool index_order, const FrameWords &fw,
                          uint32_t *sb_order, uint32_t *zero_classes,
                          hipStream_t s, uint32_t tb_split = 0, uint32_t *host_sblist = nullptr);
void launch_binning_scatter(int P, const Camera &cam, const GeomState &gs, const BinningState &bs, bool index_order,
                            hipStream_t s);
// local_sort: sb_sort_bin (exits when *maxsb > sort_cap()); else tile_bin over depth-ordered lists
void launch_binning_tiles(int P, const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                          bool local_sort, const uint32_t *maxsb, hipStream_t s, bool tb_split = false,
                          hipStream_t split_stream = nullptr);

// The gradient arrays render_bwd zeroes beside its replay (ZeroRows): up to six arrays (float
// counts n[k], 16-B aligned; unused entries n = 0) as one concatenated float4 range split evenly
// over the backward's workgroups (per4 float4 each; c4 the cumulative float4 counts).  render_bwd
// also stamps the Gaussians it stages (GeomState.live_stamp = this backward's stamp), and
// preprocess_bwd then runs the chain rule over the stamped rows only and writes nothing else.
constexpr int kZeroArrays = 6;
struct ZeroRows {
    float *p[kZeroArrays];
    uint64_t n[kZeroArrays];
    uint64_t c4[kZeroArrays + 1];
    uint64_t per4;
    uint32_t zfrom;    // workgroups below zfrom carry no zero rows (workgroup b >= zfrom: slice b - zfrom)
    uint32_t *stamps;  // != NULL: render_bwd stamps every staged Gaussian (live_stamp) with `stamp`
    uint32_t stamp;
};

// render.hip
void launch_render_fwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const float *bg, float *out_color, float *out_invdepth, hipStream_t s, bool need_bwd = true,
                       bool sb_order = false, uint32_t seg_len = 0, uint32_t fseg_len = 0,
                       hipStream_t worker_stream = nullptr, bool workers_launched = false,
                       const uint32_t *longest = nullptr, uint32_t *host_words = nullptr, uint32_t fseg_min = 0,
                       FwdSpin spin = FwdSpin{kFwdReadySpins, kFwdFlagSpins, nullptr});
// Forward segments' worker pool launched ahead of tile_order (on a side stream that has waited for
// the binning and the colour pass): its workgroups are resident before render_fwd's grid fills the
// CUs and start on the queue as soon as tile_order (given the same word) releases `ready`
// (dsort_fwdready_word: zero since the frame's preprocess).
void launch_render_fwd_workers(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                               const float *bg, float *out_color, float *out_invdepth, bool need_bwd, uint32_t seg_len,
                               uint32_t fseg_len, hipStream_t ws, const uint32_t *ready, FwdSpin spin);
// The pool's second launch, on the main stream after render_fwd when the pool was launched ahead:
// a small grid that takes whatever the early workers left in the queue (nothing, unless some gave up
// waiting for tile_order's ready word because the two streams did not run concurrently).
void launch_render_fwd_cleanup(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                               const float *bg, float *out_color, float *out_invdepth, bool need_bwd, uint32_t seg_len,
                               uint32_t fseg_len, hipStream_t s, FwdSpin spin);
// the workers' spin limits (gsr_set_fwd_spin_limits) with the pinned host words
FwdSpin fwd_spin(uint32_t *host_words);
void set_fwd_spin_limits(uint32_t ready, uint32_t flag);
// GSR_FWD_EARLY_WORKERS (default 1): launch_render_fwd_workers before tile_order; 0: beside render_fwd
bool fwd_early_workers();
// seg_len != 0: the backward's heavy tiles are cut into segments of seg_len list positions
// (gsr_set_bwd_segment; the backward must get the value its forward was made with)
void launch_render_bwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const int *radii, const float *bg, const float *dL_dpix, const float *dL_dinvdepth,
                       const BwdScratch &sc, hipStream_t s, const ZeroRows *zr = nullptr, uint32_t seg_len = 0);
bool bwd_segments_supported();
bool fwd_segments_supported();
bool fwd_segments_in_kernel();  // the worker pool inside render_fwd's launch (no side stream)
uint32_t fseg_min_len(uint32_t Lf);  // the shortest list the forward split takes
uint32_t set_fwd_split_min(uint32_t len);  // gsr_set_fwd_split_min

// backward.hip
// sparse_rows (the native train step only, set_sparse_grad_rows): the rows of Gaussians with ten
// zero accumulated sums (every gradient zero) are not written in dmeans3D / dsh / dscales / drots,
// and dmeans2D's third column carries the row's liveness (1 written, 0 not) instead of its zero.
// Only rows whose opacity gradient is nonzero are read by the sparse Adam (OurAdam's `relevant`,
// train_single.py:226), and its dense fallback reads the liveness column.
struct GaussianGrads {
    float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *dsh, *dscales, *drots;
    int sparse_rows;
};
// rasterizer.hip: gsr_rasterize_backward on this thread writes sparse rows (see above)
void set_sparse_grad_rows(bool on);

// The native step's activation backward fused into the live-row pass of preprocess_bwd
// (set_step_act around gsr_rasterize_backward): the gradient outputs are then the raw parameters'
// gradients (dscales / drots / dopacity: of the log-scales, the unnormalised quaternions and the
// logits, skybox rows' opacity gradient locked at zero, train_single.py:217-223), the
// densification statistics of every visible row are updated (train_single.py:193-194) and *flag
// is set when a row's opacity gradient is nonzero (OurAdam's `relevant`).  step_act_done() says
// whether the last backward on this thread did it (else the caller runs the activation backward).
struct StepAct {
    const float *s_raw, *o_raw;
    const float4 *q_raw;
    int64_t skybox;
    const int *radii;
    float *maxr, *accum, *denom;
    int *flag;
    int on;
};
void set_step_act(const StepAct *a);
StepAct step_act();
bool live_list();  // gsr_set_live_list
void note_step_act_done(bool done);
bool step_act_done();
void launch_preprocess_bwd(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const ImageState &is,
                           const int *radii, const BwdScratch &sc, const GaussianGrads &out, hipStream_t s,
                           const ZeroRows *zr = nullptr);
// the frame's gradient arrays for render_bwd to zero and its live stamps (false: preprocess_bwd
// writes the zeros itself -- record mode, the single-kernel path, unaligned arrays or
// GSR_BWD_ZERO_IN_RENDER=0)
bool bwd_zero_rows(const GaussianInputs &in, const GaussianGrads &out, const BwdScratch &sc, uint32_t *gs_stamps,
                   int nblocks, ZeroRows *z);

// train.hip: the native train step's fused launches (train_step.hip).  sparse_adam is
// gsr_sparse_adam_step (flag_ready: the relevance flag is already computed; shrink_raw != NULL:
// train_single.py:235-241's scale shrink of rows >= shrink_first in the same launch).
// live3 != NULL (sparse gradient rows): when no row is relevant, the dense fallback takes a zero
// gradient for rows whose live3[3 row + 2] is 0 (never written) and for the locked skybox rows
// below `skybox` (train_single.py:217-223 zeroes all six of their gradients).
// row_list: scratch of >= P + 64 ints for the compacted row list (the train context's grow-only
// slot); NULL: allocated per call in stream order, and the row-block kernel (no scratch) runs when
// that allocation fails.
int sparse_adam(int n_groups, const gsr_adam_group *groups, int64_t P, const float *relevance, double beta1,
                double beta2, double eps, int *flag_scratch, bool flag_ready, hipStream_t s, float *shrink_raw,
                int64_t shrink_first, float shrink_limit, const float *live3 = nullptr, int64_t skybox = 0,
                int *row_list = nullptr);
// SSIM map forward (+ masked inverse-depth L1 forward with its gradient for an upstream of 1 when
// mono != NULL) and the loss epilogue: losses[0..2] photometric, [3..4] depth, [5] total; *flag = 0.
// one != NULL: gmap receives the photometric gradient itself (dL/dloss = *one, times alpha when
// given), and *gmap_is_photo says so (the streaming SSIM kernel; the tile kernel writes G)
int step_loss_forward(const float *img, const float *gt, int H, int W, double lambda_dssim, void *loss_scratch,
                      float *gmap, const float *invd, const float *mono, const float *mask, float depth_w,
                      void *depth_scratch, float *d_invd, float *losses, int *flag, hipStream_t s,
                      const float *one = nullptr, const float *alpha = nullptr, bool *gmap_is_photo = nullptr);
// the depth-only view's loss (gsr_depth_only_loss) with its gradient for an upstream of 1 in d_invd;
// losses = (dens, 0, 0, pure, loss, loss); *flag = 0
int step_depth_only_forward(const float *invd, const float *mono, const float *mask, int64_t n, float w, double a,
                            void *depth_scratch, float *d_invd, float *losses, int *flag, hipStream_t s);
int launch_exposure_forward(const float *color, const float *E, int64_t npix, float *out, const float *alpha,
                            hipStream_t s);
// photometric gradient (x alpha) through the exposure into d_color, the exposure gradient and the
// exposure optimizer's dense Adam step
int step_loss_backward(const float *img, const float *gt, const float *gmap, const float *one, double lambda_dssim,
                       const float *alpha, const float *color, const float *E_view, int64_t npix, float *d_color,
                       void *exp_scratch, int n_images, int view, const gsr_adam_group &eg, float *exposure_grad,
                       double b1, double b2, double eps, hipStream_t s, bool gmap_is_photo = false);
// activation backward + skybox lock + relevance flag + densification statistics.  sparse_rows:
// the rasterizer backward wrote sparse rows (GaussianGrads): the scale / rotation gradients of
// rows it did not write are neither read nor written.
// scales / opac NULL: recomputed from the raw parameters (scaling_raw, opacity_raw) -- the raw mode
int step_activate_backward(int64_t P, const float *rotation_raw, const float *scales, const float *opac,
                           const float *d_scales, const float *d_rots, const float *d_opac, float *scaling_grad,
                           float *rotation_grad, float *opacity_grad, int64_t skybox, int *flag, const int *radii,
                           const float *d_means2D, float *max_radii2D, float *accum, float *denom, hipStream_t s,
                           bool sparse_rows = false, const float *scaling_raw = nullptr,
                           const float *opacity_raw = nullptr);

// kernel stamps of each translation unit (GSR_KSTAMP builds; gsr_kstamp_read)
int kstamp_read_preprocess(unsigned long long *out);
int kstamp_read_dsort(unsigned long long *out);
int kstamp_read_binning(unsigned long long *out);
int kstamp_read_render(unsigned long long *out);
int kstamp_read_backward(unsigned long long *out);

}  // namespace gsr
