// train_step.hip -- the native train-step executor (include/gsr_train.h gsr_train_step): one host
// call runs a whole Street-sparse iteration (train_single.py:65-247, as gs_train/harness.py
// TrainStep.step drives it from Python) with the arithmetic of the same entry points, in the same
// order:
//
//   activations -> rasterizer forward -> exposure (x alpha mask) -> photometric loss with the SSIM
//   gradient field, masked inverse-depth L1 with its gradient -> loss epilogue -> photometric
//   gradient through the exposure, exposure gradient + exposure Adam -> rasterizer backward ->
//   activation backward + skybox lock + relevance flag + densification statistics -> sparse
//   Adam -> scale shrink
//
// Knowing the whole step lets it fuse what the autograd graph keeps apart: the depth gradient is
// formed in the depth loss's pass (the upstream is 1), the photometric gradient inside the
// exposure backward (no (3, H, W) image gradient is written and re-read), the exposure Adam in the
// exposure gradient's reduction, the skybox lock / relevance test / densification statistics in
// the activation backward: 11 fewer launches and ~50 MB less traffic than the Python step, with
// identical results (bit for bit with the deterministic backward; tests/test_gpu_train.py).
// Every per-step intermediate lives in grow-only device buffers owned by the context and reused
// across steps (no allocation in steady state).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_train.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

enum Slot {
    kGeom, kBinning, kImage, kBwdScratch,                                  // rasterizer buffers
    kColor, kInvDepth, kExposed, kGradMap, kDColor, kDInvDepth,            // image-sized
    kScales, kRots, kOpac, kDScales, kDRots, kDOpac, kDMeans2D, kRadii,    // per-Gaussian
    kLossScratch, kExpScratch, kDepthScratch, kWords,                      // small
    kAdamList,                                                             // sparse Adam's row list
    kSlots
};


}  // namespace
}  // namespace gsr

using namespace gsr;

struct gsr_train_ctx {
    struct Buf {
        void *p = nullptr;
        size_t cap = 0;
    } buf[kSlots];
    hipStream_t stream = nullptr;
    bool failed_alloc = false;
    bool one_written = false;
    int64_t growths = 0;  // gsr_train_ctx_stats
    // Stream-ordered growth (hipFreeAsync / hipMallocFromPoolAsync from the context's own memory pool,
    // which keeps what is freed): a training loop whose P and K grow over its densification events
    // re-sizes its buffers without a host wait -- the synchronous form (GSR_STEP_SYNC_ALLOC=1: wait for
    // the stream, hipFree, hipMalloc) stalls the host at every growth and hipMalloc of a large block
    // maps its pages.  The pool is the context's, not the device's default pool, so other
    // stream-ordered users in the process keep the default pool's release behaviour.
    const bool async_alloc = [] {
        const char *e = std::getenv("GSR_STEP_SYNC_ALLOC");
        return !(e && e[0] == '1');
    }();
    bool pool_ready = false;
    hipMemPool_t pool = nullptr;

    void pool_setup() {
        if (pool_ready) return;
        pool_ready = true;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return;
        hipMemPoolProps props;
        std::memset(&props, 0, sizeof(props));
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
            pool = nullptr;  // hipMallocAsync from the default pool, with its own release threshold
            (void)hipGetLastError();
            return;
        }
        uint64_t keep = UINT64_MAX;  // freed blocks stay in this pool for the next growth
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }

    // grow-only, 1/4 more than asked (rasterizer buffers follow K)
    void *get(int slot, size_t bytes) {
        Buf &b = buf[slot];
        if (bytes <= b.cap && b.p) return b.p;
        growths++;
        const size_t want = std::max<size_t>(256, bytes + bytes / 4);
        if (async_alloc) {
            pool_setup();
            // in stream order: work queued before (and the side streams joined into it) still reads the
            // old block; everything after uses the new one
            if (b.p) (void)hipFreeAsync(b.p, stream);
            b.p = nullptr;
            b.cap = 0;
            const hipError_t e = pool ? hipMallocFromPoolAsync(&b.p, want, pool, stream)
                                      : hipMallocAsync(&b.p, want, stream);
            if (e != hipSuccess) {
                b.p = nullptr;
                failed_alloc = true;
                return nullptr;
            }
            b.cap = want;
            return b.p;
        }
        if (b.p) {  // queued kernels may still use the old allocation
            if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
            (void)hipFree(b.p);
            b.p = nullptr;
            b.cap = 0;
        }
        if (hipMalloc(&b.p, want) != hipSuccess) {
            b.p = nullptr;
            failed_alloc = true;
            return nullptr;
        }
        b.cap = want;
        return b.p;
    }
    int64_t held() const {
        int64_t n = 0;
        for (const auto &b : buf) n += (int64_t)b.cap;
        return n;
    }
    float *f32(int slot, size_t n) { return static_cast<float *>(get(slot, n * sizeof(float))); }

    ~gsr_train_ctx() {
        if (async_alloc) {
            for (auto &b : buf)
                if (b.p) (void)hipFreeAsync(b.p, stream);
            (void)hipStreamSynchronize(stream);
            if (pool) (void)hipMemPoolDestroy(pool);
        } else {
            for (auto &b : buf)
                if (b.p) (void)hipFree(b.p);
        }
    }
};

namespace {

void *buf_ptr(gsr_train_ctx *c, int slot) { return c->buf[slot].p; }
void *resize_geom(void *c, size_t n) { return static_cast<gsr_train_ctx *>(c)->get(kGeom, n); }
void *resize_binning(void *c, size_t n) { return static_cast<gsr_train_ctx *>(c)->get(kBinning, n); }
void *resize_image(void *c, size_t n) { return static_cast<gsr_train_ctx *>(c)->get(kImage, n); }
void *resize_scratch(void *c, size_t n) { return static_cast<gsr_train_ctx *>(c)->get(kBwdScratch, n); }

int fail_step(int rc, const char *what) {
    if (rc == GSR_OK) return rc;
    set_last_error(std::string("gsr_train_step: ") + what + ": " + gsr_last_error());
    return rc;
}

// GSR_STEP_ACTIVATIONS=1: activations written by their own launch and read by the rasterizer (the
// Python-driven step's form); default: the rasterizer and the activation backward read the raw
// parameters and activate them where they are used (GaussianInputs.raw)
#ifndef GSR_STEP_FUSE_ACT
#define GSR_STEP_FUSE_ACT 1
#endif
#ifndef GSR_STEP_PHOTO_IN_SSIM
#define GSR_STEP_PHOTO_IN_SSIM 1  // 0: the SSIM pass writes G and the exposure backward forms the gradient
#endif

bool step_raw_params() {
    const char *e = std::getenv("GSR_STEP_ACTIVATIONS");
    return !(e != nullptr && e[0] == '1');
}

bool step_sparse_rows() {
    const char *e = std::getenv("GSR_STEP_DENSE_ROWS");  // read per call: A/B runs switch it
    return !(e != nullptr && e[0] == '1');
}

int invalid(const char *msg) {
    set_last_error(std::string("gsr_train_step: ") + msg);
    return GSR_ERR_INVALID_ARGUMENT;
}

}  // namespace

extern "C" {

gsr_train_ctx *gsr_train_ctx_create(void) { return new (std::nothrow) gsr_train_ctx(); }

int gsr_train_ctx_stats(const gsr_train_ctx *ctx, int64_t *out, int n) {
    if (!ctx || !out || n < 0) return invalid("NULL context or stats buffer");
    const int64_t v[3] = {ctx->growths, ctx->held(), ctx->async_alloc ? 1 : 0};
    int k = 0;
    for (; k < n && k < 3; k++) out[k] = v[k];
    return k;
}

void gsr_train_ctx_destroy(gsr_train_ctx *ctx) {
    if (!ctx) return;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    delete ctx;
}

int gsr_train_step(gsr_train_ctx *ctx, const gsr_train_step_args *a, int64_t *num_rendered) {
    if (num_rendered) *num_rendered = 0;
    if (!ctx || !a) return invalid("NULL context or arguments");
    const int64_t P = a->P;
    const int W = a->width, H = a->height;
    if (P <= 0 || P > 0x7fffffff || W <= 0 || H <= 0 || a->M <= 0 || a->D < 0 || (a->D + 1) * (a->D + 1) > a->M)
        return invalid("bad sizes");
    if (!a->xyz || !a->features || !a->opacity || !a->scaling || !a->rotation || !a->xyz_grad ||
        !a->features_grad || !a->opacity_grad || !a->scaling_grad || !a->rotation_grad)
        return invalid("NULL parameter or gradient");
    if (!a->exposure || !a->exposure_grad || a->n_images <= 0 || a->image_index < 0 || a->image_index >= a->n_images)
        return invalid("bad exposure arguments");
    const bool depth_only = a->depth_only != 0;
    if (!a->viewmatrix || !a->projmatrix || !a->campos || !a->background || (!a->gt && !depth_only) || !a->losses)
        return invalid("NULL camera, background, target or loss output");
    if (depth_only && (!a->mono_invdepth || !(a->depth_weight > 0.f)))
        return invalid("a depth-only view needs its inverse-depth map and a positive depth weight "
                       "(train_single.py:158-161 has no loss otherwise)");
    if (depth_only && !(a->depth_dens_weight >= 0.0 && a->depth_dens_weight <= 1.0))
        return invalid("depth_dens_weight outside [0, 1]");
    if (!a->max_radii2D || !a->xyz_gradient_accum || !a->denom) return invalid("NULL densification statistics");
    if (a->n_groups <= 0 || !a->groups || !a->exposure_group) return invalid("no optimizer groups");
    if (a->skybox_rows < 0 || a->skybox_rows > P || a->scaffold_rows < 0)
        return invalid("skybox / scaffold rows outside [0, P]");
    if (!(a->lambda_dssim >= 0.0 && a->lambda_dssim <= 1.0)) return invalid("lambda_dssim outside [0, 1]");

    hipStream_t s = static_cast<hipStream_t>(a->stream);
    // the grow-only buffers are freed after a wait on ctx->stream only: a caller that switches
    // streams first drains the previous one, whose queued kernels may still use them
    if (ctx->stream != s) {
        if (ctx->stream && hipStreamSynchronize(ctx->stream) != hipSuccess)
            return fail_step(GSR_ERR_DEVICE, "previous stream");
        ctx->stream = s;
    }
    void *sv = a->stream;
    const int64_t npix = (int64_t)W * H;
    const bool depth = a->mono_invdepth != nullptr && a->depth_weight > 0.f;

    float *scales = ctx->f32(kScales, 3 * P), *rots = ctx->f32(kRots, 4 * P), *opac = ctx->f32(kOpac, P);
    float *d_scales = ctx->f32(kDScales, 3 * P), *d_rots = ctx->f32(kDRots, 4 * P), *d_opac = ctx->f32(kDOpac, P);
    float *d_means2D = ctx->f32(kDMeans2D, 3 * P);
    int *radii = static_cast<int *>(ctx->get(kRadii, sizeof(int) * P));
    float *color = ctx->f32(kColor, 3 * npix), *invd = ctx->f32(kInvDepth, npix);
    float *image = ctx->f32(kExposed, 3 * npix), *gmap = ctx->f32(kGradMap, 3 * npix);
    float *d_color = ctx->f32(kDColor, 3 * npix);
    float *d_invd = ctx->f32(kDInvDepth, npix);
    void *loss_scratch = ctx->get(kLossScratch, gsr_l1_ssim_scratch_bytes(3, H, W));
    void *exp_scratch = ctx->get(kExpScratch, gsr_exposure_scratch_bytes(npix));
    void *depth_scratch =
        ctx->get(kDepthScratch, std::max(gsr_depth_l1_scratch_bytes(npix), gsr_depth_only_scratch_bytes(npix)));
    // words: [0] the Adam relevance flag, [1] dL/dloss = 1 (the upstream of loss.backward())
    void *words = ctx->get(kWords, 64);
    // the sparse Adam's compacted row list (grow-only; without it the row-block kernel runs)
    int *adam_list = static_cast<int *>(ctx->get(kAdamList, sizeof(int) * ((size_t)P + 64)));
    if (ctx->failed_alloc || !scales || !rots || !opac || !d_scales || !d_rots || !d_opac || !d_means2D || !radii ||
        !color || !invd || !image || !gmap || !d_color || !d_invd || !loss_scratch || !exp_scratch ||
        !depth_scratch || !words) {
        ctx->failed_alloc = false;
        set_last_error("gsr_train_step: device allocation failed");
        return GSR_ERR_ALLOCATION;
    }
    int *flag = static_cast<int *>(words);
    float *one = static_cast<float *>(words) + 1;
    if (!ctx->one_written) {  // once per context (the words slot is never re-allocated: 64 B)
        const uint32_t w[4] = {0u, 0x3f800000u /* 1.0f */, 0u, 0u};
        if (hipMemcpy(words, w, sizeof(w), hipMemcpyHostToDevice) != hipSuccess)
            return fail_step(GSR_ERR_DEVICE, "step words");
        ctx->one_written = true;
    }
    int rc;

    // render(): activations, rasterizer, exposure of this view (harness.py TrainStep.render).  Raw
    // mode: the preprocess activates the parameters it reads (no activated copy written and re-read)
    const bool raw = step_raw_params();
    if (!raw && (rc = gsr_activate_forward(P, a->scaling, a->rotation, a->opacity, scales, rots, opac, sv)))
        return fail_step(rc, "activations");
    const float *r_scales = raw ? a->scaling : scales, *r_rots = raw ? a->rotation : rots,
                *r_opac = raw ? a->opacity : opac;
    int64_t K = 0;
    set_raw_params(raw);
    rc = gsr_rasterize_forward_ex(resize_geom, resize_binning, resize_image, ctx, (int)P, a->D, a->M, a->background,
                                  W, H, a->xyz, a->features, nullptr, r_opac, r_scales, 1.0f, r_rots, nullptr,
                                  a->viewmatrix, a->projmatrix, a->campos, a->tan_fovx, a->tan_fovy, 0, color, invd,
                                  radii, nullptr, nullptr, nullptr, nullptr, 0, 0, sv, &K, 0);
    set_raw_params(false);
    if (rc) return fail_step(rc, "rasterizer forward");
    const float *E = a->exposure + 12 * (int64_t)a->image_index;
    if (depth_only) {
        // a depth-only view (train_single.py:145-161): the rendered image is in no loss, so the
        // exposure pass, the SSIM pass and the exposure step (:213-214) do not run; the colour
        // gradient is zero and the exposure gradient is zeroed (:203-209)
        if ((rc = step_depth_only_forward(invd, a->mono_invdepth, a->depth_mask, npix, a->depth_weight,
                                          a->depth_dens_weight, depth_scratch, d_invd, a->losses, flag, s)))
            return fail_step(rc, "depth-only loss");
        if (hipMemsetAsync(d_color, 0, sizeof(float) * 3 * npix, s) != hipSuccess ||
            hipMemsetAsync(a->exposure_grad, 0, sizeof(float) * 12 * (size_t)a->n_images, s) != hipSuccess)
            return fail_step(GSR_ERR_DEVICE, "depth-only zero gradients");
    } else {
        // exposure (x the alpha mask, train_single.py:117-119, in the same pass)
        if ((rc = launch_exposure_forward(color, E, npix, image, a->alpha_mask, s)))
            return fail_step(rc, "exposure");

        // losses (train_single.py:121-141): the SSIM map pass with its gradient field, the depth L1
        // with its gradient (the loss is the root: dL/dloss = 1), one epilogue for both values and
        // the total
        bool photo = false;  // the SSIM pass wrote the photometric gradient itself (gsr_launch.h)
        if ((rc = step_loss_forward(image, a->gt, H, W, a->lambda_dssim, loss_scratch, gmap, invd,
                                    depth ? a->mono_invdepth : nullptr, a->depth_mask, a->depth_weight,
                                    depth_scratch, d_invd, a->losses, flag, s, GSR_STEP_PHOTO_IN_SSIM ? one : nullptr,
                                    a->alpha_mask, &photo)))
            return fail_step(rc, "losses");

        // loss.backward(): photometric gradient -> alpha mask -> exposure (colour gradient, exposure
        // gradient and the exposure optimizer's step in the same two launches)
        gsr_adam_group eg = *a->exposure_group;
        if ((rc = step_loss_backward(image, a->gt, gmap, one, a->lambda_dssim, a->alpha_mask, color, E, npix, d_color,
                                     exp_scratch, a->n_images, a->image_index, eg, a->exposure_grad,
                                     a->exposure_beta1, a->exposure_beta2, a->exposure_eps, s, photo)))
            return fail_step(rc, "loss backward");
    }
    // sparse gradient rows (gsr_launch.h GaussianGrads): the Gaussians no pixel's backward reached
    // (88% of the bench scene) have zero gradients and are never relevant to the sparse Adam, so
    // their 232 B of gradient rows are not written (GSR_STEP_DENSE_ROWS=1: every row, as the
    // Python-driven step)
    const bool sparse_rows = step_sparse_rows();
    // the activation backward (skybox lock, relevance flag, densification statistics:
    // train_single.py:193-194, 217-223) fused into the rasterizer backward's live-row pass, which
    // then writes the raw parameters' gradients itself (gsr_launch.h StepAct); the conditions
    // mirror backward.hip's split path (GSR_STEP_FUSE_ACT=0: the separate activation backward)
    const bool fuse_act = GSR_STEP_FUSE_ACT && raw && sparse_rows && a->M == 16 &&
                          (reinterpret_cast<uintptr_t>(a->features) & 15u) == 0 &&
                          (reinterpret_cast<uintptr_t>(a->features_grad) & 15u) == 0;
    const StepAct act{a->scaling, a->opacity, reinterpret_cast<const float4 *>(a->rotation), a->skybox_rows, radii,
                      a->max_radii2D, a->xyz_gradient_accum, a->denom, flag, 1};
    set_sparse_grad_rows(sparse_rows);
    set_raw_params(raw);
    set_step_act(fuse_act ? &act : nullptr);
    rc = gsr_rasterize_backward(resize_scratch, ctx, (int)P, a->D, a->M, K, a->background, W, H, a->xyz,
                                     a->features, nullptr, r_scales, 1.0f, r_rots, nullptr, a->viewmatrix, a->projmatrix,
                                     a->campos, a->tan_fovx, a->tan_fovy, radii, buf_ptr(ctx, kGeom),
                                     buf_ptr(ctx, kBinning), buf_ptr(ctx, kImage), d_color, depth ? d_invd : nullptr,
                                     d_means2D, nullptr, fuse_act ? a->opacity_grad : d_opac, a->xyz_grad, nullptr,
                                     a->features_grad, fuse_act ? a->scaling_grad : d_scales,
                                     fuse_act ? a->rotation_grad : d_rots, nullptr, nullptr, nullptr, nullptr, 0, 0, sv);
    set_sparse_grad_rows(false);
    set_raw_params(false);
    set_step_act(nullptr);
    if (rc) return fail_step(rc, "rasterizer backward");
    if (fuse_act != step_act_done())
        return invalid("the rasterizer backward did not take the fused activation backward it was given");
    // otherwise the activation backward on its own; then the sparse Adam and the shrink (:225-241)
    if (!fuse_act &&
        (rc = step_activate_backward(P, a->rotation, raw ? nullptr : scales, raw ? nullptr : opac, d_scales, d_rots,
                                     d_opac, a->scaling_grad, a->rotation_grad, a->opacity_grad, a->skybox_rows, flag,
                                     radii, d_means2D, a->max_radii2D, a->xyz_gradient_accum, a->denom, s, sparse_rows,
                                     a->scaling, a->opacity)))
        return fail_step(rc, "activation backward");
    if (!a->skip_gaussian_step &&
        (rc = sparse_adam(a->n_groups, a->groups, P, a->opacity_grad, a->beta1, a->beta2, a->eps, flag, true, s,
                          a->scaling, a->scaffold_rows, a->max_scale, sparse_rows ? d_means2D : nullptr,
                          a->skybox_rows, adam_list)))
        return fail_step(rc, "sparse Adam + shrink");
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_train_step: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    if (num_rendered) *num_rendered = K;
    return GSR_OK;
}

}  // extern "C"
