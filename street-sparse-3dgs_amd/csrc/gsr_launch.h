// gsr_launch.h -- host-side launchers for the gfx950 kernels (one translation unit each).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "gsr_device.h"

namespace gsr {

// rasterizer.hip: message returned by gsr_last_error() for the calling thread.
void set_last_error(const std::string &msg);

struct Camera {
    const float *view;  // device, 16
    const float *proj;  // device, 16
    const float *campos;  // device, 3
    float tanx, tany, fx, fy;
    int W, H, gx, gy;
};

struct GaussianInputs {
    int P, D, M;
    const float *means3D, *shs, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp;
    float scale_modifier;
};

// preprocess.hip
void launch_preprocess(const GaussianInputs &in, const Camera &cam, const GeomState &gs, int *radii,
                       hipStream_t s, bool split_color);
// SH colour of the visible Gaussians (rec.col, clamped) after a split_color preprocess
bool color_split_supported(const GaussianInputs &in);
void launch_preprocess_color(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const int *radii,
                             hipStream_t s);
// render.hip: tiles ordered heaviest first by work[t] (or, with work == NULL, by list length).
void launch_tile_order(const uint32_t *work, const uint2 *ranges, int T, int shift, uint32_t *order, hipStream_t s);
void launch_mark_visible(int P, const float *means3D, const float *view, uint8_t *present, hipStream_t s);

// sort.hip (rocPRIM)
size_t scan_temp_bytes(int P);
hipError_t inclusive_scan(void *tmp, size_t tmp_bytes, const uint32_t *in, uint32_t *out, int P, hipStream_t s);
// Stable LSD sort of n (key, value) pairs over key bits [0, end_bit) (kNN Morton order).
size_t sort_pairs_temp_bytes(size_t n, int end_bit);
hipError_t sort_pairs(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                      uint32_t *vout, size_t n, int end_bit, hipStream_t s);
size_t depth_sort_temp_bytes(int P);
hipError_t depth_sort(void *tmp, size_t tmp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                      uint32_t *vout, int P, hipStream_t s);
// binning.hip: per-tile lists from the depth-ordered Gaussians (two stable counting levels).
SBGrid sb_grid(int gx, int gy, int P);
// Depth-ordered copies of each Gaussian's tile rect and tile count (one gather pass after the sort).
void launch_depth_gather(int P, const GeomState &gs, hipStream_t s);
bool sb_grid_supported(const SBGrid &g);
void launch_binning_superblocks(int P, const Camera &cam, const GeomState &gs, const BinningState &bs,
                                const ImageState &is, hipStream_t s);
void launch_binning_tiles(int P, const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                          hipStream_t s);

// render.hip
void launch_render_fwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const float *bg, float *out_color, float *out_invdepth, hipStream_t s);
void launch_render_bwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const int *radii, const float *bg, const float *dL_dpix, const float *dL_dinvdepth,
                       const BwdScratch &sc, hipStream_t s);

// backward.hip
struct GaussianGrads {
    float *dmeans2D, *dcolors, *dopacity, *dmeans3D, *dcov3D, *dsh, *dscales, *drots;
};
void launch_preprocess_bwd(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const ImageState &is,
                           const int *radii, const BwdScratch &sc, const GaussianGrads &out, hipStream_t s);

}  // namespace gsr
