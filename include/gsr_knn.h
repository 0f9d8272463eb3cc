/*
 * gsr_knn.h -- C ABI of the nearest-neighbour scale initialisation.
 * Exported by libgsr_hip.so.
 *
 *   gsr_knn_mean_dist2  replaces simple_knn._C.distCUDA2 (submodules/simple-knn, not vendored
 *                       in the reference), called at scene/gaussian_model.py:207:
 *                         dist2 = torch.clamp_min(distCUDA2(points), 0.0000001)
 *                         scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
 *                       out[i] = (d0 + d1 + d2) / 3 with d0 <= d1 <= d2 the three smallest
 *                       squared distances from point i to the points j != i (by index: duplicate
 *                       positions count as distance 0), summed left to right in fp32; missing
 *                       neighbours (N < 4) are FLT_MAX, as upstream's initial best list.
 *                       Squared distance order: fma(dz, dz, fma(dy, dy, dx * dx)), d = p_j - p_i.
 *
 * Conventions as in gsr.h: device pointers, fp32, `stream` a hipStream_t.
 */
#ifndef GSR_KNN_H
#define GSR_KNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes of device scratch gsr_knn_mean_dist2 needs for N points. */
size_t gsr_knn_scratch_bytes(int64_t N);

/* points: (N, 3) contiguous fp32; out: (N) fp32.  Exact (conservative box pruning). */
int gsr_knn_mean_dist2(int64_t N, const float *points, float *out, void *scratch, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GSR_KNN_H */
