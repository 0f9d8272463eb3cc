// backward.hip -- per-Gaussian backward: sums the Gaussian's
// per-tile-instance records written by render_bwd (one contiguous run per Gaussian, at its
// exclusive-scan offset), then chains conic -> 2D covariance -> (3D covariance, mean) with the
// EWA Jacobian, screen-space mean -> mean3D through projmatrix, inverse depth -> mean3D,
// SH -> (coefficients, view direction -> mean3D) and 3D covariance -> (scale, rotation).
// Every output row is written (zeros for culled Gaussians and unused SH coefficients), so
// the caller's gradient tensors need no memset pass.
#include <algorithm>
#include <atomic>

#include "gsr_launch.h"

namespace gsr {

#ifndef GSR_RED_SERIAL
#define GSR_RED_SERIAL 32
#endif
constexpr uint32_t kRedSerial = GSR_RED_SERIAL;  // splats up to this many tiles: summed by their own lane
#ifndef GSR_REC_BATCH
#define GSR_REC_BATCH 4
#endif
#ifndef GSR_LIVE_UNROLL
#define GSR_LIVE_UNROLL 8
#endif
#ifndef GSR_BIG_BLOCK
#define GSR_BIG_BLOCK 2
#endif
constexpr int kRecBatch = GSR_REC_BATCH;  // live records loaded together per Gaussian (record_sum)

// SH backward for degree D: rgb_ch = sum_k B_k(dir) sh[k][ch] (+0.5, clamp handled by the caller
// zeroing gc).  dL/dsh[k][ch] = B_k gc[ch];  dL/ddir = sum_k dB_k/ddir * (sum_ch sh[k][ch] gc[ch]).
// The basis and its gradient are evaluated once and shared by the three channels; with M = 16
// the 192-B coefficient row is read and the gradient row written as 12 float4s.
template <int D, bool kRow = false>
__device__ __forceinline__ void sh_backward(const float *__restrict__ sh, int M, bool vec, const float dir[3],
                                            const float gc[3], float *__restrict__ dsh, float gd[3]) {
    // kRow: `sh` / `dsh` are this lane's 12-float4 rows of the wave's LDS tile (staged reads,
    // staged coalesced writes; see preprocess_bwd_kernel)
    constexpr int NC = (D + 1) * (D + 1);
    const float x = dir[0], y = dir[1], z = dir[2];
    float B[16], Bx[16], By[16], Bz[16];
#pragma unroll
    for (int k = 0; k < 16; k++) B[k] = Bx[k] = By[k] = Bz[k] = 0.f;
    B[0] = GSR_SH_C0;
    if (D > 0) {
        B[1] = -GSR_SH_C1 * y; By[1] = -GSR_SH_C1;
        B[2] = GSR_SH_C1 * z;  Bz[2] = GSR_SH_C1;
        B[3] = -GSR_SH_C1 * x; Bx[3] = -GSR_SH_C1;
    }
    if (D > 1) {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        B[4] = GSR_SH_C2_0 * xy; Bx[4] = GSR_SH_C2_0 * y; By[4] = GSR_SH_C2_0 * x;
        B[5] = GSR_SH_C2_1 * yz; By[5] = GSR_SH_C2_1 * z; Bz[5] = GSR_SH_C2_1 * y;
        B[6] = GSR_SH_C2_2 * (2.f * zz - xx - yy);
        Bx[6] = GSR_SH_C2_2 * 2.f * -x; By[6] = GSR_SH_C2_2 * 2.f * -y; Bz[6] = GSR_SH_C2_2 * 2.f * 2.f * z;
        B[7] = GSR_SH_C2_3 * xz; Bx[7] = GSR_SH_C2_3 * z; Bz[7] = GSR_SH_C2_3 * x;
        B[8] = GSR_SH_C2_4 * (xx - yy); Bx[8] = GSR_SH_C2_4 * 2.f * x; By[8] = GSR_SH_C2_4 * 2.f * -y;
        if (D > 2) {
            B[9] = GSR_SH_C3_0 * y * (3.f * xx - yy);
            Bx[9] = GSR_SH_C3_0 * 3.f * 2.f * xy; By[9] = GSR_SH_C3_0 * 3.f * (xx - yy);
            B[10] = GSR_SH_C3_1 * xy * z;
            Bx[10] = GSR_SH_C3_1 * yz; By[10] = GSR_SH_C3_1 * xz; Bz[10] = GSR_SH_C3_1 * xy;
            B[11] = GSR_SH_C3_2 * y * (4.f * zz - xx - yy);
            Bx[11] = GSR_SH_C3_2 * -2.f * xy; By[11] = GSR_SH_C3_2 * (-3.f * yy + 4.f * zz - xx);
            Bz[11] = GSR_SH_C3_2 * 4.f * 2.f * yz;
            B[12] = GSR_SH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy);
            Bx[12] = GSR_SH_C3_3 * -3.f * 2.f * xz; By[12] = GSR_SH_C3_3 * -3.f * 2.f * yz;
            Bz[12] = GSR_SH_C3_3 * 3.f * (2.f * zz - xx - yy);
            B[13] = GSR_SH_C3_4 * x * (4.f * zz - xx - yy);
            Bx[13] = GSR_SH_C3_4 * (-3.f * xx + 4.f * zz - yy); By[13] = GSR_SH_C3_4 * -2.f * xy;
            Bz[13] = GSR_SH_C3_4 * 4.f * 2.f * xz;
            B[14] = GSR_SH_C3_5 * z * (xx - yy);
            Bx[14] = GSR_SH_C3_5 * 2.f * xz; By[14] = GSR_SH_C3_5 * -2.f * yz; Bz[14] = GSR_SH_C3_5 * (xx - yy);
            B[15] = GSR_SH_C3_6 * x * (xx - 3.f * yy);
            Bx[15] = GSR_SH_C3_6 * 3.f * (xx - yy); By[15] = GSR_SH_C3_6 * -3.f * 2.f * xy;
        }
    }
    float c[48];
    if (kRow || vec) {
        const float4 *s4 = reinterpret_cast<const float4 *>(sh);
#pragma unroll
        for (int q = 0; q < 12; q++) {
            if (4 * q < NC * 3) {
                const float4 v = s4[q];
                c[4 * q] = v.x; c[4 * q + 1] = v.y; c[4 * q + 2] = v.z; c[4 * q + 3] = v.w;
            } else {
                c[4 * q] = c[4 * q + 1] = c[4 * q + 2] = c[4 * q + 3] = 0.f;
            }
        }
    } else {
#pragma unroll
        for (int e = 0; e < 48; e++) c[e] = e < NC * 3 ? sh[e] : 0.f;
    }
    gd[0] = gd[1] = gd[2] = 0.f;
#pragma unroll
    for (int k = 1; k < NC; k++) {
        const float vk = c[3 * k] * gc[0] + c[3 * k + 1] * gc[1] + c[3 * k + 2] * gc[2];
        gd[0] = fmaf(Bx[k], vk, gd[0]);
        gd[1] = fmaf(By[k], vk, gd[1]);
        gd[2] = fmaf(Bz[k], vk, gd[2]);
    }
    if (kRow || vec) {
        float4 *d4 = reinterpret_cast<float4 *>(dsh);
#pragma unroll
        for (int q = 0; q < 12; q++) {
            float e4[4];
#pragma unroll
            for (int t = 0; t < 4; t++) {
                const int e = 4 * q + t;
                e4[t] = e < NC * 3 ? B[e / 3] * gc[e % 3] : 0.f;
            }
            d4[q] = make_float4(e4[0], e4[1], e4[2], e4[3]);
        }
    } else {
        for (int e = 0; e < M * 3; e++) dsh[e] = 0.f;
#pragma unroll
        for (int e = 0; e < NC * 3; e++) dsh[e] = B[e / 3] * gc[e % 3];
    }
}


// Per-Gaussian sum of its per-tile records (contiguous at its exclusive-scan offset).  A record
// exists only for tiles where this Gaussian sits in front of the tile's boundary (the last list
// entry any pixel used, render.hip); elsewhere the instance contributed nothing.  The liveness of
// all (<= kRedSerial) tiles is gathered first so the boundary loads and then the record loads are
// issued back to back; larger splats are summed by the whole wave (coalesced loads + DPP).  Kept
// apart from the chain rule below: this half is memory-latency bound and wants occupancy
// (few VGPRs), the other half is arithmetic with ~130 VGPRs.
// The splat's tile rect comes from the compact per-Gaussian rect array (4 or 8 B; an empty rect marks
// a culled Gaussian) and its depth bits are recomputed from the mean exactly as the preprocess
// forms them -- reading them from the GRec line fetched a whole 64-B line per Gaussian.
__global__ __launch_bounds__(256) void record_sum_kernel(int P, int gx, const float *__restrict__ means3D,
                                                         const float *__restrict__ viewmatrix,
                                                         const uint2 *__restrict__ rect8,
                                                         const uint32_t *__restrict__ rect4,
                                                         const uint32_t *__restrict__ offsets,
                                                         const uint64_t *__restrict__ boundary, BwdScratch sc,
                                                         float *__restrict__ dmeans2D, float *__restrict__ dopacity) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1);
    const bool valid = i < P;
    const uint2 rr = !valid ? make_uint2(0u, 0u) : rect4 ? unpack_rect4(rect4[i]) : rect8[i];
    const bool vis = rr.y != 0u;  // x1 | y1 << 16 with x1 > x0 >= 0: zero only when culled
    float g[10];
#pragma unroll
    for (int k = 0; k < 10; k++) g[k] = 0.f;
    uint32_t n = 0, x0 = 0, y0 = 0, w = 1, off = 0;
    uint64_t key = 0;
    if (vis) {
        x0 = rr.x & 0xFFFFu;
        y0 = rr.x >> 16;
        w = (rr.y & 0xFFFFu) - x0;
        n = w * ((rr.y >> 16) - y0);
        const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
        const float z = xf_point43(p, load_mat4(viewmatrix)).z;
        key = ((uint64_t)__float_as_uint(z) << 32) | (uint32_t)i;
        off = offsets[i];
    }
    auto accumulate = [&](float *acc, uint32_t u) {
        const float4 a = sc.rec[4 * (size_t)u + 0];
        const float4 b = sc.rec[4 * (size_t)u + 1];
        const float4 c = sc.rec[4 * (size_t)u + 2];
        acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
        acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
        acc[8] += c.x; acc[9] += c.y;
    };
    if (n <= kRedSerial && n > 0) {
        uint32_t live = 0, x = x0, y = y0;
        const uint32_t xe = x0 + w;
#pragma unroll GSR_LIVE_UNROLL
        for (uint32_t k = 0; k < n; k++) {
            const uint64_t bk = boundary[y * (uint32_t)gx + x];
            live |= (uint32_t)(bk != 0 && key <= bk) << k;
            if (++x == xe) {
                x = x0;
                ++y;
            }
        }
        // live records kRecBatch at a time: all their loads in flight before the adds
        while (live) {
            uint32_t ks[kRecBatch];
            bool has[kRecBatch];
#pragma unroll
            for (int q = 0; q < kRecBatch; q++) {
                has[q] = live != 0u;
                ks[q] = has[q] ? (uint32_t)__ffs(live) - 1u : 0u;
                live &= live - 1u;
            }
            float4 ra[kRecBatch], rb[kRecBatch], rc[kRecBatch];
#pragma unroll
            for (int q = 0; q < kRecBatch; q++) {
                const size_t u = 4 * (size_t)(off + ks[q]);
                ra[q] = has[q] ? sc.rec[u + 0] : make_float4(0.f, 0.f, 0.f, 0.f);
                rb[q] = has[q] ? sc.rec[u + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
                rc[q] = has[q] ? sc.rec[u + 2] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int q = 0; q < kRecBatch; q++) {
                g[0] += ra[q].x; g[1] += ra[q].y; g[2] += ra[q].z; g[3] += ra[q].w;
                g[4] += rb[q].x; g[5] += rb[q].y; g[6] += rb[q].z; g[7] += rb[q].w;
                g[8] += rc[q].x; g[9] += rc[q].y;
            }
        }
    }
    // Splats over more than kRedSerial tiles (the near, large ones -- a few per wave) are summed by
    // the whole wave, one at a time, in blocks of 2 x 64 tiles whose boundary keys are all loaded
    // before any is tested and whose live records are all loaded before any is added: two memory
    // round trips per block instead of two per 64 tiles.
    for (uint64_t big = __ballot(n > kRedSerial); big; big &= big - 1) {
        const int bl = __ffsll((unsigned long long)big) - 1;
        const uint32_t boff = (uint32_t)__builtin_amdgcn_readlane((int)off, bl);
        const uint32_t bn = (uint32_t)__builtin_amdgcn_readlane((int)n, bl);
        const uint32_t bx0 = (uint32_t)__builtin_amdgcn_readlane((int)x0, bl);
        const uint32_t by0 = (uint32_t)__builtin_amdgcn_readlane((int)y0, bl);
        const uint32_t bw = (uint32_t)__builtin_amdgcn_readlane((int)w, bl);
        const uint64_t bkey = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(key >> 32), bl) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, bl);
        float q[10];
#pragma unroll
        for (int k = 0; k < 10; k++) q[k] = 0.f;
        constexpr int kBigBlock = GSR_BIG_BLOCK;
        for (uint32_t b0 = 0; b0 < bn; b0 += kBigBlock * kWave) {
            uint64_t bk[kBigBlock];
#pragma unroll
            for (int j = 0; j < kBigBlock; j++) {
                const uint32_t idx = min(b0 + (uint32_t)(j * kWave + lane), bn - 1u);  // clamped: always a tile of the splat
                bk[j] = boundary[(by0 + idx / bw) * (uint32_t)gx + bx0 + idx % bw];
            }
            float4 ra[kBigBlock], rb[kBigBlock], rc[kBigBlock];
#pragma unroll
            for (int j = 0; j < kBigBlock; j++) {
                const uint32_t idx = b0 + (uint32_t)(j * kWave + lane);
                ra[j] = rb[j] = rc[j] = make_float4(0.f, 0.f, 0.f, 0.f);  // set before the masked loads
                if (idx < bn && bk[j] != 0 && bkey <= bk[j]) {
                    const size_t u = 4 * (size_t)(boff + idx);
                    ra[j] = sc.rec[u + 0];
                    rb[j] = sc.rec[u + 1];
                    rc[j] = sc.rec[u + 2];
                }
            }
#pragma unroll
            for (int j = 0; j < kBigBlock; j++) {
                q[0] += ra[j].x; q[1] += ra[j].y; q[2] += ra[j].z; q[3] += ra[j].w;
                q[4] += rb[j].x; q[5] += rb[j].y; q[6] += rb[j].z; q[7] += rb[j].w;
                q[8] += rc[j].x; q[9] += rc[j].y;
            }
        }
#pragma unroll
        for (int k = 0; k < 10; k++) {
            const float t = wave_sum(q[k]);
            if (lane == bl) g[k] = t;
        }
    }
    if (!valid) return;
    dmeans2D[3 * i + 0] = g[0];
    dmeans2D[3 * i + 1] = g[1];
    dmeans2D[3 * i + 2] = 0.f;
    dopacity[i] = g[5];
    sc.gsum[2 * (size_t)i] = make_float4(g[2], g[3], g[4], g[9]);
    sc.gsum[2 * (size_t)i + 1] = make_float4(g[6], g[7], g[8], 0.f);
}

constexpr int kShPitch = 13;  // padded LDS row pitch (float4) of the staged SH rows
#ifndef GSR_BWD_NT
#define GSR_BWD_NT 1  // gradient rows written with non-temporal stores (streamed once, never re-read here)
#endif
#ifndef GSR_ACC_LD_NT
#define GSR_ACC_LD_NT 0  // measured: non-temporal accumulator loads slow preprocess_bwd (82 -> 85 us)
#endif
__device__ __forceinline__ float4 ld_acc(const float4 *p) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    if (!GSR_ACC_LD_NT) return *p;
    const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(p));
    return make_float4(t.x, t.y, t.z, t.w);
}
__device__ __forceinline__ void st_out(float *p, float v) {
    if (GSR_BWD_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st_out(float4 *p, float4 v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    if (GSR_BWD_NT) __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4 *>(p));
    else *p = v;
}
#ifndef GSR_BWD_SKIP_DEAD
#define GSR_BWD_SKIP_DEAD 1
#endif

// The chain rule of one live Gaussian's geometry (its ten accumulated sums g): conic -> 2D
// covariance -> (3D covariance, mean) through the EWA Jacobian, screen-space mean -> mean3D
// through projmatrix, inverse depth -> mean3D.  Leaves the 3D-covariance gradient in dcov, the mean
// gradient in dm, and the covariance, rotation and scale it read in c3 / q / s_in.
__device__ __forceinline__ void geom_chain(int i, float3 p, const Mat4 &V, const float *__restrict__ projmatrix, float fx,
                                           float fy, float tanx, float tany, bool has_scales,
                                           const float *__restrict__ scales, const float *__restrict__ rotations,
                                           float mod, const float *__restrict__ cov3D_precomp, const float g[10],
                                           float c3[6], float4 &q, float3 &s_in, float dm[3], float dcov[6],
                                           int raw) {
    // ---- conic -> cov2D -> cov3D and mean ----
    if (has_scales) {
        s_in = make_float3(scales[3 * i], scales[3 * i + 1], scales[3 * i + 2]);
        q = reinterpret_cast<const float4 *>(rotations)[i];
        if (raw) {  // pre-activation parameters (GaussianInputs.raw)
            s_in = make_float3(act_scale(s_in.x), act_scale(s_in.y), act_scale(s_in.z));
            q = act_rot(q);
        }
        cov3d_from_scale_rot(s_in, mod, q, c3);
    } else {
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = cov3D_precomp[6 * i + k];
    }
    const Ewa e = ewa_rows(p, V, fx, fy, tanx, tany);
    const float a = quad_form(e.m0, c3, e.m0) + 0.3f;
    const float b = quad_form(e.m0, c3, e.m1);
    const float c = quad_form(e.m1, c3, e.m1) + 0.3f;
    const float gca = g[2], gcb = g[3], gcc = g[4];
    const float denom = a * c - b * b;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    if (denom2inv != 0.f) {
        dL_da = denom2inv * (-c * c * gca + 2.f * b * c * gcb + (denom - a * c) * gcc);
        dL_dc = denom2inv * (-a * a * gcc + 2.f * a * b * gcb + (denom - a * c) * gca);
        dL_db = denom2inv * 2.f * (b * c * gca - (denom + 2.f * b * b) * gcb + a * b * gcc);
        const float *m0 = e.m0, *m1 = e.m1;
        dcov[0] = m0[0] * m0[0] * dL_da + m0[0] * m1[0] * dL_db + m1[0] * m1[0] * dL_dc;
        dcov[3] = m0[1] * m0[1] * dL_da + m0[1] * m1[1] * dL_db + m1[1] * m1[1] * dL_dc;
        dcov[5] = m0[2] * m0[2] * dL_da + m0[2] * m1[2] * dL_db + m1[2] * m1[2] * dL_dc;
        dcov[1] = 2.f * m0[0] * m0[1] * dL_da + (m0[0] * m1[1] + m0[1] * m1[0]) * dL_db +
                  2.f * m1[0] * m1[1] * dL_dc;
        dcov[2] = 2.f * m0[0] * m0[2] * dL_da + (m0[0] * m1[2] + m0[2] * m1[0]) * dL_db +
                  2.f * m1[0] * m1[2] * dL_dc;
        dcov[4] = 2.f * m0[2] * m0[1] * dL_da + (m0[1] * m1[2] + m0[2] * m1[1]) * dL_db +
                  2.f * m1[1] * m1[2] * dL_dc;
    }
    float Sm0[3], Sm1[3];
    const float *m0 = e.m0, *m1 = e.m1;
    Sm0[0] = c3[0] * m0[0] + c3[1] * m0[1] + c3[2] * m0[2];
    Sm0[1] = c3[1] * m0[0] + c3[3] * m0[1] + c3[4] * m0[2];
    Sm0[2] = c3[2] * m0[0] + c3[4] * m0[1] + c3[5] * m0[2];
    Sm1[0] = c3[0] * m1[0] + c3[1] * m1[1] + c3[2] * m1[2];
    Sm1[1] = c3[1] * m1[0] + c3[3] * m1[1] + c3[4] * m1[2];
    Sm1[2] = c3[2] * m1[0] + c3[4] * m1[1] + c3[5] * m1[2];
    float dm0[3], dm1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        dm0[k] = 2.f * Sm0[k] * dL_da + Sm1[k] * dL_db;
        dm1[k] = 2.f * Sm1[k] * dL_dc + Sm0[k] * dL_db;
    }
    const float *v = V.m;
    const float dj00 = v[0] * dm0[0] + v[4] * dm0[1] + v[8] * dm0[2];
    const float dj02 = v[2] * dm0[0] + v[6] * dm0[1] + v[10] * dm0[2];
    const float dj11 = v[1] * dm1[0] + v[5] * dm1[1] + v[9] * dm1[2];
    const float dj12 = v[2] * dm1[0] + v[6] * dm1[1] + v[10] * dm1[2];
    const float tz = 1.f / e.t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dtx = e.xmul * -fx * tz2 * dj02;
    const float dty = e.ymul * -fy * tz2 * dj12;
    const float dtz = -fx * tz2 * dj00 - fy * tz2 * dj11 + (2.f * fx * e.t.x) * tz3 * dj02 +
                      (2.f * fy * e.t.y) * tz3 * dj12;
    dm[0] = v[0] * dtx + v[1] * dty + v[2] * dtz;
    dm[1] = v[4] * dtx + v[5] * dty + v[6] * dtz;
    dm[2] = v[8] * dtx + v[9] * dty + v[10] * dtz;

    // ---- screen-space mean -> mean3D ----
    const Mat4 Pm = load_mat4(projmatrix);
    const float *pr = Pm.m;
    const float4 mh = xf_point44(p, Pm);
    const float mw = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = mh.x * mw * mw, mul2 = mh.y * mw * mw;
    dm[0] += (pr[0] * mw - pr[3] * mul1) * g[0] + (pr[1] * mw - pr[3] * mul2) * g[1];
    dm[1] += (pr[4] * mw - pr[7] * mul1) * g[0] + (pr[5] * mw - pr[7] * mul2) * g[1];
    dm[2] += (pr[8] * mw - pr[11] * mul1) * g[0] + (pr[9] * mw - pr[11] * mul2) * g[1];

    // ---- inverse depth -> mean3D ----
    {
        const float3 pv = xf_point43(p, V);
        const float dz = -g[9] / (pv.z * pv.z);
        dm[0] += dz * v[2];
        dm[1] += dz * v[6];
        dm[2] += dz * v[10];
    }
}

// 3D covariance gradient -> scale and rotation gradients (dscale_mod: 1 for upstream's convention,
// scale_modifier for the exact derivative).
__device__ __forceinline__ void scale_rot_chain(float4 q, float3 s_in, float mod, float dscale_mod, const float dcov[6],
                                                float ds[3], float dq[4]) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const float s[3] = {mod * s_in.x, mod * s_in.y, mod * s_in.z};
    const Rot3 R = quat_to_rot(q);
    const float G3[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                            {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                            {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
    float dLL[3][3];
#pragma unroll
    for (int rr = 0; rr < 3; rr++)
#pragma unroll
        for (int cc = 0; cc < 3; cc++)
            dLL[rr][cc] = 2.f * (G3[rr][0] * R.m[0][cc] * s[cc] + G3[rr][1] * R.m[1][cc] * s[cc] +
                                 G3[rr][2] * R.m[2][cc] * s[cc]);
#pragma unroll
    for (int k = 0; k < 3; k++)
        // dscale_mod = 1 (upstream: dL/d(mod s) reported as dL/ds) or mod (the exact
        // derivative, gsr_set_true_scale_gradient)
        ds[k] = dscale_mod * (dLL[0][k] * R.m[0][k] + dLL[1][k] * R.m[1][k] + dLL[2][k] * R.m[2][k]);
    float Gr[3][3];
#pragma unroll
    for (int rr = 0; rr < 3; rr++)
#pragma unroll
        for (int cc = 0; cc < 3; cc++) Gr[rr][cc] = dLL[rr][cc] * s[cc];
    dq[0] = 2.f * (-z * Gr[0][1] + y * Gr[0][2] + z * Gr[1][0] - x * Gr[1][2] - y * Gr[2][0] + x * Gr[2][1]);
    dq[1] = 2.f * (y * Gr[0][1] + z * Gr[0][2] + y * Gr[1][0] - 2.f * x * Gr[1][1] - r * Gr[1][2] +
                   z * Gr[2][0] + r * Gr[2][1] - 2.f * x * Gr[2][2]);
    dq[2] = 2.f * (-2.f * y * Gr[0][0] + x * Gr[0][1] + r * Gr[0][2] + x * Gr[1][0] + z * Gr[1][2] -
                   r * Gr[2][0] + z * Gr[2][1] - 2.f * y * Gr[2][2]);
    dq[3] = 2.f * (-2.f * z * Gr[0][0] - r * Gr[0][1] + x * Gr[0][2] + r * Gr[1][0] - 2.f * z * Gr[1][1] +
                   y * Gr[1][2] + x * Gr[2][0] + y * Gr[2][1]);
}

// d normalize(v)/dv applied to the SH direction gradient gd, added into the mean gradient
__device__ __forceinline__ void dir_chain(const float dor[3], const float gd[3], float dm[3]) {
    const float s2 = dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2];
    const float inv32 = 1.0f / sqrtf(s2 * s2 * s2);
    dm[0] += ((s2 - dor[0] * dor[0]) * gd[0] - dor[1] * dor[0] * gd[1] - dor[2] * dor[0] * gd[2]) * inv32;
    dm[1] += (-dor[0] * dor[1] * gd[0] + (s2 - dor[1] * dor[1]) * gd[1] - dor[2] * dor[1] * gd[2]) * inv32;
    dm[2] += (-dor[0] * dor[2] * gd[0] - dor[1] * dor[2] * gd[1] + (s2 - dor[2] * dor[2]) * gd[2]) * inv32;
}

__global__ __launch_bounds__(256) void preprocess_bwd_kernel(
    int P, int D, int M, const float *__restrict__ means3D, const int *__restrict__ radii,
    const float *__restrict__ shs, const uint8_t *__restrict__ clamped, const float *__restrict__ scales,
    const float *__restrict__ rotations, float mod, float dscale_mod, const float *__restrict__ cov3D_precomp,
    const float *__restrict__ viewmatrix, const float *__restrict__ projmatrix, const float *__restrict__ campos_p,
    float tanx, float tany, float fx, float fy, int gx, const uint32_t *__restrict__ tiles,
    const GRec *__restrict__ rec, const uint64_t *__restrict__ boundary, BwdScratch sc, GaussianGrads out, int raw) {
    __shared__ float4 s_sh[4 * kWave * kShPitch];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1);
    const bool valid = i < P;
    const bool has_shs = shs != nullptr;
    const bool has_scales = cov3D_precomp == nullptr;
    const bool vis = valid && radii[i] > 0;
    const bool vec_sh = M == 16 && (reinterpret_cast<uintptr_t>(shs) % 16 == 0) &&
                        (reinterpret_cast<uintptr_t>(out.dsh) % 16 == 0);

    // lanes past P stay to the end of the SH staging (the wave loads and stores rows together)
    const int iv = valid ? i : 0;
    float g[10];
    if (sc.atomic) {
        // render_bwd's atomic accumulator row (zeroed by render_fwd; untouched rows stay zero)
        // the rows are dead after this read: non-temporal loads keep them out of the caches
        const float4 a0 = ld_acc(sc.acc + 4 * (size_t)iv), a1 = ld_acc(sc.acc + 4 * (size_t)iv + 1),
                     a2 = ld_acc(sc.acc + 4 * (size_t)iv + 2);
        g[0] = a0.x; g[1] = a0.y; g[2] = a0.z; g[3] = a0.w;
        g[4] = a1.x; g[5] = a1.y; g[6] = a1.z; g[7] = a1.w;
        g[8] = a2.x; g[9] = a2.y;
        if (!vis) {
#pragma unroll
            for (int k = 0; k < 10; k++) g[k] = 0.f;
        }
        if (valid) {
            st_out(&out.dmeans2D[3 * i + 0], g[0]);
            st_out(&out.dmeans2D[3 * i + 1], g[1]);
            if (!out.sparse_rows) st_out(&out.dmeans2D[3 * i + 2], 0.f);  // sparse rows: the liveness, below
            st_out(&out.dopacity[i], g[5]);
        }
    } else {
        const float4 s0 = sc.gsum[2 * (size_t)iv], s1 = sc.gsum[2 * (size_t)iv + 1];
        g[0] = g[1] = g[5] = 0.f;  // screen-space mean and opacity: written by record_sum_kernel
        g[2] = s0.x; g[3] = s0.y; g[4] = s0.z; g[9] = s0.w;
        g[6] = s1.x; g[7] = s1.y; g[8] = s1.z;
        if (vis) {
            g[0] = out.dmeans2D[3 * i + 0];
            g[1] = out.dmeans2D[3 * i + 1];
        }
    }
    // A visible Gaussian in front of no tile's last contributor (occluded, or outside every
    // pixel's reach) has ten zero sums, so every gradient below is zero: its coefficient and
    // parameter rows are not read (88% of the bench scene's Gaussians; only its zero rows are
    // written)
    bool live = vis;
    {
        bool nz = false;
#pragma unroll
        for (int t = 0; t < 10; t++) nz = nz || g[t] != 0.f;
        if (sc.atomic && vis && nz) {
            // the row is consumed: clear it, so a second backward through the same saved buffers
            // (retain_graph, torch.autograd.grad twice, gradcheck) sums from zero again, as
            // upstream's stateless backward does.  Only the ~12% of rows render_bwd added into
            // are written, as whole 64-B lines (no partial-line read-modify-write).
            float4 *a = sc.acc + 4 * (size_t)i;
#pragma unroll
            for (int q = 0; q < 4; q++) a[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (GSR_BWD_SKIP_DEAD) {
            if (!sc.atomic && vis) nz = nz || out.dopacity[i] != 0.f;  // record mode: summed by record_sum
            live = vis && nz;
        }
    }
    // sparse rows (the native train step): the liveness column; a dead row's other gradient rows
    // are not written
    const bool wr = live || !out.sparse_rows;
    if (valid && out.sparse_rows) st_out(&out.dmeans2D[3 * i + 2], live ? 1.f : 0.f);

    float dm[3] = {0.f, 0.f, 0.f};
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const Mat4 V = load_mat4(viewmatrix);
    const int ip = live ? i : 0;
    const float3 p = make_float3(means3D[3 * ip], means3D[3 * ip + 1], means3D[3 * ip + 2]);
    float c3[6];
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float3 s_in = make_float3(0.f, 0.f, 0.f);
    if (live) {
        geom_chain(i, p, V, projmatrix, fx, fy, tanx, tany, has_scales, scales, rotations, mod, cov3D_precomp, g,
                   c3, q, s_in, dm, dcov, raw);
    }

    // ---- colour ----
    if (has_shs && vec_sh) {
        // Staged SH rows: the wave's 64 coefficient rows come in as 1 KiB contiguous loads (load k of
        // lane l = float4 k*64 + l) into a tile with rows padded to 13 float4, each lane reads and
        // overwrites its own row with dL/dsh, and the tile goes out with the same contiguous stores:
        // one lane per row would put 64 rows, 192 B apart, under every load and store.
        const int wv = threadIdx.x >> 6;
        float4 *S = s_sh + wv * kWave * kShPitch;
        const uint64_t need = __ballot(live);
        const int64_t row0 = (int64_t)blockIdx.x * blockDim.x + wv * kWave;
        const int cols = ((D + 1) * (D + 1) * 3 + 3) / 4;
        const float4 *src4 = reinterpret_cast<const float4 *>(shs) + row0 * 12;
        float4 v[12];
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int f = k * kWave + lane, row = f / 12;
            v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (((need >> row) & 1ull) && f - row * 12 < cols) v[k] = src4[f];
        }
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int f = k * kWave + lane, row = f / 12;
            S[row * kShPitch + (f - row * 12)] = v[k];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        float4 *mine = S + lane * kShPitch;
        if (live) {
            float dir[3], dor[3];
            sh_dir(p, make_float3(campos_p[0], campos_p[1], campos_p[2]), dir, dor);
            const uint8_t cl = clamped[i];
            float gc[3];
#pragma unroll
            for (int ch = 0; ch < 3; ch++) gc[ch] = (cl >> ch) & 1 ? 0.f : g[6 + ch];
            float gd[3];
            const float *row = reinterpret_cast<const float *>(mine);
            float *drow = reinterpret_cast<float *>(mine);
            switch (D) {
                case 0: sh_backward<0, true>(row, M, true, dir, gc, drow, gd); break;
                case 1: sh_backward<1, true>(row, M, true, dir, gc, drow, gd); break;
                case 2: sh_backward<2, true>(row, M, true, dir, gc, drow, gd); break;
                default: sh_backward<3, true>(row, M, true, dir, gc, drow, gd); break;
            }
            dir_chain(dor, gd, dm);
        } else {
#pragma unroll
            for (int c = 0; c < 12; c++) mine[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        float4 *dst4 = reinterpret_cast<float4 *>(out.dsh) + row0 * 12;
#pragma unroll
        for (int k = 0; k < 12; k++) {
            const int f = k * kWave + lane, row = f / 12;
            if (row0 + row < P && (!out.sparse_rows || ((need >> row) & 1ull)))
                st_out(&dst4[f], S[row * kShPitch + (f - row * 12)]);
        }
        if (valid && out.dcolors) {
            out.dcolors[3 * i + 0] = 0.f;
            out.dcolors[3 * i + 1] = 0.f;
            out.dcolors[3 * i + 2] = 0.f;
        }
    }
    if (!valid) return;
    if (has_shs && vec_sh) {
        // done above
    } else if (has_shs) {
        float *dsh = out.dsh + (size_t)i * M * 3;
        if (!live) {
            if (out.sparse_rows) {
                // not written
            } else if (vec_sh) {
                float4 *d4 = reinterpret_cast<float4 *>(dsh);
#pragma unroll
                for (int c = 0; c < 12; c++) d4[c] = make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                for (int k = 0; k < M * 3; k++) dsh[k] = 0.f;
            }
        } else {
            float dir[3], dor[3];
            sh_dir(p, make_float3(campos_p[0], campos_p[1], campos_p[2]), dir, dor);
            const uint8_t cl = clamped[i];
            float gc[3];
#pragma unroll
            for (int ch = 0; ch < 3; ch++) gc[ch] = (cl >> ch) & 1 ? 0.f : g[6 + ch];
            float gd[3];
            const float *sh = shs + (size_t)i * M * 3;
            switch (D) {
                case 0: sh_backward<0>(sh, M, vec_sh, dir, gc, dsh, gd); break;
                case 1: sh_backward<1>(sh, M, vec_sh, dir, gc, dsh, gd); break;
                case 2: sh_backward<2>(sh, M, vec_sh, dir, gc, dsh, gd); break;
                default: sh_backward<3>(sh, M, vec_sh, dir, gc, dsh, gd); break;
            }
            // d normalize(v)/dv applied to the direction gradient
            dir_chain(dor, gd, dm);
        }
        if (out.dcolors) {  // optional with shs (no colors_precomp input to differentiate)
            out.dcolors[3 * i + 0] = 0.f;
            out.dcolors[3 * i + 1] = 0.f;
            out.dcolors[3 * i + 2] = 0.f;
        }
    } else {
        out.dcolors[3 * i + 0] = g[6];
        out.dcolors[3 * i + 1] = g[7];
        out.dcolors[3 * i + 2] = g[8];
    }
    if (wr) {
        st_out(&out.dmeans3D[3 * i + 0], dm[0]);
        st_out(&out.dmeans3D[3 * i + 1], dm[1]);
        st_out(&out.dmeans3D[3 * i + 2], dm[2]);
    }

    // ---- cov3D -> scale / rotation ----
    if (has_scales) {
        float ds[3] = {0.f, 0.f, 0.f};
        float dq[4] = {0.f, 0.f, 0.f, 0.f};
        if (live) {
            scale_rot_chain(q, s_in, mod, dscale_mod, dcov, ds, dq);
        }
        if (wr) {
            st_out(&out.dscales[3 * i + 0], ds[0]);
            st_out(&out.dscales[3 * i + 1], ds[1]);
            st_out(&out.dscales[3 * i + 2], ds[2]);
            st_out(&reinterpret_cast<float4 *>(out.drots)[i], make_float4(dq[0], dq[1], dq[2], dq[3]));
        }
        if (out.dcov3D)  // optional with scales/rotations (no cov3D_precomp input)
#pragma unroll
            for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = 0.f;
    } else {
#pragma unroll
        for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = dcov[k];
    }
}

// ---- split form (atomic mode, M = 16 SH rows, scales / rotations): the dead rows and the live rows
// in two launches.  In the single kernel every wave (64 rows, ~8 of them live on the bench scene)
// carried its live rows' two extra dependent round trips (parameters, then SH rows) in front of
// the dead rows' zero stores, and its 53-KiB SH staging tile held occupancy to 3 blocks per CU:
// ~4.2 TB/s.  grad_rows_kernel streams every row's screen-space mean / opacity gradient and the
// dead rows' zero rows (skipped in sparse-rows mode) and publishes the live rows as one 64-bit
// mask per wave; grad_live_kernel compacts each kLiveRange-row range's live rows in LDS, so its lanes are
// all live, and runs the chain rule on them.  The arithmetic is the single kernel's (geom_chain,
// sh_backward, dir_chain, scale_rot_chain): the bits do not change.
// The ten per-Gaussian sums: the atomic accumulator row, or (record mode) record_sum's gsum row
// with the screen-space mean and opacity gradients it wrote; zero for an invisible Gaussian.
__device__ __forceinline__ void load_sums(const BwdScratch &sc, const GaussianGrads &out, int i, bool vis, float g[10]) {
    if (sc.atomic) {
        const float4 a0 = ld_acc(sc.acc + 4 * (size_t)i), a1 = ld_acc(sc.acc + 4 * (size_t)i + 1),
                     a2 = ld_acc(sc.acc + 4 * (size_t)i + 2);
        g[0] = a0.x; g[1] = a0.y; g[2] = a0.z; g[3] = a0.w;
        g[4] = a1.x; g[5] = a1.y; g[6] = a1.z; g[7] = a1.w;
        g[8] = a2.x; g[9] = a2.y;
    } else {
        const float4 s0 = sc.gsum[2 * (size_t)i], s1 = sc.gsum[2 * (size_t)i + 1];
        g[2] = s0.x; g[3] = s0.y; g[4] = s0.z; g[9] = s0.w;
        g[6] = s1.x; g[7] = s1.y; g[8] = s1.z;
        g[0] = vis ? out.dmeans2D[3 * i + 0] : 0.f;
        g[1] = vis ? out.dmeans2D[3 * i + 1] : 0.f;
        g[5] = vis ? out.dopacity[i] : 0.f;
    }
    if (!vis)
#pragma unroll
        for (int k = 0; k < 10; k++) g[k] = 0.f;
}

#ifndef GSR_GRAD_WIDE
#define GSR_GRAD_WIDE 0  // 1: float4 stores of whole waves' 3-float rows; measured slower (r03k: 0.0943 vs 0.0901 ms)
#endif
__device__ __forceinline__ bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

__global__ __launch_bounds__(256) void grad_rows_kernel(int P, const int *__restrict__ radii, BwdScratch sc,
                                                        GaussianGrads out, int zero_dead) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1);
    const bool valid = i < P;
    const int iv = valid ? i : 0;
    const bool vis = valid && radii[iv] > 0;
    float g[10];
    load_sums(sc, out, iv, vis, g);
    bool nz = false;
#pragma unroll
    for (int t = 0; t < 10; t++) nz = nz || g[t] != 0.f;
    const bool live = vis && nz;
    const uint64_t lm = __ballot(live);
    if (lane == 0 && (i >> 6) < (P + 63) / 64) sc.live[i >> 6] = lm;
    const int64_t row0 = (int64_t)i - lane;
    // GSR_GRAD_WIDE: a full wave's 3-float rows (768 B per array) go out as 48 float4 stores instead
    // of three strided dword stores per lane -- the mean2D values staged through a wave-private LDS
    // row, the zero rows of means3D / scales written as float4s wherever no live row shares them
    const bool wide = GSR_GRAD_WIDE && row0 + kWave <= P && aligned16(out.dmeans2D) && aligned16(out.dmeans3D) &&
                      aligned16(out.dscales);
    __shared__ __attribute__((aligned(16))) float s_m2[256 / kWave][3 * kWave];
    float *m2 = s_m2[threadIdx.x >> 6];
    if (valid) {
        const float c2 = out.sparse_rows && live ? 1.f : 0.f;
        if (wide && sc.atomic) {
            m2[3 * lane + 0] = g[0];
            m2[3 * lane + 1] = g[1];
            m2[3 * lane + 2] = c2;
        } else {
            if (sc.atomic) {  // record mode: written by record_sum_kernel
                st_out(&out.dmeans2D[3 * i + 0], g[0]);
                st_out(&out.dmeans2D[3 * i + 1], g[1]);
            }
            if (sc.atomic || out.sparse_rows) st_out(&out.dmeans2D[3 * i + 2], c2);
        }
        if (sc.atomic) st_out(&out.dopacity[i], g[5]);
        if (out.dcolors) {
            out.dcolors[3 * i + 0] = 0.f;
            out.dcolors[3 * i + 1] = 0.f;
            out.dcolors[3 * i + 2] = 0.f;
        }
        if (out.dcov3D)
#pragma unroll
            for (int k = 0; k < 6; k++) out.dcov3D[6 * i + k] = 0.f;
    }
    if (wide && sc.atomic) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS row is complete
        __builtin_amdgcn_wave_barrier();
        if (lane < 48) {
            const float4 v = *reinterpret_cast<const float4 *>(m2 + 4 * lane);
            st_out(reinterpret_cast<float4 *>(out.dmeans2D + 3 * row0) + lane, v);
        }
    }
    if (out.sparse_rows || !zero_dead) return;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (wide) {
        if (lane < 48) {
            // floats 4 lane .. 4 lane + 3 of the wave's rows: rows 4 lane / 3 and (4 lane + 3) / 3
            const int ra = (4 * lane) / 3, rb = (4 * lane + 3) / 3;
            float4 *m3 = reinterpret_cast<float4 *>(out.dmeans3D + 3 * row0) + lane;
            float4 *sc3 = reinterpret_cast<float4 *>(out.dscales + 3 * row0) + lane;
            if (!(((lm >> ra) | (lm >> rb)) & 1ull)) {
                st_out(m3, z4);
                st_out(sc3, z4);
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++)
                    if (!((lm >> ((4 * lane + e) / 3)) & 1ull)) {
                        st_out(reinterpret_cast<float *>(m3) + e, 0.f);
                        st_out(reinterpret_cast<float *>(sc3) + e, 0.f);
                    }
            }
        }
    } else if (valid && !live) {
        st_out(&out.dmeans3D[3 * i + 0], 0.f);
        st_out(&out.dmeans3D[3 * i + 1], 0.f);
        st_out(&out.dmeans3D[3 * i + 2], 0.f);
        st_out(&out.dscales[3 * i + 0], 0.f);
        st_out(&out.dscales[3 * i + 1], 0.f);
        st_out(&out.dscales[3 * i + 2], 0.f);
    }
    if (valid && !live) st_out(&reinterpret_cast<float4 *>(out.drots)[i], z4);
    // the wave's 64 zero SH rows as 1 KiB contiguous stores (float4 k*64 + l of the wave's rows)
    float4 *dst4 = reinterpret_cast<float4 *>(out.dsh) + row0 * 12;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const int f = k * kWave + lane, row = f / 12;
        if (row0 + row < P && !((lm >> row) & 1ull)) st_out(&dst4[f], z4);
    }
}

// The live rows' chain rule: per 2048-row range, 256 threads of 8 rows each (a byte of a 64-row live
// mask) compact the range's live rows in LDS (range_compact), then either
//   grad_range_kernel  the range's own workgroup walks them (one launch; the default), or
//   grad_live_list_kernel + grad_live_kernel  the ranges append them to one list (one atomic per
//                      workgroup on a frame control word) and a grid of two workgroups per CU walks
//                      that list, every thread the same share of rows however they fall
//                      (gsr_set_live_list(1)).
// Rows in spatial order (gs_train.chunk.reorder_rows) put a view's live rows in runs: a range can be
// all live and its 256 threads walk 8 rows each, one after the other, while most ranges have none
// (config-3 chunk: 0.155 ms per call per range, 0.125 through the list).  Scattered live rows
// (the bench frame, a chunk in the reference's row order) fill every range a little: the list's
// second launch and its ~1500 same-word atomics cost more than they balance (0.025 -> 0.054 ms).
constexpr int kLiveRange = 2048;
constexpr int kLiveBlocksPerCU = 2;  // 185 VGPRs: two 256-thread workgroups per CU

struct LiveArgs {
    int P, D;
    const float *means3D, *shs;
    const uint8_t *clamped;
    const float *scales, *rotations;
    float mod, dscale_mod;
    const float *viewmatrix, *projmatrix, *campos;
    float tanx, tany, fx, fy;
    BwdScratch sc;
    GaussianGrads out;
    int raw, stamped;  // stamped: render_bwd zeroed the dense rows and stamped the live ones
    StepAct act;
};

// One live row: the chain rule from its ten screen-space sums to its parameters' gradients.
// (pointer arguments __restrict__: the inputs' loads are not ordered behind the gradient stores)
__device__ __forceinline__ void live_row(int i, const Mat4 &V, int D, const float *__restrict__ means3D,
                                         const float *__restrict__ shs, const uint8_t *__restrict__ clamped,
                                         const float *__restrict__ scales, const float *__restrict__ rotations,
                                         float mod, float dscale_mod, const float *__restrict__ projmatrix,
                                         const float *__restrict__ campos_p, float tanx, float tany, float fx, float fy,
                                         const BwdScratch &sc, const GaussianGrads &out, int raw, int stamped,
                                         const StepAct &act) {
    float g[10];
    load_sums(sc, out, i, true, g);
    const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    float dm[3] = {0.f, 0.f, 0.f};
    float dcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float c3[6];
    float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
    float3 s_in = make_float3(0.f, 0.f, 0.f);
    geom_chain(i, p, V, projmatrix, fx, fy, tanx, tany, true, scales, rotations, mod, nullptr, g, c3, q,
               s_in, dm, dcov, raw);
    if (stamped) {  // the live rows' screen-space mean / opacity gradients (render_bwd zeroed the rest)
        st_out(&out.dmeans2D[3 * i + 0], g[0]);
        st_out(&out.dmeans2D[3 * i + 1], g[1]);
        st_out(&out.dmeans2D[3 * i + 2], out.sparse_rows ? 1.f : 0.f);
        st_out(&out.dopacity[i], g[5]);
    }
    if (sc.atomic) {
        // the row is consumed: cleared for a repeated backward (see preprocess_bwd_kernel)
        float4 *acc = sc.acc + 4 * (size_t)i;
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] = z4;
    }
    float dir[3], dor[3];
    sh_dir(p, make_float3(campos_p[0], campos_p[1], campos_p[2]), dir, dor);
    const uint8_t cl = clamped[i];
    float gc[3];
#pragma unroll
    for (int ch = 0; ch < 3; ch++) gc[ch] = (cl >> ch) & 1 ? 0.f : g[6 + ch];
    float gd[3];
    const float *sh = shs + (size_t)i * 48;
    float *dsh = out.dsh + (size_t)i * 48;
    switch (D) {
        case 0: sh_backward<0>(sh, 16, true, dir, gc, dsh, gd); break;
        case 1: sh_backward<1>(sh, 16, true, dir, gc, dsh, gd); break;
        case 2: sh_backward<2>(sh, 16, true, dir, gc, dsh, gd); break;
        default: sh_backward<3>(sh, 16, true, dir, gc, dsh, gd); break;
    }
    dir_chain(dor, gd, dm);
    st_out(&out.dmeans3D[3 * i + 0], dm[0]);
    st_out(&out.dmeans3D[3 * i + 1], dm[1]);
    st_out(&out.dmeans3D[3 * i + 2], dm[2]);
    float ds[3], dq[4];
    scale_rot_chain(q, s_in, mod, dscale_mod, dcov, ds, dq);
    if (act.on) {
        // the activation backward (train.hip activate_bwd_step_kernel's expressions): exp,
        // normalise and sigmoid with the skybox lock, the densification statistics and the
        // relevance flag of this live row
#pragma unroll
        for (int k = 0; k < 3; k++) ds[k] = ds[k] * act_scale(act.s_raw[3 * i + k]);
        const float4 x = act.q_raw[i];
        const float4 gq = make_float4(dq[0], dq[1], dq[2], dq[3]);
        const float nq = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
        const float d = fmaxf(nq, 1e-12f);
        const float gd =
            -(gq.x * ((x.x / d) / d) + gq.y * ((x.y / d) / d) + gq.z * ((x.z / d) / d) + gq.w * ((x.w / d) / d));
        const float gn = nq >= 1e-12f && nq != 0.f ? gd / nq : 0.f;
        dq[0] = gq.x / d + x.x * gn;
        dq[1] = gq.y / d + x.y * gn;
        dq[2] = gq.z / d + x.z * gn;
        dq[3] = gq.w / d + x.w * gn;
        const float y = act_opacity(act.o_raw[i]);
        const float go = (int64_t)i < act.skybox ? 0.f : g[5] * (1.f - y) * y;
        st_out(&out.dopacity[i], go);
        if (go != 0.f) *act.flag = 1;
        const int r = act.radii[i];
        if (r > 0) {
            const float gx = g[0], gy = g[1];
            const float nn = sqrtf(gx * gx + gy * gy);
            act.maxr[i] = fmaxf(act.maxr[i], (float)r);
            act.accum[i] = fmaxf(nn, act.accum[i]);
            act.denom[i] = act.denom[i] + 1.f;
        }
    }
    st_out(&out.dscales[3 * i + 0], ds[0]);
    st_out(&out.dscales[3 * i + 1], ds[1]);
    st_out(&out.dscales[3 * i + 2], ds[2]);
    st_out(&reinterpret_cast<float4 *>(out.drots)[i], make_float4(dq[0], dq[1], dq[2], dq[3]));
}

// The range's live rows compacted: thread t's mask bits, s_off[] their exclusive offsets, s_off[nw]
// the range's count.
__device__ __forceinline__ void range_compact(const LiveArgs a, int64_t base, const uint32_t *__restrict__ stamps,
                                              uint32_t stamp, uint32_t *s_off, uint8_t *s_byte, uint64_t &m,
                                              uint32_t &byte) {
    const int t = threadIdx.x;
    const int P = a.P;
    const int nw = (P + 63) / 64;
    // thread t owns rows [8t, 8t + 8) of the range: byte t % 8 of live mask t / 8 -- from
    // grad_rows_kernel's masks, or (stamps != NULL) from the rows render_bwd stamped this backward
    const int wi = (int)(base / 64) + t / 8;
    if (stamps) {
        byte = 0u;
        const int64_t r0 = base + 8 * t;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (r0 + k < P && stamps[r0 + k] == stamp) byte |= 1u << k;
        s_byte[t] = (uint8_t)byte;
        __syncthreads();
        m = 0ull;
#pragma unroll
        for (int k = 0; k < 8; k++) m |= (uint64_t)s_byte[(t & ~7) + k] << (8 * k);
    } else {
        m = wi < nw ? a.sc.live[wi] : 0ull;
        byte = (uint32_t)(m >> (8 * (t & 7))) & 0xFFu;
    }
    if ((t & 7) == 0) s_off[t / 8] = (uint32_t)__popcll(m);
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (int k = 0; k < kLiveRange / 64; k++) {
            const uint32_t c = s_off[k];
            s_off[k] = run;
            run += c;
        }
        s_off[kLiveRange / 64] = run;
    }
    __syncthreads();
}

// The native step: densification statistics of this thread's visible rows that are not live (their
// screen-space gradient is zero: densify_stats_kernel's arithmetic with n = 0).
__device__ __forceinline__ void nonlive_stats(const LiveArgs a, int64_t base, uint32_t byte) {
    if (!a.act.on) return;
    const int64_t r0 = base + 8 * threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int64_t i = r0 + k;
        if (i >= a.P || ((byte >> k) & 1u)) continue;
        const int r = a.act.radii[i];
        if (r > 0) {
            const float nn = sqrtf(0.f * 0.f + 0.f * 0.f);
            a.act.maxr[i] = fmaxf(a.act.maxr[i], (float)r);
            a.act.accum[i] = fmaxf(nn, a.act.accum[i]);
            a.act.denom[i] = a.act.denom[i] + 1.f;
        }
    }
}

__global__ __launch_bounds__(256) void grad_range_kernel(
    int P, int D, const float *__restrict__ means3D, const float *__restrict__ shs, const uint8_t *__restrict__ clamped,
    const float *__restrict__ scales, const float *__restrict__ rotations, float mod, float dscale_mod,
    const float *__restrict__ viewmatrix, const float *__restrict__ projmatrix, const float *__restrict__ campos_p,
    float tanx, float tany, float fx, float fy, BwdScratch sc, GaussianGrads out, int raw,
    const uint32_t *__restrict__ stamps, uint32_t stamp, StepAct act) {
    GSR_KS(kKsGradRange);
    __shared__ uint16_t s_list[kLiveRange];
    __shared__ uint32_t s_off[kLiveRange / 64 + 1];
    __shared__ uint8_t s_byte[256];
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kLiveRange;
    LiveArgs a{};
    a.P = P;
    a.sc = sc;
    a.act = act;
    uint64_t m;
    uint32_t byte;
    range_compact(a, base, stamps, stamp, s_off, s_byte, m, byte);
    {
        uint32_t pos = s_off[t / 8] + (uint32_t)__popcll(m & ((1ull << (8 * (t & 7))) - 1ull));
        for (uint32_t b = byte; b; b &= b - 1u) s_list[pos++] = (uint16_t)(8 * t + __builtin_ctz(b));
    }
    __syncthreads();
    const uint32_t n = s_off[kLiveRange / 64];
    nonlive_stats(a, base, byte);
    const Mat4 V = load_mat4(viewmatrix);
    for (uint32_t e = (uint32_t)t; e < n; e += blockDim.x)
        live_row((int)(base + s_list[e]), V, D, means3D, shs, clamped, scales, rotations, mod, dscale_mod, projmatrix,
                 campos_p, tanx, tany, fx, fy, sc, out, raw, stamps != nullptr, act);
}

__global__ __launch_bounds__(256) void grad_live_list_kernel(LiveArgs a, const uint32_t *__restrict__ stamps,
                                                             uint32_t stamp, uint32_t *__restrict__ ctr) {
    GSR_KS(kKsLiveList);
    __shared__ uint32_t s_off[kLiveRange / 64 + 1];
    __shared__ uint8_t s_byte[256];
    __shared__ uint32_t s_base;
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kLiveRange;
    uint64_t m;
    uint32_t byte;
    range_compact(a, base, stamps, stamp, s_off, s_byte, m, byte);
    if (t == 0) {
        const uint32_t n = s_off[kLiveRange / 64];
        s_base = n ? __hip_atomic_fetch_add(ctr, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    }
    __syncthreads();
    uint32_t pos = s_base + s_off[t / 8] + (uint32_t)__popcll(m & ((1ull << (8 * (t & 7))) - 1ull));
    for (uint32_t b = byte; b; b &= b - 1u) a.sc.list[pos++] = (uint32_t)(base + 8 * t + __builtin_ctz(b));
    nonlive_stats(a, base, byte);
}

// ctr[0]: the list's length (grad_live_list_kernel), ctr[1]: finished workgroups; the last one
// to finish zeroes both for the next backward of the frame (the preprocess zeroed them first).
__global__ __launch_bounds__(256) void grad_live_kernel(LiveArgs a, uint32_t *__restrict__ ctr) {
    GSR_KS(kKsGradLive);
    const uint32_t n = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const Mat4 V = load_mat4(a.viewmatrix);
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const int i_ = (int)a.sc.list[e];
        live_row(i_, V, a.D, a.means3D, a.shs, a.clamped, a.scales, a.rotations, a.mod, a.dscale_mod, a.projmatrix, a.campos,
                 a.tanx, a.tany, a.fx, a.fy, a.sc, a.out, a.raw, a.stamped, a.act);
    }
    // every workgroup has read n before it counts itself in
    __syncthreads();
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&ctr[1], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u) {
        __hip_atomic_store(&ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&ctr[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

#ifndef GSR_BWD_ZERO_IN_RENDER
#define GSR_BWD_ZERO_IN_RENDER 1  // the dense zero rows stored by render_bwd's waves after their replay
#endif
#ifndef GSR_BWD_ZERO_PCT
#define GSR_BWD_ZERO_PCT 100
#endif
#ifndef GSR_BWD_MEMSET
#define GSR_BWD_MEMSET 0  // 1: hipMemsetAsync fills; preprocess_bwd 0.0891 -> 0.0866 ms but the fills leave dirty lines that slow the next frame (preprocess 0.035 -> 0.040, sort 0.106 -> 0.111 ms; r03n)
#endif
#ifndef GSR_BWD_SPLIT
#define GSR_BWD_SPLIT 1  // 0: the single preprocess_bwd_kernel for every frame
#endif

namespace {
bool split_ok(const GaussianInputs &in, const GaussianGrads &out, const BwdScratch &sc) {
    return GSR_BWD_SPLIT && GSR_BWD_SKIP_DEAD && sc.live && in.shs && in.M == 16 && !in.cov3D_precomp && in.scales &&
           in.rotations && reinterpret_cast<uintptr_t>(in.shs) % 16 == 0 &&
           reinterpret_cast<uintptr_t>(out.dsh) % 16 == 0;
}
}  // namespace

bool bwd_zero_rows(const GaussianInputs &in, const GaussianGrads &out, const BwdScratch &sc, uint32_t *gs_stamps,
                   int nblocks, ZeroRows *z) {
    if (!GSR_BWD_ZERO_IN_RENDER || in.P == 0 || nblocks <= 0 || !sc.atomic || !gs_stamps || !split_ok(in, out, sc))
        return false;
    // sparse rows: only the screen-space mean and opacity gradients are dense
    const uint64_t P = (uint64_t)in.P;
    float *p[kZeroArrays] = {out.dmeans2D, out.dopacity, out.dsh, out.dmeans3D, out.dscales, out.drots};
    const uint64_t n[kZeroArrays] = {3 * P, P, 48 * P, 3 * P, 3 * P, 4 * P};
    const int na = out.sparse_rows ? 2 : kZeroArrays;
    for (int k = 0; k < na; k++)
        if (!p[k] || (reinterpret_cast<uintptr_t>(p[k]) & 15u)) return false;
    z->c4[0] = 0;
    for (int k = 0; k < kZeroArrays; k++) {
        z->p[k] = k < na ? p[k] : nullptr;
        z->n[k] = k < na ? n[k] : 0;
        z->c4[k + 1] = z->c4[k] + z->n[k] / 4;
    }
    static std::atomic<uint32_t> g_stamp{0};
    z->stamps = gs_stamps;
    z->stamp = g_stamp.fetch_add(1, std::memory_order_relaxed) + 1u;
    // only the first GSR_BWD_ZERO_PCT % of the backward's workgroups in launch order (the heaviest
    // tiles first) carry zero rows: the light tiles at the end of the launch finish without them
    // GSR_BWD_ZERO_FROM (environment, measurement A/B): the zero rows go to the workgroups from that
    // percentage of the grid on (launch order: the light tiles and the idle segment slots last)
    static const int zfrom_pct = [] {
        const char *e = getenv("GSR_BWD_ZERO_FROM");
        const int v = e ? atoi(e) : 0;
        return v > 0 && v < 100 ? v : 0;
    }();
    z->zfrom = (uint32_t)((uint64_t)nblocks * zfrom_pct / 100);
    const uint64_t nz = std::max<uint64_t>(1, ((uint64_t)nblocks - z->zfrom) * GSR_BWD_ZERO_PCT / 100);
    z->per4 = (z->c4[kZeroArrays] + nz - 1) / nz;
    return true;
}

void launch_preprocess_bwd(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const ImageState &is,
                           const int *radii, const BwdScratch &sc, const GaussianGrads &out, hipStream_t s,
                           const ZeroRows *zr) {
    const bool rows_zeroed = zr != nullptr;
    if (in.P == 0) return;
    if (!sc.atomic)  // atomic mode: the sums are already in GeomState.acc
        hipLaunchKernelGGL(record_sum_kernel, dim3((in.P + 255) / 256), dim3(256), 0, s, in.P, cam.gx, in.means3D,
                       cam.view, gs.rect8, gs.rect4, gs.offsets, is.boundary, sc, out.dmeans2D, out.dopacity);
    const bool split = split_ok(in, out, sc);
    note_step_act_done(false);
    // the native step's fused activation backward needs the raw parameters (GaussianInputs.raw)
    StepAct act = step_act();
    if (!in.raw || !out.sparse_rows) act.on = 0;
    if (split) {
        // dense rows: the dead rows' zeros as one fill per gradient array (streaming stores of whole
        // arrays) instead of grad_rows_kernel's per-row stores; grad_live_kernel then overwrites the
        // live rows (GSR_BWD_MEMSET=0: grad_rows_kernel writes the zeros)
        const bool fill = GSR_BWD_MEMSET && !out.sparse_rows && !rows_zeroed;
        if (fill) {
            const size_t P = (size_t)in.P;
            (void)hipMemsetAsync(out.dsh, 0, sizeof(float) * P * 48, s);
            (void)hipMemsetAsync(out.dmeans3D, 0, sizeof(float) * P * 3, s);
            (void)hipMemsetAsync(out.dscales, 0, sizeof(float) * P * 3, s);
            (void)hipMemsetAsync(out.drots, 0, sizeof(float) * P * 4, s);
        }
        // rows zeroed by render_bwd: its stamps name the live rows (no grad_rows pass)
        if (!rows_zeroed)
            hipLaunchKernelGGL(grad_rows_kernel, dim3((in.P + 255) / 256), dim3(256), 0, s, in.P, radii, sc, out,
                               fill ? 0 : 1);
        const LiveArgs la{in.P, in.D, in.means3D, in.shs, gs.clamped, in.scales, in.rotations, in.scale_modifier,
                          true_scale_gradient() ? in.scale_modifier : 1.0f, cam.view, cam.proj, cam.campos, cam.tanx,
                          cam.tany, cam.fx, cam.fy, sc, out, in.raw, rows_zeroed ? 1 : 0, act};
        const uint32_t *stamps = rows_zeroed ? zr->stamps : nullptr;
        const uint32_t stamp = rows_zeroed ? zr->stamp : 0u;
        const int nr = (in.P + kLiveRange - 1) / kLiveRange;
        if (sc.list) {  // gsr_set_live_list(1) when the scratch was carved
            uint32_t *const ctr = dsort_live_words(gs);
            hipLaunchKernelGGL(grad_live_list_kernel, dim3(nr), dim3(256), 0, s, la, stamps, stamp, ctr);
            const int nb = std::max(1, std::min((in.P + 255) / 256, kLiveBlocksPerCU * device_cus()));
            hipLaunchKernelGGL(grad_live_kernel, dim3(nb), dim3(256), 0, s, la, ctr);
        } else {
            hipLaunchKernelGGL(grad_range_kernel, dim3(nr), dim3(256), 0, s, in.P, in.D, in.means3D, in.shs, gs.clamped,
                               in.scales, in.rotations, in.scale_modifier, la.dscale_mod, cam.view, cam.proj,
                               cam.campos, cam.tanx, cam.tany, cam.fx, cam.fy, sc, out, in.raw, stamps, stamp, act);
        }
        note_step_act_done(act.on != 0);
        return;
    }
    hipLaunchKernelGGL(preprocess_bwd_kernel, dim3((in.P + 255) / 256), dim3(256), 0, s, in.P, in.D, in.M, in.means3D,
                       radii, in.shs, gs.clamped, in.scales, in.rotations, in.scale_modifier,
                       true_scale_gradient() ? in.scale_modifier : 1.0f, in.cov3D_precomp,
                       cam.view, cam.proj, cam.campos, cam.tanx, cam.tany, cam.fx, cam.fy, cam.gx, gs.tiles, gs.rec,
                       is.boundary, sc, out, in.raw);
}

GSR_KSTAMP_READER(kstamp_read_backward)

}  // namespace gsr
