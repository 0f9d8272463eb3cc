// preprocess.hip -- per-Gaussian forward preprocess and the frustum test (SURVEY.md 8(a) rows
// A4, A12).  Key duplication / sorting / tile ranges (A6-A8) are binning.hip.
//
// Layout: inputs are the caller's AoS tensors (means (P,3), scales (P,3), rotations (P,4),
// shs (P,M,3)); the output is one 64-B GRec per Gaussian (gsr_device.h) so that every tile
// instance the render kernels touch is a single cache-line gather.
#include <algorithm>

#include "gsr_launch.h"

#ifndef GSR_SH_NT
#define GSR_SH_NT 0  // SH coefficient rows read with non-temporal loads in the colour pass
#endif

namespace gsr {

#ifndef GSR_PARAM_NT
#define GSR_PARAM_NT 1  // parameter rows read with non-temporal loads in the preprocess (read once per frame)
#endif
__device__ __forceinline__ float ldp(const float *p) { return GSR_PARAM_NT ? __builtin_nontemporal_load(p) : *p; }

template <bool kVecSH, bool kSplitColor>
__global__ __launch_bounds__(256) void preprocess_kernel(
    int P, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales, float mod,
    const float *__restrict__ rotations, const float *__restrict__ opacities, const float *__restrict__ shs,
    const float *__restrict__ colors_precomp, const float *__restrict__ cov3D_precomp,
    const float *__restrict__ viewmatrix, const float *__restrict__ projmatrix, const float *__restrict__ campos,
    int W, int H, float tanx, float tany, float fx, float fy, int gx, int gy, GeomState gs, int *__restrict__ radii,
    int raw, CutRef cut) {
    GSR_KS(kKsPreprocess);
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    // the depth sort's control words (tickets, histograms, lookback status) start at zero
    for (uint32_t c = (uint32_t)i; c < gs.ctrl_zero; c += gridDim.x * blockDim.x) gs.ctrl[c] = 0u;
    if (i >= P) return;
    const Mat4 V = load_mat4(viewmatrix);
    const Mat4 Pm = load_mat4(projmatrix);
    radii[i] = 0;
    gs.tiles[i] = 0;
    gs.dkey[i] = 0xFFFFFFFFu;  // culled Gaussians sort behind every visible one
    if (gs.rect4)
        gs.rect4[i] = 0u;
    else
        gs.rect8[i] = make_uint2(0u, 0u);
    // a fused hierarchy cut: the row is the blend of its child and parent rows (plain loads: siblings
    // share their parent's row, which then hits in cache)
    const bool fused = cut.ri != nullptr;
    int64_t ci = i, pi = i;
    float ct = 1.f;
    if (fused) cut_source(cut, i, ci, pi, ct);
    const float3 p = fused ? make_float3(cut_lerp(ct, means3D[3 * ci], means3D[3 * pi]),
                                         cut_lerp(ct, means3D[3 * ci + 1], means3D[3 * pi + 1]),
                                         cut_lerp(ct, means3D[3 * ci + 2], means3D[3 * pi + 2]))
                           : make_float3(ldp(means3D + 3 * i), ldp(means3D + 3 * i + 1), ldp(means3D + 3 * i + 2));
    const float3 pv = xf_point43(p, V);
    if (pv.z <= 0.2f) return;  // in_frustum (prefiltered is treated as a plain cull)
    const float4 ph = xf_point44(p, Pm);
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ndcx = ph.x * pw, ndcy = ph.y * pw;

    float c3[6];
    if (cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; k++) c3[k] = cov3D_precomp[6 * i + k];
    } else {
        float3 s;
        float4 q;
        if (fused) {
            s = make_float3(cut_lerp(ct, scales[3 * ci], scales[3 * pi]), cut_lerp(ct, scales[3 * ci + 1], scales[3 * pi + 1]),
                            cut_lerp(ct, scales[3 * ci + 2], scales[3 * pi + 2]));
            const float4 qc = reinterpret_cast<const float4 *>(rotations)[ci];
            float4 qp = reinterpret_cast<const float4 *>(rotations)[pi];
            const float dot = qc.x * qp.x + qc.y * qp.y + qc.z * qp.z + qc.w * qp.w;  // torch.bmm, left to right
            if (dot < 0.f) qp = make_float4(-qp.x, -qp.y, -qp.z, -qp.w);
            q = make_float4(cut_lerp(ct, qc.x, qp.x), cut_lerp(ct, qc.y, qp.y), cut_lerp(ct, qc.z, qp.z),
                            cut_lerp(ct, qc.w, qp.w));
        } else {
            s = make_float3(ldp(scales + 3 * i), ldp(scales + 3 * i + 1), ldp(scales + 3 * i + 2));
            q = make_float4(ldp(rotations + 4 * i), ldp(rotations + 4 * i + 1), ldp(rotations + 4 * i + 2),
                            ldp(rotations + 4 * i + 3));
        }
        if (raw) {  // the native step's pre-activation parameters (GaussianInputs.raw)
            s = make_float3(act_scale(s.x), act_scale(s.y), act_scale(s.z));
            q = act_rot(q);
        }
        cov3d_from_scale_rot(s, mod, q, c3);
    }
    const Ewa e = ewa_rows(p, V, fx, fy, tanx, tany);
    const float ca = quad_form(e.m0, c3, e.m0) + 0.3f;
    const float cb = quad_form(e.m0, c3, e.m1);
    const float cc = quad_form(e.m1, c3, e.m1) + 0.3f;
    const float det = ca * cc - cb * cb;
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (ca + cc);
    const float lambda1 = mid + sqrtf(fmax_(0.1f, mid * mid - det));
    const float radius = ceilf(3.f * sqrtf(lambda1));
    const float px = ndc2pix(ndcx, W), py = ndc2pix(ndcy, H);
    const Rect r = get_rect(px, py, (int)radius, gx, gy);
    const int area = (r.x1 - r.x0) * (r.y1 - r.y0);
    if (area == 0) return;

    float4 col = make_float4(0.f, 0.f, 0.f, 0.f);
    uint8_t clamp_bits = 0;
    if (kSplitColor) {
        // colour + clamp bits come from preprocess_color_kernel on the side stream
    } else if (colors_precomp) {
        col = make_float4(colors_precomp[3 * i], colors_precomp[3 * i + 1], colors_precomp[3 * i + 2], 0.f);
    } else {
        float dir[3], dor[3];
        sh_dir(p, make_float3(campos[0], campos[1], campos[2]), dir, dor);
        const int nc = (D + 1) * (D + 1);
        float sh[48];
        const float *src = shs + (size_t)i * M * 3;
        if (kVecSH) {
            const float4 *s4 = reinterpret_cast<const float4 *>(src);
#pragma unroll
            for (int k = 0; k < 12; k++) {
                if (4 * k < nc * 3) {
                    const float4 v = s4[k];
                    sh[4 * k] = v.x; sh[4 * k + 1] = v.y; sh[4 * k + 2] = v.z; sh[4 * k + 3] = v.w;
                } else {
                    sh[4 * k] = sh[4 * k + 1] = sh[4 * k + 2] = sh[4 * k + 3] = 0.f;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 48; k++) sh[k] = k < nc * 3 ? src[k] : 0.f;
        }
        float rgb[3];
#pragma unroll
        for (int ch = 0; ch < 3; ch++) {
            const float v = sh_channel(D, sh + ch, dir[0], dir[1], dir[2]);
            if (v < 0.f) clamp_bits |= (uint8_t)(1u << ch);
            rgb[ch] = v < 0.f ? 0.f : v;
        }
        col = make_float4(rgb[0], rgb[1], rgb[2], 0.f);
    }
    if (!kSplitColor) col.w = 1.f / pv.z;
    const float op = fused ? cut_lerp(ct, opacities[ci], opacities[pi])
                           : raw ? act_opacity(ldp(opacities + i)) : ldp(opacities + i);
    const float ca_ = cc * det_inv, cb_ = -cb * det_inv, cc_ = ca * det_inv;
    // Half-extents of the region where alpha = op * exp(power) can reach 1/255:
    // power >= -t, t = ln(255 op)  <=>  d^T Q d <= 2t  ->  |dx| <= sqrt(2t (Q^-1)_xx).  Evaluated
    // from the stored conic in double with a relative + absolute margin, so culling against it
    // never drops an instance that changes any pixel (render.hip).
    float ex = -1.f, ey = -1.f;
    const double t = log(255.0 * (double)op);
    if (t >= 0.0) {
        const double qa = ca_, qb = cb_, qc = cc_;
        const double dq = qa * qc - qb * qb;
        if (dq > 0.0 && qa > 0.0 && qc > 0.0) {
            ex = (float)(sqrt(2.0 * t * qc / dq) * 1.001 + 0.1);
            ey = (float)(sqrt(2.0 * t * qa / dq) * 1.001 + 0.1);
        } else {
            ex = ey = 3.0e38f;  // degenerate conic: never cull
        }
    }
    radii[i] = (int)radius;
    float4 *R = reinterpret_cast<float4 *>(gs.rec + i);
    R[0] = make_float4(px, py, ca_, cb_);
    R[1] = make_float4(cc_, op, ex, ey);
    if (!kSplitColor) R[2] = col;
    // cull threshold of ellipse_meets_box (gsr_device.h): tau = 2 ln(255 op) with its margin,
    // formed once here instead of per tile instance (a v_log + 4 VALU per instance per batch)
    const float tau = (float)(2.0 * t);
    const float tm = fmaf(fabsf(tau), 1.0e-3f, tau) + 1.0e-2f;
    R[3] = make_float4(__uint_as_float((uint32_t)r.x0 | ((uint32_t)r.y0 << 16)), __uint_as_float((uint32_t)(r.x1 - r.x0)),
                       __uint_as_float(__float_as_uint(pv.z)), tm);
    if (!kSplitColor) gs.clamped[i] = clamp_bits;
    gs.tiles[i] = (uint32_t)area;
    if (gs.rect4)
        gs.rect4[i] = (uint32_t)r.x0 | ((uint32_t)r.y0 << 8) | ((uint32_t)r.x1 << 16) | ((uint32_t)r.y1 << 24);
    else
        gs.rect8[i] = make_uint2((uint32_t)r.x0 | ((uint32_t)r.y0 << 16), (uint32_t)r.x1 | ((uint32_t)r.y1 << 16));
    gs.dkey[i] = __float_as_uint(pv.z);
}

// The SH colour of the visible Gaussians, split off the preprocess so that it streams its 192 B
// SH rows on a side stream while the depth sort and the binning (latency-bound, little HBM
// traffic) run on the main one.  Each wave stages its 64 rows (12 KiB, contiguous) through LDS:
// load k of lane l is float4 k*64 + l of the block, so every load instruction reads 1 KiB
// contiguously (one lane per row would put 64 rows, 192 B apart, under each instruction), and
// rows land in a per-wave tile padded to 13 float4 (ds_read_b128 of one row per lane is then
// conflict-free: 52-dword stride).  Rows of culled Gaussians and coefficients above the active
// degree are not fetched.
constexpr int kShRow = 12;                 // float4 per row (M = 16)
constexpr int kShPitch = 13;               // padded LDS row pitch, in float4
#ifndef GSR_COLOR_WAVES
#define GSR_COLOR_WAVES 8  // 104 KiB per block, one block per CU: it interferes less with the binning beside it
#endif
constexpr int kColorWaves = GSR_COLOR_WAVES;  // waves per block (13 KiB of LDS each)
// A fused hierarchy cut (config 5: two SH-row gathers per row) in 10-wave blocks, still one per CU
// (140 KiB with the cut's index slice): the pass 1.42-1.44 -> 1.39-1.40 ms, the frame's raster part
// 2.28-2.30 -> 2.25-2.28 ms (r06zk, r06zm, interleaved; a next-row-block prefetch instead,
// GSR_COLOR_PF: 3.31 against 3.26 ms per frame)
#ifndef GSR_COLOR_WAVES_CUT
#define GSR_COLOR_WAVES_CUT 10
#endif
#ifndef GSR_COLOR_BLOCKS
#define GSR_COLOR_BLOCKS 0
#endif
constexpr int kColorThreads = kColorWaves * kWave;

// GSR_COLOR_CHUNKED: the rows pass through LDS in three 16-float chunks instead of whole (5 instead of
// 13 float4 of LDS per row), so a block holds 40 instead of 104 KiB and the VGPRs, not the LDS,
// bound the waves per CU; each load instruction reads 64 B of each of 16 rows.
#ifndef GSR_COLOR_CHUNKED
#define GSR_COLOR_CHUNKED 0
#endif
constexpr int kChPitch = 5;  // chunked LDS row pitch, in float4 (20 dwords: ds_read_b128 of 16 lanes conflict-free)
constexpr int kColorPitch = GSR_COLOR_CHUNKED ? kChPitch : kShPitch;

// GSR_COLOR_PF: each wave issues the next row block's SH loads before it evaluates the current
// one (the persistent grid walks row blocks; with one 8-wave block per CU the VGPR budget, not
// occupancy, pays for the second 48-VGPR buffer), so a CU keeps twice the bytes in flight
#ifndef GSR_COLOR_PF
#define GSR_COLOR_PF 0  // measured: no step-time change (r03x), the pass is off the critical path
#endif

struct ShRows {
    float4 v[kShRow];
    bool vis;
    int64_t c, p;  // a fused cut: the lane's row's child and parent rows, weight t
    float t;
};

// The wave's 64 SH rows of row block vb into registers, 1 KiB contiguous per load instruction.
// kCut (a fused hierarchy cut): each row is the blend of a child and a parent row -- both fetched
// float4 by float4 as above from the rows' own places (the (child, parent, weight) of the wave's 64
// rows staged in the wave's slice of s_idx), the blend formed in registers.
template <bool kCut>
__device__ __forceinline__ void color_fetch(int vb, ShRows &r, int P, int D, const float *__restrict__ shs,
                                            const int *__restrict__ radii, const CutRef &cut, int4 *s_idx) {
    const int i = vb * blockDim.x + threadIdx.x;
    r.vis = i < P && (!radii || radii[i] > 0);  // radii NULL: forked before the preprocess, every row
    const int nc = (D + 1) * (D + 1);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t need = __ballot(r.vis);
    const int64_t row0 = (int64_t)vb * blockDim.x + wv * kWave;
    const int cols = (nc * 3 + 3) / 4;  // float4 per row that hold active coefficients
    const float4 *src4 = reinterpret_cast<const float4 *>(shs) + (kCut ? 0 : row0 * kShRow);
    if (kCut) {
        r.c = r.p = 0;
        r.t = 1.f;
        if (r.vis) cut_source(cut, i, r.c, r.p, r.t);
        __builtin_amdgcn_wave_barrier();  // the wave's previous reads of its slice are done
        s_idx[wv * kWave + lane] = make_int4((int)r.c, (int)r.p, __float_as_int(r.t), 0);
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int k = 0; k < kShRow; k++) {
        // whole rows: float4 k*64 + l of the wave's rows; chunked: chunk k / 4 (float4 4(k/4) .. +3 of
        // every row), 16 rows per instruction
        const int f = GSR_COLOR_CHUNKED ? (k & 3) * kWave + lane : k * kWave + lane;
        const int row = GSR_COLOR_CHUNKED ? f >> 2 : f / kShRow;
        const int col = GSR_COLOR_CHUNKED ? 4 * (k >> 2) + (f & 3) : f - row * kShRow;
        r.v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kCut) {
            if (((need >> row) & 1ull) && col < cols) {
                const int4 x = s_idx[wv * kWave + row];
                const float t = __int_as_float(x.z);
                const float4 a = src4[(int64_t)x.x * kShRow + col], b = src4[(int64_t)x.y * kShRow + col];
                r.v[k] = make_float4(cut_lerp(t, a.x, b.x), cut_lerp(t, a.y, b.y), cut_lerp(t, a.z, b.z),
                                     cut_lerp(t, a.w, b.w));
            }
            continue;
        }
        if (((need >> row) & 1ull) && col < cols) {
            const int e = row * kShRow + col;  // == f for whole rows
            if (GSR_SH_NT) {
                typedef float f4 __attribute__((ext_vector_type(4)));
                const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(src4 + e));
                r.v[k] = make_float4(t.x, t.y, t.z, t.w);
            } else {
                r.v[k] = src4[e];
            }
        }
    }
}

// Rows through the wave's LDS tile to one row per lane, then the colour of that lane's Gaussian.
template <bool kCut>
__device__ __forceinline__ void color_finish(int vb, const ShRows &r, float4 *s_sh, int P, int D,
                                             const float *__restrict__ means3D, const float *__restrict__ campos,
                                             const float *__restrict__ viewmatrix, const GeomState &gs) {
    const int i = vb * blockDim.x + threadIdx.x;
    const int nc = (D + 1) * (D + 1);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4 *S = s_sh + wv * kWave * kColorPitch;
    float sh[48];
    if (GSR_COLOR_CHUNKED) {
#pragma unroll
        for (int q = 0; q < 3; q++) {
            __builtin_amdgcn_wave_barrier();  // the wave's previous reads of its tile are done
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const int f = kk * kWave + lane;
                S[(f >> 2) * kChPitch + (f & 3)] = r.v[4 * q + kk];
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes landed
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const float4 w = S[lane * kChPitch + c];
                sh[16 * q + 4 * c] = w.x; sh[16 * q + 4 * c + 1] = w.y;
                sh[16 * q + 4 * c + 2] = w.z; sh[16 * q + 4 * c + 3] = w.w;
            }
        }
    } else {
        __builtin_amdgcn_wave_barrier();  // the wave's previous reads of its tile are done
#pragma unroll
        for (int k = 0; k < kShRow; k++) {
            const int f = k * kWave + lane, row = f / kShRow, col = f - row * kShRow;
            S[row * kShPitch + col] = r.v[k];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < kShRow; c++) {
            const float4 w = S[lane * kShPitch + c];
            sh[4 * c] = w.x; sh[4 * c + 1] = w.y; sh[4 * c + 2] = w.z; sh[4 * c + 3] = w.w;
        }
    }
    if (i >= P) return;
    if (!r.vis) {
        gs.clamped[i] = 0;
        return;
    }
#pragma unroll
    for (int k = 0; k < 48; k++) sh[k] = k < nc * 3 ? sh[k] : 0.f;  // tail of a partial float4
    // the mean as the preprocess formed it (a fused cut: the same blend)
    const float3 p = kCut ? make_float3(cut_lerp(r.t, means3D[3 * r.c], means3D[3 * r.p]),
                                        cut_lerp(r.t, means3D[3 * r.c + 1], means3D[3 * r.p + 1]),
                                        cut_lerp(r.t, means3D[3 * r.c + 2], means3D[3 * r.p + 2]))
                          : make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    float dir[3], dor[3];
    sh_dir(p, make_float3(campos[0], campos[1], campos[2]), dir, dor);
    uint8_t clamp_bits = 0;
    float rgb[3];
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
        const float val = sh_channel(D, sh + ch, dir[0], dir[1], dir[2]);
        if (val < 0.f) clamp_bits |= (uint8_t)(1u << ch);
        rgb[ch] = val < 0.f ? 0.f : val;
    }
    // view depth recomputed exactly as the preprocess forms it (same operations, same order)
    // instead of read back from the GRec line: that read fetched a whole 64-B line per Gaussian
    const float z = xf_point43(p, load_mat4(viewmatrix)).z;
    reinterpret_cast<float4 *>(gs.rec + i)[2] = make_float4(rgb[0], rgb[1], rgb[2], 1.f / z);
    gs.clamped[i] = clamp_bits;
}

// GSR_COLOR_BLOCKS > 0: a persistent grid of that many blocks walks the row blocks (so the pass
// can be held to part of the chip while latency-bound work runs beside it).  Each wave owns its
// LDS tile (no block-wide barrier between row blocks).
template <bool kCut, int kWaves>
__global__ __launch_bounds__(kWaves * kWave) void preprocess_color_kernel(int P, int D, const float *__restrict__ means3D,
                                                                          const float *__restrict__ shs,
                                                                          const float *__restrict__ campos,
                                                                          const float *__restrict__ viewmatrix,
                                                                          const int *__restrict__ radii, GeomState gs,
                                                                          int nvb, CutRef cut) {
    GSR_KS(kKsColor);
    __shared__ float4 s_sh[kWaves * kWave * kColorPitch];
    __shared__ int4 s_idx[kCut ? kWaves * kWave : 1];
    if (GSR_COLOR_PF) {
        ShRows cur, nxt;
        int vb = blockIdx.x;
        if (vb < nvb) color_fetch<kCut>(vb, cur, P, D, shs, radii, cut, s_idx);
        for (; vb < nvb; vb += gridDim.x) {
            const int vn = vb + (int)gridDim.x;
            if (vn < nvb) color_fetch<kCut>(vn, nxt, P, D, shs, radii, cut, s_idx);
            color_finish<kCut>(vb, cur, s_sh, P, D, means3D, campos, viewmatrix, gs);
            cur = nxt;
        }
    } else {
        for (int vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
            ShRows cur;
            color_fetch<kCut>(vb, cur, P, D, shs, radii, cut, s_idx);
            color_finish<kCut>(vb, cur, s_sh, P, D, means3D, campos, viewmatrix, gs);
        }
    }
}

bool cut_fusable(const GaussianInputs &in) {
    return in.shs && !in.colors_precomp && in.M == 16 && (reinterpret_cast<uintptr_t>(in.shs) % 16 == 0) &&
           in.scales && in.rotations && !in.cov3D_precomp && (reinterpret_cast<uintptr_t>(in.rotations) % 16 == 0) &&
           !in.raw;
}

bool color_split_supported(const GaussianInputs &in) {
    return in.shs && !in.colors_precomp && in.M == 16 && (reinterpret_cast<uintptr_t>(in.shs) % 16 == 0);
}

void launch_preprocess(const GaussianInputs &in, const Camera &cam, const GeomState &gs, int *radii,
                       hipStream_t s, bool split_color) {
    if (in.P == 0) return;
    const int blocks = (in.P + 255) / 256;
    const bool vec = in.shs && (in.M * 3) % 4 == 0 && (reinterpret_cast<uintptr_t>(in.shs) % 16 == 0) && in.M >= 16;
#define GSR_PRE_ARGS                                                                                                 \
    in.P, in.D, in.M, in.means3D, in.scales, in.scale_modifier, in.rotations, in.opacities, in.shs, in.colors_precomp, \
        in.cov3D_precomp, cam.view, cam.proj, cam.campos, cam.W, cam.H, cam.tanx, cam.tany, cam.fx, cam.fy, cam.gx,   \
        cam.gy, gs, radii, in.raw, in.cut
    if (split_color)
        hipLaunchKernelGGL((preprocess_kernel<true, true>), dim3(blocks), dim3(256), 0, s, GSR_PRE_ARGS);
    else if (vec)
        hipLaunchKernelGGL((preprocess_kernel<true, false>), dim3(blocks), dim3(256), 0, s, GSR_PRE_ARGS);
    else
        hipLaunchKernelGGL((preprocess_kernel<false, false>), dim3(blocks), dim3(256), 0, s, GSR_PRE_ARGS);
#undef GSR_PRE_ARGS
}

// blocks < 0: a full grid of 4-wave blocks (52 KiB, three per CU), for a pass forked after the depth
// sort beside the binning: config 5's 7.46M-row pass 1.16 -> 1.06 ms (r05f, vlibs cw4).  Beside the
// sort itself they take the CUs its passes need (config 5: sort 0.36 -> 1.05 ms, r05g), so a pass
// forked before the sort (blocks == 0) or a persistent grid (blocks > 0) runs 8-wave blocks.
void launch_preprocess_color(const GaussianInputs &in, const Camera &cam, const GeomState &gs, const int *radii,
                             hipStream_t s, int blocks) {
    if (in.P == 0) return;
    const bool four = blocks < 0;
    if (blocks < 0) blocks = 0;
    const int cap = blocks > 0 ? blocks : GSR_COLOR_BLOCKS;
    const auto go = [&](auto kw) {
        constexpr int kW = decltype(kw)::value, kT = kW * kWave;
        const int nvb = (in.P + kT - 1) / kT;
        const int grid = cap > 0 ? std::min(nvb, cap) : nvb;
        if (in.cut.ri)
            hipLaunchKernelGGL((preprocess_color_kernel<true, kW>), dim3(grid), dim3(kT), 0, s, in.P, in.D, in.means3D,
                               in.shs, cam.campos, cam.view, radii, gs, nvb, in.cut);
        else
            hipLaunchKernelGGL((preprocess_color_kernel<false, kW>), dim3(grid), dim3(kT), 0, s, in.P, in.D,
                               in.means3D, in.shs, cam.campos, cam.view, radii, gs, nvb, in.cut);
    };
    if (four && cap == 0) go(std::integral_constant<int, 4>{});
    else if (in.cut.ri) go(std::integral_constant<int, GSR_COLOR_WAVES_CUT>{});
    else go(std::integral_constant<int, kColorWaves>{});
}

__global__ __launch_bounds__(256) void mark_visible_kernel(int P, const float *__restrict__ means3D,
                                                           const float *__restrict__ viewmatrix,
                                                           uint8_t *__restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const Mat4 V = load_mat4(viewmatrix);
    const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    present[i] = xf_point43(p, V).z > 0.2f ? 1 : 0;
}

void launch_mark_visible(int P, const float *means3D, const float *view, uint8_t *present, hipStream_t s) {
    if (P == 0) return;
    hipLaunchKernelGGL(mark_visible_kernel, dim3((P + 255) / 256), dim3(256), 0, s, P, means3D, view, present);
}

GSR_KSTAMP_READER(kstamp_read_preprocess)

}  // namespace gsr
