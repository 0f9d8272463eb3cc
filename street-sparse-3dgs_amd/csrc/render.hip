// render.hip -- tile blending forward and backward.
//
// MI355X mapping: one 64-lane wave owns one 16x16 tile; lane l holds pixels
// (l & 15, (l >> 4) + 4k), k = 0..3.  A workgroup is a single wave, so the batch staging
// through LDS needs no workgroup barrier cost beyond the wave's own s_waitcnt, and the
// tile-wide early exit of the upstream design (__syncthreads_count) becomes a wave vote.
//
// Backward: upstream accumulates ~10 float atomics per (pixel, Gaussian) pair.  On gfx950
// float atomics execute at the memory side (MI355X_MICROARCH.md, Global float atomics) and
// 64 lanes adding into one address serialise, so instead every wave reduces each instance's
// 10 gradient terms across its 256 pixels with DPP (row_ror + row_bcast, no LDS), parks the
// sum in lane j of the batch (lane-select), and stores one 40-B record per tile instance
// with plain stores at the instance's unsorted (Gaussian-major) index.  backward.hip then sums
// each Gaussian's contiguous run of records: no atomics, bitwise reproducible.
#include "gsr_launch.h"

namespace gsr {

// ------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void render_fwd_kernel(
    const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H, int gx,
    const float2 *__restrict__ xy, const float4 *__restrict__ conic_o, const float4 *__restrict__ rgbd,
    const float *__restrict__ bg, float *__restrict__ out_color, float *__restrict__ out_invd,
    float *__restrict__ final_T, uint32_t *__restrict__ n_contrib) {
    __shared__ float4 s_pa[kWave];  // x, y, conic.a, conic.b
    __shared__ float2 s_pb[kWave];  // conic.c, opacity
    __shared__ float4 s_c[kWave];   // r, g, b, 1/depth

    const int tile = blockIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const int py0 = ty * kTile + (lane >> 4);
    const float pfx = (float)px;

    float T[kPixPerLane], C0[kPixPerLane], C1[kPixPerLane], C2[kPixPerLane], ID[kPixPerLane];
    uint32_t last[kPixPerLane];
    bool done[kPixPerLane];
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        T[k] = 1.f; C0[k] = C1[k] = C2[k] = ID[k] = 0.f; last[k] = 0;
        done[k] = !(px < W && py0 + 4 * k < H);
    }
    const uint2 rg = ranges[tile];
    for (uint32_t base = rg.x; base < rg.y; base += kWave) {
        const bool lane_done = done[0] && done[1] && done[2] && done[3];
        if (__all(lane_done)) break;
        const uint32_t n = min((uint32_t)kWave, rg.y - base);
        if ((uint32_t)lane < n) {
            const uint32_t g = point_list[base + lane];
            const float2 p = xy[g];
            const float4 co = conic_o[g];
            s_pa[lane] = make_float4(p.x, p.y, co.x, co.y);
            s_pb[lane] = make_float2(co.z, co.w);
            s_c[lane] = rgbd[g];
        }
        __syncthreads();
        for (uint32_t j = 0; j < n; j++) {
            const float4 a = s_pa[j];
            const float2 b = s_pb[j];
            const uint32_t contributor = base - rg.x + j + 1;
            const float dx = a.x - pfx;
            const float adxdx = a.z * dx * dx;
            const float bdx = a.w * dx;
#pragma unroll
            for (int k = 0; k < kPixPerLane; k++) {
                if (done[k]) continue;
                const float dy = a.y - (float)(py0 + 4 * k);
                const float power = -0.5f * (adxdx + b.x * dy * dy) - bdx * dy;
                if (power > 0.0f) continue;
                const float alpha = fmin_(0.99f, b.y * expf(power));
                if (alpha < 1.0f / 255.0f) continue;
                const float test_T = T[k] * (1.f - alpha);
                if (test_T < 0.0001f) { done[k] = true; continue; }
                const float w = alpha * T[k];
                const float4 c = s_c[j];
                C0[k] += c.x * w;
                C1[k] += c.y * w;
                C2[k] += c.z * w;
                ID[k] += c.w * w;
                T[k] = test_T;
                last[k] = contributor;
            }
        }
        __syncthreads();
    }
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        const int py = py0 + 4 * k;
        if (px < W && py < H) {
            const int pix = py * W + px;
            final_T[pix] = T[k];
            n_contrib[pix] = last[k];
            out_color[pix] = C0[k] + T[k] * b0;
            out_color[H * W + pix] = C1[k] + T[k] * b1;
            out_color[2 * H * W + pix] = C2[k] + T[k] * b2;
            if (out_invd) out_invd[pix] = ID[k];
        }
    }
}

void launch_render_fwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const float *bg, float *out_color, float *out_invdepth, hipStream_t s) {
    const int T = cam.gx * cam.gy;
    if (T == 0) return;
    hipLaunchKernelGGL(render_fwd_kernel, dim3(T), dim3(kWave), 0, s, is.ranges, bs.point_list, cam.W, cam.H, cam.gx,
                       gs.xy, gs.conic_o, gs.rgbd, bg, out_color, out_invdepth, is.final_T, is.n_contrib);
}

// ------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------
template <bool kDepth>
__global__ __launch_bounds__(64) void render_bwd_kernel(
    const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H, int gx, int gy,
    const float2 *__restrict__ xy, const float4 *__restrict__ conic_o, const float4 *__restrict__ rgbd,
    const int *__restrict__ radii, const uint32_t *__restrict__ offsets, const float *__restrict__ bg,
    const float *__restrict__ final_Ts, const uint32_t *__restrict__ n_contrib, const float *__restrict__ dL_dpix,
    const float *__restrict__ dL_dinvd, BwdScratch sc) {
    __shared__ float4 s_pa[kWave];
    __shared__ float2 s_pb[kWave];
    __shared__ float4 s_c[kWave];

    const int tile = blockIdx.x;
    const int tx = tile % gx, ty = tile / gx;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const int py0 = ty * kTile + (lane >> 4);
    const float pfx = (float)px;
    const float ddelx_dx = 0.5f * (float)W, ddely_dy = 0.5f * (float)H;
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];

    float T[kPixPerLane], Tf[kPixPerLane], dp0[kPixPerLane], dp1[kPixPerLane], dp2[kPixPerLane], did[kPixPerLane];
    float acc0[kPixPerLane], acc1[kPixPerLane], acc2[kPixPerLane], acci[kPixPerLane];
    float la[kPixPerLane], lc0[kPixPerLane], lc1[kPixPerLane], lc2[kPixPerLane], lid[kPixPerLane];
    float bgdot[kPixPerLane];
    uint32_t last[kPixPerLane];
    uint32_t mylast = 0;
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        const int py = py0 + 4 * k;
        const bool inside = px < W && py < H;
        const int pix = py * W + px;
        Tf[k] = inside ? final_Ts[pix] : 0.f;
        T[k] = Tf[k];
        last[k] = inside ? n_contrib[pix] : 0u;
        dp0[k] = inside ? dL_dpix[pix] : 0.f;
        dp1[k] = inside ? dL_dpix[H * W + pix] : 0.f;
        dp2[k] = inside ? dL_dpix[2 * H * W + pix] : 0.f;
        did[k] = (kDepth && inside) ? dL_dinvd[pix] : 0.f;
        acc0[k] = acc1[k] = acc2[k] = acci[k] = 0.f;
        la[k] = lc0[k] = lc1[k] = lc2[k] = lid[k] = 0.f;
        bgdot[k] = b0 * dp0[k] + b1 * dp1[k] + b2 * dp2[k];
        mylast = last[k] > mylast ? last[k] : mylast;
    }
    const uint2 rg = ranges[tile];
    const uint32_t len = rg.y - rg.x;
    const uint32_t maxlast = wave_max_u32(mylast);

    // unsorted (Gaussian-major) index of the instance of `g` that lives in this tile
    auto unsorted_index = [&](uint32_t g) -> uint32_t {
        const float2 p = xy[g];
        const Rect r = get_rect(p.x, p.y, radii[g], gx, gy);
        const uint32_t off = g == 0 ? 0u : offsets[g - 1];
        return off + (uint32_t)((ty - r.y0) * (r.x1 - r.x0) + (tx - r.x0));
    };

    // instances behind every pixel's last contributor receive zero gradient
    for (uint32_t pos = maxlast + lane; pos < len; pos += kWave) {
        const uint32_t u = unsorted_index(point_list[rg.x + pos]);
        sc.ga[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        sc.gb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        sc.gc[u] = make_float2(0.f, 0.f);
    }

    for (int hi = (int)maxlast; hi > 0; hi -= kWave) {
        const int n = hi < kWave ? hi : kWave;
        uint32_t my_u = 0;
        if (lane < n) {
            const uint32_t g = point_list[rg.x + (uint32_t)(hi - 1 - lane)];
            const float2 p = xy[g];
            const float4 co = conic_o[g];
            s_pa[lane] = make_float4(p.x, p.y, co.x, co.y);
            s_pb[lane] = make_float2(co.z, co.w);
            s_c[lane] = rgbd[g];
            my_u = unsorted_index(g);
        }
        __syncthreads();
        float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f, r4 = 0.f, r5 = 0.f, r6 = 0.f, r7 = 0.f, r8 = 0.f, r9 = 0.f;
        for (int j = 0; j < n; j++) {
            const uint32_t pos = (uint32_t)(hi - 1 - j);
            const float4 a = s_pa[j];
            const float2 b = s_pb[j];
            const float4 c = s_c[j];
            const float dx = a.x - pfx;
            const float adxdx = a.z * dx * dx;
            const float bdx = a.w * dx;
            float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f, q4 = 0.f, q5 = 0.f, q6 = 0.f, q7 = 0.f, q8 = 0.f, q9 = 0.f;
            bool any = false;
#pragma unroll
            for (int k = 0; k < kPixPerLane; k++) {
                if (pos >= last[k]) continue;
                const float dy = a.y - (float)(py0 + 4 * k);
                const float power = -0.5f * (adxdx + b.x * dy * dy) - bdx * dy;
                if (power > 0.0f) continue;
                const float G = expf(power);
                const float alpha = fmin_(0.99f, b.y * G);
                if (alpha < 1.0f / 255.0f) continue;
                any = true;
                T[k] = T[k] / (1.f - alpha);
                const float dchannel = alpha * T[k];
                float dL_dalpha = 0.f;
                acc0[k] = la[k] * lc0[k] + (1.f - la[k]) * acc0[k];
                lc0[k] = c.x;
                dL_dalpha += (c.x - acc0[k]) * dp0[k];
                q6 += dchannel * dp0[k];
                acc1[k] = la[k] * lc1[k] + (1.f - la[k]) * acc1[k];
                lc1[k] = c.y;
                dL_dalpha += (c.y - acc1[k]) * dp1[k];
                q7 += dchannel * dp1[k];
                acc2[k] = la[k] * lc2[k] + (1.f - la[k]) * acc2[k];
                lc2[k] = c.z;
                dL_dalpha += (c.z - acc2[k]) * dp2[k];
                q8 += dchannel * dp2[k];
                if (kDepth) {
                    acci[k] = la[k] * lid[k] + (1.f - la[k]) * acci[k];
                    lid[k] = c.w;
                    dL_dalpha += (c.w - acci[k]) * did[k];
                    q9 += dchannel * did[k];
                }
                dL_dalpha *= T[k];
                la[k] = alpha;
                dL_dalpha += (-Tf[k] / (1.f - alpha)) * bgdot[k];
                const float dL_dG = b.y * dL_dalpha;
                const float gdx = G * dx, gdy = G * dy;
                const float dG_ddelx = -gdx * a.z - gdy * a.w;
                const float dG_ddely = -gdy * b.x - gdx * a.w;
                q0 += dL_dG * dG_ddelx * ddelx_dx;
                q1 += dL_dG * dG_ddely * ddely_dy;
                q2 += -0.5f * gdx * dx * dL_dG;
                q3 += -0.5f * gdx * dy * dL_dG;
                q4 += -0.5f * gdy * dy * dL_dG;
                q5 += G * dL_dalpha;
            }
            if (__any(any)) {
                const bool mine = lane == j;  // park instance j's sums in lane j
                { const float t = wave_sum(q0); r0 = mine ? t : r0; }
                { const float t = wave_sum(q1); r1 = mine ? t : r1; }
                { const float t = wave_sum(q2); r2 = mine ? t : r2; }
                { const float t = wave_sum(q3); r3 = mine ? t : r3; }
                { const float t = wave_sum(q4); r4 = mine ? t : r4; }
                { const float t = wave_sum(q5); r5 = mine ? t : r5; }
                { const float t = wave_sum(q6); r6 = mine ? t : r6; }
                { const float t = wave_sum(q7); r7 = mine ? t : r7; }
                { const float t = wave_sum(q8); r8 = mine ? t : r8; }
                if (kDepth)
                {
                    const float t = wave_sum(q9);
                    r9 = mine ? t : r9;
                }
            }
        }
        if (lane < n) {
            sc.ga[my_u] = make_float4(r0, r1, r2, r3);
            sc.gb[my_u] = make_float4(r4, r5, r6, r7);
            sc.gc[my_u] = make_float2(r8, r9);
        }
        __syncthreads();
    }
}

void launch_render_bwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const int *radii, const float *bg, const float *dL_dpix, const float *dL_dinvdepth,
                       const BwdScratch &sc, hipStream_t s) {
    const int T = cam.gx * cam.gy;
    if (T == 0) return;
    if (dL_dinvdepth)
        hipLaunchKernelGGL(render_bwd_kernel<true>, dim3(T), dim3(kWave), 0, s, is.ranges, bs.point_list, cam.W,
                           cam.H, cam.gx, cam.gy, gs.xy, gs.conic_o, gs.rgbd, radii, gs.offsets, bg, is.final_T,
                           is.n_contrib, dL_dpix, dL_dinvdepth, sc);
    else
        hipLaunchKernelGGL(render_bwd_kernel<false>, dim3(T), dim3(kWave), 0, s, is.ranges, bs.point_list, cam.W,
                           cam.H, cam.gx, cam.gy, gs.xy, gs.conic_o, gs.rgbd, radii, gs.offsets, bg, is.final_T,
                           is.n_contrib, dL_dpix, dL_dinvdepth, sc);
}

}  // namespace gsr
