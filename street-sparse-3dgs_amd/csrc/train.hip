// train.hip -- the device work of one train_single.py iteration around the rasterizer
// (8(f) rows 1-2): fused L1 + SSIM loss forward/backward, the fused sparse
// Adam step over all six Gaussian parameter groups, and the densification statistics.
//
// Loss.  The reference evaluates SSIM with five depthwise 11x11 conv2d passes
// (utils/loss_utils.py:44-63) plus elementwise torch ops and autograd replays them in backward.
// Here one launch computes both means (L1 and SSIM) from one read of the two images: a 64x16
// output tile per workgroup stages its 74x26 input halo in LDS, runs the separable Gaussian
// window as a horizontal then a vertical pass over the five moments (x, y, x^2, y^2, xy), and
// reduces per block (fixed-order second pass, so the loss is deterministic).  The backward
// recomputes the moments over a 2-radius halo instead of storing per-pixel partials: it reads
// the two images once and writes the gradient once, with every intermediate in LDS.
//
// Adam.  OurAdam (scene/OurAdam.py:249-337) gathers the `relevant` rows of every group,
// updates them and scatters them back, one torch op at a time, after a host-synchronising
// nonzero().  Here one launch walks all six groups' (param, grad, m, v) arrays once, testing
// relevance (opacity grad != 0) per row on the device.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <string>

#include "../../include/gsr.h"
#include "../../include/gsr_train.h"
#include "gsr_launch.h"

namespace gsr {
namespace {

constexpr int kR = 5;  // window radius: 11 taps
constexpr int kTW = 64;
constexpr int kTH = 16;
constexpr int kLossThreads = 256;
constexpr float kC1 = 0.01f * 0.01f;  // utils/loss_utils.py:54-55 (C1 = 0.01^2, C2 = 0.03^2)
constexpr float kC2 = 0.03f * 0.03f;

struct Window {
    float w[2 * kR + 1];
};

// utils/loss_utils.py:24-26: exp(-(x - 5)^2 / (2 sigma^2)) as fp32, normalised by its fp32 sum.
Window ssim_window() {
    Window win;
    float sum = 0.f;
    for (int i = 0; i < 2 * kR + 1; i++) {
        win.w[i] = (float)std::exp(-(double)((i - kR) * (i - kR)) / (2.0 * 1.5 * 1.5));
        sum += win.w[i];
    }
    for (int i = 0; i < 2 * kR + 1; i++) win.w[i] /= sum;
    return win;
}

struct Moments {
    float m1, m2, a11, a22, a12;
};

// SSIM map value at one pixel from its windowed moments (utils/loss_utils.py:44-58 op order).
__device__ __forceinline__ float ssim_value(const Moments &s) {
    const float mu1_sq = s.m1 * s.m1, mu2_sq = s.m2 * s.m2, mu12 = s.m1 * s.m2;
    const float s1 = s.a11 - mu1_sq, s2 = s.a22 - mu2_sq, s12 = s.a12 - mu12;
    return ((2.f * mu12 + kC1) * (2.f * s12 + kC2)) / ((mu1_sq + mu2_sq + kC1) * (s1 + s2 + kC2));
}

// dS/d(mu1), dS/d(E[x^2]), dS/d(E[xy]) at one pixel, mu1 derivative including its appearance in
// sigma1^2 = E[x^2] - mu1^2 and sigma12 = E[xy] - mu1 mu2.
__device__ __forceinline__ void ssim_partials(const Moments &s, float &a, float &b, float &c) {
    const float mu1_sq = s.m1 * s.m1, mu2_sq = s.m2 * s.m2, mu12 = s.m1 * s.m2;
    const float s1 = s.a11 - mu1_sq, s2 = s.a22 - mu2_sq, s12 = s.a12 - mu12;
    const float n1 = 2.f * mu12 + kC1, n2 = 2.f * s12 + kC2;
    const float d1 = mu1_sq + mu2_sq + kC1, d2 = s1 + s2 + kC2;
    // one division: S / d2 = S d1 inv and S / d1 = S d2 inv
    const float inv = 1.f / (d1 * d2);
    const float S = n1 * n2 * inv;
    const float Sinv = S * inv;
    const float ds1 = -Sinv * d1;
    const float ds12 = 2.f * n1 * inv;
    const float dmu = 2.f * s.m2 * n2 * inv - 2.f * s.m1 * (Sinv * d2);
    a = dmu - 2.f * s.m1 * ds1 - s.m2 * ds12;
    b = ds1;
    c = ds12;
}

// LDS layout: every staged map is row-major with an odd row pitch (an odd number of floats), so
// the passes below, whose 32-lane halves walk down consecutive rows of a map, touch 32
// different banks.
constexpr int odd_pitch(int cols) { return cols | 1; }

// Load a rows x cols region of one plane with origin (oy, ox), zero outside the image, into a
// map of row pitch `pitch`.
__device__ __forceinline__ void load_halo(const float *__restrict__ x, const float *__restrict__ y, int H, int W,
                                          int oy, int ox, int rows, int cols, int pitch, float *sx, float *sy) {
    for (int i = threadIdx.x; i < rows * cols; i += kLossThreads) {
        const int r = i / cols, c = i - r * cols;
        const int gy = oy + r, gx = ox + c;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        const size_t o = (size_t)gy * W + gx;
        sx[r * pitch + c] = in ? x[o] : 0.f;
        sy[r * pitch + c] = in ? y[o] : 0.f;
    }
}

// Horizontal pass of the five moments: out[q][r][c] = sum_j w_j f_q(in[r][c + j]).  A task is a
// kS-column segment of one row: kS + 10 inputs are loaded once into registers, so LDS reads drop
// from 22 per output to (2 kS + 20) / kS.  Consecutive tasks (lanes) take consecutive rows.
template <int kS>
__device__ __forceinline__ void hpass5(const float *sx, const float *sy, int rows, int in_cols, int in_pitch,
                                       int out_cols, int out_pitch, int plane, const Window &win, float *hs) {
    const int segs = (out_cols + kS - 1) / kS;
    for (int task = threadIdx.x; task < rows * segs; task += kLossThreads) {
        const int s = task / rows, r = task - s * rows, c0 = s * kS;
        const float *px = sx + r * in_pitch + c0, *py = sy + r * in_pitch + c0;
        float u[kS + 2 * kR], v[kS + 2 * kR];
#pragma unroll
        for (int k = 0; k < kS + 2 * kR; k++) {
            const bool ok = c0 + k < in_cols;
            u[k] = ok ? px[k] : 0.f;
            v[k] = ok ? py[k] : 0.f;
        }
#pragma unroll
        for (int o = 0; o < kS; o++) {
            float m1 = 0.f, m2 = 0.f, a11 = 0.f, a22 = 0.f, a12 = 0.f;
#pragma unroll
            for (int j = 0; j < 2 * kR + 1; j++) {
                const float w = win.w[j];
                m1 = fmaf(w, u[o + j], m1);
                m2 = fmaf(w, v[o + j], m2);
                a11 = fmaf(w, u[o + j] * u[o + j], a11);
                a22 = fmaf(w, v[o + j] * v[o + j], a22);
                a12 = fmaf(w, u[o + j] * v[o + j], a12);
            }
            if (c0 + o < out_cols) {
                const int i = r * out_pitch + c0 + o;
                hs[i] = m1;
                hs[plane + i] = m2;
                hs[2 * plane + i] = a11;
                hs[3 * plane + i] = a22;
                hs[4 * plane + i] = a12;
            }
        }
    }
}

// Vertical pass for the 64 x 16 output tile: lane column c = tid & 63 and four consecutive rows
// r0..r0+3 per thread, a 14-row sliding window per quantity.
template <int NQ>
__device__ __forceinline__ void vpass_tile(const float *hs, int pitch, int plane, const Window &win,
                                           float (&acc)[NQ][4]) {
    const int c = threadIdx.x & 63, r0 = (threadIdx.x >> 6) * 4;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
#pragma unroll
        for (int k = 0; k < 4; k++) acc[q][k] = 0.f;
        const float *h = hs + q * plane + r0 * pitch + c;
#pragma unroll
        for (int t = 0; t < 2 * kR + 4; t++) {
            const float v = h[t * pitch];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int j = t - k;
                if (j >= 0 && j <= 2 * kR) acc[q][k] = fmaf(win.w[j], v, acc[q][k]);
            }
        }
    }
}

template <int kThreads = kLossThreads>
__device__ __forceinline__ float block_sum(float v, float *red) {
    v = wave_sum(v);
    const int wv = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[wv] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kThreads / 64; k++) s += red[k];
    return s;
}

constexpr int kFwdRH = kTH + 2 * kR, kFwdRW = kTW + 2 * kR;  // 26 x 74 input halo
constexpr int kFwdIP = odd_pitch(kFwdRW), kFwdHP = odd_pitch(kTW);
constexpr size_t kFwdLds = sizeof(float) * (2 * kFwdRH * kFwdIP + 5 * kFwdRH * kFwdHP + 8);

__global__ __launch_bounds__(kLossThreads) void l1_ssim_fwd_kernel(const float *__restrict__ x,
                                                                    const float *__restrict__ y, int H, int W,
                                                                    Window win, float2 *__restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *sx = reinterpret_cast<float *>(smem);
    float *sy = sx + kFwdRH * kFwdIP;
    float *hs = sy + kFwdRH * kFwdIP;
    float *red = hs + 5 * kFwdRH * kFwdHP;
    const size_t plane_off = (size_t)blockIdx.z * H * W;
    x += plane_off;
    y += plane_off;
    const int ox = blockIdx.x * kTW, oy = blockIdx.y * kTH;

    load_halo(x, y, H, W, oy - kR, ox - kR, kFwdRH, kFwdRW, kFwdIP, sx, sy);
    __syncthreads();
#ifndef GSR_SSIM_FWD_SEG
#define GSR_SSIM_FWD_SEG 8
#endif
    hpass5<GSR_SSIM_FWD_SEG>(sx, sy, kFwdRH, kFwdRW, kFwdIP, kTW, kFwdHP, kFwdRH * kFwdHP, win, hs);  // 26 x 8 tasks
    __syncthreads();
    float acc[5][4];
    vpass_tile<5>(hs, kFwdHP, kFwdRH * kFwdHP, win, acc);

    const int c = threadIdx.x & 63, r0 = (threadIdx.x >> 6) * 4;
    float l1 = 0.f, ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int gy = oy + r0 + k, gx = ox + c;
        if (gy < H && gx < W) {
            const Moments m{acc[0][k], acc[1][k], acc[2][k], acc[3][k], acc[4][k]};
            ss += ssim_value(m);
            const int li = (r0 + k + kR) * kFwdIP + c + kR;
            l1 += fabsf(sx[li] - sy[li]);
        }
    }
    l1 = block_sum(l1, red);
    ss = block_sum(ss, red + 4);
    if (threadIdx.x == 0) {
        const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
        partials[b] = make_float2(l1, ss);
    }
}

// fixed-order fp64 reduction of the per-block (L1, SSIM) sums (1024 threads)
__device__ __forceinline__ void loss_finalize_body(const float2 *__restrict__ partials, int n, double inv_n,
                                                   float *__restrict__ out, float w_l1, float w_ssim) {
    __shared__ double s1[1024], s2[1024];
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < n; i += 1024) {
        a += partials[i].x;
        b += partials[i].y;
    }
    s1[threadIdx.x] = a;
    s2[threadIdx.x] = b;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s1[threadIdx.x] += s1[threadIdx.x + w];
            s2[threadIdx.x] += s2[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = (float)(s1[0] * inv_n);
        out[1] = (float)(s2[0] * inv_n);
        // photo loss (train_single.py:121-123) in torch's fp32 op order: (1-l) * L1 + l * (1 - SSIM)
        if (w_l1 >= 0.f)
            out[2] = __fadd_rn(__fmul_rn(w_l1, out[0]), __fmul_rn(w_ssim, __fsub_rn(1.f, out[1])));
    }
}

__global__ __launch_bounds__(1024) void loss_finalize_kernel(const float2 *__restrict__ partials, int n, double inv_n,
                                                             float *__restrict__ out, float w_l1,
                                                             float w_ssim) {
    loss_finalize_body(partials, n, inv_n, out, w_l1, w_ssim);
}

constexpr int kBwdIH = kTH + 4 * kR, kBwdIW = kTW + 4 * kR;  // 36 x 84 inputs
constexpr int kBwdSH = kTH + 2 * kR, kBwdSW = kTW + 2 * kR;  // 26 x 74 SSIM-map positions
constexpr int kBwdIP = odd_pitch(kBwdIW), kBwdSP = odd_pitch(kBwdSW), kBwdTP = odd_pitch(kTW);
constexpr int kBwdVS = 9;  // rows per task of the vertical stats pass; its last task reads one row past the moments
constexpr size_t kBwdLds = sizeof(float) * (2 * kBwdIH * kBwdIP + 5 * kBwdIH * kBwdSP + kBwdSP);
static_assert(3 * kBwdVS - 1 + 2 * kR <= kBwdIH, "vertical stats pass reads at most one row past the moments");
static_assert(3 * kBwdSH * kBwdSP <= 2 * kBwdIH * kBwdIP, "a/b/c maps alias the input halo");
static_assert(3 * kBwdSH * kBwdTP <= 5 * kBwdIH * kBwdSP, "second horizontal pass aliases the moments");

// dx = (dout[0] sign(x - y) + dout[1] G) / n from the field l1_ssim_grad_kernel<true> stored.
// Upstream (dL/dL1, dL/dSSIM) scaled by 1/n: from the 2-vector dout, or (photo loss, w_l1 >= 0)
// from the scalar dL/dloss as torch's backward of (1-l) * L1 + l * (1 - SSIM) forms them.
__device__ __forceinline__ float2 loss_upstream(const float *dout, float inv_n, float w_l1, float w_ssim) {
    if (w_l1 >= 0.f) return make_float2((w_l1 * dout[0]) * inv_n, (-(w_ssim * dout[0])) * inv_n);
    return make_float2(dout[0] * inv_n, dout[1] * inv_n);
}

// The photometric loss gradient at one pixel from its SSIM gradient field value G: upstream
// (L1, SSIM) weights up times (sign(x - y), G) -- the one expression every kernel that forms it uses
// (exposure_bwd_kernel, the native step's SSIM pass), so they agree bit for bit.
__device__ __forceinline__ float photo_value(float2 up, float x, float y, float G) {
    const float d = x - y;
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    return up.x * sgn + up.y * G;
}

// The native step's SSIM pass writes the photometric gradient itself instead of G (one != NULL):
// dL/dloss = *one (1), the loss weights and 1/n, times the alpha mask (NULL: none) as torch's
// multiply backward -- so the exposure backward reads one (3, H, W) field instead of the image,
// the target and G.
struct PhotoOut {
    const float *one;
    const float *alpha;
    float inv_n, w_l1, w_ssim;
};

// kMap = false: dx = dL/d(img) for the upstream 2-vector dout (the backward proper).
// kMap = true: the forward with the gradient field: per block the L1 and SSIM sums (as
// l1_ssim_fwd_kernel) and per pixel G = dSSIM_sum/dx (unscaled), from which the backward is the
// elementwise dx = (dout[0] sign(x - y) + dout[1] G) / n.  dL/dx is linear in dout, so a training
// step pays the halo recomputation once instead of twice.
template <bool kMap>
__global__ __launch_bounds__(kLossThreads) void l1_ssim_grad_kernel(const float *__restrict__ x,
                                                                     const float *__restrict__ y, int H, int W,
                                                                     Window win, const float *__restrict__ dout,
                                                                     float inv_n, float *__restrict__ dx,
                                                                     float2 *__restrict__ partials) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *sx = reinterpret_cast<float *>(smem);
    float *sy = sx + kBwdIH * kBwdIP;
    float *hs = sy + kBwdIH * kBwdIP;
    float *abc = sx;  // after the first horizontal pass the halo is dead
    float *h3 = hs;   // after the vertical pass the moments are dead
    const size_t plane_off = (size_t)blockIdx.z * H * W;
    x += plane_off;
    y += plane_off;
    dx += plane_off;
    const int ox = blockIdx.x * kTW, oy = blockIdx.y * kTH;
    const float g_l1 = kMap ? 0.f : dout[0] * inv_n, g_ssim = kMap ? 0.f : dout[1] * inv_n;
    float ss = 0.f;  // kMap: SSIM summed over this thread's interior positions
    constexpr int hp = kBwdIH * kBwdSP, sp = kBwdSH * kBwdSP, tp = kBwdSH * kBwdTP;

    load_halo(x, y, H, W, oy - 2 * kR, ox - 2 * kR, kBwdIH, kBwdIW, kBwdIP, sx, sy);
    __syncthreads();
    hpass5<12>(sx, sy, kBwdIH, kBwdIW, kBwdIP, kBwdSW, kBwdSP, hp, win, hs);  // 36 x 7 tasks
    __syncthreads();
    // Moments and dS/d(moment) at every SSIM-map position the tile's gradient reads; positions
    // outside the image have no SSIM term (zero).  A task is a kVS-row column segment: kVS + 10
    // rows of the five horizontal moments are read once.
    constexpr int kVS = kBwdVS, rsegs = (kBwdSH + kVS - 1) / kVS;  // 74 x 3 tasks
    for (int task = threadIdx.x; task < kBwdSW * rsegs; task += kLossThreads) {
        const int sg = task / kBwdSW, c = task - sg * kBwdSW, r0 = sg * kVS;
        float m[5][kVS];
#pragma unroll
        for (int q = 0; q < 5; q++) {
#pragma unroll
            for (int o = 0; o < kVS; o++) m[q][o] = 0.f;
            const float *h = hs + q * hp + r0 * kBwdSP + c;
#pragma unroll
            for (int t = 0; t < kVS + 2 * kR; t++) {
                const float v = h[t * kBwdSP];  // rows past kBwdIH only feed discarded outputs
#pragma unroll
                for (int o = 0; o < kVS; o++) {
                    const int j = t - o;
                    if (j >= 0 && j <= 2 * kR) m[q][o] = fmaf(win.w[j], v, m[q][o]);
                }
            }
        }
        const int gx = ox - kR + c;
        const bool col_in = gx >= 0 && gx < W;
#pragma unroll
        for (int o = 0; o < kVS; o++) {
            const int r = r0 + o, gy = oy - kR + r;
            float a, b, cc;
            ssim_partials(Moments{m[0][o], m[1][o], m[2][o], m[3][o], m[4][o]}, a, b, cc);
            const bool in = col_in && gy >= 0 && gy < H;
            if (kMap && in && r >= kR && r < kR + kTH && c >= kR && c < kR + kTW)
                ss += ssim_value(Moments{m[0][o], m[1][o], m[2][o], m[3][o], m[4][o]});
            if (r < kBwdSH) {
                const int i = r * kBwdSP + c;
                abc[i] = in ? a : 0.f;
                abc[sp + i] = in ? b : 0.f;
                abc[2 * sp + i] = in ? cc : 0.f;
            }
        }
    }
    __syncthreads();
    // Horizontal pass of the three partial maps (the window is symmetric: the transposed
    // convolution is the same correlation), 8-column segments, lanes down consecutive rows.
    constexpr int kHS = 8, csegs = kTW / kHS;  // 26 x 8 tasks
    for (int task = threadIdx.x; task < kBwdSH * csegs; task += kLossThreads) {
        const int sg = task / kBwdSH, r = task - sg * kBwdSH, c0 = sg * kHS;
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const float *p = abc + q * sp + r * kBwdSP + c0;
            float v[kHS + 2 * kR];
#pragma unroll
            for (int k = 0; k < kHS + 2 * kR; k++) v[k] = p[k];
#pragma unroll
            for (int o = 0; o < kHS; o++) {
                float sum = 0.f;
#pragma unroll
                for (int j = 0; j < 2 * kR + 1; j++) sum = fmaf(win.w[j], v[o + j], sum);
                h3[q * tp + r * kBwdTP + c0 + o] = sum;
            }
        }
    }
    __syncthreads();
    float acc[3][4];
    vpass_tile<3>(h3, kBwdTP, tp, win, acc);
    const int c = threadIdx.x & 63, r0 = (threadIdx.x >> 6) * 4;
    float l1 = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int gy = oy + r0 + k, gx = ox + c;
        if (gy < H && gx < W) {
            const size_t o = (size_t)gy * W + gx;
            const float xv = x[o], yv = y[o];
            const float d = xv - yv;
            const float G = acc[0][k] + 2.f * xv * acc[1][k] + yv * acc[2][k];
            if (kMap) {
                dx[o] = G;
                l1 += fabsf(d);
            } else {
                const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                dx[o] = g_l1 * sgn + g_ssim * G;
            }
        }
    }
    if (kMap) {
        float *red = sx;  // the a/b/c maps are dead after the second horizontal pass
        l1 = block_sum(l1, red);
        ss = block_sum(ss, red + 4);
        if (threadIdx.x == 0) {
            const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
            partials[b] = make_float2(l1, ss);
        }
    }
}

// Streaming form of l1_ssim_grad_kernel: a block owns a 64-column x seg-row strip of one plane
// and walks it top to bottom kStep rows at a time.  Each step stages kStep input rows, and each
// stage of the separable pipeline (horizontal moments -> vertical moments and dS/d(moment) ->
// horizontal pass of a/b/c -> vertical pass to G) advances by kStep rows, the vertical passes
// reading kRing-deep LDS rings.  Only the 2R-column side halo is recomputed (plus 4R rows per
// strip instead of per 16-row tile), LDS is 43 KiB instead of 79 KiB, and the next step's input
// rows are in flight while the current step computes.  Every value is formed with the same fmaf
// order as l1_ssim_grad_kernel, so G and dx are bit-identical to it.
constexpr int kStW = 64;
#ifndef GSR_SSIM_SEG_H
#define GSR_SSIM_SEG_H 0  // rows per strip; 0: chosen per image (stream_seg)
#endif
// GSR_SSIM_STEP: rows per step (4: 256 threads, 16-row rings, 40 KiB, four workgroups per CU; 8: 512
// threads, 32-row rings, 79 KiB, two per CU -- half the barriers per row and a thinner strip halo)
#ifndef GSR_SSIM_STEP
#define GSR_SSIM_STEP 4
#endif
static_assert(GSR_SSIM_STEP == 4 || GSR_SSIM_STEP == 8, "GSR_SSIM_STEP: 4 or 8");
constexpr int kStep = GSR_SSIM_STEP;
constexpr int kRing = kStep == 4 ? 16 : 32;
constexpr int kStThreads = kStep * 64;
constexpr int kStPerCU = kStep == 4 ? 4 : 2;  // resident workgroups per CU (LDS)
#ifndef GSR_SSIM_PF
#define GSR_SSIM_PF 1  // steps of input rows in flight; 2 measured no faster (r03j: train step 0.951-0.958 vs 0.949-0.958 ms)
#endif
static_assert(GSR_SSIM_PF == 1 || GSR_SSIM_PF == 2, "GSR_SSIM_PF: 1 or 2");
constexpr int kStIC = kStW + 4 * kR, kStMC = kStW + 2 * kR;  // 84 input, 74 SSIM-map columns
// Even pitches: the row-pair passes (2) and (4) move two adjacent columns per LDS instruction
// (8-B aligned float2), lanes on consecutive pairs, so they are conflict-free without padding.
constexpr int kStIP = kStIC, kStMP = kStMC, kStTP = kStW;
static_assert(kStIP % 2 == 0 && kStMP % 2 == 0 && kStTP % 2 == 0, "float2 rows");
constexpr int kStInElems = kStep * kStIC;
constexpr int kStInPer = (kStInElems + kStThreads - 1) / kStThreads;
constexpr int kStHSeg = kStMC / 2;  // horizontal-moment tasks per row (two columns each)
static_assert(kStMC % 2 == 0 && kStep * kStHSeg <= kStThreads, "one horizontal-moment task per thread");
static_assert(kStep % 2 == 0 && (kStep / 2) * kStMC <= kStThreads, "one task per thread");
static_assert(kRing >= 2 * kR + 1 + kStep - 1 && (kRing & (kRing - 1)) == 0, "ring holds a step's window rows");

// Workgroup barrier for LDS hand-offs only: drains this wave's LDS operations but not its global
// loads (__syncthreads waits for vmcnt(0) too), so the next step's rows stay in flight.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool kMap>
__global__ __launch_bounds__(kStThreads) void l1_ssim_stream_kernel(const float *__restrict__ x,
                                                                       const float *__restrict__ y, int H, int W,
                                                                       Window win, const float *__restrict__ dout,
                                                                       float inv_n, float *__restrict__ dx,
                                                                       float2 *__restrict__ partials, int seg,
                                                                       PhotoOut po) {
    // The staged input rows (read by (2)) and the a/b/c rows ((3) -> (4)) share one buffer: (3)
    // writes after the barrier that ends (2), and the next step's (1) writes after the barrier
    // that ends (4).  40.1 KiB in all, so four workgroups fit a CU.
    __shared__ __attribute__((aligned(16))) union {
        float in[2][kStep][kStIP];
        float abc[3][kStep][kStMP];
    } s_u;
    __shared__ __attribute__((aligned(16))) float s_hm[5][kRing][kStMP];
    __shared__ __attribute__((aligned(16))) float s_h3[3][kRing][kStTP];
    auto &s_in = s_u.in;
    auto &s_abc = s_u.abc;
    __shared__ float s_red[2 * kStThreads / 64];
    const size_t plane_off = (size_t)blockIdx.z * H * W;
    x += plane_off;
    y += plane_off;
    dx += plane_off;
    const int tid = threadIdx.x;
    const int cx = blockIdx.x * kStW, r0 = blockIdx.y * seg, r1 = min(r0 + seg, H);
    const float g_l1 = kMap ? 0.f : dout[0] * inv_n, g_ssim = kMap ? 0.f : dout[1] * inv_n;
    const float2 up = kMap && po.one ? loss_upstream(po.one, po.inv_n, po.w_l1, po.w_ssim) : make_float2(0.f, 0.f);
    const int nsteps = (r1 - r0 + 4 * kR + kStep - 1) / kStep;
    float l1 = 0.f, ss = 0.f;

    // Loads are unconditional (clamped coordinates) and the zero padding is applied when the
    // values are staged: no branch around a load, so the compiler does not drain the loads early.
    // GSR_SSIM_PF = 2: the input rows of the next two steps in flight (two register sets, the step
    // loop unrolled by two so each set stays in fixed registers).  Measured no faster than one step
    // ahead (profiles/r03j_ab_ssim_prefetch_negative.txt): a step's time is its four dependent LDS
    // stages and barriers, not the row loads.
    struct InRows {
        float px[kStInPer], py[kStInPer];
        bool pin[kStInPer];
    };
    const auto fetch = [&](InRows &f, int p0) {
#pragma unroll
        for (int k = 0; k < kStInPer; k++) {
            const int e = min(tid + k * kStThreads, kStInElems - 1);
            const int r = e / kStIC, c = e - r * kStIC;
            const int gy = p0 + r, gx = cx - 2 * kR + c;
            f.pin[k] = gy >= 0 && gy < H && gx >= 0 && gx < W;
            const size_t o = (size_t)min(max(gy, 0), H - 1) * W + min(max(gx, 0), W - 1);
            f.px[k] = x[o];
            f.py[k] = y[o];
        }
    };
    constexpr int kPf = GSR_SSIM_PF;
    InRows fa, fb;
    fetch(fa, r0 - 2 * kR);
    if (kPf == 2) fetch(fb, r0 - 2 * kR + kStep);

    const auto step = [&](int st, InRows &cur) {
        const int p0 = r0 - 2 * kR + kStep * st;  // first input row of this step
        // (1) stage input rows p0 .. p0 + kStep - 1 and start loading those kPf steps ahead
#pragma unroll
        for (int k = 0; k < kStInPer; k++) {
            const int e = tid + k * kStThreads;
            if (e < kStInElems) {
                const int r = e / kStIC, c = e - r * kStIC;
                s_in[0][r][c] = cur.pin[k] ? cur.px[k] : 0.f;
                s_in[1][r][c] = cur.pin[k] ? cur.py[k] : 0.f;
            }
        }
        // (5)'s output pixels: rows orow, orow + 1 of column ocol (tasks tid < 128)
        const int orow = p0 + 2 * ((tid >> 6) % (kStep / 2)) - 2 * kR, ocol = cx + (tid & 63);
        float xv[2], yv[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const size_t oo = (size_t)min(max(orow + k, 0), H - 1) * W + min(ocol, W - 1);
            xv[k] = x[oo];
            yv[k] = y[oo];
        }
        fetch(cur, p0 + kPf * kStep);  // unconditional (clamped): a branch here would make every wait a full drain
        lds_barrier();

        // (2) horizontal moments of the staged rows at the 74 map columns, two per task
        if (tid < kStep * kStHSeg) {
            const int r = tid / kStHSeg, c0 = 2 * (tid - r * kStHSeg);
            float u[2 + 2 * kR], v[2 + 2 * kR];
#pragma unroll
            for (int k = 0; k < 2 + 2 * kR; k += 2) {
                const float2 a = *reinterpret_cast<const float2 *>(&s_in[0][r][c0 + k]);
                const float2 b = *reinterpret_cast<const float2 *>(&s_in[1][r][c0 + k]);
                u[k] = a.x;
                u[k + 1] = a.y;
                v[k] = b.x;
                v[k + 1] = b.y;
            }
            const int ring = (p0 + r) & (kRing - 1);
            float m[5][2];
#pragma unroll
            for (int o = 0; o < 2; o++) {
                float m1 = 0.f, m2 = 0.f, a11 = 0.f, a22 = 0.f, a12 = 0.f;
#pragma unroll
                for (int j = 0; j < 2 * kR + 1; j++) {
                    const float w = win.w[j];
                    m1 = fmaf(w, u[o + j], m1);
                    m2 = fmaf(w, v[o + j], m2);
                    a11 = fmaf(w, u[o + j] * u[o + j], a11);
                    a22 = fmaf(w, v[o + j] * v[o + j], a22);
                    a12 = fmaf(w, u[o + j] * v[o + j], a12);
                }
                m[0][o] = m1;
                m[1][o] = m2;
                m[2][o] = a11;
                m[3][o] = a22;
                m[4][o] = a12;
            }
#pragma unroll
            for (int q = 0; q < 5; q++)
                *reinterpret_cast<float2 *>(&s_hm[q][ring][c0]) = make_float2(m[q][0], m[q][1]);
        }
        lds_barrier();

        // (3) vertical moments and dS/d(moment) at map rows p0 - R .. p0 + kStep - 1 - R, two rows
        // per task.  Rows above r0 - R read ring rows never written; (5) never reads them.
        if (tid < (kStep / 2) * kStMC) {
            const int pr = tid / kStMC, c = tid - pr * kStMC;
            const int qa = p0 + 2 * pr - kR;
            float m[5][2];
#pragma unroll
            for (int q = 0; q < 5; q++) {
                m[q][0] = m[q][1] = 0.f;
#pragma unroll
                for (int t = 0; t < 2 * kR + 2; t++) {
                    const float v = s_hm[q][(qa - kR + t) & (kRing - 1)][c];
#pragma unroll
                    for (int o = 0; o < 2; o++) {
                        const int j = t - o;
                        if (j >= 0 && j <= 2 * kR) m[q][o] = fmaf(win.w[j], v, m[q][o]);
                    }
                }
            }
            const int gx = cx - kR + c;
            const bool col_in = gx >= 0 && gx < W;
#pragma unroll
            for (int o = 0; o < 2; o++) {
                const int q = qa + o;
                const Moments mo{m[0][o], m[1][o], m[2][o], m[3][o], m[4][o]};
                float a, b, cc;
                ssim_partials(mo, a, b, cc);
                const bool in = col_in && q >= 0 && q < H;
                if (kMap && in && q >= r0 && q < r1 && c >= kR && c < kR + kStW) ss += ssim_value(mo);
                s_abc[0][2 * pr + o][c] = in ? a : 0.f;
                s_abc[1][2 * pr + o][c] = in ? b : 0.f;
                s_abc[2][2 * pr + o][c] = in ? cc : 0.f;
            }
        }
        lds_barrier();

        // (4) horizontal pass of a/b/c (symmetric window: the transposed convolution is the same
        // correlation), two adjacent output columns per task: 128 tasks, two waves
        if (tid < kStep * kStW / 2) {
            const int r = tid / (kStW / 2), c0 = 2 * (tid - r * (kStW / 2));
            const int ring = (p0 + r - kR) & (kRing - 1);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                float a[2 + 2 * kR];
#pragma unroll
                for (int k = 0; k < 2 + 2 * kR; k += 2) {
                    const float2 t = *reinterpret_cast<const float2 *>(&s_abc[q][r][c0 + k]);
                    a[k] = t.x;
                    a[k + 1] = t.y;
                }
                float sum0 = 0.f, sum1 = 0.f;
#pragma unroll
                for (int j = 0; j < 2 * kR + 1; j++) {
                    sum0 = fmaf(win.w[j], a[j], sum0);
                    sum1 = fmaf(win.w[j], a[j + 1], sum1);
                }
                *reinterpret_cast<float2 *>(&s_h3[q][ring][c0]) = make_float2(sum0, sum1);
            }
        }
        lds_barrier();

        // (5) vertical pass and the gradient at output rows orow, orow + 1 (p0 + r - 2R), two rows
        // per task from 12 ring rows: 128 tasks, two waves
        if (tid < kStep * 64 / 2) {
            const int c = tid & 63;
            float acc[3][2];
#pragma unroll
            for (int q = 0; q < 3; q++) {
                acc[q][0] = acc[q][1] = 0.f;
#pragma unroll
                for (int t = 0; t < 2 * kR + 2; t++) {
                    const float v = s_h3[q][(orow - kR + t) & (kRing - 1)][c];
#pragma unroll
                    for (int k = 0; k < 2; k++) {
                        const int j = t - k;
                        if (j >= 0 && j <= 2 * kR) acc[q][k] = fmaf(win.w[j], v, acc[q][k]);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int row = orow + k;
                if (row < r0 || row >= r1 || ocol >= W) continue;
                const size_t o = (size_t)row * W + ocol;
                const float d = xv[k] - yv[k];
                const float G = acc[0][k] + 2.f * xv[k] * acc[1][k] + yv[k] * acc[2][k];
                if (kMap) {
                    if (po.one) {
                        const float g = photo_value(up, xv[k], yv[k], G);
                        dx[o] = po.alpha ? g * po.alpha[o] : g;
                    } else {
                        dx[o] = G;
                    }
                    l1 += fabsf(d);
                } else {
                    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                    dx[o] = g_l1 * sgn + g_ssim * G;
                }
            }
        }
    };
    if (kPf == 2) {
        for (int st = 0; st < nsteps; st += 2) {
            step(st, fa);
            if (st + 1 < nsteps) step(st + 1, fb);
        }
    } else {
        for (int st = 0; st < nsteps; st++) step(st, fa);
    }
    if (kMap) {
        l1 = block_sum<kStThreads>(l1, s_red);
        ss = block_sum<kStThreads>(ss, s_red + kStThreads / 64);
        if (tid == 0) {
            const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
            partials[b] = make_float2(l1, ss);
        }
    }
}


__global__ __launch_bounds__(256) void l1_ssim_bwd_map_kernel(const float4 *__restrict__ x, const float4 *__restrict__ y,
                                                              const float4 *__restrict__ G, int64_t n4,
                                                              const float *__restrict__ dout, float inv_n,
                                                              float4 *__restrict__ dx, float w_l1, float w_ssim) {
    const float2 up = loss_upstream(dout, inv_n, w_l1, w_ssim);
    const float g_l1 = up.x, g_ssim = up.y;
    const auto one = [&](float xv, float yv, float gv) {
        const float d = xv - yv;
        const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        return g_l1 * sgn + g_ssim * gv;
    };
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 a = x[i], b = y[i], g = G[i];
        dx[i] = make_float4(one(a.x, b.x, g.x), one(a.y, b.y, g.y), one(a.z, b.z, g.z), one(a.w, b.w, g.w));
    }
}

__global__ __launch_bounds__(256) void l1_ssim_bwd_map_tail_kernel(const float *__restrict__ x,
                                                                   const float *__restrict__ y,
                                                                   const float *__restrict__ G, int64_t begin,
                                                                   int64_t n, const float *__restrict__ dout,
                                                                   float inv_n, float *__restrict__ dx, float w_l1,
                                                                   float w_ssim) {
    const int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 up = loss_upstream(dout, inv_n, w_l1, w_ssim);
    const float g_l1 = up.x, g_ssim = up.y;
    const float d = x[i] - y[i];
    const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    dx[i] = g_l1 * sgn + g_ssim * G[i];
}

// ---------------------------------------------------------------------------------------------
// Sparse Adam.

constexpr int kMaxGroups = 8;
constexpr int kAdamThreads = 256;

struct AdamArgs {
    gsr_adam_group g[kMaxGroups];
    int64_t block_start[kMaxGroups + 1];
    int n;
};

__global__ __launch_bounds__(256) void any_nonzero_kernel(const float *__restrict__ v, int64_t n,
                                                          int *__restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool nz = i < n && v[i] != 0.f;
    if (__ballot(nz) != 0 && (threadIdx.x & 63) == 0) *flag = 1;
}

template <int Wd>
__device__ __forceinline__ int64_t row_of(int64_t e, int64_t w) {
    return Wd > 0 ? e / Wd : e / w;
}

template <int Wd>
__device__ __forceinline__ void adam_element(const gsr_adam_group &G, int64_t e, const float *rel, bool dense,
                                             float b1, float b2, float omb1, float omb2, float eps) {
    const int64_t row = row_of<Wd>(e, G.width);
    if (!dense && rel[row] == 0.f) return;
    // element e of the group's (P, width) block sits at row * row_stride + col of its arrays
    const int64_t width = Wd > 0 ? Wd : G.width;
    e += row * (G.row_stride - width);
    const float g = G.grad[e];
    // scene/OurAdam.py:297-324: exp_avg.mul_(b1).add_(g, alpha=1-b1);
    // exp_avg_sq.mul_(b2).addcmul_(g, g, value=1-b2); denom = sqrt(v)/bc2_sqrt + eps;
    // param.addcdiv_(exp_avg, denom, value=-step_size)
    const float m = G.exp_avg[e] * b1 + omb1 * g;
    const float v = G.exp_avg_sq[e] * b2 + omb2 * (g * g);
    const float denom = sqrtf(v) / G.bias_correction2_sqrt + eps;
    G.exp_avg[e] = m;
    G.exp_avg_sq[e] = v;
    G.param[e] = G.param[e] + (-G.step_size) * (m / denom);
}

__global__ __launch_bounds__(kAdamThreads) void sparse_adam_kernel(AdamArgs a, const float *__restrict__ rel,
                                                                   int64_t P, float b1, float b2, float omb1,
                                                                   float omb2, float eps,
                                                                   const int *__restrict__ flag) {
    int gi = 0;
    while (gi + 1 < a.n && (int64_t)blockIdx.x >= a.block_start[gi + 1]) gi++;
    const gsr_adam_group &G = a.g[gi];
    const int64_t e = ((int64_t)blockIdx.x - a.block_start[gi]) * kAdamThreads + threadIdx.x;
    if (e >= P * G.width) return;
    const bool dense = flag == nullptr || *flag == 0;  // no relevance given, or no relevant row
    switch (G.width) {
        case 1: adam_element<1>(G, e, rel, dense, b1, b2, omb1, omb2, eps); break;
        case 3: adam_element<3>(G, e, rel, dense, b1, b2, omb1, omb2, eps); break;
        case 4: adam_element<4>(G, e, rel, dense, b1, b2, omb1, omb2, eps); break;
        case 45: adam_element<45>(G, e, rel, dense, b1, b2, omb1, omb2, eps); break;
        default: adam_element<0>(G, e, rel, dense, b1, b2, omb1, omb2, eps); break;
    }
}

// Row-block form: one wave per 64 consecutive rows.  The relevance of the 64 rows is one
// coalesced load and a ballot; a block of irrelevant rows costs nothing more.  Narrow groups
// (xyz, opacity, scaling, rotation, f_dc) are updated lane = row; a wide group (f_rest) row by
// relevant row, lanes across its columns (one contiguous 180-B segment per row).  The per-element
// arithmetic is adam_element's, so the result is bit-identical to sparse_adam_kernel's; the
// element-per-thread form launched P x 59 threads that mostly only read rel[row].
__device__ __forceinline__ void adam_at_g(const gsr_adam_group &G, int64_t e, float g, float b1, float b2, float omb1,
                                          float omb2, float eps) {
    const float m = G.exp_avg[e] * b1 + omb1 * g;
    const float v = G.exp_avg_sq[e] * b2 + omb2 * (g * g);
    const float denom = sqrtf(v) / G.bias_correction2_sqrt + eps;
    G.exp_avg[e] = m;
    G.exp_avg_sq[e] = v;
    G.param[e] = G.param[e] + (-G.step_size) * (m / denom);
}

__device__ __forceinline__ void adam_at(const gsr_adam_group &G, int64_t e, float b1, float b2, float omb1,
                                        float omb2, float eps) {
    adam_at_g(G, e, G.grad[e], b1, b2, omb1, omb2, eps);
}

constexpr int kAdamNarrow = 8;
// The native step's scale shrink (shrink_scales_kernel's arithmetic), applied by the lane that
// owns the row after its Adam update: s_raw NULL = none.
struct ShrinkArgs {
    float *s_raw;
    int64_t first;
    float limit;
};
// Sparse gradient rows (the native step): in the dense fallback (no relevant row) a row takes a
// zero gradient when the rasterizer backward did not write it (live3[3 row + 2] == 0) or when it is
// a locked skybox row (train_single.py:217-223 zeroes its six gradients).  live3 NULL: every row
// is read.
struct DenseRows {
    const float *live3;
    int64_t skybox;
};

// One wave per (64 consecutive rows, group): blockIdx.y is the group, so the groups' updates run
// in parallel waves instead of one after the other in one wave (each group's loads were a
// dependent round trip behind the previous group's stores).  Every element's loads are issued
// before its stores in program order (the arrays may alias as far as the compiler knows), so a
// lane's loads are in flight together.  The scale shrink runs in the wave that updates the
// scaling group (sh_group; -1: group 0's wave, no group writes the scales).
template <int kW>
__device__ __forceinline__ void adam_narrow(const gsr_adam_group &G, int64_t base, bool z, float b1, float b2,
                                            float omb1, float omb2, float eps) {
    float g[kW], m[kW], v[kW], p[kW];
#pragma unroll
    for (int c = 0; c < kW; c++) {
        g[c] = z ? 0.f : G.grad[base + c];
        m[c] = G.exp_avg[base + c];
        v[c] = G.exp_avg_sq[base + c];
        p[c] = G.param[base + c];
    }
#pragma unroll
    for (int c = 0; c < kW; c++) {
        const float mm = m[c] * b1 + omb1 * g[c];
        const float vv = v[c] * b2 + omb2 * (g[c] * g[c]);
        const float denom = sqrtf(vv) / G.bias_correction2_sqrt + eps;
        G.exp_avg[base + c] = mm;
        G.exp_avg_sq[base + c] = vv;
        G.param[base + c] = p[c] + (-G.step_size) * (mm / denom);
    }
}

__global__ __launch_bounds__(kAdamThreads) void sparse_adam_rows_kernel(AdamArgs a, const float *__restrict__ rel,
                                                                        int64_t P, float b1, float b2, float omb1,
                                                                        float omb2, float eps,
                                                                        const int *__restrict__ flag, ShrinkArgs sh,
                                                                        DenseRows dr, int sh_group) {
    __shared__ uint8_t s_idx[kAdamThreads / 64][64];  // the wave's relevant rows, compacted
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t r0 = (((int64_t)blockIdx.x * kAdamThreads + threadIdx.x) >> 6) * 64;
    if (r0 >= P) return;  // wave-uniform
    const int gi = (int)blockIdx.y;
    const gsr_adam_group &G = a.g[gi];
    const int64_t row = r0 + lane;
    const bool dense = flag == nullptr || *flag == 0;  // no relevance given, or no relevant row
    const bool relv = row < P && (dense || rel[row] != 0.f);
    const uint64_t mask = __ballot(relv);
    // dense fallback over sparse rows: rows whose gradient reads as zero
    const bool zrow = dense && row < P && (row < dr.skybox || (dr.live3 && dr.live3[3 * row + 2] == 0.f));
    const uint64_t zmask = __ballot(zrow);
    const int w = G.width;
    const int64_t rs = G.row_stride;
    if (mask != 0) {
        if (w <= kAdamNarrow) {
            if (relv) {
                const int64_t base = row * rs;
                switch (w) {
                    case 1: adam_narrow<1>(G, base, zrow, b1, b2, omb1, omb2, eps); break;
                    case 3: adam_narrow<3>(G, base, zrow, b1, b2, omb1, omb2, eps); break;
                    case 4: adam_narrow<4>(G, base, zrow, b1, b2, omb1, omb2, eps); break;
                    default:
                        for (int c = 0; c < w; c++) adam_narrow<1>(G, base + c, zrow, b1, b2, omb1, omb2, eps);
                        break;
                }
            }
        } else {
            // wide group: the relevant rows' elements flattened over the lanes (element e of the
            // wave's n rows: row slot e / w, column e % w), two per lane per trip with both loads
            // issued first
            if (relv) s_idx[wv][__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u))] = (uint8_t)lane;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const int tot = __popcll(mask) * w;
            for (int e0 = 0; e0 < tot; e0 += 128) {
                int64_t off[2];
                bool ok[2];
                float g[2], m[2], v[2], p[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int e = e0 + 64 * h + lane;
                    ok[h] = e < tot;
                    const int slot = ok[h] ? e / w : 0;
                    const int rl = s_idx[wv][slot];
                    off[h] = (r0 + rl) * rs + (e - slot * w);
                    const bool z = (zmask >> rl) & 1ull;
                    if (ok[h]) {
                        g[h] = z ? 0.f : G.grad[off[h]];
                        m[h] = G.exp_avg[off[h]];
                        v[h] = G.exp_avg_sq[off[h]];
                        p[h] = G.param[off[h]];
                    }
                }
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    if (!ok[h]) continue;
                    const float mm = m[h] * b1 + omb1 * g[h];
                    const float vv = v[h] * b2 + omb2 * (g[h] * g[h]);
                    const float denom = sqrtf(vv) / G.bias_correction2_sqrt + eps;
                    G.exp_avg[off[h]] = mm;
                    G.exp_avg_sq[off[h]] = vv;
                    G.param[off[h]] = p[h] + (-G.step_size) * (mm / denom);
                }
            }
        }
    }
    if (gi == (sh_group < 0 ? 0 : sh_group) && sh.s_raw && row >= sh.first && row < P) {
        float *sr = sh.s_raw + 3 * row;
        const float x = expf(sr[0]), y = expf(sr[1]), z = expf(sr[2]);
        if (fmaxf(fmaxf(x, y), z) > sh.limit) {
            sr[0] = logf(x * 0.8f);
            sr[1] = logf(y * 0.8f);
            sr[2] = logf(z * 0.8f);
        }
    }
}

// The dense step over whole rows (no relevance, no zero rows, no fused shrink: torch.optim.Adam's
// update of every element, train_post's optimizer): each group is one flat run of P * row_stride
// floats, streamed as float4.  A column-split pair (the DC and rest SH blocks of one buffer, each
// with its own learning rate) is merged on the host into one run whose step size switches at
// split_col, so the buffer is read once in full rows instead of twice in strided blocks.  Same
// arithmetic as adam_narrow, element for element.
struct FlatAdamRun {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;         // floats
    int row;           // floats per row (the column of element e is e % row)
    int split_col;     // columns < split_col take step0, the rest step1 (row: one step size)
    float step0, step1;
    float bc2s;
    int vec;           // all four arrays 16-B aligned and row % 4 == 0: float4 access
};
struct FlatAdamArgs {
    FlatAdamRun r[kMaxGroups];
    int64_t block_start[kMaxGroups + 1];
    int n;
};
constexpr int kFlatPerThread = 8;  // two float4 per lane
constexpr int64_t kFlatPerBlock = (int64_t)kAdamThreads * kFlatPerThread;

__device__ __forceinline__ void flat_adam_one(const FlatAdamRun &R, float &p, float &m, float &v, float g, float ss,
                                              float b1, float b2, float omb1, float omb2, float eps) {
    const float mm = m * b1 + omb1 * g;
    const float vv = v * b2 + omb2 * (g * g);
    const float denom = sqrtf(vv) / R.bc2s + eps;
    m = mm;
    v = vv;
    p = p + (-ss) * (mm / denom);
}

__global__ __launch_bounds__(kAdamThreads) void dense_adam_flat_kernel(FlatAdamArgs a, float b1, float b2, float omb1,
                                                                       float omb2, float eps) {
    int k = 0;
    while (k + 1 < a.n && (int64_t)blockIdx.x >= a.block_start[k + 1]) k++;
    const FlatAdamRun &R = a.r[k];
    const int64_t b0 = ((int64_t)blockIdx.x - a.block_start[k]) * kFlatPerBlock;
    if (R.vec) {
        float4 g[2], m[2], v[2], p[2];
        bool ok[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int64_t e = b0 + (int64_t)h * (kAdamThreads * 4) + 4 * threadIdx.x;
            ok[h] = e < R.n;  // n is a multiple of 4 (row % 4 == 0)
            if (ok[h]) {
                g[h] = *reinterpret_cast<const float4 *>(R.grad + e);
                m[h] = *reinterpret_cast<const float4 *>(R.exp_avg + e);
                v[h] = *reinterpret_cast<const float4 *>(R.exp_avg_sq + e);
                p[h] = *reinterpret_cast<const float4 *>(R.param + e);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (!ok[h]) continue;
            const int64_t e = b0 + (int64_t)h * (kAdamThreads * 4) + 4 * threadIdx.x;
            // the four share a row (row % 4 == 0); one step size: no column needed
            const int c = R.split_col < R.row ? (int)(e % R.row) : 0;
            float ss[4];
#pragma unroll
            for (int j = 0; j < 4; j++) ss[j] = c + j < R.split_col ? R.step0 : R.step1;
            flat_adam_one(R, p[h].x, m[h].x, v[h].x, g[h].x, ss[0], b1, b2, omb1, omb2, eps);
            flat_adam_one(R, p[h].y, m[h].y, v[h].y, g[h].y, ss[1], b1, b2, omb1, omb2, eps);
            flat_adam_one(R, p[h].z, m[h].z, v[h].z, g[h].z, ss[2], b1, b2, omb1, omb2, eps);
            flat_adam_one(R, p[h].w, m[h].w, v[h].w, g[h].w, ss[3], b1, b2, omb1, omb2, eps);
            *reinterpret_cast<float4 *>(R.exp_avg + e) = m[h];
            *reinterpret_cast<float4 *>(R.exp_avg_sq + e) = v[h];
            *reinterpret_cast<float4 *>(R.param + e) = p[h];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kFlatPerThread; j++) {
            const int64_t e = b0 + (int64_t)j * kAdamThreads + threadIdx.x;
            if (e >= R.n) break;
            float p = R.param[e], m = R.exp_avg[e], v = R.exp_avg_sq[e];
            const float ss = (int)(e % R.row) < R.split_col ? R.step0 : R.step1;
            flat_adam_one(R, p, m, v, R.grad[e], ss, b1, b2, omb1, omb2, eps);
            R.exp_avg[e] = m;
            R.exp_avg_sq[e] = v;
            R.param[e] = p;
        }
    }
}

// Builds the flat runs of a dense step.  A group that is a column block not pairing with its
// neighbour into whole rows is left for the row-block kernel: its index goes to rest[].  Returns
// the number of flat runs.
int flat_adam_runs(int n_groups, const gsr_adam_group *groups, int64_t P, FlatAdamArgs &fa, int *rest,
                   int &n_rest) {
    std::memset(&fa, 0, sizeof(fa));
    n_rest = 0;
    int64_t blocks = 0;
    for (int i = 0; i < n_groups; i++) {
        const gsr_adam_group &g = groups[i];
        const int64_t rs = g.row_stride == 0 ? g.width : g.row_stride;
        FlatAdamRun r;
        std::memset(&r, 0, sizeof(r));
        r.param = g.param;
        r.grad = g.grad;
        r.exp_avg = g.exp_avg;
        r.exp_avg_sq = g.exp_avg_sq;
        r.step0 = r.step1 = g.step_size;
        r.bc2s = g.bias_correction2_sqrt;
        r.split_col = (int)rs;
        if (rs > 0x7fffffff) {
            rest[n_rest++] = i;
            continue;
        }
        if (rs != g.width) {
            const gsr_adam_group *h = i + 1 < n_groups ? &groups[i + 1] : nullptr;
            const int64_t hs = h ? (h->row_stride == 0 ? h->width : h->row_stride) : 0;
            if (!h || hs != rs || g.width + h->width != rs || h->param != g.param + g.width ||
                h->grad != g.grad + g.width || h->exp_avg != g.exp_avg + g.width ||
                h->exp_avg_sq != g.exp_avg_sq + g.width || h->bias_correction2_sqrt != g.bias_correction2_sqrt) {
                rest[n_rest++] = i;
                continue;
            }
            r.split_col = (int)g.width;
            r.step1 = h->step_size;
            i++;
        }
        r.row = (int)rs;
        r.n = P * rs;
        const uintptr_t al = reinterpret_cast<uintptr_t>(r.param) | reinterpret_cast<uintptr_t>(r.grad) |
                             reinterpret_cast<uintptr_t>(r.exp_avg) | reinterpret_cast<uintptr_t>(r.exp_avg_sq);
        r.vec = (al & 15) == 0 && rs % 4 == 0;
        fa.r[fa.n] = r;
        fa.block_start[fa.n] = blocks;
        blocks += (r.n + kFlatPerBlock - 1) / kFlatPerBlock;
        fa.n++;
    }
    fa.block_start[fa.n] = blocks;
    return fa.n;
}

// The relevant rows compacted first (sparse steps: OurAdam's `relevant` rows, train_single.py:226).
// The row-block kernel above launches a wave per (64 rows, group) -- P / 64 x groups waves, most of
// which (88% of the rows are irrelevant late in a street chunk) only read 64 flags and leave -- and
// updates a relevant row's narrow groups lane = row, one 64-B line per few useful bytes.  Here:
//   adam_compact_kernel  a grid-stride pass over the flags: each wave's relevant rows appended to a
//                        list (one atomic per wave; Adam's rows are independent, so the order is
//                        free), and the scale shrink of the rows no update touches;
//   adam_rowlist_kernel  one wave per listed row (grid-stride): lane l updates element l of the
//                        row's groups concatenated (59 at SH degree 3: xyz 3, f_dc 3, f_rest 45,
//                        opacity 1, scaling 3, rotation 4), so the SH pair's 48 floats are ONE
//                        192-B contiguous access per array, then the shrink of the row's scales.
// With no relevant row (the dense fallback, OurAdam.py:214) the list pass is skipped and the row
// kernel walks every row (the sparse-rows zero gradients of DenseRows applied).  Same per-element
// arithmetic as adam_narrow (bits unchanged).  GSR_ADAM_ROWBLOCK=1: the row-block kernel (A/B).
constexpr int kAdamListMaxLanes = 64;
__device__ __forceinline__ uint32_t lane_prefix_u64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
struct AdamLaneMap {
    uint8_t group[kAdamListMaxLanes], col[kAdamListMaxLanes];
    int lanes;      // elements per row (sum of the group widths)
    int sh_lane0;   // the first of the three scaling lanes (the shrink), -1: none
};

// Workgroup b owns the contiguous rows [b * per, (b + 1) * per): a first walk counts its relevant
// rows (ballots) and shrinks the rows no update touches, ONE atomic reserves the workgroup's run
// of the list, a second walk (the flags again, now cache-hot) writes the rows.  One atomic per
// wave instead (the first version) put ~16K returning atomics on one word per call, which
// saturates at ~88 per us (MI355X_MICROARCH.md, dequeue): 164 us per call at 1M rows.
constexpr int kCompactThreads = 1024;
constexpr int kCompactWaves = kCompactThreads / 64;
constexpr int kCompactMaxBlocks = 256;
__global__ __launch_bounds__(kCompactThreads) void adam_compact_kernel(const float *__restrict__ rel, int64_t P,
                                                                       const int *__restrict__ flag, int *__restrict__ list,
                                                                       int *__restrict__ count, ShrinkArgs sh) {
    if (*flag == 0) return;  // the dense fallback: the row kernel takes every row (and shrinks them)
    __shared__ uint32_t s_wc[kCompactWaves];
    __shared__ int s_base;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t per = ((P + gridDim.x - 1) / gridDim.x + kCompactThreads - 1) / kCompactThreads * kCompactThreads;
    const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min(P, r0 + per);
    uint32_t cnt = 0;
    for (int64_t b = r0 + (int64_t)w * 64; b < r1; b += kCompactThreads) {
        const int64_t row = b + lane;
        const bool relv = row < r1 && rel[row] != 0.f;
        cnt += (uint32_t)__popcll(__ballot(relv));
        if (!relv && sh.s_raw && row >= sh.first && row < r1) {  // rows no update touches: shrunk here
            float *sr = sh.s_raw + 3 * row;
            const float x = expf(sr[0]), y = expf(sr[1]), z = expf(sr[2]);
            if (fmaxf(fmaxf(x, y), z) > sh.limit) {
                sr[0] = logf(x * 0.8f);
                sr[1] = logf(y * 0.8f);
                sr[2] = logf(z * 0.8f);
            }
        }
    }
    if (lane == 0) s_wc[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int k = 0; k < kCompactWaves; k++) tot += s_wc[k];
        s_base = tot ? atomicAdd(count, (int)tot) : 0;
    }
    __syncthreads();
    if (r0 >= r1) return;
    int at = s_base;
    for (int k = 0; k < w; k++) at += (int)s_wc[k];
    for (int64_t b = r0 + (int64_t)w * 64; b < r1; b += kCompactThreads) {
        const int64_t row = b + lane;
        const bool relv = row < r1 && rel[row] != 0.f;
        const uint64_t m = __ballot(relv);
        if (relv) list[at + (int)lane_prefix_u64(m)] = (int)row;
        at += __popcll(m);
    }
}

// Four listed rows per wave and trip: the four rows' list entries, then all their loads, then the
// updates -- one row at a time left each wave a chain of dependent round trips per row (~32 rows per
// resident wave at 3M rows, 8.5% relevant: 140 us per call in the config-3 chunk, r05e).
#ifndef GSR_ADAM_ROWS
#define GSR_ADAM_ROWS 1  // r05i: 4 rows per trip 42.9 / 163.4 us per call (1M / 3M rows), 1 row 38.0 / 161.5 us
#endif
constexpr int kAdamRowsPerTrip = GSR_ADAM_ROWS;
__global__ __launch_bounds__(256) void adam_rowlist_kernel(AdamArgs a, AdamLaneMap lm, const int *__restrict__ list,
                                                           const int *__restrict__ count, int64_t P,
                                                           const int *__restrict__ flag, float b1, float b2, float omb1,
                                                           float omb2, float eps, ShrinkArgs sh, DenseRows dr) {
    constexpr int R = kAdamRowsPerTrip;
    const int lane = threadIdx.x & 63;
    const bool dense = *flag == 0;
    const int64_t n = dense ? P : (int64_t)*count;
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
    const bool act = lane < lm.lanes;
    const gsr_adam_group &G = a.g[act ? lm.group[lane] : 0];
    const int64_t col = act ? lm.col[lane] : 0;
    const bool shrink = sh.s_raw && lm.sh_lane0 >= 0;
    for (int64_t k0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * R; k0 < n; k0 += waves * R) {
        int64_t row[R];
        bool ok[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            ok[r] = k0 + r < n;
            row[r] = !ok[r] ? 0 : dense ? k0 + r : (int64_t)list[k0 + r];
        }
        float g[R], m0[R], v0[R], p0[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            g[r] = m0[r] = v0[r] = p0[r] = 0.f;
            if (act && ok[r]) {
                // the dense fallback over sparse rows: rows whose gradient reads as zero
                const bool z = dense && (row[r] < dr.skybox || (dr.live3 && dr.live3[3 * row[r] + 2] == 0.f));
                const int64_t e = row[r] * G.row_stride + col;
                g[r] = z ? 0.f : G.grad[e];
                m0[r] = G.exp_avg[e];
                v0[r] = G.exp_avg_sq[e];
                p0[r] = G.param[e];
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            if (!ok[r]) break;  // wave-uniform
            float p = 0.f;
            if (act) {
                const int64_t e = row[r] * G.row_stride + col;
                const float mm = m0[r] * b1 + omb1 * g[r];
                const float vv = v0[r] * b2 + omb2 * (g[r] * g[r]);
                const float denom = sqrtf(vv) / G.bias_correction2_sqrt + eps;
                G.exp_avg[e] = mm;
                G.exp_avg_sq[e] = vv;
                p = p0[r] + (-G.step_size) * (mm / denom);
                G.param[e] = p;
            }
            if (shrink && row[r] >= sh.first) {
                // the shrink of the row's freshly updated scales (shrink_scales_kernel's arithmetic)
                const float sx = __shfl(p, lm.sh_lane0, 64), sy = __shfl(p, lm.sh_lane0 + 1, 64),
                            sz = __shfl(p, lm.sh_lane0 + 2, 64);
                const float x = expf(sx), y = expf(sy), zz = expf(sz);
                if (fmaxf(fmaxf(x, y), zz) > sh.limit && lane >= lm.sh_lane0 && lane < lm.sh_lane0 + 3) {
                    const float c = lane == lm.sh_lane0 ? x : lane == lm.sh_lane0 + 1 ? y : zz;
                    sh.s_raw[3 * row[r] + (lane - lm.sh_lane0)] = logf(c * 0.8f);
                }
            }
        }
    }
}

bool adam_rowblock() {  // read per call: A/B runs switch it
    const char *e = std::getenv("GSR_ADAM_ROWBLOCK");
    return e != nullptr && e[0] == '1';
}

// GSR_ADAM_DENSE_ROWS=1 sends a dense step through the row-block kernel instead (A/B).
bool adam_dense_rows() {
    const char *e = std::getenv("GSR_ADAM_DENSE_ROWS");
    return e != nullptr && e[0] == '1';
}

// GSR_ADAM_ELEMENTWISE=1 selects the element-per-thread kernel (same bits; A/B test and
// measurements).  Read per call so a test can switch it.
bool adam_elementwise() {
    const char *e = std::getenv("GSR_ADAM_ELEMENTWISE");
    return e != nullptr && e[0] == '1';
}

__global__ __launch_bounds__(256) void densify_stats_kernel(int64_t P, const int *__restrict__ radii,
                                                            const float *__restrict__ g2d, float *__restrict__ maxr,
                                                            float *__restrict__ accum, float *__restrict__ denom) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    const float gx = g2d[3 * i], gy = g2d[3 * i + 1];
    const float n = sqrtf(gx * gx + gy * gy);
    maxr[i] = fmaxf(maxr[i], (float)r);
    accum[i] = fmaxf(n, accum[i]);
    denom[i] = denom[i] + 1.f;
}

// ---------------------------------------------------------------------------------------------
// Parameter activations (scene/gaussian_model.py:39-47, getters :125-156) and the per-step
// shrink of over-large Gaussians (train_single.py:235-241).  One lane per Gaussian; the
// backward follows torch's autograd formulas (exp: g*y; sigmoid: g*(1-y)*y; normalize =
// x / max(||x||, 1e-12): dx = g/d - x * (sum(g * ((x/d)/d)) / n)).

__global__ __launch_bounds__(256) void activate_fwd_kernel(int64_t P, const float *__restrict__ s_raw,
                                                           const float4 *__restrict__ q_raw,
                                                           const float *__restrict__ o_raw, float *__restrict__ scales,
                                                           float4 *__restrict__ rots, float *__restrict__ opac) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
#pragma unroll
    for (int k = 0; k < 3; k++) scales[3 * i + k] = act_scale(s_raw[3 * i + k]);
    rots[i] = act_rot(q_raw[i]);
    opac[i] = act_opacity(o_raw[i]);
}

__global__ __launch_bounds__(256) void activate_bwd_kernel(int64_t P, const float4 *__restrict__ q_raw,
                                                           const float *__restrict__ scales,
                                                           const float *__restrict__ opac,
                                                           const float *__restrict__ g_s,
                                                           const float4 *__restrict__ g_q,
                                                           const float *__restrict__ g_o, float *__restrict__ d_s,
                                                           float4 *__restrict__ d_q, float *__restrict__ d_o) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
#pragma unroll
    for (int k = 0; k < 3; k++) d_s[3 * i + k] = g_s[3 * i + k] * scales[3 * i + k];
    const float4 x = q_raw[i], g = g_q[i];
    const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
    const float d = fmaxf(n, 1e-12f);
    const float gd = -(g.x * ((x.x / d) / d) + g.y * ((x.y / d) / d) + g.z * ((x.z / d) / d) + g.w * ((x.w / d) / d));
    const float gn = n >= 1e-12f && n != 0.f ? gd / n : 0.f;  // clamp_min and norm backward
    d_q[i] = make_float4(g.x / d + x.x * gn, g.y / d + x.y * gn, g.z / d + x.z * gn, g.w / d + x.w * gn);
    const float y = opac[i];
    d_o[i] = g_o[i] * (1.f - y) * y;
}

// The native step's form: also the skybox lock (rows below `skybox` get a zero opacity gradient,
// train_single.py:217-223), the sparse Adam's "any relevant row" flag (zeroed earlier in the step)
// and the densification statistics of the same row (densify_stats_kernel's arithmetic).
__global__ __launch_bounds__(256) void activate_bwd_step_kernel(
    int64_t P, const float4 *__restrict__ q_raw, const float *__restrict__ scales, const float *__restrict__ opac,
    const float *__restrict__ g_s, const float4 *__restrict__ g_q, const float *__restrict__ g_o,
    float *__restrict__ d_s, float4 *__restrict__ d_q, float *__restrict__ d_o, int64_t skybox, int *__restrict__ flag,
    const int *__restrict__ radii, const float *__restrict__ g2d, float *__restrict__ maxr, float *__restrict__ accum,
    float *__restrict__ denom, int sparse_rows, const float *__restrict__ s_raw, const float *__restrict__ o_raw) {
    // scales / opac NULL: the raw mode (the rasterizer read the pre-activation parameters): the
    // activations are recomputed here from s_raw / o_raw, with the forward's expressions
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float go = 0.f;
    if (i < P) {
        const int r = radii[i];
        // sparse rows: only the rows the rasterizer backward wrote (liveness in g2d's third column;
        // invisible rows never are) have scale / rotation gradients -- the others are never relevant
        bool live = !sparse_rows;
        if (r > 0) {
            const float gx = g2d[3 * i], gy = g2d[3 * i + 1];
            if (sparse_rows) live = g2d[3 * i + 2] != 0.f;
            const float nn = sqrtf(gx * gx + gy * gy);
            maxr[i] = fmaxf(maxr[i], (float)r);
            accum[i] = fmaxf(nn, accum[i]);
            denom[i] = denom[i] + 1.f;
        }
        if (live) {
#pragma unroll
            for (int k = 0; k < 3; k++)
                d_s[3 * i + k] = g_s[3 * i + k] * (scales ? scales[3 * i + k] : act_scale(s_raw[3 * i + k]));
            const float4 x = q_raw[i], g = g_q[i];
            const float n = sqrtf(x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w);
            const float d = fmaxf(n, 1e-12f);
            const float gd =
                -(g.x * ((x.x / d) / d) + g.y * ((x.y / d) / d) + g.z * ((x.z / d) / d) + g.w * ((x.w / d) / d));
            const float gn = n >= 1e-12f && n != 0.f ? gd / n : 0.f;
            d_q[i] = make_float4(g.x / d + x.x * gn, g.y / d + x.y * gn, g.z / d + x.z * gn, g.w / d + x.w * gn);
        }
        const float y = opac ? opac[i] : act_opacity(o_raw[i]);
        go = i < skybox ? 0.f : g_o[i] * (1.f - y) * y;
        d_o[i] = go;
    }
    if (__ballot(go != 0.f) != 0 && (threadIdx.x & 63) == 0) *flag = 1;
}

__global__ __launch_bounds__(256) void shrink_scales_kernel(int64_t P, int64_t first, float *__restrict__ s_raw,
                                                            float limit) {
    const int64_t i = first + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float a = expf(s_raw[3 * i]), b = expf(s_raw[3 * i + 1]), c = expf(s_raw[3 * i + 2]);
    if (fmaxf(fmaxf(a, b), c) > limit) {
        s_raw[3 * i] = logf(a * 0.8f);
        s_raw[3 * i + 1] = logf(b * 0.8f);
        s_raw[3 * i + 2] = logf(c * 0.8f);
    }
}

// ---------------------------------------------------------------------------------------------
// Exposure affine + clamp (gaussian_renderer/__init__.py:115-120).

constexpr int kExpBlocks = 1024;
constexpr int kExpThreads = 256;

__device__ __forceinline__ void exposure_pre(const float *__restrict__ E, float c0, float c1, float c2, float &o0,
                                             float &o1, float &o2) {
    // matmul(img.permute(1, 2, 0), E[:3, :3]) + E[:3, 3]: out_c = sum_k img_k E[k][c] + E[c][3]
    o0 = c0 * E[0] + c1 * E[4] + c2 * E[8] + E[3];
    o1 = c0 * E[1] + c1 * E[5] + c2 * E[9] + E[7];
    o2 = c0 * E[2] + c1 * E[6] + c2 * E[10] + E[11];
}

// alpha (the native step): the image times the view's alpha mask (train_single.py:117-119) in the
// same pass -- one rounding, as torch's separate multiply
__global__ __launch_bounds__(kExpThreads) void exposure_fwd_kernel(const float *__restrict__ color,
                                                                   const float *__restrict__ E, int64_t n,
                                                                   float *__restrict__ out,
                                                                   const float *__restrict__ alpha) {
    for (int64_t p = (int64_t)blockIdx.x * kExpThreads + threadIdx.x; p < n; p += (int64_t)gridDim.x * kExpThreads) {
        float o0, o1, o2;
        exposure_pre(E, color[p], color[n + p], color[2 * n + p], o0, o1, o2);
        o0 = fminf(fmaxf(o0, 0.f), 1.f);
        o1 = fminf(fmaxf(o1, 0.f), 1.f);
        o2 = fminf(fmaxf(o2, 0.f), 1.f);
        if (alpha) {
            const float a = alpha[p];
            o0 = o0 * a;
            o1 = o1 * a;
            o2 = o2 * a;
        }
        out[p] = o0;
        out[n + p] = o1;
        out[2 * n + p] = o2;
    }
}

// The photometric loss gradient for kPhoto (the native step): gout is formed here from the
// SSIM gradient field as l1_ssim_bwd_map_kernel forms it (then times the alpha mask, torch's
// multiply backward) instead of being read, which saves writing and re-reading the (3, H, W)
// image gradient.  Same loop and reduction order either way, so dcolor and the dE partials are
// bit-identical.
struct PhotoGrad {
    const float *x, *y, *G;  // the (masked) exposed image, the target, the SSIM gradient field
    const float *dout;       // dL/dloss (device)
    const float *alpha;      // (H, W) or NULL
    float inv_n, w_l1, w_ssim;
};

template <bool kPhoto>
__global__ __launch_bounds__(kExpThreads) void exposure_bwd_kernel(const float *__restrict__ color,
                                                                   const float *__restrict__ E, int64_t n,
                                                                   const float *__restrict__ gout,
                                                                   float *__restrict__ gcolor,
                                                                   float *__restrict__ partials, PhotoGrad pg) {
    __shared__ float red[12][kExpThreads / 64];
    float acc[12];
#pragma unroll
    for (int k = 0; k < 12; k++) acc[k] = 0.f;
    float2 up = make_float2(0.f, 0.f);
    if (kPhoto) up = loss_upstream(pg.dout, pg.inv_n, pg.w_l1, pg.w_ssim);
    const auto photo = [&](int64_t i, float a) {
        const float g = photo_value(up, pg.x[i], pg.y[i], pg.G[i]);
        return pg.alpha ? g * a : g;
    };
    for (int64_t p = (int64_t)blockIdx.x * kExpThreads + threadIdx.x; p < n; p += (int64_t)gridDim.x * kExpThreads) {
        const float c0 = color[p], c1 = color[n + p], c2 = color[2 * n + p];
        float o0, o1, o2;
        exposure_pre(E, c0, c1, c2, o0, o1, o2);
        float u0, u1, u2;
        if (kPhoto) {
            const float a = pg.alpha ? pg.alpha[p] : 1.f;
            u0 = photo(p, a);
            u1 = photo(n + p, a);
            u2 = photo(2 * n + p, a);
        } else {
            u0 = gout[p];
            u1 = gout[n + p];
            u2 = gout[2 * n + p];
        }
        const float g0 = (o0 >= 0.f && o0 <= 1.f) ? u0 : 0.f;
        const float g1 = (o1 >= 0.f && o1 <= 1.f) ? u1 : 0.f;
        const float g2 = (o2 >= 0.f && o2 <= 1.f) ? u2 : 0.f;
        gcolor[p] = E[0] * g0 + E[1] * g1 + E[2] * g2;
        gcolor[n + p] = E[4] * g0 + E[5] * g1 + E[6] * g2;
        gcolor[2 * n + p] = E[8] * g0 + E[9] * g1 + E[10] * g2;
        // dE[k][c] = sum_p img_k g_c ; dE[c][3] = sum_p g_c   (row-major 3x4 slots)
        acc[0] += c0 * g0; acc[1] += c0 * g1; acc[2] += c0 * g2; acc[3] += g0;
        acc[4] += c1 * g0; acc[5] += c1 * g1; acc[6] += c1 * g2; acc[7] += g1;
        acc[8] += c2 * g0; acc[9] += c2 * g1; acc[10] += c2 * g2; acc[11] += g2;
    }
    const int wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const float v = wave_sum(acc[k]);
        if ((threadIdx.x & 63) == 0) red[k][wv] = v;
    }
    __syncthreads();
    if (threadIdx.x < 12) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kExpThreads / 64; w++) s += red[threadIdx.x][w];
        partials[(size_t)blockIdx.x * 12 + threadIdx.x] = s;
    }
}

// One wave per output value; each lane sums a fixed strided subset, then a fixed-order wave sum.
__global__ __launch_bounds__(768) void exposure_finalize_kernel(const float *__restrict__ partials, int nblocks,
                                                                float *__restrict__ dE) {
    const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float s = 0.f;
    for (int b = lane; b < nblocks; b += 64) s += partials[(size_t)b * 12 + k];
    s = wave_sum(s);
    if (lane == 0) dE[k] = s;
}

// The native step: the exposure gradient's reduction, then the exposure optimizer's dense Adam
// step over all n_images x 12 values in the same launch (the gradient is dE in the view's row and
// zero elsewhere, as autograd's index backward leaves it); adam_at's arithmetic, so the bits of
// gsr_sparse_adam_step's dense step.
__global__ __launch_bounds__(768) void exposure_finalize_adam_kernel(const float *__restrict__ partials, int nblocks,
                                                                     int n_images, int view, gsr_adam_group G,
                                                                     float *__restrict__ grad_out, float b1, float b2,
                                                                     float omb1, float omb2, float eps) {
    __shared__ float dE[12];
    const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float s = 0.f;
    for (int b = lane; b < nblocks; b += 64) s += partials[(size_t)b * 12 + k];
    s = wave_sum(s);
    if (lane == 0) dE[k] = s;
    __syncthreads();
    for (int e = threadIdx.x; e < 12 * n_images; e += 768) {
        const int row = e / 12;
        const float g = row == view ? dE[e - 12 * view] : 0.f;
        grad_out[e] = g;
        adam_at_g(G, e, g, b1, b2, omb1, omb2, eps);
    }
}

int exposure_blocks(int64_t n) {
    const int64_t b = (n + kExpThreads - 1) / kExpThreads;
    return (int)(b < kExpBlocks ? (b > 0 ? b : 1) : kExpBlocks);
}

dim3 loss_grid(int C, int H, int W) { return dim3((W + kTW - 1) / kTW, (H + kTH - 1) / kTH, C); }
// Rows per strip of the streaming kernel: enough strips to fill the resident workgroup slots once
// (four per CU at 40 KiB of LDS), so every workgroup starts in the first round and the 4R rows of
// halo each strip recomputes are spread over as many rows as that allows; at least 64 rows.
int stream_seg(int C, int H, int W) {
    if (GSR_SSIM_SEG_H > 0) return GSR_SSIM_SEG_H;
    static int cus[16] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = -1;
    int n = 256;
    if (dev >= 0) {
        if (!cus[dev]) {
            int c = 0;
            cus[dev] = hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0
                           ? c : 256;
        }
        n = cus[dev];
    }
    const int cols = (W + kStW - 1) / kStW;
    const int strips = std::max(1, kStPerCU * n / std::max(1, C * cols));
    int seg = (H + strips - 1) / strips;
    seg = (seg + kStep - 1) / kStep * kStep;
    return std::max(seg, 64);
}

dim3 stream_grid(int C, int H, int W) {
    const int seg = stream_seg(C, H, W);
    return dim3((W + kStW - 1) / kStW, (H + seg - 1) / seg, C);
}

// GSR_SSIM_TILED=1 selects the 64 x 16 tile gradient kernel instead of the streaming one (same
// bits; kept for the A/B test and measurements).  Read per call so a test can switch it.
bool ssim_tiled() {
    const char *e = std::getenv("GSR_SSIM_TILED");
    return e != nullptr && e[0] == '1';
}


// ---- masked inverse-depth L1 (train_single.py:135-141) ----------------------------------------
// forward: per-block partial sums of |(invd - mono) * mask| (fp32 per thread over a float4 stride,
// fp64 across threads and blocks), then mean and weight; backward: torch's chain
// * w -> * (1/N) -> * sgn(d) -> * mask for d = (invd - mono) * mask, in that order (bit-identical to
// autograd through the reference's expression).
constexpr int kDepthThreads = 256;
constexpr int kDepthPerBlock = 4 * kDepthThreads * 4;  // float4 per thread, 4 strides

__device__ __forceinline__ float depth_term(float x, float y, float m) { return (x - y) * m; }

// kGrad: also dL/dinvdepth for an upstream of 1 (the native step, where the loss is the root):
// the backward kernel's chain with gout = 1, element for element
template <bool kGrad>
__global__ __launch_bounds__(kDepthThreads) void depth_l1_fwd_kernel(const float *__restrict__ invd,
                                                                    const float *__restrict__ mono,
                                                                    const float *__restrict__ mask, int64_t n,
                                                                    double *__restrict__ partials, float w,
                                                                    float inv_count, float *__restrict__ dinvd) {
    __shared__ double red[kDepthThreads / 64];
    const int64_t b0 = (int64_t)blockIdx.x * kDepthPerBlock;
    const float g = kGrad ? __fmul_rn(__fmul_rn(1.f, w), inv_count) : 0.f;
    const auto grad = [&](float d, float m) {
        const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
        return __fmul_rn(__fmul_rn(g, sg), m);
    };
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t i = b0 + 4 * ((int64_t)k * kDepthThreads + threadIdx.x);
        if (i + 3 < n) {
            const float4 x = *reinterpret_cast<const float4 *>(invd + i);
            const float4 y = *reinterpret_cast<const float4 *>(mono + i);
            const float4 m = mask ? *reinterpret_cast<const float4 *>(mask + i) : make_float4(1.f, 1.f, 1.f, 1.f);
            const float d0 = depth_term(x.x, y.x, m.x), d1 = depth_term(x.y, y.y, m.y);
            const float d2 = depth_term(x.z, y.z, m.z), d3 = depth_term(x.w, y.w, m.w);
            acc += fabsf(d0) + fabsf(d1) + fabsf(d2) + fabsf(d3);
            if (kGrad)
                *reinterpret_cast<float4 *>(dinvd + i) =
                    make_float4(grad(d0, m.x), grad(d1, m.y), grad(d2, m.z), grad(d3, m.w));
        } else {
            for (int64_t j = i; j < n && j < i + 4; j++) {
                const float mj = mask ? mask[j] : 1.f;
                const float d = depth_term(invd[j], mono[j], mj);
                acc += fabsf(d);
                if (kGrad) dinvd[j] = grad(d, mj);
            }
        }
    }
    double v = acc;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < kDepthThreads / 64; k++) t += red[k];
        partials[blockIdx.x] = t;
    }
}

__device__ __forceinline__ void depth_finalize_body(const double *__restrict__ partials, int nb, double inv_n,
                                                    float w, float *__restrict__ out) {
    __shared__ double red[1024];
    double a = 0.0;
    for (int i = threadIdx.x; i < nb; i += 1024) a += partials[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int k = 512; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = (float)(red[0] * inv_n);       // Ll1depth_pure
        out[1] = __fmul_rn(w, out[0]);          // depth_l1_weight(iteration) * Ll1depth_pure
    }
}

__global__ __launch_bounds__(1024) void depth_l1_finalize_kernel(const double *__restrict__ partials, int nb,
                                                                 double inv_n, float w, float *__restrict__ out) {
    depth_finalize_body(partials, nb, inv_n, w, out);
}

// The native step's loss epilogue: the photometric and (dp != NULL) depth reductions of
// loss_finalize_kernel / depth_l1_finalize_kernel, the step's total loss (torch's fp32 add of the
// two terms) in out[5], and the sparse Adam's relevance flag cleared for activate_bwd_step_kernel.
__global__ __launch_bounds__(1024) void step_finalize_kernel(const float2 *__restrict__ pp, int np, double inv_np,
                                                             float w_l1, float w_ssim, const double *__restrict__ dp,
                                                             int nd, double inv_nd, float w, float *__restrict__ out,
                                                             int *__restrict__ flag) {
    loss_finalize_body(pp, np, inv_np, out, w_l1, w_ssim);
    if (dp) {
        __syncthreads();
        depth_finalize_body(dp, nd, inv_nd, w, out + 3);
    }
    if (threadIdx.x == 0) {
        out[5] = dp ? __fadd_rn(out[2], out[4]) : out[2];
        *flag = 0;
    }
}

__global__ __launch_bounds__(256) void depth_l1_bwd_kernel(const float *__restrict__ invd, const float *__restrict__ mono,
                                                           const float *__restrict__ mask, int64_t n,
                                                           const float *__restrict__ gout, float w, float inv_count,
                                                           float *__restrict__ dinvd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // MeanBackward divides by the element count as a CPU scalar, which ATen turns into a
    // multiply by its fp32 reciprocal
    const float g = __fmul_rn(__fmul_rn(gout[0], w), inv_count);
    const float m = mask ? mask[i] : 1.f;
    const float d = depth_term(invd[i], mono[i], m);
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    dinvd[i] = __fmul_rn(__fmul_rn(g, sg), m);
}

// ---- the depth-only view's loss (train_single.py:145-156, Street-sparse's additional depth maps) --
//   pure = mean |(invd - mono) * mask|,  dens = mean clamp(mono - invd, min=0)
//   loss = w * (a * dens + (1 - a) * pure)          (a = additional_depth_maps_weight)
// Both sums in one pass (fp32 per thread, fp64 across threads and blocks).  The gradient follows
// torch's autograd through that expression term by term: g = gout * w; the clamp branch
// -(g * a) * (1/N) where mono - invd >= 0 (clamp passes the gradient at the bound); the L1 branch
// ((g * (1 - a)) * (1/N)) * sgn(d) * mask; their sum (the two uses of invDepth).
struct DepthOnlyW {
    float g_dens, g_pure;  // gout * w * a * (1/N), gout * w * (1 - a) * (1/N), in torch's order
};

__device__ __forceinline__ float depth_only_grad(float x, float y, float m, const DepthOnlyW &q) {
    const float d = depth_term(x, y, m);
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
    const float t2 = __fmul_rn(__fmul_rn(q.g_pure, sg), m);
    const float t1 = (y - x) >= 0.f ? -q.g_dens : 0.f;
    return __fadd_rn(t1, t2);
}

// host and device (the native step forms it on the host for an upstream of 1); products only, so
// -ffp-contract=off leaves each one a rounded fp32 multiply
__host__ __device__ __forceinline__ DepthOnlyW depth_only_w(float gout, float w, float a, float oma,
                                                            float inv_count) {
    const float g = gout * w;
    return DepthOnlyW{(g * a) * inv_count, (g * oma) * inv_count};
}

// kGrad: dL/dinvdepth for an upstream of 1 in the same pass (the native step)
template <bool kGrad>
__global__ __launch_bounds__(kDepthThreads) void depth_only_fwd_kernel(const float *__restrict__ invd,
                                                                      const float *__restrict__ mono,
                                                                      const float *__restrict__ mask, int64_t n,
                                                                      double2 *__restrict__ partials, DepthOnlyW q,
                                                                      float *__restrict__ dinvd) {
    __shared__ double2 red[kDepthThreads / 64];
    const int64_t b0 = (int64_t)blockIdx.x * kDepthPerBlock;
    float acc_p = 0.f, acc_d = 0.f;
    const auto one = [&](float x, float y, float m, float &g) {
        acc_p += fabsf(depth_term(x, y, m));
        acc_d += fmaxf(y - x, 0.f);
        if (kGrad) g = depth_only_grad(x, y, m, q);
    };
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t i = b0 + 4 * ((int64_t)k * kDepthThreads + threadIdx.x);
        if (i + 3 < n) {
            const float4 x = *reinterpret_cast<const float4 *>(invd + i);
            const float4 y = *reinterpret_cast<const float4 *>(mono + i);
            const float4 m = mask ? *reinterpret_cast<const float4 *>(mask + i) : make_float4(1.f, 1.f, 1.f, 1.f);
            float4 g;
            one(x.x, y.x, m.x, g.x);
            one(x.y, y.y, m.y, g.y);
            one(x.z, y.z, m.z, g.z);
            one(x.w, y.w, m.w, g.w);
            if (kGrad) *reinterpret_cast<float4 *>(dinvd + i) = g;
        } else {
            for (int64_t j = i; j < n && j < i + 4; j++) {
                float g;
                one(invd[j], mono[j], mask ? mask[j] : 1.f, g);
                if (kGrad) dinvd[j] = g;
            }
        }
    }
    double vp = acc_p, vd = acc_d;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        vp += __shfl_xor(vp, o, 64);
        vd += __shfl_xor(vd, o, 64);
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_double2(vp, vd);
    __syncthreads();
    if (threadIdx.x == 0) {
        double2 t = make_double2(0.0, 0.0);
        for (int k = 0; k < kDepthThreads / 64; k++) {
            t.x += red[k].x;
            t.y += red[k].y;
        }
        partials[blockIdx.x] = t;
    }
}

// out3 = (pure, dens, loss); step != 0 (the native step's epilogue): out6 = (dens, 0, 0, pure, loss,
// loss) and the sparse Adam's relevance flag cleared
__global__ __launch_bounds__(1024) void depth_only_finalize_kernel(const double2 *__restrict__ partials, int nb,
                                                                   double inv_n, float w, float a, float oma,
                                                                   float *__restrict__ out, int *__restrict__ flag) {
    __shared__ double2 red[1024];
    double2 v = make_double2(0.0, 0.0);
    for (int i = threadIdx.x; i < nb; i += 1024) {
        v.x += partials[i].x;
        v.y += partials[i].y;
    }
    red[threadIdx.x] = v;
    __syncthreads();
    for (int k = 512; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            red[threadIdx.x].x += red[threadIdx.x + k].x;
            red[threadIdx.x].y += red[threadIdx.x + k].y;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const float pure = (float)(red[0].x * inv_n), dens = (float)(red[0].y * inv_n);
        // w * (a * dens + (1 - a) * pure) in torch's fp32 op order
        const float loss = __fmul_rn(__fadd_rn(__fmul_rn(dens, a), __fmul_rn(pure, oma)), w);
        if (flag) {
            out[0] = dens;
            out[1] = 0.f;
            out[2] = 0.f;
            out[3] = pure;
            out[4] = loss;
            out[5] = loss;
            *flag = 0;
        } else {
            out[0] = pure;
            out[1] = dens;
            out[2] = loss;
        }
    }
}

__global__ __launch_bounds__(256) void depth_only_bwd_kernel(const float *__restrict__ invd,
                                                             const float *__restrict__ mono,
                                                             const float *__restrict__ mask, int64_t n,
                                                             const float *__restrict__ gout, float w, float a,
                                                             float oma, float inv_count, float *__restrict__ dinvd) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dinvd[i] = depth_only_grad(invd[i], mono[i], mask ? mask[i] : 1.f, depth_only_w(gout[0], w, a, oma, inv_count));
}

bool g_lds_attr = false;

void set_lds_attr() {
    if (g_lds_attr) return;
    (void)hipFuncSetAttribute((const void *)l1_ssim_grad_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kBwdLds);
    (void)hipFuncSetAttribute((const void *)l1_ssim_grad_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kBwdLds);
    g_lds_attr = true;
}

}  // namespace

// flag_ready: *flag_scratch already holds "some row is relevant" (the native step's
// activate_bwd_step_kernel computed it), so the any_nonzero pass is skipped.
int sparse_adam(int n_groups, const gsr_adam_group *groups, int64_t P, const float *relevance, double beta1,
                double beta2, double eps, int *flag_scratch, bool flag_ready, hipStream_t s, float *shrink_raw,
                int64_t shrink_first, float shrink_limit, const float *live3, int64_t skybox, int *row_list) {
    if ((shrink_raw || live3) && adam_elementwise()) {
        set_last_error("sparse Adam: the fused scale shrink / sparse rows need the row-block kernel");
        return GSR_ERR_UNSUPPORTED;
    }
    if (n_groups < 0 || n_groups > kMaxGroups || P < 0 || (P > 0 && (!groups || (relevance && !flag_scratch)))) {
        set_last_error("gsr_sparse_adam_step: bad group count or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (P == 0 || n_groups == 0) return GSR_OK;
    AdamArgs a;
    std::memset(&a, 0, sizeof(a));
    a.n = n_groups;
    int64_t blocks = 0;
    for (int i = 0; i < n_groups; i++) {
        const gsr_adam_group &g = groups[i];
        if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq || g.width <= 0 ||
            (g.row_stride != 0 && g.row_stride < g.width)) {
            set_last_error("gsr_sparse_adam_step: group has a NULL array, non-positive width or row_stride < width");
            return GSR_ERR_INVALID_ARGUMENT;
        }
        a.g[i] = g;
        if (a.g[i].row_stride == 0) a.g[i].row_stride = g.width;
        a.block_start[i] = blocks;
        blocks += (P * g.width + kAdamThreads - 1) / kAdamThreads;
    }
    a.block_start[n_groups] = blocks;
    if (blocks > 0x7fffffff) {
        set_last_error("gsr_sparse_adam_step: parameter set too large for one launch");
        return GSR_ERR_UNSUPPORTED;
    }
    // relevance NULL: a dense step (torch.optim.Adam over every row), one launch
    int *flag = relevance ? flag_scratch : nullptr;
    if (relevance && !flag_ready) {
        (void)hipMemsetAsync(flag_scratch, 0, sizeof(int), s);
        hipLaunchKernelGGL(any_nonzero_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, relevance, P,
                           flag_scratch);
    }
    // torch applies python-float hyper-parameters as fp32 scalars: b, (1 - b) rounded from double
    if (!relevance && !live3 && skybox == 0 && !shrink_raw && !adam_elementwise() && !adam_dense_rows()) {
        // the dense step: flat runs, and the row-block kernel for any group that is not one
        FlatAdamArgs fa;
        int rest[kMaxGroups], n_rest = 0;
        if (flat_adam_runs(n_groups, groups, P, fa, rest, n_rest) > 0)
            hipLaunchKernelGGL(dense_adam_flat_kernel, dim3((unsigned)fa.block_start[fa.n]), dim3(kAdamThreads), 0, s,
                               fa, (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2),
                               (float)eps);
        if (n_rest > 0) {
            AdamArgs ar;
            std::memset(&ar, 0, sizeof(ar));
            ar.n = n_rest;
            for (int j = 0; j < n_rest; j++) ar.g[j] = a.g[rest[j]];
            hipLaunchKernelGGL(sparse_adam_rows_kernel,
                               dim3((unsigned)((P + kAdamThreads - 1) / kAdamThreads), (unsigned)n_rest),
                               dim3(kAdamThreads), 0, s, ar, relevance, P, (float)beta1, (float)beta2,
                               (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps, (const int *)nullptr,
                               ShrinkArgs{nullptr, 0, 0.f}, DenseRows{nullptr, 0}, -1);
        }
    }
    else if (!adam_elementwise())
    {
        // the shrink reads the scales after their Adam update: it runs in the scaling group's wave
        int sh_group = -1;
        for (int i = 0; i < n_groups; i++)
            if (shrink_raw && groups[i].param == shrink_raw) sh_group = i;
        // the compacted form when the row's elements fit one wave (and the shrink, if any, has its
        // three scale lanes)
        AdamLaneMap lm;
        std::memset(&lm, 0, sizeof(lm));
        lm.sh_lane0 = -1;
        bool fits = relevance != nullptr && !adam_rowblock() && (!shrink_raw || (sh_group >= 0 && groups[sh_group].width == 3));
        for (int i = 0; fits && i < n_groups; i++) {
            if (lm.lanes + groups[i].width > kAdamListMaxLanes) {
                fits = false;
                break;
            }
            if (i == sh_group) lm.sh_lane0 = lm.lanes;
            for (int c = 0; c < (int)groups[i].width; c++) {
                lm.group[lm.lanes] = (uint8_t)i;
                lm.col[lm.lanes++] = (uint8_t)c;
            }
        }
        // the row list and its counter: the caller's scratch, or stream-ordered scratch of this call;
        // if that allocation fails the row-block kernel (which needs none) runs instead
        int *buf = row_list;
        bool own = false;
        if (fits && P <= 0x7fffffff && !buf) {
            if (hipMallocAsync(reinterpret_cast<void **>(&buf), sizeof(int) * ((size_t)P + 64), s) == hipSuccess) own = true;
            else {
                (void)hipGetLastError();
                buf = nullptr;
            }
        }
        if (fits && P <= 0x7fffffff && buf) {
            int *count = buf, *list = buf + 64;
            const ShrinkArgs sha{shrink_raw, shrink_first, shrink_limit};
            (void)hipMemsetAsync(count, 0, sizeof(int), s);
            const unsigned cb = (unsigned)std::max<int64_t>(
                1, std::min<int64_t>((P + kCompactThreads - 1) / kCompactThreads, kCompactMaxBlocks));
            hipLaunchKernelGGL(adam_compact_kernel, dim3(cb), dim3(kCompactThreads), 0, s, relevance, P, flag, list,
                               count, sha);
            hipLaunchKernelGGL(adam_rowlist_kernel, dim3(4096), dim3(256), 0, s, a, lm, (const int *)list,
                               (const int *)count, P, flag, (float)beta1, (float)beta2, (float)(1.0 - beta1),
                               (float)(1.0 - beta2), (float)eps, sha, DenseRows{live3, skybox});
            if (own) (void)hipFreeAsync(buf, s);
        } else
            hipLaunchKernelGGL(sparse_adam_rows_kernel,
                           dim3((unsigned)((P + kAdamThreads - 1) / kAdamThreads), (unsigned)n_groups),
                           dim3(kAdamThreads), 0, s, a, relevance, P, (float)beta1, (float)beta2,
                           (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps, flag,
                           ShrinkArgs{shrink_raw, shrink_first, shrink_limit}, DenseRows{live3, skybox}, sh_group);
    }
    else
        hipLaunchKernelGGL(sparse_adam_kernel, dim3((unsigned)blocks), dim3(kAdamThreads), 0, s, a, relevance, P,
                           (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), (float)eps,
                           flag);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_sparse_adam_step: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

// ---- the native step's fused launches (csrc/train_step.hip) -------------------------------------

int step_loss_forward(const float *img, const float *gt, int H, int W, double lambda_dssim, void *loss_scratch,
                      float *gmap, const float *invd, const float *mono, const float *mask, float depth_w,
                      void *depth_scratch, float *d_invd, float *losses, int *flag, hipStream_t s, const float *one,
                      const float *alpha, bool *gmap_is_photo) {
    set_lds_attr();
    const int C = 3;
    const bool tiled = ssim_tiled();
    const dim3 g = tiled ? loss_grid(C, H, W) : stream_grid(C, H, W);
    const int np = (int)(g.x * g.y * g.z);
    float2 *pp = static_cast<float2 *>(loss_scratch);
    if (tiled)
        hipLaunchKernelGGL(l1_ssim_grad_kernel<true>, g, dim3(kLossThreads), kBwdLds, s, img, gt, H, W, ssim_window(),
                           nullptr, 0.f, gmap, pp);
    else
        hipLaunchKernelGGL(l1_ssim_stream_kernel<true>, g, dim3(kStThreads), 0, s, img, gt, H, W, ssim_window(),
                           nullptr, 0.f, gmap, pp, stream_seg(C, H, W),
                           PhotoOut{one, alpha, (float)(1.0 / (double)(3 * (int64_t)H * W)), (float)(1.0 - lambda_dssim),
                                    (float)lambda_dssim});
    if (gmap_is_photo) *gmap_is_photo = !tiled && one != nullptr;
    const int64_t n = (int64_t)H * W;
    const int nd = (int)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
    double *dp = static_cast<double *>(depth_scratch);
    if (mono)
        hipLaunchKernelGGL(depth_l1_fwd_kernel<true>, dim3(nd), dim3(kDepthThreads), 0, s, invd, mono, mask, n, dp,
                           depth_w, 1.0f / (float)n, d_invd);
    hipLaunchKernelGGL(step_finalize_kernel, dim3(1), dim3(1024), 0, s, pp, np, 1.0 / ((double)C * H * W),
                       (float)(1.0 - lambda_dssim), (float)lambda_dssim, mono ? dp : nullptr, nd, 1.0 / (double)n,
                       depth_w, losses, flag);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("step loss forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int step_depth_only_forward(const float *invd, const float *mono, const float *mask, int64_t n, float w, double a,
                            void *depth_scratch, float *d_invd, float *losses, int *flag, hipStream_t s) {
    const int nb = (int)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
    double2 *part = static_cast<double2 *>(depth_scratch);
    const float af = (float)a, omaf = (float)(1.0 - a);
    if (n > 0)
        hipLaunchKernelGGL(depth_only_fwd_kernel<true>, dim3(nb), dim3(kDepthThreads), 0, s, invd, mono, mask, n, part,
                           depth_only_w(1.f, w, af, omaf, 1.0f / (float)n), d_invd);
    else if (hipMemsetAsync(part, 0, sizeof(double2), s) != hipSuccess)
        return GSR_ERR_DEVICE;
    hipLaunchKernelGGL(depth_only_finalize_kernel, dim3(1), dim3(1024), 0, s, part, nb, n > 0 ? 1.0 / (double)n : 0.0,
                       w, af, omaf, losses, flag);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("step depth-only loss: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int launch_exposure_forward(const float *color, const float *E, int64_t npix, float *out, const float *alpha,
                            hipStream_t s) {
    hipLaunchKernelGGL(exposure_fwd_kernel, dim3(exposure_blocks(npix)), dim3(kExpThreads), 0, s, color, E, npix, out,
                       alpha);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("exposure forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int step_loss_backward(const float *img, const float *gt, const float *gmap, const float *one, double lambda_dssim,
                       const float *alpha, const float *color, const float *E_view, int64_t npix, float *d_color,
                       void *exp_scratch, int n_images, int view, const gsr_adam_group &eg, float *exposure_grad,
                       double b1, double b2, double eps, hipStream_t s, bool gmap_is_photo) {
    const int nb = exposure_blocks(npix);
    float *part = static_cast<float *>(exp_scratch);
    const PhotoGrad pg{img, gt, gmap, one, alpha, (float)(1.0 / (double)(3 * npix)), (float)(1.0 - lambda_dssim),
                       (float)lambda_dssim};
    if (gmap_is_photo)  // the SSIM pass already formed the photometric gradient (PhotoOut)
        hipLaunchKernelGGL(exposure_bwd_kernel<false>, dim3(nb), dim3(kExpThreads), 0, s, color, E_view, npix, gmap,
                           d_color, part, pg);
    else
        hipLaunchKernelGGL(exposure_bwd_kernel<true>, dim3(nb), dim3(kExpThreads), 0, s, color, E_view, npix, nullptr,
                           d_color, part, pg);
    hipLaunchKernelGGL(exposure_finalize_adam_kernel, dim3(1), dim3(768), 0, s, part, nb, n_images, view, eg,
                       exposure_grad, (float)b1, (float)b2, (float)(1.0 - b1), (float)(1.0 - b2), (float)eps);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("step loss backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int step_activate_backward(int64_t P, const float *rotation_raw, const float *scales, const float *opac,
                           const float *d_scales, const float *d_rots, const float *d_opac, float *scaling_grad,
                           float *rotation_grad, float *opacity_grad, int64_t skybox, int *flag, const int *radii,
                           const float *d_means2D, float *max_radii2D, float *accum, float *denom, hipStream_t s,
                           bool sparse_rows, const float *scaling_raw, const float *opacity_raw) {
    hipLaunchKernelGGL(activate_bwd_step_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, P,
                       reinterpret_cast<const float4 *>(rotation_raw), scales, opac, d_scales,
                       reinterpret_cast<const float4 *>(d_rots), d_opac, scaling_grad,
                       reinterpret_cast<float4 *>(rotation_grad), opacity_grad, skybox, flag, radii, d_means2D,
                       max_radii2D, accum, denom, sparse_rows ? 1 : 0, scaling_raw, opacity_raw);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("step activation backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // namespace gsr

using namespace gsr;

extern "C" {

size_t gsr_l1_ssim_scratch_bytes(int C, int H, int W) {
    if (C <= 0 || H <= 0 || W <= 0) return 0;
    const dim3 g = loss_grid(C, H, W), gs = stream_grid(C, H, W);
    return sizeof(float2) * std::max<size_t>((size_t)g.x * g.y * g.z, (size_t)gs.x * gs.y * gs.z);
}

int gsr_l1_ssim_forward(const float *img, const float *gt, int C, int H, int W, void *scratch, float *out,
                        void *stream) {
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !scratch || !out) {
        set_last_error("gsr_l1_ssim_forward: empty image or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    set_lds_attr();
    const dim3 g = loss_grid(C, H, W);
    const int nb = (int)(g.x * g.y * g.z);
    float2 *part = static_cast<float2 *>(scratch);
    hipLaunchKernelGGL(l1_ssim_fwd_kernel, g, dim3(kLossThreads), kFwdLds, s, img, gt, H, W, ssim_window(), part);
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), 0, s, part, nb, 1.0 / ((double)C * H * W), out,
                       -1.f, 0.f);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_l1_ssim_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_l1_ssim_backward(const float *img, const float *gt, int C, int H, int W, const float *dL_dout,
                         float *dL_dimg, void *stream) {
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !dL_dout || !dL_dimg) {
        set_last_error("gsr_l1_ssim_backward: empty image or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    set_lds_attr();
    const float inv_n = (float)(1.0 / ((double)C * H * W));
    if (ssim_tiled())
        hipLaunchKernelGGL(l1_ssim_grad_kernel<false>, loss_grid(C, H, W), dim3(kLossThreads), kBwdLds, s, img, gt, H,
                           W, ssim_window(), dL_dout, inv_n, dL_dimg, nullptr);
    else
        hipLaunchKernelGGL(l1_ssim_stream_kernel<false>, stream_grid(C, H, W), dim3(kStThreads), 0, s, img, gt, H,
                           W, ssim_window(), dL_dout, inv_n, dL_dimg, nullptr, stream_seg(C, H, W), PhotoOut{});
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_l1_ssim_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"

namespace {

// w_l1 < 0: out = (L1, SSIM); else also out[2] = the photo loss with weights (w_l1, w_ssim)
int forward_with_map(const char *who, const float *img, const float *gt, int C, int H, int W, void *scratch,
                     float *out, float *ssim_grad_map, float w_l1, float w_ssim, void *stream) {
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !scratch || !out || !ssim_grad_map) {
        set_last_error(std::string(who) + ": empty image or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    set_lds_attr();
    const bool tiled = ssim_tiled();
    const dim3 g = tiled ? loss_grid(C, H, W) : stream_grid(C, H, W);
    const int nb = (int)(g.x * g.y * g.z);
    float2 *part = static_cast<float2 *>(scratch);
    if (tiled)
        hipLaunchKernelGGL(l1_ssim_grad_kernel<true>, g, dim3(kLossThreads), kBwdLds, s, img, gt, H, W, ssim_window(),
                           nullptr, 0.f, ssim_grad_map, part);
    else
        hipLaunchKernelGGL(l1_ssim_stream_kernel<true>, g, dim3(kStThreads), 0, s, img, gt, H, W, ssim_window(),
                           nullptr, 0.f, ssim_grad_map, part, stream_seg(C, H, W), PhotoOut{});
    hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), 0, s, part, nb, 1.0 / ((double)C * H * W), out,
                       w_l1, w_ssim);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string(who) + ": " + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int backward_from_map(const char *who, const float *img, const float *gt, const float *ssim_grad_map, int C, int H,
                      int W, const float *dL_dout, float w_l1, float w_ssim, float *dL_dimg, void *stream) {
    if (C <= 0 || H <= 0 || W <= 0 || !img || !gt || !ssim_grad_map || !dL_dout || !dL_dimg) {
        set_last_error(std::string(who) + ": empty image or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)C * H * W;
    const float inv_n = (float)(1.0 / (double)n);
    const bool vec = ((reinterpret_cast<uintptr_t>(img) | reinterpret_cast<uintptr_t>(gt) |
                       reinterpret_cast<uintptr_t>(ssim_grad_map) | reinterpret_cast<uintptr_t>(dL_dimg)) & 15) == 0;
    const int64_t n4 = vec ? n / 4 : 0;
    if (n4 > 0) {
        const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 256 * 8);
        hipLaunchKernelGGL(l1_ssim_bwd_map_kernel, dim3(blocks), dim3(256), 0, s,
                           reinterpret_cast<const float4 *>(img), reinterpret_cast<const float4 *>(gt),
                           reinterpret_cast<const float4 *>(ssim_grad_map), n4, dL_dout, inv_n,
                           reinterpret_cast<float4 *>(dL_dimg), w_l1, w_ssim);
    }
    if (4 * n4 < n) {
        const int64_t rest = n - 4 * n4;
        hipLaunchKernelGGL(l1_ssim_bwd_map_tail_kernel, dim3((unsigned)((rest + 255) / 256)), dim3(256), 0, s, img, gt,
                           ssim_grad_map, 4 * n4, n, dL_dout, inv_n, dL_dimg, w_l1, w_ssim);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string(who) + ": " + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

bool bad_lambda(const char *who, double lambda_dssim) {
    if (!(lambda_dssim >= 0.0 && lambda_dssim <= 1.0)) {
        set_last_error(std::string(who) + ": lambda_dssim outside [0, 1]");
        return true;
    }
    return false;
}

}  // namespace

extern "C" {

int gsr_l1_ssim_forward_with_map(const float *img, const float *gt, int C, int H, int W, void *scratch, float *out,
                                 float *ssim_grad_map, void *stream) {
    return forward_with_map("gsr_l1_ssim_forward_with_map", img, gt, C, H, W, scratch, out, ssim_grad_map, -1.f, 0.f,
                            stream);
}

int gsr_l1_ssim_backward_from_map(const float *img, const float *gt, const float *ssim_grad_map, int C, int H, int W,
                                  const float *dL_dout, float *dL_dimg, void *stream) {
    return backward_from_map("gsr_l1_ssim_backward_from_map", img, gt, ssim_grad_map, C, H, W, dL_dout, -1.f, 0.f,
                             dL_dimg, stream);
}

int gsr_photo_loss_forward(const float *img, const float *gt, int C, int H, int W, double lambda_dssim, void *scratch,
                           float *out3, float *ssim_grad_map, void *stream) {
    if (bad_lambda("gsr_photo_loss_forward", lambda_dssim)) return GSR_ERR_INVALID_ARGUMENT;
    // torch applies the python floats (1 - lambda) and lambda as fp32 scalars
    return forward_with_map("gsr_photo_loss_forward", img, gt, C, H, W, scratch, out3, ssim_grad_map,
                            (float)(1.0 - lambda_dssim), (float)lambda_dssim, stream);
}

int gsr_photo_loss_backward(const float *img, const float *gt, const float *ssim_grad_map, int C, int H, int W,
                            double lambda_dssim, const float *dL_dloss, float *dL_dimg, void *stream) {
    if (bad_lambda("gsr_photo_loss_backward", lambda_dssim)) return GSR_ERR_INVALID_ARGUMENT;
    return backward_from_map("gsr_photo_loss_backward", img, gt, ssim_grad_map, C, H, W, dL_dloss,
                             (float)(1.0 - lambda_dssim), (float)lambda_dssim, dL_dimg, stream);
}

int gsr_sparse_adam_step(int n_groups, const gsr_adam_group *groups, int64_t P, const float *relevance,
                         double beta1, double beta2, double eps, int *flag_scratch, void *stream) {
    return gsr::sparse_adam(n_groups, groups, P, relevance, beta1, beta2, eps, flag_scratch, false,
                            static_cast<hipStream_t>(stream), nullptr, 0, 0.f);
}

int gsr_exposure_forward(const float *color, const float *exposure, int64_t npix, float *out, void *stream) {
    if (npix < 0 || (npix > 0 && (!color || !exposure || !out))) {
        set_last_error("gsr_exposure_forward: NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (npix == 0) return GSR_OK;
    hipLaunchKernelGGL(exposure_fwd_kernel, dim3(exposure_blocks(npix)), dim3(kExpThreads), 0,
                       static_cast<hipStream_t>(stream), color, exposure, npix, out, nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_exposure_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

size_t gsr_exposure_scratch_bytes(int64_t npix) { return sizeof(float) * 12 * (size_t)exposure_blocks(npix); }

int gsr_exposure_backward(const float *color, const float *exposure, int64_t npix, const float *dL_dout,
                          float *dL_dcolor, float *dL_dexposure, void *scratch, void *stream) {
    if (npix < 0 || !dL_dexposure || !scratch || (npix > 0 && (!color || !exposure || !dL_dout || !dL_dcolor))) {
        set_last_error("gsr_exposure_backward: NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nb = exposure_blocks(npix);
    float *part = static_cast<float *>(scratch);
    if (npix > 0)
        hipLaunchKernelGGL(exposure_bwd_kernel<false>, dim3(nb), dim3(kExpThreads), 0, s, color, exposure, npix,
                           dL_dout, dL_dcolor, part, PhotoGrad{});
    else
        (void)hipMemsetAsync(part, 0, sizeof(float) * 12, s);
    hipLaunchKernelGGL(exposure_finalize_kernel, dim3(1), dim3(768), 0, s, part, npix > 0 ? nb : 1, dL_dexposure);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_exposure_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_densify_stats(int64_t P, const int *radii, const float *dL_dmeans2D, float *max_radii2D, float *grad_accum,
                      float *denom, void *stream) {
    if (P < 0 || (P > 0 && (!radii || !dL_dmeans2D || !max_radii2D || !grad_accum || !denom))) {
        set_last_error("gsr_densify_stats: NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (P == 0) return GSR_OK;
    hipLaunchKernelGGL(densify_stats_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), P, radii, dL_dmeans2D, max_radii2D, grad_accum, denom);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_densify_stats: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_activate_forward(int64_t P, const float *scaling_raw, const float *rotation_raw, const float *opacity_raw,
                         float *scales, float *rotations, float *opacities, void *stream) {
    if (P < 0 || (P > 0 && (!scaling_raw || !rotation_raw || !opacity_raw || !scales || !rotations || !opacities)) ||
        (P > 0 && ((reinterpret_cast<uintptr_t>(rotation_raw) | reinterpret_cast<uintptr_t>(rotations)) & 15))) {
        set_last_error("gsr_activate_forward: NULL or misaligned (rotations need 16 B) pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (P == 0) return GSR_OK;
    hipLaunchKernelGGL(activate_fwd_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), P, scaling_raw,
                       reinterpret_cast<const float4 *>(rotation_raw), opacity_raw, scales,
                       reinterpret_cast<float4 *>(rotations), opacities);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_activate_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_activate_backward(int64_t P, const float *rotation_raw, const float *scales, const float *opacities,
                          const float *dL_dscales, const float *dL_drotations, const float *dL_dopacities,
                          float *dL_dscaling_raw, float *dL_drotation_raw, float *dL_dopacity_raw, void *stream) {
    if (P < 0 || (P > 0 && (!rotation_raw || !scales || !opacities || !dL_dscales || !dL_drotations ||
                            !dL_dopacities || !dL_dscaling_raw || !dL_drotation_raw || !dL_dopacity_raw)) ||
        (P > 0 && ((reinterpret_cast<uintptr_t>(rotation_raw) | reinterpret_cast<uintptr_t>(dL_drotations) |
                    reinterpret_cast<uintptr_t>(dL_drotation_raw)) & 15))) {
        set_last_error("gsr_activate_backward: NULL or misaligned (rotations need 16 B) pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (P == 0) return GSR_OK;
    hipLaunchKernelGGL(activate_bwd_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), P, reinterpret_cast<const float4 *>(rotation_raw), scales,
                       opacities, dL_dscales, reinterpret_cast<const float4 *>(dL_drotations), dL_dopacities,
                       dL_dscaling_raw, reinterpret_cast<float4 *>(dL_drotation_raw), dL_dopacity_raw);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_activate_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_shrink_scales(int64_t P, int64_t first_row, float *scaling_raw, float max_scale, void *stream) {
    if (P < 0 || first_row < 0 || (P > 0 && !scaling_raw)) {
        set_last_error("gsr_shrink_scales: bad sizes or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (first_row >= P) return GSR_OK;
    const int64_t n = P - first_row;
    hipLaunchKernelGGL(shrink_scales_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), P, first_row, scaling_raw, max_scale);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_shrink_scales: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

size_t gsr_depth_l1_scratch_bytes(int64_t n) {
    return sizeof(double) * (size_t)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
}

int gsr_depth_l1_forward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                         float weight, void *scratch, float *out2, void *stream) {
    if (n < 0 || (n > 0 && (!invdepth || !mono_invdepth || !scratch)) || !out2) {
        set_last_error("gsr_depth_l1_forward: bad size or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    const bool aligned = (reinterpret_cast<uintptr_t>(invdepth) | reinterpret_cast<uintptr_t>(mono_invdepth) |
                          reinterpret_cast<uintptr_t>(mask)) % 16 == 0;
    if (!aligned) {
        set_last_error("gsr_depth_l1_forward: arrays must be 16-byte aligned");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nb = (int)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
    double *part = static_cast<double *>(scratch);
    if (n > 0)
        hipLaunchKernelGGL(depth_l1_fwd_kernel<false>, dim3(nb), dim3(kDepthThreads), 0, s, invdepth, mono_invdepth,
                           mask, n, part, 0.f, 0.f, nullptr);
    else if (hipMemsetAsync(part, 0, sizeof(double), s) != hipSuccess)
        return GSR_ERR_DEVICE;
    hipLaunchKernelGGL(depth_l1_finalize_kernel, dim3(1), dim3(1024), 0, s, part, nb,
                       n > 0 ? 1.0 / (double)n : 0.0, weight, out2);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_depth_l1_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_depth_l1_backward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                          float weight, const float *dL_dloss, float *dL_dinvdepth, void *stream) {
    if (n < 0 || (n > 0 && (!invdepth || !mono_invdepth || !dL_dloss || !dL_dinvdepth))) {
        set_last_error("gsr_depth_l1_backward: bad size or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return GSR_OK;
    hipLaunchKernelGGL(depth_l1_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), invdepth, mono_invdepth, mask, n, dL_dloss, weight,
                       1.0f / (float)n, dL_dinvdepth);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_depth_l1_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

size_t gsr_depth_only_scratch_bytes(int64_t n) {
    return sizeof(double2) * (size_t)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
}

int gsr_depth_only_loss_forward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                                float weight, double dens_weight, void *scratch, float *out3, void *stream) {
    if (n < 0 || (n > 0 && (!invdepth || !mono_invdepth)) || !scratch || !out3 ||
        !(dens_weight >= 0.0 && dens_weight <= 1.0)) {
        set_last_error("gsr_depth_only_loss_forward: bad size, weight or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if ((reinterpret_cast<uintptr_t>(invdepth) | reinterpret_cast<uintptr_t>(mono_invdepth) |
         reinterpret_cast<uintptr_t>(mask)) % 16 != 0) {
        set_last_error("gsr_depth_only_loss_forward: arrays must be 16-byte aligned");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int nb = (int)std::max<int64_t>(1, (n + kDepthPerBlock - 1) / kDepthPerBlock);
    double2 *part = static_cast<double2 *>(scratch);
    const float af = (float)dens_weight, omaf = (float)(1.0 - dens_weight);
    if (n > 0)
        hipLaunchKernelGGL(depth_only_fwd_kernel<false>, dim3(nb), dim3(kDepthThreads), 0, s, invdepth, mono_invdepth,
                           mask, n, part, DepthOnlyW{0.f, 0.f}, nullptr);
    else if (hipMemsetAsync(part, 0, sizeof(double2), s) != hipSuccess)
        return GSR_ERR_DEVICE;
    hipLaunchKernelGGL(depth_only_finalize_kernel, dim3(1), dim3(1024), 0, s, part, nb,
                       n > 0 ? 1.0 / (double)n : 0.0, weight, af, omaf, out3, nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_depth_only_loss_forward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

int gsr_depth_only_loss_backward(const float *invdepth, const float *mono_invdepth, const float *mask, int64_t n,
                                 float weight, double dens_weight, const float *dL_dloss, float *dL_dinvdepth,
                                 void *stream) {
    if (n < 0 || (n > 0 && (!invdepth || !mono_invdepth || !dL_dloss || !dL_dinvdepth)) ||
        !(dens_weight >= 0.0 && dens_weight <= 1.0)) {
        set_last_error("gsr_depth_only_loss_backward: bad size, weight or NULL pointer");
        return GSR_ERR_INVALID_ARGUMENT;
    }
    if (n == 0) return GSR_OK;
    hipLaunchKernelGGL(depth_only_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), invdepth, mono_invdepth, mask, n, dL_dloss, weight,
                       (float)dens_weight, (float)(1.0 - dens_weight), 1.0f / (float)n, dL_dinvdepth);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_last_error(std::string("gsr_depth_only_loss_backward: ") + hipGetErrorString(e));
        return GSR_ERR_DEVICE;
    }
    return GSR_OK;
}

}  // extern "C"
