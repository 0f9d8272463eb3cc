// gsr_device.h -- device-side maths and state layouts shared by the gfx950 kernels.
//
// Every index-producing expression (projection, EWA covariance, radius, tile rect, depth key)
// is evaluated in a fixed IEEE operation order and compiled with -ffp-contract=off, so the
// integer outputs (radii, tiles, keys, ranges, n_contrib away from exp() ulp ties) are
// reproducible bit for bit by the CPU restatement in oracle/gs_oracle.c.
//
// Algorithm: the graphdeco 3DGS / hierarchy-rasterizer preprocess,
// whose CUDA source is not vendored in the reference; the pure-Python twins it must agree
// with are utils/sh_utils.py:57-112 (SH), scene/gaussian_model.py:33-37 +
// utils/general_utils.py:68-114 (cov3D) and scene/cameras.py:96-99 (matrices).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

constexpr int kTile = 16;              // 16x16 pixel tiles (T = ceil(W/16)*ceil(H/16))
constexpr int kWave = 64;              // CDNA wavefront
constexpr int kPixPerLane = kTile * kTile / kWave;  // 4: one wave owns one tile

// ---- SH constants: utils/sh_utils.py:26-43 ----
#define GSR_SH_C0 0.28209479177387814f
#define GSR_SH_C1 0.4886025119029199f
#define GSR_SH_C2_0 1.0925484305920792f
#define GSR_SH_C2_1 -1.0925484305920792f
#define GSR_SH_C2_2 0.31539156525252005f
#define GSR_SH_C2_3 -1.0925484305920792f
#define GSR_SH_C2_4 0.5462742152960396f
#define GSR_SH_C3_0 -0.5900435899266435f
#define GSR_SH_C3_1 2.890611442640554f
#define GSR_SH_C3_2 -0.4570457994644658f
#define GSR_SH_C3_3 0.3731763325901154f
#define GSR_SH_C3_4 -0.4570457994644658f
#define GSR_SH_C3_5 1.445305721320277f
#define GSR_SH_C3_6 -0.5900435899266435f

__device__ __forceinline__ float fmin_(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float fmax_(float a, float b) { return a > b ? a : b; }

struct Mat4 {  // column-major 4x4 held in registers (wave-uniform -> SGPRs)
    float m[16];
};

__device__ __forceinline__ Mat4 load_mat4(const float *__restrict__ p) {
    Mat4 r;
    const float4 *q = reinterpret_cast<const float4 *>(p);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float4 v = q[i];
        r.m[4 * i + 0] = v.x; r.m[4 * i + 1] = v.y; r.m[4 * i + 2] = v.z; r.m[4 * i + 3] = v.w;
    }
    return r;
}

__device__ __forceinline__ float3 xf_point43(float3 p, const Mat4 &M) {
    const float *m = M.m;
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}

__device__ __forceinline__ float4 xf_point44(float3 p, const Mat4 &M) {
    const float *m = M.m;
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                       m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// upstream evaluates ((v + 1.0) * S - 1.0) * 0.5 in double
__device__ __forceinline__ float ndc2pix(float v, int S) {
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

struct Rect { int x0, y0, x1, y1; };

__device__ __forceinline__ int clampi(int a, int hi) { a = a > 0 ? a : 0; return a < hi ? a : hi; }

__device__ __forceinline__ Rect get_rect(float px, float py, int r, int gx, int gy) {
    Rect R;
    R.x0 = clampi((int)((px - (float)r) / (float)kTile), gx);
    R.y0 = clampi((int)((py - (float)r) / (float)kTile), gy);
    R.x1 = clampi((int)((px + (float)r + (float)(kTile - 1)) / (float)kTile), gx);
    R.y1 = clampi((int)((py + (float)r + (float)(kTile - 1)) / (float)kTile), gy);
    return R;
}

struct Rot3 { float m[3][3]; };

__device__ __forceinline__ Rot3 quat_to_rot(float4 q) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    Rot3 R;
    R.m[0][0] = 1.f - 2.f * (y * y + z * z); R.m[0][1] = 2.f * (x * y - r * z); R.m[0][2] = 2.f * (x * z + r * y);
    R.m[1][0] = 2.f * (x * y + r * z); R.m[1][1] = 1.f - 2.f * (x * x + z * z); R.m[1][2] = 2.f * (y * z - r * x);
    R.m[2][0] = 2.f * (x * z - r * y); R.m[2][1] = 2.f * (y * z + r * x); R.m[2][2] = 1.f - 2.f * (x * x + y * y);
    return R;
}

// cov3D = (R S)(R S)^T, S = diag(mod * s); 6-pack xx,xy,xz,yy,yz,zz
__device__ __forceinline__ void cov3d_from_scale_rot(float3 s_in, float mod, float4 q, float c[6]) {
    const float sx = mod * s_in.x, sy = mod * s_in.y, sz = mod * s_in.z;
    Rot3 R = quat_to_rot(q);
    float L[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++) { L[i][0] = R.m[i][0] * sx; L[i][1] = R.m[i][1] * sy; L[i][2] = R.m[i][2] * sz; }
    c[0] = L[0][0] * L[0][0] + L[0][1] * L[0][1] + L[0][2] * L[0][2];
    c[1] = L[0][0] * L[1][0] + L[0][1] * L[1][1] + L[0][2] * L[1][2];
    c[2] = L[0][0] * L[2][0] + L[0][1] * L[2][1] + L[0][2] * L[2][2];
    c[3] = L[1][0] * L[1][0] + L[1][1] * L[1][1] + L[1][2] * L[1][2];
    c[4] = L[1][0] * L[2][0] + L[1][1] * L[2][1] + L[1][2] * L[2][2];
    c[5] = L[2][0] * L[2][0] + L[2][1] * L[2][1] + L[2][2] * L[2][2];
}

struct Ewa {
    float m0[3], m1[3];  // first two rows of J * W_view
    float3 t;            // view-space mean with the 1.3*tanfov clamp applied
    float xmul, ymul;    // 0 where the clamp is active (gradient mask)
};

__device__ __forceinline__ Ewa ewa_rows(float3 mean, const Mat4 &V, float fx, float fy, float tanx, float tany) {
    Ewa e;
    float3 t = xf_point43(mean, V);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    e.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    e.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    t.x = fmin_(limx, fmax_(-limx, txtz)) * t.z;
    t.y = fmin_(limy, fmax_(-limy, tytz)) * t.z;
    const float j00 = fx / t.z, j02 = -(fx * t.x) / (t.z * t.z);
    const float j11 = fy / t.z, j12 = -(fy * t.y) / (t.z * t.z);
    const float *v = V.m;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        e.m0[c] = j00 * v[4 * c + 0] + j02 * v[4 * c + 2];
        e.m1[c] = j11 * v[4 * c + 1] + j12 * v[4 * c + 2];
    }
    e.t = t;
    return e;
}

__device__ __forceinline__ float quad_form(const float a[3], const float c[6], const float b[3]) {
    const float s0 = c[0] * b[0] + c[1] * b[1] + c[2] * b[2];
    const float s1 = c[1] * b[0] + c[3] * b[1] + c[4] * b[2];
    const float s2 = c[2] * b[0] + c[4] * b[1] + c[5] * b[2];
    return a[0] * s0 + a[1] * s1 + a[2] * s2;
}

// A hierarchy cut read in place (render_post's LOD blend fused into the preprocess and the SH colour
// pass): row r of the frame is t x[c] + (1 - t) x[p] with c = ri[r], p = pi[r] (-1: the last of the
// N rows, as torch's gather reads it), t = w[r], and the parent quaternion sign-aligned to the
// child's -- the expressions of hier.hip's cut_fwd_kernel (gaussian_renderer/__init__.py:200-220),
// so the fused frame's rows are bitwise the materialised blend's.  ri == nullptr: no cut.
struct CutRef {
    const int *ri, *pi;
    const float *w;
    int64_t N;
};
__device__ __forceinline__ float cut_lerp(float t, float a, float b) { return t * a + (1.f - t) * b; }
__device__ __forceinline__ void cut_source(const CutRef &c, int64_t r, int64_t &ci, int64_t &pi, float &t) {
    ci = c.ri[r];
    pi = c.pi[r];
    if (pi < 0) pi += c.N;
    t = c.w[r];
}

// Parameter activations (scene/gaussian_model.py:39-47, getters :125-156), in torch's op order:
// exp, x / max(||x||, 1e-12), sigmoid.  train.hip's activate kernels and the raw-parameter mode of
// the rasterizer (GaussianInputs.raw: the native train step) use these, so both form the same bits.
__device__ __forceinline__ float act_scale(float s) { return expf(s); }
__device__ __forceinline__ float4 act_rot(float4 q) {
    const float d = fmaxf(sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w), 1e-12f);
    return make_float4(q.x / d, q.y / d, q.z / d, q.w / d);
}
__device__ __forceinline__ float act_opacity(float o) { return 1.f / (1.f + expf(-o)); }

__device__ __forceinline__ void sh_dir(float3 mean, float3 campos, float dir[3], float dor[3]) {
    dor[0] = mean.x - campos.x;
    dor[1] = mean.y - campos.y;
    dor[2] = mean.z - campos.z;
    const float len = sqrtf(dor[0] * dor[0] + dor[1] * dor[1] + dor[2] * dor[2]);
    dir[0] = dor[0] / len; dir[1] = dor[1] / len; dir[2] = dor[2] / len;
}

// SH -> RGB for one channel; sh points at coefficient 0 of that channel, stride 3 floats
__device__ __forceinline__ float sh_channel(int deg, const float *sh, float x, float y, float z) {
    float r = GSR_SH_C0 * sh[0];
    if (deg > 0) {
        r = r - GSR_SH_C1 * y * sh[1 * 3] + GSR_SH_C1 * z * sh[2 * 3] - GSR_SH_C1 * x * sh[3 * 3];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            r = r + GSR_SH_C2_0 * xy * sh[4 * 3] + GSR_SH_C2_1 * yz * sh[5 * 3] +
                GSR_SH_C2_2 * (2.0f * zz - xx - yy) * sh[6 * 3] + GSR_SH_C2_3 * xz * sh[7 * 3] +
                GSR_SH_C2_4 * (xx - yy) * sh[8 * 3];
            if (deg > 2) {
                r = r + GSR_SH_C3_0 * y * (3.0f * xx - yy) * sh[9 * 3] + GSR_SH_C3_1 * xy * z * sh[10 * 3] +
                    GSR_SH_C3_2 * y * (4.0f * zz - xx - yy) * sh[11 * 3] +
                    GSR_SH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * sh[12 * 3] +
                    GSR_SH_C3_4 * x * (4.0f * zz - xx - yy) * sh[13 * 3] + GSR_SH_C3_5 * z * (xx - yy) * sh[14 * 3] +
                    GSR_SH_C3_6 * x * (xx - 3.0f * yy) * sh[15 * 3];
            }
        }
    }
    return r + 0.5f;
}

// True if some pixel centre of the box [x0, x1] x [y0, y1] may reach alpha >= 1/255, i.e. the
// conic form Q(d) = a dx^2 + 2 b dx dy + c dy^2 (power = -Q/2) gets down to tau = 2 ln(255 op)
// somewhere on the box.  The minimum of the convex Q over a box not containing the centre lies on
// a face turned towards the centre; each face is a 1-D quadratic minimised in closed form.  `tm`
// is tau with a relative + absolute margin (formed once by the preprocess, GRec.cull_tm) that
// keeps the test conservative against the kernels' float evaluation of power and exp, so culling
// with it never changes an output.  The face minimiser comes from an approximate reciprocal: any
// point of the face bounds the face minimum from above, here by O(ulp^2) of Q -- far inside the
// margin.
__device__ __forceinline__ bool ellipse_meets_box(float cx, float cy, float a, float b, float c, float tm, float x0,
                                                  float x1, float y0, float y1) {
    if (!(a > 0.f && c > 0.f)) return true;
    const float X0 = x0 - cx, X1 = x1 - cx, Y0 = y0 - cy, Y1 = y1 - cy;
    const bool outx = X0 > 0.f || X1 < 0.f, outy = Y0 > 0.f || Y1 < 0.f;
    if (!outx && !outy) return true;
    float q = 3.0e38f;
    if (outx) {
        const float xe = X0 > 0.f ? X0 : X1;
        const float ys = fminf(fmaxf(-b * xe * __builtin_amdgcn_rcpf(c), Y0), Y1);
        q = fminf(q, fmaf(a * xe, xe, fmaf(2.f * b * xe, ys, c * ys * ys)));
    }
    if (outy) {
        const float ye = Y0 > 0.f ? Y0 : Y1;
        const float xs = fminf(fmaxf(-b * ye * __builtin_amdgcn_rcpf(a), X0), X1);
        q = fminf(q, fmaf(a * xs, xs, fmaf(2.f * b * xs, ye, c * ye * ye)));
    }
    return q <= tm;
}

// ------------------------------------------------------------------------------------------
// Wave64 primitives (DPP; no LDS)
// ------------------------------------------------------------------------------------------
template <int kCtrl, int kRowMask = 0xF, int kBankMask = 0xF>
__device__ __forceinline__ float dpp_f(float src) {
    return __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(src), kCtrl, kRowMask, kBankMask, false));
}

// Sum over the 64 lanes; result is wave-uniform.  Requires a full exec mask.
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1>(v);        // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);        // quad_perm [2,3,0,1]
    v += dpp_f<0x124>(v);       // row_ror:4
    v += dpp_f<0x128>(v);       // row_ror:8  -> every lane holds its row (16 lanes) sum
    v += dpp_f<0x142, 0xA>(v);  // row_bcast:15 -> rows 1,3 += rows 0,2
    v += dpp_f<0x143, 0xC>(v);  // row_bcast:31 -> rows 2,3 += lane 31
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Sum each of N independent values over the 64 lanes; every lane receives every total.
// Stage-major order (each DPP stage issued for all N values before the next) lets the N chains
// hide each other's DPP read-after-write hazards instead of padding every step with s_nop.
// Rows of 16 are reduced with DPP (quad_perm, row_ror); the row pairs and wave halves are
// combined with gfx950's v_permlane16_swap / v_permlane32_swap (no LDS, no readlane).
template <int N>
__device__ __forceinline__ void wave_allreduce(float *v) {
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_f<0xB1>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_f<0x4E>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_f<0x124>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) v[i] += dpp_f<0x128>(v[i]);
#pragma unroll
    for (int i = 0; i < N; i++) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i]), false, false);
        v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
}

// Sum each of N values over its 16-lane row; every lane of row r receives row r's totals.  The
// four row partials are combined later, off the per-instance path.  Written as one asm block of
// fused DPP adds (v_add_f32 with a quad_perm / row_ror source modifier), stage-major over the N
// values: left to the compiler, the SLP vectoriser pairs the adds into v_pk_add_f32 fed by
// separate v_mov_b32_dpp + register-pair moves, ~2.5x the instructions.  The leading s_nop
// covers the VALU-write -> DPP-read hazard of the first stage; later stages read values
// written >= N-1 instructions earlier.
template <int N>
__device__ __forceinline__ void wave_rowsum(float *v);

#define GSR_DPP_STAGE(CTRL)                                                                               \
    "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %6, %6, %6 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %7, %7, %7 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %8, %8, %8 " CTRL " row_mask:0xf bank_mask:0xf\n"                                       \
    "v_add_f32_dpp %9, %9, %9 " CTRL " row_mask:0xf bank_mask:0xf\n"

template <>
__device__ __forceinline__ void wave_rowsum<10>(float *v) {
    asm volatile("s_nop 1\n" GSR_DPP_STAGE("quad_perm:[1,0,3,2]") GSR_DPP_STAGE("quad_perm:[2,3,0,1]")
                     GSR_DPP_STAGE("row_ror:4") GSR_DPP_STAGE("row_ror:8")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                   "+v"(v[7]), "+v"(v[8]), "+v"(v[9]));
}
#undef GSR_DPP_STAGE

#define GSR_DPP_BCAST15(I) "v_add_f32_dpp %" #I ", %" #I ", %" #I " row_bcast:15 row_mask:0xa bank_mask:0xf\n"
// wave_rowsum, then rows 1 and 3 add the row before them (row_bcast:15): lanes 16-31 hold
// rows 0+1 and lanes 48-63 rows 2+3 -- two half-wave partials per value.
template <int N>
__device__ __forceinline__ void wave_halfsum(float *v);

template <>
__device__ __forceinline__ void wave_halfsum<10>(float *v) {
    wave_rowsum<10>(v);
    asm volatile("s_nop 1\n" GSR_DPP_BCAST15(0) GSR_DPP_BCAST15(1) GSR_DPP_BCAST15(2) GSR_DPP_BCAST15(3)
                     GSR_DPP_BCAST15(4) GSR_DPP_BCAST15(5) GSR_DPP_BCAST15(6) GSR_DPP_BCAST15(7)
                         GSR_DPP_BCAST15(8) GSR_DPP_BCAST15(9)
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                   "+v"(v[7]), "+v"(v[8]), "+v"(v[9]));
}
#undef GSR_DPP_BCAST15

template <>
__device__ __forceinline__ void wave_halfsum<9>(float *v) {
    float t[10];
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = v[i];
    t[9] = 0.f;
    wave_halfsum<10>(t);
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = t[i];
}

// N = 9 (no depth term): pad with a dummy value so one asm block serves both.
template <>
__device__ __forceinline__ void wave_rowsum<9>(float *v) {
    float t[10];
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = v[i];
    t[9] = 0.f;
    wave_rowsum<10>(t);
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = t[i];
}

// Reduce-scatter of 10 values over every 16-lane row, then rows 0+1 and 2+3 added: each lane
// ends with ONE half-wave partial, of value index wave_rs10_slot(lane) (-1: a padding slot).
// Four exchange stages (partners l^8, l^7, l^2, l^1 -- row_ror:8, row_half_mirror and two
// quad_perms; after each, a lane keeps half of its values, chosen by one bit of its index).  In
// the first two stages that bit is a DPP bank bit (bank = 4-lane group: bit 3 splits banks {0,1}
// from {2,3}, bit 2 banks {0,2} from {1,3}), so each kept value is ONE bank-masked DPP add per
// half -- own + partner's copy of the SAME value -- with no selects (10 + 5 VALU instead of
// 15 + 9); the last two stages select within a bank (6 + 3).  Sums are formed in the same order
// as before (partner + own), so the bits do not change.
#define GSR_DPP_RS(CTRL, I, N) "v_add_f32_dpp %" #I ", %" #N ", %" #I " " CTRL " row_mask:0xf bank_mask:0xf\n"
#define GSR_DPP_KEEP(CTRL, BANKS, D, S) "v_add_f32_dpp %" #D ", %" #S ", %" #S " " CTRL " row_mask:0xf bank_mask:" BANKS "\n"
__device__ __forceinline__ float wave_rs10(const float *v, int lane) {
    const bool b1 = (lane >> 1) & 1, b0 = lane & 1;
    // stage 1 (l^8): banks 0,1 keep values 0..4, banks 2,3 values 5..9
    float k0, k1, k2, k3, k4;
    asm volatile("s_nop 1\n" GSR_DPP_KEEP("row_ror:8", "0x3", 0, 5) GSR_DPP_KEEP("row_ror:8", "0xc", 0, 10)
                     GSR_DPP_KEEP("row_ror:8", "0x3", 1, 6) GSR_DPP_KEEP("row_ror:8", "0xc", 1, 11)
                         GSR_DPP_KEEP("row_ror:8", "0x3", 2, 7) GSR_DPP_KEEP("row_ror:8", "0xc", 2, 12)
                             GSR_DPP_KEEP("row_ror:8", "0x3", 3, 8) GSR_DPP_KEEP("row_ror:8", "0xc", 3, 13)
                                 GSR_DPP_KEEP("row_ror:8", "0x3", 4, 9) GSR_DPP_KEEP("row_ror:8", "0xc", 4, 14)
                 : "=&v"(k0), "=&v"(k1), "=&v"(k2), "=&v"(k3), "=&v"(k4)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
                   "v"(v[8]), "v"(v[9]));
    // stage 2 (l^7, row_half_mirror): values a0..a4 (+ a5 = pad): banks 0,2 keep a0..a2, banks 1,3
    // a3, a4 and the pad (left unwritten: it only ever reaches padding slots)
    float c0, c1, c2;
    asm volatile("s_nop 1\n" GSR_DPP_KEEP("row_half_mirror", "0x5", 0, 3) GSR_DPP_KEEP("row_half_mirror", "0xa", 0, 6)
                     GSR_DPP_KEEP("row_half_mirror", "0x5", 1, 4) GSR_DPP_KEEP("row_half_mirror", "0xa", 1, 7)
                         GSR_DPP_KEEP("row_half_mirror", "0x5", 2, 5)
                 : "=&v"(c0), "=&v"(c1), "=&v"(c2)
                 : "v"(k0), "v"(k1), "v"(k2), "v"(k3), "v"(k4));
    // b0..b2 (+ b3 = 0): bit 1 keeps b0, b1 or b2, b3
    float d0 = b1 ? c2 : c0, d1 = b1 ? 0.f : c1;
    float u0 = b1 ? c0 : c2, u1 = b1 ? c1 : 0.f;
    asm volatile("s_nop 1\n" GSR_DPP_RS("quad_perm:[2,3,0,1]", 0, 2) GSR_DPP_RS("quad_perm:[2,3,0,1]", 1, 3)
                 : "+v"(d0), "+v"(d1)
                 : "v"(u0), "v"(u1));
    float e0 = b0 ? d1 : d0;
    const float w0 = b0 ? d0 : d1;
    asm volatile("s_nop 1\n" GSR_DPP_RS("quad_perm:[1,0,3,2]", 0, 1) : "+v"(e0) : "v"(w0));
    // rows 0+1 and 2+3 (both rows of a pair hold the sum): v_permlane16_swap hands every lane its
    // partner row's value without the LDS round trip of a ds_bpermute (same sum, same bits)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(e0), __float_as_uint(e0), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// The same reduce-scatter over TWO instances' ten values at once (v = instance A's, w = B's): the
// same partners in the same order (l^8, l^7, l^2, l^1, then rows 0+1 / 2+3), so every sum has the
// bits wave_rs10 gives it, but the 20 values fill the stages that pad a lone instance's 10, and the
// row pair ends in a reduce-scatter too (row 0 keeps one value, row 1 another) instead of both rows
// holding the same sum: 47 VALU per pair instead of 2 x 26.  Each lane ends with ONE half-wave partial,
// of value index wave_rs20_slot(lane) (0..9: A's, 10..19: B's, -1: padding).
__device__ __forceinline__ float wave_rs20(const float *v, const float *w, int lane) {
    const bool b1 = (lane >> 1) & 1, b0 = lane & 1;
    // stage 1 (l^8): banks 0,1 (bit 3 clear) keep A's ten values, banks 2,3 B's
    float k0, k1, k2, k3, k4, k5, k6, k7, k8, k9;
    asm volatile("s_nop 1\n"
                 GSR_DPP_KEEP("row_ror:8", "0x3", 0, 10) GSR_DPP_KEEP("row_ror:8", "0xc", 0, 20)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 1, 11) GSR_DPP_KEEP("row_ror:8", "0xc", 1, 21)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 2, 12) GSR_DPP_KEEP("row_ror:8", "0xc", 2, 22)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 3, 13) GSR_DPP_KEEP("row_ror:8", "0xc", 3, 23)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 4, 14) GSR_DPP_KEEP("row_ror:8", "0xc", 4, 24)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 5, 15) GSR_DPP_KEEP("row_ror:8", "0xc", 5, 25)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 6, 16) GSR_DPP_KEEP("row_ror:8", "0xc", 6, 26)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 7, 17) GSR_DPP_KEEP("row_ror:8", "0xc", 7, 27)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 8, 18) GSR_DPP_KEEP("row_ror:8", "0xc", 8, 28)
                 GSR_DPP_KEEP("row_ror:8", "0x3", 9, 19) GSR_DPP_KEEP("row_ror:8", "0xc", 9, 29)
                 : "=&v"(k0), "=&v"(k1), "=&v"(k2), "=&v"(k3), "=&v"(k4), "=&v"(k5), "=&v"(k6), "=&v"(k7),
                   "=&v"(k8), "=&v"(k9)
                 : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
                   "v"(v[8]), "v"(v[9]), "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]),
                   "v"(w[6]), "v"(w[7]), "v"(w[8]), "v"(w[9]));
    // stage 2 (l^7, row_half_mirror): banks 0,2 (bit 2 clear) keep k0..k4, banks 1,3 k5..k9
    float c0, c1, c2, c3, c4;
    asm volatile("s_nop 1\n"
                 GSR_DPP_KEEP("row_half_mirror", "0x5", 0, 5) GSR_DPP_KEEP("row_half_mirror", "0xa", 0, 10)
                 GSR_DPP_KEEP("row_half_mirror", "0x5", 1, 6) GSR_DPP_KEEP("row_half_mirror", "0xa", 1, 11)
                 GSR_DPP_KEEP("row_half_mirror", "0x5", 2, 7) GSR_DPP_KEEP("row_half_mirror", "0xa", 2, 12)
                 GSR_DPP_KEEP("row_half_mirror", "0x5", 3, 8) GSR_DPP_KEEP("row_half_mirror", "0xa", 3, 13)
                 GSR_DPP_KEEP("row_half_mirror", "0x5", 4, 9) GSR_DPP_KEEP("row_half_mirror", "0xa", 4, 14)
                 : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3), "=&v"(c4)
                 : "v"(k0), "v"(k1), "v"(k2), "v"(k3), "v"(k4), "v"(k5), "v"(k6), "v"(k7), "v"(k8), "v"(k9));
    // stage 3 (l^2): c0..c4 (+ c5 = 0): bit 1 keeps c0..c2 or c3, c4, pad
    float d0 = b1 ? c3 : c0, d1 = b1 ? c4 : c1, d2 = b1 ? 0.f : c2;
    const float u0 = b1 ? c0 : c3, u1 = b1 ? c1 : c4, u2 = b1 ? c2 : 0.f;
    asm volatile("s_nop 1\n" GSR_DPP_RS("quad_perm:[2,3,0,1]", 0, 3) GSR_DPP_RS("quad_perm:[2,3,0,1]", 1, 4)
                     GSR_DPP_RS("quad_perm:[2,3,0,1]", 2, 5)
                 : "+v"(d0), "+v"(d1), "+v"(d2)
                 : "v"(u0), "v"(u1), "v"(u2));
    // stage 4 (l^1): d0..d2 (+ d3 = 0): bit 0 keeps d0, d1 or d2, pad
    float e0 = b0 ? d2 : d0, e1 = b0 ? 0.f : d1;
    const float x0 = b0 ? d0 : d2, x1 = b0 ? d1 : 0.f;
    asm volatile("s_nop 1\n" GSR_DPP_RS("quad_perm:[1,0,3,2]", 0, 2) GSR_DPP_RS("quad_perm:[1,0,3,2]", 1, 3)
                 : "+v"(e0), "+v"(e1)
                 : "v"(x0), "v"(x1));
    // rows 0+1 and 2+3: v_permlane16_swap(e0, e1) hands the even row the odd row's e0 and the odd row
    // the even row's e1, so the even row keeps e0's sum and the odd row e1's
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(e0), __float_as_uint(e1), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
#undef GSR_DPP_RS
#undef GSR_DPP_KEEP

// Value index of lane's wave_rs20 result (0..19), or -1 for a padding slot: 10 b3 + 5 b2 + c with
// t = row bit + 2 b0 (3: pad) and c = t + 3 b1 (5: pad).
__device__ __forceinline__ int wave_rs20_slot(int lane) {
    const int b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, b1 = (lane >> 1) & 1, b0 = lane & 1, row = (lane >> 4) & 1;
    const int t = row + 2 * b0;
    const int c = t + 3 * b1;
    return (t == 3 || c >= 5) ? -1 : 10 * b3 + 5 * b2 + c;
}

// Value index of lane's wave_rs10 result: 5 b3 + 3 b2 + (2 b1 + b0), or -1 for a padding slot.
__device__ __forceinline__ int wave_rs10_slot(int lane) {
    const int b3 = (lane >> 3) & 1, b2 = (lane >> 2) & 1, c = lane & 3;
    return (c == 3 || (b2 && c == 2)) ? -1 : 5 * b3 + 3 * b2 + c;
}

// Max over the 64 lanes, in every lane: DPP within the 16-lane rows, then gfx950's row and half
// swaps (no LDS round trips, unlike a __shfl_xor butterfly).
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, dpp_u<0xB1>(v));   // quad_perm [1,0,3,2]
    v = max(v, dpp_u<0x4E>(v));   // quad_perm [2,3,0,1]
    v = max(v, dpp_u<0x124>(v));  // row_ror:4
    v = max(v, dpp_u<0x128>(v));  // row_ror:8 -> every lane holds its row's max
    const auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = max(r16[0], r16[1]);
    const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return max(r32[0], r32[1]);
}

// ------------------------------------------------------------------------------------------
// Scratch-state layouts (carved out of the caller's byte buffers, 256-B aligned arrays)
// ------------------------------------------------------------------------------------------
constexpr float kLog2e = 1.4426950408889634f;

// The Gaussian's exponent in base 2, p2 = log2(G) = log2(e) (-0.5 (a dx^2 + c dy^2) - b dx dy), from
// the conic scaled once per instance: a_s = a (-0.5 log2e), b_s = b log2e, c_s = c (-0.5 log2e)
// (render kernels scale it when they stage an instance in LDS).  Per pixel:
//   p2 = fma(-(b_s dx), dy, fma(c_s dy, dy, a_s dx dx)),  G = exp2(p2)
// -- two multiplies fewer than forming -0.5(...) and scaling by log2e per pixel.  The oracle
// restates this order exactly (oracle/gs_oracle.c gauss_p2).
constexpr float kHalfLog2e = -0.5f * 1.4426950408889634f;  // exact: a power-of-two scaling
__device__ __forceinline__ float gauss_p2(float adxdx_s, float bdx_s, float c_s, float dy) {
    return fmaf(-bdx_s, dy, fmaf(c_s * dy, dy, adxdx_s));
}

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// One 64-B render record per Gaussian (written by the preprocess): everything a
// tile instance needs sits in one cache line, so the render kernels gather 1 line per instance.
struct alignas(16) GRec {
    float x, y, ca, cb;       // q0: pixel-space mean, conic (a, b)
    float cc, op, ex, ey;     // q1: conic c, opacity, half-extents of the alpha >= 1/255 ellipse
                              //     (ex < 0: can never reach alpha >= 1/255)
    float r, g, b, invd;      // q2: colour, 1 / view depth
    uint32_t rect0, rectw, dbits;       // q3: tile rect x0 | y0 << 16, width; depth bits;
    float cull_tm;                      //     the cull threshold of ellipse_meets_box
};
static_assert(sizeof(GRec) == 64, "GRec must be one 64-B line");

// Superblock grid of the two-level binning (binning.hip): SB = 2^shift x 2^shift tiles.
#ifndef GSR_SB_CHUNK
#define GSR_SB_CHUNK 1024
#endif
constexpr int kSBChunk = GSR_SB_CHUNK;  // smallest level-1 chunk (SBGrid.chunk doubles for large P)
#ifndef GSR_MAX_CHUNKS
#define GSR_MAX_CHUNKS 3072  // config 5 (7.4M): 3072 -> bin_superblocks 0.40 ms, 1536 -> 0.43, 768 -> 0.51
#endif
constexpr int kMaxChunks = GSR_MAX_CHUNKS;  // chunks before SBGrid.chunk doubles
constexpr int kMaxSB = 1536;          // superblocks (3 x 8 waves x 4 B of LDS each in sb_scatter)
constexpr int kMaxTilesPerSB = 256;   // up to 16 x 16 tiles per superblock
// Level 2 of long superblock lists (tile_bin split, binning.hip): an SB list longer than
// GSR_TB_SPLIT entries is binned in up to kTBMaxSlices slices by tb_split_kernel's work items
// (queued by sb_colscan's last workgroup, at most kTBMaxItems per frame; a full queue leaves the
// rest to tile_bin).
#ifndef GSR_TB_SPLIT
#define GSR_TB_SPLIT 16384
#endif
constexpr int kTBMaxItems = 4096;
constexpr uint32_t kTBMaxSlices = 63;
constexpr uint32_t kTBVoid = 0xFFFFFFFFu;
struct SBGrid {
    int shift, nsbx, nsby, nsb, nchunks, chunk;  // chunk: depth-ordered Gaussians per level-1 chunk
    int cper, ccols;                             // counter columns per XCD, row stride of the counters
};
// GSR_BWD_CLS: render_fwd's workgroups place their tile in one of kBwdClasses backward work
// classes (a counter atomic) and render_bwd's workgroups find their tile from the class counts --
// the backward launch order without a tile_order launch between the forward and the backward
#ifndef GSR_BWD_CLS
#define GSR_BWD_CLS 1
#endif
constexpr int kBwdClasses = 256;
// GSR_FWD_SB_ORDER: the forward's launch order is by superblock (heaviest SB first, by its mean
// tile-instance count; an SB's tiles consecutive), bucketed by the level-1 column scan's last
// workgroup -- no tile_order launch between the tile binning and render_fwd
#ifndef GSR_FWD_SB_ORDER
#define GSR_FWD_SB_ORDER 0  // measured slower: render_fwd +11.5 us for the 10-us launch it saves (r03z)
#endif
constexpr int kBwdClassShift = 2;  // class = 255 - min(work >> 2, 255): heaviest first

// Backward segments (gsr_set_bwd_segment): a tile whose backward work (last contributor position)
// exceeds L list positions is replayed as ceil(work / L) independent work items of L positions, the
// later ones starting from checkpoints render_fwd stores at every L-th position of the tile's list
// (per pixel: the transmittance there and the colour / inverse depth accumulated behind it), so one
// street view's vanishing-point tiles (tens of thousands of instances) no longer set the kernel's
// tail.  The checkpoints and the segment list live in the binning buffer past the point list (the
// level-1 lists are dead once the tiles are binned): slot floor(position / L) is unique per
// checkpoint (any two are >= L positions apart in the point list).
constexpr int kBwdSegCount = kBwdClasses;  // bwd_cnt[kBwdSegCount]: full segments listed by render_fwd
constexpr int kCkFloats = 5;               // T, behind r, g, b, inverse depth (x 256 pixels per slot)
__host__ __device__ __forceinline__ size_t ck_offset(int64_t K) { return (size_t)(((4 * K) + 255) / 256 * 256); }
__host__ __device__ __forceinline__ size_t ck_slots(int64_t K, uint32_t L) { return L ? (size_t)(K / L) + 2 : 0; }
constexpr uint32_t kMinBwdSeg = 512;     // the shortest segment (with kMinFwdSeg: all fits in 16 B / instance + kSegReserve)
constexpr size_t kSegReserve = 32768;    // carved past the level-1 lists (a small K's slots)
// render_bwd's grid: every tile's last segment plus at most K / L full segments
inline int64_t bwd_grid(int T, int64_t K, uint32_t L) { return (int64_t)T + (L ? K / L : 0); }
__host__ __device__ __forceinline__ size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Forward segments (gsr_set_fwd_segment): a tile whose list is longer than fseg_min_len(Lf) is
// blended as ceil(len / Lf) work items by render_fwd_seg_kernel's kFwdPoolWorkers workgroups (an item
// queue tile_order fills), launched ahead of tile_order on a side stream.  Item s first multiplies
// out (1 - alpha) over its positions (the pixels' transmittance through the segment), publishes it,
// waits for its predecessors' and takes their product in segment order, then blends its positions
// from that transmittance with the usual stop rule; the tile's last item to finish sums the items' colours in order and writes the
// pixels.  Per item, past the backward's region: its queue entry, a ticket (the tile's first
// item's counts the finished items), a flag (1: its transmittance row is published; zeroed with
// the queue), 4 checkpoint counts, the per-pixel transmittance row and 256 x 6 partials.
constexpr uint32_t kMinFwdSeg = 1024;
// a tile is split when its list is longer than fseg_min (kFsegFactor segments by default: a tile
// of a few segments whose pixels saturate early gains little)
#ifndef GSR_FSEG_FACTOR
// config-3 with the workers ahead of tile_order (r04zc, Lf 4096): 4 -> 57.3 / 56.9 s, 16 -> 57.0 s (workers
// beside render_fwd: 58.5 s); street views with 60k-110k lists: 4 -> 0.81 ms render_fwd, 16 -> 2.96 ms
// (r04zb).  At Lf 2048 (r05t, two rounds): 3 -> 51.8 s, 4 -> 52.2 / 51.1 s, 6 -> 50.9 / 50.9 s, 8 -> 50.9 s
#define GSR_FSEG_FACTOR 6
#endif
__host__ __device__ __forceinline__ bool fseg_splits(uint32_t len, uint32_t fseg_min) { return fseg_min && len > fseg_min; }
constexpr int kFwdWorkers = 256;      // the in-kernel variant's pool (GSR_FWD_SEG_INKERNEL)
// render_fwd_seg_kernel's pool, launched ahead of tile_order: street views with 300k+ lists 1.40 /
// 1.59 ms render_fwd at 256, 1.24 / 1.28 at 512, 1.24 / 1.27 at 1024 (r04zd)
constexpr int kFwdPoolWorkers = 512;
constexpr int kFwdPartials = 6;  // r, g, b, inverse depth, T at the end, last contributor | stop << 31
// bwd_cnt's words past the backward's: the item count tile_order wrote, the queue's next item
constexpr int kFwdItemsWord = kBwdSegCount + 1, kFwdNextWord = kBwdSegCount + 2;
struct FwdSegLayout {
    uint32_t *items, *tickets, *flags, *nc;
    float *agg;  // per item x 256 pixels: the transmittance through the segment
    float *part;
};
__host__ __device__ __forceinline__ size_t fseg_max_items(int64_t K, uint32_t Lf) { return Lf ? (size_t)(2 * K / Lf) + 2 : 0; }
__host__ __device__ __forceinline__ FwdSegLayout fseg_layout(void *bin_base, int64_t K, uint32_t L, uint32_t Lf) {
    const size_t n = fseg_max_items(K, Lf);
    size_t off = ck_offset(K) + (L ? align256(ck_slots(K, L) * (kCkFloats * 256) * 4 + ck_slots(K, L) * 4) : 0);
    char *b = static_cast<char *>(bin_base);
    FwdSegLayout f;
    f.items = reinterpret_cast<uint32_t *>(b + off);
    off = align256(off + 4 * n);
    f.tickets = reinterpret_cast<uint32_t *>(b + off);
    off = align256(off + 4 * n);
    f.flags = reinterpret_cast<uint32_t *>(b + off);
    off = align256(off + 4 * n);
    f.nc = reinterpret_cast<uint32_t *>(b + off);
    off = align256(off + 16 * n);
    f.agg = reinterpret_cast<float *>(b + off);
    off = align256(off + 4 * 256 * n);
    f.part = reinterpret_cast<float *>(b + off);
    return f;
}

#ifndef GSR_RECT4
#define GSR_RECT4 1
#endif
#ifndef GSR_CNT_XCD
#define GSR_CNT_XCD 1
#endif
// Counter column of a level-1 chunk.  Chunk c runs as workgroup c, and workgroups are dealt to
// the 8 XCDs round-robin, so the columns of one XCD's chunks are made adjacent: its 4-B counter
// stores then fill whole lines in its own L2 instead of sharing every line with the 7 other XCDs.
// GSR_SB_XCD_GROUP = G > 1: runs of G consecutive chunks go to one XCD (workgroup b runs chunk
// chunk_of_block(b)), so the adjacent level-1 list runs that consecutive chunks write meet in one L2
// (a chunk's run per superblock is ~7 entries, less than a line); G = 1 is the plain order.
#ifndef GSR_SB_XCD_GROUP
#define GSR_SB_XCD_GROUP 4  // r05g A/B: bin_superblocks 0.0808 (G = 1) -> 0.0803 (2) -> 0.0783 ms (4), parity bit-exact
#endif
constexpr int kXcdGroup = GSR_SB_XCD_GROUP;
__host__ __device__ __forceinline__ int chunk_of_block(int b) {
    const int k = b >> 3;
    return kXcdGroup == 1 ? b : (k / kXcdGroup) * 8 * kXcdGroup + (b & 7) * kXcdGroup + k % kXcdGroup;
}
// workgroups of the level-1 kernels: the chunks rounded up to whole XCD groups
__host__ __device__ __forceinline__ int sb_blocks(const SBGrid &g) {
    return kXcdGroup == 1 ? g.nchunks : (g.nchunks + 8 * kXcdGroup - 1) / (8 * kXcdGroup) * 8 * kXcdGroup;
}
__host__ __device__ __forceinline__ int cnt_col(const SBGrid &g, int chunk) {
    if (!GSR_CNT_XCD) return chunk;
    if (kXcdGroup == 1) return (chunk & 7) * g.cper + (chunk >> 3);
    return ((chunk / kXcdGroup) & 7) * g.cper + (chunk / (8 * kXcdGroup)) * kXcdGroup + chunk % kXcdGroup;
}

struct GeomState {          // per Gaussian, written by preprocess
    GRec *rec;
    uint32_t *tiles;        // tiles_touched
    uint32_t *dkey;         // depth sort key: depth bits, 0xFFFFFFFF when culled (clobbered by the sort)
    uint32_t *dkey_sorted;  // sort ping-pong buffer
    uint32_t *ids;          // sort ping-pong buffer (values)
    uint32_t *order;        // Gaussian ids in (depth, id) order
    uint32_t *offsets;      // exclusive scan of tiles_touched in Gaussian order: each Gaussian's first
                            // backward record (dsort.hip pass 0)
    uint8_t *clamped;       // bit c set: SH channel c clamped at 0
    uint32_t *ctrl;         // depth-sort control words (dsort.hip); the first ctrl_zero are zeroed by
    uint32_t ctrl_zero;     // the preprocess
    uint2 *drect;           // per depth-order slot: tile rect (x0 | y0 << 16, x1 | y1 << 16), 0/0 = none
    uint2 *rect8;           // per Gaussian (index order): the same rect, written by the preprocess
                            // unless rect4 is set
    uint32_t *rect4;        // the same rect in 8-bit fields when the tile grid is <= 255 x 255 (else
                            // nullptr), then written instead of rect8: the depth sort's last pass
                            // gathers these 4 B, and drect holds them in that form too (drect4_of)
    SBGrid sb;              // level-1 binning counters: [nsb][ccols] Gaussians / instances (cnt_col),
    uint32_t *sb_cnt_g;     // per-SB bases (nsb + 1 each)
    uint32_t *sb_cnt_i;
    uint32_t *sb_base_g;
    uint32_t *sb_base_i;
    float4 *acc;            // backward accumulators, 4 float4 (64 B) per Gaussian, zeroed by render_fwd
    int nacc;               // rows of acc (P)
    uint32_t *live_stamp;   // per Gaussian: the stamp of the last backward whose render_bwd staged it
    uint32_t *tb_flag;      // tile_bin split: per SB 1 = binned in slices; [nsb] = queued items
    uint32_t *tb_items;     // ... the slice items (kTBMaxItems: SB | slice << 12 | slices << 18)
    uint32_t *tb_cnt;       // ... per item and SB tile: the slice's instance count
};
// a 4-B packed rect (x0 | y0 << 8 | x1 << 16 | y1 << 24) in the 8-B form (x0 | y0 << 16, x1 | y1 << 16)
__host__ __device__ __forceinline__ uint2 unpack_rect4(uint32_t q) {
    return make_uint2((q & 0xFFu) | ((q << 8) & 0xFF0000u), ((q >> 16) & 0xFFu) | ((q >> 8) & 0xFF0000u));
}
// drect as 4-B packed rects (the depth sort's last pass wrote rect4's form), or nullptr
__host__ __device__ __forceinline__ const uint32_t *drect4_of(const GeomState &g) {
    return g.rect4 ? reinterpret_cast<const uint32_t *>(g.drect) : nullptr;
}

// Frame words a local-sort frame's column scan publishes (binning.hip): device copies for the
// kernels (dev_K = the depth sort's K word, which every capacity test reads) and, when host is set,
// the pinned host words the host waits on.  host[kHostK] is stored last.
// kHostSBList / kHostTileList: every frame's longest superblock list (sb_colscan) and longest tile
// list (the forward's tile_order), read by the host as the split gate's hint (rasterizer.hip)
#ifndef GSR_HOST_WORDS
#define GSR_HOST_WORDS 1  // split gate hints: 1 stored by tile_order / sb_colscan, 2 forwarded by render_fwd, 0 none (A/B)
#endif
// Sticky flags the kernels set with plain system-scope stores (read-modify-write atomics on pinned host
// memory need PCIe atomics, which a host may not have) and the host's next call takes:
// kHostErr: a depth-sort lookback spin gave up; kHostFwdErr: a forward worker's wait for a
// predecessor segment gave up (both frames' images are NaN: the call fails); kHostFwdGiveUp: forward
// workers gave up waiting for tile_order's ready word (the frame is completed exactly by the pool's
// second launch; counted in gsr_forward_stats).
enum HostWord { kHostK = 0, kHostErr = 1, kHostMaxSB = 2, kHostP1 = 3, kHostSBList = 4, kHostTileList = 5,
                kHostFwdGiveUp = 6, kHostFwdErr = 7, kHostWords = 8 };
// The forward workers' bounded spins (render.hip fwd_seg_worker): `ready` = tile_order's release of
// the queue, `flag` = a predecessor item's transmittance row; loop trips of ~256 / ~128 clocks.
// gsr_set_fwd_spin_limits changes them (tests); `host` = the pinned words above.
struct FwdSpin {
    uint32_t ready, flag;
    uint32_t *host;
};
constexpr uint32_t kFwdReadySpins = 1u << 18;  // ~28 ms: tile_order normally releases within ~10 us
constexpr uint32_t kFwdFlagSpins = 1u << 22;
constexpr uint32_t kFwdReadyNever = 0xFFFFFFFFu;  // tests: the workers give up without waiting
struct FrameWords {
    uint32_t *dev_K;      // nullptr: global-sort frame (dsort publishes K)
    uint32_t *dev_maxsb;  // longest SB list
    uint32_t *host;       // pinned host words (HostWord indices) or nullptr
};

struct BinningState {       // per tile instance
    uint2 *sblist;          // level 1: (Gaussian id, footprint in SB-local tiles) per superblock, depth order
    uint4 *sblist4;         // the same memory on the local-sort path: (id, footprint, depth key, 0), id order
    uint32_t *point_list;   // Gaussian ids, per tile contiguous in (depth, id) order; tiles SB-major
    uint32_t cap;           // entries carved for sblist and point_list
    const uint32_t *kdev;   // the frame's K on the device (forward): kernels exit if K > cap
};

struct ImageState {
    uint2 *ranges;          // per tile [start, end) in point_list
    uint64_t *boundary;     // per tile: (depth bits << 32 | id) of the last instance any pixel uses
    float *final_T;         // per pixel
    uint32_t *n_contrib;    // per pixel: 1-based list position of the last contributor
    uint32_t *tile_work;    // per tile: backward work (last contributor position, max over pixels)
    uint32_t *tile_ids;     // forward launch order (tiles by descending list length)
    uint32_t *tile_order;   // backward launch order (tiles by descending tile_work; GSR_BWD_CLS = 0)
    uint32_t *bwd_cnt;      // GSR_BWD_CLS: per backward work class, the tiles render_fwd placed in it
    uint32_t *bwd_cls;      // ... and those tiles, class c at [c * T, c * T + bwd_cnt[c])
};

// Backward per-instance gradient records, one 64-B line each, indexed by the instance's unsorted
// (Gaussian-major) position u:  q0 = dmean2D.x, dmean2D.y, dconic.a, dconic.b;
// q1 = dconic.c, dopacity, drgb.r, drgb.g;  q2 = drgb.b, dinvdepth, 0, 0;  q3 = 0.
// Only instances at list positions below their tile's boundary are written.
//
// Default (atomic) mode: no records; render_bwd adds each live instance's ten values (same order:
// dmean2D x, y, dconic a, b, c, dopacity, drgb r, g, b, dinvdepth) into the Gaussian's 64-B
// accumulator row GeomState.acc with no-return float atomics, one 40-B segment per instance.
struct BwdScratch {
    float4 *rec;
    float4 *gsum;  // per Gaussian: {dconic a, b, c, dinvdepth}, {drgb r, g, b, 0} (record_sum -> preprocess_bwd)
    float4 *acc;   // atomic mode: GeomState.acc (rec / gsum unused)
    uint64_t *live;  // atomic mode: one mask of live rows (nonzero sums) per 64 Gaussians (backward.hip)
    uint32_t *list;  // the live rows, grad_live_list_kernel -> grad_live_kernel (P entries)
    int atomic;
};


// ---- kernel stamps (measurement builds only: -DGSR_KSTAMP=1, tools/kstamp.py) ----------------------
// The frame's kernels on the GPU's own clock, without a profiler in the way (rocprofv3's kernel
// trace adds ~10 us between some kernels): each instrumented kernel's block 0 stores its start
// (s_memrealtime, 100 MHz) into a 4-entry ring, every wave's lane 0 stores its end into a slot of its
// own (plain stores; the reader takes the max -- atomics on shared lines serialised at the L2 and
// doubled the step).  Kernels of more than 16384 waves alias slots.
// The arrays are per translation unit (no relocatable device code); each TU exports a reader.
#ifndef GSR_KSTAMP
#define GSR_KSTAMP 0
#endif
constexpr int kKsIds = 24, kKsRing = 4, kKsSlots = 16384;
enum KsId {
    kKsPreprocess, kKsColor, kKsUpsweep, kKsPass0, kKsPass1, kKsPass2, kKsPass3, kKsSbCount, kKsSbColscan,
    kKsSbScatter, kKsTileBin, kKsTileOrder, kKsRenderFwd, kKsRenderBwd, kKsGradRange, kKsFwdSeg, kKsLiveList,
    kKsGradLive
};
#if GSR_KSTAMP
static __device__ unsigned long long g_ks_start[kKsIds][kKsRing];
static __device__ unsigned long long g_ks_end[kKsIds][kKsRing][kKsSlots];
static __device__ unsigned int g_ks_cnt[kKsIds];
struct KStampScope {
    int id;
    __device__ __forceinline__ explicit KStampScope(int i) : id(i) {
        if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
            const unsigned c = __hip_atomic_load(&g_ks_cnt[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g_ks_start[id][c % kKsRing] = wall_clock64();
            __hip_atomic_store(&g_ks_cnt[id], c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __device__ __forceinline__ ~KStampScope() {
        if ((threadIdx.x & 63) == 0) {
            const unsigned c = __hip_atomic_load(&g_ks_cnt[id], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1u;  // relaxed: an acquire invalidates the CU's L1 per wave
            const unsigned w = ((blockIdx.x + blockIdx.y * gridDim.x) * ((blockDim.x + 63) / 64) + threadIdx.x / 64);
            __hip_atomic_store(&g_ks_end[id][c % kKsRing][w % kKsSlots], wall_clock64(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
};
#define GSR_KS(id) const gsr::KStampScope gsr_ks_scope_((int)(id))
// out[id * (1 + 2 kKsRing)]: the kernel's launch count, then the ring's starts, then its ends
#define GSR_KSTAMP_READER(name)                                                                         \
    int name(unsigned long long *out) {                                                                 \
        static unsigned long long st[kKsIds][kKsRing], en[kKsIds][kKsRing][kKsSlots];                   \
        static unsigned int cnt[kKsIds];                                                                \
        if (hipDeviceSynchronize() != hipSuccess ||                                                     \
            hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ks_start), sizeof(st)) != hipSuccess ||               \
            hipMemcpyFromSymbol(en, HIP_SYMBOL(g_ks_end), sizeof(en)) != hipSuccess ||                 \
            hipMemcpyFromSymbol(cnt, HIP_SYMBOL(g_ks_cnt), sizeof(cnt)) != hipSuccess)                 \
            return -1;                                                                                  \
        for (int i = 0; i < kKsIds; i++) {                                                              \
            unsigned long long *o = out + (size_t)i * (1 + 2 * kKsRing);                                \
            o[0] = cnt[i];                                                                              \
            for (int r = 0; r < kKsRing; r++) {                                                         \
                o[1 + r] = st[i][r];                                                                    \
                unsigned long long m = 0;                                                               \
                for (int k = 0; k < kKsSlots; k++) m = en[i][r][k] > m ? en[i][r][k] : m;               \
                o[1 + kKsRing + r] = m;                                                                 \
            }                                                                                           \
        }                                                                                               \
        return 0;                                                                                       \
    }
#else
#define GSR_KS(id) ((void)0)
#define GSR_KSTAMP_READER(name) \
    int name(unsigned long long *) { return -1; }
#endif

}  // namespace gsr
