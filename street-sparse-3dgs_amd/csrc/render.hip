// render.hip -- tile blending forward and backward.
//
// MI355X mapping: one 64-lane wave owns one 16x16 tile.  Lane l holds pixels
// (x = l & 15, y = (l >> 4) + 4k), k = 0..3, so for a fixed k the wave covers the 16x4 sub-block
// k of the tile.  Instances are staged through LDS 64 at a time: every lane gathers one 64-B
// GRec (one cache line), tests the instance's opacity-aware ellipse AABB against the four
// sub-blocks, and a wave ballot + mbcnt prefix sum compacts the survivors (with their 4-bit
// sub-block masks) into LDS.  The blend loop then runs over survivors only, skipping culled
// sub-blocks (forward: scalar branch; backward: predicate, see there).  The cull is conservative (preprocess.hip), so colour, depth,
// final T and n_contrib are exactly those of the uncompacted upstream loop.  The per-pixel work
// is branch-free (selects, no exec-mask divergence); the tile-wide early exit of the upstream
// design (__syncthreads_count) becomes a wave vote.
//
// Backward: upstream accumulates ~10 float atomics per (pixel, Gaussian) pair.  On gfx950 float
// atomics execute at the memory side (MI355X_MICROARCH.md, Global float atomics) and 64 lanes
// adding into one address serialise, so each wave first reduces every instance's 10 gradient
// terms over its 256 pixels in registers (a DPP reduce-scatter, gsr_device.h wave_rs10, whose
// half-wave partials go to LDS and are combined once per batch of 64 instances).  The per-batch
// sums then leave either as ten wave-wide float-atomic instructions into per-Gaussian rows (the
// default: one contiguous 40-B segment per instance, one memory-side request) or, in
// deterministic mode, as one 64-B record per instance at its Gaussian-major index, summed by
// backward.hip in a fixed order (bitwise reproducible).  Only instances in front of the tile's
// last contributor are visited (13% of them on the 1M-Gaussian bench scene).
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "gsr_launch.h"

namespace gsr {

__device__ __forceinline__ float gexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Measurement builds only (GSR_BLEND_STATS=1, a variant library): lane-liveness statistics of the
// blend kernels, read back with gsr_blend_stats.  Per evaluated (instance, 16x4 sub-block) pair:
// the lanes whose pixel passes the alpha / position tests, and how many finer cells (8x4 halves,
// 16x1 rows, 4x4 quads) hold at least one such lane -- what a finer cull could skip.
#ifndef GSR_BLEND_STATS
#define GSR_BLEND_STATS 0
#endif
__device__ unsigned long long g_blend_stats[16];
// The forward-split worker pool's time (always on; gsr_fwd_pool_stats): s_memrealtime ticks (100 MHz)
// summed over workgroups -- [0] waiting for tile_order's release of the queue (workers launched
// ahead), [1] waiting for predecessor segments' transmittance rows, [2] workgroup lifetimes, [3]
// workgroups.  Busy = [2] - [0] - [1] (dequeues, blends, the tiles' final sums).
#ifndef GSR_FWD_POOL_STATS
#define GSR_FWD_POOL_STATS 1
#endif
__device__ unsigned long long g_fwd_pool_ticks[4];
// StatAcc::flush writes (pairs, live lanes, live halves, live rows, live quads) at its base index
enum BlendStat { kBwdPairs, kBwdLive, kBwdHalves, kBwdRows, kBwdQuads, kBwdInst, kBwdBatches, kFwdPairs, kFwdLive,
                 kFwdHalves, kFwdRows, kFwdQuads, kFwdAcc, kBwdTiles };
struct StatAcc {
    uint64_t v[5] = {0, 0, 0, 0, 0};
    __device__ __forceinline__ void add(uint64_t live) {
        constexpr uint64_t kLeft = 0x00FF00FF00FF00FFull;
        v[0] += 1;
        v[1] += (uint64_t)__popcll(live);
        v[2] += (uint64_t)((live & kLeft) != 0) + (uint64_t)((live & ~kLeft) != 0);
#pragma unroll
        for (int r = 0; r < 4; r++) v[3] += (uint64_t)(((live >> (16 * r)) & 0xFFFFull) != 0);
#pragma unroll
        for (int q = 0; q < 4; q++) v[4] += (uint64_t)((live & (0x000F000F000F000Full << (4 * q))) != 0);
    }
    __device__ __forceinline__ void flush(int base) {
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 5; k++) atomicAdd(&g_blend_stats[base + k], (unsigned long long)v[k]);
    }
};

#ifndef GSR_EXACT_CULL
#define GSR_EXACT_CULL 3  // bit 0: forward, bit 1: backward
#endif

__device__ __forceinline__ uint32_t sub_block_mask(const float4 &qa, const float4 &qb, float tm, float tx0,
                                                   float ty0) {
    // bit k: the alpha >= 1/255 ellipse of the instance (its box, then the ellipse itself) meets
    // pixel rows ty0+4k..ty0+4k+3
    const float X = qa.x, Y = qa.y, ex = qb.z, ey = qb.w;
    if (!(X + ex >= tx0 && X - ex <= tx0 + 15.f)) return 0u;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        const float y0 = ty0 + (float)(4 * k);
        if (Y + ey >= y0 && Y - ey <= y0 + 3.f &&
            (!(GSR_EXACT_CULL & 2) || ellipse_meets_box(X, Y, qa.z, qa.w, qb.x, tm, tx0, tx0 + 15.f, y0, y0 + 3.f)))
            m |= 1u << k;
    }
    return m;
}

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ------------------------------------------------------------------------------------------
// Forward
// ------------------------------------------------------------------------------------------
// A 256-thread workgroup per tile, wave w owning the 16x4 sub-block w with one pixel per lane.
// Each wave walks the tile's list on its own (gather, cull to its sub-block with the exact
// ellipse-vs-box test, ballot-compact into its own LDS slice) and stops when its own 64 pixels
// saturate, so a heavy tile is spread over four waves and culled sub-blocks cost nothing.
//
// The gather is software-pipelined: while batch b blends, the GRec lines of batch b+1 and the
// point-list ids of batch b+2 are in flight (two dependent round trips per batch -- id, then the
// line -- that were otherwise exposed once per batch per wave).
#ifndef GSR_ACC_NT
#define GSR_ACC_NT 1
#endif
#ifndef GSR_FWD_ACC_CLEAR
#define GSR_FWD_ACC_CLEAR 1  // 0: measurement builds only (the backward's sums then start from garbage)
#endif
#ifndef GSR_FWD_SUB
#define GSR_FWD_SUB 1  // 16x4 sub-blocks per wave (measured: 1 -> 0.139 ms, 2 -> 0.176, 4 -> 0.242)
#endif
struct FwdBatch {
    float4 a, b, c;  // GRec q0..q2
    float tm;        // GRec.cull_tm
};

// Unconditional loads (lanes past the list end re-read the last entry; their hit test is false):
// a load under a lane mask would make the compiler join the old and new register values at the
// end of the branch, which waits for the load right there -- no overlap.
__device__ __forceinline__ void fwd_gather(const GRec *__restrict__ rec, uint32_t g, FwdBatch &o) {
    const float4 *R = reinterpret_cast<const float4 *>(rec + g);
    o.a = R[0];
    o.b = R[1];
    o.c = R[2];
    o.tm = rec[g].cull_tm;
}

// kSub sub-blocks per wave (4 / kSub waves per tile): lane l holds pixels (l & 15, (l >> 4) + 4k) of
// its wave's sub-blocks k = 0..kSub-1, and the instance's dx terms, LDS reads and list position
// are shared by the lane's kSub rows.  Fewer waves per tile are slower despite the shared work
// (kSub 2: 0.176 ms, 4: 0.242 ms vs 0.139 ms for kSub 1 on the bench frame): 4% of the pixels never
// saturate, so their waves walk the whole list (1700 instances on average), and that walk is
// serial per wave.  The wave's walk stops when all its pixels have saturated; saturated
// sub-blocks drop out of the cull mask at the next batch and an instance's culled sub-blocks are
// skipped with scalar branches.  The list position comes from LDS with the instance (no scalar
// bit scan and no SGPR->VGPR move per pixel).  Per-pixel arithmetic in the oracle's order.
// GSR_FWD_POLY=1 evaluates the exponent as a quadratic in the pixel's offset from its sub-block's
// centre (5 FMAs; ~3 us faster on the bench frame) -- off: its p2 differs from the backward's
// replay (and the oracle's) by up to 3e-5, and the backward reconstructs T from final_T by
// dividing out (1 - alpha) of every instance, so the forward and the replay must agree on alpha
// bit for bit.  With the quadratic, near Gaussians clamped at alpha = 0.99 amplified the mismatch
// into 1e-3 relative gradient errors (1536x1536 street frame, SH degree 1: means3D 3.5e-4 rel L2).
#ifndef GSR_FWD_POLY
#define GSR_FWD_POLY 0
#endif
#ifndef GSR_FWD_MASKSEL
#define GSR_FWD_MASKSEL 1
#endif
constexpr int kFcmpUGE = 11, kFcmpULE = 13;  // llvm::CmpInst unordered-or predicates: !(x < y), !(x > y)
// per-lane select by a wave mask held in SGPRs (mask bit set: t)
__device__ __forceinline__ float lane_select(uint64_t mask, float t, float f) {
    float r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(mask));
    return r;
}

#ifndef GSR_FWD_EARLY_EXIT
#define GSR_FWD_EARLY_EXIT 1  // leave a batch once every pixel of the sub-block has saturated
#endif
template <int kSub>
__device__ __forceinline__ uint32_t sub_block_mask_n(const float4 &qa, const float4 &qb, float tm, float tx0,
                                                     float ty0) {
    const float X = qa.x, Y = qa.y, ex = qb.z, ey = qb.w;
    if (!(X + ex >= tx0 && X - ex <= tx0 + 15.f)) return 0u;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kSub; k++) {
        const float y0 = ty0 + (float)(4 * k);
        if (Y + ey >= y0 && Y - ey <= y0 + 3.f &&
            (!(GSR_EXACT_CULL & 1) || ellipse_meets_box(X, Y, qa.z, qa.w, qb.x, tm, tx0, tx0 + 15.f, y0, y0 + 3.f)))
            m |= 1u << k;
    }
    return m;
}

// The tile's backward work (last contributor position): tile_work, and with bwd_cnt its slot in
// the backward's heaviest-first class lists.  With backward segments (seg_len != 0) a tile of more
// than seg_len positions of work is cut into ceil(work / seg_len) backward items (tile + ntiles *
// segment): all but the last go to the segment list (past the checkpoints), run first; the last one
// goes into its work class like a whole tile.
__device__ __forceinline__ void fwd_publish(uint32_t mx, int tile, uint32_t *__restrict__ tile_work,
                                            uint32_t *__restrict__ bwd_cnt, uint32_t *__restrict__ bwd_cls, int ntiles,
                                            uint32_t seg_len, float *ck, uint32_t kf) {
    tile_work[tile] = mx;
    if (!bwd_cnt) return;
    uint32_t item = (uint32_t)tile, wk = mx;
    if (seg_len && mx > seg_len) {
        const uint32_t nseg = (mx + seg_len - 1u) / seg_len;
        uint32_t *items = reinterpret_cast<uint32_t *>(ck + ck_slots(kf, seg_len) * (kCkFloats * 256));
        const uint32_t b = atomicAdd(&bwd_cnt[kBwdSegCount], nseg - 1u);
        for (uint32_t sgi = 0; sgi + 1u < nseg; sgi++) items[b + sgi] = (uint32_t)tile + (uint32_t)ntiles * sgi;
        item = (uint32_t)tile + (uint32_t)ntiles * (nseg - 1u);
        wk = mx - (nseg - 1u) * seg_len;
    }
    const uint32_t k = wk >> kBwdClassShift;
    const uint32_t c = (uint32_t)(kBwdClasses - 1) - (k < (uint32_t)(kBwdClasses - 1) ? k : (uint32_t)(kBwdClasses - 1));
    const uint32_t r = atomicAdd(&bwd_cnt[c], 1u);
    bwd_cls[(size_t)c * ntiles + r] = item;
}


// One wave's pass over list positions [p0, p1) of its 16x4 sub-block (forward segments), with the
// arithmetic of render_fwd's blend (kSub 1, wave masks).
// kBlend = false: the transmittance through the positions -- T *= 1 - alpha for every alpha the
//   blend would take (inside the ellipse, alpha >= 1/255) -- without the stop rule; a lane whose
//   product fell below 1e-4 leaves (any later position stops at its first contributor anyway).
// kBlend = true: the blend from the lane's T with the stop rule (stopm: lanes that stopped here)
//   and the backward checkpoints (colour accumulated in front of them since p0).
template <bool kBlend>
__device__ __forceinline__ void fwd_seg_pass(const uint32_t *__restrict__ point_list, const GRec *__restrict__ rec,
                                             uint32_t rgx, uint32_t p0, uint32_t p1, float4 *sa, float4 *sb, float4 *sc,
                                             float pfx, float pfy, float tx0, float sy0, uint64_t &livem, uint64_t &stopm,
                                             float &T, float &C0, float &C1, float &C2, float &ID, uint32_t &last,
                                             float *ck, uint32_t seg_len, uint32_t &ncross) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t lastpos = p1 - 1u;
    FwdBatch cur;
    fwd_gather(rec, point_list[min(p0 + (uint32_t)lane, lastpos)], cur);
    uint32_t gnext = point_list[min(p0 + kWave + (uint32_t)lane, lastpos)];
    for (uint32_t base = p0; base < p1; base += kWave) {
        if (!livem) break;
        if (kBlend && ck && base > rgx && (base - rgx) % seg_len == 0u) {
            float *c = ck + (size_t)(base / seg_len) * (kCkFloats * 256) + w * kWave + lane;
            c[0] = T;
            c[256] = C0;
            c[512] = C1;
            c[768] = C2;
            c[1024] = ID;
            ncross++;
        }
        const bool valid = base + (uint32_t)lane < p1;
        const float4 qa = cur.a, qb = cur.b, qc = cur.c;
        const uint32_t m = valid ? sub_block_mask_n<1>(qa, qb, cur.tm, tx0, sy0) : 0u;
        fwd_gather(rec, gnext, cur);
        gnext = point_list[min(base + 2 * kWave + (uint32_t)lane, lastpos)];
        const uint64_t keep = __ballot(m != 0u);
        const uint32_t cnt = (uint32_t)__popcll(keep);
        if (m) {
            const uint32_t slot = lane_prefix(keep);
            sa[slot] = make_float4(qa.x, qa.y, qa.z * kHalfLog2e, qa.w * kLog2e);
            sb[slot] = make_float4(qb.x * kHalfLog2e, qb.y, 0.f, __uint_as_float(base - rgx + (uint32_t)lane + 1u));
            if (kBlend) sc[slot] = qc;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t j = 0; j < cnt; j++) {
            const float4 a = sa[j];
            const float4 b = sb[j];
            const float dx = a.x - pfx;
            const float adxdx_s = a.z * dx * dx;
            const float bdx_s = a.w * dx;
            const float dy = a.y - pfy;
            const float p2 = gauss_p2(adxdx_s, bdx_s, b.x, dy);
            const float alpha = fminf(0.99f, b.y * gexp2(p2));
            const uint64_t okm = livem & __builtin_amdgcn_fcmpf(p2, 0.0f, kFcmpULE) &
                                 __builtin_amdgcn_fcmpf(alpha, 1.0f / 255.0f, kFcmpUGE);
            const float test_T = T * (1.f - alpha);
            if (kBlend) {
                const float4 c = sc[j];
                const uint64_t contm = __builtin_amdgcn_fcmpf(test_T, 0.0001f, kFcmpUGE);
                const uint64_t accm = okm & contm;
                stopm |= okm & ~contm;
                livem &= ~okm | contm;
                const float wgt = lane_select(accm, alpha * T, 0.f);
                C0 = fmaf(c.x, wgt, C0);
                C1 = fmaf(c.y, wgt, C1);
                C2 = fmaf(c.z, wgt, C2);
                ID = fmaf(c.w, wgt, ID);
                T = lane_select(accm, test_T, T);
                last = __float_as_uint(lane_select(accm, b.w, __uint_as_float(last)));
            } else {
                T = lane_select(okm, test_T, T);
                livem &= __builtin_amdgcn_fcmpf(T, 0.0001f, kFcmpUGE);
            }
            if (!livem) break;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Cross-workgroup hand-offs of the forward segments (MI355X_MICROARCH.md, the hand-off rules):
// producer -- every wave drains its stores, the workgroup meets, lane 0 writes the XCD's L2 back
// (agent release) and drains that before the flag / counter; consumer -- after lane 0 saw the flag,
// one agent acquire, drained, then the barrier, then plain loads.
__device__ __forceinline__ void wg_release() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
__device__ __forceinline__ void wg_acquire() {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// render_fwd_seg_kernel's workgroups (forward segments): items from the queue tile_order
// filled until it is empty (FwdSegLayout).  Item i = segment s of its tile: (1) the transmittance
// through the segment published per pixel (skipped for the tile's last segment; segment 0 publishes
// the transmittance its blend ends with instead, so a tile whose pixels saturate early costs about
// what it costs unsplit); (2) the product of
// the predecessors', in segment order once every predecessor's flag is set (each row made visible
// with a release fence before its flag; items of a tile are taken in order, so every predecessor's
// workgroup is resident), so the product does not depend on which item finished first; (3) the blend from that transmittance into the item's partials; (4) the
// tile's last item to finish (a ticket) adds the partials in segment order (up to the pixel's stop),
// turns the backward checkpoints into colour-behind and writes the tile's pixels.
__device__ void fwd_seg_worker(const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H,
                               int gx, const GRec *__restrict__ rec, const float *__restrict__ bg, float *__restrict__ out_color,
                               float *__restrict__ out_invd, float *__restrict__ final_T, uint32_t *__restrict__ n_contrib,
                               uint32_t *__restrict__ tile_work, uint32_t kf, const uint32_t *__restrict__ sort_err,
                               uint32_t *__restrict__ bwd_cnt, uint32_t *__restrict__ bwd_cls, int ntiles, uint32_t seg_len,
                               uint32_t fseg_len, uint32_t *bin_base, uint32_t *fctl, float4 *sa, float4 *sb,
                               float4 *sc, uint32_t *s_work, uint32_t *s_scalar, const uint32_t *ready,
                               FwdSpin spin, uint64_t &t_ready, uint64_t &t_flags) {
    // t_ready / t_flags (thread 0, GSR_FWD_POOL_STATS): s_memrealtime ticks spent waiting for the
    // queue's release and for predecessor segments' flags
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const FwdSegLayout f = fseg_layout(bin_base, kf, seg_len, fseg_len);
    float *ck = seg_len && bwd_cnt ? reinterpret_cast<float *>(reinterpret_cast<char *>(bin_base) + ck_offset(kf)) : nullptr;
    if (ready) {
        // launched ahead of tile_order on another stream: wait for its release of the queue.  Nothing
        // guarantees the two streams run concurrently (they may share a hardware queue, and counter
        // collection serialises dispatches), so the spin is bounded: a worker that gives up has
        // dequeued nothing, counts itself in the pinned kHostFwdGiveUp word (the host reports it:
        // gsr_forward_stats) and leaves; the pool's second launch after render_fwd on the main
        // stream (launch_render_fwd_cleanup) then takes every item still queued -- the frame stays
        // exact, only slower.
        if (threadIdx.x == 0) {
            const uint64_t t0 = GSR_FWD_POOL_STATS ? __builtin_amdgcn_s_memrealtime() : 0ull;
            uint32_t ok = 1u, spins = 0;
            // spin.ready == kFwdReadyNever (fault injection, tests): leave as if the word never came
            while (spin.ready == kFwdReadyNever || !__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                if (++spins > spin.ready || spin.ready == kFwdReadyNever) {
                    ok = 0u;
                    if (spin.host) __hip_atomic_store(spin.host + kHostFwdGiveUp, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            if (GSR_FWD_POOL_STATS) t_ready += __builtin_amdgcn_s_memrealtime() - t0;
            s_scalar[2] = ok;
        }
        wg_acquire();
        if (!s_scalar[2]) return;
        __syncthreads();  // s_scalar[2] is reused below
    }
    const uint32_t nitems = fctl[0];
    if (blockIdx.x >= nitems) return;  // more workers than items: the rest leave without a dequeue
    for (;;) {
        if (threadIdx.x == 0) s_scalar[0] = __hip_atomic_fetch_add(&fctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const uint32_t i = s_scalar[0];
        __syncthreads();
        if (i >= nitems) return;
        const uint32_t item = f.items[i];
        const int tile = (int)(item % (uint32_t)ntiles);
        const uint32_t sgi = item / (uint32_t)ntiles;
        const uint2 rg = ranges[tile];
        const uint32_t nseg = (rg.y - rg.x + fseg_len - 1u) / fseg_len;
        const uint32_t p0 = rg.x + sgi * fseg_len, p1 = min(p0 + fseg_len, rg.y);
        const uint32_t i0 = i - sgi;  // the tile's first item
        const int tx = tile % gx, ty = tile / gx;
        const int px = tx * kTile + (lane & 15), py = ty * kTile + 4 * w + (lane >> 4);
        const bool inside = px < W && py < H;
        const float pfx = (float)px, pfy = (float)py, tx0 = (float)(tx * kTile), sy0 = (float)(ty * kTile + 4 * w);
        const uint64_t insm = __ballot(inside);
        float Ta = 1.f, d0 = 0.f, d1 = 0.f, d2 = 0.f, d3 = 0.f;
        uint32_t du = 0, dn = 0;
        if (sgi > 0 && sgi + 1u < nseg) {  // (1) (item 0 publishes its blend's end transmittance instead)
            uint64_t lm = insm, sm = 0;
            fwd_seg_pass<false>(point_list, rec, rg.x, p0, p1, sa, sb, sc, pfx, pfy, tx0, sy0, lm, sm, Ta, d0, d1, d2, d3,
                                du, nullptr, 0u, dn);
            f.agg[(size_t)i * 256 + threadIdx.x] = Ta < 0.0001f ? 0.f : Ta;
            wg_release();
            if (threadIdx.x == 0) __hip_atomic_store(f.flags + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // (2) the predecessors' rows, multiplied in segment order (the same product whichever
        // finished first: the frame is bitwise repeatable)
        float Tin = 1.f;
        bool hung = false;
        if (sgi > 0) {
            if (threadIdx.x == 0) {
                const uint64_t t0 = GSR_FWD_POOL_STATS ? __builtin_amdgcn_s_memrealtime() : 0ull;
                uint32_t ok = 1u;
                for (uint32_t j = 0; j < sgi && ok; j++) {
                    uint32_t spins = 0;
                    while (!__hip_atomic_load(f.flags + i0 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        if (++spins > spin.flag) {
                            // never expected (every predecessor was dequeued earlier, so its workgroup
                            // is resident): the tile's pixels become NaN and the sticky error word
                            // makes the host's next rasterizer call fail (gsr_last_error)
                            ok = 0u;
                            if (spin.host) __hip_atomic_store(spin.host + kHostFwdErr, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_SYSTEM);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
                if (GSR_FWD_POOL_STATS) t_flags += __builtin_amdgcn_s_memrealtime() - t0;
                s_scalar[2] = ok;
            }
            wg_acquire();
            hung = s_scalar[2] == 0u;
            for (uint32_t j = 0; j < sgi; j++) Tin *= f.agg[(size_t)(i0 + j) * 256 + threadIdx.x];
        }
        // (3)
        float T = Tin, C0 = 0.f, C1 = 0.f, C2 = 0.f, ID = 0.f;
        uint32_t last = 0, ncross = 0;
        {
            uint64_t lm = insm, sm = 0;
            fwd_seg_pass<true>(point_list, rec, rg.x, p0, p1, sa, sb, sc, pfx, pfy, tx0, sy0, lm, sm, T, C0, C1, C2, ID,
                               last, ck, seg_len, ncross);
            if (sgi == 0) {
                // item 0's row: the transmittance its blend ended with (exactly the sequential one;
                // 0 for pixels that stopped), published as soon as the blend is done
                f.agg[(size_t)i * 256 + threadIdx.x] = ((sm >> lane) & 1ull) ? 0.f : T;
                wg_release();
                if (threadIdx.x == 0) __hip_atomic_store(f.flags + i, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            float *q = f.part + (size_t)i * (kFwdPartials * 256) + threadIdx.x;
            q[0] = C0;
            q[256] = C1;
            q[512] = C2;
            q[768] = ID;
            q[1024] = T;
            q[1280] = __uint_as_float(last | (((sm >> lane) & 1ull) ? 0x80000000u : 0u) | (hung ? 0x40000000u : 0u));
            if (lane == 0) f.nc[(size_t)i * 4 + w] = ncross;
        }
        wg_release();
        if (threadIdx.x == 0)
            s_scalar[1] = __hip_atomic_fetch_add(&f.tickets[i0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (s_scalar[1] + 1u != nseg) continue;
        wg_acquire();
        // (4) the tile's pixels: partials added in segment order up to the segment the pixel stopped in
        float A0 = 0.f, A1 = 0.f, A2 = 0.f, A3 = 0.f, Tf = 1.f;
        uint32_t lp = 0;
        bool bad = sort_err && *sort_err;
        for (uint32_t k = 0; k < nseg; k++) {
            const float *q = f.part + (size_t)(i0 + k) * (kFwdPartials * 256) + threadIdx.x;
            const uint32_t lw = __float_as_uint(q[1280]);
            A0 += q[0];
            A1 += q[256];
            A2 += q[512];
            A3 += q[768];
            Tf = q[1024];
            if (lw & 0x3FFFFFFFu) lp = lw & 0x3FFFFFFFu;
            bad = bad || (lw & 0x40000000u);
            if (lw & 0x80000000u) break;
        }
        if (ck) {
            // backward checkpoints: colour in front (the segments before + the segment's own part in
            // front of the checkpoint) -> colour still to come, B = C_final - C(in front)
            float P0 = 0.f, P1 = 0.f, P2 = 0.f, P3 = 0.f;
            bool stopped = false;
            for (uint32_t k = 0; k < nseg; k++) {
                const uint32_t nc = f.nc[(size_t)(i0 + k) * 4 + w];
                const uint32_t m0 = max(1u, (k * fseg_len + seg_len - 1u) / seg_len);
                for (uint32_t m = 0; m < nc; m++) {
                    float *c = ck + (size_t)((rg.x + (m0 + m) * seg_len) / seg_len) * (kCkFloats * 256) + w * kWave + lane;
                    c[256] = A0 - (P0 + c[256]);
                    c[512] = A1 - (P1 + c[512]);
                    c[768] = A2 - (P2 + c[768]);
                    c[1024] = A3 - (P3 + c[1024]);
                }
                if (!stopped) {
                    const float *q = f.part + (size_t)(i0 + k) * (kFwdPartials * 256) + threadIdx.x;
                    P0 += q[0];
                    P1 += q[256];
                    P2 += q[512];
                    P3 += q[768];
                    stopped = (__float_as_uint(q[1280]) & 0x80000000u) != 0u;
                }
            }
        }
        if (inside) {
            const int pix = py * W + px;
            const float nan = __builtin_nanf("");
            final_T[pix] = Tf;
            n_contrib[pix] = lp;
            out_color[pix] = bad ? nan : A0 + Tf * bg[0];
            out_color[H * W + pix] = bad ? nan : A1 + Tf * bg[1];
            out_color[2 * H * W + pix] = bad ? nan : A2 + Tf * bg[2];
            if (out_invd) out_invd[pix] = bad ? nan : A3;
        }
        const uint32_t wl = wave_max_u32(lp);
        if (lane == 0) s_work[w] = wl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t mx = s_work[0];
            for (int k = 1; k < kPixPerLane; k++) mx = s_work[k] > mx ? s_work[k] : mx;
            fwd_publish(mx, tile, tile_work, bwd_cnt, bwd_cls, ntiles, ck ? seg_len : 0u, ck, kf);
        }
        __syncthreads();
    }
}

// Forward segments' worker pool: kFwdPoolWorkers workgroups, launched beside render_fwd (which skips
// the split tiles) on a side stream, until the item queue is empty.
__global__ __launch_bounds__(kWave * kPixPerLane) void render_fwd_seg_kernel(
    const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H, int gx,
    const GRec *__restrict__ rec, const float *__restrict__ bg, float *__restrict__ out_color,
    float *__restrict__ out_invd, float *__restrict__ final_T, uint32_t *__restrict__ n_contrib,
    uint32_t *__restrict__ tile_work, const uint32_t *__restrict__ kdev, uint32_t cap,
    const uint32_t *__restrict__ sort_err, uint32_t *__restrict__ bwd_cnt, uint32_t *__restrict__ bwd_cls, int ntiles,
    uint32_t seg_len, uint32_t *bin_base, uint32_t fseg_len, uint32_t *fctl, const uint32_t *ready, FwdSpin spin) {
    GSR_KS(kKsFwdSeg);
    if (kdev && *kdev > cap) return;  // the point-list capacity is short: the host re-runs at K
    __shared__ float4 s_a[kPixPerLane][kWave];
    __shared__ float4 s_b[kPixPerLane][kWave];
    __shared__ float4 s_c[kPixPerLane][kWave];
    __shared__ uint32_t s_work[kPixPerLane], s_scalar[3];
    const int w = threadIdx.x >> 6;
    const uint64_t t0 = GSR_FWD_POOL_STATS ? __builtin_amdgcn_s_memrealtime() : 0ull;
    uint64_t t_ready = 0, t_flags = 0;
    fwd_seg_worker(ranges, point_list, W, H, gx, rec, bg, out_color, out_invd, final_T, n_contrib, tile_work,
                   kdev ? *kdev : cap, sort_err, bwd_cnt, bwd_cls, ntiles, seg_len, fseg_len, bin_base, fctl, s_a[w],
                   s_b[w], s_c[w], s_work, s_scalar, ready, spin, t_ready, t_flags);
    if (GSR_FWD_POOL_STATS && threadIdx.x == 0) {
        // the pool's time split (gsr_fwd_pool_stats): four no-return atomics per workgroup and frame
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_fwd_pool_ticks[0], (unsigned long long)t_ready);
        atomicAdd(&g_fwd_pool_ticks[1], (unsigned long long)t_flags);
        atomicAdd(&g_fwd_pool_ticks[2], (unsigned long long)(t1 - t0));
        atomicAdd(&g_fwd_pool_ticks[3], 1ull);
    }
}

#ifndef GSR_FWD_SEG_INKERNEL
#define GSR_FWD_SEG_INKERNEL 0  // 1: the worker pool as render_fwd's first workgroups (no side stream)
#endif
#if GSR_FWD_SEG_INKERNEL
#define GSR_FWD_ATTR __attribute__((amdgpu_waves_per_eu(8)))
#else
#define GSR_FWD_ATTR
#endif
template <int kSub>
__global__ __launch_bounds__(kWave * (kPixPerLane / kSub)) GSR_FWD_ATTR void render_fwd_kernel(
    const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H, int gx,
    const GRec *__restrict__ rec, const float *__restrict__ bg, float *__restrict__ out_color,
    float *__restrict__ out_invd, float *__restrict__ final_T, uint32_t *__restrict__ n_contrib,
    uint32_t *__restrict__ tile_work, const uint32_t *__restrict__ fwd_order, const uint32_t *__restrict__ kdev,
    uint32_t cap, const uint32_t *__restrict__ sort_err, float4 *__restrict__ acc, uint32_t acc_n4,
    uint32_t *__restrict__ bwd_cnt, uint32_t *__restrict__ bwd_cls, int ntiles, int gy, int sb_nsbx, int sb_shift,
    uint32_t seg_len, uint32_t *__restrict__ bin_base, uint32_t fseg_len, uint32_t *__restrict__ fctl, uint32_t fseg_min,
    const uint32_t *__restrict__ longest, uint32_t *host_words, FwdSpin spin) {
    GSR_KS(kKsRenderFwd);
    constexpr int kWaves = kPixPerLane / kSub;
    if (kdev && *kdev > cap) return;  // the point-list capacity is short: the host re-runs at K
    if (host_words && blockIdx.x == 0 && threadIdx.x == 0) {
        // the split gate's hints, written to pinned host memory here rather than by tile_order /
        // sb_colscan: the PCIe store's completion is hidden in this long launch instead of ending
        // a short one
        __hip_atomic_store(host_words + kHostTileList, longest[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_words + kHostSBList, longest[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (GSR_FWD_ACC_CLEAR) {
        // the backward's per-Gaussian accumulator rows (atomic mode) start at zero: every
        // workgroup clears one slice with streaming stores that drain while it blends (the
        // blend is VALU-bound; HBM is nearly idle here)
        const uint32_t per = (acc_n4 + gridDim.x - 1) / gridDim.x;
        const uint32_t a0 = blockIdx.x * per, a1 = min(acc_n4, a0 + per);
        for (uint32_t k = a0 + threadIdx.x; k < a1; k += blockDim.x)
        {
            typedef float f4 __attribute__((ext_vector_type(4)));
            if (GSR_ACC_NT) __builtin_nontemporal_store(f4{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f4 *>(acc + k));
            else acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __shared__ float4 s_a[kWaves][kWave];  // x, y, a_s, b_s (conic scaled for gauss_p2)
    __shared__ float4 s_b[kWaves][kWave];  // c_s, opacity, sub-block mask, list position + 1
    __shared__ float4 s_c[kWaves][kWave];  // r, g, b, 1 / depth
    __shared__ uint32_t s_work[kWaves];

#if GSR_FWD_SEG_INKERNEL
    // forward segments: the first kFwdWorkers workgroups are the worker pool (fwd_seg_worker)
    uint32_t bidx = blockIdx.x;
    if constexpr (kSub == 1) {
        if (fseg_len) {
            if (bidx < (uint32_t)kFwdWorkers) {
                __shared__ uint32_t s_scalar[3];
                uint64_t t_ready = 0, t_flags = 0;
                fwd_seg_worker(ranges, point_list, W, H, gx, rec, bg, out_color, out_invd, final_T, n_contrib,
                               tile_work, kdev ? *kdev : cap, sort_err, bwd_cnt, bwd_cls, ntiles, seg_len, fseg_len,
                               bin_base, fctl, s_a[threadIdx.x >> 6], s_b[threadIdx.x >> 6], s_c[threadIdx.x >> 6],
                               s_work, s_scalar, nullptr, spin, t_ready, t_flags);
                return;
            }
            bidx -= (uint32_t)kFwdWorkers;
        }
    }
#else
    const uint32_t bidx = blockIdx.x;
#endif

    int tile, tx, ty;
    if (sb_shift >= 0) {
        // superblock launch order (GSR_FWD_SB_ORDER): fwd_order lists the SBs, a workgroup per SB
        // tile slot; slots past the grid's edge have no tile
        const uint32_t per = 1u << (2 * sb_shift), b = bidx;
        const uint32_t k = fwd_order[b >> (2 * sb_shift)], t = b & (per - 1u);
        tx = (int)(k % (uint32_t)sb_nsbx) * (1 << sb_shift) + (int)(t & ((1u << sb_shift) - 1u));
        ty = (int)(k / (uint32_t)sb_nsbx) * (1 << sb_shift) + (int)(t >> sb_shift);
        if (tx >= gx || ty >= gy) return;
        tile = ty * gx + tx;
    } else {
        tile = (int)fwd_order[bidx];
        tx = tile % gx;
        ty = tile / gx;
    }
    if (fseg_splits(ranges[tile].y - ranges[tile].x, fseg_min)) return;  // render_fwd_seg_kernel's tile
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int px = tx * kTile + (lane & 15);
    const int sy = ty * kTile + 4 * kSub * w;  // the wave's first pixel row
    const float pfx = (float)px;
    // kPoly: the lane's offset from its sub-block's centre and its products (exact in fp32)
    constexpr bool kPoly = GSR_FWD_POLY && kSub == 1;
    const float lx = (float)(lane & 15) - 7.5f, ly = (float)(lane >> 4) - 1.5f;
    const float lxx = lx * lx, lxy = lx * ly, lyy = ly * ly;
    const float tx0 = (float)(tx * kTile), sy0 = (float)sy;

    // liveness: kSub == 1 keeps a lane mask (no branches in the blend); otherwise a dead pixel's
    // alpha threshold is 2 (above any alpha)
    float T[kSub], C0[kSub], C1[kSub], C2[kSub], ID[kSub], pfy[kSub], amin[kSub];
    uint32_t last[kSub];
    bool alive[kSub];
#pragma unroll
    for (int k = 0; k < kSub; k++) {
        const int py = sy + (lane >> 4) + 4 * k;
        pfy[k] = (float)py;
        T[k] = 1.f;
        C0[k] = C1[k] = C2[k] = ID[k] = 0.f;
        last[k] = 0u;
        alive[k] = px < W && py < H;
        amin[k] = alive[k] ? 1.0f / 255.0f : 2.f;
    }
    uint64_t livem = __ballot(alive[0]);  // GSR_FWD_MASKSEL: the live pixels as a wave mask
    StatAcc fst;
    uint64_t fwd_acc = 0;
    const uint2 rg = ranges[tile];
    FwdBatch cur;
    uint32_t gnext = 0;
    const uint32_t lastpos = rg.y > rg.x ? rg.y - 1u : rg.x;
    if (rg.y > rg.x) {
        fwd_gather(rec, point_list[min(rg.x + (uint32_t)lane, lastpos)], cur);
        gnext = point_list[min(rg.x + kWave + (uint32_t)lane, lastpos)];
    }
    // backward segments (seg_len != 0, kSub == 1): at every seg_len-th list position of the tile the
    // wave checkpoints its pixels' transmittance and accumulated colour / inverse depth (the state
    // in front of that position) into the binning buffer past the point list (bwd_segments)
    const bool segs = kSub == 1 && seg_len != 0u && bwd_cnt != nullptr;
    float *ck = nullptr;
    uint32_t ncross = 0;
    if (segs) ck = reinterpret_cast<float *>(reinterpret_cast<char *>(bin_base) + ck_offset(kdev ? *kdev : cap));
    for (uint32_t base = rg.x; base < rg.y; base += kWave) {
        uint32_t live = 0;  // sub-blocks with a pixel still accumulating (wave-uniform)
#pragma unroll
        for (int k = 0; k < kSub; k++)
            live |= (kSub == 1 && GSR_FWD_MASKSEL ? livem != 0 : __ballot(kSub == 1 ? alive[k] : amin[k] < 1.f) != 0)
                        ? 1u << k
                        : 0u;
        if (!live) break;
        if (segs && base > rg.x && (base - rg.x) % seg_len == 0u) {
            float *c = ck + (size_t)(base / seg_len) * (kCkFloats * 256) + w * kWave + lane;
            c[0] = T[0];
            c[256] = C0[0];
            c[512] = C1[0];
            c[768] = C2[0];
            c[1024] = ID[0];
            ncross++;
        }
        const bool valid = base + (uint32_t)lane < rg.y;
        const float4 qa = cur.a, qb = cur.b, qc = cur.c;
        const uint32_t m = valid ? sub_block_mask_n<kSub>(qa, qb, cur.tm, tx0, sy0) & live : 0u;
        // next batch in flight while this one blends
        fwd_gather(rec, gnext, cur);
        gnext = point_list[min(base + 2 * kWave + (uint32_t)lane, lastpos)];
        const uint64_t keep = __ballot(m != 0u);
        const uint32_t cnt = (uint32_t)__popcll(keep);
        if (m) {
            const uint32_t slot = lane_prefix(keep);
            const uint32_t pos1 = base - rg.x + (uint32_t)lane + 1u;  // n_contrib counts list positions from 1
            const float as = qa.z * kHalfLog2e, bs = qa.w * kLog2e, cs = qb.x * kHalfLog2e;
            if (kPoly) {
                // the exponent as a quadratic in the pixel's offset (lx, ly) from the sub-block
                // centre: p2 = F + D lx + E ly + a lx^2 - b lx ly + c ly^2
                const float X = qa.x - (tx0 + 7.5f), Y = qa.y - (sy0 + 1.5f);
                const float F = fmaf(-(bs * X), Y, fmaf(cs * Y, Y, (as * X) * X));
                const float D = fmaf(bs, Y, (-2.f * as) * X);
                const float E = fmaf(bs, X, (-2.f * cs) * Y);
                s_a[w][slot] = make_float4(F, D, E, as);
                s_b[w][slot] = make_float4(-bs, qb.y, cs, __uint_as_float(pos1));
            } else {
                s_a[w][slot] = make_float4(qa.x, qa.y, as, bs);
                s_b[w][slot] = make_float4(cs, qb.y, __uint_as_float(m), __uint_as_float(pos1));
            }
            s_c[w][slot] = qc;
        }
        // wave-private LDS slice: the wave's own writes are visible after its lgkmcnt drain
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const auto blend = [&](uint32_t j) {
            const float4 a = s_a[w][j];
            const float4 b = s_b[w][j];
            const float4 c = s_c[w][j];
            const uint32_t mk = kSub > 1 ? __builtin_amdgcn_readfirstlane(__float_as_uint(b.z)) : 1u;
            // kPoly: a = (F, D, E, a_s), b = (-b_s, opacity, c_s, position)
            const uint32_t pos = __float_as_uint(b.w);
            const float dx = kPoly ? 0.f : a.x - pfx;
            const float adxdx_s = a.z * dx * dx;
            const float bdx_s = a.w * dx;
#pragma unroll
            for (int k = 0; k < kSub; k++) {
                if (kSub > 1 && !(mk & (1u << k))) continue;
                const float dy = a.y - pfy[k];
                const float p2 = kPoly ? fmaf(a.w, lxx, fmaf(b.x, lxy, fmaf(b.z, lyy, fmaf(a.y, lx, fmaf(a.z, ly, a.x)))))
                                       : gauss_p2(adxdx_s, bdx_s, b.x, dy);
                const float alpha = fminf(0.99f, b.y * gexp2(p2));
                if (kSub == 1 && GSR_FWD_MASKSEL) {
                    // the three tests as wave masks, combined on the scalar unit, and the three
                    // selects from one mask: one compare of test_T instead of two (the compiler
                    // materialises both the stop test and its negation)
                    const float test_T = T[k] * (1.f - alpha);
                    const uint64_t okm = livem & __builtin_amdgcn_fcmpf(p2, 0.0f, kFcmpULE) &
                                         __builtin_amdgcn_fcmpf(alpha, 1.0f / 255.0f, kFcmpUGE);
                    const uint64_t contm = __builtin_amdgcn_fcmpf(test_T, 0.0001f, kFcmpUGE);
                    const uint64_t accm = okm & contm;
                    if (GSR_BLEND_STATS) {
                        fst.add(okm);
                        fwd_acc += (uint64_t)__popcll(accm);
                    }
                    livem &= ~okm | contm;
                    const float wgt = lane_select(accm, alpha * T[k], 0.f);
                    C0[k] = fmaf(c.x, wgt, C0[k]);
                    C1[k] = fmaf(c.y, wgt, C1[k]);
                    C2[k] = fmaf(c.z, wgt, C2[k]);
                    ID[k] = fmaf(c.w, wgt, ID[k]);
                    T[k] = lane_select(accm, test_T, T[k]);
                    last[k] = __float_as_uint(lane_select(accm, b.w, __uint_as_float(last[k])));
                    continue;
                }
                const bool ok = kSub == 1 ? alive[k] && !(p2 > 0.0f) && !(alpha < 1.0f / 255.0f)
                                          : !(p2 > 0.0f) && !(alpha < amin[k]);
                const float test_T = T[k] * (1.f - alpha);
                const bool cont = !(test_T < 0.0001f);
                const bool accept = ok && cont;
                if (kSub == 1) alive[k] = alive[k] && !(ok && !cont);
                else amin[k] = ok && !cont ? 2.f : amin[k];
                const float wgt = accept ? alpha * T[k] : 0.f;
                C0[k] = fmaf(c.x, wgt, C0[k]);
                C1[k] = fmaf(c.y, wgt, C1[k]);
                C2[k] = fmaf(c.z, wgt, C2[k]);
                ID[k] = fmaf(c.w, wgt, ID[k]);
                T[k] = accept ? test_T : T[k];
                last[k] = accept ? pos : last[k];
            }
        };
        // two instances per iteration (by hand: the wave-mask compares are convergent, which
        // blocks the compiler's runtime unrolling) so their independent chains interleave
        uint32_t j = 0;
        for (; j + 1 < cnt; j += 2) {
            blend(j);
            blend(j + 1);
            if (GSR_FWD_EARLY_EXIT && !livem) break;  // every pixel of the sub-block has saturated
        }
        if (j < cnt && (!GSR_FWD_EARLY_EXIT || livem)) blend(j);
        __builtin_amdgcn_wave_barrier();
    }
    if (GSR_BLEND_STATS) {
        fst.flush(kFwdPairs);
        if (lane == 0) atomicAdd(&g_blend_stats[kFwdAcc], (unsigned long long)fwd_acc);
    }
    // the checkpoints' colour as the part still to come: B = C_final - C(in front)
    for (uint32_t i = 1; i <= ncross; i++) {
        float *c = ck + (size_t)((rg.x + i * seg_len) / seg_len) * (kCkFloats * 256) + w * kWave + lane;
        c[256] = C0[0] - c[256];
        c[512] = C1[0] - c[512];
        c[768] = C2[0] - c[768];
        c[1024] = ID[0] - c[1024];
    }
    const bool bad = sort_err && *sort_err;  // the depth sort gave up on a lookback: NaN frame
    uint32_t wl = 0;
#pragma unroll
    for (int k = 0; k < kSub; k++) {
        wl = last[k] > wl ? last[k] : wl;
        const int py = sy + (lane >> 4) + 4 * k;
        if (px < W && py < H) {
            const int pix = py * W + px;
            const float nan = __builtin_nanf("");
            final_T[pix] = T[k];
            n_contrib[pix] = last[k];
            out_color[pix] = bad ? nan : C0[k] + T[k] * bg[0];
            out_color[H * W + pix] = bad ? nan : C1[k] + T[k] * bg[1];
            out_color[2 * H * W + pix] = bad ? nan : C2[k] + T[k] * bg[2];
            if (out_invd) out_invd[pix] = bad ? nan : ID[k];
        }
    }
    wl = wave_max_u32(wl);
    // the tile's backward work (last contributor position): tile_work, and with bwd_cnt its slot in
    // the backward's heaviest-first class lists
    const auto publish = [&](uint32_t mx) {
        fwd_publish(mx, tile, tile_work, bwd_cnt, bwd_cls, ntiles, segs ? seg_len : 0u, ck, kdev ? *kdev : cap);
    };
    if (kWaves == 1) {
        if (lane == 0) publish(wl);
    } else {
        if (lane == 0) s_work[w] = wl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t mx = s_work[0];
            for (int k = 1; k < kWaves; k++) mx = s_work[k] > mx ? s_work[k] : mx;
            publish(mx);
        }
    }
}

// render_bwd's tile with GSR_BWD_CLS: workgroup b takes the (b - first)-th tile of the class whose
// range of launch positions holds b (class c covers [sum of counts below c, + count c)), from the
// 256 class counts render_fwd left (4 per lane, one wave scan).
__device__ __forceinline__ int bwd_tile_of(uint32_t b, const uint32_t *__restrict__ cnt, const uint32_t *__restrict__ cls,
                                           int T) {
    const int lane = threadIdx.x & 63;
    const uint4 c4 = reinterpret_cast<const uint4 *>(cnt)[lane];
    const uint32_t s4 = c4.x + c4.y + c4.z + c4.w;
    uint32_t incl = s4;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)incl, o, 64);
        if (lane >= o) incl += t;
    }
    const uint32_t excl = incl - s4;
    const uint64_t hit = __ballot(b >= excl && b < incl);
    if (!hit) return -1;  // past the listed items (the grid's room for segments)
    const int L = __ffsll((unsigned long long)hit) - 1;
    uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)excl, L);
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)c4.x, L), y = (uint32_t)__builtin_amdgcn_readlane((int)c4.y, L),
                   z = (uint32_t)__builtin_amdgcn_readlane((int)c4.z, L);
    int c = 4 * L;
    if (b >= off + x) { off += x; c++;
        if (b >= off + y) { off += y; c++;
            if (b >= off + z) { off += z; c++; } } }
    return (int)cls[(size_t)c * T + (b - off)];
}

// the shortest list the forward split takes: gsr_set_fwd_split_min's length, else GSR_FSEG_FACTOR
// segments (measurement A/B: gsr_set_fwd_split_min, or a -DGSR_FSEG_FACTOR build)
std::atomic<uint32_t> g_fseg_min{0};
uint32_t fseg_min_len(uint32_t Lf) {
    const uint32_t m = g_fseg_min.load(std::memory_order_relaxed);
    return m ? std::max(m, Lf) : (uint32_t)GSR_FSEG_FACTOR * Lf;
}
uint32_t set_fwd_split_min(uint32_t len) { return g_fseg_min.exchange(len); }

// Launch order for a tile pass, heaviest first (longest-processing-time-first list scheduling):
// one 1024-thread workgroup buckets the T work estimates into 256 descending classes of
// 2^shift instances (LDS histogram, scan, scatter).  Order within a class is arbitrary; every
// tile writes only its own outputs, so results do not depend on it.
__global__ __launch_bounds__(1024) void tile_order_kernel(const uint32_t *__restrict__ work, const uint2 *__restrict__ ranges,
                                                          int T, int shift, uint32_t *__restrict__ order, const uint32_t *__restrict__ kdev, uint32_t cap,
                                                          uint32_t *__restrict__ zero_classes, uint32_t *__restrict__ fctl,
                                                          void *bin_base, uint32_t seg_len, uint32_t fseg_len,
                                                          uint32_t fseg_min, uint32_t *__restrict__ host_tilelist,
                                                          uint32_t *fwd_ready) {
    GSR_KS(kKsTileOrder);
    // the forward order's launch also zeroes the backward class counters render_fwd fills
    if (zero_classes && threadIdx.x < kBwdClasses) zero_classes[threadIdx.x] = 0u;
    if (zero_classes && threadIdx.x == 0) zero_classes[kBwdSegCount] = 0u;
    if (kdev && *kdev > cap) return;  // ranges / work were not written this pass (capacity re-run)
    __shared__ uint32_t hist[256];
    __shared__ uint32_t s_items, s_max;
    if (threadIdx.x < 256) hist[threadIdx.x] = 0u;
    if (threadIdx.x == 0) s_items = s_max = 0u;
    __syncthreads();
    auto bucket = [&](int t) {
        const uint32_t wk = work ? work[t] : ranges[t].y - ranges[t].x;
        const uint32_t k = wk >> shift;
        return 255u - (k < 255u ? k : 255u);
    };
    // one pass over the tiles: the work histogram, the longest list (the split gate's hint) and,
    // with forward segments, the work-item queue of the tiles longer than fseg_min (a tile's items
    // consecutive, segment order; their tickets and flags zeroed)
    FwdSegLayout f{};
    if (fseg_len) f = fseg_layout(bin_base, kdev ? *kdev : cap, seg_len, fseg_len);
    uint32_t mx = 0;
    for (int t = threadIdx.x; t < T; t += 1024) {
        const uint32_t len = ranges[t].y - ranges[t].x;
        const uint32_t k = (work ? work[t] : len) >> shift;
        atomicAdd(&hist[255u - (k < 255u ? k : 255u)], 1u);
        mx = max(mx, len);
        if (fseg_splits(len, fseg_min)) {
            const uint32_t n = (len + fseg_len - 1u) / fseg_len;
            const uint32_t b = atomicAdd(&s_items, n);
            for (uint32_t q = 0; q < n; q++) {
                f.items[b + q] = (uint32_t)t + (uint32_t)T * q;
                f.tickets[b + q] = 0u;
                f.flags[b + q] = 0u;
            }
        }
    }
    if (host_tilelist) {
        // the wave's maximum first (DPP): one LDS atomic per wave instead of 1024 on one word
        mx = wave_max_u32(mx);
        if ((threadIdx.x & 63) == 0) atomicMax(&s_max, mx);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (host_tilelist) {
            if (GSR_HOST_WORDS == 2) *host_tilelist = s_max;  // a device word render_fwd forwards
            else __hip_atomic_store(host_tilelist, s_max, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (fseg_len) {
            fctl[0] = s_items;  // kFwdItemsWord
            fctl[1] = 0u;       // kFwdNextWord
        }
    }
    if (fseg_len && fwd_ready) {
        // the workers already wait: queue, tickets and flags released before the ready word
        wg_release();
        if (threadIdx.x == 0) __hip_atomic_store(fwd_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of 256 counts, 4 per lane
        const int l = threadIdx.x;
        const uint32_t a = hist[4 * l], b = hist[4 * l + 1], c = hist[4 * l + 2], d = hist[4 * l + 3];
        uint32_t sum = a + b + c + d, incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
            if (l >= o) incl += v;
        }
        const uint32_t ex = incl - sum;
        hist[4 * l] = ex;
        hist[4 * l + 1] = ex + a;
        hist[4 * l + 2] = ex + a + b;
        hist[4 * l + 3] = ex + a + b + c;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += 1024) order[atomicAdd(&hist[bucket(t)], 1u)] = (uint32_t)t;
}

void launch_tile_order(const uint32_t *work, const uint2 *ranges, int T, int shift, uint32_t *order, hipStream_t s,
                       const uint32_t *kdev, uint32_t cap, uint32_t *zero_classes, uint32_t *fctl, void *bin_base,
                       uint32_t seg_len, uint32_t fseg_len, uint32_t *host_tilelist, uint32_t *fwd_ready, uint32_t fseg_min) {
    if (T == 0) return;
    // fseg_min: the frame's split minimum, computed once by the caller (render_fwd's skip test must see
    // the same value, or a tile could be skipped without being queued)
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, s, work, ranges, T, shift, order, kdev, cap, zero_classes,
                       fctl, bin_base, seg_len, fctl ? fseg_len : 0u, fctl && fseg_len ? fseg_min : 0u,
                       host_tilelist, fwd_ready);
}

// the worker pool's size: kFwdPoolWorkers, or GSR_FWD_WORKERS from the environment (measurement A/B)
static int fwd_workers() {
    static const int n = [] {
        const char *e = getenv("GSR_FWD_WORKERS");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? v : kFwdPoolWorkers;
    }();
    return n;
}

bool fwd_early_workers() {  // read per frame, so a test can switch it
    const char *e = getenv("GSR_FWD_EARLY_WORKERS");
    return !(e && e[0] == '0');
}

static void launch_workers(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                           const float *bg, float *out_color, float *out_invdepth, bool need_bwd, uint32_t seg_len,
                           uint32_t fseg_len, hipStream_t ws, const uint32_t *ready, FwdSpin spin, int grid) {
    uint32_t *const bcnt = GSR_BWD_CLS && need_bwd ? is.bwd_cnt : nullptr;
    hipLaunchKernelGGL(render_fwd_seg_kernel, dim3(grid), dim3(kWave * kPixPerLane), 0, ws, is.ranges,
                       bs.point_list, cam.W, cam.H, cam.gx, gs.rec, bg, out_color, out_invdepth, is.final_T,
                       is.n_contrib, is.tile_work, bs.kdev, bs.cap, bs.kdev ? dsort_err_word(gs) : nullptr, bcnt,
                       is.bwd_cls, cam.gx * cam.gy, seg_len, bs.point_list, fseg_len, is.bwd_cnt + kFwdItemsWord,
                       ready, spin);
}

void launch_render_fwd_workers(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                               const float *bg, float *out_color, float *out_invdepth, bool need_bwd, uint32_t seg_len,
                               uint32_t fseg_len, hipStream_t ws, const uint32_t *ready, FwdSpin spin) {
    if (cam.gx * cam.gy == 0 || !fseg_len || GSR_FWD_SUB != 1 || GSR_FWD_SEG_INKERNEL) return;
    launch_workers(cam, gs, bs, is, bg, out_color, out_invdepth, need_bwd, seg_len, fseg_len, ws, ready, spin,
                   fwd_workers());
}

// 64 workgroups: normally they find the queue drained (or take a straggler's last items); if the early
// pool gave up entirely they blend every item, slowly but exactly
constexpr int kFwdCleanupWorkers = 64;
void launch_render_fwd_cleanup(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                               const float *bg, float *out_color, float *out_invdepth, bool need_bwd, uint32_t seg_len,
                               uint32_t fseg_len, hipStream_t s, FwdSpin spin) {
    if (cam.gx * cam.gy == 0 || !fseg_len || GSR_FWD_SUB != 1 || GSR_FWD_SEG_INKERNEL) return;
    launch_workers(cam, gs, bs, is, bg, out_color, out_invdepth, need_bwd, seg_len, fseg_len, s, nullptr, spin,
                   kFwdCleanupWorkers);
}

std::atomic<uint32_t> g_fwd_ready_spins{kFwdReadySpins}, g_fwd_flag_spins{kFwdFlagSpins};
FwdSpin fwd_spin(uint32_t *host_words) {
    return FwdSpin{g_fwd_ready_spins.load(std::memory_order_relaxed), g_fwd_flag_spins.load(std::memory_order_relaxed),
                   host_words};
}
void set_fwd_spin_limits(uint32_t ready, uint32_t flag) {
    g_fwd_ready_spins.store(ready ? ready : kFwdReadySpins);
    g_fwd_flag_spins.store(flag ? flag : kFwdFlagSpins);
}

void launch_render_fwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const float *bg, float *out_color, float *out_invdepth, hipStream_t s, bool need_bwd,
                       bool sb_order, uint32_t seg_len, uint32_t fseg_len, hipStream_t worker_stream,
                       bool workers_launched, const uint32_t *longest, uint32_t *host_words, uint32_t fseg_min,
                       FwdSpin spin) {
    const int T = cam.gx * cam.gy;
    if (T == 0) return;
    const SBGrid &sg = gs.sb;
    if (sb_order || GSR_FWD_SUB != 1) fseg_len = 0;
    const int grid = (sb_order ? sg.nsb << (2 * sg.shift) : T) + (GSR_FWD_SEG_INKERNEL && fseg_len ? kFwdWorkers : 0);
    if (fseg_len && !GSR_FWD_SEG_INKERNEL && !workers_launched)
        launch_workers(cam, gs, bs, is, bg, out_color, out_invdepth, need_bwd, seg_len, fseg_len,
                       worker_stream ? worker_stream : s, nullptr, spin, fwd_workers());
    // launch order: is.tile_ids (rasterizer.hip, by list length)
#define GSR_FWD_LAUNCH(K, NT)                                                                                       \
    hipLaunchKernelGGL(K, dim3(grid), dim3(NT), 0, s, is.ranges, bs.point_list, cam.W, cam.H, cam.gx, gs.rec, bg,   \
                       out_color, out_invdepth, is.final_T, is.n_contrib, is.tile_work, is.tile_ids, bs.kdev, bs.cap, \
                       bs.kdev ? dsort_err_word(gs) : nullptr, gs.acc, (uint32_t)(4 * (size_t)gs.nacc),              \
                       GSR_BWD_CLS && need_bwd ? is.bwd_cnt : nullptr, is.bwd_cls, T, cam.gy, sg.nsbx,        \
                       sb_order ? sg.shift : -1, seg_len, bs.point_list, fseg_len, is.bwd_cnt + kFwdItemsWord,       \
                       fseg_len ? fseg_min : 0u, longest, longest ? host_words : nullptr, spin)
    static_assert(GSR_FWD_SUB == 1 || GSR_FWD_SUB == 2 || GSR_FWD_SUB == 4, "GSR_FWD_SUB: 1, 2 or 4");
    GSR_FWD_LAUNCH(render_fwd_kernel<GSR_FWD_SUB>, kWave * (kPixPerLane / GSR_FWD_SUB));
#undef GSR_FWD_LAUNCH
}

// ------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------
// Per pixel the replay keeps only S = sum_c A_c dL/dpix_c (not the four accumulated channels) and
// sums G dL/dalpha moments in dy (sum u, sum u dy, sum u dy^2); the lane's dx, the opacity and
// the conic are applied once per instance after the k loop / the wave sum.  37 instead of 52
// VALU per active (instance, pixel), 104 instead of 152 VGPRs: 0.35 vs 0.48 ms.
//
// Sub-blocks an instance cannot touch (ellipse box, or past the sub-block's last contributor) are
// skipped with a scalar branch on the wave-uniform mask: 0.479 vs 0.502 ms for the predicated
// form on the 1M-Gaussian 1080p bench scene once tiles run heaviest-first.
#ifndef GSR_BWD_BG_IN_S
#define GSR_BWD_BG_IN_S 1  // 0: upstream's separate background term (one more FMA per pixel)
#endif
#ifndef GSR_BWD_WAVES_PER_EU
#define GSR_BWD_WAVES_PER_EU 4  // 4 waves per SIMD: the instance pairs would otherwise take 129 VGPRs (3 waves)
#endif
#ifndef GSR_TILE_REVERSE
#define GSR_TILE_REVERSE 0
#endif
#ifndef GSR_BWD_HALVES
#define GSR_BWD_HALVES 1  // 0: halves added per instance (5.5 KiB of LDS, 29 instead of 17 waves per CU): 0.2259 -> 0.2333 ms (r03f)
#endif
#ifndef GSR_REC_PAD
#define GSR_REC_PAD 1  // write the unused 4th float4 of a 64-B record (full 64-B segments)
#endif
struct BwdBatch {
    float4 a, b, c;  // GRec q0..q2
    uint4 q3;        // tile rect, depth bits, cull threshold
    uint32_t goff;   // record mode: the Gaussian's first backward record; atomic mode: its id
};

template <bool kAtomic>
__device__ __forceinline__ void bwd_gather(const GRec *__restrict__ rec, const uint32_t *__restrict__ goff, uint32_t g,
                                           BwdBatch &o) {
    const float4 *R = reinterpret_cast<const float4 *>(rec + g);
    o.a = R[0];
    o.b = R[1];
    o.c = R[2];
    o.q3 = reinterpret_cast<const uint4 *>(rec + g)[3];
    o.goff = kAtomic ? g : goff[g];
}

// this workgroup's share of the frame's dense zero gradient rows (ZeroRows): issued after the
// replay, so no wait of the replay covers them -- the VALU-bound replay leaves HBM nearly idle, and
// preprocess_bwd no longer streams these bytes on its own
__device__ __forceinline__ void bwd_zero_slice(const ZeroRows &zr) {
    const int lane = threadIdx.x;
    if (!zr.per4 || blockIdx.x < zr.zfrom) return;
    {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const uint64_t q0 = (uint64_t)(blockIdx.x - zr.zfrom) * zr.per4, q1 = min(zr.c4[kZeroArrays], q0 + zr.per4);
        for (uint64_t q = q0 + (uint64_t)lane; q < q1; q += kWave) {
            int k = 0;
#pragma unroll
            for (int a = 1; a < kZeroArrays; a++) k += q >= zr.c4[a];
            __builtin_nontemporal_store(f4{0.f, 0.f, 0.f, 0.f}, reinterpret_cast<f4 *>(zr.p[k]) + (q - zr.c4[k]));
        }
        if (blockIdx.x == zr.zfrom && lane < 4 * kZeroArrays) {  // the floats past each array's last whole float4
            const int k = lane >> 2, t = lane & 3;
            const uint64_t e = 4 * (zr.c4[k + 1] - zr.c4[k]) + (uint64_t)t;
            if (e < zr.n[k]) __builtin_nontemporal_store(0.f, zr.p[k] + e);
        }
    }
}

// kAtomic (default): every live instance's ten sums are added into its Gaussian's accumulator row
// (GeomState.acc) with no-return float atomics once per batch -- ten wave-wide atomic instructions,
// lanes = (instance, value) pairs, so each instance is ONE contiguous 40-B segment of a 64-B row
// (one memory-side request; MI355X_MICROARCH.md, Global float atomics).  Otherwise each instance
// writes a 64-B record at its Gaussian-major index and the tile's boundary key, and
// backward.hip's record_sum adds them up in a fixed order (bitwise reproducible).
template <bool kDepth, bool kAtomic>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(GSR_BWD_WAVES_PER_EU))) void render_bwd_kernel(
    const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list, int W, int H, int gx,
    const GRec *__restrict__ rec, const float *__restrict__ bg, const float *__restrict__ final_Ts,
    const uint32_t *__restrict__ n_contrib, const float *__restrict__ dL_dpix, const float *__restrict__ dL_dinvd,
    const uint32_t *__restrict__ tile_order, const uint32_t *__restrict__ goff, uint64_t *__restrict__ boundary,
    float4 *__restrict__ out, ZeroRows zr, const uint32_t *__restrict__ bwd_cnt, const uint32_t *__restrict__ bwd_cls,
    uint32_t ntiles, uint32_t seg_len, const float *__restrict__ ck, const uint32_t *__restrict__ seg_items) {
    GSR_KS(kKsRenderBwd);
    // 9 KiB of LDS per wave: each compacted instance's mean and conic (scaled for gauss_p2 by the
    // lane that stages it, once per instance instead of by the whole wave), opacity, list position
    // << 4 | sub-block mask, Gaussian id (atomic mode) or record index, colour, and the unscaled
    // conic for the batch epilogue
    __shared__ float4 s_a[kWave];  // x, y, a_s, b_s
    __shared__ float4 s_b[kWave];  // c_s, opacity, list position << 4 | sub-block mask, id / record index
    __shared__ float4 s_c[kWave];  // r, g, b, 1 / depth
    // per compacted instance: the two half-wave partials of its 10 sums, added once per batch
    // (GSR_BWD_HALVES = 0: the halves added per instance, half the LDS -- 29 instead of 17 waves per
    // CU -- but two more VALU per instance: slower, the kernel is issue-bound, not latency-bound)
    __shared__ float s_red[kWave * 10 * (GSR_BWD_HALVES ? 2 : 1)];
    __shared__ float4 s_d[GSR_BWD_HALVES ? kWave : 1];  // GSR_BWD_HALVES: conic a, b, c for the epilogue

    // Tiles run heaviest first (longest-processing-time order from the forward's per-tile work):
    // with ~2.7 tiles per wave slot, index order leaves a tail of a few heavy tiles.
    // With segments (seg_len != 0) the full segments render_fwd listed run first, then the class
    // lists; workgroups past both only zero their share of the gradient rows.
    int item;
    if (GSR_TILE_REVERSE) item = (int)blockIdx.x;
    else if (GSR_BWD_CLS) {
        const uint32_t nsg = seg_len ? bwd_cnt[kBwdSegCount] : 0u;
        item = blockIdx.x < nsg ? (int)seg_items[blockIdx.x] : bwd_tile_of(blockIdx.x - nsg, bwd_cnt, bwd_cls, (int)ntiles);
    } else item = (int)tile_order[blockIdx.x];
    if (item < 0) {
        bwd_zero_slice(zr);
        return;
    }
    const int tile = (int)((uint32_t)item % ntiles), seg = (int)((uint32_t)item / ntiles);
    const int tx = tile % gx, ty = tile / gx;
    const int lane = threadIdx.x;
    const int px = tx * kTile + (lane & 15);
    const int py0 = ty * kTile + (lane >> 4);
    const float pfx = (float)px;
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);
    const float b0 = bg[0], b1 = bg[1], b2 = bg[2];

    float T[kPixPerLane], dp0[kPixPerLane], dp1[kPixPerLane], dp2[kPixPerLane], did[kPixPerLane];
    // S = sum_c A_c dL/dpix_c: the colour (and inverse depth) accumulated behind the current
    // instance, already dotted with the pixel's upstream gradient -- the only form dL/dalpha needs.
    // The background is the layer behind the last contributor (alpha 1, colour bg): S starts at
    // bg . dL/dpix, which folds upstream's -T_final (bg . dL/dpix) / (1 - alpha) term into
    // T (cd - S) -- T_i S_i then carries T_final bg / (1 - alpha_i) by the same recurrence.
    float S[kPixPerLane], pfy[kPixPerLane], TfB[kPixPerLane];
    uint32_t last[kPixPerLane], lastk[kPixPerLane];
    uint32_t maxlast = 0;
    // every per-pixel input load first (clamped to the image, zeroed outside it), so the 24 loads
    // of a lane are in flight together instead of one round trip per pixel row
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        const int py = py0 + 4 * k;
        const int pix = min(py, H - 1) * W + min(px, W - 1);
        pfy[k] = (float)py;
        T[k] = final_Ts[pix];
        last[k] = n_contrib[pix];
        dp0[k] = dL_dpix[pix];
        dp1[k] = dL_dpix[H * W + pix];
        dp2[k] = dL_dpix[2 * H * W + pix];
        did[k] = kDepth ? dL_dinvd[pix] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < kPixPerLane; k++) {
        const bool inside = px < W && py0 + 4 * k < H;
        T[k] = inside ? T[k] : 0.f;
        last[k] = inside ? last[k] : 0u;
        dp0[k] = inside ? dp0[k] : 0.f;
        dp1[k] = inside ? dp1[k] : 0.f;
        dp2[k] = inside ? dp2[k] : 0.f;
        did[k] = inside ? did[k] : 0.f;
        S[k] = GSR_BWD_BG_IN_S ? fmaf(b2, dp2[k], fmaf(b1, dp1[k], b0 * dp0[k])) : 0.f;
        TfB[k] = GSR_BWD_BG_IN_S ? 0.f : -T[k] * (b0 * dp0[k] + b1 * dp1[k] + b2 * dp2[k]);
        lastk[k] = wave_max_u32(last[k]);  // sub-block k needs list positions < lastk[k]
        maxlast = lastk[k] > maxlast ? lastk[k] : maxlast;
    }
    const uint2 rg = ranges[tile];
    // the item's list positions [lo, hi): the whole tile's [0, maxlast), or segment `seg` of
    // ceil(maxlast / seg_len).  A pixel still accumulating past hi starts from the forward's
    // checkpoint at hi: T there, and S from the colour still to come B = C_final - C(hi),
    // S = ((B + T_final bg) . dL/dpix + B_d dL/dinvdepth) / T.
    uint32_t lo = 0, hi0 = maxlast;
    if (seg_len && maxlast > seg_len) {
        const uint32_t nseg = (maxlast + seg_len - 1u) / seg_len;
        lo = (uint32_t)seg * seg_len;
        hi0 = (uint32_t)seg + 1u == nseg ? maxlast : lo + seg_len;
    }
    if (hi0 < maxlast) {
        const float *c = ck + (size_t)((rg.x + hi0) / seg_len) * (kCkFloats * 256) + lane;
#pragma unroll
        for (int k = 0; k < kPixPerLane; k++) {
            if (last[k] > hi0) {
                const float Tb = c[k * kWave];
                float num = fmaf(c[256 + k * kWave] + T[k] * b0, dp0[k],
                                 fmaf(c[512 + k * kWave] + T[k] * b1, dp1[k], (c[768 + k * kWave] + T[k] * b2) * dp2[k]));
                if (kDepth) num = fmaf(c[1024 + k * kWave], did[k], num);
                S[k] = num / Tb;
                T[k] = Tb;
            }
        }
    }
    const float sx = 0.5f * (float)W, sy = 0.5f * (float)H;
    const int rs_slot = wave_rs10_slot(lane);
    const int rs20_slot = wave_rs20_slot(lane);
    (void)rs_slot;
    (void)rs20_slot;
    StatAcc bst;
    uint64_t b_inst = 0, b_batches = 0;

    // The gather is software-pipelined as in the forward: batch b-1's GRec lines and record bases
    // and batch b-2's ids are in flight while batch b replays (unconditional loads at clamped list
    // positions -- a masked load would be waited for at the end of its branch).
    BwdBatch cur;
    uint32_t gnext = 0;
    if (maxlast > 0) {
        const uint32_t g0 = point_list[rg.x + (uint32_t)max((int)hi0 - 1 - lane, (int)lo)];
        bwd_gather<kAtomic>(rec, goff, g0, cur);
        gnext = point_list[rg.x + (uint32_t)max((int)hi0 - 1 - kWave - lane, (int)lo)];
        // the tile's boundary key (its last segment): lane 0 holds the last instance any pixel uses
        if (!kAtomic && lane == 0 && hi0 == maxlast) boundary[tile] = ((uint64_t)cur.q3.z << 32) | g0;
    } else if (!kAtomic && lane == 0) {
        boundary[tile] = 0ull;
    }
    for (int hi = (int)hi0; hi > (int)lo; hi -= kWave) {
        const int n = hi - (int)lo < kWave ? hi - (int)lo : kWave;
        uint32_t m = 0, u = 0, pos = 0;
        const float4 qa = cur.a, qb = cur.b, qc = cur.c;
        if (lane < n) {
            pos = (uint32_t)(hi - 1 - lane);
            const uint4 q3 = cur.q3;
            u = kAtomic ? cur.goff  // the Gaussian id
                        : cur.goff + (uint32_t)((ty - (int)(q3.x >> 16)) * (int)q3.y + (tx - (int)(q3.x & 0xFFFFu)));
            m = sub_block_mask(qa, qb, __uint_as_float(q3.w), tx0, ty0);
#pragma unroll
            for (int k = 0; k < kPixPerLane; k++)
                if (pos >= lastk[k]) m &= ~(1u << k);
        }
        // next batch in flight while this one replays
        bwd_gather<kAtomic>(rec, goff, gnext, cur);
        gnext = point_list[rg.x + (uint32_t)max(hi - 1 - 2 * kWave - lane, (int)lo)];
        if (!kAtomic && lane < n && m == 0u) {  // in the live range but touches no pixel that needs it: zero record
            const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
            out[4 * (size_t)u + 0] = z;
            out[4 * (size_t)u + 1] = z;
            out[4 * (size_t)u + 2] = z;
            if (GSR_REC_PAD) out[4 * (size_t)u + 3] = z;
        }
        const uint64_t keep = __ballot(m != 0u);
        const uint32_t cnt = (uint32_t)__popcll(keep);
        if (GSR_BLEND_STATS) {
            b_inst += cnt;
            b_batches += 1;
        }
        const uint32_t slot = lane_prefix(keep);
        if (m) {
            s_a[slot] = make_float4(qa.x, qa.y, qa.z * kHalfLog2e, qa.w * kLog2e);  // scaled conic: gauss_p2
            s_b[slot] = make_float4(qb.x * kHalfLog2e, qb.y, __uint_as_float(pos << 4 | m), __uint_as_float(u));
            s_c[slot] = qc;
            if (GSR_BWD_HALVES) s_d[slot] = make_float4(qa.z, qa.w, qb.x, 0.f);
        }
        __syncthreads();
        // one compacted instance's replay over its sub-blocks: the ten lane sums q (dx moments
        // included); returns whether any lane's pixel took it
        const auto replay = [&](uint32_t j, float (&q)[10]) -> bool {
            const float4 a = s_a[j];
            const float4 b = s_b[j];
            const float4 c = s_c[j];
            const uint32_t pm = __builtin_amdgcn_readfirstlane(__float_as_uint(b.z));
            const uint32_t mk = pm & 0xFu;  // != 0: compacted instances touch a sub-block
            const uint32_t jpos = pm >> 4;
            const float dx = a.x - pfx;
            const float adxdx_s = a.z * dx * dx;
            const float bdx_s = a.w * dx;
            bool any = false;
            // Sub-block k's replay.  The first active sub-block sets the ten lane sums, later ones
            // add to them, so a culled sub-block 0 costs no zero moves (the compiler had peeled
            // k = 0 and materialised the zeros on that path).
            const auto pix = [&](auto kk, auto ff) {
                constexpr int k = decltype(kk)::value;
                constexpr bool first = decltype(ff)::value;
                const float dy = a.y - pfy[k];
                const float p2 = gauss_p2(adxdx_s, bdx_s, b.x, dy);
                const float G = gexp2(p2);
                const float alpha = fminf(0.99f, b.y * G);
                const bool ok = jpos < last[k] && !(p2 > 0.0f) && !(alpha < 1.0f / 255.0f);
                if (GSR_BLEND_STATS) bst.add(__ballot(ok));
                any = first ? ok : (any || ok);
                const float ae = ok ? alpha : 0.f;
                const float rc = __builtin_amdgcn_rcpf(1.f - ae);
                T[k] = T[k] * rc;
                const float dch = ae * T[k];
                // dL/dalpha colour part: sum_c (c_c - A_c) dp_c = (c . dp) - S;  S += alpha (c . dp - S)
                float cd = fmaf(c.z, dp2[k], fmaf(c.y, dp1[k], c.x * dp0[k]));
                if (kDepth) cd = fmaf(c.w, did[k], cd);
                const float dlac = cd - S[k];
                S[k] = fmaf(ae, dlac, S[k]);
                const float dla = GSR_BWD_BG_IN_S ? dlac * T[k] : fmaf(TfB[k], rc, dlac * T[k]);
                // u = G dL/dalpha: the conic / mean terms are opacity * u times (dx, dy) moments,
                // summed here as sum u, sum u dy, sum u dy^2 (dx is the lane's column: applied
                // once per instance below; opacity and the conic after the wave sum)
                const float u = ok ? G * dla : 0.f;
                const float uy = u * dy;
                if constexpr (first) {
                    q[6] = dch * dp0[k];
                    q[7] = dch * dp1[k];
                    q[8] = dch * dp2[k];
                    q[9] = kDepth ? dch * did[k] : 0.f;
                    q[5] = u;
                    q[1] = uy;
                    q[4] = uy * dy;
                } else {
                    q[6] = fmaf(dch, dp0[k], q[6]);
                    q[7] = fmaf(dch, dp1[k], q[7]);
                    q[8] = fmaf(dch, dp2[k], q[8]);
                    if (kDepth) q[9] = fmaf(dch, did[k], q[9]);
                    q[5] += u;
                    q[1] += uy;
                    q[4] = fmaf(uy, dy, q[4]);
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I3 = std::integral_constant<int, 3>;
            using First = std::true_type;
            using Next = std::false_type;
#ifndef GSR_BWD_FULLSWITCH
#define GSR_BWD_FULLSWITCH 0  // measured: 0.2257 -> 0.249 ms (r03j A/B), the larger basic blocks did not pay
#endif
            // scalar branches on the wave-uniform mask: sub-blocks the instance cannot touch are
            // skipped.  GSR_BWD_FULLSWITCH: one case per mask, so all of an instance's active
            // sub-blocks are one basic block and their independent p2 -> exp -> alpha -> rcp -> T
            // chains interleave (nested ifs put every sub-block in a block of its own: each chain's
            // latency was exposed)
            if (GSR_BWD_FULLSWITCH) {
                switch (mk) {
                    case 1: pix(I0{}, First{}); break;
                    case 2: pix(I1{}, First{}); break;
                    case 3: pix(I0{}, First{}); pix(I1{}, Next{}); break;
                    case 4: pix(I2{}, First{}); break;
                    case 5: pix(I0{}, First{}); pix(I2{}, Next{}); break;
                    case 6: pix(I1{}, First{}); pix(I2{}, Next{}); break;
                    case 7: pix(I0{}, First{}); pix(I1{}, Next{}); pix(I2{}, Next{}); break;
                    case 8: pix(I3{}, First{}); break;
                    case 9: pix(I0{}, First{}); pix(I3{}, Next{}); break;
                    case 10: pix(I1{}, First{}); pix(I3{}, Next{}); break;
                    case 11: pix(I0{}, First{}); pix(I1{}, Next{}); pix(I3{}, Next{}); break;
                    case 12: pix(I2{}, First{}); pix(I3{}, Next{}); break;
                    case 13: pix(I0{}, First{}); pix(I2{}, Next{}); pix(I3{}, Next{}); break;
                    case 14: pix(I1{}, First{}); pix(I2{}, Next{}); pix(I3{}, Next{}); break;
                    default: pix(I0{}, First{}); pix(I1{}, Next{}); pix(I2{}, Next{}); pix(I3{}, Next{}); break;
                }
            } else
            switch (__builtin_ctz(mk)) {
                case 0:
                    pix(I0{}, First{});
                    if (mk & 2u) pix(I1{}, Next{});
                    if (mk & 4u) pix(I2{}, Next{});
                    if (mk & 8u) pix(I3{}, Next{});
                    break;
                case 1:
                    pix(I1{}, First{});
                    if (mk & 4u) pix(I2{}, Next{});
                    if (mk & 8u) pix(I3{}, Next{});
                    break;
                case 2:
                    pix(I2{}, First{});
                    if (mk & 8u) pix(I3{}, Next{});
                    break;
                default:
                    pix(I3{}, First{});
                    break;
            }
            // lane moments in dx: q0 = sum u dx, q2 = sum u dx^2, q3 = sum u dx dy (q1 = sum u dy,
            // q4 = sum u dy^2, q5 = sum u)
            q[0] = dx * q[5];
            q[2] = dx * q[0];
            q[3] = dx * q[1];
            return any;
        };
        // Instances in pairs: the two instances' twenty sums share one reduce-scatter (wave_rs20:
        // 23.5 instead of 26 VALU per instance, one LDS park per pair); a lone last instance takes
        // wave_rs10.  The sums' bits are the same either way (same partners, same order).
        uint32_t j = 0;
#ifndef GSR_BWD_PAIRS
#define GSR_BWD_PAIRS 1
#endif
        if (GSR_BWD_PAIRS && GSR_BWD_HALVES) {
            for (; j + 1 < cnt; j += 2) {
                float qa[10], qb[10];
                const bool anya = replay(j, qa);
                const bool anyb = replay(j + 1, qb);
                const float h = __any(anya || anyb) ? wave_rs20(qa, qb, lane) : 0.f;
                if (rs20_slot >= 0) s_red[((j + (rs20_slot >= 10 ? 1u : 0u)) * 2 + (lane >> 5)) * 10 + rs20_slot % 10] = h;
            }
        }
        for (; j < cnt; j++) {
            float q[10];
            const bool any = replay(j, q);
            // reduce-scatter: lane `rs_slot` of rows 1 and 3 parks its half-wave partial; the two
            // halves are added once per batch below instead of per instance
            float h = __any(any) ? wave_rs10(q, lane) : 0.f;
            if (GSR_BWD_HALVES) {
                if ((lane & 16) && rs_slot >= 0) s_red[(j * 2 + (lane >> 5)) * 10 + rs_slot] = h;
            } else {
                // the two halves added here (lanes l and l ^ 32 hold them): one sum per instance
                const auto hs = __builtin_amdgcn_permlane32_swap(__float_as_uint(h), __float_as_uint(h), false, false);
                h = __uint_as_float(hs[0]) + __uint_as_float(hs[1]);
                if (lane < 16 && rs_slot >= 0) s_red[j * 10 + rs_slot] = h;
            }
        }
        __syncthreads();
        float r[10];
        // GSR_BWD_HALVES: the epilogue in slot order (lane < cnt); otherwise in the batch's own lane
        // order (its instance's conic, opacity and id are still in this lane's registers)
        const bool ep = GSR_BWD_HALVES ? (uint32_t)lane < cnt : m != 0u;
        const uint32_t es = GSR_BWD_HALVES ? (uint32_t)lane : slot;
        if (ep) {
            if (GSR_BWD_HALVES) {
                const float2 *d = reinterpret_cast<const float2 *>(s_red) + es * 10;
#pragma unroll
                for (int t = 0; t < 5; t++) {
                    const float2 p0 = d[t], p1 = d[5 + t];
                    r[2 * t] = p0.x + p1.x;
                    r[2 * t + 1] = p0.y + p1.y;
                }
            } else {
                const float2 *d = reinterpret_cast<const float2 *>(s_red) + es * 5;
#pragma unroll
                for (int t = 0; t < 5; t++) {
                    const float2 p = d[t];
                    r[2 * t] = p.x;
                    r[2 * t + 1] = p.y;
                }
            }
            const size_t o = 4 * (size_t)(GSR_BWD_HALVES ? __float_as_uint(s_b[es].w) : u);
            {
                // moments -> (dmean2D, dconic): dL/dG = opacity dL/dalpha, dG/d(dx) = -G (a dx + b dy), ...
                const float4 id = GSR_BWD_HALVES ? s_d[es] : make_float4(qa.z, qa.w, qb.x, 0.f);
                const float op = GSR_BWD_HALVES ? s_b[es].y : qb.y, ca = id.x, cb = id.y, cc = id.z;
                const float m0 = r[0], m1 = r[1], mxx = r[2], mxy = r[3], myy = r[4];
                r[0] = -op * fmaf(cb, m1, ca * m0);
                r[1] = -op * fmaf(cb, m0, cc * m1);
                r[2] = op * mxx;
                r[3] = op * mxy;
                r[4] = op * myy;
            }
            r[0] *= sx;
            r[1] *= sy;
            r[2] *= -0.5f;
            r[3] *= -0.5f;
            r[4] *= -0.5f;
            // the Gaussian is live for preprocess_bwd (its sums may still be zero: harmless)
            if (kAtomic && zr.stamps) zr.stamps[o / 4] = zr.stamp;
            if (!kAtomic) {
                out[o + 0] = make_float4(r[0], r[1], r[2], r[3]);
                out[o + 1] = make_float4(r[4], r[5], r[6], r[7]);
                out[o + 2] = make_float4(r[8], r[9], 0.f, 0.f);
                if (GSR_REC_PAD) out[o + 3] = make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
        if (kAtomic) {
            // the batch's sums, instance-major, through LDS (s_red is free again: every lane has
            // read its halves), then ten atomic instructions: lane l of round k adds value
            // (64k + l) % 10 of instance (64k + l) / 10 -- consecutive lanes, consecutive floats
            // of one Gaussian's row
            if (GSR_BWD_HALVES) __syncthreads();  // otherwise each lane rewrites the slot it read
            float *st = s_red;
            if (ep) {
#pragma unroll
                for (int t = 0; t < 10; t++) st[es * 10 + t] = r[t];
            }
            __syncthreads();
#pragma unroll 1
            for (uint32_t pidx = (uint32_t)lane; pidx < 10u * cnt; pidx += (uint32_t)kWave) {
                const uint32_t j = pidx / 10u, v = pidx - 10u * j;
                const float val = st[pidx];
                const uint32_t g = __float_as_uint(s_b[j].w);
                if (val != 0.f) unsafeAtomicAdd(reinterpret_cast<float *>(out + 4 * (size_t)g) + v, val);
            }
        }
        __syncthreads();
    }
    bwd_zero_slice(zr);
    if (GSR_BLEND_STATS) {
        bst.flush(kBwdPairs);
        if (lane == 0) {
            atomicAdd(&g_blend_stats[kBwdInst], (unsigned long long)b_inst);
            atomicAdd(&g_blend_stats[kBwdBatches], (unsigned long long)b_batches);
            atomicAdd(&g_blend_stats[kBwdTiles], 1ull);
        }
    }
}

bool fwd_segments_supported() { return GSR_FWD_SUB == 1 && !GSR_FWD_SB_ORDER; }
bool fwd_segments_in_kernel() { return GSR_FWD_SEG_INKERNEL != 0; }

bool bwd_segments_supported() { return GSR_BWD_CLS && GSR_FWD_SUB == 1 && GSR_BWD_BG_IN_S && !GSR_TILE_REVERSE; }

void launch_render_bwd(const Camera &cam, const GeomState &gs, const BinningState &bs, const ImageState &is,
                       const int *radii, const float *bg, const float *dL_dpix, const float *dL_dinvdepth,
                       const BwdScratch &sc, hipStream_t s, const ZeroRows *zr, uint32_t seg_len) {
    (void)radii;
    const int T = cam.gx * cam.gy;
    if (T == 0) return;
    const ZeroRows z = zr ? *zr : ZeroRows{};
    const float *ck = nullptr;
    const uint32_t *items = nullptr;
    if (seg_len) {
        ck = reinterpret_cast<const float *>(reinterpret_cast<const char *>(bs.point_list) + ck_offset(bs.cap));
        items = reinterpret_cast<const uint32_t *>(ck + ck_slots(bs.cap, seg_len) * (kCkFloats * 256));
    }
    const unsigned grid = (unsigned)bwd_grid(T, bs.cap, seg_len);
#define GSR_BWD_LAUNCH(D, A)                                                                                       \
    hipLaunchKernelGGL((render_bwd_kernel<D, A>), dim3(grid), dim3(kWave), 0, s, is.ranges, bs.point_list, cam.W,   \
                       cam.H, cam.gx, gs.rec, bg, is.final_T, is.n_contrib, dL_dpix, dL_dinvdepth, is.tile_order,    \
                       gs.offsets, is.boundary, A ? sc.acc : sc.rec, z, is.bwd_cnt, is.bwd_cls, (uint32_t)T, seg_len, \
                       ck, items)
    if (dL_dinvdepth) {
        if (sc.atomic) GSR_BWD_LAUNCH(true, true);
        else GSR_BWD_LAUNCH(true, false);
    } else {
        if (sc.atomic) GSR_BWD_LAUNCH(false, true);
        else GSR_BWD_LAUNCH(false, false);
    }
#undef GSR_BWD_LAUNCH
}

GSR_KSTAMP_READER(kstamp_read_render)

}  // namespace gsr

extern "C" int gsr_blend_stats(int64_t *out, int n, int reset) {
    unsigned long long v[16] = {};
    if (!out || n < 0) return -1;
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(gsr::g_blend_stats), sizeof(v)) != hipSuccess) return -3;
    if (reset) {
        const unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_blend_stats), z, sizeof(z)) != hipSuccess) return -3;
    }
    int k = 0;
    for (; k < n && k < 16; k++) out[k] = (int64_t)v[k];
    return k;
}

extern "C" int gsr_fwd_pool_stats(int64_t *out, int n, int reset) {
    unsigned long long v[4] = {};
    if (!out || n < 0) return -1;
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(gsr::g_fwd_pool_ticks), sizeof(v)) != hipSuccess) return -3;
    if (reset) {
        const unsigned long long z[4] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_fwd_pool_ticks), z, sizeof(z)) != hipSuccess) return -3;
    }
    int k = 0;
    for (; k < n && k < 4; k++) out[k] = (int64_t)v[k];
    return k;
}
