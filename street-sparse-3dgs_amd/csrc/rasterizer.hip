// rasterizer.hip -- the C ABI (include/gsr.h): buffer carving, stage orchestration, the one
// device->host read of K (num_rendered), debug checking and per-stage HIP-event timing.
//
// Flow per frame:  preprocess -> depth sort (histograms + tile scan ->
// [K to the host] -> 4 radix passes, the last one gathering the depth-ordered tile rects) ->
// two-level binning (tile lists + ranges) -> render fwd;
// backward: render bwd (per-instance records) -> preprocess bwd (per-Gaussian sum + chain).
#include <cstdio>
#include <cstring>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <algorithm>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/gsr.h"
#include "../../include/gsr_hier.h"
#include "gsr_launch.h"

using namespace gsr;

namespace gsr {
// compute units of the current device (cached per device)
int device_cus() {
    static int cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cache[dev]) {
        int n = 0;
        cache[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
    }
    return cache[dev];
}
}  // namespace gsr

namespace {

thread_local std::string g_err;
// K (num_rendered) arrives in pinned, host-coherent memory written by the depth sort's first
// kernel; the host waits on an event recorded right after it, so the sort passes keep running
// while the host sizes the binning buffer.
// g_pinned[kHostK] = K, [kHostErr] = sticky depth-sort error (a lookback spin gave up; never
// expected), [kHostMaxSB] / [kHostP1] = a local-sort frame's longest SB list / level-1 total
thread_local uint32_t *g_pinned = nullptr;
thread_local uint32_t *g_pinned_dev = nullptr;
// forward statistics (gsr_forward_stats): frames, binning re-runs at K (capacity hint short)
std::atomic<int64_t> g_frames{0}, g_reruns{0}, g_local_frames{0}, g_fallbacks{0};
// binning mode (gsr_set_binning): 0 = local sort where it applies, 1 = always the global depth sort.
// Default 1: on the 1M-Gaussian 1080p bench frame the local path measured 2801 Mpix/s against
// 2909 (its level-1 kernels and the LDS sort share the chip with the SH colour pass, which the
// global sort leaves half of the CUs to)
#ifndef GSR_BINNING_DEFAULT
#define GSR_BINNING_DEFAULT 1
#endif
std::atomic<int> g_binning_mode{GSR_BINNING_DEFAULT};
// the native train step's sparse gradient rows (gsr_launch.h GaussianGrads), per calling thread
thread_local bool g_sparse_grad_rows = false;
thread_local bool g_raw_params = false;  // GaussianInputs.raw, per calling thread
thread_local gsr::StepAct g_step_act{};    // set_step_act
std::atomic<int> g_live_list{0};           // gsr_set_live_list
thread_local bool g_step_act_done = false;
constexpr int kMaxDevicesK = 64;
// The backward's per-Gaussian accumulator rows (64 B each: render_bwd's ten float-atomic sums),
// GSR_PERSISTENT_ACC (default): one grow-only array per device, all zero between backwards --
// render_bwd adds into the rows of the Gaussians it reaches and the consumer (preprocess_bwd or
// the live-row pass) zeroes every row it reads (it always did, for a repeated backward), so the
// forward no longer clears P rows per frame (1M x 64 B on the bench frame: 10 us of the step,
// r06r).  A backward that fails between render_bwd and the consumer leaves the rows marked dirty
// (cleared by the next backward); a backward on another stream than the previous one first waits
// for that stream.  GSR_PERSISTENT_ACC=0: the rows in the frame's geometry buffer, cleared by
// render_fwd (rounds 1-5).
#ifndef GSR_PERSISTENT_ACC
#define GSR_PERSISTENT_ACC 1
#endif
struct AccRows {
    float4 *p = nullptr;
    size_t rows = 0;
    bool dirty = false;
    hipStream_t last = nullptr;  // the stream of the last backward that used the rows
};
std::mutex g_acc_mu;
AccRows g_acc_rows[kMaxDevicesK];
// The device's rows for a backward of n rows on stream s (stream-ordered growth and clears); marked
// dirty until acc_rows_consumed() -- the backward has queued the consumer.  NULL on failure.
float4 *acc_rows(hipStream_t s, size_t n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevicesK) return nullptr;
    std::lock_guard<std::mutex> lk(g_acc_mu);
    AccRows &a = g_acc_rows[dev];
    // another stream's backward may still be adding into / consuming the rows (a stream may since
    // have been destroyed, so the whole device is waited for; backwards on one stream need nothing)
    if (a.last && a.last != s && hipDeviceSynchronize() != hipSuccess) return nullptr;
    const size_t row = 4 * sizeof(float4);
    if (a.rows < n) {
        const size_t want = std::max(n, a.rows + a.rows / 4);
        float4 *p = nullptr;
        if (hipMallocAsync(reinterpret_cast<void **>(&p), want * row, s) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        if (hipMemsetAsync(p, 0, want * row, s) != hipSuccess) return nullptr;
        if (a.p) (void)hipFreeAsync(a.p, s);  // after the work queued before on this stream
        a.p = p;
        a.rows = want;
    } else if (a.dirty && hipMemsetAsync(a.p, 0, a.rows * row, s) != hipSuccess) {
        return nullptr;
    }
    a.dirty = true;
    a.last = s;
    return a.p;
}
void acc_rows_consumed() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevicesK) return;
    std::lock_guard<std::mutex> lk(g_acc_mu);
    g_acc_rows[dev].dirty = false;
}
thread_local hipEvent_t g_k_ready[kMaxDevicesK] = {};
// per device: capacity for the next frame's point list, 0 = none yet.  It is the largest K of the
// last kKHist (256) frames + 1/8 + 4096, so a training loop cycling its cameras (whose K differs from
// view to view) rarely comes up short and re-runs the binning (gsr_forward_stats counts re-runs).
constexpr int kKHist = 256;
thread_local int64_t g_khint[kMaxDevicesK] = {};
thread_local int64_t g_khist[kMaxDevicesK][kKHist] = {};
thread_local int g_khead[kMaxDevicesK] = {};
#ifndef GSR_DEFER_K
#define GSR_DEFER_K 1
#endif
constexpr uint32_t kKPending = 0xFFFFFFFFu;
// The split gate (gsr_set_split_gate): the forward split and the tile_bin split cost launches and
// stream hand-offs on every frame they are armed for, and pay only on frames with very long lists
// (a street view after an opacity reset), so they are armed for kSplitMemory frames after a frame
// (per device and thread) whose longest tile / superblock list called for them -- the kernels report
// those lengths in pinned memory, read at the next forward.
constexpr int64_t kSplitMemory = 256;
thread_local int64_t g_frame_no[kMaxDevicesK] = {};
thread_local int64_t g_long_tile_at[kMaxDevicesK] = {};
thread_local int64_t g_long_sb_at[kMaxDevicesK] = {};
std::atomic<int> g_split_gate{1};

// Stage profiling is process-wide: torch runs the backward on its autograd device thread.
constexpr int kStages = 10;
std::mutex g_prof_mu;
int g_profile = 0;
bool g_ev_init = false;
hipEvent_t g_ev_begin[kStages], g_ev_end[kStages];
bool g_ev_recorded[kStages];

// Side stream for work that overlaps the main stream's latency-bound stages (the SH colour
// pass runs beside the depth sort and the binning); fork / join with events, so it also works
// inside a captured HIP graph.  One per device, created on first use.
constexpr int kMaxDevices = 64;
std::mutex g_side_mu;
constexpr int kSides = 2;  // 0: the colour pass and the forward segments' workers; 1: the tile_bin split
hipStream_t g_side[kSides][kMaxDevices] = {};
hipEvent_t g_fork[kSides][kMaxDevices] = {}, g_join[kSides][kMaxDevices] = {};

#ifndef GSR_SIDE_STREAM
#define GSR_SIDE_STREAM 1
#endif
#ifndef GSR_COLOR_SERIAL
#define GSR_COLOR_SERIAL 0  // 1: SH colour pass on the main stream after the preprocess (measured: no faster)
#endif
#ifndef GSR_K_POLL
#define GSR_K_POLL 1  // deferred K read by polling the pinned word (0: an event after the upsweep)
#endif
bool side_stream(hipStream_t main, hipStream_t *side, hipEvent_t *fork, hipEvent_t *join, int which = 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return false;
    std::lock_guard<std::mutex> lk(g_side_mu);
    if (!g_side[which][dev]) {
        if (hipStreamCreateWithFlags(&g_side[which][dev], hipStreamNonBlocking) != hipSuccess) return false;
        if (hipEventCreateWithFlags(&g_fork[which][dev], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g_join[which][dev], hipEventDisableTiming) != hipSuccess)
            return false;
    }
    *side = GSR_SIDE_STREAM ? g_side[which][dev] : main;  // 0: the colour pass serialises (timing experiments)
    *fork = g_fork[which][dev];
    *join = g_join[which][dev];
    return true;
}

// tile_bin split of long superblock lists: the list length past which an SB is sliced, GSR_TB_SPLIT
// or the environment's GSR_TB_SPLIT (measurement A/B; 0 = off)
uint32_t tb_split_len() {
    static const uint32_t len = [] {
        const char *e = getenv("GSR_TB_SPLIT");
        return e ? (uint32_t)std::max(0, atoi(e)) : (uint32_t)GSR_TB_SPLIT;
    }();
    return len;
}

// Joins the side stream into the main one when the forward leaves early (errors), so the
// caller's buffers are never released under side-stream work.
struct SideJoin {
    hipStream_t s = nullptr;
    hipEvent_t join = nullptr;
    bool pending = false;
    ~SideJoin() {
        if (pending) (void)hipStreamWaitEvent(s, join, 0);
    }
};


// Frames whose depth sort fills every CU (P above ~1M): the SH colour pass forks right after the
// preprocess at full width instead of after the sort (GSR_COLOR_EARLY_BIG=0 for the A/B).
// Measured on config 5 (7.46M rows, GSR_COLOR_FORK=0 variant, r05e): 3.73 -> 3.63 ms per frame.
bool color_early_big() {
    static const bool v = [] {
        const char *e = std::getenv("GSR_COLOR_EARLY_BIG");
        return !(e && e[0] == '0');
    }();
    return v;
}
// The same frames' colour pass as a persistent grid of this many blocks (GSR_COLOR_BIG_BLOCKS; 0 = a
// full grid of 4-wave blocks), for the A/B of config 3's 20-30 ms stalls (a depth-sort or binning
// kernel and the full-grid colour pass both stretched to the same end, r05f spikes.json)
// A full-grid colour pass forked after the sort: 8-wave blocks (0, default) or 4-wave blocks
// (GSR_COLOR_LATE_WAVES=4, -1; launch_preprocess_color).  Config 3 (r05h): 8 waves 55.8 s, 4 waves
// 56.3 s -- the colour pass itself 0.224 -> 0.139 ms, but beside it bin_superblocks 0.153 -> 0.186 ms.
int color_late_grid() {
    static const int v = [] {
        const char *e = std::getenv("GSR_COLOR_LATE_WAVES");
        return e && std::atoi(e) == 4 ? -1 : 0;
    }();
    return v;
}
int color_big_blocks() {
    static const int v = [] {
        const char *e = std::getenv("GSR_COLOR_BIG_BLOCKS");
        return e ? std::max(0, std::atoi(e)) : 0;
    }();
    return v;
}

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

// A lookback timeout of this or an earlier frame's depth sort (the pass kernels store the pinned
// word; its frame's render_fwd already wrote NaN pixels): fail this call, once per occurrence.
// kHostFwdErr: a forward worker's predecessor wait timed out (that tile's pixels are NaN).  Forward
// workers that gave up on tile_order's ready word are counted instead (kHostFwdGiveUp, frames with
// give-ups; their items were blended by the pool's second launch, the frame is exact).
// g_kwait_ns: host time spent waiting for K (num_rendered) in the forward, summed (gsr_forward_stats[5]).
std::atomic<int64_t> g_fwd_giveups{0}, g_kwait_ns{0};
// frames whose forward ran with the forward split / the tile binning's superblock split armed
std::atomic<int64_t> g_fsplit_frames{0}, g_tbsplit_frames{0};
constexpr int kFwdStats = 8;
void collect_giveups() {
    if (!g_pinned) return;
    const uint32_t gu = __atomic_exchange_n(&g_pinned[kHostFwdGiveUp], 0u, __ATOMIC_SEQ_CST);
    if (gu && g_fwd_giveups.fetch_add(1) == 0)
        fprintf(stderr, "[gsr] forward split: workers gave up waiting for tile_order (side and main streams not "
                        "concurrent); the frame was completed by the pool's second launch, slower "
                        "(gsr_forward_stats[4] counts such frames)\n");
}
int sticky_sort_error() {
    if (!g_pinned) return GSR_OK;
    collect_giveups();
    const uint32_t e = __atomic_exchange_n(&g_pinned[kHostErr], 0u, __ATOMIC_SEQ_CST);
    const uint32_t fe = __atomic_exchange_n(&g_pinned[kHostFwdErr], 0u, __ATOMIC_SEQ_CST);
    if (e) return fail(GSR_ERR_DEVICE, "depth sort: a lookback spin timed out (this or an earlier frame; its image is NaN)");
    if (fe)
        return fail(GSR_ERR_DEVICE, "forward split: a worker's wait for a predecessor segment timed out (this or an "
                                    "earlier frame; the tile's pixels are NaN)");
    return GSR_OK;
}

void ensure_events() {
    if (g_ev_init) return;
    for (int k = 0; k < kStages; k++) {
        (void)hipEventCreate(&g_ev_begin[k]);
        (void)hipEventCreate(&g_ev_end[k]);
        g_ev_recorded[k] = false;
    }
    g_ev_init = true;
}

// Measurement builds only (-DGSR_HOST_TRACE=1, a variant library): the host time spent issuing each
// stage (StageTimer's scope) and whole forward / backward calls, read with gsr_debug_trace:
// out[0..11] = nanoseconds (stages 0-9, forward call, backward call), out[12..23] = counts.
#ifndef GSR_HOST_TRACE
#define GSR_HOST_TRACE 0
#endif
constexpr int kHostTrace = 12;
std::atomic<int64_t> g_htrace_ns[kHostTrace], g_htrace_cnt[kHostTrace];
struct HostScope {
    int k;
    std::chrono::steady_clock::time_point t0;
    explicit HostScope(int slot) : k(slot) {
        if (GSR_HOST_TRACE) t0 = std::chrono::steady_clock::now();
    }
    ~HostScope() {
        if (!GSR_HOST_TRACE) return;
        g_htrace_ns[k].fetch_add(
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
        g_htrace_cnt[k].fetch_add(1);
    }
};

// Brackets exactly the device work of one stage (no host gaps inside the bracket).
struct StageTimer {
    int k;
    hipStream_t s;
    bool on;
    HostScope hs;
    StageTimer(int stage, hipStream_t stream) : k(stage), s(stream), on(g_profile != 0), hs(stage) {
        if (on) (void)hipEventRecord(g_ev_begin[k], s);
    }
    ~StageTimer() {
        if (on) {
            (void)hipEventRecord(g_ev_end[k], s);
            g_ev_recorded[k] = true;
        }
    }
};

int check(const char *stage, int debug, hipStream_t s) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && debug) {
        e = hipStreamSynchronize(s);
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (e != hipSuccess) return fail(GSR_ERR_DEVICE, std::string(stage) + ": " + hipGetErrorString(e));
    return GSR_OK;
}

struct Carver {
    char *base;
    size_t off = 0;
    explicit Carver(void *b) : base(static_cast<char *>(b)) {}
    template <class T>
    T *take(size_t n) {
        off = align_up(off, 256);
        T *p = base ? reinterpret_cast<T *>(base + off) : nullptr;
        off += n * sizeof(T);
        return p;
    }
};

GeomState carve_geom(void *base, int P, int gx, int gy, size_t *bytes) {
    Carver c(base);
    GeomState g;
    g.rec = c.take<GRec>(P);
    g.tiles = c.take<uint32_t>(P);
    g.dkey = c.take<uint32_t>(P);
    g.dkey_sorted = c.take<uint32_t>(P);
    g.ids = c.take<uint32_t>(P);
    g.order = c.take<uint32_t>(P);
    g.offsets = c.take<uint32_t>(P);
    g.clamped = c.take<uint8_t>(P);
    g.ctrl_zero = (uint32_t)dsort_ctrl_zero_words(P);
    g.ctrl = c.take<uint32_t>(dsort_ctrl_words(P));
    g.drect = c.take<uint2>(P);
    g.rect8 = c.take<uint2>(P);
    g.rect4 = c.take<uint32_t>(P);
    if (!GSR_RECT4 || gx > 255 || gy > 255) g.rect4 = nullptr;
    g.sb = sb_grid(gx, gy, P);
    g.sb_cnt_g = c.take<uint32_t>((size_t)g.sb.nsb * g.sb.ccols);
    g.sb_cnt_i = c.take<uint32_t>((size_t)g.sb.nsb * g.sb.ccols);
    g.sb_base_g = c.take<uint32_t>((size_t)g.sb.nsb + 1);
    g.sb_base_i = c.take<uint32_t>((size_t)g.sb.nsb + 1);
    // GSR_PERSISTENT_ACC: the backward's accumulator rows are the device's persistent rows
    // (acc_rows below), not part of the frame's buffer
    g.acc = GSR_PERSISTENT_ACC ? nullptr : c.take<float4>(4 * (size_t)P);
    g.nacc = GSR_PERSISTENT_ACC ? 0 : P;
    g.live_stamp = c.take<uint32_t>(P);
    g.tb_flag = c.take<uint32_t>((size_t)g.sb.nsb + 1);
    g.tb_items = c.take<uint32_t>(kTBMaxItems);
    g.tb_cnt = c.take<uint32_t>((size_t)kTBMaxItems << (2 * g.sb.shift));
    if (bytes) *bytes = align_up(c.off, 256);
    return g;
}

// point_list first: the backward re-carves this buffer with num_rendered, which may be smaller
// than the capacity the forward carved it with.
// End of the backward checkpoints (L) and the forward items (Lf) past the start of the binning
// buffer (they use the level-1 lists' room past the point list).
size_t segment_end(int64_t K, uint32_t L, uint32_t Lf) {
    size_t end = ck_offset(K);
    if (L) end += align256(ck_slots(K, L) * (kCkFloats * 256) * 4 + ck_slots(K, L) * 4);
    if (Lf) {
        const FwdSegLayout f = fseg_layout(nullptr, K, L, Lf);
        end = (size_t)reinterpret_cast<uintptr_t>(f.part) + fseg_max_items(K, Lf) * kFwdPartials * 256 * 4;
    }
    return end;
}

// L / Lf: the frame's segment lengths -- the buffer reaches past the level-1 lists when their
// regions need it (L = 512 with Lf = 1024: 28 B per instance against the lists' 20 B)
BinningState carve_binning(void *base, int64_t K, size_t *bytes, uint32_t L = 0, uint32_t Lf = 0) {
    Carver c(base);
    BinningState b;
    b.point_list = c.take<uint32_t>(K);
    // level-1 entries: 8 B (id, footprint) on the global-sort path, 16 B (id, footprint, depth key,
    // -) on the local-sort path -- carved for the larger
    b.sblist4 = c.take<uint4>(K);
    b.sblist = reinterpret_cast<uint2 *>(b.sblist4);
    const size_t end = (L || Lf) ? segment_end(K, L, Lf) : 0;
    if (end > c.off) (void)c.take<uint8_t>(end - c.off);
    (void)c.take<uint8_t>(kSegReserve);
    b.cap = (uint32_t)K;
    b.kdev = nullptr;
    if (bytes) *bytes = align_up(c.off, 256);
    return b;
}

ImageState carve_image(void *base, int T, int npix, size_t *bytes) {
    Carver c(base);
    ImageState s;
    s.ranges = c.take<uint2>(T);
    s.boundary = c.take<uint64_t>(T);
    s.final_T = c.take<float>(npix);
    s.n_contrib = c.take<uint32_t>(npix);
    s.tile_work = c.take<uint32_t>(T);
    s.tile_ids = c.take<uint32_t>(T);
    s.tile_order = c.take<uint32_t>(T);
    s.bwd_cnt = c.take<uint32_t>(kBwdClasses + 64);  // + the segment count (kBwdSegCount)
    s.bwd_cls = c.take<uint32_t>((size_t)kBwdClasses * T);
    if (bytes) *bytes = align_up(c.off, 256);
    return s;
}

// atomic mode needs no scratch (the accumulators live in the geometry buffer, GeomState.acc)
BwdScratch carve_bwd(void *base, int64_t K, int P, bool atomic, size_t *bytes, bool list) {
    Carver c(base);
    BwdScratch s{};
    s.atomic = atomic ? 1 : 0;
    if (!atomic) {
        s.rec = c.take<float4>(4 * (size_t)K);
        s.gsum = c.take<float4>(2 * (size_t)P);
    }
    s.live = c.take<uint64_t>(((size_t)P + 63) / 64);
    if (list) s.list = c.take<uint32_t>((size_t)P);  // the backward's live-row list (gsr_set_live_list)
    if (bytes) *bytes = align_up(c.off, 256);
    return s;
}

// Rows blended from the hierarchy cut when render_indices is non-empty (gsr.h): carved after the
// geometry state, read back by the backward from the same buffer.
struct CutRows {
    float *means, *scales, *rots, *opac, *shs;
};

CutRows carve_cut(Carver &c, int R, int M) {
    CutRows r;
    r.means = c.take<float>(3 * (size_t)R);
    r.scales = c.take<float>(3 * (size_t)R);
    r.rots = c.take<float>(4 * (size_t)R);
    r.opac = c.take<float>((size_t)R);
    r.shs = c.take<float>(3 * (size_t)M * R);
    return r;
}

size_t geom_bytes(int P, int gx, int gy, int R, int M) {
    size_t b = 0;
    carve_geom(nullptr, P, gx, gy, &b);
    if (R > 0) {
        Carver c(nullptr);
        c.off = b;
        carve_cut(c, R, M);
        b = align_up(c.off, 256);
    }
    return b;
}

CutRows cut_rows_of(void *geom, int P, int gx, int gy, int M) {
    size_t b = 0;
    carve_geom(nullptr, P, gx, gy, &b);
    Carver c(geom);
    c.off = b;
    return carve_cut(c, P, M);
}

int validate_cut(int R, int64_t N, const float *shs, const float *scales, const float *rotations,
                 const int *render_indices, const int *parent_indices, const float *interpolation_weights) {
    if (R < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "num_render must be >= 0");
    if (R == 0) return GSR_OK;
    if (!shs || !scales || !rotations)
        return fail(GSR_ERR_UNSUPPORTED,
                    "render_indices needs shs, scales and rotations (render_post's blend is defined for them only)");
    if (!render_indices || !parent_indices || !interpolation_weights)
        return fail(GSR_ERR_INVALID_ARGUMENT, "render_indices given without parent_indices / interpolation_weights");
    if (N <= 0) return fail(GSR_ERR_INVALID_ARGUMENT, "render_indices given with no Gaussians");
    for (const void *p : {(const void *)render_indices, (const void *)parent_indices,
                          (const void *)interpolation_weights}) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeDevice)
            return fail(GSR_ERR_INVALID_ARGUMENT, "render_indices / parent_indices / interpolation_weights must be "
                                                  "device memory when non-empty");
    }
    return GSR_OK;
}

Camera make_camera(const float *view, const float *proj, const float *campos, float tanx, float tany, int W, int H) {
    Camera c;
    c.view = view;
    c.proj = proj;
    c.campos = campos;
    c.tanx = tanx;
    c.tany = tany;
    // rasterizer_impl: focal = size / (2 * tan(fov/2)), evaluated in fp32
    c.fy = (float)H / (2.0f * tany);
    c.fx = (float)W / (2.0f * tanx);
    c.W = W;
    c.H = H;
    c.gx = (W + kTile - 1) / kTile;
    c.gy = (H + kTile - 1) / kTile;
    return c;
}

int validate_common(int P, int D, int M, const float *shs, const float *colors_precomp, const float *scales,
                    const float *rotations, const float *cov3D_precomp, int W, int H) {
    if (P < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "P must be >= 0");
    if (W <= 0 || H <= 0) return fail(GSR_ERR_INVALID_ARGUMENT, "image size must be positive");
    if ((shs == nullptr) == (colors_precomp == nullptr) && P > 0)
        return fail(GSR_ERR_INVALID_ARGUMENT, "Please provide exactly one of either SHs or precomputed colors!");
    if (((scales == nullptr || rotations == nullptr) && cov3D_precomp == nullptr) ||
        ((scales != nullptr || rotations != nullptr) && cov3D_precomp != nullptr)) {
        if (P > 0)
            return fail(GSR_ERR_INVALID_ARGUMENT,
                        "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    }
    if (shs && (D < 0 || D > 3 || (D + 1) * (D + 1) > M || M > 16))
        return fail(GSR_ERR_INVALID_ARGUMENT, "sh degree / coefficient count out of range (need (D+1)^2 <= M <= 16)");
    return GSR_OK;
}

}  // namespace

void gsr::set_last_error(const std::string &msg) { g_err = msg; }

namespace {
std::atomic<int> g_true_scale_grad{0};
#ifndef GSR_DETERMINISTIC_DEFAULT
#define GSR_DETERMINISTIC_DEFAULT 0  // backward accumulation: 0 float atomics, 1 records + ordered sums
#endif
std::atomic<int> g_deterministic{GSR_DETERMINISTIC_DEFAULT};
}
bool gsr::true_scale_gradient() { return g_true_scale_grad.load(std::memory_order_relaxed) != 0; }
void gsr::set_sparse_grad_rows(bool on) { g_sparse_grad_rows = on; }
void gsr::set_raw_params(bool on) { g_raw_params = on; }
void gsr::set_step_act(const StepAct *a) { g_step_act = a ? *a : StepAct{}; }
bool gsr::live_list() { return g_live_list.load(std::memory_order_relaxed) != 0; }
gsr::StepAct gsr::step_act() { return g_step_act; }
void gsr::note_step_act_done(bool done) { g_step_act_done = done; }
bool gsr::step_act_done() { return g_step_act_done; }

namespace {
// Geometry buffers whose accumulator rows the forward did not clear: forwards made with
// GSR_FWD_NO_BACKWARD (a backward handed one fails loudly) and forwards made in deterministic
// mode (their backward uses the record path even if the mode was switched in between).  Every
// forward first removes its own buffer, so an address the caching allocator hands out again is
// judged by the forward that carved it last.  Bounded: past kUnclearedMax entries the map is
// cleared (those forwards lose the check; their buffers are normally long released by then).
enum Uncleared : uint8_t { kNoBackward = 1, kDeterministicFwd = 2 };
std::mutex g_unclr_mu;
std::unordered_map<const void *, uint8_t> g_unclr;
constexpr size_t kUnclearedMax = 4096;
void note_forward_geom(const void *geom, bool need_bwd, bool cleared) {
    std::lock_guard<std::mutex> lk(g_unclr_mu);
    if (cleared) {
        if (!g_unclr.empty()) g_unclr.erase(geom);
        return;
    }
    if (g_unclr.size() >= kUnclearedMax) g_unclr.clear();
    g_unclr[geom] = need_bwd ? kDeterministicFwd : kNoBackward;
}
uint8_t forward_uncleared(const void *geom) {
    std::lock_guard<std::mutex> lk(g_unclr_mu);
    if (g_unclr.empty()) return 0;
    const auto it = g_unclr.find(geom);
    return it == g_unclr.end() ? 0 : it->second;
}

// Backward segments (gsr_set_bwd_segment): the segment length a forward published its backward
// items with, per image buffer (the backward must cut tiles the same way).  Same bookkeeping as
// g_unclr: a forward made without segments erases its buffer's entry; bounded by kUnclearedMax (a
// backward whose entry was dropped takes the current setting).
#ifndef GSR_BWD_SEG_DEFAULT
#define GSR_BWD_SEG_DEFAULT 512  // measured: bench render_bwd 0.2463 -> 0.2344 ms, config-3 chunk 106.2 -> 67.3 s (r04h, r04i)
#endif
std::atomic<uint32_t> g_bwd_seg{GSR_BWD_SEG_DEFAULT};
#ifndef GSR_FWD_SEG_DEFAULT
#define GSR_FWD_SEG_DEFAULT 2048  // behind the split gate; config 3 (r05j/r05k): 4096 55.8-56.0 s, 2048 53.9 s, 1024 54.2-54.8 s
#endif
std::atomic<uint32_t> g_fwd_seg{GSR_FWD_SEG_DEFAULT};
std::mutex g_seg_mu;
std::unordered_map<const void *, uint32_t> g_seg_of;
// A forward made without segments (L = 0: switched off, or the 32-bit item-numbering guard) is
// recorded as 0 too -- its backward must not cut tiles at the current setting and read checkpoints
// render_fwd never wrote.  Only an entry dropped by the kUnclearedMax clear falls back to the setting.
void note_forward_seg(const void *image, uint32_t L) {
    std::lock_guard<std::mutex> lk(g_seg_mu);
    if (g_seg_of.size() >= kUnclearedMax) g_seg_of.clear();
    g_seg_of[image] = L;
}
uint32_t forward_seg(const void *image) {
    std::lock_guard<std::mutex> lk(g_seg_mu);
    const auto it = g_seg_of.find(image);
    return it == g_seg_of.end() ? g_bwd_seg.load(std::memory_order_relaxed) : it->second;
}
}  // namespace

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }

const char *gsr_last_error(void) { return g_err.c_str(); }

const char *gsr_build_info(void) {
    return "gsr_hip gfx950: preprocess (preprocess.hip), onesweep depth sort with fused tile scan / gather "
           "(dsort.hip), two-level counting binning (binning.hip), sub-block render fwd / wave-per-tile render bwd "
           "with DPP reductions (render.hip), per-Gaussian backward (backward.hip)";
}

int gsr_set_profiling(int enable) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (enable) ensure_events();
    for (int k = 0; k < kStages; k++) g_ev_recorded[k] = false;
    g_profile = enable ? 1 : 0;
    return GSR_OK;
}

int gsr_stage_times_ms(float *out, int max_stages) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    if (!g_ev_init) return 0;
    int n = 0;
    for (; n < kStages && n < max_stages; n++) {
        float ms = 0.f;
        if (g_ev_recorded[n] && hipEventSynchronize(g_ev_end[n]) == hipSuccess &&
            hipEventElapsedTime(&ms, g_ev_begin[n], g_ev_end[n]) == hipSuccess)
            out[n] = ms;
        else
            out[n] = 0.f;
    }
    return n;
}

int gsr_rasterize_forward(gsr_resize_fn geom_buffer, gsr_resize_fn binning_buffer, gsr_resize_fn image_buffer,
                          void *resize_ctx, int P, int D, int M, const float *background, int width, int height,
                          const float *means3D, const float *shs, const float *colors_precomp,
                          const float *opacities, const float *scales, float scale_modifier,
                          const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                          const float *projmatrix, const float *cam_pos, float tan_fovx, float tan_fovy,
                          int prefiltered, float *out_color, float *out_invdepth, int *radii,
                          const int *render_indices, const int *parent_indices,
                          const float *interpolation_weights, const int *num_node_kids, int num_render,
                          int debug, void *stream, int64_t *num_rendered) {
    return gsr_rasterize_forward_ex(geom_buffer, binning_buffer, image_buffer, resize_ctx, P, D, M, background, width,
                                    height, means3D, shs, colors_precomp, opacities, scales, scale_modifier, rotations,
                                    cov3D_precomp, viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, prefiltered,
                                    out_color, out_invdepth, radii, render_indices, parent_indices,
                                    interpolation_weights, num_node_kids, num_render, debug, stream, num_rendered, 0u);
}

int gsr_rasterize_forward_ex(gsr_resize_fn geom_buffer, gsr_resize_fn binning_buffer, gsr_resize_fn image_buffer,
                             void *resize_ctx, int P, int D, int M, const float *background, int width, int height,
                             const float *means3D, const float *shs, const float *colors_precomp,
                             const float *opacities, const float *scales, float scale_modifier,
                             const float *rotations, const float *cov3D_precomp, const float *viewmatrix,
                             const float *projmatrix, const float *cam_pos, float tan_fovx, float tan_fovy,
                             int prefiltered, float *out_color, float *out_invdepth, int *radii,
                             const int *render_indices, const int *parent_indices,
                             const float *interpolation_weights, const int *num_node_kids, int num_render,
                             int debug, void *stream, int64_t *num_rendered, unsigned flags) {
    (void)prefiltered;
    (void)num_node_kids;  // accepted; render_post's blend (which this reproduces) does not read it
    HostScope host_scope(10);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (flags & ~(unsigned)GSR_FWD_NO_BACKWARD) return fail(GSR_ERR_INVALID_ARGUMENT, "unknown forward flags");
    // the backward's accumulator rows are cleared (and its launch order built) only for a frame a
    // backward may follow: atomic mode, GSR_FWD_NO_BACKWARD not set
    const bool need_bwd = !(flags & GSR_FWD_NO_BACKWARD);
    const bool det_fwd = g_deterministic.load(std::memory_order_relaxed) != 0;
    const bool clear_acc = need_bwd && !det_fwd;
    if (num_rendered) *num_rendered = 0;
    int rc = validate_common(P, D, M, shs, colors_precomp, scales, rotations, cov3D_precomp, width, height);
    if (rc) return rc;
    if ((rc = validate_cut(num_render, P, shs, scales, rotations, render_indices, parent_indices,
                           interpolation_weights)))
        return rc;
    if (!geom_buffer || !binning_buffer || !image_buffer)
        return fail(GSR_ERR_INVALID_ARGUMENT, "resize callbacks must be non-NULL");
    if (!background || !out_color || !viewmatrix || !projmatrix || !cam_pos || (P > 0 && !radii))
        return fail(GSR_ERR_INVALID_ARGUMENT, "NULL required pointer");
    if (P > 0 && (!means3D || !opacities))
        return fail(GSR_ERR_INVALID_ARGUMENT, "NULL means3D / opacities");

    // Hierarchy cut: the rasterizer renders the num_render rows blended from (render_indices,
    // parent_indices, interpolation_weights) over the P input rows -- render_post's LOD blend
    // (gaussian_renderer/__init__.py:200-243) done here, into the geometry buffer.
    const int64_t Nin = P;
    const int R = num_render;
    if (R > 0) P = R;
    // render_post's blend fused into the preprocess and the SH colour pass (the cut's rows read in
    // place, no R-row copy written and re-read) for frames no backward follows (render_hierarchy.py's
    // no_grad frames); a frame a backward may follow keeps the blended rows in its geometry buffer,
    // where the backward reads them
#ifndef GSR_CUT_FUSED
#define GSR_CUT_FUSED 1
#endif
    GaussianInputs probe{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                         scale_modifier, g_raw_params ? 1 : 0};
    const bool fuse_cut = GSR_CUT_FUSED && R > 0 && !need_bwd && cut_fusable(probe);

    const Camera cam = make_camera(viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, width, height);
    const int T = cam.gx * cam.gy;
    const int npix = width * height;

    size_t ibytes = 0;
    const size_t gbytes = geom_bytes(P, cam.gx, cam.gy, fuse_cut ? 0 : R, M);
    if (!sb_grid_supported(sb_grid(cam.gx, cam.gy, P)))
        return fail(GSR_ERR_UNSUPPORTED, "image too large for the superblock grid");
    carve_image(nullptr, T, npix, &ibytes);
    void *gbase = geom_buffer(resize_ctx, gbytes);
    void *ibase = image_buffer(resize_ctx, ibytes);
    if (!gbase || !ibase) return fail(GSR_ERR_ALLOCATION, "geometry/image buffer allocation failed");
    GeomState gs = carve_geom(gbase, P, cam.gx, cam.gy, nullptr);
    if (!clear_acc) gs.nacc = 0;
    note_forward_geom(gbase, need_bwd, clear_acc);
    const ImageState is = carve_image(ibase, T, npix, nullptr);
    if (R > 0 && !fuse_cut) {
        const CutRows cr = cut_rows_of(gbase, P, cam.gx, cam.gy, M);
        if ((rc = gsr_interpolate_cut_forward(Nin, M, R, 0, render_indices, parent_indices, interpolation_weights,
                                              means3D, scales, rotations, opacities, shs, cr.means, cr.scales,
                                              cr.rots, cr.opac, cr.shs, stream)))
            return rc;
        means3D = cr.means;
        scales = cr.scales;
        rotations = cr.rots;
        opacities = cr.opac;
        shs = cr.shs;
        if ((rc = check("hierarchy cut blend", debug, s))) return rc;
    }

    if (g_raw_params && (R > 0 || cov3D_precomp))
        return fail(GSR_ERR_UNSUPPORTED, "raw parameters with a hierarchy cut or precomputed covariances");
    GaussianInputs in{P, D, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                      scale_modifier, g_raw_params ? 1 : 0};
    if (fuse_cut) in.cut = CutRef{render_indices, parent_indices, interpolation_weights, Nin};
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // GSR_COLOR_SERIAL=1 runs the SH colour pass on the main stream right after the preprocess:
    // beside the binning on the side stream it slows the binning by about its own length (both
    // want the CUs), but run serially it costs the same (2490-2498 vs 2540 Mpix/s), so the side
    // stream stays the default.
    const bool split = P > 0 && color_split_supported(in) &&
                       (GSR_COLOR_SERIAL || side_stream(s, &side, &fork, &join));
    if (fuse_cut && !split) return fail(GSR_ERR_DEVICE, "hierarchy cut: the fused blend needs the SH colour pass");
    SideJoin sj;
#ifndef GSR_COLOR_FORK
#define GSR_COLOR_FORK 2  // 0: beside the sort and the binning; 1: beside the binning only; 2: chosen per frame
#endif
#ifndef GSR_COLOR_LOCAL_BLOCKS
#define GSR_COLOR_LOCAL_BLOCKS 128  // local-sort frames: the colour pass's persistent grid beside the binning
#endif
    // Depth order (binning.hip): the local sort (level 1 in index order, each superblock list sorted
    // in LDS) unless the frame is in deterministic mode (its backward needs the global sort's
    // record offsets) or the global sort is forced; a local frame whose longest SB list exceeds
    // what the LDS sort holds is re-run through the global sort.
    bool local = P > 0 && g_binning_mode.load(std::memory_order_relaxed) == 0 && !det_fwd;
    // The depth sort runs one 1024-thread workgroup per 8192 keys (dsort_blocks) and leaves the
    // other CUs idle: when it leaves a good share of them, the SH colour pass forks right after the
    // preprocess as a persistent grid on those CUs (1M Gaussians: 123 sort workgroups, 128 colour
    // blocks; 2640 -> 2696 Mpix/s, 133 blocks already slowed the sort); otherwise it forks after the sort, beside the
    // binning, at full width.  Local-sort frames fork it right after the preprocess too, as a
    // persistent grid of GSR_COLOR_LOCAL_BLOCKS blocks beside the binning.
    int color_blocks = 0;
    bool color_early = GSR_COLOR_FORK == 0;
    if (local && split && !GSR_COLOR_SERIAL) {
        color_early = GSR_COLOR_FORK != 1;  // 1: after the level-1 counts, beside the scatter and the sort
        color_blocks = GSR_COLOR_LOCAL_BLOCKS;
    } else if (GSR_COLOR_FORK == 2 && split && !GSR_COLOR_SERIAL) {
        {
            // workgroups are dealt round-robin over the 8 XCDs: leave every XCD room for its share
            // of the sort's workgroups (123 of them -> 16 per XCD -> 8 x (32 - 16) = 128 colour blocks)
            const int per_xcd = device_cus() / 8;
            const int free_cus = 8 * (per_xcd - (dsort_blocks(P) + 7) / 8);
            if (free_cus >= 2 * per_xcd) {
                color_early = true;
                color_blocks = free_cus;
            } else {
                // the sort fills the chip (large P).  Two rounds of it or more (config 5's 7.46M rows):
                // the colour pass forks right after the preprocess, so it overlaps the sort as well
                // as the binning (config 5 3.62 -> 3.51 ms, r05f); config 3's 3M-row frames measured
                // no gain (55.0 vs 55.3 s), so they keep the fork after the sort
                color_early = color_early_big() && dsort_blocks(P) >= 2 * device_cus();
                color_blocks = color_big_blocks() ? color_big_blocks() : color_early ? 0 : color_late_grid();
            }
        }
    }
    auto fork_color = [&](const int *vis_radii) -> int {
        // fork: the SH colours stream in beside latency-bound main-stream stages; joined before render_fwd
        if (hipEventRecord(fork, s) != hipSuccess || hipStreamWaitEvent(side, fork, 0) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "side stream fork failed");
        {
            StageTimer st(8, side);
            launch_preprocess_color(in, cam, gs, vis_radii, side, color_blocks);
        }
        if (hipEventRecord(join, side) != hipSuccess) return fail(GSR_ERR_DEVICE, "side stream join record failed");
        sj.s = s;
        sj.join = join;
        sj.pending = true;
        return check("preprocess colour", debug, side);
    };
#ifndef GSR_COLOR_PRE_CUT
#define GSR_COLOR_PRE_CUT 1
#endif
    // A fused hierarchy cut whose colour pass forks early (config 5): forked before the preprocess,
    // so it overlaps the preprocess as well; it then colours every row (no radii yet: a cut frame's
    // rows are all in view) and writes only the colour quarter of each render record and the clamp
    // bits, which the preprocess leaves to it.  Config 5's raster part 2.30 -> 2.28 ms (r06zt,
    // interleaved; the pass itself 1.44 -> 1.85 ms, longer but off the critical path).
    const bool pre_fork = GSR_COLOR_PRE_CUT && fuse_cut && split && !GSR_COLOR_SERIAL && color_early;
    if (pre_fork && (rc = fork_color(nullptr))) return rc;
    {
        StageTimer st(0, s);
        launch_preprocess(in, cam, gs, radii, s, split);
    }
    if ((rc = check("preprocess", debug, s))) return rc;
    if (split && GSR_COLOR_SERIAL) {
        {
            StageTimer st(8, s);
            launch_preprocess_color(in, cam, gs, radii, s);
        }
        if ((rc = check("preprocess colour", debug, s))) return rc;
    }
    if (split && !GSR_COLOR_SERIAL && color_early && !pre_fork && (rc = fork_color(radii))) return rc;
    // K sizes the point list.  With a capacity hint from this device's previous frame the binning
    // and the forward render are queued first and K is read afterwards (the GPU never waits on
    // the host's hand-off); kernels that would overrun the capacity exit at once (they compare the
    // device's K / instance totals with bs.cap) and the frame's binning and render are queued
    // again at the real K.  Without a hint (first frame, debug) K is read before the binning.
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevicesK)
        return fail(GSR_ERR_DEVICE, "no current device");
    const bool defer = GSR_DEFER_K && P > 0 && !debug && g_khint[dev] > 0;
    hipEvent_t k_ready = nullptr;
    if (P > 0) {
        if (!g_pinned) {
            if (hipHostMalloc(reinterpret_cast<void **>(&g_pinned), kHostWords * sizeof(uint32_t),
                              hipHostMallocCoherent) != hipSuccess ||
                hipHostGetDevicePointer(reinterpret_cast<void **>(&g_pinned_dev), g_pinned, 0) != hipSuccess)
                return fail(GSR_ERR_ALLOCATION, "pinned host allocation failed");
            for (int k = 0; k < kHostWords; k++) g_pinned[k] = 0u;
            for (int d = 0; d < kMaxDevicesK; d++) g_long_tile_at[d] = g_long_sb_at[d] = -2 * kSplitMemory;
        }
        if (!g_k_ready[dev] && hipEventCreateWithFlags(&g_k_ready[dev], hipEventDisableTiming) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "event creation failed");
        // deferred K: no event -- its marker packet cost a ~7 us gap before the first sort pass;
        // the host polls the pinned word the upsweep / column scan stores instead (read_K)
        k_ready = (defer && GSR_K_POLL) ? nullptr : g_k_ready[dev];
        __atomic_store_n(&g_pinned[kHostK], kKPending, __ATOMIC_SEQ_CST);
    }
    const FrameWords fw_local{dsort_K_word(gs), dsort_maxsb_word(gs), g_pinned_dev};
    const FrameWords fw_none{nullptr, nullptr, nullptr};
    // the forward's launch order by superblock and the backward class counters zeroed, both by the
    // level-1 column scan (no tile_order launch); P == 0 frames run no binning: tile_order does both
    const bool sb_order = GSR_FWD_SB_ORDER && P > 0;
    uint32_t *const order_sb = sb_order ? is.tile_ids : nullptr;
    uint32_t *const zero_cls = GSR_BWD_CLS && need_bwd && sb_order ? is.bwd_cnt : nullptr;
    if (local) {
        {
            StageTimer st(1, s);  // level-1 counts, SB bases, K
            launch_binning_count(P, cam, gs, true, fw_local, order_sb, zero_cls, s, false);
            if (k_ready) (void)hipEventRecord(k_ready, s);
        }
        if ((rc = check("binning (counts)", debug, s))) return rc;
    } else if (P > 0) {
        {
            StageTimer st(1, s);
            launch_depth_sort(P, gs, g_pinned_dev + kHostK, g_pinned_dev + kHostErr, s, k_ready);
        }
        if ((rc = check("depth sort", debug, s))) return rc;
    }
    int64_t K = 0;
    uint32_t maxsb = 0;
    bool have_K = P == 0;
    auto read_K = [&]() -> int {
        const auto t_wait = std::chrono::steady_clock::now();
        if (k_ready) {
            if (hipEventSynchronize(k_ready) != hipSuccess) return fail(GSR_ERR_DEVICE, "num_rendered wait failed");
        } else {
            // the frame is queued; the upsweep's (column scan's) last workgroup stores K into the
            // pinned word (it is normally there already: the host runs ahead of the GPU).  A drained
            // stream with the word still pending falls through to the device copy below.
            while (__atomic_load_n(&g_pinned[kHostK], __ATOMIC_SEQ_CST) == kKPending) {
                const hipError_t q = hipStreamQuery(s);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) return fail(GSR_ERR_DEVICE, "num_rendered wait failed");
                std::this_thread::yield();
            }
        }
        g_kwait_ns.fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                   t_wait).count(),
                             std::memory_order_relaxed);
        uint32_t k = __atomic_load_n(&g_pinned[kHostK], __ATOMIC_ACQUIRE);
        uint32_t m = __atomic_load_n(&g_pinned[kHostMaxSB], __ATOMIC_ACQUIRE);
        if (k == kKPending) {  // not expected: read the device copies instead (a local frame's K
                               // word may read "capacity short": its instance total is K)
            const uint32_t *kw = local ? gs.sb_base_i + gs.sb.nsb : dsort_K_word(gs);
            if (hipMemcpy(&k, kw, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(&m, dsort_maxsb_word(gs), sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
                return fail(GSR_ERR_DEVICE, "num_rendered copy failed");
        }
        if (debug && !local) {  // the sort passes are complete here (debug syncs after every stage)
            uint32_t err = 0;
            if (hipMemcpy(&err, dsort_err_word(gs), sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess || err)
                return fail(GSR_ERR_DEVICE, "depth sort: a lookback spin timed out");
        }
        if ((rc = sticky_sort_error())) return rc;
        K = (int64_t)k;
        maxsb = local ? m : 0u;
        have_K = true;
        return GSR_OK;
    };
    // a local frame re-run through the global sort: the head control words (tickets, counters, K)
    // start from zero again, the lookback status words are still zero (the local path never
    // touches them)
    auto to_global = [&]() -> int {
        local = false;
        g_fallbacks.fetch_add(1, std::memory_order_relaxed);
        if (hipMemsetAsync(gs.ctrl, 0, sizeof(uint32_t) * (size_t)dsort_head_words(), s) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "depth sort control reset failed");
        {
            StageTimer st(1, s);
            launch_depth_sort(P, gs, nullptr, g_pinned_dev + kHostErr, s, nullptr);
        }
        return check("depth sort", debug, s);
    };
    if (P > 0 && !defer) {
        if ((rc = read_K())) return rc;
        if (local && maxsb > (uint32_t)sort_cap() && (rc = to_global())) return rc;
    }
    if (split && !GSR_COLOR_SERIAL && !color_early && (rc = fork_color(radii))) return rc;
    bool joined = false;
    const uint32_t seg_req = need_bwd && bwd_segments_supported() ? g_bwd_seg.load(std::memory_order_relaxed) : 0u;
    uint32_t fseg_req = fwd_segments_supported() && !sb_order ? g_fwd_seg.load(std::memory_order_relaxed) : 0u;
    uint32_t tb_req = tb_split_len();
    // the split's minimum list length, read once per frame: tile_order's queue, render_fwd's skip test
    // and the gate must agree even if gsr_set_fwd_split_min runs meanwhile
    const uint32_t fseg_min = fseg_req ? fseg_min_len(fseg_req) : 0u;
    const FwdSpin spin = fwd_spin(g_pinned_dev);
    if (P > 0) {
        // the split gate: the longest lists of the frames before (whatever the pinned words hold now)
        const int64_t f = ++g_frame_no[dev];
        const uint32_t tl = __atomic_load_n(&g_pinned[kHostTileList], __ATOMIC_RELAXED);
        const uint32_t sl = __atomic_load_n(&g_pinned[kHostSBList], __ATOMIC_RELAXED);
        if (fseg_req && tl > fseg_min) g_long_tile_at[dev] = f;
        if (tb_req && sl > tb_req) g_long_sb_at[dev] = f;
        if (g_split_gate.load(std::memory_order_relaxed)) {
            if (f - g_long_tile_at[dev] > kSplitMemory) fseg_req = 0;
            if (f - g_long_sb_at[dev] > kSplitMemory) tb_req = 0;
        }
    }
    uint32_t seg_used = 0;
    bool fsplit_armed = false, tbsplit_armed = false;
    auto bin_and_render = [&](int64_t cap, bool counted) -> int {
        const uint32_t tbs = !local && P > 0 ? tb_req : 0u;
        tbsplit_armed = tbs != 0u;
        // backward / forward items are numbered tile + T * segment (32 bits)
        seg_used = seg_req && (uint64_t)T * (uint64_t)(cap / seg_req + 1) < (1ull << 32) ? seg_req : 0u;
        const uint32_t fseg_used =
            fseg_req && cap > 0 && (uint64_t)T * (uint64_t)(cap / fseg_req + 1) < (1ull << 32) ? fseg_req : 0u;
        fsplit_armed = fseg_used != 0u;
        size_t bbytes = 0;
        carve_binning(nullptr, cap, &bbytes, seg_used, fseg_used);
        void *bbase = binning_buffer(resize_ctx, bbytes);
        if (!bbase) return fail(GSR_ERR_ALLOCATION, "binning buffer allocation failed");
        BinningState bs = carve_binning(bbase, cap, nullptr, seg_used, fseg_used);
        // P == 0: no depth sort ran, its control words are not initialised (no capacity test)
        bs.kdev = P > 0 ? dsort_K_word(gs) : nullptr;
        int r;
        {
            StageTimer st(2, s);
            if (!local && !counted)
                launch_binning_count(P, cam, gs, false, fw_none, order_sb, zero_cls, s, tbs,
                                     GSR_HOST_WORDS == 2 ? dsort_longest_words(gs) + 1
                                     : GSR_HOST_WORDS ? g_pinned_dev + kHostSBList : nullptr);
            launch_binning_scatter(P, cam, gs, bs, local, s);
        }
        if ((r = check("binning (superblocks)", debug, s))) return r;
        {
            StageTimer st(3, s);
            // long superblock lists in slices beside tile_bin (a second side stream: the first may
            // still carry the colour pass)
            hipStream_t ts = s;
            hipEvent_t tf = nullptr, tj = nullptr;
            const bool tfork = tbs != 0u && side_stream(s, &ts, &tf, &tj, 1) && ts != s;
            if (tfork && (hipEventRecord(tf, s) != hipSuccess || hipStreamWaitEvent(ts, tf, 0) != hipSuccess))
                return fail(GSR_ERR_DEVICE, "side stream fork failed");
            launch_binning_tiles(P, cam, gs, bs, is, local, dsort_maxsb_word(gs), s, tbs != 0u, tfork ? ts : nullptr);
            if (tfork && (hipEventRecord(tj, ts) != hipSuccess || hipStreamWaitEvent(s, tj, 0) != hipSuccess))
                return fail(GSR_ERR_DEVICE, "side stream join failed");
        }
        if ((r = check("binning (tiles)", debug, s))) return r;
        // forward segments: the worker pool launched now, on the second side stream once the binning
        // (and the colour pass) are done, so its workgroups are resident before render_fwd's grid
        // fills the CUs; they start on the queue when tile_order releases it.  Joined after render_fwd.
        hipStream_t ws = s;
        hipEvent_t wf = nullptr, wj = nullptr;
        bool early = false;
        if (fseg_used && !sb_order && fwd_early_workers() && !fwd_segments_in_kernel() &&
            side_stream(s, &ws, &wf, &wj, 1) && ws != s) {
            if (hipEventRecord(wf, s) != hipSuccess || hipStreamWaitEvent(ws, wf, 0) != hipSuccess ||
                (split && !GSR_COLOR_SERIAL && !joined && hipStreamWaitEvent(ws, join, 0) != hipSuccess))
                return fail(GSR_ERR_DEVICE, "side stream fork failed");
            launch_render_fwd_workers(cam, gs, bs, is, background, out_color, out_invdepth, need_bwd, seg_used,
                                      fseg_used, ws, dsort_fwdready_word(gs), spin);
            if (hipEventRecord(wj, ws) != hipSuccess) return fail(GSR_ERR_DEVICE, "side stream join record failed");
            early = true;
        }
        if (!sb_order) {
            StageTimer st(4, s);
            // forward order: by list length (and the backward's class counters zeroed)
            launch_tile_order(nullptr, is.ranges, T, 4, is.tile_ids, s, bs.kdev, bs.cap,
                              GSR_BWD_CLS && need_bwd ? is.bwd_cnt : nullptr, is.bwd_cnt + kFwdItemsWord, bs.point_list,
                              seg_used, fseg_used,
                              P > 0 && GSR_HOST_WORDS == 2 ? dsort_longest_words(gs)
                              : P > 0 && GSR_HOST_WORDS ? g_pinned_dev + kHostTileList : nullptr,
                              early ? dsort_fwdready_word(gs) : nullptr, fseg_min);
        }
        if ((r = check("tile order", debug, s))) return r;
        if (split && !GSR_COLOR_SERIAL && !joined) {
            sj.pending = false;
            joined = true;
            if (hipStreamWaitEvent(s, join, 0) != hipSuccess) return fail(GSR_ERR_DEVICE, "side stream join failed");
        }
        {
            StageTimer st(5, s);
            // forward segments: the worker pool on the side stream, beside render_fwd (which skips the
            // split tiles); joined before anything reads the frame
            hipStream_t wside = s;
            hipEvent_t wfork = nullptr, wjoin = nullptr;
            if (fseg_used && !early && !fwd_segments_in_kernel() && !side_stream(s, &wside, &wfork, &wjoin)) wside = s;
            const bool forked = fseg_used && !early && wside != s;
            if (forked && (hipEventRecord(wfork, s) != hipSuccess || hipStreamWaitEvent(wside, wfork, 0) != hipSuccess))
                return fail(GSR_ERR_DEVICE, "side stream fork failed");
            launch_render_fwd(cam, gs, bs, is, background, out_color, out_invdepth, s, need_bwd, sb_order, seg_used,
                              fseg_used, wside, early, P > 0 && GSR_HOST_WORDS == 2 ? dsort_longest_words(gs) : nullptr,
                              g_pinned_dev, fseg_min, spin);
            // the early pool's workers may have given up on the ready word (the two streams did not
            // run concurrently): a small second launch on this stream, after tile_order, takes any
            // item still queued -- no frame depends on the streams' concurrency
            if (early)
                launch_render_fwd_cleanup(cam, gs, bs, is, background, out_color, out_invdepth, need_bwd, seg_used,
                                          fseg_used, s, spin);
            if (forked && (hipEventRecord(wjoin, wside) != hipSuccess || hipStreamWaitEvent(s, wjoin, 0) != hipSuccess))
                return fail(GSR_ERR_DEVICE, "side stream join failed");
            if (early && hipStreamWaitEvent(s, wj, 0) != hipSuccess) return fail(GSR_ERR_DEVICE, "side stream join failed");
        }
        if (need_bwd && !GSR_BWD_CLS) {
            StageTimer st(9, s);  // backward launch order, from the forward's per-tile work
            launch_tile_order(is.tile_work, is.ranges, T, 2, is.tile_order, s, bs.kdev, bs.cap);
        }
        return check("render", debug, s);
    };
    const int64_t cap0 = defer ? g_khint[dev] : K;
    if ((rc = bin_and_render(cap0, false))) return rc;
    if (!have_K && (rc = read_K())) return rc;
    if (debug && P > 0) {  // the binning's instance total must be K (the kernels' capacity test is on K)
        uint32_t bi = 0;
        if (hipMemcpy(&bi, gs.sb_base_i + gs.sb.nsb, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "binning total copy failed");
        if ((int64_t)bi != K) return fail(GSR_ERR_DEVICE, "binning: superblock instance total differs from K");
    }
    if (P > 0) g_frames.fetch_add(1, std::memory_order_relaxed);
    if (fsplit_armed) g_fsplit_frames.fetch_add(1, std::memory_order_relaxed);
    if (tbsplit_armed) g_tbsplit_frames.fetch_add(1, std::memory_order_relaxed);
    if (local && maxsb > (uint32_t)sort_cap()) {
        // an SB list too long for the LDS sort (the sort kernel wrote nothing): the frame again
        // through the global depth sort, at the capacity it needs
        if ((rc = to_global())) return rc;
        if ((rc = bin_and_render(std::max(K, cap0), false))) return rc;
    } else if (K > cap0) {  // the capacity was short: again at K
        g_reruns.fetch_add(1, std::memory_order_relaxed);
        // global sort: sb_colscan's last-workgroup counter (a depth-sort control word the
        // preprocess zeroes once per frame) must start from zero again; local sort: the counts and
        // SB bases stand, only the scatter and the LDS sort re-run
        if (!local && hipMemsetAsync(dsort_aux_word(gs), 0, sizeof(uint32_t), s) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "binning counter reset failed");
        if ((rc = bin_and_render(K, local))) return rc;
    }
    note_forward_seg(ibase, seg_used);  // the re-run's segment length (its capacity may differ)
    if (P > 0 && local) g_local_frames.fetch_add(1, std::memory_order_relaxed);
    // the kernels compare K with a 32-bit capacity: keep the hint representable
    if (P > 0) {
        g_khist[dev][g_khead[dev]] = K;
        g_khead[dev] = (g_khead[dev] + 1) % kKHist;
        int64_t kmax = 0;
        for (int i = 0; i < kKHist; i++) kmax = std::max(kmax, g_khist[dev][i]);
        // the kernels compare K with a 32-bit capacity: keep the hint representable
        g_khint[dev] = std::min<int64_t>(kmax + kmax / 8 + 4096, (int64_t)UINT32_MAX);
    }
    if (num_rendered) *num_rendered = K;
    return GSR_OK;
}

int gsr_rasterize_backward(gsr_resize_fn scratch, void *resize_ctx, int P, int D, int M, int64_t R_inst,
                           const float *background, int width, int height, const float *means3D,
                           const float *shs, const float *colors_precomp, const float *scales,
                           float scale_modifier, const float *rotations, const float *cov3D_precomp,
                           const float *viewmatrix, const float *projmatrix, const float *cam_pos,
                           float tan_fovx, float tan_fovy, const int *radii, void *geom_buffer,
                           void *binning_buffer, void *image_buffer, const float *dL_dpix,
                           const float *dL_dinvdepth, float *dL_dmeans2D, float *dL_dcolors, float *dL_dopacity,
                           float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscales,
                           float *dL_drotations, const int *render_indices, const int *parent_indices,
                           const float *interpolation_weights, const int *num_node_kids, int num_render,
                           int debug, void *stream) {
    (void)num_node_kids;
    HostScope host_scope(11);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int rc = validate_common(P, D, M, shs, colors_precomp, scales, rotations, cov3D_precomp, width, height);
    if (rc) return rc;
    if ((rc = validate_cut(num_render, P, shs, scales, rotations, render_indices, parent_indices,
                           interpolation_weights)))
        return rc;
    if (R_inst < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "num_rendered must be >= 0");
    if (!scratch) return fail(GSR_ERR_INVALID_ARGUMENT, "scratch callback must be non-NULL");
    if (!geom_buffer || !binning_buffer || !image_buffer || !dL_dpix)
        return fail(GSR_ERR_INVALID_ARGUMENT, "NULL state buffer / dL_dpix");
    if (P > 0 && !radii) return fail(GSR_ERR_INVALID_ARGUMENT, "NULL radii");
    if (P > 0 && (!dL_dmeans2D || !dL_dopacity || !dL_dmeans3D || (!shs && !dL_dcolors) ||
                  (cov3D_precomp && !dL_dcov3D)))
        return fail(GSR_ERR_INVALID_ARGUMENT, "NULL gradient output");
    if (P > 0 && shs && !dL_dsh) return fail(GSR_ERR_INVALID_ARGUMENT, "NULL dL_dsh");
    if (P > 0 && !cov3D_precomp && (!dL_dscales || !dL_drotations))
        return fail(GSR_ERR_INVALID_ARGUMENT, "NULL dL_dscales / dL_drotations");
    if ((rc = sticky_sort_error())) return rc;
    const uint8_t uncleared = forward_uncleared(geom_buffer);
    if (uncleared == kNoBackward)
        return fail(GSR_ERR_INVALID_ARGUMENT, "backward of a forward made with GSR_FWD_NO_BACKWARD (its accumulator "
                                              "rows were not cleared); run the forward without the flag");

    const int64_t Nin = P;
    const int R = num_render;
    const float *rotations_in = rotations;
    if (R > 0) P = R;
    const Camera cam = make_camera(viewmatrix, projmatrix, cam_pos, tan_fovx, tan_fovy, width, height);
    const int T = cam.gx * cam.gy;
    const GeomState gs = carve_geom(geom_buffer, P, cam.gx, cam.gy, nullptr);
    const BinningState bs = carve_binning(binning_buffer, R_inst, nullptr);
    const ImageState is = carve_image(image_buffer, T, width * height, nullptr);
    // a frame's accumulation mode is the one in force at its forward: one forwarded in
    // deterministic mode has no cleared accumulators (record path), one forwarded in atomic mode
    // may have no record offsets (the local sort computes none)
    const bool atomic = uncleared != kDeterministicFwd;
    size_t sbytes = 0;
    const bool list = live_list();  // read once: the carve must match the size
    carve_bwd(nullptr, R_inst, P, atomic, &sbytes, list);
    // hierarchy cut: gradients of the R blended rows first, then scattered to the input rows
    size_t cut_off = 0;
    if (R > 0) {
        Carver c(nullptr);
        c.off = sbytes;
        carve_cut(c, R, M);
        cut_off = sbytes;
        sbytes = align_up(c.off, 256);
    }
    void *sbase = scratch(resize_ctx, std::max<size_t>(sbytes, 256));  // atomic mode: the live masks only
    if (!sbase) return fail(GSR_ERR_ALLOCATION, "backward scratch allocation failed");
    BwdScratch sc = carve_bwd(sbase, R_inst, P, atomic, nullptr, list);
    sc.acc = gs.acc;
    if (GSR_PERSISTENT_ACC && atomic && P > 0 && !(sc.acc = acc_rows(s, (size_t)P)))
        return fail(GSR_ERR_ALLOCATION, "backward accumulator rows allocation failed");

    // sparse rows only for plain frames (the cut's rows are scattered to the input rows below)
    GaussianGrads out{dL_dmeans2D, dL_dcolors, dL_dopacity, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales,
                      dL_drotations, g_sparse_grad_rows && R == 0 ? 1 : 0};
    CutRows rows{}, grows{};
    if (R > 0) {
        rows = cut_rows_of(geom_buffer, P, cam.gx, cam.gy, M);
        Carver c(sbase);
        c.off = cut_off;
        grows = carve_cut(c, R, M);
        means3D = rows.means;
        scales = rows.scales;
        rotations = rows.rots;
        shs = rows.shs;
        out.dmeans3D = grows.means;
        out.dscales = grows.scales;
        out.drots = grows.rots;
        out.dopacity = grows.opac;
        out.dsh = grows.shs;
        // means2D: the rendered rows' screen-space gradient lands in rows [0, R) of the input's
        // gradient (render_post slices means2D[:R + skybox] the same way); the rest is zero
        if (Nin > R && hipMemsetAsync(dL_dmeans2D + 3 * (size_t)R, 0, sizeof(float) * 3 * (size_t)(Nin - R), s) !=
                           hipSuccess)
            return fail(GSR_ERR_DEVICE, "means2D gradient clear failed");
    }
    if (g_raw_params && (R > 0 || cov3D_precomp))
        return fail(GSR_ERR_UNSUPPORTED, "raw parameters with a hierarchy cut or precomputed covariances");
    GaussianInputs in{P, D, M, means3D, shs, colors_precomp, nullptr, scales, rotations, cov3D_precomp,
                      scale_modifier, g_raw_params ? 1 : 0};
    bool zeroed = false;
    ZeroRows zr{};
    {
        StageTimer st(6, s);
        // the dense zero gradient rows go out beside render_bwd's replay (bwd_zero_rows)
        const uint32_t seg = forward_seg(image_buffer);
        zeroed = R_inst > 0 && bwd_zero_rows(in, out, sc, gs.live_stamp, (int)bwd_grid(T, R_inst, seg), &zr);
        if (R_inst > 0)
            launch_render_bwd(cam, gs, bs, is, radii, background, dL_dpix, dL_dinvdepth, sc, s, zeroed ? &zr : nullptr,
                              seg);
    }
    if ((rc = check("render backward", debug, s))) return rc;
    {
        StageTimer st(7, s);
        launch_preprocess_bwd(in, cam, gs, is, radii, sc, out, s, zeroed ? &zr : nullptr);
    }
    if (GSR_PERSISTENT_ACC && atomic && P > 0) acc_rows_consumed();  // the consumer zeroes what it reads
    if ((rc = check("preprocess backward", debug, s))) return rc;
    if (R > 0) {
        const size_t n3 = sizeof(float) * 3 * (size_t)Nin;
        if (hipMemsetAsync(dL_dmeans3D, 0, n3, s) != hipSuccess || hipMemsetAsync(dL_dscales, 0, n3, s) != hipSuccess ||
            hipMemsetAsync(dL_drotations, 0, sizeof(float) * 4 * (size_t)Nin, s) != hipSuccess ||
            hipMemsetAsync(dL_dopacity, 0, sizeof(float) * (size_t)Nin, s) != hipSuccess ||
            hipMemsetAsync(dL_dsh, 0, sizeof(float) * 3 * (size_t)M * Nin, s) != hipSuccess)
            return fail(GSR_ERR_DEVICE, "gradient clear failed");
        if ((rc = gsr_interpolate_cut_backward(Nin, M, R, 0, render_indices, parent_indices, interpolation_weights,
                                               rotations_in, grows.means,
                                               grows.scales, grows.rots, grows.opac, grows.shs, dL_dmeans3D,
                                               dL_dscales, dL_drotations, dL_dopacity, dL_dsh, stream)))
            return rc;
        if ((rc = check("hierarchy cut blend backward", debug, s))) return rc;
    }
    return GSR_OK;
}

int gsr_set_true_scale_gradient(int enable) {
    const int prev = g_true_scale_grad.exchange(enable ? 1 : 0);
    return prev;
}

int gsr_set_deterministic(int enable) { return g_deterministic.exchange(enable ? 1 : 0); }

int gsr_set_split_gate(int enable) { return g_split_gate.exchange(enable ? 1 : 0); }

int gsr_set_live_list(int enable) { return g_live_list.exchange(enable ? 1 : 0); }

int gsr_set_fwd_spin_limits(int64_t ready, int64_t flag) {
    if (ready < -1 || flag < 0 || ready >= UINT32_MAX || flag > UINT32_MAX)
        return fail(GSR_ERR_INVALID_ARGUMENT, "spin limits: ready -1 or 0 (default) .. 2^32 - 2, flag 0 .. 2^32 - 1");
    set_fwd_spin_limits(ready < 0 ? kFwdReadyNever : (uint32_t)ready, (uint32_t)flag);
    return GSR_OK;
}

int gsr_set_fwd_split_min(int len) {
    if (len < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "forward split minimum list length must be >= 0");
    return (int)set_fwd_split_min((uint32_t)len);
}

int gsr_set_fwd_segment(int L) {
    if (L < 0 || (L > 0 && (L < (int)kMinFwdSeg || L % kWave != 0)))
        return fail(GSR_ERR_INVALID_ARGUMENT, "forward segment length: 0 (off) or a multiple of 64 >= 1024");
    if (L > 0 && !fwd_segments_supported())
        return fail(GSR_ERR_UNSUPPORTED, "forward segments need the list-length launch order and the 1-row sub-block forward");
    return (int)g_fwd_seg.exchange((uint32_t)L);
}

int gsr_set_bwd_segment(int L) {
    if (L < 0 || (L > 0 && (L < (int)kMinBwdSeg || L % kWave != 0)))
        return fail(GSR_ERR_INVALID_ARGUMENT, "backward segment length: 0 (off) or a multiple of 64 >= 512");
    if (L > 0 && !bwd_segments_supported())
        return fail(GSR_ERR_UNSUPPORTED, "backward segments need the class launch order and the 1-row sub-block forward");
    return (int)g_bwd_seg.exchange((uint32_t)L);
}

int gsr_set_binning(int mode) {
    if (mode < 0 || mode > 1) return fail(GSR_ERR_INVALID_ARGUMENT, "gsr_set_binning: mode 0 or 1");
    return g_binning_mode.exchange(mode);
}

int gsr_forward_stats(int64_t *out, int n) {
    if (!out || n < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "NULL stats buffer");
    collect_giveups();
    const int64_t v[kFwdStats] = {g_frames.load(), g_reruns.load(), g_local_frames.load(), g_fallbacks.load(),
                                  g_fwd_giveups.load(), g_kwait_ns.load(), g_fsplit_frames.load(),
                                  g_tbsplit_frames.load()};
    int k = 0;
    for (; k < n && k < kFwdStats; k++) out[k] = v[k];
    return k;
}

int gsr_segment_layout_check(int64_t K, int L, int Lf, int64_t *need, int64_t *have) {
    if (K < 0 || L < 0 || Lf < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "negative size");
    size_t bytes = 0;
    carve_binning(nullptr, K, &bytes, (uint32_t)L, (uint32_t)Lf);
    const size_t end = segment_end(K, (uint32_t)L, (uint32_t)Lf);
    if (need) *need = (int64_t)end;
    if (have) *have = (int64_t)bytes;
    return end <= bytes ? GSR_OK : GSR_ERR_INVALID_ARGUMENT;
}

int gsr_reset_capacity_hint(void) {
    if (g_pinned) g_pinned[kHostTileList] = g_pinned[kHostSBList] = 0u;
    for (int d = 0; d < kMaxDevicesK; d++) {
        g_long_tile_at[d] = g_long_sb_at[d] = g_frame_no[d] - 2 * kSplitMemory;
        g_khint[d] = 0;
        g_khead[d] = 0;
        for (int i = 0; i < kKHist; i++) g_khist[d][i] = 0;
    }
    return GSR_OK;
}

int gsr_frame_stats(const void *geom_buffer, int P, int width, int height, int64_t *out, int n) {
    if (!out || n < 0 || P < 0 || width <= 0 || height <= 0)
        return fail(GSR_ERR_INVALID_ARGUMENT, "gsr_frame_stats: bad arguments");
    if (P == 0 || n == 0) {
        for (int k = 0; k < n && k < 4; k++) out[k] = 0;
        return n < 4 ? n : 4;
    }
    if (!geom_buffer) return fail(GSR_ERR_INVALID_ARGUMENT, "gsr_frame_stats: NULL geometry buffer");
    const int gx = (width + kTile - 1) / kTile, gy = (height + kTile - 1) / kTile;
    const GeomState gs = carve_geom(const_cast<void *>(geom_buffer), P, gx, gy, nullptr);
    std::vector<uint32_t> bg((size_t)gs.sb.nsb + 1);
    uint32_t v[4] = {0u, 0u, 0u, 0u};
    if (hipMemcpy(bg.data(), gs.sb_base_g, sizeof(uint32_t) * bg.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&v[1], gs.sb_base_i + gs.sb.nsb, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&v[2], gs.tb_flag + gs.sb.nsb, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return fail(GSR_ERR_DEVICE, "gsr_frame_stats: copy failed");
    v[0] = bg[gs.sb.nsb];
    for (int k = 0; k < gs.sb.nsb; k++) v[3] = std::max(v[3], bg[k + 1] - bg[k]);
    int k = 0;
    for (; k < n && k < 4; k++) out[k] = (int64_t)v[k];
    return k;
}

// Kernel stamps (GSR_KSTAMP measurement builds, tools/kstamp.py): out[kKsIds * (1 + 2 * kKsRing)], per
// kernel id its launch count, then its last 64 launches' starts and ends (s_memrealtime ticks,
// 100 MHz).  GSR_ERR_UNSUPPORTED in a normal build.
int gsr_kstamp_read(unsigned long long *out, int n) {
    constexpr int per = 1 + 2 * kKsRing;
    if (!out || n < kKsIds * per) return fail(GSR_ERR_INVALID_ARGUMENT, "kstamp buffer too small");
    if (!GSR_KSTAMP) return fail(GSR_ERR_UNSUPPORTED, "not a GSR_KSTAMP build");
    static std::vector<unsigned long long> tmp((size_t)kKsIds * per);
    for (int i = 0; i < kKsIds * per; i++) out[i] = 0;
    int (*readers[])(unsigned long long *) = {kstamp_read_preprocess, kstamp_read_dsort, kstamp_read_binning,
                                              kstamp_read_render, kstamp_read_backward};
    for (auto rd : readers) {
        if (rd(tmp.data()) != 0) return fail(GSR_ERR_DEVICE, "kstamp read failed");
        for (int i = 0; i < kKsIds; i++)
            if (tmp[(size_t)i * per] > out[(size_t)i * per])
                for (int k = 0; k < per; k++) out[(size_t)i * per + k] = tmp[(size_t)i * per + k];
    }
    return GSR_OK;
}

int gsr_debug_trace(int64_t *out, int n, int reset) {
    if (!GSR_HOST_TRACE) return gsr::debug_trace(out, n, reset);
    if (!out || n < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "NULL trace buffer");
    int k = 0;
    for (; k < n && k < 2 * kHostTrace; k++)
        out[k] = k < kHostTrace ? g_htrace_ns[k].load() : g_htrace_cnt[k - kHostTrace].load();
    if (reset)
        for (int i = 0; i < kHostTrace; i++) g_htrace_ns[i] = g_htrace_cnt[i] = 0;
    return k;
}

int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_INVALID_ARGUMENT, "P must be >= 0");
    if (P > 0 && (!means3D || !viewmatrix || !present)) return fail(GSR_ERR_INVALID_ARGUMENT, "NULL pointer");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    launch_mark_visible(P, means3D, viewmatrix, present, s);
    return check("markVisible", 0, s);
}

}  // extern "C"
