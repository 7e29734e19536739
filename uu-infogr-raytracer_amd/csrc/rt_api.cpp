// rt_api.cpp -- C ABI of libraytracer_hip (include/raytracer_hip.h).
//
// Host side of the drop-in: context lifetime, scene upload (with the scene-constant
// precomputation described in rt_internal.h), camera math (RayTracer.cs:511-523,
// :543-554, :892-896, :1058-1061), frame rendering (single GPU, row bands, and the
// single-process multi-GPU Tick: every device traces its interleaved row bands and hands
// them to the caller's Surface.pixels over its own PCIe link; device-resident frames are
// gathered to device 0 over RCCL/xGMI), HIP-event timing and work counters.  Never throws
// across the ABI; no CPU fallback.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <link.h>
#include <new>
#include <string>
#include <vector>

#include "../../include/raytracer_hip.h"
#include "rt_internal.h"

using namespace rtk;

// ----------------------------------------------------------------------------
// minimal RCCL binding (resolved with dlopen only for multi-GPU contexts, so a
// single-GPU process never needs librccl)
// ----------------------------------------------------------------------------
namespace {
typedef void* ncclComm_t;
typedef int ncclResult_t;
enum { ncclUint8 = 1, ncclInt32 = 2, ncclInt64 = 4 };
enum { ncclMax = 2 };
struct ncclUniqueId {
    char internal[RT_COMM_ID_BYTES];
};
// The librccl already mapped into the process (torch's, in a torch.distributed job), so that our
// communicator and the framework's share one RCCL instance; else the first that dlopen finds.
// Only the library itself: its basename is "librccl.so" or "librccl.so.<version>" (RCCL's net and
// tuner plugins, e.g. librccl-net.so, also contain "librccl" but lack the nccl* entry points).
bool is_librccl(const char* path) {
    const char* base = std::strrchr(path, '/');
    base = base ? base + 1 : path;
    if (std::strncmp(base, "librccl.so", 10) != 0) return false;
    for (const char* p = base + 10; *p; ++p)
        if (!(*p == '.' || (*p >= '0' && *p <= '9'))) return false;
    return true;
}
int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* out) {
    if (info->dlpi_name && is_librccl(info->dlpi_name)) {
        *(std::string*)out = info->dlpi_name;
        return 1;
    }
    return 0;
}
struct Rccl {
    void* h = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Gather)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    bool load(std::string& err) {
        if (h) return true;
        std::string loaded;
        dl_iterate_phdr(find_loaded_rccl, &loaded);
        if (!loaded.empty()) h = dlopen(loaded.c_str(), RTLD_NOW | RTLD_NOLOAD);
        // RTLD_LOCAL: a RCCL loaded here must not interpose on one the process loads later (torch's own
        // librccl, pulled in by an `import torch` after our first RCCL context): with RTLD_GLOBAL the two
        // copies shared symbols and the process aborted at exit ("double free or corruption (!prev)", r05b) --
        // the one cause, profiles/r06_exit_abort.txt (RCCL then `import torch` aborts under RTLD_GLOBAL only)
        const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char* n : names)
            if (!h && (h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            err = "dlopen(librccl) failed";
            return false;
        }
        CommInitAll = (decltype(CommInitAll))dlsym(h, "ncclCommInitAll");
        CommDestroy = (decltype(CommDestroy))dlsym(h, "ncclCommDestroy");
        Gather = (decltype(Gather))dlsym(h, "ncclGather");
        GroupStart = (decltype(GroupStart))dlsym(h, "ncclGroupStart");
        GroupEnd = (decltype(GroupEnd))dlsym(h, "ncclGroupEnd");
        GetUniqueId = (decltype(GetUniqueId))dlsym(h, "ncclGetUniqueId");
        CommInitRank = (decltype(CommInitRank))dlsym(h, "ncclCommInitRank");
        AllReduce = (decltype(AllReduce))dlsym(h, "ncclAllReduce");
        Send = (decltype(Send))dlsym(h, "ncclSend");
        Recv = (decltype(Recv))dlsym(h, "ncclRecv");
        GetErrorString = (decltype(GetErrorString))dlsym(h, "ncclGetErrorString");
        if (!CommInitAll || !CommDestroy || !Gather || !GroupStart || !GroupEnd || !GetUniqueId || !CommInitRank ||
            !AllReduce || !Send || !Recv) {
            err = "librccl lacks a symbol (ncclCommInitAll/InitRank/GetUniqueId/Gather/AllReduce/Send/Recv/Group*)";
            return false;
        }
        return true;
    }
};
Rccl g_rccl;

thread_local std::string g_last_error;

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    int kind = 0;  // 0 kernel, 1 copy, 2 gather
};

struct Device {
    int id = 0;
    hipStream_t stream = nullptr;
    void* d_scene = nullptr;
    size_t scene_cap = 0;
    int32_t* d_frame = nullptr;  // full frame (device 0 of multi-GPU contexts)
    size_t frame_cap = 0;
    int32_t* d_bands = nullptr;  // this device's packed row bands (multi-GPU)
    size_t bands_cap = 0;
    int32_t* d_gather = nullptr;  // device 0: n_gpus x padded band sets
    size_t gather_cap = 0;
    void* d_stage = nullptr;  // rt_encode_bands scratch (encodes on one context are stream-ordered)
    size_t stage_cap = 0;
    // the batch whose tiles rt_render_bands_tiles last staged in d_stage (rt_finish_wire finishes only
    // that one; rt_encode_bands reuses the scratch and clears it)
    struct {
        bool valid = false;
        int W = 0, H = 0, band_rows = 0, rank = 0, world = 0, batch_frames = 0;
        const void* wire = nullptr;
    } staged;
    int32_t* d_frames2[2] = {nullptr, nullptr};  // rt_render_async double buffer (this device's band set)
    size_t frames2_cap[2] = {0, 0};
    // rt_render_async: one in-order stream per device; frame k's D2H rides in frame k+1's launch (the
    // copy slice, LaunchParams::copy) or is issued by rt_wait -- `hand` is that pending copy
    hipStream_t async_stream = nullptr;
    struct {
        int32_t* host = nullptr;  // caller's buffer (one contiguous band set: hipMemcpyAsync on a flush)
        CopyJob job{};            // the band set -> the buffer's device-mapped address (job.words 0: none)
    } hand;
    hipEvent_t ev_join = nullptr;  // rt_render_device at n > 1: ordering against the caller's stream
    // the synchronous Tick's copy-engine hand-off of chunk c on its own stream, after the chunk's trace
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_chunk[8] = {};
    // rt_render_async's copy-engine hand-off (RT_TICK_ASYNC=stream): slot s traced -> copied events
    hipEvent_t ev_traced[2] = {}, ev_copied[2] = {};
    bool copy_pending[2] = {false, false};
    // frames in flight of the copy-engine hand-off (rt_ctx::tick_inflight): frame f's copy done -> ring[f % 16]
    static constexpr int RING = 16;
    hipEvent_t ev_ring[RING] = {};
    uint64_t frames_issued = 0;
    float* d_view_tab = nullptr;  // lx[W] then ly[H] (view_tables)
    size_t view_tab_cap = 0;
    int tab_w = -1, tab_h = -1;
    float tab_pw = 0, tab_ph = 0;
    int async_next = 0;
    unsigned long long* d_counters = nullptr;
    unsigned long long* d_counters_diag = nullptr;  // rt_count_work
    std::vector<EventPair> pending, pool;
    uint64_t op_count[3] = {0, 0, 0};  // operations per timing kind (sampling phase)
    // Dispatch order of single-frame launches (order_pick): which of the ORDER_CANDIDATES the direct
    // kernel's workgroups follow, chosen by timing a few launches of each for the current scene and
    // frame size.  Every order traces the same tiles the same way: only their start order differs.
    struct OrderTuner {
        int chosen = -1;           // -1: measuring
        int turn = 0;              // next candidate to measure
        int W = 0, H = 0;          // frame size and scene generation the measurements belong to
        uint64_t scene_gen = 0, gen = 0;
        uint64_t since = 0;        // single-frame launches since the choice (re-measured every ORDER_RETUNE)
        std::vector<float> ms[4];
        // candidate 3: the tiles in decreasing order of their measured duration (the first single-frame
        // launch of a measuring round records every tile's duration; tile_order_prepare)
        struct Tiles {
            int W = 0, H = 0;
            uint64_t gen = 0, scene_gen = 0;
            bool recorded = false, built = false;
            rt_camera cam{};         // the camera of the recorded durations
            uint64_t uses = 0;       // candidate-3 launches since they were recorded
            uint32_t* d_order = nullptr;  // padded to SINGLE_WPG (ty = 0xffff past the last tile)
            uint32_t* d_cost = nullptr;   // RTC ticks per tile
            size_t order_cap = 0, cost_cap = 0;
        } tiles;
        struct Probe {
            hipEvent_t a = nullptr, b = nullptr;
            int cand = 0;
            uint64_t gen = 0;
        };
        std::vector<Probe> pending, pool;
    } order;
    ncclComm_t comm = nullptr;
    int comm_rank = 0, comm_world = 0;  // rt_comm_init (one rank per process); 0 = none
};

struct SceneLayout {
    int S = 0, P = 0, L = 0, limit = 0;
    size_t off_sph = 0, off_mat = 0, off_pl = 0, off_li = 0, off_cull = 0, off_shcull = 0, bytes = 0;
    size_t off_shg = 0, off_shgrid = 0, off_shslab = 0, off_clus = 0, off_shpre = 0;
    bool has_shpre = false;  // the direct kernel's shadow pre-test records (DevShadowCull [L][S + (S & 1)])
    int n_clus = 0;  // DevCluster records (the bundle kernel's per-lane pre-cull), 0: none
    bool has_shcull = false;
    bool has_shg = false;  // per-light shadow grids (DevShadowGrid) for the merged shadow pass
    std::vector<unsigned char> host_blob;  // the uploaded scene image (host tests read the tables)
    bool generic_pow = false;        // a specular material with n not in {0.5, 1, 2}
    bool lights_a2_ok = true;        // every light's 2a = 2 p.p finite and > 0
    std::vector<DevSphere> host_sph;  // for the per-frame primary constants
    std::vector<DevPlane> host_pl;    // for the single-frame launches' row order (row_order)
};
}  // namespace

// rt_render_async's frames in flight per worker behind the copy engine (rt_create_ex; RT_TICK_INFLIGHT)
constexpr int TICK_INFLIGHT = 2;

struct rt_ctx {
    int n_gpus = 1;            // band workers: devices, or streams on one device (RT_CREATE_SHARED_DEVICE)
    bool rccl_gather = false;  // RT_CREATE_RCCL_GATHER: rt_render gathers the bands to device 0 over RCCL, one D2H
    bool shared_device = false;  // RT_CREATE_SHARED_DEVICE: every worker on the caller's device
    bool comm_all = false;       // the single-process communicators (ncclCommInitAll) exist
    std::vector<Device> dev;
    bool has_scene = false;
    SceneLayout layout;
    rt_camera cam{};
    std::string last_error;
    uint64_t frames = 0, pixels = 0, launches = 0;
    uint64_t prim_rays = 0;  // traced pixels (the kernels count only reflect/shadow rays)
    double kernel_ms = 0, last_kernel_ms = 0, copy_ms = 0, gather_ms = 0;
    uint64_t timed[3] = {0, 0, 0};  // timed launches, copies, gathers
    int timing_every = 64;
    bool counting = true;  // rt_set_counting: trace launches add to the ray counters
    uint64_t scene_gen = 0;  // rt_set_scene calls (the dispatch-order measurements belong to one scene)
    int order_fixed = -1;    // RT_DISPATCH_ORDER=0/1/2: that candidate for every single-frame launch
    int tick_inflight = 0;   // rt_render_async: frames queued per worker before the host waits (0: no bound)
    int32_t* host_staging = nullptr;
    // host ranges registered through rt_register_host and their device-mapped addresses (one per
    // worker: each device writes its band set through its own mapping): only these are written by the
    // Tick hand-off's copy kernels (anything else takes the runtime's copies)
    struct HostRange {
        char* host;
        size_t bytes;
        std::vector<char*> mapped;  // [worker], nullptr where the device has no mapping
    };
    std::vector<HostRange> host_ranges;
    // view_params cache: the camera and frame size of the last call (this scene) and the view part
    // of LaunchParams they gave (per-sphere screen boxes: a few us of host trig per launch)
    bool view_ok = false;
    rt_camera view_cam{};
    int view_w = 0, view_h = 0, view_rows = 0;
    int view_height = 0;  // rt_set_view_height: the view's height (0: each render's own frame height)
    LaunchParams view_lp{};
};

// ----------------------------------------------------------------------------
// error helpers
// ----------------------------------------------------------------------------
static int fail(rt_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    if (ctx) ctx->last_error = buf;
    return code;
}

#define HIP_TRY(ctx, call)                                                                                 \
    do {                                                                                                   \
        hipError_t e_ = (call);                                                                            \
        if (e_ != hipSuccess) return fail((ctx), RT_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

namespace {
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int grow(rt_ctx* ctx, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return RT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) return fail(ctx, RT_ERR_OOM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    *cap = bytes;
    return RT_OK;
}

// Sum completed event pairs into the context totals (waits for them).
void drain_events(rt_ctx* ctx, Device& d) {
    for (EventPair& ep : d.pending) {
        float ms = 0.0f;
        (void)hipEventSynchronize(ep.b);
        if (hipEventElapsedTime(&ms, ep.a, ep.b) == hipSuccess) {
            if (ep.kind == 0) {
                ctx->kernel_ms += ms;
                ctx->last_kernel_ms = ms;
            } else if (ep.kind == 1) {
                ctx->copy_ms += ms;
            } else {
                ctx->gather_ms += ms;
            }
            ctx->timed[ep.kind]++;
        }
        d.pool.push_back(ep);
    }
    d.pending.clear();
}

// Sampled device timing: the every-th operation of each kind on each device is bracketed
// by an event pair (rt_set_timing).  Returns whether this one is.
bool begin_timed(rt_ctx* ctx, Device& d, int kind) {
    const int every = ctx->timing_every;
    if (every <= 0 || (d.op_count[kind]++ % (uint64_t)every) != 0) return false;
    if (d.pending.size() >= 4096) drain_events(ctx, d);  // bound host memory; stalls only then
    EventPair ep;
    if (!d.pool.empty()) {
        ep = d.pool.back();
        d.pool.pop_back();
    } else {
        if (hipEventCreate(&ep.a) != hipSuccess || hipEventCreate(&ep.b) != hipSuccess) return false;
    }
    ep.kind = kind;
    (void)hipEventRecord(ep.a, d.stream);
    d.pending.push_back(ep);
    return true;
}

void end_timed(Device& d, bool timed) {
    if (timed) (void)hipEventRecord(d.pending.back().b, d.stream);
}

// Host-side Vector3 helpers (binary32, no contraction: built with -ffp-contract=off).
struct H3 {
    float x, y, z;
};
H3 h3(rt_vec3 v) { return H3{v.x, v.y, v.z}; }
float hdot(H3 a, H3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
H3 hcross(H3 l, H3 r) {
    return H3{(l.y * r.z) - (l.z * r.y), (l.z * r.x) - (l.x * r.z), (l.x * r.y) - (l.y * r.x)};
}
H3 hnormalize(H3 a) {
    float s = 1.0f / std::sqrt(hdot(a, a));
    return H3{a.x * s, a.y * s, a.z * s};
}
bool hzero(rt_vec3 v) { return v.x == 0 && v.y == 0 && v.z == 0; }

DevMaterial dev_material(const rt_material& m, rt_vec3 ambient) {
    DevMaterial d;
    std::memset(&d, 0, sizeof d);
    d.kd[0] = m.kd.x, d.kd[1] = m.kd.y, d.kd[2] = m.kd.z;
    d.amb[0] = ambient.x * m.ka.x, d.amb[1] = ambient.y * m.ka.y, d.amb[2] = ambient.z * m.ka.z;
    d.ks[0] = m.ks.x, d.ks[1] = m.ks.y, d.ks[2] = m.ks.z;
    d.n = m.n;
    d.km[0] = m.km.x, d.km[1] = m.km.y, d.km[2] = m.km.z;
    d.flags = (hzero(m.km) ? 0u : MAT_MIRROR) | (hzero(m.kd) ? 0u : MAT_DIFFUSE) |
              ((!hzero(m.ks) && m.n > 0.0f) ? MAT_SPEC : 0u);
    d.pow_kind = m.n == 1.0f ? POW_ONE : m.n == 0.5f ? POW_HALF : m.n == 2.0f ? POW_TWO : POW_GENERIC;
    return d;
}

// Shadow rays (IntersectShadowLight, RayTracer.cs:573-582 -> IntersectsSphere with epsilon
// 0.001f, :613-636): with 2a finite and > 0 the ray collides iff fl(fl(n / 2a) - e) > 0, n =
// fl(-b - sqrt(disc)) (the near root decides, rt_kernel.hip shadow_blocked).  For floats q and
// e the sign of fl(q - e) is that of q - e, so the test is fl(n / 2a) > e.  Correct rounding is
// monotonic: fl(z) > e iff z > m, m = e + ulp(e)/2 the midpoint above e, except z == m, which
// rounds to the even neighbour -- succ(e) when e's significand is odd.  So the collision is
// n >= m * 2a (odd e) or n > m * 2a (even e); m has 25 significant bits and 2a 24, so the
// product is exact in double, and for a float n, "n >= T" equals "n >= the smallest float >= T"
// (and "n > T" equals "n >= the smallest float > T").  Returns that float (+inf above FLT_MAX).
float shadow_threshold(float a2) {
    const float e = 0.001f;
    int ex = 0;
    (void)std::frexp(e, &ex);                                // e = f * 2^ex, f in [0.5, 1)
    const double m = (double)e + std::ldexp(1.0, ex - 25);  // + ulp(e) / 2 (ulp = 2^(ex - 24))
    uint32_t eb;
    std::memcpy(&eb, &e, sizeof eb);
    const bool odd = (eb & 1u) != 0;
    const double T = m * (double)a2;                         // exact
    float t = (float)T;
    if ((double)t < T || (!odd && (double)t == T)) t = std::nextafter(t, INFINITY);
    return t;
}

int total_bands(int H, int band_rows) { return (H + band_rows - 1) / band_rows; }
int bands_of(int H, int band_rows, int first, int step) {
    int tb = total_bands(H, band_rows);
    return first < tb ? (tb - 1 - first) / step + 1 : 0;
}

// Conservative screen box of a sphere for primary rays (culling only; computed in double).
//
// Pixel (x, y) traces the line from the camera along D = R lx + U ly + F lz with
// lx = (x/W - 0.5) pw, ly = (y/H - 0.5) ph, lz = near (TracePixel :963-971).  By the
// cull_mask analysis the binary32 IntersectsSphere cannot select the sphere when that line
// passes at distance >= rho = r (1 + 2^-8) + 2^-8 |u| from its centre (u = C - camera), with
// |u| also scaled by the kernel's direction error (cancellation in vp - cam, bounded by
// 2^-20 (|cam| + |D|) / |D|; no box when that exceeds 2^-12).  The distance to the line is at
// least the distance to the plane through it containing the camera's up (right) axis, so
// in camera coordinates (cx, cy, cz) the x range follows from the 2-D circle (cx, cz; rho):
// lx / lz in [tan(phi - g), tan(phi + g)], phi = atan2(cx, cz), g = asin(rho / |(cx, cz)|),
// valid when cz > rho (sphere strictly in front); same for y with (cy, cz).  Two pixels of
// slack cover the binary32 pixel-to-direction mapping and the basis' non-orthogonality.
PrimBox prim_box(const LaunchParams& lp, const DevSphere& s) {
    const PrimBox all{INT_MIN / 2, INT_MAX / 2, INT_MIN / 2, INT_MAX / 2};
    const double pw = lp.pw, ph = lp.ph, lz = lp.nearc;
    if (!(pw > 0) || !(ph > 0) || !(lz > 0) || !std::isfinite(pw) || !std::isfinite(ph) || !std::isfinite(lz))
        return all;
    const double cam[3] = {lp.cam[0], lp.cam[1], lp.cam[2]};
    const double u[3] = {s.cx - cam[0], s.cy - cam[1], s.cz - cam[2]};
    auto dot3 = [](const double* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    const double ulen = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    const double camlen = std::sqrt(cam[0] * cam[0] + cam[1] * cam[1] + cam[2] * cam[2]);
    const double dmax = std::sqrt(0.25 * pw * pw + 0.25 * ph * ph + lz * lz);
    const double dir_err = 0x1p-20 * (camlen + dmax) / lz + 0x1p-20;
    const double r = std::sqrt((double)s.r2);
    if (!std::isfinite(ulen) || !std::isfinite(r) || !(dir_err <= 0x1p-12)) return all;
    const double rho = (r * (1.0 + 0x1p-8) + (0x1p-8 + 0x1p-20 + dir_err) * ulen) * (1.0 + 0x1p-16) + 0x1p-60;
    auto fdot = [](const float* a, const float* b) { return (double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2]; };
    const double ortho = std::fabs(fdot(lp.right, lp.up)) + std::fabs(fdot(lp.right, lp.fwd)) +
                         std::fabs(fdot(lp.up, lp.fwd)) + std::fabs(fdot(lp.right, lp.right) - 1.0) +
                         std::fabs(fdot(lp.up, lp.up) - 1.0) + std::fabs(fdot(lp.fwd, lp.fwd) - 1.0);
    if (!(ortho < 0x1p-18)) return all;  // the camera basis is orthonormal up to rounding
    const double cx = dot3(u, lp.right), cy = dot3(u, lp.up), cz = dot3(u, lp.fwd);
    if (!(cz > rho * (1.0 + 0x1p-10))) return all;
    auto range = [&](double c, double plane, int n, int& lo, int& hi) {
        const double phi = std::atan2(c, cz);
        const double g = std::asin(std::min(1.0, rho / std::sqrt(c * c + cz * cz)));
        const double tlo = std::tan(phi - g), thi = std::tan(phi + g);
        const double flo = n * (0.5 + lz * tlo / plane), fhi = n * (0.5 + lz * thi / plane);
        if (!std::isfinite(flo) || !std::isfinite(fhi)) {
            lo = INT_MIN / 2, hi = INT_MAX / 2;
            return;
        }
        lo = (int)std::max(-1e9, std::floor(flo) - 2.0);
        hi = (int)std::min(1e9, std::ceil(fhi) + 2.0);
    };
    PrimBox b;
    range(cx, pw, lp.W, b.x0, b.x1);
    range(cy, ph, lp.H, b.y0, b.y1);
    return b;
}

// Order of a single-frame launch's tile rows (LaunchParams::row_order).  The launch's last waves set
// its tail, so the expensive rows should start first and the cheap ones come last.  A tile row's cost
// is estimated from eight primary rays through its middle pixel row: 1 for a ray that meets nothing,
// 1 + L when it meets a plane in front of the camera or falls inside a diffuse sphere's screen box
// (prim_box: shaded, with shadow rays), (1 + L)(1 + min(limit, 4)) inside a mirror sphere's box (its
// reflected chain is shaded too).  Rows are sorted by decreasing estimate, ties in natural order.
// The estimate only orders the workgroups: every tile is traced exactly as before.
int row_order(const LaunchParams& lp, const SceneLayout& L, uint16_t* order) {
    const int rows = (lp.H + 7) / 8;
    if (rows < 2 || rows > ROW_ORDER_MAX) return 0;
    const DevMaterial* mat = L.host_blob.size() >= L.off_mat + sizeof(DevMaterial) * (size_t)(L.S + L.P)
                                 ? (const DevMaterial*)(L.host_blob.data() + L.off_mat)
                                 : nullptr;
    const double shade = 1.0 + L.L, mirror = shade * (1.0 + std::min(L.limit, 4));
    std::vector<double> cost((size_t)rows, 0.0);
    for (int r = 0; r < rows; ++r) {
        const int y = std::min(lp.H - 1, r * 8 + 4);
        const double ly = ((double)y / lp.H - 0.5) * lp.ph;
        for (int j = 0; j < 8; ++j) {
            const int x = (int)(((2 * j + 1) * (long long)lp.W) / 16);
            const double lx = ((double)x / lp.W - 0.5) * lp.pw;
            double d[3];
            for (int k = 0; k < 3; ++k) d[k] = lp.right[k] * lx + lp.up[k] * ly + lp.fwd[k] * lp.nearc;
            double w = 1.0;
            for (const DevPlane& q : L.host_pl) {
                const double den = d[0] * q.nx + d[1] * q.ny + d[2] * q.nz;
                const double num = q.cn - (lp.cam[0] * q.nx + lp.cam[1] * q.ny + lp.cam[2] * q.nz);
                if (den != 0 && num / den > 0) w = std::max(w, shade);
            }
            if (lp.prim_const)
                for (int i = 0; i < L.S; ++i)
                    if (x >= lp.pbox[i].x0 && x <= lp.pbox[i].x1 && y >= lp.pbox[i].y0 && y <= lp.pbox[i].y1)
                        w = std::max(w, mat && (mat[i].flags & MAT_MIRROR) ? mirror : shade);
            cost[(size_t)r] += w;
        }
    }
    std::vector<int> idx((size_t)rows);
    for (int r = 0; r < rows; ++r) idx[(size_t)r] = r;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return cost[(size_t)a] > cost[(size_t)b]; });
    for (int r = 0; r < rows; ++r) order[r] = (uint16_t)idx[(size_t)r];
    return rows;
}

void copy_view(const LaunchParams& from, LaunchParams& to) {
    std::memcpy(to.cam, from.cam, sizeof to.cam);
    std::memcpy(to.right, from.right, sizeof to.right);
    std::memcpy(to.up, from.up, sizeof to.up);
    std::memcpy(to.fwd, from.fwd, sizeof to.fwd);
    to.pw = from.pw, to.ph = from.ph, to.nearc = from.nearc;
    to.W = from.W, to.H = from.H;
    to.prim_const = from.prim_const;
    std::memcpy(to.pc, from.pc, sizeof to.pc);
    std::memcpy(to.pbox, from.pbox, sizeof to.pbox);
    to.row_order_n = from.row_order_n;
    to.col_major = from.col_major;
    std::memcpy(to.row_order, from.row_order, sizeof(uint16_t) * (size_t)from.row_order_n);
}

// The view of a W x VH frame (VH: rt_set_view_height, else H), of which a render traces rows [0, H).
int view_params(rt_ctx* ctx, int W, int H, LaunchParams& lp) {
    const int VH = ctx->view_height > 0 ? ctx->view_height : H;
    if (H > VH) return fail(ctx, RT_ERR_INVALID_ARG, "frame height %d above the view height %d", H, VH);
    if (ctx->view_ok && ctx->view_w == W && ctx->view_h == VH && ctx->view_rows == H &&
        std::memcmp(&ctx->view_cam, &ctx->cam, sizeof ctx->cam) == 0) {
        copy_view(ctx->view_lp, lp);
        return RT_OK;
    }
    rt_view v;
    int rc = rt_camera_view(&ctx->cam, W, VH, &v);
    if (rc != RT_OK) return fail(ctx, rc, "invalid frame size %dx%d", W, VH);
    lp.cam[0] = v.position.x, lp.cam[1] = v.position.y, lp.cam[2] = v.position.z;
    lp.right[0] = v.right.x, lp.right[1] = v.right.y, lp.right[2] = v.right.z;
    lp.up[0] = v.up.x, lp.up[1] = v.up.y, lp.up[2] = v.up.z;
    lp.fwd[0] = v.forward.x, lp.fwd[1] = v.forward.y, lp.fwd[2] = v.forward.z;
    lp.pw = v.plane_width, lp.ph = v.plane_height, lp.nearc = v.near_clip;
    lp.W = W, lp.H = VH;  // (the screen boxes and the row order in the view's pixels)
    // primary-segment sphere constants (origin = camera for every pixel)
    const std::vector<DevSphere>& sph = ctx->layout.host_sph;
    lp.prim_const = sph.size() <= (size_t)MAX_PRIM_CONST ? 1 : 0;
    if (lp.prim_const)
        for (size_t i = 0; i < sph.size(); ++i) {
            const H3 oc{lp.cam[0] - sph[i].cx, lp.cam[1] - sph[i].cy, lp.cam[2] - sph[i].cz};
            lp.pc[i] = PrimConst{oc.x, oc.y, oc.z, hdot(oc, oc) - sph[i].r2};
            lp.pbox[i] = prim_box(lp, sph[i]);
        }
    lp.row_order_n = row_order(lp, ctx->layout, lp.row_order);  // dispatch-order candidate 0 (order_pick)
    lp.H = H;  // the rows traced (validity, band counts); a cut view's row order no longer matches: not lone
    copy_view(lp, ctx->view_lp);
    ctx->view_cam = ctx->cam, ctx->view_w = W, ctx->view_h = VH, ctx->view_rows = H, ctx->view_ok = true;
    return RT_OK;
}

void scene_params(const rt_ctx* ctx, const Device& d, LaunchParams& lp) {
    const SceneLayout& L = ctx->layout;
    const char* base = (const char*)d.d_scene;
    lp.sph = (const DevSphere*)(base + L.off_sph);
    lp.mat = (const DevMaterial*)(base + L.off_mat);
    lp.pl = (const DevPlane*)(base + L.off_pl);
    lp.li = (const DevLight*)(base + L.off_li);
    lp.scull = (const DevSphereCull*)(base + L.off_cull);
    lp.shcull = L.has_shcull ? (const DevShadowCull*)(base + L.off_shcull) : nullptr;
    lp.shg = L.has_shg ? (const DevShadowGrid*)(base + L.off_shg) : nullptr;
    lp.shgrid = L.has_shg ? (const unsigned long long*)(base + L.off_shgrid) : nullptr;
    lp.shslab = L.has_shg ? (const unsigned long long*)(base + L.off_shslab) : nullptr;
    lp.clus = L.n_clus ? (const DevCluster*)(base + L.off_clus) : nullptr;
    lp.shpre = L.has_shpre ? (const DevShadowCull*)(base + L.off_shpre) : nullptr;
    lp.n_clus = L.n_clus;
    lp.S = L.S, lp.P = L.P, lp.L = L.L, lp.limit = L.limit;
    lp.lights_a2_ok = L.lights_a2_ok ? 1 : 0;
    lp.counters = ctx->counting ? d.d_counters : nullptr;  // nullptr: the kernels count nothing (rt_set_counting)
}

// Per-column / per-row view-plane coordinates of TracePixel (:963-965), computed with the
// same binary32 operations as the kernel would (-ffp-contract=off, correctly rounded
// division): lx[x] = ((float)x / W - 0.5f) * pw, ly[y] = ((float)y / H - 0.5f) * ph.
// Rebuilt only when the frame size or view-plane size changes; frames in flight may read
// the old table, so the device is synchronised first.
int view_tables(rt_ctx* ctx, Device& d, LaunchParams& lp) {
    const int VH = ctx->view_height > 0 ? ctx->view_height : lp.H;  // the view's height (ly of row y)
    if (d.tab_w != lp.W || d.tab_h != VH || d.tab_pw != lp.pw || d.tab_ph != lp.ph || !d.d_view_tab) {
        std::vector<float> t((size_t)lp.W + (size_t)VH);
        for (int x = 0; x < lp.W; ++x) {
            const float px = (float)x / (float)lp.W - 0.5f;
            t[(size_t)x] = px * lp.pw;
        }
        for (int y = 0; y < VH; ++y) {
            const float py = (float)y / (float)VH - 0.5f;
            t[(size_t)lp.W + (size_t)y] = py * lp.ph;
        }
        HIP_TRY(ctx, hipDeviceSynchronize());
        int rc = grow(ctx, (void**)&d.d_view_tab, &d.view_tab_cap, t.size() * sizeof(float));
        if (rc != RT_OK) return rc;
        HIP_TRY(ctx, hipMemcpy(d.d_view_tab, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice));
        d.tab_w = lp.W, d.tab_h = VH, d.tab_pw = lp.pw, d.tab_ph = lp.ph;
    }
    lp.lxt = d.d_view_tab;
    lp.lyt = d.d_view_tab + lp.W;
    return RT_OK;
}

// Single-frame dispatch order.  A lone frame's launch ends with its slowest waves, so the order in which
// the workgroups start sets its tail (tools/wave_times.py): cheap rows last shortens it when the costly
// tiles are moderate (C1, C2: rows reversed or sorted by the cost estimate, -3 ... -9 %), while deep mirror
// chains (C3: waves of 25-40 us) run faster spread over the whole launch among cheap ones (rows varying
// fastest, -5 %) -- no one order wins every scene (profiles/ab/r04_dispatch_orders.txt).  So the library
// measures: the first single-frame launches of a scene and frame size take the candidates in turn, each
// bracketed by an event pair; once every candidate has ORDER_SAMPLES durations the one with the least
// median is kept, and measured again after ORDER_RETUNE launches (the view drifts).  Candidates:
// 0 tile rows by decreasing estimated cost (row_order), 1 tile rows bottom to top, 2 rows varying fastest
// (column-major over the 4-tile workgroups), natural row order, 3 every tile by decreasing measured
// duration (longest first: a lone frame's tail is its costliest waves started late; C3 36.3 -> 30.8 us,
// profiles/ab/r05_tile_order.txt).  The bundle kernel's lone frames (its all-lights-ok merged
// instantiation) take the same tuner: 0-2 are its natural order, 3 the measured one (C4 338 -> 302 us,
// C5 1,136 -> 1,109 us -- faster than a frame of a 64-frame batch launch, 309 / 1,125 us).
constexpr int ORDER_CANDIDATES = 4, ORDER_SAMPLES = 7;
constexpr float ORDER_MARGIN = 1.01f;  // another order replaces candidate 0 only when > 1 % faster (median)
constexpr uint64_t ORDER_RETUNE = 1u << 14;

void order_collect(Device& d) {
    Device::OrderTuner& t = d.order;
    size_t keep = 0;
    for (size_t i = 0; i < t.pending.size(); ++i) {
        Device::OrderTuner::Probe& pr = t.pending[i];
        if (hipEventQuery(pr.b) != hipSuccess) {
            t.pending[keep++] = pr;
            continue;
        }
        float ms = 0;
        if (pr.gen == t.gen && hipEventElapsedTime(&ms, pr.a, pr.b) == hipSuccess)
            t.ms[pr.cand].push_back(ms);
        t.pool.push_back(pr);
    }
    t.pending.resize(keep);
}

// The candidate for this single-frame launch; *probe: bracket it with order_begin / order_end.
int order_pick(rt_ctx* ctx, Device& d, int W, int H, bool* probe) {
    *probe = false;
    if (ctx->order_fixed >= 0) return ctx->order_fixed;
    Device::OrderTuner& t = d.order;
    if (t.W != W || t.H != H || t.scene_gen != ctx->scene_gen || (t.chosen >= 0 && ++t.since > ORDER_RETUNE)) {
        t.W = W, t.H = H, t.scene_gen = ctx->scene_gen;
        t.chosen = -1, t.turn = 0, t.since = 0, t.gen++;
        for (std::vector<float>& v : t.ms) v.clear();
    }
    if (t.chosen >= 0) return t.chosen;
    order_collect(d);
    // candidate 3 packs tile coordinates in 16 bits each (tile_order_prepare): not for frames beyond that
    const int nc = (W + 7) / 8 > 0xffff || (H + 7) / 8 > 0xffff ? 3 : ORDER_CANDIDATES;
    bool done = true;
    for (int k = 0; k < nc; ++k) done = done && t.ms[k].size() >= (size_t)ORDER_SAMPLES;
    if (done) {
        // the least median, unless candidate 0 is within the margin of it: the launches of a bench or of
        // another process on the GPU can overlap the probes, and a noise-driven choice should not stick
        float best = 0, med0 = 0;
        for (int k = 0; k < nc; ++k) {
            std::vector<float> v = t.ms[k];
            std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
            if (k == 0) med0 = v[v.size() / 2];
            if (t.chosen < 0 || v[v.size() / 2] < best) t.chosen = k, best = v[v.size() / 2];
        }
        if (med0 <= best * ORDER_MARGIN) t.chosen = 0;
        return t.chosen;
    }
    const int k = t.turn++ % nc;
    // bound the probes in flight (results arrive as the launches complete)
    *probe = t.ms[k].size() + t.pending.size() < (size_t)(4 * ORDER_SAMPLES * ORDER_CANDIDATES);
    return k;
}

bool order_begin(Device& d, int cand, hipStream_t s) {
    Device::OrderTuner& t = d.order;
    Device::OrderTuner::Probe pr;
    if (!t.pool.empty()) {
        pr = t.pool.back();
        t.pool.pop_back();
    } else if (hipEventCreate(&pr.a) != hipSuccess || hipEventCreate(&pr.b) != hipSuccess) {
        return false;
    }
    pr.cand = cand, pr.gen = t.gen;
    (void)hipEventRecord(pr.a, s);
    t.pending.push_back(pr);
    return true;
}

void order_end(Device& d, hipStream_t s) { (void)hipEventRecord(d.order.pending.back().b, s); }

// The measured tile order: tiles 0..n-1 (row-major, tx per row) by decreasing cost, ties in natural order, as
// ty << 16 | tx entries.  A stable counting sort in 16-tick (160 ns) buckets (wider ones past 2^20 ticks): linear
// in the tile count -- an 8K frame's 518,400 tiles sort in a few ms, once per measuring round.
void tiles_by_cost(const uint32_t* cost, size_t n, uint32_t tx, uint32_t* order) {
    uint32_t cmax = 0;
    for (size_t i = 0; i < n; ++i) cmax = std::max(cmax, cost[i]);
    const int shift = cmax >> 4 < (1u << 16) ? 4 : 4 + (32 - __builtin_clz(cmax >> 20 | 1u));
    const size_t nb = (size_t)(cmax >> shift) + 1;
    std::vector<uint32_t> start(nb + 1, 0);
    for (size_t i = 0; i < n; ++i) start[nb - (cost[i] >> shift)]++;  // bucket 0 = the longest
    for (size_t b = 1; b <= nb; ++b) start[b] += start[b - 1];
    for (size_t i = 0; i < n; ++i) {
        const uint32_t t = (uint32_t)i;
        order[start[nb - 1 - (cost[i] >> shift)]++] = (t / tx) << 16 | (t % tx);
    }
}

// Candidate 3 of a single-frame launch (the direct kernel's 4-tile workgroups): the first launch of each
// measuring round (and of each frame size / scene) records every tile's duration instead of being timed as a
// probe; the first candidate-3 launch after it reads the durations back and uploads the tiles sorted by
// decreasing duration, ties in natural order.  The readback and the upload wait for the whole device (once
// per measuring round): the recording launch and the launches still reading the previous order may sit on
// any stream of the context (d.stream, the async stream, a caller's stream of rt_render_device).  The order
// is recorded again when the camera has moved and TILE_ORDER_REFRESH launches have used it (an interactive
// view drifts; pixels never depend on the order).  Returns the candidate to launch (candidate 3 falls back to
// 0 while its order is not ready), -1 when the buffers cannot be allocated, -2 on a HIP error (recorded).
constexpr uint64_t TILE_ORDER_REFRESH = 256;
int tile_order_prepare(rt_ctx* ctx, Device& d, int W, int H, LaunchParams& lp, int cand, bool* probe) {
    Device::OrderTuner::Tiles& o = d.order.tiles;
    if (o.gen != d.order.gen || o.scene_gen != ctx->scene_gen || o.W != W || o.H != H ||
        (o.built && o.uses >= TILE_ORDER_REFRESH && std::memcmp(&o.cam, &ctx->cam, sizeof o.cam) != 0)) {
        o.gen = d.order.gen, o.scene_gen = ctx->scene_gen, o.W = W, o.H = H;
        o.recorded = o.built = false;
    }
    const size_t tx = (size_t)(W + 7) / 8, ty = (size_t)(H + 7) / 8, n = tx * ty;
    const size_t padded = (n + SINGLE_WPG - 1) / SINGLE_WPG * SINGLE_WPG;
    if (ty > 0xffff || tx > 0xffff) return cand == 3 ? 0 : cand;  // (not representable: candidates 0-2 only)
    if (!o.recorded) {
        int rc = grow(ctx, (void**)&o.d_cost, &o.cost_cap, n * sizeof(uint32_t));
        if (rc == RT_OK) rc = grow(ctx, (void**)&o.d_order, &o.order_cap, padded * sizeof(uint32_t));
        if (rc != RT_OK) return -1;
        lp.tile_cost = o.d_cost;
        o.recorded = true;
        o.cam = ctx->cam, o.uses = 0;
        *probe = false;  // (the duration stores are not the candidate's own cost)
        return cand == 3 ? 0 : cand;
    }
    if (cand == 3 && !o.built) {
        std::vector<uint32_t> cost(n), order(padded, 0xffff0000u);
        hipError_t e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipMemcpy(cost.data(), o.d_cost, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess) {
            tiles_by_cost(cost.data(), n, (uint32_t)tx, order.data());
            e = hipMemcpy(o.d_order, order.data(), padded * sizeof(uint32_t), hipMemcpyHostToDevice);
        }
        if (e != hipSuccess) {
            fail(ctx, RT_ERR_HIP, "tile order readback / upload: %s", hipGetErrorString(e));
            return -2;
        }
        o.built = true;
    }
    if (cand == 3) {
        lp.tile_order = o.d_order;
        o.uses++;
    }
    return cand;
}

// The fused encoder's target of a trace with out_fmt OUT_TILES (rt_render_bands_tiles).
struct EncTarget {
    unsigned char* wire;
    uint32_t* stage;
    int tiles_x, tpf, frame0;
};

// Launch the trace of bands (first, step) of `band_rows` rows (at most max_bands of them) into `out` on
// device d.  `slice`: a Tick hand-off (CopyJob) that rides in the launch as its copy slice.
int trace_bands(rt_ctx* ctx, Device& d, hipStream_t stream, int W, int H, int band_rows, int first, int step,
                int32_t* out, int* n_bands, int fmt = RT_BANDS_INT32, int n_frames = 1, size_t frame_bytes = 0,
                const EncTarget* enc = nullptr, const CopyJob* slice = nullptr, int max_bands = INT_MAX) {
    LaunchParams lp;
    std::memset(&lp, 0, sizeof lp);
    int rc = view_params(ctx, W, H, lp);
    if (rc != RT_OK) return rc;
    scene_params(ctx, d, lp);
    rc = view_tables(ctx, d, lp);
    if (rc != RT_OK) return rc;
    const int nb = std::min(bands_of(H, band_rows, first, step), max_bands);
    if (n_bands) *n_bands = nb;
    lp.band_rows = band_rows, lp.band_first = first, lp.band_step = step;
    lp.local_rows = nb * band_rows;
    lp.out = out;
    lp.out_fmt = fmt;
    lp.n_frames = n_frames;
    lp.out_frame_bytes = frame_bytes;
    // single-frame launches of a whole frame on the direct kernel: the dispatch order (order_pick)
    const bool with_copy = slice && slice->words;
    const bool whole = !enc && !with_copy && band_rows >= lp.local_rows && lp.local_rows == H;
    const bool lone = n_frames <= 1 && whole && lp.S < CULL_MIN_SPHERES && lp.row_order_n == (H + 7) / 8;
    // the bundle kernel's all-lights-ok merged instantiation (C4/C5): natural or measured tile order
    const SceneLayout& L = ctx->layout;
    const bool lone_bundle = n_frames <= 1 && whole && lp.S >= CULL_MIN_SPHERES && lp.S <= 64 && lp.L >= 1 &&
                             lp.L <= SHADOW_MERGE_L && L.lights_a2_ok && !L.generic_pow;
    bool probe = false;
    int cand = -1;
    if (lone || lone_bundle) {
        cand = order_pick(ctx, d, W, H, &probe);
        // (candidates 1 and 2 order the direct kernel's 4-tile groups: a bundle launch under them is natural order)
        if (ctx->order_fixed < 0 ? d.order.chosen < 0 || cand == 3 : cand == 3)  // measuring, or the measured order
            cand = tile_order_prepare(ctx, d, W, H, lp, cand, &probe);
        if (cand == -2) return RT_ERR_HIP;  // (rt_last_error holds the HIP error)
        if (cand < 0) return fail(ctx, RT_ERR_OOM, "tile order buffers");
        if (lone && cand == 1)
            for (int r = 0; r < lp.row_order_n; ++r) lp.row_order[r] = (uint16_t)(lp.row_order_n - 1 - r);
        if (lone && cand == 2) lp.row_order_n = 0, lp.col_major = 1;
        if (lone_bundle) lp.row_order_n = 0;
    } else {
        lp.row_order_n = 0;  // (batch launches keep the natural order: the measured one measured no better,
                             //  profiles/ab/r05_batch_tile_order_rejected.txt)
    }
    if (enc) {
        lp.out_fmt = OUT_TILES;
        lp.enc_wire = enc->wire, lp.enc_stage = enc->stage;
        lp.enc_tiles_x = enc->tiles_x, lp.enc_tpf = enc->tpf, lp.enc_frame0 = enc->frame0;
    }
    if (with_copy) {  // the previous frame's (chunk's) hand-off rides along
        lp.copy = *slice;
        lp.copy_z = 1;
        lp.out_frame_bytes = 0;
    }
    hipStream_t saved = d.stream;
    d.stream = stream;
    const bool timed = begin_timed(ctx, d, 0);
    probe = probe && order_begin(d, cand, stream);
    int e = launch_trace(lp, ctx->layout.generic_pow, false, stream);
    if (probe) order_end(d, stream);
    end_timed(d, timed);
    d.stream = saved;
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "trace launch failed: %s", hipGetErrorString((hipError_t)e));
    ctx->launches++;
    for (int k = 0; k < nb && ctx->counting; ++k) {  // pixels of rows < H in the launched bands (counted launches)
        const long long y0 = (long long)(first + k * step) * band_rows;
        ctx->prim_rays += (uint64_t)std::min<long long>(band_rows, (long long)H - y0) * (uint64_t)W * (uint64_t)n_frames;
    }
    return RT_OK;
}

int check_ctx(rt_ctx* ctx, int W, int H) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_set_scene has not been called");
    if (W <= 0 || H <= 0 || (long long)W * H > (1LL << 31) - 1)
        return fail(ctx, RT_ERR_INVALID_ARG, "invalid frame size %dx%d", W, H);
    return RT_OK;
}

// Worker g's device-mapped address of [host, host + bytes) when it lies inside a range registered
// through rt_register_host and both ends allow the copy kernels' 16-byte stores; else nullptr.
int32_t* mapped_host(const rt_ctx* ctx, int g, void* host, size_t bytes) {
    if (((uintptr_t)host & 15) != 0) return nullptr;
    const char* h = (const char*)host;
    for (const rt_ctx::HostRange& r : ctx->host_ranges)
        if (h >= r.host && bytes <= r.bytes && (size_t)(h - r.host) <= r.bytes - bytes) {
            char* base = (size_t)g < r.mapped.size() ? r.mapped[(size_t)g] : nullptr;
            if (!base) return nullptr;
            char* m = base + (h - r.host);
            return ((uintptr_t)m & 15) == 0 ? (int32_t*)m : nullptr;
        }
    return nullptr;
}

// The band pipeline of the Tick (the reference's only parallel loop is the row-parallel
// one of RayTracer.cs:898-901).  Worker g of n (a device; RT_CREATE_SHARED_DEVICE: a stream of one
// device) traces the interleaved 8-row bands b = g, g + n, ... of the frame (n == 1: the frame as one
// band) -- balanced however the scene's cost is spread over the rows (the top ~45 % of C2 is sky) --
// packed band after band, and hands them to the caller's frame itself.
constexpr int TICK_BAND_ROWS = 8;
struct Share {
    int band_rows, first, step, nb;  // bands (first, step) of band_rows rows, nb of them
    size_t words;                    // int32 of the packed band set inside the frame (a cut last band)
};
// The int32 of bands [k0, k1) of a share (the frame's last band may be cut at H).
size_t share_words(const Share& sh, int W, int H, int k0, int k1) {
    size_t rows = 0;
    for (int k = k0; k < k1; ++k) {
        const long long y0 = (long long)(sh.first + (long long)k * sh.step) * sh.band_rows;
        rows += (size_t)std::max(0LL, std::min<long long>(sh.band_rows, (long long)H - y0));
    }
    return rows * (size_t)W;
}
Share share_of(int W, int H, int g, int n, bool banded) {
    Share sh;
    sh.band_rows = (n == 1 && !banded) ? H : TICK_BAND_ROWS;
    sh.first = g, sh.step = n;
    sh.nb = bands_of(H, sh.band_rows, g, n);
    sh.words = share_words(sh, W, H, 0, sh.nb);
    return sh;
}
// The hand-off of bands [k0, k1) of a share, traced at src (packed from band k0), into the frame whose
// row 0 is at `frame` (a device-mapped host address or device memory of this worker).
CopyJob share_job(const Share& sh, int W, int H, int k0, int k1, const int32_t* src, int32_t* frame) {
    CopyJob j{};
    const size_t bw = (size_t)sh.band_rows * (size_t)W;
    j.src = src;
    j.dst = frame + (size_t)(sh.first + (size_t)k0 * sh.step) * bw;
    j.words = share_words(sh, W, H, k0, k1);
    j.band_words = sh.step == 1 ? 0u : (unsigned)bw;  // one worker: the bands are one contiguous run
    j.dst_stride = (unsigned long long)sh.step * bw;
    return j;
}

// Issue each worker's pending rt_render_async hand-off (the last frame's D2H) on its async stream.
int flush_hand(rt_ctx* ctx) {
    if (!ctx) return RT_OK;
    for (Device& d : ctx->dev) {
        if (!d.hand.job.words) continue;
        DeviceGuard guard(d.id);
        const auto h = d.hand;
        d.hand = {};
        if (h.host && h.job.band_words == 0) {  // one contiguous band set: the runtime's copy
            HIP_TRY(ctx, hipMemcpyAsync(h.host, h.job.src, h.job.words * sizeof(int32_t), hipMemcpyDeviceToHost,
                                        d.async_stream));
        } else {
            const int e = launch_band_copy(h.job, d.async_stream);
            if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "hand-off copy: %s", hipGetErrorString((hipError_t)e));
        }
    }
    return RT_OK;
}

// A worker's band set (src, packed) into the host frame by the runtime's copies: one contiguous copy
// (one worker), a pitched 2-D copy over the whole bands plus the frame's cut last band (a registered,
// pinned frame: the copy engine writes the rows in place), or one copy per band (an unregistered frame
// -- the slow path; callers register Surface.pixels once -- where a pitched copy would be staged).
int runtime_band_copy(rt_ctx* ctx, const Share& sh, int W, int H, const int32_t* src, int32_t* host, hipStream_t st,
                      bool pinned = false, int k0 = 0, int k1 = -1) {
    if (k1 < 0) k1 = sh.nb;  // bands [k0, k1) of the share; src = the packed band set (band 0)
    if (k1 <= k0) return RT_OK;
    const size_t bw = (size_t)sh.band_rows * (size_t)W;
    auto dst = [&](int k) { return host + (size_t)(sh.first + (size_t)k * sh.step) * bw; };
    if (sh.step == 1) {
        HIP_TRY(ctx, hipMemcpyAsync(dst(k0), src + (size_t)k0 * bw, share_words(sh, W, H, k0, k1) * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, st));
        return RT_OK;
    }
    if (pinned) {
        const bool cut = share_words(sh, W, H, k1 - 1, k1) < bw;
        const int full = k1 - k0 - (cut ? 1 : 0);
        if (full > 0)
            HIP_TRY(ctx, hipMemcpy2DAsync(dst(k0), (size_t)sh.step * bw * sizeof(int32_t), src + (size_t)k0 * bw,
                                          bw * sizeof(int32_t), bw * sizeof(int32_t), (size_t)full,
                                          hipMemcpyDeviceToHost, st));
        if (cut)
            HIP_TRY(ctx, hipMemcpyAsync(dst(k1 - 1), src + (size_t)(k1 - 1) * bw,
                                        share_words(sh, W, H, k1 - 1, k1) * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        return RT_OK;
    }
    for (int k = k0; k < k1; ++k)
        HIP_TRY(ctx, hipMemcpyAsync(dst(k), src + (size_t)k * bw, share_words(sh, W, H, k, k + 1) * sizeof(int32_t),
                                    hipMemcpyDeviceToHost, st));
    return RT_OK;
}

// The single-process communicators of a multi-GPU context (ncclCommInitAll over its devices), made on
// first use: the xGMI gather of rt_render_device at n > 1 and of RT_CREATE_RCCL_GATHER contexts.
int ensure_comm_all(rt_ctx* ctx) {
    if (ctx->comm_all) return RT_OK;
    if (ctx->shared_device && ctx->n_gpus > 1)
        return fail(ctx, RT_ERR_UNSUPPORTED, "RCCL needs one device per rank (RT_CREATE_SHARED_DEVICE context)");
    std::string err;
    if (!g_rccl.load(err)) return fail(ctx, RT_ERR_RCCL, "%s", err.c_str());
    const int n = ctx->n_gpus;
    std::vector<ncclComm_t> comms((size_t)n);
    std::vector<int> ids((size_t)n);
    for (int g = 0; g < n; ++g) ids[(size_t)g] = ctx->dev[(size_t)g].id;
    const ncclResult_t r = g_rccl.CommInitAll(comms.data(), n, ids.data());
    if (r != 0) return fail(ctx, RT_ERR_RCCL, "ncclCommInitAll: %s", g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?");
    for (int g = 0; g < n; ++g) ctx->dev[(size_t)g].comm = comms[(size_t)g];
    ctx->comm_all = true;
    return RT_OK;
}

// Every worker's bands gathered into dst (device 0, row-major frame) on device 0's stream: each device
// traces its band set into its slot, a grouped ncclGather moves the slots to device 0 over xGMI, one
// scatter launch per worker reassembles them there.
int gather_frame(rt_ctx* ctx, int width, int height, int32_t* dst) {
    int rc = ensure_comm_all(ctx);
    if (rc != RT_OK) return rc;
    const int n = ctx->n_gpus;
    const int band_rows = TICK_BAND_ROWS;
    const int max_nb = bands_of(height, band_rows, 0, n);
    const size_t slot = (size_t)max_nb * band_rows * width;  // int32 elements per device
    Device& d0 = ctx->dev[0];
    for (int g = 0; g < n; ++g) {
        Device& d = ctx->dev[(size_t)g];
        DeviceGuard guard(d.id);
        rc = grow(ctx, (void**)&d.d_bands, &d.bands_cap, slot * sizeof(int32_t));
        if (rc == RT_OK && g == 0) rc = grow(ctx, (void**)&d.d_gather, &d.gather_cap, slot * n * sizeof(int32_t));
        if (rc == RT_OK) rc = trace_bands(ctx, d, d.stream, width, height, band_rows, g, n, d.d_bands, nullptr);
        if (rc != RT_OK) return rc;
    }
    std::vector<char> gtimed((size_t)n, 0);
    for (int g = 0; g < n; ++g) {
        DeviceGuard guard(ctx->dev[(size_t)g].id);
        gtimed[(size_t)g] = begin_timed(ctx, ctx->dev[(size_t)g], 2);
    }
    if (g_rccl.GroupStart() != 0) return fail(ctx, RT_ERR_RCCL, "ncclGroupStart failed");
    for (int g = 0; g < n; ++g) {
        Device& d = ctx->dev[(size_t)g];
        DeviceGuard guard(d.id);
        const ncclResult_t r = g_rccl.Gather(d.d_bands, g == 0 ? d.d_gather : nullptr, slot, ncclInt32, 0, d.comm,
                                             d.stream);
        if (r != 0) {
            (void)g_rccl.GroupEnd();
            return fail(ctx, RT_ERR_RCCL, "ncclGather: %s", g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?");
        }
    }
    if (g_rccl.GroupEnd() != 0) return fail(ctx, RT_ERR_RCCL, "ncclGroupEnd failed");
    for (int g = 0; g < n; ++g) {
        DeviceGuard guard(ctx->dev[(size_t)g].id);
        end_timed(ctx->dev[(size_t)g], gtimed[(size_t)g]);
    }
    DeviceGuard guard(d0.id);
    for (int g = 0; g < n; ++g) {
        const int nb = bands_of(height, band_rows, g, n);
        const int e = launch_scatter_bands(d0.d_gather + slot * g, dst, width, height, band_rows, g, n, nb, d0.stream);
        if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "scatter: %s", hipGetErrorString((hipError_t)e));
    }
    return RT_OK;
}
}  // namespace

// ============================================================================
// exported C ABI
// ============================================================================
extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_device_count(int* out_count) {
    if (!out_count) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL out_count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) n = 0;
    else if (e != hipSuccess) return fail(nullptr, RT_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    *out_count = n;
    return RT_OK;
}

const char* rt_last_error(const rt_ctx* ctx) {
    if (ctx) return ctx->last_error.c_str();
    return g_last_error.c_str();
}

int rt_create(int n_gpus, rt_ctx** out_ctx) { return rt_create_ex(n_gpus, 0, out_ctx); }

int rt_create_ex(int n_gpus, int flags, rt_ctx** out_ctx) {
    if (!out_ctx || n_gpus < 1 || n_gpus > RT_MAX_WORKERS ||
        (flags & ~(RT_CREATE_RCCL_GATHER | RT_CREATE_SHARED_DEVICE)) != 0 ||
        ((flags & RT_CREATE_RCCL_GATHER) && (flags & RT_CREATE_SHARED_DEVICE) && n_gpus > 1))
        return fail(nullptr, RT_ERR_INVALID_ARG, "rt_create: bad arguments");
    *out_ctx = nullptr;
    const bool shared = (flags & RT_CREATE_SHARED_DEVICE) != 0;
    int ndev = 0;
    if (rt_device_count(&ndev) != RT_OK || ndev == 0)
        return fail(nullptr, RT_ERR_NO_DEVICE, "no HIP device visible (libraytracer_hip has no CPU fallback)");
    if (n_gpus > ndev && !shared)
        return fail(nullptr, RT_ERR_NO_DEVICE, "rt_create(%d): only %d devices visible", n_gpus, ndev);
    rt_ctx* ctx = new (std::nothrow) rt_ctx();
    if (!ctx) return fail(nullptr, RT_ERR_OOM, "out of host memory");
    ctx->n_gpus = n_gpus;
    ctx->rccl_gather = (flags & RT_CREATE_RCCL_GATHER) != 0;
    ctx->shared_device = shared;
    // RT_DISPATCH_ORDER=0/1/2 fixes the single-frame dispatch order (order_pick; A/B and tests)
    if (const char* o = std::getenv("RT_DISPATCH_ORDER"))
        if (o[0] >= '0' && o[0] < '0' + ORDER_CANDIDATES && o[1] == 0) ctx->order_fixed = o[0] - '0';
    // rt_render_async keeps at most TICK_INFLIGHT frames per worker queued behind the copy engine: with more, one
    // hipMemcpyAsync of the hand-off now and then blocked the host for 6-7 ms (the runtime, not the copy: 5.4-7.0 ms
    // for an 8.3 MB copy that takes 160 us) -- a queued C3 run of 20 frames at 2.1-2.7k fps instead of 5.8k, in
    // runs 0 and 2 of 4 unbounded, 1 of 4 at 4, every run at 8, none at 2 or 3 (profiles/r06_tick_deep.txt).  The
    // double buffer needs no more than 2: frame k+2 is traced into frame k's buffer after frame k's copy anyway.
    // RT_TICK_INFLIGHT=0..16 overrides (0: no bound; A/B)
    ctx->tick_inflight = TICK_INFLIGHT;
    if (const char* q = std::getenv("RT_TICK_INFLIGHT")) ctx->tick_inflight = std::max(0, std::min(16, std::atoi(q)));
    ctx->dev.resize((size_t)n_gpus);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int g = 0; g < n_gpus; ++g) {
        Device& d = ctx->dev[(size_t)g];
        d.id = (n_gpus == 1 || shared) ? cur : g;  // one device: the caller's current one
        DeviceGuard guard(d.id);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d.id) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
            int rc = fail(ctx, RT_ERR_NO_DEVICE, "device %d is %s, this build targets gfx950", d.id, prop.gcnArchName);
            g_last_error = ctx->last_error;
            rt_destroy(ctx);
            return rc;
        }
        hipError_t e = hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipMalloc((void**)&d.d_counters, COUNTER_WORDS * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMemset(d.d_counters, 0, COUNTER_WORDS * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipDeviceSynchronize();  // kernels run on non-blocking streams
        if (e != hipSuccess) {
            int rc = fail(ctx, RT_ERR_HIP, "device %d init: %s", d.id, hipGetErrorString(e));
            g_last_error = ctx->last_error;
            rt_destroy(ctx);
            return rc;
        }
    }
    if (ctx->rccl_gather) {  // the gather's communicators now, so that a missing RCCL fails here
        const int rc = ensure_comm_all(ctx);
        if (rc != RT_OK) {
            g_last_error = ctx->last_error;
            rt_destroy(ctx);
            return rc;
        }
    }
    *out_ctx = ctx;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    (void)flush_hand(ctx);  // the last rt_render_async frame still reaches its (registered) buffer
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        (void)hipDeviceSynchronize();  // kernels on caller streams may still read our buffers
        for (EventPair& ep : d.pending) (void)hipEventDestroy(ep.a), (void)hipEventDestroy(ep.b);
        for (EventPair& ep : d.pool) (void)hipEventDestroy(ep.a), (void)hipEventDestroy(ep.b);
        for (auto* v : {&d.order.pending, &d.order.pool})
            for (Device::OrderTuner::Probe& pr : *v) (void)hipEventDestroy(pr.a), (void)hipEventDestroy(pr.b);
        if (d.ev_join) (void)hipEventDestroy(d.ev_join);
        for (hipEvent_t& ev : d.ev_chunk)
            if (ev) (void)hipEventDestroy(ev);
        for (int i = 0; i < 2; ++i) {
            if (d.ev_traced[i]) (void)hipEventDestroy(d.ev_traced[i]);
            if (d.ev_copied[i]) (void)hipEventDestroy(d.ev_copied[i]);
        }
        for (hipEvent_t& ev : d.ev_ring)
            if (ev) (void)hipEventDestroy(ev);
        if (d.copy_stream) (void)hipStreamDestroy(d.copy_stream);
        if (d.comm && g_rccl.CommDestroy) (void)g_rccl.CommDestroy(d.comm);
        if (d.d_scene) (void)hipFree(d.d_scene);
        if (d.d_frame) (void)hipFree(d.d_frame);
        if (d.d_bands) (void)hipFree(d.d_bands);
        if (d.d_gather) (void)hipFree(d.d_gather);
        for (int i = 0; i < 2; ++i)
            if (d.d_frames2[i]) (void)hipFree(d.d_frames2[i]);
        if (d.d_counters) (void)hipFree(d.d_counters);
        if (d.d_counters_diag) (void)hipFree(d.d_counters_diag);
        if (d.d_view_tab) (void)hipFree(d.d_view_tab);
        if (d.order.tiles.d_order) (void)hipFree(d.order.tiles.d_order);
        if (d.order.tiles.d_cost) (void)hipFree(d.order.tiles.d_cost);
        if (d.d_stage) (void)hipFree(d.d_stage);
        if (d.async_stream) (void)hipStreamDestroy(d.async_stream);
        if (d.stream) (void)hipStreamDestroy(d.stream);
    }
    delete ctx;
}

namespace {
// Light frame in double (the DevLight frame is its binary32 rounding).
struct Frame3 {
    double U[3], V[3], A[3];
};

// The lowest value x (double) that binary32 fma(x, s, o) can map to a value >= k (k integer): every
// x_f with floor(fl(x_f * s + o)) == k satisfies x_f >= cell_lo(k, s, o), and every x_f with that
// floor <= k - 1 satisfies x_f < cell_lo(k, s, o)... up to the allowance eps_k (a relative 2^-24 of
// the fma result plus double rounding here, taken 4x).  s > 0.
double cell_lo(int k, float s, float o) { return ((double)k - 0x1p-22 * (std::fabs((double)k) + 2.0) - (double)o) / (double)s; }
double cell_hi(int k, float s, float o) {  // the highest x that can map to k (exclusive bound of k + 1)
    return ((double)(k + 1) + 0x1p-22 * (std::fabs((double)k + 1.0) + 2.0) - (double)o) / (double)s;
}
float down(double v) { float f = (float)v; return (double)f > v ? std::nextafter(f, -INFINITY) : f; }
float up(double v) { float f = (float)v; return (double)f < v ? std::nextafter(f, INFINITY) : f; }

// The direct kernel's shadow pre-test records (rt_kernel.hip shadow_pre_keep; culling only).  The kernel drops
// sphere i for a lane's shadow ray toward light l only under shadow_sphere_cull's rules for a single ray (R = 0)
// from the lane's hit point O: w = C - O in the light's frame, margin 2^-8 dc + 2^-18 |O| with dc >= |C - O|,
// line miss if w_u^2 + w_v^2 > (r' + 2^-18 |C| + margin)^2, behind if -w_a > margin.  Here dc is bounded by
// |O_f|_1 + |C_f|_1 (frame coordinates), so the margin splits into a lane part m_l = 2^-8 (1 + 2^-8) |O_f|_1 +
// 2^-30 (kernel: it also covers the 2^-18 |O| projection allowance, and its 2^-30 floor makes every cull imply
// |C - O| > 2^-30) and a sphere part m_c = 2^-8 (1 + 2^-20) |C_f|_1, folded in here: ca' = ca + m_c and
// rr' = r' + 2^-18 |C| + m_c, both rounded up.  Records that allow no culling -- a light whose a = p.p is outside
// [2^-40, 2^40] or whose 2a is not finite, a sphere without a usable cull radius (NaN, < 2^-50), |C_f|_1 >= 2^38
// or non-finite -- get ca' = rr' = +inf (no rule can hold); the padding sphere of an odd count gets cu = +inf
// (always dropped: it never hits).
void build_shadow_pre(const DevLight* li, int n_lights, const DevSphereCull* cull, int n_spheres, int s_pad,
                      DevShadowCull* out) {
    for (int j = 0; j < n_lights; ++j) {
        const DevLight& d = li[j];
        const bool l_ok = d.a >= 0x1p-40f && d.a <= 0x1p40f && d.a2 > 0.0f && d.a2 < INFINITY;
        for (int i = 0; i < s_pad; ++i) {
            DevShadowCull& e = out[(size_t)j * (size_t)s_pad + (size_t)i];
            if (i >= n_spheres) {
                e = DevShadowCull{INFINITY, 0.0f, 0.0f, 0.0f};
                continue;
            }
            const double c[3] = {cull[i].cx, cull[i].cy, cull[i].cz};
            const double clen = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
            const double cu = c[0] * d.ux + c[1] * d.uy + c[2] * d.uz;
            const double cv = c[0] * d.vx + c[1] * d.vy + c[2] * d.vz;
            const double ca = c[0] * d.ax + c[1] * d.ay + c[2] * d.az;
            const double l1 = std::fabs((double)(float)cu) + std::fabs((double)(float)cv) + std::fabs((double)(float)ca);
            const double mc = 0x1p-8 * l1 * (1.0 + 0x1p-20);
            const bool ok = l_ok && cull[i].rr >= 0x1p-50f && l1 < 0x1p38 && std::isfinite(cull[i].rr) && std::isfinite(clen);
            if (!ok) {
                e = DevShadowCull{0.0f, 0.0f, INFINITY, INFINITY};
                continue;
            }
            e.cu = (float)cu;
            e.cv = (float)cv;
            e.ca = std::nextafter((float)((double)(float)ca + mc), INFINITY);
            e.rr = std::nextafter((float)((double)cull[i].rr + 0x1p-18 * clen + mc), INFINITY);
        }
    }
}

// Shadow grid of one light (DevShadowGrid; culling only -- a sphere left out of a lane's mask must
// provably not block that lane's shadow ray in binary32).  The argument (rt_kernel.hip cull_mask):
// IntersectsSphere yields disc < 0 when the exact line-to-centre distance D >= r (1 + 3 eps) +
// 9.2e-4 |u| (u = hp - C), and b >= 0 when (hp - C).A >= 4 eps |u|; either makes the ray unblocked.
// For a lane with |hp|_1 <= B: |u| <= |C|_1 + B, and its binary32 projections u_f = hp.U etc. are
// within 2^-21 |hp|_1 <= 2^-21 B of the exact ones in the double frame (U_f rounds U to 2^-24, three
// products and two sums round to 2^-24 each).  So, with T_j = r'_j + 2^-8 (|C_j|_1 + B) + 2^-20 B
// (r' >= r (1 + 2^-8) from DevSphereCull): a sphere whose centre lies farther than T_j from every
// (u, v) a lane of cell (iu, iv) can have -- the cell's interval from the device's own fma/floor
// mapping (cell_lo/cell_hi), grown by 2^-20 B -- has D > r (1 + 3 eps) + 2^-8 |u| (a 4x margin
// over 9.2e-4); cells outside the grid hold no such disc at all.  Axially, sphere j may be ahead of
// slab k only if ca_j + mB_j > a_lo(k), mB_j = 2^-8 (|C_j|_1 + B) + 2^-20 B; otherwise every lane in
// the slab has (hp - C).A >= 2^-8 (|C_j|_1 + B) >> 4 eps |u| (b >= 0).  Lanes beyond B: their own
// margin far_k |hp|_1 (far_k = 2^-8 + 2^-20, rounded up) on the box of all discs, and the slab of
// a_f - (far_k |hp|_1 - 2^-8 B), which raises the slab rule's margin from B to |hp|_1.  Spheres
// without a valid record (NaN/inf, r^2 < 2^-100, |C|_1 >= 2^30) are never culled (`always`); a
// light whose |p|^2 lies outside [2^-40, 2^40] (the analysis' range) culls nothing.
// The bundle kernel's sphere clusters (rt_internal.h DevCluster): median splits of the sphere centres along the
// widest axis of their box until a group holds at most `size` spheres; each cluster's centre is the middle of
// its members' box (rounded to float) and R, computed in double from that rounded centre and rounded up, bounds
// |c_i - centre| + r'_i for every member (r' = the DevSphereCull radius, itself >= r (1 + 2^-8)).  A member
// without a usable cull record (NaN / infinite centre or radius) makes its cluster's R NaN: never culled.
// Returns the cluster count (<= MAX_CLUSTERS).
int build_clusters(const DevSphereCull* cull, int S, int size, DevCluster* out) {
    std::vector<std::vector<int>> todo(1, std::vector<int>((size_t)S)), groups;
    for (int i = 0; i < S; ++i) todo[0][(size_t)i] = i;
    while (!todo.empty()) {
        std::vector<int> g = std::move(todo.back());
        todo.pop_back();
        if ((int)g.size() <= size) {
            groups.push_back(std::move(g));
            continue;
        }
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i : g) {
            const double c[3] = {cull[i].cx, cull[i].cy, cull[i].cz};
            for (int k = 0; k < 3; ++k) lo[k] = std::fmin(lo[k], c[k]), hi[k] = std::fmax(hi[k], c[k]);
        }
        int ax = 0;
        for (int k = 1; k < 3; ++k)
            if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
        auto key = [&](int i) {  // (NaN last: a strict weak order for the sort)
            const float k = ax == 0 ? cull[i].cx : ax == 1 ? cull[i].cy : cull[i].cz;
            return std::isnan(k) ? INFINITY : k;
        };
        std::stable_sort(g.begin(), g.end(), [&](int a, int b) { return key(a) < key(b); });
        const size_t h = g.size() / 2;
        todo.emplace_back(g.begin(), g.begin() + (long)h);
        todo.emplace_back(g.begin() + (long)h, g.end());
    }
    if ((int)groups.size() > MAX_CLUSTERS) return 0;
    int n = 0;
    for (const std::vector<int>& g : groups) {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool usable = true;
        unsigned long long m = 0;
        for (int i : g) {
            const double c[3] = {cull[i].cx, cull[i].cy, cull[i].cz};
            for (int k = 0; k < 3; ++k) lo[k] = std::fmin(lo[k], c[k]), hi[k] = std::fmax(hi[k], c[k]);
            usable = usable && std::isfinite(c[0]) && std::isfinite(c[1]) && std::isfinite(c[2]) &&
                     std::isfinite((double)cull[i].rr) && cull[i].rr >= 0x1p-50f;
            m |= 1ull << i;
        }
        DevCluster& c = out[n++];
        c.cx = (float)((lo[0] + hi[0]) / 2), c.cy = (float)((lo[1] + hi[1]) / 2), c.cz = (float)((lo[2] + hi[2]) / 2);
        double R = 0;
        for (int i : g) {
            const double dx = (double)cull[i].cx - c.cx, dy = (double)cull[i].cy - c.cy, dz = (double)cull[i].cz - c.cz;
            R = std::fmax(R, std::sqrt(dx * dx + dy * dy + dz * dz) + (double)cull[i].rr);
        }
        c.R = usable && R < 0x1p40 ? std::nextafter((float)(R * (1.0 + 0x1p-20)), INFINITY) : NAN;
        c.members = m;
        c.pad = 0;
    }
    return n;
}

void build_shadow_grid(const DevLight& l, const Frame3& f, const DevSphere* sph, const DevSphereCull* cull, int S,
                       DevShadowGrid& g, unsigned long long* grid, unsigned long long* slab) {
    std::memset(&g, 0, sizeof g);
    std::memset(grid, 0, sizeof(unsigned long long) * SHGRID_N * SHGRID_N);
    std::memset(slab, 0, sizeof(unsigned long long) * (SHGRID_SLABS + 2));
    const unsigned long long all = S >= 64 ? ~0ull : ((1ull << S) - 1ull);
    g.bu0 = g.bv0 = INFINITY, g.bu1 = g.bv1 = -INFINITY;  // empty box: every far lane outside
    const bool light_ok = l.a >= 0x1p-40f && l.a <= 0x1p40f && l.a2 < INFINITY;
    std::vector<double> cu(S), cv(S), ca(S), c1(S), rr(S);
    std::vector<bool> ok(S);
    double cmax1 = 0.0;
    for (int j = 0; j < S; ++j) {
        const double c[3] = {sph[j].cx, sph[j].cy, sph[j].cz};
        c1[j] = std::fabs(c[0]) + std::fabs(c[1]) + std::fabs(c[2]);
        rr[j] = cull[j].rr;
        ok[j] = light_ok && std::isfinite(c1[j]) && c1[j] < 0x1p30 && std::isfinite(rr[j]) &&
                (double)sph[j].r2 >= 0x1p-100 && rr[j] > 0.0;
        if (!ok[j]) {
            g.always |= 1ull << j;
            continue;
        }
        cu[j] = c[0] * f.U[0] + c[1] * f.U[1] + c[2] * f.U[2];
        cv[j] = c[0] * f.V[0] + c[1] * f.V[1] + c[2] * f.V[2];
        ca[j] = c[0] * f.A[0] + c[1] * f.A[1] + c[2] * f.A[2];
        cmax1 = std::max(cmax1, c1[j]);
    }
    if (g.always == all) {  // nothing to cull: no lane looks anything up that matters
        g.bound = -1.0f;    // every lane "far"
        g.far_k = 0.0f;
        return;
    }
    const double B = std::min(std::max(8.0, 1.5 * cmax1), 0x1p30);
    g.bound = down(B);
    g.far_k = up(0x1p-8 + 0x1p-20);
    g.far_b = down(0x1p-8 * B);
    double ulo = INFINITY, uhi = -INFINITY, vlo = INFINITY, vhi = -INFINITY, alo = INFINITY, ahi = -INFINITY;
    double bu0 = INFINITY, bu1 = -INFINITY, bv0 = INFINITY, bv1 = -INFINITY;
    std::vector<double> T(S), mB(S);
    for (int j = 0; j < S; ++j) {
        if (!ok[j]) continue;
        T[j] = rr[j] + 0x1p-8 * (c1[j] + B) + 0x1p-20 * B;
        mB[j] = 0x1p-8 * (c1[j] + B) + 0x1p-20 * B;
        ulo = std::min(ulo, cu[j] - T[j]), uhi = std::max(uhi, cu[j] + T[j]);
        vlo = std::min(vlo, cv[j] - T[j]), vhi = std::max(vhi, cv[j] + T[j]);
        alo = std::min(alo, ca[j] + mB[j]), ahi = std::max(ahi, ca[j] + mB[j]);
        const double t0 = rr[j] + 0x1p-8 * c1[j];  // far lanes add their own |hp| term
        bu0 = std::min(bu0, cu[j] - t0), bu1 = std::max(bu1, cu[j] + t0);
        bv0 = std::min(bv0, cv[j] - t0), bv1 = std::max(bv1, cv[j] + t0);
    }
    g.bu0 = down(bu0), g.bu1 = up(bu1), g.bv0 = down(bv0), g.bv1 = up(bv1);
    // grid over [lo, hi] padded by half a cell (lanes mapped outside it see no disc: checked below)
    auto axis = [](double lo, double hi, int n, float& s, float& o) {
        const double cs = (hi - lo) / (n - 1);  // n - 1 cells span the range, half a cell of pad each side
        const double lo2 = lo - 0.5 * cs;
        s = (float)(1.0 / cs);
        o = (float)(-lo2 * (double)s);
    };
    axis(ulo, uhi, SHGRID_N, g.su, g.ou);
    axis(vlo, vhi, SHGRID_N, g.sv, g.ov);
    bool sound = g.su > 0.0f && g.sv > 0.0f && std::isfinite(g.su) && std::isfinite(g.sv) && std::isfinite(g.ou) &&
                 std::isfinite(g.ov);
    // a lane mapped below cell 0 / above cell N-1 lies outside every disc
    sound = sound && cell_hi(-1, g.su, g.ou) + 0x1p-20 * B < ulo && cell_lo(SHGRID_N, g.su, g.ou) - 0x1p-20 * B > uhi &&
            cell_hi(-1, g.sv, g.ov) + 0x1p-20 * B < vlo && cell_lo(SHGRID_N, g.sv, g.ov) - 0x1p-20 * B > vhi;
    if (sound) {
        for (int iv = 0; iv < SHGRID_N; ++iv) {
            const double v0 = cell_lo(iv, g.sv, g.ov) - 0x1p-20 * B, v1 = cell_hi(iv, g.sv, g.ov) + 0x1p-20 * B;
            for (int iu = 0; iu < SHGRID_N; ++iu) {
                const double u0 = cell_lo(iu, g.su, g.ou) - 0x1p-20 * B, u1 = cell_hi(iu, g.su, g.ou) + 0x1p-20 * B;
                unsigned long long m = 0;
                for (int j = 0; j < S; ++j) {
                    if (!ok[j]) continue;
                    const double du = std::max(0.0, std::max(u0 - cu[j], cu[j] - u1));
                    const double dv = std::max(0.0, std::max(v0 - cv[j], cv[j] - v1));
                    if (du * du + dv * dv <= T[j] * T[j] * (1.0 + 0x1p-30)) m |= 1ull << j;
                }
                grid[iv * SHGRID_N + iu] = m;
            }
        }
    } else {  // (degenerate extents) every lane takes every sphere through the far path
        g.bound = -1.0f;
        g.bu0 = -INFINITY, g.bu1 = INFINITY, g.bv0 = -INFINITY, g.bv1 = INFINITY;
    }
    // axial slabs over [alo, ahi]: entry k + 1 for slab k (-1: below the range, every sphere)
    {
        const double cs = std::max((ahi - alo) / SHGRID_SLABS, 1e-30);
        g.sa = (float)(1.0 / cs);
        g.oa = (float)(-alo * (double)g.sa);
        const bool sa_ok = g.sa > 0.0f && std::isfinite(g.sa) && std::isfinite(g.oa);
        slab[0] = all;
        for (int k = 0; k <= SHGRID_SLABS; ++k) {
            const double a_lo = sa_ok ? cell_lo(k, g.sa, g.oa) : -INFINITY;
            unsigned long long m = 0;
            for (int j = 0; j < S; ++j)
                if (ok[j] && ca[j] + mB[j] > a_lo) m |= 1ull << j;
            slab[k + 1] = m;
        }
        if (!sa_ok) g.sa = 0.0f, g.oa = 0.0f;  // every lane in slab 0 (= every valid sphere)
    }
}
}  // namespace

int rt_set_scene(rt_ctx* ctx, const rt_sphere* spheres, int n_spheres, const rt_plane* planes, int n_planes,
                 const rt_light* lights, int n_lights, rt_vec3 ambient, int recursion_limit) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    if (n_spheres < 0 || n_planes < 0 || n_lights < 0 || (n_spheres && !spheres) || (n_planes && !planes) ||
        (n_lights && !lights))
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_scene: bad primitive arrays");
    if (recursion_limit < 0) return fail(ctx, RT_ERR_INVALID_ARG, "recursion_limit must be >= 0");
    if (n_lights > RT_MAX_LIGHTS)
        return fail(ctx, RT_ERR_UNSUPPORTED, "n_lights %d > RT_MAX_LIGHTS (%d)", n_lights, RT_MAX_LIGHTS);
    if (recursion_limit > RT_MAX_RECURSION_LIMIT)
        return fail(ctx, RT_ERR_UNSUPPORTED, "recursion_limit %d > RT_MAX_RECURSION_LIMIT (%d)", recursion_limit,
                    RT_MAX_RECURSION_LIMIT);

    SceneLayout L;
    L.S = n_spheres, L.P = n_planes, L.L = n_lights, L.limit = recursion_limit;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    // the sphere table is padded to an even count (the direct kernel's loops take spheres in
    // pairs) with a sphere that never hits: NaN centre and radius^2 make every comparison of
    // IntersectsSphere false (no candidate, t = 0, no shadow)
    const int s_pad = n_spheres + (n_spheres & 1);
    L.off_sph = 0;
    L.off_mat = al(L.off_sph + sizeof(DevSphere) * (size_t)s_pad);
    L.off_pl = al(L.off_mat + sizeof(DevMaterial) * (size_t)(n_spheres + n_planes));
    L.off_li = al(L.off_pl + sizeof(DevPlane) * (size_t)n_planes);
    L.off_cull = al(L.off_li + sizeof(DevLight) * (size_t)n_lights);
    L.off_shcull = al(L.off_cull + sizeof(DevSphereCull) * (size_t)n_spheres);
    L.has_shcull = (long long)n_lights * (long long)n_spheres <= SHADOW_CULL_MAX_ENTRIES;
    // shadow grids: the bundle kernel's merged pass only (CULL_MIN_SPHERES <= S <= 64, 1 <= L <=
    // SHADOW_MERGE_L); RT_SHADOW_GRID=0 keeps the per-level bound (A/B and fallback tests)
    const char* gv = std::getenv("RT_SHADOW_GRID");
    L.has_shg = n_spheres >= CULL_MIN_SPHERES && n_spheres <= 64 && n_lights >= 1 && n_lights <= SHADOW_MERGE_L &&
                !(gv && std::strcmp(gv, "0") == 0);
    L.off_shg = al(L.off_shcull + (L.has_shcull ? sizeof(DevShadowCull) * (size_t)n_lights * (size_t)n_spheres : 0));
    L.off_shgrid = al(L.off_shg + (L.has_shg ? sizeof(DevShadowGrid) * (size_t)n_lights : 0));
    L.off_shslab = al(L.off_shgrid + (L.has_shg ? sizeof(unsigned long long) * SHGRID_N * SHGRID_N * (size_t)n_lights : 0));
    L.off_clus = al(L.off_shslab + (L.has_shg ? sizeof(unsigned long long) * (SHGRID_SLABS + 2) * (size_t)n_lights : 0));
    // per-lane cluster pre-cull of the bundle kernel's trace bundles (CULL_MIN_SPHERES <= S <= 64);
    // RT_TRACE_CLUSTERS=0 turns it off, =2..16 sets the cluster size (A/B)
    int csize = CLUSTER_SIZE;
    if (const char* cv = std::getenv("RT_TRACE_CLUSTERS")) csize = std::atoi(cv);
    const bool want_clus = n_spheres >= CULL_MIN_SPHERES && n_spheres <= 64 && csize >= 1;
    L.off_shpre = al(L.off_clus + (want_clus ? sizeof(DevCluster) * MAX_CLUSTERS : 0));
    // the direct kernel's shadow pre-test (S < CULL_MIN_SPHERES); RT_SHADOW_PRE=0 turns it off (A/B)
    const char* pv = std::getenv("RT_SHADOW_PRE");
    L.has_shpre = n_spheres < CULL_MIN_SPHERES && n_lights >= 1 && !(pv && std::strcmp(pv, "0") == 0);
    L.bytes = al(L.off_shpre + (L.has_shpre ? sizeof(DevShadowCull) * (size_t)n_lights * (size_t)s_pad : 0)) + 256;

    std::vector<unsigned char> blob(L.bytes, 0);
    DevSphere* sph = (DevSphere*)(blob.data() + L.off_sph);
    DevMaterial* mat = (DevMaterial*)(blob.data() + L.off_mat);
    DevPlane* pl = (DevPlane*)(blob.data() + L.off_pl);
    DevLight* li = (DevLight*)(blob.data() + L.off_li);
    DevSphereCull* cull = (DevSphereCull*)(blob.data() + L.off_cull);
    for (int i = 0; i < n_spheres; ++i) {
        const rt_sphere& s = spheres[i];
        sph[i] = DevSphere{s.center.x, s.center.y, s.center.z, s.radius * s.radius};  // :336
        mat[i] = dev_material(s.material, ambient);
        // cull radius: an upper bound of sqrt(r^2) (1 + 2^-8), rounded up (NaN stays NaN)
        const double rr = std::sqrt((double)sph[i].r2) * (1.0 + 0x1p-8);
        cull[i] = DevSphereCull{sph[i].cx, sph[i].cy, sph[i].cz, std::nextafter((float)rr, INFINITY)};
    }
    for (int i = n_spheres; i < s_pad; ++i) sph[i] = DevSphere{NAN, NAN, NAN, NAN};
    L.host_sph.assign(sph, sph + n_spheres);
    for (int i = 0; i < n_planes; ++i) {
        const rt_plane& p = planes[i];
        const H3 n = h3(p.normal);
        DevPlane d;
        std::memset(&d, 0, sizeof d);
        d.cx = p.center.x, d.cy = p.center.y, d.cz = p.center.z;
        d.cn = hdot(h3(p.center), n);  // Vector3.Dot(plane.center, plane.normal), :594
        d.nx = n.x, d.ny = n.y, d.nz = n.z;
        H3 e1 = hnormalize(hcross(n, H3{1.0f, 0.0f, 0.0f}));  // :760-763
        if (e1.x == 0 && e1.y == 0 && e1.z == 0) e1 = hnormalize(hcross(n, H3{0.0f, 0.0f, 1.0f}));
        H3 e2 = hnormalize(hcross(n, e1));  // :765
        d.e1x = e1.x, d.e1y = e1.y, d.e1z = e1.z;
        d.e2x = e2.x, d.e2y = e2.y, d.e2z = e2.z;
        pl[i] = d;
        mat[n_spheres + i] = dev_material(p.material, ambient);
    }
    L.host_pl.assign(pl, pl + n_planes);
    std::vector<Frame3> frames((size_t)n_lights);
    for (int i = 0; i < n_lights; ++i) {
        const rt_light& l = lights[i];
        const H3 p = h3(l.position);
        DevLight d;
        std::memset(&d, 0, sizeof d);
        d.px = p.x, d.py = p.y, d.pz = p.z, d.intensity = l.intensity;
        d.a = hdot(p, p);  // IntersectsSphere's a = Dot(direction, direction), :617
        d.a2 = 2.0f * d.a;
        d.a4 = 4.0f * d.a;
        d.sh_t = shadow_threshold(d.a2);  // used only when a2 is finite and > 0 (wave-uniform per light)
        if (!(d.a2 > 0.0f && d.a2 < INFINITY)) L.lights_a2_ok = false;
        // shadow-cull frame (kernel uses it only when a is in [2^-40, 2^40])
        const double len = std::sqrt((double)p.x * p.x + (double)p.y * p.y + (double)p.z * p.z);
        double A[3] = {0.0, 0.0, 1.0};
        if (len > 0 && std::isfinite(len)) A[0] = p.x / len, A[1] = p.y / len, A[2] = p.z / len;
        const double h[3] = {std::fabs(A[0]) < 0.9 ? 1.0 : 0.0, std::fabs(A[0]) < 0.9 ? 0.0 : 1.0, 0.0};
        double U[3] = {A[1] * h[2] - A[2] * h[1], A[2] * h[0] - A[0] * h[2], A[0] * h[1] - A[1] * h[0]};
        const double ul = std::sqrt(U[0] * U[0] + U[1] * U[1] + U[2] * U[2]);
        for (double& c : U) c /= ul;
        const double V[3] = {A[1] * U[2] - A[2] * U[1], A[2] * U[0] - A[0] * U[2], A[0] * U[1] - A[1] * U[0]};
        d.ax = (float)A[0], d.ay = (float)A[1], d.az = (float)A[2];
        d.ux = (float)U[0], d.uy = (float)U[1], d.uz = (float)U[2];
        d.vx = (float)V[0], d.vy = (float)V[1], d.vz = (float)V[2];
        li[i] = d;
        for (int k = 0; k < 3; ++k) frames[(size_t)i].U[k] = U[k], frames[(size_t)i].V[k] = V[k], frames[(size_t)i].A[k] = A[k];
    }
    if (L.has_shg)
        for (int j = 0; j < n_lights; ++j)
            build_shadow_grid(li[j], frames[(size_t)j], sph, cull, n_spheres, ((DevShadowGrid*)(blob.data() + L.off_shg))[j],
                              (unsigned long long*)(blob.data() + L.off_shgrid) + (size_t)j * SHGRID_N * SHGRID_N,
                              (unsigned long long*)(blob.data() + L.off_shslab) + (size_t)j * (SHGRID_SLABS + 2));
    if (want_clus) L.n_clus = build_clusters(cull, n_spheres, csize, (DevCluster*)(blob.data() + L.off_clus));
    if (L.has_shcull) {  // sphere centres in each light's shadow-cull frame (culling only)
        DevShadowCull* sc = (DevShadowCull*)(blob.data() + L.off_shcull);
        for (int j = 0; j < n_lights; ++j)
            for (int i = 0; i < n_spheres; ++i) {
                const DevLight& d = li[j];
                const double c[3] = {cull[i].cx, cull[i].cy, cull[i].cz};
                const double clen = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
                DevShadowCull& e = sc[(size_t)j * (size_t)n_spheres + (size_t)i];
                e.cu = (float)(c[0] * d.ux + c[1] * d.uy + c[2] * d.uz);
                e.cv = (float)(c[0] * d.vx + c[1] * d.vy + c[2] * d.vz);
                e.ca = (float)(c[0] * d.ax + c[1] * d.ay + c[2] * d.az);
                // r' + 2^-18 |C|, rounded up (NaN / inf stay: the kernel keeps such spheres)
                e.rr = std::nextafter((float)((double)cull[i].rr + 0x1p-18 * clen), INFINITY);
            }
    }
    if (L.has_shpre) build_shadow_pre(li, n_lights, cull, n_spheres, s_pad, (DevShadowCull*)(blob.data() + L.off_shpre));
    for (int i = 0; i < n_spheres + n_planes; ++i)
        if ((mat[i].flags & MAT_SPEC) && mat[i].pow_kind == POW_GENERIC) L.generic_pow = true;
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        // frames in flight on any stream (rt_render_device callers', the async slots) read
        // the scene being replaced
        HIP_TRY(ctx, hipDeviceSynchronize());
        int rc = grow(ctx, &d.d_scene, &d.scene_cap, L.bytes);
        if (rc != RT_OK) return rc;
        HIP_TRY(ctx, hipMemcpy(d.d_scene, blob.data(), L.bytes, hipMemcpyHostToDevice));
    }
    L.host_blob = std::move(blob);
    ctx->layout = std::move(L);
    ctx->has_scene = true;
    ctx->view_ok = false;
    ctx->scene_gen++;
    return RT_OK;
}

int rt_set_view_height(rt_ctx* ctx, int view_height) {
    if (!ctx || view_height < 0) return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_view_height: bad arguments");
    ctx->view_height = view_height;
    return RT_OK;
}

int rt_set_camera(rt_ctx* ctx, const rt_camera* camera) {
    if (!ctx || !camera) return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_camera: NULL argument");
    ctx->cam = *camera;
    return RT_OK;
}

int rt_get_camera(const rt_ctx* ctx, rt_camera* camera) {
    if (!ctx || !camera) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_get_camera: NULL argument");
    *camera = ctx->cam;
    return RT_OK;
}

// CameraForwardDirection / CameraRightDirection / CameraUpDirection (RayTracer.cs:511-523):
// double trig of the float yaw/pitch, each component cast to float; Up = Cross(Right, Fwd).
// View params (Tick, :892-896): planeHeight = 0.3f * (float)Math.Tan(30f * (MathF.PI/180f)) * 2,
// planeWidth = planeHeight * ((float)width / height).
int rt_camera_view(const rt_camera* c, int width, int height, rt_view* out) {
    if (!c || !out || width <= 0 || height <= 0) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_camera_view: bad args");
    const double p = (double)c->pitch, y = (double)c->yaw;
    const H3 f{(float)(std::cos(p) * std::sin(y)), (float)-std::sin(p), (float)(std::cos(p) * std::cos(y))};
    const H3 r{(float)std::cos(y), 0.0f, (float)-std::sin(y)};
    const H3 u = hcross(r, f);
    out->position = c->position;
    out->right = rt_vec3{r.x, r.y, r.z};
    out->up = rt_vec3{u.x, u.y, u.z};
    out->forward = rt_vec3{f.x, f.y, f.z};
    const float near_clip = 0.3f, fov = 60.0f;
    const float deg2rad = (float)M_PI / 180.0f;  // MathHelper.DegreesToRadians: d * (MathF.PI / 180f)
    const float rad = (fov * 0.5f) * deg2rad;
    const float plane_height = near_clip * (float)std::tan((double)rad) * 2;
    const float aspect = (float)width / (float)height;
    out->plane_width = plane_height * aspect;
    out->plane_height = plane_height;
    out->near_clip = near_clip;
    return RT_OK;
}

// OnKeyPress, RayTracer.cs:543-554: position +/- direction * (0.05, 0.05, 0.05).
int rt_camera_on_key(rt_camera* c, int key) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_camera_on_key: NULL camera");
    rt_view v;
    rt_camera_view(c, 1, 1, &v);
    const float m = 0.05f;
    rt_vec3 dir;
    float sign;
    switch (key) {
        case RT_KEY_W: dir = v.forward, sign = 1.0f; break;
        case RT_KEY_A: dir = v.right, sign = -1.0f; break;
        case RT_KEY_S: dir = v.forward, sign = -1.0f; break;
        case RT_KEY_D: dir = v.right, sign = 1.0f; break;
        case RT_KEY_SPACE: dir = v.up, sign = -1.0f; break;
        case RT_KEY_SHIFT: dir = v.up, sign = 1.0f; break;
        default: return RT_OK;  // `_ => _cameraPosition`
    }
    const rt_vec3 d{dir.x * m, dir.y * m, dir.z * m};
    if (sign > 0) c->position = rt_vec3{c->position.x + d.x, c->position.y + d.y, c->position.z + d.z};
    else c->position = rt_vec3{c->position.x - d.x, c->position.y - d.y, c->position.z - d.z};
    return RT_OK;
}

// OnMouseMove, RayTracer.cs:1058-1061: _yaw += DeltaX / 360; _pitch += DeltaY / 360.
int rt_camera_on_mouse_move(rt_camera* c, float dx, float dy) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_camera_on_mouse_move: NULL camera");
    c->yaw = c->yaw + dx / 360.0f;
    c->pitch = c->pitch + dy / 360.0f;
    return RT_OK;
}

int rt_render_device(rt_ctx* ctx, int width, int height, int32_t* d_pixels, void* hip_stream) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (!d_pixels) return fail(ctx, RT_ERR_INVALID_ARG, "NULL d_pixels");
    Device& d0 = ctx->dev[0];
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the HIP null stream
    if (ctx->n_gpus == 1 && !ctx->rccl_gather) {
        DeviceGuard guard(d0.id);
        rc = trace_bands(ctx, d0, s, width, height, height, 0, 1, d_pixels, nullptr);
    } else {
        // n > 1: the workers start after the work already on the caller's stream (d_pixels may be in use)
        // and the caller's stream waits for the whole frame
        for (Device& d : ctx->dev)
            if (!d.ev_join) {
                DeviceGuard guard(d.id);
                HIP_TRY(ctx, hipEventCreateWithFlags(&d.ev_join, hipEventDisableTiming));
            }
        {
            DeviceGuard guard(d0.id);
            HIP_TRY(ctx, hipEventRecord(d0.ev_join, s));
        }
        for (Device& d : ctx->dev) {
            DeviceGuard guard(d.id);
            HIP_TRY(ctx, hipStreamWaitEvent(d.stream, d0.ev_join, 0));
        }
        if (ctx->shared_device) {  // one device: every worker writes its bands straight into the frame
            for (int g = 0; g < ctx->n_gpus && rc == RT_OK; ++g)
                rc = trace_bands(ctx, ctx->dev[(size_t)g], ctx->dev[(size_t)g].stream, width, height, TICK_BAND_ROWS,
                                 g, ctx->n_gpus, d_pixels, nullptr, RT_BANDS_FRAME);
        } else {  // the RCCL gather to device 0 over xGMI, reassembled into d_pixels on device 0's stream
            rc = gather_frame(ctx, width, height, d_pixels);
        }
        if (rc != RT_OK) return rc;
        DeviceGuard guard(d0.id);
        for (size_t g = 0; g < (ctx->shared_device ? ctx->dev.size() : 1); ++g) {
            HIP_TRY(ctx, hipEventRecord(ctx->dev[g].ev_join, ctx->dev[g].stream));
            HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->dev[g].ev_join, 0));
        }
    }
    if (rc == RT_OK) {
        ctx->frames++;
        ctx->pixels += (uint64_t)width * (uint64_t)height;
    }
    return rc;
}

int rt_render_bands(rt_ctx* ctx, int width, int height, int band_rows, int band_first, int band_step,
                    int32_t* d_out, void* hip_stream, int* out_n_bands) {
    return rt_render_bands_ex(ctx, width, height, band_rows, band_first, band_step, d_out, RT_BANDS_INT32, hip_stream,
                              out_n_bands);
}

int rt_render_bands_ex(rt_ctx* ctx, int width, int height, int band_rows, int band_first, int band_step, void* d_out,
                       int format, void* hip_stream, int* out_n_bands) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (band_rows <= 0 || band_first < 0 || band_step <= 0 || !d_out ||
        (format != RT_BANDS_INT32 && format != RT_BANDS_RGB24 && format != RT_BANDS_FRAME))
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands: bad band arguments");
    if (ctx->n_gpus != 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands needs a single-GPU context");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the HIP null stream
    int nb = 0;
    rc = trace_bands(ctx, d, s, width, height, band_rows, band_first, band_step, (int32_t*)d_out, &nb, format);
    if (out_n_bands) *out_n_bands = nb;
    if (rc == RT_OK) ctx->pixels += (uint64_t)nb * band_rows * width;
    return rc;
}

int rt_render_bands_batch(rt_ctx* ctx, int width, int height, int band_rows, int band_first, int band_step,
                          int n_frames, void* d_out, size_t frame_stride_bytes, int format, void* hip_stream,
                          int* out_n_bands) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (band_rows <= 0 || band_first < 0 || band_step <= 0 || !d_out || n_frames <= 0 || n_frames > 65535 ||
        (format != RT_BANDS_INT32 && format != RT_BANDS_RGB24 && format != RT_BANDS_FRAME))
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands_batch: bad band arguments");
    if (ctx->n_gpus != 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands_batch needs a single-GPU context");
    const int nb = bands_of(height, band_rows, band_first, band_step);
    const size_t need = format == RT_BANDS_FRAME ? (size_t)width * height * 4
                                                 : (size_t)nb * band_rows * width * (format == RT_BANDS_RGB24 ? 3 : 4);
    if (n_frames > 1 && frame_stride_bytes < need)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands_batch: frame stride smaller than a frame's output");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    rc = trace_bands(ctx, d, (hipStream_t)hip_stream, width, height, band_rows, band_first, band_step, (int32_t*)d_out,
                     nullptr, format, n_frames, frame_stride_bytes);
    if (out_n_bands) *out_n_bands = nb;
    if (rc == RT_OK) ctx->pixels += (uint64_t)nb * band_rows * width * (uint64_t)n_frames;
    return rc;
}

int rt_scatter_bands(rt_ctx* ctx, int width, int height, int band_rows, int band_first, int band_step,
                     const int32_t* d_bands, int32_t* d_frame, void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    if (width <= 0 || height <= 0 || band_rows <= 0 || band_first < 0 || band_step <= 0 || !d_bands || !d_frame)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_scatter_bands: bad arguments");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    hipStream_t s = (hipStream_t)hip_stream;  // NULL = the HIP null stream
    const int nb = bands_of(height, band_rows, band_first, band_step);
    int e = launch_scatter_bands(d_bands, d_frame, width, height, band_rows, band_first, band_step, nb, s);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "scatter launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int rt_scatter_gathered(rt_ctx* ctx, int width, int height, int band_rows, int world, const void* d_gathered,
                        size_t slot_bytes, int format, int32_t* d_frame, void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    const size_t bpp = format == RT_BANDS_INT32 ? 4 : 3;
    if (width <= 0 || height <= 0 || band_rows <= 0 || world <= 0 || !d_gathered || !d_frame ||
        (format != RT_BANDS_INT32 && format != RT_BANDS_RGB24) ||
        slot_bytes < (size_t)bands_of(height, band_rows, 0, world) * band_rows * width * bpp)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_scatter_gathered: bad arguments");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    int e = launch_scatter_gathered((const unsigned char*)d_gathered, slot_bytes, format, d_frame, width, height,
                                    band_rows, world, hip_stream);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "scatter launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

// Tile-codec wire geometry (raytracer_hip/tilecodec.py.layout): the tile grid of the
// largest band set, n_frames grids per batch, chunks of 64 tiles.
static bool codec_geom(int width, int height, int band_rows, int world, int n_frames, rtk::CodecGeom& g,
                       rt_wire_layout* lay) {
    if (width <= 0 || height <= 0 || band_rows <= 0 || world <= 0 || n_frames <= 0) return false;
    const int rows = std::max(1, bands_of(height, band_rows, 0, world)) * band_rows;
    const long long tx = (width + 7) / 8, ty = (rows + 7) / 8;
    const long long tpf = tx * ty, nt = tpf * (long long)n_frames;
    if (nt > (1LL << 26)) return false;  // 32-bit word offsets (<= 48 words per tile)
    const long long nc = (nt + 7) / 8;  // chunks of 8 tiles (one wave's)
    g = rtk::CodecGeom{};
    g.W = width, g.H = height, g.band_rows = band_rows, g.world = world;
    g.tiles_x = (int)tx, g.tiles_y = (int)ty, g.tiles_per_frame = (int)tpf, g.n_tiles = (int)nt, g.n_chunks = (int)nc;
    g.fixed_bytes = ((size_t)16 + 4 * (size_t)nt + 4 * (size_t)nc + 7) / 8 * 8;  // header, tile headers, chunk bases
    if (lay) {
        lay->fixed_bytes = g.fixed_bytes;
        lay->max_bytes = g.fixed_bytes + 8 * 24 * (size_t)nt;
        lay->tiles_x = (int32_t)tx, lay->tiles_y = (int32_t)ty, lay->tiles_per_frame = (int32_t)tpf;
        lay->n_frames = n_frames, lay->n_tiles = (int32_t)nt, lay->n_chunks = (int32_t)nc;
    }
    return true;
}

// Codec scratch of device d for geometry g (staged segments + workgroup sums), grown on demand:
// the previous user of the old buffer may still run, so growing waits for the device first.
static int ensure_stage(rt_ctx* ctx, Device& d, const rtk::CodecGeom& g) {
    const size_t need = encode_stage_bytes(g);
    if (need > d.stage_cap) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (d.d_stage) HIP_TRY(ctx, hipFree(d.d_stage));
        d.d_stage = nullptr, d.stage_cap = 0;
        HIP_TRY(ctx, hipMalloc(&d.d_stage, need));
        d.stage_cap = need;
    }
    return RT_OK;
}

int rt_wire_layout_of(int width, int height, int band_rows, int world, int n_frames, rt_wire_layout* out) {
    rtk::CodecGeom g;
    if (!out || !codec_geom(width, height, band_rows, world, n_frames, g, out))
        return fail(nullptr, RT_ERR_INVALID_ARG, "rt_wire_layout_of: bad arguments");
    return RT_OK;
}

int rt_encode_bands(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world, const int32_t* d_bands,
                    size_t frame_stride, int n_frames, void* d_wire, int64_t* d_wire_bytes, void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    rtk::CodecGeom g;
    if (!codec_geom(width, height, band_rows, world, n_frames, g, nullptr) || rank < 0 || rank >= world ||
        !d_bands || !d_wire || ((uintptr_t)d_wire & 7) != 0 ||
        frame_stride < (size_t)std::max(1, bands_of(height, band_rows, 0, world)) * band_rows * width)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_encode_bands: bad arguments");
    g.rank = rank;
    g.n_bands = bands_of(height, band_rows, rank, world);
    g.frame_stride = frame_stride;
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    const int rc = ensure_stage(ctx, d, g);
    if (rc != RT_OK) return rc;
    d.staged.valid = false;  // the scratch now holds this encode's segments
    int e = launch_encode_bands(d_bands, (unsigned char*)d_wire, g, d_wire_bytes, d.d_stage, hip_stream);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "encode launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int rt_render_bands_tiles(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world, int frame0,
                          int n_frames, int batch_frames, void* d_wire, void* hip_stream) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    rtk::CodecGeom g;
    if (!codec_geom(width, height, band_rows, world, batch_frames, g, nullptr) || rank < 0 || rank >= world ||
        frame0 < 0 || n_frames <= 0 || n_frames > 65535 || frame0 + n_frames > batch_frames || !d_wire ||
        ((uintptr_t)d_wire & 7) != 0)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands_tiles: bad arguments");
    if (ctx->n_gpus != 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_bands_tiles needs a single-GPU context");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    rc = ensure_stage(ctx, d, g);
    if (rc != RT_OK) return rc;
    const EncTarget enc{(unsigned char*)d_wire, (uint32_t*)d.d_stage, g.tiles_x, g.tiles_per_frame, frame0};
    int nb = 0;
    rc = trace_bands(ctx, d, (hipStream_t)hip_stream, width, height, band_rows, rank, world, (int32_t*)d_wire, &nb,
                     RT_BANDS_INT32, n_frames, 0, &enc);
    if (rc == RT_OK) {
        ctx->pixels += (uint64_t)nb * band_rows * width * (uint64_t)n_frames;
        if (frame0 == 0 || !d.staged.valid || d.staged.wire != d_wire)
            d.staged = {true, width, height, band_rows, rank, world, batch_frames, d_wire};
    }
    return rc;
}

int rt_finish_wire(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world, int n_frames,
                   void* d_wire, int64_t* d_wire_bytes, void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    rtk::CodecGeom g;
    if (!codec_geom(width, height, band_rows, world, n_frames, g, nullptr) || rank < 0 || rank >= world ||
        !d_wire || ((uintptr_t)d_wire & 7) != 0)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_finish_wire: bad arguments");
    if (ctx->n_gpus != 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_finish_wire needs a single-GPU context");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    // only the batch rt_render_bands_tiles staged last, with the same geometry and wire
    const auto& sb = d.staged;
    if (!d.d_stage || encode_stage_bytes(g) > d.stage_cap || !sb.valid || sb.W != width || sb.H != height ||
        sb.band_rows != band_rows || sb.rank != rank || sb.world != world || sb.wire != d_wire ||
        n_frames > sb.batch_frames)
        return fail(ctx, RT_ERR_INVALID_ARG,
                    "rt_finish_wire: no rt_render_bands_tiles batch of this geometry and wire with >= %d frames",
                    n_frames);
    const int traced_rows = (bands_of(height, band_rows, rank, world) * band_rows + 7) / 8;
    int e = launch_finish_wire((unsigned char*)d_wire, g, traced_rows, d_wire_bytes, d.d_stage, hip_stream);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "finish launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int rt_decode_gathered(rt_ctx* ctx, int width, int height, int band_rows, int world, int first_rank,
                       const void* d_gathered, size_t rank_stride, int n_frames, int32_t* d_frames,
                       size_t frame_stride, void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    rtk::CodecGeom g;
    rt_wire_layout lay;
    if (!codec_geom(width, height, band_rows, world, n_frames, g, &lay) || !d_gathered || !d_frames ||
        first_rank < 0 || first_rank > world || ((uintptr_t)d_gathered & 7) != 0 || (rank_stride & 7) != 0 ||
        (world - first_rank > 1 && rank_stride < lay.max_bytes) || frame_stride < (size_t)width * height)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_decode_gathered: bad arguments");
    if (first_rank == world) return RT_OK;
    g.rank = first_rank;
    g.frame_stride = frame_stride;
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    int e = launch_decode_gathered((const unsigned char*)d_gathered, rank_stride, d_frames, g, hip_stream);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "decode launch: %s", hipGetErrorString((hipError_t)e));
    return RT_OK;
}

int rt_comm_probe(void) {
    std::string err;
    if (!g_rccl.load(err)) return fail(nullptr, RT_ERR_RCCL, "%s", err.c_str());
    return RT_OK;
}

int rt_comm_unique_id(void* out_id) {
    if (!out_id) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_comm_unique_id: NULL");
    std::string err;
    if (!g_rccl.load(err)) return fail(nullptr, RT_ERR_RCCL, "%s", err.c_str());
    ncclUniqueId id;
    const ncclResult_t r = g_rccl.GetUniqueId(&id);
    if (r != 0) return fail(nullptr, RT_ERR_RCCL, "ncclGetUniqueId: %s", g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?");
    std::memcpy(out_id, id.internal, RT_COMM_ID_BYTES);
    return RT_OK;
}

int rt_comm_init(rt_ctx* ctx, int world, int rank, const void* id) {
    if (!ctx || !id || world < 1 || rank < 0 || rank >= world)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_init: bad arguments");
    if (ctx->n_gpus != 1 || ctx->rccl_gather)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_init needs a single-GPU context without RT_CREATE_RCCL_GATHER");
    Device& d = ctx->dev[0];
    if (d.comm) return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_init: the context already has a communicator");
    std::string err;
    if (!g_rccl.load(err)) return fail(ctx, RT_ERR_RCCL, "%s", err.c_str());
    DeviceGuard guard(d.id);
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, RT_COMM_ID_BYTES);
    const ncclResult_t r = g_rccl.CommInitRank(&d.comm, world, uid, rank);
    if (r != 0) {
        d.comm = nullptr;
        return fail(ctx, RT_ERR_RCCL, "ncclCommInitRank: %s", g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?");
    }
    d.comm_rank = rank, d.comm_world = world;
    return RT_OK;
}

int rt_comm_allreduce_max_i64(rt_ctx* ctx, int64_t* d_values, int count, void* hip_stream) {
    if (!ctx || !d_values || count < 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_allreduce_max_i64: bad arguments");
    Device& d = ctx->dev[0];
    if (!d.comm || !d.comm_world) return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_allreduce_max_i64: no rt_comm_init");
    DeviceGuard guard(d.id);
    const ncclResult_t r =
        g_rccl.AllReduce(d_values, d_values, (size_t)count, ncclInt64, ncclMax, d.comm, (hipStream_t)hip_stream);
    if (r != 0) return fail(ctx, RT_ERR_RCCL, "ncclAllReduce: %s", g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?");
    return RT_OK;
}

int rt_comm_gather(rt_ctx* ctx, const void* d_send, size_t n_bytes, void* d_recv, size_t recv_stride, int rotate,
                   void* hip_stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    Device& d = ctx->dev[0];
    if (!d.comm || !d.comm_world) return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_gather: no rt_comm_init");
    const int world = d.comm_world, rank = d.comm_rank;
    if ((n_bytes && !d_send) || (rank == 0 && n_bytes && (!d_recv || recv_stride < n_bytes)))
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_comm_gather: bad arguments");
    if (!n_bytes) return RT_OK;
    DeviceGuard guard(d.id);
    const hipStream_t st = (hipStream_t)hip_stream;
    auto slot = [&](int r) { return (size_t)(((r - rotate) % world + world) % world) * recv_stride; };
    if (world > 1) {
        if (g_rccl.GroupStart() != 0) return fail(ctx, RT_ERR_RCCL, "ncclGroupStart failed");
        ncclResult_t r = 0;
        if (rank != 0) {
            r = g_rccl.Send(d_send, n_bytes, ncclUint8, 0, d.comm, st);
        } else {
            for (int q = 1; q < world && r == 0; ++q)
                r = g_rccl.Recv((char*)d_recv + slot(q), n_bytes, ncclUint8, q, d.comm, st);
        }
        const ncclResult_t e = g_rccl.GroupEnd();
        if (r != 0 || e != 0)
            return fail(ctx, RT_ERR_RCCL, "ncclSend/Recv: %s",
                        g_rccl.GetErrorString ? g_rccl.GetErrorString(r ? r : e) : "?");
    }
    if (rank == 0)  // rank 0's own slot
        HIP_TRY(ctx, hipMemcpyAsync((char*)d_recv + slot(0), d_send, n_bytes, hipMemcpyDeviceToDevice, st));
    return RT_OK;
}

int rt_register_host(rt_ctx* ctx, void* host_ptr, size_t bytes) {
    if (!ctx || !host_ptr || !bytes) return fail(ctx, RT_ERR_INVALID_ARG, "rt_register_host: bad arguments");
    DeviceGuard guard(ctx->dev[0].id);
    // mapped into every device's address space: each worker's copy kernel writes its own bands (a
    // coarse-grained lock, hipExtHostRegisterCoarseGrained, measured the same copy rates: r05f)
    hipError_t e = hipHostRegister(host_ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        HIP_TRY(ctx, hipHostRegister(host_ptr, bytes, hipHostRegisterDefault));
    }
    rt_ctx::HostRange r{(char*)host_ptr, bytes, std::vector<char*>(ctx->dev.size(), nullptr)};
    for (size_t g = 0; g < ctx->dev.size(); ++g) {
        DeviceGuard dg(ctx->dev[g].id);
        void* mapped = nullptr;
        if (hipHostGetDevicePointer(&mapped, host_ptr, 0) == hipSuccess && mapped)
            r.mapped[g] = (char*)mapped;
        else
            (void)hipGetLastError();  // not mapped on this device: its hand-off takes the runtime's copies
    }
    ctx->host_ranges.push_back(std::move(r));
    return RT_OK;
}

int rt_unregister_host(rt_ctx* ctx, void* host_ptr) {
    if (!ctx || !host_ptr) return fail(ctx, RT_ERR_INVALID_ARG, "rt_unregister_host: bad arguments");
    // a hand-off still pending into this range is written first: nothing may touch it afterwards
    int rc = rt_wait(ctx);
    if (rc != RT_OK) return rc;
    for (size_t i = 0; i < ctx->host_ranges.size(); ++i)
        if (ctx->host_ranges[i].host == (char*)host_ptr) {
            ctx->host_ranges.erase(ctx->host_ranges.begin() + (long)i);
            break;
        }
    DeviceGuard guard(ctx->dev[0].id);
    HIP_TRY(ctx, hipHostUnregister(host_ptr));
    return RT_OK;
}

namespace {
// How a registered frame's hand-off is copied in the synchronous Tick (RT_TICK_COPY): runtime -- the
// runtime's copy engine after the trace, same stream; kernel -- the copy kernel through the device-mapped
// address, chunked (chunk c's copy rides in chunk c+1's launch, the last by the copy kernel alone);
// stream -- chunked, each chunk's copy by the copy engine on a second stream after the chunk's trace
// (event-ordered), so it runs under the next chunk's trace.  Default: stream (r05k, one GPU: C5 271 ->
// 391 fps at 4 chunks, C4 1,028 -> 1,250; the copy kernel writes host memory at ~35 GB/s against the
// copy engine's ~52).  A share of one chunk (a 1080p frame) takes the runtime's copy after the trace at
// n = 1 and the copy kernel at n > 1, whose bands are too short for pitched copies.
enum TickCopy { TICK_RUNTIME = 0, TICK_KERNEL = 1, TICK_STREAM = 2 };
TickCopy tick_copy_mode() {
    if (const char* e = std::getenv("RT_TICK_COPY")) {
        if (std::strcmp(e, "kernel") == 0) return TICK_KERNEL;
        if (std::strcmp(e, "runtime") == 0) return TICK_RUNTIME;
    }
    return TICK_STREAM;
}

// Chunks of a worker's share in a synchronous Tick.  RT_TICK_CHUNKS=1..8 fixes the count; by default one
// chunk per ~2 M pixels of the share, at most 8 (1080p: 1; C4 at n = 1: 4; C5: 8 at n = 1, 2 at n = 8;
// r05k: C4 4 chunks 1,250 fps against 8 chunks 1,016, C5 8 chunks ~ 4).
int tick_chunks(const rt_ctx* ctx, int W, int H) {
    if (const char* e = std::getenv("RT_TICK_CHUNKS")) {
        const int k = std::atoi(e);
        if (k >= 1 && k <= 8) return k;
    }
    const double share = (double)W * H / ctx->n_gpus;
    return (int)std::min(8.0, std::max(1.0, std::floor(share / 2.0e6 + 0.5)));
}

// The synchronous Tick of every worker: each traces its band set and copies it into `pixels` on its
// own stream (its own device and PCIe link); the host waits for all of them at the end.
int tick_sync(rt_ctx* ctx, int W, int H, int32_t* pixels) {
    const int n = ctx->n_gpus;
    const size_t frame_bytes = (size_t)W * H * sizeof(int32_t);
    const int chunks = tick_chunks(ctx, W, H);
    for (int g = 0; g < n; ++g) {
        Device& d = ctx->dev[(size_t)g];
        DeviceGuard guard(d.id);
        int32_t* mapped = mapped_host(ctx, g, pixels, frame_bytes);
        const TickCopy mode = mapped ? tick_copy_mode() : TICK_RUNTIME;
        const int nc = mode != TICK_RUNTIME ? chunks : 1;
        const Share sh = share_of(W, H, g, n, nc > 1);
        if (sh.nb <= 0) continue;
        int rc = grow(ctx, (void**)&d.d_bands, &d.bands_cap, (size_t)sh.nb * sh.band_rows * W * sizeof(int32_t));
        if (rc != RT_OK) return rc;
        if (mode == TICK_STREAM && nc > 1) {  // chunk c: trace (stream) -> event -> copy engine (copy stream)
            if (!d.copy_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&d.copy_stream, hipStreamNonBlocking));
            for (int c = 0; c < nc; ++c) {
                const int k0 = (int)((long long)sh.nb * c / nc), k1 = (int)((long long)sh.nb * (c + 1) / nc);
                if (k1 <= k0) continue;
                if (!d.ev_chunk[c]) HIP_TRY(ctx, hipEventCreateWithFlags(&d.ev_chunk[c], hipEventDisableTiming));
                rc = trace_bands(ctx, d, d.stream, W, H, sh.band_rows, sh.first + k0 * sh.step, sh.step,
                                 d.d_bands + (size_t)k0 * sh.band_rows * W, nullptr, RT_BANDS_INT32, 1, 0, nullptr,
                                 nullptr, k1 - k0);
                if (rc != RT_OK) return rc;
                HIP_TRY(ctx, hipEventRecord(d.ev_chunk[c], d.stream));
                HIP_TRY(ctx, hipStreamWaitEvent(d.copy_stream, d.ev_chunk[c], 0));
                rc = runtime_band_copy(ctx, sh, W, H, d.d_bands, pixels, d.copy_stream, true, k0, k1);
                if (rc != RT_OK) return rc;
            }
            continue;
        }
        if (mode == TICK_RUNTIME || (nc == 1 && n == 1)) {  // the runtime's copy after the trace
            rc = trace_bands(ctx, d, d.stream, W, H, sh.band_rows, sh.first, sh.step, d.d_bands, nullptr);
            if (rc != RT_OK) return rc;
            const bool ctimed = begin_timed(ctx, d, 1);
            rc = runtime_band_copy(ctx, sh, W, H, d.d_bands, pixels, d.stream, mapped != nullptr);
            end_timed(d, ctimed);
            if (rc != RT_OK) return rc;
            continue;
        }
        CopyJob prev{};
        for (int c = 0; c < nc; ++c) {
            const int k0 = (int)((long long)sh.nb * c / nc), k1 = (int)((long long)sh.nb * (c + 1) / nc);
            if (k1 <= k0) continue;
            int32_t* out = d.d_bands + (size_t)k0 * sh.band_rows * W;
            rc = trace_bands(ctx, d, d.stream, W, H, sh.band_rows, sh.first + k0 * sh.step, sh.step, out, nullptr,
                             RT_BANDS_INT32, 1, 0, nullptr, &prev, k1 - k0);
            if (rc != RT_OK) return rc;
            prev = share_job(sh, W, H, k0, k1, out, mapped);
        }
        const bool ctimed = begin_timed(ctx, d, 1);
        const int e = launch_band_copy(prev, d.stream);
        end_timed(d, ctimed);
        if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "hand-off copy: %s", hipGetErrorString((hipError_t)e));
    }
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        HIP_TRY(ctx, hipStreamSynchronize(d.stream));
        if (d.copy_stream) HIP_TRY(ctx, hipStreamSynchronize(d.copy_stream));
    }
    return RT_OK;
}
}  // namespace

// Tick(): full frame into the caller's Surface.pixels, synchronous.
int rt_render(rt_ctx* ctx, int width, int height, int32_t* pixels) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (!pixels) return fail(ctx, RT_ERR_INVALID_ARG, "NULL pixels");
    for (const Device& d : ctx->dev)
        if (d.hand.job.words || d.copy_pending[0] || d.copy_pending[1]) {  // rt_render_async frames first (the
            rc = rt_wait(ctx);                                             // caller may reuse their buffers)
            if (rc != RT_OK) return rc;
            break;
        }
    if (ctx->rccl_gather) {  // bands gathered to device 0 over RCCL, then the whole frame over its link
        Device& d0 = ctx->dev[0];
        const size_t frame_bytes = (size_t)width * height * sizeof(int32_t);
        {
            DeviceGuard guard(d0.id);
            rc = grow(ctx, (void**)&d0.d_frame, &d0.frame_cap, frame_bytes);
            if (rc != RT_OK) return rc;
        }
        rc = gather_frame(ctx, width, height, d0.d_frame);
        if (rc != RT_OK) return rc;
        DeviceGuard guard(d0.id);
        const bool ctimed = begin_timed(ctx, d0, 1);
        HIP_TRY(ctx, hipMemcpyAsync(pixels, d0.d_frame, frame_bytes, hipMemcpyDeviceToHost, d0.stream));
        end_timed(d0, ctimed);
        HIP_TRY(ctx, hipStreamSynchronize(d0.stream));
    } else {
        rc = tick_sync(ctx, width, height, pixels);
        if (rc != RT_OK) return rc;
    }
    ctx->frames++;
    ctx->pixels += (uint64_t)width * (uint64_t)height;
    return RT_OK;
}

// Double-buffered Tick() on one in-order stream per worker.  Frame k's band set is traced into device
// buffer k % 2; its D2H copy rides in frame k+1's launch as the copy slice (grid z = 0, dispatched
// ahead of the trace workgroups, so the PCIe-bound copy of frame k runs under the trace of frame k+1)
// or is issued by rt_wait.  Buffer k % 2 is traced again by launch k+2, after launch k+1 (its copy) on
// the same stream.  The slice writes only host ranges registered through rt_register_host (their
// device-mapped addresses); any other buffer gets the runtime's copies on the same stream.  n > 1: every
// worker does the same with its own bands, stream and PCIe link.
// Measured (profiles/r03_tick_ab.txt): a trace stream and a copy stream ordered by events ran
// 175-195 us per frame in some processes and 350-1200 us in others -- torch's own kernel-on-one-
// stream / D2H-on-another pattern does the same -- while one stream ran a steady 195-200 us with
// the runtime's copy and 184-187 us with the copy slice.
int rt_render_async(rt_ctx* ctx, int width, int height, int32_t* pixels) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (!pixels) return fail(ctx, RT_ERR_INVALID_ARG, "NULL pixels");
    if (ctx->rccl_gather) return rt_render(ctx, width, height, pixels);
    const size_t frame_bytes = (size_t)width * height * sizeof(int32_t);
    const int n = ctx->n_gpus;
    // The hand-off of frame k: by the copy engine on a second stream, chunk by chunk after each chunk's trace
    // (event-ordered; the trace of frame k+2 into the same buffer waits for the copy), or as the copy slice
    // in frame k+1's launch.  Default (RT_TICK_ASYNC=stream|slice overrides): the copy engine, except for
    // shares under 0.5 M pixels at n > 1, whose short bands the pitched copies move slowly (r05l, one GPU,
    // two frames deep: C3 4,928 -> 5,167 fps, C4 1,034 -> 1,261, C5 268 -> 331; C2 at 8 workers 4,800 ->
    // 4,338 with the engine).
    const char* am = std::getenv("RT_TICK_ASYNC");
    const bool engine = am ? std::strcmp(am, "stream") == 0 : (n == 1 || (double)width * height / n >= 5e5);
    const int nc = engine ? tick_chunks(ctx, width, height) : 1;
    for (int g = 0; g < n; ++g) {
        Device& d = ctx->dev[(size_t)g];
        DeviceGuard guard(d.id);
        if (!d.async_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&d.async_stream, hipStreamNonBlocking));
        const int slot = d.async_next;
        const Share sh = share_of(width, height, g, n, nc > 1);
        const size_t bytes = std::max<size_t>(1, (size_t)sh.nb * sh.band_rows * width) * sizeof(int32_t);
        if (d.frames2_cap[slot] < bytes || sh.nb <= 0) {  // (re)allocation: the pending copy may read the
            rc = flush_hand(ctx);                         // other buffer only, but nothing may still use
            if (rc != RT_OK) return rc;                   // this one
            HIP_TRY(ctx, hipStreamSynchronize(d.async_stream));
            if (d.copy_stream) HIP_TRY(ctx, hipStreamSynchronize(d.copy_stream));
            d.copy_pending[0] = d.copy_pending[1] = false;
        }
        if (sh.nb <= 0) continue;  // (more workers than bands)
        rc = grow(ctx, (void**)&d.d_frames2[slot], &d.frames2_cap[slot], bytes);
        if (rc != RT_OK) return rc;
        if (engine) {
            if (!d.copy_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&d.copy_stream, hipStreamNonBlocking));
            for (int i = 0; i < 2; ++i) {
                if (!d.ev_traced[i]) HIP_TRY(ctx, hipEventCreateWithFlags(&d.ev_traced[i], hipEventDisableTiming));
                if (!d.ev_copied[i]) HIP_TRY(ctx, hipEventCreateWithFlags(&d.ev_copied[i], hipEventDisableTiming));
            }
            rc = flush_hand(ctx);  // (a slice-mode frame still pending)
            if (rc != RT_OK) return rc;
            const uint64_t f = d.frames_issued++;
            const int cap = ctx->tick_inflight;
            if (cap > 0 && f >= (uint64_t)cap && d.ev_ring[(f - cap) % Device::RING])  // at most cap frames queued
                HIP_TRY(ctx, hipEventSynchronize(d.ev_ring[(f - cap) % Device::RING]));
            if (d.copy_pending[slot]) HIP_TRY(ctx, hipStreamWaitEvent(d.async_stream, d.ev_copied[slot], 0));
            const bool pinned = mapped_host(ctx, g, pixels, frame_bytes) != nullptr;
            for (int c = 0; c < nc; ++c) {
                const int k0 = (int)((long long)sh.nb * c / nc), k1 = (int)((long long)sh.nb * (c + 1) / nc);
                if (k1 <= k0) continue;
                hipEvent_t& ev = nc > 1 ? d.ev_chunk[c] : d.ev_traced[slot];
                if (!ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                rc = trace_bands(ctx, d, d.async_stream, width, height, sh.band_rows, sh.first + k0 * sh.step, sh.step,
                                 d.d_frames2[slot] + (size_t)k0 * sh.band_rows * width, nullptr, RT_BANDS_INT32, 1, 0,
                                 nullptr, nullptr, k1 - k0);
                if (rc != RT_OK) return rc;
                HIP_TRY(ctx, hipEventRecord(ev, d.async_stream));
                HIP_TRY(ctx, hipStreamWaitEvent(d.copy_stream, ev, 0));
                rc = runtime_band_copy(ctx, sh, width, height, d.d_frames2[slot], pixels, d.copy_stream, pinned, k0, k1);
                if (rc != RT_OK) return rc;
            }
            HIP_TRY(ctx, hipEventRecord(d.ev_copied[slot], d.copy_stream));
            if (cap > 0) {
                hipEvent_t& er = d.ev_ring[f % Device::RING];
                if (!er) HIP_TRY(ctx, hipEventCreateWithFlags(&er, hipEventDisableTiming));
                HIP_TRY(ctx, hipEventRecord(er, d.copy_stream));
            }
            d.copy_pending[slot] = true;
            d.async_next = slot ^ 1;
            continue;
        }
        rc = trace_bands(ctx, d, d.async_stream, width, height, sh.band_rows, sh.first, sh.step, d.d_frames2[slot],
                         nullptr, RT_BANDS_INT32, 1, 0, nullptr, d.hand.job.words ? &d.hand.job : nullptr);
        if (rc != RT_OK) return rc;
        d.hand = {};  // issued (in the launch)
        int32_t* mapped = mapped_host(ctx, g, pixels, frame_bytes);
        if (mapped) {
            d.hand.host = sh.step == 1 ? pixels : nullptr;
            d.hand.job = share_job(sh, width, height, 0, sh.nb, d.d_frames2[slot], mapped);
        } else {
            rc = runtime_band_copy(ctx, sh, width, height, d.d_frames2[slot], pixels, d.async_stream);
            if (rc != RT_OK) return rc;
        }
        d.async_next = slot ^ 1;
    }
    ctx->frames++;
    ctx->pixels += (uint64_t)width * (uint64_t)height;
    return RT_OK;
}

int rt_wait(rt_ctx* ctx) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    int rc = flush_hand(ctx);
    if (rc != RT_OK) return rc;
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        HIP_TRY(ctx, hipStreamSynchronize(d.stream));
        if (d.async_stream) HIP_TRY(ctx, hipStreamSynchronize(d.async_stream));
        if (d.copy_stream) HIP_TRY(ctx, hipStreamSynchronize(d.copy_stream));
        d.copy_pending[0] = d.copy_pending[1] = false;
    }
    return RT_OK;
}

// Debug ray view: re-trace every sample_stride-th pixel and append its segments.
int rt_debug_segments(rt_ctx* ctx, int width, int height, int sample_stride, rt_segment* out, int capacity,
                      int* out_count) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (sample_stride <= 0 || capacity < 0 || (capacity > 0 && !out) || !out_count)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_debug_segments: bad arguments");
    static_assert(sizeof(rt_segment) == sizeof(DevSegment), "rt_segment layout");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    LaunchParams lp;
    std::memset(&lp, 0, sizeof lp);
    rc = view_params(ctx, width, height, lp);
    if (rc != RT_OK) return rc;
    scene_params(ctx, d, lp);
    lp.band_rows = height, lp.band_first = 0, lp.band_step = 1, lp.local_rows = height;
    DevSegment* d_out = nullptr;
    unsigned* d_count = nullptr;
    HIP_TRY(ctx, hipMalloc((void**)&d_count, sizeof(unsigned)));
    hipError_t e = hipMemsetAsync(d_count, 0, sizeof(unsigned), d.stream);  // same stream as the kernel
    if (e == hipSuccess && capacity > 0) e = hipMalloc((void**)&d_out, sizeof(DevSegment) * (size_t)capacity);
    if (e == hipSuccess) e = (hipError_t)launch_debug_segments(lp, sample_stride, d_out, capacity, d_count, d.stream);
    unsigned n = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&n, d_count, sizeof n, hipMemcpyDeviceToHost, d.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d.stream);
    const unsigned keep = n < (unsigned)capacity ? n : (unsigned)capacity;
    if (e == hipSuccess && keep) e = hipMemcpy(out, d_out, sizeof(DevSegment) * keep, hipMemcpyDeviceToHost);
    (void)hipFree(d_count);
    if (d_out) (void)hipFree(d_out);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "rt_debug_segments: %s", hipGetErrorString(e));
    *out_count = (int)n;
    return RT_OK;
}

// Binary PPM (P6) of 0x00RRGGBB pixels -- the headless stand-in for the GL texture upload
// (template.cs:188-193), also used to eyeball frames from tests.
int rt_write_ppm(const char* path, const int32_t* pixels, int width, int height) {
    if (!path || !pixels || width <= 0 || height <= 0) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_write_ppm: bad args");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_write_ppm: cannot open %s", path);
    std::fprintf(f, "P6\n%d %d\n255\n", width, height);
    std::vector<unsigned char> row((size_t)width * 3);
    bool ok = true;
    for (int y = 0; y < height && ok; ++y) {
        for (int x = 0; x < width; ++x) {
            const uint32_t v = (uint32_t)pixels[(size_t)y * width + x];
            row[(size_t)x * 3 + 0] = (unsigned char)(v >> 16);
            row[(size_t)x * 3 + 1] = (unsigned char)(v >> 8);
            row[(size_t)x * 3 + 2] = (unsigned char)v;
        }
        ok = std::fwrite(row.data(), 1, row.size(), f) == row.size();
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? RT_OK : fail(nullptr, RT_ERR_INVALID_ARG, "rt_write_ppm: write failed for %s", path);
}

int rt_get_stats(rt_ctx* ctx, rt_stats* out) {
    if (!ctx || !out) return fail(ctx, RT_ERR_INVALID_ARG, "rt_get_stats: NULL argument");
    std::memset(out, 0, sizeof *out);
    unsigned long long c[4] = {0, 0, 0, 0};
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        HIP_TRY(ctx, hipDeviceSynchronize());
        drain_events(ctx, d);
        std::vector<unsigned long long> h(COUNTER_WORDS);
        HIP_TRY(ctx, hipMemcpy(h.data(), d.d_counters, COUNTER_WORDS * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost));
        for (int slot = 0; slot < COUNTER_SLOTS; ++slot)
            for (int i = 0; i < 4; ++i) c[i] += h[(size_t)slot * COUNTER_STRIDE + i];
    }
    out->frames = ctx->frames;
    out->pixels = ctx->pixels;
    out->primary_rays = ctx->prim_rays;
    out->reflect_rays = c[CNT_REFLECT];
    out->shadow_rays = c[CNT_SHADOW];
    const uint64_t S = (uint64_t)ctx->layout.S, P = (uint64_t)ctx->layout.P;
    out->sphere_tests = (ctx->prim_rays + c[1] + c[2]) * S;
    out->plane_tests = (ctx->prim_rays + c[1]) * P;
    out->launches = ctx->launches;
    out->kernel_ms = ctx->kernel_ms;
    out->last_kernel_ms = ctx->last_kernel_ms;
    out->copy_ms = ctx->copy_ms;
    out->gather_ms = ctx->gather_ms;
    out->timed_launches = ctx->timed[0];
    out->timed_copies = ctx->timed[1];
    out->timed_gathers = ctx->timed[2];
    return RT_OK;
}

int rt_dispatch_order(rt_ctx* ctx, int* out_order) {
    if (!ctx || !out_order) return fail(ctx, RT_ERR_INVALID_ARG, "NULL argument");
    // (a new scene or frame size is measured again from its first single-frame launch)
    if (ctx->dev.empty()) return fail(ctx, RT_ERR_INVALID_ARG, "context without a device");
    const Device::OrderTuner& t = ctx->dev[0].order;
    // (the tuner measures single-frame launches of view_w x view_rows traced rows, whatever the view height)
    const bool fresh = t.scene_gen == ctx->scene_gen && ctx->view_ok && t.W == ctx->view_w && t.H == ctx->view_rows;
    *out_order = ctx->order_fixed >= 0 ? ctx->order_fixed : fresh ? ctx->dev[0].order.chosen : -1;
    return RT_OK;
}

int rt_set_timing(rt_ctx* ctx, int every) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    if (every < 0) return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_timing: every must be >= 0");
    ctx->timing_every = every;
    for (Device& d : ctx->dev) d.op_count[0] = d.op_count[1] = d.op_count[2] = 0;
    return RT_OK;
}

int rt_set_counting(rt_ctx* ctx, int on) {
    if (!ctx || (on != 0 && on != 1)) return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_counting: bad arguments");
    ctx->counting = on != 0;
    return RT_OK;
}

int rt_reset_stats(rt_ctx* ctx) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "NULL context");
    for (Device& d : ctx->dev) {
        DeviceGuard guard(d.id);
        HIP_TRY(ctx, hipDeviceSynchronize());
        drain_events(ctx, d);
        HIP_TRY(ctx, hipMemset(d.d_counters, 0, COUNTER_WORDS * sizeof(unsigned long long)));
        HIP_TRY(ctx, hipDeviceSynchronize());  // the clear lands before the next frame's atomics
    }
    ctx->frames = ctx->pixels = ctx->launches = ctx->prim_rays = 0;
    ctx->kernel_ms = ctx->last_kernel_ms = ctx->copy_ms = ctx->gather_ms = 0;
    ctx->timed[0] = ctx->timed[1] = ctx->timed[2] = 0;
    for (Device& d : ctx->dev) d.op_count[0] = d.op_count[1] = d.op_count[2] = 0;
    return RT_OK;
}

int rt_count_work(rt_ctx* ctx, int width, int height, rt_work* out) {
    int rc = check_ctx(ctx, width, height);
    if (rc != RT_OK) return rc;
    if (!out) return fail(ctx, RT_ERR_INVALID_ARG, "rt_count_work: NULL out_work");
    if (ctx->n_gpus != 1) return fail(ctx, RT_ERR_INVALID_ARG, "rt_count_work needs a single-GPU context");
    Device& d = ctx->dev[0];
    DeviceGuard guard(d.id);
    LaunchParams lp;
    std::memset(&lp, 0, sizeof lp);
    rc = view_params(ctx, width, height, lp);
    if (rc != RT_OK) return rc;
    scene_params(ctx, d, lp);
    rc = view_tables(ctx, d, lp);
    if (rc != RT_OK) return rc;
    rc = grow(ctx, (void**)&d.d_frame, &d.frame_cap, (size_t)width * height * sizeof(int32_t));
    if (rc != RT_OK) return rc;
    if (!d.d_counters_diag)
        HIP_TRY(ctx, hipMalloc((void**)&d.d_counters_diag, COUNTER_WORDS * sizeof(unsigned long long)));
    HIP_TRY(ctx, hipMemsetAsync(d.d_counters_diag, 0, COUNTER_WORDS * sizeof(unsigned long long), d.stream));
    lp.counters = d.d_counters_diag;
    lp.band_rows = height, lp.band_first = 0, lp.band_step = 1, lp.local_rows = height;
    lp.out = d.d_frame;
    lp.out_fmt = RT_BANDS_INT32;
    lp.n_frames = 1;
    if (const char* sel = getenv("RT_DIAG_SEL")) lp.enc_frame0 = atoi(sel);  // RT_SHADOW_CAT diagnostic builds only
    int e = launch_trace(lp, ctx->layout.generic_pow, true, d.stream);
    if (e != hipSuccess) return fail(ctx, RT_ERR_HIP, "rt_count_work launch: %s", hipGetErrorString((hipError_t)e));
    std::vector<unsigned long long> h(COUNTER_WORDS);
    HIP_TRY(ctx, hipMemcpyAsync(h.data(), d.d_counters_diag, COUNTER_WORDS * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(ctx, hipStreamSynchronize(d.stream));
    unsigned long long c[COUNTER_STRIDE] = {};
    for (int slot = 0; slot < COUNTER_SLOTS; ++slot)
        for (int i = 0; i < COUNTER_STRIDE; ++i) c[i] += h[(size_t)slot * COUNTER_STRIDE + i];
    const uint64_t S = (uint64_t)ctx->layout.S, P = (uint64_t)ctx->layout.P;
    std::memset(out, 0, sizeof *out);
    out->primary_rays = (uint64_t)width * (uint64_t)height;
    out->reflect_rays = c[CNT_REFLECT];
    out->shadow_rays = c[CNT_SHADOW];
    out->sphere_tests = (out->primary_rays + out->reflect_rays + out->shadow_rays) * S;
    out->plane_tests = (out->primary_rays + out->reflect_rays) * P;
    out->shadow_rays_run = c[CNT_SHADOW_RUN];
    out->sphere_tests_run = c[CNT_SPHERE_RUN];
    out->plane_tests_run = c[CNT_PLANE_RUN];
    return RT_OK;
}

}  // extern "C"
