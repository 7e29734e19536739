/*
 * raytracer_hip.h -- C ABI of libraytracer_hip, the MI355X (gfx950) drop-in for the
 * per-pixel Whitted trace of TobiasDeBruijn/UU-INFOGR-Raytracer.
 *
 * The reference has no FFI: its plugin surface is the C# class
 *   RayTracer(Surface screen)          Raytracer/RayTracer.cs:535-537
 *   public readonly Surface screen     Raytracer/RayTracer.cs:506
 *   public void Tick()                 Raytracer/RayTracer.cs:886-935
 *   OnKeyPress(KeyboardKeyEventArgs)   Raytracer/RayTracer.cs:543-554
 *   OnMouseMove(MouseMoveEventArgs)    Raytracer/RayTracer.cs:1058-1061
 * plus Surface.width/height/int[] pixels (Raytracer/surface.cs:9-20).  Every entry
 * point below replaces one piece of that surface; the C# P/Invoke shim that binds
 * them is in INTEGRATION.md / shim/csharp/RayTracer.cs.
 *
 * Conventions
 *  - Plain C, blittable POD structs of float32/int32 (no packing pragmas, no torch
 *    types).  All functions return RT_OK (0) or a negative RT_ERR_* code and never
 *    throw; rt_last_error() returns the message of the last failure.
 *  - A context is used by one thread at a time (the reference calls Tick, OnKeyPress
 *    and OnMouseMove from the GLFW render thread, template.cs:175-230).
 *  - There is NO CPU fallback: rt_create fails with RT_ERR_NO_DEVICE when no gfx950
 *    device is visible.
 */
#ifndef RAYTRACER_HIP_H
#define RAYTRACER_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 10

/* ---- status codes ---------------------------------------------------------- */
enum {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = -1,   /* NULL pointer, negative size, bad enum value          */
    RT_ERR_NO_DEVICE = -2,     /* no HIP device / not enough devices for n_gpus        */
    RT_ERR_HIP = -3,           /* a HIP runtime call failed (message has the HIP text) */
    RT_ERR_NO_SCENE = -4,      /* render before rt_set_scene                          */
    RT_ERR_UNSUPPORTED = -5,   /* e.g. recursion_limit above RT_MAX_RECURSION_LIMIT    */
    RT_ERR_RCCL = -6,          /* a RCCL call failed (multi-GPU contexts)              */
    RT_ERR_OOM = -7            /* device allocation failed                            */
};

/* Deepest mirror chain the kernel's per-lane level stack holds: a limit of L
 * shades levels 0..L (L+1 stack records).  The reference's own limit is 32
 * (RayTracer.cs:490). */
#define RT_MAX_RECURSION_LIMIT 63
#define RT_MAX_LIGHTS 65536  /* per-lane shadow-ray counts are kept in 24 bits */

/* ---- scene description (RayTracer.cs:60-338, :441-469) ---------------------- */
typedef struct rt_vec3 {
    float x, y, z;
} rt_vec3;

/* Material, RayTracer.cs:60-110.  Flags are derived exactly as the reference does:
 * IsMirror = km != 0, IsDiffuse = kd != 0, HasSpecularity = ks != 0 && n > 0
 * (RayTracer.cs:85-93). */
typedef struct rt_material {
    rt_vec3 kd;  /* diffuseColor  K_d */
    rt_vec3 ka;  /* ambientColor  K_a */
    rt_vec3 ks;  /* specularColor K_s */
    float n;     /* specularity   n   */
    rt_vec3 km;  /* mirrorColor   K_m */
} rt_material;

/* Sphere, RayTracer.cs:308-338 (radiusSquared = radius*radius, :336). */
typedef struct rt_sphere {
    rt_vec3 center;
    float radius;
    rt_material material;
} rt_sphere;

/* Plane, RayTracer.cs:260-303.  Planes are always checkerboard-tiled: the
 * reference's constructor ignores its isTiled argument (RayTracer.cs:289). */
typedef struct rt_plane {
    rt_vec3 center;
    rt_vec3 normal;
    rt_material material;
} rt_plane;

/* Light, RayTracer.cs:236-255. */
typedef struct rt_light {
    rt_vec3 position;
    float intensity;
} rt_light;

/* Camera state of the reference: _cameraPosition, _yaw, _pitch (RayTracer.cs:494-502).
 * The basis (RayTracer.cs:511-523) and view-plane size (RayTracer.cs:892-896) are
 * derived from it once per frame on the host with the reference's double-precision
 * trig (rt_camera_view). */
typedef struct rt_camera {
    rt_vec3 position;
    float yaw;
    float pitch;
} rt_camera;

/* Per-frame view derived from rt_camera and the surface size. */
typedef struct rt_view {
    rt_vec3 position;
    rt_vec3 right;    /* CameraRightDirection   RayTracer.cs:517-518 */
    rt_vec3 up;       /* CameraUpDirection      RayTracer.cs:522-523 */
    rt_vec3 forward;  /* CameraForwardDirection RayTracer.cs:511-513 */
    float plane_width, plane_height, near_clip;  /* viewParams RayTracer.cs:892-896 */
} rt_view;

/* Reference keys handled by OnKeyPress (RayTracer.cs:545-553). */
enum {
    RT_KEY_W = 1, RT_KEY_A = 2, RT_KEY_S = 3, RT_KEY_D = 4,
    RT_KEY_SPACE = 5, RT_KEY_SHIFT = 6
};

/* Work counters of the visible (nearest-hit) path, accumulated since the last
 * rt_reset_stats.  rays = primary + reflected segments (terminal segments included);
 * shadow_rays = shaded diffuse hits x lights.  Times are device time measured with
 * HIP events on the stream the operation runs on, for the sampled operations only (see
 * rt_set_timing): average kernel duration = kernel_ms / timed_launches.  rt_render_async
 * ticks hand the previous frame to its host buffer inside the next frame's launch (a copy
 * slice ahead of the trace workgroups): that copy's share is in the launch's kernel_ms, the
 * last frame's copy (issued by rt_wait / the next synchronous call) is not timed, and
 * copy_ms / timed_copies count rt_render's D2H copies only. */
typedef struct rt_stats {
    uint64_t frames;
    uint64_t pixels;
    uint64_t primary_rays;
    uint64_t reflect_rays;
    uint64_t shadow_rays;
    uint64_t sphere_tests;   /* algorithmic: (primary+reflect+shadow) x S */
    uint64_t plane_tests;    /* algorithmic: (primary+reflect) x P        */
    uint64_t launches;
    double kernel_ms;        /* sum of trace-kernel durations            */
    double last_kernel_ms;
    double copy_ms;          /* sum of D2H / reassembly copy durations    */
    double gather_ms;        /* sum of RCCL gather durations (multi-GPU)  */
    uint64_t timed_launches; /* launches whose durations are in kernel_ms  */
    uint64_t timed_copies;   /* copies in copy_ms                          */
    uint64_t timed_gathers;  /* gathers in gather_ms                       */
} rt_stats;

/* Nominal and executed work of one frame (rt_count_work, ABI 5).  The nominal counts are
 * SURVEY.md 8(d)'s (every primitive of every visible-path ray; Mray/s counts these rays).
 * The kernels skip work that provably cannot change a pixel -- shadow rays whose outcome
 * cannot matter (shadow_rays_run <= shadow_rays), sphere tests culled by screen boxes, wave
 * bundles and the terminal-segment rule -- so the *_run counts are what actually ran: per
 * lane, each exact IntersectsSphere / IntersectPlane evaluation whose result the lane used. */
typedef struct rt_work {
    uint64_t primary_rays, reflect_rays, shadow_rays;  /* nominal, as rt_stats          */
    uint64_t sphere_tests, plane_tests;                /* nominal, as rt_stats          */
    uint64_t shadow_rays_run;   /* shadow rays whose sphere loop ran                   */
    uint64_t sphere_tests_run;  /* exact sphere tests executed (trace + shadow rays)   */
    uint64_t plane_tests_run;   /* exact plane tests executed                          */
} rt_work;

typedef struct rt_ctx rt_ctx;

/* ---- library / device ------------------------------------------------------- */
int rt_abi_version(void);
/* Number of visible HIP devices (0 when none).  Returns RT_OK or RT_ERR_HIP. */
int rt_device_count(int* out_count);
/* Message of the last failure on ctx (ctx may be NULL: last failure of this thread). */
const char* rt_last_error(const rt_ctx* ctx);

/* ---- context lifetime  (replaces `new RayTracer(screen)`, RayTracer.cs:535) ---- */
/* n_gpus >= 1 band workers, one per device (devices 0 .. n_gpus-1; n_gpus == 1: the caller's
 * current device), each with its own HIP stream.  A frame is split into interleaved 8-row bands,
 * band b on worker b % n_gpus (ABI 9): rt_render / rt_render_async hand every
 * worker's bands to the caller's host frame over that device's own PCIe link (no gather, no
 * single-link copy of the whole frame); rt_render_device gathers them to device 0 over RCCL/xGMI
 * (ncclCommInitAll, made on first use). */
#define RT_MAX_WORKERS 64
int rt_create(int n_gpus, rt_ctx** out_ctx);
/* rt_create with flags.  RT_CREATE_RCCL_GATHER (ABI 5): rt_render gathers the bands to device 0 over
 * RCCL (grouped ncclGather, one-launch reassembly) and copies the whole frame over device 0's link --
 * for callers that need the frame assembled on device 0; communicators made at creation, any
 * n_gpus, 1 included.  RT_CREATE_SHARED_DEVICE (ABI 9): all n_gpus workers on the caller's current
 * device (a stream each) -- the multi-GPU band pipeline rehearsed on one GPU; rt_render_device then
 * writes the workers' bands straight into the frame (no RCCL: it refuses two ranks on one device). */
enum { RT_CREATE_RCCL_GATHER = 1, RT_CREATE_SHARED_DEVICE = 2 };
int rt_create_ex(int n_gpus, int flags, rt_ctx** out_ctx);
void rt_destroy(rt_ctx* ctx);

/* ---- scene (replaces the hard-coded fields RayTracer.cs:441-490) ------------- */
int rt_set_scene(rt_ctx* ctx,
                 const rt_sphere* spheres, int n_spheres,
                 const rt_plane* planes, int n_planes,
                 const rt_light* lights, int n_lights,
                 rt_vec3 ambient, int recursion_limit);

/* ---- camera (mirrors RayTracer.cs:511-523, :543-554, :892-896, :1058-1061) ---- */
int rt_set_camera(rt_ctx* ctx, const rt_camera* camera);
/* (ABI 9) The view's height: later renders of a width x height frame with height <= view_height trace
 * rows [0, height) of the view of a width x view_height frame (TracePixel's y / height, :963-965, with
 * the view's height) -- the multi-GPU pipeline's tracing ranks when rank 0 renders the frame's last rows
 * itself; 0 (the default) = each render's own height.  The debug view ignores it. */
int rt_set_view_height(rt_ctx* ctx, int view_height);
int rt_get_camera(const rt_ctx* ctx, rt_camera* camera);
int rt_camera_view(const rt_camera* camera, int width, int height, rt_view* out_view);
int rt_camera_on_key(rt_camera* camera, int key);
int rt_camera_on_mouse_move(rt_camera* camera, float delta_x, float delta_y);

/* ---- rendering (replaces Tick(), RayTracer.cs:886-935) ---------------------- */
/* Tick(): renders the full frame and copies it into the caller-owned host buffer
 * pixels[width*height] (Surface.pixels, 0x00RRGGBB, row-major y*width+x).
 * Synchronous: the pixels are complete on return, as template.cs:189-193 requires.
 * Every worker writes its own bands into `pixels` (registered: a copy kernel through the buffer's
 * device-mapped address, on large shares in chunks whose copies ride in the next chunk's trace
 * launch; unregistered: the runtime's copies). */
int rt_render(rt_ctx* ctx, int width, int height, int32_t* pixels);

/* Pin a caller-owned host buffer (hipHostRegister, mapped into every worker's device) so that the
 * Tick hand-off lands directly in it; the shim registers Surface.pixels once. */
int rt_register_host(rt_ctx* ctx, void* host_ptr, size_t bytes);
int rt_unregister_host(rt_ctx* ctx, void* host_ptr);

/* Device-resident variant: renders the frame into d_pixels[width*height] (device 0's memory) on
 * `hip_stream` (a hipStream_t of device 0; NULL = the HIP null stream, as everywhere in HIP) and
 * returns without synchronising.  n_gpus > 1: the workers' bands are gathered to device 0 over
 * RCCL/xGMI (RT_CREATE_SHARED_DEVICE: written straight into d_pixels), ordered after the work
 * already on hip_stream, and hip_stream waits for the frame. */
int rt_render_device(rt_ctx* ctx, int width, int height, int32_t* d_pixels, void* hip_stream);

/* Row-band shard (one process per GPU): renders the bands b = band_first,
 * band_first+band_step, ... of band_rows rows each (rows [b*band_rows, (b+1)*band_rows)
 * clipped to height) into d_out, packed band after band, each band width*band_rows
 * int32 (rows past the image are left untouched).  Returns the number of bands in
 * *out_n_bands when not NULL.  Asynchronous on hip_stream. */
int rt_render_bands(rt_ctx* ctx, int width, int height, int band_rows, int band_first,
                    int band_step, int32_t* d_out, void* hip_stream, int* out_n_bands);

/* Reassemble: copies n_bands packed bands (as written by rt_render_bands with the same
 * band_first/band_step) from d_bands into the row-major frame d_frame[width*height].
 * Asynchronous on hip_stream. */
int rt_scatter_bands(rt_ctx* ctx, int width, int height, int band_rows, int band_first,
                     int band_step, const int32_t* d_bands, int32_t* d_frame, void* hip_stream);

/* Band sets for shipping to rank 0.  Formats: RT_BANDS_INT32 (as
 * rt_render_bands) or RT_BANDS_RGB24 (3 bytes B, G, R per pixel: the top byte of
 * 0x00RRGGBB is always 0, so a quarter fewer bytes cross xGMI), or RT_BANDS_FRAME: the
 * bands straight into their rows of the row-major frame d_out[height][width] (other rows
 * untouched) -- rank 0's own share, which never travels. */
enum { RT_BANDS_INT32 = 0, RT_BANDS_RGB24 = 1, RT_BANDS_FRAME = 2 };
int rt_render_bands_ex(rt_ctx* ctx, int width, int height, int band_rows, int band_first,
                       int band_step, void* d_out, int format, void* hip_stream, int* out_n_bands);
/* n_frames frames of this rank's bands (the current camera, every frame traced in full) in
 * ONE launch: frame f's output at d_out + f * frame_stride_bytes, in `format`.  For the
 * multi-GPU pipeline, where a rank's share of a 1080p frame is a few microseconds of GPU work
 * and one launch per frame would leave the GPU waiting for the host. */
int rt_render_bands_batch(rt_ctx* ctx, int width, int height, int band_rows, int band_first,
                          int band_step, int n_frames, void* d_out, size_t frame_stride_bytes,
                          int format, void* hip_stream, int* out_n_bands);
/* Reassemble the band sets of `world` ranks (band b rendered by rank b % world with
 * band_first = rank, band_step = world), gathered rank after rank at slot_bytes intervals
 * in d_gathered, into the row-major frame d_frame[height][width] -- one launch for all
 * ranks (rank 0's side of the RCCL gather). */
int rt_scatter_gathered(rt_ctx* ctx, int width, int height, int band_rows, int world,
                        const void* d_gathered, size_t slot_bytes, int format, int32_t* d_frame,
                        void* hip_stream);

/* ---- tile codec for the gather to rank 0 (ABI 4, format 2 since ABI 6) --
 * Lossless: each rank encodes its int32 band sets (as rt_render_bands writes them, the
 * slot of the largest band set per frame) into a "wire" -- per 8x8 tile a 4-byte header (raw
 * first pixel, width code), second-difference (gradient) prediction, zigzag residuals packed
 * at 0/2/3/4/6/8 bits per channel -- and rank 0 decodes all ranks' wires straight into the
 * frames.  Rendered frames are mostly flat, so the wire is ~8-13x smaller than RGB24 at 1080p
 * (DESIGN.md 1e); the format is specified in raytracer_hip/tilecodec.py.  The wire's size
 * varies: the fixed part (header, tile headers, chunk bases) is the same on every rank, the
 * payload follows it. */
typedef struct rt_wire_layout {
    uint64_t fixed_bytes;  /* header + tile headers + chunk bases (8-aligned)          */
    uint64_t max_bytes;    /* fixed_bytes + the largest possible payload (capacity)     */
    int32_t tiles_x, tiles_y, tiles_per_frame, n_frames, n_tiles, n_chunks;
} rt_wire_layout;
/* Sizes of one rank's wire for n_frames frames (the same for every rank of `world`). */
int rt_wire_layout_of(int width, int height, int band_rows, int world, int n_frames, rt_wire_layout* out);
/* Encode n_frames band sets of `rank` (frame f at d_bands + f * frame_stride int32, each
 * at least the largest band set: bands_of(height, band_rows, 0, world) * band_rows * width)
 * into d_wire (8-aligned, max_bytes capacity).  *d_wire_bytes (device int64, may be NULL)
 * receives the wire's size in bytes.  Three launches, asynchronous on hip_stream. */
int rt_encode_bands(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world,
                    const int32_t* d_bands, size_t frame_stride, int n_frames, void* d_wire,
                    int64_t* d_wire_bytes, void* hip_stream);
/* Decode the wires of ranks first_rank .. world-1 (rank r's at d_gathered + r * rank_stride,
 * 8-aligned; each region at least max_bytes) into frame f = d_frames + f * frame_stride
 * (int32, row-major) for f < n_frames: only those ranks' rows are written (first_rank = 1:
 * rank 0 rendered its own rows with RT_BANDS_FRAME).  One launch, asynchronous on hip_stream. */
int rt_decode_gathered(rt_ctx* ctx, int width, int height, int band_rows, int world, int first_rank,
                       const void* d_gathered, size_t rank_stride, int n_frames, int32_t* d_frames,
                       size_t frame_stride, void* hip_stream);
/* The encoder fused into the trace (ABI 6): trace frames frame0 .. frame0+n_frames-1 of a batch
 * of batch_frames of `rank`'s bands straight into d_wire's tile headers and the context's codec
 * scratch -- the band set never reaches HBM -- then rt_finish_wire turns the batch's first
 * n_frames (<= batch_frames) into the same wire rt_encode_bands would have made of the band sets
 * (byte for byte).  A batch may take several rt_render_bands_tiles calls; the context's scratch
 * holds one batch at a time (stream-ordered, like rt_encode_bands').  Asynchronous on hip_stream. */
int rt_render_bands_tiles(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world,
                          int frame0, int n_frames, int batch_frames, void* d_wire, void* hip_stream);
int rt_finish_wire(rt_ctx* ctx, int width, int height, int band_rows, int rank, int world, int n_frames,
                   void* d_wire, int64_t* d_wire_bytes, void* hip_stream);

/* ---- one-process-per-GPU collectives on the trace stream (ABI 7) ---------------- */
/* The N > 1 tile pipeline's two exchange steps -- the all_reduce(MAX) of the wire sizes and the
 * gather of every rank's wire to rank 0 (the reference's only parallel loop is
 * RayTracer.cs:898-901) -- issued by the library itself on the caller's HIP stream, the stream
 * that traced and encoded the batch and that decodes it, so the exchange adds no cross-stream
 * hops (a torch.distributed collective runs on its own stream: a wait into it and one out of it,
 * ~20 us each in profiles/r03_dist_stages.txt).  The communicator is RCCL (the instance already
 * loaded in the process when there is one), one rank per process and device:
 *   rank 0: rt_comm_unique_id(id); share the RT_COMM_ID_BYTES with every rank (e.g. a broadcast);
 *   every rank: rt_comm_init(ctx, world, rank, id)          -- collective, on ctx's device. */
#define RT_COMM_ID_BYTES 128
/* (ABI 8) RT_OK when a librccl with every symbol the rt_comm_* calls use can be loaded in this
 * process; no communicator, socket or thread is created.  Ranks agree on the result (e.g. an
 * all_reduce(MIN)) before any of them starts rt_comm_init, which is collective: a rank that could
 * not join would leave the others blocked inside it. */
int rt_comm_probe(void);
int rt_comm_unique_id(void* out_id);
int rt_comm_init(rt_ctx* ctx, int world, int rank, const void* id);
/* In place, count int64 values on the device: every rank ends with the element-wise maximum. */
int rt_comm_allreduce_max_i64(rt_ctx* ctx, int64_t* d_values, int count, void* hip_stream);
/* Gather n_bytes from every rank's d_send to rank 0: rank r's bytes land at
 * d_recv + ((r - rotate) mod world) * recv_stride (rank 0 only; its own by a device copy).
 * Collective; n_bytes must be the same on every rank (0: nothing moves). */
int rt_comm_gather(rt_ctx* ctx, const void* d_send, size_t n_bytes, void* d_recv, size_t recv_stride, int rotate,
                   void* hip_stream);

/* ---- double-buffered frames ------------------------------ */
/* Asynchronous Tick(): captures the current camera, enqueues the trace and its hand-off into `pixels`
 * and returns; rt_wait blocks until every enqueued frame is in its host buffer.  With two host buffers
 * a caller overlaps the trace of frame k+1 with its own use of frame k (the camera of k+1 can already
 * be set).  Each worker double-buffers its band set in device memory: frame k's copy into `pixels`
 * runs on the copy engine on a second stream behind frame k's trace (registered `pixels`; a share
 * under 0.5 Mpixel at n_gpus > 1 rides instead as a copy slice in frame k+1's trace launch, and an
 * unregistered buffer gets the runtime's copies), while frame k+1 is traced.  At most 2 frames per
 * worker are in flight: the call for frame k+2 first waits on the host for frame k's copy (deeper
 * queues made the runtime block one copy call for 6-7 ms now and then, profiles/r06_tick_deep.txt;
 * RT_TICK_INFLIGHT overrides).  Measured on one MI355X (bench.py tick_*, C3 1080p, median of 3 x 20
 * frames): two frames deep with an rt_wait per pair 5.1-5.2k fps, 20 frames queued with one rt_wait
 * 5.7-5.8k fps, against 4.8k for the synchronous rt_render.  n_gpus > 1: every worker double-buffers
 * its own band set on its own streams and device (ABI 9; RT_CREATE_RCCL_GATHER contexts render
 * synchronously here). */
int rt_render_async(rt_ctx* ctx, int width, int height, int32_t* pixels);
int rt_wait(rt_ctx* ctx);

/* ---- headless display hand-off --------------------------- */
/* Writes pixels (0x00RRGGBB, row-major) as a binary PPM (P6).  Host only, no context. */
int rt_write_ppm(const char* path, const int32_t* pixels, int width, int height);

/* ---- debug ray view (RayTracer.cs:423-435, :903-934) ------- */
/* The reference's DEBUG_ENABLE view logs traced rays and draws 500 random ones as lines
 * (red primary, green secondary, blue shadow) into the lower-right 30 % inset.  Here the
 * pixels y*width+x with (y*width+x) % sample_stride == 0 are traced again and every segment
 * of their visible path is appended to out[] (at most `capacity`; *out_count receives the
 * total): primary/secondary segments end at the winning hit point (origin + 100*dir when
 * nothing is hit); shadow segments start at the shaded point with the light POSITION as
 * direction (Q2) and end at the first blocker's distance, or at t = 1 when unblocked.
 * Synchronous.  Composited on the host by raytracer_hip.debugview. */
typedef struct rt_segment {
    rt_vec3 origin;
    rt_vec3 end;
    int32_t kind;   /* 0 primary, 1 secondary (reflected), 2 shadow -- RayKind, :343-361 */
    int32_t pixel;  /* y*width + x */
} rt_segment;

int rt_debug_segments(rt_ctx* ctx, int width, int height, int sample_stride, rt_segment* out,
                      int capacity, int* out_count);

/* ---- statistics ------------------------------------------------------------- */
/* Synchronises the context's pending work, then returns the counters. */
/* Device timing of trace launches, copies and gathers with HIP event pairs: every
 * `every`-th operation of each kind is timed (the first one always), 0 = none.  Default 64:
 * an event pair costs several microseconds of GPU time, 17 % of a 1080p frame if every
 * frame were timed.  Counters (rays) are always exact (for the launches that count, rt_set_counting). */
int rt_set_timing(rt_ctx* ctx, int every);
/* Dispatch order of single-frame launches (rt_render, rt_render_device on scenes with fewer than
 * 12 spheres): the order in which the kernel's tiles start, which sets a lone frame's tail.  The
 * first launches of a scene and frame size time each candidate (0 tile rows by decreasing estimated
 * cost, 1 rows bottom to top, 2 rows varying fastest, 3 every tile by decreasing measured duration --
 * the round's first launch records each tile's duration) and keep the fastest; the pixels are the same
 * under every order.  *out_order: the candidate in use, -1 while still measuring (ABI 8 addition;
 * RT_DISPATCH_ORDER=0/1/2/3 in the environment at rt_create fixes it).  The choice is measured again
 * every 16,384 single-frame launches; candidate 3's tile durations are recorded again once the camera
 * has moved and 256 launches have used them (one device synchronisation per recording). */
int rt_dispatch_order(rt_ctx* ctx, int* out_order);
int rt_get_stats(rt_ctx* ctx, rt_stats* out_stats);
int rt_reset_stats(rt_ctx* ctx);
/* ABI 10.  on = 1 (the default): every trace launch adds its rays to the counters above (frame 0 of a
 * batch launch counts for all its frames; one device atomic pair per wave).  on = 0: the kernels count
 * nothing -- the display loop's setting, since the reference's Tick counts nothing and in a one-frame
 * launch every wave's atomics cost the frame 8-13 % (1080p; 4 % at 4K).  Launches made with counting
 * off still add to frames, pixels and launches, not to primary_rays (= the pixels of counted launches)
 * nor to the other ray and test counts.  Returns RT_ERR_INVALID_ARG unless on is 0 or 1. */
int rt_set_counting(rt_ctx* ctx, int on);
/* Traces one width x height frame of the current camera with the diagnostic kernels (same
 * pixels, plus executed-work tallies) into a context-owned buffer and returns its work.
 * Synchronous; single-GPU contexts; does not touch rt_get_stats' counters. */
int rt_count_work(rt_ctx* ctx, int width, int height, rt_work* out_work);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RAYTRACER_HIP_H */
