// rt_internal.h -- device-side scene layout and launch interface shared by the HIP
// kernels (rt_kernel.hip) and the C-ABI host code (rt_api.cpp).
//
// Scene layout in HBM (one contiguous, 16-byte aligned allocation per context/device,
// read through the scalar cache: every loop over primitives is wave-uniform):
//   DevSphere  [S]   {center.xyz, radius^2}                 16 B   intersection loops
//   DevMaterial[S+P] sphere materials then plane materials  64 B   shading (per-lane gather)
//   DevPlane   [P]   {center, c.n, normal, e1, e2}          64 B
//   DevLight   [L]   {position, intensity, |p|^2 terms, shadow threshold, cull frame}  64 B
// Everything that the reference recomputes per call but that depends only on scene
// constants (radius^2 :336, dot(center,normal) :594, checkerboard basis e1/e2 :760-765,
// ambient*Ka :778/:873, dot(light,light) for the shadow ray :617) is computed once on the
// host with the same binary32 operations, which yields bit-identical values.
#pragma once
#include <stdint.h>

namespace rtk {

struct DevSphere {
    float cx, cy, cz, r2;
};

enum : uint32_t { MAT_MIRROR = 1u, MAT_DIFFUSE = 2u, MAT_SPEC = 4u };

enum : uint32_t { POW_GENERIC = 0u, POW_ONE = 1u, POW_HALF = 2u, POW_TWO = 3u };

struct DevMaterial {
    float kd[3];
    float amb[3];   // ambient * Ka  (RayTracer.cs:778, :873)
    float ks[3];
    float n;
    float km[3];
    uint32_t flags;  // MAT_* (RayTracer.cs:85-93)
    uint32_t pow_kind;  // POW_* fast paths for Math.Pow(x, n) (exact; see rt_kernel.hip)
    uint32_t pad;
};

struct DevPlane {
    float cx, cy, cz, cn;  // center, dot(center, normal)
    float nx, ny, nz, pad0;
    float e1x, e1y, e1z, pad1;
    float e2x, e2y, e2z, pad2;
};

struct DevLight {
    float px, py, pz, intensity;
    float a;      // dot(p, p)       : IntersectsSphere's `a` for a shadow ray (dir = position)
    float a2;     // 2 * a
    float a4;     // 4 * a
    // Shadow threshold (2a finite and > 0): IntersectsSphere(.., 0.001f) collides iff
    // fl(-b - sqrt) >= sh_t, i.e. fl(fl(-b - sqrt) / 2a) - 0.001f > 0 without the division
    // (rt_api.cpp shadow_threshold).
    float sh_t;
    // shadow-cull frame (culling only, never in a result): A ~ p/|p| (every shadow ray of this
    // light has direction p), U, V ~ orthonormal to A
    float ax, ay, az, pad1;
    float ux, uy, uz, pad2;
    float vx, vy, vz, pad3;
};

// Per-sphere culling record: centre and a radius bound r' >= sqrt(r^2) * (1 + 2^-8).
struct DevSphereCull {
    float cx, cy, cz, rr;
};

// Sphere clusters of the bundle kernel's per-lane pre-cull (CULL_MIN_SPHERES <= S <= 64; culling only): a
// bounding sphere (centre, radius R >= |c_i - centre| + r'_i of every member, r' as in DevSphereCull) and
// the member set as a mask over sphere indices.  A trace bundle whose cone allows no culling (the reflected
// segments deep in mirror chains, where a wave's rays fan out) tests each lane's own ray against the
// clusters and takes the union of the kept clusters' members (rt_kernel.hip cluster_mask) instead of every
// sphere.  Built on the host by median splits of the centres (rt_api.cpp build_clusters).
struct DevCluster {
    float cx, cy, cz, R;
    unsigned long long members;
    unsigned long long pad;
};
// Spheres per cluster: 4, 8 and 12 measured alike (C4 303.4-304.3 us, C5 1,114.7-1,116.3 us per frame against
// 311.2-311.8 / 1,135-1,137 without clusters), 2 and 16 slower (profiles/ab/r06_clusters.txt); 8 tests the fewest
// bounds.  (tools/trace_cull_model.py ranked 2 and 4 first: it prices a cluster test too cheaply.)
constexpr int CLUSTER_SIZE = 8;
constexpr int MAX_CLUSTERS = 32;

// Per-(light, sphere) shadow-cull record (culling only): the sphere centre in the light's frame
// (C.U, C.V, C.A, rounded from double) and r' + 2^-18 |C| (the projection-error allowance,
// rt_kernel.hip shadow_sphere_cull).  [L][S], built when L * S <= SHADOW_CULL_MAX_ENTRIES (larger
// scenes trace their shadow rays without culling).
struct DevShadowCull {
    float cu, cv, ca, rr;
};
constexpr long long SHADOW_CULL_MAX_ENTRIES = 1LL << 16;
// The direct kernel's per-lane shadow pre-test (S < CULL_MIN_SPHERES; culling only): per (light, sphere) the
// centre's (u, v) in the light's frame and, with the sphere's share of the margin folded in, the axial bound
// ca' and the radius bound rr' (rt_api.cpp, rt_kernel.hip shadow_pre_keep).  Same record type, [L][S + (S & 1)].

// Per-light shadow grid (bundle kernel's merged shadow pass, S <= 64 spheres, L <= 4 lights;
// culling only).  Every shadow ray of light l has direction p_l, so whether sphere j can block a
// hit point hp depends on hp's coordinates (u, v) across the light's axis and a along it.  The host
// tabulates, per light, a SHGRID_N x SHGRID_N grid over (u, v) of 64-bit masks -- the spheres whose
// margin-grown disc reaches the cell -- and SHGRID_SLABS + 2 axial masks -- the spheres whose
// centre may lie ahead of a slab -- valid for lanes with |hp|_1 <= `bound`; each lane looks up its
// own cell and slab (rt_kernel.hip shadow_members_grid).  Lanes beyond the bound use the bounding
// box of every disc with their own margin and the slab masks shifted by it.  Margins and the
// exactness argument: rt_api.cpp build_shadow_grid.
// The merged shadow pass (and so the grid) serves scenes with at most 64 spheres and this many lights.
constexpr int SHADOW_MERGE_L = 4;
constexpr int SHGRID_N = 64;
constexpr int SHGRID_SLABS = 32;
struct DevShadowGrid {
    float su, ou, sv, ov;  // cell coordinates: floor(fma(u, su, ou)), floor(fma(v, sv, ov))
    float sa, oa;          // slab coordinate: floor(fma(a, sa, oa)), clamped to [-1, SHGRID_SLABS]
    float bound;           // lanes with |hp|_1 <= bound use the grid
    float far_k;           // lanes beyond it: own margin far_k * |hp|_1 (2^-8 + projection error) ...
    float far_b;           // ... and slab coordinate a - (far_k * |hp|_1 - far_b), far_b = 2^-8 bound
    float bu0, bu1, bv0, bv1;  // (u, v) box of every sphere's disc grown by 2^-8 |C|_1 (no |hp| term)
    float pad;
    unsigned long long always;  // spheres never culled (no valid cull record: NaN/huge/tiny)
};
// Device layout: DevShadowGrid[L], then masks [L][SHGRID_N * SHGRID_N] (row iv, column iu), then
// slab masks [L][SHGRID_SLABS + 2] (entry ia + 1, ia = -1 .. SHGRID_SLABS).

// Work counters: each workgroup adds its totals into slot (block id % COUNTER_SLOTS) so that
// the atomics of thousands of workgroups do not serialise on one address.  Per slot:
// reflected segments and shadow rays of the visible path (every launch), and the executed
// work of the diagnostic kernels (rt_count_work): shadow rays whose sphere loop ran, exact
// sphere and plane tests run.
constexpr int COUNTER_SLOTS = 256;
constexpr int COUNTER_STRIDE = 8;
constexpr int COUNTER_WORDS = COUNTER_SLOTS * COUNTER_STRIDE;
enum : int { CNT_REFLECT = 1, CNT_SHADOW = 2, CNT_SHADOW_RUN = 3, CNT_SPHERE_RUN = 4, CNT_PLANE_RUN = 5 };

// Camera-relative sphere constants of the primary segment (origin = camera position for
// every pixel): oc = cam - center and c = Dot(oc, oc) - r^2 of IntersectsSphere
// (RayTracer.cs:614-619), computed once per frame on the host with the same binary32
// operations and passed in the kernarg block for up to MAX_PRIM_CONST spheres.
// Per-frame conservative screen box of sphere i for primary rays: pixels outside
// [x0, x1] x [y0, y1] cannot select sphere i (view_params in rt_api.cpp derives it).
struct PrimBox {
    int x0, x1, y0, y1;
};

struct PrimConst {
    float ocx, ocy, ocz, c;
};
constexpr int MAX_PRIM_CONST = 64;
constexpr int ROW_ORDER_MAX = 272;  // tile rows of a 2176-row frame (4K UHD: 270)

// Scenes with at least this many spheres use wave-bundle culling (rt_kernel.hip; the bundle
// kernel on the 8-sphere configs measured +20 %, profiles/ab/r02_direct_converged_fold_rejected.txt).
constexpr int CULL_MIN_SPHERES = 12;


// A band set's copy into a frame (the Tick hand-off, rt_api.cpp share_of): `words` int32 of a packed
// band set at src -> dst, band after band: source word i of band k = i / band_words lands at dst word
// k * dst_stride + i % band_words (band_words = 0: one contiguous run).  The host guarantees 16-byte
// aligned ends and band_words, dst_stride multiples of 4 (whole 16-byte stores never straddle a band).
struct CopyJob {
    const int32_t* src;
    int32_t* dst;
    unsigned long long words;
    unsigned long long dst_stride;
    unsigned band_words;
    unsigned pad;
};

// Per-launch parameters (passed by value as the kernel argument block, < 4 KiB).
struct LaunchParams {
    const DevSphere* sph;
    const DevMaterial* mat;  // [S + P]
    const DevPlane* pl;
    const DevLight* li;
    const DevSphereCull* scull;  // [S]
    const DevShadowCull* shcull;  // [L][S] or NULL (no shadow culling)
    const DevShadowCull* shpre;   // [L][S + (S & 1)] the direct kernel's shadow pre-test, or NULL
    const DevShadowGrid* shg;     // [L] or NULL (no shadow grid: the per-level bound instead)
    const unsigned long long* shgrid;  // [L][SHGRID_N^2]
    const unsigned long long* shslab;  // [L][SHGRID_SLABS + 2]
    const DevCluster* clus;            // [n_clus] (n_clus 0: no per-lane pre-cull)
    const float* lxt;  // [W]: ((float)x / W - 0.5f) * pw, TracePixel :963-965
    const float* lyt;  // [H]: ((float)y / H - 0.5f) * ph
    int S, P, L, limit;
    int lights_a2_ok;  // every light's 2a = 2 p.p is finite and > 0 (the shadow loops' exact-threshold form)
    int n_clus;
    // view, RayTracer.cs:511-523 and :892-896 (computed on the host)
    float cam[3], right[3], up[3], fwd[3];
    float pw, ph, nearc;
    int W, H;
    // row mapping: local row r -> band (band_first + (r / band_rows) * band_step),
    // global row = band * band_rows + r % band_rows; pixel written at out[r * W + x].
    int band_rows, band_first, band_step, local_rows;
    int n_frames;  // grid z (frames of one batch launch, all with this view); 0 = 1
    int32_t* out;
    unsigned long long out_frame_bytes;  // batch launches: frame z of the grid at (char*)out + z * out_frame_bytes
    int out_fmt;  // 0: int32 0x00RRGGBB per pixel; 1: packed 24-bit (bytes B, G, R); 2: int32 at frame row y;
                  // 3 (OUT_TILES): the tile codec's encoder fused into the trace -- nothing at `out`,
                  // tile t's header into enc_wire and its segments into enc_stage[t * STAGE_WORDS],
                  // t = (enc_frame0 + frame) * enc_tpf + tile row * enc_tiles_x + tile column
    unsigned char* enc_wire;
    uint32_t* enc_stage;
    int enc_tiles_x, enc_tpf, enc_frame0;
    unsigned long long* counters;  // COUNTER_SLOTS x COUNTER_STRIDE (CNT_*)
    // The Tick hand-off fused into a trace launch (rt_render_async: the previous frame; a chunked
    // rt_render: the previous chunk): with copy_z = 1 the launch has one more grid z-slice, z = 0,
    // whose workgroups run `copy` (device band set -> the caller's registered host buffer through its
    // device-mapped address); the launch's one frame is z = 1 (out_frame_bytes 0).  copy_z = 0: none.
    CopyJob copy;
    int copy_z;
    int prim_const;                // 1: pc[0..S) and pbox[0..S) valid (S <= MAX_PRIM_CONST)
    PrimConst pc[MAX_PRIM_CONST];
    PrimBox pbox[MAX_PRIM_CONST];
    // single-frame launches of a whole frame (the direct kernel's multi-tile workgroups): dispatch
    // position -> tile row in the order the host picked (rt_api.cpp order_pick: rows by estimated
    // cost, or bottom to top; row_order_n = the launch's tile rows, 0: natural order).  A lone
    // frame's last waves set its tail.
    int row_order_n;
    int col_major;  // single-frame launches: tile rows vary fastest in dispatch order (grid x = rows)
    uint16_t row_order[ROW_ORDER_MAX];
    // single-frame launches, measured order (order_pick candidate 3): dispatch position (workgroup x
    // SINGLE_WPG + wave, a 1-D grid) -> tile (ty << 16 | tx; ty = 0xffff pads past the last tile), and
    // tile_cost: when set, each wave stores its duration (RTC ticks) at tile ty * tiles_x + tx
    const uint32_t* tile_order;
    uint32_t* tile_cost;
};
// Tiles per workgroup of the direct kernel's single-frame launches (8: +2.5 % on C2,
// profiles/r04_final_check.txt); the measured tile order (LaunchParams::tile_order) is padded to it.
constexpr int SINGLE_WPG = 4;
// The kernel argument block: raising ROW_ORDER_MAX or MAX_PRIM_CONST must not push it past 4 KiB.
static_assert(sizeof(LaunchParams) < 4096, "LaunchParams is passed by value as the kernarg block (< 4 KiB)");

// Debug-view segment (layout of rt_segment in include/raytracer_hip.h).
struct DevSegment {
    float ox, oy, oz, ex, ey, ez;
    int kind, pixel;
};

// Launchers (rt_kernel.hip).  Return hipError_t as int.
int launch_debug_segments(const LaunchParams& p, int stride, DevSegment* out, int capacity, unsigned* count,
                          void* stream);
// generic_pow: some material needs the f64 Math.Pow path (exponent not 0.5, 1 or 2).
// stats: the diagnostic kernels that also tally the executed work (CNT_*_RUN).
int launch_trace(const LaunchParams& p, bool generic_pow, bool stats, void* stream);
// All ranks' gathered band sets (rank r's at g + r * slot_bytes, format fmt) -> frame.
int launch_scatter_gathered(const unsigned char* g, size_t slot_bytes, int fmt, int32_t* frame, int W, int H,
                            int band_rows, int world, void* stream);
int launch_scatter_bands(const int32_t* bands, int32_t* frame, int W, int H, int band_rows, int band_first,
                         int band_step, int n_bands, void* stream);
// A CopyJob on its own (the Tick hand-off when no later trace launch carries it: the last chunk of a
// synchronous rt_render, rt_wait's flush of rt_render_async's last frame).
int launch_band_copy(const CopyJob& job, void* stream);

constexpr int OUT_TILES = 3;

// Band-set tile codec (rt_codec.hip; format: raytracer_hip/tilecodec.py).
struct CodecGeom {
    int W, H, band_rows, rank, world, n_bands;  // rank / n_bands: the encoder's rank; the decoder's first rank
    int tiles_x, tiles_y, tiles_per_frame, n_tiles, n_chunks;
    size_t frame_stride;  // elements between frames (input band sets / output frames)
    size_t fixed_bytes;   // wire: header + tile headers + chunk bases, 8-aligned
};
// n_frames band sets (frame_stride apart) of g.rank -> wire; *wire_bytes (device, may be
// NULL) receives the wire's byte size.  Two launches; `stage` = encode_stage_bytes(g) of
// device scratch that no other launch uses meanwhile.
int launch_encode_bands(const int32_t* bands, unsigned char* wire, const CodecGeom& g, int64_t* wire_bytes,
                        void* stage, void* stream);
size_t encode_stage_bytes(const CodecGeom& g);
// The second half of the encoder after traces with OUT_TILES filled the tile headers (tile rows
// >= traced_tile_rows of every frame were not traced: their headers are zeroed) and the staging
// slots: chunk totals from the headers, then the compaction of launch_encode_bands.  Two launches.
int launch_finish_wire(unsigned char* wire, const CodecGeom& g, int traced_tile_rows, int64_t* wire_bytes,
                       void* stage, void* stream);
// every rank's wire (rank r's at gathered + r * rank_stride) -> frames.  One launch.
int launch_decode_gathered(const unsigned char* gathered, size_t rank_stride, int32_t* frames, const CodecGeom& g,
                           void* stream);

}  // namespace rtk
