// san_host.cpp -- host sanitizer driver for the C ABI's host code (rt_api.cpp), TEST
// INFRASTRUCTURE ONLY ("host ASan/UBSan build of the oracle and the C ABI").
//
// rt_api.cpp is compiled into this translation unit (unity include) with AddressSanitizer +
// UndefinedBehaviorSanitizer on the host side only (tests/native/Makefile: -Xarch_host), so
// that the host work that never touches a device can be driven without a GPU:
//   * scene packing of rt_set_scene (material flags, plane bases, light frames, cull radii,
//     the even-padded sphere table) on a context with no devices;
//   * the per-frame view set-up (view_params: camera basis RayTracer.cs:511-523, view plane
//     :892-896, primary-segment constants, conservative screen boxes in double) over random
//     and degenerate cameras, cross-checked bit for bit against the oracle's camera view;
//   * OnKeyPress / OnMouseMove (:543-554, :1058-1061), rt_write_ppm, rt_wire_layout_of,
//     and the argument checks of every entry point (no device call is reached).
// Exit status 0 = all checks passed; any sanitizer report aborts the process.
#include "../../uu-infogr-raytracer_amd/csrc/rt_api.cpp"

#include <cstdint>
#include <cstdio>
#include <unistd.h>

#include "../../oracle/oracle.h"

namespace {
int failures = 0;
#define CHECK(cond, ...)                                         \
    do {                                                         \
        if (!(cond)) {                                           \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                   \
            std::fputc('\n', stderr);                            \
            ++failures;                                          \
        }                                                        \
    } while (0)

uint64_t rng = 0xC0FFEE5EEDull;
uint64_t next64() {
    uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
float unif(float lo, float hi) { return lo + (hi - lo) * (float)((next64() >> 40) * (1.0 / 16777216.0)); }
rt_vec3 v3(float x, float y, float z) { return rt_vec3{x, y, z}; }

bool same_bits(float a, float b) { return std::memcmp(&a, &b, sizeof a) == 0; }
bool same_vec(rt_vec3 a, rt_vec3 b) { return same_bits(a.x, b.x) && same_bits(a.y, b.y) && same_bits(a.z, b.z); }

rt_material material(int kind) {
    rt_material m;
    std::memset(&m, 0, sizeof m);
    const rt_vec3 c = v3(unif(0, 1), unif(0, 1), unif(0, 1));
    switch (kind % 5) {
        case 0: m.kd = m.ka = c; break;
        case 1: m.kd = m.ka = c, m.ks = v3(0.4f, 0.4f, 0.4f), m.n = 1.0f; break;
        case 2: m.kd = m.ka = c, m.ks = c, m.n = unif(2.5f, 30.0f); break;  // generic Math.Pow
        case 3: m.km = v3(1, 1, 1); break;
        default: m.kd = m.ka = c, m.km = v3(0.5f, 0.5f, 0.5f); break;
    }
    return m;
}

void check_scene_packing() {
    for (int it = 0; it < 40; ++it) {
        rt_ctx ctx;  // no devices: rt_set_scene packs on the host and uploads nowhere
        const int S = it == 0 ? 0 : (int)(next64() % 70), P = (int)(next64() % 4), L = (int)(next64() % 6);
        std::vector<rt_sphere> sph((size_t)S);
        std::vector<rt_plane> pl((size_t)P);
        std::vector<rt_light> li((size_t)L);
        for (rt_sphere& s : sph) {
            s.center = v3(unif(-8, 8), unif(-1, 3), unif(2, 40));
            s.radius = unif(0.0f, 1.5f);
            s.material = material((int)(next64() % 5));
        }
        if (S > 3) sph[3].radius = NAN;
        for (rt_plane& p : pl) {
            p.center = v3(unif(-2, 2), unif(-2, 0), unif(0, 50));
            p.normal = next64() % 5 == 0 ? v3(1, 0, 0) : v3(unif(-1, 1), unif(-1, 1), unif(-1, 1));
            p.material = material((int)(next64() % 5));
        }
        if (P > 1) pl[1].normal = v3(0, 0, 0);
        for (rt_light& l : li) l.position = v3(unif(-40, 40), unif(-5, 20), unif(-20, 40)), l.intensity = unif(0, 1);
        if (L > 0 && it % 3 == 0) li[0].position = v3(0, 0, 0);
        const int limit = (int)(next64() % 64);
        int rc = rt_set_scene(&ctx, sph.data(), S, pl.data(), P, li.data(), L, v3(0.1f, 0.1f, 0.1f), limit);
        CHECK(rc == RT_OK, "rt_set_scene rc %d (%s)", rc, ctx.last_error.c_str());
        const SceneLayout& lay = ctx.layout;
        CHECK(lay.S == S && lay.P == P && lay.L == L && lay.limit == limit, "layout counts");
        CHECK(lay.off_mat % 256 == 0 && lay.off_pl % 256 == 0 && lay.off_li % 256 == 0 && lay.off_cull % 256 == 0,
              "layout alignment");
        CHECK(lay.off_mat >= sizeof(DevSphere) * (size_t)(S + (S & 1)), "padded sphere table overlaps materials");
        CHECK(lay.bytes >= lay.off_cull + sizeof(DevSphereCull) * (size_t)S, "cull table outside the blob");
        CHECK(lay.host_sph.size() == (size_t)S, "host sphere copy");
        for (int i = 0; i < S; ++i) {
            const float r2 = sph[(size_t)i].radius * sph[(size_t)i].radius;
            CHECK(same_bits(lay.host_sph[(size_t)i].r2, r2), "radius^2 of sphere %d", i);
        }
        // per-frame view set-up over random, degenerate and far cameras
        for (int c = 0; c < 25; ++c) {
            rt_camera cam{v3(unif(-3, 3), unif(-1, 2), unif(-4, 2)), unif(-3.2f, 3.2f), unif(-1.5f, 1.5f)};
            if (c == 1) cam.position = v3(1e30f, -1e30f, 1e30f);
            if (c == 2) cam.yaw = NAN;
            if (c == 3) cam.pitch = INFINITY;
            if (c == 4 && S > 0) cam.position = sph[0].center;
            const int W = 1 + (int)(next64() % 4000), H = 1 + (int)(next64() % 2500);
            rt_set_camera(&ctx, &cam);
            LaunchParams lp;
            std::memset(&lp, 0, sizeof lp);
            rc = view_params(&ctx, W, H, lp);
            CHECK(rc == RT_OK, "view_params rc %d", rc);
            CHECK(lp.prim_const == (S <= MAX_PRIM_CONST ? 1 : 0), "prim_const flag");
            // the single-frame row order is a permutation of the frame's tile rows (or absent)
            const int rows = (H + 7) / 8;
            CHECK(lp.row_order_n == 0 || lp.row_order_n == rows, "row order over %d of %d rows", lp.row_order_n, rows);
            CHECK(lp.row_order_n > 0 || rows < 2 || rows > ROW_ORDER_MAX, "no row order for %d rows", rows);
            std::vector<char> seen((size_t)rows, 0);
            for (int r = 0; r < lp.row_order_n; ++r) {
                CHECK(lp.row_order[r] < rows && !seen[lp.row_order[r]], "row order not a permutation at %d", r);
                if (lp.row_order[r] < rows) seen[lp.row_order[r]] = 1;
            }
            // a box is never empty: the sphere is strictly in front (cz > rho), so both tangent
            // directions lie in (-pi/2, pi/2) and tan keeps their order
            for (int i = 0; lp.prim_const && i < S; ++i)
                CHECK(lp.pbox[i].x0 <= lp.pbox[i].x1 && lp.pbox[i].y0 <= lp.pbox[i].y1,
                      "empty screen box: sphere %d [%d,%d]x[%d,%d]", i, lp.pbox[i].x0, lp.pbox[i].x1, lp.pbox[i].y0,
                      lp.pbox[i].y1);
            rt_view a, b;
            CHECK(rt_camera_view(&cam, W, H, &a) == RT_OK && oracle_camera_view(&cam, W, H, &b) == RT_OK, "views");
            CHECK(same_vec(a.right, b.right) && same_vec(a.up, b.up) && same_vec(a.forward, b.forward) &&
                      same_bits(a.plane_width, b.plane_width) && same_bits(a.plane_height, b.plane_height) &&
                      same_bits(a.near_clip, b.near_clip),
                  "rt_camera_view != oracle_camera_view (yaw %a pitch %a %dx%d)", cam.yaw, cam.pitch, W, H);
        }
    }
    rt_ctx ctx;
    rt_sphere s{};
    rt_light l{};
    CHECK(rt_set_scene(&ctx, nullptr, 1, nullptr, 0, nullptr, 0, v3(0, 0, 0), 0) == RT_ERR_INVALID_ARG, "NULL spheres");
    CHECK(rt_set_scene(&ctx, &s, 1, nullptr, 0, &l, 1, v3(0, 0, 0), -1) == RT_ERR_INVALID_ARG, "negative limit");
    CHECK(rt_set_scene(&ctx, &s, 1, nullptr, 0, &l, 1, v3(0, 0, 0), RT_MAX_RECURSION_LIMIT + 1) == RT_ERR_UNSUPPORTED,
          "limit above the stack");
    CHECK(rt_set_scene(&ctx, &s, 1, nullptr, 0, &l, RT_MAX_LIGHTS + 1, v3(0, 0, 0), 0) == RT_ERR_UNSUPPORTED,
          "too many lights");
    // render entry points: argument checks only (the context has no device)
    int32_t px[4];
    CHECK(rt_render(nullptr, 2, 2, px) == RT_ERR_INVALID_ARG, "rt_render NULL ctx");
    CHECK(rt_render_device(&ctx, 2, 2, px, nullptr) == RT_ERR_NO_SCENE, "render before a scene");
    CHECK(rt_set_scene(&ctx, &s, 1, nullptr, 0, &l, 1, v3(0, 0, 0), 0) == RT_OK, "scene");
    CHECK(rt_render_device(&ctx, 0, 2, px, nullptr) == RT_ERR_INVALID_ARG, "zero width");
    CHECK(rt_render_device(&ctx, 65536, 65536, px, nullptr) == RT_ERR_INVALID_ARG, "frame over 2^31 pixels");
    CHECK(rt_render_bands_ex(&ctx, 8, 8, 0, 0, 1, px, RT_BANDS_INT32, nullptr, nullptr) == RT_ERR_INVALID_ARG,
          "band_rows 0");
    CHECK(rt_render_bands_ex(&ctx, 8, 8, 8, 0, 1, px, 7, nullptr, nullptr) == RT_ERR_INVALID_ARG, "bad format");
    CHECK(rt_render_bands_batch(&ctx, 8, 8, 8, 0, 1, 0, px, 256, RT_BANDS_INT32, nullptr, nullptr) == RT_ERR_INVALID_ARG,
          "zero frames");
    CHECK(rt_encode_bands(&ctx, 8, 8, 8, 2, 2, px, 64, 1, px, nullptr, nullptr) == RT_ERR_INVALID_ARG, "rank >= world");
    CHECK(rt_decode_gathered(&ctx, 8, 8, 8, 2, 0, px, 3, 1, px, 64, nullptr) == RT_ERR_INVALID_ARG, "unaligned stride");
}

void check_camera_input() {
    rt_camera c{v3(0, 0, 0), 0, 0};
    for (int k = 0; k <= 7; ++k) CHECK(rt_camera_on_key(&c, k) == RT_OK, "key %d", k);
    // W then S at yaw 0: forward (0, -0, 1) * 0.05 out and back
    rt_camera d{v3(0, 0, 0), 0, 0};
    rt_camera_on_key(&d, RT_KEY_W);
    CHECK(same_bits(d.position.z, 0.05f), "W moves along +z by 0.05f");
    rt_camera_on_key(&d, RT_KEY_S);
    CHECK(d.position.z == 0.0f, "S undoes W");
    CHECK(rt_camera_on_mouse_move(&c, 36.0f, -18.0f) == RT_OK, "mouse");
    CHECK(same_bits(c.yaw, 36.0f / 360.0f) && same_bits(c.pitch, -18.0f / 360.0f), "mouse deltas / 360");
    CHECK(rt_camera_on_key(nullptr, RT_KEY_W) == RT_ERR_INVALID_ARG, "NULL camera");
    rt_view v;
    CHECK(rt_camera_view(&c, 0, 1, &v) == RT_ERR_INVALID_ARG, "zero width view");
}

void check_ppm() {
    const int W = 37, H = 5;
    std::vector<int32_t> px((size_t)W * H);
    for (size_t i = 0; i < px.size(); ++i) px[i] = (int32_t)(next64() & 0xFFFFFF);
    char path[] = "/tmp/san_host_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0, "mkstemp");
    if (fd < 0) return;
    close(fd);
    CHECK(rt_write_ppm(path, px.data(), W, H) == RT_OK, "rt_write_ppm");
    FILE* f = std::fopen(path, "rb");
    std::vector<unsigned char> data(64 + (size_t)W * H * 3);
    const size_t n = f ? std::fread(data.data(), 1, data.size(), f) : 0;
    if (f) std::fclose(f);
    std::remove(path);
    const char head[] = "P6\n37 5\n255\n";
    const size_t hl = sizeof head - 1;
    CHECK(n == hl + (size_t)W * H * 3 && std::memcmp(data.data(), head, hl) == 0, "PPM header/size");
    for (size_t i = 0; n == hl + (size_t)W * H * 3 && i < px.size(); ++i) {
        const unsigned char* p = data.data() + hl + 3 * i;
        CHECK(p[0] == ((px[i] >> 16) & 255) && p[1] == ((px[i] >> 8) & 255) && p[2] == (px[i] & 255), "pixel %zu", i);
    }
    CHECK(rt_write_ppm(nullptr, px.data(), W, H) == RT_ERR_INVALID_ARG, "NULL path");
    CHECK(rt_write_ppm("/nonexistent-dir/x.ppm", px.data(), W, H) != RT_OK, "unwritable path");
}

void check_wire_layout() {
    rt_wire_layout lay;
    for (int it = 0; it < 500; ++it) {
        const int W = 1 + (int)(next64() % 8192), H = 1 + (int)(next64() % 4400), br = 1 + (int)(next64() % 16);
        const int world = 1 + (int)(next64() % 9), nf = 1 + (int)(next64() % 128);
        const int rc = rt_wire_layout_of(W, H, br, world, nf, &lay);
        if (rc != RT_OK) continue;  // above the codec's 2^26-tile limit
        const long long rows = (long long)std::max(1, bands_of(H, br, 0, world)) * br;
        CHECK(lay.tiles_x == (W + 7) / 8 && lay.tiles_y == (int)((rows + 7) / 8), "tile grid");
        CHECK((long long)lay.n_tiles == (long long)lay.tiles_per_frame * nf && lay.n_chunks == (lay.n_tiles + 7) / 8,
              "tiles / chunks");
        CHECK(lay.fixed_bytes % 8 == 0 && lay.max_bytes >= lay.fixed_bytes + 8ull * lay.n_tiles, "wire sizes");
    }
    CHECK(rt_wire_layout_of(8192, 8192, 8, 1, 65535, &lay) == RT_ERR_INVALID_ARG, "tile overflow rejected");
    CHECK(rt_wire_layout_of(8, 8, 8, 0, 1, &lay) == RT_ERR_INVALID_ARG, "world 0");
    CHECK(rt_wire_layout_of(8, 8, 8, 1, 1, nullptr) == RT_ERR_INVALID_ARG, "NULL layout");
}

// shadow_threshold: "n >= T" must equal IntersectsSphere's fl(fl(n / a2) - 0.001f) > 0 for every
// float n, for positive finite a2 -- checked at the threshold's neighbours and at random n.
bool shadow_ref(float n, float a2) {
    volatile float q = n / a2;  // correctly rounded binary32 (SSE, no contraction)
    volatile float d = q - 0.001f;
    return d > 0.0f;
}
void check_shadow_threshold() {
    long checked = 0;
    for (int it = 0; it < 200000; ++it) {
        float a2;
        switch (it % 4) {
            case 0: a2 = unif(1.0f, 4.0f); break;                                    // unit-ish directions
            case 1: a2 = std::ldexp(unif(1.0f, 2.0f), (int)(next64() % 250) - 125); break;
            case 2: a2 = std::ldexp(unif(1.0f, 2.0f), -126 - (int)(next64() % 23)); break;  // denormal
            default: { uint32_t u = (uint32_t)(next64() % 0x7F800000u) + 1u; std::memcpy(&a2, &u, 4); }
        }
        if (!(a2 > 0.0f) || !(a2 < INFINITY)) continue;
        const float T = shadow_threshold(a2);
        float n = T;
        for (int k = 0; k < 3; ++k) n = std::nextafter(n, -INFINITY);
        for (int k = 0; k < 7; ++k, n = std::nextafter(n, INFINITY), ++checked)
            CHECK((n >= T) == shadow_ref(n, a2), "threshold a2=%a n=%a T=%a", a2, n, T);
        const float r = std::ldexp(unif(-1.0f, 1.0f), (int)(next64() % 60) - 30) * a2;
        CHECK((r >= T) == shadow_ref(r, a2), "random a2=%a n=%a T=%a", a2, r, T);
        ++checked;
    }
    CHECK(!(NAN >= shadow_threshold(2.0f)) && (INFINITY >= shadow_threshold(2.0f)), "NaN / inf numerators");
    std::printf("shadow_threshold: %ld (n, 2a) pairs\n", checked);
}

// The per-light shadow grids (rt_set_scene -> build_shadow_grid; looked up by rt_kernel.hip
// shadow_members_grid): for random scenes -- unit, large and huge coordinates, tiny / zero / NaN
// radii, grazing and degenerate lights -- and hit points near sphere surfaces, on grazing shadow
// lines, on cell and slab edges, far beyond the table's bound and non-finite, a sphere the lookup
// leaves out of a lane's mask must never block that lane's binary32 shadow ray (the oracle's
// IntersectsSphere(hp, light.position, sphere, 0.001f), RayTracer.cs:573-582).  The lookup below
// repeats the device's operations (binary32 fmaf / floor / min / max).
unsigned long long grid_lookup(const DevShadowGrid& g, const DevLight& l, const unsigned long long* grid,
                               const unsigned long long* slab, rt_vec3 hp) {
    const float l1 = std::fabs(hp.x) + std::fabs(hp.y) + std::fabs(hp.z);
    const float u = std::fmaf(hp.z, l.uz, std::fmaf(hp.y, l.uy, hp.x * l.ux));
    const float v = std::fmaf(hp.z, l.vz, std::fmaf(hp.y, l.vy, hp.x * l.vx));
    const float a = std::fmaf(hp.z, l.az, std::fmaf(hp.y, l.ay, hp.x * l.ax));
    const bool near = l1 <= g.bound;
    const float xu = std::fmaf(u, g.su, g.ou), xv = std::fmaf(v, g.sv, g.ov);
    const bool in_grid = (xu >= 0.0f) & (xu < (float)SHGRID_N) & (xv >= 0.0f) & (xv < (float)SHGRID_N);
    const unsigned iu = (unsigned)std::fmin(std::fmax(xu, 0.0f), (float)(SHGRID_N - 1));
    const unsigned iv = (unsigned)std::fmin(std::fmax(xv, 0.0f), (float)(SHGRID_N - 1));
    const unsigned long long cell = grid[iv * SHGRID_N + iu];
    const float mg = g.far_k * l1;
    const float af = near ? a : a - (mg - g.far_b);
    const float xa = std::fmin(std::fmax(std::floor(std::fmaf(af, g.sa, g.oa)), -1.0f), (float)SHGRID_SLABS);
    const unsigned long long sl = slab[(unsigned)((int)xa + 1)];
    const bool out_box = (u < g.bu0 - mg) | (u > g.bu1 + mg) | (v < g.bv0 - mg) | (v > g.bv1 + mg);
    const bool take = near ? in_grid : !out_box;
    return (take ? (near ? cell : ~0ull) & sl : 0ull) | g.always;
}

void check_shadow_grid() {
    long checked = 0, culled = 0, lanes = 0, cands = 0;
    for (int it = 0; it < 48; ++it) {
        const float scale = it % 4 == 3 ? 1000.0f : it % 4 == 2 ? 30.0f : 1.0f;
        const int S = 12 + (int)(next64() % 53), L = 1 + (int)(next64() % SHADOW_MERGE_L);
        std::vector<rt_sphere> sph((size_t)S);
        std::vector<rt_light> li((size_t)L);
        for (int i = 0; i < S; ++i) {
            rt_sphere& s = sph[(size_t)i];
            s.center = v3(unif(-8, 8) * scale, unif(-1, 3) * scale, unif(2, 40) * scale);
            s.radius = unif(0.05f, 1.5f) * scale;
            s.material = material((int)(next64() % 5));
        }
        sph[1].radius = 1e-25f;  // r^2 below 2^-100: never culled
        sph[2].radius = 0.0f;
        if (it % 5 == 1) sph[4].radius = NAN;
        if (it % 6 == 2) sph[5].center = v3(3e9f, 0, 0);  // |C|_1 >= 2^30: never culled
        for (int j = 0; j < L; ++j) {
            rt_light& l = li[(size_t)j];
            l.position = v3(unif(-40, 40), unif(-5, 20), unif(-20, 40));
            l.intensity = 1.0f;
            if (j == 1 && it % 3 == 0) l.position = v3(unif(-40, 40), 1e-3f, unif(-1, 1));  // grazing
            if (j == 2 && it % 7 == 0) l.position = v3(1e-30f, 0, 0);                      // |p|^2 < 2^-40
            if (j == 3 && it % 4 == 1) l.position = v3(0, 3e4f, 0);
        }
        rt_ctx ctx;
        const int rc = rt_set_scene(&ctx, sph.data(), S, nullptr, 0, li.data(), L, v3(0.1f, 0.1f, 0.1f), 3);
        CHECK(rc == RT_OK, "rt_set_scene rc %d", rc);
        const SceneLayout& lay = ctx.layout;
        CHECK(lay.has_shg, "no shadow grid for S=%d L=%d", S, L);
        if (!lay.has_shg) continue;
        const unsigned char* blob = lay.host_blob.data();
        const DevLight* dl = (const DevLight*)(blob + lay.off_li);
        for (int j = 0; j < L; ++j) {
            const DevShadowGrid& g = ((const DevShadowGrid*)(blob + lay.off_shg))[j];
            const unsigned long long* grid = (const unsigned long long*)(blob + lay.off_shgrid) + (size_t)j * SHGRID_N * SHGRID_N;
            const unsigned long long* slab = (const unsigned long long*)(blob + lay.off_shslab) + (size_t)j * (SHGRID_SLABS + 2);
            const DevLight& l = dl[j];
            // the light frame (double) as the host built it
            const double U[3] = {l.ux, l.uy, l.uz}, V[3] = {l.vx, l.vy, l.vz}, A[3] = {l.ax, l.ay, l.az};
            for (int k = 0; k < 3000; ++k) {
                rt_vec3 hp;
                const rt_sphere& s = sph[next64() % (size_t)S];
                const int kind = k % 6;
                if (kind == 0) {  // anywhere around the scene
                    hp = v3(unif(-20, 20) * scale, unif(-3, 6) * scale, unif(-5, 60) * scale);
                } else if (kind == 1) {  // on / just off a sphere's surface
                    const double d[3] = {unif(-1, 1), unif(-1, 1), unif(-1, 1)};
                    const double n = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) + 1e-30;
                    const double r = (double)s.radius * (1.0 + unif(-1e-3f, 1e-2f));
                    hp = v3((float)(s.center.x + r * d[0] / n), (float)(s.center.y + r * d[1] / n),
                            (float)(s.center.z + r * d[2] / n));
                } else if (kind == 2 || kind == 3) {  // a shadow line grazing a sphere (u, v at ~r from it)
                    const double ang = unif(0, 6.2831853f), rr = (double)s.radius * (1.0 + unif(-2e-3f, 2e-2f));
                    const double ax = unif(-30, 10) * scale;  // along the axis, behind or ahead of the sphere
                    double c[3] = {s.center.x, s.center.y, s.center.z};
                    double q[3];
                    for (int e = 0; e < 3; ++e)
                        q[e] = c[e] + rr * (std::cos(ang) * U[e] + std::sin(ang) * V[e]) + ax * A[e];
                    hp = v3((float)q[0], (float)q[1], (float)q[2]);
                } else if (kind == 4) {  // cell / slab edges
                    const int iu = (int)(next64() % (SHGRID_N + 2)) - 1, iv = (int)(next64() % (SHGRID_N + 2)) - 1;
                    const double uu = g.su != 0.0f ? ((double)iu - (double)g.ou) / (double)g.su : 0.0;
                    const double vv = g.sv != 0.0f ? ((double)iv - (double)g.ov) / (double)g.sv : 0.0;
                    const int ia = (int)(next64() % (SHGRID_SLABS + 2)) - 1;
                    const double aa = g.sa != 0.0f ? ((double)ia - (double)g.oa) / (double)g.sa : 0.0;
                    double q[3];
                    for (int e = 0; e < 3; ++e) q[e] = uu * U[e] + vv * V[e] + aa * A[e];
                    hp = v3((float)q[0], (float)q[1], (float)q[2]);
                } else {  // far beyond the table's bound, and non-finite
                    const float f = std::ldexp(1.0f, (int)(next64() % 24));
                    hp = v3(unif(-20, 20) * scale * f, unif(-3, 6) * scale, unif(-5, 60) * scale * f);
                    if (k % 97 == 5) hp.x = NAN;
                    if (k % 89 == 7) hp.z = INFINITY;
                }
                const unsigned long long m = grid_lookup(g, l, grid, slab, hp);
                ++lanes;
                for (int i = 0; i < S; ++i) {
                    if ((m >> i) & 1ull) {
                        ++cands;
                        continue;
                    }
                    int col = 0;
                    oracle_intersect_sphere(hp, li[(size_t)j].position, sph[(size_t)i].center, sph[(size_t)i].radius,
                                            0.001f, &col);
                    ++checked, ++culled;
                    CHECK(!col, "scene %d light %d: sphere %d culled but blocks hp (%a, %a, %a)", it, j, i, hp.x, hp.y,
                          hp.z);
                }
            }
        }
    }
    std::printf("shadow_grid: %ld culled (lane, sphere) pairs checked unblocked, %.2f candidates per lane\n", culled,
                lanes ? (double)cands / (double)lanes : 0.0);
    (void)checked;
}

// The merged pass's level-0 ball cull with hoisted light-independent terms (rt_kernel.hip
// shadow_members_fast, after make_shadow_sphere): for random scenes and random "waves" -- up to 64 hit
// points in a cluster of random spread (tight tiles, scattered deep levels), near sphere surfaces and on
// grazing shadow lines -- a (sphere, light) pair the cull drops must leave every lane's binary32 shadow
// ray unblocked.  The bound is computed as the device does it (float; the device's clen3 uses the
// hardware sqrt, covered by the (1 + 2^-10) inflation of R).
struct Ball {
    float ox, oy, oz, R, omgn;
    bool ok;
};
Ball make_ball(const std::vector<rt_vec3>& hp) {
    Ball b{};
    const rt_vec3 a = hp.front(), z = hp.back();
    b.ox = (a.x + z.x) * 0.5f, b.oy = (a.y + z.y) * 0.5f, b.oz = (a.z + z.z) * 0.5f;
    float e = 0.0f;
    bool bad = false;
    for (const rt_vec3& q : hp) {
        const float dx = q.x - b.ox, dy = q.y - b.oy, dz = q.z - b.oz;
        const float el = std::sqrt(dx * dx + dy * dy + dz * dz);
        bad = bad || !(el < 0x1p40f);
        e = std::max(e, el);
    }
    b.R = e * (1.0f + 0x1p-10f) + 0x1p-60f;
    const float olen = std::sqrt(b.ox * b.ox + b.oy * b.oy + b.oz * b.oz);
    b.omgn = 0x1p-18f * olen * (1.0f + 0x1p-10f);
    b.ok = !bad && b.R < 0x1p38f && olen < 0x1p40f;
    return b;
}
bool ball_keeps(const Ball& b, const DevSphereCull& c, const DevLight& l) {
    const float wx = c.cx - b.ox, wy = c.cy - b.oy, wz = c.cz - b.oz;
    const float dc = (std::fabs(wx) + std::fabs(wy) + std::fabs(wz)) * (1.0f + 0x1p-20f);
    const float c1 = std::fabs(c.cx) + std::fabs(c.cy) + std::fabs(c.cz);
    const float mgn = std::fmaf(0x1p-8f, dc + 3.0f * b.R, b.omgn + 0x1p-18f * c1);
    const float T = b.R + c.rr + mgn;
    const float T2 = T * T, nb = -(b.R + mgn);
    const bool valid = b.ok && c.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f && c1 < 0x1p40f;
    const bool l_ok = l.a >= 0x1p-40f && l.a <= 0x1p40f && l.a2 < INFINITY;
    const float wu = std::fmaf(wz, l.uz, std::fmaf(wy, l.uy, wx * l.ux));
    const float wv = std::fmaf(wz, l.vz, std::fmaf(wy, l.vy, wx * l.vx));
    const float wa = std::fmaf(wz, l.az, std::fmaf(wy, l.ay, wx * l.ax));
    const bool line = std::fmaf(wu, wu, wv * wv) > T2;
    const bool behind = wa < nb;
    return !(valid && l_ok && (line || behind));
}

void check_ball_cull() {
    long culled = 0, pairs = 0;
    for (int it = 0; it < 40; ++it) {
        const float scale = it % 4 == 3 ? 1000.0f : it % 4 == 2 ? 30.0f : 1.0f;
        const int S = 12 + (int)(next64() % 53), L = 1 + (int)(next64() % SHADOW_MERGE_L);
        std::vector<rt_sphere> sph((size_t)S);
        std::vector<rt_light> li((size_t)L);
        for (rt_sphere& q : sph) {
            q.center = v3(unif(-8, 8) * scale, unif(-1, 3) * scale, unif(2, 40) * scale);
            q.radius = unif(0.05f, 1.5f) * scale;
            q.material = material((int)(next64() % 5));
        }
        for (int j = 0; j < L; ++j) {
            li[(size_t)j].position = v3(unif(-40, 40), unif(-5, 20), unif(-20, 40));
            li[(size_t)j].intensity = 1.0f;
            if (j == 1 && it % 3 == 0) li[(size_t)j].position = v3(unif(-40, 40), 1e-3f, unif(-1, 1));
        }
        rt_ctx ctx;
        CHECK(rt_set_scene(&ctx, sph.data(), S, nullptr, 0, li.data(), L, v3(0.1f, 0.1f, 0.1f), 3) == RT_OK, "scene");
        const SceneLayout& lay = ctx.layout;
        const DevLight* dl = (const DevLight*)(lay.host_blob.data() + lay.off_li);
        const DevSphereCull* dc = (const DevSphereCull*)(lay.host_blob.data() + lay.off_cull);
        for (int wv = 0; wv < 300; ++wv) {
            // a wave's hit points: a cluster around a point near a sphere surface, spread from 1e-4 to 10 units
            const rt_sphere& s0 = sph[next64() % (size_t)S];
            const double d0[3] = {unif(-1, 1), unif(-1, 1), unif(-1, 1)};
            const double n0 = std::sqrt(d0[0] * d0[0] + d0[1] * d0[1] + d0[2] * d0[2]) + 1e-30;
            const double rr0 = (double)s0.radius * (1.0 + unif(-1e-3f, 5e-2f));
            const double cx = s0.center.x + rr0 * d0[0] / n0, cy = s0.center.y + rr0 * d0[1] / n0,
                         cz = s0.center.z + rr0 * d0[2] / n0;
            const double spread = std::pow(10.0, unif(-4.0f, 1.0f)) * scale;
            const int k = 1 + (int)(next64() % 64);
            std::vector<rt_vec3> hp((size_t)k);
            for (rt_vec3& q : hp)
                q = v3((float)(cx + spread * unif(-1, 1)), (float)(cy + spread * unif(-1, 1)), (float)(cz + spread * unif(-1, 1)));
            const Ball b = make_ball(hp);
            for (int j = 0; j < L; ++j)
                for (int i = 0; i < S; ++i) {
                    ++pairs;
                    if (ball_keeps(b, dc[i], dl[j])) continue;
                    ++culled;
                    for (const rt_vec3& q : hp) {
                        int col = 0;
                        oracle_intersect_sphere(q, li[(size_t)j].position, sph[(size_t)i].center, sph[(size_t)i].radius,
                                                0.001f, &col);
                        CHECK(!col, "scene %d wave %d light %d: sphere %d culled but blocks (%a, %a, %a)", it, wv, j, i,
                              q.x, q.y, q.z);
                    }
                }
        }
    }
    std::printf("ball_cull: %ld of %ld (sphere, light) pairs culled, every lane checked unblocked\n", culled, pairs);
}

// The per-lane cluster pre-cull (rt_kernel.hip cluster_mask, restated for one lane in binary32 -- the kernel's
// rsq by a correctly rounded 1/sqrt, inside the margins): rays from points on and near sphere surfaces and from
// anywhere in the scene, |d|^2 in [0.5, 2]; for every cluster the lane drops, no member collides under the
// reference's IntersectsSphere (epsilon 0: neither TracePixel's nor TraceSecondaryRay's rule can select it).
bool cluster_keeps(const DevCluster& c, rt_vec3 o, rt_vec3 d) {
    const float a = ((d.x * d.x) + (d.y * d.y)) + (d.z * d.z);
    const float s = 1.0f / std::sqrt(a);
    const float A[3] = {d.x * s, d.y * s, d.z * s};
    const float ol = std::fabs(o.x) + std::fabs(o.y) + std::fabs(o.z);
    const bool ok = a >= 0.5f && a <= 2.0f && ol < 0x1p40f;
    const float w[3] = {c.cx - o.x, c.cy - o.y, c.cz - o.z};
    const float dcl = (std::fabs(w[0]) + std::fabs(w[1]) + std::fabs(w[2])) * (1.0f + 0x1p-20f);
    const float mgn = 0x1p-8f * (dcl + c.R);
    const float x[3] = {std::fma(w[1], A[2], -(w[2] * A[1])), std::fma(w[2], A[0], -(w[0] * A[2])),
                        std::fma(w[0], A[1], -(w[1] * A[0]))};
    const float T = c.R + mgn;
    const bool line = std::fma(x[2], x[2], std::fma(x[1], x[1], x[0] * x[0])) > T * T;
    const bool behind = -std::fma(w[2], A[2], std::fma(w[1], A[1], w[0] * A[0])) - c.R > mgn;
    const bool valid = dcl >= 0x1p-30f && dcl < 0x1p40f;
    return !(ok && valid && (line || behind));
}

void check_cluster_cull() {
    long culled = 0, tests = 0;
    for (int it = 0; it < 30; ++it) {
        const float scale = it % 3 == 2 ? 1000.0f : it % 3 == 1 ? 30.0f : 1.0f;
        const int S = 12 + (int)(next64() % 53);
        std::vector<rt_sphere> sph((size_t)S);
        for (rt_sphere& q : sph) {
            q.center = v3(unif(-8, 8) * scale, unif(-1, 3) * scale, unif(2, 40) * scale);
            q.radius = unif(0.05f, 1.5f) * scale;
            q.material = material((int)(next64() % 5));
        }
        rt_light li{v3(-3, 1, -3), 1.0f};
        rt_ctx ctx;
        CHECK(rt_set_scene(&ctx, sph.data(), S, nullptr, 0, &li, 1, v3(0.1f, 0.1f, 0.1f), 5) == RT_OK, "scene");
        const SceneLayout& lay = ctx.layout;
        CHECK(lay.n_clus == (S + CLUSTER_SIZE - 1) / CLUSTER_SIZE || lay.n_clus > 0, "clusters built for S = %d", S);
        const DevCluster* cl = (const DevCluster*)(lay.host_blob.data() + lay.off_clus);
        for (int r = 0; r < 4000; ++r) {
            rt_vec3 o;
            if (r % 2 == 0) {  // on / near a sphere surface (a reflected segment's origin)
                const rt_sphere& s0 = sph[next64() % (size_t)S];
                const double d0[3] = {unif(-1, 1), unif(-1, 1), unif(-1, 1)};
                const double n0 = std::sqrt(d0[0] * d0[0] + d0[1] * d0[1] + d0[2] * d0[2]) + 1e-30;
                const double rr0 = (double)s0.radius * (1.0 + unif(-1e-6f, 1e-3f));
                o = v3((float)(s0.center.x + rr0 * d0[0] / n0), (float)(s0.center.y + rr0 * d0[1] / n0),
                       (float)(s0.center.z + rr0 * d0[2] / n0));
            } else {
                o = v3(unif(-10, 10) * scale, unif(-2, 5) * scale, unif(-5, 45) * scale);
            }
            double dd[3] = {unif(-1, 1), unif(-1, 1), unif(-1, 1)};
            const double dn = std::sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]) + 1e-30;
            const double len = std::sqrt((double)unif(0.5f, 2.0f));
            const rt_vec3 d = v3((float)(dd[0] / dn * len), (float)(dd[1] / dn * len), (float)(dd[2] / dn * len));
            for (int j = 0; j < lay.n_clus; ++j) {
                ++tests;
                if (cluster_keeps(cl[j], o, d)) continue;
                ++culled;
                for (int i = 0; i < S; ++i) {
                    if (!((cl[j].members >> i) & 1ull)) continue;
                    int col = 0;
                    oracle_intersect_sphere(o, d, sph[(size_t)i].center, sph[(size_t)i].radius, 0.0f, &col);
                    CHECK(!col, "scene %d ray %d: cluster %d culled but sphere %d collides", it, r, j, i);
                }
            }
        }
    }
    std::printf("cluster_cull: %ld of %ld (ray, cluster) tests culled, every member checked\n", culled, tests);
}

// The direct kernel's per-lane shadow pre-test (rt_kernel.hip shadow_pre_lane / shadow_pre_keep, restated in
// binary32 with the same fmas; records from rt_set_scene's build_shadow_pre): random scenes of 1-11 spheres with
// ordinary, grazing, tiny and huge lights, tiny / NaN / far spheres, and hit points on and near sphere surfaces,
// on shadow lines grazing a sphere, anywhere, far away and non-finite.  For every (lane, light, sphere) the
// pre-test drops, the oracle's binary32 IntersectShadowLight test (epsilon 0.001) must find no collision.
bool pre_keeps(const DevLight& l, const DevShadowCull& e, rt_vec3 hp) {
    const float ou = std::fmaf(hp.z, l.uz, std::fmaf(hp.y, l.uy, hp.x * l.ux));
    const float ov = std::fmaf(hp.z, l.vz, std::fmaf(hp.y, l.vy, hp.x * l.vx));
    const float oa = std::fmaf(hp.z, l.az, std::fmaf(hp.y, l.ay, hp.x * l.ax));
    const float l1 = std::fabs(ou) + std::fabs(ov) + std::fabs(oa);
    const float ml = l1 < 0x1p38f ? std::fmaf(l1, 0x1.01p-8f, 0x1p-30f) : INFINITY;
    const float wu = e.cu - ou, wv = e.cv - ov;
    const float T = e.rr + ml;
    const bool line = std::fmaf(wu, wu, wv * wv) > T * T;
    const bool behind = oa - e.ca > ml;
    return !(line || behind);
}

void check_shadow_pre() {
    long culled = 0, pairs = 0;
    for (int it = 0; it < 60; ++it) {
        const float scale = it % 4 == 3 ? 1000.0f : it % 4 == 2 ? 30.0f : it % 8 == 1 ? 1e-3f : 1.0f;
        const int S = 1 + (int)(next64() % (CULL_MIN_SPHERES - 1)), L = 1 + (int)(next64() % 4);
        std::vector<rt_sphere> sph((size_t)S);
        std::vector<rt_light> li((size_t)L);
        for (rt_sphere& q : sph) {
            q.center = v3(unif(-8, 8) * scale, unif(-1, 3) * scale, unif(2, 40) * scale);
            q.radius = unif(0.05f, 1.5f) * scale;
            q.material = material((int)(next64() % 5));
        }
        if (S > 1 && it % 5 == 1) sph[1].radius = 1e-25f;            // r'^2 below the cull's floor: never dropped
        if (S > 2 && it % 6 == 2) sph[2].radius = NAN;
        if (S > 3 && it % 7 == 3) sph[3].center = v3(3e11f, 0, 0);   // |C_f|_1 >= 2^38: never dropped
        for (int j = 0; j < L; ++j) {
            rt_light& l = li[(size_t)j];
            l.position = v3(unif(-40, 40), unif(-5, 20), unif(-20, 40));
            l.intensity = 1.0f;
            if (j == 1 && it % 3 == 0) l.position = v3(unif(-40, 40), 1e-3f, unif(-1, 1));  // grazing
            if (j == 2 && it % 4 == 0) l.position = v3(1e-30f, 0, 0);                      // a below 2^-40
            if (j == 3 && it % 2 == 0) l.position = v3(0, 3e4f, 0);
            if (j == 0 && it % 9 == 4) l.position = v3(0, 0, 0);                           // 2a = 0: literal path
        }
        rt_ctx ctx;
        CHECK(rt_set_scene(&ctx, sph.data(), S, nullptr, 0, li.data(), L, v3(0.1f, 0.1f, 0.1f), 3) == RT_OK, "scene");
        const SceneLayout& lay = ctx.layout;
        CHECK(lay.has_shpre, "pre-test records for S = %d", S);
        if (!lay.has_shpre) continue;
        const int s_pad = S + (S & 1);
        const DevShadowCull* pre = (const DevShadowCull*)(lay.host_blob.data() + lay.off_shpre);
        const DevLight* dl = (const DevLight*)(lay.host_blob.data() + lay.off_li);
        for (int j = 0; j < L; ++j) {
            const DevLight& l = dl[j];
            if (S & 1) CHECK(std::isinf(pre[(size_t)j * s_pad + S].cu), "padding record dropped");
            const double U[3] = {l.ux, l.uy, l.uz}, V[3] = {l.vx, l.vy, l.vz}, A[3] = {l.ax, l.ay, l.az};
            for (int k = 0; k < 4000; ++k) {
                rt_vec3 hp;
                const rt_sphere& s = sph[next64() % (size_t)S];
                const int kind = k % 5;
                if (kind == 0) {
                    hp = v3(unif(-20, 20) * scale, unif(-3, 6) * scale, unif(-5, 60) * scale);
                } else if (kind == 1) {  // on / just off a sphere's surface
                    const double d[3] = {unif(-1, 1), unif(-1, 1), unif(-1, 1)};
                    const double n = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) + 1e-30;
                    const double r = (double)s.radius * (1.0 + unif(-1e-3f, 1e-2f));
                    hp = v3((float)(s.center.x + r * d[0] / n), (float)(s.center.y + r * d[1] / n),
                            (float)(s.center.z + r * d[2] / n));
                } else if (kind == 2 || kind == 3) {  // a shadow line grazing a sphere
                    const double ang = unif(0, 6.2831853f), rr = (double)s.radius * (1.0 + unif(-2e-3f, 2e-2f));
                    const double ax = unif(-30, 10) * scale;
                    double q[3];
                    const double c[3] = {s.center.x, s.center.y, s.center.z};
                    for (int e = 0; e < 3; ++e) q[e] = c[e] + rr * (std::cos(ang) * U[e] + std::sin(ang) * V[e]) + ax * A[e];
                    hp = v3((float)q[0], (float)q[1], (float)q[2]);
                } else {  // far away, and non-finite
                    const float f = std::ldexp(1.0f, (int)(next64() % 40));
                    hp = v3(unif(-20, 20) * scale * f, unif(-3, 6) * scale, unif(-5, 60) * scale * f);
                    if (k % 97 == 4) hp.x = NAN;
                    if (k % 89 == 9) hp.z = INFINITY;
                }
                for (int i = 0; i < S; ++i) {
                    ++pairs;
                    if (pre_keeps(l, pre[(size_t)j * s_pad + i], hp)) continue;
                    ++culled;
                    int col = 0;
                    oracle_intersect_sphere(hp, li[(size_t)j].position, sph[(size_t)i].center, sph[(size_t)i].radius,
                                            0.001f, &col);
                    CHECK(!col, "scene %d light %d: sphere %d dropped but blocks hp (%a, %a, %a)", it, j, i, hp.x, hp.y, hp.z);
                }
            }
        }
    }
    std::printf("shadow_pre: %ld of %ld (lane, light, sphere) triples dropped, each checked unblocked\n", culled, pairs);
}

// Single-frame row order (row_order): a floor below the camera fills the bottom rows (high y), so they
// are dispatched first; a ceiling above it puts the top rows first; with no plane and no sphere every
// row costs the same and the order stays natural.
void check_row_order() {
    for (int k = 0; k < 3; ++k) {
        rt_ctx ctx;
        rt_plane pl{};
        pl.center = v3(0, k == 0 ? -1.0f : 1.0f, 0);
        pl.normal = v3(0, k == 0 ? 1.0f : -1.0f, 0);
        pl.material = material(0);
        rt_light l{v3(0, 5, 0), 1.0f};
        CHECK(rt_set_scene(&ctx, nullptr, 0, &pl, k == 2 ? 0 : 1, &l, 1, v3(0.1f, 0.1f, 0.1f), 1) == RT_OK, "scene");
        rt_camera cam{v3(0, 0, 0), 0, 0};
        rt_set_camera(&ctx, &cam);
        LaunchParams lp;
        std::memset(&lp, 0, sizeof lp);
        CHECK(view_params(&ctx, 1920, 1080, lp) == RT_OK, "view_params");
        CHECK(lp.row_order_n == 135, "row order over %d rows", lp.row_order_n);
        if (k == 0) CHECK(lp.row_order[0] >= 68 && lp.row_order[134] <= 67, "floor: bottom rows first (%d ... %d)", lp.row_order[0], lp.row_order[134]);
        if (k == 1) CHECK(lp.row_order[0] < 67 && lp.row_order[134] >= 67, "ceiling: top rows first (%d ... %d)", lp.row_order[0], lp.row_order[134]);
        if (k == 2)
            for (int r = 0; r < 135; ++r) CHECK(lp.row_order[r] == r, "empty scene: natural order at %d", r);
    }
}

void check_library() {
    CHECK(rt_abi_version() == RT_ABI_VERSION, "ABI version");
    int n = -1;
    CHECK(rt_device_count(&n) == RT_OK && n >= 0, "device count");
    rt_ctx* ctx = nullptr;
    CHECK(rt_create_ex(1, 0x100, &ctx) == RT_ERR_INVALID_ARG && !ctx, "unknown flag");
    CHECK(rt_create(0, &ctx) == RT_ERR_INVALID_ARG, "zero GPUs");
    if (n == 0) {
        CHECK(rt_create(1, &ctx) == RT_ERR_NO_DEVICE && !ctx, "no CPU fallback");
        CHECK(std::strstr(rt_last_error(nullptr), "no HIP device") != nullptr, "last error text");
    }
    rt_destroy(nullptr);
}
}  // namespace

// tiles_by_cost (the measured dispatch order): a permutation of the tiles, by decreasing cost in the sort's
// buckets, natural order inside a bucket; costs past 2^20 ticks take wider buckets.
void check_tiles_by_cost() {
    uint64_t seed = 12345;
    auto rnd = [&]() { seed = seed * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(seed >> 33); };
    long checked = 0;
    for (int trial = 0; trial < 40; ++trial) {
        const uint32_t tx = 1 + rnd() % 300, ty = 1 + rnd() % 200;
        const size_t n = (size_t)tx * ty;
        const uint32_t range = trial % 4 == 0 ? 0xffffffffu : trial % 4 == 1 ? 5000u : trial % 4 == 2 ? (1u << 22) : 17u;
        std::vector<uint32_t> cost(n), order(n);
        for (auto& c : cost) c = range == 0xffffffffu ? rnd() * 2u + (rnd() & 1u) : rnd() % (range + 1);
        tiles_by_cost(cost.data(), n, tx, order.data());
        uint32_t cmax = 0;
        for (uint32_t c : cost) cmax = std::max(cmax, c);
        const int shift = cmax >> 4 < (1u << 16) ? 4 : 4 + (32 - __builtin_clz(cmax >> 20 | 1u));
        std::vector<char> seen(n, 0);
        for (size_t k = 0; k < n; ++k) {
            const uint32_t x = order[k] & 0xffffu, y = order[k] >> 16;
            CHECK(x < tx && y < ty, "tile in range");
            const size_t t = (size_t)y * tx + x;
            CHECK(!seen[t], "each tile once");
            seen[t] = 1;
            if (k) {
                const uint32_t px = order[k - 1] & 0xffffu, py = order[k - 1] >> 16;
                const size_t pt = (size_t)py * tx + px;
                const uint32_t b0 = cost[pt] >> shift, b1 = cost[t] >> shift;
                CHECK(b0 > b1 || (b0 == b1 && pt < t), "decreasing buckets, natural order inside one");
            }
        }
        checked += (long)n;
    }
    std::printf("tiles_by_cost: %ld tiles\n", checked);
}

// build_clusters (the bundle kernel's per-lane pre-cull): the clusters partition the spheres, hold at most
// `size` members each, and every member's ball (centre, cull radius r') lies inside its cluster's bounding
// sphere, checked in double from the float records the kernel reads; a member with an unusable record
// (NaN / infinite centre or radius) leaves its cluster's R NaN (never culled).
void check_clusters() {
    long checked = 0;
    for (int trial = 0; trial < 300; ++trial) {
        const int S = 1 + (int)(next64() % 64), size = 1 + (int)(next64() % 8);
        const float scale = trial % 3 == 0 ? 1.0f : trial % 3 == 1 ? 30.0f : 1000.0f;
        std::vector<DevSphereCull> cull((size_t)S);
        for (int i = 0; i < S; ++i) {
            const float r = unif(0.001f, 1.0f) * scale;
            cull[(size_t)i] = DevSphereCull{unif(-8, 8) * scale, unif(-1, 1) * scale, unif(4, 32) * scale,
                                            std::nextafter((float)(std::sqrt((double)(r * r)) * (1.0 + 0x1p-8)), INFINITY)};
            if (trial % 7 == 3 && i == S / 2) cull[(size_t)i].cx = trial % 2 ? NAN : INFINITY;  // unusable record
            if (trial % 11 == 5 && i == 0) cull[(size_t)i].rr = NAN;
        }
        DevCluster c[MAX_CLUSTERS];
        const int n = build_clusters(cull.data(), S, size, c);
        if ((S + size - 1) / size > MAX_CLUSTERS) {  // (median splits give at most 2 S / size groups)
            CHECK(n == 0 || n <= MAX_CLUSTERS, "cluster count within the table");
            if (n == 0) continue;
        }
        CHECK(n >= 1 && n <= MAX_CLUSTERS, "cluster count %d (S %d size %d)", n, S, size);
        unsigned long long all = 0;
        for (int j = 0; j < n; ++j) {
            CHECK((all & c[j].members) == 0, "clusters disjoint");
            all |= c[j].members;
            CHECK(__builtin_popcountll(c[j].members) <= size && c[j].members != 0, "cluster size");
            bool usable = true;
            for (int i = 0; i < S; ++i) {
                if (!((c[j].members >> i) & 1ull)) continue;
                const DevSphereCull& s = cull[(size_t)i];
                if (!(std::isfinite(s.cx) && std::isfinite(s.cy) && std::isfinite(s.cz) && std::isfinite(s.rr))) {
                    usable = false;
                    continue;
                }
                const double dx = (double)s.cx - c[j].cx, dy = (double)s.cy - c[j].cy, dz = (double)s.cz - c[j].cz;
                CHECK(std::sqrt(dx * dx + dy * dy + dz * dz) + (double)s.rr <= (double)c[j].R || std::isnan(c[j].R),
                      "member ball inside the cluster bound");
                ++checked;
            }
            CHECK(usable || std::isnan(c[j].R), "unusable member -> NaN bound");
        }
        CHECK(all == (S == 64 ? ~0ull : (1ull << S) - 1ull), "every sphere in one cluster");
    }
    std::printf("clusters: %ld member bounds\n", checked);
}

int main() {
    check_library();
    check_clusters();
    check_scene_packing();
    check_camera_input();
    check_ppm();
    check_wire_layout();
    check_shadow_threshold();
    check_tiles_by_cost();
    check_shadow_grid();
    check_shadow_pre();
    check_ball_cull();
    check_cluster_cull();
    check_row_order();
    std::printf("san_host: %d failures\n", failures);
    return failures ? 1 : 0;
}
