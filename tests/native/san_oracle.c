/*
 * san_oracle.c -- host sanitizer driver for the CPU restatement (oracle/oracle.c), TEST
 * INFRASTRUCTURE ONLY ("host ASan/UBSan build of the oracle and the C ABI").
 *
 * Built twice by tests/native/Makefile: with AddressSanitizer + UndefinedBehaviorSanitizer
 * (every check fatal) and with ThreadSanitizer.  The TSan build checks the invariant the
 * reference's parallel loop relies on (RayTracer.cs:898-901, :1038): every worker of the
 * column-outer / row-parallel loop writes a disjoint set of pixels, so the frame is race-free.
 *
 * Scenes: the verbatim reference scene (RayTracer.cs:441-469, limit 32) and seeded random
 * scenes with every material kind, generic specular exponents, degenerate primitives (zero
 * radius, NaN radius, zero normal) and cameras far away / inside a sphere.  For each scene:
 * the all-hit and nearest-hit drivers agree pixel for pixel, 1 and 4 threads agree, a row
 * range equals the slice of the whole frame, and the debug segment list is bounded by its
 * capacity.  Exit status 0 = all checks passed (sanitizer reports abort the process).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/oracle.h"

static uint64_t rng_state;
static uint64_t next64(void) { /* SplitMix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static float unif(float lo, float hi) { return lo + (hi - lo) * (float)((next64() >> 40) * (1.0 / 16777216.0)); }
static rt_vec3 v3(float x, float y, float z) { rt_vec3 v = {x, y, z}; return v; }
static rt_vec3 rcol(void) { return v3(unif(0, 1), unif(0, 1), unif(0, 1)); }

static rt_material mat_of(int kind) {
    rt_material m;
    memset(&m, 0, sizeof m);
    rt_vec3 c = rcol();
    switch (kind % 6) {
        case 0: m.kd = c, m.ka = c; break;                                             /* diffuse */
        case 1: m.kd = c, m.ka = c, m.ks = v3(0.4f, 0.4f, 0.4f), m.n = 1.0f; break;    /* plastic */
        case 2: m.kd = c, m.ka = c, m.ks = c, m.n = 0.5f; break;                       /* metal   */
        case 3: m.km = v3(1, 1, 1); break;                                             /* mirror  */
        case 4: m.kd = c, m.ka = c, m.km = v3(0.5f, 0.5f, 0.5f); break;                /* diffuse mirror */
        default: m.kd = c, m.ka = c, m.ks = c, m.n = unif(2.5f, 20.0f); break;         /* generic pow */
    }
    return m;
}

typedef struct {
    rt_sphere sph[24];
    rt_plane pl[3];
    rt_light li[4];
    int ns, np, nl, limit, w, h;
    rt_vec3 ambient;
    rt_camera cam;
} TScene;

static void reference_scene(TScene* s) {
    memset(s, 0, sizeof *s);
    const float amb = 43.0f / 255.0f;
    s->ambient = v3(amb, amb, amb);
    s->ns = 3, s->np = 1, s->nl = 2, s->limit = 32, s->w = 64, s->h = 48;
    s->sph[0].center = v3(2.5f, 0, 8), s->sph[0].radius = 1, s->sph[0].material.kd = s->sph[0].material.ka = v3(1, 0, 0);
    s->sph[1].center = v3(3, 0, 5), s->sph[1].radius = 1, s->sph[1].material.kd = s->sph[1].material.ka = v3(0, 1, 0);
    s->sph[1].material.ks = v3(0.4f, 0.4f, 0.4f), s->sph[1].material.n = 1.0f;
    s->sph[2].center = v3(-3, 1, 8), s->sph[2].radius = 1, s->sph[2].material.km = v3(1, 1, 1);
    s->pl[0].center = v3(0, -1, 0), s->pl[0].normal = v3(0, 1, 0);
    s->pl[0].material.kd = v3(1, 1, 1), s->pl[0].material.ka = v3(0.5f, 0.5f, 0.5f);
    s->pl[0].material.ks = v3(1, 1, 1), s->pl[0].material.n = 0.5f, s->pl[0].material.km = v3(1, 1, 1);
    s->li[0].position = v3(-3, 1, -3), s->li[0].intensity = 1;
    s->li[1].position = v3(33, 1, 10), s->li[1].intensity = 1;
}

static void random_scene(TScene* s, int idx) {
    memset(s, 0, sizeof *s);
    s->ambient = v3(unif(0, 0.3f), unif(0, 0.3f), unif(0, 0.3f));
    s->ns = (int)(next64() % 24), s->np = (int)(next64() % 4), s->nl = (int)(next64() % 5);
    s->limit = (int)(next64() % 9);
    s->w = 17 + (int)(next64() % 40), s->h = 9 + (int)(next64() % 30);
    for (int i = 0; i < s->ns; ++i) {
        s->sph[i].center = v3(unif(-6, 6), unif(-1, 3), unif(2, 20));
        s->sph[i].radius = unif(0.2f, 1.5f);
        s->sph[i].material = mat_of((int)(next64() % 6));
    }
    if (s->ns > 2) s->sph[0].radius = 0.0f;      /* degenerate sphere */
    if (s->ns > 3 && idx % 3 == 0) s->sph[1].radius = NAN;
    for (int i = 0; i < s->np; ++i) {
        s->pl[i].center = v3(unif(-2, 2), unif(-2, 0), unif(0, 30));
        s->pl[i].normal = v3(unif(-0.3f, 0.3f), 1.0f, unif(-0.3f, 0.3f));
        s->pl[i].material = mat_of((int)(next64() % 6));
    }
    if (s->np > 1 && idx % 4 == 1) s->pl[1].normal = v3(0, 0, 0);  /* degenerate plane */
    for (int i = 0; i < s->nl; ++i) s->li[i].position = v3(unif(-30, 30), unif(0, 15), unif(-10, 30)), s->li[i].intensity = unif(0.2f, 1.0f);
    s->cam.position = v3(unif(-1, 1), unif(-0.5f, 1), unif(-2, 1));
    s->cam.yaw = unif(-0.5f, 0.5f), s->cam.pitch = unif(-0.3f, 0.3f);
    if (idx % 5 == 2 && s->ns > 4) s->cam.position = s->sph[4].center;  /* camera inside a sphere */
    if (idx % 7 == 3) s->cam.position = v3(1e6f, 1e5f, -1e6f);           /* far camera */
}

static int failures;
#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);           \
            fprintf(stderr, __VA_ARGS__);                                  \
            fputc('\n', stderr);                                           \
            ++failures;                                                    \
        }                                                                  \
    } while (0)

static int render(const TScene* s, int mode, int threads, int r0, int r1, int32_t* px, oracle_stats* st) {
    return oracle_render(s->sph, s->ns, s->pl, s->np, s->li, s->nl, s->ambient, s->limit, &s->cam, s->w, s->h, r0, r1,
                         px, mode, threads, st);
}

static void check_scene(const TScene* s, const char* name) {
    const size_t n = (size_t)s->w * s->h;
    /* exact-size heap buffers: ASan flags any store outside the frame */
    int32_t* ref1 = (int32_t*)malloc(n * sizeof(int32_t));
    int32_t* ref4 = (int32_t*)malloc(n * sizeof(int32_t));
    int32_t* near4 = (int32_t*)malloc(n * sizeof(int32_t));
    oracle_stats a, b;
    CHECK(render(s, ORACLE_MODE_REFERENCE, 1, 0, s->h, ref1, NULL) == RT_OK, "%s: reference 1 thread", name);
    CHECK(render(s, ORACLE_MODE_REFERENCE, 4, 0, s->h, ref4, NULL) == RT_OK, "%s: reference 4 threads", name);
    CHECK(render(s, ORACLE_MODE_NEAREST, 4, 0, s->h, near4, &a) == RT_OK, "%s: nearest 4 threads", name);
    CHECK(memcmp(ref1, ref4, n * sizeof(int32_t)) == 0, "%s: 1 vs 4 threads differ", name);
    CHECK(memcmp(ref1, near4, n * sizeof(int32_t)) == 0, "%s: all-hit vs nearest-hit differ", name);
    int32_t* near1 = (int32_t*)malloc(n * sizeof(int32_t));
    CHECK(render(s, ORACLE_MODE_NEAREST, 1, 0, s->h, near1, &b) == RT_OK, "%s: nearest 1 thread", name);
    CHECK(a.primary_rays == b.primary_rays && a.reflect_rays == b.reflect_rays && a.shadow_rays == b.shadow_rays,
          "%s: ray counts depend on the thread count", name);
    CHECK(a.primary_rays == n, "%s: primary rays %llu != pixels", name, (unsigned long long)a.primary_rays);
    /* a row range writes only its rows, packed from row_begin */
    const int r0 = s->h / 3, r1 = s->h - s->h / 4;
    const size_t m = (size_t)(r1 - r0) * s->w;
    int32_t* part = (int32_t*)malloc((m ? m : 1) * sizeof(int32_t));
    CHECK(render(s, ORACLE_MODE_REFERENCE, 3, r0, r1, part, NULL) == RT_OK, "%s: row range", name);
    CHECK(memcmp(part, ref1 + (size_t)r0 * s->w, m * sizeof(int32_t)) == 0, "%s: row range differs", name);
    /* debug segments: the count is the total, the stores stop at the capacity */
    int total = -1, got = -1;
    CHECK(oracle_segments(s->sph, s->ns, s->pl, s->np, s->li, s->nl, s->ambient, s->limit, &s->cam, s->w, s->h, 7,
                          NULL, 0, &total) == RT_OK, "%s: segment count", name);
    const int cap = total / 2 + 1;
    rt_segment* seg = (rt_segment*)malloc((size_t)cap * sizeof(rt_segment));
    CHECK(oracle_segments(s->sph, s->ns, s->pl, s->np, s->li, s->nl, s->ambient, s->limit, &s->cam, s->w, s->h, 7,
                          seg, cap, &got) == RT_OK, "%s: segments", name);
    CHECK(got == total, "%s: segment total %d vs %d", name, got, total);
    free(seg);
    free(part);
    free(near1);
    free(near4);
    free(ref4);
    free(ref1);
}

int main(int argc, char** argv) {
    int n_random = argc > 1 ? atoi(argv[1]) : 24;
    TScene s;
    reference_scene(&s);
    check_scene(&s, "reference");
    rng_state = 0x5A417C0DEull;
    for (int i = 0; i < n_random; ++i) {
        char name[32];
        snprintf(name, sizeof name, "random%d", i);
        random_scene(&s, i);
        check_scene(&s, name);
    }
    /* argument validation */
    int32_t px[4];
    rt_camera cam;
    memset(&cam, 0, sizeof cam);
    rt_vec3 amb = {0, 0, 0};
    CHECK(oracle_render(NULL, 1, NULL, 0, NULL, 0, amb, 0, &cam, 2, 2, 0, 2, px, 0, 1, NULL) == RT_ERR_INVALID_ARG,
          "NULL spheres accepted");
    CHECK(oracle_render(NULL, 0, NULL, 0, NULL, 0, amb, 0, &cam, 2, 2, 1, 3, px, 0, 1, NULL) == RT_ERR_INVALID_ARG,
          "row_end > height accepted");
    CHECK(oracle_net_float_to_int(NAN) == INT32_MIN && oracle_net_float_to_int(3e9f) == INT32_MIN &&
          oracle_net_float_to_int(-2.5f) == -2, ".NET (int) semantics");
    printf("san_oracle: %d scenes, %d failures\n", n_random + 1, failures);
    return failures ? 1 : 0;
}
