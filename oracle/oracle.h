/*
 * oracle.h -- CPU restatement of the reference ray tracer, TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (libraytracer_hip) never links or calls it.
 *
 * PARITY UNPINNED by the reference itself: TobiasDeBruijn/UU-INFOGR-Raytracer ships no
 * tests, fixtures or golden images, and its C#/.NET 6 + OpenTK 4.7.1 build cannot run
 * in this image (no dotnet/mono, no NuGet cache).  The restatement is
 * cross-checked instead against an independent numpy float32 emulation
 * (tests/emu_f32.py) and pinned by hand-derived known-answer tests.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/raytracer_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    ORACLE_MODE_REFERENCE = 0, /* all-hit recursive trace, per-pixel camera basis,
                                  column-outer / row-parallel loop (RayTracer.cs:898-901) */
    ORACLE_MODE_NEAREST = 1    /* nearest-hit-only recursive restatement with ray counts */
};

typedef struct oracle_stats {
    uint64_t pixels;
    uint64_t primary_rays;
    uint64_t reflect_rays;
    uint64_t shadow_rays;
} oracle_stats;

/* Render rows [row_begin, row_end) of a width x height frame into
 * pixels[(y-row_begin)*width + x].  nthreads <= 0 means 1. */
int oracle_render(const rt_sphere* spheres, int n_spheres,
                  const rt_plane* planes, int n_planes,
                  const rt_light* lights, int n_lights,
                  rt_vec3 ambient, int recursion_limit,
                  const rt_camera* camera, int width, int height,
                  int row_begin, int row_end,
                  int32_t* pixels, int mode, int nthreads, oracle_stats* stats);

/* Visible-path segments (float hit records) of every stride-th pixel, in each pixel's walk
 * order -- the checker for rt_debug_segments.  *out_count receives the total. */
int oracle_segments(const rt_sphere* spheres, int n_spheres,
                    const rt_plane* planes, int n_planes,
                    const rt_light* lights, int n_lights,
                    rt_vec3 ambient, int recursion_limit,
                    const rt_camera* camera, int width, int height, int stride,
                    rt_segment* out, int capacity, int* out_count);

/* Per-function known-answer entry points. */
float oracle_intersect_sphere(rt_vec3 origin, rt_vec3 direction, rt_vec3 center,
                              float radius, float epsilon, int* collision);
float oracle_intersect_plane(rt_vec3 origin, rt_vec3 direction, rt_vec3 center,
                             rt_vec3 normal, int* collision);
int32_t oracle_shift_color(rt_vec3 color);
int oracle_camera_view(const rt_camera* camera, int width, int height, rt_view* out);
int32_t oracle_net_float_to_int(float v);

#ifdef __cplusplus
}
#endif
#endif
