/*
 * oracle.c -- CPU restatement of Raytracer/RayTracer.cs (TEST INFRASTRUCTURE ONLY).
 *
 * Follows the reference operation by operation.  Every float operation is a single
 * IEEE binary32 operation (x86-64 SSE, compiled with -ffp-contract=off and no
 * fast-math), exactly as .NET 6 RyuJIT executes the C# source; the places where the
 * reference goes through double precision (Math.Sqrt/Pow/Tan/Sin/Cos/Floor) do the same
 * here, through glibc libm, which is what .NET's Math.* calls on Linux x64.
 *
 * .NET / OpenTK 4.7.1 semantics restated (third-party, not vendored in the reference):
 *   Math.Max/Min(float,float)  IEEE 754-2019 maximum/minimum: NaN propagates, -0 < +0
 *   Math.Clamp(float,...)      NaN passes through
 *   (int)float, (int)double    cvttss2si/cvttsd2si: NaN / out of range -> INT_MIN
 *   Vector3.Dot                (x*x') + (y*y') + (z*z')
 *   Vector3.Length             MathF.Sqrt((x*x) + (y*y) + (z*z))
 *   Vector3.Normalize(d)       s = 1f / Length;  (x*s, y*s, z*s)
 *   Vector3.Cross              (y*z' - z*y', z*x' - x*z', x*y' - y*x')
 *   MathHelper.DegreesToRadians(d) = d * (MathF.PI / 180f)
 *
 * PARITY UNPINNED by the reference (no tests / fixtures / runnable build); see oracle.h.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* .NET semantics                                                            */
/* ------------------------------------------------------------------------- */

typedef rt_vec3 v3;

static int is_neg(float f) { return signbit(f) != 0; }

/* System.Math.Max(float, float), .NET Core 3.0+ */
static float net_max(float a, float b) {
    if (a != b) {
        if (!isnan(a)) return b < a ? a : b;
        return a;
    }
    return is_neg(b) ? a : b;
}

/* System.Math.Min(float, float), .NET Core 3.0+ */
static float net_min(float a, float b) {
    if (a != b) {
        if (!isnan(a)) return a < b ? a : b;
        return a;
    }
    return is_neg(a) ? a : b;
}

/* System.Math.Clamp(float, float, float) */
static float net_clamp(float v, float lo, float hi) {
    if (v < lo) return lo;
    if (v > hi) return hi;
    return v;
}

/* (int)x for float/double on .NET 6 x64 (cvttss2si / cvttsd2si). */
static int32_t net_f2i(float v) {
    if (v >= -2147483648.0f && v < 2147483648.0f) return (int32_t)v;
    return INT32_MIN;
}
static int32_t net_d2i(double v) {
    if (v > -2147483649.0 && v < 2147483648.0) return (int32_t)v;
    return INT32_MIN;
}

int32_t oracle_net_float_to_int(float v) { return net_f2i(v); }

/* OpenTK.Mathematics.Vector3 */
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static float vdot(v3 a, v3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
static float vlength(v3 a) { return sqrtf(((a.x * a.x) + (a.y * a.y)) + (a.z * a.z)); }
static v3 vnormalize(v3 a) {
    float s = 1.0f / vlength(a);
    return V(a.x * s, a.y * s, a.z * s);
}
static v3 vcross(v3 l, v3 r) {
    return V((l.y * r.z) - (l.z * r.y), (l.z * r.x) - (l.x * r.z), (l.x * r.y) - (l.y * r.x));
}
static int vis_zero(v3 a) { return a.x == 0 && a.y == 0 && a.z == 0; } /* VecUtil.IsZero :52-54 */
static v3 vmax_s(v3 a, float s) {                                       /* VecUtil.Max :39-45 */
    return V(net_max(a.x, s), net_max(a.y, s), net_max(a.z, s));
}
static v3 vfrom(float f) { return V(f, f, f); }                          /* VecUtil.FromFloat3 */

/* ------------------------------------------------------------------------- */
/* Scene                                                                      */
/* ------------------------------------------------------------------------- */

typedef struct {
    v3 center;
    float radius;
    float radius_sq; /* radius * radius, RayTracer.cs:336 */
    rt_material m;
} Sphere;

typedef struct {
    v3 center, normal;
    rt_material m;
} Plane;

typedef struct {
    const Sphere* sph;
    int ns;
    const Plane* pl;
    int np;
    const rt_light* li;
    int nl;
    v3 ambient;
    int limit;
    /* camera state (RayTracer.cs:494-502) */
    v3 cam_pos;
    float yaw, pitch;
    int width, height;
    v3 view_params;
} Scene;

/* Material flags, RayTracer.cs:85-93 */
static int m_is_mirror(const rt_material* m) { return !vis_zero(m->km); }
static int m_is_diffuse(const rt_material* m) { return !vis_zero(m->kd); }
static int m_has_spec(const rt_material* m) { return !vis_zero(m->ks) && m->n > 0.0f; }

/* Camera basis, RayTracer.cs:511-523 (double trig, cast to float per component). */
static v3 cam_forward(const Scene* s) {
    double p = (double)s->pitch, y = (double)s->yaw;
    return V((float)(cos(p) * sin(y)), (float)-sin(p), (float)(cos(p) * cos(y)));
}
static v3 cam_right(const Scene* s) {
    double y = (double)s->yaw;
    return V((float)cos(y), 0.0f, (float)-sin(y));
}
static v3 cam_up(const Scene* s) { return vcross(cam_right(s), cam_forward(s)); }

/* Tick() view params, RayTracer.cs:892-896 */
static v3 view_params(int width, int height) {
    const float near_clip = 0.3f, fov = 60.0f;
    const float deg2rad = (float)M_PI / 180.0f;              /* MathF.PI / 180f */
    float rad = (fov * 0.5f) * deg2rad;                       /* DegreesToRadians */
    float plane_height = near_clip * (float)tan((double)rad) * 2;
    float aspect = (float)width / (float)height;
    float plane_width = plane_height * aspect;
    return V(plane_width, plane_height, near_clip);
}

int oracle_camera_view(const rt_camera* c, int width, int height, rt_view* out) {
    if (!c || !out || width <= 0 || height <= 0) return RT_ERR_INVALID_ARG;
    Scene s;
    memset(&s, 0, sizeof s);
    s.yaw = c->yaw;
    s.pitch = c->pitch;
    out->position = c->position;
    out->right = cam_right(&s);
    out->up = cam_up(&s);
    out->forward = cam_forward(&s);
    v3 vp = view_params(width, height);
    out->plane_width = vp.x;
    out->plane_height = vp.y;
    out->near_clip = vp.z;
    return RT_OK;
}

/* ------------------------------------------------------------------------- */
/* Intersection, RayTracer.cs:573-642                                         */
/* ------------------------------------------------------------------------- */

typedef struct {
    int collision;
    float distance;
} Isect;

/* IntersectsSphere, RayTracer.cs:613-642 */
static Isect intersect_sphere(v3 o, v3 d, const Sphere* sp, float epsilon) {
    Isect r = {0, 0.0f};
    v3 oc = vsub(o, sp->center);
    float a = vdot(d, d);
    float b = 2 * vdot(oc, d);
    float c = vdot(oc, oc) - sp->radius_sq;
    float disc = b * b - 4 * a * c; /* (b*b) - ((4*a)*c) */
    if (disc >= 0) {
        float dsqrt = (float)sqrt((double)disc);
        float a2 = 2 * a;
        float distance2 = (-b + dsqrt) / a2;
        float distance1 = (-b - dsqrt) / a2;
        float d1eps = distance1 - epsilon;
        float d2eps = distance2 - epsilon;
        float distance = net_min(net_max(distance1, 0), net_max(distance2, 0));
        float distance_eps = net_min(net_max(d1eps, 0), net_max(d2eps, 0));
        if (distance_eps > 0) {
            r.collision = 1;
            r.distance = distance;
        }
    }
    return r;
}

/* IntersectPlane, RayTracer.cs:590-604 */
static Isect intersect_plane(v3 o, v3 d, const Plane* p) {
    Isect r = {0, 0.0f};
    float t = (-o.x * p->normal.x - o.y * p->normal.y - o.z * p->normal.z +
               vdot(p->center, p->normal)) /
              vdot(d, p->normal);
    if (t > 0) {
        r.collision = 1;
        r.distance = t;
    }
    return r;
}

float oracle_intersect_sphere(rt_vec3 o, rt_vec3 d, rt_vec3 center, float radius, float eps,
                              int* collision) {
    Sphere s;
    memset(&s, 0, sizeof s);
    s.center = center;
    s.radius = radius;
    s.radius_sq = radius * radius;
    Isect r = intersect_sphere(o, d, &s, eps);
    if (collision) *collision = r.collision;
    return r.distance;
}

float oracle_intersect_plane(rt_vec3 o, rt_vec3 d, rt_vec3 center, rt_vec3 normal, int* collision) {
    Plane p;
    memset(&p, 0, sizeof p);
    p.center = center;
    p.normal = normal;
    Isect r = intersect_plane(o, d, &p);
    if (collision) *collision = r.collision;
    return r.distance;
}

/* IntersectShadowLight, RayTracer.cs:573-582: origin = hit point, direction = the
 * light's POSITION, spheres only, epsilon 0.001, no early exit (kept here). */
static float shadow_light(const Scene* s, v3 hp, const rt_light* l, oracle_stats* st) {
    if (st) st->shadow_rays++;
    int blocked = 0;
    for (int i = 0; i < s->ns; ++i)
        if (intersect_sphere(hp, l->position, &s->sph[i], 0.001f).collision) blocked = 1;
    return blocked ? 0.0f : l->intensity;
}

/* ------------------------------------------------------------------------- */
/* Shading, RayTracer.cs:652-720                                              */
/* ------------------------------------------------------------------------- */

/* ShapePhongShading, RayTracer.cs:665-695 */
static v3 shape_phong(v3 hp, v3 ray_dir, v3 normal, const rt_material* m, const rt_light* l) {
    v3 light_dir = vnormalize(vsub(l->position, hp));
    v3 view = vnormalize(ray_dir);
    v3 diffuse = V(0, 0, 0);
    if (m_is_diffuse(m)) {
        float angle = vdot(normal, light_dir);
        diffuse = vscale(m->kd, net_max(0, angle));
    }
    v3 specular = V(0, 0, 0);
    if (m_has_spec(m)) {
        v3 spec_dir = vsub(light_dir, vscale(normal, 2 * vdot(light_dir, normal)));
        float spec = vdot(view, vnormalize(spec_dir));
        specular = vmul(m->ks, vfrom((float)pow((double)net_max(0, spec), (double)m->n)));
    }
    return vadd(diffuse, specular);
}

/* CalculateReflectionRay, RayTracer.cs:718-720 */
static v3 reflect(v3 v, v3 n) { return vsub(v, vscale(n, 2 * vdot(v, n))); }

/* Checkerboard tile, RayTracer.cs:757-771 (the e1 == 0 fallback is dead code --
 * Normalize(0) is NaN -- but is restated anyway). */
static float checker(const Plane* p, v3 hp) {
    v3 e1 = vnormalize(vcross(p->normal, V(1.0f, 0.0f, 0.0f)));
    if (e1.x == 0 && e1.y == 0 && e1.z == 0) e1 = vnormalize(vcross(p->normal, V(0, 0, 1)));
    v3 e2 = vnormalize(vcross(p->normal, e1));
    float u = vdot(e1, hp);
    float v = vdot(e2, hp);
    uint32_t sum = (uint32_t)net_f2i(u) + (uint32_t)net_f2i(v); /* unchecked int add */
    return (float)(int32_t)(sum & 1u);
}

/* ------------------------------------------------------------------------- */
/* Reference-faithful recursive trace, RayTracer.cs:729-876                   */
/* ------------------------------------------------------------------------- */

typedef struct {
    float distance;
    v3 color;
} TraceResult;

static v3 trace_secondary(const Scene* s, v3 hp, v3 dir, int count);

/* TracePlane, RayTracer.cs:729-780 */
static TraceResult trace_plane(const Scene* s, v3 o, v3 d, const Plane* p, int count) {
    TraceResult res;
    Isect ir = intersect_plane(o, d, p);
    res.distance = ir.distance;
    if (!ir.collision || ir.distance - 0.01f <= 0) {
        res.color = V(0, 0, 0);
        return res;
    }
    if (count > s->limit) {
        res.color = V(1, 1, 1);
        return res;
    }
    v3 hp = vadd(o, vscale(d, ir.distance));
    v3 color = V(0, 0, 0);
    if (m_is_mirror(&p->m)) {
        count++;
        v3 rd = reflect(d, p->normal);
        color = vadd(color, vmul(trace_secondary(s, hp, rd, count), p->m.km));
    }
    if (m_is_diffuse(&p->m))
        for (int i = 0; i < s->nl; ++i) {
            const rt_light* l = &s->li[i];
            float li = shadow_light(s, hp, l, NULL);
            v3 irgb = vfrom(li);
            float att = (float)(1 / pow((double)ir.distance, 2));
            float tile = checker(p, hp); /* isTiled is always true, :289 */
            v3 term = vmul(vmul(vscale(irgb, att), shape_phong(hp, d, p->normal, &p->m, l)),
                           vfrom(tile));
            color = vadd(color, vmax_s(term, 0.0f));
        }
    color = vadd(color, vmul(s->ambient, p->m.ka));
    res.color = color;
    return res;
}

/* TraceSphere, RayTracer.cs:835-876 */
static TraceResult trace_sphere(const Scene* s, v3 o, v3 d, const Sphere* sp, int count) {
    TraceResult res;
    Isect ir = intersect_sphere(o, d, sp, 0.0f);
    res.distance = ir.distance;
    if (!ir.collision || ir.distance - 0.01f <= 0) {
        res.color = V(0, 0, 0);
        return res;
    }
    if (count > s->limit) {
        res.color = V(0, 0, 0);
        return res;
    }
    v3 hp = vadd(o, vscale(d, ir.distance));
    v3 color = V(0, 0, 0);
    if (m_is_mirror(&sp->m)) {
        count++;
        v3 rd = reflect(d, vnormalize(vsub(hp, sp->center)));
        color = vadd(color, vmul(trace_secondary(s, hp, rd, count), sp->m.km));
    }
    if (m_is_diffuse(&sp->m))
        for (int i = 0; i < s->nl; ++i) {
            const rt_light* l = &s->li[i];
            float li = shadow_light(s, hp, l, NULL);
            v3 irgb = vfrom(li);
            float att = 1 / ir.distance * ir.distance; /* (1/t)*t, :866 */
            v3 normal = vnormalize(vsub(hp, sp->center)); /* SpherePhongShading :706 */
            color = vadd(color, vmul(vscale(irgb, att), shape_phong(hp, d, normal, &sp->m, l)));
        }
    color = vadd(color, vmul(s->ambient, sp->m.ka));
    res.color = color;
    return res;
}

/* TraceSecondaryRay, RayTracer.cs:789-826 */
static v3 trace_secondary(const Scene* s, v3 hp, v3 dir, int count) {
    float closest_sphere = INFINITY;
    v3 sphere_color = V(0, 0, 0);
    for (int i = 0; i < s->ns; ++i) {
        TraceResult r = trace_sphere(s, hp, dir, &s->sph[i], count);
        if (r.distance - 0.01f > 0 && r.distance - 0.01f < closest_sphere) {
            closest_sphere = r.distance;
            sphere_color = r.color;
        }
    }
    float closest_plane = INFINITY;
    v3 plane_color = V(0, 0, 0);
    for (int i = 0; i < s->np; ++i) {
        TraceResult r = trace_plane(s, hp, dir, &s->pl[i], count);
        if (r.distance > 0 && r.distance < closest_plane) {
            closest_plane = r.distance;
            plane_color = r.color;
        }
    }
    return closest_sphere < closest_plane ? sphere_color : plane_color;
}

/* ShiftColor, RayTracer.cs:1046-1052 */
int32_t oracle_shift_color(rt_vec3 c) {
    int32_t r = net_d2i(floor((double)(net_clamp(c.x, 0.0f, 1.0f) * 255.0f)));
    int32_t g = net_d2i(floor((double)(net_clamp(c.y, 0.0f, 1.0f) * 255.0f)));
    int32_t b = net_d2i(floor((double)(net_clamp(c.z, 0.0f, 1.0f) * 255.0f)));
    return (int32_t)(((uint32_t)(uint8_t)r << 16) | ((uint32_t)(uint8_t)g << 8) | (uint32_t)(uint8_t)b);
}

/* Primary ray of TracePixel, RayTracer.cs:963-971.  The camera basis is recomputed per
 * pixel through the property getters, as the reference does. */
static v3 primary_dir(const Scene* s, int x, int y) {
    float px = (float)x / (float)s->width - 0.5f;
    float py = (float)y / (float)s->height - 0.5f;
    v3 local = vmul(V(px, py, 1.0f), s->view_params);
    v3 vp = vadd(vadd(vadd(s->cam_pos, vscale(cam_right(s), local.x)), vscale(cam_up(s), local.y)),
                 vscale(cam_forward(s), local.z));
    return vnormalize(vsub(vp, s->cam_pos));
}

/* TracePixel, RayTracer.cs:962-1002 (reference: every primitive traced and shaded). */
static int32_t trace_pixel_reference(const Scene* s, int x, int y) {
    v3 dir = primary_dir(s, x, y);
    v3 o = s->cam_pos;
    v3 sphere_color = V(0, 0, 0);
    float nearest_sphere = INFINITY;
    for (int i = 0; i < s->ns; ++i) {
        TraceResult r = trace_sphere(s, o, dir, &s->sph[i], 0);
        if (r.distance > 0 && nearest_sphere > r.distance) {
            nearest_sphere = r.distance;
            sphere_color = r.color;
        }
    }
    v3 plane_color = V(0, 0, 0);
    float nearest_plane = INFINITY;
    for (int i = 0; i < s->np; ++i) {
        TraceResult r = trace_plane(s, o, dir, &s->pl[i], 0);
        if (r.distance > 0 && nearest_plane > r.distance) {
            nearest_plane = r.distance;
            plane_color = r.color;
        }
    }
    return oracle_shift_color(nearest_sphere < nearest_plane ? sphere_color : plane_color);
}

/* ------------------------------------------------------------------------- */
/* Nearest-hit-only restatement (same selection rules; only the winner of each     */
/* segment is shaded).  Output-equivalent to the reference because shading has no  */
/* side effects and the selection only reads intersection distances.              */
/* ------------------------------------------------------------------------- */

/* Colour of the ray (o,d) at bounce count `count`; primary selects with the TracePixel
 * rule (:977, :987), secondary with the TraceSecondaryRay rule (:804, :819). */
static v3 trace_nearest(const Scene* s, v3 o, v3 d, int count, int primary, oracle_stats* st) {
    if (st) {
        if (primary) st->primary_rays++;
        else st->reflect_rays++;
    }
    float best_s = INFINITY;
    int win_s = -1;
    for (int i = 0; i < s->ns; ++i) {
        float t = intersect_sphere(o, d, &s->sph[i], 0.0f).distance; /* 0 on a miss */
        if (primary ? (t > 0 && best_s > t) : (t - 0.01f > 0 && t - 0.01f < best_s)) {
            best_s = t;
            win_s = i;
        }
    }
    float best_p = INFINITY;
    int win_p = -1;
    for (int i = 0; i < s->np; ++i) {
        float t = intersect_plane(o, d, &s->pl[i]).distance;
        if (t > 0 && t < best_p) {
            best_p = t;
            win_p = i;
        }
    }
    int is_sphere;
    float t;
    if (best_s < best_p) {
        is_sphere = 1;
        t = best_s;
    } else if (win_p >= 0) {
        is_sphere = 0;
        t = best_p;
    } else {
        return V(0, 0, 0);
    }
    if (t - 0.01f <= 0) return V(0, 0, 0);
    if (count > s->limit) return is_sphere ? V(0, 0, 0) : V(1, 1, 1);

    v3 hp = vadd(o, vscale(d, t));
    const rt_material* m = is_sphere ? &s->sph[win_s].m : &s->pl[win_p].m;
    v3 normal = is_sphere ? vnormalize(vsub(hp, s->sph[win_s].center)) : s->pl[win_p].normal;
    v3 color = V(0, 0, 0);
    if (m_is_mirror(m))
        color = vadd(color, vmul(trace_nearest(s, hp, reflect(d, normal), count + 1, 0, st), m->km));
    if (m_is_diffuse(m)) {
        float tile = is_sphere ? 1.0f : checker(&s->pl[win_p], hp);
        for (int i = 0; i < s->nl; ++i) {
            const rt_light* l = &s->li[i];
            float li = shadow_light(s, hp, l, st);
            v3 phong = shape_phong(hp, d, normal, m, l);
            if (is_sphere) {
                float att = 1 / t * t;
                color = vadd(color, vmul(vscale(vfrom(li), att), phong));
            } else {
                float att = (float)(1 / pow((double)t, 2));
                color = vadd(color, vmax_s(vmul(vmul(vscale(vfrom(li), att), phong), vfrom(tile)), 0.0f));
            }
        }
    }
    return vadd(color, vmul(s->ambient, m->ka));
}

static int32_t trace_pixel_nearest(const Scene* s, int x, int y, oracle_stats* st) {
    if (st) st->pixels++;
    return oracle_shift_color(trace_nearest(s, s->cam_pos, primary_dir(s, x, y), 0, 1, st));
}

/* ------------------------------------------------------------------------- */
/* Float hit records of the visible path: every ray of every       */
/* stride-th pixel as (origin, end, kind), in the order the pixel's walk       */
/* produces them -- primary / reflected segment to its selected hit (origin +  */
/* 100 * dir when nothing is selected), then at a shaded diffuse hit one       */
/* shadow ray per light ending at the first sphere (scene order) that blocks   */
/* it, at hit + t * light.position, else at t = 1.  The checker for            */
/* rt_debug_segments.                                                         */
/* ------------------------------------------------------------------------- */

static void seg_put(rt_segment* out, int cap, int* n, v3 o, v3 e, int kind, int pixel) {
    if (*n < cap) {
        out[*n].origin = o;
        out[*n].end = e;
        out[*n].kind = kind;
        out[*n].pixel = pixel;
    }
    ++*n;
}

static void segments_pixel(const Scene* s, int x, int y, rt_segment* out, int cap, int* n) {
    const int pixel = y * s->width + x;
    v3 o = s->cam_pos, d = primary_dir(s, x, y);
    for (int level = 0;; ++level) {
        const int primary = level == 0;
        float best_s = INFINITY, best_p = INFINITY;
        int win_s = -1, win_p = -1;
        for (int i = 0; i < s->ns; ++i) {
            float t = intersect_sphere(o, d, &s->sph[i], 0.0f).distance;
            if (primary ? (t > 0 && best_s > t) : (t - 0.01f > 0 && t - 0.01f < best_s)) {
                best_s = t;
                win_s = i;
            }
        }
        for (int i = 0; i < s->np; ++i) {
            float t = intersect_plane(o, d, &s->pl[i]).distance;
            if (t > 0 && t < best_p) {
                best_p = t;
                win_p = i;
            }
        }
        int is_sphere, none = 0;
        float t = 0;
        if (best_s < best_p) {
            is_sphere = 1;
            t = best_s;
        } else if (win_p >= 0) {
            is_sphere = 0;
            t = best_p;
        } else {
            is_sphere = 0;
            none = 1;
        }
        seg_put(out, cap, n, o, vadd(o, vscale(d, none ? 100.0f : t)), primary ? 0 : 1, pixel);
        if (none || t - 0.01f <= 0 || level > s->limit) return;
        const v3 hp = vadd(o, vscale(d, t));
        const rt_material* m = is_sphere ? &s->sph[win_s].m : &s->pl[win_p].m;
        if (m_is_diffuse(m))
            for (int li = 0; li < s->nl; ++li) {
                const rt_light* l = &s->li[li];
                float tb = 1.0f;
                for (int i = 0; i < s->ns; ++i) {
                    Isect r = intersect_sphere(hp, l->position, &s->sph[i], 0.001f);
                    if (r.collision) {
                        tb = r.distance;
                        break;
                    }
                }
                seg_put(out, cap, n, hp, vadd(hp, vscale(l->position, tb)), 2, pixel);
            }
        if (!m_is_mirror(m)) return;
        const v3 normal = is_sphere ? vnormalize(vsub(hp, s->sph[win_s].center)) : s->pl[win_p].normal;
        d = reflect(d, normal);
        o = hp;
    }
}

/* ------------------------------------------------------------------------- */
/* Frame drivers                                                              */
/* ------------------------------------------------------------------------- */

typedef struct {
    const Scene* s;
    int row_begin, row_end;
    int32_t* pixels;
    int mode;
    int tid, nthreads;
    pthread_barrier_t* barrier;
    atomic_int* next_row;
    oracle_stats st;
} Worker;

static void* worker_main(void* arg) {
    Worker* w = (Worker*)arg;
    const Scene* s = w->s;
    if (w->mode == ORACLE_MODE_REFERENCE) {
        /* Tick(): for (x) Parallel.For(rows) -- one fork/join per column (:898-901). */
        for (int x = 0; x < s->width; ++x) {
            for (int y = w->row_begin + w->tid; y < w->row_end; y += w->nthreads)
                w->pixels[(size_t)(y - w->row_begin) * s->width + x] = trace_pixel_reference(s, x, y);
            if (w->nthreads > 1) pthread_barrier_wait(w->barrier);
        }
    } else {
        for (;;) {
            int y = atomic_fetch_add(w->next_row, 1);
            if (y >= w->row_end) break;
            for (int x = 0; x < s->width; ++x)
                w->pixels[(size_t)(y - w->row_begin) * s->width + x] = trace_pixel_nearest(s, x, y, &w->st);
        }
    }
    return NULL;
}

int oracle_render(const rt_sphere* spheres, int n_spheres, const rt_plane* planes, int n_planes,
                  const rt_light* lights, int n_lights, rt_vec3 ambient, int recursion_limit,
                  const rt_camera* camera, int width, int height, int row_begin, int row_end,
                  int32_t* pixels, int mode, int nthreads, oracle_stats* stats) {
    if (n_spheres < 0 || n_planes < 0 || n_lights < 0 || width <= 0 || height <= 0 || !pixels ||
        !camera || row_begin < 0 || row_end > height || row_begin > row_end || recursion_limit < 0 ||
        (n_spheres && !spheres) || (n_planes && !planes) || (n_lights && !lights))
        return RT_ERR_INVALID_ARG;
    if (nthreads <= 0) nthreads = 1;

    Sphere* sph = (Sphere*)calloc((size_t)(n_spheres ? n_spheres : 1), sizeof(Sphere));
    Plane* pl = (Plane*)calloc((size_t)(n_planes ? n_planes : 1), sizeof(Plane));
    for (int i = 0; i < n_spheres; ++i) {
        sph[i].center = spheres[i].center;
        sph[i].radius = spheres[i].radius;
        sph[i].radius_sq = spheres[i].radius * spheres[i].radius;
        sph[i].m = spheres[i].material;
    }
    for (int i = 0; i < n_planes; ++i) {
        pl[i].center = planes[i].center;
        pl[i].normal = planes[i].normal;
        pl[i].m = planes[i].material;
    }
    Scene s;
    s.sph = sph;
    s.ns = n_spheres;
    s.pl = pl;
    s.np = n_planes;
    s.li = lights;
    s.nl = n_lights;
    s.ambient = ambient;
    s.limit = recursion_limit;
    s.cam_pos = camera->position;
    s.yaw = camera->yaw;
    s.pitch = camera->pitch;
    s.width = width;
    s.height = height;
    s.view_params = view_params(width, height);

    pthread_barrier_t barrier;
    atomic_int next_row;
    atomic_init(&next_row, row_begin);
    if (nthreads > 1) pthread_barrier_init(&barrier, NULL, (unsigned)nthreads);
    Worker* ws = (Worker*)calloc((size_t)nthreads, sizeof(Worker));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        ws[t].s = &s;
        ws[t].row_begin = row_begin;
        ws[t].row_end = row_end;
        ws[t].pixels = pixels;
        ws[t].mode = mode;
        ws[t].tid = t;
        ws[t].nthreads = nthreads;
        ws[t].barrier = &barrier;
        ws[t].next_row = &next_row;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, worker_main, &ws[t]);
    worker_main(&ws[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    if (nthreads > 1) pthread_barrier_destroy(&barrier);

    if (stats) {
        memset(stats, 0, sizeof *stats);
        for (int t = 0; t < nthreads; ++t) {
            stats->pixels += ws[t].st.pixels;
            stats->primary_rays += ws[t].st.primary_rays;
            stats->reflect_rays += ws[t].st.reflect_rays;
            stats->shadow_rays += ws[t].st.shadow_rays;
        }
    }
    free(ws);
    free(th);
    free(sph);
    free(pl);
    return RT_OK;
}

int oracle_segments(const rt_sphere* spheres, int n_spheres, const rt_plane* planes, int n_planes,
                    const rt_light* lights, int n_lights, rt_vec3 ambient, int recursion_limit,
                    const rt_camera* camera, int width, int height, int stride, rt_segment* out, int capacity,
                    int* out_count) {
    if (n_spheres < 0 || n_planes < 0 || n_lights < 0 || width <= 0 || height <= 0 || !camera || stride <= 0 ||
        capacity < 0 || (capacity && !out) || !out_count || recursion_limit < 0 || (n_spheres && !spheres) ||
        (n_planes && !planes) || (n_lights && !lights))
        return RT_ERR_INVALID_ARG;
    Sphere* sph = (Sphere*)calloc((size_t)(n_spheres ? n_spheres : 1), sizeof(Sphere));
    Plane* pl = (Plane*)calloc((size_t)(n_planes ? n_planes : 1), sizeof(Plane));
    for (int i = 0; i < n_spheres; ++i) {
        sph[i].center = spheres[i].center;
        sph[i].radius = spheres[i].radius;
        sph[i].radius_sq = spheres[i].radius * spheres[i].radius;
        sph[i].m = spheres[i].material;
    }
    for (int i = 0; i < n_planes; ++i) {
        pl[i].center = planes[i].center;
        pl[i].normal = planes[i].normal;
        pl[i].m = planes[i].material;
    }
    Scene s;
    memset(&s, 0, sizeof s);
    s.sph = sph, s.ns = n_spheres, s.pl = pl, s.np = n_planes, s.li = lights, s.nl = n_lights;
    s.ambient = ambient, s.limit = recursion_limit;
    s.cam_pos = camera->position, s.yaw = camera->yaw, s.pitch = camera->pitch;
    s.width = width, s.height = height, s.view_params = view_params(width, height);
    int n = 0;
    for (long long idx = 0; idx < (long long)width * height; idx += stride)
        segments_pixel(&s, (int)(idx % width), (int)(idx / width), out, capacity, &n);
    *out_count = n;
    free(sph);
    free(pl);
    return RT_OK;
}
