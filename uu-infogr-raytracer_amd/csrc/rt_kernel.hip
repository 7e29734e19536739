// rt_kernel.hip -- gfx950 kernels for the per-pixel Whitted trace of
// Raytracer/RayTracer.cs (TracePixel :962-1002 -> TraceSphere/TracePlane :729-876 ->
// IntersectsSphere/IntersectPlane :590-642 -> IntersectShadowLight :573-582 ->
// *PhongShading :652-708 -> TraceSecondaryRay :789-826 -> ShiftColor :1046-1052).
//
// Design (MI355X-first, not a translation of the C# recursion):
//  * one wave64 lane per pixel; a wave covers an 8x8 pixel tile (ray coherence -> fewer
//    divergent primitive hits per wave) and is its own workgroup (A/B: 2x2-wave groups
//    +8 % on C4, where a group's LDS stack slots were held until its slowest wave ended);
//  * the scene is tiny (< 6 KB at 64 spheres) and every loop over spheres / planes / lights
//    is wave-uniform, so primitive data is read with scalar loads (SGPR operands); the
//    camera-relative sphere constants of the primary segment come in the kernarg block;
//  * the reference shades EVERY hit primitive and recurses from each mirror hit; only the
//    nearest (by the reference's own selection rules) reaches the pixel, so each lane walks
//    a single chain of segments forward (intersection only), pushing one record per
//    shaded hit onto a per-lane stack, then folds colours backward in the reference's
//    exact order: mirror term, then each light in order, then ambient
//    (RayTracer.cs:739-778, :850-873).  Bit-identical to the all-hit recursion.
//  * arithmetic is IEEE binary32 with no FMA contraction (-ffp-contract=off), correctly
//    rounded '/' and sqrt, IEEE-754-2019 maximum/minimum for .NET Math.Max/Min, f64 where
//    the reference uses Math.Pow, and .NET's (int) conversion (NaN/overflow -> INT_MIN).
//  * work the reference does but whose result provably cannot change a selection is
//    skipped (sqrt/divisions of spheres behind the ray, the far root) -- see root_t1.
#include <hip/hip_runtime.h>

#include "rt_fastmath.h"
#include "rt_internal.h"

// RT_FASTMATH 1 (shipped): correctly rounded sqrt / reciprocal / division through the short
// sequences of rt_fastmath.h inside their verified domains (same bits as the generic
// operations for every input, tools/fastmath_check.hip); 0 = the generic sequences.
#ifndef RT_FASTMATH
#define RT_FASTMATH 1
#endif

// RT_ABLATE (timing experiments only, tools/ab.py; never defined in the shipped build):
//   1 = no shading (fold skipped), 2 = no shadow rays, 3 = primary segment only.
#ifndef RT_ABLATE
#define RT_ABLATE 0
#endif
// RT_CULLSTATS (experiments only): the bundle kernel's reflect/shadow counters count the
// wave-iterations of its shadow exact-test loops (1) or its shadow bundles (2) instead of rays.
// Workgroup shape of the trace kernels: WG_WX x WG_WY waves, each an 8x8 pixel tile.
// A/B (C2/C3/C4): 1x1 1.00/1.00/0.92, 2x1 0.99/1.00/0.95, 2x2 = 1, 4x2 1.04/1.03/1.13,
// 4x4 1.10/1.14/1.29 (kernel time relative to 2x2).
#ifndef RT_WG_WX
#define RT_WG_WX 1
#endif
#ifndef RT_WG_WY
#define RT_WG_WY 1
#endif
constexpr int WG_WX = RT_WG_WX, WG_WY = RT_WG_WY, WG_WAVES = WG_WX * WG_WY, WG_THREADS = 64 * WG_WAVES;
[[maybe_unused]] constexpr int TILE_W = 8 * WG_WX, TILE_H = 8 * WG_WY;

#ifndef RT_CULLSTATS
#define RT_CULLSTATS 0
#endif

namespace rtk {

// Correctly rounded binary32 operations (bit-identical either way, see rt_fastmath.h).
// RT_FASTMATH bits: 1 = normalize's 1/sqrt, 2 = other sqrt, 4 = reciprocal / division.
__device__ __forceinline__ float cr_sqrt(float x) {
    if constexpr ((RT_FASTMATH & 2) != 0) return sqrt_cr(x);
    else return __builtin_sqrtf(x);
}
__device__ __forceinline__ float cr_inv_len(float x) {  // 1f / MathF.Sqrt(x)
    if constexpr ((RT_FASTMATH & 1) != 0) return inv_len_cr(x);
    else return 1.0f / __builtin_sqrtf(x);
}
__device__ __forceinline__ float cr_rcp(float x) {
    if constexpr ((RT_FASTMATH & 4) != 0) return rcp_cr(x);
    else return 1.0f / x;
}
// a / b where the quotient is used only when `need` (the generic fallback runs only there).
__device__ __forceinline__ float cr_div_if(bool need, float a, float b) {
    if constexpr ((RT_FASTMATH & 4) != 0) {
        float q = div_cr_fast(a, b);
        if (__builtin_expect(need && !(fm_in(a, FM_DIV_LO, FM_DIV_HI) && fm_in(b, FM_DIV_LO, FM_DIV_HI)), 0))
            q = a / b;
        return q;
    } else {
        (void)need;
        return a / b;
    }
}

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 scale(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
// Vector3.Dot: (x*x') + (y*y') + (z*z')
__device__ __forceinline__ float dot(f3 a, f3 b) { return ((a.x * b.x) + (a.y * b.y)) + (a.z * b.z); }
// Vector3.Normalize: s = 1f / MathF.Sqrt(x*x + y*y + z*z); v * s
__device__ __forceinline__ f3 normalize(f3 a) {
    const float s = cr_inv_len(dot(a, a));
    return scale(a, s);
}
// Math.Max(x, 0f) / Math.Min(a, b) on .NET Core 3.0+: IEEE 754-2019 maximum / minimum
// (NaN propagates, -0 < +0) -> v_maximum3_f32 / v_minimum3_f32 on gfx950.
__device__ __forceinline__ float nmax0(float a) { return __builtin_elementwise_maximum(a, 0.0f); }
__device__ __forceinline__ float nmin(float a, float b) { return __builtin_elementwise_minimum(a, b); }

// (int)float on .NET 6 x64 (cvttss2si): NaN or out of range -> int.MinValue.
__device__ __forceinline__ int32_t net_f2i(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : (int32_t)0x80000000;
}

// (float)Math.Pow((double)x, (double)n) for the shading exponent.  Exact fast paths:
// n == 1 -> x; n == 2 -> x*x (the double product of two floats is exact, so one float
// rounding of it equals binary32 x*x); n == 0.5 -> binary32 sqrt (a double result within
// glibc pow's 0.54 ulp can never straddle a binary32 rounding boundary of sqrt(float):
// the exact root is >= 2^-49 relative away from every binary32 midpoint).  Other
// exponents use the device's f64 pow (compiled in only when the scene needs it).
template <bool GPOW>
__device__ __forceinline__ float spec_pow(float x, const DevMaterial& m) {
    switch (m.pow_kind) {
        case POW_ONE: return x;
        case POW_HALF: return cr_sqrt(x);
        case POW_TWO: return x * x;
        default:
            if constexpr (GPOW) return (float)pow((double)x, (double)m.n);
            else return x;  // unreachable: the host selects GPOW when any material needs it
    }
}

// ---------------------------------------------------------------------------------
// IntersectsSphere (RayTracer.cs:613-642) for nearest-hit selection, epsilon 0.
//
// The reference returns dist = min(max(t1,0), max(t2,0)) on a collision (dist > 0) and 0
// otherwise, with t2 = (-b+sqrt)/2a, t1 = (-b-sqrt)/2a; the callers then select only
// dist > 0 (TracePixel :977) or dist - 0.01 > 0 (TraceSecondaryRay :804).  When 2a is
// finite and > 0 (always, for the normalised primary and reflected directions) the
// exactly-rounded results satisfy t2 >= t1 (numerators ordered, rounding and division by
// a positive number monotonic), so a selectable distance exists iff t1 > 0, and then it is
// t1 itself.  t1 > 0 iff fl(-b - sq) > 0 iff -b > sq (gradual underflow), which needs
// -b > 0 first.  So: no sqrt when b >= 0, no division unless -b > sq, never the t2
// division.  Returns the reference's distance or 0 (non-selectable) -- identical
// selections and identical winning distances.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ float root_t1(float b, float disc, float a2) {
    float t = 0.0f;
    if (disc >= 0.0f && b < 0.0f) {
        const float sq = cr_sqrt(disc);  // == (float)Math.Sqrt((double)disc)
        const float nb = -b;
        const bool sel = nb > sq;
        const float q = cr_div_if(sel, nb - sq, a2);  // predicated, not branched
        t = sel ? q : 0.0f;
    }
    return t;
}

// Literal formula, for directions whose 2a is not finite-positive.
__device__ __forceinline__ float root_full(float b, float disc, float a2) {
    float t = 0.0f;
    if (disc >= 0.0f) {
        const float sq = __builtin_sqrtf(disc);
        const float t2 = (-b + sq) / a2;
        const float t1 = (-b - sq) / a2;
        t = nmin(nmax0(t1), nmax0(t2));
    }
    return t;
}

__device__ __forceinline__ float sphere_t(f3 o, f3 d, float a2, float a4, bool a2_ok, const DevSphere& s) {
    const f3 oc = sub(o, mk(s.cx, s.cy, s.cz));
    const float b = 2.0f * dot(oc, d);
    const float c = dot(oc, oc) - s.r2;
    const float disc = b * b - a4 * c;
    return a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2);
}

// Shadow ray of IntersectShadowLight (origin = hit point, direction = light POSITION,
// epsilon 0.001, RayTracer.cs:574-578): collision iff min(max(t1-e,0), max(t2-e,0)) > 0.
// With 2a finite-positive (uniform per light) and t2 >= t1 that is t1 - e > 0 (and then
// t2 - e > 0 too), which again needs -b > sq.
__device__ __forceinline__ bool shadow_blocked(f3 hp, const DevLight& l, bool a2_ok, const DevSphere& s) {
    const f3 oc = sub(hp, mk(s.cx, s.cy, s.cz));
    const float b = 2.0f * dot(oc, mk(l.px, l.py, l.pz));
    const float c = dot(oc, oc) - s.r2;
    const float disc = b * b - l.a4 * c;
    if (a2_ok) {
        bool hit = false;
        if (disc >= 0.0f && b < 0.0f) {
            const float sq = cr_sqrt(disc);
            const float nb = -b;
            const bool sel = nb > sq;
            hit = sel & (cr_div_if(sel, nb - sq, l.a2) - 0.001f > 0.0f);
        }
        return hit;
    }
    if (disc >= 0.0f) {
        const float sq = __builtin_sqrtf(disc);
        const float t2 = (-b + sq) / l.a2;
        const float t1 = (-b - sq) / l.a2;
        return nmin(nmax0(t1 - 0.001f), nmax0(t2 - 0.001f)) > 0.0f;
    }
    return false;
}

// IntersectPlane, RayTracer.cs:590-604: t = (((-o.x*n.x) - o.y*n.y) - o.z*n.z + c.n) / d.n,
// hit iff t > 0.  The quotient can only be > 0 when numerator and denominator are nonzero
// with equal signs; otherwise it is <= 0 or NaN (a miss) and the division is skipped.
__device__ __forceinline__ float plane_t(f3 o, f3 d, const DevPlane& p) {
    const float num = ((-o.x * p.nx - o.y * p.ny) - o.z * p.nz) + p.cn;
    const float den = dot(d, mk(p.nx, p.ny, p.nz));
    const bool sel = (num > 0.0f && den > 0.0f) || (num < 0.0f && den < 0.0f);
    const float q = cr_div_if(sel, num, den);
    return sel ? q : 0.0f;
}

// ShiftColor, :1046-1052: Math.Clamp (NaN passes), * 255f, Math.Floor, (int), (byte).
// Branch-free: IEEE maxNum/minNum return the non-NaN operand, so NaN -> 0 -> byte 0, the
// byte .NET gives ((int)NaN = int.MinValue, (byte) of it = 0); +-inf clamp to 1 / 0 and -0
// gives 0 as in the reference.
__device__ __forceinline__ uint32_t shift_channel(float c) {
    const float cl = __builtin_fminf(__builtin_fmaxf(c, 0.0f), 1.0f);
    return (uint32_t)(int32_t)__builtin_floorf(cl * 255.0f);
}

// Frame / band output: int32 0x00RRGGBB at the packed band row r (format 0) or at the frame
// row y (format 2), or packed 24-bit (B, G, R bytes; the top byte of the int32 is always 0)
// for band sets shipped to rank 0 -- a quarter fewer bytes over xGMI (format 1).
// Format 2 (RT_BANDS_FRAME): the rank's bands straight into the row-major frame (row y).
__device__ __forceinline__ void store_pixel(const LaunchParams& p, int r, int y, int x, uint32_t px32) {
    const size_t i = (size_t)(p.out_fmt == 2 ? y : r) * (size_t)p.W + (size_t)x;
    unsigned char* base = (unsigned char*)p.out + (size_t)blockIdx.z * p.out_frame_bytes;  // batch frame z
    if (p.out_fmt != 1) {
        ((int32_t*)base)[i] = (int32_t)px32;
    } else {
        unsigned char* o = base + i * 3;
        o[0] = (unsigned char)px32;
        o[1] = (unsigned char)(px32 >> 8);
        o[2] = (unsigned char)(px32 >> 16);
    }
}

// Per-lane level stack.  Records: a = {hit point, t}, b = {incoming direction, primitive code}.
template <int K, bool SCRATCH>
struct LevelStack;

// Register stack: K fixed, static indices only (shift on push/pop) so it stays in VGPRs.
template <int K>
struct LevelStack<K, false> {
    float4 a[K], b[K];
    int n = 0;
    __device__ __forceinline__ void push(float4 x, float4 y) {
#pragma unroll
        for (int i = K - 1; i > 0; --i) {
            a[i] = a[i - 1];
            b[i] = b[i - 1];
        }
        a[0] = x;
        b[0] = y;
        ++n;
    }
    __device__ __forceinline__ void pop(float4& x, float4& y) {
        x = a[0];
        y = b[0];
#pragma unroll
        for (int i = 0; i < K - 1; ++i) {
            a[i] = a[i + 1];
            b[i] = b[i + 1];
        }
        --n;
    }
};

// Deep-recursion stack (recursion limits >= 8): dynamically indexed, lives in scratch.
template <int K>
struct LevelStack<K, true> {
    float4 a[K], b[K];
    int n = 0;
    __device__ __forceinline__ void push(float4 x, float4 y) {
        a[n] = x;
        b[n] = y;
        ++n;
    }
    __device__ __forceinline__ void pop(float4& x, float4& y) {
        --n;
        x = a[n];
        y = b[n];
    }
};

// Hybrid stack for limits 3..7: the two most recent records in VGPRs, older ones in a
// per-lane scratch array (touched only by lanes more than two levels deep -- rare), so the
// kernel keeps its occupancy: 16 VGPRs instead of 8 x K.
template <int K>
struct HybridOverflow {
    float4 a[K - 2], b[K - 2];  // older records (dynamically indexed: scratch)
};
template <int K>
struct HybridStack {
    float4 a0, b0, a1, b1;  // top record, second record (separate SSA values: VGPRs)
    HybridOverflow<K>* ov;  // a separate object, so only it is demoted to scratch
    int n = 0;
    __device__ __forceinline__ HybridStack(HybridOverflow<K>* o, float2*, float*) : ov(o) {}
    __device__ __forceinline__ void push(float4 x, float4 y) {
        if (n >= 2) {  // spill the second record
            ov->a[n - 2] = a1;
            ov->b[n - 2] = b1;
        }
        a1 = a0;
        b1 = b0;
        a0 = x;
        b0 = y;
        ++n;
    }
    __device__ __forceinline__ void origin(f3) {}
    __device__ __forceinline__ void pop(const LaunchParams&, float4& x, float4& y) {
        x = a0;
        y = b0;
        a0 = a1;
        b0 = b1;
        --n;
        if (n >= 2) {  // refill the second record
            a1 = ov->a[n - 2];
            b1 = ov->b[n - 2];
        }
    }
};

struct NoOverflow {};
template <int K, bool SCRATCH>
struct PlainStack : LevelStack<K, SCRATCH> {
    __device__ __forceinline__ PlainStack(NoOverflow*, float2*, float*) {}
    __device__ __forceinline__ void origin(f3) {}
    __device__ __forceinline__ void pop(const LaunchParams&, float4& x, float4& y) { LevelStack<K, SCRATCH>::pop(x, y); }
};

// One reflection step of the forward walk (TraceSphere :854 / TracePlane normal,
// CalculateReflectionRay :718-720): hit point of segment (o, d) at t, then the reflected
// segment.  The walks and the compact stacks' re-walk share it, so the re-walk reproduces
// every hit point and direction bit for bit.
__device__ __forceinline__ f3 reflect_at(const LaunchParams& p, f3 o, f3& d, float t, int code) {
    const f3 hp = add(o, scale(d, t));
    f3 normal;
    if (code >= 0) {
        const DevSphere& s = p.sph[code];
        normal = normalize(sub(hp, mk(s.cx, s.cy, s.cz)));
    } else {
        const DevPlane& pl = p.pl[~code];
        normal = mk(pl.nx, pl.ny, pl.nz);
    }
    d = sub(d, scale(normal, 2.0f * dot(d, normal)));
    return hp;
}

// Compact stacks: a record is fully determined by the camera ray and the (t, primitive)
// pairs of the levels above it, so older levels keep only those 8 bytes (registers,
// statically indexed) and are rebuilt by re-walking the reflection chain -- no scratch
// traffic at all.
// RT_STACK 1: every level compact, each pop re-walks (level k costs k steps).  The levels
// live in register vectors; the re-walk loop is rolled with a wave-uniform index (indirect
// register reads, no scratch), the per-lane top is picked by a select chain.
template <int K>
struct CompactStack {
    typedef float tvec __attribute__((ext_vector_type(K)));
    typedef int cvec __attribute__((ext_vector_type(K)));
    tvec t;
    cvec c;
    f3 d0;
    int n = 0;
    __device__ __forceinline__ CompactStack(NoOverflow*, float2*, float*) {}
    __device__ __forceinline__ void origin(f3 d) { d0 = d; }
    __device__ __forceinline__ void push(float4 x, float4 y) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            if (i == n) {
                t[i] = x.w;
                c[i] = __float_as_int(y.w);
            }
        ++n;
    }
    __device__ __forceinline__ void pop(const LaunchParams& p, float4& x, float4& y) {
        --n;
        f3 o = mk(p.cam[0], p.cam[1], p.cam[2]), d = d0;
#pragma unroll 1
        for (int j = 0; j < K - 1; ++j) {
            const bool go = j < n;
            if (__builtin_amdgcn_ballot_w64(go) == 0) break;
            if (go) o = reflect_at(p, o, d, t[j], c[j]);
        }
        float tk = t[0];
        int ck = c[0];
#pragma unroll
        for (int i = 1; i < K; ++i)
            if (i == n) {
                tk = t[i];
                ck = c[i];
            }
        const f3 hp = add(o, scale(d, tk));
        x = make_float4(hp.x, hp.y, hp.z, tk);
        y = make_float4(d.x, d.y, d.z, __int_as_float(ck));
    }
};

// RT_STACK 2: the two most recent records whole in VGPRs, older levels compact; only the
// refill of the second record re-walks (levels n-3.. of an n-deep chain).
template <int K>
struct CompactHybridStack {
    float4 a0, b0, a1, b1;
    float t[K - 2];
    int c[K - 2];
    f3 d0;
    int n = 0;
    __device__ __forceinline__ CompactHybridStack(NoOverflow*, float2*, float*) {}
    __device__ __forceinline__ void origin(f3 d) { d0 = d; }
    __device__ __forceinline__ void push(float4 x, float4 y) {
        if (n >= 2) {
#pragma unroll
            for (int i = 0; i < K - 2; ++i)
                if (i == n - 2) {
                    t[i] = a1.w;
                    c[i] = __float_as_int(b1.w);
                }
        }
        a1 = a0;
        b1 = b0;
        a0 = x;
        b0 = y;
        ++n;
    }
    __device__ __forceinline__ void pop(const LaunchParams& p, float4& x, float4& y) {
        x = a0;
        y = b0;
        a0 = a1;
        b0 = b1;
        --n;
        if (n >= 2) {  // rebuild level n-2 from the compact levels 0..n-2
            f3 o = mk(p.cam[0], p.cam[1], p.cam[2]), d = d0;
            float tk = t[0];
            int ck = c[0];
#pragma unroll
            for (int j = 0; j < K - 3; ++j)
                if (j < n - 2) {
                    o = reflect_at(p, o, d, t[j], c[j]);
                    tk = t[j + 1];
                    ck = c[j + 1];
                }
            const f3 hp = add(o, scale(d, tk));
            a1 = make_float4(hp.x, hp.y, hp.z, tk);
            b1 = make_float4(d.x, d.y, d.z, __int_as_float(ck));
        }
    }
};

// RT_STACK 3: the compact levels and the primary direction in LDS, one slot per thread
// ([level][thread], conflict-free), so they cost no VGPRs; pop re-walks as in CompactStack.
template <int K>
struct LdsStack {
    float2* lv;  // [K][WG_THREADS] (t, primitive code) of this workgroup
    float* dv;   // [3][WG_THREADS] primary direction
    int n = 0;
    __device__ __forceinline__ LdsStack(NoOverflow*, float2* l, float* dd) : lv(l), dv(dd) {}
    __device__ __forceinline__ void origin(f3 d) {
        dv[threadIdx.x] = d.x;
        dv[WG_THREADS + threadIdx.x] = d.y;
        dv[2 * WG_THREADS + threadIdx.x] = d.z;
    }
    __device__ __forceinline__ void push(float4 x, float4 y) {
        lv[n * WG_THREADS + threadIdx.x] = make_float2(x.w, y.w);
        ++n;
    }
    __device__ __forceinline__ void pop(const LaunchParams& p, float4& x, float4& y) {
        --n;
        f3 o = mk(p.cam[0], p.cam[1], p.cam[2]);
        f3 d = mk(dv[threadIdx.x], dv[WG_THREADS + threadIdx.x], dv[2 * WG_THREADS + threadIdx.x]);
#pragma unroll 1
        for (int j = 0; j < K - 1; ++j) {
            const bool go = j < n;
            if (__builtin_amdgcn_ballot_w64(go) == 0) break;
            if (go) {
                const float2 tc = lv[j * WG_THREADS + threadIdx.x];
                o = reflect_at(p, o, d, tc.x, __float_as_int(tc.y));
            }
        }
        const float2 tk = lv[n * WG_THREADS + threadIdx.x];
        const f3 hp = add(o, scale(d, tk.x));
        x = make_float4(hp.x, hp.y, hp.z, tk.x);
        y = make_float4(d.x, d.y, d.z, tk.y);
    }
};

#ifndef RT_STACK
#define RT_STACK 3
#endif
template <int K>
struct MidStack {  // stack for K = 4, 6, 8
#if RT_STACK == 3
    using type = LdsStack<K>;
    using overflow = NoOverflow;
    static constexpr int lds_levels = K;
#elif RT_STACK == 1
    using type = CompactStack<K>;
    using overflow = NoOverflow;
    static constexpr int lds_levels = 0;
#elif RT_STACK == 2
    using type = CompactHybridStack<K>;
    using overflow = NoOverflow;
    static constexpr int lds_levels = 0;
#else
    using type = HybridStack<K>;
    using overflow = HybridOverflow<K>;
    static constexpr int lds_levels = 0;
#endif
};

// Stack type per K: registers up to 2 records, MidStack up to 8, scratch beyond.
template <int K, bool SCRATCH>
struct StackFor {
    using type = PlainStack<K, SCRATCH>;
    using overflow = NoOverflow;
    static constexpr int lds_levels = 0;
};
#ifndef RT_LDS_SMALL
#define RT_LDS_SMALL 1
#endif
#if RT_STACK == 3 && RT_LDS_SMALL
template <>
struct StackFor<1, false> : MidStack<1> {};
template <>
struct StackFor<2, false> : MidStack<2> {};
#endif
template <>
struct StackFor<4, false> : MidStack<4> {};
template <>
struct StackFor<6, false> : MidStack<6> {};
template <>
struct StackFor<8, false> : MidStack<8> {};

// Sum of v over the wave (all lanes active): bit-sliced ballots and scalar popcounts, no
// LDS round trips; the loop runs once per significant bit of the largest v (uniform).
__device__ __forceinline__ unsigned wave_count(unsigned v) {
    unsigned s = 0;
    for (int j = 0; __builtin_amdgcn_ballot_w64(v != 0u) != 0; ++j, v >>= 1)
        s += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64((v & 1u) != 0u)) << j;
    return s;
}

#ifndef RT_COUNTERS
#define RT_COUNTERS 2
#endif
// Per-lane work counts share one register: reflected segments (<= RT_MAX_RECURSION_LIMIT + 1)
// in the low byte, shadow rays (<= lights x 64; rt_set_scene caps lights at 65536) above.
constexpr unsigned CNT_SHADOW_SHIFT = 8;
constexpr unsigned CNT_REFL_MASK = 0xFFu;
// Work counters of one wave (converged call, every lane of the workgroup reaches it):
// RT_COUNTERS 1 = shuffle sums -> LDS -> one workgroup total per spread slot;
// 2 = ballot/popcount sums, lane 0 adds the wave's reflect/shadow totals to slot
// (wave id % 256); primary rays are the traced pixels, counted on the host.
__device__ __forceinline__ unsigned wave_sum(unsigned v);
__device__ __forceinline__ void add_counters(const LaunchParams& p, int lane, int wave, unsigned n_prim,
                                             unsigned n_refl, unsigned n_shadow) {
#if RT_COUNTERS == 1
    __shared__ unsigned red[WG_WAVES][3];
    n_prim = wave_sum(n_prim);
    n_refl = wave_sum(n_refl);
    n_shadow = wave_sum(n_shadow);
    if (lane == 0) {
        red[wave][0] = n_prim;
        red[wave][1] = n_refl;
        red[wave][2] = n_shadow;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned v = 0;
        for (int w = 0; w < WG_WAVES; ++w) v += red[w][threadIdx.x];
        const unsigned slot = (blockIdx.y * gridDim.x + blockIdx.x) % COUNTER_SLOTS;
        if (v) atomicAdd(&p.counters[slot * 4 + threadIdx.x], (unsigned long long)v);
    }
#elif RT_COUNTERS == 2
    // primary rays = traced pixels, counted on the host (every atomic is a memory round trip
    // on MI355X: 32 B of HBM write traffic each)
    (void)n_prim;
    const unsigned b = wave_count(n_refl), c = wave_count(n_shadow);
    if (lane == 0) {
        const unsigned slot = ((blockIdx.y * gridDim.x + blockIdx.x) * (unsigned)WG_WAVES + (unsigned)wave) % COUNTER_SLOTS;
        unsigned long long* q = &p.counters[slot * 4];
        if (b) atomicAdd(q + 1, (unsigned long long)b);
        if (c) atomicAdd(q + 2, (unsigned long long)c);
    }
#else
    (void)p, (void)lane, (void)wave, (void)n_prim, (void)n_refl, (void)n_shadow;
#endif
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Sphere loop of the direct path: a runtime loop (SMAX = 0, shipped) or fully unrolled over
// SMAX with uniform `i < S` guards.  In-process A/B of SMAX = 8: C2 +2.7 %, C3 -3.3 % -- not
// taken.
template <int SMAX, typename F>
__device__ __forceinline__ void for_spheres(int S, F&& f) {
    if constexpr (SMAX > 0) {
#pragma unroll
        for (int i = 0; i < SMAX; ++i)
            if (i < S) f(i);
    } else {
#pragma unroll 2
        for (int i = 0; i < S; ++i) f(i);
    }
}

// Result of a nearest-hit search.
struct Hit {
    float t;
    int prim;  // >= 0 sphere, ~plane for planes, or HIT_NONE
};
constexpr int HIT_NONE = 0x7fffffff;

// DIRECT path (scenes with < CULL_MIN_SPHERES spheres): per-lane divergent loops.
// Shading of one shaded hit (TraceSphere :847-873 / TracePlane :736-778): the colour is
// accumulated in the reference's order -- mirror term (from the deeper segment `sec`),
// then each light, then ambient.  Returns the colour; adds shadow rays to *n_shadow.
// A light's shadow test can change the pixel only through I * att * phong vs 0 * phong.  When
// every phong component is +-0 or NaN and I * att is finite, both give +-0 / NaN per
// component (the sign of a zero never reaches a pixel: only additions, products, IEEE max and
// the final clamp follow), so the test is skipped (RT_SHADOW_SKIP).  Ray counters are unchanged
// (shadow rays = shaded diffuse hits x lights).
#ifndef RT_SHADOW_SKIP
#define RT_SHADOW_SKIP 1
#endif
__device__ __forceinline__ bool zero_or_nan(float v) { return !(v != 0.0f && v == v); }
__device__ __forceinline__ bool shadow_matters(f3 ph, float intensity, float att) {
    if constexpr (!RT_SHADOW_SKIP) return true;
    const float ia = intensity * att;
    const bool finite = __builtin_fabsf(ia) < __builtin_inff();
    return !(finite && zero_or_nan(ph.x) && zero_or_nan(ph.y) && zero_or_nan(ph.z));
}

// Per-lane shadow cull of the direct kernel (RT_LANE_SHADOW_CULL).  Every shadow ray of light
// l has direction p_l (Q2), so sphere i can block the ray from hp only if the line
// {hp + s p_l} passes within r of its centre C: in the light's host-built frame (U, V ~ unit,
// orthogonal to A ~ p_l/|p_l|) that distance is D = |((C - hp).U, (C - hp).V)|.  The host
// stores cu = C.U, cv = C.V and t0 >= r' + 2^-8 |C|_1 (r' >= r (1 + 2^-8)); the lane skips
// the exact test when (cu - hp.U)^2 + (cv - hp.V)^2 > (t0 + 2^-8 |hp|_1)^2.
// Exactness: with u = hp - C and N = |C|_1 + |hp|_1 >= |u|, the binary32 discriminant of
// IntersectsSphere is negative whenever D >= r (1 + 3 eps) + 9.2e-4 |u| (the error analysis
// of cull_mask, invariant in the scale of the direction; a in [2^-40, 2^40], |u| < 2^41, so
// nothing overflows and, since a culled sphere has D > t0 >= 2^-25, nothing underflows),
// and disc < 0 makes shadow_blocked false in both of its branches.  The rounding of the
// cull arithmetic (cu, cv rounded from binary64, hp.U and hp.V in binary32, the frame's own
// rounding) perturbs D by less than 2^-20 N, so a cull implies D > r (1 + 2^-8) + 2^-9 N,
// twice the 9.2e-4 |u| needed.  NaN / inf anywhere, |hp|_1 >= 2^40, or a sphere the host
// excluded (t0 = +inf) fail the comparison: the exact test runs.
#ifndef RT_LANE_SHADOW_CULL
#define RT_LANE_SHADOW_CULL 0
#endif
struct LaneShadowCull {
    float hu, hv, m;
};
__device__ __forceinline__ LaneShadowCull lane_shadow_frame(f3 hp, const DevLight& l) {
    LaneShadowCull c;
    c.hu = dot(hp, mk(l.ux, l.uy, l.uz));
    c.hv = dot(hp, mk(l.vx, l.vy, l.vz));
    const float hn = __builtin_fabsf(hp.x) + __builtin_fabsf(hp.y) + __builtin_fabsf(hp.z);
    c.m = hn < 0x1p40f ? hn * 0x1.004p-8f : __builtin_inff();  // >= 2^-8 |hp|_1
    return c;
}
__device__ __forceinline__ bool lane_shadow_far(const LaneShadowCull& c, const DevShadowCull& s) {
    const float du = s.cu - c.hu, dv = s.cv - c.hv;
    const float t = s.t0 + c.m;
    return __builtin_fmaf(du, du, dv * dv) > t * t;
}

template <bool GPOW, int SMAX>
__device__ __forceinline__ f3 shade_direct(const LaunchParams& p, bool is_sphere, int prim, f3 hp, f3 d, float t, f3 sec,
                                    unsigned* n_shadow) {
    const DevMaterial& m = p.mat[is_sphere ? prim : p.S + prim];
    const uint32_t flags = m.flags;
    f3 normal;
    float tile = 1.0f;
    if (is_sphere) {
        const DevSphere& s = p.sph[prim];
        normal = normalize(sub(hp, mk(s.cx, s.cy, s.cz)));  // SpherePhongShading :706
    } else {
        const DevPlane& pl = p.pl[prim];
        normal = mk(pl.nx, pl.ny, pl.nz);
        // checkerboard, :766-770: ((int)u + (int)v) & 1, unchecked int add
        const float u = dot(mk(pl.e1x, pl.e1y, pl.e1z), hp);
        const float v = dot(mk(pl.e2x, pl.e2y, pl.e2z), hp);
        tile = (float)(int32_t)(((uint32_t)net_f2i(u) + (uint32_t)net_f2i(v)) & 1u);
    }
    f3 col = mk(0.0f, 0.0f, 0.0f);
    if (flags & MAT_MIRROR) col = add(col, mul(sec, mk(m.km[0], m.km[1], m.km[2])));
    if (flags & MAT_DIFFUSE) {
        const f3 view = normalize(d);  // ShapePhongShading :668 (not negated)
        // sphere: (1 / t) * t (:866);  plane: (float)(1 / Math.Pow(t, 2)) (:754), exact as 1/(t*t) in f64
        const float att = is_sphere ? cr_rcp(t) * t : (float)(1.0 / ((double)t * (double)t));
        const f3 kd = mk(m.kd[0], m.kd[1], m.kd[2]);
        for (int li = 0; li < p.L; ++li) {
            const DevLight& l = p.li[li];
            const bool l_ok = l.a2 > 0.0f && l.a2 < __builtin_inff();  // wave-uniform
            // ShapePhongShading, :665-695 (first: it decides whether the shadow test matters)
            const f3 ldir = normalize(sub(mk(l.px, l.py, l.pz), hp));
            f3 ph = scale(kd, nmax0(dot(normal, ldir)));
            f3 spec = mk(0.0f, 0.0f, 0.0f);
            if (flags & MAT_SPEC) {
                const f3 rs = sub(ldir, scale(normal, 2.0f * dot(ldir, normal)));
                const float sp = spec_pow<GPOW>(nmax0(dot(view, normalize(rs))), m);
                spec = mul(mk(m.ks[0], m.ks[1], m.ks[2]), mk(sp, sp, sp));
            }
            ph = add(ph, spec);
            bool blocked = false;
            if (shadow_matters(ph, l.intensity, att)) {
                if constexpr (RT_ABLATE == 2) {
                    blocked = hp.x > 1e30f;
                } else if constexpr (SMAX > 0) {
                    for_spheres<SMAX>(p.S, [&](int i) {
                        if (!blocked) blocked = shadow_blocked(hp, l, l_ok, p.sph[i]);
                    });
                } else if (RT_LANE_SHADOW_CULL && l.lane_cull) {  // wave-uniform
                    const LaneShadowCull c = lane_shadow_frame(hp, l);
                    const DevShadowCull* sc = p.shc + li * p.S;
                    for (int i = 0; i < p.S && !blocked; ++i)
                        if (!lane_shadow_far(c, sc[i])) blocked = shadow_blocked(hp, l, l_ok, p.sph[i]);
                } else {
                    for (int i = 0; i < p.S && !blocked; ++i) blocked = shadow_blocked(hp, l, l_ok, p.sph[i]);
                }
            }
            const float inten = blocked ? 0.0f : l.intensity;
            const float ia = inten * att;
            f3 term = mul(mk(ia, ia, ia), ph);
            if (!is_sphere) {
                term = mul(term, mk(tile, tile, tile));
                term = mk(nmax0(term.x), nmax0(term.y), nmax0(term.z));  // .Max(0f), :775
            }
            col = add(col, term);
        }
        *n_shadow += (unsigned)p.L << CNT_SHADOW_SHIFT;
    }
    return add(col, mk(m.amb[0], m.amb[1], m.amb[2]));
}

// Candidate spheres of a wave's primary rays: those whose per-frame screen box (view_params)
// overlaps the wave's pixels.  Lanes 0 and 63 hold the wave's first and last pixel (the row
// mapping is monotonic).  Converged call; p.prim_const required.
#ifndef RT_PRIM_BOX
#define RT_PRIM_BOX 1
#endif
// RT_FAST_PROLOGUE (shipped): the wave's start has no dependent chain of memory round trips --
// the box is one unconditional 16-byte load (lane 0's for lanes >= S), tested without
// short-circuit branches, and the view-table loads are issued before it (tile_prologue).
#ifndef RT_FAST_PROLOGUE
#define RT_FAST_PROLOGUE 1
#endif
__device__ __forceinline__ unsigned long long prim_box_mask(const LaunchParams& p, int x, int y) {
    const int x_lo = __builtin_amdgcn_readlane(x, 0), x_hi = __builtin_amdgcn_readlane(x, 63);
    const int y_lo = __builtin_amdgcn_readlane(y, 0), y_hi = __builtin_amdgcn_readlane(y, 63);
    const int lane = threadIdx.x & 63;
    bool cand = false;
    if constexpr (RT_FAST_PROLOGUE) {
        const bool in = lane < p.S;
        const PrimBox b = p.pbox[in ? lane : 0];
        cand = in & (b.x0 <= x_hi) & (b.x1 >= x_lo) & (b.y0 <= y_hi) & (b.y1 >= y_lo);
    } else if (lane < p.S) {
        const PrimBox b = p.pbox[lane];
        cand = b.x0 <= x_hi && b.x1 >= x_lo && b.y0 <= y_hi && b.y1 >= y_lo;
    }
    return __builtin_amdgcn_ballot_w64(cand);
}

// A wave's pixels: column x, local row r -> frame row y (band band_first + (r / band_rows) *
// band_step), validity, and the view-table entries lx = lxt[x], ly = lyt[y] (0 outside).
// Fast paths without a per-lane integer division: one band (every full-frame launch) and the
// 8-row bands of the multi-GPU path.
struct TilePixel {
    int x, r, y;
    bool valid;
    float lx, ly;
};
__device__ __forceinline__ TilePixel tile_pixel(const LaunchParams& p, int x, int r) {
    TilePixel t;
    t.x = x, t.r = r;
    if (RT_FAST_PROLOGUE && p.band_rows >= p.local_rows) {  // wave-uniform branches
        t.y = p.band_first * p.band_rows + r;
    } else if (RT_FAST_PROLOGUE && p.band_rows == 8) {
        t.y = (p.band_first + (r >> 3) * p.band_step) * 8 + (r & 7);
    } else {
        const int band = p.band_first + (r / p.band_rows) * p.band_step;
        t.y = band * p.band_rows + (r % p.band_rows);
    }
    t.valid = x < p.W && r < p.local_rows && t.y < p.H;
    const float lx = p.lxt[t.valid ? x : 0], ly = p.lyt[t.valid ? t.y : 0];  // unconditional loads
    t.lx = t.valid ? lx : 0.0f, t.ly = t.valid ? ly : 0.0f;
    return t;
}

template <bool PRIMARY, int SMAX>
__device__ __forceinline__ Hit nearest_direct(const LaunchParams& p, f3 o, f3 d, unsigned long long pmask = 0) {
    const float a = dot(d, d);
    const float a2 = 2.0f * a, a4 = 4.0f * a;
    const bool a2_ok = a2 > 0.0f && a2 < __builtin_inff();
    float best_s = __builtin_inff();
    int win_s = -1;
    if (PRIMARY && p.prim_const) {
        // o == camera: oc = cam - c and c = oc.oc - r^2 are the same per frame (:614-619)
        auto test = [&](int i) {
            const PrimConst pc = p.pc[i];
            const float b = 2.0f * dot(mk(pc.ocx, pc.ocy, pc.ocz), d);
            const float disc = b * b - a4 * pc.c;
            const float t = a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2);
            if (t > 0.0f && best_s > t) {
                best_s = t;
                win_s = i;
            }
        };
        if constexpr (RT_PRIM_BOX) {
            // only the wave's candidate spheres, in ascending order (non-candidates give t <= 0)
            for (unsigned long long m = pmask; m; m &= m - 1) test((int)__builtin_ctzll(m));
        } else {
            for_spheres<SMAX>(p.S, test);
        }
    } else {
        for_spheres<SMAX>(p.S, [&](int i) {
            const float t = sphere_t(o, d, a2, a4, a2_ok, p.sph[i]);
            if (PRIMARY) {
                if (t > 0.0f && best_s > t) {
                    best_s = t;
                    win_s = i;
                }
            } else {
                const float tm = t - 0.01f;
                if (tm > 0.0f && tm < best_s) {
                    best_s = t;
                    win_s = i;
                }
            }
        });
    }
    float best_p = __builtin_inff();
    int win_p = -1;
    for (int i = 0; i < p.P; ++i) {
        const float t = plane_t(o, d, p.pl[i]);
        if (t > 0.0f && t < best_p) {
            best_p = t;
            win_p = i;
        }
    }
    if (best_s < best_p) return Hit{best_s, win_s};
    if (win_p >= 0) return Hit{best_p, ~win_p};
    return Hit{0.0f, HIT_NONE};
}

// Terminal segment (bounce count > limit): only its colour is used -- One iff a plane is
// selected with t - 0.01 > 0 and no sphere beats it (TraceSecondaryRay :789-826 with the
// terminal colours of TracePlane :734 / TraceSphere :843), otherwise Zero.  Planes first:
// with no plane hit, or the nearest within 0.01, the colour is Zero whatever the spheres do,
// so they are not tested (RT_TERMINAL).  Returns HIT_NONE (Zero) or the plane hit (One);
// the walk classifies it exactly as it would the full nearest hit.
#ifndef RT_TERMINAL
#define RT_TERMINAL 1
#endif
template <int SMAX>
__device__ __forceinline__ Hit terminal_direct(const LaunchParams& p, f3 o, f3 d) {
    float best_p = __builtin_inff();
    int win_p = -1;
    for (int i = 0; i < p.P; ++i) {
        const float t = plane_t(o, d, p.pl[i]);
        if (t > 0.0f && t < best_p) {
            best_p = t;
            win_p = i;
        }
    }
    if (win_p < 0 || !(best_p - 0.01f > 0.0f)) return Hit{0.0f, HIT_NONE};
    const float a = dot(d, d);
    const float a2 = 2.0f * a, a4 = 4.0f * a;
    const bool a2_ok = a2 > 0.0f && a2 < __builtin_inff();
    float best_s = __builtin_inff();
    for_spheres<SMAX>(p.S, [&](int i) {
        const float t = sphere_t(o, d, a2, a4, a2_ok, p.sph[i]);
        const float tm = t - 0.01f;
        if (tm > 0.0f && tm < best_s) best_s = t;
    });
    if (best_s < best_p) return Hit{0.0f, HIT_NONE};  // a sphere is selected: Zero
    return Hit{best_p, ~win_p};
}

// DIRECT kernel: each lane walks its own chain with per-lane (divergent) control flow.
template <int K, bool SCRATCH, bool GPOW, int SMAX>
// RT_PRIO (experiment): issue priority by phase.  > 0 raises it as a wave reaches its later
// phases (1: for the backward fold; 2: 1 after the primary segment, 2 for the fold) -- older
// waves win VALU arbitration even more than by age (C2 +15 %, C3 +9…17 %: rejected).  < 0 gives
// young waves the priority instead (-1: 1 until the primary segment is done; -2: 2 until then,
// 1 through the walk, 0 for the fold).
#ifndef RT_PRIO
#define RT_PRIO 0
#endif
__global__ __launch_bounds__(WG_THREADS) void trace_direct_kernel(LaunchParams p) {
    if constexpr (RT_PRIO < 0) __builtin_amdgcn_s_setprio(-RT_PRIO);
    constexpr int LDS_LEVELS = StackFor<K, SCRATCH>::lds_levels;  // LdsStack slots, else unused
    __shared__ float2 stk_lv[LDS_LEVELS > 0 ? LDS_LEVELS * WG_THREADS : 1];
    __shared__ float stk_dv[LDS_LEVELS > 0 ? 3 * WG_THREADS : 1];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const TilePixel tpx = tile_pixel(p, blockIdx.x * TILE_W + (wave % WG_WX) * 8 + (lane & 7),
                                     blockIdx.y * TILE_H + (wave / WG_WX) * 8 + (lane >> 3));
    const int x = tpx.x, r = tpx.r, y = tpx.y;
    const bool valid = tpx.valid;
    const unsigned long long pmask = (RT_PRIM_BOX && p.prim_const) ? prim_box_mask(p, x, y) : 0;

    unsigned cnt = 0;  // packed: reflected segments (bits 0-7) | shadow rays << CNT_SHADOW_SHIFT
    if (valid) {
        const f3 cam = mk(p.cam[0], p.cam[1], p.cam[2]);
        // TracePixel primary ray, :963-971 (no half-pixel offset)
        // lx = ((float)x / W - 0.5f) * pw, ly likewise: per-column / per-row tables built on
        // the host with the same binary32 operations (view_tables in rt_api.cpp)
        const float lx = tpx.lx, ly = tpx.ly, lz = 1.0f * p.nearc;
        const f3 vp = add(add(add(cam, scale(mk(p.right[0], p.right[1], p.right[2]), lx)),
                              scale(mk(p.up[0], p.up[1], p.up[2]), ly)),
                          scale(mk(p.fwd[0], p.fwd[1], p.fwd[2]), lz));
        f3 d = normalize(sub(vp, cam));
        f3 o = cam;

        typename StackFor<K, SCRATCH>::overflow ovf;
        typename StackFor<K, SCRATCH>::type stk(&ovf, stk_lv, stk_dv);
        stk.origin(d);
        f3 leaf = mk(0.0f, 0.0f, 0.0f);
        Hit h = nearest_direct<true, SMAX>(p, o, d, pmask);
        if constexpr (RT_PRIO >= 2 || RT_PRIO == -2) __builtin_amdgcn_s_setprio(1);
        if constexpr (RT_PRIO == -1) __builtin_amdgcn_s_setprio(0);
        int count = 0;
        for (;;) {
            if (h.prim == HIT_NONE) break;      // nothing hit: plane colour stays Zero
            if (h.t - 0.01f <= 0.0f) break;     // too close: Zero (:731, :839)
            const bool is_sphere = h.prim >= 0;
            if (count > p.limit) {              // terminal segment: Zero / One (:734, :843)
                if (!is_sphere) leaf = mk(1.0f, 1.0f, 1.0f);
                break;
            }
            // shaded hit: record it; mirror hits continue with the reflected segment
            const f3 hp = add(o, scale(d, h.t));
            stk.push(make_float4(hp.x, hp.y, hp.z, h.t), make_float4(d.x, d.y, d.z, __int_as_float(h.prim)));
            const int prim = is_sphere ? h.prim : ~h.prim;
            const uint32_t flags = p.mat[is_sphere ? prim : p.S + prim].flags;
            if (!(flags & MAT_MIRROR) || RT_ABLATE == 3) break;
            o = reflect_at(p, o, d, h.t, h.prim);  // :854, CalculateReflectionRay :718-720
            ++count;
            ++cnt;
            // count is the same for every lane still walking: no divergence here
            h = (RT_TERMINAL && count > p.limit) ? terminal_direct<SMAX>(p, o, d) : nearest_direct<false, SMAX>(p, o, d);
        }
        // backward fold: every recorded hit is shaded in reverse order; a mirror hit
        // consumes the colour of the segment after it (levels 0..limit push at most one
        // record each, so K = limit + 1 records suffice)
        f3 col = leaf;
        if constexpr (RT_ABLATE == 1) {  // keep the walk alive: fold the records' t into the colour
            while (stk.n > 0) {
                float4 ra, rb;
                stk.pop(p, ra, rb);
                col.x += ra.w;
            }
        }
        if constexpr (RT_PRIO >= 1) __builtin_amdgcn_s_setprio(RT_PRIO >= 2 ? 2 : 1);
        if constexpr (RT_PRIO == -2) __builtin_amdgcn_s_setprio(0);
        while (RT_ABLATE != 1 && stk.n > 0) {
            float4 ra, rb;
            stk.pop(p, ra, rb);
            const int code = __float_as_int(rb.w);
            const bool is_s = code >= 0;
            col = shade_direct<GPOW, SMAX>(p, is_s, is_s ? code : ~code, mk(ra.x, ra.y, ra.z), mk(rb.x, rb.y, rb.z), ra.w, col,
                              &cnt);
        }
        const uint32_t px32 = (shift_channel(col.x) << 16) | (shift_channel(col.y) << 8) | shift_channel(col.z);
        store_pixel(p, r, y, x, px32);
    }

    add_counters(p, lane, wave, valid ? 1u : 0u, cnt & CNT_REFL_MASK, cnt >> CNT_SHADOW_SHIFT);
}

// ---------------------------------------------------------------------------------
// Wave-level ray bundles and conservative sphere culling.
//
// A wave's active rays (origins o_l, directions d_l) are bounded by a reference origin O,
// an origin radius R >= max |o_l - O|, a unit axis A and a direction spread
// delta >= max |d_l/|d_l| - A|.  Lane i tests sphere i against the bundle and a ballot
// gives the wave's candidate mask; the exact per-lane tests then visit only candidates,
// in ascending sphere index (so the reference's tie rules are untouched).
//
// Exactness: a sphere is culled only when, for EVERY lane, the binary32 evaluation of
// IntersectsSphere provably yields disc < 0 or b >= 0 -- both make the reference's
// distance non-selectable (root_t1).  With u = o - C and a = d.d, a first-order error
// analysis of disc = fl(fl(b*b) - fl(fl(4a)*fl(fl(u.u) - r^2))) bounds its error by
// 4a(14 eps |u|^2 + 4 eps r^2) (eps = 2^-24), so disc < 0 whenever the exact
// line-to-centre distance D satisfies D >= r (1 + 3 eps) + 9.2e-4 |u|; b >= 0 whenever
// u.d/|d| >= 4 eps |u|.  The cull demands D >= r (1 + 2^-8) + 2^-8 (|C - O| + R) and
// u.A >= 2^-8 (|C - O| + R) after subtracting the bundle slack (R, delta terms) --
// a 4x margin over the analysis, far above the rounding of the cull arithmetic itself.
// Culling is disabled for a wave when any active lane has a = d.d outside [0.5, 2]
// (trace rays) or the light's a outside [2^-40, 2^40] (shadow rays), or for spheres
// with r^2 < 2^-100 or |C - O| outside [2^-30, 2^40] (no underflow/overflow).
// ---------------------------------------------------------------------------------
struct Bundle {
    f3 O, A;
    float R, delta;
    bool ok;   // culling allowed
    bool any;  // some lane active
};

__device__ __forceinline__ float readlane_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ f3 readlane3(f3 v, int lane) {
    return mk(readlane_f(v.x, lane), readlane_f(v.y, lane), readlane_f(v.z, lane));
}
// Wave-uniform maximum of a non-negative float (all 64 lanes active): DPP row rotations
// give each 16-lane row its maximum, four readlanes and integer max (bit patterns of
// non-negative floats order like the floats; a NaN pattern compares above +inf) finish it.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f<0x121>(v));  // row_ror:1
    v = fmaxf(v, dpp_f<0x122>(v));  // row_ror:2
    v = fmaxf(v, dpp_f<0x124>(v));  // row_ror:4
    v = fmaxf(v, dpp_f<0x128>(v));  // row_ror:8
    const unsigned a = (unsigned)__builtin_amdgcn_readlane(__float_as_int(v), 0);
    const unsigned b = (unsigned)__builtin_amdgcn_readlane(__float_as_int(v), 16);
    const unsigned c = (unsigned)__builtin_amdgcn_readlane(__float_as_int(v), 32);
    const unsigned d = (unsigned)__builtin_amdgcn_readlane(__float_as_int(v), 48);
    return __uint_as_float(max(max(a, b), max(c, d)));
}
__device__ __forceinline__ float len3(f3 v) { return __builtin_sqrtf(dot(v, v)); }
// Culling-only arithmetic (never feeds a result): hardware sqrt / rsq (about 1 ulp) instead of
// the correctly rounded sequences; the cull margins (2^-10 relative on R and delta, 2^-8 on
// the tests) are orders of magnitude above that error.
#ifndef RT_FAST_CULL
#define RT_FAST_CULL 1
#endif
__device__ __forceinline__ float clen3(f3 v) {
#if RT_FAST_CULL
    return __builtin_amdgcn_sqrtf(dot(v, v));
#else
    return len3(v);
#endif
}
__device__ __forceinline__ f3 cnormalize(f3 v) {
#if RT_FAST_CULL
    return scale(v, __builtin_amdgcn_rsqf(dot(v, v)));
#else
    return normalize(v);
#endif
}
__device__ __forceinline__ f3 cross3(f3 l, f3 r) {
    return mk(l.y * r.z - l.z * r.y, l.z * r.x - l.x * r.z, l.x * r.y - l.y * r.x);
}

// Converged call (all 64 lanes).  `dir_uniform`: every lane's direction is `d` itself
// (shadow rays: the light position), so delta = 0.
__device__ __forceinline__ Bundle make_bundle(f3 o, f3 d, bool active, bool dir_uniform) {
    Bundle B;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(active);
    B.any = m != 0;
    if (m == 0) {
        B.ok = false;
        B.O = o;
        B.A = d;
        B.R = B.delta = 0.0f;
        return B;
    }
    const int ref = __builtin_ctzll(m);
    B.O = readlane3(o, ref);
    const f3 dref = readlane3(d, ref);
    B.A = cnormalize(dref);
    float e = 0.0f, f = 0.0f;
    bool bad = false;
    if (active) {
        e = clen3(sub(o, B.O));
        bad = !(e < 0x1p40f);  // also NaN / inf origins
        if (!dir_uniform) {
            const float a = dot(d, d);
            f = clen3(sub(cnormalize(d), B.A));
            bad = bad || !(a >= 0.5f && a <= 2.0f) || !(f < 2.0f);
        }
    }
    const float R = wave_max(e);
    const float delta = dir_uniform ? 0.0f : wave_max(f);
    bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    B.R = R * (1.0f + 0x1p-10f) + 0x1p-60f;
    B.delta = dir_uniform ? 0.0f : delta * (1.0f + 0x1p-10f) + 0x1p-20f;
    B.ok = !bad && R < 0x1p40f && B.delta < 0.5f;
    return B;
}

// Candidate mask of spheres [base, base+n) (n <= 64) for bundle B.  Converged call.
__device__ __forceinline__ unsigned long long cull_mask(const LaunchParams& p, const Bundle& B, int base, int n) {
    const int lane = threadIdx.x & 63;
    bool cand = false;
    if (lane < n) {
        cand = true;
        if (B.ok) {
#if RT_FAST_CULL
            const DevSphereCull s = p.scull[base + lane];
            const f3 w = sub(mk(s.cx, s.cy, s.cz), B.O);
            const float dc = clen3(w) * (1.0f + 0x1p-20f);
            if (s.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f) {
                const float rr = s.rr;
#else
            const DevSphere s = p.sph[base + lane];
            const f3 w = sub(mk(s.cx, s.cy, s.cz), B.O);
            const float dc = len3(w);
            if (s.r2 >= 0x1p-100f && dc >= 0x1p-30f && dc < 0x1p40f) {
                const float rr = __builtin_sqrtf(s.r2) * (1.0f + 0x1p-8f);
#endif
                const float mgn = 0x1p-8f * (dc + B.R);
                const float x = clen3(cross3(w, B.A));
                const bool line = (x - dc * B.delta - B.R) > rr + mgn;
                const bool behind = (-dot(w, B.A) - dc * B.delta - B.R * (1.0f + B.delta)) > mgn;
                cand = !(line || behind);  // NaN anywhere -> candidate
            }
        }
    }
    return __builtin_amdgcn_ballot_w64(cand);
}

// Shadow bundles.  Every shadow ray of light l has the same direction p_l (the light
// POSITION, Q2), so a sphere can block lane k only if the line {hp_k + s p_l} passes within
// r of its centre: a 2-D test in the light's frame (U, V, A ~ p_l/|p_l|, host-built), where
// the wave's hit points spread by R_perp across A and by [-R_neg, R_pos] along it.  Cull
// rules (same error analysis and 2^-8 margin as cull_mask, with |u| bounded by the L1 norm
// of the frame coordinates plus the spreads): line miss if |w_perp| - R_perp > r' + mgn;
// behind (b >= 0 for every lane) if -w_A - R_neg > mgn, where w = C - O.
#ifndef RT_SHADOW_CULL
#define RT_SHADOW_CULL 1
#endif
struct ShadowBundle {
    f3 O;
    float Rp, Rneg, Rsum;  // perpendicular spread, backward spread, Rp + Rneg + Rpos
    bool ok;
};

__device__ __forceinline__ ShadowBundle make_shadow_bundle(f3 hp, const DevLight& l, bool active) {
    ShadowBundle B;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(active);
    B.ok = false;
    B.Rp = B.Rneg = B.Rsum = 0.0f;
    B.O = hp;
    if (m == 0) return B;
    B.O = readlane3(hp, __builtin_ctzll(m));
    float perp2 = 0.0f, neg = 0.0f, pos = 0.0f;
    bool bad = false;
    if (active) {
        const f3 e = sub(hp, B.O);
        const float eu = dot(e, mk(l.ux, l.uy, l.uz));
        const float ev = dot(e, mk(l.vx, l.vy, l.vz));
        const float ea = dot(e, mk(l.ax, l.ay, l.az));
        perp2 = eu * eu + ev * ev;
        neg = nmax0(-ea);
        pos = nmax0(ea);
        bad = !(perp2 < 0x1p80f) || !(neg < 0x1p40f) || !(pos < 0x1p40f);  // also NaN / inf
    }
    bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    const float Rp2 = wave_max(perp2);
    B.Rp = __builtin_sqrtf(Rp2) * (1.0f + 0x1p-10f) + 0x1p-60f;
    B.Rneg = wave_max(neg) * (1.0f + 0x1p-10f) + 0x1p-60f;
    const float Rpos = wave_max(pos) * (1.0f + 0x1p-10f) + 0x1p-60f;
    B.Rsum = B.Rp + B.Rneg + Rpos;
    B.ok = !bad && l.a >= 0x1p-40f && l.a <= 0x1p40f && l.a2 < __builtin_inff() && B.Rsum < 0x1p41f;
    return B;
}

// Candidate mask of spheres [base, base+n) (n <= 64) for shadow bundle B.  Converged call.
__device__ __forceinline__ unsigned long long shadow_cull_mask(const LaunchParams& p, const ShadowBundle& B,
                                                               const DevLight& l, int base, int n) {
    const int lane = threadIdx.x & 63;
    bool cand = false;
    if (lane < n) {
        cand = true;
        if (B.ok) {
            const DevSphereCull s = p.scull[base + lane];
            const f3 w = sub(mk(s.cx, s.cy, s.cz), B.O);
            const float wu = dot(w, mk(l.ux, l.uy, l.uz));
            const float wv = dot(w, mk(l.vx, l.vy, l.vz));
            const float wa = dot(w, mk(l.ax, l.ay, l.az));
            const float dc = __builtin_fabsf(wu) + __builtin_fabsf(wv) + __builtin_fabsf(wa);  // >= |w|
            if (s.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f) {
                const float mgn = 0x1p-8f * (dc + B.Rsum);
                const float T = B.Rp + s.rr + mgn;
                const bool line = wu * wu + wv * wv > T * T;
                const bool behind = -wa - B.Rneg > mgn;
                cand = !(line || behind);  // NaN anywhere -> candidate
            }
        }
    }
    return __builtin_amdgcn_ballot_w64(cand);
}

// BUNDLE path.  Nearest hit of one segment for every active lane (converged call).  PRIMARY: TracePixel's
// rule (:977, :987, :993) with the per-frame camera-relative constants; otherwise
// TraceSecondaryRay's asymmetric rule (:804-806, :819-821, :825).

template <bool PRIMARY>
__device__ __forceinline__ Hit nearest_bundle(const LaunchParams& p, f3 o, f3 d, bool active,
                                              unsigned long long pmask = 0) {
    const unsigned long long am = __builtin_amdgcn_ballot_w64(active);
    if (am == 0) return Hit{0.0f, HIT_NONE};
    // primary segment: the per-frame screen boxes replace the bundle cull
    const bool use_box = PRIMARY && RT_PRIM_BOX && p.prim_const;
    Bundle B{};
    if (!use_box) B = make_bundle(o, d, active, false);
    if (am != ~0ull) {  // idle lanes trace an exact copy of the first active lane's ray, so
        const int ref = __builtin_ctzll(am);  // they never add divergence (results ignored)
        const f3 ro = readlane3(o, ref), rd = readlane3(d, ref);
        if (!active) {
            o = ro;
            d = rd;
        }
    }
    const float a = dot(d, d);
    const float a2 = 2.0f * a, a4 = 4.0f * a;
    const bool a2_ok = a2 > 0.0f && a2 < __builtin_inff();
    float best_s = __builtin_inff();
    int win_s = -1;
    for (int base = 0; base < p.S; base += 64) {
        const int n = min(64, p.S - base);
        unsigned long long m = use_box ? pmask : cull_mask(p, B, base, n);  // use_box: S <= 64
        while (m) {
            const int i = base + (int)__builtin_ctzll(m);
            m &= m - 1;
            float t;
            if (PRIMARY && p.prim_const) {
                // o == camera: oc = cam - c and c = oc.oc - r^2 are per-frame constants (:614-619)
                const PrimConst pc = p.pc[i];
                const float b = 2.0f * dot(mk(pc.ocx, pc.ocy, pc.ocz), d);
                const float disc = b * b - a4 * pc.c;
                t = a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2);
            } else {
                t = sphere_t(o, d, a2, a4, a2_ok, p.sph[i]);
            }
            if (PRIMARY) {
                if (t > 0.0f && best_s > t) {
                    best_s = t;
                    win_s = i;
                }
            } else {
                const float tm = t - 0.01f;
                if (tm > 0.0f && tm < best_s) {
                    best_s = t;
                    win_s = i;
                }
            }
        }
    }
    float best_p = __builtin_inff();
    int win_p = -1;
    for (int i = 0; i < p.P; ++i) {
        const float t = plane_t(o, d, p.pl[i]);
        if (t > 0.0f && t < best_p) {
            best_p = t;
            win_p = i;
        }
    }
    if (!active) return Hit{0.0f, HIT_NONE};
    if (best_s < best_p) return Hit{best_s, win_s};
    if (win_p >= 0) return Hit{best_p, ~win_p};
    return Hit{0.0f, HIT_NONE};
}

// Shading of one shaded hit per active lane (TraceSphere :847-873 / TracePlane :736-778),
// converged call: the colour is accumulated in the reference's order -- mirror term (from
// the deeper segment `sec`), then each light in order, then ambient.  Inactive lanes
// return `sec` unchanged.  Shadow rays (IntersectShadowLight :573-582) of the lanes that
// need them form one bundle per light (common direction = the light position).
template <bool GPOW>
__device__ __forceinline__ f3 shade_bundle(const LaunchParams& p, bool act, bool is_sphere, int prim, f3 hp, f3 d, float t,
                                    f3 sec, unsigned* n_shadow) {
    // idle lanes (act false) carry a copy of an active lane's record: same branches, result dropped
    const DevMaterial& m = p.mat[is_sphere ? prim : p.S + prim];
    const uint32_t flags = m.flags;
    f3 normal;
    float tile = 1.0f;
    if (is_sphere) {
        const DevSphere& s = p.sph[prim];
        normal = normalize(sub(hp, mk(s.cx, s.cy, s.cz)));  // SpherePhongShading :706
    } else {
        const DevPlane& pl = p.pl[prim];
        normal = mk(pl.nx, pl.ny, pl.nz);
        // checkerboard, :766-770: ((int)u + (int)v) & 1, unchecked int add
        const float u = dot(mk(pl.e1x, pl.e1y, pl.e1z), hp);
        const float v = dot(mk(pl.e2x, pl.e2y, pl.e2z), hp);
        tile = (float)(int32_t)(((uint32_t)net_f2i(u) + (uint32_t)net_f2i(v)) & 1u);
    }
    f3 col = mk(0.0f, 0.0f, 0.0f);
    if (flags & MAT_MIRROR) col = add(col, mul(sec, mk(m.km[0], m.km[1], m.km[2])));
    const bool diff = act && (flags & MAT_DIFFUSE) != 0;
    if (__builtin_amdgcn_ballot_w64(diff) != 0) {
        const f3 view = normalize(d);  // ShapePhongShading :668 (not negated)
        // sphere: (1 / t) * t (:866);  plane: (float)(1 / Math.Pow(t, 2)) (:754), exact as 1/(t*t) in f64
        const float att = is_sphere ? cr_rcp(t) * t : (float)(1.0 / ((double)t * (double)t));
        const f3 kd = mk(m.kd[0], m.kd[1], m.kd[2]);
        for (int li = 0; li < p.L; ++li) {
            const DevLight& l = p.li[li];
            const f3 lp = mk(l.px, l.py, l.pz);
            const bool l_ok = l.a2 > 0.0f && l.a2 < __builtin_inff();  // wave-uniform
            // ShapePhongShading, :665-695 (first: it decides whether the shadow test matters)
            const f3 ldir = normalize(sub(lp, hp));
            f3 ph = scale(kd, nmax0(dot(normal, ldir)));
            f3 spec = mk(0.0f, 0.0f, 0.0f);
            if (flags & MAT_SPEC) {
                const f3 rs = sub(ldir, scale(normal, 2.0f * dot(ldir, normal)));
                const float sp = spec_pow<GPOW>(nmax0(dot(view, normalize(rs))), m);
                spec = mul(mk(m.ks[0], m.ks[1], m.ks[2]), mk(sp, sp, sp));
            }
            ph = add(ph, spec);
            const bool need = diff && shadow_matters(ph, l.intensity, att);
            bool blocked = !need;
            if (__builtin_amdgcn_ballot_w64(need) != 0) {  // some lane's pixel depends on this test

#if RT_SHADOW_CULL
                const ShadowBundle B = make_shadow_bundle(hp, l, need);
#else
                Bundle B = make_bundle(hp, lp, need, true);
                B.ok = B.ok && l_ok && l.a >= 0x1p-40f && l.a <= 0x1p40f;
#endif
                const f3 hs = need ? hp : B.O;  // idle lanes mirror a shading lane (results ignored)
                if constexpr (RT_CULLSTATS == 2) *n_shadow += (unsigned)((threadIdx.x & 63) == 0) << CNT_SHADOW_SHIFT;
                for (int base = 0; RT_ABLATE != 2 && base < p.S; base += 64) {
                    const int n = min(64, p.S - base);
#if RT_SHADOW_CULL
                    unsigned long long mk64 = shadow_cull_mask(p, B, l, base, n);
#else
                    unsigned long long mk64 = cull_mask(p, B, base, n);
#endif
                    while (mk64) {
                        const int i = base + (int)__builtin_ctzll(mk64);
                        mk64 &= mk64 - 1;
                        if constexpr (RT_CULLSTATS == 1) *n_shadow += (unsigned)((threadIdx.x & 63) == 0) << CNT_SHADOW_SHIFT;
                        blocked = blocked | shadow_blocked(hs, l, l_ok, p.sph[i]);  // no short-circuit branch
                        if (__builtin_amdgcn_ballot_w64(!blocked) == 0) break;
                    }
                    if (__builtin_amdgcn_ballot_w64(!blocked) == 0) break;
                }
            }
            const float inten = (!diff || (need && blocked)) ? 0.0f : l.intensity;
            const float ia = inten * att;
            f3 term = mul(mk(ia, ia, ia), ph);
            if (!is_sphere) {
                term = mul(term, mk(tile, tile, tile));
                term = mk(nmax0(term.x), nmax0(term.y), nmax0(term.z));  // .Max(0f), :775
            }
            if (diff) col = add(col, term);
        }
        if (diff && !RT_CULLSTATS) *n_shadow += (unsigned)p.L << CNT_SHADOW_SHIFT;
    }
    col = add(col, mk(m.amb[0], m.amb[1], m.amb[2]));
    return act ? col : sec;
}

// BUNDLE kernel (scenes with >= CULL_MIN_SPHERES spheres): converged control flow so that
// every segment and every light can form a wave bundle and cull the sphere list.
template <int K, bool SCRATCH, bool GPOW>
__global__ __launch_bounds__(WG_THREADS) void trace_bundle_kernel(LaunchParams p) {
    constexpr int LDS_LEVELS = StackFor<K, SCRATCH>::lds_levels;  // LdsStack slots, else unused
    __shared__ float2 stk_lv[LDS_LEVELS > 0 ? LDS_LEVELS * WG_THREADS : 1];
    __shared__ float stk_dv[LDS_LEVELS > 0 ? 3 * WG_THREADS : 1];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const TilePixel tpx = tile_pixel(p, blockIdx.x * TILE_W + (wave % WG_WX) * 8 + (lane & 7),
                                     blockIdx.y * TILE_H + (wave / WG_WX) * 8 + (lane >> 3));
    const int x = tpx.x, r = tpx.r, y = tpx.y;
    const bool valid = tpx.valid;

    unsigned cnt = 0;  // packed: reflected segments (bits 0-7) | shadow rays << CNT_SHADOW_SHIFT
    const f3 cam = mk(p.cam[0], p.cam[1], p.cam[2]);
    // TracePixel primary ray, :963-971 (no half-pixel offset)
    // per-column / per-row tables (see the direct kernel); lanes outside the frame read 0
    const float lx = tpx.lx, ly = tpx.ly, lz = 1.0f * p.nearc;
    const f3 vp = add(add(add(cam, scale(mk(p.right[0], p.right[1], p.right[2]), lx)),
                          scale(mk(p.up[0], p.up[1], p.up[2]), ly)),
                      scale(mk(p.fwd[0], p.fwd[1], p.fwd[2]), lz));
    f3 d = normalize(sub(vp, cam));
    f3 o = cam;

    // forward walk: all lanes advance one segment per iteration (converged loop), each
    // shaded hit pushes a record; mirror hits continue with the reflected segment
    typename StackFor<K, SCRATCH>::overflow ovf;
    typename StackFor<K, SCRATCH>::type stk(&ovf, stk_lv, stk_dv);
        stk.origin(d);
    f3 leaf = mk(0.0f, 0.0f, 0.0f);
    bool active = valid;
    const unsigned long long pmask = (RT_PRIM_BOX && p.prim_const) ? prim_box_mask(p, x, y) : 0;
    Hit h = nearest_bundle<true>(p, o, d, active, pmask);
    for (int count = 0;; ++count) {
        if (active) {
            const bool is_sphere = h.prim >= 0;
            if (h.prim == HIT_NONE || h.t - 0.01f <= 0.0f) {  // nothing hit / too close: Zero (:731, :839)
                active = false;
            } else if (count > p.limit) {  // terminal segment: Zero / One (:734, :843)
                if (!is_sphere) leaf = mk(1.0f, 1.0f, 1.0f);
                active = false;
            } else {
                const f3 hp = add(o, scale(d, h.t));
                stk.push(make_float4(hp.x, hp.y, hp.z, h.t), make_float4(d.x, d.y, d.z, __int_as_float(h.prim)));
                const int prim = is_sphere ? h.prim : ~h.prim;
                const uint32_t flags = p.mat[is_sphere ? prim : p.S + prim].flags;
                if (!(flags & MAT_MIRROR) || RT_ABLATE == 3) {
                    active = false;
                } else {
                    o = reflect_at(p, o, d, h.t, h.prim);  // :854, CalculateReflectionRay :718-720
                    ++cnt;
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(active) == 0) break;
        if (RT_TERMINAL && count + 1 > p.limit) {
            // terminal segment (see terminal_direct): only lanes whose nearest plane lies beyond
            // 0.01 need the spheres; the others are Zero
            float best_p = __builtin_inff();
            int win_p = -1;
            for (int i = 0; i < p.P; ++i) {
                const float t = plane_t(o, d, p.pl[i]);
                if (t > 0.0f && t < best_p) {
                    best_p = t;
                    win_p = i;
                }
            }
            const bool need = active && win_p >= 0 && best_p - 0.01f > 0.0f;
            h = Hit{0.0f, HIT_NONE};
            if (__builtin_amdgcn_ballot_w64(need) != 0) {
                const Hit hn = nearest_bundle<false>(p, o, d, need);
                if (need) h = hn;
            }
        } else {
            h = nearest_bundle<false>(p, o, d, active);
        }
    }

    // backward fold (converged): level by level from the deepest, every recorded hit is
    // shaded; a mirror hit consumes the colour of the segment after it (levels 0..limit
    // push at most one record each, so K = limit + 1 records suffice)
    f3 col = leaf;
    const int depth = stk.n;
    int level = (int)wave_max((float)depth);
    if constexpr (RT_ABLATE == 1) {  // keep the walk alive: fold the records' t into the colour
        while (stk.n > 0) {
            float4 ra, rb;
            stk.pop(p, ra, rb);
            col.x += ra.w;
        }
        level = 0;
    }
    while (level-- > 0) {
        const bool act = level < depth;  // this lane's top record is at `level`
        float4 ra = make_float4(0.0f, 0.0f, 0.0f, 1.0f), rb = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
        if (act) stk.pop(p, ra, rb);
        const unsigned long long am = __builtin_amdgcn_ballot_w64(act);
        if (am != ~0ull) {  // idle lanes shade a copy of the first active lane's record
            const int ref = __builtin_ctzll(am);
            const float4 qa = make_float4(readlane_f(ra.x, ref), readlane_f(ra.y, ref), readlane_f(ra.z, ref),
                                          readlane_f(ra.w, ref));
            const float4 qb = make_float4(readlane_f(rb.x, ref), readlane_f(rb.y, ref), readlane_f(rb.z, ref),
                                          readlane_f(rb.w, ref));
            if (!act) {
                ra = qa;
                rb = qb;
            }
        }
        const int code = __float_as_int(rb.w);
        const bool is_s = code >= 0;
        col = shade_bundle<GPOW>(p, act, is_s, is_s ? code : ~code, mk(ra.x, ra.y, ra.z), mk(rb.x, rb.y, rb.z), ra.w, col,
                          &cnt);
    }
    if (valid) {
        const uint32_t px32 = (shift_channel(col.x) << 16) | (shift_channel(col.y) << 8) | shift_channel(col.z);
        store_pixel(p, r, y, x, px32);
    }

    add_counters(p, lane, wave, valid ? 1u : 0u, cnt & CNT_REFL_MASK, cnt >> CNT_SHADOW_SHIFT);
}

// ---------------------------------------------------------------------------------
// Debug ray view: re-trace sampled pixels with the direct path's
// selection rules and append their visible-path segments.  Not on the timed path.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ void append_segment(DevSegment* out, int cap, unsigned* count, f3 o, f3 e, int kind,
                                               int pixel) {
    const unsigned i = atomicAdd(count, 1u);
    if (i < (unsigned)cap) out[i] = DevSegment{o.x, o.y, o.z, e.x, e.y, e.z, kind, pixel};
}

__global__ __launch_bounds__(256) void debug_segments_kernel(LaunchParams p, int stride, DevSegment* out, int cap,
                                                             unsigned* count) {
    const long long idx = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * (long long)stride;
    if (idx >= (long long)p.W * p.H) return;
    const int x = (int)(idx % p.W), y = (int)(idx / p.W);
    const f3 cam = mk(p.cam[0], p.cam[1], p.cam[2]);
    const float px = (float)x / (float)p.W - 0.5f;
    const float py = (float)y / (float)p.H - 0.5f;
    const f3 vp = add(add(add(cam, scale(mk(p.right[0], p.right[1], p.right[2]), px * p.pw)),
                          scale(mk(p.up[0], p.up[1], p.up[2]), py * p.ph)),
                      scale(mk(p.fwd[0], p.fwd[1], p.fwd[2]), 1.0f * p.nearc));
    f3 d = normalize(sub(vp, cam));
    f3 o = cam;
    Hit h = nearest_direct<true, 0>(p, o, d, p.S >= 64 ? ~0ull : (1ull << p.S) - 1);  // every sphere
    for (int level = 0;; ++level) {
        const bool none = h.prim == HIT_NONE;
        append_segment(out, cap, count, o, add(o, scale(d, none ? 100.0f : h.t)), level == 0 ? 0 : 1,
                       (int)idx);
        if (none || h.t - 0.01f <= 0.0f || level > p.limit) break;
        const bool is_sphere = h.prim >= 0;
        const int prim = is_sphere ? h.prim : ~h.prim;
        const f3 hp = add(o, scale(d, h.t));
        const DevMaterial& m = p.mat[is_sphere ? prim : p.S + prim];
        if (m.flags & MAT_DIFFUSE) {
            for (int li = 0; li < p.L; ++li) {  // IntersectShadowLight's ray per light
                const DevLight& l = p.li[li];
                const bool l_ok = l.a2 > 0.0f && l.a2 < __builtin_inff();
                const f3 lp = mk(l.px, l.py, l.pz);
                float tb = 1.0f;
                for (int i = 0; i < p.S; ++i) {
                    if (shadow_blocked(hp, l, l_ok, p.sph[i])) {
                        const f3 oc = sub(hp, mk(p.sph[i].cx, p.sph[i].cy, p.sph[i].cz));
                        const float b = 2.0f * dot(oc, lp);
                        const float c = dot(oc, oc) - p.sph[i].r2;
                        const float sq = __builtin_sqrtf(b * b - l.a4 * c);
                        tb = (-b - sq) / l.a2;
                        break;
                    }
                }
                append_segment(out, cap, count, hp, add(hp, scale(lp, tb)), 2, (int)idx);
            }
        }
        if (!(m.flags & MAT_MIRROR)) break;
        const f3 normal = is_sphere ? normalize(sub(hp, mk(p.sph[prim].cx, p.sph[prim].cy, p.sph[prim].cz)))
                                    : mk(p.pl[prim].nx, p.pl[prim].ny, p.pl[prim].nz);
        d = sub(d, scale(normal, 2.0f * dot(d, normal)));
        o = hp;
        h = nearest_direct<false, 0>(p, o, d);
    }
}

// Reassemble packed row bands (rt_render_bands layout) into a row-major frame.
__global__ __launch_bounds__(256) void scatter_bands_kernel(const int32_t* __restrict__ bands,
                                                            int32_t* __restrict__ frame, int W, int H, int band_rows,
                                                            int band_first, int band_step, int local_rows) {
    const size_t total = (size_t)local_rows * (size_t)W;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / (size_t)W);
        const int x = (int)(i - (size_t)r * W);
        const int y = (band_first + (r / band_rows) * band_step) * band_rows + r % band_rows;
        if (y < H) frame[(size_t)y * W + x] = bands[i];
    }
}

// Reassemble every rank's gathered band set into the row-major frame in one launch:
// frame row y is band b = y / band_rows, owned by rank b % world as its (b / world)-th band.
__global__ __launch_bounds__(256) void scatter_gathered_kernel(const unsigned char* __restrict__ g, size_t slot_bytes,
                                                               int fmt, int32_t* __restrict__ frame, int W, int H,
                                                               int band_rows, int world) {
    const size_t total = (size_t)W * (size_t)H;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int y = (int)(i / (size_t)W);
        const int x = (int)(i - (size_t)y * W);
        const int b = y / band_rows;
        const int rank = b % world;
        const size_t local = ((size_t)(b / world) * band_rows + (size_t)(y % band_rows)) * (size_t)W + (size_t)x;
        const unsigned char* src = g + (size_t)rank * slot_bytes;
        int32_t v;
        if (fmt == 0) {
            v = ((const int32_t*)src)[local];
        } else {
            const unsigned char* q = src + local * 3;
            v = (int32_t)((uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16));
        }
        frame[i] = v;
    }
}

#define RT_DEFINE_DISPATCH(FN, NAME, ...)                                                        \
    template <bool GPOW>                                                                         \
    static void FN(const LaunchParams& p, dim3 grid, dim3 block, hipStream_t s) {                \
        const int need = p.limit + 1; /* levels 0..limit can push a record */                    \
        if (need <= 1)                                                                           \
            hipLaunchKernelGGL((NAME<1, false, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
        else if (need <= 2)                                                                      \
            hipLaunchKernelGGL((NAME<2, false, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
        else if (need <= 4)                                                                      \
            hipLaunchKernelGGL((NAME<4, false, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
        else if (need <= 6)                                                                      \
            hipLaunchKernelGGL((NAME<6, false, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
        else if (need <= 8)                                                                      \
            hipLaunchKernelGGL((NAME<8, false, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
        else                                                                                     \
            hipLaunchKernelGGL((NAME<64, true, GPOW __VA_ARGS__>), grid, block, 0, s, p);        \
    }
RT_DEFINE_DISPATCH(launch_direct_loop, trace_direct_kernel, , 0)
RT_DEFINE_DISPATCH(launch_bundle, trace_bundle_kernel)
#undef RT_DEFINE_DISPATCH

int launch_trace(const LaunchParams& p, bool generic_pow, void* stream) {
    if (p.local_rows <= 0 || p.W <= 0) return (int)hipSuccess;
    const dim3 grid((unsigned)((p.W + TILE_W - 1) / TILE_W), (unsigned)((p.local_rows + TILE_H - 1) / TILE_H),
                    (unsigned)(p.n_frames > 1 ? p.n_frames : 1));
    const dim3 block(WG_THREADS);
    hipStream_t s = (hipStream_t)stream;
    // bundle culling pays for its per-wave bounds only with enough spheres (A/B: +15 % at
    // 8 spheres, 3x faster at 64)
    const bool bundle = p.S >= CULL_MIN_SPHERES;
    if (generic_pow) {
        if (bundle) launch_bundle<true>(p, grid, block, s);
        else launch_direct_loop<true>(p, grid, block, s);
    } else {
        if (bundle) launch_bundle<false>(p, grid, block, s);
        else launch_direct_loop<false>(p, grid, block, s);
    }
    return (int)hipGetLastError();
}

int launch_debug_segments(const LaunchParams& p, int stride, DevSegment* out, int capacity, unsigned* count,
                          void* stream) {
    const long long n = ((long long)p.W * p.H + stride - 1) / stride;
    if (n <= 0) return (int)hipSuccess;
    hipLaunchKernelGGL(debug_segments_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p,
                       stride, out, capacity, count);
    return (int)hipGetLastError();
}

int launch_scatter_gathered(const unsigned char* g, size_t slot_bytes, int fmt, int32_t* frame, int W, int H,
                            int band_rows, int world, void* stream) {
    const size_t total = (size_t)W * (size_t)H;
    if (total == 0) return (int)hipSuccess;
    size_t blocks = (total + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(scatter_gathered_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, g,
                       slot_bytes, fmt, frame, W, H, band_rows, world);
    return (int)hipGetLastError();
}

int launch_scatter_bands(const int32_t* bands, int32_t* frame, int W, int H, int band_rows, int band_first,
                         int band_step, int n_bands, void* stream) {
    const size_t total = (size_t)n_bands * band_rows * W;
    if (total == 0) return (int)hipSuccess;
    size_t blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(scatter_bands_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, bands, frame,
                       W, H, band_rows, band_first, band_step, n_bands * band_rows);
    return (int)hipGetLastError();
}

}  // namespace rtk
