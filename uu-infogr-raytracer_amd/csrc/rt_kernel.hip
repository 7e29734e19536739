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
#include "rt_codec_common.h"
#include "rt_internal.h"

// One wave (64 lanes, an 8x8 pixel tile) per workgroup: a one-wave group releases its LDS
// stack slots as soon as it ends.  The dispatcher launches one-wave groups no faster than
// ~6.9 us per 1080p frame (tools/launch_probe.hip, a store-only kernel), but with real work
// that is not the limit: 4-wave groups and waves looping over 2/4/8 tiles all measured equal
// or slower (C2 +0..16 %, C3 +3..22 %, C4 +16..37 %; profiles/ab/r02_tiles_per_wg_rejected.txt).
constexpr int WG_THREADS = 64, TILE_W = 8, TILE_H = 8;

namespace rtk {

// Correctly rounded binary32 operations.  Vector3.Normalize's 1f / MathF.Sqrt(x) runs the short
// sequence of rt_fastmath.h inside its verified domain (the same bits as the generic sequence for
// every input, tools/fastmath_check.hip); the same treatment of the other sqrt and of division
// measured slower (profiles/ab/r01_fastmath.txt), so they use the generic operations.
__device__ __forceinline__ float cr_sqrt(float x) { return __builtin_sqrtf(x); }
__device__ __forceinline__ float cr_inv_len(float x) { return inv_len_cr(x); }  // 1f / MathF.Sqrt(x)
__device__ __forceinline__ float cr_rcp(float x) { return 1.0f / x; }

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
// -b > 0 first.  So: no sqrt when b >= 0, never the t2 division.  Returns the reference's
// distance when it is selectable and otherwise a value <= 0 or NaN, which every caller's
// selection test (t > 0, t - 0.01 > 0) rejects exactly as it rejects the reference's 0:
// fl(-b - sq) <= 0 whenever -b <= sq (and NaN when disc < 0), and dividing by the positive
// 2a keeps the sign -- identical selections and identical winning distances.
//
// Scalar-issue economy (MI355X: one scalar unit per CU serves its 4 SIMDs, ~1 SALU
// instruction per CU-cycle against ~1.8 VALU, profiles/r02_issue_probe.txt): the sqrt and the
// division run under a wave-uniform branch on the ballot of the candidate lanes instead of an
// exec-mask if/else, and the result needs no select.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ bool sphere_candidate(float b, float disc) {
    // disc >= 0 && b <= 0 (b = +-0 cannot select: -b > sq fails); NaN -> false
    return __builtin_elementwise_minimum(disc, -b) >= 0.0f;
}
__device__ __forceinline__ float root_t1(float b, float disc, float a2) {
    float t = 0.0f;
    if (__builtin_amdgcn_ballot_w64(sphere_candidate(b, disc)) != 0) {  // wave-uniform
        const float sq = cr_sqrt(disc);  // == (float)Math.Sqrt((double)disc); NaN off-candidate
        t = (-b - sq) / a2;              // t1 = (-b - sqrt) / 2a, :630
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

// A2OK: 2a is finite and > 0 for every active lane (checked once per segment with a ballot,
// so the sphere loops carry no per-lane two-way split).
template <bool A2OK>
__device__ __forceinline__ float root_sel(float b, float disc, float a2, bool a2_ok) {
    if constexpr (A2OK) return root_t1(b, disc, a2);
    else return a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2);
}
template <bool A2OK>
__device__ __forceinline__ float sphere_t(f3 o, f3 d, float a2, float a4, bool a2_ok, const DevSphere& s) {
    const f3 oc = sub(o, mk(s.cx, s.cy, s.cz));
    const float b = 2.0f * dot(oc, d);
    const float c = dot(oc, oc) - s.r2;
    const float disc = b * b - a4 * c;
    return root_sel<A2OK>(b, disc, a2, a2_ok);
}

// Shadow ray of IntersectShadowLight (origin = hit point, direction = light POSITION,
// epsilon 0.001, RayTracer.cs:574-578): collision iff min(max(t1-e,0), max(t2-e,0)) > 0.
// With 2a finite-positive (uniform per light) and t2 >= t1 that is t1 - e > 0 (and then
// t2 - e > 0 too); fl(-b - sq) / 2a - e > 0 already implies -b > sq (see root_t1).
// THRESH: the same predicate without the division -- t1 - e > 0 iff fl(-b - sq) >= l.sh_t, the
// per-light threshold of the correctly rounded quotient (rt_api.cpp shadow_threshold; NaN
// compares false, as the reference's NaN distance does).  Used by the bundle kernel (C4 -3 % with
// paired candidates); in the direct kernel the division-free form measured slower (C2 +4 %, C3
// +6 %: the shading code around it was scheduled worse), so it keeps the division there.
template <bool A2OK, bool THRESH = false>
__device__ __forceinline__ bool shadow_decide(float b, float disc, const DevLight& l, bool a2_ok) {
    if (A2OK || a2_ok) {
        bool hit = false;
        if (__builtin_amdgcn_ballot_w64(sphere_candidate(b, disc)) != 0) {  // wave-uniform
            const float sq = cr_sqrt(disc);
            if constexpr (THRESH) hit = -b - sq >= l.sh_t;  // == fl(fl(-b - sq) / 2a) - 0.001f > 0
            else hit = (-b - sq) / l.a2 - 0.001f > 0.0f;
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
template <bool A2OK, bool THRESH = false>
__device__ __forceinline__ bool shadow_blocked(f3 hp, const DevLight& l, bool a2_ok, const DevSphere& s) {
    const f3 oc = sub(hp, mk(s.cx, s.cy, s.cz));
    const float b = 2.0f * dot(oc, mk(l.px, l.py, l.pz));
    const float c = dot(oc, oc) - s.r2;
    const float disc = b * b - l.a4 * c;
    return shadow_decide<A2OK, THRESH>(b, disc, l, a2_ok);
}


// IntersectPlane, RayTracer.cs:590-604: t = (((-o.x*n.x) - o.y*n.y) - o.z*n.z + c.n) / d.n,
// hit iff t > 0 -- the quotient itself.  (+inf, from a zero denominator, is a "hit" that no
// nearest-plane search can select: the best distance starts at +inf and the test is strict.)
__device__ __forceinline__ float plane_t(f3 o, f3 d, const DevPlane& p) {
    const float num = ((-o.x * p.nx - o.y * p.ny) - o.z * p.nz) + p.cn;
    const float den = dot(d, mk(p.nx, p.ny, p.nz));
    return num / den;
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
// The Tick hand-off (CopyJob): a band set, device -> the caller's registered host buffer through its
// device-mapped address, 16 bytes per lane (both ends 16-byte aligned, checked on the host), band k
// of the packed source at k * dst_stride in the frame (one band set per device of a multi-GPU Tick,
// each device's bands cross its own PCIe link).  As a trace launch's copy slice (z = 0)
// it is dispatched before the trace workgroups, so the PCIe-bound copy of frame (or chunk) k-1 runs
// under the trace of k on one in-order stream.  Only the first COPY_WAVES workgroups copy
// (grid-strided, 4 loads in flight per lane), the others exit at once: a wave holds its slot until its
// host stores are acknowledged, and a slice of one-store waves (8,100 at 1080p) held nearly every wave
// slot of the chip until PCIe had drained them, so the trace waited.
constexpr unsigned COPY_WAVES = 512;
__device__ __forceinline__ size_t band_dst(const CopyJob& j, unsigned i) {  // source word -> frame word
    if (j.band_words == 0) return i;
    const unsigned k = i / j.band_words;  // (words < 2^31: W * H is capped on the host)
    return (size_t)k * j.dst_stride + (i - k * j.band_words);
}
__device__ __forceinline__ void copy_job(const CopyJob& j, size_t wg, size_t nwg) {
    const size_t lane = threadIdx.x & 63;
    const unsigned long long n = j.words, n4 = n / 4;
    const int4* __restrict__ s4 = (const int4*)j.src;
    const size_t step = nwg * 64;
    size_t i = wg * 64 + lane;
    if (j.band_words == 0) {
        int4* __restrict__ d4 = (int4*)j.dst;
        for (; i + 3 * step < n4; i += 4 * step) {
            const int4 a = s4[i], b = s4[i + step], c = s4[i + 2 * step], d = s4[i + 3 * step];
            d4[i] = a;
            d4[i + step] = b;
            d4[i + 2 * step] = c;
            d4[i + 3 * step] = d;
        }
        for (; i < n4; i += step) d4[i] = s4[i];
    } else {  // band_words and dst_stride are multiples of 4: a 16-byte chunk never straddles a band
        // (one chunk per lane and iteration, 32-bit chunk indices: this path shares the trace kernels'
        // register allocation, which must not grow -- 512 waves keep ~0.5 MB in flight, plenty for PCIe)
        int4* __restrict__ d4 = (int4*)j.dst;
        const unsigned bq = j.band_words / 4, sq = (unsigned)(j.dst_stride / 4);
        for (unsigned c = (unsigned)i; c < (unsigned)n4; c += (unsigned)step) {
            const unsigned k = c / bq;
            d4[k * sq + (c - k * bq)] = s4[c];
        }
    }
    if (wg == 0 && lane < n - n4 * 4) j.dst[band_dst(j, (unsigned)(n4 * 4 + lane))] = j.src[n4 * 4 + lane];
}
__device__ __forceinline__ void copy_slice(const LaunchParams& p) {
    const size_t nwg = min((size_t)gridDim.x * gridDim.y, (size_t)COPY_WAVES);
    const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (wg < nwg) copy_job(p.copy, wg, nwg);
}
__global__ __launch_bounds__(64) void band_copy_kernel(CopyJob j) { copy_job(j, blockIdx.x, gridDim.x); }

__device__ __forceinline__ void store_pixel(const LaunchParams& p, int r, int y, int x, uint32_t px32) {
    const size_t i = (size_t)(p.out_fmt == 2 ? y : r) * (size_t)p.W + (size_t)x;
    // batch frame z (a launch with the copy slice has one frame and out_frame_bytes 0)
    unsigned char* base = (unsigned char*)p.out + (size_t)blockIdx.z * p.out_frame_bytes;
    if (p.out_fmt != 1) {
        ((int32_t*)base)[i] = (int32_t)px32;
    } else {
        unsigned char* o = base + i * 3;
        o[0] = (unsigned char)px32;
        o[1] = (unsigned char)(px32 >> 8);
        o[2] = (unsigned char)(px32 >> 16);
    }
}

// OUT_TILES: the tile codec's encoder (rt_codec.hip encode_group, format raytracer_hip/tilecodec.py)
// fused into the trace -- the wave's 8x8 tile (lane = ry * 8 + rx) goes straight from registers to
// its tile header and staged segments, and the band set never reaches HBM.  Converged call.
// Residuals: dx = p - left (column 0: p - the tile's first pixel), minus the row above's dx (lane
// - 8); widths from the wave OR; a row's w bytes of a segment are the OR of its 8 lanes' fields.
__device__ __forceinline__ void encode_tile_fused(const LaunchParams& p, uint32_t px, bool valid) {
    const int lane = threadIdx.x & 63, rx = lane & 7, ry = lane >> 3;
    // (cross-lane steps by DPP / bpermute, so that the tile's values stay in VGPRs: readlanes
    // here would raise the direct kernel's SGPR peak above 80 and cost it a wave per SIMD)
    const uint32_t v = valid ? px & 0xffffffu : 0u;
    const uint32_t first = (uint32_t)__shfl((int)v, 0, 64);
    const size_t t = (size_t)(p.enc_frame0 + (int)blockIdx.z) * (size_t)p.enc_tpf +
                     (size_t)blockIdx.y * (size_t)p.enc_tiles_x + blockIdx.x;
    if (__builtin_amdgcn_ballot_w64(valid && v != first) == 0) {  // one colour (sky): no residual
        if (lane == 0) wire_tile_hdr(p.enc_wire)[t] = first;
        return;
    }
    const uint32_t left = row_shr<1>(v);  // lane - 1: the same row for rx >= 1
    const uint32_t dx = sub_bytes(v, rx ? left : first);
    const uint32_t above = (uint32_t)__shfl_up((int)dx, 8, 64);  // lane - 8: the row above
    const uint32_t z = valid ? zigzag_bytes(ry ? sub_bytes(dx, above) : dx) & 0xffffffu : 0u;
    uint32_t o = group8_or(z);  // the tile's OR, in every lane
    o |= (uint32_t)__shfl_xor((int)o, 8, 64);
    o |= (uint32_t)__shfl_xor((int)o, 16, 64);
    o |= (uint32_t)__shfl_xor((int)o, 32, 64);
    const uint32_t iR = width_index((o >> 16) & 0xffu), iG = width_index((o >> 8) & 0xffu),
                   iB = width_index(o & 0xffu);
    const uint32_t wm = width_at(iR) | (width_at(iG) << 4) | (width_at(iB) << 8);
    if (lane == 0) wire_tile_hdr(p.enc_wire)[t] = first | ((iR + 6u * iG + 36u * iB) << 24);
    if (wm) {  // (the same in every lane)
        unsigned char* seg = (unsigned char*)(p.enc_stage + t * STAGE_WORDS);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const uint32_t w = (wm >> (4 * c)) & 15u;
            if (w) {
                const uint64_t f = (uint64_t)((z >> (16 - 8 * c)) & 0xffu) << (rx * w);
                const uint32_t lo = group8_or((uint32_t)f), hi = group8_or((uint32_t)(f >> 32));
                if (rx == 0) store_row_bits(seg + ry * w, w, ((uint64_t)hi << 32) | lo);
            }
            seg += 8 * w;
        }
    }
}

// Deep-recursion stack (recursion limits >= 8): whole records {hit point, t} and {incoming
// direction, primitive code}, dynamically indexed, in scratch.
template <int K>
struct ScratchStack {
    float4 a[K], b[K];
    int n = 0;
    __device__ __forceinline__ ScratchStack(float2*, float*) {}
    __device__ __forceinline__ void origin(f3) {}
    __device__ __forceinline__ void push(float4 x, float4 y) {
        a[n] = x;
        b[n] = y;
        ++n;
    }
    __device__ __forceinline__ void pop(const LaunchParams&, float4& x, float4& y) {
        --n;
        x = a[n];
        y = b[n];
    }
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

// Compact levels: a record is fully determined by the camera ray and the (t, primitive)
// pairs of the levels above it, so each level keeps only those 8 bytes and pop rebuilds the
// record by re-walking the reflection chain with reflect_at (bit-identical).
// Level stack for limits 0..7: the compact levels and the primary direction in LDS, one slot per thread
// ([level][thread], conflict-free), so they cost no VGPRs; pop re-walks as in CompactStack.
template <int K>
struct LdsStack {
    float2* lv;  // [K][WG_THREADS] (t, primitive code) of this workgroup
    float* dv;   // [3][WG_THREADS] primary direction
    int n = 0;
    __device__ __forceinline__ LdsStack(float2* l, float* dd) : lv(l), dv(dd) {}
    __device__ __forceinline__ void origin(f3 d) {
        dv[(threadIdx.x & 63)] = d.x;
        dv[WG_THREADS + (threadIdx.x & 63)] = d.y;
        dv[2 * WG_THREADS + (threadIdx.x & 63)] = d.z;
    }
    __device__ __forceinline__ void push(float4 x, float4 y) {
        lv[n * WG_THREADS + (threadIdx.x & 63)] = make_float2(x.w, y.w);
        ++n;
    }
    __device__ __forceinline__ void pop(const LaunchParams& p, float4& x, float4& y) {
        --n;
        f3 o = mk(p.cam[0], p.cam[1], p.cam[2]);
        f3 d = mk(dv[(threadIdx.x & 63)], dv[WG_THREADS + (threadIdx.x & 63)], dv[2 * WG_THREADS + (threadIdx.x & 63)]);
#pragma unroll 1
        for (int j = 0; j < K - 1; ++j) {
            const bool go = j < n;
            if (__builtin_amdgcn_ballot_w64(go) == 0) break;
            if (go) {
                const float2 tc = lv[j * WG_THREADS + (threadIdx.x & 63)];
                o = reflect_at(p, o, d, tc.x, __float_as_int(tc.y));
            }
        }
        const float2 tk = lv[n * WG_THREADS + (threadIdx.x & 63)];
        const f3 hp = add(o, scale(d, tk.x));
        x = make_float4(hp.x, hp.y, hp.z, tk.x);
        y = make_float4(d.x, d.y, d.z, tk.y);
    }
};

// Stack type per K (= recursion limit + 1 records): the LDS stack up to 8 levels (A/B round 1:
// no VGPRs for records, -2..-5.5 % on C4/C5 against register and hybrid stacks), scratch beyond.
template <int K>
struct StackFor {
    using type = ScratchStack<K>;
    static constexpr int lds_levels = 0;
};
#define RT_LDS_STACK(K)                        \
    template <>                                \
    struct StackFor<K> {                       \
        using type = LdsStack<K>;              \
        static constexpr int lds_levels = K;   \
    };
RT_LDS_STACK(1)
RT_LDS_STACK(2)
RT_LDS_STACK(4)
RT_LDS_STACK(6)
RT_LDS_STACK(8)
#undef RT_LDS_STACK

// Sum of v over the wave (all lanes active): bit-sliced ballots and scalar popcounts, no
// LDS round trips; the loop runs once per significant bit of the largest v (uniform).
__device__ __forceinline__ unsigned wave_count(unsigned v) {
    unsigned s = 0;
    for (int j = 0; __builtin_amdgcn_ballot_w64(v != 0u) != 0; ++j, v >>= 1)
        s += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64((v & 1u) != 0u)) << j;
    return s;
}

// Per-lane work counts share one register: reflected segments (<= RT_MAX_RECURSION_LIMIT + 1)
// in the low byte, shadow rays (<= lights x 64; rt_set_scene caps lights at 65536) above.
constexpr unsigned CNT_SHADOW_SHIFT = 8;
constexpr unsigned CNT_REFL_MASK = 0xFFu;

// Executed-work tally of the diagnostic kernels (STATS = true; never the timed ones): exact
// IntersectsSphere / IntersectPlane evaluations a lane actually ran, and the shadow rays whose
// sphere loop ran (a shadow ray is skipped when its outcome cannot change the pixel, and culling
// skips sphere tests that provably cannot select) -- reported beside the nominal counts of
// SURVEY.md 8(d), which count every primitive of every ray.
// SMAX > 0: the scene has at most SMAX spheres (a compile-time bound: the pair loops over the
// sphere table are unrolled, no loop counter or pointer arithmetic on the scalar unit).
#ifndef RT_SLOT_TALLY
#define RT_SLOT_TALLY 0
#endif
// RT_SHADOW_CAT=1 (diagnostic builds, tools/shadow_slots.py): sphere_tests_run counts only the
// bundle kernel's shadow-test lane slots of one category, chosen at run time by rt_count_work's
// selector (RT_DIAG_SEL = 16 * category + level + 1, level -1 = every fold level): category 1
// useful (needed, not yet blocked), 2 needed but already blocked, 3 diffuse but not needed,
// 4 active record, not diffuse, 5 no record at this level.
#ifndef RT_SHADOW_CAT
#define RT_SHADOW_CAT 0
#endif

template <bool ON, int SMAX = 0>
struct Tally {
    static constexpr int smax = SMAX;
    __device__ __forceinline__ void sphere(bool) {}
    __device__ __forceinline__ void shadow_sphere(bool) {}
    __device__ __forceinline__ void plane(bool) {}
    __device__ __forceinline__ void shadow(bool) {}
    __device__ __forceinline__ void init(const LaunchParams&) {}
    __device__ __forceinline__ void set_level(int) {}
    __device__ __forceinline__ void shadow_cat(int, unsigned) {}
    __device__ __forceinline__ void shadow_masks(int, unsigned long long) {}
};
template <int SMAX>
struct Tally<true, SMAX> {
    static constexpr int smax = SMAX;
    unsigned s = 0, pl = 0, sh = 0;
    int lvl = 0, sel_cat = 0, sel_lvl = -1;
    // RT_SLOT_TALLY (diagnostic builds, tools/slot_probe.py): lane slots of the exact tests,
    // useful or not -- 1: every sphere test, 2: the nearest-hit tests only
    __device__ __forceinline__ void sphere(bool c) { s += (!RT_SHADOW_CAT && (RT_SLOT_TALLY || c)) ? 1u : 0u; }
    __device__ __forceinline__ void shadow_sphere(bool c) {
        s += (!RT_SHADOW_CAT && (RT_SLOT_TALLY == 1 || c)) ? 1u : 0u;
    }
    __device__ __forceinline__ void plane(bool c) { pl += c ? 1u : 0u; }
    __device__ __forceinline__ void shadow(bool c) { sh += c ? 1u : 0u; }
    __device__ __forceinline__ void init(const LaunchParams& p) {
        sel_cat = p.enc_frame0 / 16;
        sel_lvl = p.enc_frame0 % 16 - 1;
    }
    __device__ __forceinline__ void set_level(int l) { lvl = l; }
    __device__ __forceinline__ void shadow_cat(int cat, unsigned n) {
        s += (RT_SHADOW_CAT && cat + 1 == sel_cat && (sel_lvl < 0 || lvl == sel_lvl)) ? n : 0u;
    }
    // categories 6 / 7 (lane 0 only): candidates per light's shadow pass / of the union of a shaded
    // level's lights -- how far the lights' candidate sets overlap
    __device__ __forceinline__ void shadow_masks(int cat, unsigned long long m) {
        if (RT_SHADOW_CAT && cat + 1 == sel_cat && (sel_lvl < 0 || lvl == sel_lvl) && (threadIdx.x & 63) == 0)
            s += (unsigned)__builtin_popcountll(m);
    }
};

// Work counters of one wave (converged call): ballot/popcount sums, lane 0 adds the wave's
// totals to slot (wave id % COUNTER_SLOTS); primary rays are the traced pixels, counted on the
// host.  Every frame of a batch launch (grid z) traces the same view with the same
// LaunchParams, so its counts are identical: frame 0 counts for all n_frames of them -- one
// atomic pair per wave per launch instead of per frame (each device-scope atomic is a memory
// round trip on MI355X, 32 B of HBM write traffic).  In a one-frame launch every wave counts, and
// the atomics cost the frame more than their round trips: C2 19.6 -> 22.5 us, C3 36.1 -> 39.6 us,
// C4 337 -> 352 us per lone frame (+15 % L2 requests, +22 % waves parked on memory; spreading them
// over 8192 slots instead of 256 changed nothing, profiles/r05_bundle_lone.txt) -- so a
// display loop that never reads rt_get_stats turns them off (rt_set_counting, ABI 10).
template <bool ST, int SM>
__device__ __forceinline__ void add_counters(const LaunchParams& p, int lane, unsigned n_refl, unsigned n_shadow,
                                             const Tally<ST, SM>& tl) {
    // wave-uniform: the first frame (behind a copy slice) counts, and only when the context counts at all
    if (blockIdx.z != (unsigned)p.copy_z || p.counters == nullptr) return;
    const unsigned long long nf = p.n_frames > 1 ? (unsigned long long)p.n_frames : 1ull;
    const unsigned b = wave_count(n_refl), c = wave_count(n_shadow);
    const unsigned slot = (blockIdx.y * gridDim.x + blockIdx.x) % COUNTER_SLOTS;
    unsigned long long* q = &p.counters[slot * COUNTER_STRIDE];
    if (lane == 0) {
        if (b) atomicAdd(q + CNT_REFLECT, b * nf);
        if (c) atomicAdd(q + CNT_SHADOW, c * nf);
    }
    if constexpr (ST) {
        const unsigned s = wave_count(tl.s), pl = wave_count(tl.pl), sh = wave_count(tl.sh);
        if (lane == 0) {
            if (sh) atomicAdd(q + CNT_SHADOW_RUN, sh * nf);
            if (s) atomicAdd(q + CNT_SPHERE_RUN, s * nf);
            if (pl) atomicAdd(q + CNT_PLANE_RUN, pl * nf);
        }
    }
}

// Result of a nearest-hit search.
struct Hit {
    float t;
    int prim;  // >= 0 sphere, ~plane for planes, or HIT_NONE
};
constexpr int HIT_NONE = 0x7fffffff;

// Nearest-hit selection rules as selects (VALU compares and cndmasks, no scalar mask logic),
// on the bit patterns: with u(x) = bits(x) - 1 (unsigned, wrapping), +0, every negative value and
// every NaN map above u(+inf) = 0x7f7fffff, and positive floats keep their order.  `best` is
// always +inf or a taken positive distance, so "x > 0 && x < best" is exactly u(x) < u(best)
// (x = +inf: u(x) = u(+inf) >= u(best), not taken, as in the float rule) -- one compare and a
// min instead of two compares and two selects (C4 -0.5 %, C2/C3 +-0,
// profiles/ab/r02_umin_take.txt).
// TracePixel (:977, :987): t is taken iff t > 0 && best > t.
__device__ __forceinline__ void take_primary(float t, int i, float& best, int& win) {
    const unsigned u = __float_as_uint(t) - 1u, ub = __float_as_uint(best) - 1u;
    win = u < ub ? i : win;
    best = __uint_as_float(min(u, ub) + 1u);
}
// TraceSecondaryRay (:804-806): t is taken iff t - 0.01 > 0 && t - 0.01 < best, and then
// best = t (the asymmetric rule, Q5/Q6).
__device__ __forceinline__ void take_secondary(float t, int i, float& best, int& win) {
    const float tm = t - 0.01f;
    const bool b = __float_as_uint(tm) - 1u < __float_as_uint(best) - 1u;
    best = b ? t : best;
    win = b ? i : win;
}

// A plane test in a nearest-plane search (TracePixel :985-991, TraceSecondaryRay :819-821 -- the same rule):
// t = num / den is selectable only when t > 0, i.e. num and den nonzero with equal signs (zeros give +-0,
// +-inf or NaN, and +inf never beats the initial +inf); when no lane of the wave (of the active lanes, in
// divergent code) has such a pair the division and the selection are skipped -- the upper half of a
// frame for a floor, rays leaving a wall -- and otherwise every lane takes the literal quotient.
__device__ __forceinline__ void plane_take(f3 o, f3 d, const DevPlane& q, int i, float& best, int& win) {
    const float num = ((-o.x * q.nx - o.y * q.ny) - o.z * q.nz) + q.cn;
    const float den = dot(d, mk(q.nx, q.ny, q.nz));
    const bool may = (num > 0.0f && den > 0.0f) || (num < 0.0f && den < 0.0f);
    if (__builtin_amdgcn_ballot_w64(may) != 0) take_primary(num / den, i, best, win);  // (wave-uniform)
}

// DIRECT path (scenes with < CULL_MIN_SPHERES spheres): per-lane divergent walks, wave-uniform
// primitive loops.  Shading of one shaded hit (TraceSphere :847-873 / TracePlane :736-778): the
// colour is accumulated in the reference's order -- mirror term (from the deeper segment `sec`),
// then each light, then ambient.  Returns the colour; adds shadow rays to *n_shadow.
// A light's shadow test can change the pixel only through I * att * phong vs 0 * phong.  When
// every phong component is +-0 or NaN and I * att is finite, both give +-0 / NaN per
// component (the sign of a zero never reaches a pixel: only additions, products, IEEE max and
// the final clamp follow), so the test is skipped.  Ray counters are unchanged
// (shadow rays = shaded diffuse hits x lights); the diagnostic tally counts the tests that ran.
__device__ __forceinline__ bool zero_or_nan(float v) { return !(v != 0.0f && v == v); }
__device__ __forceinline__ bool shadow_matters(f3 ph, float intensity, float att) {
    const float ia = intensity * att;
    const bool finite = __builtin_fabsf(ia) < __builtin_inff();
    return !(finite && zero_or_nan(ph.x) && zero_or_nan(ph.y) && zero_or_nan(ph.z));
}

// Loop over the sphere table two spheres at a time (the device table is padded to an even count
// with a sphere that never hits, rt_set_scene): body(i) tests spheres i and i + 1.  Unrolled
// when the scene's sphere count has a compile-time bound (T::smax).
template <typename T, typename F>
__device__ __forceinline__ void for_sphere_pairs(const LaunchParams& p, F body) {
    if constexpr (T::smax > 0) {
#pragma unroll
        for (int i = 0; i < T::smax; i += 2) {
            if (i >= p.S) break;  // wave-uniform
            body(i);
        }
    } else {
        for (int i = 0; i < p.S; i += 2) body(i);
    }
}

// IntersectShadowLight's sphere loop (:577-579) for the active lanes: every sphere, a lane's
// result the OR of its tests, as in the reference.  The scalar unit bounds these kernels (one per
// CU for 4 SIMDs, profiles/r02_issue_probe.txt), so the loop is shaped for scalar economy: the
// blocked state is a VGPR value (no lane-mask phi), one 32-byte scalar load per pair, no per-lane
// loop exits (their mask bookkeeping cost ~28 scalar instructions per sphere) and no wave exit
// once every lane is blocked (it almost never fires: C2 -1.4 %, C3 -1.0 % without it,
// profiles/ab/r02_shadow_loop.txt).
template <bool A2OK, typename T>
__device__ __forceinline__ bool shadow_scan(const LaunchParams& p, f3 hp, const DevLight& l, T& tl) {
    int blk = 0;
    for_sphere_pairs<T>(p, [&](int i) {
        tl.shadow_sphere(blk == 0);
        const DevSphere s0 = p.sph[i], s1 = p.sph[i + 1];
        blk = shadow_blocked<A2OK>(hp, l, false, s0) ? 1 : blk;
        tl.shadow_sphere((blk == 0) & (i + 1 < p.S));
        blk = shadow_blocked<A2OK>(hp, l, false, s1) ? 1 : blk;
    });
    return blk != 0;
}

template <bool GPOW, typename T>
__device__ __forceinline__ f3 shade_direct(const LaunchParams& p, bool is_sphere, int prim, f3 hp, f3 d, float t, f3 sec,
                                           unsigned* n_shadow, T& tl) {
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
                tl.shadow(true);
                blocked = l_ok ? shadow_scan<true>(p, hp, l, tl) : shadow_scan<false>(p, hp, l, tl);
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
// mapping is monotonic).  The wave's start has no dependent chain of memory round trips: the
// box is one unconditional 16-byte load (lane 0's for lanes >= S), tested without
// short-circuit branches.  Converged call; p.prim_const required.
__device__ __forceinline__ unsigned long long prim_box_mask(const LaunchParams& p, int x, int y) {
    const int x_lo = __builtin_amdgcn_readlane(x, 0), x_hi = __builtin_amdgcn_readlane(x, 63);
    const int y_lo = __builtin_amdgcn_readlane(y, 0), y_hi = __builtin_amdgcn_readlane(y, 63);
    const int lane = threadIdx.x & 63;
    const bool in = lane < p.S;
    const PrimBox b = p.pbox[in ? lane : 0];
    const bool cand = in & (b.x0 <= x_hi) & (b.x1 >= x_lo) & (b.y0 <= y_hi) & (b.y1 >= y_lo);
    return __builtin_amdgcn_ballot_w64(cand);
}

// A wave's pixels: column x, local row r -> frame row y (band band_first + (r / band_rows) *
// band_step), validity, and the view-table entries lx = lxt[x], ly = lyt[y] (0 outside).
// Fast paths without a per-lane integer division: one band (every full-frame launch) and the
// 8-row bands of the multi-GPU path; the view-table loads are unconditional.
struct TilePixel {
    int x, r, y;
    bool valid;
    float lx, ly;
};
__device__ __forceinline__ TilePixel tile_pixel(const LaunchParams& p, int x, int r) {
    TilePixel t;
    t.x = x, t.r = r;
    if (p.band_rows >= p.local_rows) {  // wave-uniform branches
        t.y = p.band_first * p.band_rows + r;
    } else if (p.band_rows == 8) {
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

// Sphere part of a nearest-hit search for the active lanes.  PRIMARY with p.prim_const: the
// per-frame camera-relative constants and the wave's screen-box candidates (pmask); otherwise
// every sphere (IntersectsSphere, :613-642).  A2OK: 2a finite-positive on every active lane.
template <bool PRIMARY, bool A2OK, typename T>
__device__ __forceinline__ void nearest_spheres(const LaunchParams& p, f3 o, f3 d, float a2, float a4, bool a2_ok,
                                                unsigned long long pmask, float& best_s, int& win_s, T& tl) {
    if (PRIMARY && p.prim_const) {
        // o == camera: oc = cam - c and c = oc.oc - r^2 are the same per frame (:614-619);
        // only the wave's candidate spheres, in ascending order (non-candidates give t <= 0)
        for (unsigned long long m = pmask; m;) {
            const int i = (int)__builtin_ctzll(m);
            m &= ~(1ull << i);
            tl.sphere(true);
            const PrimConst pc = p.pc[i];
            const float b = 2.0f * dot(mk(pc.ocx, pc.ocy, pc.ocz), d);
            const float disc = b * b - a4 * pc.c;
            const float t = A2OK ? root_t1(b, disc, a2) : (a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2));
            take_primary(t, i, best_s, win_s);
        }
    } else {
        // pairs (the device table is padded to an even count with a sphere that never hits)
        for_sphere_pairs<T>(p, [&](int i) {
            tl.sphere(true);
            tl.sphere(i + 1 < p.S);
            const DevSphere s0 = p.sph[i], s1 = p.sph[i + 1];
            const float t0 = sphere_t<A2OK>(o, d, a2, a4, a2_ok, s0);
            const float t1 = sphere_t<A2OK>(o, d, a2, a4, a2_ok, s1);
            if (PRIMARY) {
                take_primary(t0, i, best_s, win_s);
                take_primary(t1, i + 1, best_s, win_s);
            } else {
                take_secondary(t0, i, best_s, win_s);
                take_secondary(t1, i + 1, best_s, win_s);
            }
        });
    }
}

template <bool PRIMARY, typename T>
__device__ __forceinline__ Hit nearest_direct(const LaunchParams& p, f3 o, f3 d, T& tl, unsigned long long pmask = 0) {
    const float a = dot(d, d);
    const float a2 = 2.0f * a, a4 = 4.0f * a;
    const bool a2_ok = a2 > 0.0f && a2 < __builtin_inff();
    float best_s = __builtin_inff();
    int win_s = -1;
    if (__builtin_amdgcn_ballot_w64(!a2_ok) == 0)  // wave-uniform (the usual case)
        nearest_spheres<PRIMARY, true>(p, o, d, a2, a4, a2_ok, pmask, best_s, win_s, tl);
    else
        nearest_spheres<PRIMARY, false>(p, o, d, a2, a4, a2_ok, pmask, best_s, win_s, tl);
    float best_p = __builtin_inff();
    int win_p = -1;
    for (int i = 0; i < p.P; ++i) {
        tl.plane(true);
        plane_take(o, d, p.pl[i], i, best_p, win_p);  // t > 0 && t < best (:985-991, :819-821)
    }
    if (best_s < best_p) return Hit{best_s, win_s};
    if (win_p >= 0) return Hit{best_p, ~win_p};
    return Hit{0.0f, HIT_NONE};
}

// Terminal segment (bounce count > limit): only its colour is used -- One iff a plane is
// selected with t - 0.01 > 0 and no sphere beats it (TraceSecondaryRay :789-826 with the
// terminal colours of TracePlane :734 / TraceSphere :843), otherwise Zero.  Planes first:
// with no plane hit, or the nearest within 0.01, the colour is Zero whatever the spheres do,
// so they are not tested.  Returns HIT_NONE (Zero) or the plane hit (One);
// the walk classifies it exactly as it would the full nearest hit.
template <typename T>
__device__ __forceinline__ Hit terminal_direct(const LaunchParams& p, f3 o, f3 d, T& tl) {
    float best_p = __builtin_inff();
    int win_p = -1;
    for (int i = 0; i < p.P; ++i) {
        tl.plane(true);
        plane_take(o, d, p.pl[i], i, best_p, win_p);
    }
    if (win_p < 0 || !(best_p - 0.01f > 0.0f)) return Hit{0.0f, HIT_NONE};
    const float a = dot(d, d);
    const float a2 = 2.0f * a, a4 = 4.0f * a;
    const bool a2_ok = a2 > 0.0f && a2 < __builtin_inff();
    float best_s = __builtin_inff();
    int win_s = -1;
    if (__builtin_amdgcn_ballot_w64(!a2_ok) == 0)
        nearest_spheres<false, true>(p, o, d, a2, a4, a2_ok, 0, best_s, win_s, tl);
    else
        nearest_spheres<false, false>(p, o, d, a2, a4, a2_ok, 0, best_s, win_s, tl);
    if (best_s < best_p) return Hit{0.0f, HIT_NONE};  // a sphere is selected: Zero
    return Hit{best_p, ~win_p};
}

// DIRECT path, one 8x8 tile: each lane walks its own chain with per-lane (divergent) control
// flow.  Returns the lane's packed counts: reflected segments (bits 0-7) | shadow rays << 8.
template <int K, bool GPOW, bool TILES, typename T>
__device__ __forceinline__ unsigned trace_tile_direct(const LaunchParams& p, int tile_x, int tile_y, float2* stk_lv,
                                                      float* stk_dv, T& tl) {
    const int lane = threadIdx.x & 63;
    const TilePixel tpx = tile_pixel(p, tile_x * TILE_W + (lane & 7), tile_y * TILE_H + (lane >> 3));
    const int x = tpx.x, r = tpx.r, y = tpx.y;
    const bool valid = tpx.valid;
    const unsigned long long pmask = p.prim_const ? prim_box_mask(p, x, y) : 0;

    unsigned cnt = 0;  // packed: reflected segments (bits 0-7) | shadow rays << CNT_SHADOW_SHIFT
    typename StackFor<K>::type stk(stk_lv, stk_dv);
    f3 leaf = mk(0.0f, 0.0f, 0.0f);
    uint32_t px32 = 0;
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

        stk.origin(d);
        Hit h = nearest_direct<true>(p, o, d, tl, pmask);
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
            if (!(flags & MAT_MIRROR)) break;
            o = reflect_at(p, o, d, h.t, h.prim);  // :854, CalculateReflectionRay :718-720
            ++count;
            ++cnt;
            // count is the same for every lane still walking: no divergence here
            h = count > p.limit ? terminal_direct(p, o, d, tl) : nearest_direct<false>(p, o, d, tl);
        }
        // backward fold: every recorded hit is shaded in reverse order; a mirror hit
        // consumes the colour of the segment after it (levels 0..limit push at most one
        // record each, so K = limit + 1 records suffice).  Per lane, divergent: the bundle
        // kernel's converged fold with wave-level shadow culling measured slower here (C2
        // +14 %, C3 +17 %, profiles/ab/r02_direct_converged_fold_rejected.txt)
        f3 col = leaf;
        while (stk.n > 0) {
            float4 ra, rb;
            stk.pop(p, ra, rb);
            const int code = __float_as_int(rb.w);
            const bool is_s = code >= 0;
            col = shade_direct<GPOW>(p, is_s, is_s ? code : ~code, mk(ra.x, ra.y, ra.z),
                                           mk(rb.x, rb.y, rb.z), ra.w, col, &cnt, tl);
        }
        px32 = (shift_channel(col.x) << 16) | (shift_channel(col.y) << 8) | shift_channel(col.z);
        if constexpr (!TILES) store_pixel(p, r, y, x, px32);
    }
    if constexpr (TILES) encode_tile_fused(p, px32, valid);
    return cnt;
}

// DIRECT kernel (scenes with < CULL_MIN_SPHERES spheres).
// STATS: the diagnostic build that also tallies the work actually executed (not timed).
// TILES: out_fmt OUT_TILES (the fused encoder: its own instantiation, so that the others keep their
// register budget -- the epilogue alone raises the direct kernel's SGPR peak from 79 to 83).
// WPG: waves (8x8 tiles of a tile row) per workgroup -- 1 for batch launches; SINGLE_WPG for
// single-frame launches without a copy slice (fewer, larger workgroups: the dispatcher launches
// one-wave groups no faster than ~6.9 us per 1080p frame, a floor a lone frame's launch pays in
// full, tools/launch_probe.hip).  Each wave has its own LDS stack slice.
// TORD (single-frame launches, WPG > 1): 0 = tile rows in row_order / col_major order, 1 = the measured tile
// order (tile_order, a 1-D grid), 2 = as 0 and every wave records its duration (tile_cost).  Instantiations of
// their own: the order read and the recording, compiled into the common kernel even when unused, cost a
// one-frame launch 2 % and 10 % (C2 19.9 -> 20.3 / 22.4 us, profiles/ab/r05_tile_order.txt).
template <int K, bool GPOW, bool STATS, int SMAX, bool TILES, int WPG = 1, int TORD = 0>
__global__ __launch_bounds__(WG_THREADS * WPG) void trace_direct_kernel(LaunchParams p) {
    constexpr int LDS_LEVELS = StackFor<K>::lds_levels;  // LdsStack slots, else unused
    __shared__ float2 stk_lv[LDS_LEVELS > 0 ? LDS_LEVELS * WG_THREADS * WPG : 1];
    __shared__ float stk_dv[LDS_LEVELS > 0 ? 3 * WG_THREADS * WPG : 1];
    if (WPG == 1 && blockIdx.z < (unsigned)p.copy_z) {  // wave-uniform: the fused hand-off's copy slice
        copy_slice(p);
        return;
    }
    Tally<STATS, SMAX> tl;
    const int wave = WPG > 1 && TORD != 0 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))
                     : WPG > 1                ? (int)(threadIdx.x >> 6)
                                              : 0;
    float2* lv = stk_lv + (LDS_LEVELS > 0 ? wave * LDS_LEVELS * WG_THREADS : 0);
    float* dv = stk_dv + (LDS_LEVELS > 0 ? wave * 3 * WG_THREADS : 0);
    // single-frame launches: tile rows in the host's cost order (LaunchParams::row_order), optionally
    // with the rows varying fastest in dispatch order (col_major: grid x = tile rows), or any tile order
    // the host measured (tile_order: a 1-D grid, entry ty << 16 | tx)
    const bool cm = WPG > 1 && p.col_major;
    const int gx = cm ? (int)blockIdx.y : (int)blockIdx.x, gy = cm ? (int)blockIdx.x : (int)blockIdx.y;
    int tile_x = gx * WPG + wave, tile_y = WPG > 1 && gy < p.row_order_n ? (int)p.row_order[gy] : gy;
    if constexpr (TORD == 1) {
        const uint32_t t = p.tile_order[blockIdx.x * WPG + wave];
        tile_x = (int)(t & 0xffffu), tile_y = (int)(t >> 16);  // (0xffff: past the frame, no pixel valid)
    }
    // the host measuring tile costs (order_pick): the wave's cost slot (null when not measuring) and start
    // time wait in LDS -- nothing of it lives in registers across the trace (there it spilled: +9 VGPRs)
    struct TileRec {
        unsigned* slot;
        unsigned t0;
    };
    __shared__ TileRec t_rec[TORD == 2 ? WPG : 1];
    if (TORD == 2 && (threadIdx.x & 63) == 0) {
        const unsigned tiles_x = (unsigned)(p.W + TILE_W - 1) / TILE_W, tiles_y = (unsigned)(p.H + TILE_H - 1) / TILE_H;
        const bool in = p.tile_cost != nullptr && (unsigned)tile_x < tiles_x && (unsigned)tile_y < tiles_y;
        t_rec[wave] = TileRec{in ? p.tile_cost + ((unsigned)tile_y * tiles_x + (unsigned)tile_x) : nullptr,
                              in ? (unsigned)__builtin_amdgcn_s_memrealtime() : 0u};
    }
    const unsigned cnt = trace_tile_direct<K, GPOW, TILES>(p, tile_x, tile_y, lv, dv, tl);
    add_counters<STATS>(p, threadIdx.x & 63, cnt & CNT_REFL_MASK, cnt >> CNT_SHADOW_SHIFT, tl);
    if (TORD == 2 && (threadIdx.x & 63) == 0) {
        const TileRec r = t_rec[threadIdx.x >> 6];
        if (r.slot != nullptr) *r.slot = (unsigned)__builtin_amdgcn_s_memrealtime() - r.t0;
    }
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
// Culling-only arithmetic (never feeds a result): hardware sqrt / rsq (about 1 ulp) instead of
// the correctly rounded sequences; the cull margins (2^-10 relative on R and delta, 2^-8 on
// the tests) are orders of magnitude above that error.
__device__ __forceinline__ float clen3(f3 v) { return __builtin_amdgcn_sqrtf(dot(v, v)); }
__device__ __forceinline__ f3 cnormalize(f3 v) { return scale(v, __builtin_amdgcn_rsqf(dot(v, v))); }
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
    {  // midway between the first and the last active lane's origins (see make_shadow_sphere)
        const f3 a = readlane3(o, ref), b = readlane3(o, 63 - __builtin_clzll(m));
        B.O = scale(add(a, b), 0.5f);
    }
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
    // branch-free (no exec-mask bookkeeping on the scalar unit): every lane loads and tests, lanes
    // >= n are dropped from the ballot; a sphere is culled only when the bundle allows culling,
    // its record is in range and one of the rules holds (NaN anywhere -> candidate)
    const int lane = threadIdx.x & 63;
    const bool in = lane < n;
    const DevSphereCull s = p.scull[base + (in ? lane : 0)];
    const f3 w = sub(mk(s.cx, s.cy, s.cz), B.O);
    const float dc = clen3(w) * (1.0f + 0x1p-20f);
    const float mgn = 0x1p-8f * (dc + B.R);
    const float x = clen3(cross3(w, B.A));
    const bool line = (x - dc * B.delta - B.R) > s.rr + mgn;
    const bool behind = (-dot(w, B.A) - dc * B.delta - B.R * (1.0f + B.delta)) > mgn;
    const bool valid = s.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f;
    const bool cull = B.ok && valid && (line || behind);
    return __builtin_amdgcn_ballot_w64(in && !cull);
}

// Per-lane cluster pre-cull (p.n_clus > 0) for a trace bundle that allows no culling -- the reflected segments
// deep in mirror chains, where a wave's rays fan out into a cone of 0.5 or wider and the bundle would test
// every sphere (tools/trace_cull_model.py: such bundles hold 6.6 of the 7.3 sphere candidates a C4 wave tests
// on its reflected segments, while 1-3 spheres are reachable).  Each lane tests its own ray against the
// clusters' bounding spheres (DevCluster: R >= |c_i - Cc| + r'_i for every member) and the wave takes the
// union of the kept clusters' members.  Converged call (idle lanes carry a copy of an active lane's ray).
// Exactness (culling only, FMA allowed): cull_mask's rules for one ray (R = 0, delta = 0) applied to the
// bounding sphere -- the line misses it by the margin 2^-8 (|w|_1 + R), w = Cc - o, or its centre lies behind
// the origin by R plus that margin.  Then for every member i the line-to-centre distance exceeds
// r'_i + 2^-8 (|c_i - o| + 0) (|c_i - o| <= |w| + R) or its centre is behind by more than the margin: the
// conditions under which cull_mask drops sphere i for this lane, which make its IntersectsSphere distance
// non-selectable.  The perpendicular distance is |w x A| (no cancellation), A = d / |d| by the hardware rsq
// (~1 ulp, far inside the margin); the products are fused (culling-only arithmetic: fewer roundings).  A lane whose a = d.d is outside [0.5, 2] or whose origin is not finite
// keeps every cluster, and a cluster with a NaN R (a member without a usable cull record) is never culled.
__device__ __forceinline__ unsigned long long cluster_mask(const LaunchParams& p, f3 o, f3 d) {
    const float a = dot(d, d);
    const f3 A = cnormalize(d);
    const float ol = __builtin_fabsf(o.x) + __builtin_fabsf(o.y) + __builtin_fabsf(o.z);
    const bool ok = a >= 0.5f && a <= 2.0f && ol < 0x1p40f;
    unsigned long long m = 0;
    for (int j = 0; j < p.n_clus; ++j) {  // wave-uniform
        const DevCluster c = p.clus[j];
        const f3 w = sub(mk(c.cx, c.cy, c.cz), o);
        const float dc = (__builtin_fabsf(w.x) + __builtin_fabsf(w.y) + __builtin_fabsf(w.z)) * (1.0f + 0x1p-20f);
        const float mgn = 0x1p-8f * (dc + c.R);
        const f3 x = mk(__builtin_fmaf(w.y, A.z, -(w.z * A.y)), __builtin_fmaf(w.z, A.x, -(w.x * A.z)),
                        __builtin_fmaf(w.x, A.y, -(w.y * A.x)));  // w x A
        const float T = c.R + mgn;
        const bool line = __builtin_fmaf(x.z, x.z, __builtin_fmaf(x.y, x.y, x.x * x.x)) > T * T;
        const bool behind = -__builtin_fmaf(w.z, A.z, __builtin_fmaf(w.y, A.y, w.x * A.x)) - c.R > mgn;
        const bool valid = dc >= 0x1p-30f && dc < 0x1p40f;
        if (__builtin_amdgcn_ballot_w64(!(ok && valid && (line || behind))) != 0) m |= c.members;  // NaN: kept
    }
    return m;
}

// Shadow bundles.  Every shadow ray of light l has the same direction p_l (the light
// POSITION, Q2), so a sphere can block lane k only if the line {hp_k + s p_l} passes within
// r of its centre: a 2-D test in the light's frame (U, V, A ~ p_l/|p_l|, host-built).  One bound
// serves every light of a shaded level: the ball (O, R) around the first diffuse lane's hit
// point that holds every diffuse lane's hit point, so the hit points spread by at most R across
// and along any light's axis.  Cull rules (same error analysis and 2^-8 margin as cull_mask,
// |C - O| bounded by the L1 norm of the frame coordinates): line miss if |w_perp| - R > r' + mgn;
// behind (b >= 0 for every lane) if -w_A - R > mgn, where w = C - O.  Per light the work is the
// projection of O (uniform) and the cull itself, with the sphere centres already in each light's
// frame (DevShadowCull, host-built in double; the rounding of those projections and of O's is
// covered by the 2^-18 (|C| + |O|) allowance, far above their 2^-22 (|C| + |O|) error).  Against
// a bound per light from its exact perpendicular / axial spreads (three wave reductions per
// light): C4 -2.6 %, C5 -7.5 % (profiles/ab/r02_shadow_sphere.txt).
struct ShadowSphere {
    f3 O;
    float R, omgn;  // radius (rounded up) and 2^-18 |O|
    bool ok;
};

__device__ __forceinline__ ShadowSphere make_shadow_sphere(f3 hp, bool active) {
    ShadowSphere S;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(active);
    S.ok = false;
    S.R = 0.0f;
    S.omgn = 0.0f;
    S.O = hp;
    if (m == 0) return S;
    {
        // centre: midway between the first and the last active lane's hit points (lanes 0 and 63
        // are opposite corners of the 8x8 tile), which roughly halves R against either of them
        // (C4 -4.3 %, C5 -3.8 %, profiles/ab/r02_bundle_centre.txt); R is measured from it
        const f3 a = readlane3(hp, __builtin_ctzll(m)), b = readlane3(hp, 63 - __builtin_clzll(m));
        S.O = scale(add(a, b), 0.5f);
    }
    float e = 0.0f;
    bool bad = false;
    if (active) {
        e = clen3(sub(hp, S.O));
        bad = !(e < 0x1p40f);  // also NaN / inf
    }
    bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    S.R = wave_max(e) * (1.0f + 0x1p-10f) + 0x1p-60f;
    const float olen = clen3(S.O);
    S.omgn = 0x1p-18f * olen * (1.0f + 0x1p-10f);
    S.ok = !bad && S.R < 0x1p38f && olen < 0x1p40f;
    return S;
}

// Candidate mask of spheres [base, base+n) (n <= 64) for the shadow rays of light li from the
// ball S.  Converged call.
__device__ __forceinline__ unsigned long long shadow_sphere_cull(const LaunchParams& p, const ShadowSphere& S,
                                                                 const DevLight& l, int li, int base, int n) {
    const int lane = threadIdx.x & 63;
    const bool in = lane < n;
    const bool ok = S.ok && p.shcull != nullptr && l.a >= 0x1p-40f && l.a <= 0x1p40f && l.a2 < __builtin_inff();
    if (!ok) return __builtin_amdgcn_ballot_w64(in);  // (uniform) no culling: every sphere is a candidate
    // O in the light's frame (uniform); branch-free per lane, as cull_mask
    const float ou = dot(S.O, mk(l.ux, l.uy, l.uz)), ov = dot(S.O, mk(l.vx, l.vy, l.vz));
    const float oa = dot(S.O, mk(l.ax, l.ay, l.az));
    const DevShadowCull c = p.shcull[(size_t)li * (size_t)p.S + (size_t)(base + (in ? lane : 0))];
    const float wu = c.cu - ou, wv = c.cv - ov, wa = c.ca - oa;
    const float dc = __builtin_fabsf(wu) + __builtin_fabsf(wv) + __builtin_fabsf(wa);  // >= |C - O|
    const float mgn = 0x1p-8f * (dc + 3.0f * S.R) + S.omgn;
    const float T = S.R + c.rr + mgn;
    const bool line = wu * wu + wv * wv > T * T;
    const bool behind = -wa - S.R > mgn;
    const bool valid = c.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f;
    return __builtin_amdgcn_ballot_w64(in && !(valid && (line || behind)));  // NaN anywhere -> candidate
}

// Exact tests of the candidate spheres m (bits relative to `base`) of one bundle segment, in
// ascending order (the reference's tie rules), for every lane (idle lanes trace a copy of an active
// lane's ray).  A2OK: 2a finite-positive on every lane.
template <bool PRIMARY, bool A2OK, typename T>
__device__ __forceinline__ void bundle_candidates(const LaunchParams& p, unsigned long long m, int base, f3 o, f3 d,
                                                  float a2, float a4, bool a2_ok, bool active, float& best_s,
                                                  int& win_s, T& tl) {
    auto test = [&](int i) -> float {
        if (PRIMARY && p.prim_const) {
            // o == camera: oc = cam - c and c = oc.oc - r^2 are per-frame constants (:614-619)
            const PrimConst pc = p.pc[i];
            const float b = 2.0f * dot(mk(pc.ocx, pc.ocy, pc.ocz), d);
            const float disc = b * b - a4 * pc.c;
            return A2OK ? root_t1(b, disc, a2) : (a2_ok ? root_t1(b, disc, a2) : root_full(b, disc, a2));
        }
        return sphere_t<A2OK>(o, d, a2, a4, a2_ok, p.sph[i]);
    };
    auto take = [&](float t, int i) {
        if (PRIMARY) take_primary(t, i, best_s, win_s);
        else take_secondary(t, i, best_s, win_s);
    };
    // two candidates per iteration: independent sqrt chains (ILP), selections in ascending order;
    // an odd last candidate alone (C4 -0.9 %, C5 -1.2 %; testing it twice instead: -0.5 / -0.7 %,
    // profiles/ab/r02_near_pairs.txt)
    while (m) {
        const int i0 = base + (int)__builtin_ctzll(m);
        m &= m - 1;
        if (m) {
            const int i1 = base + (int)__builtin_ctzll(m);
            m &= m - 1;
            tl.sphere(active);
            tl.sphere(active);
            const float t0 = test(i0), t1 = test(i1);
            take(t0, i0);
            take(t1, i1);
        } else {
            tl.sphere(active);
            take(test(i0), i0);
        }
    }
}

// BUNDLE path.  Nearest hit of one segment for every active lane (converged call).  PRIMARY: TracePixel's
// rule (:977, :987, :993) with the per-frame camera-relative constants; otherwise
// TraceSecondaryRay's asymmetric rule (:804-806, :819-821, :825).
// `planes`: the segment's nearest plane hit when the caller already has it (terminal segments).
template <bool PRIMARY, typename T>
__device__ __forceinline__ Hit nearest_bundle(const LaunchParams& p, f3 o, f3 d, bool active, T& tl,
                                              unsigned long long pmask = 0, const Hit* planes = nullptr) {
    const unsigned long long am = __builtin_amdgcn_ballot_w64(active);
    if (am == 0) return Hit{0.0f, HIT_NONE};
    // primary segment: the per-frame screen boxes replace the bundle cull
    const bool use_box = PRIMARY && p.prim_const;
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
        // use_box: S <= 64.  A bundle that allows no culling (cone of 0.5 or wider, far or non-finite
        // origins) takes every sphere without the per-lane cull arithmetic, whose ballot would keep every
        // sphere anyway (C4 -0.7 %, C5 -0.6 %, profiles/ab/r04_nocull_ab.txt; culling wider cones than 0.25
        // less eagerly measured +2 %).  Wave-uniform.
        // A cone too wide for the bundle cull: the per-lane cluster pre-cull when the scene has clusters (S <= 64).
        const unsigned long long all = n == 64 ? ~0ull : (1ull << n) - 1ull;
        unsigned long long m = use_box ? pmask : B.ok ? cull_mask(p, B, base, n) : p.n_clus ? cluster_mask(p, o, d) & all : all;
        // candidates in ascending order, selection by selects (take_*, no per-lane branches); the
        // root sequence is chosen once per wave (2a finite-positive on every lane: the usual case)
        if (__builtin_amdgcn_ballot_w64(!a2_ok) == 0)
            bundle_candidates<PRIMARY, true>(p, m, base, o, d, a2, a4, a2_ok, active, best_s, win_s, tl);
        else
            bundle_candidates<PRIMARY, false>(p, m, base, o, d, a2, a4, a2_ok, active, best_s, win_s, tl);
    }
    float best_p = __builtin_inff();
    int win_p = -1;
    if (planes) {
        best_p = planes->t;
        win_p = planes->prim;
    } else {
        for (int i = 0; i < p.P; ++i) {
            tl.plane(active);
            plane_take(o, d, p.pl[i], i, best_p, win_p);  // t > 0 && t < best
        }
    }
    if (!active) return Hit{0.0f, HIT_NONE};
    if (best_s < best_p) return Hit{best_s, win_s};
    if (win_p >= 0) return Hit{best_p, ~win_p};
    return Hit{0.0f, HIT_NONE};
}

// Merged shadow pass of one shaded level (bundle kernel, S <= 64 spheres, L <= SHADOW_MERGE_L
// lights): every light's shadow rays of the wave in ONE wave-uniform loop over the union of the
// lights' candidate sets (they share the level's ShadowSphere bound, and the sets overlap: on C4
// the union holds ~1/3 of the per-light sum, profiles/r03_shadow_slots.txt).  Per candidate sphere
// oc = hp - c and c = oc.oc - r^2 are shared by the lights; b, disc and the root test are per light,
// for the lights whose candidate set holds the sphere and which still have a pending lane (both
// wave-uniform).  Operations and their order are exactly shadow_blocked's (:613-642 with
// IntersectShadowLight's :574-578), so every outcome is the same bit.  Returns the lane's blocked
// bits (bit li).  `want` (bit li): the lane's ray toward light li must be resolved -- a superset of
// the shading's `need` (shade_bundle), so every needed outcome is computed.
// Candidate sets of the lights as one register: lane i holds bit li when sphere i is a candidate
// for light li (lights some lane wants only).  Converged call.  (Hoisting the light-independent
// terms of the cull out of the light loop cut VALU 1.8 % but spilled 12 B/lane: C4 +0.8 %, C5 +0.8 %,
// profiles/ab/r03_shadow_queue_rejected.txt.)
// Candidate sets of the lights from the level's ball bound, with the light-independent terms hoisted
// out of the light loop (the merged instantiation, whose register budget has room for them; against
// one shadow_sphere_cull per light: C4 -2.6 %, profiles/ab/r04_fast_members_ab.txt): lane i loads sphere
// i's centre and r' once, w = C - O, the world-frame L1 bound dc >= |C - O| and the threshold T of
// the line rule once, and per light only projects w onto (U, V, A) -- FMA allowed, culling only --
// and applies the same two rules: line miss if |w_perp|^2 > T^2, behind if w.A < -(R + mgn).  The
// margins are shadow_sphere_cull's: 2^-8 (dc + 3R) with dc from the unprojected w, plus 2^-18
// (|O| + |C|_1) for the rounding of w and of its projections (each < 2^-21 |w|_1, far inside).
__device__ __forceinline__ unsigned shadow_members_fast(const LaunchParams& p, const ShadowSphere& SS, unsigned want) {
    const int lane = threadIdx.x & 63;
    const bool in = lane < p.S;
    const DevSphereCull c = p.scull[in ? lane : 0];
    const f3 w = sub(mk(c.cx, c.cy, c.cz), SS.O);
    const float dc = (__builtin_fabsf(w.x) + __builtin_fabsf(w.y) + __builtin_fabsf(w.z)) * (1.0f + 0x1p-20f);
    const float c1 = __builtin_fabsf(c.cx) + __builtin_fabsf(c.cy) + __builtin_fabsf(c.cz);
    const float mgn = __builtin_fmaf(0x1p-8f, dc + 3.0f * SS.R, SS.omgn + 0x1p-18f * c1);
    const float T = SS.R + c.rr + mgn;
    const float T2 = T * T, nb = -(SS.R + mgn);
    // NaN anywhere -> candidate; a ball that allows no culling keeps every sphere
    const bool valid = SS.ok && p.shcull != nullptr && c.rr >= 0x1p-50f && dc >= 0x1p-30f && dc < 0x1p40f &&
                       c1 < 0x1p40f;
    unsigned memb = 0;
    for (int li = 0; li < p.L; ++li) {
        if (__builtin_amdgcn_ballot_w64((want >> li) & 1u) == 0) continue;  // wave-uniform
        const DevLight& l = p.li[li];
        const bool l_ok = l.a >= 0x1p-40f && l.a <= 0x1p40f && l.a2 < __builtin_inff();  // wave-uniform
        const float wu = __builtin_fmaf(w.z, l.uz, __builtin_fmaf(w.y, l.uy, w.x * l.ux));
        const float wv = __builtin_fmaf(w.z, l.vz, __builtin_fmaf(w.y, l.vy, w.x * l.vx));
        const float wa = __builtin_fmaf(w.z, l.az, __builtin_fmaf(w.y, l.ay, w.x * l.ax));
        const bool line = __builtin_fmaf(wu, wu, wv * wv) > T2;
        const bool behind = wa < nb;
        const bool cull = valid & l_ok & (line | behind);
        memb |= (in & !cull) ? (1u << li) : 0u;
    }
    return memb;
}
// OR of a 32-bit value over the wave (all 64 lanes active): DPP row rotations give each 16-lane row
// its OR, four readlanes finish it.
__device__ __forceinline__ unsigned wave_or(unsigned v) {
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xf, 0xf, false);  // row_ror:1
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xf, 0xf, false);  // row_ror:2
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
    v |= (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
    return (unsigned)__builtin_amdgcn_readlane((int)v, 0) | (unsigned)__builtin_amdgcn_readlane((int)v, 16) |
           (unsigned)__builtin_amdgcn_readlane((int)v, 32) | (unsigned)__builtin_amdgcn_readlane((int)v, 48);
}

// The fold level from which the shadow grids serve (below it the ball bound; at it, per wave, whichever
// fits: shade_bundle).  Level 2 measured C4 +0.6 %, C5 -1.3 % (profiles/ab/r04_w2all_and_grid_level2.txt).
constexpr int GRID_FROM_LEVEL = 1;
// Candidate sets of the lights from the per-light shadow grids (p.shg != nullptr; rt_internal.h
// DevShadowGrid, host tables and the exactness argument in rt_api.cpp build_shadow_grid): each
// lane wanting light li looks up the grid cell of its own hit point's (u, v) and the axial slab of
// its a, ANDs the two masks, and the wave ORs them -- the union of per-lane sets instead of one bound
// around every lane's hit point, which grows with their spread (deep fold levels, where the hit
// points of a wave scatter over the scene; tools/shadow_cull_model.py: C4 sphere-light pairs per
// wave 27.4 -> 7.2).  Culling-only arithmetic (FMA allowed; the margins cover the projections'
// rounding).  Same result layout as shadow_members.  Converged call.
__device__ __forceinline__ unsigned shadow_members_grid(const LaunchParams& p, f3 hp, unsigned want) {
    const int lane = threadIdx.x & 63;
    const float l1 = __builtin_fabsf(hp.x) + __builtin_fabsf(hp.y) + __builtin_fabsf(hp.z);
    unsigned memb = 0;
    for (int li = 0; li < p.L; ++li) {
        const bool w = (want >> li) & 1u;
        if (__builtin_amdgcn_ballot_w64(w) == 0) continue;  // wave-uniform
        const DevShadowGrid& g = p.shg[li];
        const DevLight& l = p.li[li];
        const float u = __builtin_fmaf(hp.z, l.uz, __builtin_fmaf(hp.y, l.uy, hp.x * l.ux));
        const float v = __builtin_fmaf(hp.z, l.vz, __builtin_fmaf(hp.y, l.vy, hp.x * l.vx));
        const float a = __builtin_fmaf(hp.z, l.az, __builtin_fmaf(hp.y, l.ay, hp.x * l.ax));
        const bool near = l1 <= g.bound;  // NaN: far
        // grid cell (near lanes): outside the grid no disc reaches the lane.  Branch-free (bitwise
        // ands / ors): both table loads are issued unconditionally, at clamped in-range indices
        const float xu = __builtin_fmaf(u, g.su, g.ou), xv = __builtin_fmaf(v, g.sv, g.ov);
        const bool in_grid = (xu >= 0.0f) & (xu < (float)SHGRID_N) & (xv >= 0.0f) & (xv < (float)SHGRID_N);
        const unsigned iu = (unsigned)__builtin_fminf(__builtin_fmaxf(xu, 0.0f), (float)(SHGRID_N - 1));
        const unsigned iv = (unsigned)__builtin_fminf(__builtin_fmaxf(xv, 0.0f), (float)(SHGRID_N - 1));
        const unsigned long long cell = p.shgrid[(unsigned)li * (SHGRID_N * SHGRID_N) + iv * SHGRID_N + iu];
        // slab of a (far lanes: lowered by their extra margin); NaN and below the range: entry 0 (all)
        const float mg = g.far_k * l1;
        const float af = near ? a : a - (mg - g.far_b);
        const float xa = __builtin_fminf(__builtin_fmaxf(__builtin_floorf(__builtin_fmaf(af, g.sa, g.oa)), -1.0f),
                                         (float)SHGRID_SLABS);
        const unsigned long long slab = p.shslab[(unsigned)li * (SHGRID_SLABS + 2) + (unsigned)((int)xa + 1)];
        // far lanes: the box of every disc grown by the lane's own margin (NaN: inside)
        const bool out_box = (u < g.bu0 - mg) | (u > g.bu1 + mg) | (v < g.bv0 - mg) | (v > g.bv1 + mg);
        const bool take = w & (near ? in_grid : !out_box);
        const unsigned long long m = take ? (near ? cell : ~0ull) & slab : 0ull;
        const unsigned long long cm = ((unsigned long long)wave_or((unsigned)(m >> 32)) << 32) |
                                      (unsigned long long)wave_or((unsigned)m) | g.always;
        memb |= ((cm >> lane) & 1ull) ? (1u << li) : 0u;
    }
    return memb;
}

// A2OK: every light of the scene has 2a = 2 p.p finite and > 0 (LaunchParams::lights_a2_ok, host-checked; the
// kernel instantiation MERGED == 2): no per-light uniform check and no literal-formula fallback in the loop
// (C4 -0.4 %, C5 -0.4 %, profiles/ab/r05_merged_loop_ab.txt).
template <bool A2OK, typename T>
__device__ __forceinline__ unsigned shadow_merged(const LaunchParams& p, unsigned memb, f3 hp, unsigned want, bool diff,
                                                  bool act, T& tl) {
    unsigned long long U = __builtin_amdgcn_ballot_w64(memb != 0u);
    unsigned blk = 0;
    while (U) {
        const int i = (int)__builtin_ctzll(U);
        U &= U - 1;
        const unsigned mi = (unsigned)__builtin_amdgcn_readlane((int)memb, i);  // lights with sphere i
        const DevSphere sp = p.sph[i];
        const f3 oc = sub(hp, mk(sp.cx, sp.cy, sp.cz));  // shared by the lights (shadow_blocked's oc, c)
        const float c = dot(oc, oc) - sp.r2;
#pragma unroll
        for (int li = 0; li < SHADOW_MERGE_L; ++li) {
            if (((mi >> li) & 1u) == 0) continue;  // wave-uniform (li < p.L)
            const bool pending = ((want & ~blk) >> li) & 1u;
            if (__builtin_amdgcn_ballot_w64(pending) == 0) continue;  // wave-uniform
            tl.shadow_cat(pending ? 0 : (((want >> li) & 1u) ? 1 : (diff ? 2 : (act ? 3 : 4))), 1u);
            tl.shadow_sphere(pending);
            const DevLight& l = p.li[li];
            const float b = 2.0f * dot(oc, mk(l.px, l.py, l.pz));
            const float disc = b * b - l.a4 * c;
            bool hit = false;
            if (A2OK || (l.a2 > 0.0f && l.a2 < __builtin_inff())) {  // wave-uniform (shadow_blocked<.., THRESH>)
                if (__builtin_amdgcn_ballot_w64(sphere_candidate(b, disc)) != 0) {
                    const float sq = cr_sqrt(disc);
                    hit = -b - sq >= l.sh_t;
                }
            } else if (disc >= 0.0f) {
                const float sq = __builtin_sqrtf(disc);
                const float t2 = (-b + sq) / l.a2;
                const float t1 = (-b - sq) / l.a2;
                hit = nmin(nmax0(t1 - 0.001f), nmax0(t2 - 0.001f)) > 0.0f;
            }
            blk |= (pending && hit) ? (1u << li) : 0u;
        }
        if (__builtin_amdgcn_ballot_w64((want & ~blk) != 0u) == 0) break;  // every wanted ray resolved
    }
    return blk;
}

// Shading of one shaded hit per active lane (TraceSphere :847-873 / TracePlane :736-778),
// converged call: the colour is accumulated in the reference's order -- mirror term (from
// the deeper segment `sec`), then each light in order, then ambient.  Inactive lanes
// return `sec` unchanged.  Shadow rays (IntersectShadowLight :573-582) of the lanes that
// need them form one bundle per light (common direction = the light position).
template <bool GPOW, int MERGED, typename T>
__device__ __forceinline__ f3 shade_bundle(const LaunchParams& p, bool act, bool is_sphere, int prim, f3 hp, f3 d, float t,
                                           f3 sec, unsigned* n_shadow, T& tl, int level) {
    // idle lanes (act false) carry a copy of an active lane's record: same branches, result dropped
    const DevMaterial& m = p.mat[is_sphere ? prim : p.S + prim];
    const uint32_t flags = m.flags;
    const bool diff = act && (flags & MAT_DIFFUSE) != 0;
    // S <= 64 and L <= SHADOW_MERGE_L: every light's shadow rays of the level in one merged pass,
    // first -- before the shading's own state is live.  Every diffuse lane's ray toward every light
    // is resolved (a superset of the shading's `need`); a cheap back-facing filter that skipped
    // some of them measured slower (C4 420 vs 401 us: its arithmetic on every lane of every level
    // cost more than the tests it saved, profiles/ab/r03_shadow_merged.txt).
    // MERGED (an instantiation of its own, so that neither path's code and registers burden the
    // other: S <= 64, 1 <= L <= SHADOW_MERGE_L, chosen on the host)
    const bool merged = MERGED != 0 && __builtin_amdgcn_ballot_w64(diff) != 0;
    unsigned blk = 0u;
    if (merged)
        for (int li = 0; li < p.L; ++li) tl.shadow(diff);  // (diagnostic tally of the rays resolved)
    if (merged) {
        const unsigned want = diff ? (1u << p.L) - 1u : 0u;
        // per-lane grid lookups below the first fold level, where a wave's hit points scatter; at
        // level 0 (the tile's primary hits, coherent) one bound around them culls tighter than the
        // grid's cells; at the first fold level whichever fits the wave: the ball while the hit points
        // lie within one grid cell of their centre (light 0's cell size), the grid otherwise (C4 -1.3 %,
        // C5 -1.6 % against the grid there, profiles/ab/r04_adaptive_level1.txt).  Wave-uniform choices.
        unsigned memb;
        if (p.shg && level > GRID_FROM_LEVEL) {
            memb = shadow_members_grid(p, hp, want);
        } else if (p.shg && level == GRID_FROM_LEVEL) {
            const ShadowSphere SS = make_shadow_sphere(hp, diff);
            const float cell = 1.0f / __builtin_fmaxf(p.shg[0].su, p.shg[0].sv);
            memb = SS.ok && SS.R < cell ? shadow_members_fast(p, SS, want) : shadow_members_grid(p, hp, want);
        } else {
            memb = shadow_members_fast(p, make_shadow_sphere(hp, diff), want);
        }
        blk = shadow_merged<MERGED == 2>(p, memb, hp, want, diff, act, tl);
    }
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
    if (__builtin_amdgcn_ballot_w64(diff) != 0) {
        const f3 view = normalize(d);  // ShapePhongShading :668 (not negated)
        // sphere: (1 / t) * t (:866);  plane: (float)(1 / Math.Pow(t, 2)) (:754), exact as 1/(t*t) in f64
        const float att = is_sphere ? cr_rcp(t) * t : (float)(1.0 / ((double)t * (double)t));
        const f3 kd = mk(m.kd[0], m.kd[1], m.kd[2]);
        ShadowSphere SS{};
        if (MERGED == 0) SS = make_shadow_sphere(hp, diff);  // one bound for every light's shadow rays
        unsigned long long umask = 0;  // (diagnostic builds: the union of the lights' candidates)
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
            bool blocked = merged ? ((blk >> li) & 1u) != 0 : !need;
            if (MERGED == 0 && __builtin_amdgcn_ballot_w64(need) != 0) {  // some lane's pixel depends on this test
                // (MERGED without a diffuse lane: no lane needs a test)
                tl.shadow(need);
                const f3 hs = need ? hp : SS.O;  // idle lanes mirror a shading lane (results ignored)
                for (int base = 0; base < p.S; base += 64) {
                    const int n = min(64, p.S - base);
                    unsigned long long mk64 = shadow_sphere_cull(p, SS, l, li, base, n);
                    tl.shadow_masks(5, mk64);
                    umask |= mk64;
                    // candidates two at a time: independent tests (ILP across the sqrt chains),
                    // one pair of sphere loads and one exit ballot per pair; an odd last
                    // candidate is tested twice (the OR is unchanged)
                    while (mk64) {
                        const int i0 = base + (int)__builtin_ctzll(mk64);
                        mk64 &= mk64 - 1;
                        const bool two = mk64 != 0;
                        const int i1 = two ? base + (int)__builtin_ctzll(mk64) : i0;
                        if (two) mk64 &= mk64 - 1;
                        const DevSphere s0 = p.sph[i0], s1 = p.sph[i1];
                        tl.shadow_cat(need ? (blocked ? 1 : 0) : (diff ? 2 : (act ? 3 : 4)), 2u);
                        tl.shadow_sphere(!blocked);
                        const bool h0 = shadow_blocked<false, true>(hs, l, l_ok, s0);
                        tl.shadow_sphere(two && !blocked && !h0);
                        const bool h1 = shadow_blocked<false, true>(hs, l, l_ok, s1);
                        blocked = blocked | h0 | h1;  // no short-circuit branch
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
        if (diff) *n_shadow += (unsigned)p.L << CNT_SHADOW_SHIFT;
        tl.shadow_masks(6, umask);
    }
    col = add(col, mk(m.amb[0], m.amb[1], m.amb[2]));
    return act ? col : sec;
}

// Backward fold (converged call, all 64 lanes): level by level from the deepest, every recorded
// hit is shaded; a mirror hit consumes the colour of the segment after it (levels 0..limit push
// at most one record each, so K = limit + 1 records suffice).  Returns the lane's colour.
template <bool GPOW, int MERGED, typename STK, typename T>
__device__ __forceinline__ f3 fold_converged(const LaunchParams& p, STK& stk, f3 leaf, unsigned* cnt, T& tl) {
    f3 col = leaf;
    const int depth = stk.n;
    int level = (int)wave_max((float)depth);
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
        tl.set_level(level);
        col = shade_bundle<GPOW, MERGED>(p, act, is_s, is_s ? code : ~code, mk(ra.x, ra.y, ra.z), mk(rb.x, rb.y, rb.z),
                                         ra.w, col, cnt, tl, level);
    }
    return col;
}

// BUNDLE kernel (scenes with >= CULL_MIN_SPHERES spheres): converged control flow so that
// every segment and every light can form a wave bundle and cull the sphere list.
template <int K, bool GPOW, bool TILES, int MERGED, typename T>
__device__ __forceinline__ unsigned trace_tile_bundle(const LaunchParams& p, int tile_x, int tile_y, float2* stk_lv,
                                                      float* stk_dv, T& tl) {
    const int lane = threadIdx.x & 63;
    const TilePixel tpx = tile_pixel(p, tile_x * TILE_W + (lane & 7), tile_y * TILE_H + (lane >> 3));
    const int x = tpx.x, y = tpx.y;
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
    typename StackFor<K>::type stk(stk_lv, stk_dv);
    stk.origin(d);
    f3 leaf = mk(0.0f, 0.0f, 0.0f);
    bool active = valid;
    const unsigned long long pmask = p.prim_const ? prim_box_mask(p, x, y) : 0;
    Hit h = nearest_bundle<true>(p, o, d, active, tl, pmask);
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
                if (!(flags & MAT_MIRROR)) {
                    active = false;
                } else {
                    o = reflect_at(p, o, d, h.t, h.prim);  // :854, CalculateReflectionRay :718-720
                    ++cnt;
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(active) == 0) break;
        if (count + 1 > p.limit) {
            // terminal segment (see terminal_direct): only lanes whose nearest plane lies beyond
            // 0.01 need the spheres; the others are Zero
            float best_p = __builtin_inff();
            int win_p = -1;
            for (int i = 0; i < p.P; ++i) {
                tl.plane(active);
                plane_take(o, d, p.pl[i], i, best_p, win_p);  // t > 0 && t < best
            }
            const bool need = active && win_p >= 0 && best_p - 0.01f > 0.0f;
            h = Hit{0.0f, HIT_NONE};
            if (__builtin_amdgcn_ballot_w64(need) != 0) {
                const Hit pl{best_p, win_p};  // (idle lanes: replaced by a copy of an active lane's ray)
                const Hit hn = nearest_bundle<false>(p, o, d, need, tl, 0, &pl);
                if (need) h = hn;
            }
        } else {
            h = nearest_bundle<false>(p, o, d, active, tl);
        }
    }

    const f3 col = fold_converged<GPOW, MERGED>(p, stk, leaf, &cnt, tl);
    const uint32_t px32 = (shift_channel(col.x) << 16) | (shift_channel(col.y) << 8) | shift_channel(col.z);
    if constexpr (TILES) encode_tile_fused(p, px32, valid);
    else {
        // the pixel's coordinates again, from the lane id (mbcnt) and the block id: cheaper than
        // keeping x, r, y and `valid` live through the walk and the fold (64-VGPR cap: they were
        // the values spilled to scratch once the merged shadow pass raised the peak)
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const TilePixel q = tile_pixel(p, tile_x * TILE_W + (ln & 7), tile_y * TILE_H + (ln >> 3));
        if (q.valid) store_pixel(p, q.r, q.y, q.x, px32);
    }
    return cnt;
}

// Occupancy: a wave's SGPRs count against a per-SIMD file of ~800 (waves per SIMD <=
// 800 / (ceil(sgpr / 16) * 16 + 16), MI355X_MICROARCH.md 'Residency'): the compiler's 93-106
// SGPRs admitted 6-7 waves per SIMD whatever its report said.  Capped at 80 (a few uniform values
// spilled to VGPR lanes) and 64 VGPRs (8 waves): C4 -2.6 %, C5 -7.5 %.  Not with GPOW (the f64
// Math.Pow path would spill ~150 B/lane to scratch).  The direct kernel needs no cap (79 SGPRs, 48
// VGPRs).
// TORD: the single-frame launches' tile order as in the direct kernel (0 = natural, 1 = tile_order over the
// 2-D grid, 2 = natural and every wave records its duration in tile_cost)
template <int K, bool GPOW, bool STATS, bool TILES, int MERGED, int TORD = 0>
__device__ __forceinline__ void bundle_kernel_body(const LaunchParams& p) {
    constexpr int LDS_LEVELS = StackFor<K>::lds_levels;  // LdsStack slots, else unused
    __shared__ float2 stk_lv[LDS_LEVELS > 0 ? LDS_LEVELS * WG_THREADS : 1];
    __shared__ float stk_dv[LDS_LEVELS > 0 ? 3 * WG_THREADS : 1];
    if (blockIdx.z < (unsigned)p.copy_z) {  // wave-uniform: the fused hand-off's copy slice
        copy_slice(p);
        return;
    }
    Tally<STATS> tl;
    tl.init(p);
    int tile_x = (int)blockIdx.x, tile_y = (int)blockIdx.y;
    if constexpr (TORD == 1) {
        const uint32_t t = p.tile_order[blockIdx.y * gridDim.x + blockIdx.x];
        tile_x = (int)(t & 0xffffu), tile_y = (int)(t >> 16);  // (0xffff: past the frame, no pixel valid)
    }
    struct TileRec {
        unsigned* slot;
        unsigned t0;
    };
    __shared__ TileRec t_rec[1];
    if (TORD == 2 && (threadIdx.x & 63) == 0)  // (a batch launch's frame 0 records; the others store nothing)
        t_rec[0] = TileRec{blockIdx.z == (unsigned)p.copy_z ? p.tile_cost + (blockIdx.y * gridDim.x + blockIdx.x) : nullptr,
                           (unsigned)__builtin_amdgcn_s_memrealtime()};
    const unsigned cnt = trace_tile_bundle<K, GPOW, TILES, MERGED>(p, tile_x, tile_y, stk_lv, stk_dv, tl);
    add_counters<STATS>(p, threadIdx.x & 63, cnt & CNT_REFL_MASK, cnt >> CNT_SHADOW_SHIFT, tl);
    if (TORD == 2 && (threadIdx.x & 63) == 0 && t_rec[0].slot != nullptr)
        *t_rec[0].slot = (unsigned)__builtin_amdgcn_s_memrealtime() - t_rec[0].t0;
}
template <int K, bool STATS, bool TILES, int MERGED, int TORD = 0>
__global__ __launch_bounds__(WG_THREADS, 8) __attribute__((amdgpu_num_sgpr(80))) void trace_bundle_kernel(
    LaunchParams p) {
    bundle_kernel_body<K, false, STATS, TILES, MERGED, TORD>(p);
}
template <int K, bool STATS, bool TILES, int MERGED>
__global__ __launch_bounds__(WG_THREADS) void trace_bundle_kernel_gpow(LaunchParams p) {
    bundle_kernel_body<K, true, STATS, TILES, MERGED>(p);
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
    Tally<false> tl;
    Hit h = nearest_direct<true>(p, o, d, tl, p.S >= 64 ? ~0ull : (1ull << p.S) - 1);  // every sphere
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
                    if (shadow_blocked<false>(hp, l, l_ok, p.sph[i])) {
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
        h = nearest_direct<false>(p, o, d, tl);
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

// Instantiation per recursion depth: K = limit + 1 records (levels 0..limit each push at most
// one), rounded up to the LDS stack sizes; deeper limits use the scratch stack.
template <template <int> class KERNEL>
static void launch_by_depth(const LaunchParams& p, dim3 grid, dim3 block, hipStream_t s) {
    const int need = p.limit + 1;
    if (need <= 1) hipLaunchKernelGGL(KERNEL<1>::fn, grid, block, 0, s, p);
    else if (need <= 2) hipLaunchKernelGGL(KERNEL<2>::fn, grid, block, 0, s, p);
    else if (need <= 4) hipLaunchKernelGGL(KERNEL<4>::fn, grid, block, 0, s, p);
    else if (need <= 6) hipLaunchKernelGGL(KERNEL<6>::fn, grid, block, 0, s, p);
    else if (need <= 8) hipLaunchKernelGGL(KERNEL<8>::fn, grid, block, 0, s, p);
    else hipLaunchKernelGGL(KERNEL<64>::fn, grid, block, 0, s, p);
}
template <bool GPOW, bool STATS, int SMAX, bool TILES, int WPG = 1, int TORD = 0>
struct DirectK {
    template <int K>
    struct at {
        static constexpr auto fn = trace_direct_kernel<K, GPOW, STATS, SMAX, TILES, WPG, TORD>;
    };
};
template <bool GPOW, bool STATS, bool TILES, int MERGED>
struct BundleK {
    template <int K>
    struct at {
        static constexpr auto fn = GPOW ? trace_bundle_kernel_gpow<K, STATS, TILES, MERGED> : trace_bundle_kernel<K, STATS, TILES, MERGED>;
    };
};
// the all-lights-ok merged instantiation's single-frame tile orders (TORD 1 / 2; no GPOW, no diagnostics)
template <int TORD>
struct BundleOrdK {
    template <int K>
    struct at {
        static constexpr auto fn = trace_bundle_kernel<K, false, false, 2, TORD>;
    };
};

// Scenes with at most DIRECT_SMAX spheres (every BASELINE config of the direct kernel) run a
// direct kernel whose sphere-pair loops are unrolled.
constexpr int DIRECT_SMAX = 8;

template <bool GPOW, bool STATS, bool TILES = false>
static void launch_variant(const LaunchParams& p, bool bundle, dim3 grid, dim3 block, hipStream_t s) {
    if (bundle) {
        // the merged shadow pass's instantiation for S <= 64 spheres and 1..SHADOW_MERGE_L lights
        if (p.S <= 64 && p.L >= 1 && p.L <= SHADOW_MERGE_L && p.lights_a2_ok) {
            if (!GPOW && !STATS && !TILES && p.tile_cost != nullptr)
                launch_by_depth<BundleOrdK<2>::template at>(p, grid, block, s);
            else if (!GPOW && !STATS && !TILES && p.tile_order != nullptr)
                launch_by_depth<BundleOrdK<1>::template at>(p, grid, block, s);
            else launch_by_depth<BundleK<GPOW, STATS, TILES, 2>::template at>(p, grid, block, s);
        }
        else if (p.S <= 64 && p.L >= 1 && p.L <= SHADOW_MERGE_L)
            launch_by_depth<BundleK<GPOW, STATS, TILES, 1>::template at>(p, grid, block, s);
        else
            launch_by_depth<BundleK<GPOW, STATS, TILES, 0>::template at>(p, grid, block, s);
    }
    else if (SINGLE_WPG > 1 && !STATS && !TILES && p.n_frames <= 1 && p.copy_z == 0) {
        // a lone frame: SINGLE_WPG tiles of a tile row per workgroup
        const unsigned gxw = (grid.x + SINGLE_WPG - 1) / SINGLE_WPG;
        const unsigned g1 = (grid.x * grid.y + SINGLE_WPG - 1) / SINGLE_WPG;  // tile_order: a 1-D grid
        const dim3 g(p.tile_order ? g1 : p.col_major ? grid.y : gxw, p.tile_order ? 1u : p.col_major ? gxw : grid.y, grid.z),
            b(WG_THREADS * SINGLE_WPG);
        if (p.tile_cost != nullptr) {  // the host recording tile durations (natural / row / column order)
            if (p.S <= DIRECT_SMAX)
                launch_by_depth<DirectK<GPOW, false, DIRECT_SMAX, false, SINGLE_WPG, 2>::template at>(p, g, b, s);
            else launch_by_depth<DirectK<GPOW, false, 0, false, SINGLE_WPG, 2>::template at>(p, g, b, s);
        } else if (p.tile_order != nullptr) {
            if (p.S <= DIRECT_SMAX)
                launch_by_depth<DirectK<GPOW, false, DIRECT_SMAX, false, SINGLE_WPG, 1>::template at>(p, g, b, s);
            else launch_by_depth<DirectK<GPOW, false, 0, false, SINGLE_WPG, 1>::template at>(p, g, b, s);
        } else if (p.S <= DIRECT_SMAX)
            launch_by_depth<DirectK<GPOW, false, DIRECT_SMAX, false, SINGLE_WPG>::template at>(p, g, b, s);
        else launch_by_depth<DirectK<GPOW, false, 0, false, SINGLE_WPG>::template at>(p, g, b, s);
    } else if (p.S <= DIRECT_SMAX)
        launch_by_depth<DirectK<GPOW, STATS, DIRECT_SMAX, TILES>::template at>(p, grid, block, s);
    else launch_by_depth<DirectK<GPOW, STATS, 0, TILES>::template at>(p, grid, block, s);
}

int launch_trace(const LaunchParams& p, bool generic_pow, bool stats, void* stream) {
    if (p.local_rows <= 0 || p.W <= 0) return (int)hipSuccess;
    const dim3 grid((unsigned)((p.W + TILE_W - 1) / TILE_W), (unsigned)((p.local_rows + TILE_H - 1) / TILE_H),
                    (unsigned)(p.n_frames > 1 ? p.n_frames : 1) + (unsigned)p.copy_z);
    const dim3 block(WG_THREADS);
    hipStream_t s = (hipStream_t)stream;
    // bundle culling pays for its per-wave bounds only with enough spheres (A/B: +15 % at
    // 8 spheres, 3x faster at 64)
    const bool bundle = p.S >= CULL_MIN_SPHERES;
    if (p.out_fmt == OUT_TILES) {  // the fused encoder (never with the diagnostic tallies)
        if (generic_pow) launch_variant<true, false, true>(p, bundle, grid, block, s);
        else launch_variant<false, false, true>(p, bundle, grid, block, s);
    } else if (stats) {
        if (generic_pow) launch_variant<true, true>(p, bundle, grid, block, s);
        else launch_variant<false, true>(p, bundle, grid, block, s);
    } else {
        if (generic_pow) launch_variant<true, false>(p, bundle, grid, block, s);
        else launch_variant<false, false>(p, bundle, grid, block, s);
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

int launch_band_copy(const CopyJob& job, void* stream) {
    if (job.words == 0) return (int)hipSuccess;
    const unsigned long long chunks = (job.words + 3) / 4;
    const unsigned wg = (unsigned)min((unsigned long long)COPY_WAVES, (chunks + 63) / 64);
    hipLaunchKernelGGL(band_copy_kernel, dim3(wg), dim3(64), 0, (hipStream_t)stream, job);
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
