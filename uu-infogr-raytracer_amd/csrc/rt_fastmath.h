// rt_fastmath.h -- correctly rounded binary32 sqrt, reciprocal and division in fewer
// instructions than the generic sequences, for operands inside a checked domain.
//
// HIP's correctly rounded '/' (-fhip-fp32-correctly-rounded-divide-sqrt) is a scaled
// Newton sequence: v_div_scale x2, v_rcp, 5 FMAs, v_div_fmas, v_div_fixup (11 VALU), and
// sqrt scales denormal inputs, fixes the hardware result up by its neighbours and patches
// +-0 / +inf (15 VALU).  Inside the domains below the scaling and the special-value
// patches are dead code, so the same Newton / neighbour steps run alone:
//   rcp_cr_fast(x)   y = v_rcp(x); e = fma(-x, y, 1); y + e*y           (3 VALU)
//   sqrt_cr_fast(x)  s = v_sqrt(x); pick s-1ulp / s / s+1ulp by the signs of the FMA
//                    residuals x - s'*s  (LLVM's own fix-up without the scaling, 7 VALU)
//   div_cr_fast(a,b) refined reciprocal, q = a*y, two residual corrections (8 VALU)
// Each result is the correctly rounded value -- the same bits as '1.0f / x', sqrtf(x) and
// 'a / b' -- which tools/fastmath_check.hip verifies on the GPU independently of any
// compiler sequence: exhaustively over all 2^32 inputs for rcp and sqrt, and for the
// division over every divisor mantissa against a set of dividends (the result of a
// correctly rounded division is correct iff b*mid_lo < a < b*mid_hi for the midpoints
// around it, evaluated exactly in binary64).  Outside the domains (denormals, huge
// values, zeros, inf, NaN) the guarded wrappers fall back to the generic operation, so
// every input gives the generic result bit for bit.
#pragma once
#include <hip/hip_runtime.h>

namespace rtk {

// Domains (|x| bounds) in which the fast sequences are exact; the checker measures the
// real ones (profiles/fastmath_check.txt) and these sit well inside them.
constexpr float FM_RCP_LO = 0x1p-120f, FM_RCP_HI = 0x1p120f;
constexpr float FM_SQRT_LO = 0x1p-96f, FM_SQRT_HI = 0x1p120f;  // below 2^-96 the residuals lose bits (LLVM scales there too)
constexpr float FM_DIV_LO = 0x1p-60f, FM_DIV_HI = 0x1p60f;

__device__ __forceinline__ float rcp_cr_fast(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}

__device__ __forceinline__ float sqrt_cr_fast(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);
    const float sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    return r;
}

__device__ __forceinline__ float div_cr_fast(float a, float b) {
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

__device__ __forceinline__ bool fm_in(float x, float lo, float hi) {
    const float ax = __builtin_fabsf(x);
    return ax >= lo && ax <= hi;  // false for NaN
}

// Guarded forms: identical bits to the generic operation for every input.
__device__ __forceinline__ float rcp_cr(float x) {
    float r = rcp_cr_fast(x);
    if (__builtin_expect(!fm_in(x, FM_RCP_LO, FM_RCP_HI), 0)) r = 1.0f / x;
    return r;
}

__device__ __forceinline__ float sqrt_cr(float x) {
    float r = sqrt_cr_fast(x);
    if (__builtin_expect(!(x >= FM_SQRT_LO && x <= FM_SQRT_HI), 0)) r = __builtin_sqrtf(x);
    return r;
}

// 1 / sqrt(x) as Vector3.Normalize computes it: two correctly rounded steps.  x in
// [2^-96, 2^120] puts sqrt(x) in [2^-48, 2^60], inside the reciprocal's domain.
__device__ __forceinline__ float inv_len_cr(float x) {
    float r = rcp_cr_fast(sqrt_cr_fast(x));
    if (__builtin_expect(!(x >= FM_SQRT_LO && x <= FM_SQRT_HI), 0)) r = 1.0f / __builtin_sqrtf(x);
    return r;
}

__device__ __forceinline__ float div_cr(float a, float b) {
    float q = div_cr_fast(a, b);
    if (__builtin_expect(!(fm_in(a, FM_DIV_LO, FM_DIV_HI) && fm_in(b, FM_DIV_LO, FM_DIV_HI)), 0)) q = a / b;
    return q;
}

}  // namespace rtk
