// fastmath_check.hip -- GPU proof of rt_fastmath.h (run on an MI355X; not part of the library).
//
// For every binary32 input x (all 2^32 bit patterns):
//   * rcp / sqrt: the fast sequence is checked against the DEFINITION of correct rounding,
//     independently of any compiler sequence: y = RN(1/x) iff x*mid_lo < 1 < x*mid_hi and
//     s = RN(sqrt x) iff mid_lo^2 < x < mid_hi^2, where mid_lo / mid_hi are the midpoints
//     between the result and its float neighbours (exact in binary64: 24 x 25 bits), and
//     exact ties cannot occur for either function;
//   * the guarded wrappers rcp_cr / sqrt_cr / inv_len_cr are compared bit for bit with the
//     generic correctly rounded '1.0f / x', sqrtf(x), 1.0f / sqrtf(x) (NaN == NaN).
// Division: every divisor mantissa (2^23) against 64 dividend mantissas (edge patterns and
// pseudo-random), at several exponent pairs spanning the domain, plus special values; the
// fast sequence is checked against the midpoint definition (b*mid_lo < a < b*mid_hi; the
// quotient of two floats is never a midpoint), the wrapper bitwise against 'a / b'.
// Mismatch counts are reported per input exponent (inside / outside the wrappers' domains).
//
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
//         -fno-gpu-flush-denormals-to-zero -o tools/fastmath_check tools/fastmath_check.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../uu-infogr-raytracer_amd/csrc/rt_fastmath.h"

using namespace rtk;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(2);                                                                         \
        }                                                                                    \
    } while (0)

// counters[test][exponent 0..255]
enum { T_RCP_FAST, T_SQRT_FAST, T_RCP_WRAP, T_SQRT_WRAP, T_INVLEN_WRAP, T_DIV_FAST, T_DIV_WRAP, NT };

__device__ bool same_bits(float a, float b) {
    return (a != a && b != b) || __float_as_uint(a) == __float_as_uint(b);
}

__device__ void mids(float r, double& lo, double& hi) {
    const uint32_t u = __float_as_uint(r);
    lo = 0.5 * ((double)r + (double)__uint_as_float(u - 1));
    hi = 0.5 * ((double)r + (double)__uint_as_float(u + 1));
}

// positive finite x whose result is a positive normal float with normal neighbours
__device__ bool rcp_ok(float x, float y) {
    double lo, hi;
    mids(y, lo, hi);
    return (double)x * lo < 1.0 && 1.0 < (double)x * hi;
}
__device__ bool sqrt_ok(float x, float s) {
    double lo, hi;
    mids(s, lo, hi);
    return lo * lo < (double)x && (double)x < hi * hi;
}
__device__ bool div_ok(float a, float b, float q) {  // a, b > 0
    double lo, hi;
    mids(q, lo, hi);
    return (double)b * lo < (double)a && (double)a < (double)b * hi;
}

__global__ void unary_kernel(unsigned long long* cnt, uint32_t base) {
    __shared__ unsigned loc[5][256];
    for (int i = threadIdx.x; i < 5 * 256; i += blockDim.x) loc[i / 256][i % 256] = 0;
    __syncthreads();
    for (int k = 0; k < 16; ++k) {
        const uint32_t u = base + ((blockIdx.x * 16u + k) * blockDim.x + threadIdx.x);
        const float x = __uint_as_float(u);
        const int ex = (u >> 23) & 0xff;
        const float ax = __builtin_fabsf(x);
        // independent correctness of the fast sequences, inside their domains
        if (x > 0.0f && fm_in(x, FM_RCP_LO, FM_RCP_HI)) {
            if (!rcp_ok(x, rcp_cr_fast(x))) atomicAdd(&loc[0][ex], 1u);
        }
        if (x > 0.0f && x >= FM_SQRT_LO && x <= FM_SQRT_HI) {
            if (!sqrt_ok(x, sqrt_cr_fast(x))) atomicAdd(&loc[1][ex], 1u);
        }
        (void)ax;
        // wrappers == generic operation, every input
        if (!same_bits(rcp_cr(x), 1.0f / x)) atomicAdd(&loc[2][ex], 1u);
        if (!same_bits(sqrt_cr(x), __builtin_sqrtf(x))) atomicAdd(&loc[3][ex], 1u);
        if (!same_bits(inv_len_cr(x), 1.0f / __builtin_sqrtf(x))) atomicAdd(&loc[4][ex], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 5 * 256; i += blockDim.x)
        if (loc[i / 256][i % 256]) atomicAdd(&cnt[(i / 256) * 256 + i % 256], (unsigned long long)loc[i / 256][i % 256]);
}

__device__ uint32_t mix(uint32_t v) {
    v ^= v >> 16;
    v *= 0x7feb352dU;
    v ^= v >> 15;
    v *= 0x846ca68bU;
    v ^= v >> 16;
    return v;
}

// a mantissa index 0..63 -> mantissa bits
__device__ uint32_t a_mant(int j) {
    switch (j) {
        case 0: return 0;
        case 1: return 1;
        case 2: return 0x7fffff;
        case 3: return 0x7ffffe;
        case 4: return 0x400000;
        case 5: return 0x3fffff;
        case 6: return 0x555555;
        case 7: return 0x2aaaaa;
        default: return mix((uint32_t)j * 2654435761u) & 0x7fffff;
    }
}

// grid: x over divisor mantissas (2^23 / 256 blocks of 256), y over exponent pairs
__global__ void div_kernel(unsigned long long* cnt, const int* ea_list, const int* eb_list) {
    const uint32_t mb = blockIdx.x * blockDim.x + threadIdx.x;
    const int ea = ea_list[blockIdx.y], eb = eb_list[blockIdx.y];
    const float b = __uint_as_float(((uint32_t)(eb + 127) << 23) | mb);
    unsigned bad_fast = 0, bad_wrap = 0;
    for (int j = 0; j < 64; ++j) {
        const float a = __uint_as_float(((uint32_t)(ea + 127) << 23) | a_mant(j));
        const float q = div_cr_fast(a, b);
        if (!div_ok(a, b, q)) ++bad_fast;
        if (!same_bits(div_cr(a, b), a / b)) ++bad_wrap;
        if (!same_bits(div_cr(-a, b), -a / b)) ++bad_wrap;
        if (!same_bits(div_cr(a, -b), a / -b)) ++bad_wrap;
    }
    if (bad_fast) atomicAdd(&cnt[T_DIV_FAST * 256 + (eb + 127)], (unsigned long long)bad_fast);
    if (bad_wrap) atomicAdd(&cnt[T_DIV_WRAP * 256 + (eb + 127)], (unsigned long long)bad_wrap);
}

// wrapper vs generic division over special / out-of-domain operands
__global__ void div_special_kernel(unsigned long long* cnt) {
    const uint32_t ua = blockIdx.x * blockDim.x + threadIdx.x;  // 2^16 patterns for a
    const float specials[] = {0.0f, -0.0f, INFINITY, -INFINITY, NAN, 0x1p-149f, 0x1p-126f, 0x1.fffffep127f,
                              0x1p-61f, 0x1p61f, 0x1p-60f, 0x1p60f, 1.0f, 3.0f, 0.1f, 7.5e-39f};
    const float a = __uint_as_float(mix(ua) ^ (ua << 16));
    unsigned bad = 0;
    for (float b : specials) {
        if (!same_bits(div_cr(a, b), a / b)) ++bad;
        if (!same_bits(div_cr(b, a), b / a)) ++bad;
    }
    if (bad) atomicAdd(&cnt[T_DIV_WRAP * 256 + 255], (unsigned long long)bad);
}

int main() {
    unsigned long long* d_cnt;
    CK(hipMalloc(&d_cnt, sizeof(unsigned long long) * NT * 256));
    CK(hipMemset(d_cnt, 0, sizeof(unsigned long long) * NT * 256));
    // 2^32 inputs: 16 launches of 2^28 (4096 x 16 x 4096... ) -> blocks of 256 threads x 16 values
    const uint32_t per_launch = 1u << 28;
    for (uint64_t base = 0; base < (1ull << 32); base += per_launch) {
        hipLaunchKernelGGL(unary_kernel, dim3(per_launch / (256 * 16)), dim3(256), 0, 0, d_cnt, (uint32_t)base);
        CK(hipGetLastError());
    }
    const int pairs[][2] = {{0, 0}, {0, 1}, {1, 0}, {-60, 0}, {0, -60}, {59, 0}, {0, 59}, {-60, 59}, {59, -60},
                            {-60, -60}, {59, 59}, {13, -7}, {-22, 31}};
    const int np = (int)(sizeof pairs / sizeof pairs[0]);
    int ea[64], eb[64];
    for (int i = 0; i < np; ++i) ea[i] = pairs[i][0], eb[i] = pairs[i][1];
    int *d_ea, *d_eb;
    CK(hipMalloc(&d_ea, sizeof ea));
    CK(hipMalloc(&d_eb, sizeof eb));
    CK(hipMemcpy(d_ea, ea, sizeof ea, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_eb, eb, sizeof eb, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(div_kernel, dim3((1u << 23) / 256, np), dim3(256), 0, 0, d_cnt, d_ea, d_eb);
    CK(hipGetLastError());
    hipLaunchKernelGGL(div_special_kernel, dim3(256), dim3(256), 0, 0, d_cnt);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned long long cnt[NT * 256];
    CK(hipMemcpy(cnt, d_cnt, sizeof cnt, hipMemcpyDeviceToHost));
    const char* names[NT] = {"rcp_cr_fast vs definition (domain)", "sqrt_cr_fast vs definition (domain)",
                             "rcp_cr == 1.0f/x (all inputs)", "sqrt_cr == sqrtf (all inputs)",
                             "inv_len_cr == 1.0f/sqrtf (all inputs)", "div_cr_fast vs definition (domain sets)",
                             "div_cr == a/b (domain sets + specials)"};
    const unsigned long long tested[NT] = {0, 0, 1ull << 32, 1ull << 32, 1ull << 32,
                                           (unsigned long long)np << 29, 3ull * ((unsigned long long)np << 29) + 2ull * 16 * 65536};
    int fails = 0;
    for (int t = 0; t < NT; ++t) {
        unsigned long long tot = 0;
        for (int e = 0; e < 256; ++e) tot += cnt[t * 256 + e];
        printf("%-44s mismatches %llu", names[t], tot);
        if (tested[t]) printf(" of %llu", tested[t]);
        printf("\n");
        if (tot) {
            ++fails;
            for (int e = 0; e < 256; ++e)
                if (cnt[t * 256 + e]) printf("    biased exponent %3d (2^%d): %llu\n", e, e - 127, cnt[t * 256 + e]);
        }
    }
    printf(fails ? "FAIL\n" : "PASS: every fast sequence is correctly rounded in its domain and every wrapper equals the generic operation\n");
    return fails ? 1 : 0;
}
