// pow_check.hip -- the device's f64 Math.Pow against glibc's (run on an MI355X; not part of the library).
//
// The kernels' ShapePhongShading exponent (RayTracer.cs:691) for n outside {0.5, 1, 2} is
// (float)pow((double)x, (double)n) on the device (ocml), where the reference's Math.Pow is glibc's pow on
// Linux x64; TracePlane's attenuation (RayTracer.cs:754) is (float)(1 / Math.Pow(t, 2)).  Both must give the
// reference's binary32 bits.
//
// 1. Specular exponent: every binary32 x in [0, 1 + 16 ulp] (the clamped dot product of two unit vectors,
//    0x00000000 ... 0x3f800010) for n in {3.7, 7.25, 12} and 64 exponents sampled in (0, 64), for two device
//    functions: the device's own f64 pow (ocml; the kernels' path until round 6) and the library's restatement
//    of glibc's pow (csrc/rt_pow.h, the kernels' path since round 6).  The device evaluates pow in double and
//    rounds to float.  Two doubles within a few ulps of the exact power (ocml's and
//    glibc's pow are both accurate to ~1 ulp of double) round to the same float unless the exact value lies
//    near a rounding boundary of binary32 -- a midpoint between two floats.  So the device flags every x whose
//    double result lies within 2^-40 (relative; ~2^12 ulps of double) of such a midpoint, and the host
//    evaluates glibc's pow for exactly those x and compares the float results bit for bit.  As a check of that
//    argument, 1 x in 1024 (all of them unflagged or not) is also compared directly.
// 2. Plane attenuation: every positive finite binary32 t: the device's (float)(1.0 / ((double)t * (double)t))
//    (the kernels' form) against the host's (float)(1.0 / pow((double)t, 2.0)) with glibc's pow, all 2^31 - 2^23
//    values, in chunks.
// Prints the mismatch counts; exit status 1 on any mismatch of the kernels' functions (the restatement, the
// attenuation form); the ocml counts are reported for the record.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
//         -o tools/pow_check tools/pow_check.hip -lpthread
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../uu-infogr-raytracer_amd/csrc/rt_pow.h"

__device__ const rtk::glibc_pow_data::LogEntry g_log[128] = RT_POW_LOG_TAB;
__device__ const uint64_t g_exp[256] = RT_POW_EXP_TAB;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e_ = (x);                                                                 \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(2);                                                                         \
        }                                                                                    \
    } while (0)

constexpr uint32_t X_END = 0x3f800011u;  // x bits 0 .. 0x3f800010 (+0 up to 1 + 16 ulp)
constexpr unsigned CAP = 1u << 22;       // records per buffer and exponent

struct Rec {
    uint32_t x;
    float f;   // the device's (float)pow (ocml)
    float fr;  // (float)rtk::glibc_pow (the restatement)
    double dr; // rtk::glibc_pow's double
};

__device__ __forceinline__ bool near_mid(double p, float f) {
    // midpoints between f and its neighbours, exact in binary64
    const uint32_t u = __float_as_uint(f);
    const double lo = 0.5 * ((double)f + (double)__uint_as_float(u - 1u));
    const double hi = 0.5 * ((double)f + (double)__uint_as_float(u + 1u));
    const double tol = 0x1p-40 * fabs(p) + 0x1p-1074 * 4096.0;
    return (u != 0u && fabs(p - lo) <= tol) || fabs(p - hi) <= tol;
}

__global__ void pow_kernel(float n, Rec* flagged, unsigned* n_flagged, Rec* sampled, unsigned* n_sampled) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= X_END) return;
    const float x = __uint_as_float(u);
    const double p = pow((double)x, (double)n);  // ocml
    const float f = (float)p;
    const double pr = rtk::glibc_pow((double)x, (double)n, g_log, g_exp);  // the kernels' spec_pow generic path
    const float fr = (float)pr;
    if (near_mid(p, f) || near_mid(pr, fr)) {
        const unsigned i = atomicAdd(n_flagged, 1u);
        if (i < CAP) flagged[i] = Rec{u, f, fr, pr};
    }
    if ((u * 2654435761u) >> 22 == 0u) {  // 1 in 1024
        const unsigned i = atomicAdd(n_sampled, 1u);
        if (i < CAP) sampled[i] = Rec{u, f, fr, pr};
    }
}

__global__ void att_kernel(uint32_t base, uint32_t count, float* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const float t = __uint_as_float(base + i);
    out[i] = (float)(1.0 / ((double)t * (double)t));  // TracePlane's (float)(1 / Math.Pow(t, 2)) in the kernels
}

static bool same_bits(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}

// glibc's pow through a volatile function pointer: never folded or replaced by the compiler
static double (*volatile glibc_pow)(double, double) = pow;

struct Bad {
    unsigned long long ocml = 0, restated = 0, restated_dbl = 0;
};
static Bad check_recs(const std::vector<Rec>& r, unsigned n, float e, const char* what, int* shown) {
    Bad bad;
    for (unsigned i = 0; i < n && i < CAP; ++i) {
        float x;
        std::memcpy(&x, &r[i].x, 4);
        const double gd = glibc_pow((double)x, (double)e);
        const float g = (float)gd;
        if (!same_bits(g, r[i].f)) {
            ++bad.ocml;
            if ((*shown)++ < 20)
                printf("    %s mismatch (ocml): x = %a (0x%08x), n = %a: device %a, glibc %a\n", what, (double)x, r[i].x,
                       (double)e, (double)r[i].f, (double)g);
        }
        if (!same_bits(g, r[i].fr)) {
            ++bad.restated;
            if ((*shown)++ < 20)
                printf("    %s mismatch (restated): x = %a (0x%08x), n = %a: device %a, glibc %a\n", what, (double)x,
                       r[i].x, (double)e, (double)r[i].fr, (double)g);
        }
        uint64_t a, b;
        std::memcpy(&a, &gd, 8);
        std::memcpy(&b, &r[i].dr, 8);
        if (a != b) ++bad.restated_dbl;
    }
    return bad;
}

int main() {
    // exponents: the random scenes' three, then 64 sampled in (0, 64) (SplitMix64, seed 0x5EED)
    std::vector<float> ns = {3.7f, 7.25f, 12.0f};
    uint64_t s = 0x5EED;
    while (ns.size() < 67) {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const float n = (float)((double)(z >> 11) * 0x1p-53 * 64.0);
        if (n > 0.0f && n != 0.5f && n != 1.0f && n != 2.0f) ns.push_back(n);
    }
    Rec *d_flag, *d_samp;
    unsigned* d_cnt;
    CK(hipMalloc(&d_flag, sizeof(Rec) * CAP));
    CK(hipMalloc(&d_samp, sizeof(Rec) * CAP));
    CK(hipMalloc(&d_cnt, 2 * sizeof(unsigned)));
    std::vector<Rec> flag(CAP), samp(CAP);
    unsigned long long tot_flag = 0, tot_samp = 0, overflow = 0;
    Bad bf_all, bs_all;
    int shown = 0;
    for (float n : ns) {
        CK(hipMemset(d_cnt, 0, 2 * sizeof(unsigned)));
        hipLaunchKernelGGL(pow_kernel, dim3((X_END + 255) / 256), dim3(256), 0, 0, n, d_flag, d_cnt, d_samp, d_cnt + 1);
        CK(hipGetLastError());
        unsigned c[2];
        CK(hipMemcpy(c, d_cnt, sizeof c, hipMemcpyDeviceToHost));
        CK(hipMemcpy(flag.data(), d_flag, sizeof(Rec) * std::min(c[0], CAP), hipMemcpyDeviceToHost));
        CK(hipMemcpy(samp.data(), d_samp, sizeof(Rec) * std::min(c[1], CAP), hipMemcpyDeviceToHost));
        if (c[0] > CAP || c[1] > CAP) ++overflow;
        const Bad bf = check_recs(flag, c[0], n, "near-midpoint", &shown);
        const Bad bs = check_recs(samp, c[1], n, "sampled", &shown);
        printf("n = %-12a (%9.6f): %8u near a binary32 midpoint, %8u sampled; float mismatches ocml %llu / %llu, "
               "restated %llu / %llu (double %llu / %llu)\n", (double)n, (double)n, c[0], c[1], bf.ocml, bs.ocml,
               bf.restated, bs.restated, bf.restated_dbl, bs.restated_dbl);
        tot_flag += c[0], tot_samp += c[1];
        bf_all.ocml += bf.ocml, bf_all.restated += bf.restated, bf_all.restated_dbl += bf.restated_dbl;
        bs_all.ocml += bs.ocml, bs_all.restated += bs.restated, bs_all.restated_dbl += bs.restated_dbl;
    }
    printf("spec_pow: %zu exponents x %u inputs x in [0, 1 + 16 ulp]: %llu inputs near a binary32 midpoint (either "
           "function) all compared with glibc, %llu sampled inputs compared%s\n", ns.size(), X_END, tot_flag, tot_samp,
           overflow ? " -- BUFFER OVERFLOW" : "");
    printf("  device ocml pow:            float mismatches %llu near-midpoint, %llu sampled\n", bf_all.ocml, bs_all.ocml);
    printf("  restated glibc pow (rt_pow.h, the kernels'): float mismatches %llu near-midpoint, %llu sampled; "
           "double mismatches %llu / %llu\n", bf_all.restated, bs_all.restated, bf_all.restated_dbl, bs_all.restated_dbl);

    // plane attenuation over every positive finite float
    const uint32_t first = 1u, last = 0x7f7fffffu, chunk = 1u << 26;
    float* d_out;
    CK(hipMalloc(&d_out, sizeof(float) * chunk));
    std::vector<float> out(chunk);
    unsigned long long att_bad = 0, att_n = 0;
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    for (uint64_t base = first; base <= last; base += chunk) {
        const uint32_t cnt = (uint32_t)std::min<uint64_t>(chunk, (uint64_t)last + 1 - base);
        hipLaunchKernelGGL(att_kernel, dim3((cnt + 255) / 256), dim3(256), 0, 0, (uint32_t)base, cnt, d_out);
        CK(hipGetLastError());
        CK(hipMemcpy(out.data(), d_out, sizeof(float) * cnt, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> bad(nt, 0);
        std::vector<std::thread> th;
        for (unsigned k = 0; k < nt; ++k)
            th.emplace_back([&, k]() {
                for (uint32_t i = k; i < cnt; i += nt) {
                    const uint32_t u = (uint32_t)base + i;
                    float t;
                    std::memcpy(&t, &u, 4);
                    const float g = (float)(1.0 / glibc_pow((double)t, 2.0));
                    if (!same_bits(g, out[i])) ++bad[k];
                }
            });
        for (auto& t : th) t.join();
        for (unsigned long long b : bad) att_bad += b;
        att_n += cnt;
    }
    printf("plane attenuation: (float)(1 / ((double)t * t)) on the device vs (float)(1 / glibc pow(t, 2)) for all %llu "
           "positive finite t: mismatches %llu\n", att_n, att_bad);
    const bool ok = !bf_all.restated && !bs_all.restated && !bf_all.restated_dbl && !bs_all.restated_dbl && !att_bad &&
                    !overflow;
    printf(ok ? "PASS\n" : "FAIL\n");
    return ok ? 0 : 1;
}
