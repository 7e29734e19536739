// pow_host.cpp -- TEST INFRASTRUCTURE ONLY: the library's restatement of glibc's pow (csrc/rt_pow.h, the
// kernels' Math.Pow for specular exponents other than 0.5, 1, 2; RayTracer.cs:691) against the host's own glibc
// pow, bit for bit on the double result (so on the binary32 result too).  Built with hipcc as a host program
// (the restatement is __host__ __device__); run by tests/test_pow.py.
//   pow_host [samples]   -> "pow_host: N compared, M double mismatches, F float mismatches"
// Inputs: the kernels' domain -- x a binary32 in [0, 1 + 16 ulp] (uniform over bit patterns and over values),
// y a binary32 exponent in (0, 64) (the random scenes' 3.7, 7.25, 12 and sampled ones); the two inputs where
// the device's ocml pow and glibc round to different floats (profiles/r06_pow_check.txt); and random doubles
// over the whole range (x > 0 of any exponent, subnormals included; y of any sign and magnitude; x < 0 with
// integer y), which exercise log/exp's special cases, overflow and underflow.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../uu-infogr-raytracer_amd/csrc/rt_pow.h"

using rtk::glibc_pow_data::LogEntry;
static const LogEntry h_log[128] = RT_POW_LOG_TAB;
static const uint64_t h_exp[256] = RT_POW_EXP_TAB;
static double (*volatile libm_pow)(double, double) = pow;

static uint64_t bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
static bool same(double a, double b) { return bits(a) == bits(b) || (a != a && b != b); }
static bool samef(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y || (a != a && b != b);
}
static float f32(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

struct Tally {
    long n = 0, dbl = 0, flt = 0;
    int shown = 0;
    void check(double x, double y) {
        const double g = libm_pow(x, y), r = rtk::glibc_pow(x, y, h_log, h_exp);
        ++n;
        if (!same(g, r)) {
            ++dbl;
            if (shown++ < 8) std::printf("  mismatch: pow(%a, %a): glibc %a, restated %a\n", x, y, g, r);
        }
        if (!samef((float)g, (float)r)) ++flt;
    }
};

// The kernels' exact fast paths of Math.Pow (rt_kernel.hip spec_pow: n = 1 -> x, n = 2 -> x * x in binary32,
// n = 0.5 -> binary32 sqrt) against glibc's (float)pow for EVERY binary32 x in [0, 1 + 16 ulp].
static int fast_paths(unsigned nt) {
    std::vector<long> bad(nt, 0);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; ++w)
        th.emplace_back([&, w]() {
            for (uint32_t u = w; u < 0x3f800011u; u += nt) {
                const float x = f32(u);
                if (!samef((float)libm_pow((double)x, 1.0), x)) ++bad[w];
                if (!samef((float)libm_pow((double)x, 2.0), x * x)) ++bad[w];
                if (!samef((float)libm_pow((double)x, 0.5), std::sqrt(x))) ++bad[w];
            }
        });
    for (auto& x : th) x.join();
    long b = 0;
    for (long v : bad) b += v;
    std::printf("pow_host fast paths: every binary32 x in [0, 1 + 16 ulp] (%u) for n = 1, 2, 0.5: %ld mismatches\n",
                0x3f800011u, b);
    return b ? 1 : 0;
}

int main(int argc, char** argv) {
    const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    if (argc > 1 && std::strcmp(argv[1], "fast-paths") == 0) return fast_paths(nt);
    const long samples = argc > 1 ? std::atol(argv[1]) : 4000000;
    std::vector<Tally> t(nt);
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; ++w)
        th.emplace_back([&, w]() {
            Tally& T = t[w];
            uint64_t s = 0x5EEDull * (w + 1);
            auto next = [&]() {
                uint64_t z = (s += 0x9E3779B97F4A7C15ull);
                z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                return z ^ (z >> 31);
            };
            const float fixed[3] = {3.7f, 7.25f, 12.0f};
            for (long i = w; i < samples; i += nt) {
                const uint64_t a = next(), b = next();
                // the kernels' domain: binary32 x in [0, 1 + 16 ulp], binary32 y in (0, 64)
                const float x = (a & 1) ? f32((uint32_t)((a >> 1) % 0x3f800011u))  // uniform over bit patterns
                                        : (float)((double)(a >> 11) * 0x1p-53);    // uniform over values
                const float y = (b % 4) < 3 ? fixed[b % 4] : (float)((double)(b >> 11) * 0x1p-53 * 64.0);
                T.check((double)x, (double)y);
                // the whole double range every 16th sample
                if (i % 16 == 0) {
                    const uint64_t c = next(), d = next();
                    double X = std::fabs(std::ldexp((double)(c >> 11) * 0x1p-53 + 0.5, (int)(c % 2100) - 1074));
                    double Y = std::ldexp((double)(d >> 11) * 0x1p-53, (int)(d % 80) - 40) * ((d >> 7) & 1 ? -1 : 1);
                    if (d % 9 == 0) Y = (double)((int64_t)(d >> 20) % 2001 - 1000);  // integer y
                    if (c % 13 == 0 && Y == std::floor(Y)) X = -X;                   // negative x, integer y
                    T.check(X, Y);
                }
            }
        });
    for (auto& x : th) x.join();
    Tally all;
    for (const Tally& x : t) all.n += x.n, all.dbl += x.dbl, all.flt += x.flt;
    // the device / glibc disagreements of tools/pow_check.hip, specials and edges
    Tally sp;
    sp.check((double)f32(0x3dd7cf12u), (double)0x1.946b02p+4f);
    sp.check((double)f32(0x3ed34fdeu), (double)0x1.273c82p+2f);
    const double sv[] = {0.0, -0.0, 1.0, -1.0, 0.5, 2.0, 0x1p-1074, 0x1p-1022, 0x1.fffffffffffffp1023, INFINITY,
                         -INFINITY, NAN, 1e-300, 1e300, 0x1p-65, 0x1p63, 3.0, -3.0, 0.999999999, 1.000000001};
    for (double x : sv)
        for (double y : sv) sp.check(x, y);
    all.n += sp.n, all.dbl += sp.dbl, all.flt += sp.flt;
    std::printf("pow_host: %ld compared, %ld double mismatches, %ld float mismatches\n", all.n, all.dbl, all.flt);
    return all.dbl ? 1 : 0;
}
