// issue_probe.hip -- issue-rate probe for the trace kernels' instruction mix (MI355X, gfx950).
//
// The trace kernels issue ~250 scalar (SALU) and ~450 vector (VALU) instructions per wave
// (profiles/r02_C2_pmc_summary.txt).  This probe measures, with every CU full of one-wave
// workgroups (the trace kernels' shape), the time per wave-instruction of
//   salu : independent s_add_u32 chains (uniform values, scalar ALU)
//   valu : independent v_add_f32 chains
//   mix  : both interleaved 1:1
// to tell whether the CU's scalar unit (shared by its 4 SIMDs) or the SIMDs' vector issue
// bounds a mixed stream.  Register-only arithmetic: no memory traffic besides one store per
// wave of its result (so the compiler keeps the chains).
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/issue_probe tools/issue_probe.hip && tools/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

constexpr int ITERS = 4096;

template <int MODE>  // 0 salu, 1 valu, 2 mix 1:1, 3 mix 3 VALU : 1 SALU, 4 mix 6 VALU : 1 SALU
__global__ __launch_bounds__(64) void probe(unsigned* out, unsigned seed) {
    unsigned s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3;
    float v0 = (float)threadIdx.x, v1 = v0 + 1.0f, v2 = v0 + 2.0f, v3 = v0 + 3.0f;
#pragma unroll 16
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (MODE != 1) {
            asm volatile(
                "s_add_u32 %0, %0, 3\n\t"
                "s_add_u32 %1, %1, 5\n\t"
                "s_add_u32 %2, %2, 7\n\t"
                "s_add_u32 %3, %3, 9\n\t"
                : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3)
                :
                : "scc");
        }
        if constexpr (MODE != 0) {
#pragma unroll
            for (int r = 0; r < (MODE == 3 ? 3 : MODE == 4 ? 6 : 1); ++r)
                asm volatile(
                    "v_add_f32 %0, 1.0, %0\n\t"
                    "v_add_f32 %1, 1.0, %1\n\t"
                    "v_add_f32 %2, 1.0, %2\n\t"
                    "v_add_f32 %3, 1.0, %3\n\t"
                    : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        }
    }
    const unsigned r = s0 ^ s1 ^ s2 ^ s3 ^ __float_as_uint(v0 + v1 + v2 + v3);
    out[blockIdx.x * 64 + threadIdx.x] = r;  // vector store of the result
}

template <int MODE>
static int run(const char* name, int waves, unsigned* d) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(probe<MODE>, dim3(waves), dim3(64), 0, 0, d, 1u);  // warm-up
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(probe<MODE>, dim3(waves), dim3(64), 0, 0, d, (unsigned)k);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    const double per_wave = (MODE == 2 ? 8.0 : MODE == 3 ? 16.0 : MODE == 4 ? 28.0 : 4.0) * ITERS;  // instructions per wave
    const double cu_cycles = ms * 1e-3 * 2.4e9;                 // at 2.4 GHz
    std::printf("%-5s waves %7d  %.3f ms  %.3f wave-instructions per CU-cycle  (%.2f per SIMD-cycle)\n", name,
                waves, ms, waves / 256.0 * per_wave / cu_cycles, waves / 1024.0 * per_wave / cu_cycles);
    return 0;
}

int main() {
    unsigned* d = nullptr;
    const int waves = 256 * 32 * 8;  // 8 rounds of 32 one-wave workgroups per CU
    CHECK(hipMalloc(&d, (size_t)waves * 64 * sizeof(unsigned)));
    if (run<0>("salu", waves, d) || run<1>("valu", waves, d) || run<2>("mix", waves, d) || run<3>("mix31", waves, d) ||
        run<4>("mix61", waves, d))
        return 1;
    CHECK(hipFree(d));
    return 0;
}
