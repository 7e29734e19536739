// launch_probe.hip -- floor of a 1080p frame made of 8x8-pixel one-wave workgroups (MI355X, gfx950).
//
// The trace kernel takes ~7 us per 1920x1080 frame on an EMPTY scene (tools/strip_probe.sh), against
// ~1.4 us of store traffic.  This probe times, over 64 frames per launch (grid z = frame, as the bench),
// kernels that only store a constant per pixel in different shapes, to tell what the per-tile floor is:
//   tile64     : 8x8 tile per 64-thread workgroup (the trace kernels' shape)
//   tile64_ka  : same, plus a 2.3 KB kernel-argument block read by every wave (LaunchParams' size)
//   row64      : 64x1 pixel strip per 64-thread workgroup (one 256-B row segment per store)
//   tile256    : 2x2 tiles per 256-thread workgroup (4 waves)
//   loop4      : one wave stores 4 tiles one after the other (grid x / 4)
//   tile64_lat : tile64 plus a dependent global load of a per-column table before the store (the view
//                tables of the trace kernels)
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/launch_probe tools/launch_probe.hip && tools/launch_probe
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

constexpr int W = 1920, H = 1080, F = 64;

struct Big {
    int w, h;
    float pad[560];  // ~2.3 KB, like LaunchParams
    int* out;
};

__global__ __launch_bounds__(64) void tile64(int* out) {
    const int x = blockIdx.x * 8 + (threadIdx.x & 7), y = blockIdx.y * 8 + (threadIdx.x >> 3);
    if (x < W && y < H) out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = x ^ y;
}

__global__ __launch_bounds__(64) void tile64_ka(Big p) {
    const int x = blockIdx.x * 8 + (threadIdx.x & 7), y = blockIdx.y * 8 + (threadIdx.x >> 3);
    const float v = p.pad[(x + y) % 560];  // per-lane kernarg read
    if (x < p.w && y < p.h) p.out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = (int)v ^ x;
}

__global__ __launch_bounds__(64) void tile64_lat(int* out, const float* tab) {
    const int x = blockIdx.x * 8 + (threadIdx.x & 7), y = blockIdx.y * 8 + (threadIdx.x >> 3);
    const float a = tab[x < W ? x : 0], b = tab[W + (y < H ? y : 0)];
    if (x < W && y < H) out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = (int)(a * b);
}

__global__ __launch_bounds__(64) void row64(int* out) {
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y;
    if (x < W && y < H) out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = x ^ y;
}

__global__ __launch_bounds__(256) void tile256(int* out) {
    const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int x = (blockIdx.x * 2 + (wv & 1)) * 8 + (l & 7), y = (blockIdx.y * 2 + (wv >> 1)) * 8 + (l >> 3);
    if (x < W && y < H) out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = x ^ y;
}

__global__ __launch_bounds__(64) void loop4(int* out) {
    for (int k = 0; k < 4; ++k) {
        const int x = (blockIdx.x * 4 + k) * 8 + (threadIdx.x & 7), y = blockIdx.y * 8 + (threadIdx.x >> 3);
        if (x < W && y < H) out[(size_t)blockIdx.z * W * H + (size_t)y * W + x] = x ^ y;
    }
}

template <typename L>
static int timeit(const char* name, L launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int k = 0; k < 3; ++k) launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    const int reps = 20;
    for (int k = 0; k < reps; ++k) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::printf("%-11s %7.3f us per 1080p frame\n", name, ms * 1e3 / reps / F);
    return 0;
}

int main() {
    int* out = nullptr;
    float* tab = nullptr;
    CHECK(hipMalloc(&out, (size_t)F * W * H * sizeof(int)));
    CHECK(hipMalloc(&tab, (size_t)(W + H) * sizeof(float)));
    CHECK(hipMemset(tab, 0, (size_t)(W + H) * sizeof(float)));
    const dim3 g64((W + 7) / 8, (H + 7) / 8, F);
    static Big big;
    big.w = W, big.h = H, big.out = out;
    for (int rep = 0; rep < 2; ++rep) {
        if (timeit("tile64", [&] { hipLaunchKernelGGL(tile64, g64, dim3(64), 0, 0, out); }) ||
            timeit("tile64_ka", [&] { hipLaunchKernelGGL(tile64_ka, g64, dim3(64), 0, 0, big); }) ||
            timeit("tile64_lat", [&] { hipLaunchKernelGGL(tile64_lat, g64, dim3(64), 0, 0, out, tab); }) ||
            timeit("row64", [&] { hipLaunchKernelGGL(row64, dim3((W + 63) / 64, H, F), dim3(64), 0, 0, out); }) ||
            timeit("tile256", [&] {
                hipLaunchKernelGGL(tile256, dim3((W + 15) / 16, (H + 15) / 16, F), dim3(256), 0, 0, out);
            }) ||
            timeit("loop4", [&] { hipLaunchKernelGGL(loop4, dim3((W + 31) / 32, (H + 7) / 8, F), dim3(64), 0, 0, out); }))
            return 1;
    }
    CHECK(hipFree(out));
    CHECK(hipFree(tab));
    return 0;
}
