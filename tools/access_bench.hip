// access_bench.hip -- micro-benchmark of read patterns over a 1920x1080xF int32 band set
// (GPU box; tools only).  Linear stream vs the codec's 8x8-tile pattern.
//   hipcc -O3 --offload-arch=gfx950 -o tools/access_bench tools/access_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(2); } } while (0)

__global__ void linear(const int* __restrict__ a, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) acc ^= a[i];
    if (acc == 0x12345678u) out[0] = acc;
}

// one wave per 16 consecutive 8x8 tiles; W columns, rows = n / W
template <int TPW>
__global__ void tiles(const int* __restrict__ a, int W, int tiles_x, int n_tiles, unsigned* out) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned acc = 0;
    for (int g = blockIdx.x * 4 + wave; g * TPW < n_tiles; g += gridDim.x * 4) {
        unsigned v[TPW];
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
            const int t = g * TPW + j;
            const int tr = t / tiles_x, tc = t - tr * tiles_x;
            v[j] = a[(size_t)(tr * 8 + (lane >> 3)) * W + tc * 8 + (lane & 7)];
        }
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc ^= v[j];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// decoder store pattern: lane 8j+ry writes row ry (8 pixels, 2 x 16 B) of tile g*8+j
__global__ void store_rows(int* __restrict__ a, int W, int tiles_x, int n_tiles, int stride_loop) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int groups = n_tiles / 8;
    for (int g = blockIdx.x * 4 + wave; g < groups; g += stride_loop ? gridDim.x * 4 : groups) {
        const int t = g * 8 + (lane >> 3), ry = lane & 7;
        const int tr = t / tiles_x, tc = t - tr * tiles_x;
        int4* d = (int4*)(a + (size_t)(tr * 8 + ry) * W + tc * 8);
        d[0] = make_int4(t, t, t, t);
        d[1] = make_int4(t, t, t, t);
    }
}

int main() {
    const int W = 1920, H = 1080 * 8;
    const size_t n = (size_t)W * H;
    int* a;
    unsigned* out;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(a, 1, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipEventRecord(e0));
        for (int i = 0; i < 20; ++i) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 1e3 / 20, n * 4 / (ms / 20 * 1e-3) / 1e12);
    };
    const int tx = W / 8, nt = tx * (H / 8);
    run("linear grid 8192x256", [&] { hipLaunchKernelGGL(linear, dim3(8192), dim3(256), 0, 0, a, n, out); });
    run("linear grid 2048x256", [&] { hipLaunchKernelGGL(linear, dim3(2048), dim3(256), 0, 0, a, n, out); });
    run("tiles16 full grid", [&] { hipLaunchKernelGGL(tiles<16>, dim3((nt / 16 + 3) / 4), dim3(256), 0, 0, a, W, tx, nt, out); });
    run("tiles16 grid 2048", [&] { hipLaunchKernelGGL(tiles<16>, dim3(2048), dim3(256), 0, 0, a, W, tx, nt, out); });
    run("tiles4 full grid", [&] { hipLaunchKernelGGL(tiles<4>, dim3((nt / 4 + 3) / 4), dim3(256), 0, 0, a, W, tx, nt, out); });
    run("tiles1 full grid", [&] { hipLaunchKernelGGL(tiles<1>, dim3((nt + 3) / 4), dim3(256), 0, 0, a, W, tx, nt, out); });
    run("store_rows full grid", [&] { hipLaunchKernelGGL(store_rows, dim3((nt / 8 + 3) / 4), dim3(256), 0, 0, a, W, tx, nt, 0); });
    run("store_rows grid 2048", [&] { hipLaunchKernelGGL(store_rows, dim3(2048), dim3(256), 0, 0, a, W, tx, nt, 1); });
    return 0;
}
