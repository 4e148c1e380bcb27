// Calibration microbenchmarks for the round kernel's access patterns (MI355X).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy_gs(const double2* __restrict__ a, double2* __restrict__ b, uint32_t n, uint32_t span) {
    const uint32_t grp = blockIdx.x & 7u, j = blockIdx.x >> 3, per = gridDim.x >> 3;
    const uint32_t base = grp * span; uint32_t end = base + span < n ? base + span : n;
    for (uint32_t v = base + j * 256 + threadIdx.x; v < end; v += per * 256) { double2 x = a[v]; x.x += 1.0; b[v] = x; }
}
__global__ void copy_flat(const double2* __restrict__ a, double2* __restrict__ b, uint32_t n) {
    uint32_t v = blockIdx.x * 256 + threadIdx.x; if (v < n) { double2 x = a[v]; x.x += 1.0; b[v] = x; }
}
__global__ void copy_bytes(const double2* __restrict__ a, double2* __restrict__ b, const uint8_t* f, uint8_t* d, uint32_t n, uint32_t span) {
    const uint32_t grp = blockIdx.x & 7u, j = blockIdx.x >> 3, per = gridDim.x >> 3;
    const uint32_t base = grp * span; uint32_t end = base + span < n ? base + span : n;
    for (uint32_t v = base + j * 256 + threadIdx.x; v < end; v += per * 256) { double2 x = a[v]; x.x += f[v]; b[v] = x; d[v] = (uint8_t)v; }
}
__global__ void scatter16(const uint32_t* __restrict__ pos, double2* __restrict__ out, uint32_t* tag, uint32_t n, int with_tag) {
    uint32_t v = blockIdx.x * 256 + threadIdx.x; if (v < n) { uint32_t p = pos[v]; out[p] = make_double2(v, 1.0); if (with_tag) tag[p] = v; }
}
__global__ void gather_rand(const uint32_t* __restrict__ pos, const uint8_t* __restrict__ src, uint8_t* out, uint32_t n) {
    uint32_t v = blockIdx.x * 256 + threadIdx.x; if (v < n) out[v] = src[pos[v]];
}
// 7-row stencil read of double2 (own + v±1, v±G, v±P) as the pull kernel does
__global__ void stencil(const double2* __restrict__ a, double2* __restrict__ b, uint32_t n, uint32_t G, uint32_t P, uint32_t span) {
    const uint32_t grp = blockIdx.x & 7u, j = blockIdx.x >> 3, per = gridDim.x >> 3;
    const uint32_t base = grp * span; uint32_t end = base + span < n ? base + span : n;
    for (uint32_t v = base + j * 256 + threadIdx.x; v < end; v += per * 256) {
        double2 x = a[v];
        if (v >= P && v + P < n) {
            double2 y0 = a[v - P], y1 = a[v - G], y2 = a[v - 1], y3 = a[v + 1], y4 = a[v + G], y5 = a[v + P];
            x.x += y0.x + y1.x + y2.x + y3.x + y4.x + y5.x;
        }
        b[v] = x;
    }
}

int main() {
    const uint32_t n = 9938376, G = 239, P = G * G;
    double2 *a, *b; uint8_t *f, *d; uint32_t *pos, *tag;
    CK(hipMalloc(&a, n * 16ull)); CK(hipMalloc(&b, n * 16ull)); CK(hipMalloc(&f, n)); CK(hipMalloc(&d, n));
    CK(hipMalloc(&pos, n * 4ull)); CK(hipMalloc(&tag, n * 4ull));
    CK(hipMemset(a, 0, n * 16ull)); CK(hipMemset(f, 1, n));
    std::vector<uint32_t> h(n); for (uint32_t i = 0; i < n; ++i) h[i] = i;
    std::mt19937 rng(1); for (uint32_t i = n - 1; i > 0; --i) std::swap(h[i], h[rng() % (i + 1)]);
    CK(hipMemcpy(pos, h.data(), n * 4ull, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint32_t span = ((n + 7) / 8 + 255) / 256 * 256;
    auto timeit = [&](const char* name, double bytes, auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipEventRecord(e0)); for (int i = 0; i < 20; ++i) fn(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 20;
        printf("%-34s %8.1f us  %7.2f TB/s (%.0f MB)\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12, bytes / 1e6);
        return 0;
    };
    const uint32_t nb = (n + 255) / 256;
    for (int grid : {2048, 4096, 8192}) {
        char nm[64]; snprintf(nm, 64, "copy16 gridstride g=%d", grid);
        timeit(nm, n * 32.0, [&] { hipLaunchKernelGGL(copy_gs, dim3(grid), dim3(256), 0, 0, a, b, n, span); });
    }
    timeit("copy16 flat", n * 32.0, [&] { hipLaunchKernelGGL(copy_flat, dim3(nb), dim3(256), 0, 0, a, b, n); });
    timeit("copy16 + byte r/w gridstride", n * 34.0, [&] { hipLaunchKernelGGL(copy_bytes, dim3(2048), dim3(256), 0, 0, a, b, f, d, n, span); });
    timeit("stencil 7 rows gridstride", n * 32.0, [&] { hipLaunchKernelGGL(stencil, dim3(2048), dim3(256), 0, 0, a, b, n, G, P, span); });
    const uint32_t m = n / 7;
    timeit("scatter16 (n/7 random)", m * 20.0, [&] { hipLaunchKernelGGL(scatter16, dim3((m + 255) / 256), dim3(256), 0, 0, pos, b, tag, m, 0); });
    timeit("scatter16+tag4 (n/7 random)", m * 24.0, [&] { hipLaunchKernelGGL(scatter16, dim3((m + 255) / 256), dim3(256), 0, 0, pos, b, tag, m, 1); });
    timeit("gather 1B random (n)", n * 6.0, [&] { hipLaunchKernelGGL(gather_rand, dim3(nb), dim3(256), 0, 0, pos, f, d, n); });
    return 0;
}
