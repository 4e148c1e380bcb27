// Random 16-byte gathers (the push-sum round kernel's fired-link message reads) under each load
// cache policy: does any policy make the L2 fetch less than a 128 B line per gather?
//   hipcc --offload-arch=gfx950 -O3 -o gatherpol gatherpol.hip
//   ./gatherpol [policy]     (one policy per run, for rocprofv3 --pmc passes; none: all, timed)
// Policies (buffer_load_dwordx4 aux bits on gfx950): 0 plain, 1 sc0, 2 nt, 16 sc1, 17 sc0 sc1,
// 19 sc0 sc1 nt.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int AUX>
__global__ void k_gather(const double2* a, uint32_t rows, uint32_t n, double* sink) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, 0x7FFFFFFF, 0x00020000);
    double s = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t row = __umulhi(mix(i), rows);
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(row * 16u), 0, AUX);
        s += (double)v.x + (double)v.w;
    }
    if (s == -1.0) *sink = s;
}

typedef void (*Kern)(const double2*, uint32_t, uint32_t, double*);

int main(int argc, char** argv) {
    const int pols[] = {0, 1, 2, 16, 17, 19};
    const Kern ks[] = {k_gather<0>, k_gather<1>, k_gather<2>, k_gather<16>, k_gather<17>, k_gather<19>};
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    const size_t bytes = 1600ull << 20;  // 1.6 GB: far beyond the 256 MB Infinity Cache
    void* a;
    double* sink;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
    (void)hipMemset(a, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t n = 50000000u, rows = (uint32_t)(bytes / 16);
    for (int p = 0; p < 6; ++p) {
        if (only >= 0 && pols[p] != only) continue;
        float best = 1e30f;
        for (int rep = 0; rep < (only >= 0 ? 1 : 5); ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(ks[p], dim3(256 * 16), dim3(256), 0, 0, (const double2*)a, rows, n, sink);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("policy %2d: %u random 16 B gathers in %.1f us = %.2f G/s (%.2f TB/s of 128 B lines)\n", pols[p], n,
               best * 1e3, n / (best * 1e-3) / 1e9, n * 128.0 / (best * 1e-3) / 1e12);
    }
    printf("status %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
