// Random-target receipt throughput on gfx950: how fast can one kernel land N receipts at random
// targets of an array, by footprint?  (Full-topology gossip lands ~1.5e8 receipts per round.)
//   atomic      atomicAdd(u32) without return (device scope: performed beyond the XCD's L2)
//   atomic_ret  the same with the old value used
//   pack8       atomicAdd on a u32 word holding 4 u8 counters (footprint / 4)
//   store4      plain random 4-byte stores (a bucketing pass's scatter)
//   stream      coalesced 16-byte copy of the same footprint (reference)
//   hipcc --offload-arch=gfx950 -O3 -o atomics atomics.hip && ./atomics
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__global__ void k_atomic(uint32_t* a, uint32_t words, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&a[__umulhi(mix(i), words)], 1u);
}

__global__ void k_atomic_ret(uint32_t* a, uint32_t words, uint32_t n, uint32_t* sink) {
    uint32_t s = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        s += atomicAdd(&a[__umulhi(mix(i), words)], 1u);
    if (s == 0xFFFFFFFFu) *sink = s;
}

__global__ void k_pack8(uint32_t* a, uint32_t words, uint32_t n) {
    const uint32_t targets = words * 4u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t t = __umulhi(mix(i), targets);
        atomicAdd(&a[t >> 2], 1u << (8u * (t & 3u)));
    }
}

__global__ void k_store4(uint32_t* a, uint32_t words, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        a[__umulhi(mix(i), words)] = i;
}

__global__ void k_stream(const uint4* a, uint4* b, uint32_t n16) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
    const uint32_t n = 100000000u;
    const size_t mbs[] = {16, 64, 128, 192, 256, 400, 800};
    uint32_t *a, *b, *sink;
    hipMalloc(&a, 800ull << 20);
    hipMalloc(&b, 800ull << 20);
    hipMalloc(&sink, 4);
    hipMemset(a, 0, 800ull << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 16, block = 256;
    printf("footprint_MB kernel ms Gops/s\n");
    for (size_t mb : mbs) {
        const uint32_t words = (uint32_t)((mb << 20) / 4);
        for (int kind = 0; kind < 5; ++kind) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(e0);
                switch (kind) {
                case 0: k_atomic<<<grid, block>>>(a, words, n); break;
                case 1: k_atomic_ret<<<grid, block>>>(a, words, n, sink); break;
                case 2: k_pack8<<<grid, block>>>(a, words / 4u, n); break;
                case 3: k_store4<<<grid, block>>>(a, words, n); break;
                default: k_stream<<<grid, block>>>((const uint4*)a, (uint4*)b, words / 4u); break;
                }
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (rep && ms < best) best = ms;
            }
            const char* names[] = {"atomic", "atomic_ret", "pack8", "store4", "stream"};
            const double ops = kind == 4 ? (double)words / 4.0 : (double)n;
            printf("%zu %s %.3f %.2f%s\n", kind == 2 ? mb / 4 : mb, names[kind], best, ops / best / 1e6,
                   kind == 4 ? " (G x16B/s)" : "");
        }
    }
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
