// Random 16-byte gathers and random 1-byte stores on gfx950: the two random accesses of the
// push-sum round kernel (a fired link's message read from the sender's row; the link mark byte
// written into the receiver's CSR slot).  Rate by footprint and by count per launch (1.42M is
// one C3 round's worth; 100M is the steady-state rate).
//   hipcc --offload-arch=gfx950 -O3 -o gather gather.hip && ./gather
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

__global__ void k_gather16(const double2* a, uint32_t rows, uint32_t n, double* sink) {
    double s = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double2 m = a[__umulhi(mix(i), rows)];
        s += m.x + m.y;
    }
    if (s == -1.0) *sink = s;
}

__global__ void k_store1(uint8_t* a, uint32_t bytes, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        a[__umulhi(mix(i), bytes)] = (uint8_t)i;
}

int main() {
    const size_t big = 16ull << 30;
    void* a;
    double* sink;
    if (hipMalloc(&a, big) != hipSuccess) return 1;
    hipMalloc(&sink, 8);
    hipMemset(a, 0, big);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t mbs[] = {40, 160, 1600, 16000};
    const uint32_t counts[] = {1420000u, 100000000u};
    printf("kind footprint_MB count us G/s\n");
    for (size_t mb : mbs)
        for (uint32_t n : counts)
            for (int kind = 0; kind < 2; ++kind) {
                float best = 1e30f;
                for (int rep = 0; rep < 5; ++rep) {
                    hipEventRecord(e0);
                    if (kind == 0)
                        k_gather16<<<256 * 16, 256>>>((const double2*)a, (uint32_t)((mb << 20) / 16), n, sink);
                    else
                        k_store1<<<256 * 16, 256>>>((uint8_t*)a, (uint32_t)std::min<size_t>(mb << 20, 0xFFFFFFFFull), n);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                printf("%s %zu %u %.1f %.2f\n", kind == 0 ? "gather16" : "store1", mb, n, best * 1e3, n / (best * 1e-3) / 1e9);
            }
    return 0;
}
