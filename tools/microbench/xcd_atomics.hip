// Receipt atomics performed in an XCD's own L2 (workgroup scope) instead of beyond it (device
// scope), for a receipt pass whose targets are partitioned over the XCDs by the hardware XCC id:
// every workgroup reads its XCC id, takes chunks of the entry list from its XCD's queue and applies
// only the entries whose target lies in its XCD's eighth of the array.  Each word is then only ever
// updated through one L2 within the kernel, and the kernel-end writeback publishes it.  A partition
// whose XCD ran no workgroup is applied by the grid's last workgroup with device-scope atomics.
//   agent     device-scope atomicAdd per entry (the engine's unpack today)
//   xcd       the partitioned pass above (every XCD reads every entry)
//   xcd_raw   the L2 atomic rate alone: each workgroup adds random receipts in its own partition
// Checks: the partitioned histogram equals the device-scope one word for word.
//   hipcc --offload-arch=gfx950 -O3 -o xcd_atomics xcd_atomics.hip && ./xcd_atomics
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u; }

__global__ void k_fill(uint32_t* e, uint32_t n, uint32_t words) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        e[i] = __umulhi(mix(i * 2654435761u + 12345u), words);
}

__global__ void k_agent(const uint32_t* e, uint32_t n, uint32_t* a) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&a[e[i]], 1u);
}

constexpr uint32_t kChunk = 256u * 16u;

// ctl: [0..7] queue heads, [8..15] workgroups started per XCD, [16] workgroups finished
__global__ __launch_bounds__(256) void k_xcd(const uint32_t* e, uint32_t n, uint32_t* a, uint32_t words,
                                             uint32_t* ctl) {
    __shared__ uint32_t chunk_s, last_s;
    const uint32_t x = xcc_id();
    const uint32_t part = (words + 7u) / 8u;
    const uint32_t lo = x * part, hi = lo + part;
    const uint32_t nchunks = (n + kChunk - 1u) / kChunk;
    if (threadIdx.x == 0) atomicAdd(&ctl[8 + x], 1u);
    for (;;) {
        if (threadIdx.x == 0) chunk_s = atomicAdd(&ctl[x], 1u);
        __syncthreads();
        const uint32_t c = chunk_s;
        __syncthreads();
        if (c >= nchunks) break;
        const uint32_t b = c * kChunk, end = min(b + kChunk, n);
        for (uint32_t i = b + threadIdx.x; i < end; i += blockDim.x) {
            const uint32_t t = e[i];
            if (t - lo < hi - lo) __hip_atomic_fetch_add(&a[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    // the grid's last workgroup applies the partitions of XCDs that ran none (device scope: no L2
    // holds those words, since no workgroup of that XCD touched them)
    __threadfence();
    if (threadIdx.x == 0) last_s = atomicAdd(&ctl[16], 1u) == gridDim.x - 1u;
    __syncthreads();
    if (!last_s) return;
    __threadfence();
    for (uint32_t y = 0; y < 8u; ++y) {
        if (__hip_atomic_load(&ctl[8 + y], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) continue;
        const uint32_t ylo = y * part, yhi = ylo + part;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t t = e[i];
            if (t - ylo < yhi - ylo) atomicAdd(&a[t], 1u);
        }
    }
}

__global__ void k_xcd_raw(uint32_t n, uint32_t* a, uint32_t words) {
    const uint32_t x = xcc_id();
    const uint32_t part = words / 8u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        __hip_atomic_fetch_add(&a[x * part + __umulhi(mix(i), part)], 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
}

__global__ void k_agent_raw(uint32_t n, uint32_t* a, uint32_t words) {
    const uint32_t x = xcc_id();
    const uint32_t part = words / 8u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&a[x * part + __umulhi(mix(i), part)], 1u);
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t err_ = (x);                                                     \
        if (err_ != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const uint32_t wordss[] = {1u << 22, 12500000u, 1u << 25};
    const uint32_t ns[] = {5250000u, 26600000u};
    const int grid = 2048, reps = 5;
    uint32_t *e, *a, *b, *ctl;
    CK(hipMalloc(&e, 4ull * 26600000u));
    CK(hipMalloc(&a, 4ull << 25));
    CK(hipMalloc(&b, 4ull << 25));
    CK(hipMalloc(&ctl, 4 * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::printf("words n kernel ms Gatomics/s check\n");
    for (uint32_t words : wordss) {
        for (uint32_t n : ns) {
            hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, 0, e, n, words);
            float best[4] = {1e30f, 1e30f, 1e30f, 1e30f};
            bool ok = true;
            for (int rep = 0; rep < reps; ++rep) {
                CK(hipMemset(a, 0, 4ull * words));
                CK(hipMemset(b, 0, 4ull * words));
                CK(hipMemset(ctl, 0, 4 * 32));
                float ms;
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_agent, dim3(grid), dim3(256), 0, 0, e, n, a);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                best[0] = std::min(best[0], ms);
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_xcd, dim3(grid), dim3(256), 0, 0, e, n, b, words, ctl);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                best[1] = std::min(best[1], ms);
                std::vector<uint32_t> ha(words), hb(words);
                CK(hipMemcpy(ha.data(), a, 4ull * words, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hb.data(), b, 4ull * words, hipMemcpyDeviceToHost));
                if (ha != hb) ok = false;
                std::vector<uint32_t> hc(32);
                CK(hipMemcpy(hc.data(), ctl, 4 * 32, hipMemcpyDeviceToHost));
                if (rep == 0) {
                    std::printf("# workgroups per XCC:");
                    for (int y = 0; y < 8; ++y) std::printf(" %u", hc[8 + y]);
                    std::printf("\n");
                }
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_agent_raw, dim3(grid), dim3(256), 0, 0, n, a, words);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                best[2] = std::min(best[2], ms);
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_xcd_raw, dim3(grid), dim3(256), 0, 0, n, a, words);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                best[3] = std::min(best[3], ms);
            }
            const char* names[] = {"agent", "xcd", "agent_raw", "xcd_raw"};
            for (int k = 0; k < 4; ++k)
                std::printf("%u %u %s %.4f %.2f %s\n", words, n, names[k], best[k], n / (best[k] * 1e6),
                            k == 1 ? (ok ? "equal" : "DIFFER") : "-");
        }
    }
    return 0;
}
