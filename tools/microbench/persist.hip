// Prices a persistent multi-round kernel for the small graphs: one launch that
// runs R rounds with a device-wide barrier between them, against R dependent launches of the same
// round body on one stream (the engine's structure).  The barrier also carries the per-round
// completion count (the ParentActor gate, program.fs:44-63): every workgroup adds its count to the
// round's arrival counter and reads the total after the barrier, exactly what a persistent round
// kernel must do before it may start the next round.
//   hipcc --offload-arch=gfx950 -O3 -o persist persist.hip && ./persist
// Body: a 100k-actor "touch" round (each thread reads one element of the previous round's buffer
// written by another workgroup, adds one, writes the next buffer): the C2 round's size.
// Barriers: (a) one arrival counter per round (lane 0 release fence, agent atomic add, relaxed
// poll with s_sleep, acquire fence); (b) XCD-hierarchical: per-XCD counter, the XCD's last
// arriver adds to the top counter, every workgroup polls the top one.  Every spin is bounded: a
// barrier that does not complete sets an error flag and the kernel returns.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

constexpr int kN = 100000;
constexpr int kBlock = 256;
constexpr long long kSpinCap = 1ll << 22;

__device__ __forceinline__ unsigned ld_relaxed(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait until *p >= target (bounded), returns false on timeout
__device__ __forceinline__ bool spin_until(const unsigned* p, unsigned target) {
    long long spins = 0;
    while (ld_relaxed(p) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinCap) return false;
    }
    return true;
}

__device__ __forceinline__ void body(const int* __restrict__ in, int* __restrict__ out, int r) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    // read an element another workgroup wrote last round (stride 7919 actors away)
    const int j = (int)(((long long)i * 7919 + r) % kN);
    if (i < kN) out[i] = in[j] + 1;
}

__global__ void k_round(const int* in, int* out, int r) { body(in, out, r); }

// (a) flat counter barrier
__global__ __launch_bounds__(kBlock) void k_persist_flat(int* a, int* b, int rounds, unsigned* ctr, unsigned* cnt,
                                                         unsigned* err) {
    for (int r = 0; r < rounds; ++r) {
        body((r & 1) ? b : a, (r & 1) ? a : b, r);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicAdd(cnt + r, 1u);  // this round's completions ride the barrier
            atomicAdd(ctr, 1u);
            if (!spin_until(ctr, (unsigned)(r + 1) * gridDim.x)) atomicOr(err, 1u);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            (void)ld_relaxed(cnt + r);  // the gate's count after round r
        }
        __syncthreads();
        if (ld_relaxed(err)) return;
    }
}

// (b) XCD-hierarchical barrier: blocks with equal blockIdx % 8 count on one sub-counter (a
// speed hint only: correctness never depends on which XCD a block runs on)
__global__ __launch_bounds__(kBlock) void k_persist_xcd(int* a, int* b, int rounds, unsigned* sub, unsigned* top,
                                                        unsigned* cnt, unsigned* err) {
    const unsigned g = blockIdx.x & 7u, members = (gridDim.x - g + 7u) / 8u;
    for (int r = 0; r < rounds; ++r) {
        body((r & 1) ? b : a, (r & 1) ? a : b, r);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicAdd(cnt + r, 1u);
            const unsigned prev = atomicAdd(sub + g * 32, 1u);
            if (prev + 1 == (unsigned)(r + 1) * members) atomicAdd(top, 1u);  // the group's last arriver
            if (!spin_until(top, (unsigned)(r + 1) * 8u)) atomicOr(err, 1u);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            (void)ld_relaxed(cnt + r);
        }
        __syncthreads();
        if (ld_relaxed(err)) return;
    }
}

int main() {
    const int R = 2000;
    const int grid = (kN + kBlock - 1) / kBlock;  // 391: every block resident (<= 8 per CU)
    int *a, *b;
    unsigned *ctr, *sub, *top, *cnt, *err;
    if (hipMalloc(&a, kN * 4) || hipMalloc(&b, kN * 4) || hipMalloc(&ctr, 4) || hipMalloc(&sub, 8 * 32 * 4) ||
        hipMalloc(&top, 4) || hipMalloc(&cnt, R * 4) || hipMalloc(&err, 4))
        return 1;
    (void)hipMemset(a, 0, kN * 4);
    (void)hipMemset(b, 0, kN * 4);
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int pass = 0; pass < 2; ++pass) {
        float ms = 0;
        // launch per round
        (void)hipEventRecord(e0, s);
        for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_round, dim3(grid), dim3(kBlock), 0, s, (r & 1) ? b : a, (r & 1) ? a : b, r);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (pass) printf("launch per round (%d blocks): %.2f us/round\n", grid, ms * 1000.0 / R);
        for (int v = 0; v < 2; ++v) {
            (void)hipMemsetAsync(ctr, 0, 4, s);
            (void)hipMemsetAsync(sub, 0, 8 * 32 * 4, s);
            (void)hipMemsetAsync(top, 0, 4, s);
            (void)hipMemsetAsync(cnt, 0, R * 4, s);
            (void)hipMemsetAsync(err, 0, 4, s);
            (void)hipEventRecord(e0, s);
            if (v == 0) hipLaunchKernelGGL(k_persist_flat, dim3(grid), dim3(kBlock), 0, s, a, b, R, ctr, cnt, err);
            else hipLaunchKernelGGL(k_persist_xcd, dim3(grid), dim3(kBlock), 0, s, a, b, R, sub, top, cnt, err);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            unsigned e = 0;
            (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
            if (pass)
                printf("persistent, %s barrier + count (%d blocks): %.2f us/round%s\n", v ? "XCD-hierarchical" : "flat",
                       grid, ms * 1000.0 / R, e ? " (BARRIER TIMED OUT)" : "");
        }
    }
    printf("status %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
