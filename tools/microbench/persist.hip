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

// (c) one XCD only: the blocks running on XCD 0 (hardware XCC_ID, not blockIdx) do all the work and
// synchronise through that XCD's L2, which they share: release = s_waitcnt vmcnt(0) (the vector L1
// writes through), the arrival atomic at workgroup scope (performed in the shared L2), acquire =
// invalidate the vector L1 (buffer_inv sc0).  The other blocks exit at once.  Membership: every
// block registers, then all wait until every block of the grid has started (one device-wide
// rendezvous), so the XCD-0 member count is final before round 0.
__device__ __forceinline__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u; }

__global__ __launch_bounds__(kBlock) void k_persist_one_xcd(int* a, int* b, int rounds, unsigned* started,
                                                            unsigned* members, unsigned* arrive, unsigned* cnt,
                                                            unsigned* err) {
    __shared__ unsigned rank_s, nmem_s;
    const bool mine = xcc_id() == 0u;
    if (threadIdx.x == 0) {
        rank_s = mine ? atomicAdd(members, 1u) : 0u;
        atomicAdd(started, 1u);
        if (!spin_until(started, gridDim.x)) atomicOr(err, 1u);
        nmem_s = ld_relaxed(members);
    }
    __syncthreads();
    if (!mine || ld_relaxed(err)) return;
    const unsigned rank = rank_s, nmem = nmem_s;
    for (int r = 0; r < rounds; ++r) {
        const int* in = (r & 1) ? b : a;
        int* out = (r & 1) ? a : b;
        for (int i = (int)(rank * kBlock + threadIdx.x); i < kN; i += (int)(nmem * kBlock)) {
            const int j = (int)(((long long)i * 7919 + r) % kN);
            out[i] = in[j] + 1;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(cnt + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            long long spins = 0;
            while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(r + 1) * nmem) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kSpinCap) {
                    atomicOr(err, 1u);
                    break;
                }
            }
        }
        __syncthreads();
        asm volatile("buffer_inv sc0" ::: "memory");
        if (ld_relaxed(err)) return;
    }
}

int main() {
    const int R = 2000;
    const int grid = (kN + kBlock - 1) / kBlock;  // 391: every block resident (<= 8 per CU)
    int *a, *b;
    unsigned *ctr, *sub, *top, *cnt, *err, *started, *members, *arrive;
    if (hipMalloc(&a, kN * 4) || hipMalloc(&b, kN * 4) || hipMalloc(&ctr, 4) || hipMalloc(&sub, 8 * 32 * 4) ||
        hipMalloc(&top, 4) || hipMalloc(&cnt, R * 4) || hipMalloc(&err, 4) || hipMalloc(&started, 4) ||
        hipMalloc(&members, 4) || hipMalloc(&arrive, 4))
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
    // (c): 8 x 32 blocks, so about 32 land on XCD 0 (one per CU); the result is checked against
    // the launch-per-round result of the same rounds
    for (int pass = 0; pass < 2; ++pass) {
        (void)hipMemsetAsync(a, 0, kN * 4, s);
        (void)hipMemsetAsync(b, 0, kN * 4, s);
        (void)hipMemsetAsync(started, 0, 4, s);
        (void)hipMemsetAsync(members, 0, 4, s);
        (void)hipMemsetAsync(arrive, 0, 4, s);
        (void)hipMemsetAsync(cnt, 0, R * 4, s);
        (void)hipMemsetAsync(err, 0, 4, s);
        float ms = 0;
        (void)hipEventRecord(e0, s);
        hipLaunchKernelGGL(k_persist_one_xcd, dim3(256), dim3(kBlock), 0, s, a, b, R, started, members, arrive, cnt, err);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned e = 0, m = 0;
        (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&m, members, 4, hipMemcpyDeviceToHost);
        static int got[kN], want[kN];
        (void)hipMemcpy(got, (R & 1) ? b : a, kN * 4, hipMemcpyDeviceToHost);
        (void)hipMemsetAsync(a, 0, kN * 4, s);
        (void)hipMemsetAsync(b, 0, kN * 4, s);
        for (int r = 0; r < R; ++r) hipLaunchKernelGGL(k_round, dim3(grid), dim3(kBlock), 0, s, (r & 1) ? b : a, (r & 1) ? a : b, r);
        (void)hipMemcpy(want, (R & 1) ? b : a, kN * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < kN; ++i) bad += got[i] != want[i];
        if (pass)
            printf("persistent on one XCD, L2-local barrier + count (%u blocks on XCD 0): %.2f us/round, %d of %d "
                   "elements differ from the launch-per-round result%s\n",
                   m, ms * 1000.0 / R, bad, kN, e ? " (BARRIER TIMED OUT)" : "");
    }
    printf("status %s\n", hipGetErrorString(hipGetLastError()));
    return 0;
}
