// Back-to-back dependent kernel launches on one stream: host enqueue rate vs GPU-side rate, and
// the same work as one hipGraph replay.  Small-graph rounds (C2: 100k actors, 62125 rounds) cost
// ~6 us each; is that the launch path or the kernel?
//   hipcc --offload-arch=gfx950 -O3 -o launch launch.hip && ./launch
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1024) *p = 0;
}

__global__ void k_touch(const int* __restrict__ in, int* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i] + 1;
}

// three dependent loads per thread (like the round kernel's gate -> flags -> message levels)
__global__ void k_chain(const int* __restrict__ perm, int* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = perm[perm[perm[i]]] + 1;
}

// eight dependent loads: a kernel whose own latency exceeds the host enqueue interval
__global__ void k_chain8(const int* __restrict__ perm, int* __restrict__ out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        int j = i;
#pragma unroll
        for (int l = 0; l < 8; ++l) j = perm[j];
        out[i] = j;
    }
}

int main() {
    const int N = 20000, n = 100000;
    int *a, *b;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    {
        int* h = new int[n];
        for (int i = 0; i < n; ++i) h[i] = (int)((i * 2654435761u) % (unsigned)n);
        (void)hipMemcpy(a, h, n * 4, hipMemcpyHostToDevice);
        delete[] h;
    }
    for (int pass = 0; pass < 2; ++pass) {
        for (int kind = 0; kind < 4; ++kind) {
            (void)hipStreamSynchronize(s);
            auto t0 = std::chrono::steady_clock::now();
            (void)hipEventRecord(e0, s);
            for (int i = 0; i < N; ++i) {
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(392), dim3(256), 0, s, nullptr);
                else if (kind == 3) hipLaunchKernelGGL(k_chain8, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n);
                else if (kind == 2) hipLaunchKernelGGL(k_chain, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n);
                else hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, n);
            }
            auto t1 = std::chrono::steady_clock::now();
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            auto t2 = std::chrono::steady_clock::now();
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (pass)
                printf("%s x%d: enqueue %.2f us/launch, wall %.2f us/launch, device %.2f us/launch\n",
                       kind == 3 ? "chain8_100k" : kind == 2 ? "chain100k" : kind ? "touch100k" : "empty", N,
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / N, ms * 1000.0 / N);
        }
    }
    // one graph of G dependent kernels, replayed
    const int G = 200, R = 100;
    for (int kind = 1; kind < 4; ++kind) {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < G; ++i) {
            if (kind == 3) hipLaunchKernelGGL(k_chain8, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n);
            else if (kind == 2) hipLaunchKernelGGL(k_chain, dim3((n + 255) / 256), dim3(256), 0, s, a, b, n);
            else hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, n);
        }
        (void)hipStreamEndCapture(s, &g);
        auto ti = std::chrono::steady_clock::now();
        if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return 1;
        auto tj = std::chrono::steady_clock::now();
        (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        auto t0 = std::chrono::steady_clock::now();
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < R; ++i) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        auto t2 = std::chrono::steady_clock::now();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("graph of %d %s: instantiate %.1f us; wall %.2f us/kernel, device %.2f us/kernel\n", G,
               kind == 3 ? "chain8_100k" : kind == 2 ? "chain100k" : "touch100k", std::chrono::duration<double, std::micro>(tj - ti).count(),
               std::chrono::duration<double, std::micro>(t2 - t0).count() / (G * R), ms * 1000.0 / (G * R));
    }
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
