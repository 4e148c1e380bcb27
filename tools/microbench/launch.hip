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

int main() {
    const int N = 20000, n = 100000;
    int *a, *b;
    if (hipMalloc(&a, n * 4) != hipSuccess || hipMalloc(&b, n * 4) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int pass = 0; pass < 2; ++pass) {
        for (int kind = 0; kind < 2; ++kind) {
            (void)hipStreamSynchronize(s);
            auto t0 = std::chrono::steady_clock::now();
            (void)hipEventRecord(e0, s);
            for (int i = 0; i < N; ++i) {
                if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(392), dim3(256), 0, s, nullptr);
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
                       kind ? "touch100k" : "empty", N,
                       std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
                       std::chrono::duration<double, std::micro>(t2 - t0).count() / N, ms * 1000.0 / N);
        }
    }
    // one graph of G dependent touch kernels, replayed
    const int G = 200, R = 100;
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < G; ++i)
        hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, n);
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
    printf("graph of %d touch100k: instantiate %.1f us; wall %.2f us/kernel, device %.2f us/kernel\n", G,
           std::chrono::duration<double, std::micro>(tj - ti).count(),
           std::chrono::duration<double, std::micro>(t2 - t0).count() / (G * R), ms * 1000.0 / (G * R));
    hipError_t e = hipGetLastError();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
