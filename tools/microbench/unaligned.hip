// Does gfx950 (ROCm 7.2 HSA defaults) serve dword / dwordx2 / dwordx4 global loads at byte- and
// dword-unaligned addresses?  The tile round kernel reads direction / mark bytes of rows that
// start at arbitrary actor ids (v - G, v + G^2 ...) as whole dwords.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void k(const uint8_t* p, uint32_t* o1, uint2* o2, uint4* o4, const uint32_t* w, uint4* o5) {
    const int i = threadIdx.x;  // byte offset i
    o1[i] = *reinterpret_cast<const uint32_t*>(p + i);
    o2[i] = *reinterpret_cast<const uint2*>(p + i);
    o4[i] = *reinterpret_cast<const uint4*>(p + i);
    o5[i] = *reinterpret_cast<const uint4*>(w + i);  // dword-aligned dwordx4
}

int main() {
    const int N = 64;
    uint8_t h[256];
    for (int i = 0; i < 256; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t* d;
    uint32_t *o1, *w;
    uint2* o2;
    uint4 *o4, *o5;
    hipMalloc(&d, 256);
    hipMalloc(&o1, N * 4);
    hipMalloc(&o2, N * 8);
    hipMalloc(&o4, N * 16);
    hipMalloc(&o5, N * 16);
    hipMalloc(&w, 1024);
    uint32_t hw[256];
    for (int i = 0; i < 256; ++i) hw[i] = 0x1000u + i;
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    hipMemcpy(w, hw, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(N), 0, 0, d, o1, o2, o4, w, o5);
    uint32_t r1[N];
    uint2 r2[N];
    uint4 r4[N], r5[N];
    hipMemcpy(r1, o1, sizeof r1, hipMemcpyDeviceToHost);
    hipMemcpy(r2, o2, sizeof r2, hipMemcpyDeviceToHost);
    hipMemcpy(r4, o4, sizeof r4, hipMemcpyDeviceToHost);
    hipMemcpy(r5, o5, sizeof r5, hipMemcpyDeviceToHost);
    int bad1 = 0, bad2 = 0, bad4 = 0, bad5 = 0;
    for (int i = 0; i < N; ++i) {
        uint32_t e1;
        uint2 e2;
        uint4 e4;
        memcpy(&e1, h + i, 4);
        memcpy(&e2, h + i, 8);
        memcpy(&e4, h + i, 16);
        bad1 += e1 != r1[i];
        bad2 += memcmp(&e2, &r2[i], 8) != 0;
        bad4 += memcmp(&e4, &r4[i], 16) != 0;
        bad5 += memcmp(hw + i, &r5[i], 16) != 0;
    }
    printf("unaligned dword: %d bad, dwordx2: %d bad, dwordx4: %d bad (of %d); dword-aligned dwordx4: %d bad\n", bad1,
           bad2, bad4, N, bad5);
    return (bad1 || bad2 || bad4 || bad5) ? 1 : 0;
}
