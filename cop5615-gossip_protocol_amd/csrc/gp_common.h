// gp_common.h — host+device definitions shared by the gfx950 kernels and the C-ABI host code.
//
// Round semantics: DESIGN.md §2.  Topology arithmetic follows
// /root/reference/program.fs:151-313 without materialising neighbour arrays: every regular
// topology is a (GX, GY, GZ) slab of `wired` actors addressed by index arithmetic, plus a
// one-entry-per-node extra link for Imp3D.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gp {

// ---------------------------------------------------------------- Philox4x32-10 (Random123)
constexpr uint32_t kPhiloxM0 = 0xD2511F53u, kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u, kPhiloxW1 = 0xBB67AE85u;

// Stream tags (counter word 3).  Counter = {node, round, 0, stream}; draw k uses word k.
constexpr uint32_t kStreamLeader = 0x4C454144u;  // program.fs:173,211,250,316
constexpr uint32_t kStreamTopo = 0x544F504Fu;    // program.fs:309
constexpr uint32_t kStreamGossip = 0x474F5353u;  // program.fs:91
constexpr uint32_t kStreamPush = 0x50555348u;    // program.fs:112,126,142

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

__host__ __device__ __forceinline__ uint4 philox(uint32_t v, uint32_t r, uint32_t stream, uint64_t seed) {
    uint32_t c0 = v, c1 = r, c2 = 0u, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        // 32x32->64 products: one v_mad_u64_u32 each on gfx950 (a mul_hi + mul_lo pair otherwise)
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c0, p1 = (uint64_t)kPhiloxM1 * c2;
        c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        c1 = (uint32_t)p1;
        c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c3 = (uint32_t)p0;
        k0 += kPhiloxW0;
        k1 += kPhiloxW1;
    }
    return make_uint4(c0, c1, c2, c3);
}

// Word x of philox(); 32x32->64 products map to one v_mad_u64_u32 each on gfx950 (half the
// multiply instructions of separate mul_hi / mul_lo), and the dead last-round words drop out.
__host__ __device__ __forceinline__ uint32_t philox_x(uint32_t v, uint32_t r, uint32_t stream, uint64_t seed) {
    uint32_t c0 = v, c1 = r, c2 = 0u, c3 = stream;
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c0, p1 = (uint64_t)kPhiloxM1 * c2;
        c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        c1 = (uint32_t)p1;
        c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c3 = (uint32_t)p0;
        k0 += kPhiloxW0;
        k1 += kPhiloxW1;
    }
    return c0;
}

// Random().Next(0, n) replacement: floor(x * n / 2^32).
__host__ __device__ __forceinline__ uint32_t scale_draw(uint32_t x, uint32_t n) { return mulhi32(x, n); }

// Imp3D extra link of wired node v: Random().Next(0, nodes-1), i.e. [0, nodes-2] (program.fs:309).
// A pure function of (seed, v): no rank stores the link array, each recomputes what it needs.
__host__ __device__ __forceinline__ uint32_t link_of(uint64_t seed, uint32_t v, uint32_t nodes) {
    return scale_draw(philox_x(v, 0u, kStreamTopo, seed), nodes - 1u);
}

// ---------------------------------------------------------------- topology
enum Topology { kLine = 0, kFull = 1, kTwoD = 2, kImp3D = 3, kThreeD = 4 };

// Direction codes in the reference's neighbour ORDER (program.fs:295-310):
// 0:-x 1:+x 2:-y 3:+y 4:-z 5:+z 6:extra link.  7 = no message.
constexpr uint8_t kDirLink = 6, kDirNone = 7;

// Unsigned 32-bit division by a run-time constant with a precomputed multiplier
// (Granlund-Montgomery round-up method): q = (t + ((n - t) >> s1)) >> s2, t = mulhi(m, n).
struct FastDiv {
    uint32_t d, m, s1, s2;
};

__host__ __device__ inline FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;  // l = ceil(log2 d)
    FastDiv f;
    f.d = d;
    f.m = (uint32_t)((((1ull << l) - d) << 32) / d + 1ull);
    f.s1 = l < 1 ? l : 1u;
    f.s2 = l > 0 ? l - 1u : 0u;
    return f;
}

__host__ __device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    const uint32_t t = mulhi32(f.m, n);
    return (t + ((n - t) >> f.s1)) >> f.s2;
}

struct Geom {
    uint32_t actors;  // nodes + 1
    uint32_t wired;   // actors with grid neighbours: actors (line/2D) or nodes (Imp3D/3D)
    uint32_t gx, gy, gz;
    uint32_t plane;   // gx * gy
    uint32_t has_link;
    FastDiv dx, dy;   // division by gx and gy
};

// Presence mask of v's neighbour list in reference order; bit 6 = extra link.
// Imp3D/3D (program.fs:295-306): x>0, x<G-1 && i+1<nodes, y>0, y<G-1 && i+G<nodes, z>0,
// z<G-1 && i+G^2<nodes.  line/2D (program.fs:164-169, 244-247) are the gx = actors row.
__host__ __device__ __forceinline__ uint32_t presence(const Geom& g, uint32_t v) {
    if (v >= g.wired) return 0u;  // the isolated Imp3D actor `nodes` (program.fs:293)
    const uint32_t yz = fdiv(v, g.dx);
    const uint32_t x = v - yz * g.gx;
    const uint32_t z = fdiv(yz, g.dy);
    const uint32_t y = yz - z * g.gy;
    uint32_t m = 0;
    m |= (x > 0) ? 1u : 0u;
    m |= (x + 1 < g.gx && v + 1 < g.wired) ? 2u : 0u;
    m |= (y > 0) ? 4u : 0u;
    m |= (y + 1 < g.gy && v + g.gx < g.wired) ? 8u : 0u;
    m |= (z > 0) ? 16u : 0u;
    m |= (z + 1 < g.gz && v + g.plane < g.wired) ? 32u : 0u;
    m |= g.has_link ? 64u : 0u;
    return m;
}

// Index of the k-th set bit of m (k < popcount(m) <= 7: six grid directions + the extra link).
// Six predicated steps instead of a k-trip loop: no divergent branch in a wave.
__host__ __device__ __forceinline__ uint32_t kth_bit(uint32_t m, uint32_t k) {
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) m = i < k ? (m & (m - 1u)) : m;
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_ctz(m);
#else
    return (uint32_t)__builtin_ctz(m);
#endif
}

__host__ __device__ __forceinline__ uint32_t popc(uint32_t m) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__popc(m);
#else
    return (uint32_t)__builtin_popcount(m);
#endif
}

// Target actor of direction code d sent by v.
__host__ __device__ __forceinline__ uint32_t dir_target(const Geom& g, uint32_t v, uint32_t d, uint32_t link) {
    switch (d) {
    case 0: return v - 1u;
    case 1: return v + 1u;
    case 2: return v - g.gx;
    case 3: return v + g.gx;
    case 4: return v - g.plane;
    case 5: return v + g.plane;
    default: return link;
    }
}

}  // namespace gp
