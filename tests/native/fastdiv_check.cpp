// Host check of gp::FastDiv (magic-number division used by presence()) against '/' and of
// presence() against the program.fs:295-306 rules written with plain division.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "gp_common.h"

int main() {
    std::mt19937_64 rng(12345);
    const uint32_t divs[] = {1, 2, 3, 5, 7, 10, 13, 50, 239, 524, 1148, 1481, 57121, 1317904, 97337, 100490,
                             1000001, 2147483647u, 2147483648u, 4294967295u};
    for (uint32_t d : divs) {
        const gp::FastDiv f = gp::make_fastdiv(d);
        for (int i = 0; i < 200000; ++i) {
            uint32_t n = (uint32_t)rng();
            if (i < 1000) n = (uint32_t)i;
            if (i >= 1000 && i < 2000) n = 0xFFFFFFFFu - (uint32_t)(i - 1000);
            if (gp::fdiv(n, f) != n / d) {
                std::printf("FAIL d=%u n=%u got %u want %u\n", d, n, gp::fdiv(n, f), n / d);
                return 1;
            }
        }
    }
    // presence() vs the reference rules for a partial-last-layer slab (G=6, nodes=125; G=239 slab)
    const uint32_t Gs[] = {2, 6, 10, 239};
    const uint32_t Ns[] = {8, 125, 1000, 9938375};
    for (int t = 0; t < 4; ++t) {
        gp::Geom g{};
        g.actors = Ns[t] + 1;
        g.wired = Ns[t];
        g.gx = g.gy = g.gz = Gs[t];
        g.plane = Gs[t] * Gs[t];
        g.has_link = 1;
        g.dx = gp::make_fastdiv(g.gx);
        g.dy = gp::make_fastdiv(g.gy);
        for (uint32_t i = 0; i < g.actors; i += (t == 3 ? 7 : 1)) {
            uint32_t want = 0;
            if (i < g.wired) {
                const uint32_t G = Gs[t], x = i % G, y = (i / G) % G, z = i / (G * G), n = Ns[t];
                want |= x > 0 ? 1 : 0;
                want |= (x < G - 1 && i + 1 < n) ? 2 : 0;
                want |= y > 0 ? 4 : 0;
                want |= (y < G - 1 && i + G < n) ? 8 : 0;
                want |= z > 0 ? 16 : 0;
                want |= (z < G - 1 && i + G * G < n) ? 32 : 0;
                want |= 64;
            }
            if (gp::presence(g, i) != want) {
                std::printf("FAIL presence G=%u i=%u got %u want %u\n", Gs[t], i, gp::presence(g, i), want);
                return 1;
            }
        }
    }
    std::printf("ok\n");
    return 0;
}
