// Error paths of gp_create under the host AddressSanitizer / LeakSanitizer (host code only:
// built with -Xarch_host -fsanitize=address).  Every failing create must return its error code
// and free what it built; LeakSanitizer reports anything left at exit.
//   abi_errors          the cases that need no GPU (every platform)
//   abi_errors gpu      also the multi-GPU group's failure paths after shards exist (one GPU)
#include <cstdio>
#include <cstring>

#include "gossip_hip.h"

static int failures = 0;

static gp_config base(int64_t n, int32_t topo, int32_t algo) {
    gp_config c;
    std::memset(&c, 0, sizeof c);
    c.n_arg = n;
    c.topology = topo;
    c.algo = algo;
    c.seed = 1;
    c.delta = 1e-10;
    c.gossip_threshold = 10;
    c.term_init = 1;
    c.term_limit = 3;
    return c;
}

static void expect(const char* what, const gp_config& c, int want_a, int want_b) {
    void* h = reinterpret_cast<void*>(0x1);
    const int rc = gp_create(&c, nullptr, &h);
    const bool ok = (rc == want_a || rc == want_b) && h == nullptr;
    std::printf("%-48s rc=%d handle=%s %s (%s)\n", what, rc, h ? "set" : "null", ok ? "ok" : "FAIL", gp_last_error());
    if (!ok) ++failures;
    if (rc == GP_OK && h) gp_destroy(h);
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
    gp_config c = base(1000, GP_IMP3D, GP_PUSHSUM);
    c.num_gpus = 17;  // above kMaxWorld
    expect("num_gpus 17", c, GP_EINVAL, GP_EINVAL);
    c.num_gpus = 2;
    c.device = 40;  // no such device (GP_EHIP where the runtime finds no GPU at all)
    expect("num_gpus 2 from device 40", c, GP_EINVAL, GP_EHIP);
    c = base(0, GP_LINE, GP_GOSSIP);
    expect("numNodes 0", c, GP_EINVAL, GP_EINVAL);
    if (gpu) {
        // shards exist before the failure: 8 ranks of a 4-plane graph fail in the partition,
        // 2 ranks on device 0 and 1 fail at device 1 (one-GPU box) or build and are destroyed
        c = base(200, GP_THREE_D, GP_PUSHSUM);
        c.num_gpus = 8;
        c.flags = GP_FLAG_ONE_DEVICE;
        expect("8 shards of a 4-plane graph", c, GP_EINVAL, GP_EINVAL);
        c = base(100000, GP_IMP3D, GP_PUSHSUM);
        c.num_gpus = 4;
        c.flags = GP_FLAG_ONE_DEVICE;
        void* h = nullptr;
        int rc = gp_create(&c, nullptr, &h);  // a whole group, built and destroyed
        gp_status st;
        if (rc == GP_OK) rc = gp_step(h, 5, &st);
        std::printf("%-48s rc=%d %s\n", "4 shards on one device, 5 rounds", rc, rc == GP_OK ? "ok" : "FAIL");
        if (rc != GP_OK) ++failures;
        gp_destroy(h);
        c = base(100000, GP_IMP3D, GP_PUSHSUM);
        c.flags = GP_FLAG_GENERIC;  // a shard refuses the generic path after the group exists
        c.num_gpus = 2;
        c.flags |= GP_FLAG_ONE_DEVICE;
        expect("2 generic shards", c, GP_EINVAL, GP_EINVAL);
    }
    std::printf("%s\n", failures ? "FAILED" : "done");
    return failures ? 1 : 0;
}
