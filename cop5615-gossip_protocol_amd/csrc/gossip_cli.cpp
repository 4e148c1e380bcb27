// gossip_cli.cpp — drop-in replacement for the reference's program entry point.
//
//   gossip numNodes topology algorithm [--seed S] [--max-rounds R] [--device D] [--gpus N]
//          [--mode round] [--verbose] [--trace FILE]
//
// Same positional contract as /root/reference/program.fs:19-21 (argv[1] = numNodes,
// argv[2] = topology "line" | "full" | "2D" | "Imp3D" (+ build-defined "3D"), argv[3] =
// algorithm "gossip" | "push-sum"), the same banners (program.fs:180,186,217,222,257,262,
// 322,327) and the same final report (program.fs:51-52 / 58-59).  The Akka actor system is
// replaced by libgossip_hip.so.  stdout is exactly the reference's lines — the banner, the
// separator, `Convergence Time: %f ms` — plus one `Rounds: N` line; --verbose adds the layout
// (actors, nodes, leader) after the banner.
//
// --gpus N runs the one graph over N GPUs of this process (gp_config.num_gpus: node-range
// shards, RCCL exchange inside the library; bit-exact with several shards on one GPU, but an
// exchange between physical GPUs is untested so far: README.md).  --mode round is the synchronous-round engine (the
// only mode); the reference's asynchronous actor execution is not part of the engine: its
// statistical restatement is test infrastructure (oracle/gp_async.c), so --mode async is
// refused.
//
// Deliberate deviations: an invalid algorithm or topology exits with status 2
// instead of hanging at Console.ReadLine() (program.fs:188-189, 331-334); a run that hits
// --max-rounds without converging exits with status 3.
//
// --trace FILE writes the ParentActor's count after every round as CSV (round,completed): the
// convergence curve behind report.pdf p.3-4, at any size.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gossip_hip.h"

namespace {

int topology_code(const std::string& t) {  // case-sensitive, as program.fs:151,191,227,267
    if (t == "line") return GP_LINE;
    if (t == "full") return GP_FULL;
    if (t == "2D") return GP_TWO_D;
    if (t == "Imp3D") return GP_IMP3D;
    if (t == "3D") return GP_THREE_D;
    return -1;
}

const char* banner(int topo, int algo) {
    if (topo == GP_LINE) return algo == GP_GOSSIP ? "Starting Protocol Gossip" : "Starting Push Sum Protocol for Line";
    return algo == GP_GOSSIP ? "Use Of Gossip Protocol" : "Push Sum Started";
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr,
                     "usage: %s numNodes topology algorithm [--seed S] [--max-rounds R] [--device D] [--gpus N] "
                     "[--mode round] [--verbose] [--trace FILE]\n"
                     "  --gpus N: one graph over N GPUs of this process (RCCL inside the library; an exchange\n"
                     "            between physical GPUs has not been tested yet, see README.md)\n",
                     argv[0]);
        return 2;
    }
    gp_config cfg{};
    cfg.n_arg = std::strtoll(argv[1], nullptr, 10);
    const std::string topology = argv[2], protocol = argv[3];
    cfg.seed = 1;
    cfg.delta = 1e-10;  // 10.0 ** -10.0 (program.fs:187)
    cfg.gossip_threshold = 10;
    cfg.term_init = 1;
    cfg.term_limit = 3;
    long long max_rounds = 1LL << 40;
    bool verbose = false;
    const char* trace_path = nullptr;
    for (int i = 4; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--seed" && i + 1 < argc) cfg.seed = std::strtoull(argv[++i], nullptr, 10);
        else if (a == "--max-rounds" && i + 1 < argc) max_rounds = std::strtoll(argv[++i], nullptr, 10);
        else if (a == "--device" && i + 1 < argc) cfg.device = std::atoi(argv[++i]);
        else if (a == "--gpus" && i + 1 < argc) cfg.num_gpus = std::atoi(argv[++i]);
        else if (a == "--verbose") verbose = true;
        else if (a == "--trace" && i + 1 < argc) trace_path = argv[++i];
        else if (a == "--mode" && i + 1 < argc) {
            const std::string m = argv[++i];
            if (m != "round") {
                std::fprintf(stderr, "--mode %s: only the synchronous-round engine (--mode round) is built; the "
                                     "asynchronous actor model is a CPU test model (oracle/gp_async.c)\n",
                             m.c_str());
                return 2;
            }
        } else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    const int topo = topology_code(topology);
    if (topo < 0) {  // program.fs:331 `| _ -> ()` (the reference then hangs)
        std::fprintf(stderr, "unknown topology '%s'\n", topology.c_str());
        return 2;
    }
    if (protocol != "gossip" && protocol != "push-sum") {  // program.fs:188-189, 224-225, 264-265
        std::printf(topo == GP_TWO_D ? "Invalid: Please enter a proper protocol or topology\n"
                                     : "Invalid:Please enter a proper protocol or topology\n");
        return 2;
    }
    cfg.topology = topo;
    cfg.algo = protocol == "gossip" ? GP_GOSSIP : GP_PUSHSUM;

    void* h = nullptr;
    gp_layout lay{};
    if (gp_create(&cfg, &lay, &h) != GP_OK) {
        std::fprintf(stderr, "gp_create: %s\n", gp_last_error());
        return 1;
    }
    std::printf("%s\n", banner(topo, cfg.algo));
    if (verbose)
        std::printf("actors %lld (nodes %lld), leader %lld, %d GPU(s)\n", (long long)lay.actors, (long long)lay.nodes,
                    (long long)lay.leader, cfg.num_gpus > 1 ? cfg.num_gpus : 1);
    gp_status st{};
    if (gp_step(h, max_rounds, &st) != GP_OK) {
        std::fprintf(stderr, "gp_step: %s\n", gp_last_error());
        gp_destroy(h);
        return 1;
    }
    int rc = 0;
    if (st.converged) {
        std::printf("-----------------------------------------------------------\n");
        std::printf("Convergence Time: %f ms\n", st.device_ms);
        std::printf("Rounds: %lld\n", (long long)st.round);
    } else {
        std::printf("Not converged after %lld rounds (%lld of %lld reported), %f ms\n", (long long)st.round,
                    (long long)st.completed, (long long)lay.nodes, st.device_ms);
        rc = 3;
    }
    if (trace_path) {
        std::vector<int64_t> done((size_t)st.round);
        FILE* f = std::fopen(trace_path, "w");
        if (!f || (st.round && gp_read_trace(h, 0, st.round, done.data()) != GP_OK)) {
            std::fprintf(stderr, "--trace %s: %s\n", trace_path, f ? gp_last_error() : std::strerror(errno));
            if (f) std::fclose(f);
            gp_destroy(h);
            return 1;
        }
        std::fprintf(f, "round,completed\n");
        for (int64_t r = 0; r < st.round; ++r) std::fprintf(f, "%lld,%lld\n", (long long)r, (long long)done[(size_t)r]);
        std::fclose(f);
    }
    gp_destroy(h);
    return rc;
}
