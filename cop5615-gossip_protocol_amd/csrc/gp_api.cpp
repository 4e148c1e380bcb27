// gp_api.cpp — the C ABI of libgossip_hip.so (include/gossip_hip.h).
//
// Host orchestration only: sizes and geometry (program.fs:26-31, 150-313), device buffers,
// the round loop that replaces the actor dispatch (program.fs:82-146) and the ParentActor
// count (program.fs:44-63), and state read-back.  All per-actor work runs in gp_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gossip_hip.h"
#include "gp_kernels.h"

using namespace gp;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(x)                                                                                 \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess)                                                                      \
            return fail(GP_EHIP, "%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

constexpr uint32_t kNone = 0xFFFFFFFFu;

int sizes(int64_t n_arg, int32_t topology, int64_t* nodes, int64_t* actors, int64_t* grid) {
    if (n_arg < 1 || n_arg > 2147483647LL) return fail(GP_EINVAL, "numNodes must be in [1, 2^31-1], got %lld", (long long)n_arg);
    int64_t nd = n_arg, g = 0;
    switch (topology) {
    case GP_LINE:
    case GP_FULL: break;
    case GP_TWO_D:  // program.fs:228-229: round up to the nearest square
        g = (int64_t)std::ceil(std::sqrt((double)n_arg));
        nd = g * g;
        break;
    case GP_IMP3D:
    case GP_THREE_D: {  // program.fs:27-31 (cube rounding) and :268 (G from the raw argument)
        const double c = std::floor(std::pow((double)n_arg, 0.33334));
        nd = (int64_t)std::pow(c, 3.0);
        g = (int64_t)std::floor(std::pow((double)n_arg, 0.34));
        if (g * g * g < nd) return fail(GP_EINVAL, "grid %lld too small for %lld nodes", (long long)g, (long long)nd);
        break;
    }
    default: return fail(GP_EINVAL, "unknown topology %d", topology);
    }
    if (nd + 1 >= (int64_t)kNone) return fail(GP_EINVAL, "too many actors");
    *nodes = nd;
    *actors = nd + 1;
    *grid = g;
    return GP_OK;
}

struct Handle {
    gp_config cfg{};
    gp_layout lay{};
    Geom g{};
    bool full = false, generic = false, gossip = false;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int grid = 0;
    uint32_t span = 0;
    std::vector<void*> allocs;
    size_t dev_bytes = 0;
    // topology
    uint32_t* link = nullptr;
    uint32_t* rev_off = nullptr;
    uint32_t* rev_src = nullptr;
    uint32_t* lpos = nullptr;
    uint8_t* lcnt[2] = {nullptr, nullptr};   // gossip link slots
    double2* lmsg[2] = {nullptr, nullptr};   // push-sum link slots
    // push-sum
    double2* msg[2] = {nullptr, nullptr};
    uint8_t* dir[2] = {nullptr, nullptr};
    uint8_t* flags = nullptr;
    double2* frozen = nullptr;
    // gossip
    uint32_t* cnt = nullptr;
    uint8_t* gstate = nullptr;
    uint32_t* inc[2] = {nullptr, nullptr};
    // generic push-sum buckets
    uint32_t* bcnt[2] = {nullptr, nullptr};
    uint32_t* boff[2] = {nullptr, nullptr};
    uint32_t* slot[2] = {nullptr, nullptr};
    uint32_t* tgt = nullptr;
    uint32_t* pos = nullptr;
    uint32_t* scan_scratch = nullptr;
    // control
    unsigned long long* total = nullptr;
    int64_t total_cap = 0;
    uint32_t* parts = nullptr;
    double2* partials = nullptr;
    unsigned long long* h_trace = nullptr;  // pinned
    int64_t h_trace_cap = 0;
    int64_t next_kernel = 0;  // index of the next fused round kernel F(k)
    int64_t rounds = 0;       // rounds whose results are final
    int64_t completed = 0;
    bool converged = false;
    int64_t batch = 8;
    uint32_t ablate = 0;  // DEBUG: GP_ABLATE env var (cost attribution only; breaks results)
    // timing
    std::vector<hipEvent_t> kev;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;
    int64_t k_launches = 0;
    double k_total_ms = 0.0;

    ~Handle() {
        if (stream) (void)hipStreamSynchronize(stream);
        for (void* p : allocs) (void)hipFree(p);
        if (h_trace) (void)hipHostFree(h_trace);
        for (hipEvent_t e : kev) (void)hipEventDestroy(e);
        if (ev_a) (void)hipEventDestroy(ev_a);
        if (ev_b) (void)hipEventDestroy(ev_b);
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }

    template <class T>
    int alloc(T** p, size_t count) {
        void* q = nullptr;
        const size_t bytes = count * sizeof(T) + 64;  // padding: vectorised tail reads stay in bounds
        hipError_t e = hipMalloc(&q, bytes);
        if (e != hipSuccess) return fail(GP_ENOMEM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
        allocs.push_back(q);
        dev_bytes += bytes;
        *p = static_cast<T*>(q);
        return GP_OK;
    }

    Launch L() const { return Launch{grid, stream}; }

    RoundArgs args(uint32_t r) const {
        RoundArgs a{};
        a.g = g;
        a.seed = cfg.seed;
        a.r = r;
        a.target = (uint32_t)lay.nodes;
        a.full = full ? 1u : 0u;
        a.nodes = (uint32_t)lay.nodes;
        a.span = span;
        a.threshold = (uint32_t)cfg.gossip_threshold;
        a.delta = cfg.delta;
        a.term_limit = (uint32_t)cfg.term_limit;
        a.ablate = ablate;
        a.total = total;
        a.parts = parts;
        a.link = link;
        a.rev_off = rev_off;
        a.rev_src = rev_src;
        a.lpos = lpos;
        const int c = (int)(r & 1u), p = c ^ 1;
        a.lcnt_prev = lcnt[p];
        a.lcnt_cur = lcnt[c];
        a.lmsg_prev = lmsg[p];
        a.lmsg_cur = lmsg[c];
        a.msg_prev = msg[p];
        a.msg_cur = msg[c];
        a.dir_prev = dir[p];
        a.dir_cur = dir[c];
        a.flags = flags;
        a.frozen = frozen;
        a.cnt = cnt;
        a.gstate = gstate;
        a.inc_prev = inc[p];
        a.inc_cur = inc[c];
        a.bcnt_prev = bcnt[p];
        a.boff_prev = boff[p];
        a.slot_prev = slot[p];
        a.bcnt_cur = bcnt[c];
        a.tgt_cur = tgt;
        a.pos_cur = pos;
        return a;
    }
};

Handle* H(void* h) { return static_cast<Handle*>(h); }

int build_links(Handle* h) {
    const uint32_t nodes = (uint32_t)h->lay.nodes, A = h->g.actors;
    int rc;
    if ((rc = h->alloc(&h->link, nodes))) return rc;
    if ((rc = h->alloc(&h->rev_off, (size_t)A + 1))) return rc;
    if ((rc = h->alloc(&h->rev_src, nodes))) return rc;
    if (!h->generic) {  // pull kernels: sender-pushed link slots
        if ((rc = h->alloc(&h->lpos, nodes))) return rc;
        if (h->gossip) {
            if ((rc = h->alloc(&h->lcnt[0], nodes)) || (rc = h->alloc(&h->lcnt[1], nodes))) return rc;
        } else if ((rc = h->alloc(&h->lmsg[0], nodes)) || (rc = h->alloc(&h->lmsg[1], nodes))) {
            return rc;
        }
    }
    uint32_t *counts = nullptr, *scratch = nullptr;
    HIP_TRY(hipMalloc(&counts, ((size_t)A + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&scratch, scan_scratch_words(A) * sizeof(uint32_t)));
    const Launch l = h->L();
    hipError_t e = hipSuccess;
    launch_links(h->link, nodes, h->cfg.seed, l);
    e = hipMemsetAsync(counts, 0, ((size_t)A + 1) * sizeof(uint32_t), h->stream);
    if (e == hipSuccess) {
        launch_count(h->link, nodes, counts, l);
        launch_exclusive_scan(counts, h->rev_off, A, scratch, h->stream);
        e = hipMemsetAsync(counts, 0, ((size_t)A + 1) * sizeof(uint32_t), h->stream);
    }
    if (e == hipSuccess) {
        launch_rev_fill(h->link, nodes, h->rev_off, counts, h->rev_src, l);
        launch_sort_segments(h->rev_off, h->rev_src, A, l);  // ascending sources per destination
        if (h->lpos) launch_lpos(h->rev_src, nodes, h->lpos, l);
        e = hipStreamSynchronize(h->stream);
    }
    if (e == hipSuccess) e = hipGetLastError();
    (void)hipFree(counts);
    (void)hipFree(scratch);
    if (e != hipSuccess) return fail(GP_EHIP, "extra-link CSR build failed: %s", hipGetErrorString(e));
    h->lay.links = nodes;
    return GP_OK;
}

int ensure_trace(Handle* h, int64_t need) {
    if (need <= h->total_cap) return GP_OK;
    int64_t cap = std::max<int64_t>(h->total_cap * 2, 4096);
    while (cap < need) cap *= 2;
    unsigned long long* nt = nullptr;
    HIP_TRY(hipMalloc(&nt, (size_t)cap * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(nt, 0, (size_t)cap * sizeof(unsigned long long), h->stream));
    if (h->total) {
        HIP_TRY(hipMemcpyAsync(nt, h->total, (size_t)h->total_cap * sizeof(unsigned long long),
                               hipMemcpyDeviceToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        auto it = std::find(h->allocs.begin(), h->allocs.end(), (void*)h->total);
        if (it != h->allocs.end()) h->allocs.erase(it);
        h->dev_bytes -= (size_t)h->total_cap * sizeof(unsigned long long);
        (void)hipFree(h->total);
    }
    h->allocs.push_back(nt);
    h->dev_bytes += (size_t)cap * sizeof(unsigned long long);
    h->total = nt;
    h->total_cap = cap;
    return GP_OK;
}

int reset(Handle* h) {
    HIP_TRY(hipStreamSynchronize(h->stream));
    const size_t A = h->g.actors;
    HIP_TRY(hipMemsetAsync(h->total, 0, (size_t)h->total_cap * sizeof(unsigned long long), h->stream));
    HIP_TRY(hipMemsetAsync(h->parts, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t), h->stream));
    for (int i = 0; i < 2; ++i) {  // no link message in flight
        if (h->lcnt[i]) HIP_TRY(hipMemsetAsync(h->lcnt[i], 0, (size_t)h->lay.nodes, h->stream));
        if (h->lmsg[i]) launch_fill_empty_slots(h->lmsg[i], (size_t)h->lay.nodes, h->stream);
    }
    if (!h->gossip) {
        launch_ps_init(h->flags, h->g, h->full ? 1u : 0u, (uint32_t)h->cfg.term_init, h->L());
        if (h->generic) {
            HIP_TRY(hipMemsetAsync(h->bcnt[0], 0, A * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->bcnt[1], 0, A * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->tgt, 0xFF, A * sizeof(uint32_t), h->stream));
        } else {
            launch_fill_u8(h->dir[0], kDirNone, A, h->stream);
            launch_fill_u8(h->dir[1], kDirNone, A, h->stream);
        }
    } else {
        HIP_TRY(hipMemsetAsync(h->cnt, 0, A * sizeof(uint32_t), h->stream));
        HIP_TRY(hipMemsetAsync(h->gstate, 0, A, h->stream));
        if (h->generic) {
            HIP_TRY(hipMemsetAsync(h->inc[0], 0, A * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->inc[1], 0, A * sizeof(uint32_t), h->stream));
        } else {
            launch_fill_u8(h->dir[0], 0xFF, A, h->stream);
            launch_fill_u8(h->dir[1], 0xFF, A, h->stream);
        }
        // kick-off (program.fs:181/218/258/323): the leader holds one activation chain; for
        // "full" it is a CallChildActor, i.e. also its first receipt.
        const uint32_t L = (uint32_t)h->lay.leader;
        const uint8_t st = 1;
        HIP_TRY(hipMemcpyAsync(h->gstate + L, &st, 1, hipMemcpyHostToDevice, h->stream));
        if (h->full) {
            const uint32_t one = 1;
            HIP_TRY(hipMemcpyAsync(h->cnt + L, &one, sizeof one, hipMemcpyHostToDevice, h->stream));
        }
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipGetLastError());
    h->next_kernel = 0;
    h->rounds = 0;
    h->completed = 0;
    h->converged = false;
    h->batch = 8;
    return GP_OK;
}

const char* round_kernel_name(const Handle* h) {
    if (h->gossip) return h->generic ? "k_gs_push" : (h->g.has_link ? "k_gs_pull<true>" : "k_gs_pull<false>");
    return h->generic ? "k_ps_push_emit" : (h->g.has_link ? "k_ps_pull<true>" : "k_ps_pull<false>");
}

// Compulsory HBM bytes of one launch of the dominant round kernel for its data layout
// (every array element it must touch, touched once); DESIGN.md §5.
//   push-sum pull: held (S,W) read 16 + message write 16 + flags read 1 + direction byte read
//   1 (own row; neighbour rows re-read from cache) + direction write 1 per participant; Imp3D
//   adds the link CSR offsets (4 per actor) and per link slot the 16-byte slot + 4-byte source.
//   The link scatter pass (a separate kernel) is not included.
//   gossip pull: state byte read 1 + direction byte read 1 + write 1 (+ count r/w 8 on the
//   receipts, not modelled); Imp3D adds offsets 4 per actor and 1 per link slot.
double bytes_per_round(const Handle* h) {
    const double P = (double)h->lay.participants, A = (double)h->lay.actors, links = (double)h->lay.links;
    if (h->gossip) {
        if (h->generic) return P * (4 + 4 + 1 + 1) + P * 2 * 4;  // cnt r/w, inc r, state r/w, 2 atomics
        return P * (1 + 1 + 1) + (h->g.has_link ? 4 * A + 1 * links : 0);
    }
    if (h->generic) return P * (16 + 16 + 16 + 1 + 4 + 4 + 4 + 4 + 4);
    double b = P * (16 + 16 + 1 + 1 + 1);
    if (h->g.has_link) b += 4 * A + links * (16 + 4);
    return b;
}

// The dominant round kernel F(k) (timed under GP_FLAG_KERNEL_TIMING) ...
void launch_main(Handle* h, int64_t k) {
    const RoundArgs a = h->args((uint32_t)k);
    const Launch l = h->L();
    if (h->gossip) {
        if (h->generic) launch_gs_push(a, l);  // adds into inc_cur, consumed (zeroed) by F(k+1)
        else launch_gs_pull(a, l);
    } else if (h->generic) {
        launch_ps_push_emit(a, l);
    } else {
        launch_ps_pull(a, l);
    }
}

// ... and the passes that complete round k after it (link scatter; bucket scan + fill).
void launch_aux(Handle* h, int64_t k) {
    const uint32_t r = (uint32_t)k;
    const RoundArgs a = h->args(r);
    const Launch l = h->L();
    if (h->gossip) {
        if (!h->generic && h->g.has_link) launch_gs_link_scatter(a, l);
    } else if (h->generic) {
        const int c = (int)(r & 1u);
        launch_exclusive_scan(h->bcnt[c], h->boff[c], h->g.actors, h->scan_scratch, h->stream);
        launch_ps_push_fill(a, h->slot[c], h->boff[c], l);
    } else if (h->g.has_link) {
        launch_ps_link_scatter(a, l);
    }
}

int launch_round(Handle* h, int64_t k) {
    launch_main(h, k);
    launch_aux(h, k);
    return GP_OK;
}

int step(Handle* h, int64_t max_rounds, gp_status* st) {
    if (max_rounds < 0) return fail(GP_EINVAL, "max_rounds < 0");
    const bool timing = (h->cfg.flags & GP_FLAG_KERNEL_TIMING) != 0;
    HIP_TRY(hipEventRecord(h->ev_a, h->stream));
    const int64_t goal = h->rounds + max_rounds;
    while (!h->converged && h->rounds < goal) {
        const int64_t B = std::min<int64_t>(h->batch, goal - h->rounds);
        int rc;
        if ((rc = ensure_trace(h, h->next_kernel + B + 4))) return rc;
        if (h->gossip && h->next_kernel == 0) {  // F(0) only emits round 0
            if ((rc = launch_round(h, 0))) return rc;
            h->next_kernel = 1;
        }
        if (timing && (int64_t)h->kev.size() < 2 * B) {
            const size_t old = h->kev.size();
            h->kev.resize((size_t)(2 * B));
            for (size_t i = old; i < h->kev.size(); ++i) HIP_TRY(hipEventCreate(&h->kev[i]));
        }
        for (int64_t i = 0; i < B; ++i) {
            if (timing) HIP_TRY(hipEventRecord(h->kev[2 * i], h->stream));
            launch_main(h, h->next_kernel + i);
            if (timing) HIP_TRY(hipEventRecord(h->kev[2 * i + 1], h->stream));
            launch_aux(h, h->next_kernel + i);
        }
        h->next_kernel += B;
        // total[] of the last round this batch applied (F(k) applies round k, or k-1 for gossip)
        launch_finalize(h->total, h->parts, h->next_kernel - (h->gossip ? 2 : 1), h->stream);
        HIP_TRY(hipGetLastError());
        // total[] entries of the rounds completed by this batch
        if (B > h->h_trace_cap) {
            if (h->h_trace) (void)hipHostFree(h->h_trace);
            h->h_trace = nullptr;
            HIP_TRY(hipHostMalloc((void**)&h->h_trace, (size_t)B * sizeof(unsigned long long), 0));
            h->h_trace_cap = B;
        }
        HIP_TRY(hipMemcpyAsync(h->h_trace, h->total + h->rounds, (size_t)B * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        int64_t real = B;
        for (int64_t i = 0; i < B; ++i) {
            if ((int64_t)h->h_trace[i] >= h->lay.nodes) {  // ParentActor: count = AllNodes
                real = i + 1;
                h->converged = true;
                break;
            }
        }
        h->completed = (int64_t)h->h_trace[real - 1];
        h->rounds += real;
        if (timing) {
            for (int64_t i = 0; i < real; ++i) {
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, h->kev[2 * i], h->kev[2 * i + 1]));
                h->k_total_ms += ms;
            }
            h->k_launches += real;
        }
        h->batch = std::min<int64_t>(h->batch * 2, 256);
    }
    HIP_TRY(hipEventRecord(h->ev_b, h->stream));
    HIP_TRY(hipEventSynchronize(h->ev_b));
    if (st) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev_a, h->ev_b));
        std::memset(st, 0, sizeof *st);
        st->round = h->rounds;
        st->completed = h->completed;
        st->converged = h->converged ? 1 : 0;
        st->device_ms = ms;
        if (!h->gossip) {
            const int64_t last = h->rounds - 1;
            RoundArgs a = h->args((uint32_t)std::max<int64_t>(last, 0));
            a.msg_prev = h->msg[last >= 0 ? (last & 1) : 0];
            a.dir_prev = h->generic ? nullptr : h->dir[last >= 0 ? (last & 1) : 0];
            launch_ps_sums(a, last >= 0 ? 1u : 0u, h->partials, h->L());
            std::vector<double2> part((size_t)h->grid);
            HIP_TRY(hipMemcpyAsync(part.data(), h->partials, part.size() * sizeof(double2), hipMemcpyDeviceToHost,
                                   h->stream));
            HIP_TRY(hipStreamSynchronize(h->stream));
            for (const double2& p : part) {
                st->sum_s += p.x;
                st->sum_w += p.y;
            }
        }
    }
    return GP_OK;
}

int check_range(const Handle* h, int64_t first, int64_t count) {
    if (first < 0 || count < 0 || first + count > (int64_t)h->g.actors)
        return fail(GP_EINVAL, "range [%lld, %lld) outside 0..%u", (long long)first, (long long)(first + count), h->g.actors);
    return GP_OK;
}

template <class T>
int copy_slice(const Handle* h, std::vector<T>& out, const T* src, int64_t first, int64_t count) {
    out.resize((size_t)count);
    if (count) HIP_TRY(hipMemcpy(out.data(), src + first, (size_t)count * sizeof(T), hipMemcpyDeviceToHost));
    (void)h;
    return GP_OK;
}

}  // namespace

extern "C" {

int gp_abi_version(void) { return GP_ABI_VERSION; }

int gp_sizes(int64_t n_arg, int32_t topology, int64_t* nodes, int64_t* actors, int64_t* grid) {
    if (!nodes || !actors || !grid) return fail(GP_EINVAL, "null output pointer");
    return sizes(n_arg, topology, nodes, actors, grid);
}

int gp_create(const gp_config* cfg, gp_layout* out, void** handle) {
    if (!cfg || !handle) return fail(GP_EINVAL, "null argument");
    *handle = nullptr;
    if (cfg->algo != GP_GOSSIP && cfg->algo != GP_PUSHSUM) return fail(GP_EINVAL, "unknown algorithm %d", cfg->algo);
    if (cfg->term_limit < 1 || cfg->term_limit > 15 || cfg->term_init < 0 || cfg->term_init >= cfg->term_limit)
        return fail(GP_EINVAL, "term_init/term_limit out of range");
    if (cfg->gossip_threshold < 0) return fail(GP_EINVAL, "gossip_threshold < 0");
    int64_t nodes, actors, grid;
    int rc = sizes(cfg->n_arg, cfg->topology, &nodes, &actors, &grid);
    if (rc) return rc;
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) return fail(GP_EINVAL, "device %d not present (%d devices)", cfg->device, ndev);
    HIP_TRY(hipSetDevice(cfg->device));

    Handle* h = new Handle();
    h->cfg = *cfg;
    h->lay.nodes = nodes;
    h->lay.actors = actors;
    h->lay.grid = grid;
    h->gossip = cfg->algo == GP_GOSSIP;
    h->full = cfg->topology == GP_FULL;
    h->generic = h->full || (cfg->flags & GP_FLAG_GENERIC);
    Geom& g = h->g;
    g.actors = (uint32_t)actors;
    if (cfg->topology == GP_IMP3D || cfg->topology == GP_THREE_D) {
        g.gx = g.gy = g.gz = (uint32_t)grid;
        g.plane = (uint32_t)(grid * grid);
        g.wired = (uint32_t)nodes;  // actor `nodes` is isolated (program.fs:293)
        g.has_link = cfg->topology == GP_IMP3D ? 1u : 0u;
    } else {  // line / 2D / full: one row of `actors`
        g.gx = (uint32_t)actors;
        g.gy = g.gz = 1;
        g.plane = (uint32_t)actors;
        g.wired = (uint32_t)actors;
        g.has_link = 0;
    }
    g.dx = make_fastdiv(g.gx);
    g.dy = make_fastdiv(g.gy);
    // leader = Random().Next(0, nodes)  (program.fs:173/211/250/316)
    h->lay.leader = scale_draw(philox(0u, 0u, kStreamLeader, cfg->seed).x, (uint32_t)nodes);
    int64_t part = 0;
    if (h->full) part = actors;
    else
        for (int64_t v = 0; v < actors; ++v) part += presence(g, (uint32_t)v) != 0u;
    h->lay.participants = part;
    if (const char* ab = std::getenv("GP_ABLATE")) h->ablate = (uint32_t)std::strtoul(ab, nullptr, 0);
    h->grid = grid_for(g.actors);
    if (const char* gg = std::getenv("GP_GRID")) {  // tuning override (rounded to a multiple of 8)
        const long v = std::strtol(gg, nullptr, 0);
        if (v >= 8) h->grid = (int)((v + 7) / 8 * 8);
    }
    h->span = span_for(g.actors, h->grid);

    auto bail = [&](int code) {
        delete h;
        return code;
    };
    if (cfg->stream) {
        h->stream = (hipStream_t)cfg->stream;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
        if (e != hipSuccess) return bail(fail(GP_EHIP, "hipStreamCreate: %s", hipGetErrorString(e)));
        h->own_stream = true;
    }
    if (hipEventCreate(&h->ev_a) != hipSuccess || hipEventCreate(&h->ev_b) != hipSuccess)
        return bail(fail(GP_EHIP, "hipEventCreate failed"));

    const size_t A = (size_t)actors;
    if (h->gossip) {
        if ((rc = h->alloc(&h->cnt, A)) || (rc = h->alloc(&h->gstate, A))) return bail(rc);
        if (h->generic) {
            if ((rc = h->alloc(&h->inc[0], A)) || (rc = h->alloc(&h->inc[1], A))) return bail(rc);
        } else if ((rc = h->alloc(&h->dir[0], A)) || (rc = h->alloc(&h->dir[1], A))) {
            return bail(rc);
        }
    } else {
        if ((rc = h->alloc(&h->msg[0], A)) || (rc = h->alloc(&h->msg[1], A)) || (rc = h->alloc(&h->flags, A)) ||
            (rc = h->alloc(&h->frozen, A)) || (rc = h->alloc(&h->partials, (size_t)h->grid)))
            return bail(rc);
        if (h->generic) {
            for (int i = 0; i < 2; ++i)
                if ((rc = h->alloc(&h->bcnt[i], A)) || (rc = h->alloc(&h->boff[i], A + 1)) ||
                    (rc = h->alloc(&h->slot[i], A)))
                    return bail(rc);
            if ((rc = h->alloc(&h->tgt, A)) || (rc = h->alloc(&h->pos, A)) ||
                (rc = h->alloc(&h->scan_scratch, scan_scratch_words((uint32_t)A))))
                return bail(rc);
        } else if ((rc = h->alloc(&h->dir[0], A)) || (rc = h->alloc(&h->dir[1], A))) {
            return bail(rc);
        }
    }
    if (g.has_link && (rc = build_links(h))) return bail(rc);
    if ((rc = h->alloc(&h->parts, (size_t)kPartRing * kParts * kPartStride))) return bail(rc);
    if ((rc = ensure_trace(h, 4096))) return bail(rc);
    if ((rc = reset(h))) return bail(rc);
    h->lay.device_bytes = (int64_t)h->dev_bytes;
    if (out) *out = h->lay;
    *handle = h;
    return GP_OK;
}

int gp_reset(void* handle) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    return reset(H(handle));
}

int gp_step(void* handle, int64_t max_rounds, gp_status* st) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    return step(H(handle), max_rounds, st);
}

int gp_read_gossip(void* handle, int64_t first, int64_t count, uint32_t* cnt, uint8_t* flags) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (!h->gossip) return fail(GP_ESTATE, "not a gossip handle");
    int rc = check_range(h, first, count);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (cnt && count) HIP_TRY(hipMemcpy(cnt, h->cnt + first, (size_t)count * 4, hipMemcpyDeviceToHost));
    if (flags && count) HIP_TRY(hipMemcpy(flags, h->gstate + first, (size_t)count, hipMemcpyDeviceToHost));
    return GP_OK;
}

int gp_read_pushsum(void* handle, int64_t first, int64_t count, double* S, double* W, uint8_t* flags) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
    int rc = check_range(h, first, count);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    std::vector<uint8_t> f;
    std::vector<double2> fr, ms;
    if ((rc = copy_slice(h, f, (const uint8_t*)h->flags, first, count))) return rc;
    if ((rc = copy_slice(h, fr, (const double2*)h->frozen, first, count))) return rc;
    const int64_t last = h->rounds - 1;
    if (last >= 0 && (rc = copy_slice(h, ms, (const double2*)h->msg[last & 1], first, count))) return rc;
    for (int64_t i = 0; i < count; ++i) {
        const uint32_t v = (uint32_t)(first + i);
        const bool part = h->full || presence(h->g, v) != 0u;
        double2 held = make_double2((double)v, 1.0);  // InitializeVariables (program.fs:107-108, :78)
        if (part && (f[i] & 16u)) held = fr[i];
        else if (part && last >= 0) held = ms[i];
        if (S) S[i] = held.x;
        if (W) W[i] = held.y;
        if (flags) flags[i] = f[i];
    }
    return GP_OK;
}

int gp_read_messages(void* handle, int64_t first, int64_t count, uint32_t* dst, double* s, double* w) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
    int rc = check_range(h, first, count);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    const int64_t last = h->rounds - 1;
    std::vector<uint32_t> t((size_t)count, kNone);
    std::vector<double2> ms;
    if (last >= 0) {
        if ((rc = copy_slice(h, ms, (const double2*)h->msg[last & 1], first, count))) return rc;
        if (h->generic) {
            if ((rc = copy_slice(h, t, (const uint32_t*)h->tgt, first, count))) return rc;
        } else {
            std::vector<uint8_t> d;
            std::vector<uint32_t> lk;
            if ((rc = copy_slice(h, d, (const uint8_t*)h->dir[last & 1], first, count))) return rc;
            if (h->g.has_link) {
                const int64_t n = std::max<int64_t>(0, std::min<int64_t>(first + count, h->lay.nodes) - first);
                lk.assign((size_t)count, 0u);
                if (n > 0) HIP_TRY(hipMemcpy(lk.data(), h->link + first, (size_t)n * 4, hipMemcpyDeviceToHost));
            }
            for (int64_t i = 0; i < count; ++i)
                t[i] = d[i] == kDirNone ? kNone
                                        : dir_target(h->g, (uint32_t)(first + i), d[i], h->g.has_link ? lk[i] : 0u);
        }
    }
    for (int64_t i = 0; i < count; ++i) {
        if (dst) dst[i] = t[i];
        if (s) s[i] = t[i] == kNone ? 0.0 : ms[i].x;
        if (w) w[i] = t[i] == kNone ? 0.0 : ms[i].y;
    }
    return GP_OK;
}

int gp_read_trace(void* handle, int64_t first_round, int64_t count, int64_t* completed) {
    if (!handle || !completed) return fail(GP_EINVAL, "null argument");
    Handle* h = H(handle);
    if (first_round < 0 || count < 0 || first_round + count > h->rounds)
        return fail(GP_EINVAL, "trace range outside the %lld executed rounds", (long long)h->rounds);
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (count)
        HIP_TRY(hipMemcpy(completed, h->total + first_round, (size_t)count * sizeof(int64_t), hipMemcpyDeviceToHost));
    return GP_OK;
}

int gp_neighbors(void* handle, int64_t v, uint32_t* out, int32_t cap) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (v < 0 || v >= (int64_t)h->g.actors) return fail(GP_EINVAL, "actor %lld out of range", (long long)v);
    if (h->full) {  // program.fs:201-206: every j != i in ascending order
        const int64_t d = h->lay.nodes;
        for (int64_t k = 0; k < d && k < cap; ++k) out[k] = (uint32_t)(k + (k >= v));
        return (int)d;
    }
    const uint32_t m = presence(h->g, (uint32_t)v);
    uint32_t lk = 0;
    if (m & 64u) HIP_TRY(hipMemcpy(&lk, h->link + v, 4, hipMemcpyDeviceToHost));
    int d = 0;
    for (uint32_t c = 0; c < 7; ++c)
        if (m & (1u << c)) {
            if (d < cap) out[d] = dir_target(h->g, (uint32_t)v, c, lk);
            ++d;
        }
    return d;
}

int gp_kernel_stats(void* handle, gp_kstats* out, int32_t reset_counters) {
    if (!handle || !out) return fail(GP_EINVAL, "null argument");
    Handle* h = H(handle);
    std::memset(out, 0, sizeof *out);
    out->launches = h->k_launches;
    out->total_ms = h->k_total_ms;
    out->avg_ms = h->k_launches ? h->k_total_ms / (double)h->k_launches : 0.0;
    out->bytes_per_launch = bytes_per_round(h);
    std::snprintf(out->kernel, sizeof out->kernel, "%s", round_kernel_name(h));
    if (reset_counters) {
        h->k_launches = 0;
        h->k_total_ms = 0.0;
    }
    return GP_OK;
}

void gp_destroy(void* handle) { delete H(handle); }

const char* gp_last_error(void) { return g_err.c_str(); }

}  // extern "C"
