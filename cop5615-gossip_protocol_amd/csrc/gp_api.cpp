// gp_api.cpp — the C ABI of libgossip_hip.so (include/gossip_hip.h).
//
// Host orchestration only: sizes and geometry (program.fs:26-31, 150-313), device buffers,
// the round loop that replaces the actor dispatch (program.fs:82-146) and the ParentActor
// count (program.fs:44-63), and state read-back.  All per-actor work runs in gp_kernels.hip.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: RCCL itself is loaded on first use (Rccl below)

// Quiet-wave skipping of the push-sum round kernel (one GPU, from kQuietMinActors actors or under
// GP_FLAG_QUIET_WAVES): the marks are kept once this percentage of the nodes has converged (0:
// off; A/B knob).  On small graphs the round is latency-bound and the marks only add work.
#ifndef GP_ACT_PCT
#define GP_ACT_PCT 99
#endif
constexpr uint32_t kQuietMinActors = 1u << 20;
// Shards run their rounds in pieces from this many actors on every rank (GP_FLAG_PIECES):
// a piece's launches cost a few microseconds each, which 12.5M-actor ranks (100M / 8) do not earn back
// (dense rank-round 0.43 -> 0.68 ms in pieces) and 125M-actor ranks (C5 / 8) do (+2.6% of kernel time
// for an exchange of 326 MB per rank-round hidden but for its last piece).
constexpr int64_t kPieceMinActors = 1 << 25;
// Full gossip done bitmap: one bit per actor, then its summary (one bit per 32-actor word).
constexpr uint32_t kDsumMinActors = 1u << 25;  // the summary is used from here (dbits > an L2)
// Full gossip on one GPU: the receipt tally (gp_kernels.h GsTally) is built from this many actors
// and used in a round after one that emitted at least actors / kTallyThrDiv chains (scaled by
// the share of nodes not done).  With the batched placement 8 rather than 2: C4 66.7 -> 61.6 ms,
// 10M +2% (profiles/round3/c4_scatter/cli_tally_thr.txt).
constexpr size_t kTallyMinActors = 1u << 20;
// Small Imp3D push-sum graphs on one GPU (no quiet marks): link senders also write their message into
// the receiver's CSR slot (k_ps_pull<3>)
constexpr uint32_t kSlotMsgMaxActors = 1u << 18;
// Small one-GPU line grids (line / 2D push-sum) below this many actors (the quiet tail's threshold)
// run up to kTileMaxNR rounds per launch
// (k_ps_tile); GP_FLAG_ONE_ROUND keeps one round per launch.
constexpr uint32_t kTileMaxActors = 1u << 20;
constexpr int64_t kMaxBatch = 256;       // rounds per gp_step batch at most
constexpr size_t kTinyMaxActors = 8192;  // gossip in one workgroup's LDS (k_gs_tiny, <= kTinyActors)
constexpr size_t kTinyGridMaxActors = 4096;  // ... for the grid topologies too (else k_gs_pull)
#ifndef GP_TALLY_THR_DIV
#define GP_TALLY_THR_DIV 8
#endif
constexpr size_t kTallyThrDiv = GP_TALLY_THR_DIV;
#ifndef GP_SPARSE_RAMP
#define GP_SPARSE_RAMP 1  // A/B knob: full gossip's ramp on lists (k_gs_sparse), one GPU
#endif
#ifndef GP_SHARD_BINS
#define GP_SHARD_BINS 1  // A/B knob: full gossip shards' receipt wave in bins (k_gs_bins_*)
#endif
#ifndef GP_BIN_GRID
#define GP_BIN_GRID 1024  // workgroups of the bins' count and placement passes (A/B knob)
#endif
#ifndef GP_BIN_DIV
// a round runs in bins while its receipts (estimated, every rank's) are >= actors / this (C4 / 8 rank
// kernels per run, incl. the loopback copies: 2 13.14 ms, 4 13.25, 8 13.29, 16 13.31;
// profiles/round6/bins_div_ab.txt)
#define GP_BIN_DIV 2
#endif
#ifndef GP_SHARD_RAMP
#define GP_SHARD_RAMP 1  // A/B knob: the same on shards (k_gs_sparse_x)
#endif

#include <algorithm>
#include <chrono>
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

// Layout of one exchange chunk (peer p -> peer q); both ends compute it identically.
struct Chunk {
    size_t hdir = 0, hslot = 0, hmsg = 0, slot = 0, msg = 0, size = 0;  // byte offsets / total size
    size_t tail = 0;    // first byte after the header and the halo face (the parts a plan resizes)
    size_t done = 0;    // full gossip: the sender's done part (0: none)
    uint32_t dwords = 0;  // full gossip: done-bitmap words of the sender's range
    uint32_t dpairs = 0;  // done part as (index, word) pairs (capacity); 0: every word
    uint32_t halo = 0;  // halo actors carried (0: none)
    uint32_t hcap = 0;  // halo entries: push-sum messages crossing the face
    uint32_t cap = 0;   // link / receipt entries
};

constexpr size_t kAlign = 256;
size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Group;

// Restore point of a push-sum shard under activity tiers (gp_shard_sync): the state F(k0) reads
// (the round k0-1 messages, direction bytes, link marks and remote link messages, the flags and
// the quiet-tail marks of round k0) and the host's counters at that round.
struct Ckpt {
    bool valid = false;
    int64_t next_kernel = 0, rounds = 0, completed = 0;
    int64_t k_launches = 0, work_rounds = 0;
    double k_total_ms = 0.0, k_aux_ms = 0.0;
    double2* msg = nullptr;
    uint8_t* dir = nullptr;
    uint8_t* lcnt = nullptr;
    uint32_t* lref = nullptr;  // push-sum shards: the slots' references of round k0-1
    char* rin = nullptr;       // and the receive buffer they point into (recv_total bytes)
    bool has_rin = false;
    uint8_t* flags = nullptr;
    uint8_t* act = nullptr;
    unsigned long long* work = nullptr;
    // full gossip: the counts, states, round k0-1's receipts and the done-bitmap replica
    uint32_t* cnt = nullptr;
    uint8_t* gstate = nullptr;
    uint32_t* inc = nullptr;
    uint32_t* dbits = nullptr;
    uint32_t* dsum = nullptr;
    uint32_t* dship = nullptr;  // the own words as shipped (lazy done-word shipping)
    int64_t gj = 0;             // the per-round plan's chain count at that round
    double gcj = 1.0;
    bool allocated = false;
};

struct Handle {
    Group* grp = nullptr;  // num_gpus > 1: this handle is the whole graph over the group's shards
    gp_config cfg{};
    gp_layout lay{};
    Geom g{};
    bool full = false, generic = false, gossip = false;
    // node-range shard (whole graph: lo = 0, hi = actors, world = 1)
    bool sharded = false;
    int32_t rank = 0, world = 1;
    uint32_t lo = 0, hi = 0;
    uint32_t halo = 0;  // z-plane (Imp3D/3D) or 1 actor (line/2D) exchanged with rank +-1
    std::vector<int64_t> abnd, sbnd;          // actor / link-slot bounds of every rank
    // A round in pieces: piece i of every rank's range is computed, packed and
    // exchanged on its own, so the exchange of one piece overlaps the next piece's kernels.  Chunks
    // are per (piece, peer), index i * world + q, laid out piece-major in the buffers.
    // The pieces run while the exchange carries the full plan (until half the nodes have converged;
    // after that the activity tiers shrink it and the extra launches would cost more than they hide):
    // kpiece is the handle's piece count, npiece the current one (1 or kpiece, chosen at a sync from
    // the global count, so every rank agrees).
    int kpiece = 1, npiece = 1;
    std::vector<int64_t> pbnd;                // kpiece bounds of every rank: pbnd[q * (kpiece + 1) + i]
    std::vector<Chunk> full_by[2][2];         // full plans [npiece > 1][out, in]
    int piece_next = 0;                       // the next piece gp_shard_round_piece packs
    int64_t round_slot = -1;                  // timing slot of the round being packed (-1: untimed)
    std::vector<unsigned long long> lhist;    // (src piece, dst rank, degree) link counts
    std::vector<Chunk> out_chunk, in_chunk;   // per (piece, peer)
    std::vector<int64_t> out_off, in_off;     // chunk offsets inside the send / recv buffers
    std::vector<int64_t> out_poff, in_poff;   // each piece's region (npiece + 1 offsets)
    int64_t send_total = 0, recv_total = 0;
    std::vector<uint32_t> max_in_cap;         // per piece
    std::vector<Chunk> full_out, full_in;  // the full plan (the buffers are sized for it)
    uint32_t* pmax = nullptr;      // running max of link entries per sub-segment to each (piece, peer)
    // full gossip shards: a plan per round.  Inputs every rank holds alike: the global
    // chain count cj emitted in round j (chains at most double per round), and per chunk the last
    // round's largest sub-segment count (m_out from this rank's pack, m_in from the peer's header) and
    // dirty done words (dw_out / dw_in).
    uint32_t* cparts = nullptr;               // chains emitted per round: kPartRing x kParts sub-counters
    unsigned long long* self_chains = nullptr;
    uint32_t* pstat = nullptr;                // kPstatWords: the last round's plan inputs (kPs*)
    uint32_t* dship = nullptr;                // own done words as last shipped
    uint32_t* dstat = nullptr;                // kDstatWords: dirty-word counter, backlog flag
    struct GossipPlan {
        bool on = false;    // sized plans (else the full plan); a restore point exists
        bool seen = false;  // m / dw hold a round's counts
        int64_t j = 0;      // round whose global chain count is cj
        double cj = 1.0;
        std::vector<uint32_t> m_out, m_in, dw_in;
        uint32_t dw_out = 0;
    } gpl;
    int64_t bytes_sent = 0;        // exchange bytes this rank sent since the last reset (replays included)
    int64_t list_rounds = 0;       // full gossip: rounds run on the ramp's lists since the last reset
    int64_t bin_rounds = 0;        // full gossip: rounds whose receipts went out in bins since the last reset
    const void* last_recv = nullptr;  // the receive buffer of the last gp_shard_deliver
    Ckpt ck;                       // activity tiers: the restore point (push-sum shards)
    int64_t full_until = 0;        // after a restore: the full plan until this many rounds are final
    bool tiered = false;           // the batch in flight may run reduced chunks (a global decision)
    int64_t delivered = 0;         // rounds delivered since the plan was last chosen
    int64_t plan_changes = 0, restores = 0;
    uint32_t* pcount = nullptr;
    uint32_t* overflow = nullptr;
    uint32_t* xfin = nullptr;      // push-sum tail rounds: k_ps_quiet_x<true>'s finished workgroups (Xchg::fin)
    unsigned long long* self_newly = nullptr;
    void* pending_send = nullptr;  // gp_shard_round issued, gp_shard_deliver not yet
    bool awaiting_deliver = false;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    int grid = 0;
    uint32_t span = 0;
    std::vector<void*> allocs;
    size_t dev_bytes = 0;
    // topology
    uint32_t* rev_off = nullptr;
    uint32_t* rev_src = nullptr;
    uint32_t* lpos = nullptr;
    uint8_t* lcnt[2] = {nullptr, nullptr};   // gossip link slots
    double2* rmsg[2] = {nullptr, nullptr};   // small one-GPU graphs: every link message per CSR slot
    uint32_t* lref[2] = {nullptr, nullptr};  // push-sum shards: slot references (gp_kernels.h kRefShift)
    const void* msg_src = nullptr;           // the receive buffer the next round reads remote messages from
    uint32_t* slot_dst = nullptr;            // shards with the quiet tail: receiver of each own CSR slot
    // push-sum
    double2* msg[kTileBufs] = {};
    uint8_t* dir[kTileBufs] = {};
    uint8_t* flags = nullptr;
    // small one-GPU line grids: several rounds per launch (k_ps_tile);
    // msg / dir / flags then rotate over kTileBufs buffers, round k's state in [k mod kTileBufs]
    bool tiles = false;
    bool tiny = false;  // gossip on a tiny graph: a batch of rounds in one workgroup's LDS (k_gs_tiny)
    uint8_t* flg[kTileBufs] = {};
    TileArgs tl{};
    int nbuf() const { return tiles ? (int)kTileBufs : 2; }
    // the buffer of round k's state (k = -1: the initial state)
    int bidx(int64_t k) const { return (int)((k + nbuf()) % nbuf()); }
    uint8_t* flags_at(int64_t k) const { return tiles ? flg[bidx(k)] : flags; }
    double2* frozen = nullptr;
    uint8_t* act[2] = {nullptr, nullptr};  // quiet-wave marks, one byte per 64 actors (ping-pong)
    uint32_t act_thr = 0;
    // gossip
    uint32_t* cnt = nullptr;
    uint8_t* gstate = nullptr;
    uint32_t* inc[2] = {nullptr, nullptr};
    uint32_t* dbits = nullptr;  // full gossip: done bitmap (k_gs_full4's sender filter); a shard's is
                                // biased (global bit = actor id) and covers its own actors
    uint32_t* dsum = nullptr;   // its summary (one bit per all-done word), from kDsumMinActors actors
    GsTally tally{};            // full gossip on one GPU: receipt tally by target bucket (cnt null: off)
    // full gossip: the ramp's rounds on lists (k_gs_sparse; shards k_gs_sparse_x) for rounds < sp_until, a
    // bound the host extends at every sync from the holder count (shards: every rank's, from the
    // exchange headers) until it has enqueued a walk over every actor (k_gs_full4 / k_gs_full4x)
    GsSparse gsp{};
    int64_t sp_until = 0;
    bool sp_frozen = false;
    bool sp_ran = false;          // a list round ran since the last sync (its error word is read there)
    // full gossip shards: the receipt wave in bins (GsBins), decided per round with the
    // round's plan (bin_next: the round gp_shard_round packs next), from values every rank holds
    GsBins bins{};
    bool bin_next = false;
    int bin_state = 0;            // 0: no binned round yet, 1: binned rounds, 2: the wave is over
    int64_t sp_fused = -1;        // shards: the round whose list kernel also ran its done-word pass and pack
    int64_t sp_s = -1;            // the last synced holder count: sp_h holders (shards: every rank's)
    uint64_t sp_h = 1;            // after F(sp_s), which sizes a list round's grid
    uint32_t* h_spctr = nullptr;  // pinned: the lists' counters and error word, copied after each batch
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
    unsigned long long* h_trace = nullptr;  // pinned, host-mapped (coherent)
    unsigned long long* d_trace = nullptr;  // its device address
    int64_t h_trace_cap = 0;
    int64_t next_kernel = 0;  // index of the next fused round kernel F(k)
    int64_t rounds = 0;       // rounds whose results are final
    int64_t completed = 0;
    bool converged = false;
    int64_t batch = 8;
    // timing
    std::vector<hipEvent_t> kev;  // 3 per round: before main, after main, after aux
    hipEvent_t ev_a = nullptr, ev_b = nullptr;
    int64_t k_launches = 0;
    double k_total_ms = 0.0, k_aux_ms = 0.0;
    unsigned long long* work = nullptr;  // actors walked by the quiet kernel (kernel statistics)
    int64_t work_rounds = 0;             // real rounds run while it counted
    std::vector<long long> timed_round;  // sharded: round applied by each timed kernel
    int64_t timed_count = 0;

    ~Handle() {
        if (stream) (void)hipStreamSynchronize(stream);
        for (void* p : allocs) (void)hipFree(p);
        if (h_trace) (void)hipHostFree(h_trace);
        if (h_spctr) (void)hipHostFree(h_spctr);
        for (hipEvent_t e : kev) (void)hipEventDestroy(e);
        if (ev_a) (void)hipEventDestroy(ev_a);
        if (ev_b) (void)hipEventDestroy(ev_b);
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }

    // Device array holding elements [first, first + count) of a global index space; *p is
    // biased by -first so kernels index it with global actor / slot ids.  The element range is
    // widened to start at a multiple of 16 (so the tile kernel's whole-dword / 16-byte loads of
    // actors v0 .. v0+3, v0 a multiple of 4, are aligned where they must be) and padded by 256
    // bytes on both sides: the row loads of the first and last lanes (v0 - 2 .. v0 + 5, a lane's
    // 16 link marks) read a few elements past [first, first + count) and never use them.
    template <class T>
    int alloc(T** p, size_t count, int64_t first = 0) {
        constexpr size_t kPad = 256;
        const int64_t f0 = first & ~(int64_t)15;
        const size_t n = (size_t)(first - f0) + count;
        void* q = nullptr;
        const size_t bytes = n * sizeof(T) + 2 * kPad;
        hipError_t e = hipMalloc(&q, bytes);
        if (e != hipSuccess) return fail(GP_ENOMEM, "hipMalloc(%zu bytes) failed: %s", bytes, hipGetErrorString(e));
        allocs.push_back(q);
        dev_bytes += bytes;
        *p = reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(q) + kPad - (uintptr_t)f0 * sizeof(T));
        return GP_OK;
    }

    // actors whose round-to-round messages this rank keeps: own range plus both halos
    int64_t ext_lo() const { return std::max<int64_t>(0, (int64_t)lo - halo); }
    int64_t ext_hi() const { return std::min<int64_t>(g.actors, (int64_t)hi + halo); }
    uint32_t own() const { return hi - lo; }
    int64_t piece_lo(int q, int i) const {
        if (npiece == 1) return i == 0 ? abnd[q] : abnd[q + 1];
        return pbnd[(size_t)q * (kpiece + 1) + i];
    }

    Launch L() const { return Launch{grid, stream}; }

    RoundArgs args(uint32_t r) const {
        RoundArgs a{};
        a.g = g;
        a.seed = cfg.seed;
        a.lo = lo;
        a.hi = hi;
        a.tag_prev = r ? link_tag(r - 1u) : 0u;
        a.tag_cur = link_tag(r);
        a.ps_tags = gossip ? 0u : 1u;
        a.slot_lo = sbnd.empty() ? 0u : (uint32_t)sbnd[rank];
        a.sharded = sharded ? 1u : 0u;
        a.r = r;
        a.target = (uint32_t)lay.nodes;
        a.full = full ? 1u : 0u;
        a.nodes = (uint32_t)lay.nodes;
        a.span = span;
        a.olo = lo;
        a.ohi = hi;
        if (gossip) a.threshold = (uint32_t)cfg.gossip_threshold;
        else a.act_thr = act_thr;
        a.delta = cfg.delta;
        a.term_limit = (uint32_t)cfg.term_limit;
        a.total = total;
        a.parts = parts;
        a.cparts = cparts;
        a.rev_off = rev_off;
        a.rev_src = rev_src;
        a.lpos = lpos;
        const int c = (int)(r & 1u), p = c ^ 1;
        const int cm = bidx(r), pm = bidx((int64_t)r - 1);  // msg / dir (kTileBufs buffers with tiles)
        a.lcnt_prev = lcnt[p];
        a.lcnt_cur = lcnt[c];
        a.msg_prev = msg[pm];
        a.msg_cur = msg[cm];
        a.rmsg_prev = rmsg[p];
        a.rmsg_cur = rmsg[c];
        a.lref_prev = lref[p];
        a.lref_cur = lref[c];
        a.rtag_prev = r ? ref_tag(r - 1u) : 0u;
        a.rtag_cur = ref_tag(r);
        a.rin_prev = static_cast<const double2*>(msg_src);
        a.dir_prev = dir[pm];
        a.dir_cur = dir[cm];
        a.work = (cfg.flags & GP_FLAG_KERNEL_TIMING) && act[0] ? work : nullptr;
        a.flags = flags_at((int64_t)r - 1);
        a.frozen = frozen;
        if (gossip) {
            a.cnt = cnt;
            a.gstate = gstate;
        } else {
            a.act_prev = act[r & 1u];
            a.act_cur = act[(r + 1u) & 1u];
        }
        a.dbits = dbits;
        a.dsum = dsum;
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

Xchg base_xchg(const Handle* h);

// Imp3D extra links (program.fs:309) and their receiver-side CSR.  A rank keeps only its own
// slices: rev_off / rev_src for the destinations it owns ([lo, hi) and their CSR slots
// [slo, shi)), lpos for the senders it owns.  No rank stores the link array: link_of() recomputes
// a link from (seed, sender), so every rank knows every link without an exchange — which remote
// senders target its actors, at which global slot, and the per-peer link counts that size the
// exchange.  Three transient arrays over all destinations (counts, offsets, the own senders'
// offsets) live only during the build.
// A push-sum shard keeps 32-bit slot references; its link pass writes them (a
// one-rank shard too: the library group at num_gpus = 1).
bool refs(const Handle* h) { return h->sharded && !h->gossip && !h->generic; }

int build_links(Handle* h) {
    const uint32_t nodes = (uint32_t)h->lay.nodes, A = h->g.actors;
    const uint32_t lo = h->lo, hi = h->hi, shi_src = std::min(hi, nodes);  // own senders [lo, shi_src)
    const uint64_t seed = h->cfg.seed;
    int rc;
    if ((rc = h->alloc(&h->rev_off, (size_t)(hi - lo) + 1, lo))) return rc;
    if (!h->generic && shi_src > lo && (rc = h->alloc(&h->lpos, (size_t)(shi_src - lo), lo))) return rc;
    const size_t nA = (size_t)A + 1;
    uint32_t *X = nullptr, *Y = nullptr, *Z = nullptr, *list = nullptr, *scratch = nullptr;
    auto cleanup = [&]() {
        for (uint32_t* p : {X, Y, Z, list, scratch})
            if (p) (void)hipFree(p);
    };
    if (hipMalloc(&X, nA * 4) != hipSuccess || hipMalloc(&Y, nA * 4) != hipSuccess || hipMalloc(&Z, nA * 4) != hipSuccess ||
        hipMalloc(&list, ((size_t)(shi_src > lo ? shi_src - lo : 0) + 1) * 4) != hipSuccess ||
        hipMalloc(&scratch, scan_scratch_words(A + 1) * 4) != hipSuccess) {
        cleanup();
        return fail(GP_ENOMEM, "extra-link CSR build: transient arrays of %zu bytes", 3 * nA * 4);
    }
    const Launch l = h->L();
    hipStream_t s = h->stream;
    hipError_t e = hipSuccess;
    std::vector<uint32_t> sb((size_t)h->world + 1);
    // X = links per destination (all senders); Y = their exclusive scan = global CSR offsets
    e = hipMemsetAsync(X, 0, nA * 4, s);
    if (e == hipSuccess) {
        launch_dst_count(seed, nodes, 0, nodes, X, l);
        launch_exclusive_scan(X, Y, A + 1, scratch, s);
        e = hipMemcpyAsync(h->rev_off + lo, Y + lo, (size_t)(hi - lo + 1) * 4, hipMemcpyDeviceToDevice, s);
    }
    for (int q = 0; q <= h->world && e == hipSuccess; ++q)  // link-slot bounds of every rank
        e = hipMemcpyAsync(&sb[(size_t)q], Y + h->abnd[q], 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const uint32_t slo = sb[(size_t)h->rank], shi = sb[(size_t)h->rank + 1];
    if (e == hipSuccess && (rc = h->alloc(&h->rev_src, (size_t)(shi - slo), slo))) {
        cleanup();
        return rc;
    }
    // own destinations' sources, ascending per destination
    if (e == hipSuccess) e = hipMemsetAsync(X, 0, nA * 4, s);
    if (e == hipSuccess) {
        launch_dst_fill(seed, nodes, 0, nodes, lo, hi, Y, X, h->rev_src, l);
        launch_sort_segments(h->rev_off + lo, h->rev_src, hi - lo, l);
    }
    // lpos of the own senders: base[t] = Y[t] + links into t from senders below lo; the own
    // senders' per-destination lists (Z-offsets, sorted) give each one's place after that
    if (e == hipSuccess && !h->generic && shi_src > lo) {
        e = hipMemsetAsync(X, 0, nA * 4, s);
        if (e == hipSuccess) e = hipMemsetAsync(Z, 0, nA * 4, s);
        if (e == hipSuccess) {
            launch_dst_count(seed, nodes, 0, lo, X, l);
            launch_add_u32(X, Y, A + 1, l);
            launch_dst_count(seed, nodes, lo, shi_src, Z, l);
            launch_exclusive_scan(Z, Y, A + 1, scratch, s);
            e = hipMemsetAsync(Z, 0, nA * 4, s);
        }
        if (e == hipSuccess) {
            launch_dst_fill(seed, nodes, lo, shi_src, 0, A, Y, Z, list, l);
            launch_sort_segments(Y, list, A, l);
            launch_lpos_lists(Y, list, A, X, h->lpos, l);
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipGetLastError();
    cleanup();
    if (e != hipSuccess) return fail(GP_EHIP, "extra-link CSR build failed: %s", hipGetErrorString(e));
    h->lay.links = nodes;
    h->sbnd.assign(sb.begin(), sb.end());
    const int64_t nsl = (int64_t)shi - slo;
    if (!h->generic) {  // pull kernels
        // per-slot link marks of the own slots (gossip chains, push-sum round tags)
        // (a push-sum shard: 32-bit references)
        if (refs(h)) {
            if ((rc = h->alloc(&h->lref[0], (size_t)nsl, slo)) || (rc = h->alloc(&h->lref[1], (size_t)nsl, slo))) return rc;
        } else if ((rc = h->alloc(&h->lcnt[0], (size_t)nsl, slo)) || (rc = h->alloc(&h->lcnt[1], (size_t)nsl, slo))) {
            return rc;
        }
        // on a small one-GPU graph every link message lands in the receiver's slot (k_ps_pull<3>, the
        // latency-bound rounds)
        // (one GPU: up to 2^18 actors; at 1M actors the scattered 16-byte slot stores cost more than
        // the load level they save, profiles/round4/small_imp3d)
        const bool slot_msgs = !h->sharded && !h->act[0] && h->g.actors < kSlotMsgMaxActors;
        if (slot_msgs && !h->gossip &&
            ((rc = h->alloc(&h->rmsg[0], (size_t)nsl, slo)) || (rc = h->alloc(&h->rmsg[1], (size_t)nsl, slo))))
            return rc;
        // the unpack marks the segment of a remote link message's receiver (quiet tail)
        if (h->sharded && h->world > 1 && !h->gossip && h->act[0]) {
            if ((rc = h->alloc(&h->slot_dst, (size_t)nsl, slo))) return rc;
            launch_slot_owner(h->rev_off, lo, hi, h->slot_dst, h->L());
            HIP_TRY(hipStreamSynchronize(s));
            HIP_TRY(hipGetLastError());
        }
    }
    if (h->sharded) {  // link counts per (source piece, destination rank, sender degree)
        const int K = h->kpiece, W = h->world;
        const size_t nb = (size_t)W * K * W * 8;
        HistBounds hb{};
        hb.ns = (uint32_t)(W * K);
        hb.nd = (uint32_t)W;
        for (int q = 0; q < W; ++q)
            for (int i = 0; i < K; ++i) hb.sb[q * K + i] = (uint32_t)h->pbnd[(size_t)q * (K + 1) + i];
        hb.sb[W * K] = (uint32_t)h->abnd[W];
        for (int q = 0; q <= W; ++q) hb.db[q] = (uint32_t)h->abnd[q];
        unsigned long long* hist = nullptr;
        HIP_TRY(hipMalloc(&hist, nb * sizeof *hist));
        e = hipMemsetAsync(hist, 0, nb * sizeof *hist, s);
        if (e == hipSuccess) {
            launch_link_hist(seed, h->g, hb, hist, l);
            h->lhist.assign(nb, 0);
            e = hipMemcpyAsync(h->lhist.data(), hist, nb * sizeof *hist, hipMemcpyDeviceToHost, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        (void)hipFree(hist);
        if (e != hipSuccess) return fail(GP_EHIP, "link histogram failed: %s", hipGetErrorString(e));
    }
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

// Quiet-wave marks: one byte per segment of kActSeg actors, indexed by global segment (actor >>
// kActShift); a handle holds the segments of its actors [lo, hi) (+1 byte of padding).
size_t act_first(const Handle* h) { return (size_t)(h->lo >> kActShift); }
size_t act_bytes(const Handle* h) { return (size_t)((h->hi + kActSeg - 1u) >> kActShift) - act_first(h) + 1u; }
int clear_act(Handle* h, int i) {
    HIP_TRY(hipMemsetAsync(h->act[i] + act_first(h), 0, act_bytes(h), h->stream));
    return GP_OK;
}

// Full gossip's done bitmap over every actor (one bit each) and its summary (one bit per word).
size_t dbits_words_all(const Handle* h) { return ((size_t)h->g.actors + 31u) / 32u + 1u; }
size_t dsum_words_all(const Handle* h) { return ((size_t)h->g.actors + 1023u) / 1024u + 1u; }
// a shard's own words of it (global word index (lo >> 5) on)
size_t dship_words(const Handle* h) { return (size_t)(((h->hi - 1u) >> 5) - (h->lo >> 5) + 1u); }

void full_plan(Handle* h);
void use_layout(Handle* h, int K);
int want_pieces(const Handle* h);
bool tiers_on(const Handle* h);
bool gossip_plans(const Handle* h);
void gossip_round_plan(Handle* h, int64_t k);
int ensure_ckpt(Handle* h);
int ckpt_copy(Handle* h, bool save);

// The rounds after round s that may run on lists (k_gs_sparse) when `holders` actors hold a chain after
// F(s): a chain starts only on a first receipt, so the holders after F(j) are at most holders * 2^(j - s),
// and F(r) fits its lists while the holders after F(r - 1) are <= cap.  Returns the first round that
// does not (exclusive bound).
int64_t sp_bound(uint32_t cap, int64_t s, uint64_t holders) {
    int64_t k = 0;
    while (holders << (k + 1) <= cap && k < 62) ++k;
    return holders <= cap ? s + 2 + k : s + 1;
}

int reset(Handle* h) {
    HIP_TRY(hipStreamSynchronize(h->stream));
    const size_t lo = h->lo, n = h->own();
    const size_t xlo = (size_t)h->ext_lo(), xn = (size_t)(h->ext_hi() - h->ext_lo());
    HIP_TRY(hipMemsetAsync(h->total, 0, (size_t)h->total_cap * sizeof(unsigned long long), h->stream));
    HIP_TRY(hipMemsetAsync(h->parts, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t), h->stream));
    if (h->sharded) {
        HIP_TRY(hipMemsetAsync(h->pcount, 0, ((size_t)h->world + 2) * kSub * kCtrStride * sizeof(uint32_t), h->stream));
        HIP_TRY(hipMemsetAsync(h->overflow, 0, sizeof(uint32_t), h->stream));
    }
    if (h->lcnt[0] || h->lref[0]) {  // no link message in flight
        const size_t slo = (size_t)h->sbnd[h->rank], ns = (size_t)(h->sbnd[h->rank + 1] - h->sbnd[h->rank]);
        for (int i = 0; i < 2; ++i) {
            if (h->lcnt[i]) HIP_TRY(hipMemsetAsync(h->lcnt[i] + slo, 0, ns, h->stream));
            if (h->lref[i]) HIP_TRY(hipMemsetAsync(h->lref[i] + slo, 0, ns * sizeof(uint32_t), h->stream));
        }
    }
    h->msg_src = nullptr;
    if (!h->gossip) {
        for (int i = 0; i < (h->tiles ? h->nbuf() : 1); ++i)  // (tiles: every buffer; non-participants keep theirs)
            launch_ps_init(h->tiles ? h->flg[i] : h->flags, h->g, h->lo, h->hi, h->full ? 1u : 0u,
                           (uint32_t)h->cfg.term_init, h->L());
        if (h->generic) {
            HIP_TRY(hipMemsetAsync(h->bcnt[0] + lo, 0, n * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->bcnt[1] + lo, 0, n * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->tgt + lo, 0xFF, n * sizeof(uint32_t), h->stream));
        } else {
            for (int i = 0; i < h->nbuf(); ++i) launch_fill_u8(h->dir[i] + xlo, kDirNone, xn, h->stream);
            for (int i = 0; i < 2; ++i) {
                int rc;
                if (h->act[i] && (rc = clear_act(h, i))) return rc;
            }
        }
    } else {
        HIP_TRY(hipMemsetAsync(h->cnt + lo, 0, n * sizeof(uint32_t), h->stream));
        HIP_TRY(hipMemsetAsync(h->gstate + lo, 0, n, h->stream));
        if (h->generic) {
            HIP_TRY(hipMemsetAsync(h->inc[0] + lo, 0, n * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->inc[1] + lo, 0, n * sizeof(uint32_t), h->stream));
            if (h->dbits) {  // the whole bitmap (a shard's replica included), then the summary
                HIP_TRY(hipMemsetAsync(h->dbits, 0, dbits_words_all(h) * sizeof(uint32_t), h->stream));
                if (h->dsum) HIP_TRY(hipMemsetAsync(h->dsum, 0, dsum_words_all(h) * sizeof(uint32_t), h->stream));
            }
            if (h->tally.cnt) {
                HIP_TRY(hipMemsetAsync(h->tally.chains, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t),
                                       h->stream));
                HIP_TRY(hipMemsetAsync(h->tally.on, 0, 4 * sizeof(uint32_t), h->stream));
            }
            if (h->gsp.hl) {  // the holder list is the leader (program.fs:218; a shard's: if it is its actor);
                              // every count zero
                HIP_TRY(hipMemsetAsync(h->gsp.ctr, 0, (3 * 4 + 1) * kSpStride * sizeof(uint32_t), h->stream));  // (+ fin)
                HIP_TRY(hipMemsetAsync(h->gsp.err, 0, sizeof(uint32_t), h->stream));
                const uint32_t L = (uint32_t)h->lay.leader;
                h->gsp.h0 = L >= h->lo && L < h->hi ? 1u : 0u;
                if (h->gsp.h0) HIP_TRY(hipMemcpyAsync(h->gsp.hl, &L, sizeof L, hipMemcpyHostToDevice, h->stream));
                h->sp_until = sp_bound(h->gsp.cap, -1, 1);
                h->sp_frozen = false;
                h->sp_ran = false;
                h->sp_s = -1;
                h->sp_h = 1;
                h->sp_fused = -1;
            }
        } else {
            launch_fill_u8(h->dir[0] + xlo, 0xFF, xn, h->stream);
            launch_fill_u8(h->dir[1] + xlo, 0xFF, xn, h->stream);
        }
        // kick-off (program.fs:181/218/258/323): the leader holds one activation chain; for
        // "full" it is a CallChildActor, i.e. also its first receipt.
        const uint32_t L = (uint32_t)h->lay.leader;
        if (L >= h->lo && L < h->hi) {
            const uint8_t st = 1;
            HIP_TRY(hipMemcpyAsync(h->gstate + L, &st, 1, hipMemcpyHostToDevice, h->stream));
            if (h->full) {
                const uint32_t one = 1;
                HIP_TRY(hipMemcpyAsync(h->cnt + L, &one, sizeof one, hipMemcpyHostToDevice, h->stream));
            }
        }
    }
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipGetLastError());
    h->next_kernel = 0;
    h->rounds = 0;
    h->completed = 0;
    h->converged = false;
    // (tiny: the whole batch is one launch, and its rounds past convergence exit in the kernel, so
    // the largest batch from the start: one host sync for C1)
    h->batch = h->tiny || h->tiles ? kMaxBatch : 8;
    h->awaiting_deliver = false;
    h->piece_next = 0;
    h->round_slot = -1;
    h->timed_count = 0;
    if (h->sharded) {  // the full plan, no restore point
        HIP_TRY(hipMemsetAsync(h->pmax, 0, (size_t)kMaxPieces * kMaxWorld * sizeof(uint32_t), h->stream));
        if (h->cparts) {  // full gossip's per-round plan inputs and done-word shipping state
            HIP_TRY(hipMemsetAsync(h->cparts, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->pstat, 0, kPstatWords * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->dstat, 0, kDstatWords * sizeof(uint32_t), h->stream));
            HIP_TRY(hipMemsetAsync(h->dship + (h->lo >> 5), 0, dship_words(h) * sizeof(uint32_t), h->stream));
        }
        HIP_TRY(hipStreamSynchronize(h->stream));
        h->ck.valid = false;
        h->tiered = false;
        h->delivered = 0;
        h->full_until = 0;
        h->last_recv = nullptr;
        h->bytes_sent = 0;
        h->list_rounds = 0;
        h->bin_rounds = 0;
        if (h->kpiece > 1 && !h->full_out.empty()) use_layout(h, want_pieces(h));
        if (!h->full_out.empty()) full_plan(h);
        h->bin_state = 0;
        h->bin_next = false;
        if (gossip_plans(h) && !h->full_out.empty()) {
            // round 0's chains: the leader's one (program.fs:218); the sized plans run from round 0, so
            // the restore point is the initial state
            Handle::GossipPlan& P = h->gpl;
            P = Handle::GossipPlan{};
            P.m_out.assign((size_t)h->world, 0u);
            P.m_in.assign((size_t)h->world, 0u);
            P.dw_in.assign((size_t)h->world, 0u);
            P.on = tiers_on(h);
            int rc;
            if (P.on && ((rc = ensure_ckpt(h)) || (rc = ckpt_copy(h, true)))) return rc;
            h->tiered = P.on;
            gossip_round_plan(h, 0);
        }
    }
    return GP_OK;
}

// Full gossip on one GPU runs the four-actors-per-lane kernel with the done bitmap.
bool full_quad(const Handle* h) { return h->gossip && h->full && !h->sharded && h->lo == 0; }



bool fused_marks(const Handle* h) { return kFuseLinkMarks && !h->gossip && !h->generic && !h->sharded && h->g.has_link; }

const char* round_kernel_name(const Handle* h) {
    // with the receipt tally the timed bracket also holds its passes (the scans, the placement and
    // the per-bucket count, gp_kernels.hip launch_gs_tally), which run after k_gs_full4 every round
    if (h->tiny) return h->gossip ? "k_gs_tiny" : "k_ps_tiny";
    if (full_quad(h)) return h->tally.cnt ? "k_gs_full4+tally" : "k_gs_full4";
    if (h->gossip && !h->generic) {
        const bool e = gs_pull_early(h->args(0));
        return h->g.has_link ? (e ? "k_gs_pull<true, true>" : "k_gs_pull<true, false>")
                             : (e ? "k_gs_pull<false, true>" : "k_gs_pull<false, false>");
    }
    if (h->gossip) return h->sharded ? "k_gs_full4x" : "k_gs_push";
    if (h->generic) return "k_ps_push_emit";
    if (h->sharded && h->g.has_link && h->lref[0]) return h->act[0] ? "k_ps_quiet_x" : "k_ps_pull<2, false>";
    if (h->g.has_link && h->rmsg[0]) return "k_ps_pull<3, false>";
    if (h->g.has_link) return h->act[0] ? "k_ps_quiet<1>" : "k_ps_pull<1, false>";
    if (h->tiles) return "k_ps_tile";
    return h->act[0] ? "k_ps_quiet<0>" : "k_ps_pull<0, false>";
}

const char* aux_kernel_name(const Handle* h) {
    if (h->tiny) return "";
    if (h->generic) return h->gossip ? (h->sharded && h->world > 1 ? "k_shard_done_out" : "") : "k_scan_* + k_ps_push_fill";
    if (!h->g.has_link || fused_marks(h)) return "";
    if (h->sharded && !h->gossip && kShardFuse && h->act[0]) return "";  // (routed by k_ps_quiet_x)
    if (h->sharded) return h->gossip ? "k_gs_link_scatter_x" : "k_ps_link_scatter_x";
    return "k_link_count";
}

// Compulsory HBM bytes of one launch of the dominant round kernel for its data layout
// (every array element it must touch, touched once); DESIGN.md §5.
//   push-sum pull: held (S,W) read 16 + message write 16 + flags read 1 + direction byte read
//   1 (own row; neighbour rows re-read from cache) + direction write 1 per participant; Imp3D
//   adds the link CSR offsets (4 per actor), per link the 4-byte source and 1-byte slot count,
//   and the 16-byte message of every link that fired (~1 in 7: the interior degree); with the
//   marks written by the round kernel (one GPU), each sender's 4-byte CSR slot and the 1-byte
//   mark of every fired link.  A separate link count pass is not included.
//   gossip pull: state byte read 1 + direction byte read 1 + write 1 (+ count r/w 8 on the
//   receipts, not modelled); Imp3D adds offsets 4 per actor and 1 per link slot.
double bytes_per_round(const Handle* h) {
    const double frac = (double)h->own() / (double)h->g.actors;  // a shard's share
    const double P = (double)h->lay.participants * frac, A = (double)h->own(), links = (double)h->lay.links * frac;
    if (h->gossip) {
        if (h->generic) return P * (4 + 4 + 1 + 1) + P * 2 * 4;  // cnt r/w, inc r, state r/w, 2 atomics
        return P * (1 + 1 + 1) + (h->g.has_link ? 4 * A + 1 * links : 0);
    }
    if (h->generic) return P * (16 + 16 + 16 + 1 + 4 + 4 + 4 + 4 + 4);
    double b = P * (16 + 16 + 1 + 1 + 1);
    if (h->g.has_link) b += 4 * A + links * (4 + 1) + links / 7 * 16;
    if (fused_marks(h)) b += 4 * A + links / 7;
    return b;
}

// Push-sum link marks of round r go into lcnt[r & 1]; clear that array before a tag value
// repeats in it (link_tag), after F(r-1) has read it and before round r's marks are written
// (by F(r) itself when the marks are fused, else by the pass after it).
int clear_tags_if_due(Handle* h, uint32_t r) {
    if (h->gossip) return GP_OK;
    const int64_t slo = h->sbnd.empty() ? 0 : h->sbnd[h->rank], ns = h->sbnd.empty() ? 0 : h->sbnd[h->rank + 1] - slo;
    if (h->lcnt[0] && tag_clear_round(r)) HIP_TRY(hipMemsetAsync(h->lcnt[r & 1u] + slo, 0, (size_t)ns, h->stream));
    if (h->lref[0] && ref_clear_round(r))  // (references: 31 tag values, every 62 rounds)
        HIP_TRY(hipMemsetAsync(h->lref[r & 1u] + slo, 0, (size_t)ns * sizeof(uint32_t), h->stream));
    return GP_OK;
}

// The dominant round kernel F(k) (timed under GP_FLAG_KERNEL_TIMING) ...  A shard samples the
// timing of every kTimeEvery-th round (`timed`), and counts the actors its quiet kernel walks in
// exactly those rounds, so work_per_launch and avg_ms average over the same launches.
// Piece i of a shard's round: the launch walks the piece's actors on a grid for them.
void piece_args(const Handle* h, int piece, RoundArgs& a, Launch& l) {
    if (h->npiece <= 1) return;
    a.lo = (uint32_t)h->piece_lo(h->rank, piece);
    a.hi = (uint32_t)h->piece_lo(h->rank, piece + 1);
    l.grid = grid_for(a.hi - a.lo);
    a.span = span_for(a.hi - a.lo, l.grid);
}

// A list round's grid: one thread per item at most.  F(k)'s items (the holders after F(k - 1) and the
// targets of round k - 1, at most as many) are bounded by the synced holder count, doubled per round
// since (a chain starts only on a first receipt).
constexpr int kSpFusedGrid = 256;
Launch sp_launch(const Handle* h, int64_t k, Launch l) {
    const int64_t d = std::min<int64_t>(std::max<int64_t>(k - 1 - h->sp_s, 0), 40);
    const double items = 2.0 * (double)h->sp_h * std::ldexp(1.0, (int)d);
    l.grid = (int)std::max(1.0, std::min((double)l.grid, std::ceil(items / (double)kBlock)));
    return l;
}

void launch_main(Handle* h, int64_t k, const Xchg* x, bool timed, int piece = 0, int nr = 1) {
    RoundArgs a = h->args((uint32_t)k);
    if (h->tiles) {
        launch_ps_tile(a, h->tl, nr, h->stream);
        return;
    }
    if (h->tiny) {
        if (h->gossip) launch_gs_tiny(a, nr, h->stream);
        else launch_ps_tiny(a, nr, h->stream);
        return;
    }
    if (h->sharded && !timed) a.work = nullptr;
    Launch l = h->L();
    piece_args(h, piece, a, l);
    if (h->gossip) {
        if (h->generic) {  // adds into inc_cur, consumed (zeroed) by F(k+1)
            const bool lists = h->gsp.hl && !h->sp_frozen && k < h->sp_until;
            if (x && lists) {  // the ramp on this rank's lists; the round's passes in its last block
                h->sp_ran = true;
                h->sp_fused = k;
                ++h->list_rounds;
                Launch ls = sp_launch(h, k, l);
                ls.grid = std::min(ls.grid, kSpFusedGrid);  // (the last-block count: one atomic per block)
                launch_gs_sparse_x(a, *x, h->gsp, h->gossip ? (long long)k - 1 : (long long)k, ls);
            } else if (x && x->binned) {  // the receipt wave: counted, scanned, placed in bins
                h->sp_frozen = true;
                ++h->bin_rounds;
                launch_gs_bins(a, *x, h->bins, h->stream);
            } else if (x) {
                h->sp_frozen = true;
                launch_gs_full4x(a, *x, l);
            } else if (full_quad(h) && lists) {
                h->sp_ran = true;
                launch_gs_sparse(a, h->tally, h->gsp, sp_launch(h, k, l));  // the ramp: lists (no tally can be due)
            } else if (full_quad(h)) {
                h->sp_frozen = true;  // lists only before the first k_gs_full4 round
                launch_gs_full4(a, h->tally, l);
                // the tally's passes exit at once in a round that does not tally; once the synced count
                // rules the tally out for every later round (fewer than 1/kTallyLateDiv of the nodes
                // left, and fewer receipts to them than thr even at two chains per actor), they are
                // not launched at all
                const int64_t left = h->lay.nodes - h->completed;
                // (round k's choice is made by F(k - 1) on the count after round k - 3: at least the
                // synced one from k = rounds + 2; one round of margin)
                const bool never = h->tally.thr && k >= h->rounds + 3 && left * (int64_t)std::max<uint64_t>(kTallyLateDiv, 1) < h->lay.nodes &&
                                   (double)left * 2.0 * (double)h->g.actors < (double)h->tally.thr * (double)h->lay.nodes;
                if (!never) launch_gs_tally(a, h->tally, l);
            }
            else launch_gs_push(a, l);
        } else {
            launch_gs_pull(a, l);
        }
    } else if (h->generic) {
        launch_ps_push_emit(a, l);
    } else {
        launch_ps_pull(a, l, x);
    }
}

// ... and the passes that complete round k after it (link scatter; bucket scan + fill).
int launch_aux(Handle* h, int64_t k, const Xchg* x, int piece = 0) {
    const uint32_t r = (uint32_t)k;
    RoundArgs a = h->args(r);
    Launch l = h->L();
    piece_args(h, piece, a, l);
    int rc;
    if (h->tiny) return GP_OK;  // (k_ps_tiny builds its buckets itself)
    // (a shard clears before its round kernel: its tail rounds write their own link marks)
    if (!fused_marks(h) && !h->sharded && (rc = clear_tags_if_due(h, r))) return rc;
    (void)rc;
    if (h->gossip) {
        if (!h->generic && h->g.has_link) {
            if (x) launch_gs_link_scatter_x(a, *x, l);
            else launch_link_count(a, l);
        }
        // (a list round's last block ran it: k_gs_sparse_x.  A round in bins sends no done words while a
        // quarter of the nodes or more have not reported: the peers' replicas only feed the sender-side
        // filter, which those rounds do not run, and a word left unshipped goes out with a later round's,
        // as any word past a plan's capacity does; the last rounds of the wave ship them, so the filter
        // of the rounds after it starts current)
        const bool skip_done = x && x->binned && (h->lay.nodes - h->completed) * 4 > h->lay.nodes;
        if (h->generic && x && h->world > 1 && h->sp_fused != k && !skip_done) launch_shard_done_out(a, *x, h->stream);
    } else if (h->generic) {
        const int c = (int)(r & 1u);
        launch_exclusive_scan(h->bcnt[c], h->boff[c], h->g.actors, h->scan_scratch, h->stream);
        launch_ps_push_fill(a, h->slot[c], h->boff[c], l);
    } else if (h->g.has_link) {
        // a shard's quiet-tail rounds route their own link messages (k_ps_quiet_x) and the pass would
        // return at once: once the synced count has reached act_thr, every later round is such a round
        // (the count only grows), so the pass is not launched at all
        const bool tail = h->act[0] && h->act_thr && h->completed >= (int64_t)h->act_thr && k >= h->rounds + 1;
        // (k_ps_quiet_x routes a dense round's link messages itself: kShardFuse)
        if (x && !tail && !(kShardFuse && h->act[0])) launch_ps_link_scatter_x(a, *x, l);
        else if (!x && !fused_marks(h)) launch_link_count(a, l);
    }
    return GP_OK;
}

constexpr int64_t kTimeEvery = 8;  // kernel timing: one round in 8
// Kernel timing without a pass after the round kernel: one event pair per group of kTimeGroup
// consecutive rounds.  Each record stalls the queue: groups of 8 added 9.3 ms to a 129 ms C3
// run (7%, and 40% of a 20 us tail round); groups of 64 add about 1/8 of that (round 3).
constexpr int64_t kTimeGroup = 256;  // = the largest batch: one event pair per batch (round 4; 64 before)
#ifndef GP_TAIL_BATCH
#define GP_TAIL_BATCH 32
#endif
constexpr int64_t kTailBatch = GP_TAIL_BATCH;  // rounds per batch in a run's tail (0: no tail rule)

int ensure_events(Handle* h, int64_t rounds) {
    const size_t need = (size_t)(3 * rounds);
    if (h->kev.size() >= need) return GP_OK;
    const size_t old = h->kev.size();
    h->kev.resize(need);
    for (size_t i = old; i < need; ++i) HIP_TRY(hipEventCreate(&h->kev[i]));
    return GP_OK;
}

// Quiet-wave marks for round k + 1 go into act[(k + 1) & 1] during F(k), tagged link_tag(k + 1):
// clear that array before a tag value repeats in it (after F(k - 1) has read it).
int clear_act_if_due(Handle* h, int64_t k) {
    if (!h->act[0] || !tag_clear_round((uint32_t)(k + 1))) return GP_OK;
    return clear_act(h, (int)((k + 1) & 1));
}

// Round k with its three timing events (slot i of the event ring).
// (In pieces, the events bracket the whole round: piece 0's round kernel to the last piece's round
// kernel, then the last piece's pass; the earlier pieces' passes count as round kernel time.)
int launch_round(Handle* h, int64_t k, const Xchg* x, bool timing, int64_t i, int piece = 0, int nr = 1) {
    int rc;
    const bool first = piece == 0, last = piece == h->npiece - 1;
    if (first && (fused_marks(h) || h->sharded) && (rc = clear_tags_if_due(h, (uint32_t)k))) return rc;
    if (first && (rc = clear_act_if_due(h, k))) return rc;
    if (timing && first) HIP_TRY(hipEventRecord(h->kev[3 * i], h->stream));
    launch_main(h, k, x, timing, piece, nr);
    if (timing && last) HIP_TRY(hipEventRecord(h->kev[3 * i + 1], h->stream));
    if ((rc = launch_aux(h, k, x, piece))) return rc;
    if (timing && last) HIP_TRY(hipEventRecord(h->kev[3 * i + 2], h->stream));
    return GP_OK;
}

int accumulate_timing(Handle* h, int64_t n) {
    for (int64_t i = 0; i < n; ++i) {
        float m = 0.f, x = 0.f;
        HIP_TRY(hipEventElapsedTime(&m, h->kev[3 * i], h->kev[3 * i + 1]));
        HIP_TRY(hipEventElapsedTime(&x, h->kev[3 * i + 1], h->kev[3 * i + 2]));
        h->k_total_ms += m;
        h->k_aux_ms += x;
    }
    h->k_launches += n;
    return GP_OK;
}

int fill_sums(Handle* h, gp_status* st) {
    if (h->gossip) return GP_OK;
    const int64_t last = h->rounds - 1;
    RoundArgs a = h->args((uint32_t)std::max<int64_t>(last, 0));
    a.msg_prev = h->msg[h->bidx(std::max<int64_t>(last, 0))];
    a.dir_prev = h->generic ? nullptr : h->dir[h->bidx(std::max<int64_t>(last, 0))];
    a.flags = h->flags_at(last);
    launch_ps_sums(a, last >= 0 ? 1u : 0u, h->partials, h->L());
    std::vector<double2> part((size_t)h->grid);
    HIP_TRY(hipMemcpyAsync(part.data(), h->partials, part.size() * sizeof(double2), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (const double2& p : part) {
        st->sum_s += p.x;
        st->sum_w += p.y;
    }
    return GP_OK;
}

int step(Handle* h, int64_t max_rounds, gp_status* st) {
    if (max_rounds < 0) return fail(GP_EINVAL, "max_rounds < 0");
    if (h->sharded) return fail(GP_ESTATE, "a shard advances with gp_shard_round / gp_shard_deliver");
    const bool timing = (h->cfg.flags & GP_FLAG_KERNEL_TIMING) != 0;
    HIP_TRY(hipEventRecord(h->ev_a, h->stream));
    const int64_t goal = h->rounds + max_rounds;
    int rc;
    while (!h->converged && h->rounds < goal) {
        const int64_t B = std::min<int64_t>(h->batch, goal - h->rounds);
        const int64_t before = h->completed;
        const bool was_tail = kTailBatch > 0 && before * 32 >= h->lay.nodes * 31;
        if ((rc = ensure_trace(h, h->next_kernel + B + 4))) return rc;
        if (h->gossip && h->next_kernel == 0) {  // F(0) only emits round 0
            if ((rc = launch_round(h, 0, nullptr, false, 0))) return rc;
            h->next_kernel = 1;
        }
        // Kernel timing.  With no pass after the round kernel, one event pair brackets each group
        // of kTimeGroup consecutive round kernels (per-launch time = group time / rounds, launch
        // gaps included); otherwise every kTimeEvery-th round is bracketed kernel by kernel.  Either
        // way the events stay out of most of the stream (each record costs stream time).
        const bool group = timing && aux_kernel_name(h)[0] == '\0';
        const int64_t every = group ? kTimeGroup : kTimeEvery;
        const int64_t ng = (B + every - 1) / every;
        if (timing && (rc = ensure_events(h, ng))) return rc;
        for (int64_t i = 0; i < B;) {
            const int64_t j = i / every;
            // tiles: up to kTileMaxNR rounds in one launch, within this batch and timing group
            int nr = 1;
            while (h->tiles && nr < (int)kTileMaxNR && i + nr < B && (i + nr) / every == j) ++nr;
            // tiny: the batch at once (with kernel timing: its timing group)
            if (h->tiny) nr = (int)(timing ? std::min(B - i, every - i % every) : B - i);
            if (group && i % every == 0) HIP_TRY(hipEventRecord(h->kev[3 * j], h->stream));
            if ((rc = launch_round(h, h->next_kernel + i, nullptr, timing && !group && i % every == 0, j, 0, nr)))
                return rc;
            i += nr;
            if (group && (i % every == 0 || i == B)) {
                HIP_TRY(hipEventRecord(h->kev[3 * j + 1], h->stream));
                HIP_TRY(hipEventRecord(h->kev[3 * j + 2], h->stream));
            }
        }
        h->next_kernel += B;
        // total[] of the last round this batch applied (F(k) applies round k, or k-1 for gossip),
        // and the total[] entries of the rounds this batch completed, written by the same kernel
        // into host-mapped memory (a device-to-host copy after it cost ~0.3 ms of queue time per
        // batch: profiles/round3/c3/rocprof_kernel_stats_whole_run.csv, round 3)
        if (B > h->h_trace_cap) {
            if (h->h_trace) (void)hipHostFree(h->h_trace);
            h->h_trace = nullptr;
            h->d_trace = nullptr;
            HIP_TRY(hipHostMalloc((void**)&h->h_trace, (size_t)B * sizeof(unsigned long long),
                                  hipHostMallocMapped | hipHostMallocCoherent));
            HIP_TRY(hipHostGetDevicePointer((void**)&h->d_trace, h->h_trace, 0));
            h->h_trace_cap = B;
        }
        launch_finalize(h->total, h->parts, h->next_kernel - (h->gossip ? 2 : 1), h->stream, h->d_trace, h->rounds,
                        h->tiles);
        const bool sp_read = h->gsp.hl && h->sp_ran;
        if (sp_read) {  // the lists' counters and error word, into pinned memory
            HIP_TRY(hipMemcpyAsync(h->h_spctr, h->gsp.ctr, 3 * 4 * kSpStride * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   h->stream));
            HIP_TRY(hipMemcpyAsync(h->h_spctr + 3 * 4 * kSpStride, h->gsp.err, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   h->stream));
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(h->stream));
        if (sp_read && h->h_spctr[3 * 4 * kSpStride]) return fail(GP_EHIP, "k_gs_sparse: a list overflowed its capacity");
        h->sp_ran = false;
        if (sp_read && !h->sp_frozen) {  // every round so far ran on lists: extend the bound
            const uint32_t* c = h->h_spctr;  // (copied behind the batch, before the sync)
            const int64_t s = h->next_kernel - 1;
            const uint64_t holders = (uint64_t)c[(0 * 4 + (s & 3)) * kSpStride] + c[(1 * 4 + (s & 3)) * kSpStride];
            h->sp_until = std::max(h->sp_until, sp_bound(h->gsp.cap, s, holders));
            h->sp_s = s;
            h->sp_h = holders;
        }
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
        if (group) {
            // every group that holds a real round, launches = its real rounds, so the timed launches
            // are exactly the run's rounds (the walked-actor count covers the same launches); the
            // group that reaches convergence also times the gated no-op launches after it (a few us
            // each: conservative)
            for (int64_t j = 0; j < ng; ++j) {
                const int64_t first = j * every, last = std::min<int64_t>(first + every, B) - 1;
                if (first >= real) break;
                float ms = 0.f;
                HIP_TRY(hipEventElapsedTime(&ms, h->kev[3 * j], h->kev[3 * j + 1]));
                h->k_total_ms += ms;
                h->k_launches += std::min<int64_t>(last, real - 1) - first + 1;
            }
        } else if (timing && (rc = accumulate_timing(h, (real + kTimeEvery - 1) / kTimeEvery))) {
            return rc;
        }
        if (timing) h->work_rounds += real;
        // Batches double up to 256 rounds; once 31/32 of the nodes have reported, the run is in
        // its tail and the batch shrinks to GP_TAIL_BATCH, so fewer rounds are launched past
        // convergence (each exits at its gate, but still costs a launch).  A tail batch that
        // completed no node doubles again (a long quiet tail, e.g. line gossip, would otherwise
        // pay a host sync every GP_TAIL_BATCH rounds).
        const bool tail = kTailBatch > 0 && h->completed * 32 >= h->lay.nodes * 31;
        if (!tail || h->tiny || h->tiles) h->batch = std::min<int64_t>(h->batch * 2, kMaxBatch);
        else if (!was_tail || h->completed != before) h->batch = kTailBatch;
        else h->batch = std::min<int64_t>(h->batch * 2, kMaxBatch);
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
        if ((rc = fill_sums(h, st))) return rc;
    }
    return GP_OK;
}

// ------------------------------------------------------------------ node-range shards
int partition(int64_t n_arg, int32_t topology, int32_t world, std::vector<int64_t>& b) {
    if (world < 1 || world > kMaxWorld) return fail(GP_EINVAL, "world %d outside 1..%d", world, kMaxWorld);
    int64_t nodes, actors, grid;
    int rc = sizes(n_arg, topology, &nodes, &actors, &grid);
    if (rc) return rc;
    b.assign((size_t)world + 1, 0);
    if (topology == GP_IMP3D || topology == GP_THREE_D) {  // whole z-planes; the isolated actor goes last
        const int64_t plane = grid * grid, planes = (nodes + plane - 1) / plane;
        if (planes < world) return fail(GP_EINVAL, "%lld z-planes cannot be split over %d ranks", (long long)planes, world);
        for (int q = 1; q < world; ++q) b[q] = (int64_t)q * planes / world * plane;
    } else {
        if (actors < 2LL * world) return fail(GP_EINVAL, "%lld actors cannot be split over %d ranks", (long long)actors, world);
        for (int q = 1; q < world; ++q) b[q] = (int64_t)q * actors / world;
    }
    b[world] = actors;
    return GP_OK;
}

// Entries per round from rank p to rank q are bounded by the mean + 8 sigma of their (binomial)
// distribution, or the exact maximum when that is smaller: an overflow is reported, never dropped.
// Per sub-segment (kSub of them, sub = sender block % kSub): a sub-segment sees about mean / kSub
// entries; its variance also carries the static spread of which links fall into it, hence the
// doubled variance.  Never above the exact maximum.
uint32_t entry_cap_sub(double mean, double exact_max) {
    const double m = mean / (double)kSub;
    const double c = std::ceil(m + 8.0 * std::sqrt(2.0 * m) + 64.0);
    return (uint32_t)std::max(1.0, std::min(c, exact_max));
}

// Actors of rank p whose chains share one sub-segment of its chunks (k_gs_full4x: the sub-segment of
// a block-iteration is its 1024-actor chunk index mod kSub, so one holds ceil(chunks / kSub) chunks).
int64_t gs_sub_actors(const Handle* h, int p) {
    const int64_t size_p = h->abnd[p + 1] - h->abnd[p];
    const int64_t q0 = (h->abnd[p] >> 2) & ~7LL, q1 = (h->abnd[p + 1] + 3) >> 2;
    const int64_t chunks = ((q1 - 1) >> 8) - (q0 >> 8) + 1, per_sub = (chunks + kSub - 1) / kSub;
    return std::min<int64_t>(size_p, per_sub * 1024);
}

// The chunk `full` with `cap` entries per sub-segment and a done part of `dpairs` pairs (0: every
// word); the header and the halo face are unchanged.
Chunk shaped(const Chunk& full, uint32_t cap, uint32_t dpairs) {
    Chunk c = full;
    c.cap = cap;
    c.dpairs = full.done ? dpairs : 0u;
    size_t off = c.tail;
    if (full.done) {
        c.done = off;
        off = align_up(off + (c.dpairs ? (size_t)c.dpairs * 2 * sizeof(uint32_t) : (size_t)c.dwords * sizeof(uint32_t)));
    }
    c.slot = off;
    off = align_up(off + (size_t)kSub * cap * sizeof(uint32_t));
    c.msg = 0;
    if (full.msg) {
        c.msg = off;
        off = align_up(off + (size_t)kSub * cap * sizeof(double2));
    }
    c.size = off;
    return c;
}

// Chunk p -> q of piece i: the header; the halo face when the piece holds it (p's first plane, in its
// first piece, to p-1; its last plane, in its last piece, to p+1); the entries of the piece's senders.
Chunk chunk_layout(const Handle* h, int p, int q, int i) {
    Chunk c;
    size_t off = kAlign;  // ShardHeader
    const int64_t size_p = h->abnd[p + 1] - h->abnd[p];
    if (h->halo && ((q == p - 1 && i == 0) || (q == p + 1 && i == h->npiece - 1))) {
        c.halo = (uint32_t)std::min<int64_t>(h->halo, size_p);
        c.hdir = off;
        off = align_up(off + c.halo);
        if (!h->gossip) {
            // each face actor crosses with probability 1/degree (one uniform draw per round)
            const int64_t first = q < p ? h->abnd[p] : h->abnd[p + 1] - c.halo;
            double mean = 0.0;
            for (int64_t u = first; u < first + c.halo; ++u) {
                const uint32_t m = presence(h->g, (uint32_t)u);
                if (m) mean += 1.0 / (double)__builtin_popcount(m);
            }
            c.hcap = entry_cap_sub(mean, (double)c.halo);
            c.hslot = off;
            off = align_up(off + (size_t)kSub * c.hcap * sizeof(uint32_t));
            c.hmsg = off;
            off = align_up(off + (size_t)kSub * c.hcap * sizeof(double2));
        }
    }
    c.tail = off;
    if (h->full && h->gossip) {  // the sender's done-bitmap words, words (lo_p >> 5) .. ((hi_p - 1) >> 5)
        c.done = off;
        c.dwords = (uint32_t)(((h->abnd[p + 1] - 1) >> 5) - (h->abnd[p] >> 5) + 1);
    }
    double mean = 0.0, exact = 0.0;
    if (h->full) {
        // every chain of p draws a target uniform over the other actors, and on "full" an actor holds
        // one chain at most (the leader's kick-off is its first receipt, program.fs:218, so no actor
        // gains a second one, :99-100).  A sub-segment sees the chains of gs_sub_actors actors:
        // entry_cap_sub gets kSub times that
        const double share = (double)(h->abnd[q + 1] - h->abnd[q]) / (double)h->lay.nodes;
        const double chains = (double)gs_sub_actors(h, p);
        mean = (double)kSub * chains * share;
        exact = chains;  // one sub-segment's bound
    } else if (h->g.has_link) {
        for (int d = 1; d < 8; ++d) {
            // the link counts are per piece of kpiece; the round's only piece holds them all
            double n = 0.0;
            for (int j = h->npiece > 1 ? i : 0; j < (h->npiece > 1 ? i + 1 : h->kpiece); ++j)
                n += (double)h->lhist[(((size_t)p * h->kpiece + j) * h->world + q) * 8 + d];
            const double pick = h->gossip ? 1.0 - (1.0 - 1.0 / d) * (1.0 - 1.0 / d) : 1.0 / d;
            mean += n * pick;
            exact += n;
        }
    }
    c.cap = entry_cap_sub(mean, exact);
    if (exact == 0.0) c.cap = 0;
    if (!h->gossip) c.msg = 1;  // (shaped() places the messages)
    return shaped(c, c.cap, 0);
}

// The current plan: chunk (piece i, peer q), index c = i * world + q, with the link capacities
// out_cap[c] / in_cap[c] (the full plan's at most) and done parts of out_dp[c] / in_dp[c] pairs (0:
// every word), packed piece-major from offset 0 of the send / receive buffers.
void apply_plan(Handle* h, const std::vector<uint32_t>& out_cap, const std::vector<uint32_t>& in_cap,
                const std::vector<uint32_t>* out_dp = nullptr, const std::vector<uint32_t>* in_dp = nullptr) {
    const int W = h->world, K = h->npiece;
    int64_t so = 0, ro = 0;
    for (int i = 0; i < K; ++i) {
        h->out_poff[i] = so;
        h->in_poff[i] = ro;
        h->max_in_cap[i] = 0;
        for (int q = 0; q < W; ++q) {
            const size_t c = (size_t)i * W + q;
            if (q != h->rank) {
                h->out_chunk[c] = shaped(h->full_out[c], std::min(out_cap[c], h->full_out[c].cap), out_dp ? (*out_dp)[c] : 0u);
                h->in_chunk[c] = shaped(h->full_in[c], std::min(in_cap[c], h->full_in[c].cap), in_dp ? (*in_dp)[c] : 0u);
                h->max_in_cap[i] = std::max(h->max_in_cap[i], h->in_chunk[c].cap);
            }
            h->out_off[c] = so;
            h->in_off[c] = ro;
            so += (int64_t)h->out_chunk[c].size;
            ro += (int64_t)h->in_chunk[c].size;
        }
    }
    h->out_poff[K] = so;
    h->in_poff[K] = ro;
}

void full_plan(Handle* h) {
    const size_t n = (size_t)h->npiece * h->world;
    std::vector<uint32_t> o(n), i(n);
    for (size_t c = 0; c < n; ++c) {
        o[c] = h->full_out[c].cap;
        i[c] = h->full_in[c].cap;
    }
    apply_plan(h, o, i);
}

// The full plan of a round in K pieces (1 or kpiece) becomes the current layout.
void use_layout(Handle* h, int K) {
    const int W = h->world;
    const size_t n = (size_t)K * W;
    h->npiece = K;
    h->full_out = h->full_by[K > 1][0];
    h->full_in = h->full_by[K > 1][1];
    h->out_chunk.assign(n, Chunk{});
    h->in_chunk.assign(n, Chunk{});
    h->out_off.assign(n, 0);
    h->in_off.assign(n, 0);
    h->out_poff.assign((size_t)K + 1, 0);
    h->in_poff.assign((size_t)K + 1, 0);
    h->max_in_cap.assign((size_t)K, 0u);
    full_plan(h);
}

// Pieces while the run is before half its nodes converged (the full plan's exchange), one piece after.
int want_pieces(const Handle* h) {
    return h->kpiece > 1 && !h->converged && h->completed * 2 < h->lay.nodes ? h->kpiece : 1;
}

int build_plan(Handle* h) {
    const int W = h->world, p = h->rank;
    int64_t st = 0, rt = 0;
    for (int K : {1, h->kpiece}) {
        h->npiece = K;
        std::vector<Chunk>& fo = h->full_by[K > 1][0];
        std::vector<Chunk>& fi = h->full_by[K > 1][1];
        fo.assign((size_t)K * W, Chunk{});
        fi.assign((size_t)K * W, Chunk{});
        for (int i = 0; i < K; ++i)
            for (int q = 0; q < W; ++q)
                if (q != p) {
                    fo[(size_t)i * W + q] = chunk_layout(h, p, q, i);
                    fi[(size_t)i * W + q] = chunk_layout(h, q, p, i);
                }
        use_layout(h, K);
        st = std::max(st, h->out_poff[K]);  // the buffers hold either layout's full plan
        rt = std::max(rt, h->in_poff[K]);
        if (h->kpiece == 1) break;
    }
    h->send_total = st;
    h->recv_total = rt;
    if (refs(h) && (uint64_t)rt / 16u >= (1ull << (32 - kRefShift)))
        return fail(GP_ENOMEM, "a receive buffer of %lld bytes is past the slot references' reach", (long long)rt);
    int rc;
    if ((rc = h->alloc(&h->pcount, ((size_t)W + 2) * kSub * kCtrStride)) || (rc = h->alloc(&h->overflow, 1)) ||
        (rc = h->alloc(&h->self_newly, 1)) || (rc = h->alloc(&h->pmax, (size_t)kMaxPieces * kMaxWorld)) ||
        (rc = h->alloc(&h->xfin, (size_t)(kFinGroups + 1) * kFinStride)))
        return rc;
    HIP_TRY(hipMemsetAsync(h->xfin, 0, (size_t)(kFinGroups + 1) * kFinStride * sizeof(uint32_t), h->stream));
    return GP_OK;
}

// Exchange descriptor with every device pointer except the buffers.
Xchg base_xchg(const Handle* h) {
    Xchg x{};
    x.world = (uint32_t)h->world;
    x.rank = (uint32_t)h->rank;
    for (int q = 0; q <= h->world && q <= kMaxWorld; ++q) {
        x.abnd[q] = (uint32_t)h->abnd[q];
        x.sbnd[q] = q < (int)h->sbnd.size() ? (uint32_t)h->sbnd[q] : 0u;
    }
    x.pcount = h->pcount;
    x.overflow = h->overflow;
    x.self_newly = h->self_newly;
    x.pmax = h->pmax;
    x.slot_dst = h->slot_dst;
    x.self_chains = h->self_chains;
    x.pstat = h->pstat;
    x.dship = h->dship;
    x.dstat = h->dstat;
    x.binned = h->bin_next ? 1u : 0u;
    x.fin = h->xfin;
    return x;
}

// The exchange descriptor of piece i (the round's only piece unless it runs in pieces).
Xchg make_xchg(const Handle* h, void* send, const void* recv, int i = 0) {
    Xchg x = base_xchg(h);
    const int W = h->world;
    x.last = i == h->npiece - 1 ? 1u : 0u;
    x.rbase = static_cast<const char*>(recv);
    x.pmax = h->pmax + (size_t)i * kMaxWorld;
    for (int q = 0; q < h->world; ++q) {
        if (q == h->rank) continue;
        if (send) {
            char* b = static_cast<char*>(send) + h->out_off[(size_t)i * W + q];
            const Chunk& c = h->out_chunk[(size_t)i * W + q];
            x.out[q] = PeerOut{reinterpret_cast<ShardHeader*>(b), reinterpret_cast<uint32_t*>(b + c.slot),
                               c.msg ? reinterpret_cast<double2*>(b + c.msg) : nullptr, c.cap, c.dpairs,
                               c.done ? reinterpret_cast<uint32_t*>(b + c.done) : nullptr};
        }
        if (recv) {
            const char* b = static_cast<const char*>(recv) + h->in_off[(size_t)i * W + q];
            const Chunk& c = h->in_chunk[(size_t)i * W + q];
            x.in[q] = PeerIn{reinterpret_cast<const ShardHeader*>(b), reinterpret_cast<const uint32_t*>(b + c.slot),
                             c.msg ? reinterpret_cast<const double2*>(b + c.msg) : nullptr, c.cap, c.dpairs,
                             c.done ? reinterpret_cast<const uint32_t*>(b + c.done) : nullptr};
        }
    }
    // halo faces (side 0: rank-1, side 1: rank+1); the crossing code is -x/+x on a line, -z/+z on a grid
    const int p = h->rank;
    for (int side = 0; side < 2; ++side) {
        const int q = side ? p + 1 : p - 1;
        if (q < 0 || q >= h->world) continue;
        x.h.code[side] = h->g.gz > 1 ? (side ? 5u : 4u) : (side ? 1u : 0u);
        const size_t c = (size_t)i * W + q;  // (a face travels in one piece only: chunk_layout)
        const Chunk& co = h->out_chunk[c];
        if (send && co.halo) {
            char* b = static_cast<char*>(send) + h->out_off[c];
            x.h.out_n[side] = co.halo;
            x.h.out_first[side] = side ? h->hi - co.halo : h->lo;
            x.h.out_cap[side] = co.hcap;
            x.h.out_dir[side] = reinterpret_cast<uint8_t*>(b + co.hdir);
            if (co.hcap) {
                x.h.out_slot[side] = reinterpret_cast<uint32_t*>(b + co.hslot);
                x.h.out_msg[side] = reinterpret_cast<double2*>(b + co.hmsg);
            }
        }
        const Chunk& ci = h->in_chunk[c];
        if (recv && ci.halo) {
            const char* b = static_cast<const char*>(recv) + h->in_off[c];
            x.h.in_n[side] = ci.halo;
            x.h.in_first[side] = side ? h->hi : h->lo - ci.halo;
            x.h.in_cap[side] = ci.hcap;
            x.h.in_hdr[side] = reinterpret_cast<const ShardHeader*>(b);
            x.h.in_dir[side] = reinterpret_cast<const uint8_t*>(b + ci.hdir);
            if (ci.hcap) {
                x.h.in_slot[side] = reinterpret_cast<const uint32_t*>(b + ci.hslot);
                x.h.in_msg[side] = reinterpret_cast<const double2*>(b + ci.hmsg);
            }
        }
    }
    return x;
}

// Index of the round F(k) applies (its completion count), -1 for gossip's emit-only F(0).
long long applied_round(const Handle* h, int64_t k) { return h->gossip ? (long long)k - 1 : (long long)k; }

// A push-sum shard's tail round writes its halo faces in its round kernel (k_ps_quiet_x<true>,
// DESIGN.md §6.12): the rounds that are certainly tail rounds, by the rule that drops the link
// scatter (launch_aux), with links (the kernel that walks them) and one piece.
bool halo_inline(const Handle* h, int64_t k) {
    return !h->gossip && !h->generic && h->g.has_link && h->halo && h->npiece == 1 && h->act[0] && h->act_thr &&
           h->completed >= (int64_t)h->act_thr && k >= h->rounds + 1;
}

// Piece `piece` of round k: its round kernel and link pass, the halo face it holds, its headers.  The
// pieces of a round are packed in order; the last one completes the round (gp_shard_deliver next).
int shard_round_piece(Handle* h, void* send, int piece) {
    if (h->awaiting_deliver) return fail(GP_ESTATE, "gp_shard_deliver must follow gp_shard_round");
    if (piece != h->piece_next)
        return fail(GP_ESTATE, "piece %d packed out of order (next: %d of %d)", piece, h->piece_next, h->npiece);
    if (!send && h->send_total) return fail(GP_EINVAL, "null send buffer");
    if (reinterpret_cast<uintptr_t>(send) % kAlign) return fail(GP_EINVAL, "send buffer not %zu-byte aligned", kAlign);
    const bool timing = (h->cfg.flags & GP_FLAG_KERNEL_TIMING) != 0;
    const int64_t k = h->next_kernel;
    int rc;
    if (piece == 0) {
        if ((rc = ensure_trace(h, k + 4))) return rc;
        // kernel timing samples every kTimeEvery-th round (event records cost stream time)
        h->round_slot = -1;
        if (timing && k >= (h->gossip ? 1 : 0) && k % kTimeEvery == 0) {
            if ((rc = ensure_events(h, h->timed_count + 1))) return rc;
            h->timed_round.resize((size_t)h->timed_count + 1);
            h->timed_round[(size_t)h->timed_count] = applied_round(h, k);
            h->round_slot = h->timed_count++;
        }
    }
    Xchg x = make_xchg(h, send, nullptr, piece);
    x.hin = halo_inline(h, k) ? 1u : 0u;
    if ((rc = launch_round(h, k, &x, h->round_slot >= 0, std::max<int64_t>(h->round_slot, 0), piece))) return rc;
    const RoundArgs a = h->args((uint32_t)k);
    // the halo face this piece holds (the rank's first actors to rank-1, its last to rank+1), then the
    // headers
    if (!x.hin) launch_shard_halo(a, x, h->gossip ? 0 : 1, h->stream);
    // (a full-gossip list round and a push-sum tail round with the halo faces inline packed themselves)
    if (h->sp_fused != k && !x.hin) launch_shard_pack(a, x, applied_round(h, k), h->stream);
    HIP_TRY(hipGetLastError());
    for (int q = 0; q < h->world; ++q) h->bytes_sent += (int64_t)h->out_chunk[(size_t)piece * h->world + q].size;
    if (++h->piece_next == h->npiece) {
        h->piece_next = 0;
        h->awaiting_deliver = true;
        h->pending_send = send;
    }
    return GP_OK;
}

int shard_round(Handle* h, void* send) {
    if (h->piece_next) return fail(GP_ESTATE, "gp_shard_round in the middle of a round's pieces");
    for (int i = 0; i < h->npiece; ++i) {
        const int rc = shard_round_piece(h, send, i);
        if (rc) return rc;
    }
    return GP_OK;
}

int shard_deliver(Handle* h, const void* recv) {
    if (!h->awaiting_deliver) return fail(GP_ESTATE, "gp_shard_deliver without gp_shard_round");
    if (!recv && h->recv_total) return fail(GP_EINVAL, "null receive buffer");
    if (reinterpret_cast<uintptr_t>(recv) % kAlign) return fail(GP_EINVAL, "receive buffer not %zu-byte aligned", kAlign);
    // round k + 1 reads round k's remote messages where they arrived; in pieces the
    // next round's exchange overlaps that round's kernels, so the host alternates two buffers
    if (refs(h) && h->npiece > 1 && recv && recv == h->msg_src)
        return fail(GP_EINVAL, "in pieces consecutive rounds need different receive buffers (the next round reads this one)");
    const int64_t k = h->next_kernel;
    // one kernel per piece applies its halo face (rank-1's last actors land below lo, rank+1's first
    // at hi) and link entries; the last publishes the round's count
    for (int i = 0; i < h->npiece; ++i) {
        const Xchg x = make_xchg(h, h->pending_send, recv, i);
        // the grid covers the largest per-peer part: link entries, a halo face, or (full gossip) a
        // peer's done-bitmap words, which arrive whole whatever the plan
        // (the halo faces travel in the end pieces; the whole grid strides over a face, so it needs
        // 1/world of it per peer: a tail round's grid was world x the face in workgroups, 3 us of a
        // 16 us unpack at 100M / 8, profiles/round5/unpack_grid/)
        const bool face = i == 0 || i == h->npiece - 1;
        const uint32_t per_face = (h->halo + (uint32_t)h->world - 1u) / (uint32_t)h->world;
        uint32_t most = std::max(kSub * h->max_in_cap[i], face ? per_face : 0u);
        if (h->gossip && h->full)  // a peer's done part: its pairs' capacity, or every word of its range
            for (int q = 0; q < h->world; ++q) {
                const Chunk& c = h->in_chunk[(size_t)i * h->world + q];
                if (q == h->rank || !c.done) continue;
                most = std::max(most, c.dpairs ? c.dpairs : (uint32_t)((h->abnd[q + 1] - h->abnd[q]) / 32 + 2));
            }
        // F(k) ran on lists (no walk over every actor enqueued yet): the peers' first receipts list
        // their targets for F(k + 1)
        const GsSparse sp = h->gsp.hl && !h->sp_frozen ? h->gsp : GsSparse{};
        launch_shard_unpack(h->args((uint32_t)k), x, applied_round(h, k), most, h->gossip ? 1 : 0, h->full ? 1 : 0, sp,
                            h->stream);
        if (x.binned) launch_shard_unpack_bins(h->args((uint32_t)k), x, h->bins, h->stream);  // the receipts in bins
    }
    HIP_TRY(hipGetLastError());
    h->awaiting_deliver = false;
    h->last_recv = recv;
    if (refs(h)) h->msg_src = recv;
    ++h->delivered;
    h->next_kernel = k + 1;
    if (gossip_plans(h)) gossip_round_plan(h, h->next_kernel);  // full gossip: a plan per round
    return GP_OK;
}

// ---- activity tiers (push-sum shards of several ranks)
// The link entries a rank sends per round follow the run's activity: every actor sends while it
// updates, and in the converged tail only relayed messages move (a few per cent of the actors), yet
// the full plan ships the capacity of an all-sending round (C5 / 8: ~0.31 GB per rank per round).
// At every gp_shard_sync both ends of a chunk p -> q know the most entries one of its sub-segments
// held in the batch just run (p from its own counters, q from p's last header), and size the next
// batch's chunk from it: the full capacity halved while the half still holds twice that count plus
// 64.  Counts can still outgrow a reduced chunk (overflow is detected, never silent), so a reduced
// plan runs only after a restore point: the state the next round reads, copied at a sync every
// kCkptEvery rounds.  A batch that overflowed is discarded on every rank (the overflow flag travels
// in every header) and the ranks resume from the restore point with the full plan up to the round
// the failed batch reached, so the run stays exact.  Every decision is made from values every rank
// (or both ends of a chunk) holds, so the ranks agree without an extra exchange.
constexpr int64_t kCkptEvery = 256;

bool tiers_on(const Handle* h) {
    // push-sum on the pull path, and full gossip (its remote receipts thin out as targets report:
    // the senders filter them on the replicated done bitmap)
    const bool ps = !h->gossip && !h->generic, fg = h->gossip && h->full;
    return h->sharded && h->world > 1 && (ps || fg) && !(h->cfg.flags & GP_FLAG_FULL_PLAN);
}


uint32_t tier_cap(uint32_t full, uint32_t m, bool tight) {
    const uint64_t need = tight ? (uint64_t)m : 2ull * m + 64u;
    uint32_t c = full;
    while (c > 1u && (uint64_t)((c + 1u) / 2u) >= need && (c + 1u) / 2u < c) c = (c + 1u) / 2u;
    return c;
}

// ---- full gossip shards: a plan per round
// A full-gossip run ramps up (chains double per round for ~log2(actors) rounds, nearly nothing moves),
// saturates (every actor sends), then thins out as targets report and the senders filter them; a
// batch-wide plan ships the saturated capacity through the ramp.  Here each round k gets its own
// plan, computed alike at both ends of a chunk from values both hold:
//   * entries: round k's chains are at most cj * 2^(k - j) (a new chain needs a receipt, and a receipt
//     a chain), the chain holders are uniform over the actors, so a sub-segment of p -> q holds at most
//     mean + 8 sigma + 64 of that bound's share (the full plan's own rule), and, once a round was
//     seen, at most twice its largest sub-segment scaled by the same growth, plus 64;
//   * done words: the dirty words of the last round, doubled, plus 64, as (index, word) pairs, or
//     every word once pairs would cost as much.  Words past the capacity wait (k_shard_done_out).
// Counts can outgrow a sized chunk (statistics, not bounds): overflow is detected, and the batch
// replays from the restore point with the full plan, as under the push-sum tiers.
bool gossip_plans(const Handle* h) { return h->sharded && h->world > 1 && h->gossip && h->full; }

uint32_t gs_cap(const Handle* h, int p, int q, int64_t k, uint32_t m, uint32_t full_cap) {
    const Handle::GossipPlan& P = h->gpl;
    if (!P.on) return full_cap;
    const bool tight = (h->cfg.flags & GP_FLAG_TIGHT_TIERS) != 0;
    const double A = (double)h->g.actors;
    const int64_t dk = std::max<int64_t>(k - P.j, 0);
    const double cb = dk >= 62 ? A : std::min(A, P.cj * std::ldexp(1.0, (int)dk));
    const double n_sub = (double)gs_sub_actors(h, p);
    const double share = (double)(h->abnd[q + 1] - h->abnd[q]) / (double)h->lay.nodes;
    const double mean = cb * n_sub / A * share;
    double c = tight ? std::ceil(mean) : (double)entry_cap_sub((double)kSub * mean, std::min(cb, n_sub));
    if (P.seen) {
        const double grow = P.cj > 0.0 ? cb / P.cj : 1.0;
        c = std::min(c, tight ? std::ceil((double)m * grow) : std::ceil(2.0 * (double)m * grow + 64.0));
    }
    return (uint32_t)std::min(c, (double)full_cap);
}

uint32_t gs_dpairs(const Handle* h, int p, uint32_t dw) {
    if (!h->gpl.on) return 0u;
    const bool tight = (h->cfg.flags & GP_FLAG_TIGHT_TIERS) != 0;
    // the report wave (from 1/1024 of the nodes reported until 1/64 are left): nearly every word
    // changes every round, and a stale replica weakens the sender filter just as it turns on (1/16):
    // every word, so the replicas stay a round behind at most
    const int64_t n = h->lay.nodes, c = h->completed;
    if (!tight && c * 1024 >= n && (n - c) * 64 >= n) return 0u;
    const uint64_t nw = (uint64_t)(((h->abnd[p + 1] - 1) >> 5) - (h->abnd[p] >> 5) + 1);
    const uint64_t d = tight ? dw / 2u + 1u : 2ull * dw + 64u;  // tight: a backlog in most rounds
    return 2u * d >= nw ? 0u : (uint32_t)d;
}

// Whether round k's receipts travel in bins (GsBins): while the round's receipts, estimated from the
// synced values every rank holds (the chain bound of gs_cap times the share of nodes not done), are at
// least actors / GP_BIN_DIV, once per run (the wave); never in a list round (GP_FLAG_GOSSIP_TALLY: every
// other round from round 1, a test hook).
bool bins_round(Handle* h, int64_t k) {
    if (!h->bins.cnt || k < 1) return false;
    if (h->gsp.hl && !h->sp_frozen && k < h->sp_until) return false;
    if (h->cfg.flags & GP_FLAG_GOSSIP_TALLY) return true;
    if (h->bin_state == 2) return false;
    const Handle::GossipPlan& P = h->gpl;
    const double A = (double)h->g.actors, n = (double)h->lay.nodes;
    const int64_t dk = std::max<int64_t>(k - P.j, 0);
    const double cb = dk >= 62 ? A : std::min(A, P.cj * std::ldexp(1.0, (int)dk));
    const bool on = cb * ((n - (double)h->completed) / n) * GP_BIN_DIV >= A;
    if (on) h->bin_state = 1;
    else if (h->bin_state == 1) h->bin_state = 2;
    return on;
}

uint32_t bins_of(const Handle* h, int q) {
    return (uint32_t)((h->abnd[q + 1] - h->abnd[q] + (1 << kTallyShift) - 1) >> kTallyShift);
}

// Round k's plan (k = the next round gp_shard_round packs).
void gossip_round_plan(Handle* h, int64_t k) {
    const int W = h->world, p = h->rank;
    const Handle::GossipPlan& P = h->gpl;
    h->bin_next = bins_round(h, k);
    std::vector<uint32_t> oc((size_t)W, 0u), ic((size_t)W, 0u), od((size_t)W, 0u), id((size_t)W, 0u);
    for (int q = 0; q < W; ++q) {
        if (q == p) continue;
        oc[q] = gs_cap(h, p, q, k, P.seen ? P.m_out[q] : 0u, h->full_out[q].cap);
        ic[q] = gs_cap(h, q, p, k, P.seen ? P.m_in[q] : 0u, h->full_in[q].cap);
        if (h->bin_next) {  // u16 entries: half the words, and the receiver's bin starts beside them
            oc[q] = (oc[q] + 1) / 2 + (bins_of(h, q) + kSub) / kSub;
            ic[q] = (ic[q] + 1) / 2 + (bins_of(h, p) + kSub) / kSub;
        }
        od[q] = gs_dpairs(h, p, P.seen ? P.dw_out : 0u);
        id[q] = gs_dpairs(h, q, P.seen ? P.dw_in[q] : 0u);
    }
    apply_plan(h, oc, ic, &od, &id);
}

int ensure_ckpt(Handle* h) {
    Ckpt& c = h->ck;
    if (c.allocated) return GP_OK;
    const size_t xn = (size_t)(h->ext_hi() - h->ext_lo()), n = h->own();
    int rc;
    if (h->gossip) {  // full gossip
        if ((rc = h->alloc(&c.cnt, n)) || (rc = h->alloc(&c.gstate, n)) || (rc = h->alloc(&c.inc, n)) ||
            (rc = h->alloc(&c.dbits, dbits_words_all(h))) || (h->dship && (rc = h->alloc(&c.dship, dship_words(h)))))
            return rc;
        if (h->dsum && (rc = h->alloc(&c.dsum, dsum_words_all(h)))) return rc;
        c.allocated = true;
        return GP_OK;
    }
    const size_t nsl = (size_t)(h->sbnd.empty() ? 0 : h->sbnd[h->rank + 1] - h->sbnd[h->rank]);
    if ((rc = h->alloc(&c.msg, xn)) || (rc = h->alloc(&c.dir, xn)) || (rc = h->alloc(&c.flags, n))) return rc;
    if (h->work && (rc = h->alloc(&c.work, (size_t)kParts * kWorkStride))) return rc;
    if (h->lcnt[0] && (rc = h->alloc(&c.lcnt, nsl))) return rc;
    if (h->lref[0] && ((rc = h->alloc(&c.lref, nsl)) || (rc = h->alloc(&c.rin, (size_t)std::max<int64_t>(h->recv_total, 1)))))
        return rc;
    if (h->act[0] && (rc = h->alloc(&c.act, act_bytes(h)))) return rc;
    c.allocated = true;
    return GP_OK;
}

// Copy the state F(k0) reads (k0 = next_kernel) into (save) or out of (!save) the restore point.
int ckpt_copy(Handle* h, bool save) {
    Ckpt& c = h->ck;
    const int64_t k0 = h->next_kernel;
    const int p = (int)((k0 + 1) & 1);  // parity of round k0 - 1
    const size_t xlo = (size_t)h->ext_lo(), xn = (size_t)(h->ext_hi() - h->ext_lo()), lo = h->lo, n = h->own();
    hipStream_t s = h->stream;
    auto cp = [&](void* live, void* saved, size_t bytes) {
        return save ? hipMemcpyAsync(saved, live, bytes, hipMemcpyDeviceToDevice, s)
                    : hipMemcpyAsync(live, saved, bytes, hipMemcpyDeviceToDevice, s);
    };
    if (h->gossip) {  // full gossip: F(k0) reads cnt, gstate, the receipts of round k0-1 and the replica
        HIP_TRY(cp(h->cnt + lo, c.cnt, n * sizeof(uint32_t)));
        HIP_TRY(cp(h->gstate + lo, c.gstate, n));
        HIP_TRY(cp(h->inc[p] + lo, c.inc, n * sizeof(uint32_t)));
        HIP_TRY(cp(h->dbits, c.dbits, dbits_words_all(h) * sizeof(uint32_t)));
        if (h->dsum) HIP_TRY(cp(h->dsum, c.dsum, dsum_words_all(h) * sizeof(uint32_t)));
        if (h->dship) HIP_TRY(cp(h->dship + (lo >> 5), c.dship, dship_words(h) * sizeof(uint32_t)));
        // round k0's receipts accumulate in the other array, empty before F(k0): a failed batch's go
        if (!save) HIP_TRY(hipMemsetAsync(h->inc[p ^ 1] + lo, 0, n * sizeof(uint32_t), s));
        if (save) {
            c.gj = h->gpl.j;
            c.gcj = h->gpl.cj;
        } else if (h->dstat) {
            // the shipping state of the restore point: no round counted, and a scan in the next round
            // (whatever was left dirty then is found again)
            HIP_TRY(hipMemsetAsync(h->dstat, 0, kDstatWords * sizeof(uint32_t), s));
            const uint32_t one = 1u;
            HIP_TRY(hipMemcpyAsync(h->dstat + kDstatLeft, &one, sizeof one, hipMemcpyHostToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));
        }
    } else {
    HIP_TRY(cp(h->msg[p] + xlo, c.msg, xn * sizeof(double2)));
    HIP_TRY(cp(h->dir[p] + xlo, c.dir, xn));
    HIP_TRY(cp(h->flags + lo, c.flags, n));
    if (h->work) HIP_TRY(cp(h->work, c.work, (size_t)kParts * kWorkStride * sizeof *h->work));
    if (h->lcnt[0]) {
        const size_t slo = (size_t)h->sbnd[h->rank], nsl = (size_t)(h->sbnd[h->rank + 1] - h->sbnd[h->rank]);
        HIP_TRY(cp(h->lcnt[p] + slo, c.lcnt, nsl));
        // the marks of round k0 land in the other array: a failed batch's are cleared
        if (!save) HIP_TRY(hipMemsetAsync(h->lcnt[p ^ 1] + slo, 0, nsl, s));
    }
    if (h->lref[0]) {  // the references of round k0-1 and the receive buffer they point into
        const size_t slo = (size_t)h->sbnd[h->rank], nsl = (size_t)(h->sbnd[h->rank + 1] - h->sbnd[h->rank]);
        HIP_TRY(cp(h->lref[p] + slo, c.lref, nsl * sizeof(uint32_t)));
        if (!save) HIP_TRY(hipMemsetAsync(h->lref[p ^ 1] + slo, 0, nsl * sizeof(uint32_t), s));
        if (save) {
            c.has_rin = h->msg_src != nullptr;
            if (c.has_rin && h->msg_src != c.rin)
                HIP_TRY(hipMemcpyAsync(c.rin, h->msg_src, (size_t)h->recv_total, hipMemcpyDeviceToDevice, s));
        } else {
            h->msg_src = c.has_rin ? c.rin : nullptr;  // F(k0) reads round k0-1's messages from the copy
        }
    }
    if (h->act[0]) HIP_TRY(cp(h->act[k0 & 1] + act_first(h), c.act, act_bytes(h)));
    }
    if (save) {
        c.next_kernel = k0;
        c.rounds = h->rounds;
        c.completed = h->completed;
        c.k_launches = h->k_launches;
        c.k_total_ms = h->k_total_ms;
        c.k_aux_ms = h->k_aux_ms;
        c.work_rounds = h->work_rounds;
        c.valid = true;
    }
    return GP_OK;
}

// Back to the restore point after an overflowed batch (every rank of the job does the same at this
// sync); the full plan until `reached` rounds are final again.
int restore(Handle* h, int64_t reached) {
    Ckpt& c = h->ck;
    h->next_kernel = c.next_kernel;
    int rc;
    if ((rc = ckpt_copy(h, false))) return rc;
    hipStream_t s = h->stream;
    HIP_TRY(hipMemsetAsync(h->parts, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t), s));
    if (h->cparts) HIP_TRY(hipMemsetAsync(h->cparts, 0, (size_t)kPartRing * kParts * kPartStride * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(h->pcount, 0, ((size_t)h->world + 2) * kSub * kCtrStride * sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(h->overflow, 0, sizeof(uint32_t), s));
    HIP_TRY(hipMemsetAsync(h->pmax, 0, (size_t)kMaxPieces * kMaxWorld * sizeof(uint32_t), s));
    HIP_TRY(hipStreamSynchronize(s));
    if (gossip_plans(h)) {  // the chain count of the restore point; no round seen since
        h->gpl.j = c.gj;
        h->gpl.cj = c.gcj;
        h->gpl.seen = false;
        h->gpl.on = false;
    }
    // the restore point holds the arrays, not the ramp's lists: the replay walks every actor
    h->sp_frozen = true;
    h->sp_fused = -1;
    h->bin_next = false;  // (the full plan's first round runs in entries; the next plans decide again)
    h->rounds = c.rounds;
    h->completed = c.completed;
    h->converged = false;
    h->k_launches = c.k_launches;
    h->k_total_ms = c.k_total_ms;
    h->k_aux_ms = c.k_aux_ms;
    h->work_rounds = c.work_rounds;
    h->timed_count = 0;
    h->full_until = std::max(h->full_until, reached);
    ++h->restores;
    h->tiered = false;
    h->delivered = 0;
    if (h->kpiece > 1) use_layout(h, want_pieces(h));
    full_plan(h);
    return GP_OK;
}

// The next batch's plan (and a restore point when one is due), at a sync with no overflow.
int choose_plan(Handle* h) {
    // a sync with no round since the last one keeps the plan (the counters would disagree: this
    // rank's were reset, the peers' last headers were not)
    if (!h->delivered) return GP_OK;
    h->delivered = 0;
    const int W = h->world, K0 = h->npiece;
    const bool tight = (h->cfg.flags & GP_FLAG_TIGHT_TIERS) != 0;
    // per (piece, peer) of the batch just run: this rank's running maxima, and the peers' from the
    // headers they sent last
    int K = K0;
    size_t n = (size_t)K * W;
    std::vector<uint32_t> pm((size_t)kMaxPieces * kMaxWorld, 0u), mo(n, 0u), mi(n, 0u);
    HIP_TRY(hipMemcpy(pm.data(), h->pmax, pm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (int i = 0; i < K; ++i)
        for (int q = 0; q < W; ++q) {
            const size_t c = (size_t)i * W + q;
            mo[c] = pm[(size_t)i * kMaxWorld + q];
            if (q != h->rank && h->last_recv)
                HIP_TRY(hipMemcpy(&mi[c], static_cast<const char*>(h->last_recv) + h->in_off[c] + offsetof(ShardHeader, runmax),
                                  sizeof(uint32_t), hipMemcpyDeviceToHost));
        }
    HIP_TRY(hipMemsetAsync(h->pmax, 0, (size_t)kMaxPieces * kMaxWorld * sizeof(uint32_t), h->stream));
    // the pieces of the next batch (a global decision); the counts carry over: a round's pieces
    // held together at most the sum of their counts, and one piece at most the whole round's
    if (want_pieces(h) != K0) {
        K = want_pieces(h);
        const size_t n1 = (size_t)K * W;
        std::vector<uint32_t> mo1(n1, 0u), mi1(n1, 0u);
        for (int i = 0; i < std::max(K, K0); ++i)
            for (int q = 0; q < W; ++q) {
                const size_t c0 = (size_t)(K0 > 1 ? i : 0) * W + q, c1 = (size_t)(K > 1 ? i : 0) * W + q;
                if (K > 1) {  // every piece as much as the whole round
                    mo1[c1] = mo[c0];
                    mi1[c1] = mi[c0];
                } else {
                    mo1[c1] += mo[c0];
                    mi1[c1] += mi[c0];
                }
            }
        mo.swap(mo1);
        mi.swap(mi1);
        n = n1;
        use_layout(h, K);
    }
    // global conditions only (every rank decides alike): half the nodes converged (the tail), no
    // replay in progress, a batch already run
    const bool on = !h->converged && h->last_recv && h->rounds >= h->full_until &&
                    (tight || h->completed * 2 >= h->lay.nodes);
    std::vector<uint32_t> oc(n), ic(n);
    for (size_t c = 0; c < n; ++c) {
        oc[c] = on ? tier_cap(h->full_out[c].cap, mo[c], tight) : h->full_out[c].cap;
        ic[c] = on ? tier_cap(h->full_in[c].cap, mi[c], tight) : h->full_in[c].cap;
    }
    int rc;
    if (on && (!h->ck.valid || tight || h->rounds - h->ck.rounds >= kCkptEvery)) {
        if ((rc = ensure_ckpt(h)) || (rc = ckpt_copy(h, true))) return rc;
    }
    h->tiered = on;
    bool changed = false;
    for (size_t c = 0; c < n; ++c) changed |= oc[c] != h->out_chunk[c].cap || ic[c] != h->in_chunk[c].cap;
    if (changed) {
        apply_plan(h, oc, ic);
        ++h->plan_changes;
    }
    return GP_OK;
}

// Full gossip: the inputs of the next rounds' plans (the last round's counts), a restore point when
// one is due, and the plan of the next round.
int gossip_sync(Handle* h) {
    Handle::GossipPlan& P = h->gpl;
    const bool tight = (h->cfg.flags & GP_FLAG_TIGHT_TIERS) != 0;
    if (h->delivered && h->last_recv) {
        h->delivered = 0;
        uint32_t ps[kPstatWords];
        HIP_TRY(hipMemcpy(ps, h->pstat, sizeof ps, hipMemcpyDeviceToHost));
        unsigned long long c;
        std::memcpy(&c, ps + kPsChains, sizeof c);
        P.j = h->next_kernel - 1;  // the chains F(next_kernel - 1) emitted
        P.cj = (double)c;
        // the ramp on lists: every rank's chain holders after F(j) bound this rank's lists (one chain per
        // holder on "full"), so every rank extends its bound alike
        if (h->gsp.hl && !h->sp_frozen) {
            h->sp_until = std::max(h->sp_until, sp_bound(h->gsp.cap, P.j, c));
            h->sp_s = P.j;
            h->sp_h = c;
        }
        P.dw_out = ps[kPsDirty];
        for (int q = 0; q < h->world; ++q) {
            P.m_out[q] = ps[kPsOut + q];
            P.m_in[q] = ps[kPsIn + q];
            P.dw_in[q] = ps[kPsDwIn + q];
        }
        P.seen = true;
    }
    P.on = tiers_on(h) && !h->converged && h->rounds >= h->full_until;
    if (P.on && (!h->ck.valid || tight || h->rounds - h->ck.rounds >= kCkptEvery)) {
        int rc;
        if ((rc = ensure_ckpt(h)) || (rc = ckpt_copy(h, true))) return rc;
    }
    h->tiered = P.on;
    gossip_round_plan(h, h->next_kernel);
    ++h->plan_changes;
    return GP_OK;
}

int shard_sync(Handle* h, gp_status* st) {
    if (h->awaiting_deliver) return fail(GP_ESTATE, "gp_shard_sync between gp_shard_round and gp_shard_deliver");
    HIP_TRY(hipStreamSynchronize(h->stream));
    uint32_t of = 0;
    HIP_TRY(hipMemcpy(&of, h->overflow, sizeof of, hipMemcpyDeviceToHost));
    if (of & 2u) return fail(GP_EOVERFLOW, "a shard received an entry outside its range; the run is void");
    if (h->gsp.hl && h->sp_ran) {  // (a list cannot outgrow its bound: the counts are exact)
        uint32_t e = 0;
        HIP_TRY(hipMemcpy(&e, h->gsp.err, sizeof e, hipMemcpyDeviceToHost));
        if (e) return fail(GP_EHIP, "k_gs_sparse_x: a list overflowed its capacity");
        h->sp_ran = false;
    }
    const int64_t applied = (int64_t)applied_round(h, h->next_kernel - 1) + 1;  // rounds whose counts exist
    int rc;
    if (of) {
        // only a batch that may have run reduced chunks is replayed (every rank agrees on that); an
        // overflow of the full plan is fatal, as its replay would overflow again
        if (!(tiers_on(h) && h->tiered && h->ck.valid))
            return fail(GP_EOVERFLOW, "a shard exchange buffer overflowed; the run is void");
        if ((rc = restore(h, applied))) return rc;  // a reduced plan overflowed: replay with the full plan
        if (st) {
            std::memset(st, 0, sizeof *st);
            st->round = h->rounds;
            st->completed = h->completed;
            st->converged = 0;
            if ((rc = fill_sums(h, st))) return rc;
        }
        return GP_OK;
    }
    int64_t timed_real = h->converged ? 0 : h->timed_count;  // after convergence no round is real
    if (!h->converged && applied > h->rounds) {
        const int64_t n = applied - h->rounds;
        std::vector<unsigned long long> t((size_t)n);
        HIP_TRY(hipMemcpy(t.data(), h->total + h->rounds, (size_t)n * sizeof t[0], hipMemcpyDeviceToHost));
        int64_t real = n;
        for (int64_t i = 0; i < n; ++i)
            if ((int64_t)t[i] >= h->lay.nodes) {
                real = i + 1;
                h->converged = true;
                break;
            }
        h->completed = (int64_t)t[real - 1];
        h->rounds += real;
        timed_real = 0;  // sampled kernels that applied a real round (not past convergence)
        while (timed_real < h->timed_count && h->timed_round[(size_t)timed_real] < h->rounds) ++timed_real;
    }
    if (h->timed_count && (rc = accumulate_timing(h, timed_real))) return rc;
    if (h->timed_count) h->work_rounds += timed_real;  // the quiet kernel counts in timed rounds only
    h->timed_count = 0;
    if (gossip_plans(h)) {
        if ((rc = gossip_sync(h))) return rc;
    } else if (tiers_on(h)) {
        if ((rc = choose_plan(h))) return rc;  // (the pieces of the next batch too)
    } else if (h->kpiece > 1 && want_pieces(h) != h->npiece) {
        use_layout(h, want_pieces(h));
    }
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->round = h->rounds;
        st->completed = h->completed;
        st->converged = h->converged ? 1 : 0;
        if ((rc = fill_sums(h, st))) return rc;
    }
    return GP_OK;
}

// Read-back ranges must lie in the handle's own actors (a shard holds [lo, hi) only).
int check_range(const Handle* h, int64_t first, int64_t count) {
    if (first < (int64_t)h->lo || count < 0 || first + count > (int64_t)h->hi)
        return fail(GP_EINVAL, "range [%lld, %lld) outside this handle's actors [%u, %u)", (long long)first,
                    (long long)(first + count), h->lo, h->hi);
    return GP_OK;
}

template <class T>
int copy_slice(const Handle* h, std::vector<T>& out, const T* src, int64_t first, int64_t count) {
    out.resize((size_t)count);
    if (count) HIP_TRY(hipMemcpy(out.data(), src + first, (size_t)count * sizeof(T), hipMemcpyDeviceToHost));
    (void)h;
    return GP_OK;
}

int create(const gp_config* cfg, int32_t rank, int32_t world, bool sharded, gp_layout* out, gp_shard_layout* shard,
           void** handle) {
    if (!cfg || !handle) return fail(GP_EINVAL, "null argument");
    *handle = nullptr;
    if (cfg->algo != GP_GOSSIP && cfg->algo != GP_PUSHSUM) return fail(GP_EINVAL, "unknown algorithm %d", cfg->algo);
    if (cfg->term_limit < 1 || cfg->term_limit > 15 || cfg->term_init < 0 || cfg->term_init >= cfg->term_limit)
        return fail(GP_EINVAL, "term_init/term_limit out of range");
    if (cfg->gossip_threshold < 0) return fail(GP_EINVAL, "gossip_threshold < 0");
    int64_t nodes, actors, grid;
    int rc = sizes(cfg->n_arg, cfg->topology, &nodes, &actors, &grid);
    if (rc) return rc;
    std::vector<int64_t> bounds;
    if (sharded) {
        if (rank < 0 || rank >= world) return fail(GP_EINVAL, "rank %d outside 0..%d", rank, world - 1);
        if (cfg->topology == GP_FULL && cfg->algo == GP_PUSHSUM)
            return fail(GP_EINVAL, "push-sum on \"full\" runs on one GPU only (gp_create)");
        if (cfg->flags & GP_FLAG_GENERIC) return fail(GP_EINVAL, "GP_FLAG_GENERIC is single-GPU only");
        if ((rc = partition(cfg->n_arg, cfg->topology, world, bounds))) return rc;
    } else {
        bounds = {0, actors};
    }
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
    // (gossip on a tiny graph of any topology takes the generic path too: k_gs_tiny runs it in LDS; up
    // to kTinyGridMaxActors, where one workgroup's walk of the actors still beats launches of the grid
    // kernels: 4000 3D -22%, 8000 3D +55%, profiles/round5/tiny/)
    // ... and push-sum on a tiny Imp3D graph (k_ps_tiny; the other grids keep their faster kernels)
    const bool one_round = (cfg->flags & GP_FLAG_ONE_ROUND) != 0;
    h->generic = h->full || (cfg->flags & GP_FLAG_GENERIC) ||
                 (h->gossip && !sharded && (size_t)actors <= kTinyGridMaxActors && !one_round) ||
                 (!h->gossip && cfg->topology == GP_IMP3D && !sharded && actors <= kTinyPsActors && !one_round);
    h->sharded = sharded;
    h->rank = sharded ? rank : 0;
    h->world = sharded ? world : 1;
    h->abnd = bounds;
    h->lo = (uint32_t)bounds[h->rank];
    h->hi = (uint32_t)bounds[h->rank + 1];
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
    if (h->world > 1 && !h->full) h->halo = g.gz > 1 ? g.plane : 1u;  // grid rows crossing a shard face
    // A round in pieces: push-sum pull shards whose host exchanges piece by piece
    // (GP_FLAG_PIECES), from 2^25 actors on every rank (GP_FLAG_FORCE_PIECES: any size), in whole
    // z-planes (line / 2D: 256 actors), so that the faces stay in the first and the last piece.
    // The same decision on every rank: it depends on the partition only.
    if (sharded && h->world > 1 && !h->gossip && !h->generic && (cfg->flags & GP_FLAG_PIECES)) {
        const int64_t unit = g.gz > 1 ? (int64_t)g.plane : 256;
        int64_t least = INT64_MAX, units = INT64_MAX;
        for (int q = 0; q < h->world; ++q) {
            least = std::min(least, bounds[q + 1] - bounds[q]);
            units = std::min(units, (bounds[q + 1] - bounds[q]) / unit);
        }
        const bool big = least >= kPieceMinActors || (cfg->flags & GP_FLAG_FORCE_PIECES);
        h->kpiece = h->npiece = big && units >= kMaxPieces ? kMaxPieces : 1;
    }
    h->pbnd.assign((size_t)h->world * (h->kpiece + 1), 0);
    for (int q = 0; q < h->world; ++q) {
        const int64_t unit = g.gz > 1 ? (int64_t)g.plane : 256, n = (bounds[q + 1] - bounds[q]) / unit;
        for (int i = 0; i <= h->kpiece; ++i)
            h->pbnd[(size_t)q * (h->kpiece + 1) + i] = i == h->kpiece ? bounds[q + 1] : bounds[q] + n * i / h->kpiece * unit;
    }
    // leader = Random().Next(0, nodes)  (program.fs:173/211/250/316)
    h->lay.leader = scale_draw(philox(0u, 0u, kStreamLeader, cfg->seed).x, (uint32_t)nodes);
    // actors with at least one neighbour: every actor of line / 2D / full (nodes + 1 >= 2),
    // every wired node of Imp3D (its extra link, program.fs:309), every node of a 3D grid of
    // more than one node (the only grid without edges is the single node, N < 8)
    if (cfg->topology == GP_IMP3D) h->lay.participants = nodes;
    else if (cfg->topology == GP_THREE_D) h->lay.participants = nodes > 1 ? nodes : 0;
    else h->lay.participants = actors;
    h->grid = grid_for(h->own());
    h->span = span_for(h->own(), h->grid);

    auto bail = [&](int code) {
        delete h;
        return code;
    };
    if (cfg->stream || (cfg->flags & GP_FLAG_USE_STREAM)) {
        h->stream = (hipStream_t)cfg->stream;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
        if (e != hipSuccess) return bail(fail(GP_EHIP, "hipStreamCreate: %s", hipGetErrorString(e)));
        h->own_stream = true;
    }
    if (hipEventCreate(&h->ev_a) != hipSuccess || hipEventCreate(&h->ev_b) != hipSuccess)
        return bail(fail(GP_EHIP, "hipEventCreate failed"));

    // own actors [lo, hi); round-to-round messages also for the halo rows of both neighbours
    const size_t n = h->own(), A = (size_t)actors;
    const int64_t lo = h->lo, xlo = h->ext_lo();
    const size_t xn = (size_t)(h->ext_hi() - xlo);
    if (h->gossip) {
        if ((rc = h->alloc(&h->cnt, n, lo)) || (rc = h->alloc(&h->gstate, n, lo))) return bail(rc);
        if (h->generic) {
            if ((rc = h->alloc(&h->inc[0], n, lo)) || (rc = h->alloc(&h->inc[1], n, lo))) return bail(rc);
            // a tiny graph runs its batches in one workgroup's LDS (k_gs_tiny; GP_FLAG_ONE_ROUND: not)
            // (up to 8192 actors, the LDS capacity: 1000 -67%, 5000 -36%, 8191 -12%, profiles/round5/tiny/)
            static_assert(kTinyMaxActors <= kTinyActors, "k_gs_tiny's LDS");
            h->tiny = !h->sharded && A <= kTinyMaxActors && !(cfg->flags & GP_FLAG_ONE_ROUND);
            // done bitmap and summary (global bit / word numbering): one GPU, the whole graph; a shard
            // holds a replica of every rank's bitmap (its own words current, the others' as of the
            // last exchange), so its senders filter remote targets too
            if (full_quad(h) || h->sharded) {
                if ((rc = h->alloc(&h->dbits, dbits_words_all(h)))) return bail(rc);
                if (A >= kDsumMinActors && (rc = h->alloc(&h->dsum, dsum_words_all(h)))) return bail(rc);
            }
            // full gossip on shards: the per-round plans' inputs and the lazy done-word shipping
            if (h->sharded && h->world > 1 && h->full &&
                ((rc = h->alloc(&h->cparts, (size_t)kPartRing * kParts * kPartStride)) ||
                 (rc = h->alloc(&h->self_chains, 1)) || (rc = h->alloc(&h->pstat, kPstatWords)) ||
                 (rc = h->alloc(&h->dstat, kDstatWords)) ||
                 (rc = h->alloc(&h->dship, dship_words(h), (int64_t)(h->lo >> 5)))))
                return bail(rc);
            const uint32_t nb = (uint32_t)((n + (1u << kTallyShift) - 1) >> kTallyShift);
            // the tally is a speed path: where its 128 KB of dynamic LDS cannot be allowed (another
            // ARCH), the handle keeps the receipt atomics, which give the same results
            if (full_quad(h) && nb <= kMaxTallyBuckets &&
                (n >= kTallyMinActors || (cfg->flags & GP_FLAG_GOSSIP_TALLY)) && prepare_gs_tally() == 0) {
                GsTally& t = h->tally;
                t.nb = nb;
                t.W = (uint32_t)h->grid;
                // (from kDsumMinActors a quarter of it: the ramp's last atomic round, 27M receipts at C4,
                // tallies too; C4 46.06 -> 45.50 ms, 10M unchanged with 8 (+3% with 32),
                // profiles/round5/cli/c4_tally_thr_*.txt)
                const size_t div = kTallyThrDiv * (n >= kDsumMinActors ? 4u : 1u);
                t.thr = (cfg->flags & GP_FLAG_GOSSIP_TALLY) ? 0u : (uint32_t)std::min<size_t>(n / div, 0xFFFFFFFFu);
                const size_t nc = (size_t)nb * t.W;
                if ((rc = h->alloc(&t.cnt, nc)) || (rc = h->alloc(&t.off, nc + 1)) || (rc = h->alloc(&t.tgt, 2 * n)) ||
                    (rc = h->alloc(&t.scratch, scan_scratch_words((uint32_t)nc))) ||
                    (rc = h->alloc(&t.chains, (size_t)kPartRing * kParts * kPartStride)) || (rc = h->alloc(&t.on, 4)) ||
                    (rc = h->alloc(&t.inc16, (n + 7) & ~(size_t)7)))
                    return bail(rc);
                // the live fallbacks, forced by a test hook: every count through the 32-bit words, and
                // the counted-batch placement everywhere
                const bool fb = (cfg->flags & GP_FLAG_TALLY_FALLBACKS) != 0;
                t.esc = fb ? 1u : 0xFFFFu;
                t.onepass = fb ? 0u : 1u;
            }
            // the ramp on lists: capacity a quarter of the tally threshold (no round it runs could be
            // due a tally: its chains stay below thr / 2), or 1/256 of the actors without the tally
            // (shards: a bound on every rank's holders, 1/256 of all the actors and at least 64, so that
            // every shard run starts on lists; the lists hold this rank's share)
            if (GP_SPARSE_RAMP && (full_quad(h) || (GP_SHARD_RAMP && gossip_plans(h))) && !h->tiny && !(cfg->flags & GP_FLAG_ONE_ROUND)) {
                GsSparse& sp = h->gsp;
                // (a list round costs ~6 us + 0.2 us per 1000 items: below the full walk's ~85 us at 100M
                // while the holders stay under ~n / 256, profiles/round6/ramp/)
                const size_t cap = h->sharded ? std::max<size_t>(A / 256u, 64u)
                                              : std::min<size_t>(h->tally.cnt ? h->tally.thr / 4u : n, n / 256u);
                if (cap >= 64 && cap < (1u << 28)) {
                    sp.cap = (uint32_t)cap;
                    const size_t size = 2 * cap + kSpSlack;
                    if ((rc = h->alloc(&sp.hl, size)) || (rc = h->alloc(&sp.tl[0], size)) ||
                        (rc = h->alloc(&sp.tl[1], size)) || (rc = h->alloc(&sp.ctr, (size_t)3 * 4 * kSpStride + kSpStride)) ||
                        (rc = h->alloc(&sp.err, 1)))
                        return bail(rc);
                    sp.fin = sp.ctr + 3 * 4 * kSpStride;  // (its own line, after the counters)
                    if (hipHostMalloc((void**)&h->h_spctr, (3 * 4 * kSpStride + 1) * sizeof(uint32_t)) != hipSuccess)
                        return bail(fail(GP_ENOMEM, "hipHostMalloc failed"));
                }
            }
            // full gossip shards: the receipt wave in bins (the passes' counters and their scan)
            if (GP_SHARD_BINS && gossip_plans(h) && prepare_gs_bins() == 0) {
                GsBins& b = h->bins;
                uint32_t nbt = 0;
                for (int q = 0; q < h->world; ++q) {
                    b.bin0[q] = nbt;
                    nbt += bins_of(h, q);
                }
                b.bin0[h->world] = nbt;
                b.nbt = nbt;
                b.nb_self = bins_of(h, h->rank);
                b.W = (uint32_t)std::min(grid_for((uint32_t)n), GP_BIN_GRID);
                const size_t nc = (size_t)nbt * b.W;
                b.self_words = b.nb_self + 1u + (uint32_t)((n + 1) / 2) + 1u;  // one u16 receipt per own actor
                if (nbt && nbt <= kMaxBins && nc < (1u << 31)) {
                    if ((rc = h->alloc(&b.cnt, nc)) || (rc = h->alloc(&b.off, nc + 1)) ||
                        (rc = h->alloc(&b.scratch, scan_scratch_words((uint32_t)nc))) || (rc = h->alloc(&b.self, b.self_words)))
                        return bail(rc);
                }
            }
        } else if ((rc = h->alloc(&h->dir[0], xn, xlo)) || (rc = h->alloc(&h->dir[1], xn, xlo))) {
            return bail(rc);
        }
    } else {
        // message rows for the own actors and both halos; a remote extra-link sender's message
        // lands in the receiver's CSR slot (rmsg), not in a row of the sender
        if ((rc = h->alloc(&h->msg[0], xn, xlo)) || (rc = h->alloc(&h->msg[1], xn, xlo)) ||
            (rc = h->alloc(&h->flags, n, lo)) || (rc = h->alloc(&h->frozen, n, lo)) ||
            (rc = h->alloc(&h->partials, (size_t)h->grid)))
            return bail(rc);
        // quiet-wave marks (a shard: over its own actors; remote messages are marked by the unpack)
        if (GP_ACT_PCT > 0 && !h->generic && (h->own() >= kQuietMinActors || (cfg->flags & GP_FLAG_QUIET_WAVES))) {
            for (int i = 0; i < 2; ++i)
                if ((rc = h->alloc(&h->act[i], act_bytes(h), (int64_t)act_first(h)))) return bail(rc);
            if ((rc = h->alloc(&h->work, (size_t)kParts * kWorkStride))) return bail(rc);
            if (hipMemsetAsync(h->work, 0, (size_t)kParts * kWorkStride * sizeof *h->work, h->stream) != hipSuccess)
                return bail(fail(GP_EHIP, "hipMemsetAsync failed"));
            h->act_thr = (uint32_t)((uint64_t)h->lay.nodes * GP_ACT_PCT / 100u);
        }
        if (h->generic) {  // single-GPU only: whole graph
            for (int i = 0; i < 2; ++i)
                if ((rc = h->alloc(&h->bcnt[i], A)) || (rc = h->alloc(&h->boff[i], A + 1)) ||
                    (rc = h->alloc(&h->slot[i], A)))
                    return bail(rc);
            // a tiny graph runs its batches in one workgroup's LDS (k_ps_tiny; GP_FLAG_ONE_ROUND: not)
            h->tiny = !h->sharded && A <= kTinyPsActors && !(cfg->flags & GP_FLAG_ONE_ROUND);
            if ((rc = h->alloc(&h->tgt, A)) || (rc = h->alloc(&h->pos, A)) ||
                (rc = h->alloc(&h->scan_scratch, scan_scratch_words((uint32_t)A))))
                return bail(rc);
        } else if ((rc = h->alloc(&h->dir[0], xn, xlo)) || (rc = h->alloc(&h->dir[1], xn, xlo))) {
            return bail(rc);
        }
        h->tiles = !h->sharded && !h->generic && !g.has_link && g.gy == 1 && g.gz == 1 && !h->act[0] &&
                   A < kTileMaxActors && !(cfg->flags & GP_FLAG_ONE_ROUND);
        if (h->tiles) {
            TileArgs& t = h->tl;
            for (int i = 2; i < (int)kTileBufs; ++i)
                if ((rc = h->alloc(&h->msg[i], xn, xlo)) || (rc = h->alloc(&h->dir[i], xn, xlo))) return bail(rc);
            for (int i = 0; i < (int)kTileBufs; ++i) {
                if ((rc = h->alloc(&h->flg[i], n, lo))) return bail(rc);
                t.msg[i] = h->msg[i];
                t.dir[i] = h->dir[i];
                t.flg[i] = h->flg[i];
            }
        }
    }
    if (g.has_link && (rc = build_links(h))) return bail(rc);
    if (h->sharded && (rc = build_plan(h))) return bail(rc);
    // the restore point of the activity tiers, allocated here so that device_bytes counts it and a
    // shard that fits at creation cannot fail for memory in the middle of a run
    if (tiers_on(h) && (rc = ensure_ckpt(h))) return bail(rc);
    if ((rc = h->alloc(&h->parts, (size_t)kPartRing * kParts * kPartStride))) return bail(rc);
    // Set up here what gp_step would otherwise allocate inside the timed round loop of a first run
    // (pinned host memory and device reallocations cost 0.1-1 ms each: `1000 full gossip` ran in
    // 1.9 ms the first time and 0.28 ms after, tools/first_run_cost.py): the per-round count
    // array for 2^17 rounds (1 MB; `100000 3D push-sum` takes 62125) and the host-mapped batch
    // trace for the largest batch.
    if ((rc = ensure_trace(h, 1 << 17))) return bail(rc);
    if (hipHostMalloc((void**)&h->h_trace, (size_t)kMaxBatch * sizeof(unsigned long long),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&h->d_trace, h->h_trace, 0) != hipSuccess)
        return bail(fail(GP_ENOMEM, "hipHostMalloc of the batch trace failed"));
    h->h_trace_cap = kMaxBatch;
    if ((rc = reset(h))) return bail(rc);
    // the code object is loaded at the first kernel launch; a reset without kernels of this library
    // (full gossip) would leave that to the first timed round (C1 ran in 1.48 instead of 0.29 ms)
    if (launch_load(h->stream)) return bail(fail(GP_EHIP, "loading the kernels failed"));
    h->lay.device_bytes = (int64_t)h->dev_bytes;
    if (out) *out = h->lay;
    if (shard) {
        shard->lo = h->lo;
        shard->hi = h->hi;
        shard->halo = h->halo;
        shard->send_total = h->send_total;
        shard->recv_total = h->recv_total;
    }
    *handle = h;
    return GP_OK;
}

// ------------------------------------------------------------------ single-process multi-GPU
// gp_create with cfg->num_gpus = N > 1 ("the library owns ... RCCL comms; multi-GPU
// runs inside one process, one stream per device, ncclCommInitAll plus group calls").  The graph
// is split into N node-range shards (gp_partition), shard p on device device + p with its own
// stream; a round is every shard's gp_shard_round, ONE exchange of the fixed-size chunks, every
// shard's gp_shard_deliver — the same decomposition the torch.distributed host drives over one
// process per GPU (gossip_amd/sharded.py), here with the library's own transport:
//   * RCCL: one communicator per device from ncclCommInitAll; the exchange is one
//     ncclGroupStart / ncclGroupEnd around every (p, q) ncclSend / ncclRecv pair, each on the
//     sending / receiving shard's stream, so kernels and transfers stay stream-ordered;
//   * GP_FLAG_ONE_DEVICE (tests on one GPU): every shard on cfg->device, one shared stream,
//     the chunks moved by device copies.
// RCCL is opened on first use (a multi-device group), not linked: the one-GPU engine and the CLI
// load on an install without RCCL.  In a torch process dlopen by soname returns the RCCL torch
// has already loaded, so the process keeps one copy.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string why;  // the loader's error text when a symbol or the library is missing
};

// Loaded once per process by a function-local static (thread-safe initialisation); the dlerror()
// text is saved at load time, since a later dlerror() returns NULL or another call's message.
const Rccl& rccl_state() {
    static const Rccl r = [] {
        Rccl x;
        void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) so = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!so) {
            const char* e = dlerror();
            x.why = e ? e : "dlopen failed";
            return x;
        }
        auto sym = [&](const char* name) {
            void* p = dlsym(so, name);
            if (!p && x.why.empty()) x.why = std::string("missing symbol ") + name;
            return p;
        };
        x.comm_init_all = reinterpret_cast<decltype(x.comm_init_all)>(sym("ncclCommInitAll"));
        x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(sym("ncclCommDestroy"));
        x.group_start = reinterpret_cast<decltype(x.group_start)>(sym("ncclGroupStart"));
        x.group_end = reinterpret_cast<decltype(x.group_end)>(sym("ncclGroupEnd"));
        x.send = reinterpret_cast<decltype(x.send)>(sym("ncclSend"));
        x.recv = reinterpret_cast<decltype(x.recv)>(sym("ncclRecv"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(sym("ncclGetErrorString"));
        return x;
    }();
    return r;
}

const Rccl* rccl() {
    const Rccl& r = rccl_state();
    const bool ok = r.comm_init_all && r.comm_destroy && r.group_start && r.group_end && r.send && r.recv &&
                    r.error_string;
    return ok ? &r : nullptr;
}

struct Group {
    int W = 0;
    bool one_device = false;
    std::vector<Handle*> shard;
    std::vector<int> dev;
    std::vector<void*> send, recv;
    // two receive buffers per shard (round parity par): a push-sum round reads the previous round's
    // remote messages where they arrived
    std::vector<int64_t> rstride;
    int par = 0;
    char* rbuf(int p) const { return static_cast<char*>(recv[(size_t)p]) + par * rstride[(size_t)p]; }
    std::vector<ncclComm_t> comm;
    hipStream_t shared = nullptr;
    // rounds in pieces: the exchange of each piece runs on a stream of its own per
    // shard (xstream; one stream for the one-device copies), ordered after the piece's kernels by an
    // event, and the shards' unpacks wait for the last one
    std::vector<hipStream_t> xstream;
    std::vector<hipEvent_t> ev_done, ev_x;
    int64_t batch = 8;
    int64_t rounds = 0, completed = 0;
    bool converged = false;

    ~Group() {
        for (size_t p = 0; p < shard.size(); ++p) {
            if (!one_device) (void)hipSetDevice(dev[p]);
            if (shard[p]) (void)hipStreamSynchronize(shard[p]->stream);
            if (p < xstream.size() && xstream[p]) (void)hipStreamSynchronize(xstream[p]);
        }
        for (size_t p = 0; p < xstream.size(); ++p) {
            if (!one_device) (void)hipSetDevice(dev[p]);
            if (xstream[p]) (void)hipStreamDestroy(xstream[p]);
            if (p < ev_done.size() && ev_done[p]) (void)hipEventDestroy(ev_done[p]);
            if (p < ev_x.size() && ev_x[p]) (void)hipEventDestroy(ev_x[p]);
        }
        for (ncclComm_t c : comm)
            if (c) (void)rccl()->comm_destroy(c);  // a communicator exists only if RCCL loaded
        for (size_t p = 0; p < shard.size(); ++p) {
            if (!one_device) (void)hipSetDevice(dev[p]);
            if (p < send.size() && send[p]) (void)hipFree(send[p]);
            if (p < recv.size() && recv[p]) (void)hipFree(recv[p]);
            delete shard[p];
        }
        if (shared) (void)hipStreamDestroy(shared);
    }
};

#define RCCL_TRY(x)                                                                                      \
    do {                                                                                                 \
        ncclResult_t r_ = (x);                                                                           \
        if (r_ != ncclSuccess) return fail(GP_ERCCL, "%s failed: %s", #x, rccl()->error_string(r_));    \
    } while (0)

// Send / receive pairs of every (p, q) between ncclGroupStart and ncclGroupEnd.  An error inside
// the group still closes it (the group is left open otherwise, and the next RCCL call fails).
// The chunks of piece i (the whole round when it is not in pieces), on stream s(p) of each shard.
int group_exchange_rccl(Group& G, const Rccl& R, int i, bool split) {
    const int W = G.W;
    for (int p = 0; p < W; ++p) {
        const Handle* s = G.shard[p];
        hipStream_t st = split ? G.xstream[p] : s->stream;
        for (int q = 0; q < W; ++q) {
            if (q == p) continue;
            const size_t c = (size_t)i * W + q, ns = s->out_chunk[c].size, nr = s->in_chunk[c].size;
            if (ns) RCCL_TRY(R.send(static_cast<char*>(G.send[p]) + s->out_off[c], ns, ncclUint8, q, G.comm[p], st));
            if (nr) RCCL_TRY(R.recv(G.rbuf(p) + s->in_off[c], nr, ncclUint8, q, G.comm[p], st));
        }
    }
    return GP_OK;
}

// Piece i's exchange.  In pieces it runs on the exchange streams, after the piece's kernels (an event
// on each shard's stream), so the shards go on with piece i+1 meanwhile.
int group_exchange(Group& G, int i = 0) {
    const int W = G.W;
    const bool split = G.shard[0]->npiece > 1;
    if (split) {
        for (int p = 0; p < (G.one_device ? 1 : W); ++p) {
            if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
            HIP_TRY(hipEventRecord(G.ev_done[p], G.shard[p]->stream));
            HIP_TRY(hipStreamWaitEvent(G.xstream[p], G.ev_done[p], 0));
        }
    }
    if (G.one_device) {
        hipStream_t st = split ? G.xstream[0] : G.shared;
        for (int p = 0; p < W; ++p)
            for (int q = 0; q < W; ++q) {
                const size_t c = (size_t)i * W + q;
                const int64_t n = (int64_t)G.shard[p]->out_chunk[c].size;
                if (q == p || !n) continue;
                HIP_TRY(hipMemcpyAsync(G.rbuf(q) + G.shard[q]->in_off[(size_t)i * W + p],
                                       static_cast<char*>(G.send[p]) + G.shard[p]->out_off[c], (size_t)n,
                                       hipMemcpyDeviceToDevice, st));
            }
        return GP_OK;
    }
    const Rccl& R = *rccl();  // loaded: the group has communicators
    RCCL_TRY(R.group_start());
    const int rc = group_exchange_rccl(G, R, i, split);
    const ncclResult_t end = R.group_end();
    if (rc) return rc;
    if (end != ncclSuccess) return fail(GP_ERCCL, "ncclGroupEnd failed: %s", R.error_string(end));
    return GP_OK;
}

// In pieces: the shards' unpacks wait for the last piece's exchange.
int group_exchange_join(Group& G) {
    if (G.shard[0]->npiece <= 1) return GP_OK;
    for (int p = 0; p < (G.one_device ? 1 : G.W); ++p) {
        if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
        HIP_TRY(hipEventRecord(G.ev_x[p], G.xstream[p]));
        HIP_TRY(hipStreamWaitEvent(G.one_device ? G.shared : G.shard[p]->stream, G.ev_x[p], 0));
    }
    return GP_OK;
}

int group_sync(Group& G, std::vector<gp_status>& sts) {
    sts.assign((size_t)G.W, gp_status{});
    int rc;
    for (int p = 0; p < G.W; ++p) {
        if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
        if ((rc = shard_sync(G.shard[p], &sts[(size_t)p]))) return rc;
    }
    for (int p = 1; p < G.W; ++p)
        if (sts[p].round != sts[0].round || sts[p].completed != sts[0].completed || sts[p].converged != sts[0].converged)
            return fail(GP_ESTATE, "shards disagree after round %lld (rank %d)", (long long)sts[0].round, p);
    G.rounds = sts[0].round;
    G.completed = sts[0].completed;
    G.converged = sts[0].converged != 0;
    return GP_OK;
}

int group_step(Handle* h, int64_t max_rounds, gp_status* st) {
    if (max_rounds < 0) return fail(GP_EINVAL, "max_rounds < 0");
    Group& G = *h->grp;
    if (G.one_device) HIP_TRY(hipSetDevice(G.dev[0]));
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t goal = G.rounds + max_rounds;
    std::vector<gp_status> sts;
    int rc;
    // gossip's F(k) reports round k-1: a batch may run past the convergence round; those
    // rounds are no-ops on the device (gated) and the counts stay final
    if (gossip_plans(G.shard[0])) G.batch = std::min<int64_t>(G.batch, 4);
    while (!G.converged && G.rounds < goal) {
        const int64_t B = std::min<int64_t>(G.batch, goal - G.rounds);
        for (int64_t i = 0; i < B; ++i) {
            // piece by piece: every shard's piece j, then its exchange, which overlaps piece j+1
            for (int j = 0; j < G.shard[0]->npiece; ++j) {
                for (int p = 0; p < G.W; ++p) {
                    if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
                    if ((rc = shard_round_piece(G.shard[p], G.send[p], j))) return rc;
                }
                if ((rc = group_exchange(G, j))) return rc;
            }
            if ((rc = group_exchange_join(G))) return rc;
            for (int p = 0; p < G.W; ++p) {
                if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
                if ((rc = shard_deliver(G.shard[p], G.rbuf(p)))) return rc;
            }
            G.par ^= 1;
        }
        const int64_t before = G.completed;
        if ((rc = group_sync(G, sts))) return rc;
        // batches start again from 8 rounds when the run enters the half-reported phase, where the
        // activity tiers begin (a plan is chosen at every sync; sharded.py _next_batch does the same)
        // (full gossip sizes every round from the last round before a sync: 4 rounds at most, §6.10)
        const int64_t nodes = G.shard[0]->lay.nodes;
        const int64_t most = gossip_plans(G.shard[0]) ? 4 : 64;
        G.batch = (2 * before < nodes && nodes <= 2 * G.completed) ? std::min<int64_t>(8, most)
                                                                  : std::min<int64_t>(G.batch * 2, most);
    }
    if (sts.empty() && (rc = group_sync(G, sts))) return rc;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->round = G.rounds;
        st->completed = G.completed;
        st->converged = G.converged ? 1 : 0;
        st->device_ms = ms;
        for (const gp_status& s : sts) {  // rank order
            st->sum_s += s.sum_s;
            st->sum_w += s.sum_w;
        }
    }
    return GP_OK;
}

int group_reset(Handle* h) {
    Group& G = *h->grp;
    int rc;
    for (int p = 0; p < G.W; ++p) {
        if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
        if ((rc = reset(G.shard[p]))) return rc;
    }
    G.batch = 8;
    G.rounds = G.completed = 0;
    G.converged = false;
    return GP_OK;
}

int group_create(const gp_config* cfg, gp_layout* out, void** handle) {
    const int W = std::max(1, cfg->num_gpus);
    if (W > kMaxWorld) return fail(GP_EINVAL, "num_gpus %d above %d", W, kMaxWorld);
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    auto* grp = new Group();
    auto* h = new Handle();
    h->grp = grp;
    auto bail = [&](int code) {
        delete grp;
        h->grp = nullptr;
        delete h;
        return code;
    };
    Group& G = *grp;
    G.W = W;
    G.one_device = (cfg->flags & GP_FLAG_ONE_DEVICE) != 0;
    for (int p = 0; p < W; ++p) {
        const int d = G.one_device ? cfg->device : cfg->device + p;
        if (d < 0 || d >= ndev)
            return bail(fail(GP_EINVAL, "num_gpus %d from device %d: device %d not present (%d devices)", W,
                             cfg->device, d, ndev));
        G.dev.push_back(d);
    }
    // every failure below goes through bail(): the shards, streams and buffers built so far are freed
    auto set_dev = [&](int d) {
        const hipError_t e = hipSetDevice(d);
        return e == hipSuccess ? GP_OK : fail(GP_EHIP, "hipSetDevice(%d): %s", d, hipGetErrorString(e));
    };
    int rc;
    if (G.one_device) {
        if ((rc = set_dev(cfg->device))) return bail(rc);
        hipError_t e = hipStreamCreateWithFlags(&G.shared, hipStreamNonBlocking);
        if (e != hipSuccess) return bail(fail(GP_EHIP, "hipStreamCreate: %s", hipGetErrorString(e)));
    } else if (!rccl()) {
        return bail(fail(GP_ERCCL, "num_gpus %d needs RCCL: librccl.so.1 could not be loaded (%s)", W,
                         rccl_state().why.c_str()));
    }
    G.shard.assign((size_t)W, nullptr);
    G.send.assign((size_t)W, nullptr);
    G.recv.assign((size_t)W, nullptr);
    G.rstride.assign((size_t)W, 0);
    int64_t bytes = 0;
    for (int p = 0; p < W; ++p) {
        gp_config c = *cfg;
        c.device = G.dev[p];
        c.num_gpus = 0;
        c.flags &= ~(GP_FLAG_ONE_DEVICE | GP_FLAG_GROUP | GP_FLAG_USE_STREAM);
        // the group exchanges piece by piece (its own transport): always on one device (device copies on
        // a side stream, in the GPU suite); across devices only when the caller asks (GP_FLAG_PIECES): its
        // RCCL path on per-shard side streams has not run on two devices yet
        if (G.one_device) c.flags |= GP_FLAG_PIECES;
        c.stream = nullptr;
        if (G.one_device) {
            c.flags |= GP_FLAG_USE_STREAM;
            c.stream = G.shared;
        }
        void* sh = nullptr;
        gp_layout lay{};
        if ((rc = create(&c, p, W, true, &lay, nullptr, &sh))) return bail(rc);
        Handle* s = H(sh);
        G.shard[p] = s;
        if ((rc = set_dev(G.dev[p]))) return bail(rc);
        if (s->send_total && hipMalloc(&G.send[p], (size_t)s->send_total) != hipSuccess)
            return bail(fail(GP_ENOMEM, "exchange send buffer of %lld bytes", (long long)s->send_total));
        G.rstride[(size_t)p] = (s->recv_total + (int64_t)kAlign - 1) / (int64_t)kAlign * (int64_t)kAlign;
        if (s->recv_total && hipMalloc(&G.recv[p], (size_t)(2 * G.rstride[(size_t)p])) != hipSuccess)
            return bail(fail(GP_ENOMEM, "exchange receive buffers of 2 x %lld bytes", (long long)s->recv_total));
        bytes += lay.device_bytes + s->send_total + 2 * G.rstride[(size_t)p];
        if (p == 0) h->lay = lay;
    }
    if (G.shard[0]->kpiece > 1) {  // the exchange streams and events of the pieces
        G.xstream.assign((size_t)W, nullptr);
        G.ev_done.assign((size_t)W, nullptr);
        G.ev_x.assign((size_t)W, nullptr);
        for (int p = 0; p < (G.one_device ? 1 : W); ++p) {
            if ((rc = set_dev(G.dev[p]))) return bail(rc);
            if (hipStreamCreateWithFlags(&G.xstream[p], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&G.ev_done[p], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&G.ev_x[p], hipEventDisableTiming) != hipSuccess)
                return bail(fail(GP_EHIP, "exchange stream / events of device %d", G.dev[p]));
        }
    }
    if (!G.one_device) {
        G.comm.assign((size_t)W, nullptr);
        ncclResult_t r = rccl()->comm_init_all(G.comm.data(), W, G.dev.data());
        if (r != ncclSuccess) {
            G.comm.clear();
            return bail(fail(GP_ERCCL, "ncclCommInitAll(%d devices): %s", W, rccl()->error_string(r)));
        }
    }
    h->cfg = *cfg;
    h->lay.device_bytes = bytes;
    h->gossip = G.shard[0]->gossip;
    h->lo = 0;
    h->hi = (uint32_t)h->lay.actors;
    if (out) *out = h->lay;
    *handle = h;
    return GP_OK;
}

// Shard p's part [a, b) of the actor range [first, first + count), or false.
bool shard_part(const Group& G, int p, int64_t first, int64_t count, int64_t& a, int64_t& b) {
    a = std::max<int64_t>(first, G.shard[p]->lo);
    b = std::min<int64_t>(first + count, G.shard[p]->hi);
    return a < b;
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
    if (cfg->num_gpus > 1 || (cfg->flags & GP_FLAG_GROUP)) {
        *handle = nullptr;
        return group_create(cfg, out, handle);
    }
    return create(cfg, 0, 1, false, out, nullptr, handle);
}

int gp_create_shard(const gp_config* cfg, int32_t rank, int32_t world, gp_layout* out, gp_shard_layout* shard,
                    void** handle) {
    if (cfg && cfg->num_gpus > 1) return fail(GP_EINVAL, "a shard is one GPU (num_gpus %d)", cfg->num_gpus);
    return create(cfg, rank, world, true, out, shard, handle);
}

int gp_partition(int64_t n_arg, int32_t topology, int32_t world, int64_t* bounds) {
    if (!bounds) return fail(GP_EINVAL, "null bounds");
    std::vector<int64_t> b;
    const int rc = partition(n_arg, topology, world, b);
    if (rc) return rc;
    std::copy(b.begin(), b.end(), bounds);
    return GP_OK;
}

int gp_shard_pieces(void* handle) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (!h->sharded) return fail(GP_ESTATE, "not a shard handle");
    return h->npiece;
}

int gp_shard_plan_piece(void* handle, int32_t piece, int64_t* send_bytes, int64_t* recv_bytes, int64_t* offsets) {
    if (!handle || !send_bytes || !recv_bytes || !offsets) return fail(GP_EINVAL, "null argument");
    Handle* h = H(handle);
    if (!h->sharded) return fail(GP_ESTATE, "not a shard handle");
    if (piece < 0 || piece >= h->npiece) return fail(GP_EINVAL, "piece %d outside 0..%d", piece, h->npiece - 1);
    for (int q = 0; q < h->world; ++q) {
        send_bytes[q] = (int64_t)h->out_chunk[(size_t)piece * h->world + q].size;
        recv_bytes[q] = (int64_t)h->in_chunk[(size_t)piece * h->world + q].size;
    }
    offsets[0] = h->out_poff[piece];
    offsets[1] = h->in_poff[piece];
    return GP_OK;
}

int gp_shard_round_piece(void* handle, void* send_buf, int32_t piece) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (!H(handle)->sharded) return fail(GP_ESTATE, "not a shard handle");
    return shard_round_piece(H(handle), send_buf, piece);
}

int gp_shard_plan(void* handle, int64_t* send_bytes, int64_t* recv_bytes) {
    if (!handle || !send_bytes || !recv_bytes) return fail(GP_EINVAL, "null argument");
    Handle* h = H(handle);
    if (!h->sharded) return fail(GP_ESTATE, "not a shard handle");
    if (h->npiece > 1) return fail(GP_ESTATE, "the round runs in %d pieces: gp_shard_plan_piece", h->npiece);
    for (int q = 0; q < h->world; ++q) {
        send_bytes[q] = (int64_t)h->out_chunk[q].size;
        recv_bytes[q] = (int64_t)h->in_chunk[q].size;
    }
    return GP_OK;
}

int gp_shard_round(void* handle, void* send_buf) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (!H(handle)->sharded) return fail(GP_ESTATE, "not a shard handle");
    return shard_round(H(handle), send_buf);
}

int gp_shard_deliver(void* handle, const void* recv_buf) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (!H(handle)->sharded) return fail(GP_ESTATE, "not a shard handle");
    return shard_deliver(H(handle), recv_buf);
}

int gp_shard_sync(void* handle, gp_status* st) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (!H(handle)->sharded) return fail(GP_ESTATE, "not a shard handle");
    return shard_sync(H(handle), st);
}

int gp_reset(void* handle) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (H(handle)->grp) return group_reset(H(handle));
    return reset(H(handle));
}

int gp_step(void* handle, int64_t max_rounds, gp_status* st) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    if (H(handle)->grp) return group_step(H(handle), max_rounds, st);
    return step(H(handle), max_rounds, st);
}

int gp_read_gossip(void* handle, int64_t first, int64_t count, uint32_t* cnt, uint8_t* flags) {
    if (!handle) return fail(GP_EINVAL, "null handle");
    Handle* h = H(handle);
    if (h->grp) {  // the shards' parts in rank order
        if (!h->gossip) return fail(GP_ESTATE, "not a gossip handle");
        int rc = check_range(h, first, count);
        if (rc) return rc;
        const Group& G = *h->grp;
        for (int p = 0; p < G.W; ++p) {
            int64_t a, b;
            if (!shard_part(G, p, first, count, a, b)) continue;
            if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
            if ((rc = gp_read_gossip(G.shard[p], a, b - a, cnt ? cnt + (a - first) : nullptr,
                                     flags ? flags + (a - first) : nullptr)))
                return rc;
        }
        return GP_OK;
    }
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
    if (h->grp) {
        if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
        int rc = check_range(h, first, count);
        if (rc) return rc;
        const Group& G = *h->grp;
        for (int p = 0; p < G.W; ++p) {
            int64_t a, b;
            if (!shard_part(G, p, first, count, a, b)) continue;
            if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
            const int64_t o = a - first;
            if ((rc = gp_read_pushsum(G.shard[p], a, b - a, S ? S + o : nullptr, W ? W + o : nullptr,
                                      flags ? flags + o : nullptr)))
                return rc;
        }
        return GP_OK;
    }
    if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
    int rc = check_range(h, first, count);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    std::vector<uint8_t> f;
    std::vector<double2> fr, ms;
    const int64_t last = h->rounds - 1;
    if ((rc = copy_slice(h, f, (const uint8_t*)h->flags_at(last), first, count))) return rc;
    if ((rc = copy_slice(h, fr, (const double2*)h->frozen, first, count))) return rc;
    if (last >= 0 && (rc = copy_slice(h, ms, (const double2*)h->msg[h->bidx(last)], first, count))) return rc;
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
    if (h->grp) {
        if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
        int rc = check_range(h, first, count);
        if (rc) return rc;
        const Group& G = *h->grp;
        for (int p = 0; p < G.W; ++p) {
            int64_t a, b;
            if (!shard_part(G, p, first, count, a, b)) continue;
            if (!G.one_device) HIP_TRY(hipSetDevice(G.dev[p]));
            const int64_t o = a - first;
            if ((rc = gp_read_messages(G.shard[p], a, b - a, dst ? dst + o : nullptr, s ? s + o : nullptr,
                                       w ? w + o : nullptr)))
                return rc;
        }
        return GP_OK;
    }
    if (h->gossip) return fail(GP_ESTATE, "not a push-sum handle");
    int rc = check_range(h, first, count);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    const int64_t last = h->rounds - 1;
    std::vector<uint32_t> t((size_t)count, kNone);
    std::vector<double2> ms;
    if (last >= 0) {
        if ((rc = copy_slice(h, ms, (const double2*)h->msg[h->bidx(last)], first, count))) return rc;
        if (h->generic) {
            if ((rc = copy_slice(h, t, (const uint32_t*)h->tgt, first, count))) return rc;
        } else {
            std::vector<uint8_t> d;
            if ((rc = copy_slice(h, d, (const uint8_t*)h->dir[h->bidx(last)], first, count))) return rc;
            for (int64_t i = 0; i < count; ++i) {
                const uint32_t v = (uint32_t)(first + i);
                t[i] = d[i] == kDirNone ? kNone
                       : dir_target(h->g, v, d[i], d[i] == kDirLink ? link_of(h->cfg.seed, v, (uint32_t)h->lay.nodes) : 0u);
            }
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
    if (h->grp) {  // every shard holds the global count
        if (!h->grp->one_device) HIP_TRY(hipSetDevice(h->grp->dev[0]));
        h = h->grp->shard[0];
    }
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
    if (h->grp) {  // the topology is global on every shard
        if (!h->grp->one_device) HIP_TRY(hipSetDevice(h->grp->dev[0]));
        h = h->grp->shard[0];
    }
    if (v < 0 || v >= (int64_t)h->g.actors) return fail(GP_EINVAL, "actor %lld out of range", (long long)v);
    if (h->full) {  // program.fs:201-206: every j != i in ascending order
        const int64_t d = h->lay.nodes;
        for (int64_t k = 0; k < d && k < cap; ++k) out[k] = (uint32_t)(k + (k >= v));
        return (int)d;
    }
    const uint32_t m = presence(h->g, (uint32_t)v);
    const uint32_t lk = (m & 64u) ? link_of(h->cfg.seed, (uint32_t)v, (uint32_t)h->lay.nodes) : 0u;
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
    if (h->grp) h = h->grp->shard[0];  // rank 0's kernels
    std::memset(out, 0, sizeof *out);
    out->launches = h->k_launches;
    out->total_ms = h->k_total_ms;
    out->avg_ms = h->k_launches ? h->k_total_ms / (double)h->k_launches : 0.0;
    out->bytes_per_launch = bytes_per_round(h);
    std::snprintf(out->kernel, sizeof out->kernel, "%s", round_kernel_name(h));
    out->aux_avg_ms = h->k_launches ? h->k_aux_ms / (double)h->k_launches : 0.0;
    std::snprintf(out->aux_kernel, sizeof out->aux_kernel, "%s", aux_kernel_name(h));
    out->work_per_launch = (double)h->own();
    if (h->act[0] && h->work) {  // the quiet kernel counts the actors it walks
        std::vector<unsigned long long> w((size_t)kParts * kWorkStride);
        HIP_TRY(hipMemcpyAsync(w.data(), h->work, w.size() * sizeof w[0], hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        unsigned long long t = 0;
        for (int i = 0; i < kParts; ++i) t += w[(size_t)i * kWorkStride];
        out->work_per_launch = h->work_rounds ? (double)t / (double)h->work_rounds : 0.0;
    }
    if (reset_counters) {
        h->k_launches = 0;
        h->k_total_ms = 0.0;
        h->k_aux_ms = 0.0;
        h->work_rounds = 0;
        if (h->work)
            HIP_TRY(hipMemsetAsync(h->work, 0, (size_t)kParts * kWorkStride * sizeof *h->work, h->stream));
    }
    return GP_OK;
}

int gp_shard_stats(void* handle, gp_shard_counters* out) {
    if (!handle || !out) return fail(GP_EINVAL, "null argument");
    Handle* h = H(handle);
    if (h->grp) h = h->grp->shard[0];
    if (!h->sharded) return fail(GP_ESTATE, "not a shard handle");
    std::memset(out, 0, sizeof *out);
    out->plan_changes = h->plan_changes;
    out->restores = h->restores;
    out->send_bytes = h->out_poff[h->npiece];
    out->recv_bytes = h->in_poff[h->npiece];
    out->restore_round = h->ck.valid ? h->ck.rounds : -1;
    out->bytes_sent = h->bytes_sent;
    out->list_rounds = h->list_rounds;
    out->bin_rounds = h->bin_rounds;
    return GP_OK;
}

void gp_destroy(void* handle) {
    Handle* h = H(handle);
    if (h && h->grp) {
        delete h->grp;
        h->grp = nullptr;
    }
    delete h;
}

const char* gp_last_error(void) { return g_err.c_str(); }

}  // extern "C"
