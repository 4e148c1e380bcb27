// gp_kernels.hip — gfx950 kernels of the synchronous-round gossip / push-sum engine.
//
// Every round kernel F(r) is one HBM-streaming pass over the actors:
//   * collect: the messages sent to actor v in round r-1 are PULLED from v's in-neighbours —
//     implicit grid offsets (program.fs:295-306 is symmetric) plus the ascending CSR of Imp3D
//     extra-link sources — in ascending source order, so the fp64 inbox sum is the canonical
//     sequential one with no sort and no atomics;
//   * update: program.fs:97-105 (gossip) / :119-143 (push-sum) for one round;
//   * emit:   one Philox4x32-10 block per (actor, round) picks the neighbour index(es);
//             only a 1-byte direction code (+ the 16-byte (s,w) message) is stored;
//   * count:  newly reported actors are reduced per wave/block and added once per block to
//             total[r], the per-round ParentActor count (program.fs:44-63).
// Kernels are grid-stride over an XCD-aware node mapping: workgroups with equal blockIdx % 8
// (one XCD under round-robin dispatch) walk one contiguous 1/8 of the actors, so the +-1,
// +-G and +-G^2 neighbour rows they re-read stay in that XCD's L2 (placement is a speed hint
// only; correctness never depends on it).
#include "gp_kernels.h"

namespace gp {

namespace {

__device__ __forceinline__ void node_range(uint32_t lo, uint32_t hi, uint32_t span, uint32_t& v, uint32_t& end,
                                           uint32_t& step) {
    const uint32_t grp = blockIdx.x & 7u;
    const uint32_t j = blockIdx.x >> 3;
    const uint32_t per = gridDim.x >> 3;
    const uint32_t base = lo + grp * span;
    end = base + span < hi ? base + span : hi;
    if (base >= hi) end = 0;
    v = base + j * kBlock + threadIdx.x;
    step = per * kBlock;
}

__device__ __forceinline__ uint32_t* part_slot(uint32_t* parts, long long a, uint32_t j) {
    return parts + ((uint32_t)(a & (kPartRing - 1)) * kParts + j) * kPartStride;
}

// Sum of one u32 over the 64 lanes of a full wave, wave-uniform: four DPP butterflies within
// each row of 16 lanes (xor 1, xor 2, half-row mirror, row mirror), then the four row sums read
// as scalars.  No LDS round trips (a __shfl_xor ladder is six dependent ds_bpermute).
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);  // row_half_mirror
    x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, true);  // row_mirror
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) + (uint32_t)__builtin_amdgcn_readlane((int)x, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)x, 32) + (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}

// Block-wide sum of one u32 per thread; thread 0 adds it to this block's sub-counter of
// round `a` (64 sub-counters on separate lines: no single-address atomic contention).
__device__ __forceinline__ void block_add(uint32_t c, uint32_t* parts, long long a) {
    __shared__ uint32_t red[kBlock / 64];
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i) t += red[i];
        if (t) atomicAdd(part_slot(parts, a, blockIdx.x & (kParts - 1)), t);
    }
}

// Block-wide sum of one u32 per thread added to a u64 counter (kernel statistics only).
__device__ __forceinline__ void block_add_u64(uint32_t c, unsigned long long* ctr) {
    __shared__ uint32_t red[kBlock / 64];
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
#pragma unroll
        for (int i = 0; i < kBlock / 64; ++i) t += red[i];
        if (t) atomicAdd(ctr, t);
    }
}

// The same count added per wave (small graphs: no LDS round trip and no block barrier at the end
// of the round; most waves have nothing to add).
__device__ __forceinline__ void wave_add(uint32_t c, uint32_t* parts, long long a) {
    c = wave_sum(c);
    if ((threadIdx.x & 63u) == 0u && c)
        atomicAdd(part_slot(parts, a, (blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) & (kParts - 1)), c);
}

// Skip gate of a kernel that applies round `a`: the completion count after round a-1 is
// total[a-2] + the round a-1 sub-counters, all final (earlier launches).  Every block computes
// it (one wave, 64 loads), so every block takes the same branch; block 0 publishes total[a-1]
// and empties the ring slot that round a+2 will use.  Sharded: total[a-1] is the global count,
// already written by the exchange's unpack (k_shard_unpack).
__device__ __forceinline__ unsigned long long gate_count(const RoundArgs& A, long long a) {
    __shared__ unsigned long long prev_s;
    if (threadIdx.x < 64) {
        if (A.sharded) {
            if (threadIdx.x == 0) prev_s = a >= 1 ? A.total[a - 1] : 0ull;
        } else {
            // one round's completions fit in u32 (at most the node count)
            unsigned long long x = wave_sum(a >= 1 ? *part_slot(A.parts, a - 1, threadIdx.x) : 0u);
            if (threadIdx.x == 0) {
                if (a >= 2) x += A.total[a - 2];
                prev_s = x;
                if (blockIdx.x == 0 && a >= 1) A.total[a - 1] = x;
            }
        }
        if (blockIdx.x == 0) *part_slot(A.parts, a + 2, threadIdx.x) = 0u;
    }
    __syncthreads();
    return prev_s;
}

__device__ __forceinline__ bool gate(const RoundArgs& A, long long a) { return gate_count(A, a) >= A.target; }

// The same count computed by every wave for itself (no LDS, no block barrier): on a small graph
// the round is one dependent chain of a few loads, and the barrier gate sits at its head.  Every
// wave reads the same final values, so all waves of a block decide alike.
__device__ __forceinline__ unsigned long long gate_count_wave(const RoundArgs& A, long long a) {
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long x = 0;
    if (A.sharded) {
        x = a >= 1 ? A.total[a - 1] : 0ull;
    } else {
        // one round's completions fit in u32 (at most the node count)
        x = wave_sum(a >= 1 ? *part_slot(A.parts, a - 1, lane) : 0u);
        if (a >= 2) x += A.total[a - 2];
        if (blockIdx.x == 0 && threadIdx.x == 0 && a >= 1) A.total[a - 1] = x;
    }
    if (blockIdx.x == 0 && threadIdx.x < 64) *part_slot(A.parts, a + 2, lane) = 0u;
    return x;
}

// program.fs:119-143 for one actor (round 0 = :110-116): absorb, test, halve, emit.
// Returns the new message (s,w); sets conv_now when the actor converges this round.
struct PsOut {
    double2 msg;
    bool send;
    bool conv_now;
};

__device__ __forceinline__ PsOut ps_update(uint8_t& f, double2 held, double ss, double ww, uint32_t cin,
                                           double delta, uint32_t term_limit) {
    PsOut o;
    o.conv_now = false;
    if (f & 16u) {  // alreadyConverged: relay what arrived, if anything (program.fs:125-127)
        o.send = cin > 0;
        o.msg = make_double2(ss, ww);
        return o;
    }
    const double S = held.x, W = held.y;
    const double nS = S + ss, nW = W + ww;  // program.fs:120-121
    uint32_t term = f & 15u;
    if (cin > 0) {
        const double cal = fabs(S / W - nS / nW);  // program.fs:123
        term = cal > delta ? 0u : term + 1u;       // program.fs:130-133
        if (term == term_limit) {                  // program.fs:135-138
            term = 0u;
            o.conv_now = true;
        }
    }
    f = (uint8_t)(term | (o.conv_now ? 16u : 0u));
    o.msg = make_double2(nS * 0.5, nW * 0.5);  // program.fs:140-141 (x/2 == x*0.5 exactly)
    o.send = true;
    return o;
}

// ------------------------------------------------------------------ shard exchange helpers
// Lanes below this one whose bit is set in m.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Owner rank of x under the range bounds b[0..world] (world <= 16: a short uniform loop).
__device__ __forceinline__ uint32_t owner(const uint32_t* b, uint32_t world, uint32_t x) {
    uint32_t q = 0;
    for (uint32_t i = 1; i < world; ++i) q += x >= b[i] ? 1u : 0u;
    return q;
}

__device__ __forceinline__ uint32_t* ctr_at(const Xchg& x, uint32_t q, uint32_t sub) {
    return x.pcount + (q * kSub + sub) * kCtrStride;
}

__device__ __forceinline__ uint32_t my_sub() { return blockIdx.x % kSub; }

// Append (entry, msg) to peer q's chunk, sub-segment my_sub(), at pos, or flag the overflow (never
// silently dropped: gp_shard_sync fails the run with GP_EOVERFLOW).
template <bool MSG>
__device__ __forceinline__ void put(const Xchg& x, uint32_t q, uint32_t pos, uint32_t entry, double2 m,
                                    uint32_t sub = kSub) {
    const PeerOut& o = x.out[q];
    if (pos < o.cap) {
        const uint32_t i = (sub < kSub ? sub : my_sub()) * o.cap + pos;
        o.slot[i] = entry;
        if (MSG) o.msg[i] = m;
    } else {
        atomicOr(x.overflow, 1u);
    }
}

// The peers' send chunks in LDS, filled by the block's reservation (block_reserve / block_reserve_qs)
// before its first barrier: put_t reads a lane's peer there.  (put indexes the kernel arguments by a
// per-lane peer, one vector load per field and entry, which keeps the texture path busy.)
struct PeerTab {
    uint32_t* slot[kMaxWorld];
    double2* msg[kMaxWorld];
    uint32_t cap[kMaxWorld];
    uint32_t sbnd[kMaxWorld + 1];  // the ranks' slot bounds (owner_t: no SGPRs held for them in a walk)
};
__device__ __forceinline__ PeerTab& peer_tab() {
    __shared__ PeerTab t;
    return t;
}
__device__ __forceinline__ void peer_tab_fill(const Xchg& x) {
    if (threadIdx.x < kMaxWorld) {
        PeerTab& t = peer_tab();
        const PeerOut& o = x.out[threadIdx.x];
        t.slot[threadIdx.x] = o.slot;
        t.msg[threadIdx.x] = o.msg;
        t.cap[threadIdx.x] = o.cap;
    }
    if (threadIdx.x <= x.world) peer_tab().sbnd[threadIdx.x] = x.sbnd[threadIdx.x];
}
// owner(x.sbnd, x.world, lp) from the LDS table (after peer_tab_fill and a barrier).
__device__ __forceinline__ uint32_t owner_t(uint32_t world, uint32_t lp) {
    const PeerTab& t = peer_tab();
    uint32_t q = 0;
    for (uint32_t i = 1; i < world; ++i) q += lp >= t.sbnd[i] ? 1u : 0u;
    return q;
}
// The two halo faces' entry parts, likewise (a shard's tail round writes them itself).
struct HaloTab {
    uint32_t* slot[2];
    double2* msg[2];
    uint32_t cap[2];
};
__device__ __forceinline__ HaloTab& halo_tab() {
    __shared__ HaloTab t;
    return t;
}
__device__ __forceinline__ void halo_tab_fill(const Xchg& x) {
    if (threadIdx.x < 2u) {
        HaloTab& t = halo_tab();
        t.slot[threadIdx.x] = x.h.out_slot[threadIdx.x];
        t.msg[threadIdx.x] = x.h.out_msg[threadIdx.x];
        t.cap[threadIdx.x] = x.h.out_cap[threadIdx.x];
    }
}
template <bool MSG>
__device__ __forceinline__ void put_t(const Xchg& x, uint32_t q, uint32_t pos, uint32_t entry, double2 m,
                                      uint32_t sub = kSub) {
    const PeerTab& t = peer_tab();
    const uint32_t cap = t.cap[q];
    if (pos < cap) {
        const uint32_t i = (sub < kSub ? sub : my_sub()) * cap + pos;
        t.slot[q][i] = entry;
        if (MSG) t.msg[q][i] = m;
    } else {
        atomicOr(x.overflow, 1u);
    }
}

// Wave-level reservation for one entry per lane (lanes with want): one atomic per peer present on
// the sub-segment counter of peer q (the quiet-tail rounds of a shard, where entries are few and the
// walk is per wave).  Every lane of the wave must call it.
__device__ __forceinline__ uint32_t wave_reserve(const Xchg& x, bool want, uint32_t q) {
    uint64_t left = __ballot(want), mine = 0;
    if (!left) return 0;
    while (left) {  // wave-uniform: the lanes of one peer per trip (ballots only, no memory)
        const uint32_t lead = (uint32_t)__builtin_ctzll(left);
        const uint32_t pq = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)lead);
        const uint64_t m = __ballot(want && q == pq);
        if (want && q == pq) mine = m;
        left &= ~m;
    }
    // one atomic per peer, all in flight together (one after another, each waited for, they put a
    // returning atomic's latency per peer into a tail pass)
    const uint32_t lead = (uint32_t)__builtin_ctzll(mine | (1ull << 63));
    uint32_t base = 0;
    if (want && (threadIdx.x & 63u) == lead) base = atomicAdd(ctr_at(x, q, my_sub()), (uint32_t)__popcll(mine));
    base = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead << 2), (int)base);
    return want ? base + mbcnt64(mine) : 0u;
}

// A shard's dense round routes its own link messages (kShardFuse): the round kernel has each message in
// registers when its actor fires the extra link, so a remote one is staged in LDS (slot, message, peer,
// position among the block's entries to that peer) instead of being re-read from msg_cur by a separate
// pass over every actor (k_ps_link_scatter_x: 0.61 ms per C5 / 8 rank-round).  Every kFuseIters
// iterations of the walk (block-uniform) the block reserves its staged entries' positions, one atomic
// per peer, and writes the entries of the step before, whose reservation has come back meanwhile: two
// stage buffers, so no workgroup waits for a returning atomic.  A step's entries go to sub-segment
// (block + step) mod kSub, so a small grid still spreads them over every sub-segment.
#ifndef GP_FUSE_STAGE
#define GP_FUSE_STAGE 256  // (a test build with 8 sends most entries down the full-buffer path)
#endif
#ifndef GP_FUSE_ITERS
#define GP_FUSE_ITERS 4
#endif
constexpr uint32_t kFuseStage = GP_FUSE_STAGE, kFuseIters = GP_FUSE_ITERS;
struct FuseStage {
    uint32_t n[2];                  // entries staged per buffer (past kFuseStage: placed directly)
    uint32_t cnt[2][kMaxWorld];     // per peer
    uint32_t base[kMaxWorld];       // the reserved positions of the buffer being written out
    uint32_t slot[2][kFuseStage];
    uint32_t qp[2][kFuseStage];     // peer << 16 | position among the buffer's entries to that peer
    double2 msg[2][kFuseStage];
};
__device__ __forceinline__ FuseStage& fuse_stage() {
    __shared__ FuseStage s;
    return s;
}
// Walk state of the fused dense round (per thread, uniform over the block but res).
struct FuseWalk {
    uint32_t it = 0, step = 0, res = 0;  // res: thread q < world holds the last reservation of peer q
};
__device__ __forceinline__ uint32_t fuse_sub(uint32_t step) { return (blockIdx.x + step) % kSub; }
// Before the block's first barrier.
__device__ __forceinline__ void fuse_init() {
    FuseStage& S = fuse_stage();
    if (threadIdx.x < 2u) S.n[threadIdx.x] = 0u;
    if (threadIdx.x < 2u * kMaxWorld) (&S.cnt[0][0])[threadIdx.x] = 0u;
}
// Stage one entry (any lane, divergent code).
__device__ __forceinline__ void fuse_put(const Xchg& x, const FuseWalk& w, uint32_t q, uint32_t lp, double2 m) {
    FuseStage& S = fuse_stage();
    const uint32_t b = w.step & 1u;
    const uint32_t i = atomicAdd(&S.n[b], 1u);
    if (i < kFuseStage) {
        const uint32_t p = atomicAdd(&S.cnt[b][q], 1u);
        S.slot[b][i] = lp;
        S.qp[b][i] = q << 16 | p;
        S.msg[b][i] = m;
    } else {  // the buffer is full (statistically never: 4 x 256 actors stage ~128): its own position
        const uint32_t sub = fuse_sub(w.step);
        put_t<true>(x, q, atomicAdd(ctr_at(x, q, sub), 1u), lp, m, sub);
    }
}
// Write out buffer b (reserved at step s) with the bases in S.base.  Every thread calls it.
__device__ __forceinline__ void fuse_write(const Xchg& x, uint32_t b, uint32_t n, uint32_t s) {
    FuseStage& S = fuse_stage();
    const uint32_t sub = fuse_sub(s);
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) {
        const uint32_t qp = S.qp[b][i], q = qp >> 16;
        put_t<true>(x, q, S.base[q] + (qp & 0xFFFFu), S.slot[b][i], S.msg[b][i], sub);
    }
}
// End of a step (block-uniform; every thread calls it): reserve this step's entries, write the previous
// step's.  Returns whether any thread has actors left; when none has, also writes this step's (the end).
__device__ __forceinline__ bool fuse_flush(const Xchg& x, FuseWalk& w, bool left) {
    FuseStage& S = fuse_stage();
    const bool more = __syncthreads_or(left);  // (the step's staging is done)
    const uint32_t b = w.step & 1u, pb = b ^ 1u;
    const uint32_t np = min(S.n[pb], kFuseStage), nb = min(S.n[b], kFuseStage);
    if (threadIdx.x < x.world) {
        S.base[threadIdx.x] = w.res;  // the previous step's reservation (issued one step ago)
        const uint32_t c = S.cnt[b][threadIdx.x];
        w.res = c ? atomicAdd(ctr_at(x, threadIdx.x, fuse_sub(w.step)), c) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < kMaxWorld) S.cnt[pb][threadIdx.x] = 0u;
    if (threadIdx.x == 0) S.n[pb] = 0u;
    if (w.step) fuse_write(x, pb, np, w.step - 1u);
    __syncthreads();  // (buffer pb and the bases are free again)
    if (!more) {
        if (threadIdx.x < x.world) S.base[threadIdx.x] = w.res;
        __syncthreads();
        fuse_write(x, b, nb, w.step);
        return false;
    }
    w.step = (uint32_t)__builtin_amdgcn_readfirstlane((int)(w.step + 1u));
    w.it = 0;
    return true;
}

// ------------------------------------------------------------------ push-sum, grid topologies
// Grid in-neighbour slots in ascending source order: v-P, v-G, v-1, v+1, v+G, v+P (presence
// bits 4, 2, 0, 1, 3, 5); the sender in slot k targets v iff its direction code is the
// opposite one (5, 3, 1, 0, 2, 4).
// (Bit masks, not a switch or a select chain: with a run-time k those compile to a divergent
// branch tree.)
__device__ __forceinline__ uint32_t slot_src(const Geom& g, uint32_t v, uint32_t k) {
    const uint32_t kk = k < 3u ? k : 5u - k;  // 0: +-G^2, 1: +-G, 2: +-1
    const uint32_t mag = (g.plane & (0u - (uint32_t)(kk == 0u))) | (g.gx & (0u - (uint32_t)(kk == 1u))) |
                         (uint32_t)(kk == 2u);
    return k < 3u ? v - mag : v + mag;
}

// Slot k of v exists iff presence bit kSlotBit(k) is set; its sender targets v iff its
// direction code is kSlotCode(k).
__device__ __forceinline__ uint32_t slot_bit(uint32_t k) { return k == 0 ? 16u : k == 1 ? 4u : k == 2 ? 1u : k == 3 ? 2u : k == 4 ? 8u : 32u; }
__device__ __forceinline__ uint32_t slot_code(uint32_t k) { return k == 0 ? 5u : k == 1 ? 3u : k == 2 ? 1u : k == 3 ? 0u : k == 4 ? 2u : 4u; }

// Branch-free load: a predicated-off lane reads `fallback` (an element it already touches),
// so hipcc emits straight-line loads instead of one basic block + vmcnt(0) per condition
// (round 3, C3 all-sending rounds: the grid-hit and link message loads exec-masked 298 vs 202
// us; a wave-uniform skip of the 3rd / 4th link message load when no lane needs it 244 vs 200
// us, profiles/round3/load_shape_ab).
template <class T>
__device__ __forceinline__ T load_sel(const T* base, bool pred, uint32_t idx, uint32_t fallback) {
    return base[pred ? idx : fallback];
}

// The message loads of lanes without a grid hit / fired link read one row shared by the whole
// grid (msg_prev[lo]) rather than the actor's own row: a wave's predicated-off lanes then touch one
// line instead of eight, and a converged actor, which never reads its own row, no longer pulls it
// in (all-sending C3 round 195.5 -> 189.8 us, profiles/round3/fallback_ab).

// Link slots scanned with unrolled loads before the (rare) tail loop.
#ifndef GP_LINK_UNROLL
#define GP_LINK_UNROLL 4
#endif
constexpr uint32_t kLinkUnroll = GP_LINK_UNROLL;
// Message loads issued for an actor's first GP_GRID_LOADS grid hits (A/B knob); later hits are
// loaded on demand.  2 instead of 3: neutral (profiles/round3/held_ab).
#ifndef GP_GRID_LOADS
#define GP_GRID_LOADS 3
#endif
constexpr uint32_t kGridLoads = GP_GRID_LOADS;

static_assert(kGridLoads >= 1 && kGridLoads <= 6, "GP_GRID_LOADS: 1 .. 6");
// One GPU: message loads issued for the first GP_FIRED_LOADS fired link slots of an actor, the
// others on demand (GP_LINK_UNROLL: one per unrolled slot, fired or not).  1: C3 -3%, 100M -1%
// against 4 (each predicated 16-byte load instruction costs ~1.5% of an all-sending round,
// profiles/round3/load_shape_ab); 2: C3 -2%, 100M +0.5%.
#ifndef GP_FIRED_LOADS
#define GP_FIRED_LOADS 1
#endif
constexpr uint32_t kFiredLoads = GP_FIRED_LOADS;

// The CSR offsets of v (rev_off[v], rev_off[v + 1]) are one 8-byte load, the four unrolled slots'
// sources one 16-byte load and their marks two dwords (round 3: C3 -5.9%, 100M -6.1% against one
// load per element, profiles/round3/csr_vec_ab).  Dword-aligned 8- and 16-byte loads (and
// byte-aligned ones) return the right bytes on gfx950 (tools/microbench/unaligned.hip).  The marks
// as one byte-aligned dword and the +-1 neighbours' direction bytes as one dword at v - 1 as well:
// neutral (one-byte loads are cheap; the 16-byte ones fill the texture data path).
// The quiet-wave round kernel's SGPR cap (GP_PSQ_SGPR, 0 = the compiler's choice).  A 256-thread
// workgroup is admitted per CU only while 800 / (ceil(sgpr / 16) * 16 + 16) allows it
// (MI355X_MICROARCH.md, residency): 106 SGPRs -> 6 workgroups, <= 96 -> 7, <= 80 -> 8.
#ifndef GP_PSQ_SGPR
#define GP_PSQ_SGPR 96
#endif
#ifndef GP_PSQ_WAVES
#define GP_PSQ_WAVES 7
#endif
#if GP_PSQ_SGPR > 0
#define GP_PSQ_SGPR_ATTR __attribute__((amdgpu_num_sgpr(GP_PSQ_SGPR)))
#else
#define GP_PSQ_SGPR_ATTR
#endif


// Cache policy of the link-mark stores (one random byte per fired link; GP_MARK_POL, A/B knob: 0
// plain, 1 non-temporal, 2 non-temporal up to kMarkNtNodes nodes) in the one-GPU round kernel.  The marks of a round are
// ~1.4M random bytes at 10M nodes that the next round reads back in CSR order; stored plainly they
// cost 27 us of a 206 us all-sending round (a timing-only build storing them into a cache-resident
// prefix ran 179 us, profiles/round3/mark_ab), stored non-temporally 6 us less (C3 -2%), while at
// 100M nodes non-temporal marks were 1.8% slower over a run; sc1 / sc0 sc1 write-through stores
// gained nothing.  The shard passes store their marks plainly (the unpack's non-temporal marks
// cost 0.29 ms more per rank-round at C5 / 8, profiles/round3/mark_ab/loop_policies.txt).  GP_ACT_POL: the same choice for the quiet-segment marks (plain: nt was slower).
#ifndef GP_MARK_POL
#define GP_MARK_POL 2
#endif
#ifndef GP_ACT_POL
#define GP_ACT_POL 0
#endif
constexpr uint32_t kMarkNtNodes = 1u << 25;
template <int POL>
__device__ __forceinline__ void byte_store(uint8_t* p, uint8_t x) {
    if constexpr (POL == 1) {
        __builtin_nontemporal_store(x, p);
    } else {
        *p = x;
    }
}
__device__ __forceinline__ void mark_store(const RoundArgs& a, uint8_t* p, uint8_t x) {
    if (GP_MARK_POL == 1 || (GP_MARK_POL == 2 && a.nodes <= kMarkNtNodes)) {  // uniform
        byte_store<1>(p, x);
    } else {
        byte_store<0>(p, x);
    }
}

// One actor's round (program.fs:119-143 after collecting the round r-1 messages to v).
// Collect = the canonical sequential fp64 sum, from +0.0, of the messages sent to v in ascending
// source id.  Messages are never copied on one GPU: a message IS the sender's held state, so a
// grid sender's message is read from msg_prev at v-G^2, v-G, v-1, v+1, v+G or v+G^2 (a sender
// targets v iff its direction byte is the opposite code), and an extra-link sender u (CSR
// rev_src, ascending) from msg_prev[u] iff k_link_count marked u's CSR slot.  Loads are
// unconditional (clamped addresses) in three dependency levels: (1) own flags, held (S,W), the
// six neighbours' direction bytes, the CSR range; (2) the first 3 grid hits' messages and, per
// CSR slot of the first kLinkUnroll, the source id and link count (coalesced: CSR order);
// (3) the messages of the links that fired.
// LM: 0 no extra links; 1 links; 2 links on a shard of several ranks: a sender outside [lo, hi)
// is remote, and the exchange wrote its message into the receiver's slot, rmsg_prev[slot]; 3 links
// on a small one-GPU graph: every link sender writes its message into the receiver's slot
// (rmsg_cur[lpos[v]]) as well as its own row, so the receiver loads the slot messages together
// with the slot sources and marks (one dependent load level less: the round is latency-bound).

// Level 1 of one actor's loads (own flags, the six neighbours' direction bytes, the CSR range),
// split out so the small-graph kernel can issue them before its gate resolves.  PRE (small
// graphs, where the round is latency-bound and bytes are cheap): also the held (S,W) and all six
// neighbours' messages, hit or not, so the grid part of the collect needs no second level.
struct PsLevel1 {
    uint32_t m, li, nl;
    uint32_t f;
    uint32_t d[6];  // one register per byte: packing them would wait for the loads
    double2 held;
    double2 gm6[6];  // PRE: the six neighbours' messages (slot order)
};

template <int LM, bool PRE = false>
__device__ __forceinline__ PsLevel1 ps_level1(const RoundArgs& a, const Geom& g, uint32_t r, uint32_t v) {
    PsLevel1 p;
    p.m = presence(g, v);
    p.f = a.flags[v];
    p.held = make_double2((double)v, 1.0);
    p.li = 0;
    p.nl = 0;
    if (PRE || r) {  // PRE: unconditional (no join for the loaded registers; ps_finish ignores
                     // them in round 0, when the buffers hold no messages yet)
        if (PRE) p.held = a.msg_prev[v];
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k) {
            p.d[k] = load_sel(a.dir_prev, (p.m & slot_bit(k)) != 0u, slot_src(g, v, k), v);
        }
        if constexpr (PRE) {
#pragma unroll
            for (uint32_t k = 0; k < 6; ++k)
                p.gm6[k] = load_sel(a.msg_prev, (p.m & slot_bit(k)) != 0u, slot_src(g, v, k), v);
        }
        if (LM) {  // rev_off[v], rev_off[v + 1] in one 8-byte load
            typedef uint32_t u2v __attribute__((ext_vector_type(2)));
            u2v o;
            __builtin_memcpy(&o, &a.rev_off[v], sizeof o);
            p.li = o.x;
            p.nl = o.y - o.x;
        }
    }
    return p;
}

// FF: message loads for the first kFiredLoads FIRED link slots only (one GPU; the shards' quiet
// kernel, which spills with one load per unrolled slot) instead of one per unrolled slot.
// A shard's quiet-tail round routes its own link messages (the scatter pass's work in the dense
// rounds): ps_finish reports the message of an actor whose round-r message took its extra link.
// HD (a shard's tail round that writes its own halo faces, k_ps_quiet_x<true>): also every send's
// direction code and message.
struct LinkSend {
    bool fired = false;
    double2 msg;
    uint32_t dir = kDirNone;
};

template <int LM, bool PRE = false, bool FF = (LM == 1), bool HD = false>
__device__ __forceinline__ uint32_t ps_finish(const RoundArgs& a, const Geom& g, uint32_t r, uint32_t v,
                                              const PsLevel1& p, bool mark, LinkSend* ls = nullptr) {
    const uint32_t m = p.m;
    if (!m) return 0;
    const uint32_t code = kth_bit(m, scale_draw(philox_x(v, r, kStreamPush, a.seed), popc(m)));
    uint8_t f = (uint8_t)p.f;
    double2 held = (PRE && !r) ? make_double2((double)v, 1.0) : p.held;
    double ss = 0.0, ww = 0.0;
    uint32_t cin = 0;
    if (r) {
        const uint32_t* d = p.d;
        const uint32_t li = p.li, nl = p.nl;
        uint32_t hits = 0;
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k) hits |= ((m & slot_bit(k)) && d[k] == slot_code(k)) ? 1u << k : 0u;
        // The first kGridLoads grid hits (slot order = ascending source id) and their sources
        // (none: above every bound), computed once for the loads and the merge.
        uint32_t gs[kGridLoads], rest = hits;
#pragma unroll
        for (int j = 0; j < (int)kGridLoads; ++j) {
            gs[j] = slot_src(g, v, (uint32_t)__builtin_ctz(rest | 64u)) | (0u - (uint32_t)(rest == 0u));
            rest &= rest - 1u;
        }
        double2 gm[kGridLoads];
#pragma unroll
        for (int j = 0; j < (int)kGridLoads; ++j)
            gm[j] = PRE ? make_double2(0.0, 0.0) : load_sel(a.msg_prev, gs[j] != 0xFFFFFFFFu, gs[j], a.lo);
        uint32_t pend = hits;  // PRE: grid hits not yet added
        // A converged actor only relays what arrives (program.fs:125-127): its held (S,W) and so
        // its message row are not read (more than half of the C3 run's actor-rounds).  Issued
        // with the second load level, when the flags byte has long arrived.
        if constexpr (!PRE) held = load_sel(a.msg_prev, !(f & 16u), v, a.lo);
        uint32_t gi = 0;
        auto add = [&](double2 mm) {
            ss += mm.x;
            ww += mm.y;
            ++cin;
        };
        // Add the pending grid hits whose source is below `bound`, in ascending order.  (A
        // branch-free form with predicated exact +0.0 adds ran 1-4% slower: more VALU work.)
        auto flush = [&](uint32_t bound) {
            if constexpr (PRE) {  // slot order = ascending source: each test is independent
#pragma unroll
                for (uint32_t k = 0; k < 6; ++k)
                    if (((pend >> k) & 1u) && slot_src(g, v, k) < bound) {
                        add(p.gm6[k]);
                        pend &= ~(1u << k);
                    }
                return;
            }
#pragma unroll
            for (int j = 0; j < (int)kGridLoads; ++j)
                if (gi == (uint32_t)j && gs[j] < bound) {
                    add(gm[j]);
                    ++gi;
                }
            if (gi >= kGridLoads) {
                while (rest) {
                    const uint32_t k = (uint32_t)__builtin_ctz(rest);
                    const uint32_t u = slot_src(g, v, k);
                    if (u >= bound) break;
                    add(a.msg_prev[u]);
                    rest &= rest - 1u;
                }
            }
        };
        if (LM) {
            uint32_t ls[kLinkUnroll];
            bool lk[kLinkUnroll];
            double2 lm[kLinkUnroll];
            uint32_t lc[kLinkUnroll];
            uint32_t lr[kLinkUnroll];  // LM 2: the slots' references
            static_assert(kLinkUnroll == 4, "GP_LINK_UNROLL: the slots load as one 16-byte load");
            {
                // the four unrolled slots' sources as one 16-byte load and their marks as two
                // aligned dwords (slots past nl belong to the next actors and are ignored; the
                // arrays are padded past their last slot)
                typedef uint32_t u4v __attribute__((ext_vector_type(4)));
                u4v s4;
                __builtin_memcpy(&s4, &a.rev_src[li], sizeof s4);
                ls[0] = s4.x;
                ls[1] = s4.y;
                ls[2] = s4.z;
                ls[3] = s4.w;
                if constexpr (LM == 2) {  // four 32-bit references, one 16-byte load like the sources
                    u4v r4;
                    __builtin_memcpy(&r4, &a.lref_prev[li], sizeof r4);
                    lr[0] = r4.x;
                    lr[1] = r4.y;
                    lr[2] = r4.z;
                    lr[3] = r4.w;
                    // (separate registers: a select over lanes of one vector value can become an indexed
                    // read of a scratch copy when the kernel's registers are short, k_ps_quiet_x)
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) asm volatile("" : "+v"(lr[k]));
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) lc[k] = lr[k] & kRefTagMask;
                } else {
                    const uint32_t* mw = reinterpret_cast<const uint32_t*>(a.lcnt_prev + (li & ~3u));
                    const uint64_t m8 = (uint64_t)mw[0] | ((uint64_t)mw[1] << 32);
                    const uint32_t sh = 8u * (li & 3u);
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) lc[k] = (uint8_t)(m8 >> (sh + 8u * k));
                }
            }
            // ---- level 3: the messages of the sources whose slot is marked
#pragma unroll
            for (uint32_t k = 0; k < kLinkUnroll; ++k)
                lk[k] = k < nl && lc[k] == (LM == 2 ? a.rtag_prev : a.tag_prev);  // round tags
            if constexpr (LM != 0 && kFiredLoads < kLinkUnroll && FF) {
                // load the messages of the first kFiredLoads FIRED slots only (about one slot in
                // seven fires: 0.14 messages per actor), the rest on demand (rare).  A shard reads
                // a remote source's message from the receive buffer its slot's reference points into,
                // a local one from the source's row: one load through a selected address.
                uint32_t rest = 0;
#pragma unroll
                for (uint32_t k = 0; k < kLinkUnroll; ++k) rest |= lk[k] ? 1u << k : 0u;
                auto msg_of = [&](uint32_t k, uint32_t u) -> const double2* {
                    if (LM == 2 && (u < a.olo || u >= a.ohi)) {
                        uint32_t rf = lr[0];
#pragma unroll
                        for (uint32_t q = 1; q < kLinkUnroll; ++q) {
                            rf = k == q ? lr[q] : rf;
                            asm volatile("" : "+v"(rf));  // (a select chain, not an indexed read)
                        }
                        return a.rin_prev + (rf >> kRefShift);
                    }
                    return a.msg_prev + u;
                };
                uint32_t fs[kFiredLoads];
                bool fv[kFiredLoads];
                double2 fm[kFiredLoads];
#pragma unroll
                for (uint32_t j = 0; j < kFiredLoads; ++j) {
                    const uint32_t k = (uint32_t)__builtin_ctz(rest | (1u << kLinkUnroll));
                    fv[j] = rest != 0u;
                    uint32_t u = ls[0];
#pragma unroll
                    for (uint32_t q = 1; q < kLinkUnroll; ++q) u = k == q ? ls[q] : u;
                    fs[j] = u;
                    fm[j] = *(fv[j] ? msg_of(k, u) : a.msg_prev + a.lo);
                    rest &= rest - 1u;
                }
#pragma unroll
                for (uint32_t j = 0; j < kFiredLoads; ++j)
                    if (fv[j]) {
                        flush(fs[j]);
                        add(fm[j]);
                    }
                while (rest) {  // rare: more than kFiredLoads of the unrolled slots fired
                    const uint32_t k = (uint32_t)__builtin_ctz(rest);
                    uint32_t u = ls[0];
#pragma unroll
                    for (uint32_t q = 1; q < kLinkUnroll; ++q) u = k == q ? ls[q] : u;
                    flush(u);
                    add(*msg_of(k, u));
                    rest &= rest - 1u;
                }
            } else {
#pragma unroll
                for (uint32_t k = 0; k < kLinkUnroll; ++k) {
                    if constexpr (LM == 3) {  // the slot holds the message: its address needs only li,
                                              // so the load goes out with the sources and marks
                        lm[k] = load_sel(a.rmsg_prev, k < nl, li + k, a.slot_lo);
                    } else if (LM == 2 && lk[k] && (ls[k] < a.olo || ls[k] >= a.ohi)) {
                        lm[k] = a.rin_prev[lr[k] >> kRefShift];
                    } else {
                        lm[k] = load_sel(a.msg_prev, lk[k], ls[k], a.lo);
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < kLinkUnroll; ++k)
                    if (lk[k]) {
                        flush(ls[k]);
                        add(lm[k]);
                    }
            }
            for (uint32_t k = kLinkUnroll; k < nl; ++k) {  // rare: more than kLinkUnroll sources
                const uint32_t rf = LM == 2 ? a.lref_prev[li + k] : 0u;
                if (LM == 2 ? (rf & kRefTagMask) == a.rtag_prev : a.lcnt_prev[li + k] == a.tag_prev) {
                    const uint32_t u = a.rev_src[li + k];
                    flush(u);
                    add(LM == 3 ? a.rmsg_prev[li + k]
                                : LM == 2 && (u < a.olo || u >= a.ohi) ? a.rin_prev[rf >> kRefShift] : a.msg_prev[u]);
                }
            }
        }
        flush(0xFFFFFFFFu);
    }
    const uint8_t f0 = f;
    const PsOut o = ps_update(f, held, ss, ww, cin, a.delta, a.term_limit);
    // non-temporal: the round's 160 MB of messages cannot stay in L2 until the next round
    // reads them, and streaming them past it leaves L2 to the +-G, +-G^2 rows read now
    // (measured ~1.5% per round; non-temporal LOADS of the CSR were 7% slower)
    if (o.send) {
        __builtin_nontemporal_store(o.msg.x, &a.msg_cur[v].x);
        __builtin_nontemporal_store(o.msg.y, &a.msg_cur[v].y);
    }
    __builtin_nontemporal_store(o.send ? (uint8_t)code : kDirNone, &a.dir_cur[v]);
    if constexpr (LM == 1 && kFuseLinkMarks) {  // the link pass's mark, written by the sender
        if (o.send && code == kDirLink) mark_store(a, &a.lcnt_cur[a.lpos[v]], (uint8_t)a.tag_cur);
    }
    if constexpr (LM == 3) {  // small graphs: the message into the receiver's slot too, and its mark
        if (o.send && code == kDirLink) {
            const uint32_t lp = a.lpos[v];
            a.rmsg_cur[lp] = o.msg;
            a.lcnt_cur[lp] = (uint8_t)a.tag_cur;
        }
    }
    if constexpr (LM == 2 && HD) {
        ls->dir = o.send ? code : kDirNone;
        ls->fired = o.send && code == kDirLink;
        ls->msg = o.msg;
    } else if (LM == 2 && ls && o.send && code == kDirLink) {
        ls->fired = true;
        ls->msg = o.msg;
    }
    if (f != f0) a.flags[v] = f;
    if (o.conv_now) a.frozen[v] = o.msg;
    if (mark) {  // the waves with work in round r + 1: v's own if it still updates, its target's
        const uint8_t t = (uint8_t)link_tag(r + 1u);
        if (!(f & 16u)) byte_store<GP_ACT_POL>(&a.act_cur[v >> kActShift], t);
        if (o.send) {
            const uint32_t tv = dir_target(g, v, code, code == kDirLink ? link_of(a.seed, v, a.nodes) : 0u);
            // a shard marks its own actors only: the receiver of a message that leaves the range
            // marks it when the exchange delivers it (k_shard_unpack)
            // (LM 1 and 3 run on one GPU only)
            if (LM == 1 || LM == 3 || !a.sharded || tv - a.olo < a.ohi - a.olo)
                byte_store<GP_ACT_POL>(&a.act_cur[tv >> kActShift], t);
        }
    }
    return o.conv_now ? 1u : 0u;
}

template <int LM, bool FF = (LM == 1), bool HD = false>
__device__ __forceinline__ uint32_t ps_actor(const RoundArgs& a, const Geom& g, uint32_t r, uint32_t v,
                                             bool mark = false, LinkSend* ls = nullptr) {
    return ps_finish<LM, false, FF, HD>(a, g, r, v, ps_level1<LM>(a, g, r, v), mark, ls);
}

// The quiet-wave tail with compaction.  Marks are per segment of kActSeg actors: F(r) marks the
// segment of every actor that still updates and of every message's target.  In F(r + 1) a wave
// reads the marks of 64 consecutive segments (its XCD group's span, grid-stride), writes "send
// nothing" (kDirNone) into the direction bytes of the unmarked ones — they hold only converged
// actors and receive nothing, so that is their whole round — and then walks the marked
// segments only, 64 / kActSeg of them per pass of its 64 lanes (each segment's actors stay
// contiguous in a lane group, so the loads keep their coalescing).  With 64-actor marks nearly
// every wave of the tail had work (86% at 3% active actors); 4-actor segments (16 per pass) walk
// about 3.8 actors per active one at 3% active actors (16-actor segments: 12.9).
// One walk loop with one ps_actor call serves both the dense rounds and the tail (two inlined
// copies of the actor body cost 4 spilled VGPRs and a wave per SIMD).
// Walk state of the compacted tail (per wave): the next 64-segment chunk of the XCD group's span,
// the marks of that chunk and the one after it (prefetched: a chunk is opened without waiting for
// its load), and the marked segments listed but not walked yet (in LDS).
constexpr uint32_t kTailList = 128;  // >= 64 / kActSeg - 1 leftovers + one chunk of 64
static_assert(kTailList >= 64u / kActSeg - 1u + 64u, "tail list capacity");
struct TailWalk {
    uint32_t base, s1, stride, c, k;
    uint32_t* list;
    uint32_t pf0, pf1;
};

__device__ __forceinline__ uint32_t tail_mark(const RoundArgs& a, const TailWalk& t, uint32_t chunk) {
    const uint32_t seg = chunk + (threadIdx.x & 63u);
    return chunk < t.s1 && seg < t.s1 ? a.act_prev[seg] : 0u;
}

__device__ __forceinline__ TailWalk tail_walk(const RoundArgs& a, bool tail) {
    __shared__ uint32_t seg_list[kBlock / 64u * kTailList];
    TailWalk t;
    // segments are global (actor >> kActShift): a shard walks the ones that hold its actors
    // [lo, hi) (its piece's); a segment astride lo or hi is walked by both ranks, each for its own
    // actors (piece bounds inside a rank's range are whole segments)
    const uint32_t sg0 = a.lo >> kActShift, sg1 = (a.hi + kActSeg - 1u) >> kActShift, nseg = sg1 - sg0;
    const uint32_t grp = blockIdx.x & 7u, wpg = (gridDim.x >> 3) * (kBlock / 64u);
    const uint32_t wid = (blockIdx.x >> 3) * (kBlock / 64u) + (threadIdx.x >> 6);
    const uint32_t sspan = ((nseg + 7u) / 8u + 63u) / 64u * 64u;
    const uint32_t s0 = sg0 + grp * sspan;
    t.s1 = s0 + sspan < sg1 ? s0 + sspan : sg1;
    t.base = s0 + wid * 64u;
    t.stride = wpg * 64u;
    t.c = t.k = 0;
    t.list = seg_list + (threadIdx.x >> 6) * kTailList;
    t.pf0 = tail ? tail_mark(a, t, t.base) : 0u;
    t.pf1 = tail ? tail_mark(a, t, t.base + t.stride) : 0u;
    return t;
}

// The next actor of this lane in the compacted tail walk (a.hi: none this pass); false when the
// wave's span is done.  Wave-uniform.  Chunks are opened until a full pass of 64 / kActSeg marked
// segments is listed (or the span ends), so a pass of the late tail, where a chunk holds one or
// two marked segments, keeps its 64 lanes busy (one pass per chunk left 1-2 segments per pass);
// each chunk's unmarked segments get "send nothing" (kDirNone) direction bytes as it is opened.
// HIN (a shard's tail round that writes its own halo faces): those of face actors into the chunks
// of rank -+ 1 too.
template <bool HIN = false>
__device__ __forceinline__ bool tail_next(const RoundArgs& a, TailWalk& t, uint8_t tag, uint32_t& v,
                                          const Xchg* hx = nullptr) {
    constexpr uint32_t S = kActSeg, PER = 64u / kActSeg;
    const uint32_t lane = threadIdx.x & 63u;
    while (t.c - t.k < PER && t.base < t.s1) {
        if (t.k) {  // fewer than PER left: move them to the front (one read, then one write)
            const uint32_t left = t.c - t.k;
            const uint32_t x = lane < left ? t.list[t.k + lane] : 0u;
            if (lane < left) t.list[lane] = x;
            t.c = left;
            t.k = 0;
        }
        const uint32_t seg = t.base + lane;
        const bool valid = seg < t.s1;
        const bool act = valid && t.pf0 == tag;
        t.pf0 = t.pf1;
        t.pf1 = tail_mark(a, t, t.base + 2u * t.stride);
        if (valid && !act) {  // kActSeg direction bytes (the array is padded past the last actor)
            uint8_t* d = a.dir_cur + (size_t)seg * S;
            static_assert(kDirNone == 7, "kDirNone bytes");
            if constexpr (S == 16u) {
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 none = {0x07070707u, 0x07070707u, 0x07070707u, 0x07070707u};
                __builtin_nontemporal_store(none, reinterpret_cast<u4*>(d));
            } else if constexpr (S == 4u) {
                __builtin_nontemporal_store(0x07070707u, reinterpret_cast<uint32_t*>(d));
            } else {
#pragma unroll
                for (uint32_t i = 0; i < S; ++i) __builtin_nontemporal_store(kDirNone, d + i);
            }
            if constexpr (HIN) {
#pragma unroll
                for (uint32_t sd = 0; sd < 2; ++sd) {
                    const uint32_t f0 = hx->h.out_first[sd], n = hx->h.out_n[sd], b = seg * S;
                    if (b + S > f0 && b < f0 + n) {  // (a face is whole planes: rarely astride a segment)
#pragma unroll
                        for (uint32_t i = 0; i < S; ++i)
                            if (b + i - f0 < n) hx->h.out_dir[sd][b + i - f0] = kDirNone;
                    }
                }
            }
        }
        const uint64_t m = __ballot(act);
        if (act) t.list[t.c + mbcnt64(m)] = seg;
        t.c += (uint32_t)__popcll(m);
        t.base += t.stride;
    }
    if (t.k >= t.c) return false;
    const uint32_t j = t.k + lane / S;
    v = j < t.c ? t.list[j] * S + lane % S : a.hi;
    t.k += PER;
    return true;
}

// Grid-stride over the XCD-aware node range (a z-march walk, each workgroup carrying a tile up
// through the planes so the +-G^2 rows come from L2, read 10% fewer lines but ran 12-20%
// slower: DESIGN.md §8).
// Quiet waves (one GPU, once act_thr actors have converged): a wave of 64 actors that F(r - 1)
// did not mark has only converged actors and receives nothing, so its round is "send nothing":
// its direction bytes become kDirNone and nothing else changes.
// Q: quiet-wave marks allocated (a.act_cur != null); the small graphs run without (Q = false).
// HIN (LM 2, tail rounds only: the host knows from the synced count): the walk writes the halo faces
// itself, the direction byte of every face actor and the messages that cross, so k_shard_halo is not
// launched.
__device__ __forceinline__ void shard_pack_body(const RoundArgs& a, const Xchg& x, long long applied);
// A shard's tail round (k_ps_quiet_x<true>): the workgroup that finishes last packs the round's headers
// (k_shard_pack's work) — every workgroup's counts and entries are released before its arrival is
// counted and acquired by the last one — so the round is one launch fewer.  Every thread calls it.
__device__ __forceinline__ void tail_pack(const RoundArgs& a, const Xchg& x) {
    __shared__ uint32_t last_s;
    // What the pack reads was written with device-scope atomics (the entry and halo counters, the round's
    // sub-counters, the overflow flag); a wave's atomics have been performed once its memory counter is 0,
    // so a workgroup arrives without a device-scope release (an L2 write-back per workgroup: ~1800 of
    // them made the tail round 94.5 -> 155.8 us).  The arrivals go to kFinGroups counters (one XCD's
    // workgroups each), the last of each group to one counter of groups.
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t G = gridDim.x < kFinGroups ? gridDim.x : kFinGroups, g = blockIdx.x % G;
        const uint32_t in_g = (gridDim.x - g + G - 1u) / G;  // workgroups of group g
        uint32_t last = 0u;
        if (atomicAdd(x.fin + (1u + g) * kFinStride, 1u) == in_g - 1u) last = atomicAdd(x.fin, 1u) == G - 1u;
        last_s = last;
    }
    __syncthreads();
    if (!last_s) return;
    __threadfence();
    shard_pack_body(a, x, (long long)a.r);
    if (threadIdx.x <= kFinGroups) x.fin[threadIdx.x * kFinStride] = 0u;  // the next tail round counts from 0
}

template <int LM, bool Q, bool HIN = false>
__device__ __forceinline__ void ps_pull_body(const RoundArgs& a, const Xchg* xp = nullptr) {
    const Geom g = a.g;
    const uint32_t r = a.r;
    uint32_t newly = 0;
    uint32_t v, end, step;
    node_range(a.lo, a.hi, a.span, v, end, step);
    if constexpr (!Q && LM != 2) {
        // Small graphs (one GPU, no quiet waves): the round is one dependent chain of loads with
        // the gate at its head, so the first actor's level-1 loads are issued ahead of the gate's
        // and both wait together (a thread without an actor loads actor lo's and drops them).
        PsLevel1 p = ps_level1<LM, true>(a, g, r, v < end ? v : a.lo);
        const unsigned long long prev = gate_count_wave(a, a.r);
        if (prev >= a.target) return;
        // keep the uses of the level-1 bytes below the gate (hoisted above it, they would wait
        // for the loads before the gate's own loads are even issued)
#pragma unroll
        for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(p.d[k]));
        asm volatile("" : "+v"(p.f));
#pragma unroll
        for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(p.gm6[k].x), "+v"(p.gm6[k].y));
        asm volatile("" : "+v"(p.held.x), "+v"(p.held.y));
        if (v < end) {
            newly += ps_finish<LM, true>(a, g, r, v, p, false);
            for (v += step; v < end; v += step) newly += ps_actor<LM>(a, g, r, v);
        }
        wave_add(newly, a.parts, r);
        return;
    }
    // HIN (a round the host knows to be a tail round): the LDS tables filled and the walk's first marks
    // in flight before the gate, whose barrier serves the tables too
    TailWalk t0{};
    if constexpr (LM == 2 && HIN) {
        peer_tab_fill(*xp);
        halo_tab_fill(*xp);
        t0 = tail_walk(a, true);
    }
    // converged after round r - 1 (one GPU, small graphs: Q = false, the per-wave gate)
    const unsigned long long prev = (Q || LM == 2) ? gate_count(a, a.r) : gate_count_wave(a, a.r);
    if (prev >= a.target) {  // (block-uniform; a tail round's headers still go out)
        if constexpr (LM == 2 && HIN) tail_pack(a, *xp);
        return;
    }
    const bool mark = Q && prev >= a.act_thr;                          // F(r) marks round r + 1
    const bool skip = Q && r >= 2u && a.total[r - 2] >= a.act_thr;  // F(r - 1) marked round r
    const uint8_t tag = (uint8_t)a.tag_cur;  // link_tag(r)
    if constexpr (Q) {
        const bool tail = skip;  // block-uniform: the compacted segment walk of the run's tail
        if constexpr (LM == 2) {
            // a tail round's entries read the peers' chunks and the halo faces from LDS (put_t): a
            // lane's own peer or face indexing the kernel arguments is a vector load per field
            if (tail) {
                if constexpr (!HIN) {
                    peer_tab_fill(*xp);
                    halo_tab_fill(*xp);
                    __syncthreads();
                }
            } else if constexpr (kShardFuse && !HIN) {  // a dense round stages its remote link messages
                peer_tab_fill(*xp);
                fuse_init();
                __syncthreads();
            }
        }
        uint32_t walked = 0;
        if constexpr (LM == 2 && kShardFuse && !HIN) {
            if (!tail) {  // a shard's dense round: its own walk, in block-uniform steps of kFuseIters
                FuseWalk fw;
                for (;;) {
                    if (fw.it == kFuseIters && !fuse_flush(*xp, fw, v < end)) break;
                    fw.it = (uint32_t)__builtin_amdgcn_readfirstlane((int)(fw.it + 1u));  // (uniform: an SGPR)
                    const uint32_t u = v;
                    v += step;
                    if (u < end) {  // (a lane past its range walks nothing until the block's step ends)
                        // the link's slot, loaded beside the actor's own loads (every line of lpos is
                        // read anyway: one actor in seven fires its link)
                        const uint32_t lp = a.lpos[u];
                        LinkSend ls;
                        newly += ps_actor<LM, true, false>(a, g, r, u, mark, &ls);
                        ++walked;
                        if (ls.fired) {  // a local slot's mark, a remote one staged
                            const Xchg& x = *xp;
                            const uint32_t q = owner_t(x.world, lp);
                            if (q == x.rank) a.lref_cur[lp] = a.rtag_cur;
                            else fuse_put(x, fw, q, lp, ls.msg);
                        }
                    }
                }
                block_add(newly, a.parts, r);
                if (a.work) block_add_u64(walked, a.work + (blockIdx.x & (kParts - 1)) * kWorkStride);
                return;
            }
        }
        TailWalk t = HIN ? t0 : tail_walk(a, tail);
        for (;;) {
            uint32_t u;
            if (tail) {
                if (!tail_next<HIN>(a, t, tag, u, xp)) break;
            } else {
                if (v >= end) break;
                u = v;
                v += step;
            }
            LinkSend ls;
            if (u - a.lo < a.hi - a.lo) {  // lo <= u < hi (a shard's edge segments)
                newly += ps_actor<LM, LM == 1 || LM == 2, HIN>(a, g, r, u, mark, LM == 2 ? &ls : nullptr);
                ++walked;
            }
            if constexpr (LM == 2) {
                // A shard's tail round routes its own link messages (k_ps_link_scatter_x skips these
                // rounds): a slot of this rank gets its mark, another rank's an entry of its chunk.
                // HIN: it also writes the halo faces (k_shard_halo's work), the direction byte of every
                // face actor and an entry for each message that crosses.  A message takes one way, so
                // a lane needs at most one position: one reservation per wave and pass, positions
                // reserved per wave (the tail's entries are few).  Wave-uniform here.
                if (tail) {
                    const Xchg& x = *xp;
                    const uint32_t lp = load_sel(a.lpos, ls.fired, u, a.lo);
                    const bool remote = ls.fired && (lp < x.sbnd[x.rank] || lp >= x.sbnd[x.rank + 1]);
                    if (ls.fired && !remote) a.lref_cur[lp] = a.rtag_cur;
                    uint32_t q = remote ? owner(x.sbnd, x.world, lp) : 0u;
                    bool cross = false;
                    uint32_t fo = 0, sd = 0;
                    if constexpr (HIN) {
                        const bool own = u - a.lo < a.hi - a.lo;
#pragma unroll
                        for (uint32_t k = 0; k < 2; ++k) {
                            const uint32_t o = u - x.h.out_first[k];
                            const bool face = own && o < x.h.out_n[k];
                            if (face) x.h.out_dir[k][o] = (uint8_t)ls.dir;
                            if (face && ls.dir == x.h.code[k]) {
                                cross = true;
                                fo = o;
                                sd = k;
                            }
                        }
                        if (cross) q = x.world + sd;
                    }
                    const uint32_t pos = wave_reserve(x, remote || cross, q);
                    if (remote) put_t<true>(x, q, pos, lp, ls.msg);
                    if (cross) {
                        const HaloTab& ht = halo_tab();
                        const uint32_t cap = ht.cap[sd];
                        if (pos < cap) {
                            ht.slot[sd][my_sub() * cap + pos] = fo;
                            ht.msg[sd][my_sub() * cap + pos] = ls.msg;
                        } else {
                            atomicOr(x.overflow, 1u);
                        }
                    }
                }
            }
        }
        block_add(newly, a.parts, r);
        if (a.work) block_add_u64(walked, a.work + (blockIdx.x & (kParts - 1)) * kWorkStride);
        if constexpr (LM == 2 && HIN) tail_pack(a, *xp);
        return;
    }
    for (; v < end; v += step) newly += ps_actor<LM>(a, g, r, v, false);
    block_add(newly, a.parts, r);
}

template <int LM, bool Q>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GP_PS_WAVES))) void k_ps_pull(RoundArgs a) {
    ps_pull_body<LM, Q>(a);
}

// The one-GPU round kernel of large graphs (quiet waves: from 2^20 actors).  Its SGPRs are capped
// (GP_PSQ_SGPR) so that seven 256-thread workgroups fit a CU (106 SGPRs admit six: MI355X
// residency rule 800 / (ceil(sgpr / 16) * 16 + 16)), and it runs on a grid of exactly the
// resident workgroups (quiet_grid): every workgroup of an XCD sweeps its span together.
// C3 -4.0%, 100M -2% against 6 per CU on a 16-per-CU grid (profiles/round3/occupancy_ab).
template <int LM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GP_PSQ_WAVES))) GP_PSQ_SGPR_ATTR void k_ps_quiet(
    RoundArgs a) {
    ps_pull_body<LM, true>(a);
}
// A shard of several ranks (LM 2): the same kernel with the exchange descriptor, so its tail rounds
// route their own link messages (HIN: and write the halo faces).
// <false> (dense rounds, and tail rounds the host cannot yet be sure of) also routes a dense round's
// link messages through LDS (kShardFuse): a second walk loop, which needs more registers than seven
// waves per SIMD leave (80 VGPRs and 106 SGPRs: six workgroups per CU, GP_PSQX_PER_CU).
#ifndef GP_PSQX_PER_CU
#define GP_PSQX_PER_CU (kShardFuse ? 6 : GP_PSQ_PER_CU)
#endif
template <bool HIN>
__global__ void k_ps_quiet_x(RoundArgs a, Xchg x);
template <>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GP_PSQ_WAVES))) GP_PSQ_SGPR_ATTR void k_ps_quiet_x<true>(
    RoundArgs a, Xchg x) {
    ps_pull_body<2, true, true>(a, &x);
}
#if GP_SHARD_FUSE
template <>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(6))) __attribute__((amdgpu_num_sgpr(106))) void
k_ps_quiet_x<false>(RoundArgs a, Xchg x) {
    ps_pull_body<2, true, false>(a, &x);
}
#else
template <>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(GP_PSQ_WAVES))) GP_PSQ_SGPR_ATTR void k_ps_quiet_x<false>(
    RoundArgs a, Xchg x) {
    ps_pull_body<2, true, false>(a, &x);
}
#endif


// ------------------------------------------------------------------ small line grids: rounds in batches
// (TileArgs)  A small grid's round is one latency-bound launch (gate, one load level,
// stores); on a line (line and 2D topologies) one launch runs up to kTileMaxNR rounds of a segment:
// round r + q over the segment and NR - 1 - q actors either side of it, round r from round r - 1's
// state of the segment and NR actors either side (loaded into LDS), each later round from the one
// before in LDS.  The rim is computed by both segments that border it, identically (the same
// arithmetic on the same inputs).  Each segment writes every round's state of its own actors (round
// r + q is the run's state if it converges there: the host then ignores the later rounds, whose
// buffers no reader uses).  100K line: 4.85 us per one-round launch, 9.2 us per four rounds; boxes
// of a 3D grid recompute 2.3-3.4x their actors in the rim and were slower (profiles/round5/tiles/).
// One actor's round from its neighbours' direction bytes and messages in LDS (cell c), in ascending
// source order (slot order), as ps_finish sums them.
__device__ __forceinline__ PsOut tile_actor(const RoundArgs& a, uint32_t r, uint32_t v, uint32_t m, uint32_t c,
                                            const uint8_t* dir, const double2* msg, uint8_t& f, double2 held,
                                            uint32_t& code) {
    code = kth_bit(m, scale_draw(philox_x(v, r, kStreamPush, a.seed), popc(m)));
    double ss = 0.0, ww = 0.0;
    uint32_t cin = 0;
    if (r) {
        // a line's slots: v - 1 (slot 2, code 1), v + 1 (slot 3, code 0)
        if ((m & 1u) && dir[c - 1u] == 1u) {
            const double2 mm = msg[c - 1u];
            ss += mm.x;
            ww += mm.y;
            ++cin;
        }
        if ((m & 2u) && dir[c + 1u] == 0u) {
            const double2 mm = msg[c + 1u];
            ss += mm.x;
            ww += mm.y;
            ++cin;
        }
    } else {
        held = make_double2((double)v, 1.0);
    }
    return ps_update(f, held, ss, ww, cin, a.delta, a.term_limit);
}

template <int NR>
__global__ __launch_bounds__(kBlock) void k_ps_tile(RoundArgs a, TileArgs t) {
    static_assert(NR >= 1 && NR <= (int)kTileMaxNR && kTileLoad <= kBlock, "one load per thread");
    __shared__ double2 s_msg[2][kTileLoad];
    __shared__ uint8_t s_dir[2][kTileLoad], s_flg[2][kTileLoad];
    __shared__ unsigned long long prev_s;
    __shared__ uint32_t red[NR][kBlock / 64];  // each round's newly converged actors per wave
    const uint32_t r = a.r, n = a.g.actors;
    // this segment [s0, s1); cells: actors s0 - NR .. s1 + NR - 1 (those on the line)
    const uint32_t s0 = blockIdx.x * kTileSeg, s1 = min(s0 + kTileSeg, n);
    const uint32_t c0 = s0 >= (uint32_t)NR ? s0 - NR : 0u, c1 = min(s1 + NR, n);
    const uint32_t i = threadIdx.x, v = c0 + i;
    // the loads go out before the gate resolves (latency-bound rounds, as k_ps_pull's PRE)
    {
        const uint32_t pin = (r + kTileBufs - 1u) % kTileBufs;  // round r - 1's state
        const bool in = v < c1;
        const uint32_t vv = in ? v : c0;  // (unconditional loads; round 0 reads no neighbour)
        const uint8_t d = t.dir[pin][vv], f = t.flg[pin][vv];
        const double2 mm = t.msg[pin][vv];
        if (i < kTileLoad) {
            s_dir[0][i] = in ? d : (uint8_t)kDirNone;
            s_flg[0][i] = f;
            s_msg[0][i] = mm;
        }
    }
    // completion counts after rounds r - kTileMaxNR .. r - 1 (the last launch's rounds, up to
    // kTileMaxNR of them, have no total yet): block 0 writes them
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        unsigned long long x = r > kTileMaxNR ? a.total[r - kTileMaxNR - 1u] : 0ull;
#pragma unroll
        for (uint32_t q = kTileMaxNR; q >= 1u; --q) {
            if (r >= q) {
                x += wave_sum(*part_slot(a.parts, (long long)r - q, lane));
                if (blockIdx.x == 0 && lane == 0) a.total[r - q] = x;
            }
        }
        if (lane == 0) prev_s = x;
        if (blockIdx.x == 0)  // the next launch's sub-counters (ring: kPartRing >= 3 kTileMaxNR)
            for (uint32_t q = 0; q < kTileMaxNR; ++q) *part_slot(a.parts, (long long)r + NR + q, lane) = 0u;
    }
    __syncthreads();
    // The gate is checked once per launch: rounds past the target inside this launch still run and
    // write their buffers, flags and frozen values.  That is exact only because the target is EVERY
    // participating actor (push-sum: T = nodes, program.fs:178; a line / 2D grid has no inert actor but
    // the isolated last one): once all have converged no actor sets conv_now again, so no flag or frozen
    // value changes, and the host reads the state of the converged round's buffer.  A smaller target
    // would need the per-round gate on the running count (gp_api.cpp enables tiles for push-sum line /
    // 2D grids only).
    if (prev_s >= a.target) return;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        // round r + q over the segment and NR - 1 - q actors either side, from LDS side q & 1
        const uint32_t rq = r + (uint32_t)q, w = (uint32_t)(NR - 1 - q), in = (uint32_t)q & 1u, out = in ^ 1u;
        const uint32_t lo = s0 >= w ? s0 - w : 0u, hi = min(s1 + w, n);
        uint32_t newly = 0;
        if (v >= lo && v < hi) {
            const uint32_t m = presence(a.g, v);
            uint8_t f = s_flg[in][i];
            uint32_t code = kDirNone;
            PsOut o{};
            if (m) o = tile_actor(a, rq, v, m, i, s_dir[in], s_msg[in], f, s_msg[in][i], code);
            const uint8_t d = m && o.send ? (uint8_t)code : (uint8_t)kDirNone;
            if (m && v >= s0 && v < s1) {
                const uint32_t pq = rq % kTileBufs;
                if (o.send) t.msg[pq][v] = o.msg;
                t.dir[pq][v] = d;
                t.flg[pq][v] = f;
                if (o.conv_now) a.frozen[v] = o.msg;
                newly = o.conv_now ? 1u : 0u;
            }
            if (q + 1 < NR) {
                s_dir[out][i] = d;
                s_flg[out][i] = f;
                s_msg[out][i] = o.msg;
            }
        }
        newly = wave_sum(newly);
        if ((threadIdx.x & 63u) == 0) red[q][threadIdx.x >> 6] = newly;
        __syncthreads();  // round r + q in LDS
    }
    if (threadIdx.x < (uint32_t)NR) {  // one add per round and block (the counts of F, block_add's)
        uint32_t c = 0;
#pragma unroll
        for (uint32_t w = 0; w < kBlock / 64; ++w) c += red[threadIdx.x][w];
        if (c) atomicAdd(part_slot(a.parts, (long long)r + threadIdx.x, blockIdx.x & (kParts - 1)), c);
    }
}

// ------------------------------------------------------------------ gossip, grid topologies
// dir byte = chain-0 code | chain-1 code << 4 (15 = no chain)
__device__ __forceinline__ uint32_t nib_match(uint8_t b, uint32_t code) {
    return (uint32_t)((b & 15u) == code) + (uint32_t)((b >> 4) == code);
}

// One actor's loads that do not depend on other loads (state byte, receipt counter, the six
// neighbours' direction bytes, the CSR range).  PRE (small graphs): issued together, before the
// gate resolves, for every actor; otherwise gs_actor loads them lazily (a done actor reads no
// direction bytes; the counter only when something arrived).
struct GsLevel1 {
    uint32_t m, st, c0, li, nl;
    uint32_t d[6];  // one register per byte: packing them would wait for the loads
};

template <bool LINK>
__device__ __forceinline__ GsLevel1 gs_level1(const RoundArgs& a, const Geom& g, uint32_t v) {
    GsLevel1 p;
    p.m = presence(g, v);
    p.st = a.gstate[v];
    p.c0 = a.cnt[v];
#pragma unroll
    for (uint32_t k = 0; k < 6; ++k) p.d[k] = load_sel(a.dir_prev, (p.m & slot_bit(k)) != 0u, slot_src(g, v, k), v);
    p.li = 0;
    p.nl = 0;
    if (LINK) {
        p.li = a.rev_off[v];
        p.nl = a.rev_off[v + 1] - p.li;
    }
    return p;
}

// F(r) for one actor: apply round r-1's receipts (program.fs:92-105), emit round r (:89-95).
template <bool LINK, bool PRE>
__device__ __forceinline__ uint32_t gs_actor(const RoundArgs& a, const Geom& g, uint32_t r, uint32_t v,
                                             const GsLevel1& p) {
    const uint32_t m = PRE ? p.m : presence(g, v);
    if (!m) return 0;
    const uint8_t st = PRE ? (uint8_t)p.st : a.gstate[v];
    uint32_t tok = st & 3u;
    uint32_t done = (st >> 2) & 1u;
    uint32_t newly = 0;
    if (r && !done) {  // apply round r-1: receipts while not done at round start (program.fs:92)
        uint32_t d[6];
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k)
            d[k] = PRE ? p.d[k] : load_sel(a.dir_prev, (m & slot_bit(k)) != 0u, slot_src(g, v, k), v);
        uint32_t inc = 0;
#pragma unroll
        for (uint32_t k = 0; k < 6; ++k) inc += (m & slot_bit(k)) ? nib_match((uint8_t)d[k], slot_code(k)) : 0u;
        if (LINK) {
            const uint32_t li = PRE ? p.li : a.rev_off[v], nl = PRE ? p.nl : a.rev_off[v + 1] - li;
            uint8_t lc[kLinkUnroll];
#pragma unroll
            for (uint32_t k = 0; k < kLinkUnroll; ++k) lc[k] = load_sel(a.lcnt_prev, k < nl, li + k, a.slot_lo);
#pragma unroll
            for (uint32_t k = 0; k < kLinkUnroll; ++k)
                if (k < nl && lc[k]) {
                    inc += lc[k];
                    a.lcnt_prev[li + k] = 0;
                }
            for (uint32_t k = kLinkUnroll; k < nl; ++k) {
                const uint8_t c = a.lcnt_prev[li + k];
                if (c) {
                    inc += c;
                    a.lcnt_prev[li + k] = 0;
                }
            }
        }
        if (inc) {
            const uint32_t c0 = PRE ? p.c0 : a.cnt[v], c1 = c0 + inc;
            a.cnt[v] = c1;
            if (c0 == 0) ++tok;                                  // program.fs:99-100
            if (c0 <= a.threshold && c1 > a.threshold) {         // program.fs:102-104
                done = 1;
                newly = 1;
            }
            a.gstate[v] = (uint8_t)(tok | (done << 2));
        }
    }
    if (tok) {  // emit round r: one draw per activation chain (program.fs:89-95)
        const uint4 x = philox(v, r, kStreamGossip, a.seed);
        const uint32_t n = popc(m);
        const uint32_t c0 = kth_bit(m, scale_draw(x.x, n));
        const uint32_t c1 = tok > 1 ? kth_bit(m, scale_draw(x.y, n)) : 15u;
        a.dir_cur[v] = (uint8_t)(c0 | (c1 << 4));
    }
    return newly;
}

// EARLY (graphs below 2^18 actors, one GPU): the round is one dependent chain with the gate at
// its head, so the first actor's level-1 loads go out ahead of the gate's (as k_ps_pull does).
template <bool LINK, bool EARLY>
__global__ __launch_bounds__(kBlock) void k_gs_pull(RoundArgs a) {
    const Geom g = a.g;
    const uint32_t r = a.r;
    uint32_t v, end, step;
    node_range(a.lo, a.hi, a.span, v, end, step);
    uint32_t newly = 0;
    if constexpr (EARLY) {
        GsLevel1 p = gs_level1<LINK>(a, g, v < end ? v : a.lo);
        if (r && gate_count_wave(a, (long long)r - 1) >= a.target) return;
        // keep the uses of the loaded bytes below the gate (see k_ps_pull)
        asm volatile("" : "+v"(p.st), "+v"(p.c0));
#pragma unroll
        for (int k = 0; k < 6; ++k) asm volatile("" : "+v"(p.d[k]));
        if (v < end) {
            newly += gs_actor<LINK, true>(a, g, r, v, p);
            for (v += step; v < end; v += step) newly += gs_actor<LINK, true>(a, g, r, v, gs_level1<LINK>(a, g, v));
        }
        if (r) wave_add(newly, a.parts, (long long)r - 1);
    } else {
        if (r && gate(a, (long long)r - 1)) return;
        const GsLevel1 none{};
        for (; v < end; v += step) newly += gs_actor<LINK, false>(a, g, r, v, none);
        if (r) block_add(newly, a.parts, (long long)r - 1);
    }
}

// ------------------------------------------------------------------ link count pass
// After F(r): every actor whose round-r message(s) took its extra link (direction code 6;
// gossip: per activation chain) writes the count (1 or 2) into its CSR slot lpos[u], a byte
// the receiver reads — coalesced, in CSR order — in F(r+1) and empties.  Only the ~1/7 of
// senders that fired touch a random address; the receiver then reads a push-sum message
// straight from the sender's row (msg_prev[u]).  A separate pass so the round kernel's loads
// never wait behind scattered stores (vmcnt counts stores on CDNA).  Four actors per thread
// (block-strided, so every load instruction stays coalesced): their direction codes, then the
// slot indices in flight together, then the scattered stores.
constexpr uint32_t kScatterPer = 4;

// Past convergence when the round before the one F(r) applied already reached the target:
// F(r) applies round r (push-sum) or r - 1 (gossip) and publishes the count before it.
__device__ __forceinline__ bool applied_converged(const RoundArgs& a) {
    const long long ap = a.ps_tags ? (long long)a.r : (long long)a.r - 1;
    return ap >= 1 && a.total[ap - 1] >= a.target;
}

__global__ __launch_bounds__(kBlock) void k_link_count(RoundArgs a) {
    if (applied_converged(a)) return;
    const uint32_t n = a.g.wired;
    const uint32_t base = blockIdx.x * kBlock * kScatterPer + threadIdx.x;
    uint32_t nl[kScatterPer], lp[kScatterPer];
#pragma unroll
    for (uint32_t j = 0; j < kScatterPer; ++j) {
        const uint32_t u = base + j * kBlock;
        const uint8_t b = load_sel(a.dir_cur, u < n, u, 0u);
        nl[j] = u < n ? (uint32_t)((b & 15u) == kDirLink) + (uint32_t)((b >> 4) == kDirLink) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kScatterPer; ++j) lp[j] = load_sel(a.lpos, nl[j] != 0u, base + j * kBlock, 0u);
#pragma unroll
    for (uint32_t j = 0; j < kScatterPer; ++j)
        if (nl[j]) a.lcnt_cur[lp[j]] = (uint8_t)(a.ps_tags ? a.tag_cur : nl[j]);
}

// ------------------------------------------------------------------ full gossip's lists (GsSparse)
__device__ __forceinline__ uint32_t* sp_ctr(const GsSparse& sp, uint32_t field, uint32_t r) {
    return sp.ctr + (field * 4u + (r & 3u)) * kSpStride;
}
// Append val to list (a wave's wanting lanes, one atomic per wave); every active lane of the wave calls it.
__device__ __forceinline__ void wave_append(bool want, uint32_t val, uint32_t* list, uint32_t* ctr, uint32_t cap,
                                            uint32_t* err) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const uint32_t lead = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if ((threadIdx.x & 63u) == lead) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = (uint32_t)__shfl((int)base, (int)lead, 64);
    const uint32_t pos = base + mbcnt64(m);
    if (want) {
        if (pos < cap) list[pos] = val;
        else atomicOr(err, 1u);
    }
}
// Two appends at once (the wave's first active lane issues both counters' atomics, then one wait).
__device__ __forceinline__ void wave_append2(bool w1, uint32_t v1, uint32_t* l1, uint32_t* c1, uint32_t cap1, bool w2,
                                             uint32_t v2, uint32_t* l2, uint32_t* c2, uint32_t cap2, uint32_t* err) {
    const uint64_t m1 = __ballot(w1), m2 = __ballot(w2);
    if (!(m1 | m2)) return;
    const uint32_t lead = (uint32_t)__builtin_ctzll(__ballot(true));
    uint32_t b1 = 0, b2 = 0;
    if ((threadIdx.x & 63u) == lead) {
        if (m1) b1 = atomicAdd(c1, (uint32_t)__popcll(m1));
        if (m2) b2 = atomicAdd(c2, (uint32_t)__popcll(m2));
    }
    b1 = (uint32_t)__shfl((int)b1, (int)lead, 64) + mbcnt64(m1);
    b2 = (uint32_t)__shfl((int)b2, (int)lead, 64) + mbcnt64(m2);
    if (w1) {
        if (b1 < cap1) l1[b1] = v1;
        else atomicOr(err, 1u);
    }
    if (w2) {
        if (b2 < cap2) l2[b2] = v2;
        else atomicOr(err, 1u);
    }
}

// ------------------------------------------------------------------ shard exchange



// Positions of K entries per thread in their peers' chunks, reserved per BLOCK: LDS counters per
// peer, then one global atomic per (block, peer) on the block's sub-segment counter.  At 8 ranks
// ~7/8 of the link messages are remote: per-wave reservation on one counter per peer cost 8.5 ms
// per round (8 loopback shards of 80M actors).  Every thread of the block must call it.
template <uint32_t K>
__device__ __forceinline__ void block_reserve(const Xchg& x, const bool (&want)[K], const uint32_t (&q)[K],
                                              uint32_t (&pos)[K], uint32_t sub = kSub) {
    if (sub >= kSub) sub = my_sub();
    __shared__ uint32_t cnt[kMaxWorld], base[kMaxWorld];
    if (threadIdx.x < kMaxWorld) cnt[threadIdx.x] = 0u;
    peer_tab_fill(x);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) pos[j] = want[j] ? atomicAdd(&cnt[q[j]], 1u) : 0u;
    __syncthreads();
    if (threadIdx.x < x.world && cnt[threadIdx.x])
        base[threadIdx.x] = atomicAdd(ctr_at(x, threadIdx.x, sub), cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < K; ++j)
        if (want[j]) pos[j] += base[q[j]];
}


// Actors per thread of the sharded link passes (block-strided): more per block means fewer
// block-level reservations (three barriers and one global atomic per peer each).
#ifndef GP_SHARD_PER
#define GP_SHARD_PER 4  // (C5 / 8 link scatter: 4 0.61 ms, 8 0.63, 16 0.96; profiles/round6/put_ab/)
#endif
constexpr uint32_t kShardPer = GP_SHARD_PER;

// Sharded push-sum link pass: a link message whose CSR slot is this rank's gets the slot's round tag
// (the receiver reads msg_prev[u] itself, as on one GPU); one whose slot belongs to another rank goes
// to that rank's send chunk as (global slot, s, w), and the receiver's unpack points the slot at it.
__global__ __launch_bounds__(kBlock) void k_ps_link_scatter_x(RoundArgs a, Xchg x) {
    if (applied_converged(a)) return;  // block-uniform: F(r) was a no-op
    const uint32_t n = a.hi < a.g.wired ? a.hi : a.g.wired;
    const uint32_t base = a.lo + blockIdx.x * kBlock * kShardPer + threadIdx.x;
    // Quiet-tail rounds (F(r) walked the marked segments only): the round kernel routed its own
    // link messages (k_ps_quiet_x); this pass, latency-bound over every actor, would cost 33-40 us
    // per rank-round at 100M / 8 for the few that moved.
    if (a.act_prev && a.r >= 2u && a.total[a.r - 2u] >= a.act_thr) return;
    const uint32_t slo = x.sbnd[x.rank], shi = x.sbnd[x.rank + 1];
    bool l[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) {
        const uint32_t u = base + j * kBlock;
        l[j] = u < n && load_sel(a.dir_cur, u < n, u, a.lo) == kDirLink;
    }
    uint32_t lp[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) lp[j] = load_sel(a.lpos, l[j], base + j * kBlock, a.lo);
    // only a remote link needs its message: the fired ~1/7 of senders would otherwise pull in
    // ~70% of msg_cur's lines (8 messages per 128 B line)
    bool rm[kShardPer];
    double2 mm[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) {
        rm[j] = l[j] && (lp[j] < slo || lp[j] >= shi);
        mm[j] = load_sel(a.msg_cur, rm[j], base + j * kBlock, a.lo);
    }
    uint32_t q[kShardPer], pos[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) {
        if (l[j] && !rm[j]) a.lref_cur[lp[j]] = a.rtag_cur;
        q[j] = rm[j] ? owner(x.sbnd, x.world, lp[j]) : 0u;
    }
    block_reserve(x, rm, q, pos);
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j)
        if (rm[j]) put_t<true>(x, q[j], pos[j], lp[j], mm[j]);
}

__global__ __launch_bounds__(kBlock) void k_gs_link_scatter_x(RoundArgs a, Xchg x) {
    if (applied_converged(a)) return;  // block-uniform
    const uint32_t n = a.hi < a.g.wired ? a.hi : a.g.wired;
    const uint32_t base = a.lo + blockIdx.x * kBlock * kShardPer + threadIdx.x;
    const uint32_t slo = x.sbnd[x.rank], shi = x.sbnd[x.rank + 1];
    uint32_t nl[kShardPer], lp[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) {
        const uint32_t u = base + j * kBlock;
        const uint8_t b = load_sel(a.dir_cur, u < n, u, a.lo);
        nl[j] = u < n ? (uint32_t)((b & 15u) == kDirLink) + (uint32_t)((b >> 4) == kDirLink) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) lp[j] = load_sel(a.lpos, nl[j] != 0u, base + j * kBlock, a.lo);
    bool rm[kShardPer];
    uint32_t q[kShardPer], pos[kShardPer];
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j) {
        rm[j] = nl[j] && (lp[j] < slo || lp[j] >= shi);
        if (nl[j] && !rm[j]) a.lcnt_cur[lp[j]] = (uint8_t)nl[j];
        q[j] = rm[j] ? owner(x.sbnd, x.world, lp[j]) : 0u;
    }
    block_reserve(x, rm, q, pos);
#pragma unroll
    for (uint32_t j = 0; j < kShardPer; ++j)
        if (rm[j]) put_t<false>(x, q[j], pos[j], lp[j] | ((nl[j] - 1u) << 31), make_double2(0.0, 0.0));
}

// Halo faces of F(k), after the round kernel: the direction bytes of this rank's first plane go
// to rank-1 and of its last plane to rank+1 (coalesced copies), and of the push-sum messages only
// those that cross the face (about 1/7 of the plane) as (face offset, s, w) entries.  The
// receiver's halo rows keep stale messages elsewhere; its pull kernel reads a halo message only
// when the direction byte points across, so they are never read.
// Block-aggregated position on one counter (LDS first, then one global atomic per block).
// Every thread of the block must call it.
__device__ __forceinline__ uint32_t block_reserve1(uint32_t* ctr, bool want) {
    __shared__ uint32_t cnt, base;
    if (threadIdx.x == 0) cnt = 0u;
    __syncthreads();
    uint32_t pos = want ? atomicAdd(&cnt, 1u) : 0u;
    __syncthreads();
    if (threadIdx.x == 0 && cnt) base = atomicAdd(ctr, cnt);
    __syncthreads();
    return pos + (want ? base : 0u);
}

__global__ __launch_bounds__(kBlock) void k_shard_halo(RoundArgs a, Xchg x, int pushsum) {
    if (applied_converged(a)) return;  // block-uniform; the chunks' headers still go out (pack)
    for (int side = 0; side < 2; ++side) {
        const uint32_t n = x.h.out_n[side];
        const uint32_t first = x.h.out_first[side], code = x.h.code[side], cap = x.h.out_cap[side];
        uint8_t* odir = x.h.out_dir[side];
        uint32_t* oslot = x.h.out_slot[side];
        double2* omsg = x.h.out_msg[side];
        uint32_t* ctr = ctr_at(x, x.world + side, my_sub());
        const uint32_t seg = my_sub() * cap;
        // block-uniform trip count: every lane of a wave reaches reserve1
        for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
            const uint32_t i = base + threadIdx.x;
            const bool valid = i < n;
            const uint8_t b = load_sel(a.dir_cur, valid, first + i, first);
            if (valid) odir[i] = b;
            const bool cross = pushsum && valid && b == code;
            double2 m = make_double2(0.0, 0.0);
            if (pushsum) m = load_sel(a.msg_cur, cross, first + i, first);  // gossip: no msg array
            const uint32_t pos = block_reserve1(ctr, cross);
            if (cross) {
                if (pos < cap) {
                    oslot[seg + pos] = i;
                    omsg[seg + pos] = m;
                } else {
                    atomicOr(x.overflow, 1u);
                }
            }
        }
    }
}

// Round `applied`'s count into every send header; the entry counters restart at 0.  One block
// of kMaxWorld x kSub threads: thread (q, s) handles sub-segment s of peer q, all at once.
static_assert(kMaxWorld * kSub == kBlock, "k_shard_pack maps one thread per (peer, sub-segment)");

__device__ __forceinline__ void shard_pack_body(const RoundArgs& a, const Xchg& x, long long applied) {
    __shared__ unsigned long long newly_s, chains_s;
    __shared__ uint32_t of_s[kMaxWorld], max_s[kMaxWorld], last_s[kMaxWorld], dirty_s;
    if (threadIdx.x < 64) {
        unsigned long long newly = 0, chains = 0;
        if (applied >= 0) newly = *part_slot(a.parts, applied, threadIdx.x);
        if (a.cparts) chains = *part_slot(a.cparts, a.r, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            newly += __shfl_xor(newly, off, 64);
            chains += __shfl_xor(chains, off, 64);
        }
        if (threadIdx.x == 0) {
            // the round's count travels with its last piece (the round kernel's pieces all add into
            // the same sub-counters)
            if (x.last) *x.self_newly = newly;
            newly_s = x.last ? newly : 0ull;
            chains_s = chains;
            if (x.self_chains) *x.self_chains = chains;
            dirty_s = 0u;
            if (x.dstat) {  // full gossip: the round's dirty done words (k_shard_done_out); the counter restarts
                dirty_s = x.dstat[kDstatCount];
                x.dstat[kDstatCount] = 0u;
            }
        }
    }
    if (threadIdx.x < kMaxWorld) {
        of_s[threadIdx.x] = 0u;
        max_s[threadIdx.x] = 0u;
        last_s[threadIdx.x] = 0u;
    }
    __syncthreads();
    const uint32_t q = threadIdx.x / kSub, s = threadIdx.x % kSub;
    const bool peer = q < x.world && q != x.rank;
    ShardHeader* hd = peer ? x.out[q].hdr : nullptr;
    if (peer) {
        uint32_t* lc = ctr_at(x, q, s);
        const uint32_t c = *lc;
        hd->nlinks[s] = c < x.out[q].cap ? c : x.out[q].cap;
        atomicMax(&max_s[q], c);
        atomicMax(&last_s[q], hd->nlinks[s]);
        bool of = c > x.out[q].cap;
        *lc = 0u;
        const int side = q + 1 == x.rank ? 0 : q == x.rank + 1 ? 1 : -1;
        uint32_t nh = 0;
        if (side >= 0) {
            uint32_t* hc = ctr_at(x, x.world + side, s);
            const uint32_t n = *hc;
            nh = n < x.h.out_cap[side] ? n : x.h.out_cap[side];
            of = of || n > x.h.out_cap[side];
            *hc = 0u;
        }
        hd->nhalo[s] = nh;
        if (of) atomicOr(&of_s[q], 1u);
    }
    __syncthreads();
    if (peer && s == 0) {
        hd->newly = newly_s;
        hd->overflow = (of_s[q] || *x.overflow) ? 1u : 0u;
        const uint32_t m = max_s[q] > x.pmax[q] ? max_s[q] : x.pmax[q];  // one writer per peer
        x.pmax[q] = m;
        hd->runmax = m;
        hd->chains = (uint32_t)chains_s;
        hd->binned = x.binned;
        // the done part: pairs written (capped), or whether the whole words were written
        const uint32_t dp = x.out[q].dpairs;
        hd->ndone = !x.out[q].done ? 0u : dp ? (dirty_s < dp ? dirty_s : dp) : (dirty_s ? 1u : 0u);
        hd->dwant = dirty_s;
        if (x.pstat) x.pstat[kPsOut + q] = last_s[q];
    }
    if (threadIdx.x == 0 && x.dstat) {
        // words left dirty past the pair capacity go out in a later round
        bool left = false;
        for (uint32_t p = 0; p < x.world; ++p)
            if (p != x.rank && x.out[p].done && x.out[p].dpairs && dirty_s > x.out[p].dpairs) left = true;
        x.dstat[kDstatLeft] = left ? 1u : 0u;
        x.pstat[kPsDirty] = dirty_s;
    }
}

__global__ __launch_bounds__(kBlock) void k_shard_pack(RoundArgs a, Xchg x, long long applied) {
    shard_pack_body(a, x, applied);
}

// total[applied] = total[applied-1] + every rank's count; the received link entries land in
// their CSR slots (push-sum (s,w) / gossip chain count) or, for "full" gossip, as receipts.
// The used entries of a chunk's kSub sub-segments (`cap` entries each, the first count[sb] used)
// as one index range [0, total): the counts are read once, together, and an index is mapped to its
// entry with 15 compares (a walk over every sub-segment's capacity visits mostly unused entries in
// a quiet round; one loop per sub-segment waits on each count in turn).
struct SubWalk {
    uint32_t pre[kSub], cap, total;
    __device__ __forceinline__ SubWalk(const uint32_t* count, uint32_t c) : cap(c) {
        uint32_t n[kSub];
#pragma unroll
        for (uint32_t sb = 0; sb < kSub; ++sb) n[sb] = count[sb];
        uint32_t t = 0;
#pragma unroll
        for (uint32_t sb = 0; sb < kSub; ++sb) {
            pre[sb] = t;
            t += n[sb] < c ? n[sb] : c;  // a count past the capacity overflowed: those entries were not written
        }
        total = t;
    }
    __device__ __forceinline__ uint32_t at(uint32_t v) const {
        uint32_t sb = 0, base = 0;
#pragma unroll
        for (uint32_t k = 1; k < kSub; ++k)
            if (v >= pre[k]) {
                sb = k;
                base = pre[k];
            }
        return sb * cap + (v - base);
    }
};

__global__ __launch_bounds__(kBlock) void k_shard_unpack(RoundArgs a, Xchg x, long long applied, int gossip,
                                                          int full, GsSparse sp) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && applied >= 0) {
        unsigned long long t = *x.self_newly;
        uint32_t of = 0;
        for (uint32_t q = 0; q < x.world; ++q)
            if (q != x.rank) {
                t += x.in[q].hdr->newly;
                of |= x.in[q].hdr->overflow;
            }
        // every piece's headers carry the senders' overflow flags; the last one the round's counts
        if (x.last) a.total[applied] = (applied >= 1 ? a.total[applied - 1] : 0ull) + t;
        if (of) atomicOr(x.overflow, 1u);
    }
    if (x.pstat && blockIdx.x == 0 && threadIdx.x < x.world) {  // full gossip: the next plans' inputs
        const uint32_t q = threadIdx.x;
        if (q == 0) {  // every rank's chains of the round
            unsigned long long c = *x.self_chains;
            for (uint32_t p = 0; p < x.world; ++p)
                if (p != x.rank) c += x.in[p].hdr->chains;
            *reinterpret_cast<unsigned long long*>(x.pstat + kPsChains) = c;
        }
        if (q != x.rank) {  // the largest sub-segment peer q sent and its dirty done words
            uint32_t m = 0;
            for (uint32_t s = 0; s < kSub; ++s) m = max(m, x.in[q].hdr->nlinks[s]);
            x.pstat[kPsIn + q] = m;
            x.pstat[kPsDwIn + q] = x.in[q].hdr->dwant;
        }
    }
    // Quiet-tail marks (push-sum): when F(applied) marked the segments with work in
    // the next round (the count after the round before it reached act_thr), the segment of every
    // actor of this rank that a remote message reaches is marked here, with F(applied)'s tag.
    const bool mark = !gossip && a.act_cur != nullptr && applied >= 0 &&
                      (applied >= 1 ? a.total[applied - 1] : 0ull) >= (unsigned long long)a.act_thr;
    const uint8_t mtag = (uint8_t)link_tag((uint32_t)applied + 1u);
    // halo faces: direction bytes of the neighbour's face plane, then its crossing messages
    const uint32_t gtid = blockIdx.x * kBlock + threadIdx.x, gstride = gridDim.x * kBlock;
    for (int side = 0; side < 2; ++side) {
        const uint32_t n = x.h.in_n[side], first = x.h.in_first[side];
        if (!n) continue;
        const uint8_t* idir = x.h.in_dir[side];
        for (uint32_t i = gtid; i < n; i += gstride) a.dir_cur[first + i] = idir[i];
        if (!x.h.in_slot[side]) continue;
        const uint32_t cap = x.h.in_cap[side];
        if (gtid >= kSub * cap) continue;  // no entry for this thread (a tail round's chunks are small)
        const SubWalk w(x.h.in_hdr[side]->nhalo, cap);
        for (uint32_t v = gtid; v < w.total; v += gstride) {
            const uint32_t i = w.at(v);
            const uint32_t o = x.h.in_slot[side][i];
            if (o >= n) {
                atomicOr(x.overflow, 2u);
                continue;
            }
            a.msg_cur[first + o] = x.h.in_msg[side][i];
            // the message crosses the face toward this rank (code[side] is the outgoing one)
            if (mark) a.act_cur[dir_target(a.g, first + o, x.h.code[side] ^ 1u, 0u) >> kActShift] = mtag;
        }
    }
    // full gossip: the other ranks' done words into this rank's replica of the bitmap (a word of q's
    // range that also holds a neighbour's actors, the first and the last, is merged with an atomic OR)
    if (full && gossip && a.dbits && applied >= 0) {
        for (uint32_t q = 0; q < x.world; ++q) {
            // a peer whose words all match what it shipped before sent none (ndone 0: k_shard_done_out
            // skips such a round)
            if (q == x.rank || !x.in[q].done) continue;
            const uint32_t nd = x.in[q].hdr->ndone;
            if (!nd) continue;
            const uint32_t w0 = x.abnd[q] >> 5, nw = ((x.abnd[q + 1] - 1u) >> 5) - w0 + 1u;
            const uint32_t dp = x.in[q].dpairs, n = dp ? (nd < dp ? nd : dp) : nw;
            for (uint32_t i = gtid; i < n; i += gstride) {
                uint32_t w = w0 + i, val;
                if (dp) {  // (global word index, word) pairs
                    const uint2 pr = reinterpret_cast<const uint2*>(x.in[q].done)[i];
                    w = pr.x;
                    val = pr.y;
                    if (w - w0 >= nw) {  // a corrupt chunk: reported, never written
                        atomicOr(x.overflow, 2u);
                        continue;
                    }
                } else {
                    val = x.in[q].done[i];
                }
                const uint32_t old = a.dbits[w];
                if ((old | val) == old) continue;  // nothing new (most words, most rounds)
                uint32_t now = val;
                if (w == w0 || w + 1 == w0 + nw) now = atomicOr(&a.dbits[w], val) | val;
                else a.dbits[w] = val;
                // the summary bit of a word that just filled (one atomic per such word, not per round)
                if (a.dsum && now == ~0u) atomicOr(&a.dsum[w >> 5], 1u << (w & 31u));
            }
        }
    }
    // an entry outside this rank's actors / slots can only come from a corrupt chunk: it is
    // reported (GP_EOVERFLOW at the next sync), never written
    const uint32_t elo = full ? a.lo : x.sbnd[x.rank], ehi = full ? a.hi : x.sbnd[x.rank + 1];
    // the grid is world x bpp blocks: block b serves peer b / bpp, so the peers' entries are in
    // flight together (one peer after another left each thread a chain of dependent loads per peer)
    const uint32_t bpp = gridDim.x / x.world;
    const uint32_t q = blockIdx.x / bpp;
    if (q < x.world && q != x.rank && x.in[q].cap && (blockIdx.x % bpp) * kBlock + threadIdx.x < kSub * x.in[q].cap &&
        !(full && x.in[q].hdr->binned)) {  // (binned receipts: k_shard_unpack_bins)
        const PeerIn& in = x.in[q];
        // kSub sub-segments of `cap` entries, each walked up to its count only (a chunk sized for an
        // all-sending round holds a few entries in most rounds)
        const SubWalk w(in.hdr->nlinks, in.cap);
        for (uint32_t v = (blockIdx.x % bpp) * kBlock + threadIdx.x; v < w.total; v += bpp * kBlock) {
            const uint32_t i = w.at(v);
            const uint32_t e = in.slot[i];
            const uint32_t t = (gossip && !full) ? e & 0x7FFFFFFFu : e;
            if (t < elo || t >= ehi) {
                atomicOr(x.overflow, 2u);
                continue;
            }
            if (full) {  // a receipt for a done actor is dropped (program.fs:92; exact: the state after
                         // F(applied), which F(applied + 1) filters with)
                if (!sp.hl) {
                    if (!(a.dbits && ((a.dbits[t >> 5] >> (t & 31u)) & 1u))) atomicAdd(&a.inc_cur[t], 1u);
                } else {  // the round ran on lists: every receipt lists its target for F(r + 1), which
                          // drops the receipts of a done actor itself (k_gs_sparse_x / gs_apply4), as
                          // the list rounds' local receipts are dropped: no bitmap read on the way
                    atomicAdd(&a.inc_cur[t], 1u);
                    wave_append(true, t, sp.tl[a.r & 1u], sp_ctr(sp, 2, a.r), 2u * sp.cap + kSpSlack, sp.err);
                }
            }
            else if (gossip) a.lcnt_cur[t] = (uint8_t)((e >> 31) + 1u);
            else {  // the slot points at the message where it arrived: one 4-byte store per entry (the
                    // message and a mark were two scattered stores, 16 + 1 bytes: 0.6 + 0.2 ms of a 0.9 ms
                    // unpack at C5 / 8, profiles/round5/unpack_write_ab/)
                const uint32_t at = (uint32_t)((reinterpret_cast<const char*>(in.msg + i) - x.rbase) >> 4);
                a.lref_cur[t] = a.rtag_cur | (at << kRefShift);
                if (mark) a.act_cur[x.slot_dst[t] >> kActShift] = mtag;  // the receiver owning slot t
            }
        }
    }
}

// hist[(src piece * nd + dst rank) * 8 + degree] over every extra link (LDS-privatised).
__global__ __launch_bounds__(kBlock) void k_link_hist(uint64_t seed, Geom g, HistBounds b, unsigned long long* hist) {
    __shared__ uint32_t h[kMaxWorld * kMaxPieces * kMaxWorld * 8];
    const uint32_t nb = b.ns * b.nd * 8;
    for (uint32_t i = threadIdx.x; i < nb; i += kBlock) h[i] = 0;
    __syncthreads();
    for (uint32_t u = blockIdx.x * kBlock + threadIdx.x; u < g.wired; u += gridDim.x * kBlock) {
        const uint32_t sp = owner(b.sb, b.ns, u), dp = owner(b.db, b.nd, link_of(seed, u, g.wired));
        atomicAdd(&h[(sp * b.nd + dp) * 8 + popc(presence(g, u))], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += kBlock)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// ------------------------------------------------------------------ generic (bucketed) paths
__device__ __forceinline__ uint32_t generic_deg(const RoundArgs& a, uint32_t v, uint32_t& m) {
    if (a.full) {
        m = 0;
        return a.nodes;  // all j != v among 0..nodes (program.fs:201-206)
    }
    m = presence(a.g, v);
    return popc(m);
}

__device__ __forceinline__ uint32_t generic_target(const RoundArgs& a, uint32_t v, uint32_t m, uint32_t idx) {
    if (a.full) return idx + (idx >= v ? 1u : 0u);
    const uint32_t code = kth_bit(m, idx);
    return dir_target(a.g, v, code, code == kDirLink ? link_of(a.seed, v, a.nodes) : 0u);
}

// Gossip on any topology (used for "full"): receipts are integer atomics into inc_cur[t]
// (order-free, so exact); the done filter of program.fs:92 is applied receiver-side.
template <bool X>
__device__ __forceinline__ void gs_push_body(const RoundArgs& a, const Xchg* xp) {
    if (a.r && gate(a, (long long)a.r - 1)) return;
    const uint32_t r = a.r;
    uint32_t v, end, step;
    node_range(a.lo, a.hi, a.span, v, end, step);
    uint32_t newly = 0;
    // X: the walk is block-uniform (block_reserve synchronises the block); lanes past the end idle
    for (; X ? v - threadIdx.x < end : v < end; v += step) {
        uint32_t m = 0, d = 0;
        if (!X || v < end) d = generic_deg(a, v, m);
        uint32_t tok = 0;
        if (d) {
            const uint8_t st = a.gstate[v];
            tok = st & 3u;
            uint32_t done = (st >> 2) & 1u;
            if (r) {
                const uint32_t inc = a.inc_prev[v];
                if (inc) {
                    a.inc_prev[v] = 0;
                    if (!done) {
                        const uint32_t c0 = a.cnt[v], c1 = c0 + inc;
                        a.cnt[v] = c1;
                        if (c0 == 0) ++tok;
                        if (c0 <= a.threshold && c1 > a.threshold) {
                            done = 1;
                            ++newly;
                        }
                        a.gstate[v] = (uint8_t)(tok | (done << 2));
                    }
                }
            }
        }
        if (!X) {
            if (tok) {
                const uint4 px = philox(v, r, kStreamGossip, a.seed);
                const uint32_t t0 = generic_target(a, v, m, scale_draw(px.x, d));
                const uint32_t t1 = tok > 1 ? generic_target(a, v, m, scale_draw(px.y, d)) : t0;
                // The sender skips a target it sees done (program.fs:92), so ~2/3 of a run's
                // receipts never become atomics.  The byte it reads is the target's state after
                // round r-2 or r-1 (this kernel may have applied r-1 already); done only ever turns
                // on, so a target seen done is also done under the receiver's filter (state after
                // r-1), which drops the receipt anyway.
                const bool send1 = tok > 1;
                const uint8_t s0 = a.gstate[t0];
                const uint8_t s1 = send1 ? a.gstate[t1] : (uint8_t)4u;
                if (!(s0 & 4u)) atomicAdd(&a.inc_cur[t0], 1u);
                if (!(s1 & 4u)) atomicAdd(&a.inc_cur[t1], 1u);
            }
        } else {  // receipts for another rank's actors go to its send chunk (the target id)
            const Xchg& x = *xp;
            uint32_t t[2] = {0u, 0u};
            if (tok) {
                const uint4 px = philox(v, r, kStreamGossip, a.seed);
                t[0] = generic_target(a, v, m, scale_draw(px.x, d));
                t[1] = generic_target(a, v, m, scale_draw(px.y, d));
            }
            bool remote[2];
            uint32_t q[2], pos[2];
#pragma unroll
            for (uint32_t c = 0; c < 2; ++c) {
                const bool send = tok > c;
                remote[c] = send && (t[c] < a.olo || t[c] >= a.ohi);
                // local targets: the sender-side done filter of the single-GPU kernel
                if (send && !remote[c] && !(a.gstate[t[c]] & 4u)) atomicAdd(&a.inc_cur[t[c]], 1u);
                q[c] = remote[c] ? owner(x.abnd, x.world, t[c]) : 0u;
            }
            block_reserve(x, remote, q, pos);
#pragma unroll
            for (uint32_t c = 0; c < 2; ++c)
                if (remote[c]) put_t<false>(x, q[c], pos[c], t[c], make_double2(0.0, 0.0));
        }
    }
    if (r) block_add(newly, a.parts, (long long)r - 1);
}

__global__ __launch_bounds__(kBlock) void k_gs_push(RoundArgs a) { gs_push_body<false>(a, nullptr); }


// Gossip on a tiny graph (at most kTinyActors actors, one GPU, the generic path: "full"): the whole
// run in one workgroup's LDS, nk rounds per launch with workgroup barriers between them.  Iteration
// k does what the launch F(k) of gs_push_body does: the gate (count after round k - 2), applying
// round k - 1's receipts (program.fs:97-105), emitting round k (:89-95), with the same draws and
// filters; the counts go to total[] / the sub-counter ring as F(k)'s gate and block_add leave them.
// C1 (1000 full gossip): 32 rounds in one launch instead of 32 (profiles/round5/tiny/).
__global__ __launch_bounds__(kTinyBlock) void k_gs_tiny(RoundArgs a, uint32_t nk) {
    __shared__ uint32_t s_cnt[kTinyActors], s_inc[kTinyActors];
    __shared__ uint8_t s_st[kTinyActors];
    __shared__ uint32_t s_red[kTinyBlock / 64];
    const uint32_t n = a.g.actors, k0 = a.r, tid = threadIdx.x;
    for (uint32_t v = tid; v < n; v += kTinyBlock) {
        s_cnt[v] = a.cnt[v];
        s_st[v] = a.gstate[v];
        s_inc[v] = k0 ? a.inc_prev[v] : 0u;  // round k0 - 1's receipts (F(k0) applies them)
    }
    // count after round k0 - 2 (F(k0)'s gate)
    unsigned long long c2 = 0;
    if (k0 >= 2u) {
        uint32_t x = tid < 64u ? *part_slot(a.parts, (long long)k0 - 2, tid) : 0u;
        x = wave_sum(x);  // (wave 0 holds the sum; broadcast below)
        if (tid == 0) s_red[0] = x;
        __syncthreads();
        c2 = (unsigned long long)s_red[0] + (k0 >= 3u ? a.total[k0 - 3u] : 0ull);
    }
    __syncthreads();
    uint32_t k = k0;
    bool gated = false;
    for (; k < k0 + nk; ++k) {
        if (k >= 1u && c2 >= a.target) {  // F(k) exits at its gate, and every later launch too
            gated = true;
            break;
        }
        if (k >= 2u && tid == 0) a.total[k - 2u] = c2;
        uint32_t newly = 0;
        if (k >= 1u) {  // apply round k - 1
            for (uint32_t v = tid; v < n; v += kTinyBlock) {
                const uint32_t inc = s_inc[v];  // (only actors with neighbours receive)
                if (!inc) continue;
                s_inc[v] = 0u;
                const uint8_t st = s_st[v];
                uint32_t tok = st & 3u, done = (st >> 2) & 1u;
                if (done) continue;
                const uint32_t c0 = s_cnt[v], c1 = c0 + inc;
                s_cnt[v] = c1;
                if (c0 == 0) ++tok;
                if (c0 <= a.threshold && c1 > a.threshold) {
                    done = 1;
                    ++newly;
                }
                s_st[v] = (uint8_t)(tok | (done << 2));
            }
            newly = wave_sum(newly);
            if ((tid & 63u) == 0) s_red[tid >> 6] = newly;
        }
        __syncthreads();  // round k - 1 applied
        if (k >= 1u) {
            uint32_t t = 0;
#pragma unroll
            for (uint32_t w = 0; w < kTinyBlock / 64; ++w) t += s_red[w];
            // round k - 1's sub-counters as F(k)'s block_add leaves them (one slot: the sum)
            if (tid < 64u) *part_slot(a.parts, (long long)k - 1, tid) = tid == 0 ? t : 0u;
            c2 = (k >= 2u ? c2 : 0ull) + t;  // now the count after round k - 1
        }
        // emit round k (receipts to targets done after round k - 1 are dropped, as the receiver would)
        for (uint32_t v = tid; v < n; v += kTinyBlock) {
            const uint32_t tok = s_st[v] & 3u;
            if (!tok) continue;
            uint32_t m;
            const uint32_t d = generic_deg(a, v, m);
            if (!d) continue;
            const uint4 px = philox(v, k, kStreamGossip, a.seed);
            const uint32_t t0 = generic_target(a, v, m, scale_draw(px.x, d));
            if (!(s_st[t0] & 4u)) atomicAdd(&s_inc[t0], 1u);
            if (tok > 1u) {
                const uint32_t t1 = generic_target(a, v, m, scale_draw(px.y, d));
                if (!(s_st[t1] & 4u)) atomicAdd(&s_inc[t1], 1u);
            }
        }
        __syncthreads();  // round k emitted (s_red free again)
    }
    // the state F(k - 1) leaves: counts and states, round k - 1's receipts in inc[(k - 1) & 1] (what
    // F(k) reads), the other receipt array empty; a gated run also leaves the totals and sub-counters
    // that the gated launches would (the count stays)
    uint32_t* inc_last = (k & 1u) ? a.inc_prev : a.inc_cur;  // inc[(k - 1) & 1] (a = args(k0))
    uint32_t* inc_next = (k & 1u) ? a.inc_cur : a.inc_prev;
    if ((k0 & 1u) == 0u) {  // args(k0): inc_prev = inc[(k0 - 1) & 1], inc_cur = inc[k0 & 1]
        uint32_t* x = inc_last;
        inc_last = inc_next;
        inc_next = x;
    }
    for (uint32_t v = tid; v < n; v += kTinyBlock) {
        a.cnt[v] = s_cnt[v];
        a.gstate[v] = s_st[v];
        inc_last[v] = gated ? 0u : s_inc[v];
        inc_next[v] = 0u;
    }
    if (gated) {
        for (uint32_t j = k; j < k0 + nk; ++j) {  // launches F(j), j >= k: total[j - 2] = the count
            if (j >= 2u && tid == 0) a.total[j - 2u] = c2;
            if (j >= 1u && tid < 64u) *part_slot(a.parts, (long long)j - 1, tid) = 0u;
        }
    }
}

// Push-sum on a tiny graph (at most kTinyPsActors actors, one GPU, the generic path), a batch of
// rounds in one workgroup's LDS: iteration k does what k_ps_push_emit + the bucket scan + fill do for
// F(k): the gate (count after round k - 1), each actor's collect of round k - 1's messages in
// ascending source order (program.fs:119-143, the same selection walk), its update and emission with
// the same draw, then round k's buckets by destination (LDS counts, a block scan, positions), so the
// next iteration's receivers find their senders.  Totals and sub-counters as F(k) leaves them.
// (zero: cnt is not all zero yet; the round loop zeroes each receiver's count as it reads it)
__device__ __forceinline__ void tiny_buckets(uint32_t n, const uint32_t* tgt, uint32_t* cnt, uint32_t* off,
                                             uint32_t* pos, uint32_t* slot, uint32_t* wsum, bool zero) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    if (zero) {
        for (uint32_t v = tid; v < n; v += kTinyBlock) cnt[v] = 0u;
        __syncthreads();
    }
    for (uint32_t v = tid; v < n; v += kTinyBlock)
        if (tgt[v] != 0xFFFFFFFFu) pos[v] = atomicAdd(&cnt[tgt[v]], 1u);
    __syncthreads();
    // exclusive scan of cnt[0 .. n): two entries per thread, a wave scan, the waves' totals
    static_assert(2u * kTinyBlock >= kTinyPsActors, "two entries per thread");
    const uint32_t i0 = 2u * tid, i1 = i0 + 1u;
    const uint32_t a0 = i0 < n ? cnt[i0] : 0u, a1 = i1 < n ? cnt[i1] : 0u;
    uint32_t inc = a0 + a1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63u) wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t j = 0; j < w; ++j) base += wsum[j];
    const uint32_t ex = base + inc - a0 - a1;
    if (i0 < n) off[i0] = ex;
    if (i1 < n) off[i1] = ex + a0;
    __syncthreads();
    for (uint32_t v = tid; v < n; v += kTinyBlock)
        if (tgt[v] != 0xFFFFFFFFu) slot[off[tgt[v]] + pos[v]] = v;
    __syncthreads();
}

__global__ __launch_bounds__(kTinyBlock) void k_ps_tiny(RoundArgs a, uint32_t nk) {
    __shared__ double2 s_msg[2][kTinyPsActors];  // round k - 1's messages, round k's
    __shared__ uint32_t s_tgt[kTinyPsActors], s_cnt[kTinyPsActors], s_off[kTinyPsActors], s_pos[kTinyPsActors],
        s_slot[kTinyPsActors];
    __shared__ uint8_t s_flg[kTinyPsActors];
    __shared__ uint32_t s_red[kTinyBlock / 64];
    const uint32_t n = a.g.actors, k0 = a.r, tid = threadIdx.x;
    for (uint32_t v = tid; v < n; v += kTinyBlock) {
        s_flg[v] = a.flags[v];
        s_tgt[v] = k0 ? a.tgt_cur[v] : 0xFFFFFFFFu;  // round k0 - 1's targets (tgt is one array)
        s_msg[0][v] = k0 ? a.msg_prev[v] : make_double2(0.0, 0.0);
    }
    // count after round k0 - 1 (F(k0)'s gate)
    unsigned long long c1 = 0;
    if (k0 >= 1u) {
        uint32_t x = tid < 64u ? *part_slot(a.parts, (long long)k0 - 1, tid) : 0u;
        x = wave_sum(x);
        if (tid == 0) s_red[0] = x;
        __syncthreads();
        c1 = (unsigned long long)s_red[0] + (k0 >= 2u ? a.total[k0 - 2u] : 0ull);
    }
    __syncthreads();
    tiny_buckets(n, s_tgt, s_cnt, s_off, s_pos, s_slot, s_red, true);
    uint32_t k = k0, in = 0;
    bool gated = false;
    for (; k < k0 + nk; ++k, in ^= 1u) {
        if (c1 >= a.target) {  // F(k) exits at its gate, and every later launch too
            gated = true;
            break;
        }
        if (k >= 1u && tid == 0) a.total[k - 1u] = c1;
        uint32_t newly = 0;
        for (uint32_t v = tid; v < n; v += kTinyBlock) {
            uint32_t m;
            const uint32_t d = generic_deg(a, v, m);
            const uint32_t c = s_cnt[v];
            s_cnt[v] = 0u;  // (read by v only; round k's counts start from zero)
            uint32_t t = 0xFFFFFFFFu;
            if (d) {
                uint8_t f = s_flg[v];
                double ss = 0.0, ww = 0.0;
                uint32_t cin = 0;
                if (k) {
                    const uint32_t o = s_off[v];
                    long long last = -1;
                    for (uint32_t i = 0; i < c; ++i) {  // ascending source id (k_ps_push_emit's walk)
                        uint32_t best = 0xFFFFFFFFu;
                        for (uint32_t j = 0; j < c; ++j) {
                            const uint32_t sj = s_slot[o + j];
                            if ((long long)sj > last && sj < best) best = sj;
                        }
                        const double2 mm = s_msg[in][best];
                        ss += mm.x;
                        ww += mm.y;
                        last = best;
                    }
                    cin = c;
                }
                double2 held = make_double2(0.0, 0.0);
                if (!(f & 16u)) held = k ? s_msg[in][v] : make_double2((double)v, 1.0);
                const PsOut o = ps_update(f, held, ss, ww, cin, a.delta, a.term_limit);
                if (o.send) {
                    const uint4 x = philox(v, k, kStreamPush, a.seed);
                    t = generic_target(a, v, m, scale_draw(x.x, d));
                    s_msg[in ^ 1u][v] = o.msg;
                }
                s_flg[v] = f;
                if (o.conv_now) {
                    a.frozen[v] = o.msg;
                    ++newly;
                }
            }
            s_tgt[v] = t;
        }
        newly = wave_sum(newly);
        if ((tid & 63u) == 0) s_red[tid >> 6] = newly;
        __syncthreads();  // round k collected and emitted
        uint32_t tsum = 0;
#pragma unroll
        for (uint32_t w = 0; w < kTinyBlock / 64; ++w) tsum += s_red[w];
        if (tid < 64u) *part_slot(a.parts, (long long)k, tid) = tid == 0 ? tsum : 0u;
        c1 += tsum;  // now the count after round k
        __syncthreads();  // (s_red read)
        tiny_buckets(n, s_tgt, s_cnt, s_off, s_pos, s_slot, s_red, false);
    }
    // the state F(k - 1) leaves: flags, round k - 1's messages in msg[(k - 1) & 1] and their targets
    // (a = args(k0); msg_prev is the other buffer of the pair, read-only in the per-round kernels)
    double2* out = ((k - 1u) & 1u) == (k0 & 1u) ? a.msg_cur : const_cast<double2*>(a.msg_prev);
    for (uint32_t v = tid; v < n; v += kTinyBlock) {
        a.flags[v] = s_flg[v];
        if (k > k0) {
            a.tgt_cur[v] = s_tgt[v];
            if (s_tgt[v] != 0xFFFFFFFFu) out[v] = s_msg[in][v];
        }
    }
    if (gated) {
        for (uint32_t j = k; j < k0 + nk; ++j) {  // launches F(j), j >= k: total[j - 1] = the count
            if (j >= 1u && tid == 0) a.total[j - 1u] = c1;
            if (tid < 64u) *part_slot(a.parts, (long long)j, tid) = 0u;
        }
    }
}

// Full-topology gossip on one GPU (program.fs:89-105, "full" neighbours program.fs:201-206):
// four consecutive actors per lane, so the per-actor streams (state byte, receipt and count
// words) are read as one dword / dwordx4 per lane.  Receipts are u32 atomics into inc_cur[t].
// Sender-side done filter (program.fs:92): a sender skips a target whose bit in `dbits` is set.
// A bit is set (atomicOr, once per actor) in the round its actor reports; done only ever turns
// on, and the receiver applies the exact filter (state at round start) anyway, so a skipped
// receipt is one the receiver would have dropped, and a stale 0 bit only costs an atomic.  The
// filter is applied only once 1/GP_GS_FILTER_DIV of the actors have reported (a bit read costs
// less than the atomic it saves only when enough targets are done).  A summary bitmap `dsum`
// (one bit per 32-actor word of dbits, set when the word fills: 391 KB at 100M actors, L2-resident)
// answers for targets in all-done words, so the long tail of a run, where nearly every target is
// done, reads the 12.5 MB bitmap rarely (from 2^25 actors: C4 -7.5%; where dbits fits an L2 the
// extra dependent load cost more, 10M +36%, profiles/round3/c4_tally/cli_dsum.txt).
#ifndef GP_GS_FILTER_DIV
#define GP_GS_FILTER_DIV 16
#endif
// Chains emitted in round r (sum of the 64 sub-counters of ring slot r & 3), computed by every
// wave for itself: all waves read the same final values.
__device__ __forceinline__ uint32_t tally_chains(const GsTally& t, uint32_t r) {
    return wave_sum(*part_slot(t.chains, r, threadIdx.x & 63u));
}

// Column of k_gs_full4 workgroup w in cnt's rows (and its inverse).  Workgroups go round-robin to
// the 8 XCDs, so w and w + 1 run on different L2s; columns grouped per XCD (W is a multiple of 8)
// let one L2 write whole lines of a row (C4 46.36 -> 46.08 ms against column = workgroup index,
// profiles/round4/tally_rows/colxcd_ab).  Any column order serves: a bucket's segment is filled in
// column order, and k_gs_tally_count tallies the segment whole.
__device__ __forceinline__ uint32_t tally_col(uint32_t w, uint32_t W) { return (w & 7u) * (W >> 3) + (w >> 3); }
__device__ __forceinline__ uint32_t tally_wg(uint32_t c, uint32_t W) { return (c % (W >> 3)) * 8u + c / (W >> 3); }

// The state bytes (st4) and the round r - 1 receipt words of actors v0 .. v0+3.  Deep in a run's
// tail (deep: block-uniform) a quad of four done actors skips its receipt words: a done actor ignores
// receipts (program.fs:92), so its words are neither read nor cleared, and whatever lands in them
// later is ignored too (the tally's count pass rewrites them whole); elsewhere both loads go out
// together.
#ifndef GP_DEEP_DIV
#define GP_DEEP_DIV 64  // A/B knob: "deep" = fewer than 1/GP_DEEP_DIV of the nodes not done (0: off)
#endif
// i16: round r - 1 tallied into 16-bit words (k_gs_tally_count); a word holding esc sends to the
// 32-bit word (GsTally::esc).  want: the receipt words were due (read).
__device__ __forceinline__ uint4 load_quad(const RoundArgs& a, const uint16_t* i16, uint32_t v0, uint32_t r, bool deep,
                                           uint32_t& st4, bool& want, uint32_t esc = 0xFFFFu) {
    uint4 in4 = make_uint4(0u, 0u, 0u, 0u);
    st4 = *reinterpret_cast<const uint32_t*>(a.gstate + v0);
    want = r && (!deep || (st4 & 0x04040404u) != 0x04040404u);
    if (want) {
        if (i16) {
            const uint2 h = *reinterpret_cast<const uint2*>(i16 + v0);
            in4 = make_uint4(h.x & 0xFFFFu, h.x >> 16, h.y & 0xFFFFu, h.y >> 16);
            if (in4.x == esc) in4.x = a.inc_prev[v0];
            if (in4.y == esc) in4.y = a.inc_prev[v0 + 1u];
            if (in4.z == esc) in4.z = a.inc_prev[v0 + 2u];
            if (in4.w == esc) in4.w = a.inc_prev[v0 + 3u];
        } else {
            in4 = *reinterpret_cast<const uint4*>(a.inc_prev + v0);
        }
    }
    return in4;
}
__device__ __forceinline__ bool deep_tail(unsigned long long prev, uint32_t target) {
    return GP_DEEP_DIV > 0 && prev < target && (unsigned long long)(target - prev) * GP_DEEP_DIV < target;
}

// The receipts of round r - 1 into the counts and states of actors v0 .. v0+3 (program.fs:97-105; a
// done actor ignores them): returns the new state bytes; the actors that report now are added to
// done4 (bit j) and newly.  zero: clear the consumed receipt words (round r + 1 adds into them).
__device__ __forceinline__ uint32_t gs_apply4(const RoundArgs& a, uint32_t v0, uint32_t st4, const uint32_t (&inc)[4],
                                              bool zero, uint32_t& done4, uint32_t& newly) {
    if (zero) *reinterpret_cast<uint4*>(a.inc_prev + v0) = make_uint4(0u, 0u, 0u, 0u);
    uint4 c4 = *reinterpret_cast<const uint4*>(a.cnt + v0);
    uint32_t c[4] = {c4.x, c4.y, c4.z, c4.w};
    const uint32_t st0 = st4;
    bool counted = false;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t st = (st4 >> (8u * j)) & 0xFFu;
        uint32_t tok = st & 3u, done = (st >> 2) & 1u;
        if (inc[j] && !done) {
            counted = true;
            const uint32_t c0 = c[j], c1 = c0 + inc[j];
            c[j] = c1;
            if (c0 == 0) ++tok;                              // program.fs:99-100
            if (c0 <= a.threshold && c1 > a.threshold) {     // program.fs:102-104
                done = 1;
                ++newly;
                done4 |= 1u << j;
            }
            st4 = (st4 & ~(0xFFu << (8u * j))) | ((tok | (done << 2)) << (8u * j));
        }
    }
    if (counted) *reinterpret_cast<uint4*>(a.cnt + v0) = make_uint4(c[0], c[1], c[2], c[3]);
    if (st4 != st0) *reinterpret_cast<uint32_t*>(a.gstate + v0) = st4;
    return st4;
}

__global__ __launch_bounds__(kBlock) void k_gs_full4(RoundArgs a, GsTally t) {
    extern __shared__ uint32_t tcnt[];  // tally rounds: receipts per target bucket (t.nb)
    const uint32_t r = a.r;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    // Round r tallies as F(r - 1) decided (t.on[r & 3]).  F(r) decides for round r + 1, one round
    // ahead, so that it can leave the receipt words of round r + 1 unzeroed when that round tallies
    // (its count pass writes them whole): 400 MB of stores less per tallied round at C4.  The rule:
    // the chains of round r - 1 that reach a target not done yet (the atomics a round would issue,
    // estimated from the share of nodes not done after round r - 2) reach thr; or, late in the run,
    // while at least 1/kTallyLateDiv of the nodes are not done, on graphs whose done bitmap outgrows
    // an L2 (those with the summary): there the sender filter's bitmap reads (most summary words not
    // yet full) cost more per draw than the tally's passes (C4: 2.2 vs 1.67 ms per round at 90-97%
    // reported; at 10M the bitmap is L2-resident and the filter wins: profiles/round4/c4_late_tally/).
    // Uniform: every block reads the same final counts.
    const bool tally = t.cnt && r >= 1u && t.on[r & 3u];
    // round r - 1 tallied: its receipts are in t.inc16, and its 32-bit words hold stale counts (the
    // round before a round that tallies leaves them unzeroed) but for the 0xFFFF escapes
    const bool from16 = t.cnt && r >= 2u && t.on[(r - 1u) & 3u];
    const double ch = (t.cnt && r >= 1u) ? (double)tally_chains(t, r - 1u) : 0.0;  // (no tally: no chains array)
    const bool tally_next = t.cnt && r >= 1u && prev < a.target &&
                            (ch * (double)(a.target - prev) >= (double)t.thr * (double)a.target ||
                             (kTallyLateDiv && a.dsum && (unsigned long long)GP_GS_FILTER_DIV * prev >= a.target &&
                              (unsigned long long)(a.target - prev) * kTallyLateDiv >= a.target && ch >= (double)t.thr));
    if (t.cnt && blockIdx.x == 0 && threadIdx.x < 64) {
        *part_slot(t.chains, r + 2u, threadIdx.x) = 0u;  // the slot round r + 2 adds into
        if (threadIdx.x == 0) t.on[(r + 1u) & 3u] = tally_next ? 1u : 0u;
    }
    if (r && prev >= a.target) {
        // past convergence (the choice was made on an older count): this round's passes must not run
        // on counts this kernel did not write
        if (t.cnt && blockIdx.x == 0 && threadIdx.x == 0) t.on[r & 3u] = 0u;
        return;
    }
    if (tally) {
        for (uint32_t i = threadIdx.x; i < t.nb; i += kBlock) tcnt[i] = 0u;
        __syncthreads();
    }
    const bool filter = (unsigned long long)GP_GS_FILTER_DIV * prev >= a.target;
    const bool deep = deep_tail(prev, a.target);
    const uint32_t na = a.hi;  // one GPU: actors [0, na)
    const uint32_t nq = (na + 3u) >> 2;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    uint32_t q, end, step;
    node_range(0u, nq, span4, q, end, step);
    uint32_t newly = 0, chains = 0;
    const uint16_t* i16 = from16 ? t.inc16 : nullptr;
    // uniform per wave: the 8 lanes sharing a bitmap word reduce together
    for (; q - (threadIdx.x & 63u) < end; q += step) {
        const bool valid = q < end;
        const uint32_t v0 = q << 2;
        uint32_t st4 = 0, done4 = 0;
        if (valid) {
            bool want;
            uint4 in4 = load_quad(a, i16, v0, r, deep, st4, want, t.esc);
            uint32_t inc[4] = {in4.x, in4.y, in4.z, in4.w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (v0 + j >= na) inc[j] = 0u;  // the padding past the last actor
            // round r + 1 adds its receipts into the words of round r - 1 unless it tallies: after a
            // tallied round they are cleared whole (stale), else the consumed ones
            if (from16 && !tally_next && want) *reinterpret_cast<uint4*>(a.inc_prev + v0) = make_uint4(0u, 0u, 0u, 0u);
            if (inc[0] | inc[1] | inc[2] | inc[3])
                st4 = gs_apply4(a, v0, st4, inc, !tally_next && !from16, done4, newly);
            // emit round r: one draw per activation chain (program.fs:89-95)
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t v = v0 + j, tok = (st4 >> (8u * j)) & 3u;
                if (tok && v < na) {
                    const uint4 px = philox(v, r, kStreamGossip, a.seed);
                    const uint32_t t0 = scale_draw(px.x, a.nodes), u0 = t0 + (t0 >= v ? 1u : 0u);
                    const uint32_t t1 = scale_draw(px.y, a.nodes), u1 = t1 + (t1 >= v ? 1u : 0u);
                    const bool s1 = tok > 1;
                    chains += s1 ? 2u : 1u;
                    if (tally) {  // counted per target bucket (LDS); placed by k_gs_tally_scatter
                        atomicAdd(&tcnt[u0 >> kTallyShift], 1u);
                        if (s1) atomicAdd(&tcnt[u1 >> kTallyShift], 1u);
                        continue;
                    }
                    uint32_t b0 = 0, b1 = 0;
                    if (filter && a.dsum) {  // a set summary bit: all 32 actors of the word are done
                        const bool f0 = (a.dsum[u0 >> 10] >> ((u0 >> 5) & 31u)) & 1u;
                        const bool f1 = s1 && ((a.dsum[u1 >> 10] >> ((u1 >> 5) & 31u)) & 1u);
                        b0 = f0 ? ~0u : load_sel(a.dbits, true, u0 >> 5, 0u);
                        if (s1) b1 = f1 ? ~0u : load_sel(a.dbits, true, u1 >> 5, 0u);
                    } else if (filter) {
                        b0 = a.dbits[u0 >> 5];
                        if (s1) b1 = a.dbits[u1 >> 5];
                    }
                    if (!((b0 >> (u0 & 31u)) & 1u)) atomicAdd(&a.inc_cur[u0], 1u);
                    if (s1 && !((b1 >> (u1 & 31u)) & 1u)) atomicAdd(&a.inc_cur[u1], 1u);
                }
            }
        }
        // the reports of this round into the done bitmap: 8 lanes = 32 actors = one word
        uint32_t w = done4 << ((q & 7u) * 4u);
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        if (w && (q & 7u) == 0u) {
            const uint32_t wi = q >> 3;
            if (a.dsum) {  // a returning atomic: the summary bit is set by the report that fills the word
                const uint32_t old = atomicOr(&a.dbits[wi], w);
                if ((old | w) == ~0u && old != ~0u) atomicOr(&a.dsum[wi >> 5], 1u << (wi & 31u));
            } else {
                atomicOr(&a.dbits[wi], w);
            }
        }
    }
    if (r) block_add(newly, a.parts, (long long)r - 1);
    if (t.cnt) {
        __syncthreads();  // block_add's LDS slots are reused
        block_add(chains, t.chains, r);
    }
    if (tally) {  // this workgroup's counts, bucket-major for the scan
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < t.nb; i += kBlock) t.cnt[i * t.W + tally_col(blockIdx.x, t.W)] = tcnt[i];
    }
}

// Full gossip's ramp (GsSparse, gp_kernels.h): F(r) on lists.  Work items [0, tp) apply the receipts
// of round r - 1 to the listed targets (program.fs:97-105; the receiver drops receipts to done actors,
// exactly as k_gs_full4's gs_apply4), [tp, tp + hb) are the chain holders, which emit round r
// (program.fs:89-95, one draw per chain: "full" holds one chain per actor); a first receipt starts a
// chain, and its actor emits here too.  Every receipt lists its target (a target listed twice takes
// its count once: the apply exchanges the word with 0), so no atomic on the way waits for its result
// but the lists' own.  No sender-side filter (it only saves atomics).  The same gate, counts, done
// bitmap and tally bookkeeping as k_gs_full4, so a k_gs_full4 round can follow.
// F(r)'s list lengths: hb holders after F(r - 1), tp targets of round r - 1 (clamped to the lists: a
// count past them has set err, and the host fails the step); block 0 records hb and restarts the
// counters F(r + 1) appends to (F(r - 3)'s, read long ago).
__device__ __forceinline__ void sp_counts(const GsSparse& sp, uint32_t r, uint32_t& hb, uint32_t& tp) {
    const uint32_t size = 2u * sp.cap + kSpSlack;
    hb = r ? *sp_ctr(sp, 0, r - 1u) + *sp_ctr(sp, 1, r - 1u) : sp.h0;
    tp = r ? *sp_ctr(sp, 2, r - 1u) : 0u;
    hb = hb < size ? hb : size;
    tp = tp < size ? tp : size;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *sp_ctr(sp, 0, r) = hb;
        *sp_ctr(sp, 1, r + 1u) = 0u;
        *sp_ctr(sp, 2, r + 1u) = 0u;
    }
}
// F(r)'s apply of a listed target v (its receipts of round r - 1; 0 where an earlier copy of the entry
// took them): program.fs:97-105 as k_gs_full4's gs_apply4, the report into the done bitmap.  Returns
// whether a chain starts (the actor joins the holders and emits this round).
__device__ __forceinline__ bool sp_apply(const RoundArgs& a, uint32_t v, uint32_t& newly) {
    const uint32_t inc = atomicExch(&a.inc_prev[v], 0u);  // round r + 1 adds into this word
    const uint32_t st = a.gstate[v];
    uint32_t tok = st & 3u, done = (st >> 2) & 1u;
    bool start = false;
    if (inc && !done) {
        const uint32_t c0 = a.cnt[v], c1 = c0 + inc;
        a.cnt[v] = c1;
        if (c0 == 0) {  // program.fs:99-100: a chain starts, and emits this round
            ++tok;
            start = true;
        }
        if (c0 <= a.threshold && c1 > a.threshold) {  // program.fs:102-104
            done = 1u;
            ++newly;
            const uint32_t bit = 1u << (v & 31u), old = atomicOr(&a.dbits[v >> 5], bit);
            if (a.dsum && (old | bit) == ~0u && old != ~0u) atomicOr(&a.dsum[v >> 10], 1u << ((v >> 5) & 31u));
        }
        a.gstate[v] = (uint8_t)(tok | (done << 2));
    }
    return start;
}

__global__ __launch_bounds__(kBlock) void k_gs_sparse(RoundArgs a, GsTally t, GsSparse sp) {
    const uint32_t r = a.r;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    // round r + 1's tally decision and the chain ring, as k_gs_full4 makes them
    const double ch = (t.cnt && r >= 1u) ? (double)tally_chains(t, r - 1u) : 0.0;
    const bool tally_next = t.cnt && r >= 1u && prev < a.target &&
                            (ch * (double)(a.target - prev) >= (double)t.thr * (double)a.target ||
                             (kTallyLateDiv && a.dsum && (unsigned long long)GP_GS_FILTER_DIV * prev >= a.target &&
                              (unsigned long long)(a.target - prev) * kTallyLateDiv >= a.target && ch >= (double)t.thr));
    if (t.cnt && blockIdx.x == 0 && threadIdx.x < 64) {
        *part_slot(t.chains, r + 2u, threadIdx.x) = 0u;
        if (threadIdx.x == 0) {
            t.on[(r + 1u) & 3u] = tally_next ? 1u : 0u;
            t.on[r & 3u] = 0u;  // this round does not tally: F(r + 1) reads its receipts from the 32-bit words
        }
    }
    uint32_t hb, tp;
    sp_counts(sp, r, hb, tp);
    if (r && prev >= a.target) {
        if (t.cnt && blockIdx.x == 0 && threadIdx.x == 0) t.on[r & 3u] = 0u;
        return;
    }
    const uint32_t size = 2u * sp.cap + kSpSlack;
    const uint32_t* tprev = sp.tl[(r + 1u) & 1u];
    uint32_t* tcur = sp.tl[r & 1u];
    uint32_t newly = 0, chains = 0;
    const uint32_t nw = tp + hb;
    for (uint32_t i0 = blockIdx.x * kBlock; i0 < nw; i0 += gridDim.x * kBlock) {
        const uint32_t i = i0 + threadIdx.x;
        bool emit = false, newh = false;
        uint32_t v = 0;
        if (i < tp) {  // a listed target: its receipts (>= 1) of round r - 1
            v = tprev[i];
            newh = emit = sp_apply(a, v, newly);
        } else if (i < nw) {  // a chain holder
            v = sp.hl[i - tp];
            emit = true;
        }
        uint32_t u0 = 0;
        if (emit) {
            const uint4 px = philox(v, r, kStreamGossip, a.seed);
            const uint32_t t0 = scale_draw(px.x, a.nodes);
            u0 = t0 + (t0 >= v ? 1u : 0u);
            atomicAdd(&a.inc_cur[u0], 1u);
            ++chains;
        }
        // (every receipt listed, or only a first one by a returning atomic: C4 43.0-43.3 ms either way,
        // profiles/round6/shard_ramp/c4_one_gpu_ab.txt)
        wave_append2(newh, v, sp.hl + hb, sp_ctr(sp, 1, r), size - hb, emit, u0, tcur, sp_ctr(sp, 2, r), size, sp.err);
    }
    if (r) block_add(newly, a.parts, (long long)r - 1);
    if (t.cnt) {
        __syncthreads();  // block_add's LDS slots are reused
        block_add(chains, t.chains, r);
    }
}

// Full gossip on a shard of several ranks: k_gs_full4's walk over this rank's actors
// [lo, hi), four consecutive actors per lane (the quads of the first and last lanes may hold other
// ranks' actors, which are masked out: neither applied nor emitted).  Every receipt first takes the
// sender-side done filter of the one-GPU kernel on this rank's replica of the whole done bitmap
// (global bit = actor id, its summary from 2^25 actors): its own words are current, the other ranks'
// arrive with every exchange (k_shard_done_out / k_shard_unpack), a round late at most, which the
// filter tolerates (done only turns on).  A receipt for one of this rank's actors is then a
// memory-side atomic; one for another rank's actor an entry of that rank's chunk (the target id),
// reserved per block and peer.  The receiver drops the entries for its done actors before the
// atomic (k_shard_unpack): the filter program.fs:92 applies there exactly.
__global__ __launch_bounds__(kBlock) void k_gs_full4x(RoundArgs a, Xchg x) {
    const uint32_t r = a.r;
    // the chain ring slot round r + 2 adds into (the pack of round r - 2, its last reader, has run)
    if (a.cparts && blockIdx.x == 0 && threadIdx.x < 64) *part_slot(a.cparts, r + 2u, threadIdx.x) = 0u;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    if (r && prev >= a.target) return;
    const bool filter = (unsigned long long)GP_GS_FILTER_DIV * prev >= a.target;  // global count
    const bool deep = deep_tail(prev, a.target);
    const uint32_t lo = a.lo, hi = a.hi;
    // quads from a multiple of 8 (8 lanes = 32 actors = one bitmap word)
    const uint32_t q0 = (lo >> 2) & ~7u, q1 = (hi + 3u) >> 2, nq = q1 - q0;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    uint32_t q, end, step;
    node_range(q0, q1, span4, q, end, step);
    uint32_t newly = 0, chains = 0;
    // block-uniform trip count: block_reserve synchronises the block; lanes past the end idle
    for (; q - threadIdx.x < end; q += step) {
        const bool valid = q < end;
        const uint32_t v0 = q << 2;
        uint32_t st4 = 0, done4 = 0, mine = 0;  // mine: actors of this rank among v0 .. v0+3
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) mine |= (valid && v0 + j - lo < hi - lo) ? 1u << j : 0u;
        if (mine) {
            bool due;
            uint4 in4 = load_quad(a, nullptr, v0, r, deep, st4, due);
            uint32_t inc[4] = {in4.x, in4.y, in4.z, in4.w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (!((mine >> j) & 1u)) inc[j] = 0u;  // another rank's actor (or padding)
            if (inc[0] | inc[1] | inc[2] | inc[3]) st4 = gs_apply4(a, v0, st4, inc, true, done4, newly);
        }
        // emit round r: one draw per activation chain (program.fs:89-95); local receipts now, remote
        // ones after the block's reservation
        bool want[8];
        uint32_t peer[8], tgt[8], pos[8];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t v = v0 + j, tok = ((mine >> j) & 1u) ? (st4 >> (8u * j)) & 3u : 0u;
            uint32_t u[2] = {0u, 0u};
            chains += tok;
            if (tok) {
                const uint4 px = philox(v, r, kStreamGossip, a.seed);
                const uint32_t t0 = scale_draw(px.x, a.nodes), t1 = scale_draw(px.y, a.nodes);
                u[0] = t0 + (t0 >= v ? 1u : 0u);
                u[1] = t1 + (t1 >= v ? 1u : 0u);
            }
#pragma unroll
            for (uint32_t c = 0; c < 2; ++c) {
                const bool local = u[c] - lo < hi - lo;
                // the sender-side done filter on the replica: this rank's own words are current,
                // another rank's as of the last exchange (stale bits are 0, never 1 too early)
                uint32_t b = 0;
                if (tok > c && filter) {
                    if (a.dsum && ((a.dsum[u[c] >> 10] >> ((u[c] >> 5) & 31u)) & 1u)) b = ~0u;
                    else b = a.dbits[u[c] >> 5];
                }
                const bool send = tok > c && !((b >> (u[c] & 31u)) & 1u);
                want[2 * j + c] = send && !local;
                tgt[2 * j + c] = u[c];
                peer[2 * j + c] = want[2 * j + c] ? owner(x.abnd, x.world, u[c]) : 0u;
                if (send && local) atomicAdd(&a.inc_cur[u[c]], 1u);
            }
        }
        // sub-segment by the block-iteration's 1024-actor chunk (its first quad / 256, block-uniform):
        // consecutive chunks of the range cycle through the kSub sub-segments whatever the grid, so
        // gp_api.cpp sizes a sub-segment for ceil(chunks / kSub) chunks
        const uint32_t sub = ((q - threadIdx.x) >> 8) % kSub;
        bool any = false;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) any |= want[k];
        if (__syncthreads_or(any)) {  // block-uniform: most block-iterations of a quiet round send nothing
            block_reserve(x, want, peer, pos, sub);
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)
                if (want[k]) put_t<false>(x, peer[k], pos[k], tgt[k], make_double2(0.0, 0.0), sub);
        }
        // the reports of this round into the done bitmap: 8 lanes = 32 actors = one word
        uint32_t w = done4 << ((q & 7u) * 4u);
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        if (w && (q & 7u) == 0u) {
            const uint32_t wi = q >> 3;
            if (a.dsum) {
                const uint32_t old = atomicOr(&a.dbits[wi], w);
                if ((old | w) == ~0u && old != ~0u) atomicOr(&a.dsum[wi >> 5], 1u << (wi & 31u));
            } else {
                atomicOr(&a.dbits[wi], w);
            }
        }
    }
    if (r) block_add(newly, a.parts, (long long)r - 1);
    if (a.cparts) {  // the chains of round r: they size the next rounds' exchange (gp_api.cpp gs_cap)
        __syncthreads();  // block_add's LDS slots are reused
        block_add(chains, a.cparts, r);
    }
}

// ---- full gossip on shards: the receipt wave in bins (GsBins, gp_kernels.h)
// Owner rank qq of remote target u and its bin in the passes' numbering: one uniform loop over the
// ranks (scalar loads and selects; a per-lane index into the kernel arguments is a vector load per
// receipt, which kept the texture path 88% busy).
__device__ __forceinline__ void peer_bin(const Xchg& x, const GsBins& b, uint32_t u, uint32_t& qq, uint32_t& bin) {
    uint32_t q = 0, base = x.abnd[0], b0 = b.bin0[0];
    for (uint32_t i = 1; i < x.world; ++i) {
        const bool ge = u >= x.abnd[i];
        q = ge ? i : q;
        base = ge ? x.abnd[i] : base;
        b0 = ge ? b.bin0[i] : b0;
    }
    qq = q;
    bin = b0 + ((u - base) >> kTallyShift);
}
// A chunk's entry part in bins: the start table (nb + 1 words), then the u16 entries (their capacity).
__device__ __forceinline__ uint32_t bins_room(uint32_t cap, uint32_t nb) {
    const uint32_t w = kSub * cap;
    return w > nb + 1u ? 2u * (w - nb - 1u) : 0u;
}

// F(r) of a receipt-wave round: k_gs_full4x's walk, apply and draws; every receipt is counted in its
// (rank, bin) LDS counter, written out per workgroup for the scan (a local receipt too: the memory-side
// atomic it took cost ~80 us of this kernel's ~160 per rank-round at C4 / 8).  Every receipt is sent
// (no sender-side filter: a bin entry costs less than the filter's bitmap read).
__global__ __launch_bounds__(kBlock) void k_gs_bins_count(RoundArgs a, Xchg x, GsBins b) {
    extern __shared__ uint32_t lc[];
    const uint32_t r = a.r;
    if (a.cparts && blockIdx.x == 0 && threadIdx.x < 64) *part_slot(a.cparts, r + 2u, threadIdx.x) = 0u;
    for (uint32_t i = threadIdx.x; i < b.nbt; i += kBlock) lc[i] = 0u;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    const bool live = !(r && prev >= a.target);  // converged: zero counts still go out (no entry placed)
    const bool deep = deep_tail(prev, a.target);
    __syncthreads();
    const uint32_t lo = a.lo, hi = a.hi;
    const uint32_t q0 = (lo >> 2) & ~7u, q1 = (hi + 3u) >> 2, nq = q1 - q0;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    uint32_t q, end, step;
    node_range(q0, q1, span4, q, end, step);
    if (!live) end = 0;
    uint32_t newly = 0, chains = 0;
    // block-uniform trip count (the done word's shuffles); lanes past the end idle
    for (; q - threadIdx.x < end; q += step) {
        const bool valid = q < end;
        const uint32_t v0 = q << 2;
        uint32_t st4 = 0, done4 = 0, mine = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) mine |= (valid && v0 + j - lo < hi - lo) ? 1u << j : 0u;
        if (mine) {
            bool due;
            uint4 in4 = load_quad(a, nullptr, v0, r, deep, st4, due);
            uint32_t inc[4] = {in4.x, in4.y, in4.z, in4.w};
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (!((mine >> j) & 1u)) inc[j] = 0u;
            if (inc[0] | inc[1] | inc[2] | inc[3]) st4 = gs_apply4(a, v0, st4, inc, true, done4, newly);
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t v = v0 + j, tok = ((mine >> j) & 1u) ? (st4 >> (8u * j)) & 3u : 0u;
                if (!tok) continue;
                chains += tok;
                const uint4 px = philox(v, r, kStreamGossip, a.seed);  // program.fs:89-95
                const uint32_t t0 = scale_draw(px.x, a.nodes), t1 = scale_draw(px.y, a.nodes);
                const uint32_t u[2] = {t0 + (t0 >= v ? 1u : 0u), t1 + (t1 >= v ? 1u : 0u)};
#pragma unroll
                for (uint32_t c = 0; c < 2; ++c) {
                    if (tok <= c) break;
                    uint32_t qq, bin;  // (this rank's own actors too: its own chunk)
                    peer_bin(x, b, u[c], qq, bin);
                    atomicAdd(&lc[bin], 1u);
                }
            }
        }
        // the reports of this round into the done bitmap: 8 lanes = 32 actors = one word
        uint32_t w = done4 << ((q & 7u) * 4u);
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        if (w && (q & 7u) == 0u) {
            const uint32_t wi = q >> 3;
            if (a.dsum) {
                const uint32_t old = atomicOr(&a.dbits[wi], w);
                if ((old | w) == ~0u && old != ~0u) atomicOr(&a.dsum[wi >> 5], 1u << (wi & 31u));
            } else {
                atomicOr(&a.dbits[wi], w);
            }
        }
    }
    __syncthreads();
    const uint32_t col = tally_col(blockIdx.x, b.W);
    for (uint32_t i = threadIdx.x; i < b.nbt; i += kBlock) b.cnt[i * b.W + col] = lc[i];
    if (r) block_add(newly, a.parts, (long long)r - 1);
    if (a.cparts) {
        __syncthreads();  // block_add's LDS slots are reused
        block_add(chains, a.cparts, r);
    }
}

// The placement of a receipt-wave round: the same grid and walk as k_gs_bins_count, the same draws
// from the states F(r) left, so every (peer, bin, workgroup) gets exactly the count it reported; a
// receipt takes the next place of its (peer, bin) in LDS.  Block 0 writes every peer's bin starts and
// sets the entry counters the pack reports (its total over the sub-segments, within each one's
// capacity); a chunk whose entries outgrow its room overflows (replayed or fatal, as entries).
__global__ __launch_bounds__(kBlock) void k_gs_bins_place(RoundArgs a, Xchg x, GsBins b) {
    extern __shared__ uint32_t lp[];
    __shared__ uint32_t pbase[kMaxWorld], proom[kMaxWorld], pabnd[kMaxWorld];
    __shared__ uint16_t* pe16[kMaxWorld];
    const uint32_t r = a.r;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    const bool live = !(r && prev >= a.target);
    const uint32_t col = tally_col(blockIdx.x, b.W);
    for (uint32_t i = threadIdx.x; i < b.nbt; i += kBlock) lp[i] = b.off[i * b.W + col];
    // per rank: first entry, room, first actor, entries (LDS: per-lane reads).  (A per-lane index into
    // the kernel arguments, or a pointer chosen between two of them, makes the compiler copy all 1.8 KB
    // of them to every thread's scratch: 0.5 GB of writes per launch at C4 / 8.)
    if (threadIdx.x < x.world) {
        const uint32_t qq = threadIdx.x, nb = b.bin0[qq + 1u] - b.bin0[qq];
        pbase[qq] = b.off[b.bin0[qq] * b.W];
        pabnd[qq] = x.abnd[qq];
        if (qq != x.rank) {
            proom[qq] = bins_room(x.out[qq].cap, nb);
            pe16[qq] = reinterpret_cast<uint16_t*>(x.out[qq].slot + nb + 1u);
        }
    }
    const uint32_t nbs = b.bin0[x.rank + 1u] - b.bin0[x.rank];  // this rank's own chunk
    if (threadIdx.x == 0) {
        proom[x.rank] = 2u * (b.self_words - nbs - 1u);
        pe16[x.rank] = reinterpret_cast<uint16_t*>(b.self + nbs + 1u);
    }
    __syncthreads();
    if (blockIdx.x == 0) {  // the bin starts, relative to each rank's first entry
        for (uint32_t i = threadIdx.x; i <= nbs; i += kBlock) b.self[i] = b.off[(b.bin0[x.rank] + i) * b.W] - pbase[x.rank];
        for (uint32_t qq = 0; qq < x.world; ++qq) {
            if (qq == x.rank) continue;  // (its own chunk holds every own receipt: no overflow, no header)
            const uint32_t nb = b.bin0[qq + 1u] - b.bin0[qq];
            for (uint32_t i = threadIdx.x; i <= nb; i += kBlock) x.out[qq].slot[i] = b.off[(b.bin0[qq] + i) * b.W] - pbase[qq];
            if (threadIdx.x < kSub) {
                const uint32_t e = b.off[b.bin0[qq + 1u] * b.W] - pbase[qq], cap = x.out[qq].cap;
                const uint32_t per = (e + kSub - 1u) / kSub;
                *ctr_at(x, qq, threadIdx.x) = per < cap ? per : cap;
                if (threadIdx.x == 0 && e > bins_room(cap, nb)) atomicOr(x.overflow, 1u);
            }
        }
    }
    if (!live) return;
    const uint32_t lo = a.lo, hi = a.hi;
    const uint32_t q0 = (lo >> 2) & ~7u, q1 = (hi + 3u) >> 2, nq = q1 - q0;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    uint32_t q, end, step;
    node_range(q0, q1, span4, q, end, step);
    for (; q < end; q += step) {
        const uint32_t v0 = q << 2;
        uint32_t mine = 0;  // (as k_gs_bins_count: a quad with none of this rank's actors is not read)
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) mine |= v0 + j - lo < hi - lo ? 1u << j : 0u;
        if (!mine) continue;
        const uint32_t st4 = *reinterpret_cast<const uint32_t*>(a.gstate + v0);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t v = v0 + j;
            const uint32_t tok = ((mine >> j) & 1u) ? (st4 >> (8u * j)) & 3u : 0u;
            if (!tok) continue;
            const uint4 px = philox(v, r, kStreamGossip, a.seed);
            const uint32_t t0 = scale_draw(px.x, a.nodes), t1 = scale_draw(px.y, a.nodes);
            const uint32_t u[2] = {t0 + (t0 >= v ? 1u : 0u), t1 + (t1 >= v ? 1u : 0u)};
#pragma unroll
            for (uint32_t c = 0; c < 2; ++c) {
                if (tok <= c) break;
                uint32_t qq, bin;
                peer_bin(x, b, u[c], qq, bin);
                const uint32_t pos = atomicAdd(&lp[bin], 1u) - pbase[qq];
                if (pos < proom[qq]) pe16[qq][pos] = (uint16_t)((u[c] - pabnd[qq]) & ((1u << kTallyShift) - 1u));
            }
        }
    }
}

// The receiver of a receipt-wave round: workgroup = one bin of this rank's actors; every rank's entries
// of the bin (its own from its own chunk) counted in LDS, then written as the bin's receipt words, zeros
// included.  A done actor's receipts are counted too: F(r + 1) ignores them (program.fs:92's filter, at
// the receiver).
constexpr uint32_t kBinBlock = 1024;
__global__ __launch_bounds__(kBinBlock) void k_shard_unpack_bins(RoundArgs a, Xchg x, GsBins b) {
    extern __shared__ uint32_t h[];
    constexpr uint32_t S = 1u << kTallyShift;
    for (uint32_t i = threadIdx.x; i < S; i += kBinBlock) h[i] = 0u;
    __syncthreads();
    const uint32_t bin = blockIdx.x, nb = b.nb_self;
    const uint32_t base = x.abnd[x.rank] + (bin << kTallyShift), top = x.abnd[x.rank + 1u];
    const uint32_t n = top - base < S ? top - base : S;
    for (uint32_t qq = 0; qq < x.world; ++qq) {
        const bool own = qq == x.rank;
        const PeerIn& in = x.in[qq];
        if (!own && (!in.cap || !in.hdr->binned)) continue;  // uniform
        const uint32_t* tab = own ? b.self : in.slot;
        const uint32_t room = own ? 2u * (b.self_words - nb - 1u) : bins_room(in.cap, nb), e = tab[nb];
        const uint32_t s0 = tab[bin], s1 = min(tab[bin + 1u], min(e, room));
        if (s0 > s1) {  // a corrupt chunk: reported, never applied
            if (threadIdx.x == 0 && s0 > tab[bin + 1u]) atomicOr(x.overflow, 2u);
            continue;
        }
        const uint16_t* e16 = reinterpret_cast<const uint16_t*>(tab + nb + 1u);
        for (uint32_t i = s0 + threadIdx.x; i < s1; i += kBinBlock) {
            const uint32_t t = e16[i];
            if (t < n) atomicAdd(&h[t], 1u);
            else atomicOr(x.overflow, 2u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += kBinBlock) a.inc_cur[base + i] = h[i];
}

// Positions of one entry per thread in peer q's chunk, sub-segment sb (both per thread): LDS counters
// per (peer, sub-segment), then one global atomic per pair present.  Every thread of the block must
// call it.
static_assert(kMaxWorld * kSub == kBlock, "block_reserve_qs: one LDS counter per thread");
__device__ __forceinline__ uint32_t block_reserve_qs(const Xchg& x, bool want, uint32_t q, uint32_t sb) {
    __shared__ uint32_t cnt[kMaxWorld * kSub], base[kMaxWorld * kSub];
    cnt[threadIdx.x] = 0u;
    peer_tab_fill(x);
    __syncthreads();
    const uint32_t key = q * kSub + sb;
    const uint32_t pos = want ? atomicAdd(&cnt[key], 1u) : 0u;
    __syncthreads();
    if (const uint32_t c = cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(ctr_at(x, threadIdx.x / kSub, threadIdx.x % kSub), c);
    __syncthreads();
    return want ? pos + base[key] : 0u;
}

// Full gossip on shards: this rank's words of the done bitmap (after F(r)) into every peer's chunk.
// The peers' replicas only feed the sender-side filter, which stays exact however stale they are
// (done only turns on; the receiver filters exactly), so words are shipped lazily: a word goes out
// when it differs from what was last shipped (x.dship).  The plan's done part is either every word
// of the range (dpairs 0: the receivers read them all when any changed) or up to dpairs (index,
// word) pairs; words past that capacity stay dirty for a later round (x.dstat backlog flag).  Every
// peer gets the same words.
// (blocks bid of nblk: the pass's grid, or the one block that ends a list round, k_gs_sparse_x)
__device__ __forceinline__ void done_out_body(const RoundArgs& a, const Xchg& x, uint32_t bid, uint32_t nblk) {
    if (applied_converged(a)) return;  // block-uniform
    // none of this rank's actors reported in the round F(r) applied and no word is left over: no word
    // differs from what was shipped (the early rounds of a run); the header's counts stay 0
    const uint32_t newly = a.r ? wave_sum(*part_slot(a.parts, (long long)a.r - 1, threadIdx.x & 63u)) : 0u;
    if (!newly && !x.dstat[kDstatLeft]) return;  // uniform: every wave sums the same final sub-counters
    uint32_t dp = 0;
    bool any = false;
    for (uint32_t q = 0; q < x.world && !any; ++q)
        if (q != x.rank && x.out[q].done) {
            dp = x.out[q].dpairs;  // the sender's plan: the same for every peer
            any = true;
        }
    if (!any) return;
    const uint32_t w0 = a.lo >> 5, nw = ((a.hi - 1u) >> 5) - w0 + 1u;
    // block-uniform trip count: every thread reaches block_reserve1
    for (uint32_t base = bid * kBlock; base < nw; base += nblk * kBlock) {
        const uint32_t i = base + threadIdx.x;
        const bool valid = i < nw;
        const uint32_t val = valid ? a.dbits[w0 + i] : 0u;
        const bool dirty = valid && val != x.dship[w0 + i];
        const uint32_t pos = block_reserve1(&x.dstat[kDstatCount], dirty);
        if (!dp) {  // every word
            if (valid)
                for (uint32_t q = 0; q < x.world; ++q)
                    if (q != x.rank && x.out[q].done) x.out[q].done[i] = val;
            if (dirty) x.dship[w0 + i] = val;
        } else if (dirty && pos < dp) {
            for (uint32_t q = 0; q < x.world; ++q)
                if (q != x.rank && x.out[q].done) reinterpret_cast<uint2*>(x.out[q].done)[pos] = make_uint2(w0 + i, val);
            x.dship[w0 + i] = val;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_shard_done_out(RoundArgs a, Xchg x) { done_out_body(a, x, blockIdx.x, gridDim.x); }

// Full gossip's ramp on a shard (GsSparse): k_gs_sparse over this rank's lists — the targets of round
// r - 1 among its actors (its own receipts and the peers', listed by k_shard_unpack) and its chain
// holders.  A receipt for one of its actors is an atomic and a list entry, one for another rank's
// actor an entry of that rank's chunk, in the sub-segment of the sender's
// 1024-actor chunk as k_gs_full4x places it (gp_api.cpp sizes the chunks by that rule).  The same
// counts, chain ring and done bitmap as k_gs_full4x, so a k_gs_full4x round can follow, and each rank
// may leave its lists in a different round.  Its last block also runs the round's two passes after it
// (k_shard_done_out, k_shard_pack).
__global__ __launch_bounds__(kBlock) void k_gs_sparse_x(RoundArgs a, Xchg x, GsSparse sp, long long applied) {
    const uint32_t r = a.r;
    if (a.cparts && blockIdx.x == 0 && threadIdx.x < 64) *part_slot(a.cparts, r + 2u, threadIdx.x) = 0u;
    unsigned long long prev = 0;
    if (r) prev = gate_count(a, (long long)r - 1);
    uint32_t hb, tp;
    sp_counts(sp, r, hb, tp);
    if (r && prev >= a.target) hb = tp = 0u;  // converged: no work, the headers still go out
    const uint32_t size = 2u * sp.cap + kSpSlack, lo = a.lo, hi = a.hi;
    const uint32_t* tprev = sp.tl[(r + 1u) & 1u];
    uint32_t* tcur = sp.tl[r & 1u];
    uint32_t newly = 0, chains = 0;
    const uint32_t nw = tp + hb;
    // block-uniform trip count: block_reserve_qs synchronises the block
    for (uint32_t i0 = blockIdx.x * kBlock; i0 < nw; i0 += gridDim.x * kBlock) {
        const uint32_t i = i0 + threadIdx.x;
        bool emit = false, newh = false;
        uint32_t v = 0;
        if (i < tp) {  // a listed target
            v = tprev[i];
            newh = emit = sp_apply(a, v, newly);
        } else if (i < nw) {  // a chain holder
            v = sp.hl[i - tp];
            emit = true;
        }
        bool local = false, remote = false;
        uint32_t u0 = 0, q = 0;
        if (emit) {  // program.fs:89-95
            const uint4 px = philox(v, r, kStreamGossip, a.seed);
            const uint32_t t0 = scale_draw(px.x, a.nodes);
            u0 = t0 + (t0 >= v ? 1u : 0u);
            ++chains;
            local = u0 - lo < hi - lo;
            remote = !local;
            if (local) atomicAdd(&a.inc_cur[u0], 1u);
            else q = owner(x.abnd, x.world, u0);
        }
        wave_append2(newh, v, sp.hl + hb, sp_ctr(sp, 1, r), size - hb, local, u0, tcur, sp_ctr(sp, 2, r), size, sp.err);
        if (__syncthreads_or(remote)) {  // block-uniform
            const uint32_t sb = (v >> 10) % kSub;
            const uint32_t pos = block_reserve_qs(x, remote, q, sb);
            if (remote) put_t<false>(x, q, pos, u0, make_double2(0.0, 0.0), sb);
        }
    }
    if (r) block_add(newly, a.parts, (long long)r - 1);
    if (a.cparts) {
        __syncthreads();  // block_add's LDS slots are reused
        block_add(chains, a.cparts, r);
    }
    // The block that finishes last ends the round: the done-word pass (after a list round its reports,
    // if any, are few: one block) and the headers, without two more launches.  Every block's counts are
    // device-scope atomics, released before its arrival is counted and acquired by the last block.
    __shared__ uint32_t last_s;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        last_s = atomicAdd(sp.fin, 1u) == gridDim.x - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (!last_s) return;
    __threadfence();
    if (x.dstat) done_out_body(a, x, 0u, 1u);
    __syncthreads();
    shard_pack_body(a, x, applied);
    if (threadIdx.x == 0) *sp.fin = 0u;  // the next list round counts from 0 (stream order)
}

// Tallied round: place every receipt of F(r) into its bucket's segment, at this workgroup's
// offset (the scan of k_gs_full4's counts) plus an LDS position.  Same grid and walk as
// k_gs_full4, same draws, read from the states F(r) wrote, so each (bucket, workgroup) gets
// exactly the count F(r) reported.
__global__ __launch_bounds__(kBlock) void k_gs_tally_scatter(RoundArgs a, GsTally t) {
    extern __shared__ uint32_t tpos[];
    const uint32_t r = a.r;
    if (!t.on[r & 3u]) return;  // uniform
    // this workgroup's first position in every bucket's segment (then LDS atomics give each
    // receipt its place without another global read)
    for (uint32_t i = threadIdx.x; i < t.nb; i += kBlock) tpos[i] = t.off[i * t.W + tally_col(blockIdx.x, t.W)];
    __syncthreads();
    const uint32_t na = a.hi;
    const uint32_t nq = (na + 3u) >> 2;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    uint32_t q, end, step;
    node_range(0u, nq, span4, q, end, step);
    for (; q < end; q += step) {
        const uint32_t v0 = q << 2;
        const uint32_t st4 = *reinterpret_cast<const uint32_t*>(a.gstate + v0);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t v = v0 + j, tok = (st4 >> (8u * j)) & 3u;
            if (tok && v < na) {
                const uint4 px = philox(v, r, kStreamGossip, a.seed);
                const uint32_t t0 = scale_draw(px.x, a.nodes), u0 = t0 + (t0 >= v ? 1u : 0u);
                const uint32_t b0 = u0 >> kTallyShift;
                t.tgt[atomicAdd(&tpos[b0], 1u)] = (TallyTarget)(u0 & ((1u << kTallyShift) - 1u));
                if (tok > 1) {
                    const uint32_t t1 = scale_draw(px.y, a.nodes), u1 = t1 + (t1 >= v ? 1u : 0u);
                    const uint32_t b1 = u1 >> kTallyShift;
                    t.tgt[atomicAdd(&tpos[b1], 1u)] = (TallyTarget)(u1 & ((1u << kTallyShift) - 1u));
                }
            }
        }
    }
}

// The receipts of actors v0 .. v0+3 in round r (the draws of k_gs_full4), one emit(u) each.
template <class F>
__device__ __forceinline__ void gs_draws4(const RoundArgs& a, uint32_t r, uint32_t v0, uint32_t st4, uint32_t na,
                                          F&& emit) {
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t v = v0 + j, tok = (st4 >> (8u * j)) & 3u;
        if (tok && v < na) {
            const uint4 px = philox(v, r, kStreamGossip, a.seed);
            const uint32_t t0 = scale_draw(px.x, a.nodes);
            emit(t0 + (t0 >= v ? 1u : 0u));
            if (tok > 1) {
                const uint32_t t1 = scale_draw(px.y, a.nodes);
                emit(t1 + (t1 >= v ? 1u : 0u));
            }
        }
    }
}

// Exclusive scan of one u32 per thread over a workgroup of NT threads (wsum: NT / 64 words).
template <uint32_t NT>
__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t x, uint32_t* wsum, uint32_t* total = nullptr) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= (uint32_t)off) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (uint32_t i = 0; i < NT / 64; ++i) {
        if (i < w) base += wsum[i];
        all += wsum[i];
    }
    __syncthreads();
    if (total) *total = all;
    return base + inc - x;
}

// Tallied round, batched placement: a workgroup of kScatK x 256 threads places the receipts of
// k_gs_full4's workgroups kScatK*s .. kScatK*s + kScatK - 1, one after another (their segments of
// every bucket are adjacent; the first starts at the bucket's start, scanned here from
// k_tally_rows' row totals, plus that row's prefix).  k_gs_full4 counted each workgroup's receipts
// per bucket (cnt), so when they fit in LDS their bucket starts in LDS are known and the draws are
// made once: each receipt goes to its bucket's run in LDS, then consecutive lanes store
// consecutive receipts of a bucket.  A workgroup with more receipts than LDS holds is placed in
// batches of walk iterations, each drawn twice (count, then sort).  The walk of one k_gs_full4
// workgroup is dealt round-robin to the kScatK thread groups.  k_gs_tally_scatter stores each
// receipt where its LDS position falls, one 4-byte store per line: its 98M receipts per C4 peak
// round wrote 2.94 GB (7.5x the receipt bytes, profiles/round3/c4_tally/pmc_scatter.txt).
constexpr uint32_t kScatK = 4;
constexpr uint32_t kScatBlock = kScatK * kBlock;
constexpr uint32_t kScatMaxPerIter = kScatBlock * 8u;  // 4 actors x 2 chains per thread
__global__ __launch_bounds__(kScatBlock) void k_gs_tally_scatter_lds(RoundArgs a, GsTally t, uint32_t cap) {
    extern __shared__ uint32_t lds[];
    const uint32_t r = a.r;
    if (!t.on[r & 3u]) return;  // uniform
    const uint32_t nb = t.nb, W = t.W, tid = threadIdx.x;
    uint32_t* tpos = lds;             // next position in each bucket's segment
    uint32_t* hs = lds + nb;          // batch counts -> starts -> ends per bucket
    uint32_t* misc = lds + 2u * nb;   // [0]: batch total; [16, 32): scan wave sums
    uint32_t* S = misc + 32;          // the batch's receipts, bucket-sorted
    // column group sg: consecutive groups on one XCD (workgroups are dealt round-robin to the 8
    // XCDs), so the count and prefix lines they read, and the bucket segments they write next to
    // each other, meet in one L2
    const uint32_t G = W / kScatK;
    const uint32_t sg = (G & 7u) == 0u ? (blockIdx.x & 7u) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    uint4 cw[4];  // receipts of buckets 4 * tid + j from workgroups kScatK*sg + 0..3 (x..w)
    {  // bucket starts: exclusive scan of k_tally_rows' row totals, 4 buckets per thread
        const uint32_t* tot = t.off + (size_t)nb * G;
        uint32_t* bst = t.off + (size_t)nb * G + nb;  // for k_gs_tally_count (workgroup 0 stores it)
        uint32_t v[4], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t b = 4u * tid + j;
            v[j] = b < nb ? tot[b] : 0u;
            cw[j] = b < nb ? *reinterpret_cast<const uint4*>(t.cnt + (size_t)b * W + kScatK * sg)
                           : make_uint4(0u, 0u, 0u, 0u);
            s += v[j];
        }
        uint32_t run = block_excl_scan_n<kScatBlock>(s, misc + 16);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t b = 4u * tid + j;
            if (b < nb) {
                tpos[b] = run + t.off[(size_t)b * G + sg];
                if (sg == 0) bst[b] = run;
            }
            run += v[j];
        }
        if (sg == 0 && tid == kScatBlock - 1u) bst[nb] = run;  // the last thread ends at the total
    }
    // stores a sorted batch of `total` receipts (hs[b]: the end of bucket b's run) and advances tpos
    auto place = [&](uint32_t total) {
        for (uint32_t i = tid; i < total; i += kScatBlock) {
            const uint32_t u = S[i], b = u >> kTallyShift;
            t.tgt[tpos[b] + i - (b ? hs[b - 1u] : 0u)] = (TallyTarget)(u & ((1u << kTallyShift) - 1u));
        }
        __syncthreads();
        for (uint32_t b = tid; b < nb; b += kScatBlock) tpos[b] += hs[b] - (b ? hs[b - 1u] : 0u);
        __syncthreads();
    };
    const uint32_t lt = tid & (kBlock - 1u), g = tid >> 8;
    const uint32_t na = a.hi, nq = (na + 3u) >> 2;
    const uint32_t span4 = (((nq + 7u) >> 3) + kBlock - 1u) / kBlock * kBlock;
    const uint32_t step = (W >> 3) * kBlock;
    const uint32_t iters = (span4 + step - 1u) / step, sup = (iters + kScatK - 1u) / kScatK;
    for (uint32_t k = 0; k < kScatK; ++k) {  // uniform
        // k_gs_full4 workgroup w's walk (node_range, thread lt): its iteration kScatK * i + g is
        // this thread's i-th
        const uint32_t w = tally_wg(kScatK * sg + k, W);
        const uint32_t base = (w & 7u) * span4;
        const uint32_t end = base >= nq ? 0u : (base + span4 < nq ? base + span4 : nq);
        const uint32_t q0 = base + (w >> 3) * kBlock + lt;
        uint32_t v[4], s = 0, all;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            v[j] = k == 0u ? cw[j].x : k == 1u ? cw[j].y : k == 2u ? cw[j].z : cw[j].w;
            s += v[j];
        }
        uint32_t run = block_excl_scan_n<kScatBlock>(s, misc + 16, &all);
        if (t.onepass && all <= cap) {  // one pass: starts from the counts
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                const uint32_t b = 4u * tid + j;
                if (b < nb) hs[b] = run;
                run += v[j];
            }
            __syncthreads();
            for (uint32_t i = 0; i < sup; ++i) {
                const uint32_t q = q0 + (kScatK * i + g) * step;
                if (q < end)
                    gs_draws4(a, r, q << 2, *reinterpret_cast<const uint32_t*>(a.gstate + (q << 2)), na,
                              [&](uint32_t u) { S[atomicAdd(&hs[u >> kTallyShift], 1u)] = u; });
            }
            __syncthreads();
            place(all);
            continue;
        }
        for (uint32_t it = 0; it < sup;) {  // counted batches (uniform)
            for (uint32_t i = tid; i < nb; i += kScatBlock) hs[i] = 0u;
            if (tid == 0) misc[0] = 0u;
            __syncthreads();
            uint32_t it1 = it, total = 0;
            do {  // count: add iterations while one more cannot overflow S
                const uint32_t q = q0 + (kScatK * it1 + g) * step;
                uint32_t c = 0;
                if (q < end)
                    gs_draws4(a, r, q << 2, *reinterpret_cast<const uint32_t*>(a.gstate + (q << 2)), na, [&](uint32_t u) {
                        atomicAdd(&hs[u >> kTallyShift], 1u);
                        ++c;
                    });
                c = wave_sum(c);
                if ((tid & 63u) == 0) atomicAdd(&misc[0], c);
                ++it1;
                __syncthreads();
                total = misc[0];
                __syncthreads();
            } while (it1 < sup && total + kScatMaxPerIter <= cap);
            {  // starts: exclusive scan of the counts, 4 buckets per thread (nb <= 4 * kScatBlock)
                uint32_t c[4], cs = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t b = 4u * tid + j;
                    c[j] = b < nb ? hs[b] : 0u;
                    cs += c[j];
                }
                uint32_t crun = block_excl_scan_n<kScatBlock>(cs, misc + 16);
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t b = 4u * tid + j;
                    if (b < nb) hs[b] = crun;
                    crun += c[j];
                }
            }
            __syncthreads();
            for (uint32_t i = it; i < it1; ++i) {  // sort: the same draws, placed by bucket
                const uint32_t q = q0 + (kScatK * i + g) * step;
                if (q < end)
                    gs_draws4(a, r, q << 2, *reinterpret_cast<const uint32_t*>(a.gstate + (q << 2)), na,
                              [&](uint32_t u) { S[atomicAdd(&hs[u >> kTallyShift], 1u)] = u; });
            }
            __syncthreads();
            place(total);
            it = it1;
        }
    }
}

// Tallied round: one workgroup per target bucket counts its receipts in LDS and writes the
// bucket's whole range of t.inc16, zeros included, so nothing is left to clear: 16-bit words (half
// the bytes here and in F(r + 1); a count from t.esc up escapes to the 32-bit word).  Its 128 KB of
// LDS admit one workgroup per CU: 1024 threads keep that many in flight.
constexpr uint32_t kCountBlock = 1024;
__global__ __launch_bounds__(kCountBlock) void k_gs_tally_count(RoundArgs a, GsTally t, const uint32_t* bst) {
    extern __shared__ uint32_t h[];
    if (!t.on[a.r & 3u]) return;  // uniform
    constexpr uint32_t S = 1u << kTallyShift;
    for (uint32_t i = threadIdx.x; i < S; i += kCountBlock) h[i] = 0u;
    __syncthreads();
    const uint32_t b = blockIdx.x;
    // bucket starts: k_gs_tally_scatter_lds's (bst) or the full scan's
    const uint32_t s0 = bst ? bst[b] : t.off[b * t.W], s1 = bst ? bst[b + 1u] : t.off[(b + 1u) * t.W];
    for (uint32_t i = s0 + threadIdx.x; i < s1; i += kCountBlock) atomicAdd(&h[(uint32_t)t.tgt[i] & (S - 1u)], 1u);
    __syncthreads();
    const uint32_t base = b << kTallyShift, na = a.hi;
    const uint32_t n = na - base < S ? na - base : S;
    const uint32_t esc = t.esc;
    for (uint32_t i = threadIdx.x; i < n; i += kCountBlock) {
        const uint32_t c = h[i];
        t.inc16[base + i] = (uint16_t)(c < esc ? c : esc);
        if (c >= esc) a.inc_cur[base + i] = c;
    }
}

// Push-sum on any topology (used for "full"): messages are bucketed by destination with an
// integer atomic (slot order is arbitrary), then each receiver visits its bucket in ascending
// source order (selection by repeated minimum; buckets hold ~1 entry), so the fp64 sum is the
// canonical one.
__global__ __launch_bounds__(kBlock) void k_ps_push_emit(RoundArgs a) {
    if (gate(a, a.r)) return;
    const uint32_t r = a.r;
    uint32_t v, end, step;
    node_range(a.lo, a.hi, a.span, v, end, step);
    uint32_t newly = 0;
    for (; v < end; v += step) {
        uint32_t m;
        const uint32_t d = generic_deg(a, v, m);
        if (!d) continue;
        uint8_t f = a.flags[v];
        double ss = 0.0, ww = 0.0;
        uint32_t cin = 0;
        if (r) {
            const uint32_t n = a.bcnt_prev[v];
            if (n) {
                const uint32_t o = a.boff_prev[v];
                long long last = -1;
                for (uint32_t i = 0; i < n; ++i) {
                    uint32_t best = 0xFFFFFFFFu;
                    for (uint32_t j = 0; j < n; ++j) {
                        const uint32_t s = a.slot_prev[o + j];
                        if ((long long)s > last && s < best) best = s;
                    }
                    const double2 mm = a.msg_prev[best];
                    ss += mm.x;
                    ww += mm.y;
                    last = best;
                }
                cin = n;
                a.bcnt_prev[v] = 0;  // bucket consumed; buffer is reused two rounds later
            }
        }
        double2 held;
        if (!(f & 16u)) held = r ? a.msg_prev[v] : make_double2((double)v, 1.0);
        const uint8_t f0 = f;
        const PsOut o = ps_update(f, held, ss, ww, cin, a.delta, a.term_limit);
        uint32_t t = 0xFFFFFFFFu;
        if (o.send) {
            const uint4 x = philox(v, r, kStreamPush, a.seed);
            t = generic_target(a, v, m, scale_draw(x.x, d));
            a.msg_cur[v] = o.msg;
            a.pos_cur[v] = atomicAdd(&a.bcnt_cur[t], 1u);
        }
        a.tgt_cur[v] = t;
        if (f != f0) a.flags[v] = f;
        if (o.conv_now) {
            a.frozen[v] = o.msg;
            ++newly;
        }
    }
    block_add(newly, a.parts, r);
}

__global__ __launch_bounds__(kBlock) void k_ps_push_fill(RoundArgs a, uint32_t* slot_cur, const uint32_t* boff_cur) {
    unsigned long long prev = 0;  // completion after round r-1 (published by this round's emit)
    if (a.r) prev = a.total[a.r - 1];
    if (prev >= a.target) return;
    uint32_t v, end, step;
    node_range(a.lo, a.hi, a.span, v, end, step);
    for (; v < end; v += step) {
        const uint32_t t = a.tgt_cur[v];
        if (t != 0xFFFFFFFFu) slot_cur[boff_cur[t] + a.pos_cur[v]] = v;
    }
}

// ------------------------------------------------------------------ setup / utility kernels
// ---- extra-link CSR construction (Imp3D, program.fs:309): links recomputed by link_of()
// counts[link_of(u)] += 1 for the senders u in [ulo, uhi)
__global__ void k_dst_count(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t* counts) {
    for (uint32_t u = ulo + blockIdx.x * blockDim.x + threadIdx.x; u < uhi; u += gridDim.x * blockDim.x)
        atomicAdd(&counts[link_of(seed, u, nodes)], 1u);
}

// out[off[t] + k] = u for the senders u in [ulo, uhi) whose destination t lies in [tlo, thi)
// (k from fill[t]: unordered; k_sort_segments restores ascending sources)
__global__ void k_dst_fill(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t tlo, uint32_t thi,
                           const uint32_t* off, uint32_t* fill, uint32_t* out) {
    for (uint32_t u = ulo + blockIdx.x * blockDim.x + threadIdx.x; u < uhi; u += gridDim.x * blockDim.x) {
        const uint32_t t = link_of(seed, u, nodes);
        if (t >= tlo && t < thi) out[off[t] + atomicAdd(&fill[t], 1u)] = u;
    }
}

__global__ void k_add_u32(uint32_t* x, const uint32_t* y, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] += y[i];
}

// lpos[u] = base[t] + (p - off[t]) for every position p of destination t's list of senders:
// a sender's global CSR slot = its destination's first slot + the senders before it
__global__ void k_lpos_lists(const uint32_t* off, const uint32_t* list, uint32_t nt, const uint32_t* base, uint32_t* lpos) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x)
        for (uint32_t p = off[t]; p < off[t + 1]; ++p) lpos[list[p]] = base[t] + (p - off[t]);
}

__global__ void k_slot_owner(const uint32_t* off, uint32_t lo, uint32_t hi, uint32_t* dst) {
    for (uint32_t v = lo + blockIdx.x * blockDim.x + threadIdx.x; v < hi; v += gridDim.x * blockDim.x)
        for (uint32_t s = off[v]; s < off[v + 1]; ++s) dst[s] = v;
}

__global__ void k_sort_segments(const uint32_t* off, uint32_t* vals, uint32_t n) {
    for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const uint32_t b = off[v], e = off[v + 1];
        for (uint32_t i = b + 1; i < e; ++i) {  // insertion sort; segments are short
            const uint32_t x = vals[i];
            uint32_t j = i;
            while (j > b && vals[j - 1] > x) {
                vals[j] = vals[j - 1];
                --j;
            }
            vals[j] = x;
        }
    }
}

constexpr uint32_t kScanPer = 8;
constexpr uint32_t kScanTile = kBlock * kScanPer;

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t& total) {
    __shared__ uint32_t wsum[kBlock / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= (uint32_t)off) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
#pragma unroll
    for (uint32_t i = 0; i < kBlock / 64; ++i) {
        if (i < w) base += wsum[i];
        total += wsum[i];
    }
    __syncthreads();
    return base + inc - x;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* in, uint32_t n, uint32_t* sums,
                                                         const uint32_t* gate) {
    if (gate && !*gate) return;
    const uint32_t b0 = blockIdx.x * kScanTile;
    uint32_t s = 0;
    for (uint32_t i = threadIdx.x; i < kScanTile; i += kBlock) {
        const uint32_t k = b0 + i;
        if (k < n) s += in[k];
    }
    uint32_t total;
    block_excl_scan(s, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(kBlock) void k_scan_top(uint32_t* sums, uint32_t nb, const uint32_t* gate) {
    if (gate && !*gate) return;
    uint32_t carry = 0;
    for (uint32_t b = 0; b < nb; b += kBlock) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t x = i < nb ? sums[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan(x, total);
        if (i < nb) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ __launch_bounds__(kBlock) void k_scan_apply(const uint32_t* in, uint32_t* off, uint32_t n,
                                                        const uint32_t* sums, const uint32_t* gate) {
    if (gate && !*gate) return;
    const uint32_t b0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint32_t vals[kScanPer];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
        const uint32_t k = b0 + j;
        vals[j] = k < n ? in[k] : 0u;
        s += vals[j];
    }
    uint32_t total;
    uint32_t run = sums[blockIdx.x] + block_excl_scan(s, total);
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
        const uint32_t k = b0 + j;
        if (k < n) off[k] = run;
        run += vals[j];
        if (k + 1 == n) off[n] = run;
    }
}

// Tallied round, batched placement: the part of the scan k_gs_tally_scatter_lds reads.  One
// workgroup per bucket row of cnt stores the row's prefix at each scatter workgroup's first column
// (off[b * G + s], G = W / kScatK) and the row total (off[nb * G + b]); the scatter workgroups scan
// the nb totals themselves.  One pass reading cnt once, in place of the reduce / top / apply scan
// of all nb * W counts (two reads and a whole write of cnt, profiles/round4/tally_rows).
constexpr uint32_t kRowP = ((uint32_t)kMaxGrid / kScatK + kBlock - 1u) / kBlock;
__global__ __launch_bounds__(kBlock) void k_tally_rows(GsTally t, const uint32_t* gate) {
    if (!*gate) return;
    const uint32_t b = blockIdx.x, G = t.W / kScatK, P = (G + kBlock - 1u) / kBlock;
    const uint4* row = reinterpret_cast<const uint4*>(t.cnt + (size_t)b * t.W);
    const uint32_t g0 = threadIdx.x * P;
    uint32_t v[kRowP], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < kRowP; ++j) {
        v[j] = 0u;
        if (j < P && g0 + j < G) {
            const uint4 q = row[g0 + j];
            v[j] = q.x + q.y + q.z + q.w;
        }
        s += v[j];
    }
    uint32_t total;
    uint32_t run = block_excl_scan(s, total);
    uint32_t* o = t.off + (size_t)b * G;
#pragma unroll
    for (uint32_t j = 0; j < kRowP; ++j) {
        if (j < P && g0 + j < G) o[g0 + j] = run;
        run += v[j];
    }
    if (threadIdx.x == 0) t.off[(size_t)t.nb * G + b] = total;
}

__global__ void k_fill_u8(uint8_t* p, uint8_t val, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = val;
}


// total[a] from the round-a sub-counters; with `out`, also total[first .. a] into out[0 ..
// a - first] (host-mapped memory: the host reads the batch's counts without a copy).
// total[b0 .. a] from the sub-counters (b0 < a: the rounds of the last launch of a batch that ran
// several, k_ps_tile), one wave, the running count carried in registers
__global__ void k_finalize(unsigned long long* total, uint32_t* parts, long long a, unsigned long long* out,
                           long long first, long long b0) {
    unsigned long long x = b0 >= 1 ? total[b0 - 1] : 0ull;
    for (long long b = b0; b <= a; ++b) {
        unsigned long long y = *part_slot(parts, b, threadIdx.x);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) y += __shfl_xor(y, off, 64);
        x += y;
        if (threadIdx.x == 0) total[b] = x;
    }
    if (b0 < a) __threadfence();  // (lane 0's totals, read back below by other lanes)
    if (out)
        for (long long i = threadIdx.x; first + i <= a; i += 64) out[i] = first + i == a ? x : total[first + i];
}

__global__ void k_ps_init(uint8_t* flags, Geom g, uint32_t lo, uint32_t hi, uint32_t full, uint32_t term_init) {
    for (uint32_t v = lo + blockIdx.x * blockDim.x + threadIdx.x; v < hi; v += gridDim.x * blockDim.x) {
        const bool part = full ? true : presence(g, v) != 0u;
        flags[v] = part ? (uint8_t)term_init : (uint8_t)0;  // termRound = 1 (program.fs:79)
    }
}

// Held + in-flight (s, w) per block (fixed-order partials; the host adds them in order).
__global__ __launch_bounds__(kBlock) void k_ps_sums(RoundArgs a, uint32_t valid, double2* partials) {
    __shared__ double2 red[kBlock];
    double s = 0.0, w = 0.0;
    for (uint32_t v = a.lo + blockIdx.x * kBlock + threadIdx.x; v < a.hi; v += gridDim.x * kBlock) {
        uint32_t m;
        if (!generic_deg(a, v, m)) continue;
        const uint8_t f = a.flags[v];
        double2 held = make_double2((double)v, 1.0);
        if (f & 16u) held = a.frozen[v];
        else if (valid) held = a.msg_prev[v];
        s += held.x;
        w += held.y;
        if (valid) {
            const bool sent = a.dir_prev ? a.dir_prev[v] != kDirNone : a.tgt_cur[v] != 0xFFFFFFFFu;
            if (sent) {
                const double2 mm = a.msg_prev[v];
                s += mm.x;
                w += mm.y;
            }
        }
    }
    red[threadIdx.x] = make_double2(s, w);
    __syncthreads();
    for (int k = kBlock / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) {
            red[threadIdx.x].x += red[threadIdx.x + k].x;
            red[threadIdx.x].y += red[threadIdx.x + k].y;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = red[0];
}

}  // namespace

// ------------------------------------------------------------------ launchers
int grid_for(uint32_t n) {
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    blocks = (blocks + 7u) & ~7u;  // a multiple of 8: one group per XCD
    if (blocks < 8) blocks = 8;
    return (int)(blocks < (uint32_t)kMaxGrid ? blocks : (uint32_t)kMaxGrid);
}

uint32_t span_for(uint32_t n, int grid) {
    (void)grid;
    uint32_t s = (n + 7u) / 8u;
    return (s + kBlock - 1) / kBlock * kBlock;
}

// The quiet-wave kernel's grid: the workgroups resident at once (GP_PSQ_PER_CU per CU; 7 with the
// SGPR cap), unless the node range needs fewer.
#ifndef GP_PSQ_PER_CU
#define GP_PSQ_PER_CU 7
#endif
static int quiet_grid(const Launch& l) { return l.grid < 256 * GP_PSQ_PER_CU ? l.grid : 256 * GP_PSQ_PER_CU; }
static int quiet_grid_x(const Launch& l) { return l.grid < 256 * GP_PSQX_PER_CU ? l.grid : 256 * GP_PSQX_PER_CU; }

void launch_ps_tiny(const RoundArgs& a, int nk, hipStream_t s) {
    hipLaunchKernelGGL(k_ps_tiny, dim3(1), dim3(kTinyBlock), 0, s, a, (uint32_t)nk);
}

void launch_gs_tiny(const RoundArgs& a, int nk, hipStream_t s) {
    hipLaunchKernelGGL(k_gs_tiny, dim3(1), dim3(kTinyBlock), 0, s, a, (uint32_t)nk);
}

void launch_ps_tile(const RoundArgs& a, const TileArgs& t, int nr, hipStream_t s) {
    const int boxes = (int)((a.g.actors + kTileSeg - 1) / kTileSeg);
    static_assert(kTileMaxNR == 8, "one instantiation per round count");
    switch (nr) {
        case 8: hipLaunchKernelGGL(k_ps_tile<8>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 7: hipLaunchKernelGGL(k_ps_tile<7>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 6: hipLaunchKernelGGL(k_ps_tile<6>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 5: hipLaunchKernelGGL(k_ps_tile<5>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 4: hipLaunchKernelGGL(k_ps_tile<4>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 3: hipLaunchKernelGGL(k_ps_tile<3>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        case 2: hipLaunchKernelGGL(k_ps_tile<2>, dim3(boxes), dim3(kBlock), 0, s, a, t); break;
        default: hipLaunchKernelGGL(k_ps_tile<1>, dim3(boxes), dim3(kBlock), 0, s, a, t);
    }
}

void launch_ps_pull(const RoundArgs& a, const Launch& l, const Xchg* x) {
    constexpr unsigned lds = 0;
    const bool q = a.act_cur != nullptr;
    if (!a.g.has_link) {
        if (q) hipLaunchKernelGGL((k_ps_quiet<0>), dim3(quiet_grid(l)), dim3(kBlock), lds, l.stream, a);
        else hipLaunchKernelGGL((k_ps_pull<0, false>), dim3(l.grid), dim3(kBlock), lds, l.stream, a);
    } else if (a.rmsg_prev && !a.sharded) {  // one GPU, small graph: link messages by slot
        hipLaunchKernelGGL((k_ps_pull<3, false>), dim3(l.grid), dim3(kBlock), lds, l.stream, a);
    } else if (a.lref_prev) {  // a push-sum shard (slot references)
        if (q && x->hin) hipLaunchKernelGGL(k_ps_quiet_x<true>, dim3(quiet_grid(l)), dim3(kBlock), lds, l.stream, a, *x);
        else if (q) hipLaunchKernelGGL(k_ps_quiet_x<false>, dim3(quiet_grid_x(l)), dim3(kBlock), lds, l.stream, a, *x);
        else hipLaunchKernelGGL((k_ps_pull<2, false>), dim3(l.grid), dim3(kBlock), lds, l.stream, a);
    } else if (q) {
        hipLaunchKernelGGL((k_ps_quiet<1>), dim3(quiet_grid(l)), dim3(kBlock), lds, l.stream, a);
    } else {
        hipLaunchKernelGGL((k_ps_pull<1, false>), dim3(l.grid), dim3(kBlock), lds, l.stream, a);
    }
}

void launch_gs_pull(const RoundArgs& a, const Launch& l) {
    const bool e = gs_pull_early(a);
    if (a.g.has_link && e) hipLaunchKernelGGL((k_gs_pull<true, true>), dim3(l.grid), dim3(kBlock), 0, l.stream, a);
    else if (a.g.has_link) hipLaunchKernelGGL((k_gs_pull<true, false>), dim3(l.grid), dim3(kBlock), 0, l.stream, a);
    else if (e) hipLaunchKernelGGL((k_gs_pull<false, true>), dim3(l.grid), dim3(kBlock), 0, l.stream, a);
    else hipLaunchKernelGGL((k_gs_pull<false, false>), dim3(l.grid), dim3(kBlock), 0, l.stream, a);
}

// Flat grids (one actor per thread): a grid-stride loop would make each iteration's load wait
// behind the previous iteration's scattered store.
void launch_link_count(const RoundArgs& a, const Launch& l) {
    hipLaunchKernelGGL(k_link_count, dim3((a.g.wired + kScatterPer * kBlock - 1) / (kScatterPer * kBlock)), dim3(kBlock), 0, l.stream, a);
}

void launch_ps_push_emit(const RoundArgs& a, const Launch& l) {
    hipLaunchKernelGGL(k_ps_push_emit, dim3(l.grid), dim3(kBlock), 0, l.stream, a);
}

void launch_ps_push_fill(const RoundArgs& a, uint32_t* slot_cur, const uint32_t* boff_cur, const Launch& l) {
    hipLaunchKernelGGL(k_ps_push_fill, dim3(l.grid), dim3(kBlock), 0, l.stream, a, slot_cur, boff_cur);
}

void launch_gs_sparse(const RoundArgs& a, const GsTally& t, const GsSparse& sp, const Launch& l) {
    hipLaunchKernelGGL(k_gs_sparse, dim3(l.grid), dim3(kBlock), 0, l.stream, a, t, sp);
}

void launch_gs_full4(const RoundArgs& a, const GsTally& t, const Launch& l) {
    const unsigned lds = t.cnt ? t.nb * (unsigned)sizeof(uint32_t) : 0u;
    hipLaunchKernelGGL(k_gs_full4, dim3(t.cnt ? t.W : (uint32_t)l.grid), dim3(kBlock), lds, l.stream, a, t);
}

// Batched placement (k_gs_tally_scatter_lds) where its 160 KB of LDS can be allowed, else one store
// per receipt (k_gs_tally_scatter, after the full scan).
constexpr uint32_t kScatLdsBytes = 160u * 1024u;  // one workgroup per CU
bool g_scatter_lds = false;

int prepare_gs_tally() {
    // the per-bucket tally keeps 32768 u32 counters (128 KB) in LDS
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gs_tally_count), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)((1u << kTallyShift) * sizeof(uint32_t))) != hipSuccess)
        return -1;
    g_scatter_lds =
                    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gs_tally_scatter_lds),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScatLdsBytes) == hipSuccess;
    (void)hipGetLastError();
    return 0;
}

void launch_gs_tally(const RoundArgs& a, const GsTally& t, const Launch& l) {
    if (!t.cnt || !a.r) return;
    const uint32_t* gate = t.on + (a.r & 3u);
    const uint32_t cap = kScatLdsBytes / 4u - 2u * t.nb - 32u;
    const uint32_t* bst = nullptr;
    if (g_scatter_lds && t.W % kScatK == 0 && t.W <= (uint32_t)kMaxGrid && t.nb <= 4u * kScatBlock &&
        cap >= kScatMaxPerIter) {
        hipLaunchKernelGGL(k_tally_rows, dim3(t.nb), dim3(kBlock), 0, l.stream, t, gate);
        hipLaunchKernelGGL(k_gs_tally_scatter_lds, dim3(t.W / kScatK), dim3(kScatBlock), kScatLdsBytes, l.stream, a, t, cap);
        bst = t.off + (size_t)t.nb * (t.W / kScatK) + t.nb;
    } else {
        const uint32_t n = t.nb * t.W, nb = (n + kScanTile - 1) / kScanTile;
        hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kBlock), 0, l.stream, t.cnt, n, t.scratch, gate);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, l.stream, t.scratch, nb, gate);
        hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(kBlock), 0, l.stream, t.cnt, t.off, n, t.scratch, gate);
        hipLaunchKernelGGL(k_gs_tally_scatter, dim3(t.W), dim3(kBlock), t.nb * (unsigned)sizeof(uint32_t), l.stream, a, t);
    }
    hipLaunchKernelGGL(k_gs_tally_count, dim3(t.nb), dim3(kCountBlock), (1u << kTallyShift) * (unsigned)sizeof(uint32_t),
                       l.stream, a, t, bst);
}

void launch_gs_push(const RoundArgs& a, const Launch& l) {
    hipLaunchKernelGGL(k_gs_push, dim3(l.grid), dim3(kBlock), 0, l.stream, a);
}

static unsigned scatter_blocks(const RoundArgs& a) {
    const uint32_t n = a.hi < a.g.wired ? a.hi : a.g.wired;
    return n > a.lo ? (n - a.lo + kShardPer * kBlock - 1) / (kShardPer * kBlock) : 0u;
}

void launch_ps_link_scatter_x(const RoundArgs& a, const Xchg& x, const Launch& l) {
    if (const unsigned b = scatter_blocks(a)) hipLaunchKernelGGL(k_ps_link_scatter_x, dim3(b), dim3(kBlock), 0, l.stream, a, x);
}

void launch_gs_link_scatter_x(const RoundArgs& a, const Xchg& x, const Launch& l) {
    if (const unsigned b = scatter_blocks(a)) hipLaunchKernelGGL(k_gs_link_scatter_x, dim3(b), dim3(kBlock), 0, l.stream, a, x);
}

void launch_shard_done_out(const RoundArgs& a, const Xchg& x, hipStream_t s) {
    const uint32_t nw = ((a.hi - 1u) >> 5) - (a.lo >> 5) + 1u;
    uint32_t blocks = (nw + kBlock - 1) / kBlock;
    blocks = blocks > 1024u ? 1024u : blocks;
    hipLaunchKernelGGL(k_shard_done_out, dim3(blocks), dim3(kBlock), 0, s, a, x);
}

void launch_gs_full4x(const RoundArgs& a, const Xchg& x, const Launch& l) {
    hipLaunchKernelGGL(k_gs_full4x, dim3(l.grid), dim3(kBlock), 0, l.stream, a, x);
}

int prepare_gs_bins() {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_shard_unpack_bins), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)((1u << kTallyShift) * sizeof(uint32_t))) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return 0;
}

void launch_gs_bins(const RoundArgs& a, const Xchg& x, const GsBins& b, hipStream_t s) {
    const unsigned lds = b.nbt * (unsigned)sizeof(uint32_t);
    hipLaunchKernelGGL(k_gs_bins_count, dim3(b.W), dim3(kBlock), lds, s, a, x, b);
    launch_exclusive_scan(b.cnt, b.off, b.nbt * b.W, b.scratch, s);
    hipLaunchKernelGGL(k_gs_bins_place, dim3(b.W), dim3(kBlock), lds, s, a, x, b);
}

void launch_shard_unpack_bins(const RoundArgs& a, const Xchg& x, const GsBins& b, hipStream_t s) {
    if (!b.nb_self) return;
    hipLaunchKernelGGL(k_shard_unpack_bins, dim3(b.nb_self), dim3(kBinBlock), (1u << kTallyShift) * (unsigned)sizeof(uint32_t),
                       s, a, x, b);
}

void launch_gs_sparse_x(const RoundArgs& a, const Xchg& x, const GsSparse& sp, long long applied, const Launch& l) {
    hipLaunchKernelGGL(k_gs_sparse_x, dim3(l.grid), dim3(kBlock), 0, l.stream, a, x, sp, applied);
}

void launch_shard_halo(const RoundArgs& a, const Xchg& x, int pushsum, hipStream_t s) {
    const uint32_t n = x.h.out_n[0] > x.h.out_n[1] ? x.h.out_n[0] : x.h.out_n[1];
    if (!n) return;
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    blocks = blocks > (uint32_t)kMaxGrid ? (uint32_t)kMaxGrid : blocks;
    hipLaunchKernelGGL(k_shard_halo, dim3(blocks), dim3(kBlock), 0, s, a, x, pushsum);
}

void launch_shard_pack(const RoundArgs& a, const Xchg& x, long long applied, hipStream_t s) {
    hipLaunchKernelGGL(k_shard_pack, dim3(1), dim3(kBlock), 0, s, a, x, applied);
}

void launch_shard_unpack(const RoundArgs& a, const Xchg& x, long long applied, uint32_t max_entries, int gossip,
                         int full, const GsSparse& sp, hipStream_t s) {
    const uint32_t cap = (uint32_t)kMaxGrid / x.world;
    uint32_t bpp = (max_entries + kBlock - 1) / kBlock;
    bpp = bpp < 1u ? 1u : (bpp > cap ? cap : bpp);
    hipLaunchKernelGGL(k_shard_unpack, dim3(bpp * x.world), dim3(kBlock), 0, s, a, x, applied, gossip, full, sp);
}

void launch_link_hist(uint64_t seed, const Geom& g, const HistBounds& b, unsigned long long* hist, const Launch& l) {
    hipLaunchKernelGGL(k_link_hist, dim3(l.grid), dim3(kBlock), 0, l.stream, seed, g, b, hist);
}

void launch_dst_count(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t* counts, const Launch& l) {
    if (uhi > ulo) hipLaunchKernelGGL(k_dst_count, dim3(l.grid), dim3(kBlock), 0, l.stream, seed, nodes, ulo, uhi, counts);
}

void launch_dst_fill(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t tlo, uint32_t thi,
                     const uint32_t* off, uint32_t* fill, uint32_t* out, const Launch& l) {
    if (uhi > ulo)
        hipLaunchKernelGGL(k_dst_fill, dim3(l.grid), dim3(kBlock), 0, l.stream, seed, nodes, ulo, uhi, tlo, thi, off, fill, out);
}

void launch_add_u32(uint32_t* x, const uint32_t* y, uint32_t n, const Launch& l) {
    hipLaunchKernelGGL(k_add_u32, dim3(l.grid), dim3(kBlock), 0, l.stream, x, y, n);
}

void launch_lpos_lists(const uint32_t* off, const uint32_t* list, uint32_t nt, const uint32_t* base, uint32_t* lpos,
                       const Launch& l) {
    hipLaunchKernelGGL(k_lpos_lists, dim3(l.grid), dim3(kBlock), 0, l.stream, off, list, nt, base, lpos);
}

void launch_slot_owner(const uint32_t* off, uint32_t lo, uint32_t hi, uint32_t* dst, const Launch& l) {
    if (hi > lo) hipLaunchKernelGGL(k_slot_owner, dim3(l.grid), dim3(kBlock), 0, l.stream, off, lo, hi, dst);
}

void launch_sort_segments(const uint32_t* off, uint32_t* vals, uint32_t n, const Launch& l) {
    hipLaunchKernelGGL(k_sort_segments, dim3(l.grid), dim3(kBlock), 0, l.stream, off, vals, n);
}

size_t scan_scratch_words(uint32_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

void launch_exclusive_scan(const uint32_t* in, uint32_t* off, uint32_t n, uint32_t* scratch, hipStream_t s) {
    const uint32_t nb = (n + kScanTile - 1) / kScanTile;
    if (nb == 0) return;
    const uint32_t* gate = nullptr;
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kBlock), 0, s, in, n, scratch, gate);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kBlock), 0, s, scratch, nb, gate);
    hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(kBlock), 0, s, in, off, n, scratch, gate);
}

// Empty kernel launched once by gp_create: the runtime loads the library's code object at its first
// kernel launch (~1.5 ms), which must not fall inside the first gp_step's timed rounds.
__global__ void k_load() {}

int launch_load(hipStream_t s) {
    hipLaunchKernelGGL(k_load, dim3(1), dim3(64), 0, s);
    return hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

void launch_fill_u8(uint8_t* p, uint8_t v, size_t n, hipStream_t s) {
    size_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > (size_t)kMaxGrid) blocks = kMaxGrid;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_fill_u8, dim3((unsigned)blocks), dim3(kBlock), 0, s, p, v, n);
}


void launch_finalize(unsigned long long* total, uint32_t* parts, long long a, hipStream_t s, unsigned long long* out,
                     long long first, bool pairs) {
    // (pairs: the last launch's earlier rounds have no total yet either)
    const long long b0 = pairs ? std::max(a - (long long)kTileMaxNR + 1, 0ll) : a;
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, total, parts, a, out, first, b0);
}

void launch_ps_init(uint8_t* flags, const Geom& g, uint32_t lo, uint32_t hi, uint32_t full, uint32_t term_init,
                    const Launch& l) {
    hipLaunchKernelGGL(k_ps_init, dim3(l.grid), dim3(kBlock), 0, l.stream, flags, g, lo, hi, full, term_init);
}

void launch_ps_sums(const RoundArgs& a, uint32_t valid, double2* partials, const Launch& l) {
    hipLaunchKernelGGL(k_ps_sums, dim3(l.grid), dim3(kBlock), 0, l.stream, a, valid, partials);
}

}  // namespace gp
