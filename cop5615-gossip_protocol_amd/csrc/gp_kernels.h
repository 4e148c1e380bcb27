// gp_kernels.h — parameter blocks and launchers of the gfx950 round kernels (gp_kernels.hip).
#pragma once
#include "gp_common.h"

namespace gp {

constexpr int kBlock = 256;       // 4 waves of 64
// Grid cap: 256 CUs x GP_GRID_PER_CU workgroups, grid-stride beyond that (A/B knob).
#ifndef GP_GRID_PER_CU
#define GP_GRID_PER_CU 16
#endif
constexpr int kMaxGrid = 256 * GP_GRID_PER_CU;
// Waves per SIMD the push-sum round kernel is compiled for (VGPR budget 512 / waves; A/B knob,
// 7 ties, 8 spills and is 20% slower).
#ifndef GP_PS_WAVES
#define GP_PS_WAVES 6
#endif
constexpr int kParts = 64;          // completion sub-counters per round (one 64 B line each)
constexpr int kPartStride = 16;     // u32 words between sub-counters
constexpr int kPartRing = 32;       // rounds kept in the sub-counter ring (k_ps_tile uses 24 at once)
constexpr int kWorkStride = 8;      // u64 words between the walked-actor sub-counters
constexpr int kMaxWorld = 16;
constexpr int kMaxPieces = 4;       // a shard's round in at most this many pieces
// Exchange entries to one peer are appended into kSub sub-segments (sub = blockIdx % kSub), each
// with its own counter on its own 128 B line: same-address atomics serialise in L2 (measured at
// 8 loopback shards: one counter per peer cost 8.5 ms per round).
constexpr uint32_t kSub = 16;
constexpr uint32_t kCtrStride = 32;  // u32 words between counters
// Full gossip's done-word shipping state (Xchg::dstat), one 128 B line each: the dirty-word counter of
// the round (k_shard_done_out adds, the pack reads and zeroes), the backlog flag (words left dirty
// after a capped round) and the last round's dirty count (read by the host at a sync).
constexpr uint32_t kDstatCount = 0, kDstatLeft = 32, kDstatWords = 64;
// The per-round plan's inputs the host reads at a sync, in one 256-byte array (Xchg::pstat, u32 words):
// every rank's chains of the last round delivered (u64), this rank's dirty done words of that round,
// and per peer its largest sub-segment sent (pack), received (unpack, from the header) and the peer's
// dirty words (unpack).
constexpr uint32_t kPsChains = 0, kPsDirty = 2, kPsOut = 16, kPsIn = 32, kPsDwIn = 48, kPstatWords = 64;
static_assert(kPsOut + kMaxWorld <= kPsIn && kPsDwIn + kMaxWorld <= kPstatWords, "pstat layout");

// Single-GPU Imp3D push-sum: the round kernel writes the link marks of its own messages (no
// k_link_count pass; 1% faster than the separate pass at 10M).
constexpr bool kFuseLinkMarks = true;

// Push-sum link-slot marks carry their round: the pass after F(r) writes link_tag(r) into the
// CSR slot of every actor whose round-r message took its extra link, into the array of parity
// r & 1; F(r+1) reads a slot as fired iff it holds link_tag(r).  One array sees 255 distinct
// tags before a value repeats, and it is cleared (hipMemsetAsync) right before that happens
// (tag_clear_round), so no consumer ever clears a slot and no stale mark can match.
__host__ __device__ inline uint8_t link_tag(uint32_t r) { return (uint8_t)((r >> 1) % 255u + 1u); }
__host__ __device__ inline bool tag_clear_round(uint32_t r) { return r >= 2u && (r >> 1) % 255u == 0u; }
// A push-sum shard's link slots hold 32-bit references instead: the round tag in
// the low kRefShift bits (ref_tag, 31 values, the same ping-pong rule, cleared every 62 rounds) and,
// for a remote sender's message, its 16-byte index in the receive buffer of the exchange that
// delivered it (the pull reads it there).
constexpr uint32_t kRefShift = 5, kRefTagMask = (1u << kRefShift) - 1u;
__host__ __device__ inline uint32_t ref_tag(uint32_t r) { return (r >> 1) % kRefTagMask + 1u; }
__host__ __device__ inline bool ref_clear_round(uint32_t r) { return r >= 2u && (r >> 1) % kRefTagMask == 0u; }

// One synchronous round kernel F(r) fuses phase 2 of round r-1 (collect the messages sent to
// this actor, read from the round r-1 buffers) with phase 1 of round r (update, convergence
// test, emit).  Buffers ping-pong on r & 1.
struct RoundArgs {
    Geom g;
    uint64_t seed;
    uint32_t lo, hi;       // actors this kernel updates: [0, actors), a shard's node range, or one piece
                           // of it when a shard's round runs in pieces
    uint32_t tag_prev;     // link_tag(r - 1): marks of the messages collected by F(r)
    uint32_t tag_cur;      // link_tag(r): marks written for the messages F(r) emits
    uint32_t slot_lo;      // first link slot held here (0, or the shard's first): the in-bounds
                           // fallback index of predicated-off link-slot loads
    uint32_t sharded;      // completion counts come from the exchange (total[] is global)
    uint32_t r;            // round index
    uint32_t target;       // completion target T = nodes (program.fs:178, AllNodes)
    uint32_t full;         // full topology (implicit k + (k >= v) neighbour map)
    uint32_t nodes;        // `nodes` (full topology degree)
    uint32_t span;         // per-XCD contiguous node range (XCD-aware block mapping)
    // The rank's own actors [olo, ohi) (= [lo, hi) unless the launch walks one piece): which sources
    // are remote, which targets a shard marks itself.
    uint32_t olo, ohi;
    union {  // gossip | push-sum (a handle runs one algorithm; the kernel arguments stay small)
        uint32_t threshold;  // gossip report threshold (program.fs:102)
        uint32_t act_thr;    // quiet-wave marks kept from this many converged actors (below)
    };
    double delta;          // push-sum delta (program.fs:187)
    uint32_t term_limit;   // program.fs:135
    uint32_t ps_tags;      // push-sum: link marks are round tags (link_tag); gossip: chain counts
    unsigned long long* total;  // total[a] = completion count after round a (trace)
    uint32_t* parts;            // kPartRing x kParts padded sub-counters of newly reported actors
    uint32_t* cparts;           // full gossip shards: the same ring for the chains emitted in round r
                                // (F(r) adds, the pack of round r reads; null: not counted)
    // topology side data (Imp3D)
    const uint32_t* rev_off;  // CSR of link sources per destination, ascending
    const uint32_t* rev_src;
    const uint32_t* lpos;     // CSR slot of v's own link edge: rev_src[lpos[v]] == v
    // Link marks per CSR slot, written by k_link_count or the exchange (ping-pong on r & 1):
    // gossip: the chains that took the link (emptied by the receiver); push-sum: link_tag(r)
    // when the sender's round-r message took it (the receiver then reads msg_prev[u]; a
    // shard's remote sender's message is written into rmsg by the exchange).
    uint8_t* lcnt_prev;
    uint8_t* lcnt_cur;
    // push-sum shards: the slots' 32-bit references (kRefShift above), ref_tag(r - 1) / ref_tag(r),
    // and the receive buffer of round r - 1's exchange (the remote messages F(r) reads, 16 bytes each)
    const uint32_t* lref_prev;
    uint32_t* lref_cur;
    uint32_t rtag_prev, rtag_cur;
    const double2* rin_prev;
    // push-sum state
    const double2* msg_prev;  // message emitted in round r-1 (= held S,W when not converged)
    double2* msg_cur;
    // small one-GPU graphs (LM 3): every link message by CSR slot
    const double2* rmsg_prev;
    double2* rmsg_cur;
    const uint8_t* dir_prev;  // direction code of that message (kDirNone: none)
    uint8_t* dir_cur;
    uint8_t* flags;           // termRound (bits 0-3) | converged (bit 4)
    double2* frozen;          // (S,W) frozen at convergence (program.fs:125-127)
    // gossip state
    union {
        struct {  // gossip state
            uint32_t* cnt;     // messageCount (program.fs:75)
            uint8_t* gstate;   // tok (bits 0-1) | done (bit 2)
        };
        // Quiet-wave skipping (one GPU, push-sum): act_cur[w] = link_tag(r + 1) when the 64 actors
        // of wave w may have work in round r + 1 (one of them has not converged, or a round-r
        // message targets one of them); written by F(r) once act_thr actors have converged, read
        // by F(r + 1).
        struct {
            const uint8_t* act_prev;  // marks for this round (written by F(r - 1)); null: off
            uint8_t* act_cur;
        };
    };
    uint32_t* dbits;          // full gossip, one GPU: done bitmap (sender-side filter)
    uint32_t* dsum;           // its summary: bit w set once word w of dbits is all ones
    uint32_t* inc_prev;       // generic path: receipts of round r-1 (atomics)
    uint32_t* inc_cur;
    // generic push-sum buckets (ping-pong)
    uint32_t* bcnt_prev;      // messages per destination
    const uint32_t* boff_prev;  // exclusive scan of bcnt
    const uint32_t* slot_prev;  // source ids grouped by destination (unordered inside)
    uint32_t* bcnt_cur;
    uint32_t* tgt_cur;        // destination of v's message (UINT32_MAX none)
    uint32_t* pos_cur;        // slot of v's message inside its destination bucket
    // kernel statistics (GP_FLAG_KERNEL_TIMING, one-GPU quiet kernel): actors walked, summed over
    // launches into kParts sub-counters kWorkStride apart (one per workgroup slot: a single
    // counter serialised 1792 atomics per round); null: not counted
    unsigned long long* work;
};

// Shard exchange (gp_shard_*).  Send chunk to peer q (built by this rank) and receive chunk from
// peer q (built by q for this rank) share one layout: a 256-byte header; when q is a z-neighbour
// (rank +-1) the halo face: the direction bytes of the face plane, then (push-sum) kSub x `hcap`
// halo entries, u32 face offsets then (s, w) pairs, for the messages that cross the face only;
// then kSub x `cap` link entries: u32 slot (global link-CSR slot; gossip: slot | (chains-1) << 31;
// full gossip: the target actor), then push-sum (s, w) pairs.  See DESIGN.md §6.
struct ShardHeader {
    unsigned long long newly;  // actors that reported in the round (sender's range)
    uint32_t overflow;         // sender dropped entries: the run is void (GP_EOVERFLOW) unless a
                               // checkpoint restores it (activity tiers, gp_api.cpp)
    uint32_t runmax;           // the sender's most link entries in one sub-segment of its chunk to
                               // this peer, over the rounds since the plan was last chosen: both
                               // ends size the next batch's chunk from it
    uint32_t nlinks[kSub];     // link entries written per sub-segment (<= cap)
    uint32_t nhalo[kSub];      // halo entries written per sub-segment (<= hcap)
    // full gossip
    uint32_t chains;           // activation chains the sender's actors emitted in the round
    uint32_t ndone;            // done part: (index, word) pairs written, or (whole-word plan) 1 when
                               // the words were written, 0 when no word changed
    uint32_t dwant;            // the sender's own done words that differed from what it had shipped
                               // (before the pair capacity): both ends size the next done parts from it
    uint32_t binned;           // full gossip: the receipts travel in bins (GsBins below), not as entries
};
static_assert(sizeof(ShardHeader) <= 256, "the chunk header is 256 bytes");

struct PeerOut {
    ShardHeader* hdr;
    uint32_t* slot;
    double2* msg;
    uint32_t cap;
    uint32_t dpairs;  // full gossip: the done part holds up to dpairs (index, word) pairs; 0: every word
    uint32_t* done;   // full gossip: the sender's done-bitmap words (its range) or pairs, or null
};

struct PeerIn {
    const ShardHeader* hdr;
    const uint32_t* slot;
    const double2* msg;
    uint32_t cap;
    uint32_t dpairs;
    const uint32_t* done;
};

// The halo faces of a shard, side 0 = rank-1 (this rank's first plane / the halo below lo),
// side 1 = rank+1 (last plane / the halo from hi).  n == 0: no such neighbour.
struct HaloX {
    uint32_t out_first[2], out_n[2], out_cap[2];  // face actors sent (global ids), entries per sub-segment
    uint32_t in_first[2], in_n[2], in_cap[2];     // halo rows received
    uint32_t code[2];                             // direction code that crosses the face
    uint8_t* out_dir[2];
    uint32_t* out_slot[2];
    double2* out_msg[2];
    const ShardHeader* in_hdr[2];
    const uint8_t* in_dir[2];
    const uint32_t* in_slot[2];
    const double2* in_msg[2];
};

struct Xchg {
    uint32_t world, rank;
    uint32_t last;                 // the round's last piece: its headers carry the
                                   // round's count (pack), its unpack publishes total[applied]
    uint32_t hin;                  // push-sum tail round: the round kernel writes the halo faces
                                   // (k_ps_quiet_x<true>; k_shard_halo is not launched)
    const char* rbase;             // the receive buffer (the unpack's message references count from it)
    uint32_t abnd[kMaxWorld + 1];  // actor range of every rank
    uint32_t sbnd[kMaxWorld + 1];  // link-slot range of every rank (global CSR numbering)
    uint32_t* pcount;              // entry counters of the current round, (peer, sub) then (world +
                                   // halo side, sub), kCtrStride apart (zeroed by pack)
    uint32_t* overflow;            // sticky local overflow flag
    unsigned long long* self_newly;  // this rank's count of the round (pack -> unpack)
    uint32_t* pmax;                // [kMaxWorld] running max of link entries per sub-segment to each
                                   // peer (reset when the host chooses the plan)
    const uint32_t* slot_dst;      // push-sum, quiet tail: the receiver of each own link slot (the
                                   // unpack marks the segment of a remote link message's receiver)
    // full gossip: the per-round plan's inputs
    unsigned long long* self_chains;  // this rank's chains of the round (pack -> unpack)
    uint32_t* pstat;                  // [kPstatWords] the plan inputs of the last round (-> host; kPs*)
    uint32_t* dship;                  // own done words as last shipped (global word index)
    uint32_t* dstat;                  // [kDstatWords]: dirty-word counter, backlog flag
    uint32_t binned;                  // full gossip: this round's receipts travel in bins (GsBins)
    uint32_t* fin;                    // push-sum, tail rounds: workgroups of k_ps_quiet_x<true> finished, per
                                      // group ([1 + g] * kFinStride) and groups finished ([0]); the last one
                                      // packs the headers (0 between launches)
    PeerOut out[kMaxWorld];
    PeerIn in[kMaxWorld];
    HaloX h;
};

struct Launch {
    int grid;
    hipStream_t stream;
};

int grid_for(uint32_t n);
uint32_t span_for(uint32_t n, int grid);

// Quiet-wave marks: one byte per segment of kActSeg actors.  4: C3 -8%, 100M -4% against 16
// (profiles/round3/tail_ab); one mark per actor with 1024-actor compaction was slower than 4
// (scattered actors cost their own lines).  The compacted walk lists 64 / kActSeg segments per pass
// (a power of two below 64: k_ps_quiet's tail walk).
constexpr uint32_t kActShift = 2;
constexpr uint32_t kActSeg = 1u << kActShift;
static_assert(kActSeg >= 2u && kActSeg < 64u, "segments of 2 .. 32 actors");

// round kernels
void launch_ps_pull(const RoundArgs& a, const Launch& l, const Xchg* x = nullptr);  // x: a shard of several ranks
// Small one-GPU line grids (line / 2D push-sum): one launch runs rounds r .. r + nr - 1
// (nr <= kTileMaxNR) of a segment of kTileSeg actors: round r + q over the segment and nr - 1 - q
// actors either side of it, round r from round r - 1's state of the segment and nr actors either side
// (loaded into LDS), each later round from the one before in LDS.  Round k's state is in buffer
// [k mod kTileBufs] (round -1's: the last): a launch reads one buffer and writes nr others.
constexpr uint32_t kTileMaxNR = 8, kTileBufs = kTileMaxNR + 1;
struct TileArgs {
    double2* msg[kTileBufs];
    uint8_t* dir[kTileBufs];
    uint8_t* flg[kTileBufs];
};
constexpr uint32_t kTileSeg = 256 - 2 * kTileMaxNR, kTileLoad = kTileSeg + 2 * kTileMaxNR;
void launch_ps_tile(const RoundArgs& a, const TileArgs& t, int nr, hipStream_t s);
// Gossip on tiny graphs (generic path, one GPU): nk rounds F(r) .. F(r + nk - 1) in one workgroup's LDS
constexpr uint32_t kTinyActors = 8192, kTinyBlock = 1024;
void launch_gs_tiny(const RoundArgs& a, int nk, hipStream_t s);
// ... and push-sum (generic path): the buckets by destination rebuilt in LDS every round
constexpr uint32_t kTinyPsActors = 2048;
void launch_ps_tiny(const RoundArgs& a, int nk, hipStream_t s);
void launch_gs_pull(const RoundArgs& a, const Launch& l);
// Gossip grid rounds on graphs below 2^18 actors (one GPU) issue their level-1 loads ahead of
// the gate: k_gs_pull<LINK, true>.  (At 1M actors the unconditional loads cost more than the
// latency they hide: profiles/round2/ab_round_kernel.md.)
inline bool gs_pull_early(const RoundArgs& a) { return !a.sharded && a.hi - a.lo < (1u << 18); }
void launch_link_count(const RoundArgs& a, const Launch& l);
void launch_ps_push_emit(const RoundArgs& a, const Launch& l);
void launch_ps_push_fill(const RoundArgs& a, uint32_t* slot_cur, const uint32_t* boff_cur, const Launch& l);
void launch_gs_push(const RoundArgs& a, const Launch& l);
// Full gossip on one GPU: receipt tally by target bucket.  In a round that follows
// one with at least `thr` emitted chains, k_gs_full4 counts its receipts per (target bucket,
// workgroup) in LDS instead of adding each with a memory-side atomic; a scan of those counts, a
// scatter of the receipts by bucket (the draws recomputed) and an LDS tally per bucket then write
// inc_cur whole.  Receipts to done targets are not filtered there (the receiver drops them).
constexpr uint32_t kTallyShift = 15;          // 32768 targets per bucket: 128 KB of LDS counters
typedef uint16_t TallyTarget;                 // a placed receipt: its target's offset in the bucket
constexpr uint32_t kMaxTallyBuckets = 4096;   // k_gs_full4's LDS counters: 16 KB at most
#ifndef GP_TALLY_LATE_DIV
#define GP_TALLY_LATE_DIV 64  // A/B knob; 0: no late tally
#endif
constexpr uint64_t kTallyLateDiv = GP_TALLY_LATE_DIV;  // also tally (filter on) while >= 1/64 of the nodes are not done
struct GsTally {
    uint32_t* cnt;     // [nb * W] receipts per (bucket, workgroup), bucket-major; null: no tally
    uint32_t* off;     // [nb * W + 1] exclusive scan of cnt
    TallyTarget* tgt;  // receipts grouped by bucket (2 per actor at most): the target's offset in
                       // its bucket (16 bits: 32768 targets per bucket)
    uint32_t* scratch; // scan scratch (scan_scratch_words(nb * W))
    uint32_t* chains;  // [4][kParts * kPartStride]: chains emitted in round r, ring slot r & 3
    uint32_t* on;      // [4]: round r tallies (written by block 0 of F(r))
    uint16_t* inc16;   // [actors] receipts of the last tallied round; a word holding esc: the count
                       // is in that round's 32-bit receipt word
    uint32_t thr;      // tally in round r >= 1 when round r - 1 emitted at least thr chains to
                       // targets not done yet (estimated from the share of nodes not done)
    uint32_t nb, W;    // buckets; k_gs_full4's grid
    // the live fallbacks (GP_FLAG_TALLY_FALLBACKS forces both; the same results either way):
    uint32_t esc;      // 16-bit receipt words escape to the 32-bit word from this count on (0xFFFF;
                       // the test hook: 1, every nonzero count)
    uint32_t onepass;  // the placement draws once when a workgroup's receipts fit LDS (1), else in
                       // counted batches (the test hook: 0, counted batches everywhere)
};
void launch_gs_full4(const RoundArgs& a, const GsTally& t, const Launch& l);  // full gossip, one GPU (lo == 0)
// Full gossip's ramp on one GPU: while few actors hold a chain, F(r) walks lists instead
// of every actor — the receipt targets of round r - 1 (apply; a first receipt starts a chain) and the
// chain holders (emit).  Every receipt lists its target for F(r + 1) (a target listed twice is applied
// once); a first receipt appends its actor to the holders.  The host runs these rounds while a bound on the holder count (a
// chain starts only on a first receipt, so holders at most double per round) keeps every list within
// cap; later rounds run k_gs_full4.  ctr: u32 words kSpStride apart, [field][round & 3]: holders before
// the round (0), holders added by it (1), receipt targets it listed (2).
// On shards (k_gs_sparse_x) the lists hold this rank's actors; the bound is on every rank's holders
// (the global chain count of the exchange headers), and a remote peer's receipts are listed by the
// unpack (k_shard_unpack, a first receipt of this rank's actor).
struct GsSparse {
    uint32_t* hl;     // chain holders (the leader first), 2 cap + kSpSlack
    uint32_t* tl[2];  // receipt targets of round r, list r & 1
    uint32_t* ctr;
    uint32_t* err;    // a list would have overflowed (the host fails the step)
    uint32_t cap;     // a round runs here only if its holders and last round's targets are <= cap
    uint32_t h0;      // holders before round 0: 1 (the leader), on a shard 0 where another rank holds it
    uint32_t* fin;    // shards: blocks of k_gs_sparse_x finished (its last block runs the done-word pass
                      // and the pack; 0 between launches)
};
constexpr uint32_t kSpStride = 32, kSpSlack = 1024;
// A push-sum shard's dense round kernel (k_ps_quiet_x) routes its own link messages through LDS, and
// k_ps_link_scatter_x is not launched (gp_kernels.hip, FuseStage).
#ifndef GP_SHARD_FUSE
#define GP_SHARD_FUSE 1
#endif
constexpr bool kShardFuse = GP_SHARD_FUSE != 0;
// A push-sum shard's tail round counts its finished workgroups in kFinGroups groups (one counter per
// 128-byte line) before one counter of groups (Xchg::fin).
constexpr uint32_t kFinGroups = 32, kFinStride = 32;
void launch_gs_sparse(const RoundArgs& a, const GsTally& t, const GsSparse& sp, const Launch& l);
// shards: F(k) on lists, then (its last block) k_shard_done_out's and k_shard_pack's work for round k
void launch_gs_sparse_x(const RoundArgs& a, const Xchg& x, const GsSparse& sp, long long applied, const Launch& l);
// full gossip on shards: this rank's done-bitmap words into every peer's chunk (after F(k))
void launch_shard_done_out(const RoundArgs& a, const Xchg& x, hipStream_t s);
// the scan, scatter and tally passes of a tallied round (each exits at once otherwise)
void launch_gs_tally(const RoundArgs& a, const GsTally& t, const Launch& l);
int prepare_gs_tally();  // once per process: allow the tally pass's 128 KB of dynamic LDS (0: ok)
// Full gossip on shards, the receipt wave: the remote receipts of a round travel
// binned by target, bin b of peer q holding q's actors [abnd[q] + b * 2^kTallyShift, ...).  F(k)
// (k_gs_bins_count) counts them per (peer, bin) and workgroup in LDS, an exclusive scan gives every
// (peer, bin, workgroup) its place, and k_gs_bins_place draws the same receipts again into their places,
// as u16 offsets in the bin.  The chunk's entry part then holds the bins' starts (nb + 1 u32 words,
// nb = the receiver's bins) and the u16 entries.  The rank's own receipts take the same way into a
// chunk of its own (`self`), so the receiver counts every receipt of a bin per workgroup in LDS and
// writes its receipt words whole (k_shard_unpack_bins): no fabric atomics anywhere, 2 bytes a receipt.
// No sender-side done filter in these rounds: F(k + 1) drops the receipts of done actors itself.
struct GsBins {
    uint32_t* cnt;                 // [nbt][W]: receipts per (rank, bin) and workgroup (tally_col order)
    uint32_t* off;                 // its exclusive scan, nbt * W + 1 words
    uint32_t* scratch;             // the scan's scratch
    uint32_t* self;                // the own receipts' chunk: nb_self + 1 starts, then u16 entries
    uint32_t self_words;           // its size (room for one receipt per own actor: "full" holds one chain)
    uint32_t W;                    // grid of k_gs_bins_count / k_gs_bins_place (a multiple of 8)
    uint32_t nbt;                  // bins over every rank (this one's too)
    uint32_t nb_self;              // bins of this rank's range (the receiver's grid)
    uint32_t bin0[kMaxWorld + 1];  // first bin of each rank, bin0[world] = nbt
};
constexpr uint32_t kMaxBins = 8192;  // the passes' LDS counters (u32 per bin)
int prepare_gs_bins();               // once per process: the receiver's 128 KB of dynamic LDS (0: ok)
// F(k) in bins: k_gs_bins_count, the scan, k_gs_bins_place (the chunks' entry parts)
void launch_gs_bins(const RoundArgs& a, const Xchg& x, const GsBins& b, hipStream_t s);
// after the exchange: every peer's bins of this rank into inc_cur (one workgroup per bin)
void launch_shard_unpack_bins(const RoundArgs& a, const Xchg& x, const GsBins& b, hipStream_t s);
// sharded variants: remote link / full-topology messages go to the send chunks of x
void launch_ps_link_scatter_x(const RoundArgs& a, const Xchg& x, const Launch& l);
void launch_gs_link_scatter_x(const RoundArgs& a, const Xchg& x, const Launch& l);
void launch_gs_full4x(const RoundArgs& a, const Xchg& x, const Launch& l);  // full gossip, shards
// halo faces of F(k) into the send chunks of rank +-1: direction bytes, crossing push-sum messages
void launch_shard_halo(const RoundArgs& a, const Xchg& x, int pushsum, hipStream_t s);
// headers of round `applied` (-1: none) into every send chunk; zero the per-peer counters
void launch_shard_pack(const RoundArgs& a, const Xchg& x, long long applied, hipStream_t s);
// total[applied] from the headers; halo faces into the halo rows of dir_cur / msg_cur; link
// entries into msg_cur + lcnt_cur / lcnt_cur / inc_cur (full gossip with sp.hl: every receipt also
// lists its target in sp.tl[r & 1], the round ran on lists)
void launch_shard_unpack(const RoundArgs& a, const Xchg& x, long long applied, uint32_t max_cap, int gossip,
                         int full, const GsSparse& sp, hipStream_t s);
// per-(source piece, destination rank, degree) counts of extra links, for the exchange plan: sb[0..ns]
// the source pieces' actor bounds (every rank's pieces in order), db[0..nd] the ranks'
struct HistBounds {
    uint32_t sb[kMaxWorld * kMaxPieces + 1], db[kMaxWorld + 1];
    uint32_t ns, nd;
};
void launch_link_hist(uint64_t seed, const Geom& g, const HistBounds& b, unsigned long long* hist, const Launch& l);

// setup / utility kernels
// extra-link CSR construction (links recomputed by link_of)
void launch_dst_count(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t* counts, const Launch& l);
void launch_dst_fill(uint64_t seed, uint32_t nodes, uint32_t ulo, uint32_t uhi, uint32_t tlo, uint32_t thi,
                     const uint32_t* off, uint32_t* fill, uint32_t* out, const Launch& l);
void launch_add_u32(uint32_t* x, const uint32_t* y, uint32_t n, const Launch& l);
void launch_sort_segments(const uint32_t* off, uint32_t* vals, uint32_t n, const Launch& l);
// dst[s] = v for every slot s of the CSR segments of actors [lo, hi)
void launch_slot_owner(const uint32_t* off, uint32_t lo, uint32_t hi, uint32_t* dst, const Launch& l);
void launch_lpos_lists(const uint32_t* off, const uint32_t* list, uint32_t nt, const uint32_t* base, uint32_t* lpos,
                       const Launch& l);
// exclusive scan of n u32 counts into off[0..n]; scratch >= scan_scratch_words(n) u32
size_t scan_scratch_words(uint32_t n);
void launch_exclusive_scan(const uint32_t* in, uint32_t* off, uint32_t n, uint32_t* scratch, hipStream_t s);
void launch_fill_u8(uint8_t* p, uint8_t v, size_t n, hipStream_t s);
int launch_load(hipStream_t s);  // load the code object now (an empty kernel, synchronised): 0 ok
// total[a] = total[a-1] + sum of the round-a sub-counters (after the last kernel of a batch)
// (out: also total[first .. a] into out[], e.g. host-mapped memory)
// pairs (k_ps_tile): total[a - 1] may be unwritten (round a - 1 was a launch's first round)
void launch_finalize(unsigned long long* total, uint32_t* parts, long long a, hipStream_t s,
                     unsigned long long* out = nullptr, long long first = 0, bool pairs = false);
void launch_ps_init(uint8_t* flags, const Geom& g, uint32_t lo, uint32_t hi, uint32_t full, uint32_t term_init,
                    const Launch& l);
// push-sum sums for gp_status: per-block partials of held + in-flight (s, w)
void launch_ps_sums(const RoundArgs& a, uint32_t last_round_valid, double2* partials, const Launch& l);

}  // namespace gp
