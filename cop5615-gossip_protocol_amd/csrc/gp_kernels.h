// gp_kernels.h — parameter blocks and launchers of the gfx950 round kernels (gp_kernels.hip).
#pragma once
#include "gp_common.h"

namespace gp {

constexpr int kBlock = 256;       // 4 waves of 64
constexpr int kMaxGrid = 256 * 16; // 256 CUs x 16 workgroups: grid-stride beyond that
constexpr int kParts = 64;          // completion sub-counters per round (one 64 B line each)
constexpr int kPartStride = 16;     // u32 words between sub-counters
constexpr int kPartRing = 4;        // rounds kept in the sub-counter ring
// empty link slot: w holds this quiet-NaN bit pattern (a real weight is finite and >= 0)
constexpr unsigned long long kEmptySlot = 0x7FF800000000DEADull;

// One synchronous round kernel F(r) fuses phase 2 of round r-1 (collect the messages sent to
// this actor, read from the round r-1 buffers) with phase 1 of round r (update, convergence
// test, emit).  Buffers ping-pong on r & 1.
struct RoundArgs {
    Geom g;
    uint64_t seed;
    uint32_t r;            // round index
    uint32_t target;       // completion target T = nodes (program.fs:178, AllNodes)
    uint32_t full;         // full topology (implicit k + (k >= v) neighbour map)
    uint32_t nodes;        // `nodes` (full topology degree)
    uint32_t span;         // per-XCD contiguous node range (XCD-aware block mapping)
    uint32_t threshold;    // gossip report threshold (program.fs:102)
    double delta;          // push-sum delta (program.fs:187)
    uint32_t term_limit;   // program.fs:135
    uint32_t ablate;       // DEBUG ONLY (env GP_ABLATE): bits skip work for cost attribution; results invalid
    unsigned long long* total;  // total[a] = completion count after round a (trace)
    uint32_t* parts;            // kPartRing x kParts padded sub-counters of newly reported actors
    // topology side data (Imp3D)
    const uint32_t* link;     // extra link per wired node (program.fs:309)
    const uint32_t* rev_off;  // CSR of link sources per destination, ascending
    const uint32_t* rev_src;
    const uint32_t* lpos;     // CSR slot of v's own link edge: rev_src[lpos[v]] == v
    // extra-link messages are PUSHED by the sender into its CSR slot (ping-pong); the receiver
    // scans its slots in order and empties what it consumed (push-sum: w = kEmptySlot NaN;
    // gossip: a u8 chain count set back to 0).
    uint8_t* lcnt_prev;
    uint8_t* lcnt_cur;
    double2* lmsg_prev;
    double2* lmsg_cur;
    // push-sum state
    const double2* msg_prev;  // message emitted in round r-1 (= held S,W when not converged)
    double2* msg_cur;
    const uint8_t* dir_prev;  // direction code of that message (kDirNone: none)
    uint8_t* dir_cur;
    uint8_t* flags;           // termRound (bits 0-3) | converged (bit 4)
    double2* frozen;          // (S,W) frozen at convergence (program.fs:125-127)
    // gossip state
    uint32_t* cnt;            // messageCount (program.fs:75)
    uint8_t* gstate;          // tok (bits 0-1) | done (bit 2)
    uint32_t* inc_prev;       // generic path: receipts of round r-1 (atomics)
    uint32_t* inc_cur;
    // generic push-sum buckets (ping-pong)
    uint32_t* bcnt_prev;      // messages per destination
    const uint32_t* boff_prev;  // exclusive scan of bcnt
    const uint32_t* slot_prev;  // source ids grouped by destination (unordered inside)
    uint32_t* bcnt_cur;
    uint32_t* tgt_cur;        // destination of v's message (UINT32_MAX none)
    uint32_t* pos_cur;        // slot of v's message inside its destination bucket
};

struct Launch {
    int grid;
    hipStream_t stream;
};

int grid_for(uint32_t n);
uint32_t span_for(uint32_t n, int grid);

// round kernels
void launch_ps_pull(const RoundArgs& a, const Launch& l);
void launch_gs_pull(const RoundArgs& a, const Launch& l);
void launch_ps_link_scatter(const RoundArgs& a, const Launch& l);
void launch_gs_link_scatter(const RoundArgs& a, const Launch& l);
void launch_ps_push_emit(const RoundArgs& a, const Launch& l);
void launch_ps_push_fill(const RoundArgs& a, uint32_t* slot_cur, const uint32_t* boff_cur, const Launch& l);
void launch_gs_push(const RoundArgs& a, const Launch& l);

// setup / utility kernels
void launch_links(uint32_t* link, uint32_t nodes, uint64_t seed, const Launch& l);
void launch_count(const uint32_t* idx, uint32_t n, uint32_t* counts, const Launch& l);
void launch_rev_fill(const uint32_t* link, uint32_t nodes, const uint32_t* rev_off, uint32_t* fillc,
                     uint32_t* rev_src, const Launch& l);
void launch_sort_segments(const uint32_t* off, uint32_t* vals, uint32_t n, const Launch& l);
void launch_lpos(const uint32_t* rev_src, uint32_t nlinks, uint32_t* lpos, const Launch& l);
// exclusive scan of n u32 counts into off[0..n]; scratch >= scan_scratch_words(n) u32
size_t scan_scratch_words(uint32_t n);
void launch_exclusive_scan(const uint32_t* in, uint32_t* off, uint32_t n, uint32_t* scratch, hipStream_t s);
void launch_fill_u8(uint8_t* p, uint8_t v, size_t n, hipStream_t s);
void launch_fill_empty_slots(double2* p, size_t n, hipStream_t s);
// total[a] = total[a-1] + sum of the round-a sub-counters (after the last kernel of a batch)
void launch_finalize(unsigned long long* total, uint32_t* parts, long long a, hipStream_t s);
void launch_ps_init(uint8_t* flags, const Geom& g, uint32_t full, uint32_t term_init, const Launch& l);
// push-sum sums for gp_status: per-block partials of held + in-flight (s, w)
void launch_ps_sums(const RoundArgs& a, uint32_t last_round_valid, double2* partials, const Launch& l);

}  // namespace gp
