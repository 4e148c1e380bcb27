/*
 * gossip_hip.h — C ABI of libgossip_hip.so, the MI355X (gfx950) gossip / push-sum engine.
 *
 * The reference (/root/reference/program.fs) has no FFI layer: its hot path is fused into the
 * ChildActor closure (program.fs:74-147), the ParentActor (program.fs:38-67) and the top-level
 * `match topology` builders (program.fs:150-331).  This ABI is the seam those pieces are cut
 * at.  Each entry point names the reference code it replaces.
 *
 * Conventions
 *   - plain C, cdecl, blittable POD structs, no C++/torch types;
 *   - return 0 on success, a negative GP_E* code on failure; gp_last_error() describes it;
 *   - the library owns every device buffer and its HIP stream (or uses cfg->stream);
 *     callers own the host buffers passed to gp_read_*;
 *   - one host thread per handle; a handle is not re-entrant.
 *
 * Flag / state encodings shared with the tests and the CPU oracle:
 *   gossip   flags: bits 0-1 = activation chains (tok, 0..2), bit 2 = done (reported)
 *   push-sum flags: bits 0-3 = termRound, bit 4 = converged (alreadyConverged)
 */
#ifndef GOSSIP_HIP_H
#define GOSSIP_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP_ABI_VERSION 8

/* program.fs:151 "line", :191 "full", :227 "2D", :267 "Imp3D"; "3D" is build-defined (Q9) */
enum gp_topology { GP_LINE = 0, GP_FULL = 1, GP_TWO_D = 2, GP_IMP3D = 3, GP_THREE_D = 4 };
/* program.fs:177 "gossip", :183 "push-sum" */
enum gp_algo { GP_GOSSIP = 0, GP_PUSHSUM = 1 };

enum gp_error {
    GP_OK = 0,
    GP_EINVAL = -1, /* bad argument / unsupported combination            */
    GP_ENOMEM = -2, /* device or host allocation failed                  */
    GP_EHIP = -3,   /* a HIP runtime call failed                         */
    GP_ESTATE = -4, /* call not valid in the handle's current state      */
    GP_EOVERFLOW = -5, /* a shard's fixed-capacity message buffer overflowed (results void) */
    GP_ERCCL = -6,  /* an RCCL call failed (num_gpus > 1)                  */
};

enum gp_flags {
    GP_FLAG_KERNEL_TIMING = 1, /* hipEvent kernel timing (gp_kernel_stats): gp_step brackets groups of 64 rounds (or every 8th kernel when a pass follows it); a shard brackets every 8th round */
    GP_FLAG_GENERIC = 2,       /* force the generic bucketed push path on grid topologies    */
    GP_FLAG_USE_STREAM = 4,    /* run on cfg->stream even when it is NULL (the null stream)  */
    GP_FLAG_ONE_DEVICE = 8,    /* num_gpus > 1: every shard on cfg->device, exchange by device
                                  copies on one stream (tests the multi-GPU engine on one GPU) */
    GP_FLAG_GROUP = 16,        /* use the multi-GPU engine (shards + RCCL) also at num_gpus = 1 */
    GP_FLAG_QUIET_WAVES = 32,  /* push-sum, one GPU: skip quiet waves at any graph
                                  size (default: from 2^20 actors on); a test hook, same results */
    GP_FLAG_GOSSIP_TALLY = 64, /* full gossip, one GPU: tally receipts by target bucket in every
                                  round from round 1 at any graph size (default: from 2^20 actors,
                                  after a round with many chains); full-gossip shards (ABI 8): send
                                  the receipts in bins in every round from round 1 that does not
                                  run on the ramp's lists (default: the receipt wave); a test hook,
                                  same results */
    GP_FLAG_FULL_PLAN = 128,   /* push-sum and full-gossip shards: keep the full exchange plan (no
                                  activity tiers, no per-round plans) */
    GP_FLAG_TIGHT_TIERS = 256, /* push-sum and full-gossip shards: sized plans from the first batch
                                  with no headroom and a restore point at every sync, so reduced
                                  chunks overflow and batches replay often (full gossip: done words
                                  also wait for a later round); a test hook, same results */
    GP_FLAG_TALLY_FALLBACKS = 512, /* full gossip, one GPU, receipt tally: run the paths a large
                                  graph takes only at extreme counts, everywhere: the counted-batch
                                  placement (a workgroup's receipts past its LDS) and the 32-bit
                                  escape of the 16-bit receipt words (counts >= 0xFFFF); a test
                                  hook, same results */
    GP_FLAG_PIECES = 1024,     /* push-sum shards: the host exchanges each round piece by piece
                                  (gp_shard_round_piece / gp_shard_plan_piece), so the exchange of
                                  one piece overlaps the next piece's kernels; the library runs 4
                                  pieces when every rank holds 2^25 actors or more, until half the
                                  nodes have converged, else 1 (gp_shard_pieces, re-read after
                                  every gp_shard_sync).  The library's own group
                                  (num_gpus > 1) runs pieces always under GP_FLAG_ONE_DEVICE and
                                  across devices only with this flag (ABI 8) */
    GP_FLAG_FORCE_PIECES = 2048, /* with GP_FLAG_PIECES: 4 pieces at any size (whole z-planes, or
                                  256 actors on line / 2D, permitting); a test hook, same results */
    GP_FLAG_ONE_ROUND = 4096,    /* one GPU: one round per launch, also where the library batches
                                  rounds into one launch (push-sum on small line / 2D grids, gossip
                                  on graphs of up to 8192 actors through the generic path); a test
                                  hook, same results */
};

typedef struct gp_config {
    int64_t n_arg;            /* argv[1] (program.fs:19)                                */
    int32_t topology;         /* gp_topology, argv[2] (program.fs:20)                   */
    int32_t algo;             /* gp_algo, argv[3] (program.fs:21)                       */
    uint64_t seed;            /* Philox4x32-10 key; replaces unseeded Random()          */
    double delta;             /* push-sum threshold, program.fs:187 (1e-10)             */
    int32_t gossip_threshold; /* program.fs:102 (10)                                    */
    int32_t term_init;        /* program.fs:79 (1)                                      */
    int32_t term_limit;       /* program.fs:135 (3)                                     */
    int32_t device;           /* HIP device ordinal (the first one when num_gpus > 1)    */
    int32_t flags;            /* gp_flags                                               */
    int32_t num_gpus;         /* 0 or 1: one GPU.  N > 1: one graph split into N node-range
                                 shards on devices device .. device+N-1 inside this process;
                                 the library owns one stream per device and the RCCL
                                 communicators (ncclCommInitAll), and exchanges each round
                                 with grouped ncclSend / ncclRecv     */
    void* stream;             /* hipStream_t to run on; NULL without GP_FLAG_USE_STREAM:
                                 a library-owned stream (ignored when num_gpus > 1)      */
} gp_config;

typedef struct gp_layout {
    int64_t nodes;        /* `nodes` after rounding = completion target (program.fs:27-31,229) */
    int64_t actors;       /* nodes + 1 actors are spawned (program.fs:152,192,233,269)        */
    int64_t grid;         /* G (Imp3D/3D, program.fs:268) or g (2D, program.fs:228); else 0   */
    int64_t leader;       /* program.fs:173/211/250/316                                       */
    int64_t participants; /* actors with at least one neighbour                              */
    int64_t links;        /* Imp3D extra links (program.fs:309), 0 otherwise                   */
    int64_t device_bytes; /* device memory held by the handle                                 */
} gp_layout;

typedef struct gp_status {
    int64_t round;     /* synchronous rounds executed                                     */
    int64_t completed; /* CompletedMessage / PushSumResult count (ParentActor count)       */
    int32_t converged; /* completed >= nodes (program.fs:49,56)                           */
    int32_t pad;
    double sum_s;      /* push-sum: sum of held S plus in-flight s (conservation check)    */
    double sum_w;      /* push-sum: sum of held W plus in-flight w                         */
    double device_ms;  /* wall time of the round loop in this gp_step call (hipEvents)     */
} gp_status;

typedef struct gp_kstats {
    int64_t launches;   /* rounds timed since the last reset                               */
    double total_ms;    /* summed durations of the dominant round kernel                   */
    double avg_ms;      /* total_ms / launches                                             */
    double bytes_per_launch; /* compulsory HBM bytes of one launch of it     */
    char kernel[64];    /* name of the dominant round kernel                               */
    double aux_avg_ms;  /* the pass that completes a round after it (0 if none)            */
    char aux_kernel[64];
    double work_per_launch; /* actor updates one launch of it performs, mean over the rounds run
                               since the last reset: every actor of the range, except that the
                               one-GPU quiet-tail kernel counts the actors it walks (ABI 4)      */
} gp_kstats;

int gp_abi_version(void);

/* Node-count rounding of program.fs:26-31 (Imp3D, G from the raw N at :268) and :228-229 (2D). */
int gp_sizes(int64_t n_arg, int32_t topology, int64_t* nodes, int64_t* actors, int64_t* grid);

/* Replaces the topology builders + actor spawn + InitializeVariables + leader pick
 * (program.fs:150-175, 191-211, 227-252, 267-317).  Builds the implicit topology and the
 * Imp3D extra-link CSR on the device and initialises the protocol state.  With
 * cfg->num_gpus = N > 1 the handle is one graph over N GPUs of this process: gp_step, gp_reset,
 * gp_read_*, gp_kernel_stats and gp_destroy act on all of them (reads may span shards). */
int gp_create(const gp_config* cfg, gp_layout* out, void** handle);

/* Re-initialise protocol state (same topology/links) so a run can be repeated. */
int gp_reset(void* handle);

/* Replaces the actor message loop (ChildActor, program.fs:82-146) and the ParentActor
 * termination count (program.fs:44-63): advance at most max_rounds synchronous rounds, or
 * until completed >= nodes.  device_ms is the round loop's time: hipEvents on one GPU, the
 * host clock around the loop (every GPU drained) for num_gpus > 1. */
int gp_step(void* handle, int64_t max_rounds, gp_status* st);

/* State read-back (the caller owns the host buffers; any pointer may be NULL). */
int gp_read_gossip(void* handle, int64_t first, int64_t count, uint32_t* cnt, uint8_t* flags);
int gp_read_pushsum(void* handle, int64_t first, int64_t count, double* S, double* W, uint8_t* flags);
/* Push-sum messages emitted in the last executed round: dst (UINT32_MAX = none), s, w. */
int gp_read_messages(void* handle, int64_t first, int64_t count, uint32_t* dst, double* s, double* w);
/* Completion count after each round: completed[i] = count after round first_round + i. */
int gp_read_trace(void* handle, int64_t first_round, int64_t count, int64_t* completed);
/* Neighbour list of actor v in the reference's order (program.fs:162-171,201-206,242-248,295-311);
 * returns the degree (writes at most cap entries) or a negative error. */
int gp_neighbors(void* handle, int64_t v, uint32_t* out, int32_t cap);

/* Per-kernel timing collected under GP_FLAG_KERNEL_TIMING; reset=1 clears the counters. */
int gp_kernel_stats(void* handle, gp_kstats* out, int32_t reset);

/* ---------------------------------------------------------------- node-range shards
 * Multi-GPU: one process per GPU, each owning a contiguous actor range of the
 * same global graph.  The reference has no counterpart (its only parallelism is the Akka
 * dispatcher over the .NET thread pool, program.fs:23); these entry points split gp_step
 * (program.fs:82-146 + :44-63) into the per-round pieces around ONE exchange, which the
 * caller performs with any all-to-all (RCCL via torch.distributed on MI355X, gloo on CPU, a
 * device copy for in-process shards).  Every buffer size is fixed at creation, so the
 * exchange needs no per-round size negotiation and the round loop never waits on the host.
 *
 * Per round k:  gp_shard_round(send)  -> caller all-to-all(send -> recv) -> gp_shard_deliver(recv)
 * and every few rounds gp_shard_sync() to learn the global completion count. */

/* Actor range of every rank: bounds[0] = 0 < ... < bounds[world] = actors.  Grid topologies
 * (Imp3D/3D) split on whole z-planes (G*G actors); line/2D/full split evenly. */
int gp_partition(int64_t n_arg, int32_t topology, int32_t world, int64_t* bounds);

typedef struct gp_shard_layout {
    int64_t lo, hi;         /* this rank's actors [lo, hi)                                   */
    int64_t halo;           /* actors exchanged with each z-neighbour rank per round (0: none) */
    int64_t send_total;     /* bytes of the send buffer (sum of send_bytes)                  */
    int64_t recv_total;     /* bytes of the receive buffer                                   */
} gp_shard_layout;

/* Create rank `rank` of `world` (cfg->device is this rank's GPU).  Supported: gossip on every
 * topology, push-sum on line/2D/Imp3D/3D (push-sum on "full" is single-GPU only). */
int gp_create_shard(const gp_config* cfg, int32_t rank, int32_t world, gp_layout* out,
                    gp_shard_layout* shard, void** handle);
/* Per-peer byte counts of the next round's exchange (arrays of `world`; peer order): chunk p -> q is
 * sent_bytes[q] bytes at the running offset of the send buffer, and likewise for the receive
 * buffer.  The buffers are allocated for the full plan (gp_shard_layout send_total / recv_total),
 * and plans only shrink from it:
 *   - push-sum shards size each batch's chunks from the activity of the batch before (activity
 *     tiers: the converged tail ships a fraction of an all-sending round);
 *   - full-gossip shards size every round's chunks (ABI 6): from the chain count, which at most
 *     doubles per round, during the ramp, and from the last round's counts after it.
 * The plan of round k holds from the gp_shard_deliver of round k-1 (or the gp_shard_sync / gp_reset
 * before round k) to the gp_shard_deliver of round k, so a host reads it after every
 * gp_shard_round.  Both ends of a chunk always agree on its size. */
int gp_shard_plan(void* handle, int64_t* send_bytes, int64_t* recv_bytes);
/* Enqueue one round on the handle's stream and pack what other ranks need into send_buf
 * (device memory, send_total bytes, 256-byte aligned).  Asynchronous.  (In pieces: every piece in
 * turn, for a host that exchanges the round's pieces one after another afterwards.) */
int gp_shard_round(void* handle, void* send_buf);
/* A round in pieces (GP_FLAG_PIECES, ABI 6).  gp_shard_pieces: the pieces per round
 * (1: gp_shard_round / gp_shard_plan as above).  Piece i of a round is gp_shard_round_piece(h, send,
 * i), i = 0 .. pieces-1 in order, each followed by its own all-to-all of the per-peer sizes
 * gp_shard_plan_piece gives, at offsets[0] of the send buffer and offsets[1] of the receive buffer
 * (pieces are laid out one after another); the exchange of piece i runs while piece i+1 is computed.
 * gp_shard_deliver follows the last piece's exchange.  gp_shard_plan fails with GP_ESTATE when the
 * round runs in pieces. */
int gp_shard_pieces(void* handle);
int gp_shard_round_piece(void* handle, void* send_buf, int32_t piece);
int gp_shard_plan_piece(void* handle, int32_t piece, int64_t* send_bytes, int64_t* recv_bytes, int64_t* offsets);
/* Enqueue the unpacking of what the other ranks sent for that round (recv_buf: recv_total
 * bytes of device memory, 256-byte aligned).  Must follow each gp_shard_round.  Asynchronous.
 * ABI 7: a push-sum shard's next round reads the remote link messages where they arrived (the slots
 * keep references into recv_buf), so round k's receive buffer must stay unchanged
 * until round k+1's kernels have run: with one piece an exchange that is stream-ordered after
 * gp_shard_round may reuse it; in pieces (where round k+1's exchange overlaps its kernels) the host
 * alternates two buffers — the same buffer twice in a row fails with GP_EINVAL. */
int gp_shard_deliver(void* handle, const void* recv_buf);
/* Wait for the enqueued rounds and fill st from the global completion counts (st->sum_s /
 * sum_w are this rank's share), then choose the next batch's plan (gp_shard_plan).  If a reduced
 * (activity-tier) chunk overflowed in the batch, every rank discards the batch and returns to its
 * restore point: st->round goes back to that round and the host simply runs on from there (the
 * run stays exact).  Fails with GP_EOVERFLOW if a full-plan buffer overflowed. */
int gp_shard_sync(void* handle, gp_status* st);

typedef struct gp_shard_counters {
    int64_t plan_changes;   /* exchange plans chosen since creation (activity tiers)            */
    int64_t restores;       /* overflowed batches replayed from a restore point                 */
    int64_t send_bytes;     /* bytes of the current plan's send / receive chunks                */
    int64_t recv_bytes;
    int64_t restore_round;  /* round of the current restore point (-1: none)                     */
    int64_t bytes_sent;     /* exchange bytes this rank sent since the last reset, summed over the
                               rounds packed (replayed rounds included) (ABI 6)                  */
    int64_t list_rounds;    /* full gossip: rounds this rank ran on its ramp lists since the last
                               reset (ABI 8)                                                     */
    int64_t bin_rounds;     /* full gossip: rounds whose receipts this rank sent in bins since the
                               last reset (ABI 8)                                                */
} gp_shard_counters;
/* Exchange-plan counters of a shard (num_gpus > 1 handle: rank 0's). */
int gp_shard_stats(void* handle, gp_shard_counters* out);

void gp_destroy(void* handle);

/* Thread-local description of the last failure on this thread. */
const char* gp_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
