/*
 * gp_oracle.h — CPU restatement of the reference gossip / push-sum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (libgossip_hip.so) never links or calls it.
 *
 * Follows /root/reference/program.fs recast into the synchronous-round semantics
 * frozen in DESIGN.md §2.  Pinning status:
 *   - Philox4x32-10: pinned to the Random123 known-answer vectors (tests/test_oracle.py).
 *   - size arithmetic (program.fs:26-31, 228-229, 268): pinned to SURVEY App. B.
 *   - round semantics: PARITY UNPINNED against the reference itself — the reference is an
 *     unseeded asynchronous Akka.NET program with no tests or fixtures, and it cannot run
 *     here (no dotnet).  It is cross-checked against an independent pure-Python restatement
 *     (tests/golden/make_golden.py) whose vectors are committed under tests/golden/.
 */
#ifndef GP_ORACLE_H
#define GP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* topology / algorithm codes — identical numbering to include/gossip_hip.h */
enum { GPO_LINE = 0, GPO_FULL = 1, GPO_TWO_D = 2, GPO_IMP3D = 3, GPO_THREE_D = 4 };
enum { GPO_GOSSIP = 0, GPO_PUSHSUM = 1 };

typedef struct {
    int64_t n_arg;            /* raw argv[1]                                   */
    int32_t topology;         /* GPO_*                                          */
    int32_t algo;             /* GPO_GOSSIP / GPO_PUSHSUM                       */
    uint64_t seed;            /* Philox key                                     */
    double delta;             /* push-sum threshold (program.fs:187: 1e-10)     */
    int32_t gossip_threshold; /* program.fs:102 (10)                            */
    int32_t term_init;        /* program.fs:79 (1)                              */
    int32_t term_limit;       /* program.fs:135 (3)                             */
} gpo_config;

typedef struct {
    int64_t nodes;        /* `nodes` after rounding (completion target T)      */
    int64_t actors;       /* nodes + 1 (program.fs:152,192,233,269)            */
    int64_t grid;         /* G for Imp3D/3D (program.fs:268), g for 2D, 0 else */
    int64_t leader;       /* program.fs:173/211/250/316                        */
    int64_t participants; /* actors with at least one neighbour                */
} gpo_layout;

typedef struct {
    int64_t round;      /* rounds executed so far                              */
    int64_t completed;  /* CompletedMessage / PushSumResult count              */
    int32_t converged;  /* completed >= nodes                                  */
    int32_t pad;
    double sum_s, sum_w; /* push-sum: held + in-flight mass                    */
} gpo_status;

void gpo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
int  gpo_sizes(int64_t n_arg, int32_t topology, int64_t* nodes, int64_t* actors, int64_t* grid);

void* gpo_create(const gpo_config* cfg, gpo_layout* out);
/* threads == 0: canonical single-thread scatter order; threads > 0: OpenMP pull mode
 * (in-neighbour CSR, receiver-side filter) with that many threads. Same results. */
int  gpo_step(void* h, int64_t max_rounds, int32_t threads, gpo_status* st);
int  gpo_degree(void* h, int64_t v);
int  gpo_neighbors(void* h, int64_t v, uint32_t* out, int32_t cap);
int  gpo_read_gossip(void* h, int64_t first, int64_t count, uint32_t* cnt, uint8_t* flags);
int  gpo_read_pushsum(void* h, int64_t first, int64_t count, double* S, double* W, uint8_t* flags);
int  gpo_read_messages(void* h, int64_t first, int64_t count, uint32_t* dst, double* s, double* w);
int  gpo_read_trace(void* h, int64_t first_round, int64_t count, int64_t* completed);
void gpo_destroy(void* h);

/* Shard mode (checker for the multi-GPU decomposition): rank `rank` of
 * `world` owns actors [bounds[rank], bounds[rank+1]) of the same global graph.  Independent of
 * the product's halo/slot scheme: every message whose destination belongs to another rank is
 * shipped as an explicit (source, destination, s, w) record, and the receiver merges the
 * records of all ranks in rank order — i.e. ascending source order, the canonical inbox order.
 * Completion counts travel in each chunk's header.  Per round: gpo_shard_round(send) ->
 * any all-to-all -> gpo_shard_deliver(recv); gpo_shard_sync reports the global count. */
void* gpo_shard_create(const gpo_config* cfg, int32_t rank, int32_t world, const int64_t* bounds, gpo_layout* out);
int  gpo_shard_plan(void* h, int64_t* send_bytes, int64_t* recv_bytes);
int  gpo_shard_round(void* h, void* send);
int  gpo_shard_deliver(void* h, const void* recv);
int  gpo_shard_sync(void* h, gpo_status* st);

/* Asynchronous actor run (gp_async.c): the reference's Akka execution model — per-actor FIFO
 * mailboxes, a seeded random interleaving of runnable actors — over the same neighbour lists
 * and leader, for statistical sanity checks only.  Time unit: one processed
 * message.  Any output pointer may be NULL; arrays hold `actors` entries. */
typedef struct {
    int64_t steps;      /* messages processed                                   */
    int64_t completed;  /* reports received by the parent                      */
    int32_t converged;  /* completed >= nodes                                   */
    int32_t pad;
    int64_t messages;   /* messages sent (incl. kick-off and self-activations)  */
    double sum_s, sum_w; /* push-sum mass held + in mailboxes                   */
} gpo_async_status;

int gpo_async_run(const gpo_config* cfg, int64_t max_steps, gpo_async_status* st, uint32_t* cnt, double* S,
                  double* W, uint8_t* flags);

#ifdef __cplusplus
}
#endif
#endif
