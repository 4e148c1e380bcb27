/*
 * gp_async.c — the reference's ASYNCHRONOUS actor run, restated for a statistical sanity check
 * (SURVEY.md §4.7, §8(f) 2).  TEST INFRASTRUCTURE ONLY (see gp_oracle.h).
 *
 * The product engine and gp_oracle.c run the synchronous-round recast.  This file
 * instead models what program.fs does under Akka.NET: one FIFO mailbox per actor, actors run
 * one message at a time, and the order in which runnable actors take their next message is an
 * arbitrary interleaving — here a seeded uniform choice among actors with a non-empty mailbox
 * (splitmix64; the reference's unseeded System.Random, Q21, is irreproducible anyway).
 *
 *   ChildActor   program.fs:74-147
 *     ActivateChildActor (:89-95): draw a neighbour; send CallChildActor unless it is done (no
 *                                  redraw, Q14); re-enqueue ActivateChildActor to self (Q13)
 *     CallChildActor (:97-105):    first receipt starts the activation loop; the 11th receipt
 *                                  reports to the parent and marks the actor done (Q12)
 *     PushSum (:110-116):          halve, send the half to a random neighbour (kick-off, Q17)
 *     ComputePushSum (:119-143):   cal = |S/W - (S+s)/(W+w)|, termRound (starts at 1, Q18);
 *                                  at 3: converged, report; a converged actor relays (Q19)
 *   ParentActor  program.fs:38-67  stop when the report count reaches AllNodes = nodes (Q3, Q22)
 *   kick-off     program.fs:173-187, 209-223, 250-263, 316-328 (Q15: full gossip starts with a
 *                CallChildActor, the other topologies with an ActivateChildActor)
 *
 * Neighbour lists come from gp_oracle.c (literal program.fs arrays, same Philox extra links and
 * leader), so only the execution model differs from the round-mode oracle.  The unit of time
 * is one processed message ("step"); a run stops at convergence or after max_steps.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gp_oracle.h"

enum { M_ACTIVATE = 0, M_CALL = 1, M_PUSHSUM = 2, M_COMPUTE = 3 };

typedef struct {
    uint8_t kind;
    double s, w;
} amsg;

typedef struct {  /* growable ring buffer */
    amsg* q;
    uint32_t head, len, cap;
} mailbox;

static uint64_t sm_next(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* uniform in [0, n) (Random().Next(0, n)) */
static uint32_t sm_below(uint64_t* x, uint32_t n) { return (uint32_t)(((sm_next(x) >> 32) * (uint64_t)n) >> 32); }

typedef struct {
    int64_t actors;
    mailbox* mb;
    uint32_t* ready;  /* actors with a non-empty mailbox */
    uint32_t* pos;    /* index in ready, or UINT32_MAX */
    uint32_t nready;
    int oom;
} sched;

static void post(sched* s, uint32_t to, amsg m) {
    mailbox* b = &s->mb[to];
    if (b->len == b->cap) {
        uint32_t nc = b->cap ? b->cap * 2 : 4;
        amsg* nq = (amsg*)malloc((size_t)nc * sizeof(amsg));
        if (!nq) {
            s->oom = 1;
            return;
        }
        for (uint32_t i = 0; i < b->len; ++i) nq[i] = b->q[(b->head + i) % b->cap];
        free(b->q);
        b->q = nq;
        b->head = 0;
        b->cap = nc;
    }
    b->q[(b->head + b->len) % b->cap] = m;
    if (b->len++ == 0) {
        s->pos[to] = s->nready;
        s->ready[s->nready++] = to;
    }
}

static amsg take(sched* s, uint32_t a) {
    mailbox* b = &s->mb[a];
    amsg m = b->q[b->head];
    b->head = (b->head + 1) % b->cap;
    if (--b->len == 0) {  /* swap-remove from the ready set */
        uint32_t i = s->pos[a], last = s->ready[--s->nready];
        s->ready[i] = last;
        s->pos[last] = i;
        s->pos[a] = UINT32_MAX;
    }
    return m;
}

int gpo_async_run(const gpo_config* cfg, int64_t max_steps, gpo_async_status* st, uint32_t* cnt_out, double* S_out,
                  double* W_out, uint8_t* flags_out) {
    gpo_layout lay;
    void* h = gpo_create(cfg, &lay);
    if (!h) return -1;
    const int64_t A = lay.actors;
    /* neighbour CSR in reference order */
    uint32_t* off = (uint32_t*)malloc(((size_t)A + 1) * sizeof(uint32_t));
    int64_t total = 0;
    for (int64_t v = 0; v < A; ++v) total += gpo_degree(h, v);
    uint32_t* nb = (uint32_t*)malloc((size_t)(total ? total : 1) * sizeof(uint32_t));
    sched s = {0};
    s.actors = A;
    s.mb = (mailbox*)calloc((size_t)A, sizeof(mailbox));
    s.ready = (uint32_t*)malloc((size_t)A * sizeof(uint32_t));
    s.pos = (uint32_t*)malloc((size_t)A * sizeof(uint32_t));
    uint32_t* cnt = (uint32_t*)calloc((size_t)A, sizeof(uint32_t));
    uint8_t* done = (uint8_t*)calloc((size_t)A, 1);
    uint8_t* conv = (uint8_t*)calloc((size_t)A, 1);
    uint8_t* term = (uint8_t*)malloc((size_t)A);
    double* S = (double*)malloc((size_t)A * sizeof(double));
    double* W = (double*)malloc((size_t)A * sizeof(double));
    int rc = 0;
    if (!off || !nb || !s.mb || !s.ready || !s.pos || !cnt || !done || !conv || !term || !S || !W) {
        rc = -2;
        goto out;
    }
    off[0] = 0;
    for (int64_t v = 0; v < A; ++v) {
        const int d = gpo_degree(h, v);
        gpo_neighbors(h, v, nb + off[v], d);
        off[v + 1] = off[v] + (uint32_t)d;
        s.pos[v] = UINT32_MAX;
        S[v] = (double)v; /* InitializeVariables (program.fs:107-108, Q16) */
        W[v] = 1.0;
        term[v] = (uint8_t)cfg->term_init;
    }
    uint64_t rng = cfg->seed ^ 0xA5F1C0DEull;
    const uint32_t L = (uint32_t)lay.leader;
    const int gossip = cfg->algo == GPO_GOSSIP;
    if (gossip) {
        amsg m = {cfg->topology == GPO_FULL ? M_CALL : M_ACTIVATE, 0.0, 0.0};
        post(&s, L, m);
    } else {
        amsg m = {M_PUSHSUM, 0.0, 0.0};
        post(&s, L, m);
    }
    int64_t steps = 0, completed = 0, sent = 1;
    const int64_t target = lay.nodes;
    while (completed < target && steps < max_steps && s.nready && !s.oom) {
        const uint32_t a = s.ready[sm_below(&rng, s.nready)];
        const amsg m = take(&s, a);
        ++steps;
        const uint32_t deg = off[a + 1] - off[a];
        if (m.kind == M_ACTIVATE) {
            if (deg) {
                const uint32_t t = nb[off[a] + sm_below(&rng, deg)];
                if (!done[t]) {
                    amsg c = {M_CALL, 0.0, 0.0};
                    post(&s, t, c);
                    ++sent;
                }
            }
            amsg self = {M_ACTIVATE, 0.0, 0.0};
            post(&s, a, self);
            ++sent;
        } else if (m.kind == M_CALL) {
            if (cnt[a] == 0) {
                amsg self = {M_ACTIVATE, 0.0, 0.0};
                post(&s, a, self);
                ++sent;
            }
            if (cnt[a] == (uint32_t)cfg->gossip_threshold) {
                ++completed;
                done[a] = 1;
            }
            ++cnt[a];
        } else if (deg) { /* push-sum: an actor without neighbours cannot send (never reached) */
            double os, ow;
            if (m.kind == M_PUSHSUM) {
                S[a] = S[a] / 2.0;
                W[a] = W[a] / 2.0;
                os = S[a];
                ow = W[a];
            } else if (conv[a]) {
                os = m.s;
                ow = m.w;
            } else {
                const double ns = S[a] + m.s, nw = W[a] + m.w;
                const double cal = fabs(S[a] / W[a] - ns / nw);
                term[a] = cal > cfg->delta ? 0 : (uint8_t)(term[a] + 1);
                if (term[a] == cfg->term_limit) {
                    term[a] = 0;
                    conv[a] = 1;
                    ++completed;
                }
                S[a] = ns / 2.0;
                W[a] = nw / 2.0;
                os = S[a];
                ow = W[a];
            }
            amsg c = {M_COMPUTE, os, ow};
            post(&s, nb[off[a] + sm_below(&rng, deg)], c);
            ++sent;
        }
    }
    if (s.oom) {
        rc = -2;
        goto out;
    }
    if (st) {
        memset(st, 0, sizeof *st);
        st->steps = steps;
        st->completed = completed;
        st->converged = completed >= target;
        st->messages = sent;
        double ss = 0.0, ww = 0.0;
        for (int64_t v = 0; v < A; ++v) {
            ss += S[v];
            ww += W[v];
            const mailbox* b = &s.mb[v];
            for (uint32_t i = 0; i < b->len; ++i) {
                ss += b->q[(b->head + i) % b->cap].s;
                ww += b->q[(b->head + i) % b->cap].w;
            }
        }
        st->sum_s = ss;
        st->sum_w = ww;
    }
    for (int64_t v = 0; v < A; ++v) {
        if (cnt_out) cnt_out[v] = cnt[v];
        if (S_out) S_out[v] = S[v];
        if (W_out) W_out[v] = W[v];
        if (flags_out) flags_out[v] = (uint8_t)(gossip ? (done[v] ? 4 : 0) : (conv[v] ? 16 : 0));
    }
out:
    if (s.mb)
        for (int64_t v = 0; v < A; ++v) free(s.mb[v].q);
    free(s.mb);
    free(s.ready);
    free(s.pos);
    free(off);
    free(nb);
    free(cnt);
    free(done);
    free(conv);
    free(term);
    free(S);
    free(W);
    gpo_destroy(h);
    return rc;
}
