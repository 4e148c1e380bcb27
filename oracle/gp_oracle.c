/*
 * gp_oracle.c — CPU restatement of the reference's gossip / push-sum hot path,
 * recast as deterministic synchronous rounds (DESIGN.md §2 = SURVEY.md App. A).
 *
 * TEST INFRASTRUCTURE ONLY (see gp_oracle.h): the checker for the HIP product and the
 * CPU baseline timed by bench.py.  Never linked into libgossip_hip.so.
 *
 * PARITY UNPINNED for the round semantics: /root/reference/program.fs is asynchronous,
 * unseeded (System.Random per draw, program.fs:91,112,126,142) and has no tests or
 * fixtures; it cannot be run here (no dotnet).  Philox is pinned to the Random123 KATs and
 * the size arithmetic to SURVEY App. B; everything else is cross-checked against the
 * independent Python restatement in tests/golden/make_golden.py.
 *
 * Written independently of the product's csrc/ (no shared headers) so that a bug in one
 * is not silently mirrored in the other.
 */
#include "gp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ Philox4x32-10 */
/* Random123 constants (Salmon et al. 2011; same values as rocrand_philox4x32_10.h:62-65) */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void gpo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int i = 0; i < 10; ++i) {
        if (i) { k0 += PHILOX_W0; k1 += PHILOX_W1; }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Stream tags (counter word 3).  One Philox block per (node, round, stream); draw k uses
 * output word k.  index = (u64(x_k) * n) >> 32  — replaces Random().Next(0, n). */
#define ST_LEADER 0x4C454144u /* 'LEAD'  program.fs:173,211,250,316 */
#define ST_TOPO   0x544F504Fu /* 'TOPO'  program.fs:309             */
#define ST_GOSSIP 0x474F5353u /* 'GOSS'  program.fs:91              */
#define ST_PUSH   0x50555348u /* 'PUSH'  program.fs:112,126,142     */

static uint32_t draw(uint64_t seed, uint32_t stream, uint32_t r, uint32_t v, int k, uint32_t n) {
    uint32_t ctr[4] = {v, r, 0u, stream};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    gpo_philox4x32_10(ctr, key, out);
    return (uint32_t)(((uint64_t)out[k] * (uint64_t)n) >> 32);
}

/* ------------------------------------------------------------------ sizes */
/* program.fs:26-31 (Imp3D rounding), :228-229 (2D), :268 (G from the RAW argument). */
int gpo_sizes(int64_t n_arg, int32_t topology, int64_t* nodes, int64_t* actors, int64_t* grid) {
    if (n_arg < 1 || n_arg > 2147483647LL) return -1;
    int64_t nd = n_arg, g = 0;
    switch (topology) {
    case GPO_LINE:
    case GPO_FULL: break;
    case GPO_TWO_D:
        g = (int64_t)ceil(sqrt((double)n_arg));
        nd = g * g;
        break;
    case GPO_IMP3D:
    case GPO_THREE_D: {
        double c = floor(pow((double)n_arg, 0.33334));
        nd = (int64_t)pow(c, 3.0);
        g = (int64_t)floor(pow((double)n_arg, 0.34));
        if (g * g * g < nd) return -1; /* never happens for n_arg >= 1 (G >= cube root) */
        break;
    }
    default: return -1;
    }
    if (nd + 1 > 0xFFFFFFFELL) return -1;
    *nodes = nd;
    *actors = nd + 1;
    *grid = g;
    return 0;
}

/* ------------------------------------------------------------------ state */
typedef struct {
    gpo_config cfg;
    gpo_layout lay;
    int64_t A;
    /* out-neighbour CSR in the reference's ORDER (empty for FULL: implicit) */
    int64_t* off;
    uint32_t* adj;
    /* in-neighbour CSR, ascending, de-duplicated (pull mode; not built for FULL) */
    int64_t* ioff;
    uint32_t* iadj;
    int64_t round, completed;
    int converged;
    int64_t* trace;
    int64_t trace_cap;
    /* gossip */
    uint32_t *cnt, *inc;
    uint8_t *tok, *done;
    /* push-sum */
    double *S, *W, *Sin, *Win, *NSin, *NWin, *ms, *mw;
    uint32_t *cin, *Ncin, *tgt;
    uint8_t *term, *conv;
    /* shard mode */
    int shard, rank, world;
    int64_t lo, hi, bnd[17];
    int64_t calls;        /* gpo_shard_round calls so far                    */
    int64_t own_newly;    /* this rank's count of the round being exchanged   */
    int stopped;          /* global count reached nodes: later rounds are no-ops */
} oracle_t;

static int64_t deg_of(const oracle_t* o, int64_t v) {
    if (o->cfg.topology == GPO_FULL) return o->lay.nodes; /* all j != i among 0..nodes */
    return o->off[v + 1] - o->off[v];
}

static uint32_t nbr_of(const oracle_t* o, int64_t v, int64_t k) {
    if (o->cfg.topology == GPO_FULL) return (uint32_t)(k + (k >= v)); /* program.fs:201-206 */
    return o->adj[o->off[v] + k];
}

/* Build the reference's neighbour arrays literally (program.fs:162-171, 242-248, 287-313). */
static int build_topology(oracle_t* o) {
    const int64_t nodes = o->lay.nodes, A = o->A;
    const int topo = o->cfg.topology;
    if (topo == GPO_FULL) return 0;
    o->off = (int64_t*)calloc((size_t)A + 1, sizeof(int64_t));
    size_t cap = (size_t)A * 7 + 8;
    o->adj = (uint32_t*)malloc(cap * sizeof(uint32_t));
    if (!o->off || !o->adj) return -1;
    size_t e = 0;
    if (topo == GPO_LINE) {
        for (int64_t i = 0; i <= nodes; ++i) {
            o->off[i] = (int64_t)e;
            if (i == 0) o->adj[e++] = 1;                    /* :164-165 */
            else if (i == nodes) o->adj[e++] = (uint32_t)(i - 1); /* :166-167 */
            else { o->adj[e++] = (uint32_t)(i - 1); o->adj[e++] = (uint32_t)(i + 1); } /* :169 */
        }
    } else if (topo == GPO_TWO_D) {
        for (int64_t i = 0; i <= nodes; ++i) {
            o->off[i] = (int64_t)e;
            if (i > 0) o->adj[e++] = (uint32_t)(i - 1);     /* :244-245 */
            if (i < nodes) o->adj[e++] = (uint32_t)(i + 1); /* :246-247 */
        }
    } else { /* IMP3D / THREE_D */
        const int64_t G = o->lay.grid, zM = G * G, yM = G;
        const int64_t lim = G - 1;
        for (int64_t i = 0; i < nodes; ++i) { /* loop z,y,x of :287-292 visits i ascending */
            const int64_t x = i % G, y = (i / G) % G, z = i / zM;
            o->off[i] = (int64_t)e;
            if (x > 0) o->adj[e++] = (uint32_t)(i - 1);                          /* :295 */
            if (x < lim && i + 1 < nodes) o->adj[e++] = (uint32_t)(i + 1);       /* :297 */
            if (y > 0) o->adj[e++] = (uint32_t)(i - yM);                         /* :299 */
            if (y < lim && i + yM < nodes) o->adj[e++] = (uint32_t)(i + yM);     /* :301 */
            if (z > 0) o->adj[e++] = (uint32_t)(i - zM);                         /* :303 */
            if (z < lim && i + zM < nodes) o->adj[e++] = (uint32_t)(i + zM);     /* :305 */
            if (topo == GPO_IMP3D) /* :309 Random().Next(0, nodes-1): [0, nodes-2] */
                o->adj[e++] = draw(o->cfg.seed, ST_TOPO, 0u, (uint32_t)i, 0, (uint32_t)(nodes - 1));
        }
        o->off[nodes] = (int64_t)e; /* actor `nodes` is never wired (:293) */
    }
    o->off[A] = (int64_t)e;
    return 0;
}

static int build_in_csr(oracle_t* o) {
    if (o->ioff || o->cfg.topology == GPO_FULL) return 0;
    const int64_t A = o->A;
    int64_t* cnt = (int64_t*)calloc((size_t)A + 1, sizeof(int64_t));
    if (!cnt) return -1;
    for (int64_t u = 0; u < A; ++u)
        for (int64_t e = o->off[u]; e < o->off[u + 1]; ++e) cnt[o->adj[e] + 1]++;
    for (int64_t v = 0; v < A; ++v) cnt[v + 1] += cnt[v];
    o->ioff = (int64_t*)malloc(((size_t)A + 1) * sizeof(int64_t));
    o->iadj = (uint32_t*)malloc(((size_t)cnt[A] + 1) * sizeof(uint32_t));
    int64_t* fill = (int64_t*)malloc(((size_t)A + 1) * sizeof(int64_t));
    if (!o->ioff || !o->iadj || !fill) { free(cnt); free(fill); return -1; }
    memcpy(fill, cnt, ((size_t)A + 1) * sizeof(int64_t));
    for (int64_t u = 0; u < A; ++u) /* ascending u => each in-list is ascending */
        for (int64_t e = o->off[u]; e < o->off[u + 1]; ++e) {
            uint32_t v = o->adj[e];
            int64_t p = fill[v];
            if (p > cnt[v] && o->iadj[p - 1] == (uint32_t)u) continue; /* duplicate edge u->v */
            o->iadj[p] = (uint32_t)u;
            fill[v] = p + 1;
        }
    /* compact (duplicates leave holes at the end of a list) */
    int64_t w = 0;
    for (int64_t v = 0; v < A; ++v) {
        int64_t b = cnt[v], n = fill[v] - cnt[v];
        o->ioff[v] = w;
        memmove(o->iadj + w, o->iadj + b, (size_t)n * sizeof(uint32_t));
        w += n;
    }
    o->ioff[A] = w;
    free(cnt);
    free(fill);
    return 0;
}

static void push_trace(oracle_t* o, int64_t r, int64_t completed) {
    if (r >= o->trace_cap) {
        int64_t nc = o->trace_cap ? o->trace_cap * 2 : 1024;
        while (nc <= r) nc *= 2;
        o->trace = (int64_t*)realloc(o->trace, (size_t)nc * sizeof(int64_t));
        o->trace_cap = nc;
    }
    o->trace[r] = completed;
}

void gpo_destroy(void* h) {
    oracle_t* o = (oracle_t*)h;
    if (!o) return;
    free(o->off); free(o->adj); free(o->ioff); free(o->iadj); free(o->trace);
    free(o->cnt); free(o->inc); free(o->tok); free(o->done);
    free(o->S); free(o->W); free(o->Sin); free(o->Win); free(o->NSin); free(o->NWin);
    free(o->ms); free(o->mw); free(o->cin); free(o->Ncin); free(o->tgt);
    free(o->term); free(o->conv);
    free(o);
}

void* gpo_create(const gpo_config* cfg, gpo_layout* out) {
    oracle_t* o = (oracle_t*)calloc(1, sizeof(oracle_t));
    if (!o) return NULL;
    o->cfg = *cfg;
    if (cfg->algo != GPO_GOSSIP && cfg->algo != GPO_PUSHSUM) { free(o); return NULL; }
    if (gpo_sizes(cfg->n_arg, cfg->topology, &o->lay.nodes, &o->lay.actors, &o->lay.grid)) {
        free(o);
        return NULL;
    }
    const int64_t A = o->lay.actors, nodes = o->lay.nodes;
    o->A = A;
    if (build_topology(o)) { gpo_destroy(o); return NULL; }
    int64_t part = 0;
    for (int64_t v = 0; v < A; ++v) part += deg_of(o, v) > 0;
    o->lay.participants = part;
    /* leader = Random().Next(0, nodes) */
    o->lay.leader = draw(cfg->seed, ST_LEADER, 0u, 0u, 0, (uint32_t)nodes);
    const size_t n = (size_t)A;
    if (cfg->algo == GPO_GOSSIP) {
        o->cnt = (uint32_t*)calloc(n, 4); o->inc = (uint32_t*)calloc(n, 4);
        o->tok = (uint8_t*)calloc(n, 1); o->done = (uint8_t*)calloc(n, 1);
        if (!o->cnt || !o->inc || !o->tok || !o->done) { gpo_destroy(o); return NULL; }
        const int64_t L = o->lay.leader;
        if (cfg->topology == GPO_FULL) { o->cnt[L] = 1; o->tok[L] = 1; } /* CallChildActor :218 */
        else o->tok[L] = 1; /* ActivateChildActor :181,258,323 */
    } else {
        o->S = (double*)malloc(n * 8); o->W = (double*)malloc(n * 8);
        o->Sin = (double*)calloc(n, 8); o->Win = (double*)calloc(n, 8);
        o->NSin = (double*)calloc(n, 8); o->NWin = (double*)calloc(n, 8);
        o->ms = (double*)calloc(n, 8); o->mw = (double*)calloc(n, 8);
        o->cin = (uint32_t*)calloc(n, 4); o->Ncin = (uint32_t*)calloc(n, 4);
        o->tgt = (uint32_t*)malloc(n * 4);
        o->term = (uint8_t*)calloc(n, 1); o->conv = (uint8_t*)calloc(n, 1);
        if (!o->S || !o->W || !o->Sin || !o->Win || !o->NSin || !o->NWin || !o->ms || !o->mw ||
            !o->cin || !o->Ncin || !o->tgt || !o->term || !o->conv) {
            gpo_destroy(o);
            return NULL;
        }
        for (int64_t v = 0; v < A; ++v) {
            o->S[v] = (double)v; /* InitializeVariables x (:107-108) */
            o->W[v] = 1.0;       /* weight = 1.0 (:78) */
            o->term[v] = deg_of(o, v) > 0 ? (uint8_t)cfg->term_init : 0; /* termRound = 1 (:79) */
            o->tgt[v] = 0xFFFFFFFFu;
        }
    }
    if (out) *out = o->lay;
    return o;
}

/* ------------------------------------------------------------------ gossip round */
/* program.fs:89-105 recast: every activation chain (tok) draws one neighbour per round
 * and sends unless the target was done at round start (:92); a receipt that moves the
 * count from <=thr to >thr reports (:102-104); the first receipt adds a chain (:99-100). */
static int64_t gossip_round(oracle_t* o, uint32_t r, int threads) {
    const int64_t A = o->A;
    const uint32_t thr = (uint32_t)o->cfg.gossip_threshold;
    const uint64_t seed = o->cfg.seed;
    int64_t newly = 0;
    if (threads <= 0) {
        for (int64_t v = 0; v < A; ++v) {
            const int64_t d = deg_of(o, v);
            for (int k = 0; k < o->tok[v] && d > 0; ++k) {
                uint32_t t = nbr_of(o, v, draw(seed, ST_GOSSIP, r, (uint32_t)v, k, (uint32_t)d));
                if (!o->done[t]) o->inc[t]++;
            }
        }
        for (int64_t v = 0; v < A; ++v) {
            uint32_t c0 = o->cnt[v], c1 = c0 + o->inc[v];
            o->inc[v] = 0;
            o->cnt[v] = c1;
            if (c0 == 0 && c1 > 0) o->tok[v]++;
            if (c0 <= thr && c1 >= thr + 1) { o->done[v] = 1; newly++; }
        }
        return newly;
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
    for (int64_t v = 0; v < A; ++v) {
        const int64_t d = deg_of(o, v);
        for (int k = 0; k < o->tok[v] && d > 0; ++k) {
            uint32_t t = nbr_of(o, v, draw(seed, ST_GOSSIP, r, (uint32_t)v, k, (uint32_t)d));
            if (!o->done[t]) __atomic_fetch_add(&o->inc[t], 1u, __ATOMIC_RELAXED); /* integer: order-free */
        }
    }
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : newly)
#endif
    for (int64_t v = 0; v < A; ++v) {
        uint32_t c0 = o->cnt[v], c1 = c0 + o->inc[v];
        o->inc[v] = 0;
        o->cnt[v] = c1;
        if (c0 == 0 && c1 > 0) o->tok[v]++;
        if (c0 <= thr && c1 >= thr + 1) { o->done[v] = 1; newly++; }
    }
    return newly;
}

/* ------------------------------------------------------------------ push-sum round */
/* Phase 1 for one node (program.fs:110-143 recast).  Returns 1 when the node
 * converges this round.  Writes the emitted message into tgt/ms/mw. */
static int ps_phase1(oracle_t* o, int64_t v, uint32_t r) {
    const int64_t d = deg_of(o, v);
    o->tgt[v] = 0xFFFFFFFFu;
    if (d == 0) return 0; /* non-participant (isolated Imp3D actor, :293) */
    int conv_now = 0;
    const uint32_t cin = o->cin[v];
    if (o->conv[v]) { /* :125-127 relay, own (S,W) frozen */
        if (cin > 0) {
            o->tgt[v] = nbr_of(o, v, draw(o->cfg.seed, ST_PUSH, r, (uint32_t)v, 0, (uint32_t)d));
            o->ms[v] = o->Sin[v];
            o->mw[v] = o->Win[v];
        }
        return 0;
    }
    const double S = o->S[v], W = o->W[v];
    const double nS = S + o->Sin[v], nW = W + o->Win[v]; /* :120-121 */
    if (cin > 0) {
        const double cal = fabs(S / W - nS / nW); /* :123 */
        if (cal > o->cfg.delta) o->term[v] = 0;   /* :130-131 */
        else o->term[v]++;                        /* :133 */
        if (o->term[v] == o->cfg.term_limit) {    /* :135-138 */
            o->term[v] = 0;
            o->conv[v] = 1;
            conv_now = 1;
        }
    }
    o->S[v] = nS / 2.0; /* :140-141 (also :114-115 in round 0) */
    o->W[v] = nW / 2.0;
    o->tgt[v] = nbr_of(o, v, draw(o->cfg.seed, ST_PUSH, r, (uint32_t)v, 0, (uint32_t)d)); /* :142-143 */
    o->ms[v] = o->S[v];
    o->mw[v] = o->W[v];
    return conv_now;
}

static int64_t pushsum_round(oracle_t* o, uint32_t r, int threads) {
    const int64_t A = o->A;
    int64_t newly = 0;
    if (threads <= 0 || o->cfg.topology == GPO_FULL) {
        for (int64_t v = 0; v < A; ++v) newly += ps_phase1(o, v, r);
        /* phase 2: inbox sums from +0.0 in ASCENDING source order (the loop order) */
        for (int64_t v = 0; v < A; ++v) { o->NSin[v] = 0.0; o->NWin[v] = 0.0; o->Ncin[v] = 0; }
        for (int64_t u = 0; u < A; ++u) {
            uint32_t t = o->tgt[u];
            if (t == 0xFFFFFFFFu) continue;
            o->NSin[t] += o->ms[u];
            o->NWin[t] += o->mw[u];
            o->Ncin[t]++;
        }
    } else {
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static) reduction(+ : newly)
#endif
        for (int64_t v = 0; v < A; ++v) newly += ps_phase1(o, v, r);
#ifdef _OPENMP
#pragma omp parallel for num_threads(threads) schedule(static)
#endif
        for (int64_t v = 0; v < A; ++v) { /* pull over the ascending in-list: same order */
            double s = 0.0, w = 0.0;
            uint32_t c = 0;
            for (int64_t e = o->ioff[v]; e < o->ioff[v + 1]; ++e) {
                uint32_t u = o->iadj[e];
                if (o->tgt[u] == (uint32_t)v) { s += o->ms[u]; w += o->mw[u]; c++; }
            }
            o->NSin[v] = s; o->NWin[v] = w; o->Ncin[v] = c;
        }
    }
    double* t;
    t = o->Sin; o->Sin = o->NSin; o->NSin = t;
    t = o->Win; o->Win = o->NWin; o->NWin = t;
    uint32_t* tc = o->cin; o->cin = o->Ncin; o->Ncin = tc;
    return newly;
}

int gpo_step(void* h, int64_t max_rounds, int32_t threads, gpo_status* st) {
    oracle_t* o = (oracle_t*)h;
    if (!o) return -1;
    if (threads > 0 && o->cfg.algo == GPO_PUSHSUM && build_in_csr(o)) return -2;
    for (int64_t i = 0; i < max_rounds && !o->converged; ++i) {
        const uint32_t r = (uint32_t)o->round;
        int64_t newly = o->cfg.algo == GPO_GOSSIP ? gossip_round(o, r, threads)
                                                  : pushsum_round(o, r, threads);
        o->completed += newly;
        push_trace(o, o->round, o->completed);
        o->round++;
        if (o->completed >= o->lay.nodes) o->converged = 1; /* ParentActor :49,56 */
    }
    if (st) {
        st->round = o->round;
        st->completed = o->completed;
        st->converged = o->converged;
        st->pad = 0;
        st->sum_s = st->sum_w = 0.0;
        if (o->cfg.algo == GPO_PUSHSUM) {
            double s = 0.0, w = 0.0;
            for (int64_t v = 0; v < o->A; ++v) {
                if (deg_of(o, v) > 0) { s += o->S[v]; w += o->W[v]; }
                s += o->Sin[v];
                w += o->Win[v];
            }
            st->sum_s = s;
            st->sum_w = w;
        }
    }
    return 0;
}

int gpo_degree(void* h, int64_t v) {
    oracle_t* o = (oracle_t*)h;
    if (!o || v < 0 || v >= o->A) return -1;
    return (int)deg_of(o, v);
}

int gpo_neighbors(void* h, int64_t v, uint32_t* out, int32_t cap) {
    oracle_t* o = (oracle_t*)h;
    if (!o || v < 0 || v >= o->A) return -1;
    int64_t d = deg_of(o, v);
    for (int64_t k = 0; k < d && k < cap; ++k) out[k] = nbr_of(o, v, k);
    return (int)d;
}

static int range_ok(const oracle_t* o, int64_t first, int64_t count) {
    return o && first >= 0 && count >= 0 && first + count <= o->A;
}

int gpo_read_gossip(void* h, int64_t first, int64_t count, uint32_t* cnt, uint8_t* flags) {
    oracle_t* o = (oracle_t*)h;
    if (!range_ok(o, first, count) || o->cfg.algo != GPO_GOSSIP) return -1;
    for (int64_t i = 0; i < count; ++i) {
        int64_t v = first + i;
        if (cnt) cnt[i] = o->cnt[v];
        if (flags) flags[i] = (uint8_t)((o->tok[v] & 3u) | (o->done[v] ? 4u : 0u));
    }
    return 0;
}

int gpo_read_pushsum(void* h, int64_t first, int64_t count, double* S, double* W, uint8_t* flags) {
    oracle_t* o = (oracle_t*)h;
    if (!range_ok(o, first, count) || o->cfg.algo != GPO_PUSHSUM) return -1;
    for (int64_t i = 0; i < count; ++i) {
        int64_t v = first + i;
        if (S) S[i] = o->S[v];
        if (W) W[i] = o->W[v];
        if (flags) flags[i] = (uint8_t)((o->term[v] & 15u) | (o->conv[v] ? 16u : 0u));
    }
    return 0;
}

int gpo_read_messages(void* h, int64_t first, int64_t count, uint32_t* dst, double* s, double* w) {
    oracle_t* o = (oracle_t*)h;
    if (!range_ok(o, first, count) || o->cfg.algo != GPO_PUSHSUM) return -1;
    for (int64_t i = 0; i < count; ++i) {
        int64_t v = first + i;
        uint32_t t = o->round ? o->tgt[v] : 0xFFFFFFFFu;
        if (dst) dst[i] = t;
        if (s) s[i] = t == 0xFFFFFFFFu ? 0.0 : o->ms[v];
        if (w) w[i] = t == 0xFFFFFFFFu ? 0.0 : o->mw[v];
    }
    return 0;
}

int gpo_read_trace(void* h, int64_t first_round, int64_t count, int64_t* completed) {
    oracle_t* o = (oracle_t*)h;
    if (!o || first_round < 0 || count < 0 || first_round + count > o->round) return -1;
    memcpy(completed, o->trace + first_round, (size_t)count * sizeof(int64_t));
    return 0;
}

/* ------------------------------------------------------------------ shard mode */
typedef struct { int64_t newly, count; } shard_hdr;              /* 16 bytes */
typedef struct { uint32_t src, dst; double s, w; } shard_msg;    /* 24 bytes */

static int owner_of(const oracle_t* o, int64_t v) {
    int q = 0;
    while (q + 1 < o->world && v >= o->bnd[q + 1]) ++q;
    return q;
}

/* Chunk from rank p: header + room for every message p's actors can emit in one round
 * (push-sum: one per actor; gossip: one per activation chain, at most two per actor). */
static int64_t chunk_bytes(const oracle_t* o, int p) {
    const int64_t n = o->bnd[p + 1] - o->bnd[p];
    return (int64_t)sizeof(shard_hdr) + (o->cfg.algo == GPO_GOSSIP ? 2 : 1) * n * (int64_t)sizeof(shard_msg);
}

void* gpo_shard_create(const gpo_config* cfg, int32_t rank, int32_t world, const int64_t* bounds, gpo_layout* out) {
    if (world < 1 || world > 16 || rank < 0 || rank >= world || !bounds) return NULL;
    oracle_t* o = (oracle_t*)gpo_create(cfg, out);
    if (!o) return NULL;
    if (bounds[0] != 0 || bounds[world] != o->A) { gpo_destroy(o); return NULL; }
    for (int q = 0; q < world; ++q)
        if (bounds[q + 1] <= bounds[q]) { gpo_destroy(o); return NULL; }
    o->shard = 1;
    o->rank = rank;
    o->world = world;
    for (int q = 0; q <= world; ++q) o->bnd[q] = bounds[q];
    o->lo = bounds[rank];
    o->hi = bounds[rank + 1];
    return o;
}

int gpo_shard_plan(void* h, int64_t* send_bytes, int64_t* recv_bytes) {
    oracle_t* o = (oracle_t*)h;
    if (!o || !o->shard) return -1;
    for (int q = 0; q < o->world; ++q) {
        send_bytes[q] = q == o->rank ? 0 : chunk_bytes(o, o->rank);
        recv_bytes[q] = q == o->rank ? 0 : chunk_bytes(o, q);
    }
    return 0;
}

static char* chunk_at(const oracle_t* o, char* base, int peer, int sending) {
    int64_t off = 0;
    for (int q = 0; q < peer; ++q)
        if (q != o->rank) off += chunk_bytes(o, sending ? o->rank : q);
    return base + off;
}

static void put_msg(oracle_t* o, char* send, uint32_t u, uint32_t t, double s, double w) {
    const int q = owner_of(o, t);
    shard_hdr* hd = (shard_hdr*)chunk_at(o, send, q, 1);
    shard_msg* m = (shard_msg*)(hd + 1) + hd->count++;
    m->src = u; m->dst = t; m->s = s; m->w = w;
}

/* Apply the receipts gathered for round a (program.fs:97-105) on this rank's actors. */
static int64_t gossip_apply_own(oracle_t* o) {
    const uint32_t thr = (uint32_t)o->cfg.gossip_threshold;
    int64_t newly = 0;
    for (int64_t v = o->lo; v < o->hi; ++v) {
        uint32_t c0 = o->cnt[v], c1 = c0 + o->inc[v];
        o->inc[v] = 0;
        o->cnt[v] = c1;
        if (c0 == 0 && c1 > 0) o->tok[v]++;
        if (c0 <= thr && c1 >= thr + 1) { o->done[v] = 1; newly++; }
    }
    return newly;
}

int gpo_shard_round(void* h, void* send) {
    oracle_t* o = (oracle_t*)h;
    if (!o || !o->shard) return -1;
    const uint32_t r = (uint32_t)o->calls;
    for (int q = 0; q < o->world; ++q)
        if (q != o->rank) { shard_hdr* hd = (shard_hdr*)chunk_at(o, (char*)send, q, 1); hd->newly = 0; hd->count = 0; }
    int64_t newly = 0;
    if (!o->stopped) {
        if (o->cfg.algo == GPO_GOSSIP) {
            /* the receipts of round r-1 are applied first (their count travels now), then the
             * chains of round r draw; local receipts are filtered by done at round start */
            if (r >= 1) newly = gossip_apply_own(o);
            for (int64_t v = o->lo; v < o->hi; ++v) {
                const int64_t d = deg_of(o, v);
                for (int k = 0; k < o->tok[v] && d > 0; ++k) {
                    uint32_t t = nbr_of(o, v, draw(o->cfg.seed, ST_GOSSIP, r, (uint32_t)v, k, (uint32_t)d));
                    if (t >= o->lo && t < o->hi) { if (!o->done[t]) o->inc[t]++; }
                    else put_msg(o, (char*)send, (uint32_t)v, t, 0.0, 0.0);
                }
            }
        } else {
            for (int64_t v = o->lo; v < o->hi; ++v) {
                newly += ps_phase1(o, v, r);
                const uint32_t t = o->tgt[v];
                if (t != 0xFFFFFFFFu && (t < o->lo || t >= o->hi)) put_msg(o, (char*)send, (uint32_t)v, t, o->ms[v], o->mw[v]);
            }
        }
    }
    for (int q = 0; q < o->world; ++q)
        if (q != o->rank) ((shard_hdr*)chunk_at(o, (char*)send, q, 1))->newly = newly;
    o->own_newly = newly;
    o->calls++;
    return 0;
}

int gpo_shard_deliver(void* h, const void* recv) {
    oracle_t* o = (oracle_t*)h;
    if (!o || !o->shard || o->calls == 0) return -1;
    const int64_t k = o->calls - 1;
    int64_t newly = o->own_newly;
    for (int q = 0; q < o->world; ++q)
        if (q != o->rank) newly += ((const shard_hdr*)chunk_at(o, (char*)recv, q, 0))->newly;
    if (!o->stopped) {
        if (o->cfg.algo == GPO_GOSSIP) {
            for (int q = 0; q < o->world; ++q) {
                if (q == o->rank) continue;
                const shard_hdr* hd = (const shard_hdr*)chunk_at(o, (char*)recv, q, 0);
                const shard_msg* m = (const shard_msg*)(hd + 1);
                for (int64_t i = 0; i < hd->count; ++i)
                    if (!o->done[m[i].dst]) o->inc[m[i].dst]++;
            }
        } else {
            /* inbox sums from +0.0 in ascending source order: ranks in order, own in place */
            for (int64_t v = o->lo; v < o->hi; ++v) { o->NSin[v] = 0.0; o->NWin[v] = 0.0; o->Ncin[v] = 0; }
            for (int q = 0; q < o->world; ++q) {
                if (q == o->rank) {
                    for (int64_t u = o->lo; u < o->hi; ++u) {
                        const uint32_t t = o->tgt[u];
                        if (t == 0xFFFFFFFFu || t < o->lo || t >= o->hi) continue;
                        o->NSin[t] += o->ms[u]; o->NWin[t] += o->mw[u]; o->Ncin[t]++;
                    }
                    continue;
                }
                const shard_hdr* hd = (const shard_hdr*)chunk_at(o, (char*)recv, q, 0);
                const shard_msg* m = (const shard_msg*)(hd + 1);
                for (int64_t i = 0; i < hd->count; ++i) {
                    o->NSin[m[i].dst] += m[i].s; o->NWin[m[i].dst] += m[i].w; o->Ncin[m[i].dst]++;
                }
            }
            double* t;
            t = o->Sin; o->Sin = o->NSin; o->NSin = t;
            t = o->Win; o->Win = o->NWin; o->NWin = t;
            uint32_t* tc = o->cin; o->cin = o->Ncin; o->Ncin = tc;
        }
        const int64_t applied = o->cfg.algo == GPO_GOSSIP ? k - 1 : k;
        if (applied >= 0) {
            o->completed += newly;
            push_trace(o, o->round, o->completed);
            o->round++;
            if (o->completed >= o->lay.nodes) { o->converged = 1; o->stopped = 1; }
        }
    }
    return 0;
}

int gpo_shard_sync(void* h, gpo_status* st) {
    oracle_t* o = (oracle_t*)h;
    if (!o || !o->shard) return -1;
    st->round = o->round;
    st->completed = o->completed;
    st->converged = o->converged;
    st->pad = 0;
    st->sum_s = st->sum_w = 0.0;
    if (o->cfg.algo == GPO_PUSHSUM) {
        /* this rank's held mass plus what its actors sent in the last round */
        for (int64_t v = o->lo; v < o->hi; ++v) {
            if (deg_of(o, v) > 0) { st->sum_s += o->S[v]; st->sum_w += o->W[v]; }
            if (o->calls > 0 && o->tgt[v] != 0xFFFFFFFFu) { st->sum_s += o->ms[v]; st->sum_w += o->mw[v]; }
        }
    }
    return 0;
}
