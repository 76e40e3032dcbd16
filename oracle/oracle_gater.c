/*
 * oracle_gater.c — the peer gater (peer_gater.go), restated over the
 * oracle's network.  TEST INFRASTRUCTURE (see oracle.h).
 *
 * Every router i keeps (peer_gater.go:118-152):
 *   validate, throttle     ValidateMessage / RejectMessage(throttled) counts  (:123-124, 386-391, 402-409)
 *   lastThrottle           time of the last throttled validation               (:127)
 *   ipStats[ip]            deliver, duplicate, ignore, reject + connected and
 *                          expire, shared by the peers of one IP               (:131-152, 243-259)
 * A peer's stats object is its IP's (getPeerIP: the first IP of the peer,
 * "<unknown>" when it has none).  Over the CSR it lives at the group's
 * representative edge: the lowest position of router i's row whose peer has
 * the same IP key.
 *
 * Deterministic restatement:
 *   * AcceptFrom (peer_gater.go:320-363) is evaluated per message copy (every
 *     forwarded message and every IWANT answer is its own RPC) against the
 *     state at the start of the round; rand.Float64() is a Philox-keyed
 *     uniform (round, receiver, slot | purpose, sender).  AcceptControl drops
 *     the message and calls ThrottlePeer (gossip_tracer.go:182-200: the
 *     receiver's promises from that peer are forgotten).  Control-only RPCs
 *     are not gated.
 *   * The tracer events of a round are counted as integers and added once at
 *     the end of the round (deliveries weighted by TopicDeliveryWeights in
 *     fixed point, 2^-16 units), so the sums do not depend on the order in
 *     which a round's copies are handled.
 *   * decayStats (:207-241) runs once per heartbeat, at the score refresh.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

#define GATER_NONE_KEY 0xFFFFFFFFu   /* "<unknown>": a peer without an IP */
#define GATER_NEVER INT64_MIN         /* lastThrottle before any throttle: time.Time{} */

struct orc_gater {
    gsim_peer_gater_params p;
    int64_t n, e;
    int32_t t;
    uint64_t* tw;          /* [T] delivery weight per topic, 2^-16 units (0 -> 1.0) */
    double *val, *thr;     /* [N] */
    int64_t* last;         /* [N] */
    uint32_t* rep;         /* [E] representative edge of (row owner, IP key of col[e]) */
    double *del, *dup, *ign, *rej;   /* [E] at representative edges */
    int32_t* con;          /* [E] connected peers of the group */
    int64_t* exp;          /* [E] retention expiry while con == 0 */
    uint64_t* a_del;       /* [E] this round's events, fixed point */
    uint32_t *a_dup, *a_ign, *a_rej;
    uint32_t *a_val, *a_thr;   /* [N] */
    uint8_t* a_last;       /* [N] a throttled validation this round */
    uint8_t* act;          /* [N] AcceptFrom may throttle this round */
    int64_t throttled;     /* copies dropped (AcceptControl) */
};

static uint32_t ip_key(const orc_net* s, uint32_t p)
{
    if (!s->ip_ptr || s->ip_ptr[p] == s->ip_ptr[p + 1]) return GATER_NONE_KEY;
    return s->ip_ids[s->ip_ptr[p]];
}

int orc_gater_validate(const gsim_peer_gater_params* p)
{
    /* PeerGaterParams.validate (peer_gater.go:57-90) */
    if (p->threshold <= 0) return 1;
    if (p->global_decay <= 0 || p->global_decay >= 1) return 2;
    if (p->source_decay <= 0 || p->source_decay >= 1) return 3;
    if (p->decay_interval_ns < 1000000000LL) return 4;
    if (p->decay_to_zero <= 0 || p->decay_to_zero >= 1) return 5;
    if (p->quiet_ns < 1000000000LL) return 6;
    if (p->duplicate_weight <= 0) return 7;
    if (p->ignore_weight < 1) return 8;
    if (p->reject_weight < 1) return 9;
    return 0;
}

uint64_t orc_gater_weight_fp(double w)
{
    /* TopicDeliveryWeights[topic], 0 -> 1 (peer_gater.go:374-381), in 2^-16 units */
    if (w == 0) w = 1;
    return (uint64_t)llround(w * 65536.0);
}

orc_gater* orc_gater_new(orc_net* s, const gsim_peer_gater_params* p, const double* topic_w)
{
    orc_gater* g = (orc_gater*)calloc(1, sizeof(orc_gater));
    g->p = *p;
    g->n = s->n; g->e = s->e; g->t = s->t;
    const size_t N = (size_t)s->n, E = (size_t)s->e, T = (size_t)(s->t > 0 ? s->t : 1);
    g->tw = (uint64_t*)malloc(T * 8);
    for (size_t t = 0; t < T; ++t) g->tw[t] = orc_gater_weight_fp(topic_w ? topic_w[t] : 0.0);
    g->val = (double*)calloc(N, 8); g->thr = (double*)calloc(N, 8);
    g->last = (int64_t*)malloc(N * 8);
    for (size_t i = 0; i < N; ++i) g->last[i] = GATER_NEVER;
    g->rep = (uint32_t*)malloc(E * 4);
    g->del = (double*)calloc(E, 8); g->dup = (double*)calloc(E, 8);
    g->ign = (double*)calloc(E, 8); g->rej = (double*)calloc(E, 8);
    g->con = (int32_t*)calloc(E, 4); g->exp = (int64_t*)calloc(E, 8);
    g->a_del = (uint64_t*)calloc(E, 8);
    g->a_dup = (uint32_t*)calloc(E, 4); g->a_ign = (uint32_t*)calloc(E, 4); g->a_rej = (uint32_t*)calloc(E, 4);
    g->a_val = (uint32_t*)calloc(N, 4); g->a_thr = (uint32_t*)calloc(N, 4);
    g->a_last = (uint8_t*)calloc(N, 1); g->act = (uint8_t*)calloc(N, 1);
    for (int64_t i = 0; i < s->n; ++i)
        for (uint32_t e = s->row_ptr[i]; e < s->row_ptr[i + 1]; ++e) {
            const uint32_t k = ip_key(s, s->col[e]);
            uint32_t r = e;
            for (uint32_t f = s->row_ptr[i]; f < e; ++f)
                if (ip_key(s, s->col[f]) == k) { r = f; break; }
            g->rep[e] = r;
            /* AddPeer of every connection the router already has (peer_gater.go:370-376) */
            if (s->estate[e] & GSIM_ES_CONNECTED) g->con[r]++;
        }
    s->gater = g;
    return g;
}

void orc_gater_free(orc_gater* g)
{
    if (!g) return;
    free(g->tw); free(g->val); free(g->thr); free(g->last); free(g->rep);
    free(g->del); free(g->dup); free(g->ign); free(g->rej); free(g->con); free(g->exp);
    free(g->a_del); free(g->a_dup); free(g->a_ign); free(g->a_rej);
    free(g->a_val); free(g->a_thr); free(g->a_last); free(g->act);
    free(g);
}

/* AcceptFrom's preamble (peer_gater.go:327-343) at round time now: whether
 * router i may throttle at all this round. */
void orc_gater_round_begin(orc_net* s, int64_t now)
{
    orc_gater* g = s->gater;
    if (!g) return;
    for (int64_t i = 0; i < g->n; ++i) {
        int a = 1;
        if (g->last[i] == GATER_NEVER || now - g->last[i] > g->p.quiet_ns) a = 0;   /* quiet */
        else if (g->thr[i] == 0) a = 0;
        else if (g->val[i] != 0 && g->thr[i] / g->val[i] < g->p.threshold) a = 0;
        g->act[i] = (uint8_t)a;
    }
}

double orc_gater_uniform(uint64_t seed, int64_t g, uint32_t recv, uint32_t slot, uint32_t sender)
{
    uint32_t ctr[4] = {(uint32_t)g, recv, (slot << 8) | P_GATER, sender};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    orc_philox4x32_10(ctr, key, out);
    const uint64_t r53 = ((uint64_t)out[0] << 21) | (out[1] >> 11);
    return (double)r53 * (1.0 / 9007199254740992.0);
}

/* AcceptFrom(p) at router i for a copy over i's edge er (peer_gater.go:320-363):
 * 1 = AcceptAll, 0 = AcceptControl (the caller drops the message). */
int orc_gater_accept(orc_net* s, uint64_t seed, int64_t g_round, uint32_t i, uint32_t er, uint32_t slot)
{
    orc_gater* g = s->gater;
    if (!g || !g->act[i]) return 1;
    const uint32_t r = g->rep[er];
    const double total = g->del[r] + g->p.duplicate_weight * g->dup[r] + g->p.ignore_weight * g->ign[r] +
                         g->p.reject_weight * g->rej[r];
    if (total == 0) return 1;
    const double threshold = (1 + g->del[r]) / (1 + total);
    if (orc_gater_uniform(seed, g_round, i, slot, s->col[er]) < threshold) return 1;
#pragma omp atomic
    g->throttled++;
    return 0;
}

/* one RawTracer event of the gater at router i about the peer of edge er
 * (peer_gater.go:386-432), counted for the end of the round */
void orc_gater_event(orc_net* s, uint32_t i, uint32_t er, int32_t topic, int32_t kind)
{
    orc_gater* g = s->gater;
    if (!g) return;
    const uint32_t r = g->rep[er];
    switch (kind) {
    case ORC_GATE_VALIDATE: g->a_val[i]++; break;                      /* ValidateMessage   :386-391 */
    case ORC_GATE_DELIVER: g->a_del[r] += g->tw[topic]; break;         /* DeliverMessage    :393-406 */
    case ORC_GATE_DUPLICATE: g->a_dup[r]++; break;                     /* DuplicateMessage  :425-432 */
    case ORC_GATE_IGNORE: g->a_ign[r]++; break;                        /* RejectValidationIgnored :414-416 */
    case ORC_GATE_REJECT: g->a_rej[r]++; break;                        /* any other reason  :418-420 */
    case ORC_GATE_THROTTLE:                                            /* throttled / queue full :404-412 */
        g->a_thr[i]++;
        g->a_last[i] = 1;
        break;
    }
}

/* the round's events into the counters (end of round at time now) */
void orc_gater_round_end(orc_net* s, int64_t now)
{
    orc_gater* g = s->gater;
    if (!g) return;
    for (int64_t i = 0; i < g->n; ++i) {
        if (g->a_val[i]) g->val[i] += (double)g->a_val[i];
        if (g->a_thr[i]) g->thr[i] += (double)g->a_thr[i];
        if (g->a_last[i]) g->last[i] = now;
        g->a_val[i] = g->a_thr[i] = 0;
        g->a_last[i] = 0;
    }
    for (int64_t r = 0; r < g->e; ++r) {
        if (g->a_del[r]) g->del[r] += (double)g->a_del[r] * (1.0 / 65536.0);
        if (g->a_dup[r]) g->dup[r] += (double)g->a_dup[r];
        if (g->a_ign[r]) g->ign[r] += (double)g->a_ign[r];
        if (g->a_rej[r]) g->rej[r] += (double)g->a_rej[r];
        g->a_del[r] = 0;
        g->a_dup[r] = g->a_ign[r] = g->a_rej[r] = 0;
    }
}

static double decay1(double x, double d, double dtz)
{
    x *= d;
    return x < dtz ? 0 : x;
}

/* decayStats (peer_gater.go:207-241) at time now */
void orc_gater_decay(orc_net* s, int64_t now)
{
    orc_gater* g = s->gater;
    if (!g) return;
    const double dtz = g->p.decay_to_zero;
    for (int64_t i = 0; i < g->n; ++i) {
        g->val[i] = decay1(g->val[i], g->p.global_decay, dtz);
        g->thr[i] = decay1(g->thr[i], g->p.global_decay, dtz);
    }
    for (int64_t r = 0; r < g->e; ++r) {
        if (g->rep[r] != (uint32_t)r) continue;
        if (g->con[r] > 0) {
            g->del[r] = decay1(g->del[r], g->p.source_decay, dtz);
            g->dup[r] = decay1(g->dup[r], g->p.source_decay, dtz);
            g->ign[r] = decay1(g->ign[r], g->p.source_decay, dtz);
            g->rej[r] = decay1(g->rej[r], g->p.source_decay, dtz);
        } else if (g->exp[r] < now) {                 /* delete(pg.ipStats, ip): a fresh object next time */
            g->del[r] = g->dup[r] = g->ign[r] = g->rej[r] = 0;
        }
    }
}

/* AddPeer / RemovePeer of router o's connection e (peer_gater.go:366-384) */
void orc_gater_connection(orc_net* s, int64_t e, int32_t up, int64_t now)
{
    orc_gater* g = s->gater;
    if (!g) return;
    const uint32_t r = g->rep[e];
    if (up) {
        g->con[r]++;
    } else {
        g->con[r]--;
        g->exp[r] = now + g->p.retain_stats_ns;
    }
}

int64_t orc_gater_throttled(const orc_gater* g) { return g ? g->throttled : 0; }

/* the state, for comparison with the engine (gsim_read_field views) */
void orc_gater_read(const orc_gater* g, double* val, double* thr, int64_t* last, double* counters4, int32_t* con,
                    int64_t* exp)
{
    const size_t N = (size_t)g->n, E = (size_t)g->e;
    if (val) memcpy(val, g->val, N * 8);
    if (thr) memcpy(thr, g->thr, N * 8);
    if (last) memcpy(last, g->last, N * 8);
    if (counters4) {
        memcpy(counters4, g->del, E * 8);
        memcpy(counters4 + E, g->dup, E * 8);
        memcpy(counters4 + 2 * E, g->ign, E * 8);
        memcpy(counters4 + 3 * E, g->rej, E * 8);
    }
    if (con) memcpy(con, g->con, E * 4);
    if (exp) memcpy(exp, g->exp, E * 8);
}
