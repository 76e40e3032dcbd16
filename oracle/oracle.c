/*
 * oracle.c — CPU restatement of the reference scoring path.  TEST INFRASTRUCTURE
 * (see oracle.h): the parity checker and the timed CPU baseline, never shipped.
 *
 * Each function cites the reference lines it follows (mouzzarr/go-libp2p-pubsub).
 * Compiled with -ffp-contract=off so every fp64 operation rounds exactly as the
 * reference's Go code (Go never fuses a*b+c into an FMA on amd64).
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TF_IN_MESH GSIM_TF_IN_MESH
#define TF_ACTIVE  GSIM_TF_ACTIVE
#define ES_TRACKED GSIM_ES_TRACKED
#define ES_CONN    GSIM_ES_CONNECTED

static inline int64_t te(const orc_net* s, int32_t t, int64_t e) { return (int64_t)t * s->e + e; }

/* ------------------------------------------------------------------------ */
/* score.go:504-565 refreshScores.  Disconnected peers past their retention are
 * purged (score.go:510-523); retained ones are not decayed.  Connected peers:
 * every counter *= decay and snaps to 0 below DecayToZero (score.go:533-549);
 * meshTime/activation refreshed for in-mesh topics (score.go:550-556); P7
 * counter decays (score.go:559-563). */
void orc_refresh_scores(orc_net* s, int64_t now)
{
    const gsim_peer_score_params* pp = s->pp;
    const double dtz = pp->decay_to_zero;
    /* edges are independent: the OpenMP split gives identical results */
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < s->e; ++e) {
        uint8_t st = s->estate[e];
        if (!(st & ES_TRACKED)) continue;
        if (!(st & ES_CONN)) {
            if (now > s->expire[e]) {                 /* now.After(pstats.expire) */
                s->estate[e] = 0;                     /* delete(ps.peerStats, p) */
                s->bp[e] = 0.0;
                s->expire[e] = 0;
                for (int32_t t = 0; t < s->t; ++t) {
                    int64_t i = te(s, t, e);
                    s->first[i] = s->meshd[i] = s->fail[i] = s->invalid[i] = 0.0;
                    s->graft_time[i] = s->mesh_time[i] = 0;
                    s->tflags[i] &= (uint8_t)(GSIM_TF_MESH | GSIM_TF_FANOUT);   /* router membership is not score state */
                }
            }
            continue;
        }
        for (int32_t t = 0; t < s->t; ++t) {
            const gsim_topic_score_params* tp = &s->tp[t];
            if (!tp->scored) continue;                /* not scoring this topic */
            int64_t i = te(s, t, e);
            double x;
            x = s->first[i] * tp->first_message_deliveries_decay;
            if (x < dtz) x = 0.0;
            s->first[i] = x;
            x = s->meshd[i] * tp->mesh_message_deliveries_decay;
            if (x < dtz) x = 0.0;
            s->meshd[i] = x;
            x = s->fail[i] * tp->mesh_failure_penalty_decay;
            if (x < dtz) x = 0.0;
            s->fail[i] = x;
            x = s->invalid[i] * tp->invalid_message_deliveries_decay;
            if (x < dtz) x = 0.0;
            s->invalid[i] = x;
            if (s->tflags[i] & TF_IN_MESH) {
                int64_t mt = now - s->graft_time[i];  /* now.Sub(tstats.graftTime) */
                s->mesh_time[i] = mt;
                if (mt > tp->mesh_message_deliveries_activation_ns) s->tflags[i] |= TF_ACTIVE;
            } else {
                /* meshTime of a record outside the mesh is never read (score.go:286,
                 * 486) and Graft resets it; the restatement normalizes it to 0 so the
                 * engine may rewrite the plane densely. */
                s->mesh_time[i] = 0;
            }
        }
        double b = s->bp[e] * pp->behaviour_penalty_decay;
        if (b < dtz) b = 0.0;
        s->bp[e] = b;
    }
}

/* score.go:265-342 score(p): per-topic P1..P4 accumulated in ascending topic
 * order, mixed with TopicWeight, capped by TopicScoreCap,
 * then P5, P6, P7. */
double orc_score_edge(const orc_net* s, int64_t e)
{
    if (!(s->estate[e] & ES_TRACKED)) return 0.0;     /* !ok -> 0 */
    const gsim_peer_score_params* pp = s->pp;
    double score = 0.0;
    for (int32_t t = 0; t < s->t; ++t) {
        const gsim_topic_score_params* tp = &s->tp[t];
        if (!tp->scored) continue;
        int64_t i = te(s, t, e);
        uint8_t f = s->tflags[i];
        double ts = 0.0;
        if (f & TF_IN_MESH) {                          /* P1 */
            double p1 = 0.0;
            if (tp->time_in_mesh_quantum_ns != 0)      /* Go would panic on /0 */
                p1 = (double)(s->mesh_time[i] / tp->time_in_mesh_quantum_ns);
            if (p1 > tp->time_in_mesh_cap) p1 = tp->time_in_mesh_cap;
            ts += p1 * tp->time_in_mesh_weight;
        }
        ts += s->first[i] * tp->first_message_deliveries_weight;       /* P2 */
        if (f & TF_ACTIVE) {                                           /* P3 */
            double md = s->meshd[i];
            if (md < tp->mesh_message_deliveries_threshold) {
                double deficit = tp->mesh_message_deliveries_threshold - md;
                double p3 = deficit * deficit;
                ts += p3 * tp->mesh_message_deliveries_weight;
            }
        }
        ts += s->fail[i] * tp->mesh_failure_penalty_weight;            /* P3b */
        double p4 = s->invalid[i] * s->invalid[i];                     /* P4 */
        ts += p4 * tp->invalid_message_deliveries_weight;
        score += ts * tp->topic_weight;
    }
    if (pp->topic_score_cap > 0 && score > pp->topic_score_cap) score = pp->topic_score_cap;
    double p5 = s->p5 ? s->p5[s->col[e]] : 0.0;                        /* P5 */
    score += p5 * pp->app_specific_weight;
    score += s->p6[e] * pp->ip_colocation_factor_weight;               /* P6 */
    if (s->bp[e] > pp->behaviour_penalty_threshold) {                  /* P7 */
        double excess = s->bp[e] - pp->behaviour_penalty_threshold;
        double p7 = excess * excess;
        score += p7 * pp->behaviour_penalty_weight;
    }
    return score;
}

/* OpenMP threads of the parallel phases (the CPU baseline's single-core and
 * all-core legs); returns the number in effect (1 without OpenMP) */
int orc_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

void orc_compute_scores(orc_net* s)
{
#pragma omp parallel for schedule(static)
    for (int64_t e = 0; e < s->e; ++e) s->score[e] = orc_score_edge(s, e);
}

/* score.go:344-388 ipColocationFactor.  peersInIP = len(ps.peerIPs[ip]) counts
 * every tracked peer of this observer (connected or retained) that has the IP
 * (setIPs/removeIPs keep the map in step with peerStats, score.go:1028-1081). */
void orc_ip_colocation(orc_net* s)
{
    const int32_t thr = s->pp->ip_colocation_factor_threshold;
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < s->n; ++i) {
        uint32_t b = s->row_ptr[i], en = s->row_ptr[i + 1];
        for (uint32_t e = b; e < en; ++e) {
            double res = 0.0;
            if (s->estate[e] & ES_TRACKED) {
                uint32_t j = s->col[e];
                for (uint32_t q = s->ip_ptr[j]; q < s->ip_ptr[j + 1]; ++q) {
                    uint32_t ip = s->ip_ids[q];
                    if (s->ip_white && s->ip_white[ip]) continue;   /* whitelisted */
                    int32_t cnt = 0;
                    for (uint32_t e2 = b; e2 < en; ++e2) {
                        if (!(s->estate[e2] & ES_TRACKED)) continue;
                        uint32_t j2 = s->col[e2];
                        for (uint32_t q2 = s->ip_ptr[j2]; q2 < s->ip_ptr[j2 + 1]; ++q2)
                            if (s->ip_ids[q2] == ip) { ++cnt; break; }
                    }
                    if (cnt > thr) {
                        double surplus = (double)(cnt - thr);
                        res += surplus * surplus;
                    }
                }
            }
            s->p6[e] = res;
        }
    }
}

/* score.go:391-405 AddPenalty. */
void orc_add_penalty(orc_net* s, int64_t e, int32_t count)
{
    if (!(s->estate[e] & ES_TRACKED)) return;
    s->bp[e] += (double)count;
}

/* score.go:649-667 Graft (getTopicStats creates stats only for scored topics,
 * score.go:882-897). */
void orc_graft(orc_net* s, int64_t e, int32_t topic, int64_t now)
{
    if (!(s->estate[e] & ES_TRACKED)) return;
    if (!s->tp[topic].scored) return;
    int64_t i = te(s, topic, e);
    s->tflags[i] = (uint8_t)((s->tflags[i] | TF_IN_MESH) & ~TF_ACTIVE);
    s->graft_time[i] = now;
    s->mesh_time[i] = 0;
}

/* score.go:669-691 Prune: sticky P3b penalty when the mesh delivery deficit is
 * active; meshMessageDeliveriesActive is deliberately NOT cleared. */
void orc_prune(orc_net* s, int64_t e, int32_t topic)
{
    if (!(s->estate[e] & ES_TRACKED)) return;
    if (!s->tp[topic].scored) return;
    int64_t i = te(s, topic, e);
    double thr = s->tp[topic].mesh_message_deliveries_threshold;
    if ((s->tflags[i] & TF_ACTIVE) && s->meshd[i] < thr) {
        double deficit = thr - s->meshd[i];
        s->fail[i] += deficit * deficit;
    }
    /* meshTime outside the mesh is never read; normalized to 0 */
    if (s->tflags[i] & TF_IN_MESH) s->mesh_time[i] = 0;
    s->tflags[i] &= (uint8_t)~TF_IN_MESH;
}

/* score.go:595-609 AddPeer. */
void orc_add_peer(orc_net* s, int64_t e)
{
    if (!(s->estate[e] & ES_TRACKED)) {
        s->bp[e] = 0.0;
        s->expire[e] = 0;
        for (int32_t t = 0; t < s->t; ++t) {
            int64_t i = te(s, t, e);
            s->first[i] = s->meshd[i] = s->fail[i] = s->invalid[i] = 0.0;
            s->graft_time[i] = s->mesh_time[i] = 0;
            s->tflags[i] &= (uint8_t)(GSIM_TF_MESH | GSIM_TF_FANOUT);   /* router membership is not score state */
        }
    }
    s->estate[e] = ES_TRACKED | ES_CONN;
}

/* score.go:611-644 RemovePeer: positive scores are dropped, non-positive ones
 * retained for RetainScore with P2 reset and the P3b penalty applied. */
void orc_remove_peer(orc_net* s, int64_t e, int64_t now)
{
    if (!(s->estate[e] & ES_TRACKED)) return;
    if (orc_score_edge(s, e) > 0) {
        s->estate[e] = 0;
        s->bp[e] = 0.0;
        s->expire[e] = 0;
        for (int32_t t = 0; t < s->t; ++t) {
            int64_t i = te(s, t, e);
            s->first[i] = s->meshd[i] = s->fail[i] = s->invalid[i] = 0.0;
            s->graft_time[i] = s->mesh_time[i] = 0;
            s->tflags[i] &= (uint8_t)(GSIM_TF_MESH | GSIM_TF_FANOUT);   /* router membership is not score state */
        }
        return;
    }
    for (int32_t t = 0; t < s->t; ++t) {
        if (!s->tp[t].scored) continue;
        int64_t i = te(s, t, e);
        s->first[i] = 0.0;
        double thr = s->tp[t].mesh_message_deliveries_threshold;
        if ((s->tflags[i] & TF_IN_MESH) && (s->tflags[i] & TF_ACTIVE) && s->meshd[i] < thr) {
            double deficit = thr - s->meshd[i];
            s->fail[i] += deficit * deficit;
        }
        if (s->tflags[i] & TF_IN_MESH) s->mesh_time[i] = 0;   /* as in orc_prune */
        s->tflags[i] &= (uint8_t)~TF_IN_MESH;
    }
    s->estate[e] = ES_TRACKED;                      /* connected = false */
    s->expire[e] = now + s->pp->retain_score_ns;
}

/* score.go:201-241 SetTopicScoreParams: install, recap counters if caps drop. */
void orc_set_topic_params(orc_net* s, int32_t topic, gsim_topic_score_params* slot,
                          const gsim_topic_score_params* np)
{
    gsim_topic_score_params old = *slot;
    *slot = *np;
    if (!old.scored) return;
    int recap = 0;
    if (np->first_message_deliveries_cap < old.first_message_deliveries_cap) recap = 1;
    if (np->mesh_message_deliveries_cap < old.mesh_message_deliveries_cap) recap = 1;
    if (!recap) return;
    for (int64_t e = 0; e < s->e; ++e) {
        if (!(s->estate[e] & ES_TRACKED)) continue;
        int64_t i = te(s, topic, e);
        if (s->first[i] > np->first_message_deliveries_cap) s->first[i] = np->first_message_deliveries_cap;
        if (s->meshd[i] > np->mesh_message_deliveries_cap) s->meshd[i] = np->mesh_message_deliveries_cap;
    }
}

/* score.go:901-914 */
void orc_mark_invalid(orc_net* s, int64_t e, int32_t topic)
{
    if (!(s->estate[e] & ES_TRACKED) || !s->tp[topic].scored) return;
    s->invalid[te(s, topic, e)] += 1;
}

/* score.go:919-946 */
void orc_mark_first(orc_net* s, int64_t e, int32_t topic)
{
    if (!(s->estate[e] & ES_TRACKED) || !s->tp[topic].scored) return;
    const gsim_topic_score_params* tp = &s->tp[topic];
    int64_t i = te(s, topic, e);
    double x = s->first[i] + 1;
    if (x > tp->first_message_deliveries_cap) x = tp->first_message_deliveries_cap;
    s->first[i] = x;
    if (!(s->tflags[i] & TF_IN_MESH)) return;
    x = s->meshd[i] + 1;
    if (x > tp->mesh_message_deliveries_cap) x = tp->mesh_message_deliveries_cap;
    s->meshd[i] = x;
}

/* score.go:951-981; has_validated = !validated.IsZero(). */
void orc_mark_duplicate(orc_net* s, int64_t e, int32_t topic, int32_t has_validated,
                        int64_t validated, int64_t now)
{
    if (!(s->estate[e] & ES_TRACKED) || !s->tp[topic].scored) return;
    int64_t i = te(s, topic, e);
    if (!(s->tflags[i] & TF_IN_MESH)) return;
    const gsim_topic_score_params* tp = &s->tp[topic];
    if (has_validated && (now - validated) > tp->mesh_message_deliveries_window_ns) return;
    double x = s->meshd[i] + 1;
    if (x > tp->mesh_message_deliveries_cap) x = tp->mesh_message_deliveries_cap;
    s->meshd[i] = x;
}

/* ------------------------------------------------------------------------ */
/* Delivery records, score.go:90-120 and 693-877 (one observer). */
enum { D_UNKNOWN = 0, D_VALID, D_INVALID, D_IGNORED, D_THROTTLED };

typedef struct drec {
    uint64_t mid;
    int32_t status;
    int32_t live;
    int64_t first_seen, validated, expire;
    int64_t* peers;       /* edge ids; NULL after release (peers = nil) */
    int32_t npeers, cappeers;
    int32_t peers_nil;
} drec;

struct orc_drecs {
    int64_t ttl;
    drec* r;
    int32_t n, cap;
    int32_t head;         /* gc queue = creation order */
};

orc_drecs* orc_drecs_new(int64_t seen_ttl)
{
    orc_drecs* d = (orc_drecs*)calloc(1, sizeof(orc_drecs));
    d->ttl = seen_ttl ? seen_ttl : 120000000000LL;   /* TimeCacheDuration, pubsub.go:32 */
    return d;
}

void orc_drecs_free(orc_drecs* d)
{
    if (!d) return;
    for (int32_t i = 0; i < d->n; ++i) free(d->r[i].peers);
    free(d->r);
    free(d);
}

/* score.go:840-861 getRecord */
static drec* get_record(orc_drecs* d, uint64_t mid, int64_t now)
{
    for (int32_t i = d->head; i < d->n; ++i)
        if (d->r[i].live && d->r[i].mid == mid) return &d->r[i];
    if (d->n == d->cap) {
        d->cap = d->cap ? 2 * d->cap : 16;
        d->r = (drec*)realloc(d->r, sizeof(drec) * (size_t)d->cap);
    }
    drec* r = &d->r[d->n++];
    memset(r, 0, sizeof(*r));
    r->mid = mid;
    r->live = 1;
    r->status = D_UNKNOWN;
    r->first_seen = now;
    r->expire = now + d->ttl;
    return r;
}

static int drec_has_peer(const drec* r, int64_t e)
{
    for (int32_t i = 0; i < r->npeers; ++i) if (r->peers[i] == e) return 1;
    return 0;
}

static void drec_add_peer(drec* r, int64_t e)
{
    if (r->npeers == r->cappeers) {
        r->cappeers = r->cappeers ? 2 * r->cappeers : 8;
        r->peers = (int64_t*)realloc(r->peers, sizeof(int64_t) * (size_t)r->cappeers);
    }
    r->peers[r->npeers++] = e;
}

static void drec_release(drec* r) { r->npeers = 0; r->peers_nil = 1; }

void orc_validate_message(orc_net* s, orc_drecs* d, uint64_t mid, int64_t now)
{
    (void)s;
    (void)get_record(d, mid, now);
}

void orc_deliver_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                         int32_t topic, int64_t now)
{
    orc_mark_first(s, from_e, topic);
    drec* r = get_record(d, mid, now);
    if (r->status != D_UNKNOWN) return;
    r->status = D_VALID;
    r->validated = now;
    for (int32_t i = 0; i < r->npeers; ++i)
        if (r->peers[i] != from_e) orc_mark_duplicate(s, r->peers[i], topic, 0, 0, now);
}

void orc_reject_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                        int32_t topic, int32_t reason, int64_t now)
{
    switch (reason) {
    case ORC_REJECT_MISSING_SIGNATURE: case ORC_REJECT_INVALID_SIGNATURE:
    case ORC_REJECT_UNEXPECTED_SIGNATURE: case ORC_REJECT_UNEXPECTED_AUTH_INFO:
    case ORC_REJECT_SELF_ORIGIN:
        orc_mark_invalid(s, from_e, topic);
        return;
    case ORC_REJECT_BLACKLISTED_PEER: case ORC_REJECT_BLACKLISTED_SOURCE:
    case ORC_REJECT_VALIDATION_QUEUE_FULL:
        return;
    default: break;
    }
    drec* r = get_record(d, mid, now);
    if (r->status != D_UNKNOWN) return;
    if (reason == ORC_REJECT_VALIDATION_THROTTLED) { r->status = D_THROTTLED; drec_release(r); return; }
    if (reason == ORC_REJECT_VALIDATION_IGNORED)   { r->status = D_IGNORED;   drec_release(r); return; }
    r->status = D_INVALID;
    orc_mark_invalid(s, from_e, topic);
    for (int32_t i = 0; i < r->npeers; ++i) orc_mark_invalid(s, r->peers[i], topic);
    drec_release(r);
}

void orc_duplicate_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                           int32_t topic, int64_t now)
{
    drec* r = get_record(d, mid, now);
    if (drec_has_peer(r, from_e)) return;          /* already seen this duplicate */
    switch (r->status) {
    case D_UNKNOWN:
        drec_add_peer(r, from_e);
        break;
    case D_VALID:
        drec_add_peer(r, from_e);
        orc_mark_duplicate(s, from_e, topic, 1, r->validated, now);
        break;
    case D_INVALID:
        orc_mark_invalid(s, from_e, topic);
        break;
    default:                                         /* throttled / ignored */
        break;
    }
}

/* score.go:863-877 gc: drop records whose expiry is strictly in the past. */
void orc_drecs_gc(orc_drecs* d, int64_t now)
{
    while (d->head < d->n && now > d->r[d->head].expire) {
        d->r[d->head].live = 0;
        free(d->r[d->head].peers);
        d->r[d->head].peers = NULL;
        d->head++;
    }
}

void orc_drecs_expire_head(orc_drecs* d, int64_t expire)
{
    if (d->head < d->n) d->r[d->head].expire = expire;
}

/* ------------------------------------------------------------------------ */
/* mcache.go: MessageCache with `history` windows; gossip ids come from the
 * first `gossip` windows in window order then insertion order. */
typedef struct mc_entry { uint64_t mid; int32_t topic; } mc_entry;
typedef struct mc_win { mc_entry* v; int32_t n, cap; } mc_win;
typedef struct mc_tx { uint64_t mid; uint32_t peer; int32_t count; } mc_tx;

struct orc_mcache {
    int32_t gossip, history;
    mc_win* win;                 /* win[0] = newest */
    uint64_t* msgs; int32_t nmsgs, capmsgs;
    mc_tx* tx; int32_t ntx, captx;
};

orc_mcache* orc_mcache_new(int32_t gossip, int32_t history)
{
    if (gossip > history) return NULL;   /* NewMessageCache panics, mcache.go:22-26 */
    orc_mcache* m = (orc_mcache*)calloc(1, sizeof(orc_mcache));
    m->gossip = gossip;
    m->history = history;
    m->win = (mc_win*)calloc((size_t)history, sizeof(mc_win));
    return m;
}

void orc_mcache_free(orc_mcache* m)
{
    if (!m) return;
    for (int32_t i = 0; i < m->history; ++i) free(m->win[i].v);
    free(m->win); free(m->msgs); free(m->tx); free(m);
}

static int mc_find_msg(orc_mcache* m, uint64_t mid)
{
    for (int32_t i = 0; i < m->nmsgs; ++i) if (m->msgs[i] == mid) return i;
    return -1;
}

void orc_mcache_put(orc_mcache* m, uint64_t mid, int32_t topic)
{
    if (mc_find_msg(m, mid) < 0) {
        if (m->nmsgs == m->capmsgs) {
            m->capmsgs = m->capmsgs ? 2 * m->capmsgs : 64;
            m->msgs = (uint64_t*)realloc(m->msgs, sizeof(uint64_t) * (size_t)m->capmsgs);
        }
        m->msgs[m->nmsgs++] = mid;
    }
    mc_win* w = &m->win[0];
    if (w->n == w->cap) {
        w->cap = w->cap ? 2 * w->cap : 16;
        w->v = (mc_entry*)realloc(w->v, sizeof(mc_entry) * (size_t)w->cap);
    }
    w->v[w->n].mid = mid;
    w->v[w->n].topic = topic;
    w->n++;
}

int orc_mcache_get(orc_mcache* m, uint64_t mid) { return mc_find_msg(m, mid) >= 0; }

int orc_mcache_get_for_peer(orc_mcache* m, uint64_t mid, uint32_t peer, int32_t* count)
{
    if (mc_find_msg(m, mid) < 0) { *count = 0; return 0; }
    for (int32_t i = 0; i < m->ntx; ++i)
        if (m->tx[i].mid == mid && m->tx[i].peer == peer) { *count = ++m->tx[i].count; return 1; }
    if (m->ntx == m->captx) {
        m->captx = m->captx ? 2 * m->captx : 64;
        m->tx = (mc_tx*)realloc(m->tx, sizeof(mc_tx) * (size_t)m->captx);
    }
    m->tx[m->ntx].mid = mid; m->tx[m->ntx].peer = peer; m->tx[m->ntx].count = 1;
    m->ntx++;
    *count = 1;
    return 1;
}

int orc_mcache_gossip_ids(orc_mcache* m, int32_t topic, uint64_t* out, int32_t cap)
{
    int32_t n = 0;
    for (int32_t w = 0; w < m->gossip; ++w)
        for (int32_t i = 0; i < m->win[w].n; ++i)
            if (m->win[w].v[i].topic == topic) {
                if (n < cap) out[n] = m->win[w].v[i].mid;
                ++n;
            }
    return n;
}

void orc_mcache_shift(orc_mcache* m)
{
    mc_win last = m->win[m->history - 1];
    for (int32_t i = 0; i < last.n; ++i) {
        uint64_t mid = last.v[i].mid;
        int32_t k = mc_find_msg(m, mid);
        if (k >= 0) m->msgs[k] = m->msgs[--m->nmsgs];
        for (int32_t q = 0; q < m->ntx;) {
            if (m->tx[q].mid == mid) m->tx[q] = m->tx[--m->ntx];
            else ++q;
        }
    }
    free(last.v);
    for (int32_t i = m->history - 2; i >= 0; --i) m->win[i + 1] = m->win[i];
    memset(&m->win[0], 0, sizeof(mc_win));
}

int orc_mcache_len(orc_mcache* m) { return m->nmsgs; }

/* ------------------------------------------------------------------------ */
/* gossip_tracer.go: promises[mid][peer] = expire. */
typedef struct gt_prom { uint64_t mid; uint32_t peer; int64_t expire; } gt_prom;
struct orc_gtracer { int64_t followup; gt_prom* p; int32_t n, cap; };

orc_gtracer* orc_gtracer_new(int64_t followup)
{
    orc_gtracer* g = (orc_gtracer*)calloc(1, sizeof(orc_gtracer));
    g->followup = followup;
    return g;
}

void orc_gtracer_free(orc_gtracer* g) { if (g) { free(g->p); free(g); } }

void orc_gtracer_add_promise(orc_gtracer* g, uint32_t peer, const uint64_t* mids, int32_t n,
                             int32_t pick, int64_t now)
{
    if (n <= 0) return;
    uint64_t mid = mids[pick];
    for (int32_t i = 0; i < g->n; ++i)
        if (g->p[i].mid == mid && g->p[i].peer == peer) return;   /* already promised */
    if (g->n == g->cap) {
        g->cap = g->cap ? 2 * g->cap : 64;
        g->p = (gt_prom*)realloc(g->p, sizeof(gt_prom) * (size_t)g->cap);
    }
    g->p[g->n].mid = mid; g->p[g->n].peer = peer; g->p[g->n].expire = now + g->followup;
    g->n++;
}

static int cmp_u32(const void* a, const void* b)
{
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

int orc_gtracer_broken(orc_gtracer* g, int64_t now, uint32_t* peers, int32_t* counts, int32_t cap)
{
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(g->n + 1));
    int32_t nb = 0;
    for (int32_t i = 0; i < g->n;) {
        if (g->p[i].expire < now) {                  /* expire.Before(now) */
            tmp[nb++] = g->p[i].peer;
            g->p[i] = g->p[--g->n];
        } else ++i;
    }
    qsort(tmp, (size_t)nb, sizeof(uint32_t), cmp_u32);
    int32_t np = 0;
    for (int32_t i = 0; i < nb;) {
        int32_t j = i;
        while (j < nb && tmp[j] == tmp[i]) ++j;
        if (np < cap) { peers[np] = tmp[i]; counts[np] = j - i; }
        ++np;
        i = j;
    }
    free(tmp);
    return np;
}

void orc_gtracer_fulfill(orc_gtracer* g, uint64_t mid)
{
    for (int32_t i = 0; i < g->n;) {
        if (g->p[i].mid == mid) g->p[i] = g->p[--g->n];
        else ++i;
    }
}

void orc_gtracer_throttle(orc_gtracer* g, uint32_t peer)
{
    for (int32_t i = 0; i < g->n;) {
        if (g->p[i].peer == peer) g->p[i] = g->p[--g->n];
        else ++i;
    }
}

int orc_gtracer_peer_promises(orc_gtracer* g)
{
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(g->n + 1));
    for (int32_t i = 0; i < g->n; ++i) tmp[i] = g->p[i].peer;
    qsort(tmp, (size_t)g->n, sizeof(uint32_t), cmp_u32);
    int32_t np = 0;
    for (int32_t i = 0; i < g->n; ++i) if (i == 0 || tmp[i] != tmp[i - 1]) ++np;
    free(tmp);
    return np;
}

/* ------------------------------------------------------------------------ */
/* timecache/: FirstSeenCache (expiry fixed at first Add) and LastSeenCache
 * (expiry slides on Add and Has); background sweep drops expiry < now. */
typedef struct tc_ent { uint64_t id; int64_t expiry; } tc_ent;
struct orc_tcache { int32_t strategy; int64_t ttl; tc_ent* v; int32_t n, cap; };

orc_tcache* orc_tcache_new(int32_t strategy, int64_t ttl)
{
    orc_tcache* c = (orc_tcache*)calloc(1, sizeof(orc_tcache));
    c->strategy = strategy;
    c->ttl = ttl;
    return c;
}

void orc_tcache_free(orc_tcache* c) { if (c) { free(c->v); free(c); } }

static int tc_find(orc_tcache* c, uint64_t id)
{
    for (int32_t i = 0; i < c->n; ++i) if (c->v[i].id == id) return i;
    return -1;
}

int orc_tcache_add(orc_tcache* c, uint64_t id, int64_t now)
{
    int32_t k = tc_find(c, id);
    if (k >= 0) {
        if (c->strategy == 1) c->v[k].expiry = now + c->ttl;
        return 0;
    }
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 64;
        c->v = (tc_ent*)realloc(c->v, sizeof(tc_ent) * (size_t)c->cap);
    }
    c->v[c->n].id = id;
    c->v[c->n].expiry = now + c->ttl;
    c->n++;
    return 1;
}

int orc_tcache_has(orc_tcache* c, uint64_t id, int64_t now)
{
    int32_t k = tc_find(c, id);
    if (k < 0) return 0;
    if (c->strategy == 1) c->v[k].expiry = now + c->ttl;
    return 1;
}

void orc_tcache_sweep(orc_tcache* c, int64_t now)
{
    for (int32_t i = 0; i < c->n;) {
        if (c->v[i].expiry < now) c->v[i] = c->v[--c->n];
        else ++i;
    }
}

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11), the counter-based generator the
 * engine uses for every random choice the reference makes with math/rand. */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
