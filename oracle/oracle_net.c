/*
 * oracle_net.c — network-level restatement of the GossipSub heartbeat and
 * control handlers.  TEST INFRASTRUCTURE (see oracle.h).
 *
 * Every observer runs gossipsub.go's heartbeat (1345-1606) on its own row of
 * the CSR graph.  The reference's random choices (shufflePeers, getPeers;
 * gossipsub.go:1908-1973) are restated as "order by a Philox key" so the
 * choice is reproducible; sort.Slice ties are broken by that
 * key.  Observers are independent within a phase, so the OpenMP split over
 * observers gives identical results.
 */
#include "oracle_internal.h"

#include <stdlib.h>
#include <string.h>

#define TF_IN_MESH GSIM_TF_IN_MESH
#define TF_MESH    GSIM_TF_MESH
#define ES_TRACKED GSIM_ES_TRACKED
#define ES_CONN    GSIM_ES_CONNECTED


static const int64_t kSecond = 1000000000LL;
/* clearBackoff adds 2*GossipSubHeartbeatInterval — the package default
 * (gossipsub.go:44), not params.HeartbeatInterval (gossipsub.go:1638). */
static const int64_t kBackoffSlack = 2 * 1000000000LL;

typedef struct cand { uint64_t key; uint32_t e; double score; } cand;

static int cmp_key(const void* a, const void* b)
{
    uint64_t x = ((const cand*)a)->key, y = ((const cand*)b)->key;
    return x < y ? -1 : x > y;
}

typedef struct hb {
    orc_net* s;
    uint32_t i, b, en;
    int32_t t;
    uint64_t tick, seed;
    int64_t now;
    uint8_t* out;            /* inbox buffer the replies/heartbeat messages go to */
    int unsub;               /* the PRUNE being handled is Leave's (GSIM_CTL_UNSUB) */
} hb;

static inline int64_t ti(const hb* h, uint32_t e) { return (int64_t)h->t * h->s->e + e; }
static inline int in_mesh(const hb* h, uint32_t e) { return (h->s->tflags[ti(h, e)] & TF_MESH) != 0; }
static inline int has_backoff(const hb* h, uint32_t e) { return h->s->backoff[ti(h, e)] != 0; }
static inline int topic_peer(const hb* h, uint32_t e)
{
    /* gs.p.topics[topic]: connected peers that announced the subscription */
    return (h->s->estate[e] & ES_CONN) && ((h->s->sub[h->s->col[e]] >> h->t) & 1u);
}

/* gs.direct (WithDirectPeers, gossipsub.go:352-374): never grafted, always sent to */
static inline int is_direct(const hb* h, uint32_t e) { return h->s->direct && h->s->direct[e]; }

static int mesh_count(const hb* h)
{
    int c = 0;
    for (uint32_t e = h->b; e < h->en; ++e) c += in_mesh(h, e);
    return c;
}

/* doAddBackoff, gossipsub.go:881-891: keep the later expiry. */
static void do_add_backoff(hb* h, uint32_t e, int64_t interval)
{
    int64_t expire = h->now + interval;
    int64_t* bo = &h->s->backoff[ti(h, e)];
    if (*bo < expire) *bo = expire;
}

static void send_ctl(hb* h, uint32_t e, uint8_t bits)
{
    h->out[(int64_t)h->t * h->s->e + h->s->rev[e]] |= bits;
}

/* heartbeat prunePeer closure, gossipsub.go:1387-1393 */
static void prune_peer(hb* h, uint32_t e)
{
    orc_log_net(ORC_EV_PRUNE, h->i, h->s->col[e], h->t, h->now);
    orc_prune(h->s, e, h->t);
    h->s->tflags[ti(h, e)] &= (uint8_t)~TF_MESH;
    do_add_backoff(h, e, h->s->gp->prune_backoff_ns);
    send_ctl(h, e, GSIM_CTL_PRUNE);
}

/* heartbeat graftPeer closure, gossipsub.go:1395-1401 */
static void graft_peer(hb* h, uint32_t e)
{
    orc_log_net(ORC_EV_GRAFT, h->i, h->s->col[e], h->t, h->now);
    orc_graft(h->s, e, h->t, h->now);
    h->s->tflags[ti(h, e)] |= TF_MESH;
    send_ctl(h, e, GSIM_CTL_GRAFT);
}

/* Peer exchange of one PRUNE (observer h->i to col[ep], topic h->t):
 * makePrune's getPeers(topic, PrunePeers, xp != p && Score(xp) >= 0)
 * (gossipsub.go:1866-1906) and the pruned peer's handlePrune / pxConnect
 * (860-869, 893-939).  live: Score is the observer's live score (the
 * heartbeat's sendGraftPrune, Leave's sendPrune); else its snapshot
 * (handleGraft's replies, the control rounds' declared divergence).  The keys
 * (opx_key) mix the topic's draw per candidate with the pruned peer's row
 * position: each PRUNE's list is its own shuffle.  The list is what the PRUNE carries, whatever the
 * receiver then does with it (ORC_EV_PX_PEER events, in list order).  The
 * receiver ignores PX from a peer it scores below acceptPXThreshold (its
 * snapshot); every listed peer it is not connected to is a connection
 * attempt, marked at its edge to that peer when the address is known (a CSR
 * edge).  Attempts are resolved between ticks (orc_px_connect).  pend: Leave's
 * PRUNEs -- the receiver handles them with the tick's control (its snapshot
 * after the next refresh), so the list waits in the pending table
 * (px_pending) until orc_px_connect. */
static int64_t find_edge(const orc_net* s, uint32_t i, uint32_t j);

static int px_list(hb* h, uint32_t ep, int live, uint32_t purpose, uint64_t key_tick, cand* c)
{
    orc_net* s = h->s;
    int n = 0;
    for (uint32_t e = h->b; e < h->en; ++e) {
        if (e == ep || !topic_peer(h, e)) continue;
        const double sc = live ? orc_score_edge(s, e) : s->score[e];
        if (sc < 0) continue;
        c[n].key = opx_key(opx_base(h->seed, key_tick, h->i, h->t, purpose, s->col[e]), ep - h->b, e - h->b);
        c[n].e = e;
        c[n].score = sc;
        ++n;
    }
    qsort(c, (size_t)n, sizeof(cand), cmp_key);
    if (n > s->gp->prune_peers) n = s->gp->prune_peers;
    for (int q = 0; q < n; ++q)
        orc_log_net_x(ORC_EV_PX_PEER, h->i, s->col[c[q].e], h->t, s->col[ep], q, h->now);
    return n;
}

/* the pruned peer's handlePrune PX part: acceptPXThreshold, then pxConnect */
static void px_accept(orc_net* s, uint32_t ep, const uint32_t* listed, int n)
{
    if (s->score[s->rev[ep]] < s->th->accept_px_threshold) return;
    const uint32_t p = s->col[ep];
    for (int q = 0; q < n; ++q) {
        const int64_t ex = find_edge(s, p, listed[q]);
        if (ex < 0) continue;                                  /* no known address */
        if (s->estate[ex] & ES_CONN) continue;                 /* pxConnect: already connected */
#pragma omp atomic write
        s->px[ex] = 1;
    }
}

/* Leave's PX lists until orc_px_connect: (pruner's edge, listed peer) per
 * entry, in the network's own table (orc_net.px_pend) */
typedef struct orc_px_pend { uint64_t* ent; int64_t n, cap; } px_pend;

struct orc_px_pend* orc_px_pend_new(void) { return (px_pend*)calloc(1, sizeof(px_pend)); }

void orc_px_pend_free(struct orc_px_pend* p)
{
    if (!p) return;
    free(p->ent);
    free(p);
}

static void px_emit(hb* h, uint32_t ep, int live, uint32_t purpose, uint64_t key_tick, int pend)
{
    orc_net* s = h->s;
    if (!s->px) return;
    const uint32_t deg = h->en - h->b;
    cand buf[1024];
    cand* c = deg <= 1024 ? buf : (cand*)malloc(sizeof(cand) * deg);
    const int n = px_list(h, ep, live, purpose, key_tick, c);
    uint32_t listed[256];
    for (int q = 0; q < n && q < 256; ++q) listed[q] = s->col[c[q].e];
    if (c != buf) free(c);
    if (!pend) {
        px_accept(s, ep, listed, n < 256 ? n : 256);
        return;
    }
    px_pend* pp = s->px_pend;
    if (!pp) return;
    for (int q = 0; q < n && q < 256; ++q) {
        if (pp->n == pp->cap) {
            pp->cap = pp->cap ? 2 * pp->cap : 256;
            pp->ent = (uint64_t*)realloc(pp->ent, sizeof(uint64_t) * (size_t)pp->cap);
        }
        pp->ent[pp->n++] = (uint64_t)ep | ((uint64_t)listed[q] << 32);
    }
}

typedef int (*filter_fn)(const hb* h, uint32_t e, double arg);

/* getPeers, gossipsub.go:1908-1928: filter the topic peers, shuffle (= order
 * by Philox key), truncate to count when count > 0. */
static int get_peers(const hb* h, int count, filter_fn f, double arg, uint32_t purpose, cand* out)
{
    int n = 0;
    for (uint32_t e = h->b; e < h->en; ++e) {
        if (!topic_peer(h, e) || !f(h, e, arg)) continue;
        out[n].key = okey(h->seed, h->tick, h->i, h->t, purpose, h->s->col[e], e - h->b);
        out[n].e = e;
        out[n].score = h->s->score[e];
        ++n;
    }
    qsort(out, (size_t)n, sizeof(cand), cmp_key);
    if (count > 0 && n > count) n = count;
    return n;
}

static int f_graft(const hb* h, uint32_t e, double arg)      /* gossipsub.go:1416-1422 */
{
    (void)arg;
    return !in_mesh(h, e) && !has_backoff(h, e) && !is_direct(h, e) && h->s->score[e] >= 0;
}

static int f_dout(const hb* h, uint32_t e, double arg)       /* gossipsub.go:1506-1512 */
{
    (void)arg;
    return !in_mesh(h, e) && !has_backoff(h, e) && !is_direct(h, e) && h->s->outbound[e] && h->s->score[e] >= 0;
}

static int f_opp(const hb* h, uint32_t e, double median)     /* gossipsub.go:1540-1545 */
{
    return !in_mesh(h, e) && !has_backoff(h, e) && !is_direct(h, e) && h->s->score[e] > median;
}

/* stable insertion sort by score descending (sort.Slice with the score
 * closure; ties keep the prior shuffle order, gossipsub.go:1434-1437) */
static void sort_score_desc(cand* v, int n)
{
    for (int a = 1; a < n; ++a) {
        cand x = v[a];
        int b = a - 1;
        while (b >= 0 && v[b].score < x.score) { v[b + 1] = v[b]; --b; }
        v[b + 1] = x;
    }
}

static int cmp_score_asc(const void* a, const void* b)
{
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

/* Mesh maintenance for one (observer, topic), gossipsub.go:1386-1552. */
static void maintain(hb* h)
{
    orc_net* s = h->s;
    const gsim_gossipsub_params* gp = s->gp;
    cand buf[4096];
    const uint32_t deg = h->en - h->b;
    cand* c = deg <= 4096 ? buf : (cand*)malloc(sizeof(cand) * deg);

    /* drop all peers with negative score, without PX (1403-1410) */
    for (uint32_t e = h->b; e < h->en; ++e)
        if (in_mesh(h, e) && s->score[e] < 0) prune_peer(h, e);

    /* do we have enough peers? (1412-1427) */
    int l = mesh_count(h);
    if (l < gp->dlo) {
        int n = get_peers(h, gp->d - l, f_graft, 0, P_GRAFT_DLO, c);
        for (int q = 0; q < n; ++q) graft_peer(h, c[q].e);
    }

    /* do we have too many peers? (1429-1490) */
    l = mesh_count(h);
    if (l > gp->dhi) {
        int n = 0;
        for (uint32_t e = h->b; e < h->en; ++e) {
            if (!in_mesh(h, e)) continue;
            c[n].key = okey(h->seed, h->tick, h->i, h->t, P_PRUNE_SHUF1, s->col[e], e - h->b);
            c[n].e = e;
            c[n].score = s->score[e];
            ++n;
        }
        qsort(c, (size_t)n, sizeof(cand), cmp_key);           /* shufflePeers(plst) */
        sort_score_desc(c, n);                                 /* sort by score desc */
        int ds = gp->dscore < n ? gp->dscore : n;
        for (int q = ds; q < n; ++q)                           /* shufflePeers(plst[Dscore:]) */
            c[q].key = okey(h->seed, h->tick, h->i, h->t, P_PRUNE_SHUF2, s->col[c[q].e], c[q].e - h->b);
        qsort(c + ds, (size_t)(n - ds), sizeof(cand), cmp_key);
        int outbound = 0;
        for (int q = 0; q < gp->d && q < n; ++q) outbound += s->outbound[c[q].e] != 0;
        if (outbound < gp->dout) {
            #define ROTATE(idx) do { cand p_ = c[idx]; for (int j_ = (idx); j_ > 0; --j_) c[j_] = c[j_ - 1]; c[0] = p_; } while (0)
            if (outbound > 0) {
                int ihave = outbound;
                for (int q = 1; q < gp->d && ihave > 0; ++q)
                    if (s->outbound[c[q].e]) { ROTATE(q); --ihave; }
            }
            int ineed = gp->dout - outbound;
            for (int q = gp->d; q < n && ineed > 0; ++q)
                if (s->outbound[c[q].e]) { ROTATE(q); --ineed; }
            #undef ROTATE
        }
        for (int q = gp->d; q < n; ++q) {
            prune_peer(h, c[q].e);
            /* sendGraftPrune: makePrune(p, topic, doPX && !noPX[p]); noPX marks the
             * negative-score prunes only (1404-1410, 1690) */
            if (gp->do_px) send_ctl(h, c[q].e, GSIM_CTL_PX);
        }
    }

    /* do we have enough outbound peers? (1492-1518) */
    l = mesh_count(h);
    if (l >= gp->dlo) {
        int outbound = 0;
        for (uint32_t e = h->b; e < h->en; ++e) outbound += in_mesh(h, e) && s->outbound[e];
        if (outbound < gp->dout) {
            int n = get_peers(h, gp->dout - outbound, f_dout, 0, P_GRAFT_DOUT, c);
            for (int q = 0; q < n; ++q) graft_peer(h, c[q].e);
        }
    }

    /* opportunistic grafting (1520-1552) */
    l = mesh_count(h);
    if (gp->opportunistic_graft_ticks && h->tick % gp->opportunistic_graft_ticks == 0 && l > 1) {
        double* sc = (double*)malloc(sizeof(double) * (size_t)l);
        int n = 0;
        for (uint32_t e = h->b; e < h->en; ++e) if (in_mesh(h, e)) sc[n++] = s->score[e];
        qsort(sc, (size_t)n, sizeof(double), cmp_score_asc);
        double median = sc[n / 2];
        free(sc);
        if (median < s->th->opportunistic_graft_threshold) {
            int m = get_peers(h, gp->opportunistic_graft_peers, f_opp, median, P_GRAFT_OPP, c);
            for (int q = 0; q < m; ++q) graft_peer(h, c[q].e);
        }
    }
    if (c != buf) free(c);
}

static inline int in_fanout(const hb* h, uint32_t e) { return (h->s->tflags[ti(h, e)] & GSIM_TF_FANOUT) != 0; }

static int f_fanout(const hb* h, uint32_t e, double thr)     /* gossipsub.go:1580-1584, 1020-1023 */
{
    return !in_fanout(h, e) && !is_direct(h, e) && h->s->score[e] >= thr;
}

/* Fanout expiry and maintenance for one observer, after its mesh topics
 * (gossipsub.go:1558-1596): drop fanouts not published to for FanoutTTL;
 * for each remaining fanout topic drop peers that left the topic or score
 * below publishThreshold, top up to D with getPeers, then emitGossip
 * excluding the fanout peers.  Topics in ascending order. */
static void fanout(hb* h, orc_msgs* m)
{
    orc_net* s = h->s;
    if (!s->lastpub || !s->fan_topics) return;
    const gsim_gossipsub_params* gp = s->gp;
    const double thr = s->th->publish_threshold;
    for (int32_t t = 0; t < s->t; ++t) {
        int64_t* lp = &s->lastpub[(int64_t)h->i * s->t + t];
        if (*lp != 0 && *lp + gp->fanout_ttl_ns < h->now) {
            h->t = t;
            for (uint32_t e = h->b; e < h->en; ++e) s->tflags[ti(h, e)] &= (uint8_t)~GSIM_TF_FANOUT;
            s->fan_topics[h->i] &= ~(1ull << t);
            *lp = 0;
        }
    }
    cand buf[4096];
    const uint32_t deg = h->en - h->b;
    cand* c = deg <= 4096 ? buf : (cand*)malloc(sizeof(cand) * deg);
    for (int32_t t = 0; t < s->t; ++t) {
        if (!((s->fan_topics[h->i] >> t) & 1u)) continue;
        h->t = t;
        int have = 0;
        for (uint32_t e = h->b; e < h->en; ++e) {
            if (!in_fanout(h, e)) continue;
            if (!topic_peer(h, e) || s->score[e] < thr) s->tflags[ti(h, e)] &= (uint8_t)~GSIM_TF_FANOUT;
            else ++have;
        }
        if (have < gp->d) {
            const int n = get_peers(h, gp->d - have, f_fanout, thr, P_FANOUT, c);
            for (int q = 0; q < n; ++q) s->tflags[ti(h, c[q].e)] |= GSIM_TF_FANOUT;
        }
        if (m) orc_gossip_emit(s, m, h->i, t, h->tick, h->seed, GSIM_TF_FANOUT);
    }
    if (c != buf) free(c);
}

/* Publish's fanout branch for an origin that has not joined the topic
 * (gossipsub.go:1011-1028): with no fanout peers yet, pick D topic peers
 * with score >= publishThreshold (getPeers, key counter = the round); then
 * lastpub = now.  Scores are the snapshot. */
void orc_fanout_publish(orc_net* s, uint32_t origin, int32_t topic, int64_t g, int64_t now, uint64_t seed)
{
    hb h = {s, origin, s->row_ptr[origin], s->row_ptr[origin + 1], topic, (uint64_t)g, seed, now, NULL, 0};
    int have = 0;
    if ((s->fan_topics[origin] >> topic) & 1u)
        for (uint32_t e = h.b; e < h.en; ++e) have |= in_fanout(&h, e);
    if (!have) {
        cand buf[4096];
        const uint32_t deg = h.en - h.b;
        cand* c = deg <= 4096 ? buf : (cand*)malloc(sizeof(cand) * deg);
        const int n = get_peers(&h, s->gp->d, f_fanout, s->th->publish_threshold, P_FANOUT_NEW, c);
        for (int q = 0; q < n; ++q) s->tflags[ti(&h, c[q].e)] |= GSIM_TF_FANOUT;
        if (n > 0) s->fan_topics[origin] |= 1ull << topic;
        if (c != buf) free(c);
    }
    s->lastpub[(int64_t)origin * s->t + topic] = now;
}

/* The network's Philox seed as the last heartbeat received it: the control
 * rounds' PX choices (GRAFT replies) use it too. */
static uint64_t g_px_seed;

void orc_heartbeat_gossip(orc_net* s, orc_msgs* m, uint64_t tick, int64_t now, uint64_t seed)
{
    g_px_seed = seed;
    uint8_t* out = s->ctl;   /* heartbeat output = parity-0 inbox, handled in round 0 */
    if (m) {
        priv* p = orc_msgs_priv(m);
        const size_t te = (size_t)s->t * (size_t)s->e;
        if (!p->ihave || p->te_alloc != (int64_t)te) {
            free(p->ihave);
            p->ihave = (uint8_t*)calloc(te ? te : 1, 1);
            p->te_alloc = (int64_t)te;
        }
        memset(p->ihave, 0, te);
        p->ihave_tick = (int64_t)tick;
        p->seed = seed;
        orc_gossip_index(s, m, (int64_t)tick);
        if (!p->npr) {
            p->pr = (promise**)calloc((size_t)s->n, sizeof(promise*));
            p->npr = (int32_t*)calloc((size_t)s->n, sizeof(int32_t));
            p->cappr = (int32_t*)calloc((size_t)s->n, sizeof(int32_t));
            p->n_alloc = s->n;
        }
    }
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < s->n; ++i) {
        hb h = {s, (uint32_t)i, s->row_ptr[i], s->row_ptr[i + 1], 0, tick, seed, now, out, 0};
        /* clearBackoff every 15 ticks (gossipsub.go:1627-1646) */
        if (tick % 15 == 0)
            for (int32_t t = 0; t < s->t; ++t)
                for (uint32_t e = h.b; e < h.en; ++e) {
                    int64_t* bo = &s->backoff[(int64_t)t * s->e + e];
                    if (*bo != 0 && *bo + kBackoffSlack < now) *bo = 0;
                }
        /* maintain the mesh for topics we have joined (1385-1557), each
         * followed by emitGossip(topic, mesh) */
        for (int32_t t = 0; t < s->t; ++t) {
            if (!((s->sub[i] >> t) & 1u)) continue;
            h.t = t;
            maintain(&h);
            if (m) orc_gossip_emit(s, m, (uint32_t)i, t, tick, seed, GSIM_TF_MESH);
        }
        /* sendGraftPrune (1672-1707) after every topic: PX with the live scores */
        if (s->gp->do_px)
            for (int32_t t = 0; t < s->t; ++t) {
                h.t = t;
                for (uint32_t e = h.b; e < h.en; ++e)
                    /* (a Leave's PRUNE in the same inbox was listed at the Leave) */
                    if ((out[(int64_t)t * s->e + s->rev[e]] & (GSIM_CTL_PX | GSIM_CTL_UNSUB)) == GSIM_CTL_PX)
                        px_emit(&h, e, 1, P_PX, tick, 0);
            }
        fanout(&h, m);
    }
}

void orc_heartbeat(orc_net* s, uint64_t tick, int64_t now, uint64_t seed)
{
    orc_heartbeat_gossip(s, NULL, tick, now, seed);
}

/* handleGraft for one (receiver, sender edge, topic), gossipsub.go:748-825.
 * Returns 1 when the GRAFT turns off PX for the whole RPC (doPX = false:
 * unknown topic, direct peer, backoff, negative score). */
static int handle_graft(hb* h, uint32_t e)
{
    orc_net* s = h->s;
    const gsim_gossipsub_params* gp = s->gp;
    if (!((s->sub[h->i] >> h->t) & 1u)) return 1;             /* unknown topic: ignore, no PX */
    if (in_mesh(h, e)) return 0;                               /* already in mesh */
    if (is_direct(h, e)) {                                     /* no GRAFT from direct peers: PRUNE */
        send_ctl(h, e, GSIM_CTL_PRUNE);
        return 1;
    }
    int64_t expire = s->backoff[ti(h, e)];
    if (expire != 0 && h->now < expire) {                      /* backing off that peer */
        orc_add_penalty(s, e, 1);
        int64_t flood_cutoff = expire + (gp->graft_flood_threshold_ns - gp->prune_backoff_ns);
        if (h->now < flood_cutoff) orc_add_penalty(s, e, 1);
        do_add_backoff(h, e, gp->prune_backoff_ns);
        send_ctl(h, e, GSIM_CTL_PRUNE);
        return 1;
    }
    if (s->score[e] < 0) {                                     /* negative score */
        send_ctl(h, e, GSIM_CTL_PRUNE);
        do_add_backoff(h, e, gp->prune_backoff_ns);
        return 1;
    }
    if (mesh_count(h) >= gp->dhi && !s->outbound[e]) {         /* mesh full, inbound: PRUNE with PX */
        send_ctl(h, e, (uint8_t)(GSIM_CTL_PRUNE | (gp->do_px ? GSIM_CTL_PX : 0)));
        do_add_backoff(h, e, gp->prune_backoff_ns);
        return 0;
    }
    orc_log_net(ORC_EV_GRAFT, h->i, s->col[e], h->t, h->now);
    orc_graft(s, e, h->t, h->now);                             /* tracer.Graft + mesh add */
    s->tflags[ti(h, e)] |= TF_MESH;
    return 0;
}

/* handlePrune for one (receiver, sender edge, topic), gossipsub.go:842-870. */
static void handle_prune(hb* h, uint32_t e)
{
    orc_net* s = h->s;
    if (!((s->sub[h->i] >> h->t) & 1u)) return;
    orc_log_net(ORC_EV_PRUNE, h->i, s->col[e], h->t, h->now);  /* tracer.Prune (gossipsub.go:849) */
    orc_prune(s, e, h->t);
    s->tflags[ti(h, e)] &= (uint8_t)~TF_MESH;
    /* makePrune sends Backoff = PruneBackoff / time.Second (whole seconds),
     * UnsubscribeBackoff for Leave's PRUNE (isUnsubscribe, gossipsub.go:1870-1872);
     * handlePrune obeys it when > 0, else uses its own PruneBackoff. */
    int64_t secs = (h->unsub ? s->gp->unsubscribe_backoff_ns : s->gp->prune_backoff_ns) / kSecond;
    if (secs > 0) do_add_backoff(h, e, secs * kSecond);
    else do_add_backoff(h, e, s->gp->prune_backoff_ns);
}

int64_t orc_handle_control(orc_net* s, int32_t round, int64_t now)
{
    const uint64_t seed = g_px_seed;
    const int64_t TE = (int64_t)s->t * s->e;
    uint8_t* in = s->ctl + (int64_t)(round & 1) * TE;
    uint8_t* out = s->ctl + (int64_t)((round + 1) & 1) * TE;
    int64_t handled = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : handled)
    for (int64_t j = 0; j < s->n; ++j) {
        hb h = {s, (uint32_t)j, s->row_ptr[j], s->row_ptr[j + 1], 0, 0, s->gp->do_px ? seed : 0, now, out, 0};
        uint8_t* nopx = s->gp->do_px ? (uint8_t*)calloc((size_t)(h.en - h.b) + 1, 1) : NULL;
        for (int32_t t = 0; t < s->t; ++t) {
            h.t = t;
            for (uint32_t e = h.b; e < h.en; ++e) {     /* senders in row order */
                uint8_t c = in[(int64_t)t * s->e + e];
                if (!c) continue;
                in[(int64_t)t * s->e + e] = 0;
                ++handled;
                if (c & GSIM_CTL_GRAFT) {
                    const int off = handle_graft(&h, e);
                    if (nopx && off) nopx[e - h.b] = 1;
                }
                if (c & GSIM_CTL_PRUNE) {
                    h.unsub = (c & GSIM_CTL_UNSUB) != 0;
                    handle_prune(&h, e);
                    h.unsub = 0;
                }
            }
        }
        if (nopx) {
            /* the replies of one RPC carry PX only if no GRAFT of it turned doPX off
             * (gossipsub.go:744-834) */
            const uint64_t kt = (uint64_t)now ^ ((uint64_t)now >> 32);
            for (int32_t t = 0; t < s->t; ++t) {
                h.t = t;
                for (uint32_t e = h.b; e < h.en; ++e) {
                    uint8_t* r = &out[(int64_t)t * s->e + s->rev[e]];
                    if (!(*r & GSIM_CTL_PX)) continue;
                    if (nopx[e - h.b]) *r &= (uint8_t)~GSIM_CTL_PX;
                    else px_emit(&h, e, 0, P_PX_GRAFT, kt, 0);
                }
            }
            free(nopx);
        }
    }
    return handled;
}

/* ---- connection churn ---------------------------------------------------- */

static int64_t find_edge(const orc_net* s, uint32_t i, uint32_t j)
{
    uint32_t lo = s->row_ptr[i], hi = s->row_ptr[i + 1];
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (s->col[mid] < j) lo = mid + 1; else hi = mid;
    }
    return (lo < s->row_ptr[i + 1] && s->col[lo] == j) ? (int64_t)lo : -1;
}

/* Connections going down or up between two ticks, both endpoints notified
 * (handleDeadPeers pubsub.go:711-759 / the new-peer case of processLoop
 * pubsub.go:575-595).
 * Down: the router's RemovePeer (gossipsub.go:554-567: out of every mesh,
 * no PRUNE, pending control dropped, backoff kept) and the score tracer's
 * RemovePeer (score.go:611-644: drop a positive score, else retain with P2
 * reset and the P3b penalty).  Up: the router's AddPeer (gossipsub.go:525-552)
 * and peerScore.AddPeer (score.go:595-609).  The live score of a removed peer
 * uses ipColocationFactor over the tracked set as the batch starts (Go
 * computes it live, score.go:344-388; an earlier up batch of the same tick
 * has changed that set), the same for every removal of the batch.  Returns
 * the index of the first pair that is not a connection, or -1. */
int32_t orc_churn(orc_net* s, const uint32_t* pairs, int32_t count, int32_t up, int64_t now)
{
    for (int32_t q = 0; q < count; ++q) {
        const uint32_t a = pairs[2 * q], b = pairs[2 * q + 1];
        if (a >= s->n || b >= s->n || find_edge(s, a, b) < 0) return q;
    }
    if (!up) orc_ip_colocation(s);
    for (int32_t q = 0; q < count; ++q) {
        for (int d = 0; d < 2; ++d) {
            const uint32_t o = pairs[2 * q + d], p = pairs[2 * q + 1 - d];
            const int64_t e = find_edge(s, o, p);
            orc_log_net(up ? ORC_EV_ADD_PEER : ORC_EV_REMOVE_PEER, o, p, -1, now);
            orc_gater_connection(s, e, up, now);
            if (up) {
                orc_add_peer(s, e);
                continue;
            }
            for (int32_t t = 0; t < s->t; ++t) {
                const int64_t i = (int64_t)t * s->e + e;
                s->tflags[i] &= (uint8_t)~(GSIM_TF_MESH | GSIM_TF_FANOUT);   /* out of mesh and fanout */
                if (s->ctl) {
                    s->ctl[i] = 0;
                    s->ctl[(int64_t)s->t * s->e + i] = 0;
                }
            }
            orc_remove_peer(s, e, now);
            s->estate[e] &= (uint8_t)~GSIM_ES_CONNECTED;
        }
    }
    return -1;
}

int64_t orc_px_connect(orc_net* s, int64_t now, uint32_t* pairs, int64_t cap)
{
    if (!s->px) return 0;
    if (s->px_pend) {   /* Leave's PRUNEs: their receivers' PX handling, with this tick's snapshot */
        px_pend* pp = s->px_pend;
        for (int64_t q = 0; q < pp->n;) {
            const uint32_t ep = (uint32_t)pp->ent[q];
            if ((int64_t)ep >= s->e) { ++q; continue; }          /* (a list of another graph: cannot happen) */
            uint32_t listed[256];
            int n = 0;
            while (q < pp->n && (uint32_t)pp->ent[q] == ep && n < 256) listed[n++] = (uint32_t)(pp->ent[q++] >> 32);
            px_accept(s, ep, listed, n);
        }
        pp->n = 0;
    }
    uint32_t* conn = NULL;
    int64_t n = 0, capc = 0;
    for (int64_t u = 0; u < s->n; ++u)
        for (uint32_t e = s->row_ptr[u]; e < s->row_ptr[u + 1]; ++e) {
            const uint32_t v = s->col[e], r = s->rev[e];
            if ((uint32_t)u > v || !(s->px[e] | s->px[r])) continue;      /* each pair once, from its lower end */
            const int a = s->px[e] != 0;
            s->px[e] = s->px[r] = 0;
            if (s->estate[e] & ES_CONN) continue;                        /* connector: already connected */
            if (n == capc) {
                capc = capc ? 2 * capc : 256;
                conn = (uint32_t*)realloc(conn, sizeof(uint32_t) * 2 * (size_t)capc);
            }
            conn[2 * n] = a ? (uint32_t)u : v;                           /* the dialer */
            conn[2 * n + 1] = a ? v : (uint32_t)u;
            ++n;
        }
    for (int64_t q = 0; q < n; ++q) {
        const int64_t ed = find_edge(s, conn[2 * q], conn[2 * q + 1]);
        ((uint8_t*)s->outbound)[ed] = 1;                                  /* gs.outbound (gossipsub.go:532-551) */
        ((uint8_t*)s->outbound)[s->rev[ed]] = 0;
        if (q < cap && pairs) { pairs[2 * q] = conn[2 * q]; pairs[2 * q + 1] = conn[2 * q + 1]; }
    }
    if (n) orc_churn(s, conn, (int32_t)n, 1, now);
    free(conn);
    return n;
}

/* ---- Join / Leave (gossipsub.go:1047-1124) ------------------------------- */

static int f_join(const hb* h, uint32_t e, double arg)        /* gossipsub.go:1084-1090 */
{
    (void)arg;
    return !is_direct(h, e) && !has_backoff(h, e) && orc_score_edge(h->s, e) >= 0;   /* the live Score (1091) */
}

static int f_join_more(const hb* h, uint32_t e, double arg)   /* gossipsub.go:1070-1077 */
{
    return !in_fanout(h, e) && f_join(h, e, arg);
}

void orc_set_subscriptions(orc_net* s, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick, int64_t now,
                           uint64_t seed)
{
    uint64_t* sub = (uint64_t*)s->sub;
    const gsim_gossipsub_params* gp = s->gp;
    for (int32_t q = 0; q < count; ++q) {
        const uint32_t p = pairs[2 * q];
        const int32_t t = (int32_t)pairs[2 * q + 1];
        const uint64_t bit = 1ull << t;
        hb h = {s, p, s->row_ptr[p], s->row_ptr[p + 1], t, tick, seed, now, s->ctl, 0};
        if (join) {
            if (sub[p] & bit) continue;                          /* gs.mesh[topic] exists */
            sub[p] |= bit;                                       /* the announcement */
            orc_log_net(ORC_EV_JOIN, p, p, t, now);
            cand buf[4096];
            const uint32_t deg = h.en - h.b;
            cand* c = deg <= 4096 ? buf : (cand*)malloc(sizeof(cand) * deg);
            if (s->fan_topics && ((s->fan_topics[p] >> t) & 1u)) {
                int have = 0;
                for (uint32_t e = h.b; e < h.en; ++e) {
                    if (!in_fanout(&h, e)) continue;
                    if (orc_score_edge(s, e) < 0 || has_backoff(&h, e))                 /* live Score (1063) */
                        s->tflags[ti(&h, e)] &= (uint8_t)~GSIM_TF_FANOUT;
                    else ++have;
                }
                if (have < gp->d) {
                    const int n = get_peers(&h, gp->d - have, f_join_more, 0, P_JOIN, c);
                    for (int k = 0; k < n; ++k) s->tflags[ti(&h, c[k].e)] |= GSIM_TF_FANOUT;
                }
                for (uint32_t e = h.b; e < h.en; ++e)
                    if (in_fanout(&h, e))
                        s->tflags[ti(&h, e)] = (uint8_t)((s->tflags[ti(&h, e)] & ~GSIM_TF_FANOUT) | TF_MESH);
                s->fan_topics[p] &= ~bit;                        /* delete(gs.fanout, topic), lastpub */
                if (s->lastpub) s->lastpub[(int64_t)p * s->t + t] = 0;
            } else {
                const int n = get_peers(&h, gp->d, f_join, 0, P_JOIN, c);
                for (int k = 0; k < n; ++k) s->tflags[ti(&h, c[k].e)] |= TF_MESH;
            }
            if (c != buf) free(c);
            for (uint32_t e = h.b; e < h.en; ++e) {
                if (!in_mesh(&h, e)) continue;
                orc_log_net(ORC_EV_GRAFT, p, s->col[e], t, now);   /* tracer.Graft + sendGraft */
                orc_graft(s, e, t, now);
                send_ctl(&h, e, GSIM_CTL_GRAFT);
            }
        } else {
            if (!(sub[p] & bit)) continue;                       /* no mesh for the topic */
            sub[p] &= ~bit;
            orc_log_net(ORC_EV_LEAVE, p, p, t, now);
            for (uint32_t e = h.b; e < h.en; ++e) {
                if (!in_mesh(&h, e)) continue;
                orc_log_net(ORC_EV_PRUNE, p, s->col[e], t, now);   /* tracer.Prune, sendPrune, addBackoff */
                orc_prune(s, e, t);
                s->tflags[ti(&h, e)] &= (uint8_t)~TF_MESH;
                send_ctl(&h, e, GSIM_CTL_PRUNE | GSIM_CTL_UNSUB | (gp->do_px ? GSIM_CTL_PX : 0));
                do_add_backoff(&h, e, gp->unsubscribe_backoff_ns);
                /* sendPrune(p, topic, true) -> makePrune(p, topic, gs.doPX, true): the list with
                 * the live scores after the Prunes so far (gossipsub.go:1118, 1132-1133) */
                if (gp->do_px) px_emit(&h, e, 1, P_PX_LEAVE, tick, 1);
            }
        }
    }
}
