/*
 * oracle_gossip.c — network-level restatement of GossipSub gossip: emitGossip
 * (gossipsub.go:1711-1775), handleIHave (630-692), handleIWant (694-739),
 * the message cache's gossip/history windows (mcache.go:55-104) and the
 * gossip tracer's IWANT promises (gossip_tracer.go:48-141) with the broken-
 * promise penalty (applyIwantPenalties, gossipsub.go:1620-1625).
 * TEST INFRASTRUCTURE (see oracle.h).
 *
 * BSP placement: a heartbeat emits IHAVE; control round 0
 * of the tick handles IHAVE and sends IWANT; control round 1 handles IWANT
 * and sends the messages, which arrive with the copies of round 2.  The
 * mcache of a peer is its first receptions (puts) by heartbeat window:
 * window w at heartbeat k holds the puts of tick k-1-w, and from the shift at
 * heartbeat k on window 0 collects tick k's puts.  A receiver that rejects a
 * message does not put it; its origin does (Publish puts before validation
 * matters to anyone else).  Control handlers use the heartbeat's score
 * snapshot (declared divergence, as for handleGraft).
 */
#include "oracle_internal.h"

#include <stdlib.h>
#include <string.h>

#define UNSEEN 0xFFFFFFFFu

static inline int64_t te(const orc_net* s, int32_t t, int64_t e) { return (int64_t)t * s->e + e; }

/* Keys of choices made per (observer, other peer, message): the other peer
 * goes into the Philox key's high word. */
static inline uint64_t okey_pair(uint64_t seed, uint64_t tick, uint32_t obs, int32_t topic, uint32_t purpose,
                                 uint32_t slot, uint32_t other)
{
    uint32_t ctr[4] = {(uint32_t)tick, obs, ((uint32_t)topic << 8) | purpose, slot};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ other};
    uint32_t out[4];
    orc_philox4x32_10(ctr, key, out);
    return ((uint64_t)out[0] << 32) | slot;
}

/* The tick in which peer i put the message of `slot` into its mcache, if it
 * did (mcache.Put at first reception of a valid message, or at Publish). */
static int put_tick(const orc_net* s, const orc_msgs* m, uint32_t slot, uint32_t i, int64_t* tick)
{
    const uint32_t c = m->seen[(int64_t)slot * s->n + i];
    if (c == UNSEEN) return 0;
    if (m->invalid[slot] && i != m->origin[slot]) return 0;
    *tick = (int64_t)c / m->rounds;
    return 1;
}

/* Slots of topic t that anyone can hold in a gossip window at heartbeat
 * `tick`: a first reception (or the publication) in ticks >= tick-HG.
 * Rebuilt once per heartbeat (an index, not a semantic filter). */
static int gossip_ids(const orc_net* s, const orc_msgs* m, uint32_t i, int32_t t, int64_t tick, uint32_t* out);

void orc_gossip_index(const orc_net* s, orc_msgs* m, int64_t tick)
{
    priv* p = orc_msgs_priv(m);
    free(p->cand);
    free(p->cand_ptr);
    p->cand_ptr = (int32_t*)calloc((size_t)s->t + 1, sizeof(int32_t));
    p->cand = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(m->ring + 1));
    const int64_t lo = (tick - s->gp->history_gossip) * m->rounds;
    int32_t n = 0;
    for (int32_t t = 0; t < s->t; ++t) {
        p->cand_ptr[t] = n;
        for (int32_t slot = 0; slot < m->ring; ++slot)
            if (p->slot_last && p->slot_last[slot] >= lo && (int32_t)m->topic[slot] == t) p->cand[n++] = (uint32_t)slot;
    }
    p->cand_ptr[s->t] = n;
    if (p->log_on) {                     /* every router's GetGossipIDs(topic) at this heartbeat */
        orc_log(m, ORC_EV_HEARTBEAT, 0, 0, 0, 0, 0, tick);
        uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(m->ring + 1));
        for (int64_t i = 0; i < s->n; ++i)
            for (int32_t t = 0; t < s->t; ++t) {
                const int k = gossip_ids(s, m, (uint32_t)i, t, tick, ids);
                for (int q = 0; q < k; ++q) orc_log(m, ORC_EV_GOSSIP_ID, (uint32_t)i, 0, ids[q], t, 0, 0);
            }
        free(ids);
    }
}

/* MessageCache.GetGossipIDs(topic) of peer i at heartbeat `tick` (before
 * its Shift): the puts of ticks tick-HistoryGossip .. tick-1, slot order. */
static int gossip_ids(const orc_net* s, const orc_msgs* m, uint32_t i, int32_t t, int64_t tick, uint32_t* out)
{
    const priv* p = (const priv*)m->priv;
    int n = 0;
    const int64_t lo = tick - s->gp->history_gossip;
    if (!p || !p->cand_ptr) return 0;
    for (int32_t q = p->cand_ptr[t]; q < p->cand_ptr[t + 1]; ++q) {
        const uint32_t slot = p->cand[q];
        int64_t pt;
        if (!put_tick(s, m, slot, i, &pt)) continue;
        if (pt >= lo && pt <= tick - 1) out[n++] = slot;
    }
    return n;
}

typedef struct kv { uint64_t key; uint32_t v; } kv;

static int cmp_kv(const void* a, const void* b)
{
    uint64_t x = ((const kv*)a)->key, y = ((const kv*)b)->key;
    return x < y ? -1 : x > y;
}

static int topic_peer(const orc_net* s, uint32_t e, int32_t t)
{
    return (s->estate[e] & GSIM_ES_CONNECTED) && ((s->sub[s->col[e]] >> t) & 1u);
}

/* emitGossip(topic, exclude) for observer i: exclude = its mesh after the mesh
 * maintenance of a joined topic (gossipsub.go:1554-1556), its fanout peers for
 * a fanout topic (1593-1595); gossipsub.go:1711-1775. */
void orc_gossip_emit(orc_net* s, orc_msgs* m, uint32_t i, int32_t t, uint64_t tick, uint64_t seed,
                     uint8_t exclude)
{
    priv* p = orc_msgs_priv(m);
    uint32_t* mids = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(m->ring > 0 ? m->ring : 1));
    const int nm = gossip_ids(s, m, i, t, (int64_t)tick, mids);
    free(mids);
    if (nm == 0) return;
    const gsim_gossipsub_params* gp = s->gp;
    const uint32_t b = s->row_ptr[i], en = s->row_ptr[i + 1];
    const uint32_t deg = en - b;
    kv* L = (kv*)malloc(sizeof(kv) * (size_t)(2 * deg + 1));
    int n = 0;
    for (uint32_t e = b; e < en; ++e) {
        if (!topic_peer(s, e, t)) continue;
        if (s->tflags[te(s, t, e)] & exclude) continue;                    /* exclude: mesh / fanout */
        if (s->direct && s->direct[e]) continue;                           /* no gossip to direct peers */
        if (orc_score_edge(s, e) < s->th->gossip_threshold) continue;        /* live Score(p) */
        L[n].key = okey(seed, tick, i, t, P_GOSSIP, s->col[e], e - b);
        L[n].v = e;
        ++n;
    }
    if (n < gp->dlo) {
        /* fill from the topic peers in map order until Dlo (gossipsub.go:1739-1748);
         * peers already selected can be appended again */
        kv* fill = (kv*)malloc(sizeof(kv) * (size_t)(deg + 1));
        int nf = 0;
        for (uint32_t e = b; e < en; ++e) {
            if (!topic_peer(s, e, t)) continue;
            fill[nf].key = okey(seed, tick, i, t, P_GOSSIP_FILL, s->col[e], e - b);
            fill[nf].v = e;
            ++nf;
        }
        qsort(fill, (size_t)nf, sizeof(kv), cmp_kv);
        for (int q = 0; q < nf; ++q) {
            const uint32_t e = fill[q].v;
            L[n].key = okey(seed, tick, i, t, P_GOSSIP_DUP, s->col[e], e - b);
            L[n].v = e;
            ++n;
            if (n >= gp->dlo) break;
        }
        free(fill);
    }
    int target = gp->dlazy;
    const int factor = (int)(gp->gossip_factor * (double)n);
    if (factor > target) target = factor;
    if (target > n) target = n;
    else qsort(L, (size_t)n, sizeof(kv), cmp_kv);                           /* shufflePeers */
    for (int q = 0; q < target; ++q) p->ihave[te(s, t, s->rev[L[q].v])] = 1;  /* enqueueGossip */
    free(L);
}

/* ---- promises (gossip_tracer.go) ---------------------------------------- */

static int cmp_u32(const void* a, const void* b)
{
    uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
    return x < y ? -1 : x > y;
}

static void promise_add(priv* p, uint32_t peer, uint32_t e, uint32_t slot, uint64_t mid, int64_t expire)
{
    for (int32_t q = 0; q < p->npr[peer]; ++q)
        if (p->pr[peer][q].mid == mid && p->pr[peer][q].e == e) return;      /* promises[mid][p] exists */
    if (p->npr[peer] == p->cappr[peer]) {
        p->cappr[peer] = p->cappr[peer] ? 2 * p->cappr[peer] : 8;
        p->pr[peer] = (promise*)realloc(p->pr[peer], sizeof(promise) * (size_t)p->cappr[peer]);
    }
    promise* x = &p->pr[peer][p->npr[peer]++];
    x->e = e; x->slot = slot; x->mid = mid; x->expire = expire;
}

/* fulfillPromise at the receiver's first reception (DeliverMessage /
 * RejectMessage / ValidateMessage, gossip_tracer.go:119-170). */
void orc_gossip_fulfill(orc_msgs* m, uint32_t peer, uint32_t slot)
{
    priv* p = orc_msgs_priv(m);
    orc_log(m, ORC_EV_FULFILL, peer, 0, slot, 0, 0, 0);
    if (!p->npr) return;
    const uint64_t mid = m->mid ? m->mid[slot] : slot;
    int32_t w = 0;
    for (int32_t q = 0; q < p->npr[peer]; ++q)
        if (p->pr[peer][q].mid != mid) p->pr[peer][w++] = p->pr[peer][q];
    p->npr[peer] = w;
}

/* applyIwantPenalties at heartbeat time `now` (gossipsub.go:1620-1625 with
 * GetBrokenPromises gossip_tracer.go:79-115): every promise that expired
 * before now is broken; AddPenalty(peer, count) per peer. */
void orc_gossip_penalties(orc_net* s, orc_msgs* m, int64_t now)
{
    priv* p = orc_msgs_priv(m);
    orc_log(m, ORC_EV_PENALTIES, 0, 0, 0, 0, 0, now);
    if (!p->npr) return;
    uint32_t* broken = NULL;
    int32_t capb = 0;
    for (int64_t peer = 0; peer < s->n; ++peer) {
        promise* v = p->pr[peer];
        int32_t w = 0, nb = 0;
        for (int32_t q = 0; q < p->npr[peer]; ++q) {
            if (v[q].expire < now) {                 /* expire.Before(now): broken */
                if (nb == capb) {
                    capb = capb ? 2 * capb : 16;
                    broken = (uint32_t*)realloc(broken, sizeof(uint32_t) * (size_t)capb);
                }
                broken[nb++] = v[q].e;
            } else {
                v[w++] = v[q];
            }
        }
        p->npr[peer] = w;
        if (nb) qsort(broken, (size_t)nb, sizeof(uint32_t), cmp_u32);
        for (int32_t q = 0; q < nb;) {               /* AddPenalty(p, count) once per peer */
            int32_t r = q;
            while (r < nb && broken[r] == broken[q]) ++r;
            orc_add_penalty(s, broken[q], r - q);
            orc_log(m, ORC_EV_BROKEN, (uint32_t)peer, s->col[broken[q]], 0, 0, 0, r - q);
            q = r;
        }
    }
    free(broken);
}

/* ---- mcache.peertx ------------------------------------------------------ */

static uint64_t tx_hash(uint64_t mid, uint32_t e)
{
    uint64_t x = mid * 0x9E3779B97F4A7C15ull ^ ((uint64_t)e * 0xC2B2AE3D27D4EB4Full);
    x ^= x >> 29;
    return x;
}

static int32_t* tx_slot(priv* p, uint64_t mid, uint32_t e)
{
    if (2 * (p->ntx + 1) > p->captx) {
        const int64_t nc = p->captx ? 2 * p->captx : 1024;
        peertx_ent* nt = (peertx_ent*)calloc((size_t)nc, sizeof(peertx_ent));
        for (int64_t q = 0; q < p->captx; ++q) {
            if (!p->tx[q].count) continue;
            uint64_t h = tx_hash(p->tx[q].mid, p->tx[q].e) & (uint64_t)(nc - 1);
            while (nt[h].count) h = (h + 1) & (uint64_t)(nc - 1);
            nt[h] = p->tx[q];
        }
        free(p->tx);
        p->tx = nt;
        p->captx = nc;
    }
    uint64_t h = tx_hash(mid, e) & (uint64_t)(p->captx - 1);
    while (p->tx[h].count && !(p->tx[h].mid == mid && p->tx[h].e == e)) h = (h + 1) & (uint64_t)(p->captx - 1);
    if (!p->tx[h].count) { p->tx[h].mid = mid; p->tx[h].e = e; ++p->ntx; }
    return &p->tx[h].count;
}

/* ---- control round 0: handleIHave --------------------------------------- */

/* Test access: the last heartbeat's IHAVE marks, [T][E] at the receivers'
 * edges (n = T * E bytes; zeros when gossip is off). */
int64_t orc_msgs_ihave_marks(orc_msgs* m, uint8_t* out, int64_t n)
{
    priv* p = orc_msgs_priv(m);
    if (!p->ihave) {
        memset(out, 0, (size_t)n);
        return 0;
    }
    memcpy(out, p->ihave, (size_t)n);
    return n;
}

void orc_gossip_ihave(orc_net* s, orc_msgs* m, int64_t g)
{
    priv* p = orc_msgs_priv(m);
    if (!p->ihave) return;
    const gsim_gossipsub_params* gp = s->gp;
    const int64_t tick = p->ihave_tick, now = orc_round_time(m, g);
    uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(m->ring + 1));
    kv* want = (kv*)malloc(sizeof(kv) * (size_t)(m->ring + 1));
    uint8_t* mark = (uint8_t*)calloc((size_t)m->ring + 1, 1);
    for (int64_t pr = 0; pr < s->n; ++pr) {
        for (uint32_t e = s->row_ptr[pr]; e < s->row_ptr[pr + 1]; ++e) {
            int any = 0;
            for (int32_t t = 0; t < s->t; ++t) any |= p->ihave[te(s, t, e)];
            if (!any) continue;
            const uint32_t i = s->col[e];
            if (s->score[e] < s->th->gossip_threshold) continue;     /* IHAVE from a low-score peer */
            if (1 > gp->max_ihave_messages) continue;                 /* peerhave flood protection */
            if (0 >= gp->max_ihave_length) continue;                  /* iasked */
            int nw = 0;
            for (int32_t t = 0; t < s->t; ++t) {
                if (!p->ihave[te(s, t, e)]) continue;
                if (!((s->sub[pr] >> t) & 1u)) continue;              /* not joined */
                int nm = gossip_ids(s, m, i, t, tick, ids);
                if (nm > gp->max_ihave_length) {
                    /* the sender truncated this peer's IHAVE to a random subset
                     * (gossipsub.go:1766-1771) */
                    kv* tmp = (kv*)malloc(sizeof(kv) * (size_t)nm);
                    for (int q = 0; q < nm; ++q) {
                        tmp[q].key = okey_pair(p->seed, (uint64_t)tick, i, t, P_IHAVE_TRUNC, ids[q], (uint32_t)pr);
                        tmp[q].v = ids[q];
                    }
                    qsort(tmp, (size_t)nm, sizeof(kv), cmp_kv);
                    nm = gp->max_ihave_length;
                    for (int q = 0; q < nm; ++q) ids[q] = tmp[q].v;
                    free(tmp);
                    qsort(ids, (size_t)nm, sizeof(uint32_t), cmp_u32);
                }
                for (int q = 0; q < nm; ++q) {
                    const uint32_t slot = ids[q];
                    if (m->seen[(int64_t)slot * s->n + pr] != UNSEEN) continue;   /* seenMessage */
                    if (mark[slot]) continue;
                    mark[slot] = 1;
                    want[nw].key = okey_pair(p->seed, (uint64_t)tick, (uint32_t)pr, 0, P_IWANT, slot, i);
                    want[nw].v = slot;
                    ++nw;
                }
            }
            for (int q = 0; q < nw; ++q) mark[want[q].v] = 0;
            if (nw == 0) continue;
            int iask = nw;
            if (iask > gp->max_ihave_length) iask = gp->max_ihave_length;
            qsort(want, (size_t)nw, sizeof(kv), cmp_kv);              /* shuffleStrings(iwantlst) */
            /* AddPromise: one random id of the list */
            int pick = 0;
            uint64_t best = ~0ull;
            for (int q = 0; q < iask; ++q) {
                const uint64_t k = okey_pair(p->seed, (uint64_t)tick, (uint32_t)pr, 0, P_PROMISE, want[q].v, i);
                if (k < best) { best = k; pick = q; }
            }
            const uint32_t ps = want[pick].v;
            orc_log(m, ORC_EV_PROMISE, (uint32_t)pr, i, ps, 0, g, now);
            promise_add(p, (uint32_t)pr, e, ps, m->mid ? m->mid[ps] : ps, now + gp->iwant_followup_time_ns);
            for (int q = 0; q < iask; ++q) {                         /* IWANT to i */
                orc_log(m, ORC_EV_RPC_IWANT, (uint32_t)pr, i, want[q].v, (int32_t)m->topic[want[q].v], g, 0);
                if (p->niw == p->capiw) {
                    p->capiw = p->capiw ? 2 * p->capiw : 1024;
                    p->iw = (iwant_ent*)realloc(p->iw, sizeof(iwant_ent) * (size_t)p->capiw);
                }
                p->iw[p->niw].er = e;
                p->iw[p->niw].slot = want[q].v;
                p->niw++;
            }
        }
    }
    free(ids);
    free(want);
    free(mark);
    memset(p->ihave, 0, (size_t)s->t * (size_t)s->e);
}

/* ---- control round 1: handleIWant --------------------------------------- */

void orc_gossip_iwant(orc_net* s, orc_msgs* m, int64_t g)
{
    priv* p = orc_msgs_priv(m);
    const gsim_gossipsub_params* gp = s->gp;
    const int64_t tick = g / m->rounds;
    for (int64_t q = 0; q < p->niw; ++q) {
        const uint32_t er = p->iw[q].er, slot = p->iw[q].slot;   /* er: requester p's edge to i */
        const uint32_t i = s->col[er], ei = s->rev[er];          /* ei: i's edge to p */
        if (s->score[ei] < s->th->gossip_threshold) continue;     /* IWANT from a low-score peer */
        if (m->behaviour && (m->behaviour[i] & ORC_BEHAVE_IGNORE_IWANT)) continue;
        int64_t pt;
        /* mcache.GetForPeer: in the history window after the shift at this tick */
        if (!put_tick(s, m, slot, i, &pt) || pt < tick - gp->history_length + 1 || pt > tick) continue;
        int32_t* cnt = tx_slot(p, m->mid ? m->mid[slot] : slot, ei);
        *cnt += 1;
        orc_log(m, ORC_EV_SERVE, i, s->col[ei], slot, 0, g, *cnt);
        if (*cnt > gp->gossip_retransmission) continue;
        if (p->ngr == p->capgr) {
            p->capgr = p->capgr ? 2 * p->capgr : 1024;
            p->gr = (arr_ent*)realloc(p->gr, sizeof(arr_ent) * (size_t)p->capgr);
        }
        p->gr[p->ngr].recv = s->col[ei];
        p->gr[p->ngr].slot = slot;
        p->gr[p->ngr].er = er;
        p->gr[p->ngr].resp = 1;
        p->ngr++;
    }
    p->niw = 0;
}
