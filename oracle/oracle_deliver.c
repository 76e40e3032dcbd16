/*
 * oracle_deliver.c — network-level restatement of message propagation.
 * TEST INFRASTRUCTURE (see oracle.h).
 *
 * Round g:
 *  1. every peer that saw a message for the first time in round g-1 (or
 *     published it in round g-1) forwards it to its current mesh except the
 *     sender and the origin (Publish, gossipsub.go:975-1045); a message whose
 *     ring slot was reused since is no longer forwarded;
 *  2. every receiver handles those copies in (receiver, message,
 *     receiving-edge) order — the lowest receiving edge of a round is the
 *     first delivery — exactly as pushMsg would for those RPCs
 *     (pubsub.go:1118-1162);
 *  3. the control inbox of the round is handled.
 */
#include "oracle_internal.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define UNSEEN 0xFFFFFFFFu

priv* orc_msgs_priv(orc_msgs* m)
{
    if (!m->priv) m->priv = calloc(1, sizeof(priv));
    return (priv*)m->priv;
}

static priv* P(orc_msgs* m) { return orc_msgs_priv(m); }

/* Router-level events (GRAFT/PRUNE/ADD/REMOVE) have no message log at hand
 * in oracle_net.c: they go to one buffer the oracle owns, on while any
 * message log is, and are handed out with the next orc_msgs_events. */
static int g_net_on;
static orc_event* g_net_ev;
static int64_t g_net_n, g_net_cap;

void orc_msgs_log(orc_msgs* m, int32_t on)
{
    P(m)->log_on = on;
    g_net_on = on;
    g_net_n = 0;
}

void orc_log_net(int32_t kind, uint32_t a, uint32_t b, int32_t topic, int64_t now)
{
    orc_log_net_x(kind, a, b, topic, 0, 0, now);
}

void orc_log_net_x(int32_t kind, uint32_t a, uint32_t b, int32_t topic, uint64_t mid, int64_t g, int64_t x)
{
    if (!g_net_on) return;
#pragma omp critical(orc_log)
    {
        if (g_net_n == g_net_cap) {
            g_net_cap = g_net_cap ? 2 * g_net_cap : 4096;
            g_net_ev = (orc_event*)realloc(g_net_ev, sizeof(orc_event) * (size_t)g_net_cap);
        }
        orc_event* v = &g_net_ev[g_net_n++];
        v->kind = kind; v->topic = topic; v->a = a; v->b = b; v->g = g; v->mid = mid; v->x = x;
    }
}

void orc_log(orc_msgs* m, int32_t kind, uint32_t a, uint32_t b, uint32_t slot, int32_t topic, int64_t g, int64_t x)
{
    priv* p = P(m);
    if (!p->log_on) return;
    if (p->nev == p->capev) {
        p->capev = p->capev ? 2 * p->capev : 4096;
        p->ev = (orc_event*)realloc(p->ev, sizeof(orc_event) * (size_t)p->capev);
    }
    orc_event* v = &p->ev[p->nev++];
    v->kind = kind; v->topic = topic; v->a = a; v->b = b; v->g = g;
    v->mid = m->mid ? m->mid[slot] : slot;
    v->x = x;
}

int64_t orc_msgs_events(orc_msgs* m, orc_event* out, int64_t cap)
{
    priv* p = P(m);
    const int64_t n = p->nev, nn = p->log_on ? g_net_n : 0;
    if (out) {
        memcpy(out, p->ev, sizeof(orc_event) * (size_t)(n < cap ? n : cap));
        if (cap > n) memcpy(out + n, g_net_ev, sizeof(orc_event) * (size_t)(nn < cap - n ? nn : cap - n));
        p->nev = 0;
        if (p->log_on) g_net_n = 0;
    }
    return n + nn;
}

void orc_msgs_free_priv(orc_msgs* m)
{
    if (m->priv && ((priv*)m->priv)->log_on) g_net_on = 0;
    if (!m->priv) return;
    priv* p = (priv*)m->priv;
    free(p->ev);
    free(p->fr);
    free(p->fp);
    free(p->ar);
    free(p->gr);
    free(p->ihave);
    free(p->iw);
    if (p->pr) for (int64_t q = 0; q < p->n_alloc; ++q) free(p->pr[q]);
    free(p->pr);
    free(p->npr);
    free(p->cappr);
    free(p->tx);
    free(p->slot_last);
    free(p->vd);
    free(p->tcount);
    free(p->pq);
    free(p->cand);
    free(p->cand_ptr);
    free(p);
    m->priv = NULL;
}

static void fr_push(priv* p, uint32_t peer, uint32_t slot, uint32_t from)
{
    if (p->nfr == p->capfr) {
        p->capfr = p->capfr ? 2 * p->capfr : 1024;
        p->fr = (fr_ent*)realloc(p->fr, sizeof(fr_ent) * (size_t)p->capfr);
    }
    p->fr[p->nfr].peer = peer; p->fr[p->nfr].slot = slot; p->fr[p->nfr].from = from;
    p->nfr++;
}

static void ar_push(priv* p, uint32_t recv, uint32_t slot, uint32_t er, uint32_t resp)
{
    if (p->nar == p->capar) {
        p->capar = p->capar ? 2 * p->capar : 4096;
        p->ar = (arr_ent*)realloc(p->ar, sizeof(arr_ent) * (size_t)p->capar);
    }
    p->ar[p->nar].recv = recv; p->ar[p->nar].slot = slot; p->ar[p->nar].er = er; p->ar[p->nar].resp = resp;
    p->nar++;
}

static void pq_push(priv* p, int64_t c, uint32_t recv, uint32_t slot, uint32_t er, int32_t first)
{
    if (p->npq == p->cappq) {
        p->cappq = p->cappq ? 2 * p->cappq : 1024;
        p->pq = (pend_ent*)realloc(p->pq, sizeof(pend_ent) * (size_t)p->cappq);
    }
    pend_ent* x = &p->pq[p->npq++];
    x->c = c; x->recv = recv; x->slot = slot; x->er = er; x->first = first;
}

static int cmp_arr(const void* a, const void* b)
{
    const arr_ent* x = (const arr_ent*)a;
    const arr_ent* y = (const arr_ent*)b;
    if (x->recv != y->recv) return x->recv < y->recv ? -1 : 1;
    if (x->slot != y->slot) return x->slot < y->slot ? -1 : 1;
    return x->er < y->er ? -1 : x->er > y->er;
}

int64_t orc_layout_size(int32_t which)
{
    return which == 0 ? (int64_t)sizeof(orc_net) : which == 1 ? (int64_t)sizeof(orc_msgs) : -1;
}

int64_t orc_round_time(const orc_msgs* m, int64_t g)
{
    const int64_t r = g % m->rounds, k = g / m->rounds;
    return m->t0 + k * m->hb + (r + 1) * m->hb / (m->rounds + 1);
}

void orc_publish(orc_net* s, orc_msgs* m, uint64_t id, uint32_t topic, uint32_t origin, uint8_t invalid,
                 int64_t g)
{
    orc_publish_v(s, m, id, topic, origin, invalid, 0, g);
}

void orc_publish_v(orc_net* s, orc_msgs* m, uint64_t id, uint32_t topic, uint32_t origin, uint8_t invalid,
                   uint8_t vdelay, int64_t g)
{
    uint32_t slot = (uint32_t)(id % (uint64_t)m->ring);
    if (m->topic_slots > 0) {
        priv* pv = P(m);
        if (!pv->tcount) pv->tcount = (int64_t*)calloc(64, sizeof(int64_t));
        slot = (uint32_t)((int64_t)topic * m->topic_slots + pv->tcount[topic]++ % m->topic_slots);
    }
    {
        priv* pv = P(m);
        if (!pv->vd) pv->vd = (uint8_t*)calloc((size_t)m->ring, 1);
        pv->vd[slot] = vdelay;
    }
    m->topic[slot] = topic;
    m->origin[slot] = origin;
    m->invalid[slot] = invalid;
    if (m->mid) m->mid[slot] = id;
    {
        priv* pv = P(m);
        if (!pv->slot_last) {
            pv->slot_last = (int64_t*)malloc(sizeof(int64_t) * (size_t)m->ring);
            for (int32_t q = 0; q < m->ring; ++q) pv->slot_last[q] = -1;
        }
        pv->slot_last[slot] = g;
    }
    uint32_t* row = m->seen + (int64_t)slot * s->n;
    for (int64_t i = 0; i < s->n; ++i) row[i] = UNSEEN;
    /* the origin validated and saw its own message (markSeen) and puts it in
     * its mcache (gossipsub.go:976); its own DeliverMessage is not scored
     * (trace.go skips ReceivedFrom == self) */
    row[origin] = (uint32_t)g;
    orc_log(m, ORC_EV_SEEN, origin, 0xFFFFFFFFu, slot, (int32_t)topic, g, 1);
    orc_log(m, ORC_EV_PUT, origin, 0, slot, (int32_t)topic, g, 0);
    orc_log(m, ORC_EV_PUBLISH, origin, origin, slot, (int32_t)topic, g, 0);
    /* Publish: an origin that has not joined the topic sends to its fanout
     * (gossipsub.go:1011-1028); flood publishing sends to every topic peer */
    if (!s->gp->flood_publish && !((s->sub[origin] >> topic) & 1u) && s->lastpub && s->fan_topics)
        orc_fanout_publish(s, origin, (int32_t)topic, g, orc_round_time(m, g), P(m)->seed);
    m->lastput[(int64_t)topic * s->n + origin] = (int32_t)(g / m->rounds);
    fr_push(P(m), origin, slot, origin);
}

/* Validations completing at the start of round g (orc_publish_v): the first
 * copy's DeliverMessage (markFirstMessageDelivery, then every pending peer's
 * markDuplicateMessageDelivery with validated zero, score.go:702-726) or
 * RejectMessage (score.go:728-793: markInvalidMessageDelivery for the first
 * and every pending peer; ignored / throttled: nothing), mcache.Put and
 * forwarding in round g + 1 (validation.go:334-341, pubsub.go:1159-1161). */
static void complete_validations(orc_net* s, orc_msgs* m, int64_t g, int64_t now)
{
    priv* p = P(m);
    int64_t keep = 0;
    for (int64_t q = 0; q < p->npq; ++q) {
        const pend_ent x = p->pq[q];
        if (x.c != g) { p->pq[keep++] = x; continue; }
        const int32_t t = (int32_t)m->topic[x.slot];
        const uint8_t verdict = m->invalid[x.slot];
        if (verdict == GSIM_VERDICT_REJECT) orc_mark_invalid(s, x.er, t);
        else if (verdict == GSIM_VERDICT_ACCEPT) {
            if (x.first) orc_mark_first(s, x.er, t);
            else orc_mark_duplicate(s, x.er, t, 0, 0, now);
        }
        if (!x.first) continue;
        if (p->slot_last && p->slot_last[x.slot] < g) p->slot_last[x.slot] = g;
        orc_log(m, ORC_EV_SEEN, x.recv, s->col[x.er], x.slot, t, g, 1);
        if (verdict == GSIM_VERDICT_ACCEPT) {
            m->lastput[(int64_t)t * s->n + x.recv] = (int32_t)(g / m->rounds);
            orc_log(m, ORC_EV_PUT, x.recv, 0, x.slot, t, g, 0);
            fr_push(p, x.recv, x.slot, s->col[x.er]);
        }
    }
    p->npq = keep;
}

typedef struct frbuf { fr_ent* v; int64_t n, cap; } frbuf;

static void frb_push(frbuf* b, uint32_t peer, uint32_t slot, uint32_t from)
{
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 1024;
        b->v = (fr_ent*)realloc(b->v, sizeof(fr_ent) * (size_t)b->cap);
    }
    b->v[b->n].peer = peer; b->v[b->n].slot = slot; b->v[b->n].from = from;
    b->n++;
}

/* One copy at receiver i (step 2 of orc_round): AcceptFrom (graylist, the
 * peer gater), the subscription, pushMsg's seen check and the score
 * tracer's Deliver / Duplicate / RejectMessage. */
static void handle_copy(orc_net* s, orc_msgs* m, priv* p, int64_t g, int64_t now, double gray, arr_ent x, frbuf* fb,
                        int64_t* stats)
{
    const uint32_t i = x.recv, slot = x.slot, er = x.er;
    const int32_t t = (int32_t)m->topic[slot];
    if (s->score[er] < gray && !(s->direct && s->direct[er])) {   /* AcceptFrom -> AcceptNone; direct: AcceptAll */
        stats[3]++;
        return;
    }
    if (s->gater && !(s->direct && s->direct[er]) &&
        !orc_gater_accept(s, p->seed, g, i, er, x.resp ? ORC_GATER_RPC_SLOT : slot)) {
        /* the peer gater's AcceptControl: the message is dropped and the
         * receiver forgets its promises from the sender (ThrottlePeer,
         * gossip_tracer.go:182-200) */
        if (p->npr) {
            int32_t w = 0;
            for (int32_t q2 = 0; q2 < p->npr[i]; ++q2)
                if (p->pr[i][q2].e != er) p->pr[i][w++] = p->pr[i][q2];
            p->npr[i] = w;
        }
        orc_log(m, ORC_EV_THROTTLE, i, s->col[er], slot, t, g, now);
        return;
    }
    /* a topic the receiver no longer subscribes to: the message is skipped
     * (pubsub.go:1094-1098; only after a Leave, orc_set_subscriptions) */
    if (!((s->sub[i] >> t) & 1u)) return;
    stats[0]++;
    uint32_t* cell = &m->seen[(int64_t)slot * s->n + i];
    const uint8_t verdict = m->invalid[slot];
    if (verdict == GSIM_VERDICT_SIGNATURE) {
        orc_gater_event(s, i, er, t, ORC_GATE_REJECT);      /* RejectInvalidSignature */
        /* RejectInvalidSignature before markSeen (validation.go:282-290):
         * every copy's sender is penalised, nothing is seen, no promise is
         * fulfilled (gossip_tracer.go:148-162) */
        stats[2]++;
        orc_mark_invalid(s, er, t);
        orc_log(m, ORC_EV_REJECT_SIG, i, s->col[er], slot, t, g, 0);
        return;
    }
    const uint8_t vdelay = p->vd ? p->vd[slot] : 0;
    if (!vdelay || *cell != UNSEEN) orc_log(m, ORC_EV_SEEN, i, s->col[er], slot, t, g, *cell == UNSEEN);
    if (s->gater) {
        /* first delivery: ValidateMessage, then the verdict's tracer call */
        static const int32_t kind[4] = {ORC_GATE_DELIVER, ORC_GATE_REJECT, ORC_GATE_IGNORE, ORC_GATE_THROTTLE};
        if (*cell == UNSEEN) orc_gater_event(s, i, er, t, ORC_GATE_VALIDATE);
        orc_gater_event(s, i, er, t, *cell == UNSEEN ? kind[verdict] : ORC_GATE_DUPLICATE);
    }
    if (*cell == UNSEEN && vdelay) {
        /* markSeen + ValidateMessage (promises fulfilled); the verdict
         * lands vdelay rounds later (complete_validations) */
        *cell = (uint32_t)(g + vdelay);
        stats[1]++;
        orc_gossip_fulfill(m, i, slot);
        if (p->slot_last) p->slot_last[slot] = g;
        pq_push(p, g + vdelay, i, slot, er, 1);
    } else if (*cell != UNSEEN && (int64_t)*cell > g) {
        /* DuplicateMessage while the first copy validates
         * (deliveryUnknown: drec.peers, score.go:806-809) */
        stats[2]++;
        if (verdict == GSIM_VERDICT_REJECT || verdict == GSIM_VERDICT_ACCEPT) pq_push(p, *cell, i, slot, er, 0);
    } else if (*cell == UNSEEN) {
        *cell = (uint32_t)g;               /* markSeen */
        stats[1]++;
        orc_gossip_fulfill(m, i, slot);    /* gossipTracer: promises for it are kept */
        if (p->slot_last) {
#pragma omp atomic write
            p->slot_last[slot] = g;
        }
        if (verdict == GSIM_VERDICT_REJECT) {
            /* ValidateMessage + RejectMessage(ValidationFailed), score.go:728-793 */
            orc_mark_invalid(s, er, t);
        } else if (verdict == GSIM_VERDICT_ACCEPT) {
            /* DeliverMessage, score.go:702-726; mcache.Put; forward next round */
            orc_mark_first(s, er, t);
            m->lastput[(int64_t)t * s->n + i] = (int32_t)(g / m->rounds);
            orc_log(m, ORC_EV_PUT, i, 0, slot, t, g, 0);
            frb_push(fb, i, slot, s->col[er]);
        }
        /* RejectValidationIgnored / Throttled: deliveryIgnored / deliveryThrottled,
         * no penalty and no credit (score.go:759-781) */
    } else {
        stats[2]++;                        /* DuplicateMessage, score.go:795-827 */
        if (verdict == GSIM_VERDICT_REJECT) orc_mark_invalid(s, er, t);
        else if (verdict == GSIM_VERDICT_ACCEPT)
            orc_mark_duplicate(s, er, t, 1, orc_round_time(m, (int64_t)*cell), now);
    }
}

void orc_round(orc_net* s, orc_msgs* m, int64_t g)
{
    priv* p = P(m);
    const int64_t now = orc_round_time(m, g);
    const double gray = s->th->graylist_threshold;

    if (p->npq) complete_validations(s, m, g, now);
    orc_gater_round_begin(s, now);

    /* 1. last round's first receivers (and publishers) forward to their mesh */
    for (int64_t q = 0; q < p->nfp; ++q) {
        const uint32_t j = p->fp[q].peer, slot = p->fp[q].slot, from = p->fp[q].from;
        if (m->seen[(int64_t)slot * s->n + j] != (uint32_t)(g - 1)) continue;   /* slot reused */
        const int32_t t = (int32_t)m->topic[slot];
        const uint32_t origin = m->origin[slot];
        /* the origin's own Publish: flood to every topic peer with score >=
         * publishThreshold (gossipsub.go:989-995), or its mesh, or its fanout
         * when it has not joined the topic (1011-1028); everyone else
         * forwards to its mesh */
        const int flood = j == origin && s->gp->flood_publish;
        const uint8_t want = (j == origin && !((s->sub[j] >> t) & 1u)) ? GSIM_TF_FANOUT : GSIM_TF_MESH;
        for (uint32_t e = s->row_ptr[j]; e < s->row_ptr[j + 1]; ++e) {
            const uint32_t i = s->col[e];
            /* direct peers in the topic always get it (gossipsub.go:991-1003) */
            const int direct = s->direct && s->direct[e] && ((s->sub[i] >> t) & 1u);
            if (flood) {
                if (!direct && (!((s->sub[i] >> t) & 1u) || s->score[e] < s->th->publish_threshold)) continue;
            } else if (!direct && !(s->tflags[(int64_t)t * s->e + e] & want)) {
                continue;
            }
            if (!(s->estate[e] & GSIM_ES_CONNECTED)) continue;
            if (i == from || i == origin) continue;
            orc_log(m, ORC_EV_RPC_MSG, j, i, slot, t, g, 0);     /* the copy's RPC (sendRPC, gossipsub.go:1195-1200) */
            ar_push(p, i, slot, s->rev[e], 0);
        }
    }
    p->nfp = 0;
    /* IWANT responses sent in the previous round arrive with them */
    for (int64_t q = 0; q < p->ngr; ++q) {
        orc_log(m, ORC_EV_RPC_MSG, s->col[p->gr[q].er], p->gr[q].recv, p->gr[q].slot, (int32_t)m->topic[p->gr[q].slot],
                g, 1);
        ar_push(p, p->gr[q].recv, p->gr[q].slot, p->gr[q].er, 1);
    }
    p->ngr = 0;

    /* 2. receivers handle the copies, in canonical order: by receiver
     * (counting sort, stable), then by (slot, receiver edge) within one */
    arr_ent* ar = p->ar;
    const int64_t nar = p->nar;
    p->ar = NULL; p->nar = 0; p->capar = 0;
    arr_ent* sorted = (arr_ent*)malloc(sizeof(arr_ent) * (size_t)(nar > 0 ? nar : 1));
    int64_t* start = (int64_t*)calloc((size_t)s->n + 1, sizeof(int64_t));
    for (int64_t q = 0; q < nar; ++q) start[ar[q].recv + 1]++;
    for (int64_t i = 0; i < s->n; ++i) start[i + 1] += start[i];
    {
        int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(s->n > 0 ? s->n : 1));
        memcpy(fill, start, sizeof(int64_t) * (size_t)s->n);
        for (int64_t q = 0; q < nar; ++q) sorted[fill[ar[q].recv]++] = ar[q];
        free(fill);
    }
    free(ar);
    /* receivers are independent (each copy touches its receiver's records,
     * cell, mcache and promises), so they run in parallel unless the event
     * log or validation latency needs one global order */
    int serial = p->log_on != 0;
    if (p->vd)
        for (int32_t q = 0; q < m->ring && !serial; ++q) serial = p->vd[q] != 0;
    int nth = 1;
#ifdef _OPENMP
    nth = serial ? 1 : omp_get_max_threads();
#endif
    frbuf* fb = (frbuf*)calloc((size_t)nth, sizeof(frbuf));
    int64_t stats[4] = {0, 0, 0, 0};
#pragma omp parallel num_threads(nth) reduction(+ : stats[:4])
    {
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
#pragma omp for schedule(dynamic, 256)
        for (int64_t i = 0; i < s->n; ++i) {
            arr_ent* seg = sorted + start[i];
            const int64_t len = start[i + 1] - start[i];
            for (int64_t a = 1; a < len; ++a) {          /* by (slot, er): a handful of copies */
                arr_ent x = seg[a];
                int64_t b = a - 1;
                while (b >= 0 && cmp_arr(&seg[b], &x) > 0) { seg[b + 1] = seg[b]; --b; }
                seg[b + 1] = x;
            }
            for (int64_t q = 0; q < len; ++q) handle_copy(s, m, p, g, now, gray, seg[q], &fb[tid], stats);
        }
    }
    for (int k = 0; k < 4; ++k) m->stats[k] += stats[k];
    for (int t = 0; t < nth; ++t) {
        for (int64_t q = 0; q < fb[t].n; ++q) fr_push(p, fb[t].v[q].peer, fb[t].v[q].slot, fb[t].v[q].from);
        free(fb[t].v);
    }
    free(fb);
    free(start);
    free(sorted);
    orc_gater_round_end(s, now);

    /* 3. control records of this round: GRAFT/PRUNE, then IHAVE (round 0)
     * and IWANT (round 1) */
    orc_handle_control(s, (int32_t)(g % m->rounds), now);
    if (g % m->rounds == 0) orc_gossip_ihave(s, m, g);
    if (g % m->rounds == 1) orc_gossip_iwant(s, m, g);

    /* this round's first receivers forward in the next one */
    fr_ent* tmp = p->fp; const int64_t cap = p->capfp;
    p->fp = p->fr; p->nfp = p->nfr; p->capfp = p->capfr;
    p->fr = tmp; p->nfr = 0; p->capfr = cap;
}
