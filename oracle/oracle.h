/*
 * oracle.h — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE.
 *
 * This library is the parity checker for the HIP engine and the timed
 * `cpu_baseline` in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path never does.
 *
 * It restates, function by function, mouzzarr/go-libp2p-pubsub:
 *   score.go (peerScore), score_params.go, gossipsub.go (heartbeat, handlers,
 *   emitGossip), mcache.go, timecache/, gossip_tracer.go
 * over the same structure-of-arrays/CSR layout the engine uses, executing the
 * deterministic BSP semantics of DESIGN.md §3 (virtual clock, ascending topic
 * order, Philox4x32-10 selection).  Parity is pinned by the reference's own
 * known-answer tests (score_test.go, score_params_test.go, mcache_test.go,
 * gossip_tracer_test.go, timecache tests) ported in tests/test_oracle_kats.py.
 */
#ifndef GSIM_ORACLE_H
#define GSIM_ORACLE_H

#include <stdint.h>
#include "../include/gsim.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Every array is caller-owned (numpy in the tests). [T][E] = topic-major. */
typedef struct orc_net {
    int64_t n, e;
    int32_t t;
    int32_t _pad;
    const uint32_t* row_ptr;   /* [N+1] */
    const uint32_t* col;       /* [E]   */
    const uint32_t* rev;       /* [E]   reverse edge index */
    const uint64_t* sub;       /* [N]   topic bitmask */
    const uint8_t*  outbound;  /* [E]   */
    const uint32_t* ip_ptr;    /* [N+1] */
    const uint32_t* ip_ids;    /* [ip_ptr[N]] */
    const uint8_t*  ip_white;  /* [n_ips] or NULL */
    const double*   p5;        /* [N] AppSpecificScore per peer, or NULL (=0) */
    double*  first;            /* [T][E] */
    double*  meshd;            /* [T][E] */
    double*  fail;             /* [T][E] */
    double*  invalid;          /* [T][E] */
    int64_t* graft_time;       /* [T][E] */
    int64_t* mesh_time;        /* [T][E] */
    uint8_t* tflags;           /* [T][E] */
    double*  bp;               /* [E] */
    uint8_t* estate;           /* [E] */
    int64_t* expire;           /* [E] */
    double*  p6;               /* [E] */
    double*  score;            /* [E] */
    int64_t* backoff;          /* [T][E] */
    const gsim_peer_score_params*  pp;
    const gsim_topic_score_params* tp;   /* [T] */
    const gsim_thresholds*         th;
    const gsim_gossipsub_params*   gp;
    uint8_t* ctl;              /* [2][T][E] control inbox by round parity */
    int64_t* lastpub;          /* [N][T] gs.lastpub[topic] (ns), 0 = none (peer-major) */
    uint64_t* fan_topics;      /* [N] bit t: gs.fanout[topic t] exists */
    const uint8_t* direct;     /* [E] col[e] is in the observer's gs.direct set (WithDirectPeers), or NULL */
    uint8_t* px;               /* [E] peer exchange (WithPeerExchange): 1 = the row's owner tries to
                                  connect to col[e] (pxConnect), or NULL */
    struct orc_gater* gater;   /* peer gater (oracle_gater.c, orc_gater_new), or NULL */
    struct orc_px_pend* px_pend;   /* Leave's pending PX lists (orc_px_pend_new), owned by the caller
                                      with the network; NULL: Leave's PRUNEs carry no lists */
} orc_net;

/* ---- message propagation (oracle_deliver.c) ------------------------------ */
/* Message ring and seen-set of the whole network (caller-owned arrays).
 * seen[slot][peer] = first-seen round (timecache + mcache put time), or
 * 0xFFFFFFFF when unseen.  Round g happens at
 *   T(g) = t0 + (g / R) * HB + (g % R + 1) * HB / (R + 1)   (integer ns). */
typedef struct orc_msgs {
    int32_t ring, rounds;
    int64_t t0, hb;
    uint32_t* topic;           /* [ring] */
    uint32_t* origin;          /* [ring] */
    uint8_t*  invalid;         /* [ring] validator verdict GSIM_VERDICT_*: 0 = accept (gsim.h) */
    uint32_t* seen;            /* [ring][N] */
    int32_t*  lastput;         /* [T][N] tick of the newest mcache.Put per (peer, topic) */
    int64_t   stats[4];        /* arrivals, first deliveries, duplicates, graylisted */
    void*     priv;            /* frontier / gossip storage (oracle-owned) */
    uint64_t* mid;             /* [ring] message id of the slot's current message (or NULL) */
    const uint8_t* behaviour;  /* [N] ORC_BEHAVE_* per peer, or NULL */
    int32_t topic_slots;       /* 0: slot = id % ring; > 0: per-topic sub-rings, topic t's messages take
                                  slots t * topic_slots + (its earlier messages mod topic_slots), as
                                  gsim_msg_config.topic_slots (the engine's seen-set layout, not the
                                  reference's: its timecache is keyed by message id) */
} orc_msgs;

#define ORC_BEHAVE_IGNORE_IWANT 0x01   /* never answers IWANT (gossipsub_spam_test.go:134-286) */

int64_t orc_round_time(const orc_msgs* m, int64_t g);
/* sizeof(orc_net), sizeof(orc_msgs): the ctypes mirrors (tests/oracle_binding.py)
 * check their own size against these when the library loads, so a field added
 * on one side only fails loudly instead of reading past the caller's struct. */
int64_t orc_layout_size(int32_t which);
/* Topic.Publish at the origin (pubsub.go:1196-1202 via pushMsg): slot =
 * id % ring is reset, the origin marks it seen at round g and forwards it in
 * round g+1. */
void orc_publish(orc_net* s, orc_msgs* m, uint64_t id, uint32_t topic, uint32_t origin, uint8_t invalid,
                 int64_t g);
/* orc_publish with a validation latency of `vdelay` rounds at every receiver
 * (async validation, validation.go:246-407): a receiver that first sees the
 * message in round g marks it seen and fulfils its promises then, but its
 * Deliver/RejectMessage (score.go:702-793), mcache.Put and forwarding happen
 * at the start of round c = g + vdelay (forwarding in round c + 1); copies
 * arriving in rounds [g, c) are pending duplicates, credited (or penalised)
 * at c with validated zero (score.go:719-725, 807-811); later copies are
 * duplicates validated at round c.  seen[] holds c. */
void orc_publish_v(orc_net* s, orc_msgs* m, uint64_t id, uint32_t topic, uint32_t origin, uint8_t invalid,
                   uint8_t vdelay, int64_t g);
/* One propagation round g: every peer that first saw (or published) a
 * message in round g-1 forwards it to its current mesh peers except the
 * sender and the origin (Publish, gossipsub.go:975-1045); receivers process
 * those copies (AcceptFrom graylist gossipsub.go:598-609; pushMsg
 * pubsub.go:1118-1162: seen-set check, DeliverMessage/DuplicateMessage/
 * RejectMessage score.go 702-827); then the control inbox of round (g % R)
 * is handled.  A message whose slot was reused is no longer forwarded. */
void orc_round(orc_net* s, orc_msgs* m, int64_t g);
void orc_msgs_free_priv(orc_msgs* m);

/* ---- gossip (oracle_gossip.c) -------------------------- */
/* heartbeat (as orc_heartbeat) followed, per joined topic, by emitGossip
 * (gossipsub.go:1554-1556, 1711-1775); IHAVE are handled in control round 0
 * and IWANT in control round 1 of the tick by orc_round. */
void orc_heartbeat_gossip(orc_net* s, orc_msgs* m, uint64_t tick, int64_t now, uint64_t seed);
/* applyIwantPenalties (gossipsub.go:1620-1625) at heartbeat time now: call
 * after orc_refresh_scores and before orc_compute_scores of the tick. */
void orc_gossip_penalties(orc_net* s, orc_msgs* m, int64_t now);

/* ---- gossipsub.go heartbeat / control handling (oracle_net.c) ----------- */
/* One heartbeat (gossipsub.go:1345-1606) for every observer at tick `tick`
 * (heartbeatTicks after the increment) and virtual time now; mesh
 * maintenance uses the score snapshot s->score (the heartbeat's lazy score
 * cache, gossipsub.go:1375-1383).  GRAFT/PRUNE go to ctl[tick parity 0]. */
void orc_heartbeat(orc_net* s, uint64_t tick, int64_t now, uint64_t seed);
/* HandleRPC control processing (handleGraft gossipsub.go:741-837, handlePrune
 * 839-871) of every receiver for the inbox of `round` (parity round&1);
 * PRUNE replies go to parity (round+1)&1.  Returns #records handled. */
int64_t orc_handle_control(orc_net* s, int32_t round, int64_t now);

/* ---- score.go ---------------------------------------------------------- */
void   orc_refresh_scores(orc_net* s, int64_t now);              /* score.go:504-565 */
double orc_score_edge(const orc_net* s, int64_t e);              /* score.go:265-342 */
void   orc_compute_scores(orc_net* s);                           /* score() for every edge */
int    orc_set_threads(int n);                                   /* OpenMP threads (n <= 0: query) */
void   orc_ip_colocation(orc_net* s);                            /* score.go:344-388 */
void   orc_add_penalty(orc_net* s, int64_t e, int32_t count);    /* score.go:391-405 */
void   orc_graft(orc_net* s, int64_t e, int32_t topic, int64_t now); /* score.go:649-667 */
void   orc_prune(orc_net* s, int64_t e, int32_t topic);          /* score.go:669-691 */
void   orc_add_peer(orc_net* s, int64_t e);                      /* score.go:595-609 */
void   orc_remove_peer(orc_net* s, int64_t e, int64_t now);      /* score.go:611-644 */
/* connection churn between ticks, both endpoints (oracle_net.c) */
int32_t orc_churn(orc_net* s, const uint32_t* pairs, int32_t count, int32_t up, int64_t now);
/* The connector (gossipsub.go:941-973) for the attempts pxConnect queued
 * (893-939): every marked pair that is a known address (a CSR edge) and not
 * connected becomes a connection, dialled by the peer that asked (the lower
 * id when both did: outbound on its side), with AddPeer at both ends.  The
 * connections made go to pairs (dialer, peer), at most cap; returns their
 * number.  Clears the marks. */
int64_t orc_px_connect(orc_net* s, int64_t now, uint32_t* pairs, int64_t cap);
/* Leave's PX lists wait here until orc_px_connect: one table per network */
struct orc_px_pend* orc_px_pend_new(void);
void orc_px_pend_free(struct orc_px_pend* p);
/* Join / Leave of (peer, topic) pairs between ticks (gossipsub.go:1047-1124,
 * gsim_set_subscriptions). */
void orc_set_subscriptions(orc_net* s, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick, int64_t now,
                           uint64_t seed);
void   orc_set_topic_params(orc_net* s, int32_t topic, gsim_topic_score_params* tp_slot,
                            const gsim_topic_score_params* np); /* score.go:201-241 */
void   orc_mark_first(orc_net* s, int64_t e, int32_t topic);     /* score.go:919-946 */
void   orc_mark_duplicate(orc_net* s, int64_t e, int32_t topic, int32_t has_validated,
                          int64_t validated, int64_t now);      /* score.go:951-981 */
void   orc_mark_invalid(orc_net* s, int64_t e, int32_t topic);   /* score.go:901-914 */

/* Message delivery records of ONE observer (score.go:90-120, 693-877). */
typedef struct orc_drecs orc_drecs;
orc_drecs* orc_drecs_new(int64_t seen_ttl);
void orc_drecs_free(orc_drecs* d);
void orc_validate_message(orc_net* s, orc_drecs* d, uint64_t mid, int64_t now);   /* 693-700 */
void orc_deliver_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                         int32_t topic, int64_t now);                            /* 702-726 */
/* reason codes = order of tracer.go:28-38 (see ORC_REJECT_*) */
void orc_reject_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                        int32_t topic, int32_t reason, int64_t now);             /* 728-793 */
void orc_duplicate_message(orc_net* s, orc_drecs* d, int64_t from_e, uint64_t mid,
                           int32_t topic, int64_t now);                          /* 795-827 */
void orc_drecs_gc(orc_drecs* d, int64_t now);                                    /* 863-877 */
void orc_drecs_expire_head(orc_drecs* d, int64_t expire);  /* test hack: score_test.go:595 */

enum {
    ORC_REJECT_BLACKLISTED_PEER = 0, ORC_REJECT_BLACKLISTED_SOURCE, ORC_REJECT_MISSING_SIGNATURE,
    ORC_REJECT_UNEXPECTED_SIGNATURE, ORC_REJECT_UNEXPECTED_AUTH_INFO, ORC_REJECT_INVALID_SIGNATURE,
    ORC_REJECT_VALIDATION_QUEUE_FULL, ORC_REJECT_VALIDATION_THROTTLED, ORC_REJECT_VALIDATION_FAILED,
    ORC_REJECT_VALIDATION_IGNORED, ORC_REJECT_SELF_ORIGIN
};

/* ---- event log of the network oracle (tests/test_oracle_linkage.py) ----- */
/* With logging on, the network oracle records what each simulated router's
 * MessageCache, seen cache and gossip tracer observe, so the KAT-pinned
 * single-router structures below can be driven with the same events and
 * compared with the network oracle's implicit windows, seen cells and
 * promise lists. */
enum {
    ORC_EV_PUT = 1,        /* a: peer, mid, topic            mcache.Put            */
    ORC_EV_SEEN = 2,       /* a: peer, b: sender (0xFFFFFFFF: its own publication), mid,
                              x: 1 new / 0 seen  seenMessage/markSeen */
    ORC_EV_SERVE = 3,      /* a: advertiser, b: requester, mid, x: GetForPeer count */
    ORC_EV_PROMISE = 4,    /* a: requester, b: advertiser, mid, x: now (AddPromise)  */
    ORC_EV_FULFILL = 5,    /* a: peer, mid                   fulfillPromise        */
    ORC_EV_BROKEN = 6,     /* a: peer, b: advertiser, x: count (GetBrokenPromises)  */
    ORC_EV_PENALTIES = 7,  /* x: now: applyIwantPenalties (every peer)              */
    ORC_EV_HEARTBEAT = 8,  /* x: tick: GetGossipIDs then Shift (every peer)         */
    ORC_EV_GOSSIP_ID = 9,  /* a: peer, mid, topic: one id of GetGossipIDs(topic)    */
    /* the tracer's view (trace export, include/gsim.h gsim_trace_event) */
    ORC_EV_REJECT_SIG = 10,  /* a: peer, b: sender, mid, topic: a bad-signature copy  */
    ORC_EV_PUBLISH = 11,     /* a: origin, mid, topic                                */
    ORC_EV_GRAFT = 12,       /* a: router, b: peer, topic, x: now  tracer.Graft      */
    ORC_EV_PRUNE = 13,       /* a: router, b: peer, topic, x: now  tracer.Prune      */
    ORC_EV_ADD_PEER = 14,    /* a: router, b: peer, x: now                           */
    ORC_EV_REMOVE_PEER = 15, /* a: router, b: peer, x: now                           */
    ORC_EV_THROTTLE = 16,    /* a: receiver, b: sender, x: now: AcceptControl -> ThrottlePeer */
    ORC_EV_JOIN = 17,        /* a: router, topic, x: now    tracer.Join              */
    ORC_EV_LEAVE = 18,       /* a: router, topic, x: now    tracer.Leave             */
    ORC_EV_PX_PEER = 19,     /* a: pruner, b: a peer of the PRUNE's PX list, topic,
                                mid: the pruned peer, g: its rank in the list (makePrune) */
    ORC_EV_RPC_MSG = 20,     /* a: sender, b: receiver, mid, topic, g: the round it arrives in,
                                x: 0 a forwarded copy (sent in g), 1 an IWANT answer (sent in g - 1) */
    ORC_EV_RPC_IWANT = 21,   /* a: requester, b: advertiser, mid, topic, g: the round the IWANT is sent
                                in (handleIHave's reply, gossipsub.go:611-627); it arrives in g + 1 */
};
typedef struct orc_event { int32_t kind, topic; uint32_t a, b; int64_t g; uint64_t mid; int64_t x; } orc_event;
void    orc_msgs_log(orc_msgs* m, int32_t on);
int64_t orc_msgs_events(orc_msgs* m, orc_event* out, int64_t cap);   /* copies and clears; returns the count */
int64_t orc_msgs_ihave_marks(orc_msgs* m, uint8_t* out, int64_t n);   /* last heartbeat's [T][E] IHAVE marks */

/* ---- mcache.go (one router's MessageCache) ------------------------------ */
typedef struct orc_mcache orc_mcache;
orc_mcache* orc_mcache_new(int32_t gossip, int32_t history);            /* mcache.go:21-36 */
void orc_mcache_free(orc_mcache* m);
void orc_mcache_put(orc_mcache* m, uint64_t mid, int32_t topic);        /* mcache.go:55-59 */
int  orc_mcache_get(orc_mcache* m, uint64_t mid);                       /* mcache.go:61-64 */
int  orc_mcache_get_for_peer(orc_mcache* m, uint64_t mid, uint32_t peer, int32_t* count); /* 66-80 */
int  orc_mcache_gossip_ids(orc_mcache* m, int32_t topic, uint64_t* out, int32_t cap);     /* 82-92 */
void orc_mcache_shift(orc_mcache* m);                                   /* mcache.go:94-104 */
int  orc_mcache_len(orc_mcache* m);

/* ---- gossip_tracer.go (one router's promise tracker) -------------------- */
typedef struct orc_gtracer orc_gtracer;
orc_gtracer* orc_gtracer_new(int64_t followup);
void orc_gtracer_free(orc_gtracer* g);
/* AddPromise picks msg_ids[pick] (the reference uses rand.Intn; the caller
 * supplies the index, gossip_tracer.go:48-75). */
void orc_gtracer_add_promise(orc_gtracer* g, uint32_t peer, const uint64_t* mids, int32_t n,
                             int32_t pick, int64_t now);
/* GetBrokenPromises, gossip_tracer.go:79-115: fills peers/counts (sorted by
 * peer), returns the number of peers with broken promises. */
int  orc_gtracer_broken(orc_gtracer* g, int64_t now, uint32_t* peers, int32_t* counts, int32_t cap);
void orc_gtracer_fulfill(orc_gtracer* g, uint64_t mid);                 /* 119-141 */
void orc_gtracer_throttle(orc_gtracer* g, uint32_t peer);               /* 182-200 */
int  orc_gtracer_peer_promises(orc_gtracer* g);                         /* len(peerPromises) */

/* ---- timecache/ --------------------------------------------------------- */
typedef struct orc_tcache orc_tcache;
orc_tcache* orc_tcache_new(int32_t strategy /*0 first-seen, 1 last-seen*/, int64_t ttl);
void orc_tcache_free(orc_tcache* c);
int  orc_tcache_add(orc_tcache* c, uint64_t id, int64_t now);  /* first_seen_cache.go:47-56 / last_seen_cache.go:38-45 */
int  orc_tcache_has(orc_tcache* c, uint64_t id, int64_t now);  /* first_seen_cache.go:37-45 / last_seen_cache.go:47-58 */
void orc_tcache_sweep(orc_tcache* c, int64_t now);             /* timecache/util.go:26-35 */

/* ---- peer gater (oracle_gater.c, peer_gater.go) ------------------------- */
typedef struct orc_gater orc_gater;
enum { ORC_GATE_VALIDATE = 0, ORC_GATE_DELIVER, ORC_GATE_DUPLICATE, ORC_GATE_IGNORE, ORC_GATE_REJECT,
       ORC_GATE_THROTTLE };
int orc_gater_validate(const gsim_peer_gater_params* p);                /* peer_gater.go:57-90 */
uint64_t orc_gater_weight_fp(double w);
orc_gater* orc_gater_new(orc_net* s, const gsim_peer_gater_params* p, const double* topic_w);   /* sets s->gater */
void orc_gater_free(orc_gater* g);
void orc_gater_round_begin(orc_net* s, int64_t now);                    /* AcceptFrom preamble :327-343 */
double orc_gater_uniform(uint64_t seed, int64_t g, uint32_t recv, uint32_t slot, uint32_t sender);
int orc_gater_accept(orc_net* s, uint64_t seed, int64_t g, uint32_t i, uint32_t er, uint32_t slot);   /* :320-363 */
void orc_gater_event(orc_net* s, uint32_t i, uint32_t er, int32_t topic, int32_t kind);   /* :386-432 */
void orc_gater_round_end(orc_net* s, int64_t now);
void orc_gater_decay(orc_net* s, int64_t now);                          /* decayStats :207-241 */
void orc_gater_connection(orc_net* s, int64_t e, int32_t up, int64_t now);   /* AddPeer/RemovePeer :366-384 */
int64_t orc_gater_throttled(const orc_gater* g);
void orc_gater_read(const orc_gater* g, double* val, double* thr, int64_t* last, double* counters4, int32_t* con,
                    int64_t* exp);

/* ---- Philox4x32-10 (the canonical selection stream) ----- */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
