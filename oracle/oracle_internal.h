/*
 * oracle_internal.h — state shared by the oracle's network-level files.
 * TEST INFRASTRUCTURE (see oracle.h).
 */
#ifndef GSIM_ORACLE_INTERNAL_H
#define GSIM_ORACLE_INTERNAL_H

#include "oracle.h"

/* Purposes of the Philox selection keys (counter word 2 = topic << 8 |
 * purpose); the engine's csrc/philox.h uses the same numbers. */
enum {
    P_GRAFT_DLO = 1, P_PRUNE_SHUF1 = 2, P_PRUNE_SHUF2 = 3, P_GRAFT_DOUT = 4, P_GRAFT_OPP = 5,
    P_GOSSIP = 6,       /* emitGossip: shufflePeers(peers)             gossipsub.go:1758 */
    P_IWANT = 7,        /* handleIHave: shuffleStrings(iwantlst)       gossipsub.go:687  */
    P_PROMISE = 8,      /* AddPromise: rand.Intn(len(msgIDs))          gossip_tracer.go:53 */
    P_GOSSIP_FILL = 9,  /* emitGossip: map order of the Dlo fill loop  gossipsub.go:1739-1748 */
    P_GOSSIP_DUP = 10,  /* emitGossip: shuffle key of a fill duplicate */
    P_IHAVE_TRUNC = 11, /* emitGossip: per-peer shuffleStrings(mids)   gossipsub.go:1766-1771 */
    P_FANOUT_NEW = 12,  /* Publish: getPeers for a new fanout          gossipsub.go:1020-1023 */
    P_FANOUT = 13,      /* heartbeat: getPeers for the fanout top-up  gossipsub.go:1578-1585 */
    P_PX = 14,          /* makePrune: getPeers for PX (heartbeat)      gossipsub.go:1879-1882 */
    P_PX_GRAFT = 15,    /* makePrune: getPeers for PX (GRAFT reply)    gossipsub.go:831-834 */
    P_GATER = 16,       /* peer gater: rand.Float64() of AcceptFrom    peer_gater.go:357 */
    P_JOIN = 17,        /* Join: getPeers for the new mesh             gossipsub.go:1068-1092 */
    P_PX_LEAVE = 18,    /* makePrune: getPeers for PX (Leave's PRUNEs)  gossipsub.go:1118, 1866-1906 */
};

static inline uint64_t okey(uint64_t seed, uint64_t tick, uint32_t obs, int32_t topic, uint32_t purpose,
                            uint32_t item, uint32_t pos)
{
    uint32_t ctr[4] = {(uint32_t)tick, obs, ((uint32_t)topic << 8) | purpose, item};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    orc_philox4x32_10(ctr, key, out);
    return ((uint64_t)out[0] << 32) | pos;
}

/* PX keys (csrc/philox.h px_base / px_key): one draw per (observer, topic,
 * candidate) and pass, mixed with the pruned peer's row position per PRUNE */
static inline uint32_t opx_base(uint64_t seed, uint64_t tick, uint32_t obs, int32_t topic, uint32_t purpose,
                                uint32_t item)
{
    uint32_t ctr[4] = {(uint32_t)tick, obs, ((uint32_t)topic << 8) | purpose, item};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t out[4];
    orc_philox4x32_10(ctr, key, out);
    return out[0];
}

static inline uint64_t opx_key(uint32_t base, uint32_t pruned_pos, uint32_t pos)
{
    uint32_t h = base ^ ((pruned_pos + 1u) * 0x9E3779B9u);
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return ((uint64_t)h << 32) | pos;
}

typedef struct fr_ent { uint32_t peer, slot, from; } fr_ent;
/* a copy at its receiver; resp: an IWANT answer (one RPC per sender and round) */
typedef struct arr_ent { uint32_t recv, slot, er, resp; } arr_ent;
/* the peer gater's draw key of an IWANT answer: one draw per (round, receiver,
 * sender) covers the whole answer RPC (AcceptFrom per RPC, pubsub.go) */
#define ORC_GATER_RPC_SLOT 0xFFFFFFu
/* a copy whose receiver is still validating the message: credited or
 * penalised when validation completes in round c (orc_publish_v) */
typedef struct pend_ent { int64_t c; uint32_t recv, slot, er; int32_t first; } pend_ent;

/* one outstanding IWANT promise of a receiver (gossip_tracer.go:21-27) */
typedef struct promise { uint32_t e; uint32_t slot; uint64_t mid; int64_t expire; } promise;
/* one IWANT in flight from round 0 to round 1: receiver edge er (at the
 * requester), message slot */
typedef struct iwant_ent { uint32_t er, slot; } iwant_ent;

typedef struct peertx_ent { uint64_t mid; uint32_t e; int32_t count; } peertx_ent;

typedef struct priv {
    fr_ent* fr; int64_t nfr, capfr;     /* peers that first-saw a message this round */
    fr_ent* fp; int64_t nfp, capfp;     /* ... in the previous round: they forward now */
    arr_ent* ar; int64_t nar, capar;    /* copies delivered this round */
    arr_ent* gr; int64_t ngr, capgr;    /* IWANT responses: delivered next round */
    /* gossip (emitGossip / handleIHave / handleIWant / gossipTracer) */
    uint8_t* ihave;                     /* [T][E] receiver edge: IHAVE(topic) from col[e] this heartbeat */
    int64_t ihave_tick;                 /* heartbeat that emitted them */
    uint64_t seed;
    iwant_ent* iw; int64_t niw, capiw;  /* IWANTs sent in control round 0 */
    promise** pr; int32_t* npr; int32_t* cappr;   /* [N] promises per receiver */
    peertx_ent* tx; int64_t ntx, captx; /* mcache.peertx: (mid, edge i->p) -> count, open addressing */
    int64_t n_alloc, te_alloc;
    int64_t* slot_last;                 /* [ring] last round with a first reception (or the publication) */
    uint32_t* cand; int32_t* cand_ptr;  /* per-topic recent slots at the current heartbeat (CSR) */
    uint8_t* vd;                        /* [ring] validation latency of the slot's message, rounds */
    int64_t* tcount;                    /* [64] messages published per topic (orc_msgs.topic_slots) */
    pend_ent* pq; int64_t npq, cappq;   /* copies pending validation */
    int32_t log_on;                     /* event log (orc_msgs_log) */
    orc_event* ev; int64_t nev, capev;
} priv;

/* one event, when logging is on */
void orc_log(orc_msgs* m, int32_t kind, uint32_t a, uint32_t b, uint32_t slot, int32_t topic, int64_t g, int64_t x);
/* router-level events (GRAFT/PRUNE/ADD/REMOVE) go to the message log that
 * last turned logging on (orc_msgs_log); safe inside the OpenMP phases */
void orc_log_net(int32_t kind, uint32_t a, uint32_t b, int32_t topic, int64_t now);
void orc_log_net_x(int32_t kind, uint32_t a, uint32_t b, int32_t topic, uint64_t mid, int64_t g, int64_t x);

priv* orc_msgs_priv(orc_msgs* m);
int64_t orc_round_time(const orc_msgs* m, int64_t g);

/* gossip (oracle_gossip.c) */
void orc_gossip_emit(orc_net* s, orc_msgs* m, uint32_t i, int32_t t, uint64_t tick, uint64_t seed,
                     uint8_t exclude);
/* Publish's fanout branch (oracle_net.c) */
void orc_fanout_publish(orc_net* s, uint32_t origin, int32_t topic, int64_t g, int64_t now, uint64_t seed);
void orc_gossip_fulfill(orc_msgs* m, uint32_t p, uint32_t slot);
void orc_gossip_ihave(orc_net* s, orc_msgs* m, int64_t g);
void orc_gossip_index(const orc_net* s, orc_msgs* m, int64_t tick);
void orc_gossip_iwant(orc_net* s, orc_msgs* m, int64_t g);

#endif
