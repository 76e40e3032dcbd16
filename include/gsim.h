/*
 * gsim.h — C ABI of the MI355X-native GossipSub scoring + heartbeat engine.
 *
 * This is the drop-in boundary for the reference's hot path.
 * Every entry point names the reference interface it replaces (file:line into
 * mouzzarr/go-libp2p-pubsub).  Conventions:
 *   - plain C types only; durations are int64 nanoseconds (Go time.Duration);
 *   - every function returns int: 0 = OK, negative errno-style on error;
 *     a human-readable message is available from gsim_last_error(h)
 *     (the reference returns Go `error`s with the same meaning);
 *   - no allocation crosses the boundary; callers own every buffer they pass,
 *     inputs are copied in, readbacks copy out (blocking);
 *   - a handle is single-threaded (the reference serializes all router and
 *     peerScore work on one event loop, pubsub.go:561-675);
 *   - topics cross as dense indices 0..T-1 (the Go shim maps topic strings to
 *     indices in sorted order); peers cross as dense indices 0..N-1.
 */
#ifndef GSIM_H
#define GSIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define GSIM_OK        0
#define GSIM_EINVAL  (-22) /* invalid argument / parameter validation failed */
#define GSIM_ENOMEM  (-12) /* device or host allocation failed               */
#define GSIM_EDEVICE  (-5) /* HIP runtime error, or no gfx950 device           */
#define GSIM_ERANGE  (-34) /* size outside what the engine supports           */
#define GSIM_ESTATE  (-71) /* call out of order (e.g. step before load_graph)  */

/* ---- parameter blocks (field-for-field mirrors of the Go structs) ------- */

/* TopicScoreParams, score_params.go:117-170. */
typedef struct gsim_topic_score_params {
    int32_t skip_atomic_validation;
    int32_t scored;                 /* 1 if present in PeerScoreParams.Topics */
    double  topic_weight;
    /* P1 */
    double  time_in_mesh_weight;
    int64_t time_in_mesh_quantum_ns;
    double  time_in_mesh_cap;
    /* P2 */
    double  first_message_deliveries_weight;
    double  first_message_deliveries_decay;
    double  first_message_deliveries_cap;
    /* P3 */
    double  mesh_message_deliveries_weight;
    double  mesh_message_deliveries_decay;
    double  mesh_message_deliveries_cap;
    double  mesh_message_deliveries_threshold;
    int64_t mesh_message_deliveries_window_ns;
    int64_t mesh_message_deliveries_activation_ns;
    /* P3b */
    double  mesh_failure_penalty_weight;
    double  mesh_failure_penalty_decay;
    /* P4 */
    double  invalid_message_deliveries_weight;
    double  invalid_message_deliveries_decay;
} gsim_topic_score_params;

/* PeerScoreParams, score_params.go:66-115.  AppSpecificScore (a Go callback)
 * is replaced by a per-peer array set with gsim_set_app_score();
 * IPColocationFactorWhitelist (CIDR list) by a per-IP flag array set with
 * gsim_set_ip_whitelist(). */
typedef struct gsim_peer_score_params {
    int32_t skip_atomic_validation;
    int32_t has_app_specific_score;   /* AppSpecificScore != nil */
    double  topic_score_cap;
    double  app_specific_weight;
    double  ip_colocation_factor_weight;
    int32_t ip_colocation_factor_threshold;
    int32_t _pad0;
    double  behaviour_penalty_weight;
    double  behaviour_penalty_threshold;
    double  behaviour_penalty_decay;
    int64_t decay_interval_ns;
    double  decay_to_zero;
    int64_t retain_score_ns;
    int64_t seen_msg_ttl_ns;
} gsim_peer_score_params;

/* PeerScoreThresholds, score_params.go:12-35. */
typedef struct gsim_thresholds {
    int32_t skip_atomic_validation;
    int32_t _pad0;
    double  gossip_threshold;
    double  publish_threshold;
    double  graylist_threshold;
    double  accept_px_threshold;
    double  opportunistic_graft_threshold;
} gsim_thresholds;

/* GossipSubParams, gossipsub.go:63-205 (defaults gossipsub.go:244-275). */
typedef struct gsim_gossipsub_params {
    int32_t d, dlo, dhi, dscore, dout;
    int32_t history_length, history_gossip;
    int32_t dlazy;
    double  gossip_factor;
    int32_t gossip_retransmission;
    int32_t prune_peers;
    int64_t heartbeat_initial_delay_ns;
    int64_t heartbeat_interval_ns;
    double  slow_heartbeat_warning;
    int64_t fanout_ttl_ns;
    int64_t prune_backoff_ns;
    int64_t unsubscribe_backoff_ns;
    int32_t connectors;
    int32_t max_pending_connections;
    int64_t connection_timeout_ns;
    uint64_t direct_connect_ticks;
    int64_t direct_connect_initial_delay_ns;
    uint64_t opportunistic_graft_ticks;
    int32_t opportunistic_graft_peers;
    int32_t max_ihave_length;
    int64_t graft_flood_threshold_ns;
    int32_t max_ihave_messages;
    int32_t flood_publish;   /* router option WithFloodPublish (gossipsub.go:321-334); this fork's default is 0 */
    int64_t iwant_followup_time_ns;
    int32_t do_px;           /* router option WithPeerExchange (gossipsub.go:340-350): PRUNEs carry PX; default 0 */
    int32_t _pad_px;
} gsim_gossipsub_params;

/* ---- host-side parameter API (no device needed) ------------------------ */

/* DefaultGossipSubParams(), gossipsub.go:244-275. */
void gsim_default_gossipsub_params(gsim_gossipsub_params* out);

/* TopicScoreParams.validate(), score_params.go:236-398.  err may be NULL. */
int gsim_validate_topic_params(const gsim_topic_score_params* p, char* err, size_t errlen);
/* PeerScoreParams.validate(), score_params.go:173-234 (validates every scored
 * topic first, as the reference does). */
int gsim_validate_peer_params(const gsim_peer_score_params* p,
                              const gsim_topic_score_params* topics, int32_t n_topics,
                              char* err, size_t errlen);
/* PeerScoreThresholds.validate(), score_params.go:37-64. */
int gsim_validate_thresholds(const gsim_thresholds* p, char* err, size_t errlen);
/* NewMessageCache(gossip, history) panics if gossip > history, mcache.go:21-26;
 * here it is a GSIM_EINVAL from gsim_create. */

/* ScoreParameterDecay / ScoreParameterDecayWithBase, score_params.go:405-417. */
double gsim_score_parameter_decay(int64_t decay_ns);
double gsim_score_parameter_decay_with_base(int64_t decay_ns, int64_t base_ns, double decay_to_zero);

/* ---- engine lifecycle -------------------------------------------------- */

typedef struct gsim_handle gsim_handle;

/* Replaces WithPeerScore(params, thresholds) (gossipsub.go:278-319) +
 * WithGossipSubParams (gossipsub.go:398-411) + newPeerScore (score.go:183-195).
 * Validates like the reference (GSIM_EINVAL + message; the message is also
 * written to err when err != NULL since no handle exists on failure).
 * device: HIP device ordinal. */
int gsim_create(const gsim_peer_score_params* params,
                const gsim_topic_score_params* topics, int32_t n_topics,
                const gsim_thresholds* thresholds,
                const gsim_gossipsub_params* gossip,
                int32_t device, gsim_handle** out, char* err, size_t errlen);
/* newPeerScore (score.go:183-195) without WithPeerScore's validation: the
 * reference's unit tests build peerScore this way with parameters validate()
 * would reject (e.g. decay 1.0).  Also disables validation in
 * gsim_set_topic_params for this handle. */
int gsim_create_unvalidated(const gsim_peer_score_params* params,
                            const gsim_topic_score_params* topics, int32_t n_topics,
                            const gsim_thresholds* thresholds,
                            const gsim_gossipsub_params* gossip,
                            int32_t device, gsim_handle** out, char* err, size_t errlen);
int gsim_destroy(gsim_handle* h);
const char* gsim_last_error(const gsim_handle* h);

/* Load the simulated network: a CSR of N observers.  Row i lists the peers i
 * is connected to (must be symmetric: j in row i <=> i in row j; rows sorted
 * ascending, no self loops, no duplicates).  outbound[e] = 1 if observer
 * row(e) initiated the connection to col[e] (gossipsub.go:525-552).
 * subscriptions[i] = bitmask of topics peer i subscribes to (T <= 64).
 * ip_ptr/ip_ids = per-peer CSR of IP ids as seen by its neighbours
 * (score.go:984-1024 getIPs; IPv6 /64 prefixes are just more ids).
 * Every edge starts tracked+connected (AddPeer, score.go:595-609) with zero
 * counters, nothing in any mesh.  Copies everything. */
int gsim_load_graph(gsim_handle* h, int64_t n_peers,
                    const uint32_t* row_ptr, const uint32_t* col_idx,
                    const uint8_t* outbound, const uint64_t* subscriptions,
                    const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips);

/* AppSpecificScore(p) for every peer (score_params.go:78) — host refreshes. */
int gsim_set_app_score(gsim_handle* h, const double* p5);
/* IPColocationFactorWhitelist (score_params.go:91): whitelisted[ip_id] = 1 if
 * any whitelisted CIDR contains that IP (host precomputes net.IPNet.Contains). */
int gsim_set_ip_whitelist(gsim_handle* h, const uint8_t* whitelisted);
/* WithDirectPeers (gossipsub.go:352-374): flags[e] != 0 when col[e] is in
 * the observer's direct set (E bytes, edge order; NULL clears).  Direct
 * peers are never grafted or gossiped to, GRAFTs from them are answered
 * with PRUNE (gossipsub.go:768-776), they receive every message of a topic
 * they joined (991-1003) and AcceptFrom accepts them whatever their score
 * (598-609).  The reconnect loop (directConnect) is not modelled. */
int gsim_set_direct_peers(gsim_handle* h, const uint8_t* flags);
/* SetTopicScoreParams (score.go:201-241, topic.go:44-82): validates, installs,
 * and recaps first/mesh counters when caps are lowered. */
int gsim_set_topic_params(gsim_handle* h, int32_t topic, const gsim_topic_score_params* p);

/* ---- hot path ---------------------------------------------------------- */

/* peerScore.refreshScores (score.go:504-565) for every observer at virtual
 * time now_ns, fused with peerScore.score (score.go:265-342) of every edge into
 * the score snapshot; P6 (score.go:344-388) is re-derived first when the
 * tracked set changed. */
int gsim_refresh_scores(gsim_handle* h, int64_t now_ns);
/* peerScore.score only (no decay) for every edge -> score snapshot. */
int gsim_compute_scores(gsim_handle* h);
/* ipColocationFactor (score.go:344-388) for every edge (segmented count over
 * each observer's neighbour IPs). */
int gsim_compute_ip_colocation(gsim_handle* h);

/* Seed of the Philox stream that replaces the reference's global math/rand
 * (gossipsub.go:1954-1973, gossip_tracer.go:53). */
int gsim_set_seed(gsim_handle* h, uint64_t seed);

/* GossipSubRouter.heartbeat (gossipsub.go:1345-1606) for every observer at
 * heartbeat tick `tick` (heartbeatTicks after its increment, so the first
 * heartbeat is tick 1) and virtual time now_ns: clearBackoff every 15 ticks,
 * per joined topic in ascending order: negative-score prune, Dlo graft, Dhi
 * score/random prune with the Dout rotation, Dout top-up, opportunistic graft
 * every OpportunisticGraftTicks; Graft/Prune traced into the score counters.
 * Uses the current score snapshot as the heartbeat's score cache
 * (gossipsub.go:1375-1383): call gsim_refresh_scores first.  GRAFT/PRUNE
 * records land in the receivers' control inbox for round 0.  Fails with the
 * previous tick's delivery error, if any (GSIM_ERANGE: the IWANT response
 * queue overflowed; GSIM_ESTATE: a slot was republished too early). */
int gsim_heartbeat(gsim_handle* h, uint64_t tick, int64_t now_ns);
/* Control-message round: every receiver handles the GRAFT/PRUNE records in
 * its inbox for `round` (handleGraft gossipsub.go:741-837, handlePrune
 * 839-871), senders in ascending peer order; PRUNE replies land in the inbox
 * of round+1. */
int gsim_handle_control(gsim_handle* h, int32_t round, int64_t now_ns);

/* Connections going down (up = 0) or up (up = 1) between two ticks, both
 * endpoints notified (handleDeadPeers pubsub.go:711-759; the new-peer case of
 * processLoop pubsub.go:575-595).  pairs = count (peer a, peer b) u32 pairs,
 * each an existing CSR connection, each at most once.
 *   down: router RemovePeer (gossipsub.go:554-567): out of every mesh without
 *         PRUNE, pending control dropped, backoff kept; score tracer
 *         RemovePeer (score.go:611-644): a positive live score is dropped,
 *         otherwise retained until now + RetainScore with P2 reset and the
 *         P3b penalty applied.
 *   up:   router AddPeer (gossipsub.go:525-552), peerScore.AddPeer
 *         (score.go:595-609): a retained record is reused, else a fresh one.
 * The removed peer's live score uses P6 over the tracked set as the batch
 * starts (re-derived if an up batch changed it).  GSIM_EINVAL if a
 * pair is not a connection or is listed twice (nothing is changed then). */
int gsim_set_connections(gsim_handle* h, const uint32_t* pairs, int32_t count, int32_t up, int64_t now_ns);

/* Peer exchange (WithPeerExchange: gsim_gossipsub_params.do_px).  PRUNEs
 * carry PX (makePrune, gossipsub.go:1866-1906: the heartbeat's Dhi prunes and
 * handleGraft's mesh-full replies); the pruned peer's handlePrune accepts it
 * from peers it scores at least acceptPXThreshold and pxConnect queues a
 * connection attempt to every listed peer it is not connected to
 * (gossipsub.go:860-869, 893-939).  This call is the connector
 * (gossipsub.go:941-973), run between ticks: every attempt whose peers know
 * each other's address (an edge of the loaded graph) and are not connected
 * becomes a connection, dialled by the peer that asked (outbound on its side;
 * the lower id when both asked), with AddPeer at both ends as in
 * gsim_set_connections.  pairs (optional, cap entries): the (dialer, peer)
 * pairs connected, sorted.  Single engines only. */
int gsim_px_connect(gsim_handle* h, int64_t now_ns, uint32_t* pairs, int64_t cap, int64_t* n_connected);

/* ---- message propagation ------------------------------ */
/* Rounds are numbered globally: round g belongs to heartbeat tick g / rounds
 * and happens at virtual time
 *   T(g) = t0 + (g / rounds) * heartbeat + (g % rounds + 1) * heartbeat / (rounds + 1).
 * The seen-set is a ring of `ring` message slots x N peers (u32 first-seen
 * round, 0xFFFFFFFF = unseen): the timecache (timecache/first_seen_cache.go)
 * restricted to messages that can still arrive.  Publishing into a slot ends
 * the propagation of its previous message; SeenMsgTTL and the ring must
 * outlast a message's propagation (they do for every reference configuration). */
/* Subscription changes between ticks (Topic.Subscribe / Cancel through
 * pubsub.go:1051-1079 announcements and the router's Join / Leave,
 * gossipsub.go:1047-1124), for (peer, topic) pairs.  join = 1: Join(topic):
 * the peer announces the topic; its fanout peers (score >= 0, no backoff)
 * become the mesh, topped up to D with getPeers (not direct, no backoff,
 * score >= 0), or D such peers without a fanout; tracer.Graft and a GRAFT to
 * each.  join = 0: Leave(topic): the announcement is withdrawn; every mesh
 * peer gets tracer.Prune, a PRUNE whose backoff is UnsubscribeBackoff and an
 * UnsubscribeBackoff of its own.  A change that is already in effect is a
 * no-op.  Scores are the snapshot; getPeers keys use `tick` (call before that
 * tick's refresh, as gsim_set_connections); the GRAFT/PRUNE are handled with
 * the heartbeat's in control round 0.  Peers that withdrew a topic drop its
 * messages (pubsub.go:1094-1098).  Leave's PRUNEs carry no peer exchange.
 * JOIN / LEAVE / GRAFT / PRUNE trace events.  Single engine. */
int gsim_set_subscriptions(gsim_handle* h, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick,
                           int64_t now_ns);

/* ---- peer gater (peer_gater.go) ------------------------------------------
 * WithPeerGater(params) (peer_gater.go:161-186): every router's AcceptFrom
 * adds the random-early-drop gate of peer_gater.go:320-363 behind the
 * graylist (gossipsub.go:598-609): once the router's validation throttles
 * (a message with GSIM_VERDICT_THROTTLE) and throttle/validate reaches
 * Threshold within Quiet of the last throttle, a message from a peer is
 * accepted with probability (1 + deliver) / (1 + weighted total) of its
 * IP's counters, else dropped (AcceptControl; the receiver's IWANT promises
 * from that peer are forgotten, gossip_tracer.go:182-200).  Field for field
 * PeerGaterParams (peer_gater.go:31-55); durations in ns.  Restatement
 * (DESIGN.md §3.9 step 7): the gate is drawn per message copy (Philox), a
 * round's tracer events are added to the counters at the end of the round,
 * TopicDeliveryWeights in 2^-16 units, decayStats at every score refresh
 * (DecayInterval must equal the heartbeat interval); single engine, no
 * validation latency. */
typedef struct gsim_peer_gater_params {
    double threshold;          /* Threshold: throttle / validate ratio that turns the gate on */
    double global_decay;       /* GlobalDecay (validate, throttle) */
    double source_decay;       /* SourceDecay (per-IP counters) */
    int64_t decay_interval_ns; /* DecayInterval */
    double decay_to_zero;      /* DecayToZero */
    int64_t retain_stats_ns;   /* RetainStats: an IP's stats after its last peer left */
    int64_t quiet_ns;          /* Quiet: the gate turns off this long after the last throttle */
    double duplicate_weight;   /* DuplicateWeight */
    double ignore_weight;      /* IgnoreWeight */
    double reject_weight;      /* RejectWeight */
} gsim_peer_gater_params;

/* PeerGaterParams.validate (peer_gater.go:57-90), the reference's messages. */
int gsim_validate_peer_gater_params(const gsim_peer_gater_params* p, char* err, size_t errlen);
/* NewPeerGaterParams(threshold, globalDecay, sourceDecay) defaults (peer_gater.go:99-111). */
int gsim_default_peer_gater_params(double threshold, double global_decay, double source_decay,
                                   gsim_peer_gater_params* out);
/* Turn the gater on for every router (after gsim_msgs_init).  topic_weights:
 * TopicDeliveryWeights per topic index ([T], 0 = 1.0; multiples of 2^-16),
 * or NULL.  GSIM_EINVAL: invalid params or weights; GSIM_ESTATE: a shard,
 * a message with validation latency published, or DecayInterval not the
 * heartbeat interval. */
int gsim_set_peer_gater(gsim_handle* h, const gsim_peer_gater_params* p, const double* topic_weights);
/* Message copies dropped by the gate (AcceptControl) so far. */
int gsim_gater_throttled(gsim_handle* h, int64_t* out);
/* The gater state (host buffers, each may be NULL): per router validate,
 * throttle [N] and lastThrottle [N] (INT64_MIN: never); per connection
 * e (edge order) the counters deliver, duplicate, ignore, reject [4][E],
 * connected [E] and expire [E] of its IP group, held at the group's
 * representative edge (the row's lowest position of that IP; other
 * positions read 0). */
int gsim_gater_read(gsim_handle* h, double* validate, double* throttle, int64_t* last, double* counters4,
                    int32_t* connected, int64_t* expire);

typedef struct gsim_msg_config {
    int32_t ring;            /* message slots (live-message window), 1..8192 */
    int32_t rounds;          /* propagation rounds per heartbeat, >= 2 */
    int64_t t0_ns;           /* virtual time of tick 0 */
    int64_t heartbeat_ns;    /* heartbeat interval (GossipSubParams.HeartbeatInterval) */
    int64_t max_frontier;    /* 0: default.  > 0: a memory bound on the round lists of member-compacted
                                layouts (topic_slots > 0): the claim list holds this many entries
                                (default max(4 N, 2^20)), each forwarder list half as many; a round
                                that overflows either is completed by the word scans (k_commit,
                                k_send_tm) -- the same results, slower.  A sharded group also sizes
                                its frontier export with it (gsim_group_msgs_init) */
    int64_t max_arrivals;    /* capacity of the IWANT response queue per tick (0: max(8 N, 2^20)) */
    int64_t topic_slots;     /* 0: one ring shared by every topic, a message's slot is id % ring, and
                                every slot keeps a seen-set cell per peer.  > 0: per-topic sub-rings
                                (ring = n_topics * topic_slots): topic t owns slots [t * topic_slots,
                                (t + 1) * topic_slots) and its messages take them in publication
                                order; each slot keeps cells only for the peers holding topic t (its
                                slot mask), so the seen-set scales with the topics'
                                members, not with the network (timecache, pubsub.go:987-995) */
} gsim_msg_config;

/* The validation verdict every receiver reaches for a message (validation
 * is instantaneous here, validation.go:282-407), with the score tracer's
 * handling of it (score.go:693-827) and the gossip tracer's (gossip_tracer.go
 * 148-170).  The origin publishes its message whatever the verdict. */
#define GSIM_VERDICT_ACCEPT    0  /* DeliverMessage: P2 / P3 credit, forwarded, mcache.Put           */
#define GSIM_VERDICT_REJECT    1  /* RejectValidationFailed: seen, P4 for the first and every later
                                     sender, not forwarded                                          */
#define GSIM_VERDICT_IGNORE    2  /* RejectValidationIgnored: seen, no credit and no penalty for any
                                     copy, not forwarded                                            */
#define GSIM_VERDICT_THROTTLE  3  /* RejectValidationThrottled: as IGNORE                           */
#define GSIM_VERDICT_SIGNATURE 4  /* RejectInvalidSignature (before markSeen, validation.go:282-290):
                                     every copy's sender gets P4, the message is never seen (so IWANT
                                     asks again) and the IWANT promise is not fulfilled            */

/* One published message (Topic.Publish, topic.go:217-283, at its origin). */
typedef struct gsim_msg {
    uint64_t id;             /* message id; slot = id % ring */
    uint32_t topic;          /* dense topic index */
    uint32_t origin;         /* publishing peer (must be subscribed) */
    uint8_t  verdict;        /* GSIM_VERDICT_* at every receiver */
    uint8_t  vdelay;         /* validation latency at every receiver, in rounds (0..GSIM_MAX_VDELAY):
                                async validation (validation.go:246-407) — a receiver that first sees
                                the message in round g marks it seen then, and its Deliver/Reject
                                verdict, mcache.Put and forwarding happen at round g + vdelay; copies
                                arriving meanwhile are pending duplicates (score.go:719-725, 806-809).
                                Needs the topic-major delivery on a single engine (not a shard). */
    uint8_t  _pad[6];
} gsim_msg;

#define GSIM_MAX_VDELAY 7

/* Allocate the message ring and seen-set (after load_graph). */
int gsim_msgs_init(gsim_handle* h, const gsim_msg_config* cfg);
/* Publish `count` messages in round g: each slot is reset, the origin marks
 * the message seen (markSeen, pubsub.go:987-995) and puts it in its mcache
 * (gossipsub.go:976); the origin forwards it in round g+1. */
int gsim_publish(gsim_handle* h, const gsim_msg* msgs, int32_t count, int64_t round);
/* Propagation round g for the whole network:
 *  1. every peer that saw a message for the first time in round g-1 (or
 *     published it then) forwards it to its current mesh except the sender
 *     and the origin (gossipsub.go:975-1045; receivers do not forward an
 *     invalid message);
 *  2. every receiver handles those copies: AcceptFrom graylist
 *     (gossipsub.go:598-609), seen-set check (pubsub.go:1118-1162), then
 *     DeliverMessage / DuplicateMessage / RejectMessage (score.go:693-827);
 *     of several same-round copies the lowest connection is the first;
 *  3. control inbox of round g % rounds (rounds 0 and 1 of a heartbeat). */
int gsim_round(gsim_handle* h, int64_t round);
/* Host synchronisations the library has made in this process (stream
 * synchronisations and blocking copies, every handle and group together):
 * read it around a tick to count the host round trips the tick paid. */
int gsim_host_sync_count(uint64_t* out);
/* n_ticks whole heartbeat ticks in one call (SURVEY.md §8(b) gsim_step; the
 * heartbeat timer loop, gossipsub.go:1320-1343): for tick k = tick ..
 * tick + n_ticks - 1 at now = t0 + k * heartbeat (gsim_msg_config):
 * gsim_refresh_scores, gsim_heartbeat, then the rounds g = k * rounds ..
 * k * rounds + rounds - 1, each with its publications (gsim_publish) and
 * gsim_round.  msgs / round_off: the publications of the call's rounds,
 * msgs[round_off[q] .. round_off[q + 1]) in round q of the call
 * (n_ticks * rounds + 1 offsets, round_off[0] = 0; both NULL: none), uploaded
 * once.  The same results as the calls it stands for; the error flags the
 * heartbeat checks (response-queue overflow, early slot reuse) are read once
 * per call, at its end (a tick after a failing one ran on flagged state).
 * Single engines only (a sharded group steps through gsim_group_*). */
int gsim_step(gsim_handle* h, uint64_t tick, int32_t n_ticks, const gsim_msg* msgs, const int64_t* round_off);
/* Cumulative totals since gsim_msgs_init: out4 = {msg-edge deliveries
 * (accepted arrivals, duplicates included), first deliveries, duplicates,
 * graylisted arrivals}.  Synchronizes.  GSIM_ERANGE if the IWANT response
 * queue overflowed, GSIM_ESTATE if a slot was republished while its message
 * could still be gossiped (results are then incomplete). */
int gsim_msg_stats(gsim_handle* h, int64_t* out4);

/* Per-peer behaviour flags for adversarial configurations:
 * GSIM_BEHAVE_IGNORE_IWANT = the peer advertises (IHAVE) but never answers
 * IWANT (gossipsub_spam_test.go:134-286), so the requesters' promises break
 * and P7 penalties follow (gossip_tracer.go:79-115, gossipsub.go:1620-1625). */
#define GSIM_BEHAVE_IGNORE_IWANT 0x01u
int gsim_set_peer_behaviour(gsim_handle* h, const uint8_t* flags);
/* Cumulative gossip totals: out4 = {(receiver, message) pairs handleIHave
 * examined for an unseen advertised id, IWANT ids sent, messages sent in
 * answer to IWANT, broken promises penalised}. */
int gsim_gossip_stats(gsim_handle* h, int64_t* out4);

/* Aggregate census of the state (the network-wide analogue of the
 * reference's score inspection, score.go:448-500): out8 = {connected scored
 * edge-topic records, of those inMesh, non-zero firstMessageDeliveries,
 * non-zero meshMessageDeliveries, non-zero meshFailurePenalty, non-zero
 * invalidMessageDeliveries, router mesh links, tracked edges}. */
int gsim_census(gsim_handle* h, int64_t* out8);

/* ---- trace export (pb/trace.proto, trace.go) ------ */
/* The events the routers [peer_lo, peer_hi) hand their tracer
 * (pubsubTracer, trace.go:70-530), one record each, in the order of
 * pb/trace.proto's TraceEvent.Type:
 *   PUBLISH_MESSAGE   the origin publishes (trace.go:70-91)
 *   REJECT_MESSAGE    first reception of a message that failed validation
 *                     (reason = the verdict), or every copy with a bad
 *                     signature (105-134)
 *   DUPLICATE_MESSAGE a copy of a message already seen (136-164)
 *   DELIVER_MESSAGE   first reception of an accepted message (166-194)
 *   ADD_PEER / REMOVE_PEER   connections made or lost (196-248)
 *   RECV_RPC / SEND_RPC  the message RPCs (trace.go:250-297): every copy a
 *                     router forwards is its own RPC (Publish -> sendRPC per
 *                     peer, gossipsub.go:1032-1044, 1195-1200), SEND_RPC at
 *                     the sender (other = the receiver) and RECV_RPC at the
 *                     receiver (other = the sender; handleIncomingRPC,
 *                     pubsub.go:1039, before AcceptFrom), reason 0; an
 *                     advertiser's IWANT answers to one requester in a round
 *                     are one RPC (handleIWant, gossipsub.go:700-739): reason
 *                     1, sent the round before they arrive, one record per
 *                     message (gsim_trace_encode joins them); reason 2:
 *                     handleIHave's IWANT request (HandleRPC -> sendRPC,
 *                     gossipsub.go:611-627), SEND_RPC at the requester in
 *                     control round 0 and RECV_RPC at the advertiser in round
 *                     1, one record per requested id (encoded as one
 *                     ControlMeta.iwant; ids in (topic, id) order).
 *                     Modelled difference: the reference's HandleRPC sends the
 *                     IWANT request, the IWANT answers and the PRUNEs of one
 *                     incoming RPC as ONE sendRPC (gossipsub.go:617-627); here
 *                     the request (control round 0) and the answers (round 1)
 *                     happen in different rounds, so they are separate RPCs
 *                     (no reference fixture pins this: parity unpinned).  The
 *                     heartbeat's control / IHAVE RPCs are traced from their
 *                     encoding (gsim_trace_rpc_encode, include/gsim_wire.h)
 *   JOIN / LEAVE      gsim_set_subscriptions (1047-1124)
 *   GRAFT / PRUNE     the router adds / drops a mesh link: heartbeat,
 *                     handleGraft, handlePrune (468-520)
 * Not produced: DROP_RPC (no outbound queue is modelled, so no RPC is
 * dropped: doDropRPC needs a full queue, gossipsub.go:1185-1200).  Copies
 * dropped by AcceptFrom produce no message event, as in pushMsg. */
#define GSIM_TRACE_PUBLISH_MESSAGE   0
#define GSIM_TRACE_REJECT_MESSAGE    1
#define GSIM_TRACE_DUPLICATE_MESSAGE 2
#define GSIM_TRACE_DELIVER_MESSAGE   3
#define GSIM_TRACE_ADD_PEER          4
#define GSIM_TRACE_REMOVE_PEER       5
#define GSIM_TRACE_RECV_RPC          6   /* a message RPC received: reason 0 a forwarded message, 1 an IWANT answer */
#define GSIM_TRACE_SEND_RPC          7   /* a message RPC sent (same reasons)                                     */
#define GSIM_TRACE_JOIN              9
#define GSIM_TRACE_LEAVE             10
#define GSIM_TRACE_GRAFT             11
#define GSIM_TRACE_PRUNE             12

typedef struct gsim_trace_event {
    int64_t  timestamp_ns;    /* TraceEvent.timestamp */
    uint64_t msg_id;          /* gsim_msg.id of message events */
    uint32_t peer;            /* TraceEvent.peerID: the router */
    uint32_t other;           /* receivedFrom (message events); the peer (ADD/REMOVE_PEER, GRAFT, PRUNE) */
    int32_t  topic;           /* message events, GRAFT, PRUNE; -1 otherwise */
    uint8_t  type;            /* GSIM_TRACE_* */
    uint8_t  reason;          /* REJECT_MESSAGE: GSIM_VERDICT_* */
    uint16_t _pad;
} gsim_trace_event;

/* Start tracing the routers [peer_lo, peer_hi) into a device buffer of cap
 * events (0: stop and free it).  A shard of a group: gsim_group_trace_config. */
int gsim_trace_config(gsim_handle* h, uint32_t peer_lo, uint32_t peer_hi, int64_t cap);

/* The events traced since the last call, sorted by (timestamp, peer, type,
 * other, reason, topic, msg_id); *n is their number (GSIM_ERANGE, nothing lost from
 * the buffer, when it exceeds cap; GSIM_ERANGE when the device buffer
 * overflowed). */
int gsim_trace_read(gsim_handle* h, gsim_trace_event* out, int64_t cap, int64_t* n);

/* Copy the score snapshot (E doubles, edge order) to host. */
int gsim_read_scores(gsim_handle* h, double* out);

/* WithPeerScoreInspect's ExtendedPeerScoreInspectFn (score.go:127-180),
 * filled as inspectScoresExtended does (score.go:472-500) for every
 * connection of the observers [obs_lo, obs_hi): peers[x] for the x-th edge of
 * those rows (edge order), topics[x * T + t] its topic t.  Score is the live
 * score(p) (deliveries since the last refresh included); a topic without
 * events reads as a zero record; an untracked edge (no peerStats) has
 * tracked = 0 and zeros. */
typedef struct gsim_topic_score_snapshot {
    int64_t time_in_mesh_ns;            /* meshTime while inMesh, else 0 */
    double  first_message_deliveries;
    double  mesh_message_deliveries;
    double  invalid_message_deliveries;
} gsim_topic_score_snapshot;
typedef struct gsim_peer_score_snapshot {
    double   score;
    double   app_specific_score;
    double   ip_colocation_factor;       /* the P6 value before its weight */
    double   behaviour_penalty;
    uint32_t observer, peer;             /* peer ids (global ids on a shard) */
    int32_t  tracked;
    int32_t  _pad;
} gsim_peer_score_snapshot;
int gsim_read_snapshot(gsim_handle* h, int64_t obs_lo, int64_t obs_hi, gsim_peer_score_snapshot* peers,
                       gsim_topic_score_snapshot* topics);

/* refreshIPs (score.go:568-585): replace every peer's IP list (CSR as for
 * gsim_load_graph); P6 is re-derived before the next score.  The whitelist
 * stays if n_ips is unchanged, else it is cleared.  GSIM_ESTATE once the peer
 * gater is on (its per-IP groups are fixed by gsim_set_peer_gater). */
int gsim_set_ips(gsim_handle* h, const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips);

/* ---- raw state access (tests, checkpoint/resume, golden fixtures) ------- */
typedef enum gsim_field {
    GSIM_F_FIRST = 0,     /* f64 [T][E] firstMessageDeliveries          score.go:49 */
    GSIM_F_MESHD,         /* f64 [T][E] meshMessageDeliveries           score.go:52 */
    GSIM_F_FAIL,          /* f64 [T][E] meshFailurePenalty              score.go:58 */
    GSIM_F_INVALID,       /* f64 [T][E] invalidMessageDeliveries        score.go:61 */
    GSIM_F_GRAFT_TIME,    /* i64 [T][E] graftTime (ns)                  score.go:42 */
    GSIM_F_MESH_TIME,     /* i64 [T][E] meshTime (ns)                   score.go:46 */
    GSIM_F_TFLAGS,        /* u8  [T][E] bit0 inMesh, bit1 meshMessageDeliveriesActive, bit2 mesh, bit3 fanout */
    GSIM_F_BP,            /* f64 [E]    behaviourPenalty                score.go:34 */
    GSIM_F_ESTATE,        /* u8  [E]    bit0 tracked (peerStats exists), bit1 connected */
    GSIM_F_EXPIRE,        /* i64 [E]    retention expiry (ns)           score.go:22 */
    GSIM_F_P6,            /* f64 [E]    ipColocationFactor value        */
    GSIM_F_SCORE,         /* f64 [E]    score snapshot                  */
    GSIM_F_BACKOFF,       /* i64 [T][E] prune backoff expiry, 0 = none gossipsub.go:432 */
    GSIM_F_CTL,           /* u8 [2][T][E] control inbox by round parity (receiver's edge) */
    GSIM_F_SEEN,          /* u32 [ring][N] first-seen round, 0xFFFFFFFF unseen (after msgs_init) */
    GSIM_F_LASTPUT,       /* i32 [T][N] tick of the newest mcache.Put, -1 none (after msgs_init) */
    GSIM_F_LASTPUB,       /* i64 [N][T] gs.lastpub[topic] (ns), 0 = none  gossipsub.go:426 (peer-major) */
    GSIM_F_FANOUT_TOPICS, /* u64 [N]    bit t: gs.fanout[topic t] exists  gossipsub.go:425 */
    GSIM_F__COUNT
} gsim_field;

#define GSIM_TF_IN_MESH   0x01u  /* topicStats.inMesh (score.go:39)               */
#define GSIM_TF_ACTIVE    0x02u  /* topicStats.meshMessageDeliveriesActive         */
#define GSIM_TF_MESH      0x04u  /* router membership: gs.mesh[topic][p] (gossipsub.go:424) */
#define GSIM_TF_FANOUT    0x08u  /* router fanout: gs.fanout[topic][p] (gossipsub.go:425) */
/* control inbox bits (GSIM_F_CTL), one byte per [parity][topic][receiver edge] */
#define GSIM_CTL_GRAFT    0x01u  /* ControlGraft  (pb/rpc.proto) */
#define GSIM_CTL_PRUNE    0x02u  /* ControlPrune with Backoff = PruneBackoff/1s */
#define GSIM_CTL_PX       0x04u  /* the PRUNE carries peer exchange (makePrune doPX, gossipsub.go:1878-1903) */
#define GSIM_CTL_IHAVE    0x08u  /* ControlIHave for this topic */
#define GSIM_CTL_UNSUB    0x10u  /* the PRUNE is Leave's (makePrune isUnsubscribe, gossipsub.go:1104-1124):
                                    Backoff = UnsubscribeBackoff/1s */
#define GSIM_ES_TRACKED   0x01u
#define GSIM_ES_CONNECTED 0x02u

/* Size in bytes of a field for the loaded graph. */
int gsim_field_bytes(gsim_handle* h, int32_t field, size_t* out);
int gsim_read_field(gsim_handle* h, int32_t field, void* dst, size_t bytes);
int gsim_write_field(gsim_handle* h, int32_t field, const void* src, size_t bytes);

/* ---- device timing on the engine's own stream (bench/profiling) -------- */
/* Record HIP event `slot` (0..511) on the engine stream. */
int gsim_event_record(gsim_handle* h, int32_t slot);
/* Milliseconds between two recorded events (synchronizes on `to`). */
int gsim_event_elapsed(gsim_handle* h, int32_t from, int32_t to, float* ms);
int gsim_synchronize(gsim_handle* h);
/* Per-kernel-class device time, measured with HIP events recorded on the
 * engine stream around each class's launches while profiling is enabled. */
typedef enum gsim_kernel_class {
    GSIM_K_REFRESH_SCORE = 0,  /* refreshScores (+ fused score) pass */
    GSIM_K_SCORE,              /* score-only pass */
    GSIM_K_IP_COLOCATION,      /* P6 segmented count */
    GSIM_K_HEARTBEAT,          /* mesh maintenance */
    GSIM_K_CONTROL,            /* GRAFT/PRUNE handling */
    GSIM_K_PUBLISH,            /* slot reset + origin self-delivery */
    GSIM_K_SEND,               /* mesh forwarding: AcceptFrom, seen-set claims, duplicate/invalid counters */
    GSIM_K_COMMIT,             /* seen commit + first-delivery credit */
    GSIM_K_ACCEPT,             /* AcceptFrom verdicts from a new score snapshot */
    GSIM_K_GOSSIP,             /* handleIHave/handleIWant + IWANT response delivery */
    GSIM_K_CHURN,              /* AddPeer/RemovePeer of gsim_set_connections */
    GSIM_K__COUNT
} gsim_kernel_class;
/* Enable (1) or disable (0) recording; clears recorded totals. */
int gsim_profile(gsim_handle* h, int32_t enable);
/* Synchronize, then write per-class milliseconds and launch counts recorded
 * since the last read (n entries, indexed by gsim_kernel_class) and reset. */
int gsim_profile_read(gsim_handle* h, double* ms, int64_t* launches, int32_t n);
/* Select an implementation variant of a hot-path kernel for A/B timing in
 * one process.  Results are identical across variants (the GPU tests run
 * each).  which = 2: the delivery kernel; 3 (topic-major k_send_tm) is the
 * only one.  which = 3: the IHAVE walk's lane
 * group width (8, 16, 32 or 64 lanes per row; 0 = chosen from the row lengths).
 * which = 6: the topic-major kernel's blocks: 0 (default) shared out among
 * the topics by their subscribers, 1 the same number for every topic, >= 64
 * shared out by subscribers, this many in all. */
int gsim_set_kernel_variant(gsim_handle* h, int32_t which, int32_t variant);

/* ---- synthetic inputs -------------------------------- */
/* Random k-regular simple graph on n vertices (configuration model, bad
 * pairs repaired by random double-edge swaps), seeded.  row_ptr (n+1) and
 * col_idx (n*k) are caller-allocated; rows come out sorted.  outbound
 * (n*k, may be NULL) gets a Bernoulli(0.5) initiator per undirected edge. */
int gsim_gen_random_regular(int64_t n, int32_t k, uint64_t seed,
                            uint32_t* row_ptr, uint32_t* col_idx, uint8_t* outbound);
/* Chung-Lu power law (C5 inputs): expected degree of peer i proportional to
 * (i + i0)^(-1/(exponent-1)) scaled to `mean`, capped at max_degree; pairs
 * drawn by inverse CDF, self loops and repeats dropped, then accepted in
 * drawing order while both ends are below the cap.  Call with col_idx NULL
 * for the directed edge count (*n_edges), then with row_ptr (n+1), col_idx
 * and outbound (may be NULL) sized to it; rows come out sorted. */
int gsim_gen_power_law(int64_t n, double mean, double exponent, int32_t max_degree, double i0, uint64_t seed,
                       uint32_t* row_ptr, uint32_t* col_idx, uint8_t* outbound, int64_t* n_edges);
/* Fill every edge-topic record with seeded steady-state-like counters on the
 * device (mesh membership with probability p_mesh, graft times within the
 * last hour of now_ns); every edge tracked+connected.  Records of topics the
 * two endpoints do not both announce stay empty.  For benchmarking at sizes
 * where a host upload would dominate. */
int gsim_fill_synthetic(gsim_handle* h, uint64_t seed, int64_t now_ns, double p_mesh);

/* ---- graph sharding across GPUs -------- */
/* The reference simulates nothing across processes: one GossipSubRouter per
 * host, RPCs over libp2p streams (gossipsub.go:1138-1202 sendRPC).  Here one
 * network is split into contiguous peer ranges, one per shard (GPU); a shard
 * holds its peers' rows in full plus a "ghost" row per remote neighbour (that
 * neighbour's connections into the shard), so every record an owned observer
 * keeps is local.  Copies are pulled: each round every shard sends the
 * others its forwarders of the round (peer, first sender, slot), and a shard
 * walks the ghost rows of the remote forwarders itself, so each copy is
 * delivered by the receiver's shard.  GRAFT/PRUNE records, the router state
 * of cross edges (mesh / fanout bits, connected, direct, publish gate) and
 * gossip marks move the same way.  At most 2^24 - 2 peers per network. */
#define GSIM_MAX_SHARDS 64

/* Contiguous peer ranges for `shards` shards balanced by the sum of (row
 * length x joined topics): bounds[0] = 0 < bounds[1] < ... < bounds[shards]
 * = n, interior bounds multiples of 64.  sub may be NULL (one topic each). */
int gsim_shard_partition(int64_t n, const uint32_t* row_ptr, const uint64_t* sub, int32_t shards,
                         int64_t* bounds);

typedef struct gsim_shard_info {
    int32_t shard, shards;
    int64_t n_local, e_local;   /* local peers (owned + ghosts) and edges (owned rows + ghost rows) */
    int64_t own_lo, own_hi;     /* owned peers: local ids [own_lo, own_hi) = global [bounds[s], bounds[s+1]) */
    int64_t own_e_lo, own_e_hi; /* local edges of the owned rows */
    int64_t n_cross;            /* owned-row edges whose column belongs to another shard */
} gsim_shard_info;
int gsim_shard_layout_info(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds,
                           int32_t shards, int32_t shard, gsim_shard_info* out);
/* The local graph of one shard (sizes from gsim_shard_layout_info; any output
 * may be NULL): gid[n_local] global id of each local peer (ascending);
 * row_ptr_l/col_l the local CSR; gidx[e_local] the global index of each local
 * edge; per other shard s, ghost_base[s]/ghost_count[s] the local edges of the
 * ghost rows of s's peers, and cross_count[s] owned-row edges into s, listed
 * in edge order one shard after the other in cross_out (n_cross entries).
 * Two shards enumerate their common cross edges in the same order:
 * cross_out of a into b, position q, is the edge ghost_base[a] + q of b. */
int gsim_shard_layout(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds,
                      int32_t shards, int32_t shard, uint32_t* gid, uint32_t* row_ptr_l, uint32_t* col_l,
                      uint64_t* gidx, int64_t* ghost_base, int64_t* ghost_count, uint32_t* cross_out,
                      int64_t* cross_count);

/* A sharded network: a group of shards, each an engine handle over its
 * local graph.  gsim_group_create puts every shard in this process (shard s
 * on devices[s]; devices NULL: all on device 0), exchanging with device
 * copies.  gsim_group_create_rccl is one shard of a multi-process job (one
 * process per GPU): `unique_id` comes from gsim_rccl_unique_id on rank 0,
 * shared by the caller (128 bytes), and the exchanges run over RCCL. */
typedef struct gsim_group gsim_group;
int gsim_rccl_unique_id(void* out, size_t bytes);
int gsim_group_create(const gsim_peer_score_params* params, const gsim_topic_score_params* topics, int32_t n_topics,
                      const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip, int32_t shards,
                      const int32_t* devices, gsim_group** out, char* err, size_t errlen);
int gsim_group_create_rccl(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                           int32_t n_topics, const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip,
                           int32_t shards, int32_t rank, int32_t device, const void* unique_id, gsim_group** out,
                           char* err, size_t errlen);
/* One shard of a multi-process job whose exchanges go through the caller's
 * own collectives over host memory (device -> pinned host -> callback ->
 * device): the one-shard-per-process code path of gsim_group_create_rccl
 * without RCCL (tests on one GPU with gloo; hosts without xGMI).  Callbacks
 * return 0 on success and are called by every rank in the same order.
 *   alltoallv: send[sdisp[d] .. + sbytes[d]) to rank d; recv[rdisp[s] .. +
 *              rbytes[s]) from rank s (sizes agreed beforehand; the rank's own
 *              entries are 0);
 *   allreduce: elementwise over `count` values of every rank, in place;
 *              dtype 0 = u32, 1 = i32, 2 = u64; op 0 = sum, 1 = max. */
typedef struct gsim_host_transport {
    void* ctx;
    int (*alltoallv)(void* ctx, const uint8_t* send, const uint64_t* sbytes, const uint64_t* sdisp, uint8_t* recv,
                     const uint64_t* rbytes, const uint64_t* rdisp);
    int (*allreduce)(void* ctx, void* buf, int64_t count, int32_t dtype, int32_t op);
} gsim_host_transport;
int gsim_group_create_host(const gsim_peer_score_params* params, const gsim_topic_score_params* topics,
                           int32_t n_topics, const gsim_thresholds* thresholds, const gsim_gossipsub_params* gossip,
                           int32_t shards, int32_t rank, int32_t device, const gsim_host_transport* transport,
                           gsim_group** out, char* err, size_t errlen);
int gsim_group_destroy(gsim_group* g);
const char* gsim_group_last_error(const gsim_group* g);
/* The handle of a shard hosted by this process (NULL otherwise): its state is
 * read and written through the gsim_*_field calls in the local view (owned
 * rows are edges [own_e_lo, own_e_hi) of gsim_shard_layout_info). */
gsim_handle* gsim_group_shard(gsim_group* g, int32_t shard);
int gsim_group_bounds(const gsim_group* g, int64_t* bounds);
/* The whole network's CSR and inputs, as for gsim_load_graph (every process
 * passes the same); bounds NULL: gsim_shard_partition. */
int gsim_group_load_graph(gsim_group* g, int64_t n_peers, const uint32_t* row_ptr, const uint32_t* col_idx,
                          const uint8_t* outbound, const uint64_t* subscriptions, const uint32_t* ip_ptr,
                          const uint32_t* ip_ids, uint32_t n_ips, const int64_t* bounds);
/* The single-handle calls over the whole network (global peer / edge
 * indexing; the per-round halo exchange happens inside). */
int gsim_group_set_app_score(gsim_group* g, const double* p5);
int gsim_group_set_ip_whitelist(gsim_group* g, const uint8_t* whitelisted);
int gsim_group_set_direct_peers(gsim_group* g, const uint8_t* flags);
int gsim_group_set_peer_behaviour(gsim_group* g, const uint8_t* flags);
int gsim_group_set_topic_params(gsim_group* g, int32_t topic, const gsim_topic_score_params* p);
int gsim_group_set_seed(gsim_group* g, uint64_t seed);
int gsim_group_fill_synthetic(gsim_group* g, uint64_t seed, int64_t now_ns, double p_mesh);
/* max_frontier > 0: the initial size of the per-shard forwarder lists
 * (default max(8 x owned peers, 65536) entries; they grow when a round needs
 * more). */
int gsim_group_msgs_init(gsim_group* g, const gsim_msg_config* cfg);
int gsim_group_refresh_scores(gsim_group* g, int64_t now_ns);
int gsim_group_heartbeat(gsim_group* g, uint64_t tick, int64_t now_ns);
int gsim_group_publish(gsim_group* g, const gsim_msg* msgs, int32_t count, int64_t round);
int gsim_group_round(gsim_group* g, int64_t round);
int gsim_group_set_connections(gsim_group* g, const uint32_t* pairs, int32_t count, int32_t up, int64_t now_ns);
/* gsim_px_connect over the shards (every rank calls it between ticks): PX
 * lists PRUNEs carried to other shards' peers are checked there
 * (acceptPXThreshold on the pruned peer's score, a known address, not
 * connected), every attempt is resolved once (the asker dials, the lower id
 * when both asked) and connected at both ends; pairs: the (dialer, peer)
 * global ids, sorted.  The same connections as one engine's gsim_px_connect. */
int gsim_group_px_connect(gsim_group* g, int64_t now_ns, uint32_t* pairs, int64_t cap, int64_t* n_connected);
/* gsim_set_subscriptions over the shards (global peer ids; every rank passes
 * the same list): the same Joins / Leaves as one engine. */
int gsim_group_set_subscriptions(gsim_group* g, const uint32_t* pairs, int32_t count, int32_t join, uint64_t tick,
                                 int64_t now_ns);
int gsim_group_set_ips(gsim_group* g, const uint32_t* ip_ptr, const uint32_t* ip_ids, uint32_t n_ips);
/* Router state (mesh / fanout flags, connection state, direct flags) was
 * written through gsim_write_field on a shard handle: the ghost rows are
 * refreshed from their owners before the next round. */
int gsim_group_state_written(gsim_group* g);
/* Totals of the whole job (summed over every shard, every process). */
int gsim_group_msg_stats(gsim_group* g, int64_t* out4);
int gsim_group_gossip_stats(gsim_group* g, int64_t* out4);
int gsim_group_census(gsim_group* g, int64_t* out8);
int gsim_group_synchronize(gsim_group* g);
/* WithPeerScoreInspect over a sharded network (score.go:152-180, 448-500):
 * the whole network's view, filled from the rows this process's shards own
 * (every shard with gsim_group_create; one rank's range with the RCCL / host
 * transports, the rest of dst left as it was).
 * gsim_group_field_bytes: the size of a field for the whole network (N peers,
 *   E edges; gsim_field_bytes's shapes).
 * gsim_group_read_field: gsim_read_field in global peer / edge order.
 * gsim_group_read_scores: the score snapshot, E doubles in global edge order.
 * gsim_group_read_snapshot: gsim_read_snapshot for the global observers
 *   [obs_lo, obs_hi): peers[x] for the x-th edge of those rows (global edge
 *   order from row_ptr[obs_lo]), topics[x * T + t]; observer and peer are
 *   global ids. */
int gsim_group_field_bytes(gsim_group* g, int32_t field, size_t* out);
int gsim_group_read_field(gsim_group* g, int32_t field, void* dst, size_t bytes);
int gsim_group_read_scores(gsim_group* g, double* out);
int gsim_group_read_snapshot(gsim_group* g, int64_t obs_lo, int64_t obs_hi, gsim_peer_score_snapshot* peers,
                             gsim_topic_score_snapshot* topics);
/* WithPeerGater over a sharded network (peer_gater.go:161-186): every
 * shard's routers; gsim_group_gater_throttled sums the drops over the job,
 * gsim_group_gater_read is gsim_gater_read in global peer / edge order (the
 * parts this process's shards own). */
int gsim_group_set_peer_gater(gsim_group* g, const gsim_peer_gater_params* p, const double* topic_weights);
int gsim_group_gater_throttled(gsim_group* g, int64_t* out);
int gsim_group_gater_read(gsim_group* g, double* validate, double* throttle, int64_t* last, double* counters4,
                          int32_t* connected, int64_t* expire);
/* gsim_trace_config / gsim_trace_read over a sharded network: the routers
 * [peer_lo, peer_hi) (global ids) that this process's shards own, every
 * event in global ids, sorted as gsim_trace_read sorts.  Needs the copy push
 * exchange (the default). */
int gsim_group_trace_config(gsim_group* g, uint32_t peer_lo, uint32_t peer_hi, int64_t cap);
int gsim_group_trace_read(gsim_group* g, gsim_trace_event* out, int64_t cap, int64_t* n);
/* Per-kernel-class time of this process's shards (summed). */
int gsim_group_profile(gsim_group* g, int32_t enable);
int gsim_group_profile_read(gsim_group* g, double* ms, int64_t* launches, int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* GSIM_H */
