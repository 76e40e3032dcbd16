// params.cpp — parameter defaults and validation behind the C ABI.
//
// Restates score_params.go:37-64 (PeerScoreThresholds.validate),
// score_params.go:173-398 (PeerScoreParams/TopicScoreParams.validate),
// score_params.go:405-417 (ScoreParameterDecay*), gossipsub.go:244-275
// (DefaultGossipSubParams).  Error texts keep the reference's wording so the
// Go shim can surface them unchanged.
#include "gsim.h"

#include <cmath>
#include <cstdio>
#include <cstring>

namespace {

constexpr int64_t kSecond = 1000000000LL;
constexpr int64_t kMilli = 1000000LL;

bool invalid_number(double x) { return std::isnan(x) || std::isinf(x); }

int fail(char* err, size_t errlen, const char* msg)
{
    if (err && errlen) std::snprintf(err, errlen, "%s", msg);
    return GSIM_EINVAL;
}

// score_params.go:269-294
int validate_time_in_mesh(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (p->skip_atomic_validation && p->time_in_mesh_weight == 0 &&
        p->time_in_mesh_quantum_ns == 0 && p->time_in_mesh_cap == 0)
        return GSIM_OK;
    if (p->time_in_mesh_quantum_ns == 0) return fail(err, n, "invalid TimeInMeshQuantum; must be non zero");
    if (p->time_in_mesh_weight < 0 || invalid_number(p->time_in_mesh_weight))
        return fail(err, n, "invalid TimeInMeshWeight; must be positive (or 0 to disable) and a valid number");
    if (p->time_in_mesh_weight != 0 && p->time_in_mesh_quantum_ns <= 0)
        return fail(err, n, "invalid TimeInMeshQuantum; must be positive");
    if (p->time_in_mesh_weight != 0 && (p->time_in_mesh_cap <= 0 || invalid_number(p->time_in_mesh_cap)))
        return fail(err, n, "invalid TimeInMeshCap; must be positive and a valid number");
    return GSIM_OK;
}

// score_params.go:296-318
int validate_first_deliveries(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (p->skip_atomic_validation && p->first_message_deliveries_weight == 0 &&
        p->first_message_deliveries_cap == 0 && p->first_message_deliveries_decay == 0)
        return GSIM_OK;
    if (p->first_message_deliveries_weight < 0 || invalid_number(p->first_message_deliveries_weight))
        return fail(err, n, "invallid FirstMessageDeliveriesWeight; must be positive (or 0 to disable) and a valid number");
    if (p->first_message_deliveries_weight != 0 &&
        (p->first_message_deliveries_decay <= 0 || p->first_message_deliveries_decay >= 1 ||
         invalid_number(p->first_message_deliveries_decay)))
        return fail(err, n, "invalid FirstMessageDeliveriesDecay; must be between 0 and 1");
    if (p->first_message_deliveries_weight != 0 &&
        (p->first_message_deliveries_cap <= 0 || invalid_number(p->first_message_deliveries_cap)))
        return fail(err, n, "invalid FirstMessageDeliveriesCap; must be positive and a valid number");
    return GSIM_OK;
}

// score_params.go:320-356
int validate_mesh_deliveries(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (p->skip_atomic_validation && p->mesh_message_deliveries_weight == 0 &&
        p->mesh_message_deliveries_cap == 0 && p->mesh_message_deliveries_decay == 0 &&
        p->mesh_message_deliveries_threshold == 0 && p->mesh_message_deliveries_window_ns == 0 &&
        p->mesh_message_deliveries_activation_ns == 0)
        return GSIM_OK;
    const double w = p->mesh_message_deliveries_weight;
    if (w > 0 || invalid_number(w))
        return fail(err, n, "invalid MeshMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
    if (w != 0 && (p->mesh_message_deliveries_decay <= 0 || p->mesh_message_deliveries_decay >= 1 ||
                   invalid_number(p->mesh_message_deliveries_decay)))
        return fail(err, n, "invalid MeshMessageDeliveriesDecay; must be between 0 and 1");
    if (w != 0 && (p->mesh_message_deliveries_cap <= 0 || invalid_number(p->mesh_message_deliveries_cap)))
        return fail(err, n, "invalid MeshMessageDeliveriesCap; must be positive and a valid number");
    if (w != 0 && (p->mesh_message_deliveries_threshold <= 0 ||
                   invalid_number(p->mesh_message_deliveries_threshold)))
        return fail(err, n, "invalid MeshMessageDeliveriesThreshold; must be positive and a valid number");
    if (p->mesh_message_deliveries_window_ns < 0)
        return fail(err, n, "invalid MeshMessageDeliveriesWindow; must be non-negative");
    if (w != 0 && p->mesh_message_deliveries_activation_ns < kSecond)
        return fail(err, n, "invalid MeshMessageDeliveriesActivation; must be at least 1s");
    return GSIM_OK;
}

// score_params.go:358-377
int validate_failure_penalty(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (p->skip_atomic_validation && p->mesh_failure_penalty_decay == 0 && p->mesh_failure_penalty_weight == 0)
        return GSIM_OK;
    if (p->mesh_failure_penalty_weight > 0 || invalid_number(p->mesh_failure_penalty_weight))
        return fail(err, n, "invalid MeshFailurePenaltyWeight; must be negative (or 0 to disable) and a valid number");
    if (p->mesh_failure_penalty_weight != 0 &&
        (invalid_number(p->mesh_failure_penalty_decay) || p->mesh_failure_penalty_decay <= 0 ||
         p->mesh_failure_penalty_decay >= 1))
        return fail(err, n, "invalid MeshFailurePenaltyDecay; must be between 0 and 1");
    return GSIM_OK;
}

// score_params.go:379-398
int validate_invalid_deliveries(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (p->skip_atomic_validation && p->invalid_message_deliveries_decay == 0 &&
        p->invalid_message_deliveries_weight == 0)
        return GSIM_OK;
    if (p->invalid_message_deliveries_weight > 0 || invalid_number(p->invalid_message_deliveries_weight))
        return fail(err, n, "invalid InvalidMessageDeliveriesWeight; must be negative (or 0 to disable) and a valid number");
    if (p->invalid_message_deliveries_decay <= 0 || p->invalid_message_deliveries_decay >= 1 ||
        invalid_number(p->invalid_message_deliveries_decay))
        return fail(err, n, "invalid InvalidMessageDeliveriesDecay; must be between 0 and 1");
    return GSIM_OK;
}

}  // namespace

extern "C" {

void gsim_default_gossipsub_params(gsim_gossipsub_params* o)
{
    std::memset(o, 0, sizeof(*o));
    o->d = 6;
    o->dlo = 5;
    o->dhi = 12;
    o->dscore = 4;
    o->dout = 2;
    o->history_length = 5;
    o->history_gossip = 3;
    o->dlazy = 6;
    o->gossip_factor = 0.25;
    o->gossip_retransmission = 3;
    o->heartbeat_initial_delay_ns = 100 * kMilli;
    o->heartbeat_interval_ns = kSecond;
    o->fanout_ttl_ns = 60 * kSecond;
    o->prune_peers = 16;
    o->prune_backoff_ns = 60 * kSecond;
    o->unsubscribe_backoff_ns = 10 * kSecond;
    o->connectors = 8;
    o->max_pending_connections = 128;
    o->connection_timeout_ns = 30 * kSecond;
    o->direct_connect_ticks = 300;
    o->direct_connect_initial_delay_ns = kSecond;
    o->opportunistic_graft_ticks = 60;
    o->opportunistic_graft_peers = 2;
    o->graft_flood_threshold_ns = 10 * kSecond;
    o->max_ihave_length = 5000;
    o->max_ihave_messages = 10;
    o->iwant_followup_time_ns = 3 * kSecond;
    o->slow_heartbeat_warning = 0.1;
}

// score_params.go:236-267
int gsim_validate_topic_params(const gsim_topic_score_params* p, char* err, size_t n)
{
    if (!p) return fail(err, n, "nil topic score params");
    if (p->topic_weight < 0 || invalid_number(p->topic_weight))
        return fail(err, n, "invalid topic weight; must be >= 0 and a valid number");
    int rc;
    if ((rc = validate_time_in_mesh(p, err, n))) return rc;
    if ((rc = validate_first_deliveries(p, err, n))) return rc;
    if ((rc = validate_mesh_deliveries(p, err, n))) return rc;
    if ((rc = validate_failure_penalty(p, err, n))) return rc;
    if ((rc = validate_invalid_deliveries(p, err, n))) return rc;
    return GSIM_OK;
}

// score_params.go:173-234
int gsim_validate_peer_params(const gsim_peer_score_params* p, const gsim_topic_score_params* topics,
                              int32_t n_topics, char* err, size_t n)
{
    if (!p) return fail(err, n, "nil peer score params");
    for (int32_t t = 0; t < n_topics; ++t) {
        if (!topics[t].scored) continue;
        char inner[256] = {0};
        if (gsim_validate_topic_params(&topics[t], inner, sizeof inner)) {
            if (err && n) std::snprintf(err, n, "invalid score parameters for topic %d: %s", t, inner);
            return GSIM_EINVAL;
        }
    }
    const bool skip = p->skip_atomic_validation != 0;
    if (!skip || p->topic_score_cap != 0) {
        if (p->topic_score_cap < 0 || invalid_number(p->topic_score_cap))
            return fail(err, n, "invalid topic score cap; must be positive (or 0 for no cap) and a valid number");
    }
    // AppSpecificScore == nil is an error unless skipping (then it scores 0).
    if (!p->has_app_specific_score && !skip) return fail(err, n, "missing application specific score function");
    if (!skip || p->ip_colocation_factor_weight != 0) {
        if (p->ip_colocation_factor_weight > 0 || invalid_number(p->ip_colocation_factor_weight))
            return fail(err, n, "invalid IPColocationFactorWeight; must be negative (or 0 to disable) and a valid number");
        if (p->ip_colocation_factor_weight != 0 && p->ip_colocation_factor_threshold < 1)
            return fail(err, n, "invalid IPColocationFactorThreshold; must be at least 1");
    }
    if (!skip || p->behaviour_penalty_weight != 0 || p->behaviour_penalty_threshold != 0) {
        if (p->behaviour_penalty_weight > 0 || invalid_number(p->behaviour_penalty_weight))
            return fail(err, n, "invalid BehaviourPenaltyWeight; must be negative (or 0 to disable) and a valid number");
        if (p->behaviour_penalty_weight != 0 &&
            (p->behaviour_penalty_decay <= 0 || p->behaviour_penalty_decay >= 1 ||
             invalid_number(p->behaviour_penalty_decay)))
            return fail(err, n, "invalid BehaviourPenaltyDecay; must be between 0 and 1");
        if (p->behaviour_penalty_threshold < 0 || invalid_number(p->behaviour_penalty_threshold))
            return fail(err, n, "invalid BehaviourPenaltyThreshold; must be >= 0 and a valid number");
    }
    if (!skip || p->decay_interval_ns != 0 || p->decay_to_zero != 0) {
        if (p->decay_interval_ns < kSecond) return fail(err, n, "invalid DecayInterval; must be at least 1s");
        if (p->decay_to_zero <= 0 || p->decay_to_zero >= 1 || invalid_number(p->decay_to_zero))
            return fail(err, n, "invalid DecayToZero; must be between 0 and 1");
    }
    return GSIM_OK;
}

// score_params.go:37-64
int gsim_validate_thresholds(const gsim_thresholds* p, char* err, size_t n)
{
    if (!p) return fail(err, n, "nil thresholds");
    const bool skip = p->skip_atomic_validation != 0;
    if (!skip || p->publish_threshold != 0 || p->gossip_threshold != 0 || p->graylist_threshold != 0) {
        if (p->gossip_threshold > 0 || invalid_number(p->gossip_threshold))
            return fail(err, n, "invalid gossip threshold; it must be <= 0 and a valid number");
        if (p->publish_threshold > 0 || p->publish_threshold > p->gossip_threshold ||
            invalid_number(p->publish_threshold))
            return fail(err, n, "invalid publish threshold; it must be <= 0 and <= gossip threshold and a valid number");
        if (p->graylist_threshold > 0 || p->graylist_threshold > p->publish_threshold ||
            invalid_number(p->graylist_threshold))
            return fail(err, n, "invalid graylist threshold; it must be <= 0 and <= publish threshold and a valid number");
    }
    if (!skip || p->accept_px_threshold != 0) {
        if (p->accept_px_threshold < 0 || invalid_number(p->accept_px_threshold))
            return fail(err, n, "invalid accept PX threshold; it must be >= 0 and a valid number");
    }
    if (!skip || p->opportunistic_graft_threshold != 0) {
        if (p->opportunistic_graft_threshold < 0 || invalid_number(p->opportunistic_graft_threshold))
            return fail(err, n, "invalid opportunistic grafting threshold; it must be >= 0 and a valid number");
    }
    return GSIM_OK;
}

// score_params.go:412-417: ticks = float64(decay / base) (integer Duration
// division first), factor = decayToZero^(1/ticks).
double gsim_score_parameter_decay_with_base(int64_t decay_ns, int64_t base_ns, double decay_to_zero)
{
    double ticks = (double)(decay_ns / base_ns);
    return std::pow(decay_to_zero, 1.0 / ticks);
}

// score_params.go:407-409 (DefaultDecayInterval = 1s, DefaultDecayToZero = 0.01)
double gsim_score_parameter_decay(int64_t decay_ns)
{
    return gsim_score_parameter_decay_with_base(decay_ns, kSecond, 0.01);
}

}  // extern "C"
