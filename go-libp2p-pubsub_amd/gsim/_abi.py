"""ctypes mirror of include/gsim.h (the engine's C ABI).

The structures below are field-for-field copies of the C structs, which are
themselves field-for-field copies of the Go structs in score_params.go and
gossipsub.go.  Loading fails loudly: there is no CPU fallback for the engine.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int32, c_int64, c_size_t,
                    c_uint8, c_uint32, c_uint64, c_void_p)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libgsim.so")

GSIM_OK = 0
GSIM_EINVAL = -22
GSIM_ENOMEM = -12
GSIM_EDEVICE = -5
GSIM_ERANGE = -34
GSIM_ESTATE = -71

(F_FIRST, F_MESHD, F_FAIL, F_INVALID, F_GRAFT_TIME, F_MESH_TIME, F_TFLAGS, F_BP, F_ESTATE,
 F_EXPIRE, F_P6, F_SCORE, F_BACKOFF, F_CTL, F_SEEN, F_LASTPUT, F_LASTPUB, F_FANOUT_TOPICS) = range(18)

TF_IN_MESH = 0x01
TF_ACTIVE = 0x02
TF_MESH = 0x04
TF_FANOUT = 0x08
CTL_GRAFT = 0x01
CTL_PRUNE = 0x02
CTL_PX = 0x04
CTL_UNSUB = 0x10
CTL_IHAVE = 0x08
ES_TRACKED = 0x01
ES_CONNECTED = 0x02


class CTopicScoreParams(Structure):
    _fields_ = [
        ("skip_atomic_validation", c_int32), ("scored", c_int32), ("topic_weight", c_double),
        ("time_in_mesh_weight", c_double), ("time_in_mesh_quantum_ns", c_int64), ("time_in_mesh_cap", c_double),
        ("first_message_deliveries_weight", c_double), ("first_message_deliveries_decay", c_double),
        ("first_message_deliveries_cap", c_double),
        ("mesh_message_deliveries_weight", c_double), ("mesh_message_deliveries_decay", c_double),
        ("mesh_message_deliveries_cap", c_double), ("mesh_message_deliveries_threshold", c_double),
        ("mesh_message_deliveries_window_ns", c_int64), ("mesh_message_deliveries_activation_ns", c_int64),
        ("mesh_failure_penalty_weight", c_double), ("mesh_failure_penalty_decay", c_double),
        ("invalid_message_deliveries_weight", c_double), ("invalid_message_deliveries_decay", c_double),
    ]


class CPeerScoreParams(Structure):
    _fields_ = [
        ("skip_atomic_validation", c_int32), ("has_app_specific_score", c_int32),
        ("topic_score_cap", c_double), ("app_specific_weight", c_double),
        ("ip_colocation_factor_weight", c_double), ("ip_colocation_factor_threshold", c_int32), ("_pad0", c_int32),
        ("behaviour_penalty_weight", c_double), ("behaviour_penalty_threshold", c_double),
        ("behaviour_penalty_decay", c_double),
        ("decay_interval_ns", c_int64), ("decay_to_zero", c_double), ("retain_score_ns", c_int64),
        ("seen_msg_ttl_ns", c_int64),
    ]


class CThresholds(Structure):
    _fields_ = [
        ("skip_atomic_validation", c_int32), ("_pad0", c_int32),
        ("gossip_threshold", c_double), ("publish_threshold", c_double), ("graylist_threshold", c_double),
        ("accept_px_threshold", c_double), ("opportunistic_graft_threshold", c_double),
    ]


class CGossipSubParams(Structure):
    _fields_ = [
        ("d", c_int32), ("dlo", c_int32), ("dhi", c_int32), ("dscore", c_int32), ("dout", c_int32),
        ("history_length", c_int32), ("history_gossip", c_int32), ("dlazy", c_int32),
        ("gossip_factor", c_double), ("gossip_retransmission", c_int32), ("prune_peers", c_int32),
        ("heartbeat_initial_delay_ns", c_int64), ("heartbeat_interval_ns", c_int64),
        ("slow_heartbeat_warning", c_double), ("fanout_ttl_ns", c_int64), ("prune_backoff_ns", c_int64),
        ("unsubscribe_backoff_ns", c_int64), ("connectors", c_int32), ("max_pending_connections", c_int32),
        ("connection_timeout_ns", c_int64), ("direct_connect_ticks", c_uint64),
        ("direct_connect_initial_delay_ns", c_int64), ("opportunistic_graft_ticks", c_uint64),
        ("opportunistic_graft_peers", c_int32), ("max_ihave_length", c_int32),
        ("graft_flood_threshold_ns", c_int64), ("max_ihave_messages", c_int32), ("flood_publish", c_int32),
        ("iwant_followup_time_ns", c_int64), ("do_px", c_int32), ("_pad_px", c_int32),
    ]


class CPeerGaterParams(Structure):
    _fields_ = [
        ("threshold", c_double), ("global_decay", c_double), ("source_decay", c_double),
        ("decay_interval_ns", c_int64), ("decay_to_zero", c_double), ("retain_stats_ns", c_int64),
        ("quiet_ns", c_int64), ("duplicate_weight", c_double), ("ignore_weight", c_double),
        ("reject_weight", c_double),
    ]


# gsim_trace_event (include/gsim.h): TraceEvent.Type values
TRACE_PUBLISH_MESSAGE, TRACE_REJECT_MESSAGE, TRACE_DUPLICATE_MESSAGE, TRACE_DELIVER_MESSAGE = 0, 1, 2, 3
TRACE_ADD_PEER, TRACE_REMOVE_PEER, TRACE_GRAFT, TRACE_PRUNE = 4, 5, 11, 12
TRACE_JOIN, TRACE_LEAVE = 9, 10
TRACE_RECV_RPC, TRACE_SEND_RPC = 6, 7          # reason 0: a forwarded message, 1: an IWANT answer


# (name, restype, argtypes) for every symbol include/gsim.h declares.
class CMsgConfig(Structure):
    _fields_ = [("ring", c_int32), ("rounds", c_int32), ("t0_ns", c_int64), ("heartbeat_ns", c_int64),
                ("max_frontier", c_int64), ("max_arrivals", c_int64), ("topic_slots", c_int64)]


class CMsg(Structure):
    _fields_ = [("id", c_uint64), ("topic", c_uint32), ("origin", c_uint32), ("verdict", ctypes.c_uint8),
                ("vdelay", ctypes.c_uint8), ("_pad", ctypes.c_uint8 * 6)]


# numpy view of gsim_msg (24 bytes)
MSG_DTYPE = [("id", "<u8"), ("topic", "<u4"), ("origin", "<u4"), ("verdict", "u1"), ("vdelay", "u1"),
             ("_pad", "u1", (6,))]
MAX_VDELAY = 7          # gsim.h GSIM_MAX_VDELAY
# gsim.h GSIM_VERDICT_*: the validation verdict of a message at every receiver
VERDICT_ACCEPT, VERDICT_REJECT, VERDICT_IGNORE, VERDICT_THROTTLE, VERDICT_SIGNATURE = 0, 1, 2, 3, 4

UNSEEN = 0xFFFFFFFF

# numpy views of gsim_peer_score_snapshot (48 bytes) / gsim_topic_score_snapshot (32 bytes)
PEER_SNAPSHOT_DTYPE = [("score", "<f8"), ("app_specific_score", "<f8"), ("ip_colocation_factor", "<f8"),
                       ("behaviour_penalty", "<f8"), ("observer", "<u4"), ("peer", "<u4"), ("tracked", "<i4"),
                       ("_pad", "<i4")]
TOPIC_SNAPSHOT_DTYPE = [("time_in_mesh_ns", "<i8"), ("first_message_deliveries", "<f8"),
                        ("mesh_message_deliveries", "<f8"), ("invalid_message_deliveries", "<f8")]

KERNEL_CLASSES = ["refresh_score", "score", "ip_colocation", "heartbeat", "control", "publish", "send",
                  "commit", "accept", "gossip", "churn"]
BEHAVE_IGNORE_IWANT = 0x01

# gsim_host_transport callbacks (include/gsim.h)
HOST_A2A = ctypes.CFUNCTYPE(c_int32, c_void_p, POINTER(c_uint8), POINTER(c_uint64), POINTER(c_uint64),
                            POINTER(c_uint8), POINTER(c_uint64), POINTER(c_uint64))
HOST_ALLREDUCE = ctypes.CFUNCTYPE(c_int32, c_void_p, c_void_p, c_int64, c_int32, c_int32)


class CHostTransport(Structure):
    _fields_ = [("ctx", c_void_p), ("alltoallv", HOST_A2A), ("allreduce", HOST_ALLREDUCE)]


class CShardInfo(Structure):
    _fields_ = [("shard", c_int32), ("shards", c_int32), ("n_local", c_int64), ("e_local", c_int64),
                ("own_lo", c_int64), ("own_hi", c_int64), ("own_e_lo", c_int64), ("own_e_hi", c_int64),
                ("n_cross", c_int64)]


MAX_SHARDS = 64


# ---- gsim_wire.h ------------------------------------------------------------------
class CBytes(Structure):
    _fields_ = [("p", c_void_p), ("n", c_uint32)]


class CWireSub(Structure):
    _fields_ = [("subscribe", c_int32), ("topic", CBytes)]


class CWireMsg(Structure):
    _fields_ = [("from_", CBytes), ("data", CBytes), ("seqno", CBytes), ("topic", CBytes), ("signature", CBytes),
                ("key", CBytes)]


class CWireIHave(Structure):
    _fields_ = [("topic", CBytes), ("id0", c_uint32), ("nid", c_uint32)]


class CWireIWant(Structure):
    _fields_ = [("id0", c_uint32), ("nid", c_uint32)]


class CWireGraft(Structure):
    _fields_ = [("topic", CBytes)]


class CWirePx(Structure):
    _fields_ = [("peer", CBytes), ("record", CBytes)]


class CWirePrune(Structure):
    _fields_ = [("topic", CBytes), ("px0", c_uint32), ("npx", c_uint32), ("has_backoff", c_int32),
                ("backoff", c_uint64)]


class CWireRpc(Structure):
    _fields_ = [("subs", c_void_p), ("nsubs", c_uint32), ("msgs", c_void_p), ("nmsgs", c_uint32),
                ("has_control", c_int32), ("ihave", c_void_p), ("nihave", c_uint32), ("iwant", c_void_p),
                ("niwant", c_uint32), ("graft", c_void_p), ("ngraft", c_uint32), ("prune", c_void_p),
                ("nprune", c_uint32), ("ids", c_void_p), ("nids", c_uint32), ("px", c_void_p), ("npx", c_uint32)]


class CWireTables(Structure):
    _fields_ = [("subs", c_void_p), ("msgs", c_void_p), ("ihave", c_void_p), ("iwant", c_void_p), ("graft", c_void_p),
                ("prune", c_void_p), ("ids", c_void_p), ("px", c_void_p),
                ("subs_cap", c_uint32), ("msgs_cap", c_uint32), ("ihave_cap", c_uint32), ("iwant_cap", c_uint32),
                ("graft_cap", c_uint32), ("prune_cap", c_uint32), ("ids_cap", c_uint32), ("px_cap", c_uint32)]


class CWireNames(Structure):
    _fields_ = [("topic_names", c_void_p), ("peer_ids", c_void_p), ("peer_id_len", c_uint32),
                ("prune_backoff_s", c_uint64)]


# numpy view of gsim_wire_ref (24 bytes)
WIRE_REF_DTYPE = [("from", "<u4"), ("to", "<u4"), ("len", "<u4"), ("pad", "<u4"), ("offset", "<u8")]

SIGNATURES = [
    ("gsim_default_gossipsub_params", None, [POINTER(CGossipSubParams)]),
    ("gsim_validate_topic_params", c_int32, [POINTER(CTopicScoreParams), c_char_p, c_size_t]),
    ("gsim_validate_peer_params", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, c_char_p, c_size_t]),
    ("gsim_validate_thresholds", c_int32, [POINTER(CThresholds), c_char_p, c_size_t]),
    ("gsim_score_parameter_decay", c_double, [c_int64]),
    ("gsim_score_parameter_decay_with_base", c_double, [c_int64, c_int64, c_double]),
    ("gsim_create", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, POINTER(CThresholds),
      POINTER(CGossipSubParams), c_int32, POINTER(c_void_p), c_char_p, c_size_t]),
    ("gsim_create_unvalidated", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, POINTER(CThresholds),
      POINTER(CGossipSubParams), c_int32, POINTER(c_void_p), c_char_p, c_size_t]),
    ("gsim_destroy", c_int32, [c_void_p]),
    ("gsim_last_error", c_char_p, [c_void_p]),
    ("gsim_load_graph", c_int32,
     [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
    ("gsim_set_app_score", c_int32, [c_void_p, c_void_p]),
    ("gsim_set_ip_whitelist", c_int32, [c_void_p, c_void_p]),
    ("gsim_set_topic_params", c_int32, [c_void_p, c_int32, POINTER(CTopicScoreParams)]),
    ("gsim_refresh_scores", c_int32, [c_void_p, c_int64]),
    ("gsim_compute_scores", c_int32, [c_void_p]),
    ("gsim_compute_ip_colocation", c_int32, [c_void_p]),
    ("gsim_read_scores", c_int32, [c_void_p, c_void_p]),
    ("gsim_field_bytes", c_int32, [c_void_p, c_int32, POINTER(c_size_t)]),
    ("gsim_read_field", c_int32, [c_void_p, c_int32, c_void_p, c_size_t]),
    ("gsim_write_field", c_int32, [c_void_p, c_int32, c_void_p, c_size_t]),
    ("gsim_event_record", c_int32, [c_void_p, c_int32]),
    ("gsim_event_elapsed", c_int32, [c_void_p, c_int32, c_int32, POINTER(c_float)]),
    ("gsim_synchronize", c_int32, [c_void_p]),
    ("gsim_set_kernel_variant", c_int32, [c_void_p, c_int32, c_int32]),
    ("gsim_gen_random_regular", c_int32, [c_int64, c_int32, c_uint64, c_void_p, c_void_p, c_void_p]),
    ("gsim_gen_power_law", c_int32, [c_int64, c_double, c_double, c_int32, c_double, c_uint64, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    ("gsim_fill_synthetic", c_int32, [c_void_p, c_uint64, c_int64, c_double]),
    ("gsim_set_seed", c_int32, [c_void_p, c_uint64]),
    ("gsim_census", c_int32, [c_void_p, c_void_p]),
    ("gsim_heartbeat", c_int32, [c_void_p, c_uint64, c_int64]),
    ("gsim_handle_control", c_int32, [c_void_p, c_int32, c_int64]),
    ("gsim_msgs_init", c_int32, [c_void_p, POINTER(CMsgConfig)]),
    ("gsim_publish", c_int32, [c_void_p, c_void_p, c_int32, c_int64]),
    ("gsim_round", c_int32, [c_void_p, c_int64]),
    ("gsim_step", c_int32, [c_void_p, c_uint64, c_int32, c_void_p, c_void_p]),
    ("gsim_host_sync_count", c_int32, [c_void_p]),
    ("gsim_msg_stats", c_int32, [c_void_p, c_void_p]),
    ("gsim_set_peer_behaviour", c_int32, [c_void_p, c_void_p]),
    ("gsim_gossip_stats", c_int32, [c_void_p, c_void_p]),
    ("gsim_set_connections", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int64]),
    ("gsim_px_connect", c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_void_p]),
    ("gsim_trace_config", c_int32, [c_void_p, c_uint32, c_uint32, c_int64]),
    ("gsim_trace_read", c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    ("gsim_set_direct_peers", c_int32, [c_void_p, c_void_p]),
    ("gsim_profile", c_int32, [c_void_p, c_int32]),
    ("gsim_profile_read", c_int32, [c_void_p, c_void_p, c_void_p, c_int32]),
    ("gsim_shard_partition", c_int32, [c_int64, c_void_p, c_void_p, c_int32, c_void_p]),
    ("gsim_shard_layout_info", c_int32, [c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                                         POINTER(CShardInfo)]),
    ("gsim_shard_layout", c_int32, [c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gsim_read_snapshot", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    ("gsim_set_ips", c_int32, [c_void_p, c_void_p, c_void_p, c_uint32]),
    ("gsim_set_subscriptions", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_uint64, c_int64]),
    ("gsim_validate_peer_gater_params", c_int32, [POINTER(CPeerGaterParams), c_char_p, c_size_t]),
    ("gsim_default_peer_gater_params", c_int32, [c_double, c_double, c_double, POINTER(CPeerGaterParams)]),
    ("gsim_set_peer_gater", c_int32, [c_void_p, POINTER(CPeerGaterParams), c_void_p]),
    ("gsim_gater_throttled", c_int32, [c_void_p, POINTER(c_int64)]),
    ("gsim_gater_read", c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gsim_rccl_unique_id", c_int32, [c_void_p, c_size_t]),
    ("gsim_group_create", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, POINTER(CThresholds),
      POINTER(CGossipSubParams), c_int32, c_void_p, POINTER(c_void_p), c_char_p, c_size_t]),
    ("gsim_group_create_rccl", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, POINTER(CThresholds),
      POINTER(CGossipSubParams), c_int32, c_int32, c_int32, c_void_p, POINTER(c_void_p), c_char_p, c_size_t]),
    ("gsim_group_create_host", c_int32,
     [POINTER(CPeerScoreParams), POINTER(CTopicScoreParams), c_int32, POINTER(CThresholds),
      POINTER(CGossipSubParams), c_int32, c_int32, c_int32, POINTER(CHostTransport), POINTER(c_void_p), c_char_p,
      c_size_t]),
    ("gsim_group_px_connect", c_int32, [c_void_p, c_int64, c_void_p, c_int64, POINTER(c_int64)]),
    ("gsim_group_set_subscriptions", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_uint64, c_int64]),
    ("gsim_group_destroy", c_int32, [c_void_p]),
    ("gsim_group_last_error", c_char_p, [c_void_p]),
    ("gsim_group_shard", c_void_p, [c_void_p, c_int32]),
    ("gsim_group_bounds", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_load_graph", c_int32,
     [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_void_p]),
    ("gsim_group_set_app_score", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_set_ip_whitelist", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_set_direct_peers", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_set_peer_behaviour", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_set_topic_params", c_int32, [c_void_p, c_int32, POINTER(CTopicScoreParams)]),
    ("gsim_group_set_seed", c_int32, [c_void_p, c_uint64]),
    ("gsim_group_fill_synthetic", c_int32, [c_void_p, c_uint64, c_int64, c_double]),
    ("gsim_group_msgs_init", c_int32, [c_void_p, POINTER(CMsgConfig)]),
    ("gsim_group_refresh_scores", c_int32, [c_void_p, c_int64]),
    ("gsim_group_heartbeat", c_int32, [c_void_p, c_uint64, c_int64]),
    ("gsim_group_publish", c_int32, [c_void_p, c_void_p, c_int32, c_int64]),
    ("gsim_group_round", c_int32, [c_void_p, c_int64]),
    ("gsim_group_set_connections", c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int64]),
    ("gsim_group_set_ips", c_int32, [c_void_p, c_void_p, c_void_p, c_uint32]),
    ("gsim_group_state_written", c_int32, [c_void_p]),
    ("gsim_group_msg_stats", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_gossip_stats", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_census", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_synchronize", c_int32, [c_void_p]),
    ("gsim_group_profile", c_int32, [c_void_p, c_int32]),
    ("gsim_group_profile_read", c_int32, [c_void_p, c_void_p, c_void_p, c_int32]),
    ("gsim_group_field_bytes", c_int32, [c_void_p, c_int32, POINTER(c_size_t)]),
    ("gsim_group_read_field", c_int32, [c_void_p, c_int32, c_void_p, c_size_t]),
    ("gsim_group_read_scores", c_int32, [c_void_p, c_void_p]),
    ("gsim_group_read_snapshot", c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p]),
    ("gsim_group_trace_config", c_int32, [c_void_p, c_uint32, c_uint32, c_int64]),
    ("gsim_group_set_peer_gater", c_int32, [c_void_p, POINTER(CPeerGaterParams), c_void_p]),
    ("gsim_group_gater_throttled", c_int32, [c_void_p, POINTER(c_int64)]),
    ("gsim_group_gater_read", c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    ("gsim_group_trace_read", c_int32, [c_void_p, c_void_p, c_int64, POINTER(c_int64)]),
    # gsim_wire.h
    ("gsim_wire_size", c_uint64, [POINTER(CWireRpc)]),
    ("gsim_trace_delimited", c_int32, [c_void_p, c_uint64, c_void_p, c_uint64, POINTER(c_uint64)]),
    ("gsim_wire_decode", c_int32, [c_void_p, c_uint64, POINTER(CWireTables), POINTER(CWireRpc)]),
    ("gsim_wire_frames", c_int32, [c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_int32, POINTER(c_int32),
                                   POINTER(c_uint64)]),
    ("gsim_wire_encode", c_int32, [POINTER(CWireRpc), c_void_p, c_uint64, POINTER(c_uint64)]),
    ("gsim_trace_encode", c_int32, [c_void_p, c_int64, POINTER(CWireNames), ctypes.c_char_p, c_void_p, c_uint64,
                                    POINTER(c_uint64)]),
    ("gsim_wire_fragment", c_int32, [POINTER(CWireRpc), c_int64, c_void_p, c_uint64, POINTER(c_uint64), c_void_p,
                                     c_int32, POINTER(c_int32)]),
    ("gsim_trace_rpc_encode", c_int32, [c_void_p, c_void_p, c_int64, POINTER(CWireNames), c_int64, c_int32, c_void_p,
                                        c_uint64, POINTER(c_uint64)]),
    ("gsim_wire_heartbeat", c_int32, [c_void_p, c_int64, c_uint32, c_uint32, POINTER(CWireNames), c_void_p, c_uint64,
                                      c_void_p, c_int64, POINTER(c_int64), POINTER(c_uint64)]),
]

_lib = None


def load(path: str | None = None) -> ctypes.CDLL:
    """Load libgsim.so (built in-tree by `make -C go-libp2p-pubsub_amd`).

    torch is imported first when available so that the HIP runtime torch
    bundles and the one libgsim links resolve to a single copy (both carry the
    SONAME libamdhip64.so.7).
    """
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("GSIM_LIB") or LIB_PATH      # GSIM_LIB: another build, for A/B runs
    if not os.path.exists(p):
        raise ImportError(f"libgsim.so not built at {p}; run `make -C go-libp2p-pubsub_amd` "
                          "(the engine has no CPU fallback)")
    try:  # share one HIP runtime with torch if the caller uses torch
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is present in this image
        pass
    lib = ctypes.CDLL(p)
    older = p != LIB_PATH                                    # an A/B build may predate newer entry points
    for name, res, args in SIGNATURES:
        if older and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib
