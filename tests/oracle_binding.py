"""ctypes binding of oracle/liboracle.so (test infrastructure only).

`NetState` holds every state array of a simulated network in numpy, in the
exact layout the engine uses, and exposes an `orc_net` view for the oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, Structure, c_double, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
# GSIM_ORACLE_LIB: another build of the same sources (tools/asan_oracle.py: ASan/UBSan)
ORACLE_LIB = os.environ.get("GSIM_ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle.so")

import sys  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "go-libp2p-pubsub_amd"))
from gsim import _abi  # noqa: E402


class OrcNet(Structure):
    _fields_ = [
        ("n", c_int64), ("e", c_int64), ("t", c_int32), ("_pad", c_int32),
        ("row_ptr", c_void_p), ("col", c_void_p), ("rev", c_void_p), ("sub", c_void_p), ("outbound", c_void_p),
        ("ip_ptr", c_void_p), ("ip_ids", c_void_p), ("ip_white", c_void_p), ("p5", c_void_p),
        ("first", c_void_p), ("meshd", c_void_p), ("fail", c_void_p), ("invalid", c_void_p),
        ("graft_time", c_void_p), ("mesh_time", c_void_p), ("tflags", c_void_p),
        ("bp", c_void_p), ("estate", c_void_p), ("expire", c_void_p), ("p6", c_void_p), ("score", c_void_p),
        ("backoff", c_void_p),
        ("pp", c_void_p), ("tp", c_void_p), ("th", c_void_p), ("gp", c_void_p),
        ("ctl", c_void_p), ("lastpub", c_void_p), ("fan_topics", c_void_p), ("direct", c_void_p),
        ("px", c_void_p), ("gater", c_void_p), ("px_pend", c_void_p),
    ]


class OrcMsgs(Structure):
    _fields_ = [
        ("ring", c_int32), ("rounds", c_int32), ("t0", c_int64), ("hb", c_int64),
        ("topic", c_void_p), ("origin", c_void_p), ("invalid", c_void_p), ("seen", c_void_p),
        ("lastput", c_void_p), ("stats", c_int64 * 4), ("priv", c_void_p),
        ("mid", c_void_p), ("behaviour", c_void_p), ("topic_slots", c_int32),
    ]


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        lib = ctypes.CDLL(ORACLE_LIB)
        # the ctypes mirrors must match the C structs field for field: a field
        # added to orc_net on one side only made orc_round read past the struct
        # (round 3's segfault under test_churn_ticks_bit_exact)
        lib.orc_layout_size.restype = c_int64
        lib.orc_layout_size.argtypes = [c_int32]
        for which, st in ((0, OrcNet), (1, OrcMsgs)):
            got = lib.orc_layout_size(which)
            if got != ctypes.sizeof(st):
                raise RuntimeError(f"{st.__name__}: ctypes size {ctypes.sizeof(st)} != C size {got} ({ORACLE_LIB})")
        P = POINTER(OrcNet)
        sig = {
            "orc_refresh_scores": (None, [P, c_int64]),
            "orc_score_edge": (c_double, [P, c_int64]),
            "orc_compute_scores": (None, [P]),
            "orc_set_threads": (ctypes.c_int, [ctypes.c_int]),
            "orc_ip_colocation": (None, [P]),
            "orc_add_penalty": (None, [P, c_int64, c_int32]),
            "orc_graft": (None, [P, c_int64, c_int32, c_int64]),
            "orc_prune": (None, [P, c_int64, c_int32]),
            "orc_add_peer": (None, [P, c_int64]),
            "orc_remove_peer": (None, [P, c_int64, c_int64]),
            "orc_churn": (c_int32, [P, c_void_p, c_int32, c_int32, c_int64]),
            "orc_set_topic_params": (None, [P, c_int32, c_void_p, c_void_p]),
            "orc_mark_first": (None, [P, c_int64, c_int32]),
            "orc_mark_duplicate": (None, [P, c_int64, c_int32, c_int32, c_int64, c_int64]),
            "orc_mark_invalid": (None, [P, c_int64, c_int32]),
            "orc_drecs_new": (c_void_p, [c_int64]),
            "orc_drecs_free": (None, [c_void_p]),
            "orc_validate_message": (None, [P, c_void_p, c_uint64, c_int64]),
            "orc_deliver_message": (None, [P, c_void_p, c_int64, c_uint64, c_int32, c_int64]),
            "orc_reject_message": (None, [P, c_void_p, c_int64, c_uint64, c_int32, c_int32, c_int64]),
            "orc_duplicate_message": (None, [P, c_void_p, c_int64, c_uint64, c_int32, c_int64]),
            "orc_drecs_gc": (None, [c_void_p, c_int64]),
            "orc_drecs_expire_head": (None, [c_void_p, c_int64]),
            "orc_mcache_new": (c_void_p, [c_int32, c_int32]),
            "orc_mcache_free": (None, [c_void_p]),
            "orc_mcache_put": (None, [c_void_p, c_uint64, c_int32]),
            "orc_mcache_get": (c_int32, [c_void_p, c_uint64]),
            "orc_mcache_get_for_peer": (c_int32, [c_void_p, c_uint64, c_uint32, POINTER(c_int32)]),
            "orc_mcache_gossip_ids": (c_int32, [c_void_p, c_int32, c_void_p, c_int32]),
            "orc_mcache_shift": (None, [c_void_p]),
            "orc_mcache_len": (c_int32, [c_void_p]),
            "orc_gtracer_new": (c_void_p, [c_int64]),
            "orc_gtracer_free": (None, [c_void_p]),
            "orc_gtracer_add_promise": (None, [c_void_p, c_uint32, c_void_p, c_int32, c_int32, c_int64]),
            "orc_gtracer_broken": (c_int32, [c_void_p, c_int64, c_void_p, c_void_p, c_int32]),
            "orc_gtracer_fulfill": (None, [c_void_p, c_uint64]),
            "orc_gtracer_throttle": (None, [c_void_p, c_uint32]),
            "orc_gtracer_peer_promises": (c_int32, [c_void_p]),
            "orc_msgs_log": (None, [POINTER(OrcMsgs), c_int32]),
            "orc_msgs_events": (c_int64, [POINTER(OrcMsgs), c_void_p, c_int64]),
            "orc_msgs_ihave_marks": (c_int64, [POINTER(OrcMsgs), c_void_p, c_int64]),
            "orc_tcache_new": (c_void_p, [c_int32, c_int64]),
            "orc_tcache_free": (None, [c_void_p]),
            "orc_tcache_add": (c_int32, [c_void_p, c_uint64, c_int64]),
            "orc_tcache_has": (c_int32, [c_void_p, c_uint64, c_int64]),
            "orc_tcache_sweep": (None, [c_void_p, c_int64]),
            "orc_philox4x32_10": (None, [c_void_p, c_void_p, c_void_p]),
            "orc_heartbeat": (None, [P, c_uint64, c_int64, c_uint64]),
            "orc_handle_control": (c_int64, [P, c_int32, c_int64]),
            "orc_round_time": (c_int64, [POINTER(OrcMsgs), c_int64]),
            "orc_publish": (None, [P, POINTER(OrcMsgs), c_uint64, c_uint32, c_uint32, ctypes.c_uint8, c_int64]),
            "orc_publish_v": (None, [P, POINTER(OrcMsgs), c_uint64, c_uint32, c_uint32, ctypes.c_uint8, ctypes.c_uint8,
                                     c_int64]),
            "orc_round": (None, [P, POINTER(OrcMsgs), c_int64]),
            "orc_msgs_free_priv": (None, [POINTER(OrcMsgs)]),
            "orc_heartbeat_gossip": (None, [P, POINTER(OrcMsgs), c_uint64, c_int64, c_uint64]),
            "orc_gossip_penalties": (None, [P, POINTER(OrcMsgs), c_int64]),
            "orc_px_connect": (c_int64, [P, c_int64, c_void_p, c_int64]),
"orc_set_subscriptions": (None, [P, c_void_p, c_int32, c_int32, c_uint64, c_int64, c_uint64]),
            "orc_gater_validate": (c_int32, [POINTER(_abi.CPeerGaterParams)]),
            "orc_gater_new": (c_void_p, [P, POINTER(_abi.CPeerGaterParams), c_void_p]),
            "orc_gater_free": (None, [c_void_p]),
            "orc_px_pend_new": (c_void_p, []),
            "orc_px_pend_free": (None, [c_void_p]),
            "orc_gater_round_begin": (None, [P, c_int64]),
            "orc_gater_accept": (c_int32, [P, c_uint64, c_int64, c_uint32, c_uint32, c_uint32]),
            "orc_gater_event": (None, [P, c_uint32, c_uint32, c_int32, c_int32]),
            "orc_gater_round_end": (None, [P, c_int64]),
            "orc_gater_decay": (None, [P, c_int64]),
            "orc_gater_connection": (None, [P, c_int64, c_int32, c_int64]),
            "orc_gater_throttled": (c_int64, [c_void_p]),
            "orc_gater_read": (None, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
            "orc_gater_uniform": (ctypes.c_double, [c_uint64, c_int64, c_uint32, c_uint32, c_uint32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


class NetState:
    """All engine state of one network, host-side, in engine layout."""

    TOPIC_FIELDS = ("first", "meshd", "fail", "invalid", "graft_time", "mesh_time", "tflags", "backoff")
    EDGE_FIELDS = ("bp", "estate", "expire", "p6", "score")
    DTYPES = {"first": np.float64, "meshd": np.float64, "fail": np.float64, "invalid": np.float64,
              "graft_time": np.int64, "mesh_time": np.int64, "tflags": np.uint8, "backoff": np.int64,
              "bp": np.float64, "estate": np.uint8, "expire": np.int64, "p6": np.float64, "score": np.float64}
    FIELD_IDS = {"first": _abi.F_FIRST, "meshd": _abi.F_MESHD, "fail": _abi.F_FAIL, "invalid": _abi.F_INVALID,
                 "graft_time": _abi.F_GRAFT_TIME, "mesh_time": _abi.F_MESH_TIME, "tflags": _abi.F_TFLAGS,
                 "backoff": _abi.F_BACKOFF, "bp": _abi.F_BP, "estate": _abi.F_ESTATE, "expire": _abi.F_EXPIRE,
                 "p6": _abi.F_P6, "score": _abi.F_SCORE}

    def __init__(self, net, params, thresholds=None, gossip=None, topics=None, p5=None, ip_white=None):
        from gsim.params import GossipSubParams, PeerScoreThresholds
        self.net = net
        self.params = params
        self.topics = sorted(set(topics or []) | set(params.Topics))
        self.T = max(1, len(self.topics))
        E = net.e
        for f in self.TOPIC_FIELDS:
            setattr(self, f, np.zeros((self.T, E), dtype=self.DTYPES[f]))
        for f in self.EDGE_FIELDS:
            setattr(self, f, np.zeros(E, dtype=self.DTYPES[f]))
        self.estate[:] = _abi.ES_TRACKED | _abi.ES_CONNECTED
        self.ctl = np.zeros((2, self.T, E), dtype=np.uint8)
        self.lastpub = np.zeros((net.n, self.T), dtype=np.int64)
        self.fan_topics = np.zeros(net.n, dtype=np.uint64)
        self.direct = np.zeros(E, dtype=np.uint8)          # gs.direct flags (configuration, not state)
        # peer exchange attempts (WithPeerExchange), when on
        self.px = np.zeros(E, dtype=np.uint8) if (gossip is not None and gossip.PeerExchange) else None
        # Leave's pending PX lists (oracle_net.c), owned with this network
        self._px_pend = load().orc_px_pend_new() if self.px is not None else None
        self.rev = net.rev()
        self.p5 = np.zeros(net.n) if p5 is None else np.ascontiguousarray(p5, dtype=np.float64)
        self.ip_white = None if ip_white is None else np.ascontiguousarray(ip_white, dtype=np.uint8)
        self.pp = params.to_c()
        self.tp = params.topic_array(self.topics)
        self.th = (thresholds or PeerScoreThresholds()).to_c()
        self.gp = (gossip or GossipSubParams()).to_c()
        self.gater = None            # orc_gater* (enable_gater)
        self._view = None

    def __del__(self):
        try:
            if self._px_pend:
                load().orc_px_pend_free(self._px_pend)
                self._px_pend = None
        except Exception:
            pass

    def view(self):
        n = self.net
        v = OrcNet()
        v.n, v.e, v.t = n.n, n.e, len(self.topics)
        v.row_ptr, v.col, v.rev, v.sub, v.outbound = _p(n.row_ptr), _p(n.col), _p(self.rev), _p(n.sub), _p(n.outbound)
        v.ip_ptr, v.ip_ids = _p(n.ip_ptr), _p(n.ip_ids)
        if n.ip_ptr is None:  # no IPs known (ps.host == nil in the reference tests)
            self._zero_ip_ptr = np.zeros(n.n + 1, dtype=np.uint32)
            self._zero_ip_ids = np.zeros(1, dtype=np.uint32)
            v.ip_ptr, v.ip_ids = _p(self._zero_ip_ptr), _p(self._zero_ip_ids)
        v.ip_white = _p(self.ip_white)
        v.p5 = _p(self.p5)
        for f in self.TOPIC_FIELDS + self.EDGE_FIELDS:
            setattr(v, f, _p(getattr(self, f)))
        v.pp = ctypes.cast(ctypes.byref(self.pp), c_void_p)
        v.tp = ctypes.cast(self.tp, c_void_p)
        v.th = ctypes.cast(ctypes.byref(self.th), c_void_p)
        v.gp = ctypes.cast(ctypes.byref(self.gp), c_void_p)
        v.ctl = _p(self.ctl)
        v.lastpub, v.fan_topics = _p(self.lastpub), _p(self.fan_topics)
        v.direct = _p(self.direct)
        v.px = _p(self.px)
        v.gater = self.gater
        v.px_pend = self._px_pend
        self._view = v
        return ctypes.byref(v)

    # ---- peer gater (oracle_gater.c) ----
    GATE_VALIDATE, GATE_DELIVER, GATE_DUPLICATE, GATE_IGNORE, GATE_REJECT, GATE_THROTTLE = range(6)

    def enable_gater(self, params, topic_weights=None):
        """orc_gater_new: WithPeerGater on every router of the oracle network."""
        c = params.to_c()
        T = max(1, len(self.topics))
        w = np.zeros(T, dtype=np.float64)
        for t, x in (params.TopicDeliveryWeights or {}).items():
            w[int(t)] = float(x)
        if topic_weights is not None:
            w = np.ascontiguousarray(topic_weights, dtype=np.float64)
        self._gater_w = w
        self.gater = None
        self.gater = load().orc_gater_new(self.view(), ctypes.byref(c), _p(w))

    def gater_decay(self, now):
        load().orc_gater_decay(self.view(), int(now))

    def gater_read(self) -> dict:
        N, E = self.net.n, self.net.e
        out = {"validate": np.zeros(N), "throttle": np.zeros(N), "last": np.zeros(N, dtype=np.int64),
               "counters": np.zeros((4, E)), "connected": np.zeros(E, dtype=np.int32),
               "expire": np.zeros(E, dtype=np.int64)}
        load().orc_gater_read(self.gater, _p(out["validate"]), _p(out["throttle"]), _p(out["last"]),
                              _p(out["counters"]), _p(out["connected"]), _p(out["expire"]))
        return out

    def gater_throttled(self) -> int:
        return int(load().orc_gater_throttled(self.gater))

    def copy_fields_from(self, other):
        for f in self.TOPIC_FIELDS + self.EDGE_FIELDS:
            getattr(self, f)[...] = getattr(other, f)

    def churn(self, pairs, up, now):
        """orc_churn: connections going down / up between ticks, both endpoints."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        bad = load().orc_churn(self.view(), _p(p), int(p.shape[0]), 1 if up else 0, int(now))
        assert bad < 0, f"pair {bad} is not a connection"

    def set_subscriptions(self, pairs, join, tick, now, seed):
        """orc_set_subscriptions: Join / Leave of (peer, topic) pairs between ticks."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        load().orc_set_subscriptions(self.view(), _p(p), int(p.shape[0]), 1 if join else 0, int(tick), int(now),
                                     int(seed))

    def px_connect(self, now):
        """orc_px_connect: the connector for this tick's PX attempts; returns
        the (dialer, peer) pairs connected, sorted (outbound flags updated in
        the network's array)."""
        cap = max(1, self.net.e // 2)
        out = np.zeros((cap, 2), dtype=np.uint32)
        n = load().orc_px_connect(self.view(), int(now), _p(out), cap)
        out = out[:n]
        return out[np.lexsort((out[:, 1], out[:, 0]))] if n else out

    def push_to_engine(self, eng):
        for f in self.TOPIC_FIELDS + self.EDGE_FIELDS:
            eng.write(self.FIELD_IDS[f], getattr(self, f))
        eng.write(_abi.F_CTL, self.ctl)
        eng.write(_abi.F_LASTPUB, self.lastpub)
        eng.write(_abi.F_FANOUT_TOPICS, self.fan_topics)
        eng.set_direct_peers(self.direct)

    def pull_from_engine(self, eng, base=None):
        """The engine's state; base: a NetState whose values stand for the
        parts no shard of this process owns (a one-shard-per-process group)."""
        def rd(fid, name):
            return eng.read(fid) if base is None else eng.read(fid, into=getattr(base, name).copy())
        for f in self.TOPIC_FIELDS + self.EDGE_FIELDS:
            getattr(self, f)[...] = rd(self.FIELD_IDS[f], f)
        self.ctl[...] = rd(_abi.F_CTL, "ctl")
        self.lastpub[...] = rd(_abi.F_LASTPUB, "lastpub")
        self.fan_topics[...] = rd(_abi.F_FANOUT_TOPICS, "fan_topics")


UNSEEN = 0xFFFFFFFF
ORC_BEHAVE_IGNORE_IWANT = 0x01   # oracle.h: never answers IWANT


# oracle.h ORC_EV_*: the network oracle's event log
EV_PUT, EV_SEEN, EV_SERVE, EV_PROMISE, EV_FULFILL, EV_BROKEN, EV_PENALTIES, EV_HEARTBEAT, EV_GOSSIP_ID = range(1, 10)
EV_REJECT_SIG, EV_PUBLISH, EV_GRAFT, EV_PRUNE, EV_ADD_PEER, EV_REMOVE_PEER = range(10, 16)
EV_THROTTLE, EV_JOIN, EV_LEAVE, EV_PX_PEER, EV_RPC_MSG, EV_RPC_IWANT = range(16, 22)
EVENT_DTYPE = np.dtype([("kind", np.int32), ("topic", np.int32), ("a", np.uint32), ("b", np.uint32),
                        ("g", np.int64), ("mid", np.uint64), ("x", np.int64)])


class Msgs:
    """Oracle message ring + seen-set of a network (oracle_deliver.c)."""

    def __init__(self, n, T, ring, rounds, t0, hb, behaviour=None, topic_slots=0):
        self.seen = np.full((ring, n), UNSEEN, dtype=np.uint32)
        self.topic = np.zeros(ring, dtype=np.uint32)
        self.origin = np.zeros(ring, dtype=np.uint32)
        self.invalid = np.zeros(ring, dtype=np.uint8)
        self.mid = np.zeros(ring, dtype=np.uint64)
        self.lastput = np.full((T, n), -1, dtype=np.int32)
        self.behaviour = None if behaviour is None else np.ascontiguousarray(behaviour, dtype=np.uint8)
        m = OrcMsgs()
        m.ring, m.rounds, m.t0, m.hb = ring, rounds, t0, hb
        m.topic, m.origin, m.invalid = _p(self.topic), _p(self.origin), _p(self.invalid)
        m.seen, m.lastput = _p(self.seen), _p(self.lastput)
        m.mid, m.behaviour = _p(self.mid), _p(self.behaviour)
        m.topic_slots = int(topic_slots)     # per-topic sub-rings (gsim_msg_config.topic_slots)
        if topic_slots:
            self.topic[:] = np.arange(ring, dtype=np.uint32) // np.uint32(topic_slots)
        self.m = m

    @property
    def stats(self):
        return list(self.m.stats)

    def round_time(self, g):
        return load().orc_round_time(ctypes.byref(self.m), g)

    def publish(self, st, mid, topic, origin, invalid, g, vdelay=0):
        """orc_publish_v: vdelay = validation latency in rounds at every receiver."""
        load().orc_publish_v(st.view(), ctypes.byref(self.m), mid, topic, origin, invalid, vdelay, g)

    def round(self, st, g):
        load().orc_round(st.view(), ctypes.byref(self.m), g)

    def heartbeat(self, st, tick, now, seed):
        """orc_heartbeat_gossip: mesh maintenance + emitGossip for every peer."""
        load().orc_heartbeat_gossip(st.view(), ctypes.byref(self.m), tick, now, seed)

    def penalties(self, st, now):
        """applyIwantPenalties at heartbeat time now (after refresh, before scoring)."""
        load().orc_gossip_penalties(st.view(), ctypes.byref(self.m), now)

    def log(self, on=True):
        """Record the events the routers' caches and tracers observe (orc_msgs_log)."""
        load().orc_msgs_log(ctypes.byref(self.m), 1 if on else 0)

    def ihave_marks(self, E):
        """The last heartbeat's IHAVE marks [T][E] (receivers' edges)."""
        out = np.zeros((self.lastput.shape[0], E), dtype=np.uint8)
        load().orc_msgs_ihave_marks(ctypes.byref(self.m), out.ctypes.data_as(c_void_p), out.size)
        return out

    def events(self):
        """The events recorded since the last call (and clear them)."""
        lib = load()
        n = lib.orc_msgs_events(ctypes.byref(self.m), None, 0)
        out = np.zeros(n, dtype=EVENT_DTYPE)
        if n:
            lib.orc_msgs_events(ctypes.byref(self.m), out.ctypes.data_as(c_void_p), n)
        return out

    def __del__(self):
        try:
            load().orc_msgs_free_priv(ctypes.byref(self.m))
        except Exception:
            pass
