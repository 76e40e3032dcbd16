"""Host-side engine handle over the C ABI (include/gsim.h).

`Engine` plays the role the reference's GossipSubRouter+peerScore pair plays
for one node (gossipsub.go:420-477, score.go:64-86), but for a whole simulated
network held on one MI355X.  Everything computational runs in libgsim.so's HIP
kernels; this module only marshals arrays.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _abi
from .params import GossipSubParams, PeerScoreParams, PeerScoreThresholds

_FIELD_DTYPES = {
    _abi.F_FIRST: np.float64, _abi.F_MESHD: np.float64, _abi.F_FAIL: np.float64, _abi.F_INVALID: np.float64,
    _abi.F_GRAFT_TIME: np.int64, _abi.F_MESH_TIME: np.int64, _abi.F_TFLAGS: np.uint8, _abi.F_BP: np.float64,
    _abi.F_ESTATE: np.uint8, _abi.F_EXPIRE: np.int64, _abi.F_P6: np.float64, _abi.F_SCORE: np.float64,
    _abi.F_BACKOFF: np.int64, _abi.F_CTL: np.uint8, _abi.F_SEEN: np.uint32, _abi.F_LASTPUT: np.int32,
    _abi.F_LASTPUB: np.int64, _abi.F_FANOUT_TOPICS: np.uint64,
}
TOPIC_FIELDS = {_abi.F_FIRST, _abi.F_MESHD, _abi.F_FAIL, _abi.F_INVALID, _abi.F_GRAFT_TIME,
                _abi.F_MESH_TIME, _abi.F_TFLAGS, _abi.F_BACKOFF}
PARITY_TOPIC_FIELDS = {_abi.F_CTL}


class GsimError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"gsim error {rc}: {msg}")
        self.rc = rc


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class Network:
    """A simulated peer graph: CSR rows = observers, columns = neighbours."""
    n: int
    row_ptr: np.ndarray           # uint32 [n+1]
    col: np.ndarray               # uint32 [E]
    outbound: np.ndarray          # uint8  [E]
    sub: np.ndarray               # uint64 [n] topic bitmask
    ip_ptr: Optional[np.ndarray] = None   # uint32 [n+1]
    ip_ids: Optional[np.ndarray] = None   # uint32
    n_ips: int = 0

    @property
    def e(self) -> int:
        return int(self.row_ptr[-1])

    def rev(self) -> np.ndarray:
        """Reverse-edge index (j->i for every i->j)."""
        owner = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.row_ptr.astype(np.int64)))
        key_fwd = owner * self.n + self.col.astype(np.int64)
        key_rev = self.col.astype(np.int64) * self.n + owner
        order = np.argsort(key_fwd, kind="stable")
        pos = np.searchsorted(key_fwd[order], key_rev)
        return order[pos].astype(np.uint32)

    def owner(self) -> np.ndarray:
        return np.repeat(np.arange(self.n, dtype=np.uint32), np.diff(self.row_ptr.astype(np.int64)))


def random_regular(n: int, k: int, seed: int = 1, n_topics: int = 1, unique_ips: bool = True) -> Network:
    """Seeded random k-regular network; all peers join all topics."""
    lib = _abi.load()
    row_ptr = np.empty(n + 1, dtype=np.uint32)
    col = np.empty(n * k, dtype=np.uint32)
    ob = np.empty(n * k, dtype=np.uint8)
    rc = lib.gsim_gen_random_regular(n, k, seed, _ptr(row_ptr), _ptr(col), _ptr(ob))
    if rc != 0:
        raise GsimError(rc, "gsim_gen_random_regular failed")
    mask = (1 << n_topics) - 1 if n_topics < 64 else (1 << 64) - 1
    sub = np.full(n, mask, dtype=np.uint64)
    ip_ptr = ip_ids = None
    n_ips = 0
    if unique_ips:
        ip_ptr = np.arange(n + 1, dtype=np.uint32)
        ip_ids = np.arange(n, dtype=np.uint32)
        n_ips = n
    return Network(n, row_ptr, col, ob, sub, ip_ptr, ip_ids, n_ips)


def app_scores(fn, n: int) -> np.ndarray:
    """AppSpecificScore(p) for every peer index (score_params.go:78), the array
    gsim_set_app_score installs.  A callback marked ``fn.vectorized = True``
    takes the whole index array at once; any other is called once per peer.
    Every peer's value is evaluated: there is no size above which it is skipped."""
    if getattr(fn, "vectorized", False):
        out = np.asarray(fn(np.arange(n, dtype=np.int64)), dtype=np.float64)
        if out.shape != (n,):
            raise ValueError("a vectorized AppSpecificScore must return one value per peer")
        return np.ascontiguousarray(out)
    return np.fromiter((fn(p) for p in range(n)), dtype=np.float64, count=n)


class Engine:
    """One simulated GossipSub network on one GPU."""

    def __init__(self, params: PeerScoreParams, thresholds: PeerScoreThresholds,
                 gossip: Optional[GossipSubParams] = None, topics: Optional[Sequence[str]] = None,
                 device: int = 0, validate: bool = True):
        """validate=False mirrors newPeerScore (score.go:183) as the reference's
        unit tests use it; the default mirrors WithPeerScore (gossipsub.go:278)."""
        self.lib = _abi.load()
        self.params = params
        self.thresholds = thresholds
        self.gossip = gossip or GossipSubParams()
        self.topics: List[str] = sorted(set(topics or []) | set(params.Topics))
        self.topic_index = {t: i for i, t in enumerate(self.topics)}
        pc = params.to_c()
        self._tarr = params.topic_array(self.topics)
        tc = thresholds.to_c()
        gc = self.gossip.to_c()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(512)
        create = self.lib.gsim_create if validate else self.lib.gsim_create_unvalidated
        rc = create(ctypes.byref(pc), self._tarr, len(self.topics), ctypes.byref(tc),
                                  ctypes.byref(gc), device, ctypes.byref(h), buf, len(buf))
        if rc != 0:
            if rc == _abi.GSIM_EINVAL:
                raise ValueError(buf.value.decode())
            raise GsimError(rc, buf.value.decode())
        self.h = h
        self.device = device
        self.net: Optional[Network] = None

    # -- lifecycle -----------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.gsim_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != 0:
            msg = self.lib.gsim_last_error(self.h)
            msg = msg.decode() if msg else ""
            if rc == _abi.GSIM_EINVAL:
                raise ValueError(msg)
            raise GsimError(rc, msg)

    # -- setup -----------------------------------------------------------------
    def load_graph(self, net: Network):
        self._check(self.lib.gsim_load_graph(
            self.h, net.n, _ptr(net.row_ptr), _ptr(net.col), _ptr(net.outbound), _ptr(net.sub),
            _ptr(net.ip_ptr), _ptr(net.ip_ids), net.n_ips))
        self.net = net
        if self.params.AppSpecificScore is not None:
            self.set_app_score(app_scores(self.params.AppSpecificScore, net.n))

    def set_app_score(self, p5: np.ndarray):
        p5 = np.ascontiguousarray(p5, dtype=np.float64)
        self._check(self.lib.gsim_set_app_score(self.h, _ptr(p5)))

    def set_ips(self, ip_ptr: np.ndarray, ip_ids: np.ndarray, n_ips: int):
        """refreshIPs (score.go:568-585): every peer's IP list replaced (gsim_set_ips)."""
        p = np.ascontiguousarray(ip_ptr, dtype=np.uint32)
        i = np.ascontiguousarray(ip_ids, dtype=np.uint32)
        self._check(self.lib.gsim_set_ips(self.h, _ptr(p), _ptr(i), int(n_ips)))

    def snapshot(self, obs_lo: int = 0, obs_hi: Optional[int] = None):
        """ExtendedPeerScoreInspectFn's view (score.go:127-140, 472-500) of the
        observers [obs_lo, obs_hi): one PeerScoreSnapshot per connection (edge
        order) and its TopicScoreSnapshots [edges, T] (gsim_read_snapshot)."""
        hi = self.net.n if obs_hi is None else obs_hi
        ne = int(self.net.row_ptr[hi]) - int(self.net.row_ptr[obs_lo])
        T = max(1, len(self.topics))
        peers = np.zeros(ne, dtype=_abi.PEER_SNAPSHOT_DTYPE)
        topics = np.zeros((ne, T), dtype=_abi.TOPIC_SNAPSHOT_DTYPE)
        self._check(self.lib.gsim_read_snapshot(self.h, int(obs_lo), int(hi), _ptr(peers), _ptr(topics)))
        return peers, topics

    def set_ip_whitelist(self, white: Optional[np.ndarray]):
        w = None if white is None else np.ascontiguousarray(white, dtype=np.uint8)
        self._check(self.lib.gsim_set_ip_whitelist(self.h, _ptr(w)))

    def set_topic_score_params(self, topic: str, p):
        """Topic.SetScoreParams -> peerScore.SetTopicScoreParams (topic.go:44-82, score.go:201-241)."""
        c = p.to_c(True)
        self._check(self.lib.gsim_set_topic_params(self.h, self.topic_index[topic], ctypes.byref(c)))
        self.params.Topics[topic] = p

    # -- hot path ----------------------------------------------------------------
    def refresh_scores(self, now: int):
        self._check(self.lib.gsim_refresh_scores(self.h, int(now)))

    def compute_scores(self):
        self._check(self.lib.gsim_compute_scores(self.h))

    def compute_ip_colocation(self):
        self._check(self.lib.gsim_compute_ip_colocation(self.h))

    def fill_synthetic(self, seed: int, now: int, p_mesh: float):
        self._check(self.lib.gsim_fill_synthetic(self.h, int(seed), int(now), float(p_mesh)))

    def scores(self) -> np.ndarray:
        out = np.empty(self.net.e, dtype=np.float64)
        self._check(self.lib.gsim_read_scores(self.h, _ptr(out)))
        return out

    # -- raw state ----------------------------------------------------------------
    def field_shape(self, f: int):
        e = self.net.e
        if f in PARITY_TOPIC_FIELDS:
            return (2, max(1, len(self.topics)), e)
        if f == _abi.F_SEEN:
            return (self._msg_cfg.ring, self.net.n)
        if f == _abi.F_LASTPUT:
            return (max(1, len(self.topics)), self.net.n)
        if f == _abi.F_LASTPUB:
            return (self.net.n, max(1, len(self.topics)))
        if f == _abi.F_FANOUT_TOPICS:
            return (self.net.n,)
        return (max(1, len(self.topics)), e) if f in TOPIC_FIELDS else (e,)

    # -- heartbeat / control ------------------------------------------------------
    def census(self) -> dict:
        out = np.zeros(8, dtype=np.int64)
        self._check(self.lib.gsim_census(self.h, _ptr(out)))
        keys = ["records", "in_mesh", "nz_first", "nz_meshd", "nz_fail", "nz_invalid", "mesh_links",
                "tracked_edges"]
        return {k: int(v) for k, v in zip(keys, out)}

    def set_seed(self, seed: int):
        self._check(self.lib.gsim_set_seed(self.h, int(seed)))

    def heartbeat(self, tick: int, now: int):
        """GossipSubRouter.heartbeat for every observer (gossipsub.go:1345-1606)."""
        self._check(self.lib.gsim_heartbeat(self.h, int(tick), int(now)))

    def handle_control(self, rnd: int, now: int):
        """handleGraft/handlePrune for the inbox of control round `rnd`."""
        self._check(self.lib.gsim_handle_control(self.h, int(rnd), int(now)))

    # -- message propagation ------------------------------------------------------
    def msgs_init(self, ring: int, rounds: int, t0: int, heartbeat: Optional[int] = None,
                  max_frontier: Optional[int] = None, max_arrivals: Optional[int] = None,
                  topic_slots: int = 0):
        """Allocate the message ring / seen-set (gsim_msgs_init).  topic_slots > 0:
        per-topic sub-rings (a message takes its topic's next slot in publication
        order) with member-compacted seen-set cells."""
        c = _abi.CMsgConfig()
        c.ring, c.rounds, c.t0_ns = int(ring), int(rounds), int(t0)
        c.heartbeat_ns = int(heartbeat if heartbeat is not None else self.gossip.HeartbeatInterval)
        # max_frontier bounds the claim / forwarder lists of member-compacted layouts
        # (0: the default; overflow falls back to the word scans); max_arrivals
        # sizes the IWANT response queue (0: the library default, gsim.h)
        c.max_frontier = int(max_frontier or 0)
        c.max_arrivals = int(max_arrivals or 0)
        # > 0: per-topic sub-rings of this many slots (ring = n_topics * topic_slots),
        # seen-set cells only for each topic's members (gsim.h gsim_msg_config)
        c.topic_slots = int(topic_slots or 0)
        self._check(self.lib.gsim_msgs_init(self.h, ctypes.byref(c)))
        self._msg_cfg = c

    def round_time(self, g: int) -> int:
        c = self._msg_cfg
        return c.t0_ns + (g // c.rounds) * c.heartbeat_ns + (g % c.rounds + 1) * c.heartbeat_ns // (c.rounds + 1)

    def publish(self, msgs, rnd: int):
        """Topic.Publish of each (id, topic, origin, verdict[, vdelay]) at its origin in
        round `rnd` (verdict: _abi.VERDICT_*, the validation result at every receiver;
        vdelay: the validation latency at every receiver in rounds, gsim_msg.vdelay)."""
        arr = np.zeros(len(msgs), dtype=_abi.MSG_DTYPE)
        for k, msg in enumerate(msgs):
            mid, topic, origin, verdict = msg[:4]
            arr[k]["id"], arr[k]["topic"], arr[k]["origin"], arr[k]["verdict"] = mid, topic, origin, verdict
            arr[k]["vdelay"] = msg[4] if len(msg) > 4 else 0
        self._check(self.lib.gsim_publish(self.h, _ptr(arr), len(arr), int(rnd)))

    def publish_array(self, arr: np.ndarray, rnd: int):
        """Like publish() for a prebuilt numpy array of dtype _abi.MSG_DTYPE."""
        a = np.ascontiguousarray(arr)
        self._check(self.lib.gsim_publish(self.h, _ptr(a), len(a), int(rnd)))

    def round(self, rnd: int):
        """One propagation round for the whole network (gsim_round)."""
        self._check(self.lib.gsim_round(self.h, int(rnd)))

    def step(self, tick: int, n_ticks: int = 1, sched: Optional[dict] = None):
        """n_ticks whole heartbeat ticks in one call (gsim_step): refresh,
        heartbeat and the rounds of each tick, with sched[g] (an array of
        dtype _abi.MSG_DTYPE or a list of (id, topic, origin, verdict[, vdelay])
        tuples) published in round g.  The heartbeat timer loop,
        gossipsub.go:1320-1343."""
        R = self._msg_cfg.rounds
        g0 = int(tick) * R
        parts, off = [], [0]
        for q in range(int(n_ticks) * R):
            m = (sched or {}).get(g0 + q)
            if m is not None and len(m):
                if not isinstance(m, np.ndarray):
                    arr = np.zeros(len(m), dtype=_abi.MSG_DTYPE)
                    for k, msg in enumerate(m):
                        arr[k]["id"], arr[k]["topic"], arr[k]["origin"], arr[k]["verdict"] = msg[:4]
                        if len(msg) > 4:
                            arr[k]["vdelay"] = msg[4]
                    m = arr
                parts.append(np.ascontiguousarray(m))
            off.append(off[-1] + (len(parts[-1]) if m is not None and len(m) else 0))
        if off[-1]:
            msgs = np.ascontiguousarray(np.concatenate(parts))
            offs = np.asarray(off, dtype=np.int64)
            self._check(self.lib.gsim_step(self.h, int(tick), int(n_ticks), _ptr(msgs), _ptr(offs)))
        else:
            self._check(self.lib.gsim_step(self.h, int(tick), int(n_ticks), None, None))

    def set_peer_behaviour(self, flags: np.ndarray):
        """Per-peer adversarial behaviour (gsim_set_peer_behaviour)."""
        f = np.ascontiguousarray(flags, dtype=np.uint8)
        self._check(self.lib.gsim_set_peer_behaviour(self.h, _ptr(f)))

    def set_connections(self, pairs, up: bool, now: int):
        """Connections (a, b) going down or up between ticks, both endpoints
        notified: the router's and the score tracer's RemovePeer / AddPeer
        (gsim_set_connections; gossipsub.go:525-567, score.go:595-644)."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        self._check(self.lib.gsim_set_connections(self.h, _ptr(p), int(p.shape[0]), 1 if up else 0, int(now)))

    def set_subscriptions(self, pairs, join: bool, tick: int, now: int):
        """Join (join=True) or Leave the (peer, topic) pairs between ticks
        (gsim_set_subscriptions; gossipsub.go:1047-1124, pubsub.go:1051-1079),
        before the refresh of `tick`."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        self._check(self.lib.gsim_set_subscriptions(self.h, _ptr(p), int(p.shape[0]), 1 if join else 0, int(tick),
                                                    int(now)))

    def set_peer_gater(self, params, topic_weights=None):
        """WithPeerGater (peer_gater.go:161-186) on every router (gsim_set_peer_gater):
        params is a gsim.PeerGaterParams; its TopicDeliveryWeights (topic index ->
        weight) unless topic_weights ([T]) is given."""
        c = params.to_c()
        T = max(1, len(self.topics))
        w = np.zeros(T, dtype=np.float64)
        for t, x in (params.TopicDeliveryWeights or {}).items():
            w[int(t)] = float(x)
        if topic_weights is not None:
            w = np.ascontiguousarray(topic_weights, dtype=np.float64)
        self._check(self.lib.gsim_set_peer_gater(self.h, ctypes.byref(c), _ptr(w)))

    def gater_throttled(self) -> int:
        """Message copies the peer gater dropped (AcceptControl) so far."""
        n = ctypes.c_int64(0)
        self._check(self.lib.gsim_gater_throttled(self.h, ctypes.byref(n)))
        return n.value

    def gater_read(self) -> dict:
        """The peer gater's state (gsim_gater_read): validate / throttle / last per
        router, and per connection (edge order) the IP group's counters
        [deliver, duplicate, ignore, reject], connected and expire at the group's
        representative position."""
        N, E = self.net.n, self.net.e
        out = {"validate": np.zeros(N), "throttle": np.zeros(N), "last": np.zeros(N, dtype=np.int64),
               "counters": np.zeros((4, E)), "connected": np.zeros(E, dtype=np.int32),
               "expire": np.zeros(E, dtype=np.int64)}
        self._check(self.lib.gsim_gater_read(self.h, _ptr(out["validate"]), _ptr(out["throttle"]), _ptr(out["last"]),
                                             _ptr(out["counters"]), _ptr(out["connected"]), _ptr(out["expire"])))
        return out

    def px_connect(self, now: int, want_pairs: bool = True):
        """The connector for the attempts peer exchange queued this tick
        (gsim_px_connect; pxConnect gossipsub.go:893-973): returns the
        (dialer, peer) pairs that became connections, sorted (want_pairs
        False: only their number, nothing read back or sorted)."""
        n = ctypes.c_int64(0)
        if not want_pairs:
            self._check(self.lib.gsim_px_connect(self.h, int(now), None, 0, ctypes.byref(n)))
            return n.value
        cap = max(1, self.net.e // 2)
        out = np.zeros((cap, 2), dtype=np.uint32)
        self._check(self.lib.gsim_px_connect(self.h, int(now), _ptr(out), int(cap), ctypes.byref(n)))
        return out[:min(n.value, cap)].copy()

    # gsim_trace_event
    TRACE_DTYPE = np.dtype([("timestamp", np.int64), ("msg_id", np.uint64), ("peer", np.uint32),
                            ("other", np.uint32), ("topic", np.int32), ("type", np.uint8), ("reason", np.uint8),
                            ("_pad", np.uint16)])

    def trace_config(self, peer_lo: int, peer_hi: int, cap: int = 1 << 20):
        """Trace the routers [peer_lo, peer_hi) (gsim_trace_config; cap 0 stops)."""
        self._check(self.lib.gsim_trace_config(self.h, int(peer_lo), int(peer_hi), int(cap)))

    def trace_read(self) -> np.ndarray:
        """The traced events since the last read, sorted (gsim_trace_read):
        the pubsubTracer events of trace.go:70-530 as TRACE_DTYPE records."""
        n = ctypes.c_int64(0)
        self._check(self.lib.gsim_trace_read(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=self.TRACE_DTYPE)
        self._check(self.lib.gsim_trace_read(self.h, _ptr(out) if n.value else None, n.value, ctypes.byref(n)))
        return out[:n.value]

    def set_direct_peers(self, flags):
        """WithDirectPeers as per-edge flags (edge order; None clears)
        (gsim_set_direct_peers; gossipsub.go:352-374)."""
        if flags is None:
            self._check(self.lib.gsim_set_direct_peers(self.h, None))
            return
        f = np.ascontiguousarray(flags, dtype=np.uint8)
        if f.shape != (self.net.e,):
            raise ValueError("direct flags: one byte per edge")
        self._check(self.lib.gsim_set_direct_peers(self.h, _ptr(f)))

    def gossip_stats(self) -> dict:
        out = np.zeros(4, dtype=np.int64)
        self._check(self.lib.gsim_gossip_stats(self.h, _ptr(out)))
        return dict(zip(["ihave_walks", "iwant_ids", "iwant_responses", "broken_promises"], (int(x) for x in out)))

    def msg_stats(self) -> list:
        out = np.zeros(4, dtype=np.int64)
        self._check(self.lib.gsim_msg_stats(self.h, _ptr(out)))
        return [int(x) for x in out]

    def read(self, f: int) -> np.ndarray:
        out = np.empty(self.field_shape(f), dtype=_FIELD_DTYPES[f])
        self._check(self.lib.gsim_read_field(self.h, f, _ptr(out), out.nbytes))
        return out

    def write(self, f: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr, dtype=_FIELD_DTYPES[f]).reshape(self.field_shape(f))
        self._check(self.lib.gsim_write_field(self.h, f, _ptr(a), a.nbytes))

    # -- timing on the engine stream ----------------------------------------------
    def event_record(self, slot: int):
        self._check(self.lib.gsim_event_record(self.h, slot))

    def event_elapsed_ms(self, a: int, b: int) -> float:
        ms = ctypes.c_float()
        self._check(self.lib.gsim_event_elapsed(self.h, a, b, ctypes.byref(ms)))
        return float(ms.value)

    def synchronize(self):
        self._check(self.lib.gsim_synchronize(self.h))

    def profile(self, enable: bool = True):
        """Record per-kernel-class device time with HIP events (gsim_profile)."""
        self._check(self.lib.gsim_profile(self.h, int(bool(enable))))

    def profile_read(self) -> dict:
        """{class: (ms, launches)} since the last read (synchronizes)."""
        n = len(_abi.KERNEL_CLASSES)
        ms = np.zeros(n, dtype=np.float64)
        cnt = np.zeros(n, dtype=np.int64)
        self._check(self.lib.gsim_profile_read(self.h, _ptr(ms), _ptr(cnt), n))
        return {c: (float(ms[i]), int(cnt[i])) for i, c in enumerate(_abi.KERNEL_CLASSES)}

    def set_kernel_variant(self, which: int, variant: int):
        self._check(self.lib.gsim_set_kernel_variant(self.h, which, variant))
