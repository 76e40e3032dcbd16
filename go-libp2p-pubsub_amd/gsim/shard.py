"""Graph sharding over several GPUs.

The reference runs one router per host and moves RPCs over libp2p streams
(gossipsub.go:1138-1202 sendRPC).  Here one simulated network is split into
contiguous peer ranges, one per shard; each shard is an engine over a local
graph of its owned rows plus ghost rows (a remote neighbour's connections
into the shard), and the halo exchange between rounds carries message copies,
GRAFT/PRUNE records and gossip marks.  This module holds the host-side
bookkeeping (partition, local graphs, global <-> local views); the exchange
itself runs in libgsim.so (gsim_group_*).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _abi
from .engine import GsimError, Network, _ptr


def partition(net: Network, shards: int) -> np.ndarray:
    """gsim_shard_partition: contiguous peer ranges balanced by row length x
    joined topics; interior bounds are multiples of 64."""
    lib = _abi.load()
    b = np.zeros(shards + 1, dtype=np.int64)
    rc = lib.gsim_shard_partition(net.n, _ptr(net.row_ptr), _ptr(net.sub), shards, _ptr(b))
    if rc != 0:
        raise GsimError(rc, f"cannot split {net.n} peers into {shards} shards")
    return b


@dataclass
class ShardPlan:
    """One shard's local graph and its exchange bookkeeping (gsim_shard_layout)."""
    shard: int
    shards: int
    bounds: np.ndarray
    gid: np.ndarray            # uint32 [n_local] global id of each local peer, ascending
    row_ptr: np.ndarray        # uint32 [n_local + 1]
    col: np.ndarray            # uint32 [e_local]
    gidx: np.ndarray           # uint64 [e_local] global edge index of each local edge
    own_lo: int
    own_hi: int
    own_e_lo: int
    own_e_hi: int
    ghost_base: np.ndarray     # int64 [shards]
    ghost_count: np.ndarray    # int64 [shards]
    cross_out: List[np.ndarray]   # [shards] owned-row edges into each shard, edge order

    @property
    def n_local(self) -> int:
        return len(self.gid)

    @property
    def e_local(self) -> int:
        return len(self.col)

    @classmethod
    def build(cls, net: Network, bounds: np.ndarray, shard: int) -> "ShardPlan":
        lib = _abi.load()
        K = len(bounds) - 1
        b = np.ascontiguousarray(bounds, dtype=np.int64)
        info = _abi.CShardInfo()
        rc = lib.gsim_shard_layout_info(net.n, _ptr(net.row_ptr), _ptr(net.col), _ptr(b), K, shard,
                                        ctypes.byref(info))
        if rc != 0:
            raise GsimError(rc, "gsim_shard_layout_info")
        gid = np.empty(info.n_local, dtype=np.uint32)
        rp = np.empty(info.n_local + 1, dtype=np.uint32)
        col = np.empty(info.e_local, dtype=np.uint32)
        gidx = np.empty(info.e_local, dtype=np.uint64)
        gb = np.zeros(K, dtype=np.int64)
        gc = np.zeros(K, dtype=np.int64)
        xo = np.empty(max(1, info.n_cross), dtype=np.uint32)
        xc = np.zeros(K, dtype=np.int64)
        rc = lib.gsim_shard_layout(net.n, _ptr(net.row_ptr), _ptr(net.col), _ptr(b), K, shard, _ptr(gid), _ptr(rp),
                                   _ptr(col), _ptr(gidx), _ptr(gb), _ptr(gc), _ptr(xo), _ptr(xc))
        if rc != 0:
            raise GsimError(rc, "gsim_shard_layout")
        offs = np.concatenate([[0], np.cumsum(xc)])
        cross = [xo[offs[s]:offs[s + 1]].copy() for s in range(K)]
        return cls(shard, K, b, gid, rp, col, gidx, int(info.own_lo), int(info.own_hi), int(info.own_e_lo),
                   int(info.own_e_hi), gb, gc, cross)

    # -- global <-> local views -------------------------------------------------
    def local_network(self, net: Network) -> Network:
        """The shard's local graph as a Network: the global per-peer and
        per-edge inputs (subscriptions, outbound flags, IPs) gathered."""
        ip_ptr = ip_ids = None
        if net.ip_ptr is not None:
            lens = np.diff(net.ip_ptr.astype(np.int64))[self.gid]
            ip_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
            starts = net.ip_ptr[self.gid].astype(np.int64)
            idx = np.repeat(starts - ip_ptr[:-1].astype(np.int64), lens) + np.arange(int(lens.sum()))
            ip_ids = np.ascontiguousarray(net.ip_ids[idx], dtype=np.uint32)
        return Network(self.n_local, self.row_ptr, self.col, np.ascontiguousarray(net.outbound[self.gidx]),
                       np.ascontiguousarray(net.sub[self.gid]), ip_ptr, ip_ids, net.n_ips)

    def edge_view(self, arr: np.ndarray) -> np.ndarray:
        """Local edge-order view [..., e_local] of a global [..., E] array."""
        return np.ascontiguousarray(arr[..., self.gidx])

    def peer_view(self, arr: np.ndarray, axis: int = -1) -> np.ndarray:
        """Local per-peer view of a global per-peer array."""
        return np.ascontiguousarray(np.take(arr, self.gid.astype(np.int64), axis=axis))

    def global_edges(self) -> slice:
        """Global edge range of the owned rows (contiguous, same order)."""
        return slice(int(self.gidx[self.own_e_lo]) if self.own_e_hi > self.own_e_lo else 0,
                     int(self.gidx[self.own_e_hi - 1]) + 1 if self.own_e_hi > self.own_e_lo else 0)

    def owned_edges(self, arr: np.ndarray) -> np.ndarray:
        """The owned rows' slice [..., own_e_lo:own_e_hi] of a local edge array."""
        return arr[..., self.own_e_lo:self.own_e_hi]

    def owned_peers(self, arr: np.ndarray, axis: int = -1) -> np.ndarray:
        sl = [slice(None)] * arr.ndim
        sl[axis] = slice(self.own_lo, self.own_hi)
        return arr[tuple(sl)]


def plan(net: Network, shards: int, bounds: Optional[np.ndarray] = None) -> List[ShardPlan]:
    """Partition `net` and build every shard's local graph."""
    b = partition(net, shards) if bounds is None else np.asarray(bounds, dtype=np.int64)
    return [ShardPlan.build(net, b, s) for s in range(len(b) - 1)]


class HostCollectives:
    """gsim_host_transport over a torch.distributed process group (gloo on
    host tensors): the exchanges of a one-shard-per-process group staged
    through host memory (gsim_group_create_host).  Keep the object alive as
    long as the group."""

    _DT = {0: np.uint32, 1: np.int32, 2: np.uint64}

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self._a2a = _abi.HOST_A2A(self._alltoallv)
        self._ar = _abi.HOST_ALLREDUCE(self._allreduce)
        self.c = _abi.CHostTransport(None, self._a2a, self._ar)
        self.error = None

    def _alltoallv(self, ctx, send, sbytes, sdisp, recv, rbytes, rdisp):
        import torch
        try:
            K = self.world
            sb = [int(sbytes[i]) for i in range(K)]
            rb = [int(rbytes[i]) for i in range(K)]
            st, rt = sum(sb), sum(rb)
            s_np = np.ctypeslib.as_array(send, shape=(st,)).copy() if st else np.zeros(0, np.uint8)
            r_t = torch.empty(rt, dtype=torch.uint8)
            self.dist.all_to_all_single(r_t, torch.from_numpy(s_np), rb, sb, group=self.group)
            if rt:
                ctypes.memmove(recv, r_t.numpy().ctypes.data, rt)
            return 0
        except Exception as ex:                 # reported by the group call's error
            self.error = ex
            return 1

    def _allreduce(self, ctx, buf, count, dtype, op):
        import torch
        try:
            dt = self._DT[int(dtype)]
            a = np.ctypeslib.as_array(ctypes.cast(buf, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                      shape=(int(count),))
            t = torch.from_numpy(a.astype(np.int64))
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM if op == 0 else self.dist.ReduceOp.MAX,
                                 group=self.group)
            a[...] = t.numpy().astype(dt)
            return 0
        except Exception as ex:
            self.error = ex
            return 1


class ShardedEngine:
    """One simulated network split over shards (gsim_group_*): the Engine API
    with global peer / edge indexing.  In-process (``shards`` handles in this
    process, device copies between them) or one shard of an RCCL job
    (``rccl=(rank, unique_id, device)``, one process per GPU)."""

    def __init__(self, params, thresholds, gossip=None, topics=None, shards: int = 2, devices=None,
                 rccl=None, host=None):
        """Parameters are validated like WithPeerScore (gossipsub.go:278-319)
        by every shard's gsim_create."""
        from .engine import Engine
        from .params import GossipSubParams
        self.lib = _abi.load()
        self.params = params
        self.thresholds = thresholds
        self.gossip = gossip or GossipSubParams()
        self.topics = sorted(set(topics or []) | set(params.Topics))
        self.topic_index = {t: i for i, t in enumerate(self.topics)}
        self.shards = shards
        pc, tc, gc = params.to_c(), thresholds.to_c(), self.gossip.to_c()
        self._tarr = params.topic_array(self.topics)
        g = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(512)
        if host is not None:
            rank, coll, device = host          # (rank, HostCollectives, device)
            self._coll = coll
            rc = self.lib.gsim_group_create_host(ctypes.byref(pc), self._tarr, len(self.topics), ctypes.byref(tc),
                                                 ctypes.byref(gc), shards, rank, device, ctypes.byref(coll.c),
                                                 ctypes.byref(g), buf, len(buf))
            self.local = [rank]
        elif rccl is None:
            dev = None if devices is None else (ctypes.c_int32 * shards)(*devices)
            rc = self.lib.gsim_group_create(ctypes.byref(pc), self._tarr, len(self.topics), ctypes.byref(tc),
                                            ctypes.byref(gc), shards, dev, ctypes.byref(g), buf, len(buf))
            self.local = list(range(shards))
        else:
            rank, uid, device = rccl
            ub = ctypes.create_string_buffer(bytes(uid), 128)
            rc = self.lib.gsim_group_create_rccl(ctypes.byref(pc), self._tarr, len(self.topics), ctypes.byref(tc),
                                                 ctypes.byref(gc), shards, rank, device, ub, ctypes.byref(g), buf,
                                                 len(buf))
            self.local = [rank]
        if rc != 0:
            raise GsimError(rc, buf.value.decode())
        self.g = g
        self.net: Optional[Network] = None
        self.plans: List[ShardPlan] = []
        self._msg_cfg = None
        self._engine_cls = Engine

    @staticmethod
    def rccl_unique_id() -> bytes:
        lib = _abi.load()
        b = ctypes.create_string_buffer(128)
        rc = lib.gsim_rccl_unique_id(b, 128)
        if rc != 0:
            raise GsimError(rc, "ncclGetUniqueId failed")
        return b.raw

    def close(self):
        if getattr(self, "g", None):
            self.lib.gsim_group_destroy(self.g)
            self.g = None

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
            msg = self.lib.gsim_group_last_error(self.g)
            msg = msg.decode() if msg else ""
            if rc == _abi.GSIM_EINVAL:
                raise ValueError(msg)
            raise GsimError(rc, msg)

    # -- setup ------------------------------------------------------------------------
    def load_graph(self, net: Network, bounds: Optional[np.ndarray] = None):
        b = None if bounds is None else np.ascontiguousarray(bounds, dtype=np.int64)
        self._check(self.lib.gsim_group_load_graph(self.g, net.n, _ptr(net.row_ptr), _ptr(net.col), _ptr(net.outbound),
                                                   _ptr(net.sub), _ptr(net.ip_ptr), _ptr(net.ip_ids), net.n_ips,
                                                   _ptr(b)))
        self.net = net
        self.bounds = np.zeros(self.shards + 1, dtype=np.int64)
        self._check(self.lib.gsim_group_bounds(self.g, _ptr(self.bounds)))
        self.plans = [ShardPlan.build(net, self.bounds, s) for s in self.local]
        if self.params.AppSpecificScore is not None:
            from .engine import app_scores
            self.set_app_score(app_scores(self.params.AppSpecificScore, net.n))

    def set_app_score(self, p5: np.ndarray):
        p5 = np.ascontiguousarray(p5, dtype=np.float64)
        self._check(self.lib.gsim_group_set_app_score(self.g, _ptr(p5)))

    def set_ip_whitelist(self, white: Optional[np.ndarray]):
        w = None if white is None else np.ascontiguousarray(white, dtype=np.uint8)
        self._check(self.lib.gsim_group_set_ip_whitelist(self.g, _ptr(w)))

    def set_direct_peers(self, flags):
        f = None if flags is None else np.ascontiguousarray(flags, dtype=np.uint8)
        self._check(self.lib.gsim_group_set_direct_peers(self.g, _ptr(f)))

    def set_peer_behaviour(self, flags: np.ndarray):
        f = np.ascontiguousarray(flags, dtype=np.uint8)
        self._check(self.lib.gsim_group_set_peer_behaviour(self.g, _ptr(f)))

    def set_topic_score_params(self, topic: str, p):
        c = p.to_c(True)
        self._check(self.lib.gsim_group_set_topic_params(self.g, self.topic_index[topic], ctypes.byref(c)))
        self.params.Topics[topic] = p

    def set_kernel_variant(self, which: int, variant: int):
        """gsim_set_kernel_variant on every shard of this process."""
        for s in self.local:
            h = self._shard_handle(s)
            rc = self.lib.gsim_set_kernel_variant(h, int(which), int(variant))
            if rc != 0:
                raise GsimError(rc, (self.lib.gsim_last_error(h) or b"").decode())

    def set_seed(self, seed: int):
        self._check(self.lib.gsim_group_set_seed(self.g, int(seed)))

    def fill_synthetic(self, seed: int, now: int, p_mesh: float):
        self._check(self.lib.gsim_group_fill_synthetic(self.g, int(seed), int(now), float(p_mesh)))

    # -- hot path -------------------------------------------------------------------
    def msgs_init(self, ring: int, rounds: int, t0: int, heartbeat: Optional[int] = None,
                  max_frontier: Optional[int] = None, max_arrivals: Optional[int] = None,
                  topic_slots: int = 0):
        c = _abi.CMsgConfig()
        c.ring, c.rounds, c.t0_ns = int(ring), int(rounds), int(t0)
        c.heartbeat_ns = int(heartbeat if heartbeat is not None else self.gossip.HeartbeatInterval)
        c.max_frontier = int(max_frontier or 0)      # forwarders one shard exports per round (0: default)
        c.max_arrivals = int(max_arrivals or 0)
        # > 0: per-topic sub-rings of this many slots (ring = n_topics * topic_slots),
        # seen-set cells only for each topic's members (gsim.h gsim_msg_config)
        c.topic_slots = int(topic_slots or 0)
        self._check(self.lib.gsim_group_msgs_init(self.g, ctypes.byref(c)))
        self._msg_cfg = c

    def refresh_scores(self, now: int):
        self._check(self.lib.gsim_group_refresh_scores(self.g, int(now)))

    def heartbeat(self, tick: int, now: int):
        self._check(self.lib.gsim_group_heartbeat(self.g, int(tick), int(now)))

    def publish(self, msgs, rnd: int):
        """As Engine.publish: (id, topic, origin, verdict[, vdelay]) with global origins."""
        arr = np.zeros(len(msgs), dtype=_abi.MSG_DTYPE)
        for k, msg in enumerate(msgs):
            mid, topic, origin, verdict = msg[:4]
            arr[k]["id"], arr[k]["topic"], arr[k]["origin"], arr[k]["verdict"] = mid, topic, origin, verdict
            arr[k]["vdelay"] = msg[4] if len(msg) > 4 else 0
        self.publish_array(arr, rnd)

    def publish_array(self, arr: np.ndarray, rnd: int):
        a = np.ascontiguousarray(arr)
        self._check(self.lib.gsim_group_publish(self.g, _ptr(a), len(a), int(rnd)))

    def round(self, rnd: int):
        self._check(self.lib.gsim_group_round(self.g, int(rnd)))

    def set_connections(self, pairs, up: bool, now: int):
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        self._check(self.lib.gsim_group_set_connections(self.g, _ptr(p), int(p.shape[0]), 1 if up else 0, int(now)))

    def set_ips(self, ip_ptr: np.ndarray, ip_ids: np.ndarray, n_ips: int):
        pp = np.ascontiguousarray(ip_ptr, dtype=np.uint32)
        ii = np.ascontiguousarray(ip_ids, dtype=np.uint32)
        self._check(self.lib.gsim_group_set_ips(self.g, _ptr(pp), _ptr(ii), int(n_ips)))

    def set_subscriptions(self, pairs, join: bool, tick: int, now: int):
        """Join / Leave of (peer, topic) pairs between ticks, over the shards
        (gsim_group_set_subscriptions; every rank passes the same pairs)."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.uint32).reshape(-1, 2))
        self._check(self.lib.gsim_group_set_subscriptions(self.g, _ptr(p), int(p.shape[0]), 1 if join else 0,
                                                          int(tick), int(now)))

    def px_connect(self, now: int, want_pairs: bool = True):
        """The connector over the shards (gsim_group_px_connect; every rank
        calls it): the (dialer, peer) pairs that became connections, sorted
        (want_pairs False: only their number)."""
        n = ctypes.c_int64(0)
        if not want_pairs:
            self._check(self.lib.gsim_group_px_connect(self.g, int(now), None, 0, ctypes.byref(n)))
            return n.value
        cap = max(1, self.net.e // 2)
        out = np.zeros((cap, 2), dtype=np.uint32)
        self._check(self.lib.gsim_group_px_connect(self.g, int(now), _ptr(out), int(cap), ctypes.byref(n)))
        return out[:min(n.value, cap)].copy()

    def set_peer_gater(self, params, topic_weights=None):
        """Engine.set_peer_gater on every shard (gsim_group_set_peer_gater)."""
        c = params.to_c()
        T = max(1, len(self.topics))
        w = np.zeros(T, dtype=np.float64)
        for t, x in (params.TopicDeliveryWeights or {}).items():
            w[int(t)] = float(x)
        if topic_weights is not None:
            w = np.ascontiguousarray(topic_weights, dtype=np.float64)
        self._check(self.lib.gsim_group_set_peer_gater(self.g, ctypes.byref(c), _ptr(w)))

    def gater_throttled(self) -> int:
        """Copies the peer gaters of the whole job dropped so far."""
        n = ctypes.c_int64(0)
        self._check(self.lib.gsim_group_gater_throttled(self.g, ctypes.byref(n)))
        return n.value

    def gater_read(self) -> dict:
        """Engine.gater_read in the whole network's view (gsim_group_gater_read)."""
        N, E = self.net.n, self.net.e
        out = {"validate": np.zeros(N), "throttle": np.zeros(N), "last": np.zeros(N, dtype=np.int64),
               "counters": np.zeros((4, E)), "connected": np.zeros(E, dtype=np.int32),
               "expire": np.zeros(E, dtype=np.int64)}
        self._check(self.lib.gsim_group_gater_read(self.g, _ptr(out["validate"]), _ptr(out["throttle"]),
                                                   _ptr(out["last"]), _ptr(out["counters"]), _ptr(out["connected"]),
                                                   _ptr(out["expire"])))
        return out

    def trace_config(self, peer_lo: int, peer_hi: int, cap: int = 1 << 20):
        """Trace the routers [peer_lo, peer_hi) (global ids) over the shards
        (gsim_group_trace_config; cap 0 stops)."""
        self._check(self.lib.gsim_group_trace_config(self.g, int(peer_lo), int(peer_hi), int(cap)))

    def trace_read(self) -> np.ndarray:
        """Engine.trace_read over the shards of this process, in global ids
        (gsim_group_trace_read)."""
        from .engine import Engine
        n = ctypes.c_int64(0)
        self._check(self.lib.gsim_group_trace_read(self.g, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=Engine.TRACE_DTYPE)
        self._check(self.lib.gsim_group_trace_read(self.g, _ptr(out) if n.value else None, n.value, ctypes.byref(n)))
        return out[:n.value]

    def msg_stats(self) -> list:
        out = np.zeros(4, dtype=np.int64)
        self._check(self.lib.gsim_group_msg_stats(self.g, _ptr(out)))
        return [int(x) for x in out]

    def local_msg_stats(self) -> list:
        """gsim_msg_stats of this process's shards only (deliveries to their peers)."""
        tot = np.zeros(4, dtype=np.int64)
        for s in self.local:
            out = np.zeros(4, dtype=np.int64)
            h = self._shard_handle(s)
            rc = self.lib.gsim_msg_stats(h, _ptr(out))
            if rc != 0:
                raise GsimError(rc, (self.lib.gsim_last_error(h) or b"").decode())
            tot += out
        return [int(x) for x in tot]

    def gossip_stats(self) -> dict:
        out = np.zeros(4, dtype=np.int64)
        self._check(self.lib.gsim_group_gossip_stats(self.g, _ptr(out)))
        return dict(zip(["ihave_walks", "iwant_ids", "iwant_responses", "broken_promises"], (int(x) for x in out)))

    def census(self) -> dict:
        out = np.zeros(8, dtype=np.int64)
        self._check(self.lib.gsim_group_census(self.g, _ptr(out)))
        keys = ["records", "in_mesh", "nz_first", "nz_meshd", "nz_fail", "nz_invalid", "mesh_links", "tracked_edges"]
        return {k: int(v) for k, v in zip(keys, out)}

    def synchronize(self):
        self._check(self.lib.gsim_group_synchronize(self.g))

    def profile(self, enable: bool = True):
        self._check(self.lib.gsim_group_profile(self.g, int(bool(enable))))

    def profile_read(self) -> dict:
        n = len(_abi.KERNEL_CLASSES)
        ms = np.zeros(n, dtype=np.float64)
        cnt = np.zeros(n, dtype=np.int64)
        self._check(self.lib.gsim_group_profile_read(self.g, _ptr(ms), _ptr(cnt), n))
        return {c: (float(ms[i]), int(cnt[i])) for i, c in enumerate(_abi.KERNEL_CLASSES)}

    def profile_read_shards(self) -> list:
        """profile_read of each shard of this process (list in shard order)."""
        n = len(_abi.KERNEL_CLASSES)
        res = []
        for s in self.local:
            ms = np.zeros(n, dtype=np.float64)
            cnt = np.zeros(n, dtype=np.int64)
            h = self._shard_handle(s)
            rc = self.lib.gsim_profile_read(h, _ptr(ms), _ptr(cnt), n)
            if rc != 0:
                raise GsimError(rc, (self.lib.gsim_last_error(h) or b"").decode())
            res.append({c: (float(ms[i]), int(cnt[i])) for i, c in enumerate(_abi.KERNEL_CLASSES)})
        return res

    # -- state in the whole network's view (this process's shards) --------------------
    _PEER_LAST = {_abi.F_SEEN, _abi.F_LASTPUT}          # [..., N]
    _PEER_FIRST = {_abi.F_LASTPUB, _abi.F_FANOUT_TOPICS}   # [N, ...]

    def _shard_handle(self, s: int):
        h = self.lib.gsim_group_shard(self.g, s)
        if not h:
            raise GsimError(_abi.GSIM_EINVAL, f"shard {s} is not in this process")
        return ctypes.c_void_p(h)

    def _shape(self, f: int, n: int, e: int):
        T = max(1, len(self.topics))
        from .engine import PARITY_TOPIC_FIELDS, TOPIC_FIELDS
        if f in PARITY_TOPIC_FIELDS:
            return (2, T, e)
        if f == _abi.F_SEEN:
            return (self._msg_cfg.ring, n)
        if f == _abi.F_LASTPUT:
            return (T, n)
        if f == _abi.F_LASTPUB:
            return (n, T)
        if f == _abi.F_FANOUT_TOPICS:
            return (n,)
        return (T, e) if f in TOPIC_FIELDS else (e,)

    def read_local(self, s: int, f: int) -> np.ndarray:
        """Shard s's field in its local view."""
        from .engine import _FIELD_DTYPES
        p = self.plans[self.local.index(s)]
        out = np.empty(self._shape(f, p.n_local, p.e_local), dtype=_FIELD_DTYPES[f])
        h = self._shard_handle(s)
        rc = self.lib.gsim_read_field(h, f, _ptr(out), out.nbytes)
        if rc != 0:
            raise GsimError(rc, (self.lib.gsim_last_error(h) or b"").decode())
        return out

    def read(self, f: int, into: Optional[np.ndarray] = None) -> np.ndarray:
        """A field of the whole network, assembled from the owned parts of
        every shard by gsim_group_read_field (every shard must be in this
        process).  into: an array of the whole network's shape whose parts
        owned by this process's shards are overwritten (any subset of the
        shards; returned)."""
        from .engine import _FIELD_DTYPES
        if into is None and len(self.local) != self.shards:
            raise GsimError(_abi.GSIM_EINVAL, "the whole network's view needs every shard in this process")
        out = np.zeros(self._shape(f, self.net.n, self.net.e), dtype=_FIELD_DTYPES[f]) if into is None else into
        assert out.flags.c_contiguous and out.dtype == _FIELD_DTYPES[f]
        self._check(self.lib.gsim_group_read_field(self.g, int(f), _ptr(out), out.nbytes))
        return out

    def snapshot(self, obs_lo: int = 0, obs_hi: Optional[int] = None):
        """Engine.snapshot over the whole network (gsim_group_read_snapshot):
        the global observers [obs_lo, obs_hi) of this process's shards."""
        hi = self.net.n if obs_hi is None else obs_hi
        ne = int(self.net.row_ptr[hi]) - int(self.net.row_ptr[obs_lo])
        T = max(1, len(self.topics))
        peers = np.zeros(ne, dtype=_abi.PEER_SNAPSHOT_DTYPE)
        topics = np.zeros((ne, T), dtype=_abi.TOPIC_SNAPSHOT_DTYPE)
        self._check(self.lib.gsim_group_read_snapshot(self.g, int(obs_lo), int(hi), _ptr(peers), _ptr(topics)))
        return peers, topics

    def write(self, f: int, arr: np.ndarray):
        """Install a field given in the whole network's view on every local shard."""
        from .engine import _FIELD_DTYPES
        a = np.asarray(arr, dtype=_FIELD_DTYPES[f]).reshape(self._shape(f, self.net.n, self.net.e))
        for p in self.plans:
            if f in self._PEER_LAST:
                loc = p.peer_view(a, axis=-1)
            elif f in self._PEER_FIRST:
                loc = p.peer_view(a, axis=0)
            else:
                loc = p.edge_view(a)
            h = self._shard_handle(p.shard)
            loc = np.ascontiguousarray(loc)
            rc = self.lib.gsim_write_field(h, f, _ptr(loc), loc.nbytes)
            if rc != 0:
                raise GsimError(rc, (self.lib.gsim_last_error(h) or b"").decode())
        self._check(self.lib.gsim_group_state_written(self.g))

    def scores(self) -> np.ndarray:
        out = np.zeros(self.net.e, dtype=np.float64)
        self._check(self.lib.gsim_group_read_scores(self.g, _ptr(out)))
        return out
