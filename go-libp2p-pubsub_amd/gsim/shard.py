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
