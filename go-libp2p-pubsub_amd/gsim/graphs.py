"""Synthetic peer graphs and subscriptions for the SURVEY.md §8 configurations.

The reference builds its test networks from libp2p hosts (`getDefaultHosts`,
`denseConnect`, `connectSome` in floodsub_test.go / gossipsub_test.go); the
engine needs a CSR peer graph instead.  These generators are host-side setup
(seeded numpy), not part of the hot path:

* `power_law`     Chung-Lu graph with expected degrees from a power law
                  (C5: exponent 2.5, mean ~16), rows capped at `max_degree`
                  (the wave-per-row kernels take rows of at most 64);
* `zipf_subscriptions`  each peer joins ~`per_peer` of T topics with Zipf
                  topic popularity (C5: 64 topics, ~8 per peer);
* `sybil_ips`     honest peers on unique IPs, a fraction of sybils sharing one
                  IP per `per_ip` (C4: 20 % sybils, 50 per IP).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .engine import Network


def _csr_from_pairs(n: int, u: np.ndarray, v: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Symmetric CSR with sorted rows from undirected pairs (u dialed v)."""
    src = np.concatenate([u, v]).astype(np.int64)
    dst = np.concatenate([v, u]).astype(np.int64)
    out = np.concatenate([np.ones(len(u), np.uint8), np.zeros(len(v), np.uint8)])
    order = np.lexsort((dst, src))
    src, dst, out = src[order], dst[order], out[order]
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    np.add.at(row_ptr, src + 1, 1)
    row_ptr = np.cumsum(row_ptr).astype(np.uint32)
    return row_ptr, dst.astype(np.uint32), out


def power_law(n: int, mean_degree: float = 16.0, exponent: float = 2.5, max_degree: int = 64,
              seed: int = 1, n_topics: int = 1, i0: float = None) -> Network:
    """Chung-Lu random graph: expected degree of peer i proportional to
    (i + i0)^(-1/(exponent-1)), scaled to `mean_degree`, at most `max_degree`
    connections per peer.  Every peer joins every topic (see
    zipf_subscriptions).  i0 (default n/1000) flattens the head: the largest
    expected degree is about mean * (exponent-2)/(exponent-1) * (n/i0)^(1/(exponent-1)),
    so i0 = 1 gives the plain Chung-Lu hubs (capped at max_degree)."""
    rng = np.random.default_rng(seed)
    i0 = max(1.0, n / 1000.0) if i0 is None else float(i0)
    w = (np.arange(n, dtype=np.float64) + i0) ** (-1.0 / (exponent - 1.0))
    w *= mean_degree * n / w.sum()
    w = np.minimum(w, max_degree)
    m = int(round(w.sum() / 2))
    p = w / w.sum()
    u = rng.choice(n, size=m, p=p)
    v = rng.choice(n, size=m, p=p)
    keep = u != v
    u, v = u[keep], v[keep]
    a, b = np.minimum(u, v), np.maximum(u, v)
    key = a.astype(np.int64) * n + b
    _, first = np.unique(key, return_index=True)
    first = np.sort(first)                       # keep the sampling order for the cap below
    u, v = u[first], v[first]
    # cap the degree: edges are accepted in sampling order while both ends have room
    deg = np.zeros(n, dtype=np.int64)
    ok = np.zeros(len(u), dtype=bool)
    # vectorised in passes: each pass accepts the edges whose endpoints stay under the cap
    pend = np.arange(len(u))
    while len(pend):
        uu, vv = u[pend], v[pend]
        # rank of each pending edge among all pending edges at the same peer
        r = _rank_within(np.concatenate([uu, vv]))
        ru, rv = r[:len(uu)], r[len(uu):]
        acc = (deg[uu] + ru < max_degree) & (deg[vv] + rv < max_degree)
        # at most `room` edges of a peer have a rank below its room, so the cap holds
        if not acc.any():
            break
        ok[pend[acc]] = True
        np.add.at(deg, uu[acc], 1)
        np.add.at(deg, vv[acc], 1)
        room = (deg[uu] < max_degree) & (deg[vv] < max_degree)
        pend = pend[~acc & room]
    u, v = u[ok], v[ok]
    row_ptr, col, outbound = _csr_from_pairs(n, u, v)
    mask = (1 << n_topics) - 1 if n_topics < 64 else (1 << 64) - 1
    sub = np.full(n, mask, dtype=np.uint64)
    ip_ptr = np.arange(n + 1, dtype=np.uint32)
    ip_ids = np.arange(n, dtype=np.uint32)
    return Network(n, row_ptr, col, outbound, sub, ip_ptr, ip_ids, n)


def power_law_native(n: int, mean_degree: float = 16.0, exponent: float = 2.5, max_degree: int = 4096,
                     seed: int = 1, n_topics: int = 1, i0: float = None) -> Network:
    """The Chung-Lu model of `power_law` drawn by the library's C++ generator
    (gsim_gen_power_law: the same distribution from its own seeded stream,
    seconds at 10M peers where the numpy one takes minutes)."""
    import ctypes
    from . import _abi
    lib = _abi.load()
    i0 = max(1.0, n / 1000.0) if i0 is None else float(i0)
    ne = ctypes.c_int64(0)
    rc = lib.gsim_gen_power_law(n, float(mean_degree), float(exponent), int(max_degree), i0, int(seed),
                                None, None, None, ctypes.byref(ne))
    if rc != 0:
        raise RuntimeError(f"gsim_gen_power_law failed ({rc})")
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    col = np.zeros(ne.value, dtype=np.uint32)
    out = np.zeros(ne.value, dtype=np.uint8)
    rc = lib.gsim_gen_power_law(n, float(mean_degree), float(exponent), int(max_degree), i0, int(seed),
                                row_ptr.ctypes.data, col.ctypes.data, out.ctypes.data, ctypes.byref(ne))
    if rc != 0:
        raise RuntimeError(f"gsim_gen_power_law failed ({rc})")
    mask = (1 << n_topics) - 1 if n_topics < 64 else (1 << 64) - 1
    sub = np.full(n, mask, dtype=np.uint64)
    ip_ptr = np.arange(n + 1, dtype=np.uint32)
    ip_ids = np.arange(n, dtype=np.uint32)
    return Network(n, row_ptr, col, out, sub, ip_ptr, ip_ids, n)


def _rank_within(keys: np.ndarray) -> np.ndarray:
    """0-based rank of each element among the equal keys, in array order."""
    order = np.argsort(keys, kind="stable")
    k = keys[order]
    start = np.r_[0, np.nonzero(k[1:] != k[:-1])[0] + 1]
    run = np.repeat(start, np.diff(np.r_[start, len(k)]))
    rank = np.empty(len(keys), dtype=np.int64)
    rank[order] = np.arange(len(k)) - run
    return rank


def zipf_subscriptions(n: int, n_topics: int, per_peer: int = 8, s: float = 1.0, seed: int = 1) -> np.ndarray:
    """Each peer joins `per_peer` distinct topics drawn by Zipf(s) popularity
    (Gumbel top-k).  Returns the u64 subscription masks."""
    rng = np.random.default_rng(seed)
    logw = -s * np.log(np.arange(1, n_topics + 1, dtype=np.float64))
    sub = np.zeros(n, dtype=np.uint64)
    k = min(per_peer, n_topics)
    for lo in range(0, n, 1 << 16):
        hi = min(n, lo + (1 << 16))
        g = logw[None, :] - np.log(-np.log(rng.random((hi - lo, n_topics))))
        top = np.argpartition(-g, k - 1, axis=1)[:, :k]
        bits = (np.uint64(1) << top.astype(np.uint64))
        sub[lo:hi] = np.bitwise_or.reduce(bits, axis=1)
    return sub


def sybil_ips(n: int, frac: float, per_ip: int, seed: int = 1) -> Tuple[np.ndarray, np.ndarray, int, np.ndarray]:
    """Honest peers get a unique IP; a random `frac` of peers (the sybils)
    share one IP per `per_ip`.  Returns (ip_ptr, ip_ids, n_ips, is_sybil)."""
    rng = np.random.default_rng(seed)
    ip_of = np.arange(n, dtype=np.int64)
    syb = rng.permutation(n)[: int(n * frac)]
    ip_of[syb] = n + (np.arange(len(syb)) // per_ip)
    ips, inv = np.unique(ip_of, return_inverse=True)
    is_sybil = np.zeros(n, dtype=bool)
    is_sybil[syb] = True
    return np.arange(n + 1, dtype=np.uint32), inv.astype(np.uint32), len(ips), is_sybil


def with_subscriptions(net: Network, sub: np.ndarray) -> Network:
    return Network(net.n, net.row_ptr, net.col, net.outbound, np.ascontiguousarray(sub, dtype=np.uint64),
                   net.ip_ptr, net.ip_ids, net.n_ips)


def with_ips(net: Network, ip_ptr: np.ndarray, ip_ids: np.ndarray, n_ips: int) -> Network:
    return Network(net.n, net.row_ptr, net.col, net.outbound, net.sub, ip_ptr, ip_ids, n_ips)
