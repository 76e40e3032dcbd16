"""Graph sharding bookkeeping on the CPU (no GPU needed): the partition, every
shard's local graph, and the index translations the halo exchange relies on
(DESIGN.md §5).  The world_size-2 test runs two processes over torch.distributed
(gloo) that each build only their own shard and exchange copies, control
records and gossip marks the way the engine's transports do, checking that
every entry lands on the record / edge of the same global connection."""
import os

import numpy as np
import pytest

from gsim import graphs, shard
from gsim.engine import Network, random_regular


def _weights(net):
    """gsim_shard_partition's peer weight (shard_plan.cpp): per joined topic the
    row length, 16 for the observer's lane group, d^2 / 512 for a hub row."""
    d = np.diff(net.row_ptr.astype(np.int64)).astype(np.float64)
    s = np.array([bin(int(x)).count("1") for x in net.sub], dtype=np.float64)
    hub = np.where(d > 64, d * d / 512.0, 0.0)
    return np.maximum(s, 1) * (d + 16.0 + hub) + 1.0


@pytest.mark.parametrize("K", [1, 2, 3, 4, 8])
def test_partition_balanced_word_aligned(K):
    net = graphs.power_law(20_000, 16, 2.5, 256, seed=3, n_topics=16)
    net = graphs.with_subscriptions(net, graphs.zipf_subscriptions(net.n, 16, 4, seed=5))
    b = shard.partition(net, K)
    assert b[0] == 0 and b[-1] == net.n and (np.diff(b) > 0).all()
    assert (b[1:-1] % 64 == 0).all()
    w = _weights(net)
    per = np.array([w[b[s]:b[s + 1]].sum() for s in range(K)])
    assert per.max() <= per.mean() * 1.02 + w.max() + 64 * w.max()


def _check_plans(net, plans):
    K = len(plans)
    rev_g = net.rev()
    owner_g = net.owner()
    for p in plans:
        loc = Network(p.n_local, p.row_ptr, p.col, np.zeros(p.e_local, np.uint8), np.zeros(p.n_local, np.uint64))
        own = loc.owner()
        assert (np.diff(p.gid.astype(np.int64)) > 0).all(), "local ids keep the global order"
        assert (p.col[loc.rev()] == own).all(), "the local graph is symmetric"
        g_own, g_col = p.gid[own].astype(np.int64), p.gid[p.col].astype(np.int64)
        assert (owner_g[p.gidx] == g_own).all() and (net.col[p.gidx] == g_col).all(), "gidx names the same edge"
        lo, hi = p.bounds[p.shard], p.bounds[p.shard + 1]
        assert (p.gid[p.own_lo:p.own_hi] == np.arange(lo, hi)).all()
        sl = p.global_edges()
        assert (p.gidx[p.own_e_lo:p.own_e_hi] == np.arange(sl.start, sl.stop)).all(), "owned rows are whole rows"
        ghost = np.ones(p.n_local, bool)
        ghost[p.own_lo:p.own_hi] = False
        gedges = ghost[own]
        assert ((p.col[gedges] >= p.own_lo) & (p.col[gedges] < p.own_hi)).all(), "ghost rows hold owned peers only"
        # record order: every record an owned observer keeps is local
        assert (p.gidx[loc.rev()] == rev_g[p.gidx]).all()
    for a in range(K):
        for b in range(K):
            if a == b:
                continue
            pa, pb = plans[a], plans[b]
            xo = pa.cross_out[b]
            assert len(xo) == pb.ghost_count[a]
            # copies / gossip marks a -> b: cross-out q is b's edge ghost_base[a] + q
            assert (pa.gidx[xo] == pb.gidx[pb.ghost_base[a] + np.arange(len(xo))]).all()
            # control a -> b: a's ghost-row edge ghost_base[b] + q is b's cross-out q
            qb = np.arange(pa.ghost_count[b])
            assert (pa.gidx[pa.ghost_base[b] + qb] == pb.gidx[pb.cross_out[a][qb]]).all()


@pytest.mark.parametrize("K", [2, 3, 4])
def test_layouts_random_regular(K):
    net = random_regular(6000, 32, seed=11, n_topics=4)
    _check_plans(net, shard.plan(net, K))


def test_layouts_power_law_hubs():
    net = graphs.power_law(8000, 16, 2.5, 512, seed=7, n_topics=8)
    _check_plans(net, shard.plan(net, 4))


def test_local_network_inputs():
    net = graphs.power_law(3000, 12, 2.5, 64, seed=2, n_topics=8)
    ip_ptr, ip_ids, n_ips, _ = graphs.sybil_ips(net.n, 0.2, 10, seed=4)
    net = graphs.with_ips(net, ip_ptr, ip_ids, n_ips)
    for p in shard.plan(net, 3):
        ln = p.local_network(net)
        assert (ln.sub == net.sub[p.gid]).all()
        assert (ln.outbound == net.outbound[p.gidx]).all()
        for l in range(0, p.n_local, 37):
            g = p.gid[l]
            assert (ln.ip_ids[ln.ip_ptr[l]:ln.ip_ptr[l + 1]] == net.ip_ids[net.ip_ptr[g]:net.ip_ptr[g + 1]]).all()


# ---- world_size 2 over gloo: each rank builds only its own shard -----------------

def _exchange(dist, torch, send_lists, K):
    """all_to_all of int64 arrays (one list per destination)."""
    cnt = torch.tensor([len(x) for x in send_lists], dtype=torch.int64)
    rcnt = torch.zeros(K, dtype=torch.int64)
    dist.all_to_all_single(rcnt, cnt)
    send = torch.from_numpy(np.concatenate(send_lists).astype(np.int64)) if sum(len(x) for x in send_lists) \
        else torch.zeros(0, dtype=torch.int64)
    recv = torch.zeros(int(rcnt.sum()), dtype=torch.int64)
    dist.all_to_all_single(recv, send, [int(x) for x in rcnt], [int(x) for x in cnt])
    out, off = [], 0
    for s in range(K):
        out.append(recv[off:off + int(rcnt[s])].numpy())
        off += int(rcnt[s])
    return out


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        net = random_regular(4000, 24, seed=21, n_topics=2)
        b = shard.partition(net, world)
        p = shard.ShardPlan.build(net, b, rank)
        gid = p.gid.astype(np.int64)
        loc = Network(p.n_local, p.row_ptr, p.col, np.zeros(p.e_local, np.uint8), np.zeros(p.n_local, np.uint64))
        own = loc.owner()
        # 1. copy push (shard.hip exchange_copies): each shard learns where its
        # ghost block starts at every other shard (gsim_group_load_graph's count
        # exchange), then sends a copy over every cross edge as the edge's index
        # at the receiver's shard (xre = rbase[d] + cross-out position), with
        # (sender gid, receiver gid) to check it against
        rbase = _exchange(dist, torch, [np.array([p.ghost_base[d] if d != rank else 0]) for d in range(world)],
                          world)
        sends = []
        for d in range(world):
            xo = p.cross_out[d] if d != rank else np.zeros(0, np.uint32)
            xre = (int(rbase[d][0]) if d != rank else 0) + np.arange(len(xo))
            sends.append(np.stack([xre, gid[own[xo]], gid[p.col[xo]]], 1).ravel())
        got = _exchange(dist, torch, sends, world)
        n_copies = 0
        for s in range(world):
            if s == rank:
                continue
            e = got[s].reshape(-1, 3)
            r = e[:, 0]                                    # the receiver's record of the sender
            assert (gid[own[r]] == e[:, 1]).all() and (gid[p.col[r]] == e[:, 2]).all()
            assert ((p.col[r] >= p.own_lo) & (p.col[r] < p.own_hi)).all(), "lands on an owned receiver"
            n_copies += len(e)
        # 2. control records from ghost rows: (ghost-block index q, sender gid, receiver gid)
        sends = []
        for d in range(world):
            if d == rank:
                sends.append(np.zeros(0, np.int64))
                continue
            x = p.ghost_base[d] + np.arange(p.ghost_count[d])
            sends.append(np.stack([x - p.ghost_base[d], gid[p.col[x]], gid[own[x]]], 1).ravel())
        got = _exchange(dist, torch, sends, world)
        for s in range(world):
            if s == rank:
                continue
            e = got[s].reshape(-1, 3)
            idx = p.cross_out[s][e[:, 0]]                  # the receiver's own edge to the sender
            assert (gid[own[idx]] == e[:, 2]).all() and (gid[p.col[idx]] == e[:, 1]).all()
        q.put((rank, n_copies, None))
        dist.destroy_process_group()
    except Exception as ex:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, -1, traceback.format_exc() + str(ex)))


def test_two_ranks_gloo_exchange_bookkeeping():
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    for rank, n, err in res:
        assert err is None, err
        assert n > 0
