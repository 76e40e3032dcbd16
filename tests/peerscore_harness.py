"""A reference-shaped `peerScore` over the oracle (test infrastructure).

score_test.go builds one peerScore with newPeerScore and drives its RawTracer
methods by hand.  `PeerScore` here is that object, restated on top of the
oracle's SoA layout: the observer is peer 0 of a star network whose other
vertices are the reference test's peers ("A", "B", ...).  Time is a virtual
clock (`self.now`, int ns) so the reference's sleep-based tests become exact.
The same class can drive the HIP engine (`engine=`) for the GPU parity KATs.
"""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_binding as ob
from gsim import _abi
from gsim.engine import Network

T0 = 1_000_000_000_000  # virtual epoch (ns); non-zero so "zero time" stays distinct


def star_network(peers, n_topics, ips=None):
    """Observer 0 connected to every test peer; ips = {peer: [ip strings]}."""
    m = len(peers)
    n = m + 1
    rows = [list(range(1, n))] + [[0] for _ in range(m)]
    row_ptr = np.zeros(n + 1, dtype=np.uint32)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.array([c for r in rows for c in r], dtype=np.uint32)
    outbound = np.zeros(len(col), dtype=np.uint8)
    sub = np.full(n, (1 << n_topics) - 1, dtype=np.uint64)
    ip_ptr = ip_ids = None
    n_ips = 0
    ip_names = []
    if ips is not None:
        ip_names = sorted({ip for lst in ips.values() for ip in lst})
        idx = {ip: i for i, ip in enumerate(ip_names)}
        lists = [[]] + [[idx[ip] for ip in ips.get(p, [])] for p in peers]
        ip_ptr = np.zeros(n + 1, dtype=np.uint32)
        ip_ptr[1:] = np.cumsum([len(lst) for lst in lists])
        ip_ids = np.array([i for lst in lists for i in lst] or [0], dtype=np.uint32)
        n_ips = len(ip_names)
    return Network(n, row_ptr, col, outbound, sub, ip_ptr, ip_ids, n_ips), ip_names


class PeerScore:
    def __init__(self, params, peers=("A", "B", "C", "D"), extra_topics=(), ips=None, seen_ttl=0):
        self.lib = ob.load()
        self.params = params
        self.peers = list(peers)
        self.topics = sorted(set(params.Topics) | set(extra_topics))
        self.net, ip_names = star_network(self.peers, max(1, len(self.topics)), ips)
        white = None
        if params.IPColocationFactorWhitelist and ip_names:
            white = np.array([params.whitelisted(ip) for ip in ip_names], dtype=np.uint8)
        p5 = np.zeros(self.net.n)
        self.st = ob.NetState(self.net, params, topics=self.topics, p5=p5, ip_white=white)
        self.st.estate[:] = 0                     # nobody added yet (newPeerScore)
        self.v = self.st.view()
        self.drecs = self.lib.orc_drecs_new(int(params.SeenMsgTTL))
        self.now = T0

    def __del__(self):
        try:
            self.lib.orc_drecs_free(self.drecs)
        except Exception:
            pass

    # peer name -> edge index in the observer's row
    def e(self, p):
        return self.peers.index(p)

    def t(self, topic):
        return self.topics.index(topic)

    def sleep(self, ns):
        self.now += int(ns)

    # ---- RawTracer / router surface -------------------------------------
    def AddPeer(self, p):
        self.lib.orc_add_peer(self.v, self.e(p))

    def RemovePeer(self, p):
        self._refresh_p5()
        self.lib.orc_ip_colocation(self.v)
        self.lib.orc_remove_peer(self.v, self.e(p), self.now)

    def Graft(self, p, topic):
        self.lib.orc_graft(self.v, self.e(p), self.t(topic), self.now)

    def Prune(self, p, topic):
        self.lib.orc_prune(self.v, self.e(p), self.t(topic))

    def AddPenalty(self, p, count):
        self.lib.orc_add_penalty(self.v, self.e(p), count)

    def refreshScores(self):
        self.lib.orc_refresh_scores(self.v, self.now)

    def _refresh_p5(self):
        f = self.params.AppSpecificScore
        for i, p in enumerate(self.peers):
            self.st.p5[i + 1] = f(p) if f else 0.0

    def Score(self, p):
        self._refresh_p5()
        self.lib.orc_ip_colocation(self.v)
        return self.lib.orc_score_edge(self.v, self.e(p))

    def ValidateMessage(self, msg):
        self.lib.orc_validate_message(self.v, self.drecs, msg.mid, self.now)

    def DeliverMessage(self, msg):
        self.lib.orc_deliver_message(self.v, self.drecs, self.e(msg.ReceivedFrom), msg.mid, self.t(msg.topic),
                                     self.now)

    def RejectMessage(self, msg, reason):
        self.lib.orc_reject_message(self.v, self.drecs, self.e(msg.ReceivedFrom), msg.mid, self.t(msg.topic),
                                    reason, self.now)

    def DuplicateMessage(self, msg):
        self.lib.orc_duplicate_message(self.v, self.drecs, self.e(msg.ReceivedFrom), msg.mid,
                                       self.t(msg.topic), self.now)

    def SetTopicScoreParams(self, topic, p):
        ti = self.t(topic)
        slot = ctypes.cast(ctypes.addressof(self.st.tp) + ti * ctypes.sizeof(_abi.CTopicScoreParams),
                           ctypes.c_void_p)
        newp = p.to_c(True)
        self.lib.orc_set_topic_params(self.v, ti, slot, ctypes.cast(ctypes.byref(newp), ctypes.c_void_p))
        self.params.Topics[topic] = p

    def gc_deliveries(self):
        self.lib.orc_drecs_gc(self.drecs, self.now)

    def expire_head_now(self):
        """ps.deliveries.head.expire = time.Now(); time.Sleep(1ms) (score_test.go:595-596)."""
        self.lib.orc_drecs_expire_head(self.drecs, self.now)
        self.sleep(1_000_000)

    # ---- introspection (ps.peerStats[p].topics[t].field) -------------------
    def topic_stat(self, p, topic, field):
        return getattr(self.st, field)[self.t(topic), self.e(p)]


class Msg:
    """makeTestMessage(i) with a topic and ReceivedFrom (mcache_test.go:156-167)."""

    def __init__(self, i, topic, frm):
        self.mid = int(i)
        self.topic = topic
        self.ReceivedFrom = frm
