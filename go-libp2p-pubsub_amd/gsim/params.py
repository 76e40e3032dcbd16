"""Reference-shaped parameter API (score_params.go, gossipsub.go).

Field names are the Go field names, durations are integer nanoseconds
(``Second``/``Millisecond`` mirror Go's ``time`` constants), and ``validate()``
raises ``ValueError`` carrying the reference's error text.  Validation is
executed by the engine library (csrc/params.cpp), the same code gsim_create
runs, so Python and the C ABI cannot disagree.
"""
from __future__ import annotations

import ctypes
import ipaddress
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from . import _abi

Nanosecond = 1
Microsecond = 1000
Millisecond = 1000 * Microsecond
Second = 1000 * Millisecond
Minute = 60 * Second
Hour = 60 * Minute

DefaultDecayInterval = Second          # score_params.go:401
DefaultDecayToZero = 0.01              # score_params.go:402
TimeCacheDuration = 120 * Second       # pubsub.go:32


@dataclass
class TopicScoreParams:
    """TopicScoreParams, score_params.go:117-170."""
    SkipAtomicValidation: bool = False
    TopicWeight: float = 0.0
    TimeInMeshWeight: float = 0.0
    TimeInMeshQuantum: int = 0
    TimeInMeshCap: float = 0.0
    FirstMessageDeliveriesWeight: float = 0.0
    FirstMessageDeliveriesDecay: float = 0.0
    FirstMessageDeliveriesCap: float = 0.0
    MeshMessageDeliveriesWeight: float = 0.0
    MeshMessageDeliveriesDecay: float = 0.0
    MeshMessageDeliveriesCap: float = 0.0
    MeshMessageDeliveriesThreshold: float = 0.0
    MeshMessageDeliveriesWindow: int = 0
    MeshMessageDeliveriesActivation: int = 0
    MeshFailurePenaltyWeight: float = 0.0
    MeshFailurePenaltyDecay: float = 0.0
    InvalidMessageDeliveriesWeight: float = 0.0
    InvalidMessageDeliveriesDecay: float = 0.0

    def to_c(self, scored: bool = True) -> _abi.CTopicScoreParams:
        return _abi.CTopicScoreParams(
            int(self.SkipAtomicValidation), int(scored), self.TopicWeight,
            self.TimeInMeshWeight, int(self.TimeInMeshQuantum), self.TimeInMeshCap,
            self.FirstMessageDeliveriesWeight, self.FirstMessageDeliveriesDecay, self.FirstMessageDeliveriesCap,
            self.MeshMessageDeliveriesWeight, self.MeshMessageDeliveriesDecay, self.MeshMessageDeliveriesCap,
            self.MeshMessageDeliveriesThreshold, int(self.MeshMessageDeliveriesWindow),
            int(self.MeshMessageDeliveriesActivation),
            self.MeshFailurePenaltyWeight, self.MeshFailurePenaltyDecay,
            self.InvalidMessageDeliveriesWeight, self.InvalidMessageDeliveriesDecay)

    def validate(self) -> None:
        """score_params.go:236-267."""
        buf = ctypes.create_string_buffer(512)
        c = self.to_c()
        if _abi.load().gsim_validate_topic_params(ctypes.byref(c), buf, len(buf)) != 0:
            raise ValueError(buf.value.decode())


@dataclass
class PeerScoreParams:
    """PeerScoreParams, score_params.go:66-115.

    ``AppSpecificScore`` is called once per peer index when the engine needs
    the P5 array (the Go callback is replaced by a host-refreshed array at the
    C boundary).  ``IPColocationFactorWhitelist`` holds ``ipaddress`` networks.
    """
    SkipAtomicValidation: bool = False
    Topics: Dict[str, TopicScoreParams] = field(default_factory=dict)
    TopicScoreCap: float = 0.0
    AppSpecificScore: Optional[Callable[[int], float]] = None
    AppSpecificWeight: float = 0.0
    IPColocationFactorWeight: float = 0.0
    IPColocationFactorThreshold: int = 0
    IPColocationFactorWhitelist: List = field(default_factory=list)
    BehaviourPenaltyWeight: float = 0.0
    BehaviourPenaltyThreshold: float = 0.0
    BehaviourPenaltyDecay: float = 0.0
    DecayInterval: int = 0
    DecayToZero: float = 0.0
    RetainScore: int = 0
    SeenMsgTTL: int = 0

    def to_c(self) -> _abi.CPeerScoreParams:
        return _abi.CPeerScoreParams(
            int(self.SkipAtomicValidation), int(self.AppSpecificScore is not None),
            self.TopicScoreCap, self.AppSpecificWeight,
            self.IPColocationFactorWeight, int(self.IPColocationFactorThreshold), 0,
            self.BehaviourPenaltyWeight, self.BehaviourPenaltyThreshold, self.BehaviourPenaltyDecay,
            int(self.DecayInterval), self.DecayToZero, int(self.RetainScore), int(self.SeenMsgTTL))

    def topic_array(self, topic_names: List[str]):
        arr = (_abi.CTopicScoreParams * max(1, len(topic_names)))()
        for i, name in enumerate(topic_names):
            tp = self.Topics.get(name)
            arr[i] = tp.to_c(True) if tp is not None else TopicScoreParams().to_c(False)
        return arr

    def validate(self) -> None:
        """score_params.go:173-234 (topics first, as the reference does)."""
        lib = _abi.load()
        names = sorted(self.Topics)
        for name in names:
            try:
                self.Topics[name].validate()
            except ValueError as e:
                raise ValueError(f"invalid score parameters for topic {name}: {e}") from None
        buf = ctypes.create_string_buffer(512)
        c = self.to_c()
        if lib.gsim_validate_peer_params(ctypes.byref(c), None, 0, buf, len(buf)) != 0:
            raise ValueError(buf.value.decode())
        if self.SkipAtomicValidation and self.AppSpecificScore is None:
            self.AppSpecificScore = lambda p: 0.0          # score_params.go:190-193

    def whitelisted(self, ip: str) -> bool:
        """net.IPNet.Contains over the whitelist (score.go:353-369)."""
        if not self.IPColocationFactorWhitelist:
            return False
        addr = ipaddress.ip_address(ip)
        return any(addr in net for net in self.IPColocationFactorWhitelist)


@dataclass
class PeerScoreThresholds:
    """PeerScoreThresholds, score_params.go:12-35."""
    SkipAtomicValidation: bool = False
    GossipThreshold: float = 0.0
    PublishThreshold: float = 0.0
    GraylistThreshold: float = 0.0
    AcceptPXThreshold: float = 0.0
    OpportunisticGraftThreshold: float = 0.0

    def to_c(self) -> _abi.CThresholds:
        return _abi.CThresholds(int(self.SkipAtomicValidation), 0, self.GossipThreshold, self.PublishThreshold,
                                self.GraylistThreshold, self.AcceptPXThreshold, self.OpportunisticGraftThreshold)

    def validate(self) -> None:
        """score_params.go:37-64."""
        buf = ctypes.create_string_buffer(512)
        c = self.to_c()
        if _abi.load().gsim_validate_thresholds(ctypes.byref(c), buf, len(buf)) != 0:
            raise ValueError(buf.value.decode())


@dataclass
class GossipSubParams:
    """GossipSubParams, gossipsub.go:63-205."""
    D: int = 6
    Dlo: int = 5
    Dhi: int = 12
    Dscore: int = 4
    Dout: int = 2
    HistoryLength: int = 5
    HistoryGossip: int = 3
    Dlazy: int = 6
    GossipFactor: float = 0.25
    GossipRetransmission: int = 3
    HeartbeatInitialDelay: int = 100 * Millisecond
    HeartbeatInterval: int = Second
    SlowHeartbeatWarning: float = 0.1
    FanoutTTL: int = 60 * Second
    PrunePeers: int = 16
    PruneBackoff: int = Minute
    UnsubscribeBackoff: int = 10 * Second
    Connectors: int = 8
    MaxPendingConnections: int = 128
    ConnectionTimeout: int = 30 * Second
    DirectConnectTicks: int = 300
    DirectConnectInitialDelay: int = Second
    OpportunisticGraftTicks: int = 60
    OpportunisticGraftPeers: int = 2
    GraftFloodThreshold: int = 10 * Second
    MaxIHaveLength: int = 5000
    MaxIHaveMessages: int = 10
    IWantFollowupTime: int = 3 * Second
    # router option WithFloodPublish (gossipsub.go:321-334), not a GossipSubParams field
    FloodPublish: bool = False
    # router option WithPeerExchange (gossipsub.go:340-350): PRUNEs carry PX
    PeerExchange: bool = False

    def to_c(self) -> _abi.CGossipSubParams:
        c = _abi.CGossipSubParams()
        c.d, c.dlo, c.dhi, c.dscore, c.dout = self.D, self.Dlo, self.Dhi, self.Dscore, self.Dout
        c.history_length, c.history_gossip, c.dlazy = self.HistoryLength, self.HistoryGossip, self.Dlazy
        c.gossip_factor, c.gossip_retransmission = self.GossipFactor, self.GossipRetransmission
        c.prune_peers = self.PrunePeers
        c.heartbeat_initial_delay_ns, c.heartbeat_interval_ns = self.HeartbeatInitialDelay, self.HeartbeatInterval
        c.slow_heartbeat_warning, c.fanout_ttl_ns = self.SlowHeartbeatWarning, self.FanoutTTL
        c.prune_backoff_ns, c.unsubscribe_backoff_ns = self.PruneBackoff, self.UnsubscribeBackoff
        c.connectors, c.max_pending_connections = self.Connectors, self.MaxPendingConnections
        c.connection_timeout_ns, c.direct_connect_ticks = self.ConnectionTimeout, self.DirectConnectTicks
        c.direct_connect_initial_delay_ns = self.DirectConnectInitialDelay
        c.opportunistic_graft_ticks, c.opportunistic_graft_peers = (self.OpportunisticGraftTicks,
                                                                     self.OpportunisticGraftPeers)
        c.max_ihave_length, c.graft_flood_threshold_ns = self.MaxIHaveLength, self.GraftFloodThreshold
        c.flood_publish = 1 if self.FloodPublish else 0
        c.do_px = 1 if self.PeerExchange else 0
        c.max_ihave_messages, c.iwant_followup_time_ns = self.MaxIHaveMessages, self.IWantFollowupTime
        return c


def DefaultGossipSubParams() -> GossipSubParams:
    """gossipsub.go:244-275 (defaults come from the engine library)."""
    c = _abi.CGossipSubParams()
    _abi.load().gsim_default_gossipsub_params(ctypes.byref(c))
    return GossipSubParams(
        D=c.d, Dlo=c.dlo, Dhi=c.dhi, Dscore=c.dscore, Dout=c.dout, HistoryLength=c.history_length,
        HistoryGossip=c.history_gossip, Dlazy=c.dlazy, GossipFactor=c.gossip_factor,
        GossipRetransmission=c.gossip_retransmission, HeartbeatInitialDelay=c.heartbeat_initial_delay_ns,
        HeartbeatInterval=c.heartbeat_interval_ns, SlowHeartbeatWarning=c.slow_heartbeat_warning,
        FanoutTTL=c.fanout_ttl_ns, PrunePeers=c.prune_peers, PruneBackoff=c.prune_backoff_ns,
        UnsubscribeBackoff=c.unsubscribe_backoff_ns, Connectors=c.connectors,
        MaxPendingConnections=c.max_pending_connections, ConnectionTimeout=c.connection_timeout_ns,
        DirectConnectTicks=c.direct_connect_ticks, DirectConnectInitialDelay=c.direct_connect_initial_delay_ns,
        OpportunisticGraftTicks=c.opportunistic_graft_ticks, OpportunisticGraftPeers=c.opportunistic_graft_peers,
        GraftFloodThreshold=c.graft_flood_threshold_ns, MaxIHaveLength=c.max_ihave_length,
        MaxIHaveMessages=c.max_ihave_messages, IWantFollowupTime=c.iwant_followup_time_ns)


def ScoreParameterDecay(decay: int) -> float:
    """score_params.go:405-409."""
    return _abi.load().gsim_score_parameter_decay(int(decay))


def ScoreParameterDecayWithBase(decay: int, base: int, decayToZero: float) -> float:
    """score_params.go:411-417."""
    return _abi.load().gsim_score_parameter_decay_with_base(int(decay), int(base), float(decayToZero))


@dataclass
class PeerGaterParams:
    """PeerGaterParams, peer_gater.go:31-55 (durations in ns).  TopicDeliveryWeights
    maps a topic index to its weight (0 / absent: 1.0; multiples of 2**-16)."""
    Threshold: float
    GlobalDecay: float
    SourceDecay: float
    DecayInterval: int = Second
    DecayToZero: float = 0.01
    RetainStats: int = 6 * Hour
    Quiet: int = Minute
    DuplicateWeight: float = 0.125
    IgnoreWeight: float = 1.0
    RejectWeight: float = 16.0
    TopicDeliveryWeights: Dict[int, float] = field(default_factory=dict)

    def to_c(self) -> _abi.CPeerGaterParams:
        c = _abi.CPeerGaterParams()
        c.threshold, c.global_decay, c.source_decay = self.Threshold, self.GlobalDecay, self.SourceDecay
        c.decay_interval_ns, c.decay_to_zero = int(self.DecayInterval), self.DecayToZero
        c.retain_stats_ns, c.quiet_ns = int(self.RetainStats), int(self.Quiet)
        c.duplicate_weight, c.ignore_weight, c.reject_weight = (self.DuplicateWeight, self.IgnoreWeight,
                                                                self.RejectWeight)
        return c

    def validate(self) -> None:
        """PeerGaterParams.validate (peer_gater.go:57-90)."""
        buf = ctypes.create_string_buffer(256)
        c = self.to_c()
        if _abi.load().gsim_validate_peer_gater_params(ctypes.byref(c), buf, len(buf)) != 0:
            raise ValueError(buf.value.decode())


def NewPeerGaterParams(threshold: float, globalDecay: float, sourceDecay: float) -> PeerGaterParams:
    """NewPeerGaterParams (peer_gater.go:99-111), defaults from the engine library."""
    c = _abi.CPeerGaterParams()
    _abi.load().gsim_default_peer_gater_params(threshold, globalDecay, sourceDecay, ctypes.byref(c))
    return PeerGaterParams(Threshold=c.threshold, GlobalDecay=c.global_decay, SourceDecay=c.source_decay,
                           DecayInterval=c.decay_interval_ns, DecayToZero=c.decay_to_zero,
                           RetainStats=c.retain_stats_ns, Quiet=c.quiet_ns, DuplicateWeight=c.duplicate_weight,
                           IgnoreWeight=c.ignore_weight, RejectWeight=c.reject_weight)


def DefaultPeerGaterParams() -> PeerGaterParams:
    """DefaultPeerGaterParams (peer_gater.go:113-116): Threshold 0.33, GlobalDecay
    ScoreParameterDecay(2m), SourceDecay ScoreParameterDecay(1h)."""
    return NewPeerGaterParams(0.33, ScoreParameterDecay(2 * Minute), ScoreParameterDecay(Hour))
