"""gsim — MI355X-native GossipSub scoring + heartbeat simulation engine.

Host-side mirror of the reference's plugin surface for the hot path:
``PeerScoreParams``/``TopicScoreParams``/``PeerScoreThresholds``/
``GossipSubParams`` (score_params.go, gossipsub.go) and an ``Engine`` that
drives libgsim.so's HIP kernels through the C ABI in include/gsim.h.
"""
from . import _abi
from .engine import Engine, GsimError, Network, random_regular
from .params import (DefaultDecayInterval, DefaultDecayToZero, DefaultGossipSubParams, DefaultPeerGaterParams,
                     GossipSubParams, Hour, Microsecond, Millisecond, Minute, Nanosecond, NewPeerGaterParams,
                     PeerGaterParams, PeerScoreParams, PeerScoreThresholds, ScoreParameterDecay,
                     ScoreParameterDecayWithBase, Second, TimeCacheDuration, TopicScoreParams)

__all__ = [
    "Engine", "GsimError", "Network", "random_regular", "PeerScoreParams", "TopicScoreParams",
    "PeerScoreThresholds", "GossipSubParams", "DefaultGossipSubParams", "ScoreParameterDecay",
    "ScoreParameterDecayWithBase", "Nanosecond", "Microsecond", "Millisecond", "Second", "Minute", "Hour",
    "DefaultDecayInterval", "DefaultDecayToZero", "TimeCacheDuration", "PeerGaterParams", "NewPeerGaterParams",
    "DefaultPeerGaterParams", "_abi",
]
