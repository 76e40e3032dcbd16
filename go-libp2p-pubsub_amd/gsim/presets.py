"""Parameter presets taken from the reference: the beacon-chain-style
TopicScoreParams / PeerScoreParams / thresholds of gossipsub_spam_test.go
(the only production-like set the reference holds), used by the bench
workload and the parity tests."""
from __future__ import annotations

import numpy as np

from .params import Minute, PeerScoreParams, PeerScoreThresholds, Second, TopicScoreParams


def zero_app_score(p):
    """AppSpecificScore that is 0 for every peer (vectorized: takes a peer
    index or an array of them, see gsim.engine.app_scores)."""
    return np.zeros(np.shape(p)) if np.ndim(p) else 0.0


zero_app_score.vectorized = True


def beacon_topic(**over) -> TopicScoreParams:
    """The only production-like TopicScoreParams set in the reference
    (gossipsub_spam_test.go:638-656), used as the "beacon-style" fixture."""
    kw = dict(TopicWeight=0.25, TimeInMeshWeight=0.0027, TimeInMeshQuantum=Second, TimeInMeshCap=3600,
              FirstMessageDeliveriesWeight=0.664, FirstMessageDeliveriesDecay=0.9916,
              FirstMessageDeliveriesCap=1500, MeshMessageDeliveriesWeight=-0.25, MeshMessageDeliveriesDecay=0.97,
              MeshMessageDeliveriesCap=400, MeshMessageDeliveriesThreshold=100,
              MeshMessageDeliveriesActivation=30 * Second, MeshMessageDeliveriesWindow=5 * Minute,
              MeshFailurePenaltyWeight=-0.25, MeshFailurePenaltyDecay=0.997,
              InvalidMessageDeliveriesWeight=-99, InvalidMessageDeliveriesDecay=0.9994)
    kw.update(over)
    return TopicScoreParams(**kw)


def beacon_params(n_topics: int, topic_cap: float = 0.0, **over) -> PeerScoreParams:
    """gossipsub_spam_test.go:627-637 peer params (+P6/P7 enabled for coverage)."""
    kw = dict(AppSpecificScore=zero_app_score, AppSpecificWeight=1.0, IPColocationFactorWeight=-35.11,
              IPColocationFactorThreshold=2, BehaviourPenaltyWeight=-15.92, BehaviourPenaltyThreshold=6,
              BehaviourPenaltyDecay=0.986, DecayInterval=Second, DecayToZero=0.01, RetainScore=10 * Second,
              TopicScoreCap=topic_cap)
    kw.update(over)
    p = PeerScoreParams(**kw)
    # vary the topics a little so per-topic parameters are exercised
    for t in range(n_topics):
        p.Topics[f"topic{t:02d}"] = beacon_topic(TopicWeight=0.25 + 0.05 * t,
                                                 MeshMessageDeliveriesThreshold=max(4, 100 - 3 * t))
    return p


def beacon_thresholds() -> PeerScoreThresholds:
    """gossipsub_spam_test.go:657-662."""
    return PeerScoreThresholds(GossipThreshold=-100, PublishThreshold=-200, GraylistThreshold=-300,
                               AcceptPXThreshold=0)
