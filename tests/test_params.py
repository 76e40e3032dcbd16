"""score_params_test.go ported: parameter validation tables and the decay KAT.

These run the engine library's validation (csrc/params.cpp, the code
gsim_create executes) through the Python mirror of the reference API; no GPU.
"""
import math

import pytest

from gsim.params import (DefaultGossipSubParams, Millisecond, Hour, PeerScoreParams, PeerScoreThresholds,
                         ScoreParameterDecay, Second, TopicScoreParams)

INF, NAN = math.inf, math.nan


def app(p):
    return 0.0


# ---- TestPeerScoreThreshold_{Atomic,Skip}Validation (score_params_test.go:11-119)
THRESH_INVALID = [
    dict(GossipThreshold=1), dict(PublishThreshold=1), dict(GossipThreshold=-1, PublishThreshold=0),
    dict(GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=0), dict(AcceptPXThreshold=-1),
    dict(OpportunisticGraftThreshold=-1),
    dict(GossipThreshold=-INF, PublishThreshold=-2, GraylistThreshold=-3, AcceptPXThreshold=1,
         OpportunisticGraftThreshold=2),
    dict(GossipThreshold=-1, PublishThreshold=-INF, GraylistThreshold=-3, AcceptPXThreshold=1,
         OpportunisticGraftThreshold=2),
    dict(GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-INF, AcceptPXThreshold=1,
         OpportunisticGraftThreshold=2),
    dict(GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-3, AcceptPXThreshold=NAN,
         OpportunisticGraftThreshold=2),
    dict(GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-3, AcceptPXThreshold=1,
         OpportunisticGraftThreshold=INF),
]


@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("kw", THRESH_INVALID)
def test_thresholds_invalid(skip, kw):
    with pytest.raises(ValueError):
        PeerScoreThresholds(SkipAtomicValidation=skip, **kw).validate()


@pytest.mark.parametrize("skip", [False, True])
def test_thresholds_valid(skip):
    PeerScoreThresholds(SkipAtomicValidation=skip, GossipThreshold=-1, PublishThreshold=-2, GraylistThreshold=-3,
                        AcceptPXThreshold=1, OpportunisticGraftThreshold=2).validate()


# ---- testTopicScoreParamsValidationWithInvalidParameters (score_params_test.go:129-360)
S = Second
TOPIC_INVALID = [
    dict(TopicWeight=-1),
    dict(TimeInMeshWeight=-1, TimeInMeshQuantum=S),
    dict(TimeInMeshWeight=1, TimeInMeshQuantum=-1),
    dict(TimeInMeshWeight=1, TimeInMeshQuantum=S, TimeInMeshCap=-1),
    dict(TimeInMeshQuantum=S, FirstMessageDeliveriesWeight=-1),
    dict(TimeInMeshQuantum=S, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=-1),
    dict(TimeInMeshQuantum=S, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=2),
    dict(TimeInMeshQuantum=S, FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=.5,
         FirstMessageDeliveriesCap=-1),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=1),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=-1),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=2),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5,
         MeshMessageDeliveriesCap=-1),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5,
         MeshMessageDeliveriesCap=5, MeshMessageDeliveriesThreshold=-3),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5,
         MeshMessageDeliveriesCap=5, MeshMessageDeliveriesThreshold=3, MeshMessageDeliveriesWindow=-1),
    dict(TimeInMeshQuantum=S, MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=.5,
         MeshMessageDeliveriesCap=5, MeshMessageDeliveriesThreshold=3, MeshMessageDeliveriesWindow=Millisecond,
         MeshMessageDeliveriesActivation=Millisecond),
    dict(TimeInMeshQuantum=S, MeshFailurePenaltyWeight=1),
    dict(TimeInMeshQuantum=S, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=-1),
    dict(TimeInMeshQuantum=S, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=2),
    dict(TimeInMeshQuantum=S, InvalidMessageDeliveriesWeight=1),
    dict(TimeInMeshQuantum=S, InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=-1),
    dict(TimeInMeshQuantum=S, InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=2),
]


@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("kw", TOPIC_INVALID)
def test_topic_params_invalid(skip, kw):
    with pytest.raises(ValueError):
        TopicScoreParams(SkipAtomicValidation=skip, **kw).validate()


def test_topic_params_empty():
    """Zero params fail atomically, pass in skip mode (score_params_test.go:131-140)."""
    TopicScoreParams(SkipAtomicValidation=True).validate()
    with pytest.raises(ValueError):
        TopicScoreParams().validate()


GOOD_TOPIC = dict(TopicWeight=1, TimeInMeshWeight=0.01, TimeInMeshQuantum=S, TimeInMeshCap=10,
                  FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.5, FirstMessageDeliveriesCap=10,
                  MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=0.5, MeshMessageDeliveriesCap=10,
                  MeshMessageDeliveriesThreshold=5, MeshMessageDeliveriesWindow=Millisecond,
                  MeshMessageDeliveriesActivation=S, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=0.5,
                  InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=0.5)


def test_topic_params_valid_atomic():
    """score_params_test.go:362-386."""
    TopicScoreParams(**GOOD_TOPIC).validate()


def test_topic_params_non_atomic_incremental():
    """score_params_test.go:388-433: each group may be set on its own in skip mode."""
    p = TopicScoreParams(SkipAtomicValidation=True)
    p.validate()
    steps = [dict(TopicWeight=1), dict(TimeInMeshWeight=0.01, TimeInMeshQuantum=S, TimeInMeshCap=10),
             dict(FirstMessageDeliveriesWeight=1, FirstMessageDeliveriesDecay=0.5, FirstMessageDeliveriesCap=10),
             dict(MeshMessageDeliveriesWeight=-1, MeshMessageDeliveriesDecay=0.5, MeshMessageDeliveriesCap=10,
                  MeshMessageDeliveriesThreshold=5, MeshMessageDeliveriesWindow=Millisecond,
                  MeshMessageDeliveriesActivation=S),
             dict(MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=0.5),
             dict(InvalidMessageDeliveriesWeight=-1, InvalidMessageDeliveriesDecay=0.5)]
    for kw in steps:
        for k, v in kw.items():
            setattr(p, k, v)
        p.validate()


# ---- testPeerScoreParamsValidationWithInvalidParams (score_params_test.go:443-618)
BAD_NUM_TOPIC = dict(TopicWeight=INF, TimeInMeshWeight=NAN, TimeInMeshQuantum=S, TimeInMeshCap=10,
                     FirstMessageDeliveriesWeight=INF, FirstMessageDeliveriesDecay=0.5, FirstMessageDeliveriesCap=10,
                     MeshMessageDeliveriesWeight=-INF, MeshMessageDeliveriesDecay=NAN, MeshMessageDeliveriesCap=INF,
                     MeshMessageDeliveriesThreshold=5, MeshMessageDeliveriesWindow=Millisecond,
                     MeshMessageDeliveriesActivation=S, MeshFailurePenaltyWeight=-1, MeshFailurePenaltyDecay=NAN,
                     InvalidMessageDeliveriesWeight=INF, InvalidMessageDeliveriesDecay=NAN)
PEER_INVALID = [
    dict(TopicScoreCap=-1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, IPColocationFactorWeight=1),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, IPColocationFactorWeight=-1,
         IPColocationFactorThreshold=-1),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=Millisecond, DecayToZero=0.01,
         IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=-1, IPColocationFactorWeight=-1,
         IPColocationFactorThreshold=1),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=2, IPColocationFactorWeight=-1,
         IPColocationFactorThreshold=1),
    dict(AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, BehaviourPenaltyWeight=1),
    dict(AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, BehaviourPenaltyWeight=-1),
    dict(AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, BehaviourPenaltyWeight=-1,
         BehaviourPenaltyDecay=2),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, IPColocationFactorWeight=-1,
         IPColocationFactorThreshold=1, Topics={"test": TopicScoreParams(**BAD_NUM_TOPIC)}),
    dict(AppSpecificScore=app, DecayInterval=S, DecayToZero=INF, IPColocationFactorWeight=-INF,
         IPColocationFactorThreshold=1, BehaviourPenaltyWeight=INF, BehaviourPenaltyDecay=NAN),
    dict(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, IPColocationFactorWeight=-1,
         IPColocationFactorThreshold=1, Topics={"test": TopicScoreParams(**{**GOOD_TOPIC, "TopicWeight": -1})}),
]


@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("kw", PEER_INVALID)
def test_peer_params_invalid(skip, kw):
    with pytest.raises(ValueError):
        PeerScoreParams(SkipAtomicValidation=skip, **kw).validate()


def test_peer_params_missing_app_score():
    """Missing AppSpecificScore: error when atomic, defaulted to 0 when skipping."""
    with pytest.raises(ValueError, match="missing application specific score function"):
        PeerScoreParams(TopicScoreCap=1, DecayInterval=S, DecayToZero=0.01).validate()
    p = PeerScoreParams(SkipAtomicValidation=True, TopicScoreCap=1, DecayInterval=S, DecayToZero=0.01)
    p.validate()
    assert p.AppSpecificScore("x") == 0


def test_peer_params_valid_atomic():
    """score_params_test.go:620-680."""
    PeerScoreParams(AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01, IPColocationFactorWeight=-1,
                    IPColocationFactorThreshold=1, BehaviourPenaltyWeight=-1, BehaviourPenaltyDecay=0.999).validate()
    PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01,
                    IPColocationFactorWeight=-1, IPColocationFactorThreshold=1, BehaviourPenaltyWeight=-1,
                    BehaviourPenaltyDecay=0.999).validate()
    PeerScoreParams(TopicScoreCap=1, AppSpecificScore=app, DecayInterval=S, DecayToZero=0.01,
                    IPColocationFactorWeight=-1, IPColocationFactorThreshold=1,
                    Topics={"test": TopicScoreParams(**GOOD_TOPIC)}).validate()


def test_peer_params_skip_incremental():
    """score_params_test.go:682-718."""
    p = PeerScoreParams(SkipAtomicValidation=True)
    p.validate()
    for kw in [dict(AppSpecificScore=app), dict(DecayInterval=S, DecayToZero=0.01),
               dict(IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
               dict(BehaviourPenaltyWeight=-1, BehaviourPenaltyDecay=0.999)]:
        for k, v in kw.items():
            setattr(p, k, v)
        p.validate()
    p = PeerScoreParams(SkipAtomicValidation=True, AppSpecificScore=app)
    for kw in [dict(TopicScoreCap=1), dict(DecayInterval=S, DecayToZero=0.01),
               dict(IPColocationFactorWeight=-1, IPColocationFactorThreshold=1),
               dict(BehaviourPenaltyWeight=-1, BehaviourPenaltyDecay=0.999),
               dict(Topics={"test": TopicScoreParams(**GOOD_TOPIC)})]:
        for k, v in kw.items():
            setattr(p, k, v)
        p.validate()


def test_score_parameter_decay():
    """score_params_test.go:720-725: ScoreParameterDecay(1h) == .9987216039048303 exactly."""
    assert ScoreParameterDecay(Hour) == .9987216039048303


def test_default_gossipsub_params():
    """gossipsub.go:244-275."""
    p = DefaultGossipSubParams()
    assert (p.D, p.Dlo, p.Dhi, p.Dscore, p.Dout) == (6, 5, 12, 4, 2)
    assert (p.HistoryLength, p.HistoryGossip, p.Dlazy, p.GossipFactor) == (5, 3, 6, 0.25)
    assert p.HeartbeatInterval == Second and p.PruneBackoff == 60 * Second
    assert (p.OpportunisticGraftTicks, p.OpportunisticGraftPeers) == (60, 2)
    assert (p.MaxIHaveLength, p.MaxIHaveMessages, p.IWantFollowupTime) == (5000, 10, 3 * Second)
