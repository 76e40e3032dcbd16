"""Replay the reference's known answers in tests/golden/reference_kats.json
(hand-extracted from score_test.go / score_params_test.go, cited per case)
against the C oracle: the data-driven twin of test_oracle_kats.py, pinning
the oracle before it checks the GPU."""
import json
import os

import pytest

from gsim.params import PeerScoreParams, ScoreParameterDecay, TopicScoreParams
from peerscore_harness import Msg, PeerScore

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")
DATA = json.load(open(GOLDEN))
TOPIC = "mytopic"


def build(case):
    pp = dict(case["peer_params"])
    app = pp.pop("AppSpecificScore", 0.0)
    params = PeerScoreParams(AppSpecificScore=lambda p, v=app: v, **pp)
    extra = []
    if case["topic_params"] is not None:
        if case["topic_params"]:
            params.Topics[TOPIC] = TopicScoreParams(**case["topic_params"])
        else:
            extra = [TOPIC]
    return PeerScore(params, peers=["A"], extra_topics=extra)


@pytest.mark.parametrize("case", DATA["cases"], ids=[c["name"] for c in DATA["cases"]])
def test_reference_kat(case):
    ps = build(case)
    expected = None
    mid = 0
    for ev in case["events"]:
        op = ev[0]
        if op == "add_peer":
            ps.AddPeer("A")
        elif op == "remove_peer":
            ps.RemovePeer("A")
        elif op == "add_penalty":
            ps.AddPenalty("A", ev[1])
        elif op == "graft":
            ps.Graft("A", TOPIC)
        elif op == "sleep":
            ps.sleep(ev[1])
        elif op == "refresh":
            ps.refreshScores()
        elif op == "refresh_n":
            for _ in range(ev[1]):
                ps.refreshScores()
        elif op == "deliver_first":
            for _ in range(ev[1]):
                m = Msg(mid, TOPIC, "A")
                mid += 1
                ps.ValidateMessage(m)
                ps.DeliverMessage(m)
        elif op == "expect":
            expected = float(ev[1])
            assert ps.Score("A") == expected, f"{case['source']}: after {ev}"
        elif op == "expect_mul":
            expected = 1.0
            for f in ev[1]:
                expected *= f
            assert ps.Score("A") == expected, f"{case['source']}: after {ev}"
        elif op == "expect_scale":
            for _ in range(ev[2]):
                expected *= ev[1]
            assert ps.Score("A") == expected, f"{case['source']}: after {ev}"
        else:
            raise AssertionError(f"unknown event {op}")


def test_reference_decay_kat():
    d = DATA["score_parameter_decay"]
    assert ScoreParameterDecay(d["decay_ns"]) == d["expected"], d["source"]
