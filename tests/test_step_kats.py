"""Hand-derived known-answer traces under the canonical STEP schedule
(tests/golden/kat_step_schedule.json: the FIFO max(s + d, last_due) rule,
an isolation window that swallows a Propose before a Q6 panic, and a skewed
duel with a NACK ahead of the majority index and a Q10 abort).  They pin the
part of the contract the global-FIFO KATs (kat_global_fifo.json) do not
cover: per-link delays, isolation, Tick skew and the acceptor-then-proposer
phase order.  Checked here against both CPU oracles; test_gpu_parity.py
checks the GPU results and per-step traces against the same fixture."""
import json
import os

import pytest

import oracle_c
import paxos_ref as R
import pxb

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = json.load(open(os.path.join(HERE, "golden", "kat_step_schedule.json")))["cases"]
IDS = [c["name"] for c in KATS]


def config(case):
    return pxb.Config(**case["config"])


def meaningful_prop(p):
    """[ticket, cmd, acks, state] of a proposer (the fields the reference's
    ClientState holds in every round state, Client.hs:58-67)."""
    return [p[0], p[1], p[2], p[3]]


@pytest.mark.parametrize("case", KATS, ids=IDS)
def test_draws_are_the_fixture_inputs(case):
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import step_kat_draws
    assert step_kat_draws.case_draws(case) == case["draws"]


@pytest.mark.parametrize("case", KATS, ids=IDS)
def test_python_oracle_matches_hand_derivation(case):
    cfg = R.Config(**case["config"])
    states = {}

    def snap(s, accs, props, in_flight):
        states[s] = {"in_flight": in_flight,
                     "acc": [[a.t_max, a.t_store, a.val, len(a.log) | (int(a.dead) << 31)] for a in accs],
                     "prop": [[p.ticket, p.cmd, p.acks, p.rs] for p in props]}
    r = R.run_instance(cfg, case["instance"], trace=snap)
    want = case["result"]
    assert (r.decided_val, r.decided_ticket, r.rounds, r.flags, r.steps) == \
        (want["decided_val"], want["decided_ticket"], want["rounds"], want["flags"], want["steps"])
    assert (r.messages, r.canon_bytes, r.executes) == (want["messages"], want["canon_bytes"], want["executes"])
    assert [list(a.log) for a in r.acceptors] == want["logs"]
    for cp in case["checkpoints"]:
        got = states[cp["step"]]
        assert got["acc"] == cp["acc"], cp["step"]
        assert [meaningful_prop(p) for p in got["prop"]] == cp["prop"], cp["step"]
        if "in_flight" in cp:
            assert got["in_flight"] == cp["in_flight"], cp["step"]


@pytest.mark.parametrize("case", KATS, ids=IDS)
def test_c_oracle_matches_hand_derivation(case):
    cfg = config(case)
    res, dig, acc, cnt = oracle_c.run_cpu(cfg, case["instance"], 1, threads=1, want_acceptors=True)
    want = case["result"]
    assert list(res[0]) == [want["decided_val"], want["decided_ticket"], want["rounds"],
                            want["flags"] | (want["steps"] << 16)]
    assert (cnt["messages"], cnt["canon_bytes"], cnt["executes"], cnt["steps"]) == \
        (want["messages"], want["canon_bytes"], want["executes"], want["steps"])
    final = [cp for cp in case["checkpoints"] if cp["step"] == want["steps"] - 1][0]
    assert acc[0].tolist() == final["acc"]
    for a, log in enumerate(want["logs"]):
        h = R.FNV_BASIS
        for v in log:
            h = R.fnv1a_u32(h, v)
        assert dig[0][a] == R.fnv1a_u32(h, len(log))
