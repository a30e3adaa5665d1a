"""CPU tests of the oracle (oracle/): Philox KATs, the hand-derived protocol
KATs of SURVEY.md §8.0 (global-FIFO schedule), canonical-schedule properties,
and the C restatement against the Python restatement and golden fixtures."""
import glob
import json
import os

import numpy as np
import pytest

import oracle_c
import paxos_ref as R
import pxb

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


# ---- Philox4x32-10, Random123 known-answer vectors --------
@pytest.mark.parametrize("key,ctr,out", [
    ((0, 0), (0, 0, 0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff, 0xffffffff), (0xffffffff,) * 4, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0xa4093822, 0x299f31d0), (0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_kat(key, ctr, out):
    assert R.philox4x32_10(ctr, key) == out


# ---- protocol KATs under the global-FIFO schedule ----------------------------
def _fifo(P, N, drops=()):
    r = R.run_global_fifo(P, N, drops)
    logs = [[R.cmd_str(v) for v in a.log] for a in r.acceptors]
    return r, logs


def test_kat1_single_proposer():
    r, logs = _fifo(1, 3)
    assert R.cmd_str(r.decided_val) == "c1.1" and r.decided_ticket == 1
    assert r.rounds == 1 and r.messages == 15 and r.flags == 0
    assert logs == [["c1.1"]] * 3
    assert all(a.t_max == 1 and a.val == R.NOTHING for a in r.acceptors)
    p = r.proposers[0]
    assert (p.ticket, p.cmd, p.rs) == (1, R.NOTHING, R.IDLE)


def test_kat2_duelling_proposers():
    r, logs = _fifo(2, 3)
    assert R.cmd_str(r.decided_val) == "c1.1" and r.decided_ticket == 1
    assert r.rounds == 4 and r.messages == 51 and r.flags == 0
    assert logs == [["c1.1", "c2.1"]] * 3
    assert all(a.t_max == 3 for a in r.acceptors)


def test_stock_main_hs_topology():
    # app/Main.hs:41,45 — 2 acceptors, 2 proposers
    r, logs = _fifo(2, 2)
    assert logs == [["c1.1", "c2.1"]] * 2 and r.rounds == 4 and r.messages == 34


def test_kat3_lost_propose_panics():
    r, logs = _fifo(1, 3, [(("c", 1), ("s", 3), 2)])
    assert r.flags & R.F_PANIC and R.cmd_str(r.decided_val) == "c1.1"
    assert logs == [["c1.1"], ["c1.1"], []]
    assert r.acceptors[2].dead


def test_kat4_lost_asks_stuck():
    r, logs = _fifo(1, 3, [(("c", 1), ("s", 2), 1), (("c", 1), ("s", 3), 1)])
    assert r.flags == R.F_UNDECIDED | R.F_STUCK and r.rounds == 1
    assert [a.t_max for a in r.acceptors] == [1, 0, 0]


def test_kat5_lost_execute_keeps_proposal():
    r, logs = _fifo(1, 3, [(("c", 1), ("s", 3), 3)])
    assert logs == [["c1.1"], ["c1.1"], []] and r.flags == 0
    assert (r.acceptors[2].t_store, R.cmd_str(r.acceptors[2].val)) == (1, "c1.1")


def test_kat6_lost_reply_same_as_kat2():
    r, logs = _fifo(2, 3, [(("s", 3), ("c", 1), 1)])
    r2, logs2 = _fifo(2, 3)
    assert logs == logs2 and r.rounds == r2.rounds and r.decided_val == r2.decided_val


def test_kat_json_fixture_matches():
    with open(os.path.join(GOLDEN, "kat_global_fifo.json")) as f:
        kats = json.load(f)
    for name, k in kats.items():
        drops = [tuple(tuple(x) if isinstance(x, list) else x for x in d) for d in k["drops"]]
        r, logs = _fifo(k["P"], k["N"], drops)
        assert logs == k["logs"], name
        assert (r.rounds, r.messages, r.flags) == (k["rounds"], k["messages"], k["flags"]), name


# ---- handler-level quirks -----------------------------
def test_q2_stale_round2success_counts():
    p = R.Proposer(client_id=1, ticket=5, cmd=R.cmd_code(1, 1), rs=R.ROUND2, r2_t=5,
                   r2_v=R.cmd_code(1, 1))
    R.proposer_handle(p, 3, R.R2S)
    out = R.proposer_handle(p, 3, R.R2S)
    assert out == [(R.EXECUTE, 5, R.NOTHING)] and p.rs == R.IDLE


def test_q4_most_recent_tie_keeps_earlier():
    assert R.most_recent(3, 111, 3, 222) == (3, 111)
    assert R.most_recent(2, 111, 3, 222) == (3, 222)
    assert R.most_recent(0, R.NOTHING, 3, 222) == (3, 222)


def test_q5_pending_on_own_command():
    own = R.cmd_code(1, 1)
    p = R.Proposer(client_id=1, ticket=4, cmd=own, rs=R.ROUND1)
    R.proposer_handle(p, 3, R.R1OK, 4, 2, own)
    out = R.proposer_handle(p, 3, R.R1OK, 4, 0, R.NOTHING)
    assert p.pending and out == [(R.PROPOSE, 4, own)]


def test_acceptor_propose_needs_equality():
    a = R.Acceptor(t_max=5)
    assert R.acceptor_handle(a, R.PROPOSE, 4, 7) == (R.HAVE, 5, 0, 0)
    assert R.acceptor_handle(a, R.PROPOSE, 5, 7) == (R.R2S, 0, 0, 0)


# ---- canonical step schedule ----------------------------------------------------
def test_config1_every_instance_is_kat1():
    cfg = R.config(1)
    for i in range(20):
        r = R.run_instance(cfg, i)
        assert R.cmd_str(r.decided_val) == "c1.1" and r.rounds == 1 and r.flags == 0
        assert r.messages == 15 and r.steps == 6
        assert all([R.cmd_str(v) for v in a.log] == ["c1.1"] for a in r.acceptors)


@pytest.mark.parametrize("N", [2, 3, 5, 7, 9])
def test_nofault_canonical_bytes(N):
    cfg = R.Config(seed=7, n_proposers=1, n_acceptors=N)
    r = R.run_instance(cfg, 3)
    assert r.canon_bytes == 196 * N + 160 == pxb.canonical_bytes_nofault(N)


def test_agreement_without_loss_single_proposer():
    cfg = R.Config(seed=11, n_proposers=1, n_acceptors=5, delay_max=6, skew_max=3,
                   crash_ppm=300000, crash_len_max=4, crash_start_max=3)
    for i in range(200):
        r = R.run_instance(cfg, i)
        assert not (r.flags & R.F_LOG_DIVERGENCE)


# ---- log mode (docs/SEMANTICS.md §9): the reference's periodic ticker -------------
def test_log_mode_each_tick_commits_a_new_slot():
    """Client.hs:96-100 ticks a proposer forever; with ticks far enough apart
    every Tick finds it Idle (Client.hs:199), starts "c1.<t>" at the next
    ticket (Client.hs:200-203) and the acceptors log one command per slot."""
    cfg = R.Config(seed=1, n_proposers=1, n_acceptors=3, n_ticks=3, tick_period=10)
    r = R.run_instance(cfg, 0)
    assert r.flags == 0 and r.rounds == 3 and r.executes == 3
    assert R.cmd_str(r.decided_val) == "c1.1" and r.decided_ticket == 1
    assert r.messages == 3 * 15 and r.steps == 20 + 6
    for a in r.acceptors:
        assert [R.cmd_str(v) for v in a.log] == ["c1.1", "c1.2", "c1.3"] and a.t_max == 3


def test_log_mode_tick_while_busy_is_dropped():
    """A Tick that finds the proposer in Round1/Round2 is ignored
    (Client.hs:196-199): ticks at 0, 2, 4, 6 commit c1.1 and c1.2 only."""
    cfg = R.Config(seed=1, n_proposers=1, n_acceptors=3, n_ticks=4, tick_period=2)
    r = R.run_instance(cfg, 0)
    assert r.executes == 2 and r.rounds == 2
    for a in r.acceptors:
        assert [R.cmd_str(v) for v in a.log] == ["c1.1", "c1.2"]


def test_single_tick_config_is_unchanged_by_log_fields():
    base = R.Config(seed=9, n_proposers=2, n_acceptors=5, loss_ppm=100000, delay_max=4, skew_max=3)
    one = R.Config(seed=9, n_proposers=2, n_acceptors=5, loss_ppm=100000, delay_max=4, skew_max=3,
                   n_ticks=1, tick_period=7)
    for i in range(30):
        a, b = R.run_instance(base, i), R.run_instance(one, i)
        assert (a.decided_val, a.rounds, a.packed_flags(), a.canon_bytes) == \
               (b.decided_val, b.rounds, b.packed_flags(), b.canon_bytes)


@pytest.mark.parametrize("P,N,loss,delay,ticks,period", [
    (1, 3, 0, 1, 4, 3), (2, 5, 50000, 3, 6, 9), (3, 7, 150000, 4, 5, 20), (2, 4, 0, 6, 8, 5)])
def test_c_oracle_matches_python_log_mode(P, N, loss, delay, ticks, period):
    cfg = pxb.Config(seed=0x10C + P * N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=2, step_cap=400, n_ticks=ticks, tick_period=period)
    rcfg = R.Config(**{k: getattr(cfg, k) for k in R.Config.__dataclass_fields__})
    n = 40
    res, dig, acc, cnt = oracle_c.run_cpu(cfg, 5, n, threads=2, want_acceptors=True)
    canon = execs = 0
    for i in range(n):
        r = R.run_instance(rcfg, 5 + i)
        canon += r.canon_bytes
        execs += r.executes
        assert list(res[i]) == [r.decided_val, r.decided_ticket, r.rounds, r.packed_flags()]
        assert list(dig[i]) == [r.digest(a) for a in range(N)]
        assert [int(x) for x in acc[i, :, 3]] == [len(a.log) | (int(a.dead) << 31) for a in r.acceptors]
    assert cnt["canon_bytes"] == canon and cnt["executes"] == execs


# ---- C restatement == Python restatement == golden fixtures ----------------------
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "cfg*.npz"))))
def test_c_oracle_matches_golden(path):
    z = np.load(path)
    c, first, n = (int(x) for x in z["meta"])
    res, dig, acc, cnt = oracle_c.run_cpu(pxb.CONFIGS[c], first, n, threads=4, want_acceptors=True)
    assert np.array_equal(res, z["results"])
    assert np.array_equal(dig, z["digests"])
    assert np.array_equal(acc, z["acceptors"])
    assert cnt["canon_bytes"] == int(z["canon_bytes"][0])
    assert cnt["instances"] == n


@pytest.mark.parametrize("P,N,loss,delay,skew,crash", [
    (1, 2, 0, 1, 0, 0), (2, 3, 50000, 3, 2, 0), (3, 4, 200000, 8, 5, 100000),
    (2, 6, 0, 15, 0, 500000), (3, 9, 400000, 2, 1, 0), (1, 8, 900000, 5, 0, 0)])
def test_c_oracle_matches_python_sweep(P, N, loss, delay, skew, crash):
    cfg = pxb.Config(seed=0xABCDEF0123 + P * N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=skew, crash_ppm=crash, crash_len_max=6,
                     crash_start_max=10, step_cap=160)
    rcfg = R.Config(**{k: getattr(cfg, k) for k in R.Config.__dataclass_fields__})
    n = 60
    res, dig, acc, cnt = oracle_c.run_cpu(cfg, 77, n, threads=2, want_acceptors=True)
    canon = 0
    for i in range(n):
        r = R.run_instance(rcfg, 77 + i)
        canon += r.canon_bytes
        assert list(res[i]) == [r.decided_val, r.decided_ticket, r.rounds, r.packed_flags()]
        assert list(dig[i]) == [r.digest(a) for a in range(N)]
    assert cnt["canon_bytes"] == canon


def test_c_handlers_match_python_random():
    rng = np.random.default_rng(5)
    n = 3000
    st = np.zeros((n, 4), np.uint32)
    st[:, 0] = rng.integers(0, 6, n)
    st[:, 1] = rng.integers(0, 6, n)
    st[:, 2] = np.where(rng.random(n) < 0.5, 0, rng.integers(1, 4, n) << 24 | 1)
    st[:, 3] = rng.integers(0, 4, n)
    msg = np.zeros((n, 4), np.uint32)
    msg[:, 0] = rng.integers(0, 3, n)
    msg[:, 1] = rng.integers(0, 7, n)
    msg[:, 3] = rng.integers(1, 4, n) << 24 | 1
    st2, rep = oracle_c.acceptor_handle(st, msg)
    for i in range(n):
        a = R.Acceptor(t_max=int(st[i, 0]), t_store=int(st[i, 1]), val=int(st[i, 2]),
                       log=[0] * int(st[i, 3]))
        r = R.acceptor_handle(a, int(msg[i, 0]), int(msg[i, 1]), int(msg[i, 3]))
        exp_rep = [pxb.MSG_NONE, 0, 0, 0] if r is None else list(r)
        assert list(rep[i]) == exp_rep
        assert list(st2[i]) == [a.t_max, a.t_store, a.val, len(a.log) | (int(a.dead) << 31)]


def test_ticket_limit_matches_kernel_packing():
    """The kernel packs tickets into 14-bit fields; TICKET_OVERFLOW must fire
    at 2^14 in the header, the C oracle (via the header) and the Python oracle."""
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "paxos_batch.h")).read()
    assert re.search(r"#define PXB_TICKET_LIMIT \(1 << 14\)", hdr)
    assert R.TICKET_LIMIT == 1 << 14


def test_ticket_at_the_limit_sets_the_flag():
    """A duel drives tickets up; with the limit lowered to a reachable value the
    flag is set exactly when some proposer's ticket reaches it (a proposer's
    ticket never decreases, so its final value is its maximum)."""
    cfg = R.Config(seed=5, n_proposers=2, n_acceptors=3, delay_max=3, step_cap=60)
    for inst in range(40):
        top = max(p.ticket for p in R.run_instance(cfg, inst).proposers)
        assert R.run_instance(cfg, inst, ticket_limit=top).flags & R.F_TICKET_OVERFLOW
        assert not R.run_instance(cfg, inst, ticket_limit=top + 1).flags & R.F_TICKET_OVERFLOW


def test_trace_callback_ends_at_the_final_state():
    """run_instance's per-step trace (the oracle side of pxb_trace_instance):
    one call per step, and the last snapshot is the final state."""
    cfg = R.Config(seed=5, n_proposers=2, n_acceptors=5, loss_ppm=100000, delay_max=4, skew_max=3, step_cap=200)
    for inst in range(20):
        seen = []
        res = R.run_instance(cfg, inst, trace=lambda s, a, p, f: seen.append(
            (s, [(x.t_max, x.t_store, x.val, tuple(x.log)) for x in a], [(y.ticket, y.rs) for y in p], f)))
        assert [x[0] for x in seen] == list(range(res.steps))
        assert seen[-1][1] == [(x.t_max, x.t_store, x.val, tuple(x.log)) for x in res.acceptors]
        assert seen[-1][2] == [(y.ticket, y.rs) for y in res.proposers]
        assert (seen[-1][3] == 0) or (res.flags & R.F_STEP_CAP)
