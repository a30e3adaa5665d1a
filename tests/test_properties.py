"""Hypothesis properties of the oracle (SURVEY.md §8(c) "Pins"), CPU only.

Each property holds for the reference's protocol (Server.hs:44-89,
Client.hs:85-207) under the canonical Philox schedule (docs/SEMANTICS.md), so
the search covers configurations the fixed seeded sweeps of test_oracle.py do
not name.  The properties restate what the reference's source implies; the
reference's own test suite (test/Spec.hs:1-2) holds none, so they pin the
restatement against itself and the handler contract, not against a run of the
Haskell binary (parity unpinned).
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle_c
import paxos_ref as R
import pxb

SETTINGS = settings(max_examples=40, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@st.composite
def configs(draw, faulty=True, log_mode=True):
    P = draw(st.integers(1, 3))
    N = draw(st.integers(2, 9))
    kw = dict(seed=draw(st.integers(0, 2**64 - 1)), n_proposers=P, n_acceptors=N,
              delay_max=draw(st.integers(1, 15)), skew_max=draw(st.integers(0, 6)),
              step_cap=draw(st.integers(1, 300)))
    if faulty:
        kw.update(loss_ppm=draw(st.sampled_from([0, 1000, 100000, 400000, 1000000])),
                  crash_ppm=draw(st.sampled_from([0, 200000, 1000000])),
                  crash_len_max=draw(st.integers(1, 16)),
                  crash_start_max=draw(st.integers(0, 20)),
                  randomize=draw(st.booleans()))     # config-5 per-instance fuzzing
    if log_mode and draw(st.booleans()):
        kw.update(n_ticks=draw(st.integers(2, 8)), tick_period=draw(st.integers(1, 30)))
    return pxb.Config(**kw)


def _rcfg(cfg):
    return R.Config(**{k: getattr(cfg, k) for k in R.Config.__dataclass_fields__})


@SETTINGS
@given(cfg=configs(), first=st.integers(0, 2**40))
def test_c_restatement_equals_python_restatement(cfg, first):
    """oracle/paxos_oracle.c and oracle/paxos_ref.py are two restatements of
    the same handlers and schedule: results, digests, final acceptor records
    and the canonical byte count agree on any configuration."""
    n = 6
    res, dig, acc, cnt = oracle_c.run_cpu(cfg, first, n, threads=1, want_acceptors=True)
    rc = _rcfg(cfg)
    canon = 0
    for i in range(n):
        r = R.run_instance(rc, first + i)
        canon += r.canon_bytes
        assert list(res[i]) == [r.decided_val, r.decided_ticket, r.rounds, r.packed_flags()]
        assert list(dig[i]) == [r.digest(a) for a in range(cfg.n_acceptors)]
        assert [int(x) for x in acc[i, :, 3]] == [len(a.log) | (int(a.dead) << 31) for a in r.acceptors]
    assert cnt["canon_bytes"] == canon and cnt["instances"] == n


@SETTINGS
@given(cfg=configs(), first=st.integers(0, 2**40), split=st.integers(0, 24),
       threads=st.integers(1, 4))
def test_results_do_not_depend_on_sharding(cfg, first, split, threads):
    """SURVEY.md §8(e) G-invariance: every draw is keyed by the global instance
    id, so any contiguous split of a batch (and any thread count) gives the
    same per-instance results and the same summed totals."""
    n = 24
    whole = oracle_c.run_cpu(cfg, first, n, threads=1)
    a = oracle_c.run_cpu(cfg, first, split, threads=threads)
    b = oracle_c.run_cpu(cfg, first + split, n - split, threads=threads)
    assert np.array_equal(whole[0], np.concatenate([a[0], b[0]]))
    assert np.array_equal(whole[1], np.concatenate([a[1], b[1]]))
    for k, v in whole[3].items():
        assert v == a[3][k] + b[3][k], k


@SETTINGS
@given(seed=st.integers(0, 2**64 - 1), N=st.integers(2, 9), delay=st.integers(1, 15),
       skew=st.integers(0, 6), first=st.integers(0, 2**40))
def test_lone_proposer_without_loss_decides_its_own_command(seed, N, delay, skew, first):
    """One proposer, no loss, no crashes: per-link FIFO delivery makes every
    Ask granted (Server.hs:56-62), the majority Round1OKs carry no proposal
    (MostRecent = Nothing, Client.hs:157-170), so the proposer's own "c1.1"
    at ticket 1 is decided in one round (KAT-1 under any delay and skew)."""
    cfg = pxb.Config(seed=seed, n_proposers=1, n_acceptors=N, delay_max=delay, skew_max=skew,
                     step_cap=256)
    res, dig, acc, cnt = oracle_c.run_cpu(cfg, first, 16, threads=1, want_acceptors=True)
    assert (res[:, 0] == R.cmd_code(1, 1)).all()
    assert (res[:, 1] == 1).all() and (res[:, 2] == 1).all()
    assert ((res[:, 3] & 0xFF) == 0).all()
    assert (acc[:, :, 3] == 1).all()                 # one executed command, nobody dead
    assert cnt["decided"] == 16 and cnt["divergence"] == 0


@SETTINGS
@given(cfg=configs(faulty=False, log_mode=False), first=st.integers(0, 2**40))
def test_no_loss_single_decree_logs_never_diverge(cfg, first):
    """Without loss or crashes, the acceptors' executed logs
    (Server.hs:73-78) are prefixes of one another on the first slot: an
    Execute only lands where t_max equals its ticket, and the proposal stored
    under that ticket is the one the majority accepted."""
    if cfg.n_proposers > 1:
        cfg = pxb.Config(**{**cfg.__dict__, "n_proposers": 1})
    res, _, _, cnt = oracle_c.run_cpu(cfg, first, 16, threads=1)
    assert cnt["divergence"] == 0
    assert ((res[:, 3] & R.F_LOG_DIVERGENCE) == 0).all()


@settings(max_examples=200, deadline=None)
@given(t_max=st.integers(0, 40), t_store=st.integers(0, 40), has=st.booleans(),
       kind=st.sampled_from([R.ASK, R.PROPOSE, R.EXECUTE]), ticket=st.integers(0, 45),
       cid=st.integers(1, 3))
def test_acceptor_handler_invariants(t_max, t_store, has, kind, ticket, cid):
    """handleClientRequest (Server.hs:51-78): the largest issued ticket never
    decreases, a grant is exactly the strictly larger ticket, a proposal is
    stored only under the current ticket, and the C handler (the GPU hook's
    checker) makes the same transition as the Python one."""
    val = R.cmd_code(cid, 1) if has else R.NOTHING
    a = R.Acceptor(t_max=t_max, t_store=t_store if has else 0, val=val)
    before = (a.t_max, a.t_store, a.val)
    rep = R.acceptor_handle(a, kind, ticket, R.cmd_code(cid, 1))
    assert a.t_max >= before[0]
    if kind == R.ASK:
        assert (rep[0] == R.R1OK) == (ticket > before[0])
        assert a.t_max == max(before[0], ticket)
    if kind == R.PROPOSE:
        assert (rep[0] == R.R2S) == (ticket == before[0])
        assert (a.t_store == ticket) if rep[0] == R.R2S else (a.t_store, a.val) == before[1:]
    if kind == R.EXECUTE:
        assert rep is None
    st_in = np.array([[t_max, before[1], val, 0]], np.uint32)
    msg = np.array([[kind, ticket, 0, R.cmd_code(cid, 1)]], np.uint32)
    st2, crep = oracle_c.acceptor_handle(st_in, msg)
    exp = [pxb.MSG_NONE, 0, 0, 0] if rep is None else list(rep)
    assert list(crep[0]) == exp
    assert list(st2[0]) == [a.t_max, a.t_store, a.val, len(a.log) | (int(a.dead) << 31)]
