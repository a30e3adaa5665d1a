"""The per-lane kernel's state machine (csrc/paxos_ev.h), compiled for the HOST
(tests/native/ev_host.cpp) and diffed against the CPU oracle instance by
instance: results, log digests, final acceptor records and run totals.

This checks the exact code the GPU runs (EvLane::init/step/finish) without a
GPU; tests/test_gpu_parity.py then checks the device build end to end.
Instances the kernel hands to the general kernel ("bailed": a FIFO, pool or
ring capacity exceeded) are excluded here and must stay rare."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_c
import paxos_ref
import pxb

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "ev_host.cpp")
# PXB_EV_HOST_DEFS="-DX -DY": build the state machine with extra defines (kernel
# variants under evaluation) into a library of its own
DEFS = os.environ.get("PXB_EV_HOST_DEFS", "").split()
OUT = os.path.join(HERE, "native", "_build", "libev_host%s.so" % ("".join(d.replace("-D", "_") for d in DEFS)))
DEPS = [SRC] + [os.path.join(HERE, "..", "cloud-haskell-paxos_amd", "csrc", f)
                for f in ("paxos_ev.h", "paxos_ev_kernel.h", "paxos_device.h")] + [os.path.join(HERE, "..", "include", "paxos_batch.h")]
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in DEPS):
            os.makedirs(os.path.dirname(OUT), exist_ok=True)
            tmp = "%s.%d" % (OUT, os.getpid())          # (parallel workers: build, then rename)
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-fPIC", *DEFS,
                            "-shared", "-o", tmp, SRC], check=True)
            os.replace(tmp, OUT)
        _lib = C.CDLL(OUT)
    return _lib


def ev_run(cfg, first, n):
    N = cfg.n_acceptors
    res = np.zeros((n, 4), np.uint32)
    dig = np.zeros((n, N), np.uint32)
    acc = np.zeros((n, N, 4), np.uint32)
    tot = (C.c_int64 * 16)()
    bail = np.zeros(max(n, 1), np.uint32)
    nb, ms = C.c_uint32(0), C.c_uint64(0)
    c = cfg.to_c(first, n)
    p = lambda a: C.c_void_p(a.ctypes.data)  # noqa: E731
    rc = lib().ev_host_run(C.byref(c), p(res), p(dig), p(acc), tot, p(bail), C.byref(nb), C.byref(ms))
    assert rc == 0, "ev_host_run rc=%d" % rc
    return res, dig, acc, pxb.counters_dict(list(tot)), bail[:nb.value].copy()


def check(cfg, first, n, max_bail_frac=0.02):
    res, dig, acc, cnt, bails = ev_run(cfg, first, n)
    eres, edig, eacc, ecnt = oracle_c.run_cpu(cfg, first, n, threads=8, want_acceptors=True)
    ok = np.ones(n, bool)
    ok[bails] = False
    bad = np.nonzero(((res != eres).any(1) | (dig != edig).any(1) | (acc != eacc).any((1, 2))) & ok)[0]
    assert bad.size == 0, "instance %d: ev %s/%s oracle %s/%s" % (
        first + bad[0], res[bad[0]], acc[bad[0]].tolist(), eres[bad[0]], eacc[bad[0]].tolist())
    # totals: the oracle's minus the bailed instances' own
    for b in bails:
        _, _, _, bc = oracle_c.run_cpu(cfg, first + int(b), 1)
        for k in ecnt:
            ecnt[k] -= bc[k]
    assert cnt == ecnt
    assert len(bails) <= max_bail_frac * n + 1, "%d of %d instances bailed" % (len(bails), n)
    return res, cnt, bails


@pytest.mark.parametrize("c,n", [(3, 4000), (4, 3000), (5, 3000)])
def test_baseline_configs(c, n):
    """Default layouts (compact for configs 3 and 4): bails stay rare."""
    _, cnt, bails = check(pxb.CONFIGS[c], 0, n, max_bail_frac=0.02)
    if c == 3:
        assert len(bails) <= 2


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("N", [2, 3, 4, 5, 6, 7, 8, 9])
def test_topology_sweep(P, N):
    cfg = pxb.Config(seed=0x1234 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=150000,
                     delay_max=5, skew_max=2, crash_ppm=150000, crash_len_max=8,
                     crash_start_max=6, step_cap=200)
    check(cfg, 1000, 1500)


@pytest.mark.parametrize("kw", [
    dict(loss_ppm=0, delay_max=15),
    dict(loss_ppm=1000000),
    dict(loss_ppm=500000, step_cap=1),
    dict(crash_ppm=1000000, crash_len_max=1, crash_start_max=0),
    dict(skew_max=4096, step_cap=4095),
    dict(loss_ppm=350000, delay_max=15, step_cap=4095),
    dict(delay_max=2, crash_ppm=400000, crash_len_max=4096, crash_start_max=65535),
])
def test_edge_schedules(kw):
    base = dict(seed=99, n_proposers=2, n_acceptors=5)
    base.update(kw)
    check(pxb.Config(**base), 0, 1500, max_bail_frac=0.5)


def test_instance_ids_cross_32bit():
    check(pxb.CONFIGS[3], (1 << 32) - 1000, 2000)


@pytest.mark.parametrize("i", range(24))
def test_random_schedules(i):
    rng = np.random.default_rng(0xE7 + i)
    cfg = pxb.Config(
        seed=int(rng.integers(0, 1 << 63)), n_proposers=int(rng.integers(1, 4)),
        n_acceptors=int(rng.integers(2, 10)),
        loss_ppm=int(rng.choice([0, rng.integers(1, 600000), 1000000])),
        delay_max=int(rng.integers(2, 16)),
        crash_ppm=int(rng.choice([0, rng.integers(1, 1000001)])),
        crash_len_max=int(rng.integers(1, 40)), crash_start_max=int(rng.integers(0, 30)),
        skew_max=int(rng.choice([0, rng.integers(1, 12)])),
        step_cap=int(rng.choice([int(rng.integers(1, 64)), 256, 1024])),
        randomize=bool(rng.random() < 0.3))
    check(cfg, int(rng.integers(0, 1 << 34)), int(rng.integers(1, 800)), max_bail_frac=0.5)


@pytest.mark.parametrize("layout", [0, 2, 3, 5])
@pytest.mark.parametrize("c", [3, 4])
def test_layouts(c, layout, monkeypatch):
    """Every link layout (4-entry FIFOs; the compact 3-entry FIFOs with the
    reply seq packed beside the request FIFO, on the 8- and on the 4-step
    timing wheel; the slim 4-entry layout with byte reply seqs in registers)
    on the short-delay configs."""
    monkeypatch.setenv("EV_LAYOUT", str(layout))
    _, _, bails = check(pxb.CONFIGS[c], 5000, 2000, max_bail_frac=0.03)
    if layout in (0, 5):
        assert len(bails) == 0


@pytest.mark.parametrize("layout", [0, 5])
@pytest.mark.parametrize("pm", [2, 3])
def test_config5_8step_layouts(pm, layout, monkeypatch):
    """Config 5 (fuzzed P <= 3, delays to 8) on both 8-step-wheel layouts and
    both shapes of the split routing (EV_PM: the shape's proposer capacity;
    instances that drew more bail at init): the slim layout (byte reply seqs,
    4 ring slots, 44- / 30-word pools) bails about as rarely as the full one."""
    monkeypatch.setenv("EV_LAYOUT", str(layout))
    monkeypatch.setenv("EV_PM", str(pm))
    check(pxb.CONFIGS[5], 3000, 1500, max_bail_frac=0.75 if pm == 2 else 0.03)


def test_config5_three_proposer_deep_response_fifos(monkeypatch):
    """The slim three-proposer shape's 5-deep response FIFOs (entries pool
    index + 1, the tail's due read from its pool word): exact against the
    oracle, and config 5 bails ~0.4 % of its P = 3 instances (1.7 % with
    4-deep FIFOs, most of them on a full response FIFO)."""
    monkeypatch.setenv("EV_LAYOUT", "5")
    monkeypatch.setenv("EV_PM", "3")
    _, _, bails = check(pxb.CONFIGS[5], 9000, 6000, max_bail_frac=0.003)
    assert len(bails) > 0                            # (the pool and the rings still bail)


@pytest.mark.parametrize("layout", [6, 7])
@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("N", [2, 5, 7, 9])
def test_simple_schedule_layout(P, N, layout, monkeypatch):
    """Layout 6 (compact, 4-step wheel, simple schedule: no loss, no Tick
    skew, single decree; BASELINE config 4's routing): every proposer's Tick
    is handled at init and the sends skip the loss test.  Layout 7 is layout 6
    with 3-deep response FIFOs in halfwords and a 23-word pool (the first
    launch of config 4's tight routing).  Exact against the oracle on every
    topology."""
    monkeypatch.setenv("EV_LAYOUT", str(layout))
    cfg = pxb.Config(seed=0x51 + 16 * P + N, n_proposers=P, n_acceptors=N, delay_max=4,
                     crash_ppm=250000, crash_len_max=12, crash_start_max=10, step_cap=300)
    # (three proposers overflow the 3-deep response FIFOs of layout 7 often:
    # the routing takes it only for P <= 2)
    check(cfg, 99, 1200, max_bail_frac=0.5 if layout == 6 or P < 3 else 1.0)
    check(pxb.CONFIGS[4], 777, 1000, max_bail_frac=0.03)
    # a lossy or skewed batch is refused by the simple layouts
    with pytest.raises(AssertionError):
        ev_run(pxb.CONFIGS[3], 0, 10)


def test_tight_layout_config4(monkeypatch):
    """Config 4 on layout 7 (50 LDS words: 12 waves per CU): exact against the
    oracle, and it bails under 1 % of the instances (host model, 2^16: 0.76 %,
    60 % on a full 3-deep response FIFO, the rest on the 21-word pool), which
    the tight routing re-runs on layout 6."""
    monkeypatch.setenv("EV_LAYOUT", "7")
    _, _, bails = check(pxb.CONFIGS[4], 1 << 20, 6000, max_bail_frac=0.015)
    assert len(bails) > 0


@pytest.mark.parametrize("layout", [2, 3])
@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("N", [2, 5, 9])
def test_compact_layout_topologies(P, N, layout, monkeypatch):
    monkeypatch.setenv("EV_LAYOUT", str(layout))
    cfg = pxb.Config(seed=0x77 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=100000,
                     delay_max=4, skew_max=2, crash_ppm=150000, crash_len_max=8,
                     crash_start_max=6, step_cap=300)
    check(cfg, 77, 1200, max_bail_frac=0.5)


def test_bailed_instances_are_reported():
    """Long delays with duelling proposers overflow the 4-slot physical FIFOs:
    those instances are handed back (not silently wrong)."""
    cfg = pxb.Config(seed=7, n_proposers=3, n_acceptors=9, delay_max=15, skew_max=0, step_cap=300)
    _, _, bails = check(cfg, 0, 400, max_bail_frac=1.0)
    assert len(bails) > 0


@pytest.mark.parametrize("P,N", [(1, 9), (2, 5), (2, 9), (3, 9)])
def test_delay8_on_8step_wheel(P, N):
    """delay_max 8 runs on the 8-step timing wheel (due steps of the sends of
    step s, carried-over copies included, stay within s .. s + 8)."""
    cfg = pxb.Config(seed=0x8D + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=200000,
                     delay_max=8, skew_max=3, crash_ppm=200000, crash_len_max=16,
                     crash_start_max=16, step_cap=512)
    check(cfg, 4321, 1200, max_bail_frac=0.05)


@pytest.mark.parametrize("first", [0, (1 << 32) - 700])
def test_split_shape_config5(first, monkeypatch):
    """Config 5 split routing: a two-proposer shape runs the fuzzed instances
    that drew P <= 2 and hands every P = 3 instance (about a third) to the
    general kernel at init; what it runs matches the oracle exactly."""
    monkeypatch.setenv("EV_PM", "2")
    _, cnt, bails = check(pxb.CONFIGS[5], first, 1500, max_bail_frac=0.45)
    assert len(bails) > 300
    # exactly the P = 3 instances bail at init; capacity bails come on top
    drawn = np.array([paxos_ref.instance_params(pxb.CONFIGS[5], first + g).P for g in range(1500)])
    p3 = np.nonzero(drawn == 3)[0]
    assert set(p3.tolist()) <= set(bails.tolist())
    assert len(bails) - len(p3) <= 0.02 * 1500


# ---- log mode (docs/SEMANTICS.md §9) on the per-lane state machine's log-mode
# fields: periodic Ticks, 14-bit commands "c<id>.<t>", logs past LOG_TRACK ----
@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (1, 5, 0, 1, 8, 6, 0),
    (1, 3, 0, 1, 6, 2, 0),
    (2, 5, 50000, 3, 6, 9, 0),
    (3, 7, 150000, 4, 5, 20, 150000),
    (2, 9, 0, 6, 12, 5, 300000),
    (3, 4, 300000, 8, 16, 3, 0),
    (2, 2, 0, 1, 16, 8, 0),              # the stock Main.hs topology, fault-free
    (2, 5, 100000, 4, 16, 4, 200000)])   # BASELINE-like faulty log mode
def test_log_mode(P, N, loss, delay, ticks, period, crash):
    cfg = pxb.Config(seed=0x1060 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=3, crash_ppm=crash, crash_len_max=12,
                     crash_start_max=30, step_cap=1024, n_ticks=ticks, tick_period=period)
    _, cnt, _ = check(cfg, 321, 1500, max_bail_frac=0.05)
    assert cnt["executes"] >= cnt["decided"]


@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (2, 5, 100000, 4, 16, 8, 200000),    # faulty log mode (BASELINE-like, extra.log_mode_faulty)
    (1, 9, 300000, 8, 10, 3, 300000),
    (3, 3, 200000, 6, 12, 5, 100000),
    (2, 2, 0, 1, 16, 8, 0)])
def test_log_mode_second_stage_layout(P, N, loss, delay, ticks, period, crash, monkeypatch):
    """Layout 8, the log-mode shape on the 16-step wheel with its topology's
    larger pool (32 words over <= 10 links): the second stage of two-stage
    faulty log mode (pxb_run_device re-runs the first stage's hand-offs on
    it).  Exact against the oracle, and it hands on nothing here."""
    monkeypatch.setenv("EV_LAYOUT", "8")
    cfg = pxb.Config(seed=0x1C8 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=3, crash_ppm=crash, crash_len_max=12,
                     crash_start_max=30, step_cap=1024, n_ticks=ticks, tick_period=period)
    _, cnt, bails = check(cfg, 77, 1500, max_bail_frac=0.0)
    assert cnt["executes"] >= cnt["decided"] and len(bails) == 0


@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (2, 5, 100000, 4, 16, 8, 200000),    # faulty log mode (BASELINE-like, extra.log_mode_faulty)
    (1, 9, 300000, 4, 10, 3, 300000),
    (3, 3, 200000, 3, 12, 5, 100000),
    (2, 2, 0, 1, 16, 8, 0),
    (2, 4, 0, 4, 16, 2, 0),              # responses pile up
    (1, 5, 10000, 2, 100, 8, 150000)])   # logs past LOG_TRACK: every packed canonical-log position
def test_log_mode_slim_4step_layout(P, N, loss, delay, ticks, period, crash, monkeypatch):
    """Layout 9: the log-mode shape with byte reply seqs in registers, on the
    4-step wheel, its canonical log packed (14 words), a 19-word pool (75 LDS
    words, 8 waves per CU): the first stage of log mode with delays <= 4 over
    <= 10 links.  Exact against the oracle, its hand-offs rare."""
    monkeypatch.setenv("EV_LAYOUT", "9")
    cfg = pxb.Config(seed=0x1C9 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=3, crash_ppm=crash, crash_len_max=12,
                     crash_start_max=30, step_cap=1024, n_ticks=ticks, tick_period=period)
    _, cnt, bails = check(cfg, 91, 1500, max_bail_frac=0.01)
    assert cnt["executes"] >= cnt["decided"]


@pytest.mark.parametrize("P,loss,crash,period,delay,clen",[(1, 10000, 150000, 8, 2, 20), (2, 0, 100000, 12, 1, 30)])
def test_log_mode_past_log_track(P, loss, crash, period, delay, clen):
    """100 Ticks per proposer: logs past LOG_TRACK = 32 set LOG_TRUNC; the
    divergence check covers the first 32 positions (as the oracle's)."""
    cfg = pxb.Config(seed=0x7A0C + P, n_proposers=P, n_acceptors=5, loss_ppm=loss, delay_max=delay, skew_max=2,
                     crash_ppm=crash, crash_len_max=clen, crash_start_max=400 if P == 1 else 600, step_cap=2048,
                     n_ticks=100, tick_period=period)
    res, cnt, _ = check(cfg, 11, 600, max_bail_frac=0.05)
    assert cnt["log_trunc"] > 0 and cnt["divergence"] > 0


@pytest.mark.parametrize("i", range(12))
def test_random_log_mode_schedules(i):
    rng = np.random.default_rng(0x10E7 + i)
    cfg = pxb.Config(
        seed=int(rng.integers(0, 1 << 63)), n_proposers=int(rng.integers(1, 4)),
        n_acceptors=int(rng.integers(2, 10)),
        loss_ppm=int(rng.choice([0, rng.integers(1, 400000)])),
        delay_max=int(rng.integers(1, 9)),
        crash_ppm=int(rng.choice([0, rng.integers(1, 600000)])),
        crash_len_max=int(rng.integers(1, 40)), crash_start_max=int(rng.integers(0, 200)),
        skew_max=int(rng.choice([0, rng.integers(1, 12)])),
        step_cap=int(rng.choice([int(rng.integers(1, 64)), 512, 2048])),
        n_ticks=int(rng.integers(2, 60)), tick_period=int(rng.integers(1, 16)),
        randomize=bool(rng.random() < 0.3))
    check(cfg, int(rng.integers(0, 1 << 34)), int(rng.integers(1, 500)), max_bail_frac=0.5)


# LDS per lane of the shapes the bench workloads run, and the residency it buys.
# A 64-lane block of W words takes 256 W bytes of the CU's 160 KiB; blocks that
# fill it to within ~1 KiB measured no gain ("LDS to spare"; LDS
# is allocated in 1 KiB steps per block), so every shape keeps >= 4 KiB free at
# its residency (round 5: the tight layout's 12 x 13 KiB, measured resident).
@pytest.mark.parametrize("c,pm,layout,words,blocks", [
    (4, 2, None, 60, 10),   # compact, 4-step wheel (layout 6: the tight routing's second launch)
    (4, 2, "7", 50, 12),    # tight (layout 7: halfword response FIFOs, 21-word pool)
    (3, 2, None, 44, 12),   # compact, 16-word pool (12 = the VGPR limit)
    (5, 3, None, 120, 5),   # slim, P = 3 share
    (5, 2, None, 75, 8),    # slim, P <= 2 share (halfword response links, 28-word pool)
    (7, 2, None, 86, 7),    # faulty log mode (layout 4, 19-word pool: delays above 4)
    (7, 2, "9", 75, 8),     # faulty log mode's first stage (layout 9: byte reply seqs, 4-step wheel, packed log)
])
def test_layout_words_leave_lds_to_spare(c, pm, layout, words, blocks, monkeypatch):
    if layout:
        monkeypatch.setenv("EV_LAYOUT", layout)
    cfg = pxb.CONFIGS[c]
    if pm != cfg.n_proposers:
        monkeypatch.setenv("EV_PM", str(pm))
    ev_run(cfg, 0, 1)
    assert lib().ev_host_last_words() == words
    assert blocks * ((256 * words + 1023) // 1024) <= 160 - 4



# ---- the hand-derived step-schedule KATs (tests/golden/kat_step_schedule.json)
# on the host build of the per-lane state machine: every case, whatever layout
# its config routes to (S4/S5: faulty log mode; S6: the randomized draw) ----
_KATS = __import__("json").load(open(os.path.join(HERE, "golden", "kat_step_schedule.json")))["cases"]


@pytest.mark.parametrize("case", _KATS, ids=[c["name"] for c in _KATS])
def test_step_kats_on_host(case):
    cfg = pxb.Config(**case["config"])
    want = case["result"]
    res, dig, acc, cnt, bails = ev_run(cfg, case["instance"], 1)
    assert len(bails) == 0
    assert list(res[0]) == [want["decided_val"], want["decided_ticket"], want["rounds"],
                            want["flags"] | (want["steps"] << 16)]
    assert (cnt["messages"], cnt["canon_bytes"], cnt["executes"]) == \
        (want["messages"], want["canon_bytes"], want["executes"])
    final = [cp for cp in case["checkpoints"] if cp["step"] == want["steps"] - 1][0]
    assert acc[0].tolist() == final["acc"]
