"""The per-lane kernel's state machine (csrc/paxos_ev.h) built for the HOST with
AddressSanitizer + UndefinedBehaviorSanitizer (no recovery: the first report
aborts) and a checked LDS accessor (every word / halfword index asserted
against the shape's S::WORDS before the access; the buffer holds exactly those
words, so ASan also sees any access past them), then run over the host matrix
and diffed against the CPU oracle like tests/test_ev_host.py.  The build also
turns shift-count warnings into errors: a shift by >= 32 in a branch that a
shape never takes (8108609: `15u << S::RD` with RD = 33 in the slim >18-link
response word) is UB that no runtime check sees.

The sanitizers run on host code only (the GPU box has no GPU ASan); the
device build of the same code is checked end to end by tests/test_gpu_parity.py.
"""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_c
import pxb

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "ev_host.cpp")
EXE = os.path.join(HERE, "native", "_build", "ev_host_san")
DEPS = [SRC] + [os.path.join(ROOT, "cloud-haskell-paxos_amd", "csrc", f)
                for f in ("paxos_ev.h", "paxos_ev_kernel.h", "paxos_device.h")] + \
       [os.path.join(ROOT, "include", "paxos_batch.h")]
FLAGS = ["--offload-arch=gfx950", "-O1", "-g0", "-std=c++17", "-DPXB_HOST_CHECKED", "-DPXB_EV_HOST_MAIN",
         "-DPXB_EV_HOST_FEW_N",
         "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
         "-Xarch_host", "-fno-sanitize-recover=all",
         "-Werror=shift-count-overflow", "-Werror=shift-count-negative"]


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(EXE) or any(os.path.getmtime(d) > os.path.getmtime(EXE) for d in DEPS):
        os.makedirs(os.path.dirname(EXE), exist_ok=True)
        # (built under a name of its own, then renamed: parallel test workers may
        # build at once, and none may run a half-written binary)
        tmp = "%s.%d" % (EXE, os.getpid())
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-o", tmp, SRC], check=True, timeout=600)
        os.replace(tmp, EXE)
    return EXE


def san_run(exe, cfg, first, n, env=None):
    """One batch through the sanitized state machine: results, digests,
    acceptor records, totals, bailed ids."""
    N = cfg.n_acceptors
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "o.bin")
        args = [exe, out, hex(cfg.seed), str(first), str(n), str(cfg.n_proposers), str(N), str(cfg.loss_ppm),
                str(cfg.delay_max), str(cfg.crash_ppm), str(cfg.crash_len_max), str(cfg.crash_start_max),
                str(cfg.skew_max), str(cfg.step_cap), str(pxb.CFG_RANDOMIZE if cfg.randomize else 0),
                str(cfg.n_ticks), str(cfg.tick_period)]
        e = dict(os.environ)
        e.update(env or {})
        e["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
        p = subprocess.run(args, capture_output=True, text=True, env=e, timeout=600)
        assert p.returncode == 0, "sanitized run failed (rc %d): %s" % (p.returncode, p.stderr[-4000:])
        w = np.fromfile(out, dtype=np.uint32)
    rc, nn, NN, nb = (int(x) for x in w[:4])
    assert rc == 0 and nn == n and NN == N
    o = 4
    res = w[o:o + 4 * n].reshape(n, 4); o += 4 * n
    dig = w[o:o + n * N].reshape(n, N); o += n * N
    acc = w[o:o + 4 * n * N].reshape(n, N, 4); o += 4 * n * N
    tot = w[o:o + 32].view(np.int64); o += 32
    bails = w[o:o + nb]
    return res, dig, acc, pxb.counters_dict(list(tot)), bails


def check(exe, cfg, first, n, env=None, max_bail_frac=0.05):
    res, dig, acc, cnt, bails = san_run(exe, cfg, first, n, env)
    eres, edig, eacc, ecnt = oracle_c.run_cpu(cfg, first, n, threads=8, want_acceptors=True)
    ok = np.ones(n, bool)
    ok[bails] = False
    bad = np.nonzero(((res != eres).any(1) | (dig != edig).any(1) | (acc != eacc).any((1, 2))) & ok)[0]
    assert bad.size == 0, "instance %d differs from the oracle" % (first + bad[0])
    for b in bails:
        _, _, _, bc = oracle_c.run_cpu(cfg, first + int(b), 1)
        for k in ecnt:
            ecnt[k] -= bc[k]
    assert cnt == ecnt
    assert len(bails) <= max_bail_frac * n + 1
    return cnt, bails


# (layout, config, EV_PM): every layout, the BASELINE configs on their own routing
@pytest.mark.parametrize("layout,c,pm", [
    (None, 3, None),        # compact, 4-step wheel (layout 3)
    (None, 4, None),        # simple schedule (layout 6)
    ("7", 4, None),         # tight simple schedule (layout 7: halfword response FIFOs with a sentinel)
    ("3", 4, None),         # config 4 on the general compact layout
    ("2", 3, None),         # compact, 8-step wheel
    ("0", 3, None),         # 4-entry FIFOs, 8-step wheel
    (None, 5, "2"),         # slim, the two-proposer share of the split routing
    (None, 5, "3"),         # slim, three proposers (5-deep response FIFOs)
    ("0", 5, "3"),
])
def test_baseline_layouts_sanitized(exe, layout, c, pm):
    env = {}
    if layout:
        env["EV_LAYOUT"] = layout
    if pm:
        env["EV_PM"] = pm
    check(exe, pxb.CONFIGS[c], 2024, 600, env, max_bail_frac=0.75 if pm == "2" else 0.05)


@pytest.mark.parametrize("P,N", [(1, 2), (2, 5), (2, 9), (3, 9)])
def test_tight_layout_topologies_sanitized(exe, P, N):
    """Layout 7 on small and large topologies: its 5-bit response entries
    (pool index + 1, or a Round2Success code) index only the lane's words (the
    checked accessor asserts it; small shapes clamp a code's unused pool load)."""
    cfg = pxb.Config(seed=0x7A + 16 * P + N, n_proposers=P, n_acceptors=N, delay_max=4, crash_ppm=250000,
                     crash_len_max=12, crash_start_max=10, step_cap=300)
    check(exe, cfg, 99, 300, {"EV_LAYOUT": "7"}, max_bail_frac=1.0)


@pytest.mark.parametrize("P,N,delay", [(1, 9, 12), (3, 9, 15), (2, 5, 9)])
def test_16step_wheel_sanitized(exe, P, N, delay):
    """Layout 1 (16-step wheel: delays above 8)."""
    cfg = pxb.Config(seed=0x5A + P * 16 + N, n_proposers=P, n_acceptors=N, loss_ppm=150000, delay_max=delay,
                     skew_max=3, crash_ppm=150000, crash_len_max=10, crash_start_max=12, step_cap=600)
    check(exe, cfg, 31, 300, max_bail_frac=0.5)


@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (2, 2, 0, 1, 16, 8, 0),                 # the stock Main.hs topology
    (2, 5, 100000, 4, 16, 8, 200000),       # faulty log mode (bench extra.log_mode_faulty)
    (3, 7, 150000, 4, 5, 20, 150000),
    (1, 5, 10000, 2, 100, 8, 150000),       # logs past LOG_TRACK
])
def test_log_mode_sanitized(exe, P, N, loss, delay, ticks, period, crash):
    cfg = pxb.Config(seed=0x1061 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss, delay_max=delay,
                     skew_max=3, crash_ppm=crash, crash_len_max=12, crash_start_max=30,
                     step_cap=2048 if ticks > 50 else 1024, n_ticks=ticks, tick_period=period)
    check(exe, cfg, 321, 300)


@pytest.mark.parametrize("layout", ["8", "9"])
@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (2, 5, 100000, 4, 16, 8, 200000),       # faulty log mode (bench extra.log_mode_faulty)
    (1, 5, 10000, 2, 100, 8, 150000),       # logs past LOG_TRACK: every packed canonical-log position
    (2, 5, 0, 4, 16, 2, 0),                 # responses pile up (the sanitized build has N = 2, 5, 7, 9)
])
def test_log_mode_stages_sanitized(exe, layout, P, N, loss, delay, ticks, period, crash):
    """The two-stage log mode's shapes: layout 9 (first stage, delays <= 4:
    byte reply seqs, 4-step wheel, the canonical log's 14-bit commands packed
    across words) and layout 8 (second stage: 16-step wheel, 32-word pool),
    with every word and halfword index checked."""
    cfg = pxb.Config(seed=0x1D61 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss, delay_max=delay,
                     skew_max=3, crash_ppm=crash, crash_len_max=12, crash_start_max=30,
                     step_cap=2048 if ticks > 50 else 1024, n_ticks=ticks, tick_period=period)
    check(exe, cfg, 55, 300, {"EV_LAYOUT": layout}, max_bail_frac=0.05)


@pytest.mark.parametrize("i", range(8))
def test_random_schedules_sanitized(exe, i):
    rng = np.random.default_rng(0x5A71 + i)
    N = int(rng.choice([2, 5, 7, 9]))
    cfg = pxb.Config(
        seed=int(rng.integers(0, 1 << 63)), n_proposers=int(rng.integers(1, 4)), n_acceptors=N,
        loss_ppm=int(rng.choice([0, rng.integers(1, 400000)])), delay_max=int(rng.integers(1, 16)),
        crash_ppm=int(rng.choice([0, rng.integers(1, 600000)])), crash_len_max=int(rng.integers(1, 40)),
        crash_start_max=int(rng.integers(0, 30)), skew_max=int(rng.choice([0, rng.integers(1, 12)])),
        step_cap=int(rng.choice([int(rng.integers(1, 64)), 256, 1024])),
        n_ticks=int(rng.choice([1, 1, rng.integers(2, 20)])), tick_period=int(rng.integers(1, 12)),
        randomize=bool(rng.random() < 0.3))
    if cfg.n_ticks > 1 and cfg.delay_max > 8:
        cfg.delay_max = 8                   # (log mode runs on the 8-step wheel only)
    check(exe, cfg, int(rng.integers(0, 1 << 34)), 250, max_bail_frac=0.6)


def test_ids_crossing_2p32_sanitized(exe):
    check(exe, pxb.CONFIGS[4], (1 << 32) - 150, 300)


def test_checked_build_flags_out_of_range_shifts():
    """The sanitizer build's -Werror=shift-count-overflow rejects the
    out-of-range shift constant that 8108609 removed: reintroduced into a
    scratch copy of the sources, the build fails."""
    with tempfile.TemporaryDirectory() as td:
        for d in ("cloud-haskell-paxos_amd/csrc", "include"):
            shutil.copytree(os.path.join(ROOT, d), os.path.join(td, d),
                            ignore=shutil.ignore_patterns("_build", "*.so", "*.o"))
        os.makedirs(os.path.join(td, "tests", "native"))
        shutil.copy(SRC, os.path.join(td, "tests", "native"))
        h = os.path.join(td, "cloud-haskell-paxos_amd", "csrc", "paxos_ev.h")
        s = open(h).read()
        good = "& ~(15u << RD)) | (due4 << RD);"
        assert good in s
        open(h, "w").write(s.replace(good, "& ~(15u << S::RD)) | (due4 << S::RD);"))
        p = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-fsyntax-only",
                            os.path.join(td, "tests", "native", "ev_host.cpp")],
                           capture_output=True, text=True, timeout=600)
        assert p.returncode != 0 and "shift count >= width of type" in p.stderr
