"""GPU parity: the HIP path (through the C ABI) against the CPU oracle,
bit-exact on results, per-acceptor log digests, final acceptor records and
run counters; plus size-independent properties at BASELINE.json sizes."""
import os

import numpy as np
import pytest

import oracle_c
import pxb

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
THREADS = min(16, os.cpu_count() or 1)


def _fnv(h, v):
    """FNV-1a-32 over the 4 little-endian bytes of v (SEMANTICS §7)."""
    for i in range(4):
        h = ((h ^ ((v >> (8 * i)) & 0xFF)) * 0x01000193) & 0xFFFFFFFF
    return h


def _cmp(cfg, first, n, want_acc=True):
    res, dig, acc, cnt = pxb.run(cfg, first, n, want_acceptors=want_acc)
    eres, edig, eacc, ecnt = oracle_c.run_cpu(cfg, first, n, threads=THREADS, want_acceptors=want_acc)
    bad = np.nonzero((res != eres).any(axis=1))[0]
    assert bad.size == 0, "first mismatching instance %d: gpu %s oracle %s" % (
        first + bad[0], res[bad[0]], eres[bad[0]])
    assert np.array_equal(dig, edig)
    if want_acc:
        assert np.array_equal(acc, eacc)
    assert cnt == ecnt
    return res, cnt


@pytest.mark.parametrize("c,n", [(1, 8192), (2, 262144), (3, 65536), (4, 8192), (5, 16384)])
def test_configs_match_oracle(gpu_lib, c, n):
    _cmp(pxb.CONFIGS[c], 0, n)


@pytest.mark.parametrize("path", sorted(p for p in os.listdir(GOLDEN) if p.endswith(".npz")))
def test_golden_fixtures(gpu_lib, path):
    z = np.load(os.path.join(GOLDEN, path))
    c, first, n = (int(x) for x in z["meta"])
    res, dig, acc, cnt = pxb.run(pxb.CONFIGS[c], first, n, want_acceptors=True)
    assert np.array_equal(res, z["results"])
    assert np.array_equal(dig, z["digests"])
    assert np.array_equal(acc, z["acceptors"])
    assert cnt["canon_bytes"] == int(z["canon_bytes"][0])


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("N", [2, 3, 4, 5, 6, 7, 8, 9])
def test_topology_sweep(gpu_lib, P, N):
    cfg = pxb.Config(seed=0x1234 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=150000,
                     delay_max=5, skew_max=2, crash_ppm=150000, crash_len_max=8,
                     crash_start_max=6, step_cap=200)
    _cmp(cfg, 1000, 3001)


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("N", [2, 3, 5, 8, 9])
def test_fault_free_topology_sweep(gpu_lib, P, N):
    """Fault-free schedules run the FF kernels (due counts from queue lengths,
    no Philox): duelling proposers with Tick skew, single decree and log mode."""
    for ticks in (1, 5):
        cfg = pxb.Config(seed=0xFF00 + 16 * P + N, n_proposers=P, n_acceptors=N, skew_max=2,
                         step_cap=600, n_ticks=ticks, tick_period=7)
        _cmp(cfg, 77, 2501)


@pytest.mark.parametrize("kw", [
    dict(loss_ppm=0, delay_max=15),                 # max delay, FIFO max() rule
    dict(loss_ppm=1000000),                          # everything lost
    dict(loss_ppm=500000, step_cap=1),               # cap at the first step
    dict(crash_ppm=1000000, crash_len_max=1, crash_start_max=0),
    dict(skew_max=4096, step_cap=8192),              # long idle gaps
    dict(loss_ppm=350000, delay_max=15, step_cap=8192),
])
def test_edge_schedules(gpu_lib, kw):
    base = dict(seed=99, n_proposers=2, n_acceptors=5)
    base.update(kw)
    _cmp(pxb.Config(**base), 0, 2000)


# ---- log mode (docs/SEMANTICS.md §9): periodic Ticks, Execute-driven slots -------
@pytest.mark.parametrize("P,N,loss,delay,ticks,period,crash", [
    (1, 5, 0, 1, 8, 6, 0),            # every Tick commits (period > one slot)
    (1, 3, 0, 1, 6, 2, 0),            # Ticks while busy are dropped
    (2, 5, 50000, 3, 6, 9, 0),        # duelling proposers, Q5 re-proposals in the log
    (3, 7, 150000, 4, 5, 20, 150000),
    (2, 9, 0, 6, 12, 5, 300000),
    (3, 4, 300000, 8, 16, 3, 0)])
def test_log_mode_matches_oracle(gpu_lib, P, N, loss, delay, ticks, period, crash):
    cfg = pxb.Config(seed=0x1060 + 16 * P + N, n_proposers=P, n_acceptors=N, loss_ppm=loss,
                     delay_max=delay, skew_max=3, crash_ppm=crash, crash_len_max=12,
                     crash_start_max=30, step_cap=1024, n_ticks=ticks, tick_period=period)
    res, cnt = _cmp(cfg, 321, 4001)
    assert cnt["executes"] >= cnt["decided"]


@pytest.mark.parametrize("P,loss,crash,period,delay,clen", [(1, 10000, 150000, 8, 2, 20), (2, 0, 100000, 12, 1, 30)])
def test_log_mode_past_log_track(gpu_lib, P, loss, crash, period, delay, clen):
    """Faulty log mode with 100 Ticks per proposer: logs grow past LOG_TRACK = 32
    positions (SEMANTICS §7, §9).  LOG_TRUNC, LOG_DIVERGENCE (checked over the
    first 32 positions only), the digests of the whole logs and the log lengths
    equal the oracle's, instance by instance; the batch holds truncated
    instances, divergent ones, and truncated divergent ones."""
    cfg = pxb.Config(seed=0x7A0C + P, n_proposers=P, n_acceptors=5, loss_ppm=loss, delay_max=delay, skew_max=2,
                     crash_ppm=crash, crash_len_max=clen, crash_start_max=400 if P == 1 else 600, step_cap=2048,
                     n_ticks=100, tick_period=period)
    res, cnt = _cmp(cfg, 11, 3000)
    flags = res[:, 3] & 0xFF
    trunc = (flags & pxb.F_LOG_TRUNC) != 0
    div = (flags & pxb.F_LOG_DIVERGENCE) != 0
    assert cnt["log_trunc"] == int(trunc.sum()) > 0 and cnt["divergence"] == int(div.sum())
    assert trunc.sum() > 100 and div.sum() > 0 and (trunc & div).sum() > 0, (trunc.sum(), div.sum())
    _, _, acc, _ = pxb.run(cfg, 11, 200, want_acceptors=True)
    assert ((acc[:, :, 3] & 0x7FFFFFFF) > 32).any()


@pytest.mark.parametrize("n", [1 << 20, 1 << 25])
def test_log_mode_full_size_properties(gpu_lib, n):
    """Fault-free log mode: every one of the 8 Ticks commits its own command,
    so every acceptor log is c1.1 .. c1.8.  2^25 instances take two launches
    (16-bit canonical-log epochs cap a launch at 60000 instances per block)."""
    cfg = pxb.Config(seed=0x5EED0006, n_proposers=1, n_acceptors=5, n_ticks=8, tick_period=6)
    res, dig, _, cnt = pxb.run(cfg, 0, n)
    assert cnt["executes"] == 8 * n and cnt["rounds"] == 8 * n and cnt["decided"] == n
    assert (res[:, 3] == ((7 * 6 + 6) << 16)).all()
    _, edig, _, _ = oracle_c.run_cpu(cfg, 0, 1)
    assert (dig == edig[0]).all()


@pytest.mark.parametrize("n", [1, 7, 63, 64, 65, 1000])
def test_ragged_batch_sizes(gpu_lib, n):
    _cmp(pxb.CONFIGS[3], 5, n)


@pytest.mark.parametrize("n", [1, 11, 12, 13, 143, 144, 145, 4097, 50001])
@pytest.mark.parametrize("c", [2, 6, "p3"])
def test_ragged_block_queue_sizes(gpu_lib, c, n):
    """Fault-free kernels run multi-wave blocks that share the block's range
    through an LDS counter, one slot-generation (G instances) per grab: batch
    sizes around G, the block width and the grid edge."""
    cfg = pxb.Config(seed=0x3F, n_proposers=3, n_acceptors=4, skew_max=2) if c == "p3" else pxb.CONFIGS[c]
    _cmp(cfg, 9, n)


def test_instance_ids_cross_32bit(gpu_lib):
    _cmp(pxb.CONFIGS[3], (1 << 32) - 3000, 6000)


def test_empty_batch(gpu_lib):
    res, dig, acc, cnt = pxb.run(pxb.CONFIGS[2], 0, 0)
    assert cnt["instances"] == 0


def test_shard_invariance(gpu_lib):
    """Results depend only on (seed, global instance id): sharded runs
    concatenate to the unsharded run (the multi-GPU contract)."""
    cfg = pxb.CONFIGS[5]
    n = 40000
    full, dfull, _, cfull = pxb.run(cfg, 0, n)
    parts, cnts = [], []
    for k in range(4):
        r, d, _, c = pxb.run(cfg, k * n // 4, n // 4)
        parts.append((r, d))
        cnts.append(c)
    assert np.array_equal(full, np.concatenate([p[0] for p in parts]))
    assert np.array_equal(dfull, np.concatenate([p[1] for p in parts]))
    for key in cfull:
        assert cfull[key] == sum(c[key] for c in cnts)


def test_config2_full_size_properties(gpu_lib):
    """BASELINE config 2 at full size (2^20): every instance decides c1.1 at
    ticket 1 in one round, 6 steps, no flag; totals = closed forms."""
    n = pxb.CONFIG_INSTANCES[2]
    res, dig, _, cnt = pxb.run(pxb.CONFIGS[2], 0, n)
    assert (res[:, 0] == pxb.command(1, 1)).all() and (res[:, 1] == 1).all()
    assert (res[:, 2] == 1).all() and (res[:, 3] == (6 << 16)).all()
    assert (dig == dig[0, 0]).all()
    assert cnt["decided"] == n and cnt["messages"] == 25 * n
    assert cnt["canon_bytes"] == pxb.canonical_bytes_nofault(5) * n


def test_config3_full_size_sampled(gpu_lib):
    """BASELINE config 3 at full size (2^24): a random sample of instances
    checked against the oracle, plus counter consistency."""
    cfg = pxb.CONFIGS[3]
    n = pxb.CONFIG_INSTANCES[3]
    res, dig, _, cnt = pxb.run(cfg, 0, n)
    assert cnt["instances"] == n and cnt["decided"] + cnt["undecided"] == n
    flags = res[:, 3] & 0xFF
    assert cnt["undecided"] == int(((flags & pxb.F_UNDECIDED) != 0).sum())
    assert cnt["divergence"] == int(((flags & pxb.F_LOG_DIVERGENCE) != 0).sum())
    assert cnt["rounds"] == int(res[:, 2].astype(np.int64).sum())
    rng = np.random.default_rng(3)
    for i in rng.choice(n, 64, replace=False):
        eres, edig, _, _ = oracle_c.run_cpu(cfg, int(i), 1)
        assert np.array_equal(res[i], eres[0]) and np.array_equal(dig[i], edig[0])


def test_config5_per_gpu_share_sampled(gpu_lib):
    """BASELINE config 5 at its per-GPU share (2^28 over 8 GPUs = 2^25
    instances in one call): totals equal the per-instance flags, and a random
    sample of 64 instances matches the oracle bit-exact."""
    cfg = pxb.CONFIGS[5]
    n = pxb.CONFIG_INSTANCES[5] // 8
    res, dig, _, cnt = pxb.run(cfg, 0, n)
    assert cnt["instances"] == n and cnt["decided"] + cnt["undecided"] == n
    flags = res[:, 3] & 0xFF
    for key, bit in (("undecided", pxb.F_UNDECIDED), ("stuck", pxb.F_STUCK), ("panic", pxb.F_PANIC),
                     ("divergence", pxb.F_LOG_DIVERGENCE), ("step_cap", pxb.F_STEP_CAP)):
        assert cnt[key] == int(((flags & bit) != 0).sum()), key
    assert cnt["rounds"] == int(res[:, 2].astype(np.int64).sum())
    assert cnt["steps"] == int((res[:, 3] >> 16).astype(np.int64).sum())
    rng = np.random.default_rng(55)
    for i in rng.choice(n, 64, replace=False):
        eres, edig, _, _ = oracle_c.run_cpu(cfg, int(i), 1)
        assert np.array_equal(res[i], eres[0]) and np.array_equal(dig[i], edig[0])


def test_config4_north_star_full_size_sampled(gpu_lib):
    """The north star at its size on one GPU: BASELINE config 4, 2^26
    instances in one call (one per-lane chunk, its bailed instances on the
    general kernel): totals equal the per-instance flags and 64 random
    instances match the oracle bit-exact."""
    cfg = pxb.CONFIGS[4]
    n = 1 << 26
    res, dig, _, cnt = pxb.run(cfg, 0, n)
    assert cnt["instances"] == n and cnt["decided"] + cnt["undecided"] == n
    flags = res[:, 3] & 0xFF
    for key, bit in (("undecided", pxb.F_UNDECIDED), ("stuck", pxb.F_STUCK), ("panic", pxb.F_PANIC),
                     ("divergence", pxb.F_LOG_DIVERGENCE), ("step_cap", pxb.F_STEP_CAP)):
        assert cnt[key] == int(((flags & bit) != 0).sum()), key
    assert cnt["rounds"] == int(res[:, 2].astype(np.int64).sum())
    assert cnt["steps"] == int((res[:, 3] >> 16).astype(np.int64).sum())
    rng = np.random.default_rng(44)
    for i in rng.choice(n, 64, replace=False):
        eres, edig, _, _ = oracle_c.run_cpu(cfg, int(i), 1)
        assert np.array_equal(res[i], eres[0]) and np.array_equal(dig[i], edig[0])


@pytest.mark.parametrize("cap", [0, 3, 1 << 20])
def test_per_lane_bail_list_overflow(gpu_lib, cap):
    """Instances the per-lane kernel cannot hold go to a capped id list for the
    general kernel; when the list overflows, the general kernel re-runs the
    whole chunk and the per-lane totals are dropped.  Results and totals stay
    exact either way (config 4 bails ~1.4 % of instances)."""
    with pxb.hooks(PXB_EV_BAIL_CAP=str(cap)):
        _cmp(pxb.CONFIGS[4], 1 << 30, 30000)


def test_per_lane_matches_general_kernel(gpu_lib):
    """The per-lane kernel (default for faulty single-decree batches) and the
    general kernel (PXB_NO_EV=1) give identical results, digests and totals."""
    cfg = pxb.CONFIGS[4]
    a = pxb.run(cfg, 777, 50000, want_acceptors=True)
    with pxb.hooks(PXB_NO_EV="1"):
        b = pxb.run(cfg, 777, 50000, want_acceptors=True)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3] == b[3]


@pytest.mark.parametrize("first", [4242, (1 << 32) - 30000])
def test_config5_split_matches_other_routings(gpu_lib, first):
    """Config 5 (fuzzed P up to 3, N = 9) runs split: the two-proposer per-lane
    shape over the chunk, the three-proposer shape over the instances that drew
    P = 3, the general kernel over the rest's bails.  Identical to the
    three-proposer shape alone (PXB_NO_SPLIT=1) and to the general kernel
    alone (PXB_NO_EV=1)."""
    cfg = pxb.CONFIGS[5]
    a = pxb.run(cfg, first, 60000, want_acceptors=True)
    for env in ("PXB_NO_SPLIT", "PXB_NO_EV"):
        with pxb.hooks(**{env: "1"}):
            b = pxb.run(cfg, first, 60000, want_acceptors=True)
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y), env
        assert a[3] == b[3], env


def _with_env(env, fn):
    with pxb.hooks(**env):
        return fn()


@pytest.mark.parametrize("first", [31337, (1 << 32) - 25000])
def test_config4_tight_matches_other_routings(gpu_lib, first):
    """Config 4 runs tight: layout 7 (52 LDS words, 12 waves per CU) over the
    chunk, layout 6 over the instances it handed on, the general kernel over
    that one's.  Identical to layout 6 alone (PXB_NO_TIGHT=1) and to the
    general kernel alone (PXB_NO_EV=1); the tight launch does hand some on."""
    cfg = pxb.CONFIGS[4]
    pxb.handoff_counts(0, reset=True)
    a = pxb.run(cfg, first, 60000, want_acceptors=True)
    h1, h2 = pxb.handoff_counts(0, reset=True)
    assert h1 > 0 and h2 <= h1
    for env in ("PXB_NO_TIGHT", "PXB_NO_EV"):
        b = _with_env({env: "1"}, lambda: pxb.run(cfg, first, 60000, want_acceptors=True))
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y), env
        assert a[3] == b[3], env


@pytest.mark.parametrize("cap", [0, 40, 1 << 20])
def test_config4_tight_list_overflow(gpu_lib, cap):
    """The tight routing's id lists capped (0: the layout-7 list overflows at
    once, so layout 6 runs nothing and the general kernel re-runs the chunk;
    40: either list may overflow): exact either way."""
    _with_env({"PXB_EV_BAIL_CAP": str(cap)}, lambda: _cmp(pxb.CONFIGS[4], (1 << 31) + 5, 30000))


def test_config4_contiguous_at_production_bail_rate(gpu_lib):
    """2^21 contiguous config-4 instances, bit-exact against the oracle
    (results, digests, totals) through both routings: the tight one (layout 7
    hands ~0.5 % on to layout 6, which hands a few on to the general kernel)
    and layout 6 alone (~0.01 % to the general kernel).  Each hand-off path
    carries at least 100 instances, so the hand-offs are exercised at the
    north star's own rate, not only at small sizes."""
    cfg, first, n = pxb.CONFIGS[4], 1 << 36, 1 << 21
    eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, n, threads=THREADS)
    for env in ({}, {"PXB_NO_TIGHT": "1"}):
        pxb.handoff_counts(0, reset=True)
        res, dig, _, cnt = _with_env(env, lambda: pxb.run(cfg, first, n))
        h1, h2 = pxb.handoff_counts(0, reset=True)
        bad = np.nonzero((res != eres).any(axis=1))[0]
        assert bad.size == 0, "%s: first mismatch at %d" % (env, first + bad[0])
        assert np.array_equal(dig, edig) and cnt == ecnt, env
        if env:
            assert h1 >= 100 and h2 == 0, (env, h1, h2)          # layout 6 -> general kernel
        else:
            assert h1 >= 5000 and h2 >= 1, (h1, h2)              # layout 7 -> layout 6 -> general


def test_config5_contiguous_at_production_bail_rate(gpu_lib):
    """2^20 contiguous config-5 instances (the split routing: the two-proposer
    shape over the chunk, the three-proposer shape over the P = 3 third, the
    general kernel over its bails), bit-exact against the oracle, with >= 100
    instances reaching the general kernel."""
    cfg, first, n = pxb.CONFIGS[5], 3 << 34, 1 << 20
    eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, n, threads=THREADS)
    pxb.handoff_counts(0, reset=True)
    res, dig, _, cnt = pxb.run(cfg, first, n)
    h1, h2 = pxb.handoff_counts(0, reset=True)
    bad = np.nonzero((res != eres).any(axis=1))[0]
    assert bad.size == 0, "first mismatch at %d" % (first + bad[0])
    assert np.array_equal(dig, edig) and cnt == ecnt
    assert h1 > n // 4 and h2 >= 100, (h1, h2)


@pytest.mark.parametrize("cap", [0, 5000])
def test_config5_split_list_overflow(gpu_lib, cap):
    """The split routing's id lists overflowing (cap 0: the P = 3 list, so the
    second per-lane kernel runs nothing and marks its own list overflowed;
    5000: either): the general kernel re-runs the chunk; exact either way."""
    with pxb.hooks(PXB_EV_BAIL_CAP=str(cap)):
        _cmp(pxb.CONFIGS[5], (1 << 32) - 7000, 14000)


@pytest.mark.parametrize("c", [2, 6])
def test_fault_free_grid_oversubscription(gpu_lib, c):
    """The fault-free per-lane kernels run a grid of several times the
    resident blocks (default 16): results, digests and totals are the same
    for 1x, the default and 64x, and equal the oracle's."""
    cfg, first, n = pxb.CONFIGS[c], 12345, 300000
    env = "PXB_FF1_OVERSUB" if c == 2 else "PXB_FFP_OVERSUB"
    a = pxb.run(cfg, first, n)
    for k in ("1", "64"):
        b = _with_env({env: k}, lambda: pxb.run(cfg, first, n))
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[3] == b[3], k
    eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, 20000, threads=THREADS)
    assert np.array_equal(a[0][:20000], eres) and np.array_equal(a[1][:20000], edig)


@pytest.mark.parametrize("c,n", [(1, 5000), (2, 20000), ("skew", 9000)])
def test_ff1_bails_run_on_general_kernel(gpu_lib, c, n):
    """Fault-free single-proposer batches run one instance per lane
    (paxos_ff1.h); an instance it hands back runs on the general faulty
    kernel.  PXB_FF1_BAIL=1 hands back every instance: still exact."""
    cfg = pxb.Config(seed=0xFF1, n_proposers=1, n_acceptors=7, skew_max=5) if c == "skew" else pxb.CONFIGS[c]
    with pxb.hooks(PXB_FF1_BAIL="1"):
        _cmp(cfg, 123, n)


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6, 7, 8, 9])
def test_ff1_matches_general_fault_free_kernel(gpu_lib, N):
    """The fault-free per-lane kernel against the general fault-free kernel
    (PXB_NO_FF1=1) and the oracle, with Tick skew and a step cap that cuts
    some instances."""
    cfg = pxb.Config(seed=0xF0 + N, n_proposers=1, n_acceptors=N, skew_max=9, step_cap=12)
    a = _cmp(cfg, (1 << 32) - 5000, 10000)
    with pxb.hooks(PXB_NO_FF1="1"):
        b = _cmp(cfg, (1 << 32) - 5000, 10000)
    assert np.array_equal(a[0], b[0]) and a[1] == b[1]
    assert a[1]["step_cap"] > 0 and a[1]["decided"] > 0


@pytest.mark.parametrize("P,N,ticks,period,skew,cap", [
    (2, 2, 16, 8, 0, 1024), (2, 5, 1, 1, 2, 600), (3, 9, 1, 1, 3, 300), (1, 3, 40, 2, 1, 1024),
    (3, 4, 6, 3, 2, 64), (2, 7, 5, 7, 4, 9)])
def test_ffp_matches_general_fault_free_kernel(gpu_lib, P, N, ticks, period, skew, cap):
    """Duelling / log-mode fault-free batches on their per-lane kernel
    (paxos_ffp.h) against the oracle and the general fault-free kernel
    (PXB_NO_FFP=1), logs past PXB_LOG_TRACK and step caps included; and with
    every instance handed to the general faulty kernel (PXB_FF1_BAIL=1)."""
    cfg = pxb.Config(seed=0xFF9 + 16 * P + N, n_proposers=P, n_acceptors=N, skew_max=skew, step_cap=cap,
                     n_ticks=ticks, tick_period=period)
    a = _cmp(cfg, (1 << 32) - 1500, 3000)
    for env in ("PXB_NO_FFP", "PXB_FF1_BAIL"):
        with pxb.hooks(**{env: "1"}):
            b = _cmp(cfg, (1 << 32) - 1500, 3000)
        assert np.array_equal(a[0], b[0]) and a[1] == b[1], env


@pytest.mark.parametrize("cap", [1, 2, 3, 4, 5, 6, 7])
def test_ff1_step_cap_at_every_phase(gpu_lib, cap):
    """The fault-free per-lane kernel runs the proposer phase of step s + 1
    inside step s; at s = step_cap - 1 it must not: caps that cut every phase
    of the six-step round, with Tick skews 0..3, against the oracle."""
    cfg = pxb.Config(seed=0xCA9 + cap, n_proposers=1, n_acceptors=4, skew_max=3, step_cap=cap)
    _cmp(cfg, 99, 4000)


def test_device_entry_accumulates_totals(gpu_lib):
    import torch
    cfg = pxb.CONFIGS[3]
    n = 10000
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    out = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    pxb.run_device(cfg, 0, n, d_results=out, d_totals=tot)
    pxb.run_device(cfg, n, n, d_totals=tot)
    torch.cuda.synchronize()
    _, _, _, c1 = oracle_c.run_cpu(cfg, 0, 2 * n, threads=THREADS)
    assert pxb.counters_dict(tot.cpu().tolist()) == c1
    eres, _, _, _ = oracle_c.run_cpu(cfg, 0, n, threads=THREADS)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), eres)


def test_work_queue_flush_keeps_totals_exact(gpu_lib):
    """Faulty kernels take instances from a device work queue and flush their
    partial totals mid-run: the general kernel its packed 16-bit per-slot
    counts every FLUSH_EVERY (30000) taken instances, the per-lane kernel
    (which this single-decree schedule takes) its per-lane register sums
    every EV_FLUSH (256) instances of a lane.  With one wave per CU each lane
    takes ~1K instances here, so every wave flushes mid-run; the totals must
    still equal the per-instance results."""
    cfg = pxb.Config(seed=0xF1, n_proposers=1, n_acceptors=3, delay_max=2, step_cap=64)
    n = 1 << 24
    with pxb.hooks(PXB_BLOCKS_PER_CU="1"):
        res, _, _, cnt = pxb.run(cfg, 5, n, want_digests=False)
    flags = res[:, 3] & 0xFF
    assert cnt["instances"] == n
    assert cnt["decided"] == int((res[:, 0] != 0).sum())
    assert cnt["undecided"] == int(((flags & pxb.F_UNDECIDED) != 0).sum())
    assert cnt["step_cap"] == int(((flags & pxb.F_STEP_CAP) != 0).sum())
    assert cnt["rounds"] == int(res[:, 2].astype(np.int64).sum())
    assert cnt["steps"] == int((res[:, 3] >> 16).astype(np.int64).sum())
    rng = np.random.default_rng(5)
    for i in rng.choice(n, 32, replace=False):
        eres, _, _, _ = oracle_c.run_cpu(cfg, 5 + int(i), 1)
        assert np.array_equal(res[i], eres[0])


def test_work_queue_many_launches(gpu_lib):
    """The queue counter pairs are reused round-robin (64 per device) and reset
    by each launch's last wave: 150 back-to-back launches on one stream must
    each run their whole batch."""
    import torch
    cfg = pxb.CONFIGS[4]
    n, k = 211, 150
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    out = torch.zeros((k * n, 4), dtype=torch.int32, device="cuda")
    for j in range(k):
        pxb.run_device(cfg, j * n, n, d_results=out[j * n:(j + 1) * n], d_totals=tot)
    torch.cuda.synchronize()
    eres, _, _, ecnt = oracle_c.run_cpu(cfg, 0, k * n, threads=THREADS)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), eres)
    assert pxb.counters_dict(tot.cpu().tolist()) == ecnt


def test_scratch_slots_across_streams_without_sync(gpu_lib):
    """120 config-4 chunks enqueued round-robin on 3 streams with no host sync
    in between: far more than the device's 64 scratch slots are in flight at
    once, so chunk k + 64 takes the slot of chunk k while chunk k may still run
    on another stream.  Each slot's event (recorded behind its finalize) makes
    the new user's stream wait for it: results, digests and the per-stream
    totals equal the oracle's (a shared slot would mix queue words and partial
    rows of two chunks)."""
    import torch
    cfg = pxb.CONFIGS[4]
    n, k, S = 211, 120, 3
    streams = [torch.cuda.Stream() for _ in range(S)]
    out = torch.zeros((k * n, 4), dtype=torch.int32, device="cuda")
    dig = torch.zeros((k * n, cfg.n_acceptors), dtype=torch.int32, device="cuda")
    tots = [torch.zeros(16, dtype=torch.int64, device="cuda") for _ in range(S)]
    torch.cuda.synchronize()
    for j in range(k):
        st = streams[j % S]
        pxb.run_device(cfg, j * n, n, d_results=out[j * n:(j + 1) * n], d_digests=dig[j * n:(j + 1) * n],
                       d_totals=tots[j % S], stream=st.cuda_stream)
    torch.cuda.synchronize()
    eres, edig, _, _ = oracle_c.run_cpu(cfg, 0, k * n, threads=THREADS)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), eres)
    assert np.array_equal(dig.cpu().numpy().view(np.uint32), edig)
    for s in range(S):
        ids = [j for j in range(k) if j % S == s]
        want = None
        for j in ids:
            _, _, _, c = oracle_c.run_cpu(cfg, j * n, n, threads=THREADS)
            want = c if want is None else {key: want[key] + c[key] for key in want}
        assert pxb.counters_dict(tots[s].cpu().tolist()) == want, s


@pytest.mark.parametrize("N", [6, 8])
def test_tight_routing_topologies(gpu_lib, N):
    """The tight routing (layout 7 first) is taken only where its hand-off rate
    is measured small: P = 2 with N = 6 or 7 on a simple schedule (host model,
    tools/wave_model.cpp: N = 6 0.11 %, N = 7 0.76 %, N = 8 2.8 %).  N = 6 runs
    tight and hands on < 1 %; N = 8 runs layout 6 alone (no second per-lane
    stage: h2 == 0).  Both exact against the oracle."""
    cfg = pxb.Config(seed=0x5EED0004 + N, n_proposers=2, n_acceptors=N, delay_max=4, crash_ppm=200000,
                     crash_len_max=16, crash_start_max=8, step_cap=256)
    n = 60000
    pxb.handoff_counts(0, reset=True)
    _cmp(cfg, 1 << 33, n, want_acc=False)
    h1, h2 = pxb.handoff_counts(0, reset=True)
    if N == 6:
        assert 0 < h1 < n // 100, (h1, h2)
    else:
        assert h1 < n // 100 and h2 == 0, (h1, h2)


def test_handoff_counts_read_and_reset(gpu_lib):
    """pxb_handoff_counts reads and zeroes in one device atomic per count: a
    read without reset keeps the counts, a reset read returns them and leaves
    zero."""
    pxb.handoff_counts(0, reset=True)
    pxb.run(pxb.CONFIGS[4], 1 << 34, 60000, want_results=False, want_digests=False)
    a = pxb.handoff_counts(0, reset=False)
    b = pxb.handoff_counts(0, reset=True)
    c = pxb.handoff_counts(0, reset=True)
    assert a == b and a[0] > 0 and c == (0, 0)


# ---- single-handler hooks: the kernel's device functions vs oracle handlers --
def test_acceptor_hook_matches_oracle(gpu_lib):
    rng = np.random.default_rng(1)
    n = 20000
    st = np.zeros((n, 4), np.uint32)
    st[:, 0] = rng.integers(0, 8, n)
    st[:, 1] = rng.integers(0, 8, n)
    st[:, 2] = np.where(rng.random(n) < 0.5, 0, (rng.integers(1, 4, n) << 24) | 1)
    st[:, 3] = rng.integers(0, 5, n) | (np.where(rng.random(n) < 0.1, 1, 0) << 31).astype(np.uint32)
    msg = np.zeros((n, 4), np.uint32)
    msg[:, 0] = rng.integers(0, 3, n)
    msg[:, 1] = rng.integers(0, 9, n)
    msg[:, 3] = (rng.integers(1, 4, n) << 24) | 1
    est, erep = oracle_c.acceptor_handle(st, msg)
    gst = st.copy()
    grep = pxb.acceptor_handle(gst, msg)
    assert np.array_equal(gst, est) and np.array_equal(grep, erep)


def test_proposer_hook_matches_oracle(gpu_lib):
    rng = np.random.default_rng(2)
    n = 20000
    st = np.zeros((n, 10), np.uint32)
    st[:, 0] = rng.integers(0, 8, n)                       # ticket
    st[:, 1] = (rng.integers(1, 4, n) << 24) | 1           # cmd
    st[:, 2] = rng.integers(0, 5, n)                       # acks
    st[:, 3] = rng.integers(0, 3, n)                       # state
    st[:, 4] = rng.integers(0, 8, n)                       # mr_t
    st[:, 5] = np.where(rng.random(n) < 0.5, 0, (rng.integers(1, 4, n) << 24) | 1)
    st[:, 6] = st[:, 0]
    st[:, 7] = (rng.integers(1, 4, n) << 24) | 1
    st[:, 8] = rng.integers(0, 2, n)
    st[:, 9] = rng.integers(1, 4, n)
    msg = np.zeros((n, 4), np.uint32)
    msg[:, 0] = rng.integers(0, 4, n)                      # 3 = Tick
    msg[:, 1] = rng.integers(0, 9, n)
    msg[:, 2] = rng.integers(0, 8, n)
    msg[:, 3] = np.where(rng.random(n) < 0.4, 0, (rng.integers(1, 4, n) << 24) | 1)
    for N in (2, 3, 5, 9):
        est, ebc, enb = oracle_c.proposer_handle(st, N, msg)
        gst = st.copy()
        gbc, gnb = pxb.proposer_handle(gst, N, msg)
        assert np.array_equal(gst, est) and np.array_equal(gbc, ebc) and np.array_equal(gnb, enb)


def test_run_multi_matches_single_device(gpu_lib):
    """pxb_run_multi (thread per GPU + RCCL all-reduce of the totals) on the
    visible devices reproduces pxb_run bit-exact."""
    cfg = pxb.CONFIGS[3]
    res, dig, cnt = pxb.run_multi(cfg, 0, 20000)
    eres, edig, _, ecnt = pxb.run(cfg, 0, 20000)
    assert np.array_equal(res, eres) and np.array_equal(dig, edig) and cnt == ecnt


def test_many_streams_concurrent(gpu_lib):
    """More concurrent streams than a device keeps bailed-id lists for (8):
    12 host threads, each on its own HIP stream, run config 4 (which bails
    ~0.5 % of its instances to a per-stream list) at once, twice over.  An
    evicted list is only handed to a new stream after the old owner's launches
    on it are done, so every thread's results and totals equal its own
    single-stream run."""
    import threading
    import torch
    cfg = pxb.CONFIGS[4]
    n, T = 20000, 12
    want = [pxb.run(cfg, 100000 * t, n) for t in range(T)]
    got = [None] * T
    errs = []

    def worker(t):
        try:
            st = torch.cuda.Stream()
            out = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
            dig = torch.zeros((n, cfg.n_acceptors), dtype=torch.int32, device="cuda")
            tot = torch.zeros(16, dtype=torch.int64, device="cuda")
            torch.cuda.current_stream().synchronize()     # (the zeros above are on this thread's stream)
            for _ in range(2):
                with torch.cuda.stream(st):
                    tot.zero_()                           # (on st: ordered before the launch)
                    pxb.run_device(cfg, 100000 * t, n, d_results=out, d_digests=dig, d_totals=tot,
                                   stream=st.cuda_stream)
                st.synchronize()
            got[t] = (out.cpu().numpy().view(np.uint32), dig.cpu().numpy().view(np.uint32),
                      pxb.counters_dict(tot.cpu().tolist()))
        except Exception as e:   # (reported by the main thread)
            errs.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for t in range(T):
        assert np.array_equal(got[t][0], want[t][0]) and np.array_equal(got[t][1], want[t][1])
        assert got[t][2] == want[t][3]


def test_run_multi_repeated_calls_release_stream_lists(gpu_lib):
    """pxb_run_multi makes a stream per device and call and gives its lists
    back when it tears the stream down: 12 calls in a row (more than the 8
    list entries of a device) stay exact."""
    cfg = pxb.CONFIGS[4]
    want = pxb.run(cfg, 5, 8000)
    for _ in range(12):
        res, dig, cnt = pxb.run_multi(cfg, 5, 8000)
        assert np.array_equal(res, want[0]) and np.array_equal(dig, want[1]) and cnt == want[3]


def test_run_multi_concurrent_callers(gpu_lib):
    """pxb_run_multi from four host threads at once, two configs and instance
    ranges: the calls share the cached RCCL communicators, so the library runs
    them one after another; every call's results and reduced totals equal its
    single-device run."""
    import threading
    jobs = [(pxb.CONFIGS[3], 1000 * t, 6000) for t in range(2)] + [(pxb.CONFIGS[4], 1000 * t, 6000) for t in range(2)]
    want = [pxb.run(cfg, f, n) for cfg, f, n in jobs]
    got = [None] * len(jobs)
    errs = []

    def worker(i):
        try:
            cfg, f, n = jobs[i]
            got[i] = pxb.run_multi(cfg, f, n)
        except Exception as e:   # (reported by the main thread)
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs
    for i in range(len(jobs)):
        assert np.array_equal(got[i][0], want[i][0]) and np.array_equal(got[i][1], want[i][1])
        assert got[i][2] == want[i][3]


def test_stream_release_with_caller_streams(gpu_lib):
    """pxb_stream_release through the public ABI: 12 caller-created streams in
    turn (more than a device's 8 list entries), each released before the next
    is made, on config 5's split routing (both list kinds) and config 4; every
    batch matches the one made on the default stream."""
    import torch
    for c in (5, 4):
        cfg = pxb.CONFIGS[c]
        want = pxb.run(cfg, 77, 6000)
        for _ in range(12):
            st = torch.cuda.Stream()
            out = torch.empty((6000, 4), dtype=torch.int32, device="cuda")
            dig = torch.empty((6000, cfg.n_acceptors), dtype=torch.int32, device="cuda")
            tot = torch.zeros(16, dtype=torch.int64, device="cuda")
            torch.cuda.current_stream().synchronize()     # (zeros before the launch on st)
            pxb.run_device(cfg, 77, 6000, d_results=out, d_digests=dig, d_totals=tot, stream=st.cuda_stream)
            st.synchronize()
            pxb.stream_release(torch.cuda.current_device(), st.cuda_stream)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want[0])
            assert np.array_equal(dig.cpu().numpy().view(np.uint32), want[1])
            assert pxb.counters_dict(tot.cpu().tolist()) == want[3]
            del st
        pxb.stream_release(0, 0)                  # (unknown / null streams are ignored)


def _device_run(cfg, first, n, stream):
    import torch
    out = torch.zeros((n, 4), dtype=torch.int32, device="cuda")
    dig = torch.zeros((n, cfg.n_acceptors), dtype=torch.int32, device="cuda")
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    torch.cuda.current_stream().synchronize()     # (the zeros before the launch on `stream`)
    pxb.run_device(cfg, first, n, d_results=out, d_digests=dig, d_totals=tot,
                   stream=stream.cuda_stream if stream is not None else None)
    return out, dig, tot


def _host(out, dig, tot):
    return (out.cpu().numpy().view(np.uint32), dig.cpu().numpy().view(np.uint32),
            pxb.counters_dict(tot.cpu().tolist()))


@pytest.mark.parametrize("c", [4, 5])
def test_failure_after_first_launch_then_more_streams(gpu_lib, c):
    """A chunk that fails right after its first per-lane launch (test hook
    PXB_FAIL_AFTER_FIRST: the two-stage routings' first list is then in use by
    a queued kernel) still records its lists' event, so the streams that take
    those lists over later -- nine more streams, one past the device's eight
    entries, then the failed stream again -- wait for that kernel: every run
    after the failure is exact."""
    import torch
    cfg, n = pxb.CONFIGS[c], 30000
    want = pxb.run(cfg, 4096, n)
    bad = torch.cuda.Stream()
    with pytest.raises(pxb.PaxosError):
        _with_env({"PXB_FAIL_AFTER_FIRST": "1"}, lambda: _device_run(cfg, 4096, n, bad))
    for st in [torch.cuda.Stream() for _ in range(9)] + [bad]:
        res = _device_run(cfg, 4096, n, st)
        st.synchronize()
        got = _host(*res)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[3]


def test_release_in_flight_then_default_stream(gpu_lib):
    """A caller stream released while its launch still runs (its lists are
    free for the next owner), then batches on the default stream, which takes
    the entry over: the default stream waits for the released stream's event
    on the device (ownership is a flag, so the null stream is an owner like
    any other), and both streams' results are exact."""
    import torch
    cfg, n = pxb.CONFIGS[4], 1 << 20
    want = pxb.run(cfg, 1 << 33, n)
    small = pxb.run(cfg, 99, 20000)
    st = torch.cuda.Stream()
    dev = torch.cuda.current_device()
    res = _device_run(cfg, 1 << 33, n, st)         # (~20 ms on the device)
    pxb.stream_release(dev, st.cuda_stream)
    for _ in range(3):
        got = pxb.run(cfg, 99, 20000)               # (pxb_run: the default stream)
        assert np.array_equal(got[0], small[0]) and got[3] == small[3]
    st.synchronize()
    got = _host(*res)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1]) and got[2] == want[3]
    pxb.stream_release(dev, 0)                      # (the default stream's entry back too)
    got = pxb.run(cfg, 99, 20000)
    assert np.array_equal(got[0], small[0]) and got[3] == small[3]


def test_config5_full_sweep_totals(gpu_lib):
    """BASELINE config 5 at its stated size: all 2^28 randomized schedules on
    one GPU in one call (run totals only, no per-instance outputs).  The
    totals equal the sum of the eight 2^25 per-GPU shares run separately (the
    8-GPU sharding), and every schedule is counted decided or undecided."""
    import torch
    cfg = pxb.CONFIGS[5]
    n = pxb.CONFIG_INSTANCES[5]
    tot = torch.zeros(16, dtype=torch.int64, device="cuda")
    pxb.run_device(cfg, 0, n, d_totals=tot)
    torch.cuda.synchronize()
    full = pxb.counters_dict(tot.cpu().tolist())
    assert full["instances"] == n and full["decided"] + full["undecided"] == n
    shares = torch.zeros(16, dtype=torch.int64, device="cuda")
    for k in range(8):
        pxb.run_device(cfg, k * (n // 8), n // 8, d_totals=shares)
    torch.cuda.synchronize()
    assert pxb.counters_dict(shares.cpu().tolist()) == full


@pytest.mark.parametrize("phase", ["setup", "compute"])
def test_run_multi_shard_failure_returns_promptly(gpu_lib, phase):
    """A device that fails before the collective makes pxb_run_multi return its
    error at once (no device is left blocked in the all-reduce); the next call
    works."""
    import time
    cfg = pxb.CONFIGS[3]
    with pxb.hooks(PXB_MULTI_FAIL_PHASE=phase, PXB_MULTI_FAIL_DEVICE="0"):
        t0 = time.perf_counter()
        with pytest.raises(pxb.PaxosError):
            pxb.run_multi(cfg, 0, 5000)
        assert time.perf_counter() - t0 < 60
    res, _, cnt = pxb.run_multi(cfg, 0, 5000)
    assert cnt["instances"] == 5000


def test_init_shutdown_cycles(gpu_lib):
    """pxb_init / pxb_shutdown release and rebuild every per-device buffer and
    the cached communicators; runs in between stay exact."""
    cfg = pxb.CONFIGS[4]
    want = pxb.run(cfg, 0, 3000)
    for _ in range(3):
        pxb.init(0)
        got = pxb.run(cfg, 0, 3000)
        assert np.array_equal(got[0], want[0]) and got[3] == want[3]
        pxb.run_multi(cfg, 0, 1000)
        pxb.shutdown()
    pxb.shutdown()
    got = pxb.run(cfg, 0, 3000)
    assert np.array_equal(got[0], want[0])


def test_host_driver_binary(gpu_lib):
    """The C++ batch driver (the app/Main.hs role) runs config 1 end to end."""
    import subprocess
    exe = os.path.join(os.path.dirname(pxb.LIB_PATH), "..", "host", "paxos_batch_main")
    out = subprocess.run([exe, "--config", "1", "--show", "2"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "decided c1.1 @ Ticket 1, rounds 1, steps 6, flags -" in out.stdout
    assert "decided          1024" in out.stdout


def _random_config(rng, i):
    """A schedule drawn from the whole validated parameter space."""
    log = rng.random() < 0.3
    return pxb.Config(
        seed=int(rng.integers(0, 1 << 63)), n_proposers=int(rng.integers(1, 4)),
        n_acceptors=int(rng.integers(2, 10)),
        loss_ppm=int(rng.choice([0, 0, rng.integers(1, 600000), 1000000])),
        delay_max=int(rng.choice([1, 1, rng.integers(2, 16)])),
        crash_ppm=int(rng.choice([0, rng.integers(1, 1000001)])),
        crash_len_max=int(rng.integers(1, 40)), crash_start_max=int(rng.integers(0, 30)),
        skew_max=int(rng.choice([0, rng.integers(1, 12)])),
        step_cap=int(rng.choice([int(rng.integers(1, 64)), 256, 1024])),
        randomize=bool(rng.random() < 0.25),
        n_ticks=int(rng.integers(2, 9)) if log else 1,
        tick_period=int(rng.integers(1, 21)) if log else 1)


@pytest.mark.parametrize("i", range(48))
def test_random_schedules_match_oracle(gpu_lib, i):
    """48 seeded draws over every knob (proposers, acceptors, loss, delay, crash
    windows, skew, step cap, per-instance fuzzing, log mode): results,
    digests, acceptor records and totals (canonical bytes included) equal the
    oracle's."""
    rng = np.random.default_rng(0xF022 + i)
    cfg = _random_config(rng, i)
    _cmp(cfg, int(rng.integers(0, 1 << 34)), int(rng.integers(1, 1500)))


@pytest.mark.parametrize("i", range(24))
def test_random_fault_free_schedules_match_oracle(gpu_lib, i):
    """24 seeded fault-free draws (the per-lane fault-free kernels: one or more
    proposers, Tick skew, step caps, single decree or log mode with up to 40
    Ticks): everything equals the oracle's."""
    rng = np.random.default_rng(0xFF0 + i)
    log = rng.random() < 0.5
    cfg = pxb.Config(seed=int(rng.integers(0, 1 << 63)), n_proposers=int(rng.integers(1, 4)),
                     n_acceptors=int(rng.integers(2, 10)), skew_max=int(rng.choice([0, rng.integers(1, 12)])),
                     step_cap=int(rng.choice([int(rng.integers(1, 40)), 256, 1024])),
                     n_ticks=int(rng.integers(2, 41)) if log else 1,
                     tick_period=int(rng.integers(1, 12)) if log else 1)
    _cmp(cfg, int(rng.integers(0, 1 << 34)), int(rng.integers(1, 2500)))


# ---- per-instance trace (pxb_trace_instance; Server.hs:85 / Client.hs:108) ----
def _oracle_trace(cfg, inst):
    import paxos_ref as R
    recs = []

    def snap(s, accs, props, in_flight):
        recs.append({"step": s, "in_flight": in_flight,
                     "acc": [(a.t_max, a.t_store, a.val, len(a.log) | (int(a.dead) << 31)) for a in accs],
                     "digest": [_digest(a.log) for a in accs],
                     "prop": [(p.ticket, p.cmd, p.acks, p.rs, p.mr_t, p.mr_v, p.r2_v, int(p.pending))
                              for p in props]})
    res = R.run_instance(R.Config(**cfg.__dict__) if not isinstance(cfg, R.Config) else cfg, inst, trace=snap)
    return recs, res


def _digest(log):
    import paxos_ref as R
    h = R.FNV_BASIS
    for v in log:
        h = R.fnv1a_u32(h, v)
    return R.fnv1a_u32(h, len(log))


def _as_rec(g):
    return {"step": g["step"], "in_flight": g["in_flight"],
            "acc": [tuple(int(x) for x in r) for r in g["acc"]], "digest": [int(x) for x in g["digest"]],
            "prop": [tuple(int(x) for x in r) for r in g["prop"]]}


@pytest.mark.parametrize("c,inst", [(3, 0), (3, 17), (4, 5), (4, 123456), (5, 9), (5, 1000),
                                    (7, 3), (7, 2024), (7, 77777)])
def test_trace_matches_oracle_steps(gpu_lib, c, inst):
    """Every step the GPU trace records equals the oracle's state at the end of
    that step (acceptor records, log digests, proposer states, messages in
    flight); the steps it skips change nothing in the oracle either."""
    cfg = pxb.CONFIGS[c]
    try:
        g, gres = pxb.trace_instance(cfg, inst)
    except pxb.PaxosError:
        pytest.skip("instance beyond the trace kernel's link capacities")
    want, res = _oracle_trace(cfg, inst)
    by_step = {r["step"]: r for r in want}
    prev = None
    gi = iter(_as_rec(x) for x in g)
    cur = next(gi)
    for r in want:
        if cur is not None and r["step"] == cur["step"]:
            assert r == cur, "step %d: oracle %s gpu %s" % (r["step"], r, cur)
            prev, cur = cur, next(gi, None)
        else:                                          # a skipped step: nothing changed
            assert prev is not None and {k: r[k] for k in ("acc", "digest", "prop", "in_flight")} == \
                {k: prev[k] for k in ("acc", "digest", "prop", "in_flight")}, r["step"]
    assert cur is None and g[-1]["step"] == want[-1]["step"] and by_step
    assert list(gres) == [res.decided_val, res.decided_ticket, res.rounds, res.packed_flags()]


@pytest.mark.parametrize("c,inst", [(3, 0), (3, 17), (4, 5), (4, 123456), (5, 9), (5, 1000), (4, 77), (3, 4242),
                                    (7, 3), (7, 2024), (7, 555)])
def test_trace_production_variant_matches_oracle_steps(gpu_lib, c, inst):
    """The carry-over variant the batch kernels run (a step may end with the
    copies of its last broadcast still to send): at every step it records, the
    acceptor records, log digests and proposer states equal the oracle's state
    at the end of that step (or of the last step the oracle visited before it:
    a carried step may hold nothing else); the oracle steps it skips change
    nothing; in_flight equals the oracle's whenever no copy is pending."""
    cfg = pxb.CONFIGS[c]
    try:
        g, gres = pxb.trace_instance(cfg, inst, production=True)
    except pxb.PaxosError:
        pytest.skip("instance beyond the trace kernel's link capacities")
    want, res = _oracle_trace(cfg, inst)
    steps = [r["step"] for r in want]
    gsteps = [int(x["step"]) for x in g]
    assert gsteps == sorted(set(gsteps))
    keys = ("acc", "digest", "prop", "in_flight")
    for k, r in enumerate(want):                       # skipped steps change nothing
        if r["step"] not in gsteps:
            assert k > 0 and {q: r[q] for q in keys} == {q: want[k - 1][q] for q in keys}, r["step"]
    import bisect
    carried = 0
    for x in g:
        r = _as_rec(x)
        k = bisect.bisect_right(steps, r["step"]) - 1
        assert k >= 0, r["step"]
        w = want[k]
        for key in ("acc", "digest", "prop"):
            assert r[key] == w[key], "step %d %s: oracle %s gpu %s" % (r["step"], key, w[key], r[key])
        if r["in_flight"] != pxb.TRACE_IN_FLIGHT_UNKNOWN:
            assert r["in_flight"] == w["in_flight"], r["step"]
        else:
            carried += 1
    assert gsteps[-1] == steps[-1]
    assert list(gres) == [res.decided_val, res.decided_ticket, res.rounds, res.packed_flags()]


def test_log_mode_two_stage_routing(gpu_lib):
    """Faulty log mode over <= 10 links runs in two per-lane stages: the
    log-mode shape (18-word pool) over the chunk, the same shape on the 16-step
    wheel with a 32-word pool over what it hands on, the general log-mode
    kernel over that one's.  A schedule whose responses pile up (delays to 8,
    no loss, a Tick every 2 steps: ~0.15 % stage-1 hand-offs, host model):
    stage 1 hands >= 20 on, stage 2 nearly none; results, digests, acceptor
    records and totals equal the oracle's, the one-stage routing's
    (PXB_NO_LG2=1) and, with the id lists capped (0: the first list overflows,
    so the general kernel re-runs the chunk; 3: either may), the same again."""
    cfg = pxb.Config(seed=0x7C, n_proposers=2, n_acceptors=5, delay_max=8, skew_max=3, step_cap=1024,
                     n_ticks=16, tick_period=2)
    first, n = 1 << 35, 60000
    pxb.handoff_counts(0, reset=True)
    _cmp(cfg, first, n)
    h1, h2 = pxb.handoff_counts(0, reset=True)
    assert h1 >= 20 and h2 <= h1 // 4, (h1, h2)
    a = pxb.run(cfg, first, n, want_acceptors=True)
    for env in ({"PXB_NO_LG2": "1"}, {"PXB_EV_BAIL_CAP": "0"}, {"PXB_EV_BAIL_CAP": "3"}, {"PXB_NO_LGS": "1"},
                {"PXB_NO_LGS": "1", "PXB_NO_LG2": "1"}):
        b = _with_env(env, lambda: pxb.run(cfg, first, n, want_acceptors=True))
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y), env
        assert a[3] == b[3], env


def test_log_mode_first_stage_layouts(gpu_lib):
    """Faulty log mode with delays <= 4 over <= 10 links runs its first stage on
    layout 9 (byte reply seqs, 4-step wheel, packed canonical log: 8 waves per
    CU), with longer delays on layout 4: both against the oracle, and layout 9
    against layout 4 (PXB_NO_LGS=1) on the bench's batch, logs past LOG_TRACK
    included."""
    for cfg in (pxb.LOG_FAULTY_CONFIG,
                pxb.Config(seed=0x7A0D, n_proposers=1, n_acceptors=5, loss_ppm=10000, delay_max=2, skew_max=2,
                           crash_ppm=150000, crash_len_max=20, crash_start_max=400, step_cap=2048, n_ticks=100,
                           tick_period=8),
                pxb.Config(seed=0x7A0E, n_proposers=2, n_acceptors=5, loss_ppm=100000, delay_max=6, skew_max=3,
                           crash_ppm=200000, crash_len_max=16, crash_start_max=64, step_cap=1024, n_ticks=16,
                           tick_period=8)):
        _cmp(cfg, 777, 6000)
        a = pxb.run(cfg, 1 << 37, 30000, want_acceptors=True)
        b = _with_env({"PXB_NO_LGS": "1"}, lambda: pxb.run(cfg, 1 << 37, 30000, want_acceptors=True))
        for x, y in zip(a[:3], b[:3]):
            assert np.array_equal(x, y)
        assert a[3] == b[3]


def test_log_mode_contiguous_faulty_config(gpu_lib):
    """2^21 contiguous faulty-log-mode instances (pxb.LOG_FAULTY_CONFIG, the
    bench's log_mode_faulty) through the two-stage routing, bit-exact against
    the oracle: results, digests and totals."""
    cfg, first, n = pxb.LOG_FAULTY_CONFIG, 5 << 33, 1 << 21
    eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, n, threads=THREADS)
    res, dig, _, cnt = pxb.run(cfg, first, n)
    bad = np.nonzero((res != eres).any(axis=1))[0]
    assert bad.size == 0, "first mismatch at %d" % (first + bad[0])
    assert np.array_equal(dig, edig) and cnt == ecnt


@pytest.mark.parametrize("cfg", [pxb.LOG_FAULTY_CONFIG, pxb.Config(seed=0x10E, n_proposers=3, n_acceptors=9, loss_ppm=300000,
                                                        delay_max=8, skew_max=3, crash_ppm=200000,
                                                        crash_len_max=16, crash_start_max=16, step_cap=512,
                                                        randomize=True, n_ticks=12, tick_period=6)])
def test_log_mode_per_lane_matches_general_kernel(gpu_lib, cfg):
    """Faulty log mode runs on the per-lane kernel's log-mode shape (bails on
    the general LOGM kernel); the general kernel alone (PXB_NO_EV=1) and the
    oracle give identical results, digests, acceptor records and totals."""
    a = pxb.run(cfg, 99, 40000, want_acceptors=True)
    with pxb.hooks(PXB_NO_EV="1"):
        b = pxb.run(cfg, 99, 40000, want_acceptors=True)
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)
    assert a[3] == b[3]
    _cmp(cfg, 99, 4000)


# ---- hand-derived step-schedule KATs (tests/golden/kat_step_schedule.json) ----
_STEP_KATS = __import__("json").load(open(os.path.join(GOLDEN, "kat_step_schedule.json")))["cases"]


@pytest.mark.parametrize("case", _STEP_KATS, ids=[c["name"] for c in _STEP_KATS])
@pytest.mark.parametrize("production", [False, True])
def test_step_kats_on_gpu(gpu_lib, case, production):
    """The GPU result, acceptor records and per-step trace (both variants of
    the per-lane state machine) equal the hand-derived trace."""
    import bisect
    cfg = pxb.Config(**case["config"])
    want = case["result"]
    res, dig, acc, cnt = pxb.run(cfg, case["instance"], 1, want_acceptors=True)
    assert list(res[0]) == [want["decided_val"], want["decided_ticket"], want["rounds"],
                            want["flags"] | (want["steps"] << 16)]
    assert (cnt["messages"], cnt["canon_bytes"], cnt["executes"]) == \
        (want["messages"], want["canon_bytes"], want["executes"])
    final = [cp for cp in case["checkpoints"] if cp["step"] == want["steps"] - 1][0]
    assert acc[0].tolist() == final["acc"]
    for a, log in enumerate(want["logs"]):
        h = 0x811C9DC5
        for v in log:
            h = _fnv(h, v)
        assert int(dig[0][a]) == _fnv(h, len(log))
    # (log mode too, ABI 5: S4's Q5 double execution and S5's Q7 stale
    # execution are pinned step by step, not only in the final records)
    recs, tres = pxb.trace_instance(cfg, case["instance"], production=production)
    assert list(tres) == list(res[0])
    steps = [r["step"] for r in recs]
    for cp in case["checkpoints"]:
        r = recs[bisect.bisect_right(steps, cp["step"]) - 1]
        assert [[int(x) for x in a] for a in r["acc"]] == cp["acc"], cp["step"]
        assert [[int(x) for x in p[:4]] for p in r["prop"]] == cp["prop"], cp["step"]
        if "in_flight" in cp and r["in_flight"] != pxb.TRACE_IN_FLIGHT_UNKNOWN:
            assert r["in_flight"] == cp["in_flight"], cp["step"]


@pytest.mark.parametrize("kind", ["simple", "compact", "split", "log"])
def test_fuzz_per_lane_shapes(gpu_lib, kind):
    """A slice of tests/fuzz_gpu.py in the suite: 12 schedules per per-lane
    shape family (the simple schedule of BASELINE config 4, the compact
    layouts, the fuzzed-P split, faulty log mode) x 2048 instances, GPU
    against the oracle instance by instance and in the run totals."""
    import fuzz_gpu
    rng = np.random.default_rng({"simple": 11, "compact": 12, "split": 13, "log": 14}[kind])
    for _ in range(12):
        cfg = fuzz_gpu.draw(rng, kind)
        first = int(rng.integers(0, 1 << 40))
        res, dig, _, cnt = pxb.run(cfg, first, 2048)
        eres, edig, _, ecnt = oracle_c.run_cpu(cfg, first, 2048, threads=THREADS)
        assert np.array_equal(res, eres) and np.array_equal(dig, edig), cfg
        assert cnt == ecnt, cfg
