"""Benchmark: Paxos instances decided per second on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4]

One step = one pxb_run_device call over one batch of fresh synthetic
instances.  The headline workload is the north star, BASELINE config 4: 2^26
(64M) instances per step with 2 duelling proposers, 7 acceptors, delays in
[1, 4] and seeded acceptor crash windows, split over the job's GPUs (strong
scaling: 2^26 / N contiguous global ids per rank and step).  Instances are
generated on the device from (seed, global instance id), so the inputs are
resident before the timed region; outputs (16 B result + 4 B/acceptor digest
per instance) are written to HBM.  `value` = decided instances / s over the
whole job.

For N > 1 (one process per GPU, torchrun) each rank runs its own instance
range (no data-path collective) and the run totals (decided counts,
violation flags) are summed with one RCCL all-reduce after the timed region.
`--gpus N` without torchrun spawns the N ranks itself (a child
torch.distributed.run, started before this process touches a GPU).  Prints
ONE JSON line on rank 0: the headline first (with its roofline and the CPU
baseline of the same config), then, on one GPU, `extra`: config 2 (the
fault-free 2^28-instance batch, the round-1..3 headline), config 4 at 2^23 (the
per-GPU share at N = 8), configs 3 and 5 at scale, config 5's whole 2^28 sweep
(totals only), fault-free and faulty log mode, and the wire codec.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))

# HIP hardware queues per process (HIP's default, and the GPU box's setting: 4).
# The faulty-log-mode lines keep LOG_STREAMS calls in flight, one step stream
# each, and streams beyond the queue count share a queue, where they run one
# after the other; workloads on one stream are unaffected.  Raised before
# anything initialises HIP (torch is imported lazily), never lowered.
HW_QUEUES = 16


def _hw_queues():
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        return 4


if _hw_queues() < HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
# VALU issue peak: 256 CUs x 4 SIMDs, a wave64 VALU instruction every 2 cycles
# per SIMD (MI355X_MICROARCH.md, "Wave scheduling") = 2 wave-instructions per
# CU-cycle, at the 2.4 GHz peak engine clock
CUS = 256
VALU_PEAK_G = CUS * 2 * 2.4  # G wave64 VALU instructions / s (1228.8)
PROFILES = os.path.join(ROOT, "profiles")
PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")   # the newest committed profile set of a workload wins
BATCHES_PER_STEP = 256       # config-2 batches of 2^20 per timed step (>= 100 ms over 20 steps)
STEP_STREAMS = 0             # --streams (A/B; --one-stream = 1; 0: by step size, GpuLeg)
DRY_NORTH_STAR = 1 << 12     # --dry-run stand-in for the headline's 2^26 instances per step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=[2, 3, 4, 5, 6, 7],
                    help="BASELINE config (6: log mode, 7: faulty log mode).  Configs 4 and 5 are one "
                         "batch over the job (2^26 and 2^28 instances per step, each rank 1/N of it: a "
                         "one-GPU --config 5 run takes all 2^28 per step); config 2 is 2^28 per GPU")
    ap.add_argument("--instances", type=int, default=0, help="per GPU per step (default: the config's step size)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--dry-run", action="store_true", help="CPU ranks (gloo), synthetic work: launcher test only")
    ap.add_argument("--streams", type=int, default=0, help="step streams (default: faulty steps of up to 2^24 instances 4, larger ones 1; fault-free 2)")
    ap.add_argument("--one-stream", action="store_true",
                    help="all steps on one stream (A/B of the two-stream step pipeline)")
    return ap.parse_args()


def spawn_ranks(args) -> int:
    """--gpus N outside torchrun: run N ranks as a child torch.distributed.run
    (one process per GPU) and return its exit code.  Called before any GPU use."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def step_instances(c: int, override: int, world: int = 1) -> int:
    """Instances per GPU per step.  Config 2 is weak-scaled (a fixed batch per
    GPU); configs 4 and 5 are quoted as one batch over the node (64M over 8
    GPUs, 256M), so each rank runs its 1/world share of that batch."""
    import pxb
    if override:
        return override
    if c == 2:
        return BATCHES_PER_STEP * pxb.CONFIG_INSTANCES[2]
    if c in (4, 5):
        return pxb.CONFIG_INSTANCES[c] // world
    return pxb.CONFIG_INSTANCES[c]


def scaling_of(c: int) -> str:
    return "strong" if c in (4, 5) else "weak"


_STREAM_POOL = []


def step_streams(stream, dev, ns):
    """The first ns step streams: the main stream, then streams created once per
    process and shared by every workload.  (A process gets GPU_MAX_HW_QUEUES
    hardware queues, which its streams share round-robin in creation order: a
    workload that made streams of its own after the earlier ones' could land two
    of its step streams on one queue, where they run one after the other; main()
    creates them all first.)"""
    import torch
    if not _STREAM_POOL:
        _STREAM_POOL.append(stream)
    while len(_STREAM_POOL) < ns:
        _STREAM_POOL.append(torch.cuda.Stream(dev))
    assert _STREAM_POOL[0] is stream
    return _STREAM_POOL[:ns]


class GpuLeg:
    """The measured work of one rank: pxb_run_device over fresh instance ids,
    asynchronous, timed with an event pair.  Steps of up to 2^24 instances
    rotate over four HIP streams (hardware queues: HW_QUEUES) with their own
    output buffers (round 6, MI355X, 8 steps: config 3 at 2^24 341 -> 346 M/s,
    config 4 at 2^23 67.8 -> 68.5 M/s against two; profiles/r06_notes/
    ab_log_streams.txt): the per-lane kernel is persistent (its grid is the resident
    capacity), so step k + 1's waves are dispatched onto the CUs that step k's
    last waves free up -- its tail (the slowest instances of the last waves,
    then the general kernel over its bailed ones: 2.5 % + 1 % of a
    2^23-instance step, tools/ev_wave_times.py) overlaps the next step's work.
    Larger faulty steps use one stream: there the overlapped launches slow each other
    (the general kernel co-runs with the next per-lane kernel at a fraction
    of its speed, and the 1-block finalize behind it waits for that kernel to
    end), MI355X A/B (profiles/r04_notes/wave_times.txt): 2^23 +1.9 %, 2^24
    +0.4 %, 2^25 +-0, 2^26 -0.7 % for two streams (round 6, 16 queues: 2^26 +-0.5 %,
    config 5 at 2^25 -10 % on 2 or 3).  Fault-free batches (config 2:
    the fault-free per-lane kernel, not persistent) keep two streams at any
    size: 2^28 per step, 4.3 ms with two against 5.4 ms alone (4 streams: the same).  All K steps complete
    inside the timed region either way."""

    def __init__(self, cfg, n, rank, world, stream, dev, outputs=True, streams=0):
        import torch
        import pxb
        self.torch, self.pxb = torch, pxb
        self.cfg, self.n, self.rank, self.world, self.stream, self.dev = cfg, n, rank, world, stream, dev
        fault_free = cfg.loss_ppm == 0 and cfg.crash_ppm == 0      # (the fault-free kernels: not persistent)
        ns = streams or STEP_STREAMS or (2 if fault_free else 4 if n <= (1 << 24) else 1)
        self.streams = step_streams(stream, dev, ns)
        ns = len(self.streams)
        # (outputs=False: run totals only, no per-instance records)
        self.out = [torch.empty((n, 4), dtype=torch.int32, device=dev) if outputs else None for _ in range(ns)]
        self.dig = [torch.empty((n, cfg.n_acceptors), dtype=torch.int32, device=dev) if outputs else None
                    for _ in range(ns)]
        self.tot = torch.zeros(16, dtype=torch.int64, device=dev)
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e1 = torch.cuda.Event(enable_timing=True)

    def launch(self, step, count):
        first = (step * self.world + self.rank) * self.n      # fresh global instance ids per step/rank
        k = step % len(self.streams)
        st = self.streams[k]
        with self.torch.cuda.stream(st):
            self.pxb.run_device(self.cfg, first, count, d_results=self.out[k], d_digests=self.dig[k],
                                d_totals=self.tot, stream=st.cuda_stream)

    def prime(self):
        # one small launch on each stream before the warmup steps: the library's
        # per-stream state (bail and split lists) is allocated on a stream's
        # first launch, which must not fall inside the timed region when the
        # warmup steps (W = 1) touch only the first stream
        for k, st in enumerate(self.streams):
            with self.torch.cuda.stream(st):
                self.pxb.run_device(self.cfg, 1 << 48, min(self.n, 1 << 12), d_results=self.out[k],
                                    d_digests=self.dig[k], d_totals=self.tot, stream=st.cuda_stream)

    def sync(self):
        self.torch.cuda.synchronize()

    def mark(self, which):
        # (e1 - e0) / K is the mean step time over all step streams, gaps between kernels included
        a = self.streams[0]
        if which == 0:
            self.e0.record(a)
            for b in self.streams[1:]:
                b.wait_event(self.e0)
        else:
            for b in self.streams[1:]:
                done_b = self.torch.cuda.Event()
                done_b.record(b)
                a.wait_event(done_b)
            self.e1.record(a)

    def event_ms(self):
        return self.e0.elapsed_time(self.e1)


class DryLeg:
    """--dry-run: the same launcher, barriers, timing and collectives on CPU
    ranks (gloo) with a synthetic stand-in for the work (no Paxos is run: the
    'totals' are instance counts).  Lets tests/test_bench_launch.py exercise the
    N-rank path of this file without GPUs."""

    def __init__(self, n, rank, world):
        import torch
        self.torch, self.n = torch, n
        self.tot = torch.zeros(16, dtype=torch.int64)
        self.t = [0.0, 0.0]

    def launch(self, step, count):
        time.sleep(0.002)
        self.tot[13] += count            # PXB_C_INSTANCES
        self.tot[0] += count             # PXB_C_DECIDED

    def sync(self):
        pass

    def mark(self, which):
        self.t[which] = time.perf_counter()

    def event_ms(self):
        return (self.t[1] - self.t[0]) * 1e3


def run_workload(leg, n, steps, warmup, world, warm_n=None):
    """Times `steps` back-to-back launches of n fresh instances per rank.
    Returns (wall seconds for the timed steps, max over ranks; mean ms per step
    from the leg's events; run totals summed over ranks)."""
    import torch
    import torch.distributed as dist
    if hasattr(leg, "prime") and warmup < len(getattr(leg, "streams", ())):   # (else the warmup touches every stream)
        leg.prime()
    for w in range(warmup):
        leg.launch(w, warm_n or n)
    leg.sync()
    leg.tot.zero_()
    if world > 1:
        dist.barrier()
    leg.sync()
    t0 = time.perf_counter()
    leg.mark(0)
    for k in range(steps):
        leg.launch(warmup + k, n)
    leg.mark(1)
    leg.sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=leg.tot.device)
    if world > 1:
        # after the timed region: the run totals (decided counts, violation
        # flags) summed over the node -- RCCL over xGMI, the only collective
        dist.all_reduce(leg.tot)
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    kms = leg.event_ms() / steps
    return float(elapsed.item()), kms, counters_dict(leg.tot.cpu().tolist())


def counters_dict(v):
    import pxb                      # the names only (pxb.COUNTER_NAMES); loads no GPU code
    return pxb.counters_dict(v)


def step_profile(workload: str):
    """The committed rocprofv3 profile of this workload (tools/profile_set.sh
    + tools/roofline.py): PMC counts per instance processed, or None."""
    for rnd in PROFILE_ROUNDS:
        path = os.path.join(PROFILES, "%s_%s" % (rnd, workload), "step.json")
        try:
            with open(path) as f:
                return json.load(f), path
        except (OSError, ValueError):
            continue
    return None, path


def roofline(workload, n, kms, canon_bytes_per_step):
    """VALU-issue roofline of one step (per GPU): the PMC-counted VALU
    wave-instructions per instance of this workload (committed profile of the
    same command) x the step's instances, over the step time measured now with
    HIP events on the launch stream; HBM bytes from the same profile's FETCH /
    WRITE passes.  The canonical SURVEY.md 8(d) byte count is reported beside
    it, never as frac: this engine does not move those bytes."""
    prof, path = step_profile(workload)
    step_s = kms * 1e-3
    r = {"bound": "valu_issue", "unit": "G VALU wave-instructions/s", "peak": VALU_PEAK_G,
         "achieved": None, "frac": None, "traffic": None,
         "peak_basis": "256 CUs x 2 wave64 VALU instructions per CU-cycle x 2.4 GHz (MI355X_MICROARCH.md)",
         "canonical_equiv_GBps": canon_bytes_per_step / step_s / 1e9,
         "canonical_note": "SURVEY.md 8(d) canonical bytes / step time: the traffic of a design whose "
                           "SoA state round-trips HBM every step; this engine keeps it on chip, so this "
                           "is not a bandwidth measurement",
         "physical_GBps": None, "physical_frac": None, "profile": os.path.relpath(path, ROOT)}
    if prof:
        valu = prof["valu_insts_per_instance"] * n
        r["achieved"] = valu / step_s / 1e9
        r["frac"] = r["achieved"] / VALU_PEAK_G
        r["valu_insts_per_step"] = valu
        r["valu_insts_per_instance"] = prof["valu_insts_per_instance"]
        r["dominant_kernel"] = prof["dominant_kernel"]
        r["dominant_share_of_kernel_time"] = prof["dominant_share"]
        r["profile_kernel_ns_per_instance"] = prof["kernel_ns_per_instance"]
        hbm = prof["hbm_bytes_per_instance"] * n
        r["traffic"] = hbm
        r["physical_GBps"] = hbm / step_s / 1e9
        r["physical_frac"] = r["physical_GBps"] / HBM_PEAK_GBS
    return r


def wire_bench(stream, dev, n=1 << 24, reps=5):
    """Wire codec: Data.Binary encode / decode of n
    ServerResponse records resident in HBM (a Round1OK-heavy mix with real
    commands), HIP events on the launch stream.  Algorithmic HBM bytes per
    message: encode (sizes, offsets and records in one call) 16 (pxb_msg) +
    8 (offset) + record; decode record + 16 offset reads + 16 (pxb_msg) + 4
    (status)."""
    import numpy as np
    import torch
    import pxb
    rng = np.random.default_rng(0)
    kind = rng.choice([0, 0, 1, 2], size=n).astype(np.uint32)
    msgs = np.zeros((n, 4), np.uint32)
    msgs[:, 0] = kind
    msgs[:, 1] = np.where(kind == 2, 0, rng.integers(1, 1 << 13, n))   # Round2Success has no field
    just = (kind == 0) & (rng.random(n) < 0.5)
    msgs[:, 2] = np.where(just, rng.integers(1, 1 << 13, n), 0)
    msgs[:, 3] = np.where(just, (rng.integers(1, 4, n) << 24) | rng.integers(1, 1 << 13, n), 0)
    d_m = torch.from_numpy(msgs.view(np.int32)).to(dev)
    d_o = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_b = torch.zeros(n * pxb.WIRE_MAX_BYTES, dtype=torch.uint8, device=dev)
    d_back = torch.zeros_like(d_m)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    sp = stream.cuda_stream

    def enc():   # fused size + encode (pxb_wire_encode_all)
        pxb.wire_encode_device(d_m, pxb.WIRE_RESPONSE, d_o, d_b, stream=sp)

    def dec():
        pxb.wire_decode_device(d_b, d_o, n, pxb.WIRE_RESPONSE, d_back, d_st, stream=sp)

    out = {"messages": n}
    with torch.cuda.stream(stream):
        for name, fn in (("encode", enc), ("decode", dec)):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(reps):
                fn()
            e1.record(stream)
            stream.synchronize()
            ms = e0.elapsed_time(e1) / reps
            nbytes = int(d_o[-1].item())
            moved = (24 * n + nbytes) if name == "encode" else (nbytes + 16 * n + 20 * n)
            out[name] = {"ms": ms, "messages_per_s": n / ms * 1e3, "wire_bytes": nbytes,
                         "hbm_GBps": moved / (ms * 1e-3) / 1e9}
    assert torch.equal(d_back, d_m) and int(d_st.abs().sum().item()) == 0
    return out


def host_cores():
    """(threads to use, CPUs in the process affinity, cgroup CPU quota or None).
    The GPU box shows the whole machine in nproc / affinity but allots a 1-GPU
    job its share (cgroup quota, and OMP_NUM_THREADS set to it): the baseline
    runs one thread per CPU of that share, every CPU it may actually use."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    n = aff
    if quota:
        n = min(n, max(1, int(quota)))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n, aff, quota


def cpu_baseline(cfg, budget_s):
    """The oracle's C port (oracle/paxos_oracle.c) on every host core the
    process may use (nproc), on a bounded sample of the same config (ids from
    2^40), then on one core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_c                          # CPU restatement (oracle/), baseline only
    threads, aff, quota = host_cores()
    chunk = 1 << 17
    done, first = 0, 1 << 40
    t0 = time.perf_counter()
    while True:
        oracle_c.run_cpu(cfg, first + done, chunk, threads=threads)
        done += chunk
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    one, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < min(3.0, budget_s):
        oracle_c.run_cpu(cfg, first + done + one, 1 << 14, threads=1)
        one += 1 << 14
    dt1 = time.perf_counter() - t1
    return {"value": done / dt, "unit": "instances/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample": "%d instances of the same config (ids from 2^40), oracle/paxos_oracle.c "
                      "on %d host threads (every CPU of the job's share), %.1f s" % (done, threads, dt),
            "one_core": {"value": one / dt1, "sample": "%d further instances, 1 thread, %.1f s" % (one, dt1)}}


def faulty_line(name, c, n, steps, warmup, stream, dev, warm_n, rank=0, world=1, leg=None, outputs=True):
    """One workload: n instances per rank per step, on every rank of the job
    (barriers, max-over-ranks time, all-reduced totals: run_workload)."""
    import pxb
    leg = leg or GpuLeg(pxb.CONFIGS[c], n, rank, world, stream, dev, outputs=outputs)
    es, ek, ecnt = run_workload(leg, n, steps, warmup, world, warm_n=warm_n)
    line = {"workload": name, "instances_per_step": n * world, "instances_per_gpu_per_step": n, "n_gpus": world,
            "instances_per_s": ecnt["instances"] / es, "decided_per_s": ecnt["decided"] / es,
            "ms_per_step": es / steps * 1e3, "kernel_ms": ek,
            "mean_steps_per_instance": ecnt["steps"] / max(1, ecnt["instances"]), "counters": ecnt}
    if leg.__class__ is GpuLeg:
        line["roofline"] = roofline("config%d" % c, n, ek, ecnt["canon_bytes"] / (steps * world))
    assert ecnt["instances"] == n * steps * world, ecnt
    assert ecnt["decided"] + ecnt["undecided"] == ecnt["instances"]
    return line


LOG_STEPS = 8                # timed steps of the faulty-log-mode lines (round 5: 2)
LOG_SAME_TOTAL = 8 << 22     # (the 2^20 line's second rate: as many instances as the 2^22 line's 8 steps)
LOG_STREAMS = 8              # their step streams: every call in flight on its own stream and hardware queue
# (MI355X, 8 steps, profiles/r06_notes/ab_log_streams.txt: 2^20 144 / 153 / 161 / 162-171 M/s
# on 2 / 3 / 4 / 8 streams, 2^22 180 / 183 / 186 / 188-191; 8 streams need the 8 queues above)


def log_faulty_line(stream, dev, n=1 << 22, general=True):
    """Faulty log mode (pxb.LOG_FAULTY_CONFIG: P = 2, N = 5, 10 % loss, delays
    to 4, crash windows, 16 Ticks 8 steps apart) on the per-lane kernel's
    log-mode shape, and (general=True) the same batch on the general kernel
    (PXB_NO_EV=1) for the speed-up; the totals of the two must be identical.
    LOG_STEPS timed steps on LOG_STREAMS step streams.  The batch's instance
    lengths have a heavy tail (median 124 steps, the longest ~950: 7.7 x), so
    a call's last waves run its longest instances for 2-5 ms after its work
    queue drained (profiles/r06_notes/lg_wave_times_2p20.txt: at 2^20 the
    queue drains at 5.0 ms and the last wave ends at 10.2 ms); the other calls
    in flight on their own streams fill that tail, and one tail stays exposed
    per measurement.  Round 5 timed 2 steps on 2 streams (that rate is
    reported beside it)."""
    import pxb
    cfg = pxb.LOG_FAULTY_CONFIG
    es, ek, ecnt = run_workload(GpuLeg(cfg, n, 0, 1, stream, dev, streams=LOG_STREAMS), n, LOG_STEPS, 1, 1)
    e2s, _, e2cnt = run_workload(GpuLeg(cfg, n, 0, 1, stream, dev), n, 2, 1, 1)
    line = {"workload": "faulty log mode: P=2, N=5, 10% loss, delay [1,4], crash windows, 16 Ticks / 8 steps",
            "instances_per_step": n, "steps": LOG_STEPS, "step_streams": LOG_STREAMS,
            "hw_queues": _hw_queues(),
            "instances_per_s": ecnt["instances"] / es,
            "commands_committed_per_s": ecnt["executes"] / es, "kernel_ms": ek,
            "instances_per_s_2_steps": e2cnt["instances"] / e2s,     # (2 steps on 2 streams: round 5's measurement)
            "roofline": roofline("config7", n, ek, ecnt["canon_bytes"] / LOG_STEPS), "counters": ecnt}
    if n < LOG_SAME_TOTAL // LOG_STEPS:
        # (the same total instances per measurement as the 2^22 line, so that
        # its one exposed tail weighs the same: steady-state calls of n)
        k = LOG_SAME_TOTAL // n
        ts, _, tcnt = run_workload(GpuLeg(cfg, n, 0, 1, stream, dev, streams=LOG_STREAMS), n, k, 1, 1)
        line["same_total"] = {"steps": k, "instances_per_s": tcnt["instances"] / ts}
    if general:
        with pxb.hooks(PXB_NO_EV="1"):
            gs, gk, gcnt = run_workload(GpuLeg(cfg, n, 0, 1, stream, dev, streams=LOG_STREAMS), n, LOG_STEPS, 1, 1)
        assert gcnt == ecnt, (gcnt, ecnt)
        line["general_kernel"] = {"instances_per_s": gcnt["instances"] / gs, "kernel_ms": gk}
        line["speedup_vs_general_kernel"] = gk / ek
    return line


def headline_workload(c, n, world):
    if c == 4:
        return ("BASELINE config 4 (north star): 2^26 instances per step, 2 duelling proposers, 7 acceptors, "
                "delays [1,4], seeded crash windows, over %d GPU%s (%d per GPU)" % (world, "s" if world > 1 else "", n))
    if c == 2:
        return "BASELINE config 2: %d fresh instances per GPU per step (%d x the 2^20 batch)" % (n, n >> 20)
    return "BASELINE config %d: %d instances per GPU per step" % (c, n)


def dry_main(args, rank, world):
    """--dry-run: the N-rank launcher path on CPU (gloo); prints the JSON line
    shape with a synthetic workload and "data": "dry-run" (not a measurement).
    The headline is strong-scaled like config 4's: one batch of --instances
    (default DRY_NORTH_STAR) per step split over the ranks."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    total = args.instances or DRY_NORTH_STAR
    n = total // world
    secs, kms, cnt = run_workload(DryLeg(n, rank, world), n, args.steps, args.warmup, world)
    assert cnt["instances"] == n * world * args.steps, cnt
    if rank == 0:
        line = {"metric": "dry-run", "value": cnt["decided"] / secs, "unit": "instances/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": secs / args.steps * 1e3,
                "scaling": "strong", "data": "dry-run",
                "config": {"workload": headline_workload(4, n, world), "instances_per_step": n * world,
                           "instances_per_gpu_per_step": n, "rccl_world": world},
                "counters": cnt}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if args.dry_run:
        return dry_main(args, rank, world)
    global STEP_STREAMS
    STEP_STREAMS = 1 if args.one_stream else args.streams
    import pxb
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(dev)
    # (every step stream a workload may take, created first: consecutive
    # creations get distinct hardware queues, HW_QUEUES)
    step_streams(stream, dev, max(LOG_STREAMS, 4))
    c = args.config
    cfg = pxb.CONFIGS[c]
    n = step_instances(c, args.instances, world)

    # the headline: K timed steps of n fresh instances per rank (BASELINE
    # config 4 by default: 2^26 / N per rank, strong scaling)
    secs, kms, cnt = run_workload(GpuLeg(cfg, n, rank, world, stream, dev), n, args.steps, args.warmup, world)
    total_inst = n * world * args.steps
    assert cnt["instances"] == total_inst, cnt
    assert cnt["decided"] + cnt["undecided"] == total_inst, cnt
    if c == 2:   # closed forms of the fault-free config: every instance decides
        assert cnt["decided"] == total_inst and cnt["canon_bytes"] == 1140 * total_inst, cnt
    value = cnt["decided"] / secs                         # decided instances / s, whole job
    line = {
        "metric": "Paxos instances decided/sec (node)",
        "value": value,
        "unit": "instances/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": secs / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling_of(c),
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (Philox4x32-10 schedule from seed + global instance id)",
        "config": {"workload": headline_workload(c, n, world),
                   "instances_per_step": n * world, "instances_per_gpu_per_step": n,
                   "proposers": cfg.n_proposers, "acceptors": cfg.n_acceptors,
                   "loss_ppm": cfg.loss_ppm, "delay_max": cfg.delay_max, "skew_max": cfg.skew_max,
                   "crash_ppm": cfg.crash_ppm, "step_cap": cfg.step_cap,
                   "randomize": cfg.randomize, "seed": hex(cfg.seed),
                   "parallelism": "instance-range shards x%d" % world, "rccl_world": world},
        "instances_per_s": cnt["instances"] / secs,
        "kernel_ms_per_step": kms,
        "roofline": roofline("config%d" % c, n, kms, cnt["canon_bytes"] / (args.steps * world)),
        "counters": cnt,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0 and not args.no_extra and c == 4 and world == 1:
        extra = {}
        # config 2 (fault-free, 1 proposer, 5 acceptors): 2^28 fresh instances
        # per step, the round 1-3 headline
        extra["config2"] = faulty_line(headline_workload(2, step_instances(2, 0), 1), 2, step_instances(2, 0),
                                       10, 1, stream, dev, None)
        if not args.no_cpu:
            extra["config2"]["cpu_baseline"] = cpu_baseline(pxb.CONFIGS[2], 3.0)
        # config 4 at its per-GPU share at N = 8 (2^23): the chunk-tail cost at
        # that size, before any 8-GPU run
        extra["config4_share"] = faulty_line("BASELINE config 4: 2^23 instances (the per-GPU share of 2^26 "
                                             "over 8 GPUs) on 1 GPU", 4, pxb.CONFIG_INSTANCES[4] // 8, 4, 1,
                                             stream, dev, 1 << 22)
        extra["config3"] = faulty_line("BASELINE config 3: 2^24 instances", 3, pxb.CONFIG_INSTANCES[3],
                                       4, 1, stream, dev, 1 << 22)
        extra["config5"] = faulty_line("BASELINE config 5: 2^25 instances (the per-GPU share of 2^28 "
                                       "over 8 GPUs)", 5, pxb.CONFIG_INSTANCES[5] // 8, 1, 1, stream, dev,
                                       1 << 22)
        # config 5 at its stated size: the whole 2^28-schedule sweep on this
        # one GPU, run totals only (agreement-violation flags summed)
        extra["config5_full"] = faulty_line("BASELINE config 5: all 2^28 randomized schedules on 1 GPU, "
                                            "run totals only", 5, pxb.CONFIG_INSTANCES[5], 1, 0, stream, dev,
                                            None, outputs=False)
        extra["wire_codec"] = wire_bench(stream, dev)
        # log mode: stock Main.hs topology with the ticker running (SEMANTICS §9)
        en = 1 << 20
        es, ek, ecnt = run_workload(GpuLeg(pxb.LOG_CONFIG, en, 0, 1, stream, dev), en, 2, 1, 1)
        extra["log_mode"] = {"instances_per_step": en, "ticks_per_proposer": pxb.LOG_CONFIG.n_ticks,
                             "commands_committed_per_s": ecnt["executes"] / es,
                             "instances_per_s": ecnt["instances"] / es, "kernel_ms": ek, "counters": ecnt}
        extra["log_mode_faulty"] = log_faulty_line(stream, dev, 1 << 22)
        extra["log_mode_faulty_2p20"] = log_faulty_line(stream, dev, 1 << 20, general=False)
        line["extra"] = extra
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
