"""Python host binding of the batched Paxos C ABI (include/paxos_batch.h).

This is the host side above the C-ABI for environments without GHC (the
reference's own host is Haskell: /root/reference/app/Main.hs; the Haskell
binding a maintainer would add lives in hs/ and INTEGRATION.md).  It mirrors
the reference's vocabulary (/root/reference/src/Common.hs:20-68): ``Ticket``,
``Command`` ("c<clientId>.<t>", Client.hs:202-203), ``Proposal``,
``ClientRequest`` / ``ServerResponse`` constructors.

The product path is ``libpaxos_batch.so`` (HIP kernels for gfx950).  There is
NO CPU fallback here: when the library (or a GPU) is missing every entry point
raises.  The CPU restatement used as test oracle lives in ``oracle/`` and is
never imported by this module.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PXB_LIB") or os.path.join(_HERE, "csrc", "libpaxos_batch.so")

# ---- constants (include/paxos_batch.h) ------------------------------------
PXB_OK, PXB_E_INVAL, PXB_E_HIP, PXB_E_OOM, PXB_E_NODEV, PXB_E_RCCL = 0, -1, -2, -3, -4, -5
MAX_PROPOSERS, MIN_ACCEPTORS, MAX_ACCEPTORS = 3, 2, 9
MAX_DELAY, MAX_STEP_CAP, QUEUE_DEPTH, LOG_TRACK, MAX_TICKS = 15, 8192, 8, 32, 4096
CFG_RANDOMIZE = 1
CFG_TRACE_PRODUCTION = 2         # pxb_trace_instance: the batch kernels' carry-over variant
TRACE_IN_FLIGHT_UNKNOWN = 0xFFFFFFFF

F_UNDECIDED, F_STUCK, F_PANIC, F_LOG_DIVERGENCE = 1, 2, 4, 8
F_STEP_CAP, F_QUEUE_OVERFLOW, F_TICKET_OVERFLOW, F_LOG_TRUNC = 16, 32, 64, 128
FLAG_NAMES = {F_UNDECIDED: "UNDECIDED", F_STUCK: "STUCK", F_PANIC: "PANIC",
              F_LOG_DIVERGENCE: "LOG_DIVERGENCE", F_STEP_CAP: "STEP_CAP",
              F_QUEUE_OVERFLOW: "QUEUE_OVERFLOW", F_TICKET_OVERFLOW: "TICKET_OVERFLOW",
              F_LOG_TRUNC: "LOG_TRUNC"}

NCOUNTERS = 16
COUNTER_NAMES = ["decided", "undecided", "stuck", "panic", "divergence", "step_cap",
                 "rounds", "messages", "queue_overflow", "ticket_overflow", "log_trunc",
                 "canon_bytes", "steps", "instances", "executes", "reserved15"]

# ClientRequest (Common.hs:41-45) / ServerResponse (Common.hs:49-53) tags
AskForTicket, Propose, Execute = 0, 1, 2
Round1OK, HaveTicket, Round2Success = 0, 1, 2
Tick = 3
MSG_NONE = 0xFFFFFFFF
Idle, Round1, Round2 = 0, 1, 2


class pxb_config(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("first_instance", C.c_uint64),
                ("n_instances", C.c_uint64), ("n_proposers", C.c_uint32),
                ("n_acceptors", C.c_uint32), ("loss_ppm", C.c_uint32),
                ("delay_max", C.c_uint32), ("crash_ppm", C.c_uint32),
                ("crash_len_max", C.c_uint32), ("crash_start_max", C.c_uint32),
                ("skew_max", C.c_uint32), ("step_cap", C.c_uint32), ("flags", C.c_uint32),
                ("n_ticks", C.c_uint32), ("tick_period", C.c_uint32)]


class pxb_result(C.Structure):
    _fields_ = [("decided_val", C.c_uint32), ("decided_ticket", C.c_int32),
                ("rounds", C.c_uint32), ("flags", C.c_uint32)]


class pxb_acceptor_rec(C.Structure):
    _fields_ = [("t_max", C.c_int32), ("t_store", C.c_int32), ("val", C.c_uint32),
                ("meta", C.c_uint32)]


class pxb_counters(C.Structure):
    _fields_ = [("c", C.c_int64 * NCOUNTERS)]


class pxb_msg(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("x", C.c_int32), ("y", C.c_int32), ("z", C.c_uint32)]


class pxb_proposer_rec(C.Structure):
    _fields_ = [("ticket", C.c_int32), ("cmd", C.c_uint32), ("acks", C.c_uint32),
                ("state", C.c_uint32), ("mr_t", C.c_int32), ("mr_v", C.c_uint32),
                ("r2_t", C.c_int32), ("r2_v", C.c_uint32), ("pending", C.c_uint32),
                ("client_id", C.c_uint32)]


assert C.sizeof(pxb_config) == 72 and C.sizeof(pxb_result) == 16
assert C.sizeof(pxb_acceptor_rec) == 16 and C.sizeof(pxb_msg) == 16

# ---- Common.hs vocabulary ------------------------------------------------


def command(client_id: int, t: int) -> int:
    """Encode the Command "c<clientId>.<t>" (Client.hs:202-203)."""
    return ((client_id & 0xFF) << 24) | (t & 0xFFFFFF)


def command_str(code: int) -> Optional[str]:
    """Decode a Command code back into the reference's String (None = Nothing)."""
    if code == 0:
        return None
    return "c%d.%d" % (code >> 24, code & 0xFFFFFF)


def flag_names(flags: int):
    return [n for b, n in FLAG_NAMES.items() if flags & b]


# ---- named configurations (BASELINE.json configs) -------
@dataclass
class Config:
    seed: int
    n_proposers: int = 1
    n_acceptors: int = 5
    loss_ppm: int = 0
    delay_max: int = 1
    crash_ppm: int = 0
    crash_len_max: int = 1
    crash_start_max: int = 0
    skew_max: int = 0
    step_cap: int = 256
    randomize: bool = False
    n_ticks: int = 1          # log mode when > 1: Ticks per proposer (Client.hs:96-100)
    tick_period: int = 1      # steps between Ticks

    def to_c(self, first_instance: int, n_instances: int) -> pxb_config:
        return pxb_config(self.seed, first_instance, n_instances, self.n_proposers,
                          self.n_acceptors, self.loss_ppm, self.delay_max, self.crash_ppm,
                          self.crash_len_max, self.crash_start_max, self.skew_max,
                          self.step_cap, CFG_RANDOMIZE if self.randomize else 0,
                          self.n_ticks, self.tick_period)


CONFIGS = {
    1: Config(seed=0x5EED0001, n_proposers=1, n_acceptors=3),
    2: Config(seed=0x5EED0002, n_proposers=1, n_acceptors=5),
    3: Config(seed=0x5EED0003, n_proposers=2, n_acceptors=5, loss_ppm=100000,
              delay_max=4, skew_max=3, step_cap=256),
    4: Config(seed=0x5EED0004, n_proposers=2, n_acceptors=7, delay_max=4,
              crash_ppm=200000, crash_len_max=16, crash_start_max=8, step_cap=256),
    5: Config(seed=0x5EED0005, n_proposers=3, n_acceptors=9, loss_ppm=300000,
              delay_max=8, crash_ppm=200000, crash_len_max=16, crash_start_max=16,
              skew_max=3, step_cap=512, randomize=True),
}
CONFIG_INSTANCES = {1: 1 << 10, 2: 1 << 20, 3: 1 << 24, 4: 1 << 26, 5: 1 << 28, 6: 1 << 20, 7: 1 << 20}

# Log mode (docs/SEMANTICS.md §9): the stock app/Main.hs
# topology (2 proposers, 2 acceptors, Main.hs:41-46) with the ticker running
# (Client.hs:96-100): 16 Ticks per proposer, 8 steps apart.
LOG_CONFIG = Config(seed=0x5EED0006, n_proposers=2, n_acceptors=2, step_cap=1024,
                    n_ticks=16, tick_period=8)
CONFIGS[6] = LOG_CONFIG
# Faulty log mode: config 3's duel and loss with crash windows, 16 Ticks per
# proposer (the per-lane kernel's log-mode shape; bench.py extra.log_mode_faulty)
LOG_FAULTY_CONFIG = Config(seed=0x5EED0007, n_proposers=2, n_acceptors=5, loss_ppm=100000, delay_max=4,
                           skew_max=3, crash_ppm=200000, crash_len_max=16, crash_start_max=64, step_cap=1024,
                           n_ticks=16, tick_period=8)
CONFIGS[7] = LOG_FAULTY_CONFIG


def canonical_bytes_nofault(n_acceptors: int) -> int:
    """B = 196 N + 160 for a fault-free P = 1 instance."""
    return 196 * n_acceptors + 160


# ---- library loading --------------------------------------------------------
_lib = None
ABI_VERSION = 5          # PXB_ABI_VERSION of include/paxos_batch.h this mirror binds


class PaxosError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load libpaxos_batch.so.  Raises (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise PaxosError("libpaxos_batch.so not built at %s — run __graft_entry__.build()" % path)
    lib = C.CDLL(path)
    vp = C.c_void_p
    lib.pxb_run.argtypes = [C.POINTER(pxb_config), vp, vp, vp, vp]
    lib.pxb_run.restype = C.c_int
    lib.pxb_run_device.argtypes = [C.POINTER(pxb_config), vp, vp, vp, vp, vp]
    lib.pxb_run_device.restype = C.c_int
    lib.pxb_run_multi.argtypes = [C.POINTER(pxb_config), C.c_int, vp, vp, vp, vp]
    lib.pxb_run_multi.restype = C.c_int
    lib.pxb_acceptor_handle.argtypes = [vp, vp, vp, C.c_uint32]
    lib.pxb_acceptor_handle.restype = C.c_int
    lib.pxb_proposer_handle.argtypes = [vp, C.c_uint32, vp, vp, vp, C.c_uint32]
    lib.pxb_proposer_handle.restype = C.c_int
    lib.pxb_strerror.argtypes = [C.c_int]
    lib.pxb_strerror.restype = C.c_char_p
    lib.pxb_last_hip_error.restype = C.c_int
    lib.pxb_abi_version.restype = C.c_int
    lib.pxb_canonical_bytes_nofault.argtypes = [C.c_uint32]
    lib.pxb_canonical_bytes_nofault.restype = C.c_uint64
    for name, args in (("pxb_wire_size", [vp, C.c_uint64, C.c_uint32, vp, vp]),
                       ("pxb_wire_encode", [vp, C.c_uint64, C.c_uint32, vp, vp, vp]),
                       ("pxb_wire_encode_all", [vp, C.c_uint64, C.c_uint32, vp, vp, vp]),
                       ("pxb_wire_decode", [vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, vp, vp]),
                       ("pxb_wire_encode_host", [vp, C.c_uint64, C.c_uint32, vp, vp, vp]),
                       ("pxb_wire_decode_host", [vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, vp]),
                       ("pxb_init", [C.c_int]), ("pxb_shutdown", []),
                       ("pxb_trace_instance", [vp, C.c_uint64, vp, C.c_uint32, vp, vp])):
        getattr(lib, name).argtypes = args
        getattr(lib, name).restype = C.c_int
    lib.pxb_stream_release.argtypes = [C.c_int, vp]
    lib.pxb_stream_release.restype = None
    lib.pxb_handoff_counts.argtypes = [C.c_int, vp, C.c_int]
    lib.pxb_handoff_counts.restype = C.c_int
    lib.pxb_reload_hooks.argtypes = []
    lib.pxb_reload_hooks.restype = None
    if lib.pxb_abi_version() != ABI_VERSION:          # (a stale build: its struct layouts may differ)
        raise PaxosError("libpaxos_batch.so has ABI %d, this binding expects %d — rebuild it"
                         % (lib.pxb_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(rc: int):
    if rc != PXB_OK:
        lib = load()
        raise PaxosError("pxb error %d: %s (hip %d)" % (rc, lib.pxb_strerror(rc).decode(),
                                                         lib.pxb_last_hip_error()))


def _ptr(a):
    """Address of a numpy array / torch tensor / None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return C.c_void_p(a.ctypes.data)


def run(cfg: Config, first_instance: int, n_instances: int, want_results=True,
        want_digests=True, want_acceptors=False):
    """Host-buffer batch run (pxb_run).  Returns numpy arrays + counters dict."""
    import numpy as np
    lib = load()
    N = cfg.n_acceptors
    res = np.zeros((n_instances, 4), dtype=np.uint32) if want_results else None
    dig = np.zeros((n_instances, N), dtype=np.uint32) if want_digests else None
    acc = np.zeros((n_instances, N, 4), dtype=np.uint32) if want_acceptors else None
    tot = pxb_counters()
    c = cfg.to_c(first_instance, n_instances)
    check(lib.pxb_run(C.byref(c), _ptr(res), _ptr(dig), _ptr(acc), C.cast(C.byref(tot), C.c_void_p)))
    return res, dig, acc, counters_dict(tot.c)


def run_multi(cfg: Config, first_instance: int, n_instances: int, n_devices: int = 0,
              want_results=True, want_digests=True):
    """Host-buffer batch sharded over devices 0..n_devices-1 (pxb_run_multi):
    one thread per GPU, one RCCL all-reduce of the run totals."""
    import numpy as np
    lib = load()
    N = cfg.n_acceptors
    res = np.zeros((n_instances, 4), dtype=np.uint32) if want_results else None
    dig = np.zeros((n_instances, N), dtype=np.uint32) if want_digests else None
    tot = pxb_counters()
    c = cfg.to_c(first_instance, n_instances)
    check(lib.pxb_run_multi(C.byref(c), n_devices, _ptr(res), _ptr(dig), None,
                            C.cast(C.byref(tot), C.c_void_p)))
    return res, dig, counters_dict(tot.c)


def _check_buf(name, t, words, itemsize):
    """A device output buffer must be a contiguous GPU tensor of 4-byte (or, for
    the totals, 8-byte) integers holding at least `words` elements: the kernels
    write through its raw address."""
    if t is None:
        return
    if not getattr(t, "is_cuda", False):
        raise ValueError("%s: a CUDA (HIP) tensor is required" % name)
    if t.element_size() != itemsize or t.dtype.is_floating_point or not t.is_contiguous():
        raise ValueError("%s: contiguous %d-byte integer tensor required" % (name, itemsize))
    if t.numel() < words:
        raise ValueError("%s: %d elements, %d needed" % (name, t.numel(), words))


def _check_bytes(name, t, nbytes):
    """A device byte buffer: contiguous GPU uint8 tensor of at least nbytes
    (its element count is the byte bound handed to the C ABI)."""
    import torch
    if not getattr(t, "is_cuda", False):
        raise ValueError("%s: a CUDA (HIP) tensor is required" % name)
    if t.dtype != torch.uint8 or not t.is_contiguous():
        raise ValueError("%s: contiguous uint8 tensor required" % name)
    if t.numel() < nbytes:
        raise ValueError("%s: %d bytes, %d needed" % (name, t.numel(), nbytes))


def run_device(cfg: Config, first_instance: int, n_instances: int, d_results=None,
               d_digests=None, d_acceptors=None, d_totals=None, stream=None):
    """Device-buffer, asynchronous batch run (pxb_run_device) on torch tensors
    (sizes and dtypes checked here: the C ABI takes raw pointers)."""
    N = cfg.n_acceptors
    _check_buf("d_results", d_results, 4 * n_instances, 4)
    _check_buf("d_digests", d_digests, N * n_instances, 4)
    _check_buf("d_acceptors", d_acceptors, 4 * N * n_instances, 4)
    if d_totals is None:
        raise ValueError("d_totals is required")
    _check_buf("d_totals", d_totals, NCOUNTERS, 8)
    lib = load()
    c = cfg.to_c(first_instance, n_instances)
    s = C.c_void_p(stream) if stream else None
    check(lib.pxb_run_device(C.byref(c), _ptr(d_results), _ptr(d_digests), _ptr(d_acceptors),
                             _ptr(d_totals), s))


def counters_dict(c) -> dict:
    return {COUNTER_NAMES[i]: int(c[i]) for i in range(NCOUNTERS)}


def acceptor_handle(states, msgs):
    """GPU hook: handleClientRequest (Server.hs:51-78) on arrays of
    pxb_acceptor_rec / pxb_msg (numpy uint32 views, shape (n, 4))."""
    import numpy as np
    lib = load()
    n = len(states)
    reply = np.zeros((n, 4), dtype=np.uint32)
    check(lib.pxb_acceptor_handle(_ptr(states), _ptr(msgs), _ptr(reply), n))
    return reply


def proposer_handle(states, n_acceptors, msgs):
    """GPU hook: handleServerResponse / handleTick (Client.hs:125-207) on
    arrays of pxb_proposer_rec (uint32 (n,10)) / pxb_msg (uint32 (n,4))."""
    import numpy as np
    lib = load()
    n = len(states)
    bc = np.zeros((n, 2, 4), dtype=np.uint32)
    nb = np.zeros(n, dtype=np.uint32)
    check(lib.pxb_proposer_handle(_ptr(states), n_acceptors, _ptr(msgs), _ptr(bc), _ptr(nb), n))
    return bc, nb


# ---- wire format (include/paxos_batch.h) ------------------
WIRE_REQUEST, WIRE_RESPONSE, WIRE_MAX_BYTES = 0, 1, 39
WIRE_OK, WIRE_E_LENGTH, WIRE_E_TAG, WIRE_E_STRING, WIRE_E_RANGE = 0, 1, 2, 3, 4


def wire_encode(msgs, wire_type):
    """Data.Binary encoding (Common.hs:24,47,55) of pxb_msg records
    (numpy uint32 (n, 4)) on the GPU.  Returns (bytes, offsets[n + 1])."""
    import numpy as np
    lib = load()
    msgs = np.ascontiguousarray(msgs, dtype=np.uint32)
    n = len(msgs)
    out = np.zeros(max(1, n * WIRE_MAX_BYTES), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.uint64)
    nb = C.c_uint64(0)
    check(lib.pxb_wire_encode_host(_ptr(msgs), n, wire_type, _ptr(out), _ptr(offs), C.byref(nb)))
    return out[:nb.value].tobytes(), offs


def wire_encode_device(d_msgs, wire_type, d_offsets, d_bytes, stream=None):
    """Fused size + encode on device tensors (pxb_wire_encode_all): d_msgs
    int32 (n, 4), d_offsets int64 (n + 1), d_bytes uint8 (n * WIRE_MAX_BYTES),
    asynchronous on `stream` (a raw hipStream_t handle, default stream if None)."""
    n = d_msgs.shape[0]
    _check_buf("d_msgs", d_msgs, 4 * n, 4)
    _check_bytes("d_bytes", d_bytes, max(1, n * WIRE_MAX_BYTES))
    _check_buf("d_offsets", d_offsets, n + 1, 8)
    lib = load()
    check(lib.pxb_wire_encode_all(C.c_void_p(d_msgs.data_ptr()), n, wire_type, C.c_void_p(d_offsets.data_ptr()),
                                  C.c_void_p(d_bytes.data_ptr()), C.c_void_p(stream or 0)))


def wire_decode_device(d_bytes, d_offsets, n, wire_type, d_msgs, d_status=None, stream=None):
    """pxb_wire_decode on device tensors: d_bytes uint8 (its whole length is the
    buffer bound), d_offsets int64 (n + 1), d_msgs int32 (n, 4), d_status int32
    (n,) or None; asynchronous on `stream` (raw hipStream_t, default if None)."""
    _check_bytes("d_bytes", d_bytes, 1)
    _check_buf("d_offsets", d_offsets, n + 1, 8)
    _check_buf("d_msgs", d_msgs, 4 * n, 4)
    _check_buf("d_status", d_status, n, 4)
    lib = load()
    check(lib.pxb_wire_decode(C.c_void_p(d_bytes.data_ptr()), d_bytes.numel(), C.c_void_p(d_offsets.data_ptr()), n,
                              wire_type, C.c_void_p(d_msgs.data_ptr()),
                              C.c_void_p(d_status.data_ptr() if d_status is not None else 0), C.c_void_p(stream or 0)))


TRACE_WORDS = 4 + 9 * 4 + 9 + 3 * 8      # pxb_trace_step, uint32 words


def trace_instance(cfg: Config, instance: int, max_records: int = 8192, production: bool = False):
    """pxb_trace_instance: the state at the end of every visited step of one
    instance, as a list of dicts (step, in_flight, acc (N, 4), digest (N,),
    prop (P, 8): ticket, cmd, acks, state, mr_t, mr_v, r2_v, pending), and its
    pxb_result.  production=True traces the batch kernels' carry-over variant
    (PXB_CFG_TRACE_PRODUCTION; in_flight may be TRACE_IN_FLIGHT_UNKNOWN)."""
    import numpy as np
    lib = load()
    buf = np.zeros((max_records, TRACE_WORDS), dtype=np.uint32)
    nrec = C.c_uint32(0)
    res = np.zeros(4, dtype=np.uint32)
    c = cfg.to_c(instance, 1)
    if production:
        c.flags |= CFG_TRACE_PRODUCTION
    check(lib.pxb_trace_instance(C.byref(c), instance, _ptr(buf), max_records, C.byref(nrec), _ptr(res)))
    out = []
    for r in buf[:nrec.value]:
        N, P = int(r[2]), int(r[3])
        out.append({"step": int(r[0]), "in_flight": int(r[1]),
                    "acc": r[4:4 + 36].reshape(9, 4)[:N].copy(), "digest": r[40:49][:N].copy(),
                    "prop": r[49:49 + 24].reshape(3, 8)[:P].copy()})
    return out, res


def init(n_devices: int = 0):
    """pxb_init: allocate the per-device scratch of devices 0..n-1 up front."""
    check(load().pxb_init(n_devices))


def stream_release(dev: int, stream: int):
    """pxb_stream_release: a stream used with run_device is about to be
    destroyed; its bailed-id lists go back to the library."""
    load().pxb_stream_release(dev, C.c_void_p(stream))


def handoff_counts(dev: int = 0, reset: bool = True):
    """pxb_handoff_counts: (first per-lane kernel, second per-lane kernel)
    hand-off counts of device dev since its scratch was created or last reset."""
    out = (C.c_uint64 * 2)()
    check(load().pxb_handoff_counts(dev, C.cast(out, C.c_void_p), 1 if reset else 0))
    return int(out[0]), int(out[1])


def reload_hooks():
    """pxb_reload_hooks: re-read the library's test / A-B hooks (PXB_NO_EV,
    PXB_NO_TIGHT, PXB_EV_BAIL_CAP, ...) from the environment."""
    load().pxb_reload_hooks()


class hooks:
    """Context manager for tests and A/B runs: sets the given PXB_* hooks in
    the environment, has the library re-read them, and restores both on exit.

        with pxb.hooks(PXB_NO_EV="1"):
            pxb.run(cfg, 0, n)
    """

    def __init__(self, **env):
        self.env = {k: str(v) for k, v in env.items()}
        self.old = {}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.env}
        os.environ.update(self.env)
        reload_hooks()
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        reload_hooks()
        return False


def shutdown():
    """pxb_shutdown: free every per-device scratch buffer and the cached RCCL
    communicators (the next call allocates them again)."""
    check(load().pxb_shutdown())


def wire_decode(data: bytes, offsets, wire_type):
    """Inverse of wire_encode: (msgs (n, 4) uint32, status (n,) uint32)."""
    import numpy as np
    lib = load()
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = len(offs) - 1
    buf = np.frombuffer(data, dtype=np.uint8) if data else np.zeros(1, np.uint8)
    buf = np.ascontiguousarray(buf)
    msgs = np.zeros((max(n, 0), 4), dtype=np.uint32)
    st = np.zeros(max(n, 0), dtype=np.uint32)
    check(lib.pxb_wire_decode_host(_ptr(buf), len(data), _ptr(offs), n, wire_type, _ptr(msgs), _ptr(st)))
    return msgs, st
