"""ctypes binding of the C oracle (oracle/paxos_oracle.c) — TEST INFRASTRUCTURE
AND CPU BASELINE ONLY (tests/, __graft_entry__.smoke, bench.py cpu_baseline).

Uses the ABI structs of the product binding (cloud-haskell-paxos_amd/pxb.py);
the product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.join(os.path.dirname(_HERE), "cloud-haskell-paxos_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)
import pxb  # noqa: E402

LIB_PATH = os.path.join(_HERE, "_build", "libpaxos_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        lib = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        lib.pxb_run_cpu.argtypes = [C.POINTER(pxb.pxb_config), vp, vp, vp, vp, C.c_int]
        lib.pxb_run_cpu.restype = C.c_int
        lib.pxb_oracle_acceptor_handle.argtypes = [vp, vp, vp, C.c_uint32]
        lib.pxb_oracle_proposer_handle.argtypes = [vp, C.c_uint32, vp, vp, vp, C.c_uint32]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def run_cpu(cfg: "pxb.Config", first: int, n: int, threads: int = 1, want_acceptors=False):
    lib = load()
    N = cfg.n_acceptors
    res = np.zeros((n, 4), dtype=np.uint32)
    dig = np.zeros((n, N), dtype=np.uint32)
    acc = np.zeros((n, N, 4), dtype=np.uint32) if want_acceptors else None
    tot = pxb.pxb_counters()
    c = cfg.to_c(first, n)
    rc = lib.pxb_run_cpu(C.byref(c), _p(res), _p(dig), _p(acc), C.cast(C.byref(tot), C.c_void_p), threads)
    if rc != 0:
        raise ValueError("pxb_run_cpu rc=%d" % rc)
    return res, dig, acc, pxb.counters_dict(tot.c)


def acceptor_handle(states: np.ndarray, msgs: np.ndarray):
    lib = load()
    st = np.ascontiguousarray(states, dtype=np.uint32).copy()
    reply = np.zeros((len(st), 4), dtype=np.uint32)
    lib.pxb_oracle_acceptor_handle(_p(st), _p(np.ascontiguousarray(msgs, dtype=np.uint32)), _p(reply), len(st))
    return st, reply


def proposer_handle(states: np.ndarray, n_acceptors: int, msgs: np.ndarray):
    lib = load()
    st = np.ascontiguousarray(states, dtype=np.uint32).copy()
    bc = np.zeros((len(st), 2, 4), dtype=np.uint32)
    nb = np.zeros(len(st), dtype=np.uint32)
    lib.pxb_oracle_proposer_handle(_p(st), n_acceptors, _p(np.ascontiguousarray(msgs, dtype=np.uint32)),
                                   _p(bc), _p(nb), len(st))
    return st, bc, nb
