"""CPU-side checks of the C-ABI boundary (include/paxos_batch.h): the HIP
library loads without a GPU, exports every declared entry point, its structs
match the header, and it fails loudly (never falls back to a CPU path)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import pxb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "paxos_batch.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\*?\s+\*?(pxb_[a-z_]+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    names = _declared()
    for f in ("pxb_run", "pxb_run_device", "pxb_acceptor_handle", "pxb_proposer_handle",
              "pxb_strerror", "pxb_last_hip_error", "pxb_abi_version", "pxb_init", "pxb_shutdown",
              "pxb_run_multi", "pxb_stream_release", "pxb_handoff_counts", "pxb_reload_hooks"):
        assert f in names


def test_library_exports_every_declared_symbol():
    lib = pxb.load()
    out = subprocess.run(["nm", "-D", "--defined-only", pxb.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (pxb_\w+)", out))
    for name in _declared():
        assert name in exported, name
        assert hasattr(lib, name)


def test_struct_layout_matches_header():
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "paxos_batch.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(pxb_config), sizeof(pxb_result),
         sizeof(pxb_acceptor_rec), sizeof(pxb_counters), sizeof(pxb_msg), sizeof(pxb_proposer_rec),
         offsetof(pxb_config, step_cap), offsetof(pxb_config, tick_period));
  return 0;
}'''
    tmp = "/tmp/pxb_layout"
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", tmp, tmp + ".c"], check=True)
    got = [int(x) for x in subprocess.run([tmp], capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(pxb.pxb_config), C.sizeof(pxb.pxb_result), C.sizeof(pxb.pxb_acceptor_rec),
                   C.sizeof(pxb.pxb_counters), C.sizeof(pxb.pxb_msg), C.sizeof(pxb.pxb_proposer_rec),
                   pxb.pxb_config.step_cap.offset, pxb.pxb_config.tick_period.offset]


def test_misc_entry_points_without_gpu():
    lib = pxb.load()
    assert lib.pxb_abi_version() == 5            # 5: pxb_reload_hooks, log-mode traces
    assert "#define PXB_ABI_VERSION 5" in open(HEADER).read()
    assert pxb.ABI_VERSION == 5
    # the test hooks are re-read on request (no GPU call), and restored
    import os
    with pxb.hooks(PXB_NO_EV="1", PXB_EV_BAIL_CAP="3"):
        assert os.environ["PXB_NO_EV"] == "1"
    assert "PXB_NO_EV" not in os.environ and "PXB_EV_BAIL_CAP" not in os.environ
    # no scratch on a device yet (no GPU here): zero counts, no HIP call
    out = (C.c_uint64 * 2)(7, 7)
    assert lib.pxb_handoff_counts(0, C.cast(out, C.c_void_p), 0) == 0 and list(out) == [0, 0]
    assert lib.pxb_handoff_counts(0, None, 0) == pxb.PXB_E_INVAL
    assert lib.pxb_handoff_counts(64, C.cast(out, C.c_void_p), 0) == pxb.PXB_E_INVAL
    assert lib.pxb_strerror(pxb.PXB_E_INVAL) == b"invalid argument"
    assert lib.pxb_canonical_bytes_nofault(5) == 1140


def test_invalid_config_rejected():
    lib = pxb.load()
    bad = pxb.Config(seed=1, n_proposers=4).to_c(0, 10)
    tot = (C.c_int64 * 16)()
    assert lib.pxb_run_device(C.byref(bad), None, None, None, C.cast(tot, C.c_void_p), None) == pxb.PXB_E_INVAL
    bad = pxb.Config(seed=1, delay_max=16).to_c(0, 10)
    assert lib.pxb_run_device(C.byref(bad), None, None, None, C.cast(tot, C.c_void_p), None) == pxb.PXB_E_INVAL


def test_trace_log_mode_validation():
    """pxb_trace_instance runs log mode (ABI 5) on the batch kernels' LG shape:
    a log-mode config passes validation (PXB_E_NODEV without a GPU, OK with
    one); delays above the LG shape's 8-step wheel, or a tick period of 0, are
    PXB_E_INVAL, checked before any device call (so on every host)."""
    import dataclasses
    import numpy as np
    lib = pxb.load()
    buf = np.zeros((16, pxb.TRACE_WORDS), dtype=np.uint32)
    n = C.c_uint32(0)
    res = np.zeros(4, dtype=np.uint32)

    def rc(cfg):
        c = cfg.to_c(0, 1)
        return lib.pxb_trace_instance(C.byref(c), 0, C.c_void_p(buf.ctypes.data), 16, C.byref(n),
                                      C.c_void_p(res.ctypes.data))
    for cfg in (pxb.LOG_CONFIG, pxb.LOG_FAULTY_CONFIG):
        assert rc(cfg) in (pxb.PXB_OK, pxb.PXB_E_NODEV)
    assert rc(dataclasses.replace(pxb.LOG_FAULTY_CONFIG, delay_max=9)) == pxb.PXB_E_INVAL
    assert rc(dataclasses.replace(pxb.LOG_FAULTY_CONFIG, tick_period=0)) == pxb.PXB_E_INVAL
    with pytest.raises(pxb.PaxosError, match="invalid argument"):
        pxb.trace_instance(dataclasses.replace(pxb.LOG_FAULTY_CONFIG, delay_max=12), 0, max_records=16)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pxb.PaxosError):
        pxb.run(pxb.CONFIGS[2], 0, 16)


def test_init_and_shutdown_without_gpu():
    """The context entry points fail cleanly without a device; shutdown with
    nothing allocated is a no-op, and may be repeated."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = pxb.load()
    assert lib.pxb_init(0) == pxb.PXB_E_NODEV
    assert lib.pxb_shutdown() == pxb.PXB_OK
    assert lib.pxb_shutdown() == pxb.PXB_OK
    pxb.stream_release(0, 0x1234)              # (a stream the library never saw: ignored)
    pxb.stream_release(-1, 0)


def test_multi_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = pxb.load()
    c = pxb.CONFIGS[3].to_c(0, 100)
    assert lib.pxb_run_multi(C.byref(c), 0, None, None, None, None) == pxb.PXB_E_NODEV


def test_run_device_checks_buffers_before_the_abi():
    """pxb.run_device hands raw addresses to pxb_run_device, so the Python
    mirror checks every device buffer first: host tensors, wrong element sizes
    and short buffers raise instead of letting a kernel write past them."""
    import torch
    cfg = pxb.CONFIGS[3]
    n = 100
    with pytest.raises(ValueError, match="CUDA"):
        pxb.run_device(cfg, 0, n, d_totals=torch.zeros(16, dtype=torch.int64))
    with pytest.raises(ValueError, match="required"):
        pxb.run_device(cfg, 0, n)

    class Fake:   # a stand-in for a device tensor (no GPU here)
        def __init__(self, numel, size=4, contiguous=True):
            self.is_cuda, self._n, self._s, self._c = True, numel, size, contiguous
            self.dtype = torch.int32 if size == 4 else torch.int64

        def element_size(self):
            return self._s

        def is_contiguous(self):
            return self._c

        def numel(self):
            return self._n

    with pytest.raises(ValueError, match="needed"):
        pxb.run_device(cfg, 0, n, d_results=Fake(4 * n - 1), d_totals=Fake(16, 8))
    with pytest.raises(ValueError, match="needed"):
        pxb.run_device(cfg, 0, n, d_digests=Fake(5 * n - 1), d_totals=Fake(16, 8))
    with pytest.raises(ValueError, match="integer"):
        pxb.run_device(cfg, 0, n, d_results=Fake(4 * n, 8), d_totals=Fake(16, 8))
    with pytest.raises(ValueError, match="integer"):
        pxb.run_device(cfg, 0, n, d_results=Fake(4 * n, 4, False), d_totals=Fake(16, 8))
    with pytest.raises(ValueError, match="needed"):
        pxb.run_device(cfg, 0, n, d_totals=Fake(15, 8))


def test_wire_device_entry_points_check_their_buffers():
    """The device wire calls take raw pointers: host tensors, wrong dtypes and
    short buffers are refused before anything reaches the C ABI."""
    import torch
    n = 4
    msgs = torch.zeros((n, 4), dtype=torch.int32)
    offs = torch.zeros(n + 1, dtype=torch.int64)
    byts = torch.zeros(n * pxb.WIRE_MAX_BYTES, dtype=torch.uint8)
    with pytest.raises(ValueError, match="CUDA"):
        pxb.wire_encode_device(msgs, pxb.WIRE_RESPONSE, offs, byts)
    with pytest.raises(ValueError, match="CUDA"):
        pxb.wire_decode_device(byts, offs, n, pxb.WIRE_RESPONSE, msgs)
    class _PosingAsDevice:                # a device-looking int32 buffer reaches the dtype check
        is_cuda = True
        dtype = torch.int32

        def is_contiguous(self):
            return True

        def numel(self):
            return 64
    with pytest.raises(ValueError, match="uint8"):
        pxb._check_bytes("d_bytes", _PosingAsDevice(), 1)

def test_trace_record_layout_matches_bindings():
    """pxb_trace_step as the Python mirror (pxb.TRACE_WORDS, word offsets in
    trace_instance) and the Haskell binding (PaxosBatch.traceInstance: 73
    words, digests from word 40, proposers from word 49, 8 words each) read it."""
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "paxos_batch.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(pxb_trace_step), offsetof(pxb_trace_step, acc),
         offsetof(pxb_trace_step, log_digest), offsetof(pxb_trace_step, prop), sizeof(pxb_trace_prop));
  return 0;
}'''
    tmp = "/tmp/pxb_trace_layout"
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), "-o", tmp, tmp + ".c"], check=True)
    size, acc, dig, prop, psize = (int(x) for x in subprocess.run([tmp], capture_output=True, text=True).stdout.split())
    assert (size, acc, dig, prop, psize) == (4 * pxb.TRACE_WORDS, 16, 160, 196, 32)
    hs = open(os.path.join(os.path.dirname(HEADER), "..", "cloud-haskell-paxos_amd", "hs", "PaxosBatch.hs")).read()
    assert "let nw = 73" in hs and "at (40 + a)" in hs and "let b = 49 + 8 * q" in hs and "let b = 4 + 4 * a" in hs
