"""The diagnostic builds of the library (-DPXB_WAVE_TIMES: per-wave timelines,
tools/build_wt.sh; -DPXB_STAMPS: per-section cycle stamps) are code no
production run compiles.  Round 4's GPU fault came from one of them (the
general kernel stored to a null timeline buffer behind the per-lane kernel,
32ad52a), so the CPU suite at least compiles them for gfx950 (host and device
semantics, every instantiation of the units that carry the switches), so that
the diagnostic paths cannot rot unseen.  The null-buffer guards they rely on
are asserted on the source."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cloud-haskell-paxos_amd", "csrc")
UNITS = [("paxos_batch.hip", []), ("paxos_ev.hip", ["-DPXB_EV_P=2"]),
         ("paxos_inst.hip", ["-DPXB_INST_P=2", "-DPXB_INST_LOGM=0"])]


@pytest.mark.parametrize("flag", ["PXB_WAVE_TIMES", "PXB_STAMPS"])
@pytest.mark.parametrize("unit,defs", UNITS, ids=[u for u, _ in UNITS])
def test_diagnostic_build_compiles(flag, unit, defs):
    p = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only",
                        "-D" + flag, *defs, os.path.join(CSRC, unit)],
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]


def test_diagnostic_stores_are_guarded():
    """Every kernel that stores a timeline or stamp does so only through a
    non-null buffer pointer (the launch leaves it null where no timeline is
    wanted: the second launch of a two-stage routing, the general kernel)."""
    for f in ("paxos_ev_kernel.h", "paxos_kernel.h"):
        src = open(os.path.join(CSRC, f)).read()
        blocks = re.findall(r"#ifdef PXB_WAVE_TIMES(.*?)#endif", src, re.S)
        stores = [b for b in blocks if "dbg[" in b]
        assert stores, f
        for b in stores:
            assert re.search(r"if \(kp\.dbg", b), (f, b[:200])
