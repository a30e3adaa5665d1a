#!/usr/bin/env python3
"""Per-section instruction budget of a per-lane kernel instantiation.

Compiles one paxos_ev_kernel<...> instantiation for gfx950 twice from the
repo headers (assembly, for the basic blocks and loop depths; a device object
with line tables, for the inline stacks), symbolizes every instruction of the
kernel with llvm-symbolizer --inlining, and attributes it to the EvLane
section it was inlined from (prop_op, broadcast, copy_send, acc_op,
send_first, end_op, enter, finish, kernel driver), split by instruction
class (VALU / SALU / LDS / other) and by helper (philox draw, one-hot
selects).  Prints a table per basic block and a per-section total over the
blocks of the iteration path.

  python3 tools/isa_budget.py "2, 7, 4, true, false, false" [extra hipcc flags]

(llvm-symbolizer, clang-offload-bundler and llvm-objdump from /opt/rocm/lib/llvm/bin.)
"""
from __future__ import annotations

import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
SECTIONS = ["prop_op", "broadcast", "copy_send", "copy_ctr", "acc_ready_mask", "acc_op", "send_first",
            "end_op", "enter", "finish", "init", "flush", "step"]
HELPERS = {"philox_rk": "philox", "philox_round": "philox", "mulhi_n": "mulhi",
           "get_from": "select", "set_from": "select", "bfi": "select", "lane_mask": "select",
           "get": "select", "put": "select", "fnv_u32": "fnv"}


def klass(op: str) -> str:
    if op.startswith("v_"):
        return "V"
    if op.startswith("s_"):
        return "S"
    if op.startswith("ds_"):
        return "DS"
    return "M"


def main() -> None:
    targs = sys.argv[1] if len(sys.argv) > 1 else "2, 7, 4, true, false, false"
    extra = sys.argv[2:]
    flags_extra = [a for a in extra if not a.startswith("--lines")]
    if "--lines" in extra:
        k = extra.index("--lines")
        flags_extra = extra[:k] + extra[k + 3:]
    tmp = tempfile.mkdtemp(prefix="isa_budget_")
    src = os.path.join(tmp, "k.hip")
    with open(src, "w") as f:
        f.write('#include "%s/cloud-haskell-paxos_amd/csrc/paxos_ev_kernel.h"\n'
                "namespace pxb { namespace ev {\n"
                "template __global__ void paxos_ev_kernel<%s>(EvKParams);\n}}\n" % (ROOT, targs))
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only", "-gline-tables-only",
             *g.EV_FLAGS, *flags_extra]
    asm = os.path.join(tmp, "k.s")
    obj = os.path.join(tmp, "k.o")
    subprocess.run([g.HIPCC, *flags, "-S", "-o", asm, src], check=True, stderr=subprocess.DEVNULL)
    subprocess.run([g.HIPCC, *flags, "-c", "-o", obj, src], check=True, stderr=subprocess.DEVNULL)
    elf = os.path.join(tmp, "k.elf")
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + obj,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + elf], check=True)

    # ---- blocks from the assembly ----
    blocks = []          # [label, depth, [mnemonics]]
    cur = None
    in_kernel = False
    for line in open(asm):
        if re.match(r"^_ZN3pxb2ev15paxos_ev_kernel\S*:", line):
            in_kernel = True
            cur = ["entry", 0, []]
            blocks.append(cur)
            continue
        if not in_kernel:
            continue
        if line.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?(.*)$", line)
        if m:
            d = re.search(r"Depth=(\d+)", m.group(2))
            cur = [m.group(1).replace("; %bb.", "bb."), int(d.group(1)) if d else 0, []]
            blocks.append(cur)
            continue
        t = line.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        cur[2].append(t.split()[0])
    nasm = sum(len(b[2]) for b in blocks)
    res = [l.strip("; \n") for l in open(asm) if re.match(r"^\s*; (NumVgprs|NumAgprs|TotalNumVgprs|NumSgprs|ScratchSize|Occupancy):", l)]
    print("resources: " + ", ".join(res[:6]))

    # ---- instruction addresses from the object ----
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", elf],
                         check=True, capture_output=True, text=True).stdout
    insts = []
    on = False
    for line in dis.split("\n"):
        if re.match(r"^[0-9a-f]+ <_ZN3pxb2ev15paxos_ev_kernel", line):
            on = True
            continue
        if on and re.match(r"^[0-9a-f]+ <", line):
            break
        m = re.match(r"^\s+(\S+).*// ([0-9A-F]+):", line)
        if on and m:
            insts.append((int(m.group(2), 16), m.group(1)))
    # (s_code_end padding after the kernel)
    while insts and insts[-1][1] in ("s_code_end", "s_nop"):
        insts.pop()
    if len(insts) < nasm:
        raise SystemExit("instruction count mismatch: asm %d, object %d" % (nasm, len(insts)))
    insts = insts[:nasm]

    # ---- inline stacks ----
    sym = subprocess.run([os.path.join(LLVM, "llvm-symbolizer"), "--inlining", "--functions=short",
                          "--obj=" + elf], input="\n".join(hex(a) for a, _ in insts) + "\n",
                         capture_output=True, text=True, check=True).stdout
    chunks = sym.strip().split("\n\n")
    stacks = [[ln for ln in chunk.split("\n")[0::2] if ln] for chunk in chunks]
    locs = [[ln for ln in chunk.split("\n")[1::2] if ln] for chunk in chunks]
    if len(stacks) != len(insts):
        raise SystemExit("symbolizer output mismatch")

    def attribute(st):
        sec = "driver"
        for fn in reversed(st):                       # outermost first
            base = fn.split("<")[0]
            if base in SECTIONS:
                sec = base if base not in ("enter", "finish", "broadcast") else base
        helper = "-"
        for fn in st:                                 # innermost first
            base = fn.split("<")[0]
            if base in HELPERS:
                helper = HELPERS[base]
                break
        return sec, helper

    # --lines FIRST LAST: per source line of paxos_ev.h (innermost frame in it),
    # VALU/SALU over the blocks FIRST..LAST (labels as printed)
    lines_mode = None
    if "--lines" in extra:
        k = extra.index("--lines")
        lines_mode = (extra[k + 1], extra[k + 2])
    i = 0
    per_block = []
    per_line = collections.Counter()
    in_range = False
    for lab, depth, ops in blocks:
        c = collections.Counter()
        if lines_mode and lab == lines_mode[0]:
            in_range = True
        for op in ops:
            if in_range:
                ln = next((l for l in locs[i] if "paxos_ev.h" in l or "paxos_ev_kernel.h" in l), "?")
                ln = ln.split("/")[-1].rsplit(":", 1)[0]
                per_line[(ln, klass(op))] += 1
            a_op = insts[i][1]
            if a_op != op and not (a_op.split("_e")[0] == op.split("_e")[0]):
                pass                                   # (encoding suffixes may differ)
            sec, helper = attribute(stacks[i])
            c[(sec, helper, klass(op))] += 1
            i += 1
        per_block.append((lab, depth, len(ops), c))
        if lines_mode and lab == lines_mode[1]:
            in_range = False

    if lines_mode:
        keys = sorted({k for k, _ in per_line}, key=lambda x: (x.split(":")[0], int(x.split(":")[1]) if x != "?" else 0))
        for k in keys:
            print("%-26s V %3d  S %3d  DS %2d" % (k, per_line[(k, "V")], per_line[(k, "S")], per_line[(k, "DS")]))
        return
    secs = SECTIONS + ["driver"]
    print("kernel paxos_ev_kernel<%s> %s" % (targs, " ".join(extra)))
    print("%-10s %3s %5s  " % ("block", "dep", "insts") + " ".join("%14s" % s[:14] for s in secs))
    for lab, depth, n, c in per_block:
        if n == 0:
            continue
        row = []
        for s in secs:
            v = sum(k for (sc, _, kl), k in c.items() if sc == s and kl == "V")
            sa = sum(k for (sc, _, kl), k in c.items() if sc == s and kl == "S")
            row.append("%6s" % ("" if v + sa == 0 else "%d/%d" % (v, sa)))
        print("%-10s %3d %5d  " % (lab, depth, n) + " ".join("%14s" % r for r in row))
    print("\n(cells: VALU/SALU)")
    # (the iteration's loop depth: 1, or 2 since the step loop nests in the
    # refill loop; BUDGET_DEPTH overrides)
    loop_depth = int(os.environ.get("BUDGET_DEPTH", "2" if any(d == 2 and "prop_op" in str(c) for _, d, _, c in per_block) else "1"))
    print("\nper section over all depth-%d blocks (static), by helper:" % loop_depth)
    tot = collections.Counter()
    for lab, depth, n, c in per_block:
        if depth == loop_depth:
            tot.update(c)
    for s in secs:
        items = {(h, kl): k for (sc, h, kl), k in tot.items() if sc == s}
        if not items:
            continue
        v = sum(k for (h, kl), k in items.items() if kl == "V")
        sa = sum(k for (h, kl), k in items.items() if kl == "S")
        ds = sum(k for (h, kl), k in items.items() if kl == "DS")
        hs = ", ".join("%s %d" % (h, sum(k for (hh, kl), k in items.items() if hh == h and kl == "V"))
                       for h in sorted({h for h, _ in items}) if h != "-")
        print("  %-15s V %4d  S %4d  DS %3d   (VALU in helpers: %s)" % (s, v, sa, ds, hs or "none"))


if __name__ == "__main__":
    main()
