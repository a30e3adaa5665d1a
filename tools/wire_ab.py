"""A/B timing of the wire codec across library variants (diagnostic).
    python tools/wire_ab.py lib1.so [lib2.so ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402
import bench  # noqa: E402
import pxb  # noqa: E402

for lib in sys.argv[1:]:
    pxb._lib = None
    pxb.load(os.path.join(ROOT, lib))
    st = torch.cuda.Stream()
    print(lib, json.dumps(bench.wire_bench(st, torch.device("cuda:0"))), flush=True)
