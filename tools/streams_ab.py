"""A/B of bench.py's step streams for one workload (diagnostic; never the bench
number): python tools/streams_ab.py <config> <log2 n> <steps> <streams,streams,...>
Runs bench.run_workload over a GpuLeg with each stream count in turn (the
process's stream pool is shared, as in bench.py) and prints instances/s.
Set GPU_MAX_HW_QUEUES in the environment to vary the hardware queues."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cloud-haskell-paxos_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import pxb  # noqa: E402


def main():
    c, lg, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    cfg = pxb.LOG_FAULTY_CONFIG if c == "7" else pxb.CONFIGS[int(c)]
    n = 1 << lg
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.Stream(dev)
    for ns in [int(x) for x in sys.argv[4].split(",")]:
        leg = bench.GpuLeg(cfg, n, 0, 1, stream, dev, streams=ns)
        es, ek, cnt = bench.run_workload(leg, n, steps, 1, 1)
        print(json.dumps({"config": c, "n": n, "steps": steps, "streams": ns,
                          "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                          "instances_per_s": cnt["instances"] / es, "kernel_ms": ek}), flush=True)
        del leg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
