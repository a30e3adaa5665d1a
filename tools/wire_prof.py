"""Wire codec kernels under rocprofv3 (diagnostic): encode / decode of 2^24
ServerResponse records as in bench.py's wire_bench, a few repetitions each.
    rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/wire_prof.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cloud-haskell-paxos_amd"))


def main():
    import torch
    import bench
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    r = bench.wire_bench(st, dev)
    print(r)


if __name__ == "__main__":
    main()
