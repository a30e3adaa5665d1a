"""Wire codec A/B (diagnostic): pxb_wire_encode_all over bench.wire_bench's 2^24
ServerResponse mix with the library PXB_LIB names (one process per library),
HIP events on the launch stream; no output check (tests/test_wire.py is the
check).  python tools/wire_ab.py [reps]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cloud-haskell-paxos_amd"))


def main():
    import numpy as np
    import torch
    import pxb
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = 1 << 24
    rng = np.random.default_rng(0)
    kind = rng.choice([0, 0, 1, 2], size=n).astype(np.uint32)
    msgs = np.zeros((n, 4), np.uint32)
    msgs[:, 0] = kind
    msgs[:, 1] = np.where(kind == 2, 0, rng.integers(1, 1 << 13, n))
    just = (kind == 0) & (rng.random(n) < 0.5)
    msgs[:, 2] = np.where(just, rng.integers(1, 1 << 13, n), 0)
    msgs[:, 3] = np.where(just, (rng.integers(1, 4, n) << 24) | rng.integers(1, 1 << 13, n), 0)
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    d_m = torch.from_numpy(msgs.view(np.int32)).to(dev)
    d_o = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_b = torch.zeros(n * pxb.WIRE_MAX_BYTES, dtype=torch.uint8, device=dev)
    with torch.cuda.stream(st):
        pxb.wire_encode_device(d_m, pxb.WIRE_RESPONSE, d_o, d_b, stream=st.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            pxb.wire_encode_device(d_m, pxb.WIRE_RESPONSE, d_o, d_b, stream=st.cuda_stream)
        e1.record(st)
        st.synchronize()
    print(json.dumps({"lib": os.path.basename(os.environ.get("PXB_LIB", "libpaxos_batch.so")),
                      "encode_ms": e0.elapsed_time(e1) / reps}), flush=True)


if __name__ == "__main__":
    main()
