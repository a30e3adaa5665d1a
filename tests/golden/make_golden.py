"""Generate the golden fixtures under tests/golden/ from the pure-Python
oracle (oracle/paxos_ref.py).  The reference (Haskell) cannot run here, so
these vectors pin the C oracle and the GPU to the Python restatement, which
is itself pinned by SURVEY.md §8.0's hand-derived KATs (tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import paxos_ref as R  # noqa: E402

# (config, first_instance, count): small enough for pure Python in seconds
CASES = [(1, 0, 64), (2, 0, 64), (3, 0, 400), (3, (1 << 32) - 50, 100), (4, 0, 200), (5, 0, 300),
         (6, 0, 200)]


def main():
    for (c, first, n) in CASES:
        cfg = R.config(c)
        res = np.zeros((n, 4), np.uint32)
        dig = np.zeros((n, cfg.n_acceptors), np.uint32)
        acc = np.zeros((n, cfg.n_acceptors, 4), np.uint32)
        canon = 0
        for i in range(n):
            r = R.run_instance(cfg, first + i)
            res[i] = [r.decided_val, r.decided_ticket, r.rounds, r.packed_flags()]
            dig[i] = [r.digest(a) for a in range(cfg.n_acceptors)]
            acc[i] = [[x.t_max, x.t_store, x.val, len(x.log) | (int(x.dead) << 31)] for x in r.acceptors]
            canon += r.canon_bytes
        name = os.path.join(HERE, "cfg%d_first%d_n%d.npz" % (c, first, n))
        np.savez_compressed(name, results=res, digests=dig, acceptors=acc,
                            canon_bytes=np.array([canon], np.uint64),
                            meta=np.array([c, first, n], np.uint64))
        print("wrote", os.path.basename(name))
    kats = {}
    cases = {
        "KAT-1": (1, 3, []), "KAT-2": (2, 3, []), "Main.hs": (2, 2, []),
        "KAT-3": (1, 3, [(("c", 1), ("s", 3), 2)]),
        "KAT-4": (1, 3, [(("c", 1), ("s", 2), 1), (("c", 1), ("s", 3), 1)]),
        "KAT-5": (1, 3, [(("c", 1), ("s", 3), 3)]),
        "KAT-6": (2, 3, [(("s", 3), ("c", 1), 1)]),
    }
    for name, (P, N, drops) in cases.items():
        r = R.run_global_fifo(P, N, drops)
        kats[name] = {
            "P": P, "N": N, "drops": drops, "decided": R.cmd_str(r.decided_val) if r.decided_val else None,
            "decided_ticket": r.decided_ticket, "rounds": r.rounds, "messages": r.messages, "flags": r.flags,
            "logs": [[R.cmd_str(v) for v in a.log] for a in r.acceptors],
            "t_max": [a.t_max for a in r.acceptors],
            "prop": [R.cmd_str(a.val) if a.val else None for a in r.acceptors],
        }
    with open(os.path.join(HERE, "kat_global_fifo.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("wrote kat_global_fifo.json")


if __name__ == "__main__":
    main()
