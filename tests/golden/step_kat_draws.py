"""The schedule inputs of the step-schedule known-answer traces
(tests/golden/kat_step_schedule.json): Philox4x32-10 draws (the
implementation pinned by the three Random123 vectors, tests/test_oracle.py)
for a case's links, Tick skews and isolation windows, and the search that
picked each (seed, instance).  The traces themselves are derived by hand
from the handler tables and docs/SEMANTICS.md §4-6; nothing here runs the
schedule.

    python tests/golden/step_kat_draws.py          # print every case's draws
    python tests/golden/step_kat_draws.py search   # re-run the searches"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import paxos_ref as R  # noqa: E402  (Philox, mulhi and thresholds only)

M32 = 0xFFFFFFFF


def w(seed, inst, c2, c3):
    return R.philox4x32_10((inst & M32, (inst >> 32) & M32, c2, c3), (seed & M32, (seed >> 32) & M32))


def msg_delay(seed, inst, dirn, p, a, k, delay_max):
    """SEMANTICS §4 message draw: link (dirn, p, a), seq k -> delay (no loss here)."""
    return 1 + R.mulhi(w(seed, inst, k, (1 << 24) | (dirn << 16) | (p << 8) | a)[1], delay_max)


def window(seed, inst, a, ppm, start_max, len_max):
    x = w(seed, inst, 0, (3 << 24) | a)
    if x[0] < R.prob_threshold(ppm):
        c0 = R.mulhi(x[1], start_max + 1)
        return [c0, c0 + 1 + R.mulhi(x[2], len_max)]
    return None


def skews(seed, inst, P, skew_max):
    x = w(seed, inst, 0, 2 << 24)
    return [R.mulhi(x[p], skew_max + 1) for p in range(P)]


def case_draws(case):
    """The draws a case lists, recomputed: {'p0->a0': [d0, d1, ...], 'a0->p0': ..., 'skew': ..., 'isolation': ...}."""
    c, inst = case["config"], case["instance"]
    out = {}
    for key, want in case["draws"].items():
        if key == "skew":
            out[key] = skews(c["seed"], inst, c["n_proposers"], c["skew_max"])
        elif key == "isolation":
            out[key] = [window(c["seed"], inst, a, c["crash_ppm"], c["crash_start_max"], c["crash_len_max"])
                        for a in range(c["n_acceptors"])]
        else:
            src, dst = key.split("->")
            if src[0] == "p":
                dirn, p, a = 0, int(src[1:]), int(dst[1:])
            else:
                dirn, p, a = 1, int(dst[1:]), int(src[1:])
            out[key] = [msg_delay(c["seed"], inst, dirn, p, a, k, c["delay_max"]) for k in range(len(want))]
    return out


def search():
    """The searches that picked the instances (first hits)."""
    D = msg_delay
    s1 = 0x57E90001
    hit = next(i for i in range(10 ** 6) if (D(s1, i, 0, 0, 0, 0, 4), D(s1, i, 0, 0, 1, 0, 4), D(s1, i, 0, 0, 2, 0, 4),
                                             D(s1, i, 1, 0, 1, 0, 4), D(s1, i, 1, 0, 2, 0, 4), D(s1, i, 0, 0, 0, 1, 4))
               == (3, 1, 1, 1, 1, 1))
    print("S1 first instance", hit)
    s2 = 0x57E90002
    hit = [i for i in range(200) if [window(s2, i, a, 500000, 7, 1) for a in range(3)] == [None, None, [3, 4]]]
    print("S2 instances", hit)
    s3 = 0x57E90003
    hit = next(i for i in range(10 ** 6) if skews(s3, i, 2, 1) == [1, 0]
               and [D(s3, i, 0, 1, a, 0, 2) for a in range(3)] == [1, 2, 2]
               and [D(s3, i, 0, 0, a, 0, 2) for a in range(3)] == [1, 1, 1]
               and [D(s3, i, 1, 0, a, 0, 2) for a in range(3)] == [1, 1, 1])
    print("S3 first instance", hit)


if __name__ == "__main__":
    if sys.argv[1:] == ["search"]:
        search()
    else:
        kats = json.load(open(os.path.join(HERE, "kat_step_schedule.json")))
        for case in kats["cases"]:
            print(case["name"], case_draws(case))
