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


def msg_lost(seed, inst, dirn, p, a, k, loss_ppm):
    """SEMANTICS §4 message draw: link (dirn, p, a), seq k -> lost iff w0 < thr(loss)."""
    return int(w(seed, inst, k, (1 << 24) | (dirn << 16) | (p << 8) | a)[0] < R.prob_threshold(loss_ppm))


def params(seed, inst, c):
    """SEMANTICS §4 randomized parameters (PXB_CFG_RANDOMIZE): the draw and what it gives."""
    x = w(seed, inst, 0, 4 << 24)
    return {"w": list(x), "P": 1 + R.mulhi(x[0], c["n_proposers"]), "loss_ppm": R.mulhi(x[1], c["loss_ppm"] + 1),
            "delay_max": 1 + R.mulhi(x[2], c["delay_max"]), "crash_ppm": R.mulhi(x[3], c["crash_ppm"] + 1)}


def _link(key):
    src, dst = key.split("->")
    if src[0] == "p":
        return 0, int(src[1:]), int(dst[1:])
    return 1, int(dst[1:]), int(src[1:])


def case_draws(case):
    """The draws a case lists, recomputed: {'p0->a0': [d0, d1, ...] (delays), 'loss:p0->a0': [0, 1, ...]
    (lost flags), 'params': {...} (randomized), 'skew': ..., 'isolation': ...}."""
    c, inst = case["config"], case["instance"]
    out = {}
    loss = c["loss_ppm"]
    if c.get("randomize"):
        loss = params(c["seed"], inst, c)["loss_ppm"]
    for key, want in case["draws"].items():
        if key == "params":
            out[key] = params(c["seed"], inst, c)
        elif key.startswith("loss:"):
            dirn, p, a = _link(key[5:])
            out[key] = [msg_lost(c["seed"], inst, dirn, p, a, k, loss) for k in range(len(want))]
        elif key == "skew":
            out[key] = skews(c["seed"], inst, c["n_proposers"], c["skew_max"])
        elif key == "isolation":
            out[key] = [window(c["seed"], inst, a, c["crash_ppm"], c["crash_start_max"], c["crash_len_max"])
                        for a in range(c["n_acceptors"])]
        else:
            dirn, p, a = _link(key)
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

    # S4 / S5: per-link loss patterns at 5 % (every other message delivered)
    def pattern(seed, i, ppm, req_n, req_lost, rep_n, rep_lost):
        return all(msg_lost(seed, i, 0, 0, a, k, ppm) == ((a, k) in req_lost) for a in range(3) for k in range(req_n[a])) \
            and all(msg_lost(seed, i, 1, 0, a, k, ppm) == ((a, k) in rep_lost) for a in range(3) for k in range(rep_n[a]))
    s4 = 0x57E90004
    print("S4 first instance", next(i for i in range(10 ** 7) if pattern(s4, i, 50000, [9, 9, 9], {(2, 2)},
                                                                      [6, 6, 6], {(1, 2)})))
    s5 = 0x57E90005
    print("S5 first instance", next(i for i in range(10 ** 7) if pattern(s5, i, 50000, [6, 6, 6], {(2, 2), (2, 4)},
                                                                      [4, 4, 3], set())))
    # S6: the randomized draw gives P = 3, delay_max 1, loss > 0, and none of
    # the 51 messages of the run is lost
    s6 = 0x57E90006
    cfg6 = {"n_proposers": 3, "loss_ppm": 100000, "delay_max": 2, "crash_ppm": 0}
    req, rep = [3, 3, 3], [2, 3, 3]
    for i in range(10 ** 6):
        q = params(s6, i, cfg6)
        if q["P"] != 3 or q["delay_max"] != 1 or q["loss_ppm"] == 0:
            continue
        L = q["loss_ppm"]
        if not any(msg_lost(s6, i, 0, p, a, k, L) for p in range(3) for a in range(3) for k in range(req[p])) and \
                not any(msg_lost(s6, i, 1, p, a, k, L) for p in range(3) for a in range(3) for k in range(rep[p])):
            print("S6 first instance", i, q)
            break


if __name__ == "__main__":
    if sys.argv[1:] == ["search"]:
        search()
    else:
        kats = json.load(open(os.path.join(HERE, "kat_step_schedule.json")))
        for case in kats["cases"]:
            print(case["name"], case_draws(case))
