"""CPU oracle for the batched ticket-Paxos engine — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``libpaxos_batch.so``, HIP kernels) never calls it.

It is a line-by-line restatement, in plain Python, of the reference's
message handlers:

* acceptor  ``handleClientRequest``   /root/reference/src/Server.hs:54-78
* proposer  ``handleServerResponse``  /root/reference/src/Client.hs:128-189
            ``haveMajority``          /root/reference/src/Client.hs:191-194
            ``handleTick``            /root/reference/src/Client.hs:196-207
* ``MostRecentProposal`` monoid       /root/reference/src/Common.hs:57-68

plus two drivers:

* ``run_global_fifo``  — one global FIFO mailbox, messages handled in send
  order (the zero-delay special case used by the hand-derived KATs of
  SURVEY.md §8.0, KAT-1..KAT-6 and the stock ``app/Main.hs`` topology).
* ``run_instance``     — the canonical batched step schedule (docs/SEMANTICS.md),
  the contract the HIP kernel reproduces bit-exact.

Parity status: the reference is Haskell (GHC 8.4 / stack lts-12.18) and
cannot be built or run in this image (no ghc/stack/cabal, no network;
SURVEY.md §8c).  The restatement is pinned by the hand-derived KATs of
SURVEY.md §8.0 (tests/test_oracle.py) and the Random123 Philox4x32-10
known-answer vectors; it is NOT pinned by executions of the reference itself.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Deque, List, Optional, Sequence, Tuple

M32 = 0xFFFFFFFF

# --------------------------------------------------------------------------
# Philox4x32-10 (Salmon et al., SC'11; Random123 reference constants)
# --------------------------------------------------------------------------
PHILOX_M0 = 0xD2511F53
PHILOX_M1 = 0xCD9E8D57
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85


def philox4x32_10(ctr: Sequence[int], key: Sequence[int]) -> Tuple[int, int, int, int]:
    c0, c1, c2, c3 = (x & M32 for x in ctr)
    k0, k1 = key[0] & M32, key[1] & M32
    for _ in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = (p0 >> 32) & M32, p0 & M32
        hi1, lo1 = (p1 >> 32) & M32, p1 & M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + PHILOX_W0) & M32
        k1 = (k1 + PHILOX_W1) & M32
    return c0, c1, c2, c3


def mulhi(w: int, n: int) -> int:
    """floor(w * n / 2^32): maps a uniform u32 onto [0, n)."""
    return ((w & M32) * n) >> 32


def prob_threshold(ppm: int) -> int:
    """u64 threshold T with  (w < T)  <=>  w * 1e6 < ppm * 2^32  for u32 w."""
    return -((-ppm << 32) // 1_000_000)  # ceil(ppm * 2^32 / 1e6)


# Philox purposes (counter word 3, bits 31..24) — docs/SEMANTICS.md §4
PURPOSE_MSG = 1
PURPOSE_SKEW = 2
PURPOSE_CRASH = 3
PURPOSE_PARAMS = 4

# --------------------------------------------------------------------------
# Encodings (SURVEY.md §8.0 "Encodings")
# --------------------------------------------------------------------------
# Command  "c<clientId>.<t>"  (Client.hs:202-203)  ->  (clientId << 24) | t
NOTHING = 0  # val == 0 encodes `Nothing` (no real command has code 0)


def cmd_code(client_id: int, t: int) -> int:
    return ((client_id & 0xFF) << 24) | (t & 0xFFFFFF)


def cmd_str(code: int) -> str:
    return "c%d.%d" % (code >> 24, code & 0xFFFFFF)


# ClientRequest constructors  (Common.hs:41-45)
ASK, PROPOSE, EXECUTE = 0, 1, 2
# ServerResponse constructors (Common.hs:49-53)
R1OK, HAVE, R2S = 0, 1, 2

# payload bytes per message type, used by the canonical
# byte accounting of §8(d)
REQ_BYTES = {ASK: 8, PROPOSE: 12, EXECUTE: 8}
RSP_BYTES = {R1OK: 16, HAVE: 8, R2S: 4}

# round states (Client.hs:51-56)
IDLE, ROUND1, ROUND2 = 0, 1, 2

# result flags (SURVEY.md §8.0 "Per-instance outputs")
F_UNDECIDED = 1 << 0
F_STUCK = 1 << 1
F_PANIC = 1 << 2
F_LOG_DIVERGENCE = 1 << 3
F_STEP_CAP = 1 << 4
F_QUEUE_OVERFLOW = 1 << 5
F_TICKET_OVERFLOW = 1 << 6
F_LOG_TRUNC = 1 << 7

TICKET_LIMIT = 1 << 14      # tickets at/above this set F_TICKET_OVERFLOW (14-bit kernel fields)
QUEUE_DEPTH = 8             # per directed link (docs/SEMANTICS.md §3)
LOG_TRACK = 32              # log positions checked for divergence

FNV_BASIS = 0x811C9DC5
FNV_PRIME = 0x01000193


def fnv1a_u32(h: int, v: int) -> int:
    for i in range(4):
        h ^= (v >> (8 * i)) & 0xFF
        h = (h * FNV_PRIME) & M32
    return h


# --------------------------------------------------------------------------
# Acceptor  (Server.hs:24-31 state, :54-78 handlers)
# --------------------------------------------------------------------------
@dataclass
class Acceptor:
    t_max: int = 0          # _largestIssuedTicket   Server.hs:26
    t_store: int = 0        # _proposal :: Maybe Proposal  Server.hs:27
    val: int = NOTHING      #   (val == 0  <=>  Nothing)
    log: List[int] = field(default_factory=list)   # _executed  Server.hs:28
    dead: bool = False      # pattern-match failure at Server.hs:76 (Q6)


def acceptor_handle(acc: Acceptor, kind: int, ticket: int, val: int = NOTHING):
    """handleClientRequest (Server.hs:51-78).

    Returns the single reply ``(kind, a, b, c)`` or ``None``; sets
    ``acc.dead`` on the Q6 panic.  Reply encodings:
    Round1OK -> (R1OK, granted, t_store, val); HaveTicket -> (HAVE, t_max, 0, 0);
    Round2Success -> (R2S, 0, 0, 0).
    """
    if kind == ASK:                               # Server.hs:54
        if acc.t_max >= ticket:                   # Server.hs:56  (>=)
            return (HAVE, acc.t_max, 0, 0)        # Server.hs:58
        acc.t_max = ticket                        # Server.hs:60
        return (R1OK, ticket, acc.t_store, acc.val)   # Server.hs:61-62
    if kind == PROPOSE:                           # Server.hs:64
        if ticket == acc.t_max:                   # Server.hs:66  (equality)
            acc.t_store, acc.val = ticket, val    # Server.hs:68
            return (R2S, 0, 0, 0)                 # Server.hs:69
        return (HAVE, acc.t_max, 0, 0)            # Server.hs:71
    if kind == EXECUTE:                           # Server.hs:73
        if acc.t_max == ticket:                   # Server.hs:75
            if acc.val == NOTHING:                # Server.hs:76 `Just (_, c) <-` fails
                acc.dead = True                   #   lazy-RWS fail = bottom -> actor dies
                return None
            acc.log.append(acc.val)               # Server.hs:78  executed <>= [c]
            acc.t_store, acc.val = 0, NOTHING     # Server.hs:77  proposal .= Nothing
        return None
    raise ValueError(kind)


# --------------------------------------------------------------------------
# Proposer  (Client.hs:36-67 state, :125-207 handlers)
# --------------------------------------------------------------------------
@dataclass
class Proposer:
    client_id: int
    ticket: int = 0         # _ticket     Client.hs:60
    cmd: int = NOTHING      # _mCommand   Client.hs:61
    acks: int = 0           # _numAcks    Client.hs:62
    rs: int = IDLE          # _roundState Client.hs:63
    mr_t: int = 0           # Round1State._mostRecentProposal  Client.hs:36-41
    mr_v: int = NOTHING
    r2_t: int = 0           # Round2State._proposal            Client.hs:43-49
    r2_v: int = NOTHING
    pending: bool = False   # Round2State._originalCommandPending


def have_majority(acks: int, n_acceptors: int) -> bool:
    """haveMajority (Client.hs:191-194): numAcks > floor(N / 2)."""
    return acks > n_acceptors // 2


def most_recent(mr_t: int, mr_v: int, t: int, v: int) -> Tuple[int, int]:
    """``MostRecent (mr) <> MostRecent (t, v)``  (Common.hs:61-65).

    Nothing is the identity; for two Justs the LEFT (earlier) wins iff
    t1 >= t2 (Q4: ties keep the earlier-delivered proposal)."""
    if mr_v == NOTHING:
        return t, v
    if v == NOTHING:
        return mr_t, mr_v
    return (mr_t, mr_v) if mr_t >= t else (t, v)


def proposer_tick(pr: Proposer) -> List[Tuple[int, int, int]]:
    """handleTick (Client.hs:196-207). Returns the broadcast requests."""
    if pr.rs != IDLE:                             # Client.hs:199
        return []
    pr.ticket += 1                                # Client.hs:200  (<+= returns new)
    t = pr.ticket
    pr.cmd = cmd_code(pr.client_id, t)            # Client.hs:202-204
    pr.acks = 0                                   # Client.hs:205
    pr.rs, pr.mr_t, pr.mr_v = ROUND1, 0, NOTHING  # Client.hs:206
    return [(ASK, t, NOTHING)]                    # Client.hs:207


def proposer_handle(pr: Proposer, n_acceptors: int, kind: int, a: int = 0, b: int = 0,
                    c: int = NOTHING) -> List[Tuple[int, int, int]]:
    """handleServerResponse (Client.hs:125-189). The sender pid is ignored
    (Client.hs:128,142,172 bind sPid, never used — Q3).  Returns the list of
    broadcasts ``(kind, ticket, val)`` in tell order."""
    out: List[Tuple[int, int, int]] = []
    if kind == HAVE:                              # Client.hs:128
        u = a
        if pr.rs != IDLE and u >= pr.ticket:      # Client.hs:130-132
            pr.ticket = u + 1                     # Client.hs:134-135
            pr.acks = 0                           # Client.hs:137
            pr.rs, pr.mr_t, pr.mr_v = ROUND1, 0, NOTHING   # Client.hs:138
            out.append((ASK, pr.ticket, NOTHING))  # Client.hs:140
        return out
    if kind == R1OK:                              # Client.hs:142
        g, t_store, v = a, b, c
        if pr.rs == ROUND1 and pr.ticket == g:    # Client.hs:144-145
            pr.acks += 1                          # Client.hs:146
            mr_t, mr_v = most_recent(pr.mr_t, pr.mr_v, t_store, v)   # :147-151
            if not have_majority(pr.acks, n_acceptors):   # Client.hs:152-154
                pr.mr_t, pr.mr_v = mr_t, mr_v
            else:
                assert pr.cmd != NOTHING          # Client.hs:156 (Q11: unreachable)
                if mr_v == NOTHING:               # Client.hs:159-162
                    pr.r2_t, pr.r2_v, pr.pending = g, pr.cmd, False
                else:                             # Client.hs:163-167 (Q5)
                    pr.r2_t, pr.r2_v, pr.pending = g, mr_v, True
                pr.acks = 0                       # Client.hs:168
                pr.rs, pr.mr_t, pr.mr_v = ROUND2, 0, NOTHING   # Client.hs:169
                out.append((PROPOSE, pr.r2_t, pr.r2_v))        # Client.hs:170
        return out
    if kind == R2S:                               # Client.hs:172
        if pr.rs == ROUND2:                       # Client.hs:174 (no ticket: Q2)
            pr.acks += 1                          # Client.hs:175
            if have_majority(pr.acks, n_acceptors):   # Client.hs:176-177
                out.append((EXECUTE, pr.ticket, NOTHING))   # Client.hs:178
                if pr.pending:                    # Client.hs:179
                    pr.ticket += 1                # Client.hs:182 (<+= new value)
                    pr.acks = 0                   # Client.hs:183
                    pr.rs, pr.mr_t, pr.mr_v = ROUND1, 0, NOTHING   # :184
                    out.append((ASK, pr.ticket, NOTHING))          # :185
                else:
                    pr.cmd = NOTHING              # Client.hs:187
                    pr.acks = 0                   # Client.hs:188
                    pr.rs = IDLE                  # Client.hs:189
        return out
    raise ValueError(kind)


# --------------------------------------------------------------------------
# Driver 1: global FIFO (KAT schedule, SURVEY.md §8.0 "Known-answer traces")
# --------------------------------------------------------------------------
@dataclass
class FifoResult:
    acceptors: List[Acceptor]
    proposers: List[Proposer]
    decided_val: int
    decided_ticket: int
    rounds: int
    messages: int
    flags: int


def run_global_fifo(n_proposers: int, n_acceptors: int, drops: Sequence[Tuple] = (),
                    max_events: int = 100000) -> FifoResult:
    """One global FIFO queue; every process handles messages in send order.

    ``drops`` is a set of ``(src, dst, nth)`` triples: the nth (1-based)
    message sent on the directed link src->dst is lost at send time.  Process
    names: ``("c", i)`` proposer i (1-based, = clientId), ``("s", j)`` acceptor j
    (1-based).  Every proposer gets one Tick up front, c1's first
    (Client.hs:96-100 ticker; ordering per SURVEY.md KAT-2).  Messages to a
    dead acceptor are dropped (Cloud Haskell drop-to-dead).
    """
    accs = [Acceptor() for _ in range(n_acceptors)]
    props = [Proposer(client_id=i + 1) for i in range(n_proposers)]
    drops = set(drops)
    link_count = {}
    q: Deque = deque()
    for i in range(n_proposers):
        q.append((("c", i + 1), None, ("tick",)))
    messages = 0
    rounds = 0
    decided = None

    def send(src, dst, payload):
        nonlocal messages
        messages += 1
        k = link_count.get((src, dst), 0) + 1
        link_count[(src, dst)] = k
        if (src, dst, k) in drops:
            return
        q.append((dst, src, payload))

    events = 0
    while q:
        events += 1
        if events > max_events:
            raise RuntimeError("global FIFO did not quiesce")
        dst, src, payload = q.popleft()
        if dst[0] == "s":
            acc = accs[dst[1] - 1]
            if acc.dead:
                continue
            kind, ticket, val = payload
            rep = acceptor_handle(acc, kind, ticket, val)
            if rep is not None:
                send(dst, src, rep)
        else:
            pr = props[dst[1] - 1]
            if payload[0] == "tick":
                out = proposer_tick(pr)
            else:
                out = proposer_handle(pr, n_acceptors, *payload)
            for (kind, ticket, val) in out:
                if kind == ASK:
                    rounds += 1
                if kind == EXECUTE and decided is None:
                    decided = (pr.r2_v, ticket)
                for j in range(n_acceptors):       # sendToAllServers, list order
                    send(dst, ("s", j + 1), (kind, ticket, val))
    flags = 0
    if decided is None:
        flags |= F_UNDECIDED
    if any(p.rs != IDLE for p in props):
        flags |= F_STUCK
    if any(a.dead for a in accs):
        flags |= F_PANIC
    if _diverged([a.log for a in accs]):
        flags |= F_LOG_DIVERGENCE
    dv, dt = decided if decided else (NOTHING, 0)
    return FifoResult(accs, props, dv, dt, rounds, messages, flags)


def _diverged(logs: Sequence[Sequence[int]], limit: Optional[int] = None) -> bool:
    """True iff two logs differ at a common position (< limit if given)."""
    for i in range(len(logs)):
        for j in range(i + 1, len(logs)):
            n = min(len(logs[i]), len(logs[j]))
            if limit is not None:
                n = min(n, limit)
            if any(logs[i][k] != logs[j][k] for k in range(n)):
                return True
    return False


# --------------------------------------------------------------------------
# Driver 2: canonical batched step schedule (docs/SEMANTICS.md)
# --------------------------------------------------------------------------
@dataclass
class Config:
    seed: int
    n_proposers: int = 1
    n_acceptors: int = 5
    loss_ppm: int = 0
    delay_max: int = 1
    crash_ppm: int = 0
    crash_len_max: int = 1
    crash_start_max: int = 0
    skew_max: int = 0
    step_cap: int = 256
    randomize: bool = False   # config-5 fuzz: per-instance P/loss/delay/crash
    n_ticks: int = 1          # log mode when > 1 (docs/SEMANTICS.md §9)
    tick_period: int = 1      # steps between a proposer's Ticks


@dataclass
class InstanceParams:
    P: int
    loss_thr: int
    delay_max: int
    skew: List[int]
    iso: List[Tuple[int, int]]   # per acceptor isolation window [c0, c1)


def instance_params(cfg: Config, inst: int) -> InstanceParams:
    """docs/SEMANTICS.md §4: all per-instance draws."""
    key = (cfg.seed & M32, (cfg.seed >> 32) & M32)
    lo, hi = inst & M32, (inst >> 32) & M32
    P, loss_ppm, delay_max, crash_ppm = (cfg.n_proposers, cfg.loss_ppm,
                                         cfg.delay_max, cfg.crash_ppm)
    if cfg.randomize:
        w = philox4x32_10((lo, hi, 0, PURPOSE_PARAMS << 24), key)
        P = 1 + mulhi(w[0], cfg.n_proposers)
        loss_ppm = mulhi(w[1], cfg.loss_ppm + 1)
        delay_max = 1 + mulhi(w[2], cfg.delay_max)
        crash_ppm = mulhi(w[3], cfg.crash_ppm + 1)
    skew = [0] * P
    if cfg.skew_max > 0:
        w = philox4x32_10((lo, hi, 0, PURPOSE_SKEW << 24), key)
        skew = [mulhi(w[p], cfg.skew_max + 1) for p in range(P)]
    iso = [(0, 0)] * cfg.n_acceptors
    if crash_ppm > 0:
        thr = prob_threshold(crash_ppm)
        iso = []
        for a in range(cfg.n_acceptors):
            w = philox4x32_10((lo, hi, 0, (PURPOSE_CRASH << 24) | a), key)
            if w[0] < thr:
                c0 = mulhi(w[1], cfg.crash_start_max + 1)
                iso.append((c0, c0 + 1 + mulhi(w[2], cfg.crash_len_max)))
            else:
                iso.append((0, 0))
    return InstanceParams(P, prob_threshold(loss_ppm), delay_max, skew, iso)


@dataclass
class InstanceResult:
    decided_val: int
    decided_ticket: int
    rounds: int
    flags: int
    steps: int
    messages: int
    canon_bytes: int
    acceptors: List[Acceptor]
    proposers: List[Proposer]
    max_queue: int
    executes: int = 0       # Execute broadcasts (commands committed)

    def digest(self, a: int) -> int:
        acc = self.acceptors[a]
        h = FNV_BASIS
        for v in acc.log:
            h = fnv1a_u32(h, v)
        return fnv1a_u32(h, len(acc.log))

    def packed_flags(self) -> int:
        return (self.flags & 0xFF) | (min(self.steps, 0xFFFF) << 16)


class _Link:
    __slots__ = ("q", "seq", "last_due")

    def __init__(self):
        self.q: Deque = deque()
        self.seq = 0
        self.last_due = 0


def run_instance(cfg: Config, inst: int, queue_depth: int = QUEUE_DEPTH,
                 log_track: int = LOG_TRACK, ticket_limit: int = TICKET_LIMIT, trace=None) -> InstanceResult:
    """Run one instance under the canonical step schedule (docs/SEMANTICS.md).
    ``trace(s, accs, props, in_flight)``, if given, is called at the end of
    every step with the live state (the reference's per-message `say` dumps,
    Server.hs:85 / Client.hs:108, at step granularity)."""
    N = cfg.n_acceptors
    prm = instance_params(cfg, inst)
    P = prm.P
    key = (cfg.seed & M32, (cfg.seed >> 32) & M32)
    lo, hi = inst & M32, (inst >> 32) & M32
    accs = [Acceptor() for _ in range(N)]
    props = [Proposer(client_id=p + 1) for p in range(P)]
    req = [[_Link() for _ in range(N)] for _ in range(P)]   # p -> a
    rsp = [[_Link() for _ in range(P)] for _ in range(N)]   # a -> p
    flags = 0
    rounds = 0
    messages = 0
    canon = 0
    decided = None
    max_queue = 0
    canon_log = [NOTHING] * log_track
    # the ticker (Client.hs:96-100): one Tick at skew_p (single decree) or
    # n_ticks Ticks tick_period steps apart (log mode, docs/SEMANTICS.md §9)
    n_ticks = max(1, cfg.n_ticks)
    period = cfg.tick_period if n_ticks > 1 else 1
    last_tick = max(prm.skew) + (n_ticks - 1) * period
    executes = 0
    faulty = prm.loss_thr > 0 or prm.delay_max > 1

    def send(link: _Link, s: int, dirn: int, p: int, a: int, msg):
        nonlocal messages, flags, max_queue
        messages += 1
        k = link.seq
        link.seq += 1
        d = 1
        if faulty:
            w = philox4x32_10((lo, hi, k, (PURPOSE_MSG << 24) | (dirn << 16) | (p << 8) | a), key)
            if w[0] < prm.loss_thr:
                return
            d = 1 + mulhi(w[1], prm.delay_max)
        if len(link.q) >= queue_depth:
            flags |= F_QUEUE_OVERFLOW
            return
        due = max(s + d, link.last_due)
        link.last_due = due
        link.q.append((due, msg))
        max_queue = max(max_queue, len(link.q))

    def bcast(p: int, s: int, out):
        nonlocal rounds, decided, executes
        for (kind, ticket, val) in out:
            if kind == ASK:
                rounds += 1
            if kind == EXECUTE:
                executes += 1
            if kind == EXECUTE and decided is None:
                decided = (props[p].r2_v, ticket)
            for a in range(N):
                send(req[p][a], s, 0, p, a, (kind, ticket, val))

    steps = 0
    for s in range(cfg.step_cap):
        steps = s + 1
        # -- acceptor phase: inbox ordered by (proposer index, link seq)
        for a in range(N):
            acc = accs[a]
            c0, c1 = prm.iso[a]
            isolated = c0 <= s < c1
            for p in range(P):
                link = req[p][a]
                while link.q and link.q[0][0] <= s:
                    _, (kind, ticket, val) = link.q.popleft()
                    if acc.dead or isolated:
                        canon += REQ_BYTES[kind]          # written, discarded
                        continue
                    canon += 2 * REQ_BYTES[kind] + 32
                    before = len(acc.log)
                    rep = acceptor_handle(acc, kind, ticket, val)
                    if acc.dead:
                        flags |= F_PANIC
                    if len(acc.log) != before:
                        pos = before
                        if pos < log_track:
                            if canon_log[pos] == NOTHING:
                                canon_log[pos] = acc.log[-1]
                            elif canon_log[pos] != acc.log[-1]:
                                flags |= F_LOG_DIVERGENCE
                        else:
                            flags |= F_LOG_TRUNC
                    if rep is not None:
                        send(rsp[a][p], s, 1, p, a, rep)
        # -- proposer phase: tick, then inbox ordered by (acceptor index, link seq)
        for p in range(P):
            pr = props[p]
            active = False
            since = s - prm.skew[p]
            if since >= 0 and since % period == 0 and since // period < n_ticks:
                active = True
                bcast(p, s, proposer_tick(pr))
            for a in range(N):
                link = rsp[a][p]
                while link.q and link.q[0][0] <= s:
                    _, (kind, x, y, z) = link.q.popleft()
                    active = True
                    canon += 2 * RSP_BYTES[kind]
                    bcast(p, s, proposer_handle(pr, N, kind, x, y, z))
            if active:
                canon += 48
            if pr.ticket >= ticket_limit:
                flags |= F_TICKET_OVERFLOW
        # -- quiescence
        in_flight = any(l.q for row in req for l in row) or any(l.q for row in rsp for l in row)
        if trace is not None:
            trace(s, accs, props, sum(len(l.q) for row in req for l in row) +
                  sum(len(l.q) for row in rsp for l in row))
        if not in_flight and s >= last_tick:
            break
    else:
        flags |= F_STEP_CAP
    if decided is None:
        flags |= F_UNDECIDED
    if not (flags & F_STEP_CAP) and any(p.rs != IDLE for p in props):
        flags |= F_STUCK
    canon += 16 + 4 * N
    dv, dt = decided if decided else (NOTHING, 0)
    return InstanceResult(dv, dt, rounds, flags, steps, messages, canon, accs, props, max_queue,
                          executes)


def run_batch(cfg: Config, first: int, count: int, **kw) -> List[InstanceResult]:
    return [run_instance(cfg, first + i, **kw) for i in range(count)]


# Named configurations (BASELINE.json configs / SURVEY.md §8(d))
def config(n: int) -> Config:
    if n == 1:
        return Config(seed=0x5EED0001, n_proposers=1, n_acceptors=3)
    if n == 2:
        return Config(seed=0x5EED0002, n_proposers=1, n_acceptors=5)
    if n == 3:
        return Config(seed=0x5EED0003, n_proposers=2, n_acceptors=5, loss_ppm=100000,
                      delay_max=4, skew_max=3, step_cap=256)
    if n == 4:
        return Config(seed=0x5EED0004, n_proposers=2, n_acceptors=7, delay_max=4,
                      crash_ppm=200000, crash_len_max=16, crash_start_max=8, step_cap=256)
    if n == 5:
        return Config(seed=0x5EED0005, n_proposers=3, n_acceptors=9, loss_ppm=300000,
                      delay_max=8, crash_ppm=200000, crash_len_max=16, crash_start_max=16,
                      skew_max=3, step_cap=512, randomize=True)
    if n == 6:   # log mode (docs/SEMANTICS.md §9): stock Main.hs topology, ticker running
        return Config(seed=0x5EED0006, n_proposers=2, n_acceptors=2, step_cap=1024,
                      n_ticks=16, tick_period=8)
    raise ValueError(n)
