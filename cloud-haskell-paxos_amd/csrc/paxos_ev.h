// paxos_ev.h — the per-lane ("event") batched ticket-Paxos kernel for faulty
// single-decree schedules (loss, delay, crash windows, duelling, fuzzing).
//
// One lane runs one whole instance: its N acceptors (Server.hs:44-89), its P
// proposers (Client.hs:85-207) and its 2·P·N directed links.  The reference's
// actors are replaced by a per-lane state machine that, every wave iteration,
// performs ONE micro-step of its own instance in canonical order
// (docs/SEMANTICS.md §6):
//
//   ACC   one request handled by one acceptor (handleClientRequest,
//         Server.hs:51-78) + its reply sent on link a -> p;
//   PROP  one Tick (handleTick, Client.hs:196-207) or one response folded
//         by one proposer (handleServerResponse, Client.hs:125-189), and the
//         next copy of a pending broadcast (sendToAllServers,
//         Client.hs:122-123) sent on link p -> a;
//   ADV   end of step: quiescence / step cap (the role of Main.hs:49-53),
//         then the next step's due links from a timing wheel.
//
// Lanes are independent (instances share nothing: Main.hs:41-45), so a wave
// never waits on its slowest instance: a lane whose instance ends writes its
// outputs and takes the next instance from the work queue.  Every lane sends
// at most one message per micro-step, so the wave issues one Philox4x32-10
// draw per iteration for all 64 lanes.
//
// Per-lane state (LDS words are lane-interleaved, [word][lane]: every access
// is bank-conflict free):
//   registers  proposer states, pending-broadcast queue, link-free masks,
//              counters;
//   LDS        request-link FIFOs (4 x {broadcast slot, due} per link, the
//              payload lives once per broadcast in a per-proposer ring),
//              response-link FIFOs (indices into a per-lane pool of response
//              words), the reply sequence numbers, acceptor states and
//              digests, isolation windows, and a timing wheel of per-step
//              due-link masks.
//
// The semantic queue depth stays PXB_QUEUE_DEPTH = 8; the physical FIFOs hold
// 4 (and the pool POOL responses).  An instance that would need more is
// "bailed": its id goes to a list that the general kernel (paxos_kernel.h)
// re-runs from scratch, so results stay exact for every schedule.  Measured
// on the BASELINE configs (tools/ study): config 4 never
// bails, config 5 bails ~0.3 % of instances.
//
// This file is plain C++ over a memory accessor, so the same code runs on the
// device (LDS accessor) and in the host unit test (tests/test_ev_host.py),
// which checks it against the CPU oracle instance by instance.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/paxos_batch.h"
#include "paxos_device.h"

namespace pxb {
namespace ev {

constexpr uint32_t CPHYS = 4;     // physical FIFO slots per link
constexpr uint32_t BR = 8;        // broadcast ring slots per proposer
constexpr uint32_t PQ_CAP = 4;    // pending broadcasts per lane
constexpr uint32_t MAX_STEP_CAP = 4095;   // 12-bit tickets (tickets <= step_cap, SEMANTICS §6)
static_assert(MAX_STEP_CAP < PXB_TICKET_LIMIT, "EV tickets never reach the overflow limit");

// lane modes
constexpr uint32_t M_IDLE = 0, M_ACC = 1, M_PROP = 2;

template <int PM_, int N_, int POOL_, int W_>
struct Shape {
  static constexpr int PM = PM_, N = N_, POOL = POOL_, W = W_;
  static constexpr int NL = PM * N;                  // links per direction
  static constexpr int IB = POOL <= 32 ? 5 : 6;      // pool index bits
  static constexpr int WW = (NL <= 16) ? 1 : 2;      // wheel words per slot
  static constexpr int PSH = (WW == 1) ? 16 : 0;     // proposer-link bit offset in the wheel word
  // LDS word offsets
  static constexpr int REQM = 0;                     // NL: request links, index a*PM + p
  static constexpr int RSPM = REQM + NL;             // NL: response links, index p*N + a
  static constexpr int RSEQ = RSPM + NL;             // NL halfwords: reply seq, index a*PM + p
  static constexpr int POOLW = RSEQ + (NL + 1) / 2;  // POOL response words
  static constexpr int BRING = POOLW + POOL;         // PM*BR halfwords: broadcast payloads
  static constexpr int ACCW = BRING + PM * BR / 2;   // N acceptor words
  static constexpr int ACCD = ACCW + N;              // N digests
  static constexpr int ACCC = ACCD + N;              // N isolation windows
  static constexpr int WHEEL = ACCC + N;             // W * WW due-link masks
  static constexpr int WORDS = WHEEL + W * WW;
  static_assert(W == 8 || W == 16, "wheel of 8 or 16 steps");
  static_assert(NL <= 32, "link masks are 32-bit");
  static_assert(4 * IB + 7 <= 32, "response-link word");
};

// Layouts (docs/SEMANTICS.md §2 encodings; tickets < 2^12):
//   request-link word   entry i (7 bits at 7i): broadcast slot [2:0] | due&15 [6:3];  len [30:28]
//   response-link word  pool index i (IB bits at IB*i); len [4IB+2:4IB]; last due&15 [4IB+6:4IB+3]
//   response word       x [11:0] | y [23:12] | z [25:24] | due&15 [29:26] | kind [31:30]
//   broadcast payload   x [11:0] | z [13:12] | kind [15:14]
//   acceptor word       t_max [11:0] | t_store [23:12] | val [25:24] | dead [26] | log_len [31:27]
//   window              c0 [15:0] | c1 [31:16]  (clamped to 4096: steps are < 4095)

// Per-launch parameters shared by the device kernel and the host test.
struct EvParams {
  uint64_t first_instance;
  uint32_t k0, k1;
  uint32_t cfg;                       // CFG_* bits (paxos_kernel.h)
  uint32_t n_prop, delay_max;
  uint32_t loss_m1, crash_m1;
  uint32_t loss_ppm, crash_ppm;
  uint32_t crash_len_max, crash_start_max, skew_max, step_cap;
};
constexpr uint32_t EV_CFG_RANDOMIZE = 1u << 0, EV_CFG_LOSSY = 1u << 1, EV_CFG_CRASHY = 1u << 2;

__host__ __device__ inline uint64_t ev_threshold(uint32_t ppm) {
  return ((((uint64_t)ppm) << 32) + 999999ull) / 1000000ull;
}

__host__ __device__ __forceinline__ uint32_t ctz32(uint32_t x) { return x ? (uint32_t)__builtin_ctz(x) : 32u; }

// Per-instance outcome handed to the driver when a lane finishes.
struct EvOut {
  uint32_t res[4];                    // pxb_result
  uint32_t flags;                     // PXB_F_* (low byte) for the counters
  uint32_t steps;
};

template <int PM, int N, int POOL, int W, class Mem>
struct EvLane {
  using S = Shape<PM, N, POOL, W>;
  using pool_mask_t = typename std::conditional<(POOL > 32), unsigned long long, uint32_t>::type;
  static constexpr uint32_t NL = S::NL;

  Mem m;
  // ---- instance ----
  uint32_t mode;
  uint32_t gid;                       // instance index within the launch
  uint32_t lo, hi;                    // global instance id (Philox counter words 0, 1)
  uint32_t P, dmax, loss_m1;
  bool lossy, faulty;
  int32_t s, last_tick;
  uint32_t acc_mask, prop_mask;       // this step's links with due messages left
  uint32_t tickp, stepped, pcur;      // Ticks due this step, proposers with input, proposer in turn
  // proposer states (ClientState, Client.hs:58-67): tickets < 2^12, commands = clientId
  uint32_t ticket[PM], cmd[PM], acks[PM], rs[PM], mr_t[PM], mr_v[PM], r2_v[PM], pending[PM];
  uint32_t skew[PM];
  uint32_t nsent[PM];                 // broadcasts of p whose copies have started (request-link seq)
  uint32_t bnext[PM];                 // next broadcast-ring slot
  uint32_t refc[PM];                  // ring-slot reference counts (4-bit nibbles)
  uint32_t pq, pq_len, acur;          // pending broadcasts (p << 3 | slot, 5 bits each), next acceptor
  pool_mask_t pfree;                  // free response-pool words
  uint32_t in_flight;
  uint32_t lflags, rounds, dval, dtick, execs, msgs, canon;
  unsigned long long clog;            // canonical log, 2-bit values (divergence check, SEMANTICS §7)
  uint32_t clog_len;
  bool bailed;

  __host__ __device__ static constexpr pool_mask_t full_pool() {
    return (POOL == 8 * (int)sizeof(pool_mask_t)) ? ~(pool_mask_t)0
                                                   : (pool_mask_t)(((pool_mask_t)1 << (POOL % (8 * sizeof(pool_mask_t)))) - 1u);
  }

  // ---- helpers over the per-proposer register arrays (q may differ per lane) ----
  __host__ __device__ static uint32_t getp(const uint32_t (&v)[PM], uint32_t q) {
    uint32_t r = v[0];
#pragma unroll
    for (int i = 1; i < PM; ++i) r = (q == (uint32_t)i) ? v[i] : r;
    return r;
  }
  __host__ __device__ static void setp(uint32_t (&v)[PM], uint32_t q, uint32_t x) {
#pragma unroll
    for (int i = 0; i < PM; ++i) v[i] = (q == (uint32_t)i) ? x : v[i];
  }

  // ---- instance start: parameters, Tick skews, isolation windows (SEMANTICS §4) ----
  __host__ __device__ void init(const EvParams& kp, uint32_t g) {
    gid = g;
    const uint64_t inst = kp.first_instance + g;
    lo = (uint32_t)inst;
    hi = (uint32_t)(inst >> 32);
    P = kp.n_prop;
    dmax = kp.delay_max;
    lossy = (kp.cfg & EV_CFG_LOSSY) != 0u;
    bool crashy = (kp.cfg & EV_CFG_CRASHY) != 0u;
    loss_m1 = kp.loss_m1;
    uint32_t crash_m1 = kp.crash_m1;
    if (kp.cfg & EV_CFG_RANDOMIZE) {                  // config-5 fuzz (SEMANTICS §4)
      const uint4 w = philox(lo, hi, 0u, 4u << 24, kp.k0, kp.k1);
      P = 1u + mulhi_n(w.x, kp.n_prop);
      const uint64_t lt = ev_threshold(mulhi_n(w.y, kp.loss_ppm + 1u));
      dmax = 1u + mulhi_n(w.z, kp.delay_max);
      const uint64_t ct = ev_threshold(mulhi_n(w.w, kp.crash_ppm + 1u));
      lossy = lt != 0ull;
      loss_m1 = (uint32_t)(lt - 1ull);
      crashy = ct != 0ull;
      crash_m1 = (uint32_t)(ct - 1ull);
    }
    faulty = lossy || dmax > 1u;
    uint4 wsk = make_uint4(0, 0, 0, 0);
    if (kp.skew_max > 0u) wsk = philox(lo, hi, 0u, 2u << 24, kp.k0, kp.k1);
    last_tick = 0;
    tickp = 0;
#pragma unroll
    for (int p = 0; p < PM; ++p) {
      const uint32_t wp = (p == 0) ? wsk.x : (p == 1) ? wsk.y : wsk.z;
      skew[p] = (kp.skew_max > 0u) ? mulhi_n(wp, kp.skew_max + 1u) : 0u;
      if ((uint32_t)p < P) {
        last_tick = ((int32_t)skew[p] > last_tick) ? (int32_t)skew[p] : last_tick;
        tickp |= (skew[p] == 0u) ? (1u << p) : 0u;
      }
      ticket[p] = cmd[p] = acks[p] = mr_t[p] = mr_v[p] = r2_v[p] = pending[p] = 0u;
      rs[p] = IDLE;
      nsent[p] = bnext[p] = refc[p] = 0u;
    }
#pragma unroll
    for (int a = 0; a < N; ++a) {
      uint32_t c0 = 0, c1 = 0;
      if (crashy) {
        const uint4 w = philox(lo, hi, 0u, (3u << 24) | (uint32_t)a, kp.k0, kp.k1);
        if (w.x <= crash_m1) {
          c0 = mulhi_n(w.y, kp.crash_start_max + 1u);
          c1 = c0 + 1u + mulhi_n(w.z, kp.crash_len_max);
        }
      }
      c0 = c0 < 4096u ? c0 : 4096u;
      c1 = c1 < 4096u ? c1 : 4096u;
      m.st(S::ACCW + a, 0u);
      m.st(S::ACCD + a, 0x811C9DC5u);
      m.st(S::ACCC + a, c0 | (c1 << 16));
    }
#pragma unroll
    for (int L = 0; L < (int)NL; ++L) {
      m.st(S::REQM + L, 0u);
      m.st(S::RSPM + L, 0u);
    }
#pragma unroll
    for (int i = 0; i < ((int)NL + 1) / 2; ++i) m.st(S::RSEQ + i, 0u);
#pragma unroll
    for (int i = 0; i < W * S::WW; ++i) m.st(S::WHEEL + i, 0u);
    pq = pq_len = acur = 0u;
    pfree = full_pool();
    in_flight = 0u;
    lflags = rounds = dval = dtick = execs = msgs = canon = 0u;
    clog = 0ull;
    clog_len = 0u;
    s = 0;
    acc_mask = prop_mask = 0u;
    stepped = pcur = 0u;
    bailed = false;
    mode = M_PROP;
  }

  // broadcast o = (kind, x, z) by proposer q: bookkeeping of bcast() (oracle)
  // and a pending entry whose N copies go out one per micro-step
  __host__ __device__ void broadcast(uint32_t q, uint32_t kind, uint32_t x, uint32_t z, bool pred) {
    rounds += (pred && kind == ASK) ? 1u : 0u;
    const bool ex = pred && kind == EXECUTE;
    execs += ex ? 1u : 0u;
    if (ex && dval == 0u) {                          // the decided value: first Execute (Client.hs:178)
      dval = getp(r2_v, q);
      dtick = x;
    }
    const uint32_t slot = getp(bnext, q);
    const uint32_t busy = (getp(refc, q) >> (4u * slot)) & 15u;
    if (pred && busy != 0u) bailed = true;           // ring slot still referenced by a queued copy
    if (pred) {
      m.st16(S::BRING, q * BR + slot, x | (z << 12) | (kind << 14));
      setp(bnext, q, (slot + 1u) & (BR - 1u));
      pq |= ((q << 3) | slot) << (5u * pq_len);
      pq_len += 1u;
    }
  }

  // the proposer q still has input this step (its Tick or a due response)
  __host__ __device__ bool has_input(uint32_t q) const {
    return ((tickp >> q) & 1u) != 0u || ctz32(prop_mask) < (q + 1u) * (uint32_t)N;
  }

  // move past proposers without input left: per (proposer, step) with input
  // the canonical accounting charges 48 B (SEMANTICS §8)
  __host__ __device__ void skip_idle() {
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      if (pcur < P && !has_input(pcur)) {
        canon += ((stepped >> pcur) & 1u) ? 48u : 0u;
        pcur += 1u;
      }
    }
  }

  // one micro-step; returns true when the instance ended (outputs in o)
  __host__ __device__ bool step(const EvParams& kp, EvOut& o) {
    bool snd = false;
    uint32_t sdir = 0, sp = 0, sa = 0, sword = 0, sk = 0;

    // ---------------- acceptor: one request (Server.hs:51-78) ----------------
    if (mode == M_ACC) {
      const uint32_t L = ctz32(acc_mask);
      const uint32_t a = L / PM, p = L - a * PM;
      const uint32_t rm = m.ld(S::REQM + L);
      const uint32_t len = rm >> 28;
      const uint32_t bslot = rm & 7u;
      const uint32_t rm2 = ((rm & 0x0FFFFFFFu) >> 7) | ((len - 1u) << 28);
      m.st(S::REQM + L, rm2);
      const bool keep = len > 1u && ((rm2 >> 3) & 15u) == ((uint32_t)s & 15u);
      acc_mask = keep ? acc_mask : (acc_mask & ~(1u << L));
      in_flight -= 1u;
      const uint32_t w16 = m.ld16(S::BRING, p * BR + bslot);
      setp(refc, p, getp(refc, p) - (1u << (4u * bslot)));
      const uint32_t kind = w16 >> 14, x = w16 & 0xFFFu, z = (w16 >> 12) & 3u;
      uint32_t A = m.ld(S::ACCW + a);
      const uint32_t win = m.ld(S::ACCC + a);
      const bool iso = (win & 0xFFFFu) <= (uint32_t)s && (uint32_t)s < (win >> 16);
      const bool dead = ((A >> 26) & 1u) != 0u;
      const uint32_t rb = (kind == PROPOSE) ? 12u : 8u;
      if (dead || iso) {
        canon += rb;                                 // discarded at a dead / isolated acceptor
      } else {
        canon += 2u * rb + 32u;
        const uint32_t t_max = A & 0xFFFu, t_store = (A >> 12) & 0xFFFu, val = (A >> 24) & 3u;
        uint32_t log_len = A >> 27;
        const bool is_ask = kind == ASK, is_prop = kind == PROPOSE, is_exec = kind == EXECUTE;
        const bool grant = is_ask && !(t_max >= x);              // Server.hs:56
        const bool accept = is_prop && x == t_max;               // :66 (equality, not >=)
        const bool hit = is_exec && t_max == x;                  // :75
        const bool panic = hit && val == 0u;                     // :76 (Q6)
        const bool run = hit && val != 0u;                       // :77-78
        const uint32_t rk = grant ? R1OK : accept ? R2S : (is_ask || is_prop) ? HAVE : 3u;
        const uint32_t rx = grant ? x : (accept ? 0u : t_max);
        const uint32_t ry = grant ? t_store : 0u;
        const uint32_t rz = grant ? val : 0u;
        const uint32_t nt_max = grant ? x : t_max;
        const uint32_t nt_store = accept ? x : (run ? 0u : t_store);
        const uint32_t nval = accept ? z : (run ? 0u : val);
        lflags |= panic ? (uint32_t)PXB_F_PANIC : 0u;
        if (run) {                                   // executed <>= [c]: log, digest, divergence
          if (log_len >= 31u) bailed = true;
          const uint32_t dg = m.ld(S::ACCD + a);
          m.st(S::ACCD + a, fnv_u32(dg, (val << 24) | 1u));
          if (log_len < clog_len) {
            if (((uint32_t)(clog >> (2u * log_len)) & 3u) != val) lflags |= PXB_F_LOG_DIVERGENCE;
          } else {
            clog |= (unsigned long long)val << (2u * log_len);
            clog_len += 1u;
          }
          log_len += 1u;
        }
        A = nt_max | (nt_store << 12) | (nval << 24) | ((dead || panic) ? (1u << 26) : 0u) | (log_len << 27);
        m.st(S::ACCW + a, A);
        if (rk != 3u) {                              // the reply, on link a -> p
          snd = true;
          sdir = 1u;
          sp = p;
          sa = a;
          sword = rx | (ry << 12) | (rz << 24) | (rk << 30);
        }
      }
      if (acc_mask == 0u) mode = M_PROP;
    }

    // ---------------- proposers: Tick, then responses in (a, seq) order -------
    if (mode == M_PROP) {
      skip_idle();
      // the next copy of a pending broadcast (sendToAllServers, Client.hs:122-123)
      if (!snd && pq_len != 0u) {
        const uint32_t e = pq & 31u;
        snd = true;
        sdir = 0u;
        sp = e >> 3;
        sa = acur;
        sword = e & 7u;
        sk = getp(nsent, sp);                         // the broadcast's index = the link's seq
        acur += 1u;
        if (acur == (uint32_t)N) {
          pq >>= 5;
          pq_len -= 1u;
          acur = 0u;
          setp(nsent, sp, getp(nsent, sp) + 1u);
        }
      }
      // one input of proposer pcur (room for the up to two broadcasts it may make)
      if (pcur < P && pq_len + 2u <= PQ_CAP) {
        const uint32_t q = pcur;
        uint32_t T = getp(ticket, q), R = getp(rs, q), K = getp(acks, q);
        uint32_t MT = getp(mr_t, q), MV = getp(mr_v, q), C2 = getp(r2_v, q), PD = getp(pending, q), CM = getp(cmd, q);
        uint32_t k0o = NONE, x0o = 0, z0o = 0;
        bool b1 = false;                              // the restart's AskForTicket (Client.hs:185)
        stepped |= 1u << q;
        if ((tickp >> q) & 1u) {                      // handleTick, Client.hs:196-207
          tickp &= ~(1u << q);
          if (R == IDLE) {
            T += 1u;
            CM = q + 1u;
            K = 0u;
            R = ROUND1;
            MT = MV = 0u;
            k0o = ASK;
            x0o = T;
          }
        } else {                                      // handleServerResponse, Client.hs:125-189
          const uint32_t Lr = ctz32(prop_mask);
          const uint32_t rm = m.ld(S::RSPM + Lr);
          const uint32_t len = (rm >> (4 * S::IB)) & 7u;
          const uint32_t im = (1u << S::IB) - 1u;
          const uint32_t k = rm & im;
          const uint32_t pe = m.ld(S::POOLW + k);
          const uint32_t pn = (len > 1u) ? m.ld(S::POOLW + ((rm >> S::IB) & im)) : 0u;
          pfree |= (pool_mask_t)1 << k;
          m.st(S::RSPM + Lr, (((rm & ((1u << (4 * S::IB)) - 1u)) >> S::IB)) | ((len - 1u) << (4 * S::IB)) |
                                 (rm & (15u << (4 * S::IB + 3))));
          const bool keep = len > 1u && ((pn >> 26) & 15u) == ((uint32_t)s & 15u);
          prop_mask = keep ? prop_mask : (prop_mask & ~(1u << Lr));
          in_flight -= 1u;
          const uint32_t kind = pe >> 30, x = pe & 0xFFFu, y = (pe >> 12) & 0xFFFu, z = (pe >> 24) & 3u;
          canon += 2u * (16u >> kind);                // Round1OK 16, HaveTicket 8, Round2Success 4
          const uint32_t maj = (uint32_t)N >> 1;      // haveMajority: acks > floor(N/2), :191-194
          if (kind == HAVE) {                         // :128-140
            if (R != IDLE && x >= T) {
              T = x + 1u;
              K = 0u;
              R = ROUND1;
              MT = MV = 0u;
              k0o = ASK;
              x0o = T;
            }
          } else if (kind == R1OK) {                  // :142-170
            if (R == ROUND1 && T == x) {
              K += 1u;
              uint32_t mt = MT, mv = MV;              // mr <> MostRecent mp (Common.hs:61-65)
              if (mv == 0u) {
                mt = y;
                mv = z;
              } else if (z != 0u && !(mt >= y)) {
                mt = y;
                mv = z;
              }
              if (K <= maj) {
                MT = mt;
                MV = mv;
              } else {                                // Q5: pending whenever mr is Just
                C2 = (mv == 0u) ? CM : mv;
                PD = (mv != 0u) ? 1u : 0u;
                K = 0u;
                R = ROUND2;
                MT = MV = 0u;
                k0o = PROPOSE;
                x0o = x;
                z0o = C2;
              }
            }
          } else {                                    // Round2Success, :172-189 (no ticket: Q2)
            if (R == ROUND2) {
              K += 1u;
              if (K > maj) {
                k0o = EXECUTE;
                x0o = T;
                if (PD) {
                  T += 1u;
                  K = 0u;
                  R = ROUND1;
                  MT = MV = 0u;
                  b1 = true;
                } else {
                  CM = 0u;
                  K = 0u;
                  R = IDLE;
                }
              }
            }
          }
        }
        setp(ticket, q, T);
        setp(rs, q, R);
        setp(acks, q, K);
        setp(mr_t, q, MT);
        setp(mr_v, q, MV);
        setp(r2_v, q, C2);
        setp(pending, q, PD);
        setp(cmd, q, CM);
        broadcast(q, k0o, x0o, z0o, k0o != NONE);
        broadcast(q, ASK, T, 0u, b1);
        skip_idle();
      }
    }

    // ---------------- the micro-step's one send (SEMANTICS §5) ----------------
    if (snd) {
      msgs += 1u;
      uint32_t k;
      const uint32_t Lq = sa * PM + sp;              // request-link / reply-seq index
      if (sdir == 0u) {
        k = sk;                                       // every broadcast tries every acceptor
      } else {
        k = m.ld16(S::RSEQ, Lq);
        if (k == 0xFFFFu) bailed = true;
        m.st16(S::RSEQ, Lq, k + 1u);
      }
      uint32_t d = 1u;
      bool ok = true;
      if (faulty) {
        const uint4 w = philox(lo, hi, k, (1u << 24) | (sdir << 16) | (sp << 8) | sa, kp.k0, kp.k1);
        ok = !(lossy && w.x <= loss_m1);
        d = 1u + mulhi_n(w.y, dmax);
      }
      if (ok) {
        const uint32_t s4 = (uint32_t)s & 15u;
        uint32_t due_rel, wbit;
        if (sdir == 0u) {                            // request copy on link p -> a
          const uint32_t rm = m.ld(S::REQM + Lq);
          const uint32_t len = rm >> 28;
          if (len >= CPHYS) bailed = true;
          const uint32_t rel = len ? (((rm >> (7u * (len - 1u) + 3u)) & 15u) - s4) & 15u : 0u;
          due_rel = d > rel ? d : rel;
          const uint32_t ent = sword | (((s4 + due_rel) & 15u) << 3);
          m.st(S::REQM + Lq, (rm & 0x0FFFFFFFu) | (ent << (7u * len)) | ((len + 1u) << 28));
          setp(refc, sp, getp(refc, sp) + (1u << (4u * sword)));
          wbit = 1u << Lq;
        } else {                                     // reply on link a -> p
          const uint32_t Lr = sp * (uint32_t)N + sa;
          const uint32_t rm = m.ld(S::RSPM + Lr);
          const uint32_t len = (rm >> (4 * S::IB)) & 7u;
          if (len >= CPHYS || pfree == 0) bailed = true;
          const uint32_t rel = len ? (((rm >> (4 * S::IB + 3)) & 15u) - s4) & 15u : 0u;
          due_rel = d > rel ? d : rel;
          const uint32_t due4 = (s4 + due_rel) & 15u;
          const uint32_t k2 = (POOL > 32) ? (uint32_t)__builtin_ctzll((unsigned long long)pfree | (1ull << 63))
                                          : ctz32((uint32_t)pfree) & 31u;
          pfree &= ~((pool_mask_t)1 << k2);
          m.st(S::POOLW + k2, sword | (due4 << 26));
          m.st(S::RSPM + Lr, (rm & ((1u << (S::IB * len)) - 1u)) | (k2 << (S::IB * len)) | ((len + 1u) << (4 * S::IB)) |
                                 (due4 << (4 * S::IB + 3)));
          wbit = 1u << (S::WW == 1 ? (S::PSH + Lr) : Lr);
        }
        const uint32_t slot = ((uint32_t)s + due_rel) & (uint32_t)(W - 1);
        const uint32_t wi = S::WHEEL + slot * S::WW + ((S::WW == 2 && sdir == 1u) ? 1u : 0u);
        m.st(wi, m.ld(wi) | wbit);
        in_flight += 1u;
      }
    }

    // ---------------- end of step: quiescence, step cap, next step ------------
    if (mode == M_PROP && pcur >= P && pq_len == 0u) {
      const bool quiet = in_flight == 0u && s >= last_tick;
      if (quiet || s + 1 >= (int32_t)kp.step_cap) {
        finish(!quiet, o);
        return true;
      }
      s += 1;
      const uint32_t slot = (uint32_t)s & (uint32_t)(W - 1);
      if (S::WW == 1) {
        const uint32_t wv = m.ld(S::WHEEL + slot);
        m.st(S::WHEEL + slot, 0u);
        acc_mask = wv & 0xFFFFu;
        prop_mask = wv >> 16;
      } else {
        acc_mask = m.ld(S::WHEEL + 2 * slot);
        prop_mask = m.ld(S::WHEEL + 2 * slot + 1);
        m.st(S::WHEEL + 2 * slot, 0u);
        m.st(S::WHEEL + 2 * slot + 1, 0u);
      }
      tickp = 0u;
#pragma unroll
      for (int p = 0; p < PM; ++p) tickp |= ((uint32_t)p < P && skew[p] == (uint32_t)s) ? (1u << p) : 0u;
      pcur = 0u;
      stepped = 0u;
      mode = acc_mask ? M_ACC : M_PROP;
    }
    return false;
  }

  // ---- outputs of an ended instance (SEMANTICS §7) ----
  __host__ __device__ void finish(bool capped, EvOut& o) {
    const uint32_t steps = (uint32_t)s + 1u;
    uint32_t f = lflags | (capped ? (uint32_t)PXB_F_STEP_CAP : 0u) | (dval ? 0u : (uint32_t)PXB_F_UNDECIDED);
#pragma unroll
    for (int p = 0; p < PM; ++p)
      f |= (!capped && (uint32_t)p < P && rs[p] != IDLE) ? (uint32_t)PXB_F_STUCK : 0u;
    canon += 16u + 4u * (uint32_t)N;
    o.res[0] = dval ? ((dval << 24) | 1u) : 0u;
    o.res[1] = dval ? dtick : 0u;
    o.res[2] = rounds;
    o.res[3] = (f & 0xFFu) | (steps << 16);
    o.flags = f;
    o.steps = steps;
    mode = M_IDLE;
  }

  // final per-acceptor outputs (digest, record) of an ended instance
  __host__ __device__ uint32_t digest_of(int a) const {
    return fnv_u32(m.ld(S::ACCD + a), m.ld(S::ACCW + a) >> 27);
  }
  __host__ __device__ void record_of(int a, uint32_t r[4]) const {
    const uint32_t A = m.ld(S::ACCW + a);
    const uint32_t val = (A >> 24) & 3u;
    r[0] = A & 0xFFFu;
    r[1] = (A >> 12) & 0xFFFu;
    r[2] = val ? ((val << 24) | 1u) : 0u;
    r[3] = (A >> 27) | (((A >> 26) & 1u) << 31);
  }
};

// EV eligibility of a launch (host side): single decree, faulty, 12-bit tickets,
// delays inside the 16-step wheel.  Fault-free and log-mode batches keep the
// paxos_kernel.h kernels.
__host__ inline bool eligible(const pxb_config* c) {
  return c->n_ticks <= 1 && c->step_cap <= MAX_STEP_CAP && c->delay_max <= 15;
}

}  // namespace ev
}  // namespace pxb

namespace pxb {
namespace ev {

// Launch parameters from the ABI config (host side; mirrors pxb_run_device).
__host__ inline EvParams make_params(const pxb_config* c) {
  EvParams p{};
  p.first_instance = c->first_instance;
  p.k0 = (uint32_t)c->seed;
  p.k1 = (uint32_t)(c->seed >> 32);
  p.n_prop = c->n_proposers;
  p.delay_max = c->delay_max;
  p.loss_ppm = c->loss_ppm;
  p.crash_ppm = c->crash_ppm;
  p.crash_len_max = c->crash_len_max;
  p.crash_start_max = c->crash_start_max;
  p.skew_max = c->skew_max;
  p.step_cap = c->step_cap;
  const uint64_t lt = ev_threshold(c->loss_ppm), ct = ev_threshold(c->crash_ppm);
  p.cfg = ((c->flags & PXB_CFG_RANDOMIZE) ? EV_CFG_RANDOMIZE : 0u) | (lt ? EV_CFG_LOSSY : 0u) | (ct ? EV_CFG_CRASHY : 0u);
  p.loss_m1 = (uint32_t)(lt - 1ull);
  p.crash_m1 = (uint32_t)(ct - 1ull);
  return p;
}

// the timing wheel must outlast the longest delay
__host__ inline int wheel_for(uint32_t delay_max) { return delay_max <= 7 ? 8 : 16; }

}  // namespace ev
}  // namespace pxb
