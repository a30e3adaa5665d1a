// paxos_ffp.h — per-lane kernel for the other fault-free batches: duelling
// proposers (P = 2, 3) and log mode (several Ticks per proposer: the stock
// Main.hs topology with its ticker running, docs/SEMANTICS.md §9), one lane
// per instance.  The single-proposer single-decree case has its own leaner
// kernel (paxos_ff1.h); this one follows the same plan:
//
//   * fault-free: a message sent in step s is handled in step s + 1, so the
//     in-flight state is each proposer's broadcasts of the last two steps
//     (one word each: every copy carries the same payload) — registers;
//   * step s runs the acceptor phase (acceptor a takes the broadcasts of
//     s - 1 in (proposer, seq) order, Server.hs:51-78) and, fused with it, the
//     proposer phase of s + 1: each proposer's Tick of s + 1 (Client.hs:196-207),
//     then every reply as the acceptor makes it (Client.hs:125-189).  Exact
//     because proposer p's phase in s + 1 reads only p's state and its replies
//     of s, in acceptor order (FIFO per link) after its Tick, and the acceptor
//     phase reads nothing a proposer writes; at s = step_cap - 1 nothing is
//     fused and the replies stay in flight;
//   * commands are 16-bit (clientId << 14 | t), as in the general kernel's log
//     mode, widened to (clientId << 24 | t) for digests and results; the
//     canonical log (first PXB_LOG_TRACK positions, the divergence check) is
//     kept per lane in LDS, lane-interleaved.
//
// An instance whose proposer makes more than two broadcasts in one step is
// bailed to the general kernel (its link FIFOs hold up to 8).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "paxos_ff1.h"

namespace pxb {
namespace ffp {

using ff1::req_bytes;
using ff1::rsp_bytes;

// for (I = B; I < E; ++I) f(I) with I a compile-time constant, so the
// per-proposer / per-acceptor register arrays are only ever indexed by
// constants (a plain unrolled loop left some of them in scratch memory)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}
constexpr uint32_t TM = 0x3FFFu;              // ticket field
constexpr int LT = PXB_LOG_TRACK;             // canonical-log positions checked

struct FfpParams {
  uint64_t first_instance;
  uint32_t k0, k1;                            // Philox key (Tick skew draws)
  uint32_t n_prop, skew_max, step_cap, n_ticks, tick_period;
  uint32_t n_instances;
  uint4* out;                                 // pxb_result records (nullable)
  uint32_t* dig;                              // log digests (nullable)
  uint4* acc;                                 // final acceptor records (nullable)
  unsigned long long* part;                   // ev::EV_TCOPIES partial run-total rows
  uint32_t* bail_ids;                         // ids of bailed instances (capacity bail_cap)
  uint32_t* bail_n;                           // their count, 0 on entry
  uint32_t bail_cap;
  uint32_t bail_all;                          // tests: bail every instance
};

// a 16-bit command as the reference's code (id << 24) | t
__device__ __forceinline__ uint32_t code32(uint32_t v) { return v ? (((v >> 14) << 24) | (v & TM)) : 0u; }

template <int PM, int N>
struct FfpLane {
  uint32_t* clog;                             // this lane's canonical log: LT halfwords, interleaved by lane
  // acceptors: t_max [13:0] | t_store [27:14] | dead [30]; value (16-bit command, 0 = Nothing)
  uint32_t aw[N], av[N], llen[N], accd[N];
  PropState S[PM];                            // cmd / mr_v / r2_v as 16-bit commands
  uint32_t nt[PM], tl[PM];                    // next Tick step, Ticks left
  // broadcasts in flight per proposer: sent in s - 1 (cur) and in s (mid);
  // words x [13:0] | cmd [29:14] | kind [31:30]
  uint32_t nc[PM], c0[PM], c1[PM], nm[PM], m0[PM], m1[PM];
  uint32_t P, last_tick, lflags, rounds, msgs, execs, canon, dval, dtick, clog_len;
  bool bailed;

  __device__ __forceinline__ void init(const FfpParams& kp, uint64_t inst) {
    P = kp.n_prop;
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (kp.skew_max > 0u)                                       // SEMANTICS §4, purpose "skew"
      w = philox((uint32_t)inst, (uint32_t)(inst >> 32), 0u, 2u << 24, kp.k0, kp.k1);
    last_tick = 0u;
    sfor<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      const uint32_t wp = (p == 0) ? w.x : (p == 1) ? w.y : w.z;
      const uint32_t sk = (kp.skew_max > 0u && (uint32_t)p < P) ? mulhi_n(wp, kp.skew_max + 1u) : 0u;
      nt[p] = sk;
      tl[p] = ((uint32_t)p < P) ? kp.n_ticks : 0u;
      const uint32_t lt = sk + (kp.n_ticks - 1u) * kp.tick_period;
      last_tick = ((uint32_t)p < P && lt > last_tick) ? lt : last_tick;
      S[p] = PropState{0, 0u, 0u, IDLE, 0, 0u, 0, 0u, 0u};        // Client.hs:90-95
      nc[p] = c0[p] = c1[p] = nm[p] = m0[p] = m1[p] = 0u;
    });
#pragma unroll
    for (int a = 0; a < N; ++a) {
      aw[a] = av[a] = llen[a] = 0u;                             // Server.hs:46
      accd[a] = 0x811C9DC5u;
    }
    lflags = rounds = msgs = execs = canon = dval = dtick = clog_len = 0u;
    bailed = false;
    // step 0's proposer phase: the Ticks of step 0
    sfor<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      uint32_t n0 = 0u, n1 = 0u, nn = 0u;
      canon += tick_due<p>(0u, kp.tick_period, n0, n1, nn) ? 48u : 0u;
      m0[p] = n0;
      m1[p] = n1;
      nm[p] = nn;
    });
  }

  // a broadcast of proposer p (Client.hs:122-123), predicated on go
  template <int p>
  __device__ __forceinline__ void bcast(bool go, uint32_t kind, uint32_t x, uint32_t cmd, uint32_t& n0,
                                        uint32_t& n1, uint32_t& nn) {
    const uint32_t w = x | (cmd << 14) | (kind << 30);
    bailed = bailed | (go & (nn >= 2u));
    n0 = (go & (nn == 0u)) ? w : n0;
    n1 = (go & (nn == 1u)) ? w : n1;
    nn += go ? 1u : 0u;
    msgs += go ? (uint32_t)N : 0u;
    rounds += (go & (kind == ASK)) ? 1u : 0u;
    const bool ex = go & (kind == EXECUTE);
    execs += ex ? 1u : 0u;
    const bool first = ex & (dval == 0u);                    // the first Execute decides (SEMANTICS §7)
    dval = first ? S[p].r2_v : dval;
    dtick = first ? x : dtick;
  }

  // handleTick (Client.hs:196-207): a Tick while busy is dropped
  template <int p>
  __device__ __forceinline__ void tick(uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    PropState& R = S[p];
    const bool t_go = R.rs == IDLE;                           // :199
    R.ticket = t_go ? R.ticket + 1 : R.ticket;                // :200
    R.cmd = t_go ? (((uint32_t)p + 1u) << 14) | ((uint32_t)R.ticket & TM) : R.cmd;   // :202-204 "c<id>.<t>"
    R.acks = t_go ? 0u : R.acks;                              // :205
    R.rs = t_go ? ROUND1 : R.rs;                              // :206
    R.mr_t = t_go ? 0 : R.mr_t;
    R.mr_v = t_go ? 0u : R.mr_v;
    bcast<p>(t_go, ASK, (uint32_t)R.ticket, 0u, n0, n1, nn);  // :207
  }
  // the Tick of proposer p due at step t, if any (then its next one)
  template <int p>
  __device__ __forceinline__ bool tick_due(uint32_t t, uint32_t period, uint32_t& n0, uint32_t& n1,
                                           uint32_t& nn) {
    const bool d = (tl[p] != 0u) & (nt[p] == t);
    if (d) {
      tick<p>(n0, n1, nn);
      nt[p] += period;
      tl[p] -= 1u;
    }
    return d;
  }

  // handleServerResponse (Client.hs:125-189) of one reply to p, one function
  // per reply kind, predicated on go (Q3: the sender is not checked)
  template <int p>
  __device__ __forceinline__ void fold_r1ok(bool go, int32_t px, int32_t py, uint32_t pz, uint32_t& n0,
                                            uint32_t& n1, uint32_t& nn) {
    PropState& R = S[p];
    canon += go ? 2u * 16u : 0u;
    const bool o_go = go & (R.rs == ROUND1) & (R.ticket == px);       // :144-145
    const uint32_t K1 = R.acks + 1u;                                    // :146
    const bool take = (R.mr_v == 0u) | ((pz != 0u) & !(R.mr_t >= py));  // MostRecent (Common.hs:61-65)
    const int32_t mt = take ? py : R.mr_t;
    const uint32_t mv = take ? pz : R.mr_v;
    const bool maj = o_go & (K1 > ((uint32_t)N >> 1));                 // :152-154, :191-194
    R.r2_t = maj ? px : R.r2_t;                                        // :157-167 (Q5)
    R.r2_v = maj ? ((mv == 0u) ? R.cmd : mv) : R.r2_v;
    R.pending = maj ? ((mv != 0u) ? 1u : 0u) : R.pending;
    R.acks = maj ? 0u : (o_go ? K1 : R.acks);                          // :168
    R.rs = maj ? ROUND2 : R.rs;                                        // :169
    R.mr_t = maj ? 0 : (o_go ? mt : R.mr_t);
    R.mr_v = maj ? 0u : (o_go ? mv : R.mr_v);
    bcast<p>(maj, PROPOSE, (uint32_t)px, R.r2_v, n0, n1, nn);          // :170
  }
  template <int p>
  __device__ __forceinline__ void fold_have(bool go, int32_t px, uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    PropState& R = S[p];
    canon += go ? 2u * 8u : 0u;
    const bool h = go & (R.rs != IDLE) & (px >= R.ticket);              // :130-132
    R.ticket = h ? px + 1 : R.ticket;                                   // :134-135
    R.acks = h ? 0u : R.acks;                                           // :137
    R.rs = h ? ROUND1 : R.rs;                                           // :138
    R.mr_t = h ? 0 : R.mr_t;
    R.mr_v = h ? 0u : R.mr_v;
    bcast<p>(h, ASK, (uint32_t)R.ticket, 0u, n0, n1, nn);               // :140
  }
  template <int p>
  __device__ __forceinline__ void fold_r2s(bool go, uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    PropState& R = S[p];
    canon += go ? 2u * 4u : 0u;
    const bool s_go = go & (R.rs == ROUND2);                            // :172-174 (no ticket: Q2)
    const uint32_t K1 = R.acks + 1u;                                    // :175
    const bool maj = s_go & (K1 > ((uint32_t)N >> 1));                 // :176-177
    const bool restart = maj & (R.pending != 0u);                       // :179
    bcast<p>(maj, EXECUTE, (uint32_t)R.ticket, 0u, n0, n1, nn);         // :178 Execute (s ^. ticket)
    R.ticket = restart ? R.ticket + 1 : R.ticket;                       // :182
    R.acks = maj ? 0u : (s_go ? K1 : R.acks);                          // :183 / :188
    R.rs = restart ? ROUND1 : (maj ? IDLE : R.rs);                      // :184 / :189
    R.mr_t = restart ? 0 : R.mr_t;
    R.mr_v = restart ? 0u : R.mr_v;
    R.cmd = (maj & !restart) ? 0u : R.cmd;                              // :187
    bcast<p>(restart, ASK, (uint32_t)R.ticket, 0u, n0, n1, nn);         // :185
  }

  // handleClientRequest (Server.hs:51-78) of broadcast q of proposer p by
  // acceptor a; with fuse its reply goes straight to p (an input of step s + 1)
  template <int a, int p>
  __device__ __forceinline__ void accept(uint32_t q, bool fuse, uint32_t& nrep, bool& inp,
                                         uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    const uint32_t kind = q >> 30, x = q & TM, z = (q >> 14) & 0xFFFFu;
    const uint32_t pay = req_bytes(kind);
    const uint32_t A = aw[a], t_max = A & TM;
    const bool live = (A >> 30) == 0u;
    canon += live ? 2u * pay + 32u : pay;
    const bool rep = live & (kind != EXECUTE);
    nrep += rep ? 1u : 0u;
    msgs += rep ? 1u : 0u;
    inp = inp | (fuse & rep);
    if (kind == ASK) {                                        // :54-62
      const bool grant = live & !(t_max >= x);                // :56
      aw[a] = grant ? (A & ~TM) | x : A;                      // :60
      // :61-62 Round1OK t prop, or :58 HaveTicket T_max
      fold_r1ok<p>(fuse & grant, (int32_t)x, (int32_t)((A >> 14) & TM), av[a], n0, n1, nn);
      if (fuse & live & !grant) fold_have<p>(true, (int32_t)t_max, n0, n1, nn);
    } else if (kind == PROPOSE) {                             // :64-71
      const bool acc = live & (x == t_max);                   // :66 (equality, not >=)
      aw[a] = acc ? t_max | (x << 14) : A;                    // :68 prop := Just (t, c)
      av[a] = acc ? z : av[a];
      fold_r2s<p>(fuse & acc, n0, n1, nn);                    // :70 Round2Success
      if (fuse & live & !acc) fold_have<p>(true, (int32_t)t_max, n0, n1, nn);   // :71
    } else {                                                  // Execute, :73-78 (no reply)
      const uint32_t v = av[a];
      const bool hit = live & (t_max == x);                   // :75
      if (hit & (v == 0u)) {                                  // :76 pattern failure: dead forever (Q6)
        aw[a] = A | (1u << 30);
        lflags |= PXB_F_PANIC;
      } else if (hit) {                                       // :77-78 executed <>= [c]; prop := Nothing
        aw[a] = t_max;
        av[a] = 0u;
        const uint32_t pos = llen[a];
        accd[a] = fnv_u32(accd[a], code32(v));
        if (pos < (uint32_t)LT) {                             // divergence over the first LT positions
          uint16_t* h = reinterpret_cast<uint16_t*>(clog);
          const uint32_t i = ((pos >> 1) * 64u) * 2u + (pos & 1u);
          if (pos < clog_len) {
            if (h[i] != v) lflags |= PXB_F_LOG_DIVERGENCE;
          } else {
            h[i] = (uint16_t)v;
            clog_len = pos + 1u;
          }
        } else {
          lflags |= PXB_F_LOG_TRUNC;
        }
        llen[a] = pos + 1u;
      }
    }
  }

  // one step s (see the file comment); returns true when the instance ended after it
  __device__ __forceinline__ bool step(uint32_t s, const FfpParams& kp, uint32_t& steps, bool& capped) {
    const bool fuse = s + 1u < kp.step_cap;
    uint32_t n0[PM], n1[PM], nn[PM];
    bool inp[PM];
    sfor<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      n0[p] = n1[p] = nn[p] = 0u;
      inp[p] = fuse && tick_due<p>(s + 1u, kp.tick_period, n0[p], n1[p], nn[p]);
    });
    uint32_t nrep = 0u;
    sfor<0, N>([&](auto ac) {
      constexpr int a = decltype(ac)::value;
      sfor<0, PM>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        if (nc[p] > 0u) accept<a, p>(c0[p], fuse, nrep, inp[p], n0[p], n1[p], nn[p]);
        if (__builtin_expect(nc[p] > 1u, 0)) accept<a, p>(c1[p], fuse, nrep, inp[p], n0[p], n1[p], nn[p]);
      });
    });
    bool mid_any = false;
    sfor<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      canon += inp[p] ? 48u : 0u;                             // proposer p had an input in s + 1
      mid_any = mid_any | (nm[p] != 0u);
      nc[p] = nm[p];
      c0[p] = m0[p];
      c1[p] = m1[p];
      nm[p] = nn[p];
      m0[p] = n0[p];
      m1[p] = n1[p];
    });
    // ---- end of step s: nothing in flight (the broadcasts of s, the replies of s) ----
    const bool quiet = !mid_any & (nrep == 0u) & (s >= last_tick);
    capped = !quiet & !fuse;
    steps = s + 1u;
    return quiet | capped;
  }

  __device__ __forceinline__ void finish(bool capped, uint32_t steps, uint32_t (&res)[4], uint32_t& f) {
    bool busy = false;
    sfor<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      busy = busy | (((uint32_t)p < P) & (S[p].rs != IDLE));
    });
    f = lflags | (capped ? (uint32_t)PXB_F_STEP_CAP : 0u) | (dval ? 0u : (uint32_t)PXB_F_UNDECIDED) |
        ((!capped && busy) ? (uint32_t)PXB_F_STUCK : 0u);
    canon += 16u + 4u * (uint32_t)N;
    res[0] = code32(dval);
    res[1] = dval ? dtick : 0u;
    res[2] = rounds;
    res[3] = (f & 0xFFu) | (steps << 16);
  }

  __device__ __forceinline__ uint4 record(int a) const {
    const uint32_t A = aw[a];
    return make_uint4(A & TM, (A >> 14) & TM, code32(av[a]), llen[a] | ((A >> 30) << 31));
  }
};

// Grid-stride over the launch's instances, one per lane at a time (as
// paxos_ff1_kernel); run totals in registers, wave-reduced into one of
// EV_TCOPIES partial rows (plus the log-truncation count).
// Waves per SIMD the register allocation targets (1 = the compiler's choice):
// the stock Main.hs log-mode workload, P = 2 and N = 2, at 6 (1.55 -> 1.73 G
// instances/s on MI355X); one proposer over five acceptors with 8 Ticks at 5
// (3.35 -> 3.59 G/s); the other small shapes where that spills at most a few
// words (one proposer, N <= 3: 6)
template <int PM, int N>
constexpr int ffp_waves() {
  return (PM == 2 && N == 2) ? 6 : (PM == 1 && N <= 3) ? 6 : (PM == 1 && N == 5) ? 5 : 1;
}
template <int PM, int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(ffp_waves<PM, N>())))
void paxos_ffp_kernel(FfpParams kp) {
  __shared__ uint32_t s_clog[4][LT / 2][64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + wib));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  unsigned long long* const trow = kp.part + (size_t)(wave % ev::EV_TCOPIES) * 16u;
  ev::EvTotals tot;
  tot.clear();
  uint32_t ltrunc = 0u;
  for (uint32_t w0 = wave * 64u; w0 < kp.n_instances; w0 += n_waves * 64u) {
    if (__builtin_amdgcn_ballot_w64(tot.c[0] >= ev::EV_FLUSH) != 0ull) {
      tot.flush(trow, lane);
      const uint64_t t = ev::EvTotals::wave_sum((uint64_t)ltrunc);
      if (lane == 0 && t) atomicAdd(&trow[PXB_C_LOG_TRUNC], (unsigned long long)t);
      ltrunc = 0u;
    }
    const uint32_t g = w0 + lane;
    if (g < kp.n_instances) {
      FfpLane<PM, N> L;
      L.clog = &s_clog[wib][0][lane];
      L.init(kp, kp.first_instance + g);
      L.bailed = L.bailed | (kp.bail_all != 0u);
      uint32_t steps = 0u;
      bool capped = false;
#pragma nounroll
      for (uint32_t s = 0;; ++s)
        if (L.step(s, kp, steps, capped) || L.bailed) break;
      if (__builtin_expect(L.bailed, 0)) {
        const uint32_t pos = atomicAdd(kp.bail_n, 1u);
        if (pos < kp.bail_cap) kp.bail_ids[pos] = g;
      } else {
        uint32_t res[4], f;
        L.finish(capped, steps, res, f);
        tot.c[0] += 1u;
        tot.c[1] += (f & PXB_F_UNDECIDED) ? 1u : 0u;
        tot.c[2] += (f & PXB_F_STUCK) ? 1u : 0u;
        tot.c[3] += (f & PXB_F_PANIC) ? 1u : 0u;
        tot.c[4] += (f & PXB_F_LOG_DIVERGENCE) ? 1u : 0u;
        tot.c[5] += (f & PXB_F_STEP_CAP) ? 1u : 0u;
        tot.c[6] += L.rounds;
        tot.c[7] += steps;
        tot.c[8] += L.msgs;
        tot.c[9] += L.execs;
        tot.canon += L.canon;
        ltrunc += (f & PXB_F_LOG_TRUNC) ? 1u : 0u;
        if (kp.out) kp.out[g] = make_uint4(res[0], res[1], res[2], res[3]);
        if (kp.dig) {
#pragma unroll
          for (int a = 0; a < N; ++a) kp.dig[(uint64_t)g * N + a] = fnv_u32(L.accd[a], L.llen[a]);
        }
        if (kp.acc) {
#pragma unroll
          for (int a = 0; a < N; ++a) kp.acc[(uint64_t)g * N + a] = L.record(a);
        }
      }
    }
  }
  tot.flush(trow, lane);
  const uint64_t t = ev::EvTotals::wave_sum((uint64_t)ltrunc);
  if (lane == 0 && t) atomicAdd(&trow[PXB_C_LOG_TRUNC], (unsigned long long)t);
}

}  // namespace ffp
}  // namespace pxb
