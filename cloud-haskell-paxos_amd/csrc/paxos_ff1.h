// paxos_ff1.h — per-lane kernel for fault-free single-proposer batches
// (BASELINE configs 1 and 2: P = 1, no loss, delay 1, no crash windows; Tick
// skew allowed), one lane per instance.
//
// Fault-free means every message sent in step s is handled in step s + 1
// (docs/SEMANTICS.md §5-§6), so an instance's in-flight state is just the
// broadcasts its proposer made in the previous step (all N copies carry the
// same payload) and one reply per acceptor.  A lane keeps all of it — N
// acceptors (Server.hs:24-31), the proposer's ClientState (Client.hs:58-67),
// the in-flight messages and the run totals — in registers and runs each step
// as the two phases of §6:
//   proposer phase   its Tick at the skew step (handleTick, Client.hs:196-207),
//                    then the replies of acceptors 0..N-1 in order
//                    (handleServerResponse, Client.hs:125-189);
//   acceptor phase   acceptors 0..N-1 each handle the previous step's
//                    broadcasts in order (handleClientRequest, Server.hs:51-78)
//                    and reply (Common.hs:36-39 sendToAllServers / send).
// The two phases of one step are independent (every send is due one step
// later), so the proposer phase runs first and the acceptor phase overwrites
// the replies it consumed.  The handlers are the shared ones of
// paxos_device.h.
//
// Compared with the general kernel (one lane per (instance, acceptor), the
// proposer state replicated in the instance's N lanes and its fold done with
// cross-lane ballots and DPP reductions), nothing is replicated and nothing
// crosses lanes.  An instance this layout cannot hold (more than two
// broadcasts in one step, two replies from one acceptor in one step, a log of
// 17 entries: none happens with one proposer) is "bailed" to the general
// kernel, like the per-lane event kernel's (paxos_ev_kernel.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "paxos_ev_kernel.h"

namespace pxb {
namespace ff1 {

struct Ff1Params {
  uint64_t first_instance;
  uint32_t k0, k1;                            // Philox key (Tick skew draws)
  uint32_t skew_max, step_cap;
  uint32_t n_instances;
  uint4* out;                                 // pxb_result records (nullable)
  uint32_t* dig;                              // log digests (nullable)
  uint4* acc;                                 // final acceptor records (nullable)
  unsigned long long* part;                   // ev::EV_TCOPIES partial run-total rows
  uint32_t* bail_ids;                         // ids of bailed instances (capacity bail_cap)
  uint32_t* bail_n;                           // their count, 0 on entry
  uint32_t bail_cap;
  uint32_t bail_all;                          // tests: bail every instance (exercises the general kernel)
};

// request payload bytes (SEMANTICS §8): Ask 8, Propose 12, Execute 8
__device__ __forceinline__ uint32_t req_bytes(uint32_t kind) { return kind == PROPOSE ? 12u : 8u; }
// response payload bytes: Round1OK 16, HaveTicket 8, Round2Success 4
__device__ __forceinline__ uint32_t rsp_bytes(uint32_t kind) { return 16u >> kind; }

// The lanes of a wave run in lockstep (every instance of a skew-free batch
// takes the same steps), so the handlers branch on the message kind and the
// proposer state: a wave runs only the path its instances are on (measured on
// MI355X: 10 % faster than the predicated select form of the event kernel,
// which pays for every path of every handler).
constexpr uint32_t TM = 0x3FFFu;              // ticket field

template <int N>
struct Ff1Lane {
  // acceptors, packed: t_max [13:0] | t_store [27:14] | val [29:28] | dead [30]
  // (tickets <= step_cap <= 8192 < 2^14, SEMANTICS §6; commands travel as the
  // clientId, 0 = Nothing); log lengths; running log digests
  uint32_t aw[N], llen[N], accd[N];
  // the proposer (clientId 1): its command travels as the clientId, 1
  PropState S;
  // in flight: the broadcasts sent in the previous step (cur, handled by the
  // acceptors now) and in this step (mid), as words x [13:0] | z [29:28] | kind [31:30]
  uint32_t ncur, cur0, cur1, nmid, mid0, mid1;
  // per-instance outputs and counters
  uint32_t skew, lflags, rounds, msgs, execs, canon, dval, dtick;
  uint32_t clog;                              // canonical log, 2-bit values (divergence, SEMANTICS §7)
  uint32_t clog_len;
  bool bailed;

  __device__ __forceinline__ void init(const Ff1Params& kp, uint64_t inst) {
    skew = 0u;
    if (kp.skew_max > 0u) {                                     // SEMANTICS §4, purpose "skew"
      const uint4 w = philox((uint32_t)inst, (uint32_t)(inst >> 32), 0u, 2u << 24, kp.k0, kp.k1);
      skew = mulhi_n(w.x, kp.skew_max + 1u);
    }
#pragma unroll
    for (int a = 0; a < N; ++a) {
      aw[a] = 0u;                                               // Server.hs:46
      llen[a] = 0u;
      accd[a] = 0x811C9DC5u;
    }
    S = PropState{0, 0u, 0u, IDLE, 0, 0u, 0, 0u, 0u};           // Client.hs:90-95
    ncur = cur0 = cur1 = nmid = mid0 = mid1 = 0u;
    lflags = rounds = msgs = execs = canon = dval = dtick = 0u;
    clog = 0u;
    clog_len = 0u;
    bailed = false;
    // step 0's proposer phase: its Tick (the replies of a step are handled
    // within the step before, see step())
    if (skew == 0u) tick(mid0, mid1, nmid);
  }

  // handleTick, Client.hs:196-207 (48 canonical bytes: an input of the proposer)
  __device__ __forceinline__ void tick(uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    canon += 48u;
    const bool t_go = S.rs == IDLE;                           // :199
    S.ticket = t_go ? S.ticket + 1 : S.ticket;                // :200
    S.cmd = t_go ? 1u : S.cmd;                                // :202-204 "c1.1" as clientId 1
    S.acks = t_go ? 0u : S.acks;                              // :205
    S.rs = t_go ? ROUND1 : S.rs;                              // :206
    S.mr_t = t_go ? 0 : S.mr_t;
    S.mr_v = t_go ? 0u : S.mr_v;
    bcast(t_go, ASK, (uint32_t)S.ticket, 0u, n0, n1, nn);     // :207
  }

  // a broadcast of the proposer phase (Client.hs:122-123): N copies, due next
  // step, as one word x [13:0] | z [29:28] | kind [31:30] (predicated on go)
  __device__ __forceinline__ void bcast(bool go, uint32_t kind, uint32_t x, uint32_t z, uint32_t& n0, uint32_t& n1,
                                        uint32_t& nn) {
    const uint32_t w = x | (z << 28) | (kind << 30);
    bailed = bailed | (go & (nn >= 2u));
    n0 = (go & (nn == 0u)) ? w : n0;
    n1 = (go & (nn == 1u)) ? w : n1;
    nn += go ? 1u : 0u;
    msgs += go ? (uint32_t)N : 0u;
    rounds += (go & (kind == ASK)) ? 1u : 0u;
    const bool ex = go & (kind == EXECUTE);
    execs += ex ? 1u : 0u;
    const bool first = ex & (dval == 0u);                    // the first Execute decides (SEMANTICS §7)
    dval = first ? S.r2_v : dval;
    dtick = first ? x : dtick;
  }

  // handleServerResponse (Client.hs:125-189) of acceptor a's reply, one
  // function per reply kind, predicated on go (Q3: the sender is not checked)
  // (returns whether it reached the majority: its Propose is then the pass's
  // only broadcast, Round2 ignores further Round1OKs)
  __device__ __forceinline__ bool fold_r1ok(bool go, int32_t px, int32_t py, uint32_t pz) {
    canon += go ? 2u * 16u : 0u;
    const bool o_go = go & (S.rs == ROUND1) & (S.ticket == px);        // :144-145
    const uint32_t K1 = S.acks + 1u;                                     // :146
    const bool take = (S.mr_v == 0u) | ((pz != 0u) & !(S.mr_t >= py));   // mr <> MostRecent (Common.hs:61-65)
    const int32_t mt = take ? py : S.mr_t;
    const uint32_t mv = take ? pz : S.mr_v;
    const bool maj = o_go & (K1 > ((uint32_t)N >> 1));                  // :152-154, haveMajority :191-194
    S.r2_t = maj ? px : S.r2_t;                                         // :157-167 (Q5: pending whenever mr is Just)
    S.r2_v = maj ? ((mv == 0u) ? S.cmd : mv) : S.r2_v;
    S.pending = maj ? ((mv != 0u) ? 1u : 0u) : S.pending;
    S.acks = maj ? 0u : (o_go ? K1 : S.acks);                           // :168
    S.rs = maj ? ROUND2 : S.rs;                                         // :169
    S.mr_t = maj ? 0 : (o_go ? mt : S.mr_t);
    S.mr_v = maj ? 0u : (o_go ? mv : S.mr_v);
    return maj;                                                         // :170 Propose (r2_t, r2_v)
  }
  __device__ __forceinline__ void fold_have(bool go, int32_t px, uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    canon += go ? 2u * 8u : 0u;
    const bool h = go & (S.rs != IDLE) & (px >= S.ticket);               // :130-132
    S.ticket = h ? px + 1 : S.ticket;                                    // :134-135
    S.acks = h ? 0u : S.acks;                                            // :137
    S.rs = h ? ROUND1 : S.rs;                                            // :138
    S.mr_t = h ? 0 : S.mr_t;
    S.mr_v = h ? 0u : S.mr_v;
    bcast(h, ASK, (uint32_t)S.ticket, 0u, n0, n1, nn);                   // :140
  }
  // (returns whether it reached the majority: Execute, then with a pending
  // command the restart's AskForTicket; Idle / Round1 ignore further ones)
  __device__ __forceinline__ bool fold_r2s(bool go, bool& restart) {
    canon += go ? 2u * 4u : 0u;
    const bool s_go = go & (S.rs == ROUND2);                             // :172-174 (no ticket: Q2)
    const uint32_t K1 = S.acks + 1u;                                     // :175
    const bool maj = s_go & (K1 > ((uint32_t)N >> 1));                  // :176-177
    restart = maj & (S.pending != 0u);                                   // :179
    S.ticket = restart ? S.ticket + 1 : S.ticket;                        // :182
    S.acks = maj ? 0u : (s_go ? K1 : S.acks);                           // :183 / :188
    S.rs = restart ? ROUND1 : (maj ? IDLE : S.rs);                       // :184 / :189
    S.mr_t = restart ? 0 : S.mr_t;
    S.mr_v = restart ? 0u : S.mr_v;
    S.cmd = (maj & !restart) ? 0u : S.cmd;                               // :187
    return maj;
  }
  // the broadcasts of a Round2Success majority: Execute (s ^. ticket), :178,
  // and after a restart AskForTicket with the new ticket, :185
  __device__ __forceinline__ void r2s_bcast(bool maj, bool restart, uint32_t& n0, uint32_t& n1, uint32_t& nn) {
    const uint32_t t = (uint32_t)S.ticket;
    bcast(maj, EXECUTE, restart ? t - 1u : t, 0u, n0, n1, nn);
    bcast(restart, ASK, t, 0u, n0, n1, nn);
  }

  // the reply of acceptor a (predicated on go): counted, at most one per
  // acceptor per step (two would need a FIFO: bail)
  __device__ __forceinline__ void reply(bool go, int a, uint32_t& nmask) {
    bailed = bailed | (go & (((nmask >> a) & 1u) != 0u));
    nmask |= go ? (1u << a) : 0u;
    msgs += go ? 1u : 0u;
  }

  // handleClientRequest (Server.hs:51-78) of broadcast q by every acceptor, in
  // acceptor order: one branch on the broadcast's kind, then selects (the
  // acceptors of one instance may differ: a dead one, a refused ticket).
  // With fuse, each reply is handed straight to the proposer as an input of
  // the next step (its proposer phase only reads the proposer state and these
  // replies, in acceptor order, after that step's Tick): the next step's
  // broadcasts go to n0/n1/nn.  A Round1OK / Round2Success pass issues its
  // one broadcast after the pass unless a HaveTicket comes first.
  __device__ __forceinline__ void accept_all(uint32_t q, bool fuse, uint32_t& nmask, uint32_t& n0, uint32_t& n1,
                                             uint32_t& nn) {
    const uint32_t kind = q >> 30, z = (q >> 28) & 3u, x = q & TM;
    const uint32_t pay = req_bytes(kind);
    constexpr uint32_t MAJ = (uint32_t)N >> 1;               // haveMajority: acks > floor(N/2), Client.hs:191-194
    if (kind == ASK) {                                        // :54-62
      uint32_t G = 0u, L = 0u;                                // granting / live acceptors
#pragma unroll
      for (int a = 0; a < N; ++a) {
        const uint32_t A = aw[a], t_max = A & TM;
        const bool live = (A >> 30) == 0u;
        canon += live ? 2u * pay + 32u : pay;
        const bool grant = live & !(t_max >= x);              // :56
        aw[a] = grant ? (A & ~TM) | x : A;                    // :60 (t_store, val unchanged)
        reply(live, a, nmask);                                // :61-62 Round1OK t prop / :58 HaveTicket T_max
        G |= grant ? 1u << a : 0u;
        L |= live ? 1u << a : 0u;
      }
      if (fuse & (L != 0u)) {
        if (__builtin_expect(L == G, 1)) {
          // only Round1OKs (Client.hs:142-170), in acceptor order: while in
          // Round1 at ticket x each one counts, up to the majority, folding its
          // proposal into mr (Common.hs:61-65); after it, Round2 ignores them
          canon += 2u * 16u * (uint32_t)__builtin_popcount(G);
          const bool o_go = (S.rs == ROUND1) & (S.ticket == (int32_t)x);
          const uint32_t need = MAJ + 1u - S.acks, cnt = (uint32_t)__builtin_popcount(G);
          const bool maj = o_go & (cnt >= need);
          int32_t mt = S.mr_t;
          uint32_t mv = S.mr_v, seen = 0u;
#pragma unroll
          for (int a = 0; a < N; ++a) {
            const bool g = (((G >> a) & 1u) != 0u) & (seen < need);
            seen += ((G >> a) & 1u);
            const int32_t py = (int32_t)((aw[a] >> 14) & TM);
            const uint32_t pz = (aw[a] >> 28) & 3u;
            const bool take = g & ((mv == 0u) | ((pz != 0u) & !(mt >= py)));
            mt = take ? py : mt;
            mv = take ? pz : mv;
          }
          S.r2_t = maj ? (int32_t)x : S.r2_t;                 // :157-167 (Q5: pending whenever mr is Just)
          S.r2_v = maj ? ((mv == 0u) ? S.cmd : mv) : S.r2_v;
          S.pending = maj ? ((mv != 0u) ? 1u : 0u) : S.pending;
          S.acks = maj ? 0u : (o_go ? S.acks + cnt : S.acks);   // :146 / :168
          S.rs = maj ? ROUND2 : S.rs;                          // :169
          S.mr_t = maj ? 0 : (o_go ? mt : S.mr_t);
          S.mr_v = maj ? 0u : (o_go ? mv : S.mr_v);
          bcast(maj, PROPOSE, x, S.r2_v, n0, n1, nn);          // :170
        } else {
          // a HaveTicket among them: every reply through its handler, in order
          bool m = false;
#pragma unroll
          for (int a = 0; a < N; ++a) {
            const uint32_t A = aw[a];
            if ((G >> a) & 1u) {
              m = m | fold_r1ok(true, (int32_t)x, (int32_t)((A >> 14) & TM), (A >> 28) & 3u);
            } else if ((L >> a) & 1u) {
              bcast(m, PROPOSE, (uint32_t)S.r2_t, S.r2_v, n0, n1, nn);
              m = false;
              fold_have(true, (int32_t)(A & TM), n0, n1, nn);
            }
          }
          bcast(m, PROPOSE, (uint32_t)S.r2_t, S.r2_v, n0, n1, nn);
        }
      }
    } else if (kind == PROPOSE) {                             // :64-71
      uint32_t G = 0u, L = 0u;                                // accepting / live acceptors
#pragma unroll
      for (int a = 0; a < N; ++a) {
        const uint32_t A = aw[a], t_max = A & TM;
        const bool live = (A >> 30) == 0u;
        canon += live ? 2u * pay + 32u : pay;
        const bool acc = live & (x == t_max);                 // :66 (equality, not >=)
        aw[a] = acc ? t_max | (x << 14) | (z << 28) : A;      // :68 prop := Just (t, c)
        reply(live, a, nmask);                                // :70 Round2Success / :71 HaveTicket T_max
        G |= acc ? 1u << a : 0u;
        L |= live ? 1u << a : 0u;
      }
      if (fuse & (L != 0u)) {
        if (__builtin_expect(L == G, 1)) {
          // only Round2Successes (Client.hs:172-189): in Round2 each counts (no
          // ticket: Q2) up to the majority; then Idle or, pending, Round1 ignore them
          canon += 2u * 4u * (uint32_t)__builtin_popcount(G);
          const bool s_go = S.rs == ROUND2;
          const uint32_t need = MAJ + 1u - S.acks, cnt = (uint32_t)__builtin_popcount(G);
          const bool maj = s_go & (cnt >= need);
          const bool restart = maj & (S.pending != 0u);       // :179
          S.ticket = restart ? S.ticket + 1 : S.ticket;       // :182
          S.acks = maj ? 0u : (s_go ? S.acks + cnt : S.acks); // :175 / :183 / :188
          S.rs = restart ? ROUND1 : (maj ? IDLE : S.rs);      // :184 / :189
          S.mr_t = restart ? 0 : S.mr_t;
          S.mr_v = restart ? 0u : S.mr_v;
          S.cmd = (maj & !restart) ? 0u : S.cmd;              // :187
          r2s_bcast(maj, restart, n0, n1, nn);                // :178 Execute, :185 AskForTicket
        } else {
          bool m = false, re = false;
#pragma unroll
          for (int a = 0; a < N; ++a) {
            if ((G >> a) & 1u) {
              bool r;
              m = m | fold_r2s(true, r);
              re = re | r;
            } else if ((L >> a) & 1u) {
              r2s_bcast(m, re, n0, n1, nn);
              m = re = false;
              fold_have(true, (int32_t)(aw[a] & TM), n0, n1, nn);
            }
          }
          r2s_bcast(m, re, n0, n1, nn);
        }
      }
    } else {                                                  // Execute, :73-78 (no reply)
#pragma unroll
      for (int a = 0; a < N; ++a) {
        const uint32_t A = aw[a], v = (A >> 28) & 3u;
        const bool live = (A >> 30) == 0u;
        canon += live ? 2u * pay + 32u : pay;
        const bool hit = live & ((A & TM) == x);              // :75
        const bool panic = hit & (v == 0u);                   // :76 pattern failure: dead forever (Q6)
        const bool run = hit & (v != 0u);                     // :77-78 executed <>= [c]; prop := Nothing
        lflags |= panic ? (uint32_t)PXB_F_PANIC : 0u;
        aw[a] = run ? (A & TM) : (panic ? (A | (1u << 30)) : A);
        bailed = bailed | (run & (llen[a] >= 16u));           // (16 positions of the 32-bit canonical log)
        accd[a] = run ? fnv_u32(accd[a], (v << 24) | 1u) : accd[a];
        const bool old = llen[a] < clog_len;
        lflags |= (run & old & (((clog >> (2u * llen[a])) & 3u) != v)) ? (uint32_t)PXB_F_LOG_DIVERGENCE : 0u;
        clog |= (run & !old) ? v << (2u * llen[a]) : 0u;
        clog_len += (run & !old) ? 1u : 0u;
        llen[a] += run ? 1u : 0u;
      }
    }
  }

  // One step s (SEMANTICS §6); returns true when the instance ended after it.
  // Its acceptor phase handles the broadcasts sent in s - 1 and, fused with
  // it, the proposer phase of step s + 1 runs: that step's Tick, then each
  // reply as it is made (a reply sent in s is an input of s + 1; the proposer
  // phase of s + 1 reads nothing else).  Below the step cap only: at s =
  // step_cap - 1 the instance ends with those replies in flight.
  __device__ __forceinline__ bool step(uint32_t s, uint32_t step_cap, uint32_t& steps, bool& capped) {
    const bool fuse = s + 1u < step_cap;
    uint32_t n0 = 0u, n1 = 0u, nn = 0u;                       // the broadcasts of step s + 1
    if (fuse & (s + 1u == skew)) tick(n0, n1, nn);
    uint32_t nmask = 0u;
    if (ncur > 0u) accept_all(cur0, fuse, nmask, n0, n1, nn);
    if (__builtin_expect(ncur > 1u, 0)) accept_all(cur1, fuse, nmask, n0, n1, nn);
    // 48 canonical bytes for the proposer's input in s + 1 (its Tick counted them)
    canon += (fuse & (nmask != 0u) & (s + 1u != skew)) ? 48u : 0u;
    // ---- end of step s: nothing in flight (the broadcasts of s, the replies of s) ----
    const bool quiet = (nmid == 0u) & (nmask == 0u) & (s >= skew);
    ncur = nmid;
    cur0 = mid0;
    cur1 = mid1;
    nmid = nn;
    mid0 = n0;
    mid1 = n1;
    capped = !quiet & !fuse;
    steps = s + 1u;
    return quiet | capped;
  }

  __device__ __forceinline__ void finish(bool capped, uint32_t steps, uint32_t (&res)[4], uint32_t& f) {
    f = lflags | (capped ? (uint32_t)PXB_F_STEP_CAP : 0u) | (dval ? 0u : (uint32_t)PXB_F_UNDECIDED) |
        ((!capped && S.rs != IDLE) ? (uint32_t)PXB_F_STUCK : 0u);
    canon += 16u + 4u * (uint32_t)N;
    res[0] = dval ? ((dval << 24) | 1u) : 0u;
    res[1] = dval ? dtick : 0u;
    res[2] = rounds;
    res[3] = (f & 0xFFu) | (steps << 16);
  }

  __device__ __forceinline__ uint4 record(int a) const {
    const uint32_t A = aw[a], val = (A >> 28) & 3u;
    return make_uint4(A & TM, (A >> 14) & TM, val ? ((val << 24) | 1u) : 0u, llen[a] | ((A >> 30) << 31));
  }
};

// Grid-stride over the launch's instances, one per lane at a time; the lanes
// of a wave run in lockstep (every instance of a skew-free batch takes the
// same steps).  The grid holds several times the resident blocks
// (pxb_run_device): a block that ends early leaves its CU to the next one, so
// slower CUs take fewer blocks (one launch of equal static shares per
// resident wave ran 20 % slower than two launches overlapped on two streams,
// at every size from 2^26 to 2^29; a work queue inside the kernel spilled).
// Run totals as in the per-lane event kernel: register sums, wave-reduced
// into one of EV_TCOPIES partial rows.
// (N <= 5: 5 waves per SIMD, 96 VGPRs; the compiler's own choice, 101, fits 4
// and is 5 % slower on config 2)
template <int N>
#ifndef PXB_FF1_W5
#define PXB_FF1_W5 5
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(N <= 5 ? PXB_FF1_W5 : 1))) void paxos_ff1_kernel(
    Ff1Params kp) {
  const uint32_t lane = threadIdx.x & 63u;
  // (wave-uniform, so kept in an SGPR: 28 B of scratch spill per lane instead of 36)
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
  const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
  unsigned long long* const trow = kp.part + (size_t)(wave % ev::EV_TCOPIES) * 16u;
  ev::EvTotals tot;
  tot.clear();
  for (uint32_t w0 = wave * 64u; w0 < kp.n_instances; w0 += n_waves * 64u) {
    // (wave-uniform: flush the sums before any could wrap)
    if (__builtin_amdgcn_ballot_w64(tot.c[0] >= ev::EV_FLUSH) != 0ull) tot.flush(trow, lane);
    const uint32_t g = w0 + lane;
    if (g < kp.n_instances) {
      Ff1Lane<N> L;
      L.init(kp, kp.first_instance + g);
      L.bailed = kp.bail_all != 0u;
      uint32_t steps = 0u;
      bool capped = false;
#pragma nounroll   // (unrolled by 2: 7 % slower on config 2)
      for (uint32_t s = 0;; ++s)
        if (L.step(s, kp.step_cap, steps, capped) || L.bailed) break;
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
}

}  // namespace ff1
}  // namespace pxb
