// paxos_ev.h — the per-lane ("event") batched ticket-Paxos kernel for faulty
// single-decree schedules (loss, delay, crash windows, duelling, fuzzing).
//
// One lane runs one whole instance: its N acceptors (Server.hs:44-89), its P
// proposers (Client.hs:85-207) and its 2·P·N directed links.  Within a step
// the acceptor phase and the proposer phase are independent (every send is
// due one step later at the earliest, docs/SEMANTICS.md §6), so every wave
// iteration a lane does, predicated and without branches:
//
//   ACC   one due request handled by one acceptor (handleClientRequest,
//         Server.hs:51-78) and its reply sent on link a -> p;
//   COPY  the next copy of a pending broadcast sent on link p -> a
//         (sendToAllServers, Client.hs:122-123);
//   PROP  one input of one proposer: its Tick (handleTick, Client.hs:196-207)
//         or one due response (handleServerResponse, Client.hs:125-189),
//         whose broadcasts join the pending queue;
//   END   when the step has no work left: quiescence / step cap (the role of
//         Main.hs:49-53), then the next step that has a due message or a Tick
//         (steps without either change nothing and are skipped).
//
// The canonical order (§6) only constrains each process: acceptor a takes
// its requests by (p, seq), proposer p its Tick and then its responses by
// (a, seq).  The due-request mask has bit a*PM+p, so its lowest set bit
// serves each acceptor in proposer order; the proposer-input mask has bit
// p*(N+1) for the Tick and p*(N+1)+1+a for link a -> p.
//
// Lanes are independent (instances share nothing: Main.hs:41-45), so a wave
// never waits on its slowest instance: a lane whose instance ends writes its
// outputs and takes the next instance from the work queue.
//
// Per-lane state:
//   registers  proposer states, acceptor words (T_max, T_store, val, dead,
//              log length) and isolation windows, pending-broadcast queue,
//              ring reference counts, due masks, counters;
//   LDS        (lane-interleaved words, [word][lane]: every access is
//              bank-conflict free) request-link FIFOs (4 x {broadcast ring
//              slot, due} per link; the payload lives once per broadcast in a
//              per-proposer ring), response-link FIFOs (indices into a
//              per-lane pool of response words), reply sequence numbers, log
//              digests, and a timing wheel of per-step due-link masks.
//
// The semantic queue depth stays PXB_QUEUE_DEPTH = 8; the physical FIFOs hold
// 4 (and the pool POOL responses).  An instance that would need more is
// "bailed": its id goes to a list that the general kernel (paxos_kernel.h)
// re-runs from scratch, so results stay exact for every schedule.
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

#ifndef PXB_EV_SL_RH
#define PXB_EV_SL_RH 1
#endif
#ifndef PXB_EV_LG_RH
#define PXB_EV_LG_RH 0
#endif
#ifndef PXB_EV_STORE_BACK
#define PXB_EV_STORE_BACK 1
#endif
#ifndef PXB_EV_PQ_CAP
#define PXB_EV_PQ_CAP 4
#endif
constexpr uint32_t PQ_CAP = PXB_EV_PQ_CAP;    // pending broadcasts per lane
constexpr uint32_t MAX_STEP_CAP = 4095;   // 12-bit tickets (tickets <= step_cap, SEMANTICS §6)
static_assert(MAX_STEP_CAP < PXB_TICKET_LIMIT, "EV tickets never reach the overflow limit");

// lane modes
constexpr uint32_t M_IDLE = 0, M_RUN = 1;

template <int PM_, int N_, int POOL_, int W_, bool CMP_, bool LG_ = false, bool SL_ = false, int SP_ = 0>
struct Shape {
  static constexpr int PM = PM_, N = N_, POOL = POOL_, W = W_;
  static constexpr bool SP = SP_ != 0;               // simple schedule: no loss, no Tick skew, single decree
  // tight (SP_ == 2, layout 7): the simple schedule's compact layout with the
  // response FIFOs in halfwords (3 entries of pool index + 1 or a Round2Success
  // code, zero above the length), so that a lane fits 52 LDS words (13 KB per
  // wave: 12 waves per CU, 3 on every SIMD); its bails re-run on layout 6
  // (also the faulty log-mode shape over <= 10 links on the 8-step wheel:
  // 75 words with a 15-word pool, 8 waves per CU instead of 7)
  static constexpr bool RH = SP_ == 2 || (PXB_EV_LG_RH && LG_ && PM_ * N_ <= 10 && W_ == 8) ||
                             (PXB_EV_SL_RH && SL_ && PM_ == 2 && PM_ * N_ > 16 && PM_ * N_ <= 18 && W_ == 8);
  static constexpr bool CMP = CMP_;                  // compact links (see Layouts)
  static constexpr bool LG = LG_;                    // log mode (several Ticks, long logs; see Layouts)
  static constexpr bool SL = SL_;                    // slim 4-entry layout (see Layouts)
  static constexpr int NLQ = PM * N;                 // request (and response) links
  // proposer-input bits: a Tick bit and N link bits per proposer (the simple
  // schedule has no Tick after init: N link bits, so that an input bit is its
  // response link's index)
  static constexpr int IT = SP ? 0 : 1, IW = N + IT;
  static constexpr int NIN = PM * IW;
  static constexpr int WW = (NLQ + NIN <= 32) ? 1 : 2;   // wheel words per slot
  static constexpr int ISH = (WW == 1) ? NLQ : 0;    // input-bit offset in its wheel word
  static constexpr int IB = POOL <= 32 ? 5 : 6;      // pool index bits
  // request FIFO: QC entries of EB bits (ring slot SB bits, due mod 2^DB), length
  // at QL (QLB bits); compact: the reply seq of the same (a, p) pair in the
  // word's top KB bits.  Compact on the 4-step wheel (delays <= 4): 5-bit
  // entries (4 ring slots: 2 bits; every queued due lies in [sb, sb + 5]: due
  // mod 8), so 4 of them fit beside a 9-bit reply seq (3-entry FIFOs bailed
  // 0.46 % of config 4's instances, 98 % of them on a full request FIFO;
  // tools/wave_model.cpp)
  static constexpr bool C5 = CMP && W == 4;
  static constexpr int EB = C5 ? 5 : 7, SB = C5 ? 2 : 3, DB = EB - SB;
  static constexpr int QC = (CMP && !C5) ? 3 : 4, QL = EB * QC, QLB = (QC == 4) ? 3 : 2;
  static constexpr int KSH = QL + QLB, KB = 32 - KSH;
  // response FIFO: RC pool indices of IB bits, length at RL (RLB bits), tail due at RD;
  // slim over > 18 links (RSN): RC = 5 entries, each its pool index + 1 (0: empty),
  // no length or due field (the length from the highest set bit, the tail's due
  // from its pool word).  Config 5's three-proposer shape: P = 3 bails 1.7 % ->
  // 0.4 % of instances, the general kernel 53 -> 17 ms at 2^25, the per-lane kernel
  // +28 ms (it now runs those long instances itself): +0.7 % end to end.  On the
  // two-proposer shape (0.01 % bails) it only costs (-1 %): not used there.
  static constexpr bool RSN = SL && PM * N > 18;
  // (RZ: entries are pool index + 1, zero above the length, the length from
  // the highest set bit and the tail's due from its pool word or code)
  static constexpr bool RZ = RSN || RH;

  static constexpr int RC = RH ? 3 : RSN ? 5 : 4, RL = IB * RC, RLB = 3, RD = RL + RLB;
  static constexpr int POOLB_SHIFT = RZ ? 1 : 0;     // entry e's pool word: POOLW - POOLB_SHIFT + e
  // compact layouts with a pool of <= 24 words: a Round2Success (no payload)
  // takes no pool word; its FIFO entry is the code RCB + (due & 7) instead
#ifdef PXB_EV_NO_RCODE
  static constexpr bool RCODE = false;               // (A/B: every response takes a pool word)
#else
  static constexpr bool RCODE = CMP && POOL <= 24 && IB == 5;
#endif
  static constexpr uint32_t RCB = 24;
  // LDS word offsets
  static constexpr int REQ = 0;                      // NLQ: request links, index a*PM + p (CMP: + reply seq)
  static constexpr int RSEQ = REQ + NLQ;             // !CMP: NLQ halfwords of reply seq, index a*PM + p
  // (slim: the reply seqs are bytes in registers)
  static constexpr int RSP0 = RSEQ + ((CMP || SL) ? 0 : (NLQ + 1) / 2);   // NLQ response links, index p*N + a
  // (RH: the halfword links go last, after the wheel, so that every pool
  // load of a 5-bit entry, Round2Success codes included, stays in the lane's words)
  static constexpr int POOLW = RH ? RSP0 : RSP0 + NLQ;   // POOL response words
  // broadcast ring slots per proposer: short-delay (compact) schedules never
  // hold more than 4 broadcasts of one proposer in flight (BASELINE configs
  // 3 and 4: the bail rate is the same with 4 slots as with 8), nor does
  // faulty log mode (extra.log_mode_faulty: no bail with 4)
  static constexpr uint32_t BR = (CMP || LG || SL) ? 4 : 8;
  // log mode: the responses' 14-bit commands in a halfword array beside the
  // pool (+ one dummy halfword), the first LOG_TRACK positions of the
  // canonical log (halfwords), 32-bit broadcast payloads
  static constexpr int POOLZ = POOLW + POOL;         // LG: POOL + 1 halfwords
  static constexpr int BRING = POOLZ + (LG ? POOL / 2 + 1 : 0);   // PM*BR payloads: halfwords (LG: words)
  static constexpr int CLOG = BRING + (LG ? PM * BR : PM * BR / 2);   // LG: PXB_LOG_TRACK halfwords
  // (CLP: the slim log-mode shape packs its canonical log's 14-bit commands
  // end to end, 14 words instead of 16)
  static constexpr bool CLP = LG && SL;
  static constexpr int CLW = !LG ? 0 : CLP ? (PXB_LOG_TRACK * 14 + 31) / 32 : PXB_LOG_TRACK / 2;
  static constexpr int WHEEL = CLOG + CLW;           // W * WW due masks
  static constexpr int RSP = RH ? WHEEL + W * WW : RSP0;
  static constexpr int WORDS = WHEEL + W * WW + (RH ? (NLQ + 1) / 2 : 0);
  static_assert(W == 4 || W == 8 || W == 16, "wheel of 4, 8 or 16 steps");
  static_assert(NIN <= 32 && NLQ <= 32, "masks are 32-bit");
  static_assert(RH ? (IB * RC <= 16 && POOL < (1 << IB) - 1) : RSN ? (IB * RC <= 32 && POOL < (1 << IB)) : (RD + 4 <= 32),
                "response-link word");
  // (index + 1 below the Round2Success codes)
  static_assert(!(RZ && RCODE) || POOL < (int)RCB, "pool entries and codes");
  static_assert(!RH || (SP && !LG && RCODE && DB == 3) || ((LG || SL) && !RCODE), "halfword links: layouts 7, 4, 5");
  // (every 5-bit entry indexes the lane's words: else send_first clamps the code's pool load)
  static constexpr bool TE_SAFE = POOLW - POOLB_SHIFT + 31 < WORDS;
  static constexpr int POOLB = POOLW - POOLB_SHIFT;
  static_assert(QL + QLB <= 31, "request-link word");
};

// Layouts (docs/SEMANTICS.md §2 encodings; tickets < 2^12):
//   request-link word   entry i (7 bits at 7i): broadcast slot [2:0] | due&15 [6:3]; len at QL
//                       (compact: 3 entries, len [22:21], and the reply seq of the same
//                       (a, p) pair in [31:23], one word for both; compact on the 4-step
//                       wheel: 4 entries of 5 bits, slot [1:0] | due&7 [4:2], len [22:20],
//                       reply seq [31:23]; else 4 entries, len [30:28], reply seq in its
//                       own halfword)
//   response-link word  pool index i (IB bits at IB*i); len [4IB+2:4IB]; last due&15 above it
//                       (compact, pool <= 24: index 24 + (due & 7) = a Round2Success, no
//                       pool word; dues stay within s + delay_max <= s + 4;
//                       slim over > 18 links: 5 entries of pool index + 1, 0 above the
//                       length, nothing else)
//   response word       x [11:0] | y [23:12] | z [25:24] | kind [31:30]
//   broadcast payload   x [11:0] | z [13:12] | kind [15:14]
//   acceptor word       t_max [11:0] | t_store [23:12] | val [25:24] | dead [26] | log_len [31:27]
//   window              c0 [15:0] | c1 [31:16]  (clamped to 4096: steps are < 4095)
// Slim (SL, layout 5: the 4-entry layout on the 8-step wheel for runs of at
// most 512 steps, BASELINE config 5): the reply seqs are bytes in registers
// (a 256th reply on one link bails), 4 broadcast ring slots per proposer, and
// the response pools of EvPool: 120 LDS words per lane for P = 3, N = 9 (5
// waves per CU instead of 4), 86 for P = 2 (7 instead of 6).
// Log mode (LG) carries commands "c<id>.<t>" as 14 bits, id [13:12] | t [11:0]
// (t >= 1; 0 = Nothing) and keeps 4 broadcast ring slots per proposer (with
// the 19-word response pool of topologies of <= 10 links, EvPool: 86 words per
// lane for P = 2, N = 5, 7 waves per CU), so:
//   acceptor word       t_max [11:0] | t_store [23:12] | dead [24]; a second word (accv):
//                       the stored command [13:0] | log_len [31:14]
//   response word       z [25:24] unused: the command in the pool's halfword array
//   broadcast payload   x [11:0] | z [25:12] | kind [31:30], one word
//   proposer            pw1 = mr_v [13:0] | r2_v [27:14], pw2 = the t of its own command
// The due step of a queued response is kept in its link word only for the
// tail (the FIFO max-chain of §5); "is the next one due now" reads the
// response's own due nibble [29:26] (x, y < 2^12, z < 4: bits 26..29 free).

// Per-launch parameters shared by the device kernel and the host test.
struct EvParams {
  uint64_t first_instance;
  uint32_t k0, k1;
  uint32_t cfg;                       // EV_CFG_* bits
  uint32_t n_prop, delay_max;
  uint32_t loss_m1, crash_m1;
  uint32_t loss_ppm, crash_ppm;
  uint32_t crash_len_max, crash_start_max, skew_max, step_cap;
  uint32_t n_ticks, tick_period;      // log mode: Ticks per proposer (> 1) and their spacing
};
constexpr uint32_t EV_CFG_RANDOMIZE = 1u << 0, EV_CFG_LOSSY = 1u << 1, EV_CFG_CRASHY = 1u << 2;
constexpr uint32_t EV_CFG_DRAWS = 1u << 3;    // some instance may draw message loss / delay

__host__ __device__ inline uint64_t ev_threshold(uint32_t ppm) {
  return ((((uint64_t)ppm) << 32) + 999999ull) / 1000000ull;
}

// true in every lane when the predicate holds in any lane of the wave (host: the
// lane's own value): guards code that only a few lanes of a wave ever need
__host__ __device__ __forceinline__ bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(p) != 0ull;
#else
  return p;
#endif
}

// Host-only probes (tools/wave_model.cpp): which wave-level branches and slots
// a lane uses in an iteration.  Nothing on the device.
enum : uint32_t {
  EVP_END = 1u << 0, EVP_FIN = 1u << 1, EVP_RUN = 1u << 2, EVP_TICK_ENTER = 1u << 3, EVP_TICK_END = 1u << 4,
  EVP_ACC = 1u << 5, EVP_PROP = 1u << 6, EVP_COPY = 1u << 7, EVP_SEND1 = 1u << 8, EVP_BCAST = 1u << 9,
  // bail causes: ring slot still referenced, response FIFO full, response pool
  // empty, request FIFO full, log length, reply seq
  EVB_RING = 1u << 16, EVB_RFIFO = 1u << 17, EVB_POOL = 1u << 18, EVB_QFIFO = 1u << 19, EVB_LOG = 1u << 20,
  EVB_RSEQ = 1u << 21,
};
#if defined(PXB_EV_PROBES) && !defined(__HIP_DEVICE_COMPILE__)
extern thread_local uint32_t ev_probe_bits;
#define PXB_EV_PROBE(b, c) (ev_probe_bits |= (c) ? (uint32_t)(b) : 0u)
#else
#define PXB_EV_PROBE(b, c) ((void)0)
#endif

// (a small index times a constant: the 24-bit mask lets LLVM use
// v_mad_u32_u24 / v_mul_u32_u24, full rate, where it cannot bound the operand
// itself -- it had emitted v_mad_u64_u32 and v_mul_lo_u32)
__host__ __device__ __forceinline__ uint32_t u24(uint32_t x) { return x & 0xFFFFFFu; }
// x * C: a shift for a power of two (where the mask only costs), else the 24-bit form
template <uint32_t C>
__host__ __device__ __forceinline__ uint32_t mulc(uint32_t x) { return ((C & (C - 1u)) == 0u) ? x * C : u24(x) * C; }
__host__ __device__ __forceinline__ uint32_t ctz32(uint32_t x) { return x ? (uint32_t)__builtin_ctz(x) : 32u; }
__host__ __device__ __forceinline__ uint32_t popc32(uint32_t x) { return (uint32_t)__builtin_popcount(x); }
__host__ __device__ __forceinline__ uint32_t nbits32(uint32_t x) { return x ? 32u - (uint32_t)__builtin_clz(x) : 0u; }

// Per-instance outcome handed to the driver when a lane finishes.
struct EvOut {
  uint32_t res[4];                    // pxb_result
  uint32_t flags;                     // PXB_F_* (low byte) for the counters
  uint32_t steps;
};

// EARLY: a step may end with the copies of its last broadcast still to send
// (see end_op); the trace kernel turns it off so that its per-step records
// hold every message of the step in flight, as the oracle's do.
template <int PM, int N, int POOL, int W, bool CMP, class Mem, bool EARLY = true, bool LG = false, bool SL = false,
          int SP = 0>
struct EvLane {
  using S = Shape<PM, N, POOL, W, CMP, LG, SL, SP>;
  static constexpr bool kEarly = EARLY;
  // acceptor fields (Layouts): dead bit, log-length shift (LG: in accv) and its limit
  static constexpr uint32_t A_DEAD = LG ? 24 : 26, A_LEN = LG ? 14 : 27, A_LEN_MAX = LG ? (1u << 18) - 1u : 31;
  using pool_mask_t = typename std::conditional<(POOL > 32), unsigned long long, uint32_t>::type;
  static constexpr uint32_t NLQ = S::NLQ;
  static constexpr uint32_t WM = (uint32_t)W - 1u;
  static constexpr uint32_t QLM = (1u << S::QLB) - 1u, RLM = (1u << S::RLB) - 1u;
  static constexpr uint32_t IM = (1u << S::IB) - 1u;
  static constexpr uint32_t DM = (1u << S::DB) - 1u;     // request-entry due mask

  Mem m;
  uint32_t rk[20];                    // Philox round keys (set_keys): uniform, held in VGPRs
  // ---- instance ----
  uint32_t mode;
  uint32_t gid;                       // instance index within the launch
  uint32_t lo, hi;                    // global instance id (Philox counter words 0, 1)
  uint32_t P, dmax, loss_m1;
  bool lossy;
  // (SP: loss-free batches, whose sends never test a loss draw)
  static constexpr bool kLossy = !SP;
  int32_t s, last_tick;
  uint32_t acc_mask;                  // this step's request links with due messages left
  uint32_t in_mask;                   // this step's proposer inputs left (Tick / response links)
  // wheel slots holding due bits, twice (bits k and W + k): the slots from
  // any step on are one bit-field extract
  uint32_t occ;
  static constexpr uint32_t OCC1 = 1u | (1u << W);
  static_assert(2 * W <= 32, "doubled wheel occupancy");
  // proposer states (ClientState, Client.hs:58-67), packed (tickets < 2^12,
  // commands = clientId, acks <= N/2 + 1):
  //   pw0 = ticket [11:0] | mr_t [23:12] | acks [27:24] | state [29:28] | pending [30]
  //   pw1 = mr_v [1:0] | r2_v [3:2] | cmd [5:4]
  uint32_t pw0[PM], pw1[PM];
  uint32_t pw2[PM];                   // LG: the t of the proposer's own command (0: Nothing)
  uint32_t skew[PM];                  // the (next) Tick step of each proposer
  uint32_t tk_end[PM];                // LG: its last Tick step
  uint32_t tper;                      // LG: steps between Ticks
  uint32_t nsent[PM];                 // broadcasts of p whose copies have started (request-link seq)
  uint32_t bnext[PM];                 // next broadcast-ring slot
  // ring-slot reference counts, 4-bit nibbles: one 32- or 64-bit word for
  // every proposer when they fit (nibble p * BR + slot: an add, no one-hot
  // select), else a word each
  static constexpr bool RPK = PM * S::BR * 4 <= 64;
  using ref_t = typename std::conditional<(PM * S::BR * 4 > 32), unsigned long long, uint32_t>::type;
  ref_t refp;
  uint32_t refc[RPK ? 1 : PM];
  // acceptor states (Server.hs:24-31), isolation windows, log digests
  uint32_t accw[N], win[N], accd[N];
  uint32_t accv[LG ? N : 1];          // LG: the stored command and log length of each acceptor
  // SL: the reply seqs, a byte per request link: four links a word, or (RSA:
  // three proposers) a word per acceptor, byte p, so that the selects share the
  // acceptor's one-hot masks with its state words (2 VGPRs more)
  static constexpr bool RSA = SL && PM == 3;
  static constexpr int NRS = RSA ? N : (NLQ + 3) / 4;
  uint32_t rseqv[SL ? NRS : 1];
  uint32_t pq, pq_len, acur;          // pending broadcasts (p << 3 | slot, 5 bits each), next acceptor
  // pending broadcasts at the head of pq made at step s - 1 (carried over by
  // end_op: at most one, or two on the simple schedule, CARRY2)
  // (CARRY2, opt-in: two broadcasts carried over on the simple schedule.
  // Host model, config 4: 0.4 % fewer iterations -- the carried copies then
  // hold up the next step instead -- for 5 more VALU per iteration: not used)
#ifdef PXB_EV_CARRY2
  static constexpr bool CARRY2 = SP && EARLY;
#else
  static constexpr bool CARRY2 = false;
#endif
  // (a count only with CARRY2: a lane-mask bool is one scalar op to update)
  typename std::conditional<CARRY2, uint32_t, bool>::type pqo;
  uint32_t canon0;                    // canon on entering a step that carries one over (else canon - 1)
  pool_mask_t pfree;                  // free response-pool words
  uint32_t lflags, rounds, dval, dtick, execs, msgs, canon;   // (msgs: the replies; see msgs_sent)
  unsigned long long clog;            // canonical log, 2-bit values (divergence check, SEMANTICS §7)
  uint32_t clog_len;
  bool bailed;

  // (slim: bit e for pool word e - 1, bit 0 unused)
  __host__ __device__ static constexpr pool_mask_t full_pool() {
    return (POOL == 8 * (int)sizeof(pool_mask_t)) ? ~(pool_mask_t)0
                                                   : (pool_mask_t)((((pool_mask_t)1 << (POOL % (8 * sizeof(pool_mask_t)))) - 1u) << S::POOLB_SHIFT);
  }
  static_assert(POOL + S::POOLB_SHIFT <= 8 * (int)sizeof(pool_mask_t), "pool mask");

  // ---- selects over per-proposer / per-acceptor register arrays (index may differ per lane) ----
  // The operands go through an empty asm: otherwise LLVM folds the select
  // chain into one load at a selected offset, and the dynamic offset keeps
  // the whole lane state in scratch memory instead of VGPRs.
  __host__ __device__ static __forceinline__ uint32_t opaque(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    __asm__("" : "+v"(x));
#endif
    return x;
  }
  // keeps a rarely taken branch a branch: SimplifyCFG's speculation would
  // otherwise run its body as selects in every iteration
  __host__ __device__ static __forceinline__ void opaque_barrier() {
#if defined(__HIP_DEVICE_COMPILE__)
    __asm__ volatile("");
#endif
  }
  // Selects by a per-lane index q over a small register array, as bit
  // operations on the one-hot word 1 << q: element i's lane mask is bit i of
  // it sign-extended (one v_bfe_i32), merged with v_bfi_b32.  A compare per
  // element would hold one 64-bit SGPR mask each, live across the step: for
  // the N-acceptor arrays that pushed ~70 SGPRs into VGPR spill slots.
  // (in asm: LLVM folds the bit form back into compares + v_cndmask)
  template <int I>
  __host__ __device__ static __forceinline__ uint32_t lane_mask(uint32_t onehot) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    __asm__("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(onehot), "i"(I));
    return r;
#else
    return (uint32_t)(((int32_t)(onehot << (31 - I))) >> 31);
#endif
  }
  __host__ __device__ static __forceinline__ uint32_t bfi(uint32_t mk, uint32_t x, uint32_t y) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(PXB_EV_BITOP3_BFI)
    // (v_bitop3_b32 with the bitwise-select table, 0xCA, as a builtin: no
    // s_nop before each dependent select, but LLVM then adds copies around it;
    // MI355X A/B: config 4 -7 %, config 3 -1 %: not used)
    return __builtin_amdgcn_bitop3_b32(mk, x, y, 0xCA);
#elif defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    __asm__("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mk), "v"(x), "v"(y));
    return r;
#else
    return (mk & x) | (~mk & y);
#endif
  }
  template <int K, int I = 1>
  __host__ __device__ static __forceinline__ uint32_t get_from(const uint32_t (&v)[K], uint32_t oh, uint32_t r) {
    if constexpr (I < K) return get_from<K, I + 1>(v, oh, bfi(lane_mask<I>(oh), v[I], r));
    else return r;
  }
  template <int K>
  __host__ __device__ static __forceinline__ uint32_t get(const uint32_t (&v)[K], uint32_t q) {
    return get_from<K>(v, 1u << q, v[0]);
  }
  template <int K, int I = 0>
  __host__ __device__ static __forceinline__ void set_from(uint32_t (&v)[K], uint32_t oh, uint32_t x) {
    if constexpr (I < K) {
#if defined(__HIP_DEVICE_COMPILE__)
      // (the element's new value in its own register, a tied operand: LLVM
      // otherwise gave some loop-carried elements a second register and
      // copied them back at the loop's end)
      __asm__("v_bfi_b32 %0, %1, %2, %0" : "+v"(v[I]) : "v"(lane_mask<I>(oh)), "v"(x));
#else
      v[I] = bfi(lane_mask<I>(oh), x, v[I]);
#endif
      set_from<K, I + 1>(v, oh, x);
    }
  }

  // element q := x for every lane (a lane that keeps its element passes the
  // old value): the same one-hot masks as get(v, q), which LLVM then shares
  template <int K>
  __host__ __device__ static __forceinline__ void put(uint32_t (&v)[K], uint32_t q, uint32_t x) {
    set_from<K>(v, 1u << q, x);
  }

  // the reference-count nibble of q's ring slot k, and adding d to it
  __host__ __device__ __forceinline__ uint32_t ref_nib(uint32_t q, uint32_t k) const {
    return RPK ? (uint32_t)(refp >> (4u * (q * (uint32_t)S::BR + k))) & 15u : (get(refc, q) >> (4u * k)) & 15u;
  }
  // (d: 1, 0 or ~0u = -1)
  __host__ __device__ __forceinline__ void ref_add(uint32_t q, uint32_t k, uint32_t d) {
    if constexpr (RPK) refp += (ref_t)(typename std::make_signed<ref_t>::type)(int32_t)d << (4u * (q * (uint32_t)S::BR + k));
    else put(refc, q, get(refc, q) + (d << (4u * k)));
  }

  // a value as the reference's command code (id << 24) | t (SEMANTICS §2)
  __host__ __device__ static __forceinline__ uint32_t code_of(uint32_t v) {
    return LG ? (((v >> 12) << 24) | (v & 0xFFFu)) : ((v << 24) | 1u);
  }

  // fields of the packed proposer state of p (finish, trace)
  __host__ __device__ uint32_t p_ticket(int p) const { return pw0[p] & 0xFFFu; }
  __host__ __device__ uint32_t p_mr_t(int p) const { return (pw0[p] >> 12) & 0xFFFu; }
  __host__ __device__ uint32_t p_acks(int p) const { return (pw0[p] >> 24) & 15u; }
  __host__ __device__ uint32_t p_state(int p) const { return (pw0[p] >> 28) & 3u; }
  __host__ __device__ uint32_t p_pending(int p) const { return (pw0[p] >> 30) & 1u; }
  __host__ __device__ uint32_t p_mr_v(int p) const { return pw1[p] & 3u; }
  __host__ __device__ uint32_t p_r2_v(int p) const { return (pw1[p] >> 2) & 3u; }
  __host__ __device__ uint32_t p_cmd(int p) const { return (pw1[p] >> 4) & 3u; }

  // broadcast ring slot `slot` of proposer q: halfword `half` of word `word`
  // (two proposers: one word per slot, the proposer picks the half)
  __host__ __device__ static __forceinline__ uint32_t bring_word(uint32_t q, uint32_t slot) {
    if (PM == 2) return slot;
    return q * (S::BR / 2u) + (slot >> 1);
  }
  __host__ __device__ static __forceinline__ uint32_t bring_half(uint32_t q, uint32_t slot) {
    if (PM == 2) return q;
    return slot & 1u;
  }
  __host__ __device__ __forceinline__ uint32_t rsp_ld(uint32_t Lr) const {
    return S::RH ? m.ldh(S::RSP, Lr) : m.ld(S::RSP + Lr);
  }
  __host__ __device__ __forceinline__ void rsp_st(uint32_t Lr, uint32_t v) const {
    if constexpr (S::RH) m.sth(S::RSP, Lr, v);
    else m.st(S::RSP + Lr, v);
  }

  // the Tick bits of step t
  __host__ __device__ __forceinline__ uint32_t ticks_at(int32_t t) const {
    uint32_t r = 0u;
#pragma unroll
    for (int p = 0; p < PM; ++p) r |= ((uint32_t)p < P && skew[p] == (uint32_t)t) ? (1u << (p * (N + 1))) : 0u;
    return r;
  }

  // enter step t: its due links from the wheel, its Ticks;
  // 48 canonical bytes per proposer with an input (SEMANTICS §8)
  __host__ __device__ __forceinline__ void enter(int32_t t) {
    s = t;
    pqo = CARRY2 ? pq_len : (pq_len != 0u);          // (at most one, CARRY2 two: end_op)
    if constexpr (!SP) canon0 = pqo ? canon : canon - 1u;   // (SP: see end_op)
    const uint32_t slot = (uint32_t)t & WM;
    uint32_t wq, wi;
    if (S::WW == 1) {
      const uint32_t wv = m.ld(S::WHEEL + slot);
      wq = wv & ((1u << NLQ) - 1u);
      wi = wv >> S::ISH;
    } else {
      wq = m.ld(S::WHEEL + 2u * slot);
      wi = m.ld(S::WHEEL + 2u * slot + 1u);
      m.st(S::WHEEL + 2u * slot + 1u, 0u);
    }
    m.st(S::WHEEL + S::WW * slot, 0u);
    occ &= ~(OCC1 << slot);
    acc_mask = wq;
    // Ticks only up to the last skew
    uint32_t tk = 0u;
    PXB_EV_PROBE(EVP_TICK_ENTER, t <= last_tick);
    if (!SP && any_lane(t <= last_tick)) {          // (single decree: the first steps only; SP: init)
      opaque_barrier();
      tk = (t <= last_tick) ? ticks_at(t) : 0u;
      if constexpr (LG) {                            // the next Tick of each proposer that ticked
#pragma unroll
        for (int p = 0; p < PM; ++p)
          skew[p] = (((tk >> (p * (N + 1))) & 1u) && skew[p] < tk_end[p]) ? skew[p] + tper : skew[p];
      }
    }
    in_mask = wi | tk;
#pragma unroll
    for (int p = 0; p < PM; ++p) {
      const uint32_t grp = ((1u << S::IW) - 1u) << (p * S::IW);
      canon += (in_mask & grp) ? 48u : 0u;
    }
  }

  // the launch's Philox round keys, once per wave: as VGPRs they cost no
  // per-round key arithmetic, and (unlike 20 SGPRs) push nothing into spills
  __host__ __device__ __forceinline__ void set_keys(const EvParams& kp) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
#if defined(PXB_EV_SGPR_KEYS) && defined(__HIP_DEVICE_COMPILE__)
      // (A/B: the keys as SGPRs)
      uint32_t a = kp.k0 + (uint32_t)r * 0x9E3779B9u, b = kp.k1 + (uint32_t)r * 0xBB67AE85u;
      __asm__ volatile("" : "+s"(a));
      __asm__ volatile("" : "+s"(b));
      rk[2 * r] = a;
      rk[2 * r + 1] = b;
#else
      rk[2 * r] = opaque(kp.k0 + (uint32_t)r * 0x9E3779B9u);
      rk[2 * r + 1] = opaque(kp.k1 + (uint32_t)r * 0xBB67AE85u);
#endif
    }
  }
  __host__ __device__ __forceinline__ uint4 draw(uint32_t c2, uint32_t c3) const {
    return philox_rk(lo, hi, c2, c3, rk);
  }

  // the isolation window of acceptor a of global instance (lo, hi) given its
  // draw w (SEMANTICS §4): c0 | c1 << 16, both clamped to 4096 (0: none)
  __host__ __device__ static __forceinline__ uint32_t window_of(const EvParams& kp, const uint4& w, uint32_t crash_m1) {
    uint32_t c0 = 0, c1 = 0;
    if (w.x <= crash_m1) {
      c0 = mulhi_n(w.y, kp.crash_start_max + 1u);
      c1 = c0 + 1u + mulhi_n(w.z, kp.crash_len_max);
    }
    c0 = c0 < 4096u ? c0 : 4096u;
    c1 = c1 < 4096u ? c1 : 4096u;
    return c0 | (c1 << 16);
  }

  // ---- instance start: parameters, Tick skews, isolation windows (SEMANTICS §4) ----
  __host__ __device__ __forceinline__ void init(const EvParams& kp, uint32_t g) {
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
      const uint4 w = draw(0u, 4u << 24);
      P = 1u + mulhi_n(w.x, kp.n_prop);
      const uint64_t lt = ev_threshold(mulhi_n(w.y, kp.loss_ppm + 1u));
      dmax = 1u + mulhi_n(w.z, kp.delay_max);
      const uint64_t ct = ev_threshold(mulhi_n(w.w, kp.crash_ppm + 1u));
      lossy = lt != 0ull;
      loss_m1 = (uint32_t)(lt - 1ull);
      crashy = ct != 0ull;
      crash_m1 = (uint32_t)(ct - 1ull);
    }
    // (slim two-proposer shape, config 5's first launch: a fuzzed P above the
    // shape's is handed on right here when no lane of the refill keeps its
    // instance, so a third of its instances skip the rest of init.  Only
    // there: in every shape, the same code cost configs 3 and 4 1.5 %)
    if constexpr (SL && PM < 3) {
      if ((kp.cfg & EV_CFG_RANDOMIZE) && !any_lane(P <= (uint32_t)PM)) {
        bailed = true;
        mode = M_RUN;
        return;
      }
    }
    uint4 wsk = make_uint4(0, 0, 0, 0);
    if (kp.skew_max > 0u) wsk = draw(0u, 2u << 24);
    last_tick = 0;
    tper = kp.tick_period;
#pragma unroll
    for (int p = 0; p < PM; ++p) {
      const uint32_t wp = (p == 0) ? wsk.x : (p == 1) ? wsk.y : wsk.z;
      skew[p] = (kp.skew_max > 0u && (uint32_t)p < P) ? mulhi_n(wp, kp.skew_max + 1u) : 0u;
      // log mode: n_ticks Ticks tick_period apart (SEMANTICS §9)
      tk_end[p] = LG ? skew[p] + (kp.n_ticks - 1u) * kp.tick_period : skew[p];
      const int32_t lt = (int32_t)(((uint32_t)p < P) ? tk_end[p] : 0u);
      last_tick = (lt > last_tick) ? lt : last_tick;
      pw0[p] = pw1[p] = pw2[p] = 0u;               // ticket 0, Idle, no command (Client.hs:90-95)
      nsent[p] = bnext[p] = 0u;
      refc[RPK ? 0 : p] = 0u;
      refp = 0u;
    }
#pragma unroll
    for (int a = 0; a < N; ++a) {
      win[a] = crashy ? window_of(kp, draw(0u, (3u << 24) | (uint32_t)a), crash_m1) : 0u;
      accw[a] = 0u;
      if constexpr (LG) accv[a] = 0u;
      accd[a] = 0x811C9DC5u;
    }
#pragma unroll
    for (int i = S::REQ; i < S::POOLW; ++i) m.st(i, 0u);   // request links, reply seqs, response links (RH: below)
    if constexpr (S::RH) {                           // (halfword rows shared with the other lanes' words)
#pragma unroll
      for (int i = 0; i < NLQ; ++i) m.sth(S::RSP, i, 1u);   // empty: the sentinel
    }
    if constexpr (SL) {
#pragma unroll
      for (int i = 0; i < NRS; ++i) rseqv[i] = 0u;
    }
#pragma unroll
    for (int i = 0; i < W * S::WW; ++i) m.st(S::WHEEL + i, 0u);
    pq = pq_len = acur = 0u;
    pqo = 0;
    pfree = full_pool();
    lflags = rounds = dval = dtick = execs = msgs = canon = 0u;
    clog = 0ull;
    clog_len = 0u;
    occ = 0u;
    // a fuzzed instance with more proposers than this shape holds goes to the
    // general kernel (config 5 runs its P <= 2 instances here: pxb_run_device)
    bailed = P > (uint32_t)PM;
    mode = M_RUN;
    enter(0);
    if constexpr (SP) {
      // Skew-free single decree: every proposer's only Tick is at step 0; it
      // is handled here (handleTick, Client.hs:196-207: Idle -> Round1 with
      // ticket 1, command c<id>, AskForTicket broadcast), so the proposer op
      // never sees one.  Its copies go out over the next iterations in the
      // order the proposer op would have queued them (proposer 0 first).
#pragma unroll
      for (int p = 0; p < PM; ++p) {
        if ((uint32_t)p < P) {
          canon += 48u;                              // (the Tick: a proposer input of step 0)
          pw0[p] = 1u | (ROUND1 << 28);
          pw1[p] = ((uint32_t)p + 1u) << 4;
          broadcast((uint32_t)p, ASK, 1u, 0u, true, 1u, false, 0u);
        }
      }
      in_mask = 0u;
    }
  }

  // The handler's broadcasts (kind0, x0, z0) [and the restart's AskForTicket
  // x1, Client.hs:185, only after an Execute] by proposer q: bookkeeping of
  // bcast() (oracle) and pending entries whose N copies go out over the next
  // iterations.  Payloads go to the next ring slots of q.
  __host__ __device__ __forceinline__ void broadcast(uint32_t q, uint32_t kind0, uint32_t x0, uint32_t z0, bool p0,
                                                     uint32_t x1, bool p1, uint32_t val) {
    rounds += ((p0 & (kind0 == ASK)) ? 1u : 0u) + (p1 ? 1u : 0u);
    const bool ex = p0 & (kind0 == EXECUTE);
    execs += ex ? 1u : 0u;
    const bool first = ex & (dval == 0u);             // the decided value: first Execute (Client.hs:178)
    dval = first ? val : dval;
    dtick = first ? x0 : dtick;
    const uint32_t slot0 = get(bnext, q), slot1 = (slot0 + 1u) & (S::BR - 1u);
    // a ring slot still referenced by a queued copy
    // (non-short-circuit: || here became two exec-mask branches)
    bailed = bailed | (p0 & (ref_nib(q, slot0) != 0u)) | (p1 & (ref_nib(q, slot1) != 0u));
    PXB_EV_PROBE(EVB_RING, (p0 & (ref_nib(q, slot0) != 0u)) | (p1 & (ref_nib(q, slot1) != 0u)));
    PXB_EV_PROBE(EVP_BCAST, p0);
    if (p0) {                                        // (p1 only with p0)
      if constexpr (LG && !PXB_EV_STORE_BACK) {
        m.st(S::BRING + q * S::BR + slot0, x0 | (z0 << 12) | (kind0 << 30));
        if (p1) m.st(S::BRING + q * S::BR + slot1, x1 | (ASK << 30));
      } else if constexpr (!LG && !PXB_EV_STORE_BACK) {
        m.st16h(S::BRING + bring_word(q, slot0), bring_half(q, slot0), x0 | (z0 << 12) | (kind0 << 14));
        if (p1) m.st16h(S::BRING + bring_word(q, slot1), bring_half(q, slot1), x1 | (ASK << 14));
      }
    }
    if constexpr (LG && PXB_EV_STORE_BACK) {       // (the same with the log mode's payload words)
      const uint32_t w0a = S::BRING + q * S::BR + slot0, w1a = S::BRING + q * S::BR + slot1;
      const uint32_t o0 = m.ld(w0a), o1 = m.ld(w1a);
      m.st(w0a, p0 ? x0 | (z0 << 12) | (kind0 << 30) : o0);
      m.st(w1a, p1 ? x1 | (ASK << 30) : o1);
    }
    if constexpr (!LG && PXB_EV_STORE_BACK) {
      // (without a branch: a lane that makes no broadcast stores the slots'
      // halfwords back; slot1 = slot0 + 1 mod BR, so the two never alias)
      const uint32_t w0a = S::BRING + bring_word(q, slot0), h0a = bring_half(q, slot0);
      const uint32_t w1a = S::BRING + bring_word(q, slot1), h1a = bring_half(q, slot1);
      const uint32_t o0 = m.ld16h(w0a, h0a), o1 = m.ld16h(w1a, h1a);
      m.st16h(w0a, h0a, p0 ? x0 | (z0 << 12) | (kind0 << 14) : o0);
      m.st16h(w1a, h1a, p1 ? x1 | (ASK << 14) : o1);
    }
    pq |= (p0 ? ((q << 3) | slot0) << (5u * pq_len) : 0u) | (p1 ? ((q << 3) | slot1) << (5u * pq_len + 5u) : 0u);
    const uint32_t nb = (p0 ? 1u : 0u) + (p1 ? 1u : 0u);
    pq_len += nb;
    put(bnext, q, (slot0 + nb) & (S::BR - 1u));
  }

  // the next copy of the oldest pending broadcast, on link cp -> ca (Philox
  // seq = the broadcast index, the link's seq: every broadcast tries every acceptor)
  __host__ __device__ __forceinline__ bool copy_ready() const { return pq_len != 0u; }
  // the acceptor's reply, handed to send_first: link, pool word (without its
  // due), proposer-input bit
  struct Reply {
    bool snd;
    uint32_t Lr, pw, bit;
    uint32_t z;                       // LG: the Round1OK's command (the pool's halfword array)
  };

  // The iteration's first send, on draw w: the acceptor's reply on link
  // a -> p (response FIFO + pool word) when there is one, else the next copy
  // of the oldest pending broadcast (request FIFO); one code path for both.
  __host__ __device__ __forceinline__ void send_first(const EvParams& kp, const uint4& w, const Reply& rp,
                                                     bool act = true) {
    const bool isR = rp.snd;                         // (only with act: acc_op)
    // the copy's bookkeeping (as in copy_send)
    const uint32_t sb = (uint32_t)s - (pqo ? 1u : 0u);
    const bool csnd = act & !isR & (pq_len != 0u);
    const uint32_t ce = pq & 31u;
    const uint32_t cp = ce >> 3, cslot = ce & 7u, ca = acur;
    const uint32_t ck = get(nsent, cp);
    {
      const uint32_t a1 = acur + 1u;
      const bool wrap = csnd & (a1 == (uint32_t)N);
      acur = wrap ? 0u : (csnd ? a1 : acur);
      pq = wrap ? pq >> 5 : pq;
      pq_len -= wrap ? 1u : 0u;
      if constexpr (CARRY2) pqo -= (wrap & (pqo != 0u)) ? 1u : 0u;
      else pqo = pqo & !wrap;
      put(nsent, cp, ck + (wrap ? 1u : 0u));
    }
    const bool snd = isR | csnd;
    PXB_EV_PROBE(EVP_SEND1, snd);
    const bool ok = !(kLossy & lossy & (w.x <= loss_m1));
    const uint32_t d = 1u + mulhi_n(w.y, dmax);
    const bool go = snd & ok;
    const uint32_t base = isR ? (uint32_t)s : sb;   // the send step (a carried copy's is s - 1)
    const uint32_t b4 = base & 15u;
    const uint32_t Lq = mulc<PM>(ca) + cp;
    // (a Round2Success in a compact link word needs no pool word)
    const bool r2c = S::RCODE & isR & ((rp.pw >> 30) == R2S);
    const uint32_t k2 = (POOL > 32) ? (uint32_t)__builtin_ctzll((unsigned long long)pfree | (1ull << 63))
                                    : ctz32((uint32_t)pfree) & 31u;
    uint32_t due_rel, due4;
    if constexpr (S::RH) {
      // Halfword response links (layout 7): both link words are loaded (the
      // request word of the copy, the response halfword of the reply) and
      // both are stored back, so no halfword is extracted from a shared word.
      // A response halfword holds its entries (pool index + 1, or a
      // Round2Success code) from bit 0 and a sentinel bit above the last
      // (empty: 1), so its highest set bit gives the tail's offset (+ 5)
      // and the append position.
      const uint32_t wq = m.ld(S::REQ + Lq);
      const uint32_t h = rsp_ld(rp.Lr);
      const uint32_t msb = 31u - (uint32_t)__builtin_clz(h | 1u);   // (h >= 1: the sentinel)
      const uint32_t te = (h >> ((msb - (uint32_t)S::IB) & 31u)) & IM;   // (empty: >> 27 = 0)
      // (a Round2Success code carries its due & 7; a code's or an empty link's pool load is unused)
      const bool tcode = S::RCODE && te >= S::RCB;       // (without codes every entry is a pool word's)
      const uint32_t tp = (m.ld(S::POOLB + ((S::TE_SAFE || !tcode) ? te : 0u)) >> 26) & 15u;
      const uint32_t rtail = tcode ? te & 7u : tp;
      const uint32_t qlen = (wq >> S::QL) & QLM;
      const uint32_t qtail = (wq >> (((uint32_t)S::EB * qlen - (uint32_t)S::DB) & 31u)) & DM;
      const uint32_t nz = isR ? h - 1u : qlen;           // (0: the link is empty)
      // (a code's due is mod 8: RCODE only on the 4-step wheel, DM = 7; log
      // mode's pool dues and request dues are mod 16)
      constexpr uint32_t RM = S::RCODE ? 7u : 15u;
      static_assert(!S::RCODE || DM == 7u, "codes on the 4-step wheel");
      const uint32_t rel = ((isR ? rtail : qtail) - b4) & (nz ? (isR ? RM : DM) : 0u);
      due_rel = d > rel ? d : rel;
      due4 = (b4 + due_rel) & 15u;
      // (as integers: a select of two booleans became five instructions)
      const uint32_t pool_out = ((pfree == 0) & !r2c) ? 1u : 0u;
      const uint32_t full = isR ? (h >> (S::IB * S::RC)) | pool_out : qlen >> 2;   // (QC = 4, qlen <= 4)
      static_assert(S::QC == 4, "request FIFOs of 4");
      bailed = bailed | (go & (full != 0u));
      PXB_EV_PROBE(EVB_RFIFO, go & isR & (h >= (1u << (S::IB * S::RC))));
      PXB_EV_PROBE(EVB_POOL, go & isR & (pfree == 0) & !r2c);
      PXB_EV_PROBE(EVB_QFIFO, go & !isR & (qlen >= (uint32_t)S::QC));
      // the pool word: to a free entry (harmless unless a reply goes), or, with
      // none free, to the request word, which the next store rewrites
      m.st(pfree ? S::POOLB + k2 : S::REQ + Lq, rp.pw | (due4 << 26));
      if constexpr (LG) {                            // (entry k2 = pool index + 1; no free entry: the dummy halfword)
        const uint32_t zi = pfree ? k2 - 1u : (uint32_t)POOL;
        m.st16h(S::POOLZ + (zi >> 1), zi & 1u, rp.z);
      }
      const uint32_t ent = r2c ? S::RCB + (due4 & 7u) : k2;
      // (the entry replaces the sentinel, the sentinel moves up one entry)
      const uint32_t nR = h + ((ent + (1u << S::IB) - 1u) << msb);
      const uint32_t nQ = wq + (1u << S::QL) + ((cslot | ((due4 & DM) << S::SB)) << ((uint32_t)S::EB * qlen));
      m.st(S::REQ + Lq, (go & !isR) ? nQ : wq);
      rsp_st(rp.Lr, (go & isR) ? nR : h);
    } else {
      const uint32_t lw = isR ? S::RSP + rp.Lr : S::REQ + Lq;   // the link word
      const uint32_t wv = m.ld(lw);
      uint32_t rlen, rtail;
      if constexpr (S::RZ) {                         // (the tail entry's pool word holds its due)
        rlen = (nbits32(wv) + (uint32_t)S::IB - 1u) / (uint32_t)S::IB;
        const uint32_t te = (wv >> ((S::IB * rlen - S::IB) & 31u)) & (isR ? IM : 0u);
        rtail = (m.ld(S::POOLB + te) >> 26) & 15u;
      } else {
        rlen = (wv >> S::RL) & RLM;
        rtail = (wv >> S::RD) & 15u;
      }
      // (both links' fields in plain variables, then selects: clang made the
      // selects over expressions branches, with the tail's pool load inside)
      const uint32_t qlen = (wv >> S::QL) & QLM;
      // (a request entry's due is mod 2^DB: every queued due lies within 2^DB of the send step)
      const uint32_t qtail = (wv >> (((uint32_t)S::EB * qlen - (uint32_t)S::DB) & 31u)) & DM;
      const uint32_t len = isR ? rlen : qlen;
      const uint32_t tail = isR ? rtail : qtail;
      const uint32_t lm = isR ? 15u : DM;
      const uint32_t rel = (tail - b4) & (len ? lm : 0u);
      due_rel = d > rel ? d : rel;
      due4 = (b4 + due_rel) & 15u;
      // (as integers, as in the halfword path)
      const uint32_t pool_out = ((pfree == 0) & !r2c) ? 1u : 0u;
      const uint32_t rfull = (rlen >= (uint32_t)S::RC) ? 1u : 0u, qfull = (qlen >= (uint32_t)S::QC) ? 1u : 0u;
      const uint32_t full = isR ? rfull | pool_out : qfull;
      bailed = bailed | (go & (full != 0u));
      PXB_EV_PROBE(EVB_RFIFO, go & isR & (len >= (uint32_t)S::RC));
      PXB_EV_PROBE(EVB_POOL, go & isR & (pfree == 0) & !r2c);
      PXB_EV_PROBE(EVB_QFIFO, go & !isR & (len >= (uint32_t)S::QC));
      // the pool word: to a free entry (harmless unless a reply goes), or, with
      // none free, to the link word, which the next store rewrites
      m.st(pfree ? S::POOLB + k2 : lw, rp.pw | (due4 << 26));
      if constexpr (LG) {                            // (no free entry: the dummy halfword)
        const uint32_t zi = pfree ? k2 : (uint32_t)POOL;
        m.st16h(S::POOLZ + (zi >> 1), zi & 1u, rp.z);
      }
      const uint32_t ent = r2c ? S::RCB + (due4 & 7u) : k2;
      // (entries above a FIFO's length are 0: appends are additions)
      constexpr int RD = S::RZ ? 0 : S::RD;         // (no due field in a slim >18-link word)
      const uint32_t nR = S::RZ ? wv | (ent << ((S::IB * len) & 31u))
                                : ((wv + (1u << S::RL) + (ent << (S::IB * len))) & ~(15u << RD)) | (due4 << RD);
      const uint32_t nQ = wv + (1u << S::QL) + ((cslot | ((due4 & DM) << S::SB)) << ((uint32_t)S::EB * len));
      m.st(lw, go ? (isR ? nR : nQ) : wv);
    }
    pfree &= (go & isR & !r2c) ? ~((pool_mask_t)1 << k2) : ~(pool_mask_t)0;
    ref_add(cp, cslot, (go & !isR) ? 1u : 0u);
    // a carried copy due now joins this step's due links, the rest the wheel
    const bool now = EARLY & !isR & (base + due_rel == (uint32_t)s);
    const uint32_t slot = (base + due_rel) & WM;
    m.orw(S::WHEEL + slot * S::WW + ((S::WW == 2 && isR) ? 1u : 0u), (go & !now) ? 1u << (isR ? rp.bit : Lq) : 0u);
    occ |= (go & !now) ? (OCC1 << slot) : 0u;
    acc_mask |= (go & now) ? (1u << Lq) : 0u;
  }

  // the Philox counter words of the next copy (seq = the broadcast's index on
  // its proposer, tag = (proposer, acceptor))
  __host__ __device__ __forceinline__ uint2 copy_ctr() const {
    const uint32_t cp = (pq & 31u) >> 3;
    return make_uint2(get(nsent, cp), (1u << 24) | (cp << 8) | acur);
  }
  __host__ __device__ __forceinline__ void copy_send(const EvParams& kp, bool act, const uint4& w) {
    // the broadcast's own step: s, or s - 1 for one carried over by end_op
    const uint32_t sb = (uint32_t)s - (pqo ? 1u : 0u);
    const uint32_t s4 = sb & 15u;
    const bool snd = act & (pq_len != 0u);
    PXB_EV_PROBE(EVP_COPY, snd);
    const uint32_t ce = pq & 31u;
    const uint32_t cp = ce >> 3, cslot = ce & 7u, ca = acur;
    const uint32_t ck = get(nsent, cp);
    {                                                // (branch-free: selects, no exec-mask branches)
      const uint32_t a1 = acur + 1u;
      const bool wrap = snd & (a1 == (uint32_t)N);    // the broadcast's last copy
      acur = wrap ? 0u : (snd ? a1 : acur);
      pq = wrap ? pq >> 5 : pq;
      pq_len -= wrap ? 1u : 0u;
      if constexpr (CARRY2) pqo -= (wrap & (pqo != 0u)) ? 1u : 0u;
      else pqo = pqo & !wrap;
      put(nsent, cp, ck + (wrap ? 1u : 0u));
    }
    // (w: the draw of copy_ctr() taken before this call)
    const bool ok = !(kLossy & lossy & (w.x <= loss_m1));
    const uint32_t d = 1u + mulhi_n(w.y, dmax);      // (delay_max <= 1: always 1)
    // enqueue (predicated: inactive lanes store to the dummy word)
    const bool go = snd & ok;
    const uint32_t Lq = mulc<PM>(ca) + cp;
    const uint32_t wq = m.ld(S::REQ + Lq);
    const uint32_t qlen = (wq >> S::QL) & QLM;
    bailed = bailed | (go & (qlen >= (uint32_t)S::QC));
    PXB_EV_PROBE(EVB_QFIFO, go & (qlen >= (uint32_t)S::QC));
    const uint32_t rel = (((wq >> (((uint32_t)S::EB * qlen - (uint32_t)S::DB) & 31u)) & DM) - s4) & (qlen ? DM : 0u);   // tail's due - sb
    const uint32_t due_rel = d > rel ? d : rel;
    const uint32_t ent = cslot | (((s4 + due_rel) & DM) << S::SB);
    // (inactive lanes store their word back unchanged)
    // (entries above the length are 0: a pop shifts zeros in; a full FIFO bails)
    m.st(S::REQ + Lq, go ? wq + (1u << S::QL) + (ent << ((uint32_t)S::EB * qlen)) : wq);
    ref_add(cp, cslot, go ? 1u : 0u);
    // due at s (a carried-over copy with the shortest delay): straight into
    // this step's due links, else into the wheel
    const bool now = EARLY & (sb + due_rel == (uint32_t)s);
    const uint32_t slot = (sb + due_rel) & WM;
    m.orw(S::WHEEL + slot * S::WW, (go & !now) ? 1u << Lq : 0u);
    occ |= (go & !now) ? (OCC1 << slot) : 0u;
    acc_mask |= (go & now) ? (1u << Lq) : 0u;
  }

  // One iteration: the proposer part, a copy, the acceptor part, another
  // copy (when the acceptor sent no reply), the step end; returns true when
  // the instance ended (outputs in o).  Two Philox draws per iteration: the
  // copy's, and the reply's or else the second copy's (1.4 of the 3 sends an
  // iteration can make are used on average; that copy's counter is known
  // before the acceptor part, which does not touch the pending queue).
  // (act = false: an idle lane of the wave, every op predicated off: the
  // driver runs the iteration without an exec-mask branch around it)
  // (fin: called with the outputs inside the step end's finishing branch,
  // where the lane state is still live in its registers: the kernel stores
  // the outputs there)
  struct NoFin {
    __host__ __device__ void operator()(const EvOut&) const {}
  };
  template <class Fin = NoFin>
  __host__ __device__ __forceinline__ bool step(const EvParams& kp, EvOut& o, bool act = true, const Fin& fin = Fin()) {
    // The proposer input first, so its link and pool loads start the
    // iteration instead of waiting behind the acceptor op; a pop and an append
    // on one FIFO commute (bails may differ, and stay exact).  MI355X, 2^24
    // instances: config 3 +2.7 %, config 4 +1.3 %, config 5 +2.3 %.
    // The copy's counter is then known at the start too, so its Philox chain
    // overlaps the acceptor op (config 4 +1.7 %, config 3 +0.7 %, config 5 +0.9 %);
    // the copy before the proposer op measured 1-3 % slower.
    Reply rp;
    prop_op(kp, act);
    const uint2 c = copy_ctr();
    copy_send(kp, act, draw(c.x, c.y));
    // (taking the acceptor op's choice before the copy is exact too, and
    // measured 1.5-2.5 % slower)
    const uint32_t ready = acc_ready_mask();
    const uint4 w0 = acc_op(kp, act, copy_ctr(), rp, ready);
    send_first(kp, w0, rp, act);
    return end_op(kp, o, act, fin);
  }

  // ================= ACC: one due request (Server.hs:51-78) and its reply =================
  __host__ __device__ __forceinline__ bool acc_ready() const { return acc_ready_mask() != 0u; }
  // the due requests the acceptor op may take: while a carried-over broadcast
  // has copies left, only those of the acceptors it has reached (its copy to
  // acceptor a may be due now, and a takes its requests in (p, seq) order)
  __host__ __device__ __forceinline__ uint32_t acc_ready_mask() const {
#ifdef PXB_EV_OLD_READY
    return (EARLY & (pqo != 0)) ? acc_mask & ((1u << (acur * (uint32_t)PM)) - 1u) : acc_mask;
#else
    // (an acceptor it has not reached takes its requests from proposers up to
    // the broadcast's own: the copy, due now at the earliest, goes after them
    // on its link, and links of higher proposers come after it, SEMANTICS §6)
    // (PM = 2: all links, or the p = 0 ones, by pq's proposer bit 3 sign-extended)
    const uint32_t cp = (pq & 31u) >> 3;
    const uint32_t upto = (PM == 1) ? ~0u : (PM == 2) ? 0x55555555u | (uint32_t)((int32_t)(pq << 28) >> 31)
                                                      : (cp == 0u ? 0x49249249u : cp == 1u ? 0xDB6DB6DBu : ~0u);
    uint32_t ok = ((1u << (acur * (uint32_t)PM)) - 1u) | upto;
    if constexpr (CARRY2) {
      // (a second carried broadcast, whose copies all wait: no acceptor takes
      // requests of proposers above its own)
      const uint32_t c2 = (pq >> 8) & 3u;
      const uint32_t upto2 = (PM == 1) ? ~0u : (PM == 2) ? 0x55555555u | (uint32_t)((int32_t)(pq << 23) >> 31)
                                                         : (c2 == 0u ? 0x49249249u : c2 == 1u ? 0xDB6DB6DBu : ~0u);
      ok &= ((uint32_t)pqo > 1u) ? upto2 : ~0u;
    }
    return (EARLY & (pqo != 0)) ? acc_mask & ok : acc_mask;
#endif
  }
  // (ready: acc_ready_mask(); it could be taken before this iteration's copy:
  // a request that copy makes due now belongs to an acceptor it had not reached)
  __host__ __device__ __forceinline__ uint4 acc_op(const EvParams& kp, bool act, uint2 cc, Reply& rp,
                                                   uint32_t ready) {
    const uint32_t s4 = (uint32_t)s & 15u;
    const bool acc = act & (ready != 0u);
    PXB_EV_PROBE(EVP_ACC, acc);
    const uint32_t L = acc ? ctz32(ready) : 0u;
    const uint32_t a = L / (uint32_t)PM, p = L - a * (uint32_t)PM;
    const uint32_t wq = m.ld(S::REQ + L);
    // the reply's link sequence number
    const uint32_t kw = SL ? get(rseqv, RSA ? a : L >> 2) : 0u;
    const uint32_t ksh = 8u * (RSA ? p : (L & 3u));   // (its byte)
    const uint32_t kr = S::CMP ? (wq >> S::KSH) : SL ? (kw >> ksh) & 0xFFu : m.ld16(S::RSEQ, L);
    const uint32_t len = (wq >> S::QL) & QLM;
    const uint32_t bslot = wq & ((1u << S::SB) - 1u);
    // the popped word: entries shifted down one, length - 1 (fields above the
    // entries, length and reply seq, adjusted in place)
    const uint32_t rq2 = ((wq & ((1u << S::QL) - 1u)) >> S::EB) + ((wq & ~((1u << S::QL) - 1u)) - (1u << S::QL));
    const bool keep = (len > 1u) & (((wq >> (S::EB + S::SB)) & DM) == (s4 & DM));   // the next entry due now too
    acc_mask = (acc & !keep) ? (acc_mask & ~(1u << L)) : acc_mask;
    uint32_t kind, x, z;
    if constexpr (LG) {
      const uint32_t w32 = m.ld(S::BRING + p * S::BR + bslot);
      kind = w32 >> 30, x = w32 & 0xFFFu, z = (w32 >> 12) & 0x3FFFu;
    } else {
      const uint32_t w16 = m.ld16h(S::BRING + bring_word(p, bslot), bring_half(p, bslot));
      kind = w16 >> 14, x = w16 & 0xFFFu, z = (w16 >> 12) & 3u;
    }
    ref_add(p, bslot, acc ? ~0u : 0u);
    const uint32_t A = get(accw, a);
    const bool dead = ((A >> A_DEAD) & 1u) != 0u;
    const uint32_t wa = get(win, a);                 // isolated at s: c0 <= s < c1 (SEMANTICS §4)
    const bool isol = ((wa & 0xFFFFu) <= (uint32_t)s) & ((uint32_t)s < (wa >> 16));
    const bool live = acc & !dead & !isol;
    const uint32_t rb = (kind == PROPOSE) ? 12u : 8u;
    canon += acc ? (live ? 2u * rb + 32u : rb) : 0u;
    const uint32_t t_max = A & 0xFFFu;
    const uint32_t V = LG ? get(accv, a) : A;
    const uint32_t val = LG ? V & 0x3FFFu : (A >> 24) & 3u;
    uint32_t log_len = V >> A_LEN;
    const bool is_ask = live & (kind == ASK), is_prop = live & (kind == PROPOSE), is_exec = live & (kind == EXECUTE);
    const bool grant = is_ask & !(t_max >= x);                // Server.hs:56
    const bool accept = is_prop & (x == t_max);                 // :66 (equality, not >=)
    const bool hit = is_exec & (t_max == x);                    // :75
    const bool panic = hit & (val == 0u);                       // :76 (Q6)
    const bool run = hit & (val != 0u);                         // :77-78
    const uint32_t rz = grant ? val : 0u;             // LG: the Round1OK's command (rp.z)
    lflags |= panic ? (uint32_t)PXB_F_PANIC : 0u;
    PXB_EV_PROBE(EVP_RUN, run);
    if (__builtin_expect(run, 0)) {                  // executed <>= [c]: log, digest, divergence
      if (log_len >= A_LEN_MAX) bailed = true;
      PXB_EV_PROBE(EVB_LOG, log_len >= A_LEN_MAX);
      put(accd, a, fnv_u32(get(accd, a), code_of(val)));
      if constexpr (LG) {                            // the canonical log's first LOG_TRACK positions (LDS)
        // (straight-line: compare or append at position log_len, the halfword
        // stored back when neither; a position past LOG_TRACK only flags.
        // Log mode's Execute branch runs in 91 % of its wave-iterations, for
        // 4 % of the lanes: nested exec-mask branches cost every one of them)
        const bool trk = log_len < (uint32_t)PXB_LOG_TRACK;
        const uint32_t li = trk ? log_len : (uint32_t)PXB_LOG_TRACK - 1u;
        const bool seen = log_len < clog_len;
        const bool app = trk & !seen;
        uint32_t old;
        if constexpr (S::CLP) {
          // position li at bit 14 li of the packed words: a 64-bit window of
          // words w and w + 1 (the last position ends at bit 32 of word CLW - 1,
          // whose window is that word twice: stored high half first, low last)
          const uint32_t b = mulc<14>(li), w = b >> 5, sh = b & 31u;
          const uint32_t w1 = (w + 1u < (uint32_t)S::CLW) ? w + 1u : w;
          const uint32_t lo = m.ld(S::CLOG + w), hi = m.ld(S::CLOG + w1);
          const unsigned long long v = ((unsigned long long)hi << 32) | lo;
          old = (uint32_t)(v >> sh) & 0x3FFFu;
          const unsigned long long nv = app ? (v & ~(0x3FFFull << sh)) | ((unsigned long long)val << sh) : v;
          m.st(S::CLOG + w1, (uint32_t)(nv >> 32));
          m.st(S::CLOG + w, (uint32_t)nv);
        } else {
          const uint32_t cw = S::CLOG + (li >> 1), ch = li & 1u;
          old = m.ld16h(cw, ch);
          m.st16h(cw, ch, app ? val : old);
        }
        lflags |= (trk & seen & (old != val)) ? (uint32_t)PXB_F_LOG_DIVERGENCE : 0u;
        lflags |= trk ? 0u : (uint32_t)PXB_F_LOG_TRUNC;
        clog_len += app ? 1u : 0u;
      } else {
        if (log_len < clog_len) {
          if (((uint32_t)(clog >> (2u * log_len)) & 3u) != val) lflags |= PXB_F_LOG_DIVERGENCE;
        } else {
          clog |= (unsigned long long)val << (2u * log_len);
          clog_len += 1u;
        }
      }
      log_len += 1u;
    }
    // (a lane without a live request rebuilds its old word unchanged)
    uint32_t pw;                                     // the reply's response word
    if constexpr (LG) {
      // (as below: accw = t_max | t_store << 12 | dead << 24, accv = the
      // stored command | log length << 14; the Round1OK's command goes in rp.z)
      const uint32_t c_gr = (A & ~0xFFFu) | x, c_ac = (A & ~0xFFF000u) | (x << 12);
      const uint32_t c_rn = A & ~0xFFF000u, c_pn = A | (1u << A_DEAD);
      uint32_t An = panic ? c_pn : A;
      An = run ? c_rn : An;
      An = accept ? c_ac : An;
      An = grant ? c_gr : An;
      put(accw, a, An);
      const uint32_t v_ac = (V & ~0x3FFFu) | z, v_rn = (V & ~0x3FFFu) + (1u << A_LEN);
      uint32_t Vn = run ? v_rn : V;
      Vn = accept ? v_ac : Vn;
      put(accv, a, Vn);
      const uint32_t p_gr = x | (A & 0xFFF000u) | (R1OK << 30), p_hv = (A & 0xFFFu) | (HAVE << 30);
      constexpr uint32_t p_ac = R2S << 30;
      pw = accept ? p_ac : p_hv;
      pw = grant ? p_gr : pw;
    } else {
      // whole-word updates (candidates, then selects of plain values): grant
      // sets t_max; accept sets t_store and val; Execute clears them and
      // appends (log length + 1; a 32nd entry bailed above); panic sets dead.
      // A Round1OK carries (x, t_store, val), which sit in the reply's fields
      // at their acceptor-word offsets.
      const uint32_t c_gr = (A & ~0xFFFu) | x, c_ac = (A & 0xFC000FFFu) | (x << 12) | (z << 24);
      const uint32_t c_rn = (A & 0xFC000FFFu) + (1u << 27), c_pn = A | (1u << 26);
      uint32_t An = panic ? c_pn : A;
      An = run ? c_rn : An;
      An = accept ? c_ac : An;
      An = grant ? c_gr : An;
      put(accw, a, An);
      const uint32_t p_gr = x | (A & 0x03FFF000u) | (R1OK << 30), p_hv = (A & 0xFFFu) | (HAVE << 30);
      constexpr uint32_t p_ac = R2S << 30;
      pw = accept ? p_ac : p_hv;
      pw = grant ? p_gr : pw;
    }
    const bool snd1 = live & !is_exec;              // the reply, on link a -> p
    m.st(S::REQ + L, acc ? rq2 + ((S::CMP && snd1) ? 1u << S::KSH : 0u) : wq);

    // ================= the reply, on a -> p (SEMANTICS §5) =================
    // Philox seq = the link's reply count.  Sent before the proposer part so its
    // state dies early; the proposer part only pops due-now heads, so the order
    // of the two on one link does not matter.
    // (one draw: this reply's, or, without one, the next copy's: cc)
    const uint4 w1 = draw(snd1 ? kr : cc.x, snd1 ? (1u << 24) | (1u << 16) | (p << 8) | a : cc.y);
    msgs += snd1 ? 1u : 0u;
    bailed = bailed | (snd1 & (kr == (S::CMP ? (1u << S::KB) - 1u : SL ? 0xFFu : 0xFFFFu)));
    PXB_EV_PROBE(EVB_RSEQ, snd1 & (kr == (S::CMP ? (1u << S::KB) - 1u : SL ? 0xFFu : 0xFFFFu)));
    if constexpr (SL) put(rseqv, RSA ? a : L >> 2, kw + (snd1 ? 1u << ksh : 0u));
    else if constexpr (!S::CMP) m.st16(S::RSEQ, L, snd1 ? kr + 1u : kr);
    rp.snd = snd1;
    rp.Lr = p * (uint32_t)N + a;
    rp.pw = pw;
    rp.z = rz;
    rp.bit = S::ISH + (SP ? rp.Lr : mulc<N + 1>(p) + 1u + a);
    return w1;
  }

  // ================= PROP: one input of one proposer =================
  __host__ __device__ __forceinline__ bool prop_ready() const { return in_mask != 0u && pq_len + 2u <= PQ_CAP; }
  __host__ __device__ __forceinline__ void prop_op(const EvParams& kp, bool act) {
    const uint32_t s4 = (uint32_t)s & 15u;
    const bool pin = act & (in_mask != 0u) & (pq_len + 2u <= PQ_CAP);
    PXB_EV_PROBE(EVP_PROP, pin);
    {
      const uint32_t j = pin ? ctz32(in_mask) : 0u;
      // (SP: bit j is response link j; j / N as a multiply-shift, exact for j < 2^10)
      const uint32_t q = SP ? (j * ((65536u + N - 1u) / N)) >> 16 : j / (uint32_t)(N + 1);
      const uint32_t r = SP ? 1u : j - mulc<N + 1>(q);
      const bool resp = pin & (r != 0u);
      const uint32_t ra = r - 1u;
      const uint32_t Lr = SP ? j : mulc<N>(q) + (resp ? ra : 0u);
      const uint32_t rr = rsp_ld(Lr);
      const uint32_t rlen = (rr >> S::RL) & RLM;
      // (RH: with one entry, nk is the sentinel: rkeep tests for a second entry)
      const uint32_t k = rr & IM, nk = (rr >> S::IB) & IM;
      // (a Round2Success code: no pool word, its due in the code)
      const bool kc = S::RCODE & (k >= S::RCB), nkc = S::RCODE & (nk >= S::RCB);
      // (a code's load is unused; with TE_SAFE every 5-bit entry indexes the lane's words)
      const uint32_t pe0 = m.ld(S::POOLB + ((S::TE_SAFE || !kc) ? k : 0u));
      const uint32_t pn = m.ld(S::POOLB + ((S::TE_SAFE || !nkc) ? nk : 0u));
      const uint32_t pe = kc ? (R2S << 30) : pe0;
      pfree |= (resp & !kc) ? ((pool_mask_t)1 << k) : (pool_mask_t)0;
      const uint32_t popped = S::RZ ? rr >> S::IB
                                    : ((rr & ((1u << S::RL) - 1u)) >> S::IB) + ((rr & ~((1u << S::RL) - 1u)) - (1u << S::RL));
      rsp_st(Lr, resp ? popped : rr);                // (popped: entries down one, length - 1)
      const bool nnow = nkc ? ((nk & 7u) == (s4 & 7u)) : (((pn >> 26) & 15u) == s4);
      const bool rkeep = resp & (S::RH ? rr >= (1u << (2 * S::IB)) : S::RZ ? nk != 0u : rlen > 1u) & nnow;
      in_mask = (pin & !rkeep) ? (in_mask & ~(1u << j)) : in_mask;
      const uint32_t rkind = pe >> 30, px = pe & 0xFFFu, py = (pe >> 12) & 0xFFFu;
      const uint32_t kz = k - (uint32_t)S::POOLB_SHIFT;   // (the pool index of entry k)
      const uint32_t pz = LG ? m.ld16h(S::POOLZ + ((kz >> 1) & 31u), kz & 1u) : (pe >> 24) & 3u;
      canon += resp ? 32u >> rkind : 0u;               // 2 x: Round1OK 16, HaveTicket 8, Round2Success 4

      const uint32_t w0 = get(pw0, q), w1 = get(pw1, q);
      const uint32_t T = w0 & 0xFFFu, MT = (w0 >> 12) & 0xFFFu, K = (w0 >> 24) & 15u, R = (w0 >> 28) & 3u;
      uint32_t MV, C2, CM, CT = 0u;
      if constexpr (LG) {                            // 14-bit commands; own command c<q+1>.<CT>
        CT = get(pw2, q);
        MV = w1 & 0x3FFFu, C2 = (w1 >> 14) & 0x3FFFu, CM = CT ? (((q + 1u) << 12) | CT) : 0u;
      } else {
        MV = w1 & 3u, C2 = (w1 >> 2) & 3u, CM = (w1 >> 4) & 3u;
      }
      {
        // The handlers (Client.hs:128-207) as whole-word updates of the packed
        // state: one select among the few outcomes instead of a select per
        // field (config 4: -1.8 % time against the field form, round 5)
        const uint32_t maj = (uint32_t)N >> 1;        // haveMajority: acks > floor(N/2), :191-194
        const uint32_t key = (pin ? ((!SP && r == 0u) ? 3u : rkind) : 4u) * 4u + R;
        const bool t_go = !SP && key == 3u * 4u + IDLE;                  // handleTick, :196-207
        const bool h_go = (key - (HAVE * 4u + ROUND1) < 2u) & (px >= T);  // HaveTicket, :128-140
        const bool o_go = (key == R1OK * 4u + ROUND1) & (T == px);        // Round1OK, :142-170
        const bool s_go = key == R2S * 4u + ROUND2;                      // Round2Success, :172-189 (Q2)
        const bool maj1 = K >= maj;                                      // acks + 1 > maj
        const bool o_take = (MV == 0u) | ((pz != 0u) & !(MT >= py));     // MostRecent (Common.hs:61-65)
        const uint32_t mv = o_take ? pz : MV;
        const bool o_maj = o_go & maj1, s_maj = s_go & maj1;
        const uint32_t PDb = w0 & (1u << 30);
        const bool sPD = s_maj & (PDb != 0u);                            // Execute + restart (:185)
        const bool ask = t_go | h_go;
        const bool restart = ask | sPD;                                  // -> Round1 with a new ticket
        const uint32_t Tn = (h_go ? px : T) + (restart ? 1u : 0u);
        const uint32_t C2n = o_maj ? ((mv == 0u) ? CM : mv) : C2;        // Q5: pending whenever mr is Just
        // pw0: restart: Tn, Round1, acks 0, mr_t 0, pending kept; Round2 entry:
        // T, acks 0, mr_t 0, pending = mr is Just; done (Idle): T and mr_t kept;
        // an ack below the majority: acks + 1 (Round1OK: mr_t := the MostRecent ticket)
        // (candidates first, then selects of plain values: clang emits a
        // conditional operator over larger expressions as branches)
        const uint32_t dmt = (py - MT) << 12;
        const uint32_t inc = (1u << 24) + ((o_go & o_take) ? dmt : 0u);
        const uint32_t pdo = (mv != 0u) ? 1u << 30 : 0u;
        const uint32_t c_rs = Tn | (ROUND1 << 28) | PDb, c_om = T | (ROUND2 << 28) | pdo;
        const uint32_t c_sd = w0 & 0xFFFFFFu, c_in = w0 + inc;
        uint32_t w0n = (o_go | s_go) ? c_in : w0;
        w0n = s_maj ? c_sd : w0n;
        w0n = o_maj ? c_om : w0n;
        w0n = restart ? c_rs : w0n;
        // pw1: mr_v := 0 (restart, Round2 entry) or the MostRecent value (an ack
        // below the majority); r2_v := C2n on Round2 entry; cmd := 0 when done,
        // c<id> on a Tick (LG: 14-bit mr_v | r2_v << 14, the command's t in pw2)
        constexpr uint32_t MVM = LG ? 0x3FFFu : 3u, C2S = LG ? 14u : 2u;
        const uint32_t tick_cm = (SP || LG) ? 0u : ((q + 1u) << 4);
        const uint32_t c1_rs = (!LG && t_go) ? (w1 & 0xCu) | tick_cm : w1 & ~MVM;
        const uint32_t c1_om = (LG ? 0u : (w1 & 0x30u)) | (C2n << C2S);
        const uint32_t c1_ok = (w1 & ~MVM) | mv, c1_sd = LG ? w1 : w1 & 0xFu;
        uint32_t w1n = s_maj ? c1_sd : w1;
        w1n = o_go ? c1_ok : w1n;
        w1n = o_maj ? c1_om : w1n;
        w1n = restart ? c1_rs : w1n;
        put(pw0, q, w0n);
        put(pw1, q, w1n);
        if constexpr (LG) put(pw2, q, t_go ? Tn : (s_maj & (PDb == 0u)) ? 0u : CT);   // handleTick: c<id>.<Tn>
        const uint32_t k0o = ask ? ASK : o_maj ? PROPOSE : s_maj ? EXECUTE : NONE;
        broadcast(q, k0o, ask ? Tn : T, C2n, k0o != NONE, Tn, sPD, C2n);
      }
    }
  }

  // ================= END of step: quiescence, step cap, next step =================
  // A step ends when its due messages and inputs are handled and its
  // broadcasts' copies are sent, except for the copies of one broadcast of
  // this step below the step cap: those go out during step s + 1 (next to
  // its own work), which is then the next step whatever else is due.  Their
  // delays are counted from s, so none is due before s + 1.
  __host__ __device__ __forceinline__ bool end_ready(const EvParams& kp) const {
    // (non-short-circuit: && / || here became a tree of exec-mask branches)
    // (CARRY2: the copies of two broadcasts of this step; a carried broadcast
    // is never carried again: its copies' delays count from its own step)
    const bool carry = EARLY & (pq_len <= (CARRY2 ? 2u : 1u)) & !pqo & ((uint32_t)s + 1u < kp.step_cap);
    return (acc_mask == 0u) & (in_mask == 0u) & ((pq_len == 0u) | carry);
  }
  template <class Fin = NoFin>
  __host__ __device__ __forceinline__ bool end_op(const EvParams& kp, EvOut& o, bool act, const Fin& fin = Fin()) {
    if (act && end_ready(kp)) {
      PXB_EV_PROBE(EVP_END, true);
      // (no message in flight: every queued one falls due after s and holds a
      // bit of its due step's wheel slot, which only entering that step clears)
      const bool quiet = (pq_len == 0u) & (occ == 0u) & (SP || s >= last_tick);
      // nothing but lost copies at a carried-over step: the instance was quiet at s - 1
      // (SP: never at a quiet step -- without loss, the carried copies sent
      // at s were handled at s (canonical bytes) or hold a wheel slot)
      const bool back = EARLY & !SP & (canon == canon0);
      // the next step with a due message or a Tick (skews of absent proposers are 0)
      const uint32_t s1 = (uint32_t)s + 1u;
      const uint32_t rot = (occ >> (s1 & WM)) & ((1u << W) - 1u);   // (occupied slots from s1 on)
      uint32_t nx = ((occ != 0u) & (pq_len == 0u)) ? s1 + ctz32(rot) : (pq_len ? s1 : 0xFFFFu);
      PXB_EV_PROBE(EVP_TICK_END, s < last_tick);
      if (!SP && any_lane(s < last_tick)) {           // (a later Tick: first steps only)
        opaque_barrier();
#pragma unroll
        for (int q = 0; q < PM; ++q) nx = ((skew[q] > (uint32_t)s) & (skew[q] < nx)) ? skew[q] : nx;
      }
      const bool capped = !quiet & (nx >= kp.step_cap);
      PXB_EV_PROBE(EVP_FIN, quiet | capped);
      if (__builtin_expect(quiet | capped, 0)) {
        s = capped ? (int32_t)kp.step_cap - 1 : (back ? s - 1 : s);
        finish(capped, o);
        fin(o);
        return true;
      }
      enter((int32_t)nx);
    }
    return false;
  }

  // messages sent by an ended instance: its replies plus N copies of every
  // broadcast, counted from nsent (an instance ends -- quiet or at the step
  // cap -- only with no broadcast left to send, end_op, so every broadcast
  // has sent its last copy and bumped nsent)
  __host__ __device__ __forceinline__ uint32_t msgs_sent() const {
    uint32_t b = 0u;
#pragma unroll
    for (int p = 0; p < PM; ++p) b += nsent[p];
    return msgs + b * (uint32_t)N;
  }

  // ---- outputs of an ended instance (SEMANTICS §7) ----
  __host__ __device__ __forceinline__ void finish(bool capped, EvOut& o) {
    const uint32_t steps = (uint32_t)s + 1u;
    uint32_t f = lflags | (capped ? (uint32_t)PXB_F_STEP_CAP : 0u) | (dval ? 0u : (uint32_t)PXB_F_UNDECIDED);
#pragma unroll
    for (int p = 0; p < PM; ++p)
      f |= (!capped && (uint32_t)p < P && p_state(p) != IDLE) ? (uint32_t)PXB_F_STUCK : 0u;
    canon += 16u + 4u * (uint32_t)N;
    o.res[0] = dval ? code_of(dval) : 0u;
    o.res[1] = dval ? dtick : 0u;
    o.res[2] = rounds;
    o.res[3] = (f & 0xFFu) | (steps << 16);
    o.flags = f;
    o.steps = steps;
    mode = M_IDLE;
  }

  // messages queued on the links (the trace's in_flight; the kernels test the wheel)
  __host__ __device__ uint32_t links_in_flight() const {
    uint32_t n = 0u;
    for (uint32_t L = 0; L < NLQ; ++L) {
      const uint32_t rw = rsp_ld(L);
      n += ((m.ld(S::REQ + L) >> S::QL) & QLM)
           + (S::RH ? (nbits32(rw) - 1u) / (uint32_t)S::IB
              : S::RZ ? (nbits32(rw) + (uint32_t)S::IB - 1u) / (uint32_t)S::IB : (rw >> S::RL) & RLM);
    }
    return n;
  }

  // final per-acceptor outputs (digest, record) of an ended instance
  __host__ __device__ uint32_t log_len_of(int a) const { return (LG ? accv[LG ? a : 0] : accw[a]) >> A_LEN; }
  // (single decree: log lengths < 32 fit the first byte, so FNV-1a over the
  // bytes (len, 0, 0, 0) is (h ^ len) * prime^4)
  __host__ __device__ uint32_t digest_of(int a) const {
    if constexpr (LG) {
      return fnv_u32(accd[a], log_len_of(a));
    } else {
      constexpr uint32_t P = 0x01000193u, P2 = P * P, P4 = P2 * P2;
      static_assert(A_LEN_MAX < 256, "one-byte log length");
      return (accd[a] ^ log_len_of(a)) * P4;
    }
  }
  __host__ __device__ void record_of(int a, uint32_t r[4]) const {
    const uint32_t A = accw[a];
    const uint32_t val = LG ? accv[LG ? a : 0] & 0x3FFFu : (A >> 24) & 3u;
    r[0] = A & 0xFFFu;
    r[1] = (A >> 12) & 0xFFFu;
    r[2] = val ? code_of(val) : 0u;
    r[3] = log_len_of(a) | (((A >> A_DEAD) & 1u) << 31);
  }
};

// EV eligibility of a launch (host side): single decree, faulty, 12-bit tickets,
// delays inside the 16-step wheel.  Fault-free and log-mode batches keep the
// paxos_kernel.h kernels.
__host__ inline bool eligible(const pxb_config* c) {
  // (log mode: the 8-step wheel layout only)
  return c->step_cap <= MAX_STEP_CAP && c->delay_max <= (c->n_ticks > 1 ? 8u : 15u);
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
  p.n_ticks = c->n_ticks > 1 ? c->n_ticks : 1u;
  p.tick_period = c->n_ticks > 1 ? c->tick_period : 1u;
  const uint64_t lt = ev_threshold(c->loss_ppm), ct = ev_threshold(c->crash_ppm);
  p.cfg = ((c->flags & PXB_CFG_RANDOMIZE) ? EV_CFG_RANDOMIZE : 0u) | (lt ? EV_CFG_LOSSY : 0u) | (ct ? EV_CFG_CRASHY : 0u);
  if ((c->flags & PXB_CFG_RANDOMIZE) || lt || c->delay_max > 1) p.cfg |= EV_CFG_DRAWS;
  p.loss_m1 = (uint32_t)(lt - 1ull);
  p.crash_m1 = (uint32_t)(ct - 1ull);
  return p;
}

// the timing wheel must outlast the longest delay: sends at step s (or s - 1
// for a carried-over copy) fall due in [s, s + delay_max] (a link's FIFO tail
// is at most its last send step + delay_max), the slot of s is emptied on
// entering s and a copy due at s goes straight to the step's due links, so
// the wheel holds dues in [s + 1, s + delay_max]: 8 slots serve delays up to 8
// (4 slots up to 4)
__host__ inline int wheel_for(uint32_t delay_max) { return delay_max <= 8 ? 8 : 16; }

// Kernel layout of a launch: 0 = 8-step wheel, 1 = 16-step wheel, 2 = compact
// links (3-entry request FIFOs sharing a word with the reply seq, a 24-word
// response pool, 8-step wheel).  Short delays keep FIFOs short (BASELINE
// config 4: 0.9 % of instances ever hold a fourth request on one link, config
// 3: 0.02 %; those are bailed to the general kernel), so they take the compact
// layout, which fits more resident waves; fuzzed or long-delay schedules keep
// 4-entry FIFOs.  The compact reply seq has 9 bits (config 4 reaches 68 in 256
// steps), so long runs keep the separate 16-bit one; three duelling proposers
// over 9 acceptors overflow the 3-entry FIFOs too often (25 % of instances at
// 10 % loss), so the compact layout is kept to topologies of <= 16 links.
// Layout 3 is the compact layout with a 4-step wheel (delays up to 4: BASELINE
// configs 3 and 4), 4 words per lane fewer.  Layout 5 is layout 0 slimmed
// (Shape::SL) for runs of at most 512 steps (BASELINE config 5).
__host__ inline int layout_for(const pxb_config* c) {
  if (c->n_ticks > 1) return 4;                      // log mode: 8-step wheel, 4-entry FIFOs, LG fields
  if (!(c->flags & PXB_CFG_RANDOMIZE) && c->delay_max <= 4 && c->step_cap <= 512 &&
      c->n_proposers * c->n_acceptors <= 16)
    return (c->loss_ppm == 0 && c->skew_max == 0) ? 6 : 3;   // 6: layout 3, simple schedule (Shape::SP)
  if (wheel_for(c->delay_max) != 8) return 1;
#ifndef PXB_EV_NO_SLIM
  if (c->step_cap <= 512) return 5;                  // slim: byte reply seqs suffice
#endif
  return 0;
}
__host__ inline int layout_wheel(int layout) {
  return (layout == 1 || layout == 8) ? 16 : (layout == 3 || layout == 6 || layout == 7 || layout == 9) ? 4 : 8;
}
__host__ inline bool layout_compact(int layout) { return layout == 2 || layout == 3 || layout == 6 || layout == 7; }
__host__ inline bool layout_simple(int layout) { return layout == 6 || layout == 7; }
// (8: layout 4 on the 16-step wheel with its topology's larger pool, the
// second stage of two-stage log mode, pxb_run_device)
// (9: layout 4 slimmed -- byte reply seqs in registers -- on the 4-step wheel,
// for log mode with delays <= 4 over <= 10 links: the first stage there)
__host__ inline bool layout_log(int layout) { return layout == 4 || layout == 8 || layout == 9; }

}  // namespace ev
}  // namespace pxb
