// paxos_kernel.h — the gfx950 batched ticket-Paxos kernel (device code).
//
// Replaces the reference's per-message actors (Server.hs:44-89 acceptor loop,
// Client.hs:85-111 proposer loop, spawned by Main.hs:41-46) with one GPU wave
// per group of independent instances:
//
//   * lane = (instance slot g, acceptor a): G = 64 / N instance slots per wave,
//     lanes g*N .. g*N+N-1 hold the N acceptors of one instance (SoA in VGPRs).
//     The kernel is VALU-issue bound (throughput saturates at 2-3 waves per
//     SIMD), so state stays unpacked and every hot-path instruction counts.
//   * each acceptor lane owns its directed links: the request queue from every
//     proposer p (p -> a) and the response queue to every proposer (a -> p),
//     PXB_QUEUE_DEPTH deep, as lane-interleaved LDS rings (bank-conflict free)
//     with the due steps nibble-packed in one register per link.
//   * the P proposers of an instance are replicated in all N lanes of its
//     slot.  Responses are folded in canonical (acceptor, link seq) order:
//     quorum counting with __ballot + popcount, the majority acceptor from a
//     prefix popcount, MostRecent (Common.hs:61-65) from a slot max-reduction;
//     a wave where some link holds 2+ due responses folds per-lane lists
//     instead (lane scans + slot prefix sums + DPP max).  Each lane enqueues
//     its own copy of a broadcast on its own link (Philox loss/delay per
//     link, in parallel).
//   * waves are persistent: when a slot's instance quiesces (or hits
//     step_cap) the slot writes its 16-B result + 4-B/acceptor digests and
//     refills from the wave's contiguous instance range.
//   * run totals: slot leaders count finished instances in packed 16-bit
//     per-lane counters, reduced once per wave when the wave exits.
//
// Semantics: docs/SEMANTICS.md; checked bit-exact against oracle/.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>

#include "../../include/paxos_batch.h"
#include "paxos_device.h"

namespace pxb {

constexpr int QD = PXB_QUEUE_DEPTH;   // 8: ring slots per directed link
constexpr int LT = PXB_LOG_TRACK;
static_assert(QD == 8, "due-nibble word and ring masks assume 8 slots");
static_assert(PXB_MAX_STEP_CAP <= 8192, "14-bit packed tickets / steps");
static_assert(PXB_TICKET_LIMIT <= (1 << 14), "the overflow flag must fire before a 14-bit ticket field wraps");
#ifndef PXB_OCC_P1
#define PXB_OCC_P1 4
#endif
#ifndef PXB_OCC_P1_FF
#define PXB_OCC_P1_FF 6   // measured on config 2: 4 -> 6 is +6 % (80 VGPRs, 12-wave blocks); 5 is 30 % slower
#endif
#ifndef PXB_OCC_P2
#define PXB_OCC_P2 4   // measured: 3 -> 4 is +10 % on configs 3, 4; 5, 6 no better
#endif
#ifndef PXB_OCC_P3
#define PXB_OCC_P3 3   // measured: 2 -> 3 is +25 % on config 5 (VGPRs fit 3 waves without spills)
#endif
// Faulty kernels hand out instances from a device work queue in chunks of
// QCHUNK (instance lengths vary from a few steps to step_cap, so a static
// split leaves the slowest waves running alone at the end).  One counter is
// enough: eight sub-queues with stealing measured no faster, and the
// fault-free kernels keep their static slices (a queue there costs 4x: every
// wave would hit the counter every ~12 steps).
#ifndef PXB_QCHUNK
#define PXB_QCHUNK 8    // measured: 8 = 16 > 32 > 64 > 256 on configs 3-5; under the
                        // iterative-ILP scheduler 8 is +2 % on config 5, +0.5 % on 3/4
#endif
constexpr uint32_t QCHUNK = PXB_QCHUNK;
// Run totals: each wave adds its counts into row (wave % TCOPIES) of a
// partial-totals block, and finalize_kernel (launched right after on the same
// stream) sums the rows into the caller's totals, zeroes them and resets the
// queue.  All waves adding into one 128-B row serialise at the L2: 4096 waves
// x 15 counters cost ~70-100 us per launch, a third of a config-2 launch.
constexpr uint32_t TCOPIES = 256;
// a wave flushes its packed 16-bit run totals after taking this many
// instances from the queue (a slot finishes at most that + QCHUNK + G since)
constexpr uint32_t FLUSH_EVERY = 30000;

// kp.cfg bit layout
constexpr uint32_t CFG_RANDOMIZE = 1u << 0;
constexpr uint32_t CFG_LOSSY = 1u << 1;     // loss threshold > 0
constexpr uint32_t CFG_CRASHY = 1u << 2;    // crash threshold > 0

struct KParams {
  uint64_t first_instance;
  uint32_t n_instances;               // this launch (host chunks larger batches)
  uint32_t k0, k1;                    // Philox key = seed
  uint32_t cfg;                       // CFG_*
  uint32_t n_prop, delay_max;
  uint32_t loss_m1, crash_m1;         // thr-1 (valid when LOSSY / CRASHY)
  uint32_t loss_ppm, crash_ppm;       // maxima for RANDOMIZE
  uint32_t crash_len_max, crash_start_max, skew_max, step_cap;
  uint32_t n_ticks, tick_period;      // log mode (LOGM kernels): Ticks per proposer, spacing
  uint4* out;                         // pxb_result records (nullable)
  uint32_t* dig;
  uint4* acc;
  unsigned long long* part;           // TCOPIES partial run-total rows (16 counters, 128 B each)
  uint32_t* queue;                    // faulty kernels: next instance, 0 on entry
  unsigned long long* dbg;            // diagnostic builds only (PXB_STAMPS)
  // faulty kernels only: run the instances listed in ids[0 .. *n_ids) (the
  // per-lane kernel's bailed instances, paxos_ev.h) instead of 0 .. n_instances;
  // a count above ids_cap means the list overflowed: run every instance
  const uint32_t* ids;
  const uint32_t* n_ids;
  uint32_t ids_cap;
};

__host__ __device__ inline uint64_t prob_threshold(uint32_t ppm) {
  return ((((uint64_t)ppm) << 32) + 999999ull) / 1000000ull;
}

// wave ballot straight from the lane predicate (HIP's __ballot(int) adds a
// bool -> int -> compare round trip per call)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; }

// compile-time loop: every per-proposer register index is a constant
template <int I, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < E) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, E>(f);
  }
}

// ---- diagnostic section stamps (separate build: -DPXB_STAMPS; never timed) --
#ifdef PXB_STAMPS
#define STAMP_DECL                                                \
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};                  \
  uint32_t st_cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};                  \
  uint64_t st_prev = __builtin_amdgcn_s_memtime();
#define SCOUNT(i) (st_cnt[i]++)
#define STAMP(i)                                                  \
  do {                                                            \
    __builtin_amdgcn_sched_barrier(0);                            \
    const uint64_t st_now = __builtin_amdgcn_s_memtime();         \
    __builtin_amdgcn_sched_barrier(0);                            \
    st_acc[i] += st_now - st_prev;                                \
    st_prev = st_now;                                             \
  } while (0)
#define STAMP_FLUSH(ptr)                                          \
  if (lane == 0 && (ptr)) {                                       \
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&(ptr)[i_], (unsigned long long)st_acc[i_]); \
    for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&(ptr)[8 + i_], (unsigned long long)st_cnt[i_]); \
  }
#else
#define STAMP_DECL
#define STAMP(i) do {} while (0)
#define SCOUNT(i) do {} while (0)
#define STAMP_FLUSH(ptr)
#endif

// ---- one directed link = LDS ring (payload) + 3 registers ------------------
// Every message is one 32-bit word:
//   request   x[13:0] | val[15:14] | kind[17:16]
//   response  x[13:0] | y[27:14]   | val[29:28] | kind[31:30]
// The due steps (mod 16) of the queued messages sit in one register as a
// nibble shift-queue, so "how many are due now" needs no LDS access.
struct Link {
  uint32_t dn;    // due&15 of entry i in bits [4i+3:4i], entry 0 = head
  uint32_t hl;    // len[3:0] | head[6:4] | 0[7] | last_due[31:8]
  uint32_t seq;   // sends attempted on this link (Philox counter word 2)
};
__device__ __forceinline__ uint32_t l_len(const Link& L) { return L.hl & 15u; }
__device__ __forceinline__ uint32_t l_head(const Link& L) { return (L.hl >> 4) & 7u; }
__device__ __forceinline__ int32_t l_last(const Link& L) { return (int32_t)(L.hl >> 8); }
// find-first-set-bit with the hardware's "none" value (v_ffbl_b32: ~0u for 0)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) { return x ? (uint32_t)__builtin_ctz(x) : ~0u; }
// number of entries at the head that are due at step s (due == s <=> nibble ==
// s&15, because every queued due lies in [s, s+15]); srep = (s&15) * 0x11111111
__device__ __forceinline__ uint32_t l_due_count(const Link& L, uint32_t srep) {
  return min(ffbl(L.dn ^ srep) >> 2, l_len(L));
}
// pop the head when `p`: len - 1, head + 1 (mod 8: the carry into bit 7 is cleared)
__device__ __forceinline__ void l_pop_if(Link& L, bool p) {
  L.dn = p ? (L.dn >> 4) : L.dn;
  L.hl = p ? ((L.hl + 15u) & ~0x80u) : L.hl;
}

// pop n <= len entries at once
__device__ __forceinline__ void l_pop_n(Link& L, uint32_t n) {
  L.dn = (n >= 8u) ? 0u : (L.dn >> (4u * n));
  L.hl = (L.hl & ~0x7Fu) | (((l_head(L) + n) & 7u) << 4) | (l_len(L) - n);
}

// Log mode (several Ticks per proposer, SEMANTICS §9) carries full commands
// "c<id>.<t>" (16 bits: id << 14 | t) instead of the single-decree clientId:
// a Round1OK then needs a second word, kept in a parallel ring.
template <int PM, bool LOGM> struct Ring2 { uint32_t w[PM][QD][64]; };
template <int PM> struct Ring2<PM, false> { uint32_t w[1][1][1]; };

// Canonical-log entry (epoch << CB | command).  Single decree: 2-bit clientId,
// 30-bit epochs.  Log mode: 16-bit commands; the fault-free kernels keep each
// wave's / block's instance range below 2^16 (host) so the entry fits 32 bits
// (half the LDS: config 6 goes from 7 to 9 resident waves per CU); the queue
// kernels' epochs need 32 bits and a 64-bit entry.
template <bool LOGM, bool FF> struct ClogFmt { using type = uint32_t; static constexpr uint32_t cb = 2u; };
template <> struct ClogFmt<true, true> { using type = uint32_t; static constexpr uint32_t cb = 16u; };
template <> struct ClogFmt<true, false> { using type = unsigned long long; static constexpr uint32_t cb = 32u; };

template <int PM, int N, bool LOGM, bool FF>
struct Lds {
  static constexpr int G = 64 / N;
  using clog_t = typename ClogFmt<LOGM, FF>::type;
  uint32_t rq[PM][QD][64];       // links p -> a   (lane-interleaved: conflict-free)
  uint32_t sq[PM][QD][64];       // links a -> p
  clog_t clog[G][LT + 1];        // per-slot canonical log (+1 pad: rows on distinct banks);
                                 // entries are (epoch << CB | command), epoch = instance tag
  Ring2<PM, LOGM> sq2;           // links a -> p, command word (log mode)
};

// command word -> the result encoding (clientId << 24) | t of "c<id>.<t>"
template <bool LOGM>
__device__ __forceinline__ uint32_t code32(uint32_t v) {
  if constexpr (LOGM) return v ? (((v >> 14) << 24) | (v & 0x3FFFu)) : 0u;
  else return v ? ((v << 24) | 1u) : 0u;
}

// occupancy target (waves per SIMD) by proposer count and schedule kind:
// bounds the VGPR budget (launch bounds) and the host's residency
template <int PM, bool FF> struct Occ {
  static constexpr int waves = PM == 1 ? (FF ? PXB_OCC_P1_FF : PXB_OCC_P1) : PM == 2 ? PXB_OCC_P2 : PXB_OCC_P3;
};

// Waves per block (LDS is carved per wave).  Faulty kernels: one wave per
// block, balanced by the device work queue.  Fault-free kernels: as many of a
// CU's waves as the LDS allows in one block (16 at 4 waves/SIMD), sharing the
// block's instance range through an LDS counter.  The SIMD arbiter favours
// older waves, so with a static slice per wave the waves of a SIMD finish up
// to 1.5x apart and the SIMD runs its tail with 1-3 waves; a shared range
// keeps all of them busy until the block's range is done.
constexpr int LDS_BYTES = 163840;
template <int PM, int N, bool LOGM, bool FF>
struct Shape {
  static constexpr int lds = (int)sizeof(Lds<PM, N, LOGM, FF>);
  static constexpr int occ = Occ<PM, FF>::waves;
  static constexpr int cap = 4 * occ;              // waves per CU at the occupancy target
#ifdef PXB_WPB
  static constexpr int wpb = PXB_WPB;
#else
  // waves resident per CU with w waves per block: whole blocks, LDS- and
  // target-limited
  static constexpr int resident(int w) {
    return (w * lds > LDS_BYTES) ? 0 : ((LDS_BYTES / (w * lds)) < (cap / w) ? (LDS_BYTES / (w * lds)) : (cap / w)) * w;
  }
  // the largest block (<= 16 waves) that keeps the most waves resident
  static constexpr int best() {
    int b = 1;
    for (int w = 2; w <= 16; ++w)
      if (resident(w) >= resident(b)) b = w;
    return b;
  }
  static constexpr int wpb = FF ? best() : 1;
#endif
  static constexpr int block = 64 * wpb;
};

// Philox with its inputs made opaque, so the compiler cannot hoist the
// per-instance half of the rounds (quarter-rate multiplies) out of the rare
// fault branch into every step.
__device__ __forceinline__ uint4 philox_here(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                             uint32_t k0, uint32_t k1) {
  asm volatile("" : "+v"(c0), "+v"(c1), "+s"(k0), "+s"(k1));
#ifdef PXB_PHILOX_TWICE_DIAG   // diagnostic: the marginal cost of the draws
  {
    uint32_t d0 = c0 ^ 1u;
    asm volatile("" : "+v"(d0));
    const uint4 w2 = philox(d0, c1, c2, c3, k0, k1);
    asm volatile("" ::"v"(w2.x), "v"(w2.y));
  }
#endif
  return philox(c0, c1, c2, c3, k0, k1);
}

// FF = fault-free schedule (no loss, delay 1, no crash windows, no fuzzing):
// every message is due exactly one step after it is sent, so a link's due
// count is its length (requests) or its length before this step's acceptor
// phase (responses), and no Philox draw, due-nibble or isolation test is needed.
template <int PM, int N, bool LOGM, bool FF>
__global__ __launch_bounds__((Shape<PM, N, LOGM, FF>::block), (Occ<PM, FF>::waves)) void paxos_batch_kernel(KParams kp) {
  constexpr int WPB = Shape<PM, N, LOGM, FF>::wpb;
  constexpr int G = 64 / N;
  constexpr uint32_t NM = (1u << N) - 1u;     // slot-local lane mask
  constexpr uint32_t ENONE = 16u;             // "no event" acceptor index (N <= 9 < 16)
  // command field of a request word: single decree = clientId (2 bits, t = 1),
  // log mode = id << 14 | t (16 bits); the kind sits above it
  constexpr uint32_t ZM = LOGM ? 0xFFFFu : 3u, KSH = LOGM ? 30u : 16u;
  using clog_t = typename Lds<PM, N, LOGM, FF>::clog_t;
  constexpr uint32_t CB = ClogFmt<LOGM, FF>::cb;   // epoch shift of a canonical-log entry
  // A lone proposer on a fault-free schedule is never NACKed (its tickets only
  // grow and nobody else raises T_max) and gets at most one response per link
  // per step, so the NACK handling and the multi-response fold compile out.
  constexpr bool CONTENDED = !(FF && PM == 1);
  __shared__ Lds<PM, N, LOGM, FF> s_lds[WPB];

  const int lane = threadIdx.x & 63;
  const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  Lds<PM, N, LOGM, FF>& L = s_lds[wib];
  const int g = lane / N;
  const int a = lane - g * N;
  const bool used = g < G;
  const int base = g * N;
  const uint32_t ltm = (1u << a) - 1u;        // slot-local lanes below me
  clog_t* clog = &L.clog[used ? g : 0][0];
  for (int k = lane; k < G * (LT + 1); k += 64) (&L.clog[0][0])[k] = 0u;   // epoch 0 = empty
  // a ballot restricted to my slot, as an N-bit mask indexed by acceptor
  auto slot = [&](uint64_t b) -> uint32_t { return (uint32_t)(b >> base) & NM; };   // unused lanes never act

  const uint32_t wave = blockIdx.x * WPB + wib;
  const uint32_t nwaves = gridDim.x * WPB;
  // faulty kernels may take their instances from a device-side list (its
  // length is written by the kernel launched before this one)
  const uint32_t n_listed = (!FF && kp.n_ids) ? (uint32_t)__builtin_amdgcn_readfirstlane((int)*kp.n_ids) : 0u;
  const bool listed = !FF && kp.n_ids && n_listed <= kp.ids_cap;
  const uint32_t n = listed ? n_listed : kp.n_instances;
  // an empty list (the usual case behind the per-lane kernels): leave at once,
  // before any wave touches the work queue (grid-uniform)
  if (listed && n == 0u) return;
  // faulty kernels: chunks from the device work queue (DYN); fault-free
  // kernels: one-generation chunks of the block's contiguous range from an
  // LDS counter (BQ); diagnostic builds: a static slice per wave
#ifdef PXB_STATIC_SPLIT
  constexpr bool DYN = false, BQ = false;
#else
  // (a one-wave block gains nothing from the LDS counter: measured 2 % slower)
  constexpr bool DYN = !FF, BQ = FF && WPB > 1;
#endif
  __shared__ uint32_t s_bq;
  const uint32_t blo = (uint32_t)((uint64_t)n * blockIdx.x / gridDim.x);
  const uint32_t bhi = (uint32_t)((uint64_t)n * (blockIdx.x + 1) / gridDim.x);
  if constexpr (BQ) {
    if (threadIdx.x == 0) s_bq = 0u;
    __syncthreads();
  }
  uint32_t next = (DYN || BQ) ? 0u : (uint32_t)((uint64_t)n * wave / nwaves);
  uint32_t end = (DYN || BQ) ? 0u : (uint32_t)((uint64_t)n * (wave + 1) / nwaves);
  // epoch tags of the canonical log (idx - first_idx + 1) must grow along a
  // slot's instances: both queues hand out chunks in increasing order
  const uint32_t first_idx = BQ ? blo : next;
  bool drained = false;                   // DYN: the queue is empty (wave-uniform)
  uint32_t grabbed = 0;                   // DYN: instances taken since the last flush (wave-uniform)
  const uint32_t k0 = kp.k0, k1 = kp.k1;
#ifdef PXB_WAVE_TIMES   // diagnostic: per-wave start / end (100 MHz constant clock)
  const uint64_t wt0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t wm0 = __builtin_amdgcn_s_memtime();
#endif

  // ---- slot state (replicated in the slot's lanes unless marked "lane") ----
  bool active = false;
  uint32_t P = 0, dmax = 1;
  bool faulty = false, lossy = false, tovf = false;
  int32_t last_tick = 0;
  int32_t s = 0;                          // current step
  uint32_t idx = 0;                       // local instance index (queue position)
  uint32_t gid = 0;                       // instance index within the launch (ids[idx] with a list)
  uint32_t loss_m1 = 0;
  uint32_t rounds = 0, dval = 0;          // dval: decided clientId (0 = none)
  int32_t dtick = 0;
  int32_t c0 = 0, c1 = 0;                 // lane: isolation window of acceptor a
  AccState A{0, 0, 0, false};             // lane: acceptor a (ServerState)
  uint32_t log_len = 0, lflags = 0, digest = 0;   // lane
  uint32_t canon = 0;                     // lane: canonical bytes of the current instance
  PropState S[PM];                        // replicated proposers (ClientState)
  int32_t skew[PM];
  int32_t ntick[PM];                      // log mode: step of proposer p's next Tick
  uint32_t tleft[PM];                     // log mode: Ticks still to come
  uint32_t execs = 0, execs_acc = 0;      // Execute broadcasts (commands committed)
  Link R[PM], Sx[PM];                     // lane: links p -> a, a -> p
  uint32_t msgs_acc = 0;                  // lane totals across instances
  uint64_t canon_acc = 0;
  // slot-leader run totals, two 16-bit counts per register (the host sizes
  // launches so no slot finishes 65536 instances):
  //   ca = instances | undecided<<16, cb = stuck | panic<<16,
  //   cc = divergence | step_cap<<16, cd = queue_ovf | ticket_ovf<<16, ce = log_trunc
  uint32_t ca = 0, cb = 0, cc = 0, cd = 0, ce = 0, rounds_acc = 0, steps_acc = 0;
#pragma unroll
  for (int p = 0; p < PM; ++p) {
    S[p] = PropState{0, 0, 0, IDLE, 0, 0, 0, 0, 0u};
    skew[p] = 0;
    ntick[p] = 0;
    tleft[p] = 0;
    R[p] = Link{0, 0, 0};
    Sx[p] = Link{0, 0, 0};
  }

  unsigned long long* const trow = kp.part + (size_t)(wave % TCOPIES) * 16u;
  // ---- run totals: wave reduction + one atomic per counter, counters zeroed
  auto flush_totals = [&]() {
    uint32_t v[14] = {ca & 0xFFFFu, ca >> 16, cb & 0xFFFFu, cb >> 16, cc & 0xFFFFu, cc >> 16,
                      cd & 0xFFFFu, cd >> 16, ce, rounds_acc, steps_acc, msgs_acc, execs_acc, 0u};
    uint64_t c64 = canon_acc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
      for (int q = 0; q < 13; ++q) v[q] += (uint32_t)__shfl_xor((int)v[q], off);
      const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)c64, off);
      const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(c64 >> 32), off);
      c64 += ((uint64_t)hi << 32) | lo;
    }
    if (lane < 14) {
      // lane q adds counter q (one atomic per lane, no serialisation within the wave)
      const int slot_of[14] = {PXB_C_INSTANCES, PXB_C_UNDECIDED, PXB_C_STUCK, PXB_C_PANIC, PXB_C_DIVERGENCE,
                               PXB_C_STEP_CAP, PXB_C_QUEUE_OVERFLOW, PXB_C_TICKET_OVERFLOW, PXB_C_LOG_TRUNC,
                               PXB_C_ROUNDS, PXB_C_STEPS, PXB_C_MESSAGES, PXB_C_EXECUTES, PXB_C_DECIDED};
      unsigned long long val = 0;
#pragma unroll
      for (int q = 0; q < 13; ++q) val = (lane == q) ? (unsigned long long)v[q] : val;
      if (lane == 13) val = (unsigned long long)v[0] - (unsigned long long)v[1];   // decided
#ifndef PXB_NO_TOTALS_DIAG   // diagnostic: the cost of the totals atomics
      if (val) atomicAdd(&trow[slot_of[lane]], val);
#endif
    }
#ifndef PXB_NO_TOTALS_DIAG
    if (lane == 14) atomicAdd(&trow[PXB_C_CANON_BYTES], (unsigned long long)c64);
#endif
    ca = cb = cc = cd = ce = rounds_acc = steps_acc = msgs_acc = execs_acc = 0u;
    canon_acc = 0ull;
  };

  // rare in-loop variant (every FLUSH_EVERY started instances): each lane adds
  // its own counts, no wave reduction (keeps register pressure off the loop)
  auto flush_lanes = [&]() {
    auto add = [&](int c, uint32_t v) {
      if (v) atomicAdd(&trow[c], (unsigned long long)v);
    };
    add(PXB_C_INSTANCES, ca & 0xFFFFu);
    add(PXB_C_UNDECIDED, ca >> 16);
    add(PXB_C_DECIDED, (ca & 0xFFFFu) - (ca >> 16));
    add(PXB_C_STUCK, cb & 0xFFFFu);
    add(PXB_C_PANIC, cb >> 16);
    add(PXB_C_DIVERGENCE, cc & 0xFFFFu);
    add(PXB_C_STEP_CAP, cc >> 16);
    add(PXB_C_QUEUE_OVERFLOW, cd & 0xFFFFu);
    add(PXB_C_TICKET_OVERFLOW, cd >> 16);
    ca = cb = cc = cd = 0u;
  };

  STAMP_DECL
  // common link send, predicated on `pred` (docs/SEMANTICS.md §5): Philox
  // loss/delay, FIFO due, bounded ring (overflow -> flag, message dropped);
  // returns whether the message was queued
  auto link_send = [&](Link& Lk, uint32_t* ring, uint32_t* ring2, uint32_t dirbits, uint32_t word,
                       uint32_t word2, bool pred) -> bool {
    msgs_acc += pred ? 1u : 0u;
    const uint32_t k = Lk.seq;
    Lk.seq = pred ? k + 1u : k;
    int32_t d = 1;
    bool ok = true;
#ifdef PXB_STAMPS
    if (!FF && any(pred && faulty)) SCOUNT(5);
#endif
    if (!FF && pred && faulty) {
      const uint64_t inst = kp.first_instance + gid;
      const uint4 w = philox_here((uint32_t)inst, (uint32_t)(inst >> 32), k, (1u << 24) | dirbits | (uint32_t)a, k0, k1);
      ok = !(lossy && w.x <= loss_m1);
      d = 1 + (int32_t)mulhi_n(w.y, dmax);
    }
    const uint32_t len = l_len(Lk);
    const bool full = len >= (uint32_t)QD;
    const bool push = pred && ok && !full;
    const bool ovf = pred && ok && full;
    if (any(ovf)) lflags |= ovf ? (uint32_t)PXB_F_QUEUE_OVERFLOW : 0u;
    const int32_t due = FF ? s + 1 : max(s + d, l_last(Lk));
    if (push) {
      const uint32_t at = ((l_head(Lk) + len) & 7u) * 64u + (uint32_t)lane;
      ring[at] = word;
      if (ring2) ring2[at] = word2;
    }
    if constexpr (FF) {
      Lk.hl = push ? Lk.hl + 1u : Lk.hl;        // no due bookkeeping: all due next step
    } else {
      Lk.dn = push ? (Lk.dn | (((uint32_t)due & 15u) << (4u * len))) : Lk.dn;
      Lk.hl = push ? (((Lk.hl & 0x7Fu) + 1u) | ((uint32_t)due << 8)) : Lk.hl;
    }
    return push;
  };
  // proposer p's broadcast copy on link p -> a (sendToAllServers, Client.hs:122-123)
  auto send_req = [&](auto pc, bool has, uint32_t kind, int32_t x, uint32_t z) {
    constexpr int p = decltype(pc)::value;
    rounds += (has && kind == ASK) ? 1u : 0u;
    const bool ex = has && kind == EXECUTE;
    if (any(ex)) {                      // a slot committed (Client.hs:178)
      execs += ex ? 1u : 0u;
      const bool first_exec = ex && dval == 0u;   // the decided value
      dval = first_exec ? S[p].r2_v : dval;
      dtick = first_exec ? x : dtick;
    }
    link_send(R[p], &L.rq[p][0][0], nullptr, (uint32_t)p << 8, (uint32_t)x | (z << 14) | (kind << KSH), 0u, has);
  };
  // one request from the head of link p -> a (Rl; the reply goes on Sl,
  // link a -> p), predicated on `due`: handleClientRequest, Server.hs:51-78
  // (dead / isolated acceptors discard it).  p may differ between lanes.
  auto acc_take = [&](Link& Rl, Link& Sl, uint32_t p, bool due, bool isolated) {
    const uint32_t w = (&L.rq[0][0][0])[(p * QD + l_head(Rl)) * 64u + (uint32_t)lane];
    l_pop_if(Rl, due);
    const uint32_t kind = (w >> KSH) & 3u;
    const bool live = due && !A.dead && !isolated;
    const uint32_t rb = 8u + ((kind & 1u) << 2);       // payload: Propose 12, Ask / Execute 8
    canon += live ? 2u * rb + 32u : (due ? rb : 0u);    // discarded: written, not read
    int32_t rx, ry;
    uint32_t rz, ev;
    const uint32_t rk = acceptor_step(A, live, kind, (int32_t)(w & 0x3FFFu), (w >> 14) & ZM, rx, ry, rz, ev);
    if (any(ev != 0u)) {
      if (ev != 0u) {
        digest = fnv_u32(digest, code32<LOGM>(ev));
        if (log_len < (uint32_t)LT) {
          // two acceptors of this instance executed different commands at
          // the same position iff the max already holds this epoch with
          // another command (order-independent, SEMANTICS §7)
          const clog_t tag = (clog_t)(idx - first_idx + 1u);
          const clog_t old = atomicMax(&clog[log_len], (tag << CB) | (clog_t)ev);
          if ((old >> CB) == tag && (uint32_t)(old & (((clog_t)1 << CB) - 1u)) != ev) lflags |= PXB_F_LOG_DIVERGENCE;
        } else {
          lflags |= PXB_F_LOG_TRUNC;
        }
        log_len++;
      }
    }
    // tickets are < 2^14 (SEMANTICS §6), so the fields need no masking
    // (log mode: the clientId field says Just / Nothing, the full command
    // travels in the second ring)
    const bool queued =
        link_send(Sl, &L.sq[0][0][0] + p * (QD * 64u), LOGM ? &L.sq2.w[0][0][0] + p * (QD * 64u) : nullptr,
                  (1u << 16) | (p << 8),
                  (uint32_t)rx | ((uint32_t)ry << 14) | ((LOGM ? (rz >> 14) : rz) << 28) | (rk << 30), rz,
                  rk != NONE);
    // a queued response is charged here as delivered (payload written + read,
    // Round1OK 16, HaveTicket 8, Round2Success 4 B): every queued response is
    // consumed before quiescence, and a step-capped instance gives back the
    // ones still queued when it stops
    canon += queued ? 2u * (16u >> (rk & 3u)) : 0u;
  };

  for (;;) {
    // ---------------- refill free slots from this wave's range -------------
    const uint64_t freeb = ballot(used && !active && a == 0);
    if (BQ && freeb != 0ull && next >= end && !drained) {
      uint32_t c = 0u;
      if (lane == 0) c = atomicAdd(&s_bq, (uint32_t)G);
      c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
      drained = c >= bhi - blo;
      next = drained ? next : blo + c;
      end = drained ? end : min(blo + c + (uint32_t)G, bhi);
    }
    if (DYN && freeb != 0ull && next >= end && !drained) {
      uint32_t c = 0u;
      if (lane == 0) c = atomicAdd(&kp.queue[0], QCHUNK);
      c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
      drained = c >= n;
      next = drained ? next : c;
      end = drained ? end : min(c + QCHUNK, n);
      grabbed += QCHUNK;
      if (grabbed >= FLUSH_EVERY) {   // keep the 16-bit slot counts below 2^16
        flush_lanes();
        grabbed = 0;
      }
    }
    if (freeb != 0ull && next < end) {
      const uint32_t cand = next + (uint32_t)__popcll(freeb & ((1ull << base) - 1ull));
      if (used && !active && cand < end) {
        idx = cand;
        gid = listed ? kp.ids[cand] : cand;
        const uint64_t inst = kp.first_instance + gid;
        const uint32_t ilo = (uint32_t)inst, ihi = (uint32_t)(inst >> 32);
        P = kp.n_prop;
        dmax = kp.delay_max;
        lossy = (kp.cfg & CFG_LOSSY) != 0u;
        bool crashy = (kp.cfg & CFG_CRASHY) != 0u;
        loss_m1 = kp.loss_m1;
        uint32_t crash_m1 = kp.crash_m1;
        if (!FF && (kp.cfg & CFG_RANDOMIZE)) {         // SEMANTICS §4 (config-5 fuzz)
          const uint4 w = philox(ilo, ihi, 0u, 4u << 24, k0, k1);
          P = 1u + mulhi_n(w.x, kp.n_prop);
          const uint64_t lt = prob_threshold(mulhi_n(w.y, kp.loss_ppm + 1u));
          dmax = 1u + mulhi_n(w.z, kp.delay_max);
          const uint64_t ct = prob_threshold(mulhi_n(w.w, kp.crash_ppm + 1u));
          lossy = lt != 0ull;
          loss_m1 = (uint32_t)(lt - 1ull);
          crashy = ct != 0ull;
          crash_m1 = (uint32_t)(ct - 1ull);
        }
        uint4 wsk = make_uint4(0, 0, 0, 0);
        if (kp.skew_max > 0u) wsk = philox(ilo, ihi, 0u, 2u << 24, k0, k1);
        last_tick = 0;
        static_for<0, PM>([&](auto pc) {
          constexpr int p = decltype(pc)::value;
          const uint32_t wp = (p == 0) ? wsk.x : (p == 1) ? wsk.y : wsk.z;
          skew[p] = (kp.skew_max > 0u) ? (int32_t)mulhi_n(wp, kp.skew_max + 1u) : 0;
          ntick[p] = skew[p];
          tleft[p] = kp.n_ticks;
          // the last Tick: skew + (n_ticks - 1) * period (single decree: skew)
          if ((uint32_t)p < P)
            last_tick = max(last_tick, skew[p] + (LOGM ? (int32_t)((kp.n_ticks - 1u) * kp.tick_period) : 0));
          S[p] = PropState{0, 0, 0, IDLE, 0, 0, 0, 0, 0u};
          R[p] = Link{0, 0, 0};
          Sx[p] = Link{0, 0, 0};
        });
        c0 = c1 = 0;
        if (!FF && crashy) {
          const uint4 w = philox(ilo, ihi, 0u, (3u << 24) | (uint32_t)a, k0, k1);
          if (w.x <= crash_m1) {
            c0 = (int32_t)mulhi_n(w.y, kp.crash_start_max + 1u);
            c1 = c0 + 1 + (int32_t)mulhi_n(w.z, kp.crash_len_max);
          }
        }
        faulty = lossy || dmax > 1u;
        tovf = false;
        A = AccState{0, 0, 0, false};
        log_len = lflags = 0;
        canon = 0;
        digest = 0x811C9DC5u;
        rounds = dval = execs = 0;
        dtick = 0;
        s = 0;
        active = true;
      }
      next = min(next + (uint32_t)__popcll(freeb), end);
    }
    if (!any(active)) break;
    SCOUNT(0);
#ifdef PXB_STAMPS
    uint32_t st_sr = 0;   // this slot's fold rounds over all proposers this step
    st_cnt[7] += (uint32_t)__popcll(ballot(active && a == 0));
#endif
    STAMP(0);

    const uint32_t srep = ((uint32_t)s & 15u) * 0x11111111u;
    // FF: the responses due now are exactly those queued before this step's
    // acceptor phase (the replies it sends are due next step)
    uint32_t sx_due[PM];
#pragma unroll
    for (int p = 0; p < PM; ++p) sx_due[p] = FF ? l_len(Sx[p]) : 0u;
    // ---------------- acceptor phase: (proposer index, link seq) order -------
    // handleClientRequest, Server.hs:51-78, for every due request of lane a,
    // one request per lane per iteration (predicated, no divergent branches)
    {
      const bool isolated = !FF && (c0 <= s) && (s < c1);
      if constexpr (PM == 1) {
        uint32_t cnt = active ? (FF ? l_len(R[0]) : l_due_count(R[0], srep)) : 0u;
        if (any(cnt > 0u)) {
          do {
            SCOUNT(1);
            acc_take(R[0], Sx[0], 0u, cnt > 0u, isolated);
            cnt = (cnt > 0u) ? cnt - 1u : 0u;
          } while (any(cnt > 0u));
        }
      } else {
        // every lane walks its own (p, seq) list, so the wave iterates
        // max over lanes of the lane's total, not the sum over p of per-link
        // maxima; the link of the current request is selected per lane
        uint32_t cn[PM];
        uint32_t left = 0;
#pragma unroll
        for (int p = 0; p < PM; ++p) {
          cn[p] = active ? (FF ? l_len(R[p]) : l_due_count(R[p], srep)) : 0u;
          left += cn[p];
        }
        if (any(left > 0u)) {
          do {
            SCOUNT(1);
            uint32_t ps = PM - 1;
#pragma unroll
            for (int p = PM - 2; p >= 0; --p) ps = (cn[p] != 0u) ? (uint32_t)p : ps;
            Link Rl = R[PM - 1], Sl = Sx[PM - 1];
#pragma unroll
            for (int p = 0; p < PM - 1; ++p) {
              Rl.dn = (ps == (uint32_t)p) ? R[p].dn : Rl.dn;
              Rl.hl = (ps == (uint32_t)p) ? R[p].hl : Rl.hl;
              Sl.dn = (ps == (uint32_t)p) ? Sx[p].dn : Sl.dn;
              Sl.hl = (ps == (uint32_t)p) ? Sx[p].hl : Sl.hl;
              Sl.seq = (ps == (uint32_t)p) ? Sx[p].seq : Sl.seq;
            }
            const bool due = left > 0u;
            acc_take(Rl, Sl, ps, due, isolated);
#pragma unroll
            for (int p = 0; p < PM; ++p) {
              const bool me = due && ps == (uint32_t)p;
              R[p].dn = me ? Rl.dn : R[p].dn;
              R[p].hl = me ? Rl.hl : R[p].hl;
              Sx[p].dn = me ? Sl.dn : Sx[p].dn;
              Sx[p].hl = me ? Sl.hl : Sx[p].hl;
              Sx[p].seq = me ? Sl.seq : Sx[p].seq;
              cn[p] -= me ? 1u : 0u;
            }
            left -= due ? 1u : 0u;
          } while (any(left > 0u));
        }
      }
    }
    STAMP(1);

    // ---------------- proposer phase: Tick, then (acceptor, link seq) order --
    static_for<0, PM>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      const bool pact = active && (uint32_t)p < P;
      bool stepped = false;
      // the ticker (Client.hs:96-100): one Tick at skew_p (single decree), or
      // n_ticks Ticks tick_period steps apart (log mode)
      const bool tick = LOGM ? (pact && tleft[p] != 0u && s == ntick[p]) : (pact && s == skew[p]);
      if (any(tick)) {                          // handleTick, Client.hs:196-207
        Req o0{NONE, 0, 0};
        uint32_t no = 0;
        if (tick) {
          // command "c<id>.<t>" with t the new ticket (Client.hs:200-203);
          // single decree: t = 1, carried as the clientId alone
          const uint32_t cmd = LOGM ? (((uint32_t)(p + 1) << 14) | (uint32_t)(S[p].ticket + 1)) : (uint32_t)(p + 1);
          no = proposer_tick(S[p], cmd, o0);
          stepped = true;
          if (LOGM) {
            ntick[p] += (int32_t)kp.tick_period;
            tleft[p] -= 1u;
          }
        }
        send_req(pc, no > 0u, o0.kind, o0.x, o0.z);
      }
      const uint32_t cnt_p = pact ? (FF ? sx_due[p] : l_due_count(Sx[p], srep)) : 0u;
      const uint64_t anyb = ballot(cnt_p > 0u);
      STAMP(2);
      if (anyb != 0ull) {
        const uint32_t mine_slot = slot(anyb);
        stepped = stepped || mine_slot != 0u;
        const bool slot_multi = slot(ballot(cnt_p > 1u)) != 0u;
        // ---- fast path: every link a -> p of the slot has <= 1 due response.
        // The serial fold of Client.hs:125-189 over acceptors 0..N-1 is done in
        // rounds, one per state-changing event (majority or NACK):
        // acks = __ballot + popcount, the majority acceptor = the lane whose
        // prefix popcount hits the quorum, MostRecent (Common.hs:61-65) = a
        // slot max-reduction of (t_store, -lane) over the counted acks.  After
        // an event only a NACK (not Idle) or a stale Round2Success (in Round2)
        // can still act: a fresh Round1OK for the new ticket cannot exist yet.
        // Every round is a select network (no divergent branches).
        // A wave with any multi slot runs every slot through the multi path
        // (it is exact for <= 1 response per link too): the slots of a wave
        // would otherwise pay for both paths.
        const bool wave_multi = CONTENDED && any(pact && slot_multi);
        const bool fast = pact && !wave_multi && mine_slot != 0u;
        if (any(fast)) {
          const bool has = fast && cnt_p == 1u;
          const uint32_t w = L.sq[p][l_head(Sx[p])][lane];
          const uint32_t w2 = LOGM ? L.sq2.w[p][l_head(Sx[p])][lane] : 0u;
          l_pop_if(Sx[p], has);
          const uint32_t kind = has ? (w >> 30) : 3u;       // 3: no response
          const int32_t x = (int32_t)(w & 0x3FFFu);
          const int32_t y = (int32_t)((w >> 14) & 0x3FFFu);
          const uint32_t z = has ? (LOGM ? w2 : ((w >> 28) & 3u)) : 0u;
          uint32_t rem = slot(ballot(has));                 // unprocessed responses
          const uint32_t havem = slot(ballot(kind == HAVE));
          const uint32_t r2sm = slot(ballot(kind == R2S));
          bool go = fast;
          do {
            SCOUNT(2);
#ifdef PXB_STAMPS
            st_sr += go ? 1u : 0u;
#endif
            PropState& Sp = S[p];
            const uint32_t rs = Sp.rs;
            const int32_t T = Sp.ticket;
            const bool mine = go && ((rem >> a) & 1u) != 0u;
            const bool is_ack = mine && ((rs == ROUND1 && kind == R1OK && x == T) ||
                                         (rs == ROUND2 && kind == R2S));
            const bool is_ab = CONTENDED && mine && rs != IDLE && kind == HAVE && x >= T;
            const uint32_t ackm = slot(ballot(is_ack));
            const uint32_t abm = slot(ballot(is_ab));
            const uint32_t need = (uint32_t)(N >> 1) + 1u - Sp.acks;
            const bool is_maj = is_ack && (uint32_t)__popc(ackm & ltm) + 1u == need;
            const uint32_t majm = slot(ballot(is_maj));
            const uint32_t e_ab = min(ffbl(abm), ENONE);
            const uint32_t e_mj = min(ffbl(majm), ENONE);
            const bool mj = e_mj < e_ab;                    // majority before any NACK
            const uint32_t e = min(e_ab, e_mj);
            // acks counted before the event (and the majority ack itself)
            const uint32_t counted = ackm & ((1u << (e + (mj ? 1u : 0u))) - 1u);
            // MostRecent over the counted Round1OKs that carry a proposal
            const bool elig = rs == ROUND1 && ((counted >> a) & 1u) != 0u && z != 0u;
            const uint32_t zb = slot(ballot(elig));
            uint32_t key = elig ? (((uint32_t)y << 5) | (31u - (uint32_t)a)) : 0u;
            uint32_t bz = 0;
            if (any(zb != 0u)) {              // some slot saw a stored proposal
              if (any(__popc(zb) > 1)) {
#pragma unroll
                for (int off = 1; off < N; off <<= 1) {
                  const uint32_t o = (uint32_t)__shfl((int)key, lane + off);
                  if (a + off < N) key = max(key, o);
                }
              }
              const int src = zb ? ((__popc(zb) > 1) ? base : base + __builtin_ctz(zb)) : lane;
              key = (uint32_t)__shfl((int)key, src);
              bz = (uint32_t)__shfl((int)z, zb ? base + 31 - (int)(key & 31u) : lane);
            }
            int32_t u = 0;
            if (any(abm != 0u)) u = __shfl(x, abm ? base + (int)e_ab : lane);
            // ---- the state transition of this round (Client.hs:128-189) ----
            int32_t mt = Sp.mr_t;
            uint32_t mv = Sp.mr_v;
            const bool take = zb != 0u && (mv == 0u || (int32_t)(key >> 5) > mt);
            mt = take ? (int32_t)(key >> 5) : mt;
            mv = take ? bz : mv;
            const bool ev = go && e != ENONE;
            const bool r1maj = go && mj && rs == ROUND1;    // Client.hs:157-170
            const bool r2maj = go && mj && rs == ROUND2;    // Client.hs:177-189
            const bool nack = ev && !mj;                    // Client.hs:130-140
            const bool restart = r2maj && Sp.pending;       // Client.hs:179-185
            const bool idle = r2maj && !Sp.pending;         // Client.hs:186-189
            const uint32_t r2v = (mv == 0u) ? Sp.cmd : mv;
            const int32_t tn = nack ? u + 1 : T + 1;
            // outputs: o0 (Propose / Execute / AskForTicket), o1 (AskForTicket on restart)
            const uint32_t k0o = r1maj ? PROPOSE : (r2maj ? EXECUTE : ASK);
            const int32_t x0o = nack ? tn : T;
            const uint32_t z0o = r1maj ? r2v : 0u;
            Sp.r2_v = r1maj ? r2v : Sp.r2_v;
            Sp.pending = r1maj ? (mv != 0u) : Sp.pending;
            Sp.ticket = (nack || restart) ? tn : T;
            Sp.cmd = idle ? 0u : Sp.cmd;
            Sp.acks = go ? (ev ? 0u : Sp.acks + (uint32_t)__popc(counted)) : Sp.acks;
            Sp.rs = r1maj ? ROUND2 : ((nack || restart) ? ROUND1 : (idle ? IDLE : rs));
            const bool keep_mr = go && !ev && rs == ROUND1;
            Sp.mr_t = keep_mr ? mt : (ev ? 0 : Sp.mr_t);
            Sp.mr_v = keep_mr ? mv : (ev ? 0u : Sp.mr_v);
            rem = ev ? rem & ~((2u << e) - 1u) : 0u;
            go = ev && Sp.rs != IDLE && (rem & (havem | (Sp.rs == ROUND2 ? r2sm : 0u))) != 0u;
            if (any(ev)) send_req(pc, ev, k0o, x0o, z0o);
            if (any(restart)) send_req(pc, restart, ASK, tn, 0u);
          } while (any(go));
        }
        STAMP(3);
        // ---- multi path (some link of the slot holds >= 2 due responses).
        // The canonical order is (acceptor a, link seq k); between events the
        // proposer only counts acks, so the fold runs in rounds again, now over
        // per-lane lists: every lane scans its own due responses (acks before
        // its first qualifying NACK), a slot prefix sum of those counts finds
        // the majority acceptor and the majority ack inside its list, the
        // first NACK lane cuts the rest, MostRecent is a max over
        // (t_store, -a, -k) of the counted proposals.  Same transitions as the
        // fast path (Client.hs:128-189); all due responses are consumed.
        const bool multi = pact && wave_multi && mine_slot != 0u;
        if (CONTENDED && any(multi)) {
          SCOUNT(3);
          const uint32_t h0 = l_head(Sx[p]);
          const uint32_t cntm = multi ? cnt_p : 0u;
          uint32_t kp = 0;                                   // next unprocessed response of my list
          bool go = multi;
#pragma unroll 1
          while (any(go)) {
            SCOUNT(4);
#ifdef PXB_STAMPS
            st_sr += go ? 1u : 0u;
#endif
            PropState& Sp = S[p];
            const uint32_t rs = Sp.rs;
            const int32_t T = Sp.ticket;
            // scan: acks before my first qualifying NACK (count and position
            // mask), that NACK, and the best MostRecent candidate among those
            // acks, key (t_store, -a, -k)
            const bool r1 = rs == ROUND1;
            uint32_t c = 0, nk = 0xFFu, ackb = 0, bkey = 0, bz = 0;
            int32_t ux = 0;
#pragma unroll 1
            for (uint32_t j = 0; any(go && kp + j < cntm && nk == 0xFFu); ++j) {
              const uint32_t k = kp + j;
              const bool v = go && k < cntm && nk == 0xFFu;
              const uint32_t w = L.sq[p][(h0 + k) & 7u][lane];
              const uint32_t kind = w >> 30;
              const int32_t x = (int32_t)(w & 0x3FFFu);
              const bool ack = v && ((r1 && kind == R1OK && x == T) || (rs == ROUND2 && kind == R2S));
              const bool nack = v && rs != IDLE && kind == HAVE && x >= T;
              c += ack ? 1u : 0u;
              ackb |= ack ? (1u << k) : 0u;
              ux = nack ? x : ux;
              nk = nack ? k : nk;
              const uint32_t zc = LOGM ? L.sq2.w[p][(h0 + k) & 7u][lane] : ((w >> 28) & 3u);
              const uint32_t key = (((w >> 14) & 0x3FFFu) << 8) | ((15u - (uint32_t)a) << 4) | (15u - k);
              const bool el = ack && r1 && zc != 0u && key > bkey;
              bkey = el ? key : bkey;
              bz = el ? zc : bz;
            }
            const uint32_t A = min(ffbl(slot(ballot(nk != 0xFFu))), ENONE);   // first NACK lane
            const uint32_t ce = ((uint32_t)a <= A) ? c : 0u;
            // inclusive prefix of ce over the slot's lanes (log-step shuffles)
            uint32_t incl = ce;
#pragma unroll
            for (int off = 1; off < N; off <<= 1) {
              const uint32_t o = (uint32_t)__shfl((int)incl, lane - off);
              incl += (a >= off) ? o : 0u;
            }
            const uint32_t excl = incl - ce;
            const uint32_t need = (uint32_t)(N >> 1) + 1u - Sp.acks;    // haveMajority, Client.hs:191-194
            const bool majl = go && ce != 0u && excl < need && need <= incl;
            const uint32_t M = min(ffbl(slot(ballot(majl))), ENONE);    // majority lane (<= A)
            const bool mj = M != ENONE;
            const uint32_t e = mj ? M : A;                              // event lane (ENONE: none)
            const uint32_t r = need - excl;                             // majority = my r-th ack
            // the majority ack's index: the r-th set bit of the ack mask
            // (r <= need <= N/2 + 1 <= 5)
            uint32_t bits = ackb;
#pragma unroll
            for (uint32_t i = 1; i < 5u; ++i) bits = (i < r) ? (bits & (bits - 1u)) : bits;
            const uint32_t kmaj = ffbl(bits);
            // MostRecent counts the acks of the lanes before the event lane (all
            // lanes when there is none) and of the event lane up to its majority
            // ack or its NACK (where the scan stopped).  Only an event lane with
            // acks after its majority ack needs a shorter candidate scan: it has
            // 2+ acks, which a Round1 list never holds (one Round1OK per Ask,
            // tickets strictly increase) but the fold stays exact regardless.
            const bool counted_lane = go && ((uint32_t)a < e || e == ENONE || (uint32_t)a == e);
            const bool redo = go && r1 && mj && (uint32_t)a == e && c > r;
            bkey = counted_lane ? bkey : 0u;
            if (any(redo)) {
              uint32_t rk2 = 0, rz2 = 0;
#pragma unroll 1
              for (uint32_t j = 0; any(redo && kp + j <= kmaj); ++j) {
                const uint32_t k = kp + j;
                const bool v = redo && k <= kmaj && ((ackb >> k) & 1u) != 0u;
                const uint32_t w = L.sq[p][(h0 + k) & 7u][lane];
                const uint32_t zc = LOGM ? L.sq2.w[p][(h0 + k) & 7u][lane] : ((w >> 28) & 3u);
                const uint32_t key = (((w >> 14) & 0x3FFFu) << 8) | ((15u - (uint32_t)a) << 4) | (15u - k);
                const bool el = v && zc != 0u && key > rk2;
                rk2 = el ? key : rk2;
                rz2 = el ? zc : rz2;
              }
              bkey = redo ? rk2 : bkey;
              bz = redo ? rz2 : bz;
            }
            // slot max of the candidates: DPP wave_shl:1 chain, result in lane base
            uint32_t mkey = bkey;
            if (any(bkey != 0u)) {
#pragma unroll
              for (int i = 1; i < N; ++i) {
                const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mkey, 0x130, 0xF, 0xF, false);
                mkey = (a + 1 < N) ? max(mkey, nb) : mkey;
              }
              mkey = (uint32_t)__shfl((int)mkey, base);
            }
            const uint32_t wz = (uint32_t)__shfl((int)bz, base + 15 - (int)((mkey >> 4) & 15u));
            int32_t u = 0;
            if (any(A != ENONE)) u = __shfl(ux, (A != ENONE) ? base + (int)A : lane);
            const uint32_t total = (uint32_t)__shfl((int)incl, base + N - 1);   // acks counted, no event
            // ---- the transition (Client.hs:128-189), as in the fast path ----
            int32_t mt = Sp.mr_t;
            uint32_t mv = Sp.mr_v;
            const bool take = mkey != 0u && (mv == 0u || (int32_t)(mkey >> 8) > mt);
            mt = take ? (int32_t)(mkey >> 8) : mt;
            mv = take ? wz : mv;
            const bool ev = go && e != ENONE;
            const bool r1maj = ev && mj && rs == ROUND1;
            const bool r2maj = ev && mj && rs == ROUND2;
            const bool nack = ev && !mj;
            const bool restart = r2maj && Sp.pending != 0u;
            const bool idle = r2maj && Sp.pending == 0u;
            const uint32_t r2v = (mv == 0u) ? Sp.cmd : mv;
            const int32_t tn = nack ? u + 1 : T + 1;
            const uint32_t k0o = r1maj ? PROPOSE : (r2maj ? EXECUTE : ASK);
            const int32_t x0o = nack ? tn : T;
            const uint32_t z0o = r1maj ? r2v : 0u;
            Sp.r2_v = r1maj ? r2v : Sp.r2_v;
            Sp.pending = r1maj ? ((mv != 0u) ? 1u : 0u) : Sp.pending;
            Sp.ticket = (nack || restart) ? tn : T;
            Sp.cmd = idle ? 0u : Sp.cmd;
            Sp.acks = go ? (ev ? 0u : Sp.acks + total) : Sp.acks;
            Sp.rs = r1maj ? ROUND2 : ((nack || restart) ? ROUND1 : (idle ? IDLE : rs));
            const bool keep_mr = go && !ev && rs == ROUND1;
            Sp.mr_t = keep_mr ? mt : (ev ? 0 : Sp.mr_t);
            Sp.mr_v = keep_mr ? mv : (ev ? 0u : Sp.mr_v);
            // consumed: lanes before the event lane all, the event lane through
            // the event response, later lanes nothing; no event: everything
            const uint32_t kev = (mj ? kmaj : nk) + 1u;
            kp = !go ? kp : (e == ENONE || (uint32_t)a < e) ? cntm : ((uint32_t)a == e ? kev : kp);
            if (any(ev)) send_req(pc, ev, k0o, x0o, z0o);
            if (any(restart)) send_req(pc, restart, ASK, tn, 0u);
            go = go && Sp.rs != IDLE && slot(ballot(kp < cntm)) != 0u;
          }
          l_pop_n(Sx[p], cntm);                              // every due response is consumed
        }
      }
      canon += (stepped && a == 0) ? 48u : 0u;
      tovf = tovf || (pact && S[p].ticket >= PXB_TICKET_LIMIT);
      STAMP(4);
    });
#ifdef PXB_STAMPS
    {
      uint32_t m = st_sr;
      for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off));
      st_cnt[6] += m;
    }
#endif

    // ---------------- end of step: quiescence / step cap ---------------------
    uint32_t lens = 0;
#pragma unroll
    for (int p = 0; p < PM; ++p) lens |= R[p].hl | Sx[p].hl;
    const uint64_t busyb = ballot(active && (lens & 15u) != 0u);
    const bool quiet = active && slot(busyb) == 0u && s >= last_tick;
    const bool cap = active && !quiet && (s + 1 >= (int32_t)kp.step_cap);
    s += active ? 1 : 0;
    const bool done = quiet || cap;
    STAMP(5);
    if (any(cap)) {                             // responses charged but never delivered
#pragma unroll
      for (int p = 0; p < PM; ++p) {
        const uint32_t len = cap ? l_len(Sx[p]) : 0u;
#pragma unroll 1
        for (uint32_t k = 0; any(k < len); ++k) {
          const uint32_t w = L.sq[p][(l_head(Sx[p]) + k) & 7u][lane];
          canon -= (k < len) ? 2u * (16u >> (w >> 30)) : 0u;
        }
      }
    }
    if (any(done)) {

      const uint32_t pan = slot(ballot(A.dead));             // Q6: dead <=> panicked
      const uint32_t dvg = slot(ballot((lflags & PXB_F_LOG_DIVERGENCE) != 0u));
      const uint32_t qov = slot(ballot((lflags & PXB_F_QUEUE_OVERFLOW) != 0u));
      const uint32_t trc = slot(ballot((lflags & PXB_F_LOG_TRUNC) != 0u));
      if (done) {
        uint32_t f = tovf ? (uint32_t)PXB_F_TICKET_OVERFLOW : 0u;
        f |= pan ? (uint32_t)PXB_F_PANIC : 0u;
        f |= dvg ? (uint32_t)PXB_F_LOG_DIVERGENCE : 0u;
        f |= qov ? (uint32_t)PXB_F_QUEUE_OVERFLOW : 0u;
        f |= trc ? (uint32_t)PXB_F_LOG_TRUNC : 0u;
        f |= cap ? (uint32_t)PXB_F_STEP_CAP : 0u;
        f |= dval ? 0u : (uint32_t)PXB_F_UNDECIDED;
#pragma unroll
        for (int p = 0; p < PM; ++p)
          f |= (!cap && (uint32_t)p < P && S[p].rs != IDLE) ? (uint32_t)PXB_F_STUCK : 0u;
        canon_acc += canon + ((a == 0) ? 20u : 4u);          // + result record + this digest
        if (a == 0) {
          ca += 1u + ((f & PXB_F_UNDECIDED) ? 0x10000u : 0u);
          cb += ((f & PXB_F_STUCK) ? 1u : 0u) + ((f & PXB_F_PANIC) ? 0x10000u : 0u);
          cc += ((f & PXB_F_LOG_DIVERGENCE) ? 1u : 0u) + ((f & PXB_F_STEP_CAP) ? 0x10000u : 0u);
          cd += ((f & PXB_F_QUEUE_OVERFLOW) ? 1u : 0u) + ((f & PXB_F_TICKET_OVERFLOW) ? 0x10000u : 0u);
          ce += (f & PXB_F_LOG_TRUNC) ? 1u : 0u;
          rounds_acc += rounds;
          steps_acc += (uint32_t)s;
          execs_acc += execs;
        }
        if (a == 0 && kp.out) {
          uint4 r;
          r.x = code32<LOGM>(dval);
          r.y = dval ? (uint32_t)dtick : 0u;
          r.z = rounds;
          r.w = (f & 0xFFu) | ((uint32_t)s << 16);
          kp.out[gid] = r;
        }
        if (kp.dig) kp.dig[(uint64_t)gid * N + a] = fnv_u32(digest, log_len);
        if (kp.acc) {
          uint4 r;
          r.x = (uint32_t)A.t_max;
          r.y = (uint32_t)A.t_store;
          r.z = code32<LOGM>(A.val);
          r.w = log_len | ((A.dead ? 1u : 0u) << 31);
          kp.acc[(uint64_t)gid * N + a] = r;
        }
        active = false;
      }
    }
    STAMP(6);
  }

  STAMP(7);
  STAMP_FLUSH(kp.dbg);
#ifdef PXB_WAVE_TIMES
  {
    const uint64_t wt1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t wm1 = __builtin_amdgcn_s_memtime();
    // HW_ID (SIMD, CU, SE fields) and XCC_ID hardware registers
    const uint64_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint64_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);
    // (only launches given a buffer: the general kernel behind the per-lane
    // kernels runs with kp.dbg null -- an unguarded store here faulted)
    if (kp.dbg && lane < 6 && wave < 65536u)
      kp.dbg[6 * wave + lane] = lane == 0 ? wt0 : lane == 1 ? wt1 : lane == 2 ? hw : lane == 3 ? xcc : lane == 4 ? wm0 : wm1;
  }
#endif
  flush_totals();
}

}  // namespace pxb
