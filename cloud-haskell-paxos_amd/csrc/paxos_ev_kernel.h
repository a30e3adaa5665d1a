// paxos_ev_kernel.h — gfx950 wave driver of the per-lane kernel (paxos_ev.h).
//
// One 64-lane wave per block, persistent: every lane runs its own instance one
// iteration at a time and, when the instance ends (or bails), writes its
// outputs and takes the next instance id from the wave's chunk of the launch's
// work queue.  The per-lane state lives in registers and in the block's LDS,
// lane-interleaved; the block's resident count is set by that LDS (the kernel
// is latency-bound, so every byte per lane matters: DESIGN.md §3).
#pragma once
#include <hip/hip_runtime.h>

#include "paxos_ev.h"

namespace pxb {
namespace ev {

// lane-interleaved LDS words: word i of lane l at w[i * 64 + l]
struct LdsMem {
  uint32_t* w;
  uint32_t lane;
  __host__ __device__ uint32_t ld(uint32_t i) const { return w[i * 64u + lane]; }
  __host__ __device__ void st(uint32_t i, uint32_t v) const { w[i * 64u + lane] = v; }
  // halfword i of the array starting at word `base`
  __host__ __device__ uint32_t ld16(uint32_t base, uint32_t i) const {
    return reinterpret_cast<const uint16_t*>(w)[((base + (i >> 1)) * 64u + lane) * 2u + (i & 1u)];
  }
  __host__ __device__ void st16(uint32_t base, uint32_t i, uint32_t v) const {
    reinterpret_cast<uint16_t*>(w)[((base + (i >> 1)) * 64u + lane) * 2u + (i & 1u)] = (uint16_t)v;
  }
  // halfword `half` (0, 1) of word i
  __host__ __device__ uint32_t ld16h(uint32_t i, uint32_t half) const {
    return reinterpret_cast<const uint16_t*>(w)[(i * 64u + lane) * 2u + half];
  }
  __host__ __device__ void st16h(uint32_t i, uint32_t half, uint32_t v) const {
    reinterpret_cast<uint16_t*>(w)[(i * 64u + lane) * 2u + half] = (uint16_t)v;
  }
  // element i of a lane-interleaved halfword array at word `base`: [i][lane]
  // (a halfword per lane and row: the address is one shift-add)
  __host__ __device__ uint32_t ldh(uint32_t base, uint32_t i) const {
    return reinterpret_cast<const uint16_t*>(w + base * 64u)[i * 64u + lane];
  }
  __host__ __device__ void sth(uint32_t base, uint32_t i, uint32_t v) const {
    reinterpret_cast<uint16_t*>(w + base * 64u)[i * 64u + lane] = (uint16_t)v;
  }
  // OR into a word (ds_or_b32: no read-back on the critical path)
  __device__ void orw(uint32_t i, uint32_t v) const { atomicOr(&w[i * 64u + lane], v); }
};

constexpr uint32_t EV_QCHUNK = 64;            // instances per work-queue grab (one per lane)
constexpr uint32_t EV_TCOPIES = 256;          // partial-total rows (= TCOPIES in paxos_kernel.h)

struct EvKParams {
  EvParams p;
  uint32_t n_instances;
  uint4* out;                                 // pxb_result records (nullable)
  uint32_t* dig;                              // log digests (nullable)
  uint4* acc;                                 // final acceptor records (nullable)
  unsigned long long* part;                   // EV_TCOPIES partial run-total rows
  uint32_t* queue;                            // next instance, 0 on entry
  uint32_t* bail_ids;                         // ids of bailed instances (capacity bail_cap)
  uint32_t* bail_n;                           // their count, 0 on entry (may exceed bail_cap: overflow)
  uint32_t bail_cap;
  // optional: run only the instances listed in ids[0 .. *n_ids) (another
  // per-lane kernel's bails); a count above ids_cap (that list overflowed)
  // runs none and marks this kernel's own list overflowed, so the general
  // kernel re-runs the whole chunk
  const uint32_t* ids;
  const uint32_t* n_ids;
  uint32_t ids_cap;
#ifdef PXB_WAVE_TIMES
  unsigned long long* dbg;                    // diagnostic: per-wave (start, end, last grab, instances, HW_ID, XCC_ID)
#endif
};

// response-pool words per lane of a shape (the compact layout is picked for
// schedules with short delays, whose responses in flight stay fewer)
#ifndef PXB_EV_CMP_POOL
#define PXB_EV_CMP_POOL 24
#endif
// (log mode over at most 10 links: 19 words, 86 per lane, 7 waves per CU instead
// of 5 (9.5 KiB of LDS to spare).  Round 6: with 18 words (85 per lane) faulty
// log mode handed on 2 instances per million (host model), one of the
// longest each time, so nearly every 2^20-instance call waited 4-5 ms for its
// re-run after the per-lane kernel (kernel trace,
// profiles/r06_notes/lg2_kernel_trace_2p20.txt); with 19, none in 4 million.
// Round 5 measured the halfword response links
// here too (PXB_EV_LG_RH=1 with PXB_EV_LG_POOL=15: 75 words, 8 waves per CU,
// 9 bails in 20000): 2^22 +-1 %, 2^20 -11 % (the chunk tail): not used)
// (slim: 44 words hold the responses of 99.6 % of config 5's P = 3 instances
// (with its 5-deep response FIFOs, whose entries are pool index + 1: < 64
// words), 28 those of 99.8 % of its P = 2 ones with halfword response links
// (75 words per lane, 8 waves per CU; round 4: 30 words and 86, 7); compact over <= 10 links:
// config 3 bails no more with 16 words than with 24, and its shape then leaves
// LDS to spare at 12 waves per CU)
// (tight, layout 7: 21 words, 50 per lane: 12 resident waves per CU need
// <= 50 (measured: 52-word lanes ran 11, the 12th block waited); 5-bit
// entries of pool index + 1 beside the 8 Round2Success codes allow <= 23;
// config 4 bails 0.76 % on it, host model)
// (compact over > 16 links; tools/wave_model.cpp C5W4=1 varies it)
#ifndef PXB_EV_CMPW_POOL
#define PXB_EV_CMPW_POOL 48
#endif
#ifndef PXB_EV_SL2_POOL
#define PXB_EV_SL2_POOL 28
#endif
#ifndef PXB_EV_LG_POOL
#define PXB_EV_LG_POOL 19
#endif
// (slim log mode on the 4-step wheel, layout 9: see pxb_run_device; a 17-word
// pool, 74 words, handed 5.5 instances per million on and measured slower)
#ifndef PXB_EV_LGS_POOL
#define PXB_EV_LGS_POOL 19
#endif
#ifndef PXB_EV_TIGHT_POOL
#define PXB_EV_TIGHT_POOL 21
#endif
// (W: the log-mode shape on the 16-step wheel, the second stage behind the
// 8-step one, takes the larger pool of its topology)
#ifndef PXB_EV_SLW4_POOL
#define PXB_EV_SLW4_POOL 31
#endif
template <int PM, int N, bool CMP, bool LG = false, bool SL = false, int SP = 0, int W = 8>
struct EvPool {
  static constexpr int value = (SP == 2)             ? PXB_EV_TIGHT_POOL
                               : (SL && !LG && W == 4 && PM * N > 18) ? PXB_EV_SLW4_POOL
                               : (LG && SL && W == 4 && PM * N <= 10) ? PXB_EV_LGS_POOL
                               : (LG && PM * N <= 10 && W <= 8) ? PXB_EV_LG_POOL
                               : (CMP && PM * N <= 10) ? 16
                               : (PM * N <= 16)      ? (CMP ? PXB_EV_CMP_POOL : 32)
                               : CMP                ? PXB_EV_CMPW_POOL
                               : (PM * N <= 18)     ? (SL ? PXB_EV_SL2_POOL : 32)
                               : SL                 ? 44
                                                    : 64;
};

// Run totals: each lane sums its finished instances in registers; the wave
// adds the lane sums into its partial row (finalize_kernel sums the rows)
// when it ends, or earlier once a lane has summed EV_FLUSH instances, which
// keeps every 32-bit sum from wrapping (an instance runs < 2^12 steps and
// sends < 2^10 messages per step: at most 2^8 x 2^22; canonical bytes are
// summed in 64 bits).
constexpr int EV_NTOT = 12;
constexpr uint32_t EV_FLUSH = 1u << 8;
__device__ constexpr int tot_slot[EV_NTOT] = {PXB_C_INSTANCES, PXB_C_UNDECIDED, PXB_C_STUCK, PXB_C_PANIC,
                                              PXB_C_DIVERGENCE, PXB_C_STEP_CAP, PXB_C_ROUNDS, PXB_C_STEPS,
                                              PXB_C_MESSAGES, PXB_C_EXECUTES, PXB_C_LOG_TRUNC, PXB_C_CANON_BYTES};

struct EvTotals {
  uint32_t c[EV_NTOT - 1];            // the 32-bit sums, in tot_slot order
  uint64_t canon;
  __device__ void clear() {
#pragma unroll
    for (int q = 0; q < EV_NTOT - 1; ++q) c[q] = 0u;
    canon = 0ull;
  }
  __device__ static uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
  }
  // the wave's sums into its partial row (all 64 lanes of the wave call this)
  __device__ void flush(unsigned long long* trow, uint32_t lane) {
#pragma unroll
    for (int q = 0; q < EV_NTOT - 1; ++q) {
      const uint64_t t = wave_sum((uint64_t)c[q]);
      if (lane == 0 && t) atomicAdd(&trow[tot_slot[q]], (unsigned long long)t);
    }
    const uint64_t t = wave_sum(canon);
    if (lane == 0 && t) atomicAdd(&trow[PXB_C_CANON_BYTES], (unsigned long long)t);
    const uint64_t d = wave_sum((uint64_t)(c[0] - c[1]));        // decided = instances - undecided
    if (lane == 0 && d) atomicAdd(&trow[PXB_C_DECIDED], (unsigned long long)d);
    clear();
  }
};

// The compact layout leaves room for 10 resident waves per CU (LDS), i.e. 3
// on some SIMDs: its register budget is then 168 VGPRs, which the second
// bound (minimum waves per SIMD) makes the compiler keep to.
// The slim layout fits 5 or more waves per CU, 2 on some SIMDs: <= 256 VGPRs.
template <int PM, int N, int W, bool CMP, bool LG = false, bool SL = false, int SP = 0>
__global__ __launch_bounds__(64, CMP ? 3 : SL ? 2 : 1) void paxos_ev_kernel(EvKParams kp) {
  constexpr int POOL = EvPool<PM, N, CMP, LG, SL, SP, W>::value;
  using S = Shape<PM, N, POOL, W, CMP, LG, SL, SP>;
  __shared__ uint32_t lds[S::WORDS * 64];
  const uint32_t lane = threadIdx.x;
  unsigned long long* const trow = kp.part + (size_t)(blockIdx.x % EV_TCOPIES) * 16u;
  EvTotals tot;
  tot.clear();
  EvLane<PM, N, POOL, W, CMP, LdsMem, true, LG, SL, SP> L;
  L.m = LdsMem{lds, lane};
  L.set_keys(kp.p);
  L.mode = M_IDLE;
  L.bailed = false;
  uint32_t n = kp.n_instances;
  if (kp.n_ids) {
    const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)*kp.n_ids);
    n = (c <= kp.ids_cap) ? c : 0u;
    if (c > kp.ids_cap && blockIdx.x == 0 && lane == 0) atomicAdd(kp.bail_n, kp.bail_cap + 1u);
  }
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t next = 0, end = 0;
  bool drained = false;
#ifdef PXB_WAVE_TIMES   // diagnostic: wave start / end / last chunk grab (100 MHz constant clock), instances taken
  const uint64_t wt0 = __builtin_amdgcn_s_memrealtime();
  uint64_t wgrab = wt0;
  uint32_t wtaken = 0;
#endif

#ifndef PXB_EV_REFILL_MIN
#define PXB_EV_REFILL_MIN 2
#endif
  // Idle lanes of the wave (wave-uniform, kept in a scalar): the refill below
  // runs only once it can start PXB_EV_REFILL_MIN lanes, or when no lane is
  // live, and the count is only re-taken after a lane ended or bailed.  A
  // refill costs the wave ~600 instructions whether it starts one lane or
  // several, and a lane ends every ~17 wave-iterations (config 4), so nearly
  // every refill started one lane; waiting for a second costs each instance
  // ~8 idle lane-iterations of its ~1090 (tools/wave_model.cpp refill_min):
  // MI355X A/B, config 4 at 2^24: +1.3 %.  The refill test is taken only
  // where the idle count changes (a refill leaves no idle lane unless the
  // chunk drained, so it clears the flag), and the steps in between run in an
  // inner loop whose back edge is one ballot (round 5: with the outputs stored
  // in the finishing branch, config 4 +3.4 %).  (Measured and not kept,
  // profiles/r04_notes: idle lanes running the iteration predicated off
  // instead of masked, -0.9 %; the crash-window draws spread over the wave,
  // -0.3 %; grabs of as many instances as idle lanes near the end of the
  // queue, config 4 +-0, configs 3 and 5 -10 % (queue-word contention); a
  // 2x-unrolled step loop spills.)
  uint32_t nidle = 64u;
  bool refill = true;
  for (;;) {
    if (refill) {
      // ---- refill idle lanes from the wave's chunk of the queue ----
      uint64_t freeb = __builtin_amdgcn_ballot_w64(L.mode == M_IDLE);
      while (freeb != 0ull && !drained) {
        // (wave-uniform; a lane's sums only grow by instances it takes here)
        if (__builtin_amdgcn_ballot_w64(tot.c[0] >= EV_FLUSH) != 0ull) tot.flush(trow, lane);
        if (next >= end) {
          uint32_t c = 0;
          if (lane == 0) c = atomicAdd(kp.queue, EV_QCHUNK);
          c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
          if (c >= n) {
            drained = true;
            break;
          }
          next = c;
          end = min(c + EV_QCHUNK, n);
#ifdef PXB_WAVE_TIMES
          wgrab = __builtin_amdgcn_s_memrealtime();
          wtaken += EV_QCHUNK;
#endif
        }
        const uint32_t take = min((uint32_t)__popcll(freeb), end - next);
        const uint32_t rank = (uint32_t)__popcll(freeb & below);
        if (((freeb >> lane) & 1ull) && rank < take) L.init(kp.p, kp.n_ids ? kp.ids[next + rank] : next + rank);
        if (((freeb >> lane) & 1ull) && rank < take) {
          if (__builtin_expect(L.bailed, 0)) {   // (a fuzzed P above this shape's: the general kernel's)
            const uint32_t pos = atomicAdd(kp.bail_n, 1u);
            if (pos < kp.bail_cap) kp.bail_ids[pos] = L.gid;
            L.mode = M_IDLE;
            L.bailed = false;
          }
        }
        next += take;
        freeb = __builtin_amdgcn_ballot_w64(L.mode == M_IDLE);
      }
      const uint64_t idleb = __builtin_amdgcn_ballot_w64(L.mode == M_IDLE);
      if (idleb == ~0ull) break;                   // (drained: nothing left to run)
      nidle = (uint32_t)__popcll(idleb);
      refill = false;                              // (nidle == 0, or drained with a live lane)
    }

    // ---- one iteration of every live lane ----
    // (an ended instance's outputs and sums are taken in the step end's
    // finishing branch, where its state is live: stored here instead, LLVM
    // kept a copy of the acceptor registers for them in every iteration)
    EvOut o;
    bool done = false;
    // (an instance that bailed in its last iteration is re-run: no outputs here)
    auto fin = [&](const EvOut& o) {
        if (L.bailed) return;
        const uint32_t f = o.flags;
        tot.c[0] += 1u;
        tot.c[1] += (f & PXB_F_UNDECIDED) ? 1u : 0u;
        tot.c[2] += (f & PXB_F_STUCK) ? 1u : 0u;
        tot.c[3] += (f & PXB_F_PANIC) ? 1u : 0u;
        tot.c[4] += (f & PXB_F_LOG_DIVERGENCE) ? 1u : 0u;
        tot.c[5] += (f & PXB_F_STEP_CAP) ? 1u : 0u;
        tot.c[6] += L.rounds;
        tot.c[7] += o.steps;
        tot.c[8] += L.msgs_sent();
        tot.c[9] += L.execs;
        if (LG) tot.c[10] += (f & PXB_F_LOG_TRUNC) ? 1u : 0u;
        tot.canon += L.canon;
        if (kp.out) kp.out[L.gid] = make_uint4(o.res[0], o.res[1], o.res[2], o.res[3]);
        if (kp.dig) {
#pragma unroll
          for (int a = 0; a < N; ++a) kp.dig[(uint64_t)L.gid * N + a] = L.digest_of(a);
        }
        if (kp.acc) {
#pragma unroll
          for (int a = 0; a < N; ++a) {
            uint32_t r[4];
            L.record_of(a, r);
            kp.acc[(uint64_t)L.gid * N + a] = make_uint4(r[0], r[1], r[2], r[3]);
          }
        }
    };
    // (iterations until some lane ends or bails: the inner loop's back edge
    // is the one ballot)
    do {
      if (L.mode != M_IDLE) done = L.step(kp.p, o, true, fin);
    } while (__builtin_amdgcn_ballot_w64(done | L.bailed) == 0ull);
    if (__builtin_expect(L.bailed, 0)) {      // beyond this kernel's capacities: re-run by the general kernel
      const uint32_t pos = atomicAdd(kp.bail_n, 1u);
      if (pos < kp.bail_cap) kp.bail_ids[pos] = L.gid;
      L.mode = M_IDLE;
      L.bailed = false;
    }
    nidle = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(L.mode == M_IDLE));
    refill = nidle == 64u || (nidle >= (uint32_t)PXB_EV_REFILL_MIN && !drained);
  }
#ifdef PXB_WAVE_TIMES
  if (kp.dbg && blockIdx.x < 65536u) {
    const uint64_t wt1 = __builtin_amdgcn_s_memrealtime();
    const uint64_t hw = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    const uint64_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);
    if (lane < 6)
      kp.dbg[6ull * blockIdx.x + lane] = lane == 0 ? wt0 : lane == 1 ? wt1 : lane == 2 ? wgrab : lane == 3 ? wtaken
                                        : lane == 4 ? hw : xcc;
  }
#endif
  tot.flush(trow, lane);
}

}  // namespace ev
}  // namespace pxb
