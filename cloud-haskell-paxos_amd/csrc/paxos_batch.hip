// paxos_batch.hip — host side of the gfx950 batched ticket-Paxos engine: the
// C ABI (include/paxos_batch.h), launch configuration, dispatch over the
// kernel instantiations, and the single-handler hook kernels.
//
// The batch kernel itself is paxos_kernel.h (design notes there and in
// DESIGN.md); its instantiations are compiled by paxos_inst.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/paxos_batch.h"
#include "paxos_ev_kernel.h"
#include "paxos_ff1.h"
#include "paxos_ffp.h"
#include "paxos_kernel.h"

namespace pxb {

// The kernel instantiations live in paxos_inst.hip (compiled once per
// proposer count, in parallel); declared here for the dispatch table.
#define PXB_FOR_N(M, PM, LOGM, FF) M(PM, 2, LOGM, FF) M(PM, 3, LOGM, FF) M(PM, 4, LOGM, FF) M(PM, 5, LOGM, FF) \
  M(PM, 6, LOGM, FF) M(PM, 7, LOGM, FF) M(PM, 8, LOGM, FF) M(PM, 9, LOGM, FF)
#define PXB_FOR_MODES(M, PM) PXB_FOR_N(M, PM, false, false) PXB_FOR_N(M, PM, false, true) \
  PXB_FOR_N(M, PM, true, false) PXB_FOR_N(M, PM, true, true)
#define PXB_EXTERN(PM, N, LOGM, FF) extern template __global__ void paxos_batch_kernel<PM, N, LOGM, FF>(KParams);
PXB_FOR_MODES(PXB_EXTERN, 1)
PXB_FOR_MODES(PXB_EXTERN, 2)
PXB_FOR_MODES(PXB_EXTERN, 3)
// per-lane kernels (paxos_ev.hip): P x N x {8, 16}-step wheels
#define PXB_EV_EXTERN(PM, N, W, C) extern template __global__ void ev::paxos_ev_kernel<PM, N, W, C>(ev::EvKParams);
#define PXB_EV_FOR(M, PM, W, C) M(PM, 2, W, C) M(PM, 3, W, C) M(PM, 4, W, C) M(PM, 5, W, C) M(PM, 6, W, C) \
  M(PM, 7, W, C) M(PM, 8, W, C) M(PM, 9, W, C)
PXB_EV_FOR(PXB_EV_EXTERN, 1, 8, false) PXB_EV_FOR(PXB_EV_EXTERN, 1, 16, false) PXB_EV_FOR(PXB_EV_EXTERN, 1, 8, true)
PXB_EV_FOR(PXB_EV_EXTERN, 2, 8, false) PXB_EV_FOR(PXB_EV_EXTERN, 2, 16, false) PXB_EV_FOR(PXB_EV_EXTERN, 2, 8, true)
PXB_EV_FOR(PXB_EV_EXTERN, 3, 8, false) PXB_EV_FOR(PXB_EV_EXTERN, 3, 16, false) PXB_EV_FOR(PXB_EV_EXTERN, 3, 8, true)
#define PXB_EV_EXTERN_SL(PM, N, W, C) extern template __global__ void ev::paxos_ev_kernel<PM, N, W, C, false, true>(ev::EvKParams);
PXB_EV_FOR(PXB_EV_EXTERN_SL, 1, 8, false) PXB_EV_FOR(PXB_EV_EXTERN_SL, 2, 8, false) PXB_EV_FOR(PXB_EV_EXTERN_SL, 3, 8, false)
// (the compact 4-step, log-mode and simple-schedule shapes: instantiated in paxos_ev.hip too)
PXB_EV_FOR(PXB_EV_EXTERN, 1, 4, true) PXB_EV_FOR(PXB_EV_EXTERN, 2, 4, true) PXB_EV_FOR(PXB_EV_EXTERN, 3, 4, true)
#define PXB_EV_EXTERN_LG(PM, N, W, C) extern template __global__ void ev::paxos_ev_kernel<PM, N, W, C, true>(ev::EvKParams);
PXB_EV_FOR(PXB_EV_EXTERN_LG, 1, 8, false) PXB_EV_FOR(PXB_EV_EXTERN_LG, 2, 8, false) PXB_EV_FOR(PXB_EV_EXTERN_LG, 3, 8, false)
PXB_EV_FOR(PXB_EV_EXTERN_LG, 1, 16, false) PXB_EV_FOR(PXB_EV_EXTERN_LG, 2, 16, false) PXB_EV_FOR(PXB_EV_EXTERN_LG, 3, 16, false)
#define PXB_EV_EXTERN_LGS(PM, N, W, C) extern template __global__ void ev::paxos_ev_kernel<PM, N, W, C, true, true>(ev::EvKParams);
PXB_EV_FOR(PXB_EV_EXTERN_LGS, 1, 4, false) PXB_EV_FOR(PXB_EV_EXTERN_LGS, 2, 4, false) PXB_EV_FOR(PXB_EV_EXTERN_LGS, 3, 4, false)
#define PXB_EV_EXTERN_SP(PM, N, W, SP) extern template __global__ void ev::paxos_ev_kernel<PM, N, W, true, false, false, SP>(ev::EvKParams);
PXB_EV_FOR(PXB_EV_EXTERN_SP, 1, 4, 1) PXB_EV_FOR(PXB_EV_EXTERN_SP, 2, 4, 1) PXB_EV_FOR(PXB_EV_EXTERN_SP, 3, 4, 1)
PXB_EV_FOR(PXB_EV_EXTERN_SP, 2, 4, 2)
#define PXB_FF1_EXTERN(N) extern template __global__ void ff1::paxos_ff1_kernel<N>(ff1::Ff1Params);
PXB_FF1_EXTERN(2) PXB_FF1_EXTERN(3) PXB_FF1_EXTERN(4) PXB_FF1_EXTERN(5)
PXB_FF1_EXTERN(6) PXB_FF1_EXTERN(7) PXB_FF1_EXTERN(8) PXB_FF1_EXTERN(9)
#define PXB_FFP_EXTERN(P, N) extern template __global__ void ffp::paxos_ffp_kernel<P, N>(ffp::FfpParams);
#define PXB_FFP_EXTERN_N(P) PXB_FFP_EXTERN(P, 2) PXB_FFP_EXTERN(P, 3) PXB_FFP_EXTERN(P, 4) PXB_FFP_EXTERN(P, 5) \
  PXB_FFP_EXTERN(P, 6) PXB_FFP_EXTERN(P, 7) PXB_FFP_EXTERN(P, 8) PXB_FFP_EXTERN(P, 9)
PXB_FFP_EXTERN_N(1) PXB_FFP_EXTERN_N(2) PXB_FFP_EXTERN_N(3)

// ---- single-handler hook kernels ------------------------------------------
__global__ void acceptor_hook_kernel(pxb_acceptor_rec* st, const pxb_msg* in, pxb_msg* out, uint32_t count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  AccState A{st[i].t_max, st[i].t_store, st[i].val, (st[i].meta >> 31) != 0u};
  uint32_t log_len = st[i].meta & 0x7FFFFFFFu;
  pxb_msg r{NONE, 0, 0, 0};
  if (!A.dead) {
    int32_t rx, ry;
    uint32_t rz, ev;
    const uint32_t rk = acceptor_step(A, true, in[i].kind, in[i].x, in[i].z, rx, ry, rz, ev);
    if (ev) log_len++;
    if (rk != NONE) r = pxb_msg{rk, rx, ry, rz};
  }
  st[i] = pxb_acceptor_rec{A.t_max, A.t_store, A.val, log_len | ((A.dead ? 1u : 0u) << 31)};
  out[i] = r;
}

__global__ void proposer_hook_kernel(pxb_proposer_rec* st, uint32_t n_acc, const pxb_msg* in,
                                     pxb_msg* bc, uint32_t* nb, uint32_t count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  pxb_proposer_rec R = st[i];
  PropState S{R.ticket, R.cmd, R.acks, R.state, R.mr_t, R.mr_v, R.r2_t, R.r2_v, R.pending != 0u ? 1u : 0u};
  Req o0{NONE, 0, 0}, o1{NONE, 0, 0};
  uint32_t no;
  if (in[i].kind == 3u)
    no = proposer_tick(S, (R.client_id << 24) | ((uint32_t)(S.ticket + 1) & 0xFFFFFFu), o0);
  else
    no = proposer_step(S, n_acc, in[i].kind, in[i].x, in[i].y, in[i].z, o0, o1);
  st[i] = pxb_proposer_rec{S.ticket, S.cmd, S.acks, S.rs, S.mr_t, S.mr_v, S.r2_t, S.r2_v,
                           S.pending ? 1u : 0u, R.client_id};
  bc[2 * i] = (no > 0) ? pxb_msg{o0.kind, o0.x, 0, o0.z} : pxb_msg{NONE, 0, 0, 0};
  bc[2 * i + 1] = (no > 1) ? pxb_msg{o1.kind, o1.x, 0, o1.z} : pxb_msg{NONE, 0, 0, 0};
  nb[i] = no;
}

constexpr uint32_t QWORDS = 8;          // per-slot queue / counter words (finalize_kernel resets them)
// queue words: [0] the general kernel's work queue, [1] the per-lane kernel's,
// [2] its bailed-instance count; split routing: [3] the second per-lane
// kernel's queue, [4] its bailed-instance count
[[maybe_unused]] constexpr uint32_t Q_GEN = 0, Q_EV = 1, Q_BAIL = 2, Q_EV2 = 3, Q_BAIL2 = 4;   // (Q_GEN: kp.queue itself)

// Sums the TCOPIES partial rows of the general kernel, and those of the
// per-lane kernels unless the bailed-id list the general kernel ran
// (queue[bail_word]) overflowed (then it re-ran every instance of the chunk),
// into the caller's totals; zeroes them and resets the queue words, so the
// launch slot is clean for its next use.  One block of TCOPIES threads;
// thread t reads column t % 16 of rows t/16, t/16+16, ...
__global__ __launch_bounds__(TCOPIES) void finalize_kernel(unsigned long long* part, unsigned long long* part_ev,
                                                            uint32_t* queue, uint32_t bail_word, uint32_t bail_cap,
                                                            unsigned long long* totals, unsigned long long* hand) {
  __shared__ unsigned long long acc[16];
  const uint32_t t = threadIdx.x;
  if (t < 16) acc[t] = 0ull;
  // the device's hand-off counts (pxb_handoff_counts): instances the first
  // per-lane kernel handed on, and those a second one handed on
  if (t < 2 && queue[t ? Q_BAIL2 : Q_BAIL]) atomicAdd(&hand[t], (unsigned long long)queue[t ? Q_BAIL2 : Q_BAIL]);
  __syncthreads();
  const bool ev_ok = queue[bail_word] <= bail_cap;
  unsigned long long v = 0ull;
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {
    v += part[t + j * TCOPIES] + (ev_ok ? part_ev[t + j * TCOPIES] : 0ull);
    part[t + j * TCOPIES] = 0ull;
    part_ev[t + j * TCOPIES] = 0ull;
  }
  if (v) atomicAdd(&acc[t % 16u], v);
  __syncthreads();
  if (t < 16 && acc[t]) atomicAdd(&totals[t], acc[t]);
  if (t >= 16 && t < 16 + QWORDS) queue[t - 16] = 0u;
}

// the device's hand-off counts read (pxb_handoff_counts) of the device's hand-off counts (pxb_handoff_counts):
// out[t] = the count, zeroed in the same atomic when reset, so a finalize_kernel
// of another thread's chunk never adds between the read and the zeroing
__global__ void hand_xchg_kernel(unsigned long long* h, unsigned long long* out, int reset) {
  const uint32_t t = threadIdx.x;
  if (t < 2) out[t] = reset ? atomicExch(&h[t], 0ull) : atomicAdd(&h[t], 0ull);
}

// ---- host side ----------------------------------------------------------------
typedef void (*kernel_ptr)(KParams);
typedef void (*ev_kernel_ptr)(ev::EvKParams);

template <int PM, int W, bool C, bool L = false, bool S = false, int SP = 0>
static ev_kernel_ptr ev_pick_n(uint32_t n) {
  switch (n) {
    case 2: return ev::paxos_ev_kernel<PM, 2, W, C, L, S, SP>;
    case 3: return ev::paxos_ev_kernel<PM, 3, W, C, L, S, SP>;
    case 4: return ev::paxos_ev_kernel<PM, 4, W, C, L, S, SP>;
    case 5: return ev::paxos_ev_kernel<PM, 5, W, C, L, S, SP>;
    case 6: return ev::paxos_ev_kernel<PM, 6, W, C, L, S, SP>;
    case 7: return ev::paxos_ev_kernel<PM, 7, W, C, L, S, SP>;
    case 8: return ev::paxos_ev_kernel<PM, 8, W, C, L, S, SP>;
    case 9: return ev::paxos_ev_kernel<PM, 9, W, C, L, S, SP>;
  }
  return nullptr;
}

typedef void (*ff1_kernel_ptr)(ff1::Ff1Params);
static ff1_kernel_ptr ff1_pick(uint32_t n) {
  switch (n) {
    case 2: return ff1::paxos_ff1_kernel<2>;
    case 3: return ff1::paxos_ff1_kernel<3>;
    case 4: return ff1::paxos_ff1_kernel<4>;
    case 5: return ff1::paxos_ff1_kernel<5>;
    case 6: return ff1::paxos_ff1_kernel<6>;
    case 7: return ff1::paxos_ff1_kernel<7>;
    case 8: return ff1::paxos_ff1_kernel<8>;
    case 9: return ff1::paxos_ff1_kernel<9>;
  }
  return nullptr;
}

typedef void (*ffp_kernel_ptr)(ffp::FfpParams);
template <int P>
static ffp_kernel_ptr ffp_pick_n(uint32_t n) {
  switch (n) {
    case 2: return ffp::paxos_ffp_kernel<P, 2>;
    case 3: return ffp::paxos_ffp_kernel<P, 3>;
    case 4: return ffp::paxos_ffp_kernel<P, 4>;
    case 5: return ffp::paxos_ffp_kernel<P, 5>;
    case 6: return ffp::paxos_ffp_kernel<P, 6>;
    case 7: return ffp::paxos_ffp_kernel<P, 7>;
    case 8: return ffp::paxos_ffp_kernel<P, 8>;
    case 9: return ffp::paxos_ffp_kernel<P, 9>;
  }
  return nullptr;
}
static ffp_kernel_ptr ffp_pick(uint32_t p, uint32_t n) {
  return p == 1 ? ffp_pick_n<1>(n) : p == 2 ? ffp_pick_n<2>(n) : p == 3 ? ffp_pick_n<3>(n) : nullptr;
}

// layout index: 0 = 8-step wheel, 1 = 16-step wheel, 2 / 3 = compact links (8- / 4-step wheel),
// 4 = log mode (8-step wheel), 5 = slim (8-step wheel, byte reply seqs), 6 = layout 3 for
// simple schedules (no loss, no Tick skew: ev::layout_for), 7 = layout 6 with halfword
// response FIFOs (tight: the first launch of the two-proposer simple schedules, P = 2 only),
// 8 = log mode on the 16-step wheel with its topology's larger pool (the second stage
// behind layout 4 over <= 10 links), 9 = layout 4 slimmed (byte reply seqs in registers) on
// the 4-step wheel (the first stage of log mode over <= 10 links with delays <= 4)
static ev_kernel_ptr ev_pick(uint32_t pm, uint32_t n, int layout) {
  switch (pm * 10 + (uint32_t)layout) {
    case 10: return ev_pick_n<1, 8, false>(n);
    case 11: return ev_pick_n<1, 16, false>(n);
    case 12: return ev_pick_n<1, 8, true>(n);
    case 13: return ev_pick_n<1, 4, true>(n);
    case 14: return ev_pick_n<1, 8, false, true>(n);
    case 15: return ev_pick_n<1, 8, false, false, true>(n);
    case 16: return ev_pick_n<1, 4, true, false, false, 1>(n);
    case 18: return ev_pick_n<1, 16, false, true>(n);
    case 19: return ev_pick_n<1, 4, false, true, true>(n);
    case 20: return ev_pick_n<2, 8, false>(n);
    case 21: return ev_pick_n<2, 16, false>(n);
    case 22: return ev_pick_n<2, 8, true>(n);
    case 23: return ev_pick_n<2, 4, true>(n);
    case 24: return ev_pick_n<2, 8, false, true>(n);
    case 25: return ev_pick_n<2, 8, false, false, true>(n);
    case 26: return ev_pick_n<2, 4, true, false, false, 1>(n);
    case 27: return ev_pick_n<2, 4, true, false, false, 2>(n);
    case 28: return ev_pick_n<2, 16, false, true>(n);
    case 29: return ev_pick_n<2, 4, false, true, true>(n);
    case 30: return ev_pick_n<3, 8, false>(n);
    case 31: return ev_pick_n<3, 16, false>(n);
    case 32: return ev_pick_n<3, 8, true>(n);
    case 33: return ev_pick_n<3, 4, true>(n);
    case 34: return ev_pick_n<3, 8, false, true>(n);
    case 35: return ev_pick_n<3, 8, false, false, true>(n);
    case 36: return ev_pick_n<3, 4, true, false, false, 1>(n);
    case 38: return ev_pick_n<3, 16, false, true>(n);
    case 39: return ev_pick_n<3, 4, false, true, true>(n);
  }
  return nullptr;
}
struct kernel_fn {
  kernel_ptr fn;
  int wpb;                       // waves per block (Shape<>::wpb)
  int occ;                       // waves per SIMD target (Shape<>::occ)
  explicit operator bool() const { return fn != nullptr; }
};

template <int PM, int N, bool LOGM, bool FF>
static kernel_fn kfn() { return kernel_fn{paxos_batch_kernel<PM, N, LOGM, FF>, Shape<PM, N, LOGM, FF>::wpb, Shape<PM, N, LOGM, FF>::occ}; }

template <int PM, bool LOGM, bool FF>
static kernel_fn pick_n(uint32_t n) {
  switch (n) {
    case 2: return kfn<PM, 2, LOGM, FF>();
    case 3: return kfn<PM, 3, LOGM, FF>();
    case 4: return kfn<PM, 4, LOGM, FF>();
    case 5: return kfn<PM, 5, LOGM, FF>();
    case 6: return kfn<PM, 6, LOGM, FF>();
    case 7: return kfn<PM, 7, LOGM, FF>();
    case 8: return kfn<PM, 8, LOGM, FF>();
    case 9: return kfn<PM, 9, LOGM, FF>();
  }
  return kernel_fn{nullptr, 0, 0};
}

template <int PM>
static kernel_fn pick_mode(uint32_t n, bool logm, bool ff) {
  if (logm) return ff ? pick_n<PM, true, true>(n) : pick_n<PM, true, false>(n);
  return ff ? pick_n<PM, false, true>(n) : pick_n<PM, false, false>(n);
}

// single decree (one Tick per proposer) or log mode (several); fault-free or not
static kernel_fn pick(uint32_t pm, uint32_t n, bool logm, bool ff) {
  switch (pm) {
    case 1: return pick_mode<1>(n, logm, ff);
    case 2: return pick_mode<2>(n, logm, ff);
    case 3: return pick_mode<3>(n, logm, ff);
  }
  return kernel_fn{nullptr, 0, 0};
}

// Test and A/B hooks (environment variables), read once -- on the first
// launch, or by pxb_reload_hooks() -- and never by getenv in the launch path,
// which is not safe against a concurrent setenv (tests/conftest.py's
// `hooks` helper sets them and reloads)
struct Hooks {
  bool no_ev, no_ff1, no_ffp, no_split, no_tight, no_lg2, no_lgs, fail_after_first, ff1_bail;
  int bail_cap;                   // PXB_EV_BAIL_CAP (-1: the default)
  int blocks_per_cu;              // PXB_BLOCKS_PER_CU (0: none)
  int ff1_oversub, ffp_oversub;   // PXB_FF1_OVERSUB / PXB_FFP_OVERSUB (0: FF1_OVERSUB)
  char multi_fail_phase[16];      // PXB_MULTI_FAIL_PHASE / _DEVICE (paxos_multi.cpp)
  int multi_fail_device;
};
static Hooks g_hooks;
static bool g_hooks_read = false;

static thread_local int g_last_hip = 0;
#ifdef PXB_STAMPS
static unsigned long long* g_dbg = nullptr;
#endif
static std::mutex g_mu;
static int g_occ[4][4][10][64];         // [logm*2+ff][pm][n][device] blocks per CU (0 = unknown)
static int g_cus[64];
// Per-launch scratch: QSLOTS slots per device, each two sets of TCOPIES
// partial-total rows (16 x u64; the general kernel's and the per-lane
// kernel's) + the queue words on their own 128-B line.  Each launch takes the
// next slot round-robin; its finalize_kernel leaves the slot zeroed, so
// consecutive launches need no memset.  Up to QSLOTS launches of one device
// may be in flight at once (on any streams).
constexpr int QSLOTS = 64;
constexpr size_t ROWS_U64 = (size_t)TCOPIES * 16;
constexpr size_t SLOT_U64 = 2 * ROWS_U64 + 16;
// (+ 16 words after the last slot: the device's hand-off counts)
constexpr size_t HAND_U64 = (size_t)QSLOTS * SLOT_U64;
static unsigned long long* g_slots[64];
static uint32_t g_qseq[64];
// Each slot's event is recorded behind the last chunk that used it (its
// finalize_kernel, or the zeroing of a failed chunk), and a chunk that takes
// the slot makes its stream wait for it (hipStreamWaitEvent, on the device),
// so a 65th chunk in flight across streams waits for the first one's slot
// instead of sharing its queue words and partial rows
static hipEvent_t g_slot_ev[64][QSLOTS];
static bool g_slot_ev_set[64][QSLOTS];
// (slot creation: a device's own lock, so that its allocation and wait never
// hold up launches on other devices under g_mu)
static std::mutex g_dev_mu[64];
// Per-lane kernel: one launch per EV_CHUNK instances; its bailed ids go to a
// list of EV_BAIL_CAP entries (16 MB) kept per (device, stream): launches of
// one stream run in order, so they can share it.  Bails are rare
// (BASELINE configs: <= 1.5 %); a chunk whose list overflows is re-run whole
// by the general kernel (finalize_kernel then drops the per-lane totals).
// Big chunks matter: each one ends with a tail (the slowest instances of the
// last waves, then of the bailed ones on the general kernel); config 4 at 2^26
// on one GPU: 2^24-instance chunks 1292.6 ms, 2^25 1283.8, 2^26 1277.3.  The
// list holds 1/16 of a chunk (16 MB per slot).
constexpr uint64_t EV_CHUNK = 1ull << 26;
constexpr uint32_t EV_BAIL_CAP = 1u << 22;
// split routing (fuzzed P = 3 batches, config 5): the per-lane kernel of a
// two-proposer shape takes the instances that drew P <= 2 and lists the P = 3
// ones (a third) with its bails for the three-proposer shape, so that list
// holds half a chunk; split chunks are 2^25 instances (64 MB lists, allocated
// for the slots split launches use; config 5 at 2^25: 34.9 M/s with 2^24
// chunks, 36.2 with 2^25)
constexpr uint64_t EV_SPLIT_CHUNK = 1ull << 25;
// fault-free per-lane kernels: blocks per launch, in multiples of the resident
// ones (the dispatcher then hands a freed CU the next block, which balances
// waves that run slower; one 2^28 config-2 launch: x1 5.26 ms, x2 4.76, x4 4.42,
// x8 4.30, x16 4.25)
constexpr uint64_t FF1_OVERSUB = 16;
constexpr uint32_t EV_SPLIT_CAP = (uint32_t)(EV_SPLIT_CHUNK / 2);
// At most EV_LIST_STREAMS streams per device hold lists (created lazily, 16 MB
// each + 64 MB for the two-stage routings).  An entry records an event behind
// the last launches that use its lists (on every exit of a chunk once one of
// them is queued, failures included); they are enqueued with g_mu held, so
// whoever takes the entry over later (a stream beyond EV_LIST_STREAMS evicting
// the oldest, or any stream taking one that pxb_stream_release freed) first
// makes its own stream wait for that event (hipStreamWaitEvent: no host wait,
// so no thread blocks under g_mu): two streams never share a list while
// either may still run on it.  Ownership is a flag, not the stream handle:
// the null (default) stream is a stream like any other.
constexpr int EV_LIST_STREAMS = 8;
struct EvLists {
  hipStream_t s;                // owner, when owned
  bool owned;                   // (false: free, buffers kept for the next owner)
  uint32_t* bail;
  uint32_t* split;
  hipEvent_t ev;                // behind the owner's last launches on these lists
  bool ev_set;
};
static EvLists g_lists[64][EV_LIST_STREAMS];
static int g_nlists[64], g_lnext[64];
static int g_eocc[11][4][10][64];
static int g_ff1occ[10][64];
static int g_ffpocc[4][10][64];

static int hip_fail(hipError_t e) {
  g_last_hip = (int)e;
  return (e == hipErrorOutOfMemory) ? PXB_E_OOM : PXB_E_HIP;
}
#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t _e = (x);                            \
    if (_e != hipSuccess) return hip_fail(_e);      \
  } while (0)

static int validate(const pxb_config* c) {
  if (!c) return PXB_E_INVAL;
  if (c->n_proposers < 1 || c->n_proposers > PXB_MAX_PROPOSERS) return PXB_E_INVAL;
  if (c->n_acceptors < PXB_MIN_ACCEPTORS || c->n_acceptors > PXB_MAX_ACCEPTORS) return PXB_E_INVAL;
  if (c->loss_ppm > 1000000u || c->crash_ppm > 1000000u) return PXB_E_INVAL;
  if (c->delay_max < 1 || c->delay_max > PXB_MAX_DELAY) return PXB_E_INVAL;
  if (c->crash_len_max < 1 || c->crash_len_max > 4096 || c->crash_start_max > 65535) return PXB_E_INVAL;
  if (c->skew_max > 4096) return PXB_E_INVAL;
  if (c->step_cap < 1 || c->step_cap > PXB_MAX_STEP_CAP) return PXB_E_INVAL;
  if (c->n_instances > (1ull << 40)) return PXB_E_INVAL;
  if (c->n_ticks > PXB_MAX_TICKS) return PXB_E_INVAL;
  if (c->n_ticks > 1 && (c->tick_period < 1 || c->tick_period > PXB_MAX_STEP_CAP)) return PXB_E_INVAL;
  return PXB_OK;
}

}  // namespace pxb

using namespace pxb;

extern "C" {

int pxb_abi_version(void) { return PXB_ABI_VERSION; }

#ifdef PXB_STAMPS
// diagnostic build only: cycles per kernel section and event counts, summed over waves (and reset)
int pxb_debug_stamps(unsigned long long* out16) {
  if (!g_dbg) return PXB_E_INVAL;
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out16, g_dbg, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(g_dbg, 0, 16 * sizeof(unsigned long long)));
  return PXB_OK;
}
#endif
#ifdef PXB_WAVE_TIMES
// diagnostic build only: (start, end, HW_ID, XCC_ID, shader-clock start, end) of every wave of the last launch
static unsigned long long* g_wt = nullptr;
static unsigned g_wt_waves = 0;
int pxb_debug_wave_times(unsigned long long* out, unsigned max_waves) {
  if (!g_wt) return PXB_E_INVAL;
  HIPCHK(hipDeviceSynchronize());
  const unsigned nw = std::min(g_wt_waves, max_waves);
  HIPCHK(hipMemcpy(out, g_wt, 6ull * nw * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return (int)nw;
}
#endif
int pxb_last_hip_error(void) { return g_last_hip; }

// the bailed-id lists of (dev, stream) (callers hold g_mu until their launches
// on the lists are enqueued and a ListUse has recorded the entry's event)
static int stream_lists(int dev, hipStream_t st, bool need_split, uint32_t** bail, uint32_t** split,
                        EvLists** ent) {
  EvLists* e = nullptr;
  for (int k = 0; k < g_nlists[dev] && !e; ++k)
    if (g_lists[dev][k].owned && g_lists[dev][k].s == st) e = &g_lists[dev][k];
  bool handover = e == nullptr;
  for (int k = 0; k < g_nlists[dev] && !e; ++k)      // a freed entry (its owner released it)
    if (!g_lists[dev][k].owned) e = &g_lists[dev][k];
  if (!e) {
    if (g_nlists[dev] < EV_LIST_STREAMS) e = &g_lists[dev][g_nlists[dev]++];
    else e = &g_lists[dev][g_lnext[dev]++ % EV_LIST_STREAMS];   // every entry owned: take the oldest over
  }
  if (handover) {                                    // new owner: after the old owner's launches
    if (e->ev_set) HIPCHK(hipStreamWaitEvent(st, e->ev, 0));
    e->s = st;
    e->owned = true;
  }
  if (!e->ev) HIPCHK(hipEventCreateWithFlags(&e->ev, hipEventDisableTiming));
  if (!e->bail) HIPCHK(hipMalloc(&e->bail, (size_t)EV_BAIL_CAP * sizeof(uint32_t)));
  if (need_split && !e->split) HIPCHK(hipMalloc(&e->split, (size_t)EV_SPLIT_CAP * sizeof(uint32_t)));
  *bail = e->bail;
  *split = need_split ? e->split : nullptr;
  *ent = e;
  return PXB_OK;
}

// Records an entry's event behind the launches of a chunk that use its lists,
// on every exit of the chunk (success or failure) once the first of them is
// queued (g_mu held: declared after the chunk's lock, so destroyed before it)
struct ListUse {
  EvLists* e;
  hipStream_t st;
  bool queued = false;
  ~ListUse() {
    if (!e || !queued) return;
    if (hipEventRecord(e->ev, st) == hipSuccess) {
      e->ev_set = true;
    } else {
      // (no event behind these launches: wait for them here, so that a later
      // owner taking the entry over cannot share the lists with them)
      (void)hipStreamSynchronize(st);
      e->ev_set = false;
    }
  }
};

// The same for the chunk's scratch slot (g_slot_ev), on every exit of the chunk
struct SlotUse {
  int dev, sidx;
  hipStream_t st;
  ~SlotUse() {
    if (sidx < 0) return;
    if (hipEventRecord(g_slot_ev[dev][sidx], st) == hipSuccess) {
      g_slot_ev_set[dev][sidx] = true;
    } else {
      (void)hipStreamSynchronize(st);
      g_slot_ev_set[dev][sidx] = false;
    }
  }
};

// A stream that is about to be destroyed gives up its lists (paxos_multi.cpp
// creates a stream per device and call): the entry is freed for the next stream
// (which waits for the event first), so lists never outlive their stream's use.
extern "C" void pxb_stream_release(int dev, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dev < 0 || dev >= 64) return;
  std::lock_guard<std::mutex> lk(g_mu);
  for (int k = 0; k < g_nlists[dev]; ++k)
    if (g_lists[dev][k].owned && g_lists[dev][k].s == st) g_lists[dev][k].owned = false;
}

// per-device scratch of pxb_run_device, created on the current device `dev`
// (callers do NOT hold g_mu: the allocation and the wait for its zeroing take
// only this device's lock, so a device's first launch holds up no launch on
// another device); published under g_mu
static int ensure_slots(int dev) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_slots[dev]) return PXB_OK;
  }
  std::lock_guard<std::mutex> dl(g_dev_mu[dev]);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_slots[dev]) return PXB_OK;            // (another thread made them meanwhile)
  }
  unsigned long long* q = nullptr;
  hipStream_t zs = nullptr;
  hipError_t e = hipMalloc(&q, (HAND_U64 + 16) * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&zs, hipStreamNonBlocking);
  // (the zeroing completes before any launch can use the slots: a private
  // stream, so this waits for nothing else on the device)
  if (e == hipSuccess) e = hipMemsetAsync(q, 0, (HAND_U64 + 16) * sizeof(unsigned long long), zs);
  if (e == hipSuccess) e = hipStreamSynchronize(zs);
  for (int k = 0; k < QSLOTS && e == hipSuccess; ++k)
    if (!g_slot_ev[dev][k]) e = hipEventCreateWithFlags(&g_slot_ev[dev][k], hipEventDisableTiming);
  if (zs) (void)hipStreamDestroy(zs);
  if (e != hipSuccess) {
    if (q) (void)hipFree(q);
    return hip_fail(e);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  for (int k = 0; k < QSLOTS; ++k) g_slot_ev_set[dev][k] = false;
  g_slots[dev] = q;
  return PXB_OK;
}

static void read_hooks_locked() {
  Hooks h;
  memset(&h, 0, sizeof(h));
  auto flag = [](const char* name) {
    const char* v = getenv(name);
    return v && atoi(v) > 0;
  };
  auto num = [](const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
  };
  h.no_ev = flag("PXB_NO_EV");
  h.no_ff1 = flag("PXB_NO_FF1");
  h.no_ffp = flag("PXB_NO_FFP");
  h.no_split = flag("PXB_NO_SPLIT");
  h.no_tight = flag("PXB_NO_TIGHT");
  h.no_lg2 = flag("PXB_NO_LG2");
  h.no_lgs = flag("PXB_NO_LGS");
  h.fail_after_first = flag("PXB_FAIL_AFTER_FIRST");
  h.ff1_bail = flag("PXB_FF1_BAIL");
  h.bail_cap = num("PXB_EV_BAIL_CAP", -1);
  h.blocks_per_cu = std::max(0, num("PXB_BLOCKS_PER_CU", 0));
  const int fo = num("PXB_FF1_OVERSUB", 0), po = num("PXB_FFP_OVERSUB", 0);
  h.ff1_oversub = (fo > 0 && fo <= 64) ? fo : 0;
  h.ffp_oversub = (po > 0 && po <= 64) ? po : 0;
  const char* ph = getenv("PXB_MULTI_FAIL_PHASE");
  if (ph) snprintf(h.multi_fail_phase, sizeof(h.multi_fail_phase), "%s", ph);
  h.multi_fail_device = num("PXB_MULTI_FAIL_DEVICE", -1);
  g_hooks = h;
  g_hooks_read = true;
}

// the hooks in force (a copy: callers read it without the lock)
static Hooks hooks() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_hooks_read) read_hooks_locked();
  return g_hooks;
}

// (paxos_multi.cpp's failure injection: device g fails in `phase`)
bool multi_fail_injected(const char* phase, int g) {
  const Hooks h = hooks();
  return h.multi_fail_phase[0] && strcmp(h.multi_fail_phase, phase) == 0 && h.multi_fail_device == g;
}


extern "C" void pxb_multi_release(void);   // paxos_multi.cpp
extern "C" void pxb_wire_release(void);    // paxos_wire.hip

int pxb_init(int n_devices) {
  int visible = 0;
  if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) return PXB_E_NODEV;
  const int G = (n_devices <= 0) ? visible : n_devices;
  if (G > visible || G > 64) return PXB_E_INVAL;
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  (void)hooks();                       // (the test hooks: read now, not in a launch)
  for (int d = 0; d < G; ++d) {
    HIPCHK(hipSetDevice(d));
    if (int rc = ensure_slots(d)) {
      (void)hipSetDevice(cur);
      return rc;
    }
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, d));
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_cus[d]) g_cus[d] = prop.multiProcessorCount;
  }
  HIPCHK(hipSetDevice(cur));
  return PXB_OK;
}

void pxb_reload_hooks(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  read_hooks_locked();
}

int pxb_shutdown(void) {
  int cur = 0;
  const bool have_dev = hipGetDevice(&cur) == hipSuccess;
  int rc = PXB_OK;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    for (int d = 0; d < 64; ++d) {
      const bool any = g_slots[d] != nullptr || g_nlists[d] > 0;
      if (!any) continue;
      if (hipSetDevice(d) != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = PXB_E_HIP;
      if (g_slots[d]) (void)hipFree(g_slots[d]);
      g_slots[d] = nullptr;
      for (int k = 0; k < QSLOTS; ++k) {
        if (g_slot_ev[d][k]) (void)hipEventDestroy(g_slot_ev[d][k]);
        g_slot_ev[d][k] = nullptr;
        g_slot_ev_set[d][k] = false;
      }
      for (int k = 0; k < g_nlists[d]; ++k) {
        if (g_lists[d][k].bail) (void)hipFree(g_lists[d][k].bail);
        if (g_lists[d][k].split) (void)hipFree(g_lists[d][k].split);
        if (g_lists[d][k].ev) (void)hipEventDestroy(g_lists[d][k].ev);
        g_lists[d][k] = EvLists{};
      }
      g_nlists[d] = g_lnext[d] = 0;
      g_qseq[d] = 0;
    }
  }
  pxb_multi_release();
  pxb_wire_release();
  if (have_dev) (void)hipSetDevice(cur);
  return rc;
}

const char* pxb_strerror(int code) {
  switch (code) {
    case PXB_OK: return "ok";
    case PXB_E_INVAL: return "invalid argument";
    case PXB_E_HIP: return "HIP runtime error";
    case PXB_E_OOM: return "device out of memory";
    case PXB_E_NODEV: return "no GPU device";
    case PXB_E_RCCL: return "collective failure";
  }
  return "unknown error";
}

uint64_t pxb_canonical_bytes_nofault(uint32_t n_acceptors) { return 196ull * n_acceptors + 160ull; }

int pxb_handoff_counts(int dev, uint64_t* out2, int reset) {
  if (!out2 || dev < 0 || dev >= 64) return PXB_E_INVAL;
  unsigned long long* h = nullptr;
  {
    // (the device wait below runs without g_mu: launches on other devices go on)
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_slots[dev]) h = g_slots[dev] + HAND_U64;
  }
  if (!h) {
    out2[0] = out2[1] = 0;
    return PXB_OK;
  }
  // (one reader at a time: the exchange's two output words are shared)
  static std::mutex hand_mu;
  std::lock_guard<std::mutex> hl(hand_mu);
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  HIPCHK(hipSetDevice(dev));
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) {
    // read and (reset) zero in one atomic per count, on the device
    hipLaunchKernelGGL(hand_xchg_kernel, dim3(1), dim3(64), 0, nullptr, h, h + 2, reset ? 1 : 0);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out2, h + 2, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost);
  (void)hipSetDevice(cur);
  return e == hipSuccess ? PXB_OK : hip_fail(e);
}

int pxb_run_device(const pxb_config* cfg, pxb_result* d_out, uint32_t* d_log_digest,
                   pxb_acceptor_rec* d_acc, int64_t* d_totals, void* stream) {
  int rc = validate(cfg);
  if (rc) return rc;
  if (!d_totals) return PXB_E_INVAL;
  if (cfg->n_instances == 0) return PXB_OK;
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return PXB_E_NODEV;
  const Hooks hk = hooks();
  const bool logm = cfg->n_ticks > 1;   // log mode: several Ticks per proposer
  // fault-free schedule: no message is lost, delayed past the next step or sent
  // to an isolated acceptor (Tick skew is allowed)
  const bool ff = !(cfg->flags & PXB_CFG_RANDOMIZE) && cfg->loss_ppm == 0 && cfg->delay_max == 1 &&
                  cfg->crash_ppm == 0;
  // faulty single-decree batches run on the per-lane kernel (paxos_ev.h), its
  // bailed instances on the general faulty kernel.  Per-lane beats the general
  // kernel on every topology, even where its layout fits 3 waves per CU
  // (MI355X, 2^22 instances, ms: config 5 148 vs 247; P = 3, N = 9 with delays
  // to 12: 347 vs 689; P = 2, N = 9, delays to 12: 97 vs 247).
  // PXB_NO_EV=1 forces the general kernel.
  // (faulty log mode too: the per-lane kernel's log-mode fields, 8-step wheel)
  bool use_ev = !ff && ev::eligible(cfg) && !hk.no_ev;
  // tests: a smaller bailed-id list, to exercise its overflow path
  const uint32_t bail_cap = hk.bail_cap >= 0 ? std::min<uint32_t>((uint32_t)hk.bail_cap, EV_BAIL_CAP) : EV_BAIL_CAP;
  // fault-free single-proposer batches (configs 1, 2) run one instance per
  // lane on paxos_ff1_kernel, its (never expected) bails on the general
  // faulty kernel; PXB_NO_FF1=1 keeps them on the general fault-free kernel
  const bool use_ff1 = ff && !logm && cfg->n_proposers == 1 && !hk.no_ff1;
  // the other fault-free batches (duelling proposers, log mode) on
  // paxos_ffp_kernel, its bails on the general faulty kernel; PXB_NO_FFP=1
  // keeps them on the general fault-free kernel
  const bool use_ffp = ff && !use_ff1 && !hk.no_ffp;
  kernel_fn fn = pick(cfg->n_proposers, cfg->n_acceptors, logm, ff && !use_ff1 && !use_ffp);
  if (!fn) return PXB_E_INVAL;
  const ff1_kernel_ptr ffn = use_ff1 ? ff1_pick(cfg->n_acceptors) : nullptr;
  if (use_ff1 && !ffn) return PXB_E_INVAL;
  const ffp_kernel_ptr pfn = use_ffp ? ffp_pick(cfg->n_proposers, cfg->n_acceptors) : nullptr;
  if (use_ffp && !pfn) return PXB_E_INVAL;
  const int layout = ev::layout_for(cfg);
  // Two-stage faulty log mode over <= 10 links: the log-mode shape (layout 4,
  // a 19-word response pool: 86 words, 7 waves per CU) over the chunk, the
  // same shape on the 16-step wheel with a 32-word pool (layout 8) over what
  // it hands on (pool overflows: none in 4 million instances of
  // extra.log_mode_faulty, host model; 2 per million with an 18-word pool),
  // the general log-mode kernel over that one's.  A handed-on instance is one
  // of the longest; on the general kernel it held a 2^20-instance call 4-5 ms
  // and a 2^22 one up to 22 ms after the per-lane kernel, on layout 8 0.9-6 ms
  // (kernel traces, profiles/r06_notes/lg_kernel_trace.txt,
  // lg2_kernel_trace_2p20.txt).  PXB_NO_LG2=1 turns it off.
  const bool may_lg2 = use_ev && layout == 4 && cfg->n_proposers * cfg->n_acceptors <= 10 && !hk.no_lg2;
  // With delays <= 4 the first stage is layout 9: layout 4 with its reply seqs
  // as bytes in registers, the 4-step wheel and its canonical log packed (14
  // words), the same 19-word pool: 75 LDS words, 8 waves per CU instead of 7
  // (residency sweep, faulty log mode at 2^22, PXB_BLOCKS_PER_CU 5 / 6 / 7:
  // 32.7 / 29.6 / 27.5 ms; layout 9: 2^22 +5.6 %, 2^20 +2.5 %,
  // profiles/r06_notes/ab_lg_layout9.txt).  PXB_NO_LGS=1 keeps layout 4.
  const bool lgs = use_ev && layout == 4 && cfg->delay_max <= 4 && cfg->n_proposers * cfg->n_acceptors <= 10 &&
                   !hk.no_lgs;
  const int flayout = lgs ? 9 : layout;     // (the first per-lane stage's)
  const int elayout = may_lg2 ? 8 : flayout;
  const ev_kernel_ptr efn = use_ev ? ev_pick(cfg->n_proposers, cfg->n_acceptors, elayout) : nullptr;
  if (use_ev && !efn) return PXB_E_INVAL;
  // Split routing of fuzzed three-proposer batches (config 5): the
  // two-proposer shape's layout fits more waves (config 5: 6 vs 4 per CU), so
  // it runs first, over the chunk, and lists the instances that drew P = 3
  // (bailed at init) for the three-proposer shape, whose own bails go to the
  // general kernel.  PXB_NO_SPLIT=1 turns it off.
  // tests only: PXB_FAIL_AFTER_FIRST=1 fails every chunk right after its first
  // per-lane launch (the list and slot bookkeeping of the failure path)
  const bool fail_after_first = hk.fail_after_first;
  const bool may_split = use_ev && (cfg->flags & PXB_CFG_RANDOMIZE) && cfg->n_proposers == 3 && !hk.no_split;
  // Tight routing of two-proposer simple schedules whose layout-6 lane takes
  // more than 52 LDS words (config 4: 60 words, 10 waves per CU, so half the
  // SIMDs run 2 waves and half 3): layout 7 (52 words, 12 waves per CU)
  // runs over the chunk first and lists its bails (config 4: 0.5 %, nearly all
  // a full 3-deep response FIFO) for layout 6 over that list, whose own bails
  // go to the general kernel.  PXB_NO_TIGHT=1 turns it off.
  // Only where its hand-off rate is measured small: N = 6, 7 (host model,
  // tools/wave_model.cpp NACC=6/7/8 TIGHT=1 on config 4's schedule: 0.11 %,
  // 0.76 %, 2.8 %; at N = 8 the tight lane has 53 words, so it would not reach
  // 12 waves per CU anyway, and its 21-word pool serves 16 response links).
  // A list that overflowed (above a quarter of the chunk) would have the
  // general kernel re-run the whole chunk: exact, but slow.
  const bool may_tight = use_ev && layout == 6 && cfg->n_proposers == 2 && cfg->n_acceptors >= 6 &&
                         cfg->n_acceptors <= 7 && !hk.no_tight;
  const ev_kernel_ptr sfn = may_split ? ev_pick(2, cfg->n_acceptors, layout)
                            : may_tight ? ev_pick(2, cfg->n_acceptors, 7)
                            : may_lg2 ? ev_pick(cfg->n_proposers, cfg->n_acceptors, flayout) : nullptr;
  // (split: the two-stage routing of either kind)
  bool split = false;
  const hipStream_t st = (hipStream_t)stream;
  int occ, cus, eocc = 0, socc = 0;
  if (int rc2 = ensure_slots(dev)) return rc2;   // (not under g_mu: see ensure_slots)
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_cus[dev]) {
      hipDeviceProp_t prop;
      HIPCHK(hipGetDeviceProperties(&prop, dev));
      g_cus[dev] = prop.multiProcessorCount;
    }
    int& o = g_occ[(logm ? 2 : 0) + ((ff && !use_ff1 && !use_ffp) ? 1 : 0)][cfg->n_proposers][cfg->n_acceptors][dev];
    if (!o) {
      int nb = 0;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)fn.fn, 64 * fn.wpb, 0));
      o = std::max(1, nb);
    }
    // Residency: the launch-bounds target (waves per SIMD x 4 SIMDs), even when
    // a small kernel would fit more (measured: 4 -> 6 waves/SIMD costs 5 % on
    // config 2: more, more often partially filled slot generations per wave).
    const int target = 4 * fn.occ;
    occ = std::min(o, std::max(1, target / fn.wpb));   // blocks per CU
    cus = g_cus[dev];
    auto ev_occ = [&](ev_kernel_ptr k, uint32_t pm, int lay, int* out) -> int {
      int& eo = g_eocc[lay][pm][cfg->n_acceptors][dev];
      if (!eo) {
        int nb = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k, 64, 0));
        eo = std::max(1, nb);
      }
      *out = eo;
      return PXB_OK;
    };
    if (use_ff1) {
      int& fo = g_ff1occ[cfg->n_acceptors][dev];
      if (!fo) {
        int nb = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)ffn, 256, 0));
        fo = std::max(1, nb);
      }
      eocc = fo;
    }
    if (use_ffp) {
      int& fo = g_ffpocc[cfg->n_proposers][cfg->n_acceptors][dev];
      if (!fo) {
        int nb = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)pfn, 256, 0));
        fo = std::max(1, nb);
      }
      eocc = fo;
    }
    if (use_ev) {
      if (int rc2 = ev_occ(efn, cfg->n_proposers, elayout, &eocc)) return rc2;
      if (sfn) {
        if (int rc2 = ev_occ(sfn, may_lg2 ? cfg->n_proposers : 2, may_tight ? 7 : flayout, &socc)) return rc2;
        split = may_lg2 || socc > eocc;
      }
    }
    if (hk.blocks_per_cu > 0) {                 // tests / experiments: cap residency
      occ = std::min(occ, hk.blocks_per_cu);
      if (eocc) eocc = std::min(eocc, hk.blocks_per_cu);
      if (socc) socc = std::min(socc, hk.blocks_per_cu);
    }
  }
  KParams kp;
  memset(&kp, 0, sizeof(kp));
  kp.k0 = (uint32_t)cfg->seed;
  kp.k1 = (uint32_t)(cfg->seed >> 32);
  kp.n_prop = cfg->n_proposers;
  kp.delay_max = cfg->delay_max;
  kp.loss_ppm = cfg->loss_ppm;
  kp.crash_ppm = cfg->crash_ppm;
  kp.crash_len_max = cfg->crash_len_max;
  kp.crash_start_max = cfg->crash_start_max;
  kp.skew_max = cfg->skew_max;
  kp.step_cap = cfg->step_cap;
  kp.n_ticks = logm ? cfg->n_ticks : 1u;
  kp.tick_period = logm ? cfg->tick_period : 1u;
  const uint64_t lt = prob_threshold(cfg->loss_ppm), ct = prob_threshold(cfg->crash_ppm);
  kp.cfg = ((cfg->flags & PXB_CFG_RANDOMIZE) ? CFG_RANDOMIZE : 0u) | (lt ? CFG_LOSSY : 0u) | (ct ? CFG_CRASHY : 0u);
  kp.loss_m1 = (uint32_t)(lt - 1ull);
  kp.crash_m1 = (uint32_t)(ct - 1ull);
  unsigned long long* const totals = reinterpret_cast<unsigned long long*>(d_totals);
#ifdef PXB_STAMPS
  {
    static unsigned long long* dbg = nullptr;
    if (!dbg) {
      HIPCHK(hipMalloc(&dbg, 16 * sizeof(unsigned long long)));
      HIPCHK(hipMemset(dbg, 0, 16 * sizeof(unsigned long long)));
    }
    kp.dbg = dbg;
    g_dbg = dbg;
  }
#endif
  const uint64_t G = 64 / cfg->n_acceptors;
  const uint64_t resident = (uint64_t)occ * (uint64_t)cus;
  // a launch must not give any slot 65536 instances (16-bit packed run totals):
  // on average 30000 per slot for the block-queue kernels (uniform instance
  // lengths), 60000 for the work-queue kernels (which also flush mid-run);
  // epoch tags (idx + 1 under the work queue) stay below 2^30.  Per-lane
  // chunks are bounded by the bailed-id buffer of a scratch slot.
  const uint64_t wpb = (uint64_t)fn.wpb;
  // fault-free log mode: 16-bit epochs, so every block's range (static slices:
  // every wave's) stays below 2^16 instances
  // (tight: bails are rare, so whole chunks; the list holds a quarter of one)
  // (log mode's second stage too)
  const uint64_t ev_chunk = (split && !may_tight && !may_lg2) ? EV_SPLIT_CHUNK : EV_CHUNK;
  // fault-free per-lane kernels: as few launches as the general faulty kernel
  // allows (it may have to re-run a whole chunk); A/B on config 2 at 2^26:
  // 2^24-instance launches 2 % slower, 2^22 10 %, 2^20 33 %
  const uint64_t chunk_max = (use_ff1 || use_ffp) ? std::min<uint64_t>((1ull << 30) - 1, resident * wpb * G * 60000ull)
                             : use_ev ? ev_chunk
                             : (ff && logm) ? std::min<uint64_t>(resident * wpb * G * 30000ull, resident * 60000ull)
                             : ff ? std::min<uint64_t>(1ull << 31, resident * wpb * G * 30000ull)
                                  : std::min<uint64_t>((1ull << 30) - 1, resident * wpb * G * 60000ull);
  for (uint64_t done = 0; done < cfg->n_instances; done += chunk_max) {
    const uint64_t nc = std::min<uint64_t>(chunk_max, cfg->n_instances - done);
    kp.first_instance = cfg->first_instance + done;
    kp.n_instances = (uint32_t)nc;
    kp.out = d_out ? reinterpret_cast<uint4*>(d_out + done) : nullptr;
    kp.dig = d_log_digest ? d_log_digest + done * cfg->n_acceptors : nullptr;
    kp.acc = d_acc ? reinterpret_cast<uint4*>(d_acc + done * cfg->n_acceptors) : nullptr;
    uint32_t *bail = nullptr, *slist = nullptr;
    unsigned long long* slot = nullptr;
    EvLists* lent = nullptr;
    // (held until this chunk's launches are enqueued: see EvLists)
    std::unique_lock<std::mutex> lk(g_mu);
    const int sidx = (int)(g_qseq[dev]++ % QSLOTS);
    slot = g_slots[dev] + (size_t)sidx * SLOT_U64;
    kp.part = slot;
    kp.queue = reinterpret_cast<uint32_t*>(slot + 2 * ROWS_U64);
    // after the slot's last user (another stream's chunk may still run on it)
    if (g_slot_ev_set[dev][sidx]) HIPCHK(hipStreamWaitEvent(st, g_slot_ev[dev][sidx], 0));
    // the slot's event goes behind whatever this chunk queues, on every exit
    SlotUse suse{dev, sidx, st};
    if (use_ev || use_ff1 || use_ffp)
      if (int rc2 = stream_lists(dev, st, split, &bail, &slist, &lent)) return rc2;
    // the lists' event likewise
    ListUse use{lent, st, lent != nullptr};
    // a launch that fails after an earlier one of this chunk has queued leaves
    // the slot half used: zero it behind the queued work before reporting
    auto fail = [&](hipError_t e) {
      (void)hipMemsetAsync(slot, 0, SLOT_U64 * sizeof(unsigned long long), st);
      return hip_fail(e);
    };
    uint32_t bail_word = Q_BAIL;
    if (use_ff1) {
      // the fault-free per-lane kernel over the chunk, the general kernel over its bailed ids
      ff1::Ff1Params fp;
      memset(&fp, 0, sizeof(fp));
      fp.first_instance = kp.first_instance;
      fp.k0 = kp.k0;
      fp.k1 = kp.k1;
      fp.skew_max = cfg->skew_max;
      fp.step_cap = cfg->step_cap;
      fp.n_instances = (uint32_t)nc;
      fp.out = kp.out;
      fp.dig = kp.dig;
      fp.acc = kp.acc;
      fp.part = kp.part + ROWS_U64;
      fp.bail_ids = bail;
      fp.bail_n = kp.queue + Q_BAIL;
      fp.bail_cap = bail_cap;
      fp.bail_all = hk.ff1_bail ? 1u : 0u;               // tests: hand every instance to the general kernel
      // FF1_OVERSUB x the resident blocks (PXB_FF1_OVERSUB=k: k, A/B)
      const uint64_t over = hk.ff1_oversub ? (uint64_t)hk.ff1_oversub : FF1_OVERSUB;
      const uint64_t fres = (uint64_t)eocc * (uint64_t)cus * over;
      const unsigned fgrid = (unsigned)std::min<uint64_t>((nc + 255) / 256, fres);
      hipLaunchKernelGGL(ffn, dim3(fgrid), dim3(256), 0, st, fp);
      if (hipError_t e = hipGetLastError()) return fail(e);
      kp.ids = bail;
      kp.n_ids = kp.queue + Q_BAIL;
      kp.ids_cap = bail_cap;
      hipLaunchKernelGGL(fn.fn, dim3((unsigned)resident), dim3(64 * fn.wpb), 0, st, kp);
      if (hipError_t e = hipGetLastError()) return fail(e);
    } else if (use_ffp) {
      // the fault-free per-lane kernel for duelling proposers / log mode, then
      // the general faulty kernel over its bailed ids
      ffp::FfpParams fp;
      memset(&fp, 0, sizeof(fp));
      fp.first_instance = kp.first_instance;
      fp.k0 = kp.k0;
      fp.k1 = kp.k1;
      fp.n_prop = cfg->n_proposers;
      fp.skew_max = cfg->skew_max;
      fp.step_cap = cfg->step_cap;
      fp.n_ticks = kp.n_ticks;
      fp.tick_period = kp.tick_period;
      fp.n_instances = (uint32_t)nc;
      fp.out = kp.out;
      fp.dig = kp.dig;
      fp.acc = kp.acc;
      fp.part = kp.part + ROWS_U64;
      fp.bail_ids = bail;
      fp.bail_n = kp.queue + Q_BAIL;
      fp.bail_cap = bail_cap;
      fp.bail_all = hk.ff1_bail ? 1u : 0u;               // tests: hand every instance to the general kernel
      const uint64_t over = hk.ffp_oversub ? (uint64_t)hk.ffp_oversub : FF1_OVERSUB;   // (A/B)
      const uint64_t fres = (uint64_t)eocc * (uint64_t)cus * over;
      const unsigned fgrid = (unsigned)std::min<uint64_t>((nc + 255) / 256, fres);
      hipLaunchKernelGGL(pfn, dim3(fgrid), dim3(256), 0, st, fp);
      if (hipError_t e = hipGetLastError()) return fail(e);
      kp.ids = bail;
      kp.n_ids = kp.queue + Q_BAIL;
      kp.ids_cap = bail_cap;
      hipLaunchKernelGGL(fn.fn, dim3((unsigned)resident), dim3(64 * fn.wpb), 0, st, kp);
      if (hipError_t e = hipGetLastError()) return fail(e);
    } else if (use_ev) {
      // the per-lane kernel over the chunk, then the general kernel over its
      // bailed ids; split: the two-proposer shape over the chunk, the
      // three-proposer shape over its list, the general kernel over that one's;
      // tight: layout 7 over the chunk, layout 6 over its list, the general
      // kernel over that one's
      ev::EvKParams ek;
      memset(&ek, 0, sizeof(ek));
      ek.p = ev::make_params(cfg);
      ek.p.first_instance = kp.first_instance;
      ek.n_instances = (uint32_t)nc;
      ek.out = kp.out;
      ek.dig = kp.dig;
      ek.acc = kp.acc;
      ek.part = kp.part + ROWS_U64;
      ek.queue = kp.queue + Q_EV;
      ek.bail_ids = bail;
      ek.bail_n = kp.queue + Q_BAIL;
      ek.bail_cap = bail_cap;
      if (split) {
        ev::EvKParams sk = ek;
        sk.bail_ids = slist;
        sk.bail_cap = std::min<uint32_t>(bail_cap == EV_BAIL_CAP ? EV_SPLIT_CAP : bail_cap, EV_SPLIT_CAP);
        const unsigned sgrid = (unsigned)std::min<uint64_t>((nc + 63) / 64, (uint64_t)socc * (uint64_t)cus);
#ifdef PXB_WAVE_TIMES   // (two-stage: the first per-lane launch's timeline)
        if (!g_wt) HIPCHK(hipMalloc(&g_wt, 6ull * 65536 * sizeof(unsigned long long)));
        sk.dbg = g_wt;
        g_wt_waves = sgrid;
#endif
        hipLaunchKernelGGL(sfn, dim3(sgrid), dim3(64), 0, st, sk);
        if (hipError_t e = hipGetLastError()) return fail(e);
        // (tests: a launch failure right after the first per-lane launch)
        if (fail_after_first) return fail(hipErrorLaunchFailure);
        ek.ids = slist;
        ek.n_ids = kp.queue + Q_BAIL;
        ek.ids_cap = sk.bail_cap;
        ek.queue = kp.queue + Q_EV2;
        ek.bail_n = kp.queue + Q_BAIL2;
        bail_word = Q_BAIL2;
      }
      const uint64_t eres = (uint64_t)eocc * (uint64_t)cus;
      const unsigned egrid = (unsigned)std::min<uint64_t>((nc + 63) / 64, eres);
#ifdef PXB_WAVE_TIMES
      if (!g_wt) HIPCHK(hipMalloc(&g_wt, 6ull * 65536 * sizeof(unsigned long long)));
      ek.dbg = split ? nullptr : g_wt;
      if (!split) g_wt_waves = egrid;
#endif
      hipLaunchKernelGGL(efn, dim3(egrid), dim3(64), 0, st, ek);
      if (hipError_t e = hipGetLastError()) return fail(e);
      if (fail_after_first) return fail(hipErrorLaunchFailure);
      kp.ids = bail;
      kp.n_ids = kp.queue + bail_word;
      kp.ids_cap = bail_cap;
      hipLaunchKernelGGL(fn.fn, dim3((unsigned)resident), dim3(64 * fn.wpb), 0, st, kp);
      if (hipError_t e = hipGetLastError()) return fail(e);
    } else {
      const uint64_t waves_needed = (nc + G - 1) / G;
      const uint64_t blocks_needed = (waves_needed + wpb - 1) / wpb;
      const unsigned grid = (unsigned)std::min<uint64_t>(blocks_needed, resident);
#ifdef PXB_WAVE_TIMES
      if (!g_wt) HIPCHK(hipMalloc(&g_wt, 6ull * 65536 * sizeof(unsigned long long)));
      kp.dbg = g_wt;
      g_wt_waves = grid * fn.wpb;
      if (grid * fn.wpb > 65536) return PXB_E_INVAL;
#endif
      hipLaunchKernelGGL(fn.fn, dim3(grid), dim3(64 * fn.wpb), 0, st, kp);
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(TCOPIES), 0, st, kp.part, kp.part + ROWS_U64, kp.queue,
                       bail_word, bail_cap, totals, g_slots[dev] + HAND_U64);
    if (hipError_t e = hipGetLastError()) return fail(e);
  }
  return PXB_OK;
}

int pxb_run(const pxb_config* cfg, pxb_result* out, uint32_t* log_digest, pxb_acceptor_rec* acc,
            pxb_counters* totals) {
  int rc = validate(cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  const uint64_t n = cfg->n_instances, N = cfg->n_acceptors;
  pxb_result* d_out = nullptr;
  uint32_t* d_dig = nullptr;
  pxb_acceptor_rec* d_acc = nullptr;
  int64_t* d_tot = nullptr;
  hipError_t e = hipSuccess;
  rc = PXB_OK;
  do {
    if (out && n && (e = hipMalloc(&d_out, n * sizeof(pxb_result))) != hipSuccess) break;
    if (log_digest && n && (e = hipMalloc(&d_dig, n * N * sizeof(uint32_t))) != hipSuccess) break;
    if (acc && n && (e = hipMalloc(&d_acc, n * N * sizeof(pxb_acceptor_rec))) != hipSuccess) break;
    if ((e = hipMalloc(&d_tot, PXB_NCOUNTERS * sizeof(int64_t))) != hipSuccess) break;
    if ((e = hipMemset(d_tot, 0, PXB_NCOUNTERS * sizeof(int64_t))) != hipSuccess) break;
    rc = pxb_run_device(cfg, d_out, d_dig, d_acc, d_tot, nullptr);
    if (rc) break;
    if ((e = hipDeviceSynchronize()) != hipSuccess) break;
    if (out && n && (e = hipMemcpy(out, d_out, n * sizeof(pxb_result), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (log_digest && n &&
        (e = hipMemcpy(log_digest, d_dig, n * N * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (acc && n && (e = hipMemcpy(acc, d_acc, n * N * sizeof(pxb_acceptor_rec), hipMemcpyDeviceToHost)) != hipSuccess)
      break;
    if (totals && (e = hipMemcpy(totals->c, d_tot, PXB_NCOUNTERS * sizeof(int64_t), hipMemcpyDeviceToHost)) != hipSuccess)
      break;
  } while (0);
  if (e != hipSuccess) rc = hip_fail(e);
  if (d_out) (void)hipFree(d_out);
  if (d_dig) (void)hipFree(d_dig);
  if (d_acc) (void)hipFree(d_acc);
  if (d_tot) (void)hipFree(d_tot);
  return rc;
}

static int run_hook(bool acceptor, void* st, size_t st_bytes, uint32_t n_acc, const pxb_msg* in, pxb_msg* out,
                    size_t out_n, uint32_t* nb, uint32_t count) {
  if (!st || !in || !out || (!acceptor && !nb)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  void *d_st = nullptr, *d_in = nullptr, *d_out = nullptr, *d_nb = nullptr;
  hipError_t e = hipSuccess;
  do {
    if ((e = hipMalloc(&d_st, st_bytes * count)) != hipSuccess) break;
    if ((e = hipMalloc(&d_in, sizeof(pxb_msg) * count)) != hipSuccess) break;
    if ((e = hipMalloc(&d_out, sizeof(pxb_msg) * out_n * count)) != hipSuccess) break;
    if (!acceptor && (e = hipMalloc(&d_nb, sizeof(uint32_t) * count)) != hipSuccess) break;
    if ((e = hipMemcpy(d_st, st, st_bytes * count, hipMemcpyHostToDevice)) != hipSuccess) break;
    if ((e = hipMemcpy(d_in, in, sizeof(pxb_msg) * count, hipMemcpyHostToDevice)) != hipSuccess) break;
    const unsigned grid = (count + 255) / 256;
    if (acceptor)
      hipLaunchKernelGGL(acceptor_hook_kernel, dim3(grid), dim3(256), 0, 0, (pxb_acceptor_rec*)d_st,
                         (const pxb_msg*)d_in, (pxb_msg*)d_out, count);
    else
      hipLaunchKernelGGL(proposer_hook_kernel, dim3(grid), dim3(256), 0, 0, (pxb_proposer_rec*)d_st, n_acc,
                         (const pxb_msg*)d_in, (pxb_msg*)d_out, (uint32_t*)d_nb, count);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipDeviceSynchronize()) != hipSuccess) break;
    if ((e = hipMemcpy(st, d_st, st_bytes * count, hipMemcpyDeviceToHost)) != hipSuccess) break;
    if ((e = hipMemcpy(out, d_out, sizeof(pxb_msg) * out_n * count, hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (!acceptor && (e = hipMemcpy(nb, d_nb, sizeof(uint32_t) * count, hipMemcpyDeviceToHost)) != hipSuccess) break;
  } while (0);
  if (d_st) (void)hipFree(d_st);
  if (d_in) (void)hipFree(d_in);
  if (d_out) (void)hipFree(d_out);
  if (d_nb) (void)hipFree(d_nb);
  return (e == hipSuccess) ? PXB_OK : hip_fail(e);
}

int pxb_acceptor_handle(pxb_acceptor_rec* states, const pxb_msg* req, pxb_msg* reply, uint32_t count) {
  return run_hook(true, states, sizeof(pxb_acceptor_rec), 0, req, reply, 1, nullptr, count);
}

int pxb_proposer_handle(pxb_proposer_rec* states, uint32_t n_acceptors, const pxb_msg* msg, pxb_msg* bcast,
                        uint32_t* n_bcast, uint32_t count) {
  if (n_acceptors < PXB_MIN_ACCEPTORS || n_acceptors > PXB_MAX_ACCEPTORS) return PXB_E_INVAL;
  return run_hook(false, states, sizeof(pxb_proposer_rec), n_acceptors, msg, bcast, 2, n_bcast, count);
}

}  // extern "C"
