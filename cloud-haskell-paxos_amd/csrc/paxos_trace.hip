// paxos_trace.hip — pxb_trace_instance: one instance through the per-lane state
// machine (paxos_ev.h) on one GPU lane, with its state recorded at the end of
// every visited step: the device counterpart of the reference's per-message
// `say` dumps (Server.hs:85, Client.hs:108), used to localise a parity break.
#include <hip/hip_runtime.h>
#include <string.h>

#include "../../include/paxos_batch.h"
#include "paxos_ev_kernel.h"

namespace pxb {
namespace ev {

template <class Lane>
__device__ void trace_record(const Lane& L, uint32_t step, pxb_trace_step* r) {
  constexpr int PM = Lane::S::PM, N = Lane::S::N;
  constexpr bool LG = Lane::S::LG;
  constexpr bool EARLY = Lane::kEarly;
  r->step = step;
  // (production variant: copies of a broadcast still to send are not on the
  // links yet, so the count is not the oracle's end-of-step one)
  r->in_flight = (EARLY && L.pq_len != 0u) ? PXB_TRACE_IN_FLIGHT_UNKNOWN : L.links_in_flight();
  r->n_acceptors = N;
  r->n_proposers = L.P;
  for (int a = 0; a < PXB_MAX_ACCEPTORS; ++a) {
    uint32_t rec[4] = {0, 0, 0, 0};
    if (a < N) L.record_of(a, rec);
    r->acc[a].t_max = (int32_t)rec[0];
    r->acc[a].t_store = (int32_t)rec[1];
    r->acc[a].val = rec[2];
    r->acc[a].meta = rec[3];
    r->log_digest[a] = a < N ? L.digest_of(a) : 0u;
  }
  for (int p = 0; p < PXB_MAX_PROPOSERS; ++p) {
    pxb_trace_prop q = {0, 0, 0, 0, 0, 0, 0, 0};
    if (p < PM && (uint32_t)p < L.P) {
      q.ticket = (int32_t)L.p_ticket(p);
      q.acks = L.p_acks(p);
      q.state = L.p_state(p);
      q.mr_t = (int32_t)L.p_mr_t(p);
      q.pending = L.p_pending(p);
      if constexpr (LG) {
        // log mode: 14-bit commands id [13:12] | t [11:0] (mr_v | r2_v << 14 in
        // pw1), the proposer's own command c<p+1>.<t> with t in pw2 (0: Nothing)
        const uint32_t mv = L.pw1[p] & 0x3FFFu, rv = (L.pw1[p] >> 14) & 0x3FFFu, ct = L.pw2[p];
        q.cmd = ct ? (((uint32_t)p + 1u) << 24) | ct : 0u;
        q.mr_v = mv ? Lane::code_of(mv) : 0u;
        q.r2_v = rv ? Lane::code_of(rv) : 0u;
      } else {
        const uint32_t code = 1u;   // every command is c<id>.1 (docs/SEMANTICS.md §2)
        q.cmd = L.p_cmd(p) ? ((L.p_cmd(p) << 24) | code) : 0u;
        q.mr_v = L.p_mr_v(p) ? ((L.p_mr_v(p) << 24) | code) : 0u;
        q.r2_v = L.p_r2_v(p) ? ((L.p_r2_v(p) << 24) | code) : 0u;
      }
    }
    r->prop[p] = q;
  }
}

// one wave, lane 0 runs the instance; status[0] = records written,
// status[1] = 1 bailed / 2 out of records.  EARLY = false (the default trace):
// every step drains its copies, so each record is the oracle's end-of-step
// state exactly; EARLY = true (PXB_CFG_TRACE_PRODUCTION): the carry-over
// variant the batch kernels run (paxos_ev.h, end_op), recorded on entering the
// next step.
// LG: log mode (several Ticks per proposer, logs of commands c<id>.<t>): the
// batch kernels' log-mode shape (layout 4, EvLane<..., LG = true>, 8-step wheel)
template <int PM, int N, int W, bool EARLY, bool LG = false>
__global__ __launch_bounds__(64) void paxos_trace_kernel(EvParams p, uint32_t gid, pxb_trace_step* out, uint32_t max,
                                                         uint32_t* status, uint4* res) {
  constexpr int POOL = EvPool<PM, N, false, LG>::value;
  using S = Shape<PM, N, POOL, W, false, LG>;
  __shared__ uint32_t lds[S::WORDS * 64];
  if (threadIdx.x != 0) return;
  EvLane<PM, N, POOL, W, false, LdsMem, EARLY, LG> L;
  L.m = LdsMem{lds, 0u};
  L.set_keys(p);
  L.init(p, gid);
  uint32_t n = 0;
  for (;;) {
    const int32_t s0 = L.s;
    EvOut o;
    const bool done = L.step(p, o);
    if (L.bailed) {
      status[1] = 1u;
      break;
    }
    if (done || L.s != s0) {
      const uint32_t step = (uint32_t)(done ? L.s : s0);
      // (production variant: an instance whose carried step held only lost
      // copies ends at the step before it, already recorded: rewrite that record)
      const bool again = EARLY && done && n > 0 && out[n - 1].step == step;
      if (!again && n >= max) {
        status[1] = 2u;
        break;
      }
      trace_record(L, step, out + (again ? n - 1 : n));
      n += again ? 0u : 1u;
    }
    if (done) {
      *res = make_uint4(o.res[0], o.res[1], o.res[2], o.res[3]);
      break;
    }
  }
  status[0] = n;
}

typedef void (*trace_ptr)(EvParams, uint32_t, pxb_trace_step*, uint32_t, uint32_t*, uint4*);

template <int PM, int W, bool E, bool LG = false>
static trace_ptr pick_n(uint32_t n) {
  switch (n) {
    case 2: return paxos_trace_kernel<PM, 2, W, E, LG>;
    case 3: return paxos_trace_kernel<PM, 3, W, E, LG>;
    case 4: return paxos_trace_kernel<PM, 4, W, E, LG>;
    case 5: return paxos_trace_kernel<PM, 5, W, E, LG>;
    case 6: return paxos_trace_kernel<PM, 6, W, E, LG>;
    case 7: return paxos_trace_kernel<PM, 7, W, E, LG>;
    case 8: return paxos_trace_kernel<PM, 8, W, E, LG>;
    case 9: return paxos_trace_kernel<PM, 9, W, E, LG>;
  }
  return nullptr;
}

// (log mode: the 8-step wheel only, as the batch kernels' LG shape)
template <bool E>
static trace_ptr pick(uint32_t pm, uint32_t n, int w, bool lg) {
  switch (pm * 1000 + (lg ? 500u : 0u) + (uint32_t)w) {
    case 1008: return pick_n<1, 8, E>(n);
    case 1016: return pick_n<1, 16, E>(n);
    case 2008: return pick_n<2, 8, E>(n);
    case 2016: return pick_n<2, 16, E>(n);
    case 3008: return pick_n<3, 8, E>(n);
    case 3016: return pick_n<3, 16, E>(n);
    case 1508: return pick_n<1, 8, E, true>(n);
    case 2508: return pick_n<2, 8, E, true>(n);
    case 3508: return pick_n<3, 8, E, true>(n);
  }
  return nullptr;
}

}  // namespace ev
}  // namespace pxb

extern "C" int pxb_trace_instance(const pxb_config* cfg, uint64_t instance, pxb_trace_step* out, uint32_t max_records,
                                  uint32_t* n_records, pxb_result* result) {
  using namespace pxb::ev;
  if (!cfg || !out || !n_records || max_records == 0) return PXB_E_INVAL;
  if (cfg->n_proposers < 1 || cfg->n_proposers > PXB_MAX_PROPOSERS || cfg->n_acceptors < PXB_MIN_ACCEPTORS ||
      cfg->n_acceptors > PXB_MAX_ACCEPTORS || cfg->delay_max < 1 || cfg->delay_max > PXB_MAX_DELAY ||
      cfg->step_cap < 1 || !eligible(cfg))
    return PXB_E_INVAL;
  // log mode (n_ticks > 1, ABI 5): the batch kernels' log-mode shape (its
  // ticker, 14-bit commands, Execute-driven logs); eligible() holds its delays
  // to the 8-step wheel
  if (cfg->n_ticks > PXB_MAX_TICKS || (cfg->n_ticks > 1 && (cfg->tick_period < 1 || cfg->tick_period > PXB_MAX_STEP_CAP)))
    return PXB_E_INVAL;
  const bool lg = cfg->n_ticks > 1;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  const bool prod = (cfg->flags & PXB_CFG_TRACE_PRODUCTION) != 0u;
  const trace_ptr fn = prod ? pick<true>(cfg->n_proposers, cfg->n_acceptors, wheel_for(cfg->delay_max), lg)
                            : pick<false>(cfg->n_proposers, cfg->n_acceptors, wheel_for(cfg->delay_max), lg);
  if (!fn) return PXB_E_INVAL;
  EvParams p = make_params(cfg);
  p.first_instance = instance;
  pxb_trace_step* d_out = nullptr;
  uint32_t* d_st = nullptr;
  uint4* d_res = nullptr;
  int rc = PXB_OK;
  hipError_t e = hipSuccess;
  uint32_t st[2] = {0, 0};
  do {
    if ((e = hipMalloc(&d_out, (size_t)max_records * sizeof(pxb_trace_step))) != hipSuccess) break;
    if ((e = hipMalloc(&d_st, 2 * sizeof(uint32_t))) != hipSuccess) break;
    if ((e = hipMalloc(&d_res, sizeof(uint4))) != hipSuccess) break;
    if ((e = hipMemset(d_st, 0, 2 * sizeof(uint32_t))) != hipSuccess) break;
    hipLaunchKernelGGL(fn, dim3(1), dim3(64), 0, 0, p, 0u, d_out, max_records, d_st, d_res);
    if ((e = hipGetLastError()) != hipSuccess) break;
    if ((e = hipDeviceSynchronize()) != hipSuccess) break;
    if ((e = hipMemcpy(st, d_st, sizeof(st), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (st[1]) {
      rc = PXB_E_INVAL;
      break;
    }
    if ((e = hipMemcpy(out, d_out, (size_t)st[0] * sizeof(pxb_trace_step), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (result && (e = hipMemcpy(result, d_res, sizeof(uint4), hipMemcpyDeviceToHost)) != hipSuccess) break;
    *n_records = st[0];
  } while (0);
  if (d_out) (void)hipFree(d_out);
  if (d_st) (void)hipFree(d_st);
  if (d_res) (void)hipFree(d_res);
  if (e != hipSuccess) return (e == hipErrorOutOfMemory) ? PXB_E_OOM : PXB_E_HIP;
  return rc;
}
