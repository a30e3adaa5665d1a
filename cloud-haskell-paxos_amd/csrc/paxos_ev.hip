// paxos_ev.hip — explicit instantiations of the per-lane kernel
// (paxos_ev_kernel.h) for one proposer count (-DPXB_EV_P=1|2|3): 8 acceptor
// counts x {8, 16}-step timing wheels (plus the compact-link
// layout with the 8- and 4-step wheels, the log-mode fields on the 8-step
// wheel, the slim 8-step layout, and the tight layout 7 for P = 2).  Split by P so the units build in
// parallel.
#include "paxos_ev_kernel.h"

#if !defined(PXB_EV_P)
#error "compile with -DPXB_EV_P=1|2|3"
#endif

namespace pxb {
namespace ev {
#define PXB_EV_INST(N, W, C, L, S, SP) template __global__ void paxos_ev_kernel<PXB_EV_P, N, W, C, L, S, SP>(EvKParams);
#define PXB_EV_FOR_N(W, C, L, S, SP) PXB_EV_INST(2, W, C, L, S, SP) PXB_EV_INST(3, W, C, L, S, SP) \
  PXB_EV_INST(4, W, C, L, S, SP) PXB_EV_INST(5, W, C, L, S, SP) PXB_EV_INST(6, W, C, L, S, SP) \
  PXB_EV_INST(7, W, C, L, S, SP) PXB_EV_INST(8, W, C, L, S, SP) PXB_EV_INST(9, W, C, L, S, SP)
// (PXB_EV_PART 0: the wide, compact and simple-schedule shapes; 1: the log-mode
// and slim ones -- two units per proposer count, so that each builds in
// parallel and takes its own scheduler flags, __graft_entry__.py)
#if !defined(PXB_EV_PART) || PXB_EV_PART == 0
PXB_EV_FOR_N(8, false, false, false, false)
PXB_EV_FOR_N(16, false, false, false, false)
PXB_EV_FOR_N(8, true, false, false, false)
PXB_EV_FOR_N(4, true, false, false, false)
PXB_EV_FOR_N(4, true, false, false, 1)         // simple schedule (layout 6)
#if PXB_EV_P == 2
PXB_EV_FOR_N(4, true, false, false, 2)         // tight simple schedule (layout 7; two proposers only)
#endif
#endif
#if !defined(PXB_EV_PART) || PXB_EV_PART == 1
PXB_EV_FOR_N(8, false, true, false, false)     // log mode
PXB_EV_FOR_N(16, false, true, false, false)    // log mode, second stage (layout 8: 16-step wheel, larger pool)
PXB_EV_FOR_N(8, false, false, true, false)     // slim
PXB_EV_FOR_N(4, false, true, true, false)      // log mode, slim, 4-step wheel (layout 9)
#endif
}  // namespace ev
}  // namespace pxb
