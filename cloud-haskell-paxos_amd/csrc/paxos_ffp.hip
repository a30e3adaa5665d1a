// paxos_ffp.hip — explicit instantiations of the fault-free per-lane kernel for
// duelling proposers and log mode (paxos_ffp.h): P = 1..3 x 8 acceptor counts.
#include "paxos_ffp.h"

namespace pxb {
namespace ffp {
#define PXB_FFP_INST(P, N) template __global__ void paxos_ffp_kernel<P, N>(FfpParams);
#define PXB_FFP_FOR_N(P) PXB_FFP_INST(P, 2) PXB_FFP_INST(P, 3) PXB_FFP_INST(P, 4) PXB_FFP_INST(P, 5) \
  PXB_FFP_INST(P, 6) PXB_FFP_INST(P, 7) PXB_FFP_INST(P, 8) PXB_FFP_INST(P, 9)
PXB_FFP_FOR_N(1)
PXB_FFP_FOR_N(2)
PXB_FFP_FOR_N(3)
}  // namespace ffp
}  // namespace pxb
