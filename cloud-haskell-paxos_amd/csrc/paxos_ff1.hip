// paxos_ff1.hip — explicit instantiations of the fault-free single-proposer
// per-lane kernel (paxos_ff1.h) for the 8 acceptor counts.
#include "paxos_ff1.h"

namespace pxb {
namespace ff1 {
#define PXB_FF1_INST(N) template __global__ void paxos_ff1_kernel<N>(Ff1Params);
PXB_FF1_INST(2) PXB_FF1_INST(3) PXB_FF1_INST(4) PXB_FF1_INST(5)
PXB_FF1_INST(6) PXB_FF1_INST(7) PXB_FF1_INST(8) PXB_FF1_INST(9)
}  // namespace ff1
}  // namespace pxb
