// paxos_inst.hip — explicit instantiations of the batch kernel for one
// proposer count and mode (-DPXB_INST_P=1|2|3 -DPXB_INST_LOGM=0|1): 8 acceptor
// counts x {faulty, fault-free}.  Split out so the six objects build in
// parallel.
#include "paxos_kernel.h"

#if !defined(PXB_INST_P) || !defined(PXB_INST_LOGM)
#error "compile with -DPXB_INST_P=1|2|3 -DPXB_INST_LOGM=0|1"
#endif

namespace pxb {
#define PXB_FOR_N(M, PM, LOGM, FF) M(PM, 2, LOGM, FF) M(PM, 3, LOGM, FF) M(PM, 4, LOGM, FF) M(PM, 5, LOGM, FF) \
  M(PM, 6, LOGM, FF) M(PM, 7, LOGM, FF) M(PM, 8, LOGM, FF) M(PM, 9, LOGM, FF)
#define PXB_INSTANTIATE(PM, N, LOGM, FF) template __global__ void paxos_batch_kernel<PM, N, LOGM, FF>(KParams);
PXB_FOR_N(PXB_INSTANTIATE, PXB_INST_P, (PXB_INST_LOGM != 0), false)
PXB_FOR_N(PXB_INSTANTIATE, PXB_INST_P, (PXB_INST_LOGM != 0), true)
}  // namespace pxb
