// Reproducer (diagnostic, not built into the library): the ROCm 7.2 / clang-22
// AMDGPU backend segfaults in the greedy register allocator
// (VirtRegAuxInfo::isRematerializable) on one per-lane kernel shape when the
// iterative-ILP machine scheduler is on and the one-hot selects are inline-asm
// v_bfi_b32 (the library's form; -DPXB_EV_BITOP3_BFI swaps in the builtin
// v_bitop3_b32, which compiles).  See repro.sh.
#include "../../cloud-haskell-paxos_amd/csrc/paxos_ev_kernel.h"

namespace pxb {
namespace ev {
template __global__ void paxos_ev_kernel<3, 2, 8, false>(EvKParams);
}  // namespace ev
}  // namespace pxb
