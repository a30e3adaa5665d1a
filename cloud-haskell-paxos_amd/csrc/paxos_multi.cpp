// paxos_multi.cpp — multi-GPU entry of the C ABI (pxb_run_multi).
//
// One host thread per device runs the device's contiguous share of the global
// instance range (instances share no state — Main.hs:41-45,
// Server.hs:58-71 — and every Philox draw is keyed by the GLOBAL instance id,
// so results do not depend on the device count).  The only collective is one
// RCCL all-reduce (sum, int64 x PXB_NCOUNTERS) of the run totals over xGMI,
// issued once per run by every device thread on its own communicator.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string.h>
#include <thread>
#include <vector>

#include "../../include/paxos_batch.h"

namespace {

std::mutex g_comm_mu;
std::vector<ncclComm_t> g_comms;   // cached communicator set for devices 0..n-1

int comms_for(int n, std::vector<ncclComm_t>& out) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  if ((int)g_comms.size() != n) {
    for (ncclComm_t c : g_comms) ncclCommDestroy(c);
    g_comms.assign(n, nullptr);
    std::vector<int> devs(n);
    for (int i = 0; i < n; ++i) devs[i] = i;
    if (ncclCommInitAll(g_comms.data(), n, devs.data()) != ncclSuccess) {
      g_comms.clear();
      return PXB_E_RCCL;
    }
  }
  out = g_comms;
  return PXB_OK;
}

}  // namespace

extern "C" {

// Same outputs as pxb_run (host buffers, all nullable) for a batch sharded over
// devices 0..n_devices-1 (n_devices <= 0: every visible device).  totals are the
// RCCL-all-reduced run totals.
int pxb_run_multi(const pxb_config* cfg, int n_devices, pxb_result* out, uint32_t* log_digest,
                  pxb_acceptor_rec* acc, pxb_counters* totals) {
  if (!cfg) return PXB_E_INVAL;
  int visible = 0;
  if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) return PXB_E_NODEV;
  const int G = (n_devices <= 0) ? visible : n_devices;
  if (G > visible) return PXB_E_INVAL;
  std::vector<ncclComm_t> comms;
  int rc = comms_for(G, comms);
  if (rc) return rc;
  const uint64_t n = cfg->n_instances, N = cfg->n_acceptors;
  std::vector<int> rcs(G, PXB_OK);
  std::vector<int64_t> host_tot((size_t)G * PXB_NCOUNTERS, 0);
  std::vector<std::thread> th;
  for (int g = 0; g < G; ++g) {
    th.emplace_back([&, g]() {
      const uint64_t lo = n * (uint64_t)g / (uint64_t)G, hi = n * (uint64_t)(g + 1) / (uint64_t)G;
      pxb_config c = *cfg;
      c.first_instance = cfg->first_instance + lo;
      c.n_instances = hi - lo;
      int r = PXB_OK;
      pxb_result* d_out = nullptr;
      uint32_t* d_dig = nullptr;
      pxb_acceptor_rec* d_acc = nullptr;
      int64_t* d_tot = nullptr;
      hipStream_t st = nullptr;
      do {
        if (hipSetDevice(g) != hipSuccess || hipStreamCreate(&st) != hipSuccess) { r = PXB_E_HIP; break; }
        if (hipMalloc(&d_tot, PXB_NCOUNTERS * sizeof(int64_t)) != hipSuccess) { r = PXB_E_OOM; break; }
        const uint64_t m = c.n_instances;
        if (out && m && hipMalloc(&d_out, m * sizeof(pxb_result)) != hipSuccess) { r = PXB_E_OOM; break; }
        if (log_digest && m && hipMalloc(&d_dig, m * N * sizeof(uint32_t)) != hipSuccess) { r = PXB_E_OOM; break; }
        if (acc && m && hipMalloc(&d_acc, m * N * sizeof(pxb_acceptor_rec)) != hipSuccess) { r = PXB_E_OOM; break; }
        if (hipMemsetAsync(d_tot, 0, PXB_NCOUNTERS * sizeof(int64_t), st) != hipSuccess) { r = PXB_E_HIP; break; }
        r = pxb_run_device(&c, d_out, d_dig, d_acc, d_tot, st);
        if (r) break;
        if (hipStreamSynchronize(st) != hipSuccess) { r = PXB_E_HIP; break; }
        if (out && m && hipMemcpy(out + lo, d_out, m * sizeof(pxb_result), hipMemcpyDeviceToHost) != hipSuccess) { r = PXB_E_HIP; break; }
        if (log_digest && m &&
            hipMemcpy(log_digest + lo * N, d_dig, m * N * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) { r = PXB_E_HIP; break; }
        if (acc && m &&
            hipMemcpy(acc + lo * N, d_acc, m * N * sizeof(pxb_acceptor_rec), hipMemcpyDeviceToHost) != hipSuccess) { r = PXB_E_HIP; break; }
      } while (0);
      rcs[g] = r;
      // the run's one collective: every device joins it (with zeros on failure)
      if (d_tot && st) {
        if (ncclAllReduce(d_tot, d_tot, PXB_NCOUNTERS, ncclInt64, ncclSum, comms[g], st) != ncclSuccess)
          rcs[g] = PXB_E_RCCL;
        else if (hipStreamSynchronize(st) != hipSuccess ||
                 hipMemcpy(&host_tot[(size_t)g * PXB_NCOUNTERS], d_tot, PXB_NCOUNTERS * sizeof(int64_t),
                           hipMemcpyDeviceToHost) != hipSuccess)
          rcs[g] = PXB_E_HIP;
      }
      if (d_out) (void)hipFree(d_out);
      if (d_dig) (void)hipFree(d_dig);
      if (d_acc) (void)hipFree(d_acc);
      if (d_tot) (void)hipFree(d_tot);
      if (st) (void)hipStreamDestroy(st);
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (rcs[g]) return rcs[g];
  if (totals) memcpy(totals->c, host_tot.data(), PXB_NCOUNTERS * sizeof(int64_t));   // rank 0's reduced copy
  return PXB_OK;
}

}  // extern "C"
