// paxos_multi.cpp — multi-GPU entry of the C ABI (pxb_run_multi).
//
// Each device runs its contiguous share of the global instance range on its own
// host thread (instances share no state — Main.hs:41-45,
// Server.hs:58-71 — and every Philox draw is keyed by the GLOBAL instance id,
// so results do not depend on the device count).  The only collective is one
// RCCL all-reduce (sum, int64 x PXB_NCOUNTERS) of the run totals over xGMI.
// shard_runner.h orders the phases so that the collective is issued for all
// devices together (one RCCL group from one thread) or not at all: a device
// that fails never leaves the others blocked in the all-reduce.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string.h>
#include <string>
#include <vector>

#include "../../include/paxos_batch.h"
#include "shard_runner.h"

extern "C" bool multi_fail_injected(const char* phase, int g);   // paxos_batch.hip

namespace {

std::mutex g_comm_mu;
// one pxb_run_multi at a time: concurrent calls would issue collectives on the
// same cached communicators (and a call with another device count would
// destroy them under the first); the per-device work inside a call is
// parallel, so this costs a multi-device host nothing
std::mutex g_multi_mu;
std::vector<ncclComm_t> g_comms;   // cached communicators ...
std::string g_comm_key;            // ... for this device list (PCI bus ids)

std::string device_key(int G) {
  std::string key;
  for (int g = 0; g < G; ++g) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), g) != hipSuccess) snprintf(bus, sizeof(bus), "dev%d", g);
    key += bus;
    key += ';';
  }
  return key;
}

void release_locked() {
  for (ncclComm_t c : g_comms)
    if (c) ncclCommDestroy(c);
  g_comms.clear();
  g_comm_key.clear();
}

int comms_for(int G, std::vector<ncclComm_t>& out) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  const std::string key = device_key(G);
  if (key != g_comm_key) {
    release_locked();
    g_comms.assign(G, nullptr);
    std::vector<int> devs(G);
    for (int i = 0; i < G; ++i) devs[i] = i;
    if (ncclCommInitAll(g_comms.data(), G, devs.data()) != ncclSuccess) {
      g_comms.clear();
      return PXB_E_RCCL;
    }
    g_comm_key = key;
  }
  out = g_comms;
  return PXB_OK;
}

// after a failed collective the communicators may hold half-issued work: abort
// and forget them (the next call builds new ones)
void abort_comms() {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  for (ncclComm_t c : g_comms)
    if (c) ncclCommAbort(c);
  g_comms.clear();
  g_comm_key.clear();
}

// tests: make device `g` fail in a phase ("setup" / "compute"), to check that
// the call returns the error promptly instead of hanging in the collective
// (PXB_MULTI_FAIL_PHASE / _DEVICE, read with the library's other test hooks)
bool injected(const char* phase, int g) { return multi_fail_injected(phase, g); }


struct HipShards {
  const pxb_config* cfg;
  int G;
  pxb_result* out;
  uint32_t* log_digest;
  pxb_acceptor_rec* acc;
  std::vector<ncclComm_t> comms;
  struct Dev {
    hipStream_t st = nullptr;
    pxb_result* d_out = nullptr;
    uint32_t* d_dig = nullptr;
    pxb_acceptor_rec* d_acc = nullptr;
    int64_t* d_tot = nullptr;
    uint64_t lo = 0, m = 0;
    int64_t tot[PXB_NCOUNTERS] = {0};
  };
  std::vector<Dev> dv;

  int setup(int g) {
    Dev& d = dv[g];
    const uint64_t n = cfg->n_instances, N = cfg->n_acceptors;
    d.lo = n * (uint64_t)g / (uint64_t)G;
    d.m = n * (uint64_t)(g + 1) / (uint64_t)G - d.lo;
    if (injected("setup", g)) return PXB_E_HIP;
    if (hipSetDevice(g) != hipSuccess || hipStreamCreate(&d.st) != hipSuccess) return PXB_E_HIP;
    if (hipMalloc(&d.d_tot, PXB_NCOUNTERS * sizeof(int64_t)) != hipSuccess) return PXB_E_OOM;
    if (out && d.m && hipMalloc(&d.d_out, d.m * sizeof(pxb_result)) != hipSuccess) return PXB_E_OOM;
    if (log_digest && d.m && hipMalloc(&d.d_dig, d.m * N * sizeof(uint32_t)) != hipSuccess) return PXB_E_OOM;
    if (acc && d.m && hipMalloc(&d.d_acc, d.m * N * sizeof(pxb_acceptor_rec)) != hipSuccess) return PXB_E_OOM;
    if (hipMemsetAsync(d.d_tot, 0, PXB_NCOUNTERS * sizeof(int64_t), d.st) != hipSuccess) return PXB_E_HIP;
    return PXB_OK;
  }

  int compute(int g) {
    Dev& d = dv[g];
    if (injected("compute", g)) return PXB_E_HIP;
    if (hipSetDevice(g) != hipSuccess) return PXB_E_HIP;
    pxb_config c = *cfg;
    c.first_instance = cfg->first_instance + d.lo;
    c.n_instances = d.m;
    if (int r = pxb_run_device(&c, d.d_out, d.d_dig, d.d_acc, d.d_tot, d.st)) return r;
    if (hipStreamSynchronize(d.st) != hipSuccess) return PXB_E_HIP;
    const uint64_t N = cfg->n_acceptors;
    if (out && d.m && hipMemcpy(out + d.lo, d.d_out, d.m * sizeof(pxb_result), hipMemcpyDeviceToHost) != hipSuccess)
      return PXB_E_HIP;
    if (log_digest && d.m &&
        hipMemcpy(log_digest + d.lo * N, d.d_dig, d.m * N * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
      return PXB_E_HIP;
    if (acc && d.m &&
        hipMemcpy(acc + d.lo * N, d.d_acc, d.m * N * sizeof(pxb_acceptor_rec), hipMemcpyDeviceToHost) != hipSuccess)
      return PXB_E_HIP;
    return PXB_OK;
  }

  // the run's one collective, issued for every device in one group
  int reduce_all() {
    if (ncclGroupStart() != ncclSuccess) return PXB_E_RCCL;
    bool ok = true;
    for (int g = 0; g < G; ++g)
      ok = ok && ncclAllReduce(dv[g].d_tot, dv[g].d_tot, PXB_NCOUNTERS, ncclInt64, ncclSum, comms[g], dv[g].st) ==
                     ncclSuccess;
    if (ncclGroupEnd() != ncclSuccess || !ok) return PXB_E_RCCL;
    return PXB_OK;
  }
  void abort_reduce() { abort_comms(); }

  int fetch(int g) {
    Dev& d = dv[g];
    if (hipSetDevice(g) != hipSuccess || hipStreamSynchronize(d.st) != hipSuccess) return PXB_E_HIP;
    if (hipMemcpy(d.tot, d.d_tot, PXB_NCOUNTERS * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
      return PXB_E_HIP;
    return PXB_OK;
  }

  void teardown(int g) {
    Dev& d = dv[g];
    (void)hipSetDevice(g);
    if (d.st) (void)hipStreamSynchronize(d.st);
    if (d.d_out) (void)hipFree(d.d_out);
    if (d.d_dig) (void)hipFree(d.d_dig);
    if (d.d_acc) (void)hipFree(d.d_acc);
    if (d.d_tot) (void)hipFree(d.d_tot);
    if (d.st) {
      pxb_stream_release(g, d.st);      // (its bailed-id lists go back to the device's pool)
      (void)hipStreamDestroy(d.st);
    }
    d.st = nullptr;                  // (the fetched totals stay: they are the result)
    d.d_out = nullptr;
    d.d_dig = nullptr;
    d.d_acc = nullptr;
    d.d_tot = nullptr;
  }
};

}  // namespace

extern "C" {

// internal (pxb_shutdown): destroy the cached communicators
void pxb_multi_release(void) {
  std::lock_guard<std::mutex> lk(g_comm_mu);
  release_locked();
}

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
  std::lock_guard<std::mutex> serial(g_multi_mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  HipShards b{cfg, G, out, log_digest, acc, {}, std::vector<HipShards::Dev>(G)};
  if (int rc = comms_for(G, b.comms)) return rc;
  const int rc = pxb::run_shards(b, G);
  (void)hipSetDevice(cur);
  if (rc) return rc;
  if (totals) memcpy(totals->c, b.dv[0].tot, PXB_NCOUNTERS * sizeof(int64_t));   // the reduced totals
  return PXB_OK;
}

}  // extern "C"
