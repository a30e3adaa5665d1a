// shard_host.cpp — TEST ONLY: drives shard_runner.h (the phase order of
// pxb_run_multi, paxos_multi.cpp) with a fake backend on the host, so the
// failure handling is checked without GPUs: a shard that fails in setup or
// compute must make the call return its error with NO collective issued (a
// real all-reduce would then block the healthy devices forever), a failing
// collective must be aborted, and every shard that was set up is torn down.
#include <atomic>
#include <chrono>
#include <thread>

#include "../../cloud-haskell-paxos_amd/csrc/shard_runner.h"

namespace {

struct Fake {
  int fail_phase;     // 0 none, 1 setup, 2 compute, 3 reduce, 4 fetch
  int fail_shard;
  std::atomic<int> setups{0}, computes{0}, reduces{0}, aborts{0}, fetches{0}, teardowns{0};
  int setup(int g) {
    setups++;
    return (fail_phase == 1 && g == fail_shard) ? -2 : 0;
  }
  int compute(int g) {
    std::this_thread::sleep_for(std::chrono::milliseconds(2 * (g % 3)));   // uneven shards
    computes++;
    return (fail_phase == 2 && g == fail_shard) ? -3 : 0;
  }
  int reduce_all() {
    reduces++;
    return fail_phase == 3 ? -5 : 0;
  }
  void abort_reduce() { aborts++; }
  int fetch(int g) {
    fetches++;
    return (fail_phase == 4 && g == fail_shard) ? -2 : 0;
  }
  void teardown(int) { teardowns++; }
};

}  // namespace

extern "C" int shard_test(int G, int fail_phase, int fail_shard, int* counts /* 6 */) {
  Fake f;
  f.fail_phase = fail_phase;
  f.fail_shard = fail_shard;
  const int rc = pxb::run_shards(f, G);
  counts[0] = f.setups;
  counts[1] = f.computes;
  counts[2] = f.reduces;
  counts[3] = f.aborts;
  counts[4] = f.fetches;
  counts[5] = f.teardowns;
  return rc;
}
