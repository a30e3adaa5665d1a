// shard_runner.h — failure-safe orchestration of a run sharded over devices
// (pxb_run_multi, paxos_multi.cpp).  Backend-agnostic so the failure handling
// is unit-tested on the host with a fake backend (tests/native/shard_host.cpp).
//
// The reference's instances share nothing (Main.hs:41-45), so a node run is G
// independent device runs plus ONE collective: the all-reduce of the run
// totals.  A collective that only some devices join blocks
// the others forever, so the phases are:
//   1. setup    every device in its own thread (device, stream, buffers);
//   2. compute  every device in its own thread (its instance range);
//   3. reduce   only if every device got here without error: the G
//               all-reduce calls are issued together from THIS thread (one
//               RCCL group), so either all devices join or none does;
//   4. fetch    every device in its own thread (its reduced totals);
//   5. teardown every device that was set up, whatever happened.
// Any failure returns its error code after teardown; no thread is left waiting.
#pragma once
#include <functional>
#include <thread>
#include <vector>

namespace pxb {

inline void for_each_shard(int G, const std::function<void(int)>& f) {
  std::vector<std::thread> th;
  th.reserve(G);
  for (int g = 0; g < G; ++g) th.emplace_back(f, g);
  for (auto& t : th) t.join();
}

// Backend B: int setup(int g); int compute(int g); int reduce_all();
//            void abort_reduce(); int fetch(int g); void teardown(int g).
template <class B>
int run_shards(B& b, int G) {
  std::vector<int> rc(G, 0), up(G, 0);
  auto first_error = [&]() {
    for (int g = 0; g < G; ++g)
      if (rc[g]) return rc[g];
    return 0;
  };
  auto finish = [&](int r) {
    for_each_shard(G, [&](int g) {
      if (up[g]) b.teardown(g);
    });
    return r;
  };
  for_each_shard(G, [&](int g) {
    rc[g] = b.setup(g);
    up[g] = 1;                       // teardown also undoes a partial setup
  });
  if (int r = first_error()) return finish(r);
  for_each_shard(G, [&](int g) { rc[g] = b.compute(g); });
  if (int r = first_error()) return finish(r);
  if (int r = b.reduce_all()) {
    b.abort_reduce();
    return finish(r);
  }
  for_each_shard(G, [&](int g) { rc[g] = b.fetch(g); });
  return finish(first_error());
}

}  // namespace pxb
