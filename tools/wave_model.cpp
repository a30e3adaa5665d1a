// wave_model.cpp — host model of the per-lane kernel's wave loop
// (paxos_ev_kernel.h): 64 EvLane state machines in lockstep, refilled from
// 64-instance chunks, one iteration of every live lane per wave-iteration.
// Reports how often each wave-level branch region of the loop body runs (a
// region runs when any lane of the wave needs it), the slot use of the
// predicated ops, and refill / output frequencies.  With the per-block
// instruction counts of tools/isa_budget.py this gives the dynamic
// instruction budget per instance (profiles/r04_notes/ev_budget.txt).
//
//   hipcc -O2 -std=c++17 -DPXB_EV_PROBES -o /tmp/wave_model tools/wave_model.cpp
//   /tmp/wave_model <config 3|4|5|7> <n_instances> [refill_min]
//
// refill_min > 1 models a refill that waits until that many lanes are idle
// (or the wave has nothing else to run).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../cloud-haskell-paxos_amd/csrc/paxos_ev_kernel.h"

namespace pxb { namespace ev { thread_local uint32_t ev_probe_bits = 0; } }

using namespace pxb;
using namespace pxb::ev;

namespace {

struct HostMem {
  uint32_t* w;
  uint32_t ld(uint32_t i) const { return w[i]; }
  void st(uint32_t i, uint32_t v) const { w[i] = v; }
  uint32_t ld16(uint32_t base, uint32_t i) const { return reinterpret_cast<const uint16_t*>(w + base)[i]; }
  void st16(uint32_t base, uint32_t i, uint32_t v) const { reinterpret_cast<uint16_t*>(w + base)[i] = (uint16_t)v; }
  uint32_t ld16h(uint32_t i, uint32_t half) const { return reinterpret_cast<const uint16_t*>(w + i)[half]; }
  void st16h(uint32_t i, uint32_t half, uint32_t v) const { reinterpret_cast<uint16_t*>(w + i)[half] = (uint16_t)v; }
  uint32_t ldh(uint32_t base, uint32_t i) const { return ld16(base, i); }
  void sth(uint32_t base, uint32_t i, uint32_t v) const { st16(base, i, v); }
  void orw(uint32_t i, uint32_t v) const { w[i] |= v; }
};

constexpr int NB = 10;
const char* names[NB] = {"END", "FIN", "RUN", "TICK_ENTER", "TICK_END", "ACC", "PROP", "COPY", "SEND1", "BCAST"};

// (ids: run only these instances, as a second-stage kernel over another's
// hand-offs; bailed_out: the ids this shape hands on)
template <int PM, int N, int W, bool CMP, bool LG, bool SL, int SP = 0>
void model(const pxb_config* cfg, uint32_t n, uint32_t refill_min, const std::vector<uint32_t>* ids = nullptr,
           std::vector<uint32_t>* bailed_out = nullptr) {
  if (ids) n = (uint32_t)ids->size();
  constexpr int POOL = EvPool<PM, N, CMP, LG, SL, SP, W>::value;
  using S = Shape<PM, N, POOL, W, CMP, LG, SL, SP>;
  const EvParams p = make_params(cfg);
  using Lane = EvLane<PM, N, POOL, W, CMP, HostMem, true, LG, SL, SP>;
  std::vector<uint32_t> mem(64 * (S::WORDS + 1));
  std::vector<Lane> L(64);
  for (int l = 0; l < 64; ++l) {
    L[l].m = HostMem{&mem[l * (S::WORDS + 1)]};
    L[l].set_keys(p);
    L[l].mode = M_IDLE;
  }
  uint64_t wave_it = 0, live_lane_it = 0, any[NB] = {}, sum[NB] = {};
  uint64_t refills = 0, inits = 0, out_its = 0, outs = 0, bails = 0, bail_its = 0, done_inst = 0;
  uint64_t bcause[6] = {};
  uint32_t next = 0;
  for (;;) {
    // refill (the kernel: every idle lane, from the wave's chunk of the queue)
    int idle = 0, live = 0;
    for (int l = 0; l < 64; ++l) (L[l].mode == M_IDLE ? idle : live)++;
    if (idle && next < n && (idle >= (int)refill_min || live == 0)) {
      ++refills;
      for (int l = 0; l < 64 && next < n; ++l)
        if (L[l].mode == M_IDLE) {
          L[l].init(p, ids ? (*ids)[next] : next);
          ++next;
          ++inits;
          if (L[l].bailed) {
            if (bailed_out) bailed_out->push_back(L[l].gid);
            L[l].mode = M_IDLE;
            L[l].bailed = false;
            ++bails;
          }
        }
    }
    live = 0;
    for (int l = 0; l < 64; ++l) live += L[l].mode != M_IDLE;
    if (!live) {
      if (next >= n) break;
      continue;
    }
    ++wave_it;
    uint32_t orb = 0;
    bool anyout = false, anybail = false;
    for (int l = 0; l < 64; ++l) {
      if (L[l].mode == M_IDLE) continue;
      ++live_lane_it;
      ev_probe_bits = 0;
      EvOut o;
      const bool done = L[l].step(p, o);
      orb |= ev_probe_bits;
      for (int b = 0; b < NB; ++b) sum[b] += (ev_probe_bits >> b) & 1u;
      if (L[l].bailed) {
        if (bailed_out) bailed_out->push_back(L[l].gid);
        for (int b = 0; b < 6; ++b) bcause[b] += (ev_probe_bits >> (16 + b)) & 1u;
        L[l].mode = M_IDLE;
        L[l].bailed = false;
        ++bails;
        anybail = true;
      } else if (done) {
        ++outs;
        ++done_inst;
        anyout = true;
      }
    }
    for (int b = 0; b < NB; ++b) any[b] += (orb >> b) & 1u;
    out_its += anyout;
    bail_its += anybail;
  }
  const double I = (double)n;
  printf("instances %u (done %llu, bailed %llu), LDS words %d, pool %d\n", n, (unsigned long long)done_inst,
         (unsigned long long)bails, S::WORDS, POOL);
  printf("wave-iterations per instance %.2f; lane-iterations per instance %.2f; live lanes per wave-iteration %.2f\n",
         64.0 * wave_it / I, live_lane_it / I, (double)live_lane_it / wave_it);
  printf("refills per instance (wave-level) %.4f, lanes per refill %.2f; output blocks per instance %.4f\n",
         refills / I, (double)inits / refills, out_its / I);
  printf("bail causes (an instance may have several): ring %llu, response FIFO %llu, pool %llu, request FIFO %llu, "
         "log %llu, reply seq %llu\n", (unsigned long long)bcause[0], (unsigned long long)bcause[1],
         (unsigned long long)bcause[2], (unsigned long long)bcause[3], (unsigned long long)bcause[4],
         (unsigned long long)bcause[5]);
  printf("%-11s %10s %10s\n", "region", "wave-frac", "lane-frac");
  for (int b = 0; b < NB; ++b)
    printf("%-11s %10.4f %10.4f\n", names[b], (double)any[b] / wave_it, (double)sum[b] / live_lane_it);
}

}  // namespace

int main(int argc, char** argv) {
  const int c = argc > 1 ? atoi(argv[1]) : 4;
  const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 64 * 64;
  const uint32_t rmin = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
  pxb_config cfg{};
  cfg.first_instance = 0;
  cfg.n_instances = n;
  // BASELINE configs (pxb.CONFIGS)
  if (c == 3) {
    cfg.seed = 0x5EED0003; cfg.n_proposers = 2; cfg.n_acceptors = 5; cfg.loss_ppm = 100000;
    cfg.delay_max = 4; cfg.skew_max = 3; cfg.step_cap = 256;
    model<2, 5, 4, true, false, false>(&cfg, n, rmin);
  } else if (c == 4) {
    cfg.seed = 0x5EED0004; cfg.n_proposers = 2; cfg.n_acceptors = 7; cfg.delay_max = 4;
    cfg.crash_ppm = 200000; cfg.crash_len_max = 16; cfg.crash_start_max = 8; cfg.step_cap = 256;
    // (NACC=6 / 8: the other topologies the tight routing may take, P = 2, N * P <= 16)
    const int na = getenv("NACC") ? atoi(getenv("NACC")) : 7;
    cfg.n_acceptors = (uint32_t)na;
    const bool t = getenv("TIGHT") != nullptr;
    if (na == 6) t ? model<2, 6, 4, true, false, false, 2>(&cfg, n, rmin) : model<2, 6, 4, true, false, false, 1>(&cfg, n, rmin);
    else if (na == 8) t ? model<2, 8, 4, true, false, false, 2>(&cfg, n, rmin) : model<2, 8, 4, true, false, false, 1>(&cfg, n, rmin);
    else if (t) model<2, 7, 4, true, false, false, 2>(&cfg, n, rmin);   // layout 7 (tight)
    else model<2, 7, 4, true, false, false, 1>(&cfg, n, rmin);   // layout 6 (simple schedule)
  } else if (c == 5) {
    // the three-proposer slim shape over every instance (P <= 3 drawn per instance)
    cfg.seed = 0x5EED0005; cfg.n_proposers = 3; cfg.n_acceptors = 9; cfg.loss_ppm = 300000;
    cfg.delay_max = 8; cfg.crash_ppm = 200000; cfg.crash_len_max = 16; cfg.crash_start_max = 16;
    cfg.skew_max = 3; cfg.step_cap = 512; cfg.flags = PXB_CFG_RANDOMIZE;
    if (getenv("C5W4")) {   // (its delay_max <= 4 instances on the compact 4-step wheel)
      cfg.delay_max = 4;
      model<3, 9, 4, true, false, false>(&cfg, n, rmin);
    } else if (getenv("C5SW4")) {
      // the slim P = 3 shape on the 4-step wheel over the P = 3, delay <= 4
      // instances among the first n (a first stage in front of layout 5's)
      const EvParams p = make_params(&cfg);
      using Probe = EvLane<3, 9, 44, 8, false, HostMem, true, false, true, 0>;
      std::vector<uint32_t> mem(256), ids, bailed;
      Probe q;
      q.m = HostMem{mem.data()};
      q.set_keys(p);
      for (uint32_t g = 0; g < n; ++g) {
        q.init(p, g);
        if (q.P == 3u && q.dmax <= 4u) ids.push_back(g);
      }
      printf("-- slim W4 over %zu P = 3, delay <= 4 instances of %u\n", ids.size(), n);
      model<3, 9, 4, false, false, true>(&cfg, 0, rmin, &ids, &bailed);
    } else {
      std::vector<uint32_t> bailed;
      model<3, 9, 8, false, false, true>(&cfg, n, rmin, nullptr, &bailed);
      if (getenv("STAGE2")) {   // a third per-lane stage over the P = 3 shape's hand-offs: layout 0 / 1
        std::vector<uint32_t> p3;
        for (uint32_t g : bailed) p3.push_back(g);
        printf("-- layout 0 over %zu hand-offs\n", p3.size());
        std::vector<uint32_t> b2, b3;
        model<3, 9, 8, false, false, false>(&cfg, 0, rmin, &p3, &b2);
        printf("-- layout 1 over %zu hand-offs\n", p3.size());
        model<3, 9, 16, false, false, false>(&cfg, 0, rmin, &p3, &b3);
      }
    }
  } else if (c == 7) {
    // faulty log mode (pxb.LOG_FAULTY_CONFIG): the LG shape, layout 4
    cfg.seed = 0x5EED0007; cfg.n_proposers = 2; cfg.n_acceptors = 5; cfg.loss_ppm = 100000;
    cfg.delay_max = 4; cfg.skew_max = 3; cfg.crash_ppm = 200000; cfg.crash_len_max = 16;
    cfg.crash_start_max = 64; cfg.step_cap = 1024; cfg.n_ticks = 16; cfg.tick_period = 8;
    std::vector<uint32_t> bailed;
    // (LGW=4: the log-mode shape slimmed -- byte reply seqs in registers -- on the
    // 4-step wheel, for delays <= 4; LGW=8: the same on the 8-step wheel)
    if (getenv("LGW")) {
      if (atoi(getenv("LGW")) == 4) model<2, 5, 4, false, true, true>(&cfg, n, rmin, nullptr, &bailed);
      else model<2, 5, 8, false, true, true>(&cfg, n, rmin, nullptr, &bailed);
    } else {
      model<2, 5, 8, false, true, false>(&cfg, n, rmin, nullptr, &bailed);
    }
    if (getenv("STAGE2")) {   // the LG shape on the 16-step wheel (its larger pool) over the hand-offs
      printf("-- second stage over %zu hand-offs\n", bailed.size());
      std::vector<uint32_t> b2;
      model<2, 5, 16, false, true, false>(&cfg, 0, rmin, &bailed, &b2);
      printf("-- still handed on: %zu\n", b2.size());
    }
  } else {
    fprintf(stderr, "config 3, 4, 5 or 7\n");
    return 1;
  }
  return 0;
}
