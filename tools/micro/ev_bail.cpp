// ev_bail.cpp — layout experiment (host only): bail rate, iterations per
// instance and LDS words of candidate per-lane shapes for a config.
//   hipcc -O2 -std=c++17 -o /tmp/ev_bail tools/micro/ev_bail.cpp && /tmp/ev_bail [n] [first]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../cloud-haskell-paxos_amd/csrc/paxos_ev_kernel.h"

using namespace pxb;
using namespace pxb::ev;

struct HostMem {
  uint32_t* w;
  uint32_t ld(uint32_t i) const { return w[i]; }
  void st(uint32_t i, uint32_t v) const { w[i] = v; }
  uint32_t ld16(uint32_t base, uint32_t i) const { return reinterpret_cast<const uint16_t*>(w + base)[i]; }
  void st16(uint32_t base, uint32_t i, uint32_t v) const { reinterpret_cast<uint16_t*>(w + base)[i] = (uint16_t)v; }
  uint32_t ld16h(uint32_t i, uint32_t half) const { return reinterpret_cast<const uint16_t*>(w + i)[half]; }
  void st16h(uint32_t i, uint32_t half, uint32_t v) const { reinterpret_cast<uint16_t*>(w + i)[half] = (uint16_t)v; }
  void orw(uint32_t i, uint32_t v) const { w[i] |= v; }
};

template <int PM, int N, int POOL, int W, bool CMP>
void run(const char* name, const pxb_config* cfg, uint32_t only_p = 0) {
  using S = Shape<PM, N, POOL, W, CMP>;
  std::vector<uint32_t> buf(S::WORDS + 1, 0xDEADBEEFu);
  const EvParams p = make_params(cfg);
  EvLane<PM, N, POOL, W, CMP, HostMem> L;
  L.m = HostMem{buf.data()};
  L.set_keys(p);
  uint64_t it = 0, it_ok = 0, nb = 0, steps = 0, cnt = 0;
  for (uint32_t g = 0; g < (uint32_t)cfg->n_instances; ++g) {
    L.init(p, g);
    if (only_p && L.P != only_p) continue;
    ++cnt;
    EvOut o;
    uint64_t k = 0;
    for (;;) {
      const bool done = L.step(p, o);
      ++k;
      if (L.bailed) { ++nb; break; }
      if (done) { it_ok += k; steps += o.steps; break; }
    }
    it += k;
  }
  const double n = (double)cnt;
  printf("%-28s words %3d (waves/CU %2d)  bail %.4f  iters/inst %.1f (ok %.1f)  steps/inst %.1f\n", name, S::WORDS,
         (int)(160 * 1024 / (S::WORDS * 256)), nb / n, it / n, it_ok / (n - nb), steps / (n - nb));
}

int main(int argc, char** argv) {
  pxb_config c{};
  c.first_instance = argc > 2 ? strtoull(argv[2], 0, 0) : 0;
  c.n_instances = argc > 1 ? strtoull(argv[1], 0, 0) : 20000;
  const int which = argc > 3 ? atoi(argv[3]) : 5;
  if (which == 4) {                       // BASELINE config 4
    c.seed = 0x5EED0004;
    c.n_proposers = 2;
    c.n_acceptors = 7;
    c.delay_max = 4;
    c.crash_ppm = 200000;
    c.crash_len_max = 16;
    c.crash_start_max = 8;
    c.step_cap = 256;
    run<2, 7, 24, 8, true>("c4 cur <2,7,24,W8,cmp>", &c);
    run<2, 7, 24, 4, true>("c4 <2,7,24,W4,cmp>", &c);
    run<2, 7, 22, 4, true>("c4 <2,7,22,W4,cmp>", &c);
    run<2, 7, 20, 4, true>("c4 <2,7,20,W4,cmp>", &c);
    run<2, 7, 16, 4, true>("c4 <2,7,16,W4,cmp>", &c);
    return 0;
  }
  c.seed = 0x5EED0005;
  c.n_proposers = 3;
  c.n_acceptors = 9;
  c.loss_ppm = 300000;
  c.delay_max = 8;
  c.crash_ppm = 200000;
  c.crash_len_max = 16;
  c.crash_start_max = 16;
  c.skew_max = 3;
  c.step_cap = 512;
  c.flags = PXB_CFG_RANDOMIZE;
  run<3, 9, 64, 8, false>("P=3 <3,9,64,W8,full>", &c, 3);
  run<3, 9, 48, 8, false>("P=3 <3,9,48,W8,full>", &c, 3);
  run<2, 9, 32, 8, false>("P=2 <2,9,32,W8,full>", &c, 2);
  run<2, 9, 32, 8, true>("P=2 <2,9,32,W8,cmp>", &c, 2);
  return 0;
}
