// ev_host.cpp — TEST ONLY: runs the per-lane kernel's state machine
// (cloud-haskell-paxos_amd/csrc/paxos_ev.h) on the host, one instance at a
// time, so tests/test_ev_host.py can diff it against the CPU oracle without a
// GPU.  The product runs the same EvLane code on the device
// (paxos_ev_kernel.h); nothing here is linked into libpaxos_batch.so.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../cloud-haskell-paxos_amd/csrc/paxos_ev_kernel.h"

using namespace pxb;
using namespace pxb::ev;

namespace {

int g_words = 0;                                           // LDS words per lane of the last shape run

// PXB_HOST_CHECKED (the sanitizer build, tests/test_ev_sanitized.py): every
// access is checked against the shape's LDS words (S::WORDS), halfword
// accesses against 2 * WORDS halfwords, before it is made
#ifdef PXB_HOST_CHECKED
#define PXB_HCHK(c)                                                                                   \
  do {                                                                                              \
    if (!(c)) {                                                                                     \
      fprintf(stderr, "ev_host: LDS access out of the shape's words: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
      abort();                                                                                      \
    }                                                                                               \
  } while (0)
#else
#define PXB_HCHK(c) ((void)0)
#endif
struct HostMem {
  uint32_t* w;
  uint32_t n;                                              // the shape's words (S::WORDS)
  uint32_t ld(uint32_t i) const { PXB_HCHK(i < n); return w[i]; }
  void st(uint32_t i, uint32_t v) const { PXB_HCHK(i < n); w[i] = v; }
  uint32_t ld16(uint32_t base, uint32_t i) const {
    PXB_HCHK(2u * base + i < 2u * n);
    return reinterpret_cast<const uint16_t*>(w + base)[i];
  }
  void st16(uint32_t base, uint32_t i, uint32_t v) const {
    PXB_HCHK(2u * base + i < 2u * n);
    reinterpret_cast<uint16_t*>(w + base)[i] = (uint16_t)v;
  }
  uint32_t ld16h(uint32_t i, uint32_t half) const {
    PXB_HCHK(i < n && half < 2u);
    return reinterpret_cast<const uint16_t*>(w + i)[half];
  }
  void st16h(uint32_t i, uint32_t half, uint32_t v) const {
    PXB_HCHK(i < n && half < 2u);
    reinterpret_cast<uint16_t*>(w + i)[half] = (uint16_t)v;
  }
  // (the device's lane-interleaved halfword arrays: per lane, halfword i of the array at word base)
  uint32_t ldh(uint32_t base, uint32_t i) const { return ld16(base, i); }
  void sth(uint32_t base, uint32_t i, uint32_t v) const { st16(base, i, v); }
  void orw(uint32_t i, uint32_t v) const { PXB_HCHK(i < n); w[i] |= v; }
};

template <int PM, int N, int W, bool CMP, bool LG, bool SL, int SP>
int run_shape(const pxb_config* cfg, pxb_result* out, uint32_t* dig, pxb_acceptor_rec* acc, int64_t* tot,
              uint32_t* bail_ids, uint32_t* n_bail, uint64_t* micro_steps) {
  constexpr int POOL = EvPool<PM, N, CMP, LG, SL, SP, W>::value;
  using S = Shape<PM, N, POOL, W, CMP, LG, SL, SP>;
  g_words = S::WORDS;
  // garbage: init must set what it reads (checked builds: exactly WORDS, so
  // ASan sees an access past them even where PXB_HCHK would not)
#ifdef PXB_HOST_CHECKED
  std::vector<uint32_t> buf(S::WORDS, 0xDEADBEEFu);
#else
  std::vector<uint32_t> buf(S::WORDS + 1, 0xDEADBEEFu);
#endif
  const EvParams p = make_params(cfg);
  EvLane<PM, N, POOL, W, CMP, HostMem, true, LG, SL, SP> L;
  L.m = HostMem{buf.data(), (uint32_t)S::WORDS};
  L.set_keys(p);
  uint32_t nb = 0;
  uint64_t ms = 0;
  for (uint32_t g = 0; g < (uint32_t)cfg->n_instances; ++g) {
    L.init(p, g);
    EvOut o;
    uint64_t guard = 0;
    if (L.bailed) {                                        // fuzzed P above the shape's (split routing)
      bail_ids[nb++] = g;
      continue;
    }
    for (;;) {
      const bool done = L.step(p, o);
      ++ms;
      if (++guard > 100000ull * cfg->step_cap) return -100;   // a hang is a test failure
      if (L.bailed) {
        bail_ids[nb++] = g;
        break;
      }
      if (done) {
        if (out) memcpy(&out[g], o.res, 16);
        for (int a = 0; a < N; ++a) {
          if (dig) dig[(uint64_t)g * N + a] = L.digest_of(a);
          if (acc) {
            uint32_t r[4];
            L.record_of(a, r);
            memcpy(&acc[(uint64_t)g * N + a], r, 16);
          }
        }
        const uint32_t f = o.flags;
        tot[PXB_C_INSTANCES] += 1;
        tot[PXB_C_DECIDED] += !(f & PXB_F_UNDECIDED);
        tot[PXB_C_UNDECIDED] += !!(f & PXB_F_UNDECIDED);
        tot[PXB_C_STUCK] += !!(f & PXB_F_STUCK);
        tot[PXB_C_PANIC] += !!(f & PXB_F_PANIC);
        tot[PXB_C_DIVERGENCE] += !!(f & PXB_F_LOG_DIVERGENCE);
        tot[PXB_C_STEP_CAP] += !!(f & PXB_F_STEP_CAP);
        tot[PXB_C_ROUNDS] += L.rounds;
        tot[PXB_C_STEPS] += o.steps;
#ifdef PXB_HOST_CHECKED
        // msgs_sent() counts N copies of every broadcast from nsent: an ended
        // instance has no broadcast left to send
        if (L.pq_len != 0u) {
          fprintf(stderr, "ev_host: instance ended with %u pending broadcasts\n", L.pq_len);
          abort();
        }
#endif
        tot[PXB_C_MESSAGES] += L.msgs_sent();
        tot[PXB_C_EXECUTES] += L.execs;
        tot[PXB_C_LOG_TRUNC] += !!(f & PXB_F_LOG_TRUNC);
        tot[PXB_C_CANON_BYTES] += L.canon;
        break;
      }
    }
  }
  *n_bail = nb;
  if (micro_steps) *micro_steps = ms;
  return 0;
}

template <int PM, int W, bool CMP, bool LG, bool SL, int SP>
int run_n(const pxb_config* c, pxb_result* o, uint32_t* d, pxb_acceptor_rec* a, int64_t* t, uint32_t* b, uint32_t* nb,
          uint64_t* ms) {
  switch (c->n_acceptors) {
    case 2: return run_shape<PM, 2, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 5: return run_shape<PM, 5, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 7: return run_shape<PM, 7, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 9: return run_shape<PM, 9, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
#ifndef PXB_EV_HOST_FEW_N   // (the sanitizer build: the acceptor counts above only, half the compile time)
    case 3: return run_shape<PM, 3, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 4: return run_shape<PM, 4, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 6: return run_shape<PM, 6, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 8: return run_shape<PM, 8, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
#endif
  }
  return -1;
}

template <int W, bool CMP, bool LG = false, bool SL = false, int SP = 0>
int run_w(const pxb_config* c, uint32_t pm, pxb_result* o, uint32_t* d, pxb_acceptor_rec* a, int64_t* t, uint32_t* b,
          uint32_t* nb, uint64_t* ms) {
  switch (pm) {
    case 1: return run_n<1, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 2: return run_n<2, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
    case 3: return run_n<3, W, CMP, LG, SL, SP>(c, o, d, a, t, b, nb, ms);
  }
  return -1;
}

}  // namespace

extern "C" int ev_host_run(const pxb_config* cfg, pxb_result* out, uint32_t* dig, pxb_acceptor_rec* acc,
                           int64_t* totals, uint32_t* bail_ids, uint32_t* n_bail, uint64_t* micro_steps) {
  if (!cfg || !eligible(cfg)) return -1;
  const char* lv = getenv("EV_LAYOUT");                 // tests: force a layout
  const int layout = lv ? atoi(lv) : layout_for(cfg);
  if (layout == 2 && cfg->delay_max > 8) return -1;
  if ((layout == 3 || layout == 6 || layout == 7) && cfg->delay_max > 4) return -1;
  if ((layout == 6 || layout == 7) && (cfg->loss_ppm || cfg->skew_max || (cfg->flags & PXB_CFG_RANDOMIZE) || cfg->n_ticks > 1)) return -1;
  if ((layout == 4 || layout == 8 || layout == 9) != (cfg->n_ticks > 1)) return -1;   // log mode runs on the log-mode fields only
  if (layout == 9 && cfg->delay_max > 4) return -1;
  if ((layout == 0 || layout == 5) && cfg->delay_max > 8) return -1;
  // tests: the shape's proposer capacity; below n_proposers (fuzzed batches
  // only) it is the split routing of pxb_run_device, whose instances with more
  // proposers than the shape bail at init
  const char* pv = getenv("EV_PM");
  uint32_t pm = cfg->n_proposers;
  if (pv && atoi(pv) > 0) {
    pm = (uint32_t)atoi(pv);
    if (pm > cfg->n_proposers || (pm < cfg->n_proposers && !(cfg->flags & PXB_CFG_RANDOMIZE))) return -1;
  }
  switch (layout) {
    case 0: return run_w<8, false>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 1: return run_w<16, false>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 2: return run_w<8, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 3: return run_w<4, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 4: return run_w<8, false, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 5: return run_w<8, false, false, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 6: return run_w<4, true, false, false, 1>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 7: return run_w<4, true, false, false, 2>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 8: return run_w<16, false, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
    case 9: return run_w<4, false, true, true>(cfg, pm, out, dig, acc, totals, bail_ids, n_bail, micro_steps);
  }
  return -1;
}

// the LDS words per lane of the shape the last ev_host_run used (tests: layout sizes)
extern "C" int ev_host_last_words(void) { return g_words; }

#ifdef PXB_EV_HOST_MAIN
// Sanitizer-build driver (tests/test_ev_sanitized.py): one batch from the
// command line, outputs to a file as raw little-endian words:
//   rc, n, N, n_bail | results n x 4 | digests n x N | acceptor records n x N x 4
//   | totals 16 x int64 | bailed ids n_bail
// argv: out seed first n P N loss delay crash clen cstart skew cap flags ticks period
int main(int argc, char** argv) {
  if (argc != 17) {
    fprintf(stderr, "usage: %s out seed first n P N loss delay crash clen cstart skew cap flags ticks period\n", argv[0]);
    return 2;
  }
  pxb_config c{};
  c.seed = strtoull(argv[2], nullptr, 0);
  c.first_instance = strtoull(argv[3], nullptr, 0);
  c.n_instances = strtoull(argv[4], nullptr, 0);
  uint32_t* f[] = {&c.n_proposers, &c.n_acceptors, &c.loss_ppm, &c.delay_max, &c.crash_ppm, &c.crash_len_max,
                   &c.crash_start_max, &c.skew_max, &c.step_cap, &c.flags, &c.n_ticks, &c.tick_period};
  for (int i = 0; i < 12; ++i) *f[i] = (uint32_t)strtoul(argv[5 + i], nullptr, 0);
  const uint64_t n = c.n_instances, N = c.n_acceptors;
  std::vector<pxb_result> res(n);
  std::vector<uint32_t> dig(n * N), bails(n + 1);
  std::vector<pxb_acceptor_rec> acc(n * N);
  int64_t tot[16] = {0};
  uint32_t nb = 0;
  uint64_t ms = 0;
  const int rc = ev_host_run(&c, res.data(), dig.data(), acc.data(), tot, bails.data(), &nb, &ms);
  FILE* o = fopen(argv[1], "wb");
  if (!o) return 3;
  const uint32_t hdr[4] = {(uint32_t)rc, (uint32_t)n, (uint32_t)N, nb};
  fwrite(hdr, 4, 4, o);
  fwrite(res.data(), sizeof(pxb_result), n, o);
  fwrite(dig.data(), 4, n * N, o);
  fwrite(acc.data(), sizeof(pxb_acceptor_rec), n * N, o);
  fwrite(tot, 8, 16, o);
  fwrite(bails.data(), 4, nb, o);
  fclose(o);
  return rc == 0 ? 0 : 4;
}
#endif
