// paxos_batch_main.cpp — C++ batch driver over the C ABI.
//
// This is the role app/Main.hs (/root/reference/app/Main.hs:27-53) plays in the
// reference, turned into a batch driver: instead of spawning 2 servers and 2
// clients on one Cloud Haskell node and logging forever (Main.hs:41-53), it runs
// many independent single-decree instances of the same protocol on the GPU(s)
// through include/paxos_batch.h and prints the outcome in the reference's
// vocabulary (Command "c<id>.<t>", Ticket, Client.hs:202-203, Common.hs:20-30).
// The Haskell binding of the same entry points is hs/PaxosBatch.hs.
//
//   paxos_batch_main [--config K] [--instances N] [--first F] [--gpus G] [--show S]
//                    [--ticks T --period D]   (log mode: T Ticks per proposer, D steps apart)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/paxos_batch.h"

static pxb_config named_config(int k) {
  pxb_config c;
  memset(&c, 0, sizeof(c));
  c.n_proposers = 1;
  c.n_acceptors = 5;
  c.delay_max = 1;
  c.crash_len_max = 1;
  c.step_cap = 256;
  switch (k) {  // BASELINE.json configs
    case 1: c.seed = 0x5EED0001; c.n_acceptors = 3; c.n_instances = 1 << 10; break;
    case 2: c.seed = 0x5EED0002; c.n_instances = 1 << 20; break;
    case 3: c.seed = 0x5EED0003; c.n_proposers = 2; c.loss_ppm = 100000; c.delay_max = 4; c.skew_max = 3;
            c.n_instances = 1 << 24; break;
    case 4: c.seed = 0x5EED0004; c.n_proposers = 2; c.n_acceptors = 7; c.delay_max = 4; c.crash_ppm = 200000;
            c.crash_len_max = 16; c.crash_start_max = 8; c.n_instances = 1 << 26; break;
    case 5: c.seed = 0x5EED0005; c.n_proposers = 3; c.n_acceptors = 9; c.loss_ppm = 300000; c.delay_max = 8;
            c.crash_ppm = 200000; c.crash_len_max = 16; c.crash_start_max = 16; c.skew_max = 3; c.step_cap = 512;
            c.flags = PXB_CFG_RANDOMIZE; c.n_instances = 1ull << 28; break;
    default: fprintf(stderr, "unknown config %d\n", k); exit(2);
  }
  return c;
}

static std::string command(uint32_t code) {   // "c<clientId>.<t>"  (Client.hs:202-203)
  if (code == 0) return "Nothing";
  return "c" + std::to_string(code >> 24) + "." + std::to_string(code & 0xFFFFFFu);
}

static std::string flag_names(uint32_t f) {
  static const char* names[8] = {"UNDECIDED", "STUCK", "PANIC", "LOG_DIVERGENCE",
                                 "STEP_CAP", "QUEUE_OVERFLOW", "TICKET_OVERFLOW", "LOG_TRUNC"};
  std::string s;
  for (int b = 0; b < 8; ++b)
    if (f & (1u << b)) s += (s.empty() ? "" : "|") + std::string(names[b]);
  return s.empty() ? "-" : s;
}

int main(int argc, char** argv) {
  int cfg_id = 2, gpus = 1, show = 4, ticks = 0, period = 8;
  long long instances = -1, first = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return (i + 1 < argc) ? argv[++i] : (char*)"0"; };
    if (a == "--config") cfg_id = atoi(next());
    else if (a == "--instances") instances = atoll(next());
    else if (a == "--first") first = atoll(next());
    else if (a == "--gpus") gpus = atoi(next());
    else if (a == "--show") show = atoi(next());
    else if (a == "--ticks") ticks = atoi(next());      // log mode: Ticks per proposer
    else if (a == "--period") period = atoi(next());    // steps between Ticks
    else {
      fprintf(stderr, "usage: %s [--config K] [--instances N] [--first F] [--gpus G] [--show S] "
              "[--ticks T --period D]\n", argv[0]);
      return 2;
    }
  }
  pxb_config cfg = named_config(cfg_id);
  if (instances >= 0) cfg.n_instances = (uint64_t)instances;
  cfg.first_instance = (uint64_t)first;
  if (ticks > 1) {
    cfg.n_ticks = (uint32_t)ticks;
    cfg.tick_period = (uint32_t)period;
    const uint32_t need = (uint32_t)(ticks - 1) * (uint32_t)period + 64u;
    if (cfg.step_cap < need) cfg.step_cap = need > PXB_MAX_STEP_CAP ? PXB_MAX_STEP_CAP : need;
  }
  const uint64_t n = cfg.n_instances, N = cfg.n_acceptors;
  std::vector<pxb_result> res(n);
  std::vector<uint32_t> dig(n * N);
  pxb_counters tot;
  memset(&tot, 0, sizeof(tot));
  const auto t0 = std::chrono::steady_clock::now();
  int rc = pxb_run_multi(&cfg, gpus, res.data(), dig.data(), nullptr, &tot);
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc != PXB_OK) {
    fprintf(stderr, "pxb_run_multi: %s (%d, hip %d)\n", pxb_strerror(rc), rc, pxb_last_hip_error());
    return 1;
  }
  printf("config %d: %llu instances (P=%u, N=%u, loss %u ppm, delay<=%u, crash %u ppm) on %d GPU(s) in %.3f s "
         "(host-buffer path, incl. PCIe copies)\n",
         cfg_id, (unsigned long long)n, cfg.n_proposers, cfg.n_acceptors, cfg.loss_ppm, cfg.delay_max, cfg.crash_ppm,
         gpus, dt);
  static const char* cn[PXB_NCOUNTERS] = {"decided", "undecided", "stuck", "panic", "divergence", "step_cap",
                                          "rounds", "messages", "queue_overflow", "ticket_overflow", "log_trunc",
                                          "canon_bytes", "steps", "instances", "executes", "-"};
  for (int k = 0; k < 15; ++k) printf("  %-16s %lld\n", cn[k], (long long)tot.c[k]);
  for (uint64_t i = 0; i < n && i < (uint64_t)show; ++i) {
    const pxb_result& r = res[i];
    printf("instance %llu: decided %s @ Ticket %d, rounds %u, steps %u, flags %s, log digests",
           (unsigned long long)(cfg.first_instance + i), command(r.decided_val).c_str(), r.decided_ticket, r.rounds,
           PXB_RESULT_STEPS(r.flags), flag_names(r.flags & 0xFFu).c_str());
    for (uint64_t a = 0; a < N; ++a) printf(" %08x", dig[i * N + a]);
    printf("\n");
  }
  return 0;
}
