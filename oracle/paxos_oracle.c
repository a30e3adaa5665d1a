/*
 * paxos_oracle.c — CPU restatement of the canonical batched ticket-Paxos step
 * schedule.  TEST INFRASTRUCTURE AND CPU BASELINE ONLY: linked/loaded by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
 * the product library (cloud-haskell-paxos_amd/csrc).
 *
 * Semantics: docs/SEMANTICS.md.  This file mirrors oracle/paxos_ref.py
 * (run_instance) statement for statement; the handlers restate
 *   acceptor handleClientRequest   /root/reference/src/Server.hs:54-78
 *   proposer handleServerResponse  /root/reference/src/Client.hs:128-189
 *            haveMajority          /root/reference/src/Client.hs:191-194
 *            handleTick            /root/reference/src/Client.hs:196-207
 *   MostRecentProposal monoid      /root/reference/src/Common.hs:57-68
 * Parity: pinned to SURVEY.md §8.0's hand-derived KATs through paxos_ref.py
 * (tests cross-check this file against it); the Haskell reference itself
 * cannot be built here (no GHC) — see DESIGN.md "Oracle".
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/paxos_batch.h"

/* ---- Philox4x32-10 ------------------------------------------------------- */
typedef struct { uint32_t v[4]; } u32x4;

static u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  u32x4 o = {{c0, c1, c2, c3}};
  return o;
}

static inline uint32_t mulhi(uint32_t w, uint32_t n) { return (uint32_t)(((uint64_t)w * n) >> 32); }
static inline uint64_t prob_threshold(uint32_t ppm) {
  return (((uint64_t)ppm << 32) + 999999u) / 1000000u;
}

enum { PURPOSE_MSG = 1, PURPOSE_SKEW = 2, PURPOSE_CRASH = 3, PURPOSE_PARAMS = 4 };
enum { ASK = 0, PROPOSE = 1, EXECUTE = 2 };
enum { R1OK = 0, HAVE = 1, R2S = 2 };
enum { IDLE = 0, ROUND1 = 1, ROUND2 = 2 };
static const int REQ_BYTES[3] = {8, 12, 8};
static const int RSP_BYTES[3] = {16, 8, 4};

#define QD PXB_QUEUE_DEPTH
#define MAXP PXB_MAX_PROPOSERS
#define MAXN PXB_MAX_ACCEPTORS

typedef struct { uint32_t kind; int32_t x, y; uint32_t z; int32_t due; } msg_t;
typedef struct { msg_t q[QD]; int head, len; uint32_t seq; int32_t last_due; } link_t;

typedef struct {
  int32_t t_max, t_store;
  uint32_t val;
  uint32_t log_len;
  uint32_t digest;
  int dead;
  int32_t c0, c1;
} acc_t;

typedef struct {
  int32_t ticket;
  uint32_t cmd, acks, rs;
  int32_t mr_t; uint32_t mr_v;
  int32_t r2_t; uint32_t r2_v;
  int pending;
  uint32_t client_id;
} prop_t;

typedef struct {
  /* inputs */
  const pxb_config* cfg;
  uint32_t k0, k1, lo, hi;
  int P, N;
  uint64_t loss_thr;
  uint32_t delay_max;
  int faulty;
  int32_t skew[MAXP];
  /* state */
  acc_t acc[MAXN];
  prop_t prop[MAXP];
  link_t req[MAXP][MAXN];
  link_t rsp[MAXN][MAXP];
  uint32_t canon_log[PXB_LOG_TRACK];
  uint32_t flags, rounds;
  uint64_t messages, canon, executes;
  int decided;
  uint32_t decided_val; int32_t decided_ticket;
} inst_t;

static inline uint32_t fnv_u32(uint32_t h, uint32_t v) {
  for (int i = 0; i < 4; ++i) { h ^= (v >> (8 * i)) & 0xFFu; h *= 0x01000193u; }
  return h;
}

/* ---- link send (docs/SEMANTICS.md §5) ---- */
static void send(inst_t* I, link_t* L, int s, int dirn, int p, int a, msg_t m) {
  I->messages++;
  uint32_t k = L->seq++;
  int d = 1;
  if (I->faulty) {
    u32x4 w = philox(I->lo, I->hi, k, (PURPOSE_MSG << 24) | (dirn << 16) | (p << 8) | a, I->k0, I->k1);
    if ((uint64_t)w.v[0] < I->loss_thr) return;
    d = 1 + (int)mulhi(w.v[1], I->delay_max);
  }
  if (L->len >= QD) { I->flags |= PXB_F_QUEUE_OVERFLOW; return; }
  int32_t due = s + d;
  if (due < L->last_due) due = L->last_due;
  L->last_due = due;
  m.due = due;
  L->q[(L->head + L->len) % QD] = m;
  L->len++;
}

static inline int pop_due(link_t* L, int s, msg_t* m) {
  if (L->len == 0 || L->q[L->head].due > s) return 0;
  *m = L->q[L->head];
  L->head = (L->head + 1) % QD;
  L->len--;
  return 1;
}

/* ---- acceptor: handleClientRequest, Server.hs:54-78 ---- */
static int acceptor_handle(acc_t* A, const msg_t* m, msg_t* rep) {
  if (m->kind == ASK) {                                   /* Server.hs:54 */
    if (A->t_max >= m->x) {                               /* :56 */
      rep->kind = HAVE; rep->x = A->t_max; rep->y = 0; rep->z = 0;   /* :58 */
      return 1;
    }
    A->t_max = m->x;                                      /* :60 */
    rep->kind = R1OK; rep->x = m->x; rep->y = A->t_store; rep->z = A->val;  /* :61-62 */
    return 1;
  }
  if (m->kind == PROPOSE) {                               /* :64 */
    if (m->x == A->t_max) {                               /* :66 equality */
      A->t_store = m->x; A->val = m->z;                   /* :68 */
      rep->kind = R2S; rep->x = rep->y = 0; rep->z = 0;   /* :69 */
      return 1;
    }
    rep->kind = HAVE; rep->x = A->t_max; rep->y = 0; rep->z = 0;     /* :71 */
    return 1;
  }
  /* EXECUTE, :73 */
  if (A->t_max == m->x) {                                 /* :75 */
    if (A->val == 0) { A->dead = 1; return 0; }          /* :76 Q6 */
    A->log_len++;                                         /* :78 */
    A->digest = fnv_u32(A->digest, A->val);
    A->t_store = 0; A->val = 0;                           /* :77 */
  }
  return 0;
}

/* ---- proposer (Client.hs:128-207); returns number of broadcasts ---- */
static int proposer_tick(prop_t* pr, msg_t out[2]) {
  if (pr->rs != IDLE) return 0;                           /* :199 */
  pr->ticket += 1;                                        /* :200 */
  pr->cmd = (pr->client_id << 24) | ((uint32_t)pr->ticket & 0xFFFFFFu);   /* :202-204 */
  pr->acks = 0; pr->rs = ROUND1; pr->mr_t = 0; pr->mr_v = 0;              /* :205-206 */
  out[0].kind = ASK; out[0].x = pr->ticket; out[0].y = 0; out[0].z = 0;   /* :207 */
  return 1;
}

static int proposer_handle(prop_t* pr, int N, const msg_t* m, msg_t out[2]) {
  if (m->kind == HAVE) {                                  /* :128 */
    if (pr->rs != IDLE && m->x >= pr->ticket) {           /* :130-132 */
      pr->ticket = m->x + 1;                              /* :134-135 */
      pr->acks = 0; pr->rs = ROUND1; pr->mr_t = 0; pr->mr_v = 0;   /* :137-138 */
      out[0].kind = ASK; out[0].x = pr->ticket; out[0].y = 0; out[0].z = 0;   /* :140 */
      return 1;
    }
    return 0;
  }
  if (m->kind == R1OK) {                                  /* :142 */
    if (pr->rs == ROUND1 && pr->ticket == m->x) {         /* :144-145 */
      pr->acks += 1;                                      /* :146 */
      int32_t mt = pr->mr_t; uint32_t mv = pr->mr_v;      /* MostRecent fold :147-151, Common.hs:61-65 */
      if (mv == 0) { mt = m->y; mv = m->z; }
      else if (m->z != 0 && !(mt >= m->y)) { mt = m->y; mv = m->z; }
      if (!(pr->acks > (uint32_t)(N / 2))) {              /* :152-154, haveMajority :191-194 */
        pr->mr_t = mt; pr->mr_v = mv;
        return 0;
      }
      if (mv == 0) { pr->r2_t = m->x; pr->r2_v = pr->cmd; pr->pending = 0; }   /* :159-162 */
      else         { pr->r2_t = m->x; pr->r2_v = mv;      pr->pending = 1; }   /* :163-167 */
      pr->acks = 0; pr->rs = ROUND2; pr->mr_t = 0; pr->mr_v = 0;              /* :168-169 */
      out[0].kind = PROPOSE; out[0].x = pr->r2_t; out[0].y = 0; out[0].z = pr->r2_v;   /* :170 */
      return 1;
    }
    return 0;
  }
  /* R2S, :172 */
  if (pr->rs == ROUND2) {                                 /* :174 */
    pr->acks += 1;                                        /* :175 */
    if (pr->acks > (uint32_t)(N / 2)) {                   /* :176-177 */
      out[0].kind = EXECUTE; out[0].x = pr->ticket; out[0].y = 0; out[0].z = 0;   /* :178 */
      if (pr->pending) {                                  /* :179 */
        pr->ticket += 1;                                  /* :182 */
        pr->acks = 0; pr->rs = ROUND1; pr->mr_t = 0; pr->mr_v = 0;   /* :183-184 */
        out[1].kind = ASK; out[1].x = pr->ticket; out[1].y = 0; out[1].z = 0;   /* :185 */
        return 2;
      }
      pr->cmd = 0; pr->acks = 0; pr->rs = IDLE;           /* :187-189 */
      return 1;
    }
  }
  return 0;
}

static void bcast(inst_t* I, int p, int s, const msg_t* out, int nout) {
  for (int i = 0; i < nout; ++i) {
    if (out[i].kind == ASK) I->rounds++;
    if (out[i].kind == EXECUTE) I->executes++;
    if (out[i].kind == EXECUTE && !I->decided) {
      I->decided = 1; I->decided_val = I->prop[p].r2_v; I->decided_ticket = out[i].x;
    }
    for (int a = 0; a < I->N; ++a) send(I, &I->req[p][a], s, 0, p, a, out[i]);
  }
}

static void run_instance(const pxb_config* cfg, uint64_t inst, pxb_result* res,
                         uint32_t* digest, pxb_acceptor_rec* accrec, int64_t* cnt) {
  inst_t I_;
  inst_t* I = &I_;
  memset(I, 0, sizeof(*I));
  I->cfg = cfg;
  I->k0 = (uint32_t)cfg->seed; I->k1 = (uint32_t)(cfg->seed >> 32);
  I->lo = (uint32_t)inst; I->hi = (uint32_t)(inst >> 32);
  I->N = (int)cfg->n_acceptors;
  int P = (int)cfg->n_proposers;
  uint32_t loss_ppm = cfg->loss_ppm, delay_max = cfg->delay_max, crash_ppm = cfg->crash_ppm;
  if (cfg->flags & PXB_CFG_RANDOMIZE) {                   /* SEMANTICS §4 */
    u32x4 w = philox(I->lo, I->hi, 0, PURPOSE_PARAMS << 24, I->k0, I->k1);
    P = 1 + (int)mulhi(w.v[0], cfg->n_proposers);
    loss_ppm = mulhi(w.v[1], cfg->loss_ppm + 1);
    delay_max = 1 + mulhi(w.v[2], cfg->delay_max);
    crash_ppm = mulhi(w.v[3], cfg->crash_ppm + 1);
  }
  I->P = P;
  I->loss_thr = prob_threshold(loss_ppm);
  I->delay_max = delay_max;
  I->faulty = (I->loss_thr > 0) || (delay_max > 1);
  int last_tick = 0;
  if (cfg->skew_max > 0) {
    u32x4 w = philox(I->lo, I->hi, 0, PURPOSE_SKEW << 24, I->k0, I->k1);
    for (int p = 0; p < P; ++p) {
      I->skew[p] = (int32_t)mulhi(w.v[p], cfg->skew_max + 1);
      if (I->skew[p] > last_tick) last_tick = I->skew[p];
    }
  }
  /* ticker (Client.hs:96-100): n_ticks Ticks tick_period steps apart from
   * skew_p (single decree: n_ticks <= 1, one Tick at skew_p) — SEMANTICS §9 */
  const int n_ticks = cfg->n_ticks > 1 ? (int)cfg->n_ticks : 1;
  const int period = cfg->n_ticks > 1 ? (int)cfg->tick_period : 1;
  last_tick += (n_ticks - 1) * period;
  for (int a = 0; a < I->N; ++a) { I->acc[a].digest = 0x811C9DC5u; }
  if (crash_ppm > 0) {
    uint64_t thr = prob_threshold(crash_ppm);
    for (int a = 0; a < I->N; ++a) {
      u32x4 w = philox(I->lo, I->hi, 0, (PURPOSE_CRASH << 24) | a, I->k0, I->k1);
      if ((uint64_t)w.v[0] < thr) {
        I->acc[a].c0 = (int32_t)mulhi(w.v[1], cfg->crash_start_max + 1);
        I->acc[a].c1 = I->acc[a].c0 + 1 + (int32_t)mulhi(w.v[2], cfg->crash_len_max);
      }
    }
  }
  for (int p = 0; p < P; ++p) I->prop[p].client_id = (uint32_t)(p + 1);

  int steps = 0, capped = 1;
  msg_t m, rep, out[2];
  for (int s = 0; s < (int)cfg->step_cap; ++s) {
    steps = s + 1;
    /* acceptor phase: inbox ordered by (proposer index, link seq) */
    for (int a = 0; a < I->N; ++a) {
      acc_t* A = &I->acc[a];
      int isolated = (A->c0 <= s) && (s < A->c1);
      for (int p = 0; p < P; ++p) {
        while (pop_due(&I->req[p][a], s, &m)) {
          if (A->dead || isolated) { I->canon += REQ_BYTES[m.kind]; continue; }
          I->canon += 2 * REQ_BYTES[m.kind] + 32;
          uint32_t before = A->log_len;
          uint32_t v = A->val;
          int r = acceptor_handle(A, &m, &rep);
          if (A->dead) I->flags |= PXB_F_PANIC;
          if (A->log_len != before) {
            if (before < PXB_LOG_TRACK) {
              if (I->canon_log[before] == 0) I->canon_log[before] = v;
              else if (I->canon_log[before] != v) I->flags |= PXB_F_LOG_DIVERGENCE;
            } else {
              I->flags |= PXB_F_LOG_TRUNC;
            }
          }
          if (r) send(I, &I->rsp[a][p], s, 1, p, a, rep);
        }
      }
    }
    /* proposer phase: Tick, then inbox ordered by (acceptor index, link seq) */
    for (int p = 0; p < P; ++p) {
      prop_t* pr = &I->prop[p];
      int active = 0;
      const int since = s - I->skew[p];
      if (since >= 0 && since % period == 0 && since / period < n_ticks) {
        active = 1;
        int n = proposer_tick(pr, out);
        bcast(I, p, s, out, n);
      }
      for (int a = 0; a < I->N; ++a) {
        while (pop_due(&I->rsp[a][p], s, &m)) {
          active = 1;
          I->canon += 2 * RSP_BYTES[m.kind];
          int n = proposer_handle(pr, I->N, &m, out);
          bcast(I, p, s, out, n);
        }
      }
      if (active) I->canon += 48;
      if (pr->ticket >= PXB_TICKET_LIMIT) I->flags |= PXB_F_TICKET_OVERFLOW;
    }
    /* quiescence */
    int in_flight = 0;
    for (int p = 0; p < P; ++p)
      for (int a = 0; a < I->N; ++a) in_flight |= I->req[p][a].len | I->rsp[a][p].len;
    if (!in_flight && s >= last_tick) { capped = 0; break; }
  }
  if (capped) I->flags |= PXB_F_STEP_CAP;
  if (!I->decided) I->flags |= PXB_F_UNDECIDED;
  if (!capped) {
    for (int p = 0; p < P; ++p) if (I->prop[p].rs != IDLE) { I->flags |= PXB_F_STUCK; break; }
  }
  I->canon += 16 + 4 * (uint64_t)I->N;

  if (res) {
    res->decided_val = I->decided ? I->decided_val : 0;
    res->decided_ticket = I->decided ? I->decided_ticket : 0;
    res->rounds = I->rounds;
    res->flags = (I->flags & 0xFFu) | ((uint32_t)(steps > 0xFFFF ? 0xFFFF : steps) << 16);
  }
  for (int a = 0; a < I->N; ++a) {
    if (digest) digest[a] = fnv_u32(I->acc[a].digest, I->acc[a].log_len);
    if (accrec) {
      accrec[a].t_max = I->acc[a].t_max;
      accrec[a].t_store = I->acc[a].t_store;
      accrec[a].val = I->acc[a].val;
      accrec[a].meta = I->acc[a].log_len | ((uint32_t)(I->acc[a].dead != 0) << 31);
    }
  }
  uint32_t f = I->flags;
  cnt[PXB_C_DECIDED] += !(f & PXB_F_UNDECIDED);
  cnt[PXB_C_UNDECIDED] += !!(f & PXB_F_UNDECIDED);
  cnt[PXB_C_STUCK] += !!(f & PXB_F_STUCK);
  cnt[PXB_C_PANIC] += !!(f & PXB_F_PANIC);
  cnt[PXB_C_DIVERGENCE] += !!(f & PXB_F_LOG_DIVERGENCE);
  cnt[PXB_C_STEP_CAP] += !!(f & PXB_F_STEP_CAP);
  cnt[PXB_C_ROUNDS] += I->rounds;
  cnt[PXB_C_MESSAGES] += (int64_t)I->messages;
  cnt[PXB_C_QUEUE_OVERFLOW] += !!(f & PXB_F_QUEUE_OVERFLOW);
  cnt[PXB_C_TICKET_OVERFLOW] += !!(f & PXB_F_TICKET_OVERFLOW);
  cnt[PXB_C_LOG_TRUNC] += !!(f & PXB_F_LOG_TRUNC);
  cnt[PXB_C_CANON_BYTES] += (int64_t)I->canon;
  cnt[PXB_C_STEPS] += steps;
  cnt[PXB_C_INSTANCES] += 1;
  cnt[PXB_C_EXECUTES] += (int64_t)I->executes;
}

/* ---- threaded batch runner -------------------------------------------- */
typedef struct {
  const pxb_config* cfg;
  pxb_result* out; uint32_t* digest; pxb_acceptor_rec* acc;
  uint64_t begin, end;
  int64_t cnt[PXB_NCOUNTERS];
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  const pxb_config* cfg = j->cfg;
  uint32_t N = cfg->n_acceptors;
  for (uint64_t i = j->begin; i < j->end; ++i) {
    run_instance(cfg, cfg->first_instance + i, j->out ? j->out + i : NULL,
                 j->digest ? j->digest + i * N : NULL, j->acc ? j->acc + i * N : NULL, j->cnt);
  }
  return NULL;
}

int pxb_oracle_validate(const pxb_config* c) {
  if (!c) return PXB_E_INVAL;
  if (c->n_proposers < 1 || c->n_proposers > PXB_MAX_PROPOSERS) return PXB_E_INVAL;
  if (c->n_acceptors < PXB_MIN_ACCEPTORS || c->n_acceptors > PXB_MAX_ACCEPTORS) return PXB_E_INVAL;
  if (c->loss_ppm > 1000000u || c->crash_ppm > 1000000u) return PXB_E_INVAL;
  if (c->delay_max < 1 || c->delay_max > PXB_MAX_DELAY) return PXB_E_INVAL;
  if (c->crash_len_max < 1 || c->crash_len_max > 4096 || c->crash_start_max > 65535) return PXB_E_INVAL;
  if (c->skew_max > 4096) return PXB_E_INVAL;
  if (c->step_cap < 1 || c->step_cap > PXB_MAX_STEP_CAP) return PXB_E_INVAL;
  if (c->n_ticks > PXB_MAX_TICKS) return PXB_E_INVAL;
  if (c->n_ticks > 1 && (c->tick_period < 1 || c->tick_period > PXB_MAX_STEP_CAP)) return PXB_E_INVAL;
  return PXB_OK;
}

/* Same contract as pxb_run (include/paxos_batch.h) on host threads.
 * threads <= 0: one. Counters are ADDED into totals. */
int pxb_run_cpu(const pxb_config* cfg, pxb_result* out, uint32_t* log_digest,
                pxb_acceptor_rec* acc, pxb_counters* totals, int threads) {
  int rc = pxb_oracle_validate(cfg);
  if (rc) return rc;
  if (threads < 1) threads = 1;
  if ((uint64_t)threads > cfg->n_instances) threads = cfg->n_instances ? (int)cfg->n_instances : 1;
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return PXB_E_OOM; }
  uint64_t n = cfg->n_instances;
  for (int t = 0; t < threads; ++t) {
    jobs[t].cfg = cfg; jobs[t].out = out; jobs[t].digest = log_digest; jobs[t].acc = acc;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
  }
  for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, worker, &jobs[t]);
  worker(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
  if (totals)
    for (int t = 0; t < threads; ++t)
      for (int k = 0; k < PXB_NCOUNTERS; ++k) totals->c[k] += jobs[t].cnt[k];
  free(jobs); free(th);
  return PXB_OK;
}

/* Single-handler oracles (same message encoding as the GPU hooks). */
int pxb_oracle_acceptor_handle(pxb_acceptor_rec* st, const pxb_msg* req, pxb_msg* reply, uint32_t count) {
  for (uint32_t i = 0; i < count; ++i) {
    acc_t A; memset(&A, 0, sizeof(A));
    A.t_max = st[i].t_max; A.t_store = st[i].t_store; A.val = st[i].val;
    A.log_len = st[i].meta & 0x7FFFFFFFu; A.dead = (int)(st[i].meta >> 31);
    msg_t m = {req[i].kind, req[i].x, req[i].y, req[i].z, 0}, rep;
    int r = A.dead ? 0 : acceptor_handle(&A, &m, &rep);
    st[i].t_max = A.t_max; st[i].t_store = A.t_store; st[i].val = A.val;
    st[i].meta = A.log_len | ((uint32_t)(A.dead != 0) << 31);
    if (r) { reply[i].kind = rep.kind; reply[i].x = rep.x; reply[i].y = rep.y; reply[i].z = rep.z; }
    else   { reply[i].kind = PXB_MSG_NONE; reply[i].x = reply[i].y = 0; reply[i].z = 0; }
  }
  return PXB_OK;
}

int pxb_oracle_proposer_handle(pxb_proposer_rec* st, uint32_t N, const pxb_msg* msg,
                               pxb_msg* bc, uint32_t* nb, uint32_t count) {
  for (uint32_t i = 0; i < count; ++i) {
    prop_t pr = {st[i].ticket, st[i].cmd, st[i].acks, st[i].state, st[i].mr_t, st[i].mr_v,
                 st[i].r2_t, st[i].r2_v, (int)st[i].pending, st[i].client_id};
    msg_t m = {msg[i].kind, msg[i].x, msg[i].y, msg[i].z, 0}, out[2];
    int n = (msg[i].kind == 3) ? proposer_tick(&pr, out) : proposer_handle(&pr, (int)N, &m, out);
    st[i].ticket = pr.ticket; st[i].cmd = pr.cmd; st[i].acks = pr.acks; st[i].state = pr.rs;
    st[i].mr_t = pr.mr_t; st[i].mr_v = pr.mr_v; st[i].r2_t = pr.r2_t; st[i].r2_v = pr.r2_v;
    st[i].pending = (uint32_t)pr.pending;
    nb[i] = (uint32_t)n;
    for (int k = 0; k < 2; ++k) {
      if (k < n) { bc[2*i+k].kind = out[k].kind; bc[2*i+k].x = out[k].x; bc[2*i+k].y = out[k].y; bc[2*i+k].z = out[k].z; }
      else { bc[2*i+k].kind = PXB_MSG_NONE; bc[2*i+k].x = bc[2*i+k].y = 0; bc[2*i+k].z = 0; }
    }
  }
  return PXB_OK;
}
