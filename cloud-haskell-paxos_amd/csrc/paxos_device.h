// paxos_device.h — device-side protocol functions shared by the batch kernel
// and the single-handler hook kernels (paxos_batch.hip).
//
// These are the reference's message handlers restated for one GPU lane:
//   acceptor  handleClientRequest   /root/reference/src/Server.hs:54-78
//   proposer  handleServerResponse  /root/reference/src/Client.hs:128-189
//             haveMajority          /root/reference/src/Client.hs:191-194
//             handleTick            /root/reference/src/Client.hs:196-207
//   MostRecentProposal (<>)         /root/reference/src/Common.hs:61-65
// Semantics and quirks Q1..Q12: docs/SEMANTICS.md (= SURVEY.md §8.0).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pxb {

// ClientRequest tags (Common.hs:41-45)
constexpr uint32_t ASK = 0, PROPOSE = 1, EXECUTE = 2;
// ServerResponse tags (Common.hs:49-53)
constexpr uint32_t R1OK = 0, HAVE = 1, R2S = 2;
constexpr uint32_t NONE = 0xFFFFFFFFu;
// RoundState (Client.hs:51-56)
constexpr uint32_t IDLE = 0, ROUND1 = 1, ROUND2 = 2;

// ---- Philox4x32-10 (Random123 constants) --------------------------------
// Each round needs the full 64-bit products of two 32-bit words: written as
// 64-bit multiplies they compile to one v_mad_u64_u32 each instead of a
// v_mul_lo_u32 + v_mul_hi_u32 pair.
// three-input xor as one gfx950 v_bitop3_b32 (truth table 0x96); LLVM emits
// two v_xor_b32 for it
__host__ __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // one v_bitop3_b32 (truth table of a^b^c)
#else
  return a ^ b ^ c;
#endif
}

__host__ __device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0), n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

// the same with its 2 x 10 round keys precomputed: rk[2r], rk[2r+1] = the keys
// of round r (k0 + r * 0x9E3779B9, k1 + r * 0xBB67AE85)
__host__ __device__ __forceinline__ uint4 philox_rk(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                           const uint32_t (&rk)[20]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, rk[2 * r]), n2 = xor3((uint32_t)(p0 >> 32), c3, rk[2 * r + 1]);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  return make_uint4(c0, c1, c2, c3);
}

__host__ __device__ __forceinline__ uint32_t mulhi_n(uint32_t w, uint32_t n) {
  return (uint32_t)(((uint64_t)w * n) >> 32);   // v_mul_hi_u32 on the device
}

__host__ __device__ __forceinline__ uint32_t fnv_u32(uint32_t h, uint32_t v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    h ^= (v >> (8 * i)) & 0xFFu;
    h *= 0x01000193u;
  }
  return h;
}

// ---- acceptor: handleClientRequest (Server.hs:51-78) ----------------------
struct AccState {
  int32_t t_max;    // _largestIssuedTicket  Server.hs:26
  int32_t t_store;  // _proposal = Just (t_store, val) | Nothing (val == 0)
  uint32_t val;
  bool dead;        // Server.hs:76 pattern failure kills the actor (Q6)
};

// Returns the reply tag (or NONE).  exec_val != 0 when `executed <>= [c]` ran.
// Written as selects (no branches): every lane of a wave may hold a different
// request kind, and a branchy body costs exec-mask juggling on all of them.
// `live` = false makes the call a no-op (no state change, reply NONE), so the
// batch kernel can run it predicated instead of under a branch.
__device__ __forceinline__ uint32_t acceptor_step(AccState& A, bool live, uint32_t kind, int32_t x, uint32_t z,
                                                  int32_t& rx, int32_t& ry, uint32_t& rz,
                                                  uint32_t& exec_val) {
  const bool is_ask = live && kind == ASK;               // Server.hs:54
  const bool is_prop = live && kind == PROPOSE;          // Server.hs:64
  const bool is_exec = live && kind == EXECUTE;          // Server.hs:73
  const bool grant = is_ask && !(A.t_max >= x);          // :56  T_max >= t -> HaveTicket
  const bool accept = is_prop && (x == A.t_max);         // :66  equality, not >=
  const bool hit = is_exec && (A.t_max == x);            // :75
  const bool panic = hit && A.val == 0u;                 // :76 `Just (_, c) <-` fails (Q6)
  const bool run = hit && A.val != 0u;                   // :77-78
  const uint32_t rk = grant ? R1OK : accept ? R2S : ((is_ask || is_prop) ? HAVE : NONE);
  rx = grant ? x : (accept ? 0 : A.t_max);               // :58/:71 HaveTicket T_max; :62 Round1OK t
  ry = grant ? A.t_store : 0;                            // :61-62 Round1OK t prop
  rz = grant ? A.val : 0u;
  exec_val = run ? A.val : 0u;                           // :78 executed <>= [c]
  A.t_max = grant ? x : A.t_max;                         // :60
  A.t_store = accept ? x : (run ? 0 : A.t_store);        // :68 / :77
  A.val = accept ? z : (run ? 0u : A.val);
  A.dead = A.dead || panic;
  return rk;
}

// ---- proposer: ClientState (Client.hs:58-67) -------------------------------
struct PropState {
  int32_t ticket;   // _ticket
  uint32_t cmd;     // _mCommand (0 = Nothing)
  uint32_t acks;    // _numAcks
  uint32_t rs;      // _roundState tag
  int32_t mr_t;     // Round1State._mostRecentProposal
  uint32_t mr_v;
  int32_t r2_t;     // Round2State._proposal
  uint32_t r2_v;
  uint32_t pending; // Round2State._originalCommandPending (0 / 1)
};

struct Req {
  uint32_t kind;    // ASK / PROPOSE / EXECUTE, or NONE
  int32_t x;        // ticket
  uint32_t z;       // command (PROPOSE)
};

// handleTick (Client.hs:196-207).  `cmd_of_ticket` supplies the encoding of
// "c<clientId>.<t>" (compact kernels pass clientId itself, t is always 1).
__device__ __forceinline__ uint32_t proposer_tick(PropState& S, uint32_t cmd_code, Req& o0) {
  if (S.rs != IDLE) return 0;              // :199
  S.ticket += 1;                           // :200  (<+= returns the new value)
  S.cmd = cmd_code;                        // :202-204
  S.acks = 0;                              // :205
  S.rs = ROUND1;                           // :206
  S.mr_t = 0;
  S.mr_v = 0;
  o0.kind = ASK;                           // :207
  o0.x = S.ticket;
  o0.z = 0;
  return 1;
}

// handleServerResponse (Client.hs:125-189) for one response; the sender pid
// is ignored (Q3).  Returns the number of broadcasts (0..2) in tell order.
__device__ __forceinline__ uint32_t proposer_step(PropState& S, uint32_t n_acc, uint32_t kind,
                                                  int32_t x, int32_t y, uint32_t z, Req& o0, Req& o1) {
  const uint32_t maj = n_acc >> 1;         // haveMajority: acks > floor(N/2), :191-194
  if (kind == HAVE) {                      // :128
    if (S.rs != IDLE && x >= S.ticket) {   // :130-132
      S.ticket = x + 1;                    // :134-135
      S.acks = 0;                          // :137
      S.rs = ROUND1;                       // :138
      S.mr_t = 0;
      S.mr_v = 0;
      o0.kind = ASK;                       // :140
      o0.x = S.ticket;
      o0.z = 0;
      return 1;
    }
    return 0;
  }
  if (kind == R1OK) {                      // :142
    if (S.rs == ROUND1 && S.ticket == x) { // :144-145
      S.acks += 1;                         // :146
      int32_t mt = S.mr_t;                 // :147-151  mr <> MostRecent mp  (Common.hs:61-65)
      uint32_t mv = S.mr_v;
      if (mv == 0 || (z != 0 && !(mt >= y))) {
        mt = y;
        mv = z;
      }
      if (S.acks <= maj) {                 // :152-154
        S.mr_t = mt;
        S.mr_v = mv;
        return 0;
      }
      S.r2_t = x;                          // :157-167 (Q5: pending whenever mr is Just)
      S.r2_v = (mv == 0) ? S.cmd : mv;
      S.pending = (mv != 0) ? 1u : 0u;
      S.acks = 0;                          // :168
      S.rs = ROUND2;                       // :169
      S.mr_t = 0;
      S.mr_v = 0;
      o0.kind = PROPOSE;                   // :170
      o0.x = S.r2_t;
      o0.z = S.r2_v;
      return 1;
    }
    return 0;
  }
  if (S.rs == ROUND2) {                    // Round2Success, :172-174 (no ticket: Q2)
    S.acks += 1;                           // :175
    if (S.acks > maj) {                    // :176-177
      o0.kind = EXECUTE;                   // :178 Execute (s ^. ticket)
      o0.x = S.ticket;
      o0.z = 0;
      if (S.pending) {                     // :179
        S.ticket += 1;                     // :182
        S.acks = 0;                        // :183
        S.rs = ROUND1;                     // :184
        S.mr_t = 0;
        S.mr_v = 0;
        o1.kind = ASK;                     // :185
        o1.x = S.ticket;
        o1.z = 0;
        return 2;
      }
      S.cmd = 0;                           // :187
      S.acks = 0;                          // :188
      S.rs = IDLE;                         // :189
      return 1;
    }
  }
  return 0;
}

}  // namespace pxb
