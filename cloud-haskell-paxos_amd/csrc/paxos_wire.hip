// paxos_wire.hip — batch codec for the reference's wire format.
//
// Encodes / decodes the `Data.Binary` payloads of the message vocabulary,
// the bytes `send` serialises for `contentOf m` (Common.hs:36-39):
//   ClientRequest  = AskForTicket Ticket | Propose (Ticket, Command) | Execute Ticket
//   ServerResponse = Round1OK Ticket (Maybe Proposal) | HaveTicket Ticket | Round2Success
// with the GHC.Generics instances of binary-0.8.5.1 (Common.hs:24,47,55): a
// Word8 constructor tag (0, 1, 2 in declaration order), Int = Int64 big-endian,
// Maybe = Word8 0 | 1 + value, String = Int length + UTF-8 chars.  Restated
// and pinned in oracle/wire_ref.py.
//
// One thread per message.  Sizes -> exclusive offsets (hipCUB scan) ->
// bytes; decoding takes the offsets (the transport frames every message) and
// reports a status per message.  HBM-bound byte work: 16 B of pxb_msg plus
// 1..39 B of wire bytes per message.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <mutex>
#include <stdint.h>
#include <string.h>

#include "../../include/paxos_batch.h"

namespace pxw {

// constructor tags in declaration order (putSum of Data.Binary.Generic)
constexpr uint32_t PROPOSE = 1;                         // ClientRequest: AskForTicket 0, Propose 1, Execute 2
constexpr uint32_t R1OK = 0, HAVE = 1;                  // ServerResponse: Round1OK 0, HaveTicket 1, Round2Success 2

__device__ __forceinline__ uint32_t ndigits(uint32_t v) {
  uint32_t n = 1;
#pragma unroll
  for (uint32_t p = 10; p <= 10000000u; p *= 10) n += (v >= p) ? 1u : 0u;
  return n;                                              // v < 10^8 (t < 2^24)
}
// length of "c<id>.<t>" (Client.hs:202-203)
__device__ __forceinline__ uint32_t cmd_len(uint32_t code) {
  return 2u + ndigits(code >> 24) + ndigits(code & 0xFFFFFFu);
}

__device__ __forceinline__ uint32_t record_size(const pxb_msg& m, uint32_t type) {
  if (m.kind > 2u) return 0u;                            // not a constructor: empty record
  if (type == PXB_WIRE_REQUEST) return (m.kind == PROPOSE) ? 17u + cmd_len(m.z) : 9u;
  if (m.kind == R1OK) return (m.z == 0u) ? 10u : 26u + cmd_len(m.z);
  return (m.kind == HAVE) ? 9u : 1u;
}

__global__ void size_kernel(const pxb_msg* __restrict__ msgs, uint64_t n, uint32_t type,
                            uint64_t* __restrict__ offs) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) offs[0] = 0;
  if (i < n) offs[i + 1] = record_size(msgs[i], type);
}

struct Out {
  uint8_t* p;
  __device__ __forceinline__ void u8(uint32_t v) { *p++ = (uint8_t)v; }
  __device__ __forceinline__ void i64(int32_t v) {       // Binary Int: Int64 big-endian
    const uint64_t w = (uint64_t)(int64_t)v;
#pragma unroll
    for (int k = 7; k >= 0; --k) u8((uint32_t)(w >> (8 * k)) & 0xFFu);
  }
  __device__ __forceinline__ void digits(uint32_t v) {
    const uint32_t nd = ndigits(v);
    for (uint32_t k = 0; k < nd; ++k) {
      p[nd - 1 - k] = (uint8_t)('0' + v % 10u);
      v /= 10u;
    }
    p += nd;
  }
  __device__ __forceinline__ void command(uint32_t code) {   // Binary [Char]
    i64((int32_t)cmd_len(code));
    u8('c');
    digits(code >> 24);
    u8('.');
    digits(code & 0xFFFFFFu);
  }
};

__global__ void encode_kernel(const pxb_msg* __restrict__ msgs, uint64_t n, uint32_t type,
                              const uint64_t* __restrict__ offs, uint8_t* __restrict__ bytes) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const pxb_msg m = msgs[i];
  if (m.kind > 2u) return;
  Out o{bytes + offs[i]};
  o.u8(m.kind);                                          // constructor tag
  if (type == PXB_WIRE_REQUEST) {
    o.i64(m.x);                                          // the Ticket of every request
    if (m.kind == PROPOSE) o.command(m.z);               // Proposal = (Ticket, Command)
  } else if (m.kind == R1OK) {
    o.i64(m.x);
    if (m.z == 0u) {
      o.u8(0);                                           // Nothing
    } else {
      o.u8(1);                                           // Just (t_store, command)
      o.i64(m.y);
      o.command(m.z);
    }
  } else if (m.kind == HAVE) {
    o.i64(m.x);
  }
}

struct In {
  const uint8_t* p;
  const uint8_t* end;
  uint32_t err;
  __device__ __forceinline__ bool need(uint64_t k) {
    if (err == 0u && (uint64_t)(end - p) < k) err = PXB_WIRE_E_LENGTH;
    return err == 0u;
  }
  __device__ __forceinline__ uint32_t u8() { return need(1) ? *p++ : 0u; }
  __device__ __forceinline__ int64_t i64() {
    if (!need(8)) return 0;
    uint64_t w = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) w = (w << 8) | p[k];
    p += 8;
    return (int64_t)w;
  }
  __device__ __forceinline__ int32_t int32() {
    const int64_t v = i64();
    if (err == 0u && (v < -(int64_t)2147483648ll || v > 2147483647ll)) err = PXB_WIRE_E_RANGE;
    return (int32_t)v;
  }
  // one run of `show` digits (no leading zero), returns the value (64-bit: <= 11 digits)
  __device__ __forceinline__ uint64_t digits(const uint8_t* s, uint32_t n, uint32_t& i) {
    const uint32_t i0 = i;
    uint64_t v = 0;
    while (i < n && s[i] >= '0' && s[i] <= '9') v = v * 10u + (uint64_t)(s[i++] - '0');
    if (i == i0 || (i - i0 > 1 && s[i0] == '0')) err = err ? err : PXB_WIRE_E_STRING;
    return v;
  }
  __device__ __forceinline__ uint32_t command() {
    const int64_t n64 = i64();
    if (err) return 0u;
    if (n64 < 4 || n64 > 13) { err = PXB_WIRE_E_STRING; return 0u; }
    const uint32_t n = (uint32_t)n64;
    if (!need(n)) return 0u;
    const uint8_t* s = p;
    p += n;
    if (s[0] != 'c') { err = PXB_WIRE_E_STRING; return 0u; }
    uint32_t i = 1;
    const uint64_t id = digits(s, n, i);
    if (err) return 0u;
    if (i >= n || s[i] != '.') { err = PXB_WIRE_E_STRING; return 0u; }
    ++i;
    const uint64_t t = digits(s, n, i);
    if (err) return 0u;
    if (i != n) { err = PXB_WIRE_E_STRING; return 0u; }
    if (id > 255u || t > 0xFFFFFFu) { err = PXB_WIRE_E_RANGE; return 0u; }
    return (uint32_t)((id << 24) | t);
  }
};

__global__ void decode_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ offs, uint64_t n,
                              uint32_t type, pxb_msg* __restrict__ msgs, uint32_t* __restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = offs[i], e = offs[i + 1];
  In r{bytes + b, bytes + (e >= b ? e : b), 0u};
  pxb_msg m{0, 0, 0, 0};
  const uint32_t tag = r.u8();
  if (!r.err) {
    if (tag > 2u) {
      r.err = PXB_WIRE_E_TAG;
    } else if (type == PXB_WIRE_REQUEST) {
      m.x = r.int32();
      if (tag == PROPOSE) m.z = r.command();
    } else if (tag == R1OK) {
      m.x = r.int32();
      const uint32_t just = r.u8();
      if (!r.err) {
        if (just == 1u) {
          m.y = r.int32();
          m.z = r.command();
        } else if (just != 0u) {
          r.err = PXB_WIRE_E_TAG;
        }
      }
    } else if (tag == HAVE) {
      m.x = r.int32();
    }
  }
  if (!r.err && r.p != r.end) r.err = PXB_WIRE_E_LENGTH;   // trailing bytes
  m.kind = tag;
  if (r.err) m = pxb_msg{0, 0, 0, 0};
  msgs[i] = m;
  if (status) status[i] = r.err;
}

// scan scratch (grown on demand, one buffer per device)
std::mutex g_mu;
void* g_tmp[64];
size_t g_tmp_bytes[64];

int hip_fail(hipError_t e) { return (e == hipErrorOutOfMemory) ? PXB_E_OOM : PXB_E_HIP; }

unsigned grid_of(uint64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace pxw

using namespace pxw;

extern "C" {

int pxb_wire_size(const pxb_msg* d_msgs, uint64_t count, uint32_t type, uint64_t* d_offsets, void* stream) {
  if (type > PXB_WIRE_RESPONSE || !d_offsets || (count && !d_msgs) || count > (1ull << 40)) return PXB_E_INVAL;
  const hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(size_kernel, dim3(grid_of(count ? count : 1)), dim3(256), 0, st, d_msgs, count, type,
                     d_offsets);
  if (hipGetLastError() != hipSuccess) return PXB_E_HIP;
  if (count == 0) return PXB_OK;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return PXB_E_NODEV;
  std::lock_guard<std::mutex> lk(g_mu);
  size_t need = 0;
  if (hipcub::DeviceScan::InclusiveSum(nullptr, need, d_offsets + 1, d_offsets + 1, (int64_t)count, st) !=
      hipSuccess)
    return PXB_E_HIP;
  if (need > g_tmp_bytes[dev]) {
    if (g_tmp[dev]) (void)hipFree(g_tmp[dev]);
    g_tmp[dev] = nullptr;
    g_tmp_bytes[dev] = 0;
    hipError_t e = hipMalloc(&g_tmp[dev], need);
    if (e != hipSuccess) return hip_fail(e);
    g_tmp_bytes[dev] = need;
  }
  size_t have = g_tmp_bytes[dev];
  hipError_t e = hipcub::DeviceScan::InclusiveSum(g_tmp[dev], have, d_offsets + 1, d_offsets + 1, (int64_t)count, st);
  return (e == hipSuccess) ? PXB_OK : hip_fail(e);
}

int pxb_wire_encode(const pxb_msg* d_msgs, uint64_t count, uint32_t type, const uint64_t* d_offsets,
                    uint8_t* d_bytes, void* stream) {
  if (type > PXB_WIRE_RESPONSE || count > (1ull << 40)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  if (!d_msgs || !d_offsets || !d_bytes) return PXB_E_INVAL;
  hipLaunchKernelGGL(encode_kernel, dim3(grid_of(count)), dim3(256), 0, (hipStream_t)stream, d_msgs, count, type,
                     d_offsets, d_bytes);
  return (hipGetLastError() == hipSuccess) ? PXB_OK : PXB_E_HIP;
}

int pxb_wire_decode(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t count, uint32_t type,
                    pxb_msg* d_msgs, uint32_t* d_status, void* stream) {
  if (type > PXB_WIRE_RESPONSE || count > (1ull << 40)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  if (!d_offsets || !d_msgs || !d_bytes) return PXB_E_INVAL;
  hipLaunchKernelGGL(decode_kernel, dim3(grid_of(count)), dim3(256), 0, (hipStream_t)stream, d_bytes, d_offsets,
                     count, type, d_msgs, d_status);
  return (hipGetLastError() == hipSuccess) ? PXB_OK : PXB_E_HIP;
}

int pxb_wire_encode_host(const pxb_msg* msgs, uint64_t count, uint32_t type, uint8_t* out, uint64_t* offsets,
                         uint64_t* nbytes) {
  if (type > PXB_WIRE_RESPONSE || !offsets || !nbytes || (count && (!msgs || !out))) return PXB_E_INVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  pxb_msg* d_m = nullptr;
  uint64_t* d_o = nullptr;
  uint8_t* d_b = nullptr;
  hipError_t e = hipSuccess;
  int rc = PXB_OK;
  do {
    if ((e = hipMalloc(&d_o, (count + 1) * sizeof(uint64_t))) != hipSuccess) break;
    if (count && (e = hipMalloc(&d_m, count * sizeof(pxb_msg))) != hipSuccess) break;
    if (count && (e = hipMemcpy(d_m, msgs, count * sizeof(pxb_msg), hipMemcpyHostToDevice)) != hipSuccess) break;
    if ((rc = pxb_wire_size(d_m, count, type, d_o, nullptr)) != PXB_OK) break;
    if ((e = hipMemcpy(offsets, d_o, (count + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost)) != hipSuccess) break;
    *nbytes = offsets[count];
    if (count && (e = hipMalloc(&d_b, *nbytes ? *nbytes : 1)) != hipSuccess) break;
    if ((rc = pxb_wire_encode(d_m, count, type, d_o, d_b, nullptr)) != PXB_OK) break;
    if (*nbytes && (e = hipMemcpy(out, d_b, *nbytes, hipMemcpyDeviceToHost)) != hipSuccess) break;
  } while (0);
  if (d_m) (void)hipFree(d_m);
  if (d_o) (void)hipFree(d_o);
  if (d_b) (void)hipFree(d_b);
  if (e != hipSuccess) return hip_fail(e);
  return rc;
}

int pxb_wire_decode_host(const uint8_t* in, const uint64_t* offsets, uint64_t count, uint32_t type, pxb_msg* msgs,
                         uint32_t* status) {
  if (type > PXB_WIRE_RESPONSE || !offsets || (count && (!in || !msgs))) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  const uint64_t nb = offsets[count];
  pxb_msg* d_m = nullptr;
  uint64_t* d_o = nullptr;
  uint8_t* d_b = nullptr;
  uint32_t* d_s = nullptr;
  hipError_t e = hipSuccess;
  int rc = PXB_OK;
  do {
    if ((e = hipMalloc(&d_o, (count + 1) * sizeof(uint64_t))) != hipSuccess) break;
    if ((e = hipMalloc(&d_m, count * sizeof(pxb_msg))) != hipSuccess) break;
    if ((e = hipMalloc(&d_b, nb ? nb : 1)) != hipSuccess) break;
    if (status && (e = hipMalloc(&d_s, count * sizeof(uint32_t))) != hipSuccess) break;
    if ((e = hipMemcpy(d_o, offsets, (count + 1) * sizeof(uint64_t), hipMemcpyHostToDevice)) != hipSuccess) break;
    if (nb && (e = hipMemcpy(d_b, in, nb, hipMemcpyHostToDevice)) != hipSuccess) break;
    if ((rc = pxb_wire_decode(d_b, d_o, count, type, d_m, d_s, nullptr)) != PXB_OK) break;
    if ((e = hipMemcpy(msgs, d_m, count * sizeof(pxb_msg), hipMemcpyDeviceToHost)) != hipSuccess) break;
    if (status && (e = hipMemcpy(status, d_s, count * sizeof(uint32_t), hipMemcpyDeviceToHost)) != hipSuccess) break;
  } while (0);
  if (d_m) (void)hipFree(d_m);
  if (d_o) (void)hipFree(d_o);
  if (d_b) (void)hipFree(d_b);
  if (d_s) (void)hipFree(d_s);
  if (e != hipSuccess) return hip_fail(e);
  return rc;
}

}  // extern "C"
