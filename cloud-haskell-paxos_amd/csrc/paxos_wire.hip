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
// One thread per message.  Sizes: one hipCUB scan over the record sizes
// computed on the fly (no size pass in HBM).  Encoding: a tile of ETILE
// messages builds its records in LDS at their tile-local offsets (block scan
// of the sizes, one global offset per tile) and writes the tile's contiguous
// byte range with aligned 16-B stores.  pxb_wire_encode_all fuses the two:
// per-tile size sums, a scan of those, then the encode tiles also write the
// offsets (HBM: the messages twice, offsets and bytes once).  Decoding stages the tile's byte range
// through LDS with aligned 16-B loads and parses from LDS (records outside a
// well-formed tile range are parsed straight from HBM).  Every message gets a
// status.  HBM-bound byte work: 16 B of pxb_msg plus 1..39 B of wire bytes per
// message.
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

// messages per block, one per thread (measured: small encode tiles overlap
// their scan / LDS / store phases better; decode prefers long staged ranges)
constexpr int ETILE = 256;
constexpr int DTILE = 1024;
// LDS stage of a tile's bytes in uint4: worst case + the alignment head
template <int T> struct Stage { static constexpr int n = (T * PXB_WIRE_MAX_BYTES + 16 + 15) / 16; };

struct SizeOp {
  uint32_t type;
  __device__ __forceinline__ uint64_t operator()(const pxb_msg& m) const { return record_size(m, type); }
};

// inclusive scan over the threads of a T-thread block (wave scans + LDS)
template <int T>
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, off);
    v += (lane >= off) ? o : 0u;
  }
  if (lane == 63) s_w[w] = v;
  __syncthreads();
  if (w == 0) {
    uint32_t t = (lane < T / 64) ? s_w[lane] : 0u;
#pragma unroll
    for (int off = 1; off < T / 64; off <<= 1) {
      const uint32_t o = (uint32_t)__shfl_up((int)t, off);
      t += (lane >= off) ? o : 0u;
    }
    if (lane < T / 64) s_w[lane] = t;
  }
  __syncthreads();
  total = s_w[T / 64 - 1];
  return v + (w ? s_w[w - 1] : 0u);
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

__device__ __forceinline__ void encode_record(Out& o, const pxb_msg& m, uint32_t type) {
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

// sum of the record sizes of every ETILE-message tile (encode_all pass 1); a
// block covers SUM_TILES tiles so every thread keeps that many loads in flight
constexpr int SUM_TILES = 4;
__global__ __launch_bounds__(ETILE) void tile_sum_kernel(const pxb_msg* __restrict__ msgs, uint64_t n, uint32_t type,
                                                         uint64_t ntiles, uint64_t* __restrict__ tsum) {
  __shared__ uint32_t s_w[SUM_TILES][ETILE / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * SUM_TILES;
  pxb_msg m[SUM_TILES];
#pragma unroll
  for (int j = 0; j < SUM_TILES; ++j) {
    const uint64_t i = (t0 + j) * ETILE + threadIdx.x;
    m[j] = (i < n) ? msgs[i] : pxb_msg{3u, 0, 0, 0};
  }
#pragma unroll
  for (int j = 0; j < SUM_TILES; ++j) {
    uint32_t v = (m[j].kind <= 2u) ? record_size(m[j], type) : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    if ((threadIdx.x & 63) == 0) s_w[j][threadIdx.x >> 6] = v;
  }
  __syncthreads();
  if (threadIdx.x < SUM_TILES && t0 + threadIdx.x < ntiles) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < ETILE / 64; ++w) t += s_w[threadIdx.x][w];
    tsum[t0 + threadIdx.x] = t;
  }
}

// One tile: records built in LDS, then the tile's byte range [base, base +
// total) written with aligned 16-B stores (byte stores only for the partial
// 16-B chunks at its two ends, which neighbouring tiles share).  The tile's
// base is offs[first] (pxb_wire_encode) or the scanned tile sum, in which case
// the tile also writes its offsets (pxb_wire_encode_all).
template <bool WRITE_OFFS>
__global__ __launch_bounds__(ETILE) void encode_kernel(const pxb_msg* __restrict__ msgs, uint64_t n, uint32_t type,
                                                       uint64_t* __restrict__ offs, const uint64_t* __restrict__ toff,
                                                       uint8_t* __restrict__ bytes) {
  __shared__ uint4 s_buf[Stage<ETILE>::n];
  __shared__ uint32_t s_w[ETILE / 64];
  uint8_t* buf = reinterpret_cast<uint8_t*>(s_buf);
  const uint64_t first = (uint64_t)blockIdx.x * ETILE;
  const uint64_t i = first + threadIdx.x;
  pxb_msg m{3u, 0, 0, 0};
  if (i < n) m = msgs[i];
  const uint32_t sz = (m.kind <= 2u) ? record_size(m, type) : 0u;
  uint32_t total;
  const uint32_t loc = block_scan<ETILE>(sz, s_w, total) - sz;
  const uint64_t base = WRITE_OFFS ? toff[blockIdx.x] : offs[first];
  if (WRITE_OFFS) {
    if (i < n) offs[i + 1] = base + loc + sz;
    if (i == 0) offs[0] = 0;
  }
  uint8_t* gdst = bytes + base;
  const uint32_t pad = (uint32_t)((uintptr_t)gdst & 15u);  // LDS byte k <-> global gdst - pad + k
  if (sz) {
    Out o{buf + pad + loc};
    encode_record(o, m, type);
  }
  __syncthreads();
  const uint32_t span = pad + total;
  uint8_t* g0 = gdst - pad;                              // 16-B aligned
  for (uint32_t c = threadIdx.x; c * 16u < span; c += ETILE) {
    const uint32_t k0 = c * 16u;
    if (k0 >= pad && k0 + 16u <= span) {
      *reinterpret_cast<uint4*>(g0 + k0) = s_buf[c];
    } else {
      for (uint32_t k = max(k0, pad); k < min(k0 + 16u, span); ++k) g0[k] = buf[k];
    }
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

__device__ __forceinline__ uint32_t decode_record(In& r, uint32_t type, pxb_msg& m) {
  m = pxb_msg{0, 0, 0, 0};
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
  return r.err;
}

// One tile: when its offsets are monotone and its byte range fits the stage,
// the range is loaded with aligned 16-B loads into LDS and each record parsed
// from there; any record outside that range (or a tile with malformed
// offsets) is parsed straight from HBM.
__global__ __launch_bounds__(DTILE) void decode_kernel(const uint8_t* __restrict__ bytes, uint64_t nbytes,
                                                      const uint64_t* __restrict__ offs, uint64_t n, uint32_t type,
                                                      pxb_msg* __restrict__ msgs, uint32_t* __restrict__ status) {
  __shared__ uint4 s_buf[Stage<DTILE>::n];
  const uint8_t* buf = reinterpret_cast<const uint8_t*>(s_buf);
  const uint64_t first = (uint64_t)blockIdx.x * DTILE;
  const uint64_t last = min(first + (uint64_t)DTILE, n);
  const uint64_t lo = offs[first], hi = offs[last];
  const bool staged = hi >= lo && hi <= nbytes && hi - lo <= (uint64_t)DTILE * PXB_WIRE_MAX_BYTES;
  const uint8_t* gsrc = bytes + lo;
  const uint32_t pad = (uint32_t)((uintptr_t)gsrc & 15u);   // LDS byte k <-> global gsrc - pad + k
  if (staged) {
    const uint32_t span = pad + (uint32_t)(hi - lo);
    const uint8_t* g0 = gsrc - pad;
    for (uint32_t c = threadIdx.x; c * 16u < span; c += DTILE) {
      const uint32_t k0 = c * 16u;
      if (k0 >= pad && k0 + 16u <= span) {
        s_buf[c] = *reinterpret_cast<const uint4*>(g0 + k0);
      } else {
        uint8_t* d = reinterpret_cast<uint8_t*>(s_buf);
        for (uint32_t k = max(k0, pad); k < min(k0 + 16u, span); ++k) d[k] = g0[k];
      }
    }
  }
  __syncthreads();
  const uint64_t i = first + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = offs[i], e = offs[i + 1];
  const uint64_t ee = (e >= b) ? e : b;
  pxb_msg m;
  uint32_t err;
  if (ee > nbytes) {                       // the record reaches past the buffer
    m = pxb_msg{0, 0, 0, 0};
    err = PXB_WIRE_E_LENGTH;
  } else if (staged && b >= lo && ee <= hi) {
    const uint8_t* p = buf + pad + (uint32_t)(b - lo);
    In r{p, p + (uint32_t)(ee - b), 0u};
    err = decode_record(r, type, m);
  } else {
    In r{bytes + b, bytes + ee, 0u};
    err = decode_record(r, type, m);
  }
  msgs[i] = m;
  if (status) status[i] = err;
}

// Per-call scratch (the scans' temporary storage, the tile sums and offsets)
// comes from a stream-ordered pool per device: allocated and freed on the
// caller's stream, so calls on different streams never share a buffer and a
// buffer is never freed under a kernel still using it.
std::mutex g_mu;
hipMemPool_t g_pool[64];

int hip_fail(hipError_t e) { return (e == hipErrorOutOfMemory) ? PXB_E_OOM : PXB_E_HIP; }

unsigned tiles_of(uint64_t n, int tile) { return (unsigned)((n + tile - 1) / tile); }

int scratch(int dev, size_t bytes, hipStream_t st, void** p) {
  hipMemPool_t pool;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_pool[dev]) {
      hipMemPoolProps props;
      memset(&props, 0, sizeof(props));
      props.allocType = hipMemAllocationTypePinned;
      props.location.type = hipMemLocationTypeDevice;
      props.location.id = dev;
      hipError_t e = hipMemPoolCreate(&g_pool[dev], &props);
      if (e != hipSuccess) {
        g_pool[dev] = nullptr;
        return hip_fail(e);
      }
      uint64_t keep = 64ull << 20;                       // (kept across synchronisations)
      (void)hipMemPoolSetAttribute(g_pool[dev], hipMemPoolAttrReleaseThreshold, &keep);
    }
    pool = g_pool[dev];
  }
  hipError_t e = hipMallocFromPoolAsync(p, bytes ? bytes : 1, pool, st);
  return (e == hipSuccess) ? PXB_OK : hip_fail(e);
}

}  // namespace pxw

using namespace pxw;

extern "C" {

// internal (pxb_shutdown): destroy the per-device scratch pools
void pxb_wire_release(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  int cur = 0;
  const bool have = hipGetDevice(&cur) == hipSuccess;
  for (int d = 0; d < 64; ++d) {
    if (!g_pool[d]) continue;
    (void)hipSetDevice(d);
    (void)hipDeviceSynchronize();
    (void)hipMemPoolDestroy(g_pool[d]);
    g_pool[d] = nullptr;
  }
  if (have) (void)hipSetDevice(cur);
}

int pxb_wire_size(const pxb_msg* d_msgs, uint64_t count, uint32_t type, uint64_t* d_offsets, void* stream) {
  if (type > PXB_WIRE_RESPONSE || !d_offsets || (count && !d_msgs) || count > (1ull << 40)) return PXB_E_INVAL;
  const hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), st) != hipSuccess) return PXB_E_HIP;
  if (count == 0) return PXB_OK;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return PXB_E_NODEV;
  // offsets[1..count] = inclusive sum of the record sizes, computed as the
  // scan reads the messages
  hipcub::TransformInputIterator<uint64_t, SizeOp, const pxb_msg*> sizes(d_msgs, SizeOp{type});
  size_t need = 0;
  if (hipcub::DeviceScan::InclusiveSum(nullptr, need, sizes, d_offsets + 1, (int64_t)count, st) != hipSuccess)
    return PXB_E_HIP;
  void* tmp = nullptr;
  if (int rc = scratch(dev, need, st, &tmp)) return rc;
  hipError_t e = hipcub::DeviceScan::InclusiveSum(tmp, need, sizes, d_offsets + 1, (int64_t)count, st);
  const hipError_t f = hipFreeAsync(tmp, st);
  if (e == hipSuccess) e = f;
  return (e == hipSuccess) ? PXB_OK : hip_fail(e);
}

int pxb_wire_encode(const pxb_msg* d_msgs, uint64_t count, uint32_t type, const uint64_t* d_offsets,
                    uint8_t* d_bytes, void* stream) {
  if (type > PXB_WIRE_RESPONSE || count > (1ull << 40)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  if (!d_msgs || !d_offsets || !d_bytes) return PXB_E_INVAL;
  hipLaunchKernelGGL(encode_kernel<false>, dim3(tiles_of(count, ETILE)), dim3(ETILE), 0, (hipStream_t)stream, d_msgs,
                     count, type, const_cast<uint64_t*>(d_offsets), nullptr, d_bytes);
  return (hipGetLastError() == hipSuccess) ? PXB_OK : PXB_E_HIP;
}

int pxb_wire_encode_all(const pxb_msg* d_msgs, uint64_t count, uint32_t type, uint64_t* d_offsets,
                        uint8_t* d_bytes, void* stream) {
  if (type > PXB_WIRE_RESPONSE || !d_offsets || count > (1ull << 40)) return PXB_E_INVAL;
  const hipStream_t st = (hipStream_t)stream;
  if (count == 0) return (hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), st) == hipSuccess) ? PXB_OK : PXB_E_HIP;
  if (!d_msgs || !d_bytes) return PXB_E_INVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return PXB_E_NODEV;
  const uint64_t tiles = tiles_of(count, ETILE);
  size_t need = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, need, (uint64_t*)nullptr, (uint64_t*)nullptr, (int64_t)tiles, st) !=
      hipSuccess)
    return PXB_E_HIP;
  const size_t arr = ((tiles * sizeof(uint64_t)) + 255) & ~(size_t)255;
  void* buf = nullptr;
  if (int rc = scratch(dev, 2 * arr + need, st, &buf)) return rc;
  uint64_t* tsum = reinterpret_cast<uint64_t*>(buf);
  uint64_t* toff = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(buf) + arr);
  void* tmp = reinterpret_cast<char*>(buf) + 2 * arr;
  hipLaunchKernelGGL(tile_sum_kernel, dim3((unsigned)((tiles + SUM_TILES - 1) / SUM_TILES)), dim3(ETILE), 0, st, d_msgs,
                     count, type, tiles, tsum);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, need, tsum, toff, (int64_t)tiles, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(encode_kernel<true>, dim3((unsigned)tiles), dim3(ETILE), 0, st, d_msgs, count, type, d_offsets,
                       toff, d_bytes);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(buf, st);     // (stream-ordered: after the launches above)
  if (e == hipSuccess) e = f;
  return (e == hipSuccess) ? PXB_OK : hip_fail(e);
}

int pxb_wire_decode(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_offsets, uint64_t count,
                    uint32_t type, pxb_msg* d_msgs, uint32_t* d_status, void* stream) {
  if (type > PXB_WIRE_RESPONSE || count > (1ull << 40)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  if (!d_offsets || !d_msgs || (n_bytes && !d_bytes)) return PXB_E_INVAL;
  hipLaunchKernelGGL(decode_kernel, dim3(tiles_of(count, DTILE)), dim3(DTILE), 0, (hipStream_t)stream, d_bytes, n_bytes,
                     d_offsets, count, type, d_msgs, d_status);
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

int pxb_wire_decode_host(const uint8_t* in, uint64_t n_bytes, const uint64_t* offsets, uint64_t count, uint32_t type,
                         pxb_msg* msgs, uint32_t* status) {
  if (type > PXB_WIRE_RESPONSE || !offsets || (count && !msgs) || (n_bytes && !in)) return PXB_E_INVAL;
  if (count == 0) return PXB_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return PXB_E_NODEV;
  uint64_t nb = 0;                                       // bytes the offsets reach inside the buffer
  for (uint64_t k = 0; k <= count; ++k) nb = (offsets[k] > nb) ? offsets[k] : nb;
  nb = (nb < n_bytes) ? nb : n_bytes;
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
    if ((rc = pxb_wire_decode(d_b, nb, d_o, count, type, d_m, d_s, nullptr)) != PXB_OK) break;
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
