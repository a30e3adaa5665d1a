/*
 * paxos_batch.h — C ABI of the MI355X batched single-decree ticket-Paxos engine.
 *
 * This is the drop-in boundary for the hot path of rgrover/cloud-haskell-paxos.
 * The reference has NO FFI of its own: its externally visible
 * surface is
 *     server :: Process ()                        /root/reference/src/Server.hs:44
 *     client :: [ProcessId] -> Int -> Process ()  /root/reference/src/Client.hs:85
 * spawned N x / P x by  main  (/root/reference/app/Main.hs:41-46), with the
 * message vocabulary of /root/reference/src/Common.hs:20-68.  A batch driver in
 * app/Main.hs binds the functions below with `foreign import ccall safe`
 * (INTEGRATION.md shows the binding).  Each call runs many independent Paxos
 * instances (N acceptors + P proposers each) under the canonical step schedule
 * of docs/SEMANTICS.md on the GPU and returns the per-instance outcome.
 *
 * Plain C types only.  No C++ exceptions cross this boundary.  All functions
 * return 0 on success or a negative PXB_E_* code.  Protocol failures (panic,
 * stuck, divergence, ...) are DATA in pxb_result.flags, not errors.
 */
#ifndef PAXOS_BATCH_H
#define PAXOS_BATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PXB_ABI_VERSION 5   /* 3: pxb_init / pxb_shutdown, n_bytes bound on wire decode;
                               4: pxb_stream_release, pxb_handoff_counts;
                               5: pxb_reload_hooks, pxb_trace_instance in log mode */

/* ---- error codes ---------------------------------------------------------- */
#define PXB_OK          0
#define PXB_E_INVAL    -1   /* bad config / null pointer / out-of-range field  */
#define PXB_E_HIP      -2   /* HIP runtime error (detail: pxb_last_hip_error)   */
#define PXB_E_OOM      -3   /* device allocation failed                          */
#define PXB_E_NODEV    -4   /* no GPU visible                                    */
#define PXB_E_RCCL     -5   /* collective failure                                */

/* ---- limits of the canonical schedule (docs/SEMANTICS.md §3) ------------ */
#define PXB_MAX_PROPOSERS   3
#define PXB_MIN_ACCEPTORS   2
#define PXB_MAX_ACCEPTORS   9
#define PXB_MAX_DELAY      15
#define PXB_MAX_STEP_CAP 8192
#define PXB_QUEUE_DEPTH     8    /* messages per directed link              */
#define PXB_LOG_TRACK      32    /* log positions checked for divergence    */
#define PXB_TICKET_LIMIT (1 << 14)   /* = the 14-bit ticket fields of the kernel words */
#define PXB_MAX_TICKS    4096    /* log mode: Ticks per proposer            */

/* pxb_config.flags */
#define PXB_CFG_RANDOMIZE 1u     /* config-5 fuzz: per-instance P, loss, delay,
                                    crash drawn from Philox (n_proposers,
                                    loss_ppm, delay_max, crash_ppm are maxima) */
#define PXB_CFG_TRACE_PRODUCTION 2u  /* pxb_trace_instance only (batch runs ignore
                                    it): trace the carry-over variant the batch
                                    kernels run instead of the draining one    */
#define PXB_TRACE_IN_FLIGHT_UNKNOWN 0xFFFFFFFFu  /* trace record: copies of a
                                    broadcast not yet on the links (production
                                    variant), so no end-of-step count          */

/* Everything that defines a batch.  Mirrors the hard-coded constants of the
 * reference (N = 2 acceptors Main.hs:41, P = 2 proposers Main.hs:45, majority
 * rule Client.hs:191-194) plus the new fault schedule. */
typedef struct pxb_config {
  uint64_t seed;             /* Philox key                                     */
  uint64_t first_instance;   /* global id of the first instance (sharding)    */
  uint64_t n_instances;      /* instances in this call                        */
  uint32_t n_proposers;      /* P: 1..3   (clientId = p+1, Client.hs:85)      */
  uint32_t n_acceptors;      /* N: 2..9   (length serverPids, Client.hs:193)  */
  uint32_t loss_ppm;         /* per-message loss probability, ppm             */
  uint32_t delay_max;        /* link delay uniform in [1, delay_max], 1..15   */
  uint32_t crash_ppm;        /* per-acceptor isolation-window probability     */
  uint32_t crash_len_max;    /* window length uniform in [1, crash_len_max]   */
  uint32_t crash_start_max;  /* window start uniform in [0, crash_start_max]  */
  uint32_t skew_max;         /* proposer Tick step uniform in [0, skew_max]   */
  uint32_t step_cap;         /* 1..8192                                        */
  uint32_t flags;            /* PXB_CFG_*                                      */
  /* log mode (ABI 2): the reference's ticker sends a Tick every second,
   * forever (Client.hs:96-100).  n_ticks <= 1 = single decree (one Tick per
   * proposer, at its skew step); n_ticks > 1 = proposer p gets Ticks at steps
   * skew_p + j * tick_period, j = 0..n_ticks-1, and the acceptor logs grow one
   * command per committed slot (Server.hs:73-78). */
  uint32_t n_ticks;          /* 0 / 1 = single decree, else 2..PXB_MAX_TICKS   */
  uint32_t tick_period;      /* steps between Ticks (log mode), 1..8192        */
} pxb_config;

/* Per-instance outcome (16 B).  decided_val is the Command of the first
 * `Execute` broadcast (Client.hs:178) encoded (clientId << 24) | t, i.e.
 * "c<clientId>.<t>" (Client.hs:202-203); 0 = none.  flags bits 0..7 are the
 * PXB_F_* bits, bits 16..31 the number of steps the instance ran. */
typedef struct pxb_result {
  uint32_t decided_val;
  int32_t  decided_ticket;   /* Ticket of that Execute (Common.hs:20)          */
  uint32_t rounds;           /* AskForTicket broadcasts, all proposers         */
  uint32_t flags;
} pxb_result;

#define PXB_F_UNDECIDED       (1u << 0)  /* no Execute ever sent               */
#define PXB_F_STUCK           (1u << 1)  /* quiescent, some proposer not Idle  */
#define PXB_F_PANIC           (1u << 2)  /* Server.hs:76 pattern failure (Q6)  */
#define PXB_F_LOG_DIVERGENCE  (1u << 3)  /* two acceptor logs differ           */
#define PXB_F_STEP_CAP        (1u << 4)
#define PXB_F_QUEUE_OVERFLOW  (1u << 5)
#define PXB_F_TICKET_OVERFLOW (1u << 6)
#define PXB_F_LOG_TRUNC       (1u << 7)  /* a log longer than PXB_LOG_TRACK    */
#define PXB_RESULT_STEPS(f)   ((f) >> 16)

/* Final acceptor record (16 B) — ServerState, Server.hs:24-31.
 * meta = log_len | (dead << 31).  val == 0 means `_proposal = Nothing`. */
typedef struct pxb_acceptor_rec {
  int32_t  t_max;            /* _largestIssuedTicket */
  int32_t  t_store;          /* fst of _proposal     */
  uint32_t val;              /* snd of _proposal     */
  uint32_t meta;
} pxb_acceptor_rec;

/* Run totals (SURVEY.md §8(e) slots 0..7, extended). */
#define PXB_NCOUNTERS 16
enum {
  PXB_C_DECIDED = 0, PXB_C_UNDECIDED, PXB_C_STUCK, PXB_C_PANIC,
  PXB_C_DIVERGENCE, PXB_C_STEP_CAP, PXB_C_ROUNDS, PXB_C_MESSAGES,
  PXB_C_QUEUE_OVERFLOW, PXB_C_TICKET_OVERFLOW, PXB_C_LOG_TRUNC,
  PXB_C_CANON_BYTES,         /* SURVEY.md §8(d) canonical accounting v1       */
  PXB_C_STEPS, PXB_C_INSTANCES,
  PXB_C_EXECUTES,            /* Execute broadcasts (commands committed)       */
  PXB_C_RESERVED15
};
typedef struct pxb_counters { int64_t c[PXB_NCOUNTERS]; } pxb_counters;

/* ---- batch entry points ---------------------------------------------------
 * pxb_run: HOST buffers.  Runs cfg->n_instances instances on the current HIP
 * device, copies the outputs back.  out: n_instances results; log_digest:
 * n_instances * n_acceptors FNV-1a digests (instance-major); acc:
 * n_instances * n_acceptors final acceptor records; totals: run totals.  Every
 * output pointer is nullable.  Blocks until done.
 * Replaces: Main.hs:37-53 (spawn servers/clients, run forever) for a batch.   */
int pxb_run(const pxb_config* cfg, pxb_result* out, uint32_t* log_digest,
            pxb_acceptor_rec* acc, pxb_counters* totals);

/* pxb_run_device: DEVICE buffers, asynchronous on `stream` (a hipStream_t;
 * NULL = default stream).  Same outputs as pxb_run but all pointers are device
 * pointers on the current device.  d_totals (PXB_NCOUNTERS int64) is ADDED to,
 * not overwritten, so many launches can accumulate into one vector.  The
 * batch runs in chunks; each chunk enqueues its kernels and a one-block
 * finalize kernel that folds the chunk's partial totals into d_totals:
 *   fault-free, one proposer, single decree: the fault-free per-lane kernel,
 *     then the general faulty kernel over the instances it handed back
 *     (chunks up to 2^30 - 1);
 *   other fault-free (duelling proposers, log mode): the fault-free per-lane
 *     kernel for those, then the general faulty kernel over its bails;
 *   faulty single decree: the per-lane event kernel, then the general faulty
 *     kernel over its bailed instances; loss-free, skew-free batches with
 *     delays <= 4 (BASELINE config 4) take its simple-schedule shape, and
 *     with two proposers over more than 10 links its tight layout first
 *     (12 waves per CU), the simple-schedule shape over what that hands on;
 *     fuzzed three-proposer batches run the two-proposer event kernel first
 *     and the three-proposer one over the instances that drew P = 3 (chunks
 *     of 2^26; 2^25 split);
 *   faulty log mode (n_ticks > 1, delays <= 8): the per-lane event kernel's
 *     log-mode shape, over <= 10 links the same shape on the 16-step wheel
 *     with a larger pool over what it hands on, then the general log-mode
 *     kernel over the rest (chunks of 2^26; longer delays: the general
 *     log-mode kernel).
 * Each chunk
 * uses one of 64 per-device scratch slots round-robin; a chunk that takes a
 * slot makes its stream wait (on the device, hipStreamWaitEvent) for the
 * event recorded behind the slot's previous chunk, so any number of chunks
 * may be in flight across streams (a 65th waits for the first's slot).  A
 * launch failure after a chunk's first kernel zeroes its slot (behind the
 * queued work) before the error is returned.                                 */
int pxb_run_device(const pxb_config* cfg, pxb_result* d_out, uint32_t* d_log_digest,
                   pxb_acceptor_rec* d_acc, int64_t* d_totals, void* stream);

/* pxb_run_multi: HOST buffers, sharded over devices 0..n_devices-1 (<= 0: all
 * visible) by contiguous global-instance ranges, one host thread per device;
 * totals = one RCCL all-reduce (sum) of the per-device run totals over xGMI.
 * Results are identical to pxb_run for any device count (Philox is keyed by
 * the global instance id).  Concurrent calls from several threads run one
 * after another (they share the cached communicators).
 * Replaces: Main.hs:37-53 for a multi-GPU node.                               */
int pxb_run_multi(const pxb_config* cfg, int n_devices, pxb_result* out, uint32_t* log_digest,
                  pxb_acceptor_rec* acc, pxb_counters* totals);

/* ---- context ------------------------------------------------------------------
 * The library keeps per-device scratch (64 launch slots of partial totals and
 * queue words, 2 MB per device; the wire codec's scan buffer) and the RCCL
 * communicators of pxb_run_multi, created lazily on first use.  The per-lane
 * kernels' bailed-id lists are kept per (device, stream) of pxb_run_device,
 * allocated on that stream's first faulty or per-lane launch: 16 MB each, plus
 * 64 MB for the two-stage routings (config 5's split, config 4's tight), for
 * at most 8 streams per device (a ninth stream takes over the oldest entry:
 * its launches wait on the device for an event recorded behind that entry's
 * last launches, failed chunks included; a stream destroyed by the library
 * hands its entry back).  pxb_init(n) creates the launch slots of devices 0..n-1
 * (n <= 0: all visible) up front; pxb_shutdown() waits for those devices, frees everything
 * and destroys the communicators; the next call starts afresh.  Both are
 * optional.  Do not call pxb_shutdown while other threads have calls in
 * flight.  (A CPU pxb_run_cpu is NOT part of this library: the CPU
 * restatement of the schedule is test infrastructure in oracle/ — the checker
 * and the timed baseline — and the GPU entry points never fall back to it.) */
int pxb_init(int n_devices);
int pxb_shutdown(void);

/* pxb_stream_release (ABI 4): `stream` (a hipStream_t used with pxb_run_device on device
 * `dev`; NULL = the default stream) is about to be destroyed or has no more
 * work for the library: its bailed-id lists go back to the library for the
 * next stream, whose launches first wait (on the device, hipStreamWaitEvent)
 * for the event behind their last launches, even while those still run.
 * Optional (without it a ninth stream takes the oldest entry over the same
 * way); pxb_run_multi calls it for the streams it creates.  Unknown streams
 * are ignored.  First use of a stream allocates its lists: a timed loop should
 * make one small untimed launch on every stream it will use (bench.py does).  */
void pxb_stream_release(int dev, void* stream);

/* ---- per-instance trace (the build counterpart of the reference's `say`
 * state dumps, Server.hs:85 and Client.hs:108) ---------------------------------
 * Runs ONE instance of a single-decree batch on the current device through the
 * per-lane state machine of the faulty kernels (csrc/paxos_ev.h) and records
 * the state at the end of every step it visits: steps with no due message and
 * no Tick change nothing and are skipped (their state is the previous
 * record's).  Host buffers; out holds max_records records; *n_records is the
 * count written (the last one is the final step); result (nullable) is the
 * instance's pxb_result, as pxb_run gives it.  By default the trace runs the
 * variant of the state machine in which every step sends all of its copies
 * before the next begins, so every record is the schedule's end-of-step state.
 * The batch kernels run a variant that may carry the copies of a step's last
 * broadcast into the next step; with PXB_CFG_TRACE_PRODUCTION in cfg->flags the
 * trace runs that variant instead: records are taken on entering the next step
 * (acceptor and proposer states are the end-of-step ones; in_flight is
 * PXB_TRACE_IN_FLIGHT_UNKNOWN while copies are still to send, and a carried
 * step may be recorded although nothing else falls due in it).
 * Log mode (n_ticks > 1, ABI 5) runs the batch kernels' log-mode shape: the
 * ticker, Execute-driven logs (the acceptor records' log lengths and digests
 * per step) and commands c<id>.<t> in the proposer fields.
 * PXB_E_INVAL for step_cap > 4095, for log mode with delays above 8, or if the
 * instance outgrows the state machine's link capacities (its FIFOs hold 4
 * messages; the batch kernels then hand it to the general kernel) or
 * max_records.                                                               */
typedef struct pxb_trace_prop {
  int32_t  ticket;           /* _ticket                      Client.hs:60    */
  uint32_t cmd;              /* _mCommand, (id << 24) | t or 0 (t = 1 single decree) */
  uint32_t acks;             /* _numAcks                                     */
  uint32_t state;            /* 0 Idle, 1 Round1, 2 Round2                    */
  int32_t  mr_t;             /* Round1: MostRecent (ticket, command)          */
  uint32_t mr_v;
  uint32_t r2_v;             /* Round2: the proposed command                  */
  uint32_t pending;          /* Round2: _originalCommandPending               */
} pxb_trace_prop;
typedef struct pxb_trace_step {
  uint32_t step;             /* the step that just ended                      */
  uint32_t in_flight;        /* messages queued on the links after it         */
  uint32_t n_acceptors, n_proposers;
  pxb_acceptor_rec acc[PXB_MAX_ACCEPTORS];
  uint32_t log_digest[PXB_MAX_ACCEPTORS];
  pxb_trace_prop prop[PXB_MAX_PROPOSERS];
} pxb_trace_step;
int pxb_trace_instance(const pxb_config* cfg, uint64_t instance, pxb_trace_step* out, uint32_t max_records,
                       uint32_t* n_records, pxb_result* result);

/* ---- single-handler hooks (run the kernel's own device functions) -------- */
/* One message in or out.  Requests (ClientRequest, Common.hs:41-45):
 *   kind 0 AskForTicket t | 1 Propose (t, c) | 2 Execute t ; x = t, z = c.
 * Responses (ServerResponse, Common.hs:49-53):
 *   kind 0 Round1OK g (t_store, val) | 1 HaveTicket u | 2 Round2Success ;
 *   x = g or u, y = t_store, z = val.                                        */
typedef struct pxb_msg { uint32_t kind; int32_t x; int32_t y; uint32_t z; } pxb_msg;
#define PXB_MSG_NONE 0xFFFFFFFFu   /* kind of an absent reply */

/* ClientState, Client.hs:58-67 (+ Round1State/Round2State :36-49). */
typedef struct pxb_proposer_rec {
  int32_t  ticket;
  uint32_t cmd;              /* 0 = Nothing          */
  uint32_t acks;
  uint32_t state;            /* 0 Idle, 1 Round1, 2 Round2 */
  int32_t  mr_t;             /* Round1: MostRecent   */
  uint32_t mr_v;
  int32_t  r2_t;             /* Round2: _proposal    */
  uint32_t r2_v;
  uint32_t pending;          /* Round2: _originalCommandPending */
  uint32_t client_id;
} pxb_proposer_rec;

/* handleClientRequest (Server.hs:51-78) applied to count independent
 * (state, message) pairs on the GPU.  reply[i].kind = PXB_MSG_NONE when the
 * handler tells nothing.  A panic (Server.hs:76) sets bit 31 of meta.  Host
 * pointers.                                                                  */
int pxb_acceptor_handle(pxb_acceptor_rec* states, const pxb_msg* req,
                        pxb_msg* reply, uint32_t count);

/* handleServerResponse / handleTick (Client.hs:125-207) applied to count
 * independent (state, message) pairs on the GPU.  msg kind 3 = Tick.  Each
 * handler broadcasts at most two requests (Client.hs:178,185): bcast[2*i],
 * bcast[2*i+1], with n_bcast[i] of them valid.  Host pointers.               */
int pxb_proposer_handle(pxb_proposer_rec* states, uint32_t n_acceptors,
                        const pxb_msg* msg, pxb_msg* bcast, uint32_t* n_bcast,
                        uint32_t count);

/* ---- wire format ----------------------------------------
 * Batch codec for the Data.Binary payloads the reference sends: the generic
 * `instance Binary ClientRequest` / `instance Binary ServerResponse`
 * (Common.hs:24,47,55; binary-0.8.5.1 from the lts-12.18 resolver): Word8
 * constructor tag, Int = Int64 big-endian, Maybe = Word8 0|1 (+ value),
 * Command = Int length + UTF-8 chars of "c<clientId>.<t>".  Messages use
 * pxb_msg: requests kind 0/1/2 with x = ticket, z = command code
 * ((clientId << 24) | t, Propose only); responses kind 0/1/2 with x = ticket,
 * (y, z) = Round1OK's stored proposal (z == 0: Nothing).  A kind above 2
 * encodes to an empty record.  Offsets are exclusive prefix sums
 * (count + 1 entries): message i occupies bytes [off[i], off[i+1]).
 * Replaces: Cloud Haskell's serialisation of `contentOf m` in sendMessages
 * (Common.hs:36-39) for a batch of messages; the envelope (sender ProcessId,
 * type fingerprint, TCP framing) is not part of it.                        */
#define PXB_WIRE_REQUEST   0u     /* ClientRequest  (Common.hs:41-47)        */
#define PXB_WIRE_RESPONSE  1u     /* ServerResponse (Common.hs:49-55)        */
#define PXB_WIRE_MAX_BYTES 39     /* longest record: Round1OK with a Just    */
/* per-message decode status */
#define PXB_WIRE_OK        0u
#define PXB_WIRE_E_LENGTH  1u     /* truncated record or trailing bytes      */
#define PXB_WIRE_E_TAG     2u     /* constructor / Maybe tag out of range    */
#define PXB_WIRE_E_STRING  3u     /* not a "c<id>.<t>" the reference prints  */
#define PXB_WIRE_E_RANGE   4u     /* Int beyond int32, id > 255, t >= 2^24   */

/* DEVICE buffers, asynchronous on `stream`.  pxb_wire_size writes the
 * offsets of `count` encoded messages (d_offsets: count + 1 entries);
 * pxb_wire_encode takes exactly those offsets (it writes the records of each
 * message tile contiguously from the tile's first offset).  Decode
 * accepts any offsets: a record with off[i+1] < off[i] is empty, and one that
 * reaches past n_bytes (the size of d_bytes) is never read; both are
 * PXB_WIRE_E_LENGTH. */
int pxb_wire_size(const pxb_msg* d_msgs, uint64_t count, uint32_t type, uint64_t* d_offsets, void* stream);
int pxb_wire_encode(const pxb_msg* d_msgs, uint64_t count, uint32_t type, const uint64_t* d_offsets,
                    uint8_t* d_bytes, void* stream);
/* size + encode fused: writes the offsets (count + 1 entries) and the records;
 * d_bytes must hold count * PXB_WIRE_MAX_BYTES bytes (or the encoded total).
 * The size / encode_all calls of one device share a scratch buffer: issue
 * them on one stream. */
int pxb_wire_encode_all(const pxb_msg* d_msgs, uint64_t count, uint32_t type, uint64_t* d_offsets,
                        uint8_t* d_bytes, void* stream);
/* d_status (nullable): PXB_WIRE_* per message; failed messages decode to 0s */
int pxb_wire_decode(const uint8_t* d_bytes, uint64_t n_bytes, const uint64_t* d_offsets, uint64_t count,
                    uint32_t type, pxb_msg* d_msgs, uint32_t* d_status, void* stream);
/* HOST-buffer forms (blocking).  encode: `out` holds count * PXB_WIRE_MAX_BYTES
 * bytes, offsets count + 1 entries, *nbytes = total bytes written. */
int pxb_wire_encode_host(const pxb_msg* msgs, uint64_t count, uint32_t type, uint8_t* out, uint64_t* offsets,
                         uint64_t* nbytes);
int pxb_wire_decode_host(const uint8_t* in, uint64_t n_bytes, const uint64_t* offsets, uint64_t count,
                         uint32_t type, pxb_msg* msgs, uint32_t* status);

/* pxb_handoff_counts: instances the per-lane kernels of device `dev` handed on
 * since the device's scratch was created (pxb_init or its first launch) or
 * last reset: out2[0] = by the first per-lane kernel of a chunk (its bails; for
 * the two-stage routings also what the second per-lane kernel re-runs:
 * config 5's P = 3 instances, or config 4's instances that outgrew the tight
 * layout), out2[1] = by a second per-lane kernel (two-stage routings only).
 * What reaches the general kernel is out2[1] for two-stage chunks, out2[0]
 * otherwise.  A list that overflowed counts cap + 1 more.  Waits for the
 * device; reset != 0 zeroes the counts after reading.  Observability only:
 * results never depend on it.                                                */
int pxb_handoff_counts(int dev, uint64_t* out2, int reset);

/* pxb_reload_hooks (ABI 5): re-reads the library's test / A-B hooks from the
 * environment (PXB_NO_EV, PXB_NO_TIGHT, PXB_EV_BAIL_CAP, PXB_BLOCKS_PER_CU, ...:
 * routing and capacity switches the GPU tests use).  They are read once, on
 * pxb_init or the first launch, and then only by this call: the launch path
 * never calls getenv.  Not for production use; unset, nothing changes.       */
void pxb_reload_hooks(void);

/* ---- misc ----------------------------------------------------------------- */
const char* pxb_strerror(int code);
int         pxb_last_hip_error(void);
int         pxb_abi_version(void);
/* canonical algorithmic bytes for a fault-free P = 1 instance */
uint64_t    pxb_canonical_bytes_nofault(uint32_t n_acceptors);

#ifdef __cplusplus
}
#endif
#endif /* PAXOS_BATCH_H */
