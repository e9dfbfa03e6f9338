/*
 * dash.h -- C-ABI of libdash, the MI355X batched DASH directory-coherence
 * simulator (drop-in for the hot path of vibhav950/UE22CS343BB1-OpenMP-Assignment).
 *
 * The reference (assignment.c) simulates ONE system of NUM_PROCS nodes with
 * one OpenMP thread per node. libdash simulates up to millions of independent
 * systems per GPU under the deterministic lockstep schedule,
 * one wave64 lane per node. Plain pointers and sizes only; no torch types.
 *
 * Reference interfaces each entry point replaces (file:line in assignment.c):
 *   dash_parse_core_file   initializeProcessor's trace parse         :822-850
 *   dash_init_node_state   initializeProcessor's state init          :806-821
 *   dash_load_traces/_dir  per-thread traces in processorNode        :89-95, :152
 *   dash_run               the OpenMP parallel region: event loop,
 *                          13-way dispatch, sendMessage,
 *                          handleCacheReplacement, locks/queues      :135-155, :149-738,
 *                                                                    :741-765, :767-804
 *   dash_read_state        the private processorNode after the run   :145, :149
 *   dash_dump_node/_file   printProcessorState                       :853-905
 *   dash_simulate_dir      main() end to end                         :126-739
 *
 * Errors: negative return codes (DASH_E*); nothing exits or throws across the
 * ABI. Per-system protocol faults are reported as DASH_ERR_* bits.
 */
#ifndef DASH_H
#define DASH_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DASH_MEM_SIZE 16   /* MEM_SIZE (ref :8) */
#define DASH_MAX_PROCS 8   /* bitVector is one byte (ref :63) */
#define DASH_MAX_CACHE 16
#define DASH_RING_DEPTH 256 /* per-node queue capacity = ref MSG_BUFFER_SIZE (:9); the engine
                              runs shallower LDS queues first and re-runs, from scratch, any
                              system that would fill one (16 -> 32 -> 256) */
#define DASH_NUM_TIERS 3
#define DASH_NUM_TXN 13    /* transactionType (ref :30-44) */

/* return codes */
#define DASH_OK 0
#define DASH_EINVAL -1   /* bad argument / configuration */
#define DASH_EIO -2      /* trace file missing or unreadable (ref :826-828) */
#define DASH_EPARSE -3   /* a line the reference would turn into garbage */
#define DASH_EADDR -4    /* trace address homed on a node >= num_procs */
#define DASH_EDEVICE -5  /* HIP runtime error (no device, launch failure, ...) */
#define DASH_ENOMEM -6
#define DASH_ESTATE -7   /* call out of order (e.g. read_state before run) */
#define DASH_ETRUNC -8   /* an event log reached its capacity: later events were not kept */

/* per-system protocol fault bits (reference UB made defined) */
#define DASH_ERR_OVERFLOW 1u  /* receiver queue (256) full: dropped (ref :754-761) */
#define DASH_ERR_OOB 2u       /* receiver >= N: dropped (ref :751 via :772,786) */
#define DASH_ERR_CTZ0 4u      /* ctz(0) on an EM entry: dropped (ref :209,451) */
#define DASH_ERR_DEADLOCK 8u  /* quiescent with a node still waiting */
#define DASH_ERR_ROUNDCAP 16u /* stopped at max_rounds */
#define DASH_ERR_STUCK 32u    /* a receiver queue reached MSG_BUFFER_SIZE (256): head == tail, so the
                                 reference never drains it again (:167-170); its messages stay
                                 unhandled and later sends to it drop (:754-761). Modelled exactly. */
#define DASH_ERR_SCHEDULE 64u /* a micro-step schedule stepped a node whose outbox still held sends
                                 (not a reference interleaving: sendMessage is synchronous,
                                 :741-765); the system stops there and its results are void */

/* transactionType ordinals (ref :30-44) */
enum dash_txn {
    DASH_READ_REQUEST, DASH_WRITE_REQUEST, DASH_REPLY_RD, DASH_REPLY_WR, DASH_REPLY_ID,
    DASH_INV, DASH_UPGRADE, DASH_WRITEBACK_INV, DASH_WRITEBACK_INT, DASH_FLUSH,
    DASH_FLUSH_INVACK, DASH_EVICT_SHARED, DASH_EVICT_MODIFIED
};

/* flags */
#define DASH_KEEP_STATE 1u    /* write full final node state (needed by dash_read_state) */
#define DASH_TIER_FROM_32 2u  /* start at queue depth 32 (testing: exercises that kernel) */
#define DASH_TIER_FROM_256 4u /* run every system at depth 256 directly; with no TIER flag
                                 the first depth adapts to the previous run's overflow rate */
#define DASH_TEST_SHORT_ARB 8u /* testing only: the seeded schedule's round table holds 8 rounds,
                                  so later rounds take the in-kernel hashing path */

typedef struct dash_cfg {
    uint32_t num_procs;   /* NUM_PROCS (ref :6): 4 or 8 */
    uint32_t cache_size;  /* CACHE_SIZE (ref :7): 1..16 (powers of two have specialised kernels) */
    uint32_t max_instr;   /* longest trace per node (ref MAX_INSTR_NUM 32, :10) */
    uint32_t flags;       /* DASH_KEEP_STATE */
    uint64_t num_systems; /* independent systems in the batch */
    uint64_t max_rounds;  /* per-system round cap (engine-defined: the reference never exits),
                             clamped to 2^31 - 4, then rounded up to a multiple of 4;
                             0 = 1024 + 256*max_instr */
    int32_t device;       /* HIP device ordinal */
    uint32_t trace_events; /* event log capacity for DEBUG_MSG / DEBUG_INSTR emission
                              (ref :179-182, :649-652), in rounds: every node's events of the
                              first trace_events rounds, rounded up to a multiple of 4 (a node
                              logs at most one event per round, so also at most that many events
                              per node); 0 = no log; < 2^30; device memory num_systems x
                              num_procs x 4 B per kept round */
    uint64_t schedule_seed; /* 0: lowest-sender-first lockstep (the parity schedule); else a
                               seeded legal schedule: per round a node sits out w.p. 1/4 and
                               senders deliver in a seeded order */
} dash_cfg;

/* Final node state in the reference's own terms (processorNode, ref :89-95). */
typedef struct dash_node_state {
    uint8_t memory[DASH_MEM_SIZE];
    uint8_t dir_bitvector[DASH_MEM_SIZE];
    uint8_t dir_state[DASH_MEM_SIZE];     /* EM=0, S=1, U=2 (ref :28) */
    uint8_t cache_addr[DASH_MAX_CACHE];
    uint8_t cache_value[DASH_MAX_CACHE];
    uint8_t cache_state[DASH_MAX_CACHE];  /* MODIFIED=0 .. INVALID=3 (ref :17) */
} dash_node_state;

typedef struct dash_stats {
    uint64_t hist[DASH_NUM_TXN]; /* messages handled per transactionType */
    uint64_t instructions;       /* instructions issued */
    uint64_t rounds_total;       /* sum over systems of lockstep rounds */
    uint64_t rounds_max;
    uint64_t systems;
    uint64_t err_systems;        /* systems with any DASH_ERR_* bit */
    uint64_t err_bits;           /* OR of all DASH_ERR_* bits */
    uint64_t dropped;            /* messages dropped */
    uint64_t max_depth;          /* deepest queue after any delivery */
    double kernel_ms;            /* simulation kernel time (HIP events, engine stream) */
    uint64_t tier_systems[DASH_NUM_TIERS]; /* systems simulated at queue depth 16, 32, 256 */
    uint64_t wave_rounds;        /* lockstep-loop trips summed over wavefronts (all tiers) */
} dash_stats;

/* Synthetic trace generator (counter-based, identical host spec in DESIGN.md §gen). */
#define DASH_GEN_UNIFORM 0u
#define DASH_GEN_CONTENTION 1u /* 90 %: WR to 0x00..0x03 (homed on node 0) */
#define DASH_GEN_LOCALITY 2u   /* node == own w.p. locality/65536, else another node */
typedef struct dash_gen {
    uint64_t seed;
    uint64_t sys_base;  /* global id of this handle's system 0 (multi-GPU sharding) */
    uint32_t kind;
    uint32_t locality;
    uint32_t len;       /* instructions per node (<= cfg.max_instr) */
    uint32_t _reserved;
} dash_gen;

/* One logged step of one node (cfg.trace_events > 0), in lockstep order. */
#define DASH_EV_MSG 0u   /* handled a message: word = message word (type[3:0], sender[6:4],
                            address[14:8], value|bitVector[23:16], secondReceiver[26:24];
                            the other bits are zero; a REPLY_ID's bitVector is the directory's,
                            the receiving requester leaves itself out of the INV fan-out) */
#define DASH_EV_INSTR 1u /* issued an instruction: word = packed instruction */
typedef struct dash_event {
    uint32_t round;
    uint32_t node;
    uint32_t kind;
    uint32_t word;
} dash_event;

typedef struct dash_ctx dash_t;

/* ---- lifecycle / device path (libdash.so, HIP) ---- */
int dash_create(const dash_cfg *cfg, dash_t **out);
void dash_destroy(dash_t *h);
/* the handle's last error message; dash_last_error(NULL) = the message of the last failed
   handle-less call (dash_create, dash_run_host_batched) on the calling thread. The library
   never writes to stderr. */
const char *dash_last_error(const dash_t *h);

/* traces: packed u16 (bit15 = WR, bits 14..8 = address, bits 7..0 = value),
   layout [sys][node][stride]; lens[sys*num_procs + node]. Synchronous: the caller's
   buffer is read (for power-of-two num_procs, by one strided H2D copy) before return;
   words at or past a node's length are never simulated. An RD word's value bits are
   ignored: the reference parses every RD with value 0 (:839) and later fills REPLY_ID /
   REPLY_WR / FLUSH_INVACK lines with the last issued value (:383,470,531), so the library
   clears them on the device after the copy (one pass over the trace buffer). */
int dash_load_traces(dash_t *h, const uint16_t *packed, uint64_t stride, const uint32_t *lens,
                     uint64_t num_systems);
/* Host-buffer throughput path (replaces the same load+run for callers whose traces sit in
   host memory): num_systems (a multiple of batches) go through in `batches` equal batches
   on two handles made from *cfg (num_systems = the batch size), each driven by its own host
   thread and HIP stream, so one batch's H2D copy overlaps another's run. Results equal one
   dash_load_traces + dash_run over all systems: merged *stats (kernel_ms = sum over
   batches), and per-system digests / rounds / errors into the optional arrays. The handles
   are made without DASH_KEEP_STATE and event logs (nothing here returns them); the first
   failing batch stops both threads, and dash_last_error(NULL) then holds its message. */
int dash_run_host_batched(const dash_cfg *cfg, const uint16_t *packed, uint64_t stride,
                          const uint32_t *lens, uint64_t num_systems, uint32_t batches,
                          dash_stats *stats, uint64_t *digests, uint32_t *rounds, uint32_t *errors);
int dash_generate(dash_t *h, const dash_gen *g);
/* An explicit round schedule, replacing the seeded rounds of a handle created with
   schedule_seed != 0 (DASH_ESTATE otherwise): sched[r * num_procs + t] = DASH_SIT_OUT when node
   t sits round r out, else t's delivery position in round r (< next_pow2(num_procs), distinct
   among the round's stepping nodes; DASH_EINVAL otherwise). Rounds >= `rounds` are lockstep
   rounds (every node steps, ascending sender order). Every system of the batch follows it.
   The whole run must fit the handle's round table: cfg.max_rounds (rounded) <= 2^22 and no
   DASH_TEST_SHORT_ARB. Each round is a legal reference execution (the stepping
   threads run their handlers, then complete their sendMessage calls (:741-765) one thread after
   another in delivery order), so a schedule pins one chosen interleaving of the reference, e.g.
   the one behind an accepted racy-test output (tests/golden/schedules/). */
#define DASH_SIT_OUT 0xFFu
int dash_set_schedule(dash_t *h, const uint8_t *sched, uint32_t rounds);
/* A micro-step schedule, the finer-grained twin of dash_set_schedule (same handle requirements):
   acts[r * num_procs + t] = DASH_SIT_OUT, DASH_MICRO_STEP (node t pops or issues, as in a round,
   and its sends wait in its outbox) or DASH_MICRO_SEND (node t delivers its oldest held message);
   at most one node acts per round, and every node sits out past `rounds`. This is the
   reference's own granularity: a thread handles a message, then completes its sendMessage
   calls (:741-765) one by one while other threads run, so any interleaving of the reference's
   threads -- e.g. the one the oracle recovers from a reference run's DEBUG logs -- is one such
   schedule (tests/golden/ref_runs/). A valid schedule never steps a node whose outbox holds
   messages; a system whose schedule does stops at that round with DASH_ERR_SCHEDULE. Runs at
   queue depth 256 only (no tiers); pass max_rounds >= the schedule's rounds:
   a system still active (or holding sends) at the round cap stops with DASH_ERR_ROUNDCAP. */
#define DASH_MICRO_STEP 0u
#define DASH_MICRO_SEND 1u
int dash_set_micro_schedule(dash_t *h, const uint8_t *acts, uint32_t rounds);
int dash_run(dash_t *h, dash_stats *stats);
int dash_read_state(dash_t *h, uint64_t sys, dash_node_state *out /* [num_procs] */);
int dash_read_results(dash_t *h, uint64_t first, uint64_t count, uint64_t *digests,
                      uint32_t *rounds, uint32_t *errors);
int dash_read_hist(dash_t *h, uint64_t sys, uint32_t *hist /* [DASH_NUM_TXN] */);
/* The event log of one system, merged in lockstep order (round, then node): up to
   cap events into out, the total into *n (cap 0 with out NULL: count only). The log keeps
   trace_events rounds rounded up to a multiple of 4 (a node logs at most one event per round);
   DASH_ETRUNC if events fell past them (counted in *n, not kept). */
int dash_read_events(dash_t *h, uint64_t sys, dash_event *out, uint32_t cap, uint32_t *n);
/* HIP stream the engine launches on (hipStream_t as void*) */
void *dash_stream(dash_t *h);

/* Box calibration (not a reference interface: it makes a benchmark line explain the box it ran
   on). The device's identity and clock limits, and one timed launch of a fixed VALU-bound
   probe kernel (CUs x 8 workgroups of 256 threads, eight add/xor chains per lane): its time,
   its rate, and the shader clock the box actually held meanwhile (shader-clock cycles over the
   100-MHz reference counter, read by every workgroup around its loop). A box whose clock or
   issue rate is low shows it here, whatever the simulation kernel did. */
typedef struct dash_box_probe {
    char name[64];
    char arch[32];
    int32_t compute_units;
    int32_t clock_khz;        /* hipDeviceProp_t.clockRate (the maximum shader clock) */
    int32_t mem_clock_khz;    /* hipDeviceProp_t.memoryClockRate */
    int32_t pci_domain, pci_bus, pci_device;
    uint64_t total_mem;
    double probe_ms;          /* the probe launch (HIP events) */
    double probe_valu_per_s;  /* wave64 VALU instructions of the chains per second */
    double probe_sclk_mhz;    /* mean shader clock over the workgroups' loops */
    double probe_sclk_min_mhz, probe_sclk_max_mhz;
} dash_box_probe;
int dash_probe_box(int device, dash_box_probe *out);

/* ---- host boundary (pure C, no device) ---- */
/* initializeProcessor's parse (ref :822-850): up to max_instr records into out[]. */
int dash_parse_core_file(const char *path, uint32_t num_procs, uint32_t max_instr,
                         uint16_t *out, uint32_t *len);
/* Resolve the reference's `tests/<dir>/core_<n>.txt` rule (ref :824); also accepts a
   directory that directly holds core_<n>.txt. Writes the resolved path. */
int dash_resolve_dir(const char *dir, char *resolved, size_t cap);
int dash_load_dir(dash_t *h, const char *dir, uint64_t sys);
/* Bulk ingest: system k = trace directory dirs[k] (same rules as dash_load_dir, ref
   :822-850; parsed on host threads, no "initialized" lines); n == cfg.num_systems. */
int dash_load_dirs(dash_t *h, const char *const *dirs, uint64_t n);
/* Bulk emission: one system's printProcessorState files (ref :853-905) into out_dir
   (created if missing; needs DASH_KEEP_STATE), and a text file with one line
   "system digest(hex) rounds errors(hex)" for every system. */
int dash_dump_system(dash_t *h, uint64_t sys, const char *out_dir);
int dash_write_digests(dash_t *h, const char *path);
void dash_init_node_state(dash_node_state *s, uint32_t node_id, uint32_t cache_size);
/* printProcessorState byte-exact (ref :853-905). Returns bytes written, or < 0. */
int dash_dump_node(const dash_node_state *s, uint32_t node_id, uint32_t cache_size, char *buf,
                   size_t cap);
int dash_dump_file(const dash_node_state *s, uint32_t node_id, uint32_t cache_size,
                   const char *path);
uint64_t dash_digest_node(const dash_node_state *s, uint32_t node_id, uint32_t cache_size);
/* One event as the reference prints it: DEBUG_MSG "Processor %d msg from: %d, type: %d,
   address: 0x%02X" (ref :180-181) or DEBUG_INSTR "Processor %d: instr type=%c,
   address=0x%02X, value=%hhu" (ref :650-651), newline included. Returns bytes or < 0. */
int dash_format_event(const dash_event *e, char *buf, size_t cap);
/* main() end to end for one system: parse dir, run on the GPU, write
   core_<n>_output.txt into out_dir (ref :126-739, :860). */
int dash_simulate_dir(const char *dir, uint32_t num_procs, uint32_t cache_size,
                      uint32_t max_instr, const char *out_dir, int device, dash_stats *stats);

#ifdef __cplusplus
}
#endif
#endif
