/*
 * dash_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the DASH directory-coherence protocol of
 * /root/reference/assignment.c (vibhav950/UE22CS343BB1-OpenMP-Assignment), run
 * under the deterministic lockstep schedule the GPU engine implements
 * (SURVEY.md App. C). It is the parity checker: only tests/, the smoke()
 * entry and bench.py's cpu_baseline leg may load it. The product path
 * (libdash.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked byte-for-byte against the
 * reference's own golden dumps (tests/golden/reference/..., copied from
 * /root/reference/tests) and, where the reference builds here, against the
 * reference binary itself on schedule-independent traces (oracle/build_ref.sh).
 */
#ifndef DASH_ORACLE_H
#define DASH_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_PROCS 8
#define ORC_MEM_SIZE 16
#define ORC_MAX_CACHE 16
#define ORC_NUM_TXN 13

/* error bits (same values as the product's DASH_ERR_*) */
#define ORC_ERR_OVERFLOW 1u  /* receiver queue full: message dropped (ref :754-761) */
#define ORC_ERR_OOB 2u       /* receiver >= N: message dropped (ref UB :751 via :772,786) */
#define ORC_ERR_CTZ0 4u      /* ctz(0) on an EM entry: message dropped (ref UB :209,451) */
#define ORC_ERR_DEADLOCK 8u  /* quiescent while some node still waits for a reply */
#define ORC_ERR_ROUNDCAP 16u /* stopped at max_rounds */
#define ORC_ERR_STUCK 32u    /* a queue reached capacity: head == tail, never drained again (ref :167-170) */

/* micro-step models (orc_cfg.micro) */
#define ORC_MICRO_BUFFERED 0 /* a thread may pop/issue again while its earlier sends are still
                                buffered (the round-1..3 checker: a superset of the reference) */
#define ORC_MICRO_STRICT 1   /* a thread's sends all complete before its next pop or issue, as
                                sendMessage is synchronous in the reference (:741-765): exactly
                                the race-free reference */
#define ORC_MICRO_RACE 2     /* STRICT plus the reference's unlocked count-- (:177) racing the
                                locked count++ (:757): see orc_reach in dash_oracle.c */

typedef struct orc_cfg {
    int num_procs;       /* N (NUM_PROCS, ref :6) 1..8 */
    int cache_size;      /* CACHE_SIZE (ref :7), 1..16 */
    int ring_depth;      /* queue capacity (ref MSG_BUFFER_SIZE, :9): 256 is the reference and the
                            engine; a queue that reaches it is stuck (ref :167-170). Smaller
                            values model a reference built with a smaller MSG_BUFFER_SIZE, NOT
                            the engine's shallow tiers (the engine re-runs a system that would
                            exceed a tier at the next depth, so it never freezes below 256) */
    uint64_t max_rounds; /* 0 = unlimited; else clamped to 2^31 - 4 and rounded up to a
                            multiple of 4 like the engine's */
    int log_msgs;        /* log also DEBUG_MSG lines (ref :180-181), not only DEBUG_INSTR */
    int micro;           /* micro-step model of the legality checker (ORC_MICRO_*); the lockstep
                            runner ignores it */
    uint64_t arb_seed;   /* 0: deliver in ascending sender order; else the seeded per-round
                            sender order of orc_arb_prio */
    const uint8_t *sched; /* explicit round schedule (twin of dash_set_schedule), or NULL:
                             sched[r * num_procs + t] = 0xFF when node t sits round r out, else
                             its delivery position (distinct among the round's stepping nodes);
                             rounds >= sched_rounds are lockstep rounds. Overrides arb_seed. */
    uint32_t sched_rounds;
    int count_msgs;      /* legality checker: an outcome is (final state, messages handled per
                            type), as the reference's DEBUG_MSG lines (:179-182) count them */
} orc_cfg;

/* Delivery priority of sender t in round r under a seeded arbitration (same spec as
   the kernel): an affine permutation of 0..P-1, P = next power of two >= N. */
uint32_t orc_arb_prio(uint64_t seed, uint64_t round, uint32_t t, uint32_t P);
/* Whether node t sits out round r under a seeded arbitration (probability 1/4; a
   thread of the reference may be descheduled for any time, so every subset of
   nodes stepping in a round is a legal schedule). */
int orc_arb_stall(uint64_t seed, uint64_t round, uint32_t t);

/* Final per-node state, in the reference's own terms (processorNode, ref :89-95). */
typedef struct orc_node_state {
    uint8_t memory[ORC_MEM_SIZE];
    uint8_t dir_bitvector[ORC_MEM_SIZE];
    uint8_t dir_state[ORC_MEM_SIZE];   /* EM=0, S=1, U=2 (ref :28) */
    uint8_t cache_addr[ORC_MAX_CACHE];
    uint8_t cache_value[ORC_MAX_CACHE];
    uint8_t cache_state[ORC_MAX_CACHE]; /* M=0, E=1, S=2, I=3 (ref :17) */
} orc_node_state;

typedef struct orc_result {
    orc_node_state node[ORC_MAX_PROCS];
    uint64_t hist[ORC_NUM_TXN]; /* messages handled, by transactionType (ref :30-44) */
    uint64_t rounds;            /* lockstep rounds until quiescence */
    uint64_t instructions;      /* instructions issued */
    uint32_t errors;            /* ORC_ERR_* bits */
    uint32_t dropped;           /* messages dropped */
    uint32_t max_depth;         /* deepest queue observed after delivery */
    uint32_t _pad;
    uint64_t digest;            /* dash digest of the final state */
} orc_result;

/*
 * Simulate one system. trace = N rows of packed instructions, row stride
 * `stride` (u16 each: bit15 = WR, bits 14..8 = address, bits 7..0 = value).
 * If `log` is non-NULL, every issued instruction is appended as a
 * DEBUG_INSTR line (ref :650-651) while it fits in log_cap bytes.
 * Returns 0, or -1 on a bad config / malformed trace address.
 */
int orc_run_system(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride,
                   const uint32_t *lens, orc_result *out, char *log, uint64_t log_cap);

/* Synthetic generator: identical spec to the device generator. */
typedef struct orc_gen {
    uint64_t seed;
    uint32_t kind;      /* 0 uniform, 1 contention, 2 locality */
    uint32_t locality;  /* P(node == own) in 1/65536 units (kind 2) */
    uint32_t len;       /* instructions per node */
    uint32_t num_procs;
} orc_gen;

uint16_t orc_gen_instr(const orc_gen *g, uint64_t sys, uint32_t node, uint32_t i);
void orc_gen_system(const orc_gen *g, uint64_t sys, uint16_t *trace, uint64_t stride);

/*
 * Batch mode (CPU baseline / large parity sets): systems [sys_first,
 * sys_first+count) generated by `g` and simulated with `threads` OpenMP
 * threads. Per-system digests/rounds/errors are written if the arrays are
 * non-NULL; hist_total accumulates the histogram. Returns wall seconds.
 */
double orc_run_batch(const orc_cfg *cfg, const orc_gen *g, uint64_t sys_first, uint64_t count,
                     int threads, uint64_t *digests, uint32_t *rounds, uint32_t *errors,
                     uint64_t *hist_total, uint64_t *instr_total);

/* Dump text of one node exactly as printProcessorState (ref :853-905). Returns bytes. */
int orc_dump_node(const orc_node_state *s, int node_id, int cache_size, char *buf, int cap);

uint64_t orc_digest_node(const orc_node_state *s, int node_id, int cache_size);

/* ---- legality checker (race-free micro-step model) ---- */
typedef struct orc_outcome {
    orc_node_state node[ORC_MAX_PROCS];
    uint64_t digest;  /* same digest as orc_result.digest (with cfg.count_msgs: folded with hist) */
    uint32_t errors;  /* ORC_ERR_* (DEADLOCK when a node still waits) */
    uint32_t _pad;
    uint32_t hist[ORC_NUM_TXN]; /* cfg.count_msgs: messages handled per type */
    uint32_t _pad2;
} orc_outcome;

/* The lockstep schedule executed as micro-steps (each step checked enabled). */
int orc_replay_lockstep(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                        orc_outcome *out, uint64_t *steps);
/* One uniformly random legal schedule (a random enabled micro-step at a time). */
int orc_random_schedule(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                        uint64_t seed, orc_outcome *out);
/* Exhaustive search (pop-first persistent sets) of terminal outcomes; stops adding
   states at max_states (complete = 0 then). Distinct outcomes by digest. */
int orc_explore(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                uint64_t max_states, orc_outcome *outs, int max_outs, int *n_outs, uint64_t *states,
                int *complete);

/* Goal-directed DFS over the micro-step model cfg->micro (pop-first persistent sets, visited
   hash set, at most race_max RACE steps under ORC_MICRO_RACE): stops at the first terminal
   state whose digest is in targets (*hit = its index, else -1) and writes the witness, one
   step word (kind << 8 | aux << 4 | node; kind 0 POP, 1 ISSUE, 2 SEND, 3 RACE with aux the
   sender whose count++ is lost) per step. prio[t] (lower first) orders the successors;
   order_seed != 0 shuffles them instead. *complete: every reachable state was visited without
   a hit (the targets are unreachable in this model). With found_flags != NULL the search goes
   on until every target is found (found_flags[k] = 1 for each found; *hit = how many; the
   witness is the first hit's). */
int orc_reach(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
              int race_max, const uint64_t *targets, int n_targets, uint64_t max_states,
              const uint8_t *prio, uint64_t order_seed, int *hit, uint16_t *witness, uint32_t wit_cap,
              uint32_t *wit_len, uint64_t *states, int *complete, int *found_flags);
/* One random schedule with per-node and per-kind (POP, ISSUE, SEND, RACE) step weights (NULL:
   uniform), and its witness. */
int orc_random_walk(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                    int race_max, uint64_t seed, const uint32_t *weights, const uint32_t *kind_w,
                    orc_outcome *out, uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len);
/* Re-execute a witness: 0, or -(k+1) if step k is not enabled in the full model. */
int orc_replay_steps(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                     int race_max, const uint16_t *steps, uint32_t n, orc_outcome *out, int *terminal);

/* The engine's schedule (lockstep, cfg->arb_seed or cfg->sched) as a micro-step witness, each
   step checked enabled in the model cfg->micro. 0, -2 (a step not enabled), -3 (cap). */
int orc_schedule_witness(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len, orc_outcome *out);

/* Log-guided replay (STRICT model): an interleaving in which every node pops exactly the
   messages of its reference DEBUG_MSG log, in order, and issues where its DEBUG_INSTR log does.
   events: the nodes' logs concatenated (ev_count[t] words for node t); POP word = type |
   sender << 8 | address << 16, ISSUE word = 1u << 31. *found, the final *out; *complete = the
   search was exhaustive (found 0 and complete 1: no such interleaving exists). */
int orc_guided(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
               const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
               orc_outcome *out, uint64_t *states, int *complete);

/* orc_guided plus the interleaving it found: *wit_len micro-steps (XSTEP: pop / issue / one
   send of node t), the order in which the reference's threads took them; -3 if more than
   wit_cap (the witness is then cut). */
int orc_guided_witness(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                       const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
                       orc_outcome *out, uint64_t *states, uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len);

/* An engine round schedule (dash_set_schedule form, [rounds][num_procs]) under which every node
   pops exactly its logged messages and issues where its log says (events as for orc_guided).
   *found = 0 when the search ends without one (the run is not a round-model execution, or the
   state budget ran out). */
int orc_rounds_from_logs(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         const uint32_t *events, const uint32_t *ev_count, uint64_t max_states,
                         uint8_t *sched, uint32_t sched_cap, uint32_t *n_rounds, int *found, uint64_t *states);

#ifdef __cplusplus
}
#endif
#endif
