/*
 * dash_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker, never shipped).
 *
 * Sequential restatement of /root/reference/assignment.c's per-node event
 * loop (:149-738), sendMessage (:741-765) and handleCacheReplacement
 * (:767-804), driven by the deterministic lockstep schedule of SURVEY.md
 * App. C:
 *   - every round, each node takes ONE step on start-of-round state: pop and
 *     handle one message if its queue is non-empty (ref :167-619), else issue
 *     one instruction if it is not waiting and has instructions left
 *     (ref :624-735), else idle;
 *   - messages sent during the round are appended to the receivers' queues at
 *     the end of the round, ascending sender id, program order within a sender;
 *   - the system is quiescent when every queue is empty and no node can issue.
 * Defined behaviour where the reference is undefined (SURVEY.md App. B 5,8,9):
 * a send to a node >= N, ctz(0) and queue overflow drop the message and raise
 * an error bit.
 *
 * The code mirrors the reference's control structure handler by handler (no
 * packing, no predication) so it can be read side by side with
 * assignment.c; the GPU kernel is a different, predicated formulation.
 */
#include "dash_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* cacheLineState (ref :17), directoryEntryState (ref :28), transactionType (ref :30-44) */
enum { MODIFIED, EXCLUSIVE, SHARED, INVALID };
enum { EM, S, U };
enum {
    READ_REQUEST, WRITE_REQUEST, REPLY_RD, REPLY_WR, REPLY_ID, INV, UPGRADE,
    WRITEBACK_INV, WRITEBACK_INT, FLUSH, FLUSH_INVACK, EVICT_SHARED, EVICT_MODIFIED
};

/* Mutation testing of the reference pin (tests/test_reference_cross_node.py): ORC_MUTANT = k
   builds oracle/_mut/libdash_oracle_m<k>.so with one plausible misreading of a cross-node
   handler (listed in tests/ref_pin.py MUTANTS). The shipped checker is ORC_MUTANT 0. */
#ifndef ORC_MUTANT
#define ORC_MUTANT 0
#endif

#define MAX_RING 256
#define MAX_OUT (ORC_MAX_PROCS + 4)

typedef struct {
    uint8_t type, sender, address, value, bitVector, secondReceiver, dirState;
} omsg; /* message (ref :70-79) */

typedef struct {
    uint8_t address, value, state;
} oline; /* cacheLine (ref :56-60) */

typedef struct {
    oline cache[ORC_MAX_CACHE];
    uint8_t memory[ORC_MEM_SIZE];
    uint8_t bitVector[ORC_MEM_SIZE];
    uint8_t dirState[ORC_MEM_SIZE];
    const uint16_t *trace;
    uint32_t count; /* instructionCount */
    uint32_t idx;   /* next instruction to issue */
    int waiting;    /* waitingForReply (ref :162) */
    uint8_t instr_type, instr_address, instr_value; /* `instr` (ref :159), last issued */
    /* incoming queue (messageBuffer, ref :81-87) */
    omsg q[MAX_RING];
    uint32_t head, qcount;
    /* this round's sends, in program order */
    int nout;
    int out_to[MAX_OUT];
    omsg out[MAX_OUT];
} onode;

typedef struct {
    int N, CS, ring, log_msgs;
    onode node[ORC_MAX_PROCS];
    orc_result *res;
    char *log;
    uint64_t log_len, log_cap;
} osys;

/* sendMessage (ref :741-765), deferred to the end of the round */
static void send_message(onode *nd, int receiver, omsg m) {
    nd->out_to[nd->nout] = receiver;
    nd->out[nd->nout] = m;
    nd->nout++;
}

/* handleCacheReplacement (ref :767-804) */
static void handle_cache_replacement(onode *nd, int sender, oline old) {
    int home = (old.address >> 4) & 0x0F;
    omsg m = {0};
    switch (old.state) {
    case EXCLUSIVE:
    case SHARED:
        m.type = EVICT_SHARED;
        m.sender = (uint8_t)sender;
        m.address = old.address;
        send_message(nd, home, m);
        break;
    case MODIFIED:
        m.type = EVICT_MODIFIED;
        m.sender = (uint8_t)sender;
        m.address = old.address;
        m.value = old.value;
        send_message(nd, home, m);
        break;
    default: /* INVALID: no action (ref :800-802) */
        break;
    }
}

static int ctz8(uint8_t v) { return __builtin_ctz((unsigned)v); }

/* One message through the 13-way dispatch (ref :186-618). */
static void handle_message(osys *sy, int tid, omsg msg) {
    onode *nd = &sy->node[tid];
    const int CS = sy->CS;
    uint8_t procNodeAddr = (msg.address >> 4) & 0x0F; /* ref :186-188 */
    uint8_t memBlockAddr = msg.address & 0x0F;
    uint8_t cacheIndex = memBlockAddr % CS;
    oline *L = &nd->cache[cacheIndex];
    omsg r = {0};

    sy->res->hist[msg.type]++;
    if (sy->log && sy->log_msgs && sy->log_len + 64 < sy->log_cap) /* DEBUG_MSG (ref :180-181) */
        sy->log_len += (uint64_t)snprintf(sy->log + sy->log_len, sy->log_cap - sy->log_len,
                                          "Processor %d msg from: %d, type: %d, address: 0x%02X\n", tid,
                                          msg.sender, msg.type, msg.address);
    switch (msg.type) {
    case READ_REQUEST: /* ref :191-237 */
        if (nd->dirState[memBlockAddr] == EM) {
            if (nd->bitVector[memBlockAddr] == 0) { sy->res->errors |= ORC_ERR_CTZ0; sy->res->dropped++; break; }
            r.type = WRITEBACK_INT;
            r.sender = (uint8_t)tid;
            r.address = msg.address;
            r.secondReceiver = msg.sender;
            send_message(nd, ctz8(nd->bitVector[memBlockAddr]), r);
        } else if (nd->dirState[memBlockAddr] == S) {
            r.type = REPLY_RD;
            r.sender = (uint8_t)tid;
            r.address = msg.address;
            r.value = nd->memory[memBlockAddr];
            r.dirState = S;
            send_message(nd, msg.sender, r);
            if (ORC_MUTANT != 8) nd->bitVector[memBlockAddr] |= (uint8_t)(1u << msg.sender);
        } else { /* U */
            r.type = REPLY_RD;
            r.sender = (uint8_t)tid;
            r.address = msg.address;
            r.value = nd->memory[memBlockAddr];
            r.dirState = EM;
            send_message(nd, msg.sender, r);
            nd->dirState[memBlockAddr] = EM;
            nd->bitVector[memBlockAddr] = (uint8_t)(1u << msg.sender);
        }
        break;

    case REPLY_RD: /* ref :239-255 */
        if (L->address != msg.address && L->state != INVALID)
            handle_cache_replacement(nd, tid, *L);
        L->address = msg.address;
        L->value = msg.value;
        L->state = (msg.dirState == S) ? SHARED : EXCLUSIVE;
        nd->waiting = 0;
        break;

    case WRITEBACK_INT: /* ref :257-286; reads/changes cache[idx] with no address check */
        r.type = FLUSH;
        r.sender = (uint8_t)tid;
        r.address = msg.address;
        r.value = L->value;
        r.secondReceiver = msg.secondReceiver;
        send_message(nd, procNodeAddr, r);
        if (procNodeAddr != msg.secondReceiver)
            send_message(nd, msg.secondReceiver, r);
        if (ORC_MUTANT != 1 || L->address == msg.address)
            L->state = SHARED;
        break;

    case FLUSH: /* ref :288-323 */
        if (tid == procNodeAddr) {
            nd->dirState[memBlockAddr] = S;
            nd->bitVector[memBlockAddr] |= (uint8_t)(1u << msg.secondReceiver);
            nd->memory[memBlockAddr] = msg.value;
        }
        if (tid == msg.secondReceiver) {
            if (L->address != msg.address && L->state != INVALID)
                handle_cache_replacement(nd, tid, *L);
            L->address = msg.address;
            L->value = msg.value;
            L->state = SHARED;
        }
        if (ORC_MUTANT != 2 || tid == msg.secondReceiver)
            nd->waiting = 0; /* unconditional (App. B 2) */
        break;

    case UPGRADE: { /* ref :325-349; no directory-state check */
        uint8_t others = nd->bitVector[memBlockAddr] & (uint8_t)~(1u << msg.sender);
        r.type = REPLY_ID;
        r.sender = (uint8_t)tid;
        r.address = msg.address;
        r.bitVector = ORC_MUTANT == 3 ? nd->bitVector[memBlockAddr] : others;
        send_message(nd, msg.sender, r);
        nd->dirState[memBlockAddr] = EM;
        nd->bitVector[memBlockAddr] = (uint8_t)(1u << msg.sender);
        break;
    }

    case REPLY_ID: /* ref :351-387; fills with the last issued instr.value */
        for (int i = 0; i < sy->N; i++) {
            if (msg.bitVector & (1u << i)) {
                omsg inv = {0};
                inv.type = INV;
                inv.sender = (uint8_t)tid;
                inv.address = msg.address;
                send_message(nd, i, inv);
            }
        }
        if (L->address != msg.address && L->state != INVALID)
            handle_cache_replacement(nd, tid, *L);
        L->address = msg.address;
        L->value = nd->instr_value;
        L->state = MODIFIED;
        nd->waiting = 0;
        break;

    case INV: /* ref :389-399; state not checked */
        if (L->address == msg.address && (ORC_MUTANT != 11 || L->state == SHARED))
            L->state = INVALID;
        break;

    case WRITE_REQUEST: /* ref :401-459 */
        if (nd->dirState[memBlockAddr] == U) {
            r.type = REPLY_WR;
            r.sender = (uint8_t)tid;
            r.address = msg.address;
            send_message(nd, msg.sender, r);
        } else if (nd->dirState[memBlockAddr] == S) {
            r.type = REPLY_ID;
            r.sender = (uint8_t)tid;
            r.address = msg.address;
            r.bitVector = nd->bitVector[memBlockAddr] & (uint8_t)~(1u << msg.sender);
            send_message(nd, msg.sender, r);
        } else { /* EM */
            if (nd->bitVector[memBlockAddr] == 0) {
                sy->res->errors |= ORC_ERR_CTZ0;
                sy->res->dropped++;
            } else {
                r.type = WRITEBACK_INV;
                r.sender = (uint8_t)tid;
                r.address = msg.address;
                r.value = msg.value;
                r.secondReceiver = msg.sender;
                send_message(nd, ctz8(nd->bitVector[memBlockAddr]), r);
            }
        }
        if (ORC_MUTANT == 9 && nd->dirState[memBlockAddr] == S) break;
        nd->dirState[memBlockAddr] = EM; /* ref :456-457, every branch */
        nd->bitVector[memBlockAddr] = (uint8_t)(1u << msg.sender);
        break;

    case REPLY_WR: /* ref :461-474; replacement is unconditional (App. B 6) */
        if (ORC_MUTANT != 10 || L->address != msg.address)
            handle_cache_replacement(nd, tid, *L);
        L->address = msg.address;
        L->value = nd->instr_value;
        L->state = MODIFIED;
        nd->waiting = 0;
        break;

    case WRITEBACK_INV: /* ref :476-503; FLUSH_INVACK twice when home == requester */
        r.type = FLUSH_INVACK;
        r.sender = (uint8_t)tid;
        r.address = msg.address;
        r.value = L->value;
        r.secondReceiver = msg.secondReceiver;
        send_message(nd, procNodeAddr, r);
        if (ORC_MUTANT != 4 || procNodeAddr != msg.secondReceiver)
            send_message(nd, msg.secondReceiver, r);
        L->state = INVALID;
        break;

    case FLUSH_INVACK: /* ref :505-536 */
        if (tid == procNodeAddr) {
            nd->bitVector[memBlockAddr] = (uint8_t)(1u << msg.secondReceiver);
            nd->memory[memBlockAddr] = msg.value;
        }
        if (tid == msg.secondReceiver) {
            if (L->address != msg.address && L->state != INVALID)
                handle_cache_replacement(nd, tid, *L);
            L->address = msg.address;
            L->value = ORC_MUTANT == 5 ? msg.value : nd->instr_value;
            L->state = MODIFIED;
        }
        nd->waiting = 0;
        break;

    case EVICT_SHARED: /* ref :538-590 */
        if (tid != procNodeAddr) {
            if (ORC_MUTANT != 7 || L->address == msg.address)
                L->state = EXCLUSIVE; /* no address check (App. B 5) */
        } else {
            nd->bitVector[memBlockAddr] &= (uint8_t)~(1u << msg.sender);
            int numSharers = __builtin_popcount(nd->bitVector[memBlockAddr]);
            if (numSharers == 0) {
                nd->dirState[memBlockAddr] = U;
            } else if (numSharers == 1) {
                nd->dirState[memBlockAddr] = EM;
                int newOwner = ctz8(nd->bitVector[memBlockAddr]);
                if (newOwner != procNodeAddr) {
                    r.type = EVICT_SHARED;
                    r.sender = (uint8_t)tid;
                    r.address = msg.address;
                    r.value = nd->memory[memBlockAddr];
                    send_message(nd, newOwner, r);
                } else if (ORC_MUTANT != 6) {
                    L->state = EXCLUSIVE;
                }
            }
        }
        break;

    case EVICT_MODIFIED: /* ref :592-617 */
        if (ORC_MUTANT == 12 && nd->bitVector[memBlockAddr] != (uint8_t)(1u << msg.sender)) break;
        nd->memory[memBlockAddr] = msg.value;
        nd->bitVector[memBlockAddr] = 0;
        nd->dirState[memBlockAddr] = U;
        break;
    }
}

/* Issue one instruction (ref :647-735). */
static void issue_instruction(osys *sy, int tid) {
    onode *nd = &sy->node[tid];
    uint16_t w = nd->trace[nd->idx++];
    uint8_t type = (w & 0x8000) ? 'W' : 'R';
    uint8_t address = (uint8_t)((w >> 8) & 0x7F);
    /* initializeProcessor parses every RD with value 0 (ref :839), whatever the packed word's
       bits 7..0 hold; the value is used later by REPLY_ID/REPLY_WR/FLUSH_INVACK (:383,470,531) */
    uint8_t value = type == 'W' ? (uint8_t)(w & 0xFF) : 0;
    nd->instr_type = type;
    nd->instr_address = address;
    nd->instr_value = value;
    sy->res->instructions++;

    if (sy->log && sy->log_len + 64 < sy->log_cap) /* DEBUG_INSTR (ref :650-651) */
        sy->log_len += (uint64_t)snprintf(sy->log + sy->log_len, sy->log_cap - sy->log_len,
                                          "Processor %d: instr type=%c, address=0x%02X, value=%hhu\n",
                                          tid, type, address, value);

    uint8_t procNodeAddr = (address >> 4) & 0x0F;
    uint8_t memBlockAddr = address & 0x0F;
    uint8_t cacheIndex = memBlockAddr % sy->CS;
    oline *L = &nd->cache[cacheIndex];
    int hit = L->address == address ? (L->state == INVALID ? 0 : 1) : 0; /* ref :662-664 */
    omsg m = {0};
    if (type == 'R') {
        if (!hit) {
            m.type = READ_REQUEST;
            m.sender = (uint8_t)tid;
            m.address = address;
            send_message(nd, procNodeAddr, m);
            nd->waiting = 1;
        }
    } else {
        if (hit) {
            if (L->state == MODIFIED || L->state == EXCLUSIVE) {
                L->value = value;
                if (ORC_MUTANT != 13 || L->state == MODIFIED) L->state = MODIFIED;
            } else {
                m.type = UPGRADE;
                m.sender = (uint8_t)tid;
                m.address = address;
                m.value = value;
                send_message(nd, procNodeAddr, m);
                nd->waiting = 1;
            }
        } else {
            m.type = WRITE_REQUEST;
            m.sender = (uint8_t)tid;
            m.address = address;
            m.value = value;
            send_message(nd, procNodeAddr, m);
            nd->waiting = 1;
        }
    }
}

/* initializeProcessor's state part (ref :806-821) */
static void init_node(onode *nd, int tid, int CS) {
    for (int i = 0; i < ORC_MEM_SIZE; i++) {
        nd->memory[i] = (uint8_t)(20 * tid + i);
        nd->bitVector[i] = 0;
        nd->dirState[i] = U;
    }
    for (int i = 0; i < CS; i++) {
        nd->cache[i].address = 0xFF;
        nd->cache[i].value = 0;
        nd->cache[i].state = INVALID;
    }
    nd->head = nd->qcount = 0;
    nd->nout = 0;
    nd->waiting = 0;
}

static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

int orc_arb_stall(uint64_t seed, uint64_t round, uint32_t t) {
    const uint64_t key = fmix64(seed ^ (round * 0x9E3779B97F4A7C15ULL) ^ 0xD1B54A32D192ED03ULL);
    return (int)((key >> (8 * t)) & 3u) == 0;
}

uint32_t orc_arb_prio(uint64_t seed, uint64_t round, uint32_t t, uint32_t P) {
    const uint64_t key = fmix64(seed ^ (round * 0x9E3779B97F4A7C15ULL));
    const uint32_t A = ((uint32_t)key & (P - 1)) | 1u, B = (uint32_t)(key >> 8) & (P - 1);
    return (t * A + B) & (P - 1);
}

uint64_t orc_digest_node(const orc_node_state *s, int node_id, int cache_size) {
    uint64_t h = 0x243F6A8885A308D3ULL ^ ((uint64_t)node_id << 56);
    for (int b = 0; b < ORC_MEM_SIZE; b++)
        h = fmix64(h ^ ((uint64_t)s->memory[b] | ((uint64_t)s->dir_bitvector[b] << 8) |
                        ((uint64_t)s->dir_state[b] << 16)));
    for (int i = 0; i < cache_size; i++)
        h = fmix64(h ^ ((uint64_t)s->cache_addr[i] | ((uint64_t)s->cache_value[i] << 8) |
                        ((uint64_t)s->cache_state[i] << 16) | (1ULL << 24)));
    return h;
}

/* the engine's round cap: clamped to 2^31 - 4 first, then rounded up to a multiple of 4
   (dash_create does the same) */
static uint64_t round_cap(uint64_t max_rounds) {
    return ((max_rounds < 0x7FFFFFFCULL ? max_rounds : 0x7FFFFFFCULL) + 3) & ~3ULL;
}

int orc_run_system(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride,
                   const uint32_t *lens, orc_result *out, char *log, uint64_t log_cap) {
    const int N = cfg->num_procs, CS = cfg->cache_size;
    if (N < 1 || N > ORC_MAX_PROCS || CS < 1 || CS > ORC_MAX_CACHE ||
        cfg->ring_depth < 1 || cfg->ring_depth > MAX_RING)
        return -1;
    for (int t = 0; t < N; t++)
        for (uint32_t i = 0; i < lens[t]; i++)
            if (((trace[t * stride + i] >> 12) & 0x7) >= (unsigned)N) return -1;

    osys *sy = (osys *)calloc(1, sizeof(osys));
    if (!sy) return -1;
    memset(out, 0, sizeof(*out));
    sy->N = N;
    sy->CS = CS;
    sy->ring = cfg->ring_depth;
    sy->log_msgs = cfg->log_msgs;
    sy->res = out;
    sy->log = log;
    sy->log_cap = log ? log_cap : 0;
    if (log && log_cap) log[0] = 0;
    for (int t = 0; t < N; t++) {
        init_node(&sy->node[t], t, CS);
        sy->node[t].trace = trace + t * stride;
        sy->node[t].count = lens[t];
    }

    for (;;) {
        int active = 0;
        for (int t = 0; t < N; t++) {
            onode *nd = &sy->node[t];
            /* a full queue (qcount == capacity) has head == tail: the reference's drain loop
               (ref :167-170) never pops it again */
            if ((nd->qcount > 0 && nd->qcount < (uint32_t)sy->ring) || (!nd->waiting && nd->idx < nd->count))
                active = 1;
        }
        if (!active) break;
        /* the engine's round cap (not the reference's: it never exits) is a multiple of 4 */
        if (cfg->max_rounds && out->rounds >= round_cap(cfg->max_rounds)) {
            out->errors |= ORC_ERR_ROUNDCAP;
            break;
        }
        out->rounds++;

        /* every node steps on start-of-round state (unless a seeded arbitration stalls it) */
        for (int t = 0; t < N; t++) {
            onode *nd = &sy->node[t];
            nd->nout = 0;
            if (cfg->sched) {
                if (out->rounds - 1 < cfg->sched_rounds && cfg->sched[(out->rounds - 1) * (uint64_t)N + t] == 0xFF)
                    continue;
            } else if (cfg->arb_seed && orc_arb_stall(cfg->arb_seed, out->rounds - 1, (uint32_t)t)) {
                continue;
            }
            if (nd->qcount > 0 && nd->qcount < (uint32_t)sy->ring) {
                omsg m = nd->q[nd->head];
                nd->head = (nd->head + 1) % (uint32_t)sy->ring;
                nd->qcount--;
                handle_message(sy, t, m);
            } else if (!nd->waiting && nd->idx < nd->count) {
                issue_instruction(sy, t);
            }
        }
        /* end-of-round delivery: ascending sender (or the seeded sender order), program
           order within a sender (sendMessage ref :741-765) */
        int order[ORC_MAX_PROCS];
        for (int s = 0; s < N; s++) order[s] = s;
        if (cfg->sched) {
            if (out->rounds - 1 < cfg->sched_rounds) {
                const uint8_t *row = cfg->sched + (out->rounds - 1) * (uint64_t)N;
                int k = 0;
                for (int pos = 0; pos < ORC_MAX_PROCS; pos++)
                    for (int s = 0; s < N; s++)
                        if (row[s] == pos) order[k++] = s;
                for (int s = 0; s < N; s++) /* sitting-out nodes send nothing; keep them listed */
                    if (row[s] == 0xFF || row[s] >= ORC_MAX_PROCS) order[k++] = s;
            }
        } else if (cfg->arb_seed) {
            uint32_t P = 1;
            while (P < (uint32_t)N) P <<= 1;
            int k = 0;
            for (uint32_t pr = 0; pr < P; pr++)
                for (int s = 0; s < N; s++)
                    if (orc_arb_prio(cfg->arb_seed, out->rounds - 1, (uint32_t)s, P) == pr) order[k++] = s;
        }
        for (int si = 0; si < N; si++) {
            const int s = order[si];
            onode *src = &sy->node[s];
            for (int k = 0; k < src->nout; k++) {
                int rcv = src->out_to[k];
                if (rcv < 0 || rcv >= N) {
                    out->errors |= ORC_ERR_OOB;
                    out->dropped++;
                    continue;
                }
                onode *dst = &sy->node[rcv];
                if (dst->qcount < (uint32_t)sy->ring) {
                    dst->q[(dst->head + dst->qcount) % (uint32_t)sy->ring] = src->out[k];
                    if (++dst->qcount == (uint32_t)sy->ring) out->errors |= ORC_ERR_STUCK;
                } else {
                    out->errors |= ORC_ERR_OVERFLOW;
                    out->dropped++;
                }
            }
        }
        for (int t = 0; t < N; t++)
            if (sy->node[t].qcount > out->max_depth) out->max_depth = sy->node[t].qcount;
    }

    uint64_t d = 0x9E3779B97F4A7C15ULL;
    for (int t = 0; t < N; t++) {
        onode *nd = &sy->node[t];
        if (nd->waiting && !(out->errors & ORC_ERR_ROUNDCAP)) out->errors |= ORC_ERR_DEADLOCK;
        orc_node_state *st = &out->node[t];
        for (int b = 0; b < ORC_MEM_SIZE; b++) {
            st->memory[b] = nd->memory[b];
            st->dir_bitvector[b] = nd->bitVector[b];
            st->dir_state[b] = nd->dirState[b];
        }
        for (int i = 0; i < CS; i++) {
            st->cache_addr[i] = nd->cache[i].address;
            st->cache_value[i] = nd->cache[i].value;
            st->cache_state[i] = nd->cache[i].state;
        }
        d = fmix64(d ^ orc_digest_node(st, t, CS));
    }
    out->digest = d;
    free(sy);
    return 0;
}

/* ---- synthetic traces (spec shared with the device generator) ---- */

uint16_t orc_gen_instr(const orc_gen *g, uint64_t sys, uint32_t node, uint32_t i) {
    const uint64_t N = g->num_procs;
    uint64_t key = fmix64(g->seed ^ (sys * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL));
    uint64_t r = fmix64(key ^ (((uint64_t)node << 32) | i) ^ 0x8CB92BA72F3D8DD7ULL);
    uint32_t value = (uint32_t)(r & 0xFF);
    uint32_t blk = (uint32_t)((r >> 8) & 0xF);
    uint32_t is_w = (uint32_t)((r >> 12) & 1);
    uint32_t c16 = (uint32_t)((r >> 16) & 0xFFFF);
    uint64_t u32 = r >> 32;
    uint32_t nd = (uint32_t)((u32 * N) >> 32);
    if (g->kind == 1) {
        if (c16 < 58982u) { /* 90 %: WR to one of 0x00..0x03 (homed on node 0) */
            is_w = 1;
            nd = 0;
            blk &= 3;
        }
    } else if (g->kind == 2) {
        if (c16 < g->locality || N == 1)
            nd = node;
        else
            nd = (uint32_t)((node + 1 + ((u32 * (N - 1)) >> 32)) % N);
    }
    if (!is_w) value = 0; /* RD carries value 0 (ref :839) */
    return (uint16_t)((is_w << 15) | (((nd << 4) | blk) << 8) | value);
}

void orc_gen_system(const orc_gen *g, uint64_t sys, uint16_t *trace, uint64_t stride) {
    for (uint32_t t = 0; t < g->num_procs; t++)
        for (uint32_t i = 0; i < g->len; i++)
            trace[t * stride + i] = orc_gen_instr(g, sys, t, i);
}

double orc_run_batch(const orc_cfg *cfg, const orc_gen *g, uint64_t sys_first, uint64_t count,
                     int threads, uint64_t *digests, uint32_t *rounds, uint32_t *errors,
                     uint64_t *hist_total, uint64_t *instr_total) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint64_t hist[ORC_NUM_TXN] = {0};
    uint64_t instr = 0;
    int nthr = threads > 0 ? threads : 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthr)
#endif
    {
        uint16_t *tr = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)g->num_procs * (g->len ? g->len : 1));
        uint32_t lens[ORC_MAX_PROCS];
        for (int t = 0; t < ORC_MAX_PROCS; t++) lens[t] = g->len;
        orc_result *res = (orc_result *)malloc(sizeof(orc_result));
        uint64_t lh[ORC_NUM_TXN] = {0};
        uint64_t li = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = 0; k < (int64_t)count; k++) {
            uint64_t sys = sys_first + (uint64_t)k;
            orc_gen_system(g, sys, tr, g->len);
            orc_run_system(cfg, tr, g->len, lens, res, NULL, 0);
            if (digests) digests[k] = res->digest;
            if (rounds) rounds[k] = (uint32_t)res->rounds;
            if (errors) errors[k] = res->errors;
            for (int j = 0; j < ORC_NUM_TXN; j++) lh[j] += res->hist[j];
            li += res->instructions;
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            for (int j = 0; j < ORC_NUM_TXN; j++) hist[j] += lh[j];
            instr += li;
        }
        free(res);
        free(tr);
    }
    (void)nthr;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (hist_total)
        for (int j = 0; j < ORC_NUM_TXN; j++) hist_total[j] += hist[j];
    if (instr_total) *instr_total += instr;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- printProcessorState (ref :853-905), binary digits hand-formatted (no %B) ---- */

int orc_dump_node(const orc_node_state *s, int id, int cache_size, char *buf, int cap) {
    static const char *cst[] = {"MODIFIED", "EXCLUSIVE", "SHARED", "INVALID"};
    static const char *dst[] = {"EM", "S", "U"};
    int n = 0;
#define P(...) n += snprintf(buf + n, (size_t)(cap > n ? cap - n : 0), __VA_ARGS__)
    P("=======================================\n");
    P(" Processor Node: %d\n", id);
    P("=======================================\n\n");
    P("-------- Memory State --------\n");
    P("| Index | Address |   Value  |\n");
    P("|----------------------------|\n");
    for (int i = 0; i < ORC_MEM_SIZE; i++)
        P("|  %3d  |  0x%02X   |  %5d   |\n", i, (id << 4) + i, s->memory[i]);
    P("------------------------------\n\n");
    P("------------ Directory State ---------------\n");
    P("| Index | Address | State |    BitVector   |\n");
    P("|------------------------------------------|\n");
    for (int i = 0; i < ORC_MEM_SIZE; i++) {
        char bits[9];
        for (int k = 0; k < 8; k++) bits[k] = (char)('0' + ((s->dir_bitvector[i] >> (7 - k)) & 1));
        bits[8] = 0;
        P("|  %3d  |  0x%02X   |  %2s   |   0x%s   |\n", i, (id << 4) + i,
          dst[s->dir_state[i] % 3], bits);
    }
    P("--------------------------------------------\n\n");
    P("------------ Cache State ----------------\n");
    P("| Index | Address | Value |    State    |\n");
    P("|---------------------------------------|\n");
    for (int i = 0; i < cache_size; i++)
        P("|  %3d  |  0x%02X   |  %3d  |  %8s \t|\n", i, s->cache_addr[i], s->cache_value[i],
          cst[s->cache_state[i] & 3]);
    P("----------------------------------------\n\n");
#undef P
    return n;
}

/* ==== legality checker: the race-free micro-step model ====
 *
 * A reference thread's observable behaviour is a sequence of operations on the
 * shared queues (:102): pops from its own queue (:167-177) and appends to other
 * queues (sendMessage :741-765); everything else touches thread-private state
 * (private(node), :149). The micro-step model has one step kind per such
 * operation, with each thread's sends buffered in an outbox (FIFO) between the
 * handler that produced them and the append -- any gap is a legal delay of the
 * sending thread:
 *   POP(t)    pop t's queue head and run the handler (local effects, sends -> outbox)
 *   ISSUE(t)  t's queue is empty, t is not waiting, instructions remain (:624-647):
 *             issue one instruction (local effects, sends -> outbox)
 *   SEND(t)   append the head of t's outbox to its receiver's queue
 * Every total order of enabled steps is a legal execution of the reference
 * with race-free queues (App. B 12: the unlocked count-- race is the
 * reference's bug, not part of its semantics). Terminal: no step enabled.
 *
 * Exhaustive search uses the persistent set {POP(t)} for the lowest t with a
 * non-empty queue: a pop commutes with every other thread's steps (appends go to
 * the tail of a non-empty queue) and with t's own SEND (outbox FIFO), and no
 * other step of t is enabled while t's queue is non-empty, so terminal states
 * are preserved. */

#define XQ 40 /* explorer per-node queue / outbox capacity */

typedef struct {
    oline cache[ORC_MAX_CACHE];
    uint8_t memory[ORC_MEM_SIZE], bitVector[ORC_MEM_SIZE], dirState[ORC_MEM_SIZE];
    uint16_t idx;
    uint8_t waiting, instr_value, qn, on, _pad[2];
    omsg q[XQ];        /* incoming queue, head first */
    omsg o[XQ];        /* outbox, head first */
    uint8_t oto[XQ];   /* outbox receivers */
} xnode;

typedef struct {
    xnode n[ORC_MAX_PROCS];
    uint32_t errors;
    int8_t deficit[ORC_MAX_PROCS]; /* ORC_MICRO_RACE: appends whose count++ was lost (:757 vs :177) */
    uint8_t races, _pad[3];
    uint16_t hist[ORC_NUM_TXN + 1]; /* cfg->count_msgs: messages handled per type so far */
    uint16_t npop[ORC_MAX_PROCS];   /* guided search: messages each node has popped */
} xsys;

typedef struct {
    int N, CS, micro, race_max, count_msgs, guided;
    const uint16_t *trace[ORC_MAX_PROCS];
    uint32_t count[ORC_MAX_PROCS];
    osys *scratch; /* the oracle's handlers run on a scratch node */
    orc_result scratch_res;
} xctx;
static void x_init(xctx *c, xsys *s) {
    memset(s, 0, sizeof *s);
    for (int t = 0; t < c->N; t++) {
        onode tmp;
        init_node(&tmp, t, c->CS);
        xnode *x = &s->n[t];
        memcpy(x->cache, tmp.cache, sizeof x->cache);
        memcpy(x->memory, tmp.memory, sizeof x->memory);
        memcpy(x->bitVector, tmp.bitVector, sizeof x->bitVector);
        memcpy(x->dirState, tmp.dirState, sizeof x->dirState);
    }
}

/* run one POP (msg != NULL) or ISSUE step of node t through the oracle's handlers */
static void x_step(xctx *c, xsys *s, int t, const omsg *msg) {
    xnode *x = &s->n[t];
    onode *nd = &c->scratch->node[t];
    memcpy(nd->cache, x->cache, sizeof x->cache);
    memcpy(nd->memory, x->memory, sizeof x->memory);
    memcpy(nd->bitVector, x->bitVector, sizeof x->bitVector);
    memcpy(nd->dirState, x->dirState, sizeof x->dirState);
    nd->trace = c->trace[t];
    nd->count = c->count[t];
    nd->idx = x->idx;
    nd->waiting = x->waiting;
    nd->instr_value = x->instr_value;
    nd->nout = 0;
    c->scratch->res = &c->scratch_res;
    c->scratch_res.errors = 0;
    if (msg)
        handle_message(c->scratch, t, *msg);
    else
        issue_instruction(c->scratch, t);
    s->errors |= c->scratch_res.errors;
    memcpy(x->cache, nd->cache, sizeof x->cache);
    memcpy(x->memory, nd->memory, sizeof x->memory);
    memcpy(x->bitVector, nd->bitVector, sizeof x->bitVector);
    memcpy(x->dirState, nd->dirState, sizeof x->dirState);
    x->idx = (uint16_t)nd->idx;
    x->waiting = (uint8_t)nd->waiting;
    x->instr_value = nd->instr_value;
    for (int k = 0; k < nd->nout; k++) {
        if (x->on >= XQ) { s->errors |= ORC_ERR_OVERFLOW; continue; }
        x->o[x->on] = nd->out[k];
        x->oto[x->on] = (uint8_t)nd->out_to[k];
        x->on++;
    }
}

static void x_pop(xctx *c, xsys *s, int t) {
    xnode *x = &s->n[t];
    omsg m = x->q[0];
    if (c->count_msgs && m.type < ORC_NUM_TXN) s->hist[m.type]++;
    if (c->guided) s->npop[t]++;
    memmove(&x->q[0], &x->q[1], sizeof(omsg) * (size_t)(x->qn - 1));
    x->qn--;
    memset(&x->q[x->qn], 0, sizeof(omsg));
    x_step(c, s, t, &m);
}

static void x_send(xctx *c, xsys *s, int t) {
    xnode *x = &s->n[t];
    omsg m = x->o[0];
    int rcv = x->oto[0];
    memmove(&x->o[0], &x->o[1], sizeof(omsg) * (size_t)(x->on - 1));
    memmove(&x->oto[0], &x->oto[1], (size_t)(x->on - 1));
    x->on--;
    memset(&x->o[x->on], 0, sizeof(omsg));
    x->oto[x->on] = 0;
    if (rcv < 0 || rcv >= c->N) { s->errors |= ORC_ERR_OOB; return; }
    xnode *d = &s->n[rcv];
    if (d->qn >= XQ) { s->errors |= ORC_ERR_OVERFLOW; return; }
    d->q[d->qn++] = m;
}

/* The visible queue count: the reference's `count` (:168) lags the true queue length by the
   appends whose count++ (:757) a racing count-- (:177) overwrote (ORC_MICRO_RACE only). */
static int x_vis(const xctx *c, const xsys *s, int t) {
    return (int)s->n[t].qn - (c->micro == ORC_MICRO_RACE ? s->deficit[t] : 0);
}

/* POP(t): the drain loop's test `count > 0 && head != tail` (:167-170); STRICT / RACE: t's
   earlier sends are done (sendMessage returns before the loop tests again). */
static int x_can_pop(const xctx *c, const xsys *s, int t) {
    return x_vis(c, s, t) > 0 && (c->micro == ORC_MICRO_BUFFERED || s->n[t].on == 0);
}

/* ISSUE(t): the drain loop found nothing, not waiting, instructions left (:624-647). */
static int x_can_issue(const xctx *c, const xsys *s, int t) {
    const xnode *x = &s->n[t];
    return x_vis(c, s, t) <= 0 && (c->micro == ORC_MICRO_BUFFERED || x->on == 0) && !x->waiting &&
           x->idx < c->count[t];
}

/* micro-steps, encoded kind << 8 | aux << 4 | node */
enum { XK_POP, XK_ISSUE, XK_SEND, XK_RACE };
#define XSTEP(k, aux, t) ((uint16_t)((k) << 8 | (aux) << 4 | (t)))

/* Every enabled step, in node order (POP, ISSUE, SEND, then RACE). RACE(x -> t): t's pop and
   x's append to t overlap so that t's unlocked count-- (:177) overwrites x's count++ (:757);
   the message is in the queue but not counted, so t may find its queue "empty" (issue, or stop
   draining) with it inside, until a later append is counted (one message stranded, or dropped
   for good at the end). */
static int x_enabled(const xctx *c, const xsys *s, uint16_t *st) {
    int n = 0;
    for (int t = 0; t < c->N; t++) {
        if (x_can_pop(c, s, t)) st[n++] = XSTEP(XK_POP, 0, t);
        if (x_can_issue(c, s, t)) st[n++] = XSTEP(XK_ISSUE, 0, t);
        if (s->n[t].on > 0) st[n++] = XSTEP(XK_SEND, 0, t);
    }
    if (c->micro == ORC_MICRO_RACE && s->races < c->race_max)
        for (int t = 0; t < c->N; t++) {
            if (s->n[t].on == 0) continue;
            const int r = s->n[t].oto[0];
            if (r != t && r < c->N && x_can_pop(c, s, r) && s->n[r].qn < XQ) st[n++] = XSTEP(XK_RACE, t, r);
        }
    return n;
}

/* The persistent set the exhaustive search expands: {POP(t)} for the lowest t that can pop (a
   pop commutes with every other thread's step and no other step of t is enabled beside it),
   else every enabled step. While races are left the pop is not independent of a RACE on the
   same queue, so everything is expanded. */
static int x_succ(const xctx *c, const xsys *s, uint16_t *st) {
    if (c->micro != ORC_MICRO_RACE || s->races >= c->race_max)
        for (int t = 0; t < c->N; t++)
            if (x_can_pop(c, s, t)) {
                st[0] = XSTEP(XK_POP, 0, t);
                return 1;
            }
    return x_enabled(c, s, st);
}

static void x_apply(xctx *c, xsys *s, uint16_t step) {
    const int t = step & 15, aux = (step >> 4) & 15;
    switch (step >> 8) {
    case XK_POP: x_pop(c, s, t); break;
    case XK_ISSUE: x_step(c, s, t, NULL); break;
    case XK_SEND: x_send(c, s, t); break;
    default: /* XK_RACE: t pops while aux's append to t loses its count++ */
        x_pop(c, s, t);
        x_send(c, s, aux);
        s->deficit[t]++;
        s->races++;
        break;
    }
}

/* Hash of the meaningful bytes of a state (unused queue slots excluded). */
static uint64_t x_hash(const xctx *c, const xsys *s) {
    uint64_t h = 0x243F6A8885A308D3ULL;
#define XH(ptr, len)                                                                           \
    do {                                                                                       \
        const uint8_t *p_ = (const uint8_t *)(ptr);                                            \
        size_t l_ = (len);                                                                     \
        while (l_ >= 8) { uint64_t w_; memcpy(&w_, p_, 8); h = (h ^ w_) * 0x9E3779B97F4A7C15ULL; h ^= h >> 29; p_ += 8; l_ -= 8; } \
        uint64_t w_ = 0; memcpy(&w_, p_, l_); h = (h ^ w_ ^ ((uint64_t)l_ << 56)) * 0xff51afd7ed558ccdULL; h ^= h >> 32; \
    } while (0)
    for (int t = 0; t < c->N; t++) {
        const xnode *x = &s->n[t];
        XH(x, offsetof(xnode, q));
        XH(x->q, sizeof(omsg) * x->qn);
        XH(x->o, sizeof(omsg) * x->on);
        XH(x->oto, x->on);
    }
    XH(&s->errors, sizeof(uint32_t) + ORC_MAX_PROCS + 1);
    if (c->count_msgs) XH(s->hist, sizeof s->hist);
    if (c->guided) XH(s->npop, sizeof s->npop);
#undef XH
    return fmix64(h);
}

static void x_outcome(const xctx *c, const xsys *s, orc_outcome *o) {
    memset(o, 0, sizeof *o);
    uint64_t d = 0x9E3779B97F4A7C15ULL;
    for (int t = 0; t < c->N; t++) {
        const xnode *x = &s->n[t];
        orc_node_state *st = &o->node[t];
        memcpy(st->memory, x->memory, ORC_MEM_SIZE);
        memcpy(st->dir_bitvector, x->bitVector, ORC_MEM_SIZE);
        memcpy(st->dir_state, x->dirState, ORC_MEM_SIZE);
        for (int i = 0; i < c->CS; i++) {
            st->cache_addr[i] = x->cache[i].address;
            st->cache_value[i] = x->cache[i].value;
            st->cache_state[i] = x->cache[i].state;
        }
        if (x->waiting) o->errors |= ORC_ERR_DEADLOCK;
        d = fmix64(d ^ orc_digest_node(st, t, c->CS));
    }
    o->errors |= s->errors;
    if (c->count_msgs) { /* the outcome is (final state, messages handled per type) */
        uint64_t hk = 0x452821E638D01377ULL;
        for (int k = 0; k < ORC_NUM_TXN; k++) {
            o->hist[k] = s->hist[k];
            hk = fmix64(hk ^ ((uint64_t)k << 32 | s->hist[k]));
        }
        d = fmix64(d ^ hk);
    }
    o->digest = d;
}

static int x_setup(xctx *c, const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                   int race_max) {
    memset(c, 0, sizeof *c);
    c->N = cfg->num_procs;
    c->CS = cfg->cache_size;
    c->micro = cfg->micro;
    c->count_msgs = cfg->count_msgs;
    c->race_max = c->micro == ORC_MICRO_RACE ? race_max : 0;
    if (c->N < 1 || c->N > ORC_MAX_PROCS || c->CS < 1 || c->CS > ORC_MAX_CACHE) return -1;
    if (c->micro < ORC_MICRO_BUFFERED || c->micro > ORC_MICRO_RACE || race_max < 0 || race_max > 100) return -1;
    for (int t = 0; t < c->N; t++) {
        c->trace[t] = trace + (uint64_t)t * stride;
        c->count[t] = lens[t];
        if (lens[t] > 0xFFFF) return -1;
        for (uint32_t i = 0; i < lens[t]; i++)
            if (((c->trace[t][i] >> 12) & 0x7) >= (unsigned)c->N) return -1;
    }
    c->scratch = (osys *)calloc(1, sizeof(osys));
    if (!c->scratch) return -1;
    c->scratch->N = c->N;
    c->scratch->CS = c->CS;
    c->scratch->ring = MAX_RING;
    return 0;
}

int orc_replay_lockstep(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                        orc_outcome *out, uint64_t *steps) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, 0)) return -1;
    xsys *s = (xsys *)malloc(sizeof(xsys));
    x_init(&c, s);
    uint64_t n = 0;
    int rc = 0;
    for (;;) {
        /* a lockstep round as micro-steps: every node's POP or ISSUE on start-of-round
           queues (no SEND has run yet), then every outbox drained in sender order */
        int any = 0;
        int popq[ORC_MAX_PROCS];
        for (int t = 0; t < c.N; t++) popq[t] = s->n[t].qn > 0;
        for (int t = 0; t < c.N; t++) {
            if (popq[t]) {
                if (s->n[t].qn == 0) { rc = -2; break; } /* not enabled: cannot happen */
                x_pop(&c, s, t);
                any = 1;
                n++;
            } else if (x_can_issue(&c, s, t)) {
                x_step(&c, s, t, NULL);
                any = 1;
                n++;
            }
        }
        for (int t = 0; t < c.N; t++)
            while (s->n[t].on > 0) { x_send(&c, s, t); n++; }
        if (!any || rc) break;
    }
    x_outcome(&c, s, out);
    if (steps) *steps = n;
    free(s);
    free(c.scratch);
    return rc;
}

static uint64_t x_rng(uint64_t *st) {
    *st += 0x9E3779B97F4A7C15ULL;
    return fmix64(*st);
}

int orc_random_schedule(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                        uint64_t seed, orc_outcome *out) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, 0)) return -1;
    xsys *s = (xsys *)malloc(sizeof(xsys));
    x_init(&c, s);
    uint64_t st = seed;
    uint16_t en[4 * ORC_MAX_PROCS];
    for (;;) {
        const int ne = x_enabled(&c, s, en);
        if (ne == 0) break;
        x_apply(&c, s, en[x_rng(&st) % (uint64_t)ne]);
    }
    x_outcome(&c, s, out);
    free(s);
    free(c.scratch);
    return 0;
}

typedef struct {
    uint64_t *keys;
    uint64_t cap, n;
} xset;

static int xset_insert(xset *v, uint64_t h) { /* 1 if newly inserted */
    if (h == 0) h = 1;
    uint64_t i = h & (v->cap - 1);
    while (v->keys[i]) {
        if (v->keys[i] == h) return 0;
        i = (i + 1) & (v->cap - 1);
    }
    v->keys[i] = h;
    v->n++;
    return 1;
}

int orc_explore(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                uint64_t max_states, orc_outcome *outs, int max_outs, int *n_outs, uint64_t *states,
                int *complete) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, 0)) return -1;
    xset vis;
    vis.cap = 1;
    while (vis.cap < 2 * max_states + 2) vis.cap <<= 1;
    vis.keys = (uint64_t *)calloc(vis.cap, sizeof(uint64_t));
    vis.n = 0;
    size_t scap = 1024, sn = 0;
    xsys *stack = (xsys *)malloc(sizeof(xsys) * scap);
    if (!vis.keys || !stack) { free(vis.keys); free(stack); free(c.scratch); return -1; }
    int nout = 0, full = 1;
    x_init(&c, &stack[sn++]);
    xset_insert(&vis, x_hash(&c, &stack[0]));
    xsys cur, nxt;
    while (sn > 0) {
        cur = stack[--sn];
        uint16_t succ[4 * ORC_MAX_PROCS];
        const int ns = x_succ(&c, &cur, succ);
        if (ns == 0) { /* terminal: record the outcome if new */
            orc_outcome o;
            x_outcome(&c, &cur, &o);
            int seen = 0;
            for (int k = 0; k < nout && k < max_outs; k++)
                if (outs[k].digest == o.digest) seen = 1;
            if (!seen) {
                if (nout < max_outs) outs[nout] = o;
                nout++;
            }
            continue;
        }
        for (int k = 0; k < ns; k++) {
            nxt = cur;
            x_apply(&c, &nxt, succ[k]);
            if (vis.n >= max_states) { full = 0; continue; }
            if (!xset_insert(&vis, x_hash(&c, &nxt))) continue;
            if (sn == scap) {
                scap *= 2;
                xsys *ns2 = (xsys *)realloc(stack, sizeof(xsys) * scap);
                if (!ns2) { full = 0; break; }
                stack = ns2;
            }
            stack[sn++] = nxt;
        }
    }
    if (n_outs) *n_outs = nout;
    if (states) *states = vis.n;
    if (complete) *complete = full;
    free(vis.keys);
    free(stack);
    free(c.scratch);
    return 0;
}

/* ==== goal-directed reachability (classify test_4 run_3 / run_4) ====
 *
 * orc_reach is a depth-first search over the micro-step model (cfg->micro; up to race_max
 * RACE steps under ORC_MICRO_RACE) with a visited-state hash set and the pop-first persistent
 * sets of x_succ. It stops at the first terminal state whose digest is one of `targets` and
 * returns the path to it (the witness: one XSTEP word per step), which orc_replay_steps
 * re-executes step by step, checking that each step is enabled in the full (unreduced) model.
 * Successors are tried in a node-priority order (`prio[t]`, lower first; a DFS that prefers
 * some threads delays the others as long as it can, which is how the racy tests' unusual
 * outcomes arise), SEND before POP before ISSUE within a node; `order_seed` != 0 shuffles
 * them instead. */

static void x_order(const xctx *c, uint16_t *st, int n, const uint8_t *prio, uint64_t *rng) {
    if (rng) {
        for (int i = n - 1; i > 0; i--) {
            const int j = (int)(x_rng(rng) % (uint64_t)(i + 1));
            const uint16_t tmp = st[i]; st[i] = st[j]; st[j] = tmp;
        }
        return;
    }
    static const int kind_rank[4] = {1, 2, 0, 3}; /* SEND, POP, ISSUE, RACE */
    for (int i = 1; i < n; i++) { /* insertion sort, preferred first */
        const uint16_t v = st[i];
        const int kv = (prio ? prio[v & 15] : 0) * 8 + kind_rank[v >> 8];
        int j = i - 1;
        while (j >= 0 && (prio ? prio[st[j] & 15] : 0) * 8 + kind_rank[st[j] >> 8] > kv) { st[j + 1] = st[j]; j--; }
        st[j + 1] = v;
    }
    (void)c;
}

typedef struct {
    xsys s;
    uint32_t depth;
    uint16_t step;
} xent;

int orc_reach(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
              int race_max, const uint64_t *targets, int n_targets, uint64_t max_states,
              const uint8_t *prio, uint64_t order_seed, int *hit, uint16_t *witness, uint32_t wit_cap,
              uint32_t *wit_len, uint64_t *states, int *complete, int *found_flags) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, race_max)) return -1;
    int n_found = 0;
    xset vis;
    vis.cap = 1;
    while (vis.cap < max_states + max_states / 2 + 2) vis.cap <<= 1;
    vis.keys = (uint64_t *)calloc(vis.cap, sizeof(uint64_t));
    vis.n = 0;
    size_t scap = 4096, sn = 0, pcap = 4096;
    xent *stack = (xent *)malloc(sizeof(xent) * scap);
    uint16_t *path = (uint16_t *)malloc(sizeof(uint16_t) * pcap);
    int rc = 0, full = 1, found = -1;
    uint32_t found_len = 0;
    uint64_t rng = order_seed, *prng = order_seed ? &rng : NULL;
    if (!vis.keys || !stack || !path) { rc = -1; goto done; }
    x_init(&c, &stack[0].s);
    if (found_flags)
        for (int k = 0; k < n_targets; k++) found_flags[k] = 0;
    stack[0].depth = 0;
    stack[0].step = 0xFFFF;
    sn = 1;
    xset_insert(&vis, x_hash(&c, &stack[0].s));
    while (sn > 0 && found < 0) {
        xent *e = &stack[--sn];
        const uint32_t d = e->depth;
        if (e->step != 0xFFFF) { /* path[0..d-1] leads to this entry's parent; d >= 1 */
            if (d > pcap) {
                pcap *= 2;
                uint16_t *np = (uint16_t *)realloc(path, sizeof(uint16_t) * pcap);
                if (!np) { rc = -1; break; }
                path = np;
            }
            path[d - 1] = e->step;
        }
        xsys cur = e->s;
        uint16_t succ[4 * ORC_MAX_PROCS];
        const int ns = x_succ(&c, &cur, succ);
        if (ns == 0) {
            orc_outcome o;
            x_outcome(&c, &cur, &o);
            for (int k = 0; k < n_targets; k++)
                if (targets[k] == o.digest) {
                    if (!found_flags) { found = k; found_len = d; break; }
                    if (!found_flags[k]) { /* multi-target: the first witness is kept */
                        found_flags[k] = 1;
                        if (n_found++ == 0 && witness && d <= wit_cap) {
                            memcpy(witness, path, sizeof(uint16_t) * d);
                            found_len = d;
                        }
                        if (n_found == n_targets) found = k;
                    }
                }
            continue;
        }
        x_order(&c, succ, ns, prio, prng);
        for (int k = ns - 1; k >= 0; k--) { /* pushed last = tried first */
            xsys nxt = cur;
            x_apply(&c, &nxt, succ[k]);
            if (vis.n >= max_states) { full = 0; continue; }
            if (!xset_insert(&vis, x_hash(&c, &nxt))) continue;
            if (sn == scap) {
                scap *= 2;
                xent *ns2 = (xent *)realloc(stack, sizeof(xent) * scap);
                if (!ns2) { full = 0; rc = -1; break; }
                stack = ns2;
            }
            stack[sn].s = nxt;
            stack[sn].depth = d + 1;
            stack[sn].step = succ[k];
            sn++;
        }
        if (rc) break;
    }
    if (found >= 0 && witness && !found_flags) {
        if (found_len > wit_cap) rc = -2;
        else memcpy(witness, path, sizeof(uint16_t) * found_len);
    }
done:
    if (hit) *hit = found_flags ? n_found : found;
    if (wit_len) *wit_len = (found >= 0 || n_found) ? found_len : 0;
    if (states) *states = vis.n;
    if (complete) *complete = found < 0 && full && rc == 0;
    free(vis.keys);
    free(stack);
    free(path);
    free(c.scratch);
    return rc;
}

/* One random schedule drawn with per-node weights and per-kind weights (POP, ISSUE, SEND, RACE;
   either NULL: 1), with its witness. A step's weight is its acting node's weight (the popping
   node's for a RACE) times its kind's: a large SEND weight models the reference, whose threads
   append their messages right after the handler that made them (:741-765). */
int orc_random_walk(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                    int race_max, uint64_t seed, const uint32_t *weights, const uint32_t *kind_w,
                    orc_outcome *out, uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, race_max)) return -1;
    xsys *s = (xsys *)malloc(sizeof(xsys));
    if (!s) { free(c.scratch); return -1; }
    x_init(&c, s);
    uint64_t st = seed;
    uint16_t en[4 * ORC_MAX_PROCS];
    uint32_t n = 0;
    int rc = 0;
    for (;;) {
        const int ne = x_enabled(&c, s, en);
        if (ne == 0) break;
        int k;
        if (weights || kind_w) {
            uint64_t wt[4 * ORC_MAX_PROCS], tot = 0;
            for (int i = 0; i < ne; i++) {
                wt[i] = (uint64_t)(weights ? weights[en[i] & 15] : 1u) * (kind_w ? kind_w[en[i] >> 8] : 1u);
                tot += wt[i];
            }
            if (tot == 0) { k = (int)(x_rng(&st) % (uint64_t)ne); }
            else {
                uint64_t r = x_rng(&st) % tot;
                for (k = 0; k < ne - 1; k++) {
                    if (r < wt[k]) break;
                    r -= wt[k];
                }
            }
        } else {
            k = (int)(x_rng(&st) % (uint64_t)ne);
        }
        if (witness) {
            if (n < wit_cap) witness[n] = en[k];
            else rc = -2;
        }
        n++;
        x_apply(&c, s, en[k]);
    }
    x_outcome(&c, s, out);
    if (wit_len) *wit_len = n;
    free(s);
    free(c.scratch);
    return rc;
}

/* Re-execute a witness. Returns 0, or -(k+1) when step k is not enabled in the full model;
   *terminal says whether no step is enabled at the end. */
int orc_replay_steps(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                     int race_max, const uint16_t *steps, uint32_t n, orc_outcome *out, int *terminal) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, race_max)) return -1;
    xsys *s = (xsys *)malloc(sizeof(xsys));
    if (!s) { free(c.scratch); return -1; }
    x_init(&c, s);
    uint16_t en[4 * ORC_MAX_PROCS];
    int rc = 0;
    for (uint32_t k = 0; k < n; k++) {
        const int ne = x_enabled(&c, s, en);
        int ok = 0;
        for (int i = 0; i < ne; i++)
            if (en[i] == steps[k]) ok = 1;
        if (!ok) { rc = -(int)(k + 1); break; }
        x_apply(&c, s, steps[k]);
    }
    if (terminal) *terminal = x_enabled(&c, s, en) == 0;
    x_outcome(&c, s, out);
    free(s);
    free(c.scratch);
    return rc;
}

/* The engine's schedule (lockstep, seeded, or the explicit cfg->sched of dash_set_schedule) as
   a micro-step witness: each round, every stepping node's POP or ISSUE on start-of-round
   queues in node order, then every outbox drained in the round's delivery order. Each step is
   checked enabled in the model cfg->micro (STRICT: these are real reference executions: the
   stepping threads run their local parts, then complete their sends one thread after
   another). Returns 0, -2 if a step was not enabled, -3 if the witness does not fit. */
int orc_schedule_witness(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len, orc_outcome *out) {
    xctx c;
    if (x_setup(&c, cfg, trace, stride, lens, 0)) return -1;
    xsys *s = (xsys *)malloc(sizeof(xsys));
    if (!s) { free(c.scratch); return -1; }
    x_init(&c, s);
    uint32_t n = 0;
    int rc = 0;
    uint32_t P = 1;
    while (P < (uint32_t)c.N) P <<= 1;
    uint16_t en[4 * ORC_MAX_PROCS];
    for (uint64_t r = 0; rc == 0; r++) {
        uint16_t round_steps[2 * ORC_MAX_PROCS];
        int nr = 0;
        int stall[ORC_MAX_PROCS] = {0}, order[ORC_MAX_PROCS];
        for (int t = 0; t < c.N; t++) order[t] = t;
        if (cfg->sched) {
            if (r < cfg->sched_rounds) {
                const uint8_t *row = cfg->sched + r * (uint64_t)c.N;
                int k = 0;
                for (int pos = 0; pos < ORC_MAX_PROCS; pos++)
                    for (int t = 0; t < c.N; t++)
                        if (row[t] == pos) order[k++] = t;
                for (int t = 0; t < c.N; t++)
                    if (row[t] == 0xFF || row[t] >= ORC_MAX_PROCS) { stall[t] = 1; order[k++] = t; }
            }
        } else if (cfg->arb_seed) {
            int k = 0;
            for (uint32_t pr = 0; pr < P; pr++)
                for (int t = 0; t < c.N; t++)
                    if (orc_arb_prio(cfg->arb_seed, r, (uint32_t)t, P) == pr) order[k++] = t;
            for (int t = 0; t < c.N; t++) stall[t] = orc_arb_stall(cfg->arb_seed, r, (uint32_t)t);
        }
        int any = 0, can_any = 0;
        for (int t = 0; t < c.N; t++) {
            if (s->n[t].qn > 0 || x_can_issue(&c, s, t)) can_any = 1;
            if (stall[t]) continue;
            if (s->n[t].qn > 0) round_steps[nr++] = XSTEP(XK_POP, 0, t);
            else if (x_can_issue(&c, s, t)) round_steps[nr++] = XSTEP(XK_ISSUE, 0, t);
        }
        if (!can_any) break; /* quiescent */
        for (int k = 0; k < nr && rc == 0; k++) {
            const int ne = x_enabled(&c, s, en);
            int ok = 0;
            for (int i = 0; i < ne; i++) ok |= en[i] == round_steps[k];
            if (!ok) { rc = -2; break; }
            if (n < wit_cap) witness[n] = round_steps[k]; else rc = -3;
            n++;
            x_apply(&c, s, round_steps[k]);
            any = 1;
        }
        for (int k = 0; k < c.N && rc == 0; k++)
            while (s->n[order[k]].on > 0) {
                if (n < wit_cap) witness[n] = XSTEP(XK_SEND, 0, order[k]); else { rc = -3; break; }
                n++;
                x_apply(&c, s, XSTEP(XK_SEND, 0, order[k]));
            }
        if (r > 100000000ULL) { rc = -2; break; }
        (void)any;
    }
    if (wit_len) *wit_len = n;
    x_outcome(&c, s, out);
    free(s);
    free(c.scratch);
    return rc;
}

/* ==== log-guided replay: the reference's own per-thread event logs (round 4) ====
 *
 * Built with -DDEBUG_MSG -DDEBUG_INSTR, the reference prints every message a thread pops
 * ("Processor t msg from: s, type: k, address: a", :179-182) and every instruction it issues
 * (:649-652), each thread's lines in its program order. orc_guided searches the STRICT
 * micro-step model for an interleaving in which every node pops exactly the messages its log
 * lists, in that order, and issues when its log says so (a node's local state, and so its
 * final state, is then fixed by its log: the handlers are deterministic). Sends are free, so
 * the search decides only when each append happens; a state in which a node's queue head is
 * not the message its log pops next (or a node whose log issues next, or has ended, holds a
 * message) can never recover and is cut. *found = 1 with the final outcome when such an
 * interleaving exists; *complete = 1 when the search was exhaustive (found = 0 then means the
 * model cannot produce the reference's run at all -- how the mutants are refuted).
 * Event words: POP = type | sender << 8 | address << 16; ISSUE = 1 << 31. */
typedef struct {
    const uint32_t *ev[ORC_MAX_PROCS];
    uint32_t n[ORC_MAX_PROCS];
} xguide;

static int g_cursor(const xsys *s, int t) { return (int)s->n[t].idx + (int)s->npop[t]; }

/* A node pops while its queue is non-empty and its queue is FIFO, so every queued message must
 * be the node's next logged pops, in order, with no logged issue among them (the whole queue,
 * not only its head: a wrong message behind the head can never leave without a mismatch). */
static int g_dead(const xctx *c, const xguide *g, const xsys *s) {
    for (int t = 0; t < c->N; t++) {
        const xnode *x = &s->n[t];
        const int k = g_cursor(s, t);
        if ((uint64_t)k + x->qn > g->n[t]) return 1;
        for (int i = 0; i < (int)x->qn; i++) {
            const uint32_t e = g->ev[t][k + i];
            const omsg *h = &x->q[i];
            if ((e >> 31) || (e & 0xFF) != h->type || ((e >> 8) & 0xFF) != h->sender ||
                ((e >> 16) & 0xFF) != h->address)
                return 1;
        }
    }
    return 0;
}

static int g_succ(const xctx *c, const xguide *g, const xsys *s, uint16_t *st) {
    int n = 0;
    for (int t = 0; t < c->N; t++) { /* pop-first: a pop the log allows commutes with the rest */
        const int k = g_cursor(s, t);
        if ((uint32_t)k < g->n[t] && !(g->ev[t][k] >> 31) && x_can_pop(c, s, t)) {
            st[0] = XSTEP(XK_POP, 0, t);
            return 1;
        }
    }
    for (int t = 0; t < c->N; t++) {
        const int k = g_cursor(s, t);
        if ((uint32_t)k < g->n[t] && (g->ev[t][k] >> 31) && x_can_issue(c, s, t)) st[n++] = XSTEP(XK_ISSUE, 0, t);
        if (s->n[t].on > 0) st[n++] = XSTEP(XK_SEND, 0, t);
    }
    return n;
}

static int guided_search(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
                         orc_outcome *out, uint64_t *states, int *complete, uint16_t *witness, uint32_t wit_cap,
                         uint32_t *wit_len);

int orc_guided(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
               const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
               orc_outcome *out, uint64_t *states, int *complete) {
    return guided_search(cfg, trace, stride, lens, events, ev_count, max_states, found, out, states, complete,
                         NULL, 0, NULL);
}

int orc_guided_witness(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                       const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
                       orc_outcome *out, uint64_t *states, uint16_t *witness, uint32_t wit_cap, uint32_t *wit_len) {
    int complete = 0;
    return guided_search(cfg, trace, stride, lens, events, ev_count, max_states, found, out, states, &complete,
                         witness, wit_cap, wit_len);
}

/* The DFS keeps each stack entry's depth and the step that made it, so the steps of the path
   to the state being expanded are path[0 .. depth - 1]: the witness when the logs are met. */
static int guided_search(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         const uint32_t *events, const uint32_t *ev_count, uint64_t max_states, int *found,
                         orc_outcome *out, uint64_t *states, int *complete, uint16_t *witness, uint32_t wit_cap,
                         uint32_t *wit_len) {
    xctx c;
    if (cfg->micro != ORC_MICRO_STRICT) return -1;
    if (x_setup(&c, cfg, trace, stride, lens, 0)) return -1;
    c.guided = 1;
    xguide g;
    uint64_t off = 0;
    for (int t = 0; t < c.N; t++) {
        g.ev[t] = events + off;
        g.n[t] = ev_count[t];
        off += ev_count[t];
    }
    xset vis;
    vis.cap = 1;
    while (vis.cap < max_states + max_states / 2 + 2) vis.cap <<= 1;
    vis.keys = (uint64_t *)calloc(vis.cap, sizeof(uint64_t));
    vis.n = 0;
    size_t scap = 1024, sn = 0, pcap = 1024;
    xsys *stack = (xsys *)malloc(sizeof(xsys) * scap);
    uint32_t *sdepth = (uint32_t *)malloc(sizeof(uint32_t) * scap);
    uint16_t *sstep = (uint16_t *)malloc(sizeof(uint16_t) * scap);
    uint16_t *path = (uint16_t *)malloc(sizeof(uint16_t) * pcap);
    uint32_t hit_depth = 0;
    int rc = 0, full = 1, hit = 0;
    if (!vis.keys || !stack || !sdepth || !sstep || !path) { rc = -1; goto done; }
    x_init(&c, &stack[sn]);
    sdepth[sn] = 0;
    sstep[sn++] = 0;
    xset_insert(&vis, x_hash(&c, &stack[0]));
    while (sn > 0 && !hit) {
        --sn;
        xsys cur = stack[sn];
        const uint32_t depth = sdepth[sn];
        if (depth > 0) { /* the path to cur: its parent's path, then the step that made cur */
            if (depth > pcap) {
                pcap *= 2;
                uint16_t *p2 = (uint16_t *)realloc(path, sizeof(uint16_t) * pcap);
                if (!p2) { rc = -1; break; }
                path = p2;
            }
            path[depth - 1] = sstep[sn];
        }
        uint16_t succ[4 * ORC_MAX_PROCS];
        const int ns = g_succ(&c, &g, &cur, succ);
        if (ns == 0) {
            int all = 1;
            for (int t = 0; t < c.N; t++)
                if ((uint32_t)g_cursor(&cur, t) != g.n[t] || cur.n[t].qn || cur.n[t].on) all = 0;
            if (all) {
                uint16_t en[4 * ORC_MAX_PROCS];
                if (x_enabled(&c, &cur, en) == 0) { /* terminal in the full model too */
                    x_outcome(&c, &cur, out);
                    hit = 1;
                    hit_depth = depth;
                }
            }
            continue;
        }
        for (int k = 0; k < ns; k++) {
            xsys nxt = cur;
            x_apply(&c, &nxt, succ[k]);
            if (g_dead(&c, &g, &nxt)) continue;
            if (vis.n >= max_states) { full = 0; continue; }
            if (!xset_insert(&vis, x_hash(&c, &nxt))) continue;
            if (sn == scap) {
                scap *= 2;
                xsys *ns2 = (xsys *)realloc(stack, sizeof(xsys) * scap);
                uint32_t *d2 = ns2 ? (uint32_t *)realloc(sdepth, sizeof(uint32_t) * scap) : NULL;
                uint16_t *s2 = d2 ? (uint16_t *)realloc(sstep, sizeof(uint16_t) * scap) : NULL;
                if (ns2) stack = ns2;
                if (d2) sdepth = d2;
                if (s2) sstep = s2;
                if (!ns2 || !d2 || !s2) { full = 0; rc = -1; break; }
            }
            stack[sn] = nxt;
            sdepth[sn] = depth + 1;
            sstep[sn++] = succ[k];
        }
        if (rc) break;
    }
    if (hit && witness) {
        for (uint32_t i = 0; i < hit_depth && i < wit_cap; i++) witness[i] = path[i];
        if (hit_depth > wit_cap) rc = -3;
    }
    if (wit_len) *wit_len = hit ? hit_depth : 0;
done:
    if (found) *found = hit;
    if (states) *states = vis.n;
    if (complete) *complete = hit || (full && rc == 0);
    free(vis.keys);
    free(stack);
    free(sdepth);
    free(sstep);
    free(path);
    free(c.scratch);
    return rc;
}

/* ==== engine round schedules from the reference's own logs (round 4) ====
 *
 * orc_rounds_from_logs searches the ENGINE's round model -- each round, a chosen set of nodes
 * each takes one step on start-of-round state (pop if its queue is non-empty, else issue), then
 * the round's messages are appended sender by sender in a chosen order -- for a schedule under
 * which every node pops exactly the messages of its reference log, in order, and issues where
 * the log says. The resulting table is a dash_set_schedule input: the GPU engine then re-enacts
 * that reference run, and its own DEBUG event log must equal the reference's, thread by thread.
 * A round is built from the optional nodes (a queued head that is the node's next logged pop, or
 * an issue its log expects next); nodes whose log waits for a message sit out. The messages in a
 * queue must always be a prefix of the node's upcoming run of logged pops (a message arriving
 * before the node's logged issue would be popped first), which fixes, per receiver, the order of
 * the round's senders; the senders are then ordered by those precedences. Subsets of the
 * optional nodes are tried largest first (depth-first, visited states hashed). */

typedef struct {
    xsys s;
    uint32_t depth;
    uint8_t row[ORC_MAX_PROCS];
} xrent;

/* round with stepping set `mask` from state *s; on success writes the delivery row and returns
   1 (*s advanced), else 0 */
static int r_try(xctx *c, const xguide *g, xsys *s, uint32_t mask, uint8_t *row) {
    for (int t = 0; t < c->N; t++) {
        if (!((mask >> t) & 1)) continue;
        if (s->n[t].qn > 0) x_pop(c, s, t);
        else x_step(c, s, t, NULL);
    }
    /* precedences among senders: prec[a] has bit b when a must deliver before b */
    uint32_t prec[ORC_MAX_PROCS] = {0};
    for (int r = 0; r < c->N; r++) {
        const xnode *x = &s->n[r];
        const int k0 = g_cursor(s, r);
        /* the queue, then this round's arrivals, must follow r's upcoming run of logged pops */
        int run = 0;
        while ((uint32_t)(k0 + run) < g->n[r] && !(g->ev[r][k0 + run] >> 31)) run++;
        int pos = x->qn;
        if (pos > run) return 0;
        for (int i = 0; i < x->qn; i++) {
            const uint32_t e = g->ev[r][k0 + i];
            if ((e & 0xFF) != x->q[i].type || ((e >> 8) & 0xFF) != x->q[i].sender ||
                ((e >> 16) & 0xFF) != x->q[i].address)
                return 0;
        }
        /* each sender's block to r, in program order: match it at the position its first
           message has in the run */
        int placed = 0, last = -1;
        uint32_t done = 0;
        for (;;) {
            int total = 0;
            for (int snd = 0; snd < c->N; snd++)
                if (!((done >> snd) & 1))
                    for (int k = 0; k < s->n[snd].on; k++) total += s->n[snd].oto[k] == r;
            if (total == 0) break;
            if (pos >= run) return 0;  /* more arrivals than logged pops before r's next issue */
            const uint32_t e = g->ev[r][k0 + pos];
            const int snd = (int)((e >> 8) & 0xFF);
            if (snd >= c->N || ((done >> snd) & 1)) return 0;
            const xnode *sx = &s->n[snd];
            int n_to = 0;
            for (int k = 0; k < sx->on; k++) {
                if (sx->oto[k] != r) continue;
                if (pos + n_to >= run) return 0;
                const uint32_t f = g->ev[r][k0 + pos + n_to];
                if ((f & 0xFF) != sx->o[k].type || ((f >> 8) & 0xFF) != sx->o[k].sender ||
                    ((f >> 16) & 0xFF) != sx->o[k].address)
                    return 0;
                n_to++;
            }
            if (n_to == 0) return 0;  /* the logged next sender sent r nothing this round */
            pos += n_to;
            done |= 1u << snd;
            if (last >= 0) prec[last] |= 1u << snd;
            last = snd;
            placed++;
        }
        (void)placed;
    }
    /* a delivery order honouring the precedences (Kahn), stepping senders first by id */
    uint32_t left = (1u << c->N) - 1, p = 0;
    uint8_t order[ORC_MAX_PROCS];
    while (left) {
        int pick = -1;
        for (int a = 0; a < c->N && pick < 0; a++) {
            if (!((left >> a) & 1)) continue;
            int blocked = 0;
            for (int b = 0; b < c->N; b++)
                if (((left >> b) & 1) && ((prec[b] >> a) & 1)) blocked = 1;
            if (!blocked) pick = a;
        }
        if (pick < 0) return 0;  /* contradictory orders across receivers */
        order[p++] = (uint8_t)pick;
        left &= ~(1u << pick);
    }
    for (int k = 0; k < c->N; k++) {
        const int snd = order[k];
        while (s->n[snd].on > 0) x_send(c, s, snd);
    }
    for (int t = 0; t < c->N; t++) row[t] = 0xFF;
    for (int k = 0; k < c->N; k++)
        if ((mask >> order[k]) & 1) row[order[k]] = (uint8_t)k;
    /* positions must be distinct among stepping nodes only; the rest sit out */
    return 1;
}

int orc_rounds_from_logs(const orc_cfg *cfg, const uint16_t *trace, uint64_t stride, const uint32_t *lens,
                         const uint32_t *events, const uint32_t *ev_count, uint64_t max_states,
                         uint8_t *sched, uint32_t sched_cap, uint32_t *n_rounds, int *found, uint64_t *states) {
    xctx c;
    orc_cfg cf = *cfg;
    cf.micro = ORC_MICRO_STRICT;
    if (x_setup(&c, &cf, trace, stride, lens, 0)) return -1;
    c.guided = 1;
    xguide g;
    uint64_t off = 0;
    for (int t = 0; t < c.N; t++) {
        g.ev[t] = events + off;
        g.n[t] = ev_count[t];
        off += ev_count[t];
    }
    xset vis;
    vis.cap = 1;
    while (vis.cap < max_states + max_states / 2 + 2) vis.cap <<= 1;
    vis.keys = (uint64_t *)calloc(vis.cap, sizeof(uint64_t));
    vis.n = 0;
    size_t scap = 256, sn = 0, pcap = 1024;
    xrent *stack = (xrent *)malloc(sizeof(xrent) * scap);
    uint8_t *path = (uint8_t *)malloc((size_t)pcap * ORC_MAX_PROCS);
    int rc = 0, hit = 0;
    uint32_t hit_len = 0;
    if (!vis.keys || !stack || !path) { rc = -1; goto done; }
    x_init(&c, &stack[0].s);
    stack[0].depth = 0;
    sn = 1;
    while (sn > 0 && !hit) {
        const xrent e = stack[--sn];
        if (e.depth > 0) {
            if (e.depth > pcap) {
                pcap *= 2;
                uint8_t *np = (uint8_t *)realloc(path, (size_t)pcap * ORC_MAX_PROCS);
                if (!np) { rc = -1; break; }
                path = np;
            }
            memcpy(path + (size_t)(e.depth - 1) * ORC_MAX_PROCS, e.row, ORC_MAX_PROCS);
        }
        const xsys *s = &e.s;
        /* optional nodes; dead if a queued head is not the node's next logged pop */
        uint32_t opt = 0;
        int dead = 0, finished = 1;
        for (int t = 0; t < c.N && !dead; t++) {
            const xnode *x = &s->n[t];
            const int k = g_cursor(s, t);
            const int more = (uint32_t)k < g.n[t];
            if (more || x->qn) finished = 0;
            if (x->qn > 0) {
                if (!more || (g.ev[t][k] >> 31)) { dead = 1; break; }
                opt |= 1u << t;  /* the head was checked when it arrived */
            } else if (!x->waiting && x->idx < c.count[t]) {
                if (!more) { dead = 1; break; }
                if (g.ev[t][k] >> 31) opt |= 1u << t;
            }
        }
        if (dead) continue;
        if (finished) {
            hit = 1;
            hit_len = e.depth;
            break;
        }
        /* subsets of opt, largest first; pushed in reverse so the largest is tried first */
        uint32_t subs[256];
        int ns = 0;
        for (int bits = c.N; bits >= 1; bits--)
            for (uint32_t m = opt; m; m = (m - 1) & opt)
                if (__builtin_popcount(m) == bits) subs[ns++] = m;
        for (int i = ns - 1; i >= 0; i--) {
            xrent nx;
            nx.s = *s;
            if (!r_try(&c, &g, &nx.s, subs[i], nx.row)) continue;
            if (vis.n >= max_states) continue;
            if (!xset_insert(&vis, x_hash(&c, &nx.s))) continue;
            nx.depth = e.depth + 1;
            if (sn == scap) {
                scap *= 2;
                xrent *ns2 = (xrent *)realloc(stack, sizeof(xrent) * scap);
                if (!ns2) { rc = -1; break; }
                stack = ns2;
            }
            stack[sn++] = nx;
        }
        if (rc) break;
    }
    if (hit) {
        if (hit_len > sched_cap) rc = -2;
        else
            for (uint32_t r = 0; r < hit_len; r++)
                memcpy(sched + (size_t)r * c.N, path + (size_t)r * ORC_MAX_PROCS, (size_t)c.N);
    }
done:
    if (found) *found = hit;
    if (n_rounds) *n_rounds = hit ? hit_len : 0;
    if (states) *states = vis.n;
    free(vis.keys);
    free(stack);
    free(path);
    free(c.scratch);
    return rc;
}
