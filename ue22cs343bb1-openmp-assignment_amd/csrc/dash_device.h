// dash_device.h -- argument blocks shared by the HIP kernels and the host API.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dash {

// DASH_ERR_* of include/dash.h, restated for device code
constexpr uint32_t DASH_ERR_OVERFLOW_D = 1u;
constexpr uint32_t DASH_ERR_OOB_D = 2u;
constexpr uint32_t DASH_ERR_CTZ0_D = 4u;
constexpr uint32_t DASH_ERR_DEADLOCK_D = 8u;
constexpr uint32_t DASH_ERR_ROUNDCAP_D = 16u;
constexpr uint32_t DASH_ERR_STUCK_D = 32u;
constexpr uint32_t DASH_ERR_SCHEDULE_D = 64u;

// device statistics block (u64 words)
enum : uint32_t {
    STAT_HIST = 0,  // 13 words
    STAT_INSTR = 13,
    STAT_ROUNDS = 14,
    STAT_ROUNDS_MAX = 15,
    STAT_SYSTEMS = 16,
    STAT_ERRSYS = 17,
    STAT_ERRBITS = 18,
    STAT_DROPS = 19,
    STAT_MAXDEPTH = 20,
    STAT_WAVE_ROUNDS = 21,  // loop trips summed over waves (the kernel's unit of work)
    STAT_WORDS = 32
};

struct SimArgs {
    const uint2* trace;       // [group][64 lanes][chunk] x 8 B (4 packed instructions)
    const uint32_t* lens;     // [sys * N + node]
    uint64_t nsys;
    uint32_t nchunks;
    uint32_t num_procs;
    uint32_t max_rounds;
    uint32_t final_tier;      // 1: queue overflow drops (reference semantics); 0: hand off
    const uint32_t* sys_list; // systems to (re)run; nullptr = all systems in order
    uint64_t list_len;
    uint32_t* ovf_list;       // systems handed to the next queue-depth tier
    uint32_t* ovf_count;
    uint64_t* digests;        // [sys]
    uint32_t* rounds;         // [sys]
    uint32_t* errors;         // [sys]
    uint32_t* state;          // optional [(sys*N+node)*(16+CS)] directory/cache words
    uint32_t* hist;           // [sys*13] messages handled per type; written when keep
    uint32_t keep;
    uint32_t event_cap;       // event log capacity in rounds, a multiple of 4 (0: no log)
    uint32_t* events;         // [sys][round / 4][node][round % 4]: one word per node and round, 0 = none
    uint32_t* event_count;    // [sys*N+node] events produced (may exceed event_cap)
    unsigned long long* stats;  // [STAT_WORDS]
    uint64_t arb_seed;        // 0: lowest-sender-first lockstep; else the seeded schedule
    const uint32_t* arb_tab;  // seeded schedule: per-round word (arb_word) for rounds < arb_len
    uint32_t arb_len;         // a multiple of 4; rounds beyond it hash their key in the kernel
    uint32_t micro;           // 1: arb_tab is a micro-step table (dash_set_micro_schedule, MODE 4)
    const uint8_t* skip;      // optional [sys]: 1 = run elsewhere this pass (a deeper tier, concurrently)
    uint32_t cache_size;      // CACHE_SIZE (ref :7); read by the generic (non-power-of-two) kernels
    uint64_t cs_lut;          // nibble b = b % cache_size, b < 16 (generic kernels)
};

struct GenArgs {
    uint2* trace;
    uint32_t* lens;
    uint64_t nsys;
    uint64_t ngroups;
    uint64_t seed;
    uint64_t sys_base;
    uint32_t nchunks;
    uint32_t num_procs;
    uint32_t seg;
    uint32_t kind;
    uint32_t locality;
    uint32_t len;
};

hipError_t launch_sim(const SimArgs& a, uint32_t seg, uint32_t cs, uint32_t ring, uint64_t groups,
                      hipStream_t s);

// queue-depth tiers: each re-runs the systems that overflowed the previous one;
// the last is the reference's MSG_BUFFER_SIZE (ref :9) and drops like it
constexpr int NUM_TIERS = 3;
constexpr uint32_t RING_TIERS[NUM_TIERS] = {16, 32, 256};
constexpr uint32_t CHUNK_INSTR = 4;  // instructions per 8-B trace chunk
// spare 8-B chunks after the trace buffer: a lane's window refill reads up to two chunks past
// its last instruction (never issued), so the last lane's stream needs no bounds test
constexpr uint64_t TRACE_PAD = 64;
hipError_t launch_gen(const GenArgs& g, hipStream_t s);
// the seeded schedule's table: each node's word (arb_node) of rounds [0, n), n a multiple of 4,
// laid out [round / 4][node < seg][round % 4]; rounds past it are hashed in sim_kernel
constexpr uint32_t ARB_TABLE_MAX = 1u << 22;
hipError_t launch_arb_table(uint64_t seed, uint32_t seg, uint32_t* out, uint32_t n, hipStream_t s);
// skip[list[i]] = 1 for i < n
// RD words carry value 0 (ref :839): clears bits 7..0 of every word whose bit 15 is 0
hipError_t launch_clear_rd(uint2* trace, uint64_t words, hipStream_t s);
hipError_t launch_mark(const uint32_t* list, uint64_t n, uint8_t* skip, hipStream_t s);
// box probe: blocks x 256 threads, 8 full-rate VALU per trip; clk[2 * block] = shader cycles,
// clk[2 * block + 1] = 100-MHz reference ticks of that block's loop
constexpr uint32_t PROBE_VALU_PER_TRIP = 8;
hipError_t launch_probe(uint32_t blocks, uint32_t iters, uint32_t* sink, unsigned long long* clk, hipStream_t s);

}  // namespace dash
