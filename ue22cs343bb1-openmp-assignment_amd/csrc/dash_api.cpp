// dash_api.cpp -- C-ABI of libdash over HIP (handles, device buffers, launches).
//
// Replaces main()'s OpenMP plumbing in /root/reference/assignment.c:
// omp_set_num_threads / queue + lock init (:135-144), the parallel region
// (:149-155) and the per-thread private processorNode (:145).
#include <hip/hip_runtime.h>

#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdarg>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <memory>
#include <vector>

#include "dash.h"
#include "dash_device.h"

struct dash_ctx {
    dash_cfg cfg{};
    uint32_t seg = 0;       // lanes per system (next pow2 of num_procs)
    uint64_t groups = 0;    // waves (64/seg systems each)
    uint32_t nchunks = 0;   // lane stride of the trace layout in 4-instruction (8-B) chunks
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    uint2* d_trace = nullptr;
    uint32_t* d_lens = nullptr;
    uint64_t* d_digests = nullptr;
    uint32_t* d_rounds = nullptr;
    uint32_t* d_errors = nullptr;
    uint32_t* d_state = nullptr;
    uint32_t* d_hist = nullptr;
    unsigned long long* d_stats = nullptr;
    uint32_t* d_list[2] = {nullptr, nullptr};  // overflow hand-off lists (ping-pong)
    uint32_t* d_count = nullptr;
    uint32_t* d_events = nullptr;       // [sys][round / 4][node][round % 4] (rounds: ev_rounds)
    uint32_t* d_arb = nullptr;          // seeded schedule: one word per node and round (dash::arb_node)
    uint32_t arb_len = 0;
    bool micro = false;                 // the round table is a micro-step schedule (MODE 4)
    uint32_t* d_event_count = nullptr;  // [sys*N+node]
    uint32_t ev_rounds = 0;             // trace_events rounded up to a multiple of 4
    uint64_t tier_systems[dash::NUM_TIERS] = {};  // systems run per queue-depth tier, last run
    int auto_tier = 0;                         // adaptive first tier
    // overflow hint: the systems that overflowed the first tier in earlier
    // runs of the same traces; the next run starts them one tier deeper on a side stream,
    // concurrently with the first tier, which skips them. Reset whenever traces change.
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint32_t* d_hint = nullptr;  // [num_systems] system ids
    uint8_t* d_skip = nullptr;   // [num_systems] 1 = in the hint
    uint64_t hint_n = 0;
    int hint_tier = -1;
    bool loaded = false;
    bool ran = false;
    char msg[256] = {0};
};

static int fail(dash_t* h, int code, const char* fmt, ...) {
    if (h) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(h->msg, sizeof h->msg, fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(h, expr)                                                                  \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return fail((h), DASH_EDEVICE, "%s: %s", #expr, hipGetErrorString(e_));      \
    } while (0)

static uint32_t next_pow2(uint32_t n) {
    uint32_t p = 1;
    while (p < n) p <<= 1;
    return p;
}

// new traces: the overflow hint no longer applies
static hipError_t reset_hint(dash_t* h) {
    if (h->hint_n == 0) return hipSuccess;
    h->hint_n = 0;
    h->hint_tier = -1;
    return hipMemsetAsync(h->d_skip, 0, std::max<uint64_t>(h->cfg.num_systems, 1), h->stream);
}

// message of the last failed handle-less call (dash_create, dash_run_host_batched, ...) on this thread
static thread_local char g_msg[256] = "";

static void set_global_msg(const char* m) { snprintf(g_msg, sizeof g_msg, "%s", m ? m : ""); }

// Runs an entry point's body so that no C++ exception crosses the C-ABI: a failed allocation
// becomes DASH_ENOMEM (on the handle, or dash_last_error(NULL) without one).
template <class F>
static int guarded(dash_t* h, const char* what, F&& body) {
    char m[256];
    try {
        return body();
    } catch (const std::bad_alloc&) {
        snprintf(m, sizeof m, "%s: out of host memory", what);
        if (h) return fail(h, DASH_ENOMEM, "%s", m);
        set_global_msg(m);
        return DASH_ENOMEM;
    } catch (...) {
        snprintf(m, sizeof m, "%s: unexpected host failure", what);
        if (h) return fail(h, DASH_EDEVICE, "%s", m);
        set_global_msg(m);
        return DASH_EDEVICE;
    }
}

extern "C" {

// largest round cap: event words carry the round in bits 30..0 (bit 31 = issued instruction)
static constexpr uint64_t MAX_ROUNDS_CAP = 0x7FFFFFFCull;

const char* dash_last_error(const dash_t* h) { return h ? h->msg : g_msg; }

void* dash_stream(dash_t* h) { return h ? (void*)h->stream : nullptr; }

static void release(dash_t* h) {
    if (!h) return;
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    (void)hipFree(h->d_trace);
    (void)hipFree(h->d_lens);
    (void)hipFree(h->d_digests);
    (void)hipFree(h->d_rounds);
    (void)hipFree(h->d_errors);
    (void)hipFree(h->d_state);
    (void)hipFree(h->d_hist);
    (void)hipFree(h->d_stats);
    (void)hipFree(h->d_list[0]);
    (void)hipFree(h->d_list[1]);
    (void)hipFree(h->d_count);
    (void)hipFree(h->d_events);
    (void)hipFree(h->d_event_count);
    (void)hipFree(h->d_hint);
    (void)hipFree(h->d_skip);
    (void)hipFree(h->d_arb);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
    if (h->ev_join) (void)hipEventDestroy(h->ev_join);
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->stream) (void)hipStreamDestroy(h->stream);
}

void dash_destroy(dash_t* h) {
    release(h);
    delete h;
}

int dash_create(const dash_cfg* cfg, dash_t** out) {
    set_global_msg("");  // dash_last_error(NULL) describes this call only
    auto invalid = [](const char* why) {
        set_global_msg(why);
        return DASH_EINVAL;
    };
    if (!cfg || !out) return invalid("dash_create: null cfg or out");
    *out = nullptr;
    const uint32_t N = cfg->num_procs, CS = cfg->cache_size;
    if (N < 1 || N > DASH_MAX_PROCS) return invalid("dash_create: num_procs must be 1..8");
    if (CS < 1 || CS > DASH_MAX_CACHE) return invalid("dash_create: cache_size must be 1..16");  // (ref :7)
    if (cfg->max_instr > (1u << 24)) return invalid("dash_create: max_instr above 2^24");
    if (cfg->num_systems > 0xFFFFFFFFull)  // system ids are u32 in the lists
        return invalid("dash_create: num_systems above 2^32 - 1");
    if (cfg->trace_events >= (1u << 30))
        return invalid("dash_create: trace_events must be below 2^30");
    if (cfg->trace_events && (double)cfg->num_systems * N * (cfg->trace_events + 3u) * 4.0 > 64.0 * (1ull << 30))
        return invalid("dash_create: event log larger than 64 GiB");
    dash_t* h = new (std::nothrow) dash_ctx();
    if (!h) {
        set_global_msg("dash_create: out of host memory");
        return DASH_ENOMEM;
    }
    h->cfg = *cfg;
    if (h->cfg.max_rounds == 0) h->cfg.max_rounds = 1024ull + 256ull * cfg->max_instr;
    // clamped below 2^31 (event words keep the round in bits 30..0) before it is rounded up to
    // the multiple of 4 the kernel tests at the first round of every trip (no wrap to 0)
    h->cfg.max_rounds = (std::min<uint64_t>(h->cfg.max_rounds, MAX_ROUNDS_CAP) + 3) & ~3ull;
    h->seg = next_pow2(N);
    const uint64_t spw = 64 / h->seg;
    h->groups = (cfg->num_systems + spw - 1) / spw;
    {
        // lane stride of the trace layout: an odd number of 128-B lines, so the
        // streams of a wave's lanes (and of consecutive waves) spread over L2 sets
        // and channels instead of aliasing at a power-of-two stride
        const uint32_t raw = (cfg->max_instr + dash::CHUNK_INSTR - 1) / dash::CHUNK_INSTR;
        uint32_t lines = (raw * 8 + 127) / 128;
        // (measured: 359 vs 389 GB of L2 fills per 1M-system launch)
        h->nchunks = (lines + ((lines && !(lines & 1)) ? 1u : 0u)) * 16;
    }
    int rc = DASH_OK;
    auto chk = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == DASH_OK)
            rc = fail(h, e == hipErrorOutOfMemory ? DASH_ENOMEM : DASH_EDEVICE, "%s: %s", what,
                      hipGetErrorString(e));
    };
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        delete h;
        set_global_msg("dash_create: no HIP device");
        return DASH_EDEVICE;
    }
    if (cfg->device < 0 || cfg->device >= ndev) {
        delete h;
        return invalid("dash_create: device ordinal out of range");
    }
    chk(hipSetDevice(cfg->device), "hipSetDevice");
    chk(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), "hipStreamCreate");
    chk(hipEventCreate(&h->ev0), "hipEventCreate");
    chk(hipEventCreate(&h->ev1), "hipEventCreate");
    const uint64_t nsys = cfg->num_systems;
    const uint64_t trace_words = h->groups * (uint64_t)std::max<uint32_t>(h->nchunks, 1) * 64;
    chk(hipMalloc(&h->d_trace, (trace_words + dash::TRACE_PAD) * sizeof(uint2)), "hipMalloc(trace)");
    chk(hipMalloc(&h->d_lens, std::max<uint64_t>(nsys * N, 1) * sizeof(uint32_t)), "hipMalloc(lens)");
    chk(hipMalloc(&h->d_digests, std::max<uint64_t>(nsys, 1) * sizeof(uint64_t)), "hipMalloc(digests)");
    chk(hipMalloc(&h->d_rounds, std::max<uint64_t>(nsys, 1) * sizeof(uint32_t)), "hipMalloc(rounds)");
    chk(hipMalloc(&h->d_errors, std::max<uint64_t>(nsys, 1) * sizeof(uint32_t)), "hipMalloc(errors)");
    chk(hipMalloc(&h->d_stats, dash::STAT_WORDS * sizeof(unsigned long long)), "hipMalloc(stats)");
    chk(hipMalloc(&h->d_hist, std::max<uint64_t>(nsys, 1) * 13 * sizeof(uint32_t)), "hipMalloc(hist)");
    chk(hipMalloc(&h->d_list[0], std::max<uint64_t>(nsys, 1) * sizeof(uint32_t)), "hipMalloc(list)");
    chk(hipMalloc(&h->d_list[1], std::max<uint64_t>(nsys, 1) * sizeof(uint32_t)), "hipMalloc(list)");
    chk(hipMalloc(&h->d_count, 2 * sizeof(uint32_t)), "hipMalloc(count)");
    chk(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking), "hipStreamCreate(side)");
    chk(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming), "hipEventCreate");
    chk(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming), "hipEventCreate");
    chk(hipMalloc(&h->d_hint, std::max<uint64_t>(nsys, 1) * sizeof(uint32_t)), "hipMalloc(hint)");
    chk(hipMalloc(&h->d_skip, std::max<uint64_t>(nsys, 1)), "hipMalloc(skip)");
    if (rc == DASH_OK) chk(hipMemset(h->d_skip, 0, std::max<uint64_t>(nsys, 1)), "hipMemset(skip)");
    if (cfg->trace_events) {
        h->ev_rounds = (cfg->trace_events + 3u) & ~3u;
        chk(hipMalloc(&h->d_events, std::max<uint64_t>(nsys * N * h->ev_rounds, 1) * 4), "hipMalloc(events)");
        chk(hipMalloc(&h->d_event_count, std::max<uint64_t>(nsys * N, 1) * 4), "hipMalloc(event_count)");
    }
    if (cfg->schedule_seed) {  // the seeded schedule's round words, built once per handle
        // DASH_TEST_SHORT_ARB (tests only) cuts the table to 8 rounds so the in-kernel hashing
        // past its end runs
        const uint64_t cap = (cfg->flags & DASH_TEST_SHORT_ARB) ? 8u : dash::ARB_TABLE_MAX;
        h->arb_len = (uint32_t)std::min<uint64_t>(h->cfg.max_rounds, std::min<uint64_t>(cap, dash::ARB_TABLE_MAX));
        chk(hipMalloc(&h->d_arb, ((uint64_t)h->arb_len + 4) * h->seg * sizeof(uint32_t)), "hipMalloc(arb)");
        if (rc == DASH_OK) chk(dash::launch_arb_table(cfg->schedule_seed, h->seg, h->d_arb, h->arb_len, h->stream),
                               "arb table");
        if (rc == DASH_OK) chk(hipStreamSynchronize(h->stream), "arb table");
    }
    if (cfg->flags & DASH_KEEP_STATE)
        chk(hipMalloc(&h->d_state, std::max<uint64_t>(nsys * N, 1) * (16 + CS) * sizeof(uint32_t)),
            "hipMalloc(state)");
    if (rc != DASH_OK) {
        set_global_msg(h->msg);  // no stderr from the library: dash_last_error(NULL) has it
        dash_destroy(h);
        return rc;
    }
    *out = h;
    return DASH_OK;
}

int dash_load_traces(dash_t* h, const uint16_t* packed, uint64_t stride, const uint32_t* lens,
                     uint64_t num_systems) {
    return guarded(h, "dash_load_traces", [&]() -> int {
        if (!h || (!packed && num_systems) || !lens) return DASH_EINVAL;
        const uint32_t N = h->cfg.num_procs, P = h->seg;
        if (num_systems != h->cfg.num_systems) return fail(h, DASH_EINVAL, "num_systems mismatch");
        for (uint64_t i = 0; i < num_systems * N; i++)
            if (lens[i] > h->cfg.max_instr || lens[i] > stride)
                return fail(h, DASH_EINVAL, "trace %llu longer than max_instr", (unsigned long long)i);
        // the 3-bit node field cannot name a node >= 8, so only N < 8 needs the address scan
        if (N < 8)
            for (uint64_t r = 0; r < num_systems * N; r++)
                for (uint32_t i = 0; i < lens[r]; i++) {
                    const uint16_t w = packed[r * stride + i];
                    if (((w >> 12) & 7u) >= N)
                        return fail(h, DASH_EADDR, "system %llu node %u: address 0x%02X homed on node >= %u",
                                    (unsigned long long)(r / N), (unsigned)(r % N), (w >> 8) & 0x7F, N);
                }
        // lane-contiguous layout: [group][lane][chunk][4 x u16]
        const uint64_t words = h->groups * (uint64_t)h->nchunks * 64;
        constexpr uint32_t C = dash::CHUNK_INSTR;
        const uint64_t pitch = (uint64_t)h->nchunks * 8;  // lane stride in bytes
        HIPCHK(h, hipSetDevice(h->cfg.device));
        if (P == N) {
            // system s node t is lane row s*N + t in both layouts: one strided H2D copy, no
            // host staging. Words past a node's length are never issued (the kernel's pc < len
            // guard), so they need no zeroing.
            if (num_systems)
                HIPCHK(h, hipMemcpy2DAsync(h->d_trace, pitch, packed, stride * 2, std::min<uint64_t>(stride * 2, pitch),
                                           num_systems * N, hipMemcpyHostToDevice, h->stream));
        } else {
            std::vector<uint16_t> host(words * C, 0);
            for (uint64_t s = 0; s < num_systems; s++) {
                const uint64_t g = s / (64 / P);
                const uint32_t lane0 = (uint32_t)(s % (64 / P)) * P;
                for (uint32_t t = 0; t < N; t++) {
                    const uint16_t* src = packed + (s * N + t) * stride;
                    for (uint32_t i = 0; i < lens[s * N + t]; i++)
                        host[((g * 64 + lane0 + t) * h->nchunks + i / C) * C + (i % C)] = src[i];
                }
            }
            if (words)
                HIPCHK(h, hipMemcpyAsync(h->d_trace, host.data(), words * 8, hipMemcpyHostToDevice, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));  // `host` is pageable and local
        }
        // RD carries value 0 whatever the caller's bits 7..0 say (ref :839; dash.h)
        HIPCHK(h, dash::launch_clear_rd(h->d_trace, words, h->stream));
        if (num_systems)
            HIPCHK(h, hipMemcpyAsync(h->d_lens, lens, num_systems * N * 4, hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, reset_hint(h));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->loaded = true;
        h->ran = false;
        return DASH_OK;
    });
}

int dash_generate(dash_t* h, const dash_gen* g) {
    if (!h || !g) return DASH_EINVAL;
    if (g->len > h->cfg.max_instr) return fail(h, DASH_EINVAL, "gen len > max_instr");
    if (g->kind > DASH_GEN_LOCALITY) return fail(h, DASH_EINVAL, "unknown generator kind");
    dash::GenArgs a{};
    a.trace = h->d_trace;
    a.lens = h->d_lens;
    a.nsys = h->cfg.num_systems;
    a.ngroups = h->groups;
    a.seed = g->seed;
    a.sys_base = g->sys_base;
    a.nchunks = h->nchunks;
    a.num_procs = h->cfg.num_procs;
    a.seg = h->seg;
    a.kind = g->kind;
    a.locality = g->locality;
    a.len = g->len;
    HIPCHK(h, hipSetDevice(h->cfg.device));
    HIPCHK(h, dash::launch_gen(a, h->stream));
    HIPCHK(h, reset_hint(h));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    h->loaded = true;
    h->ran = false;
    return DASH_OK;
}

int dash_set_schedule(dash_t* h, const uint8_t* sched, uint32_t rounds) {
    return guarded(h, "dash_set_schedule", [&]() -> int {
        if (!h || (!sched && rounds)) return DASH_EINVAL;
        if (!h->d_arb) return fail(h, DASH_ESTATE, "dash_set_schedule: handle created with schedule_seed = 0");
        const uint32_t N = h->cfg.num_procs, P = h->seg;
        if (h->arb_len < h->cfg.max_rounds)
            return fail(h, DASH_EINVAL, "dash_set_schedule: the round table holds %u of max_rounds %llu rounds",
                        h->arb_len, (unsigned long long)h->cfg.max_rounds);
        if (rounds > h->arb_len) return fail(h, DASH_EINVAL, "dash_set_schedule: %u rounds > max_rounds", rounds);
        for (uint32_t r = 0; r < rounds; r++) {
            uint32_t used = 0;
            for (uint32_t t = 0; t < N; t++) {
                const uint8_t v = sched[(uint64_t)r * N + t];
                if (v == DASH_SIT_OUT) continue;
                if (v >= P || (used >> v) & 1u)
                    return fail(h, DASH_EINVAL, "dash_set_schedule: round %u node %u: position %u invalid or repeated",
                                r, t, (unsigned)v);
                used |= 1u << v;
            }
        }
        // the kernel's table layout (dash_kernels.hip arb_table_kernel): [round / 4][lane][round % 4],
        // each word 0 for a node sitting out, else its primary arrival bit 2 << 4 * position
        std::vector<uint32_t> tab(((uint64_t)h->arb_len + 4) * P, 0);
        for (uint64_t r = 0; r < (uint64_t)h->arb_len + 4; r++)
            for (uint32_t t = 0; t < P; t++) {
                uint32_t w = 0;
                if (t < N) {
                    const uint32_t v = r < rounds ? sched[r * N + t] : t;  // later rounds: lockstep
                    w = v == DASH_SIT_OUT ? 0u : 2u << (4u * v);
                }
                tab[((r >> 2) * P + t) * 4 + (r & 3)] = w;
            }
        HIPCHK(h, hipSetDevice(h->cfg.device));
        HIPCHK(h, hipMemcpyAsync(h->d_arb, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->ran = false;
        h->micro = false;
        return DASH_OK;
    });
}

int dash_set_micro_schedule(dash_t* h, const uint8_t* acts, uint32_t rounds) {
    return guarded(h, "dash_set_micro_schedule", [&]() -> int {
        if (!h || (!acts && rounds)) return DASH_EINVAL;
        if (!h->d_arb) return fail(h, DASH_ESTATE, "dash_set_micro_schedule: handle created with schedule_seed = 0");
        const uint32_t N = h->cfg.num_procs, P = h->seg;
        if (h->arb_len < h->cfg.max_rounds)
            return fail(h, DASH_EINVAL, "dash_set_micro_schedule: the round table holds %u of max_rounds %llu rounds",
                        h->arb_len, (unsigned long long)h->cfg.max_rounds);
        if (rounds > h->arb_len)
            return fail(h, DASH_EINVAL, "dash_set_micro_schedule: %u rounds > max_rounds", rounds);
        for (uint32_t r = 0; r < rounds; r++) {
            uint32_t acting = 0;
            for (uint32_t t = 0; t < N; t++) {
                const uint8_t v = acts[(uint64_t)r * N + t];
                if (v == DASH_SIT_OUT) continue;
                if (v != DASH_MICRO_STEP && v != DASH_MICRO_SEND)
                    return fail(h, DASH_EINVAL, "dash_set_micro_schedule: round %u node %u: action %u invalid", r, t,
                                (unsigned)v);
                ++acting;
            }
            if (acting > 1) return fail(h, DASH_EINVAL, "dash_set_micro_schedule: round %u: %u nodes act", r, acting);
        }
        // table words (dash_kernels.hip MODE 4): 0 = sits out, 1 = steps, 2 = sends one held
        // message; every node sits out past the schedule
        std::vector<uint32_t> tab(((uint64_t)h->arb_len + 4) * P, 0);
        for (uint64_t r = 0; r < rounds; r++)
            for (uint32_t t = 0; t < N; t++) {
                const uint8_t v = acts[r * N + t];
                tab[((r >> 2) * P + t) * 4 + (r & 3)] = v == DASH_SIT_OUT ? 0u : v == DASH_MICRO_STEP ? 1u : 2u;
            }
        HIPCHK(h, hipSetDevice(h->cfg.device));
        HIPCHK(h, hipMemcpyAsync(h->d_arb, tab.data(), tab.size() * sizeof(uint32_t), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->ran = false;
        h->micro = true;
        return DASH_OK;
    });
}

int dash_run(dash_t* h, dash_stats* stats) {
    if (!h) return DASH_EINVAL;
    if (!h->loaded) return fail(h, DASH_ESTATE, "no traces loaded");
    dash::SimArgs a{};
    a.trace = h->d_trace;
    a.lens = h->d_lens;
    a.nsys = h->cfg.num_systems;
    a.nchunks = h->nchunks;
    a.num_procs = h->cfg.num_procs;
    a.max_rounds = (uint32_t)h->cfg.max_rounds;
    a.digests = h->d_digests;
    a.rounds = h->d_rounds;
    a.errors = h->d_errors;
    a.state = h->d_state;
    a.hist = h->d_hist;
    a.keep = (h->cfg.flags & DASH_KEEP_STATE) ? 1u : 0u;
    a.event_cap = h->ev_rounds;
    a.arb_seed = h->cfg.schedule_seed;
    a.arb_tab = h->d_arb;
    a.arb_len = h->arb_len;
    a.micro = h->micro ? 1u : 0u;
    a.cache_size = h->cfg.cache_size;
    for (uint32_t b = 0; b < 16; b++)  // b % CACHE_SIZE for the generic (non-power-of-two) kernels
        a.cs_lut |= (uint64_t)(b % h->cfg.cache_size) << (4 * b);
    a.events = h->d_events;
    a.event_count = h->d_event_count;
    a.stats = h->d_stats;
    const uint64_t spw = 64 / h->seg;
    HIPCHK(h, hipSetDevice(h->cfg.device));
    HIPCHK(h, hipMemsetAsync(h->d_stats, 0, dash::STAT_WORDS * sizeof(unsigned long long), h->stream));
    HIPCHK(h, hipEventRecord(h->ev0, h->stream));
    // queue-depth tiers: every system runs at the first depth; systems that would
    // overflow it are listed and re-run from scratch at the next depth (exact:
    // the lockstep schedule is deterministic); the last tier drops like the reference.
    // Without a DASH_TIER_FROM_* flag the first depth adapts: when more than 1/32 of
    // the systems overflowed the first depth of a run, later runs start one deeper.
    uint64_t todo = h->cfg.num_systems;
    const uint32_t* list = nullptr;
    const uint32_t f = h->cfg.flags;
    // a micro-step schedule runs at the reference's queue depth only (sim_kernel MODE 4)
    const int first = (h->micro || (f & DASH_TIER_FROM_256)) ? 2 : (f & DASH_TIER_FROM_32) ? 1 : h->auto_tier;
    if (h->hint_n && h->hint_tier != first) HIPCHK(h, reset_hint(h));
    // Systems that overflowed the first tier in an earlier run of these traces (the
    // schedule is deterministic, so they will again) start one tier deeper on the side
    // stream right away, while the first tier -- which skips them -- runs on the main
    // stream: the deeper pass no longer waits for the first tier's tail.
    const bool hint = h->hint_n > 0 && first < dash::NUM_TIERS - 1;
    const int ht = first + 1;
    if (hint) {
        HIPCHK(h, hipMemsetAsync(h->d_count + (ht & 1), 0, sizeof(uint32_t), h->stream));
        HIPCHK(h, hipEventRecord(h->ev_fork, h->stream));
        HIPCHK(h, hipStreamWaitEvent(h->side, h->ev_fork, 0));
        dash::SimArgs b = a;
        b.sys_list = h->d_hint;
        b.list_len = h->hint_n;
        b.final_tier = ht == dash::NUM_TIERS - 1 ? 1u : 0u;
        b.ovf_list = h->d_list[ht & 1];  // shared with the main stream's pass at this tier
        b.ovf_count = h->d_count + (ht & 1);
        HIPCHK(h, dash::launch_sim(b, h->seg, h->cfg.cache_size, dash::RING_TIERS[ht],
                                   (h->hint_n + spw - 1) / spw, h->side));
        HIPCHK(h, hipEventRecord(h->ev_join, h->side));
    }
    uint64_t first_ovf = 0;  // systems that overflowed the first tier in this run
    for (int tier = 0; tier < dash::NUM_TIERS; ++tier) h->tier_systems[tier] = 0;
    for (int tier = first; tier < dash::NUM_TIERS; ++tier) {
        const bool last = tier == dash::NUM_TIERS - 1;
        const bool joined = hint && tier == ht;  // the hinted pass ran this tier too
        h->tier_systems[tier] = todo + (joined ? h->hint_n : 0);
        uint32_t* out = h->d_list[tier & 1];
        uint32_t* cnt = h->d_count + (tier & 1);
        if (!joined) HIPCHK(h, hipMemsetAsync(cnt, 0, sizeof(uint32_t), h->stream));
        if (todo) {
            a.sys_list = list;
            a.list_len = todo;
            a.final_tier = last ? 1u : 0u;
            a.ovf_list = out;
            a.ovf_count = cnt;
            a.skip = (hint && tier == first) ? h->d_skip : nullptr;
            HIPCHK(h, dash::launch_sim(a, h->seg, h->cfg.cache_size, dash::RING_TIERS[tier],
                                       (todo + spw - 1) / spw, h->stream));
        }
        if (joined) HIPCHK(h, hipStreamWaitEvent(h->stream, h->ev_join, 0));
        if (last) break;
        uint32_t next = 0;
        if (todo || joined) {
            HIPCHK(h, hipMemcpyAsync(&next, cnt, sizeof next, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
        if (tier == first) first_ovf = next;
        todo = next;
        list = out;
    }
    if (first < dash::NUM_TIERS - 1 && first_ovf) {  // they join the hint for the next run
        HIPCHK(h, hipMemcpyAsync(h->d_hint + h->hint_n, h->d_list[first & 1], first_ovf * sizeof(uint32_t),
                                 hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(h, dash::launch_mark(h->d_list[first & 1], first_ovf, h->d_skip, h->stream));
        h->hint_n += first_ovf;
        h->hint_tier = first;
    }
    if (!(f & (DASH_TIER_FROM_32 | DASH_TIER_FROM_256)) && first < dash::NUM_TIERS - 1 &&
        h->tier_systems[first + 1] * 32 > h->tier_systems[first])
        h->auto_tier = first + 1;
    HIPCHK(h, hipEventRecord(h->ev1, h->stream));
    unsigned long long s[dash::STAT_WORDS];
    HIPCHK(h, hipMemcpyAsync(s, h->d_stats, sizeof s, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    float ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
    h->ran = true;
    if (stats) {
        memset(stats, 0, sizeof *stats);
        for (int k = 0; k < DASH_NUM_TXN; k++) stats->hist[k] = s[dash::STAT_HIST + k];
        stats->instructions = s[dash::STAT_INSTR];
        stats->rounds_total = s[dash::STAT_ROUNDS];
        stats->rounds_max = s[dash::STAT_ROUNDS_MAX];
        stats->systems = s[dash::STAT_SYSTEMS];
        stats->err_systems = s[dash::STAT_ERRSYS];
        stats->err_bits = s[dash::STAT_ERRBITS];
        stats->dropped = s[dash::STAT_DROPS];
        stats->max_depth = s[dash::STAT_MAXDEPTH];
        stats->kernel_ms = ms;
        for (int k = 0; k < dash::NUM_TIERS; k++) stats->tier_systems[k] = h->tier_systems[k];
        stats->wave_rounds = s[dash::STAT_WAVE_ROUNDS];
    }
    return DASH_OK;
}

int dash_read_results(dash_t* h, uint64_t first, uint64_t count, uint64_t* digests,
                      uint32_t* rounds, uint32_t* errors) {
    if (!h) return DASH_EINVAL;
    if (!h->ran) return fail(h, DASH_ESTATE, "dash_run has not completed");
    if (first + count > h->cfg.num_systems || first + count < first)
        return fail(h, DASH_EINVAL, "range out of bounds");
    HIPCHK(h, hipSetDevice(h->cfg.device));
    if (digests && count)
        HIPCHK(h, hipMemcpyAsync(digests, h->d_digests + first, count * 8, hipMemcpyDeviceToHost, h->stream));
    if (rounds && count)
        HIPCHK(h, hipMemcpyAsync(rounds, h->d_rounds + first, count * 4, hipMemcpyDeviceToHost, h->stream));
    if (errors && count)
        HIPCHK(h, hipMemcpyAsync(errors, h->d_errors + first, count * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return DASH_OK;
}

int dash_read_state(dash_t* h, uint64_t sys, dash_node_state* out) {
    return guarded(h, "dash_read_state", [&]() -> int {
        if (!h || !out) return DASH_EINVAL;
        if (!h->ran) return fail(h, DASH_ESTATE, "dash_run has not completed");
        if (!h->d_state) return fail(h, DASH_ESTATE, "created without DASH_KEEP_STATE");
        if (sys >= h->cfg.num_systems) return fail(h, DASH_EINVAL, "system out of range");
        const uint32_t N = h->cfg.num_procs, CS = h->cfg.cache_size, W = 16 + CS;
        std::vector<uint32_t> w((size_t)N * W);
        HIPCHK(h, hipSetDevice(h->cfg.device));
        HIPCHK(h, hipMemcpyAsync(w.data(), h->d_state + sys * N * W, w.size() * 4, hipMemcpyDeviceToHost,
                                 h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        for (uint32_t t = 0; t < N; t++) {
            dash_node_state* s = &out[t];
            memset(s, 0, sizeof *s);
            for (uint32_t b = 0; b < 16; b++) {
                const uint32_t e = w[t * W + b];
                s->memory[b] = (uint8_t)(e & 0xFF);
                s->dir_bitvector[b] = (uint8_t)((e >> 8) & 0xFF);
                s->dir_state[b] = (uint8_t)((e >> 16) & 3);
            }
            for (uint32_t i = 0; i < CS; i++) {
                const uint32_t l = w[t * W + 16 + i];
                s->cache_addr[i] = (uint8_t)(l & 0xFF);
                s->cache_value[i] = (uint8_t)((l >> 8) & 0xFF);
                s->cache_state[i] = (uint8_t)((l >> 16) & 3);
            }
        }
        return DASH_OK;
    });
}

int dash_read_hist(dash_t* h, uint64_t sys, uint32_t* hist) {
    if (!h || !hist) return DASH_EINVAL;
    if (!h->ran) return fail(h, DASH_ESTATE, "dash_run has not completed");
    if (!(h->cfg.flags & DASH_KEEP_STATE)) return fail(h, DASH_ESTATE, "created without DASH_KEEP_STATE");
    if (sys >= h->cfg.num_systems) return fail(h, DASH_EINVAL, "system out of range");
    HIPCHK(h, hipSetDevice(h->cfg.device));
    HIPCHK(h, hipMemcpyAsync(hist, h->d_hist + sys * 13, 13 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                             h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return DASH_OK;
}

int dash_read_events(dash_t* h, uint64_t sys, dash_event* out, uint32_t cap, uint32_t* n) {
    return guarded(h, "dash_read_events", [&]() -> int {
        if (!h || (!out && cap) || !n) return DASH_EINVAL;
        if (!h->ran) return fail(h, DASH_ESTATE, "dash_run has not completed");
        if (!h->d_events) return fail(h, DASH_ESTATE, "created with trace_events = 0");
        if (sys >= h->cfg.num_systems) return fail(h, DASH_EINVAL, "system out of range");
        const uint32_t N = h->cfg.num_procs, R = h->ev_rounds;
        std::vector<uint32_t> cnt(N);
        uint32_t sys_rounds = 0;
        HIPCHK(h, hipSetDevice(h->cfg.device));
        HIPCHK(h, hipMemcpyAsync(cnt.data(), h->d_event_count + sys * N, N * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipMemcpyAsync(&sys_rounds, h->d_rounds + sys, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        uint64_t total = 0, logged = 0;
        for (uint32_t t = 0; t < N; t++) total += cnt[t];
        // count-only call (out NULL, cap 0) on a log that holds every round the system ran: the
        // per-node counts are the answer and nothing can be truncated, so skip the row copy
        if (!out && sys_rounds <= R) {
            *n = (uint32_t)std::min<uint64_t>(total, 0xFFFFFFFFull);
            return DASH_OK;
        }
        // only this run's rounds: the kernel writes the log up to its wave's last trip and never
        // clears it, so rows past the system's last active round may hold an earlier run's words
        // (ADVICE r4). Events only happen in rounds < rounds[sys]; copy whole 4-round rows of those.
        const uint32_t Rs = std::min<uint32_t>(R, (uint32_t)std::min<uint64_t>(((uint64_t)sys_rounds + 3u) & ~3ull,
                                                                                 0xFFFFFFFCull));
        std::vector<uint32_t> ev((size_t)N * Rs);
        if (Rs) {
            HIPCHK(h, hipMemcpyAsync(ev.data(), h->d_events + sys * N * (uint64_t)R, ev.size() * 4,
                                     hipMemcpyDeviceToHost, h->stream));
            HIPCHK(h, hipStreamSynchronize(h->stream));
        }
        // the log is round-major (a node logs at most one event per round): reading it round by
        // round, node by node, is the lockstep order
        uint32_t k = 0;
        for (uint32_t r = 0; r < std::min(Rs, sys_rounds); r++)
            for (uint32_t t = 0; t < N; t++) {
                const uint32_t w = ev[(size_t)(r / 4) * N * 4 + t * 4 + r % 4];
                if (!(w & 0x01000000u)) continue;  // bit 24: an event
                ++logged;
                if (k < cap) {
                    out[k].round = r;
                    out[k].node = t;
                    out[k].kind = (w & 0x80000000u) ? DASH_EV_INSTR : DASH_EV_MSG;
                    // a message word without the kernel's internal bits (7: REPLY_RD's dirState,
                    // 15: the reply-table flag, 24) and with secondReceiver moved from bits 30..28
                    // to 26..24, as include/dash.h documents it
                    out[k].word = (w & 0x80000000u) ? (w & 0xFFFFu) : (w & 0x00FF7F7Fu) | (((w >> 28) & 7u) << 24);
                }
                ++k;
            }
        const bool trunc = logged < total;  // events past the log's rounds were counted, not stored
        *n = (uint32_t)std::min<uint64_t>(total, 0xFFFFFFFFull);
        return trunc ? fail(h, DASH_ETRUNC, "event log truncated at %u rounds", R) : DASH_OK;
    });
}

int dash_load_dir(dash_t* h, const char* dir, uint64_t sys) {
    return guarded(h, "dash_load_dir", [&]() -> int {
        if (!h || !dir) return DASH_EINVAL;
        if (h->cfg.num_systems != 1 || sys != 0)
            return fail(h, DASH_EINVAL, "dash_load_dir loads a batch of one system");
        char base[4096], path[4200];
        int rc = dash_resolve_dir(dir, base, sizeof base);
        const uint32_t N = h->cfg.num_procs, M = h->cfg.max_instr;
        std::vector<uint16_t> tr((size_t)N * std::max<uint32_t>(M, 1), 0);
        std::vector<uint32_t> lens(N, 0);
        for (uint32_t t = 0; t < N; t++) {
            snprintf(path, sizeof path, "%s/core_%u.txt", base, t);
            rc = dash_parse_core_file(path, N, M, tr.data() + (size_t)t * std::max<uint32_t>(M, 1), &lens[t]);
            if (rc != DASH_OK) return fail(h, rc, "%s: parse failed (%d)", path, rc);
            printf("Processor %u initialized\n", t); /* ref :850 */
        }
        return dash_load_traces(h, tr.data(), std::max<uint32_t>(M, 1), lens.data(), 1);
    });
}

int dash_load_dirs(dash_t* h, const char* const* dirs, uint64_t n) {
    return guarded(h, "dash_load_dirs", [&]() -> int {
        if (!h || (!dirs && n)) return DASH_EINVAL;
        if (n != h->cfg.num_systems) return fail(h, DASH_EINVAL, "%llu directories for %llu systems",
                                                 (unsigned long long)n, (unsigned long long)h->cfg.num_systems);
        const uint32_t N = h->cfg.num_procs, M = h->cfg.max_instr, stride = std::max<uint32_t>(M, 1);
        std::vector<uint16_t> tr((size_t)n * N * stride, 0);
        std::vector<uint32_t> lens((size_t)n * N, 0);
        std::atomic<uint64_t> next{0}, bad{~0ull};
        std::atomic<int> bad_rc{DASH_OK};
        auto worker = [&]() {
            char base[4096], path[4200];
            for (uint64_t k; (k = next.fetch_add(1)) < n;) {
                int rc = dash_resolve_dir(dirs[k], base, sizeof base);
                for (uint32_t t = 0; rc == DASH_OK && t < N; t++) {
                    snprintf(path, sizeof path, "%s/core_%u.txt", base, t);
                    rc = dash_parse_core_file(path, N, M, tr.data() + (k * N + t) * stride, &lens[k * N + t]);
                }
                if (rc != DASH_OK) {
                    uint64_t prev = bad.load();
                    while (k < prev && !bad.compare_exchange_weak(prev, k)) {
                    }
                    bad_rc = rc;
                }
            }
        };
        const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({n, 16, std::max(1u, std::thread::hardware_concurrency())}));
        std::vector<std::thread> pool;
        try {
            for (unsigned i = 1; i < nt; i++) pool.emplace_back(worker);
        } catch (...) {  // no thread: the calling thread takes the remaining directories
        }
        worker();
        for (auto& th : pool) th.join();
        if (bad.load() != ~0ull)
            return fail(h, bad_rc.load(), "%s: trace directory rejected (%d)", dirs[bad.load()], bad_rc.load());
        return dash_load_traces(h, tr.data(), stride, lens.data(), n);
    });
}

int dash_dump_system(dash_t* h, uint64_t sys, const char* out_dir) {
    return guarded(h, "dash_dump_system", [&]() -> int {
        if (!h || !out_dir) return DASH_EINVAL;
        std::vector<dash_node_state> st(h->cfg.num_procs);
        int rc = dash_read_state(h, sys, st.data());
        if (rc != DASH_OK) return rc;
        if (mkdir(out_dir, 0755) != 0 && errno != EEXIST) return fail(h, DASH_EIO, "mkdir %s", out_dir);
        for (uint32_t t = 0; t < h->cfg.num_procs; t++) {
            char path[4200];
            snprintf(path, sizeof path, "%s/core_%u_output.txt", out_dir, t);
            rc = dash_dump_file(&st[t], t, h->cfg.cache_size, path);
            if (rc != DASH_OK) return fail(h, rc, "write %s", path);
        }
        return DASH_OK;
    });
}

// dash_write_digests: the lines of fprintf("%llu %016llx %u %x\n") for every system, formatted by
// hand in parallel chunks (one fprintf per line ran at ~4e6 lines/s) and written in order. The
// results are read and formatted one window of chunks (2 per thread) at a time, into buffers
// reused from window to window, so host memory stays bounded (~8 MiB of text per thread) at
// any num_systems.
static int write_digests_impl(dash_t* h, const char* path) {
    const uint64_t n = h->cfg.num_systems;
    constexpr uint64_t CHUNK = 1u << 16;  // lines per chunk: <= 64 B each
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const uint64_t window = std::max<uint64_t>(1, std::min<uint64_t>(n, 2ull * nt * CHUNK));
    // default-initialised (new T[]): zero-filling ~100 MB of buffers the writer overwrites anyway
    // cost as much as the formatting (round 4: 26.5 ms per 1M systems)
    std::unique_ptr<uint64_t[]> d(new uint64_t[window]);
    std::unique_ptr<uint32_t[]> r(new uint32_t[window]), e(new uint32_t[window]);
    const uint64_t wch = (window + CHUNK - 1) / CHUNK;
    std::vector<std::unique_ptr<char[]>> buf(wch);
    for (auto& b : buf) b.reset(new char[CHUNK * 64]);
    std::vector<size_t> used(wch);
    FILE* f = fopen(path, "w");
    if (!f) return fail(h, DASH_EIO, "open %s", path);
    bool ok = true;
    for (uint64_t w0 = 0; ok && w0 < n; w0 += window) {
        const uint64_t wn = std::min(window, n - w0);
        int rc = dash_read_results(h, w0, wn, d.get(), r.get(), e.get());
        if (rc != DASH_OK) {
            fclose(f);
            return rc;
        }
        const uint64_t nch = (wn + CHUNK - 1) / CHUNK;
        std::atomic<uint64_t> next{0};
        auto work = [&] {  // touches only its chunks' preallocated buffers: nothing here allocates
            static const char HEX[] = "0123456789abcdef";
            for (uint64_t c; (c = next.fetch_add(1)) < nch;) {
                char* o = buf[c].get();
                auto dec = [&o](uint64_t v) {
                    char t[20];
                    int m = 0;
                    do t[m++] = (char)('0' + v % 10); while ((v /= 10) != 0);
                    while (m) *o++ = t[--m];
                };
                for (uint64_t k = c * CHUNK; k < std::min<uint64_t>(wn, (c + 1) * CHUNK); k++) {
                    dec(w0 + k);
                    *o++ = ' ';
                    for (int sh = 60; sh >= 0; sh -= 4) *o++ = HEX[(d[k] >> sh) & 15];
                    *o++ = ' ';
                    dec(r[k]);
                    *o++ = ' ';
                    int sh = 28;
                    while (sh > 0 && ((e[k] >> sh) & 15) == 0) sh -= 4;
                    for (; sh >= 0; sh -= 4) *o++ = HEX[(e[k] >> sh) & 15];
                    *o++ = '\n';
                }
                used[c] = (size_t)(o - buf[c].get());
            }
        };
        std::vector<std::thread> pool;
        try {
            for (uint64_t i = 1; i < std::min<uint64_t>(nch, nt); i++) pool.emplace_back(work);
        } catch (...) {  // no thread: the calling thread formats the remaining chunks
        }
        work();
        for (auto& th : pool) th.join();
        for (uint64_t c = 0; ok && c < nch; c++) ok = fwrite(buf[c].get(), 1, used[c], f) == used[c];
    }
    return (fclose(f) == 0 && ok) ? DASH_OK : fail(h, DASH_EIO, "write %s", path);
}

int dash_write_digests(dash_t* h, const char* path) {
    if (!h || !path) return DASH_EINVAL;
    try {  // no C++ exception crosses the C-ABI
        return write_digests_impl(h, path);
    } catch (const std::bad_alloc&) {
        return fail(h, DASH_ENOMEM, "dash_write_digests: out of host memory");
    } catch (...) {
        return fail(h, DASH_EIO, "dash_write_digests: unexpected failure");
    }
}

int dash_probe_box(int device, dash_box_probe* out) {
    return guarded(nullptr, "dash_probe_box", [&]() -> int {
        set_global_msg("");
        if (!out) return DASH_EINVAL;
        memset(out, 0, sizeof *out);
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
            set_global_msg("dash_probe_box: no such HIP device");
            return DASH_EDEVICE;
        }
        hipDeviceProp_t p;
        if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&p, device) != hipSuccess) {
            set_global_msg("dash_probe_box: hipGetDeviceProperties failed");
            return DASH_EDEVICE;
        }
        snprintf(out->name, sizeof out->name, "%s", p.name);
        if (!out->name[0] && hipDeviceGetName(out->name, (int)sizeof out->name, device) != hipSuccess) out->name[0] = 0;
        snprintf(out->arch, sizeof out->arch, "%s", p.gcnArchName);
        out->compute_units = p.multiProcessorCount;
        out->clock_khz = p.clockRate;
        out->mem_clock_khz = p.memoryClockRate;
        out->pci_domain = p.pciDomainID;
        out->pci_bus = p.pciBusID;
        out->pci_device = p.pciDeviceID;
        out->total_mem = p.totalGlobalMem;
        const uint32_t blocks = (uint32_t)std::max(1, p.multiProcessorCount) * 8u;
        // ~170 ms at 2.4 GHz (2 wave64 VALU per cycle per CU): long enough for the clock to settle
    // (a 20-ms probe measured 1.88 GHz on a box whose sysfs clock read 2.39 GHz under load)
    const uint32_t iters = 1u << 21;
        uint32_t* sink = nullptr;
        unsigned long long* clk = nullptr;
        hipStream_t st = nullptr;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        int rc = DASH_OK;
        auto chk = [&](hipError_t e, const char* what) {
            if (e != hipSuccess && rc == DASH_OK) {
                rc = DASH_EDEVICE;
                char m[256];
                snprintf(m, sizeof m, "dash_probe_box: %s: %s", what, hipGetErrorString(e));
                set_global_msg(m);
            }
        };
        chk(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
        chk(hipEventCreate(&e0), "event");
        chk(hipEventCreate(&e1), "event");
        chk(hipMalloc(&sink, 4), "hipMalloc");
        chk(hipMalloc(&clk, (size_t)blocks * 2 * sizeof(unsigned long long)), "hipMalloc");
        if (rc == DASH_OK) chk(dash::launch_probe(blocks, 1024, sink, clk, st), "warm-up launch");
        if (rc == DASH_OK) chk(hipEventRecord(e0, st), "event");
        if (rc == DASH_OK) chk(dash::launch_probe(blocks, iters, sink, clk, st), "launch");
        if (rc == DASH_OK) chk(hipEventRecord(e1, st), "event");
        std::vector<unsigned long long> c((size_t)blocks * 2);
        if (rc == DASH_OK) chk(hipMemcpyAsync(c.data(), clk, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost, st), "copy");
        if (rc == DASH_OK) chk(hipStreamSynchronize(st), "sync");
        float ms = 0.f;
        if (rc == DASH_OK) chk(hipEventElapsedTime(&ms, e0, e1), "elapsed");
        if (rc == DASH_OK) {
            double cyc = 0, ref = 0, lo = 1e30, hi = 0;
            for (uint32_t b = 0; b < blocks; b++) {
                cyc += (double)c[2 * b];
                ref += (double)c[2 * b + 1];
                if (c[2 * b + 1]) {
                    const double f = (double)c[2 * b] / (double)c[2 * b + 1] * 100.0;  // MHz
                    lo = std::min(lo, f);
                    hi = std::max(hi, f);
                }
            }
            out->probe_ms = ms;
            out->probe_valu_per_s = (double)blocks * 4.0 * iters * dash::PROBE_VALU_PER_TRIP / (ms / 1e3);
            out->probe_sclk_mhz = ref > 0 ? cyc / ref * 100.0 : 0.0;
            out->probe_sclk_min_mhz = hi > 0 ? lo : 0.0;
            out->probe_sclk_max_mhz = hi;
        }
        (void)hipFree(sink);
        (void)hipFree(clk);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (st) (void)hipStreamDestroy(st);
        return rc;
    });
}

int dash_simulate_dir(const char* dir, uint32_t num_procs, uint32_t cache_size, uint32_t max_instr,
                      const char* out_dir, int device, dash_stats* stats) {
    return guarded(nullptr, "dash_simulate_dir", [&]() -> int {
        dash_cfg cfg{};
        cfg.num_procs = num_procs;
        cfg.cache_size = cache_size;
        cfg.max_instr = max_instr;
        cfg.flags = DASH_KEEP_STATE;
        cfg.num_systems = 1;
        cfg.device = device;
        dash_t* h = nullptr;
        int rc = dash_create(&cfg, &h);
        if (rc != DASH_OK) return rc;
        rc = dash_load_dir(h, dir, 0);
        if (rc != DASH_OK) {
            set_global_msg(h->msg);
            dash_destroy(h);
            return rc;
        }
        rc = dash_run(h, stats);
        std::vector<dash_node_state> st(num_procs);
        if (rc == DASH_OK) rc = dash_read_state(h, 0, st.data());
        for (uint32_t t = 0; rc == DASH_OK && t < num_procs; t++) {
            char path[4200];
            snprintf(path, sizeof path, "%s/core_%u_output.txt", out_dir ? out_dir : ".", t);
            rc = dash_dump_file(&st[t], t, cache_size, path);
        }
        if (rc != DASH_OK) set_global_msg(h->msg);
        dash_destroy(h);
        return rc;
    });
}

}  // extern "C"

// ---- host-buffer throughput path: batches on two handles, copies overlapped with runs ----
extern "C" int dash_run_host_batched(const dash_cfg* cfg, const uint16_t* packed, uint64_t stride,
                                     const uint32_t* lens, uint64_t num_systems, uint32_t batches,
                                     dash_stats* stats, uint64_t* digests, uint32_t* rounds,
                                     uint32_t* errors) {
    return guarded(nullptr, "dash_run_host_batched", [&]() -> int {
        if (!cfg || !packed || !lens || !stats || batches == 0 || num_systems == 0 || num_systems % batches)
            return DASH_EINVAL;
        const uint64_t nb = num_systems / batches, N = cfg->num_procs;
        dash_cfg c = *cfg;
        c.num_systems = nb;
        // throughput path: per-system state snapshots and event logs are not returned here,
        // so the handles do not allocate them
        c.flags &= ~(uint32_t)DASH_KEEP_STATE;
        c.trace_events = 0;
        const unsigned nh = batches < 2 ? 1u : 2u;
        dash_t* h[2] = {nullptr, nullptr};
        set_global_msg("");
        int rc = DASH_OK;
        for (unsigned i = 0; i < nh && rc == DASH_OK; i++) rc = dash_create(&c, &h[i]);
        dash_stats part[2];
        memset(part, 0, sizeof part);
        int trc[2] = {DASH_OK, DASH_OK};
        std::atomic<bool> stop{false};  // the first failing lane stops the other one too
        // handle i (its own HIP stream) takes batches i, i+2, ...: while one copies, the other runs
        auto lane = [&](unsigned i) {
            for (uint64_t b = i; b < batches && !stop.load(); b += nh) {
                int r = dash_load_traces(h[i], packed + b * nb * N * stride, stride, lens + b * nb * N, nb);
                dash_stats st;
                if (r == DASH_OK) r = dash_run(h[i], &st);
                if (r == DASH_OK && (digests || rounds || errors))
                    r = dash_read_results(h[i], 0, nb, digests ? digests + b * nb : nullptr,
                                          rounds ? rounds + b * nb : nullptr, errors ? errors + b * nb : nullptr);
                if (r != DASH_OK) {
                    trc[i] = r;
                    stop.store(true);
                    break;
                }
                dash_stats& p = part[i];
                for (int k = 0; k < DASH_NUM_TXN; k++) p.hist[k] += st.hist[k];
                p.instructions += st.instructions;
                p.rounds_total += st.rounds_total;
                p.rounds_max = std::max(p.rounds_max, st.rounds_max);
                p.systems += st.systems;
                p.err_systems += st.err_systems;
                p.err_bits |= st.err_bits;
                p.dropped += st.dropped;
                p.max_depth = std::max(p.max_depth, st.max_depth);
                p.kernel_ms += st.kernel_ms;
                for (int k = 0; k < DASH_NUM_TIERS; k++) p.tier_systems[k] += st.tier_systems[k];
                p.wave_rounds += st.wave_rounds;
            }
        };
        if (rc == DASH_OK) {
            std::vector<std::thread> pool;
            for (unsigned i = 0; i < nh; i++) {
                try {
                    pool.emplace_back(lane, i);
                } catch (...) {  // no thread: this lane's batches run on the calling thread
                    lane(i);
                }
            }
            for (auto& t : pool) t.join();
            rc = trc[0] != DASH_OK ? trc[0] : trc[1];
            if (rc != DASH_OK) set_global_msg(h[trc[0] != DASH_OK ? 0 : 1]->msg);
        }
        for (unsigned i = 0; i < nh; i++)
            if (h[i]) dash_destroy(h[i]);
        if (rc != DASH_OK) return rc;
        *stats = part[0];
        if (nh == 2) {
            const dash_stats& q = part[1];
            for (int k = 0; k < DASH_NUM_TXN; k++) stats->hist[k] += q.hist[k];
            stats->instructions += q.instructions;
            stats->rounds_total += q.rounds_total;
            stats->rounds_max = std::max(stats->rounds_max, q.rounds_max);
            stats->systems += q.systems;
            stats->err_systems += q.err_systems;
            stats->err_bits |= q.err_bits;
            stats->dropped += q.dropped;
            stats->max_depth = std::max(stats->max_depth, q.max_depth);
            stats->kernel_ms += q.kernel_ms;
            for (int k = 0; k < DASH_NUM_TIERS; k++) stats->tier_systems[k] += q.tier_systems[k];
            stats->wave_rounds += q.wave_rounds;
        }
        return DASH_OK;
    });
}
