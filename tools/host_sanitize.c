/*
 * host_sanitize.c -- sanitizer run (gcc ASan + UBSan) of the host-side C code:
 *   * the CPU half of the boundary, csrc/dash_host.c: core_<n>.txt ingest
 *     (initializeProcessor's parse, assignment.c:822-850), printProcessorState
 *     dump (:853-905), digest, DEBUG_MSG / DEBUG_INSTR formatting (:179-182,
 *     :649-652);
 *   * the CPU oracle, oracle/dash_oracle.c: lockstep restatement, seeded
 *     schedules, legality checker (replay, random schedules, exhaustive search).
 * Driven over the reference's golden directories, fuzzed trace files and random
 * systems (every N, CACHE_SIZE, shallow queues that overflow, round caps).
 * GPU sanitizers are not available on this pool; the device code is covered by
 * the bit-exact parity tests instead. Built and run by tests/test_host_sanitizers.py.
 *
 * usage: host_sanitize SCRATCH_DIR GOLDEN_DIR...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dash.h"
#include "dash_oracle.h"

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return rng_state;
}
static uint32_t rndn(uint32_t n) { return (uint32_t)(rnd() % n); }

static int failures = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fputc('\n', stderr);                       \
            failures++;                                \
        }                                              \
    } while (0)

/* the boundary's dump/digest and the oracle's agree on a result */
static void check_result(const orc_result *r, int N, int CS) {
    static char a[16384], b[16384];
    for (int n = 0; n < N; n++) {
        dash_node_state d;
        memcpy(&d, &r->node[n], sizeof d); /* identical layouts (include/dash.h, oracle) */
        int la = dash_dump_node(&d, (uint32_t)n, (uint32_t)CS, a, sizeof a);
        int lb = orc_dump_node(&r->node[n], n, CS, b, (int)sizeof b);
        CHECK(la > 0 && la == lb && memcmp(a, b, (size_t)la) == 0, "dump mismatch node %d", n);
        CHECK(dash_digest_node(&d, (uint32_t)n, (uint32_t)CS) == orc_digest_node(&r->node[n], n, CS),
              "digest mismatch node %d", n);
        /* a too-small buffer is an error, never an overflow */
        CHECK(dash_dump_node(&d, (uint32_t)n, (uint32_t)CS, a, 100) < 0, "short buffer accepted");
    }
}

static void golden_dir(const char *dir) {
    enum { N = 4, L = 32 };
    uint16_t tr[N * L];
    uint32_t lens[N];
    char path[4096];
    memset(tr, 0, sizeof tr);
    for (int n = 0; n < N; n++) {
        snprintf(path, sizeof path, "%s/core_%d.txt", dir, n);
        int rc = dash_parse_core_file(path, N, L, tr + n * L, &lens[n]);
        CHECK(rc == DASH_OK, "parse %s rc %d", path, rc);
    }
    orc_cfg cfg = {N, 4, 256, 0, 1, 0, 0};
    static orc_result r;
    static char log[1 << 16];
    CHECK(orc_run_system(&cfg, tr, L, lens, &r, log, sizeof log) == 0, "oracle %s", dir);
    check_result(&r, N, 4);
    static orc_outcome o;
    uint64_t steps = 0;
    CHECK(orc_replay_lockstep(&cfg, tr, L, lens, &o, &steps) == 0, "replay %s", dir);
    CHECK(o.digest == r.digest, "replay digest %s", dir);
    for (uint64_t seed = 1; seed <= 20; seed++)
        CHECK(orc_random_schedule(&cfg, tr, L, lens, seed, &o) == 0, "random schedule %s", dir);
    cfg.arb_seed = 87;
    CHECK(orc_run_system(&cfg, tr, L, lens, &r, NULL, 0) == 0, "seeded %s", dir);
}

static const char *fuzz_line(char *buf, size_t cap) {
    static const char *const pieces[] = {"RD", "WR", "rd", " ", "\t", "0x", "0X", "-", "+", "ff", "1F",
                                         "99999999999", "300", "x", "\r", "RDWR", "WR 0x10", "RD 0x"};
    switch (rndn(6)) {
    case 0: snprintf(buf, cap, "RD 0x%02X\n", rndn(256)); break;
    case 1: snprintf(buf, cap, "WR 0x%02X %d\n", rndn(256), (int)rndn(2000) - 1000); break;
    case 2: snprintf(buf, cap, "\n"); break;
    case 3: { /* a long line: fgets(line, 20) splits it (ref :831) */
        size_t n = 20 + rndn(60);
        for (size_t i = 0; i < n && i + 2 < cap; i++) buf[i] = (char)('!' + rndn(90));
        buf[n < cap - 2 ? n : cap - 2] = '\n';
        buf[n < cap - 2 ? n + 1 : cap - 1] = 0;
        break;
    }
    default: {
        buf[0] = 0;
        for (int k = 0, m = 1 + (int)rndn(5); k < m; k++)
            strncat(buf, pieces[rndn(sizeof pieces / sizeof *pieces)], cap - strlen(buf) - 2);
        strncat(buf, "\n", cap - strlen(buf) - 1);
    }
    }
    return buf;
}

static void fuzz_ingest(const char *scratch) {
    char path[4096], line[256];
    snprintf(path, sizeof path, "%s/core_0.txt", scratch);
    uint16_t out[64];
    for (int it = 0; it < 3000; it++) {
        FILE *f = fopen(path, "w");
        if (!f) { CHECK(0, "cannot write %s", path); return; }
        for (int k = 0, n = (int)rndn(50); k < n; k++) fputs(fuzz_line(line, sizeof line), f);
        fclose(f);
        uint32_t len = 0xFFFFFFFFu;
        const uint32_t N = 1 + rndn(8), cap = rndn(65);
        int rc = dash_parse_core_file(path, N, cap, out, &len);
        CHECK(rc == DASH_OK || rc == DASH_EPARSE || rc == DASH_EADDR, "parse rc %d", rc);
        CHECK(len <= cap, "parsed %u > cap %u", len, cap);
        for (uint32_t i = 0; i < len; i++) CHECK(((out[i] >> 12) & 7u) < N, "address beyond N");
    }
    uint32_t len;
    CHECK(dash_parse_core_file("/nonexistent/core_9.txt", 4, 32, out, &len) == DASH_EIO, "missing file");
}

static void random_systems(void) {
    enum { MAXL = 48 };
    static uint16_t tr[ORC_MAX_PROCS * MAXL];
    static orc_result r;
    static orc_outcome outs[64];
    static const int depths[] = {2, 4, 8, 256};
    for (int it = 0; it < 400; it++) {
        const int N = 1 + (int)rndn(8), CS = 1 << rndn(5);
        uint32_t lens[ORC_MAX_PROCS];
        for (int n = 0; n < N; n++) {
            lens[n] = rndn(MAXL + 1);
            for (uint32_t i = 0; i < lens[n]; i++) {
                const uint32_t w = rndn(2), node = rndn((uint32_t)N), blk = rndn(it % 3 ? 16 : 2);
                tr[n * MAXL + i] = (uint16_t)((w << 15) | (((node << 4) | blk) << 8) | (w ? rndn(256) : 0));
            }
        }
        orc_cfg cfg = {N, CS, depths[rndn(4)], rndn(4) == 0 ? 1 + rndn(40) : 0, (int)rndn(2), 0,
                       rndn(3) == 0 ? rnd() | 1 : 0};
        static char log[1 << 16];
        CHECK(orc_run_system(&cfg, tr, MAXL, lens, &r, log, sizeof log) == 0, "oracle it %d", it);
        check_result(&r, N, CS);
        dash_event e = {rndn(1000), rndn(8), rndn(3), (uint32_t)rnd()};
        char buf[128];
        const int n = dash_format_event(&e, buf, sizeof buf);
        CHECK(e.kind > 1 ? n < 0 : (n > 0 && n < (int)sizeof buf), "format_event kind %u", e.kind);
        if (it % 8 == 0) { /* legality checker on small systems */
            orc_cfg c2 = {N, CS, 256, 0, 0, 0, 0};
            uint32_t small[ORC_MAX_PROCS];
            for (int k = 0; k < N; k++) small[k] = lens[k] < 3 ? lens[k] : 3;
            orc_outcome o;
            uint64_t steps;
            CHECK(orc_replay_lockstep(&c2, tr, MAXL, small, &o, &steps) == 0, "replay it %d", it);
            int nout = 0, complete = 0;
            uint64_t states = 0;
            CHECK(orc_explore(&c2, tr, MAXL, small, 2000, outs, 64, &nout, &states, &complete) == 0,
                  "explore it %d", it);
        }
    }
    /* batch mode with threads (the CPU baseline path) */
    orc_cfg cfg = {8, 4, 256, 0, 0, 0, 0};
    orc_gen g = {0x5EED, 1, 0, 64, 8};
    uint64_t dig[16], hist[ORC_NUM_TXN] = {0}, instr = 0;
    uint32_t rounds[16], errs[16];
    orc_run_batch(&cfg, &g, 0, 16, 2, dig, rounds, errs, hist, &instr);
    CHECK(instr == 16 * 8 * 64, "batch instructions %llu", (unsigned long long)instr);
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s SCRATCH_DIR GOLDEN_DIR...\n", argv[0]);
        return 2;
    }
    for (int i = 2; i < argc; i++) golden_dir(argv[i]);
    fuzz_ingest(argv[1]);
    random_systems();
    if (failures) fprintf(stderr, "%d check(s) failed\n", failures);
    else printf("host sanitizer run clean\n");
    return failures ? 1 : 0;
}
