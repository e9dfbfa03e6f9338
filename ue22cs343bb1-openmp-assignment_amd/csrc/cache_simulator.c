/*
 * cache_simulator.c -- CLI with the reference's argv contract
 * (/root/reference/assignment.c:126-131): `cache_simulator <test_directory>`
 * reads tests/<dir>/core_<n>.txt (or <dir>/core_<n>.txt), prints
 * "Processor N initialized" per node, simulates on the GPU and writes
 * core_<n>_output.txt (printProcessorState bytes) into the CWD. Unlike the
 * reference it exits 0 at quiescence instead of spinning until killed.
 *
 * Extra options (defaults = the reference's #defines, :6-10):
 *   -n NUM_PROCS (4)  -c CACHE_SIZE (4)  -m MAX_INSTR_NUM (32)
 *   -o OUT_DIR (.)    -d DEVICE (0)      -s  print run statistics to stderr
 *   --debug-instr / --debug-msg  print the reference's DEBUG_INSTR (:650-651) /
 *       DEBUG_MSG (:180-181) lines to stdout, in lockstep order (the reference's
 *       -D DEBUG_INSTR / -D DEBUG_MSG builds, README :104)
 *   --schedule SEED   a seeded legal schedule instead of lowest-sender-first (DESIGN.md §2;
 *       e.g. --schedule 87 lands tests/test_4 on its accepted run_2); also in bulk modes
 *   --rounds FILE     an explicit round schedule (dash_set_schedule): one row per round, one
 *       character per node, '-' = the node sits the round out, else its delivery position;
 *       later rounds are lockstep. FILE is plain rows, or a JSON record of tests/golden/schedules
 *       record (its "rounds" strings): e.g. tests/golden/schedules/test_4_run_3.json makes
 *       `cache_simulator test_4` write the accepted run_3
 *   --micro FILE      a micro-step schedule (dash_set_micro_schedule): whitespace-separated
 *       tokens, one per round, "P<t>" / "I<t>" / "S<t>" = node t steps (pops or issues, its
 *       sends held), "D<t>" = node t delivers its oldest held message; plain text, or the
 *       "steps" string of a JSON record (tests/golden/ref_runs/micro4.json's cases)
 *
 * Bulk modes (one GPU batch, many systems; dumps go to OUT_DIR/<k>/):
 *   --batch LIST        system k = the k-th trace directory listed in LIST (one per line)
 *   --synthetic COUNT   COUNT generated systems: --len L (4096) --kind uniform|contention|
 *                       locality --locality P (0.5) --seed S (0x5EED) --dump K[,K...]
 *   --digests FILE      "system digest rounds errors" for every system
 */
#define _POSIX_C_SOURCE 200809L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "dash.h"

static const char *txn_names[DASH_NUM_TXN] = {
    "READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV", "UPGRADE",
    "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK", "EVICT_SHARED", "EVICT_MODIFIED"};

/* --rounds FILE: rows of n characters ('-' or a position digit); from a JSON record, the quoted
   strings after its "rounds" key. Returns the row count, or -1 on a malformed file. */
static long read_micro(const char *path, unsigned n, uint8_t **out);

static long read_rounds(const char *path, unsigned n, uint8_t **out) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    static char text[1 << 20];
    size_t len = fread(text, 1, sizeof text - 1, f);
    const int more = fgetc(f) != EOF; /* a longer file would be cut: refuse it */
    fclose(f);
    if (more) return -1;
    text[len] = 0;
    const char *p = strstr(text, "\"rounds\"");
    const int json = p != NULL;
    if (!json) p = text;
    else p += 8;
    long rows = 0, cap = 0;
    uint8_t *r = NULL;
    while (*p) {
        const char *q;
        if (json) {  /* next quoted string, up to the array's end */
            while (*p && *p != '"' && *p != ']') p++;
            if (*p != '"') break;
            q = ++p;
            while (*p && *p != '"') p++;
        } else {     /* next non-empty line */
            while (*p == '\n' || *p == '\r' || *p == ' ') p++;
            if (!*p) break;
            q = p;
            while (*p && *p != '\n' && *p != '\r' && *p != ' ') p++;
        }
        if ((unsigned)(p - q) != n) { free(r); return -1; }
        if (rows == cap) {
            cap = cap ? 2 * cap : 64;
            r = (uint8_t *)realloc(r, (size_t)cap * n);
        }
        for (unsigned t = 0; t < n; t++) {
            const char c = q[t];
            if (c == '-') r[rows * n + t] = DASH_SIT_OUT;
            else if (c >= '0' && c <= '7') r[rows * n + t] = (uint8_t)(c - '0');
            else { free(r); return -1; }
        }
        rows++;
        if (*p) p++;
    }
    *out = r;
    return rows;
}

/* --micro FILE: one token per round, [PIS]<t> (a step) or D<t> (a delivery); from a JSON record, the
   string after its "steps" key. Returns the round count, or -1 on a malformed file. */
static long read_micro(const char *path, unsigned n, uint8_t **out) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    static char text[1 << 22];
    size_t len = fread(text, 1, sizeof text - 1, f);
    const int more = fgetc(f) != EOF;
    fclose(f);
    if (more) return -1;
    text[len] = 0;
    char *p = strstr(text, "\"steps\"");
    if (p) {
        p = strchr(p + 7, '"');
        if (!p) return -1;
        char *end = strchr(++p, '"');
        if (!end) return -1;
        *end = 0;
    } else {
        p = text;
    }
    long rows = 0, cap = 0;
    uint8_t *r = NULL;
    for (char *tok = strtok(p, " \t\r\n"); tok; tok = strtok(NULL, " \t\r\n")) {
        char *e;
        const long t = strtol(tok + 1, &e, 10);
        if (!strchr("PISD", tok[0]) || e == tok + 1 || *e || t < 0 || t >= (long)n) { free(r); return -1; }
        if (rows == cap) {
            cap = cap ? 2 * cap : 256;
            uint8_t *r2 = (uint8_t *)realloc(r, (size_t)cap * n);
            if (!r2) { free(r); return -1; }
            r = r2;
        }
        memset(r + rows * n, DASH_SIT_OUT, n);
        r[rows * n + t] = tok[0] == 'D' ? DASH_MICRO_SEND : DASH_MICRO_STEP;
        rows++;
    }
    *out = r;
    return rows;
}

/* dash_simulate_dir plus a schedule (seed, explicit rounds or micro-steps) and the event log of the
   one system */
static int simulate_traced(const char *dir, unsigned n, unsigned cs, unsigned m, const char *out, int dev,
                           int dbg_instr, int dbg_msg, unsigned long long sched, const uint8_t *rounds,
                           long nrounds, int micro, dash_stats *st) {
    dash_cfg cfg = {0};
    cfg.num_procs = n;
    cfg.cache_size = cs;
    cfg.max_instr = m;
    cfg.flags = DASH_KEEP_STATE;
    cfg.num_systems = 1;
    cfg.device = dev;
    /* the log holds every round the run may take (the default round cap, 1024 + 256 x max_instr,
       up to 2^22): n x 4 B per round on the device */
    uint64_t log_rounds = 1024u + 256ull * m;
    if (log_rounds > (1u << 22)) log_rounds = 1u << 22;
    cfg.trace_events = (dbg_instr || dbg_msg) ? (uint32_t)log_rounds : 0;
    cfg.schedule_seed = rounds ? (sched ? sched : 1) : sched;
    dash_t *h = NULL;
    int rc = dash_create(&cfg, &h);
    if (rc != DASH_OK) return rc;
    if (rounds) rc = micro ? dash_set_micro_schedule(h, rounds, (uint32_t)nrounds)
                           : dash_set_schedule(h, rounds, (uint32_t)nrounds);
    if (rc == DASH_OK && (rc = dash_load_dir(h, dir, 0)) == DASH_OK && (rc = dash_run(h, st)) == DASH_OK) {
        dash_node_state nodes[DASH_MAX_PROCS];
        rc = dash_read_state(h, 0, nodes);
        for (unsigned t = 0; rc == DASH_OK && t < n; t++) {
            char path[4200];
            snprintf(path, sizeof path, "%s/core_%u_output.txt", out, t);
            rc = dash_dump_file(&nodes[t], t, cs, path);
        }
        uint32_t cap = 0, total = 0;
        dash_event *ev = NULL;
        if (rc == DASH_OK && cfg.trace_events) {  /* the count first, then the events */
            int erc = dash_read_events(h, 0, NULL, 0, &cap);
            if (erc == DASH_OK || erc == DASH_ETRUNC)
                ev = (dash_event *)malloc(sizeof(dash_event) * (cap ? cap : 1));
            if (!ev) rc = (erc == DASH_OK || erc == DASH_ETRUNC) ? DASH_ENOMEM : erc;
        }
        if (rc == DASH_OK && ev) {
            int erc = dash_read_events(h, 0, ev, cap, &total);
            for (uint32_t k = 0; k < total && k < cap; k++) {
                char line[128];
                if ((ev[k].kind == DASH_EV_INSTR && dbg_instr) || (ev[k].kind == DASH_EV_MSG && dbg_msg))
                    if (dash_format_event(&ev[k], line, sizeof line) > 0) fputs(line, stdout);
            }
            if (erc != DASH_OK) rc = erc;
        }
        free(ev);
    }
    if (rc != DASH_OK) fprintf(stderr, "%s\n", dash_last_error(h));
    dash_destroy(h);
    return rc;
}

typedef struct {
    unsigned n, cs, m, len, kind, locality;
    unsigned long long seed, sched;
    int dev, show;
    const char *out, *digests, *dump;
} bulk_opts;

static void print_stats(const dash_stats *st);

static int finish_bulk(dash_t *h, const bulk_opts *o, const dash_stats *st, uint64_t count, int dump_all) {
    int rc = DASH_OK;
    if (o->digests) rc = dash_write_digests(h, o->digests);
    if (rc == DASH_OK && (dump_all || o->dump)) {
        mkdir(o->out, 0755);
        const char *p = o->dump;
        for (uint64_t k = 0; rc == DASH_OK && (dump_all ? k < count : (p && *p)); k++) {
            uint64_t sys = dump_all ? k : strtoull(p, (char **)&p, 0);
            if (!dump_all && *p == ',') p++;
            char dir[4200];
            snprintf(dir, sizeof dir, "%s/%llu", o->out, (unsigned long long)sys);
            rc = dash_dump_system(h, sys, dir);
        }
    }
    if (rc != DASH_OK) fprintf(stderr, "%s\n", dash_last_error(h));
    if (o->show) print_stats(st);
    return rc;
}

static int run_batch_list(const char *list, const bulk_opts *o) {
    FILE *f = fopen(list, "r");
    if (!f) {
        fprintf(stderr, "Error: could not open %s\n", list);
        return DASH_EIO;
    }
    char **dirs = NULL, line[4096];
    uint64_t n = 0, cap = 0;
    while (fgets(line, sizeof line, f)) {
        size_t l = strcspn(line, "\r\n");
        line[l] = 0;
        if (!l || line[0] == '#') continue;
        if (n == cap) {
            cap = cap ? 2 * cap : 64;
            dirs = (char **)realloc(dirs, cap * sizeof *dirs);
        }
        dirs[n++] = strdup(line);
    }
    fclose(f);
    dash_cfg cfg = {0};
    cfg.num_procs = o->n;
    cfg.cache_size = o->cs;
    cfg.max_instr = o->m;
    cfg.flags = DASH_KEEP_STATE;
    cfg.num_systems = n;
    cfg.device = o->dev;
    cfg.schedule_seed = o->sched;
    dash_t *h = NULL;
    dash_stats st;
    int rc = n ? dash_create(&cfg, &h) : DASH_EINVAL;
    if (rc == DASH_OK && (rc = dash_load_dirs(h, (const char *const *)dirs, n)) == DASH_OK &&
        (rc = dash_run(h, &st)) == DASH_OK)
        rc = finish_bulk(h, o, &st, n, 1);
    else if (h)
        fprintf(stderr, "%s\n", dash_last_error(h));
    dash_destroy(h);
    for (uint64_t k = 0; k < n; k++) free(dirs[k]);
    free(dirs);
    return rc;
}

static int run_synthetic(uint64_t count, const bulk_opts *o) {
    dash_cfg cfg = {0};
    cfg.num_procs = o->n;
    cfg.cache_size = o->cs;
    cfg.max_instr = o->len;
    cfg.flags = o->dump ? DASH_KEEP_STATE : 0;
    cfg.num_systems = count;
    cfg.device = o->dev;
    cfg.schedule_seed = o->sched;
    dash_gen g = {0};
    g.seed = o->seed;
    g.kind = o->kind;
    g.locality = o->locality;
    g.len = o->len;
    dash_t *h = NULL;
    dash_stats st;
    int rc = dash_create(&cfg, &h);
    if (rc == DASH_OK && (rc = dash_generate(h, &g)) == DASH_OK && (rc = dash_run(h, &st)) == DASH_OK) {
        printf("%llu systems, %llu instructions, %.3f ms, %.4g instr/s\n", (unsigned long long)st.systems,
               (unsigned long long)st.instructions, st.kernel_ms, st.instructions / (st.kernel_ms * 1e-3));
        rc = finish_bulk(h, o, &st, count, 0);
    } else if (h) {
        fprintf(stderr, "%s\n", dash_last_error(h));
    }
    dash_destroy(h);
    return rc;
}

int main(int argc, char *argv[]) {
    unsigned n = 4, cs = 4, m = 32;
    int dev = 0, show = 0, dbg_instr = 0, dbg_msg = 0, n_given = 0;
    const char *out = ".", *dir = NULL, *batch = NULL, *digests = NULL, *dump = NULL, *rounds_file = NULL,
               *micro_file = NULL;
    unsigned long long synth = 0, seed = 0x5EED, sched = 0;
    unsigned len = 4096, kind = DASH_GEN_UNIFORM;
    double loc = 0.5;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) n = (unsigned)atoi(argv[++i]), n_given = 1;
        else if (!strcmp(argv[i], "-c") && i + 1 < argc) cs = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-m") && i + 1 < argc) m = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!strcmp(argv[i], "-d") && i + 1 < argc) dev = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s")) show = 1;
        else if (!strcmp(argv[i], "--debug-instr")) dbg_instr = 1;
        else if (!strcmp(argv[i], "--debug-msg")) dbg_msg = 1;
        else if (!strcmp(argv[i], "--batch") && i + 1 < argc) batch = argv[++i];
        else if (!strcmp(argv[i], "--synthetic") && i + 1 < argc) synth = strtoull(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--digests") && i + 1 < argc) digests = argv[++i];
        else if (!strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
        else if (!strcmp(argv[i], "--len") && i + 1 < argc) len = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) seed = strtoull(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--schedule") && i + 1 < argc) sched = strtoull(argv[++i], NULL, 0);
        else if (!strcmp(argv[i], "--rounds") && i + 1 < argc) rounds_file = argv[++i];
        else if (!strcmp(argv[i], "--micro") && i + 1 < argc) micro_file = argv[++i];
        else if (!strcmp(argv[i], "--locality") && i + 1 < argc) loc = atof(argv[++i]);
        else if (!strcmp(argv[i], "--kind") && i + 1 < argc) {
            const char *k = argv[++i];
            kind = !strcmp(k, "contention") ? DASH_GEN_CONTENTION : !strcmp(k, "locality") ? DASH_GEN_LOCALITY
                                                                                         : DASH_GEN_UNIFORM;
        }
        else if (!dir) dir = argv[i];
    }
    if (batch || synth) {
        if (synth && !n_given) n = 8; /* synthetic systems default to 8 nodes (BASELINE configs) */
        bulk_opts o = {n, cs, m, len, kind, (unsigned)(loc * 65536.0), seed, sched, dev, show, out, digests, dump};
        if (o.locality > 65536u) o.locality = 65536u;
        int rc = batch ? run_batch_list(batch, &o) : run_synthetic(synth, &o);
        return rc == DASH_OK ? EXIT_SUCCESS : EXIT_FAILURE;
    }
    if (!dir) {
        fprintf(stderr, "Usage: %s <test_directory>\n", argv[0]); /* ref :128 */
        return EXIT_FAILURE;
    }
    uint8_t *rounds = NULL;
    long nrounds = 0;
    if (rounds_file && micro_file) {  /* two schedules for one run: refuse rather than drop one */
        fprintf(stderr, "cache_simulator: --rounds and --micro are exclusive\n");
        return EXIT_FAILURE;
    }
    if (rounds_file && (nrounds = read_rounds(rounds_file, n, &rounds)) < 0) {
        fprintf(stderr, "cache_simulator: %s: not a round schedule for %u nodes\n", rounds_file, n);
        return EXIT_FAILURE;
    }
    if (micro_file && (nrounds = read_micro(micro_file, n, &rounds)) <= 0) {
        /* an empty micro-step schedule would fall through to a plain lockstep run */
        fprintf(stderr, "cache_simulator: %s: %s\n", micro_file,
                nrounds == 0 ? "empty micro-step schedule" : "not a micro-step schedule");
        free(rounds);
        return EXIT_FAILURE;
    }
    dash_stats st;
    int rc = (dbg_instr || dbg_msg || sched || rounds)
                 ? simulate_traced(dir, n, cs, m, out, dev, dbg_instr, dbg_msg, sched, rounds, nrounds,
                                   micro_file != NULL, &st)
                 : dash_simulate_dir(dir, n, cs, m, out, dev, &st);
    free(rounds);
    if (rc != DASH_OK) {
        const char *why = dash_last_error(NULL);
        fprintf(stderr, "cache_simulator: %s (%d)\n", why[0] ? why : "failed", rc);
        return EXIT_FAILURE;
    }
    if (show) print_stats(&st);
    return st.err_bits ? 2 : EXIT_SUCCESS;
}

static void print_stats(const dash_stats *st) {
    fprintf(stderr, "rounds %llu instructions %llu errors 0x%llx dropped %llu\n",
            (unsigned long long)st->rounds_total, (unsigned long long)st->instructions,
            (unsigned long long)st->err_bits, (unsigned long long)st->dropped);
    for (int k = 0; k < DASH_NUM_TXN; k++)
        fprintf(stderr, "  %-15s %llu\n", txn_names[k], (unsigned long long)st->hist[k]);
}
