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
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dash.h"

static const char *txn_names[DASH_NUM_TXN] = {
    "READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV", "UPGRADE",
    "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK", "EVICT_SHARED", "EVICT_MODIFIED"};

/* dash_simulate_dir plus the event log of the one system */
static int simulate_traced(const char *dir, unsigned n, unsigned cs, unsigned m, const char *out, int dev,
                           int dbg_instr, int dbg_msg, dash_stats *st) {
    dash_cfg cfg = {0};
    cfg.num_procs = n;
    cfg.cache_size = cs;
    cfg.max_instr = m;
    cfg.flags = DASH_KEEP_STATE;
    cfg.num_systems = 1;
    cfg.device = dev;
    cfg.trace_events = 1u << 16;
    dash_t *h = NULL;
    int rc = dash_create(&cfg, &h);
    if (rc != DASH_OK) return rc;
    if ((rc = dash_load_dir(h, dir, 0)) == DASH_OK && (rc = dash_run(h, st)) == DASH_OK) {
        dash_node_state nodes[DASH_MAX_PROCS];
        rc = dash_read_state(h, 0, nodes);
        for (unsigned t = 0; rc == DASH_OK && t < n; t++) {
            char path[4200];
            snprintf(path, sizeof path, "%s/core_%u_output.txt", out, t);
            rc = dash_dump_file(&nodes[t], t, cs, path);
        }
        uint32_t cap = cfg.trace_events * n, total = 0;
        dash_event *ev = (dash_event *)malloc(sizeof(dash_event) * cap);
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

int main(int argc, char *argv[]) {
    unsigned n = 4, cs = 4, m = 32;
    int dev = 0, show = 0, dbg_instr = 0, dbg_msg = 0;
    const char *out = ".", *dir = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) n = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-c") && i + 1 < argc) cs = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-m") && i + 1 < argc) m = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!strcmp(argv[i], "-d") && i + 1 < argc) dev = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s")) show = 1;
        else if (!strcmp(argv[i], "--debug-instr")) dbg_instr = 1;
        else if (!strcmp(argv[i], "--debug-msg")) dbg_msg = 1;
        else if (!dir) dir = argv[i];
    }
    if (!dir) {
        fprintf(stderr, "Usage: %s <test_directory>\n", argv[0]); /* ref :128 */
        return EXIT_FAILURE;
    }
    dash_stats st;
    int rc = (dbg_instr || dbg_msg) ? simulate_traced(dir, n, cs, m, out, dev, dbg_instr, dbg_msg, &st)
                                    : dash_simulate_dir(dir, n, cs, m, out, dev, &st);
    if (rc != DASH_OK) {
        fprintf(stderr, "cache_simulator: failed (%d)\n", rc);
        return EXIT_FAILURE;
    }
    if (show) {
        fprintf(stderr, "rounds %llu instructions %llu errors 0x%llx dropped %llu\n",
                (unsigned long long)st.rounds_total, (unsigned long long)st.instructions,
                (unsigned long long)st.err_bits, (unsigned long long)st.dropped);
        for (int k = 0; k < DASH_NUM_TXN; k++)
            fprintf(stderr, "  %-15s %llu\n", txn_names[k], (unsigned long long)st.hist[k]);
    }
    return st.err_bits ? 2 : EXIT_SUCCESS;
}
