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
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dash.h"

static const char *txn_names[DASH_NUM_TXN] = {
    "READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV", "UPGRADE",
    "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK", "EVICT_SHARED", "EVICT_MODIFIED"};

int main(int argc, char *argv[]) {
    unsigned n = 4, cs = 4, m = 32;
    int dev = 0, show = 0;
    const char *out = ".", *dir = NULL;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) n = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-c") && i + 1 < argc) cs = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-m") && i + 1 < argc) m = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
        else if (!strcmp(argv[i], "-d") && i + 1 < argc) dev = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s")) show = 1;
        else if (!dir) dir = argv[i];
    }
    if (!dir) {
        fprintf(stderr, "Usage: %s <test_directory>\n", argv[0]); /* ref :128 */
        return EXIT_FAILURE;
    }
    dash_stats st;
    int rc = dash_simulate_dir(dir, n, cs, m, out, dev, &st);
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
