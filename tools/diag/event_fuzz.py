#!/usr/bin/env python3
"""Differential fuzz of the DEBUG_MSG / DEBUG_INSTR event log (round-major layout, MODE 2 / 3)
against the oracle on one MI355X (measurement / test infrastructure: the oracle is the checker).

For every (num_procs, cache_size, schedule, trace shape) configuration: a random batch, one
engine run with the log sized to the run's round cap, and every system's formatted log compared
with the oracle's log of the same schedule, line for line; digests compared too.
Usage (through gpurun): python3 tools/diag/event_fuzz.py [configs] [systems] [maxlen] OUT.json
"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from oracle_ctypes import run_system  # noqa: E402
from test_gpu_parity import random_batch  # noqa: E402


def main():
    ncfg = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    nsys = int(sys.argv[2]) if len(sys.argv) > 2 else 192
    maxlen = int(sys.argv[3]) if len(sys.argv) > 3 else 96
    out = sys.argv[4] if len(sys.argv) > 4 else None
    dash = bench.load_dash()
    rng = np.random.default_rng(0xE7E7)
    report = {"configs": [], "systems": 0, "events": 0, "mismatched_systems": 0}
    t0 = time.time()
    for c in range(ncfg):
        N = int(rng.integers(1, 9))
        CS = int(rng.choice([1, 2, 3, 4, 5, 8, 16]))
        seed = 0 if c % 2 == 0 else int(rng.integers(1, 1 << 32))
        span = int(rng.choice([2, 4, 16]))
        hot = float(rng.choice([0.0, 0.0, 0.5, 0.8]))
        L = int(rng.integers(1, maxlen + 1))
        packed, lens = random_batch(rng, nsys, N, L, block_span=span, hot_frac=hot)
        R = 1024 + 256 * packed.shape[2]
        bad, events = [], 0
        with dash.Engine(nsys, num_procs=N, cache_size=CS, max_instr=packed.shape[2], trace_events=R,
                         schedule_seed=seed) as eng:
            eng.load_traces(packed, lens)
            eng.run()
            dig = eng.read_results()[0]
            for s in range(nsys):
                res, log = run_system(packed[s], lens[s], num_procs=N, cache_size=CS, log=True, log_msgs=True,
                                      arb_seed=seed, log_bytes=1 << 24)
                ev = eng.read_events(s)
                events += len(ev)
                if dash.format_events(ev) != log or int(dig[s]) != res.digest:
                    bad.append(s)
        report["configs"].append({"num_procs": N, "cache_size": CS, "schedule_seed": seed, "block_span": span,
                                  "hot_frac": hot, "max_len": L, "systems": nsys, "events": events,
                                  "mismatched": bad[:8], "n_mismatched": len(bad)})
        report["systems"] += nsys
        report["events"] += events
        report["mismatched_systems"] += len(bad)
        print(f"[{time.time() - t0:.0f}s] cfg {c}: N={N} CS={CS} seed={seed:#x} L={L} events={events} "
              f"mismatched={len(bad)}", flush=True)
    report["seconds"] = time.time() - t0
    print(json.dumps({k: v for k, v in report.items() if k != "configs"}), flush=True)
    if out:
        pathlib.Path(out).write_text(json.dumps(report, indent=1))
    return 1 if report["mismatched_systems"] else 0


if __name__ == "__main__":
    sys.exit(main())
