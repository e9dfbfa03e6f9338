#!/usr/bin/env python3
"""One launch of the headline kernel for the LDS attribution probe (tools/lds_variants.py,
tools/lds_probe.sh): quarter-size uniform workload (2^18 systems x 8 nodes x 4096, CACHE_SIZE 4,
seed 0x5EED), with a round cap so a variant whose messages go astray still ends. Loads the library
DASH_LIB names. Prints one JSON line: the launch's wave-rounds, kernel time, tier systems, and
whether the totals are the product's (the base variant's must be)."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
CAP = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
REPS = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # launches; the fastest is reported

dash = bench.load_dash()
with dash.Engine(M, num_procs=8, cache_size=4, max_instr=4096, max_rounds=CAP) as eng:
    eng.generate(0x5EED, 4096, kind=dash.GEN_UNIFORM)
    runs = [eng.run() for _ in range(REPS)]
    st = min(runs, key=lambda x: x["kernel_ms"])
    d, r, e = eng.read_results()
print(json.dumps({"lib": str(dash.LIB_PATH.name), "systems": M, "round_cap": CAP, "wave_rounds": st["wave_rounds"],
                  "kernel_ms": st["kernel_ms"], "kernel_ms_all": [x["kernel_ms"] for x in runs], "tier_systems": st["tier_systems"], "rounds_total": st["rounds_total"],
                  "err_systems": st["err_systems"], "roundcap_systems": int(((e & 16) != 0).sum()),
                  "digest_sum": bench.digest_sum(d)}), flush=True)
