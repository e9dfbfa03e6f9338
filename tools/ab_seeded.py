#!/usr/bin/env python3
"""Seeded-schedule / event-log A/B (experiments): kernel ms and the digest checksum of one build.

Usage (through gpurun): DASH_LIB=... python3 tools/ab_seeded.py [systems] [steps] [events]
Runs the headline workload shape (8 nodes x 4096 uniform, CACHE_SIZE 4, device generator
seed 0x5EED) under schedule seed 0x5EED5EED, or (events = 1) in lockstep with the DEBUG event
log on (8 x 4096 events per node, as bench_next.py's events row); two builds that simulate the
same schedule must print the same checksum."""
import importlib.util
import json
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("dash", ROOT / "ue22cs343bb1-openmp-assignment_amd" / "dash.py")
dash = importlib.util.module_from_spec(spec)
spec.loader.exec_module(dash)

systems = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
events = len(sys.argv) > 3 and sys.argv[3] == "1"
opts = {"trace_events": 8 * 4096} if events else {"schedule_seed": 0x5EED5EED}
with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=4096, **opts) as eng:
    eng.generate(0x5EED, 4096, kind=dash.GEN_UNIFORM)
    eng.run()
    ks = [eng.run()["kernel_ms"] for _ in range(steps)]
    st = eng.run()
    d = eng.read_results()[0]
    chk = [int((d & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64)), int((d >> np.uint64(32)).sum(dtype=np.uint64))]
print(json.dumps({"kernel_ms": ks, "kernel_ms_avg": sum(ks) / len(ks), "digest_sum": chk,
                  "rounds_total": st["rounds_total"], "instructions": st["instructions"], "hist": st["hist"]}))
