"""Golden totals for BASELINE.json configs[4] (the CACHE_SIZE x locality sweep), at a reduced
but non-trivial size: 4096 systems x 8 nodes x 4096 instructions per grid point, seed 0x5EED,
CACHE_SIZE in {1,2,4,8,16} x locality p in {0, 0.25, 0.5, 0.75, 1} (w.p. p an instruction's
home node is the issuing node, else uniform over the others; DESIGN.md §5 generator spec).
The oracle (oracle/dash_oracle.c, test infrastructure) runs every point; tests/golden/sweep.json
keeps per point the per-type histogram, instruction / round / error-system / drop totals and
bench.digest_sum of the per-system state digests. tests/test_gpu_sweep.py runs all 25 points
through dash_generate + dash_run on the GPU and compares; tests/test_oracle_sweep.py re-derives
three points on the CPU. The grid exercises cacheIndex = blockIndex % CACHE_SIZE
(assignment.c:7,188,659) at CS = 1..16.

Usage: python tests/golden/make_sweep.py [threads]   (~2 min on 8 host threads)
"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (digest_sum)
import oracle_ctypes as oc  # noqa: E402

SYSTEMS, LEN, SEED = 4096, 4096, 0x5EED
CACHE_SIZES = (1, 2, 4, 8, 16)
LOCALITIES = (0.0, 0.25, 0.5, 0.75, 1.0)
GEN_LOCALITY = 2


def point(cs, p, threads, systems=SYSTEMS):
    r = oc.run_batch(SEED, 0, systems, num_procs=8, cache_size=cs, length=LEN, kind=GEN_LOCALITY,
                     locality=int(round(p * 65536)), threads=threads)
    return {"cache_size": cs, "locality": p, "hist": [int(x) for x in r["hist"]],
            "instructions": r["instructions"], "rounds_total": int(r["rounds"].astype(np.uint64).sum()),
            "err_systems": int((r["errors"] != 0).sum()), "digest_sum": bench.digest_sum(r["digests"])}


if __name__ == "__main__":
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    pts, t0 = [], time.time()
    for cs in CACHE_SIZES:
        for p in LOCALITIES:
            pts.append(point(cs, p, threads))
            print(f"CS={cs} p={p}: {time.time() - t0:.0f} s", flush=True)
    out = {"systems": SYSTEMS, "num_procs": 8, "instr_per_node": LEN, "seed": SEED,
           "generator": "locality (kind 2), oracle/dash_oracle.c orc_run_batch", "points": pts}
    f = pathlib.Path(__file__).resolve().parent / "sweep.json"
    f.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {f}")
