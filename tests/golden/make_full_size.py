"""Full-size golden totals for the headline workloads (BASELINE.json configs[2] and [3]):
the oracle (oracle/dash_oracle.c, test infrastructure) run over ALL 2^20 systems x 8 nodes x
4096 instructions, CACHE_SIZE 4, seed 0x5EED, for the uniform and contention generators.
Writes tests/golden/full_size.json: per kind the per-type histogram, instruction / round /
error-system totals and bench.digest_sum of the per-system state digests, so
tests/test_gpu_parity.py::test_full_size_totals_match_oracle can check the GPU's whole
headline run bit-exactly on the box without re-running the oracle there (≈10 min per kind
on 8 host threads).

Usage: python tests/golden/make_full_size.py [threads]
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

SYSTEMS, LEN, SEED, CS, CHUNK = 1 << 20, 4096, 0x5EED, 4, 1 << 15


def totals(kind, threads):
    hist = np.zeros(13, dtype=np.uint64)
    instr = rounds = errsys = 0
    lo = hi = 0
    t0 = time.time()
    for first in range(0, SYSTEMS, CHUNK):
        r = oc.run_batch(SEED, first, CHUNK, num_procs=8, cache_size=CS, length=LEN, kind=kind,
                         threads=threads)
        hist += r["hist"]
        instr += r["instructions"]
        rounds += int(r["rounds"].astype(np.uint64).sum())
        errsys += int((r["errors"] != 0).sum())
        a, b = bench.digest_sum(r["digests"])
        lo, hi = lo + a, hi + b
        print(f"kind {kind}: {first + CHUNK}/{SYSTEMS} systems, {time.time() - t0:.0f} s", flush=True)
    return {"hist": [int(x) for x in hist], "instructions": instr, "rounds_total": rounds,
            "err_systems": errsys, "digest_sum": [lo, hi]}


if __name__ == "__main__":
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    out = {"systems": SYSTEMS, "num_procs": 8, "instr_per_node": LEN, "cache_size": CS, "seed": SEED,
           "generator": "oracle/dash_oracle.c orc_run_batch (counter-based, keyed by global system id)",
           "uniform": totals(0, threads), "contention": totals(1, threads)}
    p = pathlib.Path(__file__).resolve().parent / "full_size.json"
    p.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {p}")
