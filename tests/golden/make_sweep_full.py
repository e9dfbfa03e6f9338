"""Full-size golden totals for points of BASELINE.json configs[4] (the CACHE_SIZE x
locality sweep; all 25 points are committed since round 6, the file lists them): the oracle (oracle/dash_oracle.c, test infrastructure) run over ALL 2^20
systems x 8 nodes x 4096 instructions of the locality generator, seed 0x5EED, at
  CACHE_SIZE 1, locality 0.0;  CACHE_SIZE 4, locality 0.5;  CACHE_SIZE 16, locality 1.0
(the corners and the middle of the grid; round 4) and, since round 5, CACHE_SIZE 8, locality 0.0
and CACHE_SIZE 16, locality 0.25 (the kernels round 5 changed: the 2-instruction trace window at
CACHE_SIZE 8, the INV fan-out everywhere; 16 / 0.25 has the most REPLY_ID fan-outs and the most
systems on the reference's undefined paths); later in round 5 more points one at a time
(`make_sweep_full.py 8 CS:P ...`); round 6 the last two, CACHE_SIZE 2 and 16 at locality 0 (about
30 min each on 7 threads). Writes tests/golden/sweep_full.json: per point the
per-type histogram, instruction / round / error-system totals and bench.digest_sum of the
per-system digests, so the `sweep` object of the default bench.py line (1M systems per GPU
per point) is checked bit-exactly against the oracle: tests/test_full_size_golden.py
(committed lines) and tests/test_gpu_sweep.py (live, on the GPU box).

Usage: python tests/golden/make_sweep_full.py [threads] [CS:P ...]   (about 10 min per point on 8
threads; with points given, only those are computed and merged into the existing file)
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

SYSTEMS, LEN, SEED, CHUNK = 1 << 20, 4096, 0x5EED, 1 << 15
POINTS = [(1, 0.0), (4, 0.5), (16, 1.0), (8, 0.0), (16, 0.25)]  # the default set; more are added by CS:P


def totals(cs, p, threads):
    loc = int(round(p * 65536))
    hist = np.zeros(13, dtype=np.uint64)
    instr = rounds = errsys = 0
    lo = hi = 0
    t0 = time.time()
    for first in range(0, SYSTEMS, CHUNK):
        r = oc.run_batch(SEED, first, CHUNK, num_procs=8, cache_size=cs, length=LEN, kind=2, locality=loc,
                         threads=threads)
        hist += r["hist"]
        instr += r["instructions"]
        rounds += int(r["rounds"].astype(np.uint64).sum())
        errsys += int((r["errors"] != 0).sum())
        a, b = bench.digest_sum(r["digests"])
        lo, hi = lo + a, hi + b
        print(f"CS {cs} locality {p}: {first + CHUNK}/{SYSTEMS} systems, {time.time() - t0:.0f} s", flush=True)
    return {"cache_size": cs, "locality": p, "hist": [int(x) for x in hist], "instructions": instr,
            "rounds_total": rounds, "err_systems": errsys, "digest_sum": [lo, hi]}


if __name__ == "__main__":
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    only = [(int(a.split(":")[0]), float(a.split(":")[1])) for a in sys.argv[2:]]
    path = pathlib.Path(__file__).resolve().parent / "sweep_full.json"
    out = {"systems": SYSTEMS, "num_procs": 8, "instr_per_node": LEN, "seed": SEED, "generator":
           "oracle/dash_oracle.c orc_run_batch, locality kind (counter-based, keyed by global system id)",
           "points": []}
    if path.exists():  # always merge: a run never drops points it did not compute
        out = json.loads(path.read_text())
    for cs, p in (only or POINTS):
        pt = totals(cs, p, threads)
        out["points"] = [q for q in out["points"] if (q["cache_size"], q["locality"]) != (cs, p)] + [pt]
        path.write_text(json.dumps(out, indent=1) + "\n")  # after every point: a long run keeps what it did
        print(f"wrote {path} ({len(out['points'])} points)", flush=True)
