"""Full-size golden totals of every rank's slice of the driver's 8-GPU layout (round 6): the
oracle (oracle/dash_oracle.c, test infrastructure) over global systems [r * 2^20, (r + 1) * 2^20)
x 8 nodes x 4096 instructions, CACHE_SIZE 4, seed 0x5EED, for slices r = 1..7 of the headline
workloads (BASELINE.json configs[2] uniform, configs[3] contention). Slice 0 is
tests/golden/full_size.json. With these, every rank of a bench.py line at 2^20 systems per GPU
checks its own whole slice (bench.slice_golden, the counters ride in the one all-reduce), so an
N-GPU line certifies all N x 2^20 systems, not rank 0's alone.

Writes tests/golden/full_slices.json {"<kind>": {"<r>": totals}} after every slice (a long run
keeps what it did; existing slices are kept unless recomputed).
Usage: python tests/golden/make_full_slices.py [--out FILE] [threads] [kind@r ...]   (about 27 min per
slice on 7 threads; default: uniform 1..7, then contention 1..7; --out writes another file, merged
into this one by hand: the contention slices were computed on the GPU box's 16 host CPUs). kind is
uniform, contention or a configs[4] point locality:<CS>:<p> (bench.golden_key), e.g. locality:16:0.5@1
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
KINDS = {"uniform": 0, "contention": 1}


def workload(kind):
    """(generator kind, CACHE_SIZE, locality fixed-point) of a fixture key: "uniform", "contention"
    or a configs[4] point "locality:<CS>:<p>" (bench.golden_key)."""
    if kind.startswith("locality:"):
        _, cs, p = kind.split(":")
        return 2, int(cs), int(round(float(p) * 65536))
    return KINDS[kind], CS, 0


def totals(kind, r, threads):
    hist = np.zeros(13, dtype=np.uint64)
    instr = rounds = errsys = 0
    lo = hi = 0
    t0 = time.time()
    base = r * SYSTEMS
    gen, cs, loc = workload(kind)
    for first in range(base, base + SYSTEMS, CHUNK):
        res = oc.run_batch(SEED, first, CHUNK, num_procs=8, cache_size=cs, length=LEN, kind=gen, locality=loc,
                           threads=threads)
        hist += res["hist"]
        instr += res["instructions"]
        rounds += int(res["rounds"].astype(np.uint64).sum())
        errsys += int((res["errors"] != 0).sum())
        a, b = bench.digest_sum(res["digests"])
        lo, hi = lo + a, hi + b
        print(f"{kind} slice {r}: {first + CHUNK - base}/{SYSTEMS} systems, {time.time() - t0:.0f} s", flush=True)
    return {"hist": [int(x) for x in hist], "instructions": instr, "rounds_total": rounds,
            "err_systems": errsys, "digest_sum": [lo, hi]}


if __name__ == "__main__":
    argv = sys.argv[1:]
    path = pathlib.Path(__file__).resolve().parent / "full_slices.json"
    if argv[:1] == ["--out"]:  # another file (e.g. under gpurun_out/ when run on a bigger host)
        path, argv = pathlib.Path(argv[1]), argv[2:]
    threads = int(argv[0]) if argv else 8
    # kind@r, e.g. uniform@3 or locality:16:0.5@1
    todo = [(a.rsplit("@", 1)[0], int(a.rsplit("@", 1)[1])) for a in argv[1:]] or \
        [(k, r) for k in ("uniform", "contention") for r in range(1, 8)]
    out = json.loads(path.read_text()) if path.exists() else {
        "systems_per_slice": SYSTEMS, "num_procs": 8, "instr_per_node": LEN, "cache_size": CS, "seed": SEED,
        "generator": "oracle/dash_oracle.c orc_run_batch (counter-based, keyed by global system id); slice r = "
                     "global systems [r * 2^20, (r + 1) * 2^20); slice 0 is full_size.json",
        "uniform": {}, "contention": {}}
    for kind, r in todo:
        out.setdefault(kind, {})[str(r)] = totals(kind, r, threads)
        path.write_text(json.dumps(out, indent=1) + "\n")
        print(f"wrote {path} ({kind} slice {r})", flush=True)
