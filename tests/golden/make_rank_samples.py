"""Per-system golden results at sampled global system ids, for every workload bench.py times
(BASELINE.json configs[2] uniform, configs[3] contention, the 25 points of configs[4]), so that
EVERY rank of an N-GPU bench run can check its own slice, not only rank 0 (whose slice
[0, 2^20) the full-size totals of full_size.json / sweep_full.json cover). VERDICT r5 next #1.

The oracle (oracle/dash_oracle.c, test infrastructure) runs each sampled system alone: 8 nodes x
4096 instructions, seed 0x5EED, traces keyed by the global system id exactly as the GPU
generator keys them. Sampled ids:
  * "high": 16 per rank slice [r*2^20, (r+1)*2^20) for r < 8 (the driver's 1/2/4/8-GPU runs at
    2^20 systems per GPU), spread over the slice;
  * "low": every 61st id below 7808, so small rehearsals (a few hundred systems per rank,
    tests/test_gpu_distributed.py) also hold samples on every rank.
Writes tests/golden/rank_samples.json: per workload the digest (hex), lockstep rounds and error
bits of each sampled id (parallel lists in the order of "ids").

Usage: python tests/golden/make_rank_samples.py   (about 1-2 min)
"""
import json
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ctypes as oc  # noqa: E402

SEED, LEN, PER_RANK = 0x5EED, 4096, 1 << 20
LOW = [k * 61 for k in range(128)]
HIGH = [r * PER_RANK + k * 65536 + (k * 7919) % 65536 for r in range(8) for k in range(16)]
IDS = sorted(set(LOW) | set(HIGH))
GRID = [(cs, p) for cs in (1, 2, 4, 8, 16) for p in (0.0, 0.25, 0.5, 0.75, 1.0)]


def workloads():
    """(key, cache_size, generator kind, locality fixed-point) -- the keys bench.py looks up."""
    yield "uniform", 4, 0, 0
    yield "contention", 4, 1, 0
    for cs, p in GRID:
        yield f"locality:{cs}:{p:g}", cs, 2, int(round(p * 65536))


def main():
    out = {"seed": SEED, "instr_per_node": LEN, "num_procs": 8, "systems_per_rank": PER_RANK,
           "generator": "oracle/dash_oracle.c orc_run_batch, one system per call (keyed by global id)",
           "ids": IDS, "workloads": {}}
    t0 = time.time()
    for key, cs, kind, loc in workloads():
        d, r, e = [], [], []
        for g in IDS:
            res = oc.run_batch(SEED, g, 1, num_procs=8, cache_size=cs, length=LEN, kind=kind, locality=loc)
            d.append(f"{int(res['digests'][0]):016x}")
            r.append(int(res["rounds"][0]))
            e.append(int(res["errors"][0]))
        out["workloads"][key] = {"cache_size": cs, "digest": d, "rounds": r, "errors": e}
        print(f"{key}: {len(IDS)} systems, {time.time() - t0:.0f} s", flush=True)
    path = pathlib.Path(__file__).resolve().parent / "rank_samples.json"
    path.write_text(json.dumps(out, separators=(",", ":")) + "\n")
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
