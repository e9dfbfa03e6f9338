#!/usr/bin/env python3
"""Micro-step schedule campaign on one MI355X (test infrastructure; tests/micro_fuzz.py does the
check): random (num_procs, cache_size) configurations, random traces, one random STRICT-model
interleaving per system, engine through dash_set_micro_schedule vs the oracle's final state.
Usage: python3 tools/diag/micro_campaign.py [configs] [systems] [maxlen] OUT.json"""
import json
import pathlib
import sys
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import micro_fuzz  # noqa: E402
from test_gpu_parity import random_batch  # noqa: E402


def main():
    ncfg = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    nsys = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    maxlen = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    out = sys.argv[4] if len(sys.argv) > 4 else None
    dash = bench.load_dash()
    rng = np.random.default_rng(0x3C3C)
    rep = {"configs": [], "systems": 0, "mismatched_systems": 0, "skipped_model_overflow": 0}
    t0 = time.time()
    for c in range(ncfg):
        N = int(rng.integers(1, 9))
        CS = int(rng.choice([1, 2, 3, 4, 5, 8, 16]))
        L = int(rng.integers(1, maxlen + 1))
        bad, skipped = micro_fuzz.one_config(dash, rng, N, CS, nsys, L, random_batch)
        rep["configs"].append({"num_procs": N, "cache_size": CS, "max_len": L, "systems": nsys,
                               "mismatched": bad[:8], "n_mismatched": len(bad), "skipped": skipped})
        rep["systems"] += nsys - len(skipped)
        rep["mismatched_systems"] += len(bad)
        rep["skipped_model_overflow"] += len(skipped)
        print(f"[{time.time() - t0:.0f}s] cfg {c}: N={N} CS={CS} L={L} mismatched={len(bad)} skipped={len(skipped)}",
              flush=True)
    rep["seconds"] = time.time() - t0
    print(json.dumps({k: v for k, v in rep.items() if k != "configs"}), flush=True)
    if out:
        pathlib.Path(out).write_text(json.dumps(rep, indent=1))
    return 1 if rep["mismatched_systems"] else 0


if __name__ == "__main__":
    sys.exit(main())
