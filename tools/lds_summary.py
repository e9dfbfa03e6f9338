#!/usr/bin/env python3
"""Summary of tools/lds_probe.sh: per variant, the first-tier headline kernel's
(sim_kernel<8, 4, 16u, 0>) LDS counters per wave-round from its --pmc pass, its bank-conflict
share of LDS-active cycles, and the fastest of three timed launches; deltas against `base`.
Usage: python3 tools/lds_summary.py [name ...]  (reads gpurun_out/lds/)"""
import collections
import csv
import glob
import json
import sys

KERNEL = "sim_kernel<8, 4, 16u, 0>"
OUT = "gpurun_out/lds"


def counters(name):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{OUT}/{name}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def last_json(path):
    return json.loads([ln for ln in open(path) if ln.startswith("{")][-1])


def main(names):
    rows = {}
    for n in names:
        c = counters(n)
        p = last_json(f"{OUT}/{n}.pmc.json")
        t = last_json(f"{OUT}/{n}.time.json")
        wr = max(p["wave_rounds"], 1)
        rows[n] = {"kernel_ms": t["kernel_ms"], "kernel_ms_all": t["kernel_ms_all"], "wave_rounds": t["wave_rounds"],
                   "roundcap_systems": t["roundcap_systems"], "digest_sum": t["digest_sum"],
                   "lds_bank_conflict_per_wr": c.get("SQ_LDS_BANK_CONFLICT", 0) / wr,
                   "lds_idx_active_per_wr": c.get("SQ_LDS_IDX_ACTIVE", 0) / wr,
                   "lds_insts_per_wr": c.get("SQ_INSTS_LDS", 0) / wr,
                   "wait_inst_lds_per_wr": c.get("SQ_WAIT_INST_LDS", 0) / wr,
                   "valu_per_wr": c.get("SQ_INSTS_VALU", 0) / wr,
                   "conflict_frac": (c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
                                     if c.get("SQ_LDS_IDX_ACTIVE") else None),
                   "ns_per_wave_round": t["kernel_ms"] * 1e6 / max(t["wave_rounds"], 1)}
    base = rows.get("base")
    if base:
        for n, r in rows.items():
            r["conflict_delta_per_wr"] = r["lds_bank_conflict_per_wr"] - base["lds_bank_conflict_per_wr"]
            r["conflict_share_removed"] = (-r["conflict_delta_per_wr"] / base["lds_bank_conflict_per_wr"]
                                           if base["lds_bank_conflict_per_wr"] else None)
            r["time_per_wr_vs_base"] = r["ns_per_wave_round"] / base["ns_per_wave_round"]
    print(json.dumps({"kernel": KERNEL, "workload": "2^18 systems x 8 nodes x 4096 uniform, CACHE_SIZE 4, seed 0x5EED, "
                      "round cap 65536", "variants": rows}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:] or ["base", "ring", "arrive", "hist", "window", "swizzle"])
