#!/usr/bin/env python3
"""Point-by-point account of the configs[4] CACHE_SIZE cost from the committed
rocprofv3 PMC summaries of the sweep points (profiles/pmc_sweep_cs<CS>_p0.json, made by
tools/evidence_sweep_pmc.sh + tools/pmc_summary.py) and the engine statistics in each pass's line.

Kernel time per launch = wave-rounds x time per wave-round, and time per wave-round follows
  * the issued VALU + SALU per wave-round: +0.45 % per instruction (padding probes
    measured 0.43-0.49 % per VALU or SALU instruction on this kernel), and
  * the resident waves per CU: 16 instead of 18 costs 6.4 % (profiles/r04/occupancy_vs_fetch:
    the same kernel with 1,540 B of LDS padding, 653.0 / 613.6 ms).
The model's prediction against the measured ratio to CACHE_SIZE 4 is printed per point; the
REPLY_ID fan-out share (the cold INV loop) explains where the extra instructions of
the larger caches come from: P(a wave pops any REPLY_ID in a round) = 1 - (1 - p)^64 with p the
REPLY_ID pops per lane-round.

Usage: python3 tools/sweep_account.py [--dir DIR] [--json out.json]   (DIR holds the summaries; default
profiles/, the final library's; profiles/r05/pmc_sweep/summaries_before_fanout/ holds round 5's first
measurements, before the INV fan-out change)
"""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
PER_INSTR = 0.0045
OCC = {18: 1.0, 16: 653.0 / 613.6}


def point(cs, d):
    prof = json.loads((d / f"pmc_sweep_cs{cs}_p0.json").read_text())
    src = ROOT / prof["source"].split()[0].rstrip("/")
    line = json.loads([x for x in pathlib.Path(str(src) + ".log").read_text().splitlines() if x.startswith("{")][-1])
    if "totals" not in line:  # round-5 compact line: the pass's side file holds the record
        line = json.loads(pathlib.Path(str(src) + ".detail.json").read_text())
    hist, wr = line["totals"]["hist"], line["wave_rounds"]
    rid = hist[4] / (wr * 64)
    waves = prof["waves_per_cu"]
    return {"cache_size": cs, "kernel_ms": prof["kernel_ms"], "wave_rounds": wr,
            "ns_per_wave_round_per_cu": prof["ns_per_wave_round_per_cu"],
            "valu": prof["valu_per_wave_round"], "salu": prof["salu_per_wave_round"],
            "lds": prof["lds_per_wave_round"], "branch": prof.get("branch_per_wave_round"),
            "waves_per_cu": waves, "waves_slots": 18 if waves > 16.8 else 16,
            "lds_bank_conflict_frac": prof["lds_bank_conflict_frac"], "valu_exec_lanes": prof["valu_exec_lanes"],
            "fill_x": prof.get("fill_bytes_per_algorithmic_byte"), "p_wave_rid": 1 - (1 - rid) ** 64,
            "err_frac": line["totals"]["err_systems"] / (1 << 20), "kernel_fingerprint": prof["kernel_fingerprint"]}


def main():
    d = pathlib.Path(sys.argv[sys.argv.index("--dir") + 1]) if "--dir" in sys.argv else ROOT / "profiles"
    pts = {cs: point(cs, d if d.is_absolute() else ROOT / d) for cs in (1, 4, 8, 16)}
    base = pts[4]
    rows = []
    for cs, p in pts.items():
        wr = p["wave_rounds"] / base["wave_rounds"]
        instr = 1 + PER_INSTR * ((p["valu"] + p["salu"]) - (base["valu"] + base["salu"]))
        occ = OCC[p["waves_slots"]] / OCC[base["waves_slots"]]
        model = wr * instr * occ
        meas = p["kernel_ms"] / base["kernel_ms"]
        rows.append(dict(p, ratio_measured=meas, ratio_model=model, f_wave_rounds=wr, f_instr=instr, f_occupancy=occ,
                         residual=meas / model - 1))
    print(f"{'CS':>3} {'ms':>7} {'t/CS4':>6} {'model':>6} {'resid':>6} | {'wr':>6} {'instr':>6} {'occ':>6} | "
          f"{'VALU':>6} {'SALU':>6} {'br':>5} {'waves':>6} {'P(RID)':>6} {'err':>6}")
    for r in rows:
        print(f"{r['cache_size']:>3} {r['kernel_ms']:7.1f} {r['ratio_measured']:6.3f} {r['ratio_model']:6.3f} "
              f"{r['residual']:+6.1%} | {r['f_wave_rounds']:6.3f} {r['f_instr']:6.3f} {r['f_occupancy']:6.3f} | "
              f"{r['valu']:6.1f} {r['salu']:6.1f} {r['branch']:5.1f} {r['waves_per_cu']:6.2f} {r['p_wave_rid']:6.2f} "
              f"{r['err_frac']:6.3f}")
    if "--json" in sys.argv:
        out = pathlib.Path(sys.argv[sys.argv.index("--json") + 1])
        out.write_text(json.dumps({"model": "t/t(CS4) = wave-round ratio x (1 + 0.45 % x extra VALU+SALU per "
                                            "wave-round) x occupancy factor (16 waves: 653.0/613.6)",
                                   "points": rows}, indent=1))


if __name__ == "__main__":
    main()
