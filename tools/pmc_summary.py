"""Per-launch summary of the first-tier sim_kernel from rocprofv3 PMC passes
(FETCH_SIZE, WRITE_SIZE and an SQ pass), written to profiles/pmc_<kind>.json
and read by bench.py for roofline.traffic and valu_issue.

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters); bytes are
reported as measured (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for
16-B-per-lane streaming reads, which this kernel does not do -- its 8-B trace
loads are uncalibrated, so the figure is indicative).
Usage: python tools/pmc_summary.py KIND OUT_JSON DIR [DIR ...]"""
import collections, csv, glob, json, sys

kind, out = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(float)
dur = {}
for d in sys.argv[3:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "sim_kernel<8, 4, 16" not in row["Kernel_Name"]:
                continue
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
            dur[row["Counter_Name"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
res = {"kernel": "dash::sim_kernel<8, 4, 16u>", "workload": kind, "source": " ".join(sys.argv[3:])}
if "FETCH_SIZE" in agg:
    res["fetch_bytes_per_launch"] = agg["FETCH_SIZE"] * 1024
if "WRITE_SIZE" in agg:
    res["write_bytes_per_launch"] = agg["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
    res["hbm_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"):
    if k in agg:
        res[k.lower()] = agg[k]
if "SQ_INSTS_VALU" in agg:
    res["valu_per_launch"] = agg["SQ_INSTS_VALU"]
    res["kernel_ms"] = dur["SQ_INSTS_VALU"]
if len(sys.argv) > 4 and "wave_rounds" in res:
    pass
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
