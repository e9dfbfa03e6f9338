"""Sum rocprofv3 counter CSVs of one pmc_cmp/pmc_passes directory for the first-tier
simulation kernel (sim_kernel<8, 4, ...> or swar_kernel<4, ...>)."""
import collections, csv, glob, sys
for d in sys.argv[1:]:
    agg = collections.defaultdict(float); dur = {}
    for f in glob.glob(f"{d}/*/run_counter_collection.csv") + glob.glob(f"{d}/run_counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if ("sim_kernel" in name and "8, 4" in name) or ("swar_kernel" in name and "<4" in name):
                agg[row["Counter_Name"]] += float(row["Counter_Value"])
                dur[f] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
    print(d, "kernel ms", sorted(set(round(v, 1) for v in dur.values())))
    for k, v in sorted(agg.items()):
        print(f"  {k:28s} {v:.4g}")
