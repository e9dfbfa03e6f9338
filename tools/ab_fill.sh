#!/bin/bash
# L2 -> fabric read requests (128-B fills) of kernel variants at one configs[4] point, quarter size:
# one rocprofv3 --pmc pass per variant (TCC_EA0_RDREQ_128B), next to tools/ab_cs.sh's timing.
# Usage (through gpurun): CS=8 LOC=0 tools/ab_fill.sh NAME [NAME...]
set -uo pipefail
mkdir -p gpurun_out/ab_fill; export TMPDIR=/tmp
CS=${CS:-8}; LOC=${LOC:-0}
for n in "$@"; do
  D=gpurun_out/ab_fill/${n}_cs${CS}_p${LOC}
  DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_128B_sum TCC_REQ_sum \
      --kernel-trace --output-format csv -d "$D" -o run -- python3 bench.py --kind locality --locality $LOC \
      --cache-size $CS --systems ${SYSTEMS:-262144} --steps 1 --warmup 0 --no-cpu-baseline --contention-steps 0 \
      --line-sweep off --line-next off --detail "$D.detail.json" > "$D.log" 2>&1 || { echo "$n pmc failed"; exit 1; }
  python3 - "$D" "$n" <<PY
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))
        if "sim_kernel<8, $CS, 16u, 0>" in r["Kernel_Name"]]
grid = max(int(r["Grid_Size"]) for r in rows)
first = min(int(r["Dispatch_Id"]) for r in rows if int(r["Grid_Size"]) == grid)
v = {}
for r in rows:
    if int(r["Dispatch_Id"]) == first:
        v[r["Counter_Name"]] = v.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
print("%-8s CS $CS p $LOC fills %.1f GB, L2 requests %.3g" % (sys.argv[2], v["TCC_EA0_RDREQ_128B_sum"] * 128 / 1e9, v["TCC_REQ_sum"]))
PY
done
