#!/bin/bash
# Instruction-mix counters of kernel variants (one rocprofv3 --pmc pass each, quarter-size
# uniform headline). Usage (through gpurun): tools/ab_pmc.sh NAME [NAME...]
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
for n in "$@"; do
  DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAIT_ANY --kernel-trace --output-format csv \
      -d gpurun_out/abp/$n -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --systems 262144 \
      --contention-steps 0 > gpurun_out/abp/$n.log 2>&1 || { echo "$n pmc failed"; exit 1; }
  python3 - "$n" <<'PY'
import csv, glob, sys, collections, json
n = sys.argv[1]
agg = collections.defaultdict(float); dur = 0
for f in glob.glob(f"gpurun_out/abp/{n}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("sim_kernel<8, 4, 16u, false>", "sim_kernel<8, 4, 16u, 0>")):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
wr = json.load(open(f"gpurun_out/abp/{n}.log".replace(".log", ".log")) if False else None) if False else None
line = [l for l in open(f"gpurun_out/abp/{n}.log") if l.startswith("{")]
w = json.loads(line[-1])["wave_rounds"] if line else 1
print(f"{n:8s} {dur:7.2f} ms  per wave-round: " + "  ".join(f"{k.replace('SQ_', '')} {v / w:.1f}" for k, v in sorted(agg.items())))
PY
done
