#!/bin/bash
# LDS bank-conflict attribution on one MI355X: for each variant of
# tools/lds_variants.py (tools/var_r6/libdash_lds_<name>.so), a timing run (3 launches, the fastest
# kept) and one rocprofv3 --pmc pass of the LDS counters, quarter-size uniform headline
# (tools/lds_probe.py); then tools/lds_summary.py -> gpurun_out/lds/summary.json.
# Usage (through gpurun, from the repo root): tools/lds_probe.sh [name ...]
set -uo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/lds; mkdir -p "$OUT"
NAMES=${*:-base ring arrive hist window swizzle}
for n in $NAMES; do
  echo "[$(date +%T)] $n"
  DASH_LIB=$PWD/tools/var_r6/libdash_lds_$n.so timeout -k 10 120 python3 tools/lds_probe.py 262144 65536 3 \
      > "$OUT/$n.time.json" 2> "$OUT/$n.time.err" || { echo "$n timing failed"; exit 1; }
  DASH_LIB=$PWD/tools/var_r6/libdash_lds_$n.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT \
      SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU \
      --kernel-trace --output-format csv -d "$OUT/$n" -o run -- python3 tools/lds_probe.py 262144 65536 1 \
      > "$OUT/$n.pmc.json" 2> "$OUT/$n.pmc.err" || { echo "$n pmc failed"; exit 1; }
done
python3 tools/lds_summary.py $NAMES > "$OUT/summary.json" && cat "$OUT/summary.json"
