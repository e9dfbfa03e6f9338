#!/bin/bash
# One SQ pass (instruction mix) on a 262144-system uniform run. Usage: tools/quick_pmc.sh TAG
set -uo pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH \
  --kernel-trace --output-format csv -d "$OUT/q" -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --systems 262144 > "$OUT/q.log" 2>&1 || exit 1
python3 tools/pmc_sum.py "$OUT"
