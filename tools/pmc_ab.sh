#!/bin/bash
# SQ instruction-mix pass for both first-tier kernels (swar_kernel, then sim_kernel via
# DASH_KERNEL=lane) on a 262144-system uniform run. Usage: tools/pmc_ab.sh TAG
set -uo pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/swar" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --systems 262144 > "$OUT/swar.log" 2>&1 || exit 1
DASH_KERNEL=lane timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d "$OUT/lane" -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --systems 262144 > "$OUT/lane.log" 2>&1 || exit 1
python3 tools/pmc_sum.py "$OUT/swar" "$OUT/lane"
