#!/bin/bash
# rocprofv3 passes for the bench workload (run on the GPU box from the repo root).
#   1) kernel trace + stats (per-kernel average duration)
#   2) PMC: FETCH_SIZE      3) PMC: WRITE_SIZE      4) PMC: SQ instruction mix
# Output under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
set -euo pipefail
TAG=${1:-r01}
ARGS=${2:-"--steps 2 --warmup 1 --no-cpu-baseline"}
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/bench_fetch.log" 2>&1
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/bench_write.log" 2>&1
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/sq" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/bench_sq.log" 2>&1
fi
echo done
