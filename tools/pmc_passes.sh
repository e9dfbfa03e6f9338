#!/bin/bash
# PMC passes over a reduced bench workload (one rocprofv3 run per pass, each
# under its own time limit). Usage: tools/pmc_passes.sh TAG [bench args]
set -uo pipefail
TAG=${1:-pmc}; shift || true
ARGS=${*:-"--systems 131072 --steps 1 --warmup 0 --no-cpu-baseline"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py $ARGS > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; exit 1; }
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
echo pmc-done
