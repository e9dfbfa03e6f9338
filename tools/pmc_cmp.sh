#!/bin/bash
# Two SQ passes (LDS pipeline + instruction mix) for one bench configuration.
# Usage: tools/pmc_cmp.sh TAG [bench args]
set -uo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 $BARGS > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }; }
BARGS="$*"
run a SQ_WAIT_INST_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_BRANCH SQ_IFETCH SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS
run c SQ_LDS_ATOMIC_RETURN SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES
echo done
