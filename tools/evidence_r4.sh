#!/bin/bash
# Round-4 evidence on one MI355X (run from the repo root): the driver's bench command, rocprofv3
# kernel-trace stats of the headline (uniform launches only) and of the event-log row, and one
# rocprofv3 PMC pass per counter group (full-size workload, 1 step each, no line sweep), each
# pass's bench line carrying its `box` (tools/pmc_summary.py records them).
# Usage: tools/evidence_r4.sh TAG   -> gpurun_out/ev_TAG/
set -uo pipefail
TAG=$1; OUT=gpurun_out/ev_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ -z "${SKIP_BENCH:-}" ]; then
  step bench "(the driver's command)"
  timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
fi
step kernel trace, uniform launches only
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_uniform" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off > "$OUT/trace_uniform.log" 2>&1 || exit 1
pmc() {  # kind name counters...
  local kind=$1 name=$2; shift 2
  step pmc "$kind" "$name"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$kind/$name" -o run -- \
      python3 bench.py --kind "$kind" --steps 1 --warmup 0 --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off \
      > "$OUT/pmc_$kind/$name.log" 2>&1 || { echo "pmc $name failed"; exit 1; }
}
for kind in ${PMC_KINDS:-uniform contention}; do
  mkdir -p "$OUT/pmc_$kind"
  pmc $kind sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
  pmc $kind fetch FETCH_SIZE
  pmc $kind write WRITE_SIZE
  pmc $kind sq3 SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_CYCLES
  pmc $kind sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
  pmc $kind tcc1 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  pmc $kind tcc2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum
done
step evidence-done
