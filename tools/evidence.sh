#!/bin/bash
# Round evidence on one MI355X (run from the repo root): GPU parity suite, default bench
# (with CPU baseline), contention bench, rocprofv3 kernel-trace stats of the bench command,
# and one rocprofv3 PMC pass per counter group (full-size workload, 1 step each).
# Usage: tools/evidence.sh TAG        -> gpurun_out/ev_TAG/
set -uo pipefail
TAG=$1; OUT=gpurun_out/ev_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 \
  || { tail -20 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
step bench "(headline line: uniform + contention + CPU baselines)"
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 > "$OUT/bench_uniform.json" 2> "$OUT/bench_uniform.err" || exit 1
step kernel trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --contention-steps 2 > "$OUT/trace.log" 2>&1 || exit 1
step kernel trace, uniform launches only "(the headline kernel's own average)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_uniform" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --contention-steps 0 > "$OUT/trace_uniform.log" 2>&1 || exit 1
pmc() {  # kind name counters...
  local kind=$1 name=$2; shift 2
  step pmc "$kind" "$name"
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$OUT/pmc_$kind/$name" -o run -- \
      python3 bench.py --kind "$kind" --steps 1 --warmup 0 --no-cpu-baseline --contention-steps 0 > "$OUT/pmc_$kind/$name.log" 2>&1 \
      || { echo "pmc $name failed"; exit 1; }
}
for kind in uniform contention; do
  mkdir -p "$OUT/pmc_$kind"
  pmc $kind sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
  pmc $kind fetch FETCH_SIZE
  pmc $kind write WRITE_SIZE
  pmc $kind sq3 SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_CYCLES
done
for kind in ${SQ2_KINDS:-uniform contention}; do
  pmc $kind sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
  pmc $kind tcc1 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  pmc $kind tcc2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum
done
step evidence-done
