#!/bin/bash
# rocprofv3 PMC passes, one counter group per rocprofv3 run (separate --pmc passes, each under its
# own time limit), each pass's bench record in its own side file (DIR.detail.json) for
# tools/pmc_summary.py. Points: "CS:P" = a configs[4] point (full-size locality traces at that
# CACHE_SIZE and locality), "uniform" / "contention" = BASELINE configs[2] / [3].
# Usage: tools/evidence_sweep_pmc.sh TAG "CS:P ... uniform contention"  -> gpurun_out/sw_TAG/<point>/
set -uo pipefail
TAG=$1; POINTS=${2:-"16:0 1:0 4:0 8:0"}
OUT=gpurun_out/sw_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
for pt in $POINTS; do
  case "$pt" in
    uniform|contention) D="$OUT/pmc_$pt"; ARGS="--kind $pt" ;;
    *) cs=${pt%%:*}; p=${pt##*:}; D="$OUT/cs${cs}_p${p}"; ARGS="--kind locality --locality $p --cache-size $cs" ;;
  esac
  mkdir -p "$D"
  pass() {  # name counters...
    local name=$1; shift
    step "$pt pass $name"
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$D/$name" -o run -- \
        python3 bench.py $ARGS --steps 1 --warmup 0 \
        --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off --detail "$D/$name.detail.json" \
        > "$D/$name.log" 2>&1 || { echo "pass $name failed"; exit 1; }
  }
  pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
  pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
  pass sq3 SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_CYCLES
  pass sq4 SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD
  pass tcc1 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
  pass tcc2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_REQ_sum
  pass write WRITE_SIZE
done
step evidence-done
