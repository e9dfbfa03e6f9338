#!/bin/bash
# Round-6 evidence on one MI355X (run from the repo root): the GPU test suite, the driver's bench
# command (its printed line, stderr and side file kept separately, so their sizes are what the
# driver sees), and rocprofv3 --kernel-trace --stats of the headline's uniform launches.
# Usage: tools/evidence_r6.sh TAG   -> gpurun_out/ev6_TAG/      (SKIP_TESTS=1 / SKIP_TRACE=1)
set -uo pipefail
TAG=$1; OUT=gpurun_out/ev6_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step gpu tests
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
      > "$OUT/gpu_tests.txt" 2>&1 || { echo "gpu tests failed"; exit 1; }
  step smoke
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || exit 1
fi
step bench "(the driver's command)"
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
cp gpurun_out/bench_detail.json "$OUT/bench_detail.json"
wc -c "$OUT/bench.json" "$OUT/bench.err"
if [ -z "${SKIP_TRACE:-}" ]; then
  step kernel trace, uniform launches only
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_uniform" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off \
      --detail "$OUT/trace_uniform_detail.json" > "$OUT/trace_uniform.log" 2>&1 || exit 1
fi
if [ -n "${DEFAULT_STATS:-}" ]; then
  step "rocprofv3 --kernel-trace --stats of the whole default command"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/default_cmd_stats" -o run -- \
      python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail "$OUT/default_cmd_stats_detail.json" \
      > "$OUT/default_cmd_stats.json" 2> "$OUT/default_cmd_stats.err" || exit 1
fi
step evidence-done
