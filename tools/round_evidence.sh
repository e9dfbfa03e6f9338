#!/bin/bash
# Round evidence on one MI355X: default bench (with CPU baseline), contention bench,
# rocprofv3 kernel-trace stats of the bench command, FETCH_SIZE / WRITE_SIZE passes.
# Usage: tools/round_evidence.sh TAG
set -uo pipefail
TAG=$1; OUT=gpurun_out/ev_$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > "$OUT/bench_uniform.json" 2> "$OUT/bench_uniform.err" || exit 1
echo "uniform done"
timeout -k 10 300 python3 bench.py --kind contention --no-cpu-baseline > "$OUT/bench_contention.json" 2>/dev/null || exit 1
echo "contention done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/trace.log" 2>&1 || exit 1
echo "trace done"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/write.log" 2>&1 || exit 1
echo evidence-done
