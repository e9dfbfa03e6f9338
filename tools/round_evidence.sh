#!/bin/bash
# Everything a round's profiles/rNN/ holds, on one MI355X (run from the repo root through
# gpurun; about 6 minutes of box time): tools/evidence.sh (GPU suite, headline line with the
# CPU baselines, kernel-trace stats, every PMC pass), then the configs[4] sweep, the SURVEY 8(f)
# rows and the batched host-buffer path.
# Usage: tools/round_evidence.sh TAG      -> gpurun_out/ev_TAG/
set -uo pipefail
TAG=$1; OUT=gpurun_out/ev_$TAG; export TMPDIR=/tmp
bash tools/evidence.sh "$TAG" || exit 1
echo "[$(date +%T)] sweep"
timeout -k 10 600 python3 bench.py --sweep --steps 2 --warmup 1 > "$OUT/sweep.json" 2> "$OUT/sweep.err" || exit 1
echo "[$(date +%T)] next rows"
timeout -k 10 600 python3 bench.py --next --steps 2 > "$OUT/next_rows.json" 2> "$OUT/next_rows.err" || exit 1
echo "[$(date +%T)] host-buffer path"
timeout -k 10 300 python3 bench.py --host-traces --host-native --host-batches 16 --systems 262144 --steps 3 --warmup 1 \
    --no-cpu-baseline > "$OUT/bench_host_native_b16.json" 2> "$OUT/host.err" || exit 1
echo "[$(date +%T)] round-evidence-done"
