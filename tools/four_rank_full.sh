#!/bin/bash
# The driver's N = 4 line at full size rehearsed on the box's one GPU: `bench.py --gpus 4` over gloo,
# all four ranks on the GPU (4 x 2^20 systems, 256 GiB of traces resident at once); every rank checks
# its whole slice against tests/golden/full_slices.json. Usage (through gpurun): tools/four_rank_full.sh TAG
set -uo pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python3 bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 \
    --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "four-rank bench failed"; exit 1; }
wc -c "$OUT/bench.json" "$OUT/bench.err"
