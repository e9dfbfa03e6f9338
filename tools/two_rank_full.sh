#!/bin/bash
# The driver's N-GPU line rehearsed at full size on the box's one GPU: `bench.py --gpus 2` over gloo,
# both ranks on the GPU (2 x 2^20 systems, 128 GiB of traces), the default steps of the driver's
# command; the line must certify itself (rank 0's slice [0, 2^20) vs the full-size goldens, both
# ranks' sampled ids). Usage (through gpurun): tools/two_rank_full.sh TAG -> gpurun_out/TAG/
set -uo pipefail
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 1000 python3 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 \
    --detail "$OUT/bench_detail.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "two-rank bench failed"; exit 1; }
wc -c "$OUT/bench.json" "$OUT/bench.err"
