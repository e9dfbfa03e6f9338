#!/bin/bash
# Timing only (no parity): quarter-size headline kernel ms of probe variants, alternating.
# Usage (through gpurun): tools/ab_time.sh NAME [NAME...]
set -uo pipefail
mkdir -p gpurun_out/ab
for r in $(seq ${ROUNDS:-2}); do
  for n in "$@"; do
    DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 120 python3 bench.py --systems ${SYSTEMS:-262144} --steps 3 --warmup 1 \
        --no-cpu-baseline --contention-steps 0 > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.err || { echo "$n bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/$n.$r.json'));print('%-8s r%d kernel %.2f ms'%('$n',$r,d['kernel_ms_avg']))"
  done
done
