#!/bin/bash
# Kernel-time screen of headline-only variant builds (tools/variants/libdash_NAME.so, no parity
# subset: build flags that only change instruction scheduling). Usage: tools/sched_screen.sh NAME...
set -uo pipefail
mkdir -p gpurun_out/var
for n in "$@"; do
  DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 120 python3 bench.py --systems 262144 --steps 3 --warmup 1 \
      --no-cpu-baseline --contention-steps 0 > gpurun_out/var/$n.json 2> gpurun_out/var/$n.err || { echo "$n: bench failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var/$n.json'));print('%-12s kernel %.1f ms %s'%('$n', d['kernel_ms_avg'], d['kernel_ms_steps']))"
done
