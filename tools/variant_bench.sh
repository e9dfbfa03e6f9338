#!/bin/bash
# For each tools/variants/libdash_*.so (or the names given): quick GPU parity subset, then
# bench.py at a quarter of the headline workload. Usage: tools/variant_bench.sh [NAME...]
set -uo pipefail
mkdir -p gpurun_out/var
names=("$@")
[ ${#names[@]} -eq 0 ] && names=($(ls tools/variants | sed -n 's/^libdash_\(.*\)\.so$/\1/p'))
for n in "${names[@]}"; do
  lib=$PWD/tools/variants/libdash_$n.so
  DASH_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "${VB_K:-random_traces or generator or contention or tiers or seeded_schedule_bit or long_traces or full_size or golden or non_power}" > gpurun_out/var/$n.tests 2>&1 \
      || { echo "$n: parity FAILED"; tail -5 gpurun_out/var/$n.tests; exit 1; }
  DASH_LIB=$lib timeout -k 10 120 python3 bench.py --systems 262144 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/var/$n.json 2> gpurun_out/var/$n.err || { echo "$n: bench failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/var/$n.json'));print('%-10s kernel %.1f ms  %s'%('$n', d['kernel_ms_avg'], open('gpurun_out/var/$n.tests').read().strip().splitlines()[-1]))"
done
