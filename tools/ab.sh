#!/bin/bash
# A/B of kernel variants on one MI355X: quick GPU parity subset per variant, then the
# quarter-size headline bench alternating over the variants ROUNDS times (kernel ms each).
# Usage (through gpurun): tools/ab.sh NAME [NAME...]   (tools/variants/libdash_NAME.so)
set -uo pipefail
mkdir -p gpurun_out/ab
for n in "$@"; do
  [ "$n" = base ] && continue
  DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q \
      --timeout 120 --timeout-method thread > gpurun_out/ab/$n.tests 2>&1 \
      || { echo "$n: parity FAILED"; tail -15 gpurun_out/ab/$n.tests; exit 1; }
  echo "$n: $(tail -1 gpurun_out/ab/$n.tests)"
done
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 120 python3 bench.py --systems ${SYSTEMS:-262144} --steps 3 --warmup 1 \
        --no-cpu-baseline --contention-steps ${CSTEPS:-0} > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.err || { echo "$n bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/$n.$r.json'));c=d.get('contention') or {};print('%-8s r%d kernel %.2f ms  contention %s'%('$n',$r,d['kernel_ms_avg'],round(c.get('kernel_ms_avg',0),2)))"
  done
done
