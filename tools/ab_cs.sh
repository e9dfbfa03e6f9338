#!/bin/bash
# A/B of kernel variants at one configs[4] point (locality traces, one CACHE_SIZE), alternating
# ROUNDS times: kernel ms per variant. Quick parity subset first (tests/test_gpu_sweep.py is the
# sweep's bit-exact check). Usage (through gpurun): CS=8 LOC=0 tools/ab_cs.sh NAME [NAME...]
set -uo pipefail
mkdir -p gpurun_out/ab_cs
CS=${CS:-8}; LOC=${LOC:-0}
for n in "$@"; do
  [ -n "${SKIP_PARITY:-}" ] && break  # timing probes whose results are wrong by design
  DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -q \
      -k "test_sweep_grid_matches_oracle and 1" --timeout 300 --timeout-method thread > gpurun_out/ab_cs/$n.tests 2>&1 \
      || { echo "$n: sweep parity FAILED"; tail -15 gpurun_out/ab_cs/$n.tests; exit 1; }
  echo "$n: $(tail -1 gpurun_out/ab_cs/$n.tests)"
done
for r in $(seq ${ROUNDS:-3}); do
  for n in "$@"; do
    DASH_LIB=$PWD/tools/variants/libdash_$n.so timeout -k 10 120 python3 bench.py --kind locality --locality $LOC \
        --cache-size $CS --systems ${SYSTEMS:-262144} --steps 3 --warmup 1 --no-cpu-baseline --contention-steps 0 \
        --detail gpurun_out/ab_cs/$n.$r.detail.json > gpurun_out/ab_cs/$n.$r.json 2> gpurun_out/ab_cs/$n.err \
        || { echo "$n bench failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_cs/$n.$r.detail.json'));print('%-8s r%d CS $CS p $LOC kernel %.2f ms, %.4f ns per wave-round'%('$n',$r,d['kernel_ms_avg'],d['kernel_ms_avg']*1e6/d['wave_rounds']))"
  done
done
