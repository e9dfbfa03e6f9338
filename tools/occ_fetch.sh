#!/bin/bash
# PATCHES=tools/experiments/lds_pad_r4.patch OUT=$PWD/tools/var_r4 tools/build_variant.sh ldspad, then (through gpurun):
# occupancy vs L2 over-fetch on the headline kernel (same code, fingerprint da9f0): dynamic LDS
# padding per workgroup caps the resident waves per CU (18 / 16 / 14 / 12); per pad the kernel time
# (bench.py, full size) and one rocprofv3 PMC pass of FETCH_SIZE + TCC hits
set -uo pipefail
OUT=gpurun_out/occ_fetch; mkdir -p $OUT; export TMPDIR=/tmp
export DASH_LIB=$PWD/tools/var_r4/libdash_ldspad.so
for pad in 0 1540 3000 4950; do
  DASH_LDS_PAD=$pad timeout -k 10 150 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off > $OUT/bench_$pad.json 2> $OUT/bench_$pad.err || { echo "bench $pad failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$pad.json').read().strip().splitlines()[-1]); print('pad $pad kernel_ms', round(d['kernel_ms_avg'],1))"
  DASH_LDS_PAD=$pad timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace --output-format csv -d $OUT/pmc_$pad -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --contention-steps 0 --line-sweep off --line-next off > $OUT/pmc_$pad.log 2>&1 || { echo "pmc $pad failed"; exit 1; }
  echo "pmc $pad ok"
done
