#!/bin/bash
# Occupancy sweep: bench.py at a quarter of the headline size with dynamic LDS padding
# that caps the resident workgroups (waves) per CU. Usage: tools/occ_sweep.sh [PAD...]
# needs the DASH_LDS_PAD hook: PATCHES=tools/experiments/lds_pad.patch tools/build_variant.sh ldspad
set -uo pipefail
mkdir -p gpurun_out/occ
pads=("$@"); [ ${#pads[@]} -eq 0 ] && pads=(11264 4096 2200 1000 0)
for pad in "${pads[@]}"; do
  DASH_LDS_PAD=$pad DASH_LIB=$PWD/tools/variants/libdash_ldspad.so timeout -k 10 120 python3 bench.py --systems 262144 --steps 2 --warmup 1 --no-cpu-baseline \
      > gpurun_out/occ/pad_$pad.json 2> gpurun_out/occ/pad_$pad.err || { echo "pad $pad failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/occ/pad_$pad.json'));print('pad $pad', round(d['kernel_ms_avg'],1), d['value'])"
done
