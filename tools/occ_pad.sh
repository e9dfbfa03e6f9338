set -uo pipefail
# needs the DASH_LDS_PAD hook: PATCHES=tools/experiments/lds_pad.patch tools/build_variant.sh ldspad
for pad in 0 256 1024 0 256 1024; do
  DASH_LDS_PAD=$pad DASH_LIB=$PWD/tools/variants/libdash_ldspad.so timeout -k 10 120 python3 bench.py --systems 262144 --steps 3 --warmup 1 --no-cpu-baseline --contention-steps 0 > gpurun_out/occ_$pad.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/occ_$pad.json'));print('pad $pad kernel %.2f'%d['kernel_ms_avg'])"
done
