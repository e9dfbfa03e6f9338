#!/bin/bash
# GPU parity suite + a bench line (no CPU baseline). Usage: tools/gpu_check.sh TAG [bench args]
set -o pipefail
TAG=${1:-chk}; shift || true
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${TAG}_bench.json 2>/dev/null || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('value %.4g ms/step %.1f kernel %.1f tiers?'%(d['value'],d['ms_per_step'],d['kernel_ms_avg']))"
