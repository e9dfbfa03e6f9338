#!/bin/bash
# Event-log kernel (MODE 2) ablation on one MI355X: the bench_next events row (32,768 systems x 8 x
# 4096, fast kernel vs event-log kernel) for the product library and for the variants of
# tools/experiments/event_log_ablation.patch (built into tools/var_r4/ by tools/build_variant.sh),
# then one rocprofv3 PMC pass of SQ counters over the product's events row.
set -uo pipefail
mkdir -p gpurun_out/ev_abl; export TMPDIR=/tmp
for v in base NOLOG NOLOGLDS NOFLUSH NOSTORE NOARB; do
  L=""; [ "$v" != base ] && L=$PWD/tools/var_r4/libdash_ev_$v.so
  DASH_LIB=$L timeout -k 10 200 python -c "import bench, bench_next, json; d=bench.load_dash(); print(json.dumps([bench_next.events_row(d, 0, 0x5EED, 32768, 4096) for _ in range(2)]))" \
      > gpurun_out/ev_abl/$v.json 2> gpurun_out/ev_abl/$v.err || { echo "$v failed"; tail -3 gpurun_out/ev_abl/$v.err; exit 1; }
  python3 -c "import json; r=json.load(open('gpurun_out/ev_abl/$v.json')); print('$v', [round(x['kernel_ms'],2) for x in r], [round(x['fast_kernel_ms'],2) for x in r])"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d gpurun_out/ev_abl/pmc_sq -o run -- \
    python3 -c "import bench, bench_next; d=bench.load_dash(); bench_next.events_row(d, 0, 0x5EED, 32768, 4096)" > gpurun_out/ev_abl/pmc_sq.log 2>&1 || echo "pmc failed"
echo ablation-done
timeout -k 10 120 python -c "import bench, json; d=bench.load_dash(); print(json.dumps([d.probe_box(0) for _ in range(3)]))" > gpurun_out/ev_abl/probe.json 2>&1 || echo probe-failed
