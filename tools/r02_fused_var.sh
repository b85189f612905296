#!/bin/bash
# fused-selection timing variants (libmpcqp_<name>.so): bench step ms with --select fused
set -o pipefail
for n in default noatom wgscope plainst; do
  if [ "$n" = default ]; then L=$PWD/mpc-limx-control_amd/lib/libmpcqp.so; else L=$PWD/mpc-limx-control_amd/lib/libmpcqp_$n.so; fi
  MPCQP_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-per-config --steps 50 --warmup 5 --select fused > gpurun_out/fv_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/fv_$n.log; exit 1; }
  grep '^{' gpurun_out/fv_$n.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$n', round(d['ms_per_step'],4), d['config']['kernel_ms'])"
done
