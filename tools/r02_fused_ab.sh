#!/bin/bash
# GPU suite, then the bench step with the fused selection record against the separate
# k_select_min launch (same binary, --select), one line each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/fused_tests.log 2>&1
tail -4 gpurun_out/fused_tests.log
for sel in fused separate fused separate; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-per-config --steps 50 --warmup 5 --select $sel > gpurun_out/fused_$sel.log 2>&1 || { echo "bench $sel failed"; tail -5 gpurun_out/fused_$sel.log; exit 1; }
  grep '^{' gpurun_out/fused_$sel.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$sel', round(d['value']/1e6,2), 'M QP/s', round(d['ms_per_step'],4), 'ms/step', d['config']['kernel_ms'])"
done
