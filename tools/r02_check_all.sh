#!/bin/bash
# GPU suite + per-config kernel times (time_kernel) + the bench's own per_config line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/chk_tests.log 2>&1
tail -2 gpurun_out/chk_tests.log
AB_CONFIGS=B,C,L AB_REPS=10 bash tools/ab_libs.sh default
timeout -k 10 200 python tools/time_kernel.py --configs C --gait mixed --reps 3 2>&1 | grep -E "C:"
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/chk_bench.log 2>&1 || { echo bench failed; tail -3 gpurun_out/chk_bench.log; exit 1; }
grep '^{' gpurun_out/chk_bench.log | python3 -c "
import sys,json; d=json.loads(sys.stdin.read()); print('bench', round(d['value']/1e6,2), d['ms_per_step'], d['config']['kernel_ms'])
for k,v in d['config']['per_config'].items(): print(' ', k, round(v['kernel_ms'],4), round(v['mean_solver_iters'],3))"
