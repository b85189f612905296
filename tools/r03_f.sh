#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03f}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 200 python -u tools/r03_sweep.py --reps 30 --sizes 512,4096,8192,65536 > gpurun_out/${T}_sweep.log 2>&1 || { echo sweep failed; exit 1; }
cat gpurun_out/${T}_sweep.log
for G in 65536 8192; do for sel in separate fused; do
timeout -k 10 200 python -u bench.py --no-per-config --no-cpu-baseline --steps 100 --warmup 10 --global-batch $G --weak-batch 0 --select $sel > gpurun_out/${T}_b${G}_${sel}.log 2>&1 || { echo bench failed; tail -3 gpurun_out/${T}_b${G}_${sel}.log; exit 1; }
grep '^{' gpurun_out/${T}_b${G}_${sel}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print('$G $sel', round(d['value']/1e6,2), 'M QP/s', round(d['ms_per_step']*1e3,1), 'us/step', {k[:24]: round(v*1e3,1) for k,v in c['kernel_ms'].items()})"
done; done
