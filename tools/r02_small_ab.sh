#!/bin/bash
# fused vs separate selection at the per-GPU shard sizes of the strong-scaling runs
set -o pipefail
for G in 32768 16384 8192; do
  for sel in fused separate fused separate; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-per-config --steps 100 --warmup 10 --global-batch $G --weak-batch 0 --select $sel > gpurun_out/small_${G}_${sel}.log 2>&1 || { echo "bench $G $sel failed"; tail -3 gpurun_out/small_${G}_${sel}.log; exit 1; }
    grep '^{' gpurun_out/small_${G}_${sel}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$G $sel', round(d['value']/1e6,2), 'M QP/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in d['config']['kernel_ms'].items()})"
  done
done
