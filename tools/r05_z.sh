#!/bin/bash
# r05: the DESIGN §5 shard table at the current library (tools/r03_sweep.py sizes) and the bench
# step at --global-batch 8,192 / 4,096 (one GPU: the per-GPU shard of an 8 / 16-way split)
set -o pipefail
T=${1:-r05z}
mkdir -p gpurun_out
{ timeout -k 10 300 python3 tools/r03_sweep.py --sizes 2048,4096,6144,8192,12288,65536 --reps 50 &&
  for g in 8192 4096; do
    timeout -k 10 300 python3 bench.py --global-batch $g --no-per-config --no-host-path --no-cpu-baseline | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench --global-batch', d['config']['global_batch'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %.4f' % d['roofline']['kernel_ms'])"
  done; } > gpurun_out/${T}.txt 2>&1 || { tail -20 gpurun_out/${T}.txt; exit 1; }
cat gpurun_out/${T}.txt
