#!/bin/bash
# small-shard step: fused-record test (incl. max_free contexts without the workgroup kernel),
# then the shard sweep at the default context and at max_free = 30
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03s}
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k fused_record > gpurun_out/${T}_fused.log 2>&1 || { tail -n 30 gpurun_out/${T}_fused.log; exit 1; }
tail -n 3 gpurun_out/${T}_fused.log
timeout -k 10 300 python -u tools/r03_sweep.py --sizes 2048,4096,6144,8192,12288,65536 --reps 50 > gpurun_out/${T}_sweep.log 2>&1 || { tail gpurun_out/${T}_sweep.log; exit 1; }
timeout -k 10 300 python -u tools/r03_sweep.py --sizes 2048,4096,6144,8192,12288,65536 --reps 50 --max-free 30 >> gpurun_out/${T}_sweep.log 2>&1 || { tail gpurun_out/${T}_sweep.log; exit 1; }
cat gpurun_out/${T}_sweep.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-per-config > gpurun_out/${T}_bench.log 2>&1 || { tail gpurun_out/${T}_bench.log; exit 1; }
grep -o '"value": [0-9.e+]*, "unit"[^}]*"ms_per_step": [0-9.]*' gpurun_out/${T}_bench.log
for g in 8192 4096; do timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-per-config --global-batch $g > gpurun_out/${T}_bench$g.log 2>&1 || { tail gpurun_out/${T}_bench$g.log; exit 1; }; grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_bench$g.log; done
