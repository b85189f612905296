#!/bin/bash
# r05: GPU suite, fold A/B (B and L configs), bench --capi-group smoke (GPU box, repo root)
set -o pipefail
T=${1:-r05b}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
for r in 1 2; do
  AB_CONFIGS=B,L bash tools/ab_libs.sh default nofold
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-per-config --no-host-path --capi-group > gpurun_out/${T}_capi.log 2>&1 || { tail -20 gpurun_out/${T}_capi.log; exit 1; }
cat gpurun_out/${T}_ab.log
tail -c 600 gpurun_out/${T}_capi.log
