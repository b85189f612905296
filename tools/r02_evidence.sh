#!/bin/bash
# bench line + rocprofv3 kernel trace/stats + PMC traffic + PMC executed-flops passes, tagged.
#   tools/r02_evidence.sh TAG  -> gpurun_out/{bench_TAG.json, prof_TAG/, pmcf_TAG/}
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench_$TAG.log; exit 1; }
grep '^{' gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline" timeout -k 10 700 bash tools/profile_run.sh gpurun_out/prof_$TAG \
    || { echo "profile failed"; exit 1; }
timeout -k 10 300 bash tools/pmc_flops.sh gpurun_out/pmcf_$TAG || { echo "pmc flops failed"; exit 1; }
echo "evidence OK"
