#!/bin/bash
# Round evidence on the GPU box (repo root): the -m gpu suite, the default bench line, then the
# rocprofv3 kernel-trace + PMC traffic passes (tools/profile_run.sh).  Stops at the first
# failure; every GPU step has its own time limit.
#   tools/evidence_run.sh TAG      -> gpurun_out/{t_all.log, bench_TAG.json, prof_TAG/}
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
    > gpurun_out/t_all.log 2>&1 || { echo "gpu tests failed"; tail -n 30 gpurun_out/t_all.log; exit 1; }
tail -n 2 gpurun_out/t_all.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -n 20 gpurun_out/bench_$TAG.log; exit 1; }
grep '^{' gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline" timeout -k 10 700 bash tools/profile_run.sh gpurun_out/prof_$TAG \
    || { echo "profile failed"; exit 1; }
echo "evidence OK"
