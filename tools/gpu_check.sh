#!/bin/bash
# GPU-box check used between kernel changes (repo root): the -m gpu suite, then the per-phase
# cuts of config B.  Each GPU step has its own time limit; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
    > gpurun_out/t_all.log 2>&1 || { echo "gpu tests failed"; tail -n 30 gpurun_out/t_all.log; exit 1; }
tail -n 2 gpurun_out/t_all.log
timeout -k 10 200 python tools/phase_cuts.py --configs "${CUT_CONFIGS:-B}" > gpurun_out/cuts.log 2>&1
cat gpurun_out/cuts.log
