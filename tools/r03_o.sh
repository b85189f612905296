#!/bin/bash
# small-batch step anatomy: sweep with fused selection, and a kernel trace of the step chain
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03o}
true
true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for B in 4096 8192; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_tr$B -o run --output-format csv -- python3 tools/step_trace.py --batch $B > gpurun_out/${T}_tr$B.log 2>&1 || { tail gpurun_out/${T}_tr$B.log; exit 1; }
  f=$(find gpurun_out/${T}_tr$B -name 'run_kernel_trace.csv' | head -1)
  echo "== B $B"; python tools/step_trace.py --analyze $f
done
