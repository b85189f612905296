#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats           -> per-kernel average duration
#   2. --pmc FETCH_SIZE   (own pass)  -> HBM read bytes  (gfx950: x2 for wide streams)
#   3. --pmc WRITE_SIZE   (own pass)  -> HBM write bytes
# Counters are never combined with trace domains (pool rule).  Usage: tools/profile_run.sh OUT
set -e
OUT=${1:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
# counter passes: the headline launches only (per_config's B-standing runs the same kernel)
PMC_ARGS=${PMC_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline --no-per-config"}
mkdir -p "$OUT"
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/trace" -o run --output-format csv \
    -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/$OUT/fetch" -o run --output-format csv \
    -- python3 bench.py $PMC_ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/$OUT/write" -o run --output-format csv \
    -- python3 bench.py $PMC_ARGS > "$OUT/write.log" 2>&1
