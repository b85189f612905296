#!/bin/bash
# FP64 VALU / MFMA counters of the one-QP kernel at config C and the dense workgroup kernel at
# config E (tools/pmc_flops.sh passes, own bench runs), for profiles/pmc_flops_{C,E}.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/pmc_flops.sh gpurun_out/pmcf_C --config C --steps 3 --warmup 1 --no-cpu-baseline --no-per-config || exit 1
timeout -k 10 300 bash tools/pmc_flops.sh gpurun_out/pmcf_E --config E --global-batch 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-per-config || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_CE/C -o run --output-format csv -- python3 bench.py --config C --steps 5 --warmup 1 --no-cpu-baseline --no-per-config > gpurun_out/prof_CE_C.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_CE/E -o run --output-format csv -- python3 bench.py --config E --global-batch 16384 --steps 5 --warmup 1 --no-cpu-baseline --no-per-config > gpurun_out/prof_CE_E.log 2>&1 || exit 1
export TMPDIR=/tmp
R=$(pwd)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/trf_C/$c" -o run --output-format csv -- python3 bench.py --config C --steps 3 --warmup 1 --no-cpu-baseline --no-per-config > gpurun_out/trf_C_$c.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/trf_E/$c" -o run --output-format csv -- python3 bench.py --config E --global-batch 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-per-config > gpurun_out/trf_E_$c.log 2>&1 || exit 1
done
echo pmc OK
