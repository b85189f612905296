#!/bin/bash
# issue / stall / LDS counters of config E's k_dense_wg (16,384) and of the headline k_mpc_pair,
# two --pmc passes each (tools/pmc_stall.sh)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03ab}
ARGS="--config E --global-batch 16384 --steps 3 --warmup 1 --no-cpu-baseline --no-per-config --weak-batch 0 --no-kernel-timing" \
  timeout -k 10 300 bash tools/pmc_stall.sh gpurun_out/${T}_E || exit 1
timeout -k 10 300 bash tools/pmc_stall.sh gpurun_out/${T}_B || exit 1
echo ok
