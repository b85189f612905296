#!/bin/bash
# HBM traffic of library variants at one config (GPU box, repo root):
#   tools/traffic_ab.sh CONFIG name1 name2 ...   ("default" = lib/libmpcqp.so)
# One FETCH_SIZE and one WRITE_SIZE pass (separate, pool rule) of the config's bench line per
# variant -> gpurun_out/abt_<CONFIG>_<name>/{FETCH_SIZE,WRITE_SIZE}; tools/traffic_table.py.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
CFG=$1; shift
ARGS="--config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-per-config --no-host-path --no-kernel-timing"
for n in "$@"; do
  if [ "$n" = default ]; then L=$R/mpc-limx-control_amd/lib/libmpcqp.so; else L=$R/mpc-limx-control_amd/lib/libmpcqp_$n.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    MPCQP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/abt_${CFG}_$n/$c" -o run \
        --output-format csv -- python3 bench.py $ARGS > "gpurun_out/abt_${CFG}_${n}_$c.log" 2>&1 || { echo "$n $c failed"; exit 1; }
  done
done
echo traffic done
