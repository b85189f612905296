#!/bin/bash
# HBM traffic A/B of library variants (GPU box, repo root): tools/ab_traffic.sh name1 name2 ...
# One FETCH_SIZE and one WRITE_SIZE pass (separate, pool rule) of the headline bench per
# variant -> gpurun_out/abt_<name>/{fetch,write}; tools/traffic_table.py prints the table.
set -o pipefail
export TMPDIR=/tmp
R=$(pwd)
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --no-per-config"}
for n in "$@"; do
  if [ "$n" = default ]; then L=$R/mpc-limx-control_amd/lib/libmpcqp.so; else L=$R/mpc-limx-control_amd/lib/libmpcqp_$n.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    MPCQP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $c -d "$R/gpurun_out/abt_$n/$c" -o run \
        --output-format csv -- python3 bench.py $ARGS > "gpurun_out/abt_${n}_$c.log" 2>&1 || { echo "$n $c failed"; exit 1; }
  done
  echo "$n: $(grep '^{' gpurun_out/abt_${n}_WRITE_SIZE.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
done
