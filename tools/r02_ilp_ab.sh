#!/bin/bash
# default vs max-ilp (pair TU) vs max-ilp (every fused TU) on B, C, L, E and the overflow gaits
set -o pipefail
for n in default ilp ilpall default ilp ilpall; do
  if [ "$n" = default ]; then L=$PWD/mpc-limx-control_amd/lib/libmpcqp.so; else L=$PWD/mpc-limx-control_amd/lib/libmpcqp_$n.so; fi
  echo "== $n"
  MPCQP_LIB=$L timeout -k 10 120 python tools/time_kernel.py --configs B,C,L --reps 10 2>&1 | grep -E "B:|C:|L:" || exit 1
  MPCQP_LIB=$L timeout -k 10 120 python tools/time_kernel.py --configs E --batch 16384 --reps 5 2>&1 | grep -E "E:" || exit 1
  MPCQP_LIB=$L timeout -k 10 120 python tools/time_kernel.py --configs C --gait mixed --reps 2 2>&1 | grep -E "C:" | sed 's/C:/C-mixed:/' || exit 1
done
