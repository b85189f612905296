#!/bin/bash
# GPU box: the workgroup crash's own kernel time (cuts build: exit after the unconstrained
# minimum = cut 6, after the crash = cut 8, full = cut 0), crash on / off, B standing and E.
O=${1:-gpurun_out/r04cc}
export MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_cuts.so
for cut in 106 108 0; do
  MPCQP_CUT=$cut timeout -k 10 150 python tools/ab_env.py --slot 3 --config B --gait standing --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 65536 --rounds 3 --per 3 >> ${O}_Bst.log 2>&1 || exit 1
  MPCQP_CUT=$cut timeout -k 10 150 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 16384 --rounds 3 --per 3 >> ${O}_E.log 2>&1 || exit 1
done
echo cc done
