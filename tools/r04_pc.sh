#!/bin/bash
# GPU box: config E's crash cost against its working-set cap (cuts build, cut 108 = after the
# crash; cut 106 = before it), caps 0 / 1 / 2 / 12.
O=${1:-gpurun_out/r04pc}
export MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_cuts.so
for cut in 106 108; do
  MPCQP_CUT=$cut timeout -k 10 200 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=1 --env MPCQP_CRASH_P_WG=2 --env MPCQP_CRASH_P_WG=12 --batches 16384 --rounds 3 --per 3 >> ${O}.log 2>&1 || exit 1
done
echo pc done
