#!/bin/bash
# GPU box: workgroup crash sub-phase stamps at B standing (stamps build), and the stamps
# build's own kernel times with the crash on / off.  Usage: tools/r04_st.sh OUT
O=${1:-gpurun_out/r04st}
export MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so
MPCQP_CRASH_P_WG=12 timeout -k 10 200 python tools/phase_profile.py --config B --gait standing --batch 65536 > ${O}_Bst12.log 2>&1 || exit 1
timeout -k 10 150 python tools/ab_env.py --slot 3 --config B --gait standing --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 65536 --rounds 3 --per 3 > ${O}_ab.log 2>&1 || exit 1
echo st done
