#!/bin/bash
# GPU box: parity tests, then config E with the workgroup crash on / off (full kernel), and the
# crash's own time (cuts build: 106 = unconstrained minimum, 108 = after the crash).
O=${1:-gpurun_out/r04e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_path.py -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
timeout -k 10 150 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 16384 --rounds 4 --per 4 > ${O}_wg.log 2>&1 || exit 1
for cut in 106 108; do
  MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_cuts.so MPCQP_CUT=$cut timeout -k 10 150 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 16384 --rounds 3 --per 3 >> ${O}_cc.log 2>&1 || exit 1
done
echo e done
