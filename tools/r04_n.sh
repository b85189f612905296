#!/bin/bash
# GPU box: parity tests, then the workgroup crash on / off (full kernels: E, B standing, B mixed;
# cuts build: the crash's own time at B standing and E).  Usage: tools/r04_n.sh OUT
O=${1:-gpurun_out/r04n}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_path.py -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
timeout -k 10 150 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 16384 --rounds 4 --per 4 > ${O}_wg.log 2>&1 || exit 1
for g in standing mixed; do
  timeout -k 10 150 python tools/ab_env.py --slot 3 --config B --gait $g --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG=12 --batches 65536 --rounds 4 --per 4 >> ${O}_wg.log 2>&1 || exit 1
done
bash tools/r04_crashcut.sh ${O}_cc || exit 1
echo n done
