#!/bin/bash
# GPU box: parity tests at the 1-Newton-step rsqrt build, E / B-standing phase stamps with the
# workgroup crash on and off, then the phase cuts of configs C and B.  Usage: tools/r04_m.sh OUT
O=${1:-gpurun_out/r04m}
L=$PWD/mpc-limx-control_amd/lib
MPCQP_LIB=$L/libmpcqp_nr1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > ${O}_nr1_tests.log 2>&1 || { echo nr1 tests failed; tail -5 ${O}_nr1_tests.log; }
for c in 0 12; do
  MPCQP_CRASH_P_WG=$c timeout -k 10 200 python tools/phase_profile.py --config E --batch 16384 > ${O}_E_stamps_$c.log 2>&1 || exit 1
  MPCQP_CRASH_P_WG=$c timeout -k 10 200 python tools/phase_profile.py --config B --gait standing --batch 65536 > ${O}_Bst_stamps_$c.log 2>&1 || exit 1
done
bash tools/r04_cuts.sh ${O}_cuts || exit 1
echo m done
