#!/bin/bash
# GPU box: parity tests, then the code-size builds against the previous ones (one inlined
# diagonal factorisation, out-of-line Pade products) alternating per process: E (bigE),
# C (bigC), B standing (bigW).  Usage: tools/r04_h.sh OUT
O=${1:-gpurun_out/r04h}
L=$PWD/mpc-limx-control_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_path.py -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
ab() {  # variant slot args...
  local v=$1 s=$2; shift 2
  for i in 1 2; do
    for lib in libmpcqp.so libmpcqp_$v.so; do
      echo "== $lib" >> ${O}_$v.log
      MPCQP_LIB=$L/$lib timeout -k 10 120 python tools/ab_env.py --slot $s --env X=1 --rounds 3 --per 3 "$@" >> ${O}_$v.log 2>&1 || return 1
    done
  done
}
ab bigE 1 --config E --batches 16384 || exit 1
ab bigC 2 --config C --batches 65536 || exit 1
ab bigW 3 --config B --gait standing --batches 65536 || exit 1
echo h done
