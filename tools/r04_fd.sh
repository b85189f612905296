#!/bin/bash
# GPU box: one Newton step after v_rsq_f64 in the other translation units: parity suite per
# variant, then each against the product library, alternating processes.
O=${1:-gpurun_out/r04nr}
L=$PWD/mpc-limx-control_amd/lib
for v in fast_dense fast_srbm20 fast_literal fast_wg; do
  MPCQP_LIB=$L/libmpcqp_fd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > ${O}_tests_$v.log 2>&1 || { echo "tests failed $v"; tail -5 ${O}_tests_$v.log; exit 1; }
done
ab() {  # variant slot args...
  local v=$1 s=$2; shift 2
  for i in 1 2; do
    for lib in libmpcqp.so libmpcqp_fd_$v.so; do
      echo "== $lib" >> ${O}_$v.log
      MPCQP_LIB=$L/$lib timeout -k 10 150 python tools/ab_env.py --slot $s --env X=1 --rounds 3 --per 4 "$@" >> ${O}_$v.log 2>&1 || return 1
    done
  done
}
ab fast_dense 1 --config E --batches 16384 || exit 1
ab fast_srbm20 2 --config C --batches 65536 || exit 1
ab fast_literal 2 --config L --batches 65536 || exit 1
ab fast_wg 3 --config B --gait standing --batches 65536 || exit 1
echo fd done
