#!/bin/bash
# GPU box: parity tests, then the overflow launch (slot 3) and the paired kernel (slot 2) of the
# current library against lib/libmpcqp_prev.so, alternating processes.
O=${1:-gpurun_out/r04tk}
L=$PWD/mpc-limx-control_amd/lib
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
for i in 1 2; do
  for lib in libmpcqp.so libmpcqp_prev.so; do
    for s in 3 1; do
      echo "== $lib slot $s" >> ${O}.log
      MPCQP_LIB=$L/$lib timeout -k 10 120 python tools/ab_env.py --slot $s --env X=1 --batches 4096,65536 --rounds 4 --per 8 >> ${O}.log 2>&1 || exit 1
    done
  done
done
echo tk done
