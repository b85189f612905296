#!/bin/bash
# GPU box: config E with the Pade products out of line (default) vs inlined (lib variant
# expinl), alternating processes; then instruction-cache / instruction-mix counters.
O=${1:-gpurun_out/r04g}
L=$PWD/mpc-limx-control_amd/lib
for i in 1 2; do
  for lib in libmpcqp.so libmpcqp_expinl.so; do
    echo "== $lib" >> ${O}_E.log
    MPCQP_LIB=$L/$lib timeout -k 10 120 python tools/ab_env.py --slot 1 --config E --env X=1 --batches 16384 --rounds 3 --per 3 >> ${O}_E.log 2>&1 || exit 1
  done
done
bash tools/r04_pmcE.sh ${O}_pe || exit 1
echo g done
