#!/bin/bash
# GPU box: first 20 steps of a fresh context, the product library vs the input-alias build
# (inputs of instance b mod 128: cache-resident), twice each, alternating processes.
O=${1:-gpurun_out/r04sp3}
L=$PWD/mpc-limx-control_amd/lib
for i in 1 2; do
  for lib in libmpcqp.so libmpcqp_alias.so; do
    echo "== $lib" >> ${O}.log
    MPCQP_LIB=$L/$lib timeout -k 10 200 python tools/step_profile.py >> ${O}.log 2>&1 || exit 1
  done
done
echo sp3 done
