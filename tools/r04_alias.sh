#!/bin/bash
# GPU box: the paired kernel against its input-alias diagnostic build (inputs of instance b mod
# 128: L2-resident), alternating processes -- what the input loads' latency costs.
O=${1:-gpurun_out/r04al}
L=$PWD/mpc-limx-control_amd/lib
for i in 1 2; do
  for lib in libmpcqp.so libmpcqp_alias.so; do
    echo "== $lib" >> ${O}.log
    MPCQP_LIB=$L/$lib timeout -k 10 120 python tools/ab_env.py --env X=1 --batches 8192,65536 >> ${O}.log 2>&1 || exit 1
  done
done
echo alias done
