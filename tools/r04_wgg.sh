#!/bin/bash
# GPU box: the overflow launch's own time at config B (empty list) against its grid
# (MPCQP_WG_GRID caps it; the launch is read at every call), slots 3 (workgroup kernel) and 2.
O=${1:-gpurun_out/r04wgg}
for s in 3 2; do
  timeout -k 10 150 python tools/ab_env.py --slot $s --env MPCQP_WG_GRID= --env MPCQP_WG_GRID=64 --env MPCQP_WG_GRID=8 --batches 4096,8192,65536 --rounds 4 --per 8 >> ${O}.log 2>&1 || exit 1
done
echo wgg done
