#!/bin/bash
# GPU box: phase cuts of the paired kernel at the small shards (4,096 and 8,192 instances).
O=${1:-gpurun_out/r04cs}
for B in 4096 8192; do
  timeout -k 10 200 python tools/phase_cuts.py --configs B --batch $B --reps 20 --cuts 11,1,13,2,3,4,6,8,7,0 > ${O}_$B.log 2>&1 || exit 1
done
echo cs done
