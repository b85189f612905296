#!/bin/bash
# GPU box: the bench line as the driver runs it (20 steps after 5 warm-up), twice.
O=${1:-gpurun_out/r04drv2}
for i in 1 2; do
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 > ${O}_bench$i.log 2>&1 || exit 1
  grep '^{' ${O}_bench$i.log > ${O}_bench$i.json
done
echo drv2 done
