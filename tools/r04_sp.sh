#!/bin/bash
O=${1:-gpurun_out/r04sp2}
for ph in same-kernel C; do
  echo "== preheat $ph" >> ${O}.log
  timeout -k 10 200 python tools/step_profile.py --preheat $ph >> ${O}.log 2>&1 || exit 1
done
echo sp done
