#!/bin/bash
# A/B timing of library variants (GPU box, repo root): tools/ab_libs.sh name1 name2 ...
# [AB_CONFIGS=B,C AB_GAIT=mixed AB_BATCH=65536 AB_REPS=30 AB_B2B=1 (back-to-back launches)]
# (lib/libmpcqp_<name>.so; "default" = lib/libmpcqp.so).  One process per variant.
for n in "$@"; do
  if [ "$n" = default ]; then L=$PWD/mpc-limx-control_amd/lib/libmpcqp.so; else L=$PWD/mpc-limx-control_amd/lib/libmpcqp_$n.so; fi
  echo "== $n"
  MPCQP_LIB=$L timeout -k 10 120 python tools/time_kernel.py --configs ${AB_CONFIGS:-B} --reps ${AB_REPS:-30} --gait ${AB_GAIT:-alternating} --batch ${AB_BATCH:-65536} ${AB_B2B:+--b2b} 2>&1 | grep -v amdgpu.ids | grep -v "^lib"
done
