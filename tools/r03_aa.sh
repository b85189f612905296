#!/bin/bash
# paired kernel's R^-1 d loop in blocks of four: GPU tests, then the shard sweep alternating
# default / ru0 (MPCQP_PAIR_RU4=0 in fast_pair); C / L with the one-QP solver's R^-1 loop in blocks
# of four (cru0 / lru0 = MPCQP_REG_RU4=0)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03aa}
TAG=$T tools/gpu_tests.sh || exit 1
L=$PWD/mpc-limx-control_amd/lib
for v in default ru0 default ru0; do
  if [ $v = default ]; then lib=$L/libmpcqp.so; else lib=$L/libmpcqp_$v.so; fi
  echo "== $v"
  MPCQP_LIB=$lib timeout -k 10 200 python -u tools/r03_sweep.py --sizes 512,4096,8192,65536 --reps 40 2>&1 | grep "^B " || exit 1
done > gpurun_out/${T}_sweep.log
cat gpurun_out/${T}_sweep.log
AB_CONFIGS=C AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default cru0 default cru0 > gpurun_out/${T}_C.log 2>&1 || { cat gpurun_out/${T}_C.log; exit 1; }
cat gpurun_out/${T}_C.log
AB_CONFIGS=L AB_REPS=10 timeout -k 10 300 tools/ab_libs.sh default lru0 default lru0 > gpurun_out/${T}_L.log 2>&1 || { cat gpurun_out/${T}_L.log; exit 1; }
cat gpurun_out/${T}_L.log
