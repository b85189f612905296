#!/bin/bash
# -m gpu suite, then A/B of the workgroup-kernel configs (E, B standing, C mixed):
# lib/libmpcqp_base.so vs lib/libmpcqp.so, one process per variant and config
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/${1:-r02wab}
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu \
    > $O.tests.log 2>&1 || { tail -n 30 $O.tests.log; exit 1; }
tail -n 2 $O.tests.log
for v in ${AB_VARIANTS:-base default}; do
  if [ $v = default ]; then L=$PWD/mpc-limx-control_amd/lib/libmpcqp.so; else L=$PWD/mpc-limx-control_amd/lib/libmpcqp_$v.so; fi
  echo "== $v" >> $O.time.log
  MPCQP_LIB=$L timeout -k 10 200 python tools/time_kernel.py --configs E --batch 16384 --reps 5 >> $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
  MPCQP_LIB=$L timeout -k 10 200 python tools/time_kernel.py --configs B --gait standing --reps 5 >> $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
  MPCQP_LIB=$L timeout -k 10 200 python tools/time_kernel.py --configs C --gait mixed --reps 3 >> $O.time.log 2>&1 || { cat $O.time.log; exit 1; }
done
grep -v amdgpu.ids $O.time.log
