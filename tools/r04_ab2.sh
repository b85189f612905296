#!/bin/bash
# r04 A/B set (GPU box): parity tests, then the paired kernel of two libraries alternated per
# process (default vs lib/libmpcqp_$v.so for each v of the comma list $1), then the workgroup crash on / off at E, B standing,
# B mixed.  Usage: tools/r04_ab2.sh VARIANT OUTPREFIX
V=$1; O=${2:-gpurun_out/r04ab2}
L=$PWD/mpc-limx-control_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_host_path.py -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
for i in 1 2; do
  for lib in libmpcqp.so $(for v in ${V//,/ }; do echo libmpcqp_$v.so; done); do
    echo "== $lib" >> ${O}_pair.log
    MPCQP_LIB=$L/$lib timeout -k 10 120 python tools/ab_env.py --env X=1 --batches 4096,8192,65536 >> ${O}_pair.log 2>&1 || exit 1
  done
done
timeout -k 10 150 python tools/ab_env.py --slot 1 --config E --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG= --batches 16384 --rounds 4 --per 4 > ${O}_wg.log 2>&1 || exit 1
timeout -k 10 150 python tools/ab_env.py --slot 3 --config B --gait standing --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG= --batches 65536 --rounds 4 --per 4 >> ${O}_wg.log 2>&1 || exit 1
timeout -k 10 150 python tools/ab_env.py --slot 3 --config B --gait mixed --env MPCQP_CRASH_P_WG=0 --env MPCQP_CRASH_P_WG= --batches 65536 --rounds 4 --per 4 >> ${O}_wg.log 2>&1 || exit 1
echo ab2 done
