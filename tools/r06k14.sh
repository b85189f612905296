# round 6: the crash's working-set cap KC = 10 or 14 against 12
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh default k14 || exit 1
  done
done > gpurun_out/r06k14_ab.log 2>&1
cat gpurun_out/r06k14_ab.log
