# round 6: the small-batch paired kernel at a 2-wave register budget (w2) against 3 (default)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for b in 2048 4096 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh default w2 || exit 1
  done
done > gpurun_out/r06w2_ab.log 2>&1
cat gpurun_out/r06w2_ab.log
