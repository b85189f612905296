# round 6: scheduler strategies for the paired kernel's 4-wave (65,536) and 3-wave (8,192) builds
set -o pipefail
mkdir -p gpurun_out
V="default noilp_b sb_iterative-minreg sb_iterative-ilp"
for r in 1 2; do
  AB_CONFIGS=B AB_REPS=40 bash tools/ab_libs.sh $V || exit 1
  AB_CONFIGS=B AB_REPS=60 AB_BATCH=8192 bash tools/ab_libs.sh $V || exit 1
done
