# round 6: unmasked crash elimination (LSEL) and the S loop order (SLOOP) in the paired kernel
# (default has both, old3 neither), and config E's compile-time tile schedule (nosched_e: off);
# parity first
set -o pipefail
mkdir -p gpurun_out
TAG=r06t bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or fuzz or parity or literal or dense" || exit 1
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh old3 default nolsel noslp || exit 1
  done
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default nosched_e || exit 1
done > gpurun_out/r06t_ab.log 2>&1
cat gpurun_out/r06t_ab.log
