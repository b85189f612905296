# round 6: config E's Toeplitz tile loads without the zero selects once every row is live
# (default) against the selects throughout (nosplit_e)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default nosplit_e || exit 1; done > gpurun_out/r06u_ab.log 2>&1
cat gpurun_out/r06u_ab.log
