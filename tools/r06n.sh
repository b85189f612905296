# round 6: folded sweep with constant lane-mask selects, SGPR non-PD mask, 64-bit copies for the
# row pairs, one DPP wait per step -- GPU suite, then A/B against the r06z library (prev)
set -o pipefail
mkdir -p gpurun_out
TAG=r06n bash tools/gpu_tests.sh || exit 1
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_REPS=60 AB_BATCH=$b bash tools/ab_libs.sh prev default || exit 1
  done
done > gpurun_out/r06n_ab.log 2>&1
cat gpurun_out/r06n_ab.log
