# round 6: back-to-back A/B of the folded-sweep micro-optimisations (default) against r06z (prev)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh prev default || exit 1
  done
done > gpurun_out/r06o_ab.log 2>&1
cat gpurun_out/r06o_ab.log
