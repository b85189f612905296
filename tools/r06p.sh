# round 6: row-load lane masks and the crash's Newton reciprocal (default) against the previous
# commit (old2 = both off) and each alone; parity first
set -o pipefail
mkdir -p gpurun_out
TAG=r06p bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or fuzz or parity" || exit 1
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh old2 default nolmask norcp || exit 1
  done
done > gpurun_out/r06p_ab.log 2>&1
cat gpurun_out/r06p_ab.log
