# round 6: the crash's unmasked elimination in the 4-wave build only (LSEL=2) and the unmasked
# y sum over zeroed rows (YZERO): default both, old4 neither; parity first
set -o pipefail
mkdir -p gpurun_out
TAG=r06v bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or fuzz or parity or literal" || exit 1
for r in 1 2 3; do
  for b in 65536 8192; do
    AB_B2B=1 AB_REPS=200 AB_BATCH=$b bash tools/ab_libs.sh old4 default yz0 lsel0 || exit 1
  done
done > gpurun_out/r06v_ab.log 2>&1
cat gpurun_out/r06v_ab.log
