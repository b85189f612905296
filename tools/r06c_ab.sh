# round 6: the paired kernel at a 4-wave register budget vs 3 (one library, MPCQP_PAIR_W4_MIN) and
# against the round-5 library (base)
set -o pipefail
mkdir -p gpurun_out
K="pair or batch_vs_oracle or gait or crash or flops or fuzz"
TAG=r06d_def bash tools/gpu_tests.sh -k "$K" || exit 1
MPCQP_PAIR_W4_MIN=1 TAG=r06d_w4all bash tools/gpu_tests.sh -k "$K" || exit 1
timeout -k 10 400 python3 tools/ab_env.py --env MPCQP_PAIR_W4_MIN=0 --env MPCQP_PAIR_W4_MIN=1 \
    --batches 65536,32768,16384,8192,4096 --rounds 10 > gpurun_out/r06d_w4env.log 2>&1 || exit 1
cat gpurun_out/r06d_w4env.log
for r in 1 2; do
  for b in 65536 8192; do
    AB_REPS=60 AB_BATCH=$b bash tools/ab_libs.sh base default || exit 1
  done
done > gpurun_out/r06d_ab.log 2>&1
cat gpurun_out/r06d_ab.log
