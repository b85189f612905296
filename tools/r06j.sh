# round 6: padded one-wave Cholesky staging (config C): parity, A/B, census
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/r06j_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06j_tests.log
[ $rc = 0 ] || exit 1
for r in 1 2; do AB_CONFIGS=C AB_REPS=20 bash tools/ab_libs.sh default nopad_c || exit 1; done
bash tools/phase_pmc.sh gpurun_out/pc_r06j C > gpurun_out/r06j_C_census.txt 2>&1; cat gpurun_out/r06j_C_census.txt
