# round 6: padded diagonal staging + rotated t readout in the workgroup factorisation (E, overflow)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gait.py -m gpu > gpurun_out/r06k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06k_tests.log
[ $rc = 0 ] || exit 1
for r in 1 2; do AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default nopad_c || exit 1; done
for r in 1 2; do AB_CONFIGS=B AB_GAIT=standing AB_REPS=10 bash tools/ab_libs.sh default nopad_c || exit 1; done
bash tools/phase_pmc_e.sh gpurun_out/pe_r06k > gpurun_out/r06k_E_census.txt 2>&1; cat gpurun_out/r06k_E_census.txt
