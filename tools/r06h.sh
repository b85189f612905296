# round 6: C warm crash + B warm seeding + census of C and E (one call)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gait.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/r06h_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r06h_tests.log
timeout -k 10 200 python3 tools/warm_iters.py --states 256 > gpurun_out/r06h_warm.log 2>&1; cat gpurun_out/r06h_warm.log
bash tools/phase_pmc.sh gpurun_out/pc_r06h C > gpurun_out/r06h_C_census.txt 2>&1; cat gpurun_out/r06h_C_census.txt
bash tools/phase_pmc_e.sh gpurun_out/pe_r06h > gpurun_out/r06h_E_census.txt 2>&1; cat gpurun_out/r06h_E_census.txt
