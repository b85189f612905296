# round 6 closing set at the final library (GPU box, repo root):
#   GPU suite + smoke, the evidence set (tools/evidence.sh TAG), the shard table and the
#   --global-batch 8,192 / 4,096 bench lines, the per-phase census of k_mpc_pair (4-wave build)
#   and of configs C and E, and the driver-style bench line (20 steps after 5 warm-up).
set -o pipefail
T=${1:-r06y}
mkdir -p gpurun_out
TAG=${T} bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; exit 1; }
bash tools/evidence.sh ${T} || exit 1
bash tools/runs.sh shards ${T}_shards || exit 1
bash tools/phase_pmc_pair.sh gpurun_out/pp_${T} B > gpurun_out/${T}_census_B.txt 2>&1 || exit 1
bash tools/phase_pmc.sh gpurun_out/pc_${T} C > gpurun_out/${T}_census_C.txt 2>&1 || exit 1
bash tools/phase_pmc_e.sh gpurun_out/pe_${T} > gpurun_out/${T}_census_E.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver_style.log 2>&1 || exit 1
grep '^{' gpurun_out/${T}_bench_driver_style.log > gpurun_out/${T}_bench_driver_style.json
echo "final set ${T} OK"
