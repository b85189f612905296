# round 6: the C-ABI group's host path with page-locked caller arrays (direct DMA per member)
set -o pipefail
mkdir -p gpurun_out
TAG=r06w bash tools/gpu_tests.sh -k "group or host" || exit 1
timeout -k 10 200 python3 tools/group_host_rate.py --states 4096 > gpurun_out/r06w_group_host.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r06w_group_host.log
