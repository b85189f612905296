# round 6: the group's loopback test transport (three ranks on one device) + the group suite
set -o pipefail
mkdir -p gpurun_out
TAG=r06lb bash tools/gpu_tests.sh tests/test_group.py || exit 1
