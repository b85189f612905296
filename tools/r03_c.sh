#!/bin/bash
# R^-1 dual loop: the suite, lone-wave stamps, sweep
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03c}
TAG=$T tools/gpu_tests.sh || exit 1
MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_stamps.so timeout -k 10 200 python -u tools/r03_sweep.py --max-free 30 --reps 5 --sizes 128,512 > gpurun_out/${T}_stamps.log 2>&1 || { echo stamps failed; exit 1; }
cat gpurun_out/${T}_stamps.log
timeout -k 10 200 python -u tools/r03_sweep.py --reps 30 --sizes 512,4096,8192,16384,65536 > gpurun_out/${T}_sweep.log 2>&1 || { echo sweep failed; exit 1; }
cat gpurun_out/${T}_sweep.log
timeout -k 10 300 python -u bench.py --no-per-config --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/${T}_bench.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-per-config --no-cpu-baseline --no-kernel-timing > gpurun_out/${T}_bench_nt.log 2>&1 || { echo bench2 failed; tail -5 gpurun_out/${T}_bench_nt.log; exit 1; }
for f in gpurun_out/${T}_bench.log gpurun_out/${T}_bench_nt.log; do grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print(round(d['value']/1e6,2), 'M QP/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in c['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3), c.get('per_tick_latency'))"; done
