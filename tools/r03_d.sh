#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03d}
TAG=$T tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -u bench.py --no-per-config --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep '^{' gpurun_out/${T}_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); c=d['config']; print(round(d['value']/1e6,2), 'M QP/s', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v*1e3,1) for k,v in c['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'],3), json.dumps(c.get('per_tick_latency')))"
