# round 6: driver-style bench lines (20 steps after 5 warm-up) with the per-config lines run
# right before the headline's warm-up, twice, and once without per-config lines
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06q_drv$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06q_drv$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-style', d['value']/1e6, d['ms_per_step'], d['config']['kernel_ms'])"
done
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-per-config --no-cpu-baseline --no-host-path > gpurun_out/r06q_noper.log 2>&1 || exit 1
grep '^{' gpurun_out/r06q_noper.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no per-config', d['value']/1e6, d['ms_per_step'])"
