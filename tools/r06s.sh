# round 6: driver-style bench lines with the per-config lines (B-standing last) right before the
# headline's warm-up
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06s_drv$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/r06s_drv$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-style', d['value']/1e6, d['ms_per_step'], d['config']['kernel_ms'])"
done
