#!/bin/bash
# r05: GPU suite + headline bench (long) + small-shard step times (GPU box, repo root)
set -o pipefail
T=${1:-r05i}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
B="--no-cpu-baseline --no-per-config --no-host-path"
timeout -k 10 200 python bench.py --steps 200 --warmup 100 $B > gpurun_out/${T}_b65536.json 2>/dev/null || exit 1
for g in 4096 8192; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 100 --global-batch $g $B > gpurun_out/${T}_b$g.json 2>/dev/null || exit 1
done
python3 - $T <<'PY'
import json, sys
t = sys.argv[1]
for g in (65536, 4096, 8192):
    d = json.loads(open(f"gpurun_out/{t}_b{g}.json").read().strip().splitlines()[-1])
    print(g, round(d["value"] / 1e6, 1), "M QP/s", round(d["ms_per_step"] * 1e3, 1), "us/step",
          {k[:40]: round(v * 1e3, 1) for k, v in d["config"]["kernel_ms"].items()})
PY
