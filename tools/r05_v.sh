#!/bin/bash
# r05: GPU suite and the default bench line (driver-style 20 / 5 and a 200 / 100 steady run)
set -o pipefail
T=${1:-r05v}
mkdir -p gpurun_out
TAG=$T bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 200 --warmup 100 --no-per-config --no-host-path > gpurun_out/${T}_long.json 2> gpurun_out/${T}_long.err || exit 1
timeout -k 10 500 python3 bench.py > gpurun_out/${T}_drv.json 2> gpurun_out/${T}_drv.err || exit 1
python3 - gpurun_out/${T}_long.json gpurun_out/${T}_drv.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    r = d["roofline"]
    print(f, "value %.1f M" % (d["value"] / 1e6), "ms/step %.4f" % d["ms_per_step"], "kernel %.4f" % r["kernel_ms"],
          "frac %.4f" % r["frac"], "lane_eff", r.get("lane_efficiency"))
    pc = d["config"].get("per_config") or {}
    for k, v in pc.items():
        print("   ", k, "%.4f ms" % v.get("kernel_ms", float("nan")))
PY
