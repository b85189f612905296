#!/bin/bash
# GPU box: the bench line as the driver runs it (20 steps after 5 warm-up), GPU tests first.
O=${1:-gpurun_out/r04drv}
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > ${O}_tests.log 2>&1 || { echo tests failed; tail -5 ${O}_tests.log; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > ${O}_bench.log 2>&1 || exit 1
grep '^{' ${O}_bench.log > ${O}_bench.json
echo drv done
