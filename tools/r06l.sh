# round 6: per-step kernel chain at the headline batch (gaps between launches), fused selection
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tr_r06l -o run --output-format csv -- python3 tools/step_trace.py --batch 65536 --steps 12 > gpurun_out/r06l_tr.log 2>&1 || exit 1
f=$(find gpurun_out/tr_r06l -name "run_kernel_trace.csv" | head -1)
python3 tools/step_trace.py --analyze "$f"
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tr_r06l8 -o run --output-format csv -- python3 tools/step_trace.py --batch 8192 --steps 12 > gpurun_out/r06l_tr8.log 2>&1 || exit 1
f=$(find gpurun_out/tr_r06l8 -name "run_kernel_trace.csv" | head -1)
python3 tools/step_trace.py --analyze "$f"
