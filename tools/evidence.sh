#!/bin/bash
# Evidence set at the current library (GPU box, repo root), all tagged TAG:
#   gpurun_out/ev_TAG/bench.json            the default bench line (cpu baseline, per-config)
#   gpurun_out/ev_TAG/B/{trace,fetch,write} headline k_mpc_pair: kernel trace + HBM passes
#   gpurun_out/ev_TAG/B_flops/{sq,grbm}     executed FP64 / MFMA counters of the headline
#   gpurun_out/ev_TAG/{C,E}/{trace,fetch,write}, {C,E}_flops
#                                           configs C (65,536) and E (16,384), driven by
#                                           tools/time_kernel.py: the trace's (kernel, grid) group
#                                           is the launch per_config.kernel_ms times
#   gpurun_out/ev_TAG/Bst/trace             k_mpc_pair + k_mpc_list at B standing (overflow path)
#   gpurun_out/ev_TAG/{B,C,E}_stall          stall / issue counters (tools/pmc_stall.sh)
# Summaries are written on the CPU afterwards (tools/summarize_evidence.sh).  Counter passes
# never share a run with trace domains.
set -o pipefail
TAG=${1:-r05}
O=gpurun_out/ev_$TAG
mkdir -p $O
export TMPDIR=/tmp
R=$(pwd)
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -n 5 $O/$n.log; exit 1; }
}
run bench 500 python3 bench.py
grep '^{' $O/bench.log > $O/bench.json
# headline passes: a long warm-up so that the traced launches run at steady clocks, and no
# host-path lines (they launch the same kernel and grid between PCIe copies)
HB="--steps 20 --warmup ${HB_WARMUP:-100} --no-cpu-baseline --no-per-config --no-host-path"
run B_trace 300 rocprofv3 --kernel-trace --stats -d $R/$O/B/trace -o run --output-format csv -- python3 bench.py $HB
run B_fetch 200 rocprofv3 --pmc FETCH_SIZE -d $R/$O/B/fetch -o run --output-format csv -- python3 bench.py $HB
run B_write 200 rocprofv3 --pmc WRITE_SIZE -d $R/$O/B/write -o run --output-format csv -- python3 bench.py $HB
run B_flops 400 bash tools/pmc_flops.sh $O/B_flops $HB
for spec in "C:--configs C --batch 65536" "E:--configs E --batch 16384"; do
  c=${spec%%:*}; a="${spec#*:}"
  run ${c}_trace 300 rocprofv3 --kernel-trace --stats -d $R/$O/$c/trace -o run --output-format csv -- python3 tools/time_kernel.py $a --reps 40
  run ${c}_fetch 200 rocprofv3 --pmc FETCH_SIZE -d $R/$O/$c/fetch -o run --output-format csv -- python3 tools/time_kernel.py $a --reps 5
  run ${c}_write 200 rocprofv3 --pmc WRITE_SIZE -d $R/$O/$c/write -o run --output-format csv -- python3 tools/time_kernel.py $a --reps 5
  run ${c}_flops 400 bash tools/pmc_flops.sh $O/${c}_flops --driver "tools/time_kernel.py $a --reps 5"
done
run B_stall 400 bash tools/pmc_stall.sh $O/B_stall
run C_stall 400 bash tools/pmc_stall.sh $O/C_stall --driver "tools/time_kernel.py --configs C --batch 65536 --reps 5"
run E_stall 400 bash tools/pmc_stall.sh $O/E_stall --driver "tools/time_kernel.py --configs E --batch 16384 --reps 5"
run Bst_trace 300 rocprofv3 --kernel-trace --stats -d $R/$O/Bst/trace -o run --output-format csv -- python3 tools/time_kernel.py --configs B --gait standing --reps 10
echo "evidence $TAG OK"
