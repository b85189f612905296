#!/bin/bash
# CPU side of tools/r03_evidence.sh: turn gpurun_out/ev_TAG into the tracked profiles/ set
# (headline trace + traffic summary, executed-FP64 / MFMA counters, config C and E traffic and
# counters, the B-standing trace, the bench line).  Usage: tools/summarize_evidence.sh TAG
set -e
T=$1; O=gpurun_out/ev_$T
KB='k_mpc_pair<6, 10, 0, false>'; KC='k_mpc<6, 20, 0, true, 60>'; KE='k_dense_wg<24, 6, 16, true>'
python3 tools/summarize_profile.py $O/B $T --kernel "$KB" --grid 2097152
python3 tools/summarize_flops.py $O/B_flops $T --kernel "$KB" --grid 2097152
python3 tools/summarize_traffic.py $O/C $T --config C --batch 65536 --kernel "$KC" --grid 4194304
python3 tools/summarize_flops.py $O/C_flops $T --kernel "$KC" --config C --batch 65536 --grid 4194304 --out pmc_flops_C.json
python3 tools/summarize_traffic.py $O/E $T --config E --batch 16384 --kernel "$KE" --grid 4194304
python3 tools/summarize_flops.py $O/E_flops $T --kernel "$KE" --config E --batch 16384 --grid 4194304 --out pmc_flops_E.json
python3 tools/summarize_profile.py $O/Bst ${T}_Bstanding --kernel "$KB" --grid 2097152
cp $O/bench.json profiles/${T}_bench.json
for c in C E; do cp $O/$c/trace/run_kernel_stats.csv profiles/${T}_${c}_kernel_stats.csv; done
echo "profiles/ updated for $T"
