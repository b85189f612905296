#!/bin/bash
# CPU side of tools/evidence.sh: gpurun_out/ev_TAG -> the tracked profiles/ set.  Every
# summary is keyed by (kernel instantiation, grid): the headline (B), configs C and E, and the
# B-standing trace.  Usage: tools/summarize_evidence.sh TAG
set -e
T=$1; O=gpurun_out/ev_$T
# the library the GPU run profiled (its bench line), not whatever is built in-tree now
export MPCQP_PROFILED_BUILD_ID=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['lib_build_id'])" $O/bench.json)
KB='k_mpc_pair<6, 10, 0, false, 4>'; KC='k_mpc<6, 20, 0, true, 60>'; KE='k_dense_wg<24, 6, 16, true>'
python3 tools/summarize_profile.py $O/B $T --kernel "$KB" --grid 2097152
python3 tools/summarize_flops.py $O/B_flops $T --kernel "$KB" --grid 2097152
python3 tools/summarize_profile.py $O/C ${T}_C --config C --batch 65536 --kernel "$KC" --grid 4194304 --no-traffic-json
python3 tools/summarize_traffic.py $O/C $T --config C --batch 65536 --kernel "$KC" --grid 4194304
python3 tools/summarize_flops.py $O/C_flops $T --kernel "$KC" --config C --batch 65536 --grid 4194304 --out pmc_flops_C.json
python3 tools/summarize_profile.py $O/E ${T}_E --config E --batch 16384 --kernel "$KE" --grid 4194304 --no-traffic-json
python3 tools/summarize_traffic.py $O/E $T --config E --batch 16384 --kernel "$KE" --grid 4194304
python3 tools/summarize_flops.py $O/E_flops $T --kernel "$KE" --config E --batch 16384 --grid 4194304 --out pmc_flops_E.json
python3 tools/summarize_profile.py $O/Bst ${T}_Bstanding --kernel "$KB" --grid 2097152 --no-traffic-json
python3 tools/summarize_stall.py $O/B_stall $T --kernel "$KB"
python3 tools/summarize_stall.py $O/C_stall ${T}_C --kernel "$KC" --grid 4194304
python3 tools/summarize_stall.py $O/E_stall ${T}_E --kernel "$KE" --grid 4194304
cp $O/bench.json profiles/${T}_bench.json
echo "profiles/ updated for $T"
