#!/bin/bash
# GPU box: instruction mix / instruction-cache counters of config E with the workgroup crash
# on / off (two PMC passes each).  Usage: tools/r04_pmcE.sh OUT
O=${1:-gpurun_out/r04pe}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -io "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*" $O/avail.txt | sort -u > $O/icache_ctrs.txt || true
CONFIG=E BATCHES=16384 bash tools/pmc_env_ab.sh $O/p1 MPCQP_CRASH_P_WG=0 MPCQP_CRASH_P_WG=12 || exit 1
IC=$(head -4 $O/icache_ctrs.txt | tr '\n' ' ')
CTRS="SQ_WAVES SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU $IC" CONFIG=E BATCHES=16384 bash tools/pmc_env_ab.sh $O/p2 MPCQP_CRASH_P_WG=0 MPCQP_CRASH_P_WG=12 || exit 1
echo pe done
