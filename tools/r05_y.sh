#!/bin/bash
# r05: wave-priority A/B -- E and B standing with the one-wave serial stages at raised priority
# (MPCQP_SERIAL_PRIO), the paired kernel with raised priority during its inputs / from its
# crash start (MPCQP_PAIR_PRIO 1 / 2)
set -o pipefail
T=${1:-r05y}
mkdir -p gpurun_out
for r in 1 2 3; do
  AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384 bash tools/ab_libs.sh default prio_e
  AB_CONFIGS=C AB_GAIT=mixed AB_REPS=3 bash tools/ab_libs.sh default prio_w
  AB_CONFIGS=B AB_REPS=60 bash tools/ab_libs.sh default prio1 prio2
  AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60 bash tools/ab_libs.sh default prio1 prio2
done > gpurun_out/${T}_ab.log 2>&1 || exit 1
cat gpurun_out/${T}_ab.log
