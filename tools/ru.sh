#!/bin/bash
# register / scratch / occupancy summary per kernel of one translation unit:  tools/ru.sh csrc/X.hip [extra hipcc flags]
cd "$(dirname "$0")/../mpc-limx-control_amd"
SRC=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-value \
  -Wno-unused-variable -mllvm -pragma-unroll-threshold=1000000 "$@" -c "$SRC" -o /tmp/ru_$$.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys, re
cur = None
for line in sys.stdin:
    m = re.search(r"remark: (?:\s*)(.*?) \[-Rpass", line)
    if not m: continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip(); print(); print(cur[:90], end="")
    elif cur and any(t.startswith(k) for k in ("VGPRs:", "AGPRs:", "ScratchSize", "Occupancy", "VGPRs Spill", "SGPRs Spill")):
        print(" |", t, end="")
print()'
rm -f /tmp/ru_$$.o
