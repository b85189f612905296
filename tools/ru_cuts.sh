#!/bin/bash
# Register use of k_mpc truncated after each phase (compile-time cut), to locate pressure.
# Usage: tools/ru_cuts.sh [kernel-regex]   (CPU only; hipcc cross-compiles)
set -e
PAT=${1:-'k_mpcILi6ELi(10|20)ELi0ELb0ELi(32|64)'}
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
mkdir -p "$W/pkg" "$W/include"
cp -r "$R/mpc-limx-control_amd/csrc" "$W/pkg/"
cp "$R/include/mpcqp.h" "$W/include/"
cd "$W/pkg/csrc"
sed -i 's/MPCQP_CUT(a.cut,/MPCQP_CUT(FCUT,/; s/C.cut = a.cut;/C.cut = FCUT;/; s/if (a.cut >= 4 \&\& a.cut <= 7) return;/if (FCUT >= 4 \&\& FCUT <= 7) return;/' mpc_fused.hpp
for k in 1 2 3 4 5 6 7 0; do
  (/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=1000000 \
     -DMPCQP_CUTS -DFCUT=$k -Rpass-analysis=kernel-resource-usage -c -o "$W/c$k.o" mpcqp_kernels.hip \
     > "$W/ru_$k.txt" 2>&1) &
done
wait
for k in 1 2 3 4 5 6 7 0; do
  echo "cut $k: $(grep -A8 -E "$PAT" "$W/ru_$k.txt" | grep -E 'VGPRs:|AGPRs:|Scratch' | sed 's/.*remark: //;s/\[-Rpass.*//;s/ \[bytes\/lane\]//' | tr -s ' ' | tr '\n' ' ')"
done
rm -rf "$W"
