#!/bin/bash
# Build A/B variants of the paired kernel's translation unit (CPU; hipcc cross-compiles):
#   [TU=fast_dense] tools/build_variants.sh name1:"-DFLAG=1" name2:"" ...
# Each variant relinks the release objects with its own fast_pair.o into
# lib/libmpcqp_<name>.so (time them on the GPU box with tools/ab_libs.sh) and prints the
# compiler's VGPR spill count for the config B kernel.
R=$(cd "$(dirname "$0")/.." && pwd)
TU=${TU:-fast_pair}
cd "$R/mpc-limx-control_amd" || exit 1
HF="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -mllvm -pragma-unroll-threshold=1000000"
[ -n "$NOILP" ] || HF="$HF -mllvm -amdgpu-sched-strategy=max-ilp"  # NOILP=1: the default scheduler
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  # the variant's flags go into mpcqp_build_id() (PMC summaries of variants stay distinct)
  flags="$flags -DMPCQP_VARIANT_TAG=\"$name-$(echo "$TU $flags" | sha1sum | cut -c1-8)\""
  ( mkdir -p "build/$name" && /opt/rocm/bin/hipcc $HF $flags -c -o "build/$name/$TU.o" csrc/$TU.hip && \
    /opt/rocm/bin/hipcc $HF -shared -o "lib/libmpcqp_$name.so" $(ls build/rel/*.o | grep -v $TU.o) \
        "build/$name/$TU.o" -L/opt/rocm/lib -lrccl && \
    echo "$name $(/opt/rocm/bin/hipcc $HF $flags -Rpass-analysis=kernel-resource-usage --cuda-device-only -c \
        -o "/tmp/ru_$name.o" csrc/$TU.hip 2>&1 | grep -E 'VGPRs Spill' | head -1 \
        | sed 's/.*remark://;s/\[-R.*//')" ) &
done
wait
