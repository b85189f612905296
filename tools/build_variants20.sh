#!/bin/bash
# A/B variants of the N = 20 one-wave kernels (fast_srbm20.hip + fast_literal.hip):
#   tools/build_variants20.sh name1:"-DFLAG=1" ...  -> lib/libmpcqp_<name>.so (tools/ab_libs.sh)
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R/mpc-limx-control_amd" || exit 1
HF="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -mllvm -pragma-unroll-threshold=1000000"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( mkdir -p "build/$name" && /opt/rocm/bin/hipcc $HF $flags -c -o "build/$name/fast_srbm20.o" csrc/fast_srbm20.hip && \
    /opt/rocm/bin/hipcc $HF $flags -c -o "build/$name/fast_literal.o" csrc/fast_literal.hip && \
    /opt/rocm/bin/hipcc $HF -shared -o "lib/libmpcqp_$name.so" build/rel/mpcqp_kernels.o build/rel/estimator.o \
        build/rel/fast_srbm10.o "build/$name/fast_srbm20.o" "build/$name/fast_literal.o" build/rel/fast_pair.o \
        build/rel/fast_wg.o build/rel/fast_dense.o && echo "$name built" ) &
done
wait
