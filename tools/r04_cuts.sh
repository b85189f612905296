#!/bin/bash
# Per-phase kernel time by early exit (lib/libmpcqp_cuts.so, `make cuts`): config C's one-QP
# kernel and config B's paired kernel (crash = cut 8).  Usage: tools/r04_cuts.sh OUTPREFIX
O=${1:-gpurun_out/r04cuts}
timeout -k 10 200 python tools/phase_cuts.py --configs C --reps 8 > ${O}_C.log 2>&1 || exit 1
timeout -k 10 200 python tools/phase_cuts.py --configs B --reps 8 --cuts 1,2,3,4,6,8,7,0 > ${O}_B.log 2>&1 || exit 1
echo cuts done
