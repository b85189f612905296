#!/bin/bash
# Named GPU-box runs behind DESIGN.md's measurements (run from the repo root on the box):
#   bash tools/runs.sh <name> [tag]
# Output goes to gpurun_out/<tag>*.  The A/B runs alternate processes between the default
# library and variant libraries built here by tools/build_variants.sh (lib/libmpcqp_<v>.so):
#   tools/build_variants.sh nofold:-DMPCQP_PAIR_FOLD=0 foldasel:-DMPCQP_FOLD_ASEL=0 \
#       hbbases:-DMPCQP_HB_BASES=0
#   TU=fast_srbm20 tools/build_variants.sh diagrl_c:-DMPCQP_DIAG_DPP=0 noelide_c:-DMPCQP_ELIDE_FZ=0
#   TU=fast_dense  tools/build_variants.sh diagrl_e:-DMPCQP_DIAG_DPP=0 padelate_e:-DMPCQP_PADE_LATE=0
#   TU=fast_wg     tools/build_variants.sh diagrl_w:-DMPCQP_DIAG_DPP=0 ovfwg:-DMPCQP_OVF_ONEWAVE=0
#   NOILP=1 [TU=...] tools/build_variants.sh noilp_b: / noilp_c: / noilp_e:
#   [TU=...] tools/build_variants.sh sb_<s>:"-mllvm -amdgpu-sched-strategy=<s>" (sc_ / se_ likewise)
# (the flags' current defaults are the kept side; variants whose code was removed after a
#  negative result -- oldcrash, cpairs, pmfma, rpnew / rpasel, gj2, inc / kc10, padesw_e, prio1 / prio2 / prio_e / prio_w -- are in git history)
set -o pipefail
NAME=${1:?usage: tools/runs.sh <name> [tag]}
T=${2:-$NAME}
mkdir -p gpurun_out

rep() { local n=$1; shift; for r in $(seq "$n"); do "$@" || return 1; done; }
abl() { local e=$1; shift; env $e bash tools/ab_libs.sh "$@"; }  # one tools/ab_libs.sh round
# the paired kernel at the headline batch and at a 16-way shard; configs C and E
ab_b() { abl "AB_CONFIGS=B AB_REPS=60" default "$@" && abl "AB_CONFIGS=B AB_BATCH=4096 AB_REPS=60" default "$@"; }
ab_c() { abl "AB_CONFIGS=C AB_REPS=20" "$@"; }
ab_e() { abl "AB_CONFIGS=E AB_REPS=10 AB_BATCH=16384" "$@"; }
diag_round() { ab_c default diagrl_c && ab_e default diagrl_e &&
               abl "AB_CONFIGS=B AB_GAIT=standing AB_REPS=10" default diagrl_w; }
elide_round() { ab_c default noelide_c && ab_e default padeskip0_e; }
noilp_round() { ab_e noilp_e noilplate_e && ab_c default noilp_c && abl "AB_CONFIGS=B AB_REPS=60" default noilp_b; }
sched_round() { abl "AB_CONFIGS=B AB_REPS=60" default sb_max-memory-clause sb_iterative-ilp sb_iterative-minreg &&
                ab_c default sc_max-memory-clause sc_iterative-ilp sc_iterative-minreg &&
                ab_e default se_max-memory-clause se_iterative-ilp se_iterative-minreg; }
prio_round() { ab_e default prio_e && abl "AB_CONFIGS=C AB_GAIT=mixed AB_REPS=3" default prio_w && ab_b prio1 prio2; }
overflow_ab() { for g in standing double alternating; do
                  rep 2 abl "AB_CONFIGS=B AB_GAIT=$g AB_REPS=10" default ovfwg || return 1; done; }
pair_tests() {  # the paired-kernel tests with a variant as the library under test
  MPCQP_LIB=$PWD/mpc-limx-control_amd/lib/libmpcqp_$1.so TAG=$T \
    bash tools/gpu_tests.sh -k "pair or batch_vs_oracle or gait or crash or flops"
}
log() { "$@" > "gpurun_out/${T}_ab.log" 2>&1; local s=$?; cat "gpurun_out/${T}_ab.log"; return $s; }

case "$NAME" in
  suite)      # the GPU suite (tools/gpu_tests.sh)
    TAG=$T bash tools/gpu_tests.sh ;;
  bench)      # the bench line driver-style (20 / 5) and steady state (200 / 100)
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 100 --no-per-config --no-host-path \
      > gpurun_out/${T}_long.json 2> gpurun_out/${T}_long.err &&
    timeout -k 10 500 python3 bench.py > gpurun_out/${T}_drv.json 2> gpurun_out/${T}_drv.err ;;
  shards)     # DESIGN §5's shard table and the bench step at --global-batch 8,192 / 4,096
    { timeout -k 10 300 python3 tools/shard_sweep.py --sizes 2048,4096,6144,8192,12288,65536 --reps 50 &&
      for g in 8192 4096; do
        timeout -k 10 300 python3 bench.py --global-batch $g --no-per-config --no-host-path \
          --no-cpu-baseline > gpurun_out/${T}_b$g.json || exit 1
      done; } > gpurun_out/${T}.txt 2>&1 ;;
  smalltrace) # kernel trace of the shard sweep: the GPU's own durations at small shards
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_st -o run \
      --output-format csv -- python3 tools/shard_sweep.py --sizes 512,2048,4096,8192,65536 --reps 40 \
      > gpurun_out/${T}_st.log 2>&1 ;;
  stall)      # stall / issue profiles: headline B, config C, config E
    bash tools/pmc_stall.sh gpurun_out/st_$T/B &&
    bash tools/pmc_stall.sh gpurun_out/st_$T/C --driver "tools/time_kernel.py --configs C --batch 65536 --reps 5" &&
    bash tools/pmc_stall.sh gpurun_out/st_$T/E --driver "tools/time_kernel.py --configs E --batch 16384 --reps 5" ;;
  census)     # k_mpc_pair per-phase PMC census and early-exit cut times (config B)
    bash tools/phase_pmc_pair.sh gpurun_out/pp_$T B > gpurun_out/${T}_census.txt 2>&1 &&
    timeout -k 10 300 python3 tools/phase_cuts.py --configs B --reps 20 --cuts 11,1,13,2,3,4,6,8,7,0 \
      > gpurun_out/${T}_cuts.txt 2>&1 ;;
  phases-ce)  # configs C and E: per-phase stamps (stamps build) and C's early-exit cuts
    { timeout -k 10 120 python3 tools/phase_profile.py --config C &&
      timeout -k 10 120 python3 tools/phase_profile.py --config E --batch 16384 &&
      timeout -k 10 300 python3 tools/phase_cuts.py --configs C --reps 10 --cuts 11,13,1,2,3,4,6,7,0; } \
      > gpurun_out/${T}_phases.txt 2>&1 ;;
  # ---- round-5 A/Bs (profiles/ab_r05*.log); variants from tools/build_variants.sh
  fold)        log rep 3 ab_b nofold ;;                # folded Cholesky + J sweep
  crash-dpp)   log rep 3 ab_b oldcrash ;;              # DPP vs LDS crash
  diag-dpp)    log rep 3 diag_round ;;                 # DPP diagonal blocks (C, E, B standing)
  elide-fz)    log rep 3 elide_round ;;                # implied fz bound (C); Pade swap guard (E)
  overflow)    log overflow_ab ;;                      # overflow on k_mpc_list vs the workgroup kernel
  pade)        (cd tools/micro && timeout -k 10 60 ./pade_bench 256 4 && timeout -k 10 60 ./pade_bench 16384 2) &&
               log rep 3 ab_e default padesw_e ;;      # Pade micro-benchmark; swap form
  pade-late)   log rep 3 ab_e default noilp_e padelate_e ;;  # late column read; scheduler (E)
  noilp)       log rep 3 noilp_round ;;                # default scheduler instead of max-ilp
  sched)       log rep 2 sched_round ;;                # machine-scheduler strategies
  prio)        log rep 3 prio_round ;;                 # wave priority
  fold-asel)   log rep 3 ab_b foldasel ;;              # folded rows from a selected address
  hb-bases)    log rep 3 ab_b hbbases && pair_tests hbbases ;;  # H-build sub-block bases
  crash-pairs) log rep 3 ab_b cpairs && pair_tests cpairs ;;    # crash Gram by entry pairs
  pair-mfma)   pair_tests pmfma && log rep 3 ab_b pmfma ;;      # paired factorisation on MFMA
  rowpair)     pair_tests rpnew && log rep 3 ab_b rpnew rpasel ;;  # DPP64 broadcasts, lane-mask selects
  crash-gj2)   timeout -k 10 300 python3 tools/cmp_libs.py mpc-limx-control_amd/lib/libmpcqp.so mpc-limx-control_amd/lib/libmpcqp_gj2.so &&
               log rep 3 ab_b gj2 ;;                   # crash Gauss-Jordan, two pivots per round trip
  pair-sort)   log rep 3 ab_b nosort ;;                 # schedule-sorted pairing off (nosort: -DMPCQP_PAIR_SORT=0)
  toep-pipe)   log rep 3 ab_e default toeppipe_e ;;     # E: software-pipelined Toeplitz tiles (NOILP=1 TU=fast_dense toeppipe_e:-DMPCQP_TOEP_PIPE=1)
  wg-crash-k)  log rep 3 ab_e default kc24_e kc16_e ;;   # E: workgroup crash KC (NOILP=1 TU=fast_dense kc24_e:-DMPCQP_WG_CRASH_K=24 ...)
  *) echo "unknown run: $NAME" >&2; exit 2 ;;
esac
