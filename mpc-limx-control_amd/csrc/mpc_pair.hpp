// mpc_pair.hpp -- the fused per-tick step of mpc_fused.hpp with TWO QP instances per
// wavefront: lanes 0-31 own instance 2w, lanes 32-63 instance 2w+1.
//
// Reference: mpcQP::mpcQP + buildSystemModel (include/mpcQP.h:35-119, 121-182),
// QPSolver::discretizeSystem / buildQPParams / solveQP (src/QPSolver.cpp:21-106).
//
// For problems with at most 30 free variables -- config B (SRBM 13/6/10: the gait has one
// stance foot per horizon step, nf = 30) and the reference-literal 13/3/10 model (nf = 30) --
// the one-QP-per-wave kernel leaves lanes 32-63 idle through the factorisation, the inverse
// and the dual loop, and an FP64 wave instruction costs 4 cycles however many lanes it uses.
// Here every lane-parallel phase serves two instances for the same instruction count:
//   * lane l of a half owns row l of H_FF / L and row l of J (30 columns in registers); lane
//     31 of each half carries g through the inverse sweep (t = L^-1 g), as lane 63 does in
//     gi_reg.hpp; the Cholesky and the inverse sweep run fused (one LDS column read per step
//     feeds both)
//   * broadcasts are LDS reads at a per-half address (one address per half); cross-lane reads
//     at a constant index are DPP row_newbcast + v_permlane16_swap (half_ops.hpp)
//   * reductions: DPP inside each 16-lane row, then v_permlane16_swap across the half's rows
//   * the dual loop runs while either half is active; each half's state (q, iterations,
//     status, the selected constraint) lives in VGPRs and a finished half idles (EXEC-masked);
//     the bound states live in the owning lane's registers, the add step is a Householder
//     reflection (see the loop)
// Same algorithm, constraint order and tolerances as fast_mpc + gi_run_reg (the add step's
// reflection differs from their Givens chain only in rounding), so results match the
// one-QP kernel and the CPU oracle to rounding and iteration counts agree.
//
// LDS per instance (config B): 5.6 KB -- the early model terms keep only the support rows of
// X0 / X1 and no [Ac | Bc] copy, the condensed linear terms die before the packed H is built
// over them, and the bounds live in registers -- so three waves (six QPs) per SIMD fit in
// 160 KB.
#pragma once
#include "half_ops.hpp"
#include "mpc_fused.hpp"

namespace mpcqp {

// LDS loads in flight per step of the unrolled sweeps (a code-motion fence every PF elements):
// larger hides more LDS latency behind the FMAs, smaller bounds the registers the loads hold
// (the kernel comes in two register budgets, W = 3 and 4 waves per SIMD (fast_pair.hip); the
//  4-wave build keeps fewer LDS loads in flight per fence: PFD overrides both)
template <int W>
constexpr int pair_pf() {
#ifdef MPCQP_PF_DUAL
    return MPCQP_PF_DUAL;
#else
    return W >= 4 ? 4 : 8;
#endif
}
// Cholesky + inverse: columns per LDS round trip, and the fence period of its trailing update
// pair instances by contact schedule within aligned groups of 16 (see pair_sorted_instance)
#ifndef MPCQP_PAIR_SORT
#define MPCQP_PAIR_SORT 1
#endif
#ifndef MPCQP_CHOL_CB
#define MPCQP_CHOL_CB 2
#endif
#ifndef MPCQP_CHOL_PF
#define MPCQP_CHOL_PF 4
#endif
// Cholesky and J = L^-T folded into one register row per lane (see the sweep); 0 keeps the
// fused two-array sweep (A/B builds)
#ifndef MPCQP_PAIR_FOLD
#define MPCQP_PAIR_FOLD 1
#endif
// the folded sweep's rows load from a per-slot selected address (one LDS read per slot) instead
// of reading both candidates and selecting the value (A/B)
// MPCQP_FOLD_LMASK: the row load's lower / upper choice (q <= l) by a constant lane mask per
// slot (no v_cmp of the lane index): fewer VALU, measured neutral (r06p); 0: the compare
#ifndef MPCQP_FOLD_LMASK
#define MPCQP_FOLD_LMASK 0
#endif
// MPCQP_PAIR_CRASH_RCP: the crash's Gauss-Jordan pivot reciprocal from v_rcp_f64 and two Newton
// steps (5 VALU instead of the ~12 of the IEEE division; the pivots are positive and normal or
// the half gives up), and w = r / pivot as r times that reciprocal; 0: IEEE divisions (A/B)
#ifndef MPCQP_PAIR_CRASH_RCP
#define MPCQP_PAIR_CRASH_RCP 1
#endif
// MPCQP_PAIR_SLOOP: the S blocks' loop with the lane's entries outermost (see pair_mpc):
// 260.2 -> 253.4 us at 65,536, 58.7 -> 57.8 us at 8,192 (r06t, profiles/ab_r06t_*)
#ifndef MPCQP_PAIR_SLOOP
#define MPCQP_PAIR_SLOOP 1
#endif
// MPCQP_CRASH_LSEL: the crash's Gauss-Jordan updates unmasked with a zero multiplier on the
// lanes that do not eliminate (one select per step instead of one per updated entry): +0.3 % at
// 65,536 but -0.7 % at 8,192 (r06t), off; 0: the masked update
#ifndef MPCQP_CRASH_LSEL
#define MPCQP_CRASH_LSEL 0
#endif
#ifndef MPCQP_FOLD_ASEL
#define MPCQP_FOLD_ASEL 1
#endif
// the H build's sub-blocks address their entries from per-sub-block bases (compile-time offsets),
// and g's terms are masked by an FMA with 0 / 1 instead of a value select (A/B)
#ifndef MPCQP_HB_BASES
#define MPCQP_HB_BASES 1
#endif
// the dual loop keeps R^-1 instead of R (r = R^-1 d as a lane-parallel product, no serial
// back substitution); 0 keeps R (A/B builds)
#ifndef MPCQP_PAIR_RINV
#define MPCQP_PAIR_RINV 1
#endif
// speculative primal-dual active-set start before the dual loop (see the crash block below);
// 0 = plain Goldfarb-Idnani from the unconstrained minimum (A/B builds)
#ifndef MPCQP_PAIR_CRASH
#define MPCQP_PAIR_CRASH 1
#endif

constexpr int kPairNF = 30;  // free variables per instance; lane 31 of a half carries g

// a code-motion fence inside an unrolled dot product over an LDS buffer, with the four partial
// sums pinned in registers: the compiler can neither hoist the later loads above it nor sink the
// FMAs below it, so at most one fence period of loads is in flight (the loops' register peak)
__device__ __forceinline__ void pin_fence4(double (&s4)[4]) {
    pin(s4[0]);
    pin(s4[1]);
    pin(s4[2]);
    pin(s4[3]);
    step_fence();
}
// crash start (below): bounds per working set, working sets before giving up
#ifndef MPCQP_CRASH_K
#define MPCQP_CRASH_K 12
#endif
#ifndef MPCQP_CRASH_P
#define MPCQP_CRASH_P 8
#endif
constexpr int kPairCrashK = MPCQP_CRASH_K, kPairCrashP = MPCQP_CRASH_P;

template <int NU, int N, int MODEL>
struct PairLayout {
    static constexpr int NX = 13, NF = kPairNF, NV = NU * N, NP = kHalf;
    using Sup = XSupport<MODEL>;
    static constexpr int SD = Sup::x0hi - Sup::x0lo;
    static constexpr int NR = RegPack<NF>::doubles;  // packed L / R
    static constexpr int HB = NF * (NF + 1) / 2;     // packed H_FF
    // doubles; one region, in turn:
    //   early   : X0, X1 support rows, A x0, A^2 x0, xref, x0, then u_m / v_m   [oU, eUV)
    //   H build : packed H [oU, oU + HB) over the dead early view; S after it (R and the Q / P
    //             diagonals are read from global memory, not staged per instance)
    //   solver  : packed R^-1 [oU, oU + HB) (crash: the published J rows), then the broadcast
    //             buffers over the dead S: buf | colb | rot (2 NP) | a zero slot
    // then bytes: the parked contact mask and instance index, the free map (int8: fid[NF],
    // pos[NV]).  5 KB per instance at config B: 16 waves (32 instances) fit a CU's 160 KB.
    static constexpr int oU = 0;
    static constexpr int oX0 = oU;                       // [NU][SD]
    static constexpr int oX1 = oX0 + NU * SD;            // [NU][SD]
    static constexpr int oAx = oX1 + NU * SD;            // NX
    static constexpr int oA2x = oAx + NX;                // NX
    static constexpr int oXr = oA2x + NX;                // NX (N+1), Eigen column-major
    static constexpr int oX0v = oXr + NX * (N + 1);      // NX
    static constexpr int oUV = oX0v + NX;                // [(N+1)][2][NU]
    static constexpr int eUV = oUV + (N + 1) * 2 * NU;
    static constexpr int oS = oU + ((HB > eUV - oU ? HB : eUV - oU) + 1) / 2 * 2;  // [NU*NU][4]
    static constexpr int eMid = oS + 4 * NU * NU;
    static constexpr int oR = oU;
    static constexpr int oDump = oU + HB;  // sink of the H build's masked-off stores (past H)
    // R^-1 packed needs HB doubles; the R form of the A/B build (MPCQP_PAIR_RINV=0) NR, with its
    // 1/R(j,j) buffer after the rotations
    static constexpr int oRow = (oR + (MPCQP_PAIR_RINV ? HB : NR) + 1) & ~1;  // buf | colb | rot
    // (+ 2: the dual loop's zero slot and the crash's objective slot)
    static constexpr int eLate = oRow + 4 * NP + (MPCQP_PAIR_RINV ? 2 : NP + 2);
    static constexpr int nDoubles = ((eMid > eLate ? eMid : eLate) + 1) & ~1;
    static constexpr size_t oCt = sizeof(double) * nDoubles;  // u64 contact mask, int64 index
    static constexpr size_t oFid = oCt + 16;                  // int8 [NF]: variable of slot p
    static constexpr size_t oPos = oFid + NF;                 // int8 [NV]: slot of variable v
    static constexpr size_t bytes = (oPos + NV + 15) & ~(size_t)15;
    static constexpr size_t lds_bytes = 2 * bytes;  // both halves
    static_assert(oU % 2 == 0 && oRow % 2 == 0 && oS % 2 == 0, "16-byte aligned buffers");
    static_assert(oDump < oRow && oDump >= eUV, "the dump slot is free during the H build");
    static_assert(NV < 128 && NF < 128, "int8 free map");
    static_assert(HB <= NR, "packed H fits the L / R space");
    static_assert(NV <= NR, "the U staging row fits the L / R space");
    static_assert(N <= kHalf, "one lane per horizon step in the gait mask");
};

// bounds of variable v from the contact schedule (gen_bound, gi_solver.hpp)
template <int NU, int MODEL>
__device__ __forceinline__ void pair_bound(const MpcArgs &a, uint64_t contact, int v, double &lo,
                                           double &hi) {
    if (MODEL == 1) { lo = a.u_min; hi = a.u_max; return; }
    const int k = v / NU, c = v % NU, s = c / 3, comp = c % 3;
    if ((contact >> (2 * k + s)) & 1ull) {
        if (comp == 2) { lo = a.fz_min; hi = a.fz_max; }
        else { lo = -a.fxy_max; hi = a.fxy_max; }
    } else { lo = 0.0; hi = 0.0; }
}
// gait_mask_wave per half: lane l < N of each half evaluates step l of its own instance
__device__ __forceinline__ uint64_t gait_mask_half(int N, double Ts, double phase0, float swing,
                                                   float stance) {
    const double cycle = (double)(swing + stance), sw = (double)swing;
    const int hl = lane() & (kHalf - 1);
    const double ph = fmod(phase0 + (double)hl * Ts, cycle);
    const uint64_t right = half_ballot(hl < N && ph < sw);
    const uint64_t left = half_ballot(hl < N && !(ph < sw));
    return spread_even(left) | (spread_even(right) << 1);
}

// Which instance each half solves.  A wave runs its dual loop until BOTH halves are done, so
// the halves should need the same number of iterations.  Instances are taken in aligned
// groups of 16 (the gait candidates of one state in the batch layout), sorted by contact
// schedule (the generated-input path: by gait phase within the cycle, which orders the
// schedules), ties by index; wave w of the group gets ranks 2w' and 2w'+1.  Candidates of
// one state with the same schedule are the same QP, so they land in the same wave.  Every
// instance is still solved and written at its own index; only the pairing changes.
// lane j of this lane's 16-lane row (DPP row_newbcast; j constant after unrolling)
__device__ __forceinline__ int row_bcast_u32(int v, int j) {
    switch (j) {
#define MPCQP_RB(i) case i: return __builtin_amdgcn_mov_dpp(v, 0x150 + i, 0xf, 0xf, false);
        MPCQP_RB(0) MPCQP_RB(1) MPCQP_RB(2) MPCQP_RB(3) MPCQP_RB(4) MPCQP_RB(5) MPCQP_RB(6)
        MPCQP_RB(7) MPCQP_RB(8) MPCQP_RB(9) MPCQP_RB(10) MPCQP_RB(11) MPCQP_RB(12) MPCQP_RB(13)
        MPCQP_RB(14) MPCQP_RB(15)
#undef MPCQP_RB
        default: return 0;
    }
}
template <bool GEN, int N>
__device__ __forceinline__ int pair_sorted_instance(const MpcArgs &a) {
    const int ln = lane(), c = ln & 15;
    const int wv = xcd_order((int)blockIdx.x, (int)gridDim.x);
    const int g0 = (2 * wv) & ~15;
    const int gn = a.B - g0 < 16 ? a.B - g0 : 16;
    int rank = 0;
    if constexpr (!GEN && 2 * N <= 32) {
        // the schedule's bits (2k + foot, k < N) fit 32 bits: one DPP move and one compare per
        // candidate (bits above 2N, if a caller sets any, only change the pairing, never a result)
        unsigned key = ~0u;
        if (c < gn) key = (unsigned)a.contact[g0 + c];
#pragma unroll
        for (int j = 0; j < 16; ++j) {  // row_newbcast: key j of this 16-lane row
            const unsigned kj = (unsigned)row_bcast_u32((int)key, j);
            rank += (j < gn && (kj < key || (kj == key && j < c))) ? 1 : 0;
        }
    } else {
        unsigned long long key = ~0ull;
        if (c < gn) {
            if constexpr (GEN) {
                const double cyc = (double)(a.swing + a.stance);
                key = (unsigned long long)__double_as_longlong(fmod(a.phase[g0 + c], cyc));
            } else {
                key = a.contact[g0 + c];
            }
        }
        const int klo = (int)(key & 0xffffffffull), khi = (int)(key >> 32);
#pragma unroll
        for (int j = 0; j < 16; ++j) {  // row_newbcast: key j of this 16-lane row
            const unsigned lo = (unsigned)row_bcast_u32(klo, j);
            const unsigned hi = (unsigned)row_bcast_u32(khi, j);
            const unsigned long long kj = ((unsigned long long)hi << 32) | lo;
            rank += (j < gn && (kj < key || (kj == key && j < c))) ? 1 : 0;
        }
    }
    // ranks 2w' (lower half) and 2w'+1 (upper half), both read off lanes 0-15 (row 0)
    const int r0 = (2 * wv) & 15;
    const unsigned m0 = (unsigned)(__ballot(ln < 16 && c < gn && rank == r0) & 0xffffull);
    const unsigned m1 = (unsigned)(__ballot(ln < 16 && c < gn && rank == r0 + 1) & 0xffffull);
    const unsigned m = ln >= kHalf ? m1 : m0;
    return m ? g0 + __builtin_ctz(m) : a.B;  // a.B: no instance (rank beyond a short group)
}

// ---- the folded sweep's trailing update (see pair_mpc): slot J of every lane -= the column's
// entry of row J, broadcast in the FMA itself (v_fmac_f64_dpp row_newbcast: lane J & 15 of each
// 16-lane row, from the row copy A -- lanes 0-15 of the half -- or B -- lanes 16-31 -- of
// row_pair), times the lane's own multiplier m.  Columns k (A0/B0, m0) and k + 1 (A1/B1, m1).
// The compiler does not form DPP FMAs itself (its VOP3 v_fma_f64 has no DPP); "s_nop 1" gives
// the DPP source its two wait states after the VALU that wrote it.
template <int J, bool NOP>
__device__ __forceinline__ void fold_dpp4(double &s0, double &s1, double &s2, double &s3,
                                          double A0, double B0, double m0, double A1, double B1,
                                          double m1) {
    if constexpr (NOP) asm volatile("s_nop 1");
    asm("v_fmac_f64_dpp %0, -%4, %12 row_newbcast:%c14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%5, %12 row_newbcast:%c15 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%6, %12 row_newbcast:%c16 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, -%7, %12 row_newbcast:%c17 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, -%8, %13 row_newbcast:%c14 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%9, %13 row_newbcast:%c15 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %2, -%10, %13 row_newbcast:%c16 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %3, -%11, %13 row_newbcast:%c17 row_mask:0xf bank_mask:0xf"
        : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3)
        : "v"(J < 16 ? A0 : B0), "v"(J + 1 < 16 ? A0 : B0), "v"(J + 2 < 16 ? A0 : B0),
          "v"(J + 3 < 16 ? A0 : B0), "v"(J < 16 ? A1 : B1), "v"(J + 1 < 16 ? A1 : B1),
          "v"(J + 2 < 16 ? A1 : B1), "v"(J + 3 < 16 ? A1 : B1), "v"(m0), "v"(m1),
          "i"(J & 15), "i"((J + 1) & 15), "i"((J + 2) & 15), "i"((J + 3) & 15));
}
template <int J, bool NOP>
__device__ __forceinline__ void fold_dpp2(double &s0, double &s1, double A0, double B0, double m0,
                                          double A1, double B1, double m1) {
    if constexpr (NOP) asm volatile("s_nop 1");
    asm("v_fmac_f64_dpp %0, -%2, %6 row_newbcast:%c8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%3, %6 row_newbcast:%c9 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %0, -%4, %7 row_newbcast:%c8 row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %1, -%5, %7 row_newbcast:%c9 row_mask:0xf bank_mask:0xf"
        : "+v"(s0), "+v"(s1)
        : "v"(J < 16 ? A0 : B0), "v"(J + 1 < 16 ? A0 : B0), "v"(J < 16 ? A1 : B1),
          "v"(J + 1 < 16 ? A1 : B1), "v"(m0), "v"(m1), "i"(J & 15), "i"((J + 1) & 15));
}
// one slot, one column (the in-panel update of column k + 1 by column k)
template <int J>
__device__ __forceinline__ void fold_dpp1(double &s, double A, double B, double m) {
    asm("s_nop 1\n\t"
        "v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%c3 row_mask:0xf bank_mask:0xf"
        : "+v"(s)
        : "v"(J < 16 ? A : B), "v"(m), "i"(J & 15));
}
// the trailing update of slots k + 2 .. NF - 1 for the column pair (k, k + 1)
template <int NF, int K, int J = K + 2>
__device__ __forceinline__ void fold_trailing(double (&s)[NF], double A0, double B0, double m0,
                                              double A1, double B1, double m1) {
    // (the DPP sources A / B were written before the step's first group: only that group
    //  needs the two wait states after the VALU that wrote them)
    if constexpr (J + 3 < NF) {
        fold_dpp4<J, J == K + 2>(s[J], s[J + 1], s[J + 2], s[J + 3], A0, B0, m0, A1, B1, m1);
        fold_trailing<NF, K, J + 4>(s, A0, B0, m0, A1, B1, m1);
    } else if constexpr (J + 1 < NF) {
        fold_dpp2<J, J == K + 2>(s[J], s[J + 1], A0, B0, m0, A1, B1, m1);
        fold_trailing<NF, K, J + 2>(s, A0, B0, m0, A1, B1, m1);
    }
}
template <int NF, int K = 0>
__device__ __forceinline__ void fold_in_panel(double (&s)[NF], double A, double B, double m, int k) {
    if constexpr (K + 1 < NF) {
        if (k == K) fold_dpp1<K + 1>(s[K + 1], A, B, m);
        else fold_in_panel<NF, K + 2>(s, A, B, m, k);
    }
}
template <int NF, int K = 0>
__device__ __forceinline__ void fold_trailing_k(double (&s)[NF], int k, double A0, double B0,
                                                double m0, double A1, double B1, double m1) {
    if constexpr (K + 2 < NF) {
        if (k == K) fold_trailing<NF, K>(s, A0, B0, m0, A1, B1, m1);
        else fold_trailing_k<NF, K + 2>(s, k, A0, B0, m0, A1, B1, m1);
    }
}

// textbook flops of one crash working-set solve with k bounds and of one dual pass with q
// constraints active, nf free variables (mpcqp/flops.py, the oracle's t_sflops): the diagnostic
// solver-flops counter (MpcArgs::flops_acc)
// (integers: a half's total stays far below 2^31 -- at most max_iter passes of ~6 k each)
__device__ __forceinline__ int crash_ws_flops_i(int nf, int k) {
    return k * (k + 1) * nf + (k - 1) * k * (k + 1) + 2 * k * nf + 2 * nf * nf + nf + 3 * k;
}
__device__ __forceinline__ int pass_flops_i(int nf, int q) {
    const int r = nf > q ? nf - q : 0;
    return q * q + 4 * nf + 6 * nf * r + 2 * nf + 3 * q;
}

template <int NU, int N, int MODEL, bool GEN, int W>
__device__ __forceinline__ void pair_mpc(const MpcArgs &a, unsigned char *smem) {
    // loads in flight per code-motion fence in the unrolled dot products over LDS buffers:
    // more hides more LDS latency, fewer bounds the registers the loads hold
    constexpr int PFD = pair_pf<W>(), PFG = pair_pf<W>();
    static_assert(!GEN || MODEL == 0, "generated inputs are defined for the SRBM model");
    static_assert(MODEL == 0 || MODEL == 1, "TRON1 models only");
    using Lay = PairLayout<NU, N, MODEL>;
    using Sup = XSupport<MODEL>;
    constexpr int NX = 13, NS = NX + NU, NF = kPairNF, NV = Lay::NV, SD = Lay::SD, NP = kHalf;
    MPCQP_STAMP_INIT(tst);
    const int ln = lane(), hl = ln & (kHalf - 1);
    const bool up = ln >= kHalf;
    int bq = 2 * xcd_order((int)blockIdx.x, (int)gridDim.x) + (up ? 1 : 0);
    if constexpr (MPCQP_PAIR_SORT && MODEL == 0) bq = pair_sorted_instance<GEN, N>(a);
    const bool valid = bq < a.B;
    const int b = valid ? bq : a.B - 1;  // the spare half of an odd batch re-reads the last QP
    [[maybe_unused]] const int b_ = b;
    unsigned char *Dbase = smem + (up ? Lay::bytes : 0);
    double *D = reinterpret_cast<double *>(Dbase);
    signed char *fid = reinterpret_cast<signed char *>(Dbase + Lay::oFid);
    signed char *pos = reinterpret_cast<signed char *>(Dbase + Lay::oPos);
    double *X0 = D + Lay::oX0, *X1 = D + Lay::oX1, *Ax = D + Lay::oAx, *A2x = D + Lay::oA2x;
    double *xr = D + Lay::oXr, *x0g = D + Lay::oX0v, *UV = D + Lay::oUV;
    double *S = D + Lay::oS;
    const double *Rm = a.rmat;  // R (NU x NU) and the Q / P diagonals: global, L1/L2-resident
    const double *Qd = a.qd, *Pd = a.pd;

    // ---- per-instance inputs: all global loads back to back, then parked in LDS
    double lin[8];
    uint64_t contact = 0;
    constexpr int NRM = NU * NU;
    if constexpr (GEN) {
        // x0 = the state; xref as mpcQP::mpcQP builds it (include/mpcQP.h:74-97)
        const int s_ = b / a.cands;
        const double stv = (hl < NX) ? a.state[(size_t)s_ * NX + hl] : 0.0;
        const double wz = a.cmd[(size_t)s_ * 2], vx = a.cmd[(size_t)s_ * 2 + 1];
#pragma unroll
        for (int i = 0; i < 6; ++i) lin[1 + i] = a.feet[(size_t)s_ * 6 + i];
        lin[7] = 0.0;
        const double ph0 = a.phase[b];
        if (hl < NX) x0g[hl] = stv;
        lin[0] = hbcast<2>(stv);
        if (hl < NX) {
#pragma unroll
            for (int i = 0; i <= N; ++i) {
                const double t = (double)i * a.Ts;
                double v = stv;
                if (hl == 2) v = stv + t * wz;
                if (hl == 3) v = stv + t * vx;
                if (hl == 9 && i > 0) v = vx;
                if (hl == 12) v = -9.8;
                xr[i * NX + hl] = v;
            }
        }
        contact = gait_mask_half(N, a.Ts, ph0, a.swing, a.stance);
    } else {
        // (diagnostic MPCQP_INPUT_ALIAS=n: inputs of instance b mod n, L2-resident -- the
        //  kernel time without the input loads' HBM latency; results are not the batch's)
#ifdef MPCQP_INPUT_ALIAS
        const int b = b_ % MPCQP_INPUT_ALIAS;
#endif
#pragma unroll
        for (int i = 0; i < 8; ++i) lin[i] = stream_load(a.lin + (size_t)b * 8 + i);
        constexpr int NXR = NX * (N + 1), RX = (NXR + kHalf - 1) / kHalf;
        const double *xrg = a.xref + (size_t)b * NXR;
        double v[RX];
#pragma unroll
        for (int r = 0; r < RX; ++r) v[r] = (hl + r * kHalf < NXR) ? stream_load(xrg + hl + r * kHalf) : 0.0;
        const double x0l = (hl < NX) ? stream_load(a.x0 + (size_t)b * NX + hl) : 0.0;
        if (MODEL == 0) contact = stream_load(a.contact + b);
#pragma unroll
        for (int r = 0; r < RX; ++r)
            if (hl + r * kHalf < NXR) xr[hl + r * kHalf] = v[r];
        if (hl < NX) x0g[hl] = x0l;
    }
    wave_sync();
    MPCQP_CUT(a.cut, 11);

    // ---- free map and constraint states (gi_setup for generated bounds, no rows)
    int status = ST_OK, nf = 0;
    {
        bool infeas = false;
#pragma unroll
        for (int base = 0; base < NV; base += kHalf) {
            const int v = base + hl;
            const bool vv = v < NV;
            double lo = -kInfty, hi = kInfty;
            if (vv) pair_bound<NU, MODEL>(a, contact, v, lo, hi);
            const bool freev = vv && lo != hi;
            infeas |= half_ballot(vv && lo > hi) != 0u;
            const uint32_t m = half_ballot(freev);
            const int before = __popc(m & ((1u << hl) - 1u));
            if (vv) pos[v] = freev ? nf + before : -1;
            if (freev && nf + before < NF) fid[nf + before] = v;
            nf += __popc(m);
        }
        if (infeas) status = ST_INFEASIBLE;
        if (nf > NF) status = ST_BAD_DIMS;
    }
    if (nf > a.max_free) status = ST_BAD_DIMS;
    uint64_t *ctl = reinterpret_cast<uint64_t *>(Dbase + Lay::oCt);
    if (hl == 0) {  // reloaded for the outputs: nothing per instance stays live
        ctl[0] = contact;
        ctl[1] = (uint64_t)(valid ? bq : -1);
    }
    wave_sync();
    // a wavefront whose two instances both go elsewhere (deferred to the workgroup kernel,
    // infeasible, no free variable, past the batch) skips the model and condensed terms
    const bool work = __ballot(valid && status == ST_OK && nf > 0) != 0ull;
    MPCQP_STAMP(a.stamps, 0, tst);
    MPCQP_CUT(a.cut, 1);
    if (work) {
        if constexpr (MODEL == 0) {
            // ---- SRBM model, rows written out: Ac's nonzeros are Theta' = Rz' omega (rows 0-2),
            //      p' = v (3-5), v_z' = g (11); Bc's are omega' = Iw^-1 [r_f]x f (6-8) and
            //      v' = f / m (9-11).  Each product keeps the one-QP kernel's operation order
            //      (its zero terms are exact), without evaluating the 13 x 19 entries per lane.
            double Iwi[9];
            double cy = 1.0, sy = 0.0;
            srbm_rot_inertia(lin[0], a.Ibinv, cy, sy, Iwi);
            const double Ts = a.Ts, im = 1.0 / a.mass;
            if (hl >= Sup::x0lo && hl < Sup::x0hi) {  // X0 = Bc Ts, rows 6-11
                const int ii = hl - 6;
                const double e0 = ii == 0 ? 1.0 : 0.0, e1 = ii == 1 ? 1.0 : 0.0,
                             e2 = ii == 2 ? 1.0 : 0.0;
                const double w0 = e0 * Iwi[0] + e1 * Iwi[1] + e2 * Iwi[2];
                const double w1 = e0 * Iwi[3] + e1 * Iwi[4] + e2 * Iwi[5];
                const double w2 = e0 * Iwi[6] + e1 * Iwi[7] + e2 * Iwi[8];
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const int ft = c / 3, comp = c % 3;
                    const double r0 = lin[1 + 3 * ft], r1 = lin[2 + 3 * ft], r2 = lin[3 + 3 * ft];
                    double xa, xb, xc;  // column comp of [r]x
                    if (comp == 0) { xa = 0.0; xb = r2; xc = -r1; }
                    else if (comp == 1) { xa = -r2; xb = 0.0; xc = r0; }
                    else { xa = r1; xb = -r0; xc = 0.0; }
                    const double om = w0 * xa + w1 * xb + w2 * xc;
                    const double vv = (ii - 3 == comp) ? im : 0.0;
                    X0[c * SD + ii] = (ii < 3 ? om : vv) * Ts;
                }
            }
            // row hl of Ac times a vector y (y6, y7, y8 broadcast, yh = y[hl + 6], y12)
            auto arow_dot = [&](double y6, double y7, double y8, double yh, double y12) {
                const double s0 = fma(sy, y7, cy * y6), s1 = fma(cy, y7, -sy * y6);
                double v = 0.0;
                v = hl == 0 ? s0 : v;
                v = hl == 1 ? s1 : v;
                v = hl == 2 ? y8 : v;
                v = (hl >= 3 && hl < 6) ? yh : v;
                v = hl == 11 ? y12 : v;
                return v;
            };
            const int h6 = hl + 6 < NX ? hl + 6 : NX - 1;
            if (hl < NX)
                Ax[hl] = arow_dot(x0g[6], x0g[7], x0g[8], x0g[h6], x0g[12]) * Ts;
            wave_sync();
            if (hl >= Sup::x1lo && hl < Sup::x1hi) {  // X1 = (Ac Ts) X0, rows 0-5
#pragma unroll
                for (int c = 0; c < NU; ++c) {
                    const double *Xc = X0 + c * SD;
                    const double s0 = fma(sy, Xc[1], cy * Xc[0]), s1 = fma(cy, Xc[1], -sy * Xc[0]);
                    double v = Xc[hl < 6 ? hl : 0];
                    v = hl == 0 ? s0 : v;
                    v = hl == 1 ? s1 : v;
                    v = hl == 2 ? Xc[2] : v;
                    X1[c * SD + hl - Sup::x1lo] = v * Ts;
                }
            }
            if (hl < NX)
                A2x[hl] = arow_dot(Ax[6], Ax[7], Ax[8], Ax[h6], Ax[12]) * Ts;
        } else {
            // ---- model: lane i < NX holds row i of Ac; X0 = Bc Ts and X1 = (Ac Ts) X0 on their
            //      support rows, A x0, A^2 x0 (A = Ac Ts).  Same products, in the same order, as the
            //      one-QP kernel (the zero terms it adds are exact).
            double Iwi[9];
            double cy = 1.0, sy = 0.0;
            if (MODEL == 0) srbm_rot_inertia(lin[0], a.Ibinv, cy, sy, Iwi);
            auto entry = [&](int i, int j) -> double {  // [Ac | Bc](i, j)
                return MODEL == 0 ? srbm_entry(i, j, lin, cy, sy, Iwi, a.mass)
                                  : literal_entry(i, j, lin, a.mass);
            };
            const double Ts = a.Ts;
            double arow[NX];
    #pragma unroll
            for (int k = 0; k < NX; ++k) arow[k] = entry(hl, k);
            if (hl >= Sup::x0lo && hl < Sup::x0hi) {
    #pragma unroll
                for (int c = 0; c < NU; ++c) X0[c * SD + hl - Sup::x0lo] = entry(hl, NX + c) * Ts;
            }
            if (hl < NX) {
                double s = 0.0;
    #pragma unroll
                for (int k = 0; k < NX; ++k) s += arow[k] * x0g[k];
                Ax[hl] = s * Ts;
            }
            wave_sync();
            if (hl >= Sup::x1lo && hl < Sup::x1hi) {
    #pragma unroll
                for (int c = 0; c < NU; ++c) {
                    double s = 0.0;
    #pragma unroll
                    for (int k = Sup::x0lo; k < Sup::x0hi; ++k) s += arow[k] * X0[c * SD + k - Sup::x0lo];
                    X1[c * SD + hl - Sup::x1lo] = s * Ts;
                }
            }
            if (hl < NX) {
                double s = 0.0;
    #pragma unroll
                for (int k = 0; k < NX; ++k) s += arow[k] * Ax[k];
                A2x[hl] = s * Ts;
            }
        }
        MPCQP_CUT(a.cut, 13);

        // ---- S^W_rr = X_r' W X_r over the support rows (w: 0 = Q, 1 = P), entry o = cj NU + ci
        //      (MPCQP_PAIR_SLOOP: the lane's entries outermost, so their index arithmetic and the
        //      X rows' loads serve all four blocks; the same operations per entry; 0: the blocks
        //      outermost, A/B)
        if constexpr (MPCQP_PAIR_SLOOP) {
            for (int e = hl; e < NRM; e += kHalf) {
                const int ci = e % NU, cj = e / NU;
                double acc[4];
#pragma unroll
                for (int blk = 0; blk < 4; ++blk) {
                    const int r_ = blk & 1, w_ = blk >> 1;
                    const int lo = r_ ? Sup::x1lo : Sup::x0lo;
                    const double *Xr = r_ ? X1 : X0;
                    const double *w = w_ ? Pd : Qd;  // diag P / Q (uniform addresses: scalar loads)
                    double a_ = 0.0;
#pragma unroll
                    for (int l = 0; l < SD; ++l) a_ += Xr[ci * SD + l] * w[lo + l] * Xr[cj * SD + l];
                    acc[blk] = a_;
                }
#pragma unroll
                for (int blk = 0; blk < 4; ++blk) S[e * 4 + blk] = acc[blk];
            }
        } else {
#pragma unroll
            for (int blk = 0; blk < 4; ++blk) {
                const int r_ = blk & 1, w_ = blk >> 1;
                const int lo = r_ ? Sup::x1lo : Sup::x0lo;
                const double *Xr = r_ ? X1 : X0;
                const double *w = w_ ? Pd : Qd;
                for (int e = hl; e < NRM; e += kHalf) {
                    const int ci = e % NU, cj = e / NU;
                    double acc = 0.0;
#pragma unroll
                    for (int l = 0; l < SD; ++l) acc += Xr[ci * SD + l] * w[lo + l] * Xr[cj * SD + l];
                    S[e * 4 + blk] = acc;
                }
            }
        }
        // ---- W_m e_m once per (m, support row) -- shared by the NU components -- over the dead
        //      xref slot (e_m = x0 + m A x0 + m^2 A^2 x0 / 2 - xref_m), then
        //      u_m(c) = X0[:,c]' W_m e_m, v_m(c) = X1[:,c]' W_m e_m, m = 1..N
        wave_sync();  // (S read X0 / X1 only; xref is still whole)
        constexpr int NSUP = 2 * SD;  // support rows of X1 then X0
        for (int e = hl; e < N * NSUP; e += kHalf) {
            const int m = 1 + e / NSUP, t = e % NSUP;
            const int l = t < SD ? Sup::x1lo + t : Sup::x0lo + t - SD;
            const double md = (double)m, hm2 = 0.5 * md * md;
            const double wl = (m < N ? Qd : Pd)[l];
            xr[m * NX + l] = wl * (x0g[l] + md * Ax[l] + hm2 * A2x[l] - xr[m * NX + l]);
        }
        wave_sync();
        for (int e = hl; e < N * NU; e += kHalf) {
            const int c = e % NU, m = 1 + e / NU;
            const double *el = xr + m * NX;
            double su = 0.0, sv = 0.0;
#pragma unroll
            for (int l = Sup::x0lo; l < Sup::x0hi; ++l) su += X0[c * SD + l - Sup::x0lo] * el[l];
#pragma unroll
            for (int l = Sup::x1lo; l < Sup::x1hi; ++l) sv += X1[c * SD + l - Sup::x1lo] * el[l];
            UV[(m * 2 + 0) * NU + c] = su;
            UV[(m * 2 + 1) * NU + c] = sv;
        }
        wave_sync();
    }
    MPCQP_STAMP(a.stamps, 1, tst);
    MPCQP_CUT(a.cut, 2);

    // a wavefront with nothing to solve (both halves deferred, infeasible, nothing free, past
    // the batch: B standing's every wavefront) goes straight to the outputs
    double fval = 0.0, x = 0.0;
    int iters = 0;
    // warm start (GEN rollouts, MpcArgs::warm): the lane's bounds active at the end, bit 0 lower,
    // bit 1 upper, written back for the next tick
    [[maybe_unused]] int act2 = 0;
    int sfl = 0;  // this half's solver flops (diagnostic counter, MpcArgs::flops_acc)
    if (work) {
        // ---- g (lane p: g_p), then H_FF over the dead early view (lane p loads row p)
        const bool ok = valid && status == ST_OK && nf > 0;
        double gp = 0.0;
        if (ok && hl < nf) {
            const int vi = fid[hl], ki = vi / NU, ci = vi % NU;
            double s = 0.0;
            const double kb = (double)ki - 0.5;  // beta = (m - 1) - kb, exact: one conversion per lane
    #pragma unroll
            for (int m = 1; m <= N; ++m) {  // m > ki; unrolled, branch-free: the loads issue together
                const double beta = (double)(m - 1) - kb;
                const double tm = UV[(m * 2 + 0) * NU + ci] + beta * UV[(m * 2 + 1) * NU + ci];
                if (MPCQP_HB_BASES) s = fma((m > ki) ? 1.0 : 0.0, tm, s);  // (exact: x 1 / x 0)
                else s += (m > ki) ? tm : 0.0;
            }
            gp = 2.0 * s;
        }
        wave_sync();
        double *Hb = D + Lay::oR;
        if (ok) {
            // one lane per block pair (ki >= kj); the beta sums once per block
            constexpr int NPAIR = N * (N + 1) / 2;
            constexpr int NFT = NU / 3;
            static_assert(NU % 3 == 0, "inputs are force triples");
            for (int bp = hl; bp < NPAIR; bp += kHalf) {
                // bp = ki (ki + 1) / 2 + kj, row-major over ki >= kj (closed form, corrected)
                int ki = (int)((__builtin_sqrtf(8.0f * (float)bp + 1.0f) - 1.0f) * 0.5f);
                ki += ((ki + 1) * (ki + 2) / 2 <= bp) ? 1 : 0;
                ki -= (ki * (ki + 1) / 2 > bp) ? 1 : 0;
                const int kj = bp - ki * (ki + 1) / 2;
                double c, si, sj, sij;
                beta_sums(ki + 1, N - 1, ki, kj, c, si, sj, sij);
                const double bi = (double)(N - 1 - ki) + 0.5, bj = (double)(N - 1 - kj) + 0.5;
                const double bij = bi * bj;
                const double rf = (ki == kj) ? 1.0 : 0.0;  // R on the diagonal blocks (exact: fma by 1)
                // the free inputs of a step come in whole force triples (a foot in contact has
                // all three components free: the fast path's bounds guarantee it), so the block
                // is a set of 3x3 foot-pair sub-blocks with consecutive positions.  The triples of
                // each step are compacted (slot a: foot fI[a] at position pI[a], -1 past the step's
                // count), so a sub-block slot no lane of the wave has is skipped as a whole: one
                // stance foot per step (config B) runs one 3x3 sub-block per block pair, not four
                int pI[NFT], pJ[NFT], fI[NFT], fJ[NFT];
    #pragma unroll
                for (int t = 0; t < NFT; ++t) { pI[t] = pJ[t] = -1; fI[t] = fJ[t] = 0; }
                int nI = 0, nJ = 0;
    #pragma unroll
                for (int s_ = 0; s_ < NFT; ++s_) {
                    const int p_i = pos[ki * NU + 3 * s_], p_j = pos[kj * NU + 3 * s_];
    #pragma unroll
                    for (int t = 0; t < NFT; ++t) {
                        const bool ti = p_i >= 0 && nI == t, tj = p_j >= 0 && nJ == t;
                        pI[t] = ti ? p_i : pI[t];
                        fI[t] = ti ? s_ : fI[t];
                        pJ[t] = tj ? p_j : pJ[t];
                        fJ[t] = tj ? s_ : fJ[t];
                    }
                    nI += p_i >= 0 ? 1 : 0;
                    nJ += p_j >= 0 ? 1 : 0;
                }
#if MPCQP_HB_BASES
                // per sub-block: the S / R entry base and the three packed-row bases of H_FF;
                // the 3x3 entries then sit at compile-time offsets from them.  Positions ascend
                // with the slot (a triple per slot), so in a diagonal block (ki == kj) slot
                // pairs ta < tb are strictly upper (skipped), ta > tb strictly lower, and
                // ta == tb keeps a3 >= b3 (the others go to the dump slot, branch-free)
                const bool diag = ki == kj;
    #pragma unroll
                for (int ta = 0; ta < NFT; ++ta) {
    #pragma unroll
                    for (int tb = 0; tb < NFT; ++tb) {
                        if (pI[ta] < 0 || pJ[tb] < 0 || (ta < tb && diag)) continue;
                        const int sb = 3 * fJ[tb] * NU + 3 * fI[ta];
                        const double *Sb = S + sb * 4, *Rb = Rm + sb;
                        const int h0 = lrow(pI[ta]) + pJ[tb];
                        const int hrow[3] = {h0, h0 + pI[ta] + 1, h0 + 2 * pI[ta] + 3};
    #pragma unroll
                        for (int a3 = 0; a3 < 3; ++a3) {
    #pragma unroll
                            for (int b3 = 0; b3 < 3; ++b3) {
                                const double *So = Sb + (b3 * NU + a3) * 4;
                                double v = c * So[0] + sij * So[1];
                                v += So[2] + bij * So[3];
                                v = fma(rf, Rb[b3 * NU + a3], v);
                                const bool dump = ta == tb && a3 < b3 && diag;
                                Hb[dump ? Lay::oDump - Lay::oR : hrow[a3] + b3] = 2.0 * v;
                            }
                        }
                    }
                }
#else
    #pragma unroll
                for (int ta = 0; ta < NFT; ++ta) {
    #pragma unroll
                    for (int tb = 0; tb < NFT; ++tb) {
                        if (pI[ta] < 0 || pJ[tb] < 0) continue;
    #pragma unroll
                        for (int a3 = 0; a3 < 3; ++a3) {
    #pragma unroll
                            for (int b3 = 0; b3 < 3; ++b3) {
                                const int pp = pI[ta] + a3, qq = pJ[tb] + b3;
                                const int ci = 3 * fI[ta] + a3, cj = 3 * fJ[tb] + b3;
                                // branch-free: the strictly upper entries of a diagonal block go
                                // to the dump slot
                                const double *So = S + (cj * NU + ci) * 4;
                                double v = c * So[0] + sij * So[1];
                                v += So[2] + bij * So[3];
                                v = fma(rf, Rm[cj * NU + ci], v);
                                Hb[pp >= qq ? lrow(pp) + qq : Lay::oDump - Lay::oR] = 2.0 * v;
                            }
                        }
                    }
                }
#endif
            }
        }
        // rows without a free variable (past nf, or a half with nothing to solve) are identity
        // rows of the padded H_FF: written into the packed buffer (rare: only such waves pay), so
        // every lane then loads its row unmasked (entries right of the diagonal are never read)
        const bool pad = !ok || hl >= nf;
        if (__ballot(pad && hl < NF) != 0ull) {
            if (pad && hl < NF)
                for (int q = 0; q <= hl; ++q) Hb[lrow(hl) + q] = (q == hl) ? 1.0 : 0.0;
        }
        wave_sync();
#if !MPCQP_PAIR_FOLD
        double h[NF];
    #pragma unroll
        for (int q = 0; q < NF; ++q) h[q] = Hb[lrow(hl) + q];
        wave_sync();
#endif
        MPCQP_STAMP(a.stamps, 3, tst);
        MPCQP_CUT(a.cut, 3);

        // ---- solver (gi_run_reg with NF = 30 per half)
        constexpr bool kRinv = MPCQP_PAIR_RINV;
        double *Lc = D + Lay::oR, *R = D + Lay::oR, *Ri = D + Lay::oR;  // R (or R^-1) over dead L
        (void)Lc;
        double *rowbuf = D + Lay::oRow, *colb = rowbuf + NP, *rot = rowbuf + 2 * NP,
               *rinv = rowbuf + 4 * NP;
        double u = 0.0;
        int q = 0, act = -1;
        double Jr[NF];
        double gv = gp;
        const bool any_ok = __ballot(ok) != 0ull;
        bool ok2 = ok;
        if (any_ok) {
#if MPCQP_PAIR_FOLD
            // ---- Cholesky and the inverse sweep FOLDED into one register row per lane.  Lane l owns
            //      row l of the symmetric H_FF, whole (slots q > l read from the packed lower
            //      triangle's column l).  Right-looking, lane l is an ordinary Cholesky row for its
            //      slots q <= l: at step k its slot k becomes L(l, k), the multiplier of its trailing
            //      update s_j -= L(l, k) L(j, k).  Its slots q > l hold the J part: every step k < l
            //      applies the same update to them (the instruction is uniform), so after step l - 1
            //      they hold exactly the Schur-complement entries H'(j, l) -- the values lane j holds
            //      in its slot l, computed by the same FMAs in the same order -- i.e. L(j, l) L(l, l).
            //      Lane l sits out the trailing update of step l itself, and its own slot l is
            //      negated after the scaling (-L(l, l)): from then on [-L(l,l), H'(l+1.., l)] is
            //      -piv_l times [ik_l, -L(l+1.., l) ik_l], the forward substitution L y = e_l after its
            //      step l, and the later steps k > l (in which lane l takes part with its slot k as
            //      the multiplier y_k) finish it.  At the end slots q >= l are scaled by -1 / piv_l
            //      (row l of J = L^-T) and slots q < l (its row of L, dead) zeroed.  Lane 31 of each
            //      half carries g as row 31 of the padded matrix (below every row: a plain Cholesky
            //      row throughout) and ends with t = L^-1 g.  One FMA per (step, slot) instead of the
            //      fused sweep's two (one for H, one for J); the two triangles of the square the lanes
            //      swept are one triangle each, and the J array costs no registers of its own.
            // (lane 31 reads g from the row buffer: its row of the padded matrix)
            if (hl < NF) rowbuf[hl] = gv;
            wave_sync();
            {
                const double *Hr = hl == kHalf - 1 ? rowbuf : D + Lay::oR + lrow(hl),
                             *Hc = D + Lay::oR + hl;
    #pragma unroll
                for (int q = 0; q < NF; ++q) {
                    if (MPCQP_FOLD_ASEL && MPCQP_FOLD_LMASK) {  // lanes q .. 31 read their row
                        const unsigned long long mq = hrange_k(q, kHalf - 1);
                        int ad;
                        asm("v_cndmask_b32_e64 %0, %1, %2, %3"
                            : "=v"(ad)
                            : "v"((int)(size_t)(Hc + lrow(q))), "v"((int)(size_t)(Hr + q)), "s"(mq));
                        // (the low 32 bits of an LDS-derived generic pointer are its LDS address)
                        typedef __attribute__((address_space(3))) const double lds_cd;
                        Jr[q] = *(lds_cd *)(size_t)(unsigned)ad;
                    } else if (MPCQP_FOLD_ASEL) {  // one load from the selected address
                        Jr[q] = *((q <= hl) ? Hr + q : Hc + lrow(q));  // (q, l) read for q > l
                    } else {
                        const double lo_ = Hr[q], up_ = Hc[lrow(q)];  // (q, l) read for q > l
                        Jr[q] = (q <= hl) ? lo_ : up_;
                    }
                }
            }
            wave_sync();
            static_assert(MPCQP_CHOL_CB == 2, "the folded sweep runs column pairs");
            double *dg = rot;  // pivot of every column (uniform stores), for the final scaling
            double piv = hbcast<0>(Jr[0]);
            // non-PD flag: a lane mask in SGPRs (v_cmp + s_or per pivot), pinned every step
            unsigned long long badm = __ballot(!(piv > 0.0));
            double ik = rsqrt_nr(piv);
    #pragma unroll
            for (int k = 0; k < NF; k += 2) {
                const double pk = piv;
                // column k: lanes > k get L(l, k), lanes < k their J entry y_k; lane k L(k, k),
                // negated (its J part's first entry), and multiplier 0 (it sits out step k)
                // (lane k of each half by an SGPR constant: no per-lane compare)
                Jr[k] *= ik;
                const unsigned long long own0 = hmask_k(k);
                const double m0 = zero_if(Jr[k], own0);
                Jr[k] = neg_if(Jr[k], own0);
                double A0, B0;
                row_pair(m0, A0, B0);  // the column's rows 0-15 / 16-31 in every row of the half
                fold_in_panel<NF>(Jr, A0, B0, m0, k);  // slot k + 1 -= L(k + 1, k) m0
                const double pc = hbcast(Jr[k + 1], k + 1);
                badm |= __ballot(!(pc > 0.0));
                const double ik1 = rsqrt_nr(pc);
                Jr[k + 1] *= ik1;
                const unsigned long long own1 = hmask_k(k + 1);
                const double m1 = zero_if(Jr[k + 1], own1);
                Jr[k + 1] = neg_if(Jr[k + 1], own1);
                double A1, B1;
                row_pair(m1, A1, B1);
                double pivn = 1.0, ikn = 1.0;
                if (k + 2 < NF) {  // next pivot ahead of the trailing update (on lane k + 2)
                    double hn = Jr[k + 2 < NF ? k + 2 : k];
                    hn -= Jr[k] * Jr[k];
                    pivn = hbcast(hn - Jr[k + 1] * Jr[k + 1], k + 2);
                    badm |= __ballot(!(pivn > 0.0));
                    ikn = rsqrt_nr(pivn);
                }
                dg[k] = pk;
                dg[k + 1] = pc;
                // trailing update: slot j -= L(j, k) m0 + L(j, k + 1) m1, the L(j, .) broadcast by
                // the FMA's own DPP (no LDS round trip)
                fold_trailing_k<NF>(Jr, k, A0, B0, m0, A1, B1, m1);
    #pragma unroll
                for (int j = 0; j < NF; ++j)
                    if (j >= k) pin(Jr[j]);
                piv = pivn;
                ik = ikn;
                pin(piv);
                pin(ik);
                // the non-PD test is evaluated here, each step: left to the compiler, every
                // column's pivot stayed live to a test sunk after the sweep (60 VGPRs)
                asm volatile("" : "+s"(badm));
                step_fence();
            }
            {   // rows of J: slots >= l times -1 / piv_l, the L row below zeroed; lane 31 keeps t
                wave_sync();
                const bool gl = hl == kHalf - 1;
                const double pl = dg[hl < NF ? hl : 0];
                const double cl = gl ? 1.0 : -1.0 / pl;
                // slot j is zeroed on lanes j + 1 .. NF - 1 (their L rows) and on the padding
                // lanes NF .. 30 (lane 31 keeps t): a constant lane mask per slot
    #pragma unroll
                for (int j = 0; j < NF; ++j) {
                    Jr[j] = zero_if(Jr[j] * cl, hrange_k(j + 1, kHalf - 2));
                    pin(Jr[j]);  // (in place: the scaled row does not take a second register set)
                    if ((j & 7) == 7) step_fence();
                }
            }
            // (every pivot is uniform over its half: the half's base lane carries its votes)
            const bool bad = ((badm >> (lane() & kHalf)) & 1ull) != 0ull;
#else
            // ---- Cholesky fused with the inverse sweep.  Right-looking, lane l owns row l of H_FF
            //      (identity padding beyond nf).  Step k's column of L, broadcast from LDS for the
            //      trailing update, is also the operand of step k of the forward substitution
            //      that turns lane c's e_c into column c of L^-1 (= row c of J, in registers): one
            //      LDS read feeds two independent FMA streams.  Lane 31 of each half starts from g
            //      instead and ends with t = L^-1 g.  Same operations in the same order as a
            //      separate Cholesky then inverse sweep.
            if (hl < NF) colb[hl] = gv;
            wave_sync();
            // (branch-free: every lane reads colb -- a uniform address, two values per b128 -- and
            //  selects, instead of a predicated read per element)
            const bool gl = hl == kHalf - 1;
    #pragma unroll
            for (int l = 0; l < NF; ++l) {
                double cbl = colb[l];
                pin(cbl);  // (keeps the load unconditional: LLVM would sink it into a branch)
                Jr[l] = gl ? cbl : ((hl == l) ? 1.0 : 0.0);
            }
            double piv = hbcast<0>(h[0]);
            bool bad = !(piv > 0.0);
            double ik = rsqrt_nr(piv);
            // CB columns per LDS round trip: columns k+1 .. k+CB-1 are finished in registers from
            // the panel's DPP-broadcast entries L(k+c, k+c'), then the CB columns are written and
            // the trailing update reads them together.  Per element the operations and their
            // order are those of CB single-column steps (bitwise the same factor and J).
            constexpr int CB = MPCQP_CHOL_CB;
            static_assert(NF % CB == 0, "whole column panels");
    #pragma unroll
            for (int k = 0; k < NF; k += CB) {
                double lk[CB], ikc[CB];
                double bc[CB][CB];  // bc[c][c2] = L(k + c, k + c2), broadcast once: the panel update
                                    // and the inverse sweep's column both use it
                ikc[0] = ik;
                lk[0] = h[k] * ik;
                h[k] = lk[0];
    #pragma unroll
                for (int c = 1; c < CB; ++c) {
    #pragma unroll
                    for (int c2 = 0; c2 < c; ++c2) {
                        bc[c][c2] = hbcast(lk[c2], k + c);
                        h[k + c] -= lk[c2] * bc[c][c2];  // panel column c2's update
                    }
                    const double pc = hbcast(h[k + c], k + c);
                    bad |= !(pc > 0.0);
                    ikc[c] = rsqrt_nr(pc);
                    lk[c] = h[k + c] * ikc[c];
                    h[k + c] = lk[c];
                }
                double pivn = 1.0, ikn = 1.0;
                if (k + CB < NF) {
                    double hn = h[k + CB < NF ? k + CB : k];  // on lane k+CB
    #pragma unroll
                    for (int c = 0; c < CB - 1; ++c) hn -= lk[c] * lk[c];
                    pivn = hbcast(hn - lk[CB - 1] * lk[CB - 1], k + CB);
                    bad |= !(pivn > 0.0);
                    ikn = rsqrt_nr(pivn);
                }
                // the panel's CB columns of L go to a column buffer for the trailing update's
                // broadcast reads: every lane stores its entry at a fixed slot (no predicate, no
                // address arithmetic; entries above the diagonal are never read).  L itself is
                // not kept: the fused sweep builds J as it goes, and the region is R^-1 next.
    #pragma unroll
                for (int c = 0; c < CB; ++c) Lc[c * NP + hl] = lk[c];
    #pragma unroll
                for (int c = 0; c < CB; ++c) {
    #pragma unroll
                    for (int c2 = 0; c2 < c; ++c2) Jr[k + c] -= bc[c][c2] * Jr[k + c2];
                    Jr[k + c] *= ikc[c];
                }
                wave_sync();
    #pragma unroll
                for (int j = 0; j < NF; ++j) {
                    if (j >= k + CB) {
                        double cv[CB];
    #pragma unroll
                        for (int c = 0; c < CB; ++c) cv[c] = Lc[c * NP + j];
    #pragma unroll
                        for (int c = 0; c < CB; ++c) h[j] -= lk[c] * cv[c];
    #pragma unroll
                        for (int c = 0; c < CB; ++c) Jr[j] -= cv[c] * Jr[k + c];
                    }
                    if ((j % MPCQP_CHOL_PF) == MPCQP_CHOL_PF - 1 && j >= k + CB) step_fence();
                }
    #pragma unroll
                for (int j = 0; j < NF; ++j)
                    if (j >= k) { pin(h[j]); pin(Jr[j]); }
                piv = pivn;
                ik = ikn;
                pin(piv);
                pin(ik);
                step_fence();
            }
#endif
            if (ok && bad) status = ST_NOT_PD;
            ok2 = ok && status == ST_OK;
            MPCQP_STAMP(a.stamps, 5, tst);
            MPCQP_CUT(a.cut, 4);
            MPCQP_CUT(a.cut, 5);
            // ---- unconstrained minimum x = -J t, objective -|t|^2 / 2
            wave_sync();
            if (hl == kHalf - 1) {
    #pragma unroll
                for (int j = 0; j < NF; ++j) colb[j] = Jr[j];
            }
            wave_sync();
            gv = (hl < NF) ? colb[hl] : 0.0;
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll
            for (int j = 0; j < NF; ++j) {
                s4[j & 3] += Jr[j] * colb[j];
                if ((j % PFD) == PFD - 1) pin_fence4(s4);
            }
            x = (ok2 && hl < nf) ? -((s4[0] + s4[1]) + (s4[2] + s4[3])) : 0.0;
            fval = half_sum(hl < nf ? gv * gv : 0.0);
            fval = ok2 ? -0.5 * fval : 0.0;
        }
        MPCQP_STAMP(a.stamps, 7, tst);
        MPCQP_CUT(a.cut, 6);

        // ---- dual active-set loop (Goldfarb-Idnani), flattened: one add or drop per pass, the
        //      wave running while either half has work.  Lane l owns variable l's two bound
        //      constraints (ids l and l + nf): their b and eligibility live in registers, so the
        //      most-violated search is register arithmetic plus one half-wave argmin.
        //      Add step: J2 <- J2 (I - beta v v'), the Householder reflection that maps d2 to
        //      |d2| e_q (v_q by Parlett's cancellation-free form).  It leaves the same first
        //      column J2 d2 / |d2| and R column as the Givens chain of gi_reg.hpp / the oracle;
        //      the trailing columns of J2 are another orthonormal basis of the same subspace, which
        //      every later GI quantity (z = J2 J2' n, d1 = J1' n, r) is invariant to.  62 FMAs on
        //      the resident rows instead of 30 rotations and their suffix-scan set-up.
        //      Drop step: Givens restores R to triangular, the rotations go to LDS for J.
        const int mt = 2 * nf;
        const int max_iter = a.max_iter > 0 ? a.max_iter : 10 * (mt + nf + 1);
        // bit 0 / 1: lower / upper bound inactive (eligible); bit 2: the variable is a vertical
        // force.  A free variable is a force in contact (or a literal-model input), so its bounds
        // follow from bit 2 alone: b of x >= lo is lo, b of -x >= -hi is -hi
        int stb = 0;
        if (ok2 && hl < nf) {
            double lo, hi;
            // (a free variable is in contact: the all-ones schedule gives its bounds, and the
            //  contact register need not live from the inputs to here)
            pair_bound<NU, MODEL>(a, ~0ull, fid[hl], lo, hi);
            stb = (lo > -kInfty ? 1 : 0) | (hi < kInfty ? 2 : 0) |
                  ((MODEL == 0 && (fid[hl] % NU) % 3 == 2) ? 4 : 0);
        }
        // b and the violation threshold of the lane's two bounds: host-computed constants picked
        // by bit 2 of stb (which never changes) at each use -- the opaque copy of the bit keeps
        // the selects where they are used, so no per-lane copy lives through the loops
        auto vert = [&]() {
            int sb = stb;
            asm volatile("" : "+v"(sb));
            return (sb & 4) != 0;
        };
#define MPCQP_BLO (vert() ? a.blo_v : a.blo_t)
#define MPCQP_BHI (vert() ? a.bhi_v : a.bhi_t)
#define MPCQP_TLO (vert() ? a.tlo_v : a.tlo_t)
#define MPCQP_THI (vert() ? a.thi_v : a.thi_t)
        bool done = !ok2;
#if MPCQP_PAIR_CRASH
        // ---- crash: speculative primal-dual active-set start (oracle box_crash, DESIGN.md
        //      section 4).  Working set A = every bound the unconstrained minimum x0 violates
        //      (at most KC: the bounds already in A, then the lowest variable ids); with A's
        //      bounds as equalities the minimiser is x = x0 - J J_A' w, M w = x0_A - b_A,
        //      M = J_A J_A' = (H^-1)_AA.  Lane a of A publishes its J row (LDS, the dead L space),
        //      computes row rank(a) of M against the published rows, and the k x k system is
        //      solved by Gauss-Jordan, one pivot row broadcast per step.  The next A drops
        //      negative multipliers (lambda_a = -side_a w_a) and adds what x violates; an
        //      unchanged A is the optimum (the strictly convex QP's KKT point, within the dual
        //      loop's own tolerances), and the half skips the dual loop.  After PC working sets
        //      or a non-positive pivot the half gives up with J, x0 and f0 untouched and runs
        //      Goldfarb-Idnani as before.  Iterations = the working sets that needed a solve.
        //      One wavefront loop for both halves; every ballot runs with all lanes active.
        //      Rows of M and the terms of y go in chunks of four (one branch per chunk, the
        //      chunk's LDS reads issued together); past-k entries of a chunk are computed from
        //      clamped addresses and never read.
        {
            constexpr int KC = kPairCrashK, CH = 2;
            static_assert(KC % CH == 0, "whole chunks");
            const int PC = a.crash_p;
            static_assert(KC * NF <= Lay::HB, "the published J rows fit the dead H space");
            static_assert(KC + 2 <= NP, "the pivot row fits the row buffer");
            double *Wr = D + Lay::oR;             // [KC][NF] published J rows
            double *Pv = rowbuf;                  // pivot row [KC], its r, 1 / pivot
            double *Wv = colb;                    // w by rank
            double *Yv = rot;                     // y = J_A' w [NF]
            const double x0v = x, f0 = fval;
            double xc = x0v;
            // the objective at xc (uniform per half) is parked in LDS: a register pair less
            // through the Gram and Gauss-Jordan, the crash's register peak
            double *fcs = D + Lay::oRow + 4 * NP + 1;
            if (hl == 0) *fcs = f0;
            bool lneg = false;  // this bound's multiplier is negative (dropped next)
            int side = 0, cit = 0;
            bool crashing = !done, cok = false;
            // warm start (rollouts): the previous tick's active bound of this
            // variable, one horizon step later (step k now was step k + 1 then; the last step
            // repeats), joins the FIRST working set even when x0 does not violate it; the
            // primal-dual iteration then drops it if its multiplier is negative.  The optimum is
            // the same point (strictly convex QP); only the number of working sets changes.
            int seed = 0;
            if constexpr (GEN) {
                if (a.warm && crashing && hl < nf) {
                    const int bw = (int)(long long)ctl[1];
                    const unsigned long long *w = a.warm + (size_t)bw * a.warm_words;
                    const int v = fid[hl], kv = v / NU, cv = v % NU;
                    const int vs = (kv + 1 < N ? kv + 1 : kv) * NU + cv;
                    if (((w[vs >> 6] >> (vs & 63)) & 1ull) && (stb & 1)) seed = 1;
                    else if (((w[(NV + vs) >> 6] >> ((NV + vs) & 63)) & 1ull) && (stb & 2)) seed = -1;
                }
            }
            while (__ballot(crashing) != 0ull) {
                int nw = side;
                if (crashing && hl < nf) {
                    // (the thresholds are re-derived here: kept live across the loop they were
                    //  the kernel's spilled registers, reloaded from scratch every trip)
                    if (side == 0) {
                        if ((stb & 1) && xc - MPCQP_BLO < MPCQP_TLO) nw = 1;
                        else if ((stb & 2) && -xc - MPCQP_BHI < MPCQP_THI) nw = -1;
                        else if (GEN && cit == 0) nw = seed;
                    } else if (lneg) {
                        nw = 0;
                    }
                }
                const bool changed = half_ballot(nw != side) != 0u;
                if (crashing && !changed) { cok = true; crashing = false; }  // (cit = 0: x0 is optimal)
                if (crashing && cit >= PC) crashing = false;  // give up
                {   // at most KC bounds: those already in A, then the lowest variable ids
                    const uint32_t am = half_ballot(crashing && nw != 0);
                    const uint32_t km = half_ballot(crashing && nw != 0 && side != 0);
                    const uint32_t nm = half_ballot(crashing && nw != 0 && side == 0);
                    const int room = KC - __popc(km);
                    if (__popc(am) > KC && nw != 0 && side == 0 &&
                        __popc(nm & ((1u << hl) - 1u)) >= room)
                        nw = 0;
                }
                if (crashing) { side = nw; ++cit; }
                const uint32_t amask = half_ballot(crashing && side != 0);
                const int k = __popc(amask);
                const int rho = __popc(amask & ((1u << hl) - 1u));
                const bool solving = crashing && k > 0;
                const bool inA = solving && side != 0;
                if (crashing && k == 0) { xc = x0v; lneg = false; if (hl == 0) *fcs = f0; }
                if (solving) ++iters;
                if (a.flops_acc && solving) sfl += crash_ws_flops_i(nf, k);
                const int ks = solving ? k : 0;
                const int kmax = max(__builtin_amdgcn_readlane(ks, 0), __builtin_amdgcn_readlane(ks, kHalf));
                if (kmax == 0) continue;  // (wave-uniform)
                double rr = x0v - (side > 0 ? MPCQP_BLO : -MPCQP_BHI);
                if (inA) {
        #pragma unroll
                    for (int c = 0; c < NF; ++c) Wr[rho * NF + c] = Jr[c];
                }
                wave_sync();
                // row rank(a) of M = J_A J_A' (lane a's own J row against the published rows)
                double Mr[KC];
        #pragma unroll
                for (int m0 = 0; m0 < KC; m0 += CH) {
        #pragma unroll
                    for (int m = m0; m < m0 + CH; ++m) Mr[m] = 0.0;
                    if (m0 < kmax) {
        #pragma unroll
                        for (int c = 0; c < NF; ++c) {
        #pragma unroll
                            for (int m = 0; m < CH; ++m) Mr[m0 + m] += Jr[c] * Wr[(m0 + m) * NF + c];
                            if ((c % PFG) == PFG - 1) {
        #pragma unroll
                                for (int m = 0; m < CH; ++m) pin(Mr[m0 + m]);
                                step_fence();
                            }
                        }
                    }
                }
                // Gauss-Jordan without pivoting (M is positive definite): step j's pivot row is
                // published by the lane of rank j, every other lane of A eliminates column j.
                // (The next pivot's stores follow this step's loads of the same words, and LDS
                //  keeps a wave's program order: one wave_sync per step.)
                double dd = 1.0;
                bool bad = false;
        #pragma unroll
                for (int j = 0; j < KC; ++j) {
                    if (j < kmax) {
                        // (columns past kmax are never read: the row's tail goes in chunks of
                        //  four behind wave-uniform guards)
                        if (inA && rho == j) {
        #pragma unroll
                            for (int m0 = j & ~3; m0 < KC; m0 += 4) {
                                if (m0 < kmax) {
        #pragma unroll
                                    for (int m = m0; m < m0 + 4; ++m)
                                        if (m >= j) Pv[m] = Mr[m];
                                }
                            }
                            Pv[KC] = rr;
                            if constexpr (MPCQP_PAIR_CRASH_RCP) {
                                const double pj = Mr[j];
                                double y = __builtin_amdgcn_rcp(pj);
                                y = fma(y, fma(-pj, y, 1.0), y);
                                y = fma(y, fma(-pj, y, 1.0), y);
                                Pv[KC + 1] = y;
                                dd = y;  // (its reciprocal: w = r / pivot below)
                            } else {
                                Pv[KC + 1] = 1.0 / Mr[j];
                                dd = Mr[j];
                            }
                            bad |= !(Mr[j] > 0.0);
                        }
                        wave_sync();
                        const double pr = Pv[KC], pi = Pv[KC + 1];
                        const bool upd = inA && rho != j && j < k;
                        // MPCQP_CRASH_LSEL: the lanes that do not eliminate get multiplier 0 (one
                        // select) and run the FMAs unmasked: x - 0 * p = x for the finite pivot row
                        const double l = MPCQP_CRASH_LSEL ? (upd ? Mr[j] * pi : 0.0) : Mr[j] * pi;
                        // the pivot row in chunks of four (loads outside the divergent update,
                        // at most one chunk of it in registers)
        #pragma unroll
                        for (int m0 = (j + 1) & ~3; m0 < KC; m0 += 4) {
                            if (m0 < kmax) {
                                double pv[4];
        #pragma unroll
                                for (int m = m0; m < m0 + 4; ++m) pv[m - m0] = m > j ? Pv[m] : 0.0;
                                if (MPCQP_CRASH_LSEL || upd) {
        #pragma unroll
                                    for (int m = m0; m < m0 + 4; ++m)
                                        if (m > j) Mr[m] -= l * pv[m - m0];
                                }
                            }
                        }
                        if (MPCQP_CRASH_LSEL || upd) rr -= l * pr;
                    }
                }
                const bool gave_up = half_ballot(bad) != 0u;
                const double w = inA ? (MPCQP_PAIR_CRASH_RCP ? rr * dd : rr / dd) : 0.0;
                if (inA) Wv[rho] = w;
                // (b and the right-hand side re-derived after the elimination: not live through it)
                const double bval = side > 0 ? MPCQP_BLO : -MPCQP_BHI;
                const double wr = half_sum(inA ? w * (x0v - bval) : 0.0);
                wave_sync();
                // y = J_A' w (lane c: column c of the published rows), then x = x0 - J y
                double yv[CH] = {};
                const int cc = hl < NF ? hl : 0;
        #pragma unroll
                for (int m0 = 0; m0 < KC; m0 += CH) {
                    if (m0 < kmax) {
        #pragma unroll
                        for (int m = 0; m < CH; ++m) {
                            const double t = Wr[(m0 + m) * NF + cc] * Wv[m0 + m];
                            yv[m] += (m0 + m < k) ? t : 0.0;
                        }
                    }
                }
                double ys = 0.0;
        #pragma unroll
                for (int m = 0; m < CH; ++m) ys += yv[m];
                if (hl < NF) Yv[hl] = ys;
                wave_sync();
                double s4[4] = {0.0, 0.0, 0.0, 0.0};
        #pragma unroll
                for (int c = 0; c < NF; ++c) {
                    s4[c & 3] += Jr[c] * Yv[c];
                    if ((c % PFD) == PFD - 1) pin_fence4(s4);
                }
                wave_sync();
                if (solving && !gave_up) {
                    xc = hl < nf ? x0v - ((s4[0] + s4[1]) + (s4[2] + s4[3])) : 0.0;
                    if (inA) xc = bval;
                    lneg = inA && -(double)side * w < 0.0;
                    if (hl == 0) *fcs = f0 + 0.5 * wr;
                }
                if (solving && gave_up) crashing = false;
            }
            wave_sync();
            if (cok) {  // this half is solved: the dual loop skips it
                x = xc;
                fval = *fcs;
                done = true;
                if constexpr (GEN) act2 = side > 0 ? 1 : (side < 0 ? 2 : 0);
            }
        }
#endif
        MPCQP_CUT(a.cut, 8);
        bool fresh = true;
        int p = 0;
        // the partial multiplier of the constraint being added (slot q), in every lane of the half
        double uadd = 0.0;
        // a zero double (the masked reads of the R^-1 product point here)
        constexpr int oZ = Lay::oRow + 4 * NP;
        if (kRinv && hl == 0) D[oZ] = 0.0;
        MPCQP_SUB_INIT(tsub);
    #ifdef MPCQP_STAMPS
        unsigned long long npass = 0;  // passes of this wavefront (diagnostic slot 2)
    #endif
        while (__ballot(!done) != 0ull) {
    #ifdef MPCQP_STAMPS
            ++npass;
    #endif
            double dj = 0.0, sp = 0.0, z = 0.0, zn = 0.0, zq = 0.0, r = 0.0, t1 = INFINITY,
                   t2 = INFINITY, t = 0.0, sg = 1.0, beta = 0.0, dqv = 0.0;
            int kslot = 0x7fffffff, a_ = 0;
            bool lower = true;
            // a pass either steps on the selected constraint p or (first pass) only selects
            const bool go = !done && !fresh;
            if (go) {
                // ---- d = J' n_p = sg J(a, :)': lane a publishes its J row and the slack of p;
                //      every lane reads its d_j, then lanes j < q zero their slot, leaving d2 (the
                //      inactive part, for z and the reflection) in the buffer
                lower = p < nf;
                a_ = lower ? p : p - nf;
                sg = lower ? 1.0 : -1.0;
                if (hl == a_) {
    #pragma unroll
                    for (int c = 0; c < NF; ++c) {
                        rowbuf[c] = Jr[c];
                    }
                    rowbuf[NP - 1] = lower ? x - MPCQP_BLO : -x - MPCQP_BHI;
                }
                wave_sync();
                dj = (hl < nf) ? sg * rowbuf[hl] : 0.0;
                sp = rowbuf[NP - 1];
                if constexpr (kRinv) {
                    // r = R^-1 d(0:q): lane i < q takes row i of R^-1 (column-major packed, (i, j)
                    // at lrow(j) + i: consecutive lanes, consecutive addresses) against the
                    // published d (uniform address per half); independent products, no chain
                    // (masked terms read the zero slot: an address select instead of value selects)
                    const int qmax = max(__builtin_amdgcn_readlane(q, 0), __builtin_amdgcn_readlane(q, kHalf));
                    double r2[2] = {0.0, 0.0};
                    for (int j = 0; j < qmax; ++j) {
                        const double rij = D[hl <= j ? Lay::oR + lrow(j) + hl : oZ];
                        const double dv = D[j < q ? Lay::oRow + j : oZ];
                        r2[j & 1] = fma(rij, dv, r2[j & 1]);
                    }
                    r = (hl < q) ? sg * (r2[0] + r2[1]) : 0.0;
                }
                if (hl < q) rowbuf[hl] = 0.0;  // after every lane's read (LDS keeps program order)
                wave_sync();
                if (iters >= max_iter) { status = ST_ITER_LIMIT; done = true; }
            }
            MPCQP_SUB(tsub, 0);
            MPCQP_CUT(a.cut, 20);
            const bool stepping = go && !done;
            if (stepping) {
                ++iters;
                if (a.flops_acc) sfl += pass_flops_i(nf, q);
                // |d(0:q)|^2 and |d(q+1:nf)|^2 in one two-sum pass; zn = |d2|^2 = zq + d_q^2 and
                // dd = |d|^2 = zn + the first part
                double sq = hl < q ? dj * dj : 0.0;
                zq = (hl > q && hl < nf) ? dj * dj : 0.0;
                half_sum2(sq, zq);
                dqv = q < nf ? sg * rowbuf[q] : 0.0;  // d_q: slot q is not zeroed (only j < q)
                zn = fma(dqv, dqv, zq);
                const double dd = zn + sq;
                double z4[4] = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll
                for (int j = 0; j < NF; ++j) {
                    z4[j & 3] += Jr[j] * rowbuf[j];
                    if ((j % PFD) == PFD - 1) pin_fence4(z4);
                }
                z = sg * ((z4[0] + z4[1]) + (z4[2] + z4[3]));
                pin(z);  // here, not sunk to its use after the R solve: the row would stay live
                if (q > 0) {
                    if constexpr (!kRinv) {
                        // r = R^-1 d(0:q): uniform loop to the larger q of the two halves
                        const int qmax = max(__builtin_amdgcn_readlane(q, 0), __builtin_amdgcn_readlane(q, kHalf));
                        double val = dj;
                        for (int j = qmax - 1; j >= 0; --j) {
                            const double rj = hread_rt(val, j) * rinv[j];
                            if (j < q) {
                                if (hl == j) r = rj;
                                if (hl < j) val -= R[roff(j) + hl] * rj;
                            }
                        }
                    }
                    const double rmax = half_max(hl < q ? fabs(r) : 0.0);
                    if (hl < q && r > kRTol * rmax) t1 = u / r;
                    kslot = half_argmin_lane(t1);
                }
                const bool dep = !(zn > kDepTol * dd);
                t2 = dep ? INFINITY : -sp / zn;
                t = t1 < t2 ? t1 : t2;
                if (isinf(t)) { status = ST_INFEASIBLE; done = true; }
            }
            MPCQP_SUB(tsub, 1);
            MPCQP_CUT(a.cut, 21);
            const bool moving = stepping && !done;
            bool add = false;
            if (moving) {
                const double uq = uadd;
                if (!isinf(t2)) {
                    if (hl < nf) x += t * z;
                    fval += t * zn * (0.5 * t + uq);
                }
                if (hl < q) u -= t * r;
                uadd += t;
                if (hl == q) u = uadd;
                add = !isinf(t2) && t2 <= t1;
                if (add) {
                    // ---- add p: R column q = (d_0..d_{q-1}, r_qq); the reflection vector v = d2
                    //      - |d2| e_q goes to rowbuf (which holds d2 / sg), v = sg rowbuf
                    const double dq = dqv;
                    double rqq = dq, vq = 0.0;
                    if (zq > 0.0) {  // otherwise d2 = d_q e_q: no reflection, r_qq = d_q
                        const double nrm = sqrt(zn);
                        rqq = nrm;
                        vq = dq > 0.0 ? -zq / (dq + nrm) : dq - nrm;
                        beta = 2.0 / (vq * vq + zq);
                    }
                    wave_sync();
                    if (hl == q) rowbuf[q] = sg * vq;
                    if constexpr (kRinv) {
                        // R^-1 of [[R, d1], [0, rqq]] = [[R^-1, -R^-1 d1 / rqq], [0, 1 / rqq]], and
                        // R^-1 d1 is this pass's r
                        const double irq = 1.0 / rqq;
                        if (hl < q) Ri[lrow(q) + hl] = -r * irq;
                        if (hl == q) { Ri[lrow(q) + q] = irq; act = p; }
                    } else {
                        if (hl < q) R[roff(q) + hl] = dj;
                        if (hl == q) { R[roff(q) + q] = rqq; rinv[q] = 1.0 / rqq; act = p; }
                    }
                    if (hl == a_) stb &= lower ? ~1 : ~2;
                    ++q;
                    fresh = true;
                } else {
                    // ---- drop slot kslot: shift u / act and R's columns left, then Givens back
                    //      to triangular; the (c, s) pairs go to LDS for J
                    const int k = kslot;
                    const int dropped = hread_k(act, k);
                    const bool dlow = dropped < nf;
                    if (hl == (dlow ? dropped : dropped - nf)) stb |= dlow ? 1 : 2;
                    {
                        const int src = (hl + 1 < kHalf) ? ln + 1 : ln;
                        const double un = __shfl(u, src, kWave);
                        const int an = __shfl(act, src, kWave);
                        if (hl >= k && hl < q) { u = un; act = an; }
                    }
                    if constexpr (kRinv) {
                        // Removing column k of R and restoring the triangle with Givens G on rows
                        // (j, j+1), j = k .. q-2, is, for R^-1, R^-1 G' with row k then deleted and the
                        // last column dropped, where the same rotations zero row k of R^-1 G' left of
                        // column q-1 (row k of (G R)^-1 is a multiple of e_{q-1}').  So the rotations
                        // come from row k of R^-1 alone: every lane of the half runs the same chain
                        // a <- hypot(a, R^-1(k, j+1)) on broadcast reads; (c, s) go to LDS for J.
                        double ra = Ri[lrow(k) + k];
                        rot[2 * hl] = 1.0;
                        rot[2 * hl + 1] = 0.0;
                        wave_sync();
                        for (int j = k; j < q - 1; ++j) {
                            const double rb = Ri[lrow(j + 1) + k];
                            double c = 1.0, s_ = 0.0;
                            if (ra != 0.0) {
                                const double hh = sqrt(ra * ra + rb * rb), ih = 1.0 / hh;
                                c = rb * ih;
                                s_ = -ra * ih;
                                ra = hh;
                            } else {
                                ra = rb;
                            }
                            // lane i's entries (i, j), (i, j+1) of R^-1 G' (rows i <= j+1 are
                            // nonzero); rotated column j is final: it is written with row k deleted
                            // (rows below k move up one, so it fits its j+1 packed slots again),
                            // column j+1 goes back in place for the next rotation
                            const double y0 = (hl <= j) ? Ri[lrow(j) + hl] : 0.0;
                            const double y1 = (hl <= j + 1) ? Ri[lrow(j + 1) + hl] : 0.0;
                            if (hl == 0) {
                                rot[2 * j] = c;
                                rot[2 * j + 1] = s_;
                            }
                            if (hl <= j + 1 && hl != k) Ri[lrow(j) + hl - (hl > k ? 1 : 0)] = c * y0 + s_ * y1;
                            if (hl <= j + 1) Ri[lrow(j + 1) + hl] = -s_ * y0 + c * y1;
                            wave_sync();
                        }
                        --q;
                    } else {
                        for (int j = k; j < q - 1; ++j) {
                            const double v = (hl <= j + 1) ? R[roff(j + 1) + hl] : 0.0;
                            wave_sync();
                            if (hl <= j + 1) R[roff(j) + hl] = v;
                            wave_sync();
                        }
                        --q;
                        rot[2 * hl] = 1.0;
                        rot[2 * hl + 1] = 0.0;
                        wave_sync();
                        for (int j = k; j < q; ++j) {
                            const double aa = R[roff(j) + j], bb = R[roff(j) + j + 1];
                            if (bb != 0.0) {
                                const double hh = sqrt(aa * aa + bb * bb);
                                const double ih = 1.0 / hh;
                                const double c = aa * ih, s_ = bb * ih;
                                const int l = j + 1 + hl;
                                double r0 = 0.0, r1 = 0.0;
                                if (l < q) { r0 = R[roff(l) + j]; r1 = R[roff(l) + j + 1]; }
                                wave_sync();
                                if (l < q) {
                                    R[roff(l) + j] = c * r0 + s_ * r1;
                                    R[roff(l) + j + 1] = -s_ * r0 + c * r1;
                                }
                                if (hl == 0) {
                                    R[roff(j) + j] = hh;
                                    R[roff(j) + j + 1] = 0.0;
                                    rinv[j] = ih;
                                    rot[2 * j] = c;
                                    rot[2 * j + 1] = s_;
                                }
                                wave_sync();
                            } else {
                                if (hl == 0) rinv[j] = 1.0 / aa;
                                wave_sync();
                            }
                        }
                    }
                }
            }
            wave_sync();
            MPCQP_SUB(tsub, 2);
            MPCQP_CUT(a.cut, 22);
            if (!done && fresh) {
                // ---- most violated inactive bound (lowest id on ties): before the first step and
                //      right after every add, so a half's last add also ends its solve (no checking
                //      pass of its own, no update of J that nothing reads)
                double best = INFINITY;
                bool upb = false;  // the lane's candidate is its upper bound (id hl + nf)
                if (stb & 1) {
                    const double s_ = x - MPCQP_BLO;
                    if (s_ < MPCQP_TLO) best = s_;
                }
                if (stb & 2) {
                    const double s_ = -x - MPCQP_BHI;
                    if ((s_ < MPCQP_THI) & (s_ < best)) { best = s_; upb = true; }
                }
                // lowest id among the lanes at the minimum: a lower bound (id hl) before any upper
                // bound (hl + nf), each by lowest lane
                const double bm = half_min(best);
                const uint32_t hit = half_ballot(best == bm), hitl = half_ballot(best == bm && !upb);
                const int bid = bm == INFINITY ? 0x7fffffff
                              : hitl ? (int)__builtin_ctz(hitl) : (int)__builtin_ctz(hit) + nf;
                if (bid == 0x7fffffff) {
                    done = true;  // optimal
                } else {
                    p = bid;
                    if (hl == q) u = 0.0;
                    uadd = 0.0;
                    fresh = false;
                }
            }
            // ---- the pass's update of J, as ONE chain of wave-uniform steps (no divergent
            //      definition of Jr, so the register allocator keeps a single copy of it):
            //      add -> J2 (I - beta v v'), v = sg rowbuf (the signs cancel: J_j -= beta (J .
            //      rowbuf) rowbuf_j, f = 0 in a half that does not add); drop -> rotations from LDS,
            //      the identity in a half that does not drop
            const bool hh = moving && add && beta != 0.0 && !done;
            const bool rt = moving && !add;
            if (__ballot(hh) != 0ull) {
                double w4[4] = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll
                for (int j = 0; j < NF; ++j) {
                    w4[j & 3] += Jr[j] * rowbuf[j];
                    if ((j % PFD) == PFD - 1) pin_fence4(w4);
                }
                const double f = hh ? beta * ((w4[0] + w4[1]) + (w4[2] + w4[3])) : 0.0;
    #pragma unroll
                for (int j = 0; j < NF; ++j) {
                    Jr[j] -= f * rowbuf[j];
                    if ((j % PFD) == PFD - 1) step_fence();
                }
            }
            if (__ballot(rt) != 0ull) {
                if (!rt) {
                    rot[2 * hl] = 1.0;
                    rot[2 * hl + 1] = 0.0;
                }
                wave_sync();
    #pragma unroll
                for (int j = 0; j < NF - 1; ++j) {
                    const double c = rot[2 * j], s_ = rot[2 * j + 1];
                    const double y0 = Jr[j], y1 = Jr[j + 1];
                    Jr[j] = c * y0 + s_ * y1;
                    Jr[j + 1] = -s_ * y0 + c * y1;
                    if ((j % PFD) == PFD - 1) step_fence();
                }
            }
            wave_sync();
            MPCQP_SUB(tsub, 3);
            MPCQP_CUT(a.cut, 23);
        }
        MPCQP_SUB_FLUSH(a.stamps, tsub);
    #ifdef MPCQP_STAMPS
        if (a.stamps && ln == 0) atomicAdd(&a.stamps[2], npass);
    #endif
        if constexpr (GEN) {  // the dual loop's final active bounds (stb: bit cleared = active)
            if (a.warm && ok2 && status == ST_OK && hl < nf) {
                double lo, hi;
                pair_bound<NU, MODEL>(a, ~0ull, fid[hl], lo, hi);
                const int st0 = (lo > -kInfty ? 1 : 0) | (hi < kInfty ? 2 : 0);
                act2 |= st0 & ~stb & 3;
            }
            if (status != ST_OK) act2 = 0;
        }
    }

#undef MPCQP_BLO
#undef MPCQP_BHI
#undef MPCQP_TLO
#undef MPCQP_THI
    MPCQP_STAMP(a.stamps, 8, tst);
    MPCQP_CUT(a.cut, 7);
    // ---- outputs.  The lane-derived values (half lane, this half's LDS base and its free map)
    // are re-derived here from an opaque lane id: kept from the start they were 3 of the
    // kernel's spilled VGPRs
    int lno = lane();
    asm volatile("" : "+v"(lno));
    const int hlo = lno & (kHalf - 1);
    double *Do = reinterpret_cast<double *>(smem + (lno >= kHalf ? Lay::bytes : 0));
    const unsigned char *Dob = smem + (lno >= kHalf ? Lay::bytes : 0);
    const signed char *fido = reinterpret_cast<const signed char *>(Dob + Lay::oFid);
    const signed char *poso = reinterpret_cast<const signed char *>(Dob + Lay::oPos);
    const uint64_t *ctlo = reinterpret_cast<const uint64_t *>(Dob + Lay::oCt);
    const int bo = (int)(long long)ctlo[1];
    const bool defer = a.ovf && nf > NF && nf <= a.max_free;  // the workgroup kernel takes it
    {  // one append (one atomic) for the wavefront's deferred instances
        const int b0 = __builtin_amdgcn_readlane(bo, 0), b1 = __builtin_amdgcn_readlane(bo, kHalf);
        const uint64_t dm = __ballot(defer && bo >= 0);
        if (dm && lno == 0) wg_list_append(a.ovf, a.ovf_cap, b0, dm & 1ull, b1, (dm >> kHalf) & 1ull);
    }
    if constexpr (GEN) {
        // warm start: this tick's active bounds, in the global numbering (bit v lower, bit NV + v
        // upper: gi_reg.hpp WarmSet), for the next tick -- every instance of the launch writes
        // its words (zero when it was not solved)
        if (a.warm) {
            unsigned long long *wl = reinterpret_cast<unsigned long long *>(Do + Lay::oRow);
            wave_sync();
            if (hlo < a.warm_words) wl[hlo] = 0ull;
            wave_sync();
            if (bo >= 0 && hlo < nf && nf <= NF && act2) {
                const int v = fido[hlo];
                if (act2 & 1) atomicOr(&wl[v >> 6], 1ull << (v & 63));
                if (act2 & 2) atomicOr(&wl[(NV + v) >> 6], 1ull << ((NV + v) & 63));
            }
            wave_sync();
            if (bo >= 0 && hlo < a.warm_words) a.warm[(size_t)bo * a.warm_words + hlo] = wl[hlo];
            wave_sync();
        }
    }
    if (bo >= 0 && !defer) {
        // U assembled in LDS (the dead L / R space), then written once, coalesced: a
        // non-temporal store of a partial line is its own HBM write
        const uint64_t cto = *ctlo;
        double *U = a.U + (size_t)bo * NV;
        double *Us = Do + Lay::oR;
        const bool have_map = nf <= NF;
        wave_sync();
        for (int v = hlo; v < NV; v += kHalf) {
            const int pv = poso[v];
            if (pv < 0 || !have_map) {
                double lo, hi;
                pair_bound<NU, MODEL>(a, cto, v, lo, hi);
                Us[v] = (pv < 0) ? lo : 0.0;
            }
        }
        if (have_map && hlo < nf) Us[fido[hlo]] = x;
        wave_sync();
        for (int v = hlo; v < NV; v += kHalf) stream_store(U + v, Us[v]);
        if (hlo == 0) {
            stream_store(a.cost + bo, fval);
            stream_store(a.status + bo, status);
            stream_store(a.iters + bo, iters);
        }
    }
    if (a.flops_acc) {  // (diagnostic) both halves' solver flops, one atomic per wavefront
        const double t = (double)__builtin_amdgcn_readlane(sfl, 0) +
                         (double)__builtin_amdgcn_readlane(sfl, kHalf);
        if (lno == 0) atomicAdd(a.flops_acc + (blockIdx.x % kFlopsSlots) * kFlopsStride, t);
    }
#ifndef MPCQP_FUSED_SEL
#define MPCQP_FUSED_SEL 1
#endif
    if (MPCQP_FUSED_SEL && a.sel) {  // fused selection: the wave's smaller key (per-half status / cost)
        const unsigned long long kh =
            (bo >= 0 && !defer) ? sel_key(status, fval, a.sel_base + bo) : kSelNone;
        const unsigned long long k0 = readlane_u64(kh, 0), k1 = readlane_u64(kh, kHalf);
        wave_sync();  // the U staging reads are done: the L / R space is scratch again
        sel_commit_t(a, k0 < k1 ? k0 : k1, NV, true,
                     reinterpret_cast<unsigned long long *>(smem) + Lay::oR, -1, lno);
    }
    MPCQP_STAMP(a.stamps, 9, tst);
    (void)NS;
}

}  // namespace mpcqp
