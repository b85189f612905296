// mpc_fused.hpp -- one kernel for the whole per-tick step of the TRON1 models:
// linearise -> discretise -> condense -> solve, one QP per wavefront, nothing but U / cost /
// status / iterations leaving the chip.
//
// Reference: mpcQP::mpcQP + buildSystemModel (include/mpcQP.h:35-119, 121-182),
// QPSolver::discretizeSystem / buildQPParams / solveQP (src/QPSolver.cpp:21-106).
//
// Closed-form discretisation and condensing.  For both TRON1 models (the convex-MPC SRBM and
// the reference-literal 13x3) the continuous dynamics are nilpotent: with A = Ac Ts and
// B = Bc Ts, A^2 has a single non-zero (p_z <- g) and A^3 = 0, and the gravity row of Bc is
// zero so A^2 B = 0.  Hence, exactly,
//   exp([[A, B],[0, 0]]) = I + M + M^2/2 + M^3/6:   Ad = I + A + A^2/2,   Bd = B + AB/2
//   Ad^m = I + m A + m^2 A^2 / 2,     Phi_m = Ad^m Bd = B + (m + 1/2) A B.
// Eigen's Pade approximant (what the reference evaluates) agrees with this series to beyond
// the 4th power, so the two are equal in exact arithmetic; in fp64 they agree to ~1e-16
// (tests/test_gpu_parity.py).  With Phi_a = X0 + beta_a X1 (X0 = B, X1 = AB, beta_a = a+1/2)
// and diagonal weights W_m (Q for m < N, P for m = N):
//   H(i,j)/2 = sum_m sum_rs beta_i^r beta_j^s S^{W_m}_rs(c_i,c_j) + R(c_i,c_j)[k_i == k_j],
//   S^W_rs = X_r' W X_s  (eight 6x6 blocks, 13-deep),
// and the sums over m of 1, beta_i, beta_j, beta_i beta_j have closed forms.
//   f(i) = 2 sum_{m>k_i} (u_m(c_i) + beta_{m-1-k_i} v_m(c_i)),
//   u_m = X0' W_m e_m, v_m = X1' W_m e_m, e_m = x0 + m A x0 + m^2 A^2 x0 / 2 - xref_m.
#pragma once
#include "condense.hpp"
#include "gi_reg.hpp"
#include "gi_solver.hpp"

namespace mpcqp {

// one-QP kernels above 32 free variables start the solver with the blocked MFMA
// factorisation (chol_reg.hpp); MPCQP_REG_TILES=0 keeps the column sweeps (A/B builds)
#ifndef MPCQP_REG_TILES
#define MPCQP_REG_TILES 1
#endif
template <int NF>
constexpr bool kRegTiles = MPCQP_REG_TILES && NF > 32;

struct MpcArgs {
    int B;
    double Ts, mass;
    double Ibinv[9];
    const double *qd, *pd;  // diagonals of Q and P (device)
    const double *qm, *pm;  // Q and P, nx x nx column-major (device; the dense model)
    const double *fq, *fp;  // F with Q = F F', P = F F' (dense model, Toeplitz condensing)
    const double *rmat;     // R, nu x nu column-major (device)
    double fz_min, fz_max, fxy_max, u_min, u_max, mu;
    int max_iter, max_free;
    int crash_p;  // paired kernel: working sets of its crash start before the dual loop (0: none)
    int crash_p_wg;  // the workgroup solver's (gi_wg.hpp), box-only problems
    // paired kernel's bound constants, by kind of free variable (v: a vertical force, t: a
    // tangential force; the literal model's inputs use v): b of x >= lo (lo) and of -x >= -hi
    // (-hi), and the dual loop's violation thresholds -kFeasTol (1 + |b|), precomputed on the
    // host so the kernel selects them from scalar registers instead of keeping them per lane
    double blo_v, blo_t, bhi_v, bhi_t, tlo_v, tlo_t, thi_v, thi_t;
    const double *lin, *x0, *xref;
    const uint64_t *contact;
    double *U, *cost;
    int *status, *iters;
    unsigned long long *stamps;
    // diagnostic (mpcqp_count_solver_flops): the paired kernel adds the textbook flops of its
    // crash working-set solves and dual passes here (one atomic per wavefront, into slot
    // blockIdx % kFlopsSlots: 32,768 atomics on one address serialise); nullptr: off
    double *flops_acc;
    int cut;  // diagnostic cuts build only
    // device-generated inputs (GEN kernels): instance b = state b / cands,
    // candidate b % cands
    const double *state;  // [S][13]  [rpy, p, omega, v, g]
    const double *feet;   // [S][6]   r_L, r_R (foot minus CoM, world frame)
    const double *cmd;    // [S][2]   yaw rate, forward speed (include/mpcQP.h:75-76)
    const double *phase;  // [S * cands] gait phase of each candidate at step 0 (s)
    int cands;
    float swing, stance;  // MPCParam::swing_time / stance_time (float, include/MPCParam.h:48-49)
    int *ovf;  // overflow list (mpc_wg.hpp) for instances beyond the kernel's free capacity
    int ovf_cap;  // ids per sub-list (ovf_list_cap)
    unsigned long long *warm;  // GEN one-wave kernels: per-instance active-set words (WarmSet)
    int warm_words;
    // fused min-cost selection (mpcqp_batch_solve_select; nullptr: off).  sel: the running
    // minimum key's slots and the workgroup ticket (sel_commit); re-armed by the finalizer.
    // sel_final: this launch is the batch's last (the workgroup kernel when it runs), so its
    // last workgroup writes the record [key | winner's U] to sel_rec.
    unsigned long long *sel;
    long long sel_base;
    long long *sel_rec;
    int sel_final;
};

constexpr int kFlopsSlots = 256, kFlopsStride = 16;  // flops_acc: slots 128 B apart
constexpr int kFlopsWords = kFlopsSlots * kFlopsStride;

// ---- fused selection (the record of k_select_min, mpcqp_kernels.hip, without its launch)
constexpr unsigned long long kSelNone = 0x7fffffffffffffffull;
// order-preserving bits of a float (larger float -> larger unsigned), as k_select_min
__device__ __forceinline__ unsigned long long sel_order_bits(float c) {
    const unsigned u = __float_as_uint(c);
    return (u & 0x80000000u) ? (unsigned long long)(~u) : (unsigned long long)(u | 0x80000000u);
}
// key of a solved instance: (cost as fp32 bits) << 31 | global index; kSelNone if not solved
__device__ __forceinline__ unsigned long long sel_key(int status, double cost, long long gi) {
    return status == 0 ? (sel_order_bits((float)cost) << 31) | ((unsigned long long)gi & 0x7fffffffull)
                       : kSelNone;
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
// The running minimum lives in kSelSlots words 128 B apart (workgroup w mins into slot
// w % kSelSlots): one address taking an atomic from each of 32,768 wavefronts serialises them
// (~40 us per launch measured), 256 addresses do not.  The ticket follows the slots.
constexpr int kSelSlots = 256, kSelStride = 16, kSelTickets = 16;
// key slots, then kSelTickets ticket words and the global ticket, each on its own 128 B
constexpr int kSelWords = (kSelSlots + kSelTickets + 1) * kSelStride;
// the finalizer: the minimum over the slots (and k0), the winner's U row into the record, slots
// and tickets re-armed for the next call on the stream
__device__ __forceinline__ void sel_final_reduce(const MpcArgs &a, int nV,
                                                 unsigned long long *scratch, int tid,
                                                 unsigned long long k0) {
    const int nt = (int)blockDim.x;
    unsigned long long *sel_red = scratch;
    auto tword = [&](int i) { return reinterpret_cast<unsigned *>(&a.sel[(kSelSlots + i) * kSelStride]); };
    __syncthreads();  // (sel_red[0] may hold k0, read by every thread before this)
    unsigned long long m = k0;
    for (int sl = tid; sl < kSelSlots; sl += nt) {
        unsigned long long *w = &a.sel[sl * kSelStride];
        const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        m = v < m ? v : m;
        __hip_atomic_store(w, kSelNone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(m, o, 64);
        m = t < m ? t : m;
    }
    if ((tid & 63) == 0) sel_red[tid >> 6] = m;
    __syncthreads();
    m = sel_red[0];
    for (int w = 1; w < (nt + 63) / 64; ++w) m = sel_red[w] < m ? sel_red[w] : m;
    const bool none = m == kSelNone;
    const long long li = none ? 0 : (long long)(m & 0x7fffffffull) - (a.sel_base & 0x7fffffffll);
    double *ru = reinterpret_cast<double *>(a.sel_rec + 1);
    for (int e = tid; e < nV; e += nt) ru[e] = none ? 0.0 : a.U[(size_t)li * nV + e];
    if (tid <= kSelTickets)
        __hip_atomic_store(tword(tid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0) a.sel_rec[0] = (long long)m;
}

// Every thread of the workgroup, after its instances' U / cost / status are stored; k (thread
// 0's) is the workgroup's minimum key; wrote: it stored any instance in this launch.  In the finalizing launch the workgroup that takes the
// last ticket reduces the slots, copies the winner's U row (written by any workgroup of this or
// the previous launch: release / acquire at agent scope around the ticket) into the record and
// re-arms slots and ticket for the next call on the stream.
// scratch: 24 words of the caller's (dead) dynamic LDS, used only by a finalizing launch -- a
// static __shared__ here would add to every kernel's LDS and cost the one-QP kernel a wave per CU.
// groups: the workgroups 0 .. groups-1 that commit in a finalizing launch (the others must not
// call; default the whole grid)
// tid: the thread index (sel_commit passes threadIdx.x; a one-wave workgroup can pass its lane
// id, so that threadIdx.x need not live in a register from the kernel's entry)
// fresh: no workgroup of this launch stored an instance (the overflow list was empty), so every
// U row the finalizer may copy was stored by an earlier launch on the stream, which the kernel
// boundary makes visible; with one committing workgroup that finalizer then needs neither the
// ticket nor the agent-scope fence (~3.5 us of the empty overflow launch's ~8)
__device__ __forceinline__ void sel_commit_t(const MpcArgs &a, unsigned long long k, int nV,
                                             bool wrote, unsigned long long *scratch, int groups,
                                             int tid, bool fresh = false) {
    int &sel_last = *reinterpret_cast<int *>(scratch + 16);
    unsigned long long *sel_red = scratch;
    unsigned long long *slot = &a.sel[(blockIdx.x % kSelSlots) * kSelStride];
    if (!a.sel_final) {  // no-return atomic: the wavefront does not wait for it to complete
        if (tid == 0 && k != kSelNone)
            __hip_atomic_fetch_min(slot, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (fresh && groups == 1) {
        // the one committing workgroup of a launch that stored nothing: its own key (if any)
        // joins the slots' minimum below directly
        if (tid == 0) sel_red[0] = k;
        __syncthreads();
        sel_final_reduce(a, nV, scratch, tid, sel_red[0]);
        return;
    }
    unsigned long long prev = 0;
    if (tid == 0 && k != kSelNone)
        prev = __hip_atomic_fetch_min(slot, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the min has completed (its returned value is consumed) before the ticket below
    asm volatile("" : "+v"(prev));
    // two-level ticket: workgroup w counts into ticket word w % kSelTickets, and the one that
    // completes its word counts into the global word (the ~1,000 workgroups of a resident grid
    // on one address serialise for ~15 us)
    auto tword = [&](int i) { return reinterpret_cast<unsigned *>(&a.sel[(kSelSlots + i) * kSelStride]); };
    if (tid == 0) {
        // release this workgroup's U rows (an agent-scope fence writes L2 back: only a
        // workgroup that stored instances in this launch pays for one)
        if (wrote) __threadfence();
        // relaxed RMWs: acq_rel ones at agent scope would write L2 back in every workgroup
        const int g = groups > 0 ? groups : (int)gridDim.x, w = (int)(blockIdx.x % kSelTickets);
        const int words = g < kSelTickets ? g : kSelTickets;
        const unsigned need = (unsigned)((g - w + kSelTickets - 1) / kSelTickets);
        const unsigned t = __hip_atomic_fetch_add(tword(w), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool last = false;
        if (t == need - 1) {
            const unsigned u = __hip_atomic_fetch_add(tword(kSelTickets), 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            last = u == (unsigned)words - 1;
        }
        sel_last = last;
    }
    __syncthreads();
    if (!sel_last) return;
    __threadfence();
    sel_final_reduce(a, nV, scratch, tid, kSelNone);
}
__device__ __forceinline__ void sel_commit(const MpcArgs &a, unsigned long long k, int nV,
                                           bool wrote, unsigned long long *scratch, int groups = -1,
                                           bool fresh = false) {
    sel_commit_t(a, k, nV, wrote, scratch, groups, (int)threadIdx.x, fresh);
}

// Overflow list (int words).  One counter per 128 B line would still take one device-scope
// atomic per deferred wavefront on a single address, and those serialise (65,536 of them cost
// ~330 us per launch at B standing).  So the list is kListSubs sub-lists: wavefront w appends
// to sub-list w % kListSubs with ONE atomic for its deferred instances (both halves of a paired
// wave at once).  Layout: counter of sub-list s at word s * kListStride (its own 128 B line),
// then the sub-lists' ids, sub-list s at kListHeadWords + s * cap.  A wavefront appends at most
// two ids, so cap = ceil(B / kListSubs) + 2 (ovf_list_cap) holds every sub-list.
constexpr int kListSubs = 64, kListStride = 32;
constexpr int kListHeadWords = kListSubs * kListStride;
__host__ __device__ constexpr int ovf_list_cap(long long B) {
    return (int)((B + kListSubs - 1) / kListSubs) + 2;
}
// called by one lane: append ids b0 (if d0) and b1 (if d1) to this wavefront's sub-list
__device__ __forceinline__ void wg_list_append(int *list, int cap, int b0, bool d0, int b1,
                                               bool d1) {
    const int n = (d0 ? 1 : 0) + (d1 ? 1 : 0);
    if (!n) return;
    const int s = (int)(blockIdx.x % kListSubs);
    const int i = __hip_atomic_fetch_add(&list[s * kListStride], n, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    int *ids = list + kListHeadWords + s * cap + i;
    if (d0) *ids++ = b0;
    if (d1) *ids = b1;
}
// the reader's view (k_mpc_wg, every wavefront alike): lane l holds sub-list l's count and the
// inclusive prefix sum, so entry i of the concatenated list is one ballot away
struct OvfView {
    int *list;
    int cap, cnt, incl, total;
    __device__ __forceinline__ int id(int i) const {  // wave-uniform i < total
        const int s = __popcll(__ballot(incl <= i));
        const int excl = __shfl(incl - cnt, s, kWave);
        return list[kListHeadWords + s * cap + (i - excl)];
    }
};
__device__ __forceinline__ OvfView ovf_view(int *list, int cap) {
    static_assert(kListSubs == kWave, "one sub-list per lane");
    OvfView v;
    v.list = list;
    v.cap = cap;
    v.cnt = __hip_atomic_load(&list[lane() * kListStride], __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
    int x = v.cnt;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const int y = __shfl_up(x, o, kWave);
        if (lane() >= o) x += y;
    }
    v.incl = x;
    v.total = __builtin_amdgcn_readlane(x, kWave - 1);
    return v;
}

// Gait contact mask of one horizon: MPC::calculateGait (include/MPCController.h:61-75)
// evaluated at phase0 + k Ts for k = 0..N-1 (lane k, exact fmod as the host's math.fmod);
// bit 2k = left foot in contact, 2k+1 = right.  Wave-uniform result.
__device__ __forceinline__ uint64_t spread_even(uint64_t x) {  // bit i -> bit 2i (i < 32)
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}
__device__ __forceinline__ uint64_t gait_mask_wave(int N, double Ts, double phase0, float swing,
                                                   float stance) {
    const double cycle = (double)(swing + stance), sw = (double)swing;
    const int ln = lane();
    const double ph = fmod(phase0 + (double)ln * Ts, cycle);
    const uint64_t right = __ballot(ln < N && ph < sw) & 0xffffffffull;
    const uint64_t left = __ballot(ln < N && !(ph < sw)) & 0xffffffffull;
    return spread_even(left) | (spread_even(right) << 1);
}

// Nonzero rows of X0 = Bc Ts and X1 = Ac Bc Ts^2 for the two TRON1 models (compile time):
// SRBM: Bc rows 6-11 (omega, v), Ac maps those to rows 0-5 (Theta, p); literal: Bc rows 9-11,
// Ac maps them to rows 3-5.  The supports are disjoint, so X0' W X1 = 0 for diagonal W: only
// the (0,0) and (1,1) blocks of S^W are nonzero, each over the support rows only.
template <int MODEL>
struct XSupport {
    static constexpr int x0lo = MODEL == 0 ? 6 : 9, x0hi = 12;
    static constexpr int x1lo = MODEL == 0 ? 0 : 3, x1hi = 6;
    static_assert(x0hi - x0lo == x1hi - x1lo, "equal support sizes");
    static_assert(x1hi <= x0lo, "disjoint supports");
};

template <int NU, int N, bool FRIC, int NF>
struct MpcLayout {
    static_assert(NF <= 64, "the register solver holds at most 64 free variables");
    static constexpr int NX = 13, NV = NU * N, LD = NF | 1;
    static constexpr int NFRIC = FRIC ? 4 * N * 2 : 0;
    static constexpr int MT = 2 * NF + NFRIC;
    static constexpr bool REG = true;
    static constexpr int NR = RegPack<NF>::doubles;  // packed L / R
    // doubles.  Live for the whole kernel: the x mirror, fixed values, the bounds' b; then one
    // region the phases take turns on (relative offsets):
    //   model/condensing : T = [Ac | Bc] (scratch), X0, X1, A x0, A^2 x0, xref, x0 at [0, E)
    //   condensed terms  : S (4 nonzero blocks, entry-major), u/v, R copy at [max(E, HB), ..)
    //   H_FF build       : packed H at [0, HB), HB = NF(NF+1)/2, reading the condensed terms
    //   solver           : packed L / R at [0, NR), then 5 NF broadcast / 1/R(j,j) doubles
    static constexpr int oXS = 0;                         // x mirror (NF)
    // no xfull: every fixed input of these models is 0 (a swing foot's forces; the literal
    // model has none), so C.L.xfull = nullptr and the solver reads 0 (gi_solver.hpp)
    static constexpr int oMisc = oXS + NF;                // rowfix / ys slot
    static constexpr int oCB = oMisc + 2;                 // b of the bound constraints (2 NF)
    static constexpr int oU = (oCB + 2 * NF + 1) & ~1;    // the shared region (16-B aligned)
    // early-phase view
    static constexpr int oT = oU;                         // [Ac | Bc] (NX x (NX+NU))
    static constexpr int oX0 = oT + NX * (NX + NU);       // B  (NX x NU)
    static constexpr int oX1 = oX0 + NX * NU;             // AB (NX x NU)
    static constexpr int oAx = oX1 + NX * NU;             // A x0, A^2 x0 (2 NX)
    static constexpr int oXr = oAx + 2 * NX;              // xref (NX x (N+1))
    static constexpr int oX0v = oXr + NX * (N + 1);       // x0 (NX)
    static constexpr int nEarly = oX0v + NX + 1 - oU;
    static constexpr int HB = NF * (NF + 1) / 2;
    // condensed terms, live until H_FF and g are built
    static constexpr int oS = oU + (((nEarly > HB ? nEarly : HB) + 1) & ~1);  // [NU*NU][4]
    // u_m, v_m: [(N+1)][2][NU], m = 1..N used (slot m = 0 overlaps the end of S, never touched)
    static constexpr int oUV = oS + 4 * NU * NU - 2 * NU;
    static constexpr int oRm = oUV + (N + 1) * 2 * NU;    // R (NU x NU) copy
    static constexpr int nMid = oRm + NU * NU - oU;
    // solver view
    static constexpr int oR = oU;                         // packed L / R (and H_FF before)
    static constexpr int oRow = (oR + NR + 1) & ~1;       // broadcast buffers (4 NF) + 1/R(j,j)
    static constexpr int nLate = oRow + 5 * NF - oU;
    static constexpr int nShared = nMid > nLate ? nMid : nLate;
    static constexpr int nDoubles = oU + nShared;
    static constexpr size_t bytes =
        sizeof(double) * nDoubles + sizeof(int) * (NF + NV) + ((MT + 15) & ~15);
    static constexpr size_t lds_bytes = (bytes + 15) & ~(size_t)15;
    static_assert(oRow % 2 == 0 && oU % 2 == 0 && oS % 2 == 0, "16-byte aligned buffers");
    static_assert(NV <= NR, "gi_write stages x in the packed R space");
    static_assert(HB <= NR, "packed H fits the L / R space");
};

// sum over m in [m0, m1] of 1, beta_i, beta_j, beta_i beta_j; beta_x = m - 1 - k_x + 1/2
__device__ __forceinline__ void beta_sums(int m0, int m1, int ki, int kj, double &c, double &si,
                                          double &sj, double &sij) {
    if (m1 < m0) { c = si = sj = sij = 0.0; return; }
    const double n = (double)(m1 - m0 + 1);
    const double s1 = 0.5 * (double)(m0 + m1) * n;  // sum m
    auto S2 = [](int t) { return (double)(t * (t + 1) * (2 * t + 1) / 6); };  // exact in int
    const double s2 = S2(m1) - S2(m0 - 1);           // sum m^2
    const double oi = (double)ki + 0.5, oj = (double)kj + 0.5;
    c = n;
    si = s1 - oi * n;
    sj = s1 - oj * n;
    sij = s2 - (oi + oj) * s1 + oi * oj * n;
}

// ---- phases of the fused step shared by the one-wave kernel (fast_mpc below) and the
//      workgroup kernel (mpc_wg.hpp); each runs on ONE wave.  Lay provides the LDS offsets
//      (doubles from D): oXr, oX0v, oRm, oT, oX0, oX1, oAx, oS, oUV.

// per-instance inputs of instance b (x0, xref, R, lin)
template <class Lay, int NU, int N, bool GEN>
__device__ __forceinline__ void mpc_load_inputs(const MpcArgs &a, int b, double *D,
                                                double (&lin)[8]) {
    constexpr int NX = 13;
    const int ln = lane();
    const int st_ = GEN ? b / a.cands : b;  // state row of this instance (GEN)
    // ---- per-instance inputs: all global loads issued back to back (one HBM round trip),
    //      then parked in LDS
    double *xr = D + Lay::oXr, *x0g = D + Lay::oX0v;
    if constexpr (GEN) {
        // x0 = the state; xref as mpcQP::mpcQP builds it (include/mpcQP.h:74-97) from the
        // state and the (yaw rate, forward speed) command; lin = {yaw, r_L, r_R}
        const double st = (ln < NX) ? a.state[(size_t)st_ * NX + ln] : 0.0;
        const double wz = a.cmd[(size_t)st_ * 2], vx = a.cmd[(size_t)st_ * 2 + 1];
#pragma unroll
        for (int i = 0; i < 6; ++i) lin[1 + i] = a.feet[(size_t)st_ * 6 + i];
        lin[7] = 0.0;
        const double rml = (ln < NU * NU) ? a.rmat[ln] : 0.0;
        if (ln < NX) x0g[ln] = st;
        if (ln < NU * NU) D[Lay::oRm + ln] = rml;
        lin[0] = readlane(st, 2);
        if (ln < NX) {
#pragma unroll
            for (int i = 0; i <= N; ++i) {
                const double t = (double)i * a.Ts;
                double v = st;
                if (ln == 2) v = st + t * wz;
                if (ln == 3) v = st + t * vx;
                if (ln == 9 && i > 0) v = vx;
                if (ln == 12) v = -9.8;
                xr[i * NX + ln] = v;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) lin[i] = stream_load(a.lin + (size_t)b * 8 + i);
        constexpr int NXR = NX * (N + 1), RX = (NXR + kWave - 1) / kWave;
        const double *xrg = a.xref + (size_t)b * NXR;
        double v[RX];
#pragma unroll
        for (int r = 0; r < RX; ++r) v[r] = (ln + r * kWave < NXR) ? stream_load(xrg + ln + r * kWave) : 0.0;
        const double x0l = (ln < NX) ? stream_load(a.x0 + (size_t)b * NX + ln) : 0.0;
        const double rml = (ln < NU * NU) ? a.rmat[ln] : 0.0;
#pragma unroll
        for (int r = 0; r < RX; ++r)
            if (ln + r * kWave < NXR) xr[ln + r * kWave] = v[r];
        if (ln < NX) x0g[ln] = x0l;
        if (ln < NU * NU) D[Lay::oRm + ln] = rml;
    }
    wave_sync();
    (void)st_;
}

// model: X0 = Bc Ts, X1 = (Ac Ts)(Bc Ts); A x0, A^2 x0
template <class Lay, int NU, int MODEL>
__device__ __forceinline__ void mpc_model_terms(const MpcArgs &a, double *D,
                                                const double (&lin)[8]) {
    constexpr int NX = 13, NS = NX + NU;
    const int ln = lane();
    double *X0 = D + Lay::oX0, *X1 = D + Lay::oX1, *Ax = D + Lay::oAx, *A2x = Ax + NX;
    double *x0g = D + Lay::oX0v;
    double Iwi[9];
    double cy = 1.0, sy = 0.0;
    if (MODEL == 0) srbm_rot_inertia(lin[0], a.Ibinv, cy, sy, Iwi);
    auto entry = [&](int i, int j) -> double {  // [Ac | Bc](i, j)
        return MODEL == 0 ? srbm_entry(i, j, lin, cy, sy, Iwi, a.mass)
                          : literal_entry(i, j, lin, a.mass);
    };
    const double Ts = a.Ts;
    // [Ac | Bc] into LDS once, lane i writing row i with compile-time columns (the R space is
    // free until H_FF is built there); the products then read it
    double *T = D + Lay::oT;
    if (ln < NX) {
#pragma unroll
        for (int j = 0; j < NS; ++j) T[j * NX + ln] = entry(ln, j);
    }
    wave_sync();
    for (int e = ln; e < NX * NU; e += kWave) X0[e] = T[NX * NX + e] * Ts;
    if (ln < NX) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) s += T[k * NX + ln] * x0g[k];
        Ax[ln] = s * Ts;
    }
    wave_sync();
    for (int e = ln; e < NX * NU; e += kWave) {
        const int i = e % NX, c = e / NX;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) s += T[k * NX + i] * X0[c * NX + k];
        X1[e] = s * Ts;
    }
    if (ln < NX) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NX; ++k) s += T[k * NX + ln] * Ax[k];
        A2x[ln] = s * Ts;
    }
    wave_sync();
}

// condensed terms: the S^W blocks and u_m / v_m
template <class Lay, int NU, int N, int MODEL>
__device__ __forceinline__ void mpc_condensed_terms(const MpcArgs &a, double *D) {
    constexpr int NX = 13;
    const int ln = lane();
    double *X0 = D + Lay::oX0, *X1 = D + Lay::oX1, *S = D + Lay::oS, *UV = D + Lay::oUV;
    double *Ax = D + Lay::oAx, *A2x = Ax + NX;
    double *xr = D + Lay::oXr, *x0g = D + Lay::oX0v;
    // ---- S^W_rr = X_r' W X_r over the support rows (w: 0 = Q, 1 = P); slot blk = 2w + r of
    //      entry o = cj NU + ci (the cross blocks X0' W X1 are zero and not stored).
    //      The block loop is wave-uniform so the weights are scalar loads.
    using Sup = XSupport<MODEL>;
    constexpr int SD = Sup::x0hi - Sup::x0lo;
#pragma unroll
    for (int blk = 0; blk < 4; ++blk) {
        const int r_ = blk & 1, w_ = blk >> 1;
        const int lo = r_ ? Sup::x1lo : Sup::x0lo;
        const double *Xr = r_ ? X1 : X0;
        const double *w = w_ ? a.pd : a.qd;
        for (int e = ln; e < NU * NU; e += kWave) {
            const int ci = e % NU, cj = e / NU;
            double acc = 0.0;
#pragma unroll
            for (int l = lo; l < lo + SD; ++l) acc += Xr[ci * NX + l] * w[l] * Xr[cj * NX + l];
            S[e * 4 + blk] = acc;  // [o = cj NU + ci][blk]: one entry's terms contiguous
        }
    }
    // ---- u_m(c) = X0[:,c]' W_m e_m, v_m(c) = X1[:,c]' W_m e_m, m = 1..N (support rows only)
    for (int e = ln; e < N * NU; e += kWave) {
        const int c = e % NU, m = 1 + e / NU;
        const double md = (double)m, hm2 = 0.5 * md * md;
        auto el = [&](int l) {
            const double wl = (m < N) ? a.qd[l] : a.pd[l];
            return wl * (x0g[l] + md * Ax[l] + hm2 * A2x[l] - xr[m * NX + l]);
        };
        double su = 0.0, sv = 0.0;
#pragma unroll
        for (int l = Sup::x0lo; l < Sup::x0hi; ++l) su += X0[c * NX + l] * el(l);
#pragma unroll
        for (int l = Sup::x1lo; l < Sup::x1hi; ++l) sv += X1[c * NX + l] * el(l);
        UV[(m * 2 + 0) * NU + c] = su;
        UV[(m * 2 + 1) * NU + c] = sv;
    }
    wave_sync();
}

// H_FF(vi, vj) and g(vi) of the condensed problem from the terms above (closed form; the
// cross blocks X0' W X1 vanish, XSupport)
template <class Lay, int NU, int N>
__device__ __forceinline__ double mpc_h_entry(const double *D, int vi, int vj) {
    const int ki = vi / NU, ci = vi % NU, kj = vj / NU, cj = vj % NU;
    const int kk = ki > kj ? ki : kj;
    double c, si, sj, sij;
    beta_sums(kk + 1, N - 1, ki, kj, c, si, sj, sij);
    const double bi = (double)(N - 1 - ki) + 0.5, bj = (double)(N - 1 - kj) + 0.5;
    const double *So = D + Lay::oS + (cj * NU + ci) * 4;
    double v = c * So[0] + sij * So[1];
    v += So[2] + bi * bj * So[3];
    if (ki == kj) v += D[Lay::oRm + cj * NU + ci];
    return 2.0 * v;
}
template <class Lay, int NU, int N>
__device__ __forceinline__ double mpc_g_entry(const double *D, int vi) {
    const int ki = vi / NU, ci = vi % NU;
    const double *UV = D + Lay::oUV;
    double s = 0.0;
    for (int m = ki + 1; m <= N; ++m) {
        const double beta = (double)(m - 1 - ki) + 0.5;
        s += UV[(m * 2 + 0) * NU + ci] + beta * UV[(m * 2 + 1) * NU + ci];
    }
    return 2.0 * s;
}

// b_in < 0: instance xcd_order(blockIdx.x) of the batch, deferred to the overflow list when its
// free forces exceed NF, its key committed to the fused selection here.  b_in >= 0 (the
// overflow list's one-wave kernel, k_mpc_list): that instance, never deferred (more than NF
// free forces: ST_BAD_DIMS), its selection key returned in *key_out instead of committed.
template <int NU, int N, int MODEL, bool FRIC, int NF, bool GEN = false>
__device__ __forceinline__ void fast_mpc(const MpcArgs &a, unsigned char *smem, int b_in = -1,
                                         unsigned long long *key_out = nullptr) {
    static_assert(!GEN || MODEL == 0, "generated inputs are defined for the SRBM model");
    using Lay = MpcLayout<NU, N, FRIC, NF>;
    constexpr int NX = 13, NS = NX + NU, NV = Lay::NV, LD = Lay::LD;
    const bool listed = b_in >= 0;
    const int b = listed ? b_in : xcd_order((int)blockIdx.x, (int)gridDim.x), ln = lane();
    double *D = reinterpret_cast<double *>(smem);
    double *S = D + Lay::oS, *UV = D + Lay::oUV;
    static_assert(MODEL == 0 || MODEL == 1, "TRON1 models only");
    MPCQP_STAMP_INIT(tst);

    // ---- solver context (bounds from the contact schedule)
    SolveProblem P;
    P.nV = NV;
    P.H = nullptr; P.f = nullptr; P.lb = nullptr; P.ub = nullptr;
    P.gen_bounds = 1;
    P.model = MODEL; P.nu = NU; P.N = N; P.nfeet = 2;
    P.fz_min = a.fz_min; P.fz_max = a.fz_max; P.fxy_max = a.fxy_max;
    P.u_min = a.u_min; P.u_max = a.u_max;
    P.contact = (MODEL != 0) ? 0ull
              : GEN ? gait_mask_wave(N, a.Ts, a.phase[b], a.swing, a.stance) : stream_load(a.contact + b);
    P.friction = FRIC ? 1 : 0;
    P.mu = a.mu;
    P.mA = 0; P.A = nullptr; P.a_colmajor = 0; P.lbA = nullptr; P.ubA = nullptr;
    P.max_iter = a.max_iter;
    GiCtx C;
    C.wide = 0;
    C.stamps = a.stamps;
    C.cut = a.cut;
    C.P = &P;
    C.nfmax = NF;
    C.L.ld = LD;
    C.L.R = D + Lay::oR;
    C.L.J = nullptr;
    C.L.g = nullptr;
    C.L.xs = D + Lay::oXS;
    C.L.xfull = nullptr;  // fixed inputs are 0 (MpcLayout)
    C.L.rowfix = D + Lay::oMisc;
    C.L.ys = D + Lay::oMisc;
    int *ip = reinterpret_cast<int *>(D + Lay::nDoubles);
    C.L.fid = ip;
    C.L.pos = ip + NF;
    C.L.st = reinterpret_cast<unsigned char *>(ip + NF + NV);
    C.L.cb = D + Lay::oCB;

    double lin[8];
    mpc_load_inputs<Lay, NU, N, GEN>(a, b, D, lin);
    MPCQP_CUT(a.cut, 11);
    // the free map first (it reads only the bounds and the contact schedule): an instance the
    // workgroup kernel takes returns before the model terms
    gi_setup(C);  // free map + constraint states
    if (C.nf > a.max_free || (listed && C.nf > NF)) C.status = ST_BAD_DIMS;
    wave_sync();
    if (!listed && a.ovf && C.nf > NF && C.nf <= a.max_free) {  // the overflow kernel takes it
        if (ln == 0) wg_list_append(a.ovf, a.ovf_cap, b, true, 0, false);
        return;
    }
    mpc_model_terms<Lay, NU, MODEL>(a, D, lin);
    MPCQP_CUT(a.cut, 13);
    MPCQP_STAMP(a.stamps, 0, tst);
    MPCQP_CUT(a.cut, 1);

    mpc_condensed_terms<Lay, NU, N, MODEL>(a, D);
    MPCQP_STAMP(a.stamps, 1, tst);
    MPCQP_CUT(a.cut, 2);

    // ---- H_FF (lane p builds row p) and g
    const int nf = C.nf;
    const bool ok = C.status == ST_OK && nf > 0;
    double gp = 0.0;
    if (ok && ln < nf) {
        const int vi = C.L.fid[ln], ki = vi / NU, ci = vi % NU;
        double s = 0.0;
        for (int m = ki + 1; m <= N; ++m) {
            const double beta = (double)(m - 1 - ki) + 0.5;
            s += UV[(m * 2 + 0) * NU + ci] + beta * UV[(m * 2 + 1) * NU + ci];
        }
        gp = 2.0 * s;
    }
    C.c0 = 0.0;
    if constexpr (Lay::REG) {
        // lower triangle of H_FF, packed index e -> (p >= q), built by all lanes into the
        // (still empty) R buffer, then lane p loads row p; rows/cols >= nf are padded with
        // the identity so the register factorization runs without predicates
        double *Hb = C.L.R;
        if (ok) {
            // one lane per block pair (ki >= kj), row-major packed over the N(N+1)/2 pairs:
            // the beta sums are per block, then the lane walks its block's free entries
            constexpr int NPAIR = N * (N + 1) / 2;
            const int *pos = C.L.pos;
            int ki = 0, kj = ln;
            while (kj > ki) { kj -= ki + 1; ++ki; }
            for (int bp = ln; bp < NPAIR; bp += kWave) {
                double c, si, sj, sij;
                beta_sums(ki + 1, N - 1, ki, kj, c, si, sj, sij);
                const double bi = (double)(N - 1 - ki) + 0.5, bj = (double)(N - 1 - kj) + 0.5;
                const double bij = bi * bj;
                int mi = 0, mj = 0;
#pragma unroll
                for (int cc = 0; cc < NU; ++cc) {
                    mi |= (pos[ki * NU + cc] >= 0) << cc;
                    mj |= (pos[kj * NU + cc] >= 0) << cc;
                }
                for (int ri = mi; ri; ri &= ri - 1) {
                    const int ci = __builtin_ctz(ri), pp = pos[ki * NU + ci];
                    for (int rj = mj; rj; rj &= rj - 1) {
                        const int cj = __builtin_ctz(rj), qq = pos[kj * NU + cj];
                        if (pp >= qq) {
                            const double *So = S + (cj * NU + ci) * 4;
                            double v = c * So[0] + sij * So[1];  // cross blocks zero
                            v += So[2] + bij * So[3];
                            if (ki == kj) v += D[Lay::oRm + cj * NU + ci];
                            Hb[lrow(pp) + qq] = 2.0 * v;
                        }
                    }
                }
                kj += kWave;
                while (kj > ki) { kj -= ki + 1; ++ki; }
            }
        }
        wave_sync();
        double h[NF];
        if constexpr (!kRegTiles<NF>) {
#pragma unroll
            for (int q = 0; q < NF; ++q) {
                const bool in = ok && ln < nf && q < nf && q <= ln;
                h[q] = in ? Hb[lrow(ln) + q] : ((q == ln) ? 1.0 : 0.0);
            }
            wave_sync();
        }
        MPCQP_STAMP(a.stamps, 3, tst);
        MPCQP_CUT(a.cut, 3);
        if (GEN && a.warm) {
            WarmSet ws{a.warm + (size_t)b * a.warm_words, a.warm_words};
            gi_run_reg<NF, kRegTiles<NF>>(C, h, gp, D + Lay::oRow, &ws);
        } else {
            gi_run_reg<NF, kRegTiles<NF>>(C, h, gp, D + Lay::oRow);
        }
    }
#ifdef MPCQP_CUTS
    if (a.cut >= 4 && a.cut <= 7) return;
#endif
    MPCQP_STAMP_INIT(tw);
    SolveOut O;
    O.x = a.U + (size_t)b * NV;
    O.cost = a.cost + b;
    O.status = a.status + b;
    O.iters = a.iters + b;
    O.y = nullptr;
    O.stage = C.L.R;  // the packed R is dead after the solve
    gi_write(C, O);
    // (a deferred instance returned above; its key comes from the workgroup kernel, which then
    // is the finalizing launch)
    if (listed) {
        if (key_out) *key_out = sel_key(C.status, C.fval + C.c0, a.sel_base + b);
    } else if (a.sel) {
        sel_commit(a, sel_key(C.status, C.fval + C.c0, a.sel_base + b), NV, true,
                   reinterpret_cast<unsigned long long *>(D + Lay::oR));
    }
    MPCQP_STAMP(a.stamps, 9, tw);
    (void)NS;
}

}  // namespace mpcqp
