// wave_ops.hpp -- 64-lane wavefront primitives for the one-QP-per-wavefront kernels (gfx950).
//
// Every kernel in this library runs one problem instance per 64-lane wavefront (one wave per
// workgroup), so all control flow inside an instance is wave-uniform and these helpers can
// assume a full, converged wave.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpcqp {

constexpr int kWave = 64;

__device__ __forceinline__ int lane() { return (int)__lane_id(); }

// XCD-aware workgroup order (cdna_hip_programming.md T1, the bijective form): the dispatcher
// deals workgroups round-robin over the 8 XCDs, so workgroups w and w + 1 sit on different
// XCDs and every 128-B line shared by neighbouring instances (x0, lin, contact, the edges of
// xref and U, cost / status / iterations) is fetched, and partially written, by several XCDs'
// L2s.  Renumbered so that the workgroups of one XCD take one contiguous range of instances.
// A speed choice only: any bijection is correct.
#ifndef MPCQP_XCD_REMAP
#define MPCQP_XCD_REMAP 1
#endif
__device__ __forceinline__ int xcd_order(int w, int G) {
#if MPCQP_XCD_REMAP
    const int q = G >> 3, r = G & 7, x = w & 7, s = w >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
#else
    (void)G;
    return w;
#endif
}

// Broadcast lane `src` (wave-uniform index) of a double to the whole wave (v_readlane x2).
__device__ __forceinline__ double readlane(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ int readlane(int v, int src) {
    return __builtin_amdgcn_readlane(v, src);
}

// ---- reductions: DPP within each 16-lane row (xor 1, xor 2, half-row mirror, row mirror:
//      after the four steps every lane of a row holds the row's result, bit-identical because
//      each step combines a pair symmetrically), then the four row results are read into
//      SGPRs and combined in a fixed order, so the result is wave-uniform.  No LDS traffic
//      (ds_bpermute costs an LDS round trip per step).
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // lane i <- lane 7-i within each 8
constexpr int kDppMirror = 0x140;     // lane i <- lane 15-i within each 16

// mov_dpp (no tied `old` operand): every control used here reads a valid lane for every lane,
// or (bound_ctrl) writes 0 where it does not, so no register needs pre-loading with an old value
template <int CTRL>
__device__ __forceinline__ int dpp(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = dpp<CTRL>((int)(b & 0xffffffffll));
    const int hi = dpp<CTRL>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// DPP move that reads 0 where the source lane is outside the row
template <int CTRL>
__device__ __forceinline__ double dpp_z(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// lane l gets lane l + 1's value (DPP wave_shl:1, crosses rows; lane 63 gets 0)
__device__ __forceinline__ double wave_next(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x130, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// lane l gets lane l - 1's value (DPP wave_shr:1, crosses rows; lane 0 gets 0)
__device__ __forceinline__ double wave_prev(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffffll), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x138, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// inclusive suffix sum over the wave: lane l gets sum_{i >= l} v_i.  row_shl 1,2,4,8 scans
// each 16-lane row; the rows after this one are added from their totals (lanes 16, 32, 48).
__device__ __forceinline__ double wave_suffix_sum(double v) {
    v += dpp_z<0x101>(v);
    v += dpp_z<0x102>(v);
    v += dpp_z<0x104>(v);
    v += dpp_z<0x108>(v);
    const double r1 = readlane(v, 16), r2 = readlane(v, 32), r3 = readlane(v, 48);
    const int row = lane() >> 4;
    const double add = row == 0 ? (r1 + r2) + r3 : row == 1 ? r2 + r3 : row == 2 ? r3 : 0.0;
    return v + add;
}

// inclusive prefix sum over the wave: lane l gets sum_{i <= l} v_i.  row_shr 1,2,4,8 scans each
// 16-lane row; the rows before this one are added from their totals (lanes 15, 31, 47)
__device__ __forceinline__ double wave_prefix_sum(double v) {
    v += dpp_z<0x111>(v);
    v += dpp_z<0x112>(v);
    v += dpp_z<0x114>(v);
    v += dpp_z<0x118>(v);
    const double r0 = readlane(v, 15), r1 = readlane(v, 31), r2 = readlane(v, 47);
    const int row = lane() >> 4;
    const double add = ((row >= 1 ? r0 : 0.0) + (row >= 2 ? r1 : 0.0)) + (row >= 3 ? r2 : 0.0);
    return v + add;
}

__device__ __forceinline__ double wave_sum(double v) {
    v += dpp<kDppXor1>(v);
    v += dpp<kDppXor2>(v);
    v += dpp<kDppHalfMirror>(v);
    v += dpp<kDppMirror>(v);
    return (readlane(v, 0) + readlane(v, 16)) + (readlane(v, 32) + readlane(v, 48));
}
// two independent sums in one pass (the DPP chains interleave)
__device__ __forceinline__ void wave_sum2(double &a, double &b) {
    a += dpp<kDppXor1>(a);
    b += dpp<kDppXor1>(b);
    a += dpp<kDppXor2>(a);
    b += dpp<kDppXor2>(b);
    a += dpp<kDppHalfMirror>(a);
    b += dpp<kDppHalfMirror>(b);
    a += dpp<kDppMirror>(a);
    b += dpp<kDppMirror>(b);
    a = (readlane(a, 0) + readlane(a, 16)) + (readlane(a, 32) + readlane(a, 48));
    b = (readlane(b, 0) + readlane(b, 16)) + (readlane(b, 32) + readlane(b, 48));
}
// three independent sums in one pass
__device__ __forceinline__ void wave_sum3(double &a, double &b, double &c) {
    a += dpp<kDppXor1>(a);
    b += dpp<kDppXor1>(b);
    c += dpp<kDppXor1>(c);
    a += dpp<kDppXor2>(a);
    b += dpp<kDppXor2>(b);
    c += dpp<kDppXor2>(c);
    a += dpp<kDppHalfMirror>(a);
    b += dpp<kDppHalfMirror>(b);
    c += dpp<kDppHalfMirror>(c);
    a += dpp<kDppMirror>(a);
    b += dpp<kDppMirror>(b);
    c += dpp<kDppMirror>(c);
    a = (readlane(a, 0) + readlane(a, 16)) + (readlane(a, 32) + readlane(a, 48));
    b = (readlane(b, 0) + readlane(b, 16)) + (readlane(b, 32) + readlane(b, 48));
    c = (readlane(c, 0) + readlane(c, 16)) + (readlane(c, 32) + readlane(c, 48));
}
__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, dpp<kDppXor1>(v));
    v = fmax(v, dpp<kDppXor2>(v));
    v = fmax(v, dpp<kDppHalfMirror>(v));
    v = fmax(v, dpp<kDppMirror>(v));
    return fmax(fmax(readlane(v, 0), readlane(v, 16)), fmax(readlane(v, 32), readlane(v, 48)));
}

template <int CTRL, bool MIN>
__device__ __forceinline__ void arg_step(double &v, int &idx) {
    const double ov = dpp<CTRL>(v);
    const int oi = dpp<CTRL>(idx);
    // bitwise, not short-circuit: no branch per step
    const bool take = MIN ? ((ov < v) | ((ov == v) & (oi < idx))) : ((ov > v) | ((ov == v) & (oi < idx)));
    v = take ? ov : v;
    idx = take ? oi : idx;
}
template <bool MIN>
__device__ __forceinline__ void wave_arg(double &v, int &idx) {
    arg_step<kDppXor1, MIN>(v, idx);
    arg_step<kDppXor2, MIN>(v, idx);
    arg_step<kDppHalfMirror, MIN>(v, idx);
    arg_step<kDppMirror, MIN>(v, idx);
    double bv = readlane(v, 0);
    int bi = readlane(idx, 0);
#pragma unroll
    for (int r = 16; r < kWave; r += 16) {
        const double ov = readlane(v, r);
        const int oi = readlane(idx, r);
        const bool take = MIN ? (ov < bv || (ov == bv && oi < bi)) : (ov > bv || (ov == bv && oi < bi));
        bv = take ? ov : bv;
        bi = take ? oi : bi;
    }
    v = bv;
    idx = bi;
}
// lexicographic (value, index) minimum; lanes with nothing to offer pass (+inf, INT_MAX)
__device__ __forceinline__ void wave_argmin(double &v, int &idx) { wave_arg<true>(v, idx); }
// (value, index) maximum with the lowest index winning ties (Eigen maxCoeff semantics)
__device__ __forceinline__ void wave_argmax(double &v, int &idx) { wave_arg<false>(v, idx); }

// Ordering point between phases of a single-wave workgroup.  One wave issues its LDS
// instructions in program order and the LDS executes them in order, so a store by one lane
// is seen by a later load of another lane without any wait; only the compiler must not move
// LDS accesses across this point (wavefront-scope fences emit no instruction).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Code-motion fence for unrolled straight-line phases: no memory access moves across it at
// the IR level (empty asm with a memory clobber) nor in the machine scheduler.
__device__ __forceinline__ void step_fence() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// 1/sqrt(a) for a > 0: v_rsq_f64 plus MPCQP_RSQ_NR Newton steps -- a short dependency chain
// compared with the correctly rounded sqrt and divide sequences.  v_rsq_f64 is good to about
// 2^-23 relative; each step squares the error: one step (the default) gives about 2^-46 (tens of
// ulp, ~1e-14 relative) in every Cholesky pivot scale, two steps ~1 ulp.  The factor is then
// L (1 + e) column-wise with |e| ~ 1e-14 and J its exact inverse, so H^-1 = J J' carries ~1e-14
// relative error: four orders below the parity tolerance (1e-8 max(1, |U|)); the ill-conditioned
// parity case tests/test_gpu_parity.py::test_pair_kernel_ill_conditioned_vs_oracle guards it.
#ifndef MPCQP_RSQ_NR
// Newton steps after v_rsq_f64 (its estimate is good to about half the mantissa; one step squares
// the error): 1 since r04 -- parity suite unchanged, B 315 -> 311 us, L 2.38 -> 2.34 ms,
// C / E -0.5..0.8 % (alternating A/B); A/B builds: 2
#define MPCQP_RSQ_NR 1
#endif
__device__ __forceinline__ double rsqrt_nr(double a) {
    double y = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a;
#pragma unroll
    for (int i = 0; i < MPCQP_RSQ_NR; ++i) y = y * fma(-h * y, y, 1.5);
    return y;
}

// a / b for the dual loops' step lengths, reflector and rotation scalings: the IEEE division
// (~12 VALU: v_div_scale x2, v_rcp, five FMAs, v_div_fmas, v_div_fixup) or, with
// MPCQP_FAST_DIV, a * (1 / b) from v_rcp_f64 and two Newton steps (5 VALU; within ~2 ulp; every
// divisor there is positive and normal)
#ifndef MPCQP_FAST_DIV
#define MPCQP_FAST_DIV 0
#endif
__device__ __forceinline__ double fdiv(double a, double b) {
    if constexpr (MPCQP_FAST_DIV) {
        double y = __builtin_amdgcn_rcp(b);
        y = fma(y, fma(-b, y, 1.0), y);
        y = fma(y, fma(-b, y, 1.0), y);
        return a * y;
    } else {
        return a / b;
    }
}

// Materialise v in a VGPR at this point: arithmetic producing v cannot sink past it.
__device__ __forceinline__ void pin(double &v) { asm volatile("" : "+v"(v)); }

// Per-instance inputs and outputs are touched once: stream them past L2 (non-temporal) so they
// do not evict the scratch lines of the waves' spilled registers, which otherwise leave L2 as
// write-backs (MPCQP_STREAM=0: ordinary loads; MPCQP_STREAM_LD / _ST pick each side)
#ifndef MPCQP_STREAM
#define MPCQP_STREAM 1
#endif
#ifndef MPCQP_STREAM_LD
#define MPCQP_STREAM_LD MPCQP_STREAM
#endif
// Stores are ordinary (r04): with the XCD-aware instance order (xcd_order) neighbouring
// instances' partial output lines meet in one XCD's L2 and leave it merged -- writes at config
// B 47.3 -> 35.1 MB per launch (32.8 MB of U / cost / status / iterations), C 85.9 -> 66.1 MB
// (64.0), time unchanged; non-temporal stores leave every partial line as its own HBM write
#ifndef MPCQP_STREAM_ST
#define MPCQP_STREAM_ST 0
#endif
template <typename T>
__device__ __forceinline__ T stream_load(const T *p) {
#if MPCQP_STREAM_LD
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
template <typename T>
__device__ __forceinline__ void stream_store(T *p, T v) {
#if MPCQP_STREAM_ST
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// Diagnostic phase stamps (built only with -DMPCQP_STAMPS, lib/libmpcqp_stamps.so): cycles
// (s_memtime) since the previous stamp are added to slot k of a global array.  The real
// library compiles these to nothing.
#ifdef MPCQP_STAMPS
#define MPCQP_STAMP(ptr, k, t)                                                  \
    do {                                                                        \
        if (ptr) {                                                              \
            const unsigned long long now_ = __builtin_amdgcn_s_memtime();      \
            if (::mpcqp::lane() == 0) atomicAdd(&(ptr)[(k)], now_ - (t));      \
            (t) = now_;                                                         \
        }                                                                       \
    } while (0)
#define MPCQP_STAMP_INIT(t) unsigned long long t = __builtin_amdgcn_s_memtime()
// sub-phases inside a loop: cycles accumulate in registers (no atomic per pass) and go to
// slots 12..15 once, after the loop (MPCQP_SUB_OFF leaves 12..15 to the expm's sub-stamps)
#ifdef MPCQP_SUB_OFF
#define MPCQP_SUB_INIT(t) ((void)0)
#define MPCQP_SUB(t, k) ((void)0)
#define MPCQP_SUB_FLUSH(ptr, t) ((void)0)
#else
#define MPCQP_SUB_INIT(t) \
    unsigned long long t = __builtin_amdgcn_s_memtime(), t##_a0 = 0, t##_a1 = 0, t##_a2 = 0, t##_a3 = 0
#define MPCQP_SUB(t, k)                                                         \
    do {                                                                        \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();          \
        t##_a##k += now_ - (t);                                                 \
        (t) = now_;                                                             \
    } while (0)
#define MPCQP_SUB_FLUSH(ptr, t)                                                 \
    do {                                                                        \
        if ((ptr) && ::mpcqp::lane() == 0) {                                    \
            atomicAdd(&(ptr)[12], t##_a0); atomicAdd(&(ptr)[13], t##_a1);      \
            atomicAdd(&(ptr)[14], t##_a2); atomicAdd(&(ptr)[15], t##_a3);      \
        }                                                                       \
    } while (0)
#endif
#else
#define MPCQP_STAMP(ptr, k, t) ((void)0)
#define MPCQP_STAMP_INIT(t) ((void)0)
#define MPCQP_SUB_INIT(t) ((void)0)
#define MPCQP_SUB(t, k) ((void)0)
#define MPCQP_SUB_FLUSH(ptr, t) ((void)0)
#endif

// Diagnostic phase cuts (built only with -DMPCQP_CUTS, lib/libmpcqp_cuts.so): the kernel
// returns after phase k when the launch's cut value is k, so timing successive cuts gives
// each phase's cost at full occupancy (tools/phase_cuts.py).
#ifdef MPCQP_CUTS
#define MPCQP_CUT(cutv, k) \
    do {                   \
        if ((cutv) == (k)) return; \
    } while (0)
#elif defined(MPCQP_MARKS)
#define MPCQP_CUT(cutv, k) asm volatile(";@@CUT " #k)
#else
#define MPCQP_CUT(cutv, k) ((void)0)
#endif

}  // namespace mpcqp
