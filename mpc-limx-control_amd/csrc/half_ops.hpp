// half_ops.hpp -- half-wavefront primitives for the two-instances-per-wave kernel
// (mpc_pair.hpp): lanes 0-31 and 32-63 each run one instance.
//
// A half is two whole 16-lane DPP rows (rows 0-1 and rows 2-3), so
//   * row-local DPP steps (wave_ops.hpp) never mix halves;
//   * the cross-row step inside a half is gfx950's v_permlane16_swap: with both operands the
//     same value, the first result holds the even row's value and the second the odd row's,
//     in every lane of the half -- no SGPR round trip, no per-half select;
//   * a broadcast of lane k of each half is DPP row_newbcast (lane k & 15 of every row) then
//     the same swap, taking the even or odd row.
// All of these only read lanes of the caller's own half, so they also work inside a branch
// that one half takes and the other does not.  The v_readlane forms (hread_rt, hread_k) read
// the other half too and select; they ignore EXEC, which is equally safe.
#pragma once
#include "wave_ops.hpp"

namespace mpcqp {

constexpr int kHalf = 32;
__device__ __forceinline__ bool upper_half() { return lane() >= kHalf; }

__device__ __forceinline__ long long d2ll(double v) { return __double_as_longlong(v); }
__device__ __forceinline__ double ll2d(int lo, int hi) {
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Lane masks known at compile time: selects by an SGPR constant (s_mov_b64, scalar) instead of
// a per-lane v_cmp of the lane index on the VALU.  hmask<K>: lane K of each half.
template <int K>
__device__ __forceinline__ constexpr unsigned long long hmask() {
    return (1ull << K) | (1ull << (K + kHalf));
}
// lanes lo..hi (inclusive) of each half
template <int LO, int HI>
__device__ __forceinline__ constexpr unsigned long long hrange() {
    constexpr unsigned long long h = LO > HI ? 0ull : ((~0ull >> (63 - HI)) & ~((1ull << LO) - 1ull));
    return h | (h << kHalf);
}
// the same for indices that are constants after unrolling (the shifts fold)
__device__ __forceinline__ unsigned long long hmask_k(int k) {
    return (1ull << k) | (1ull << (k + kHalf));
}
__device__ __forceinline__ unsigned long long hrange_k(int lo, int hi) {
    const unsigned long long h = lo > hi ? 0ull : ((~0ull >> (63 - hi)) & ~((1ull << lo) - 1ull));
    return h | (h << kHalf);
}
// m ? 0.0 : v, lane by lane
__device__ __forceinline__ double zero_if(double v, unsigned long long m) {
    const long long b = d2ll(v);
    const int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    int rl, rh;  // (separate outputs: the input stays where it is, no copy)
    asm("v_cndmask_b32_e64 %0, %1, 0, %2" : "=v"(rl) : "v"(lo), "s"(m));
    asm("v_cndmask_b32_e64 %0, %1, 0, %2" : "=v"(rh) : "v"(hi), "s"(m));
    return ll2d(rl, rh);
}
// m ? -v : v, lane by lane (the sign bit of the high word flipped by the select's own source
// modifier: one instruction)
__device__ __forceinline__ double neg_if(double v, unsigned long long m) {
    const long long b = d2ll(v);
    const int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    int rh;
    asm("v_cndmask_b32_e64 %0, %1, -%1, %2" : "=v"(rh) : "v"(hi), "s"(m));
    return ll2d(lo, rh);
}

// one v_mov_b64 (the compiler copies a double it must keep as two v_mov_b32)
__device__ __forceinline__ double copy64(double v) {
    double r;
    asm("v_mov_b64 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
// (even row, odd row) of this half for a row-uniform value.  The swap overwrites both of its
// operands, so v (still live) is copied twice, 64 bits at a time.
__device__ __forceinline__ void row_pair(double v, double &even, double &odd) {
    const long long b1 = d2ll(copy64(v)), b2 = d2ll(copy64(v));
    const auto l = __builtin_amdgcn_permlane16_swap((int)(b1 & 0xffffffffll), (int)(b2 & 0xffffffffll),
                                                     false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((int)(b1 >> 32), (int)(b2 >> 32), false, false);
    even = ll2d(l[0], h[0]);
    odd = ll2d(l[1], h[1]);
}
// the same for a value that dies here: one copy, the swap takes v's own registers
__device__ __forceinline__ void row_pair_dead(double v, double &even, double &odd) {
    const long long b1 = d2ll(copy64(v)), b2 = d2ll(v);
    const auto l = __builtin_amdgcn_permlane16_swap((int)(b1 & 0xffffffffll), (int)(b2 & 0xffffffffll),
                                                     false, false);
    const auto h = __builtin_amdgcn_permlane16_swap((int)(b1 >> 32), (int)(b2 >> 32), false, false);
    even = ll2d(l[0], h[0]);
    odd = ll2d(l[1], h[1]);
}
__device__ __forceinline__ void row_pair(int v, int &even, int &odd) {
    const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    even = p[0];
    odd = p[1];
}

// lane (half base + K) of each half, K a compile-time constant
template <int K>
__device__ __forceinline__ double hbcast(double v) {
    static_assert(K >= 0 && K < kHalf, "lane within a half");
    const double r = dpp<0x150 + (K & 15)>(v);  // row_newbcast
    double e, o;
    row_pair_dead(r, e, o);
    return K < 16 ? e : o;
}
// the same for an index that is constant after unrolling (the switch folds)
__device__ __forceinline__ double hbcast(double v, int k) {
    switch (k) {
#define MPCQP_HB(i) case i: return hbcast<i>(v);
        MPCQP_HB(0) MPCQP_HB(1) MPCQP_HB(2) MPCQP_HB(3) MPCQP_HB(4) MPCQP_HB(5) MPCQP_HB(6)
        MPCQP_HB(7) MPCQP_HB(8) MPCQP_HB(9) MPCQP_HB(10) MPCQP_HB(11) MPCQP_HB(12) MPCQP_HB(13)
        MPCQP_HB(14) MPCQP_HB(15) MPCQP_HB(16) MPCQP_HB(17) MPCQP_HB(18) MPCQP_HB(19)
        MPCQP_HB(20) MPCQP_HB(21) MPCQP_HB(22) MPCQP_HB(23) MPCQP_HB(24) MPCQP_HB(25)
        MPCQP_HB(26) MPCQP_HB(27) MPCQP_HB(28) MPCQP_HB(29) MPCQP_HB(30) MPCQP_HB(31)
#undef MPCQP_HB
        default: return 0.0;
    }
}

// lane (half base + k) of each half, k wave-uniform at run time (v_readlane of both halves)
__device__ __forceinline__ double hread_rt(double v, int k) {
    const double lo = readlane(v, k), hi = readlane(v, k + kHalf);
    return upper_half() ? hi : lo;
}
// lane (half base + k) where k is uniform within each half (possibly different per half)
__device__ __forceinline__ double hread_k(double v, int k) {
    const int k0 = __builtin_amdgcn_readlane(k, 0) & (kHalf - 1);
    const int k1 = __builtin_amdgcn_readlane(k, kHalf) & (kHalf - 1);
    const double lo = readlane(v, k0), hi = readlane(v, k1 + kHalf);
    return upper_half() ? hi : lo;
}
__device__ __forceinline__ int hread_k(int v, int k) {
    const int k0 = __builtin_amdgcn_readlane(k, 0) & (kHalf - 1);
    const int k1 = __builtin_amdgcn_readlane(k, kHalf) & (kHalf - 1);
    const int lo = readlane(v, k0), hi = readlane(v, k1 + kHalf);
    return upper_half() ? hi : lo;
}
// per-half ballot (bit i = lane base + i of this half)
__device__ __forceinline__ uint32_t half_ballot(bool p) {
    const uint64_t m = __ballot(p);
    return upper_half() ? (uint32_t)(m >> 32) : (uint32_t)m;
}

// ---- reductions: DPP inside each row, then the half's two rows (even + odd, the same order
//      in every lane, so the result is bit-identical across the half)
__device__ __forceinline__ double row_sum(double v) {
    v += dpp<kDppXor1>(v);
    v += dpp<kDppXor2>(v);
    v += dpp<kDppHalfMirror>(v);
    v += dpp<kDppMirror>(v);
    return v;
}
__device__ __forceinline__ double half_sum(double v) {
    double e, o;
    row_pair(row_sum(v), e, o);
    return e + o;
}
__device__ __forceinline__ void half_sum3(double &a, double &b, double &c) {
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
    double e, o;
    row_pair(a, e, o);
    a = e + o;
    row_pair(b, e, o);
    b = e + o;
    row_pair(c, e, o);
    c = e + o;
}
__device__ __forceinline__ double half_max(double v) {
    v = fmax(v, dpp<kDppXor1>(v));
    v = fmax(v, dpp<kDppXor2>(v));
    v = fmax(v, dpp<kDppHalfMirror>(v));
    v = fmax(v, dpp<kDppMirror>(v));
    double e, o;
    row_pair(v, e, o);
    return fmax(e, o);
}
// minimum within each half (compare / select: no canonicalising v_min_f64 under IEEE mode)
__device__ __forceinline__ double half_min(double v) {
    double o = dpp<kDppXor1>(v);
    v = o < v ? o : v;
    o = dpp<kDppXor2>(v);
    v = o < v ? o : v;
    o = dpp<kDppHalfMirror>(v);
    v = o < v ? o : v;
    o = dpp<kDppMirror>(v);
    v = o < v ? o : v;
    double e, od;
    row_pair(v, e, od);
    return od < e ? od : e;
}
// two sums in one pass (the DPP chains interleave)
__device__ __forceinline__ void half_sum2(double &a, double &b) {
    a += dpp<kDppXor1>(a);
    b += dpp<kDppXor1>(b);
    a += dpp<kDppXor2>(a);
    b += dpp<kDppXor2>(b);
    a += dpp<kDppHalfMirror>(a);
    b += dpp<kDppHalfMirror>(b);
    a += dpp<kDppMirror>(a);
    b += dpp<kDppMirror>(b);
    double e, o;
    row_pair(a, e, o);
    a = e + o;
    row_pair(b, e, o);
    b = e + o;
}
// (value, lane) minimum within each half, lowest lane on ties: the minimum by compare/select,
// then one ballot of the lanes holding it (no index carried through the DPP steps).  A half
// whose values are all +inf gets lane 0x7fffffff.
__device__ __forceinline__ int half_argmin_lane(double &v) {
    const double m = half_min(v);
    const uint32_t hit = half_ballot(v == m);
    v = m;
    return m == INFINITY ? 0x7fffffff : (int)__builtin_ctz(hit);
}
// lexicographic (value, index) minimum within each half
__device__ __forceinline__ void half_argmin(double &v, int &idx) {
    arg_step<kDppXor1, true>(v, idx);
    arg_step<kDppXor2, true>(v, idx);
    arg_step<kDppHalfMirror, true>(v, idx);
    arg_step<kDppMirror, true>(v, idx);
    double ev, ov;
    int ei, oi;
    row_pair(v, ev, ov);
    row_pair(idx, ei, oi);
    const bool take = (ov < ev) | ((ov == ev) & (oi < ei));
    v = take ? ov : ev;
    idx = take ? oi : ei;
}

}  // namespace mpcqp
