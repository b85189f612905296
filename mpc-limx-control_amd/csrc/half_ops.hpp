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

// (even row, odd row) of this half for a row-uniform value
__device__ __forceinline__ void row_pair(double v, double &even, double &odd) {
    const long long b = d2ll(v);
    const int lo = (int)(b & 0xffffffffll), hi = (int)(b >> 32);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
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
    row_pair(r, e, o);
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
