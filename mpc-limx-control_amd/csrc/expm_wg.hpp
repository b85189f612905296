// expm_wg.hpp -- wave_expm (condense.hpp: Eigen's Pade degree selection and scaling and
// squaring of exp([[A, B], [0, 0]] Ts), QPSolver::discretizeSystem, src/QPSolver.cpp:21-29) run by
// a whole workgroup: the (top block, scalar) algebra products go to the FP64 matrix cores as
// 16 x 16 output tiles spread over the waves, the linear combinations over every thread; the
// Pade quotient's partial-pivot LU stays on one wave (expm_pade_solve).  Same operations and
// branch thresholds as wave_expm; products differ from it only in summation order.
#pragma once
#include "condense.hpp"
#include "mfma_ops.hpp"

namespace mpcqp {

// out = X * Y in the top-block algebra (alg_mul): out[:, j] = X1 Y[:, j] (+ sY X[:, j], j >= nx)
__device__ __forceinline__ void wg_alg_mul(int nx, int ns, const double *X, const double *Y,
                                           double sY, double *out, int wv, int nw) {
    const int tm_n = (nx + 15) >> 4, tn_n = (ns + 15) >> 4, ks = (nx + 3) >> 2;
    const int ln = lane(), li = ln & 15, lk = ln >> 4;
    for (int t = wv; t < tm_n * tn_n; t += nw) {
        const int tm = t % tm_n, tn = t / tm_n;
        const int i = tm * 16 + li, j = tn * 16 + li;
        dx4 acc = {0.0, 0.0, 0.0, 0.0};
        if (ks <= 8) {  // as mfma_gemm: operands first (clamped loads + selects), then the chain
            double av[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int kk = 4 * s + lk;
                const bool oka = s < ks && i < nx && kk < nx, okb = s < ks && j < ns && kk < nx;
                const double a = X[oka ? kk * nx + i : 0];
                const double b = Y[okb ? j * nx + kk : 0];
                av[s] = oka ? a : 0.0;
                bv[s] = okb ? b : 0.0;
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
        } else {
            for (int s = 0; s < ks; ++s) {
                const int kk = 4 * s + lk;
                const bool kin = kk < nx;
                const double a = (i < nx && kin) ? X[kk * nx + i] : 0.0;
                const double b = (j < ns && kin) ? Y[j * nx + kk] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = tm * 16 + lk + 4 * r, col = tn * 16 + li;
            if (row < nx && col < ns) {
                double v = acc[r];
                if (col >= nx) v += sY * X[col * nx + row];
                out[col * nx + row] = v;
            }
        }
    }
    __syncthreads();
}

// Two products in one pass (8 tiles over the waves, one barrier), each with its right operand a
// linear combination and a combination added to its result (degree 13's W and V, which depend
// only on A2, A4, A6):  out_p = X (sum_q cb_p[q] Mb_p[q]) + (sum_q ce_p[q] Me_p[q] + ceI_p I),
// the right operands' scalar parts 0.  Every sum in alg_comb's order, so the values are those
// of the comb / mul / add stages it replaces (five barriers fewer).
template <int K>
struct AlgComb {
    double c[K];
    const double *M[K];
    __device__ __forceinline__ double at(int e) const {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) s += c[q] * M[q][e];
        return s;
    }
};
template <int KB, int KE>
__device__ __forceinline__ void wg_alg_mul_comb2(int nx, int ns, const double *X,
                                                 const AlgComb<KB> (&cb)[2], const AlgComb<KE> (&ce)[2],
                                                 const double (&ceI)[2], double *const (&out)[2],
                                                 int wv, int nw) {
    const int tm_n = (nx + 15) >> 4, tn_n = (ns + 15) >> 4, ks = (nx + 3) >> 2, nt1 = tm_n * tn_n;
    const int ln = lane(), li = ln & 15, lk = ln >> 4;
    for (int t = wv; t < 2 * nt1; t += nw) {
        const int pr = t < nt1 ? 0 : 1, tt = t < nt1 ? t : t - nt1;
        const int tm = tt % tm_n, tn = tt / tm_n;
        const int i = tm * 16 + li, j = tn * 16 + li;
        dx4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int s = 0; s < ks; ++s) {
            const int kk = 4 * s + lk;
            const bool oka = i < nx && kk < nx, okb = j < ns && kk < nx;
            const double a = X[oka ? kk * nx + i : 0];
            double b = cb[pr].at(okb ? j * nx + kk : 0);
            if (okb && kk == j) b += 0.0;  // (alg_comb's identity term, cI = 0)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(oka ? a : 0.0, okb ? b : 0.0, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = tm * 16 + lk + 4 * r, col = tn * 16 + li;
            if (row < nx && col < ns) {
                const int e = col * nx + row;
                double w = ce[pr].at(e);
                if (row == col) w += ceI[pr];
                out[pr][e] = acc[r] + w;
            }
        }
    }
    __syncthreads();
}

// out = sum_q c[q] M[q] + cI I (alg_comb) over every thread
template <int K>
__device__ __forceinline__ void wg_alg_comb(int nx, int ns, double *out, const double (&c)[K],
                                            const double *const (&M)[K], double cI, int tid,
                                            int nt) {
    for (int e = tid; e < nx * ns; e += nt) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) s += c[q] * M[q][e];
        const int i = e % nx, j = e / nx;
        if (i == j) s += cI;
        out[e] = s;
    }
    __syncthreads();
}

// The Pade quotient (expm_pade_solve, condense.hpp) by the workgroup: denom X = numer by
// Gauss-Jordan elimination with expm_pade_solve's partial pivoting (pivot = largest |D(i, k)|,
// lowest row on ties; l_i = D(i, k) / piv; row -= l_i pivot row), applied to every row but the
// pivot's, so no back substitution (a latency chain of ~nx^2 / 2 dependent LDS reads and FMAs on
// one wave) remains: X(i, :) = row i / D(i, i).  Same pivots as the LU; X differs from its
// back substitution by rounding only.  Thread (wave w, lane j) holds column j of [D | numer'],
// rows w, w + nw, .. in registers.  Per step: the pivot candidates of column k (lane k of each
// wave) meet in LDS | barrier | rows k, p and column k are published | barrier | swap +
// elimination in registers; buffers alternate between steps, so two barriers per column.
// Needs nx <= MR nw (MR <= 8), nx + ns <= 64, and 352 doubles of scratch.
template <int MR>  // row slots per thread: nx <= MR nw
__device__ __forceinline__ void wg_pade_solve(int nx, int ns, const double *U, const double *V,
                                              double *E, double *scr, int wv, int nw) {
    const int j = lane(), ncol = nx + ns;
    const bool colok = j < ncol;
    double *redv = scr, *redi = scr + 16, *rowP = scr + 32, *rowK = scr + 160, *colK = scr + 288;
    double a[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        const int i = wv + nw * r;
        double v = 0.0;
        if (colok && i < nx) {
            const int c = j < nx ? j : j - nx;
            const int e = c * nx + i;
            const double n = U[e] + V[e], d = -U[e] + V[e];
            v = (j < nx) ? d : ((e / nx >= nx) ? n - d : n);
        }
        a[r] = v;
    }
    for (int k = 0; k < nx; ++k) {
        const int b = k & 1;
        if (j == k) {
            double best = -1.0;
            int bi = 0x7fffffff;
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int i = wv + nw * r;
                if (i >= k && i < nx) {
                    const double v = fabs(a[r]);
                    if (v > best) { best = v; bi = i; }  // rows ascend: ties keep the lowest
                }
            }
            redv[8 * b + wv] = best;
            redi[8 * b + wv] = (double)bi;
        }
        __syncthreads();
        double pv = redv[8 * b];
        int p = (int)redi[8 * b];
        for (int w = 1; w < nw; ++w) {
            const double ov = redv[8 * b + w];
            const int oi = (int)redi[8 * b + w];
            if (ov > pv || (ov == pv && oi < p)) { pv = ov; p = oi; }
        }
        const int wp = p % nw, sp = p / nw, wk = k % nw, sk = k / nw;
        if (colok) {
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                if (wv == wp && r == sp) rowP[64 * b + j] = a[r];
                if (wv == wk && r == sk) rowK[64 * b + j] = a[r];
            }
        }
        if (j == k) {
#pragma unroll
            for (int r = 0; r < MR; ++r) {
                const int i = wv + nw * r;
                if (i < nx) colK[32 * b + i] = a[r];
            }
        }
        __syncthreads();
        const double pk = colok ? rowP[64 * b + j] : 0.0;  // the pivot row after the swap
        const double piv = rowP[64 * b + k];
        const double ck = colK[32 * b + k], rk = colok ? rowK[64 * b + j] : 0.0;
        const double rp = 1.0 / piv;  // one division per step; multipliers l_i = D(i, k) / piv
#pragma unroll
        for (int r = 0; r < MR; ++r) {  // branch-free: selects instead of EXEC-masked slots
            const int i = wv + nw * r;
            const double ci = (i == p) ? ck : colK[32 * b + (i < nx ? i : 0)];
            double v = (i == k) ? pk : ((i == p) ? rk : a[r]);
            const bool upd = i != k && i < nx && j > k && colok;
            a[r] = upd ? v - (ci * rp) * pk : v;
        }
    }
    // X(i, c) = row i / D(i, i); D(i, i) sits on lane i of the same wave
#pragma unroll
    for (int r = 0; r < MR; ++r) {
        const int i = wv + nw * r;
        if (i < nx) {
            const double dii = readlane(a[r], i);
            if (colok && j >= nx) E[(j - nx) * nx + i] = a[r] / dii;
        }
    }
}

// The same Gauss-Jordan elimination (same pivots, lowest row on ties, same multipliers
// l_i = D(i, k) / piv and updates) on ONE wavefront with the nx rows of every column in
// registers (lane j = column j of [D | numer'], nx compile-time): the column-k entries reach all
// lanes by v_readlane, the pivot row is chosen by lane k from its own registers and swapped by
// selects -- no LDS and no barrier per column (the workgroup form above spent two barriers
// and three LDS round trips per column: 426 k wave-cycles per QP at config E, a quarter of the
// kernel).  MPCQP_PADE_WAVE=0 keeps the workgroup form (A/B builds).
#ifndef MPCQP_PADE_WAVE
#define MPCQP_PADE_WAVE 1
#endif
// MPCQP_PADE_LDS: column k reaches the lanes through LDS (lane k writes it, every lane reads it
// back at uniform addresses: 2 NXC / 2 b128 instructions) instead of 2 NXC v_readlane.
// Measured slower (E 6.39 vs 6.31 ms at 16,384, alternating A/B): off
#ifndef MPCQP_PADE_LDS
#define MPCQP_PADE_LDS 0
#endif
// MPCQP_PADE_NOSEL: every lane applies the step's update (no select keeping columns j <= k):
// the columns left of k are never read again (their entries are garbage afterwards), and each
// lane keeps its own pivot D(j, j) in a register from its step on.  The numerator columns
// (j >= nx > k) get exactly the same operations, so E is bit-identical.
// MPCQP_PADE_LATE: column k is read row by row in the update (after the swap) instead of 2 NXC
// v_readlane up front, whose 48 SGPR results per step the compiler hoisted together (A/B)
#ifndef MPCQP_PADE_LATE
#define MPCQP_PADE_LATE 1
#endif
#ifndef MPCQP_PADE_NOSEL
#define MPCQP_PADE_NOSEL 1
#endif
template <int NXC>
__device__ __forceinline__ void wave_pade_gj(int ns, const double *U, const double *V, double *E,
                                             double *scr) {
    static_assert(NXC <= 32, "pivot cases below");
    constexpr int nx = NXC;
    const int j = lane(), ncol = nx + ns;
    const bool colok = j < ncol;
    double a[NXC];
#pragma unroll
    for (int i = 0; i < NXC; ++i) {
        double v = 0.0;
        if (colok) {
            const int c = j < nx ? j : j - nx;
            const int e = c * nx + i;
            const double n = U[e] + V[e], d = -U[e] + V[e];
            v = (j < nx) ? d : ((e / nx >= nx) ? n - d : n);
        }
        a[i] = v;
    }
    double piv_own = 0.0;  // (MPCQP_PADE_NOSEL) lane j's pivot D(j, j), from step j on
#pragma unroll
    for (int k = 0; k < NXC; ++k) {
        // pivot: lane k's largest |a(i)|, i >= k, by a pairwise tree in which the lower row
        // wins ties (the linear scan's rule: rows ascend, ties keep the lowest)
        double tv[NXC];
        int ti[NXC];
#pragma unroll
        for (int i = k; i < NXC; ++i) { tv[i - k] = fabs(a[i]); ti[i - k] = i; }
#pragma unroll
        for (int w = 1; w < NXC - k; w *= 2) {
#pragma unroll
            for (int i = 0; i + w < NXC - k; i += 2 * w) {
                const bool t = tv[i + w] > tv[i];
                tv[i] = t ? tv[i + w] : tv[i];
                ti[i] = t ? ti[i + w] : ti[i];
            }
        }
        const int p = __builtin_amdgcn_readlane(ti[0], k);
        double ck[NXC];  // column k before the swap, every lane
        if (MPCQP_PADE_LATE) {
            // (each row's column-k entry is read in the update loop below, after the swap)
#pragma unroll
            for (int i = 0; i < NXC; ++i) ck[i] = 0.0;
        } else if (MPCQP_PADE_LDS) {
            if (j == k) {
#pragma unroll
                for (int i = 0; i < NXC; ++i) scr[i] = a[i];
            }
            wave_sync();
#pragma unroll
            for (int i = 0; i < NXC; ++i) ck[i] = scr[i];
            wave_sync();  // (the next column's writes after these reads)
        } else {
#pragma unroll
            for (int i = 0; i < NXC; ++i) ck[i] = readlane(a[i], k);
        }
        // rows k and p swap (p >= k, uniform: a scalar branch, no select chain; an if-chain of
        // uniform compares measured 2.5 % slower at E, tools/r05_t.sh)
        double pk = a[k], ckk = ck[k];
        const double rk = a[k];
        switch (p) {
#define MPCQP_PSW(i)                                          \
    case i:                                                   \
        if (i > k && i < NXC) {                               \
            pk = a[i < NXC ? i : 0];                          \
            ckk = ck[i < NXC ? i : 0];                        \
            a[i < NXC ? i : 0] = rk;                          \
        }                                                     \
        break;
            MPCQP_PSW(1) MPCQP_PSW(2) MPCQP_PSW(3) MPCQP_PSW(4) MPCQP_PSW(5) MPCQP_PSW(6)
            MPCQP_PSW(7) MPCQP_PSW(8) MPCQP_PSW(9) MPCQP_PSW(10) MPCQP_PSW(11) MPCQP_PSW(12)
            MPCQP_PSW(13) MPCQP_PSW(14) MPCQP_PSW(15) MPCQP_PSW(16) MPCQP_PSW(17) MPCQP_PSW(18)
            MPCQP_PSW(19) MPCQP_PSW(20) MPCQP_PSW(21) MPCQP_PSW(22) MPCQP_PSW(23) MPCQP_PSW(24)
            MPCQP_PSW(25) MPCQP_PSW(26) MPCQP_PSW(27) MPCQP_PSW(28) MPCQP_PSW(29) MPCQP_PSW(30)
            MPCQP_PSW(31)
#undef MPCQP_PSW
            default: break;
        }
        a[k] = pk;  // ckk = piv
        if (MPCQP_PADE_LATE) ckk = readlane(pk, k);  // D(p, k)
        if (MPCQP_PADE_NOSEL) piv_own = (j == k) ? pk : piv_own;
        const double rp = 1.0 / ckk;
#pragma unroll
        for (int i = 0; i < NXC; ++i) {
            if (i == k) continue;
            // row i's column-k entry after the swap (MPCQP_PADE_LATE: read from the row itself,
            // which the swap already placed; one short SGPR live range per row)
            const double ci = MPCQP_PADE_LATE ? readlane(a[i], k) : (i > k && p == i) ? ck[k] : ck[i];
            if (MPCQP_PADE_NOSEL) {
                a[i] = a[i] - (ci * rp) * pk;
            } else {
                const bool upd = j > k && colok;
                a[i] = upd ? a[i] - (ci * rp) * pk : a[i];
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NXC; ++i) {
        const double dii = MPCQP_PADE_NOSEL ? readlane(piv_own, i) : readlane(a[i], i);
        if (colok && j >= nx) E[(j - nx) * nx + i] = a[i] / dii;
    }
}

// 1: degree 13's two independent products fused with their combinations (wg_alg_mul_comb2):
// five barriers fewer, but the fused operands' three loads per element stretch the products'
// chains; measured slower (E 6.37 vs 6.31 ms at 16,384, alternating A/B): off
#ifndef MPCQP_EXPM_FUSE
#define MPCQP_EXPM_FUSE 0
#endif

struct NoSide {
    __device__ void operator()() const {}
};
// wave_expm by the workgroup (nt threads, nw waves).  T (nx x ns, scaled by Ts) is overwritten
// when scaling; ws: 7 nx ns doubles; E: the result top block.  Every thread must call it.
// side: one wave's independent work (it must not touch T, ws or E), run by the last wave while
// the first solves the Pade quotient alone (config E), else by the last wave after the solve.
template <class Side = NoSide>
__device__ __forceinline__ void wg_expm(int nx, int ns, double *T, double *ws, double *E, int tid,
                                        int nt, int wv, int nw,
                                        unsigned long long *stamps = nullptr,
                                        const Side &side = Side()) {
    MPCQP_STAMP_INIT(tx);
    const int sz = nx * ns;
    double *A2 = ws, *A4 = ws + sz, *A6 = ws + 2 * sz, *A8 = ws + 3 * sz, *U = ws + 4 * sz,
           *V = ws + 5 * sz, *W = ws + 6 * sz;
    double cs = 0.0;  // 1-norm, computed by every wave alike
    for (int j = lane(); j < ns; j += kWave) {
        double s = 0.0;
        for (int i = 0; i < nx; ++i) s += fabs(T[j * nx + i]);
        cs = fmax(cs, s);
    }
    const double l1 = wave_max(cs);
    int squarings = 0;
    if (l1 < 1.495585217958292e-002) {
        const double b[] = {120., 60., 12., 1.};
        wg_alg_mul(nx, ns, T, T, 0.0, A2, wv, nw);
        wg_alg_comb<1>(nx, ns, W, {b[3]}, {A2}, b[1], tid, nt);
        wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
        wg_alg_comb<1>(nx, ns, V, {b[2]}, {A2}, b[0], tid, nt);
    } else if (l1 < 2.539398330063230e-001) {
        const double b[] = {30240., 15120., 3360., 420., 30., 1.};
        wg_alg_mul(nx, ns, T, T, 0.0, A2, wv, nw);
        wg_alg_mul(nx, ns, A2, A2, 0.0, A4, wv, nw);
        wg_alg_comb<2>(nx, ns, W, {b[5], b[3]}, {A4, A2}, b[1], tid, nt);
        wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
        wg_alg_comb<2>(nx, ns, V, {b[4], b[2]}, {A4, A2}, b[0], tid, nt);
    } else if (l1 < 9.504178996162932e-001) {
        const double b[] = {17297280., 8648640., 1995840., 277200., 25200., 1512., 56., 1.};
        wg_alg_mul(nx, ns, T, T, 0.0, A2, wv, nw);
        wg_alg_mul(nx, ns, A2, A2, 0.0, A4, wv, nw);
        wg_alg_mul(nx, ns, A4, A2, 0.0, A6, wv, nw);
        wg_alg_comb<3>(nx, ns, W, {b[7], b[5], b[3]}, {A6, A4, A2}, b[1], tid, nt);
        wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
        wg_alg_comb<3>(nx, ns, V, {b[6], b[4], b[2]}, {A6, A4, A2}, b[0], tid, nt);
    } else if (l1 < 2.097847961257068e+000) {
        const double b[] = {17643225600., 8821612800., 2075673600., 302702400., 30270240.,
                            2162160.,     110880.,     3960.,       90.,        1.};
        wg_alg_mul(nx, ns, T, T, 0.0, A2, wv, nw);
        wg_alg_mul(nx, ns, A2, A2, 0.0, A4, wv, nw);
        wg_alg_mul(nx, ns, A4, A2, 0.0, A6, wv, nw);
        wg_alg_mul(nx, ns, A6, A2, 0.0, A8, wv, nw);
        wg_alg_comb<4>(nx, ns, W, {b[9], b[7], b[5], b[3]}, {A8, A6, A4, A2}, b[1], tid, nt);
        wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
        wg_alg_comb<4>(nx, ns, V, {b[8], b[6], b[4], b[2]}, {A8, A6, A4, A2}, b[0], tid, nt);
    } else {
        const double maxnorm = 5.371920351148152;
        frexp(l1 / maxnorm, &squarings);
        if (squarings < 0) squarings = 0;
        __syncthreads();  // every wave has read T for its norm
        for (int e = tid; e < sz; e += nt) T[e] = ldexp(T[e], -squarings);
        __syncthreads();
        const double b[] = {64764752532480000., 32382376266240000., 7771770303897600.,
                            1187353796428800.,  129060195264000.,   10559470521600.,
                            670442572800.,      33522128640.,       1323241920.,
                            40840800.,          960960.,            16380.,
                            182.,               1.};
        wg_alg_mul(nx, ns, T, T, 0.0, A2, wv, nw);
        wg_alg_mul(nx, ns, A2, A2, 0.0, A4, wv, nw);
        wg_alg_mul(nx, ns, A4, A2, 0.0, A6, wv, nw);
        if (MPCQP_EXPM_FUSE) {
            // W = A6 (b13 A6 + b11 A4 + b9 A2) + (b7 A6 + b5 A4 + b3 A2 + b1 I) and
            // V = A6 (b12 A6 + b10 A4 + b8 A2) + (b6 A6 + b4 A4 + b2 A2 + b0 I) in one pass
            const AlgComb<3> cb[2] = {{{b[13], b[11], b[9]}, {A6, A4, A2}},
                                      {{b[12], b[10], b[8]}, {A6, A4, A2}}};
            const AlgComb<3> ce[2] = {{{b[7], b[5], b[3]}, {A6, A4, A2}},
                                      {{b[6], b[4], b[2]}, {A6, A4, A2}}};
            const double ceI[2] = {b[1], b[0]};
            double *const outs[2] = {W, V};
            wg_alg_mul_comb2(nx, ns, A6, cb, ce, ceI, outs, wv, nw);
            wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
        } else {
            wg_alg_comb<3>(nx, ns, V, {b[13], b[11], b[9]}, {A6, A4, A2}, 0.0, tid, nt);
            wg_alg_mul(nx, ns, A6, V, 0.0, W, wv, nw);
            wg_alg_comb<3>(nx, ns, A8, {b[7], b[5], b[3]}, {A6, A4, A2}, b[1], tid, nt);
            for (int e = tid; e < sz; e += nt) W[e] += A8[e];
            __syncthreads();
            wg_alg_mul(nx, ns, T, W, b[1], U, wv, nw);
            wg_alg_comb<3>(nx, ns, W, {b[12], b[10], b[8]}, {A6, A4, A2}, 0.0, tid, nt);
            wg_alg_mul(nx, ns, A6, W, 0.0, V, wv, nw);
            wg_alg_comb<3>(nx, ns, A8, {b[6], b[4], b[2]}, {A6, A4, A2}, b[0], tid, nt);
            for (int e = tid; e < sz; e += nt) V[e] += A8[e];
            __syncthreads();
        }
    }
    MPCQP_STAMP(stamps, 12, tx);
    if (MPCQP_PADE_WAVE && nx == 24 && nx + ns <= kWave) {  // config E
#ifdef MPCQP_PADE_PROBE  // (stamps build only) wave 0's solve in slot 15, the side work in slot 0
        MPCQP_STAMP_INIT(tp);
        if (wv == 0) { wave_pade_gj<24>(ns, U, V, E, A2); MPCQP_STAMP(stamps, 15, tp); }
        else if (wv == nw - 1) { side(); MPCQP_STAMP(stamps, 0, tp); }
#else
        if (wv == 0) wave_pade_gj<24>(ns, U, V, E, A2);  // A2 .. W are dead here
        else if (wv == nw - 1) side();
#endif
    } else if (nx <= 6 * nw && nx + ns <= kWave && 4 * sz >= 352) {  // A2 .. W are dead here
        wg_pade_solve<6>(nx, ns, U, V, E, A2, wv, nw);         // config E: 24 rows, 4 waves
    } else if (nx <= 8 * nw && nx + ns <= kWave && 4 * sz >= 352) {
        wg_pade_solve<8>(nx, ns, U, V, E, A2, wv, nw);
    } else {
        if (wv == 0) expm_pade_solve(nx, ns, U, V, A2, E);
    }
    if (!(MPCQP_PADE_WAVE && nx == 24 && nx + ns <= kWave) && wv == nw - 1) side();
    __syncthreads();
    MPCQP_STAMP(stamps, 13, tx);
    for (int s = 0; s < squarings; ++s) {
        wg_alg_mul(nx, ns, E, E, 1.0, W, wv, nw);
        for (int e = tid; e < sz; e += nt) E[e] = W[e];
        __syncthreads();
    }
    MPCQP_STAMP(stamps, 14, tx);
    (void)stamps;
}

}  // namespace mpcqp
