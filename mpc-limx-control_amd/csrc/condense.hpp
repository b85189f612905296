// condense.hpp -- per-wavefront SRBM linearisation, exact ZOH discretisation and horizon
// condensing (HIP, gfx950).
//
// Reference path (Fleming-Sung/mpc-limX-control):
//   mpcQP::buildSystemModel           include/mpcQP.h:121-182   -> model_entry()
//   QPSolver::discretizeSystem        src/QPSolver.cpp:21-29    -> wave_discretize()
//   QPSolver::buildQPParams           src/QPSolver.cpp:31-81    -> wave_condense()
//
// Discretisation: the reference takes exp(M Ts) of M = [[Ac, Bc],[0, 0]] with Eigen's Pade /
// scaling-and-squaring.  Every matrix in that computation is block upper triangular with a
// zero-or-scalar*I bottom block, so here it is carried as (top nx x (nx+nu) block, scalar) --
// the same Pade degree, the same scaling, the same partial-pivot LU on the top-left block --
// at nx/(nx+nu) of the work and storage.
//
// Condensing: instead of the reference's dense 2 B'QB with a (nx(N+1))^2 block-diagonal Q,
// H(i,j) = 2 [sum_m Phi_{m-1-k_i}[:,c_i]' Q_m Phi_{m-1-k_j}[:,c_j] + R(c_i,c_j) d(k_i,k_j)]
// with Phi_a = Ad^a Bd (the block-Toeplitz structure of B_aug), and
// f(i) = 2 sum_{m>k_i} Phi_{m-1-k_i}[:,c_i]' Q_m (Ad^m x0 - xref_m).
#pragma once
#include "wave_ops.hpp"

namespace mpcqp {

struct ModelConst {
    int nx, nu, N, nV, ns;  // ns = nx + nu
    int model;              // 0 SRBM 13x6, 1 literal 13x3, 2 generic (Ac/Bc given)
    double Ts, mass;
    double Ibinv[9];        // body inertia inverse (column-major), host-computed
    const double *Q, *R, *P;
};

// ------------------------------------------------------------------ continuous-time model
// Entry (i, j) of [Ac | Bc] (nx x ns) for one instance.
__device__ __forceinline__ double srbm_entry(int i, int j, const double *lin, double cy,
                                             double sy, const double *Iwi, double mass) {
    // columns 0..12: Ac, 13..18: Bc.   state [rpy 0:3, p 3:6, w 6:9, v 9:12, g 12]
    if (j < 13) {
        if (i == 0) return j == 6 ? cy : (j == 7 ? sy : 0.0);
        if (i == 1) return j == 6 ? -sy : (j == 7 ? cy : 0.0);
        if (i == 2) return j == 8 ? 1.0 : 0.0;
        if (i >= 3 && i < 6) return j == i + 6 ? 1.0 : 0.0;
        if (i == 11) return j == 12 ? 1.0 : 0.0;
        return 0.0;
    }
    const int u = j - 13, ft = u / 3, c = u % 3;
    if (i >= 6 && i < 9) {  // Iw^-1 [r_ft]x, column c
        // selects instead of indexing, so a lane-varying i or j never forces the small
        // arrays into scratch
        const double f1 = ft ? 1.0 : 0.0, f0 = 1.0 - f1;
        const double r0 = f0 * lin[1] + f1 * lin[4], r1 = f0 * lin[2] + f1 * lin[5],
                     r2 = f0 * lin[3] + f1 * lin[6];
        // column c of [r]x
        double x0, x1, x2;
        if (c == 0) { x0 = 0.0; x1 = r2; x2 = -r1; }
        else if (c == 1) { x0 = -r2; x1 = 0.0; x2 = r0; }
        else { x0 = r1; x1 = -r0; x2 = 0.0; }
        // row ii of Iw^-1 by arithmetic blending: a select of two array loads would be folded
        // into one load with a lane-varying index, which keeps the array in scratch memory
        const int ii = i - 6;
        const double e0 = ii == 0 ? 1.0 : 0.0, e1 = ii == 1 ? 1.0 : 0.0, e2 = ii == 2 ? 1.0 : 0.0;
        const double w0 = e0 * Iwi[0] + e1 * Iwi[1] + e2 * Iwi[2];
        const double w1 = e0 * Iwi[3] + e1 * Iwi[4] + e2 * Iwi[5];
        const double w2 = e0 * Iwi[6] + e1 * Iwi[7] + e2 * Iwi[8];
        return w0 * x0 + w1 * x1 + w2 * x2;
    }
    if (i >= 9 && i < 12) return (i - 9 == c) ? 1.0 / mass : 0.0;
    return 0.0;
}

// sin and cos of x: Cody-Waite reduction by pi/2 in three parts (pio2_1 has 33 significant
// bits, so n pio2_1 and x - n pio2_1 are exact for |n| < 2^20) and fdlibm's __kernel_sin /
// __kernel_cos minimax polynomials on |r| <= pi/4 (< 1 ulp, as libm).  ~40 VALU instead of the
// library's ~150 (which also carries the Payne-Hanek path); |x| >= 2^19 goes to the library.
__device__ __forceinline__ void fast_sincos(double x, double *sp, double *cp) {
    if (!(fabs(x) < 524288.0)) {
        sincos(x, sp, cp);
        return;
    }
    const double fn = rint(x * 6.36619772367581382433e-01);
    const int n = (int)fn;
    double r = fma(-fn, 1.57079632673412561417e+00, x);
    r = fma(-fn, 6.07710050630396597660e-11, r);
    r = fma(-fn, 2.02226624879595063154e-21, r);
    const double z = r * r;
    // __kernel_sin(r, 0, 0)
    const double ps = 8.33333333332248946124e-03 +
                      z * (-1.98412698298579493134e-04 +
                           z * (2.75573137070700676789e-06 +
                                z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
    const double sn = r + (z * r) * (-1.66666666666666324348e-01 + z * ps);
    // __kernel_cos(r, 0)
    const double pc =
        z * (4.16666666666666019037e-02 +
             z * (-1.38888888888741095749e-03 +
                  z * (2.48015872894767294178e-05 +
                       z * (-2.75573143513906633035e-07 +
                            z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
    const double ar = fabs(r);
    double cs;
    if (ar < 0.3) {
        cs = 1.0 - (0.5 * z - z * pc);
    } else {
        const double qx = ar > 0.78125 ? 0.28125
                                       : __hiloint2double(__double2hiint(ar) - 0x00200000, 0);
        cs = (1.0 - qx) - ((0.5 * z - qx) - z * pc);
    }
    const int q = n & 3;
    const double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
    *sp = (q & 2) ? -s0 : s0;
    *cp = ((q + 1) & 2) ? -c0 : c0;
}

// Rz(yaw) and the world-frame inverse inertia Iw^-1 = Rz Ib^-1 Rz' (column-major)
__device__ __forceinline__ void srbm_rot_inertia(double yaw, const double *Ibinv, double &cy,
                                                 double &sy, double *Iwi) {
    fast_sincos(yaw, &sy, &cy);
    const double Rz[9] = {cy, sy, 0.0, -sy, cy, 0.0, 0.0, 0.0, 1.0};
    double Tm[9];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < 3; ++l) s += Rz[l * 3 + i] * Ibinv[j * 3 + l];
            Tm[j * 3 + i] = s;
        }
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < 3; ++l) s += Tm[l * 3 + i] * Rz[l * 3 + j];
            Iwi[j * 3 + i] = s;
        }
}

// reference mpcQP::buildSystemModel, include/mpcQP.h:154-181 (lin = {dx, dy, dz})
__device__ __forceinline__ double literal_entry(int i, int j, const double *lin, double mass) {
    const double dx = lin[0], dy = lin[1], dz = lin[2];
    if (j < 13) {
        if (i == 0) return j == 7 ? dz : (j == 8 ? dy : 0.0);
        if (i == 1) return j == 6 ? dz : (j == 8 ? dx : 0.0);
        if (i == 2) return j == 6 ? dy : (j == 7 ? dx : 0.0);
        if (i >= 3 && i < 6) return j == i + 6 ? 1.0 : 0.0;
        if (i == 11) return j == 12 ? -1.0 : 0.0;
        return 0.0;
    }
    const int c = j - 13;
    if (i >= 9 && i < 12) return (i - 9 == c) ? -mass : 0.0;
    return 0.0;
}

// Fill T = [Ac | Bc] * Ts (nx x ns, column-major, ld nx) for this instance.
__device__ __forceinline__ void wave_build_model(const ModelConst &mc, const double *lin,
                                        const double *Ac, const double *Bc, double *T) {
    const int nx = mc.nx, ns = mc.ns;
    double Iwi[9];
    double cy = 1.0, sy = 0.0;
    if (mc.model == 0) {
        fast_sincos(lin[0], &sy, &cy);
        // Iw^-1 = Rz Ib^-1 Rz'
        const double Rz[9] = {cy, sy, 0.0, -sy, cy, 0.0, 0.0, 0.0, 1.0};
        double Tm[9];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                double s = 0.0;
#pragma unroll
                for (int l = 0; l < 3; ++l) s += Rz[l * 3 + i] * mc.Ibinv[j * 3 + l];
                Tm[j * 3 + i] = s;
            }
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                double s = 0.0;
#pragma unroll
                for (int l = 0; l < 3; ++l) s += Tm[l * 3 + i] * Rz[l * 3 + j];
                Iwi[j * 3 + i] = s;
            }
    }
    for (int e = lane(); e < nx * ns; e += kWave) {
        const int i = e % nx, j = e / nx;
        double v;
        if (mc.model == 0) v = srbm_entry(i, j, lin, cy, sy, Iwi, mc.mass);
        else if (mc.model == 1) v = literal_entry(i, j, lin, mc.mass);
        else v = (j < nx) ? Ac[j * nx + i] : Bc[(j - nx) * nx + i];
        T[e] = v * mc.Ts;
    }
    wave_sync();
}

// out = X * Y in the (top block, scalar) algebra: out[:,j] = X1 Y[:,j] (+ sY X[:,j] for j>=nx)
__device__ __forceinline__ void alg_mul(int nx, int ns, const double *X, const double *Y, double sY,
                               double *out) {
    for (int e = lane(); e < nx * ns; e += kWave) {
        const int i = e % nx, j = e / nx;
        double s = 0.0;
        for (int l = 0; l < nx; ++l) s += X[l * nx + i] * Y[j * nx + l];
        if (j >= nx) s += sY * X[e];
        out[e] = s;
    }
    wave_sync();
}

// out = sum_q c[q] M[q] + cI * I (top block; diagonal of the top-left part)
template <int K>
__device__ __forceinline__ void alg_comb(int nx, int ns, double *out, const double (&c)[K],
                                const double *const (&M)[K], double cI) {
    for (int e = lane(); e < nx * ns; e += kWave) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < K; ++q) s += c[q] * M[q][e];
        const int i = e % nx, j = e / nx;
        if (i == j) s += cI;
        out[e] = s;
    }
    wave_sync();
}

__device__ __forceinline__ void expm_pade_solve(int nx, int ns, const double *U, const double *V,
                                                double *D, double *E);
__device__ __forceinline__ void pade_back_substitute(int nx, int ns, const double *D, double *X);

// E = exp([[A, B],[0, 0]]) top block, A = T (nx x ns, already scaled by Ts), Eigen's degree
// selection.  ws: 7 * nx * ns doubles of scratch.  Result written to E (nx x ns).
__device__ __forceinline__ void wave_expm(int nx, int ns, double *T, double *ws, double *E) {
    const int sz = nx * ns;
    double *A2 = ws, *A4 = ws + sz, *A6 = ws + 2 * sz, *A8 = ws + 3 * sz, *U = ws + 4 * sz,
           *V = ws + 5 * sz, *W = ws + 6 * sz;
    // 1-norm of the full (ns x ns) matrix: column sums of the top block (bottom rows are 0)
    double cs = 0.0;
    for (int j = lane(); j < ns; j += kWave) {
        double s = 0.0;
        for (int i = 0; i < nx; ++i) s += fabs(T[j * nx + i]);
        cs = fmax(cs, s);
    }
    const double l1 = wave_max(cs);
    int squarings = 0;
    double b0;
    if (l1 < 1.495585217958292e-002) {
        const double b[] = {120., 60., 12., 1.};
        alg_mul(nx, ns, T, T, 0.0, A2);
        alg_comb<1>(nx, ns, W, {b[3]}, {A2}, b[1]);
        alg_mul(nx, ns, T, W, b[1], U);
        alg_comb<1>(nx, ns, V, {b[2]}, {A2}, b[0]);
        b0 = b[0];
    } else if (l1 < 2.539398330063230e-001) {
        const double b[] = {30240., 15120., 3360., 420., 30., 1.};
        alg_mul(nx, ns, T, T, 0.0, A2);
        alg_mul(nx, ns, A2, A2, 0.0, A4);
        alg_comb<2>(nx, ns, W, {b[5], b[3]}, {A4, A2}, b[1]);
        alg_mul(nx, ns, T, W, b[1], U);
        alg_comb<2>(nx, ns, V, {b[4], b[2]}, {A4, A2}, b[0]);
        b0 = b[0];
    } else if (l1 < 9.504178996162932e-001) {
        const double b[] = {17297280., 8648640., 1995840., 277200., 25200., 1512., 56., 1.};
        alg_mul(nx, ns, T, T, 0.0, A2);
        alg_mul(nx, ns, A2, A2, 0.0, A4);
        alg_mul(nx, ns, A4, A2, 0.0, A6);
        alg_comb<3>(nx, ns, W, {b[7], b[5], b[3]}, {A6, A4, A2}, b[1]);
        alg_mul(nx, ns, T, W, b[1], U);
        alg_comb<3>(nx, ns, V, {b[6], b[4], b[2]}, {A6, A4, A2}, b[0]);
        b0 = b[0];
    } else if (l1 < 2.097847961257068e+000) {
        const double b[] = {17643225600., 8821612800., 2075673600., 302702400., 30270240.,
                            2162160.,     110880.,     3960.,       90.,        1.};
        alg_mul(nx, ns, T, T, 0.0, A2);
        alg_mul(nx, ns, A2, A2, 0.0, A4);
        alg_mul(nx, ns, A4, A2, 0.0, A6);
        alg_mul(nx, ns, A6, A2, 0.0, A8);
        alg_comb<4>(nx, ns, W, {b[9], b[7], b[5], b[3]}, {A8, A6, A4, A2}, b[1]);
        alg_mul(nx, ns, T, W, b[1], U);
        alg_comb<4>(nx, ns, V, {b[8], b[6], b[4], b[2]}, {A8, A6, A4, A2}, b[0]);
        b0 = b[0];
    } else {
        const double maxnorm = 5.371920351148152;
        frexp(l1 / maxnorm, &squarings);
        if (squarings < 0) squarings = 0;
        for (int e = lane(); e < sz; e += kWave) T[e] = ldexp(T[e], -squarings);
        wave_sync();
        const double b[] = {64764752532480000., 32382376266240000., 7771770303897600.,
                            1187353796428800.,  129060195264000.,   10559470521600.,
                            670442572800.,      33522128640.,       1323241920.,
                            40840800.,          960960.,            16380.,
                            182.,               1.};
        alg_mul(nx, ns, T, T, 0.0, A2);
        alg_mul(nx, ns, A2, A2, 0.0, A4);
        alg_mul(nx, ns, A4, A2, 0.0, A6);
        alg_comb<3>(nx, ns, V, {b[13], b[11], b[9]}, {A6, A4, A2}, 0.0);
        alg_mul(nx, ns, A6, V, 0.0, W);               // W = A6 V
        alg_comb<3>(nx, ns, A8, {b[7], b[5], b[3]}, {A6, A4, A2}, b[1]);
        for (int e = lane(); e < sz; e += kWave) W[e] += A8[e];
        wave_sync();
        alg_mul(nx, ns, T, W, b[1], U);                // U = A (A6 V + ... + b1 I)
        alg_comb<3>(nx, ns, W, {b[12], b[10], b[8]}, {A6, A4, A2}, 0.0);
        alg_mul(nx, ns, A6, W, 0.0, V);
        alg_comb<3>(nx, ns, A8, {b[6], b[4], b[2]}, {A6, A4, A2}, b[0]);
        for (int e = lane(); e < sz; e += kWave) V[e] += A8[e];
        wave_sync();
        b0 = b[0];
    }
    (void)b0;
    expm_pade_solve(nx, ns, U, V, A2, E);
    // squarings: (E,1)^2 = [E1 E1, E1 E2 + E2]
    for (int s = 0; s < squarings; ++s) {
        alg_mul(nx, ns, E, E, 1.0, W);
        for (int e = lane(); e < sz; e += kWave) E[e] = W[e];
        wave_sync();
    }
}

// The Pade quotient of wave_expm: numer = U + V (scalar b0), denom = -U + V (scalar b0).
// Solve denom X = numer:  X = [D1^-1 N1, D1^-1 (N2 - D2)]  (bottom block of X is I).
// One wave; D (nx x ns scratch), X = E (nx x ns).
__device__ __forceinline__ void expm_pade_solve(int nx, int ns, const double *U, const double *V,
                                                double *D, double *E) {
    const int sz = nx * ns;
    double *X = E;
    for (int e = lane(); e < sz; e += kWave) {
        const double n = U[e] + V[e], d = -U[e] + V[e];
        D[e] = d;
        X[e] = (e / nx >= nx) ? n - d : n;
    }
    wave_sync();
    // LU with partial pivoting on D[:, 0:nx], applied to all ns columns of X.  Lane jj owns
    // one column of [D(:, k+1:) | X] per step and updates it in registers: every load of a
    // step is issued before its stores (LDS pointers may alias, so a load-after-store chain
    // would cost a round trip per element).  nx <= 32 (MPCQP_MAX_NX), nx + ns <= 64.
    constexpr int MX = 32;
    for (int k = 0; k < nx; ++k) {
        double pv = -1.0;
        int pi = 0x7fffffff;
        for (int i = k + lane(); i < nx; i += kWave) {
            pv = fabs(D[k * nx + i]);
            pi = i;
        }
        wave_argmax(pv, pi);
        if (pi != k) {
            for (int j = lane(); j < ns; j += kWave) {
                if (j < nx) {
                    const double t = D[j * nx + k]; D[j * nx + k] = D[j * nx + pi]; D[j * nx + pi] = t;
                }
                const double t = X[j * nx + k]; X[j * nx + k] = X[j * nx + pi]; X[j * nx + pi] = t;
            }
            wave_sync();
        }
        const double piv = D[k * nx + k];
        // multipliers l_i = D(i, k) / piv, one division per row, kept in place (column k below
        // the pivot is not read again: the back substitution reads the upper factor only)
        for (int i = k + 1 + lane(); i < nx; i += kWave) D[k * nx + i] = D[k * nx + i] / piv;
        wave_sync();
        // update D(i, j) for j > k and X(i, j) for all j, i > k
        const int wD = nx - k - 1, wtot = wD + ns;
        const int jj = lane();
        if (jj < wtot) {
            double *col = jj < wD ? D + (k + 1 + jj) * nx : X + (jj - wD) * nx;
            double lm[MX], v[MX];
#pragma unroll
            for (int i = 0; i < MX; ++i) {
                const bool in = i > k && i < nx;
                lm[i] = in ? D[k * nx + i] : 0.0;
                v[i] = in ? col[i] : 0.0;
            }
            const double ck = col[k];
#pragma unroll
            for (int i = 0; i < MX; ++i)
                if (i > k && i < nx) col[i] = v[i] - lm[i] * ck;
        }
        wave_sync();
    }
    pade_back_substitute(nx, ns, D, X);
}

// U X = Y in place (X = E, nx x ns; U = the upper triangle of D), lane j owns column j of X
// (in registers); one wave
__device__ __forceinline__ void pade_back_substitute(int nx, int ns, const double *D, double *X) {
    constexpr int MX = 32;
    {
        const int j = lane();
        if (j < ns) {
            double v[MX];
#pragma unroll
            for (int i = 0; i < MX; ++i) v[i] = i < nx ? X[j * nx + i] : 0.0;
#pragma unroll
            for (int i = MX - 1; i >= 0; --i) {
                if (i >= nx) continue;
                double s = v[i];
#pragma unroll
                for (int l = i + 1; l < MX; ++l)
                    if (l < nx) s -= D[l * nx + i] * v[l];
                v[i] = s / D[i * nx + i];
            }
#pragma unroll
            for (int i = 0; i < MX; ++i)
                if (i < nx) X[j * nx + i] = v[i];
        }
    }
    wave_sync();
}

// Horizon condensing.  AB = [Ad | Bd] (nx x ns).  ws must hold
//   Phi, QPhi, PPhi: 3 * nx * nV   +   xf: nx * (N+1)   +   Qe: nx * (N+1).
// Writes H (nV x nV column-major, global) and f (nV, global).  If xf_out != nullptr the
// free response Ad^m x0 (m = 0..N) stays in ws for the caller (pointer returned there).
__device__ __forceinline__ void wave_condense(const ModelConst &mc, const double *AB, const double *x0,
                                     const double *xref, double *ws, double *H, double *f,
                                     double **Phi_out, double **xf_out) {
    const int nx = mc.nx, nu = mc.nu, N = mc.N, nV = mc.nV;
    const double *Ad = AB, *Bd = AB + nx * nx;
    double *Phi = ws, *QPhi = ws + nx * nV, *PPhi = ws + 2 * nx * nV;
    double *xf = ws + 3 * nx * nV, *Qe = xf + nx * (N + 1);
    // Phi_0 = Bd, Phi_m = Ad Phi_{m-1}
    for (int e = lane(); e < nx * nu; e += kWave) Phi[e] = Bd[e];
    wave_sync();
    for (int m = 1; m < N; ++m) {
        for (int e = lane(); e < nx * nu; e += kWave) {
            const int i = e % nx, c = e / nx;
            double s = 0.0;
            for (int l = 0; l < nx; ++l) s += Ad[l * nx + i] * Phi[((m - 1) * nu + c) * nx + l];
            Phi[(m * nu + c) * nx + i] = s;
        }
        wave_sync();
    }
    // QPhi = Q Phi, PPhi = P Phi (all columns)
    for (int e = lane(); e < nx * nV; e += kWave) {
        const int i = e % nx, col = e / nx;
        double sq = 0.0, sp = 0.0;
        for (int l = 0; l < nx; ++l) {
            const double ph = Phi[col * nx + l];
            sq += mc.Q[l * nx + i] * ph;
            sp += mc.P[l * nx + i] * ph;
        }
        QPhi[e] = sq;
        PPhi[e] = sp;
    }
    // free response xf_m = Ad^m x0 and weighted errors Qe_m = Q_m (xf_m - xref_m)
    for (int i = lane(); i < nx; i += kWave) xf[i] = x0[i];
    wave_sync();
    for (int m = 1; m <= N; ++m) {
        for (int i = lane(); i < nx; i += kWave) {
            double s = 0.0;
            for (int l = 0; l < nx; ++l) s += Ad[l * nx + i] * xf[(m - 1) * nx + l];
            xf[m * nx + i] = s;
        }
        wave_sync();
    }
    for (int e = lane(); e < nx * N; e += kWave) {
        const int i = e % nx, m = 1 + e / nx;
        const double *W = (m < N) ? mc.Q : mc.P;
        double s = 0.0;
        for (int l = 0; l < nx; ++l) s += W[l * nx + i] * (xf[m * nx + l] - xref[m * nx + l]);
        Qe[m * nx + i] = s;
    }
    wave_sync();
    // H, column-major: consecutive lanes -> consecutive rows (coalesced stores)
    for (int e = lane(); e < nV * nV; e += kWave) {
        const int i = e % nV, j = e / nV;
        const int ki = i / nu, ci = i % nu, kj = j / nu, cj = j % nu;
        const int kk = ki > kj ? ki : kj;
        double s = 0.0;
        for (int m = kk + 1; m <= N; ++m) {
            const double *a = Phi + ((m - 1 - ki) * nu + ci) * nx;
            const double *bq = ((m < N) ? QPhi : PPhi) + ((m - 1 - kj) * nu + cj) * nx;
            double t = 0.0;
            for (int l = 0; l < nx; ++l) t += a[l] * bq[l];
            s += t;
        }
        if (ki == kj) s += mc.R[cj * nu + ci];
        H[e] = 2.0 * s;
    }
    for (int i = lane(); i < nV; i += kWave) {
        const int ki = i / nu, ci = i % nu;
        double s = 0.0;
        for (int m = ki + 1; m <= N; ++m) {
            const double *a = Phi + ((m - 1 - ki) * nu + ci) * nx;
            double t = 0.0;
            for (int l = 0; l < nx; ++l) t += a[l] * Qe[m * nx + l];
            s += t;
        }
        f[i] = 2.0 * s;
    }
    if (Phi_out) *Phi_out = Phi;
    if (xf_out) *xf_out = xf;
}

}  // namespace mpcqp
