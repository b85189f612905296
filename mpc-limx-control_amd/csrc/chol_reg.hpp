// chol_reg.hpp -- the one-wave form of chol_mfma.hpp: blocked Cholesky H_FF = L L', X = L^-1,
// J = X' (row r of J on lane r) and t = L^-1 g for ONE QP held by ONE wavefront, on the FP64
// matrix cores (v_mfma_f64_16x16x4_f64) with every tile in registers.  Replaces the
// column-by-column sweeps of gi_run_reg (one LDS broadcast per FMA) for the one-QP kernels
// (configs C and L, NF = 60).  Same tile conventions as chol_mfma.hpp (a stored tile S is an
// MFMA accumulator: lane l, register s = S((l >> 4) + 4 s, l & 15), which is also the B
// operand of step s of S and the A operand of step s of S'):
//   off-diagonal L tiles hold L_ij', X tiles hold X_ij, the diagonal tile holds H_kk (lower
//   triangle valid) until its block is factored, then W_k = L_kk^-1; wt[k] holds W_k'.
// LDS: 608 doubles of scratch (diagonal-block staging and X-tile readout in the padded layout
// (68, 17) of diag_block_inverse_l, W' staging, g), over the packed H once every tile is loaded.
// (The (64, 16) slice order made every row read of the staged tile an 8-way bank conflict: the
// diagonal factorisation's loads and W' stores and the t = X g readout.)
#pragma once
#include "chol_mfma.hpp"

// MPCQP_CHOL_PAD: stage tiles in the padded (68, 17) layout; 0: the (64, 16) slice order (A/B)
#ifndef MPCQP_CHOL_PAD
#define MPCQP_CHOL_PAD 1
#endif

namespace mpcqp {

// Hb: packed lower H_FF (row-major, Hb[lrow(r) + c], c <= r < nf); identity beyond nf.
// Lane r returns row r of J in Jr (J(r, c) = X(c, r), 0 below the diagonal) and t_r.
template <int NF>
__device__ __forceinline__ void reg_chol_inverse_mfma(const double *Hb, int nf, double g,
                                                      double *scratch, double (&Jr)[NF],
                                                      double &t, bool &bad) {
    constexpr int T = (NF + 15) / 16, NT = T * (T + 1) / 2;
    const int ln = lane(), li = ln & 15, lk = ln >> 4;
    constexpr int P4 = MPCQP_CHOL_PAD ? 68 : 64, P1 = MPCQP_CHOL_PAD ? 17 : 16, PS = 272;  // padded tile layout and its footprint
    double *gbuf = scratch + 2 * PS;
    const int so = P1 * lk + li;               // this lane's slot of slice s: P4 s + so
    dx4 tl[NT];
    dx4 wt[T];
    // ---- tiles from the packed H (symmetric reads; identity padding)
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                int r, c;
                if (i != j) { r = 16 * i + li; c = 16 * j + lk + 4 * s; }      // S = H_ij'
                else        { r = 16 * i + lk + 4 * s; c = 16 * i + li; }      // S = H_ii
                const int hi = r > c ? r : c, lo = r > c ? c : r;
                tl[tix(i, j)][s] = (r < nf && c < nf) ? Hb[hi * (hi + 1) / 2 + lo] : (r == c ? 1.0 : 0.0);
            }
    const double gl = (ln < nf) ? g : 0.0;
    wave_sync();  // every read of the packed H is done: its space is the scratch from here
    gbuf[ln] = gl;
    // ---- blocked right-looking Cholesky
#pragma unroll
    for (int k = 0; k < T; ++k) {
#pragma unroll
        for (int s = 0; s < 4; ++s) scratch[P4 * s + so] = tl[tix(k, k)][s];
        wave_sync();
        diag_block_inverse_l<P4, P1, P4, P1, P4, P1>(scratch, scratch, scratch + PS, bad);
        wave_sync();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            tl[tix(k, k)][s] = scratch[P4 * s + so];
            wt[k][s] = scratch[PS + P4 * s + so];
        }
        wave_sync();
#pragma unroll
        for (int i = k + 1; i < T; ++i) {  // panel: L_ik' = W_k H_ik'
            dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(wt[k][s], tl[tix(i, k)][s], acc, 0, 0, 0);
            tl[tix(i, k)] = acc;
        }
#pragma unroll
        for (int j = k + 1; j < T; ++j)  // trailing: H_ij' -= L_jk L_ik'
#pragma unroll
            for (int i = j; i < T; ++i) {
                dx4 acc = tl[tix(i, j)];
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-tl[tix(j, k)][s], tl[tix(i, k)][s],
                                                               acc, 0, 0, 0);
                tl[tix(i, j)] = acc;
            }
    }
    // ---- X = L^-1 below the diagonal, block row by block row
#pragma unroll
    for (int i = 1; i < T; ++i) {
        dx4 xr[T];
#pragma unroll
        for (int j = 0; j < i; ++j) {
            dx4 q = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int m = j; m < i; ++m)
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    q = __builtin_amdgcn_mfma_f64_16x16x4f64(tl[tix(i, m)][s], tl[tix(m, j)][s], q,
                                                             0, 0, 0);
            dx4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                x = __builtin_amdgcn_mfma_f64_16x16x4f64(-wt[i][s], q[s], x, 0, 0, 0);
            xr[j] = x;
        }
#pragma unroll
        for (int j = 0; j < i; ++j) tl[tix(i, j)] = xr[j];
    }
    // ---- readout, one X tile at a time through the scratch: J(r, c) = X(c, r) on the lanes of
    //      block column j, t_r += X(r, c) g_c on the lanes of block row i
#pragma unroll
    for (int l = 0; l < NF; ++l) Jr[l] = 0.0;
    double tt = 0.0;
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
#pragma unroll
            for (int s = 0; s < 4; ++s) scratch[P4 * s + so] = tl[tix(i, j)][s];
            wave_sync();
            if (lk == j) {
#pragma unroll
                for (int cc = 0; cc < 16; ++cc)
                    if (16 * i + cc < NF)
                        Jr[16 * i + cc < NF ? 16 * i + cc : 0] =
                            scratch[P4 * (cc >> 2) + P1 * (cc & 3) + li];
            }
            if (lk == i) {
#pragma unroll
                for (int cc = 0; cc < 16; ++cc)
                    tt += scratch[P4 * (li >> 2) + P1 * (li & 3) + cc] * gbuf[16 * j + cc];
            }
            wave_sync();
        }
    t = tt;
}

}  // namespace mpcqp
