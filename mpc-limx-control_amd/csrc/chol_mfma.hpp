// chol_mfma.hpp -- blocked Cholesky H_FF = L L' and triangular inverse X = L^-1 of ONE QP's
// reduced Hessian on the FP64 matrix cores (v_mfma_f64_16x16x4_f64), for the workgroup
// solvers (gi_wg.hpp: the whole-body configuration E and the double-support / standing
// overflow).  The Goldfarb-Idnani start needs J = L^-T and t = L^-1 g (qpOASES's dense
// factorisation in QPSolver::solveQP, src/QPSolver.cpp:87-96); column-by-column sweeps cost one
// workgroup barrier and one LDS broadcast per column, this costs three barriers per 16 columns.
//
// Storage (LDS, per QP): the lower triangle as 16 x 16 tiles, tile (i, j) at TS * tix(i, j).
// A stored tile S is kept in the matrix cores' C/D order ("slices"): element (a, b) of S at
// 64 (a >> 2) + 16 (a & 3) + b, so slice s read at offset 64 s + lane is the accumulator
// register s of an MFMA result (lane l: row (l >> 4) + 4 s, column l & 15), the B operand of
// step s (k = (l >> 4) + 4 s, column l & 15) of S, and the A operand of step s of S' -- every
// operand below is one conflict-free ds_read_b64 at the same offset:
//   H / L tiles (i > j) store their TRANSPOSE (S = L_ij'),  X tiles store X_ij itself,
//   the diagonal tile k ends up holding W_k = L_kk^-1 (= X_kk), Wt[k] holds W_k' (padded
//   layout, see diag_block_inverse_l).
// Algorithm (T = NF / 16 block columns):
//   for k:  W_k = (chol of tile k)^-1 on wave 0 (16 lanes, registers)        | barrier
//           L_ik' = W_k H_ik'                (A = W_k, B = H_ik', 4 MFMAs)    | barrier
//           H_ij' -= L_jk L_ik'  (k < j <= i)(A = L_jk, B = L_ik', 4 MFMAs)   | barrier
//   for i:  X_ij = -W_i sum_{m=j}^{i-1} L_im X_mj  (j < i; the sum's accumulator is the B
//           operand of the W_i product in place)                              | 2 barriers
// Tiles of one step are spread round-robin over the workgroup's waves.
#pragma once
#include "mfma_ops.hpp"

namespace mpcqp {

template <int NF>
struct TileFact {
    static_assert(NF % 16 == 0, "16-column blocks");
    static constexpr int T = NF / 16;
    static constexpr int TS = 272;  // 256 + 16: tiles (i, j) and (i, j + 1) sit 16 bank pairs apart
                                    // (and a W' slot holds the padded (68, 17) layout: 271)
    static constexpr int NT = T * (T + 1) / 2;
    static constexpr int oTiles = 0;
    static constexpr int oWt = NT * TS;        // W_k' slices
    static constexpr int oG = oWt + T * TS;    // g
    static constexpr int oFlag = oG + NF;      // non-PD flag
    static constexpr int doubles = oFlag + 2;
    // X (c, r): row c, column r of X = L^-1 (c >= r) -- J(r, c)
    static __device__ __forceinline__ int xoff(int c, int r) {
        const int i = c >> 4, j = r >> 4, a = c & 15;
        return TS * (i * (i + 1) / 2 + j) + 64 * (a >> 2) + 16 * (a & 3) + (r & 15);
    }
};

__device__ __forceinline__ int tix(int i, int j) { return i * (i + 1) / 2 + j; }

// Cholesky of the 16 x 16 block in `tile` (lower triangle of the stored S = H_kk', i.e. of H_kk
// as it is symmetric) and W = L^-1, on lanes 0..15 of the calling wave: lane i owns row i of L,
// then lane c column c of W.  Writes W's slices over the tile and W' slices to wt.
// MPCQP_DIAG_FUSED: W's forward substitution runs inside the factorisation (right-looking:
// step k's broadcast L(j, k) feeds both the trailing update of row j and w[j] -= L(j, k) w[k]),
// instead of a second sweep of 120 more v_readlane pairs after it.  0 keeps the two sweeps.
#ifndef MPCQP_DIAG_FUSED
#define MPCQP_DIAG_FUSED 1
#endif
#ifndef MPCQP_DIAG_NOSEL
#define MPCQP_DIAG_NOSEL 1
#endif
// MPCQP_DIAG_DPP: every 16-lane row of the wave factors the same block (lane i of each row owns
// row i), and step k's broadcast L(j, k) comes from lane j of the lane's own row inside the FMA
// (v_fmac_f64_dpp row_newbcast), instead of 120 v_readlane pairs per block whose SGPR results
// spilled to VGPR lanes.  Same operations in the same order per element (bit-identical).
// 0: the v_readlane form (A/B builds).
#ifndef MPCQP_DIAG_DPP
#define MPCQP_DIAG_DPP 1
#endif
// acc -= (lane J of this lane's 16-lane row of b) * m; NOP: give b its two wait states after the
// VALU that wrote it
template <int J, bool NOP>
__device__ __forceinline__ void fmac_rowbcast_neg(double &acc, double b, double m) {
    if constexpr (NOP)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%c3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc) : "v"(b), "v"(m), "i"(J));
    else
        asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%c3 row_mask:0xf bank_mask:0xf"
            : "+v"(acc) : "v"(b), "v"(m), "i"(J));
}
// step K's updates of row entries and W columns j = J .. 15 (J = K + 1 first)
template <int K, int J = K + 1>
__device__ __forceinline__ void diag_step_dpp(double (&a)[16], double (&w)[16], double lk) {
    if constexpr (J < 16) {
        fmac_rowbcast_neg<J, J == K + 1>(a[J], lk, lk);     // a[j] -= L(j, k) L(ln, k)
        fmac_rowbcast_neg<J, false>(w[J], lk, w[K]);         // w[j] -= L(j, k) w[k]
        diag_step_dpp<K, J + 1>(a, w, lk);
    }
}
template <int K = 0>
__device__ __forceinline__ void diag_factor_dpp(double (&a)[16], double (&w)[16], bool &bad) {
    if constexpr (K < 16) {
        const double piv = dpp<0x150 + K>(a[K]);  // lane K of the row (row_newbcast)
        bad |= !(piv > 0.0);
        const double isq = rsqrt_nr(piv);
        const double lk = a[K] * isq;
        a[K] = lk;
        w[K] *= isq;
        diag_step_dpp<K>(a, w, lk);
        diag_factor_dpp<K + 1>(a, w, bad);
    }
}
// Layouts: element (a, b) of a 16 x 16 tile at P4 (a >> 2) + P1 (a & 3) + b.  (64, 16) is the
// MFMA slice order (register s of lane l at 64 s + l); there the row reads below (lane i reads
// row i) stride 16 doubles and land on two bank pairs: 8-way conflicts, and so do the row
// stores of W'.  (68, 17) pads each 16-double group by one and each slice by four: the 16 rows
// start on distinct bank pairs, and slice reads (68 s + 17 (l >> 4) + (l & 15)) stay
// conflict-free but for one lane pair.  diag_block_inverse_l reads the block from src in
// (S4, S1), writes W to wd in (W4, W1) and W' to td in (T4, T1); src may alias either output
// (every read precedes every write).
template <int S4, int S1, int W4, int W1, int T4, int T1>
__device__ __forceinline__ void diag_block_inverse_rl(const double *src, double *wd, double *td,
                                                      bool &bad);
template <int S4, int S1, int W4, int W1, int T4, int T1>
__device__ __forceinline__ void diag_block_inverse_l(const double *src, double *wd, double *td,
                                                     bool &bad) {
#if MPCQP_DIAG_DPP
    const int ln = lane();
    const int li = ln & 15;
    double a[16], w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        a[j] = (j <= li) ? src[S4 * (li >> 2) + S1 * (li & 3) + j] : 0.0;
        w[j] = (li == j) ? 1.0 : 0.0;
    }
    // (every row computes the same pivots; the ballot keeps the flag wave-uniform for the
    //  compiler, which otherwise treats the solver's status as divergent from here on)
    bool nb = false;
    diag_factor_dpp(a, w, nb);
    bad |= __ballot(nb) != 0ull;
    if (ln < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            wd[W4 * (i >> 2) + W1 * (i & 3) + li] = w[i];   // W(i, c), c = li
            td[T4 * (li >> 2) + T1 * (li & 3) + i] = w[i];  // W'(c, i)
        }
    }
    return;
#endif
    diag_block_inverse_rl<S4, S1, W4, W1, T4, T1>(src, wd, td, bad);
}
// the block in place in the slice order, W' to wt in the slice order
__device__ __forceinline__ void diag_block_inverse(double *tile, double *wt, bool &bad) {
    diag_block_inverse_l<64, 16, 64, 16, 64, 16>(tile, tile, wt, bad);
}
template <int S4, int S1, int W4, int W1, int T4, int T1>
__device__ __forceinline__ void diag_block_inverse_rl(const double *src, double *wd, double *td,
                                                      bool &bad) {
    const int ln = lane();
    const bool on = ln < 16;
    const int li = ln & 15;
    double a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
        a[j] = (on && j <= li) ? src[S4 * (li >> 2) + S1 * (li & 3) + j] : 0.0;
    double iq[16];
    double w[16];  // lane c: column c of W = L^-1 (fused form: e_c, reduced step by step)
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = (li == j) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const double piv = readlane(a[k], k);
        bad |= !(piv > 0.0);
        const double isq = rsqrt_nr(piv);
        iq[k] = isq;
        const double lk = a[k] * isq;  // L(ln, k); on lane k, L(k, k) = piv / sqrt(piv)
        a[k] = lk;
        if (MPCQP_DIAG_FUSED) w[k] *= isq;
#pragma unroll
        for (int j = k + 1; j < 16; ++j) {
            const double ljk = readlane(lk, j);
            // (unmasked: a lane li <= k only changes its row's entries right of the diagonal,
            //  which nothing reads -- lanes li < k hold zeros there and lk = 0 -- and no lane
            //  reads another's row but through lk of lanes j > k)
            if (MPCQP_DIAG_NOSEL || li > k) a[j] -= lk * ljk;
            if (MPCQP_DIAG_FUSED) w[j] -= ljk * w[k];
        }
    }
    if (!MPCQP_DIAG_FUSED) {
        // W = L^-1, lane c: column c by forward substitution (L entries are wave-uniform)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            double s = (li == i) ? 1.0 : 0.0;
#pragma unroll
            for (int m = 0; m < i; ++m) s -= readlane(a[m], i) * w[m];
            w[i] = s * iq[i];
        }
    }
    if (on) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            wd[W4 * (i >> 2) + W1 * (i & 3) + li] = w[i];   // W(i, c), c = li
            td[T4 * (li >> 2) + T1 * (li & 3) + i] = w[i];  // W'(c, i)
        }
    }
}

// Blocked factorisation + inverse of the NF x NF matrix whose tiles are in F (TileFact layout),
// by the workgroup's NW waves (wave index wv).  Returns the non-PD flag (same on every thread).
// MPCQP_CHOL_LOOKAHEAD: the diagonal block k + 1 is updated first in step k's trailing update,
// by wave 0, which then factors and inverts it at once while the other waves finish the step's
// remaining tiles -- the serial 16-lane factorisation leaves the critical path of every step but
// the first, and each step loses a barrier.  Same operations in the same order per element
// (bit-identical).  0: the diagonal factorisation as its own stage (A/B builds).
#ifndef MPCQP_CHOL_LOOKAHEAD
#define MPCQP_CHOL_LOOKAHEAD 1
#endif
#ifndef MPCQP_WG_DIAG_PAD
#define MPCQP_WG_DIAG_PAD 1
#endif
template <int NF, int NW>
__device__ __forceinline__ bool chol_inverse_mfma(double *F, int wv) {
    using TF = TileFact<NF>;
    constexpr int T = TF::T, TS = TF::TS;
    constexpr bool LA = MPCQP_CHOL_LOOKAHEAD && NW > 1;
    const int ln = lane();
    double *tiles = F + TF::oTiles, *Wt = F + TF::oWt;
    bool bad = false;
    // MPCQP_WG_DIAG_PAD: the diagonal block is staged into W_k''s slot in the padded (68, 17)
    // layout, factored from there (conflict-free row reads), W_k lands in the tile in slice order
    // and W_k' in the padded layout (conflict-free row stores), which the panel and X products
    // read as slices (68 s + so).  0: everything in slice order (A/B builds).
    constexpr int Q4 = MPCQP_WG_DIAG_PAD ? 68 : 64, Q1 = MPCQP_WG_DIAG_PAD ? 17 : 16;
    const int so = Q1 * (ln >> 4) + (ln & 15);
    auto diag = [&](int k) {
        double *tk = tiles + TS * tix(k, k), *wk = Wt + TS * k;
        if constexpr (MPCQP_WG_DIAG_PAD) {
            double v[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) v[s] = tk[64 * s + ln];
#pragma unroll
            for (int s = 0; s < 4; ++s) wk[Q4 * s + so] = v[s];
            wave_sync();
            diag_block_inverse_l<Q4, Q1, 64, 16, Q4, Q1>(wk, tk, wk, bad);
        } else {
            diag_block_inverse(tk, wk, bad);
        }
        if (ln == 0 && bad) F[TF::oFlag] = 1.0;
    };
    // trailing pair t of step k (k < j <= i, row-major: t = 0 is the diagonal tile (k+1, k+1))
    auto trail = [&](int k, int t) {
        int i = k + 1, rem = t;
        while (rem >= i - k) { rem -= i - k; ++i; }
        const int j = k + 1 + rem;
        const double *lj = tiles + TS * tix(j, k), *li = tiles + TS * tix(i, k);
        double *c = tiles + TS * tix(i, j);
        dx4 acc = {c[ln], c[64 + ln], c[128 + ln], c[192 + ln]};
#pragma unroll
        for (int s = 0; s < 4; ++s)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-lj[64 * s + ln], li[64 * s + ln], acc, 0, 0, 0);
#pragma unroll
        for (int s = 0; s < 4; ++s) c[64 * s + ln] = acc[s];
    };
    if (LA) {
        if (wv == 0) diag(0);
        __syncthreads();
    }
    for (int k = 0; k < T; ++k) {
        if (!LA) {
            if (wv == 0) diag(k);
            __syncthreads();
        }
        // panel: L_ik' = W_k H_ik'
        for (int i = k + 1 + wv; i < T; i += NW) {
            const double *wk = Wt + TS * k;
            double *ti = tiles + TS * tix(i, k);
            dx4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(wk[Q4 * s + so], ti[64 * s + ln], acc, 0, 0, 0);
#pragma unroll
            for (int s = 0; s < 4; ++s) ti[64 * s + ln] = acc[s];
        }
        if (k + 1 == T) break;  // (no trailing tile after the last panel: nothing follows)
        __syncthreads();
        // trailing update: H_ij' -= L_jk L_ik', k < j <= i (pairs in row-major order)
        const int np = (T - 1 - k) * (T - k) / 2;
        if (LA) {
            if (wv == 0) {  // the next diagonal tile, then its factorisation (look-ahead)
                trail(k, 0);
                wave_sync();
                diag(k + 1);
            } else {
                for (int t = wv; t < np; t += NW - 1) trail(k, t);
            }
        } else {
            for (int t = wv; t < np; t += NW) trail(k, t);
        }
        __syncthreads();
    }
    __syncthreads();
    // X = L^-1 below the diagonal, block row by block row
    constexpr int MAXJ = (T - 1 + NW - 1) / NW;
    for (int i = 1; i < T; ++i) {
        dx4 xr[MAXJ > 0 ? MAXJ : 1];
#pragma unroll
        for (int u = 0; u < MAXJ; ++u) {
            const int j = wv + u * NW;
            if (j >= i) break;
            dx4 q = {0.0, 0.0, 0.0, 0.0};
            for (int m = j; m < i; ++m) {
                const double *lim = tiles + TS * tix(i, m), *xmj = tiles + TS * tix(m, j);
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    q = __builtin_amdgcn_mfma_f64_16x16x4f64(lim[64 * s + ln], xmj[64 * s + ln], q, 0, 0, 0);
            }
            const double *wi = Wt + TS * i;
            dx4 x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < 4; ++s)
                x = __builtin_amdgcn_mfma_f64_16x16x4f64(-wi[Q4 * s + so], q[s], x, 0, 0, 0);
            xr[u] = x;
        }
        __syncthreads();  // every read of L_i* is done before X_i* overwrites it
#pragma unroll
        for (int u = 0; u < MAXJ; ++u) {
            const int j = wv + u * NW;
            if (j >= i) break;
            double *c = tiles + TS * tix(i, j);
#pragma unroll
            for (int s = 0; s < 4; ++s) c[64 * s + ln] = xr[u][s];
        }
        __syncthreads();
    }
    return F[TF::oFlag] != 0.0;
}

}  // namespace mpcqp
