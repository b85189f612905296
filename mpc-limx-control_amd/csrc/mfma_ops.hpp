// mfma_ops.hpp -- FP64 matrix-core products (v_mfma_f64_16x16x4_f64) of the small dense
// matrices of one QP, for the workgroup kernels: the condensing contractions of the dense
// (whole-body) model, where B'QB is a genuine dense contraction (SURVEY.md 8a a5,
// src/QPSolver.cpp:58).
#pragma once
#include "wave_ops.hpp"

namespace mpcqp {

typedef double dx4 __attribute__((ext_vector_type(4)));

// C = alpha op(A) B (+ D), all column-major; op(A) = A (m x k, lda) or A' (A stored k x m).
// Output tiles of 16 x 16 go to waves w0 .. w0+nw-1 of the workgroup (tile t -> wave
// w0 + t % nw; wv and the sizes are wave-uniform); rows, columns and k beyond the sizes read 0
// and are not stored.  Operand maps of the f64 16x16x4 form (cdna_hip_programming.md section
// 3): lane l supplies A(row l & 15, k = 4s + (l >> 4)) and B(k = 4s + (l >> 4), col l & 15);
// accumulator register r holds D(row (l >> 4) + 4r, col l & 15).  C must not alias A, B or D.
// BATCH: load all of a tile's operands before its MFMA chain (k <= 32); off where registers
// are scarce (the H-row staging holds each thread's row part live across the product)
template <bool TA, bool BATCH = true>
__device__ __forceinline__ void mfma_gemm(int m, int n, int k, const double *A, int lda,
                                          const double *B, int ldb, double *C, int ldc,
                                          const double *D, int ldd, double alpha, int wv, int w0,
                                          int nw) {
    if (wv < w0 || wv >= w0 + nw) return;
    const int tm_n = (m + 15) >> 4, tn_n = (n + 15) >> 4, ks = (k + 3) >> 2;
    const int ln = lane(), li = ln & 15, lk = ln >> 4;
    for (int t = wv - w0; t < tm_n * tn_n; t += nw) {
        const int tm = t % tm_n, tn = t / tm_n;
        const int i = tm * 16 + li, j = tn * 16 + li;
        dx4 acc = {0.0, 0.0, 0.0, 0.0};
        if (BATCH && ks <= 8) {
            // k <= 32 (every product of the dense path): all operands loaded first, from
            // clamped addresses with the out-of-range ones zeroed by a select (no EXEC-masked
            // loads, one wait), then the MFMA chain
            double av[8], bv[8];
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int kk = 4 * s + lk;
                const bool oka = s < ks && i < m && kk < k, okb = s < ks && j < n && kk < k;
                const double a = A[oka ? (TA ? i * lda + kk : kk * lda + i) : 0];
                const double b = B[okb ? j * ldb + kk : 0];
                av[s] = oka ? a : 0.0;
                bv[s] = okb ? b : 0.0;
            }
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s], bv[s], acc, 0, 0, 0);
        } else {
            for (int s = 0; s < ks; ++s) {
                const int kk = 4 * s + lk;
                const bool kin = kk < k;
                const double a = (i < m && kin) ? (TA ? A[i * lda + kk] : A[kk * lda + i]) : 0.0;
                const double b = (j < n && kin) ? B[j * ldb + kk] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = tm * 16 + lk + 4 * r, col = tn * 16 + li;
            if (row < m && col < n) {
                double v = alpha * acc[r];
                if (D) v += D[col * ldd + row];
                C[col * ldc + row] = v;
            }
        }
    }
}

}  // namespace mpcqp
