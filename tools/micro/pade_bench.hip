// Micro-benchmark of the one-wave Pade Gauss-Jordan (expm_wg.hpp wave_pade_gj<24>) in isolation:
// one wavefront per block, [U | V] for 24 x 30 from global memory into LDS, the solve, E back;
// per-block s_memtime cycles.  Build: hipcc -O3 --offload-arch=gfx950 -I../../mpc-limx-control_amd/csrc
// Diagnostic only (tools/): variants are compared here before one goes into expm_wg.hpp.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "expm_wg.hpp"
using namespace mpcqp;
constexpr int NX = 24, NS = 30, SZ = NX * NS;


// ---- local variants of wave_pade_gj<24> (VAR bit 0: reciprocal by v_rcp_f64 + 2 Newton steps
//      instead of the IEEE division; bit 1: column k by DPP row broadcast + lane swaps instead of
//      v_readlane)
template <int K>
__device__ __forceinline__ double bcast_k(double v) {
    const double r = dpp<0x150 + (K & 15)>(v);
    const long long bb = __double_as_longlong(r);
    const int lo = (int)(bb & 0xffffffffll), hi = (int)(bb >> 32);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const int tl = (K & 16) ? (int)l[1] : (int)l[0], th = (K & 16) ? (int)h[1] : (int)h[0];
    const auto l2 = __builtin_amdgcn_permlane32_swap(tl, tl, false, false);
    const auto h2 = __builtin_amdgcn_permlane32_swap(th, th, false, false);
    const int ol = (K & 32) ? (int)l2[1] : (int)l2[0], oh = (K & 32) ? (int)h2[1] : (int)h2[0];
    return __longlong_as_double(((long long)oh << 32) | (unsigned)ol);
}
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    return r;
}
template <int VAR, int K, int NXC>
__device__ __forceinline__ void col_k(const double (&a)[NXC], double (&ck)[NXC]) {
#pragma unroll
    for (int i = 0; i < NXC; ++i) ck[i] = (VAR & 2) ? bcast_k<K>(a[i]) : readlane(a[i], K);
}
template <int VAR, int NXC, int K = 0>
__device__ __forceinline__ void gj_steps(double (&a)[NXC], double &piv_own) {
    if constexpr (K < NXC) {
        constexpr int k = K;
        const int j = lane();
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
        double ck[NXC];
        col_k<VAR, K, NXC>(a, ck);
        double pk = a[k], ckk = ck[k];
        const double rk = a[k];
#pragma unroll
        for (int i = k + 1; i < NXC; ++i)
            if (p == i) { pk = a[i]; ckk = ck[i]; a[i] = rk; }
        a[k] = pk;
        piv_own = (j == k) ? pk : piv_own;
        const double rp = (VAR & 1) ? rcp_nr(ckk) : 1.0 / ckk;
#pragma unroll
        for (int i = 0; i < NXC; ++i) {
            if (i == k) continue;
            const double ci = (i > k && p == i) ? ck[k] : ck[i];
            a[i] = a[i] - (ci * rp) * pk;
        }
        gj_steps<VAR, NXC, K + 1>(a, piv_own);
    }
}
template <int VAR, int NXC>
__device__ __forceinline__ void pade_var(int ns, const double *U, const double *V, double *E) {
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
    double piv_own = 0.0;
    gj_steps<VAR, NXC>(a, piv_own);
#pragma unroll
    for (int i = 0; i < NXC; ++i) {
        const double dii = readlane(piv_own, i);
        if (colok && j >= nx) E[(j - nx) * nx + i] = (VAR & 1) ? a[i] * rcp_nr(dii) : a[i] / dii;
    }
}

template <int VAR>
__global__ void __launch_bounds__(64) k_pade(const double *U, const double *V, double *E,
                                             unsigned long long *cyc, int reps) {
    __shared__ double sU[SZ], sV[SZ], sE[SZ], scr[512];
    const int b = blockIdx.x, ln = threadIdx.x;
    for (int e = ln; e < SZ; e += 64) { sU[e] = U[(size_t)b * SZ + e]; sV[e] = V[(size_t)b * SZ + e]; }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (VAR < 0) wave_pade_gj<NX>(NS, sU, sV, sE, scr);
        else pade_var<VAR < 0 ? 0 : VAR, NX>(NS, sU, sV, sE);
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    for (int e = ln; e < SZ; e += 64) E[(size_t)b * SZ + e] = sE[e];
    if (ln == 0) cyc[b] = t1 - t0;
}

int main(int argc, char **argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 1024, reps = argc > 2 ? atoi(argv[2]) : 4;
    std::vector<double> hU((size_t)B * SZ), hV((size_t)B * SZ);
    srand(7);
    auto rnd = [] { return (double)rand() / RAND_MAX - 0.5; };
    for (int b = 0; b < B; ++b)
        for (int j = 0; j < NS; ++j)
            for (int i = 0; i < NX; ++i) {
                const size_t e = (size_t)b * SZ + j * NX + i;
                hU[e] = 0.3 * rnd();
                hV[e] = (i == j ? 2.0 : 0.0) + 0.2 * rnd();
            }
    double *U, *V, *E;
    unsigned long long *cyc;
    (void)hipMalloc(&U, hU.size() * 8); (void)hipMalloc(&V, hV.size() * 8);
    (void)hipMalloc(&E, hU.size() * 8); (void)hipMalloc(&cyc, B * 8);
    (void)hipMemcpy(U, hU.data(), hU.size() * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(V, hV.data(), hV.size() * 8, hipMemcpyHostToDevice);
    std::vector<unsigned long long> c(B);
    std::vector<double> ref(hU.size()), out(hU.size());
    auto run = [&](auto kern, const char *name, bool keep) {
        for (int pass = 0; pass < 2; ++pass) {
            hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            kern<<<B, 64>>>(U, V, E, cyc, reps);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
            (void)hipMemcpy(c.data(), cyc, B * 8, hipMemcpyDeviceToHost);
            (void)hipMemcpy(out.data(), E, out.size() * 8, hipMemcpyDeviceToHost);
            double s = 0; for (auto v : c) s += (double)v;
            if (keep) ref = out;
            double err = 0; for (size_t i = 0; i < out.size(); ++i) err = fmax(err, fabs(out[i] - ref[i]));
            if (pass) printf("%-28s B %d reps %d  kernel %.3f ms  cycles per solve %.0f  max|E - lib| %.2e\n", name, B, reps, ms, s / B / reps, err);
        }
    };
    run(k_pade<-1>, "library wave_pade_gj<24>", true);
    run(k_pade<0>, "var 0 (copy, if-chain swap)", false);
    run(k_pade<1>, "var 1 (rcp + Newton)", false);
    run(k_pade<2>, "var 2 (DPP broadcast)", false);
    run(k_pade<3>, "var 3 (both)", false);
    return 0;
}
