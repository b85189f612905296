// mpcqp_kernels.hip -- HIP kernels (gfx950) and the extern "C" implementation of
// include/mpcqp.h.  One QP instance per 64-lane wavefront, one wavefront per workgroup.
//
// Kernels
//   k_condense   linearise (SRBM / literal / given Ac,Bc) -> exp(M Ts) -> Phi_k = Ad^k Bd ->
//                H, f (and, for the single-instance reference API, the reference's constraint
//                arrays A_eq, b_eq, lb, ub, A_ineq, lbA, ubA).        src/QPSolver.cpp:21-81,
//                include/mpcQP.h:121-182
//   k_solve      corrected dense QP, Goldfarb-Idnani                  src/QPSolver.cpp:83-106
//   k_discretize<..>, k_condense_solve<..>   the batched hot path with compile-time dims
//                (fused.hpp): linearise + expm, then Phi, H_FF, f and the solve in LDS
//   k_mpc<..>, k_mpc_gen<..>   the whole tick in one kernel (mpc_fused.hpp), one QP per wave
//   k_mpc_pair<..>             the same, two QPs per wave for nf <= 30 (mpc_pair.hpp)
//                (instantiated in fast_srbm10 / fast_srbm20 / fast_literal / fast_pair.hip)
//   k_select_min per-rank min-cost key (multi-GPU selection)
//   k_plant      x <- Ad x + Bd u                                       src/QPSolver.cpp:108-111
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/mpcqp.h"

#include "fast_kernels.hpp"
#include "gi_solver.hpp"
#include "gi_wg.hpp"

using namespace mpcqp;

namespace {

struct CondenseArgs {
    ModelConst mc;
    int B;
    const double *x0, *xref, *lin;   // [B][nx], [B][N+1][nx], [B][8]
    const double *Ac, *Bc;           // generic model [B][nx*nx], [B][nx*nu]
    const double *ABin;              // optional [B][nx*ns] = [Ad | Bd] (skip discretisation)
    double *H, *f;                   // [B][nV*nV], [B][nV] (nullable when discretize_only)
    double *ABout;                   // optional [B][nx*ns]
    int discretize_only;
    // reference-layout extras (single instance API)
    const double *x_min, *x_max;
    double u_min, u_max;
    double *A_eq, *b_eq, *lb, *ub, *A_ineq, *lbA, *ubA;
};

size_t condense_lds_doubles(int nx, int nu, int N) {
    const int ns = nx + nu, nV = nu * N;
    const size_t ab = (size_t)nx * ns;
    const size_t expm_ws = 8 * ab;  // T + 7 scratch
    const size_t cond_ws = 3 * (size_t)nx * nV + 2 * (size_t)nx * (N + 1);
    return ab + std::max(expm_ws, cond_ws);
}

__global__ void __launch_bounds__(64) k_condense(CondenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem_d[];
    const int b = blockIdx.x;
    if (b >= a.B) return;
    const ModelConst &mc = a.mc;
    const int nx = mc.nx, ns = mc.ns, nV = mc.nV, N = mc.N;
    double *AB = smem_d;                 // [Ad | Bd]
    double *ws = smem_d + nx * ns;       // scratch
    if (a.ABin) {
        for (int e = lane(); e < nx * ns; e += kWave) AB[e] = a.ABin[(size_t)b * nx * ns + e];
        wave_sync();
    } else {
        double *T = ws;
        double lin[8];
        if (a.lin && mc.model != 2)
#pragma unroll
            for (int i = 0; i < 8; ++i) lin[i] = a.lin[(size_t)b * 8 + i];
        const double *Acb = a.Ac ? a.Ac + (size_t)b * nx * nx : nullptr;
        const double *Bcb = a.Bc ? a.Bc + (size_t)b * nx * mc.nu : nullptr;
        if (mc.model == 2 && a.lin) {  // dense model: lin = [Ac | Bc] per instance
            // (the single-instance entry points pass model 2 with Ac/Bc and no lin)
            Acb = a.lin + (size_t)b * nx * ns;
            Bcb = Acb + nx * nx;
        }
        wave_build_model(mc, lin, Acb, Bcb, T);
        wave_expm(nx, ns, T, ws + nx * ns, AB);
    }
    if (a.ABout)
        for (int e = lane(); e < nx * ns; e += kWave) a.ABout[(size_t)b * nx * ns + e] = AB[e];
    if (a.discretize_only) return;
    double *Phi = nullptr, *xf = nullptr;
    wave_condense(mc, AB, a.x0 + (size_t)b * nx, a.xref + (size_t)b * nx * (N + 1), ws,
                  a.H + (size_t)b * nV * nV, a.f + (size_t)b * nV, &Phi, &xf);
    // reference constraint arrays (src/QPSolver.cpp:63-80)
    const int nu = mc.nu, NE = nx * N, NI = 2 * nx * N;
    if (a.A_eq)
        for (int e = lane(); e < NE * nV; e += kWave) {
            const int r = e % NE, c = e / NE, m = r / nx + 1, i = r % nx, k = c / nu, cc = c % nu;
            a.A_eq[(size_t)b * NE * nV + e] = (k < m) ? Phi[((m - 1 - k) * nu + cc) * nx + i] : 0.0;
        }
    if (a.b_eq)
        for (int r = lane(); r < NE; r += kWave) a.b_eq[(size_t)b * NE + r] = xf[nx + r];
    if (a.lb)
        for (int r = lane(); r < nV; r += kWave) a.lb[(size_t)b * nV + r] = a.u_min;
    if (a.ub)
        for (int r = lane(); r < nV; r += kWave) a.ub[(size_t)b * nV + r] = a.u_max;
    if (a.A_ineq)
        for (int e = lane(); e < NI * nV; e += kWave) {
            const int r = e % NI, c = e / NI, blk = r / nx;
            double v = 0.0;
            if ((blk & 1) == 0) {
                const int m = blk / 2 + 1, i = r % nx, k = c / nu, cc = c % nu;
                v = (k < m) ? Phi[((m - 1 - k) * nu + cc) * nx + i] : 0.0;
            }
            a.A_ineq[(size_t)b * NI * nV + e] = v;
        }
    if (a.lbA || a.ubA)
        for (int r = lane(); r < NI; r += kWave) {
            const int blk = r / nx, i = r % nx;
            double lo = -kInfty, hi = kInfty;
            if ((blk & 1) == 0) {
                const double fr = xf[(blk / 2 + 1) * nx + i];
                lo = a.x_min[i] - fr;
                hi = a.x_max[i] - fr;
            }
            if (a.lbA) a.lbA[(size_t)b * NI + r] = lo;
            if (a.ubA) a.ubA[(size_t)b * NI + r] = hi;
        }
}

struct SolveArgs {
    SolveProblem P;   // per-instance pointers are offsets from these bases
    int B;
    int nfmax;
    const uint64_t *contact;  // [B] (gen_bounds) or nullptr
    size_t a_stride;          // per-instance stride of A (0 = shared)
    size_t ab_stride;         // per-instance stride of lbA/ubA (0 = shared)
    double *x, *cost, *y;
    int *status, *iters;
};

__global__ void __launch_bounds__(64) k_solve(SolveArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_b[];
    const int b = blockIdx.x;
    if (b >= a.B) return;
    SolveProblem P = a.P;
    const int nV = P.nV;
    P.H += (size_t)b * nV * nV;
    P.f += (size_t)b * nV;
    if (P.lb) P.lb += (size_t)b * nV;
    if (P.ub) P.ub += (size_t)b * nV;
    if (P.A) P.A += (size_t)b * a.a_stride;
    if (P.lbA) P.lbA += (size_t)b * a.ab_stride;
    if (P.ubA) P.ubA += (size_t)b * a.ab_stride;
    if (a.contact) P.contact = a.contact[b];
    SolveOut O;
    O.x = a.x + (size_t)b * nV;
    O.cost = a.cost + b;
    O.status = a.status + b;
    O.iters = a.iters + b;
    O.y = a.y ? a.y + (size_t)b * (nV + P.mA) : nullptr;
    wave_gi_solve(P, O, smem_b, a.nfmax);
}

__device__ __forceinline__ unsigned long long order_bits(float c) {
    const unsigned u = __float_as_uint(c);
    return (u & 0x80000000u) ? (unsigned long long)(~u) : (unsigned long long)(u | 0x80000000u);
}

// One launch: each block reduces its grid-stride share to a partial key, the last block to
// finish (ticket from a device-scope counter) reduces the partials into *key and re-arms the
// counter for the next call on this context's stream.  No pre-fill launch of the key; an
// empty batch (B = 0, one block) yields the no-valid-instance key 0x7fffffffffffffff.
constexpr int kSelMaxBlocks = 1024;
// the context's selection words: [0, kSelMaxBlocks) k_select_min partials, then its ticket,
// then the fused selection's key slots (armed to kSelNone) and ticket (MpcArgs::sel,
// sel_commit in mpc_fused.hpp)
constexpr int kFusedSel = kSelMaxBlocks + 1;
constexpr int kSelCtxWords = kFusedSel + kSelWords;
// instances per block (4 per thread): 64 blocks at B = 65,536 take 8.6 us, 256 blocks 10.9 us
constexpr int kSelPerBlock = 1024;
__global__ void __launch_bounds__(256) k_select_min(int B, const double *cost, const int *status,
                                                     long long base, unsigned long long *key,
                                                     unsigned long long *partial,
                                                     unsigned int *ticket, const double *U,
                                                     int nV, double *rec_u) {
    __shared__ unsigned long long red[4];
    __shared__ bool last;
    __shared__ unsigned long long win;
    unsigned long long best = 0x7fffffffffffffffull;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B; i += gridDim.x * blockDim.x) {
        if (status[i] != 0) continue;
        const unsigned long long k =
            (order_bits((float)cost[i]) << 31) | ((unsigned long long)(base + i) & 0x7fffffffull);
        best = k < best ? k : best;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(best, o, 64);
        best = t < best ? t : best;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = red[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = red[w] < m ? red[w] : m;
        __hip_atomic_store(&partial[blockIdx.x], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        last = t == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    best = 0x7fffffffffffffffull;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x) {
        const unsigned long long v =
            __hip_atomic_load(&partial[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        best = v < best ? v : best;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(best, o, 64);
        best = t < best ? t : best;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long m = red[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) m = red[w] < m ? red[w] : m;
        *key = m;
        win = m;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!rec_u) return;
    // selection record: the winner's U row after the key (zeros when no instance is valid)
    __syncthreads();
    const unsigned long long m = win;
    const bool none = m == 0x7fffffffffffffffull;
    const long long li = none ? 0 : (long long)(m & 0x7fffffffull) - (base & 0x7fffffffll);
    for (int e = threadIdx.x; e < nV; e += blockDim.x)
        rec_u[e] = none ? 0.0 : U[(size_t)li * nV + e];
}

// Global selection over n gathered records [key | U(nV)] (one per rank, after one all-gather):
// the minimum key's record is copied to `best`.  Keys carry the global index, so they are
// distinct unless invalid (0x7fff...); an all-invalid set yields that key and the first
// record's U, which is all zeros by construction of k_select_min.
__global__ void __launch_bounds__(64) k_reduce_records(int n, int nV, const long long *rec,
                                                       long long *best) {
    __shared__ int who;
    unsigned long long k = 0x7fffffffffffffffull;
    int idx = 0;
    for (int r = threadIdx.x; r < n; r += 64) {
        const unsigned long long v = (unsigned long long)rec[(size_t)r * (nV + 1)];
        if (v < k) { k = v; idx = r; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(k, o, 64);
        const int ti = __shfl_xor(idx, o, 64);
        if (t < k || (t == k && ti < idx)) { k = t; idx = ti; }
    }
    if (threadIdx.x == 0) who = idx;
    __syncthreads();
    const long long *src = rec + (size_t)who * (nV + 1);
    for (int e = threadIdx.x; e <= nV; e += 64) best[e] = src[e];
}

__global__ void __launch_bounds__(64) k_plant(int nx, int nu, const double *Ad, const double *Bd,
                                              double *x, const double *u) {
    __shared__ double xs[MPCQP_MAX_NX];
    const int i = threadIdx.x;
    if (i < nx) xs[i] = x[i];
    __syncthreads();
    if (i < nx) {
        double s = 0.0, t = 0.0;
        for (int l = 0; l < nx; ++l) s += Ad[l * nx + i] * xs[l];
        for (int l = 0; l < nu; ++l) t += Bd[l * nx + i] * u[l];
        x[i] = s + t;
    }
}

// linear_mpc_example's numerically integrated Bd (src/linear_mpc_example.cpp:35-46):
//   Bd = sum_{i<100} Ad (I - Ac tau_i / 100)^-1 Bc Ts/100,  tau_i = i Ts / 100
// (the reference divides by `steps` twice; kept).  One wave: lane j owns column j of the
// augmented [W | Bc] for the partial-pivot elimination, then lane (r, c) accumulates
// (Ad X)(r, c).  Ad comes from the Pade path (k_condense).
__global__ void __launch_bounds__(64) k_quad_bd(int nx, int nu, double Ts, const double *Ac,
                                                const double *Bc, const double *Ad, double *Bd) {
    __shared__ double W[MPCQP_MAX_NX * (MPCQP_MAX_NX + MPCQP_MAX_NU)];
    __shared__ double acc[MPCQP_MAX_NX * MPCQP_MAX_NU];
    const int ln = threadIdx.x, nc = nx + nu, steps = 100;
    for (int e = ln; e < nx * nu; e += 64) acc[e] = 0.0;
    for (int i = 0; i < steps; ++i) {
        const double tau = i * Ts / steps;
        __syncthreads();
        for (int e = ln; e < nx * nc; e += 64) {  // W column-major nx x nc
            const int r = e % nx, c = e / nx;
            double v;
            if (c < nx) v = -Ac[c * nx + r] * tau / steps + (r == c ? 1.0 : 0.0);
            else v = Bc[(c - nx) * nx + r];
            W[e] = v;
        }
        __syncthreads();
        for (int k = 0; k < nx; ++k) {
            int p = k;
            double amax = fabs(W[k * nx + k]);
            for (int r = k + 1; r < nx; ++r) {
                const double v = fabs(W[k * nx + r]);
                if (v > amax) { amax = v; p = r; }
            }
            const double piv = W[k * nx + p];
            __syncthreads();
            if (ln < nc && p != k) {
                const double t = W[ln * nx + k];
                W[ln * nx + k] = W[ln * nx + p];
                W[ln * nx + p] = t;
            }
            __syncthreads();
            if (ln > k && ln < nc)
                for (int r = k + 1; r < nx; ++r) W[ln * nx + r] -= (W[k * nx + r] / piv) * W[ln * nx + k];
            __syncthreads();
        }
        if (ln >= nx && ln < nc) {  // back substitution of RHS column ln - nx
            for (int r = nx - 1; r >= 0; --r) {
                double sum = W[ln * nx + r];
                for (int l = r + 1; l < nx; ++l) sum -= W[l * nx + r] * W[ln * nx + l];
                W[ln * nx + r] = sum / W[r * nx + r];
            }
        }
        __syncthreads();
        for (int e = ln; e < nx * nu; e += 64) {
            const int r = e % nx, c = e / nx;
            double sum = 0.0;
            for (int l = 0; l < nx; ++l) sum += Ad[l * nx + r] * W[(nx + c) * nx + l];
            acc[e] += sum * (Ts / steps);
        }
    }
    __syncthreads();
    for (int e = ln; e < nx * nu; e += 64) Bd[e] = acc[e];
}

// best of each state's C gait candidates: (fp32 cost order bits, candidate) minimum, the same
// rule as k_select_min; U row copied out.  One wave per state, C <= 64.
__global__ void __launch_bounds__(64) k_select_state(int S, int C, int nV, const double *cost,
                                                     const int *status, const double *U,
                                                     int *best, double *best_cost, double *Ubest) {
    const int s = blockIdx.x, c = threadIdx.x;
    if (s >= S) return;
    const size_t b = (size_t)s * C + c;
    unsigned long long k = 0x7fffffffffffffffull;
    if (c < C && status[b] == 0) k = (order_bits((float)cost[b]) << 31) | (unsigned)c;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(k, o, 64);
        k = t < k ? t : k;
    }
    const int w = (k == 0x7fffffffffffffffull) ? -1 : (int)(k & 0x7fffffffull);
    if (c == 0) {
        best[s] = w;
        if (best_cost) best_cost[s] = w >= 0 ? cost[(size_t)s * C + w] : INFINITY;
    }
    if (Ubest)
        for (int i = c; i < nV; i += 64)
            Ubest[(size_t)s * nV + i] = w >= 0 ? U[((size_t)s * C + w) * nV + i] : 0.0;
}

// SRBM plant step of each state with its chosen first-step forces:
// x <- Ad x + Bd u = x + A x + A^2 x / 2 + B u + A B u / 2 (A = Ac Ts, B = Bc Ts, the exact ZOH
// of the nilpotent model, as in k_mpc); stance feet stay fixed in the world, so both lever
// arms move by -(p+ - p); every candidate's gait phase advances by Ts.
struct PlantArgs {
    int S, C, nV;
    double Ts, mass;
    double Ibinv[9];
    double *state, *feet, *phase;
    const double *Ubest;
    const int *best;  // states with no solved candidate keep u = 0
};

__global__ void __launch_bounds__(64) k_plant_srbm(PlantArgs a) {
    constexpr int NX = 13, NS = 19;
    __shared__ double T[NX * NS], xs[NX], us[6], ax[NX], bu[NX];
    const int s = blockIdx.x, ln = threadIdx.x;
    if (s >= a.S) return;
    double lin[8];
    lin[0] = a.state[(size_t)s * NX + 2];
#pragma unroll
    for (int i = 0; i < 6; ++i) lin[1 + i] = a.feet[(size_t)s * 6 + i];
    lin[7] = 0.0;
    double cy, sy, Iwi[9];
    srbm_rot_inertia(lin[0], a.Ibinv, cy, sy, Iwi);
    if (ln < NX) {
#pragma unroll
        for (int j = 0; j < NS; ++j) T[j * NX + ln] = srbm_entry(ln, j, lin, cy, sy, Iwi, a.mass);
        xs[ln] = a.state[(size_t)s * NX + ln];
    }
    if (ln < 6) us[ln] = (a.best[s] >= 0) ? a.Ubest[(size_t)s * a.nV + ln] : 0.0;
    __syncthreads();
    if (ln < NX) {
        double p = 0.0, q = 0.0;
        for (int k = 0; k < NX; ++k) p += T[k * NX + ln] * xs[k];
        for (int c = 0; c < 6; ++c) q += T[(NX + c) * NX + ln] * us[c];
        ax[ln] = p * a.Ts;
        bu[ln] = q * a.Ts;
    }
    __syncthreads();
    double xn = 0.0;
    if (ln < NX) {
        double p = 0.0, q = 0.0;
        for (int k = 0; k < NX; ++k) {
            p += T[k * NX + ln] * ax[k];
            q += T[k * NX + ln] * bu[k];
        }
        xn = xs[ln] + ax[ln] + 0.5 * (p * a.Ts) + bu[ln] + 0.5 * (q * a.Ts);
        a.state[(size_t)s * NX + ln] = xn;
    }
    __syncthreads();
    if (ln >= 3 && ln < 6) ax[ln] = xn - xs[ln];  // CoM displacement (reuse ax)
    __syncthreads();
    if (ln < 6) a.feet[(size_t)s * 6 + ln] -= ax[3 + ln % 3];
    for (int c = ln; c < a.C; c += 64) a.phase[(size_t)s * a.C + c] += a.Ts;
}

// MPCQP_PAIR=0 in the environment keeps the one-QP-per-wave kernel (A/B measurements)
bool pair_enabled() {
    const char *e = getenv("MPCQP_PAIR");
    return !(e && e[0] == '0');
}

// instantiated configurations (BASELINE configs A/B/C and the literal model); anything else
// runs the generic runtime-dimension kernels
// The one-wave kernel is sized for min(nfmax, 64) free variables; an SRBM context whose nfmax
// exceeds what its one-wave kernel holds (30 for the paired kernel, NF for k_mpc) also gets the
// workgroup kernel (fast_wg.hip) for the instances beyond it (the overflow list).
bool pick_fast(int model, int nx, int nu, int N, bool fric, int nfmax, FastKernels &k) {
    if (nx != 13) return false;
    bool found = false;
    const int nprim = std::min(nfmax, 64);
    if (model == MPCQP_MODEL_SRBM && nu == 6) {
        if (N == 10) found = pick_fast_srbm10(fric, nprim, k);
        if (N == 20) found = pick_fast_srbm20(fric, nprim, k);
    }
    if (model == MPCQP_MODEL_LITERAL && nu == 3 && !fric) found = pick_fast_literal(N, nprim, k);
    if (found && pair_enabled()) add_fast_pair(model, N, fric, nprim, k);
    // MPCQP_CRASH_P=n in the environment: the paired kernel's crash start gives up after n
    // working sets (0: the plain dual loop from the unconstrained minimum; A/B runs and tests)
    if (k.pair && k.crash_k > 0)
        if (const char *e = getenv("MPCQP_CRASH_P")) k.crash_p = std::max(0, atoi(e));
    // the 4-wave build from this many instances per launch (MPCQP_PAIR_W4_MIN=n: A/B and tests;
    // 0 = never)
    if (k.pair) {
        k.pair_w4_min = kPairW4Min;
        if (const char *e = getenv("MPCQP_PAIR_W4_MIN")) k.pair_w4_min = std::max(0, atoi(e));
    }
    // (diagnostic MPCQP_PAIR_LDS_PAD=bytes: extra LDS per paired-kernel wave, i.e. fewer resident
    //  waves per CU -- the kernel's occupancy sensitivity, tools/ab_env.py; never in a measured line)
    if (k.pair)
        if (const char *e = getenv("MPCQP_PAIR_LDS_PAD")) k.pair_lds += (size_t)std::max(0, atoi(e));
    if (found) {
        k.prim_nf = k.pair ? kPairCap : k.nf;
        if (nfmax > k.prim_nf) add_fast_wg(model, N, fric, k);
    }
    // MPCQP_CRASH_P_WG=n: the same for the workgroup solver (overflow / dense kernels)
    if (k.crash_k_wg > 0)
        if (const char *e = getenv("MPCQP_CRASH_P_WG")) k.crash_p_wg = std::max(0, atoi(e));
    return found;
}

// ------------------------------------------------------------------------------ host side
void inv3(const double *A, double *Ai) {  // same formula as the oracle's model builder
    const double a = A[0], b = A[3], c = A[6], d = A[1], e = A[4], f = A[7], g = A[2],
                 h = A[5], i = A[8];
    const double A00 = e * i - f * h, A01 = -(d * i - f * g), A02 = d * h - e * g;
    const double det = a * A00 + b * A01 + c * A02;
    const double id = 1.0 / det;
    Ai[0] = A00 * id; Ai[3] = -(b * i - c * h) * id; Ai[6] = (b * f - c * e) * id;
    Ai[1] = A01 * id; Ai[4] = (a * i - c * g) * id;  Ai[7] = -(a * f - c * d) * id;
    Ai[2] = A02 * id; Ai[5] = -(a * h - b * g) * id; Ai[8] = (a * e - b * d) * id;
}

int hip_status(hipError_t e) { return e == hipSuccess ? MPCQP_OK : MPCQP_ERR_DEVICE; }

#define HIP_TRY(x)                                \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) { rc = MPCQP_ERR_DEVICE; goto out; } \
    } while (0)

bool have_device() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}

// scoped device buffer list for the single-instance API
struct DevBufs {
    void *p[32];
    int n = 0;
    ~DevBufs() {
        for (int i = 0; i < n; ++i) hipFree(p[i]);
    }
    template <class T>
    T *alloc(size_t count) {
        void *q = nullptr;
        if (count == 0) count = 1;
        if (hipMalloc(&q, count * sizeof(T)) != hipSuccess) return nullptr;
        p[n++] = q;
        return static_cast<T *>(q);
    }
    template <class T>
    T *upload(const T *h, size_t count) {
        if (!h) return nullptr;
        T *d = alloc<T>(count);
        if (d && hipMemcpy(d, h, count * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    }
};

size_t set_lds(const void *kernel, size_t bytes) {
    if (bytes > 64 * 1024)
        hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    return bytes;
}

}  // namespace

// ------------------------------------------------------------------------------ context
struct mpcqp_ctx {
    mpcqp_model m;
    int device;
    double *dQ = nullptr, *dR = nullptr, *dP = nullptr;
    double Ibinv[9];
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool timing = false;
    // timing (mpcqp_enable_timing): per slot a ring of begin / end event pairs, the last
    // kTimingRing launches since the last mpcqp_kernel_ms_sum (created on first enable)
    static constexpr int kTimingRing = 64;
    hipEvent_t ev[4][kTimingRing][2];
    bool ev_ok = false;
    int ev_n[4] = {0, 0, 0, 0};       // launches recorded since the last sum
    long long ev_seq[4] = {0, 0, 0, 0};  // launches recorded in total (ring position)
    double *scratchH = nullptr, *scratchF = nullptr;
    size_t scratch_cap = 0;
    // fast path
    bool fast = false;
    FastKernels fk;
    double *dqd = nullptr, *dpd = nullptr;  // diagonals of Q, P
    double *dFQ = nullptr, *dFP = nullptr;  // dense model: Q = F F', P = F F' (sym_factor)
    double *dAB = nullptr;                  // [B][nx*(nx+nu)] discretised model scratch
    size_t ab_cap = 0;
    unsigned long long *dstamps = nullptr;  // diagnostic phase cycles (stamps build)
    double *dflops = nullptr;  // diagnostic solver-flops accumulator (mpcqp_count_solver_flops)
    bool flops_on = false;
    int flops_launches = 0;
    unsigned long long *dsel = nullptr;     // k_select_min: per-block partial keys + ticket
    int *dlist = nullptr;                   // two overflow lists [count, -, ids...] (mpc_wg.hpp)
    size_t list_cap = 0;                    // instances a list holds
    int list_par = 0;                       // the list the next launch fills
    int wg_grid = 0;                        // resident workgroups of the workgroup kernel
    // host-pointer entry point (mpcqp_batch_solve_host): device staging, pinned host staging of
    // the same byte layout (one copy each way), its own stream (graph capture needs one) and
    // the instantiated graphs of the last batch size: [0] no overflow launch, [1 + parity] with
    // the overflow launch on list `parity`.  A graph holds the device addresses it was captured
    // with (staging, overflow lists, scratch): every reallocation of a context-owned device
    // buffer bumps buf_gen, and graphs captured under an older generation are dropped
    void *hbuf = nullptr;
    size_t hbuf_cap = 0;
    void *pin = nullptr;
    size_t pin_cap = 0;
    hipStream_t hstream = nullptr;
    hipEvent_t hev = nullptr;
    // the direct host path (the caller's page-locked arrays): copy-in / copy-out streams and the
    // per-chunk "inputs landed" / "solved" events of the pipeline (created on first use)
    hipStream_t hs_in = nullptr, hs_out = nullptr;
    hipEvent_t hev_in[8] = {}, hev_k[8] = {};
    bool hd_ok = false;
    bool hd_off = false;  // MPCQP_HOST_DIRECT=0: always stage (A/B of the direct path)
    int hg_B = 0;
    unsigned long long buf_gen = 0, hg_gen = 0;
    hipGraphExec_t hg_exec[3] = {nullptr, nullptr, nullptr};
    bool hg_off = false;  // capture failed once: run the host path uncaptured
    // closed-loop rollout workspace
    void *rbuf = nullptr;
    size_t rbuf_cap = 0;
    void *fkbuf = nullptr;  // mpcqp_ctx_fk_feet_host staging
    size_t fkbuf_cap = 0;
    void *dwarm = nullptr;  // warm start: per-instance active-set words (gi_reg.hpp WarmSet)
    size_t warm_cap = 0;
    int warm_on = 0, warm_fresh = 0;
};

extern "C" {

#ifndef MPCQP_BUILD_ID
#define MPCQP_BUILD_ID "unversioned"
#endif
// A/B variant builds (tools/build_variants.sh) recompile one translation unit with extra -D
// flags and relink it with the release objects; that unit then defines the strong
// mpcqp_variant_tag_fn (fast_kernels.hpp), so the id of a variant library names its flags
__attribute__((weak)) const char *mpcqp_variant_tag_fn(void) { return ""; }

const char *mpcqp_build_id(void) {
    static char id[96];
    if (!id[0]) {
        const char *v = mpcqp_variant_tag_fn();
        snprintf(id, sizeof id, "%s%s%s", MPCQP_BUILD_ID, v[0] ? "+" : "", v);
    }
    return id;
}

const char *mpcqp_status_string(int s) {
    switch (s) {
        case MPCQP_OK: return "OK";
        case MPCQP_ERR_BAD_DIMS: return "bad dimensions";
        case MPCQP_ERR_INFEASIBLE: return "infeasible";
        case MPCQP_ERR_ITER_LIMIT: return "iteration limit";
        case MPCQP_ERR_NOT_PD: return "Hessian not positive definite";
        case MPCQP_ERR_DEVICE: return "HIP device error";
        case MPCQP_ERR_BAD_ARG: return "bad argument";
        case MPCQP_ERR_NO_DEVICE: return "no HIP device";
        default: return "unknown";
    }
}

int mpcqp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

static int check_dims(int nx, int nu, int N) {
    if (nx <= 0 || nu <= 0 || N <= 0 || nx > MPCQP_MAX_NX || nu > MPCQP_MAX_NU || N > MPCQP_MAX_N ||
        nu * N > MPCQP_MAX_NV)
        return MPCQP_ERR_BAD_DIMS;
    return MPCQP_OK;
}

static ModelConst make_mc(int nx, int nu, int N, int model, double Ts, double mass,
                          const double *Ibinv, const double *Q, const double *R, const double *P) {
    ModelConst mc;
    mc.nx = nx; mc.nu = nu; mc.N = N; mc.nV = nu * N; mc.ns = nx + nu;
    mc.model = model; mc.Ts = Ts; mc.mass = mass;
    for (int i = 0; i < 9; ++i) mc.Ibinv[i] = Ibinv ? Ibinv[i] : 0.0;
    mc.Q = Q; mc.R = R; mc.P = P;
    return mc;
}

int mpcqp_discretize(int nx, int nu, double Ts, const double *Ac, const double *Bc, double *Ad,
                     double *Bd) {
    if (!Ac || !Bc || !Ad || !Bd) return MPCQP_ERR_BAD_ARG;
    if (nx <= 0 || nu <= 0 || nx > MPCQP_MAX_NX || nu > MPCQP_MAX_NU) return MPCQP_ERR_BAD_DIMS;
    if (!have_device()) return MPCQP_ERR_NO_DEVICE;
    int rc = MPCQP_OK;
    DevBufs bufs;
    const int ns = nx + nu;
    CondenseArgs a;
    memset(&a, 0, sizeof(a));
    a.mc = make_mc(nx, nu, 1, 2, Ts, 1.0, nullptr, nullptr, nullptr, nullptr);
    a.B = 1;
    a.Ac = bufs.upload(Ac, (size_t)nx * nx);
    a.Bc = bufs.upload(Bc, (size_t)nx * nu);
    a.ABout = bufs.alloc<double>((size_t)nx * ns);
    a.discretize_only = 1;
    if (!a.Ac || !a.Bc || !a.ABout) return MPCQP_ERR_DEVICE;
    {
        const size_t lds = set_lds((const void *)k_condense,
                                   sizeof(double) * condense_lds_doubles(nx, nu, 1));
        hipLaunchKernelGGL(k_condense, dim3(1), dim3(64), lds, 0, a);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(Ad, a.ABout, sizeof(double) * nx * nx, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(Bd, a.ABout + nx * nx, sizeof(double) * nx * nu, hipMemcpyDeviceToHost));
    }
out:
    return rc;
}

int mpcqp_discretize_quadrature(int nx, int nu, double Ts, const double *Ac, const double *Bc,
                                double *Ad, double *Bd) {
    if (!Ac || !Bc || !Ad || !Bd) return MPCQP_ERR_BAD_ARG;
    if (nx <= 0 || nu <= 0 || nx > MPCQP_MAX_NX || nu > MPCQP_MAX_NU || nx + nu > 64)
        return MPCQP_ERR_BAD_DIMS;
    int rc = mpcqp_discretize(nx, nu, Ts, Ac, Bc, Ad, Bd);  // Ad = exp(Ac Ts) (Pade path)
    if (rc) return rc;
    DevBufs bufs;
    double *dAc = bufs.upload(Ac, (size_t)nx * nx), *dBc = bufs.upload(Bc, (size_t)nx * nu);
    double *dAd = bufs.upload(Ad, (size_t)nx * nx), *dBd = bufs.alloc<double>((size_t)nx * nu);
    if (!dAc || !dBc || !dAd || !dBd) return MPCQP_ERR_DEVICE;
    hipLaunchKernelGGL(k_quad_bd, dim3(1), dim3(64), 0, 0, nx, nu, Ts, dAc, dBc, dAd, dBd);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(Bd, dBd, sizeof(double) * nx * nu, hipMemcpyDeviceToHost));
out:
    return rc;
}

int mpcqp_build_qp(int nx, int nu, int N, const double *Ad, const double *Bd, const double *Q,
                   const double *R, const double *P, const double *x_min, const double *x_max,
                   double u_min, double u_max, const double *xi0, const double *xi_ref,
                   double *H, double *f, double *A_eq, double *b_eq, double *lb, double *ub,
                   double *A_ineq, double *lbA, double *ubA) {
    if (!Ad || !Bd || !Q || !R || !P || !xi0 || !xi_ref) return MPCQP_ERR_BAD_ARG;
    if ((lbA || ubA) && (!x_min || !x_max)) return MPCQP_ERR_BAD_ARG;
    int rc = check_dims(nx, nu, N);
    if (rc) return rc;
    if (!have_device()) return MPCQP_ERR_NO_DEVICE;
    DevBufs bufs;
    const int ns = nx + nu, nV = nu * N, NE = nx * N, NI = 2 * nx * N;
    double *AB = (double *)malloc(sizeof(double) * nx * ns);
    memcpy(AB, Ad, sizeof(double) * nx * nx);
    memcpy(AB + nx * nx, Bd, sizeof(double) * nx * nu);
    CondenseArgs a;
    memset(&a, 0, sizeof(a));
    const double *dQ = bufs.upload(Q, (size_t)nx * nx), *dR = bufs.upload(R, (size_t)nu * nu),
                 *dP = bufs.upload(P, (size_t)nx * nx);
    a.mc = make_mc(nx, nu, N, 2, 0.0, 1.0, nullptr, dQ, dR, dP);
    a.B = 1;
    a.ABin = bufs.upload(AB, (size_t)nx * ns);
    free(AB);
    a.x0 = bufs.upload(xi0, (size_t)nx);
    a.xref = bufs.upload(xi_ref, (size_t)nx * (N + 1));
    a.H = bufs.alloc<double>((size_t)nV * nV);
    a.f = bufs.alloc<double>((size_t)nV);
    a.x_min = bufs.upload(x_min, (size_t)nx);
    a.x_max = bufs.upload(x_max, (size_t)nx);
    a.u_min = u_min;
    a.u_max = u_max;
    a.A_eq = A_eq ? bufs.alloc<double>((size_t)NE * nV) : nullptr;
    a.b_eq = b_eq ? bufs.alloc<double>((size_t)NE) : nullptr;
    a.lb = lb ? bufs.alloc<double>((size_t)nV) : nullptr;
    a.ub = ub ? bufs.alloc<double>((size_t)nV) : nullptr;
    a.A_ineq = A_ineq ? bufs.alloc<double>((size_t)NI * nV) : nullptr;
    a.lbA = lbA ? bufs.alloc<double>((size_t)NI) : nullptr;
    a.ubA = ubA ? bufs.alloc<double>((size_t)NI) : nullptr;
    if (!dQ || !dR || !dP || !a.ABin || !a.x0 || !a.xref || !a.H || !a.f) return MPCQP_ERR_DEVICE;
    {
        const size_t lds = set_lds((const void *)k_condense,
                                   sizeof(double) * condense_lds_doubles(nx, nu, N));
        hipLaunchKernelGGL(k_condense, dim3(1), dim3(64), lds, 0, a);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipDeviceSynchronize());
        if (H) HIP_TRY(hipMemcpy(H, a.H, sizeof(double) * nV * nV, hipMemcpyDeviceToHost));
        if (f) HIP_TRY(hipMemcpy(f, a.f, sizeof(double) * nV, hipMemcpyDeviceToHost));
        if (A_eq) HIP_TRY(hipMemcpy(A_eq, a.A_eq, sizeof(double) * NE * nV, hipMemcpyDeviceToHost));
        if (b_eq) HIP_TRY(hipMemcpy(b_eq, a.b_eq, sizeof(double) * NE, hipMemcpyDeviceToHost));
        if (lb) HIP_TRY(hipMemcpy(lb, a.lb, sizeof(double) * nV, hipMemcpyDeviceToHost));
        if (ub) HIP_TRY(hipMemcpy(ub, a.ub, sizeof(double) * nV, hipMemcpyDeviceToHost));
        if (A_ineq) HIP_TRY(hipMemcpy(A_ineq, a.A_ineq, sizeof(double) * NI * nV, hipMemcpyDeviceToHost));
        if (lbA) HIP_TRY(hipMemcpy(lbA, a.lbA, sizeof(double) * NI, hipMemcpyDeviceToHost));
        if (ubA) HIP_TRY(hipMemcpy(ubA, a.ubA, sizeof(double) * NI, hipMemcpyDeviceToHost));
    }
out:
    return rc;
}

int mpcqp_solve_dense(int nV, int nC, const double *H, const double *f, const double *A,
                      int a_layout, const double *lb, const double *ub, const double *lbA,
                      const double *ubA, int *nWSR, double *x, double *y, double *cost) {
    if (!H || !f || !x || (nC > 0 && !A)) return MPCQP_ERR_BAD_ARG;
    if (a_layout != MPCQP_A_ROWMAJOR && a_layout != MPCQP_A_COLMAJOR) return MPCQP_ERR_BAD_ARG;
    if (nV <= 0 || nV > MPCQP_MAX_NV || nC < 0 || nC > 4096) return MPCQP_ERR_BAD_DIMS;
    if (!have_device()) return MPCQP_ERR_NO_DEVICE;
    int rc = MPCQP_OK;
    DevBufs bufs;
    // free-variable count decides the LDS size; fixed variables (lb == ub) are eliminated
    int nfree = 0;
    for (int i = 0; i < nV; ++i) {
        const double lo = lb ? lb[i] : -MPCQP_INFTY, hi = ub ? ub[i] : MPCQP_INFTY;
        if (lo != hi) ++nfree;
    }
    if (nfree > kWave) return MPCQP_ERR_BAD_DIMS;  // the one-wave dense solver
    const int nfmax = std::max(1, nfree);
    SolveArgs a;
    memset(&a, 0, sizeof(a));
    a.B = 1;
    a.nfmax = nfmax;
    a.P.nV = nV;
    a.P.H = bufs.upload(H, (size_t)nV * nV);
    a.P.f = bufs.upload(f, (size_t)nV);
    a.P.lb = bufs.upload(lb, (size_t)nV);
    a.P.ub = bufs.upload(ub, (size_t)nV);
    a.P.mA = nC;
    a.P.A = nC ? bufs.upload(A, (size_t)nC * nV) : nullptr;
    a.P.a_colmajor = a_layout == MPCQP_A_COLMAJOR;
    a.P.lbA = nC ? bufs.upload(lbA, (size_t)nC) : nullptr;
    a.P.ubA = nC ? bufs.upload(ubA, (size_t)nC) : nullptr;
    a.P.max_iter = (nWSR && *nWSR > 0) ? *nWSR : 0;
    double *dx = bufs.alloc<double>(nV), *dc = bufs.alloc<double>(1);
    int *ds = bufs.alloc<int>(1), *di = bufs.alloc<int>(1);
    double *dy = y ? bufs.alloc<double>((size_t)nV + nC) : nullptr;
    a.x = dx; a.cost = dc; a.status = ds; a.iters = di; a.y = dy;
    if (!a.P.H || !a.P.f || !dx || !dc || !ds || !di) return MPCQP_ERR_DEVICE;
    if (nC && (!a.P.A)) return MPCQP_ERR_DEVICE;
    {
        const size_t lds = set_lds((const void *)k_solve, gi_lds_bytes(nfmax, nV, nC, 0));
        int st = 0, it = 0;
        double c = 0.0;
        hipLaunchKernelGGL(k_solve, dim3(1), dim3(64), lds, 0, a);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpy(x, dx, sizeof(double) * nV, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&st, ds, sizeof(int), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&it, di, sizeof(int), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(&c, dc, sizeof(double), hipMemcpyDeviceToHost));
        if (y) HIP_TRY(hipMemcpy(y, dy, sizeof(double) * (nV + nC), hipMemcpyDeviceToHost));
        if (nWSR) *nWSR = it;
        if (cost) *cost = c;
        rc = st;
    }
out:
    return rc;
}

int mpcqp_plant_step(int nx, int nu, const double *Ad, const double *Bd, double *x,
                     const double *u) {
    if (!Ad || !Bd || !x || !u) return MPCQP_ERR_BAD_ARG;
    if (nx <= 0 || nu <= 0 || nx > MPCQP_MAX_NX || nu > MPCQP_MAX_NU) return MPCQP_ERR_BAD_DIMS;
    if (!have_device()) return MPCQP_ERR_NO_DEVICE;
    int rc = MPCQP_OK;
    DevBufs bufs;
    const double *dA = bufs.upload(Ad, (size_t)nx * nx), *dB = bufs.upload(Bd, (size_t)nx * nu),
                 *du = bufs.upload(u, (size_t)nu);
    double *dx = bufs.upload(x, (size_t)nx);
    if (!dA || !dB || !du || !dx) return MPCQP_ERR_DEVICE;
    hipLaunchKernelGGL(k_plant, dim3(1), dim3(64), 0, 0, nx, nu, dA, dB, dx, du);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpy(x, dx, sizeof(double) * nx, hipMemcpyDeviceToHost));
out:
    return rc;
}

// ------------------------------------------------------------------------- batched path
// F (n x n, column-major) with M = F F' for a symmetric positive semi-definite M: the square
// roots of a diagonal M, otherwise cyclic Jacobi M = V L V' and F = V L^(1/2).  false if M is
// not symmetric, has an eigenvalue below -1e-12 max |eigenvalue| or Jacobi does not converge
// (the dense kernel then keeps the recursion, which takes any Q and P)
static bool sym_factor(const double *M, int n, double *F) {
    double mx = 0.0;
    for (int i = 0; i < n * n; ++i) mx = std::max(mx, std::fabs(M[i]));
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < j; ++i)
            if (std::fabs(M[j * n + i] - M[i * n + j]) > 1e-14 * mx) return false;
    bool diag = true;
    for (int j = 0; j < n && diag; ++j)
        for (int i = 0; i < n; ++i)
            if (i != j && M[j * n + i] != 0.0) { diag = false; break; }
    std::vector<double> A(M, M + (size_t)n * n), V((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) V[(size_t)i * n + i] = 1.0;
    if (!diag) {
        bool converged = false;
        for (int sweep = 0; sweep <= 64 && !converged; ++sweep) {
            double off = 0.0;
            for (int q = 0; q < n; ++q)
                for (int p = 0; p < q; ++p) off += A[(size_t)q * n + p] * A[(size_t)q * n + p];
            if (off <= 1e-32 * mx * mx) { converged = true; break; }
            if (sweep == 64) break;  // (the off-diagonal test of the 64th sweep's result)
            for (int q = 1; q < n; ++q)
                for (int p = 0; p < q; ++p) {
                    const double apq = A[(size_t)q * n + p];
                    if (apq == 0.0) continue;
                    const double app = A[(size_t)p * n + p], aqq = A[(size_t)q * n + q];
                    const double th = (aqq - app) / (2.0 * apq);
                    const double t = (th >= 0 ? 1.0 : -1.0) / (std::fabs(th) + std::sqrt(th * th + 1.0));
                    const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
                    for (int k = 0; k < n; ++k) {  // A <- J' A J, columns then rows
                        const double akp = A[(size_t)p * n + k], akq = A[(size_t)q * n + k];
                        A[(size_t)p * n + k] = c * akp - sn * akq;
                        A[(size_t)q * n + k] = sn * akp + c * akq;
                    }
                    for (int k = 0; k < n; ++k) {
                        const double apk = A[(size_t)k * n + p], aqk = A[(size_t)k * n + q];
                        A[(size_t)k * n + p] = c * apk - sn * aqk;
                        A[(size_t)k * n + q] = sn * apk + c * aqk;
                    }
                    for (int k = 0; k < n; ++k) {
                        const double vkp = V[(size_t)p * n + k], vkq = V[(size_t)q * n + k];
                        V[(size_t)p * n + k] = c * vkp - sn * vkq;
                        V[(size_t)q * n + k] = sn * vkp + c * vkq;
                    }
                }
        }
        // not diagonalised to the tolerance in 64 sweeps: F F' would not be M -- keep the
        // recursion path, which takes any Q and P
        if (!converged) return false;
    }
    double lmax = 0.0;
    for (int i = 0; i < n; ++i) lmax = std::max(lmax, std::fabs(A[(size_t)i * n + i]));
    for (int k = 0; k < n; ++k) {
        const double l = A[(size_t)k * n + k];
        if (l < -1e-12 * lmax) return false;
        const double sl = l > 0.0 ? std::sqrt(l) : 0.0;
        for (int i = 0; i < n; ++i) F[(size_t)k * n + i] = V[(size_t)k * n + i] * sl;
    }
    return true;
}

static bool is_diag(const double *M, int n) {
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i)
            if (i != j && M[j * n + i] != 0.0) return false;
    return true;
}

// initial selection words: k_select_min's partials and ticket 0, the fused key slots armed to
// kSelNone, the fused ticket 0
static std::vector<unsigned long long> sel_words_armed() {
    std::vector<unsigned long long> w((size_t)kSelCtxWords, 0ull);
    for (int s = 0; s < kSelSlots; ++s) w[(size_t)(kFusedSel + s * kSelStride)] = kSelNone;
    return w;
}

int mpcqp_ctx_create(const mpcqp_model *m, int device, mpcqp_ctx **out) {
    if (!m || !out || !m->Q || !m->R || !m->P) return MPCQP_ERR_BAD_ARG;
    *out = nullptr;
    int rc = check_dims(m->nx, m->nu, m->N);
    if (rc) return rc;
    if (m->model == MPCQP_MODEL_SRBM && (m->nx != 13 || m->nu != 6)) return MPCQP_ERR_BAD_DIMS;
    if (m->model == MPCQP_MODEL_LITERAL && (m->nx != 13 || m->nu != 3)) return MPCQP_ERR_BAD_DIMS;
    if (m->model != MPCQP_MODEL_SRBM && m->model != MPCQP_MODEL_LITERAL &&
        m->model != MPCQP_MODEL_DENSE)
        return MPCQP_ERR_BAD_ARG;
    if (m->model == MPCQP_MODEL_DENSE && !(m->u_min < m->u_max)) return MPCQP_ERR_BAD_ARG;
    // literal model: every input is free (u_min < u_max); the fused kernels read a fixed input
    // as 0, which an empty box (u_min == u_max) would contradict
    if (m->model == MPCQP_MODEL_LITERAL && !(m->u_min < m->u_max)) return MPCQP_ERR_BAD_ARG;
    if (m->constraints != MPCQP_CONS_BOX && m->constraints != MPCQP_CONS_FRICTION)
        return MPCQP_ERR_BAD_ARG;
    const int nfmax = m->max_free > 0 ? m->max_free : m->nu * m->N;
    if (nfmax > MPCQP_MAX_FREE) return MPCQP_ERR_BAD_DIMS;
    if (!have_device()) return MPCQP_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return MPCQP_ERR_DEVICE;
    mpcqp_ctx *c = new (std::nothrow) mpcqp_ctx();
    if (!c) return MPCQP_ERR_DEVICE;
    c->m = *m;
    c->device = device;
    if (const char *e = getenv("MPCQP_HOST_DIRECT")) c->hd_off = atoi(e) == 0;
    inv3(m->Ib, c->Ibinv);
    const int nx = m->nx, nu = m->nu;
    double qd[MPCQP_MAX_NX], pd[MPCQP_MAX_NX];
    for (int i = 0; i < nx; ++i) { qd[i] = m->Q[i * nx + i]; pd[i] = m->P[i * nx + i]; }
    if (hipMalloc(&c->dQ, sizeof(double) * nx * nx) != hipSuccess ||
        hipMalloc(&c->dR, sizeof(double) * nu * nu) != hipSuccess ||
        hipMalloc(&c->dP, sizeof(double) * nx * nx) != hipSuccess ||
        hipMalloc(&c->dqd, sizeof(double) * nx) != hipSuccess ||
        hipMalloc(&c->dpd, sizeof(double) * nx) != hipSuccess ||
        hipMemcpy(c->dQ, m->Q, sizeof(double) * nx * nx, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->dR, m->R, sizeof(double) * nu * nu, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->dP, m->P, sizeof(double) * nx * nx, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->dqd, qd, sizeof(double) * nx, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->dpd, pd, sizeof(double) * nx, hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc(&c->dsel, sizeof(unsigned long long) * kSelCtxWords) != hipSuccess ||
        hipMemcpy(c->dsel, sel_words_armed().data(), sizeof(unsigned long long) * kSelCtxWords,
                  hipMemcpyHostToDevice) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        mpcqp_ctx_destroy(c);
        return MPCQP_ERR_DEVICE;
    }
    c->own_stream = true;
    // fast path: compile-time dims, diagonal Q/P (the reference's asDiagonal() weights,
    // include/mpcQP.h:54-56), and in-contact forces never fixed (so fixed inputs are 0)
    const bool fric = m->model == MPCQP_MODEL_SRBM && m->constraints == MPCQP_CONS_FRICTION;
    const bool bounds_ok = m->model == MPCQP_MODEL_LITERAL ||
                           (m->fz_min < m->fz_max && m->fxy_max > 0.0);
    c->fast = m->model != MPCQP_MODEL_DENSE && is_diag(m->Q, nx) && is_diag(m->P, nx) &&
              bounds_ok && nu <= 6 && pick_fast(m->model, nx, nu, m->N, fric, nfmax, c->fk);
    if (m->model == MPCQP_MODEL_DENSE && nfmax <= 128) {
        // dense Q/R/P allowed: the kernel reads them whole; symmetric PSD Q and P are factored
        // for the Toeplitz condensing (dense_wg.hpp)
        std::vector<double> fq((size_t)nx * nx), fp((size_t)nx * nx);
        bool toep = sym_factor(m->Q, nx, fq.data()) && sym_factor(m->P, nx, fp.data());
        if (toep && (hipMalloc(&c->dFQ, sizeof(double) * nx * nx) != hipSuccess ||
                     hipMalloc(&c->dFP, sizeof(double) * nx * nx) != hipSuccess ||
                     hipMemcpy(c->dFQ, fq.data(), sizeof(double) * nx * nx, hipMemcpyHostToDevice) != hipSuccess ||
                     hipMemcpy(c->dFP, fp.data(), sizeof(double) * nx * nx, hipMemcpyHostToDevice) != hipSuccess)) {
            mpcqp_ctx_destroy(c);
            return MPCQP_ERR_DEVICE;
        }
        if (pick_fast_dense(nx, nu, m->N, toep, c->fk)) {
            c->fast = true;
            set_lds(c->fk.dense, c->fk.dense_lds);
            if (const char *e = getenv("MPCQP_CRASH_P_WG")) c->fk.crash_p_wg = std::max(0, atoi(e));
        }
    }
    if (!c->fast && nfmax > kWave) {  // the generic one-wave solver holds 64 free variables
        mpcqp_ctx_destroy(c);
        return MPCQP_ERR_BAD_DIMS;
    }
    if (c->fast && c->fk.wg) {  // resident grid of the persistent workgroup kernels
        int dev_cus = 0, nb = 0;
        hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, device);
        set_lds(c->fk.wg, c->fk.wg_lds);
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, c->fk.wg, c->fk.wg_threads, c->fk.wg_lds);
        c->wg_grid = std::max(1, nb) * std::max(1, dev_cus);
    }
    c->m.Q = c->m.R = c->m.P = nullptr;  // host pointers are not kept
    *out = c;
    return MPCQP_OK;
}

int mpcqp_ctx_fast_path(const mpcqp_ctx *c) {
    if (!c || !c->fast) return 0;
    if (c->fk.dense) return 3;
    return c->fk.pair ? 2 : 1;
}

int mpcqp_ctx_overflow_kernel(const mpcqp_ctx *c) {
    if (!c || !c->fast || !c->fk.wg) return 0;
    return c->fk.wg_threads == 64 ? 1 : 2;
}

int mpcqp_ctx_one_wave_nf(const mpcqp_ctx *c) {
    if (!c || !c->fast || c->fk.dense) return 0;
    return c->fk.prim_nf;
}

int mpcqp_ctx_crash_params(const mpcqp_ctx *c, int *kmax, int *pmax, int *kmax_wg,
                           int *pmax_wg) {
    if (!c || !kmax || !pmax || !kmax_wg || !pmax_wg) return MPCQP_ERR_BAD_ARG;
    const bool on = c->fast && c->fk.pair && !c->fk.dense;
    *kmax = on ? c->fk.crash_k : 0;
    *pmax = on ? c->fk.crash_p : 0;
    const bool wg = c->fast && (c->fk.wg || c->fk.dense);
    *kmax_wg = wg ? c->fk.crash_k_wg : 0;
    *pmax_wg = wg ? c->fk.crash_p_wg : 0;
    return MPCQP_OK;
}

int mpcqp_count_solver_flops(mpcqp_ctx *c, int on) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    if (on && !c->dflops) {
        hipSetDevice(c->device);
        // (cleared on the context's stream: a later launch on it is ordered after the clear)
        if (hipMalloc(&c->dflops, sizeof(double) * kFlopsWords) != hipSuccess ||
            hipMemsetAsync(c->dflops, 0, sizeof(double) * kFlopsWords, c->stream) != hipSuccess) {
            hipFree(c->dflops);
            c->dflops = nullptr;
            return MPCQP_ERR_DEVICE;
        }
    }
    c->flops_on = on != 0;
    return MPCQP_OK;
}

double mpcqp_solver_flops(mpcqp_ctx *c, int *launches) {
    if (launches) *launches = 0;
    if (!c || !c->dflops) return -1.0;
    double h[kFlopsWords], v = 0.0;
    hipSetDevice(c->device);
    // read and cleared on the context's stream (it may be non-blocking: a null-stream clear
    // would not be ordered before the next launch's atomics)
    if (hipMemcpyAsync(h, c->dflops, sizeof h, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemsetAsync(c->dflops, 0, sizeof h, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return -1.0;
    for (int i = 0; i < kFlopsSlots; ++i) v += h[i * kFlopsStride];
    if (launches) *launches = c->flops_launches;
    c->flops_launches = 0;
    return v;
}

int mpcqp_debug_phase_cycles(mpcqp_ctx *c, uint64_t *out, int n) {
#ifdef MPCQP_STAMPS
    if (!c || !out || n <= 0) return MPCQP_ERR_BAD_ARG;
    const int slots = 16;
    if (!c->dstamps) {
        if (hipMalloc(&c->dstamps, sizeof(unsigned long long) * slots) != hipSuccess ||
            hipMemset(c->dstamps, 0, sizeof(unsigned long long) * slots) != hipSuccess)
            return MPCQP_ERR_DEVICE;
        for (int i = 0; i < n; ++i) out[i] = 0;
        return MPCQP_OK;
    }
    unsigned long long h[16];
    if (hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(h, c->dstamps, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemset(c->dstamps, 0, sizeof(h)) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    for (int i = 0; i < n; ++i) out[i] = i < slots ? h[i] : 0;
    return MPCQP_OK;
#else
    (void)c; (void)out; (void)n;
    return MPCQP_ERR_BAD_ARG;  // only the diagnostic build (libmpcqp_stamps.so) records
#endif
}

int mpcqp_ctx_destroy(mpcqp_ctx *c) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    hipFree(c->dQ);
    hipFree(c->dR);
    hipFree(c->dP);
    hipFree(c->dqd);
    hipFree(c->dpd);
    hipFree(c->dFQ);
    hipFree(c->dFP);
    hipFree(c->dAB);
    hipFree(c->dstamps);
    hipFree(c->dflops);
    hipFree(c->dsel);
    hipFree(c->dlist);
    hipFree(c->hbuf);
    for (int i = 0; i < 3; ++i)
        if (c->hg_exec[i]) hipGraphExecDestroy(c->hg_exec[i]);
    if (c->pin) hipHostFree(c->pin);
    if (c->hev) hipEventDestroy(c->hev);
    if (c->hstream) hipStreamDestroy(c->hstream);
    for (int i = 0; i < 8; ++i) {
        if (c->hev_in[i]) hipEventDestroy(c->hev_in[i]);
        if (c->hev_k[i]) hipEventDestroy(c->hev_k[i]);
    }
    if (c->hs_in) hipStreamDestroy(c->hs_in);
    if (c->hs_out) hipStreamDestroy(c->hs_out);
    hipFree(c->rbuf);
    hipFree(c->fkbuf);
    hipFree(c->dwarm);
    hipFree(c->scratchH);
    hipFree(c->scratchF);
    if (c->ev_ok)
        for (int w = 0; w < 4; ++w)
            for (int i = 0; i < mpcqp_ctx::kTimingRing; ++i)
                for (int e = 0; e < 2; ++e) hipEventDestroy(c->ev[w][i][e]);
    if (c->own_stream && c->stream) hipStreamDestroy(c->stream);
    delete c;
    return MPCQP_OK;
}

int mpcqp_set_stream(mpcqp_ctx *c, void *stream) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    if (c->own_stream && c->stream) {
        hipStreamSynchronize(c->stream);
        hipStreamDestroy(c->stream);
    }
    c->own_stream = false;
    c->stream = (hipStream_t)stream;  // NULL = the HIP null stream
    return MPCQP_OK;
}

int mpcqp_sync(mpcqp_ctx *c) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    return hip_status(hipStreamSynchronize(c->stream));
}

int mpcqp_enable_timing(mpcqp_ctx *c, int on) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    if (on && !c->ev_ok) {
        hipSetDevice(c->device);
        hipEvent_t *evs = &c->ev[0][0][0];
        constexpr int nev = 4 * mpcqp_ctx::kTimingRing * 2;
        for (int i = 0; i < nev; ++i)
            if (hipEventCreate(&evs[i]) != hipSuccess) {
                for (int j = 0; j < i; ++j) hipEventDestroy(evs[j]);  // no partial set is kept
                return MPCQP_ERR_DEVICE;
            }
        c->ev_ok = true;
    }
    c->timing = on && c->ev_ok;
    return MPCQP_OK;
}

static double ev_ms(mpcqp_ctx *c, int which, long long seq) {
    hipEvent_t *p = c->ev[which][seq % mpcqp_ctx::kTimingRing];
    float ms = -1.0f;
    if (hipEventSynchronize(p[1]) != hipSuccess) return -1.0;
    if (hipEventElapsedTime(&ms, p[0], p[1]) != hipSuccess) return -1.0;
    return ms;
}

double mpcqp_last_kernel_ms(mpcqp_ctx *c, int which) {
    if (!c || which < 0 || which > 3 || !c->ev_ok || c->ev_seq[which] == 0) return -1.0;
    return ev_ms(c, which, c->ev_seq[which] - 1);
}

double mpcqp_kernel_ms_sum(mpcqp_ctx *c, int which, int *count) {
    if (count) *count = 0;
    if (!c || which < 0 || which > 3 || !c->ev_ok) return -1.0;
    const int n = std::min(c->ev_n[which], mpcqp_ctx::kTimingRing);
    double sum = 0.0;
    for (int i = 0; i < n; ++i) {
        const double ms = ev_ms(c, which, c->ev_seq[which] - 1 - i);
        if (ms < 0.0) return -1.0;
        sum += ms;
    }
    c->ev_n[which] = 0;
    if (count) *count = n;
    return sum;
}

static void tbegin(mpcqp_ctx *c, int which) {
    if (c->timing)
        hipEventRecord(c->ev[which][c->ev_seq[which] % mpcqp_ctx::kTimingRing][0], c->stream);
}
static void tend(mpcqp_ctx *c, int which) {
    if (c->timing) {
        hipEventRecord(c->ev[which][c->ev_seq[which] % mpcqp_ctx::kTimingRing][1], c->stream);
        ++c->ev_seq[which];
        ++c->ev_n[which];
    }
}

static CondenseArgs batch_condense_args(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                                        const double *lin, double *H, double *f) {
    CondenseArgs a;
    memset(&a, 0, sizeof(a));
    a.mc = make_mc(c->m.nx, c->m.nu, c->m.N, c->m.model, c->m.Ts, c->m.mass, c->Ibinv, c->dQ,
                   c->dR, c->dP);
    a.B = B;
    a.x0 = x0;
    a.xref = xref;
    a.lin = lin;
    a.H = H;
    a.f = f;
    return a;
}

static FastArgs fast_args(mpcqp_ctx *c, int B) {
    FastArgs a;
    memset(&a, 0, sizeof(a));
    const mpcqp_model &m = c->m;
    a.B = B;
    a.Ts = m.Ts;
    a.mass = m.mass;
    for (int i = 0; i < 9; ++i) a.Ibinv[i] = c->Ibinv[i];
    a.qd = c->dqd;
    a.pd = c->dpd;
    a.rmat = c->dR;
    a.fz_min = m.fz_min;
    a.fz_max = m.fz_max;
    a.fxy_max = m.fxy_max;
    a.u_min = m.u_min;
    a.u_max = m.u_max;
    a.mu = m.mu;
    a.max_iter = m.max_iter;
    a.max_free = m.max_free > 0 ? m.max_free : m.nu * m.N;
    a.stamps = c->dstamps;
    return a;
}

static MpcArgs mpc_args(mpcqp_ctx *c, int B) {
    MpcArgs a;
    memset(&a, 0, sizeof(a));
    const mpcqp_model &m = c->m;
    a.B = B;
    a.Ts = m.Ts;
    a.mass = m.mass;
    for (int i = 0; i < 9; ++i) a.Ibinv[i] = c->Ibinv[i];
    a.qd = c->dqd;
    a.pd = c->dpd;
    a.qm = c->dQ;
    a.pm = c->dP;
    a.fq = c->dFQ;
    a.fp = c->dFP;
    a.rmat = c->dR;
    a.fz_min = m.fz_min;
    a.fz_max = m.fz_max;
    a.fxy_max = m.fxy_max;
    a.u_min = m.u_min;
    a.u_max = m.u_max;
    a.mu = m.mu;
    a.max_iter = m.max_iter;
    a.max_free = m.max_free > 0 ? m.max_free : m.nu * m.N;
    a.crash_p = c->fk.crash_p;
    a.crash_p_wg = c->fk.crash_p_wg;
    {   // (pair_mpc's bound selection; gi_solver.hpp kFeasTol)
        const bool lit = m.model == MPCQP_MODEL_LITERAL;
        a.blo_v = lit ? m.u_min : m.fz_min;
        a.blo_t = lit ? m.u_min : -m.fxy_max;
        a.bhi_v = lit ? -m.u_max : -m.fz_max;
        a.bhi_t = lit ? -m.u_max : -m.fxy_max;
        a.tlo_v = -kFeasTol * (1.0 + fabs(a.blo_v));
        a.tlo_t = -kFeasTol * (1.0 + fabs(a.blo_t));
        a.thi_v = -kFeasTol * (1.0 + fabs(a.bhi_v));
        a.thi_t = -kFeasTol * (1.0 + fabs(a.bhi_t));
    }
    a.stamps = c->dstamps;
    a.flops_acc = c->flops_on ? c->dflops : nullptr;
    a.cut = 0;
#ifdef MPCQP_CUTS
    if (const char *e = getenv("MPCQP_CUT")) a.cut = atoi(e);
#endif
    return a;
}

static int launch(const void *k, int B, size_t lds, hipStream_t s, void *arg) {
    void *args[] = {arg};
    return hip_status(hipLaunchKernel(k, dim3(B), dim3(64), args, lds, s));
}

// grow a context-owned device buffer to `bytes` (waits for the stream before freeing the old
// one); mpcqp_ctx_reserve sizes every such buffer up front so the solve path never allocates
static int ensure_bytes(mpcqp_ctx *c, void **buf, size_t *cap, size_t bytes) {
    if (*cap >= bytes) return MPCQP_OK;
    if (*buf) hipStreamSynchronize(c->stream);
    hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    ++c->buf_gen;  // captured host-path graphs may hold the old address
    if (hipMalloc(buf, bytes) != hipSuccess) return MPCQP_ERR_DEVICE;
    *cap = bytes;
    return MPCQP_OK;
}

static size_t host_stage_bytes(const mpcqp_ctx *c, size_t B) {
    const size_t nx = c->m.nx, N = c->m.N, nV = (size_t)c->m.nu * c->m.N;
    const size_t lin_w = c->m.model == MPCQP_MODEL_DENSE ? nx * (nx + c->m.nu) : 8;
    return sizeof(double) * (nx * B + nx * (N + 1) * B + lin_w * B + nV * B + B) +
           sizeof(uint64_t) * B + 2 * sizeof(int) * B + 64;
}

static size_t rollout_bytes(const mpcqp_ctx *c, size_t S, size_t C) {
    const size_t B = S * C, nV = (size_t)c->m.nu * c->m.N;
    return sizeof(double) * (B * nV + B + S * nV + S) + sizeof(int) * (2 * B + S) + 64;
}

static int warm_words(const mpcqp_ctx *c) {
    return (2 * c->m.nu * c->m.N + 8 * c->m.N + 63) / 64;
}

// the warm-start words of B instances, zeroed (cold) after mpcqp_set_warm_start or a resize
static int ensure_warm(mpcqp_ctx *c, int B) {
    const size_t bytes = sizeof(unsigned long long) * warm_words(c) * (size_t)B;
    if (c->warm_cap < bytes) {
        int rc = ensure_bytes(c, &c->dwarm, &c->warm_cap, bytes);
        if (rc) return rc;
        c->warm_fresh = 1;
    }
    if (c->warm_fresh) {
        if (hipMemsetAsync(c->dwarm, 0, c->warm_cap, c->stream) != hipSuccess) return MPCQP_ERR_DEVICE;
        c->warm_fresh = 0;
    }
    return MPCQP_OK;
}

// overflow list for B instances (grown on demand; mpcqp_ctx_reserve sizes it up front): two
// lists (alternate launches), each kListSubs counters then kListSubs sub-lists (mpc_fused.hpp)
static size_t list_stride(size_t cap) { return kListHeadWords + kListSubs * (size_t)ovf_list_cap((long long)cap); }
static int ensure_list(mpcqp_ctx *c, int B) {
    if (c->list_cap >= (size_t)B) return MPCQP_OK;
    if (c->dlist) hipStreamSynchronize(c->stream);
    hipFree(c->dlist);
    c->dlist = nullptr;
    c->list_cap = 0;
    ++c->buf_gen;
    const size_t stride = list_stride((size_t)B);
    if (hipMalloc(&c->dlist, sizeof(int) * 2 * stride) != hipSuccess ||
        hipMemsetAsync(c->dlist, 0, sizeof(int) * kListHeadWords, c->stream) != hipSuccess ||
        hipMemsetAsync(c->dlist + stride, 0, sizeof(int) * kListHeadWords, c->stream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    c->list_cap = B;
    c->list_par = 0;
    return MPCQP_OK;
}

// the fused step: two instances per wave when the paired kernel is instantiated; instances
// beyond the one-wave kernel's free capacity go through the overflow list to the workgroup
// kernel, launched right after on the same stream
static int launch_mpc(mpcqp_ctx *c, bool gen, int B, MpcArgs *a, bool may_overflow = true) {
    a->ovf = nullptr;
    int *list = nullptr, *rearm = nullptr;
    if (c->fk.wg && !gen && may_overflow) {
        const int rc = ensure_list(c, B);
        if (rc) return rc;
        const size_t stride = list_stride(c->list_cap);
        list = c->dlist + (c->list_par ? stride : 0);
        rearm = c->dlist + (c->list_par ? 0 : stride);
        a->ovf = list;
        a->ovf_cap = ovf_list_cap((long long)c->list_cap);
    }
    const void *pk = gen ? c->fk.pair_gen : c->fk.pair;
    if (pk && B >= c->fk.pair_w4_min && c->fk.pair_w4_min > 0) {
        const void *p4 = gen ? c->fk.pair_gen_w4 : c->fk.pair_w4;
        if (p4) pk = p4;
    }
    a->sel_final = a->ovf ? 0 : 1;  // fused selection: the batch's last launch finalizes
    if (a->flops_acc && pk) ++c->flops_launches;
    tbegin(c, 2);
    int rc = pk ? launch(pk, (B + 1) / 2, c->fk.pair_lds, c->stream, a)
                : launch(gen ? c->fk.mpc_gen : c->fk.mpc, B, c->fk.mpc_lds, c->stream, a);
    tend(c, 2);
    if (rc || !a->ovf) return rc;
    a->sel_final = 1;
    void *args[] = {a, &list, &rearm};
    const int grid = std::max(1, std::min(B, c->wg_grid));
    tbegin(c, 3);
    rc = hip_status(hipLaunchKernel(c->fk.wg, dim3(grid), dim3(c->fk.wg_threads), args, c->fk.wg_lds,
                                    c->stream));
    tend(c, 3);
    c->list_par ^= 1;
    return rc;
}

int mpcqp_batch_condense(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                         const double *lin, double *H, double *f) {
    if (!c || !x0 || !xref || !lin || !H || !f || B < 0) return MPCQP_ERR_BAD_ARG;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    CondenseArgs a = batch_condense_args(c, B, x0, xref, lin, H, f);
    const size_t lds = set_lds((const void *)k_condense,
                               sizeof(double) * condense_lds_doubles(c->m.nx, c->m.nu, c->m.N));
    tbegin(c, 0);
    hipLaunchKernelGGL(k_condense, dim3(B), dim3(64), lds, c->stream, a);
    tend(c, 0);
    return hip_status(hipGetLastError());
}

static SolveArgs batch_solve_args(mpcqp_ctx *c, int B, const double *H, const double *f,
                                  const uint64_t *contact, double *U, double *cost, int *status,
                                  int *iters) {
    SolveArgs a;
    memset(&a, 0, sizeof(a));
    const mpcqp_model &m = c->m;
    a.B = B;
    // the stand-alone solve is one wave: at most 64 free variables (more -> BAD_DIMS)
    a.nfmax = std::min(kWave, m.max_free > 0 ? m.max_free : m.nu * m.N);
    a.P.nV = m.nu * m.N;
    a.P.H = H;
    a.P.f = f;
    a.P.gen_bounds = 1;
    a.P.model = m.model;
    a.P.nu = m.nu;
    a.P.N = m.N;
    a.P.nfeet = 2;
    a.P.fz_min = m.fz_min;
    a.P.fz_max = m.fz_max;
    a.P.fxy_max = m.fxy_max;
    a.P.u_min = m.u_min;
    a.P.u_max = m.u_max;
    a.P.friction = (m.model == MPCQP_MODEL_SRBM && m.constraints == MPCQP_CONS_FRICTION);
    a.P.mu = m.mu;
    a.P.max_iter = m.max_iter;
    a.contact = (m.model == MPCQP_MODEL_SRBM) ? contact : nullptr;
    a.x = U;
    a.cost = cost;
    a.status = status;
    a.iters = iters;
    return a;
}

// The stand-alone (generic) solve holds 64 free variables.  A dense-model context frees every
// input (u_min < u_max is required), so above 64 inputs no instance can be served there: the
// staged entry points refuse it (mpcqp_batch_solve runs k_dense_wg instead).
static bool generic_solve_unfit(const mpcqp_ctx *c) {
    const int nfmax = c->m.max_free > 0 ? c->m.max_free : c->m.nu * c->m.N;
    return c->m.model == MPCQP_MODEL_DENSE && std::min(nfmax, c->m.nu * c->m.N) > kWave;
}

int mpcqp_batch_solve_qp(mpcqp_ctx *c, int B, const double *H, const double *f,
                         const uint64_t *contact, double *U, double *cost, int *status,
                         int *iters) {
    if (!c || !H || !f || !U || !cost || !status || !iters || B < 0) return MPCQP_ERR_BAD_ARG;
    if (generic_solve_unfit(c)) return MPCQP_ERR_BAD_DIMS;
    if (c->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    SolveArgs a = batch_solve_args(c, B, H, f, contact, U, cost, status, iters);
    const int nfric = a.P.friction ? 4 * c->m.N * 2 : 0;
    const size_t lds = set_lds((const void *)k_solve, gi_lds_bytes(a.nfmax, a.P.nV, 0, nfric));
    tbegin(c, 1);
    hipLaunchKernelGGL(k_solve, dim3(B), dim3(64), lds, c->stream, a);
    tend(c, 1);
    return hip_status(hipGetLastError());
}

int mpcqp_batch_discretize(mpcqp_ctx *c, int B, const double *lin, double *AB) {
    if (!c || !lin || !AB || B < 0) return MPCQP_ERR_BAD_ARG;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    int rc;
    tbegin(c, 0);
    if (c->fast && c->fk.disc) {
        FastArgs a = fast_args(c, B);
        a.lin = lin;
        a.AB = AB;
        rc = launch(c->fk.disc, B, c->fk.disc_lds, c->stream, &a);
    } else {
        CondenseArgs a = batch_condense_args(c, B, nullptr, nullptr, lin, nullptr, nullptr);
        a.ABout = AB;
        a.discretize_only = 1;
        const size_t lds = set_lds((const void *)k_condense,
                                   sizeof(double) * condense_lds_doubles(c->m.nx, c->m.nu, 1));
        hipLaunchKernelGGL(k_condense, dim3(B), dim3(64), lds, c->stream, a);
        rc = hip_status(hipGetLastError());
    }
    tend(c, 0);
    return rc;
}

static int ensure_scratch_hf(mpcqp_ctx *c, int B) {
    const size_t nV = (size_t)c->m.nu * c->m.N;
    if (c->scratch_cap >= (size_t)B) return MPCQP_OK;
    if (c->scratchH) hipStreamSynchronize(c->stream);
    hipFree(c->scratchH);
    hipFree(c->scratchF);
    c->scratchH = c->scratchF = nullptr;
    c->scratch_cap = 0;
    ++c->buf_gen;
    if (hipMalloc(&c->scratchH, sizeof(double) * nV * nV * B) != hipSuccess ||
        hipMalloc(&c->scratchF, sizeof(double) * nV * B) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    c->scratch_cap = B;
    return MPCQP_OK;
}

int mpcqp_batch_condense_solve(mpcqp_ctx *c, int B, const double *AB, const double *x0,
                               const double *xref, const uint64_t *contact, double *U,
                               double *cost, int *status, int *iters) {
    if (!c || !AB || !x0 || !xref || !U || !cost || !status || !iters || B < 0)
        return MPCQP_ERR_BAD_ARG;
    if (c->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
    if (!(c->fast && c->fk.cs) && generic_solve_unfit(c)) return MPCQP_ERR_BAD_DIMS;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    if (c->fast && c->fk.cs) {
        FastArgs a = fast_args(c, B);
        a.AB = const_cast<double *>(AB);
        a.x0 = x0;
        a.xref = xref;
        a.contact = contact;
        a.U = U;
        a.cost = cost;
        a.status = status;
        a.iters = iters;
        tbegin(c, 1);
        const int rc = launch(c->fk.cs, B, c->fk.cs_lds, c->stream, &a);
        tend(c, 1);
        return rc;
    }
    // generic: condense from the given [Ad | Bd] into scratch H, f, then solve
    int rc = ensure_scratch_hf(c, B);
    if (rc) return rc;
    CondenseArgs a = batch_condense_args(c, B, x0, xref, nullptr, c->scratchH, c->scratchF);
    a.ABin = AB;
    const size_t lds = set_lds((const void *)k_condense,
                               sizeof(double) * condense_lds_doubles(c->m.nx, c->m.nu, c->m.N));
    hipLaunchKernelGGL(k_condense, dim3(B), dim3(64), lds, c->stream, a);
    rc = hip_status(hipGetLastError());
    if (rc) return rc;
    return mpcqp_batch_solve_qp(c, B, c->scratchH, c->scratchF, contact, U, cost, status, iters);
}

static int batch_solve(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                       const double *lin, const uint64_t *contact, double *U, double *cost,
                       int *status, int *iters, bool may_overflow);

int mpcqp_batch_solve(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                      const double *lin, const uint64_t *contact, double *U, double *cost,
                      int *status, int *iters) {
    return batch_solve(c, B, x0, xref, lin, contact, U, cost, status, iters, true);
}

static int batch_solve(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                       const double *lin, const uint64_t *contact, double *U, double *cost,
                       int *status, int *iters, bool may_overflow) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    if (B <= 0) return B == 0 ? MPCQP_OK : MPCQP_ERR_BAD_ARG;
    hipSetDevice(c->device);
    if (c->fast) {  // one fused kernel: closed-form linearise/discretise/condense + solve
        if (!x0 || !xref || !lin || !U || !cost || !status || !iters) return MPCQP_ERR_BAD_ARG;
        if (c->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
        MpcArgs a = mpc_args(c, B);
        a.lin = lin;
        a.x0 = x0;
        a.xref = xref;
        a.contact = contact;
        a.U = U;
        a.cost = cost;
        a.status = status;
        a.iters = iters;
        tbegin(c, 1);
        int rc;
        if (c->fk.dense) {  // one workgroup per QP
            void *args[] = {&a};
            rc = hip_status(hipLaunchKernel(c->fk.dense, dim3(B), dim3(c->fk.dense_threads), args,
                                            c->fk.dense_lds, c->stream));
        } else {
            rc = launch_mpc(c, false, B, &a, may_overflow);
        }
        tend(c, 1);
        return rc;
    }
    const size_t ab = (size_t)c->m.nx * (c->m.nx + c->m.nu);
    int rc = ensure_bytes(c, (void **)&c->dAB, &c->ab_cap, sizeof(double) * ab * B);
    if (rc) return rc;
    rc = mpcqp_batch_discretize(c, B, lin, c->dAB);
    if (rc) return rc;
    return mpcqp_batch_condense_solve(c, B, c->dAB, x0, xref, contact, U, cost, status, iters);
}

int mpcqp_batch_solve_select(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                             const double *lin, const uint64_t *contact, double *U, double *cost,
                             int *status, int *iters, int64_t index_base, int64_t *record) {
    if (!c || !record) return MPCQP_ERR_BAD_ARG;
    if (B < 0) return MPCQP_ERR_BAD_ARG;
    if (index_base < 0 || index_base + (int64_t)B > 0x7fffffffll) return MPCQP_ERR_BAD_DIMS;
    hipSetDevice(c->device);
    if (B > 0 && c->fast && !c->fk.dense && c->fk.wg) {
        // the fused kernels min their keys into the context's selection words and the last
        // workgroup of the workgroup kernel (always launched after the one-wave kernel on these
        // contexts; its resident grid takes the tickets) writes the record: no selection launch.
        // (Contexts without the workgroup kernel keep k_select_min: a ticket from every one-wave
        // workgroup costs each an agent-scope release, an L2 write-back -- 1.10 ms per launch
        // at 65,536 against 0.38 ms with the separate selection, r03s)
        if (!x0 || !xref || !lin || !U || !cost || !status || !iters) return MPCQP_ERR_BAD_ARG;
        if (c->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
        MpcArgs a = mpc_args(c, B);
        a.lin = lin;
        a.x0 = x0;
        a.xref = xref;
        a.contact = contact;
        a.U = U;
        a.cost = cost;
        a.status = status;
        a.iters = iters;
        a.sel = c->dsel + kFusedSel;
        a.sel_base = (long long)index_base;
        a.sel_rec = reinterpret_cast<long long *>(record);
        tbegin(c, 1);
        const int rc = launch_mpc(c, false, B, &a);
        tend(c, 1);
        return rc;
    }
    int rc = mpcqp_batch_solve(c, B, x0, xref, lin, contact, U, cost, status, iters);
    if (!rc) rc = mpcqp_batch_select_record(c, B, cost, status, U, index_base, record);
    return rc;
}

int mpcqp_ctx_reserve(mpcqp_ctx *c, int B) {
    if (!c || B < 0) return MPCQP_ERR_BAD_ARG;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    const size_t ab = (size_t)c->m.nx * (c->m.nx + c->m.nu);
    int rc = ensure_bytes(c, &c->hbuf, &c->hbuf_cap, host_stage_bytes(c, B));
    if (!rc) rc = ensure_bytes(c, &c->fkbuf, &c->fkbuf_cap, sizeof(double) * 15 * (size_t)B);
    if (!rc && c->fast && c->fk.wg) rc = ensure_list(c, B);
    if (!rc && c->fast && c->fk.mpc_gen)
        rc = ensure_bytes(c, &c->rbuf, &c->rbuf_cap, rollout_bytes(c, B, 1));
    if (!rc && c->warm_on && c->fast && c->fk.mpc_gen) rc = ensure_warm(c, B);
    if (!rc && !c->fast) rc = ensure_bytes(c, (void **)&c->dAB, &c->ab_cap, sizeof(double) * ab * B);
    if (!rc && !c->fast) rc = ensure_scratch_hf(c, B);
    if (!rc) rc = hip_status(hipStreamSynchronize(c->stream));
    return rc;
}

int mpcqp_ctx_fk_feet_host(mpcqp_ctx *c, int R, const double *q, const double *rpy,
                           int rpy_stride, double *feet) {
    if (!c || !q || !rpy || !feet || R < 0 || rpy_stride < 3) return MPCQP_ERR_BAD_ARG;
    if (R == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    const size_t nq = 6 * (size_t)R, nr = (size_t)rpy_stride * (R - 1) + 3, nf = 6 * (size_t)R;
    if (ensure_bytes(c, &c->fkbuf, &c->fkbuf_cap, sizeof(double) * (nq + nr + nf)))
        return MPCQP_ERR_DEVICE;
    double *dq = (double *)c->fkbuf, *dr = dq + nq, *df = dr + nr;
    if (hipMemcpyAsync(dq, q, sizeof(double) * nq, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(dr, rpy, sizeof(double) * nr, hipMemcpyHostToDevice, c->stream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    int rc = mpcqp_fk_feet(c->stream, R, dq, dr, rpy_stride, df);
    if (rc) return rc;
    if (hipMemcpyAsync(feet, df, sizeof(double) * nf, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    return hip_status(hipStreamSynchronize(c->stream));
}

// Can an instance of this host batch need more free variables than the one-wave kernel holds
// (so the overflow workgroup kernel must run)?  The free count follows from the contact word
// alone: the forces of a foot in contact are free, a swing foot's are fixed (SRBM); every input
// is free in the literal model.
static bool host_may_overflow(const mpcqp_ctx *c, int B, const uint64_t *contact) {
    if (!c->fast || !c->fk.wg) return false;
    if (c->m.model != MPCQP_MODEL_SRBM || !contact) return true;
    const int N = c->m.N;
    const uint64_t mask = N >= 32 ? ~0ull : ((1ull << (2 * N)) - 1ull);
    for (int i = 0; i < B; ++i)
        if (3 * __builtin_popcountll(contact[i] & mask) > c->fk.prim_nf) return true;
    return false;
}

// the host path's step on its staging, as the stream work of one call: H2D of the inputs, the
// solve, D2H of the outputs (captured once into a graph per batch size and list parity)
static int host_step(mpcqp_ctx *c, int B, bool ovf, size_t in_bytes, size_t out_off,
                     size_t out_bytes, bool has_contact) {
    const size_t nx = c->m.nx, N = c->m.N, nV = (size_t)c->m.nu * c->m.N;
    const size_t lin_w = c->m.model == MPCQP_MODEL_DENSE ? nx * (nx + c->m.nu) : 8;
    char *d = (char *)c->hbuf;
    double *d_x0 = (double *)d, *d_xr = d_x0 + nx * B, *d_lin = d_xr + nx * (N + 1) * B;
    uint64_t *d_ct = (uint64_t *)(d_lin + lin_w * B);
    double *d_U = (double *)(d + out_off), *d_cost = d_U + nV * B;
    int *d_st = (int *)(d_cost + B), *d_it = d_st + B;
    if (hipMemcpyAsync(d, c->pin, in_bytes, hipMemcpyHostToDevice, c->hstream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    hipStream_t keep = c->stream;
    c->stream = c->hstream;
    const int rc = batch_solve(c, B, d_x0, d_xr, d_lin, has_contact ? d_ct : nullptr, d_U, d_cost,
                               d_st, d_it, ovf);
    c->stream = keep;
    if (rc) return rc;
    if (hipMemcpyAsync((char *)c->pin + out_off, d + out_off, out_bytes, hipMemcpyDeviceToHost,
                       c->hstream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    return MPCQP_OK;
}

static void host_graphs_drop(mpcqp_ctx *c) {
    for (int i = 0; i < 3; ++i)
        if (c->hg_exec[i]) { hipGraphExecDestroy(c->hg_exec[i]); c->hg_exec[i] = nullptr; }
    c->hg_B = 0;
}

// ---- page-locked host memory (the caller's own buffers handed to the solver, as
// src/QPSolver.cpp:93-96 hands its Eigen storage to qpOASES): registered or allocated here, a host
// array is DMA'd straight to and from the device by the host-pointer entry points
int mpcqp_host_register(void *p, size_t bytes) {
    if (!p || !bytes) return MPCQP_ERR_BAD_ARG;
    // page-aligned starts only: pinning works on whole pages, and two registrations that share a
    // page (small heap arrays side by side) left the runtime with a stale mapping of it -- a
    // later pageable copy through that page faulted the device (r06y).  With aligned starts no
    // page is ever registered twice.
    const long page = sysconf(_SC_PAGESIZE);
    if (page > 0 && ((uintptr_t)p % (uintptr_t)page) != 0) return MPCQP_ERR_BAD_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MPCQP_ERR_NO_DEVICE;
    return hip_status(hipHostRegister(p, bytes, hipHostRegisterDefault));
}

int mpcqp_host_unregister(void *p) {
    if (!p) return MPCQP_ERR_BAD_ARG;
    return hip_status(hipHostUnregister(p));
}

int mpcqp_host_alloc(size_t bytes, void **p) {
    if (!p || !bytes) return MPCQP_ERR_BAD_ARG;
    *p = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MPCQP_ERR_NO_DEVICE;
    return hip_status(hipHostMalloc(p, bytes, hipHostMallocDefault));
}

int mpcqp_host_free(void *p) {
    if (!p) return MPCQP_ERR_BAD_ARG;
    return hip_status(hipHostFree(p));
}

// is [p, p + bytes) page-locked host memory the device can DMA (hipHostRegister / hipHostMalloc)?
static bool host_locked(const void *p, size_t bytes) {
    if (!p || !bytes) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    // the whole range must belong to one locked allocation: check its last byte as well
    hipPointerAttribute_t at2;
    if (hipPointerGetAttributes(&at2, (const char *)p + bytes - 1) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at2.type == hipMemoryTypeHost;
}

// batches below this go through the pinned staging and the captured graphs (the per-tick path)
constexpr int kHostDirectMin = 4096;

// The direct host path: inputs DMA'd from the caller's page-locked arrays into device staging and
// outputs DMA'd back into the caller's arrays, no host memcpy.  The batch goes in chunks
// (multiples of 16 instances: the paired kernel's candidate groups stay whole, so every instance
// is solved exactly as in one launch), pipelined over three streams: the copy-in of chunk i + 1
// and the copy-out of chunk i - 1 run beside the solve of chunk i.
static int host_direct(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                       const double *lin, const uint64_t *contact, double *U, double *cost,
                       int *status, int *iters, bool ovf, size_t out_off) {
    if (!c->hd_ok) {
        if (hipStreamCreateWithFlags(&c->hs_in, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&c->hs_out, hipStreamNonBlocking) != hipSuccess)
            return MPCQP_ERR_DEVICE;
        for (int i = 0; i < 8; ++i)
            if (hipEventCreateWithFlags(&c->hev_in[i], hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&c->hev_k[i], hipEventDisableTiming) != hipSuccess)
                return MPCQP_ERR_DEVICE;
        c->hd_ok = true;
    }
    const size_t nx = c->m.nx, N = c->m.N, nV = (size_t)c->m.nu * c->m.N;
    const size_t lin_w = c->m.model == MPCQP_MODEL_DENSE ? nx * (nx + c->m.nu) : 8;
    char *d = (char *)c->hbuf;
    double *d_x0 = (double *)d, *d_xr = d_x0 + nx * B, *d_lin = d_xr + nx * (N + 1) * B;
    uint64_t *d_ct = (uint64_t *)(d_lin + lin_w * B);
    double *d_U = (double *)(d + out_off), *d_cost = d_U + nV * B;
    int *d_st = (int *)(d_cost + B), *d_it = d_st + B;
    // four chunks of >= 8,192 instances (at most 8), multiples of 16
    int chunk = std::max(8192, (B / 4 + 15) & ~15);
    if ((B + chunk - 1) / chunk > 8) chunk = ((B + 7) / 8 + 15) & ~15;
    const int nch = (B + chunk - 1) / chunk;
    // the copy-in waits for the context's earlier work (hev was recorded on its stream)
    if (hipStreamWaitEvent(c->hs_in, c->hev, 0) != hipSuccess) return MPCQP_ERR_DEVICE;
    const hipMemcpyKind h2d = hipMemcpyHostToDevice, d2h = hipMemcpyDeviceToHost;
    for (int i = 0; i < nch; ++i) {
        const size_t i0 = (size_t)i * chunk, n = std::min((size_t)chunk, (size_t)B - i0);
        if (hipMemcpyAsync(d_x0 + i0 * nx, x0 + i0 * nx, 8 * nx * n, h2d, c->hs_in) != hipSuccess ||
            hipMemcpyAsync(d_xr + i0 * nx * (N + 1), xref + i0 * nx * (N + 1), 8 * nx * (N + 1) * n,
                           h2d, c->hs_in) != hipSuccess ||
            hipMemcpyAsync(d_lin + i0 * lin_w, lin + i0 * lin_w, 8 * lin_w * n, h2d, c->hs_in) != hipSuccess ||
            (contact && hipMemcpyAsync(d_ct + i0, contact + i0, 8 * n, h2d, c->hs_in) != hipSuccess) ||
            hipEventRecord(c->hev_in[i], c->hs_in) != hipSuccess ||
            hipStreamWaitEvent(c->hstream, c->hev_in[i], 0) != hipSuccess)
            return MPCQP_ERR_DEVICE;
        hipStream_t keep = c->stream;
        const bool timing = c->timing;
        c->stream = c->hstream;
        c->timing = false;  // (the host path does not feed the timing slots)
        const int rc = batch_solve(c, (int)n, d_x0 + i0 * nx, d_xr + i0 * nx * (N + 1),
                                   d_lin + i0 * lin_w, contact ? d_ct + i0 : nullptr,
                                   d_U + i0 * nV, d_cost + i0, d_st + i0, d_it + i0, ovf);
        c->stream = keep;
        c->timing = timing;
        if (rc) return rc;
        if (hipEventRecord(c->hev_k[i], c->hstream) != hipSuccess ||
            hipStreamWaitEvent(c->hs_out, c->hev_k[i], 0) != hipSuccess ||
            hipMemcpyAsync(U + i0 * nV, d_U + i0 * nV, 8 * nV * n, d2h, c->hs_out) != hipSuccess ||
            hipMemcpyAsync(cost + i0, d_cost + i0, 8 * n, d2h, c->hs_out) != hipSuccess ||
            hipMemcpyAsync(status + i0, d_st + i0, 4 * n, d2h, c->hs_out) != hipSuccess ||
            hipMemcpyAsync(iters + i0, d_it + i0, 4 * n, d2h, c->hs_out) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    if (hipStreamSynchronize(c->hs_out) != hipSuccess || hipStreamSynchronize(c->hstream) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    return MPCQP_OK;
}

int mpcqp_batch_solve_host(mpcqp_ctx *c, int B, const double *x0, const double *xref,
                           const double *lin, const uint64_t *contact, double *U, double *cost,
                           int *status, int *iters) {
    if (!c || !x0 || !xref || !lin || !U || !cost || !status || !iters || B < 0)
        return MPCQP_ERR_BAD_ARG;
    if (c->m.model == MPCQP_MODEL_SRBM && !contact) return MPCQP_ERR_BAD_ARG;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    // one byte layout on both sides: inputs [x0 | xref | lin | contact], then (16-B aligned)
    // outputs [U | cost | status | iters]
    const size_t nx = c->m.nx, N = c->m.N, nV = (size_t)c->m.nu * c->m.N;
    const size_t lin_w = c->m.model == MPCQP_MODEL_DENSE ? nx * (nx + c->m.nu) : 8;
    const size_t b_x0 = sizeof(double) * nx * B, b_xr = sizeof(double) * nx * (N + 1) * B,
                 b_lin = sizeof(double) * lin_w * B, b_ct = contact ? sizeof(uint64_t) * B : 0;
    const size_t in_bytes = b_x0 + b_xr + b_lin + sizeof(uint64_t) * B;
    const size_t out_off = (in_bytes + 15) & ~(size_t)15;
    const size_t b_u = sizeof(double) * nV * B, b_c = sizeof(double) * B, b_i = sizeof(int) * B;
    const size_t out_bytes = b_u + b_c + 2 * b_i, total = out_off + out_bytes;
    if (ensure_bytes(c, &c->hbuf, &c->hbuf_cap, std::max(total, host_stage_bytes(c, B))))
        return MPCQP_ERR_DEVICE;
    if (!c->hstream) {
        if (hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->hev, hipEventDisableTiming) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    const bool ovf = host_may_overflow(c, B, contact);
    if (ovf && ensure_list(c, B)) return MPCQP_ERR_DEVICE;  // (allocates outside any capture)
    // the caller's arrays page-locked (mpcqp_host_register / mpcqp_host_alloc) and a large batch:
    // one DMA each way straight from / into them, pipelined in chunks
    if (B >= kHostDirectMin && !c->hd_off && host_locked(x0, b_x0) && host_locked(xref, b_xr) &&
        host_locked(lin, b_lin) && (!contact || host_locked(contact, b_ct)) &&
        host_locked(U, b_u) && host_locked(cost, b_c) && host_locked(status, b_i) &&
        host_locked(iters, b_i)) {
        if (hipEventRecord(c->hev, c->stream) != hipSuccess) return MPCQP_ERR_DEVICE;
        return host_direct(c, B, x0, xref, lin, contact, U, cost, status, iters, ovf, out_off);
    }
    // otherwise: one memcpy into the context's pinned staging and one DMA each way
    if (c->pin_cap < total) {
        if (c->pin) hipHostFree(c->pin);
        c->pin = nullptr;
        c->pin_cap = 0;
        ++c->buf_gen;
        if (hipHostMalloc(&c->pin, total, hipHostMallocDefault) != hipSuccess) return MPCQP_ERR_DEVICE;
        c->pin_cap = total;
    }
    // (after every allocation this call may make: a graph is captured against the buffers as
    // they are now)
    if (c->hg_gen != c->buf_gen) {
        host_graphs_drop(c);
        c->hg_gen = c->buf_gen;
    }
    char *h = (char *)c->pin;
    memcpy(h, x0, b_x0);
    memcpy(h + b_x0, xref, b_xr);
    memcpy(h + b_x0 + b_xr, lin, b_lin);
    if (b_ct) memcpy(h + b_x0 + b_xr + b_lin, contact, b_ct);
    // after the context's earlier work (the overflow lists, buffers it may still use)
    if (hipEventRecord(c->hev, c->stream) != hipSuccess ||
        hipStreamWaitEvent(c->hstream, c->hev, 0) != hipSuccess)
        return MPCQP_ERR_DEVICE;
    int rc = MPCQP_OK;
    const bool graph = c->fast && !c->hg_off;
    if (graph) {
        if (c->hg_B != B) {
            host_graphs_drop(c);
            c->hg_B = B;
        }
        // one graph per (overflow launch, list parity): a contact schedule that flips the
        // overflow prediction from tick to tick replays cached graphs instead of re-capturing
        const int par = ovf ? 1 + c->list_par : 0;
        if (!c->hg_exec[par]) {
            // capture one call's stream work; the capture does not run it, so the list parity
            // the capture advanced is put back (the launch below advances it)
            const bool timing = c->timing;
            c->timing = false;
            hipGraph_t g = nullptr;
            bool ok = hipStreamBeginCapture(c->hstream, hipStreamCaptureModeThreadLocal) == hipSuccess;
            const int rcc = ok ? host_step(c, B, ovf, in_bytes, out_off, out_bytes, b_ct != 0) : MPCQP_OK;
            if (ok) ok = hipStreamEndCapture(c->hstream, &g) == hipSuccess && rcc == MPCQP_OK;
            c->list_par = ovf ? par - 1 : c->list_par;
            c->timing = timing;
            if (ok) ok = hipGraphInstantiate(&c->hg_exec[par], g, nullptr, nullptr, 0) == hipSuccess;
            if (g) hipGraphDestroy(g);
            if (!ok) {
                c->hg_exec[par] = nullptr;
                c->hg_off = true;  // fall back to direct launches from now on
                (void)hipGetLastError();
            }
        }
        if (c->hg_exec[par]) {
            if (hipGraphLaunch(c->hg_exec[par], c->hstream) != hipSuccess) return MPCQP_ERR_DEVICE;
            if (ovf) c->list_par ^= 1;
        } else {
            rc = host_step(c, B, ovf, in_bytes, out_off, out_bytes, b_ct != 0);
        }
    } else {
        rc = host_step(c, B, ovf, in_bytes, out_off, out_bytes, b_ct != 0);
    }
    if (rc) return rc;
    rc = hip_status(hipStreamSynchronize(c->hstream));
    if (rc) return rc;
    memcpy(U, h + out_off, b_u);
    memcpy(cost, h + out_off + b_u, b_c);
    memcpy(status, h + out_off + b_u + b_c, b_i);
    memcpy(iters, h + out_off + b_u + b_c + b_i, b_i);
    return MPCQP_OK;
}

int mpcqp_set_warm_start(mpcqp_ctx *c, int on) {
    if (!c) return MPCQP_ERR_BAD_ARG;
    c->warm_on = on ? 1 : 0;
    c->warm_fresh = 1;  // the next gait solve starts cold
    return MPCQP_OK;
}

int mpcqp_batch_solve_gait(mpcqp_ctx *c, int S, int C, const double *state, const double *feet,
                           const double *cmd, const double *phase, float swing, float stance,
                           double *U, double *cost, int *status, int *iters) {
    if (!c || !state || !feet || !cmd || !phase || !U || !cost || !status || !iters || S < 0 ||
        C <= 0)
        return MPCQP_ERR_BAD_ARG;
    if (!(swing > 0.0f) || !(stance >= 0.0f)) return MPCQP_ERR_BAD_ARG;
    if (!c->fast || !c->fk.mpc_gen) return MPCQP_ERR_BAD_DIMS;  // SRBM fast-path models only
    if ((long long)S * C > 0x7fffffffll) return MPCQP_ERR_BAD_DIMS;
    const int B = S * C;
    if (B == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    MpcArgs a = mpc_args(c, B);
    a.state = state;
    a.feet = feet;
    a.cmd = cmd;
    a.phase = phase;
    a.cands = C;
    a.swing = swing;
    a.stance = stance;
    a.U = U;
    a.cost = cost;
    a.status = status;
    a.iters = iters;
    if (c->warm_on) {  // the paired kernel seeds its crash start, the one-wave kernels their dual loop
        const int rw = ensure_warm(c, B);
        if (rw) return rw;
        a.warm = reinterpret_cast<unsigned long long *>(c->dwarm);
        a.warm_words = warm_words(c);
    }
    tbegin(c, 1);
    const int rc = launch_mpc(c, true, B, &a);
    tend(c, 1);
    return rc;
}

int mpcqp_batch_select_state(mpcqp_ctx *c, int S, int C, const double *cost, const int *status,
                             const double *U, int *best, double *best_cost, double *Ubest) {
    if (!c || !cost || !status || !best || S < 0 || C <= 0 || C > 64) return MPCQP_ERR_BAD_ARG;
    if (Ubest && !U) return MPCQP_ERR_BAD_ARG;
    if (S == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    hipLaunchKernelGGL(k_select_state, dim3(S), dim3(64), 0, c->stream, S, C, c->m.nu * c->m.N,
                       cost, status, U, best, best_cost, Ubest);
    return hip_status(hipGetLastError());
}

int mpcqp_batch_plant_srbm(mpcqp_ctx *c, int S, int C, double *state, double *feet,
                           double *phase, const int *best, const double *Ubest) {
    if (!c || !state || !feet || !best || !Ubest || S < 0 || C < 0 || (C > 0 && !phase))
        return MPCQP_ERR_BAD_ARG;
    if (c->m.model != MPCQP_MODEL_SRBM || c->m.nx != 13 || c->m.nu != 6) return MPCQP_ERR_BAD_DIMS;
    if (S == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    PlantArgs a;
    memset(&a, 0, sizeof(a));
    a.S = S;
    a.C = C;
    a.nV = c->m.nu * c->m.N;
    a.Ts = c->m.Ts;
    a.mass = c->m.mass;
    for (int i = 0; i < 9; ++i) a.Ibinv[i] = c->Ibinv[i];
    a.state = state;
    a.feet = feet;
    a.phase = phase;
    a.Ubest = Ubest;
    a.best = best;
    hipLaunchKernelGGL(k_plant_srbm, dim3(S), dim3(64), 0, c->stream, a);
    return hip_status(hipGetLastError());
}

int mpcqp_rollout(mpcqp_ctx *c, int S, int C, int K, double *state, double *feet,
                  const double *cmd, double *phase, float swing, float stance, double *traj,
                  int *choice) {
    if (!c || !state || !feet || !cmd || !phase || S < 0 || C <= 0 || C > 64 || K < 0)
        return MPCQP_ERR_BAD_ARG;
    if (!c->fast || !c->fk.mpc_gen) return MPCQP_ERR_BAD_DIMS;
    if (S == 0 || K == 0) return MPCQP_OK;
    hipSetDevice(c->device);
    const size_t B = (size_t)S * C, nV = (size_t)c->m.nu * c->m.N;
    if (ensure_bytes(c, &c->rbuf, &c->rbuf_cap, rollout_bytes(c, S, C))) return MPCQP_ERR_DEVICE;
    double *U = (double *)c->rbuf, *cost = U + B * nV, *Ub = cost + B, *bc = Ub + S * nV;
    int *st = (int *)(bc + S), *it = st + B, *best = it + B;
    for (int k = 0; k < K; ++k) {
        int rc = mpcqp_batch_solve_gait(c, S, C, state, feet, cmd, phase, swing, stance, U, cost,
                                        st, it);
        if (!rc) rc = mpcqp_batch_select_state(c, S, C, cost, st, U, best, bc, Ub);
        if (!rc) rc = mpcqp_batch_plant_srbm(c, S, C, state, feet, phase, best, Ub);
        if (rc) return rc;
        if (traj && hipMemcpyAsync(traj + (size_t)k * S * 13, state, sizeof(double) * S * 13,
                                   hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
            return MPCQP_ERR_DEVICE;
        if (choice && hipMemcpyAsync(choice + (size_t)k * S, best, sizeof(int) * S,
                                     hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
            return MPCQP_ERR_DEVICE;
    }
    return MPCQP_OK;
}

int mpcqp_batch_select_min(mpcqp_ctx *c, int B, const double *cost, const int *status,
                           int64_t index_base, int64_t *key) {
    if (!c || !key || B < 0 || (B > 0 && (!cost || !status))) return MPCQP_ERR_BAD_ARG;
    hipSetDevice(c->device);
    unsigned long long *k = reinterpret_cast<unsigned long long *>(key);
    const int blocks = std::max(1, std::min(kSelMaxBlocks, (B + kSelPerBlock - 1) / kSelPerBlock));
    hipLaunchKernelGGL(k_select_min, dim3(blocks), dim3(256), 0, c->stream, B, cost, status,
                       (long long)index_base, k, c->dsel,
                       reinterpret_cast<unsigned int *>(c->dsel + kSelMaxBlocks),
                       (const double *)nullptr, 0, (double *)nullptr);
    return hip_status(hipGetLastError());
}

int mpcqp_batch_select_record(mpcqp_ctx *c, int B, const double *cost, const int *status,
                              const double *U, int64_t index_base, int64_t *record) {
    if (!c || !record || B < 0 || (B > 0 && (!cost || !status || !U))) return MPCQP_ERR_BAD_ARG;
    if (index_base < 0 || index_base + (int64_t)B > 0x7fffffffll) return MPCQP_ERR_BAD_DIMS;
    hipSetDevice(c->device);
    unsigned long long *k = reinterpret_cast<unsigned long long *>(record);
    const int nV = c->m.nu * c->m.N;
    const int blocks = std::max(1, std::min(kSelMaxBlocks, (B + kSelPerBlock - 1) / kSelPerBlock));
    hipLaunchKernelGGL(k_select_min, dim3(blocks), dim3(256), 0, c->stream, B, cost, status,
                       (long long)index_base, k, c->dsel,
                       reinterpret_cast<unsigned int *>(c->dsel + kSelMaxBlocks), U, nV,
                       reinterpret_cast<double *>(record + 1));
    return hip_status(hipGetLastError());
}

int mpcqp_reduce_records(mpcqp_ctx *c, int n, const int64_t *records, int64_t *best) {
    if (!c || !records || !best || n <= 0) return MPCQP_ERR_BAD_ARG;
    hipSetDevice(c->device);
    hipLaunchKernelGGL(k_reduce_records, dim3(1), dim3(64), 0, c->stream, n, c->m.nu * c->m.N,
                       reinterpret_cast<const long long *>(records),
                       reinterpret_cast<long long *>(best));
    return hip_status(hipGetLastError());
}

// (library-internal, group.hip) the same reduction on another stream of the context's device:
// the multi-GPU group runs it on its collective stream, after the all-gather
__attribute__((visibility("hidden"))) int mpcqp_reduce_records_on(mpcqp_ctx *c, void *stream, int n,
                                                                  const int64_t *records,
                                                                  int64_t *best) {
    if (!c || !records || !best || n <= 0) return MPCQP_ERR_BAD_ARG;
    hipSetDevice(c->device);
    hipLaunchKernelGGL(k_reduce_records, dim3(1), dim3(64), 0, (hipStream_t)stream, n,
                       c->m.nu * c->m.N, reinterpret_cast<const long long *>(records),
                       reinterpret_cast<long long *>(best));
    return hip_status(hipGetLastError());
}

}  // extern "C"
