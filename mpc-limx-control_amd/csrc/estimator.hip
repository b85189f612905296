// estimator.hip -- the producers either side of the MPC step, batched:
//   k_fk_feet     foot contact points of both 3-DoF legs (one thread per robot) -> the `feet`
//                 lever arms of mpcqp_batch_solve_gait.  Reference: Pinocchio FK on PF_TRON1A
//                 (include/pinocchio_kinematics.h:30-43); the URDF is not in the repository, so
//                 the chain is MPCParam's kinematicValues (include/MPCParam.h:13-38) with
//                 abad about x, hip and knee about y (build-chosen); at q = 0 it is exactly
//                 MPCParam's static_foot_offset_{left,right} (include/MPCParam.h:64-72).
//   k_kf_update   one step of the 12-state linear Kalman filter of stateEstimator::update
//                 (include/stateEstimator.h:217-337), one wavefront per robot, all 12x12 /
//                 14x14 algebra in LDS, partial-pivot LU of S with 13 right-hand sides.
// Both restate the reference as written (quirks listed in oracle/mpcqp_oracle.c).
#include <hip/hip_runtime.h>

#include <math.h>

#include "../../include/mpcqp.h"

namespace {

constexpr double kAbad[3] = {0.05556, 0.105, -0.2602}, kHip[3] = {-0.077, 0.02050, 0.0},
                 kKnee[3] = {-0.1500, -0.02050, -0.25981}, kFoot[3] = {0.145, 0.0, -0.2598},
                 kContact[3] = {0.0, 0.0, -0.032};

__global__ void __launch_bounds__(256) k_fk_feet(int R, const double *q, const double *rpy,
                                                 int rpy_stride, double *feet) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const double *e = rpy + (size_t)r * rpy_stride;
    double sr, cr, sp, cp, syw, cyw;
    sincos(e[0], &sr, &cr);
    sincos(e[1], &sp, &cp);
    sincos(e[2], &syw, &cyw);
#pragma unroll
    for (int leg = 0; leg < 2; ++leg) {
        const double sg = leg == 0 ? -1.0 : 1.0;  // the left leg's lateral sign, MPCParam.h:67
        const double *ql = q + (size_t)r * 6 + 3 * leg;
        double v0 = kFoot[0] + kContact[0], v1 = kFoot[1] + kContact[1], v2 = kFoot[2] + kContact[2];
        double s, c, t0, t1, t2;
        sincos(ql[2], &s, &c);  // knee, about y
        t0 = c * v0 + s * v2;
        t2 = -s * v0 + c * v2;
        v0 = t0 + kKnee[0]; v1 = v1 + sg * kKnee[1]; v2 = t2 + kKnee[2];
        sincos(ql[1], &s, &c);  // hip, about y
        t0 = c * v0 + s * v2;
        t2 = -s * v0 + c * v2;
        v0 = t0 + kHip[0]; v1 = v1 + sg * kHip[1]; v2 = t2 + kHip[2];
        sincos(ql[0], &s, &c);  // abad, about x
        t1 = c * v1 - s * v2;
        t2 = s * v1 + c * v2;
        v0 = v0 + kAbad[0]; v1 = t1 + sg * kAbad[1]; v2 = t2 + kAbad[2];
        const double a1 = v1 * cr - v2 * sr, a2 = v1 * sr + v2 * cr;  // Rx(roll)
        const double b0 = v0 * cp + a2 * sp, b2 = -v0 * sp + a2 * cp;  // Ry(pitch)
        feet[(size_t)r * 6 + 3 * leg + 0] = b0 * cyw - a1 * syw;      // Rz(yaw)
        feet[(size_t)r * 6 + 3 * leg + 1] = b0 * syw + a1 * cyw;
        feet[(size_t)r * 6 + 3 * leg + 2] = b2;
    }
}

struct KfArgs {
    int R;
    double dt;
    double *xhat, *P;              // [R][12], [R][144] col-major
    const double *eePos, *eeVel;   // [R][6]
    const unsigned char *contact;  // [R][2]
    const double *quat, *acc;      // [R][4] (x y z w), [R][3]
};

// C (14 x 12) of the estimator: rows 0-5 = [I3 0 | -I6], rows 6-11 = [0 I3 | 0], (12,8), (13,11)
__device__ __forceinline__ double kf_c(int i, int j) {
    double v = 0.0;
    if (i < 6 && j == i % 3) v = 1.0;
    if (i < 6 && j == 6 + i) v = -1.0;
    if (i >= 6 && i < 12 && j == 3 + (i - 6) % 3) v = 1.0;
    if (i == 12 && j == 8) v = 1.0;
    if (i == 13 && j == 11) v = 1.0;
    return v;
}

__global__ void __launch_bounds__(64) k_kf_update(KfArgs a) {
    __shared__ double P[144], Pm[144], PC[168], W[14 * 27], xn[12], y[14], qd[12], rd[14], accw[3];
    const int r = blockIdx.x, ln = threadIdx.x;
    if (r >= a.R) return;
    const double dt = a.dt;
    for (int e = ln; e < 144; e += 64) P[e] = a.P[(size_t)r * 144 + e];
    if (ln < 12) {
        double q = ln < 3 ? (dt / 20.f) * 0.02 : ln < 6 ? (dt * 9.81f / 20.f) * 0.02 : dt * 0.002;
        if (ln >= 6 && !a.contact[(size_t)r * 2 + (ln - 6) / 3]) q *= 100.0;
        qd[ln] = q;
    }
    if (ln < 14) {
        const int f = ln < 12 ? (ln % 6) / 3 : ln - 12;
        double rv = ln < 6 ? 0.005 : ln < 12 ? 0.1 : 0.01;
        if (!a.contact[(size_t)r * 2 + f]) rv *= 100.0;
        rd[ln] = rv;
        double yv = 0.0;  // feetHeights_ (first two entries of a zero 4-vector)
        if (ln < 6) yv = -a.eePos[(size_t)r * 6 + ln] + (ln % 3 == 2 ? 0.02 : 0.0);
        else if (ln < 12) yv = -a.eeVel[(size_t)r * 6 + ln - 6];
        y[ln] = yv;
    }
    if (ln == 0) {
        // accel = R(quatToZyx(q))' a_local + g  (include/stateEstimator.h:280-281)
        const double *qq = a.quat + (size_t)r * 4;
        const double x = qq[0], yy = qq[1], z = qq[2], w = qq[3];
        double as = -2. * (x * z - w * yy);
        as = as < .99999 ? as : .99999;
        const double e0 = atan2(2 * (x * yy + w * z), w * w + x * x - yy * yy - z * z);
        const double e1 = asin(as);
        const double e2 = atan2(2 * (yy * z + w * x), w * w - x * x - yy * yy + z * z);
        const double c1 = cos(e0), c2 = cos(e1), c3 = cos(e2), s1 = sin(e0), s2 = sin(e1),
                     s3 = sin(e2);
        const double Rm[9] = {c1 * c2, c2 * s1, -s2,                           // column 0
                              c1 * s2 * s3 - s1 * c3, s1 * s2 * s3 + c1 * c3, c2 * s3,
                              c1 * s2 * c3 + s1 * s3, s1 * s2 * c3 - c1 * s3, c2 * c3};
        const double *al = a.acc + (size_t)r * 3;
        for (int i = 0; i < 3; ++i) {
            double s = 0.0;
            for (int l = 0; l < 3; ++l) s += Rm[i * 3 + l] * al[l];  // (R')(i, l) = R(l, i)
            accw[i] = s + (i == 2 ? -9.81 : 0.0);
        }
    }
    __syncthreads();
    // x- = A x + B accel, A = I + dt E(0:3, 3:6), B = [dt^2/2 I; dt I; 0]
    if (ln < 12) {
        const double *x = a.xhat + (size_t)r * 12;
        double v = x[ln];
        if (ln < 3) v = v + dt * x[ln + 3] + 0.5 * dt * dt * accw[ln];
        else if (ln < 6) v = v + dt * accw[ln - 3];
        xn[ln] = v;
    }
    // Pm = A P A' + Q
    for (int e = ln; e < 144; e += 64) {
        const int i = e % 12, j = e / 12;
        auto AP = [&](int ii, int jj) {  // (A P)(ii, jj)
            return P[jj * 12 + ii] + (ii < 3 ? dt * P[jj * 12 + ii + 3] : 0.0);
        };
        double v = AP(i, j) + (j < 3 ? dt * AP(i, j + 3) : 0.0);
        Pm[e] = v + (i == j ? qd[i] : 0.0);
    }
    __syncthreads();
    // PC = Pm C' (12 x 14)
    for (int e = ln; e < 168; e += 64) {
        const int i = e % 12, j = e / 12;
        double s = 0.0;
        for (int l = 0; l < 12; ++l) s += Pm[l * 12 + i] * kf_c(j, l);
        PC[e] = s;
    }
    __syncthreads();
    // augmented W = [S | ey | C], S = C PC + R, ey = y - C x-   (14 x 27, column-major)
    for (int e = ln; e < 14 * 27; e += 64) {
        const int i = e % 14, j = e / 14;
        double v;
        if (j < 14) {
            double s = 0.0;
            for (int l = 0; l < 12; ++l) s += kf_c(i, l) * PC[j * 12 + l];
            v = s + (i == j ? rd[i] : 0.0);
        } else if (j == 14) {
            double s = 0.0;
            for (int l = 0; l < 12; ++l) s += kf_c(i, l) * xn[l];
            v = y[i] - s;
        } else {
            v = kf_c(i, j - 15);
        }
        W[e] = v;
    }
    __syncthreads();
    // partial-pivot LU (first maximum), lane j owns column j, then back substitution of the
    // 13 right-hand sides
    for (int k = 0; k < 14; ++k) {
        int p = k;
        double amax = fabs(W[k * 14 + k]);
        for (int i = k + 1; i < 14; ++i) {
            const double v = fabs(W[k * 14 + i]);
            if (v > amax) { amax = v; p = i; }
        }
        const double piv = W[k * 14 + p];
        __syncthreads();
        if (ln < 27 && p != k) {
            const double t = W[ln * 14 + k];
            W[ln * 14 + k] = W[ln * 14 + p];
            W[ln * 14 + p] = t;
        }
        __syncthreads();
        if (ln > k && ln < 27)
            for (int i = k + 1; i < 14; ++i) W[ln * 14 + i] -= (W[k * 14 + i] / piv) * W[ln * 14 + k];
        __syncthreads();
    }
    if (ln >= 14 && ln < 27) {
        for (int i = 13; i >= 0; --i) {
            double s = W[ln * 14 + i];
            for (int l = i + 1; l < 14; ++l) s -= W[l * 14 + i] * W[ln * 14 + l];
            W[ln * 14 + i] = s / W[i * 14 + i];
        }
    }
    __syncthreads();
    // x+ = x- + PC sEy;  P+ = sym((I - PC sC) Pm), then the decoupling of P(0:2, 0:2)
    if (ln < 12) {
        double s = 0.0;
        for (int l = 0; l < 14; ++l) s += PC[l * 12 + ln] * W[14 * 14 + l];
        a.xhat[(size_t)r * 12 + ln] = xn[ln] + s;
    }
    for (int e = ln; e < 144; e += 64) {  // K = I - PC sC into P (P is free now)
        const int i = e % 12, j = e / 12;
        double s = 0.0;
        for (int l = 0; l < 14; ++l) s += PC[l * 12 + i] * W[(15 + j) * 14 + l];
        P[e] = (i == j ? 1.0 : 0.0) - s;
    }
    __syncthreads();
    for (int e = ln; e < 144; e += 64) {  // Pn = K Pm into PC (reused)
        const int i = e % 12, j = e / 12;
        double s = 0.0;
        for (int l = 0; l < 12; ++l) s += P[l * 12 + i] * Pm[j * 12 + l];
        PC[e] = s;
    }
    __syncthreads();
    for (int e = ln; e < 144; e += 64) {
        const int i = e % 12, j = e / 12;
        Pm[e] = (PC[j * 12 + i] + PC[i * 12 + j]) / 2.0;
    }
    __syncthreads();
    const double det = Pm[0] * Pm[13] - Pm[12] * Pm[1];
    for (int e = ln; e < 144; e += 64) {
        const int i = e % 12, j = e / 12;
        double v = Pm[e];
        if (det > 0.000001) {
            if ((i < 2) != (j < 2)) v = 0.0;
            else if (i < 2 && j < 2) v /= 10.;
        }
        a.P[(size_t)r * 144 + e] = v;
    }
}

int hip_rc(hipError_t e) { return e == hipSuccess ? MPCQP_OK : MPCQP_ERR_DEVICE; }

bool device_present() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

}  // namespace

extern "C" {

int mpcqp_fk_feet(void *stream, int R, const double *q, const double *rpy, int rpy_stride,
                  double *feet) {
    if (!q || !rpy || !feet || R < 0 || rpy_stride < 3) return MPCQP_ERR_BAD_ARG;
    if (R == 0) return MPCQP_OK;
    if (!device_present()) return MPCQP_ERR_NO_DEVICE;
    hipLaunchKernelGGL(k_fk_feet, dim3((R + 255) / 256), dim3(256), 0, (hipStream_t)stream, R, q,
                       rpy, rpy_stride, feet);
    return hip_rc(hipGetLastError());
}

int mpcqp_kf_update(void *stream, int R, double dt, double *xhat, double *P, const double *eePos,
                    const double *eeVel, const unsigned char *contact, const double *quat,
                    const double *acc) {
    if (!xhat || !P || !eePos || !eeVel || !contact || !quat || !acc || R < 0)
        return MPCQP_ERR_BAD_ARG;
    if (R == 0) return MPCQP_OK;
    if (!device_present()) return MPCQP_ERR_NO_DEVICE;
    KfArgs a{R, dt, xhat, P, eePos, eeVel, contact, quat, acc};
    hipLaunchKernelGGL(k_kf_update, dim3(R), dim3(64), 0, (hipStream_t)stream, a);
    return hip_rc(hipGetLastError());
}

}  // extern "C"
