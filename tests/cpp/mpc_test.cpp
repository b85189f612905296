// C++ closed-loop harness through the header-only QPSolver mirror (mpcqp::QPSolverD), the flow
// of the reference's src/linear_mpc_example.cpp:108-195 (mpc_test): the plant written as
// damping / mass, linear_mpc_example's quadrature Bd (:35-46, discretizeSystemQuadrature), xi
// carried from (2,0,0,0) by xi = Ad xi + Bd u (:124, 182), the circle reference at
// t = k Ts + i Ts, [A_eq; A_ineq] stacked as the harness stacks them (corrected on the GPU).
// Prints one line per tick: k u0 u1 x0 x1 x2 x3 status corrected (%.17g) for tests/test_cpp.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "mpcqp/qpsolver.hpp"

using mpcqp::DMat;

int main(int argc, char **argv) {
    const int ticks = argc > 1 ? std::atoi(argv[1]) : 500;
    const int N = 15;
    const double damping = 0.02, mass = 0.2, Ts = 0.01;
    DMat Ac(4, 4), Bc(4, 2), Q(4, 4), R(2, 2), P(4, 4), x_min(4), x_max(4);
    Ac(0, 1) = 1; Ac(1, 1) = -damping / mass; Ac(2, 3) = 1; Ac(3, 3) = -damping / mass;
    Bc(1, 0) = 1 / mass; Bc(3, 1) = 1 / mass;
    const double qd[4] = {50, 5, 50, 5}, xm[4] = {-5, -3, -5, -3};
    for (int i = 0; i < 4; ++i) {
        Q(i, i) = qd[i];
        P(i, i) = 20 * qd[i];
        x_min(i) = xm[i];
        x_max(i) = -xm[i];
    }
    R(0, 0) = R(1, 1) = 0.1;
    mpcqp::QPSolverD qp(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, -8.0, 8.0);
    qp.discretizeSystemQuadrature();

    DMat xi(4);
    xi(0) = 2.0;
    qp.setState(xi);
    const double radius = 2.0, angular_vel = 0.5;
    for (int k = 0; k < ticks; ++k) {
        DMat xi_ref(4, N + 1);
        for (int i = 0; i <= N; ++i) {
            const double t = k * Ts + i * Ts;
            const double theta = angular_vel * t;
            xi_ref(0, i) = radius * std::cos(theta);
            xi_ref(2, i) = radius * std::sin(theta);
            xi_ref(1, i) = -radius * angular_vel * std::sin(theta);
            xi_ref(3, i) = radius * angular_vel * std::cos(theta);
        }
        DMat H, f, A_eq, b_eq, lb, ub, A_ineq, lbA, ubA;
        qp.buildQPParams(xi, xi_ref, H, f, A_eq, b_eq, lb, ub, A_ineq, lbA, ubA);
        const long ne = A_eq.rows(), ni = A_ineq.rows(), nv = H.rows();
        DMat A_total(ne + ni, nv), lbA_total(ne + ni), ubA_total(ne + ni);
        for (long c = 0; c < nv; ++c) {
            for (long r = 0; r < ne; ++r) A_total(r, c) = A_eq(r, c);
            for (long r = 0; r < ni; ++r) A_total(ne + r, c) = A_ineq(r, c);
        }
        for (long r = 0; r < ne; ++r) lbA_total(r) = ubA_total(r) = b_eq(r);
        for (long r = 0; r < ni; ++r) {
            lbA_total(ne + r) = lbA(r);
            ubA_total(ne + r) = ubA(r);
        }
        DMat U_opt(2, N);
        if (!qp.solveQP(H, f, A_total, lb, ub, lbA_total, ubA_total, U_opt)) return 1;
        DMat u(2);
        u(0) = U_opt(0, 0);
        u(1) = U_opt(1, 0);
        qp.updateState(u);  // xi = Ad xi + Bd u on the GPU
        const DMat &s = qp.getState();
        for (int i = 0; i < 4; ++i) xi(i) = s(i);
        std::printf("%d %.17g %.17g %.17g %.17g %.17g %.17g %d %d\n", k, u(0), u(1), xi(0), xi(1),
                    xi(2), xi(3), qp.lastStatus(), (int)qp.corrected());
    }
    return 0;
}
