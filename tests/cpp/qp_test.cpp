// C++ closed-loop harness through the header-only QPSolver mirror (mpcqp::QPSolverD), the
// flow of the reference's src/qpSolver_test.cpp:4-91 (4/2/15 plant, circle reference of radius
// 2 at 0.5 rad/s, [A_eq; A_ineq] stacked as the reference stacks them, U_opt.col(0) applied).
// Prints one line per tick: k x0 x1 x2 x3 status corrected (%.17g) for tests/test_cpp.py.
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "mpcqp/qpsolver.hpp"

using mpcqp::DMat;

int main(int argc, char **argv) {
    const int ticks = argc > 1 ? std::atoi(argv[1]) : 500;
    const double Ts = 0.01;
    const int N = 15;
    DMat Ac(4, 4), Bc(4, 2), Q(4, 4), R(2, 2), P(4, 4), x_min(4), x_max(4);
    Ac(0, 1) = 1; Ac(1, 1) = -0.1; Ac(2, 3) = 1; Ac(3, 3) = -0.1;
    Bc(1, 0) = 5; Bc(3, 1) = 5;
    const double qd[4] = {50, 5, 50, 5}, xm[4] = {-5, -3, -5, -3};
    for (int i = 0; i < 4; ++i) {
        Q(i, i) = qd[i];
        P(i, i) = 20 * qd[i];
        x_min(i) = xm[i];
        x_max(i) = -xm[i];
    }
    R(0, 0) = R(1, 1) = 0.1;
    mpcqp::QPSolverD qp(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, -8.0, 8.0);

    DMat xi(4);
    xi(0) = 2.0;  // the harness's x0; the solver's own state starts at zero (quirk kept)
    for (int k = 0; k < ticks; ++k) {
        DMat xi_ref(4, N + 1);
        for (int i = 0; i <= N; ++i) {
            const double th = 0.5 * (k * Ts + i * Ts);
            xi_ref(0, i) = 2.0 * std::cos(th);
            xi_ref(2, i) = 2.0 * std::sin(th);
            xi_ref(1, i) = -2.0 * 0.5 * std::sin(th);
            xi_ref(3, i) = 2.0 * 0.5 * std::cos(th);
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
        qp.updateState(u);
        const DMat &s = qp.getState();
        for (int i = 0; i < 4; ++i) xi(i) = s(i);
        std::printf("%d %.17g %.17g %.17g %.17g %d %d\n", k, xi(0), xi(1), xi(2), xi(3),
                    qp.lastStatus(), (int)qp.corrected());
    }
    return 0;
}
