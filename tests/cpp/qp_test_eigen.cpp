// The reference harness's call pattern (src/qpSolver_test.cpp:4-91: Eigen fixed-size types,
// comma initialisers, QPSolver(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, u_min, u_max),
// buildQPParams, [A_eq; A_ineq] stacked with <<, solveQP into Matrix<double, 2, 15>,
// U_opt.col(0), updateState, getState) against the DROP-IN header compat/QPSolver.h and
// compat/MPCParam.h -- compiled here with the test-only Eigen stand-in
// (tests/cpp/eigen_shim), linked to libmpcqp.so.  One line per tick: k x0 x1 x2 x3 status
// corrected (%.17g), the format of tests/cpp/qp_test.cpp.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "MPCParam.h"
#include "QPSolver.h"

int main(int argc, char **argv) {
    const int ticks = argc > 1 ? std::atoi(argv[1]) : 500;
    const double Ts = 0.01;
    const int N = 15;
    Eigen::Matrix4d Ac;
    Eigen::Matrix<double, 4, 2> Bc;
    Ac << 0, 1, 0, 0,  //
        0, -0.1, 0, 0,  //
        0, 0, 0, 1,     //
        0, 0, 0, -0.1;
    Bc << 0, 0,  //
        5, 0,    //
        0, 0,    //
        0, 5;
    const Eigen::Matrix4d Q = (Eigen::Vector4d() << 50, 5, 50, 5).finished().asDiagonal();
    const Eigen::Matrix2d R = 0.1 * Eigen::Matrix2d::Identity();
    const Eigen::Matrix4d P = 20 * Q;
    const Eigen::Vector4d x_min = (Eigen::Vector4d() << -5, -3, -5, -3).finished();
    const Eigen::Vector4d x_max = -x_min;
    QPSolver solver(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, -8.0, 8.0);

    Eigen::Vector4d xi(2, 0, 0, 0);  // the harness's start; the solver's own state is zero
    for (int k = 0; k < ticks; ++k) {
        Eigen::Matrix<double, 4, 16> xi_ref;
        for (int i = 0; i <= N; ++i) {
            const double th = 0.5 * (k * Ts + i * Ts);
            xi_ref(0, i) = 2.0 * std::cos(th);
            xi_ref(1, i) = -2.0 * 0.5 * std::sin(th);
            xi_ref(2, i) = 2.0 * std::sin(th);
            xi_ref(3, i) = 2.0 * 0.5 * std::cos(th);
        }
        Eigen::MatrixXd H, A_eq, A_ineq;
        Eigen::VectorXd f, b_eq, lb, ub, lbA_ineq, ubA_ineq;
        solver.buildQPParams(xi, xi_ref, H, f, A_eq, b_eq, lb, ub, A_ineq, lbA_ineq, ubA_ineq);
        Eigen::MatrixXd A_total(A_eq.rows() + A_ineq.rows(), 2 * N);
        A_total << A_eq, A_ineq;
        Eigen::VectorXd lbA_total(b_eq.size() + lbA_ineq.size());
        lbA_total << b_eq, lbA_ineq;
        Eigen::VectorXd ubA_total(b_eq.size() + ubA_ineq.size());
        ubA_total << b_eq, ubA_ineq;
        Eigen::Matrix<double, 2, 15> U_opt;
        if (!solver.solveQP(H, f, A_total, lb, ub, lbA_total, ubA_total, U_opt)) return 1;
        Eigen::Vector2d u = U_opt.col(0);
        solver.updateState(u);
        xi = solver.getState();
        const Eigen::Vector2d pos(xi.transpose()[0], xi.transpose()[2]);
        const Eigen::Vector2d ref(xi_ref(0, 0), xi_ref(2, 0));
        if (!std::isfinite((pos - ref).norm())) return 3;
        std::printf("%d %.17g %.17g %.17g %.17g %d %d\n", k, xi(0), xi(1), xi(2), xi(3),
                    solver.lastStatus(), solver.corrected() ? 1 : 0);
    }
    MPCParam param;  // the compat parameter struct compiles and carries the reference's offsets
    std::cerr << "foot offset left: " << param.static_foot_offset_left.transpose() << "\n";
    return 0;
}
