// compat/QPSolver.h -- drop-in for the reference's include/QPSolver.h
// (Fleming-Sung/mpc-limX-control): same class name and method names; the Eigen types of the
// reference's signatures (include/QPSolver.h:13-37) are accepted, the work runs on MI355X
// through libmpcqp.so.  Put this directory ahead of the reference's include/ and link
// libmpcqp.so instead of QPSolver.cpp + qpOASES.
//
// Source compatibility: the reference's fixed-size arguments (Eigen::Vector4d xi0,
// Eigen::Matrix<double,2,15>& U_opt, Eigen::Vector2d& u) bind to the templated members, and so
// do generic VectorXd / MatrixXd, so the 13-state models compile too.  getState() returns a
// VectorXd, which assigns to Eigen::Vector4d for the 4-state harness.
#ifndef MPCQP_COMPAT_QP_SOLVER_H
#define MPCQP_COMPAT_QP_SOLVER_H

#if __has_include(<Eigen/Dense>)
#include <Eigen/Dense>

#include "../include/mpcqp/qpsolver.hpp"

class QPSolver : public mpcqp::BasicQPSolver<Eigen::MatrixXd, Eigen::VectorXd> {
  public:
    using mpcqp::BasicQPSolver<Eigen::MatrixXd, Eigen::VectorXd>::BasicQPSolver;
    Eigen::VectorXd getState() { return BasicQPSolver::getState(); }
};

#else
#error "compat/QPSolver.h needs Eigen 3 (as the reference does); without Eigen use <mpcqp/qpsolver.hpp> (mpcqp::QPSolverD)"
#endif

#endif
