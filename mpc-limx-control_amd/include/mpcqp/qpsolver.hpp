// qpsolver.hpp -- C++ host mirror of the reference's QPSolver (include/QPSolver.h:10-56) over
// the libmpcqp C ABI (include/mpcqp.h).  Header-only; every numerical step runs on the GPU.
//
//   QPSolver(Ts, N, Ac, Bc, Q, R, P, x_min, x_max, u_min, u_max)   src/QPSolver.cpp:3-19
//   discretizeSystem()                                               src/QPSolver.cpp:21-29
//   buildQPParams(xi0, xi_ref, H, f, A_eq, b_eq, lb, ub, A_ineq, lbA, ubA)
//                                                                    src/QPSolver.cpp:31-81
//   solveQP(H, f, A_total, lb, ub, lbA_total, ubA_total, U_opt)      src/QPSolver.cpp:83-106
//   updateState(u), getState()                                       src/QPSolver.cpp:108-116
//
// BasicQPSolver<Mat, Vec> works with any column-major dense types offering rows(), cols(),
// size(), data() and resize(): Eigen::MatrixXd / VectorXd (compat/QPSolver.h) or the DMat
// below.  Behaviour kept from the reference: solveQP returns true and only reports a failed
// status (stderr), the internal state xi starts at zero, updateState/getState print the state
// (switchable).  Differences: A_total is read column-major as Eigen stores it (the reference
// hands it to a row-major API), the status is kept in lastStatus(), and when
// the harness-stacked [A_eq; A_ineq] problem is infeasible (always) the
// equality block is dropped and the corrected QP is solved (corrected() == true).
#pragma once
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mpcqp.h"

namespace mpcqp {

// minimal column-major dense matrix / vector (Eigen-shaped API subset)
class DMat {
  public:
    DMat() = default;
    DMat(long r, long c) : r_(r), c_(c), v_((size_t)(r * c), 0.0) {}
    explicit DMat(long n) : r_(n), c_(1), v_((size_t)n, 0.0) {}
    long rows() const { return r_; }
    long cols() const { return c_; }
    long size() const { return r_ * c_; }
    void resize(long r, long c) { r_ = r; c_ = c; v_.assign((size_t)(r * c), 0.0); }
    void resize(long n) { resize(n, 1); }
    double *data() { return v_.data(); }
    const double *data() const { return v_.data(); }
    double &operator()(long i, long j) { return v_[(size_t)(j * r_ + i)]; }
    double operator()(long i, long j) const { return v_[(size_t)(j * r_ + i)]; }
    double &operator()(long i) { return v_[(size_t)i]; }
    double operator()(long i) const { return v_[(size_t)i]; }
    double &operator[](long i) { return v_[(size_t)i]; }
    double operator[](long i) const { return v_[(size_t)i]; }

  private:
    long r_ = 0, c_ = 0;
    std::vector<double> v_;
};

inline void check(int rc, const char *what) {
    if (rc != MPCQP_OK && rc != MPCQP_ERR_INFEASIBLE && rc != MPCQP_ERR_ITER_LIMIT &&
        rc != MPCQP_ERR_NOT_PD)
        throw std::runtime_error(std::string(what) + ": " + mpcqp_status_string(rc));
}

template <class Mat, class Vec>
class BasicQPSolver {
  public:
    BasicQPSolver(double Ts, int N, const Mat &Ac, const Mat &Bc, const Mat &Q, const Mat &R,
                  const Mat &P, const Vec &x_min, const Vec &x_max, double u_min, double u_max)
        : Ts_(Ts), N_(N), Ac_(Ac), Bc_(Bc), Q_(Q), R_(R), P_(P), x_min_(x_min), x_max_(x_max),
          u_min_(u_min), u_max_(u_max) {
        NX_ = (int)Ac.rows();
        NU_ = (int)Bc.cols();
        xi_.resize(NX_);
        for (int i = 0; i < NX_; ++i) xi_.data()[i] = 0.0;  // src/QPSolver.cpp:12
        discretizeSystem();
    }

    void discretizeSystem() {
        Ad_.resize(NX_, NX_);
        Bd_.resize(NX_, NU_);
        check(mpcqp_discretize(NX_, NU_, Ts_, Ac_.data(), Bc_.data(), Ad_.data(), Bd_.data()),
              "mpcqp_discretize");
    }

    // linear_mpc_example's own discretisation (src/linear_mpc_example.cpp:35-46): Ad = exp(Ac Ts),
    // Bd by the 100-step quadrature, used by the mpc_test harness instead of discretizeSystem
    void discretizeSystemQuadrature() {
        Ad_.resize(NX_, NX_);
        Bd_.resize(NX_, NU_);
        check(mpcqp_discretize_quadrature(NX_, NU_, Ts_, Ac_.data(), Bc_.data(), Ad_.data(),
                                          Bd_.data()),
              "mpcqp_discretize_quadrature");
    }

    // mpc_test carries its own xi from (2,0,0,0) (src/linear_mpc_example.cpp:124,182); the
    // reference QPSolver has no setter (its xi starts at zero, src/QPSolver.cpp:12)
    template <class V0>
    void setState(const V0 &xi) {
        for (int i = 0; i < NX_; ++i) xi_.data()[i] = xi.data()[i];
    }

    template <class V0, class M0>
    void buildQPParams(const V0 &xi0, const M0 &xi_ref, Mat &H, Vec &f, Mat &A_eq, Vec &b_eq,
                       Vec &lb, Vec &ub, Mat &A_ineq, Vec &lbA_ineq, Vec &ubA_ineq) {
        const int nV = NU_ * N_, NE = NX_ * N_, NI = 2 * NX_ * N_;
        H.resize(nV, nV);
        f.resize(nV);
        A_eq.resize(NE, nV);
        b_eq.resize(NE);
        lb.resize(nV);
        ub.resize(nV);
        A_ineq.resize(NI, nV);
        lbA_ineq.resize(NI);
        ubA_ineq.resize(NI);
        check(mpcqp_build_qp(NX_, NU_, N_, Ad_.data(), Bd_.data(), Q_.data(), R_.data(),
                             P_.data(), x_min_.data(), x_max_.data(), u_min_, u_max_,
                             xi0.data(), xi_ref.data(), H.data(), f.data(), A_eq.data(),
                             b_eq.data(), lb.data(), ub.data(), A_ineq.data(), lbA_ineq.data(),
                             ubA_ineq.data()),
              "mpcqp_build_qp");
    }

    template <class MU>
    bool solveQP(const Mat &H, const Vec &f, const Mat &A_total, const Vec &lb, const Vec &ub,
                 const Vec &lbA_total, const Vec &ubA_total, MU &U_opt) {
        const int nV = NU_ * N_, nC = (int)A_total.rows();
        std::vector<double> x((size_t)nV, 0.0);
        int nwsr = 50000;  // src/QPSolver.cpp:92
        double cost = 0.0;
        int st = mpcqp_solve_dense(nV, nC, H.data(), f.data(), A_total.data(), MPCQP_A_COLMAJOR,
                                   lb.data(), ub.data(), lbA_total.data(), ubA_total.data(),
                                   &nwsr, x.data(), nullptr, &cost);
        check(st, "mpcqp_solve_dense");
        corrected_ = false;
        const int NE = NX_ * N_;
        if (st == MPCQP_ERR_INFEASIBLE && nC == NE + 2 * NX_ * N_) {
            // the harness's [A_eq; A_ineq] stack (src/qpSolver_test.cpp:58-63) is infeasible
            // by construction: solve the corrected QP (bounds + A_ineq rows)
            std::vector<double> Ain((size_t)(nC - NE) * nV);
            for (int c = 0; c < nV; ++c)
                for (int r = NE; r < nC; ++r)
                    Ain[(size_t)c * (nC - NE) + (r - NE)] = A_total.data()[(size_t)c * nC + r];
            nwsr = 50000;
            st = mpcqp_solve_dense(nV, nC - NE, H.data(), f.data(), Ain.data(), MPCQP_A_COLMAJOR,
                                   lb.data(), ub.data(), lbA_total.data() + NE,
                                   ubA_total.data() + NE, &nwsr, x.data(), nullptr, &cost);
            check(st, "mpcqp_solve_dense");
            corrected_ = true;
        }
        last_status_ = st;
        last_iters_ = nwsr;
        last_cost_ = cost;
        if (st != MPCQP_OK) std::fprintf(stderr, "QP solve failed, status: %s\n", mpcqp_status_string(st));
        for (int i = 0; i < nV && i < (int)U_opt.size(); ++i) U_opt.data()[i] = x[(size_t)i];
        return true;  // the reference returns true regardless (src/QPSolver.cpp:105)
    }

    template <class VU>
    void updateState(const VU &u) {
        std::vector<double> x(xi_.data(), xi_.data() + NX_);
        check(mpcqp_plant_step(NX_, NU_, Ad_.data(), Bd_.data(), x.data(), u.data()),
              "mpcqp_plant_step");
        for (int i = 0; i < NX_; ++i) xi_.data()[i] = x[(size_t)i];
        if (verbose) print_state();
    }

    const Vec &getState() {
        if (verbose) print_state();
        return xi_;
    }

    int lastStatus() const { return last_status_; }
    int lastIters() const { return last_iters_; }
    double lastCost() const { return last_cost_; }
    bool corrected() const { return corrected_; }
    const Mat &Ad() const { return Ad_; }
    const Mat &Bd() const { return Bd_; }
    bool verbose = false;  // the reference prints xi in updateState/getState

  private:
    void print_state() const {
        for (int i = 0; i < NX_; ++i) std::printf(i ? " %g" : "%g", xi_.data()[i]);
        std::printf("\n");
    }
    double Ts_;
    int N_, NX_ = 0, NU_ = 0;
    Mat Ac_, Bc_, Q_, R_, P_, Ad_, Bd_;
    Vec x_min_, x_max_;
    double u_min_, u_max_;
    Vec xi_;
    int last_status_ = MPCQP_OK, last_iters_ = 0;
    double last_cost_ = 0.0;
    bool corrected_ = false;
};

using QPSolverD = BasicQPSolver<DMat, DMat>;

}  // namespace mpcqp
