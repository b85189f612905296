// convex_mpc.hpp -- C++ controller-side front end of the batched engine: the call a TRON1
// controller makes once per MPC tick from MPC::computeSupportFootForce
// (include/MPCController.h:36, empty in the reference).  Header-only over the
// C ABI (include/mpcqp.h).
//
//   srbm_model(N, friction)   model constants of include/mpcQP.h:18-60 plus the build-chosen
//                             force bounds / R of the 6-input SRBM
//   gait_contact_mask(...)    MPC::calculateGait (include/MPCController.h:61-75) per horizon step
//   ConvexMpc                 owns one mpcqp_ctx; solve() runs C gait candidates of one state
//                             and returns the minimum-cost one (lowest index on ties, fp32 cost,
//                             the same rule as mpcqp_batch_select_min and the multi-GPU path)
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/mpcqp.h"

namespace mpcqp {

constexpr double kMass = 9.585;  // include/mpcQP.h:18
constexpr double kGravity = 9.8;
constexpr double kTs = 0.001;    // include/mpcQP.h:37
constexpr double kMu = 0.6;
constexpr double kRSrbm = 1e-5;

struct ModelSpec {
    mpcqp_model m{};
    std::vector<double> Q, R, P;  // column-major, owned (m.Q/R/P point here)
    ModelSpec() = default;
    ModelSpec(const ModelSpec &o) : m(o.m), Q(o.Q), R(o.R), P(o.P) { rebind(); }
    ModelSpec &operator=(const ModelSpec &o) {
        m = o.m; Q = o.Q; R = o.R; P = o.P;
        rebind();
        return *this;
    }
    void rebind() { m.Q = Q.data(); m.R = R.data(); m.P = P.data(); }
};

// 13-state / 6-input convex-MPC model (SRBM), horizon N, box or box + friction pyramid
inline ModelSpec srbm_model(int N, bool friction) {
    static const double qd[13] = {1, 1, 10, 100, 100, 100, 50, 50, 50, 100, 100, 100, 0.1};
    static const double Ib[9] = {140110.479e-06, 534.939e-06,    28184.116e-06,
                                 534.939e-06,    110641.449e-06, -27.278e-06,
                                 28184.116e-06,  -27.278e-06,    98944.542e-06};  // :20-22
    ModelSpec s;
    s.Q.assign(169, 0.0);
    s.P.assign(169, 0.0);
    s.R.assign(36, 0.0);
    for (int i = 0; i < 13; ++i) {
        s.Q[i * 14] = qd[i];
        s.P[i * 14] = 20.0 * qd[i];  // P = 20 Q, include/mpcQP.h:56
    }
    for (int i = 0; i < 6; ++i) s.R[i * 7] = kRSrbm;
    mpcqp_model &m = s.m;
    m.nx = 13;
    m.nu = 6;
    m.N = N;
    m.model = MPCQP_MODEL_SRBM;
    m.constraints = friction ? MPCQP_CONS_FRICTION : MPCQP_CONS_BOX;
    m.Ts = kTs;
    m.mass = kMass;
    m.mu = kMu;
    std::memcpy(m.Ib, Ib, sizeof(Ib));
    m.fz_min = 0.0;
    m.fz_max = 4.0 * kMass * kGravity;
    m.fxy_max = kMu * m.fz_max;
    m.u_min = -8.0;
    m.u_max = 8.0;
    m.max_iter = 0;
    m.max_free = 0;  // nu N: every contact schedule (double support, standing)
    s.rebind();
    return s;
}

// bit 2k = left foot in contact at step k, bit 2k+1 = right; swing/stance are MPCParam floats
inline uint64_t gait_contact_mask(int N, double Ts, double phase0, float swing = 0.5f,
                                  float stance = 0.5f) {
    const double cycle = (double)(swing + stance);
    uint64_t mask = 0;
    for (int k = 0; k < N; ++k) {
        double ph = std::fmod(phase0 + (double)k * Ts, cycle);
        mask |= (ph < (double)swing) ? (1ull << (2 * k + 1)) : (1ull << (2 * k));
    }
    return mask;
}

struct MpcChoice {
    int index = -1;       // winning candidate (-1: none solved)
    double cost = 0.0;    // its objective value
    std::vector<double> U;  // nu x N column-major (U.col(0) = first step forces)
    std::vector<int> status;  // per-candidate MPCQP_* status
};

class ConvexMpc {
  public:
    explicit ConvexMpc(const ModelSpec &spec, int device = 0) : spec_(spec) {
        int rc = mpcqp_ctx_create(&spec_.m, device, &ctx_);
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_ctx_create: ") + mpcqp_status_string(rc));
    }
    ~ConvexMpc() { if (ctx_) mpcqp_ctx_destroy(ctx_); }
    ConvexMpc(const ConvexMpc &) = delete;
    ConvexMpc &operator=(const ConvexMpc &) = delete;

    int nx() const { return spec_.m.nx; }
    int nu() const { return spec_.m.nu; }
    int N() const { return spec_.m.N; }
    mpcqp_ctx *ctx() { return ctx_; }

    // One tick: the same state x0 [nx], reference xref [(N+1) nx] and lever arms lin [8] for
    // every candidate contact schedule; returns the cheapest candidate's plan.
    MpcChoice solve(const double *x0, const double *xref, const double *lin,
                    const uint64_t *contacts, int C) {
        const int nx_ = nx(), xr = (N() + 1) * nx_;
        bx0_.resize((size_t)C * nx_);
        bxr_.resize((size_t)C * xr);
        blin_.resize((size_t)C * 8);
        for (int c = 0; c < C; ++c) {
            std::memcpy(&bx0_[(size_t)c * nx_], x0, sizeof(double) * nx_);
            std::memcpy(&bxr_[(size_t)c * xr], xref, sizeof(double) * xr);
            std::memcpy(&blin_[(size_t)c * 8], lin, sizeof(double) * 8);
        }
        return solve_batch(bx0_.data(), bxr_.data(), blin_.data(), contacts, C);
    }

    // General form: C independent instances (host arrays in the mpcqp.h instance-major layout)
    MpcChoice solve_batch(const double *x0, const double *xref, const double *lin,
                          const uint64_t *contacts, int C) {
        const int nv = nu() * N();
        U_.resize((size_t)C * nv);
        cost_.resize((size_t)C);
        iters_.resize((size_t)C);
        MpcChoice out;
        out.status.resize((size_t)C);
        int rc = mpcqp_batch_solve_host(ctx_, C, x0, xref, lin, contacts, U_.data(), cost_.data(),
                                        out.status.data(), iters_.data());
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_batch_solve_host: ") + mpcqp_status_string(rc));
        float best = std::numeric_limits<float>::infinity();
        for (int c = 0; c < C; ++c) {
            if (out.status[(size_t)c] != MPCQP_OK) continue;
            float v = (float)cost_[(size_t)c];
            if (out.index < 0 || v < best) { best = v; out.index = c; }
        }
        if (out.index >= 0) {
            out.cost = cost_[(size_t)out.index];
            out.U.assign(U_.begin() + (size_t)out.index * nv, U_.begin() + (size_t)(out.index + 1) * nv);
        }
        return out;
    }

    const std::vector<double> &all_U() const { return U_; }
    const std::vector<double> &all_cost() const { return cost_; }
    const std::vector<int> &all_iters() const { return iters_; }

  private:
    ModelSpec spec_;
    mpcqp_ctx *ctx_ = nullptr;
    std::vector<double> bx0_, bxr_, blin_, U_, cost_;
    std::vector<int> iters_;
};

// The batch of S states x C gait candidates over several GPUs of one node, from one controller
// process: mpcqp_group (one context per device, the library's RCCL communicator, ONE all-gather
// of the selection records per tick).  The choice is the global minimum (fp32 cost, lowest
// global index), the same rule as ConvexMpc::solve_batch and the multi-process path.
class GroupMpc {
  public:
    GroupMpc(const ModelSpec &spec, const std::vector<int> &devices) : spec_(spec) {
        int rc = mpcqp_group_create(&spec_.m, (int)devices.size(), devices.data(), &g_);
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_group_create: ") + mpcqp_status_string(rc));
    }
    ~GroupMpc() { if (g_) mpcqp_group_destroy(g_); }
    GroupMpc(const GroupMpc &) = delete;
    GroupMpc &operator=(const GroupMpc &) = delete;

    mpcqp_group *group() { return g_; }

    // S states x C candidates (host arrays, the mpcqp.h instance-major layout, instance s*C + c)
    MpcChoice solve_batch(const double *x0, const double *xref, const double *lin,
                          const uint64_t *contacts, int S, int C) {
        const int nv = spec_.m.nu * spec_.m.N;
        const size_t B = (size_t)S * C;
        U_.resize(B * nv);
        cost_.resize(B);
        iters_.resize(B);
        rec_.resize(1 + (size_t)nv);
        MpcChoice out;
        out.status.resize(B);
        int rc = mpcqp_group_solve_select_host(g_, S, C, x0, xref, lin, contacts, U_.data(),
                                               cost_.data(), out.status.data(), iters_.data(),
                                               rec_.data());
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_group_solve_select_host: ") + mpcqp_status_string(rc));
        if (rec_[0] != INT64_MAX) {
            out.index = (int)(rec_[0] & 0x7fffffff);
            out.cost = cost_[(size_t)out.index];
            out.U.resize((size_t)nv);
            std::memcpy(out.U.data(), &rec_[1], sizeof(double) * nv);  // the record's U bits
        }
        return out;
    }

    const std::vector<double> &all_U() const { return U_; }
    const std::vector<double> &all_cost() const { return cost_; }
    const std::vector<int> &all_iters() const { return iters_; }
    const std::vector<int64_t> &record() const { return rec_; }

  private:
    ModelSpec spec_;
    mpcqp_group *g_ = nullptr;
    std::vector<double> U_, cost_;
    std::vector<int> iters_;
    std::vector<int64_t> rec_;
};

}  // namespace mpcqp
