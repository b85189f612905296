// mpc_controller.hpp -- the reference's `class MPC` tick (include/MPCController.h:9-39,
// 41-196) with its intended QP call site filled in: computeSupportFootForce
// (include/MPCController.h:178-180, empty in the reference) assembles the mpcQP inputs exactly
// as include/mpcQP.h:35-119 does and solves them on the GPU through ConvexMpc.
//
// Header-only and Eigen-free: the vector, parameter and estimator types are template
// parameters, so the same code backs compat/MPCController.h (Eigen::Vector3d, MPCParam,
// StateEstimatorFake, limxsdk::*) and the test harness (tests/cpp/mpc_controller.cpp, with
// test-only stand-ins).  Requirements:
//   Vec3       constructible from (double, double, double), operator[] (Eigen::Vector3d is)
//   Param      MPCParam's fields dt, swing_time, stance_time (float), static_foot_offset_left /
//              _right (Vec3-like)                                 (include/MPCParam.h:44-72)
//   Estimator  get_state() -> a RobotOdomState-like struct with pos[3], ori[3], quat[4] (x y z
//              w), v_pos[3], v_ori[3]                    (include/state_estimator_fake.h:19-25)
//   run()'s RobotState has a float container q (6 joint angles: abad, hip, knee left then
//   right); ImuData and RobotCmd are not read (the reference's tick does not read imu either).
//
// What a tick does (MPC::run, include/MPCController.h:183-196):
//   update_odom_state()        :45-58, as written
//   calculateGait(iter)        :61-75, as written (float dt / swing / stance kept float)
//   computeFootPlacement()     :106-132, as written
//   computeSupportFootForce()  the intended QP call (mpcQP ctor, include/mpcQP.h:35-119):
//     x0   = [rpy, p, omega, v, -9.8]                          (include/mpcQP.h:66-71)
//     xref = 13 x (N+1), column i: yaw + i Ts omega_yaw, x + i Ts v_x, v_x(i>0) = 0.5, rest
//            held at the current state                         (include/mpcQP.h:74-97)
//     lin  = {yaw, r_L, r_R, 0}: both feet from the batched FK kernel (mpcqp_ctx_fk_feet_host,
//            replacing kinematicsModel.forwardKinematics + getLinkPosition, :125-137)
//     contact per horizon step from calculateGait's rule at t = iter dt + k Ts (both feet,
//            so the 6-input SRBM sees the whole schedule, not one support leg)
//     -> ConvexMpc::solve (one GPU launch), U.col(0) = support-foot forces (f_L, f_R).
//   computeSwingFootDesiredPosition() needs Pinocchio's IK on the TRON1 URDF, neither of which
//   is in the reference repository: not built; cmd is left as passed.
//
// Lever arms.  The reference's buildSystemModel calls setBaseLinkPose(Position,
// Quaterniond(Quat(0), Quat(1), Quat(2), Quat(3))) with the odometry quaternion stored x y z w,
// i.e. w/x swapped (include/mpcQP.h:125, include/state_estimator_fake.h:69-72), but that pose
// is written to data.oMi[1], which the following forwardKinematics overwrites
// (include/pinocchio_kinematics.h:153-157, :30-33): the FK foot position is in the base frame
// and d = foot - Position mixes it with the world base position (:139-141).  So the quaternion
// (swapped or not) never reaches the result.  LeverArms::World (default) rotates the base-frame
// FK by the odometry rpy (the attitude x0 carries): r = R(rpy) FK(q), the vector the SRBM
// needs.  LeverArms::ReferenceLiteral reproduces the reference's arithmetic: r = FK(q) - p.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "convex_mpc.hpp"

namespace mpcqp {

// x0 of include/mpcQP.h:66-71
inline void mpc_x0(const double ori[3], const double pos[3], const double w[3], const double v[3],
                   double x0[13]) {
    for (int i = 0; i < 3; ++i) {
        x0[i] = ori[i];
        x0[3 + i] = pos[i];
        x0[6 + i] = w[i];
        x0[9 + i] = v[i];
    }
    x0[12] = -9.8;
}

// xref of include/mpcQP.h:74-97: 13 x (N+1) column-major (column i = step i)
inline void mpc_xref(int N, double Ts, double omega_yaw, double velocity_x, const double ori[3],
                     const double pos[3], const double w[3], const double v[3], double *xref) {
    for (int i = 0; i <= N; ++i) {
        const double t = i * Ts;
        double *c = xref + (size_t)13 * i;
        c[0] = ori[0];
        c[1] = ori[1];
        c[2] = ori[2] + t * omega_yaw;
        c[3] = pos[0] + t * velocity_x;
        c[4] = pos[1];
        c[5] = pos[2];
        c[6] = w[0];
        c[7] = w[1];
        c[8] = w[2];
        c[9] = i == 0 ? v[0] : velocity_x;
        c[10] = v[1];
        c[11] = v[2];
        c[12] = -9.8;
    }
}

enum class LeverArms { World, ReferenceLiteral };

template <class Vec3, class Param, class Estimator>
class BasicMPC {
  public:
    // N = 20, Ts = 1 ms: the reference mpcQP's horizon and sample time (include/mpcQP.h:37-38)
    explicit BasicMPC(int N = 20, bool friction = false, int device = 0)
        : mpc_(srbm_model(N, friction), device) {
        odom_state = estimates.get_state();  // include/MPCController.h:41-43
        int rc = mpcqp_ctx_reserve(mpc_.ctx(), 64);  // no device allocation per tick
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_ctx_reserve: ") + mpcqp_status_string(rc));
    }

    template <class RobotState, class ImuData, class RobotCmd>
    void run(RobotState state, ImuData imu, RobotCmd &cmd, int iter) {
        (void)imu;
        (void)cmd;
        update_odom_state();
        calculateGait(iter);
        computeFootPlacement(finalPosition);
        computeSupportFootForce(state, iter);
        // the reference's swing-leg command (cmd.q from Pinocchio IK, :134-175,195) is not
        // built: cmd goes back as passed, and this says so at run time
        if (++untouched_ticks_ == 1 && warnUntouchedCmd)
            std::fprintf(stderr, "[mpcqp] MPC::run: the swing-leg command path (Pinocchio IK, "
                                 "include/MPCController.h:134-175) is not implemented; cmd is "
                                 "returned unmodified (cmdWritten() == false)\n");
    }

    // The reference's run() also writes cmd.q for the swing leg (include/MPCController.h:
    // 134-175,195: Pinocchio IK on the TRON1 URDF, which the reference repository does not
    // hold; SURVEY.md 2 #3 puts it out of scope).  run() here leaves cmd as passed: callers that
    // publish cmd check cmdWritten() (always false) or kWritesSwingCommand;
    // untouchedCmdTicks() counts the ticks that returned cmd unmodified, and the first one prints
    // a line to stderr unless warnUntouchedCmd is cleared before it.
    static constexpr bool kWritesSwingCommand = false;
    bool cmdWritten() const { return kWritesSwingCommand; }
    long long untouchedCmdTicks() const { return untouched_ticks_; }
    bool warnUntouchedCmd = true;

    Param param;
    Estimator estimates;
    Vec3 desieredV_pos = Vec3(1.0, 0.0, 0.0);  // include/MPCController.h:16-17 (sic)
    Vec3 desieredV_ori = Vec3(0.0, 0.0, 0.0);

    // reference mpcQP constants (include/mpcQP.h:75-76)
    double omega_yaw = 0.1;
    double velocity_x = 0.5;
    LeverArms lever_arms = LeverArms::World;
    // extra gait candidates (phase offsets, s) solved beside the reference's schedule in the same
    // launch; the cheapest wins (lowest index on ties).  Empty: the reference's gait only.
    std::vector<double> candidate_offsets;

    // results of the last tick
    const double *supportForce() const { return force_; }  // U.col(0) = (f_L, f_R) [N]
    const std::vector<double> &plan() const { return plan_; }  // U, nu x N column-major
    int lastStatus() const { return status_; }
    int lastChoice() const { return choice_; }
    double lastCost() const { return cost_; }
    const double *lastX0() const { return x0_; }
    const std::vector<double> &lastXref() const { return xref_; }
    const double *lastLin() const { return lin_; }
    uint64_t lastContact() const { return contact_; }
    int leftLegState() const { return left_leg_state; }
    int rightLegState() const { return right_leg_state; }
    double gaitPhase() const { return phase; }
    double remainingSwingTime() const { return remainSwingTime; }
    const Vec3 &footPlacement() const { return finalPosition; }
    ConvexMpc &engine() { return mpc_; }

  protected:
    template <class O>
    void copy_odom(const O &o) {
        for (int i = 0; i < 3; ++i) {
            pos_[i] = o.pos[i];
            ori_[i] = o.ori[i];
            vel_[i] = o.v_pos[i];
            omega_[i] = o.v_ori[i];
        }
        for (int i = 0; i < 4; ++i) quat_[i] = o.quat[i];
    }

    // include/MPCController.h:45-58
    void update_odom_state() {
        odom_state = estimates.get_state();
        copy_odom(odom_state);
        currentPosition = Vec3(pos_[0], pos_[1], pos_[2]);
        currentVelocity = Vec3(vel_[0], vel_[1], vel_[2]);
        currentOrientation = Vec3(ori_[0], ori_[1], ori_[2]);
        currentAngularVelocity = Vec3(omega_[0], omega_[1], omega_[2]);
    }

    // include/MPCController.h:61-75 (1 = swing, 0 = stance)
    void calculateGait(int iter) {
        double currentTime = iter * param.dt;
        double cycleTime = param.swing_time + param.stance_time;
        phase = std::fmod(currentTime, cycleTime);
        if (phase < param.swing_time) {
            left_leg_state = 1;
            right_leg_state = 0;
            remainSwingTime = param.swing_time - phase;
        } else {
            left_leg_state = 0;
            right_leg_state = 1;
            remainSwingTime = cycleTime - phase;
        }
    }

    // include/MPCController.h:106-132
    void computeFootPlacement(Vec3 &fp) {
        double pred[3];
        for (int i = 0; i < 3; ++i) pred[i] = pos_[i] + desieredV_pos[i] * remainSwingTime;
        const double p_rel_max = 0.3;
        double pfx_rel = desieredV_pos[0] * 0.5 * param.stance_time;
        double pfy_rel = desieredV_pos[1] * 0.5 * param.stance_time;
        pfx_rel = std::fmin(std::fmax(pfx_rel, -p_rel_max), p_rel_max);
        pfy_rel = std::fmin(std::fmax(pfy_rel, -p_rel_max), p_rel_max);
        pred[0] += pfx_rel;
        pred[1] += pfy_rel;
        pred[2] = 0;
        if (left_leg_state == 1) {
            fp[0] = pred[0] + param.static_foot_offset_left[0];
            fp[1] = pred[1] + param.static_foot_offset_left[1];
        } else {
            fp[0] = pred[0] + param.static_foot_offset_right[0];
            fp[1] = pred[1] + param.static_foot_offset_right[1];
        }
    }

    // the intended QP call site (include/MPCController.h:178-180 -> mpcQP, include/mpcQP.h:35-119)
    template <class RobotState>
    void computeSupportFootForce(RobotState &state, int iter) {
        const int N = mpc_.N();
        const double Ts = kTs;
        mpc_x0(ori_, pos_, omega_, vel_, x0_);
        xref_.resize((size_t)13 * (N + 1));
        mpc_xref(N, Ts, omega_yaw, velocity_x, ori_, pos_, omega_, vel_, xref_.data());
        // joint angles arrive as float and widen exactly to double (include/mpcQP.h:127-128)
        double q[6];
        for (int i = 0; i < 6; ++i) q[i] = (double)state.q[(size_t)i];
        const double zero[3] = {0.0, 0.0, 0.0};
        const bool literal = lever_arms == LeverArms::ReferenceLiteral;
        double feet[6];
        int rc = mpcqp_ctx_fk_feet_host(mpc_.ctx(), 1, q, literal ? zero : ori_, 3, feet);
        if (rc != MPCQP_OK) throw std::runtime_error(std::string("mpcqp_ctx_fk_feet_host: ") + mpcqp_status_string(rc));
        lin_[0] = ori_[2];
        for (int i = 0; i < 6; ++i) lin_[1 + i] = feet[i] - (literal ? pos_[i % 3] : 0.0);
        lin_[7] = 0.0;
        // gait schedule over the horizon: calculateGait's rule at t = iter dt + k Ts
        const double t0 = (double)(iter * param.dt);
        const int C = 1 + (int)candidate_offsets.size();
        masks_.resize((size_t)C);
        masks_[0] = gait_contact_mask(N, Ts, t0, param.swing_time, param.stance_time);
        for (int c = 1; c < C; ++c)
            masks_[(size_t)c] = gait_contact_mask(N, Ts, t0 + candidate_offsets[(size_t)c - 1],
                                                  param.swing_time, param.stance_time);
        MpcChoice best = mpc_.solve(x0_, xref_.data(), lin_, masks_.data(), C);
        choice_ = best.index;
        status_ = best.index >= 0 ? MPCQP_OK : best.status[0];
        contact_ = masks_[(size_t)(best.index >= 0 ? best.index : 0)];
        cost_ = best.cost;
        plan_ = best.U;
        for (int i = 0; i < 6; ++i) force_[i] = best.index >= 0 ? best.U[(size_t)i] : 0.0;
    }

    decltype(std::declval<Estimator &>().get_state()) odom_state;
    int left_leg_state = 0;
    int right_leg_state = 0;
    double phase = 0.0;
    double remainSwingTime = 0.0;
    Vec3 finalPosition = Vec3(0.0, 0.0, 0.0);
    Vec3 currentPosition = Vec3(0.0, 0.0, 0.0);
    Vec3 currentVelocity = Vec3(0.0, 0.0, 0.0);
    Vec3 currentOrientation = Vec3(0.0, 0.0, 0.0);
    Vec3 currentAngularVelocity = Vec3(0.0, 0.0, 0.0);
    double quat_[4] = {0, 0, 0, 1};  // as stored: x y z w (kept for inspection; see header)

  private:
    ConvexMpc mpc_;
    double pos_[3] = {0, 0, 0}, ori_[3] = {0, 0, 0}, vel_[3] = {0, 0, 0}, omega_[3] = {0, 0, 0};
    double x0_[13] = {0};
    double lin_[8] = {0};
    double force_[6] = {0};
    std::vector<double> xref_, plan_;
    std::vector<uint64_t> masks_;
    uint64_t contact_ = 0;
    double cost_ = 0.0;
    int status_ = -1, choice_ = -1;
    long long untouched_ticks_ = 0;
};

}  // namespace mpcqp
