// compat/MPCController.h -- drop-in for the reference's include/MPCController.h
// (Fleming-Sung/mpc-limX-control): the same `class MPC` with the same public members
// (MPC(), run(limxsdk::RobotState, limxsdk::ImuData, limxsdk::RobotCmd&, int), param,
// estimates, desieredV_pos, desieredV_ori; include/MPCController.h:9-17), whose tick also runs
// the support-force MPC the reference leaves empty (computeSupportFootForce, :178-180) on the
// GPU through libmpcqp.so.  The logic lives in <mpcqp/mpc_controller.hpp> (mpcqp::BasicMPC,
// Eigen-free); this header binds it to the reference's types.
//
// Needs what the reference's header needs: Eigen 3, limxsdk/datatypes.h and the reference's
// state_estimator_fake.h (ROS) on the include path, with this directory ahead of the
// reference's include/ (so MPCParam.h resolves to compat/MPCParam.h).  Pinocchio is not needed:
// the foot positions come from the batched FK kernel (mpcqp_ctx_fk_feet_host).  Not built here
// (no Eigen / limxsdk / ROS in the image); tests/cpp/mpc_controller.cpp drives the same
// BasicMPC with test-only stand-ins for those types.
#ifndef MPCQP_COMPAT_MPC_CONTROLLER_H
#define MPCQP_COMPAT_MPC_CONTROLLER_H

#if __has_include(<Eigen/Dense>) && __has_include("limxsdk/datatypes.h") && \
    __has_include("state_estimator_fake.h")
#include <Eigen/Dense>

#include "MPCParam.h"
#include "limxsdk/datatypes.h"
#include "state_estimator_fake.h"
#include "../include/mpcqp/mpc_controller.hpp"

class MPC : public mpcqp::BasicMPC<Eigen::Vector3d, MPCParam, StateEstimatorFake> {
  public:
    MPC() : mpcqp::BasicMPC<Eigen::Vector3d, MPCParam, StateEstimatorFake>(20, false, 0) {}
    void run(limxsdk::RobotState state, limxsdk::ImuData imu, limxsdk::RobotCmd &cmd, int iter) {
        mpcqp::BasicMPC<Eigen::Vector3d, MPCParam, StateEstimatorFake>::run(state, imu, cmd, iter);
    }
};

#else
#error "compat/MPCController.h needs Eigen 3, limxsdk/datatypes.h and state_estimator_fake.h (as the reference does); without them use <mpcqp/mpc_controller.hpp> (mpcqp::BasicMPC)"
#endif

#endif
