// Drives the reference's `class MPC` tick (mpcqp::BasicMPC, include/mpcqp/mpc_controller.hpp;
// what compat/MPCController.h instantiates with Eigen / limxsdk / ROS types) with TEST-ONLY
// stand-ins for limxsdk::RobotState / ImuData / RobotCmd, RobotOdomState and
// StateEstimatorFake (include/state_estimator_fake.h:19-25, 118-142), none of which exist in
// this image.  Reads T ticks from a raw little-endian file written by tests/test_cpp.py:
//   per tick: int32 iter, 16 doubles odom (pos3 ori3 quat4 v_pos3 v_ori3), 6 floats q
// and prints per tick (%.17g) the gait state, foot placement, x0, xref, lin, contact, the chosen
// candidate, status, cost and the support-foot forces U.col(0).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "limxsdk/datatypes.h"      // test-only stand-ins (tests/cpp/eigen_shim)
#include "state_estimator_fake.h"
#ifdef MPCQP_COMPAT_MPC
#include "MPCController.h"  // the drop-in class MPC (compat/), over the Eigen stand-in
#else
#include "mpcqp/mpc_controller.hpp"
#endif

#ifndef MPCQP_COMPAT_MPC
struct Vec3 {
    double v[3];
    Vec3(double a, double b, double c) : v{a, b, c} {}
    double &operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
};

struct Param {  // MPCParam's fields the tick reads (include/MPCParam.h:44-72)
    float dt = 0.001f;
    float swing_time = 0.5f;
    float stance_time = 0.5f;
    // kinematicValues sums, include/MPCParam.h:13-38, 64-72 (left y negative, as the reference)
    Vec3 static_foot_offset_left{0.05556 - 0.077 - 0.15 + 0.145 + 0.0, -0.105 - 0.0205 + 0.0205 + 0.0 + 0.0,
                                 -0.2602 + 0.0 - 0.25981 - 0.2598 - 0.032};
    Vec3 static_foot_offset_right{0.05556 - 0.077 - 0.15 + 0.145 + 0.0, 0.105 + 0.0205 - 0.0205 + 0.0 + 0.0,
                                  -0.2602 + 0.0 - 0.25981 - 0.2598 - 0.032};
};

#endif

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: mpc_controller N T lever(0 world|1 literal) ncand input.bin\n");
        return 2;
    }
    const int N = std::atoi(argv[1]), T = std::atoi(argv[2]), literal = std::atoi(argv[3]),
              ncand = std::atoi(argv[4]);
    FILE *fp = std::fopen(argv[5], "rb");
    if (!fp) return 3;
#ifdef MPCQP_COMPAT_MPC
    // class MPC as the reference declares it: N = 20, world lever arms, one candidate
    if (N != 20 || literal || ncand != 1) return 5;
    MPC mpc;
#else
    mpcqp::BasicMPC<Vec3, Param, StateEstimatorFake> mpc(N, false, 0);
    mpc.lever_arms = literal ? mpcqp::LeverArms::ReferenceLiteral : mpcqp::LeverArms::World;
    for (int c = 1; c < ncand; ++c) mpc.candidate_offsets.push_back(0.0625 * c);
#endif
    limxsdk::RobotState state;
    state.q.assign(6, 0.0f);
    limxsdk::ImuData imu{};
    limxsdk::RobotCmd cmd;
    cmd.tau.assign(6, 0.0f);
    for (int t = 0; t < T; ++t) {
        int iter = 0;
        double od[16];
        float q[6];
        if (std::fread(&iter, sizeof(int), 1, fp) != 1 || std::fread(od, sizeof(double), 16, fp) != 16 ||
            std::fread(q, sizeof(float), 6, fp) != 6)
            return 4;
        RobotOdomState &s = mpc.estimates.s;
        std::memcpy(s.pos, od, 3 * sizeof(double));
        std::memcpy(s.ori, od + 3, 3 * sizeof(double));
        std::memcpy(s.quat, od + 6, 4 * sizeof(double));
        std::memcpy(s.v_pos, od + 10, 3 * sizeof(double));
        std::memcpy(s.v_ori, od + 13, 3 * sizeof(double));
        for (int i = 0; i < 6; ++i) state.q[(size_t)i] = q[i];
        mpc.run(state, imu, cmd, iter);
        std::printf("tick %d gait %d %d %.17g %.17g place %.17g %.17g", t, mpc.leftLegState(),
                    mpc.rightLegState(), mpc.gaitPhase(), mpc.remainingSwingTime(),
                    mpc.footPlacement()[0], mpc.footPlacement()[1]);
        std::printf(" x0");
        for (int i = 0; i < 13; ++i) std::printf(" %.17g", mpc.lastX0()[i]);
        std::printf(" xref");
        for (double v : mpc.lastXref()) std::printf(" %.17g", v);
        std::printf(" lin");
        for (int i = 0; i < 8; ++i) std::printf(" %.17g", mpc.lastLin()[i]);
        std::printf(" contact %llu choice %d status %d cost %.17g force",
                    (unsigned long long)mpc.lastContact(), mpc.lastChoice(), mpc.lastStatus(),
                    mpc.lastCost());
        for (int i = 0; i < 6; ++i) std::printf(" %.17g", mpc.supportForce()[i]);
        std::printf("\n");
    }
    std::fclose(fp);
    // the swing-leg command path is not built: run() must say so, and leave cmd as passed
    if (mpc.cmdWritten() || mpc.untouchedCmdTicks() != T) return 6;
    for (float v : cmd.tau)
        if (v != 0.0f) return 7;
    return 0;
}
