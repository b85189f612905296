// TEST-ONLY stand-in for limxsdk/datatypes.h (absent from this image): the fields the MPC tick
// reads and writes (src/mpc_control.cpp:170-185).  Used by tests/cpp/mpc_controller.cpp, with and
// without compat/MPCController.h.
#pragma once
#include <vector>

namespace limxsdk {
struct RobotState {
    std::vector<float> q, dq, tau;
};
struct ImuData {
    float quat[4], acc[3], gyro[3];
};
struct RobotCmd {
    std::vector<float> q, dq, tau, Kp, Kd;
};
}  // namespace limxsdk
