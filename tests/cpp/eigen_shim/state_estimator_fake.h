// TEST-ONLY stand-in for the reference's include/state_estimator_fake.h (it needs ROS / limxsdk):
// RobotOdomState as declared there (:19-25) and a StateEstimatorFake whose get_state() returns
// what the test put in `s` (the real one integrates IMU / joint data, :118-142).
#pragma once

struct RobotOdomState {
    double pos[3], ori[3], quat[4], v_pos[3], v_ori[3];
};

class StateEstimatorFake {
  public:
    RobotOdomState s{};
    RobotOdomState get_state() { return s; }
};
