// compat/MPCParam.h -- drop-in for the reference's include/MPCParam.h: the same public fields
// (include/MPCParam.h:13-59, float timing fields kept float) and errorTest(), without the
// limxsdk include it does not use.  The constructor is inline (the reference defines it in the
// header non-inline, which breaks when two translation units include it).
#ifndef MPCQP_COMPAT_MPC_PARAM_H
#define MPCQP_COMPAT_MPC_PARAM_H

#include <cmath>
#include <vector>

#if __has_include(<Eigen/Dense>)
#include <Eigen/Dense>
#else
#error "compat/MPCParam.h needs Eigen 3 (as the reference does)"
#endif

struct kinematicValues {
    double abad_offset_x = 0.05556, abad_offset_y = 0.105, abad_offset_z = -0.2602;
    double hip_offset_x = -0.077, hip_offset_y = 0.02050, hip_offset_z = 0.0;
    double knee_offset_x = -0.1500, knee_offset_y = -0.02050, knee_offset_z = -0.25981;
    double foot_offset_x = 0.145, foot_offset_y = 0.0, foot_offset_z = -0.2598;
    double contact_offset_x = 0.0, contact_offset_y = 0.0, contact_offset_z = -0.032;
};

class MPCParam {
  public:
    MPCParam() {
        const kinematicValues &k = KinematicValues;
        const double x = k.abad_offset_x + k.hip_offset_x + k.knee_offset_x + k.foot_offset_x +
                         k.contact_offset_x;
        const double z = k.abad_offset_z + k.hip_offset_z + k.knee_offset_z + k.foot_offset_z +
                         k.contact_offset_z;
        // include/MPCParam.h:66-72 (the left foot's lateral sign is the reference's)
        static_foot_offset_left << x,
            -k.abad_offset_y - k.hip_offset_y - k.knee_offset_y + k.foot_offset_y + k.contact_offset_y, z;
        static_foot_offset_right << x,
            k.abad_offset_y + k.hip_offset_y + k.knee_offset_y + k.foot_offset_y + k.contact_offset_y, z;
    }

    float dt = 0.001f;
    int milliseconds_per_step = static_cast<int>(1 / dt);
    int mpcStep = 5;
    float dtMPC = dt * mpcStep;
    float swing_time = 0.5f;
    float stance_time = 0.5f;
    float gait_height = 0.1f;
    float givenErrorRate = 0.1f;

    kinematicValues KinematicValues;
    Eigen::Vector3d static_foot_offset_right;
    Eigen::Vector3d static_foot_offset_left;

    // include/MPCParam.h:75-82: true when all 6 joints are within givenErrorRate
    bool errorTest(std::vector<float> targetPos, std::vector<float> nowPos) {
        bool ok = true;
        for (int i = 0; i < 6; ++i)
            if (std::fabs(targetPos[i] - nowPos[i]) >= givenErrorRate) ok = false;
        return ok;
    }
};

#endif
