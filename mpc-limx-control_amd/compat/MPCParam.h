// compat/MPCParam.h -- drop-in for the reference's include/MPCParam.h: the same public fields
// (include/MPCParam.h:13-59, float timing fields kept float), the same include set, and
// errorTest().  The constructor is inline (the reference defines it in the header non-inline,
// which breaks when two translation units include it).
//
// errorTest (include/MPCParam.h:75-82) calls an unqualified abs() on a float difference at
// global scope.  Which abs that is depends on the declarations visible there: with only the
// <cmath> / <cstdlib> family it is C's int abs(int), so the difference is TRUNCATED to an
// integer (any error below 1 rad passes the 0.1 rad test); once libstdc++'s <stdlib.h> or
// <math.h> wrapper is visible (`using std::abs`: x86-64 Eigen pulls it in through the SSE
// intrinsics headers -> <mm_malloc.h> -> <stdlib.h>) it is the float overload.  The body below
// is written the reference's way, after the reference's includes, so it resolves to the same
// abs as the reference does in the same translation unit.  MPCQP_ERRORTEST_ABS overrides it:
//   0 (default) the reference's unqualified abs, as resolved here
//   1           C's int abs on the truncated difference, whatever is included
//   2           the float absolute value, whatever is included
#ifndef MPCQP_COMPAT_MPC_PARAM_H
#define MPCQP_COMPAT_MPC_PARAM_H

#if __has_include("limxsdk/datatypes.h")
#include "limxsdk/datatypes.h"
#endif
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <vector>

#if __has_include(<Eigen/Dense>)
#include <Eigen/Dense>
#else
#error "compat/MPCParam.h needs Eigen 3 (as the reference does)"
#endif

#ifndef MPCQP_ERRORTEST_ABS
#define MPCQP_ERRORTEST_ABS 0
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

    // include/MPCParam.h:75-82: true when all 6 joints are within givenErrorRate (see the
    // header comment for which abs the reference's expression means)
    bool errorTest(std::vector<float> targetPos, std::vector<float> nowPos) {
        bool ok = true;
        for (int i = 0; i < 6; ++i) {
#if MPCQP_ERRORTEST_ABS == 1
            if (std::abs(static_cast<int>(targetPos[i] - nowPos[i])) >= givenErrorRate) ok = false;
#elif MPCQP_ERRORTEST_ABS == 2
            if (std::fabs(targetPos[i] - nowPos[i]) >= givenErrorRate) ok = false;
#else
            if (abs(targetPos[i] - nowPos[i]) >= givenErrorRate) ok = false;
#endif
        }
        return ok;
    }
    // which abs errorTest applies in this translation unit: true = C's int abs (truncating)
    static bool errorTestTruncates() {
#if MPCQP_ERRORTEST_ABS == 1
        return true;
#elif MPCQP_ERRORTEST_ABS == 2
        return false;
#else
        return abs(0.5f) == 0;
#endif
    }
};

#endif
