// MPCParam::errorTest through the drop-in header (compat/MPCParam.h) against two restatements
// of the reference's expression `abs(targetPos[i] - nowPos[i]) >= givenErrorRate`
// (include/MPCParam.h:75-82): C's int abs of the truncated difference, and the float absolute
// value.  Which one the reference means depends on what is visible at its definition (see
// compat/MPCParam.h); EXPECT_TRUNC names the one this build must reproduce.
//
// Checks, on seeded joint vectors:
//   * errors inside (0.1, 1) rad on one or all joints, errors of 1-3 rad, errors below 0.1 rad,
//     negative differences;
//   * the start-up loop of src/mpc_control_fake_state.cpp:57-89: joints interpolated from
//     init_pos to targetPos over 2000 iterations (r = iter / 2000), tracked exactly, until
//     errorTest passes -- the iteration at which the loop leaves must equal the restatement's.
// Prints "errortest OK trunc=<0|1> exit=<iteration>".
#include "MPCParam.h"

#include <algorithm>
#include <cstdio>
#include <random>

#ifndef EXPECT_TRUNC
#error "define EXPECT_TRUNC (1: C's int abs, 0: the float absolute value)"
#endif

static bool restated(const std::vector<float> &t, const std::vector<float> &n, float rate) {
    bool flag = true;
    for (int i = 0; i < 6; ++i) {
        const float d = t[i] - n[i];
#if EXPECT_TRUNC
        if (std::abs(static_cast<int>(d)) >= rate) flag = false;
#else
        if (std::fabs(d) >= rate) flag = false;
#endif
    }
    return flag;
}

int main() {
    MPCParam param;
    if (MPCParam::errorTestTruncates() != (EXPECT_TRUNC != 0)) {
        std::printf("errortest FAIL: the header applies %s abs, expected %s\n",
                    MPCParam::errorTestTruncates() ? "int" : "float", EXPECT_TRUNC ? "int" : "float");
        return 1;
    }
    std::mt19937 rng(20260601);
    std::uniform_real_distribution<float> pos(-2.0f, 2.0f), small(0.0f, 0.0999f),
        mid(0.1001f, 0.999f), big(1.0f, 3.0f), sgn(-1.0f, 1.0f);
    int cases = 0, passes = 0;
    for (int trial = 0; trial < 4000; ++trial) {
        std::vector<float> t(6), n(6);
        for (int i = 0; i < 6; ++i) t[i] = pos(rng);
        const int kind = trial % 4;
        for (int i = 0; i < 6; ++i) {
            float e = small(rng);
            if (kind == 1 && i == trial % 6) e = mid(rng);   // one joint in (0.1, 1)
            if (kind == 2) e = mid(rng);                      // every joint in (0.1, 1)
            if (kind == 3 && i == trial % 6) e = big(rng);    // one joint 1-3 rad off
            n[i] = t[i] - (sgn(rng) < 0.0f ? -e : e);
        }
        const bool got = param.errorTest(t, n), want = restated(t, n, param.givenErrorRate);
        if (got != want) {
            std::printf("errortest FAIL: trial %d kind %d: header %d restatement %d\n", trial, kind,
                        (int)got, (int)want);
            return 1;
        }
        ++cases;
        passes += got ? 1 : 0;
    }
    // the start-up loop: every joint starts 0.5-2 rad from its target
    std::vector<float> target(6, 0.0f), init(6);
    for (int i = 0; i < 6; ++i) init[i] = (i % 2 ? -1.0f : 1.0f) * (0.5f + 0.25f * (float)i);
    auto leave_at = [&](bool header) {
        for (int iter = 0; iter <= 4000; ++iter) {
            const double r = std::min(std::max(double(iter) / 2000.0, 0.0), 1.0);
            std::vector<float> q(6);
            for (int i = 0; i < 6; ++i) q[i] = (float)((1 - r) * init[i] + r * target[i]);
            const bool reach = header ? param.errorTest(target, q) : restated(target, q, param.givenErrorRate);
            if (reach) return iter;
        }
        return -1;
    };
    const int ih = leave_at(true), ir = leave_at(false);
    if (ih != ir || ih < 0) {
        std::printf("errortest FAIL: start-up loop leaves at %d (header) vs %d (restatement)\n", ih, ir);
        return 1;
    }
    std::printf("errortest OK trunc=%d exit=%d cases=%d passed=%d\n", EXPECT_TRUNC, ih, cases, passes);
    return 0;
}
