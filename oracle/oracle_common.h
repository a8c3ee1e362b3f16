// CPU ORACLE — test infrastructure only.
//
// This directory holds a plain C++ restatement of the GF-ORB-SLAM hot path
// (ORBextractor / ORBmatcher / Observability / Optimizer).
// It is the parity checker for the HIP implementation in gf_orb_slam_amd/csrc
// and the CPU baseline leg of bench.py. Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline may load liboracle.so; the product path never
// links or calls it.
//
// Parity pinning: the reference depends on OpenCV 3.4 / Armadillo / g2o-Eigen
// arithmetic that is not vendored in /root/reference and cannot be built here
// (SURVEY.md §8c). The restatement documents every arithmetic choice it makes
// for those libraries (see DESIGN.md "Oracle assumptions"); the kinematics and
// Jacobian rows are pinned by the reference's own known-answer tests
// (test/test_Kine_1.cpp, test/test_Kine_2.cpp, test/test_Jacobian.cpp) and the
// greedy selection by the test_Greedy.cpp property. The extractor / matcher /
// pose-optimisation rows are "parity unpinned" against the original binaries:
// they are pinned against this restatement only.
//
// Compile with -O3 -fno-tree-vectorize -ffp-contract=off: no FMA contraction
// and no auto-vectorised float conversions (GCC's vectorizer changed an
// f64->f32 rounding), so float arithmetic matches the device kernels, which
// are built with -ffp-contract=off and correctly rounded f32 div/sqrt.
// Pose LM (oracle/poseopt.cpp): parity unpinned (no PoseOptimization test
// upstream); checked by recovery/outlier properties in tests/test_oracle_pose.py.
#pragma once
#include <stdint.h>
#include <stddef.h>

#include "../include/gfslam/abi.h"

#ifdef __cplusplus
#include <vector>
#include <cmath>

namespace orc {

// cvRound for float/double: round half to even (lrint under the default mode).
static inline int cv_round(float v) { return (int)std::lrint(v); }
static inline int cv_round(double v) { return (int)std::lrint(v); }
static inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil(float v) { int i = (int)v; return i + (i < v); }

// BORDER_REFLECT_101 index (OpenCV borderInterpolate), len >= 2.
static inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - p - 2;
    }
    return p;
}

struct Image {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
};

}  // namespace orc
#endif
