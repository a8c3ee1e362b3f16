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

// Accumulation order of the reference's small cv::Mat float products
// (Rcw*x3Dw+tcw, V*LastTcw, Tcw*LastTwc, -Rcw^T*tcw). docs/ORACLE_ASSUMPTIONS.md
// A1: 0 = float products, float left-to-right sums (the parity setting, what
// the device does); 1 = products and sums in double, one rounding to float
// (cv::gemm's generic GEMMSingleMul<float,double> path); 2 = fused
// multiply-adds left to right. Modes 1 and 2 exist only for
// scripts/oracle_sensitivity.py (orc_set_gemm_mode).
extern int g_gemm_mode;
inline float dot3(float a0, float b0, float a1, float b1, float a2, float b2) {
    if (g_gemm_mode == 1) return (float)((double)a0 * b0 + (double)a1 * b1 + (double)a2 * b2);
    if (g_gemm_mode == 2) return std::fma(a2, b2, std::fma(a1, b1, a0 * b0));
    const float x = a0 * b0, y = a1 * b1, z = a2 * b2;
    return (x + y) + z;
}
inline float dot3p(float a0, float b0, float a1, float b1, float a2, float b2, float t) {
    if (g_gemm_mode == 1) return (float)((double)a0 * b0 + (double)a1 * b1 + (double)a2 * b2 + (double)t);
    if (g_gemm_mode == 2) return std::fma(a2, b2, std::fma(a1, b1, a0 * b0)) + t;
    const float x = a0 * b0, y = a1 * b1, z = a2 * b2;
    return ((x + y) + z) + t;
}
inline float dot4(const float* a, int sa, const float* b, int sb) {
    if (g_gemm_mode == 1) {
        double s = 0;
        for (int k = 0; k < 4; k++) s += (double)a[k * sa] * b[k * sb];
        return (float)s;
    }
    float s = a[0] * b[0];
    for (int k = 1; k < 4; k++) s = g_gemm_mode == 2 ? std::fma(a[k * sa], b[k * sb], s) : s + a[k * sa] * b[k * sb];
    return s;
}

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

// SearchByProjection_OnePoint over a frame grid built once (oracle/match.cpp):
// returns the keypoint the map point would claim (not claimed here) or -1.
struct OnePointGrid;
OnePointGrid* one_point_grid(const gf_frame_info* fi, const gf_keypoint* kps, int n);
void one_point_grid_free(OnePointGrid* g);
int one_point(const OnePointGrid* g, const gf_mp_view& v, const uint8_t* mp_desc, const uint8_t* desc, float th,
              float nnratio, const int32_t* kp2mp, int* dist_out);

// log-det evaluations of the last runActiveMapMatching (oracle/gf.cpp)
extern long long g_ldets;

struct Image {
    int w = 0, h = 0;
    std::vector<uint8_t> px;
    uint8_t at(int x, int y) const { return px[(size_t)y * w + x]; }
};

}  // namespace orc
#endif
