// CPU ORACLE (test infrastructure) — SURVEY.md §8(f) rank 2:
// Frame::UndistortKeyPoints (src/Frame.cc:389-423) = cv::undistortPoints(pts,
// pts, mK, mDistCoef, Mat(), mK) with a float K and 4-5 float coefficients,
// copy when k1 == 0. OpenCV is not vendored: this restates
// OpenCV 3.4's cvUndistortPointsInternal (imgproc/src/undistort.cpp) for that
// call — TermCriteria(COUNT, 5): five iterations, identity tilt, RR = K —
// keeping its expression order. Parity unpinned against OpenCV itself.
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "oracle_common.h"

extern "C" int orc_undistort_keypoints(const float K[4], const float dist[5], const gf_keypoint* in, int n,
                                       gf_keypoint* out) {
    for (int i = 0; i < n; i++) out[i] = in[i];
    if (dist[0] == 0.f) return GF_OK;  // Frame.cc:391-395
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    double k[14] = {0};
    for (int j = 0; j < 5; j++) k[j] = dist[j];
    for (int i = 0; i < n; i++) {
        double x = in[i].x, y = in[i].y;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        const double xx = fx * x + 0. * y + cx;
        const double yy = 0. * x + fy * y + cy;
        const double ww = 1. / (0. * x + 0. * y + 1.);
        out[i].x = (float)(xx * ww);
        out[i].y = (float)(yy * ww);
    }
    return GF_OK;
}

// Frame::ComputeImageBounds (Frame.cc:425-493): the four corners and four edge
// midpoints undistorted, the int bounds compared with the float coordinates
// as the reference writes it; b = {mnMinX, mnMaxX, mnMinY, mnMaxY}. k1 == 0:
// the image (:486-492).
extern "C" int orc_frame_bounds(const float K[4], const float dist[5], int w, int h, int b[4]) {
    if (dist[0] == 0.f) {
        b[0] = 0;
        b[1] = w;
        b[2] = 0;
        b[3] = h;
        return GF_OK;
    }
    gf_keypoint p[8];
    std::memset(p, 0, sizeof(p));
    const float xs[8] = {0.0f, (float)w, 0.0f, (float)w, 0.0f, float(w) / 2.0f, float(w) / 2.0f, (float)w};
    const float ys[8] = {0.0f, 0.0f, (float)h, (float)h, float(h) / 2.0f, 0.0f, (float)h, float(h) / 2.0f};
    for (int i = 0; i < 8; i++) {
        p[i].x = xs[i];
        p[i].y = ys[i];
    }
    orc_undistort_keypoints(K, dist, p, 8, p);
    int mnMinX = INT_MAX, mnMaxX = INT_MIN, mnMinY = INT_MAX, mnMaxY = INT_MIN;
    for (int i = 0; i < 8; i++) {
        if (mnMinX > p[i].x) mnMinX = (int)std::floor(p[i].x);
        if (mnMinY > p[i].y) mnMinY = (int)std::floor(p[i].y);
        if (mnMaxX < p[i].x) mnMaxX = (int)std::ceil(p[i].x);
        if (mnMaxY < p[i].y) mnMaxY = (int)std::ceil(p[i].y);
    }
    b[0] = mnMinX;
    b[1] = mnMaxX;
    b[2] = mnMinY;
    b[3] = mnMaxY;
    return GF_OK;
}
