// cv::undistortPoints for Frame::UndistortKeyPoints (Frame.cc:389-423) and
// Frame::ComputeImageBounds (Frame.cc:425-493), shared by the keypoint kernel
// (undistort.hip) and the front end's image bounds (computed on the host at
// creation, frontend.hip). OpenCV 3.4's cvUndistortPointsInternal with the
// default criteria TermCriteria(COUNT, 5, 0.01): 5 fixed-point iterations in
// double on the normalised point, 4 or 5 coefficients (k1 k2 p1 p2 [k3]), no
// tilt, then the projection through P = K (RR = K * I); f64 in OpenCV's
// expression order (compiled without contraction).
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>

namespace gfu {

struct UndistCoef {
    double fx, fy, ifx, ify, cx, cy;
    double k[5];  // k1 k2 p1 p2 k3
};

inline UndistCoef make_coef(const float K[4], const float dist[5]) {
    UndistCoef c;
    c.fx = (double)K[0];
    c.fy = (double)K[1];
    c.cx = (double)K[2];
    c.cy = (double)K[3];
    c.ifx = 1. / c.fx;
    c.ify = 1. / c.fy;
    for (int i = 0; i < 5; i++) c.k[i] = (double)dist[i];
    return c;
}

__host__ __device__ inline void undistort_point(const UndistCoef& c, float xf, float yf, float& xo, float& yo) {
    double x = (double)xf, y = (double)yf;
    x = (x - c.cx) * c.ifx;
    y = (y - c.cy) * c.ify;
    // the identity tilt: x0 = 1 * x (exact)
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        // the rational-model numerator is 1 + ((0 r2 + 0) r2 + 0) r2 = 1 exactly
        const double icdist = 1.0 / (1 + ((c.k[4] * r2 + c.k[1]) * r2 + c.k[0]) * r2);
        const double deltaX = 2 * c.k[2] * x * y + c.k[3] * (r2 + 2 * x * x);
        const double deltaY = c.k[2] * (r2 + 2 * y * y) + 2 * c.k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = K: xx = fx x + 0 y + cx, yy = 0 x + fy y + cy, ww = 1 / (0 x + 0 y + 1)
    const double xx = c.fx * x + c.cx, yy = c.fy * y + c.cy;
    xo = (float)xx;
    yo = (float)yy;
}

// Frame::ComputeImageBounds (Frame.cc:425-493): the corners and edge
// midpoints undistorted; b = {mnMinX, mnMaxX, mnMinY, mnMaxY}. k1 == 0: the
// image. The reference compares the int bound with the float coordinate.
inline void image_bounds(const float K[4], const float dist[5], int w, int h, int b[4]) {
    if (dist[0] == 0.f) {
        b[0] = 0;
        b[1] = w;
        b[2] = 0;
        b[3] = h;
        return;
    }
    const float px[8] = {0.f, (float)w, 0.f, (float)w, 0.f, (float)w / 2.0f, (float)w / 2.0f, (float)w};
    const float py[8] = {0.f, 0.f, (float)h, (float)h, (float)h / 2.0f, 0.f, (float)h, (float)h / 2.0f};
    const UndistCoef c = make_coef(K, dist);
    int mnMinX = INT_MAX, mnMaxX = INT_MIN, mnMinY = INT_MAX, mnMaxY = INT_MIN;
    for (int i = 0; i < 8; i++) {
        float x, y;
        undistort_point(c, px[i], py[i], x, y);
        if ((float)mnMinX > x) mnMinX = (int)std::floor(x);
        if ((float)mnMinY > y) mnMinY = (int)std::floor(y);
        if ((float)mnMaxX < x) mnMaxX = (int)std::ceil(x);
        if ((float)mnMaxY < y) mnMaxY = (int)std::ceil(y);
    }
    b[0] = mnMinX;
    b[1] = mnMaxX;
    b[2] = mnMinY;
    b[3] = mnMaxY;
}

}  // namespace gfu
