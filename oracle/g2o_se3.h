// CPU ORACLE (test infrastructure) — the SE(3) arithmetic g2o runs for the
// pose LM and the local BA, restated from the vendored sources:
//   SE3Quat ctor / normalizeRotation / operator* / map / exp
//     (Thirdparty/g2o/g2o/types/slam3d/se3quat.h:55-64, 104-117, 217-258),
//   Eigen Quaternion(Matrix3) / toRotationMatrix / _transformVector / product
//     (Eigen 3.3 semantics; Eigen itself is not vendored),
//   Converter::toSE3Quat / toCvMat (src/Converter.cc:38-72).
// Shared by oracle/poseopt.cpp (rows P1-P4) and oracle/lba.cpp (row B1).
#pragma once
#include <cmath>
#include <cstring>

namespace orc {

struct Quat {
    double w, x, y, z;
};

inline Quat quat_from_R(const double m[3][3]) {  // Eigen quaternionbase_assign_impl
    Quat q;
    double t = m[0][0] + (m[1][1] + m[2][2]);  // diagonal().sum(): unrolled a0 + (a1 + a2)
    if (t > 0) {
        t = std::sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[k][j] - m[j][k]) * t;
        c[j] = (m[j][i] + m[i][j]) * t;
        c[k] = (m[k][i] + m[i][k]) * t;
        q.x = c[0];
        q.y = c[1];
        q.z = c[2];
    }
    return q;
}

inline void normalize_rotation(Quat& q) {  // SE3Quat::normalizeRotation
    if (q.w < 0) {
        q.w *= -1;
        q.x *= -1;
        q.y *= -1;
        q.z *= -1;
    }
    // coeffs() = (x, y, z, w) reduced as two packets: (x^2 + z^2) + (y^2 + w^2)
    double n = std::sqrt((q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w));
    q.x /= n;
    q.y /= n;
    q.z /= n;
    q.w /= n;
}

inline void quat_to_R(const Quat& q, double R[3][3]) {  // Eigen toRotationMatrix
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0][0] = 1 - (tyy + tzz);
    R[0][1] = txy - twz;
    R[0][2] = txz + twy;
    R[1][0] = txy + twz;
    R[1][1] = 1 - (txx + tzz);
    R[1][2] = tyz - twx;
    R[2][0] = txz - twy;
    R[2][1] = tyz + twx;
    R[2][2] = 1 - (txx + tyy);
}

inline void rotate(const Quat& q, const double* v, double* o) {  // Eigen _transformVector
    double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    const double cx = q.y * uv[2] - q.z * uv[1], cy = q.z * uv[0] - q.x * uv[2], cz = q.x * uv[1] - q.y * uv[0];
    o[0] = v[0] + q.w * uv[0] + cx;
    o[1] = v[1] + q.w * uv[1] + cy;
    o[2] = v[2] + q.w * uv[2] + cz;
}

inline Quat qmul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

struct SE3 {
    Quat r;
    double t[3];
    void map(const double* p, double* o) const {
        rotate(r, p, o);
        for (int i = 0; i < 3; i++) o[i] += t[i];
    }
};

inline SE3 se3_exp(const double* u) {  // SE3Quat::exp, se3quat.h:223-258
    const double w[3] = {u[0], u[1], u[2]}, up[3] = {u[3], u[4], u[5]};
    const double theta = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
        std::memcpy(V, R, sizeof(R));
    } else {
        const double a = std::sin(theta) / theta, b = (1 - std::cos(theta)) / (theta * theta);
        const double c = (theta - std::sin(theta)) / std::pow(theta, 3);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + a * O[i][j]) + b * O2[i][j];
                V[i][j] = ((i == j ? 1.0 : 0.0) + b * O[i][j]) + c * O2[i][j];
            }
    }
    SE3 s;
    s.r = quat_from_R(R);
    for (int i = 0; i < 3; i++) s.t[i] = V[i][0] * up[0] + V[i][1] * up[1] + V[i][2] * up[2];
    normalize_rotation(s.r);
    return s;
}

inline SE3 se3_mul(const SE3& a, const SE3& b) {  // SE3Quat::operator*
    SE3 r = a;
    double rt[3];
    rotate(a.r, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] += rt[i];
    r.r = qmul(a.r, b.r);
    normalize_rotation(r.r);
    return r;
}

// Converter::toSE3Quat (Converter.cc:38-48): float cv::Mat Tcw -> SE3Quat.
inline SE3 se3_from_Tcw(const float* Tcw) {
    double R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = Tcw[4 * i + j];
    SE3 s;
    s.r = quat_from_R(R);
    for (int i = 0; i < 3; i++) s.t[i] = Tcw[4 * i + 3];
    normalize_rotation(s.r);
    return s;
}

// Converter::toCvMat(SE3Quat) (Converter.cc:50-72): to_homogeneous_matrix, cast to float.
inline void se3_to_Tcw(const SE3& s, float* Tcw) {
    double R[3][3];
    quat_to_R(s.r, R);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Tcw[4 * i + j] = (float)R[i][j];
        Tcw[4 * i + 3] = (float)s.t[i];
    }
    Tcw[12] = Tcw[13] = Tcw[14] = 0.f;
    Tcw[15] = 1.f;
}

}  // namespace orc
