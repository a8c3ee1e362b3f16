// SE(3) arithmetic of the motion-only pose LM (rows P1-P4), written to the
// exact operation order of the reference's g2o/Eigen expressions so host and
// device agree with the oracle bit for bit:
//   SE3Quat ctor / normalizeRotation / operator* / map / exp
//     (Thirdparty/g2o/g2o/types/slam3d/se3quat.h:55-64, 104-117, 217-258),
//   Eigen Quaternion(Matrix3) / toRotationMatrix / _transformVector / product,
//   Eigen::LDLT<MatrixXd> (diagonal pivoting, lower triangle) as used by
//     LinearSolverDense::solve (solvers/dense/linear_solver_dense.h:65-113).
#pragma once
#include <float.h>
#include <math.h>

#if defined(__HIPCC__)
#define SE3_HD __host__ __device__ __forceinline__
#else
#define SE3_HD inline
#endif

namespace gfse3 {

struct Quat {
    double w, x, y, z;
};

struct SE3 {
    Quat r;
    double t[3];
};

SE3_HD void normalize(Quat& q) {
    if (q.w < 0) {
        q.w = -q.w;
        q.x = -q.x;
        q.y = -q.y;
        q.z = -q.z;
    }
    // coeffs() = (x, y, z, w), squaredNorm reduced as two 2-wide packets
    const double n = sqrt((q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w));
    q.x /= n;
    q.y /= n;
    q.z /= n;
    q.w /= n;
}

// Eigen quaternionbase_assign_impl<Matrix3>; R row-major.
SE3_HD Quat from_R(const double* m) {
    Quat q;
    double t = m[0] + (m[4] + m[8]);
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = c[0];
        q.y = c[1];
        q.z = c[2];
    }
    return q;
}

SE3_HD void to_R(const Quat& q, double* R) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1 - (tyy + tzz);
    R[1] = txy - twz;
    R[2] = txz + twy;
    R[3] = txy + twz;
    R[4] = 1 - (txx + tzz);
    R[5] = tyz - twx;
    R[6] = txz - twy;
    R[7] = tyz + twx;
    R[8] = 1 - (txx + tyy);
}

SE3_HD void rotate(const Quat& q, const double* v, double* o) {
    double u0 = q.y * v[2] - q.z * v[1], u1 = q.z * v[0] - q.x * v[2], u2 = q.x * v[1] - q.y * v[0];
    u0 += u0;
    u1 += u1;
    u2 += u2;
    o[0] = v[0] + q.w * u0 + (q.y * u2 - q.z * u1);
    o[1] = v[1] + q.w * u1 + (q.z * u0 - q.x * u2);
    o[2] = v[2] + q.w * u2 + (q.x * u1 - q.y * u0);
}

SE3_HD void map(const SE3& T, const double* p, double* o) {
    rotate(T.r, p, o);
    o[0] += T.t[0];
    o[1] += T.t[1];
    o[2] += T.t[2];
}

SE3_HD Quat mul(const Quat& a, const Quat& b) {
    Quat r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

// exp(u) * T for the update u = (omega, upsilon)
SE3_HD SE3 exp_mul(const double* u, const SE3& T) {
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt((w0 * w0 + w1 * w1) + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0 ? 1.0 : 0.0) + O[i]) + O2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double s = sin(theta), c = cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), cc = (theta - s) / pow(theta, 3.0);  // libm pow(double, double)
        for (int i = 0; i < 9; i++) {
            const double I = i % 4 == 0 ? 1.0 : 0.0;
            R[i] = (I + a * O[i]) + b * O2[i];
            V[i] = (I + b * O[i]) + cc * O2[i];
        }
    }
    SE3 E;
    E.r = from_R(R);
    for (int i = 0; i < 3; i++) E.t[i] = V[3 * i] * u[3] + V[3 * i + 1] * u[4] + V[3 * i + 2] * u[5];
    normalize(E.r);
    // E * T
    SE3 P;
    double rt[3];
    rotate(E.r, T.t, rt);
    for (int i = 0; i < 3; i++) P.t[i] = E.t[i] + rt[i];
    P.r = mul(E.r, T.r);
    normalize(P.r);
    return P;
}

// Eigen::LDLT (lower, diagonal pivoting) factor + solve of the 6x6 system
// A x = b; A row-major, only its lower triangle is read. Returns isPositive().
// x is written only when the factorisation is positive.
SE3_HD bool ldlt6(const double* Ain, const double* b, double* x) {
    const int n = 6;
    double A[36];
    for (int i = 0; i < 36; i++) A[i] = Ain[i];
    int perm[6];
    bool found_zero = false;
    int sign = 0;  // 0 zero, 1 psd, 2 nsd, 3 indefinite
    double temp[6];
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(A[k * n + k]);
        for (int i = k + 1; i < n; i++)
            if (fabs(A[i * n + i]) > bv) bv = fabs(A[i * n + i]), big = i;
        perm[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) {
                double t = A[k * n + j];
                A[k * n + j] = A[big * n + j];
                A[big * n + j] = t;
            }
            for (int i = big + 1; i < n; i++) {
                double t = A[i * n + k];
                A[i * n + k] = A[i * n + big];
                A[i * n + big] = t;
            }
            double t = A[k * n + k];
            A[k * n + k] = A[big * n + big];
            A[big * n + big] = t;
            for (int i = k + 1; i < big; i++) {
                double t2 = A[i * n + k];
                A[i * n + k] = A[big * n + i];
                A[big * n + i] = t2;
            }
        }
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = A[j * n + j] * A[k * n + j];
            double s = 0;
            for (int j = 0; j < k; j++) s += A[k * n + j] * temp[j];
            A[k * n + k] -= s;
            for (int i = k + 1; i < n; i++) {
                double t = 0;
                for (int j = 0; j < k; j++) t += A[i * n + j] * temp[j];
                A[i * n + k] -= t;
            }
        }
        const double akk = A[k * n + k];
        const bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) {
            sign = 0;
            for (int j = 0; j < n; j++) perm[j] = j;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; i++) A[i * n + k] /= akk;
        if (!valid) found_zero = true;
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0)
                sign = 1;
            else if (akk < 0)
                sign = 2;
        }
    }
    (void)found_zero;
    if (!(sign == 1 || sign == 0)) return false;
    double y[6];
    for (int i = 0; i < n; i++) y[i] = b[i];
    for (int k = 0; k < n; k++) {
        double t = y[k];
        y[k] = y[perm[k]];
        y[perm[k]] = t;
    }
    for (int j = 0; j < n; j++)
        for (int i = j + 1; i < n; i++) y[i] -= A[i * n + j] * y[j];
    for (int i = 0; i < n; i++) y[i] = fabs(A[i * n + i]) > DBL_MIN ? y[i] / A[i * n + i] : 0.0;
    for (int i = n - 1; i >= 0; i--) {
        double s = 0;
        for (int k = i + 1; k < n; k++) s += A[k * n + i] * y[k];
        y[i] -= s;
    }
    for (int k = n - 1; k >= 0; k--) {
        double t = y[k];
        y[k] = y[perm[k]];
        y[perm[k]] = t;
    }
    for (int i = 0; i < n; i++) x[i] = y[i];
    return true;
}

}  // namespace gfse3
