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

// Eigen quaternionbase_assign_impl<Matrix3>; R row-major. The branch on the
// largest diagonal entry i is expanded into three compile-time cases (the
// same arithmetic), so m is never indexed by a run-time value: on the device
// that would put the matrix in scratch memory.
template <int I>
SE3_HD Quat from_R_diag(const double* m) {
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    double t = sqrt(m[4 * I] - m[4 * J] - m[4 * K] + 1.0);
    double c[3];
    c[I] = 0.5 * t;
    t = 0.5 / t;
    Quat q;
    q.w = (m[3 * K + J] - m[3 * J + K]) * t;
    c[J] = (m[3 * J + I] + m[3 * I + J]) * t;
    c[K] = (m[3 * K + I] + m[3 * I + K]) * t;
    q.x = c[0];
    q.y = c[1];
    q.z = c[2];
    return q;
}

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
        if (m[8] > (i ? m[4] : m[0])) i = 2;
        q = i == 0 ? from_R_diag<0>(m) : i == 1 ? from_R_diag<1>(m) : from_R_diag<2>(m);
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
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) O2[3 * i + j] = O[3 * i] * O[j] + O[3 * i + 1] * O[3 + j] + O[3 * i + 2] * O[6 + j];
    double R[9], V[9];
    if (theta < 0.00001) {
#pragma unroll
        for (int i = 0; i < 9; i++) R[i] = ((i % 4 == 0 ? 1.0 : 0.0) + O[i]) + O2[i];
#pragma unroll
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double s = sin(theta), c = cos(theta);
        const double a = s / theta, b = (1 - c) / (theta * theta), cc = (theta - s) / pow(theta, 3.0);  // libm pow(double, double)
#pragma unroll
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
// x is written only when the factorisation is positive. Every array index is
// a compile-time constant (template recursion over the pivot step, pivot
// swaps selected by comparison), so A stays in registers on the device; the
// arithmetic and its order are those of Eigen's ldlt_inplace<Lower>::unblocked
// and LDLT::_solve_impl.
namespace ldlt_detail {

// conditional exchange as two selects (no branch, no address arithmetic)
SE3_HD void csw(bool c, double& a, double& b) {
    const double ta = c ? b : a, tb = c ? a : b;
    a = ta;
    b = tb;
}

// symmetric swap of row/column K and B (K < B) within the lower triangle, if c
template <int K, int B>
SE3_HD void sym_swap(double (&A)[36], bool c) {
#pragma unroll
    for (int j = 0; j < K; j++) csw(c, A[K * 6 + j], A[B * 6 + j]);
#pragma unroll
    for (int i = B + 1; i < 6; i++) csw(c, A[i * 6 + K], A[i * 6 + B]);
    csw(c, A[K * 7], A[B * 7]);
#pragma unroll
    for (int i = K + 1; i < B; i++) csw(c, A[i * 6 + K], A[B * 6 + i]);
}

template <int K, int B>
SE3_HD void pivot(double (&A)[36], int big) {
    if constexpr (B < 6) {
        sym_swap<K, B>(A, big == B);
        pivot<K, B + 1>(A, big);
    }
}

template <int K, int B>
SE3_HD void perm_vec(double (&y)[6], int p) {
    if constexpr (B < 6) {
        csw(p == B, y[K], y[B]);
        perm_vec<K, B + 1>(y, p);
    }
}

template <int K>
SE3_HD void step(double (&A)[36], int (&perm)[6], int& sign, bool& stop) {
    if constexpr (K < 6) {
        int big = K;
        double bv = fabs(A[K * 7]);
#pragma unroll
        for (int i = K + 1; i < 6; i++)
            if (fabs(A[i * 7]) > bv) bv = fabs(A[i * 7]), big = i;
        perm[K] = big;
        pivot<K, K + 1>(A, big);
        if constexpr (K > 0) {
            double temp[K];
#pragma unroll
            for (int j = 0; j < K; j++) temp[j] = A[j * 7] * A[K * 6 + j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < K; j++) s += A[K * 6 + j] * temp[j];
            A[K * 7] -= s;
#pragma unroll
            for (int i = K + 1; i < 6; i++) {
                double t = 0;
#pragma unroll
                for (int j = 0; j < K; j++) t += A[i * 6 + j] * temp[j];
                A[i * 6 + K] -= t;
            }
        }
        const double akk = A[K * 7];
        const bool valid = fabs(akk) > 0;
        if (K == 0 && !valid) {  // zero matrix: identity transpositions, ZeroSign
            sign = 0;
#pragma unroll
            for (int j = 0; j < 6; j++) perm[j] = j;
            stop = true;
            return;
        }
        if (valid) {
#pragma unroll
            for (int i = K + 1; i < 6; i++) A[i * 6 + K] /= akk;
        }
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
        step<K + 1>(A, perm, sign, stop);
    }
}

}  // namespace ldlt_detail

SE3_HD bool ldlt6(const double* Ain, const double* b, double* x) {
    double A[36];
#pragma unroll
    for (int i = 0; i < 36; i++) A[i] = Ain[i];
    int perm[6];
    int sign = 0;  // 0 zero, 1 psd, 2 nsd, 3 indefinite
    bool stop = false;
    ldlt_detail::step<0>(A, perm, sign, stop);
    if (!(sign == 1 || sign == 0)) return false;
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = b[i];
    // y = P b
    ldlt_detail::perm_vec<0, 1>(y, perm[0]);
    ldlt_detail::perm_vec<1, 2>(y, perm[1]);
    ldlt_detail::perm_vec<2, 3>(y, perm[2]);
    ldlt_detail::perm_vec<3, 4>(y, perm[3]);
    ldlt_detail::perm_vec<4, 5>(y, perm[4]);
    // L^-1 (unit lower, column axpy order)
#pragma unroll
    for (int j = 0; j < 6; j++)
#pragma unroll
        for (int i = j + 1; i < 6; i++) y[i] -= A[i * 6 + j] * y[j];
    // D^+ (pseudo-inverse below numeric_limits<double>::min())
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = fabs(A[i * 7]) > DBL_MIN ? y[i] / A[i * 7] : 0.0;
    // L^-T
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = 0;
#pragma unroll
        for (int k = i + 1; k < 6; k++) s += A[k * 6 + i] * y[k];
        y[i] -= s;
    }
    // P^-1
    ldlt_detail::perm_vec<4, 5>(y, perm[4]);
    ldlt_detail::perm_vec<3, 4>(y, perm[3]);
    ldlt_detail::perm_vec<2, 3>(y, perm[2]);
    ldlt_detail::perm_vec<1, 2>(y, perm[1]);
    ldlt_detail::perm_vec<0, 1>(y, perm[0]);
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

}  // namespace gfse3
