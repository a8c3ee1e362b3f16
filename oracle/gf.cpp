// CPU ORACLE (test infrastructure) — good-feature rows G1-G7 of SURVEY.md §8a,
// restated from include/Observability.h, include/Util.hpp and
// src/Observability.cc in f64 (the reference uses Armadillo double matrices).
// Armadillo/LAPACK internals are restated as documented in DESIGN.md:
// 3x3 inverse by cofactors (arma inv_tiny), Cholesky in natural summation
// order (dpotrf), product of the Cholesky diagonal with Armadillo's two-way
// accumulation, LU log|det| fallback (dgetrf partial pivoting).
#include <stdlib.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <memory>
#include <queue>
#include <vector>

#include "oracle_common.h"

namespace orc {

// ------------------------------------------------------------ G1 kinematics
typedef double M4[4][4];

static void q2r(const double* q, double R[3][3]) {  // Util.hpp:302-316
    double x = q[1], y = q[2], z = q[3], r = q[0];
    R[0][0] = r * r + x * x - y * y - z * z;
    R[0][1] = 2.0 * (x * y - r * z);
    R[0][2] = 2.0 * (z * x + r * y);
    R[1][0] = 2.0 * (x * y + r * z);
    R[1][1] = r * r - x * x + y * y - z * z;
    R[1][2] = 2.0 * (y * z - r * x);
    R[2][0] = 2.0 * (z * x - r * y);
    R[2][1] = 2.0 * (y * z + r * x);
    R[2][2] = r * r - x * x - y * y + z * z;
}

// arma::inv for 3x3 (cofactor formula, inv_noalias_tinymat)
static bool inv3(const double X[3][3], double O[3][3]) {
    // column-major accessors of the reference: a_j = column j
    const double val1 = X[0][0] * (X[2][2] * X[1][1] - X[1][2] * X[2][1]);
    const double val2 = X[0][1] * (X[2][2] * X[1][0] - X[1][2] * X[2][0]);
    const double val3 = X[0][2] * (X[2][1] * X[1][0] - X[1][1] * X[2][0]);
    const double det = val1 - val2 + val3;
    if (std::fabs(det) < DBL_EPSILON) return false;
    O[0][0] = (X[2][2] * X[1][1] - X[1][2] * X[2][1]) / det;
    O[1][0] = -(X[2][2] * X[1][0] - X[2][0] * X[1][2]) / det;
    O[2][0] = (X[2][1] * X[1][0] - X[2][0] * X[1][1]) / det;
    O[0][1] = -(X[2][2] * X[0][1] - X[2][1] * X[0][2]) / det;
    O[1][1] = (X[2][2] * X[0][0] - X[2][0] * X[0][2]) / det;
    O[2][1] = -(X[2][1] * X[0][0] - X[2][0] * X[0][1]) / det;
    O[0][2] = (X[1][2] * X[0][1] - X[1][1] * X[0][2]) / det;
    O[1][2] = -(X[1][2] * X[0][0] - X[1][0] * X[0][2]) / det;
    O[2][2] = (X[1][1] * X[0][0] - X[1][0] * X[0][1]) / det;
    return true;
}

static double norm3(const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// dqomegadt_by_domega, Util.hpp:440-506
static void dqomegadt_by_domega(const double* w, double dt, double R[4][3]) {
    double wm = norm3(w);
    std::memset(R, 0, sizeof(double) * 12);
    if (std::fabs(wm) < 1e-8) {
        R[1][0] = R[2][1] = R[3][2] = dt / 2;
        return;
    }
    auto d0 = [&](double a) { return (-dt / 2.0) * (a / wm) * std::sin(wm * dt / 2.0); };
    auto dA = [&](double a) {
        return (dt / 2.0) * a * a / (wm * wm) * std::cos(wm * dt / 2.0) +
               (1.0 / wm) * (1.0 - a * a / (wm * wm)) * std::sin(wm * dt / 2.0);
    };
    auto dB = [&](double a, double b) {
        return (a * b / (wm * wm)) * ((dt / 2.0) * std::cos(wm * dt / 2.0) - (1.0 / wm) * std::sin(wm * dt / 2.0));
    };
    R[0][0] = d0(w[0]);
    R[0][1] = d0(w[1]);
    R[0][2] = d0(w[2]);
    R[1][0] = dA(w[0]);
    R[1][1] = dB(w[0], w[1]);
    R[1][2] = dB(w[0], w[2]);
    R[2][0] = dB(w[1], w[0]);
    R[2][1] = dA(w[1]);
    R[2][2] = dB(w[1], w[2]);
    R[3][0] = dB(w[2], w[0]);
    R[3][1] = dB(w[2], w[1]);
    R[3][2] = dA(w[2]);
}

// compute_F_subblock, Util.hpp:787-881
static void compute_F(const double* Xv, double dt, double FQ[4][4], double FO[4][3]) {
    const double* w = Xv + 10;
    const double* qo = Xv + 3;
    double v[3] = {w[0] * dt, w[1] * dt, w[2] * dt};
    double theta = norm3(v);
    double q[4];
    if (theta < 1e-6) {
        q[0] = 1;
        q[1] = q[2] = q[3] = 0;
    } else {
        double vn[3] = {v[0] / theta, v[1] / theta, v[2] / theta};
        double nn = norm3(vn), s = std::sin(theta / 2.0);
        q[0] = std::cos(theta / 2.0);
        for (int i = 0; i < 3; i++) q[1 + i] = s * (vn[i] / nn);
    }
    double R = q[0], X = q[1], Y = q[2], Z = q[3];
    double fq[4][4] = {{R, -X, -Y, -Z}, {X, R, Z, -Y}, {Y, -Z, R, X}, {Z, Y, -X, R}};
    std::memcpy(FQ, fq, sizeof(fq));
    R = qo[0], X = qo[1], Y = qo[2], Z = qo[3];
    double d31[4][4] = {{R, -X, -Y, -Z}, {X, R, -Z, Y}, {Y, Z, R, -X}, {Z, -Y, X, R}};
    double dq[4][3];
    dqomegadt_by_domega(w, dt, dq);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += d31[i][k] * dq[k][j];
            FO[i][j] = s;
        }
}

// convert_PWLS_Vec_To_Homo + QUAT2DCM_float, Util.hpp:613-635, :883-905
static void pwls_to_Tcw(const double* Xv, float* T) {
    float Rwc[3][3], twc[3];
    double x = Xv[4], y = Xv[5], z = Xv[6], r = Xv[3];
    Rwc[0][0] = (float)(r * r + x * x - y * y - z * z);
    Rwc[0][1] = (float)(2.0 * (x * y - r * z));
    Rwc[0][2] = (float)(2.0 * (z * x + r * y));
    Rwc[1][0] = (float)(2.0 * (x * y + r * z));
    Rwc[1][1] = (float)(r * r - x * x + y * y - z * z);
    Rwc[1][2] = (float)(2.0 * (y * z - r * x));
    Rwc[2][0] = (float)(2.0 * (z * x - r * y));
    Rwc[2][1] = (float)(2.0 * (y * z + r * x));
    Rwc[2][2] = (float)(r * r - x * x - y * y + z * z);
    for (int i = 0; i < 3; i++) twc[i] = (float)Xv[i];
    std::memset(T, 0, 64);
    T[15] = 1.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = Rwc[j][i];
        float a = -Rwc[0][i] * twc[0], b = -Rwc[1][i] * twc[1], c = -Rwc[2][i] * twc[2];
        T[4 * i + 3] = (a + b) + c;
    }
}

// propagate_PWLS, Util.hpp:968-1005
static void propagate(const double* Xv, double dt, double* out) {
    std::memcpy(out, Xv, 13 * sizeof(double));
    for (int i = 0; i < 3; i++) out[i] = Xv[i] + Xv[7 + i] * dt;
    double wv[3] = {Xv[10] * dt, Xv[11] * dt, Xv[12] * dt};
    double a = norm3(wv), u[3];
    if (a > 0.0000001) {
        for (int i = 0; i < 3; i++) u[i] = wv[i] / a;
    } else {
        a = 0;
        u[0] = u[1] = u[2] = 0;
    }
    double qm[4] = {std::cos(a / 2), u[0] * std::sin(a / 2), u[1] * std::sin(a / 2), u[2] * std::sin(a / 2)};
    const double* q1 = Xv + 3;
    double A = q1[0], B = q1[1], C = q1[2], D = q1[3], W = qm[0], X = qm[1], Y = qm[2], Z = qm[3];
    double qp[4] = {A * W - B * X - C * Y - D * Z, A * X + B * W + C * Z - D * Y, A * Y - B * Z + C * W + D * X,
                    A * Z + B * Y - C * X + D * W};
    double nq = std::sqrt(qp[0] * qp[0] + qp[1] * qp[1] + qp[2] * qp[2] + qp[3] * qp[3]);
    for (int i = 0; i < 4; i++) out[3 + i] = qp[i] / nq;
}

void predict(const double* Xv0, double dt_in, int nseg, gf_kine* out) {
    double cur[13];
    std::memcpy(cur, Xv0, sizeof(cur));
    for (int s = 0; s < nseg; s++) {
        gf_kine& K = out[s];
        K.dt = (float)dt_in;
        K.dt_inseg = (float)K.dt / (float)13;
        std::memcpy(K.Xv, cur, sizeof(cur));
        pwls_to_Tcw(K.Xv, K.Tcw);
        double FQ[4][4], FO[4][3];
        compute_F(K.Xv, K.dt_inseg, FQ, FO);
        std::memcpy(K.F_Q_inSeg, FQ, sizeof(FQ));
        std::memcpy(K.F_Omg_inSeg, FO, sizeof(FO));
        compute_F(K.Xv, K.dt, FQ, FO);
        std::memcpy(K.F_Q, FQ, sizeof(FQ));
        std::memcpy(K.F_Omg, FO, sizeof(FO));
        double nxt[13];
        propagate(K.Xv, K.dt, nxt);
        std::memcpy(cur, nxt, sizeof(cur));
    }
}

// DCM2QUAT_float (arma overload), Util.hpp:570-611 — float arithmetic
static void dcm2quat_float(const float R[3][3], double* q) {
    float qf[4];
    float trace = R[0][0] + R[1][1] + R[2][2];
    if (trace > 0) {
        float s = std::sqrt(trace + 1.0f) * 2;
        qf[0] = 0.25f * s;
        qf[1] = (R[2][1] - R[1][2]) / s;
        qf[2] = (R[0][2] - R[2][0]) / s;
        qf[3] = (R[1][0] - R[0][1]) / s;
    } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
        float s = 2.0f * std::sqrt(1.0f + R[0][0] - R[1][1] - R[2][2]);
        qf[0] = (R[2][1] - R[1][2]) / s;
        qf[1] = 0.25f * s;
        qf[2] = (R[0][1] + R[1][0]) / s;
        qf[3] = (R[0][2] + R[2][0]) / s;
    } else if (R[1][1] > R[2][2]) {
        float s = 2.0f * std::sqrt(1.0f + R[1][1] - R[0][0] - R[2][2]);
        qf[0] = (R[0][2] - R[2][0]) / s;
        qf[1] = (R[0][1] + R[1][0]) / s;
        qf[2] = 0.25f * s;
        qf[3] = (R[1][2] + R[2][1]) / s;
    } else {
        float s = 2.0f * std::sqrt(1.0f + R[2][2] - R[0][0] - R[1][1]);
        qf[0] = (R[1][0] - R[0][1]) / s;
        qf[1] = (R[0][2] + R[2][0]) / s;
        qf[2] = (R[1][2] + R[2][1]) / s;
        qf[3] = 0.25f * s;
    }
    for (int i = 0; i < 4; i++) q[i] = qf[i];
    if (q[0] < 0)
        for (int i = 0; i < 4; i++) q[i] = -1.0 * q[i];
}

// 4x4 float product and rigid inverse as cv::Mat ops (float, left-to-right)
static void mul44(const float* A, const float* B, float* C) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = A[4 * i] * B[j];
            for (int k = 1; k < 4; k++) s = s + A[4 * i + k] * B[4 * k + j];
            C[4 * i + j] = s;
        }
}

// convert_Homo_Pair_To_PWLS_Vec, Util.hpp:907-954. (Tcw_0 * Twc_1).inv() is
// taken as the rigid-transform inverse in float (cv::Mat::inv on a 4x4 pose;
// LU inverse of OpenCV restated as the exact rigid inverse).
void update_pwls(double t0, const float* Tcw0, double t1, const float* Twc1, double* Xv) {
    std::memset(Xv, 0, 13 * sizeof(double));
    for (int i = 0; i < 3; i++) Xv[i] = Twc1[4 * i + 3];
    float R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = Twc1[4 * i + j];
    dcm2quat_float(R, Xv + 3);
    float P[16], Ti[16];
    mul44(Tcw0, Twc1, P);
    // rigid inverse
    std::memset(Ti, 0, sizeof(Ti));
    Ti[15] = 1.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Ti[4 * i + j] = P[4 * j + i];
        float a = -P[0 * 4 + i] * P[3], b = -P[1 * 4 + i] * P[7], c = -P[2 * 4 + i] * P[11];
        Ti[4 * i + 3] = (a + b) + c;
    }
    float dt = (float)(t1 - t0);
    for (int i = 0; i < 3; i++) Xv[7 + i] = Ti[4 * i + 3] / dt;
    // get_angular_velocity_with_H: 0.5 * (R - R^T) off-diagonals, float
    float O21 = Ti[2 * 4 + 1] - Ti[1 * 4 + 2], O02 = Ti[0 * 4 + 2] - Ti[2 * 4 + 0], O10 = Ti[1 * 4 + 0] - Ti[0 * 4 + 1];
    Xv[10] = (0.5 * O21) / dt;
    Xv[11] = (0.5 * O02) / dt;
    Xv[12] = (0.5 * O10) / dt;
}

// ------------------------------------------------------------ G2/G3 Jacobian
// dRq_times_a_by_dq, Util.hpp:391-438
static void dRq_times_a(const double* q, const double* a, double RES[3][4]) {
    double q0 = q[0], qx = q[1], qy = q[2], qz = q[3];
    double D[4][3][3] = {{{2.0 * q0, -2.0 * qz, 2.0 * qy}, {2.0 * qz, 2.0 * q0, -2.0 * qx}, {-2.0 * qy, 2.0 * qx, 2.0 * q0}},
                         {{2.0 * qx, 2.0 * qy, 2.0 * qz}, {2.0 * qy, -2.0 * qx, -2.0 * q0}, {2.0 * qz, 2.0 * q0, -2.0 * qx}},
                         {{-2.0 * qy, 2.0 * qx, 2.0 * q0}, {2.0 * qx, 2.0 * qy, 2.0 * qz}, {-2.0 * q0, 2.0 * qz, -2.0 * qy}},
                         {{-2.0 * qz, -2.0 * q0, 2.0 * qx}, {2.0 * q0, -2.0 * qz, 2.0 * qy}, {2.0 * qx, 2.0 * qy, 2.0 * qz}}};
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 3; r++) RES[r][c] = D[c][r][0] * a[0] + D[c][r][1] * a[1] + D[c][r][2] * a[2];
}

// compute_H_subblock_simplied, Observability.h:460-515. H is 2x7 row-major.
bool compute_H(const gf_obs_camera* cam, const double* Xv, const double* y, bool check_viz, double* H, float* uv) {
    const double* q = Xv + 3;
    double Rq[3][3], R[3][3];
    q2r(q, Rq);
    if (!inv3(Rq, R)) std::memset(R, 0, sizeof(R));
    double t[3] = {y[0] - Xv[0], y[1] - Xv[1], y[2] - Xv[2]};
    double h[3];
    for (int i = 0; i < 3; i++) h[i] = R[i][0] * t[0] + R[i][1] * t[1] + R[i][2] * t[2];
    float u, v;
    if (h[2] > 0) {
        u = (float)((double)(float)cam->fu * h[0] / h[2] + (double)(float)cam->cx);
        v = (float)((double)(float)cam->fv * h[1] / h[2] + (double)(float)cam->cy);
    } else {
        u = FLT_MAX;
        v = FLT_MAX;
    }
    uv[0] = u;
    uv[1] = v;
    if (check_viz) {
        if (h[2] < 0.0 + cam->bound_depth) return false;
        if (u < cam->min_x - cam->bound_x || u > cam->max_x + cam->bound_x) return false;
        if (v < cam->min_y - cam->bound_y || v > cam->max_y + cam->bound_y) return false;
    }
    double dh[2][3];
    if (std::fabs(h[2]) < 1e-6) {
        std::memset(dh, 0, sizeof(dh));
    } else {
        double z2 = h[2] * h[2];
        dh[0][0] = cam->fu / h[2];
        dh[0][1] = 0.0;
        dh[0][2] = -h[0] * cam->fu / z2;
        dh[1][0] = 0.0;
        dh[1][1] = cam->fv / h[2];
        dh[1][2] = -h[1] * cam->fv / z2;
    }
    double qc[4] = {q[0], -1.0 * q[1], -1.0 * q[2], -1.0 * q[3]};  // qconj
    double dR[3][4];
    dRq_times_a(qc, t, dR);
    for (int r = 0; r < 3; r++)
        for (int c = 1; c < 4; c++) dR[r][c] = -dR[r][c];  // * dqbar_by_dq = diag(1,-1,-1,-1)
    for (int i = 0; i < 2; i++) {
        for (int j = 0; j < 3; j++) H[7 * i + j] = -1.0 * (dh[i][0] * R[0][j] + dh[i][1] * R[1][j] + dh[i][2] * R[2][j]);
        for (int j = 0; j < 4; j++) H[7 * i + 3 + j] = dh[i][0] * dR[0][j] + dh[i][1] * dR[1][j] + dh[i][2] * dR[2][j];
    }
    return true;
}

// reWeightInfoMat (Observability.h:517-596) + info = H_rw^T H_rw
static void info_block(const double* H, double sigma2, double* info) {
    double Hw[14];
    double s = std::sqrt(sigma2);
    double w = s / (s * s);  // inv(chol(sigma2 I)) by the 2x2 cofactor inverse
    for (int i = 0; i < 14; i++) Hw[i] = w * H[i];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) info[7 * i + j] = Hw[i] * Hw[j] + Hw[7 + i] * Hw[7 + j];
}

// ------------------------------------------------------------ G5 logDet
static double prod_diag(const double* L) {
    double v1 = 1, v2 = 1;
    int i, j;
    for (i = 0, j = 1; j < 7; i += 2, j += 2) {
        v1 *= L[8 * i];
        v2 *= L[8 * j];
    }
    if (i < 7) v1 *= L[8 * i];
    return v1 * v2;
}

double logdet7(const double* M) {
    double L[49];
    std::memset(L, 0, sizeof(L));
    bool ok = true;
    for (int j = 0; j < 7 && ok; j++) {
        double s = M[8 * j];
        for (int k = 0; k < j; k++) s -= L[7 * j + k] * L[7 * j + k];
        if (!(s > 0)) {
            ok = false;
            break;
        }
        double d = std::sqrt(s);
        L[8 * j] = d;
        const double rd = 1.0 / d;  // dpotf2 scales the column by ONE / AJJ
        for (int i = j + 1; i < 7; i++) {
            double t = M[7 * i + j];
            for (int k = 0; k < j; k++) t -= L[7 * i + k] * L[7 * j + k];
            L[7 * i + j] = t * rd;
        }
    }
    if (ok) return 2 * std::log(prod_diag(L));
    // arma::log_det via LU with partial pivoting, real part = sum log|u_ii|
    double A[49];
    std::memcpy(A, M, sizeof(A));
    double acc = 0;
    for (int c = 0; c < 7; c++) {
        int p = c;
        double best = std::fabs(A[7 * c + c]);
        for (int r = c + 1; r < 7; r++)
            if (std::fabs(A[7 * r + c]) > best) best = std::fabs(A[7 * r + c]), p = r;
        if (p != c)
            for (int k = 0; k < 7; k++) std::swap(A[7 * c + k], A[7 * p + k]);
        double piv = A[7 * c + c];
        if (piv != 0)
            for (int r = c + 1; r < 7; r++) {
                double f = A[7 * r + c] / piv;
                A[7 * r + c] = f;
                for (int k = c + 1; k < 7; k++) A[7 * r + k] -= f * A[7 * c + k];
            }
        acc += std::log(std::fabs(piv));
    }
    return acc;
}

// ------------------------------------------------------------ RNG
long long g_ldets = 0;
static int g_rand_calls = 0;  // rand() calls of the last active-match / max-vol call

struct Rand {  // glibc random_r TYPE_3 (the generator behind std::rand)
    struct random_data rd;
    char state[128];
    ~Rand() { g_rand_calls = calls; }
    int calls = 0;
    void seed(unsigned s) {
        std::memset(&rd, 0, sizeof(rd));
        initstate_r(s, state, sizeof(state), &rd);
    }
    // continue from a saved state (gf_rng: the 31 words and the front / rear
    // indices of glibc's random_data)
    void load(const gf_rng& g) {
        seed(1);
        for (int i = 0; i < 31; i++) rd.state[i] = g.state[i];
        rd.fptr = rd.state + g.f;
        rd.rptr = rd.state + g.r;
    }
    void save(gf_rng& g) const {
        for (int i = 0; i < 31; i++) g.state[i] = rd.state[i];
        g.f = (int32_t)(rd.fptr - rd.state);
        g.r = (int32_t)(rd.rptr - rd.state);
    }
    int next() {
        int32_t r;
        random_r(&rd, &r);
        calls++;
        return r;
    }
};

}  // namespace orc

// ============================================================== C API
extern "C" {

int orc_rand_sequence(unsigned seed, int n, int32_t* out) {
    orc::Rand R;
    R.seed(seed);
    for (int i = 0; i < n; i++) out[i] = R.next();
    return GF_OK;
}

int orc_obs_predict(const double* Xv, double dt, int nseg, gf_kine* out) {
    orc::predict(Xv, dt, nseg, out);
    return GF_OK;
}

int orc_obs_update(double t0, const float* Tcw0, double t1, const float* Twc1, double* Xv) {
    orc::update_pwls(t0, Tcw0, t1, Twc1, Xv);
    return GF_OK;
}

int orc_obs_build_info(const gf_obs_camera* cam, const double* Xv, const float* pos, const float* sigma2, int n,
                       int check_viz, double* H, double* info, float* uv, uint8_t* valid) {
    for (int i = 0; i < n; i++) {
        double y[3] = {pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]};
        double h[14];
        bool ok = orc::compute_H(cam, Xv, y, check_viz != 0, h, uv + 2 * i);
        valid[i] = ok;
        if (!ok) {
            std::memset(H + 14 * i, 0, 14 * sizeof(double));
            std::memset(info + 49 * i, 0, 49 * sizeof(double));
            continue;
        }
        std::memcpy(H + 14 * i, h, sizeof(h));
        orc::info_block(h, sigma2 ? (double)sigma2[i] : 1.0, info + 49 * i);
    }
    return GF_OK;
}

int orc_logdet(const double* M, int n, double* out) {
    for (int i = 0; i < n; i++) out[i] = orc::logdet7(M + 49 * i);
    return GF_OK;
}

// SearchByProjection_OnePoint (ORBmatcher.h:71-145) over a prebuilt grid.
int orc_match_project(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                      const gf_mp_view* views, const uint8_t* mp_desc, int m, float th, float nnratio,
                      int32_t* kp2mp, int32_t* score, int* nmatches);

// The time cap of runActiveMapMatching (Observability.cc:1260, 1275-1277,
// 1362-1370) replayed on elapsed times the device measured: round_el[i] is
// the elapsed time at round i's start, cap = time_for_match (same ticks);
// a round with round_el > cap ends at its first accepted draw, returning
// without leftovers. null round_el: no cap.
struct AmCap {
    const long long* round_el = nullptr;
    int nrec = 0;
    long long cap = 0;
    int* cut_round = nullptr;
};

// runActiveMapMatching, Observability.cc:1249-1524 (FRAME_INFO_MATRIX).
static int active_match(orc::Rand& R, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                        const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated, const double* info,
                        const double* H, int m, const double* base, const float* level_sigma2, int num_to_match,
                        float th, float nnratio, int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft,
                        int* nmatched, const AmCap& tc = AmCap{});

int orc_obs_active_match(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                         const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated, const double* info,
                         const double* H, const float* uv, int m, const double* base, const float* level_sigma2,
                         int num_to_match, float th, float nnratio, unsigned rng_seed, int32_t* kp2mp,
                         int32_t* score, int32_t* left, int* nleft, int* nmatched) {
    (void)uv;
    orc::Rand R;
    R.seed(rng_seed);
    return active_match(R, fi, kps, desc, n, views, mp_desc, updated, info, H, m, base, level_sigma2, num_to_match, th,
                        nnratio, kp2mp, score, left, nleft, nmatched);
}

// Same, continuing the caller's std::rand() state (one sequence across frames).
int orc_obs_active_match_rng(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                             const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated,
                             const double* info, const double* H, int m, const double* base,
                             const float* level_sigma2, int num_to_match, float th, float nnratio, gf_rng* rng,
                             int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft, int* nmatched) {
    orc::Rand R;
    R.load(*rng);
    int rc = active_match(R, fi, kps, desc, n, views, mp_desc, updated, info, H, m, base, level_sigma2, num_to_match,
                          th, nnratio, kp2mp, score, left, nleft, nmatched);
    R.save(*rng);
    return rc;
}

static int active_match(orc::Rand& R, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                        const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated, const double* info,
                        const double* H, int m, const double* base, const float* level_sigma2, int num_to_match,
                        float th, float nnratio, int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft,
                        int* nmatched, const AmCap& tc) {
    *nleft = 0;
    *nmatched = 0;
    orc::g_ldets = 0;
    if (tc.cut_round) *tc.cut_round = -1;
    auto push_left_all = [&]() {
        for (int i = 0; i < m; i++)
            if (views[i].in_view) left[(*nleft)++] = i;
    };
    if (m == 0 || num_to_match <= 0 || (tc.round_el && tc.cap <= 0)) {
        push_left_all();
        return GF_OK;
    }
    std::vector<int> lmkIdx;
    std::vector<double> visited;
    for (int i = 0; i < m; i++)
        if (views[i].in_view && updated[i]) {
            lmkIdx.push_back(i);
            visited.push_back(-1);
        }
    const size_t N = lmkIdx.size();
    const size_t szLazier = (size_t)((float)N / (float)num_to_match * 1.0);
    std::unique_ptr<orc::OnePointGrid, void (*)(orc::OnePointGrid*)> grid(orc::one_point_grid(fi, kps, n),
                                                                          orc::one_point_grid_free);
    double cur[49];
    std::memcpy(cur, base, sizeof(cur));
    struct SP {
        int idx;
        double score;
        bool operator<(const SP& o) const { return score < o.score; }
    };
    int nMatched = 0;
    for (size_t i = 0; i < (size_t)num_to_match; ++i) {
        std::priority_queue<SP> heap;
        std::vector<int> removeIdx;
        size_t numHit = 0, numRndQue = 0, szActual = std::min(szLazier, lmkIdx.size());
        const bool late = tc.round_el && szActual > 0 && (int)i < tc.nrec && tc.round_el[i] > tc.cap;
        while (numHit < szActual) {
            size_t j = 0;
            numRndQue = 0;
            while (numRndQue < 2000) {
                j = (size_t)(R.next() % (int)lmkIdx.size());
                if (visited[j] < (double)i) {
                    visited[j] = (double)i;
                    break;
                }
                ++numRndQue;
            }
            if (numRndQue >= 2000) break;
            int q = lmkIdx[j];
            ++numHit;
            if (late) {  // reach max time cap: return nMatched (:1366-1370)
                if (tc.cut_round) *tc.cut_round = (int)i;
                *nmatched = nMatched;
                return GF_OK;
            }
            double M[49];
            for (int k = 0; k < 49; k++) M[k] = cur[k] + info[49 * (size_t)q + k];
            heap.push(SP{q, orc::logdet7(M)});
            ++orc::g_ldets;
            if (numHit >= szActual) {
                SP top = heap.top();
                // SearchByProjection_OnePoint of map point top.idx (claims the keypoint)
                int bd = 0;
                const int bestIdx = orc::one_point(grid.get(), views[top.idx], mp_desc + 32 * (size_t)top.idx, desc,
                                                   th, nnratio, kp2mp, &bd);
                if (bestIdx >= 0) {
                    kp2mp[bestIdx] = top.idx;
                    score[bestIdx] = bd;
                    double s2 = (double)level_sigma2[kps[bestIdx].octave];
                    double blk[49];
                    orc::info_block(H + 14 * (size_t)top.idx, s2, blk);
                    for (int k = 0; k < 49; k++) cur[k] = cur[k] + blk[k];
                    removeIdx.push_back(top.idx);
                    ++nMatched;
                    break;
                } else {
                    removeIdx.push_back(top.idx);
                    heap.pop();
                    --numHit;
                }
            }
        }
        if (numRndQue >= 2000 || heap.empty() || removeIdx.empty()) break;
        if (lmkIdx.size() == removeIdx.size()) break;  // all tried: every entry stays in mLeftMapPoints
        std::sort(removeIdx.begin(), removeIdx.end());
        std::vector<int> nl;
        std::vector<double> nv;
        size_t a = 0, k = 0;
        while (a < lmkIdx.size()) {
            if (k >= removeIdx.size()) {
                nl.push_back(lmkIdx[a]);
                nv.push_back(visited[a]);
                ++a;
            } else if (lmkIdx[a] < removeIdx[k]) {
                nl.push_back(lmkIdx[a]);
                nv.push_back(visited[a]);
                ++a;
            } else {
                if (lmkIdx[a] == removeIdx[k]) ++a;
                ++k;
            }
        }
        lmkIdx.swap(nl);
        visited.swap(nv);
    }
    for (int q : lmkIdx) left[(*nleft)++] = q;
    *nmatched = nMatched;
    return GF_OK;
}

// The same under the time cap (the front end's budgets, gf_set_budgets).
int orc_obs_active_match_capped(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                                const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated,
                                const double* info, const double* H, int m, const double* base,
                                const float* level_sigma2, int num_to_match, float th, float nnratio, gf_rng* rng,
                                int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft, int* nmatched,
                                const long long* round_el, int nrec, long long cap, int* cut_round) {
    orc::Rand R;
    R.load(*rng);
    AmCap tc;
    tc.round_el = round_el;
    tc.nrec = nrec;
    tc.cap = cap;
    tc.cut_round = cut_round;
    int rc = active_match(R, fi, kps, desc, n, views, mp_desc, updated, info, H, m, base, level_sigma2, num_to_match,
                          th, nnratio, kp2mp, score, left, nleft, nmatched, tc);
    R.save(*rng);
    return rc;
}

// Max-volume selection: 1 baseline, 2 lazier selection, 3 automatic (deletion if 2k > n)
static int maxvol_select(orc::Rand& R, const double* info, const double* score, int n, int k, double sample_scale,
                         int mode, int32_t* out_idx, int* nout);

int orc_maxvol_select(const double* info, const double* score, int n, int k, double sample_scale, int mode,
                      unsigned rng_seed, int32_t* out_idx, int* nout) {
    orc::Rand R;
    R.seed(rng_seed);
    return maxvol_select(R, info, score, n, k, sample_scale, mode, out_idx, nout);
}

// Observability::setSelction_Number over map points (Observability.cc:1021-1247):
// MAP_INFO_MATRIX with the visibility check at Xv (batchInfoMat_Map, ObsScore
// 1), the pool of visible points in list order, then greedy_mtd 1 (baseline),
// 2 (lazier) or 3 (automatic, split over threadNeeded chunks when the pool is
// large: :1086-1160; the chunks run in chunk order on one rand() stream).
// setSelction_Number's greedy stage over a prepared pool (lmkSelectPool,
// Observability.cc:1072-1160): greedy_mtd 1 / 2 on the pool; 3 splits a
// large pool into threadNeeded chunks (:1086-1160) run in chunk order on one
// rand() stream (the reference runs them on threads sharing std::rand: an
// ordering assumption, docs/ORACLE_ASSUMPTIONS.md), then an automatic pass
// over the merged selections, which keep their pool scores (:1141-1146).
int orc_select_pool(const double* info, const double* score, int P, int k, int greedy_mtd, int max_threads,
                    gf_rng* rng, int32_t* out_idx, int* nout) {
    *nout = 0;
    if (greedy_mtd < 1 || greedy_mtd > 3) return GF_ERR_ARG;
    if (P <= 0) return GF_OK;
    orc::Rand R;
    R.load(*rng);
    const double scale = 6.0;
    if (greedy_mtd == 1 || greedy_mtd == 2) {
        maxvol_select(R, info, score, P, k, scale, greedy_mtd, out_idx, nout);
    } else {
        int T = 1;
        if (!((float)P - 1.2f * (float)k <= 10 || P < 2 * 1000)) T = std::min((int)std::lround((float)P / 1000.f), max_threads);
        T = std::max(T, 1);
        if (T == 1) {
            maxvol_select(R, info, score, P, k, scale, 3, out_idx, nout);
        } else {
            const int kpar = (int)std::ceil((float)k / (float)T * 1.2f);
            const int npar = (int)std::ceil((float)P / (float)T);
            std::vector<int> merged;  // pool positions, chunk by chunk
            for (int t = 0; t < T; t++) {
                const int lo = t * npar, hi = std::min(P, (t + 1) * npar);
                if (hi <= lo) continue;
                std::vector<int32_t> o(hi - lo);
                int no = 0;
                maxvol_select(R, &info[49 * (size_t)lo], &score[lo], hi - lo, kpar, scale, 3, o.data(), &no);
                for (int q = 0; q < no; q++) merged.push_back(lo + o[q]);
            }
            const int Mg = (int)merged.size();
            std::vector<double> minfo(49 * (size_t)std::max(Mg, 1)), mscore(std::max(Mg, 1));
            for (int j = 0; j < Mg; j++) {
                std::memcpy(&minfo[49 * (size_t)j], &info[49 * (size_t)merged[j]], 49 * sizeof(double));
                mscore[j] = score[merged[j]];
            }
            std::vector<int32_t> o(std::max(Mg, 1));
            int no = 0;
            maxvol_select(R, minfo.data(), mscore.data(), Mg, k, scale, 3, o.data(), &no);
            for (int q = 0; q < no; q++) out_idx[(*nout)++] = merged[o[q]];
        }
    }
    R.save(*rng);
    return GF_OK;
}

int orc_select_map_points(const gf_obs_camera* cam, const double* Xv, const float* pos, int n, int k,
                          int greedy_mtd, int max_threads, gf_rng* rng, int32_t* out_idx, int* nout) {
    *nout = 0;
    if (greedy_mtd < 1 || greedy_mtd > 3) return GF_ERR_ARG;
    std::vector<double> H(14 * (size_t)std::max(n, 1)), info(49 * (size_t)std::max(n, 1));
    std::vector<float> uv(2 * (size_t)std::max(n, 1));
    std::vector<uint8_t> valid(std::max(n, 1));
    orc_obs_build_info(cam, Xv, pos, nullptr, n, 1, H.data(), info.data(), uv.data(), valid.data());
    std::vector<int> pool;
    for (int i = 0; i < n; i++)
        if (valid[i]) pool.push_back(i);
    const int P = (int)pool.size();
    std::vector<double> pinfo(49 * (size_t)std::max(P, 1)), pscore(std::max(P, 1), 1.0);
    for (int j = 0; j < P; j++) std::memcpy(&pinfo[49 * (size_t)j], &info[49 * (size_t)pool[j]], 49 * sizeof(double));
    std::vector<int32_t> sel(std::max(P, 1));
    int ns = 0;
    int rc = orc_select_pool(pinfo.data(), pscore.data(), P, k, greedy_mtd, max_threads, rng, sel.data(), &ns);
    for (int q = 0; q < ns; q++) out_idx[(*nout)++] = pool[sel[q]];
    return rc;
}

static int maxvol_select(orc::Rand& R, const double* info, const double* score, int n, int k, double sample_scale,
                         int mode, int32_t* out_idx, int* nout) {
    *nout = 0;
    if (n == 0) return GF_OK;
    struct GP {
        int idx;
        double obs_score, upper;
        bool selected;
        std::vector<double> blk, sum;
    };
    std::vector<GP> pool(n);
    for (int i = 0; i < n; i++) {
        pool[i].idx = i;
        pool[i].obs_score = score[i];
        pool[i].selected = false;
        pool[i].upper = -DBL_MAX;
        pool[i].blk.assign(info + 49 * (size_t)i, info + 49 * (size_t)i + 49);
    }
    if (k >= n) {
        for (int i = 0; i < n; i++) out_idx[(*nout)++] = i;
        return GF_OK;
    }
    double cur[49];
    std::memset(cur, 0, sizeof(cur));
    for (int i = 0; i < 7; i++) cur[8 * i] = 0.00001;
    if (mode == 1) {  // maxVolSelection_BaselineGreedy
        for (int it = 0; it < k; ++it) {
            int maxLmk = -1;
            double maxDet = -DBL_MAX;
            for (auto& g : pool) {
                if (g.selected || g.obs_score < 0) {
                    g.upper = -DBL_MAX;
                    continue;
                }
                g.sum.resize(49);
                for (int q = 0; q < 49; q++) g.sum[q] = cur[q] + g.blk[q];
                double ub = 0;
                for (int q = 0; q < 7; q++) ub += std::log(g.sum[8 * q]);
                g.upper = ub;
            }
            std::sort(pool.begin(), pool.end(), [](const GP& a, const GP& b) { return a.upper > b.upper; });
            for (int j = 0; j < n; ++j) {
                GP& g = pool[j];
                if (g.selected || g.obs_score < 0) continue;
                if (g.upper < maxDet) break;
                double d = orc::logdet7(g.sum.data());
                if (d > maxDet) {
                    maxDet = d;
                    maxLmk = j;
                }
            }
            if (maxLmk == -1) break;
            for (int q = 0; q < 49; q++) cur[q] = cur[q] + pool[maxLmk].blk[q];
            pool[maxLmk].selected = true;
            out_idx[(*nout)++] = pool[maxLmk].idx;
        }
        return GF_OK;
    }
    const bool deletion = mode == 3 && (size_t)k * 2 > (size_t)n;
    const size_t szLazier = (size_t)((double)n / (double)k * sample_scale);
    std::vector<int> lmkIdx(n);
    std::vector<double> visited(n, -1);
    for (int i = 0; i < n; i++) lmkIdx[i] = i;
    if (!deletion) {  // maxVolSelection_LazierGreedy :2815-3029
        for (size_t i = 0; i < (size_t)k; ++i) {
            int maxLmk = -1;
            double maxDet = -DBL_MAX;
            size_t numHit = 0, numRndQue = 0, szActual = std::min(szLazier, lmkIdx.size());
            while (numHit < szActual) {
                size_t j = 0;
                numRndQue = 0;
                while (numRndQue < 2000) {
                    j = (size_t)(R.next() % (int)lmkIdx.size());
                    if (visited[j] < (double)i) {
                        visited[j] = (double)i;
                        break;
                    }
                    ++numRndQue;
                }
                if (numRndQue >= 2000) break;
                int q = lmkIdx[j];
                ++numHit;
                if (pool[q].selected || pool[q].obs_score < 0) {
                    --numHit;
                    continue;
                }
                double M[49];
                for (int t = 0; t < 49; t++) M[t] = cur[t] + pool[q].blk[t];
                double d = orc::logdet7(M);
                if (d > maxDet) {
                    maxDet = d;
                    maxLmk = q;
                }
            }
            if (maxLmk == -1) break;
            std::vector<int> nl;
            std::vector<double> nv;
            for (size_t j = 0; j < lmkIdx.size(); ++j)
                if (lmkIdx[j] != maxLmk) nl.push_back(lmkIdx[j]), nv.push_back(visited[j]);
            lmkIdx.swap(nl);
            visited.swap(nv);
            for (int t = 0; t < 49; t++) cur[t] = cur[t] + pool[maxLmk].blk[t];
            pool[maxLmk].selected = true;
            out_idx[(*nout)++] = maxLmk;
        }
        return GF_OK;
    }
    // maxVolDeletion_LazierGreedy :2339-2542
    for (int i = 0; i < n; i++) {
        for (int t = 0; t < 49; t++) cur[t] = cur[t] + pool[i].blk[t];
        pool[i].selected = true;
    }
    const size_t mDelLim = (size_t)(n - k);
    for (size_t i = 0; i < mDelLim; ++i) {
        int maxLmk = -1;
        double maxDet = -DBL_MAX;
        size_t numHit = 0, numRndQue = 0, szActual = std::min(szLazier, lmkIdx.size());
        while (numHit < szActual) {
            size_t j = 0;
            numRndQue = 0;
            while (numRndQue < 2000) {
                j = (size_t)(R.next() % (int)lmkIdx.size());
                if (visited[j] < (double)i) {
                    visited[j] = (double)i;
                    break;
                }
                ++numRndQue;
            }
            if (numRndQue >= 2000) break;
            int q = lmkIdx[j];
            ++numHit;
            if (!pool[q].selected || pool[q].obs_score < 0) {
                --numHit;
                continue;
            }
            double M[49];
            for (int t = 0; t < 49; t++) M[t] = cur[t] - pool[q].blk[t];
            double d = orc::logdet7(M);
            if (d > maxDet) {
                maxDet = d;
                maxLmk = q;
            }
        }
        if (maxLmk == -1) break;
        std::vector<int> nl;
        std::vector<double> nv;
        for (size_t j = 0; j < lmkIdx.size(); ++j)
            if (lmkIdx[j] != maxLmk) nl.push_back(lmkIdx[j]), nv.push_back(visited[j]);
        lmkIdx.swap(nl);
        visited.swap(nv);
        for (int t = 0; t < 49; t++) cur[t] = cur[t] - pool[maxLmk].blk[t];
        pool[maxLmk].selected = false;
    }
    for (int i = 0; i < n; i++)
        if (pool[i].selected) out_idx[(*nout)++] = i;
    return GF_OK;
}

// rand() calls made by the last orc_obs_active_match / orc_maxvol_select
int orc_last_rand_calls(void) { return orc::g_rand_calls; }

// logDet evaluations (heap pushes) of the last orc_obs_active_match(_rng)
long long orc_last_ldets(void) { return orc::g_ldets; }

}  // extern "C"
