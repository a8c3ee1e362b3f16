// Constant-velocity PWLS kinematics of the good-feature module (row G1):
// Observability::updatePWLSVec / predictPWLSVec (include/Observability.h:222-295)
// over Util.hpp:302-1005. Shared by the host ABI (gf_host.cpp) and the
// device kernel that keeps the per-frame state update on the GPU (gf.hip).
#pragma once
#include <math.h>
#include <stddef.h>

#if defined(__HIPCC__)
#define GFK_HD __host__ __device__ inline
#else
#define GFK_HD inline
#endif

namespace gfkine {

GFK_HD void gfk_zero(void* p, size_t bytes) {
    unsigned char* c = (unsigned char*)p;
    for (size_t i = 0; i < bytes; i++) c[i] = 0;
}
GFK_HD void gfk_copy(void* d, const void* s, size_t bytes) {
    unsigned char* o = (unsigned char*)d;
    const unsigned char* c = (const unsigned char*)s;
    for (size_t i = 0; i < bytes; i++) o[i] = c[i];
}


GFK_HD void quat_to_R(const double* q, double R[3][3]) {  // Util.hpp:302-316 (q = [r x y z])
    const double x = q[1], y = q[2], z = q[3], r = q[0];
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

GFK_HD double norm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// d(q * q(w dt)) / dw, Util.hpp:440-506
GFK_HD void dq_domega(const double* w, double dt, double out[4][3]) {
    const double wm = norm3(w);
    gfk_zero(out, sizeof(double) * 12);
    if (fabs(wm) < 1e-8) {
        out[1][0] = out[2][1] = out[3][2] = dt / 2;
        return;
    }
    const double c = cos(wm * dt / 2.0), s = sin(wm * dt / 2.0);
    for (int a = 0; a < 3; a++) out[0][a] = (-dt / 2.0) * (w[a] / wm) * s;
    for (int r = 0; r < 3; r++)
        for (int col = 0; col < 3; col++) {
            const double A = w[r];
            if (r == col)
                out[1 + r][col] = (dt / 2.0) * A * A / (wm * wm) * c + (1.0 / wm) * (1.0 - A * A / (wm * wm)) * s;
            else
                out[1 + r][col] = (A * w[col] / (wm * wm)) * ((dt / 2.0) * c - (1.0 / wm) * s);
        }
}

// F blocks of one segment, Util.hpp:787-881
GFK_HD void f_blocks(const double* Xv, double dt, double* FQ /*4x4*/, double* FO /*4x3*/) {
    const double* w = Xv + 10;
    const double* q0 = Xv + 3;
    const double v[3] = {w[0] * dt, w[1] * dt, w[2] * dt};
    const double theta = norm3(v);
    double q[4] = {1, 0, 0, 0};
    if (!(theta < 1e-6)) {
        const double vn[3] = {v[0] / theta, v[1] / theta, v[2] / theta};
        const double nn = norm3(vn), sh = sin(theta / 2.0);
        q[0] = cos(theta / 2.0);
        for (int i = 0; i < 3; i++) q[1 + i] = sh * (vn[i] / nn);
    }
    const double R = q[0], X = q[1], Y = q[2], Z = q[3];
    const double fq[16] = {R, -X, -Y, -Z, X, R, Z, -Y, Y, -Z, R, X, Z, Y, -X, R};
    gfk_copy(FQ, fq, sizeof(fq));
    const double r0 = q0[0], x0 = q0[1], y0 = q0[2], z0 = q0[3];
    const double d31[4][4] = {{r0, -x0, -y0, -z0}, {x0, r0, -z0, y0}, {y0, z0, r0, -x0}, {z0, -y0, x0, r0}};
    double dq[4][3];
    dq_domega(w, dt, dq);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 4; k++) acc += d31[i][k] * dq[k][j];
            FO[3 * i + j] = acc;
        }
}

// convert_PWLS_Vec_To_Homo (Util.hpp:883-905) with QUAT2DCM_float
GFK_HD void state_to_Tcw(const double* Xv, float* T) {
    double Rd[3][3];
    quat_to_R(Xv + 3, Rd);
    float Rwc[3][3], twc[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Rwc[i][j] = (float)Rd[i][j];
    for (int i = 0; i < 3; i++) twc[i] = (float)Xv[i];
    gfk_zero(T, 64);
    T[15] = 1.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = Rwc[j][i];
        const float a = -Rwc[0][i] * twc[0], b = -Rwc[1][i] * twc[1], c = -Rwc[2][i] * twc[2];
        T[4 * i + 3] = (a + b) + c;
    }
}

// propagate_PWLS, Util.hpp:968-1005
GFK_HD void propagate_state(const double* Xv, double dt, double* out) {
    gfk_copy(out, Xv, 13 * sizeof(double));
    for (int i = 0; i < 3; i++) out[i] = Xv[i] + Xv[7 + i] * dt;
    const double wv[3] = {Xv[10] * dt, Xv[11] * dt, Xv[12] * dt};
    double a = norm3(wv), u[3] = {0, 0, 0};
    if (a > 0.0000001) {
        for (int i = 0; i < 3; i++) u[i] = wv[i] / a;
    } else {
        a = 0;
    }
    const double qm[4] = {cos(a / 2), u[0] * sin(a / 2), u[1] * sin(a / 2), u[2] * sin(a / 2)};
    const double* p = Xv + 3;
    const double qp[4] = {p[0] * qm[0] - p[1] * qm[1] - p[2] * qm[2] - p[3] * qm[3],
                          p[0] * qm[1] + p[1] * qm[0] + p[2] * qm[3] - p[3] * qm[2],
                          p[0] * qm[2] - p[1] * qm[3] + p[2] * qm[0] + p[3] * qm[1],
                          p[0] * qm[3] + p[1] * qm[2] - p[2] * qm[1] + p[3] * qm[0]};
    const double nq = sqrt(qp[0] * qp[0] + qp[1] * qp[1] + qp[2] * qp[2] + qp[3] * qp[3]);
    for (int i = 0; i < 4; i++) out[3 + i] = qp[i] / nq;
}

// DCM2QUAT_float (Util.hpp:570-611), float arithmetic, q0 >= 0
GFK_HD void R_to_quat(const float R[3][3], double* q) {
    float qf[4];
    const float tr = R[0][0] + R[1][1] + R[2][2];
    if (tr > 0) {
        const float s = sqrt(tr + 1.0f) * 2;
        qf[0] = 0.25f * s;
        qf[1] = (R[2][1] - R[1][2]) / s;
        qf[2] = (R[0][2] - R[2][0]) / s;
        qf[3] = (R[1][0] - R[0][1]) / s;
    } else if (R[0][0] > R[1][1] && R[0][0] > R[2][2]) {
        const float s = 2.0f * sqrt(1.0f + R[0][0] - R[1][1] - R[2][2]);
        qf[0] = (R[2][1] - R[1][2]) / s;
        qf[1] = 0.25f * s;
        qf[2] = (R[0][1] + R[1][0]) / s;
        qf[3] = (R[0][2] + R[2][0]) / s;
    } else if (R[1][1] > R[2][2]) {
        const float s = 2.0f * sqrt(1.0f + R[1][1] - R[0][0] - R[2][2]);
        qf[0] = (R[0][2] - R[2][0]) / s;
        qf[1] = (R[0][1] + R[1][0]) / s;
        qf[2] = 0.25f * s;
        qf[3] = (R[1][2] + R[2][1]) / s;
    } else {
        const float s = 2.0f * sqrt(1.0f + R[2][2] - R[0][0] - R[1][1]);
        qf[0] = (R[1][0] - R[0][1]) / s;
        qf[1] = (R[0][2] + R[2][0]) / s;
        qf[2] = (R[1][2] + R[2][1]) / s;
        qf[3] = 0.25f * s;
    }
    const double sign = qf[0] < 0 ? -1.0 : 1.0;
    for (int i = 0; i < 4; i++) q[i] = sign * (double)qf[i];
}


GFK_HD void obs_update(double t_prev, const float* Tcw_prev, double t_cur, const float* Twc_cur, double* Xv) {
    gfk_zero(Xv, 13 * sizeof(double));
    for (int i = 0; i < 3; i++) Xv[i] = Twc_cur[4 * i + 3];
    float R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = Twc_cur[4 * i + j];
    R_to_quat(R, Xv + 3);
    // T_rel = (Tcw_prev * Twc_cur)^-1 (rigid inverse, float)
    float P[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = Tcw_prev[4 * i] * Twc_cur[j];
            for (int k = 1; k < 4; k++) s = s + Tcw_prev[4 * i + k] * Twc_cur[4 * k + j];
            P[4 * i + j] = s;
        }
    float Ti[16];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Ti[4 * i + j] = P[4 * j + i];
        const float a = -P[i] * P[3], b = -P[4 + i] * P[7], c = -P[8 + i] * P[11];
        Ti[4 * i + 3] = (a + b) + c;
    }
    const float dt = (float)(t_cur - t_prev);
    for (int i = 0; i < 3; i++) Xv[7 + i] = Ti[4 * i + 3] / dt;
    // get_angular_velocity_with_H (Util.hpp:749-762)
    const float o21 = Ti[9] - Ti[6], o02 = Ti[2] - Ti[8], o10 = Ti[4] - Ti[1];
    Xv[10] = (0.5 * o21) / dt;
    Xv[11] = (0.5 * o02) / dt;
    Xv[12] = (0.5 * o10) / dt;
}

// Frame::getTwc (src/Frame.cc:152-163): Rwc = Rcw^T, twc = -Rwc * tcw (float).
GFK_HD void get_Twc(const float* Tcw, float* Twc) {
    for (int i = 0; i < 16; i++) Twc[i] = (i % 5 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Twc[4 * i + j] = Tcw[4 * j + i];
        const float a = -Tcw[i] * Tcw[3], b = -Tcw[4 + i] * Tcw[7], c = -Tcw[8 + i] * Tcw[11];
        Twc[4 * i + 3] = (a + b) + c;
    }
}

}  // namespace gfkine
