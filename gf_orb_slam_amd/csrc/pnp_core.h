// EPnP RANSAC core of ORB_SLAM::PnPsolver (src/PnPsolver.cc) shared by the
// batched kernels (pnp.hip) and the relocalisation step (reloc.hip): the
// OpenCV SVD / solve restatement, EPnP, CheckInliers and one iterate() call
// split as draw (one thread), hypotheses (one thread each) and the scan (a
// workgroup). See pnp.hip for the design.
#pragma once
#include <algorithm>
#include <cmath>

#include "common.h"
#include "rng.h"

namespace gfpnp {
namespace {

constexpr int kMaxSet = 8;     // minimal-set size bound (the reference uses 4)
constexpr int kWork = 12;      // doubles per correspondence in the refine work buffer

// ----------------------------------------------------------- OpenCV restated
struct CvRng {
    uint64_t state;
    __device__ unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

template <bool V>
__device__ void jacobi_svd(double* At, double* W, double* Vt, int m, int n) {
    const double eps = 2.220446049250313e-16 * 10, minval = 2.2250738585072014e-308;
    double Wd[12];
    const int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * m + k];
            sd += t * t;
        }
        Wd[i] = sd;
        if (V) {
            for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
            Vt[i * n + i] = 1;
        }
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = Wd[i], p = 0, b = Wd[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = sqrt(p * p + beta * beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const double t0 = c * Ai[k] + s * Aj[k];
                    const double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                Wd[i] = a;
                Wd[j] = b;
                changed = true;
                if (V) {
                    double *Vi = Vt + i * n, *Vj = Vt + j * n;
                    for (int k = 0; k < n; k++) {
                        const double t0 = c * Vi[k] + s * Vj[k];
                        const double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const double t = At[i * m + k];
            sd += t * t;
        }
        Wd[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (Wd[j] < Wd[k]) j = k;
        if (i != j) {
            const double tw = Wd[i];
            Wd[i] = Wd[j];
            Wd[j] = tw;
            for (int k = 0; k < m; k++) {
                const double t = At[i * m + k];
                At[i * m + k] = At[j * m + k];
                At[j * m + k] = t;
            }
            if (V)
                for (int k = 0; k < n; k++) {
                    const double t = Vt[i * n + k];
                    Vt[i * n + k] = Vt[j * n + k];
                    Vt[j * n + k] = t;
                }
        }
    }
    for (int i = 0; i < n; i++) W[i] = Wd[i];
    CvRng rng{0x12345678};
    for (int i = 0; i < n; i++) {
        double sd = Wd[i];
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const double val0 = 1. / m;
            for (int k = 0; k < m; k++) At[i * m + k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        const double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) {
                const double t = At[i * m + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

// cv::SVD of r x c (r >= c): w, left vectors as rows (c x r), vt (c x c)
template <bool V>
__device__ void svd(const double* A, int r, int c, double* w, double* urows, double* vt) {
    for (int i = 0; i < c; i++)
        for (int k = 0; k < r; k++) urows[i * r + k] = A[k * c + i];
    jacobi_svd<V>(urows, w, vt, r, c);
}

__device__ void svbksb(int r, int c, const double* w, const double* urows, const double* vt, const double* b,
                       double* x) {
    const int nm = r < c ? r : c, nb = b ? 1 : r;
    for (int i = 0; i < c * nb; i++) x[i] = 0;
    double threshold = 0;
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= 2.220446049250313e-16 * 2;
    for (int i = 0; i < nm; i++) {
        const double* u = urows + i * r;
        const double* v = vt + i * c;
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        if (b) {
            double s = 0;
            for (int j = 0; j < r; j++) s += u[j] * b[j];
            s *= wi;
            for (int j = 0; j < c; j++) x[j] = x[j] + s * v[j];
        } else {
            double buf[3];
            for (int j = 0; j < nb; j++) buf[j] = u[j] * wi;
            for (int rr = 0; rr < c; rr++) {
                const double s = v[rr];
                for (int j = 0; j < nb; j++) x[rr * nb + j] = x[rr * nb + j] + s * buf[j];
            }
        }
    }
}

__device__ void solve_svd(const double* A, int c, const double* b, double* x) {
    double u[6 * 5], w[5], vt[5 * 5];
    svd<true>(A, 6, c, w, u, vt);
    svbksb(6, c, w, u, vt, b, x);
}

// ------------------------------------------------------------------- EPnP
__device__ __forceinline__ double dot3(const double* a, const double* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ double dist2(const double* p1, const double* p2) {
    return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

struct Cam {
    double fu, fv, uc, vc;
};

// Correspondence storage: pws[3n], us[2n], alphas[4n], pcs[3n] (private
// arrays for a minimal set, the global work buffer for a refinement).
struct Pts {
    double *pws, *us, *alphas, *pcs;
    int n;
};

__device__ void choose_control_points(const Pts& P, double cws[4][3]) {
    const int n = P.n;
    cws[0][0] = cws[0][1] = cws[0][2] = 0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) cws[0][j] += P.pws[3 * i + j];
    for (int j = 0; j < 3; j++) cws[0][j] /= n;
    double pw0tpw0[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0;
            for (int i = 0; i < n; i++) s += (P.pws[3 * i + a] - cws[0][a]) * (P.pws[3 * i + b] - cws[0][b]);
            pw0tpw0[a * 3 + b] = s;
        }
    double dc[3], uct[9], vt[9];
    svd<true>(pw0tpw0, 3, 3, dc, uct, vt);
    for (int i = 1; i < 4; i++) {
        const double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
    }
}

__device__ void barycentric(const Pts& P, double cws[4][3]) {
    double cc[9], w[3], u[9], vt[9], ci[9];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
    svd<true>(cc, 3, 3, w, u, vt);
    svbksb(3, 3, w, u, vt, nullptr, ci);
    for (int i = 0; i < P.n; i++) {
        const double* pi = P.pws + 3 * i;
        double* a = P.alphas + 4 * i;
        for (int j = 0; j < 3; j++)
            a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                       ci[3 * j + 2] * (pi[2] - cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
}

__device__ void betas_from(const double* L, const double* rho, int which, double* betas) {
    if (which == 1) {
        double l[24], b4[4];
        for (int i = 0; i < 6; i++) {
            l[i * 4 + 0] = L[i * 10 + 0];
            l[i * 4 + 1] = L[i * 10 + 1];
            l[i * 4 + 2] = L[i * 10 + 3];
            l[i * 4 + 3] = L[i * 10 + 6];
        }
        solve_svd(l, 4, rho, b4);
        if (b4[0] < 0) {
            betas[0] = sqrt(-b4[0]);
            betas[1] = -b4[1] / betas[0];
            betas[2] = -b4[2] / betas[0];
            betas[3] = -b4[3] / betas[0];
        } else {
            betas[0] = sqrt(b4[0]);
            betas[1] = b4[1] / betas[0];
            betas[2] = b4[2] / betas[0];
            betas[3] = b4[3] / betas[0];
        }
    } else {
        const int c = which == 2 ? 3 : 5;
        double l[30], bb[5];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < c; j++) l[i * c + j] = L[i * 10 + j];
        solve_svd(l, c, rho, bb);
        if (bb[0] < 0) {
            betas[0] = sqrt(-bb[0]);
            betas[1] = (bb[2] < 0) ? sqrt(-bb[2]) : 0.0;
        } else {
            betas[0] = sqrt(bb[0]);
            betas[1] = (bb[2] > 0) ? sqrt(bb[2]) : 0.0;
        }
        if (bb[1] < 0) betas[0] = -betas[0];
        betas[2] = which == 2 ? 0.0 : bb[3] / betas[0];
        betas[3] = 0.0;
    }
}

// qr_solve (PnPsolver.cc:832-922) on the 6 x 4 Gauss-Newton system
__device__ void qr_solve(double* A, double* b, double* X) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; k++) {
        double eta = fabs(A[k * nc + k]);
        for (int i = k + 1; i < nr; i++) {
            // the reference compares |A[k][k]| again on the first pass (ppAik not advanced yet)
            const double elt = fabs(A[(i - 1) * nc + k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;
        double sum = 0.0;
        const double inv_eta = 1. / eta;
        for (int i = k; i < nr; i++) {
            A[i * nc + k] *= inv_eta;
            sum += A[i * nc + k] * A[i * nc + k];
        }
        double sigma = sqrt(sum);
        if (A[k * nc + k] < 0) sigma = -sigma;
        A[k * nc + k] += sigma;
        A1[k] = sigma * A[k * nc + k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double s = 0;
            for (int i = k; i < nr; i++) s += A[i * nc + k] * A[i * nc + j];
            const double tau = s / A1[k];
            for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
        }
    }
    for (int j = 0; j < nc; j++) {
        double tau = 0;
        for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double s = 0;
        for (int j = i + 1; j < nc; j++) s += A[i * nc + j] * X[j];
        X[i] = (b[i] - s) / A2[i];
    }
}

__device__ void gauss_newton(const double* L, const double* rho, double betas[4]) {
    for (int it = 0; it < 5; it++) {
        double A[24], b[6], x[4] = {0, 0, 0, 0};
        for (int i = 0; i < 6; i++) {
            const double* r = L + i * 10;
            double* a = A + i * 4;
            a[0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
            a[1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
            a[2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
            a[3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
            b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                             r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                             r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                             r[9] * betas[3] * betas[3]);
        }
        qr_solve(A, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

__device__ double compute_R_and_t(const Pts& P, const Cam& cam, const double* ut, const double* betas,
                                  double R[3][3], double t[3]) {
    double ccs[4][3];
    for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0;
    for (int i = 0; i < 4; i++) {
        const double* v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
    }
    const int n = P.n;
    for (int i = 0; i < n; i++) {
        const double* a = P.alphas + 4 * i;
        double* pc = P.pcs + 3 * i;
        for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
    }
    if (P.pcs[2] < 0.0)
        for (int i = 0; i < n; i++) {
            P.pcs[3 * i] = -P.pcs[3 * i];
            P.pcs[3 * i + 1] = -P.pcs[3 * i + 1];
            P.pcs[3 * i + 2] = -P.pcs[3 * i + 2];
        }
    // estimate_R_and_t :541-599
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) {
            pc0[j] += P.pcs[3 * i + j];
            pw0[j] += P.pws[3 * i + j];
        }
    for (int j = 0; j < 3; j++) {
        pc0[j] /= n;
        pw0[j] /= n;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const double* pc = P.pcs + 3 * i;
        const double* pw = P.pws + 3 * i;
        for (int j = 0; j < 3; j++) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    double d[3], urows[9], vt[9], U[9], Vm[9];
    svd<true>(abt, 3, 3, d, urows, vt);
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) {
            U[i * 3 + k] = urows[k * 3 + i];
            Vm[i * 3 + k] = vt[k * 3 + i];
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = dot3(U + 3 * i, Vm + 3 * j);
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                       R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
        R[2][0] = -R[2][0];
        R[2][1] = -R[2][1];
        R[2][2] = -R[2][2];
    }
    t[0] = pc0[0] - dot3(R[0], pw0);
    t[1] = pc0[1] - dot3(R[1], pw0);
    t[2] = pc0[2] - dot3(R[2], pw0);
    // reprojection_error :522-539
    double sum2 = 0.0;
    for (int i = 0; i < n; i++) {
        const double* pw = P.pws + 3 * i;
        const double Xc = dot3(R[0], pw) + t[0];
        const double Yc = dot3(R[1], pw) + t[1];
        const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
        const double ue = cam.uc + cam.fu * Xc * inv_Zc;
        const double ve = cam.vc + cam.fv * Yc * inv_Zc;
        const double u = P.us[2 * i], v = P.us[2 * i + 1];
        sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / n;
}

__device__ void compute_pose(const Pts& P, const Cam& cam, double R[3][3], double t[3]) {
    double cws[4][3];
    choose_control_points(P, cws);
    barycentric(P, cws);
    const int n = P.n;
    // MtM = M^T M with M's rows (fill_M :408-423) generated in row order
    double ut[144];
    for (int a = 0; a < 12; a++)
        for (int b = a; b < 12; b++) {
            const int ja = a / 3, ca = a % 3, jb = b / 3, cb = b % 3;
            double s = 0;
            for (int i = 0; i < n; i++) {
                const double* as = P.alphas + 4 * i;
                const double u = P.us[2 * i], v = P.us[2 * i + 1];
                const double m1a = ca == 0 ? as[ja] * cam.fu : ca == 1 ? 0.0 : as[ja] * (cam.uc - u);
                const double m1b = cb == 0 ? as[jb] * cam.fu : cb == 1 ? 0.0 : as[jb] * (cam.uc - u);
                const double m2a = ca == 0 ? 0.0 : ca == 1 ? as[ja] * cam.fv : as[ja] * (cam.vc - v);
                const double m2b = cb == 0 ? 0.0 : cb == 1 ? as[jb] * cam.fv : as[jb] * (cam.vc - v);
                s += m1a * m1b;
                s += m2a * m2b;
            }
            ut[b * 12 + a] = ut[a * 12 + b] = s;  // symmetric: At = MtM^T = MtM
        }
    double d[12];
    jacobi_svd<false>(ut, d, nullptr, 12, 12);
    // compute_L_6x10 :732-772 and compute_rho :774-782
    double L[60], rho[6];
    {
        const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
        double dv[4][6][3];
        for (int i = 0; i < 4; i++) {
            int a = 0, b = 1;
            for (int j = 0; j < 6; j++) {
                for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
                b++;
                if (b > 3) {
                    a++;
                    b = a + 1;
                }
            }
        }
        for (int i = 0; i < 6; i++) {
            double* row = L + 10 * i;
            row[0] = dot3(dv[0][i], dv[0][i]);
            row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
            row[2] = dot3(dv[1][i], dv[1][i]);
            row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
            row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
            row[5] = dot3(dv[2][i], dv[2][i]);
            row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
            row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
            row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
            row[9] = dot3(dv[3][i], dv[3][i]);
        }
        rho[0] = dist2(cws[0], cws[1]);
        rho[1] = dist2(cws[0], cws[2]);
        rho[2] = dist2(cws[0], cws[3]);
        rho[3] = dist2(cws[1], cws[2]);
        rho[4] = dist2(cws[1], cws[3]);
        rho[5] = dist2(cws[2], cws[3]);
    }
    double best_err = 0, Rb[3][3], tb[3];
    for (int w = 1; w <= 3; w++) {
        double betas[4], Rw[3][3], tw[3];
        betas_from(L, rho, w, betas);
        gauss_newton(L, rho, betas);
        const double err = compute_R_and_t(P, cam, ut, betas, Rw, tw);
        // N = 1; if e2 < e1: N = 2; if e3 < e[N]: N = 3
        if (w == 1 || err < best_err) {
            best_err = err;
            for (int i = 0; i < 3; i++) {
                for (int j = 0; j < 3; j++) Rb[i][j] = Rw[i][j];
                tb[i] = tw[i];
            }
        }
    }
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R[i][j] = Rb[i][j];
        t[i] = tb[i];
    }
}

// CheckInliers :280-311 for one correspondence
__device__ __forceinline__ bool is_inlier(const float* p3d, const float* p2d, float max_err, const double* Rt,
                                          const Cam& cam) {
    const double x = p3d[0], y = p3d[1], z = p3d[2];
    const float Xc = (float)(Rt[0] * x + Rt[1] * y + Rt[2] * z + Rt[9]);
    const float Yc = (float)(Rt[3] * x + Rt[4] * y + Rt[5] * z + Rt[10]);
    const float invZc = (float)(1 / (Rt[6] * x + Rt[7] * y + Rt[8] * z + Rt[11]));
    const double ue = cam.uc + cam.fu * (double)Xc * (double)invZc;
    const double ve = cam.vc + cam.fv * (double)Yc * (double)invZc;
    const float distX = (float)((double)p2d[0] - ue);
    const float distY = (float)((double)p2d[1] - ve);
    const float error2 = distX * distX + distY * distY;
    return error2 < max_err;
}

// A state from device memory is clamped to what the kernels can hold: the
// minimal set to [1, kMaxSet] (private arrays), n to the problem capacity.
__device__ __forceinline__ gf_pnp_state load_state(const gf_pnp_state* states, int b, int cap) {
    gf_pnp_state st = states[b];
    st.min_set = min(max(st.min_set, 1), kMaxSet);
    st.n = min(max(st.n, 0), cap);
    return st;
}

__device__ __forceinline__ int loop_count(const gf_pnp_state& st, int n_iterations) {
    if (st.n < st.min_inliers) return 0;
    const int a = st.max_iterations - st.iterations;
    const int L = a > n_iterations ? a : n_iterations;
    return L > 0 ? L : 0;
}

__device__ __forceinline__ int random_int(int32_t* s, int32_t* f, int32_t* r, int mn, int mx) {
    const int d = mx - mn + 1;
    return int(((double)gfrng::next(s, f, r) / ((double)2147483647 + 1.0)) * d) + mn;
}

// k_pnp_draw's body for solver b (one thread).
__device__ void pnp_draw_one(const gf_pnp_state* __restrict__ states, const gf_rng* __restrict__ rngs, int b,
                             int n_iterations, int lcap, int32_t* __restrict__ draws, int cap) {
    const gf_pnp_state st = load_state(states, b, cap);
    const int L = min(loop_count(st, n_iterations), lcap);
    int32_t s[31];
    for (int i = 0; i < 31; i++) s[i] = rngs[b].state[i];
    int32_t f = rngs[b].f, r = rngs[b].r;
    int32_t* out = draws + (size_t)b * lcap * kMaxSet;
    const int ms = st.min_set;
    for (int h = 0; h < L; h++) {
        // vAvailableIndices = 0..n-1 with at most ms overwritten slots
        int opos[kMaxSet], oval[kMaxSet], no = 0, size = st.n;
        for (int i = 0; i < ms; i++) {
            const int randi = random_int(s, &f, &r, 0, size - 1);
            int idx = randi;
            for (int o = 0; o < no; o++)
                if (opos[o] == randi) idx = oval[o];
            int back = size - 1;
            for (int o = 0; o < no; o++)
                if (opos[o] == size - 1) back = oval[o];
            out[h * kMaxSet + i] = idx;
            bool found = false;  // avail[idx] = back
            for (int o = 0; o < no; o++)
                if (opos[o] == idx) {
                    oval[o] = back;
                    found = true;
                }
            if (!found) {
                opos[no] = idx;
                oval[no] = back;
                no++;
            }
            size--;
        }
    }
}

// k_pnp_hyp's body for hypothesis h of solver b (one thread).
__device__ void pnp_hyp_one(const float* __restrict__ p3d, const float* __restrict__ p2d,
                            const float* __restrict__ sigma2, int cap, const Cam& cam,
                            const gf_pnp_state* __restrict__ states, int n_iterations, int lcap,
                            const int32_t* __restrict__ draws, double* __restrict__ hyp_rt,
                            int32_t* __restrict__ hyp_cnt, int b, int h) {
    const gf_pnp_state st = load_state(states, b, cap);
    if (h >= min(loop_count(st, n_iterations), lcap)) return;
    const float* P3 = p3d + (size_t)b * cap * 3;
    const float* P2 = p2d + (size_t)b * cap * 2;
    const float* S2 = sigma2 + (size_t)b * cap;
    const int32_t* dr = draws + ((size_t)b * lcap + h) * kMaxSet;
    double pws[3 * kMaxSet], us[2 * kMaxSet], alphas[4 * kMaxSet], pcs[3 * kMaxSet];
    const int ms = st.min_set;
    for (int i = 0; i < ms; i++) {
        const int idx = dr[i];
        pws[3 * i] = P3[3 * idx];
        pws[3 * i + 1] = P3[3 * idx + 1];
        pws[3 * i + 2] = P3[3 * idx + 2];
        us[2 * i] = P2[2 * idx];
        us[2 * i + 1] = P2[2 * idx + 1];
    }
    Pts P{pws, us, alphas, pcs, ms};
    double R[3][3], t[3];
    compute_pose(P, cam, R, t);
    double Rt[12];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Rt[i * 3 + j] = R[i][j];
        Rt[9 + i] = t[i];
    }
    int cnt = 0;
    for (int i = 0; i < st.n; i++) cnt += is_inlier(P3 + 3 * i, P2 + 2 * i, S2[i] * st.th2, Rt, cam);
    double* o = hyp_rt + ((size_t)b * lcap + h) * 12;
    for (int i = 0; i < 12; i++) o[i] = Rt[i];
    hyp_cnt[(size_t)b * lcap + h] = cnt;
}

__device__ void rt_to_Tcw(const double* Rt, float* T) {
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[i * 4 + j] = (float)Rt[i * 3 + j];
        T[i * 4 + 3] = (float)Rt[9 + i];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

// Inlier test of one pose over the solver's correspondences across the
// workgroup: mask to `mask`, returns the count (all threads).
__device__ int block_inliers(const float* P3, const float* P2, const float* S2, int n, float th2, const double* Rt,
                             const Cam& cam, uint8_t* mask, int* red) {
    int c = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const bool in = is_inlier(P3 + 3 * i, P2 + 2 * i, S2[i] * th2, Rt, cam);
        mask[i] = in;
        c += in;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    int tot = 0;
    for (int w = 0; w < (int)((blockDim.x + 63) >> 6); w++) tot += red[w];
    __syncthreads();
    return tot;
}

// k_pnp_scan's body for solver b, by the whole workgroup (<= 256 threads).
__device__ void pnp_scan_block(const float* __restrict__ p3d, const float* __restrict__ p2d,
                               const float* __restrict__ sigma2, int cap, const Cam& cam,
                               gf_pnp_state* __restrict__ states, uint8_t* __restrict__ best_mask,
                               int n_iterations, int lcap, const double* __restrict__ hyp_rt,
                               const int32_t* __restrict__ hyp_cnt, double* __restrict__ work,
                               gf_rng* __restrict__ rngs, float* __restrict__ Tcw_out,
                               uint8_t* __restrict__ inliers, int32_t* __restrict__ ninliers,
                               int32_t* __restrict__ flags, int b) {
    __shared__ int red[4];
    __shared__ double sRt[12];
    __shared__ gf_pnp_state sst;
    if (threadIdx.x == 0) sst = load_state(states, b, cap);
    __syncthreads();
    gf_pnp_state st = sst;  // every wave works from the call's starting state
    const int n = st.n;
    const float* P3 = p3d + (size_t)b * cap * 3;
    const float* P2 = p2d + (size_t)b * cap * 2;
    const float* S2 = sigma2 + (size_t)b * cap;
    uint8_t* bm = best_mask + (size_t)b * cap;
    uint8_t* out_mask = inliers + (size_t)b * cap;
    const int L = min(loop_count(st, n_iterations), lcap);
    const bool truncated = loop_count(st, n_iterations) > lcap;  // max_iterations below the state's loop
    int ran = 0, fl = 0, ninl = 0;
    bool refine_pending = true;  // Refine() of the current best set not yet evaluated in this call
    float T[16];
    for (int h = 0; h < L && !(fl & GF_PNP_FOUND); h++) {
        ran = h + 1;
        const int cnt = hyp_cnt[(size_t)b * lcap + h];
        if (cnt < st.min_inliers) continue;
        const double* Rt = hyp_rt + ((size_t)b * lcap + h) * 12;
        if (cnt > st.best_inliers) {
            block_inliers(P3, P2, S2, n, st.th2, Rt, cam, bm, red);
            st.best_inliers = cnt;
            rt_to_Tcw(Rt, st.best_Tcw);
            refine_pending = true;
        }
        if (!refine_pending) continue;  // the same set refines to the same failure
        refine_pending = false;
        __syncthreads();
        if (threadIdx.x == 0) {
            // gather the best inliers in correspondence order (Refine :234-253)
            double* W = work + (size_t)b * cap * kWork;
            const int K = [&] {
                int k = 0;
                for (int i = 0; i < n; i++)
                    if (bm[i]) {
                        W[3 * k] = P3[3 * i];
                        W[3 * k + 1] = P3[3 * i + 1];
                        W[3 * k + 2] = P3[3 * i + 2];
                        k++;
                    }
                return k;
            }();
            double* us = W + 3 * (size_t)K;
            double* alphas = us + 2 * (size_t)K;
            double* pcs = alphas + 4 * (size_t)K;
            for (int i = 0, k = 0; i < n; i++)
                if (bm[i]) {
                    us[2 * k] = P2[2 * i];
                    us[2 * k + 1] = P2[2 * i + 1];
                    k++;
                }
            Pts P{W, us, alphas, pcs, K};
            double R[3][3], t[3];
            compute_pose(P, cam, R, t);
            for (int i = 0; i < 3; i++) {
                for (int j = 0; j < 3; j++) sRt[i * 3 + j] = R[i][j];
                sRt[9 + i] = t[i];
            }
        }
        __syncthreads();
        const int nref = block_inliers(P3, P2, S2, n, st.th2, sRt, cam, out_mask, red);
        if (nref > st.min_inliers) {
            rt_to_Tcw(sRt, T);
            ninl = nref;
            fl = GF_PNP_FOUND | GF_PNP_REFINED;
        }
    }
    st.iterations += ran;
    if (!(fl & GF_PNP_FOUND)) {
        if (L == 0 && n < st.min_inliers) fl = GF_PNP_NOMORE;
        if (st.iterations >= st.max_iterations) {
            fl = GF_PNP_NOMORE;
            if (st.best_inliers >= st.min_inliers) {
                ninl = st.best_inliers;
                for (int i = threadIdx.x; i < n; i += blockDim.x) out_mask[i] = bm[i];
                for (int i = 0; i < 16; i++) T[i] = st.best_Tcw[i];
                fl |= GF_PNP_FOUND;
            }
        }
        if (!(fl & GF_PNP_FOUND))
            for (int i = threadIdx.x; i < n; i += blockDim.x) out_mask[i] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 0; i < 16; i++) Tcw_out[(size_t)b * 16 + i] = (fl & GF_PNP_FOUND) ? T[i] : 0.f;
        ninliers[b] = ninl;
        flags[b] = truncated ? (fl | GF_PNP_TRUNCATED) : fl;
        states[b] = st;
        gf_rng g = rngs[b];
        for (int i = 0; i < ran * st.min_set; i++) (void)gfrng::next(g.state, &g.f, &g.r);
        rngs[b] = g;
    }
}

}  // namespace
}  // namespace gfpnp
