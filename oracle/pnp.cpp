// CPU ORACLE (test infrastructure) — SURVEY.md §8(f) rank 4: the
// relocalisation solver ORB_SLAM::PnPsolver (src/PnPsolver.cc), EPnP inside
// RANSAC. Restated from the reference text:
//   SetRansacParameters :93-129, iterate :137-230, Refine :232-277,
//   CheckInliers :280-311, EPnP compute_pose :347-497 (control points,
//   barycentric coordinates, M, L_6x10, rho, betas approx 1-3, Gauss-Newton,
//   R|t by the 3x3 SVD, reprojection error), qr_solve :832-922.
// OpenCV is not vendored. Its three calls on this path are
// restated from OpenCV 3.4 (modules/core/src/lapack.cpp): cvSVD / cv::SVD
// (one-sided Jacobi, JacobiSVDImpl_, eps = 10 DBL_EPSILON, minval = DBL_MIN,
// the cv::RNG(0x12345678) completion of null left vectors), cvSolve
// DECOMP_SVD and cvInvert DECOMP_SVD (SVBkSbImpl_, threshold = 2 DBL_EPSILON
// * sum w), all scalar (no SSE2 VBLAS pairing) and hypot(p, beta) taken as
// sqrt(p*p + beta*beta). Parity unpinned against OpenCV itself: the device
// kernel (gf_orb_slam_amd/csrc/pnp.hip) is checked against this restatement
// bit for bit, and this restatement against ground-truth poses.
// DUtils::Random::RandomInt (Thirdparty/DBoW2/DUtils/Random.cpp:47-50) over
// glibc rand(); the reference's draw bookkeeping writes the back element to
// position idx (the drawn VALUE), not randi (:171) — kept.
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "oracle_common.h"

namespace orc_pnp {

// ------------------------------------------------------ OpenCV 3.4 restated
struct CvRng {  // cv::RNG: multiply-with-carry, CV_RNG_COEFF 4164903690
    uint64_t state;
    unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

// JacobiSVDImpl_<double>: At is n rows of length m (the columns of A); on
// return rows 0..n1-1 of At are the left singular vectors, W the singular
// values (descending), Vt the right singular vectors as rows.
static void jacobi_svd(double* At, double* W, double* Vt, int m, int n, int n1) {
    const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
    std::vector<double> Wd(n);
    const int max_iter = std::max(m, 30);
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * m + k];
            sd += t * t;
        }
        Wd[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = Wd[i], p = 0, b = Wd[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = std::sqrt(p * p + beta * beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = std::sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = std::sqrt((gamma + beta) / (gamma * 2));
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
                double *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (int k = 0; k < n; k++) {
                    const double t0 = c * Vi[k] + s * Vj[k];
                    const double t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            double t = At[i * m + k];
            sd += t * t;
        }
        Wd[i] = std::sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {  // selection sort, descending
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (Wd[j] < Wd[k]) j = k;
        if (i != j) {
            std::swap(Wd[i], Wd[j]);
            for (int k = 0; k < m; k++) std::swap(At[i * m + k], At[j * m + k]);
            for (int k = 0; k < n; k++) std::swap(Vt[i * n + k], Vt[j * n + k]);
        }
    }
    for (int i = 0; i < n; i++) W[i] = Wd[i];
    CvRng rng{0x12345678};
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? Wd[i] : 0;
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
                        asum += std::fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) {
                const double t = At[i * m + k];
                sd += t * t;
            }
            sd = std::sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

// cv::SVD::compute of an r x c matrix (r >= c): w (c), u as rows (c x r),
// vt (c x c). Square inputs are symmetric-agnostic: At = A^T.
static void svd(const double* A, int r, int c, double* w, double* urows, double* vt) {
    for (int i = 0; i < c; i++)
        for (int k = 0; k < r; k++) urows[i * r + k] = A[k * c + i];
    jacobi_svd(urows, w, vt, r, c, c);
}

// SVBkSbImpl_ with one right-hand side (b) or the identity (b == NULL, an
// r x r block written to x as c x r).
static void svbksb(int r, int c, const double* w, const double* urows, const double* vt, const double* b,
                   double* x) {
    const int nm = std::min(r, c), nb = b ? 1 : r;
    for (int i = 0; i < c * nb; i++) x[i] = 0;
    double threshold = 0;
    for (int i = 0; i < nm; i++) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int i = 0; i < nm; i++) {
        const double* u = urows + i * r;
        const double* v = vt + i * c;
        double wi = w[i];
        if (std::fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        if (b) {
            double s = 0;
            for (int j = 0; j < r; j++) s += u[j] * b[j];
            s *= wi;
            for (int j = 0; j < c; j++) x[j] = x[j] + s * v[j];
        } else {
            double buf[16];
            for (int j = 0; j < nb; j++) buf[j] = u[j] * wi;
            for (int rr = 0; rr < c; rr++) {
                const double s = v[rr];
                for (int j = 0; j < nb; j++) x[rr * nb + j] = x[rr * nb + j] + s * buf[j];
            }
        }
    }
}

// cvSolve(A (6 x c), b, x, CV_SVD)
static void solve_svd(const double* A, int c, const double* b, double* x) {
    double u[6 * 6], w[6], vt[6 * 6];
    svd(A, 6, c, w, u, vt);
    svbksb(6, c, w, u, vt, b, x);
}

// ------------------------------------------------------------- EPnP
struct EPnP {
    double uc, vc, fu, fv;
    std::vector<double> pws, us, alphas, pcs;
    int number_of_correspondences = 0;
    double cws[4][3], ccs[4][3];

    void reset(int nmax) {
        pws.assign(3 * nmax, 0);
        us.assign(2 * nmax, 0);
        alphas.assign(4 * nmax, 0);
        pcs.assign(3 * nmax, 0);
        number_of_correspondences = 0;
    }
    void add(double X, double Y, double Z, double u, double v) {
        const int i = number_of_correspondences++;
        pws[3 * i] = X;
        pws[3 * i + 1] = Y;
        pws[3 * i + 2] = Z;
        us[2 * i] = u;
        us[2 * i + 1] = v;
    }
    void choose_control_points() {  // :347-381
        const int n = number_of_correspondences;
        cws[0][0] = cws[0][1] = cws[0][2] = 0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
        for (int j = 0; j < 3; j++) cws[0][j] /= n;
        double pw0tpw0[9];  // cvMulTransposed(PW0, ., 1) = PW0^T PW0
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) {
                double s = 0;
                for (int i = 0; i < n; i++) s += (pws[3 * i + a] - cws[0][a]) * (pws[3 * i + b] - cws[0][b]);
                pw0tpw0[a * 3 + b] = s;
            }
        double dc[3], uct[9], vt[9];
        svd(pw0tpw0, 3, 3, dc, uct, vt);
        for (int i = 1; i < 4; i++) {
            const double k = std::sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * uct[3 * (i - 1) + j];
        }
    }
    void compute_barycentric_coordinates() {  // :383-406
        double cc[9], w[3], u[9], vt[9], ci[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svd(cc, 3, 3, w, u, vt);
        svbksb(3, 3, w, u, vt, nullptr, ci);
        for (int i = 0; i < number_of_correspondences; i++) {
            const double* pi = &pws[3 * i];
            double* a = &alphas[4 * i];
            for (int j = 0; j < 3; j++)
                a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                           ci[3 * j + 2] * (pi[2] - cws[0][2]);
            a[0] = 1.0f - a[1] - a[2] - a[3];
        }
    }
    static double dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
    static double dist2(const double* p1, const double* p2) {
        return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) +
               (p1[2] - p2[2]) * (p1[2] - p2[2]);
    }
    void compute_L_6x10(const double* ut, double* l) {  // :732-772
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
            double* row = l + 10 * i;
            row[0] = dot(dv[0][i], dv[0][i]);
            row[1] = 2.0f * dot(dv[0][i], dv[1][i]);
            row[2] = dot(dv[1][i], dv[1][i]);
            row[3] = 2.0f * dot(dv[0][i], dv[2][i]);
            row[4] = 2.0f * dot(dv[1][i], dv[2][i]);
            row[5] = dot(dv[2][i], dv[2][i]);
            row[6] = 2.0f * dot(dv[0][i], dv[3][i]);
            row[7] = 2.0f * dot(dv[1][i], dv[3][i]);
            row[8] = 2.0f * dot(dv[2][i], dv[3][i]);
            row[9] = dot(dv[3][i], dv[3][i]);
        }
    }
    void compute_rho(double* rho) {
        rho[0] = dist2(cws[0], cws[1]);
        rho[1] = dist2(cws[0], cws[2]);
        rho[2] = dist2(cws[0], cws[3]);
        rho[3] = dist2(cws[1], cws[2]);
        rho[4] = dist2(cws[1], cws[3]);
        rho[5] = dist2(cws[2], cws[3]);
    }
    static void find_betas_approx_1(const double* L, const double* rho, double* betas) {
        double l[24], b4[4];
        for (int i = 0; i < 6; i++) {
            l[i * 4 + 0] = L[i * 10 + 0];
            l[i * 4 + 1] = L[i * 10 + 1];
            l[i * 4 + 2] = L[i * 10 + 3];
            l[i * 4 + 3] = L[i * 10 + 6];
        }
        solve_svd(l, 4, rho, b4);
        if (b4[0] < 0) {
            betas[0] = std::sqrt(-b4[0]);
            betas[1] = -b4[1] / betas[0];
            betas[2] = -b4[2] / betas[0];
            betas[3] = -b4[3] / betas[0];
        } else {
            betas[0] = std::sqrt(b4[0]);
            betas[1] = b4[1] / betas[0];
            betas[2] = b4[2] / betas[0];
            betas[3] = b4[3] / betas[0];
        }
    }
    static void find_betas_approx_2(const double* L, const double* rho, double* betas) {
        double l[18], b3[3];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 3; j++) l[i * 3 + j] = L[i * 10 + j];
        solve_svd(l, 3, rho, b3);
        if (b3[0] < 0) {
            betas[0] = std::sqrt(-b3[0]);
            betas[1] = (b3[2] < 0) ? std::sqrt(-b3[2]) : 0.0;
        } else {
            betas[0] = std::sqrt(b3[0]);
            betas[1] = (b3[2] > 0) ? std::sqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) betas[0] = -betas[0];
        betas[2] = 0.0;
        betas[3] = 0.0;
    }
    static void find_betas_approx_3(const double* L, const double* rho, double* betas) {
        double l[30], b5[5];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 5; j++) l[i * 5 + j] = L[i * 10 + j];
        solve_svd(l, 5, rho, b5);
        if (b5[0] < 0) {
            betas[0] = std::sqrt(-b5[0]);
            betas[1] = (b5[2] < 0) ? std::sqrt(-b5[2]) : 0.0;
        } else {
            betas[0] = std::sqrt(b5[0]);
            betas[1] = (b5[2] > 0) ? std::sqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) betas[0] = -betas[0];
        betas[2] = b5[3] / betas[0];
        betas[3] = 0.0;
    }
    static void qr_solve(double* A, double* b, double* X) {  // :832-922, A 6 x 4
        const int nr = 6, nc = 4;
        double A1[6], A2[6];
        double *pA = A, *ppAkk = pA;
        for (int k = 0; k < nc; k++) {
            double *ppAik = ppAkk, eta = std::fabs(*ppAik);
            for (int i = k + 1; i < nr; i++) {
                const double elt = std::fabs(*ppAik);
                if (eta < elt) eta = elt;
                ppAik += nc;
            }
            if (eta == 0) {  // "A is singular": the reference returns leaving X as it was
                A1[k] = A2[k] = 0.0;
                return;
            }
            double sum = 0.0, inv_eta = 1. / eta;
            ppAik = ppAkk;
            for (int i = k; i < nr; i++) {
                *ppAik *= inv_eta;
                sum += *ppAik * *ppAik;
                ppAik += nc;
            }
            double sigma = std::sqrt(sum);
            if (*ppAkk < 0) sigma = -sigma;
            *ppAkk += sigma;
            A1[k] = sigma * *ppAkk;
            A2[k] = -eta * sigma;
            for (int j = k + 1; j < nc; j++) {
                double* pp = ppAkk;
                double s = 0;
                for (int i = k; i < nr; i++) {
                    s += *pp * pp[j - k];
                    pp += nc;
                }
                const double tau = s / A1[k];
                pp = ppAkk;
                for (int i = k; i < nr; i++) {
                    pp[j - k] -= tau * *pp;
                    pp += nc;
                }
            }
            ppAkk += nc + 1;
        }
        double *ppAjj = pA, *pb = b;
        for (int j = 0; j < nc; j++) {
            double *ppAij = ppAjj, tau = 0;
            for (int i = j; i < nr; i++) {
                tau += *ppAij * pb[i];
                ppAij += nc;
            }
            tau /= A1[j];
            ppAij = ppAjj;
            for (int i = j; i < nr; i++) {
                pb[i] -= tau * *ppAij;
                ppAij += nc;
            }
            ppAjj += nc + 1;
        }
        X[nc - 1] = pb[nc - 1] / A2[nc - 1];
        for (int i = nc - 2; i >= 0; i--) {
            double *ppAij = pA + i * nc + (i + 1), s = 0;
            for (int j = i + 1; j < nc; j++) {
                s += *ppAij * X[j];
                ppAij++;
            }
            X[i] = (pb[i] - s) / A2[i];
        }
    }
    static void gauss_newton(const double* L, const double* rho, double betas[4]) {  // :784-830
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
    double reprojection_error(const double R[3][3], const double t[3]) {  // :522-539
        double sum2 = 0.0;
        for (int i = 0; i < number_of_correspondences; i++) {
            const double* pw = &pws[3 * i];
            const double Xc = dot(R[0], pw) + t[0];
            const double Yc = dot(R[1], pw) + t[1];
            const double inv_Zc = 1.0 / (dot(R[2], pw) + t[2]);
            const double ue = uc + fu * Xc * inv_Zc;
            const double ve = vc + fv * Yc * inv_Zc;
            const double u = us[2 * i], v = us[2 * i + 1];
            sum2 += std::sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
        return sum2 / number_of_correspondences;
    }
    void estimate_R_and_t(double R[3][3], double t[3]) {  // :541-599
        const int n = number_of_correspondences;
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs[3 * i + j];
                pw0[j] += pws[3 * i + j];
            }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= n;
            pw0[j] /= n;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; i++) {
            const double* pc = &pcs[3 * i];
            const double* pw = &pws[3 * i];
            for (int j = 0; j < 3; j++) {
                abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
        double d[3], urows[9], vt[9];
        svd(abt, 3, 3, d, urows, vt);
        // abt_u = U (columns = left vectors), abt_v = V: R = U V^T
        double U[9], V[9];
        for (int i = 0; i < 3; i++)
            for (int k = 0; k < 3; k++) {
                U[i * 3 + k] = urows[k * 3 + i];
                V[i * 3 + k] = vt[k * 3 + i];
            }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = dot(U + 3 * i, V + 3 * j);
        const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                           R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
        if (det < 0) {
            R[2][0] = -R[2][0];
            R[2][1] = -R[2][1];
            R[2][2] = -R[2][2];
        }
        t[0] = pc0[0] - dot(R[0], pw0);
        t[1] = pc0[1] - dot(R[1], pw0);
        t[2] = pc0[2] - dot(R[2], pw0);
    }
    double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {  // :623-634
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
        }
        for (int i = 0; i < number_of_correspondences; i++) {
            const double* a = &alphas[4 * i];
            double* pc = &pcs[3 * i];
            for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        if (pcs[2] < 0.0) {  // solve_for_sign :608-621
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
            for (int i = 0; i < number_of_correspondences; i++) {
                pcs[3 * i] = -pcs[3 * i];
                pcs[3 * i + 1] = -pcs[3 * i + 1];
                pcs[3 * i + 2] = -pcs[3 * i + 2];
            }
        }
        estimate_R_and_t(R, t);
        return reprojection_error(R, t);
    }
    double compute_pose(double R[3][3], double t[3]) {  // :449-497
        choose_control_points();
        compute_barycentric_coordinates();
        const int n = number_of_correspondences;
        // M (2n x 12) by fill_M :408-423, MtM = M^T M (cvMulTransposed, order 1)
        std::vector<double> M(24 * (size_t)n);
        for (int i = 0; i < n; i++) {
            const double* as = &alphas[4 * i];
            const double u = us[2 * i], v = us[2 * i + 1];
            double* M1 = &M[(size_t)2 * i * 12];
            double* M2 = M1 + 12;
            for (int j = 0; j < 4; j++) {
                M1[3 * j] = as[j] * fu;
                M1[3 * j + 1] = 0.0;
                M1[3 * j + 2] = as[j] * (uc - u);
                M2[3 * j] = 0.0;
                M2[3 * j + 1] = as[j] * fv;
                M2[3 * j + 2] = as[j] * (vc - v);
            }
        }
        double mtm[144];
        for (int a = 0; a < 12; a++)
            for (int b = a; b < 12; b++) {
                double s = 0;
                for (int r = 0; r < 2 * n; r++) s += M[(size_t)r * 12 + a] * M[(size_t)r * 12 + b];
                mtm[a * 12 + b] = mtm[b * 12 + a] = s;
            }
        double d[12], ut[144], vt[144];
        svd(mtm, 12, 12, d, ut, vt);
        double l_6x10[60], rho[6];
        compute_L_6x10(ut, l_6x10);
        compute_rho(rho);
        double Betas[4][4], rep_errors[4], Rs[4][3][3], ts[4][3];
        find_betas_approx_1(l_6x10, rho, Betas[1]);
        gauss_newton(l_6x10, rho, Betas[1]);
        rep_errors[1] = compute_R_and_t(ut, Betas[1], Rs[1], ts[1]);
        find_betas_approx_2(l_6x10, rho, Betas[2]);
        gauss_newton(l_6x10, rho, Betas[2]);
        rep_errors[2] = compute_R_and_t(ut, Betas[2], Rs[2], ts[2]);
        find_betas_approx_3(l_6x10, rho, Betas[3]);
        gauss_newton(l_6x10, rho, Betas[3]);
        rep_errors[3] = compute_R_and_t(ut, Betas[3], Rs[3], ts[3]);
        int N = 1;
        if (rep_errors[2] < rep_errors[1]) N = 2;
        if (rep_errors[3] < rep_errors[N]) N = 3;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R[i][j] = Rs[N][i][j];
            t[i] = ts[N][i];
        }
        return rep_errors[N];
    }
};

// CheckInliers :280-311 (float / double mix as in the reference)
static int check_inliers(const float* p3d, const float* p2d, const float* max_err, int n, const double R[3][3],
                         const double t[3], double uc, double vc, double fu, double fv, uint8_t* mask) {
    int cnt = 0;
    for (int i = 0; i < n; i++) {
        const float x = p3d[3 * i], y = p3d[3 * i + 1], z = p3d[3 * i + 2];
        const float Xc = R[0][0] * x + R[0][1] * y + R[0][2] * z + t[0];
        const float Yc = R[1][0] * x + R[1][1] * y + R[1][2] * z + t[1];
        const float invZc = 1 / (R[2][0] * x + R[2][1] * y + R[2][2] * z + t[2]);
        const double ue = uc + fu * Xc * invZc;
        const double ve = vc + fv * Yc * invZc;
        const float distX = p2d[2 * i] - ue;
        const float distY = p2d[2 * i + 1] - ve;
        const float error2 = distX * distX + distY * distY;
        mask[i] = error2 < max_err[i];
        cnt += mask[i];
    }
    return cnt;
}

static void to_Tcw(const double R[3][3], const double t[3], float* T) {
    for (int i = 0; i < 16; i++) T[i] = 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[i * 4 + j] = (float)R[i][j];
        T[i * 4 + 3] = (float)t[i];
    }
    T[15] = 1.f;
}

struct Rand {  // glibc random_r TYPE_3: the process-wide std::rand()
    struct random_data rd;
    char state[128];
    void seed(unsigned s) {
        std::memset(&rd, 0, sizeof(rd));
        std::memset(state, 0, sizeof(state));
        initstate_r(s, state, sizeof(state), &rd);
    }
    void load(const gf_rng& g) {  // a saved std::rand() state (gf_rng)
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
        return r;
    }
    int random_int(int mn, int mx) {  // DUtils::Random::RandomInt
        const int d = mx - mn + 1;
        return int(((double)next() / ((double)RAND_MAX + 1.0)) * d) + mn;
    }
};

}  // namespace orc_pnp

extern "C" {

// PnPsolver::SetRansacParameters :93-129 (the host set-up the library also does)
int orc_pnp_init(int n, const gf_pnp_params* p, gf_pnp_state* st) {
    std::memset(st, 0, sizeof(*st));
    st->n = n;
    st->min_set = p->min_set;
    st->th2 = p->th2;
    float eps = p->epsilon;
    int nMinInliers = n * eps;
    if (nMinInliers < p->min_inliers) nMinInliers = p->min_inliers;
    if (nMinInliers < p->min_set) nMinInliers = p->min_set;
    if (n > 0 && eps < (float)nMinInliers / n) eps = (float)nMinInliers / n;
    int nIterations;
    if (nMinInliers == n)
        nIterations = 1;
    else {
        const double it = std::ceil(std::log(1 - p->probability) / std::log(1 - std::pow(eps, 3)));
        nIterations = (it == it && it < 2147483647.0) ? (int)it : p->max_iterations;
    }
    st->min_inliers = nMinInliers;
    st->epsilon = eps;
    st->max_iterations = std::max(1, std::min(nIterations, p->max_iterations));
    return GF_OK;
}

}  // extern "C"

namespace orc_pnp {

// One PnPsolver::iterate(n_iter, bNoMore, vbInliers, nInliers) call (:137-230)
// on a solver state; draws from R (DUtils::Random::RandomInt over std::rand()),
// *calls counts them. Outputs T (zeros unless found), inl (n), ninl, flags.
static void iterate_call(const float* p3d, const float* p2d, const float* sigma2, int n, const float K[4],
                         gf_pnp_state& st, uint8_t* best_mask, int n_iter, Rand& R, int* calls, float* T,
                         uint8_t* inl, int32_t* ninliers, int32_t* flags) {
    const double fu = K[0], fv = K[1], uc = K[2], vc = K[3];
    std::vector<float> max_err(n);
    for (int i = 0; i < n; i++) max_err[i] = sigma2[i] * st.th2;  // :126-128
    std::vector<uint8_t> best(best_mask, best_mask + n), cur(n, 0), refined(n, 0);
    std::vector<int> avail(std::max(n, 1));
    EPnP E;
    E.fu = fu;
    E.fv = fv;
    E.uc = uc;
    E.vc = vc;
    for (int i = 0; i < 16; i++) T[i] = 0.f;
    for (int i = 0; i < n; i++) inl[i] = 0;
    int fl = 0, ninl = 0;
    if (n < st.min_inliers) {  // :145-149
        *flags = GF_PNP_NOMORE;
        *ninliers = 0;
        return;
    }
    int cur_it = 0;
    bool done = false;
    while (st.iterations < st.max_iterations || cur_it < n_iter) {
        cur_it++;
        st.iterations++;
        E.reset(st.min_set);
        for (int i = 0; i < n; i++) avail[i] = i;  // vAvailableIndices = mvAllIndices
        int size = n;
        for (int i = 0; i < st.min_set; i++) {
            const int randi = R.random_int(0, size - 1);
            (*calls)++;
            const int idx = avail[randi];
            E.add(p3d[3 * idx], p3d[3 * idx + 1], p3d[3 * idx + 2], p2d[2 * idx], p2d[2 * idx + 1]);
            avail[idx] = avail[size - 1];  // :171, index idx as the reference writes it
            size--;
        }
        double Ri[3][3], ti[3];
        E.compute_pose(Ri, ti);
        const int inl_i = check_inliers(p3d, p2d, max_err.data(), n, Ri, ti, uc, vc, fu, fv, cur.data());
        if (inl_i >= st.min_inliers) {
            if (inl_i > st.best_inliers) {
                best = cur;
                st.best_inliers = inl_i;
                to_Tcw(Ri, ti, st.best_Tcw);
            }
            // Refine :232-277
            int K2 = 0;
            for (int i = 0; i < n; i++) K2 += best[i];
            E.reset(K2);
            for (int i = 0; i < n; i++)
                if (best[i]) E.add(p3d[3 * i], p3d[3 * i + 1], p3d[3 * i + 2], p2d[2 * i], p2d[2 * i + 1]);
            double Rr[3][3], tr[3];
            E.compute_pose(Rr, tr);
            const int nref = check_inliers(p3d, p2d, max_err.data(), n, Rr, tr, uc, vc, fu, fv, refined.data());
            if (nref > st.min_inliers) {
                to_Tcw(Rr, tr, T);
                for (int i = 0; i < n; i++) inl[i] = refined[i];
                ninl = nref;
                fl = GF_PNP_FOUND | GF_PNP_REFINED;
                done = true;
                break;
            }
        }
    }
    if (!done && st.iterations >= st.max_iterations) {  // :213-227
        fl = GF_PNP_NOMORE;
        if (st.best_inliers >= st.min_inliers) {
            ninl = st.best_inliers;
            for (int i = 0; i < n; i++) inl[i] = best[i];
            for (int i = 0; i < 16; i++) T[i] = st.best_Tcw[i];
            fl |= GF_PNP_FOUND;
        }
    }
    std::memcpy(best_mask, best.data(), (size_t)n);
    *flags = fl;
    *ninliers = ninl;
}

}  // namespace orc_pnp

extern "C" {

// A sequence of iterate() calls on one solver of n correspondences with
// std::srand(seed) before the first: call c runs n_iter[c] iterations; its
// outputs land at Tcw[c*16], inliers[c*n], ninliers[c], flags[c];
// rand_calls[c] = std::rand() calls made so far.
int orc_pnp_run(const float* p3d, const float* p2d, const float* sigma2, int n, const float K[4],
                const gf_pnp_params* p, unsigned seed, int ncalls, const int32_t* n_iter, float* Tcw, uint8_t* inliers,
                int32_t* ninliers, int32_t* flags, int32_t* rand_calls) {
    using namespace orc_pnp;
    gf_pnp_state st;
    orc_pnp_init(n, p, &st);
    Rand R;
    R.seed(seed);
    int calls = 0;
    std::vector<uint8_t> best(std::max(n, 1), 0);
    for (int c = 0; c < ncalls; c++) {
        iterate_call(p3d, p2d, sigma2, n, K, st, best.data(), n_iter[c], R, &calls, Tcw + 16 * c,
                     inliers + (size_t)n * c, &ninliers[c], &flags[c]);
        rand_calls[c] = calls;
    }
    return GF_OK;
}

// One iterate() call on a saved solver state (gf_pnp_iterate's contract):
// rng is the std::rand() state (advanced by the draws made), best_mask
// (mvbBestInliers) persists with the state.
int orc_pnp_iterate(const float* p3d, const float* p2d, const float* sigma2, const float K[4], gf_pnp_state* st,
                    uint8_t* best_mask, int n_iterations, gf_rng* rng, float* Tcw, uint8_t* inliers, int32_t* ninliers,
                    int32_t* flags) {
    using namespace orc_pnp;
    Rand R;
    R.load(*rng);
    int calls = 0;
    iterate_call(p3d, p2d, sigma2, st->n, K, *st, best_mask, n_iterations, R, &calls, Tcw, inliers, ninliers, flags);
    R.save(*rng);
    return GF_OK;
}

}  // extern "C"
