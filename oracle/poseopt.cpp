// CPU ORACLE (test infrastructure) — pose optimisation rows P1-P4 of
// Optimizer::PoseOptimization (src/Optimizer.cc:279-413) on the
// vendored g2o arithmetic it runs: OptimizationAlgorithmLevenberg::solve
// (core/optimization_algorithm_levenberg.cpp:61-189), BaseBinaryEdge
// constructQuadraticForm (core/base_binary_edge.hpp:55-122) with the Huber
// kernel (core/robust_kernel_impl.cpp:78-88), EdgeSE3ProjectXYZ
// (types/sba/types_six_dof_expmap.cpp:384-428), SE3Quat::exp / map
// (types/slam3d/se3quat.h), Converter::toSE3Quat / toCvMat, and Eigen's
// LDLT (diagonal pivoting) for LinearSolverDense. Sums run in edge order.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "g2o_se3.h"
#include "oracle_common.h"

namespace orc {

// Eigen::LDLT<MatrixXd> (diagonal pivoting) solve of H x = b, n = 6.
// Returns false when the factorisation is not positive (isPositive()).
bool ldlt_solve(const double* Hin, const double* b, double* x, int n) {
    double A[36];
    std::memcpy(A, Hin, sizeof(double) * n * n);
    int perm[6];
    bool found_zero = false, ok = true;
    int sign = 0;  // 0 zero, 1 psd, 2 nsd, 3 indefinite
    double temp[6];
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = std::fabs(A[k * n + k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(A[i * n + i]) > bv) bv = std::fabs(A[i * n + i]), big = i;
        perm[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(A[k * n + j], A[big * n + j]);
            for (int i = big + 1; i < n; i++) std::swap(A[i * n + k], A[i * n + big]);
            std::swap(A[k * n + k], A[big * n + big]);
            for (int i = k + 1; i < big; i++) {
                double t = A[i * n + k];
                A[i * n + k] = A[big * n + i];
                A[big * n + i] = t;
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
        const bool valid = std::fabs(akk) > 0;
        if (k == 0 && !valid) {
            sign = 0;
            ok = false;
            for (int j = 0; j < n; j++) perm[j] = j;
            break;
        }
        if (valid)
            for (int i = k + 1; i < n; i++) A[i * n + k] /= akk;
        if (found_zero && valid)
            ok = false;
        else if (!valid)
            found_zero = true;
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
    (void)ok;
    if (!(sign == 1 || sign == 0)) return false;
    // x = P b
    for (int i = 0; i < n; i++) x[i] = b[i];
    for (int k = 0; k < n; k++) std::swap(x[k], x[perm[k]]);
    for (int j = 0; j < n; j++)  // L^-1 (unit lower, column axpy order)
        for (int i = j + 1; i < n; i++) x[i] -= A[i * n + j] * x[j];
    const double tol = DBL_MIN;  // numeric_limits<double>::min()
    for (int i = 0; i < n; i++) x[i] = std::fabs(A[i * n + i]) > tol ? x[i] / A[i * n + i] : 0.0;
    for (int i = n - 1; i >= 0; i--) {  // L^-T
        double s = 0;
        for (int k = i + 1; k < n; k++) s += A[k * n + i] * x[k];
        x[i] -= s;
    }
    for (int k = n - 1; k >= 0; k--) std::swap(x[k], x[perm[k]]);
    return true;
}

struct Edge {
    double X[3], z[2], info, delta;
    double err[2];
};

struct PoseProblem {
    std::vector<Edge> e;
    double fx, fy, cx, cy;
    SE3 T;
    // Solver::_x persists across optimize() calls and keeps its last value when
    // the LDLT is not positive (g2o leaves it uninitialised; zero here).
    double x[6] = {0, 0, 0, 0, 0, 0};

    void compute_error(Edge& g, const SE3& P) const {
        double pc[3];
        P.map(g.X, pc);
        const double px = pc[0] / pc[2], py = pc[1] / pc[2];
        g.err[0] = g.z[0] - (px * fx + cx);
        g.err[1] = g.z[1] - (py * fy + cy);
    }
    static double chi2(const Edge& g) { return g.err[0] * (g.info * g.err[0]) + g.err[1] * (g.info * g.err[1]); }
    static void robustify(const Edge& g, double e, double* rho) {
        const double dsqr = g.delta * g.delta;
        if (e <= dsqr) {
            rho[0] = e;
            rho[1] = 1.;
        } else {
            const double s = std::sqrt(e);
            rho[0] = 2 * s * g.delta - dsqr;
            rho[1] = g.delta / s;
        }
    }
    double robust_chi2_all(const SE3& P) {
        double chi = 0;
        for (auto& g : e) {
            compute_error(g, P);
            double rho[2];
            robustify(g, chi2(g), rho);
            chi += rho[0];
        }
        return chi;
    }
    void build(double* H, double* b) {
        std::memset(H, 0, 36 * sizeof(double));
        std::memset(b, 0, 6 * sizeof(double));
        for (auto& g : e) {
            double pc[3];
            T.map(g.X, pc);
            const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
            double J[2][6];
            J[0][0] = x * y / z2 * fx;
            J[0][1] = -(1 + (x * x / z2)) * fx;
            J[0][2] = y / z * fx;
            J[0][3] = -1. / z * fx;
            J[0][4] = 0;
            J[0][5] = x / z2 * fx;
            J[1][0] = (1 + y * y / z2) * fy;
            J[1][1] = -x * y / z2 * fy;
            J[1][2] = -x / z * fy;
            J[1][3] = 0;
            J[1][4] = -1. / z * fy;
            J[1][5] = y / z2 * fy;
            double rho[2];
            robustify(g, chi2(g), rho);
            const double w = rho[1] * g.info;
            const double orr[2] = {-(g.info * g.err[0]) * rho[1], -(g.info * g.err[1]) * rho[1]};
            for (int i = 0; i < 6; i++) {
                b[i] += J[0][i] * orr[0] + J[1][i] * orr[1];
                for (int j = 0; j < 6; j++) H[6 * i + j] += (J[0][i] * w) * J[0][j] + (J[1][i] * w) * J[1][j];
            }
        }
    }

    // SparseOptimizer::optimize(iters) with OptimizationAlgorithmLevenberg.
    int optimize(int iterations) {
        double lambda = 0, ni = 2;
        int nBad = 0, it_done = 0;
        for (int iter = 0; iter < iterations; iter++) {
            it_done++;
            double currentChi = robust_chi2_all(T);
            double iniChi = currentChi;
            double H[36], b[6];
            build(H, b);
            if (iter == 0) {
                double md = 0;
                for (int j = 0; j < 6; j++) md = std::max(std::fabs(H[7 * j]), md);
                lambda = 1e-5 * md;
                ni = 2;
                nBad = 0;
            }
            double rho = 0;
            int q = 0;
            do {
                double Hl[36];
                std::memcpy(Hl, H, sizeof(H));
                for (int j = 0; j < 6; j++) Hl[7 * j] += lambda;
                double xs[6];
                bool ok = ldlt_solve(Hl, b, xs, 6);
                if (ok) std::memcpy(x, xs, sizeof(x));
                SE3 trial = se3_mul(se3_exp(x), T);
                double tempChi = robust_chi2_all(trial);
                if (!ok) tempChi = DBL_MAX;
                rho = currentChi - tempChi;
                double scale = 0;
                for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
                scale += 1e-3;
                rho /= scale;
                if (rho > 0 && std::isfinite(tempChi)) {
                    double alpha = 1. - std::pow((2 * rho - 1), 3);
                    alpha = std::min(alpha, 2. / 3.);
                    double sf = std::max(1. / 3., alpha);
                    lambda *= sf;
                    ni = 2;
                    currentChi = tempChi;
                    T = trial;
                } else {
                    lambda *= ni;
                    ni *= 2;
                    // estimate restored; edge errors keep the trial values (g2o pops only the state)
                }
                q++;
            } while (rho < 0 && q < 10);
            if (q == 10 || rho == 0) break;
            if ((iniChi - currentChi) * 1e3 < iniChi)
                nBad++;
            else
                nBad = 0;
            if (nBad >= 3) break;
        }
        return it_done;
    }
};

}  // namespace orc

extern "C" {

// Optimizer::PoseOptimization for one frame. Edges in keypoint order: X (MP
// world position, float as cv::Mat), z (keypoint), octave; inv_sigma2 per level.
int orc_pose_opt(const float* Tcw_in, const float* X, const float* z, const int32_t* octave,
                 const float* inv_sigma2_levels, int n, float fx, float fy, float cx, float cy, float* Tcw_out,
                 uint8_t* outlier, int* ninliers, int* iterations) {
    orc::PoseProblem P;
    P.fx = fx;
    P.fy = fy;
    P.cx = cx;
    P.cy = cy;
    P.T = orc::se3_from_Tcw(Tcw_in);
    const float delta = std::sqrt(5.991);
    std::vector<float> invs(n);
    for (int i = 0; i < n; i++) {
        orc::Edge g;
        for (int k = 0; k < 3; k++) g.X[k] = X[3 * i + k];
        g.z[0] = z[2 * i];
        g.z[1] = z[2 * i + 1];
        invs[i] = inv_sigma2_levels[octave[i]];
        g.info = invs[i];
        g.delta = delta;
        g.err[0] = g.err[1] = 0;
        P.e.push_back(g);
        outlier[i] = 0;
    }
    const float chi2t[4] = {9.210f, 7.378f, 5.991f, 5.991f};
    const int its[4] = {10, 10, 7, 5};
    int nBad = 0, total_it = 0;
    for (int it = 0; it < 4 && n > 0; it++) {  // empty graph: optimize() returns -1, nothing moves
        total_it += P.optimize(its[it]);
        nBad = 0;
        for (int i = 0; i < n; i++) {
            orc::Edge& g = P.e[i];
            if (outlier[i]) {
                g.info = invs[i];
                P.compute_error(g, P.T);
            }
            const double c2 = orc::PoseProblem::chi2(g);
            if (c2 > chi2t[it]) {
                outlier[i] = 1;
                g.info = 1e-10;
                nBad++;
            } else if (c2 <= chi2t[it]) {
                outlier[i] = 0;
            }
        }
        if (n < 10) break;
    }
    orc::se3_to_Tcw(P.T, Tcw_out);
    *ninliers = n - nBad;
    if (iterations) *iterations = total_it;
    return GF_OK;
}

int orc_ldlt_solve(const double* H, const double* b, double* x) { return orc::ldlt_solve(H, b, x, 6) ? 1 : 0; }

}  // extern "C"
