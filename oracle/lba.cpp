// CPU ORACLE (test infrastructure) — row B1 of SURVEY.md §8a:
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:1515-1764) on the g2o
// machinery it configures (vendored, Thirdparty/g2o/g2o):
//   SparseOptimizer::initializeOptimization / buildIndexMapping /
//     computeActiveErrors / activeRobustChi2 / update
//     (core/sparse_optimizer.cpp:61-114, 166-267, 354-435);
//   OptimizationAlgorithmLevenberg::solve / computeLambdaInit / computeScale
//     (core/optimization_algorithm_levenberg.cpp:61-189);
//   BlockSolver::buildSystem / setLambda / solve with the Schur complement
//     (core/block_solver.hpp:354-486, 502-589; sparse_block_matrix_ccs.h:103-130);
//   BaseBinaryEdge::constructQuadraticForm, robust branch
//     (core/base_binary_edge.hpp:91-114), RobustKernelHuber
//     (core/robust_kernel_impl.cpp:78-88);
//   EdgeSE3ProjectXYZ::computeError / linearizeOplus
//     (types/sba/types_six_dof_expmap.h:162-191, .cpp:384-420);
//   VertexSE3Expmap::oplus (exp(u) * T), VertexSBAPointXYZ::oplus (X + u);
//   Eigen's 3x3 inverse (cofactors of column 0, then the helper) for Dinv.
//
// Parity unpinned for the linear solve: the reference factors the reduced
// camera system with CHOLMOD (solvers/cholmod/linear_solver_cholmod.h:115-154,
// AMD ordering; CHOLMOD is not vendored). This restatement
// factors the same matrix with a dense LL^T in natural order (divisions by
// L_jj as products with its reciprocal; forward substitution with ascending,
// back substitution with descending sums) and
// treats a non-positive pivot as CHOLMOD_NOT_POSDEF (solve() returns false,
// Solver::_x keeps its previous value). Solver::_x is zeroed whenever the
// structure is rebuilt (g2o leaves it uninitialised). Every other sum runs in
// g2o's order: edges in insertion order, landmarks in vertex order, the
// blocks of a landmark column in pose order.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "g2o_se3.h"
#include "oracle_common.h"

namespace orc {
namespace {

struct BAEdge {
    int pt, kf;
    double z[2], info, fx, fy, cx, cy;
    double err[2];
    bool active;
};

inline void huber(double e, double delta, double* rho) {  // RobustKernelHuber::robustify
    const double dsqr = delta * delta;
    if (e <= dsqr) {
        rho[0] = e;
        rho[1] = 1.;
    } else {
        const double s = std::sqrt(e);
        rho[0] = 2 * s * delta - dsqr;
        rho[1] = delta / s;
    }
}

// Eigen compute_inverse<Matrix3d>: cofactors of column 0, det, then the rest.
inline void inverse3(const double* m, double* r) {
#define M_(i, j) m[3 * (i) + (j)]
    const double c0 = M_(1, 1) * M_(2, 2) - M_(1, 2) * M_(2, 1);
    const double c1 = M_(2, 1) * M_(0, 2) - M_(2, 2) * M_(0, 1);
    const double c2 = M_(0, 1) * M_(1, 2) - M_(0, 2) * M_(1, 1);
    const double det = (c0 * M_(0, 0) + c1 * M_(1, 0)) + c2 * M_(2, 0);
    const double inv = 1.0 / det;
    r[0] = c0 * inv;
    r[1] = c1 * inv;
    r[2] = c2 * inv;
    r[3] = (M_(1, 2) * M_(2, 0) - M_(1, 0) * M_(2, 2)) * inv;
    r[4] = (M_(2, 2) * M_(0, 0) - M_(2, 0) * M_(0, 2)) * inv;
    r[5] = (M_(0, 2) * M_(1, 0) - M_(0, 0) * M_(1, 2)) * inv;
    r[6] = (M_(1, 0) * M_(2, 1) - M_(1, 1) * M_(2, 0)) * inv;
    r[7] = (M_(2, 0) * M_(0, 1) - M_(2, 1) * M_(0, 0)) * inv;
    r[8] = (M_(0, 0) * M_(1, 1) - M_(0, 1) * M_(1, 0)) * inv;
#undef M_
}

struct LBA {
    std::vector<SE3> T;         // keyframe poses, vertex order
    std::vector<uint8_t> kind;  // 0 local, 1 local fixed, 2 fixed camera
    std::vector<double> X;      // 3 per point, vertex order
    std::vector<BAEdge> E;      // insertion order
    double delta = 0;
    // index mapping of the last initializeOptimization()
    std::vector<int> pose_col, pose_kf, lm_of_pt, lm_pt;
    std::vector<std::vector<int>> lm_edges;  // landmark column: edges to free poses, by pose index
    // BlockSolver system
    std::vector<double> Hpp, bp, Hll, bl, Hpl;  // 36 / 6 per pose, 9 / 3 per landmark, 18 per edge
    std::vector<double> x;                      // Solver::_x = [6 np | 3 nl]

    static double chi2(const BAEdge& g) { return g.err[0] * (g.info * g.err[0]) + g.err[1] * (g.info * g.err[1]); }

    void project(BAEdge& g, const SE3& P, const double* Xp) const {  // EdgeSE3ProjectXYZ::computeError
        double pc[3];
        P.map(Xp, pc);
        const double px = pc[0] / pc[2], py = pc[1] / pc[2];
        g.err[0] = g.z[0] - (px * g.fx + g.cx);
        g.err[1] = g.z[1] - (py * g.fy + g.cy);
    }

    // Active vertices: those with an active edge; fixed keyframes get no
    // Hessian index; free poses first, then the marginalised points.
    bool initialize() {
        const int nkf = (int)T.size(), npt = (int)X.size() / 3;
        std::vector<int> kf_n(nkf, 0), pt_n(npt, 0);
        int nact = 0;
        for (const BAEdge& g : E)
            if (g.active) {
                kf_n[g.kf]++;
                pt_n[g.pt]++;
                nact++;
            }
        if (!nact) return false;
        pose_col.assign(nkf, -1);
        pose_kf.clear();
        for (int k = 0; k < nkf; k++)
            if (kind[k] == 0 && kf_n[k]) {
                pose_col[k] = (int)pose_kf.size();
                pose_kf.push_back(k);
            }
        lm_of_pt.assign(npt, -1);
        lm_pt.clear();
        for (int p = 0; p < npt; p++)
            if (pt_n[p]) {
                lm_of_pt[p] = (int)lm_pt.size();
                lm_pt.push_back(p);
            }
        lm_edges.assign(lm_pt.size(), {});
        for (int e = 0; e < (int)E.size(); e++)
            if (E[e].active && pose_col[E[e].kf] >= 0) lm_edges[lm_of_pt[E[e].pt]].push_back(e);
        for (auto& col : lm_edges)
            std::stable_sort(col.begin(), col.end(),
                             [&](int a, int b) { return pose_col[E[a].kf] < pose_col[E[b].kf]; });
        x.assign(6 * pose_kf.size() + 3 * lm_pt.size(), 0.0);
        return true;
    }

    double errors(const std::vector<SE3>& P, const std::vector<double>& Xs) {  // computeActiveErrors + activeRobustChi2
        double chi = 0;
        for (BAEdge& g : E) {
            if (!g.active) continue;
            project(g, P[g.kf], &Xs[3 * g.pt]);
            double rho[2];
            huber(chi2(g), delta, rho);
            chi += rho[0];
        }
        return chi;
    }

    void build() {  // BlockSolver::buildSystem
        const int np = (int)pose_kf.size(), nl = (int)lm_pt.size();
        Hpp.assign(36 * np, 0.0);
        bp.assign(6 * np, 0.0);
        Hll.assign(9 * nl, 0.0);
        bl.assign(3 * nl, 0.0);
        Hpl.assign(18 * E.size(), 0.0);
        for (int e = 0; e < (int)E.size(); e++) {
            const BAEdge& g = E[e];
            if (!g.active) continue;
            const SE3& P = T[g.kf];
            double pc[3];
            P.map(&X[3 * g.pt], pc);
            const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
            double R[3][3];
            quat_to_R(P.r, R);
            // _jacobianOplusXi = -1./z * tmp * R (point), _jacobianOplusXj (pose)
            const double tmp[2][3] = {{g.fx, 0, -x / z * g.fx}, {0, g.fy, -y / z * g.fy}};
            const double s = -1. / z;
            double A[2][3], B[2][6];
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 3; j++)
                    A[i][j] = ((s * tmp[i][0]) * R[0][j] + (s * tmp[i][1]) * R[1][j]) + (s * tmp[i][2]) * R[2][j];
            B[0][0] = x * y / z2 * g.fx;
            B[0][1] = -(1 + (x * x / z2)) * g.fx;
            B[0][2] = y / z * g.fx;
            B[0][3] = -1. / z * g.fx;
            B[0][4] = 0;
            B[0][5] = x / z2 * g.fx;
            B[1][0] = (1 + y * y / z2) * g.fy;
            B[1][1] = -x * y / z2 * g.fy;
            B[1][2] = -x / z * g.fy;
            B[1][3] = 0;
            B[1][4] = -1. / z * g.fy;
            B[1][5] = y / z2 * g.fy;
            double rho[2];
            huber(chi2(g), delta, rho);
            const double w = rho[1] * g.info;  // robustInformation = rho' * Omega
            const double o0 = -(g.info * g.err[0]) * rho[1], o1 = -(g.info * g.err[1]) * rho[1];
            const int l = lm_of_pt[g.pt];
            for (int i = 0; i < 3; i++) {
                bl[3 * l + i] += A[0][i] * o0 + A[1][i] * o1;
                for (int j = 0; j < 3; j++) Hll[9 * l + 3 * i + j] += (A[0][i] * w) * A[0][j] + (A[1][i] * w) * A[1][j];
            }
            const int c = pose_col[g.kf];
            if (c < 0) continue;
            for (int r = 0; r < 6; r++)
                for (int j = 0; j < 3; j++) Hpl[18 * e + 3 * r + j] = (B[0][r] * w) * A[0][j] + (B[1][r] * w) * A[1][j];
            for (int i = 0; i < 6; i++) {
                bp[6 * c + i] += B[0][i] * o0 + B[1][i] * o1;
                for (int j = 0; j < 6; j++) Hpp[36 * c + 6 * i + j] += (B[0][i] * w) * B[0][j] + (B[1][i] * w) * B[1][j];
            }
        }
    }

    double max_diag() const {  // computeLambdaInit over the index mapping
        double m = 0;
        for (size_t c = 0; c < pose_kf.size(); c++)
            for (int j = 0; j < 6; j++) m = std::max(std::fabs(Hpp[36 * c + 7 * j]), m);
        for (size_t l = 0; l < lm_pt.size(); l++)
            for (int j = 0; j < 3; j++) m = std::max(std::fabs(Hll[9 * l + 4 * j]), m);
        return m;
    }

    // setLambda + BlockSolver::solve (Schur) + restoreDiagonal. Writes x only
    // when the reduced camera system factors.
    bool solve(double lambda) {
        const int np = (int)pose_kf.size(), nl = (int)lm_pt.size(), n = 6 * np;
        std::vector<double> S((size_t)n * n, 0.0), coef(n, 0.0), Dinv(9 * (size_t)nl), db(3 * (size_t)nl);
        for (int c = 0; c < np; c++)  // _Hschur = _Hpp (upper blocks, lambda on the diagonal)
            for (int i = 0; i < 6; i++)
                for (int j = 0; j < 6; j++)
                    S[(size_t)(6 * c + i) * n + 6 * c + j] = Hpp[36 * c + 6 * i + j] + (i == j ? lambda : 0.0);
        for (int l = 0; l < nl; l++) {
            double D[9];
            for (int i = 0; i < 9; i++) D[i] = Hll[9 * l + i] + (i % 4 == 0 ? lambda : 0.0);
            double* Di = &Dinv[9 * (size_t)l];
            inverse3(D, Di);
            const double* b = &bl[3 * l];
            for (int i = 0; i < 3; i++) db[3 * l + i] = (Di[3 * i] * b[0] + Di[3 * i + 1] * b[1]) + Di[3 * i + 2] * b[2];
            const double* d = &db[3 * l];
            const std::vector<int>& col = lm_edges[l];
            for (size_t a = 0; a < col.size(); a++) {
                const int i1 = pose_col[E[col[a]].kf];
                const double* Bi = &Hpl[18 * (size_t)col[a]];
                double BD[18];
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++)
                        BD[3 * r + c] = (Bi[3 * r] * Di[c] + Bi[3 * r + 1] * Di[3 + c]) + Bi[3 * r + 2] * Di[6 + c];
                for (int r = 0; r < 6; r++) coef[6 * i1 + r] += (Bi[3 * r] * d[0] + Bi[3 * r + 1] * d[1]) + Bi[3 * r + 2] * d[2];
                for (size_t b2 = a; b2 < col.size(); b2++) {
                    const int i2 = pose_col[E[col[b2]].kf];
                    const double* Bj = &Hpl[18 * (size_t)col[b2]];
                    for (int r = 0; r < 6; r++)
                        for (int c = 0; c < 6; c++)
                            S[(size_t)(6 * i1 + r) * n + 6 * i2 + c] -=
                                (BD[3 * r] * Bj[3 * c] + BD[3 * r + 1] * Bj[3 * c + 1]) + BD[3 * r + 2] * Bj[3 * c + 2];
                }
            }
        }
        // dense LL^T of the upper-stored S (CHOLMOD stand-in, see header);
        // divisions by L_jj are multiplications by its reciprocal
        std::vector<double> L((size_t)n * n, 0.0), rinv(n), y(n), xs(n);
        for (int j = 0; j < n; j++) {
            double s = S[(size_t)j * n + j];
            for (int k = 0; k < j; k++) s -= L[(size_t)j * n + k] * L[(size_t)j * n + k];
            if (!(s > 0.0)) return false;
            const double dj = std::sqrt(s);
            L[(size_t)j * n + j] = dj;
            rinv[j] = 1.0 / dj;
            for (int i = j + 1; i < n; i++) {
                double t = S[(size_t)j * n + i];
                for (int k = 0; k < j; k++) t -= L[(size_t)i * n + k] * L[(size_t)j * n + k];
                L[(size_t)i * n + j] = t * rinv[j];
            }
        }
        for (int i = 0; i < n; i++) {
            double s = bp[i] - coef[i];  // _bschur = _b - coefficients
            for (int k = 0; k < i; k++) s -= L[(size_t)i * n + k] * y[k];
            y[i] = s * rinv[i];
        }
        for (int i = n - 1; i >= 0; i--) {
            double s = y[i];
            for (int k = n - 1; k > i; k--) s -= L[(size_t)k * n + i] * xs[k];
            xs[i] = s * rinv[i];
        }
        for (int i = 0; i < n; i++) x[i] = xs[i];
        // landmarks: cl = bl + Hpl^T (-xp) (column blocks in pose order), xl = Dinv cl
        for (int l = 0; l < nl; l++) {
            double cl[3] = {bl[3 * l], bl[3 * l + 1], bl[3 * l + 2]};
            for (int e : lm_edges[l]) {
                const int i1 = pose_col[E[e].kf];
                const double* B = &Hpl[18 * (size_t)e];
                double cp[6];
                for (int r = 0; r < 6; r++) cp[r] = -x[6 * i1 + r];
                for (int c = 0; c < 3; c++) {
                    double t = B[c] * cp[0];
                    for (int r = 1; r < 6; r++) t += B[3 * r + c] * cp[r];
                    cl[c] += t;
                }
            }
            const double* Di = &Dinv[9 * (size_t)l];
            for (int i = 0; i < 3; i++) x[n + 3 * l + i] = (Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1]) + Di[3 * i + 2] * cl[2];
        }
        return true;
    }

    // SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg.
    int optimize(int iterations) {
        if (!initialize()) return -1;  // empty graph / no vertex to optimise
        const int np = (int)pose_kf.size(), nl = (int)lm_pt.size();
        double lambda = 0, ni = 2;
        int nBad = 0, it_done = 0;
        for (int iter = 0; iter < iterations; iter++) {
            it_done++;
            double currentChi = errors(T, X);
            const double iniChi = currentChi;
            build();
            if (iter == 0) {
                lambda = 1e-5 * max_diag();
                ni = 2;
                nBad = 0;
            }
            double rho = 0;
            int q = 0;
            do {
                const std::vector<SE3> T0 = T;
                const std::vector<double> X0 = X;
                const bool ok = solve(lambda);
                for (int c = 0; c < np; c++) T[pose_kf[c]] = se3_mul(se3_exp(&x[6 * c]), T[pose_kf[c]]);
                for (int l = 0; l < nl; l++)
                    for (int i = 0; i < 3; i++) X[3 * lm_pt[l] + i] += x[6 * np + 3 * l + i];
                double tempChi = errors(T, X);
                if (!ok) tempChi = DBL_MAX;
                rho = currentChi - tempChi;
                double scale = 0;
                for (int j = 0; j < 6 * np; j++) scale += x[j] * (lambda * x[j] + bp[j]);
                for (int j = 0; j < 3 * nl; j++) scale += x[6 * np + j] * (lambda * x[6 * np + j] + bl[j]);
                scale += 1e-3;
                rho /= scale;
                if (rho > 0 && std::isfinite(tempChi)) {
                    double alpha = 1. - std::pow((2 * rho - 1), 3);
                    alpha = std::min(alpha, 2. / 3.);
                    const double sf = std::max(1. / 3., alpha);
                    lambda *= sf;
                    ni = 2;
                    currentChi = tempChi;
                } else {
                    lambda *= ni;
                    ni *= 2;
                    T = T0;  // pop(): the estimate is restored, the edge errors keep the trial values
                    X = X0;
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

    bool is_outlier(const BAEdge& g) const {  // chi2 > 5.991 || !isDepthPositive()
        double pc[3];
        T[g.kf].map(&X[3 * g.pt], pc);
        return chi2(g) > 5.991 || !(pc[2] > 0.0);
    }
};

}  // namespace
}  // namespace orc

extern "C" {

int orc_local_ba_iters(const gf_ba_problem* P, gf_ba_result* R, int its0, int its1);

// Optimizer::LocalBundleAdjustment on an explicit local window (gf_ba_problem).
int orc_local_ba(const gf_ba_problem* P, gf_ba_result* R) { return orc_local_ba_iters(P, R, 5, 10); }

// The same with other iteration caps for the two optimize() calls (a force
// stop after its0 iterations is optimize(its0) then optimize(0)).
int orc_local_ba_iters(const gf_ba_problem* P, gf_ba_result* R, int its0, int its1) {
    if (!P || !R) return GF_ERR_ARG;
    orc::LBA L;
    L.delta = (double)(float)std::sqrt(5.991);  // const float thHuber = sqrt(5.991)
    for (int k = 0; k < P->nkf; k++) {
        L.T.push_back(orc::se3_from_Tcw(P->kf_Tcw + 16 * k));
        L.kind.push_back(P->kf_kind[k]);
    }
    for (int i = 0; i < 3 * P->npts; i++) L.X.push_back((double)P->pt_pos[i]);
    for (int e = 0; e < P->nedges; e++) {
        orc::BAEdge g;
        g.pt = P->edge_pt[e];
        g.kf = P->edge_kf[e];
        g.z[0] = P->edge_z[2 * e];
        g.z[1] = P->edge_z[2 * e + 1];
        g.info = P->edge_inv_sigma2[e];
        const float* K = P->kf_cam + 4 * g.kf;
        g.fx = K[0];
        g.fy = K[1];
        g.cx = K[2];
        g.cy = K[3];
        g.err[0] = g.err[1] = 0;
        g.active = true;
        L.E.push_back(g);
        R->edge_outlier[e] = 0;
    }
    R->iterations[0] = L.optimize(its0);
    for (int e = 0; e < P->nedges; e++)
        if (L.is_outlier(L.E[e])) {
            L.E[e].active = false;  // EraseMapPointMatch / EraseObservation / removeEdge
            R->edge_outlier[e] = 1;
        }
    R->iterations[1] = L.optimize(its1);
    for (int e = 0; e < P->nedges; e++)
        if (L.E[e].active && L.is_outlier(L.E[e])) R->edge_outlier[e] = 2;
    for (int k = 0; k < P->nkf; k++) {
        if (L.kind[k] == 2)
            std::memcpy(R->kf_Tcw + 16 * k, P->kf_Tcw + 16 * k, 64);
        else
            orc::se3_to_Tcw(L.T[k], R->kf_Tcw + 16 * k);
    }
    for (int i = 0; i < 3 * P->npts; i++) R->pt_pos[i] = (float)L.X[i];
    return GF_OK;
}

// Eigen 3x3 inverse as used for the landmark blocks (checked against numpy).
void orc_inverse3(const double* m, double* r) { orc::inverse3(m, r); }

}  // extern "C"
