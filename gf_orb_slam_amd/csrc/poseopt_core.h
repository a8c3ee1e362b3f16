// Motion-only pose optimisation core (see poseopt.hip): the one-wave LM of
// Optimizer::PoseOptimization shared by the batched kernel and the
// relocalisation step (reloc.hip).
#pragma once
#include <cfloat>

#include "common.h"
#include "se3.h"

namespace gfpose {
namespace {
constexpr int PO_NACC = 28;  // 21 lower-triangle H + 6 b + robust chi2
constexpr int PO_CHI = 27;
constexpr int PO_SPEC = 4;   // LM trials evaluated together (see k_pose_opt)
constexpr int PO_ROWS = PO_CHI + PO_SPEC;  // term rows: H, b, one chi2 row per trial
// One wave per problem: a frame's edges (tens to a few hundred) go through in
// passes of PO_E, and the footprint (29 KB of LDS) lets four problems share a
// CU with the other stream groups' extraction workgroups. (r02 ran 256
// threads and 256-edge passes: 77 KB, one or two problems per CU.)
#ifndef PO_THREADS
#define PO_THREADS 64
#endif
constexpr int PO_T = PO_THREADS;  // threads per problem
#ifndef PO_E
#define PO_E 64                   // edges per pass (a term row's length)
#endif
constexpr int PO_TP = PO_E + 1;  // term row pitch (doubles): accumulator threads read distinct banks
constexpr int PO_STRIDE_MAX = 8192;
constexpr int PO_LDS_EDGES = 384;  // problems up to this size keep edges and residuals in LDS (18 KB)

// Phase timing (diagnostic build only: -DGF_POSE_STAMPS): problem 0, lane 0
// accumulates s_memrealtime ticks (100 MHz) per phase and prints them.
#ifdef GF_POSE_STAMPS
#define PO_ST_DECL unsigned long long _st_prev = wall_clock64(), _st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PO_ST(i)                                           \
    do {                                                   \
        const unsigned long long _n = wall_clock64();      \
        _st[i] += _n - _st_prev;                           \
        _st_prev = _n;                                     \
    } while (0)
#else
#define PO_ST_DECL
#define PO_ST(i) \
    do {         \
    } while (0)
#endif

struct PoseArgs {
    const gf_pose_edge* edges;
    const int32_t* nedges;
    int stride;
    float* Tcw;
    uint8_t* outl;
    int32_t* ninl;
    int32_t* iters;
    double* work;  // per problem: err0[stride], err1[stride], info[stride]
    double fx, fy, cx, cy;
    // optional scatter of the outlier flags to keypoint slots
    const int32_t* edge_kp;
    uint8_t* kp_outl;
    int kp_stride;
    // optional gate: problem p is not run at all (pose, flags and counts
    // untouched) when gate[p] < gate_min
    const int32_t* gate;
    int gate_min;
};

struct Lane {
    const gf_pose_edge* E;
    double* info;
    int n, l;
    double fx, fy, cx, cy, delta, dsqr;
};

__device__ __forceinline__ void robustify(double e, double delta, double dsqr, double& rho0, double& rho1) {
    if (e <= dsqr) {
        rho0 = e;
        rho1 = 1.;
    } else {
        const double s = sqrt(e);
        rho0 = 2 * s * delta - dsqr;
        rho1 = delta / s;
    }
}

__device__ __forceinline__ void edge_error(const Lane& L, const gfse3::SE3& T, int e, double* pc, double& r0,
                                           double& r1) {
    const gf_pose_edge g = L.E[e];
    const double X[3] = {(double)g.X[0], (double)g.X[1], (double)g.X[2]};
    gfse3::map(T, X, pc);
    const double px = pc[0] / pc[2], py = pc[1] / pc[2];
    r0 = (double)g.z[0] - (px * L.fx + L.cx);
    r1 = (double)g.z[1] - (py * L.fy + L.cy);
}

// acc += row[0] + ... + row[m - 1], one dependent add per term in order
// (the reference's sequential sum); the next 8 terms' LDS loads are issued
// before the current 8 are added, so the chain waits on the adds only. Loads
// are unconditional (a tail past m reads neighbouring LDS, not added) so the
// compiler can count them.
__device__ __forceinline__ double chain_sum(const double* row, int m, double acc) {
    // two named buffers alternate (no register rotation, so no wait for the
    // batch in flight before the adds)
    double a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; u++) a[u] = row[u];
    for (int j = 8;; j += 16) {
        if (j >= m) {  // a holds terms j - 8 .. m - 1
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (j - 8 + u < m) acc += a[u];
            break;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) b[u] = row[j + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += a[u];
        if (j + 8 >= m) {  // b holds terms j .. m - 1
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (j + u < m) acc += b[u];
            break;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) a[u] = row[j + 8 + u];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += b[u];
    }
    return acc;
}

// PO_MFMA (A/B build, off in the product): buildSystem's H = sum_e J^T W J
// and b on v_mfma_f64_16x16x4f64 instead of the ordered VALU sums. Per pass
// each edge writes its two Jacobian rows J_r (6) and (w J_r, o_r) (7) to LDS
// (the H / b term rows' space); wave 0 then contracts them, four edge rows
// per MFMA: A[i][k] = J_{r_k}[i], B[k][j] = w J_{r_k}[j] (j < 6), o_{r_k}
// (j = 6), so D[i][j < 6] = H[i][j] and D[i][6] = b[i], accumulated over the
// passes in registers. The sums' order is the matrix core's, not the edge
// order of g2o's buildSystem (block_solver.hpp:502-562).
#ifndef PO_MFMA
#define PO_MFMA 0
#endif
typedef double po_d4 __attribute__((ext_vector_type(4)));
constexpr int PO_JB = 6 * 2 * PO_E;  // offset of the (w J, o) rows in the buffer

__device__ __forceinline__ void mfma_store_rows(double* jb, int ll, const double* J0, const double* J1, double w,
                                                double o0, double o1) {
#pragma unroll
    for (int i = 0; i < 6; i++) {
        jb[(2 * ll) * 6 + i] = J0[i];
        jb[(2 * ll + 1) * 6 + i] = J1[i];
        jb[PO_JB + (2 * ll) * 7 + i] = J0[i] * w;
        jb[PO_JB + (2 * ll + 1) * 7 + i] = J1[i] * w;
    }
    jb[PO_JB + (2 * ll) * 7 + 6] = o0;
    jb[PO_JB + (2 * ll + 1) * 7 + 6] = o1;
}

// wave 0: acc += the pass's m edges (2 m rows)
__device__ __forceinline__ void mfma_accumulate(const double* jb, int m, int l, po_d4& acc) {
    const int i = l & 15, kk = l >> 4;
    for (int t = 0; 4 * t < 2 * m; t++) {
        const int r = 4 * t + kk;
        const bool rv = r < 2 * m;
        const double a = (rv && i < 6) ? jb[r * 6 + i] : 0.0;
        const double bb = (rv && i < 7) ? jb[PO_JB + r * 7 + i] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
    }
}

// H lower packed [0, 21) and b [21, 27) from the accumulator: lane l holds
// D[row (l >> 4) + 4 u][col l & 15] in acc[u]
__device__ __forceinline__ void mfma_write(const po_d4& acc, int l, double* sh_sum) {
    const int col = l & 15, rb = l >> 4;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const int row = rb + 4 * u;
        if (row < 6) {
            const double v = u == 0 ? acc[0] : u == 1 ? acc[1] : u == 2 ? acc[2] : acc[3];
            if (col <= row) sh_sum[row * (row + 1) / 2 + col] = v;
            if (col == 6) sh_sum[21 + row] = v;
        }
    }
}

// computeActiveErrors + activeRobustChi2 (+ buildSystem when `build`) at T.
// Returns the sums in sh_sum: [0,21) lower H row-major-packed, [21,27) b, 27 chi2.
__device__ __forceinline__ void pass(const Lane& L, const gfse3::SE3& T, bool build, double (*term)[PO_TP],
                                     double* sh_sum) {
    // (build: the H/b rows too; the chi2 row is PO_CHI)
    double acc = 0.0;
#if PO_MFMA
    po_d4 macc = {0.0, 0.0, 0.0, 0.0};
#endif
    for (int base = 0; base < L.n; base += PO_E) {
        const int e = base + L.l;
        if (L.l < PO_E && e < L.n) {
            double pc[3], r0, r1;
            edge_error(L, T, e, pc, r0, r1);
            const double info = L.info[e];
            const double chi2 = r0 * (info * r0) + r1 * (info * r1);
            double rho0, rho1;
            robustify(chi2, L.delta, L.dsqr, rho0, rho1);
            term[PO_CHI][L.l] = rho0;
            if (build) {
                const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
                double J0[6], J1[6];
                J0[0] = x * y / z2 * L.fx;
                J0[1] = -(1 + (x * x / z2)) * L.fx;
                J0[2] = y / z * L.fx;
                J0[3] = -1. / z * L.fx;
                J0[4] = 0;
                J0[5] = x / z2 * L.fx;
                J1[0] = (1 + y * y / z2) * L.fy;
                J1[1] = -x * y / z2 * L.fy;
                J1[2] = -x / z * L.fy;
                J1[3] = 0;
                J1[4] = -1. / z * L.fy;
                J1[5] = y / z2 * L.fy;
                const double w = rho1 * info;
                const double o0 = -(info * r0) * rho1, o1 = -(info * r1) * rho1;
#if PO_MFMA
                mfma_store_rows(&term[0][0], L.l, J0, J1, w, o0, o1);
#else
                int k = 0;
#pragma unroll
                for (int a = 0; a < 6; a++)
#pragma unroll
                    for (int b = 0; b <= a; b++) term[k++][L.l] = (J0[a] * w) * J0[b] + (J1[a] * w) * J1[b];
#pragma unroll
                for (int a = 0; a < 6; a++) term[21 + a][L.l] = J0[a] * o0 + J1[a] * o1;
#endif
            }
        }
        __syncthreads();
        const int m = min(PO_E, L.n - base);
#if PO_MFMA
        if (build && L.l < 64) mfma_accumulate(&term[0][0], m, L.l, macc);
        if (L.l == PO_CHI) acc = chain_sum(term[L.l], m, acc);
#else
        if ((build && L.l < PO_NACC) || L.l == PO_CHI) {
            acc = chain_sum(term[L.l], m, acc);
        }
#endif
        __syncthreads();
    }
#if PO_MFMA
    if (build && L.l < 64) mfma_write(macc, L.l, sh_sum);
    if (L.l == PO_CHI) sh_sum[L.l] = acc;
#else
    if ((build && L.l < PO_NACC) || L.l == PO_CHI) sh_sum[L.l] = acc;
#endif
    __syncthreads();
}

// computeActiveErrors + activeRobustChi2 at S trial estimates at once, and
// buildSystem at trial 0's: lane PO_CHI + s adds trial s's robust chi2 terms
// in edge order, lanes 0..26 trial 0's H and b terms. When trial 0 is
// accepted (most LM iterations) the next iteration's linearisation is
// already in sh_sum — the same arithmetic g2o's next computeActiveErrors +
// buildSystem at that estimate performs. With NT = 256 (a problem per
// workgroup, for small batches) wave s evaluates trial s, so the trials'
// edge passes run on four SIMDs instead of one after another.
template <int NT>
__device__ __forceinline__ void pass_trials(const Lane& L, const gfse3::SE3* T, int S, double (*term)[PO_TP],
                                            double* sh_sum) {
    double acc = 0.0;
#if PO_MFMA
    po_d4 macc = {0.0, 0.0, 0.0, 0.0};
#endif
    const int wv = NT > 64 ? L.l >> 6 : 0, ll = NT > 64 ? L.l & 63 : L.l;
    for (int base = 0; base < L.n; base += PO_E) {
        const int e = base + ll;
        if (ll < PO_E && e < L.n && wv < S) {
            const double info = L.info[e];
#pragma unroll
            for (int s = 0; s < PO_SPEC; s++) {
                if (s >= S) break;
                if (NT > 64 && s != wv) continue;
                double pc[3], r0, r1;
                edge_error(L, T[s], e, pc, r0, r1);
                const double chi2 = r0 * (info * r0) + r1 * (info * r1);
                double rho0, rho1;
                robustify(chi2, L.delta, L.dsqr, rho0, rho1);
                term[PO_CHI + s][ll] = rho0;
                if (s == 0) {
                    const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
                    double J0[6], J1[6];
                    J0[0] = x * y / z2 * L.fx;
                    J0[1] = -(1 + (x * x / z2)) * L.fx;
                    J0[2] = y / z * L.fx;
                    J0[3] = -1. / z * L.fx;
                    J0[4] = 0;
                    J0[5] = x / z2 * L.fx;
                    J1[0] = (1 + y * y / z2) * L.fy;
                    J1[1] = -x * y / z2 * L.fy;
                    J1[2] = -x / z * L.fy;
                    J1[3] = 0;
                    J1[4] = -1. / z * L.fy;
                    J1[5] = y / z2 * L.fy;
                    const double w = rho1 * info;
                    const double o0 = -(info * r0) * rho1, o1 = -(info * r1) * rho1;
#if PO_MFMA
                    mfma_store_rows(&term[0][0], ll, J0, J1, w, o0, o1);
#else
                    int k = 0;
#pragma unroll
                    for (int a = 0; a < 6; a++)
#pragma unroll
                        for (int b = 0; b <= a; b++) term[k++][ll] = (J0[a] * w) * J0[b] + (J1[a] * w) * J1[b];
#pragma unroll
                    for (int a = 0; a < 6; a++) term[21 + a][ll] = J0[a] * o0 + J1[a] * o1;
#endif
                }
            }
        }
        __syncthreads();
        const int m = min(PO_E, L.n - base);
#if PO_MFMA
        if (L.l < 64) mfma_accumulate(&term[0][0], m, L.l, macc);
        if (L.l >= PO_CHI && L.l < PO_CHI + S) acc = chain_sum(term[L.l], m, acc);
#else
        if (L.l < PO_CHI + S) {
            acc = chain_sum(term[L.l], m, acc);
        }
#endif
        __syncthreads();
    }
#if PO_MFMA
    if (L.l < 64) mfma_write(macc, L.l, sh_sum);
    if (L.l >= PO_CHI && L.l < PO_CHI + S) sh_sum[L.l] = acc;
#else
    if (L.l < PO_CHI + S) sh_sum[L.l] = acc;
#endif
    __syncthreads();
}

// k_pose_opt's body: problem p by NT threads (one wave, or four with the
// trials' passes split over them).
template <int NT = PO_T>
__device__ __forceinline__ void pose_opt_problem(const PoseArgs& A, int p) {
    if (A.gate && A.gate[p] < A.gate_min) return;
    __shared__ double term[PO_ROWS][PO_TP];
    __shared__ double sh_sum[PO_ROWS];
    __shared__ double sh_x[PO_SPEC][6];       // each speculative trial's solution
    __shared__ int sh_ok[PO_SPEC];
    __shared__ gfse3::SE3 sh_T[PO_SPEC];      // and its trial estimate
    // every pass re-reads each edge and its residuals: for problems up to
    // PO_LDS_EDGES edges they live in LDS (generic pointers), else in HBM
    __shared__ gf_pose_edge sh_edges[PO_LDS_EDGES];
    __shared__ double sh_info[PO_LDS_EDGES];
    PO_ST_DECL
    Lane L;
    L.l = threadIdx.x;
    L.n = min(max(A.nedges[p], 0), A.stride);
    if (L.n <= PO_LDS_EDGES) {
        const gf_pose_edge* src = A.edges + (size_t)p * A.stride;
        for (int e = L.l; e < L.n; e += NT) sh_edges[e] = src[e];
        L.E = sh_edges;
        L.info = sh_info;
        __syncthreads();
    } else {
        L.E = A.edges + (size_t)p * A.stride;
        L.info = A.work + (size_t)p * A.stride;
    }
    L.fx = A.fx;
    L.fy = A.fy;
    L.cx = A.cx;
    L.cy = A.cy;
    L.delta = (double)(float)sqrt(5.991);  // const float delta = sqrt(5.991)
    L.dsqr = L.delta * L.delta;
    uint8_t* ou = A.outl + (size_t)p * A.stride;
    float* Tp = A.Tcw + (size_t)p * 16;

    // Converter::toSE3Quat: float Tcw -> Matrix3d -> Quaterniond -> normalizeRotation
    gfse3::SE3 T;
    {
        double R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = (double)Tp[4 * i + j];
        T.r = gfse3::from_R(R);
        for (int i = 0; i < 3; i++) T.t[i] = (double)Tp[4 * i + 3];
        gfse3::normalize(T.r);
    }
    for (int e = L.l; e < L.n; e += NT) {
        L.info[e] = (double)L.E[e].inv_sigma2;
        ou[e] = 0;
    }
    __syncthreads();

    // chi2 thresholds {9.210, 7.378, 5.991, 5.991} (float) and iterations {10, 10, 7, 5}
    int nBadEdges = 0, total_it = 0;
    double xs[6] = {0, 0, 0, 0, 0, 0};
    gfse3::SE3 last_eval = T;  // the estimate whose residuals the edges hold
    for (int round = 0; round < 4 && L.n > 0; round++) {
        const double chi2th = round == 0 ? (double)9.210f : round == 1 ? (double)7.378f : (double)5.991f;
        const int its = round < 2 ? 10 : round == 2 ? 7 : 5;
        // SparseOptimizer::optimize(its) with the Levenberg algorithm
        double lambda = 0, ni = 2;
        int nBad = 0;
        bool have_build = false;  // sh_sum already holds H, b, chi2 at T (trial 0 accepted)
        for (int iter = 0; iter < its; iter++) {
            total_it++;
            PO_ST(0);
            if (!have_build) pass(L, T, true, term, sh_sum);
            PO_ST(1);
            have_build = false;
            double H[36], b[6];
            for (int a = 0, k = 0; a < 6; a++)
                for (int c = 0; c <= a; c++, k++) H[6 * a + c] = H[6 * c + a] = sh_sum[k];
            for (int a = 0; a < 6; a++) b[a] = sh_sum[21 + a];
            double currentChi = sh_sum[PO_CHI];
            const double iniChi = currentChi;
            if (iter == 0) {
                double md = 0;
                for (int j = 0; j < 6; j++) md = fmax(fabs(H[7 * j]), md);
                lambda = 1e-5 * md;
                ni = 2;
                nBad = 0;
            }
            // g2o's trial loop (levenberg.cpp:99-163): on a rejection lambda *= ni,
            // ni *= 2 and the next trial solves again. The next PO_SPEC trials'
            // lambdas are therefore known in advance; they are solved (one
            // 16-lane group per trial), their estimates built and their chi2
            // evaluated together, and the sequential decision then walks them
            // in order and stops at the first acceptance — the same trials, the
            // same arithmetic and the same outcome as one trial at a time.
            double rho = 0;
            int q = 0;
            bool more = true;
            while (more) {
                const int S = min(PO_SPEC, 10 - q);
                double lam_s[PO_SPEC], ni_s[PO_SPEC];
                lam_s[0] = lambda;
                ni_s[0] = ni;
#pragma unroll
                for (int s2 = 1; s2 < PO_SPEC; s2++) {
                    lam_s[s2] = lam_s[s2 - 1] * ni_s[s2 - 1];
                    ni_s[s2] = ni_s[s2 - 1] * 2;
                }
                {
                    const int g = (L.l & 63) >> 4;  // this lane's trial (every wave computes all four)
                    double lam_g = lam_s[0];
#pragma unroll
                    for (int s2 = 1; s2 < PO_SPEC; s2++)
                        if (g == s2) lam_g = lam_s[s2];
                    double Hl[36];
                    for (int i = 0; i < 36; i++) Hl[i] = H[i];
                    for (int j = 0; j < 6; j++) Hl[7 * j] += lam_g;
                    double xn[6];
                    const bool ok = gfse3::ldlt6(Hl, b, xn);
                    if (L.l < 64 && (L.l & 15) == 0 && g < PO_SPEC) {
                        sh_ok[g] = ok;
                        for (int j = 0; j < 6; j++) sh_x[g][j] = xn[j];
                    }
                }
                __syncthreads();
                PO_ST(2);
                // a failed factorisation keeps the previous solution (Solver::_x):
                // trial g solves with the last successful x among trials <= g
                {
                    const int g = L.l >> 4;
                    if (L.l < 64 && (L.l & 15) == 0 && g < S) {
                        double xg[6];
                        for (int j = 0; j < 6; j++) xg[j] = xs[j];
                        for (int s2 = 0; s2 <= g; s2++)
                            if (sh_ok[s2])
                                for (int j = 0; j < 6; j++) xg[j] = sh_x[s2][j];
                        sh_T[g] = gfse3::exp_mul(xg, T);
                    }
                }
                __syncthreads();
                PO_ST(3);
                pass_trials<NT>(L, sh_T, S, term, sh_sum);
                PO_ST(4);
                for (int s2 = 0; s2 < S; s2++) {
                    const bool ok = sh_ok[s2];
                    if (ok)
                        for (int j = 0; j < 6; j++) xs[j] = sh_x[s2][j];
                    double tempChi = sh_sum[PO_CHI + s2];
                    if (!ok) tempChi = DBL_MAX;
                    rho = currentChi - tempChi;
                    double scale = 0;
                    for (int j = 0; j < 6; j++) scale += xs[j] * (lam_s[s2] * xs[j] + b[j]);
                    scale += 1e-3;
                    rho /= scale;
                    last_eval = sh_T[s2];
                    q++;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * rho - 1), 3.0);
                        alpha = fmin(alpha, 2. / 3.);
                        const double sf = fmax(1. / 3., alpha);
                        lambda = lam_s[s2] * sf;
                        ni = 2;
                        currentChi = tempChi;
                        T = sh_T[s2];
                        have_build = s2 == 0;
                    } else {
                        lambda = lam_s[s2] * ni_s[s2];
                        ni = ni_s[s2] * 2;
                    }
                    if (!(rho < 0 && q < 10)) {
                        more = false;
                        break;
                    }
                }
            }
            PO_ST(5);
            if (q == 10 || rho == 0) break;
            if ((iniChi - currentChi) * 1e3 < iniChi)
                nBad++;
            else
                nBad = 0;
            if (nBad >= 3) break;
        }
        // outlier classification (Optimizer.cc:373-395); errors are those of
        // the last evaluated estimate, recomputed at the current one for
        // flagged edges.
        int nb = 0;
        for (int base = 0; base < L.n; base += NT) {
            const int e = base + L.l;
            bool bad = false;
            if (e < L.n) {
                double pc[3], r0, r1;
                if (ou[e]) {
                    L.info[e] = (double)L.E[e].inv_sigma2;
                    edge_error(L, T, e, pc, r0, r1);
                } else {
                    edge_error(L, last_eval, e, pc, r0, r1);
                }
                const double info = L.info[e];
                const double c2 = r0 * (info * r0) + r1 * (info * r1);
                if (c2 > chi2th) {
                    ou[e] = 1;
                    L.info[e] = 1e-10;
                    bad = true;
                } else if (c2 <= chi2th) {
                    ou[e] = 0;
                }
            }
            nb += __syncthreads_count(bad);
        }
        nBadEdges = nb;
        __syncthreads();
        PO_ST(6);
        if (L.n < 10) break;
    }

    // Converter::toCvMat(SE3Quat): float pose out
    __syncthreads();
    if (L.l == 0) {
        double R[9];
        gfse3::to_R(T.r, R);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) Tp[4 * i + j] = (float)R[3 * i + j];
            Tp[4 * i + 3] = (float)T.t[i];
        }
        Tp[12] = Tp[13] = Tp[14] = 0.f;
        Tp[15] = 1.f;
        A.ninl[p] = L.n - nBadEdges;
        if (A.iters) A.iters[p] = total_it;
#ifdef GF_POSE_STAMPS
        if (p == 0)
            printf("POSE_STAMPS n=%d it=%d pre=%llu build=%llu ldlt=%llu exp=%llu trials=%llu dec=%llu class=%llu\n",
                   L.n, total_it, _st[0], _st[1], _st[2], _st[3], _st[4], _st[5], _st[6]);
#endif
    }
    if (A.kp_outl)
        for (int e = L.l; e < L.n; e += NT)
            A.kp_outl[(size_t)p * A.kp_stride + A.edge_kp[(size_t)p * A.stride + e]] = ou[e];
}

}  // namespace
}  // namespace gfpose
