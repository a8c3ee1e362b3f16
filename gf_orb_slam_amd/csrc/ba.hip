// Local bundle adjustment on gfx950.
//
// Optimizer::LocalBundleAdjustment (src/Optimizer.cc:1515-1764) builds a g2o
// graph — local keyframe poses (SE3; mnId 0 fixed), fixed observer cameras,
// marginalised map points, one Huber EdgeSE3ProjectXYZ per observation — and
// runs optimize(5), removes the edges with chi2 > 5.991 or negative depth,
// runs optimize(10) and flags the outliers again. The device keeps g2o's
// Levenberg-Marquardt (core/optimization_algorithm_levenberg.cpp:61-189) and
// its Schur solve (BlockSolver::solve, core/block_solver.hpp:354-486) as a
// state machine per problem in device memory. One host-enqueued step is one
// LM trial of every problem of the batch:
//
//   k_ba_linearize  computeActiveErrors + the point half of buildSystem, one
//                   thread per map point: Hll, b_l, the 6x3 Hpl block of every
//                   edge (also written into the dense K-major panel Ht), robust
//                   chi2 partial sums
//   k_ba_poses      the pose half: Hpp, b_p, one wave per free pose over its
//                   edge list
//   k_ba_schur_pts  lambda init, Dinv = (Hll + lambda I)^-1, db = Dinv b_l and
//                   W = Hpl Dinv into the panel Wt, db as Wt's column n
//   k_ba_gemm       C = Ht^T Wt on v_mfma_f64_16x16x4 (split-K, fixed order):
//                   the Schur product Hpl Dinv Hpl^T and the coefficient
//                   vector Hpl db in one pass — the J^T J-shaped contraction;
//                   k_ba_spgemm, the same product as a host-built task list of
//                   only the nonzero tile products (batches of <= 8 windows)
//   k_ba_solve      S = Hpp + lambda I - C, b_s = b_p - C[:, n]; dense LL^T
//                   and the triangular solves in LDS; trial poses exp(x) * T
//   k_ba_update     landmark back-substitution, trial points, trial errors
//   k_ba_decide     rho, lambda schedule and stop rules (levenberg.cpp:99-163);
//                   at the end of optimize(5) / optimize(10) the outlier pass
//                   (Optimizer.cc:1680-1698, 1724-1743)
//
// Every kernel reads the problem's state first and returns at once when the
// step does not concern it, so the host enqueues steps blindly and polls the
// done flags every few steps. Floating-point parity with the oracle is a
// tolerance (the reference's CHOLMOD is unpinned, and the Schur sums run in
// MFMA order); the LL^T itself and the triangular solves use the oracle's
// exact operation order.
#include <float.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <vector>

#include "common.h"
#include "se3.h"

namespace {

constexpr int BA_T = 64;      // threads of the point / edge kernels (one wave: more CUs for one window)
constexpr int BA_MAXSPLIT = 64;  // split-K of the Schur GEMM (per plan: more splits for small batches)
constexpr int BA_MAXFREE = 32;
constexpr int BA_MAXN = 6 * BA_MAXFREE;  // LDS of k_ba_solve
constexpr int BA_MAXPTS = 65536;
constexpr int BA_MAXSTEPS = 400;

typedef double d4 __attribute__((ext_vector_type(4)));

struct BADesc {
    int nkf, npts, nedges, nfree;
    int n, npad, K, sps;  // 6 * nfree; panel width; panel rows; MFMA k-steps per split
    int ntiles, nwg;      // Schur GEMM tiles; point workgroups
    int nsplit, newg;     // GEMM k-splits; edge workgroups
    int kf0, pt0, e0, f0, fe0, pl0, tile0, wg0, mask0, ss0;
    int item0, nitems, kl0, tip0;  // Schur GEMM task list: items, k-step list, per-tile item ranges
    long long panel0;  // Ht at panel0, Wt at panel0 + K * npad (doubles)
};

struct BAState {
    int round;     // 0: optimize(5), 1: optimize(10), 2: done
    int iter, q;   // outer iteration of the round, trial of the iteration
    int need_lin;  // next step starts an iteration (errors + buildSystem)
    int cur;       // estimate buffer holding the current state
    int chol_ok, nbad, pad;
    int iters[2];
    double lambda, ni, currentChi, iniChi, scale_p;
};

struct BAArena {
    const BADesc* desc;
    BAState* st;
    int nkf_tot, npt_tot;
    // keyframes: [2][nkf_tot][8] = q(w,x,y,z), t(3), pad
    double* kfT;
    const float* kf_Tcw0;
    const uint8_t* kf_kind;
    const int32_t* kf_col;  // free pose index or -1
    // points: [2][npt_tot][4]
    double* ptX;
    const float* pt_pos0;
    const int32_t* pt_eb;  // problem-local edge range [eb, ee)
    const int32_t* pt_ee;
    double *Hll, *bl, *Dinv, *xl;  // 9, 3, 9, 3 per point
    uint8_t* pt_act;
    // edges
    const int32_t* e_pt;   // problem-local
    const int32_t* e_kf;   // problem-local
    const double* e_meas;  // 8: z0, z1, info, fx, fy, cx, cy, 0
    double* e_err;         // 2: errors of the last evaluated estimate
    uint8_t* e_act;
    uint8_t* e_out;
    double* Hpl;  // 18 per edge (6x3 row-major)
    // free poses
    const int32_t* f_kf;
    const int32_t* f_eptr;   // nfree + 1 per problem, into f_elist (problem-local)
    const int32_t* f_elist;  // problem-local edge indices, point order
    double *Hpp, *bp, *xp;   // 36, 6, 6 per free pose
    uint8_t* f_act;
    // dense panels, their per-k-step column-tile masks, GEMM tiles and their
    // split sums (S lower packed + the coefficient column), per-workgroup partials
    double* panel;
    const uint16_t* kmask;
    const int4* items;        // (ti, tj, kb, ke): tile and its k-step range in klist
    const int32_t* klist;     // k-steps (4 panel rows) where both operand tiles are nonzero
    const int32_t* tile_iptr; // per problem ntiles + 1: the items of tile t, in order
    double* tiles;
    double* Ssum;
    double *wg_chi, *wg_chi_t, *wg_maxd, *wg_scale;
    // outputs
    float* out_T;
    float* out_X;
    // diagnostics: phase stamps of k_ba_solve (s_memrealtime, 100 MHz) when non-null
    unsigned long long* tstamp;
    // setForceStopFlag (Optimizer.cc:1579-1580): != 0 ends every optimize()
    // call at its next iteration boundary (SparseOptimizer::optimize checks
    // terminate() before each iteration, sparse_optimizer.cpp:376)
    const int* stop;
};

__device__ __forceinline__ gfse3::SE3 load_T(const BAArena& A, int buf, int gk) {
    const double* p = A.kfT + ((size_t)buf * A.nkf_tot + gk) * 8;
    gfse3::SE3 s;
    s.r.w = p[0];
    s.r.x = p[1];
    s.r.y = p[2];
    s.r.z = p[3];
    s.t[0] = p[4];
    s.t[1] = p[5];
    s.t[2] = p[6];
    return s;
}

__device__ __forceinline__ void store_T(const BAArena& A, int buf, int gk, const gfse3::SE3& s) {
    double* p = A.kfT + ((size_t)buf * A.nkf_tot + gk) * 8;
    p[0] = s.r.w;
    p[1] = s.r.x;
    p[2] = s.r.y;
    p[3] = s.r.z;
    p[4] = s.t[0];
    p[5] = s.t[1];
    p[6] = s.t[2];
}

__device__ __forceinline__ double* ptX_at(const BAArena& A, int buf, int gp) {
    return A.ptX + ((size_t)buf * A.npt_tot + gp) * 4;
}

__device__ __forceinline__ void huber(double e, double& rho0, double& rho1) {
    const double delta = (double)(float)sqrt(5.991);  // const float thHuber = sqrt(5.991)
    const double dsqr = delta * delta;
    if (e <= dsqr) {
        rho0 = e;
        rho1 = 1.;
    } else {
        const double s = sqrt(e);
        rho0 = 2 * s * delta - dsqr;
        rho1 = delta / s;
    }
}

// EdgeSE3ProjectXYZ::computeError; pc = T.map(X)
// SparseOptimizer::optimize checks terminate() before every iteration
// (sparse_optimizer.cpp:376): an iteration that would start while the
// caller's stop flag is raised does not run. The step's kernels then do
// nothing and k_ba_decide ends the round. (Within a step the flag is
// constant: the host writes it on the same stream between steps.)
__device__ __forceinline__ bool ba_halted(const BAArena& A, const BAState& st) {
    return st.need_lin && A.stop && *A.stop;
}

__device__ __forceinline__ void edge_error(const double* m, const gfse3::SE3& T, const double* X, double* pc,
                                           double& e0, double& e1) {
    gfse3::map(T, X, pc);
    const double px = pc[0] / pc[2], py = pc[1] / pc[2];
    e0 = m[0] - (px * m[3] + m[5]);
    e1 = m[1] - (py * m[4] + m[6]);
}

// EdgeSE3ProjectXYZ::linearizeOplus: point (2x3) and pose (2x6) Jacobians.
__device__ __forceinline__ void edge_jac(const double* m, const gfse3::SE3& T, const double* pc, double (*Jp)[3],
                                         double (*Jc)[6], bool want_point) {
    const double fx = m[3], fy = m[4];
    const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
    if (want_point) {
        double R[9];
        gfse3::to_R(T.r, R);
        const double s = -1. / z;
        const double tmp[2][3] = {{fx, 0, -x / z * fx}, {0, fy, -y / z * fy}};
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < 3; j++)
                Jp[i][j] = ((s * tmp[i][0]) * R[j] + (s * tmp[i][1]) * R[3 + j]) + (s * tmp[i][2]) * R[6 + j];
    }
    Jc[0][0] = x * y / z2 * fx;
    Jc[0][1] = -(1 + (x * x / z2)) * fx;
    Jc[0][2] = y / z * fx;
    Jc[0][3] = -1. / z * fx;
    Jc[0][4] = 0;
    Jc[0][5] = x / z2 * fx;
    Jc[1][0] = (1 + y * y / z2) * fy;
    Jc[1][1] = -x * y / z2 * fy;
    Jc[1][2] = -x / z * fy;
    Jc[1][3] = 0;
    Jc[1][4] = -1. / z * fy;
    Jc[1][5] = y / z2 * fy;
}

// BA_EG consecutive edges [le0, le0 + BA_EG) of one point (problem-local,
// clipped at ee): active flags, measurement records, the keyframe poses of
// estimate buffer buf and the free-pose columns, every load issued before any
// of them is used. A point's edge loop pays two memory round trips per group
// instead of two or three per edge; the edges are still consumed in order.
constexpr int BA_EG = 4;
struct BAEdgeGroup {
    bool act[BA_EG];
    int col[BA_EG];
    double m[BA_EG][8];
    gfse3::SE3 T[BA_EG];
    __device__ __forceinline__ void load(const BAArena& A, const BADesc& d, int buf, int le0, int ee) {
        int kf[BA_EG];
#pragma unroll
        for (int q = 0; q < BA_EG; q++) {
            const int ge = d.e0 + min(le0 + q, ee - 1);
            const uint8_t a = A.e_act[ge];
            act[q] = le0 + q < ee && a;
            kf[q] = A.e_kf[ge];
#pragma unroll
            for (int k = 0; k < 8; k++) m[q][k] = A.e_meas[(size_t)ge * 8 + k];
        }
#pragma unroll
        for (int q = 0; q < BA_EG; q++) {
            T[q] = load_T(A, buf, d.kf0 + kf[q]);
            col[q] = A.kf_col[d.kf0 + kf[q]];
        }
    }
};

// Workgroup sum / max of one double per thread in a fixed order.
__device__ double block_reduce(double v, double* sh, bool is_max) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double u = __shfl_xor(v, o, 64);
        v = is_max ? fmax(v, u) : v + u;
    }
    if (lane == 0) sh[w] = v;
    __syncthreads();
    double r = sh[0];
    for (int i = 1; i < nw; i++) r = is_max ? fmax(r, sh[i]) : r + sh[i];
    __syncthreads();
    return r;
}

// Eigen compute_inverse<Matrix3d> (oracle/lba.cpp inverse3).
__device__ __forceinline__ void inverse3(const double* m, double* r) {
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[7] * m[2] - m[8] * m[1];
    const double c2 = m[1] * m[5] - m[2] * m[4];
    const double det = (c0 * m[0] + c1 * m[3]) + c2 * m[6];
    const double inv = 1.0 / det;
    r[0] = c0 * inv;
    r[1] = c1 * inv;
    r[2] = c2 * inv;
    r[3] = (m[5] * m[6] - m[3] * m[8]) * inv;
    r[4] = (m[8] * m[0] - m[6] * m[2]) * inv;
    r[5] = (m[2] * m[3] - m[0] * m[5]) * inv;
    r[6] = (m[3] * m[7] - m[4] * m[6]) * inv;
    r[7] = (m[6] * m[1] - m[7] * m[0]) * inv;
    r[8] = (m[0] * m[4] - m[1] * m[3]) * inv;
}

// ------------------------------------------------------------------ init
__global__ __launch_bounds__(256) void k_ba_init(BAArena A) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const BADesc d = A.desc[p];
    for (int k = tid; k < d.nkf; k += 256) {  // Converter::toSE3Quat
        const float* T = A.kf_Tcw0 + (size_t)(d.kf0 + k) * 16;
        double R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[3 * i + j] = (double)T[4 * i + j];
        gfse3::SE3 s;
        s.r = gfse3::from_R(R);
        for (int i = 0; i < 3; i++) s.t[i] = (double)T[4 * i + 3];
        gfse3::normalize(s.r);
        store_T(A, 0, d.kf0 + k, s);
    }
    for (int i = tid; i < d.npts; i += 256) {
        double* X = ptX_at(A, 0, d.pt0 + i);
        for (int c = 0; c < 3; c++) X[c] = (double)A.pt_pos0[(size_t)(d.pt0 + i) * 3 + c];
        for (int c = 0; c < 3; c++) A.xl[(size_t)(d.pt0 + i) * 3 + c] = 0.0;
    }
    for (int e = tid; e < d.nedges; e += 256) {
        A.e_act[d.e0 + e] = 1;
        A.e_out[d.e0 + e] = 0;
        // an edge's _error before any computeError: taken as 0 (g2o leaves the
        // Eigen member uninitialised; read by a stop before the first iteration)
        A.e_err[(size_t)(d.e0 + e) * 2] = 0.0;
        A.e_err[(size_t)(d.e0 + e) * 2 + 1] = 0.0;
    }
    for (int i = tid; i < 6 * d.nfree; i += 256) A.xp[(size_t)d.f0 * 6 + i] = 0.0;
    if (tid == 0) {
        BAState s{};
        s.round = d.nedges > 0 ? 0 : 2;
        s.iters[0] = d.nedges > 0 ? 0 : -1;
        s.iters[1] = d.nedges > 0 ? 0 : -1;
        s.need_lin = 1;
        s.ni = 2;
        A.st[p] = s;
    }
}

// ------------------------------------------------------------------ buildSystem, point half
__global__ __launch_bounds__(BA_T) void k_ba_linearize(BAArena A) {
    __shared__ double sh[BA_T / 64];
    const int p = blockIdx.y;
    const BADesc d = A.desc[p];
    if (blockIdx.x >= d.nwg) return;
    const BAState st = A.st[p];
    if (st.round >= 2 || !st.need_lin || ba_halted(A, st)) return;
    const int i = blockIdx.x * BA_T + threadIdx.x;
    double chi = 0.0, maxd = 0.0;
    if (i < d.npts) {
        const int gp = d.pt0 + i, cur = st.cur;
        const double* Xp = ptX_at(A, cur, gp);
        const double X[3] = {Xp[0], Xp[1], Xp[2]};
        double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
        int nact = 0;
        const int eb = A.pt_eb[gp], ee = A.pt_ee[gp];
        for (int le0 = eb; le0 < ee; le0 += BA_EG) {
            // one group of edges: their records and poses loaded before the
            // first edge's arithmetic (two memory round trips per group)
            BAEdgeGroup g;
            g.load(A, d, cur, le0, ee);
#pragma unroll
            for (int q = 0; q < BA_EG; q++) {
                if (!g.act[q]) continue;
                const int ge = d.e0 + le0 + q;
                nact++;
                const double* m = g.m[q];
                const gfse3::SE3& T = g.T[q];
                double pc[3], e0, e1;
                edge_error(m, T, X, pc, e0, e1);
                const double info = m[2];
                double rho0, rho1;
                huber(e0 * (info * e0) + e1 * (info * e1), rho0, rho1);
                chi += rho0;
                double Jp[2][3], Jc[2][6];
                edge_jac(m, T, pc, Jp, Jc, true);
                const double w = rho1 * info;
                const double o0 = -(info * e0) * rho1, o1 = -(info * e1) * rho1;
#pragma unroll
                for (int r = 0; r < 3; r++) {
                    b[r] += Jp[0][r] * o0 + Jp[1][r] * o1;
#pragma unroll
                    for (int c = 0; c < 3; c++) H[3 * r + c] += (Jp[0][r] * w) * Jp[0][c] + (Jp[1][r] * w) * Jp[1][c];
                }
                const int col = g.col[q];
                if (col >= 0) {  // Hpl = B^T W A, also the panel Ht[3 i + c][6 col + r]
                    double* hp = A.Hpl + (size_t)ge * 18;
                    double* Ht = A.panel + d.panel0;
#pragma unroll
                    for (int r = 0; r < 6; r++)
#pragma unroll
                        for (int c = 0; c < 3; c++) {
                            const double v = (Jc[0][r] * w) * Jp[0][c] + (Jc[1][r] * w) * Jp[1][c];
                            hp[3 * r + c] = v;
                            Ht[(size_t)(3 * i + c) * d.npad + 6 * col + r] = v;
                        }
                }
            }
        }
        double* Hg = A.Hll + (size_t)gp * 9;
        for (int k = 0; k < 9; k++) Hg[k] = H[k];
        for (int k = 0; k < 3; k++) A.bl[(size_t)gp * 3 + k] = b[k];
        A.pt_act[gp] = nact > 0;
        if (nact) maxd = fmax(fmax(fabs(H[0]), fabs(H[4])), fabs(H[8]));
    }
    const double cs = block_reduce(chi, sh, false);
    const double mx = block_reduce(maxd, sh, true);
    if (threadIdx.x == 0) {
        A.wg_chi[d.wg0 + blockIdx.x] = cs;
        A.wg_maxd[d.wg0 + blockIdx.x] = mx;
    }
}

// ------------------------------------------------------------------ buildSystem, pose half
constexpr int BA_PT = 256;  // threads per free pose (k_ba_poses)
__global__ __launch_bounds__(BA_PT) void k_ba_poses(BAArena A) {
    __shared__ double sacc[BA_PT / 64][28];
    const int p = blockIdx.y, a = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const BADesc d = A.desc[p];
    if (a >= d.nfree) return;
    const BAState st = A.st[p];
    if (st.round >= 2 || !st.need_lin || ba_halted(A, st)) return;
    const int cur = st.cur;
    const int kf = A.f_kf[d.f0 + a];
    const gfse3::SE3 T = load_T(A, cur, d.kf0 + kf);
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; k++) acc[k] = 0.0;
    int cnt = 0;
    const int j0 = A.f_eptr[d.fe0 + a], j1 = A.f_eptr[d.fe0 + a + 1];
    for (int jg = j0 + (int)threadIdx.x; jg < j1; jg += BA_PT * BA_EG) {
      // this thread's next BA_EG edges (j = jg, jg + BA_PT, ...): every load
      // of the group issued before the first edge's arithmetic
      bool use[BA_EG];
      double mq[BA_EG][8], Xq[BA_EG][3];
      {
        int ge[BA_EG], pt[BA_EG];
#pragma unroll
        for (int q = 0; q < BA_EG; q++) ge[q] = d.e0 + A.f_elist[d.pl0 + min(jg + q * BA_PT, j1 - 1)];
#pragma unroll
        for (int q = 0; q < BA_EG; q++) {
            const uint8_t a = A.e_act[ge[q]];
            use[q] = jg + q * BA_PT < j1 && a;
            pt[q] = A.e_pt[ge[q]];
#pragma unroll
            for (int k = 0; k < 8; k++) mq[q][k] = A.e_meas[(size_t)ge[q] * 8 + k];
        }
#pragma unroll
        for (int q = 0; q < BA_EG; q++) {
            const double* Xp = ptX_at(A, cur, d.pt0 + pt[q]);
#pragma unroll
            for (int k = 0; k < 3; k++) Xq[q][k] = Xp[k];
        }
      }
#pragma unroll
      for (int q = 0; q < BA_EG; q++) {
        if (!use[q]) continue;
        cnt++;
        const double* m = mq[q];
        const double* X = Xq[q];
        double pc[3], e0, e1;
        edge_error(m, T, X, pc, e0, e1);
        const double info = m[2];
        double rho0, rho1;
        huber(e0 * (info * e0) + e1 * (info * e1), rho0, rho1);
        double Jc[2][6];
        edge_jac(m, T, pc, nullptr, Jc, false);
        const double w = rho1 * info;
        const double o0 = -(info * e0) * rho1, o1 = -(info * e1) * rho1;
        int k = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
            for (int c = 0; c <= r; c++) acc[k++] += (Jc[0][r] * w) * Jc[0][c] + (Jc[1][r] * w) * Jc[1][c];
#pragma unroll
        for (int r = 0; r < 6; r++) acc[21 + r] += Jc[0][r] * o0 + Jc[1][r] * o1;
      }
    }
#pragma unroll
    for (int k = 0; k < 27; k++)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 64);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 27; k++) sacc[wv][k] = acc[k];
        sacc[wv][27] = (double)cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 27; k++) {
            double v = sacc[0][k];
            for (int q = 1; q < BA_PT / 64; q++) v += sacc[q][k];
            acc[k] = v;
        }
        cnt = 0;
        for (int q = 0; q < BA_PT / 64; q++) cnt += (int)sacc[q][27];
        double* H = A.Hpp + (size_t)(d.f0 + a) * 36;
        int k = 0;
        for (int r = 0; r < 6; r++)
            for (int c = 0; c <= r; c++, k++) H[6 * r + c] = H[6 * c + r] = acc[k];
        for (int r = 0; r < 6; r++) A.bp[(size_t)(d.f0 + a) * 6 + r] = acc[21 + r];
        A.f_act[d.f0 + a] = cnt > 0;
    }
}

// lambda of this trial: computeLambdaInit at the first trial of a round
// (max |diag| over the active poses and points), else the state's. Called by
// every thread of a workgroup (block_reduce inside).
__device__ double trial_lambda(const BAArena& A, const BADesc& d, const BAState& st, double* sh) {
    if (!(st.iter == 0 && st.q == 0)) return st.lambda;
    double m = 0.0;
    for (int w = threadIdx.x; w < d.nwg; w += blockDim.x) m = fmax(m, A.wg_maxd[d.wg0 + w]);
    for (int u = threadIdx.x; u < 6 * d.nfree; u += blockDim.x)
        if (A.f_act[d.f0 + u / 6]) m = fmax(m, fabs(A.Hpp[(size_t)(d.f0 + u / 6) * 36 + 7 * (u % 6)]));
    return 1e-5 * block_reduce(m, sh, true);
}

// ------------------------------------------------------------------ Schur, per edge
// One thread per edge: Dinv of its point (recomputed per edge; the same
// arithmetic as the point's own), W = Hpl Dinv into the panel Wt. The first
// active edge of a point also stores Dinv and writes db = Dinv b_l into Wt's
// column n.
__global__ __launch_bounds__(BA_T) void k_ba_schur_pts(BAArena A) {
    __shared__ double sh[BA_T / 64];
    const int p = blockIdx.y;
    const BADesc d = A.desc[p];
    if (blockIdx.x >= d.newg) return;
    const BAState st = A.st[p];
    if (st.round >= 2 || ba_halted(A, st)) return;
    const double lam = trial_lambda(A, d, st, sh);
    if (blockIdx.x == 0 && threadIdx.x == 0 && st.iter == 0 && st.q == 0) A.st[p].lambda = lam;
    const int e = blockIdx.x * BA_T + threadIdx.x;
    if (e >= d.nedges) return;
    const int ge = d.e0 + e;
    if (!A.e_act[ge]) return;
    const int i = A.e_pt[ge], gp = d.pt0 + i;
    const int col = A.kf_col[d.kf0 + A.e_kf[ge]];
    int earlier = 0;  // an active edge of this point before e (independent loads, no early exit)
#pragma unroll 8
    for (int le = A.pt_eb[gp]; le < e; le++) earlier |= A.e_act[d.e0 + le];
    const bool first = !earlier;
    if (col < 0 && !first) return;
    double D[9], Di[9];
    const double* Hg = A.Hll + (size_t)gp * 9;
#pragma unroll
    for (int k = 0; k < 9; k++) D[k] = Hg[k] + (k % 4 == 0 ? lam : 0.0);
    inverse3(D, Di);
    double* Wt = A.panel + d.panel0 + (size_t)d.K * d.npad;
    if (first) {
#pragma unroll
        for (int k = 0; k < 9; k++) A.Dinv[(size_t)gp * 9 + k] = Di[k];
        const double* b = A.bl + (size_t)gp * 3;
#pragma unroll
        for (int r = 0; r < 3; r++)
            Wt[(size_t)(3 * i + r) * d.npad + d.n] = (Di[3 * r] * b[0] + Di[3 * r + 1] * b[1]) + Di[3 * r + 2] * b[2];
    }
    if (col < 0) return;
    const double* H = A.Hpl + (size_t)ge * 18;
    double h[18];
#pragma unroll
    for (int k = 0; k < 18; k++) h[k] = H[k];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int r = 0; r < 6; r++)
            Wt[(size_t)(3 * i + c) * d.npad + 6 * col + r] =
                (h[3 * r] * Di[c] + h[3 * r + 1] * Di[3 + c]) + h[3 * r + 2] * Di[6 + c];
}

// ------------------------------------------------------------------ Schur product on MFMA
// C[i][j] = sum_k Ht[k][i] Wt[k][j] over the lower-triangle 16x16 tiles of the
// reduced camera system plus the tiles of column n (the coefficient vector).
// Workgroup = (split, problem), 8 waves; wave w owns tiles w + 8u (u < 16)
// with their accumulators in registers. The split's panel rows stream through
// LDS in chunks of BA_GCH k-steps (4 rows each, both panels, full width,
// 16-byte loads); a k-step issues the MFMA of tile (ti, tj) only when its
// column-tile mask has ti (Ht) and tj (Wt): the panels are block sparse (a
// map point is seen by a few keyframes) and the mask comes from the graph
// structure (host, gf_ba_plan_create).
constexpr int BA_GCH = 8;
constexpr int BA_GW = 8;    // waves per GEMM workgroup
constexpr int BA_GTPW = 16; // tiles per wave
__global__ __launch_bounds__(64 * BA_GW) void k_ba_gemm(BAArena A) {
    extern __shared__ __align__(16) double gs[];
    __shared__ uint16_t smask[BA_GCH];
    const int p = blockIdx.y, s = blockIdx.x;
    const BADesc d = A.desc[p];
    if (s >= d.nsplit) return;
    if (A.st[p].round >= 2 || ba_halted(A, A.st[p])) return;
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int nt = d.npad >> 4, lower = nt * (nt + 1) / 2, tdb = d.n >> 4;
    const int ld = d.npad + 2;  // padded LDS row: the 4 k-rows of an operand fall in different banks
    double* sa = gs;
    double* sw = gs + BA_GCH * 4 * ld;
    const double* Ht = A.panel + d.panel0;
    const double* Wt = Ht + (size_t)d.K * d.npad;
    const uint16_t* km = A.kmask + d.mask0;
    const int kr = l >> 4, cl = l & 15;
    int ti[BA_GTPW], tj[BA_GTPW];
#pragma unroll
    for (int u = 0; u < BA_GTPW; u++) {
        const int t = w + BA_GW * u;
        if (t >= d.ntiles) {
            ti[u] = tj[u] = -1;
        } else if (t < lower) {
            int a = 0;
            while ((a + 1) * (a + 2) / 2 <= t) a++;
            ti[u] = a;
            tj[u] = t - a * (a + 1) / 2;
        } else {
            ti[u] = t - lower;
            tj[u] = tdb;
        }
    }
    d4 acc[BA_GTPW];
#pragma unroll
    for (int u = 0; u < BA_GTPW; u++) acc[u] = (d4){0.0, 0.0, 0.0, 0.0};
    const int j0 = s * d.sps, j1 = j0 + d.sps, half = d.npad >> 1;
    for (int c0 = j0; c0 < j1; c0 += BA_GCH) {
        const int nstep = min(BA_GCH, j1 - c0), nrow = 4 * nstep;
        if (threadIdx.x < nstep) smask[threadIdx.x] = km[c0 + threadIdx.x];
        for (int q = threadIdx.x; q < nrow * half; q += 64 * BA_GW) {
            const int r = q / half, c2 = 2 * (q - r * half);
            const size_t g = (size_t)(4 * c0 + r) * d.npad + c2;
            const double2 va = *(const double2*)(Ht + g), vw = *(const double2*)(Wt + g);
            sa[r * ld + c2] = va.x;
            sa[r * ld + c2 + 1] = va.y;
            sw[r * ld + c2] = vw.x;
            sw[r * ld + c2 + 1] = vw.y;
        }
        __syncthreads();
        for (int js = 0; js < nstep; js++) {
            const unsigned ma = smask[js], mb = ma | (1u << tdb);
            if (!ma) continue;
            const double* ra = sa + (4 * js + kr) * ld + cl;
            const double* rw = sw + (4 * js + kr) * ld + cl;
#pragma unroll
            for (int u = 0; u < BA_GTPW; u++) {
                if (ti[u] >= 0 && ((ma >> ti[u]) & (mb >> tj[u]) & 1u))
                    acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ra[16 * ti[u]], rw[16 * tj[u]], acc[u], 0, 0, 0);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < BA_GTPW; u++) {
        if (ti[u] < 0) continue;
        double* out = A.tiles + ((size_t)d.tile0 + (size_t)s * d.ntiles + w + BA_GW * u) * 256;
#pragma unroll
        for (int r = 0; r < 4; r++)  // f64 16x16x4 C/D: col = lane & 15, row = (lane >> 4) + 4 r
            out[(kr + 4 * r) * 16 + cl] = acc[u][r];
    }
}

size_t ba_gemm_lds(int npad) { return sizeof(double) * 2 * BA_GCH * 4 * (npad + 2); }

// The same product as a task list: one wave per item = one output tile over
// a run of the k-steps where both its operand tiles are nonzero (listed on the
// host from the graph structure), operands read straight from the panels
// (16 consecutive doubles per row, 4 rows per MFMA), the tile's partial sum
// written per item and reduced in item order (k_ba_gemm_reduce). No k-step
// that contributes nothing is visited, and no mask test runs per tile.
constexpr int BA_SW = 4;   // waves (items) per workgroup
constexpr int BA_KCH = 16; // k-steps per item at most
__global__ __launch_bounds__(64 * BA_SW) void k_ba_spgemm(BAArena A) {
    const int p = blockIdx.y;
    const BADesc d = A.desc[p];
    const int it = blockIdx.x * BA_SW + (threadIdx.x >> 6);
    if (it >= d.nitems) return;
    if (A.st[p].round >= 2 || ba_halted(A, A.st[p])) return;
    const int4 item = A.items[d.item0 + it];
    const int l = threadIdx.x & 63, kr = l >> 4, cl = l & 15;
    const double* Ht = A.panel + d.panel0;
    const double* Wt = Ht + (size_t)d.K * d.npad;
    const int32_t* kl = A.klist + d.kl0;
    const int ca = 16 * item.x + cl, cw = 16 * item.y + cl;
    // every k-step's operands in flight at once (an item holds at most
    // BA_KCH k-steps), then the MFMA chain
    // (loads at clamped k-steps, unconditional: a load behind a branch has its
    // result merged before the next one issues, one round trip per k-step)
    double a[BA_KCH], w[BA_KCH];
    int ks[BA_KCH];
#pragma unroll
    for (int u = 0; u < BA_KCH; u++) ks[u] = kl[min(item.z + u, item.w - 1)];
#pragma unroll
    for (int u = 0; u < BA_KCH; u++) {
        const size_t r = (size_t)(4 * ks[u] + kr) * d.npad;
        a[u] = Ht[r + ca];
        w[u] = Wt[r + cw];
    }
    d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int u = 0; u < BA_KCH; u++)
        if (item.z + u < item.w) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], w[u], acc, 0, 0, 0);
    double* out = A.tiles + ((size_t)d.item0 + it) * 256;
#pragma unroll
    for (int r = 0; r < 4; r++) out[(kr + 4 * r) * 16 + cl] = acc[r];
}

__device__ __forceinline__ int tri(int i) { return i * (i + 1) / 2; }

// Item sums in item order: Ssum = [S lower packed (n(n+1)/2) | column n (n)].
__global__ __launch_bounds__(256) void k_ba_gemm_reduce(BAArena A) {
    const int p = blockIdx.y;
    const BADesc d = A.desc[p];
    const int n = d.n, npk = tri(n);
    const int u = blockIdx.x * 256 + threadIdx.x;
    if (u >= npk + n) return;
    if (A.st[p].round >= 2 || ba_halted(A, A.st[p])) return;
    int t, e;
    if (u < npk) {
        int i = (int)((sqrt(8.0 * u + 1.0) - 1.0) * 0.5);
        while (tri(i) > u) i--;
        while (tri(i + 1) <= u) i++;
        const int j = u - tri(i);
        t = tri(i >> 4) + (j >> 4);
        e = (i & 15) * 16 + (j & 15);
    } else {
        const int i = u - npk, ti = i >> 4, tdb = n >> 4, nt = d.npad >> 4;
        t = ti >= tdb ? tri(ti) + tdb : nt * (nt + 1) / 2 + ti;
        e = (i & 15) * 16 + (n & 15);
    }
    double g = 0.0;
    if (d.nitems < 0) {  // dense split-K GEMM (large batches): split sums in split order
        const double* tiles = A.tiles + (size_t)d.tile0 * 256;
        for (int s = 0; s < d.nsplit; s++) g += tiles[((size_t)s * d.ntiles + t) * 256 + e];
        A.Ssum[(size_t)d.ss0 + u] = g;
        return;
    }
    const double* part = A.tiles + (size_t)d.item0 * 256;
    const int32_t* tp = A.tile_iptr + d.tip0;
    // item order, adds in sequence; loads BA_RB at a time (independent, a
    // tile has ~90 items at config 4, so three round trips instead of twelve)
    constexpr int BA_RB = 32;
    const int i0 = tp[t], i1 = tp[t + 1];
    for (int it = i0; it < i1; it += BA_RB) {
        double v[BA_RB];
#pragma unroll
        for (int q = 0; q < BA_RB; q++) v[q] = it + q < i1 ? part[(size_t)(it + q) * 256 + e] : 0.0;
#pragma unroll
        for (int q = 0; q < BA_RB; q++)
            if (it + q < i1) g += v[q];
    }
    A.Ssum[(size_t)d.ss0 + u] = g;
}

// ------------------------------------------------------------------ reduced camera system
// S = Hpp + lambda I - C (lower, packed in LDS), b_s = b_p - C[:, n]; inactive
// poses decouple with x = 0. Blocked LL^T with one 6x6 block per pose (two
// barriers per pose), substitutions one pose block at a time on one wave —
// all in the oracle's operation order (see below).
#ifndef BA_SOLVE_THREADS
#define BA_SOLVE_THREADS 1024
#endif
constexpr int BA_ST = BA_SOLVE_THREADS;
static_assert(BA_ST >= BA_MAXN && BA_ST % 64 == 0, "k_ba_solve: one thread per panel row");

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long u = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffLL), l);
    const int hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ __launch_bounds__(BA_ST) void k_ba_solve(BAArena A) {
    __shared__ double sL[BA_MAXN * (BA_MAXN + 1) / 2];
    __shared__ double sb[BA_MAXN], sbp[BA_MAXN], srinv[BA_MAXN];
    __shared__ uint8_t sact[BA_MAXFREE];
#ifdef BA_SUBST_BLOCK
    __shared__ double scol6[6];
#endif
    __shared__ int s_fail;
    const int p = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const BADesc d = A.desc[p];
    const BAState st = A.st[p];
    if (st.round >= 2 || ba_halted(A, st)) return;
#define BA_STAMP(k)                                                                      \
    if (A.tstamp && tid == 0) A.tstamp[(size_t)p * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
    BA_STAMP(0);
    const int n = d.n, npk = tri(n);
    const double lam = st.lambda;
    for (int a = tid; a < d.nfree; a += BA_ST) sact[a] = A.f_act[d.f0 + a];
    __syncthreads();
    const double* Sg = A.Ssum + d.ss0;
    // a wave's rows i = w, w + 16, ..., four at a time with their <= 3 column
    // chunks: the batch's Sg / Hpp values loaded (clamped, unconditional)
    // before any is used, one round trip per batch instead of one per chunk
    constexpr int RB = 4, CPR = (BA_MAXN + 63) / 64;
    for (int i0 = w; i0 < n; i0 += RB * (BA_ST / 64)) {
        double sgv[RB][CPR], hpv[RB][CPR];
#pragma unroll
        for (int ri = 0; ri < RB; ri++) {
            const int i = min(i0 + ri * (BA_ST / 64), n - 1), a = i / 6;
#pragma unroll
            for (int cj = 0; cj < CPR; cj++) {
                const int j = min(lane + 64 * cj, i);
                sgv[ri][cj] = Sg[tri(i) + j];
                const int jc = min(max(j, 6 * a), 6 * a + 5);  // a column of i's own pose block
                hpv[ri][cj] = A.Hpp[(size_t)(d.f0 + a) * 36 + (i % 6) * 6 + (jc % 6)];
            }
        }
#pragma unroll
        for (int ri = 0; ri < RB; ri++) {
            const int i = i0 + ri * (BA_ST / 64);
            if (i >= n) break;
            const int a = i / 6;
#pragma unroll
            for (int cj = 0; cj < CPR; cj++) {
                const int j = lane + 64 * cj;
                if (j > i) break;
                const int c = j / 6;
                double v;
                if (!sact[a] || !sact[c]) {
                    v = (i == j) ? 1.0 : 0.0;
                } else {
                    v = 0.0;
                    if (a == c) v = hpv[ri][cj] + (i == j ? lam : 0.0);
                    v = v - sgv[ri][cj];
                }
                sL[tri(i) + j] = v;
            }
        }
    }
    for (int i = tid; i < n; i += BA_ST) {
        const double bpi = A.bp[(size_t)d.f0 * 6 + i];
        sbp[i] = bpi;
        sb[i] = sact[i / 6] ? bpi - Sg[npk + i] : 0.0;
    }
    __syncthreads();
    BA_STAMP(1);
    // Blocked LL^T, one 6x6 block per pose, in place on the packed lower
    // triangle: per block column, (1) the diagonal block factored in registers
    // by the waves that own panel rows (every lane the same values), (2) the
    // panel rows below by one thread each, (3) the trailing update by the
    // whole workgroup. Every element still sees its subtractions
    // L_ik L_jk one at a time in ascending k and a product rounded before
    // it is subtracted, so the factor is bit for bit the oracle's left-looking
    // LL^T (oracle/lba.cpp) — with 2 barriers per pose instead of one per
    // column. On exit sL holds L (scaled, j < i) and d_j on the diagonal,
    // srinv[j] = 1 / d_j.
    if (tid == 0) s_fail = 0;
    __syncthreads();
#ifdef BA_CHOL_PHASES  // diagnostic: s_memtime cycles of (diagonal + panel) and (trailing update) summed over the block steps
    unsigned long long ph_a = 0, ph_b = 0, ph_t = __builtin_amdgcn_s_memtime();
#endif
    for (int k0 = 0; k0 < n; k0 += 6) {
        const int nrow = n - k0 - 6;  // panel rows below the block
        double Db[6][6], rb[6];
        bool ok = true;
        if (tid < ((nrow + 63) & ~63) || (nrow == 0 && tid < 64)) {
#pragma unroll
            for (int c = 0; c < 6; c++) {
                double sv = sL[tri(k0 + c) + k0 + c];
#pragma unroll
                for (int m = 0; m < c; m++) sv = sv - Db[c][m] * Db[c][m];
                ok = ok && sv > 0.0;
                const double dj = sqrt(sv);
                Db[c][c] = dj;
                rb[c] = 1.0 / dj;
#pragma unroll
                for (int a2 = c + 1; a2 < 6; a2++) {
                    double t = sL[tri(k0 + a2) + k0 + c];
#pragma unroll
                    for (int m = 0; m < c; m++) t = t - Db[a2][m] * Db[c][m];
                    Db[a2][c] = t * rb[c];
                }
            }
            if (tid < nrow) {  // panel row i = k0 + 6 + tid
                const int i = k0 + 6 + tid;
                double P[6];
#pragma unroll
                for (int c = 0; c < 6; c++) {
                    double t = sL[tri(i) + k0 + c];
#pragma unroll
                    for (int m = 0; m < c; m++) t = t - P[m] * Db[c][m];
                    P[c] = t * rb[c];
                }
#pragma unroll
                for (int c = 0; c < 6; c++) sL[tri(i) + k0 + c] = P[c];
            }
        }
        __syncthreads();
#ifdef BA_CHOL_PHASES
        { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph_a += t - ph_t; ph_t = t; }
#endif
        if (tid == 0) {  // the block's factor (no one reads these rows before the substitutions)
            if (!ok) s_fail = 1;
#pragma unroll
            for (int c = 0; c < 6; c++) {
                srinv[k0 + c] = rb[c];
#pragma unroll
                for (int a2 = c; a2 < 6; a2++) sL[tri(k0 + a2) + k0 + c] = Db[a2][c];
            }
        }
        // trailing update: R_ij -= L_i,k0+m L_j,k0+m, m = 0..5, for k0+6 <= j <= i.
        // Lane l of every wave keeps the panel rows j = k0 + 6 + l + 64 q in
        // registers; wave w takes rows i = k0 + 6 + w, + 16, ... and reads
        // each row's six panel values once (a broadcast), so an element costs
        // one LDS read and one write instead of thirteen accesses.
        {
            double Lj[(BA_MAXN + 63) / 64][6];
#pragma unroll
            for (int q = 0; q < (BA_MAXN + 63) / 64; q++) {
                const int j = k0 + 6 + lane + 64 * q;
#pragma unroll
                for (int m = 0; m < 6; m++) Lj[q][m] = j < n ? sL[tri(j) + k0 + m] : 0.0;
            }
            for (int ii = w; ii < nrow; ii += BA_ST / 64) {
                const int i = k0 + 6 + ii;
                double Li[6];
#pragma unroll
                for (int m = 0; m < 6; m++) Li[m] = sL[tri(i) + k0 + m];
#pragma unroll
                for (int q = 0; q < (BA_MAXN + 63) / 64; q++) {
                    const int jj = lane + 64 * q;
                    if (jj <= ii) {
                        const int j = k0 + 6 + jj;
                        double Rv = sL[tri(i) + j];
#pragma unroll
                        for (int m = 0; m < 6; m++) Rv = Rv - Li[m] * Lj[q][m];
                        sL[tri(i) + j] = Rv;
                    }
                }
            }
        }
        __syncthreads();
#ifdef BA_CHOL_PHASES
        { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph_b += t - ph_t; ph_t = t; }
#endif
        if (s_fail) break;
    }
    const bool fail = s_fail;
    __syncthreads();
    BA_STAMP(2);
#ifdef BA_CHOL_PHASES
    if (A.tstamp && tid == 0) {
        A.tstamp[(size_t)p * 8 + 5] = ph_a;
        A.tstamp[(size_t)p * 8 + 6] = ph_b;
    }
#else
    if (A.tstamp && tid == 0) A.tstamp[(size_t)p * 8 + 5] = __builtin_amdgcn_s_memtime();
#endif
#ifndef BA_SUBST_BLOCK
    if (!fail && w == 0) {
        // Substitutions on one wave, one unknown per step: lane l holds rows
        // l, l + 64, l + 128 in registers. Step k takes y_k = r_k / d_k from
        // its owner lane (the product with 1 / d_k, then two lane reads), and
        // every row still open subtracts its one term: the forward pass in
        // ascending k (L_ik from row i), the backward pass in descending k
        // (L_ki from row k, a contiguous run of the packed triangle). Each
        // row sees its terms in the oracle's order, so x is the same bits as
        // the block-wise form (BA_SUBST_BLOCK). The L values of 8 steps are
        // loaded together (one wait per 8 steps), and the steps of one
        // owner slot (k in [64 uk, 64 uk + 64)) are a loop of their own, so
        // the owner's register and the rows a step touches are known at
        // compile time: the step's chain is a product, two lane reads, a
        // product and a difference.
        constexpr int SC = 8;
        double r[3], ri[3];
#pragma unroll
        for (int u = 0; u < 3; u++) {
            const int i = lane + 64 * u;
            r[u] = i < n ? sb[i] : 0.0;
            ri[u] = i < n ? srinv[i] : 0.0;
        }
        // forward: SC steps at a time while a whole chunk fits, then single steps
        auto fwd = [&](auto ukc, auto scc, int k0) {
            constexpr int uk = decltype(ukc)::value, S = decltype(scc)::value;
            double Lb[3][S];
#pragma unroll
            for (int u = uk; u < 3; u++) {
                const int i = min(lane + 64 * u, n - 1), base = tri(i);
#pragma unroll
                for (int s2 = 0; s2 < S; s2++) Lb[u][s2] = sL[base + min(k0 + s2, i)];
            }
#pragma unroll
            for (int s2 = 0; s2 < S; s2++) {
                const int k = k0 + s2;
                const double yk = readlane_d(r[uk] * ri[uk], k & 63);
                {
                    const int i = lane + 64 * uk;
                    const double t = r[uk] - Lb[uk][s2] * yk;
                    r[uk] = i > k ? t : (i == k ? yk : r[uk]);
                }
#pragma unroll
                for (int u = uk + 1; u < 3; u++) r[u] = r[u] - Lb[u][s2] * yk;
            }
        };
        auto fwd_seg = [&](auto ukc) {
            constexpr int uk = decltype(ukc)::value;
            const int ke = min(n, 64 * uk + 64);
            int k0 = 64 * uk;
            for (; k0 + SC <= ke; k0 += SC) fwd(ukc, std::integral_constant<int, SC>{}, k0);
            for (; k0 < ke; k0++) fwd(ukc, std::integral_constant<int, 1>{}, k0);
        };
        fwd_seg(std::integral_constant<int, 0>{});
        fwd_seg(std::integral_constant<int, 1>{});
        fwd_seg(std::integral_constant<int, 2>{});
        // backward, the same shape in descending k
        auto bwd = [&](auto ukc, auto scc, int k1) {
            constexpr int uk = decltype(ukc)::value, S = decltype(scc)::value;
            double Lb[3][S];
#pragma unroll
            for (int s2 = 0; s2 < S; s2++) {
                const int base = tri(k1 - s2);
#pragma unroll
                for (int u = 0; u <= uk; u++) Lb[u][s2] = sL[base + min(lane + 64 * u, k1 - s2)];
            }
#pragma unroll
            for (int s2 = 0; s2 < S; s2++) {
                const int k = k1 - s2;
                const double xk = readlane_d(r[uk] * ri[uk], k & 63);
                {
                    const int i = lane + 64 * uk;
                    const double t = r[uk] - Lb[uk][s2] * xk;
                    r[uk] = i < k ? t : (i == k ? xk : r[uk]);
                }
#pragma unroll
                for (int u = 0; u < uk; u++) r[u] = r[u] - Lb[u][s2] * xk;
            }
        };
        auto bwd_seg = [&](auto ukc) {
            constexpr int uk = decltype(ukc)::value;
            const int kb = 64 * uk;
            int k1 = min(n, 64 * uk + 64) - 1;
            for (; k1 - SC + 1 >= kb; k1 -= SC) bwd(ukc, std::integral_constant<int, SC>{}, k1);
            for (; k1 >= kb; k1--) bwd(ukc, std::integral_constant<int, 1>{}, k1);
        };
        bwd_seg(std::integral_constant<int, 2>{});
        bwd_seg(std::integral_constant<int, 1>{});
        bwd_seg(std::integral_constant<int, 0>{});
#pragma unroll
        for (int u = 0; u < 3; u++)
            if (lane + 64 * u < n) sb[lane + 64 * u] = r[u];
    }
#else
    if (!fail && w == 0) {
        // Substitutions on one wave, one pose block at a time: lane l holds
        // rows l, l + 64, l + 128 in registers; a block's 6 values go through
        // LDS (srow) and are solved redundantly on
        // every lane, then every row outside the block subtracts the block's
        // 6 terms in the oracle's order (forward: ascending k; backward:
        // descending k).
        double* srow = scol6;
        double r[3];
        for (int u = 0; u < 3; u++) r[u] = (lane + 64 * u < n) ? sb[lane + 64 * u] : 0.0;
        for (int k0 = 0; k0 < n; k0 += 6) {
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int i = lane + 64 * u;
                if (i >= k0 && i < k0 + 6) srow[i - k0] = r[u];
            }
            wave_lds_sync();
            double y[6];
#pragma unroll
            for (int c = 0; c < 6; c++) {
                double sv = srow[c];
#pragma unroll
                for (int m = 0; m < c; m++) sv = sv - sL[tri(k0 + c) + k0 + m] * y[m];
                y[c] = sv * srinv[k0 + c];
            }
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int i = lane + 64 * u;
                if (i >= k0 && i < k0 + 6) {
#pragma unroll
                    for (int c = 0; c < 6; c++)
                        if (i == k0 + c) r[u] = y[c];
                } else if (i >= k0 + 6 && i < n) {
                    double t = r[u];
#pragma unroll
                    for (int m = 0; m < 6; m++) t = t - sL[tri(i) + k0 + m] * y[m];
                    r[u] = t;
                }
            }
            wave_lds_sync();
        }
        for (int k0 = n - 6; k0 >= 0; k0 -= 6) {
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int i = lane + 64 * u;
                if (i >= k0 && i < k0 + 6) srow[i - k0] = r[u];
            }
            wave_lds_sync();
            double x[6];
#pragma unroll
            for (int c = 5; c >= 0; c--) {
                double sv = srow[c];
#pragma unroll
                for (int m = 5; m > c; m--) sv = sv - sL[tri(k0 + m) + k0 + c] * x[m];
                x[c] = sv * srinv[k0 + c];
            }
#pragma unroll
            for (int u = 0; u < 3; u++) {
                const int i = lane + 64 * u;
                if (i >= k0 && i < k0 + 6) {
#pragma unroll
                    for (int c = 0; c < 6; c++)
                        if (i == k0 + c) r[u] = x[c];
                } else if (i < k0) {
                    double t = r[u];
#pragma unroll
                    for (int m = 5; m >= 0; m--) t = t - sL[tri(k0 + m) + i] * x[m];
                    r[u] = t;
                }
            }
            wave_lds_sync();
        }
#pragma unroll
        for (int u = 0; u < 3; u++)
            if (lane + 64 * u < n) sb[lane + 64 * u] = r[u];
    }
#endif
    __syncthreads();
    BA_STAMP(3);
#ifndef BA_CHOL_PHASES
    if (A.tstamp && tid == 0) A.tstamp[(size_t)p * 8 + 6] = __builtin_amdgcn_s_memtime();
#endif
    if (fail) {  // Solver::_x keeps its previous value
        for (int i = tid; i < n; i += BA_ST) sb[i] = A.xp[(size_t)d.f0 * 6 + i];
    } else {
        for (int i = tid; i < n; i += BA_ST) A.xp[(size_t)d.f0 * 6 + i] = sb[i];
    }
    __syncthreads();
    // trial poses: exp(x) * T for the active free poses
    const int cur = st.cur;
    for (int k = tid; k < d.nkf; k += BA_ST) {
        gfse3::SE3 T = load_T(A, cur, d.kf0 + k);
        const int col = A.kf_col[d.kf0 + k];
        if (col >= 0 && sact[col]) {
            double x6[6];
            for (int r = 0; r < 6; r++) x6[r] = sb[6 * col + r];
            T = gfse3::exp_mul(x6, T);
        }
        store_T(A, 1 - cur, d.kf0 + k, T);
    }
    if (tid == 0) {  // computeScale, pose part (index order)
        double sc = 0.0;
        for (int i = 0; i < n; i++) sc += sb[i] * (lam * sb[i] + sbp[i]);
        A.st[p].scale_p = sc;
        A.st[p].chol_ok = fail ? 0 : 1;
    }
    BA_STAMP(4);
#undef BA_STAMP
}

// ------------------------------------------------------------------ landmarks, trial errors
__global__ __launch_bounds__(BA_T) void k_ba_update(BAArena A) {
    __shared__ double sh[BA_T / 64];
    const int p = blockIdx.y;
    const BADesc d = A.desc[p];
    if (blockIdx.x >= d.nwg) return;
    const BAState st = A.st[p];
    if (st.round >= 2 || ba_halted(A, st)) return;
    const int i = blockIdx.x * BA_T + threadIdx.x;
    double chi = 0.0, sc = 0.0;
    if (i < d.npts) {
        const int gp = d.pt0 + i, cur = st.cur, nxt = 1 - st.cur;
        const double lam = st.lambda;
        const double* Xc = ptX_at(A, cur, gp);
        double X[3] = {Xc[0], Xc[1], Xc[2]};
        const int eb = A.pt_eb[gp], ee = A.pt_ee[gp];
        if (A.pt_act[gp]) {
            double* xl = A.xl + (size_t)gp * 3;
            const double* b = A.bl + (size_t)gp * 3;
            if (st.chol_ok) {  // cl = b_l + Hpl^T (-x_p), x_l = Dinv cl
                double cl[3] = {b[0], b[1], b[2]};
                for (int le0 = eb; le0 < ee; le0 += BA_EG) {  // groups of edges, loads first (BAEdgeGroup)
                    bool use[BA_EG];
                    int col[BA_EG];
                    double H[BA_EG][18], xa[BA_EG][6];
#pragma unroll
                    for (int q = 0; q < BA_EG; q++) {
                        const int ge = d.e0 + min(le0 + q, ee - 1);
                        const uint8_t a = A.e_act[ge];
                        col[q] = A.kf_col[d.kf0 + A.e_kf[ge]];
                        use[q] = le0 + q < ee && a && col[q] >= 0;
#pragma unroll
                        for (int k = 0; k < 18; k++) H[q][k] = A.Hpl[(size_t)ge * 18 + k];
                    }
#pragma unroll
                    for (int q = 0; q < BA_EG; q++)
#pragma unroll
                        for (int k = 0; k < 6; k++) xa[q][k] = A.xp[(size_t)(d.f0 + max(col[q], 0)) * 6 + k];
#pragma unroll
                    for (int q = 0; q < BA_EG; q++) {
                        if (!use[q]) continue;
                        for (int c = 0; c < 3; c++) {
                            double t = H[q][c] * (-xa[q][0]);
                            for (int r = 1; r < 6; r++) t += H[q][3 * r + c] * (-xa[q][r]);
                            cl[c] += t;
                        }
                    }
                }
                const double* Di = A.Dinv + (size_t)gp * 9;
                for (int r = 0; r < 3; r++) xl[r] = (Di[3 * r] * cl[0] + Di[3 * r + 1] * cl[1]) + Di[3 * r + 2] * cl[2];
            }
            for (int c = 0; c < 3; c++) {
                X[c] += xl[c];
                sc += xl[c] * (lam * xl[c] + b[c]);
            }
        }
        double* Xn = ptX_at(A, nxt, gp);
        Xn[0] = X[0];
        Xn[1] = X[1];
        Xn[2] = X[2];
        for (int le0 = eb; le0 < ee; le0 += BA_EG) {  // errors at the trial estimate
            BAEdgeGroup g;
            g.load(A, d, nxt, le0, ee);
#pragma unroll
            for (int q = 0; q < BA_EG; q++) {
                if (!g.act[q]) continue;
                const int ge = d.e0 + le0 + q;
                const double* m = g.m[q];
                double pc[3], e0, e1;
                edge_error(m, g.T[q], X, pc, e0, e1);
                A.e_err[(size_t)ge * 2] = e0;
                A.e_err[(size_t)ge * 2 + 1] = e1;
                const double info = m[2];
                double rho0, rho1;
                huber(e0 * (info * e0) + e1 * (info * e1), rho0, rho1);
                chi += rho0;
            }
        }
    }
    const double cs = block_reduce(chi, sh, false);
    const double ss = block_reduce(sc, sh, false);
    if (threadIdx.x == 0) {
        A.wg_chi_t[d.wg0 + blockIdx.x] = cs;
        A.wg_scale[d.wg0 + blockIdx.x] = ss;
    }
}

// ------------------------------------------------------------------ LM decision + outlier pass
__global__ __launch_bounds__(1024) void k_ba_decide(BAArena A) {
    __shared__ int s_end, s_cnt;
    __shared__ double s_part[3][BA_MAXPTS / BA_T];
    __shared__ double s_sum[3];
    const int p = blockIdx.x, tid = threadIdx.x;
    const BADesc d = A.desc[p];
    if (A.st[p].round >= 2) return;
    for (int w = tid; w < d.nwg; w += 1024) {  // partial sums staged in LDS, summed in order by one thread
        s_part[0][w] = A.wg_chi[d.wg0 + w];
        s_part[1][w] = A.wg_chi_t[d.wg0 + w];
        s_part[2][w] = A.wg_scale[d.wg0 + w];
    }
    __syncthreads();
    // the three ordered sums on three threads at once (each in workgroup order,
    // the pose part of the scale first, as one thread summed them before)
    if (tid < 3) {
        double c = tid == 2 ? A.st[p].scale_p : 0.0;
#pragma unroll 8
        for (int w = 0; w < d.nwg; w++) c += s_part[tid][w];
        s_sum[tid] = c;
    }
    __syncthreads();
    if (tid == 0 && ba_halted(A, A.st[p])) {  // terminate() before this iteration: optimize() returns
        s_end = 1;
        s_cnt = 0;
    } else if (tid == 0) {
        BAState st = A.st[p];
        if (st.q == 0) {  // activeRobustChi2 at the iteration start
            st.currentChi = s_sum[0];
            st.iniChi = s_sum[0];
        }
        double tempChi = s_sum[1];
        if (!st.chol_ok) tempChi = DBL_MAX;
        double scale = s_sum[2];
        scale += 1e-3;
        const double rho = (st.currentChi - tempChi) / scale;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3.0);
            alpha = fmin(alpha, 2. / 3.);
            const double sf = fmax(1. / 3., alpha);
            st.lambda *= sf;
            st.ni = 2;
            st.currentChi = tempChi;
            st.cur ^= 1;  // the trial estimate becomes the current one
        } else {
            st.lambda *= st.ni;
            st.ni *= 2;
        }
        st.q++;
        int end = 0;
        if (rho < 0 && st.q < 10 && !(A.stop && *A.stop)) {  // the trial loop also ends on terminate()
            st.need_lin = 0;  // another trial on the same system
        } else {
            if (st.round == 0)  // (fixed indices: a run-time one puts st in scratch memory)
                st.iters[0]++;
            else
                st.iters[1]++;
            bool term = (st.q == 10 || rho == 0) || (A.stop && *A.stop);
            if (!term) {
                if ((st.iniChi - st.currentChi) * 1e3 < st.iniChi)
                    st.nbad++;
                else
                    st.nbad = 0;
                term = st.nbad >= 3;
            }
            st.iter++;
            if (term || st.iter >= (st.round == 0 ? 5 : 10)) {
                end = 1;
            } else {
                st.need_lin = 1;
                st.q = 0;
            }
        }
        A.st[p] = st;
        s_end = end;
        s_cnt = 0;
    }
    __syncthreads();
    if (!s_end) return;
    const BAState st = A.st[p];
    const int round = st.round, cur = st.cur;
    double* Ht = A.panel + d.panel0;
    double* Wt = Ht + (size_t)d.K * d.npad;
    int cnt = 0;
    for (int e = tid; e < d.nedges; e += 1024) {
        const int ge = d.e0 + e;
        if (!A.e_act[ge]) continue;
        const double* m = A.e_meas + (size_t)ge * 8;
        const double e0 = A.e_err[(size_t)ge * 2], e1 = A.e_err[(size_t)ge * 2 + 1], info = m[2];
        const int pt = A.e_pt[ge], kf = A.e_kf[ge];
        const double* Xp = ptX_at(A, cur, d.pt0 + pt);
        const double X[3] = {Xp[0], Xp[1], Xp[2]};
        double pc[3];
        gfse3::map(load_T(A, cur, d.kf0 + kf), X, pc);
        if (e0 * (info * e0) + e1 * (info * e1) > 5.991 || !(pc[2] > 0.0)) {
            A.e_out[ge] = (uint8_t)(round + 1);
            if (round == 0) {  // removeEdge: out of the structure of optimize(10)
                A.e_act[ge] = 0;
                const int col = A.kf_col[d.kf0 + kf];
                if (col >= 0)
                    for (int c = 0; c < 3; c++)
                        for (int r = 0; r < 6; r++) {
                            Ht[(size_t)(3 * pt + c) * d.npad + 6 * col + r] = 0.0;
                            Wt[(size_t)(3 * pt + c) * d.npad + 6 * col + r] = 0.0;
                        }
                continue;
            }
        }
        cnt++;
    }
    for (int i = tid; i < 3 * d.npts; i += 1024) Wt[(size_t)i * d.npad + d.n] = 0.0;  // db column of dropped points
    for (int i = tid; i < 6 * d.nfree; i += 1024) A.xp[(size_t)d.f0 * 6 + i] = 0.0;  // new structure: fresh _x
    for (int i = tid; i < 3 * d.npts; i += 1024) A.xl[(size_t)d.pt0 * 3 + i] = 0.0;
    atomicAdd(&s_cnt, cnt);
    __syncthreads();
    if (tid == 0) {
        BAState s2 = A.st[p];
        s2.round++;
        if (s2.round == 1 && s_cnt == 0) {  // no edge left: optimize(10) does not run
            s2.round = 2;
            s2.iters[1] = -1;
        } else if (s2.round == 1 && A.stop && *A.stop) {
            // stopped: optimize(10) returns before its first iteration; its
            // outlier check sees the estimate the first pass just checked
            s2.round = 2;
            s2.iters[1] = 0;
        }
        s2.iter = 0;
        s2.q = 0;
        s2.need_lin = 1;
        s2.ni = 2;
        s2.nbad = 0;
        A.st[p] = s2;
    }
}

// ------------------------------------------------------------------ outputs
__global__ __launch_bounds__(256) void k_ba_finish(BAArena A) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const BADesc d = A.desc[p];
    const int cur = A.st[p].cur;
    for (int k = tid; k < d.nkf; k += 256) {  // Converter::toCvMat for the local keyframes
        float* o = A.out_T + (size_t)(d.kf0 + k) * 16;
        if (A.kf_kind[d.kf0 + k] == 2) {
            for (int q = 0; q < 16; q++) o[q] = A.kf_Tcw0[(size_t)(d.kf0 + k) * 16 + q];
            continue;
        }
        const gfse3::SE3 T = load_T(A, cur, d.kf0 + k);
        double R[9];
        gfse3::to_R(T.r, R);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) o[4 * i + j] = (float)R[3 * i + j];
            o[4 * i + 3] = (float)T.t[i];
        }
        o[12] = o[13] = o[14] = 0.f;
        o[15] = 1.f;
    }
    for (int i = tid; i < d.npts; i += 256) {
        const double* X = ptX_at(A, cur, d.pt0 + i);
        for (int c = 0; c < 3; c++) A.out_X[(size_t)(d.pt0 + i) * 3 + c] = (float)X[c];
    }
}

template <typename T>
int dalloc(T** p, size_t n, std::vector<void*>& owned) {
    *p = nullptr;
    if (n == 0) n = 1;
    GF_HIP(hipMalloc((void**)p, n * sizeof(T)));
    owned.push_back((void*)*p);
    return GF_OK;
}

}  // namespace

// ====================================================================== host
struct gf_ba_plan {
    gf_ctx* ctx = nullptr;
    int nprob = 0;
    std::vector<BADesc> desc;
    int max_nwg = 1, max_free = 1, max_tiles = 1, max_newg = 1, max_split = 1, max_ss = 1, max_npad = 16;
    int max_items = 1;
    bool sparse_gemm = true;  // task-list Schur GEMM (small batches); dense split-K otherwise
    size_t panel_doubles = 0;
    BAArena A{};
    std::vector<void*> owned;
    BAState* h_state = nullptr;  // pinned
    BADesc* d_desc = nullptr;
    int* d_stop = nullptr;       // device copy of the caller's stop flag
    std::vector<uint8_t> h_out;  // scratch for results
};

namespace {

int ba_launch_step(gf_ba_plan* P, hipStream_t s) {
    const BAArena& A = P->A;
    const int B = P->nprob;
    const dim3 gpt(P->max_nwg, B), gpose(P->max_free, B), gedge(P->max_newg, B),
        ggemm((P->max_items + BA_SW - 1) / BA_SW, B), gred((P->max_ss + 255) / 256, B);
    {
        GF_PROF(P->ctx, s, "k_ba_linearize");
        GF_LAUNCH(k_ba_linearize, gpt, BA_T, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_poses");
        GF_LAUNCH(k_ba_poses, gpose, BA_PT, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_schur_pts");
        GF_LAUNCH(k_ba_schur_pts, gedge, BA_T, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_gemm");
        if (P->sparse_gemm)
            GF_LAUNCH(k_ba_spgemm, ggemm, 64 * BA_SW, 0, s, A);
        else
            GF_LAUNCH(k_ba_gemm, dim3(P->max_split, B), 64 * BA_GW, ba_gemm_lds(P->max_npad), s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_gemm_reduce");
        GF_LAUNCH(k_ba_gemm_reduce, gred, 256, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_solve");
        GF_LAUNCH(k_ba_solve, B, BA_ST, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_update");
        GF_LAUNCH(k_ba_update, gpt, BA_T, 0, s, A);
    }
    {
        GF_PROF(P->ctx, s, "k_ba_decide");
        GF_LAUNCH(k_ba_decide, B, 1024, 0, s, A);
    }
    GF_HIP(hipGetLastError());
    return GF_OK;
}

}  // namespace

extern "C" {

int gf_ba_plan_destroy(gf_ba_plan* P) {
    if (!P) return GF_OK;
    if (P->ctx) (void)hipSetDevice(P->ctx->device);
    for (void* q : P->owned) (void)hipFree(q);
    if (P->h_state) (void)hipHostFree(P->h_state);
    delete P;
    return GF_OK;
}

int gf_ba_plan_create(gf_ctx* ctx, int nprob, const gf_ba_problem* probs, gf_ba_plan** out) {
    GF_CHECK(ctx && out && (nprob == 0 || probs), GF_ERR_ARG, "null arg");
    GF_CHECK(nprob >= 0, GF_ERR_ARG, "nprob < 0");
    *out = nullptr;
    // ---- validate and lay out (host): index mapping, edge ranges, pose edge lists
    std::vector<BADesc> desc(nprob);
    std::vector<int32_t> kf_col, pt_eb, pt_ee, e_pt, e_kf, f_kf, f_eptr, f_elist;
    std::vector<double> e_meas;
    std::vector<float> kf_T, pt_pos;
    std::vector<uint16_t> kmask;
    std::vector<int4> items;
    std::vector<int32_t> klist, tile_iptr;
    // k-steps per item: short runs keep a single window's GEMM spread over the chip
    const int kch = BA_KCH;
    // few windows: the task list (only the nonzero tile products; 3.97 -> 3.64 ms
    // per window alone); many windows: the dense split-K product streams the
    // panels, which beats scattered 128-byte reads once they leave the caches
    const bool sparse = nprob <= 8;
    const int nsplit = std::max(1, std::min(BA_MAXSPLIT, (256 + std::max(nprob, 1) - 1) / std::max(nprob, 1)));
    int ss_tot = 0;
    std::vector<uint8_t> kf_kind;
    int nkf_tot = 0, npt_tot = 0, ne_tot = 0, nf_tot = 0, ntile_tot = 0, nwg_tot = 0;
    long long panel = 0;
    for (int p = 0; p < nprob; p++) {
        const gf_ba_problem& Q = probs[p];
        GF_CHECK(Q.nkf >= 0 && Q.npts >= 0 && Q.nedges >= 0, GF_ERR_ARG, "negative size");
        GF_CHECK(Q.npts <= BA_MAXPTS, GF_ERR_UNSUPPORTED, "more than 65536 points");
        GF_CHECK((Q.nkf == 0 || (Q.kf_Tcw && Q.kf_kind && Q.kf_cam)) && (Q.npts == 0 || Q.pt_pos) &&
                     (Q.nedges == 0 || (Q.edge_pt && Q.edge_kf && Q.edge_z && Q.edge_inv_sigma2)),
                 GF_ERR_ARG, "null array");
        BADesc& d = desc[p];
        d.nkf = Q.nkf;
        d.npts = Q.npts;
        d.nedges = Q.nedges;
        d.kf0 = nkf_tot;
        d.pt0 = npt_tot;
        d.e0 = ne_tot;
        d.f0 = nf_tot;
        d.fe0 = (int)f_eptr.size();
        d.pl0 = (int)f_elist.size();
        int nfree = 0;
        std::vector<int> col(Q.nkf, -1);
        for (int k = 0; k < Q.nkf; k++) {
            GF_CHECK(Q.kf_kind[k] <= 2, GF_ERR_ARG, "keyframe kind must be 0, 1 or 2");
            if (Q.kf_kind[k] == 0) {
                col[k] = nfree++;
                f_kf.push_back(k);
            }
            kf_col.push_back(col[k]);
            kf_kind.push_back(Q.kf_kind[k]);
            for (int q = 0; q < 16; q++) kf_T.push_back(Q.kf_Tcw[16 * k + q]);
        }
        GF_CHECK(nfree <= BA_MAXFREE, GF_ERR_UNSUPPORTED, "more than 32 local (non-fixed) keyframes");
        d.nfree = nfree;
        // edges of a point contiguous, one edge per (point, keyframe)
        std::vector<int> eb(Q.npts, 0), ee(Q.npts, 0), seen(Q.npts, 0);
        for (int e = 0; e < Q.nedges; e++) {
            const int pt = Q.edge_pt[e], kf = Q.edge_kf[e];
            GF_CHECK(pt >= 0 && pt < Q.npts && kf >= 0 && kf < Q.nkf, GF_ERR_ARG, "edge index out of range");
            if (!seen[pt]) {
                seen[pt] = 1;
                eb[pt] = e;
            } else {
                GF_CHECK(ee[pt] == e, GF_ERR_ARG, "edges of a map point must be contiguous");
            }
            ee[pt] = e + 1;
        }
        for (int i = 0; i < Q.npts; i++) {
            for (int a = eb[i]; a < ee[i]; a++)
                for (int b = a + 1; b < ee[i]; b++)
                    GF_CHECK(Q.edge_kf[a] != Q.edge_kf[b], GF_ERR_ARG, "two edges between one point and one keyframe");
            pt_eb.push_back(eb[i]);
            pt_ee.push_back(ee[i]);
            for (int c = 0; c < 3; c++) pt_pos.push_back(Q.pt_pos[3 * i + c]);
        }
        for (int e = 0; e < Q.nedges; e++) {
            const float* K = Q.kf_cam + 4 * Q.edge_kf[e];
            e_pt.push_back(Q.edge_pt[e]);
            e_kf.push_back(Q.edge_kf[e]);
            const double m[8] = {(double)Q.edge_z[2 * e], (double)Q.edge_z[2 * e + 1], (double)Q.edge_inv_sigma2[e],
                                 (double)K[0], (double)K[1], (double)K[2], (double)K[3], 0.0};
            e_meas.insert(e_meas.end(), m, m + 8);
        }
        // per free pose: its edges in point order
        std::vector<std::vector<int>> lists(nfree);
        for (int i = 0; i < Q.npts; i++)
            for (int e = eb[i]; e < ee[i]; e++)
                if (col[Q.edge_kf[e]] >= 0) lists[col[Q.edge_kf[e]]].push_back(e);
        int acc = 0;
        for (int a = 0; a < nfree; a++) {
            f_eptr.push_back(acc);
            for (int e : lists[a]) f_elist.push_back(e);
            acc += (int)lists[a].size();
        }
        f_eptr.push_back(acc);
        // Schur panel / GEMM geometry; per k-step (4 panel rows) the column tiles a point block touches
        d.n = 6 * nfree;
        d.npad = ((d.n + 1 + 15) / 16) * 16;
        const int steps = std::max(1, (3 * Q.npts + 3) / 4);
        d.nsplit = nsplit;
        d.sps = (steps + nsplit - 1) / nsplit;
        d.K = nsplit * d.sps * 4;
        const int nt = d.npad / 16;
        d.ntiles = nt * (nt + 1) / 2 + (d.n >> 4);
        GF_CHECK(d.ntiles <= BA_GW * BA_GTPW, GF_ERR_UNSUPPORTED, "Schur GEMM tile count");
        d.nwg = std::max(1, (Q.npts + BA_T - 1) / BA_T);
        d.newg = std::max(1, (Q.nedges + BA_T - 1) / BA_T);
        d.tile0 = ntile_tot;
        d.wg0 = nwg_tot;
        d.panel0 = panel;
        d.mask0 = (int)kmask.size();
        d.ss0 = ss_tot;
        kmask.resize(kmask.size() + (size_t)nsplit * d.sps, 0);
        for (int i = 0; i < Q.npts; i++)
            for (int e = eb[i]; e < ee[i]; e++) {
                const int c = col[Q.edge_kf[e]];
                if (c < 0) continue;
                const uint16_t bits = (uint16_t)((1u << ((6 * c) >> 4)) | (1u << ((6 * c + 5) >> 4)));
                for (int r = 3 * i; r < 3 * i + 3; r++) kmask[d.mask0 + r / 4] |= bits;
            }
        d.nitems = -1;
        if (sparse) {  // the GEMM task list: per output tile, the k-steps where both operand tiles are nonzero
            const int tdb = d.n >> 4, lower = nt * (nt + 1) / 2;
            d.item0 = (int)items.size();
            d.kl0 = (int)klist.size();
            d.tip0 = (int)tile_iptr.size();
            int nloc = 0;
            std::vector<int> ks;
            for (int t = 0; t < d.ntiles; t++) {
                int ti, tj;
                if (t < lower) {
                    int a = 0;
                    while ((a + 1) * (a + 2) / 2 <= t) a++;
                    ti = a;
                    tj = t - a * (a + 1) / 2;
                } else {
                    ti = t - lower;
                    tj = tdb;
                }
                tile_iptr.push_back(nloc);
                ks.clear();
                for (int k = 0; k < steps; k++) {
                    const unsigned m = kmask[d.mask0 + k], mb = m | (1u << tdb);
                    if (m && ((m >> ti) & (mb >> tj) & 1u)) ks.push_back(k);
                }
                for (size_t c = 0; c < ks.size(); c += kch) {
                    const int kb = (int)klist.size() - d.kl0;
                    const int ke = kb + (int)std::min<size_t>(kch, ks.size() - c);
                    for (size_t q = c; q < c + (size_t)(ke - kb); q++) klist.push_back(ks[q]);
                    items.push_back(make_int4(ti, tj, kb, ke));
                    nloc++;
                }
            }
            tile_iptr.push_back(nloc);
            d.nitems = nloc;
        }
        nkf_tot += Q.nkf;
        npt_tot += Q.npts;
        ne_tot += Q.nedges;
        nf_tot += nfree;
        ntile_tot += nsplit * d.ntiles;
        nwg_tot += d.nwg;
        ss_tot += d.n * (d.n + 1) / 2 + d.n;
        panel += 2LL * d.K * d.npad;
    }
    GF_HIP(hipSetDevice(ctx->device));
    gf_ba_plan* P = new gf_ba_plan();
    P->ctx = ctx;
    P->nprob = nprob;
    P->desc = desc;
    for (const BADesc& d : desc) {
        P->max_nwg = std::max(P->max_nwg, d.nwg);
        P->max_free = std::max(P->max_free, d.nfree);
        P->max_tiles = std::max(P->max_tiles, d.ntiles);
        P->max_newg = std::max(P->max_newg, d.newg);
        P->max_split = std::max(P->max_split, d.nsplit);
        P->max_ss = std::max(P->max_ss, d.n * (d.n + 1) / 2 + d.n);
        P->max_npad = std::max(P->max_npad, d.npad);
        P->max_items = std::max(P->max_items, d.nitems);
    }
    P->sparse_gemm = sparse;
    P->panel_doubles = (size_t)panel;
    BAArena& A = P->A;
    A.nkf_tot = nkf_tot;
    A.npt_tot = npt_tot;
    int rc = 0;
    BADesc* dd;
    BAState* ds;
    double *kfT, *ptX, *Hll, *bl, *Dinv, *xl, *e_err, *Hpl, *Hpp, *bp, *xp, *pnl, *tiles, *w0, *w1, *w2, *w3, *ssum;
    uint16_t* kmk;
    int4* itm;
    int32_t *kls, *tip;
    float *kT0, *pX0, *oT, *oX;
    uint8_t *kk, *pa, *ea, *eo, *fa;
    int32_t *kc, *peb, *pee, *ept, *ekf, *fkf, *fep, *fel;
    double* em;
    auto& o = P->owned;
    if ((rc = dalloc(&dd, nprob, o)) || (rc = dalloc(&ds, nprob, o)) || (rc = dalloc(&kfT, 16 * (size_t)nkf_tot, o)) ||
        (rc = dalloc(&kT0, 16 * (size_t)nkf_tot, o)) || (rc = dalloc(&kk, nkf_tot, o)) ||
        (rc = dalloc(&kc, nkf_tot, o)) || (rc = dalloc(&ptX, 8 * (size_t)npt_tot, o)) ||
        (rc = dalloc(&pX0, 3 * (size_t)npt_tot, o)) || (rc = dalloc(&peb, npt_tot, o)) ||
        (rc = dalloc(&pee, npt_tot, o)) || (rc = dalloc(&Hll, 9 * (size_t)npt_tot, o)) ||
        (rc = dalloc(&bl, 3 * (size_t)npt_tot, o)) || (rc = dalloc(&Dinv, 9 * (size_t)npt_tot, o)) ||
        (rc = dalloc(&xl, 3 * (size_t)npt_tot, o)) || (rc = dalloc(&pa, npt_tot, o)) ||
        (rc = dalloc(&ept, ne_tot, o)) || (rc = dalloc(&ekf, ne_tot, o)) || (rc = dalloc(&em, 8 * (size_t)ne_tot, o)) ||
        (rc = dalloc(&e_err, 2 * (size_t)ne_tot, o)) || (rc = dalloc(&ea, ne_tot, o)) || (rc = dalloc(&eo, ne_tot, o)) ||
        (rc = dalloc(&Hpl, 18 * (size_t)ne_tot, o)) || (rc = dalloc(&fkf, nf_tot, o)) ||
        (rc = dalloc(&fep, f_eptr.size(), o)) || (rc = dalloc(&fel, f_elist.size(), o)) ||
        (rc = dalloc(&Hpp, 36 * (size_t)nf_tot, o)) || (rc = dalloc(&bp, 6 * (size_t)nf_tot, o)) ||
        (rc = dalloc(&xp, 6 * (size_t)nf_tot, o)) || (rc = dalloc(&fa, nf_tot, o)) ||
        (rc = dalloc(&pnl, P->panel_doubles, o)) || (rc = dalloc(&tiles, 256 * std::max<size_t>(sparse ? items.size() : (size_t)ntile_tot, 1), o)) ||
        (rc = dalloc(&w0, nwg_tot, o)) || (rc = dalloc(&w1, nwg_tot, o)) || (rc = dalloc(&w2, nwg_tot, o)) ||
        (rc = dalloc(&w3, nwg_tot, o)) || (rc = dalloc(&oT, 16 * (size_t)nkf_tot, o)) ||
        (rc = dalloc(&oX, 3 * (size_t)npt_tot, o)) || (rc = dalloc(&kmk, kmask.size(), o)) ||
        (rc = dalloc(&ssum, ss_tot, o)) || (rc = dalloc(&itm, items.size(), o)) ||
        (rc = dalloc(&kls, klist.size(), o)) || (rc = dalloc(&tip, tile_iptr.size(), o))) {
        gf_ba_plan_destroy(P);
        return rc;
    }
    hipError_t he = hipHostMalloc((void**)&P->h_state, sizeof(BAState) * std::max(nprob, 1));
    if (he != hipSuccess) {
        gf_ba_plan_destroy(P);
        return gf::fail(GF_ERR_HIP, hipGetErrorString(he));
    }
    hipStream_t s = ctx->stream;
    auto up = [&](void* dst, const void* src, size_t bytes) {
        return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s) : hipSuccess;
    };
    if ((he = up(dd, desc.data(), sizeof(BADesc) * nprob)) || (he = up(kT0, kf_T.data(), 4 * kf_T.size())) ||
        (he = up(kk, kf_kind.data(), kf_kind.size())) || (he = up(kc, kf_col.data(), 4 * kf_col.size())) ||
        (he = up(pX0, pt_pos.data(), 4 * pt_pos.size())) || (he = up(peb, pt_eb.data(), 4 * pt_eb.size())) ||
        (he = up(pee, pt_ee.data(), 4 * pt_ee.size())) || (he = up(ept, e_pt.data(), 4 * e_pt.size())) ||
        (he = up(ekf, e_kf.data(), 4 * e_kf.size())) || (he = up(em, e_meas.data(), 8 * e_meas.size())) ||
        (he = up(fkf, f_kf.data(), 4 * f_kf.size())) || (he = up(fep, f_eptr.data(), 4 * f_eptr.size())) ||
        (he = up(fel, f_elist.data(), 4 * f_elist.size())) || (he = up(kmk, kmask.data(), 2 * kmask.size())) ||
        (he = up(itm, items.data(), sizeof(int4) * items.size())) || (he = up(kls, klist.data(), 4 * klist.size())) ||
        (he = up(tip, tile_iptr.data(), 4 * tile_iptr.size())) ||
        (he = hipStreamSynchronize(s))) {
        gf_ba_plan_destroy(P);
        return gf::fail(GF_ERR_HIP, hipGetErrorString(he));
    }
    P->d_desc = dd;
    A.desc = dd;
    A.st = ds;
    A.kfT = kfT;
    A.kf_Tcw0 = kT0;
    A.kf_kind = kk;
    A.kf_col = kc;
    A.ptX = ptX;
    A.pt_pos0 = pX0;
    A.pt_eb = peb;
    A.pt_ee = pee;
    A.Hll = Hll;
    A.bl = bl;
    A.Dinv = Dinv;
    A.xl = xl;
    A.pt_act = pa;
    A.e_pt = ept;
    A.e_kf = ekf;
    A.e_meas = em;
    A.e_err = e_err;
    A.e_act = ea;
    A.e_out = eo;
    A.Hpl = Hpl;
    A.f_kf = fkf;
    A.f_eptr = fep;
    A.f_elist = fel;
    A.Hpp = Hpp;
    A.bp = bp;
    A.xp = xp;
    A.f_act = fa;
    A.panel = pnl;
    A.tiles = tiles;
    A.kmask = kmk;
    A.items = itm;
    A.klist = kls;
    A.tile_iptr = tip;
    A.Ssum = ssum;
    A.wg_chi = w0;
    A.wg_chi_t = w1;
    A.wg_maxd = w2;
    A.wg_scale = w3;
    A.out_T = oT;
    A.out_X = oX;
    *out = P;
    return GF_OK;
}

}  // extern "C"

// Diagnostics (not in the ABI header): device buffer of 8 stamps per problem
// written by k_ba_solve, or nullptr.
extern "C" int gf_ba_plan_debug_stamps(gf_ba_plan* P, unsigned long long* d_stamps) {
    GF_CHECK(P, GF_ERR_ARG, "null plan");
    P->A.tstamp = d_stamps;
    return GF_OK;
}

extern "C" {

int gf_ba_plan_solve(gf_ba_plan* P, void* stream, int* steps) { return gf_ba_plan_solve_stop(P, stream, nullptr, steps); }

int gf_ba_plan_solve_stop(gf_ba_plan* P, void* stream, const volatile uint8_t* stop_flag, int* steps) {
    GF_CHECK(P, GF_ERR_ARG, "null plan");
    if (steps) *steps = 0;
    if (P->nprob == 0) return GF_OK;
    GF_HIP(hipSetDevice(P->ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : P->ctx->stream;
    if (!P->d_stop) {
        GF_HIP(hipMalloc(&P->d_stop, sizeof(int)));
        P->owned.push_back(P->d_stop);
        P->A.stop = P->d_stop;
    }
    GF_HIP(hipMemsetAsync(P->d_stop, 0, sizeof(int), s));
    bool stop_sent = false;
    GF_HIP(hipMemsetAsync(P->A.panel, 0, P->panel_doubles * sizeof(double), s));
    {
        GF_PROF(P->ctx, s, "k_ba_init");
        GF_LAUNCH(k_ba_init, P->nprob, 256, 0, s, P->A);
        GF_HIP(hipGetLastError());
    }
    // Steps are enqueued blindly in chunks (a finished problem's kernels
    // return at once) and the state is read back after each chunk. The first
    // chunk covers the usual optimize(5) + optimize(10) run (15 iterations,
    // one trial each), the later ones are short; every chunk ends with the
    // output conversion (idempotent), so the chunk that finishes the last
    // problem needs no further launch and wait. A host round trip costs about
    // as much as two no-op steps.
    int n = 0;
    bool done = false;
    while (!done) {
        GF_CHECK(n < BA_MAXSTEPS, GF_ERR_HIP, "local BA did not terminate");
        if (stop_flag && *stop_flag && !stop_sent) {  // the caller raised mbAbortBA
            static const int one = 1;
            GF_HIP(hipMemcpyAsync(P->d_stop, &one, sizeof(int), hipMemcpyHostToDevice, s));
            stop_sent = true;
        }
        const int chunk = n == 0 ? 12 : 4;
        for (int c = 0; c < chunk; c++, n++) {
            int rc = ba_launch_step(P, s);
            if (rc) return rc;
        }
        {
            GF_PROF(P->ctx, s, "k_ba_finish");
            GF_LAUNCH(k_ba_finish, P->nprob, 256, 0, s, P->A);
            GF_HIP(hipGetLastError());
        }
        GF_HIP(hipMemcpyAsync(P->h_state, P->A.st, sizeof(BAState) * P->nprob, hipMemcpyDeviceToHost, s));
        GF_HIP(hipStreamSynchronize(s));
        done = true;
        for (int p = 0; p < P->nprob; p++) done = done && P->h_state[p].round >= 2;
    }
    if (steps) *steps = n;
    return GF_OK;
}

int gf_ba_plan_results(gf_ba_plan* P, gf_ba_result* res) {
    GF_CHECK(P && (P->nprob == 0 || res), GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(P->ctx->device));
    hipStream_t s = P->ctx->stream;
    GF_HIP(hipMemcpyAsync(P->h_state, P->A.st, sizeof(BAState) * std::max(P->nprob, 1), hipMemcpyDeviceToHost, s));
    for (int p = 0; p < P->nprob; p++) {
        const BADesc& d = P->desc[p];
        gf_ba_result& r = res[p];
        if (d.nkf)
            GF_HIP(hipMemcpyAsync(r.kf_Tcw, P->A.out_T + (size_t)d.kf0 * 16, 64 * (size_t)d.nkf, hipMemcpyDeviceToHost, s));
        if (d.npts)
            GF_HIP(hipMemcpyAsync(r.pt_pos, P->A.out_X + (size_t)d.pt0 * 3, 12 * (size_t)d.npts, hipMemcpyDeviceToHost, s));
        if (d.nedges) GF_HIP(hipMemcpyAsync(r.edge_outlier, P->A.e_out + d.e0, d.nedges, hipMemcpyDeviceToHost, s));
    }
    GF_HIP(hipStreamSynchronize(s));
    for (int p = 0; p < P->nprob; p++) {
        res[p].iterations[0] = P->h_state[p].iters[0];
        res[p].iterations[1] = P->h_state[p].iters[1];
    }
    return GF_OK;
}

int gf_local_ba(gf_ctx* ctx, const gf_ba_problem* prob, gf_ba_result* res) {
    return gf_local_ba_stop(ctx, prob, res, nullptr);
}

int gf_local_ba_stop(gf_ctx* ctx, const gf_ba_problem* prob, gf_ba_result* res, const volatile uint8_t* stop_flag) {
    GF_CHECK(ctx && prob && res, GF_ERR_ARG, "null arg");
    gf_ba_plan* P = nullptr;
    int rc = gf_ba_plan_create(ctx, 1, prob, &P);
    if (rc) return rc;
    rc = gf_ba_plan_solve_stop(P, nullptr, stop_flag, nullptr);
    if (!rc) rc = gf_ba_plan_results(P, res);
    gf_ba_plan_destroy(P);
    return rc;
}

}  // extern "C"
