// Good-feature selection on gfx950 — SURVEY.md §8a rows G2-G7 (f64).
//
//   k_obs_info     one thread per landmark: measurement Jacobian H (2x7) and
//                  information block H_rw^T H_rw (compute_H_subblock_simplied
//                  Observability.h:460-515, reWeightInfoMat :517-596,
//                  batchInfoMat_Map/_Frame Observability.cc:386-644)
//   k_logdet       Util.hpp:714-731 (Cholesky, LU fallback)
//   k_active_match one workgroup per frame: runActiveMapMatching
//                  (Observability.cc:1249-1524). The lazier-greedy rounds are
//                  sequential in the reference (std::rand draws, a max-heap,
//                  one-point matches that claim keypoints); the workgroup keeps
//                  that order exactly — draws and heap on one lane, the
//                  log-dets of each batch of random samples across the
//                  workgroup, grid/claims/pool/heap in LDS.
//   k_maxvol       one workgroup per pool: maxVolSelection_BaselineGreedy /
//                  _LazierGreedy / maxVolDeletion_LazierGreedy
//                  (Observability.cc:2339-3155).
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>

#include <type_traits>

#include "common.h"
#include "match_common.h"
#include "rng.h"
#include "select.h"

#define POOL_MAX 4096
// AM_CC 1: the first pass's candidate arrays apart from its pool (AM_CAND_CAP
// entries; a frame whose round would draw past them is redone by the overflow
// pass). Off by default: the LDS it saves (50.7 -> 38.6 KB) did not move the
// headline, and the extra state slowed one frame's pop chain by a fifth
// (single sequence 1.28 -> 1.40 ms, profiles/r04/sp2_*.json).
#ifndef AM_CC
#define AM_CC 0
#endif
#ifndef AM_ONE_PASS_MAX
#define AM_ONE_PASS_MAX 64  // batches up to this size take the one-pass launch
#endif
#ifndef AM_CAND_CAP
#define AM_CAND_CAP 640  // first-pass capacity for a round's drawn candidates
#endif
#ifndef AM_SMALL_POOL
#define AM_SMALL_POOL 1280  // first-pass pool capacity of the two-pass active match (multiple of 64)
#endif
#ifndef AM_OVF_GRID
#define AM_OVF_GRID 256  // workgroups of the overflow pass (at most)
#endif
#define GF_THREADS 256
#define MAX_RANDOM_QUERY_TIME 2000

namespace {

// ------------------------------------------------------------- math helpers
__device__ __forceinline__ void q2r(const double* q, double R[3][3]) {
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

// arma::inv of a 3x3 (cofactors / determinant)
__device__ __forceinline__ bool inv3(const double X[3][3], double O[3][3]) {
    const double v1 = X[0][0] * (X[2][2] * X[1][1] - X[1][2] * X[2][1]);
    const double v2 = X[0][1] * (X[2][2] * X[1][0] - X[1][2] * X[2][0]);
    const double v3 = X[0][2] * (X[2][1] * X[1][0] - X[1][1] * X[2][0]);
    const double det = v1 - v2 + v3;
    if (fabs(det) < DBL_EPSILON) return false;
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

// H = [H13 H47] (2x7 row-major) and the projected pixel; false when the
// visibility check rejects the landmark.
__device__ bool landmark_jacobian(const gf_obs_camera& cam, const double* Xv, const double* y, bool check_viz,
                                  double* H, float* uv) {
    const double* q = Xv + 3;
    double Rq[3][3], R[3][3];
    q2r(q, Rq);
    if (!inv3(Rq, R))
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = 0;
    const double t[3] = {y[0] - Xv[0], y[1] - Xv[1], y[2] - Xv[2]};
    double h[3];
    for (int i = 0; i < 3; i++) h[i] = R[i][0] * t[0] + R[i][1] * t[1] + R[i][2] * t[2];
    float u = FLT_MAX, v = FLT_MAX;
    if (h[2] > 0) {
        u = (float)((double)(float)cam.fu * h[0] / h[2] + (double)(float)cam.cx);
        v = (float)((double)(float)cam.fv * h[1] / h[2] + (double)(float)cam.cy);
    }
    uv[0] = u;
    uv[1] = v;
    if (check_viz) {
        if (h[2] < 0.0 + cam.bound_depth) return false;
        if (u < cam.min_x - cam.bound_x || u > cam.max_x + cam.bound_x) return false;
        if (v < cam.min_y - cam.bound_y || v > cam.max_y + cam.bound_y) return false;
    }
    double dh[2][3] = {{0, 0, 0}, {0, 0, 0}};
    if (!(fabs(h[2]) < 1e-6)) {
        const double z2 = h[2] * h[2];
        dh[0][0] = cam.fu / h[2];
        dh[0][2] = -h[0] * cam.fu / z2;
        dh[1][1] = cam.fv / h[2];
        dh[1][2] = -h[1] * cam.fv / z2;
    }
    // dRq_times_a_by_dq(qconj(q), t) * diag(1,-1,-1,-1), Util.hpp:391-438
    const double q0 = q[0], qx = -1.0 * q[1], qy = -1.0 * q[2], qz = -1.0 * q[3];
    const double D[4][3][3] = {
        {{2.0 * q0, -2.0 * qz, 2.0 * qy}, {2.0 * qz, 2.0 * q0, -2.0 * qx}, {-2.0 * qy, 2.0 * qx, 2.0 * q0}},
        {{2.0 * qx, 2.0 * qy, 2.0 * qz}, {2.0 * qy, -2.0 * qx, -2.0 * q0}, {2.0 * qz, 2.0 * q0, -2.0 * qx}},
        {{-2.0 * qy, 2.0 * qx, 2.0 * q0}, {2.0 * qx, 2.0 * qy, 2.0 * qz}, {-2.0 * q0, 2.0 * qz, -2.0 * qy}},
        {{-2.0 * qz, -2.0 * q0, 2.0 * qx}, {2.0 * q0, -2.0 * qz, 2.0 * qy}, {2.0 * qx, 2.0 * qy, 2.0 * qz}}};
    double dR[3][4];
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 3; r++) {
            double e = D[c][r][0] * t[0] + D[c][r][1] * t[1] + D[c][r][2] * t[2];
            dR[r][c] = c ? -e : e;
        }
    for (int i = 0; i < 2; i++) {
        for (int j = 0; j < 3; j++) H[7 * i + j] = -1.0 * (dh[i][0] * R[0][j] + dh[i][1] * R[1][j] + dh[i][2] * R[2][j]);
        for (int j = 0; j < 4; j++) H[7 * i + 3 + j] = dh[i][0] * dR[0][j] + dh[i][1] * dR[1][j] + dh[i][2] * dR[2][j];
    }
    return true;
}

// information block of H / sigma (reWeightInfoMat + H_rw^T H_rw)
__device__ __forceinline__ void add_info_block(const double* H, double sigma2, double* M) {
    const double s = sqrt(sigma2);
    const double w = s / (s * s);
    double Hw[14];
    for (int i = 0; i < 14; i++) Hw[i] = w * H[i];
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) M[7 * i + j] = M[7 * i + j] + (Hw[i] * Hw[j] + Hw[7 + i] * Hw[7 + j]);
}

// rebuilds a + sign*b itself so the caller's matrix can stay in registers
__device__ __noinline__ double logdet_lu(const double* a, const double* b, double sign) {
    double A[49];
    for (int i = 0; i < 49; i++) A[i] = sign > 0 ? a[i] + b[i] : a[i] - b[i];
    double acc = 0;
    for (int c = 0; c < 7; c++) {
        int p = c;
        double best = fabs(A[7 * c + c]);
        for (int r = c + 1; r < 7; r++)
            if (fabs(A[7 * r + c]) > best) best = fabs(A[7 * r + c]), p = r;
        if (p != c)
            for (int k = 0; k < 7; k++) {
                double t = A[7 * c + k];
                A[7 * c + k] = A[7 * p + k];
                A[7 * p + k] = t;
            }
        const double piv = A[7 * c + c];
        if (piv != 0)
            for (int r = c + 1; r < 7; r++) {
                const double f = A[7 * r + c] / piv;
                A[7 * r + c] = f;
                for (int k = c + 1; k < 7; k++) A[7 * r + k] -= f * A[7 * c + k];
            }
        acc += log(fabs(piv));
    }
    return acc;
}

// logDet(a + sign*b), Util.hpp:714-731: 2 log prod diag chol, else LU.
__device__ double logdet_sum(const double* a, const double* b, double sign) {
    double M[49];
#pragma unroll
    for (int i = 0; i < 49; i++) M[i] = sign > 0 ? a[i] + b[i] : a[i] - b[i];
    double L[28];  // packed lower triangle, row-major
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 7; j++) {
        double s = M[8 * j];
#pragma unroll
        for (int k = 0; k < j; k++) s -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
        if (!(s > 0)) {
            ok = false;
            break;
        }
        const double d = sqrt(s);
        L[j * (j + 1) / 2 + j] = d;
        const double rd = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < 7; i++) {
            double t = M[7 * i + j];
#pragma unroll
            for (int k = 0; k < j; k++) t -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
            L[i * (i + 1) / 2 + j] = t * rd;
        }
    }
    if (!ok) return logdet_lu(a, b, sign);
    double v1 = 1, v2 = 1;  // Armadillo's two-accumulator product of the diagonal
    v1 *= L[0];
    v2 *= L[2];
    v1 *= L[5];
    v2 *= L[9];
    v1 *= L[14];
    v2 *= L[20];
    v1 *= L[27];
    return 2 * log(v1 * v2);
}


// logdet_sum(cur, b) (the summed block's logdet) for a matrix the Cholesky
// accepts, reading b's lower triangle from its packed record lt[i (i + 1) / 2
// + j] = b[7 i + j] (kept beside every ObsMat: the Cholesky's 28 entries are
// then two cache lines, not the four the full block's rows spread them over);
// the factor is formed in place, the same arithmetic entry for entry as the
// reference's; a matrix that is not positive definite takes logdet_sum's LU
// fallback on the full b.
__device__ __forceinline__ double logdet_sum_lower_packed(const double* cur, const double* lt, const double* b) {
    double X[28];
    const double* a = static_cast<const double*>(__builtin_assume_aligned(lt, 256));  // 32-double records
#pragma unroll
    for (int k = 0; k < 28; k++) X[k] = gfd::ldg(a + k);
#pragma unroll
    for (int i = 0; i < 7; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) X[i * (i + 1) / 2 + j] = cur[7 * i + j] + X[i * (i + 1) / 2 + j];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 7; j++) {
        double s = X[j * (j + 1) / 2 + j];
#pragma unroll
        for (int k = 0; k < j; k++) s -= X[j * (j + 1) / 2 + k] * X[j * (j + 1) / 2 + k];
        ok = ok && s > 0;
        const double d = sqrt(s);
        X[j * (j + 1) / 2 + j] = d;
        const double rd = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < 7; i++) {
            double t = X[i * (i + 1) / 2 + j];
#pragma unroll
            for (int k = 0; k < j; k++) t -= X[i * (i + 1) / 2 + k] * X[j * (j + 1) / 2 + k];
            X[i * (i + 1) / 2 + j] = t * rd;
        }
    }
    if (!ok) return logdet_lu(cur, b, 1.0);
    double v1 = 1, v2 = 1;  // Armadillo's two-accumulator product of the diagonal
    v1 *= X[0];
    v2 *= X[2];
    v1 *= X[5];
    v2 *= X[9];
    v1 *= X[14];
    v2 *= X[20];
    v1 *= X[27];
    return 2 * log(v1 * v2);
}

// the packed lower triangle of a 7x7 block (logdet_sum_lower_packed's layout)
__device__ __forceinline__ void store_lower_packed(const double* M, double* lt) {
#pragma unroll
    for (int i = 0; i < 7; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) lt[i * (i + 1) / 2 + j] = M[7 * i + j];
}

// The packed records of [F][cap] information blocks, for callers of the
// active matcher that keep only the full blocks (the C-ABI entry points).
__global__ __launch_bounds__(256) void k_pack_info(const double* __restrict__ info, int cap,
                                                   double* __restrict__ lt) {
    const int q = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (q >= cap) return;
    const size_t g = (size_t)f * cap + q;
    store_lower_packed(info + 49 * g, lt + 32 * g);
}

// ------------------------------------------------------------- k_obs_info
__global__ void k_obs_info(gf_obs_camera cam, const double* __restrict__ Xv, const float* __restrict__ pos,
                           const float* __restrict__ sigma2, const int32_t* __restrict__ n, int cap, int check_viz,
                           double* __restrict__ Hout, double* __restrict__ info, float* __restrict__ uv,
                           uint8_t* __restrict__ valid) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n[f]) return;
    const long long g = (long long)f * cap + i;
    const double y[3] = {pos[3 * g], pos[3 * g + 1], pos[3 * g + 2]};
    double H[14];
    float p[2];
    const bool ok = landmark_jacobian(cam, Xv + 13 * f, y, check_viz != 0, H, p);
    uv[2 * g] = p[0];
    uv[2 * g + 1] = p[1];
    valid[g] = ok;
    double M[49];
    for (int k = 0; k < 49; k++) M[k] = 0;
    if (ok) add_info_block(H, sigma2 ? (double)sigma2[g] : 1.0, M);
    for (int k = 0; k < 14; k++) Hout[14 * g + k] = ok ? H[k] : 0.0;
    for (int k = 0; k < 49; k++) info[49 * g + k] = M[k];
}

__global__ void k_logdet(const double* __restrict__ M, int n, double* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double z[49];
    for (int k = 0; k < 49; k++) z[k] = 0;
    out[i] = logdet_sum(M + 49LL * i, z, 1.0);
}

// Sum of information blocks of flagged entries: out[f] = base + sum info[i].
__global__ void k_obs_accumulate(const double* __restrict__ info, const uint8_t* __restrict__ flag,
                                 const int32_t* __restrict__ n, int cap, double diag, double* __restrict__ out) {
    const int f = blockIdx.x;
    const int e = threadIdx.x;  // 49 entries
    if (e >= 49) return;
    double s = (e % 8 == 0) ? diag : 0.0;
    for (int i = 0; i < n[f]; i++) {
        const long long g = (long long)f * cap + i;
        if (flag[g]) s = s + info[49 * g + e];
    }
    out[49LL * f + e] = s;
}

// ------------------------------------------------------------- active matching
struct HeapEntry {
    double s;
    int idx;
    int pad;
};
struct HeapLess {  // std::priority_queue<SimplePoint>: SimplePoint::operator< on score
    __device__ bool operator()(const HeapEntry& a, const HeapEntry& b) const { return a.s < b.s; }
};

struct ActiveArgs {
    FrameConst fc;
    const gf_keypoint* kps;
    const uint8_t* desc;
    const int32_t* n;
    int kp_cap;
    const gf_mp_view* views;
    const uint8_t* mp_desc;
    const uint8_t* updated;
    const double* info;
    const double* H;
    const int32_t* m;
    int mp_cap;
    const double* base;  // [F][49]
    float sigma2[16];
    const int32_t* num_to_match;  // [F]
    float th, nnratio;
    gf_rng* rng;  // [F]
    int32_t* kp2mp;
    int32_t* score;
    int32_t* left;
    int32_t* nleft;
    int32_t* nmatched;
    int32_t* nldet;  // [F] logDet evaluations (optional)
    const int32_t* remap;  // [F][mp_cap] map index of local point q for info / H (null: q itself)
    int32_t* err;
    const struct OnePre* pre;  // [F][mp_cap] one-point results against the starting claims
    int* grid_cs;              // [F][NCELLS + 1] keypoint grid CSR (written by k_onepoint_pre)
    int* grid_items;           // [F][kp_cap]
    int pool_cap;              // LDS pool capacity of this launch (<= POOL_MAX)
    int cand_cap;              // LDS capacity for a round's drawn candidates (<= pool_cap)
    int32_t* ovf;              // two-pass launch: [0] = count, [1 + k] = k-th frame whose pool
                               // did not fit the first pass's LDS
    int pass;                  // 0 = single launch, 1 = small-pool pass, 2 = overflow pass
    const double* info_lt;     // null, or the packed lower triangles of info ([F][mp_cap][32])
    gf::ActiveClock ck;        // the front end's time cap (ck.mat_t0 null: none)
    int lq_stage;              // 1: each pool slot's info / H row (remap) staged in LDS (when it fits)
};

// ---------------------------------------------------------------------------
// runActiveMapMatching on ONE wave per frame. Everything that is sequential in
// the reference stays sequential and in its order (std::rand draws, heap
// tops, one-point matches, claims), but each sequential step is wave-wide:
//   * the glibc random_r state lives in lanes 0..30 of a VGPR and advances
//     with readlane/writelane;
//   * the heap top is a wave arg-max over the live candidates; when the
//     maximum is tied or a score is NaN the std::priority_queue order is
//     ambiguous, and the exact heap is rebuilt by replaying the round's
//     push/pop log with the libstdc++ heap port (select.h);
//   * SearchByProjection_OnePoint scans its grid window with 64 lanes and
//     merges (distance, candidate order) top-2 lists, which is what the
//     sequential best / second-best loop keeps.
constexpr int AW = 64;

// glibc random_r TYPE_3 as a linear recurrence: with the ring read oldest
// first, s_j = st[(f + j) % 31] = o_{n-31+j}, every later word is
// o_{n+k} = o_{n+k-3} + o_{n+k-31} (mod 2^32), hence a fixed integer
// combination sum_j C[k][j] s_j. One wave produces the next 64 words at once
// (lane k: 31 multiply-adds); rand() = word >> 1.
// [j][lane]: lane-consecutive, one coalesced 256-B row per history word
__constant__ uint32_t c_rng_coef[31][64];

// A lane's row of the recurrence. AM_RCOEF_REG 1 keeps it in 31 VGPRs for the
// whole kernel; 0 (default) reads it from the table at each 64-word batch (a
// few batches per round; the 31 registers were a quarter of the budget of a
// kernel whose register pressure the compiler handled wrongly).
#ifndef AM_RCOEF_REG
#define AM_RCOEF_REG 0
#endif
struct RCoef {
#if AM_RCOEF_REG
    uint32_t c[31];
    __device__ void load() {
#pragma unroll
        for (int j = 0; j < 31; j++) c[j] = c_rng_coef[j][threadIdx.x];
    }
    __device__ uint32_t operator[](int j) const { return c[j]; }
#else
    __device__ void load() {}
    __device__ uint32_t operator[](int j) const { return c_rng_coef[j][threadIdx.x]; }
#endif
};

__device__ __forceinline__ uint32_t rng_word(uint32_t s, const RCoef& coef) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 31; j++) acc += coef[j] * (uint32_t)__builtin_amdgcn_readlane((int)s, j);
    return acc;
}

// history after consuming c (<= 64) words: s'_j = h_{c+j}, h = s ++ o
__device__ __forceinline__ uint32_t rng_advance(uint32_t s, uint32_t o, int c) {
    const int j = threadIdx.x, src = c + j;
    const uint32_t a = (uint32_t)__shfl((int)s, min(src, 30), 64);
    const uint32_t b = (uint32_t)__shfl((int)o, max(src - 31, 0), 64);
    return j < 31 ? (src < 31 ? a : b) : 0u;
}

struct IdxLess {  // SimplePoint::operator< (score only), on candidate indices
    const double* sc;
    __device__ bool operator()(int16_t a, int16_t b) const { return sc[a] < sc[b]; }
};

__device__ __forceinline__ void top2_insert(unsigned long long key, unsigned long long& k1, unsigned long long& k2) {
    if (key < k1) {
        k2 = k1;
        k1 = key;
    } else if (key < k2) {
        k2 = key;
    }
}

// Pool = lmkIdx columns: alive slots of the original in-view list, in slot
// order; bits + per-word prefix counts give the j-th column in O(log).
struct Pool {
    unsigned long long* bits;  // [64]
    int* pre;                  // [65]
};

__device__ __forceinline__ int pool_select(const Pool& P, int j) {
    int lo = 0, hi = 64;  // largest w with pre[w] <= j
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (P.pre[mid] <= j) lo = mid;
        else hi = mid;
    }
    unsigned long long w = P.bits[lo];
    int r = j - P.pre[lo], pos = 0;
#pragma unroll
    for (int half = 32; half >= 1; half >>= 1) {
        const int c = __popcll(w & ((1ull << half) - 1ull));
        if (r >= c) {
            r -= c;
            w >>= half;
            pos += half;
        }
    }
    return lo * 64 + pos;
}

__device__ __forceinline__ void pool_prefix(const Pool& P) {
    const int lane = threadIdx.x;
    int c = __popcll(P.bits[lane]), x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    P.pre[lane] = x - c;
    if (lane == 63) P.pre[64] = x;
}

// Keypoint sources for the one-point scan: the frame's arrays in HBM, or the
// copy a precompute workgroup staged in LDS (x, y, octave as float4; the
// descriptors behind a generic pointer, LDS or HBM).
struct KpGlobal {
    const gf_keypoint* K;
    const uint8_t* D;
    __device__ float4 xyo(int i) const {
        const gf_keypoint kp = K[i];
        return make_float4(kp.x, kp.y, __int_as_float(kp.octave), 0.f);
    }
    __device__ const uint8_t* desc(int i) const { return D + (long long)i * 32; }
};
struct KpStaged {
    const float4* X;
    const uint8_t* D;
    __device__ float4 xyo(int i) const { return X[i]; }
    __device__ const uint8_t* desc(int i) const { return D + (long long)i * 32; }
};

// ORBmatcher::SearchByProjection_OnePoint (ORBmatcher.h:71-145) on one lane,
// without claiming: the keypoint it would claim (or -1) and its distance,
// plus the keypoints holding first and second place in its best/second-best
// loop. Claims only remove keypoints, and the loop's outcome is a function of
// those two holders alone (the first keypoint at the minimum distance, the
// first other one at the second smallest), so a result stays exact until one
// of its two holders is claimed.
// MB > 1: the positions and descriptors of MB candidates are loaded together
// (clamped indices, unconditional) and then walked in order.
template <int MB = 1, class KP>
__device__ void one_point_scan(const ActiveArgs& A, const FrameConst& fc, int f, int mpi, const int* cell_start,
                               const int* items, const int* claim, const KP& kps, int& outIdx, int& outDist,
                               int& holder1, int& holder2) {
    outIdx = -1;
    outDist = INT_MAX;
    holder1 = holder2 = -1;
    const gf_mp_view v = A.views[(long long)f * A.mp_cap + mpi];
    if (!v.in_view) return;
    const int pl = min(max(v.level, 0), fc.nlevels - 1);
    float r = v.view_cos > 0.998 ? 2.5f : 4.0f;
    if (A.th != 1.0) r *= A.th;
    r = r * fc.scales[pl];
    int cx0, cx1, cy0, cy1;
    if (!grid_window(fc, v.u, v.v, r, cx0, cx1, cy0, cy1)) return;
    const uint8_t* qd = A.mp_desc + ((long long)f * A.mp_cap + mpi) * 32;
    int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1, secondIdx = -1;
    uint4 qa, qb;
    if constexpr (MB > 1) {
        qa = reinterpret_cast<const uint4*>(qd)[0];
        qb = reinterpret_cast<const uint4*>(qd)[1];
    }
    for (int ix = cx0; ix <= cx1; ix++) {
        const int s = cell_start[ix * GRID_ROWS + cy0], e = cell_start[ix * GRID_ROWS + cy1 + 1];
        for (int t0 = s; t0 < e; t0 += MB) {
            int id[MB];
            float4 kq[MB];
            uint4 da[MB], db[MB];
#pragma unroll
            for (int u = 0; u < MB; u++) id[u] = items[MB > 1 ? min(t0 + u, e - 1) : t0];
#pragma unroll
            for (int u = 0; u < MB; u++) {
                kq[u] = kps.xyo(id[u]);
                if constexpr (MB > 1) {
                    const uint4* pd = reinterpret_cast<const uint4*>(kps.desc(id[u]));
                    da[u] = pd[0];
                    db[u] = pd[1];
                }
            }
#pragma unroll
            for (int u = 0; u < MB; u++) {
                if (MB > 1 && t0 + u >= e) continue;
                const int idx = id[u];
                const float4 kp = kq[u];
                const int oct = __float_as_int(kp.z);
                if (!level_ok(oct, pl - 1, pl)) continue;
                if (fabsf(kp.x - v.u) > r || fabsf(kp.y - v.v) > r) continue;
                if (claim[idx] >= 0) continue;
                int dist;
                if constexpr (MB > 1)
                    dist = hamming_regs(qa, qb, da[u], db[u]);
                else
                    dist = hamming32(qd, kps.desc(idx));
                if (dist < bestDist) {
                    bestDist2 = bestDist;
                    bestDist = dist;
                    bestLevel2 = bestLevel;
                    bestLevel = oct;
                    secondIdx = bestIdx;
                    bestIdx = idx;
                } else if (dist < bestDist2) {
                    bestLevel2 = oct;
                    bestDist2 = dist;
                    secondIdx = idx;
                }
            }
        }
    }
    holder1 = bestIdx;
    holder2 = secondIdx;
    if (bestDist <= TH_HIGH) {
        if (bestLevel == bestLevel2 && (float)bestDist > A.nnratio * (float)bestDist2) return;
        outIdx = bestIdx;
        outDist = bestDist;
    }
}

struct OnePre {  // one-point result against the frame's starting claims
    int16_t idx, dist, holder1, holder2;
};

// One 1024-thread workgroup per frame: the keypoint grid, the keypoints'
// (x, y, octave) (and, up to PRE_DESC_LDS_MAX keypoints, their descriptors) in LDS, then
// one thread per in-view map point runs the one-point scan. The active
// matcher takes these results until a claim hits one of their holders.
#ifndef PRE_THREADS
#define PRE_THREADS 1024
#endif
// descriptors staged in LDS up to this capacity; 0 since r04 (see
// SEQ_PRE_DESC_MAX in match.hip)
// candidates whose loads the precompute's scan issues together
#ifndef PRE_MB
#define PRE_MB 2
#endif
#ifndef PRE_DESC_LDS_MAX
#define PRE_DESC_LDS_MAX 0
#endif
__global__ __launch_bounds__(PRE_THREADS) void k_onepoint_pre(ActiveArgs A, OnePre* __restrict__ out) {
    gfd::track_prio();
    extern __shared__ __align__(16) uint8_t smem[];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(A.n[f], KP_MAX);
    const int m = min(A.m[f], 32767);
    if (m == 0 || A.num_to_match[f] <= 0) return;  // k_active_match takes its early exit
    float4* X = (float4*)smem;                  // kp_cap
    int* cell_start = (int*)(X + A.kp_cap);     // NCELLS + 1
    int* items = cell_start + NCELLS + 1;       // kp_cap
    int* claim = items + A.kp_cap;              // kp_cap
    int* scratch = claim + A.kp_cap;            // kp_cap
    uint8_t* Ds = (uint8_t*)(scratch + A.kp_cap);  // 32 x kp_cap when kp_cap <= PRE_DESC_LDS_MAX
    const gf_keypoint* K = A.kps + (long long)f * A.kp_cap;
    const uint8_t* D = A.desc + (long long)f * A.kp_cap * 32;
    const bool dl = A.kp_cap <= PRE_DESC_LDS_MAX;
    for (int i = tid; i < n; i += PRE_THREADS) {
        const gf_keypoint kp = K[i];
        X[i] = make_float4(kp.x, kp.y, __int_as_float(kp.octave), 0.f);
    }
    if (dl)
        for (int i = tid; i < 2 * n; i += PRE_THREADS)
            reinterpret_cast<uint4*>(Ds)[i] = reinterpret_cast<const uint4*>(D)[i];
    build_grid(A.fc, K, n, A.kp2mp + (long long)f * A.kp_cap, cell_start, items, claim, scratch,
               PRE_THREADS);
    for (int c = tid; c < NCELLS + 1; c += PRE_THREADS) A.grid_cs[(long long)f * (NCELLS + 1) + c] = cell_start[c];
    for (int i = tid; i < n; i += PRE_THREADS) A.grid_items[(long long)f * A.kp_cap + i] = items[i];
    const KpStaged src{X, dl ? (const uint8_t*)Ds : D};
    for (int i = tid; i < m; i += PRE_THREADS) {
        int mi, md, h1, h2;
        one_point_scan<PRE_MB>(A, A.fc, f, i, cell_start, items, claim, src, mi, md, h1, h2);
        out[(long long)f * A.mp_cap + i] = OnePre{(int16_t)mi, (int16_t)(mi >= 0 ? md : 0), (int16_t)h1, (int16_t)h2};
    }
}

size_t onepoint_pre_lds_bytes(int kp_cap) {
    return 16 * (size_t)kp_cap + sizeof(int) * (NCELLS + 1 + 3 * (size_t)kp_cap) +
           (kp_cap <= PRE_DESC_LDS_MAX ? 32 * (size_t)kp_cap : 0);
}

#ifdef GF_AM_STAMP
// [0..7] phase cycles; [8] draw batches, [9] eval calls, [10] candidates
// evaluated, [11] one-point rescans, [12] rounds, [13] pops, [16] max and [17]
// sum of a frame's cycles
__device__ unsigned long long g_am_stamp[24];
#define AM_C(k, v)                                                              \
    do {                                                                        \
        if (threadIdx.x == 0) atomicAdd(&g_am_stamp[k], (unsigned long long)(v)); \
    } while (0)
#else
#define AM_C(k, v) (void)0
#endif
#ifdef GF_AM_GUARD
__device__ unsigned long long g_am_guard[2];  // [0] corrupted sentinel dwords, [1] frames checked
#endif
#ifdef GF_AM_CHECK
// diagnostic build: [0] commits whose batch-restart RNG history differs from
// the step-by-step one, [1] out-of-range slot indices at the commit, [2]
// out-of-range claimed keypoints, [3] sigma^2 copies that differ, [4] commits
// checked, [8..15] the first RNG mismatch (frame, round, T, nb, b, sz, npop,
// pass), [16..47] its fast history lanes, [48..79] its step-by-step lanes
__device__ unsigned long long g_am_check[80];
#endif
#ifdef GF_AM_TRACE
// diagnostic build: one 48-word record per commit of frames 0..7: round, T,
// nused, nc, nb, used, top, N, oct_b, sigma^2 bits, the round's start
// history lanes 0..30 would follow at the next record; here the committed
// history rs (lanes 0..30) at words 16..46
constexpr int AMT_REC = 48, AMT_MAX = 2048;
__device__ uint32_t g_am_trace[8][AMT_MAX][AMT_REC];
__device__ uint32_t g_am_tcnt[8];
#endif

// Per-round candidate list: the draws of the sequential loop in order (the
// initial random subset, then one replacement per failed top), produced 64
// tries at a time ahead of need.
// The active matcher is one wave per workgroup: its LDS hand-offs need the
// wave's LDS operations done and ordered, not a workgroup barrier, whose
// release fence also waits for the wave's outstanding global stores.
#ifdef AM_SYNC_BAR  // diagnostic: workgroup barriers instead of the wave-scope hand-offs
__device__ __forceinline__ void am_sync() { __syncthreads(); }
#else
__device__ __forceinline__ void am_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif

// AM_PREFETCH: each evaluated candidate's claimed-keypoint octave kept in LDS
// (beside its distance) and its H row touched into the caches, so the round's
// commit (curMat += H^T H / sigma^2 of the winner) does not wait on two
// dependent HBM loads. Measured r06 (profiles/r06/amab2): k_active_match 0.89 /
// 0.99 ms against 0.91 without, single sequence 0.967 against 0.961: off.
#ifndef AM_PREFETCH
#define AM_PREFETCH 0
#endif
struct Cands {
    int16_t* slot;   // pool slot drawn
    int32_t* tries;  // rand() calls from the round start up to this acceptance
    double* score;   // logDet(curMat + ObsMat)
    int16_t* match;  // keypoint OnePoint would claim, -1
    int16_t* dist;
    uint8_t* alive;  // still in the heap
};

// True when a lower lane of the wave holds the same value (the earlier try of
// a batch on the same column wins). Values below 2^nbits: the lanes holding
// the same value are the intersection, over the bits, of the lanes that agree
// with this lane on that bit (one ballot per bit: nbits ballots instead of 63
// lane reads). Called with every lane of the wave active (an inactive lane's
// bits would read as zeros).
__device__ __forceinline__ bool dup_of_lower_lane(int v, int nbits) {
    const int lane = threadIdx.x;
    unsigned long long same = __ballot(1);
    for (int b = 0; b < nbits; b++) {
        const unsigned long long ones = __ballot((v >> b) & 1);
        same &= ((v >> b) & 1) ? ones : ~ones;
    }
    return (same & ((1ull << lane) - 1ull)) != 0ull;
}
__device__ __forceinline__ int bits_for(int n) {  // 2^bits_for(n) >= n
    return n <= 1 ? 1 : 32 - __clz(n - 1);
}

// One batch of 64 tries: tries are accepted in order when their column was not
// visited this round and not drawn earlier in the batch; accepted columns are
// marked visited at once (unused ones are unmarked at the round end). A draw
// fails after MAX_RANDOM_QUERY_TIME rejected tries: *exh_at = tries count then.
// The batch's start history and words are left in (s0, o0): the round's
// commit advances the RNG from the batch holding its last call.
__device__ int draw_batch(uint32_t& s, uint32_t& s0, uint32_t& o0, int& tries, int& run, int N, int round,
                          const Pool& P, int16_t* vis,
                          const Cands& C, int nc, int* exh_at, const RCoef& coef, int sbits) {
    const int lane = threadIdx.x;
    AM_C(8, 1);
    const uint32_t o = rng_word(s, coef);
    const int j = (int)((o >> 1) % (uint32_t)N);
    const int sl = pool_select(P, j);
    // an earlier try of this batch that drew the same column wins
    const bool dup = dup_of_lower_lane(sl, sbits);  // all lanes: no short circuit
    const bool acc = vis[sl] < round && !dup;
    const unsigned long long m = __ballot(acc);
    const int a0 = m ? __ffsll((long long)m) - 1 : 64;
    int got = 0;
    if (run + a0 >= MAX_RANDOM_QUERY_TIME) {  // the next draw gives up inside this batch
        *exh_at = tries + (MAX_RANDOM_QUERY_TIME - run);
    } else {
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        if (acc) {
            C.slot[nc + rank] = (int16_t)sl;
            C.tries[nc + rank] = tries + lane + 1;
            vis[sl] = (int16_t)round;
        }
        got = __popcll(m);
        if (m) {
            run = __builtin_amdgcn_readfirstlane(__clzll((long long)m));  // rejected tries after the last acceptance
        } else {
            run += 64;
        }
    }
    s0 = s;
    o0 = o;
    s = rng_advance(s, o, 64);
    tries += 64;
    am_sync();
    return __builtin_amdgcn_readfirstlane(got);
}

// One-point state of every pool slot (the k_onepoint_pre result, refreshed
// when a claim hits one of its holders): keypoint it would claim (-1: none),
// distance, first- and second-place holders.
struct SlotMatch {
    int16_t* match;
    int16_t* dist;
    int16_t* h1;
    int16_t* h2;
};

// The slot's one-point result under the current claims: rescanned (and
// stored back) when a keypoint holding first or second place was claimed
// since it was computed.
__device__ __forceinline__ int slot_match(const ActiveArgs& A, const FrameConst& fc, int f, const SlotMatch& SM,
                                          int sl, int q, const int* cell_start, const int* items, const int* claim,
                                          const gf_keypoint* K, const uint8_t* D, int& md) {
    int mi = SM.match[sl];
    md = SM.dist[sl];
    const int h1 = SM.h1[sl], h2 = SM.h2[sl];
    if ((h1 >= 0 && claim[h1] >= 0) || (h2 >= 0 && claim[h2] >= 0)) {
        int n1, n2;
#ifdef GF_AM_STAMP
        atomicAdd(&g_am_stamp[11], 1ull);
#endif
        one_point_scan(A, fc, f, q, cell_start, items, claim, KpGlobal{K, D}, mi, md, n1, n2);
        if (mi < 0) md = 0;
        SM.match[sl] = (int16_t)mi;
        SM.dist[sl] = (int16_t)md;
        SM.h1[sl] = (int16_t)n1;
        SM.h2[sl] = (int16_t)n2;
    }
    return mi;
}

__device__ void eval_cands(const ActiveArgs& A, const FrameConst& fc, int f, const Cands& C, int c0, int c1,
                           const int16_t* lmk, const SlotMatch& SM, const double* cur, const double* info,
                           const double* info_lt,
                           const uint16_t* lq, const int32_t* rmp, const int* cell_start, const int* items,
                           const int* claim, const gf_keypoint* K, const uint8_t* D, const double* Hm) {
    AM_C(9, 1);
    AM_C(10, c1 - c0);
#if AM_PREFETCH
    double pf = 0.0;
#endif
    for (int c = c0 + threadIdx.x; c < c1; c += AW) {
        const int sl = C.slot[c];
        const int q = lmk[sl];
        // the slot's info / H row: staged at the pool build (lq_stage), else through the remap
        const long long qi = A.lq_stage ? (long long)lq[sl] : (rmp ? rmp[q] : q);
#if AM_PREFETCH
        // the commit's inputs, fetched while the round is still drawing: the
        // H row's two cache lines into the caches (read again only if this
        // candidate wins the round)
        pf += gfd::ldg(Hm + 14LL * qi) + gfd::ldg(Hm + 14LL * qi + 13);
#endif
        C.score[c] = logdet_sum_lower_packed(cur, info_lt + 32LL * qi, info + 49LL * qi);
        int md;
        const int mi = slot_match(A, fc, f, SM, sl, q, cell_start, items, claim, K, D, md);
        C.match[c] = (int16_t)mi;
#if AM_PREFETCH
        // the claimed keypoint's octave (the commit's sigma^2, < 16 levels) in
        // bits 12..15 of the distance (a Hamming distance <= 256)
        C.dist[c] = (int16_t)(md | (mi >= 0 ? K[mi].octave & 15 : 0) << 12);
#else
        C.dist[c] = (int16_t)md;
#endif
        C.alive[c] = 0;
    }
#if AM_PREFETCH
    if (pf == -1.2345678e-300) A.err[f] = 9;  // keeps the touch loads (a value no H row sums to)
#endif
    am_sync();
}

// A round in which no pool entry can be matched any more: every draw fails
// its one-point match, so the heap order no longer matters and the round
// (and runActiveMapMatching) ends when MAX_RANDOM_QUERY_TIME draws in a row
// hit visited columns (Observability.cc:1347-1359, 1437-1440). Only the
// accepted draws (one logDet each) and the rand() calls are observable; both
// follow from the column sequence alone, so this replays the draws on a
// column bitmask without evaluating anything. sd/tries/run continue the
// round's draw state; on return sd is the rand() state after exactly
// exh_at calls from the round start.
__device__ void exhaust_draws(uint32_t& sd, int tries, int run, int N, unsigned long long* colvis, int& nacc,
                              int& exh_at, const RCoef& coef) {
    while (true) {
        const uint32_t o = rng_word(sd, coef);
        const int j = (int)((o >> 1) % (uint32_t)N);
        const bool dup = dup_of_lower_lane(j, bits_for(N));
        const bool acc = !((colvis[j >> 6] >> (j & 63)) & 1ull) && !dup;
        const unsigned long long m = __ballot(acc);
        const int a0 = m ? __ffsll((long long)m) - 1 : 64;
        if (run + a0 >= MAX_RANDOM_QUERY_TIME) {
            const int k = MAX_RANDOM_QUERY_TIME - run;  // tries of this batch before the draw gives up
            exh_at = tries + k;
            sd = rng_advance(sd, o, k);
            am_sync();
            return;
        }
        if (acc) atomicOr(&colvis[j >> 6], 1ull << (j & 63));
        nacc += __popcll(m);
        run = m ? __clzll((long long)m) : run + 64;
        sd = rng_advance(sd, o, 64);
        tries += 64;
        am_sync();
    }
}

// Sort the wave's (score, candidate) pairs by score, descending; lanes with
// candidate < 0 sort last. Bitonic over 64 lanes.
__device__ __forceinline__ void wave_sort_desc(double& hs, int& hc) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const double os = __shfl_xor(hs, j, 64);
            const int oc = __shfl_xor(hc, j, 64);
            // "other before mine" in descending order
            const bool ogt = oc >= 0 && (hc < 0 || os > hs);
            const bool olt = hc >= 0 && (oc < 0 || os < hs);
            const bool keep_first = ((lane & j) == 0) == ((lane & k) == 0);
            if (keep_first ? ogt : olt) {
                hs = os;
                hc = oc;
            }
        }
    }
}

// The live set as K registers per lane, position p = 64 r + lane, sorted by
// score descending (positions past the set hold candidate -1 and sort last).
template <int K>
struct LiveSet {
    double s[K];
    int c[K];
    int m[K];  // the candidate's one-point match was found
};

__device__ __forceinline__ bool before_desc(double as, int ac, double bs, int bc) {  // a sorts before b
    return ac >= 0 && (bc < 0 || as > bs);
}

template <int K>
__device__ __forceinline__ void live_cmpx(LiveSet<K>& L, int r0, int r1, bool desc_first) {
    // registers r0 < r1 of one lane: position r0 gets the earlier one when desc_first
    const bool sw = desc_first ? before_desc(L.s[r1], L.c[r1], L.s[r0], L.c[r0])
                               : before_desc(L.s[r0], L.c[r0], L.s[r1], L.c[r1]);
    if (sw) {
        const double ts = L.s[r0];
        const int tc = L.c[r0];
        L.s[r0] = L.s[r1];
        L.c[r0] = L.c[r1];
        L.s[r1] = ts;
        L.c[r1] = tc;
    }
}

// Bitonic sort of the 64 K positions (payload: candidate; match flags are
// loaded after the sort).
template <int K>
__device__ __forceinline__ void live_sort(LiveSet<K>& L) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int k = 2; k <= 64 * K; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64) {
                const int rj = j >> 6;
#pragma unroll
                for (int r = 0; r < K; r++) {
                    if (r & rj) continue;
                    const bool asc_block = ((64 * r + lane) & k) != 0;  // this block sorts ascending
                    live_cmpx<K>(L, r, r | rj, !asc_block);
                }
            } else {
#pragma unroll
                for (int r = 0; r < K; r++) {
                    const double os = __shfl_xor(L.s[r], j, 64);
                    const int oc = __shfl_xor(L.c[r], j, 64);
                    const int p = 64 * r + lane;
                    const bool ogt = before_desc(os, oc, L.s[r], L.c[r]);
                    const bool olt = before_desc(L.s[r], L.c[r], os, oc);
                    const bool keep_first = ((p & j) == 0) == ((p & k) == 0);
                    if (keep_first ? ogt : olt) {
                        L.s[r] = os;
                        L.c[r] = oc;
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ double rlane(double v, int l) {  // lane l's value (l uniform)
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

__device__ __forceinline__ double rl0(double v) {  // lane 0's value
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 0);
    return __builtin_bit_cast(double, (uint64_t)hi << 32 | lo);
}

// lane i <- lane i + 1 (lane 63 keeps its own). A cross-lane permute: the DPP
// wavefront shifts (wave_shl) are gone from gfx90a on — the encoding still
// assembles for gfx950 but moves nothing, so every neighbour compare saw a
// tie and each round fell back to the heap replay.
__device__ __forceinline__ int dpp_next(int v) { return __shfl_down(v, 1, 64); }

__device__ __forceinline__ double dpp_next(double v) { return __shfl_down(v, 1, 64); }

// Heap top of the live candidates: the arg-max, unless the maximum is tied
// or a score is NaN, when std::priority_queue's order is reproduced by
// replaying its push/pop history (sz pushes, then pop/push pairs) exactly.
// The live candidates are the al[0 .. na) list (na = sz: every pop is
// followed by its replacement, which takes the popped entry's place), so a
// top costs one pass over at most sz entries, not over every draw so far.
// *pos = the top's place in al.
__device__ int wave_top(const Cands& C, const int16_t* al, int na, int sz, int npop, int16_t* rheap, int* s_res,
                        int* pos) {
    const int lane = threadIdx.x;
    double best = -INFINITY;
    int bi = -1, nan = 0;
    for (int i = lane; i < na; i += AW) {
        const double sc = C.score[al[i]];
        if (sc != sc) {
            nan = 1;
        } else if (bi < 0 || sc > best) {
            best = sc;
            bi = i;
        }
    }
    double gb = best;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) gb = fmax(gb, __shfl_xor(gb, o, 64));
    int cnt;
    if (na <= AW) {
        cnt = __popcll(__ballot(bi >= 0 && best == gb));
    } else {
        int c2 = 0;
        for (int i = lane; i < na; i += AW) c2 += C.score[al[i]] == gb;
        cnt = gfd::warp_sum(c2);
    }
    if (__ballot(nan) == 0ull && cnt == 1) {
        const unsigned long long m = __ballot(bi >= 0 && best == gb);
        const int p = __shfl(bi, __ffsll((long long)m) - 1, 64);
        *pos = p;
        return al[p];
    }
    if (lane == 0) {
        int hn = 0;
        const IdxLess cmp{C.score};
        for (int c = 0; c < sz; c++) {
            rheap[hn++] = (int16_t)c;
            gfsel::push_heap(rheap, hn, cmp);
        }
        for (int p = 0; p < npop; p++) {
            gfsel::pop_heap(rheap, hn, cmp);
            hn--;
            rheap[hn++] = (int16_t)(sz + p);
            gfsel::push_heap(rheap, hn, cmp);
        }
        *s_res = rheap[0];
    }
    am_sync();
    const int t = __builtin_amdgcn_readfirstlane(*s_res);
    int p = -1;
    for (int i0 = 0; i0 < na && p < 0; i0 += AW) {
        const unsigned long long m = __ballot(i0 + lane < na && al[i0 + lane] == t);
        if (m) p = i0 + __ffsll((long long)m) - 1;
    }
    *pos = p;
    return t;
}

#ifdef GF_AM_STAMP  // diagnostic build only: shader cycles per phase, summed over frames
#define AM_T(k)                                                               \
    do {                                                                      \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime();        \
        if (threadIdx.x == 0) atomicAdd(&g_am_stamp[k], now_ - am_last_);     \
        am_last_ = now_;                                                      \
    } while (0)
#else
#define AM_T(k) (void)0
#endif

// AM_SLOTS: the heap loop of a round (live set <= 64, no ties) by slot
// assignment instead of one pop at a time. std::priority_queue pops the
// largest live score; a failed top is replaced by the next draw, so draw i
// (i >= 1 after the round's sz initial ones) joins at pop time i. Pops in
// score order to the earliest free time are a unit-job schedule: an entry of
// score v joining at time a leaves at the first time t >= a at which every
// higher entry that joined by t has left, i.e. the first t >= a with
// x_t <= v (t >= 1) and #{initial > v} + #{x_1..x_t > v} <= t; that is the
// c-th time at which the draw is not above v, c = #{initial > v} (t = 0 when
// c = 0). The round ends at the first time whose entry is matchable: T = min
// over matchable entries of their time, T pops, the entries with time < T
// popped. One window of up to 64 draws costs one pass of broadcast LDS
// compares instead of up to 64 dependent pop steps; a tie or NaN hands the
// round to the exact heap replay as before.
#ifndef AM_SLOTS
#define AM_SLOTS 1
#endif
// AM_SORTED_WIDE: live sets of 65..256 candidates kept sorted in 2 / 4
// registers per lane (sorted_loop); off, such rounds (initial subsets above
// 64: num_to_match small against the pool) take the general wave_top loop.
// r06: with the loop's match-flag load behind a short-circuit branch, the
// register allocator put spill copies of live-through values (the rand()-call
// counter among them) in that branch's join block before its exec restore, so
// lanes outside the branch kept stale copies. The loads are
// unconditional now; tests/test_isa_guard.py checks the compiled kernels for
// the pattern.
#ifndef AM_SORTED_WIDE
#define AM_SORTED_WIDE 1
#endif
// AM_WOCT: the commit's per-octave weight from LDS (made at kernel start)
// instead of a kernel-argument load, a square root and a division per claim
#ifndef AM_WOCT
#define AM_WOCT 1
#endif
#ifndef AM_SB
#define AM_SB 16  // slot_loop: live / window scores per batch of broadcast reads
#endif
// LDS hand-over inside the one-wave workgroup
__device__ __forceinline__ void wave_sync_lds() { am_sync(); }

// position of the k-th (1-based) set bit of m, 64 if fewer
__device__ __forceinline__ int kth_bit(unsigned long long m, int k) {
    if (k <= 0 || __popcll(m) < k) return 64;
    int pos = 0, r = k - 1;
#pragma unroll
    for (int half = 32; half >= 1; half >>= 1) {
        const int c = __popcll(m & ((1ull << half) - 1ull));
        if (r >= c) {
            r -= c;
            m >>= half;
            pos += half;
        }
    }
    return pos;
}

__device__ __forceinline__ void active_match_body(const ActiveArgs& A, const int f) {
#ifdef GF_AM_STAMP
    unsigned long long am_last_ = __builtin_amdgcn_s_memtime();
    const unsigned long long am_start_ = am_last_;
#endif
    extern __shared__ __align__(16) uint8_t smem[];
    // sized for this launch: PC = pool capacity (map-list capacity rounded to 64,
    // at most POOL_MAX), claims for kp_cap keypoints
    const int PC = A.pool_cap;
    // CC: a round's drawn candidates (sz + pops + the last batch's spare
    // draws, usually ~100); a frame whose round would draw past CC returns
    // before writing its outputs and the overflow pass redoes it (as a pool
    // past PC does)
#if AM_CC
    const int CC = A.cand_cap;
#else
    const int CC = PC;
#endif
#ifdef GF_AM_GUARD  // diagnostic build: 256 sentinel bytes below the dynamic arrays, checked at the end
    uint32_t* guard = (uint32_t*)smem;
    guard[threadIdx.x] = 0xa5a5a5a5u + threadIdx.x;
    double* c_score = (double*)(smem + 256);                               // CC
#else
    double* c_score = (double*)smem;                                       // CC
#endif
    unsigned long long* pbits = (unsigned long long*)(c_score + CC);       // 64
    int* claim = (int*)(pbits + 64);                                       // kp_cap
    int* ppre = claim + A.kp_cap;                                          // 65 (+3 pad)
    int32_t* c_tries = ppre + 68;                                          // CC
    int16_t* lmk = (int16_t*)(c_tries + CC);                               // PC: map point of each slot
    int16_t* vis = lmk + PC;                                               // PC: lmkVisited per slot
    int16_t* c_slot = vis + PC;                                            // CC
    int16_t* c_match = c_slot + CC;                                        // CC
    int16_t* c_dist = c_match + CC;                                        // CC
    int16_t* rheap = c_dist + CC;                                          // PC: replay heap
    int16_t* sm_match = rheap + PC;                                        // PC: one-point state per slot
    int16_t* sm_dist = sm_match + PC;                                      // PC
    int16_t* sm_h1 = sm_dist + PC;                                         // PC
    int16_t* sm_h2 = sm_h1 + PC;                                           // PC
    int16_t* alv = sm_h2 + PC;                                             // PC: the live candidates (heap set)
    uint8_t* c_alive = (uint8_t*)(alv + PC);                               // CC
    uint16_t* lq = (uint16_t*)(((uintptr_t)(c_alive + CC) + 1) & ~(uintptr_t)1);  // PC (lq_stage): info / H row of each slot
    __shared__ double cur[49];
    __shared__ unsigned long long colvis[64];  // exhausting round: visited columns
    __shared__ int s_res, s_exh, s_nsucc;  // s_nsucc: 0 = no pool slot can be matched
#ifdef AM_LSIG  // diagnostic: the level sigma^2 from an LDS copy at the commit
    __shared__ float s_sig2[16];
#endif
#if AM_WOCT
    __shared__ double s_woct[16];
#endif
#if AM_SLOTS
    __shared__ __align__(16) double s_lsc[64];  // slot_loop: live scores, lane order (-inf past sz)
    __shared__ __align__(16) double s_xsc[64];  // slot_loop: the window's scores (-inf past W)
    __shared__ unsigned long long s_rk[2];  // slot_loop: ranks seen (distinctness)
    __shared__ int16_t s_live[128];         // slot_loop: next live set
#endif

    const int lane = threadIdx.x;
    const FrameConst& fc = A.fc;
    const int n = min(A.n[f], A.kp_cap);
    const int m = min(A.m[f], 32767);
    if (m == 0) {  // not this frame's branch: nothing to do, no LDS touched
        if (lane == 0) {
            A.nleft[f] = 0;
            A.nmatched[f] = 0;
            if (A.nldet) A.nldet[f] = 0;
        }
        return;
    }
    const gf_keypoint* K = A.kps + (long long)f * A.kp_cap;
    const uint8_t* D = A.desc + (long long)f * A.kp_cap * 32;
    int32_t* kp2mp = A.kp2mp + (long long)f * A.kp_cap;
    int32_t* left = A.left + (long long)f * A.mp_cap;
    const int num_to_match = A.num_to_match[f];
    // time cap (Observability.cc:1260, 1275-1277): time_for_match from
    // time_Mat_Online (Tracking.cc:3311 -> here) and time_Viz; <= 0 is the early exit
    const bool clocked = A.ck.mat_t0 != nullptr;
    unsigned long long t_am0 = 0;
    long long am_cap = 0;
    long long* rec = clocked ? A.ck.rec + (long long)f * A.ck.stride : nullptr;
    if (clocked) {
        t_am0 = __builtin_amdgcn_s_memrealtime();
        const long long mat = A.ck.syn ? A.ck.syn[0] : (long long)(t_am0 - A.ck.mat_t0[f]);
        am_cap = A.ck.match_ticks - mat - A.ck.viz[f];
        if (lane == 0) {
            rec[GF_CK_MAT_ONLINE] = mat;
            rec[GF_CK_AM_CUT] = -1;
        }
    }
    bool cut = false;
    bool cabort = false;  // a round would draw past CC: the overflow pass redoes the frame
    // the keypoint grid comes from k_onepoint_pre (HBM; only rescans read it)
    const int* cell_start = A.grid_cs + (long long)f * (NCELLS + 1);
    const int* items = A.grid_items + (long long)f * A.kp_cap;
    for (int i = lane; i < n; i += AW) claim[i] = kp2mp[i];
#ifdef AM_LSIG
    if (lane < 16) s_sig2[lane] = A.sigma2[lane];
#endif
#if AM_WOCT
    if (lane < 16) {  // the commit's weight per octave, s2 / (s2 s2) with s2 = sqrt(sigma^2), made once
        const double s2 = sqrt((double)A.sigma2[lane]);
        s_woct[lane] = s2 / (s2 * s2);
    }
#endif
    const int32_t* rmp = A.remap ? A.remap + (long long)f * A.mp_cap : nullptr;
    // a slot's info / H row: staged at the pool build, or read through the remap
    auto row_of = [&](int sl) -> long long {
        if (A.lq_stage) return lq[sl];
        const int q = lmk[sl];
        return rmp ? rmp[q] : q;
    };
    RCoef rcoef;  // this lane's row of the rand() recurrence
    rcoef.load();
    am_sync();
    AM_T(0);

    // ---- pool: in-view, updated map points in list order (Observability.cc:1285-1306)
    const bool early = (m == 0 || num_to_match <= 0 || (clocked && am_cap <= 0));
    int N = 0;
    for (int base = 0; base < m; base += AW) {
        const int i = base + lane;
        bool in = false, upd = false;
        int rq = i;
        if (i < m) {
            const long long g = (long long)f * A.mp_cap + i;
            in = A.views[g].in_view;
            upd = A.updated[g];
            if (A.remap && A.lq_stage) rq = A.remap[g];  // (loaded beside the flags: no extra round trip)
        }
        const bool take = in && (early || upd);
        const unsigned long long msk = __ballot(take);
        const int o = N + __popcll(msk & ((1ull << lane) - 1ull));
        if (take) {
            if (early) {
                left[o] = i;
            } else if (o < PC) {
                lmk[o] = (int16_t)i;
                if (A.lq_stage) lq[o] = (uint16_t)rq;
                vis[o] = -1;
            }
        }
        N += __popcll(msk);
    }
    if (early) {
        if (lane == 0) {
            A.nleft[f] = N;
            A.nmatched[f] = 0;
            if (A.nldet) A.nldet[f] = 0;
        }
        return;
    }
    if (N > PC) {  // nothing written yet: the overflow pass redoes this frame with a full pool
        if (lane == 0) {
            if (A.pass == 1) A.ovf[1 + atomicAdd(A.ovf, 1)] = f;
            else A.err[f] = 2;
        }
        return;
    }
    const Pool P{pbits, ppre};
#ifdef GF_AM_CHECK
    const int N0 = N;
#endif
    const int sbits = bits_for(N);  // pool slots are < N (they never move)
    {
        const int lo = lane * 64;
        pbits[lane] = N >= lo + 64 ? ~0ull : (N > lo ? ((1ull << (N - lo)) - 1ull) : 0ull);
        am_sync();
        pool_prefix(P);
    }
    const SlotMatch SM{sm_match, sm_dist, sm_h1, sm_h2};
    {  // one-point state of every slot from the precompute; matchable slots counted
        int ns = 0;
        for (int sl = lane; sl < N; sl += AW) {
            const OnePre p = A.pre[(long long)f * A.mp_cap + lmk[sl]];
            sm_match[sl] = p.idx;
            sm_dist[sl] = p.dist;
            sm_h1[sl] = p.holder1;
            sm_h2[sl] = p.holder2;
            ns += p.idx >= 0;
        }
        ns = gfd::warp_sum(ns);
        if (lane == 0) s_nsucc = ns;
    }
    if (lane < 49) cur[lane] = A.base[49LL * f + lane];
    uint32_t rs;  // RNG history (oldest first) at the last committed rand() call
    {
        const int f0 = A.rng[f].f;
        rs = lane < 31 ? (uint32_t)A.rng[f].state[(f0 + lane) % 31] : 0u;
    }
    // rand() calls, claims, logDet calls of the reference (one per draw): wave
    // counters, pinned uniform (scalar registers) at every update
    int used = 0, nm = 0, nld = 0;
    am_sync();
    AM_T(1);

    const Cands C{c_slot, c_tries, c_score, c_match, c_dist, c_alive};
    const int S = (int)((float)N / (float)num_to_match * 1.0);
    const int nw0 = (N + 63) >> 6;  // pool words (slots never move; only bits clear)
    bool nsucc_valid = true;        // s_nsucc counts the matchable pool slots
    int last_npop = 0;
    const double* info = A.info + (long long)f * A.mp_cap * 49;
    const double* info_lt = A.info_lt + (long long)f * A.mp_cap * 32;
    const double* Hm = A.H + (long long)f * A.mp_cap * 14;

    for (int round = 0; round < num_to_match; ++round) {
        AM_C(12, 1);
        const int sz = __builtin_amdgcn_readfirstlane(min(S, N));
        if (sz == 0) break;  // empty heap: early termination
        if (clocked) {
            // the time cap, read at the round's start; the reference checks it
            // after each accepted draw (Observability.cc:1362-1370), so a late
            // round ends at its first accepted draw: matches so far stand, no
            // leftovers (the return skips mLeftMapPoints)
            const long long e = gfd::ck_elapsed(t_am0, A.ck.syn ? A.ck.syn + 2 : nullptr, round);
            if (lane == 0 && round < A.ck.rounds) rec[A.ck.off + round] = e;
            if (e > am_cap) {
                uint32_t sd = rs, s0, o0;
                int tries = 0, run = 0, nc = 0, exh_at = -1;
                while (nc < 1 && exh_at < 0) {
                    if (lane == 0) s_exh = -1;
                    am_sync();
                    nc = __builtin_amdgcn_readfirstlane(
                        nc + draw_batch(sd, s0, o0, tries, run, N, round, P, vis, C, nc, &s_exh, rcoef, sbits));
                    exh_at = __builtin_amdgcn_readfirstlane(s_exh);
                }
                // an accepted draw before the draws gave out: the cap fires there;
                // otherwise the draws gave out first (early termination, :1437)
                const int T = nc >= 1 ? __builtin_amdgcn_readfirstlane(C.tries[0]) : exh_at;
                for (int t = T; t > 0; t -= 64) rs = rng_advance(rs, rng_word(rs, rcoef), min(t, 64));
                used = __builtin_amdgcn_readfirstlane(used + T);
                if (nc >= 1) {
                    cut = true;
                    if (lane == 0) rec[GF_CK_AM_CUT] = round;
                }
                am_sync();
                break;
            }
        }
        // -- draws, ahead of need
        uint32_t sd = rs;
        int tries = 0, run = 0, nc = 0, evald = 0, exh_at = -1;
        uint32_t bs0 = 0u, bo0 = 0u, bs1 = 0u, bo1 = 0u;  // start history / words of the last two batches
        int nb = 0;                                      // batches drawn this round
        AM_T(6);
        if (!nsucc_valid && last_npop > sz) {
            // the last round had to pop: count the pool entries that can still be
            // matched (slots whose holders were claimed are scanned again)
            // pass 1, loads only: a slot whose holders are unclaimed keeps its
            // result. Only "none left" matters, so the walk stops at the first
            // word holding a known matchable slot (usually the first word)
            bool known = false;
            unsigned long long stale = 0ull;  // bit w: this lane's slot in word w needs a rescan
            for (int w = 0; w < nw0; w++) {
                const int sl = w * 64 + lane;
                if ((pbits[w] >> lane) & 1ull) {
                    const int h1 = sm_h1[sl], h2 = sm_h2[sl];
                    if ((h1 >= 0 && claim[h1] >= 0) || (h2 >= 0 && claim[h2] >= 0))
                        stale |= 1ull << w;
                    else
                        known |= sm_match[sl] >= 0;
                }
                if (__ballot(known)) break;
            }
            int ns = __ballot(known) ? 1 : 0;
            // pass 2: rescans, until a matchable slot turns up
            for (int w = 0; w < nw0 && !ns; w++) {
                int mi = -1;
                if ((stale >> w) & 1ull) {
                    int md;
                    mi = slot_match(A, fc, f, SM, w * 64 + lane, lmk[w * 64 + lane], cell_start, items, claim, K, D,
                                    md);
                }
                ns = __ballot(mi >= 0) ? 1 : 0;
            }
            if (lane == 0) s_nsucc = ns;
            nsucc_valid = true;
            am_sync();
        }
        AM_T(7);
        if (nsucc_valid && __builtin_amdgcn_readfirstlane(s_nsucc) == 0) {  // nothing left to match: the round draws until the draws give out
            colvis[lane] = 0ull;
            am_sync();
            int nacc = 0, ex = 0;
            exhaust_draws(sd, 0, 0, N, colvis, nacc, ex, rcoef);
            nld = __builtin_amdgcn_readfirstlane(nld + nacc);
            used = __builtin_amdgcn_readfirstlane(used + ex);
            rs = sd;
            AM_T(2);
            break;
        }
        while (nc < sz && exh_at < 0) {
            if (AM_CC && CC < N && nc + 64 > CC) {  // the batch could write past the candidate arrays
                cabort = true;
                break;
            }
            if (lane == 0) s_exh = -1;
            am_sync();
            {
                uint32_t s0, o0;
                nc = __builtin_amdgcn_readfirstlane(nc + draw_batch(sd, s0, o0, tries, run, N, round, P, vis, C, nc,
                                                                    &s_exh, rcoef, sbits));
                bs0 = nb & 1 ? bs0 : s0;
                bo0 = nb & 1 ? bo0 : o0;
                bs1 = nb & 1 ? s0 : bs1;
                bo1 = nb & 1 ? o0 : bo1;
                nb++;
            }
            exh_at = __builtin_amdgcn_readfirstlane(s_exh);
        }
        AM_T(2);
        if (cabort) break;
        if (nc < sz) {  // the initial subset could not be completed
            nld = __builtin_amdgcn_readfirstlane(nld + nc);
            for (int c = lane; c < nc; c += AW) vis[C.slot[c]] = -1;
            used = __builtin_amdgcn_readfirstlane(used + exh_at);
            for (int T = exh_at; T > 0; T -= 64) rs = rng_advance(rs, rng_word(rs, rcoef), min(T, 64));
            break;
        }
        eval_cands(A, fc, f, C, 0, nc, lmk, SM, cur, info, info_lt, lq, rmp, cell_start, items, claim, K, D, Hm);
        evald = nc;
        AM_T(3);
        // -- the sequential heap loop, now over known scores and match results.
        // While the live set fits the wave and no two live scores tie (NaN
        // counts as a tie), it is kept sorted in registers, lane 0 = heap top:
        // a pop is a one-lane shift and a rank by ballot. Otherwise (or from
        // the first tie on) wave_top, with the exact heap replay for ties.
        int npop = 0, top = -1, tpos = -1;
        bool exh = false, success = false;
        // (a) the live set sorted in registers (K per lane, position p = 64 r +
        // lane, descending): the top is position 0; a failed top is popped by
        // shifting positions 1.. down one (DPP wave_shl, plus the neighbouring
        // register's lane 0 for lane 63) and the replacement goes to the
        // place its rank (ballots) gives. Ties (and NaN) leave for (b), where
        // the heap replay fixes their order. Alive flags are written at the end.
        auto draw_eval = [&](int rep) {
            if (rep >= nc && exh_at < 0) {
                AM_T(4);
                while (rep >= nc && exh_at < 0) {
                    if (AM_CC && CC < N && nc + 64 > CC) {
                        // past the candidate arrays: no draw, so the pop loop
                        // ends as on exhausted draws (no claim, no global write
                        // follows) and the round loop stops at the check after
                        // it; the overflow pass takes the frame
                        cabort = true;
                        break;
                    }
                    if (lane == 0) s_exh = -1;
                    am_sync();
                    {
                uint32_t s0, o0;
                nc = __builtin_amdgcn_readfirstlane(nc + draw_batch(sd, s0, o0, tries, run, N, round, P, vis, C, nc,
                                                                    &s_exh, rcoef, sbits));
                bs0 = nb & 1 ? bs0 : s0;
                bo0 = nb & 1 ? bo0 : o0;
                bs1 = nb & 1 ? s0 : bs1;
                bo1 = nb & 1 ? o0 : bo1;
                nb++;
            }
                    exh_at = __builtin_amdgcn_readfirstlane(s_exh);
                }
                AM_T(2);
            }
            if (rep < nc && rep >= evald) {
                AM_T(4);
                eval_cands(A, fc, f, C, evald, nc, lmk, SM, cur, info, info_lt, lq, rmp, cell_start, items, claim, K, D, Hm);
                evald = nc;
                AM_T(3);
            }
        };
#if AM_SLOTS
        // (a') the live set (<= 64, lane j: candidate lc) against the next
        // window of draws, by slot assignment (AM_SLOTS above). 1: round
        // decided (success / exh set), 0: leave for (b) with alv / C.alive set.
        auto slot_loop = [&]() -> int {
            constexpr int INF = 1 << 20;
            int lc = lane < sz ? lane : -1;
            while (true) {
                const int rep0 = sz + npop;
                draw_eval(rep0);
                if (nc - rep0 < 16 && exh_at < 0 && !cabort) draw_eval(nc);  // a useful window
                if (evald < nc && !cabort) {
                    AM_T(4);
                    eval_cands(A, fc, f, C, evald, nc, lmk, SM, cur, info, info_lt, lq, rmp, cell_start, items, claim, K,
                               D, Hm);
                    evald = nc;
                    AM_T(3);
                }
                if (cabort) {
                    exh = true;
                    return 1;
                }
                const int W = __builtin_amdgcn_readfirstlane(max(min(nc - rep0, 64), 0));
                const bool v0 = lc >= 0, v1 = lane < W;
                const int xc = v1 ? rep0 + lane : -1;
                const double lv = v0 ? C.score[lc] : 0.0, xv = v1 ? C.score[xc] : 0.0;
                const bool m0 = v0 && C.match[lc] >= 0, m1 = v1 && C.match[xc] >= 0;
                s_lsc[lane] = v0 ? lv : -INFINITY;  // -inf is above nothing
                s_xsc[lane] = v1 ? xv : -INFINITY;
                if (lane < 2) s_rk[lane] = 0ull;
                wave_sync_lds();
                const bool nan = (v0 && lv != lv) || (v1 && xv != xv);
                // c = #{live > v}, g = {window draws above v}: broadcast LDS
                // reads, AM_SB scores per batch in flight, no per-entry branch
                int c0 = 0, c1 = 0;
                uint32_t g0l = 0u, g0h = 0u, g1l = 0u, g1h = 0u;
#pragma unroll
                for (int kb = 0; kb < 64; kb += AM_SB) {
                    if (kb < sz) {
                        double lk[AM_SB];
#pragma unroll
                        for (int u = 0; u < AM_SB; u += 2) {
                            const double2 d2 = *reinterpret_cast<const double2*>(&s_lsc[kb + u]);
                            lk[u] = d2.x;
                            lk[u + 1] = d2.y;
                        }
#pragma unroll
                        for (int u = 0; u < AM_SB; u++) {
                            c0 += lk[u] > lv;
                            c1 += lk[u] > xv;
                        }
                    }
                    if (kb < W) {
                        double xk[AM_SB];
#pragma unroll
                        for (int u = 0; u < AM_SB; u += 2) {
                            const double2 d2 = *reinterpret_cast<const double2*>(&s_xsc[kb + u]);
                            xk[u] = d2.x;
                            xk[u + 1] = d2.y;
                        }
#pragma unroll
                        for (int u = 0; u < AM_SB; u++) {
                            const int k = kb + u;
                            if (k < 32) {
                                g0l |= xk[u] > lv ? 1u << k : 0u;
                                g1l |= xk[u] > xv ? 1u << k : 0u;
                            } else {
                                g0h |= xk[u] > lv ? 1u << (k - 32) : 0u;
                                g1h |= xk[u] > xv ? 1u << (k - 32) : 0u;
                            }
                        }
                    }
                }
                const unsigned long long g0 = (unsigned long long)g0h << 32 | g0l,
                                         g1 = (unsigned long long)g1h << 32 | g1l;
                // distinct scores: every entry's rank (#{entries above}) once
                const int r0 = c0 + __popcll(g0), r1 = c1 + __popcll(g1);
                if (v0) atomicOr(&s_rk[r0 >> 6], 1ull << (r0 & 63));
                if (v1) atomicOr(&s_rk[r1 >> 6], 1ull << (r1 & 63));
                wave_sync_lds();
                const bool tie = __popcll(s_rk[0]) + __popcll(s_rk[1]) != sz + W;
                if (__ballot(nan) || tie) {  // (b) pops the rest exactly
                    for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
                    wave_sync_lds();
                    if (v0) {
                        alv[__popcll(__ballot(v0) & ((1ull << lane) - 1ull))] = (int16_t)lc;
                        C.alive[lc] = 1;
                    }
                    wave_sync_lds();
                    return 0;
                }
                // leaving times: draw k of the window joins (and may leave) at time k + 1
                const unsigned long long wm = W >= 64 ? ~0ull : ((1ull << W) - 1ull);
                const unsigned long long z0 = ~g0 & wm, z1 = ~g1 & wm;
                const int p0 = !v0 ? INF : c0 == 0 ? 0 : (kth_bit(z0, c0) < 64 ? kth_bit(z0, c0) + 1 : INF);
                int p1 = INF;
                if (v1) {
                    const int t = c1 == 0 ? 0 : (kth_bit(z1, c1) < 64 ? kth_bit(z1, c1) + 1 : INF);
                    p1 = t >= INF ? INF : max(t, lane + 1);
                }
                int T = min(m0 ? p0 : INF, m1 ? p1 : INF);
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) T = min(T, __shfl_xor(T, o, 64));
                T = __builtin_amdgcn_readfirstlane(T);
                const bool exhausted = T > W && exh_at >= 0 && rep0 + W >= nc;
                if (T <= W || exhausted) {
                    // decided: success at time T, or the draws gave out at time W
                    // (its top popped too, as the sequential loop does)
                    const int cut = T <= W ? T : W + 1;  // entries leaving before `cut` are popped
                    const int np = T <= W ? T : W;
                    if (T <= W) {
                        const unsigned long long w0m = __ballot(m0 && p0 == T), w1m = __ballot(m1 && p1 == T);
                        if (w0m) top = __builtin_amdgcn_readlane(lc, __ffsll((long long)w0m) - 1);
                        else top = rep0 + __ffsll((long long)w1m) - 1;
                        success = true;
                    } else {
                        exh = true;
                    }
                    npop = __builtin_amdgcn_readfirstlane(npop + np);
                    for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
                    wave_sync_lds();
                    if (v0 && p0 >= cut) C.alive[lc] = 1;
                    if (v1 && lane < np && p1 >= cut) C.alive[xc] = 1;
                    wave_sync_lds();
                    return 1;
                }
                // W pops (times 0 .. W - 1); the entries still live (time >= W) become the live set
                const bool k0l = v0 && p0 >= W, k1l = v1 && p1 >= W;
                const unsigned long long b0 = __ballot(k0l), b1 = __ballot(k1l);
                const unsigned long long below = (1ull << lane) - 1ull;
                if (k0l) s_live[__popcll(b0 & below)] = (int16_t)lc;
                if (k1l) s_live[__popcll(b0) + __popcll(b1 & below)] = (int16_t)xc;
                wave_sync_lds();
                lc = lane < sz ? (int)s_live[lane] : -1;
                npop = __builtin_amdgcn_readfirstlane(npop + W);
                wave_sync_lds();
            }
        };
#endif
        auto sorted_loop = [&](auto kk) -> int {  // 1: round decided, 0: leave for (b)
            constexpr int KR = decltype(kk)::value;
            LiveSet<KR> L;
            bool bad = false;
#pragma unroll
            for (int r = 0; r < KR; r++) {
                const int p = 64 * r + lane;
                L.c[r] = p < sz ? p : -1;
                const double sp = C.score[p];  // p < 64 kreg <= PC: in the array (loads unconditional)
                L.s[r] = p < sz ? sp : -INFINITY;
                bad |= p < sz && L.s[r] != L.s[r];
            }
            if (__ballot(bad)) return 0;
            live_sort<KR>(L);
            bool tie = false;
#pragma unroll
            for (int r = 0; r < KR; r++) {
                const double nx0 = dpp_next(L.s[r]);
                const double nx = lane < 63 ? nx0 : (r + 1 < KR ? rl0(L.s[r + 1 < KR ? r + 1 : r]) : -INFINITY);
                const int p = 64 * r + lane;
                tie |= p + 1 < sz && nx == L.s[r];
                const int mt = C.match[max(L.c[r], 0)];
                L.m[r] = (L.c[r] >= 0) & (mt >= 0);
            }
            if (__ballot(tie)) return 0;
            if constexpr (KR == 1) {
                // The live set stays in place: lane i keeps its candidate and
                // its rank (0 = heap top). A pop hands the top's lane to the
                // replacement: every live score above the replacement moves up
                // one rank, the others keep theirs, and the replacement takes
                // the rank a ballot counts. No lane moves, so a pop is a few
                // ballots and lane reads; the replacements' scores and match
                // flags come from a 64-candidate window in registers.
                double& ls = L.s[0];
                int& lc = L.c[0];
                int& lm = L.m[0];
                int rk = lane;  // sorted above: rank = lane
                const unsigned long long szm = sz >= 64 ? ~0ull : ((1ull << sz) - 1ull);
                int w0 = -64, wn = 0;  // window start, candidates drawn when it was filled
                double ws = 0.0;
                int wm = 0;
                while (true) {
                    const int tl = __ffsll((long long)(__ballot(rk == 0) & szm)) - 1;  // the top's lane
                    top = __builtin_amdgcn_readlane(lc, tl);
                    if (__builtin_amdgcn_readlane(lm, tl)) {
                        success = true;
                        break;
                    }
                    const int rep = sz + npop;  // the replacement draw
                    draw_eval(rep);
                    if (rep >= nc) {
                        exh = true;
                        lc = lane == tl ? -1 : lc;  // the top was popped
                        break;
                    }
                    if (rep >= w0 + 64 || rep >= wn) {
                        w0 = rep;
                        wn = nc;
                        ws = w0 + lane < nc ? C.score[w0 + lane] : 0.0;
                        wm = w0 + lane < nc ? C.match[w0 + lane] >= 0 : 0;
                    }
                    const double x = rlane(ws, rep - w0);
                    const int xm = __builtin_amdgcn_readlane(wm, rep - w0);
                    const unsigned long long live = szm & ~(1ull << tl);
                    if (x != x || (__ballot(ls == x) & live)) {  // a tie: (b) pops it exactly
                        npop = __builtin_amdgcn_readfirstlane(npop + 1);
                        for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
                        am_sync();
                        const bool lv = (live >> lane) & 1ull;
                        if (lv) {
                            alv[__popcll(live & ((1ull << lane) - 1ull))] = (int16_t)lc;
                            C.alive[lc] = 1;
                        }
                        if (lane == 0) {
                            alv[sz - 1] = (int16_t)rep;
                            C.alive[rep] = 1;
                        }
                        am_sync();
                        return 0;
                    }
                    const unsigned long long gt = __ballot(ls > x) & live;
                    rk = (gt >> lane) & 1ull ? rk - 1 : rk;
                    if (lane == tl) {
                        ls = x;
                        lc = rep;
                        lm = xm;
                        rk = __popcll(gt);
                    }
                    npop = __builtin_amdgcn_readfirstlane(npop + 1);
                }
                // alive flags of the candidates that entered: popped 0, live 1
                for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
                am_sync();
                if (lane < sz && lc >= 0) C.alive[lc] = 1;
                am_sync();
                return 1;
            }
            while (true) {
                top = __builtin_amdgcn_readlane(L.c[0], 0);
                if (__builtin_amdgcn_readlane(L.m[0], 0)) {
                    success = true;
                    break;
                }
                const int rep = sz + npop;  // the replacement draw
                draw_eval(rep);
                if (rep >= nc) {
                    exh = true;
                    break;
                }
                const double x = C.score[rep];
                const int xm = C.match[rep] >= 0;
                bool t2 = x != x;
                int rank = 0;
#pragma unroll
                for (int r = 0; r < KR; r++) {
                    const int p = 64 * r + lane;
                    const bool live = p >= 1 && p < sz;  // position 0 is the popped top
                    t2 |= __ballot(live && L.s[r] == x) != 0ull;
                    rank += __popcll(__ballot(live && L.s[r] > x));
                }
                if (t2) {  // hand the live set (positions 1.., then the replacement) to (b)
                    npop = __builtin_amdgcn_readfirstlane(npop + 1);
                    for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
                    am_sync();
#pragma unroll
                    for (int r = 0; r < KR; r++) {
                        const int p = 64 * r + lane;
                        if (p >= 1 && p < sz) {
                            alv[p - 1] = (int16_t)L.c[r];
                            C.alive[L.c[r]] = 1;
                        }
                    }
                    if (lane == 0) {
                        alv[sz - 1] = (int16_t)rep;
                        C.alive[rep] = 1;
                    }
                    am_sync();
                    return 0;
                }
                // new[p] = old[p + 1] for p < rank, new[rank] = the replacement
                double ns[KR];
                int nc2[KR], nm[KR];
#pragma unroll
                for (int r = 0; r < KR; r++) {
                    const double a = dpp_next(L.s[r]);
                    const int b2 = dpp_next(L.c[r]), m2 = dpp_next(L.m[r]);
                    const int rn = r + 1 < KR ? r + 1 : r;
                    const double a63 = r + 1 < KR ? rl0(L.s[rn]) : -INFINITY;
                    const int b63 = r + 1 < KR ? __builtin_amdgcn_readlane(L.c[rn], 0) : -1;
                    const int m63 = r + 1 < KR ? __builtin_amdgcn_readlane(L.m[rn], 0) : 0;
                    ns[r] = lane < 63 ? a : a63;
                    nc2[r] = lane < 63 ? b2 : b63;
                    nm[r] = lane < 63 ? m2 : m63;
                }
#pragma unroll
                for (int r = 0; r < KR; r++) {
                    const int p = 64 * r + lane;
                    if (p < rank) {
                        L.s[r] = ns[r];
                        L.c[r] = nc2[r];
                        L.m[r] = nm[r];
                    } else if (p == rank) {
                        L.s[r] = x;
                        L.c[r] = rep;
                        L.m[r] = xm;
                    }
                }
                npop = __builtin_amdgcn_readfirstlane(npop + 1);
            }
            // alive flags of the candidates that entered: popped 0, live 1
            for (int c = lane; c < sz + npop; c += AW) C.alive[c] = 0;
            am_sync();
#pragma unroll
            for (int r = 0; r < KR; r++) {
                const int p = 64 * r + lane;
                if (p < sz && !(exh && p == 0)) C.alive[L.c[r]] = 1;  // on exhaustion the top was popped
            }
            am_sync();
            return 1;
        };
        const int kreg = (sz + 63) >> 6;
        int decided = 0;
        (void)sorted_loop;
#if AM_SLOTS
        if (kreg == 1)
            decided = slot_loop();
#else
        if (kreg == 1)
            decided = sorted_loop(std::integral_constant<int, 1>{});
#endif
#if AM_SORTED_WIDE
        else if (kreg == 2)
            decided = sorted_loop(std::integral_constant<int, 2>{});
        else if (kreg <= 4)
            decided = sorted_loop(std::integral_constant<int, 4>{});
#endif
        if (!decided) {
            if (npop == 0) {  // (b) from the start: the initial live set
                for (int c = lane; c < sz; c += AW) {
                    C.alive[c] = 1;
                    alv[c] = (int16_t)c;
                }
                am_sync();
            }
            // (b) general: wave_top over the live list (ties replay the heap)
            while (true) {
                top = wave_top(C, alv, sz, sz, npop, rheap, &s_res, &tpos);
                if (C.match[top] >= 0) {
                    success = true;
                    break;
                }
                if (lane == 0) C.alive[top] = 0;  // heapSubset.pop()
                const int rep = sz + npop;       // the replacement draw
                draw_eval(rep);
                if (rep >= nc) {
                    exh = true;
                    break;
                }
                if (lane == 0) {
                    C.alive[rep] = 1;
                    alv[tpos] = (int16_t)rep;  // the replacement takes the popped entry's place
                }
                npop = __builtin_amdgcn_readfirstlane(npop + 1);
                am_sync();
            }
        }
        AM_T(4);
        if (cabort) break;
        // the successful top's H row and its keypoint's octave, loaded now so
        // that their latency overlaps the commit below
        double h_i = 0.0, h_j = 0.0, h_7i = 0.0, h_7j = 0.0;
        int oct_b = 0;
        if (!exh && lane < 49) {
            // (top is wave-uniform, so are the row and the octave: scalar bases)
            const double* Hq = Hm + 14LL * __builtin_amdgcn_readfirstlane((int)row_of(C.slot[top]));
            const int i = lane / 7, jj = lane % 7;
            h_i = Hq[i];
            h_j = Hq[jj];
            h_7i = Hq[7 + i];
            h_7j = Hq[7 + jj];
#if AM_PREFETCH
            oct_b = (C.dist[top] >> 12) & 15;
#else
            oct_b = K[C.match[top]].octave;
#endif
        }
        // -- commit: RNG calls actually made, visited marks of the used draws only
        const int nused = sz + npop;  // draws that happened
        nld = __builtin_amdgcn_readfirstlane(nld + nused);
        const int T = __builtin_amdgcn_readfirstlane(exh ? exh_at : C.tries[nused - 1]);
#ifdef GF_AM_CHECK
        {
            int bad = 0;
            for (int c = nused + lane; c < nc; c += AW) bad += C.slot[c] < 0 || C.slot[c] >= N0;
            for (int c = lane; c < nused; c += AW) bad += C.slot[c] < 0 || C.slot[c] >= N0;
            if (lane == 0 && N != ppre[64]) atomicAdd(&g_am_check[5], 1ull);
            bad = gfd::warp_sum(bad);
            if (lane == 0 && bad) atomicAdd(&g_am_check[1], (unsigned long long)bad);
            if (lane == 0 && !exh && (C.match[top] < 0 || C.match[top] >= n)) atomicAdd(&g_am_check[2], 1ull);
        }
        const uint32_t rs_prev = rs;
#endif
        for (int c = nused + lane; c < nc; c += AW) vis[C.slot[c]] = -1;
        used = __builtin_amdgcn_readfirstlane(used + T);
        if (T > 0 && (T - 1) / 64 >= nb - 2) {  // the batch holding call T is one of the last two
            const int b = (T - 1) / 64;
            rs = (b & 1) ? rng_advance(bs1, bo1, T - 64 * b) : rng_advance(bs0, bo0, T - 64 * b);
        } else {
            for (int t = T; t > 0; t -= 64) rs = rng_advance(rs, rng_word(rs, rcoef), min(t, 64));
        }
#ifdef GF_AM_CHECK
        {
            uint32_t rsl = rs_prev;
            for (int t = T; t > 0; t -= 64) rsl = rng_advance(rsl, rng_word(rsl, rcoef), min(t, 64));
            const unsigned long long bad = __ballot(lane < 31 && rsl != rs);
            unsigned long long k = 0;
            if (lane == 0) {
                atomicAdd(&g_am_check[4], 1ull);
                if (bad) k = atomicAdd(&g_am_check[0], 1ull);
            }
            k = __shfl(k, 0, 64);
            if (bad && k == 0) {
                if (lane < 32) {
                    g_am_check[16 + lane] = rs;
                    g_am_check[48 + lane] = rsl;
                }
                if (lane == 0) {
                    g_am_check[8] = f;
                    g_am_check[9] = round;
                    g_am_check[10] = T;
                    g_am_check[11] = nb;
                    g_am_check[12] = T > 0 ? (T - 1) / 64 : -1;
                    g_am_check[13] = sz;
                    g_am_check[14] = npop;
                    g_am_check[15] = A.pass;
                }
            }
        }
#endif
#ifdef GF_AM_TRACE
        if (f < 8) {
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&g_am_tcnt[f], 1u);
            k = __shfl(k, 0, 64);
            if (k < AMT_MAX) {
                uint32_t* r = g_am_trace[f][k];
                if (lane < 31) r[16 + lane] = rs;
                if (lane == 0) {
                    r[0] = round;
                    r[1] = T;
                    r[2] = nused;
                    r[3] = nc;
                    r[4] = nb;
                    r[5] = used;
                    r[6] = exh ? 0xffffffffu : (uint32_t)top;
                    r[7] = N;
                    r[8] = oct_b;
                    r[9] = exh ? 0u : (uint32_t)C.match[top];
                    r[10] = A.pass;
                    r[11] = npop;
                    r[12] = sz;
                }
            }
        }
#endif
        am_sync();
        if (exh) break;
        AM_T(5);
        const int nrem = npop + 1;  // removeIdx: every top tried
        const int q = lmk[C.slot[top]];
        const int b = C.match[top];
        if (lane == 0) {  // OnePoint's claim
            claim[b] = q;
            A.score[(long long)f * A.kp_cap + b] = C.dist[top] & 0xfff;
        }
        if (lane < 49) {  // curMat += H_rw^T H_rw (sigma^2 of the matched keypoint octave)
#if AM_WOCT
            const double w = s_woct[oct_b];  // the same arithmetic, done at kernel start
#else
#ifdef AM_LSIG
            const double s2 = sqrt((double)s_sig2[oct_b]);
#ifdef GF_AM_CHECK
            if (s_sig2[oct_b] != A.sigma2[oct_b]) atomicAdd(&g_am_check[3], 1ull);
#endif
#else
            const double s2 = sqrt((double)A.sigma2[oct_b]);
#endif
            const double w = s2 / (s2 * s2);
#endif
            const double a0 = w * h_i, a1 = w * h_j, b0 = w * h_7i, b1 = w * h_7j;
            cur[lane] = cur[lane] + (a0 * a1 + b0 * b1);
        }
        nm = __builtin_amdgcn_readfirstlane(nm + 1);
        AM_C(13, npop);
        (void)success;
        am_sync();
        if (nrem == N) break;  // went through all map points: the pool stays as left-overs
        // drop the tried columns: popped candidates and the successful top
        for (int c = lane; c < nused; c += AW)
            if (!C.alive[c] || c == top) atomicAnd(&pbits[C.slot[c] >> 6], ~(1ull << (C.slot[c] & 63)));
        am_sync();
        pool_prefix(P);
        N = __builtin_amdgcn_readfirstlane(N - nrem);
        nsucc_valid = false;  // a claim and removed columns: recounted when it may pay off
        last_npop = npop;
        am_sync();
        AM_T(6);
    }
    if (cabort) {  // (the scores written at this attempt's claims are the redo's too: same arithmetic)
        if (lane == 0) {
            if (A.pass == 1) A.ovf[1 + atomicAdd(A.ovf, 1)] = f;
            else A.err[f] = 3;
        }
        return;
    }
    // ---- outputs: claims, left-over pool (alive slots in order), RNG state
    for (int i = lane; i < n; i += AW) kp2mp[i] = claim[i];
    if (cut) N = 0;
    for (int w = 0; w < 64 && !cut; w++) {
        const unsigned long long bits = pbits[w];
        if (((bits >> lane) & 1ull) && w * 64 + lane < PC)
            left[ppre[w] + __popcll(bits & ((1ull << lane) - 1ull))] = lmk[w * 64 + lane];
    }
#ifdef GF_AM_GUARD
    am_sync();
    if (guard[threadIdx.x] != 0xa5a5a5a5u + threadIdx.x) atomicAdd(&g_am_guard[0], 1ull);
    if (threadIdx.x == 0) atomicAdd(&g_am_guard[1], 1ull);
#endif
#ifdef GF_AM_STAMP
    if (threadIdx.x == 0) {
        const unsigned long long tot_ = __builtin_amdgcn_s_memtime() - am_start_;
        atomicMax(&g_am_stamp[16], tot_);
        atomicAdd(&g_am_stamp[17], tot_);
    }
#endif
    {  // back to the glibc ring: f advanced by the calls made, oldest word at f
        const int f1 = (A.rng[f].f + used) % 31;
        am_sync();
        if (lane < 31) A.rng[f].state[(f1 + lane) % 31] = (int32_t)rs;
        am_sync();
        if (lane == 0) {
            A.rng[f].f = f1;
            A.rng[f].r = (f1 + 28) % 31;
            A.nleft[f] = N;
            A.nmatched[f] = nm;
            if (A.nldet) A.nldet[f] = nld;
        }
    }
}

// AM_PRIO: the wave's issue priority (s_setprio). A frame's rounds are one
// wave's dependent chain, and in the step it shares its SIMD with other
// groups' extraction waves; VALU / LDS issue goes to the higher priority,
// then the older wave, so at the default priority the chain waits behind
// them (cdna_hip_programming / MI355X_MICROARCH: issue arbitration).
// Measured r05 (profiles/r05/ab1): priority 3 made the launch slower in the
// step (1.12-1.15 ms per 256 frames against 0.97 at 0; 3 on every tracking
// kernel, GF_TRACK_PRIO: 1.03), headline unchanged: off.
#ifndef AM_PRIO
#define AM_PRIO 0
#endif
// the same body under two names, so that profiles tell the small-pool pass
// from the overflow pass of a two-pass launch
__global__ __launch_bounds__(AW) void k_active_match(ActiveArgs A) {
    if (AM_PRIO) __builtin_amdgcn_s_setprio(AM_PRIO);
    active_match_body(A, blockIdx.x);
}

// overflow pass: a small grid walks the frames the first pass listed (one
// wave, so the LDS reuse between frames needs no barrier)
__global__ __launch_bounds__(AW) void k_active_match_overflow(ActiveArgs A) {
    if (AM_PRIO) __builtin_amdgcn_s_setprio(AM_PRIO);
    const int cnt = A.ovf[0];
    for (int k = blockIdx.x; k < cnt; k += gridDim.x) active_match_body(A, A.ovf[1 + k]);
}

#undef AM_T

size_t active_lds_bytes(int pool_cap, int cand_cap, int kp_cap, bool lq_stage = false) {
#ifdef GF_AM_GUARD
    const size_t guard = 256;
#else
    const size_t guard = 0;
#endif
    return guard + sizeof(double) * cand_cap + 8 * 64 + sizeof(int) * ((size_t)kp_cap + 68) +
           sizeof(int32_t) * cand_cap + sizeof(int16_t) * (8 * (size_t)pool_cap + 3 * (size_t)cand_cap) + cand_cap +
           (lq_stage ? 1 + sizeof(uint16_t) * (size_t)pool_cap : 0);
}
// dynamic LDS bound of the active matcher's launches: the full-capacity
// footprint without the staged rows (the static arrays take the rest of 160 KB)
static const size_t AM_LDS_LIMIT = active_lds_bytes(POOL_MAX, POOL_MAX, KP_MAX, false);

// ------------------------------------------------------------- max-volume selection
struct MaxvolArgs {
    const double* info;   // [P][cap][49]
    const double* score;  // [P][cap]
    const int32_t* n;     // [P]
    int cap, k, mode;
    double sample_scale;
    gf_rng* rng;
    int32_t* out;   // [P][cap]
    int32_t* nout;  // [P]
    int32_t* err;
};

__global__ __launch_bounds__(GF_THREADS) void k_maxvol(MaxvolArgs A) {
    __shared__ double cur[49];
    __shared__ int16_t lmk[POOL_MAX], vis[POOL_MAX], samp[POOL_MAX];
    __shared__ uint8_t sel[POOL_MAX];
    __shared__ double s_best[GF_THREADS];
    __shared__ double s_ub[GF_THREADS];
    __shared__ int s_bi[GF_THREADS];
    __shared__ int32_t s_st[31], s_rf, s_rr;
    __shared__ int s_N, s_cnt, s_nout, s_stop;
    const int p = blockIdx.x, tid = threadIdx.x;
    const int n = A.n[p], k = A.k;
    const double* info = A.info + (long long)p * A.cap * 49;
    const double* score = A.score + (long long)p * A.cap;
    int32_t* out = A.out + (long long)p * A.cap;
    if (n > POOL_MAX) {
        if (tid == 0) A.err[p] = 2;
        return;
    }
    if (k >= n) {  // every landmark is selected
        for (int i = tid; i < n; i += GF_THREADS) out[i] = i;
        if (tid == 0) A.nout[p] = n;
        return;
    }
    const bool deletion = A.mode == 3 && 2LL * k > n;
    for (int i = tid; i < n; i += GF_THREADS) {
        lmk[i] = (int16_t)i;
        vis[i] = -1;
        sel[i] = deletion ? 1 : 0;
    }
    if (tid < 49) {
        double c = (tid % 8 == 0) ? 0.00001 : 0.0;
        if (deletion)
            for (int i = 0; i < n; i++) c = c + info[49LL * i + tid];
        cur[tid] = c;
    }
    if (tid < 31) s_st[tid] = A.rng[p].state[tid];
    if (tid == 0) {
        s_rf = A.rng[p].f;
        s_rr = A.rng[p].r;
        s_N = n;
        s_nout = 0;
        s_stop = 0;
    }
    __syncthreads();
    const int rounds = deletion ? n - k : k;
    const size_t szLazier = (size_t)((double)n / (double)k * A.sample_scale);
    const double sign = deletion ? -1.0 : 1.0;
    for (int it = 0; it < rounds; it++) {
        double best = -DBL_MAX, bub = -DBL_MAX;
        int bi = INT_MAX;
        if (A.mode == 1) {
            // baseline greedy: exact argmax of log det(cur + A_j) over the pool;
            // ties keep the larger diagonal upper bound, then the lower index.
            for (int j = tid; j < n; j += GF_THREADS) {
                if (sel[j] || score[j] < 0) continue;
                const double* b = info + 49LL * j;
                double ub = 0;
                for (int q = 0; q < 7; q++) ub += log(cur[8 * q] + b[8 * q]);
                const double d = logdet_sum(cur, b, 1.0);
                if (d > best || (d == best && (ub > bub || (ub == bub && j < bi)))) {
                    best = d;
                    bub = ub;
                    bi = j;
                }
            }
        } else {
            if (tid == 0) {  // random samples in exact std::rand order
                const int N = s_N;
                const int szActual = (int)min(szLazier, (size_t)N);
                int hit = 0, cnt = 0;
                while (hit < szActual) {
                    int j = -1;
                    for (int q = 0; q < MAX_RANDOM_QUERY_TIME; q++) {
                        const int jj = (int)((uint32_t)gfrng::next(s_st, &s_rf, &s_rr) % (uint32_t)N);
                        if (vis[jj] < it) {
                            vis[jj] = (int16_t)it;
                            j = jj;
                            break;
                        }
                    }
                    if (j < 0) break;
                    const int qi = lmk[j];
                    hit++;
                    const bool valid = deletion ? (sel[qi] && score[qi] >= 0) : (!sel[qi] && score[qi] >= 0);
                    if (!valid) {
                        hit--;
                        continue;
                    }
                    samp[cnt++] = (int16_t)qi;
                }
                s_cnt = cnt;
            }
            __syncthreads();
            for (int t = tid; t < s_cnt; t += GF_THREADS) {
                const double d = logdet_sum(cur, info + 49LL * samp[t], sign);
                if (d > best || (d == best && t < bi)) {  // first sample wins ties (strict '>')
                    best = d;
                    bi = t;
                }
            }
        }
        s_best[tid] = best;
        s_ub[tid] = bub;
        s_bi[tid] = bi;
        __syncthreads();
        if (tid == 0) {
            double B = -DBL_MAX, U = -DBL_MAX;
            int I = INT_MAX;
            for (int t = 0; t < GF_THREADS; t++) {
                const double d = s_best[t];
                if (s_bi[t] == INT_MAX) continue;
                bool better;
                if (A.mode == 1)
                    better = d > B || (d == B && (s_ub[t] > U || (s_ub[t] == U && s_bi[t] < I)));
                else
                    better = d > B || (d == B && s_bi[t] < I);
                if (better) {
                    B = d;
                    U = s_ub[t];
                    I = s_bi[t];
                }
            }
            if (I == INT_MAX) {
                s_stop = 1;  // early termination (no valid candidate)
            } else {
                const int chosen = A.mode == 1 ? I : samp[I];
                for (int q = 0; q < 49; q++) cur[q] = deletion ? cur[q] - info[49LL * chosen + q] : cur[q] + info[49LL * chosen + q];
                sel[chosen] = deletion ? 0 : 1;
                if (!deletion) out[s_nout++] = chosen;
                if (A.mode != 1) {  // drop the chosen entry from the index pool
                    int w = 0;
                    for (int r = 0; r < s_N; r++)
                        if (lmk[r] != chosen) {
                            lmk[w] = lmk[r];
                            vis[w] = vis[r];
                            w++;
                        }
                    s_N = w;
                }
            }
        }
        __syncthreads();
        if (s_stop) break;
    }
    if (deletion && tid == 0) {
        for (int i = 0; i < n; i++)
            if (sel[i]) out[s_nout++] = i;
    }
    __syncthreads();
    if (tid < 31) A.rng[p].state[tid] = s_st[tid];
    if (tid == 0) {
        A.rng[p].f = s_rf;
        A.rng[p].r = s_rr;
        A.nout[p] = s_nout;
    }
}

}  // namespace

// ============================================================== ABI
static int set_lds_attr(gf_ctx* ctx, const void* fn, size_t bytes, unsigned long long* mask) {
    if (!(*mask & (1ull << ctx->device))) {
        GF_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        *mask |= 1ull << ctx->device;
    }
    return GF_OK;
}

extern "C" {

int gf_obs_build_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_pos,
                          const float* d_sigma2, const int32_t* d_n, int cap, int check_viz, double* d_H,
                          double* d_info, float* d_uv, uint8_t* d_valid, void* stream) {
    GF_CHECK(ctx && cam, GF_ERR_ARG, "null arg");
    if (nframes <= 0 || cap <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_info");
    GF_LAUNCH(k_obs_info, dim3((cap + 127) / 128, nframes), 128, 0, s, *cam, d_Xv, d_pos, d_sigma2, d_n, cap, check_viz, d_H,
                                                                 d_info, d_uv, d_valid);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_obs_accumulate_dev(gf_ctx* ctx, int nframes, const double* d_info, const uint8_t* d_flag, const int32_t* d_n,
                          int cap, double diag, double* d_out, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_accumulate");
    GF_LAUNCH(k_obs_accumulate, nframes, 64, 0, s, d_info, d_flag, d_n, cap, diag, d_out);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_obs_active_match_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                            const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                            const uint8_t* d_mp_desc, const uint8_t* d_updated, const double* d_info,
                            const double* d_H, const int32_t* d_m, int mp_cap, const double* d_base,
                            const float* level_sigma2, const int32_t* d_num_to_match, float th, float nnratio,
                            gf_rng* d_rng, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_left, int32_t* d_nleft,
                            int32_t* d_nmatched, int32_t* d_nldet, void* stream) {
    return gf::obs_active_match(ctx, fi, nframes, d_kps, d_desc, d_n, kp_cap, d_views, d_mp_desc, d_updated, d_info,
                                d_H, d_m, mp_cap, d_base, level_sigma2, d_num_to_match, th, nnratio, d_rng, d_kp2mp,
                                d_score, d_left, d_nleft, d_nmatched, d_nldet, nullptr, stream);
}

}  // extern "C"

int gf::obs_active_match(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                         const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                         const uint8_t* d_mp_desc, const uint8_t* d_updated, const double* d_info, const double* d_H,
                         const int32_t* d_m, int mp_cap, const double* d_base, const float* level_sigma2,
                         const int32_t* d_num_to_match, float th, float nnratio, gf_rng* d_rng, int32_t* d_kp2mp,
                         int32_t* d_score, int32_t* d_left, int32_t* d_nleft, int32_t* d_nmatched, int32_t* d_nldet,
                         const int32_t* d_remap, void* stream, const gf::ActiveClock& ck,
                         const double* d_info_lt) {
    GF_CHECK(ctx && fi && level_sigma2, GF_ERR_ARG, "null arg");
    GF_CHECK(!ck.mat_t0 || (ck.viz && ck.rec), GF_ERR_ARG, "bad clock");
    GF_CHECK(kp_cap <= KP_MAX && mp_cap <= 32767, GF_ERR_UNSUPPORTED, "frame exceeds active-matching limits");
    GF_CHECK(fi->nlevels >= 1 && fi->nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    if (nframes <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    ActiveArgs A{};
    A.fc = gf::make_frame_const(fi);
    A.kps = d_kps;
    A.desc = d_desc;
    A.n = d_n;
    A.kp_cap = kp_cap;
    A.views = d_views;
    A.mp_desc = d_mp_desc;
    A.updated = d_updated;
    A.info = d_info;
    if (!d_info_lt) {  // the packed records the matcher reads, built here
        void* lt = nullptr;
        int rc0 = gf::ws_get(ctx, 20, sizeof(double) * 32 * (size_t)nframes * std::max(mp_cap, 1), &lt);
        if (rc0) return rc0;
        if (mp_cap > 0) {
            GF_PROF(ctx, s, "k_pack_info");
            GF_LAUNCH(k_pack_info, dim3((mp_cap + 255) / 256, nframes), 256, 0, s, d_info, mp_cap, (double*)lt);
            GF_HIP(hipGetLastError());
        }
        d_info_lt = (const double*)lt;
    }
    A.info_lt = d_info_lt;
    A.H = d_H;
    A.m = d_m;
    A.mp_cap = mp_cap;
    A.base = d_base;
    for (int i = 0; i < fi->nlevels; i++) A.sigma2[i] = level_sigma2[i];
    A.num_to_match = d_num_to_match;
    A.th = th;
    A.nnratio = nnratio;
    A.rng = d_rng;
    A.kp2mp = d_kp2mp;
    A.score = d_score;
    A.left = d_left;
    A.nleft = d_nleft;
    A.nmatched = d_nmatched;
    A.nldet = d_nldet;
    A.remap = d_remap;
    A.ck = ck;
    void* err;
    int rc = gf::ws_get(ctx, 30, sizeof(int32_t) * nframes, &err);
    if (rc) return rc;
    A.err = (int32_t*)err;
    static unsigned long long mask = 0;  // devices whose table is set (once per process)
    if (!(mask & (1ull << ctx->device))) {  // rand() as a linear combination of the 31-word history
        uint32_t h[31 + 64][31] = {};
        for (int j = 0; j < 31; j++) h[j][j] = 1u;
        for (int k = 0; k < 64; k++)
            for (int j = 0; j < 31; j++) h[31 + k][j] = h[28 + k][j] + h[k][j];
        uint32_t t[31][64];
        for (int j = 0; j < 31; j++)
            for (int k = 0; k < 64; k++) t[j][k] = h[31 + k][j];
        GF_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_rng_coef), &t[0][0], sizeof(t)));
        mask |= 1ull << ctx->device;
    }
    void* pre;
    rc = gf::ws_get(ctx, 32, sizeof(OnePre) * (size_t)nframes * mp_cap, &pre);
    if (rc) return rc;
    A.pre = (const OnePre*)pre;
    void *gcs, *gitems;
    if ((rc = gf::ws_get(ctx, 34, sizeof(int) * (size_t)nframes * (NCELLS + 1), &gcs)) ||
        (rc = gf::ws_get(ctx, 35, sizeof(int) * (size_t)nframes * kp_cap, &gitems)))
        return rc;
    A.grid_cs = (int*)gcs;
    A.grid_items = (int*)gitems;
    static unsigned long long pre_mask = 0;
    const size_t pre_lds = onepoint_pre_lds_bytes(kp_cap);
    GF_CHECK(pre_lds <= 160 * 1024, GF_ERR_UNSUPPORTED, "keypoint capacity too large for the one-point precompute");
    if (!(pre_mask & (1ull << ctx->device))) {
        GF_HIP(hipFuncSetAttribute((const void*)k_onepoint_pre, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)onepoint_pre_lds_bytes(KP_MAX)));
        pre_mask |= 1ull << ctx->device;
    }
    {
        GF_PROF(ctx, s, "k_onepoint_pre");
        GF_LAUNCH(k_onepoint_pre, nframes, PRE_THREADS, pre_lds, s, A, (OnePre*)pre);
        GF_HIP(hipGetLastError());
    }
    const int full_pc = std::min(((mp_cap + 63) / 64) * 64, POOL_MAX);
    static unsigned long long ovf_mask = 0;
    const size_t lds_max = std::min(active_lds_bytes(POOL_MAX, POOL_MAX, KP_MAX, true), AM_LDS_LIMIT);
    if ((rc = set_lds_attr(ctx, (const void*)k_active_match, lds_max, &mask)) ||
        (rc = set_lds_attr(ctx, (const void*)k_active_match_overflow, lds_max, &ovf_mask)))
        return rc;
    // the slots' rows go to LDS when the remapped rows fit 16 bits and the launch's LDS allows
    auto lq_fits = [&](int pc, int cc) {
        return mp_cap <= 65536 && active_lds_bytes(pc, cc, kp_cap, true) <= AM_LDS_LIMIT;
    };
    // Two passes when the map list is long: most frames' pools (in-view, updated
    // points) are far below the list capacity, and a smaller LDS footprint lets
    // more workgroups of the concurrently running kernels share each CU. Frames
    // whose pool does not fit return before writing anything and are redone by
    // the overflow pass with the full capacity.
    A.pool_cap = A.cand_cap = full_pc;
    A.pass = 0;
    A.ovf = nullptr;
    // with a time budget the candidate arrays stay full size (an attempt cut
    // short by them would have spent clock time the redo does not see)
    const int cand_small = (ck.mat_t0 || !AM_CC) ? std::min(full_pc, AM_SMALL_POOL) : std::min(full_pc, AM_CAND_CAP);
    // (a small batch runs one pass at full capacity: the LDS is free, and a
    // redone frame would double a single sequence's latency)
    if (nframes > AM_ONE_PASS_MAX && (full_pc > AM_SMALL_POOL || cand_small < full_pc)) {
        void* ovf;
        if ((rc = gf::ws_get(ctx, 39, sizeof(int32_t) * (nframes + 1), &ovf))) return rc;
        GF_HIP(hipMemsetAsync(ovf, 0, sizeof(int32_t), s));
        A.ovf = (int32_t*)ovf;
        A.pool_cap = std::min(full_pc, AM_SMALL_POOL);
        A.cand_cap = cand_small;
        A.pass = 1;
    }
    {
        GF_PROF(ctx, s, "k_active_match");
        A.lq_stage = lq_fits(A.pool_cap, A.cand_cap) ? 1 : 0;
        GF_LAUNCH(k_active_match, nframes, AW, active_lds_bytes(A.pool_cap, A.cand_cap, kp_cap, A.lq_stage), s, A);
        GF_HIP(hipGetLastError());
    }
    if (A.pass == 1) {
        A.pool_cap = A.cand_cap = full_pc;
        A.pass = 2;
        GF_PROF(ctx, s, "k_active_match_overflow");
        // a workgroup per listed frame up to AM_OVF_GRID (the ones past the
        // list's count exit at once): with long maps (config 3) every frame's
        // pool is past the first pass's, and 64 workgroups walked 256 frames
        // four deep (7.7 ms of the step)
        A.lq_stage = lq_fits(full_pc, full_pc) ? 1 : 0;
        GF_LAUNCH(k_active_match_overflow, std::min(nframes, AM_OVF_GRID), AW,
                  active_lds_bytes(full_pc, full_pc, kp_cap, A.lq_stage), s, A);
        GF_HIP(hipGetLastError());
    }
    return GF_OK;
}

extern "C" {

int gf_maxvol_select_dev(gf_ctx* ctx, int npools, const double* d_info, const double* d_score, const int32_t* d_n,
                         int cap, int k, double sample_scale, int mode, gf_rng* d_rng, int32_t* d_out,
                         int32_t* d_nout, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    GF_CHECK(mode >= 1 && mode <= 3, GF_ERR_ARG, "mode must be 1, 2 or 3");
    GF_CHECK(cap <= POOL_MAX, GF_ERR_UNSUPPORTED, "pool exceeds 4096 landmarks");
    if (npools <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    MaxvolArgs A{d_info, d_score, d_n, cap, k, mode, sample_scale, d_rng, d_out, d_nout, nullptr};
    void* err;
    int rc = gf::ws_get(ctx, 29, sizeof(int32_t) * npools, &err);
    if (rc) return rc;
    A.err = (int32_t*)err;
    GF_PROF(ctx, s, "k_maxvol");
    GF_LAUNCH(k_maxvol, npools, GF_THREADS, 0, s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

// ------------------------------------------------------------ host family
int gf_obs_build_info(gf_ctx* ctx, const gf_obs_camera* cam, const double* Xv, const float* pos, const float* sigma2,
                      int n, int check_viz, double* H, double* info, float* uv, uint8_t* valid) {
    GF_CHECK(ctx && cam && Xv, GF_ERR_ARG, "null arg");
    if (n <= 0) return GF_OK;
    GF_CHECK(pos && H && info && uv && valid, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dX, *dP, *dS = nullptr, *dn, *dH, *dI, *dU, *dV;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, Xv, 13 * sizeof(double), &dX)) ||
        (rc = gf::ws_upload(ctx, 1, pos, 12 * (size_t)n, &dP)) || (rc = gf::ws_upload(ctx, 2, &n, 4, &dn)) ||
        (rc = gf::ws_get(ctx, 3, 14 * 8 * (size_t)n, &dH)) || (rc = gf::ws_get(ctx, 4, 49 * 8 * (size_t)n, &dI)) ||
        (rc = gf::ws_get(ctx, 5, 8 * (size_t)n, &dU)) || (rc = gf::ws_get(ctx, 6, (size_t)n, &dV)))
        return rc;
    if (sigma2 && (rc = gf::ws_upload(ctx, 7, sigma2, 4 * (size_t)n, &dS))) return rc;
    rc = gf_obs_build_info_dev(ctx, cam, 1, (const double*)dX, (const float*)dP, (const float*)dS, (const int32_t*)dn,
                               n, check_viz, (double*)dH, (double*)dI, (float*)dU, (uint8_t*)dV, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(H, dH, 14 * 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(info, dI, 49 * 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(uv, dU, 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(valid, dV, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_logdet(gf_ctx* ctx, const double* M, int n, double* out) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (n <= 0) return GF_OK;
    GF_CHECK(M && out, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dM, *dO;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, M, 49 * 8 * (size_t)n, &dM)) || (rc = gf::ws_get(ctx, 1, 8 * (size_t)n, &dO)))
        return rc;
    {
        GF_PROF(ctx, ctx->stream, "k_logdet");
        GF_LAUNCH(k_logdet, (n + 127) / 128, 128, 0, ctx->stream, (const double*)dM, n, (double*)dO);
    }
    GF_HIP(hipGetLastError());
    GF_HIP(hipMemcpyAsync(out, dO, 8 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_obs_active_match(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                        const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated, const double* info,
                        const double* H, const float* uv, int m, const double* base, const float* level_sigma2,
                        int num_to_match, float th, float nnratio, gf_rng* rng, int32_t* kp2mp, int32_t* score,
                        int32_t* left, int* nleft, int* nmatched) {
    GF_CHECK(ctx && fi && nleft && nmatched && rng && base && level_sigma2, GF_ERR_ARG, "null arg");
    (void)uv;  // u_proj/v_proj feed only reWeightInfoMat's residual terms, which are compiled out
    *nleft = 0;
    *nmatched = 0;
    GF_CHECK(n >= 0 && m >= 0, GF_ERR_ARG, "negative size");
    GF_CHECK(m == 0 || (views && mp_desc && updated && info && H && left), GF_ERR_ARG, "null arg");
    GF_CHECK(n == 0 || (kps && desc && kp2mp && score), GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    const int nn = n > 0 ? n : 1, mm = m > 0 ? m : 1;
    void *dK, *dD, *dn, *dV, *dQ, *dU, *dI, *dH, *dm, *dB, *dT, *dR, *dC, *dS, *dL, *dNL, *dNM;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, kps, sizeof(gf_keypoint) * n, &dK)) ||
        (rc = gf::ws_upload(ctx, 1, desc, 32 * (size_t)n, &dD)) || (rc = gf::ws_upload(ctx, 2, &n, 4, &dn)) ||
        (rc = gf::ws_upload(ctx, 3, views, sizeof(gf_mp_view) * m, &dV)) ||
        (rc = gf::ws_upload(ctx, 4, mp_desc, 32 * (size_t)m, &dQ)) ||
        (rc = gf::ws_upload(ctx, 5, updated, (size_t)m, &dU)) ||
        (rc = gf::ws_upload(ctx, 6, info, 49 * 8 * (size_t)m, &dI)) ||
        (rc = gf::ws_upload(ctx, 7, H, 14 * 8 * (size_t)m, &dH)) || (rc = gf::ws_upload(ctx, 8, &m, 4, &dm)) ||
        (rc = gf::ws_upload(ctx, 9, base, 49 * 8, &dB)) ||
        (rc = gf::ws_upload(ctx, 10, &num_to_match, 4, &dT)) ||
        (rc = gf::ws_upload(ctx, 11, rng, sizeof(gf_rng), &dR)) ||
        (rc = gf::ws_upload(ctx, 12, kp2mp, 4 * (size_t)n, &dC)) ||
        (rc = gf::ws_upload(ctx, 13, score, 4 * (size_t)n, &dS)) || (rc = gf::ws_get(ctx, 14, 4 * (size_t)mm, &dL)) ||
        (rc = gf::ws_get(ctx, 15, 4, &dNL)) || (rc = gf::ws_get(ctx, 16, 4, &dNM)))
        return rc;
    (void)nn;
    void* err;
    if ((rc = gf::ws_get(ctx, 30, 4, &err))) return rc;
    GF_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
    rc = gf_obs_active_match_dev(ctx, fi, 1, (const gf_keypoint*)dK, (const uint8_t*)dD, (const int32_t*)dn, n > 0 ? n : 1,
                                 (const gf_mp_view*)dV, (const uint8_t*)dQ, (const uint8_t*)dU, (const double*)dI,
                                 (const double*)dH, (const int32_t*)dm, mm, (const double*)dB, level_sigma2,
                                 (const int32_t*)dT, th, nnratio, (gf_rng*)dR, (int32_t*)dC, (int32_t*)dS,
                                 (int32_t*)dL, (int32_t*)dNL, (int32_t*)dNM, nullptr, ctx->stream);
    if (rc) return rc;
    int e = 0;
    GF_HIP(hipMemcpyAsync(&e, err, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(nleft, dNL, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(nmatched, dNM, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(rng, dR, sizeof(gf_rng), hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    GF_CHECK(e == 0, GF_ERR_UNSUPPORTED, "active-matching pool exceeds 4096 map points");
    if (n > 0) {
        GF_HIP(hipMemcpy(kp2mp, dC, 4 * (size_t)n, hipMemcpyDeviceToHost));
        GF_HIP(hipMemcpy(score, dS, 4 * (size_t)n, hipMemcpyDeviceToHost));
    }
    if (*nleft > 0) GF_HIP(hipMemcpy(left, dL, 4 * (size_t)*nleft, hipMemcpyDeviceToHost));
    return GF_OK;
}

int gf_maxvol_select(gf_ctx* ctx, const double* info, const double* score, int n, int k, double sample_scale, int mode,
                     gf_rng* rng, int32_t* out_idx, int* nout) {
    GF_CHECK(ctx && nout && rng, GF_ERR_ARG, "null arg");
    *nout = 0;
    if (n <= 0) return GF_OK;
    GF_CHECK(info && score && out_idx, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dI, *dS, *dn, *dR, *dO, *dN, *err;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, info, 49 * 8 * (size_t)n, &dI)) ||
        (rc = gf::ws_upload(ctx, 1, score, 8 * (size_t)n, &dS)) || (rc = gf::ws_upload(ctx, 2, &n, 4, &dn)) ||
        (rc = gf::ws_upload(ctx, 3, rng, sizeof(gf_rng), &dR)) || (rc = gf::ws_get(ctx, 4, 4 * (size_t)n, &dO)) ||
        (rc = gf::ws_get(ctx, 5, 4, &dN)) || (rc = gf::ws_get(ctx, 29, 4, &err)))
        return rc;
    GF_HIP(hipMemsetAsync(err, 0, 4, ctx->stream));
    rc = gf_maxvol_select_dev(ctx, 1, (const double*)dI, (const double*)dS, (const int32_t*)dn, n, k, sample_scale,
                              mode, (gf_rng*)dR, (int32_t*)dO, (int32_t*)dN, ctx->stream);
    if (rc) return rc;
    int e = 0;
    GF_HIP(hipMemcpyAsync(&e, err, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(nout, dN, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(rng, dR, sizeof(gf_rng), hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    GF_CHECK(e == 0, GF_ERR_UNSUPPORTED, "pool exceeds 4096 landmarks");
    if (*nout > 0) GF_HIP(hipMemcpy(out_idx, dO, 4 * (size_t)*nout, hipMemcpyDeviceToHost));
    return GF_OK;
}

// Observability::setSelction_Number's greedy stage over a prepared pool
// (lmkSelectPool, Observability.cc:1072-1160): greedy_mtd 1 / 2 on the pool,
// 3 splits a large pool into threadNeeded chunks as the reference does
// (:1086-1160), run in chunk order on the caller's rand() stream, then an
// automatic pass over the merged selections (which keep their scores).
int gf_select_pool(gf_ctx* ctx, const double* info, const double* score, int n, int k, int greedy_mtd,
                   int max_threads, gf_rng* rng, int32_t* out_idx, int* nout) {
    GF_CHECK(ctx && rng && nout, GF_ERR_ARG, "null arg");
    GF_CHECK(greedy_mtd >= 1 && greedy_mtd <= 3, GF_ERR_ARG, "greedy_mtd must be 1, 2 or 3");
    *nout = 0;
    const int P = n;
    if (P <= 0) return GF_OK;
    GF_CHECK(info && score && out_idx, GF_ERR_ARG, "null arg");
    const double scale = 6.0;  // random_sample_scale of the map overload (:1035)
    int rc;
    int T = 1;
    if (greedy_mtd == 3 && !((float)P - 1.2f * (float)k <= 10 || P < 2 * 1000))
        T = std::max(1, std::min((int)std::lround((float)P / 1000.f), max_threads));
    if (T == 1) return gf_maxvol_select(ctx, info, score, P, k, scale, greedy_mtd, rng, out_idx, nout);
    const int kpar = (int)std::ceil((float)k / (float)T * 1.2f);
    const int npar = (int)std::ceil((float)P / (float)T);
    std::vector<int> merged;
    for (int t = 0; t < T; t++) {
        const int lo = t * npar, hi = std::min(P, (t + 1) * npar);
        if (hi <= lo) continue;
        std::vector<int32_t> o(hi - lo);
        int no = 0;
        rc = gf_maxvol_select(ctx, &info[49 * (size_t)lo], &score[lo], hi - lo, kpar, scale, 3, rng, o.data(), &no);
        if (rc) return rc;
        for (int q = 0; q < no; q++) merged.push_back(lo + o[q]);
    }
    const int Mg = (int)merged.size();
    std::vector<double> minfo(49 * (size_t)std::max(Mg, 1)), mscore(std::max(Mg, 1));
    for (int j = 0; j < Mg; j++) {
        memcpy(&minfo[49 * (size_t)j], &info[49 * (size_t)merged[j]], 49 * sizeof(double));
        mscore[j] = score[merged[j]];
    }
    std::vector<int32_t> o(std::max(Mg, 1));
    int no = 0;
    rc = gf_maxvol_select(ctx, minfo.data(), mscore.data(), Mg, k, scale, 3, rng, o.data(), &no);
    if (rc) return rc;
    for (int q = 0; q < no; q++) out_idx[(*nout)++] = merged[o[q]];
    return GF_OK;
}

// Observability::setSelction_Number over fresh map points (Observability.cc:
// 1021-1247): MAP_INFO_MATRIX with the visibility check on the device (no
// point updated this frame), the visible pool in list order with ObsScore 1,
// then gf_select_pool.
int gf_select_map_points(gf_ctx* ctx, const gf_obs_camera* cam, const double* Xv, const float* pos, int n, int k,
                         int greedy_mtd, int max_threads, gf_rng* rng, int32_t* out_idx, int* nout) {
    GF_CHECK(ctx && cam && Xv && rng && nout, GF_ERR_ARG, "null arg");
    GF_CHECK(greedy_mtd >= 1 && greedy_mtd <= 3, GF_ERR_ARG, "greedy_mtd must be 1, 2 or 3");
    *nout = 0;
    if (n <= 0) return GF_OK;
    GF_CHECK(pos && out_idx, GF_ERR_ARG, "null arg");
    std::vector<double> H(14 * (size_t)n), info(49 * (size_t)n);
    std::vector<float> uv(2 * (size_t)n);
    std::vector<uint8_t> valid(n);
    int rc = gf_obs_build_info(ctx, cam, Xv, pos, nullptr, n, 1, H.data(), info.data(), uv.data(), valid.data());
    if (rc) return rc;
    std::vector<int> pool;
    for (int i = 0; i < n; i++)
        if (valid[i]) pool.push_back(i);
    const int P = (int)pool.size();
    std::vector<double> pinfo(49 * (size_t)std::max(P, 1)), pscore(std::max(P, 1), 1.0);
    for (int j = 0; j < P; j++) memcpy(&pinfo[49 * (size_t)j], &info[49 * (size_t)pool[j]], 49 * sizeof(double));
    std::vector<int32_t> sel(std::max(P, 1));
    int ns = 0;
    rc = gf_select_pool(ctx, pinfo.data(), pscore.data(), P, k, greedy_mtd, max_threads, rng, sel.data(), &ns);
    if (rc) return rc;
    for (int q = 0; q < ns; q++) out_idx[(*nout)++] = pool[sel[q]];
    return GF_OK;
}

}  // extern "C"

// G1 on the device: Observability::updatePWLSVec(mLastFrame.mTimeStamp,
// mLastFrame.mTcw, mCurrentFrame.mTimeStamp, mCurrentFrame.getTwc())
// (Tracking.cc:3168-3169) for every frame, one thread each.
#include "kine.h"

namespace {
__global__ void k_obs_update(int nframes, const double* __restrict__ t_prev, const float* __restrict__ Tcw_prev,
                             const double* __restrict__ t_cur, const float* __restrict__ Tcw_cur,
                             double* __restrict__ Xv, double* __restrict__ Xv_next,
                             const int32_t* __restrict__ gate) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    if (gate && !gate[f]) return;
    float Twc[16];
    gfkine::get_Twc(Tcw_cur + 16 * f, Twc);
    gfkine::obs_update(t_prev[f], Tcw_prev + 16 * f, t_cur[f], Twc, Xv + 13 * f);
    if (Xv_next) {  // predictPWLSVec(dt, 2): kinematic[1].Xv = propagate_PWLS(Xv, float(dt))
        const double dt = (double)(float)(t_cur[f] - t_prev[f]);
        gfkine::propagate_state(Xv + 13 * f, dt, Xv_next + 13 * f);
    }
}
}  // namespace

extern "C" int gf_obs_update_dev(gf_ctx* ctx, int nframes, const double* d_t_prev, const float* d_Tcw_prev,
                                 const double* d_t_cur, const float* d_Tcw_cur, double* d_Xv, double* d_Xv_next,
                                 void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_t_prev && d_Tcw_prev && d_t_cur && d_Tcw_cur && d_Xv, GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    return gf::obs_update_gated(ctx, nframes, d_t_prev, d_Tcw_prev, d_t_cur, d_Tcw_cur, d_Xv, d_Xv_next, nullptr, s);
}

int gf::obs_update_gated(gf_ctx* ctx, int nframes, const double* d_t_prev, const float* d_Tcw_prev,
                         const double* d_t_cur, const float* d_Tcw_cur, double* d_Xv, double* d_Xv_next,
                         const int32_t* d_gate, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_update");
    GF_LAUNCH(k_obs_update, (nframes + 63) / 64, 64, 0, s, nframes, d_t_prev, d_Tcw_prev, d_t_cur, d_Tcw_cur, d_Xv,
              d_Xv_next, d_gate);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

// ---------------------------------------------------------------------------
// Map-resident observability state (MapPoint::ObsMat / H_meas / u_proj /
// updateAtFrameId, MapPoint.h) and the three per-frame passes over it.
namespace {

struct LevelTab {
    float v[16];
};

// batchInfoMat_Frame (Observability.cc:386-554): every matched, non-outlier
// keypoint writes H/ObsMat/u_proj of its map point with the keypoint level
// sigma^2 (WITH_OCT_LEVELED_NOISE); updateAtFrameId is left alone (:498-503).
__global__ void k_obs_frame_info(gf_obs_camera cam, const double* __restrict__ Xv, const gf_keypoint* __restrict__ kps,
                                 const int32_t* __restrict__ nkps, int kp_stride, const int32_t* __restrict__ kp2mp,
                                 const uint8_t* __restrict__ outl, const float* __restrict__ mpos,
                                 const int32_t* __restrict__ nmp, int map_stride, LevelTab sig, int nlevels,
                                 double* __restrict__ Hout, double* __restrict__ info, float* __restrict__ uv,
                                 const int32_t* __restrict__ remap, double* __restrict__ info_lt) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nkps[f]) return;
    const long long k = (long long)f * kp_stride + i;
    const int mp = kp2mp[k];
    if (mp < 0 || mp >= nmp[f] || (outl && outl[k])) return;
    const long long g = (long long)f * map_stride + mp;
    const double y[3] = {mpos[3 * g], mpos[3 * g + 1], mpos[3 * g + 2]};
    double H[14];
    float p[2];
    landmark_jacobian(cam, Xv + 13 * f, y, false, H, p);
    const int oc = min(max(kps[k].octave, 0), nlevels - 1);
    double M[49];
    for (int e = 0; e < 49; e++) M[e] = 0;
    add_info_block(H, (double)sig.v[oc], M);
    const long long w = remap ? (long long)f * map_stride + remap[g] : g;
    uv[2 * w] = p[0];
    uv[2 * w + 1] = p[1];
    for (int e = 0; e < 14; e++) Hout[14 * w + e] = H[e];
    for (int e = 0; e < 49; e++) info[49 * w + e] = M[e];
    if (info_lt) store_lower_packed(M, info_lt + 32 * w);
}

// batchInfoMat_Map (Observability.cc:556-644): skip points already updated
// for this frame id, and (check_viz == false) points not mbTrackInView; on a
// visible point write H/ObsMat/u_proj and updateAtFrameId = frame_id.
// updated_out (optional) = (updateAtFrameId == frame_id) afterwards.
__global__ void k_obs_map_info(gf_obs_camera cam, const double* __restrict__ Xv, const float* __restrict__ mpos,
                               const int32_t* __restrict__ nmp, int map_stride, int check_viz,
                               const gf_mp_view* __restrict__ views, int32_t* __restrict__ upd_id, int frame_id,
                               double* __restrict__ Hout, double* __restrict__ info, float* __restrict__ uv,
                               uint8_t* __restrict__ updated_out, const int32_t* __restrict__ remap,
                               gf::StageClock ck, const long long* __restrict__ cap2, double* __restrict__ info_lt) {
    const int f = blockIdx.y;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool late = false;
    if (ck.t0) {  // the time cap, one clock read per 64-point batch (Observability.cc:573-578)
        const int w = i >> 6;
        if (w * 64 < nmp[f]) {
            const long long e = gfd::ck_elapsed(ck.t0[f], ck.syn, w);
            if ((threadIdx.x & 63) == 0) ck.rec[(long long)f * ck.stride + ck.off + w] = e;
            late = 2 * e > cap2[f];
        }
    }
    if (i >= map_stride) return;
    const long long g = (long long)f * map_stride + i;
    if (i >= nmp[f]) {
        if (updated_out) updated_out[g] = 0;
        return;
    }
    int u = upd_id[g];
    const bool skip = late || (u == frame_id) || (!check_viz && views && !views[g].in_view);
    if (!skip) {
        const double y[3] = {mpos[3 * g], mpos[3 * g + 1], mpos[3 * g + 2]};
        double H[14];
        float p[2];
        if (landmark_jacobian(cam, Xv + 13 * f, y, check_viz != 0, H, p)) {
            double M[49];
            for (int e = 0; e < 49; e++) M[e] = 0;
            add_info_block(H, 1.0, M);
            const long long w = remap ? (long long)f * map_stride + remap[g] : g;
            uv[2 * w] = p[0];
            uv[2 * w + 1] = p[1];
            for (int e = 0; e < 14; e++) Hout[14 * w + e] = H[e];
            for (int e = 0; e < 49; e++) info[49 * w + e] = M[e];
            if (info_lt) store_lower_packed(M, info_lt + 32 * w);
            u = frame_id;
            upd_id[g] = u;
        }
    }
    if (updated_out) updated_out[g] = (u == frame_id);
}

// mCurrentInfoMat = diag*I + sum over matched points (keypoint order) with
// updateAtFrameId == frame_id of their ObsMat (Tracking.cc:3184, 3195-3213).
__global__ __launch_bounds__(64) void k_obs_accumulate_matched(const int32_t* __restrict__ kp2mp,
                                                               const int32_t* __restrict__ nkps, int kp_stride,
                                                               const double* __restrict__ info,
                                                               const int32_t* __restrict__ upd_id,
                                                               const int32_t* __restrict__ nmp, int map_stride,
                                                               int frame_id, double diag, double* __restrict__ out,
                                                               const int32_t* __restrict__ remap,
                                                               const int32_t* __restrict__ gate) {
    __shared__ int list[KP_MAX];
    const int f = blockIdx.x, lane = threadIdx.x;
    if (gate && !gate[f]) return;
    const int n = min(nkps[f], KP_MAX), m = nmp[f];
    // the contributing map points in keypoint order (ballot compaction)
    int cnt = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        int mp = i < n ? kp2mp[(long long)f * kp_stride + i] : -1;
        const bool on = mp >= 0 && mp < m && upd_id[(long long)f * map_stride + mp] == frame_id;
        const unsigned long long msk = __ballot(on);
        if (on)
            list[cnt + __popcll(msk & ((1ull << lane) - 1ull))] = remap ? remap[(long long)f * map_stride + mp] : mp;
        cnt += __popcll(msk);
    }
    __syncthreads();
    if (lane >= 49) return;
    // lane = matrix entry; the additions stay in keypoint order (bit-exact with
    // the sequential loop), the loads run ahead of them
    double s = (lane % 8 == 0) ? diag : 0.0;
    const double* I = info + (long long)f * map_stride * 49 + lane;
    int i = 0;
    for (; i + 4 <= cnt; i += 4) {
        const double a = I[49LL * list[i]], b = I[49LL * list[i + 1]], c = I[49LL * list[i + 2]],
                     d = I[49LL * list[i + 3]];
        s = s + a;
        s = s + b;
        s = s + c;
        s = s + d;
    }
    for (; i < cnt; i++) s = s + I[49LL * list[i]];
    out[49LL * f + lane] = s;
}

}  // namespace

int gf::obs_frame_info(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv,
                       const gf_keypoint* d_kps, const int32_t* d_nkps, int kp_stride, const int32_t* d_kp2mp,
                       const uint8_t* d_outlier, const float* d_map_pos, const int32_t* d_nmp, int map_stride,
                       const float* level_sigma2, int nlevels, double* d_H, double* d_info, float* d_uv,
                       const int32_t* d_remap, void* stream, double* d_info_lt) {
    GF_CHECK(ctx && cam && level_sigma2, GF_ERR_ARG, "null arg");
    if (nframes <= 0 || kp_stride <= 0) return GF_OK;
    GF_CHECK(nlevels >= 1 && nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    GF_CHECK(d_Xv && d_kps && d_nkps && d_kp2mp && d_map_pos && d_nmp && d_H && d_info && d_uv, GF_ERR_ARG,
             "null arg");
    LevelTab t{};
    for (int i = 0; i < nlevels; i++) t.v[i] = level_sigma2[i];
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_frame_info");
    GF_LAUNCH(k_obs_frame_info, dim3((kp_stride + 127) / 128, nframes), 128, 0, s, 
        *cam, d_Xv, d_kps, d_nkps, kp_stride, d_kp2mp, d_outlier, d_map_pos, d_nmp, map_stride, t, nlevels, d_H,
        d_info, d_uv, d_remap, d_info_lt);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf::obs_map_info(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_map_pos,
                     const int32_t* d_nmp, int map_stride, int check_viz, const gf_mp_view* d_views,
                     int32_t* d_upd_id, int frame_id, double* d_H, double* d_info, float* d_uv, uint8_t* d_updated,
                     const int32_t* d_remap, void* stream, const gf::StageClock& ck, const long long* d_cap2,
                     double* d_info_lt) {
    GF_CHECK(ctx && cam, GF_ERR_ARG, "null arg");
    if (nframes <= 0 || map_stride <= 0) return GF_OK;
    GF_CHECK(d_Xv && d_map_pos && d_nmp && d_upd_id && d_H && d_info && d_uv, GF_ERR_ARG, "null arg");
    GF_CHECK(!ck.t0 || (ck.rec && d_cap2 && map_stride <= 4096), GF_ERR_ARG, "bad clock");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_map_info");
    GF_LAUNCH(k_obs_map_info, dim3((map_stride + 127) / 128, nframes), 128, 0, s, 
        *cam, d_Xv, d_map_pos, d_nmp, map_stride, check_viz, d_views, d_upd_id, frame_id, d_H, d_info, d_uv, d_updated,
        d_remap, ck, d_cap2, d_info_lt);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf::obs_accumulate_matched(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps,
                               int kp_stride, const double* d_info, const int32_t* d_upd_id, const int32_t* d_nmp,
                               int map_stride, int frame_id, double diag, double* d_out, const int32_t* d_remap,
                               void* stream, const int32_t* d_gate) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_kp2mp && d_nkps && d_info && d_upd_id && d_nmp && d_out, GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_obs_accumulate");
    GF_LAUNCH(k_obs_accumulate_matched, nframes, 64, 0, s, d_kp2mp, d_nkps, kp_stride, d_info, d_upd_id, d_nmp, map_stride,
              frame_id, diag, d_out, d_remap, d_gate);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

extern "C" {

int gf_obs_frame_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv,
                          const gf_keypoint* d_kps, const int32_t* d_nkps, int kp_stride, const int32_t* d_kp2mp,
                          const uint8_t* d_outlier, const float* d_map_pos, const int32_t* d_nmp, int map_stride,
                          const float* level_sigma2, int nlevels, double* d_H, double* d_info, float* d_uv,
                          void* stream) {
    return gf::obs_frame_info(ctx, cam, nframes, d_Xv, d_kps, d_nkps, kp_stride, d_kp2mp, d_outlier, d_map_pos, d_nmp,
                              map_stride, level_sigma2, nlevels, d_H, d_info, d_uv, nullptr, stream);
}

int gf_obs_map_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_map_pos,
                        const int32_t* d_nmp, int map_stride, int check_viz, const gf_mp_view* d_views,
                        int32_t* d_upd_id, int frame_id, double* d_H, double* d_info, float* d_uv,
                        uint8_t* d_updated, void* stream) {
    return gf::obs_map_info(ctx, cam, nframes, d_Xv, d_map_pos, d_nmp, map_stride, check_viz, d_views, d_upd_id,
                            frame_id, d_H, d_info, d_uv, d_updated, nullptr, stream);
}

int gf_obs_accumulate_matched_dev(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps,
                                  int kp_stride, const double* d_info, const int32_t* d_upd_id, const int32_t* d_nmp,
                                  int map_stride, int frame_id, double diag, double* d_out, void* stream) {
    return gf::obs_accumulate_matched(ctx, nframes, d_kp2mp, d_nkps, kp_stride, d_info, d_upd_id, d_nmp, map_stride,
                                      frame_id, diag, d_out, nullptr, stream);
}

}  // extern "C"

#ifdef GF_AM_GUARD
extern "C" int gf_debug_am_guard(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_am_guard), sizeof(unsigned long long) * 2) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GF_AM_TRACE
extern "C" int gf_debug_am_trace(uint32_t* out, uint32_t* cnt) {
    if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(g_am_tcnt), sizeof(uint32_t) * 8) != hipSuccess) return -1;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_am_trace), sizeof(uint32_t) * 8 * AMT_MAX * AMT_REC) == hipSuccess
               ? 0 : -1;
}
#endif
#ifdef GF_AM_CHECK
extern "C" int gf_debug_am_check(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_am_check), sizeof(unsigned long long) * 80) == hipSuccess ? 0 : -1;
}
#endif
#ifdef GF_AM_STAMP
// Diagnostic build only (not in the header): phase cycles of k_active_match.
extern "C" int gf_debug_am_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_am_stamp), sizeof(unsigned long long) * 24) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[24] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_am_stamp), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
