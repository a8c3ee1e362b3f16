// Monocular map initialisation on gfx950 — SURVEY.md §8(f) rank 4:
// ORB_SLAM::Initializer::Initialize (src/Initializer.cc:44-132) as five
// kernels:
//   k_init_prepare  block 0/1: Normalize (:873-919) of frame 1/2 — the
//                   reference's sequential float sums, one lane, LDS-staged;
//                   block 2: ordered compaction of vMatches12 (:51-63) and the
//                   mMaxIterations 8-point sets (:80-95) from the caller's
//                   std::rand() state: lane 0 runs glibc's lagged-Fibonacci
//                   recurrence with its 31-word window in registers, then one
//                   lane per iteration turns 8 draws into RandomInt values and
//                   replays the swap-remove of vAvailableIndices as an
//                   overwrite log;
//   k_init_hyp      one workgroup per RANSAC hypothesis, H and F side by side
//                   (FindHomography :241-289 / FindFundamental :292-340):
//                   lane 0 solves the 8-point system (ComputeH21 :343-383,
//                   ComputeF21 :385-421; OpenCV's float Jacobi SVD restated),
//                   the workgroup evaluates CheckHomography (:423-506) /
//                   CheckFundamental (:508-586) per match and lane 0 adds the
//                   terms in match order (the reference's float score);
//   k_init_decide   the first strict best of each search, RH = SH/(SH+SF)
//                   (:117-129), the inlier flags of both kept models, and the
//                   motion hypotheses: ReconstructH's 8 (Faugeras, :690-804) or
//                   ReconstructF's 4 (DecomposeE :1042-1062);
//   k_init_checkrt  one workgroup per motion hypothesis: CheckRT (:922-1040)
//                   per match (4x4 float SVD triangulation :858-871 in
//                   registers), nGood by count, the parallax as the
//                   min(50, nGood-1)-th smallest cosine by a 4-pass radix select
//                   (the value std::sort would put there);
//   k_init_finish   ReconstructH's / ReconstructF's acceptance rules
//                   (:807-856 / :617-688) and the accepted hypothesis' points
//                   (CheckRT re-run for that hypothesis only).
// Arithmetic follows oracle/initializer.cpp operation for operation (float,
// -ffp-contract=off, correctly rounded div/sqrt); docs/ORACLE_ASSUMPTIONS.md
// A16/A17 list the OpenCV readings. Parity: bit-exact against the oracle.
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "common.h"

namespace {

constexpr int IN_T = 256;    // k_init_hyp / k_init_checkrt workgroup
constexpr int IN_BIG = 1024; // single-workgroup kernels
constexpr double kPi = 3.1415926535897932384626433832795;  // CV_PI

// ----------------------------------------------------------- OpenCV restated
struct CvRng {  // cv::RNG
    uint64_t state;
    __device__ unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

// JacobiSVDImpl_<float> (eps 2 FLT_EPSILON, minval FLT_MIN): At holds N rows of
// length M (M x M storage, rows >= N zero); W singular values, Vt (N x N) the
// right vectors as rows. N1 > 0 completes/normalises rows 0..N1-1 of At (the
// left vectors, with cv::RNG(0x12345678) for null ones); N1 = 0 skips that
// step, which touches nothing but the left vectors.
template <int M, int N, int N1>
__device__ void jacobi_f(float* At, float* Wout, float* Vt) {
    const double minval = FLT_MIN;
    const float eps = FLT_EPSILON * 2;
    double W[N];
    constexpr int max_iter = M > 30 ? M : 30;
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const float t = At[i * M + k];
            sd += (double)t * (double)t;
        }
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < N; k++) Vt[i * N + k] = 0.f;
        Vt[i * N + i] = 1.f;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; i++)
#pragma unroll
            for (int j = i + 1; j < N; j++) {
                float *Ai = At + i * M, *Aj = At + j * M;
                double a = W[i], p = 0, b = W[j];
#pragma unroll
                for (int k = 0; k < M; k++) p += (double)Ai[k] * (double)Aj[k];
                if (fabs(p) <= (double)eps * sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = sqrt(p * p + beta * beta);
                float c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = (float)sqrt(delta / gamma);
                    c = (float)(p / (gamma * (double)s * 2));
                } else {
                    c = (float)sqrt((gamma + beta) / (gamma * 2));
                    s = (float)(p / (gamma * (double)c * 2));
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < M; k++) {
                    const float t0 = c * Ai[k] + s * Aj[k];
                    const float t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += (double)t0 * (double)t0;
                    b += (double)t1 * (double)t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                float *Vi = Vt + i * N, *Vj = Vt + j * N;
#pragma unroll
                for (int k = 0; k < N; k++) {
                    const float t0 = c * Vi[k] + s * Vj[k];
                    const float t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; k++) {
            const float t = At[i * M + k];
            sd += (double)t * (double)t;
        }
        W[i] = sqrt(sd);
    }
    // selection sort, descending (compile-time indices: the swaps are selects)
#pragma unroll
    for (int i = 0; i < N - 1; i++) {
        int j = i;
#pragma unroll
        for (int k = i + 1; k < N; k++)
            if (W[j] < W[k]) j = k;
#pragma unroll
        for (int k = i + 1; k < N; k++) {
            if (j != k) continue;
            const double tw = W[i];
            W[i] = W[k];
            W[k] = tw;
#pragma unroll
            for (int q = 0; q < M; q++) {
                const float t = At[i * M + q];
                At[i * M + q] = At[k * M + q];
                At[k * M + q] = t;
            }
#pragma unroll
            for (int q = 0; q < N; q++) {
                const float t = Vt[i * N + q];
                Vt[i * N + q] = Vt[k * N + q];
                Vt[k * N + q] = t;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < N; i++) Wout[i] = (float)W[i];
    if constexpr (N1 > 0) {
        CvRng rng{0x12345678};
        for (int i = 0; i < N1; i++) {
            double sd = i < N ? W[i < N ? i : 0] : 0.;
            for (int ii = 0; ii < 100 && sd <= minval; ii++) {
                const float val0 = (float)(1. / M);
                for (int k = 0; k < M; k++) At[i * M + k] = (rng.next() & 256) != 0 ? val0 : -val0;
                for (int it = 0; it < 2; it++)
                    for (int j = 0; j < i; j++) {
                        sd = 0;
                        for (int k = 0; k < M; k++) sd += (double)(At[i * M + k] * At[j * M + k]);
                        float asum = 0;
                        for (int k = 0; k < M; k++) {
                            const float t = (float)((double)At[i * M + k] - sd * (double)At[j * M + k]);
                            At[i * M + k] = t;
                            asum += fabsf(t);
                        }
                        asum = asum > eps * 100 ? 1 / asum : 0;
                        for (int k = 0; k < M; k++) At[i * M + k] *= asum;
                    }
                sd = 0;
                for (int k = 0; k < M; k++) {
                    const float t = At[i * M + k];
                    sd += (double)t * (double)t;
                }
                sd = sqrt(sd);
            }
            const float s = (float)(sd > minval ? 1 / sd : 0.);
            for (int k = 0; k < M; k++) At[i * M + k] *= s;
        }
    }
}

// cv::SVD::compute(A R x C, FULL_UV) on CV_32F: Ta is an M x M work buffer
// (M = max(R, C)); u (R x R) only when FULLU.
template <int R, int C, bool FULLU>
__device__ void svd_f(const float* A, float* Ta, float* w, float* u, float* vt) {
    constexpr bool at = R < C;
    constexpr int M = at ? C : R, N = at ? R : C;
#pragma unroll
    for (int i = 0; i < M * M; i++) Ta[i] = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int k = 0; k < M; k++) Ta[i * M + k] = at ? A[i * C + k] : A[k * C + i];
    float V[N * N];
    jacobi_f<M, N, FULLU ? M : 0>(Ta, w, V);
    if constexpr (!at) {
        if constexpr (FULLU)
#pragma unroll
            for (int i = 0; i < R; i++)
#pragma unroll
                for (int j = 0; j < R; j++) u[i * R + j] = Ta[j * M + i];
#pragma unroll
        for (int i = 0; i < C * C; i++) vt[i] = V[i];
    } else {
        if constexpr (FULLU)
#pragma unroll
            for (int i = 0; i < R; i++)
#pragma unroll
                for (int j = 0; j < R; j++) u[i * R + j] = V[j * N + i];
#pragma unroll
        for (int i = 0; i < C * C; i++) vt[i] = Ta[i];
    }
}

// small cv::gemm (docs A1): float products summed left to right, then the
// MatExpr scale as a double multiply rounded to float
template <int R, int K, int C>
__device__ void gemm_f(const float* A, const float* B, float* D, double alpha = 1.0) {
    float out[R * C];
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int j = 0; j < C; j++) {
            float s = A[i * K] * B[j];
#pragma unroll
            for (int q = 1; q < K; q++) s = s + A[i * K + q] * B[q * C + j];
            out[i * C + j] = alpha == 1.0 ? s : (float)((double)s * alpha);
        }
#pragma unroll
    for (int i = 0; i < R * C; i++) D[i] = out[i];
}

__device__ void transpose3(const float* A, float* T) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[j * 3 + i] = A[i * 3 + j];
}

__device__ double det3(const float* m) {
    return m[0] * ((double)m[4] * m[8] - (double)m[5] * m[7]) - m[1] * ((double)m[3] * m[8] - (double)m[5] * m[6]) +
           m[2] * ((double)m[3] * m[7] - (double)m[4] * m[6]);
}

__device__ void inv3(const float* S, float* D) {
    double d = det3(S);
    if (d == 0.) {
        for (int i = 0; i < 9; i++) D[i] = 0.f;
        return;
    }
    d = 1. / d;
    D[0] = (float)(((double)S[4] * S[8] - (double)S[5] * S[7]) * d);
    D[1] = (float)(((double)S[2] * S[7] - (double)S[1] * S[8]) * d);
    D[2] = (float)(((double)S[1] * S[5] - (double)S[2] * S[4]) * d);
    D[3] = (float)(((double)S[5] * S[6] - (double)S[3] * S[8]) * d);
    D[4] = (float)(((double)S[0] * S[8] - (double)S[2] * S[6]) * d);
    D[5] = (float)(((double)S[2] * S[3] - (double)S[0] * S[5]) * d);
    D[6] = (float)(((double)S[3] * S[7] - (double)S[4] * S[6]) * d);
    D[7] = (float)(((double)S[1] * S[6] - (double)S[0] * S[7]) * d);
    D[8] = (float)(((double)S[0] * S[4] - (double)S[1] * S[3]) * d);
}

__device__ double norm3(const float* v) {  // cv::norm NORM_L2 (double accumulation)
    double s = 0;
    for (int i = 0; i < 3; i++) s += (double)v[i] * (double)v[i];
    return sqrt(s);
}

__device__ void scale3(const float* v, double alpha, float* out) {  // MatExpr Mat / s
    const float a = (float)alpha;
    for (int i = 0; i < 3; i++) out[i] = v[i] * a;
}

// ----------------------------------------------------------------- kernels
struct InitArgs {
    float K[9];
    float sigma;
    int iters, min_tri;
    const gf_keypoint* k1;
    int n1;
    const gf_keypoint* k2;
    int n2;
    const int32_t* matches;
    gf_rng* rng;
    gf_init_result* res;
    float* p3d;
    uint8_t* tri;
    // scratch
    int32_t* m1;      // [n1] match -> keypoint of frame 1
    int32_t* m2;      // [n1] match -> keypoint of frame 2
    int32_t* ctl;     // [16] N, model, nhyp, Nin
    float* norm;      // [2][4] meanX, meanY, sX, sY
    int32_t* sets;    // [iters][8]
    float* score;     // [2 iters]
    float* mats;      // [2 iters][9]
    uint8_t* inl;     // [n1] inliers of the chosen model
    float* hyp;       // [8][12] R (9), t (3)
    int32_t* ngood;   // [8]
    float* par;       // [8]
    uint32_t* cosk;   // [8][n1] ordered keys of the good cosines
};

// A batch of independent problems (blockIdx.y = problem): problem p's view is
// the base view with the caller's arrays and the scratch block offset by p.
struct InitBatch {
    InitArgs base;
    const int32_t* n1s;  // per-problem sizes (null: base.n1 / base.n2)
    const int32_t* n2s;
    int cap1, cap2;      // rows per problem of the keypoint / match / output arrays
    size_t ws_stride;    // scratch bytes per problem
};

__device__ __forceinline__ InitArgs at(const InitBatch& B, int p) {
    InitArgs A = B.base;
    const long long c1 = (long long)p * B.cap1, c2 = (long long)p * B.cap2;
    A.k1 += c1;
    A.k2 += c2;
    A.matches += c1;
    A.p3d += 3 * c1;
    A.tri += c1;
    A.rng += p;
    A.res += p;
    if (B.n1s) {
        A.n1 = min(max(B.n1s[p], 0), B.cap1);
        A.n2 = min(max(B.n2s[p], 0), B.cap2);
    }
    const size_t o = (size_t)p * B.ws_stride;
    auto sh = [o](auto* q) { return reinterpret_cast<decltype(q)>(reinterpret_cast<char*>(q) + o); };
    A.m1 = sh(A.m1);
    A.m2 = sh(A.m2);
    A.ctl = sh(A.ctl);
    A.norm = sh(A.norm);
    A.sets = sh(A.sets);
    A.score = sh(A.score);
    A.mats = sh(A.mats);
    A.inl = sh(A.inl);
    A.hyp = sh(A.hyp);
    A.ngood = sh(A.ngood);
    A.par = sh(A.par);
    A.cosk = sh(A.cosk);
    return A;
}

enum { C_N = 0, C_MODEL = 1, C_NHYP = 2, C_NIN = 3 };

__global__ __launch_bounds__(IN_BIG) void k_init_prepare(InitBatch Bt) {
    const InitArgs A = at(Bt, blockIdx.y);
    __shared__ float xs[IN_BIG], ys[IN_BIG];
    __shared__ int tmp[IN_BIG / 64];
    const int tid = threadIdx.x;
    if (blockIdx.x < 2) {  // Normalize (:873-919)
        const int f = blockIdx.x;
        const gf_keypoint* kp = f ? A.k2 : A.k1;
        const int n = f ? A.n2 : A.n1;
        float meanX = 0, meanY = 0, devX = 0, devY = 0;
        for (int c0 = 0; c0 < n; c0 += IN_BIG) {
            const int i = c0 + tid;
            if (i < n) {
                xs[tid] = kp[i].x;
                ys[tid] = kp[i].y;
            }
            __syncthreads();
            if (tid == 0)
                for (int j = 0; j < min(IN_BIG, n - c0); j++) {
                    meanX += xs[j];
                    meanY += ys[j];
                }
            __syncthreads();
        }
        if (tid == 0) {
            meanX = meanX / (float)n;
            meanY = meanY / (float)n;
            xs[0] = meanX;
            ys[0] = meanY;
        }
        __syncthreads();
        meanX = xs[0];
        meanY = ys[0];
        __syncthreads();
        for (int c0 = 0; c0 < n; c0 += IN_BIG) {
            const int i = c0 + tid;
            if (i < n) {
                xs[tid] = fabsf(kp[i].x - meanX);
                ys[tid] = fabsf(kp[i].y - meanY);
            }
            __syncthreads();
            if (tid == 0)
                for (int j = 0; j < min(IN_BIG, n - c0); j++) {
                    devX += xs[j];
                    devY += ys[j];
                }
            __syncthreads();
        }
        if (tid == 0) {
            devX = devX / (float)n;
            devY = devY / (float)n;
            float* o = A.norm + 4 * f;
            o[0] = meanX;
            o[1] = meanY;
            o[2] = (float)(1.0 / devX);
            o[3] = (float)(1.0 / devY);
        }
        return;
    }
    // block 2: matches in frame-1 order (:51-63)
    const int lane = tid & 63, wid = tid >> 6;
    int N = 0;
    for (int c0 = 0; c0 < A.n1; c0 += IN_BIG) {
        const int i = c0 + tid;
        const int m = i < A.n1 ? A.matches[i] : -1;
        const bool on = m >= 0;
        const unsigned long long b = __ballot(on);
        const int below = __popcll(b & ((1ull << lane) - 1ull));
        if (lane == 0) tmp[wid] = __popcll(b);
        __syncthreads();
        int base = 0, tot = 0;
        for (int w = 0; w < IN_BIG / 64; w++) {
            base += w < wid ? tmp[w] : 0;
            tot += tmp[w];
        }
        if (on) {
            A.m1[N + base + below] = i;
            A.m2[N + base + below] = m;
        }
        N += tot;
        __syncthreads();
    }
    if (tid == 0) A.ctl[C_N] = N;
    if (N < 8) return;
    // the 8-point sets (:80-95). glibc's TYPE_3 generator is x_k = x_{k-31} +
    // x_{k-3}: lane 0 runs it 31 steps per unrolled block with the window in
    // registers and stores every x_k (raw, full 32 bits) into the sets buffer
    const int n = 8 * A.iters;
    uint32_t* raw = reinterpret_cast<uint32_t*>(A.sets);
    const int f0 = A.rng->f, r0 = A.rng->r;
    if (tid == 0) {
        uint32_t w[31];  // w[i] = x_{i-31}: the state word at (f0 + i) % 31
#pragma unroll
        for (int i = 0; i < 31; i++) w[i] = (uint32_t)A.rng->state[(f0 + i) % 31];
        for (int b0 = 0; b0 < n; b0 += 31) {
#pragma unroll
            for (int j = 0; j < 31; j++) {
                const uint32_t x = w[j] + w[(j + 28) % 31];
                w[j] = x;
                if (b0 + j < n) raw[b0 + j] = x;
            }
        }
    }
    __syncthreads();
    // the caller's state after n draws: x_k sits at position (f0 + k) % 31
    if (tid < 31) {
        const int k0 = (tid - f0 + 31) % 31;
        if (k0 <= n - 1) A.rng->state[tid] = (int32_t)raw[k0 + 31 * ((n - 1 - k0) / 31)];
    }
    if (tid == 31) {
        A.rng->f = (f0 + n) % 31;
        A.rng->r = (r0 + n) % 31;
    }
    __syncthreads();
    // one lane per iteration: RandomInt(0, size-1) and the swap-remove of
    // vAvailableIndices = 0..N-1, kept as an overwrite log of <= 8 entries
    for (int it = tid; it < A.iters; it += IN_BIG) {
        uint32_t x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) x[j] = raw[it * 8 + j];
        int opos[8], oval[8], no = 0, size = N;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int randi = int(((double)(int32_t)(x[j] >> 1) / ((double)2147483647 + 1.0)) * size);
            int idx = randi, back = size - 1;
#pragma unroll
            for (int o = 0; o < 8; o++)
                if (o < no) {
                    if (opos[o] == randi) idx = oval[o];
                    if (opos[o] == size - 1) back = oval[o];
                }
            A.sets[it * 8 + j] = idx;
            bool found = false;  // vAvailableIndices[randi] = back
#pragma unroll
            for (int o = 0; o < 8; o++)
                if (o < no && opos[o] == randi) {
                    oval[o] = back;
                    found = true;
                }
            if (!found) {
#pragma unroll
                for (int o = 0; o < 8; o++)
                    if (o == no) {
                        opos[o] = randi;
                        oval[o] = back;
                    }
                no++;
            }
            size--;
        }
    }
}

__device__ __forceinline__ void norm_T(const float* nm, float* T) {  // Normalize's T
    T[0] = nm[2], T[1] = 0.f, T[2] = -nm[0] * nm[2];
    T[3] = 0.f, T[4] = nm[3], T[5] = -nm[1] * nm[3];
    T[6] = 0.f, T[7] = 0.f, T[8] = 1.f;
}

// CheckHomography / CheckFundamental terms of one match: the two score
// increments (0 when the side is rejected) and the inlier flag
__device__ __forceinline__ bool check_h(const float* H21, const float* H12, float u1, float v1, float u2, float v2,
                                        float invS2, float& s1, float& s2) {
    const float th = 5.991f;
    bool in = true;
    const float w2in1inv = (float)(1.0 / (double)(H12[6] * u2 + H12[7] * v2 + H12[8]));
    const float u2in1 = (H12[0] * u2 + H12[1] * v2 + H12[2]) * w2in1inv;
    const float v2in1 = (H12[3] * u2 + H12[4] * v2 + H12[5]) * w2in1inv;
    const float c1 = ((u1 - u2in1) * (u1 - u2in1) + (v1 - v2in1) * (v1 - v2in1)) * invS2;
    s1 = 0.f;
    if (c1 > th)
        in = false;
    else
        s1 = th - c1;
    const float w1in2inv = (float)(1.0 / (double)(H21[6] * u1 + H21[7] * v1 + H21[8]));
    const float u1in2 = (H21[0] * u1 + H21[1] * v1 + H21[2]) * w1in2inv;
    const float v1in2 = (H21[3] * u1 + H21[4] * v1 + H21[5]) * w1in2inv;
    const float c2 = ((u2 - u1in2) * (u2 - u1in2) + (v2 - v1in2) * (v2 - v1in2)) * invS2;
    s2 = 0.f;
    if (c2 > th)
        in = false;
    else
        s2 = th - c2;
    return in;
}

__device__ __forceinline__ bool check_f(const float* F, float u1, float v1, float u2, float v2, float invS2,
                                        float& s1, float& s2) {
    const float th = 3.841f, thScore = 5.991f;
    bool in = true;
    const float a2 = F[0] * u1 + F[1] * v1 + F[2], b2 = F[3] * u1 + F[4] * v1 + F[5], c2 = F[6] * u1 + F[7] * v1 + F[8];
    const float num2 = a2 * u2 + b2 * v2 + c2;
    const float ch1 = (num2 * num2 / (a2 * a2 + b2 * b2)) * invS2;
    s1 = 0.f;
    if (ch1 > th)
        in = false;
    else
        s1 = thScore - ch1;
    const float a1 = F[0] * u2 + F[3] * v2 + F[6], b1 = F[1] * u2 + F[4] * v2 + F[7], c1 = F[2] * u2 + F[5] * v2 + F[8];
    const float num1 = a1 * u1 + b1 * v1 + c1;
    const float ch2 = (num1 * num1 / (a1 * a1 + b1 * b1)) * invS2;
    s2 = 0.f;
    if (ch2 > th)
        in = false;
    else
        s2 = thScore - ch2;
    return in;
}

__global__ __launch_bounds__(IN_T) void k_init_hyp(InitBatch Bt) {
    const InitArgs A = at(Bt, blockIdx.y);
    __shared__ float Ta[16 * 16];
    __shared__ float Hs[18];
    __shared__ float t1[IN_T], t2[IN_T];
    const int N = A.ctl[C_N];
    if (N < 8) return;
    const int tid = threadIdx.x;
    const bool isF = blockIdx.x >= (unsigned)A.iters;
    const int it = isF ? blockIdx.x - A.iters : blockIdx.x;
    if (tid == 0) {
        const float* n1 = A.norm;
        const float* n2 = A.norm + 4;
        float T1[9], T2[9];
        norm_T(n1, T1);
        norm_T(n2, T2);
        float p1x[8], p1y[8], p2x[8], p2y[8];
        for (int j = 0; j < 8; j++) {
            const int idx = A.sets[it * 8 + j];
            const gf_keypoint a = A.k1[A.m1[idx]], b = A.k2[A.m2[idx]];
            p1x[j] = (a.x - n1[0]) * n1[2];
            p1y[j] = (a.y - n1[1]) * n1[3];
            p2x[j] = (b.x - n2[0]) * n2[2];
            p2y[j] = (b.y - n2[1]) * n2[3];
        }
        float tmp[9], M21[9];
        if (!isF) {  // ComputeH21: A (16 x 9), SVD without the transpose
            float Am[16 * 9];
            for (int i = 0; i < 8; i++) {
                const float u1 = p1x[i], v1 = p1y[i], u2 = p2x[i], v2 = p2y[i];
                float* r0 = Am + (2 * i) * 9;
                float* r1 = Am + (2 * i + 1) * 9;
                r0[0] = 0.f, r0[1] = 0.f, r0[2] = 0.f, r0[3] = -u1, r0[4] = -v1, r0[5] = -1.f;
                r0[6] = v2 * u1, r0[7] = v2 * v1, r0[8] = v2;
                r1[0] = u1, r1[1] = v1, r1[2] = 1.f, r1[3] = 0.f, r1[4] = 0.f, r1[5] = 0.f;
                r1[6] = -u2 * u1, r1[7] = -u2 * v1, r1[8] = -u2;
            }
            float w[9], vt[81];
            svd_f<16, 9, false>(Am, Ta, w, nullptr, vt);
            float T2inv[9];
            inv3(T2, T2inv);
            gemm_f<3, 3, 3>(T2inv, vt + 72, tmp);
            gemm_f<3, 3, 3>(tmp, T1, M21);
            for (int i = 0; i < 9; i++) Hs[i] = M21[i];
            inv3(M21, Hs + 9);
        } else {  // ComputeF21: A (8 x 9) -> transposed SVD, row 8 of the completed vt
            float Am[8 * 9];
            for (int i = 0; i < 8; i++) {
                const float u1 = p1x[i], v1 = p1y[i], u2 = p2x[i], v2 = p2y[i];
                float* r = Am + i * 9;
                r[0] = u2 * u1, r[1] = u2 * v1, r[2] = u2, r[3] = v2 * u1, r[4] = v2 * v1, r[5] = v2;
                r[6] = u1, r[7] = v1, r[8] = 1.f;
            }
            float w[8], u8[64], vt[81];
            svd_f<8, 9, true>(Am, Ta, w, u8, vt);
            float w3[3], u3[9], vt3[9], D[9], UD[9], Fn[9], T2t[9];
            svd_f<3, 3, true>(vt + 72, Ta, w3, u3, vt3);
            w3[2] = 0.f;
            D[0] = w3[0], D[1] = 0.f, D[2] = 0.f, D[3] = 0.f, D[4] = w3[1], D[5] = 0.f, D[6] = 0.f, D[7] = 0.f;
            D[8] = w3[2];
            gemm_f<3, 3, 3>(u3, D, UD);
            gemm_f<3, 3, 3>(UD, vt3, Fn);
            transpose3(T2, T2t);
            gemm_f<3, 3, 3>(T2t, Fn, tmp);
            gemm_f<3, 3, 3>(tmp, T1, M21);
            for (int i = 0; i < 9; i++) Hs[i] = M21[i];
        }
        float* o = A.mats + (size_t)blockIdx.x * 9;
        for (int i = 0; i < 9; i++) o[i] = M21[i];
    }
    __syncthreads();
    float M21[9], M12[9];
    for (int i = 0; i < 9; i++) M21[i] = Hs[i];
    if (!isF)
        for (int i = 0; i < 9; i++) M12[i] = Hs[9 + i];
    const float invS2 = (float)(1.0 / (double)(A.sigma * A.sigma));
    float score = 0.f;
    for (int c0 = 0; c0 < N; c0 += IN_T) {
        const int i = c0 + tid;
        if (i < N) {
            const gf_keypoint a = A.k1[A.m1[i]], b = A.k2[A.m2[i]];
            float s1, s2;
            if (!isF)
                check_h(M21, M12, a.x, a.y, b.x, b.y, invS2, s1, s2);
            else
                check_f(M21, a.x, a.y, b.x, b.y, invS2, s1, s2);
            t1[tid] = s1;
            t2[tid] = s2;
        }
        __syncthreads();
        if (tid == 0)
            for (int j = 0; j < min(IN_T, N - c0); j++) {
                score += t1[j];
                score += t2[j];
            }
        __syncthreads();
    }
    if (tid == 0) A.score[blockIdx.x] = score;
}

// CheckRT set-up of one hypothesis (:926-950)
struct RT {
    float R[9], t[3], P1[12], P2[12], O2[3];
};

__device__ void rt_setup(const float* K, const float* Rt, RT& C) {
    for (int i = 0; i < 9; i++) C.R[i] = Rt[i];
    for (int i = 0; i < 3; i++) C.t[i] = Rt[9 + i];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) C.P1[r * 4 + c] = K[r * 3 + c];
        C.P1[r * 4 + 3] = 0.f;
    }
    float P[12];
    for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) P[r * 4 + c] = C.R[r * 3 + c];
        P[r * 4 + 3] = C.t[r];
    }
    gemm_f<3, 3, 4>(K, P, C.P2);
    float RT_[9];
    transpose3(C.R, RT_);
    gemm_f<3, 3, 1>(RT_, C.t, C.O2, -1.0);
}

// one match of CheckRT (:954-1027): 0 rejected, 1 counted, 2 counted and vbGood
__device__ int check_match(const RT& C, const float* K, float th2, const gf_keypoint& kp1, const gf_keypoint& kp2,
                           float* p, float& cosParallax) {
    float Am[16];
    auto row = [&](float x, const float* P, int r, float* out) {
#pragma unroll
        for (int c = 0; c < 4; c++)
            out[c] = (float)((double)P[8 + c] * (double)x + (double)P[4 * r + c] * -1.0 + 0.0);
    };
    row(kp1.x, C.P1, 0, Am);
    row(kp1.y, C.P1, 1, Am + 4);
    row(kp2.x, C.P2, 0, Am + 8);
    row(kp2.y, C.P2, 1, Am + 12);
    float Ta[16], w[4], vt[16];
    svd_f<4, 4, false>(Am, Ta, w, nullptr, vt);
    scale3(vt + 12, 1.0 / (double)vt[15], p);
    if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) return 0;
    const float n1v[3] = {p[0] - 0.f, p[1] - 0.f, p[2] - 0.f};
    const float dist1 = (float)norm3(n1v);
    const float n2v[3] = {p[0] - C.O2[0], p[1] - C.O2[1], p[2] - C.O2[2]};
    const float dist2 = (float)norm3(n2v);
    double dot = 0;
    for (int r = 0; r < 3; r++) dot += (double)n1v[r] * (double)n2v[r];
    cosParallax = (float)(dot / (double)(dist1 * dist2));
    if (p[2] <= 0 && (double)cosParallax < 0.99998) return 0;
    float p2[3];
    for (int r = 0; r < 3; r++) {
        const float x = C.R[3 * r] * p[0], y = C.R[3 * r + 1] * p[1], z = C.R[3 * r + 2] * p[2];
        p2[r] = ((x + y) + z) + C.t[r];
    }
    if (p2[2] <= 0 && (double)cosParallax < 0.99998) return 0;
    const float fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    const float invZ1 = (float)(1.0 / (double)p[2]);
    const float im1x = fx * p[0] * invZ1 + cx, im1y = fy * p[1] * invZ1 + cy;
    const float e1 = (im1x - kp1.x) * (im1x - kp1.x) + (im1y - kp1.y) * (im1y - kp1.y);
    if (e1 > th2) return 0;
    const float invZ2 = (float)(1.0 / (double)p2[2]);
    const float im2x = fx * p2[0] * invZ2 + cx, im2y = fy * p2[1] * invZ2 + cy;
    const float e2 = (im2x - kp2.x) * (im2x - kp2.x) + (im2y - kp2.y) * (im2y - kp2.y);
    if (e2 > th2) return 0;
    return (double)cosParallax < 0.99998 ? 2 : 1;
}

__global__ __launch_bounds__(IN_BIG) void k_init_decide(InitBatch Bt) {
    const InitArgs A = at(Bt, blockIdx.y);
    __shared__ float sh[2 * 9 + 9];
    __shared__ int si[4];
    __shared__ int cntH, cntF;
    const int tid = threadIdx.x;
    const int N = A.ctl[C_N];
    gf_init_result* R = A.res;
    for (int i = tid; i < A.n1; i += IN_BIG) {
        A.p3d[3 * i] = 0.f;
        A.p3d[3 * i + 1] = 0.f;
        A.p3d[3 * i + 2] = 0.f;
        A.tri[i] = 0;
    }
    if (tid == 0) {
        cntH = cntF = 0;
        float SH = 0.f, SF = 0.f;
        int iH = -1, iF = -1;
        if (N >= 8)
            for (int it = 0; it < A.iters; it++) {
                const float h = A.score[it], f = A.score[A.iters + it];
                if (h > SH) SH = h, iH = it;
                if (f > SF) SF = f, iF = it;
            }
        si[0] = iH;
        si[1] = iF;
        const float RH = (SH == 0.f && SF == 0.f) ? 0.f : SH / (SH + SF);  // 0/0 reported as 0
        const int model = N < 8 ? -1 : (SH == 0.f && SF == 0.f) ? -1 : (double)RH > 0.40 ? 0 : 1;
        si[2] = model;
        for (int i = 0; i < 9; i++) {
            sh[i] = iH >= 0 ? A.mats[(size_t)iH * 9 + i] : 0.f;
            sh[9 + i] = iF >= 0 ? A.mats[(size_t)(A.iters + iF) * 9 + i] : 0.f;
        }
        inv3(sh, sh + 18);
        R->ok = 0;
        R->model = model;
        R->nmatches = N;
        R->iter_H = iH;
        R->iter_F = iF;
        R->best = -1;
        R->SH = SH;
        R->SF = SF;
        R->RH = RH;
        R->parallax = 0.f;
        for (int i = 0; i < 8; i++) R->ngood[i] = 0;
        for (int i = 0; i < 9; i++) {
            R->H21[i] = sh[i];
            R->F21[i] = sh[9 + i];
            R->R21[i] = 0.f;
        }
        for (int i = 0; i < 3; i++) R->t21[i] = 0.f;
        A.ctl[C_MODEL] = model;
        A.ctl[C_NHYP] = 0;
    }
    __syncthreads();
    const int iH = si[0], iF = si[1], model = si[2];
    if (model < 0) {
        if (tid == 0) R->ninliers_H = R->ninliers_F = 0;
        return;
    }
    // inlier flags of the kept models (the same per-match test that scored them)
    float H21[9], H12[9], F21[9];
    for (int i = 0; i < 9; i++) H21[i] = sh[i], F21[i] = sh[9 + i], H12[i] = sh[18 + i];
    const float invS2 = (float)(1.0 / (double)(A.sigma * A.sigma));
    int ch = 0, cf = 0;
    for (int i = tid; i < N; i += IN_BIG) {
        const gf_keypoint a = A.k1[A.m1[i]], b = A.k2[A.m2[i]];
        float s1, s2;
        const bool inH = iH >= 0 && check_h(H21, H12, a.x, a.y, b.x, b.y, invS2, s1, s2);
        const bool inF = iF >= 0 && check_f(F21, a.x, a.y, b.x, b.y, invS2, s1, s2);
        ch += inH;
        cf += inF;
        A.inl[i] = model == 0 ? inH : inF;
    }
    atomicAdd(&cntH, ch);
    atomicAdd(&cntF, cf);
    __syncthreads();
    if (tid != 0) return;
    R->ninliers_H = cntH;
    R->ninliers_F = cntF;
    A.ctl[C_NIN] = model == 0 ? cntH : cntF;
    const float* K = A.K;
    float Ta[9];
    if (model == 0) {  // ReconstructH (:690-804)
        float invK[9], tmp[9], Am[9], w[3], U[9], Vt[9];
        inv3(K, invK);
        gemm_f<3, 3, 3>(invK, H21, tmp);
        gemm_f<3, 3, 3>(tmp, K, Am);
        svd_f<3, 3, true>(Am, Ta, w, U, Vt);
        const float s = (float)(det3(U) * det3(Vt));
        const float d1 = w[0], d2 = w[1], d3 = w[2];
        if ((double)(d1 / d2) < 1.00001 || (double)(d2 / d3) < 1.00001) return;
        const float aux1 = sqrtf((d1 * d1 - d2 * d2) / (d1 * d1 - d3 * d3));
        const float aux3 = sqrtf((d2 * d2 - d3 * d3) / (d1 * d1 - d3 * d3));
        const float x1[] = {aux1, aux1, -aux1, -aux1}, x3[] = {aux3, -aux3, aux3, -aux3};
        const float aux_stheta = sqrtf((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 + d3) * d2);
        const float ctheta = (d2 * d2 + d1 * d3) / ((d1 + d3) * d2);
        const float stheta[] = {aux_stheta, -aux_stheta, -aux_stheta, aux_stheta};
        const float aux_sphi = sqrtf((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 - d3) * d2);
        const float cphi = (d1 * d3 - d2 * d2) / ((d1 - d3) * d2);
        const float sphi[] = {aux_sphi, -aux_sphi, -aux_sphi, aux_sphi};
        for (int i = 0; i < 8; i++) {
            const bool second = i >= 4;
            const int q = i & 3;
            float Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            if (!second) {
                Rp[0] = ctheta, Rp[2] = -stheta[q], Rp[6] = stheta[q], Rp[8] = ctheta;
            } else {
                Rp[0] = cphi, Rp[2] = sphi[q], Rp[4] = -1.f, Rp[6] = sphi[q], Rp[8] = -cphi;
            }
            float URp[9];
            float* h = A.hyp + 12 * i;
            gemm_f<3, 3, 3>(U, Rp, URp, (double)s);
            gemm_f<3, 3, 3>(URp, Vt, h);
            float tp[3] = {x1[q], 0.f, second ? x3[q] : -x3[q]};
            const float sc = second ? d1 + d3 : d1 - d3;
            for (int r = 0; r < 3; r++) tp[r] = tp[r] * sc;
            float tt[3];
            gemm_f<3, 3, 1>(U, tp, tt);
            scale3(tt, 1.0 / norm3(tt), h + 9);
        }
        A.ctl[C_NHYP] = 8;
    } else {  // ReconstructF (:588-615) with DecomposeE (:1042-1062)
        float KT[9], tmp[9], E[9], w[3], u[9], vt[9];
        transpose3(K, KT);
        gemm_f<3, 3, 3>(KT, F21, tmp);
        gemm_f<3, 3, 3>(tmp, K, E);
        svd_f<3, 3, true>(E, Ta, w, u, vt);
        float t[3];
        const float tt[3] = {u[2], u[5], u[8]};
        scale3(tt, 1.0 / norm3(tt), t);
        const float W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
        float WT[9], UW[9], R1[9], R2[9];
        transpose3(W, WT);
        gemm_f<3, 3, 3>(u, W, UW);
        gemm_f<3, 3, 3>(UW, vt, R1);
        if (det3(R1) < 0)
            for (int i = 0; i < 9; i++) R1[i] = -R1[i];
        gemm_f<3, 3, 3>(u, WT, UW);
        gemm_f<3, 3, 3>(UW, vt, R2);
        if (det3(R2) < 0)
            for (int i = 0; i < 9; i++) R2[i] = -R2[i];
        for (int i = 0; i < 4; i++) {  // (R1,t) (R2,t) (R1,-t) (R2,-t)
            float* h = A.hyp + 12 * i;
            const float* Rs = (i & 1) ? R2 : R1;
            for (int k = 0; k < 9; k++) h[k] = Rs[k];
            for (int k = 0; k < 3; k++) h[9 + k] = i < 2 ? t[k] : -t[k];
        }
        A.ctl[C_NHYP] = 4;
    }
}

__device__ __forceinline__ uint32_t ord_key(float c) {  // order-preserving float -> uint
    const uint32_t u = __float_as_uint(c);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_val(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(IN_T) void k_init_checkrt(InitBatch Bt) {
    const InitArgs A = at(Bt, blockIdx.y);
    __shared__ int s_cnt;
    __shared__ int hist[256];
    __shared__ uint32_t s_prefix;
    __shared__ int s_rank;
    const int h = blockIdx.x, tid = threadIdx.x;
    if (h >= A.ctl[C_NHYP]) return;
    const int N = A.ctl[C_N];
    RT C;
    rt_setup(A.K, A.hyp + 12 * h, C);
    const float th2 = (float)(4.0 * (double)(A.sigma * A.sigma));
    if (tid == 0) s_cnt = 0;
    __syncthreads();
    uint32_t* keys = A.cosk + (size_t)h * A.n1;
    for (int i = tid; i < N; i += IN_T) {
        if (!A.inl[i]) continue;
        float p[3], cp;
        const int st = check_match(C, A.K, th2, A.k1[A.m1[i]], A.k2[A.m2[i]], p, cp);
        if (st) keys[atomicAdd(&s_cnt, 1)] = ord_key(cp);
    }
    __syncthreads();
    const int ng = s_cnt;
    float parallax = 0.f;
    if (ng > 0) {
        // the min(50, nGood-1)-th smallest: radix select, 8 bits a pass
        if (tid == 0) {
            s_prefix = 0;
            s_rank = min(50, ng - 1);
        }
        for (int pass = 0; pass < 4; pass++) {
            const int shift = 24 - 8 * pass;
            const uint32_t mask = pass ? 0xffffffffu << (32 - 8 * pass) : 0u;
            hist[tid] = 0;
            __syncthreads();
            const uint32_t pre = s_prefix;
            for (int j = tid; j < ng; j += IN_T) {
                const uint32_t k = keys[j];
                if ((k & mask) == pre) atomicAdd(&hist[(k >> shift) & 255], 1);
            }
            __syncthreads();
            if (tid == 0) {
                int r = s_rank, d = 0;
                while (r >= hist[d]) r -= hist[d++];
                s_rank = r;
                s_prefix = pre | ((uint32_t)d << shift);
            }
            __syncthreads();
        }
        const float c = key_val(s_prefix);
        const float ac = (float)acos((double)c);
        parallax = (float)((double)(ac * 180.f) / kPi);
    }
    if (tid == 0) {
        A.ngood[h] = ng;
        A.par[h] = parallax;
    }
}

__global__ __launch_bounds__(IN_BIG) void k_init_finish(InitBatch Bt) {
    const InitArgs A = at(Bt, blockIdx.y);
    __shared__ int s_best;
    const int tid = threadIdx.x;
    const int nh = A.ctl[C_NHYP];
    if (nh == 0) return;
    gf_init_result* R = A.res;
    if (tid == 0) {
        const int Nin = A.ctl[C_NIN];
        int acc = -1;
        for (int i = 0; i < nh; i++) R->ngood[i] = A.ngood[i];
        if (nh == 8) {  // ReconstructH (:807-856)
            int bestGood = 0, second = 0, best = -1;
            float bestPar = -1.f;
            for (int i = 0; i < 8; i++) {
                const int g = A.ngood[i];
                if (g > bestGood) {
                    second = bestGood;
                    bestGood = g;
                    best = i;
                    bestPar = A.par[i];
                } else if (g > second) {
                    second = g;
                }
            }
            R->best = best;
            R->parallax = bestPar;
            if (second < 0.75 * bestGood && bestPar >= 1.0f && bestGood > A.min_tri && bestGood > 0.9 * Nin)
                acc = best;
        } else {  // ReconstructF (:617-688)
            int maxGood = 0;
            for (int i = 0; i < 4; i++) maxGood = max(maxGood, A.ngood[i]);
            const int nMinGood = max(static_cast<int>(0.9 * Nin), A.min_tri);
            int nsimilar = 0;
            for (int i = 0; i < 4; i++) nsimilar += A.ngood[i] > 0.7 * maxGood;
            int b = 0;
            while (A.ngood[b] != maxGood) b++;
            R->best = b;
            R->parallax = A.par[b];
            if (!(maxGood < nMinGood || nsimilar > 1) && A.par[b] > 1.0f) acc = b;
        }
        if (acc >= 0) {
            R->ok = 1;
            for (int i = 0; i < 9; i++) R->R21[i] = A.hyp[12 * acc + i];
            for (int i = 0; i < 3; i++) R->t21[i] = A.hyp[12 * acc + 9 + i];
        }
        s_best = acc;
    }
    __syncthreads();
    const int b = s_best;
    if (b < 0) return;
    RT C;
    rt_setup(A.K, A.hyp + 12 * b, C);
    const float th2 = (float)(4.0 * (double)(A.sigma * A.sigma));
    const int N = A.ctl[C_N];
    for (int i = tid; i < N; i += IN_BIG) {
        if (!A.inl[i]) continue;
        float p[3], cp;
        const int st = check_match(C, A.K, th2, A.k1[A.m1[i]], A.k2[A.m2[i]], p, cp);
        if (!st) continue;
        const int k = A.m1[i];
        A.p3d[3 * k] = p[0];
        A.p3d[3 * k + 1] = p[1];
        A.p3d[3 * k + 2] = p[2];
        A.tri[k] = st == 2;
    }
}

static int init_launch(gf_ctx* ctx, int nprob, const float K[9], float sigma, int iterations, int min_triangulated,
                       const gf_keypoint* d_kps1, int n1, int cap1, const int32_t* d_n1, const gf_keypoint* d_kps2,
                       int n2, int cap2, const int32_t* d_n2, const int32_t* d_matches12, gf_rng* d_rng,
                       gf_init_result* d_result, float* d_p3d, uint8_t* d_triangulated, void* stream) {
    GF_CHECK(iterations > 0 && iterations <= 65536, GF_ERR_ARG, "gf_initialize: iterations out of range");
    GF_CHECK(sigma > 0.f, GF_ERR_ARG, "gf_initialize: sigma <= 0");
    const size_t nn = (size_t)std::max(cap1, 1), it = (size_t)iterations;
    // one scratch block per problem (slot 62): m1, m2, sets, ctl, norm, score, mats, hyp, ngood, par, cosk, inl
    const size_t off_m1 = 0, off_m2 = off_m1 + 4 * nn, off_sets = off_m2 + 4 * nn, off_ctl = off_sets + 32 * it,
                 off_norm = off_ctl + 64, off_score = off_norm + 32, off_mats = off_score + 8 * it,
                 off_hyp = off_mats + 72 * it, off_ngood = off_hyp + 4 * 96, off_par = off_ngood + 32,
                 off_cosk = off_par + 32, off_inl = off_cosk + 32 * nn, per = (off_inl + nn + 255) & ~(size_t)255;
    void* ws = nullptr;
    int rc = gf::ws_get(ctx, 62, per * (size_t)nprob, &ws);
    if (rc) return rc;
    char* b = (char*)ws;
    InitBatch Bt{};
    InitArgs& A = Bt.base;
    for (int i = 0; i < 9; i++) A.K[i] = K[i];
    A.sigma = sigma;
    A.iters = iterations;
    A.min_tri = min_triangulated;
    A.k1 = d_kps1;
    A.n1 = n1;
    A.k2 = d_kps2;
    A.n2 = n2;
    A.matches = d_matches12;
    A.rng = d_rng;
    A.res = d_result;
    A.p3d = d_p3d;
    A.tri = d_triangulated;
    A.m1 = (int32_t*)(b + off_m1);
    A.m2 = (int32_t*)(b + off_m2);
    A.sets = (int32_t*)(b + off_sets);
    A.ctl = (int32_t*)(b + off_ctl);
    A.norm = (float*)(b + off_norm);
    A.score = (float*)(b + off_score);
    A.mats = (float*)(b + off_mats);
    A.hyp = (float*)(b + off_hyp);
    A.ngood = (int32_t*)(b + off_ngood);
    A.par = (float*)(b + off_par);
    A.cosk = (uint32_t*)(b + off_cosk);
    A.inl = (uint8_t*)(b + off_inl);
    Bt.n1s = d_n1;
    Bt.n2s = d_n2;
    Bt.cap1 = cap1;
    Bt.cap2 = cap2;
    Bt.ws_stride = per;
    hipStream_t s = (hipStream_t)stream;
    {
        GF_PROF(ctx, s, "k_init_prepare");
        GF_LAUNCH(k_init_prepare, dim3(3, nprob), IN_BIG, 0, s, Bt);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_init_hyp");
        GF_LAUNCH(k_init_hyp, dim3(2 * iterations, nprob), IN_T, 0, s, Bt);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_init_decide");
        GF_LAUNCH(k_init_decide, dim3(1, nprob), IN_BIG, 0, s, Bt);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_init_checkrt");
        GF_LAUNCH(k_init_checkrt, dim3(8, nprob), IN_T, 0, s, Bt);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_init_finish");
        GF_LAUNCH(k_init_finish, dim3(1, nprob), IN_BIG, 0, s, Bt);
        GF_HIP(hipGetLastError());
    }
    return GF_OK;
}

}  // namespace

extern "C" {

int gf_initialize_dev(gf_ctx* ctx, const float K[9], float sigma, int iterations, int min_triangulated,
                      const gf_keypoint* d_kps1, int n1, const gf_keypoint* d_kps2, int n2,
                      const int32_t* d_matches12, gf_rng* d_rng, gf_init_result* d_result, float* d_p3d,
                      uint8_t* d_triangulated, void* stream) {
    GF_CHECK(ctx && K, GF_ERR_ARG, "gf_initialize_dev: null arg");
    GF_CHECK(d_kps1 && d_kps2 && d_matches12 && d_rng && d_result && d_p3d && d_triangulated, GF_ERR_ARG,
             "gf_initialize_dev: null buffer");
    GF_CHECK(n1 > 0 && n2 > 0, GF_ERR_ARG, "gf_initialize_dev: empty frame");
    return init_launch(ctx, 1, K, sigma, iterations, min_triangulated, d_kps1, n1, n1, nullptr, d_kps2, n2, n2,
                       nullptr, d_matches12, d_rng, d_result, d_p3d, d_triangulated, stream);
}

int gf_initialize_batch_dev(gf_ctx* ctx, int nprob, const float K[9], float sigma, int iterations,
                            int min_triangulated, const gf_keypoint* d_kps1, int cap1, const int32_t* d_n1,
                            const gf_keypoint* d_kps2, int cap2, const int32_t* d_n2, const int32_t* d_matches12,
                            gf_rng* d_rng, gf_init_result* d_result, float* d_p3d, uint8_t* d_triangulated,
                            void* stream) {
    GF_CHECK(ctx && K, GF_ERR_ARG, "gf_initialize_batch_dev: null arg");
    if (nprob <= 0) return GF_OK;
    GF_CHECK(d_kps1 && d_kps2 && d_n1 && d_n2 && d_matches12 && d_rng && d_result && d_p3d && d_triangulated,
             GF_ERR_ARG, "gf_initialize_batch_dev: null buffer");
    GF_CHECK(cap1 > 0 && cap2 > 0 && nprob <= 65535, GF_ERR_ARG, "gf_initialize_batch_dev: bad caps or batch");
    return init_launch(ctx, nprob, K, sigma, iterations, min_triangulated, d_kps1, cap1, cap1, d_n1, d_kps2, cap2,
                       cap2, d_n2, d_matches12, d_rng, d_result, d_p3d, d_triangulated, stream);
}

int gf_initialize(gf_ctx* ctx, const float K[9], float sigma, int iterations, int min_triangulated,
                  const gf_keypoint* kps1, int n1, const gf_keypoint* kps2, int n2, const int32_t* matches12,
                  gf_rng* rng, gf_init_result* result, float* p3d, uint8_t* triangulated) {
    GF_CHECK(ctx && K && kps1 && kps2 && matches12 && rng && result && p3d && triangulated, GF_ERR_ARG,
             "gf_initialize: null arg");
    GF_CHECK(n1 > 0 && n2 > 0, GF_ERR_ARG, "gf_initialize: empty frame");
    int N = 0;
    for (int i = 0; i < n1; i++) {
        GF_CHECK(matches12[i] < n2, GF_ERR_ARG, "gf_initialize: match index out of range");
        N += matches12[i] >= 0;
    }
    GF_CHECK(N >= 8, GF_ERR_ARG, "gf_initialize: fewer than 8 matches");
    GF_HIP(hipSetDevice(ctx->device));
    void *d1, *d2, *dm, *dr, *dres, *dp, *dt;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, kps1, sizeof(gf_keypoint) * (size_t)n1, &d1)) ||
        (rc = gf::ws_upload(ctx, 1, kps2, sizeof(gf_keypoint) * (size_t)n2, &d2)) ||
        (rc = gf::ws_upload(ctx, 2, matches12, sizeof(int32_t) * (size_t)n1, &dm)) ||
        (rc = gf::ws_upload(ctx, 3, rng, sizeof(gf_rng), &dr)) ||
        (rc = gf::ws_get(ctx, 4, sizeof(gf_init_result), &dres)) ||
        (rc = gf::ws_get(ctx, 5, sizeof(float) * 3 * (size_t)n1, &dp)) || (rc = gf::ws_get(ctx, 6, (size_t)n1, &dt)))
        return rc;
    rc = gf_initialize_dev(ctx, K, sigma, iterations, min_triangulated, (const gf_keypoint*)d1, n1,
                           (const gf_keypoint*)d2, n2, (const int32_t*)dm, (gf_rng*)dr, (gf_init_result*)dres,
                           (float*)dp, (uint8_t*)dt, ctx->stream);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    GF_HIP(hipMemcpyAsync(result, dres, sizeof(gf_init_result), hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(rng, dr, sizeof(gf_rng), hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(p3d, dp, sizeof(float) * 3 * (size_t)n1, hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(triangulated, dt, (size_t)n1, hipMemcpyDeviceToHost, s));
    GF_HIP(hipStreamSynchronize(s));
    return GF_OK;
}

}  // extern "C"
