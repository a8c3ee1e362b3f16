// CPU ORACLE (test infrastructure) — SURVEY.md §8(f) rank 4: the monocular
// map initialiser ORB_SLAM::Initializer (src/Initializer.cc). Restated from
// the reference text:
//   Initialize :44-132 (8-point sets from DUtils::Random::RandomInt, H and F
//   searches, RH = SH / (SH + SF) > 0.40 picks the homography),
//   FindHomography :241-289, FindFundamental :292-340, ComputeH21 :343-383,
//   ComputeF21 :385-421, CheckHomography :423-506, CheckFundamental :508-586,
//   ReconstructF :588-688, ReconstructH :690-856, Triangulate :858-871,
//   Normalize :873-919, CheckRT :922-1040, DecomposeE :1042-1062;
//   minTriangulated = THRES_INIT_MPT_NUM / 2 = 50 (include/Initializer.h).
// The reference's quirks are kept: FindFundamental sizes its result from the
// (empty) output vector, so an F search that never beats a score of 0 yields
// no inliers (the reference then reads past the empty vector; here they are
// all false); RandomInt = int(rand() / (RAND_MAX + 1.0) * (max - min + 1)) + min.
// OpenCV is not vendored: cv::SVD of CV_32F matrices is
// restated from OpenCV 3.4 lapack.cpp (JacobiSVDImpl_<float>: float
// rotations, double accumulators, eps = 2 FLT_EPSILON, the cv::RNG(0x12345678)
// completion of null left vectors — which is where ComputeF21's null vector
// comes from, the 8 x 9 system being transposed first), the 3x3 CV_32F
// inverse and determinant in double, small float products as
// docs/ORACLE_ASSUMPTIONS.md A1, MatExpr scalings as a double multiply rounded
// to float (A17). Parity unpinned against OpenCV itself.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_common.h"

namespace orc_init {

struct CvRng {  // cv::RNG, multiply-with-carry (CV_RNG_COEFF 4164903690)
    uint64_t state;
    unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690ULL + (unsigned)(state >> 32);
        return (unsigned)state;
    }
};

// JacobiSVDImpl_<float>(At, W, Vt, m, n, n1): At holds n rows of length m
// (plus n1 - n more rows when n1 > n); on return rows 0..n1-1 of At are the
// left singular vectors, W the singular values, Vt the right ones as rows.
static void jacobi_svd_f(float* At, float* Wout, float* Vt, int m, int n, int n1) {
    const double minval = FLT_MIN;
    const float eps = FLT_EPSILON * 2;
    std::vector<double> W(n);
    const int max_iter = std::max(m, 30);
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const float t = At[i * m + k];
            sd += (double)t * t;
        }
        W[i] = sd;
        for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
        Vt[i * n + i] = 1;
    }
    for (int iter = 0; iter < max_iter; iter++) {
        bool changed = false;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                float *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += (double)Ai[k] * Aj[k];
                if (std::fabs(p) <= eps * std::sqrt((double)a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = std::sqrt(p * p + beta * beta);
                float c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = (float)std::sqrt(delta / gamma);
                    c = (float)(p / (gamma * s * 2));
                } else {
                    c = (float)std::sqrt((gamma + beta) / (gamma * 2));
                    s = (float)(p / (gamma * c * 2));
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    const float t0 = c * Ai[k] + s * Aj[k];
                    const float t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += (double)t0 * t0;
                    b += (double)t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                float *Vi = Vt + i * n, *Vj = Vt + j * n;
                for (int k = 0; k < n; k++) {
                    const float t0 = c * Vi[k] + s * Vj[k];
                    const float t1 = -s * Vi[k] + c * Vj[k];
                    Vi[k] = t0;
                    Vj[k] = t1;
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) {
            const float t = At[i * m + k];
            sd += (double)t * t;
        }
        W[i] = std::sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            std::swap(W[i], W[j]);
            for (int k = 0; k < m; k++) std::swap(At[i * m + k], At[j * m + k]);
            for (int k = 0; k < n; k++) std::swap(Vt[i * n + k], Vt[j * n + k]);
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = (float)W[i];
    CvRng rng{0x12345678};
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            const float val0 = (float)(1. / m);
            for (int k = 0; k < m; k++) At[i * m + k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];  // float product
                    float asum = 0;
                    for (int k = 0; k < m; k++) {
                        const float t = (float)(At[i * m + k] - sd * At[j * m + k]);
                        At[i * m + k] = t;
                        asum += std::fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) {
                const float t = At[i * m + k];
                sd += (double)t * t;
            }
            sd = std::sqrt(sd);
        }
        const float s = (float)(sd > minval ? 1 / sd : 0.);
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

// cv::SVD::compute(A r x c, w, u, vt, FULL_UV) of a CV_32F matrix: w (min),
// u (r x r, row-major), vt (c x c, row-major).
static void svd_full(const float* A, int r, int c, float* w, float* u, float* vt) {
    const bool at = r < c;
    const int m = at ? c : r, n = at ? r : c;  // JacobiSVD sizes, m >= n
    std::vector<float> Ta((size_t)m * m, 0.f), V((size_t)n * n), W(n);
    // temp_a (n x m): A^T when r >= c, A itself otherwise
    for (int i = 0; i < n; i++)
        for (int k = 0; k < m; k++) Ta[(size_t)i * m + k] = at ? A[i * c + k] : A[k * c + i];
    jacobi_svd_f(Ta.data(), W.data(), V.data(), m, n, m);
    for (int i = 0; i < n; i++) w[i] = W[i];
    if (!at) {  // u = temp_u^T (r x r), vt = temp_v (c x c)
        for (int i = 0; i < r; i++)
            for (int j = 0; j < r; j++) u[i * r + j] = Ta[(size_t)j * m + i];
        for (int i = 0; i < c * c; i++) vt[i] = V[i];
    } else {  // u = temp_v^T (r x r), vt = temp_u (c x c)
        for (int i = 0; i < r; i++)
            for (int j = 0; j < r; j++) u[i * r + j] = V[(size_t)j * n + i];
        for (int i = 0; i < c * c; i++) vt[i] = Ta[i];
    }
}

// small float products (A1): D = alpha * (A B), a*b in float summed left to right
static void gemm(const float* A, const float* B, float* D, int r, int k, int c, double alpha = 1.0) {
    std::vector<float> out((size_t)r * c);
    for (int i = 0; i < r; i++)
        for (int j = 0; j < c; j++) {
            float s = A[i * k] * B[j];
            for (int q = 1; q < k; q++) s = s + A[i * k + q] * B[q * c + j];
            out[(size_t)i * c + j] = alpha == 1.0 ? s : (float)((double)s * alpha);
        }
    std::copy(out.begin(), out.end(), D);
}

static void transpose3(const float* A, float* T) {
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) T[j * 3 + i] = A[i * 3 + j];
}

static double det3(const float* m) {
    return m[0] * ((double)m[4] * m[8] - (double)m[5] * m[7]) - m[1] * ((double)m[3] * m[8] - (double)m[5] * m[6]) +
           m[2] * ((double)m[3] * m[7] - (double)m[4] * m[6]);
}

// cv::Mat::inv() of a 3x3 CV_32F (DECOMP_LU closed form in double; zeros when singular)
static void inv3(const float* S, float* D) {
    double d = det3(S);
    if (d == 0.) {
        for (int i = 0; i < 9; i++) D[i] = 0.f;
        return;
    }
    d = 1. / d;
    const double t[9] = {((double)S[4] * S[8] - (double)S[5] * S[7]) * d, ((double)S[2] * S[7] - (double)S[1] * S[8]) * d,
                         ((double)S[1] * S[5] - (double)S[2] * S[4]) * d, ((double)S[5] * S[6] - (double)S[3] * S[8]) * d,
                         ((double)S[0] * S[8] - (double)S[2] * S[6]) * d, ((double)S[2] * S[3] - (double)S[0] * S[5]) * d,
                         ((double)S[3] * S[7] - (double)S[4] * S[6]) * d, ((double)S[1] * S[6] - (double)S[0] * S[7]) * d,
                         ((double)S[0] * S[4] - (double)S[1] * S[3]) * d};
    for (int i = 0; i < 9; i++) D[i] = (float)t[i];
}

// cv::norm(v, NORM_L2) of a float vector (normL2_32f): squares summed in double
static double norm3(const float* v) {
    double s = 0;
    for (int i = 0; i < 3; i++) s += (double)v[i] * (double)v[i];
    return std::sqrt(s);
}

// MatExpr scaling (Mat / s, Mat *= s): convertTo with the factor cast to float
static void scale3(const float* v, double alpha, float* out) {
    const float a = (float)alpha;
    for (int i = 0; i < 3; i++) out[i] = v[i] * a;
}

struct Rand {  // glibc random_r TYPE_3 continued from a gf_rng (the process-wide std::rand())
    struct random_data rd;
    char state[128];
    explicit Rand(const gf_rng& g) {
        std::memset(&rd, 0, sizeof(rd));
        initstate_r(1, state, sizeof(state), &rd);
        for (int i = 0; i < 31; i++) rd.state[i] = g.state[i];
        rd.fptr = rd.state + g.f;
        rd.rptr = rd.state + g.r;
    }
    void save(gf_rng& g) const {
        for (int i = 0; i < 31; i++) g.state[i] = rd.state[i];
        g.f = (int32_t)(rd.fptr - rd.state);
        g.r = (int32_t)(rd.rptr - rd.state);
    }
    int random_int(int mn, int mx) {  // DUtils::Random::RandomInt (Random.cpp:47-50)
        int32_t r;
        random_r(&rd, &r);
        const int d = mx - mn + 1;
        return int(((double)r / ((double)RAND_MAX + 1.0)) * d) + mn;
    }
};

struct Pt {
    float x, y;
};

// Initializer::Normalize (:873-919)
static void normalize(const gf_keypoint* K, int n, std::vector<Pt>& P, float* T) {
    float meanX = 0, meanY = 0;
    for (int i = 0; i < n; i++) {
        meanX += K[i].x;
        meanY += K[i].y;
    }
    meanX = meanX / n;
    meanY = meanY / n;
    P.resize(n);
    float devX = 0, devY = 0;
    for (int i = 0; i < n; i++) {
        P[i].x = K[i].x - meanX;
        P[i].y = K[i].y - meanY;
        devX += std::fabs(P[i].x);
        devY += std::fabs(P[i].y);
    }
    devX = devX / n;
    devY = devY / n;
    const float sX = (float)(1.0 / devX), sY = (float)(1.0 / devY);
    for (int i = 0; i < n; i++) {
        P[i].x = P[i].x * sX;
        P[i].y = P[i].y * sY;
    }
    const float T0[9] = {sX, 0, -meanX * sX, 0, sY, -meanY * sY, 0, 0, 1};
    std::memcpy(T, T0, sizeof(T0));
}

static void compute_h21(const Pt* p1, const Pt* p2, float* H) {  // :343-383
    float A[16 * 9];
    for (int i = 0; i < 8; i++) {
        const float u1 = p1[i].x, v1 = p1[i].y, u2 = p2[i].x, v2 = p2[i].y;
        float* r0 = A + (2 * i) * 9;
        float* r1 = A + (2 * i + 1) * 9;
        r0[0] = 0, r0[1] = 0, r0[2] = 0, r0[3] = -u1, r0[4] = -v1, r0[5] = -1, r0[6] = v2 * u1, r0[7] = v2 * v1,
        r0[8] = v2;
        r1[0] = u1, r1[1] = v1, r1[2] = 1, r1[3] = 0, r1[4] = 0, r1[5] = 0, r1[6] = -u2 * u1, r1[7] = -u2 * v1,
        r1[8] = -u2;
    }
    float w[9], u[16 * 16], vt[81];
    svd_full(A, 16, 9, w, u, vt);
    for (int i = 0; i < 9; i++) H[i] = vt[8 * 9 + i];
}

static void compute_f21(const Pt* p1, const Pt* p2, float* F) {  // :385-421
    float A[8 * 9];
    for (int i = 0; i < 8; i++) {
        const float u1 = p1[i].x, v1 = p1[i].y, u2 = p2[i].x, v2 = p2[i].y;
        float* r = A + i * 9;
        r[0] = u2 * u1, r[1] = u2 * v1, r[2] = u2, r[3] = v2 * u1, r[4] = v2 * v1, r[5] = v2, r[6] = u1, r[7] = v1,
        r[8] = 1;
    }
    float w[9], u[64], vt[81];
    svd_full(A, 8, 9, w, u, vt);
    float Fpre[9], w3[3], u3[9], vt3[9];
    for (int i = 0; i < 9; i++) Fpre[i] = vt[8 * 9 + i];
    svd_full(Fpre, 3, 3, w3, u3, vt3);
    w3[2] = 0;
    const float D[9] = {w3[0], 0, 0, 0, w3[1], 0, 0, 0, w3[2]};
    float UD[9];
    gemm(u3, D, UD, 3, 3, 3);
    gemm(UD, vt3, F, 3, 3, 3);
}

// CheckHomography (:423-506): per-match chi-square terms, sequential score
static float check_h(const float* H21, const float* H12, const gf_keypoint* K1, const gf_keypoint* K2,
                     const std::vector<std::pair<int, int>>& M, std::vector<char>& in, float sigma) {
    const float th = 5.991f, invS2 = (float)(1.0 / (sigma * sigma));
    float score = 0;
    in.assign(M.size(), 0);
    for (size_t i = 0; i < M.size(); i++) {
        bool bIn = true;
        const float u1 = K1[M[i].first].x, v1 = K1[M[i].first].y, u2 = K2[M[i].second].x, v2 = K2[M[i].second].y;
        const float w2in1inv = (float)(1.0 / (H12[6] * u2 + H12[7] * v2 + H12[8]));
        const float u2in1 = (H12[0] * u2 + H12[1] * v2 + H12[2]) * w2in1inv;
        const float v2in1 = (H12[3] * u2 + H12[4] * v2 + H12[5]) * w2in1inv;
        const float sq1 = (u1 - u2in1) * (u1 - u2in1) + (v1 - v2in1) * (v1 - v2in1);
        const float c1 = sq1 * invS2;
        if (c1 > th)
            bIn = false;
        else
            score += th - c1;
        const float w1in2inv = (float)(1.0 / (H21[6] * u1 + H21[7] * v1 + H21[8]));
        const float u1in2 = (H21[0] * u1 + H21[1] * v1 + H21[2]) * w1in2inv;
        const float v1in2 = (H21[3] * u1 + H21[4] * v1 + H21[5]) * w1in2inv;
        const float sq2 = (u2 - u1in2) * (u2 - u1in2) + (v2 - v1in2) * (v2 - v1in2);
        const float c2 = sq2 * invS2;
        if (c2 > th)
            bIn = false;
        else
            score += th - c2;
        in[i] = bIn;
    }
    return score;
}

// CheckFundamental (:508-586)
static float check_f(const float* F, const gf_keypoint* K1, const gf_keypoint* K2,
                     const std::vector<std::pair<int, int>>& M, std::vector<char>& in, float sigma) {
    const float th = 3.841f, thScore = 5.991f, invS2 = (float)(1.0 / (sigma * sigma));
    float score = 0;
    in.assign(M.size(), 0);
    for (size_t i = 0; i < M.size(); i++) {
        bool bIn = true;
        const float u1 = K1[M[i].first].x, v1 = K1[M[i].first].y, u2 = K2[M[i].second].x, v2 = K2[M[i].second].y;
        const float a2 = F[0] * u1 + F[1] * v1 + F[2], b2 = F[3] * u1 + F[4] * v1 + F[5],
                    c2 = F[6] * u1 + F[7] * v1 + F[8];
        const float num2 = a2 * u2 + b2 * v2 + c2;
        const float sq1 = num2 * num2 / (a2 * a2 + b2 * b2);
        const float ch1 = sq1 * invS2;
        if (ch1 > th)
            bIn = false;
        else
            score += thScore - ch1;
        const float a1 = F[0] * u2 + F[3] * v2 + F[6], b1 = F[1] * u2 + F[4] * v2 + F[7],
                    c1 = F[2] * u2 + F[5] * v2 + F[8];
        const float num1 = a1 * u1 + b1 * v1 + c1;
        const float sq2 = num1 * num1 / (a1 * a1 + b1 * b1);
        const float ch2 = sq2 * invS2;
        if (ch2 > th)
            bIn = false;
        else
            score += thScore - ch2;
        in[i] = bIn;
    }
    return score;
}

// Triangulate (:858-871)
static void triangulate(const gf_keypoint& k1, const gf_keypoint& k2, const float* P1, const float* P2, float* x3) {
    // x * P.row(2) - P.row(0): addWeighted(P.row(2), x, P.row(0), -1, 0) in double
    auto row = [](float x, const float* P, int r, float* out) {
        for (int c = 0; c < 4; c++) out[c] = (float)((double)P[8 + c] * (double)x + (double)P[4 * r + c] * -1.0 + 0.0);
    };
    float A[16];
    row(k1.x, P1, 0, A);
    row(k1.y, P1, 1, A + 4);
    row(k2.x, P2, 0, A + 8);
    row(k2.y, P2, 1, A + 12);
    float w[4], u[16], vt[16];
    svd_full(A, 4, 4, w, u, vt);
    scale3(vt + 12, 1.0 / (double)vt[15], x3);
}

// CheckRT (:922-1040)
static int check_rt(const float* R, const float* t, const gf_keypoint* K1, const gf_keypoint* K2,
                    const std::vector<std::pair<int, int>>& M, const std::vector<char>& inl, const float* K, int n1,
                    std::vector<float>& P3D, std::vector<char>& good, float th2, float& parallax) {
    const float fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    good.assign(n1, 0);
    P3D.assign(3 * (size_t)n1, 0.f);
    std::vector<float> cosp;
    float P1[12] = {K[0], K[1], K[2], 0, K[3], K[4], K[5], 0, K[6], K[7], K[8], 0};
    float Rt[12] = {R[0], R[1], R[2], t[0], R[3], R[4], R[5], t[1], R[6], R[7], R[8], t[2]};
    float P2[12];
    gemm(K, Rt, P2, 3, 3, 4);
    float RT[9], O2[3];
    transpose3(R, RT);
    gemm(RT, t, O2, 3, 3, 1, -1.0);
    int nGood = 0;
    for (size_t i = 0; i < M.size(); i++) {
        if (i >= inl.size() || !inl[i]) continue;
        const gf_keypoint& kp1 = K1[M[i].first];
        const gf_keypoint& kp2 = K2[M[i].second];
        float p[3];
        triangulate(kp1, kp2, P1, P2, p);
        if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) {
            good[M[i].first] = 0;
            continue;
        }
        const float n1v[3] = {p[0] - 0.f, p[1] - 0.f, p[2] - 0.f};  // p3dC1 - O1
        const float dist1 = (float)norm3(n1v);
        const float n2v[3] = {p[0] - O2[0], p[1] - O2[1], p[2] - O2[2]};
        const float dist2 = (float)norm3(n2v);
        // Mat::dot (dotProd_32f): products and sum in double
        double dot = 0;
        for (int r = 0; r < 3; r++) dot += (double)n1v[r] * (double)n2v[r];
        const float cosParallax = (float)(dot / (double)(dist1 * dist2));
        if (p[2] <= 0 && (double)cosParallax < 0.99998) continue;
        float p2[3];
        for (int r = 0; r < 3; r++) p2[r] = orc::dot3p(R[3 * r], p[0], R[3 * r + 1], p[1], R[3 * r + 2], p[2], t[r]);
        if (p2[2] <= 0 && (double)cosParallax < 0.99998) continue;
        const float invZ1 = (float)(1.0 / p[2]);
        const float im1x = fx * p[0] * invZ1 + cx, im1y = fy * p[1] * invZ1 + cy;
        const float e1 = (im1x - kp1.x) * (im1x - kp1.x) + (im1y - kp1.y) * (im1y - kp1.y);
        if (e1 > th2) continue;
        const float invZ2 = (float)(1.0 / p2[2]);
        const float im2x = fx * p2[0] * invZ2 + cx, im2y = fy * p2[1] * invZ2 + cy;
        const float e2 = (im2x - kp2.x) * (im2x - kp2.x) + (im2y - kp2.y) * (im2y - kp2.y);
        if (e2 > th2) continue;
        cosp.push_back(cosParallax);
        for (int r = 0; r < 3; r++) P3D[3 * (size_t)M[i].first + r] = p[r];
        nGood++;
        if ((double)cosParallax < 0.99998) good[M[i].first] = 1;
    }
    if (nGood > 0) {
        std::sort(cosp.begin(), cosp.end());
        const size_t idx = std::min(50, int(cosp.size() - 1));
        // acos(float) = acosf, taken as correctly rounded (A17)
        const float ac = (float)std::acos((double)cosp[idx]);
        parallax = (float)((double)(ac * 180.f) / M_PI);
    } else {
        parallax = 0;
    }
    return nGood;
}

static void decompose_e(const float* E, float* R1, float* R2, float* t) {  // :1042-1062
    float w[3], u[9], vt[9];
    svd_full(E, 3, 3, w, u, vt);
    const float tt[3] = {u[2], u[5], u[8]};
    scale3(tt, 1.0 / norm3(tt), t);
    const float W[9] = {0, -1, 0, 1, 0, 0, 0, 0, 1};
    float WT[9], UW[9];
    transpose3(W, WT);
    gemm(u, W, UW, 3, 3, 3);
    gemm(UW, vt, R1, 3, 3, 3);
    if (det3(R1) < 0)
        for (int i = 0; i < 9; i++) R1[i] = -R1[i];
    gemm(u, WT, UW, 3, 3, 3);
    gemm(UW, vt, R2, 3, 3, 3);
    if (det3(R2) < 0)
        for (int i = 0; i < 9; i++) R2[i] = -R2[i];
}

}  // namespace orc_init

using namespace orc_init;

// Initializer(ReferenceFrame, sigma, iterations).Initialize(CurrentFrame, vMatches12, ...)
extern "C" int orc_initialize(const float* K, float sigma, int iterations, int min_triangulated,
                              const gf_keypoint* kps1, int n1, const gf_keypoint* kps2, int n2,
                              const int32_t* matches12, gf_rng* rng, gf_init_result* res, float* p3d,
                              uint8_t* triangulated) {
    std::memset(res, 0, sizeof(*res));
    res->best = res->iter_H = res->iter_F = -1;
    res->model = -1;
    if (n1 > 0) {
        std::memset(p3d, 0, sizeof(float) * 3 * (size_t)n1);
        std::memset(triangulated, 0, (size_t)n1);
    }
    std::vector<std::pair<int, int>> M;
    for (int i = 0; i < n1; i++)
        if (matches12[i] >= 0) M.emplace_back(i, matches12[i]);
    const int N = (int)M.size();
    res->nmatches = N;
    if (N < 8 || iterations <= 0) return GF_ERR_ARG;  // the reference needs 8 distinct matches per set
    // 8-point sets (:80-95)
    std::vector<int> sets((size_t)iterations * 8);
    std::vector<int> all(N), avail;
    for (int i = 0; i < N; i++) all[i] = i;
    Rand R(*rng);
    for (int it = 0; it < iterations; it++) {
        avail = all;
        for (int j = 0; j < 8; j++) {
            const int randi = R.random_int(0, (int)avail.size() - 1);
            const int idx = avail[randi];
            sets[(size_t)it * 8 + j] = idx;
            avail[randi] = avail.back();
            avail.pop_back();
        }
    }
    R.save(*rng);
    std::vector<Pt> Pn1, Pn2;
    float T1[9], T2[9];
    normalize(kps1, n1, Pn1, T1);
    normalize(kps2, n2, Pn2, T2);
    // FindHomography (:241-289)
    float T2inv[9];
    inv3(T2, T2inv);
    float SH = 0, H21[9] = {0};
    std::vector<char> inH, cur;
    for (int it = 0; it < iterations; it++) {
        Pt a[8], b[8];
        for (int j = 0; j < 8; j++) {
            a[j] = Pn1[M[sets[(size_t)it * 8 + j]].first];
            b[j] = Pn2[M[sets[(size_t)it * 8 + j]].second];
        }
        float Hn[9], tmp[9], H21i[9], H12i[9];
        compute_h21(a, b, Hn);
        gemm(T2inv, Hn, tmp, 3, 3, 3);
        gemm(tmp, T1, H21i, 3, 3, 3);
        inv3(H21i, H12i);
        const float sc = check_h(H21i, H12i, kps1, kps2, M, cur, sigma);
        if (sc > SH) {
            std::memcpy(H21, H21i, sizeof(H21));
            inH = cur;
            SH = sc;
            res->iter_H = it;
        }
    }
    // FindFundamental (:292-340; N taken from the empty output vector, :295)
    float T2t[9];
    transpose3(T2, T2t);
    float SF = 0, F21[9] = {0};
    std::vector<char> inF;
    for (int it = 0; it < iterations; it++) {
        Pt a[8], b[8];
        for (int j = 0; j < 8; j++) {
            a[j] = Pn1[M[sets[(size_t)it * 8 + j]].first];
            b[j] = Pn2[M[sets[(size_t)it * 8 + j]].second];
        }
        float Fn[9], tmp[9], F21i[9];
        compute_f21(a, b, Fn);
        gemm(T2t, Fn, tmp, 3, 3, 3);
        gemm(tmp, T1, F21i, 3, 3, 3);
        const float sc = check_f(F21i, kps1, kps2, M, cur, sigma);
        if (sc > SF) {
            std::memcpy(F21, F21i, sizeof(F21));
            inF = cur;
            SF = sc;
            res->iter_F = it;
        }
    }
    std::memcpy(res->H21, H21, sizeof(H21));
    std::memcpy(res->F21, F21, sizeof(F21));
    res->SH = SH;
    res->SF = SF;
    for (char c : inH) res->ninliers_H += c;
    for (char c : inF) res->ninliers_F += c;
    // both searches without a positive score: the reference divides 0/0 and
    // reconstructs from an empty cv::Mat (an OpenCV assertion); reported as no
    // model, RH = 0, here
    if (SH == 0.f && SF == 0.f) return GF_OK;
    const float RH = SH / (SH + SF);
    res->RH = RH;
    const float th2 = 4.0f * (sigma * sigma);
    std::vector<float> P3D;
    std::vector<char> good;
    const float minParallax = 1.0f;
    if ((double)RH > 0.40) {  // ReconstructH (:690-856)
        res->model = 0;
        int Nin = 0;
        for (char c : inH) Nin += c;
        float invK[9], tmp[9], A[9];
        inv3(K, invK);
        gemm(invK, H21, tmp, 3, 3, 3);
        gemm(tmp, K, A, 3, 3, 3);
        float w[3], U[9], Vt[9], V[9];
        svd_full(A, 3, 3, w, U, Vt);
        transpose3(Vt, V);
        const float s = (float)(det3(U) * det3(Vt));
        const float d1 = w[0], d2 = w[1], d3 = w[2];
        if ((double)(d1 / d2) < 1.00001 || (double)(d2 / d3) < 1.00001) return GF_OK;
        float vR[8][9], vt[8][3];
        const float aux1 = std::sqrt((d1 * d1 - d2 * d2) / (d1 * d1 - d3 * d3));
        const float aux3 = std::sqrt((d2 * d2 - d3 * d3) / (d1 * d1 - d3 * d3));
        const float x1[] = {aux1, aux1, -aux1, -aux1}, x3[] = {aux3, -aux3, aux3, -aux3};
        const float aux_stheta = std::sqrt((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 + d3) * d2);
        const float ctheta = (d2 * d2 + d1 * d3) / ((d1 + d3) * d2);
        const float stheta[] = {aux_stheta, -aux_stheta, -aux_stheta, aux_stheta};
        const float aux_sphi = std::sqrt((d1 * d1 - d2 * d2) * (d2 * d2 - d3 * d3)) / ((d1 - d3) * d2);
        const float cphi = (d1 * d3 - d2 * d2) / ((d1 - d3) * d2);
        const float sphi[] = {aux_sphi, -aux_sphi, -aux_sphi, aux_sphi};
        for (int i = 0; i < 8; i++) {
            const bool second = i >= 4;
            const int q = i & 3;
            float Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
            if (!second) {
                Rp[0] = ctheta, Rp[2] = -stheta[q], Rp[6] = stheta[q], Rp[8] = ctheta;
            } else {
                Rp[0] = cphi, Rp[2] = sphi[q], Rp[4] = -1, Rp[6] = sphi[q], Rp[8] = -cphi;
            }
            float URp[9];
            gemm(U, Rp, URp, 3, 3, 3, (double)s);  // s*U*Rp*Vt: (s U Rp) then Vt
            gemm(URp, Vt, vR[i], 3, 3, 3);
            float tp[3] = {x1[q], 0, second ? x3[q] : -x3[q]};
            const float sc = second ? d1 + d3 : d1 - d3;
            for (int r = 0; r < 3; r++) tp[r] = (float)((double)tp[r] * (double)sc);
            float tt[3];
            gemm(U, tp, tt, 3, 3, 1);
            scale3(tt, 1.0 / norm3(tt), vt[i]);
        }
        int bestGood = 0, secondBestGood = 0, best = -1;
        float bestParallax = -1;
        std::vector<float> bestP3D;
        std::vector<char> bestTri;
        for (int i = 0; i < 8; i++) {
            float parallaxi;
            const int nGood = check_rt(vR[i], vt[i], kps1, kps2, M, inH, K, n1, P3D, good, th2, parallaxi);
            res->ngood[i] = nGood;
            if (nGood > bestGood) {
                secondBestGood = bestGood;
                bestGood = nGood;
                best = i;
                bestParallax = parallaxi;
                bestP3D = P3D;
                bestTri = good;
            } else if (nGood > secondBestGood) {
                secondBestGood = nGood;
            }
        }
        res->parallax = bestParallax;
        res->best = best;
        if (secondBestGood < 0.75 * bestGood && bestParallax >= minParallax && bestGood > min_triangulated &&
            bestGood > 0.9 * Nin) {
            std::memcpy(res->R21, vR[best], sizeof(res->R21));
            std::memcpy(res->t21, vt[best], sizeof(res->t21));
            for (int i = 0; i < 3 * n1; i++) p3d[i] = bestP3D[i];
            for (int i = 0; i < n1; i++) triangulated[i] = bestTri[i];
            res->ok = 1;
        }
        return GF_OK;
    }
    // ReconstructF (:588-688)
    res->model = 1;
    int Nin = 0;
    for (char c : inF) Nin += c;
    float KT[9], tmp[9], E21[9];
    transpose3(K, KT);
    gemm(KT, F21, tmp, 3, 3, 3);
    gemm(tmp, K, E21, 3, 3, 3);
    float R1[9], R2[9], t[3], tn[3];
    decompose_e(E21, R1, R2, t);
    for (int r = 0; r < 3; r++) tn[r] = -t[r];
    const float* Rs[4] = {R1, R2, R1, R2};
    const float* ts[4] = {t, t, tn, tn};
    int nGood[4];
    float par[4];
    std::vector<float> P[4];
    std::vector<char> G[4];
    for (int i = 0; i < 4; i++) {
        nGood[i] = check_rt(Rs[i], ts[i], kps1, kps2, M, inF, K, n1, P[i], G[i], th2, par[i]);
        res->ngood[i] = nGood[i];
    }
    const int maxGood = std::max(nGood[0], std::max(nGood[1], std::max(nGood[2], nGood[3])));
    const int nMinGood = std::max(static_cast<int>(0.9 * Nin), min_triangulated);
    int nsimilar = 0;
    for (int i = 0; i < 4; i++)
        if (nGood[i] > 0.7 * maxGood) nsimilar++;
    int b = 0;  // the if / else-if chain on maxGood == nGood_i (:641-685)
    while (nGood[b] != maxGood) b++;
    res->best = b;
    res->parallax = par[b];
    if (maxGood < nMinGood || nsimilar > 1) return GF_OK;
    if (par[b] > minParallax) {
        std::memcpy(res->R21, Rs[b], sizeof(res->R21));
        std::memcpy(res->t21, ts[b], sizeof(res->t21));
        for (int k = 0; k < 3 * n1; k++) p3d[k] = P[b][k];
        for (int k = 0; k < n1; k++) triangulated[k] = G[b][k];
        res->ok = 1;
    }
    return GF_OK;
}
