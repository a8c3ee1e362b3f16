// CPU ORACLE (test infrastructure) — ORB extraction, SURVEY.md §8a rows E1-E7.
// Restates ORB_SLAM::ORBextractor (src/ORBextractor.cc) together with the
// OpenCV 3.4 internals it calls (FAST, KeyPointsFilter::retainBest, resize,
// GaussianBlur, fastAtan2) as documented in DESIGN.md "Oracle assumptions".
#include <algorithm>
#include <climits>
#include <cfloat>
#include <cstring>
#include <vector>

#include "oracle_common.h"
#include "../gf_orb_slam_amd/csrc/orb_pattern.h"

namespace orc {

static const int kPatchSize = 31;      // ORBextractor.cc:82
static const int kHalfPatch = 15;      // ORBextractor.cc:83
static const int kEdgeThreshold = 16;  // ORBextractor.cc:84

struct KP {  // cv::KeyPoint
    float x, y, size, angle, response;
    int octave, class_id;
};

struct ExtractorPlan {
    int nfeatures, nlevels, fastTh, minTh = 7;
    int scoreType = 1;  // ORB::HARRIS_SCORE 0, ORB::FAST_SCORE 1 (ORBextractor.h:57)
    double scaleFactor;  // ORBextractor.h:79 stores it as double
    std::vector<float> scale, invScale;
    std::vector<int> featPerLevel;
    int umax[kHalfPatch + 1];

    // ORBextractor::ORBextractor, ORBextractor.cc:464-524
    ExtractorPlan(int nf, float sf, int nl, int th) : nfeatures(nf), nlevels(nl), fastTh(th), scaleFactor(sf) {
        scale.resize(nl);
        invScale.resize(nl);
        scale[0] = 1.f;
        for (int i = 1; i < nl; i++) scale[i] = (float)((double)scale[i - 1] * scaleFactor);
        float inv = (float)(1.0f / scaleFactor);
        invScale[0] = 1.f;
        for (int i = 1; i < nl; i++) invScale[i] = invScale[i - 1] * inv;

        featPerLevel.resize(nl);
        float factor = (float)(1.0 / scaleFactor);
        float nd = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
        int sum = 0;
        for (int l = 0; l < nl - 1; l++) {
            featPerLevel[l] = cv_round(nd);
            sum += featPerLevel[l];
            nd *= factor;
        }
        featPerLevel[nl - 1] = std::max(nfeatures - sum, 0);

        int vmax = cv_floor(kHalfPatch * std::sqrt(2.f) / 2 + 1);
        int vmin = cv_ceil(kHalfPatch * std::sqrt(2.f) / 2);
        const double hp2 = kHalfPatch * kHalfPatch;
        for (int v = 0; v <= vmax; ++v) umax[v] = cv_round(std::sqrt(hp2 - v * v));
        for (int v = kHalfPatch, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
    }
};

// ---------------------------------------------------------------- E2 resize
// cv::resize(INTER_LINEAR) on CV_8U: 11-bit fixed-point coefficients,
// HResizeLinear (int row sums) + VResizeLinear with the
// ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2) >> 2 cast.
static Image resize_linear(const Image& src, int dw, int dh) {
    Image dst;
    dst.w = dw;
    dst.h = dh;
    dst.px.resize((size_t)dw * dh);
    const int ONE = 2048;
    double scale_x = 1. / ((double)dw / src.w), scale_y = 1. / ((double)dh / src.h);
    std::vector<int> xofs(dw), yofs(dh);
    std::vector<short> ialpha(2 * dw), ibeta(2 * dh);
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx >= src.w - 1) fx = 0, sx = src.w - 1;
        xofs[dx] = sx;
        ialpha[2 * dx] = (short)cv_round((1.f - fx) * ONE);
        ialpha[2 * dx + 1] = (short)cv_round(fx * ONE);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        yofs[dy] = sy;
        ibeta[2 * dy] = (short)cv_round((1.f - fy) * ONE);
        ibeta[2 * dy + 1] = (short)cv_round(fy * ONE);
    }
    std::vector<int> r0(dw), r1(dw);
    auto hrow = [&](int sy, std::vector<int>& out) {
        sy = std::min(std::max(sy, 0), src.h - 1);
        const uint8_t* S = &src.px[(size_t)sy * src.w];
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (sx + 1 < src.w)
                out[dx] = S[sx] * ialpha[2 * dx] + S[sx + 1] * ialpha[2 * dx + 1];
            else
                out[dx] = S[sx] * ONE;
        }
    };
    int c0 = INT_MIN, c1 = INT_MIN;  // source rows held in r0 / r1
    for (int dy = 0; dy < dh; dy++) {
        const int s0 = std::min(std::max(yofs[dy], 0), src.h - 1), s1 = std::min(std::max(yofs[dy] + 1, 0), src.h - 1);
        if (s0 == c1) {
            std::swap(r0, r1);
            std::swap(c0, c1);
        }
        if (s0 != c0) hrow(s0, r0), c0 = s0;
        if (s1 != c1) hrow(s1, r1), c1 = s1;
        int b0 = ibeta[2 * dy], b1 = ibeta[2 * dy + 1];
        uint8_t* D = &dst.px[(size_t)dy * dw];
        for (int dx = 0; dx < dw; dx++) {
            int v = (((b0 * (r0[dx] >> 4)) >> 16) + ((b1 * (r1[dx] >> 4)) >> 16) + 2) >> 2;
            D[dx] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
    return dst;
}

// ---------------------------------------------------------------- E5 blur
// GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on CV_8U: integer kernel
// round(k*256) from getGaussianKernel(7, 2, CV_32F), int row pass, column pass
// cast (sum + 2^15) >> 16 (OpenCV 3.4.1 FixedPtCastEx, bits = 16).
void gauss_kernel7(int k[7]) {
    float cf[7];
    double sum = 0, scale2X = -0.5 / (2.0 * 2.0);
    for (int i = 0; i < 7; i++) {
        double x = i - 3.0;
        cf[i] = (float)std::exp(scale2X * x * x);
        sum += cf[i];
    }
    sum = 1. / sum;
    for (int i = 0; i < 7; i++) {
        cf[i] = (float)(cf[i] * sum);
        k[i] = cv_round((double)cf[i] * 256.0);
    }
}

static Image gaussian_blur(const Image& src) {
    int k[7];
    gauss_kernel7(k);
    Image dst = src;
    const int w = src.w, h = src.h;
    std::vector<int> rows((size_t)w * h);
    for (int y = 0; y < h; y++) {
        const uint8_t* S = &src.px[(size_t)y * w];
        int* R = &rows[(size_t)y * w];
        for (int x = 0; x < w; x++) {
            if (x == 3 && w > 6) {  // interior: no border arithmetic
                const int k0 = k[0], k1 = k[1], k2 = k[2], k3 = k[3], k4 = k[4], k5 = k[5], k6 = k[6];
                for (; x + 3 < w; x++)
                    R[x] = k0 * S[x - 3] + k1 * S[x - 2] + k2 * S[x - 1] + k3 * S[x] + k4 * S[x + 1] + k5 * S[x + 2] +
                           k6 * S[x + 3];
                if (x >= w) break;
            }
            int s = 0;
            for (int i = 0; i < 7; i++) s += k[i] * S[reflect101(x + i - 3, w)];
            R[x] = s;
        }
    }
    for (int y = 0; y < h; y++) {
        const int* r[7];
        for (int i = 0; i < 7; i++) r[i] = &rows[(size_t)reflect101(y + i - 3, h) * w];
        uint8_t* D = &dst.px[(size_t)y * w];
        for (int x = 0; x < w; x++) {
            int s = 0;
            for (int i = 0; i < 7; i++) s += k[i] * r[i][x];
            int v = (s + (1 << 15)) >> 16;
            D[x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    }
    return dst;
}

// ---------------------------------------------------------------- E3 FAST
// OpenCV FAST_t<16> (TYPE_9_16) with cornerScore<16> and the 3-row strict
// non-maximum suppression, run on a ROI view (x0,y0,w,h) of a level.
static const int kCircle[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},  {3, 0},  {3, -1},
                                   {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                   {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

int fast_corner_score(const Image& im, int x, int y, int threshold) {
    int v = im.at(x, y);
    int d[25];
    for (int k = 0; k < 25; k++) d[k] = v - im.at(x + kCircle[k & 15][0], y + kCircle[k & 15][1]);
    int a0 = threshold;
    for (int k = 0; k < 16; k += 2) {
        int a = std::min(d[k + 1], d[k + 2]);
        a = std::min(a, d[k + 3]);
        if (a <= a0) continue;
        a = std::min(a, d[k + 4]);
        a = std::min(a, d[k + 5]);
        a = std::min(a, d[k + 6]);
        a = std::min(a, d[k + 7]);
        a = std::min(a, d[k + 8]);
        a0 = std::max(a0, std::min(a, d[k]));
        a0 = std::max(a0, std::min(a, d[k + 9]));
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = std::max(d[k + 1], d[k + 2]);
        b = std::max(b, d[k + 3]);
        b = std::max(b, d[k + 4]);
        b = std::max(b, d[k + 5]);
        if (b >= b0) continue;
        b = std::max(b, d[k + 6]);
        b = std::max(b, d[k + 7]);
        b = std::max(b, d[k + 8]);
        b0 = std::min(b0, std::max(b, d[k]));
        b0 = std::min(b0, std::max(b, d[k + 9]));
    }
    return -b0 - 1;
}

// 9-of-16 contiguous segment test (brighter or darker by more than th).
bool fast_is_corner(const Image& im, int x, int y, int th) {
    int v = im.at(x, y);
    int vt_lo = v - th, vt_hi = v + th;
    int cnt_d = 0, cnt_b = 0;
    for (int k = 0; k < 25; k++) {
        int p = im.at(x + kCircle[k & 15][0], y + kCircle[k & 15][1]);
        if (p < vt_lo) {
            if (++cnt_d > 8) return true;
        } else
            cnt_d = 0;
        if (p > vt_hi) {
            if (++cnt_b > 8) return true;
        } else
            cnt_b = 0;
    }
    return false;
}

static void fast_roi(const Image& im, int x0, int y0, int w, int h, int th, std::vector<KP>& out) {
    out.clear();
    if (w < 7 || h < 7) return;
    thread_local std::vector<int> score;
    thread_local std::vector<char> corner;
    score.assign((size_t)w * h, 0);
    corner.assign((size_t)w * h, 0);
    // OpenCV FAST_t's exact pre-test (threshold_tab, opposite pairs of the
    // circle): a pixel whose pairs cannot hold a 9-arc is not a corner; the
    // others get the full segment test.
    int off[16];
    for (int k = 0; k < 16; k++) off[k] = kCircle[k][1] * im.w + kCircle[k][0];
    uint8_t tab[512];
    for (int i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -th ? 1 : i > th ? 2 : 0);
    for (int i = 3; i < h - 3; i++) {
        const uint8_t* row = &im.px[(size_t)(y0 + i) * im.w + x0];
        for (int j = 3; j < w - 3; j++) {
            const uint8_t* p = row + j;
            const uint8_t* tb = tab + 255 - p[0];
            int d = tb[p[off[0]]] | tb[p[off[8]]];
            if (!d) continue;
            d &= tb[p[off[2]]] | tb[p[off[10]]];
            d &= tb[p[off[4]]] | tb[p[off[12]]];
            d &= tb[p[off[6]]] | tb[p[off[14]]];
            if (!d) continue;
            d &= tb[p[off[1]]] | tb[p[off[9]]];
            d &= tb[p[off[3]]] | tb[p[off[11]]];
            d &= tb[p[off[5]]] | tb[p[off[13]]];
            d &= tb[p[off[7]]] | tb[p[off[15]]];
            if (!d) continue;
            // the segment test (fast_is_corner) on the circle through offsets
            const int v = p[0], lo = v - th, hi = v + th;
            int cnt_d = 0, cnt_b = 0;
            bool is_corner = false;
            for (int k = 0; k < 25; k++) {
                const int q = p[off[k & 15]];
                cnt_d = q < lo ? cnt_d + 1 : 0;
                cnt_b = q > hi ? cnt_b + 1 : 0;
                if (cnt_d > 8 || cnt_b > 8) {
                    is_corner = true;
                    break;
                }
            }
            if (is_corner) {
                corner[(size_t)i * w + j] = 1;
                score[(size_t)i * w + j] = (uint8_t)fast_corner_score(im, x0 + j, y0 + i, th);
            }
        }
    }
    // Row-major scan = the order FAST_t pushes keypoints (row i-1 emitted while
    // row i is scanned); neighbours outside the detection window score 0.
    for (int i = 3; i < h - 3; i++)
        for (int j = 3; j < w - 3; j++) {
            if (!corner[(size_t)i * w + j]) continue;
            int s = score[(size_t)i * w + j];
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    if (!dx && !dy) continue;
                    if (!(s > score[(size_t)(i + dy) * w + (j + dx)])) {
                        keep = false;
                        break;
                    }
                }
            if (keep) out.push_back(KP{(float)j, (float)i, 7.f, -1.f, (float)s, 0, -1});
        }
}

// HarrisResponses(cellImage, keypoints, 7, HARRIS_K), ORBextractor.cc:86-127,
// called per cell when scoreType == HARRIS_SCORE (:667-670): keypoints are in
// cell coordinates, the ROI (x0, y0) of the level; every read lies inside the
// level (the cell ROI starts 13 px in, the block reaches 4 px out).
static void harris_responses(const Image& im, int x0, int y0, std::vector<KP>& pts) {
    const int blockSize = 7, r = blockSize / 2;
    const int step = im.w;
    float scale = (1 << 2) * blockSize * 255.0f;
    scale = 1.0f / scale;
    const float scale_sq_sq = scale * scale * scale * scale;
    const float harris_k = 0.04f;  // HARRIS_K, ORBextractor.cc:80
    for (KP& k : pts) {
        const int bx = cv_round(k.x - r), by = cv_round(k.y - r);
        const uint8_t* ptr0 = &im.px[(size_t)(y0 + by) * step + (x0 + bx)];
        int a = 0, b = 0, c = 0;
        for (int i = 0; i < blockSize; i++)
            for (int j = 0; j < blockSize; j++) {
                const uint8_t* ptr = ptr0 + i * step + j;
                const int Ix = (ptr[1] - ptr[-1]) * 2 + (ptr[-step + 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[step - 1]);
                const int Iy = (ptr[step] - ptr[-step]) * 2 + (ptr[step - 1] - ptr[-step - 1]) + (ptr[step + 1] - ptr[-step + 1]);
                a += Ix * Ix;
                b += Iy * Iy;
                c += Ix * Iy;
            }
        k.response = ((float)a * b - (float)c * c - harris_k * ((float)a + b) * ((float)a + b)) * scale_sq_sq;
    }
}

// KeyPointsFilter::retainBest (OpenCV 3.4 keypoint.cpp): nth_element at
// n_points-1 with KeypointResponseGreater, then the tie-keeping partition.
struct RespGreater {
    bool operator()(const KP& a, const KP& b) const { return a.response > b.response; }
};
static void retain_best(std::vector<KP>& kps, int n) {
    if (n >= 0 && kps.size() > (size_t)n) {
        if (n == 0) {
            kps.clear();
            return;
        }
        std::nth_element(kps.begin(), kps.begin() + n - 1, kps.end(), RespGreater());
        float amb = kps[n - 1].response;
        auto new_end = std::partition(kps.begin() + n, kps.end(), [amb](const KP& k) { return k.response >= amb; });
        kps.resize(new_end - kps.begin());
    }
}

// ---------------------------------------------------------------- E4 angle
// cv::fastAtan2 (OpenCV 3.4 mathfuncs_core), degrees in [0, 360).
float fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// IC_Angle, ORBextractor.cc:131-158 (intensity centroid on the unblurred level).
static float ic_angle(const Image& im, int cx, int cy, const int* umax) {
    int m01 = 0, m10 = 0;
    for (int u = -kHalfPatch; u <= kHalfPatch; ++u) m10 += u * im.at(cx + u, cy);
    for (int v = 1; v <= kHalfPatch; ++v) {
        int vsum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int vp = im.at(cx + u, cy + v), vm = im.at(cx + u, cy - v);
            vsum += vp - vm;
            m10 += u * (vp + vm);
        }
        m01 += v * vsum;
    }
    return fast_atan2((float)m01, (float)m10);
}

// ---------------------------------------------------------------- E6 rBRIEF
// computeOrbDescriptor, ORBextractor.cc:162-201. `(float)cos(angle)` of a
// float under `using namespace std` (:75, :167) is the C library's cosf/sinf:
// called here as such (glibc; the device restates its algorithm). Pixels
// outside the level interior come from the unblurred reflect-101 border
// (GaussianBlur writes only the ROI of the bordered level, :842).
static void orb_descriptor(const KP& kp, const Image& blurred, const Image& level, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = kp.angle * factorPI;
    float a = ::cosf(angle), b = ::sinf(angle);
    int cx = cv_round(kp.x), cy = cv_round(kp.y);
    auto value = [&](int idx) -> int {
        float px = (float)kOrbPattern31[2 * idx], py = (float)kOrbPattern31[2 * idx + 1];
        float t1 = px * b, t2 = py * a;
        int ry = cv_round(t1 + t2);
        float t3 = px * a, t4 = py * b;
        int rx = cv_round(t3 - t4);
        int x = cx + rx, y = cy + ry;
        if (x >= 0 && x < blurred.w && y >= 0 && y < blurred.h) return blurred.at(x, y);
        return level.at(reflect101(x, level.w), reflect101(y, level.h));
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; bit++) {
            int p = i * 16 + bit * 2;
            int t0 = value(p), t1 = value(p + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

// ---------------------------------------------------------------- E7
struct ExtractResult {
    std::vector<KP> kps;
    std::vector<uint8_t> desc;
    std::vector<Image> pyr, blur;
};

static void extract(const ExtractorPlan& P, const Image& img, ExtractResult& R) {
    R.kps.clear();
    R.desc.clear();
    R.pyr.assign(P.nlevels, Image());
    R.blur.assign(P.nlevels, Image());
    if (img.w == 0 || img.h == 0) return;
    // ComputePyramid :922-998 (borders are reflect-101 of each interior and are
    // addressed on the fly; FAST and IC_Angle never reach them).
    for (int l = 0; l < P.nlevels; l++) {
        int w = cv_round((float)img.w * P.invScale[l]), h = cv_round((float)img.h * P.invScale[l]);
        R.pyr[l] = l == 0 ? img : resize_linear(R.pyr[l - 1], w, h);
    }
    // ComputeKeyPoints :535-758
    std::vector<std::vector<KP>> all(P.nlevels);
    float imageRatio = (float)R.pyr[0].w / R.pyr[0].h;
    for (int level = 0; level < P.nlevels; ++level) {
        const Image& L = R.pyr[level];
        const int nDesired = P.featPerLevel[level];
        const int levelCols = (int)std::sqrt((float)nDesired / (5 * imageRatio));
        const int levelRows = (int)(imageRatio * levelCols);
        const int minBX = kEdgeThreshold, minBY = kEdgeThreshold;
        const int maxBX = L.w - kEdgeThreshold, maxBY = L.h - kEdgeThreshold;
        const int W = maxBX - minBX, H = maxBY - minBY;
        const int cellW = (int)std::ceil((float)W / levelCols);
        const int cellH = (int)std::ceil((float)H / levelRows);
        const int nCells = levelRows * levelCols;
        const int nfCell = (int)std::ceil((float)nDesired / nCells);
        std::vector<std::vector<KP>> cellKps(nCells);
        std::vector<int> nToRetain(nCells, 0), nTotal(nCells, 0), iniXCol(levelCols, 0), iniYRow(levelRows, 0);
        std::vector<char> noMore(nCells, 0);
        int nNoMore = 0, nToDistribute = 0;
        float hY = cellH + 6;
        for (int i = 0; i < levelRows; i++) {
            const float iniY = minBY + i * cellH - 3;
            iniYRow[i] = (int)iniY;
            if (i == levelRows - 1) {
                hY = maxBY + 3 - iniY;
                if (hY <= 0) continue;
            }
            float hX = cellW + 6;
            for (int j = 0; j < levelCols; j++) {
                float iniX;
                if (i == 0) {
                    iniX = minBX + j * cellW - 3;
                    iniXCol[j] = (int)iniX;
                } else
                    iniX = iniXCol[j];
                if (j == levelCols - 1) {
                    hX = maxBX + 3 - iniX;
                    if (hX <= 0) continue;
                }
                std::vector<KP>& ck = cellKps[i * levelCols + j];
                fast_roi(L, (int)iniX, (int)iniY, (int)hX, (int)hY, P.fastTh, ck);
                if (ck.size() <= 3) {
                    ck.clear();
                    fast_roi(L, (int)iniX, (int)iniY, (int)hX, (int)hY, P.minTh, ck);
                }
                if (P.scoreType == 0) harris_responses(L, (int)iniX, (int)iniY, ck);
                const int nKeys = (int)ck.size();
                nTotal[i * levelCols + j] = nKeys;
                if (nKeys > nfCell) {
                    nToRetain[i * levelCols + j] = nfCell;
                    noMore[i * levelCols + j] = 0;
                } else {
                    nToRetain[i * levelCols + j] = nKeys;
                    nToDistribute += nfCell - nKeys;
                    noMore[i * levelCols + j] = 1;
                    nNoMore++;
                }
            }
        }
        while (nToDistribute > 0 && nNoMore < nCells) {
            int nNew = nfCell + (int)std::ceil((float)nToDistribute / (nCells - nNoMore));
            nToDistribute = 0;
            for (int c = 0; c < nCells; c++) {
                if (noMore[c]) continue;
                if (nTotal[c] > nNew) {
                    nToRetain[c] = nNew;
                    noMore[c] = 0;
                } else {
                    nToRetain[c] = nTotal[c];
                    nToDistribute += nNew - nTotal[c];
                    noMore[c] = 1;
                    nNoMore++;
                }
            }
        }
        std::vector<KP>& kps = all[level];
        const int scaledPatchSize = (int)(kPatchSize * P.scale[level]);
        for (int i = 0; i < levelRows; i++)
            for (int j = 0; j < levelCols; j++) {
                std::vector<KP>& ck = cellKps[i * levelCols + j];
                retain_best(ck, nToRetain[i * levelCols + j]);
                if ((int)ck.size() > nToRetain[i * levelCols + j]) ck.resize(nToRetain[i * levelCols + j]);
                for (auto& k : ck) {
                    k.x += iniXCol[j];
                    k.y += iniYRow[i];
                    k.octave = level;
                    k.size = (float)scaledPatchSize;
                    kps.push_back(k);
                }
            }
        if ((int)kps.size() > nDesired) {
            retain_best(kps, nDesired);
            kps.resize(nDesired);
        }
    }
    for (int level = 0; level < P.nlevels; ++level)
        for (auto& k : all[level]) k.angle = ic_angle(R.pyr[level], (int)k.x, (int)k.y, P.umax);

    // operator() :803-874: blur, descriptors, scale, concatenate.
    for (int level = 0; level < P.nlevels; ++level) {
        R.blur[level] = gaussian_blur(R.pyr[level]);
        auto& kps = all[level];
        for (auto& k : kps) {
            uint8_t d[32];
            orb_descriptor(k, R.blur[level], R.pyr[level], d);
            R.desc.insert(R.desc.end(), d, d + 32);
        }
        if (level != 0) {
            float s = P.scale[level];
            for (auto& k : kps) {
                k.x = k.x * s;
                k.y = k.y * s;
            }
        }
        R.kps.insert(R.kps.end(), kps.begin(), kps.end());
    }
}

}  // namespace orc

// ---------------------------------------------------------------- C API
extern "C" {

int orc_extract_st(const uint8_t* img, int w, int h, int stride, int nfeatures, float scale_factor, int nlevels,
                   int score_type, int fast_th, gf_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
    orc::ExtractorPlan P(nfeatures, scale_factor, nlevels, fast_th);
    if (score_type != 0 && score_type != 1) return GF_ERR_ARG;
    P.scoreType = score_type;
    orc::Image im;
    im.w = w;
    im.h = h;
    im.px.resize((size_t)w * h);
    for (int y = 0; y < h; y++) std::memcpy(&im.px[(size_t)y * w], img + (size_t)y * stride, w);
    orc::ExtractResult R;
    orc::extract(P, im, R);
    int n = (int)R.kps.size();
    *n_out = n;
    if (n > cap) return GF_ERR_CAP;
    for (int i = 0; i < n; i++) {
        const orc::KP& k = R.kps[i];
        kps[i] = gf_keypoint{k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id};
    }
    if (n) std::memcpy(desc, R.desc.data(), (size_t)n * 32);
    return GF_OK;
}

int orc_extract(const uint8_t* img, int w, int h, int stride, int nfeatures, float scale_factor, int nlevels,
                int fast_th, gf_keypoint* kps, uint8_t* desc, int cap, int* n_out) {
    return orc_extract_st(img, w, h, stride, nfeatures, scale_factor, nlevels, 1, fast_th, kps, desc, cap, n_out);
}

// Plan tables: level sizes (w,h), quotas, scale factors.
int orc_extractor_plan(int w, int h, int nfeatures, float scale_factor, int nlevels, int* level_w, int* level_h,
                       int* feat_per_level, float* scales, int* umax16) {
    orc::ExtractorPlan P(nfeatures, scale_factor, nlevels, 20);
    for (int l = 0; l < nlevels; l++) {
        level_w[l] = orc::cv_round((float)w * P.invScale[l]);
        level_h[l] = orc::cv_round((float)h * P.invScale[l]);
        feat_per_level[l] = P.featPerLevel[l];
        scales[l] = P.scale[l];
    }
    if (umax16)
        for (int v = 0; v < 16; v++) umax16[v] = P.umax[v];
    return GF_OK;
}

// Intermediate planes for stage-by-stage parity: which 0 = pyramid, 1 = blur.
int orc_extract_level(const uint8_t* img, int w, int h, int nfeatures, float scale_factor, int nlevels, int level,
                      int which, uint8_t* out, int* lw, int* lh) {
    orc::ExtractorPlan P(nfeatures, scale_factor, nlevels, 20);
    orc::Image im;
    im.w = w;
    im.h = h;
    im.px.assign(img, img + (size_t)w * h);
    orc::Image cur = im;
    for (int l = 1; l <= level; l++)
        cur = orc::resize_linear(cur, orc::cv_round((float)w * P.invScale[l]), orc::cv_round((float)h * P.invScale[l]));
    if (which == 1) cur = orc::gaussian_blur(cur);
    *lw = cur.w;
    *lh = cur.h;
    if (out) std::memcpy(out, cur.px.data(), cur.px.size());
    return GF_OK;
}

void orc_gauss_kernel7(int* k) { orc::gauss_kernel7(k); }

// FAST primitives on a single plane, for brute-force invariants in the tests.
int orc_fast_score(const uint8_t* img, int w, int h, int x, int y, int th) {
    orc::Image im;
    im.w = w;
    im.h = h;
    im.px.assign(img, img + (size_t)w * h);
    if (!orc::fast_is_corner(im, x, y, th)) return 0;
    return orc::fast_corner_score(im, x, y, th);
}

float orc_fast_atan2(float y, float x) { return orc::fast_atan2(y, x); }

}  // extern "C"
