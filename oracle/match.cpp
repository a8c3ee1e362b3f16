// CPU ORACLE (test infrastructure) — matching rows E8, M1-M3, M7 of
// SURVEY.md §8a, restated sequentially from src/ORBmatcher.cc and src/Frame.cc,
// and the local-mapping rows of §8(f) rank 3: MapPoint::ComputeDistinctive-
// Descriptors (src/MapPoint.cc:197-262) and ORBmatcher::Fuse (:1590-1707).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle_common.h"

namespace orc {

static const int kGridCols = 64, kGridRows = 48;  // Frame.h:35-36
static const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;

struct FrameGrid {
    const gf_frame_info* fi;
    const gf_keypoint* kps;
    int n;
    float invW, invH;
    std::vector<float> scales;
    std::vector<int> grid[kGridCols][kGridRows];

    FrameGrid(const gf_frame_info* f, const gf_keypoint* k, int nk) : fi(f), kps(k), n(nk) {
        // Frame.cc:91-92 and :114-131
        invW = (float)kGridCols / (float)(fi->max_x - fi->min_x);
        invH = (float)kGridRows / (float)(fi->max_y - fi->min_y);
        scales.resize(fi->nlevels);
        scales[0] = 1.f;
        for (int i = 1; i < fi->nlevels; i++) scales[i] = scales[i - 1] * fi->scale_factor;
        for (int i = 0; i < n; i++) {
            int px = (int)std::round((kps[i].x - fi->min_x) * invW);
            int py = (int)std::round((kps[i].y - fi->min_y) * invH);
            if (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) continue;
            grid[px][py].push_back(i);
        }
    }

    // Frame::GetFeaturesInArea, Frame.cc:300-365
    std::vector<int> area(float x, float y, float r, int minLevel, int maxLevel) const {
        std::vector<int> out;
        int nMinCellX = (int)std::floor((x - fi->min_x - r) * invW);
        nMinCellX = std::max(0, nMinCellX);
        if (nMinCellX >= kGridCols) return out;
        int nMaxCellX = (int)std::ceil((x - fi->min_x + r) * invW);
        nMaxCellX = std::min(kGridCols - 1, nMaxCellX);
        if (nMaxCellX < 0) return out;
        int nMinCellY = (int)std::floor((y - fi->min_y - r) * invH);
        nMinCellY = std::max(0, nMinCellY);
        if (nMinCellY >= kGridRows) return out;
        int nMaxCellY = (int)std::ceil((y - fi->min_y + r) * invH);
        nMaxCellY = std::min(kGridRows - 1, nMaxCellY);
        if (nMaxCellY < 0) return out;
        bool check = !(minLevel == -1 && maxLevel == -1);
        bool same = check && minLevel == maxLevel;
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++)
                for (int idx : grid[ix][iy]) {
                    const gf_keypoint& k = kps[idx];
                    if (check && !same) {
                        if (k.octave < minLevel || k.octave > maxLevel) continue;
                    } else if (same) {
                        if (k.octave != minLevel) continue;
                    }
                    if (std::fabs(k.x - x) > r || std::fabs(k.y - y) > r) continue;
                    out.push_back(idx);
                }
        return out;
    }
};

// ORBmatcher::DescriptorDistance, ORBmatcher.cc:2384-2400
int descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t va, vb;
        std::memcpy(&va, a + 4 * i, 4);
        std::memcpy(&vb, b + 4 * i, 4);
        uint32_t v = va ^ vb;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return dist;
}

// ORBmatcher::RadiusByViewingCos, ORBmatcher.cc:696-702
static float radius_by_viewing_cos(float c) { return c > 0.998 ? 2.5f : 4.0f; }

// ORBmatcher::ComputeThreeMaxima, ORBmatcher.cc:2338-2379
void three_maxima(const int* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    ind1 = ind2 = ind3 = -1;
    for (int i = 0; i < L; i++) {
        const int s = histo[i];
        if (s > max1) {
            max3 = max2;
            max2 = max1;
            max1 = s;
            ind3 = ind2;
            ind2 = ind1;
            ind1 = i;
        } else if (s > max2) {
            max3 = max2;
            max2 = s;
            ind3 = ind2;
            ind2 = i;
        } else if (s > max3) {
            max3 = s;
            ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
}

// Pc = R * P + t, float, left-to-right, no contraction (cv::Mat
// float gemm restated).
static inline void transform(const float* T, const float* P, float* Pc) {
    for (int r = 0; r < 3; r++)
        Pc[r] = dot3p(T[4 * r + 0], P[0], T[4 * r + 1], P[1], T[4 * r + 2], P[2], T[4 * r + 3]);
}

int g_gemm_mode = 0;
// area candidates (Frame::GetFeaturesInArea sizes) of the projection matchers
// since the last orc_cand_take(): SURVEY §8d B_match's C, counted as the
// device counts it
long long g_cand = 0;

// ORBmatcher::SearchByProjection_OnePoint (ORBmatcher.h:71-145) over a grid
// built once per frame (runActiveMapMatching's one-point matches).
struct OnePointGrid {
    FrameGrid G;
    OnePointGrid(const gf_frame_info* f, const gf_keypoint* k, int n) : G(f, k, n) {}
};
OnePointGrid* one_point_grid(const gf_frame_info* fi, const gf_keypoint* kps, int n) {
    return new OnePointGrid(fi, kps, n);
}
void one_point_grid_free(OnePointGrid* g) { delete g; }

int one_point(const OnePointGrid* g, const gf_mp_view& v, const uint8_t* mp_desc, const uint8_t* desc, float th,
              float nnratio, const int32_t* kp2mp, int* dist_out) {
    const FrameGrid& G = g->G;
    if (!v.in_view) return -1;
    const int pl = v.level;
    float r = radius_by_viewing_cos(v.view_cos);
    if (th != 1.0) r *= th;
    std::vector<int> near = G.area(v.u, v.v, r * G.scales[pl], pl - 1, pl);
    if (near.empty()) return -1;
    int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
    for (int idx : near) {
        if (kp2mp[idx] >= 0) continue;
        const int dist = descriptor_distance(mp_desc, desc + 32 * (size_t)idx);
        if (dist < bestDist) {
            bestDist2 = bestDist;
            bestDist = dist;
            bestLevel2 = bestLevel;
            bestLevel = G.kps[idx].octave;
            bestIdx = idx;
        } else if (dist < bestDist2) {
            bestLevel2 = G.kps[idx].octave;
            bestDist2 = dist;
        }
    }
    if (bestDist > TH_HIGH) return -1;
    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) return -1;
    *dist_out = bestDist;
    return bestIdx;
}

}  // namespace orc

extern "C" {

int orc_descriptor_distance(const uint8_t* a, const uint8_t* b) { return orc::descriptor_distance(a, b); }

long long orc_cand_take(void) {
    const long long c = orc::g_cand;
    orc::g_cand = 0;
    return c;
}

// docs/ORACLE_ASSUMPTIONS.md A1 (sensitivity runs only; 0 = parity)
void orc_set_gemm_mode(int mode) { orc::g_gemm_mode = mode; }

// Frame::isInFrustum, Frame.cc:166-227
int orc_frustum(const gf_frame_info* fi, const float* Tcw, const gf_map_point* mps, int m, float viewCosLimit,
                gf_mp_view* views, int* n_in_view) {
    std::vector<float> scales(fi->nlevels);
    scales[0] = 1.f;
    for (int i = 1; i < fi->nlevels; i++) scales[i] = scales[i - 1] * fi->scale_factor;
    // Ow = -Rcw^T * tcw (Frame::UpdatePoseMatrices :143-148)
    float Ow[3];
    for (int c = 0; c < 3; c++) Ow[c] = -orc::dot3(Tcw[0 * 4 + c], Tcw[3], Tcw[1 * 4 + c], Tcw[7], Tcw[2 * 4 + c], Tcw[11]);
    int cnt = 0;
    for (int i = 0; i < m; i++) {
        gf_mp_view& v = views[i];
        v.in_view = 0;
        v.u = v.v = v.view_cos = 0.f;
        v.level = 0;
        const float* P = mps[i].pos;
        float Pc[3];
        orc::transform(Tcw, P, Pc);
        if (Pc[2] < 0.0) continue;
        const float invz = (float)(1.0 / (double)Pc[2]);
        const float u = fi->fx * Pc[0] * invz + fi->cx;
        const float vv = fi->fy * Pc[1] * invz + fi->cy;
        if (u < fi->min_x || u > fi->max_x) continue;
        if (vv < fi->min_y || vv > fi->max_y) continue;
        const float maxD = mps[i].max_dist, minD = mps[i].min_dist;
        const float PO[3] = {P[0] - Ow[0], P[1] - Ow[1], P[2] - Ow[2]};
        const float dist = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist < minD || dist > maxD) continue;
        const float* Pn = mps[i].normal;
        double dot = (double)PO[0] * Pn[0] + (double)PO[1] * Pn[1] + (double)PO[2] * Pn[2];
        float viewCos = (float)(dot / dist);
        if (viewCos < viewCosLimit) continue;
        float ratio = dist / minD;
        int lvl = 0;
        while (lvl < fi->nlevels && scales[lvl] < ratio) lvl++;  // lower_bound
        if (lvl >= fi->nlevels) lvl = fi->nlevels - 1;
        v.in_view = 1;
        v.u = u;
        v.v = vv;
        v.level = lvl;
        v.view_cos = viewCos;
        cnt++;
    }
    *n_in_view = cnt;
    return GF_OK;
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th), :384-465
int orc_match_project(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                      const gf_mp_view* views, const uint8_t* mp_desc, int m, float th, float nnratio,
                      int32_t* kp2mp, int32_t* score, int* nmatches) {
    orc::FrameGrid G(fi, kps, n);
    int nm = 0;
    const bool bFactor = th != 1.0;
    for (int k = 0; k < m; k++) {
        const gf_mp_view& v = views[k];
        if (!v.in_view) continue;
        const int pl = v.level;
        float r = orc::radius_by_viewing_cos(v.view_cos);
        if (bFactor) r *= th;
        std::vector<int> near = G.area(v.u, v.v, r * G.scales[pl], pl - 1, pl);
        orc::g_cand += (long long)near.size();  // B_match's C
        if (near.empty()) continue;
        int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
        for (int idx : near) {
            if (kp2mp[idx] >= 0) continue;
            const int dist = orc::descriptor_distance(mp_desc + 32 * (size_t)k, desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= orc::TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            kp2mp[bestIdx] = k;
            score[bestIdx] = bestDist;
            nm++;
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// ORBmatcher::SearchByProjection_Budget(F, vpMapPoints, th, time_constr)
// (ORBmatcher.cc:276-379) over the map points list[0 .. nlist) in list order
// (views / mp_desc indexed by map point). el (optional) holds the elapsed
// time the device measured at each list point and constr2 = 2 x time_constr
// in the same ticks: constr2 <= 0 returns at once (:281-282); otherwise the
// loop breaks after the first point that reaches the clock check (in view, a
// non-empty area, not rejected by the ratio test) with 2 el >= constr2
// (:366-371). *cut = that list position, -1 when the loop ran to the end.
int orc_match_project_list(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                           const gf_mp_view* views, const uint8_t* mp_desc, const int32_t* list, int nlist, float th,
                           float nnratio, int32_t* kp2mp, int32_t* score, int* nmatches, const long long* el,
                           long long constr2, int* cut) {
    *nmatches = 0;
    if (cut) *cut = -1;
    if (el && constr2 <= 0) return GF_OK;
    orc::FrameGrid G(fi, kps, n);
    int nm = 0;
    const bool bFactor = th != 1.0;
    for (int k = 0; k < nlist; k++) {
        const int q = list[k];
        const gf_mp_view& v = views[q];
        if (!v.in_view) continue;
        const int pl = v.level;
        float r = orc::radius_by_viewing_cos(v.view_cos);
        if (bFactor) r *= th;
        std::vector<int> near = G.area(v.u, v.v, r * G.scales[pl], pl - 1, pl);
        orc::g_cand += (long long)near.size();
        if (near.empty()) continue;
        int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
        for (int idx : near) {
            if (kp2mp[idx] >= 0) continue;
            const int dist = orc::descriptor_distance(mp_desc + 32 * (size_t)q, desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = kps[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= orc::TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            kp2mp[bestIdx] = q;
            score[bestIdx] = bestDist;
            nm++;
        }
        if (el && 2 * el[k] >= constr2) {
            if (cut) *cut = k;
            break;
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th), :2081-2202
int orc_match_lastframe(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n, const float* Tcw,
                        const gf_keypoint* last_kps, const uint8_t* last_desc, const int32_t* last_kp2mp,
                        const uint8_t* last_outlier, const float* last_pos, int n_last, float th, int check_ori,
                        int32_t* kp2mp, int32_t* score, int* nmatches) {
    orc::FrameGrid G(fi, kps, n);
    std::vector<int> rotHist[orc::HISTO_LENGTH];
    const float factor = 1.0f / orc::HISTO_LENGTH;
    int nm = 0;
    for (int i = 0; i < n_last; i++) {
        if (last_kp2mp[i] < 0 || last_outlier[i]) continue;
        float Pc[3];
        orc::transform(Tcw, last_pos + 3 * (size_t)i, Pc);
        const float xc = Pc[0], yc = Pc[1];
        const float invzc = (float)(1.0 / (double)Pc[2]);
        float u = fi->fx * xc * invzc + fi->cx;
        float v = fi->fy * yc * invzc + fi->cy;
        if (u < fi->min_x || u > fi->max_x) continue;
        if (v < fi->min_y || v > fi->max_y) continue;
        int oct = last_kps[i].octave;
        float radius = th * G.scales[oct];
        std::vector<int> idx2 = G.area(u, v, radius, oct - 1, oct + 1);
        orc::g_cand += (long long)idx2.size();  // B_match's C
        if (idx2.empty()) continue;
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (int i2 : idx2) {
            if (kp2mp[i2] >= 0) continue;
            int dist = orc::descriptor_distance(last_desc + 32 * (size_t)i, desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= orc::TH_HIGH) {
            kp2mp[bestIdx2] = last_kp2mp[i];
            score[bestIdx2] = bestDist;
            nm++;
            if (check_ori) {
                float rot = last_kps[i].angle - kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == orc::HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) {
        int sizes[orc::HISTO_LENGTH], i1, i2, i3;
        for (int b = 0; b < orc::HISTO_LENGTH; b++) sizes[b] = (int)rotHist[b].size();
        orc::three_maxima(sizes, orc::HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < orc::HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int j : rotHist[b]) {
                kp2mp[j] = -1;
                score[j] = 999;
                nm--;
            }
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:227-261) for nmp
// points: the float N x N distance table, each row copied to vector<int> and
// sorted, median = row[0.5 * (N - 1)], strict < keeps the first minimum.
int orc_distinctive_descriptors(int nmp, const uint8_t* desc, const int32_t* offsets, int32_t* best,
                                uint8_t* out_desc) {
    for (int p = 0; p < nmp; p++) {
        const int o = offsets[p], N = offsets[p + 1] - o;
        best[p] = -1;
        if (N <= 0) continue;
        std::vector<float> D((size_t)N * N);
        for (int i = 0; i < N; i++) {
            D[(size_t)i * N + i] = 0;
            for (int j = i + 1; j < N; j++) {
                const int d = orc::descriptor_distance(desc + 32 * (size_t)(o + i), desc + 32 * (size_t)(o + j));
                D[(size_t)i * N + j] = (float)d;
                D[(size_t)j * N + i] = (float)d;
            }
        }
        int BestMedian = INT_MAX, BestIdx = 0;
        for (int i = 0; i < N; i++) {
            std::vector<int> v(D.begin() + (size_t)i * N, D.begin() + (size_t)(i + 1) * N);
            std::sort(v.begin(), v.end());
            const int median = v[(size_t)(0.5 * (N - 1))];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = i;
            }
        }
        best[p] = BestIdx;
        if (out_desc) std::memcpy(out_desc + 32 * (size_t)p, desc + 32 * (size_t)(o + BestIdx), 32);
    }
    return GF_OK;
}

// ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>&, th) (ORBmatcher.cc:1590-1707),
// walked in list order with the keyframe's slots updated as the reference
// does (AddMapPoint fills a slot; Replace() leaves the slot's occupant).
int orc_fuse(const gf_frame_info* fi, const float* Tcw, const float* Ow, const gf_keypoint* kps,
             const uint8_t* desc, int n, const int32_t* kf_mp, const uint8_t* kf_mp_bad, const gf_map_point* mps,
             const uint8_t* mp_desc, const uint8_t* mp_skip, const int32_t* mp_ids, int m, float th,
             gf_fuse_result* res, int* nfused) {
    orc::FrameGrid G(fi, kps, n);
    const int nMaxLevel = fi->nlevels - 1;
    // slot -> (occupant id, occupant bad); list-point occupants are not bad
    std::vector<int> occ(kf_mp, kf_mp + n);
    std::vector<char> bad(n, 0);
    if (kf_mp_bad)
        for (int k = 0; k < n; k++) bad[k] = (char)kf_mp_bad[k];
    int nFused = 0;
    for (int i = 0; i < m; i++) {
        res[i] = gf_fuse_result{-1, GF_FUSE_NONE, -1};
        if (mp_skip && mp_skip[i]) continue;
        const gf_map_point& mp = mps[i];
        float Pc[3];
        orc::transform(Tcw, mp.pos, Pc);
        if (Pc[2] < 0.0f) continue;
        const float invz = 1 / Pc[2];
        const float x = Pc[0] * invz;
        const float y = Pc[1] * invz;
        const float u = fi->fx * x + fi->cx;
        const float v = fi->fy * y + fi->cy;
        if (!(u >= fi->min_x && u < fi->max_x && v >= fi->min_y && v < fi->max_y)) continue;  // KeyFrame::IsInImage
        const float maxDistance = mp.max_dist, minDistance = mp.min_dist;
        const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
        const float dist3D = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
        if (dot < 0.5 * dist3D) continue;
        const float ratio = dist3D / minDistance;
        const int lb = (int)(std::lower_bound(G.scales.begin(), G.scales.end(), ratio) - G.scales.begin());
        const int nPredictedLevel = std::min(lb, nMaxLevel);
        const float radius = th * G.scales[nPredictedLevel];
        const std::vector<int> idxs = G.area(u, v, radius, -1, -1);  // KeyFrame::GetFeaturesInArea
        if (idxs.empty()) continue;
        int bestDist = INT_MAX, bestIdx = -1;
        for (int idx : idxs) {
            const int kpLevel = kps[idx].octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int dist = orc::descriptor_distance(mp_desc + 32 * (size_t)i, desc + 32 * (size_t)idx);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx = idx;
            }
        }
        if (bestDist <= orc::TH_LOW) {
            gf_fuse_result& r = res[i];
            r.kp = bestIdx;
            if (occ[bestIdx] >= 0) {
                if (!bad[bestIdx]) {
                    r.action = GF_FUSE_REPLACE;  // pMP->Replace(pMPinKF)
                    r.target = occ[bestIdx];
                } else {
                    r.action = GF_FUSE_KEEP;
                }
            } else {
                r.action = GF_FUSE_ADD;
                occ[bestIdx] = mp_ids ? mp_ids[i] : i;
            }
            nFused++;
        }
    }
    *nfused = nFused;
    return GF_OK;
}


// ORBmatcher::WindowSearch(F1, F2, windowSize, vpMapPointMatches2, minScaleLevel,
// maxScaleLevel) (ORBmatcher.cc:979-1086) for the matcher TrackPreviousFrame
// builds (ORBmatcher(0.9, true), Tracking.cc:1331): F1 = the last frame (its
// undistorted keypoints, descriptors and map points, -1 = NULL), F2 = the
// current frame. out (n2 entries) = vpMapPointMatches2. max_level = INT_MAX:
// no maximum. Sequential claims; the ratio test compares int with the float
// product (:1046); rotation bins as the reference computes them (:1052-1059).
int orc_window_search(const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                      const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, int n1, int window,
                      int min_level, int max_level, float nnratio, int check_ori, int32_t* out, int* nmatches) {
    orc::FrameGrid G(fi, kps2, n2);
    for (int i = 0; i < n2; i++) out[i] = -1;
    std::vector<int> rotHist[orc::HISTO_LENGTH];
    const float factor = 1.0f / orc::HISTO_LENGTH;
    const bool bMinLevel = min_level > 0, bMaxLevel = max_level < INT_MAX;
    int nm = 0;
    for (int i1 = 0; i1 < n1; i1++) {
        if (mp1[i1] < 0) continue;
        const gf_keypoint& kp1 = kps1[i1];
        const int level1 = kp1.octave;
        if (bMinLevel && level1 < min_level) continue;
        if (bMaxLevel && level1 > max_level) continue;
        const std::vector<int> idx2 = G.area(kp1.x, kp1.y, (float)window, level1, level1);
        if (idx2.empty()) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int i2 : idx2) {
            if (out[i2] >= 0) continue;
            const int dist = orc::descriptor_distance(desc1 + 32 * (size_t)i1, desc2 + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if ((float)bestDist <= (float)bestDist2 * nnratio && bestDist <= orc::TH_HIGH) {
            out[bestIdx2] = mp1[i1];
            nm++;
            if (check_ori) {
                float rot = kp1.angle - kps2[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == orc::HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) {
        int sizes[orc::HISTO_LENGTH], i1, i2, i3;
        for (int b = 0; b < orc::HISTO_LENGTH; b++) sizes[b] = (int)rotHist[b].size();
        orc::three_maxima(sizes, orc::HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < orc::HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int j : rotHist[b]) {
                out[j] = -1;
                nm--;
            }
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// ORBmatcher::SearchByProjection(Frame& F1, Frame& F2, windowSize,
// vpMapPointMatches2) (ORBmatcher.cc:1089-1168): F1's map points (world
// positions pos1) not already among F2's matches (the set is taken at entry,
// :1092) projected with F2's pose, without a depth or bounds test, into a
// same-level window; best < ratio x second (floats, :1155) and <= TH_HIGH.
// kp2mp / score (n2 entries) are F2.mvpMapPoints in and vpMapPointMatches2 /
// mvpMatchScore out.
int orc_search_frames(const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2, const float* Tcw2,
                      const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, const float* pos1, int n1,
                      int window, float nnratio, int32_t* kp2mp, int32_t* score, int* nmatches) {
    orc::FrameGrid G(fi, kps2, n2);
    std::vector<int> found;
    for (int i = 0; i < n2; i++)
        if (kp2mp[i] >= 0) found.push_back(kp2mp[i]);
    std::sort(found.begin(), found.end());
    int nm = 0;
    for (int i1 = 0; i1 < n1; i1++) {
        const int mp = mp1[i1];
        if (mp < 0 || std::binary_search(found.begin(), found.end(), mp)) continue;
        const int level1 = kps1[i1].octave;
        float Pc[3];
        orc::transform(Tcw2, pos1 + 3 * (size_t)i1, Pc);
        const float invzc2 = (float)(1.0 / (double)Pc[2]);
        const float u2 = fi->fx * Pc[0] * invzc2 + fi->cx;
        const float v2 = fi->fy * Pc[1] * invzc2 + fi->cy;
        const std::vector<int> idx2 = G.area(u2, v2, (float)window, level1, level1);
        if (idx2.empty()) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (int i2 : idx2) {
            if (kp2mp[i2] >= 0) continue;
            const int dist = orc::descriptor_distance(desc1 + 32 * (size_t)i1, desc2 + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if ((float)bestDist <= (float)bestDist2 * nnratio && bestDist <= orc::TH_HIGH) {
            kp2mp[bestIdx2] = mp;
            score[bestIdx2] = bestDist;
            nm++;
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// ORBmatcher::SearchByProjection(Frame& F, KeyFrame* pKF, sAlreadyFound, th,
// ORBdist) (ORBmatcher.cc:2204-2336), Relocalisation's ORBmatcher(0.9, true):
// the keyframe's map points in slot order (kf_mp, -1 = NULL) not marked in
// `found` (a byte per map point) projected with the frame's pose; image bounds,
// the predicted level from the invariance distance (lower_bound of the scale
// factors), a window th x scale over levels [pred - 1, pred + 1]; the nearest
// unclaimed keypoint within ORBdist claims; rotation bins from the keyframe
// keypoint's angle. kp2mp / score are the frame's mvpMapPoints / mvpMatchScore.
int orc_search_kf_projection(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                             const float* Tcw, const gf_keypoint* kf_kps, const int32_t* kf_mp, int nslots,
                             const gf_map_point* mps, const uint8_t* mp_desc, const uint8_t* found, float th,
                             int orb_dist, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches) {
    orc::FrameGrid G(fi, kps, n);
    float Ow[3];  // -Rcw^T tcw (:2210)
    for (int c = 0; c < 3; c++) Ow[c] = -orc::dot3(Tcw[0 * 4 + c], Tcw[3], Tcw[1 * 4 + c], Tcw[7], Tcw[2 * 4 + c], Tcw[11]);
    std::vector<int> rotHist[orc::HISTO_LENGTH];
    const float factor = 1.0f / orc::HISTO_LENGTH;
    int nm = 0;
    for (int i = 0; i < nslots; i++) {
        const int mp = kf_mp[i];
        if (mp < 0 || found[mp]) continue;
        const gf_map_point& P = mps[mp];
        float Pc[3];
        orc::transform(Tcw, P.pos, Pc);
        const float invzc = (float)(1.0 / (double)Pc[2]);
        const float u = fi->fx * Pc[0] * invzc + fi->cx;
        const float v = fi->fy * Pc[1] * invzc + fi->cy;
        if (u < fi->min_x || u > fi->max_x) continue;
        if (v < fi->min_y || v > fi->max_y) continue;
        const float minDistance = P.min_dist;
        const float PO[3] = {P.pos[0] - Ow[0], P.pos[1] - Ow[1], P.pos[2] - Ow[2]};
        const float dist3D = (float)std::sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
        const float ratio = dist3D / minDistance;
        const int lb = (int)(std::lower_bound(G.scales.begin(), G.scales.end(), ratio) - G.scales.begin());
        const int nPredictedLevel = std::min(lb, fi->nlevels - 1);
        const float radius = th * G.scales[nPredictedLevel];
        const std::vector<int> idx2 = G.area(u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1);
        if (idx2.empty()) continue;
        int bestDist = INT_MAX, bestIdx2 = -1;
        for (int i2 : idx2) {
            if (kp2mp[i2] >= 0) continue;
            const int dist = orc::descriptor_distance(mp_desc + 32 * (size_t)mp, desc + 32 * (size_t)i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= orb_dist) {
            kp2mp[bestIdx2] = mp;
            score[bestIdx2] = bestDist;
            nm++;
            if (check_ori) {
                float rot = kf_kps[i].angle - kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == orc::HISTO_LENGTH) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    if (check_ori) {
        int sizes[orc::HISTO_LENGTH], i1, i2, i3;
        for (int b = 0; b < orc::HISTO_LENGTH; b++) sizes[b] = (int)rotHist[b].size();
        orc::three_maxima(sizes, orc::HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < orc::HISTO_LENGTH; b++) {
            if (b == i1 || b == i2 || b == i3) continue;
            for (int j : rotHist[b]) {
                kp2mp[j] = -1;
                score[j] = 999;
                nm--;
            }
        }
    }
    *nmatches = nm;
    return GF_OK;
}

}  // extern "C"
