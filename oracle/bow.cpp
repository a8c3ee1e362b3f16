// CPU ORACLE (test infrastructure) — rows D1 and M6 of SURVEY.md §8a:
//   DBoW2 TemplatedVocabulary::transform(features, BowVector, FeatureVector,
//     levelsup) and its per-descriptor descent
//     (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1141-1208, 1232-1273),
//   BowVector::addWeight / addIfNotExist / normalize (BowVector.cpp:34-84),
//   FeatureVector::addFeature (FeatureVector.cpp:31-45),
//   FORB::distance (FORB.cpp:81-101), the scoring objects' mustNormalize
//     (ScoringObject.h:74-89);
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...) (src/ORBmatcher.cc:724-853)
//   and SearchByBoW(KeyFrame*, KeyFrame*, ...) (:1289-1424) with
//   ComputeThreeMaxima (:2338-2379);
//   SearchForTriangulation (:1426-1588) with CheckDistEpipolarLine (:705-722).
// The vocabulary tree arrives as the loaders build it (node 0 = root, nodes
// in record order, children in record order, word ids in record order of the
// leaves). DBoW2 is vendored, so these rows restate vendored text; parity is
// pinned against this restatement (no DBoW2 test or fixture exists upstream).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <vector>

#include "oracle_common.h"

namespace orc {
namespace {

int hamming(const uint8_t* a, const uint8_t* b) {  // FORB::distance: 8 x int32 SWAR popcount
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        std::memcpy(&x, a + 4 * i, 4);
        std::memcpy(&y, b + 4 * i, 4);
        uint32_t v = x ^ y;
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        d += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return d;
}

struct Vocab {
    int k, L, scoring, weighting;
    std::vector<std::vector<int>> children;
    const uint8_t* desc;
    const double* weight;
    std::vector<int> word;
    Vocab(int k_, int L_, int sc, int wt, int nnodes, const int32_t* parent, const uint8_t* d, const double* w,
          const uint8_t* leaf)
        : k(k_), L(L_), scoring(sc), weighting(wt), children(nnodes), desc(d), weight(w), word(nnodes, 0) {
        int nw = 0;
        for (int i = 1; i < nnodes; i++) {
            children[parent[i]].push_back(i);
            if (leaf[i]) word[i] = nw++;
        }
    }
    // transform(feature, word_id, weight, &nid, levelsup)
    void descend(const uint8_t* f, int levelsup, int& wid, double& w, int& nid) const {
        const int nid_level = L - levelsup;
        if (nid_level <= 0) nid = 0;
        int final_id = 0, level = 0;
        do {
            ++level;
            const std::vector<int>& nodes = children[final_id];
            final_id = nodes[0];
            int best = hamming(f, desc + 32 * (size_t)final_id);
            for (size_t c = 1; c < nodes.size(); c++) {
                const int d = hamming(f, desc + 32 * (size_t)nodes[c]);
                if (d < best) {
                    best = d;
                    final_id = nodes[c];
                }
            }
            if (level == nid_level) nid = final_id;
        } while (!children[final_id].empty());
        wid = word[final_id];
        w = weight[final_id];
    }
};

}  // namespace

void three_maxima(const int* histo, int L, int& ind1, int& ind2, int& ind3);  // match.cpp
}  // namespace orc

extern "C" {

// TemplatedVocabulary::transform(features, v, fv, levelsup) for one frame.
// Outputs the BowVector (word ids ascending, values) and the FeatureVector
// (node ids ascending, CSR offsets, feature indices).
int orc_bow_transform(int k, int L, int scoring, int weighting, int nnodes, const int32_t* parent,
                      const uint8_t* desc, const double* weight, const uint8_t* is_leaf, const uint8_t* feats, int n,
                      int levelsup, int32_t* words, double* values, int* nwords, int32_t* fv_nodes, int32_t* fv_start,
                      int32_t* fv_feats, int* nfv) {
    orc::Vocab V(k, L, scoring, weighting, nnodes, parent, desc, weight, is_leaf);
    std::map<int, double> v;
    std::map<int, std::vector<int>> fv;
    const bool must = scoring != 5;  // DOT_PRODUCT does not normalise; the others: L2 for L2_NORM, else L1
    if (nnodes > 1) {
        for (int i = 0; i < n; i++) {
            int wid, nid = 0;
            double w;
            V.descend(feats + 32 * (size_t)i, levelsup, wid, w, nid);
            if (!(w > 0)) continue;  // stopped word
            if (weighting == 0 || weighting == 1) {  // TF_IDF, TF: addWeight
                auto it = v.lower_bound(wid);
                if (it != v.end() && it->first == wid)
                    it->second += w;
                else
                    v.insert(it, {wid, w});
            } else {  // IDF, BINARY: addIfNotExist
                if (!v.count(wid)) v[wid] = w;
            }
            fv[nid].push_back(i);
        }
        if ((weighting == 0 || weighting == 1) && !v.empty() && !must) {
            const double nd = (double)v.size();
            for (auto& e : v) e.second /= nd;
        }
        if (must) {
            double norm = 0.0;
            if (scoring == 1) {
                for (auto& e : v) norm += e.second * e.second;
                norm = std::sqrt(norm);
            } else {
                for (auto& e : v) norm += std::fabs(e.second);
            }
            if (norm > 0.0)
                for (auto& e : v) e.second /= norm;
        }
    }
    int c = 0;
    for (auto& e : v) {
        words[c] = e.first;
        values[c++] = e.second;
    }
    *nwords = c;
    c = 0;
    int off = 0;
    for (auto& e : fv) {
        fv_nodes[c] = e.first;
        fv_start[c++] = off;
        for (int f : e.second) fv_feats[off++] = f;
    }
    fv_start[c] = off;
    *nfv = c;
    return GF_OK;
}

// ORBmatcher::SearchByBoW. mode 0: (KeyFrame a, Frame b) — a feature i with
// a_mp[i] >= 0 matches an unclaimed b feature, best <= TH_LOW(50) and best <
// nnratio * second; out[b index] = a_mp[i] (vpMapPointMatches). mode 1:
// (KeyFrame a, KeyFrame b) — b features need b_mp >= 0 and !vbMatched2, best <
// TH_LOW; out[a index] = b_mp[j] (vpMatches12). Rotation consistency when
// check_ori. Features of one FeatureVector node are walked in list order.
int orc_match_bow(int mode, float nnratio, int check_ori, const int32_t* a_nodes, const int32_t* a_start,
                  const int32_t* a_feats, int a_nn, const uint8_t* a_desc, const float* a_angle, const int32_t* a_mp,
                  int a_n, const int32_t* b_nodes, const int32_t* b_start, const int32_t* b_feats, int b_nn,
                  const uint8_t* b_desc, const float* b_angle, const int32_t* b_mp, int b_n, int32_t* out,
                  int* nmatches) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    const int nout = mode == 0 ? b_n : a_n;
    for (int i = 0; i < nout; i++) out[i] = -1;
    std::vector<char> matched_b(b_n, 0);
    std::vector<int> rotHist[30];
    const float factor = 1.0f / HISTO_LENGTH;
    int nm = 0, ia = 0, ib = 0;
    while (ia < a_nn && ib < b_nn) {
        if (a_nodes[ia] == b_nodes[ib]) {
            for (int x = a_start[ia]; x < a_start[ia + 1]; x++) {
                const int idxA = a_feats[x];
                if (a_mp[idxA] < 0) continue;
                int best1 = INT32_MAX, best2 = INT32_MAX, bestB = -1;
                for (int y = b_start[ib]; y < b_start[ib + 1]; y++) {
                    const int idxB = b_feats[y];
                    if (mode == 0 ? out[idxB] >= 0 : (matched_b[idxB] || b_mp[idxB] < 0)) continue;
                    const int dist = orc::hamming(a_desc + 32 * (size_t)idxA, b_desc + 32 * (size_t)idxB);
                    if (dist < best1) {
                        best2 = best1;
                        best1 = dist;
                        bestB = idxB;
                    } else if (dist < best2) {
                        best2 = dist;
                    }
                }
                const bool ok = mode == 0 ? best1 <= TH_LOW : best1 < TH_LOW;
                if (!ok || !(static_cast<float>(best1) < nnratio * static_cast<float>(best2))) continue;
                if (mode == 0) {
                    out[bestB] = a_mp[idxA];
                } else {
                    out[idxA] = b_mp[bestB];
                    matched_b[bestB] = 1;
                }
                if (check_ori) {
                    float rot = a_angle[idxA] - b_angle[bestB];
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)std::round(rot * factor);
                    if (bin == HISTO_LENGTH) bin = 0;
                    rotHist[bin].push_back(mode == 0 ? bestB : idxA);
                }
                nm++;
            }
            ia++;
            ib++;
        } else if (a_nodes[ia] < b_nodes[ib]) {
            ia = (int)(std::lower_bound(a_nodes + ia, a_nodes + a_nn, b_nodes[ib]) - a_nodes);
        } else {
            ib = (int)(std::lower_bound(b_nodes + ib, b_nodes + b_nn, a_nodes[ia]) - b_nodes);
        }
    }
    if (check_ori) {  // ComputeThreeMaxima
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int s = (int)rotHist[i].size();
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
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int j : rotHist[i]) {
                out[j] = -1;
                nm--;
            }
        }
    }
    *nmatches = nm;
    return GF_OK;
}

// ORBmatcher::SearchForTriangulation(pKF1 = a, pKF2 = b, F12, ...)
// (ORBmatcher.cc:1426-1588). out[a index] = matched b index (vMatches12).
int orc_search_triangulation(int check_ori, const int32_t* a_nodes, const int32_t* a_start, const int32_t* a_feats,
                             int a_nn, const uint8_t* a_desc, const gf_keypoint* a_kps, const int32_t* a_mp, int a_n,
                             const int32_t* b_nodes, const int32_t* b_start, const int32_t* b_feats, int b_nn,
                             const uint8_t* b_desc, const gf_keypoint* b_kps, const int32_t* b_mp, int b_n,
                             const float* F12, const float* sigma2_b, int32_t* out, int* nmatches) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    auto epipolar = [&](const gf_keypoint& kp1, const gf_keypoint& kp2) {  // CheckDistEpipolarLine
        const float a = kp1.x * F12[0] + kp1.y * F12[3] + F12[6];
        const float b = kp1.x * F12[1] + kp1.y * F12[4] + F12[7];
        const float c = kp1.x * F12[2] + kp1.y * F12[5] + F12[8];
        const float num = a * kp2.x + b * kp2.y + c;
        const float den = a * a + b * b;
        if (den == 0) return false;
        const float dsqr = num * num / den;
        return dsqr < 3.84 * sigma2_b[kp2.octave];
    };
    std::vector<char> vbMatched2(b_n, 0);
    for (int i = 0; i < a_n; i++) out[i] = -1;
    std::vector<int> rotHist[30];
    const float factor = 1.0f / HISTO_LENGTH;
    int nm = 0, ia = 0, ib = 0;
    while (ia < a_nn && ib < b_nn) {
        if (a_nodes[ia] == b_nodes[ib]) {
            for (int x = a_start[ia]; x < a_start[ia + 1]; x++) {
                const int idx1 = a_feats[x];
                if (a_mp[idx1] >= 0) continue;
                std::vector<std::pair<int, int>> vDistIndex;
                for (int y = b_start[ib]; y < b_start[ib + 1]; y++) {
                    const int idx2 = b_feats[y];
                    if (vbMatched2[idx2] || b_mp[idx2] >= 0) continue;
                    const int dist = orc::hamming(a_desc + 32 * (size_t)idx1, b_desc + 32 * (size_t)idx2);
                    if (dist > TH_LOW) continue;
                    vDistIndex.push_back({dist, idx2});
                }
                if (vDistIndex.empty()) continue;
                std::sort(vDistIndex.begin(), vDistIndex.end());
                const int BestDist = vDistIndex.front().first;
                const int DistTh = (int)std::round(2 * BestDist);
                for (const auto& di : vDistIndex) {
                    if (di.first > DistTh) break;
                    const int idx2 = di.second;
                    if (epipolar(a_kps[idx1], b_kps[idx2])) {
                        vbMatched2[idx2] = 1;
                        out[idx1] = idx2;
                        nm++;
                        if (check_ori) {
                            float rot = a_kps[idx1].angle - b_kps[idx2].angle;
                            if (rot < 0.0) rot += 360.0f;
                            int bin = (int)std::round(rot * factor);
                            if (bin == HISTO_LENGTH) bin = 0;
                            rotHist[bin].push_back(idx1);
                        }
                        break;
                    }
                }
            }
            ia++;
            ib++;
        } else if (a_nodes[ia] < b_nodes[ib]) {
            ia = (int)(std::lower_bound(a_nodes + ia, a_nodes + a_nn, b_nodes[ib]) - a_nodes);
        } else {
            ib = (int)(std::lower_bound(b_nodes + ib, b_nodes + b_nn, a_nodes[ia]) - b_nodes);
        }
    }
    if (check_ori) {
        int sizes[30], i1, i2, i3;
        for (int b = 0; b < HISTO_LENGTH; b++) sizes[b] = (int)rotHist[b].size();
        orc::three_maxima(sizes, HISTO_LENGTH, i1, i2, i3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
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


// L1Scoring::score (DBoW2 ScoringObject.cpp): over the words both BowVectors
// hold, in ascending word order, score += |v - w| - |v| - |w|; -score / 2.
double orc_bow_score_l1(const int32_t* w1, const double* v1, int n1, const int32_t* w2, const double* v2, int n2) {
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        if (w1[i] == w2[j]) {
            const double vi = v1[i], wi = v2[j];
            score += std::fabs(vi - wi) - std::fabs(vi) - std::fabs(wi);
            i++;
            j++;
        } else if (w1[i] < w2[j]) {
            i = (int)(std::lower_bound(w1 + i, w1 + n1, w2[j]) - w1);
        } else {
            j = (int)(std::lower_bound(w2 + j, w2 + n2, w1[i]) - w2);
        }
    }
    return -score / 2.0;
}

// KeyFrameDatabase::DetectRelocalisationCandidates (KeyFrameDatabase.cc:198-308)
// for one frame (BowVector words / values, nwords entries) against nkf
// keyframes: BowVector CSR bow_off / bow_words / bow_values, the inverted file
// (mvInvertedFile: per word the non-bad keyframes in insertion order, here
// ascending keyframe index; kf_bad may be null), the first 10 of
// mvpOrderedConnectedKeyFrames (cov_off / cov), and the keyframes'
// mnRelocQuery / mnRelocWords / mRelocScore, which persist across queries
// (a keyframe sharing words but not scored keeps an older score, :272-281).
// query = the frame's mnId (never 0). Candidates in the reference's order.
int orc_reloc_candidates(const int32_t* words, const double* values, int nwords, int nkf, const uint8_t* kf_bad,
                         const int32_t* bow_off, const int32_t* bow_words, const double* bow_values,
                         const int32_t* cov_off, const int32_t* cov, uint32_t query, uint32_t* reloc_query,
                         int32_t* reloc_words, float* reloc_score, int32_t* cands, int* ncand) {
    *ncand = 0;
    // the inverted file: word -> keyframes (ascending)
    std::map<int, std::vector<int>> inv;
    for (int k = 0; k < nkf; k++) {
        if (kf_bad && kf_bad[k]) continue;
        for (int e = bow_off[k]; e < bow_off[k + 1]; e++) inv[bow_words[e]].push_back(k);
    }
    std::vector<int> sharing;  // lKFsSharingWords
    for (int i = 0; i < nwords; i++) {
        auto it = inv.find(words[i]);
        if (it == inv.end()) continue;
        for (int k : it->second) {
            if (reloc_query[k] != query) {
                reloc_words[k] = 0;
                reloc_query[k] = query;
                sharing.push_back(k);
            }
            reloc_words[k]++;
        }
    }
    if (sharing.empty()) return GF_OK;
    int maxCommonWords = 0;
    for (int k : sharing)
        if (reloc_words[k] > maxCommonWords) maxCommonWords = reloc_words[k];
    const int minCommonWords = maxCommonWords * 0.8f;
    std::vector<std::pair<float, int>> scored;  // lScoreAndMatch
    for (int k : sharing) {
        if (reloc_words[k] > minCommonWords) {
            const float si = (float)orc_bow_score_l1(words, values, nwords, bow_words + bow_off[k], bow_values + bow_off[k],
                                                     bow_off[k + 1] - bow_off[k]);
            reloc_score[k] = si;
            scored.push_back({si, k});
        }
    }
    if (scored.empty()) return GF_OK;
    std::vector<std::pair<float, int>> acc;  // lAccScoreAndMatch
    float bestAccScore = 0;
    for (auto& sk : scored) {
        const int k = sk.second;
        float bestScore = sk.first, accScore = bestScore;
        int pBest = k;
        const int nn = std::min(10, cov_off[k + 1] - cov_off[k]);  // GetBestCovisibilityKeyFrames(10)
        for (int j = 0; j < nn; j++) {
            const int k2 = cov[cov_off[k] + j];
            if (reloc_query[k2] != query) continue;
            accScore += reloc_score[k2];
            if (reloc_score[k2] > bestScore) {
                pBest = k2;
                bestScore = reloc_score[k2];
            }
        }
        acc.push_back({accScore, pBest});
        if (accScore > bestAccScore) bestAccScore = accScore;
    }
    const float minScoreToRetain = 0.75f * bestAccScore;
    std::vector<char> added(nkf, 0);
    int nc = 0;
    for (auto& a : acc) {
        if (a.first > minScoreToRetain && !added[a.second]) {
            cands[nc++] = a.second;
            added[a.second] = 1;
        }
    }
    *ncand = nc;
    return GF_OK;
}

}  // extern "C"
