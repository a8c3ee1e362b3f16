// C++ drop-in layer (include/gfslam/orbslam.h): the reference's ORBextractor /
// ORBmatcher / Frame / Observability / Optimizer interface forwarded to the
// libgfslam C-ABI. Only packing happens here: MapPoint pointers become
// indices into a per-call table, results are written back to the same
// fields the reference mutates.
#include "../../include/gfslam/orbslam.h"

#include <algorithm>
#include <cmath>
#include <thread>
#include <unordered_map>

namespace ORB_SLAM {

namespace {

thread_local gf_ctx* t_ctx = nullptr;
thread_local int t_device = 0;

void check(int rc) {
    if (rc != GF_OK) throw GpuError(rc, gf_last_error());
}

// Pointer table: map points of one call, in the order given, plus any
// pointer already held by a frame (so pre-existing claims keep an index).
struct PointTable {
    std::vector<MapPoint*> ptrs;
    std::unordered_map<const MapPoint*, int> index;
    int id(MapPoint* p) {
        if (!p) return -1;
        auto it = index.find(p);
        if (it != index.end()) return it->second;
        const int i = (int)ptrs.size();
        ptrs.push_back(p);
        index.emplace(p, i);
        return i;
    }
};

gf_map_point to_abi(const MapPoint& m) {
    gf_map_point g;
    std::memcpy(g.pos, m.mWorldPos, sizeof(g.pos));
    std::memcpy(g.normal, m.mNormalVector, sizeof(g.normal));
    g.min_dist = m.mfMinDistance;
    g.max_dist = m.mfMaxDistance;
    return g;
}

gf_mp_view view_of(const MapPoint* p) {
    gf_mp_view v;
    v.u = p->mTrackProjX;
    v.v = p->mTrackProjY;
    v.view_cos = p->mTrackViewCos;
    v.level = p->mnTrackScaleLevel;
    v.in_view = p->mbTrackInView && !p->isBad();
    return v;
}

}  // namespace

gf_ctx* Context() {
    if (!t_ctx) check(gf_ctx_create(t_device, &t_ctx));
    return t_ctx;
}

void SetDevice(int device) {
    if (t_ctx) throw GpuError(GF_ERR_ARG, "SetDevice after the context was created");
    t_device = device;
}

/* ---------------------------------------------------------------- ORBVocabulary */
ORBVocabulary::~ORBVocabulary() {
    if (voc_) gf_vocab_destroy(voc_);
}

bool ORBVocabulary::loadFromTextFile(const std::string& filename) {
    if (filename.size() < 4 || filename.compare(filename.size() - 4, 4, ".txt") != 0) return false;
    gf_vocab* v = nullptr;
    if (gf_vocab_load(Context(), filename.c_str(), &v) != GF_OK) return false;
    if (voc_) gf_vocab_destroy(voc_);
    voc_ = v;
    return true;
}

bool ORBVocabulary::loadFromBinaryFile(const std::string& filename) {
    if (filename.size() >= 4 && filename.compare(filename.size() - 4, 4, ".txt") == 0) return false;
    gf_vocab* v = nullptr;
    if (gf_vocab_load(Context(), filename.c_str(), &v) != GF_OK) return false;
    if (voc_) gf_vocab_destroy(voc_);
    voc_ = v;
    return true;
}

void ORBVocabulary::transform(const Descriptors& features, BowVector& v, FeatureVector& fv, int levelsup) const {
    if (!voc_) throw GpuError(GF_ERR_ARG, "vocabulary not loaded");
    const int n = features.rows;
    const int cap = std::max(n, 1);
    v.words.assign(cap, 0);
    v.values.assign(cap, 0.0);
    fv.nodes.assign(cap, 0);
    fv.start.assign(n + 1, 0);
    fv.feats.assign(cap, 0);
    int nw = 0, nfv = 0;
    check(gf_bow_transform(voc_, features.data.data(), n, levelsup, v.words.data(), v.values.data(), &nw,
                           fv.nodes.data(), fv.start.data(), fv.feats.data(), &nfv));
    v.words.resize(nw);
    v.values.resize(nw);
    fv.nodes.resize(nfv);
    fv.start.resize(nfv + 1);
    fv.feats.resize(fv.start[nfv]);
}

/* ---------------------------------------------------------------- ORBextractor */
ORBextractor::ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int scoreType_, int fastTh_)
    : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_), scoreType(scoreType_), fastTh(fastTh_) {}

ORBextractor::~ORBextractor() {
    if (ex_) gf_extractor_destroy(ex_);
}

void ORBextractor::operator()(const ImageView& image, std::vector<KeyPoint>& keypoints, Descriptors& descriptors) {
    keypoints.clear();
    descriptors.rows = 0;
    descriptors.data.clear();
    if (!image.data || image.cols == 0 || image.rows == 0) return;  // ORBextractor.cc:772-773
    if (!ex_ || image.cols != w_ || image.rows != h_) {
        if (ex_) gf_extractor_destroy(ex_);
        ex_ = nullptr;
        check(gf_extractor_create(Context(), nfeatures, (float)scaleFactor, nlevels, scoreType, fastTh, image.cols,
                                  image.rows, 1, &ex_));
        w_ = image.cols;
        h_ = image.rows;
    }
    int cap = 0, n = 0;
    check(gf_extractor_capacity(ex_, &cap));
    keypoints.resize(cap);
    descriptors.data.resize((size_t)cap * 32);
    check(gf_orb_extract(ex_, image.data, (int)image.step, reinterpret_cast<gf_keypoint*>(keypoints.data()),
                         descriptors.data.data(), cap, &n));
    keypoints.resize(n);
    descriptors.data.resize((size_t)n * 32);
    descriptors.rows = n;
}

/* ---------------------------------------------------------------- Frame */
Frame::Frame(const ImageView& im, double timeStamp, ORBextractor* extractor, const float K[4])
    : mTimeStamp(timeStamp), fx(K[0]), fy(K[1]), cx(K[2]), cy(K[3]) {
    static long unsigned int nNextId = 0;
    mnId = nNextId++;
    (*extractor)(im, mvKeys, mDescriptors);
    mvKeysUn = mvKeys;  // k1 == 0: UndistortKeyPoints copies (Frame.cc:391-395)
    N = (int)mvKeys.size();
    mvpMapPoints.assign(N, nullptr);
    mvpMatchScore.assign(N, 999);
    mvbOutlier.assign(N, false);
    mnMinX = 0;
    mnMaxX = im.cols;
    mnMinY = 0;
    mnMaxY = im.rows;
    mnScaleLevels = extractor->GetLevels();
    mfScaleFactor = extractor->GetScaleFactor();
    mvScaleFactors.assign(mnScaleLevels, 1.0f);
    for (int i = 1; i < mnScaleLevels; i++) mvScaleFactors[i] = mvScaleFactors[i - 1] * mfScaleFactor;
    mvLevelSigma2.resize(mnScaleLevels);
    mvInvLevelSigma2.resize(mnScaleLevels);
    for (int i = 0; i < mnScaleLevels; i++) {
        mvLevelSigma2[i] = mvScaleFactors[i] * mvScaleFactors[i];
        mvInvLevelSigma2[i] = 1.0f / mvLevelSigma2[i];
    }
}

void Frame::ComputeBoW() {
    if (!mpORBvocabulary) throw GpuError(GF_ERR_ARG, "Frame::ComputeBoW without a vocabulary");
    if (mBowVec.words.empty()) mpORBvocabulary->transform(mDescriptors, mBowVec, mFeatVec, 4);
}

KeyFrame::KeyFrame(const Frame& F)
    : mnFrameId(F.mnId), N(F.N), mvKeysUn(F.mvKeysUn), mDescriptors(F.mDescriptors), mBowVec(F.mBowVec),
      mFeatVec(F.mFeatVec), mvpMapPoints(F.mvpMapPoints) {
    static long unsigned int nNextId = 0;
    mnId = nNextId++;
}

gf_frame_info Frame::info() const {
    gf_frame_info fi;
    fi.min_x = mnMinX;
    fi.max_x = mnMaxX;
    fi.min_y = mnMinY;
    fi.max_y = mnMaxY;
    fi.fx = fx;
    fi.fy = fy;
    fi.cx = cx;
    fi.cy = cy;
    fi.nlevels = mnScaleLevels;
    fi.scale_factor = mfScaleFactor;
    return fi;
}

void Frame::getTwc(float Twc[16]) const {
    for (int i = 0; i < 16; i++) Twc[i] = (i % 5 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Twc[4 * i + j] = mTcw[4 * j + i];
        const float a = -mTcw[i] * mTcw[3], b = -mTcw[4 + i] * mTcw[7], c = -mTcw[8 + i] * mTcw[11];
        Twc[4 * i + 3] = (a + b) + c;
    }
}

int Frame::isInFrustum(const std::vector<MapPoint*>& vpMapPoints, float viewingCosLimit) {
    const int m = (int)vpMapPoints.size();
    if (m == 0) return 0;
    std::vector<gf_map_point> mps(m);
    for (int i = 0; i < m; i++) mps[i] = to_abi(*vpMapPoints[i]);
    std::vector<gf_mp_view> views(m);
    const gf_frame_info fi = info();
    int nin = 0;
    check(gf_frustum(Context(), &fi, mTcw, mps.data(), m, viewingCosLimit, views.data(), &nin));
    for (int i = 0; i < m; i++) {
        MapPoint* p = vpMapPoints[i];
        p->mbTrackInView = views[i].in_view != 0;
        if (p->mbTrackInView) {
            p->mTrackProjX = views[i].u;
            p->mTrackProjY = views[i].v;
            p->mnTrackScaleLevel = views[i].level;
            p->mTrackViewCos = views[i].view_cos;
        }
    }
    return nin;
}

bool Frame::isInFrustum(MapPoint* pMP, float viewingCosLimit) {
    return isInFrustum(std::vector<MapPoint*>{pMP}, viewingCosLimit) == 1;
}

/* ---------------------------------------------------------------- ORBmatcher */
int ORBmatcher::DescriptorDistance(const uint8_t* a, const uint8_t* b) {
    int32_t d = 0;
    check(gf_descriptor_distance(Context(), a, b, 1, &d));
    return d;
}

int ORBmatcher::SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, float th) {
    PointTable T;
    for (MapPoint* p : vpMapPoints) T.id(p);
    std::vector<int32_t> kp2mp(F.N), score(F.mvpMatchScore.begin(), F.mvpMatchScore.end());
    for (int i = 0; i < F.N; i++) kp2mp[i] = T.id(F.mvpMapPoints[i]);  // claims held by other points stay claims
    const int m = (int)T.ptrs.size();
    std::vector<gf_mp_view> views(m);
    std::vector<uint8_t> desc((size_t)m * 32);
    for (int i = 0; i < m; i++) {
        views[i] = view_of(T.ptrs[i]);
        if (i >= (int)vpMapPoints.size()) views[i].in_view = 0;  // not in the searched list
        std::memcpy(&desc[32 * (size_t)i], T.ptrs[i]->mDescriptor, 32);
    }
    const gf_frame_info fi = F.info();
    int n = 0;
    check(gf_match_project(Context(), &fi, reinterpret_cast<const gf_keypoint*>(F.mvKeysUn.data()),
                           F.mDescriptors.data.data(), F.N, views.data(), desc.data(), m, th, mfNNratio,
                           kp2mp.data(), score.data(), &n));
    for (int i = 0; i < F.N; i++) {
        F.mvpMapPoints[i] = kp2mp[i] >= 0 ? T.ptrs[kp2mp[i]] : nullptr;
        F.mvpMatchScore[i] = score[i];
    }
    return n;
}

int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, float th) {
    PointTable T;
    const int nl = LastFrame.N;
    std::vector<int32_t> last_kp2mp(nl);
    std::vector<uint8_t> last_out(nl);
    std::vector<float> last_pos((size_t)nl * 3, 0.f);
    for (int i = 0; i < nl; i++) {
        MapPoint* p = LastFrame.mvpMapPoints[i];
        last_kp2mp[i] = T.id(p);
        last_out[i] = LastFrame.mvbOutlier[i];
        if (p) p->GetWorldPos(&last_pos[3 * (size_t)i]);
    }
    std::vector<int32_t> kp2mp(CurrentFrame.N), score(CurrentFrame.mvpMatchScore.begin(),
                                                      CurrentFrame.mvpMatchScore.end());
    for (int i = 0; i < CurrentFrame.N; i++) kp2mp[i] = T.id(CurrentFrame.mvpMapPoints[i]);
    const gf_frame_info fi = CurrentFrame.info();
    int n = 0;
    check(gf_match_lastframe(Context(), &fi, reinterpret_cast<const gf_keypoint*>(CurrentFrame.mvKeysUn.data()),
                             CurrentFrame.mDescriptors.data.data(), CurrentFrame.N, CurrentFrame.mTcw,
                             reinterpret_cast<const gf_keypoint*>(LastFrame.mvKeysUn.data()),
                             LastFrame.mDescriptors.data.data(), last_kp2mp.data(), last_out.data(),
                             last_pos.data(), nl, th, mbCheckOrientation ? 1 : 0, kp2mp.data(), score.data(), &n));
    for (int i = 0; i < CurrentFrame.N; i++) {
        CurrentFrame.mvpMapPoints[i] = kp2mp[i] >= 0 ? T.ptrs[kp2mp[i]] : nullptr;
        CurrentFrame.mvpMatchScore[i] = score[i];
    }
    return n;
}

int ORBmatcher::SearchByProjection_OnePoint(Frame& F, MapPoint* pMP, const float th) {
    if (!pMP || !pMP->mbTrackInView || pMP->isBad()) return -1;  // ORBmatcher.h:75-79
    PointTable T;
    T.id(pMP);
    std::vector<int32_t> kp2mp(F.N), score(F.mvpMatchScore.begin(), F.mvpMatchScore.end());
    for (int i = 0; i < F.N; i++) kp2mp[i] = T.id(F.mvpMapPoints[i]);
    const int m = (int)T.ptrs.size();
    std::vector<gf_mp_view> views(m);
    std::vector<uint8_t> desc((size_t)m * 32);
    for (int i = 0; i < m; i++) {
        views[i] = view_of(T.ptrs[i]);
        if (i > 0) views[i].in_view = 0;  // only pMP is searched
        std::memcpy(&desc[32 * (size_t)i], T.ptrs[i]->mDescriptor, 32);
    }
    const gf_frame_info fi = F.info();
    int n = 0;
    check(gf_match_project(Context(), &fi, reinterpret_cast<const gf_keypoint*>(F.mvKeysUn.data()),
                           F.mDescriptors.data.data(), F.N, views.data(), desc.data(), m, th, mfNNratio, kp2mp.data(),
                           score.data(), &n));
    if (n == 0) return -1;
    for (int i = 0; i < F.N; i++)
        if (kp2mp[i] == 0 && F.mvpMapPoints[i] != pMP) {
            F.mvpMapPoints[i] = pMP;
            F.mvpMatchScore[i] = score[i];
            return i;
        }
    return -1;
}

int ORBmatcher::SearchByProjection_Budget(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th,
                                          const double time_constr) {
    if (time_constr <= 0) return 0;  // ORBmatcher.cc:281-282
    std::vector<MapPoint*> before(F.mvpMapPoints);
    const int n = SearchByProjection(F, vpMapPoints, th);
    for (int i = 0; i < F.N; i++)
        if (F.mvpMapPoints[i] && F.mvpMapPoints[i] != before[i]) F.mvpMapPoints[i]->IncreaseFound();  // :357
    return n;
}

namespace {
// One side of SearchByBoW: FeatureVector, descriptors, keypoints and the map
// point of each feature as an index into T (-1 = none or bad).
struct BowSide {
    std::vector<int32_t> mp;
    gf_bow_side side{};
    BowSide(const FeatureVector& fv, const Descriptors& d, const std::vector<KeyPoint>& kps,
            const std::vector<MapPoint*>* pts, PointTable& T) {
        const int n = (int)kps.size();
        mp.assign(std::max(n, 1), -1);
        if (pts)
            for (int i = 0; i < n; i++) {
                MapPoint* p = (*pts)[i];
                if (p && !p->isBad()) mp[i] = T.id(p);
            }
        side.fv_nodes = fv.nodes.data();
        side.fv_start = fv.start.data();
        side.fv_feats = fv.feats.data();
        side.nfv = (int32_t)fv.nodes.size();
        side.desc = d.data.data();
        side.kps = reinterpret_cast<const gf_keypoint*>(kps.data());
        side.mp = mp.data();
        side.n = n;
    }
};
}  // namespace

int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches) {
    if (!pKF) throw GpuError(GF_ERR_ARG, "null keyframe");
    PointTable T;
    BowSide a(pKF->mFeatVec, pKF->mDescriptors, pKF->mvKeysUn, &pKF->mvpMapPoints, T);
    BowSide b(F.mFeatVec, F.mDescriptors, F.mvKeysUn, nullptr, T);
    std::vector<int32_t> out(std::max(F.N, 1));
    int n = 0;
    check(gf_match_bow(Context(), 0, mfNNratio, mbCheckOrientation ? 1 : 0, &a.side, &b.side, out.data(), &n));
    vpMapPointMatches.assign(F.N, nullptr);  // ORBmatcher.cc:728
    for (int j = 0; j < F.N; j++)
        if (out[j] >= 0) vpMapPointMatches[j] = T.ptrs[out[j]];
    return n;
}

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12) {
    if (!pKF1 || !pKF2) throw GpuError(GF_ERR_ARG, "null keyframe");
    PointTable T;
    BowSide a(pKF1->mFeatVec, pKF1->mDescriptors, pKF1->mvKeysUn, &pKF1->mvpMapPoints, T);
    BowSide b(pKF2->mFeatVec, pKF2->mDescriptors, pKF2->mvKeysUn, &pKF2->mvpMapPoints, T);
    std::vector<int32_t> out(std::max(pKF1->N, 1));
    int n = 0;
    check(gf_match_bow(Context(), 1, mfNNratio, mbCheckOrientation ? 1 : 0, &a.side, &b.side, out.data(), &n));
    vpMatches12.assign(pKF1->N, nullptr);  // :1303
    for (int i = 0; i < pKF1->N; i++)
        if (out[i] >= 0) vpMatches12[i] = T.ptrs[out[i]];
    return n;
}

/* ---------------------------------------------------------------- Observability */
Observability::Observability(double fu, double fv, int nRows, int nCols, double cx, double cy, double, double) {
    camera.fu = fu;
    camera.fv = fv;
    camera.cx = cx;
    camera.cy = cy;
    camera.nrows = nRows;
    camera.ncols = nCols;
    camera.min_x = 0;
    camera.max_x = nCols;
    camera.min_y = 0;
    camera.max_y = nRows;
    gf_rng_seed(&rng_, 1);  // glibc: rand() without srand() behaves as srand(1)
    mNumThreads = std::max(1u, std::thread::hardware_concurrency());  // Observability.h:186
}

gf_obs_camera Observability::cam_now() const {
    gf_obs_camera c = camera;
    if (pFrame) {
        c.min_x = pFrame->mnMinX;
        c.max_x = pFrame->mnMaxX;
        c.min_y = pFrame->mnMinY;
        c.max_y = pFrame->mnMaxY;
    }
    c.bound_x = mBoundXInFrame;
    c.bound_y = mBoundYInFrame;
    c.bound_depth = mBoundDepth;
    return c;
}

void Observability::srand(unsigned seed) { gf_rng_seed(&rng_, seed); }

void Observability::updatePWLSVec(double time_prev, const float Tcw_prev[16], double time_cur,
                                  const float Twc_cur[16]) {
    check(gf_obs_update(time_prev, Tcw_prev, time_cur, Twc_cur, Xv));
}

void Observability::predictPWLSVec(double dt, size_t num_seg_pred) {
    kinematic.resize(num_seg_pred);
    check(gf_obs_predict(Xv, dt, (int)num_seg_pred, kinematic.data()));
}

bool Observability::runMatrixBuilding(size_t mat_type, double, bool, bool check_viz) {
    if (mKineIdx >= kinematic.size()) return false;
    const gf_obs_camera cam = cam_now();
    const double* xv = kinematic[mKineIdx].Xv;
    std::vector<MapPoint*> pts;
    std::vector<float> pos, sigma2;
    std::vector<int> kp;
    if (mat_type == FRAME_INFO_MATRIX) {  // batchInfoMat_Frame (Observability.cc:386-554)
        if (!pFrame) return false;
        for (int i = 0; i < pFrame->N; i++) {
            MapPoint* p = pFrame->mvpMapPoints[i];
            if (!p) continue;
            if (pFrame->mvbOutlier[i]) {
                p->ObsScore = -1.0;
                continue;
            }
            pts.push_back(p);
            kp.push_back(i);
            sigma2.push_back(pFrame->mvLevelSigma2[pFrame->mvKeysUn[i].octave]);
        }
    } else if (mat_type == MAP_INFO_MATRIX) {  // batchInfoMat_Map (Observability.cc:556-644)
        if (!mMapPoints) return false;
        for (MapPoint* p : *mMapPoints) {
            if (!p) continue;  // batchInfoMat_Map tests the pointer only (:584)
            if (p->updateAtFrameId == (long)mnFrameId) continue;
            if (!check_viz && !p->mbTrackInView) continue;
            pts.push_back(p);
        }
    } else {
        return false;
    }
    const int n = (int)pts.size();
    if (n == 0) return true;
    pos.resize(3 * (size_t)n);
    for (int i = 0; i < n; i++) pts[i]->GetWorldPos(&pos[3 * (size_t)i]);
    std::vector<double> H(14 * (size_t)n), info(49 * (size_t)n);
    std::vector<float> uv(2 * (size_t)n);
    std::vector<uint8_t> valid(n);
    const bool frame = mat_type == FRAME_INFO_MATRIX;
    check(gf_obs_build_info(Context(), &cam, xv, pos.data(), frame ? sigma2.data() : nullptr, n,
                            frame ? 0 : (check_viz ? 1 : 0), H.data(), info.data(), uv.data(), valid.data()));
    for (int i = 0; i < n; i++) {
        MapPoint* p = pts[i];
        if (!valid[i]) {
            p->ObsScore = -1.0;
            continue;
        }
        p->u_proj = uv[2 * i];
        p->v_proj = uv[2 * i + 1];
        std::memcpy(p->H_meas, &H[14 * (size_t)i], sizeof(p->H_meas));
        std::memcpy(p->ObsMat, &info[49 * (size_t)i], sizeof(p->ObsMat));
        p->hasObsMat = true;
        if (frame) {
            p->ObsScore = pFrame->mvpMatchScore[kp[i]];
        } else {
            p->ObsScore = 1.0;
            p->updateAtFrameId = (long)mnFrameId;
        }
    }
    return true;
}

int Observability::runActiveMapMatching(Frame* F, size_t, const double base[49], float th, ORBmatcher& matcher,
                                        int num_to_match, double) {
    if (!F || !mMapPoints) return 0;
    PointTable T;
    for (MapPoint* p : *mMapPoints) T.id(p);
    const int nlist = (int)T.ptrs.size();
    std::vector<int32_t> kp2mp(F->N), score(F->mvpMatchScore.begin(), F->mvpMatchScore.end());
    for (int i = 0; i < F->N; i++) kp2mp[i] = T.id(F->mvpMapPoints[i]);
    const int m = (int)T.ptrs.size();
    std::vector<gf_mp_view> views(m);
    std::vector<uint8_t> desc((size_t)m * 32), updated(m);
    std::vector<double> info((size_t)m * 49), H((size_t)m * 14);
    std::vector<float> uv((size_t)m * 2);
    for (int i = 0; i < m; i++) {
        const MapPoint* p = T.ptrs[i];
        views[i] = view_of(p);
        if (i >= nlist) views[i].in_view = 0;
        updated[i] = p->updateAtFrameId == (long)F->mnId;
        std::memcpy(&desc[32 * (size_t)i], p->mDescriptor, 32);
        std::memcpy(&info[49 * (size_t)i], p->ObsMat, sizeof(p->ObsMat));
        std::memcpy(&H[14 * (size_t)i], p->H_meas, sizeof(p->H_meas));
        uv[2 * i] = p->u_proj;
        uv[2 * i + 1] = p->v_proj;
    }
    std::vector<int32_t> left(std::max(m, 1));
    int nleft = 0, nmatched = 0;
    const gf_frame_info fi = F->info();
    check(gf_obs_active_match(Context(), &fi, reinterpret_cast<const gf_keypoint*>(F->mvKeysUn.data()),
                              F->mDescriptors.data.data(), F->N, views.data(), desc.data(), updated.data(),
                              info.data(), H.data(), uv.data(), m, base, F->mvLevelSigma2.data(), num_to_match, th,
                              matcher.mfNNratio, &rng_, kp2mp.data(), score.data(), left.data(), &nleft, &nmatched));
    for (int i = 0; i < F->N; i++) {
        F->mvpMapPoints[i] = kp2mp[i] >= 0 ? T.ptrs[kp2mp[i]] : nullptr;
        F->mvpMatchScore[i] = score[i];
    }
    for (int i = 0; i < nleft; i++) mLeftMapPoints.push_back(T.ptrs[left[i]]);
    return nmatched;
}

bool Observability::setSelction_Number(size_t num_good_inlier, int greedy_mtd, double time_for_select,
                                       std::vector<MapPoint*>* mapPoints, std::vector<GoodPoint>* mpVec) {
    if (!mapPoints || !mpVec || time_for_select <= 0) return false;  // Observability.cc:1026-1027
    if (kinematic.size() < 2) return false;
    mKineIdx = 1;
    mMapPoints = mapPoints;
    // MAP_INFO_MATRIX with the visibility check (:1039 -> batchInfoMat_Map
    // :556-644): points updated this frame keep their blocks and scores, the
    // others are rebuilt at kinematic[1] (ObsScore 1, stamped) or, not
    // visible, get ObsScore -1
    runMatrixBuilding(MAP_INFO_MATRIX, time_for_select / 2.0, true, true);
    // lmkSelectPool: ObsScore >= 0 with a block, in list order (:1046-1058)
    std::vector<size_t> pidx;
    std::vector<double> pinfo, pscore;
    for (size_t i = 0; i < mapPoints->size(); i++) {
        const MapPoint* p = (*mapPoints)[i];
        if (!p || !(p->ObsScore >= 0) || !p->hasObsMat) continue;
        pidx.push_back(i);
        pinfo.insert(pinfo.end(), p->ObsMat, p->ObsMat + 49);
        pscore.push_back(p->ObsScore);
    }
    mpVec->clear();
    const int n = (int)pidx.size();
    if (n == 0) return true;
    std::vector<int32_t> out(n);
    int nout = 0;
    check(gf_select_pool(Context(), pinfo.data(), pscore.data(), n, (int)num_good_inlier, greedy_mtd,
                         (int)mNumThreads, &rng_, out.data(), &nout));
    for (int j = 0; j < nout; j++) {
        GoodPoint g;
        g.idx = pidx[out[j]];
        g.obs_score = pscore[out[j]];
        std::memcpy(g.obs_block.data(), &pinfo[49 * (size_t)out[j]], sizeof(double) * 49);
        mpVec->push_back(g);
    }
    return true;
}

std::vector<int> Observability::maxVolSelection(const std::vector<std::array<double, 49>>& pool,
                                                const std::vector<double>& score, int k, double sample_scale,
                                                int mode) {
    const int n = (int)pool.size();
    std::vector<int> out(std::max(n, 1));
    int nout = 0;
    if (n == 0) return {};
    check(gf_maxvol_select(Context(), pool[0].data(), score.data(), n, k, sample_scale, mode, &rng_, out.data(),
                           &nout));
    out.resize(nout);
    return out;
}

/* ---------------------------------------------------------------- Optimizer */
int Optimizer::PoseOptimization(Frame* pFrame) {
    std::vector<gf_pose_edge> edges;
    std::vector<int> idx;
    for (int i = 0; i < pFrame->N; i++) {
        MapPoint* p = pFrame->mvpMapPoints[i];
        if (!p) continue;
        gf_pose_edge e;
        p->GetWorldPos(e.X);
        e.z[0] = pFrame->mvKeysUn[i].pt.x;
        e.z[1] = pFrame->mvKeysUn[i].pt.y;
        e.inv_sigma2 = pFrame->mvInvLevelSigma2[pFrame->mvKeysUn[i].octave];
        edges.push_back(e);
        idx.push_back(i);
    }
    const int n = (int)edges.size();
    std::vector<uint8_t> outl(std::max(n, 1));
    int32_t ninl = 0;
    float Tout[16];
    check(gf_pose_opt(Context(), pFrame->mTcw, n ? edges.data() : nullptr, n, pFrame->fx, pFrame->fy, pFrame->cx,
                      pFrame->cy, Tout, outl.data(), &ninl, nullptr));
    std::memcpy(pFrame->mTcw, Tout, sizeof(Tout));
    for (int j = 0; j < n; j++) pFrame->mvbOutlier[idx[j]] = outl[j] != 0;
    return ninl;
}

void Optimizer::LocalBundleAdjustment(LocalBAWindow* w, bool* pbStopFlag) {
    if (!w) throw GpuError(GF_ERR_ARG, "null window");
    gf_ba_problem P{};
    P.nkf = (int32_t)w->kf_kind.size();
    P.npts = (int32_t)(w->pt_pos.size() / 3);
    P.nedges = (int32_t)w->edge_pt.size();
    if (w->kf_Tcw.size() != 16 * (size_t)P.nkf || w->kf_cam.size() != 4 * (size_t)P.nkf ||
        w->edge_kf.size() != (size_t)P.nedges || w->edge_z.size() != 2 * (size_t)P.nedges ||
        w->edge_inv_sigma2.size() != (size_t)P.nedges)
        throw GpuError(GF_ERR_ARG, "inconsistent local BA window");
    P.kf_Tcw = w->kf_Tcw.data();
    P.kf_kind = w->kf_kind.data();
    P.kf_cam = w->kf_cam.data();
    P.pt_pos = w->pt_pos.data();
    P.edge_pt = w->edge_pt.data();
    P.edge_kf = w->edge_kf.data();
    P.edge_z = w->edge_z.data();
    P.edge_inv_sigma2 = w->edge_inv_sigma2.data();
    std::vector<float> T(w->kf_Tcw.size()), X(w->pt_pos.size());
    w->edge_outlier.assign(P.nedges, 0);
    gf_ba_result R{};
    R.kf_Tcw = T.data();
    R.pt_pos = X.data();
    R.edge_outlier = w->edge_outlier.data();
    static_assert(sizeof(bool) == 1, "bool flag read as a byte");
    check(gf_local_ba_stop(Context(), &P, &R, reinterpret_cast<const volatile uint8_t*>(pbStopFlag)));
    w->kf_Tcw = T;
    w->pt_pos = X;
    w->iterations[0] = R.iterations[0];
    w->iterations[1] = R.iterations[1];
}

}  // namespace ORB_SLAM
