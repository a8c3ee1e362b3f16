/* C++ drop-in layer over the libgfslam C-ABI.
 *
 * Re-declares the reference classes on the hot path with the same names,
 * method names and argument meaning (namespace ORB_SLAM):
 *   ORBextractor            include/ORBextractor.h:47-70
 *   ORBmatcher              include/ORBmatcher.h:40-290 (M2, M3, OnePoint, Budget, SearchByBoW x2,
 *                           distance)
 *   Frame / KeyFrame /      include/Frame.h, include/KeyFrame.h, include/MapPoint.h (the fields
 *   MapPoint                the path reads/writes)
 *   ORBVocabulary           Thirdparty/DBoW2 TemplatedVocabulary (loaders, transform)
 *   Observability           include/Observability.h:165-741 (PWLS kinematics, matrix building,
 *                           active map matching, max-volume selection, setSelction_Number)
 *   Optimizer               include/Optimizer.h:53-54 (PoseOptimization, LocalBundleAdjustment)
 * OpenCV/Armadillo types are replaced by plain value types with the same
 * memory layout where one exists (KeyPoint == cv::KeyPoint, 28 B; Tcw is a
 * row-major float 4x4 like the CV_32F cv::Mat; matrices are row-major f64).
 * Every call forwards to the GPU through include/gfslam/abi.h; nothing here
 * computes on the host beyond packing.
 */
#ifndef GFSLAM_ORBSLAM_H
#define GFSLAM_ORBSLAM_H

#include <stdint.h>

#include <array>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "abi.h"

namespace ORB_SLAM {

/* ---------------------------------------------------------------- types */
struct Point2f {
    float x = 0, y = 0;
};
/* cv::KeyPoint layout (pt, size, angle, response, octave, class_id). */
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
static_assert(sizeof(KeyPoint) == sizeof(gf_keypoint), "KeyPoint must keep the cv::KeyPoint layout");

/* A CV_8UC1 image view (cv::Mat data/cols/rows/step). */
struct ImageView {
    const uint8_t* data = nullptr;
    int cols = 0, rows = 0;
    size_t step = 0;
};

/* N x 32 CV_8U descriptor matrix. */
struct Descriptors {
    int rows = 0;
    std::vector<uint8_t> data;
    const uint8_t* ptr(int r) const { return data.data() + 32 * (size_t)r; }
    uint8_t* ptr(int r) { return data.data() + 32 * (size_t)r; }
};

/* Thrown on any non-zero libgfslam status (the reference signals failure by
 * return values; the GPU layer adds device errors that have no such value). */
struct GpuError : std::runtime_error {
    int code;
    GpuError(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

/* The per-thread libgfslam context (one HIP stream), created on first use on
 * HIP device 0 or the one given to SetDevice before any other call. */
gf_ctx* Context();
void SetDevice(int device);

/* ---------------------------------------------------------------- MapPoint
 * The fields of ORB_SLAM::MapPoint the front end reads and writes. */
struct MapPoint {
    float mWorldPos[3] = {0, 0, 0};
    float mNormalVector[3] = {0, 0, 1};
    float mfMinDistance = 0, mfMaxDistance = 0;
    uint8_t mDescriptor[32] = {};
    bool mbBad = false;
    /* written by Frame::isInFrustum (Frame.cc:166-227) */
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackViewCos = 0;
    int mnTrackScaleLevel = 0;
    /* written by Observability (MapPoint.h: H_meas, ObsMat, u/v_proj, ...) */
    double H_meas[14] = {};
    double ObsMat[49] = {};
    bool hasObsMat = false; /* ObsMat.n_rows > 0 (an arma::mat set by a build) */
    float u_proj = 0, v_proj = 0;
    double ObsScore = 0;
    long updateAtFrameId = -1;
    /* tracking counters (MapPoint.cc:298-312) */
    int mnVisible = 1, mnFound = 1;

    bool isBad() const { return mbBad; }
    void GetWorldPos(float out[3]) const { std::memcpy(out, mWorldPos, sizeof(mWorldPos)); }
    void IncreaseVisible(int n = 1) { mnVisible += n; }
    void IncreaseFound(int n = 1) { mnFound += n; }
};

/* DBoW2 BowVector (word id -> weight) and FeatureVector (node id -> feature
 * indices) as sorted arrays: node i holds feats[start[i] .. start[i+1]). */
struct BowVector {
    std::vector<int32_t> words;
    std::vector<double> values;
};
struct FeatureVector {
    std::vector<int32_t> nodes, start{0}, feats;
};

/* ORBVocabulary = TemplatedVocabulary<FORB::TDescriptor, FORB>
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h), resident on the GPU. */
class ORBVocabulary {
public:
    ORBVocabulary() = default;
    ~ORBVocabulary();
    ORBVocabulary(const ORBVocabulary&) = delete;
    ORBVocabulary& operator=(const ORBVocabulary&) = delete;
    /* loadFromTextFile (:1352-1432) / loadFromBinaryFile (:1469-1510); false on failure */
    bool loadFromTextFile(const std::string& filename);
    bool loadFromBinaryFile(const std::string& filename);
    /* transform(features, BowVector, FeatureVector, levelsup) (:1141-1270) */
    void transform(const struct Descriptors& features, BowVector& v, FeatureVector& fv, int levelsup) const;
    gf_vocab* handle() const { return voc_; }

private:
    gf_vocab* voc_ = nullptr;
};

class ORBextractor;

/* ---------------------------------------------------------------- Frame */
class Frame {
public:
    Frame() = default;
    /* Frame::Frame(im, timeStamp, extractor, K, distCoef) (Frame.cc:40-137)
     * with k1 == 0 (undistortion bypassed: mvKeysUn == mvKeys). K = fx fy cx cy. */
    Frame(const ImageView& im, double timeStamp, ORBextractor* extractor, const float K[4]);

    long unsigned int mnId = 0;
    double mTimeStamp = 0;
    float fx = 0, fy = 0, cx = 0, cy = 0;
    int mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0;
    int N = 0;
    std::vector<KeyPoint> mvKeys, mvKeysUn;
    Descriptors mDescriptors;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<int> mvpMatchScore;
    std::vector<bool> mvbOutlier;
    float mTcw[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    int mnScaleLevels = 8;
    float mfScaleFactor = 1.2f;
    std::vector<float> mvScaleFactors, mvLevelSigma2, mvInvLevelSigma2;

    /* Frame::ComputeBoW (Frame.cc:380-387): transform with levelsup 4 */
    ORBVocabulary* mpORBvocabulary = nullptr;
    BowVector mBowVec;
    FeatureVector mFeatVec;
    void ComputeBoW();

    void SetPose(const float Tcw[16]) { std::memcpy(mTcw, Tcw, sizeof(mTcw)); }
    /* Frame::getTwc (Frame.cc:152-163) */
    void getTwc(float Twc[16]) const;
    /* Frame::isInFrustum for one point (Frame.cc:166-227). */
    bool isInFrustum(MapPoint* pMP, float viewingCosLimit);
    /* The same test for a whole list in one GPU call; returns the number in view. */
    int isInFrustum(const std::vector<MapPoint*>& vpMapPoints, float viewingCosLimit);

    gf_frame_info info() const;
};

/* ---------------------------------------------------------------- KeyFrame
 * The fields of ORB_SLAM::KeyFrame that SearchByBoW reads: built from a
 * Frame as KeyFrame::KeyFrame(Frame&, Map*, KeyFrameDatabase*) copies them
 * (KeyFrame.cc:31-58). */
class KeyFrame {
public:
    explicit KeyFrame(const Frame& F);
    long unsigned int mnId = 0, mnFrameId = 0;
    int N = 0;
    std::vector<KeyPoint> mvKeysUn;
    Descriptors mDescriptors;
    BowVector mBowVec;
    FeatureVector mFeatVec;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<MapPoint*> GetMapPointMatches() const { return mvpMapPoints; }
    MapPoint* GetMapPoint(size_t idx) const { return mvpMapPoints[idx]; }
};

/* ---------------------------------------------------------------- ORBextractor */
class ORBextractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };
    ORBextractor(int nfeatures = 1000, float scaleFactor = 1.2f, int nlevels = 8, int scoreType = FAST_SCORE,
                 int fastTh = 20);
    ~ORBextractor();
    ORBextractor(const ORBextractor&) = delete;
    ORBextractor& operator=(const ORBextractor&) = delete;

    /* operator()(image, mask, keypoints, descriptors) (ORBextractor.cc:769-875).
     * The reference builds mvMaskPyramid from a mask (:929-993) but never hands
     * cellMask to FAST (:614-621), so a mask does not change the outputs: the
     * overload with a mask takes it and extracts as without one. */
    void operator()(const ImageView& image, std::vector<KeyPoint>& keypoints, Descriptors& descriptors);
    void operator()(const ImageView& image, const ImageView& mask, std::vector<KeyPoint>& keypoints,
                    Descriptors& descriptors) {
        (void)mask;
        operator()(image, keypoints, descriptors);
    }

    int GetLevels() const { return nlevels; }
    float GetScaleFactor() const { return (float)scaleFactor; }

protected:
    int nfeatures;
    double scaleFactor;
    int nlevels;
    int scoreType;
    int fastTh;
    gf_extractor* ex_ = nullptr;
    int w_ = 0, h_ = 0;
};

/* ---------------------------------------------------------------- ORBmatcher */
class ORBmatcher {
public:
    static const int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;
    ORBmatcher(float nnratio = 0.6f, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

    /* ORBmatcher::DescriptorDistance (ORBmatcher.cc:2384-2400) */
    static int DescriptorDistance(const uint8_t* a, const uint8_t* b);
    /* SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:384-465);
     * reads the isInFrustum state of each point. */
    int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, float th = 3);
    /* SearchByProjection(Frame& Cur, const Frame& Last, th) (ORBmatcher.cc:2081-2202) */
    int SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, float th);
    /* SearchByProjection_OnePoint(F, pMP, th) (ORBmatcher.h:71-145): the keypoint
     * index pMP claims in F (F.mvpMapPoints / mvpMatchScore written) or -1. */
    int SearchByProjection_OnePoint(Frame& F, MapPoint* pMP, const float th);
    /* SearchByProjection_Budget(F, vpMapPoints, th, time_constr)
     * (ORBmatcher.cc:276-379): M2 over the list in order with IncreaseFound on
     * every match. time_constr <= 0 returns 0 at once (:281-282); otherwise the
     * list is matched in one GPU call (microseconds), so the per-point wall-clock
     * cut of :366-371 is not reached. */
    int SearchByProjection_Budget(Frame& F, const std::vector<MapPoint*>& vpMapPoints, const float th,
                                  const double time_constr);
    /* SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) (ORBmatcher.cc:724-853):
     * vpMapPointMatches[j] = the keyframe's map point matched to F's feature j.
     * Needs both FeatureVectors (ComputeBoW). Returns the match count. */
    int SearchByBoW(KeyFrame* pKF, Frame& F, std::vector<MapPoint*>& vpMapPointMatches);
    /* SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vpMatches12) (:1289-1424):
     * vpMatches12[i] = pKF2's map point matched to pKF1's feature i. */
    int SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, std::vector<MapPoint*>& vpMatches12);

    float mfNNratio;
    bool mbCheckOrientation;
};

/* ---------------------------------------------------------------- Observability */
enum { FRAME_INFO_MATRIX = 0, MAP_INFO_MATRIX = 1 };

/* GoodPoint (Util.hpp:65-129): a selected map point, idx into the list given
 * to setSelction_Number; obs_block is the 7x7 ObsMat row-major. */
struct GoodPoint {
    size_t idx = 0;
    double obs_score = 0;
    bool selected = false;
    std::array<double, 49> obs_block{};
};

class Observability {
public:
    /* Observability(fu, fv, nRows, nCols, cx, cy, k1, k2) (Observability.h:165-206) */
    Observability(double fu, double fv, int nRows, int nCols, double cx, double cy, double k1, double k2);

    /* updatePWLSVec / predictPWLSVec (Observability.h:222-295); poses row-major float 4x4 */
    void updatePWLSVec(double time_prev, const float Tcw_prev[16], double time_cur, const float Twc_cur[16]);
    void predictPWLSVec(double dt, size_t num_seg_pred);

    /* runMatrixBuilding (Observability.cc:646-804), FRAME_INFO_MATRIX over
     * pFrame->mvpMapPoints or MAP_INFO_MATRIX over *mMapPoints; time caps
     * and thread counts are accepted and ignored (one GPU call). */
    bool runMatrixBuilding(size_t mat_type, double time_for_build, bool with_multi_thread, bool check_viz = false);

    /* runActiveMapMatching (Observability.cc:1249-1524) with FRAME_INFO_MATRIX;
     * mBaseInfoMat is 7x7 row-major; fills mLeftMapPoints. */
    int runActiveMapMatching(Frame* pFrame, size_t mat_type, const double mBaseInfoMat[49], float th,
                             ORBmatcher& matcher, int num_to_match, double time_for_match);

    /* maxVol*_LazierGreedy / BaselineGreedy over a pool of 7x7 blocks
     * (Observability.cc:2815-3155); mode 1 baseline, 2 lazier, 3 automatic. */
    std::vector<int> maxVolSelection(const std::vector<std::array<double, 49>>& pool,
                                     const std::vector<double>& score, int k, double sample_scale, int mode);

    /* setSelction_Number(num_good_inlier, greedy_mtd, time_for_select,
     * mapPoints, mpVec) (Observability.cc:1021-1247): MAP_INFO_MATRIX with the
     * visibility check at kinematic[1] (mKineIdx = 1) over *mapPoints, then
     * greedy_mtd 1 BaselineGreedy / 2 LazierGreedy / 3 automatic lazier greedy
     * with the reference's multi-thread split (sample scale 6). mpVec = the
     * selection in order. Null / bad points take no part. false when
     * time_for_select <= 0, mapPoints or mpVec is null, or predictPWLSVec has
     * not produced kinematic[1]. The time budget is otherwise not applied. */
    bool setSelction_Number(size_t num_good_inlier, int greedy_mtd, double time_for_select,
                            std::vector<MapPoint*>* mapPoints, std::vector<GoodPoint>* mpVec);

    /* std::srand for the lazier-greedy draws (the reference seeds once). */
    void srand(unsigned seed);

    gf_obs_camera camera{};
    int mBoundXInFrame = 20, mBoundYInFrame = 20;
    float mBoundDepth = 0;
    long unsigned int mnFrameId = 0;
    size_t mKineIdx = 0;
    double Xv[13] = {};
    std::vector<gf_kine> kinematic;
    std::vector<MapPoint*>* mMapPoints = nullptr;
    std::vector<MapPoint*> mLeftMapPoints;
    Frame* pFrame = nullptr;
    bool mbNeedVizCheck = false;
    /* std::thread::hardware_concurrency() (Observability.h:186): the thread
     * count of setSelction_Number's greedy split */
    size_t mNumThreads = 1;

private:
    gf_rng rng_{};
    gf_obs_camera cam_now() const;
};

/* ---------------------------------------------------------------- Optimizer */
class Optimizer {
public:
    /* Optimizer::PoseOptimization(Frame*) (Optimizer.cc:279-413): updates
     * pFrame->mTcw and mvbOutlier of the matched keypoints, returns the
     * number of inliers. */
    static int PoseOptimization(Frame* pFrame);

    /* Optimizer::LocalBundleAdjustment(KeyFrame* pKF, bool* pbStopFlag)
     * (Optimizer.cc:1515-1764). The local window the reference collects from
     * pKF's covisibility graph (:1518-1566) is passed as a LocalBAWindow in
     * the reference's vertex and edge orders (gf_ba_problem); the optimised
     * poses and points and the outlier flags come back in the same window.
     * *pbStopFlag (LocalMapping::mbAbortBA) is polled between iterations. */
    struct LocalBAWindow {
        std::vector<float> kf_Tcw;        /* nkf x 16 (in / out) */
        std::vector<uint8_t> kf_kind;     /* 0 local, 1 local fixed (mnId 0), 2 fixed camera */
        std::vector<float> kf_cam;        /* nkf x 4: fx fy cx cy */
        std::vector<float> pt_pos;        /* npts x 3 (in / out) */
        std::vector<int32_t> edge_pt, edge_kf;
        std::vector<float> edge_z;        /* nedges x 2 */
        std::vector<float> edge_inv_sigma2;
        std::vector<uint8_t> edge_outlier; /* out: 1 removed after optimize(5), 2 after optimize(10) */
        int iterations[2] = {0, 0};
    };
    static void LocalBundleAdjustment(LocalBAWindow* pWindow, bool* pbStopFlag);
};

}  // namespace ORB_SLAM

#endif /* GFSLAM_ORBSLAM_H */
