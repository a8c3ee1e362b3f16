/*
 * gfslam C-ABI — the drop-in boundary of the MI355X GF-ORB-SLAM front end.
 *
 * Every entry point is extern "C", takes plain pointers and sizes, returns an
 * int status (GF_OK = 0, negative = error; no exceptions cross the ABI) and
 * replaces one reference C++ operator (file:line cited per function, paths
 * relative to the reference tree Aidenryan/GF_ORB_SLAM). Two families:
 *
 *   host family   (gf_orb_extract, gf_match_project, ...): host buffers in and
 *                 out, synchronous; what a cgo/ctypes/C++ caller binds.
 *   device family (*_dev): device pointers + a hipStream_t passed as void*,
 *                 asynchronous, batched over independent frames; what the
 *                 throughput path (bench.py) and in-process pipelines use.
 *
 * Error behaviour mirrors the reference: empty inputs give empty outputs
 * (ORBextractor.cc:772 returns on an empty image, matchers return 0 matches).
 */
#ifndef GFSLAM_ABI_H
#define GFSLAM_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    GF_OK = 0,
    GF_ERR_ARG = -1,          /* bad argument (null pointer, size mismatch)     */
    GF_ERR_HIP = -2,          /* HIP runtime error (message in gf_last_error)  */
    GF_ERR_CAP = -3,          /* output capacity too small (n_out holds need)  */
    GF_ERR_UNSUPPORTED = -4,  /* option the build does not implement           */
    GF_ERR_NODEV = -5         /* no HIP device                                 */
};

/* cv::KeyPoint memory layout (28 B): pt.x, pt.y, size, angle, response,
 * octave, class_id. */
typedef struct gf_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} gf_keypoint;

typedef struct gf_ctx gf_ctx;
typedef struct gf_extractor gf_extractor;

/* ---------------------------------------------------------------- runtime */
int gf_version(void);
const char* gf_last_error(void);
int gf_device_count(int* n);
/* One context per host thread: owns one HIP stream on `hip_device`. */
int gf_ctx_create(int hip_device, gf_ctx** out);
int gf_ctx_destroy(gf_ctx* ctx);
int gf_ctx_stream(gf_ctx* ctx, void** stream);
int gf_ctx_sync(gf_ctx* ctx);
/* Per-kernel timing with HIP events recorded on each launch's own stream
 * (what bench.py reports the roofline from). gf_prof_report returns, for
 * entry idx, the kernel name, summed device time and launch count. */
int gf_prof_enable(gf_ctx* ctx, int on);
int gf_prof_reset(gf_ctx* ctx);
int gf_prof_report(gf_ctx* ctx, int idx, char* name, int name_cap, double* total_ms, int* launches);

/* ------------------------------------------------------- ORB extraction (E1-E8)
 * Replaces ORB_SLAM::ORBextractor (include/ORBextractor.h:57-70,
 * src/ORBextractor.cc:464-998): ctor(nfeatures, scaleFactor, nlevels,
 * scoreType, fastTh) and operator()(image, mask=empty, keypoints, descriptors).
 * The geometry (width x height) is fixed at creation: the pyramid, cell grids
 * and per-level quotas are planned once. score_type: FAST_SCORE (1) or HARRIS_SCORE (0);
 * any other value returns GF_ERR_ARG. max_batch bounds nframes of the
 * batched device call. */
int gf_extractor_create(gf_ctx* ctx, int nfeatures, float scale_factor, int nlevels,
                        int score_type, int fast_th, int width, int height, int max_batch,
                        gf_extractor** out);
int gf_extractor_destroy(gf_extractor* ex);
/* GetLevels()/GetScaleFactor() (ORBextractor.h:66-70) + the per-level
 * feature quotas mnFeaturesPerLevel (ORBextractor.cc:483-494). */
int gf_extractor_info(gf_extractor* ex, int* nlevels, float* scale_factor,
                      int* features_per_level /* [nlevels] or NULL */);
/* Max keypoints one frame can return (sum of level quotas). */
int gf_extractor_capacity(gf_extractor* ex, int* cap);

/* Host family: img is width x height u8 with row stride `stride`; writes up to
 * `cap` keypoints (28 B each) and descriptors (32 B rows). An empty image
 * (width/height 0) returns n_out = 0. */
int gf_orb_extract(gf_extractor* ex, const uint8_t* img, int stride, gf_keypoint* kps,
                   uint8_t* desc, int cap, int* n_out);

/* Device family: nframes images at d_imgs + f*frame_stride (row stride
 * `stride`), outputs at d_kps[f*cap + i], d_desc[(f*cap + i)*32] and
 * d_counts[f]; cap must be >= gf_extractor_capacity. Asynchronous on stream. */
int gf_orb_extract_batch_dev(gf_extractor* ex, int nframes, const uint8_t* d_imgs,
                             size_t frame_stride, int stride, gf_keypoint* d_kps,
                             uint8_t* d_desc, int32_t* d_counts, int cap, void* stream);

/* Pointer-table form of gf_orb_extract_batch_dev: level 0 of frame f is the
 * width x height image at d_img_ptrs[f] (a device array of device pointers,
 * row stride `stride`), so frames can come from anywhere in HBM (a sequence
 * ring, a staging buffer) without a gather copy. */
int gf_orb_extract_ptrs_dev(gf_extractor* ex, int nframes, const uint8_t* const* d_img_ptrs, int stride,
                            gf_keypoint* d_kps, uint8_t* d_desc, int32_t* d_counts, int cap, void* stream);

/* Debug/parity hook: copies one intermediate plane of frame f of the last
 * batch to host. which: 0 = pyramid level (unblurred, ComputePyramid
 * ORBextractor.cc:922-998), 1 = blurred level interior (GaussianBlur :842).
 * out must hold w*h bytes of that level; (w,h) returned. */
int gf_extractor_debug_level(gf_extractor* ex, int frame, int level, int which, uint8_t* out,
                             int* w, int* h);

/* ------------------------------------------------------ matching (E8, M1-M5, M7)
 * Frame view (include/Frame.h:44-150): keypoints mvKeysUn (== mvKeys when
 * k1 == 0, Frame.cc:391-395), descriptors, undistorted image bounds
 * mnMinX..mnMaxY (Frame.cc:470-476), intrinsics, scale pyramid. The 64x48
 * keypoint grid (Frame.cc:100-131) is built on the device per call. */
typedef struct gf_frame_info {
    int32_t min_x, max_x, min_y, max_y;
    float fx, fy, cx, cy;
    int32_t nlevels;
    float scale_factor; /* mvScaleFactors[l] = scale_factor^l (float products) */
} gf_frame_info;

/* MapPoint state used by the tracker (include/MapPoint.h): world position,
 * mean viewing direction, scale-invariance distances mfMinDistance /
 * mfMaxDistance (MapPoint.cc:326-336). Descriptors travel separately (32 B). */
typedef struct gf_map_point {
    float pos[3];
    float normal[3];
    float min_dist, max_dist;
} gf_map_point;

/* Projection state Frame::isInFrustum writes into a MapPoint
 * (Frame.cc:216-222): mTrackProjX/Y, mTrackViewCos, mnTrackScaleLevel,
 * mbTrackInView (in_view = mbTrackInView && !isBad()). */
typedef struct gf_mp_view {
    float u, v, view_cos;
    int32_t level;
    int32_t in_view;
} gf_mp_view;

/* Frame::isInFrustum(pMP, viewingCosLimit), Frame.cc:166-227, for m map
 * points at pose Tcw (row-major 4x4 float). */
int gf_frustum(gf_ctx* ctx, const gf_frame_info* fi, const float* Tcw, const gf_map_point* mps, int m,
               float view_cos_limit, gf_mp_view* views, int* n_in_view);

/* ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>&, th),
 * ORBmatcher.cc:384-465 (M2; with RadiusByViewingCos :696-702,
 * Frame::GetFeaturesInArea Frame.cc:300-365). Map points are processed in
 * list order; a keypoint already claimed (kp2mp[i] >= 0 on entry, or by an
 * earlier map point) is skipped, exactly as F.mvpMapPoints[idx] != NULL.
 * kp2mp/score are in/out (mvpMapPoints / mvpMatchScore, index of the map
 * point in `views`); nmatches = new matches. */
int gf_match_project(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                     const gf_mp_view* views, const uint8_t* mp_desc, int m, float th, float nnratio,
                     int32_t* kp2mp, int32_t* score, int* nmatches);

/* ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th),
 * ORBmatcher.cc:2081-2202, with the rotation-consistency histogram
 * (ComputeThreeMaxima :2338-2379) when check_ori != 0 (M3). Last-frame
 * keypoint i carries map point last_kp2mp[i] (-1: none) at world position
 * last_pos[3i..3i+2] and outlier flag last_outlier[i]. Matches write
 * kp2mp[j] = last_kp2mp[i] and score[j]; rejected rotations reset score to
 * 999 (:2183-2186). */
int gf_match_lastframe(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                       const float* Tcw, const gf_keypoint* last_kps, const uint8_t* last_desc,
                       const int32_t* last_kp2mp, const uint8_t* last_outlier, const float* last_pos, int n_last,
                       float th, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches);

/* Device family of the three above, batched over nframes independent frames.
 * Per-frame arrays are strided by their capacity (kp_cap keypoints, mp_cap /
 * last_cap queries); counts live on the device (d_n, d_m, d_n_last). Limits:
 * kp_cap <= 4096, mp_cap/last_cap <= 8192. gf_match_lastframe_dev needs
 * d_scratch of nframes*last_cap int32. */
int gf_frustum_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw, const gf_map_point* d_mps,
                   const int32_t* d_m, int mp_cap, float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview,
                   void* stream);
int gf_match_project_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                         const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                         const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, float th, float nnratio,
                         int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream);
int gf_match_lastframe_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                           const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const float* d_Tcw,
                           const gf_keypoint* d_last_kps, const uint8_t* d_last_desc, const int32_t* d_last_kp2mp,
                           const uint8_t* d_last_outlier, const float* d_last_pos, const int32_t* d_n_last,
                           int last_cap, float th, int check_ori, int32_t* d_kp2mp, int32_t* d_score,
                           int32_t* d_nmatches, int32_t* d_scratch, void* stream);

/* List forms (device family). Frame::isInFrustum for the map points
 * d_list[f][0 .. d_nlist[f]) only (the visibility pass of
 * SearchAdditionalMatchesInFrame over mLeftMapPoints, Tracking.cc:3105-3126);
 * views of other points are left as they are. And
 * ORBmatcher::SearchByProjection_Budget(F, vpMapPoints, th, time)
 * (ORBmatcher.cc:276-379) = SearchByProjection over the map points of the
 * list in list order (th != 1 scales the window; claims and the ratio test as
 * M2). Lists are strided by mp_cap. */
int gf_frustum_list_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw,
                        const gf_map_point* d_mps, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                        float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview, void* stream);
int gf_match_project_list_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                              const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                              const uint8_t* d_mp_desc, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                              float th, float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches,
                              void* stream);

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:2384-2400) over n pairs of
 * 32-byte rows: dist[i] = popcount(a[i] ^ b[i]). */
int gf_descriptor_distance(gf_ctx* ctx, const uint8_t* a, const uint8_t* b, int n, int32_t* dist);

/* ------------------------------------------------- good-feature selection (G1-G7)
 * f64 throughout, as the reference's Armadillo matrices. */

/* glibc rand() state (TYPE_3 additive feedback, 31 words): the reference draws
 * its lazier-greedy samples with std::rand() % n (Observability.cc:1348,
 * :2895). Callers keep one state per sequence across frames. */
typedef struct gf_rng {
    int32_t state[31];
    int32_t f, r;
} gf_rng;
/* std::srand(seed) */
int gf_rng_seed(gf_rng* rng, uint32_t seed);
/* n successive std::rand() values (host; for checking the device port). */
int gf_rng_next(gf_rng* rng, int32_t* out, int n);

/* Observability camera (PinHoleCamera, include/Util.hpp:136-178) and the
 * visibility margins mBoundX/YInFrame, mBoundDepth (Observability.h:727-728)
 * with Frame::mnMinX..mnMaxY. */
typedef struct gf_obs_camera {
    double fu, fv, cx, cy;
    int32_t nrows, ncols;
    int32_t min_x, max_x, min_y, max_y;
    int32_t bound_x, bound_y;
    float bound_depth;
} gf_obs_camera;

/* One predicted segment of the constant-velocity PWLS motion model
 * (KineStruct, Util.hpp:170-177): state Xv = [twc(3) q_wc(4) v(3) w(3)], the
 * quaternion/angular-rate blocks of F for the full segment and one of 13
 * sub-segments, and the predicted Tcw (float, row-major). */
typedef struct gf_kine {
    double dt, dt_inseg;
    double Xv[13];
    double F_Q[16], F_Omg[12], F_Q_inSeg[16], F_Omg_inSeg[12]; /* row-major */
    float Tcw[16];
} gf_kine;

/* Observability::updatePWLSVec (Observability.h:222-259): Xv from the last
 * frame pose Tcw_prev and the current Twc (float row-major), times in s. */
int gf_obs_update(double t_prev, const float* Tcw_prev, double t_cur, const float* Twc_cur, double* Xv);
/* Observability::predictPWLSVec(dt, nseg) (Observability.h:261-295). */
int gf_obs_predict(const double* Xv, double dt, int nseg, gf_kine* out);

/* Measurement Jacobian + information block per landmark
 * (compute_H_subblock_simplied Observability.h:460-515, reWeightInfoMat
 * :517-596, batchInfoMat_Map / batchInfoMat_Frame Observability.cc:386-644).
 * For each of n landmarks at world position pos[3i..]: H (2x7 row-major,
 * n x 14) and info = H_rw^T H_rw (7x7 row-major, n x 49) at state Xv, where
 * H_rw = H / sigma, sigma^2 = sigma2[i] (frame path: level sigma^2 of the
 * matched keypoint octave) or 1 when sigma2 == NULL (map path). uv = the
 * projected pixel (u_proj, v_proj). valid[i] = 0 when check_viz rejects the
 * landmark (ObsScore = -1). */
int gf_obs_build_info(gf_ctx* ctx, const gf_obs_camera* cam, const double* Xv, const float* pos,
                      const float* sigma2, int n, int check_viz, double* H, double* info, float* uv,
                      uint8_t* valid);

/* Util.hpp:714-731 logDet: 2 log prod diag chol(M), LU log|det| fallback;
 * n 7x7 row-major matrices. */
int gf_logdet(gf_ctx* ctx, const double* M, int n, double* out);

/* Observability::runActiveMapMatching with FRAME_INFO_MATRIX
 * (Observability.cc:1249-1524): lazier-greedy active matching of
 * num_to_match map points into frame F using SearchByProjection_OnePoint
 * (ORBmatcher.h:71-145). Pool = map points with views[i].in_view and
 * updated[i] (updateAtFrameId == frame id), in list order; info/H are their
 * map information blocks and Jacobians (gf_obs_build_info map path), uv their
 * projections. base = mCurrentInfoMat (7x7). level_sigma2 = Frame
 * mvLevelSigma2. Writes claims into kp2mp/score (in/out), the left-over pool
 * (mLeftMapPoints) into left[0..nleft), advances rng; nmatched = matches. */
int gf_obs_active_match(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                        const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated,
                        const double* info, const double* H, const float* uv, int m, const double* base,
                        const float* level_sigma2, int num_to_match, float th, float nnratio, gf_rng* rng,
                        int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft, int* nmatched);

/* Max-volume subset selection over a pool of 7x7 information blocks
 * (Observability.cc): mode 1 = maxVolSelection_BaselineGreedy (:3031-3139),
 * 2 = maxVolSelection_LazierGreedy (:2815-3029), 3 =
 * maxVolAutomatic_LazierGreedy (:3141-3155, deletion when 2k > n).
 * score[i] < 0 excludes block i (obs_score). sample_scale as
 * setSelction_Number computes it (:823). out_idx receives pool indices in
 * selection order (deletion: pool order). rng used by modes 2-3. */
int gf_maxvol_select(gf_ctx* ctx, const double* info, const double* score, int n, int k, double sample_scale,
                     int mode, gf_rng* rng, int32_t* out_idx, int* nout);

/* The greedy stage alone, over a prepared pool (lmkSelectPool,
 * Observability.cc:1046-1160): n blocks info [n][49] with their ObsScore
 * values, k = num_good_inlier; out_idx = pool positions selected (greedy_mtd
 * 3 splits large pools into threadNeeded chunks, run in chunk order on rng).
 * What setSelction_Number runs after MAP_INFO_MATRIX has left points updated
 * this frame (e.g. by FRAME_INFO_MATRIX) with their own blocks and scores. */
int gf_select_pool(gf_ctx* ctx, const double* info, const double* score, int n, int k, int greedy_mtd,
                   int max_threads, gf_rng* rng, int32_t* out_idx, int* nout);

/* Observability::setSelction_Number(num_good_inlier, greedy_mtd, time,
 * mapPoints, mpVec) (Observability.cc:1021-1247; test/test_GoodMap.cpp drives
 * it): MAP_INFO_MATRIX with the visibility check (mKineIdx = 1: Xv is the
 * predicted kinematic[1] state) over the n map points at pos, the visible ones
 * form the pool in list order, then greedy_mtd 1 = BaselineGreedy, 2 =
 * LazierGreedy, 3 = maxVolAutomatic_LazierGreedy with the multi-thread split
 * (threadNeeded = min(round(pool / 1000), max_threads) when pool >= 2000 and
 * pool - 1.2 k > 10; chunks of ceil(pool / T) selecting ceil(k / T * 1.2)
 * each, then one pass over the merged selections). sample_scale 6. The chunks
 * draw from `rng` in chunk order (the reference's threads share std::rand()
 * in race order). out_idx = map indices in selection order (deletion
 * variant: pool order); at most 4096 visible points per greedy call. */
int gf_select_map_points(gf_ctx* ctx, const gf_obs_camera* cam, const double* Xv, const float* pos, int n, int k,
                         int greedy_mtd, int max_threads, gf_rng* rng, int32_t* out_idx, int* nout);

/* Device family of the GF rows, batched over frames (per-frame arrays strided
 * by cap / mp_cap; d_Xv is [F][13], d_base [F][49], d_rng [F]). Pool limit
 * for active matching and max-volume selection: 4096 landmarks.
 * gf_obs_accumulate_dev: d_out[f] = diag*I + sum of d_info rows with d_flag
 * set (mCurrentInfoMat accumulation, Tracking.cc:3161 and :3195-3219).
 * gf_obs_active_match_dev: d_nldet (optional, [F]) = logDet evaluations the
 * reference makes (one per heap push, Observability.cc:1373); frames whose
 * d_m or d_num_to_match is 0 exit before any LDS use. */
int gf_obs_build_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_pos,
                          const float* d_sigma2, const int32_t* d_n, int cap, int check_viz, double* d_H,
                          double* d_info, float* d_uv, uint8_t* d_valid, void* stream);
int gf_obs_accumulate_dev(gf_ctx* ctx, int nframes, const double* d_info, const uint8_t* d_flag, const int32_t* d_n,
                          int cap, double diag, double* d_out, void* stream);
int gf_obs_active_match_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                            const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                            const uint8_t* d_mp_desc, const uint8_t* d_updated, const double* d_info,
                            const double* d_H, const int32_t* d_m, int mp_cap, const double* d_base,
                            const float* level_sigma2, const int32_t* d_num_to_match, float th, float nnratio,
                            gf_rng* d_rng, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_left, int32_t* d_nleft,
                            int32_t* d_nmatched, int32_t* d_nldet, void* stream);
int gf_maxvol_select_dev(gf_ctx* ctx, int npools, const double* d_info, const double* d_score, const int32_t* d_n,
                         int cap, int k, double sample_scale, int mode, gf_rng* d_rng, int32_t* d_out,
                         int32_t* d_nout, void* stream);

/* G1 on the device: Xv[f] = updatePWLSVec(t_prev[f], Tcw_prev[f], t_cur[f],
 * getTwc(Tcw_cur[f])) (Tracking.cc:3168-3169, :797-799, Frame.cc:152-163).
 * Segment 0 of predictPWLSVec keeps this Xv (the in-frame FRAME/MAP builds);
 * d_Xv_next (optional) = kinematic[1].Xv = propagate_PWLS(Xv, float(dt)), the
 * state the next-frame MAP build uses (Tracking.cc:1768, mKineIdx = 1). */
int gf_obs_update_dev(gf_ctx* ctx, int nframes, const double* d_t_prev, const float* d_Tcw_prev,
                      const double* d_t_cur, const float* d_Tcw_cur, double* d_Xv, double* d_Xv_next,
                      void* stream);

/* Map-resident observability state, map-indexed per frame (stride
 * map_stride): H [14], ObsMat [49], u/v_proj [2], updateAtFrameId (int32).
 * gf_obs_frame_info_dev = batchInfoMat_Frame (Observability.cc:386-554):
 *   matched non-outlier keypoints write their map point's H/ObsMat/uv with
 *   the keypoint level sigma^2; updateAtFrameId untouched.
 * gf_obs_map_info_dev = batchInfoMat_Map (Observability.cc:556-644): points
 *   with updateAtFrameId == frame_id are skipped, and with check_viz == 0 so
 *   are points whose view is not in_view (d_views may be NULL only with
 *   check_viz); a valid point is written and stamped frame_id. d_updated
 *   (optional) = (updateAtFrameId == frame_id) for every point afterwards.
 * gf_obs_accumulate_matched_dev: mCurrentInfoMat = diag*I + sum, in keypoint
 *   order, of the ObsMat of matched points stamped frame_id (Tracking.cc:3184,
 *   3195-3213). */
int gf_obs_frame_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv,
                          const gf_keypoint* d_kps, const int32_t* d_nkps, int kp_stride, const int32_t* d_kp2mp,
                          const uint8_t* d_outlier, const float* d_map_pos, const int32_t* d_nmp, int map_stride,
                          const float* level_sigma2, int nlevels, double* d_H, double* d_info, float* d_uv,
                          void* stream);
int gf_obs_map_info_dev(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_map_pos,
                        const int32_t* d_nmp, int map_stride, int check_viz, const gf_mp_view* d_views,
                        int32_t* d_upd_id, int frame_id, double* d_H, double* d_info, float* d_uv,
                        uint8_t* d_updated, void* stream);
int gf_obs_accumulate_matched_dev(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps,
                                  int kp_stride, const double* d_info, const int32_t* d_upd_id, const int32_t* d_nmp,
                                  int map_stride, int frame_id, double diag, double* d_out, void* stream);

/* ------------------------------------------------ pose optimisation (P1-P4)
 * Optimizer::PoseOptimization(Frame*) (src/Optimizer.cc:279-413) on g2o's
 * Levenberg-Marquardt (core/optimization_algorithm_levenberg.cpp:61-189),
 * EdgeSE3ProjectXYZ with a fixed map point (types_six_dof_expmap.cpp:384-428),
 * Huber delta^2 = 5.991 (robust_kernel_impl.cpp:78-88) and the dense LDLT
 * solver (linear_solver_dense.h:65-113). One edge per matched keypoint, in
 * keypoint order; f64 internally, float pose in and out (Converter.cc:38-72).
 * Outlier flags follow the reference: 4 rounds of {10,10,7,5} iterations with
 * chi2 thresholds {9.210,7.378,5.991,5.991}; outliers keep their edge with
 * information 1e-10. ninliers = n - nBad of the last round. */
typedef struct gf_pose_edge {
    float X[3];       /* MapPoint::GetWorldPos() */
    float z[2];       /* mvKeysUn[i].pt */
    float inv_sigma2; /* mvInvLevelSigma2[octave] */
} gf_pose_edge;

/* Host family: one problem of n edges. iterations (may be NULL) = LM
 * iterations run over the 4 rounds. */
int gf_pose_opt(gf_ctx* ctx, const float* Tcw_in, const gf_pose_edge* edges, int n, float fx, float fy, float cx,
                float cy, float* Tcw_out, uint8_t* outlier, int32_t* ninliers, int32_t* iterations);

/* Device family, nprob independent problems (one workgroup each). d_Tcw is
 * nprob x 16 floats, updated in place; problem p owns edges
 * [p*edge_stride, p*edge_stride + d_nedges[p]) and the same outlier slots.
 * d_iterations may be NULL. edge_stride <= 8192. */
int gf_pose_opt_batch_dev(gf_ctx* ctx, int nprob, float* d_Tcw, const gf_pose_edge* d_edges, const int32_t* d_nedges,
                          int edge_stride, float fx, float fy, float cx, float cy, uint8_t* d_outlier,
                          int32_t* d_ninliers, int32_t* d_iterations, void* stream);

/* Device family over Frames: gathers the edges of every keypoint with
 * d_kp2mp >= 0 (X = d_map[kp2mp].pos of that frame's map, z = keypoint,
 * inv_sigma2[octave]), optimises d_Tcw in place and writes mvbOutlier for the
 * matched keypoints (others untouched). inv_sigma2 is a host array of nlevels
 * (<= 16) floats. kp_stride <= 8192. d_nedges (nInitialCorrespondences) and
 * d_iterations may be NULL. */
int gf_pose_opt_frames_dev(gf_ctx* ctx, int nframes, float* d_Tcw, const gf_keypoint* d_kps, const int32_t* d_nkps,
                           int kp_stride, const int32_t* d_kp2mp, const gf_map_point* d_map, int map_stride,
                           const float* inv_sigma2, int nlevels, float fx, float fy, float cx, float cy,
                           uint8_t* d_outlier, int32_t* d_ninliers, int32_t* d_iterations, int32_t* d_nedges,
                           void* stream);

/* --------------------------------------- ORB vocabulary, BoW (D1), SearchByBoW (M6)
 * A DBoW2 ORB vocabulary tree (TemplatedVocabulary<FORB::TDescriptor, FORB>,
 * Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) as its loaders build it:
 * node 0 is the root; nodes 1..nnodes-1 in file record order with their
 * parent, 32-byte descriptor, weight and leaf flag; a node's children in
 * record order; word ids in record order of the leaves. scoring is DBoW2's
 * ScoringType (0 L1_NORM, 1 L2_NORM, 2 CHI_SQUARE, 3 KL, 4 BHATTACHARYYA,
 * 5 DOT_PRODUCT), weighting its WeightingType (0 TF_IDF, 1 TF, 2 IDF, 3 BINARY). */
typedef struct gf_vocab_arrays {
    int32_t k, L, scoring, weighting, nnodes;
    int32_t* parent;  /* nnodes; parent[0] = -1 */
    uint8_t* desc;    /* nnodes x 32 */
    double* weight;   /* nnodes */
    uint8_t* is_leaf; /* nnodes */
} gf_vocab_arrays;

typedef struct gf_vocab gf_vocab;

/* Host only: parse a vocabulary file — loadFromTextFile (TemplatedVocabulary.h:1352-1432)
 * for a ".txt" path, loadFromBinaryFile (:1469-1510) otherwise. With out->parent
 * == NULL only the header fields and nnodes are filled; call again with buffers
 * of nnodes entries. */
int gf_vocab_read(const char* path, gf_vocab_arrays* out);
/* Host only: TemplatedVocabulary::saveToBinaryFile (TemplatedVocabulary.h:1516-1536;
 * tools/bin_vocabulary.cc converts ORBvoc.txt with it): header {nb_nodes,
 * size_node = 41, k, L, scoring, weighting}, then nodes 1..nnodes-1 as {uint32
 * parent, 32 descriptor bytes, float weight, bool is_leaf}, is_leaf meaning "has
 * no children" as Node::isLeaf. */
int gf_vocab_save_binary(const gf_vocab_arrays* tree, const char* path);
/* Upload a tree (device-resident, shared by every frame of the context). */
int gf_vocab_create(gf_ctx* ctx, const gf_vocab_arrays* tree, gf_vocab** out);
/* gf_vocab_read + gf_vocab_create (main.cc:92-106 picks the loader by suffix). */
int gf_vocab_load(gf_ctx* ctx, const char* path, gf_vocab** out);
int gf_vocab_info(gf_vocab* voc, int* k, int* L, int* nnodes, int* nwords);
int gf_vocab_destroy(gf_vocab* voc);

/* Frame::ComputeBoW (Frame.cc:380-387) = transform(descriptors, mBowVec,
 * mFeatVec, levelsup) (TemplatedVocabulary.h:1141-1208, 1232-1273): the
 * BowVector as words[0..nwords) ascending with values, the FeatureVector as
 * fv_nodes[0..nfv) ascending with the feature indices of node i in
 * fv_feats[fv_start[i] .. fv_start[i+1]). Capacities n (fv_start n + 1).
 * At most 4096 descriptors per frame. */
int gf_bow_transform(gf_vocab* voc, const uint8_t* desc, int n, int levelsup, int32_t* words, double* values,
                     int* nwords, int32_t* fv_nodes, int32_t* fv_start, int32_t* fv_feats, int* nfv);
/* Device family: nframes frames, descriptors and outputs strided by cap. */
int gf_bow_transform_dev(gf_vocab* voc, int nframes, const uint8_t* d_desc, const int32_t* d_n, int cap, int levelsup,
                         int32_t* d_words, double* d_values, int32_t* d_nwords, int32_t* d_fv_nodes,
                         int32_t* d_fv_start, int32_t* d_fv_feats, int32_t* d_nfv, void* stream);

/* One side of ORBmatcher::SearchByBoW: its FeatureVector, descriptors,
 * keypoints (for the angle) and map point per feature (-1 = none or bad). */
typedef struct gf_bow_side {
    const int32_t* fv_nodes;
    const int32_t* fv_start;
    const int32_t* fv_feats;
    int32_t nfv;
    const uint8_t* desc;
    const gf_keypoint* kps;
    const int32_t* mp;
    int32_t n;
} gf_bow_side;

/* mode 0: SearchByBoW(KeyFrame* a, Frame& b, vpMapPointMatches)
 *   (ORBmatcher.cc:724-853): out has b.n entries, out[j] = a's map point
 *   matched to b feature j or -1; a feature needs a map point, best <= TH_LOW.
 * mode 1: SearchByBoW(KeyFrame* a, KeyFrame* b, vpMatches12) (:1289-1424):
 *   out has a.n entries, out[i] = b's map point matched to a feature i; b
 *   features need a map point, best < TH_LOW.
 * Both: best < nnratio * second, rotation consistency (ComputeThreeMaxima
 * :2338-2379) when check_ori. nmatches = the returned count. */
int gf_match_bow(gf_ctx* ctx, int mode, float nnratio, int check_ori, const gf_bow_side* a, const gf_bow_side* b,
                 int32_t* out, int* nmatches);
/* Device family: npairs (a[p], b[p]) pairs whose pointers are device
 * pointers; outs[p] device output of pair p, d_nmatches[p]. The host arrays a,
 * b, outs are copied at the call. At most 4096 features per side. */
int gf_match_bow_dev(gf_ctx* ctx, int mode, float nnratio, int check_ori, int npairs, const gf_bow_side* a,
                     const gf_bow_side* b, int32_t* const* outs, int32_t* d_nmatches, void* stream);

/* ------------------------------------------------ local bundle adjustment (B1)
 * Optimizer::LocalBundleAdjustment(KeyFrame*, bool*) (src/Optimizer.cc:1515-1764)
 * on g2o's Levenberg-Marquardt with the Schur complement over the map points
 * (core/block_solver.hpp:354-486): optimize(5), drop the edges with chi2 >
 * 5.991 or negative depth, optimize(10), flag the outliers again.
 *
 * The caller passes the graph the reference builds (Optimizer.cc:1517-1675)
 * as plain arrays, in the reference's orders:
 *   keyframes in vertex-id order (mnId), kind 0 = local keyframe, 1 = local
 *     keyframe that is fixed (mnId == 0; written back), 2 = fixed camera
 *     (lFixedCameras: a fixed vertex, not written back);
 *   map points in vertex-id order (mnId), their world positions;
 *   edges in insertion order (lLocalMapPoints, then each point's
 *     observations); the edges of one point are contiguous and a point has
 *     at most one edge per keyframe (map<KeyFrame*, size_t>).
 * Results: poses of kinds 0/1 (kind 2 copied through), point positions,
 * per-edge outlier flags (1 = removed after optimize(5), 2 = flagged after
 * optimize(10); the caller erases those observations, Optimizer.cc:1691-1696,
 * 1739-1741) and the iterations of the two optimize() calls (-1 = not run).
 * Limits: at most 32 keyframes of kind 0 per problem, 65536 points. */
typedef struct gf_ba_problem {
    int32_t nkf, npts, nedges;
    const float* kf_Tcw;          /* nkf x 16, row-major KeyFrame::GetPose() */
    const uint8_t* kf_kind;       /* nkf: 0 local, 1 local fixed, 2 fixed camera */
    const float* kf_cam;          /* nkf x 4: fx, fy, cx, cy */
    const float* pt_pos;          /* npts x 3: MapPoint::GetWorldPos() */
    const int32_t* edge_pt;       /* nedges: point index */
    const int32_t* edge_kf;       /* nedges: keyframe index */
    const float* edge_z;          /* nedges x 2: GetKeyPointUn(idx).pt */
    const float* edge_inv_sigma2; /* nedges: GetInvSigma2(octave) */
} gf_ba_problem;

typedef struct gf_ba_result {
    float* kf_Tcw;          /* nkf x 16 */
    float* pt_pos;          /* npts x 3 */
    uint8_t* edge_outlier;  /* nedges */
    int32_t iterations[2];  /* optimize(5), optimize(10) */
} gf_ba_result;

typedef struct gf_ba_plan gf_ba_plan;

/* Host family: one problem, synchronous. */
int gf_local_ba(gf_ctx* ctx, const gf_ba_problem* prob, gf_ba_result* res);

/* Batched device path: gf_ba_plan_create validates and uploads nprob
 * problems and builds their structure (index mapping, per-pose edge lists,
 * Schur panel layout) once; gf_ba_plan_solve runs every problem from its
 * uploaded initial state to the end on `stream` (all problems advance one LM
 * trial per step; the host polls a device done flag every few steps; *steps
 * = steps run); gf_ba_plan_results copies res[0..nprob) out. */
int gf_ba_plan_create(gf_ctx* ctx, int nprob, const gf_ba_problem* probs, gf_ba_plan** out);
int gf_ba_plan_solve(gf_ba_plan* plan, void* stream, int* steps);
int gf_ba_plan_results(gf_ba_plan* plan, gf_ba_result* res);
/* The abortable forms: LocalBundleAdjustment(pKF, &mbAbortBA) with
 * optimizer.setForceStopFlag(pbStopFlag) (Optimizer.cc:1515, 1579-1580;
 * LocalMapping.cc:108). The host polls *stop_flag (written by another thread,
 * as LocalMapping's mbAbortBA is) between LM iterations; once it is set every
 * problem's running optimize() call ends at its next iteration boundary (the
 * iteration in flight completes, as SparseOptimizer::optimize checks
 * terminate() before each iteration), optimize(10) then runs 0 iterations and
 * both outlier checks still run. NULL = never stop. */
int gf_ba_plan_solve_stop(gf_ba_plan* plan, void* stream, const volatile uint8_t* stop_flag, int* steps);
int gf_local_ba_stop(gf_ctx* ctx, const gf_ba_problem* prob, gf_ba_result* res, const volatile uint8_t* stop_flag);
int gf_ba_plan_destroy(gf_ba_plan* plan);

/* ------------------------------------------------ keypoint undistortion
 * Frame::UndistortKeyPoints (Frame.cc:389-423): cv::undistortPoints with
 * K = {fx, fy, cx, cy} and dist = {k1, k2, p1, p2, k3} (k3 = 0 for the 4-term
 * model); keypoints are copied unchanged when k1 == 0. Only x/y change. */
int gf_undistort_keypoints(gf_ctx* ctx, const float K[4], const float dist[5], const gf_keypoint* kps, int n,
                           gf_keypoint* out);
/* Batched: d_in/d_out are [nframes][cap], d_n[nframes] keypoints each. */
int gf_undistort_keypoints_dev(gf_ctx* ctx, int nframes, const float K[4], const float dist[5],
                               const gf_keypoint* d_in, const int32_t* d_n, int cap, gf_keypoint* d_out, void* stream);

/* ------------------------------------------ local-mapping matchers (§8f rank 3)
 * MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:197-262) for nmp
 * map points at once: point p's observation descriptors (non-bad keyframes,
 * observation-map order) are rows offsets[p] .. offsets[p+1]-1 of desc
 * (offsets has nmp + 1 entries, offsets[0] = 0). best[p] = the row (relative
 * to offsets[p]) with the least median Hamming distance to the others, -1 for
 * a point without observations; out_desc (optional, nmp x 32, in/out)
 * receives that row (mDescriptor), untouched for an empty point. */
int gf_distinctive_descriptors(gf_ctx* ctx, int nmp, const uint8_t* desc, const int32_t* offsets, int32_t* best,
                               uint8_t* out_desc);
/* Device family: total = offsets[nmp] (host value: sizes the row grid). */
int gf_distinctive_descriptors_dev(gf_ctx* ctx, int nmp, const uint8_t* d_desc, const int32_t* d_offsets,
                                   int32_t* d_best, uint8_t* d_out_desc, int total, void* stream);

/* ORBmatcher::Fuse(KeyFrame* pKF, vector<MapPoint*>& vpMapPoints, th)
 * (src/ORBmatcher.cc:1590-1707). The keyframe: bounds/intrinsics/pyramid in
 * fi, pose Tcw (row-major 4x4), camera centre Ow (KeyFrame::GetCameraCenter),
 * undistorted keypoints, descriptors, kf_mp[k] = id of the map point at slot k
 * (-1 none) and kf_mp_bad[k] its isBad() (optional). The candidates:
 * gf_map_point (mfMin/MaxDistance are the invariance distances), descriptors,
 * mp_skip[i] (optional) = NULL / isBad() / IsInKeyFrame(pKF), mp_ids[i]
 * (optional, default i) the id reported as a Replace() target. Result per
 * candidate in list order:
 *   kp      keypoint fused with (bestDist <= TH_LOW) or -1;
 *   action  GF_FUSE_ADD      pMP->AddObservation(pKF, kp), pKF->AddMapPoint;
 *           GF_FUSE_REPLACE  pMP->Replace(target): target is the slot's
 *                            occupant, or the earlier candidate that took the
 *                            empty slot in this call;
 *           GF_FUSE_KEEP     the occupant isBad(): nothing changes;
 *   nfused = number of candidates with kp >= 0 (the reference's nFused). */
enum { GF_FUSE_NONE = 0, GF_FUSE_ADD = 1, GF_FUSE_REPLACE = 2, GF_FUSE_KEEP = 3 };
typedef struct gf_fuse_result {
    int32_t kp, action, target;
} gf_fuse_result;
int gf_fuse(gf_ctx* ctx, const gf_frame_info* fi, const float* Tcw, const float* Ow, const gf_keypoint* kps,
            const uint8_t* desc, int n, const int32_t* kf_mp, const uint8_t* kf_mp_bad, const gf_map_point* mps,
            const uint8_t* mp_desc, const uint8_t* mp_skip, const int32_t* mp_ids, int m, float th,
            gf_fuse_result* res, int* nfused);
/* Device family: nprob independent (keyframe, candidate list) problems that
 * share fi; every pointer in a problem is a device pointer (the array itself
 * is host memory, copied at the call). At most 4096 keypoints per keyframe. */
typedef struct gf_fuse_problem {
    float Tcw[16];
    float Ow[3];
    const gf_keypoint* kps;
    const uint8_t* desc;
    int32_t n;
    const int32_t* kf_mp;
    const uint8_t* kf_mp_bad;
    const gf_map_point* mps;
    const uint8_t* mp_desc;
    const uint8_t* mp_skip;
    const int32_t* mp_ids;
    int32_t m;
    float th;
    gf_fuse_result* res;
    int32_t* nfused;
} gf_fuse_problem;
int gf_fuse_dev(gf_ctx* ctx, const gf_frame_info* fi, int nprob, const gf_fuse_problem* probs, void* stream);

/* ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, ...) (src/ORBmatcher.cc:
 * 1426-1588): keypoints of a (pKF1) and b (pKF2) without a map point
 * (mp < 0) that share a FeatureVector node; best distance <= TH_LOW, the
 * candidates within 2x the best walked in (distance, index) order, the first
 * passing CheckDistEpipolarLine (:705-722: squared distance to the epipolar
 * line x1' F12 < 3.84 sigma2_b[octave]) matches; rotation consistency when
 * check_ori. F12 row-major 3x3; sigma2_b = pKF2's mvLevelSigma2 (nlevels <= 16).
 * out[i] (a.n entries) = the b keypoint matched to a keypoint i or -1
 * (vMatches12; vMatchedPairs are its non-negative entries in order). */
int gf_search_for_triangulation(gf_ctx* ctx, int check_ori, const gf_bow_side* a, const gf_bow_side* b,
                                const float* F12, const float* sigma2_b, int nlevels, int32_t* out, int* nmatches);
/* Device family: npairs independent (a[p], b[p]) keyframe pairs (device
 * pointers; LocalMapping::CreateNewMapPoints pairs the new keyframe with each
 * covisible neighbour), F12 host array of npairs x 9, one sigma2 table,
 * outs[p] device output of pair p, d_nmatches[p]. One workgroup per pair. */
int gf_search_for_triangulation_dev(gf_ctx* ctx, int check_ori, int npairs, const gf_bow_side* a,
                                    const gf_bow_side* b, const float* F12, const float* sigma2_b, int nlevels,
                                    int32_t* const* outs, int32_t* d_nmatches, void* stream);

/* ----------------------------------------- local-map assembly
 * Tracking::UpdateReference (Tracking.cc:3689-3706) =
 * UpdateReferenceKeyFrames (:3768-3852) + UpdateReferencePoints (:3708-3766),
 * for a batch of frames tracking against one map:
 *   - every map point of the frame (mvpMapPoints, keypoint order) that is
 *     not bad votes once for each keyframe observing it; bad ones are set to
 *     -1 in the frame (:3778-3793);
 *   - local keyframes = the voted keyframes that are not bad, in
 *     std::map<KeyFrame*,int> order, i.e. ascending KeyFrame* — which is the
 *     order keyframes are passed in here (Map::GetAllKeyFrames iterates its
 *     std::set<KeyFrame*> that way); the reference keyframe is the first one
 *     with the most votes (:3798-3817);
 *   - while the list holds <= 80, each of the keyframes found so far adds the
 *     first of its best 10 covisible keyframes (GetBestCovisibilityKeyFrames(10))
 *     that is neither bad nor in the list (:3820-3848);
 *   - local map points = the map points of the local keyframes
 *     (GetMapPointMatches, slot order), first occurrence only, not bad
 *     (:3737-3763; GOOD_FEATURE_MAP_BOUND is off in the reference build).
 * The keyframe / map-point "mnTrackReferenceForFrame" marks are the
 * call's own: every call starts from unmarked keyframes and points. */
typedef struct gf_covis_map {
    int32_t nkf, nmp;           /* keyframes (<= 8192), map points            */
    const uint8_t* kf_bad;      /* [nkf] KeyFrame::isBad, ascending KeyFrame* */
    const int32_t* kf_mp_off;   /* [nkf+1] CSR of KeyFrame::mvpMapPoints      */
    const int32_t* kf_mp;       /*   map point index per slot, -1 = NULL      */
    const int32_t* kf_cov_off;  /* [nkf+1] CSR of mvpOrderedConnectedKeyFrames */
    const int32_t* kf_cov;      /*   keyframe indices (the first 10 are used) */
    const uint8_t* mp_bad;      /* [nmp] MapPoint::isBad                      */
    const int32_t* mp_obs_off;  /* [nmp+1] CSR of MapPoint::mObservations     */
    const int32_t* mp_obs;      /*   observing keyframe indices               */
} gf_covis_map;
/* One frame, host arrays (the map is uploaded per call). frame_mps[nkp] is
 * updated in place. Outputs up to the caps; the counts are the full sizes
 * (GF_ERR_CAP when a cap is exceeded). ref_kf = pKFmax index or -1. */
int gf_update_reference(gf_ctx* ctx, const gf_covis_map* map, int32_t* frame_mps, int nkp, int32_t* local_kfs,
                        int* n_local_kfs, int kf_cap, int32_t* local_mps, int* n_local_mps, int mp_cap,
                        int32_t* ref_kf);
/* B frames against one map whose arrays are device pointers (the struct is
 * host memory). d_frame_mps [B][stride] with d_nkps[B]; outputs
 * [B][kf_cap] / [B][mp_cap], counts [B], d_ref_kf [B]. */
int gf_update_reference_dev(gf_ctx* ctx, const gf_covis_map* d_map, int nframes, int32_t* d_frame_mps,
                            const int32_t* d_nkps, int stride, int32_t* d_local_kfs, int32_t* d_n_local_kfs,
                            int kf_cap, int32_t* d_local_mps, int32_t* d_n_local_mps, int mp_cap,
                            int32_t* d_ref_kf, void* stream);

/* ------------------------------------------------ relocalisation PnP
 * ORB_SLAM::PnPsolver (src/PnPsolver.cc, include/PnPsolver.h): EPnP
 * (Lepetit et al.) on random minimal sets inside RANSAC, then a refinement
 * over the best inlier set; Tracking::Relocalization drives it
 * (Tracking.cc:3916-3942: SetRansacParameters(0.99,10,300,4,0.5,5.991), then
 * iterate(5) per candidate keyframe). A problem is the solver's correspondence
 * list in PnPsolver order (ctor :50-72): p3d (n x 3 world points), p2d (n x 2
 * undistorted keypoints), sigma2 (level sigma^2 of each keypoint octave). The
 * keypoint-index mapping (mvKeyPointIndices) stays with the caller. */
typedef struct gf_pnp_params { /* SetRansacParameters arguments (:93) */
    double probability;
    int32_t min_inliers;
    int32_t max_iterations;
    int32_t min_set; /* 1..8 (the reference uses 4) */
    float epsilon;
    float th2;
} gf_pnp_params;
typedef struct gf_pnp_state { /* one solver across iterate() calls */
    int32_t n;              /* N correspondences */
    int32_t min_inliers;    /* mRansacMinInliers after the adjustment (:106-111) */
    int32_t max_iterations; /* mRansacMaxIts after the adjustment (:116-124) */
    int32_t min_set;        /* mRansacMinSet */
    float epsilon;          /* mRansacEpsilon after the adjustment (:113-114) */
    float th2;              /* mvMaxError[i] = sigma2[i] * th2 (:126-128) */
    int32_t iterations;     /* mnIterations */
    int32_t best_inliers;   /* mnBestInliers */
    float best_Tcw[16];     /* mBestTcw, row-major */
} gf_pnp_state;
#define GF_PNP_FOUND 1   /* iterate returned a pose (refined or best)      */
#define GF_PNP_NOMORE 2  /* bNoMore                                        */
#define GF_PNP_REFINED 4 /* the pose came from Refine() (:198-208)         */
#define GF_PNP_TRUNCATED 8 /* device path: max_iterations cut the state's loop short */
/* PnPsolver::SetRansacParameters (host scalar set-up; resets the iteration
 * count and the best hypothesis as a fresh solver has them). */
int gf_pnp_init(int n, const gf_pnp_params* params, gf_pnp_state* state);
/* PnPsolver::iterate(nIterations, bNoMore, vbInliers, nInliers) (:137-230)
 * for one solver; rng is the process-wide std::rand() state the minimal sets
 * are drawn from (DUtils::Random::RandomInt, :165), advanced by min_set draws
 * per iteration run. best_mask (n bytes, mvbBestInliers) persists across calls
 * with the state. Outputs: Tcw (row-major, valid when flags & FOUND), inliers
 * (n bytes), ninliers, flags. */
int gf_pnp_iterate(gf_ctx* ctx, const float* p3d, const float* p2d, const float* sigma2, const float K[4],
                   gf_pnp_state* state, uint8_t* best_mask, int n_iterations, gf_rng* rng, float Tcw[16],
                   uint8_t* inliers, int32_t* ninliers, int32_t* flags);
/* Device batch: nprob independent solvers, problem b's correspondences at
 * [b][cap] of d_p3d/d_p2d/d_sigma2/d_best_mask/d_inliers, its size in
 * d_state[b].n; each problem draws from its own d_rng[b]. d_Tcw is [nprob][16].
 * max_iterations bounds every problem's loop count (the params value it was
 * initialised with); a problem whose loop it cuts short gets GF_PNP_TRUNCATED.
 * States are clamped on the device (min_set to 1..8, n to cap). */
int gf_pnp_iterate_dev(gf_ctx* ctx, int nprob, const float* d_p3d, const float* d_p2d, const float* d_sigma2,
                       int cap, const float K[4], gf_pnp_state* d_state, uint8_t* d_best_mask, int n_iterations,
                       int max_iterations, gf_rng* d_rng, float* d_Tcw, uint8_t* d_inliers, int32_t* d_ninliers,
                       int32_t* d_flags, void* stream);

/* ------------------------------------------------ monocular initialisation
 * ORB_SLAM::Initializer (src/Initializer.cc, include/Initializer.h):
 * Initializer(ReferenceFrame, sigma, iterations) + Initialize(CurrentFrame,
 * vMatches12, R21, t21, vP3D, vbTriangulated) (:44-132), called by
 * Tracking::MonocularInitialization with sigma 1.0 and 200 iterations; the
 * reference passes minTriangulated = THRES_INIT_MPT_NUM / 2 = 50. Frame 1 is
 * the reference frame (mvKeys1 = its undistorted keypoints), frame 2 the
 * current one; matches12[i] (n1 entries) is the frame-2 keypoint matched to
 * keypoint i of frame 1 or -1. The 8-point sets are drawn from rng (the
 * process-wide std::rand() state, DUtils::Random::RandomInt), which advances
 * by 8 * iterations draws. Outputs p3d (n1 x 3) and triangulated (n1) are
 * vP3D / vbTriangulated when ok, zeros otherwise. */
typedef struct gf_init_result {
    int32_t ok;         /* Initialize() returned true: R21, t21, p3d, triangulated valid      */
    int32_t model;      /* 0 homography (RH > 0.40), 1 fundamental, -1 neither search scored  */
    int32_t nmatches;   /* N = entries of matches12 >= 0                                       */
    int32_t iter_H;     /* RANSAC iteration of the kept H (first strict best), -1 none         */
    int32_t iter_F;     /* same for F                                                          */
    int32_t ninliers_H; /* vbMatchesInliersH count                                             */
    int32_t ninliers_F; /* vbMatchesInliersF count                                             */
    int32_t best;       /* motion hypothesis with the most nGood (0..7 H, 0..3 F), -1 none     */
    int32_t ngood[8];   /* CheckRT nGood of each motion hypothesis                             */
    float SH, SF, RH;   /* scores and ratio (RH = 0 when both scores are 0)                    */
    float parallax;     /* parallax (degrees) of hypothesis `best`                             */
    float H21[9], F21[9]; /* kept models, row-major (zeros when none)                          */
    float R21[9], t21[3]; /* accepted motion, row-major                                        */
} gf_init_result;
/* Host family: uploads, runs the device path, downloads. GF_ERR_ARG when a
 * match index is >= n2 or fewer than 8 matches exist (nothing runs then). */
int gf_initialize(gf_ctx* ctx, const float K[9], float sigma, int iterations, int min_triangulated,
                  const gf_keypoint* kps1, int n1, const gf_keypoint* kps2, int n2, const int32_t* matches12,
                  gf_rng* rng, gf_init_result* result, float* p3d, uint8_t* triangulated);
/* Device family: all buffers in device memory; the caller guarantees the
 * match indices are < n2. With fewer than 8 matches the result reports
 * model -1 and nmatches, and rng is left as it was. */
int gf_initialize_dev(gf_ctx* ctx, const float K[9], float sigma, int iterations, int min_triangulated,
                      const gf_keypoint* d_kps1, int n1, const gf_keypoint* d_kps2, int n2,
                      const int32_t* d_matches12, gf_rng* d_rng, gf_init_result* d_result, float* d_p3d,
                      uint8_t* d_triangulated, void* stream);
/* Device batch: nprob independent initialisations in one launch set (e.g. every
 * sequence of a multi-sequence tracker at start-up). Problem p's reference /
 * current keypoints at [p][cap1] / [p][cap2] with d_n1[p] / d_n2[p] valid
 * (clamped to the caps), matches12 [p][cap1], rng [p], result [p], p3d
 * [p][cap1][3], triangulated [p][cap1]. Same per-problem results as
 * gf_initialize_dev. */
int gf_initialize_batch_dev(gf_ctx* ctx, int nprob, const float K[9], float sigma, int iterations,
                            int min_triangulated, const gf_keypoint* d_kps1, int cap1, const int32_t* d_n1,
                            const gf_keypoint* d_kps2, int cap2, const int32_t* d_n2, const int32_t* d_matches12,
                            gf_rng* d_rng, gf_init_result* d_result, float* d_p3d, uint8_t* d_triangulated,
                            void* stream);

/* ------------------------------------------------ tracking glue (device)
 * Per-frame bookkeeping of Tracking between the stages above, so a front-end
 * step stays on the device. One workgroup per frame.
 * gf_motion_predict_dev: Tcw = velocity * Tcw_last (Tracking.cc:1511).
 * gf_discard_outliers_dev: kp2mp = -1, outlier = 0 for flagged matches
 *   (Tracking.cc:1550-1563); nmatches = remaining, num_to_match = budget -
 *   nmatches (Tracking.cc:3228). Either output may be NULL.
 * gf_matched_gather_dev: keypoint-ordered compaction of the matched points:
 *   pos (map position), sigma2 (level sigma^2 of the octave), idx (keypoint),
 *   n per frame; the FRAME_INFO_MATRIX input (Observability.cc:386-520).
 * gf_views_exclude_matched_dev: views[kp2mp].in_view = 0, i.e.
 *   mbTrackInView = false for points already matched (Tracking.cc:3205). */
int gf_motion_predict_dev(gf_ctx* ctx, int nframes, const float* d_velocity, const float* d_Tcw_last, float* d_Tcw,
                          void* stream);
int gf_discard_outliers_dev(gf_ctx* ctx, int nframes, int32_t* d_kp2mp, uint8_t* d_outlier, const int32_t* d_nkps,
                            int kp_stride, int budget, int32_t* d_nmatches, int32_t* d_num_to_match, void* stream);
int gf_matched_gather_dev(gf_ctx* ctx, int nframes, const gf_keypoint* d_kps, const int32_t* d_nkps, int kp_stride,
                          const int32_t* d_kp2mp, const gf_map_point* d_map, int map_stride,
                          const float* level_sigma2, int nlevels, float* d_pos, float* d_sigma2, int32_t* d_idx,
                          int32_t* d_n, void* stream);
int gf_views_exclude_matched_dev(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps,
                                 int kp_stride, gf_mp_view* d_views, const int32_t* d_nmp, int mp_stride,
                                 void* stream);

/* ------------------------------------------------ batched tracking front end
 * Tracking::GrabImage in the WORKING state (Tracking.cc:461-917) for B
 * independent sequences ("streams"), every frame of every stream on the
 * device, no host round trip inside a step:
 *   Frame (ORB extraction, E1-E8)
 *   TrackWithMotionModel (Tracking.cc:1506-1642): Tcw = V * Tlast, M3
 *     SearchByProjection(Cur, Last, 15), PoseOptimization, discard outliers
 *   TrackLocalMap (:2732-2844) with SearchReferencePointsInFrustum
 *     (:3149-3410): updatePWLSVec, FRAME_INFO_MATRIX, mCurrentInfoMat; then
 *     num_to_match <= 0: mLeftMapPoints = in-view (stale mbTrackInView)
 *       local points, mbNeedVizCheck;
 *     else isInFrustum; nToMatch < 400: SearchByProjection(F, local, 1);
 *       else MAP_INFO_MATRIX + runActiveMapMatching (leftovers = unmatched
 *       pool); PoseOptimization (outliers kept, :2776)
 *   motion model update V = Tcw * LastTwc (:729-738), updatePWLSVec +
 *     predictPWLSVec(dt, 2), RunMapPointsSelection's MAP_INFO_MATRIX at
 *     kinematic[1] (:1717-1779), SearchAdditionalMatchesInFrame
 *     (:3097-3145: isInFrustum when mbNeedVizCheck, SearchByProjection_Budget
 *     th 0.8), outliers set NULL, mLastFrame = Frame(mCurrentFrame) (:901-910).
 * The local map (UpdateReference, :3689-3852) is the map set with
 * gf_frontend_set_map, in that order; keyframe insertion and local mapping
 * are outside the path. The tracking state machine of GrabImage
 * (:602-644, 652-716, 854-911) runs per stream (GF_FE_TRACK):
 *   WORKING with a velocity and >= 2 frames since a relocalisation:
 *     TrackWithMotionModel; it fails on < 20 matches (:1559) or < 10 after
 *     the outlier discard (:1641), and TrackPreviousFrame (:1325-1404) runs;
 *   WORKING otherwise: TrackPreviousFrame (WindowSearch 200 from the upper
 *     half of the pyramid, then 100 at any level, PoseOptimization,
 *     SearchByProjection(Last, Cur, 15 or 50), PoseOptimization);
 *   LOST: Relocalisation (:3854-4031) against the stream's keyframe
 *     database (gf_frontend_set_kfdb; none: the frame stays LOST):
 *     ComputeBoW, DetectRelocalisationCandidates, SearchByBoW(0.75) per
 *     candidate (>= 15), P4P RANSAC iterate(5) rounds over the candidates
 *     (0.99, 10, 300, 4, 0.5, 5.991) with PoseOptimization and the
 *     SearchByProjection(F, KF, found, 10 / 3, 100 / 64) refinements, until
 *     one pose keeps >= 50 inliers.
 *   A frame whose initial estimate succeeded runs TrackLocalMap (the
 *   SearchByProjection window is 5 and FRAME_INFO_MATRIX is skipped for two
 *   frames after a relocalisation, :3162, :3318-3320); it fails on < 25
 *   inliers within mMaxFrames of a relocalisation or < 15 (:2819-2824). A
 *   failed frame sets LOST, clears the velocity and skips the post-publish
 *   block: mLastFrame stays the last tracked frame.
 * Assumed of the map: >= 6 keyframes (KeyFramesInMap() >= 4 for the motion
 * model, > 5 for WindowSearch's octave floor; the keyframe graph's count when
 * one is set) and frames past the initial TIME_INIT_TRACKING window.
 * updateAtFrameId stamps are stored relative to the current frame
 * (the frame being tracked is 1, the next 2; every step shifts them by -1),
 * so a step has no per-frame host argument and can be replayed as a HIP
 * graph. Time budgets follow gf_set_budgets of the context (+inf = parity). */
typedef struct gf_frontend_params {
    int32_t width, height;
    float fx, fy, cx, cy;       /* Camera.fx/fy/cx/cy                             */
    int32_t nfeatures;          /* ORBextractor.nFeatures */
    float scale_factor;         /* ORBextractor.scaleFactor */
    int32_t nlevels;            /* ORBextractor.nLevels */
    int32_t fast_th;            /* ORBextractor.fastTh */
    int32_t batch;              /* streams B */
    int32_t map_cap;            /* local-map capacity per stream (<= 4096) */
    int32_t gf_budget;          /* num_good_inlier_predef (main.cc GF budget) */
    int32_t gf;                 /* 1 GOOD_FEATURE_MAP_MATCHING, 0 ORB-SLAM baseline matching */
    double dt;                  /* frame period 1 / Camera.fps (timestamps t_k = t_0 + k dt) */
    float dist[5];              /* Camera.k1 k2 p1 p2 [k3] (mDistCoef). k1 != 0: every
                                   frame's keypoints are undistorted after extraction
                                   (Frame::UndistortKeyPoints, Frame.cc:389-423) and the
                                   image bounds mnMinX..mnMaxY come from the undistorted
                                   corners and edge midpoints (Frame.cc:425-493); they
                                   set the projection bounds, the keypoint grid and the
                                   observability margins (Tracking.cc:876-877).
                                   k1 == 0: keypoints as extracted, bounds = the image. */
    int32_t max_frames;         /* mMaxFrames = 18 * Camera.fps / 30 (Tracking.cc:153), the
                                   window of TrackLocalMap's stricter inlier rule after a
                                   relocalisation; 0: derived from dt */
    int32_t harris_score;       /* 1: ORBextractor.nScoreType = HARRIS_SCORE (0; Tracking.cc:186),
                                   0: FAST_SCORE (1, the settings' default) */
} gf_frontend_params;
typedef struct gf_frontend gf_frontend;

// Extraction gate for several front ends sharing one GPU: before its
// extraction kernels a step waits for `wait_event` (a hipEvent_t; NULL: no
// wait), after them it records `done_event` (NULL: none). Chaining front end
// g's done event into front end g+1's wait event serialises the
// bandwidth-bound extraction stages while each front end's tracking kernels
// overlap the next one's extraction. Events stay owned by the caller.
// A gated front end cannot be captured as a graph (gf_frontend_capture
// refuses), nor can a captured one be gated.
int gf_frontend_set_gate(gf_frontend* fe, void* wait_event, void* done_event);
// The extraction stage after which the gate's done event is recorded: 0
// resize, 1 blur + FAST map, 2 cells, 3 select, 4 describe (the default, the
// whole extraction). An earlier stage lets the next front end's extraction
// start sooner (overlapping this one's later stages).
int gf_frontend_set_gate_stage(gf_frontend* fe, int stage);
// Tracking stream: the step's kernels after extraction run on a stream of
// their own created with HIP stream priority `priority` (clamped to the
// device's range; lower = more urgent), forked from and joined back into the
// context's stream each step, so results and ordering are unchanged. With
// several front ends on one GPU a high priority lets one front end's
// latency-bound tracking kernels take compute units ahead of another's
// extraction kernels. Once per front end; not with gf_frontend_capture. The
// tracking kernels use the context's scratch slots, so the front end must be
// the only one on its context (GF_ERR_ARG otherwise, and gf_frontend_create
// then refuses a second front end on that context).
int gf_frontend_set_track_priority(gf_frontend* fe, int priority);
// A hipEvent_t (timing disabled) on the context's device, for the gate.
int gf_event_create(gf_ctx* ctx, void** event_out);
int gf_event_destroy(void* event);

/* Per-stream state and outputs, readable / writable as whole-batch arrays. */
enum {
    GF_FE_KPS = 0,      /* [B][cap] gf_keypoint  mCurrentFrame.mvKeysUn      */
    GF_FE_DESC,         /* [B][cap][32] u8       mDescriptors               */
    GF_FE_NKP,          /* [B] i32               N                          */
    GF_FE_TCW,          /* [B][16] f32           mTcw                       */
    GF_FE_KP2MP,        /* [B][cap] i32          mvpMapPoints (map index)   */
    GF_FE_SCORE,        /* [B][cap] i32          mvpMatchScore              */
    GF_FE_OUTLIER,      /* [B][cap] u8           mvbOutlier                 */
    GF_FE_LAST_KPS,     /* mLastFrame: as the four above                    */
    GF_FE_LAST_DESC,
    GF_FE_LAST_NKP,
    GF_FE_LAST_KP2MP,
    GF_FE_LAST_OUTLIER, /* [B][cap] u8                                      */
    GF_FE_LAST_POS,     /* [B][cap][3] f32 world position of each last MP  */
    GF_FE_TCW_LAST,     /* [B][16] f32 mLastFrame.mTcw                      */
    GF_FE_VELOCITY,     /* [B][16] f32 mVelocity                            */
    GF_FE_T_PREV,       /* [B] f64 mLastFrame.mTimeStamp                    */
    GF_FE_T_CUR,        /* [B] f64 mCurrentFrame.mTimeStamp                 */
    GF_FE_MAP,          /* [B][M] gf_map_point                              */
    GF_FE_MAP_DESC,     /* [B][M][32] u8                                    */
    GF_FE_NMP,          /* [B] i32                                          */
    GF_FE_VIEWS,        /* [B][M] gf_mp_view (mbTrackInView & projection)   */
    GF_FE_XV,           /* [B][13] f64 kinematic[0].Xv                      */
    GF_FE_XV_NEXT,      /* [B][13] f64 kinematic[1].Xv                      */
    GF_FE_BASE,         /* [B][49] f64 mCurrentInfoMat                      */
    GF_FE_MP_H,         /* [B][M][14] f64 MapPoint::H_meas                  */
    GF_FE_MP_INFO,      /* [B][M][49] f64 MapPoint::ObsMat                  */
    GF_FE_MP_UV,        /* [B][M][2] f32 u_proj, v_proj                     */
    GF_FE_MP_UPD,       /* [B][M] i32 updateAtFrameId (relative stamps)     */
    GF_FE_RNG,          /* [B] gf_rng std::rand() state per stream          */
    GF_FE_LEFT,         /* [B][M] i32 mLeftMapPoints of the last step       */
    GF_FE_STATS,        /* [GF_FE_NSTAT][B] i32, see GF_ST_*                */
    GF_FE_HIST,         /* [B][8] i32 running counters since the last write:
                           [0..4] steps per GF_ST_BRANCH value, [5] steps in
                           which a time cap fired, [6] logDet evaluations,
                           [7] local-map search matches                      */
    GF_FE_CLOCK,        /* [B][GF_CK_WORDS(M, budget)] i64 budget clock record
                           of the last step (see gf_set_budgets)             */
    GF_FE_TRACK,        /* [B][GF_TR_N] i32 tracking state, see GF_TR_*     */
    GF_FE_RELOC,        /* [B][64] gf_reloc_kf: keyframes' relocalisation-query
                           state (mnRelocQuery / mnRelocWords / mRelocScore) */
    GF_FE_NFIELDS
};
enum {
    GF_TR_STATE = 0,    /* mState after the step: 0 WORKING, 1 LOST          */
    GF_TR_VEL,          /* 1: mVelocity holds a motion, 0: empty              */
    GF_TR_SINCE,        /* mnId - mnLastRelocFrameId (saturates at 1 << 30)  */
    GF_TR_PATH,         /* initial estimate of the last step: 0 TrackWithMotionModel,
                           1 TrackPreviousFrame after it failed, 2 TrackPreviousFrame,
                           3 Relocalisation                                  */
    GF_TR_QUERY,        /* mnId of the last frame (the keyframe database's query id) */
    GF_TR_OK,           /* bOK of the last step's initial estimate           */
    GF_TR_N = 8
};
/* KeyFrame::mnRelocQuery / mnRelocWords / mRelocScore of one keyframe of a
 * stream's database (KeyFrame.h:163-165; the reference leaves mRelocScore
 * uninitialised, here it starts at 0). */
typedef struct gf_reloc_kf {
    uint32_t query;
    int32_t words;
    float score;
} gf_reloc_kf;
enum {
    GF_ST_M3 = 0,       /* SearchByProjection(Cur, Last) matches            */
    GF_ST_FOUND,        /* nMatchesFound after the outlier discard          */
    GF_ST_TO_MATCH,     /* num_to_match = budget - nMatchesFound            */
    GF_ST_BRANCH,       /* 1 leftovers only, 2 SearchByProjection, 3 active matching, 4 nToMatch = 0 */
    GF_ST_IN_VIEW,      /* nToMatch                                         */
    GF_ST_LOCAL,        /* matches of the local-map search (M2 or active)   */
    GF_ST_INL1,         /* inliers of the first PoseOptimization            */
    GF_ST_INL2,         /* mnMatchesInliers                                 */
    GF_ST_EXTRA,        /* SearchAdditionalMatchesInFrame matches           */
    GF_ST_NLEFT,        /* mLeftMapPoints size                              */
    GF_ST_ITER1, GF_ST_ITER2, GF_ST_EDGES1, GF_ST_EDGES2,
    GF_ST_FLAGS,        /* 1: M3 < 20 (TrackPreviousFrame fall-back), 2: < 10 after PoseOptimization,
                           4: mnMatchesInliers < 15 (LOST), 8: a time budget cut a loop,
                           16: timeCost_rest <= 0 (RunMapPointsSelection and
                           SearchByProjection_Budget return at once),
                           32: isInFrustum cap, 64: MAP_INFO cap (active branch),
                           128: runActiveMapMatching cap, 256: MAP_INFO cap of
                           RunMapPointsSelection, 512: visibility cap of
                           SearchAdditionalMatchesInFrame, 1024: SearchByProjection_Budget cap,
                           2048: TrackPreviousFrame ran, 4096: Relocalisation ran,
                           8192: the initial estimate failed (no TrackLocalMap),
                           16384: TrackLocalMap failed, 32768: relocalised */
    GF_ST_FRAMES,       /* frames tracked                                   */
    GF_ST_LDETS,        /* logDet evaluations of runActiveMapMatching (heap
                           pushes, Observability.cc:1373): SURVEY §8d E_ld  */
    GF_ST_NLOCAL,       /* mvpLocalMapPoints size (keyframe graphs only)    */
    GF_ST_NCUT,         /* local points the isInFrustum cap moved to mLeftMapPoints */
    GF_ST_CAND_LAST,    /* SearchByProjection(Cur, Last): area candidates (GetFeaturesInArea
                           sizes; SURVEY §8d B_match's C)                   */
    GF_ST_CAND_PROJ,    /* the same for SearchByProjection(F, local) and
                           SearchByProjection_Budget together              */
    GF_ST_TPF,          /* TrackPreviousFrame's final nmatches (lmk_num_initTrack) */
    GF_ST_NCAND,        /* relocalisation candidates (DetectRelocalisationCandidates) */
    GF_ST_RELOC,        /* relocalisation: nGood of the last pose it optimised */
    GF_ST_RANSAC,       /* relocalisation: PnPsolver::iterate calls           */
    GF_FE_NSTAT
};
int gf_frontend_create(gf_ctx* ctx, const gf_frontend_params* params, gf_frontend** out);
int gf_frontend_destroy(gf_frontend* fe);
/* Keypoint capacity per frame (sum of the extractor's level quotas). */
int gf_frontend_capacity(gf_frontend* fe, int* cap);
/* Frame source: stream b's frame at step k is the image at d_bases[b] +
 * ((phase[b] + k) mod period) * frame_stride (device memory, row stride =
 * width). d_bases / phase are host arrays of B entries (copied). */
int gf_frontend_set_source(gf_frontend* fe, const uint8_t* const* d_bases, const int32_t* phase, int period,
                           size_t frame_stride);
/* The local map of one stream (host arrays; m <= map_cap), in
 * mvpLocalMapPoints order. Resets that stream's observability state. */
int gf_frontend_set_map(gf_frontend* fe, int stream, const gf_map_point* mps, const uint8_t* desc, int m);
int gf_frontend_set_rng(gf_frontend* fe, int stream, uint32_t seed);
/* ----------------------------------------- keyframe database (relocalisation)
 * The keyframes of a stream's map as Relocalisation reads them: per keyframe
 * its undistorted keypoints and descriptors (mvKeysUn, mDescriptors; slot i of
 * the keyframe graph's kf_mp is keypoint i), its BowVector (words ascending,
 * values) and FeatureVector (nodes ascending; node g's keypoints are
 * fv_feats[fv_start[g] .. fv_start[g + 1]), offsets absolute over all
 * keyframes, fv_start has fv_off[nkf] + 1 entries), all from
 * KeyFrame::ComputeBoW with the front end's vocabulary (levelsup 4). The
 * inverted file (KeyFrameDatabase::add, KeyFrameDatabase.cc:39-45) is built
 * from the BowVectors, keyframes in index order (= insertion order).
 * gf_kfdb_create uploads a database once (device resident; several streams
 * over one scene share it); gf_frontend_set_kfdb attaches it to a stream,
 * whose keyframe graph (gf_frontend_set_covis, same nkf and slot counts)
 * supplies the map points, isBad flags and covisibility. */
typedef struct gf_keyframe_db {
    int32_t nkf;
    const int32_t* kp_off;      /* [nkf + 1] keypoint offsets                 */
    const gf_keypoint* kps;     /* [kp_off[nkf]]                              */
    const uint8_t* desc;        /* [kp_off[nkf]][32]                          */
    const int32_t* bow_off;     /* [nkf + 1]                                  */
    const int32_t* bow_words;   /* [bow_off[nkf]]                             */
    const double* bow_values;   /* [bow_off[nkf]]                             */
    const int32_t* fv_off;      /* [nkf + 1] FeatureVector nodes per keyframe */
    const int32_t* fv_nodes;    /* [fv_off[nkf]]                              */
    const int32_t* fv_start;    /* [fv_off[nkf] + 1]                          */
    const int32_t* fv_feats;    /* [fv_start[fv_off[nkf]]] keyframe-local keypoint indices */
} gf_keyframe_db;
typedef struct gf_kfdb gf_kfdb;
int gf_kfdb_create(gf_ctx* ctx, const gf_keyframe_db* db, gf_kfdb** out);
int gf_kfdb_destroy(gf_kfdb* db);
/* NULL detaches (Relocalisation then finds no candidate). The stream's
 * keyframes' query state (GF_FE_RELOC) is reset. */
int gf_frontend_set_kfdb(gf_frontend* fe, int stream, gf_kfdb* db);
/* The vocabulary of Frame::ComputeBoW for relocalisation (mpORBVocabulary);
 * the caller keeps it alive while the front end steps. */
int gf_frontend_set_vocab(gf_frontend* fe, gf_vocab* voc);
/* The track-loss matchers of the step, one problem per call (host arrays,
 * synchronous; at most 4096 keypoints a frame and map points):
 * gf_window_search: ORBmatcher::WindowSearch(F1, F2, window,
 *   vpMapPointMatches2, min_level, max_level) (ORBmatcher.cc:979-1086) with
 *   ORBmatcher(nnratio, check_ori); F1 = keypoints / descriptors / map point
 *   per keypoint (-1 NULL) of the last frame, F2 the current frame; out (n2)
 *   = vpMapPointMatches2; max_level = INT_MAX for none.
 * gf_search_frames: ORBmatcher::SearchByProjection(F1, F2, window,
 *   vpMapPointMatches2) (:1089-1168): F1's map points (world positions pos1)
 *   projected with Tcw2; kp2mp / score (n2) are F2.mvpMapPoints /
 *   mvpMatchScore, in and out.
 * gf_search_kf_projection: ORBmatcher::SearchByProjection(F, pKF,
 *   sAlreadyFound, th, ORBdist) (:2204-2336): the keyframe's slots (kf_mp,
 *   its keypoints for the angle) against the frame at Tcw; found = a byte per
 *   map point (sAlreadyFound); kp2mp / score in and out.
 * gf_reloc_candidates: KeyFrameDatabase::DetectRelocalisationCandidates
 *   (KeyFrameDatabase.cc:198-308) for a frame's BowVector against db's
 *   keyframes (kf_bad optional; cov_off / cov = mvpOrderedConnectedKeyFrames);
 *   query = the frame's mnId (!= 0); state (db->nkf entries) persists across
 *   queries as the keyframes' fields do. */
int gf_window_search(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                     const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, int n1, int window,
                     int min_level, int max_level, float nnratio, int check_ori, int32_t* out, int* nmatches);
int gf_search_frames(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                     const float* Tcw2, const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1,
                     const float* pos1, int n1, int window, float nnratio, int32_t* kp2mp, int32_t* score,
                     int* nmatches);
int gf_search_kf_projection(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                            const float* Tcw, const gf_keypoint* kf_kps, const int32_t* kf_mp, int nslots,
                            const gf_map_point* mps, const uint8_t* mp_desc, int nmp, const uint8_t* found, float th,
                            int orb_dist, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches);
int gf_reloc_candidates(gf_ctx* ctx, const int32_t* words, const double* values, int nwords, const gf_keyframe_db* db,
                        const uint8_t* kf_bad, const int32_t* cov_off, const int32_t* cov, uint32_t query,
                        gf_reloc_kf* state, int32_t* cands, int* ncand);
/* The keyframe graph of one stream's map (host arrays, gf_covis_map over the
 * map set with gf_frontend_set_map: g->nmp must equal its size; at most 64
 * keyframes, 64 x keypoint-capacity slots and observations). Once any stream
 * has a graph, every step first runs Tracking::UpdateReference
 * (Tracking.cc:2745, 3689-3852) on the frame's matches after
 * TrackWithMotionModel and tracks the rest of the frame against the local map
 * it returns (local keyframes' points, mvpLocalMapPoints order), so the local
 * map follows the camera; every stream then needs a graph. The map fields
 * (GF_FE_MAP, VIEWS, MP_*) keep indexing the stream's map, and GF_FE_LEFT /
 * GF_FE_KP2MP map indices. The bootstrap matches the whole map. */
int gf_frontend_set_covis(gf_frontend* fe, int stream, const gf_covis_map* graph);
/* Start of tracking: the current source frame of every stream is taken at the
 * given pose (Tcw [B][16]) and matched to its local map
 * (isInFrustum + SearchByProjection(F, local, 1) with nnratio 0.8); it becomes
 * mLastFrame with timestamp t0, V [B][16] the motion model, and the step
 * counter advances by one. */
int gf_frontend_bootstrap(gf_frontend* fe, const float* Tcw, const float* V, double t0);
/* Same with the B bootstrap frames from host memory ([B][height][width] u8),
 * for callers without a device frame source (then step with
 * gf_frontend_step_host). */
int gf_frontend_bootstrap_host(gf_frontend* fe, const uint8_t* imgs, const float* Tcw, const float* V, double t0);
/* One frame per stream from the source (asynchronous on the context stream). */
int gf_frontend_step(gf_frontend* fe);
/* gf_frontend_step in two calls: the extraction gate and Frame construction
 * (ORB extraction, undistortion; the Frame(...) of Tracking.cc:521), then tracking (Track()). Lets a caller stepping several
 * gated front ends from one thread enqueue every front end's extraction before
 * any tracking. Each call fails with GF_ERR_ARG out of order; gf_frontend_step
 * fails while an extracted frame awaits tracking. Not for captured front ends. */
int gf_frontend_step_extract(gf_frontend* fe);
int gf_frontend_step_track(gf_frontend* fe);
/* Same with the B frames taken from host memory ([B][height][width] u8):
 * the PCIe copy is part of the step. */
int gf_frontend_step_host(gf_frontend* fe, const uint8_t* imgs);
/* Capture gf_frontend_step as one HIP graph; later steps replay it (and
 * capture again when gf_set_budgets changed the budgets). While the graph
 * exists the context's scratch buffers are pinned: a call on the same context
 * that would need a larger one fails with GF_ERR_ARG instead of freeing
 * memory the graph uses. */
int gf_frontend_capture(gf_frontend* fe);
int gf_frontend_sync(gf_frontend* fe);
/* Copy a whole-batch field (synchronises; bytes must equal the field size). */
int gf_frontend_read(gf_frontend* fe, int field, void* host, size_t bytes);
int gf_frontend_write(gf_frontend* fe, int field, const void* host, size_t bytes);
/* Size and device pointer of a field. */
int gf_frontend_field(gf_frontend* fe, int field, size_t* bytes, void** d_ptr);

/* Wall-clock budgets of the reference's time-capped loops, in seconds; +inf
 * (the default) is parity mode: no loop is cut and no clock is read.
 *   match_s  = time_total_match (Tracking.cc:3230, 0.015 in the reference).
 *   select_s = the post-publish frame budget 1/(0.5 fps) - 0.002
 *              (Tracking.cc:866, 0.098 at 20 fps); timeCost_rest =
 *              select_s - timeCost_sofar.
 * Every cap is the reference's rule on the device's real-time clock
 * (s_memrealtime, 100 MHz ticks), each timer started where the reference
 * starts it, at the granularity given:
 *   isInFrustum loop (Tracking.cc:3251-3270): timer at the loop start; point i
 *     (skipping points matched this frame) cuts when its elapsed > match/2:
 *     points i.. go to mLeftMapPoints and leave mvpLocalMapPoints. Per point
 *     (a wave's 64 points read the clock once). time_Viz = the last value the
 *     loop compared.
 *   MAP_INFO build (Tracking.cc:3331 -> Observability.cc:564-578), cap
 *     (match - time_Viz)/2 on a timer started after the loop (:3311); per
 *     64-point batch.
 *   runActiveMapMatching (Tracking.cc:3343-3344 -> Observability.cc:1260,
 *     1275-1277, 1366-1370), cap match - time_Mat_Online - time_Viz (<= 0:
 *     the early exit); the clock is read at each round's start and the cut
 *     takes effect at that round's first accepted draw (where the reference
 *     first checks in a round): matches so far stand, no leftovers.
 *   timeCost_sofar from the frame's start (after the extraction gate wait,
 *     so queueing behind other front ends does not count).
 *   RunMapPointsSelection (Tracking.cc:1727-1779): returns when
 *     timeCost_rest <= 0, else MAP_INFO at kinematic[1] capped at
 *     timeCost_rest; per 64-point batch.
 *   SearchAdditionalMatchesInFrame (Tracking.cc:3097-3137): visibility pass
 *     cut at timeCost_rest/2 per list point (mLeftMapPoints erased from
 *     there); SearchByProjection_Budget (ORBmatcher.cc:281-282, 366-371)
 *     returns when timeCost_rest - time_so_far <= 0, else breaks after the
 *     first point that reaches its clock check with elapsed >= that
 *     (per point, elapsed from the matcher's start).
 * The elapsed values every rule compared are written to GF_FE_CLOCK, so a
 * CPU replay can apply the same rules (oracle/chain.cpp) and check the cut
 * positions rather than be told them. */
int gf_set_budgets(gf_ctx* ctx, double match_s, double select_s);

/* GF_FE_CLOCK record of one stream (int64 words, ticks of 10 ns; -1 = not
 * reached). M = map_cap, R = max(gf_budget, 1) (rounds <= num_to_match). */
enum {
    GF_CK_FLAGS = 0,    /* bit 0 match budget on, bit 1 select budget on   */
    GF_CK_MATCH,        /* time_total_match in ticks                        */
    GF_CK_SELECT,       /* select budget in ticks                           */
    GF_CK_VIZ_CUT,      /* isInFrustum: position of the cut (list size when none) */
    GF_CK_VIZ_TIME,     /* time_Viz                                         */
    GF_CK_MAT_ONLINE,   /* time_Mat_Online                                  */
    GF_CK_AM_CUT,       /* round at which the active-matching cap fired, -1 none */
    GF_CK_SOFAR,        /* timeCost_sofar                                   */
    GF_CK_SA_CUT,       /* visibility pass cut position in mLeftMapPoints (size when none) */
    GF_CK_SA_SOFAR,     /* time_so_far before SearchByProjection_Budget     */
    GF_CK_BUDGET_CUT,   /* list position SearchByProjection_Budget broke after, -1 none */
    GF_CK_HEADER = 16
};
#define GF_CK_OFF_VIZ(M, R) (GF_CK_HEADER)                       /* [M] isInFrustum, per list point  */
#define GF_CK_OFF_MI(M, R) (GF_CK_HEADER + (M))                  /* [64] MAP_INFO batches (active)    */
#define GF_CK_OFF_AM(M, R) (GF_CK_HEADER + (M) + 64)             /* [R] active-matching rounds        */
#define GF_CK_OFF_SEL(M, R) (GF_CK_HEADER + (M) + 64 + (R))      /* [64] MAP_INFO batches (kinematic[1]) */
#define GF_CK_OFF_SA(M, R) (GF_CK_HEADER + (M) + 128 + (R))      /* [M] visibility pass, per list point */
#define GF_CK_OFF_BUD(M, R) (GF_CK_HEADER + 2 * (M) + 128 + (R)) /* [M] SearchByProjection_Budget    */
#define GF_CK_WORDS(M, R) (GF_CK_HEADER + 3 * (M) + 128 + (R))
/* Test clock (test-only): every budget check reads base + idx * slope ticks
 * instead of the device clock, idx the check's position at its site (the
 * isInFrustum list point, the MAP_INFO 64-point batch, the active-matching
 * round, the SearchByProjection_Budget point; 0 for a site read once). With
 * it a chosen cap fires at a chosen point, so the budget rules are tested
 * without wall-clock luck; the clock record (GF_FE_CLOCK) holds the values
 * read, as with the device clock. base_slope: [GF_CK_NSITE][2] i64 ticks;
 * NULL restores the device clock. Set before a graph capture. */
enum {
    GF_CK_SITE_VIZ = 0,    /* isInFrustum loop, per list point (Tracking.cc:3262) */
    GF_CK_SITE_MI,         /* MAP_INFO batches of the active branch (Observability.cc:573) */
    GF_CK_SITE_AM_START,   /* time_Mat_Online at runActiveMapMatching's start (Tracking.cc:3311) */
    GF_CK_SITE_AM_ROUND,   /* runActiveMapMatching, per round (Observability.cc:1366) */
    GF_CK_SITE_SOFAR,      /* timeCost_sofar (Tracking.cc:866) */
    GF_CK_SITE_SEL,        /* RunMapPointsSelection's MAP_INFO batches (Tracking.cc:1779) */
    GF_CK_SITE_SA,         /* SearchAdditionalMatchesInFrame's visibility pass, per point (:3107-3119) */
    GF_CK_SITE_SA_SOFAR,   /* time_so_far before SearchByProjection_Budget (:3131) */
    GF_CK_SITE_BUD,        /* SearchByProjection_Budget, per point (ORBmatcher.cc:366) */
    GF_CK_NSITE
};
int gf_frontend_set_test_clock(gf_frontend* fe, const long long* base_slope);

/* Per-frame stage log: Tracking::logCurrentFrame / SaveTimeLog
 * (Tracking.h:254-280, filled at Tracking.cc:528, 605-615, 672, 913,
 * 2808-2814, 3143, 3339). With a log of `steps` entries on, each step
 * records the device real-time clock (s_memrealtime, 100 MHz) at its stage
 * boundaries (one 1-thread launch per boundary on the step's stream) and,
 * per stream, the counts the reference's landmark columns are made of; the
 * last `steps` steps are kept in a ring. The stages are batched: a boundary
 * is where the whole batch crossed it, so a column is the batch's time in
 * that stage, which every stream of the batch shares. Off (steps = 0) by
 * default: the step then launches nothing for it. Not while a captured graph
 * exists (capture again after changing it). */
enum {
    GF_TL_BEGIN = 0,     /* the frame's start, after the extraction gate         */
    GF_TL_EXTRACTED,     /* ORB extraction (+ undistortion) done                 */
    GF_TL_MOTION,        /* TrackWithMotionModel: SearchByProjection(Cur, Last) + PoseOptimization */
    GF_TL_INIT_POSE,     /* + TrackPreviousFrame / Relocalisation, outlier discard */
    GF_TL_REF_UPDATED,   /* TrackLocalMap: UpdateReference                       */
    GF_TL_FRUSTUM,       /* SearchReferencePointsInFrustum: FRAME_INFO, isInFrustum */
    GF_TL_MAT_ONLINE,    /* MAP_INFO_MATRIX (runMatrixBuilding, time_Mat_Online) */
    GF_TL_SELECTED,      /* runActiveMapMatching                                 */
    GF_TL_SEARCHED,      /* SearchByProjection(F, local) (end of SearchReferencePointsInFrustum) */
    GF_TL_OPTIMISED,     /* PoseOptimization + statistics (end of TrackLocalMap)  */
    GF_TL_END,           /* motion update, PWLS prediction, RunMapPointsSelection, SearchAdditionalMatchesInFrame, mLastFrame */
    GF_TL_NSITE = 12
};
typedef struct gf_time_rec {
    double frame_time_stamp; /* mCurrentFrame.mTimeStamp                          */
    int32_t path;            /* GF_TR_PATH of the step                             */
    int32_t branch;          /* GF_ST_BRANCH                                       */
    int32_t found;           /* GF_ST_FOUND: TrackWithMotionModel's nmatches        */
    int32_t tpf;             /* GF_ST_TPF: TrackPreviousFrame's nmatches            */
    int32_t local;           /* GF_ST_LOCAL                                        */
    int32_t inliers;         /* GF_ST_INL2: mnMatchesInliers                       */
    int32_t extra;           /* GF_ST_EXTRA                                        */
    int32_t track_map;       /* 1: TrackLocalMap ran                               */
    int32_t flags;           /* GF_ST_FLAGS                                        */
    int32_t step;            /* the front end's step counter of the record         */
} gf_time_rec;
int gf_frontend_set_time_log(gf_frontend* fe, int steps);
/* The ring in step order, oldest first: stamps [n][GF_TL_NSITE] i64 ticks
 * (0: not reached), recs [n][B]; n (<= steps) returned in *nsteps. */
int gf_frontend_read_time_log(gf_frontend* fe, long long* stamps, gf_time_rec* recs, int* nsteps);

/* ------------------------------------------------ multi-GPU start-up exchange
 * Config 5: one process per GPU, sequences independent,
 * and one exchange step before tracking: an RCCL communicator over xGMI and
 * broadcasts from rank 0 of the shared state. The reference has no
 * distributed layer (one process, main.cc:92-157); the vocabulary it loads
 * once (main.cc:92-106, TemplatedVocabulary.h:1469-1536) and the map it
 * tracks against are what every rank receives. The communicator uses the
 * context's device and stream; calls are synchronous. */
typedef struct gf_dist gf_dist;
/* ncclGetUniqueId on one rank (128 bytes); the caller hands it to the others. */
int gf_dist_unique_id(uint8_t* id);
int gf_dist_init(gf_ctx* ctx, int rank, int world, const uint8_t* id, gf_dist** out);
int gf_dist_destroy(gf_dist* d);
int gf_dist_info(gf_dist* d, int* rank, int* world);
/* Other transports behind the same entry points (gf_dist_bcast / _allreduce /
 * _bcast_vocab / _bcast_map work unchanged on them):
 * - loopback: the ranks are host threads of one process, each with its own
 *   context, meeting in a channel of `world` ranks; a broadcast is a
 *   rendezvous and a device-to-device copy from the root's buffer, an
 *   all-reduce a rank-ordered host reduction. Every rank's call blocks until
 *   all ranks have made the same call (120 s timeout, then GF_ERR_HIP and a
 *   broken channel). One GPU runs the receiving side of config 5 this way.
 * - host-staged: device -> host, fn(user, op, host_buf, bytes, root) does the
 *   collective on host memory (op GF_DIST_OP_BCAST from root; GF_DIST_OP_SUM /
 *   _MAX / _MIN in place over bytes / 8 doubles, root -1) and returns 0,
 *   host -> device. For processes that share a GPU (a gloo group). */
enum { GF_DIST_RCCL = 0, GF_DIST_LOOPBACK = 1, GF_DIST_HOST = 2 };
enum { GF_DIST_OP_BCAST = 0, GF_DIST_OP_SUM = 1, GF_DIST_OP_MAX = 2, GF_DIST_OP_MIN = 3 };
typedef struct gf_dist_channel gf_dist_channel;
typedef int (*gf_dist_host_fn)(void* user, int op, void* host_buf, size_t bytes, int root);
int gf_dist_channel_create(int world, gf_dist_channel** out);
int gf_dist_channel_destroy(gf_dist_channel* ch);
int gf_dist_init_loopback(gf_ctx* ctx, int rank, gf_dist_channel* ch, gf_dist** out);
int gf_dist_init_host(gf_ctx* ctx, int rank, int world, gf_dist_host_fn fn, void* user, gf_dist** out);
/* GF_DIST_RCCL / _LOOPBACK / _HOST */
int gf_dist_transport(gf_dist* d, int* transport);
/* Device buffer broadcast from root. */
int gf_dist_bcast(gf_dist* d, void* d_buf, size_t bytes, int root);
/* In-place all-reduce of n doubles: op 0 sum, 1 max, 2 min. */
int gf_dist_allreduce(gf_dist* d, double* d_buf, size_t n, int op);
/* The vocabulary of root into every rank (*voc == NULL on the others: a
 * vocabulary is created on the communicator's device). */
int gf_dist_bcast_vocab(gf_dist* d, gf_vocab** voc, int root);
/* Every stream's local map (gf_frontend_set_map state) of root's front end
 * into the same-shaped front ends of the other ranks. */
int gf_dist_bcast_map(gf_dist* d, gf_frontend* fe, int root);
/* Host copy of a device vocabulary's node arrays (any may be NULL). */
int gf_vocab_download(gf_vocab* voc, uint8_t* desc, double* weight, int32_t* word, int32_t* cstart);

#ifdef __cplusplus
}
#endif
#endif /* GFSLAM_ABI_H */
