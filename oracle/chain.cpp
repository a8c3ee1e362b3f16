// CPU oracle of the batched tracking front end (test infrastructure: only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline load it).
//
// One stream of gf_frontend_step restated sequentially on the oracle
// operators, in the call order of Tracking::GrabImage in the WORKING state
// (Tracking.cc:461-917; see include/gfslam/abi.h "batched tracking front
// end"): Frame -> TrackWithMotionModel (:1506-1642) -> TrackLocalMap
// (:2732-2844) with SearchReferencePointsInFrustum (:3149-3410) -> motion
// model (:729-738) -> predictPWLSVec + RunMapPointsSelection (:795-800,
// :1717-1779) -> SearchAdditionalMatchesInFrame (:3097-3145) -> outliers NULL
// and mLastFrame = mCurrentFrame (:899-907). State lives in the same field
// layouts as the device front end (B = 1), so a test can copy a device
// stream's state in, run one frame here and compare every field.
// Parity mode only: the time budgets are infinite.
#include <algorithm>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "oracle_common.h"

extern "C" {
int orc_extract_st(const uint8_t* img, int w, int h, int stride, int nfeatures, float scale_factor, int nlevels,
                   int score_type, int fast_th, gf_keypoint* kps, uint8_t* desc, int cap, int* n_out);
int orc_extract(const uint8_t* img, int w, int h, int stride, int nfeatures, float scale_factor, int nlevels,
                int fast_th, gf_keypoint* kps, uint8_t* desc, int cap, int* n_out);
int orc_extractor_plan(int w, int h, int nfeatures, float scale_factor, int nlevels, int* level_w, int* level_h,
                       int* feat_per_level, float* scales, int* umax16);
int orc_frustum(const gf_frame_info* fi, const float* Tcw, const gf_map_point* mps, int m, float viewCosLimit,
                gf_mp_view* views, int* n_in_view);
int orc_match_project(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                      const gf_mp_view* views, const uint8_t* mp_desc, int m, float th, float nnratio,
                      int32_t* kp2mp, int32_t* score, int* nmatches);
int orc_match_lastframe(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n, const float* Tcw,
                        const gf_keypoint* last_kps, const uint8_t* last_desc, const int32_t* last_kp2mp,
                        const uint8_t* last_outlier, const float* last_pos, int n_last, float th, int check_ori,
                        int32_t* kp2mp, int32_t* score, int* nmatches);
int orc_pose_opt(const float* Tcw_in, const float* X, const float* z, const int32_t* octave,
                 const float* inv_sigma2_levels, int n, float fx, float fy, float cx, float cy, float* Tcw_out,
                 uint8_t* outlier, int* ninliers, int* iterations);
int orc_obs_update(double t0, const float* Tcw0, double t1, const float* Twc1, double* Xv);
int orc_obs_predict(const double* Xv, double dt, int nseg, gf_kine* out);
int orc_obs_build_info(const gf_obs_camera* cam, const double* Xv, const float* pos, const float* sigma2, int n,
                       int check_viz, double* H, double* info, float* uv, uint8_t* valid);
int orc_obs_active_match_rng(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                             const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated,
                             const double* info, const double* H, int m, const double* base,
                             const float* level_sigma2, int num_to_match, float th, float nnratio, gf_rng* rng,
                             int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft, int* nmatched);
long long orc_last_ldets(void);
long long orc_cand_take(void);
int orc_undistort_keypoints(const float K[4], const float dist[5], const gf_keypoint* in, int n, gf_keypoint* out);
int orc_frame_bounds(const float K[4], const float dist[5], int w, int h, int b[4]);
int orc_obs_active_match_capped(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                                const gf_mp_view* views, const uint8_t* mp_desc, const uint8_t* updated,
                                const double* info, const double* H, int m, const double* base,
                                const float* level_sigma2, int num_to_match, float th, float nnratio, gf_rng* rng,
                                int32_t* kp2mp, int32_t* score, int32_t* left, int* nleft, int* nmatched,
                                const long long* round_el, int nrec, long long cap, int* cut_round);
int orc_match_project_list(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                           const gf_mp_view* views, const uint8_t* mp_desc, const int32_t* list, int nlist, float th,
                           float nnratio, int32_t* kp2mp, int32_t* score, int* nmatches, const long long* el,
                           long long constr2, int* cut);
int orc_update_reference(const gf_covis_map* M, int32_t* frame_mps, int nkp, int32_t* local_kfs, int* n_local_kfs,
                         int kf_cap, int32_t* local_mps, int* n_local_mps, int mp_cap, int32_t* ref_kf);
int orc_window_search(const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                      const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, int n1, int window,
                      int min_level, int max_level, float nnratio, int check_ori, int32_t* out, int* nmatches);
int orc_search_frames(const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2, const float* Tcw2,
                      const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, const float* pos1, int n1,
                      int window, float nnratio, int32_t* kp2mp, int32_t* score, int* nmatches);
int orc_search_kf_projection(const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                             const float* Tcw, const gf_keypoint* kf_kps, const int32_t* kf_mp, int nslots,
                             const gf_map_point* mps, const uint8_t* mp_desc, const uint8_t* found, float th,
                             int orb_dist, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches);
int orc_bow_transform(int k, int L, int scoring, int weighting, int nnodes, const int32_t* parent,
                      const uint8_t* desc, const double* weight, const uint8_t* is_leaf, const uint8_t* feats, int n,
                      int levelsup, int32_t* words, double* values, int* nwords, int32_t* fv_nodes, int32_t* fv_start,
                      int32_t* fv_feats, int* nfv);
int orc_match_bow(int mode, float nnratio, int check_ori, const int32_t* a_nodes, const int32_t* a_start,
                  const int32_t* a_feats, int a_nn, const uint8_t* a_desc, const float* a_angle, const int32_t* a_mp,
                  int a_n, const int32_t* b_nodes, const int32_t* b_start, const int32_t* b_feats, int b_nn,
                  const uint8_t* b_desc, const float* b_angle, const int32_t* b_mp, int b_n, int32_t* out,
                  int* nmatches);
int orc_reloc_candidates(const int32_t* words, const double* values, int nwords, int nkf, const uint8_t* kf_bad,
                         const int32_t* bow_off, const int32_t* bow_words, const double* bow_values,
                         const int32_t* cov_off, const int32_t* cov, uint32_t query, uint32_t* reloc_query,
                         int32_t* reloc_words, float* reloc_score, int32_t* cands, int* ncand);
int orc_pnp_init(int n, const gf_pnp_params* p, gf_pnp_state* st);
int orc_pnp_iterate(const float* p3d, const float* p2d, const float* sigma2, const float K[4], gf_pnp_state* st,
                    uint8_t* best_mask, int n_iterations, gf_rng* rng, float* Tcw, uint8_t* inliers, int32_t* ninliers,
                    int32_t* flags);
}

namespace {

// glibc srand(): the oracle's own restatement for seeding (TYPE_3, 310 discards)
void rng_seed(gf_rng* r, uint32_t s) {
    if (s == 0) s = 1;
    r->state[0] = (int32_t)s;
    int32_t word = (int32_t)s;
    for (int i = 1; i < 31; ++i) {
        long long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        r->state[i] = word;
    }
    r->f = 3;
    r->r = 0;
    for (int k = 0; k < 310; k++) {
        uint32_t val = (uint32_t)r->state[r->f] + (uint32_t)r->state[r->r];
        r->state[r->f] = (int32_t)val;
        if (++r->f >= 31) {
            r->f = 0;
            ++r->r;
        } else if (++r->r >= 31) {
            r->r = 0;
        }
    }
}

void mat44(const float* a, const float* b, float* o) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) o[4 * i + j] = orc::dot4(a + 4 * i, 1, b + j, 4);
}

// Frame::getTwc (Frame.cc:152-163) and LastTwc (Tracking.cc:731-735):
// Rwc = R^T, twc = -Rwc * t.
void twc_of(const float* T, float* W) {
    for (int i = 0; i < 16; i++) W[i] = (i % 5 == 0) ? 1.f : 0.f;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) W[4 * i + j] = T[4 * j + i];
        W[4 * i + 3] = orc::dot3(-T[i], T[3], -T[4 + i], T[7], -T[8 + i], T[11]);
    }
}

}  // namespace

struct orc_chain {
    gf_frontend_params p{};
    int cap = 0, M = 0;
    gf_frame_info fi{};
    gf_obs_camera oc{};
    float inv_sigma2[16] = {}, level_sigma2[16] = {};
    // fields (B = 1), layouts as gf_frontend
    std::vector<gf_keypoint> kps, last_kps;
    std::vector<uint8_t> desc, last_desc, outl, last_outl, map_desc;
    int32_t nkp = 0, last_nkp = 0, nmp = 0;
    float Tcw[16] = {}, Tcw_last[16] = {}, V[16] = {};
    std::vector<int32_t> kp2mp, score, last_kp2mp, upd, left;
    std::vector<float> last_pos, mp_uv;
    double t_prev = 0, t_cur = 0;
    std::vector<gf_map_point> map;
    std::vector<gf_mp_view> views;
    double Xv[13] = {}, Xv_next[13] = {}, base[49] = {};
    std::vector<double> mp_H, mp_info;
    gf_rng rng{};
    int32_t stats[GF_FE_NSTAT] = {};
    double tm[8] = {};  // stage seconds of the last step
    // time budgets (orc_chain_set_clock): the clock record of the step to
    // replay (GF_FE_CLOCK of one device stream); the cap rules of
    // gf_set_budgets run on the elapsed times it holds. Empty: parity mode.
    std::vector<long long> clk;
    int ck_R = 1;
    // keyframe graph (orc_chain_set_covis): UpdateReference every step, the
    // frame tracked against the local map gathered from the stream map
    int refmap = 0, g_nkf = 0;
    std::vector<uint8_t> g_kf_bad, g_mp_bad;
    std::vector<int32_t> g_kf_mp_off, g_kf_mp, g_kf_cov_off, g_kf_cov, g_mp_obs_off, g_mp_obs;
    // the tracking state machine (GF_FE_TRACK) and the keyframes' query state (GF_FE_RELOC)
    int32_t track[GF_TR_N] = {};
    gf_reloc_kf rkf[64] = {};
    int max_frames = 12;
    // keyframe database (orc_chain_set_kfdb) and vocabulary (orc_chain_set_vocab)
    int has_kfdb = 0;
    std::vector<int32_t> k_kp_off, k_bow_off, k_bow_words, k_fv_off, k_fv_nodes, k_fv_start, k_fv_feats;
    std::vector<gf_keypoint> k_kps;
    std::vector<uint8_t> k_desc;
    std::vector<double> k_bow_values;
    int has_vocab = 0;
    int v_k = 0, v_L = 0, v_scoring = 0, v_weighting = 0, v_nnodes = 0;
    std::vector<int32_t> v_parent;
    std::vector<uint8_t> v_desc, v_leaf;
    std::vector<double> v_weight;
};

namespace {
// The map-point arrays of a chain: the stream map, or a step's local map.
struct MapState {
    std::vector<gf_map_point> map;
    std::vector<uint8_t> desc;
    std::vector<gf_mp_view> views;
    std::vector<double> H, info;
    std::vector<float> uv;
    std::vector<int32_t> upd;
    int32_t nmp = 0;
};

void take_map(orc_chain* c, MapState& s) {
    s.map.swap(c->map);
    s.desc.swap(c->map_desc);
    s.views.swap(c->views);
    s.H.swap(c->mp_H);
    s.info.swap(c->mp_info);
    s.uv.swap(c->mp_uv);
    s.upd.swap(c->upd);
    std::swap(s.nmp, c->nmp);
}
}  // namespace

namespace {

void field(orc_chain* c, int f, void** ptr, size_t* bytes) {
    *ptr = nullptr;
    *bytes = 0;
#define FV(v) (*ptr = (void*)c->v.data(), *bytes = sizeof(c->v[0]) * c->v.size())
#define FS(v) (*ptr = (void*)&c->v, *bytes = sizeof(c->v))
    switch (f) {
        case GF_FE_KPS: FV(kps); break;
        case GF_FE_DESC: FV(desc); break;
        case GF_FE_NKP: FS(nkp); break;
        case GF_FE_TCW: FS(Tcw); break;
        case GF_FE_KP2MP: FV(kp2mp); break;
        case GF_FE_SCORE: FV(score); break;
        case GF_FE_OUTLIER: FV(outl); break;
        case GF_FE_LAST_KPS: FV(last_kps); break;
        case GF_FE_LAST_DESC: FV(last_desc); break;
        case GF_FE_LAST_NKP: FS(last_nkp); break;
        case GF_FE_LAST_KP2MP: FV(last_kp2mp); break;
        case GF_FE_LAST_OUTLIER: FV(last_outl); break;
        case GF_FE_LAST_POS: FV(last_pos); break;
        case GF_FE_TCW_LAST: FS(Tcw_last); break;
        case GF_FE_VELOCITY: FS(V); break;
        case GF_FE_T_PREV: FS(t_prev); break;
        case GF_FE_T_CUR: FS(t_cur); break;
        case GF_FE_MAP: FV(map); break;
        case GF_FE_MAP_DESC: FV(map_desc); break;
        case GF_FE_NMP: FS(nmp); break;
        case GF_FE_VIEWS: FV(views); break;
        case GF_FE_XV: FS(Xv); break;
        case GF_FE_XV_NEXT: FS(Xv_next); break;
        case GF_FE_BASE: FS(base); break;
        case GF_FE_MP_H: FV(mp_H); break;
        case GF_FE_MP_INFO: FV(mp_info); break;
        case GF_FE_MP_UV: FV(mp_uv); break;
        case GF_FE_MP_UPD: FV(upd); break;
        case GF_FE_RNG: FS(rng); break;
        case GF_FE_LEFT: FV(left); break;
        case GF_FE_STATS: FS(stats); break;
        case GF_FE_TRACK: FS(track); break;
        case GF_FE_RELOC: FS(rkf); break;
        default: break;
    }
#undef FV
#undef FS
}

// batchInfoMat_Map (Observability.cc:556-644) over points i < m of the map:
// skip those stamped fid and (check_viz == 0) those not in view; stamp the
// valid ones. Returns updated flags (updateAtFrameId == fid). With a time cap
// (bel != null) the 64-point batch w is skipped when 2 x bel[w] > cap2
// (:573-578 on the device's per-batch clock reads); *late = a batch was.
void map_info(orc_chain* c, const double* Xv, int m, int check_viz, int fid, std::vector<uint8_t>* updated,
              const long long* bel = nullptr, long long cap2 = 0, bool* late = nullptr) {
    if (late) *late = false;
    if (bel && late)
        for (int w = 0; w * 64 < m; w++) *late = *late || 2 * bel[w] > cap2;
    // runMatrixBuilding (Observability.cc:646-713): hardware_concurrency equal
    // grains of the point list, one std::thread each (ORC_THREADS overrides)
    auto grain = [&](int lo, int hi) {
        for (int i = lo; i < hi; i++) {
            if (bel && 2 * bel[i >> 6] > cap2) continue;
            if (c->upd[i] == fid) continue;
            if (!check_viz && !c->views[i].in_view) continue;
            double H[14], info[49];
            float uv[2];
            uint8_t valid = 0;
            orc_obs_build_info(&c->oc, Xv, c->map[i].pos, nullptr, 1, check_viz, H, info, uv, &valid);
            if (!valid) continue;
            std::memcpy(&c->mp_H[14 * (size_t)i], H, sizeof(H));
            std::memcpy(&c->mp_info[49 * (size_t)i], info, sizeof(info));
            c->mp_uv[2 * i] = uv[0];
            c->mp_uv[2 * i + 1] = uv[1];
            c->upd[i] = fid;
        }
    };
    int nt = (int)std::thread::hardware_concurrency();
    if (const char* e = std::getenv("ORC_THREADS")) nt = std::atoi(e);
    nt = std::max(1, std::min(nt, m / 64));
    if (nt <= 1) {
        grain(0, m);
    } else {
        std::vector<std::thread> th;
        const int step = (m + nt - 1) / nt;
        for (int t = 0; t < nt; t++) th.emplace_back(grain, t * step, std::min(m, (t + 1) * step));
        for (auto& x : th) x.join();
    }
    if (updated) {
        updated->assign(c->M, 0);
        for (int i = 0; i < c->nmp; i++) (*updated)[i] = c->upd[i] == fid;
    }
}

// Optimizer::PoseOptimization over the matched keypoints, in keypoint order.
void pose(orc_chain* c, int* ninl, int* iters, int* nedges) {
    std::vector<float> X, z;
    std::vector<int32_t> oct, idx;
    for (int i = 0; i < c->nkp; i++) {
        const int mp = c->kp2mp[i];
        if (mp < 0) continue;
        for (int k = 0; k < 3; k++) X.push_back(c->map[mp].pos[k]);
        z.push_back(c->kps[i].x);
        z.push_back(c->kps[i].y);
        oct.push_back(c->kps[i].octave);
        idx.push_back(i);
    }
    const int n = (int)idx.size();
    std::vector<uint8_t> o(n + 1);
    float T[16];
    int ni = 0, it = 0;
    orc_pose_opt(c->Tcw, X.data(), z.data(), oct.data(), c->inv_sigma2, n, c->fi.fx, c->fi.fy, c->fi.cx, c->fi.cy, T,
                 o.data(), &ni, &it);
    std::memcpy(c->Tcw, T, sizeof(T));
    for (int e = 0; e < n; e++) c->outl[idx[e]] = o[e];
    *ninl = ni;
    *iters = it;
    *nedges = n;
}

// Matches flagged as outliers set NULL (flags reset with reset: the loops of
// TrackPreviousFrame; Relocalisation's keep them). Returns the count.
int discard(orc_chain* c, bool reset) {
    int cnt = 0;
    for (int i = 0; i < c->nkp; i++)
        if (c->outl[i] && c->kp2mp[i] >= 0) {
            c->kp2mp[i] = -1;
            if (reset) c->outl[i] = 0;
            cnt++;
        }
    return cnt;
}

int pose_n(orc_chain* c) {
    int ni = 0, it = 0, ne = 0;
    pose(c, &ni, &it, &ne);
    return ni;
}

// Tracking::TrackPreviousFrame (Tracking.cc:1325-1404): mTcw = mLastFrame.mTcw
// and no matches on entry.
bool track_previous_frame(orc_chain* c) {
    const int n = c->nkp;
    const int kfc = c->refmap ? c->g_nkf : -1;  // KeyFramesInMap (no graph: assumed > 5)
    const int minOctave = (kfc < 0 || kfc > 5) ? (c->p.nlevels - 1) / 2 + 1 : 0;
    int nm = 0;
    orc_window_search(&c->fi, c->kps.data(), c->desc.data(), n, c->last_kps.data(), c->last_desc.data(),
                      c->last_kp2mp.data(), c->last_nkp, 200, minOctave, INT_MAX, 0.9f, 1, c->kp2mp.data(), &nm);
    if (nm < 10) {
        orc_window_search(&c->fi, c->kps.data(), c->desc.data(), n, c->last_kps.data(), c->last_desc.data(),
                          c->last_kp2mp.data(), c->last_nkp, 100, 0, INT_MAX, 0.9f, 1, c->kp2mp.data(), &nm);
        if (nm < 10) {
            std::fill(c->kp2mp.begin(), c->kp2mp.begin() + n, -1);
            nm = 0;
        }
    }
    int k = 0;
    if (nm >= 10) {
        pose_n(c);
        nm -= discard(c, true);
        orc_search_frames(&c->fi, c->kps.data(), c->desc.data(), n, c->Tcw, c->last_kps.data(), c->last_desc.data(),
                          c->last_kp2mp.data(), c->last_pos.data(), c->last_nkp, 15, 0.9f, c->kp2mp.data(),
                          c->score.data(), &k);
        nm += k;
    } else {  // last opportunity
        orc_search_frames(&c->fi, c->kps.data(), c->desc.data(), n, c->Tcw, c->last_kps.data(), c->last_desc.data(),
                          c->last_kp2mp.data(), c->last_pos.data(), c->last_nkp, 50, 0.9f, c->kp2mp.data(),
                          c->score.data(), &k);
        nm = k;
    }
    if (nm >= 10) {
        pose_n(c);
        nm -= discard(c, true);
    }
    c->stats[GF_ST_TPF] = nm;
    return nm >= 10;
}

// Tracking::Relocalisation (Tracking.cc:3854-4031) against the chain's
// keyframe database.
bool relocalise(orc_chain* c) {
    if (!c->has_kfdb || !c->has_vocab) return false;
    const int n = c->nkp, cap = c->cap;
    // Frame::ComputeBoW (levelsup 4)
    std::vector<int32_t> words(std::max(n, 1)), fvn(std::max(n, 1)), fvs(n + 1), fvf(std::max(n, 1));
    std::vector<double> values(std::max(n, 1));
    int nw = 0, nfv = 0;
    orc_bow_transform(c->v_k, c->v_L, c->v_scoring, c->v_weighting, c->v_nnodes, c->v_parent.data(), c->v_desc.data(),
                      c->v_weight.data(), c->v_leaf.data(), c->desc.data(), n, 4, words.data(), values.data(), &nw,
                      fvn.data(), fvs.data(), fvf.data(), &nfv);
    // DetectRelocalisationCandidates
    const int nkf = c->g_nkf;
    std::vector<uint32_t> rq(nkf);
    std::vector<int32_t> rw(nkf), cands(64);
    std::vector<float> rs(nkf);
    for (int k = 0; k < nkf; k++) {
        rq[k] = c->rkf[k].query;
        rw[k] = c->rkf[k].words;
        rs[k] = c->rkf[k].score;
    }
    int nc = 0;
    orc_reloc_candidates(words.data(), values.data(), nw, nkf, c->g_kf_bad.data(), c->k_bow_off.data(),
                         c->k_bow_words.data(), c->k_bow_values.data(), c->g_kf_cov_off.data(), c->g_kf_cov.data(),
                         (uint32_t)c->track[GF_TR_QUERY], rq.data(), rw.data(), rs.data(), cands.data(), &nc);
    for (int k = 0; k < nkf; k++) c->rkf[k] = gf_reloc_kf{rq[k], rw[k], rs[k]};
    c->stats[GF_ST_NCAND] = nc;
    if (nc == 0) return false;
    // ORBmatcher(0.75, true).SearchByBoW per candidate, a PnPsolver for >= 15
    std::vector<std::vector<int32_t>> match(nc, std::vector<int32_t>(std::max(n, 1), -1));
    std::vector<gf_pnp_state> st(nc);
    std::vector<std::vector<uint8_t>> best(nc, std::vector<uint8_t>(std::max(n, 1), 0));
    std::vector<char> disc(nc, 0);
    std::vector<float> fangle(std::max(n, 1));
    for (int i = 0; i < n; i++) fangle[i] = c->kps[i].angle;
    std::vector<int32_t> none(std::max(n, 1), -1);
    const gf_pnp_params prm{0.99, 10, 300, 4, 0.5f, 5.991f};
    std::vector<float> p3d(3 * (size_t)std::max(n, 1)), p2d(2 * (size_t)std::max(n, 1)), s2(std::max(n, 1));
    std::vector<int32_t> pidx(std::max(n, 1));
    auto corr = [&](int i) {  // PnPsolver ctor :50-73
        int N = 0;
        for (int j = 0; j < n; j++) {
            const int mp = match[i][j];
            if (mp < 0) continue;
            for (int q = 0; q < 3; q++) p3d[3 * N + q] = c->map[mp].pos[q];
            p2d[2 * N] = c->kps[j].x;
            p2d[2 * N + 1] = c->kps[j].y;
            s2[N] = c->level_sigma2[c->kps[j].octave];
            pidx[N] = j;
            N++;
        }
        return N;
    };
    int nCandidates = 0;
    for (int i = 0; i < nc; i++) {
        const int kf = cands[i];
        if (c->g_kf_bad[kf]) {
            disc[i] = 1;
            continue;
        }
        const int a0 = c->k_fv_off[kf], ann = c->k_fv_off[kf + 1] - a0, k0 = c->k_kp_off[kf];
        const int akn = c->k_kp_off[kf + 1] - k0;
        std::vector<float> aangle(std::max(akn, 1));
        for (int j = 0; j < akn; j++) aangle[j] = c->k_kps[k0 + j].angle;
        int nmb = 0;
        orc_match_bow(0, 0.75f, 1, c->k_fv_nodes.data() + a0, c->k_fv_start.data() + a0, c->k_fv_feats.data(), ann,
                      c->k_desc.data() + 32 * (size_t)k0, aangle.data(), c->g_kf_mp.data() + c->g_kf_mp_off[kf], akn,
                      fvn.data(), fvs.data(), fvf.data(), nfv, c->desc.data(), fangle.data(), none.data(), n,
                      match[i].data(), &nmb);
        if (nmb < 15) {
            disc[i] = 1;
            continue;
        }
        orc_pnp_init(corr(i), &prm, &st[i]);
        nCandidates++;
    }
    const float K[4] = {c->p.fx, c->p.fy, c->p.cx, c->p.cy};
    bool bMatch = false;
    int attempts = 0, nGood = 0;
    std::vector<uint8_t> found(c->nmp, 0), inl(std::max(n, 1));
    auto mark = [&]() {
        std::fill(found.begin(), found.end(), 0);
        for (int j = 0; j < n; j++)
            if (c->kp2mp[j] >= 0) found[c->kp2mp[j]] = 1;
    };
    while (nCandidates > 0 && !bMatch) {
        for (int i = 0; i < nc; i++) {
            if (disc[i]) continue;
            const int N = corr(i);
            float T[16];
            int32_t ninl = 0, fl = 0;
            orc_pnp_iterate(p3d.data(), p2d.data(), s2.data(), K, &st[i], best[i].data(), 5, &c->rng, T, inl.data(),
                            &ninl, &fl);
            attempts++;
            if (fl & GF_PNP_NOMORE) {
                disc[i] = 1;
                nCandidates--;
            }
            if (!(fl & GF_PNP_FOUND)) continue;
            std::memcpy(c->Tcw, T, sizeof(T));
            std::fill(c->kp2mp.begin(), c->kp2mp.begin() + n, -1);
            for (int q = 0; q < N; q++)
                if (inl[q]) c->kp2mp[pidx[q]] = match[i][pidx[q]];
            mark();  // sFound
            nGood = pose_n(c);
            if (nGood < 10) continue;
            discard(c, false);
            if (nGood < 50) {
                const int kf = cands[i];
                const int k0 = c->k_kp_off[kf], nsl = c->k_kp_off[kf + 1] - k0;
                const int32_t* kmp = c->g_kf_mp.data() + c->g_kf_mp_off[kf];
                int nadd = 0;
                orc_search_kf_projection(&c->fi, c->kps.data(), c->desc.data(), n, c->Tcw, c->k_kps.data() + k0, kmp,
                                         nsl, c->map.data(), c->map_desc.data(), found.data(), 10.f, 100, 1,
                                         c->kp2mp.data(), c->score.data(), &nadd);
                if (nadd + nGood >= 50) {
                    nGood = pose_n(c);
                    if (nGood > 30 && nGood < 50) {
                        mark();
                        orc_search_kf_projection(&c->fi, c->kps.data(), c->desc.data(), n, c->Tcw,
                                                 c->k_kps.data() + k0, kmp, nsl, c->map.data(), c->map_desc.data(),
                                                 found.data(), 3.f, 64, 1, c->kp2mp.data(), c->score.data(), &nadd);
                        if (nGood + nadd >= 50) {
                            nGood = pose_n(c);
                            discard(c, false);
                        }
                    }
                }
            }
            if (nGood >= 50) {
                bMatch = true;
                break;
            }
        }
    }
    (void)cap;
    c->stats[GF_ST_RELOC] = nGood;
    c->stats[GF_ST_RANSAC] = attempts;
    return bMatch;
}

// isInFrustum on the points of a list (others untouched).
void frustum_list(orc_chain* c, const int32_t* list, int n) {
    for (int k = 0; k < n; k++) {
        const int i = list[k];
        int cnt = 0;
        orc_frustum(&c->fi, c->Tcw, &c->map[i], 1, 0.5f, &c->views[i], &cnt);
    }
}

}  // namespace

extern "C" {

orc_chain* orc_chain_create(const gf_frontend_params* p) {
    orc_chain* c = new orc_chain();
    c->p = *p;
    int lw[16], lh[16], fpl[16], um[16];
    float sc[16];
    orc_extractor_plan(p->width, p->height, p->nfeatures, p->scale_factor, p->nlevels, lw, lh, fpl, sc, um);
    c->cap = 0;
    for (int l = 0; l < p->nlevels; l++) c->cap += fpl[l];
    c->M = p->map_cap;
    c->ck_R = std::max(p->gf_budget, 1);
    // Frame::ComputeImageBounds (Frame.cc:425-493)
    const float K[4] = {p->fx, p->fy, p->cx, p->cy};
    int bnd[4];
    orc_frame_bounds(K, p->dist, p->width, p->height, bnd);
    c->fi = gf_frame_info{bnd[0], bnd[1], bnd[2], bnd[3], p->fx, p->fy, p->cx, p->cy, p->nlevels, p->scale_factor};
    float sf = 1.f;
    for (int l = 0; l < p->nlevels; l++) {
        if (l) sf = sf * p->scale_factor;
        c->level_sigma2[l] = sf * sf;
        c->inv_sigma2[l] = 1.0f / (sf * sf);
    }
    gf_obs_camera& oc = c->oc;
    oc.fu = p->fx;
    oc.fv = p->fy;
    oc.cx = p->cx;
    oc.cy = p->cy;
    oc.nrows = p->height;
    oc.ncols = p->width;
    oc.min_x = bnd[0];
    oc.max_x = bnd[1];
    oc.min_y = bnd[2];
    oc.max_y = bnd[3];
    // mBoundXInFrame / mBoundYInFrame (Tracking.cc:876-877)
    oc.bound_x = (int)((bnd[1] - bnd[0]) * 0.1);
    oc.bound_y = (int)((bnd[3] - bnd[2]) * 0.1);
    oc.bound_depth = 0.f;
    const size_t cap = c->cap, M = c->M;
    c->kps.assign(cap, gf_keypoint{});
    c->last_kps.assign(cap, gf_keypoint{});
    c->desc.assign(cap * 32, 0);
    c->last_desc.assign(cap * 32, 0);
    c->outl.assign(cap, 0);
    c->last_outl.assign(cap, 0);
    c->kp2mp.assign(cap, 0);
    c->score.assign(cap, 0);
    c->last_kp2mp.assign(cap, 0);
    c->last_pos.assign(cap * 3, 0.f);
    c->map.assign(M, gf_map_point{});
    c->map_desc.assign(M * 32, 0);
    c->views.assign(M, gf_mp_view{});
    c->upd.assign(M, -1000);
    c->left.assign(M, 0);
    c->mp_uv.assign(M * 2, 0.f);
    c->mp_H.assign(M * 14, 0.0);
    c->mp_info.assign(M * 49, 0.0);
    for (int i = 0; i < 4; i++) c->Tcw_last[5 * i] = c->V[5 * i] = 1.f;
    rng_seed(&c->rng, 1);
    c->max_frames = p->max_frames > 0 ? p->max_frames : (int)(18.0 / (30.0 * p->dt) + 1e-6);  // 18 * fps / 30
    return c;
}

void orc_chain_destroy(orc_chain* c) { delete c; }

int orc_chain_capacity(orc_chain* c) { return c->cap; }

int orc_chain_read(orc_chain* c, int f, void* host, size_t bytes) {
    void* p;
    size_t b;
    field(c, f, &p, &b);
    if (!p || b != bytes) return GF_ERR_ARG;
    std::memcpy(host, p, b);
    return GF_OK;
}

int orc_chain_write(orc_chain* c, int f, const void* host, size_t bytes) {
    void* p;
    size_t b;
    field(c, f, &p, &b);
    if (!p || b != bytes) return GF_ERR_ARG;
    std::memcpy(p, host, b);
    return GF_OK;
}

int orc_chain_set_map(orc_chain* c, const gf_map_point* mps, const uint8_t* desc, int m) {
    if (m < 0 || m > c->M) return GF_ERR_ARG;
    std::memcpy(c->map.data(), mps, sizeof(gf_map_point) * m);
    std::memcpy(c->map_desc.data(), desc, 32 * (size_t)m);
    c->nmp = m;
    std::fill(c->upd.begin(), c->upd.end(), -1000);
    std::fill(c->views.begin(), c->views.end(), gf_mp_view{});
    return GF_OK;
}

int orc_chain_set_rng(orc_chain* c, uint32_t seed) {
    rng_seed(&c->rng, seed);
    return GF_OK;
}

static int extract(orc_chain* c, const uint8_t* img) {
    int n = 0;
    int rc = orc_extract_st(img, c->p.width, c->p.height, c->p.width, c->p.nfeatures, c->p.scale_factor,
                            c->p.nlevels, c->p.harris_score ? 0 : 1, c->p.fast_th, c->kps.data(), c->desc.data(),
                            c->cap, &n);
    c->nkp = n;
    // mvKeysUn (Frame::UndistortKeyPoints, Frame.cc:389-423; a copy when k1 == 0)
    const float K[4] = {c->p.fx, c->p.fy, c->p.cx, c->p.cy};
    if (rc == GF_OK) orc_undistort_keypoints(K, c->p.dist, c->kps.data(), n, c->kps.data());
    return rc;
}

static void make_last(orc_chain* c) {
    const int n = c->nkp;
    for (int i = 0; i < n; i++) {
        const int mp = c->kp2mp[i];
        c->last_kp2mp[i] = mp;
        c->last_outl[i] = c->outl[i];
        c->last_kps[i] = c->kps[i];
        for (int k = 0; k < 3; k++) c->last_pos[3 * i + k] = mp >= 0 ? c->map[mp].pos[k] : 0.f;
    }
    std::memcpy(c->last_desc.data(), c->desc.data(), 32 * (size_t)n);
    c->last_nkp = n;
    std::memcpy(c->Tcw_last, c->Tcw, sizeof(c->Tcw));
    c->t_prev = c->t_cur;
}

int orc_chain_bootstrap(orc_chain* c, const uint8_t* img, const float* Tcw, const float* V, double t0) {
    std::memcpy(c->Tcw, Tcw, sizeof(c->Tcw));
    std::memcpy(c->V, V, sizeof(c->V));
    c->t_cur = t0;
    std::fill(c->kp2mp.begin(), c->kp2mp.end(), -1);
    std::fill(c->score.begin(), c->score.end(), 999);
    std::fill(c->outl.begin(), c->outl.end(), 0);
    int rc = extract(c, img);
    if (rc) return rc;
    int nv = 0, nm = 0;
    orc_frustum(&c->fi, c->Tcw, c->map.data(), c->nmp, 0.5f, c->views.data(), &nv);
    orc_match_project(&c->fi, c->kps.data(), c->desc.data(), c->nkp, c->views.data(), c->map_desc.data(), c->nmp, 1.f,
                      0.8f, c->kp2mp.data(), c->score.data(), &nm);
    make_last(c);
    c->track[GF_TR_STATE] = 0;  // WORKING, a velocity, no relocalisation so far
    c->track[GF_TR_VEL] = 1;
    c->track[GF_TR_SINCE] = 1 << 30;
    c->track[GF_TR_PATH] = 0;
    c->track[GF_TR_OK] = 1;
    return GF_OK;
}

// The keyframe database of the chain's keyframe graph (gf_keyframe_db arrays).
int orc_chain_set_kfdb(orc_chain* c, const gf_keyframe_db* db) {
    if (!db) {
        c->has_kfdb = 0;
        std::memset(c->rkf, 0, sizeof(c->rkf));
        return GF_OK;
    }
    if (!c->refmap || db->nkf != c->g_nkf || db->nkf > 64) return GF_ERR_ARG;
    const int nkf = db->nkf;
    const int nk = nkf ? db->kp_off[nkf] : 0, nb = nkf ? db->bow_off[nkf] : 0, nn = nkf ? db->fv_off[nkf] : 0;
    const int nf = nkf ? db->fv_start[nn] : 0;
    c->k_kp_off.assign(db->kp_off, db->kp_off + nkf + 1);
    c->k_kps.assign(db->kps, db->kps + nk);
    c->k_desc.assign(db->desc, db->desc + 32 * (size_t)nk);
    c->k_bow_off.assign(db->bow_off, db->bow_off + nkf + 1);
    c->k_bow_words.assign(db->bow_words, db->bow_words + nb);
    c->k_bow_values.assign(db->bow_values, db->bow_values + nb);
    c->k_fv_off.assign(db->fv_off, db->fv_off + nkf + 1);
    c->k_fv_nodes.assign(db->fv_nodes, db->fv_nodes + nn);
    c->k_fv_start.assign(db->fv_start, db->fv_start + nn + 1);
    c->k_fv_feats.assign(db->fv_feats, db->fv_feats + nf);
    for (int k = 0; k < nkf; k++)
        if (c->k_kp_off[k + 1] - c->k_kp_off[k] != c->g_kf_mp_off[k + 1] - c->g_kf_mp_off[k]) return GF_ERR_ARG;
    c->has_kfdb = 1;
    std::memset(c->rkf, 0, sizeof(c->rkf));
    return GF_OK;
}

int orc_chain_set_vocab(orc_chain* c, int k, int L, int scoring, int weighting, int nnodes, const int32_t* parent,
                        const uint8_t* desc, const double* weight, const uint8_t* is_leaf) {
    c->v_k = k;
    c->v_L = L;
    c->v_scoring = scoring;
    c->v_weighting = weighting;
    c->v_nnodes = nnodes;
    c->v_parent.assign(parent, parent + nnodes);
    c->v_desc.assign(desc, desc + 32 * (size_t)nnodes);
    c->v_weight.assign(weight, weight + nnodes);
    c->v_leaf.assign(is_leaf, is_leaf + nnodes);
    c->has_vocab = nnodes > 1;
    return GF_OK;
}

// The clock record of the next step (n = GF_CK_WORDS(map_cap, max(budget, 1))
// int64 words; n = 0 clears it: parity mode).
int orc_chain_set_clock(orc_chain* c, const long long* rec, size_t n) {
    if (n == 0) {
        c->clk.clear();
        return GF_OK;
    }
    if (!rec || n != (size_t)GF_CK_WORDS((long long)c->M, (long long)c->ck_R)) return GF_ERR_ARG;
    c->clk.assign(rec, rec + n);
    return GF_OK;
}

// The keyframe graph over the chain's map (gf_frontend_set_covis).
int orc_chain_set_covis(orc_chain* c, const gf_covis_map* g) {
    if (!g || g->nmp != c->nmp || g->nkf < 0) return GF_ERR_ARG;
    const int nkf = g->nkf, nmp = g->nmp;
    const size_t ns = nkf ? g->kf_mp_off[nkf] : 0, nc = nkf ? g->kf_cov_off[nkf] : 0, no = nmp ? g->mp_obs_off[nmp] : 0;
    c->g_nkf = nkf;
    c->g_kf_bad.assign(g->kf_bad, g->kf_bad + nkf);
    c->g_kf_mp_off.assign(g->kf_mp_off, g->kf_mp_off + (nkf ? nkf + 1 : 0));
    c->g_kf_mp.assign(g->kf_mp, g->kf_mp + ns);
    c->g_kf_cov_off.assign(g->kf_cov_off, g->kf_cov_off + (nkf ? nkf + 1 : 0));
    c->g_kf_cov.assign(g->kf_cov, g->kf_cov + nc);
    c->g_mp_bad.assign(g->mp_bad, g->mp_bad + nmp);
    c->g_mp_obs_off.assign(g->mp_obs_off, g->mp_obs_off + (nmp ? nmp + 1 : 0));
    c->g_mp_obs.assign(g->mp_obs, g->mp_obs + no);
    c->refmap = 1;
    return GF_OK;
}

int orc_chain_timings(orc_chain* c, double* out) {
    std::memcpy(out, c->tm, sizeof(c->tm));
    return GF_OK;
}

int orc_chain_step(orc_chain* c, const uint8_t* img) {
    using clk = std::chrono::steady_clock;
    auto tprev = clk::now();
    auto lap = [&](int k) {
        auto t = clk::now();
        c->tm[k] = std::chrono::duration<double>(t - tprev).count();
        tprev = t;
    };
    int32_t* st = c->stats;
    int32_t* T = c->track;
    const int frames = st[GF_ST_FRAMES];
    std::memset(st, 0, sizeof(c->stats));
    st[GF_ST_FRAMES] = frames;
    // the initial estimate's path (Tracking.cc:602-628)
    T[GF_TR_QUERY] += 1;  // mnId
    T[GF_TR_SINCE] = std::min(T[GF_TR_SINCE] + 1, 1 << 30);
    // TrackWithMotionModel needs >= 4 keyframes in the map (KeyFramesInMap, :602;
    // no keyframe graph: the map is assumed to hold more)
    const int kfc0 = c->refmap ? c->g_nkf : -1;
    int path = T[GF_TR_STATE] == 1 ? 3 : (T[GF_TR_VEL] && T[GF_TR_SINCE] >= 2 && !(kfc0 >= 0 && kfc0 < 4)) ? 0 : 2;
    c->t_cur = c->t_cur + c->p.dt;  // mCurrentFrame.mTimeStamp
    if (path == 0)
        mat44(c->V, c->Tcw_last, c->Tcw);  // TrackWithMotionModel :1519
    else
        for (int i = 0; i < 16; i++) c->Tcw[i] = path == 2 ? c->Tcw_last[i] : 0.f;  // :1353; empty
    std::fill(c->kp2mp.begin(), c->kp2mp.end(), -1);
    std::fill(c->score.begin(), c->score.end(), 999);
    std::fill(c->outl.begin(), c->outl.end(), 0);
    int rc = extract(c, img);
    if (rc) return rc;
    lap(0);
    const int n = c->nkp;
    int nm = 0;
    orc_cand_take();
    if (path == 0) {  // TrackWithMotionModel (:1506-1642)
        orc_match_lastframe(&c->fi, c->kps.data(), c->desc.data(), n, c->Tcw, c->last_kps.data(),
                            c->last_desc.data(), c->last_kp2mp.data(), c->last_outl.data(), c->last_pos.data(),
                            c->last_nkp, 15.f, 1, c->kp2mp.data(), c->score.data(), &nm);
        st[GF_ST_M3] = nm;
        st[GF_ST_CAND_LAST] = (int32_t)orc_cand_take();
        if (nm >= 20) pose(c, &st[GF_ST_INL1], &st[GF_ST_ITER1], &st[GF_ST_EDGES1]);
    }
    int found = 0;
    for (int i = 0; i < n; i++)
        if (c->kp2mp[i] >= 0) {
            if (c->outl[i]) {
                c->kp2mp[i] = -1;
                c->outl[i] = 0;
            } else {
                found++;
            }
        }
    st[GF_ST_FOUND] = found;
    st[GF_ST_TO_MATCH] = c->p.gf_budget - found;
    // the fall-backs: TrackPreviousFrame, Relocalisation
    bool ok = true;
    if (path == 0 && !(nm >= 20 && found >= 10)) {
        path = 1;
        std::fill(c->kp2mp.begin(), c->kp2mp.begin() + n, -1);
        std::memcpy(c->Tcw, c->Tcw_last, sizeof(c->Tcw));
    }
    if (path != 0) {
        ok = path == 3 ? relocalise(c) : track_previous_frame(c);
        int cnt = 0;
        for (int i = 0; i < n; i++) cnt += c->kp2mp[i] >= 0;
        st[GF_ST_FOUND] = cnt;
        st[GF_ST_TO_MATCH] = c->p.gf_budget - cnt;
        st[GF_ST_FLAGS] |= path == 3 ? 4096 : 2048;
        if (!ok) st[GF_ST_FLAGS] |= 8192;
        if (path == 3 && ok) {
            st[GF_ST_FLAGS] |= 32768;
            T[GF_TR_SINCE] = 0;  // mnLastRelocFrameId = mCurrentFrame.mnId
        }
    }
    T[GF_TR_PATH] = path;
    T[GF_TR_OK] = ok;
    const bool recent = T[GF_TR_SINCE] < 2;  // mnId < mnLastRelocFrameId + 2
    const int ntm = st[GF_ST_TO_MATCH];
    const bool gf = c->p.gf != 0;
    // TrackLocalMap (only after a successful initial estimate)
    MapState G;
    std::vector<int32_t> lmp;
    std::vector<int32_t> list;
    int branch = 5;
    bool viz = false, working = false;
    std::vector<uint8_t> seen;
    const long long* rec = c->clk.empty() ? nullptr : c->clk.data();
    const int M = c->M, R = c->ck_R;
    const bool mclk = gf && rec && (rec[GF_CK_FLAGS] & 1), sclk = gf && rec && (rec[GF_CK_FLAGS] & 2);
    const long long match_t = rec ? rec[GF_CK_MATCH] : 0, select_t = rec ? rec[GF_CK_SELECT] : 0;
    float Twc[16];
    if (ok) {
        // UpdateReference (Tracking.cc:2745, 3689-3852), then the local map in
        // mvpLocalMapPoints order replaces the map for the rest of the frame
        if (c->refmap) {
            gf_covis_map g{c->g_nkf, c->nmp, c->g_kf_bad.data(), c->g_kf_mp_off.data(), c->g_kf_mp.data(),
                           c->g_kf_cov_off.data(), c->g_kf_cov.data(), c->g_mp_bad.data(), c->g_mp_obs_off.data(),
                           c->g_mp_obs.data()};
            std::vector<int32_t> lk(64);
            lmp.assign(c->M, 0);
            int nk = 0, nl = 0, ref = -1;
            orc_update_reference(&g, c->kp2mp.data(), n, lk.data(), &nk, 64, lmp.data(), &nl, c->M, &ref);
            nl = std::min(nl, c->M);
            lmp.resize(nl);
            take_map(c, G);  // c's arrays are now empty; rebuild them as the local map
            const size_t Mz = c->M;
            c->map.assign(Mz, gf_map_point{});
            c->map_desc.assign(Mz * 32, 0);
            c->views.assign(Mz, gf_mp_view{});
            c->mp_H.assign(Mz * 14, 0.0);
            c->mp_info.assign(Mz * 49, 0.0);
            c->mp_uv.assign(Mz * 2, 0.f);
            c->upd.assign(Mz, 0);
            std::vector<int32_t> g2l(Mz, -1);
            for (int k = 0; k < nl; k++) {
                const int q = lmp[k];
                c->map[k] = G.map[q];
                std::memcpy(&c->map_desc[32 * (size_t)k], &G.desc[32 * (size_t)q], 32);
                c->views[k] = G.views[q];
                std::memcpy(&c->mp_H[14 * (size_t)k], &G.H[14 * (size_t)q], 14 * sizeof(double));
                std::memcpy(&c->mp_info[49 * (size_t)k], &G.info[49 * (size_t)q], 49 * sizeof(double));
                c->mp_uv[2 * k] = G.uv[2 * q];
                c->mp_uv[2 * k + 1] = G.uv[2 * q + 1];
                c->upd[k] = G.upd[q];
                g2l[q] = k;
            }
            c->nmp = nl;
            st[GF_ST_NLOCAL] = nl;
            for (int i = 0; i < n; i++)
                if (c->kp2mp[i] >= 0) {
                    c->kp2mp[i] = g2l[c->kp2mp[i]];
                    if (c->kp2mp[i] < 0) c->score[i] = 999;
                }
        }
        lap(1);
        // SearchReferencePointsInFrustum (Tracking.cc:3149-3410)
        if (gf) {
            if (!recent) {  // updatePWLSVec + FRAME_INFO_MATRIX (:3162-3192)
                twc_of(c->Tcw, Twc);
                orc_obs_update(c->t_prev, c->Tcw_last, c->t_cur, Twc, c->Xv);
                for (int i = 0; i < n; i++) {  // Observability.cc:386-554
                    const int mp = c->kp2mp[i];
                    if (mp < 0 || mp >= c->nmp || c->outl[i]) continue;
                    const float s2 = c->level_sigma2[c->kps[i].octave];
                    uint8_t valid;
                    orc_obs_build_info(&c->oc, c->Xv, c->map[mp].pos, &s2, 1, 0, &c->mp_H[14 * (size_t)mp],
                                       &c->mp_info[49 * (size_t)mp], &c->mp_uv[2 * mp], &valid);
                }
            }
            // mCurrentInfoMat = 1e-5 I + matched ObsMat stamped for this frame (:3161, :3195-3219)
            for (int e = 0; e < 49; e++) c->base[e] = (e % 8 == 0) ? 1e-5 : 0.0;
            for (int i = 0; i < n; i++) {
                const int mp = c->kp2mp[i];
                if (mp < 0 || mp >= c->nmp || c->upd[mp] != 1) continue;
                for (int e = 0; e < 49; e++) c->base[e] = c->base[e] + c->mp_info[49 * (size_t)mp + e];
            }
        }
        lap(2);
        for (int i = 0; i < n; i++)  // mbTrackInView = false for matched points (:3205)
            if (c->kp2mp[i] >= 0 && c->kp2mp[i] < c->nmp) c->views[c->kp2mp[i]].in_view = 0;
        // mnLastFrameSeen == mnId: the points matched before the local-map search
        seen.assign(c->nmp, 0);
        for (int i = 0; i < n; i++)
            if (c->kp2mp[i] >= 0 && c->kp2mp[i] < c->nmp) seen[c->kp2mp[i]] = 1;
        if (gf && ntm <= 0) {  // :3231-3249, stale mbTrackInView
            for (int i = 0; i < c->nmp; i++)
                if (c->views[i].in_view) list.push_back(i);
            branch = 1;
            viz = true;
        } else {
            // isInFrustum over mvpLocalMapPoints (:3251-3278); with a match budget
            // the loop stops at the first point not seen this frame whose elapsed
            // > time_total_match / 2: those points move to mLeftMapPoints and the
            // list ends there
            int mlen = c->nmp;
            long long tviz = 0;
            if (mclk) {
                const long long* el = rec + GF_CK_OFF_VIZ(M, R);
                int last = -1;
                for (int i = 0; i < c->nmp; i++) {
                    if (seen[i]) continue;
                    tviz = el[i];
                    last = i;
                    if (2 * el[i] > match_t) {
                        mlen = i;
                        break;
                    }
                }
                if (last < 0) tviz = 0;
                for (int i = mlen; i < c->nmp; i++) list.push_back(i);
                if (mlen < c->nmp) {
                    viz = true;
                    st[GF_ST_FLAGS] |= 8 | 32;
                }
                st[GF_ST_NCUT] = c->nmp - mlen;
            }
            int nv = 0;
            orc_frustum(&c->fi, c->Tcw, c->map.data(), mlen, 0.5f, c->views.data(), &nv);
            for (int i = 0; i < n; i++)
                if (c->kp2mp[i] >= 0 && c->kp2mp[i] < c->nmp) c->views[c->kp2mp[i]].in_view = 0;
            int nin = 0;
            for (int i = 0; i < mlen; i++) nin += c->views[i].in_view ? 1 : 0;
            st[GF_ST_IN_VIEW] = nin;
            if (nin == 0) {
                branch = 4;
            } else if (!gf || nin < 400 || recent) {  // :3318-3323 (th 5 after a relocalisation)
                branch = 2;
                int k = 0;
                orc_match_project(&c->fi, c->kps.data(), c->desc.data(), n, c->views.data(), c->map_desc.data(),
                                  mlen, recent ? 5.f : 1.f, 0.8f, c->kp2mp.data(), c->score.data(), &k);
                st[GF_ST_LOCAL] = k;
            } else {  // :3329-3343
                branch = 3;
                std::vector<uint8_t> updated;
                bool late = false;
                // MAP_INFO capped at (time_total_match - time_Viz) / 2 (:3331)
                map_info(c, c->Xv, mlen, 0, 1, &updated, mclk ? rec + GF_CK_OFF_MI(M, R) : nullptr, match_t - tviz,
                         &late);
                if (late) st[GF_ST_FLAGS] |= 8 | 64;
                std::vector<int32_t> left(c->M);
                int nleft = 0, nmatched = 0, cut_round = -1;
                // capped at time_total_match - time_Mat_Online - time_Viz (:3343-3344)
                orc_obs_active_match_capped(&c->fi, c->kps.data(), c->desc.data(), n, c->views.data(),
                                            c->map_desc.data(), updated.data(), c->mp_info.data(), c->mp_H.data(),
                                            mlen, c->base, c->level_sigma2, ntm, 1.f, 0.8f, &c->rng, c->kp2mp.data(),
                                            c->score.data(), left.data(), &nleft, &nmatched,
                                            mclk ? rec + GF_CK_OFF_AM(M, R) : nullptr, R,
                                            mclk ? match_t - rec[GF_CK_MAT_ONLINE] - tviz : 0, &cut_round);
                if (cut_round >= 0) st[GF_ST_FLAGS] |= 8 | 128;
                st[GF_ST_LOCAL] = nmatched;
                st[GF_ST_LDETS] = (int32_t)orc_last_ldets();
                list.insert(list.end(), left.begin(), left.begin() + nleft);  // push_back after the cut points
            }
        }
        lap(3);
        pose(c, &st[GF_ST_INL2], &st[GF_ST_ITER2], &st[GF_ST_EDGES2]);  // outliers kept (:2776)
        lap(4);
        // TrackLocalMap's verdict (:2819-2824)
        const int inl = st[GF_ST_INL2];
        working = !(T[GF_TR_SINCE] < c->max_frames && inl < 25) && inl >= 15;
        if (!working) st[GF_ST_FLAGS] |= 16384;
    }
    st[GF_ST_BRANCH] = branch;
    T[GF_TR_STATE] = working ? 0 : 1;
    T[GF_TR_VEL] = working ? 1 : 0;
    int nlist = (int)list.size();
    if (working) {
        // motion model (:729-738)
        float LastTwc[16];
        twc_of(c->Tcw_last, LastTwc);
        mat44(c->Tcw, LastTwc, c->V);
        if (gf) {
            // timeCost_rest (:866) for RunMapPointsSelection and SearchAdditionalMatchesInFrame
            const long long rest = sclk ? select_t - rec[GF_CK_SOFAR] : 0;
            if (sclk && rest <= 0) st[GF_ST_FLAGS] |= 8 | 16;
            // predictPWLSVec(dt, 2) and RunMapPointsSelection at kinematic[1] (:795-800, :1717-1779)
            twc_of(c->Tcw, Twc);
            orc_obs_update(c->t_prev, c->Tcw_last, c->t_cur, Twc, c->Xv);
            gf_kine kin[2];
            orc_obs_predict(c->Xv, c->t_cur - c->t_prev, 2, kin);
            std::memcpy(c->Xv_next, kin[1].Xv, sizeof(c->Xv_next));
            if (!sclk || rest > 0) {  // "too little budget available" (:1727-1731)
                bool late = false;
                map_info(c, c->Xv_next, c->nmp, 1, 2, nullptr, sclk ? rec + GF_CK_OFF_SEL(M, R) : nullptr,
                         2 * rest, &late);
                if (late) st[GF_ST_FLAGS] |= 8 | 256;
            }
            lap(5);
            // SearchAdditionalMatchesInFrame (:3097-3145)
            if (!list.empty()) {
                if (viz) {
                    // the visibility pass, capped at timeCost_rest / 2 per point (:3107-3119)
                    int cut = (int)list.size();
                    if (sclk) {
                        const long long* el = rec + GF_CK_OFF_SA(M, R);
                        for (int k = 0; k < (int)list.size(); k++)
                            if (!seen[list[k]] && 2 * el[k] > 2 * rest) {
                                cut = k;
                                break;
                            }
                    }
                    frustum_list(c, list.data(), cut);
                    // points seen this frame are skipped by the pass (mnLastFrameSeen, :3110-3111)
                    for (int i = 0; i < n; i++)
                        if (c->kp2mp[i] >= 0 && c->kp2mp[i] < c->nmp) c->views[c->kp2mp[i]].in_view = 0;
                    if (cut < (int)list.size()) {
                        list.resize(cut);  // mLeftMapPoints.erase(vit, vend)
                        st[GF_ST_FLAGS] |= 8 | 512;
                    }
                }
                // SearchByProjection_Budget(F, mLeftMapPoints, 0.8, rest - time_so_far)
                int k = 0, bcut = -1;
                orc_match_project_list(&c->fi, c->kps.data(), c->desc.data(), n, c->views.data(),
                                       c->map_desc.data(), list.data(), (int)list.size(), 0.8f, 0.8f,
                                       c->kp2mp.data(), c->score.data(), &k, sclk ? rec + GF_CK_OFF_BUD(M, R) : nullptr,
                                       sclk ? 2 * rest - 2 * rec[GF_CK_SA_SOFAR] : 0, &bcut);
                if (bcut >= 0) st[GF_ST_FLAGS] |= 8 | 1024;
                st[GF_ST_EXTRA] = k;
            }
        }
        nlist = (int)list.size();
    }
    for (int k = 0; k < nlist; k++) c->left[k] = list[k];
    st[GF_ST_NLEFT] = nlist;
    st[GF_ST_CAND_PROJ] = (int32_t)orc_cand_take();  // M2 and SearchByProjection_Budget (the one-point scans do not count)
    if (c->refmap && ok) {  // the local map's state back to the stream map, indices back to map indices
        const int nl = (int)lmp.size();
        for (int k = 0; k < nl; k++) {
            const int q = lmp[k];
            G.views[q] = c->views[k];
            std::memcpy(&G.H[14 * (size_t)q], &c->mp_H[14 * (size_t)k], 14 * sizeof(double));
            std::memcpy(&G.info[49 * (size_t)q], &c->mp_info[49 * (size_t)k], 49 * sizeof(double));
            G.uv[2 * q] = c->mp_uv[2 * k];
            G.uv[2 * q + 1] = c->mp_uv[2 * k + 1];
            G.upd[q] = c->upd[k];
        }
        for (int i = 0; i < n; i++)
            if (c->kp2mp[i] >= 0) c->kp2mp[i] = lmp[c->kp2mp[i]];
        for (int j = 0; j < st[GF_ST_NLEFT]; j++) c->left[j] = lmp[c->left[j]];
        take_map(c, G);  // the stream map back in place
    }
    if (working) {  // outliers NULL, mLastFrame = Frame(mCurrentFrame) (:899-910)
        for (int i = 0; i < n; i++)
            if (c->kp2mp[i] >= 0 && c->outl[i]) c->kp2mp[i] = -1;
        make_last(c);
    }
    for (int i = 0; i < c->nmp; i++) c->upd[i] -= 1;
    int fl = st[GF_ST_FLAGS];
    if (T[GF_TR_PATH] == 1) fl |= st[GF_ST_M3] < 20 ? 1 : 2;  // TrackWithMotionModel failed
    if (ok && st[GF_ST_INL2] < 15) fl |= 4;
    st[GF_ST_FLAGS] = fl;
    st[GF_ST_FRAMES] = frames + 1;
    lap(6);
    return GF_OK;
}

}  // extern "C"
