// Oracle (test infrastructure): Tracking::UpdateReference for one frame —
// UpdateReferenceKeyFrames (src/Tracking.cc:3768-3852) and
// UpdateReferencePoints (:3708-3766) restated with the reference's own
// containers: std::map<KeyFrame*,int> keyed by the keyframe index (the
// keyframes are indexed in ascending KeyFrame* order, include/gfslam/abi.h
// gf_covis_map), a vector reserved to 3x the counter size and walked with the
// end iterator taken before the neighbour loop appends, and the
// mnTrackReferenceForFrame marks as per-call flags.
#include <map>
#include <vector>

#include "oracle_common.h"

extern "C" int orc_update_reference(const gf_covis_map* M, int32_t* frame_mps, int nkp, int32_t* local_kfs,
                                    int* n_local_kfs, int kf_cap, int32_t* local_mps, int* n_local_mps, int mp_cap,
                                    int32_t* ref_kf) {
    // UpdateReferenceKeyFrames: each map point votes for the keyframes observing it (:3775-3795)
    std::map<int, int> keyframeCounter;
    for (int i = 0; i < nkp; i++) {
        const int m = frame_mps[i];
        if (m < 0) continue;
        if (!M->mp_bad[m]) {
            for (int o = M->mp_obs_off[m]; o < M->mp_obs_off[m + 1]; o++) keyframeCounter[M->mp_obs[o]]++;
        } else {
            frame_mps[i] = -1;
        }
    }
    int max = 0, kfmax = -1;
    std::vector<int> local;
    local.reserve(3 * keyframeCounter.size());
    std::vector<char> kf_mark(M->nkf, 0);
    for (auto it = keyframeCounter.begin(); it != keyframeCounter.end(); ++it) {  // :3803-3817
        const int kf = it->first;
        if (M->kf_bad[kf]) continue;
        if (it->second > max) {
            max = it->second;
            kfmax = kf;
        }
        local.push_back(kf);
        kf_mark[kf] = 1;
    }
    const size_t n0 = local.size();
    for (size_t p = 0; p < n0; p++) {  // :3820-3848 (end iterator taken before the loop)
        if (local.size() > 80) break;
        const int kf = local[p];
        const int o0 = M->kf_cov_off[kf];
        const int deg = std::min(10, M->kf_cov_off[kf + 1] - o0);  // GetBestCovisibilityKeyFrames(10)
        for (int j = 0; j < deg; j++) {
            const int nb = M->kf_cov[o0 + j];
            if (!M->kf_bad[nb]) {
                if (!kf_mark[nb]) {
                    local.push_back(nb);
                    kf_mark[nb] = 1;
                    break;
                }
            }
        }
    }
    *ref_kf = kfmax;
    // UpdateReferencePoints (:3713-3763; GOOD_FEATURE_MAP_BOUND off)
    std::vector<char> mp_mark(M->nmp, 0);
    std::vector<int> mps;
    for (int kf : local) {
        for (int o = M->kf_mp_off[kf]; o < M->kf_mp_off[kf + 1]; o++) {
            const int m = M->kf_mp[o];
            if (m < 0) continue;
            if (mp_mark[m]) continue;
            if (!M->mp_bad[m]) {
                mps.push_back(m);
                mp_mark[m] = 1;
            }
        }
    }
    *n_local_kfs = (int)local.size();
    *n_local_mps = (int)mps.size();
    for (int p = 0; p < (int)local.size() && p < kf_cap; p++) local_kfs[p] = local[p];
    for (int p = 0; p < (int)mps.size() && p < mp_cap; p++) local_mps[p] = mps[p];
    return ((int)local.size() <= kf_cap && (int)mps.size() <= mp_cap) ? GF_OK : GF_ERR_CAP;
}
