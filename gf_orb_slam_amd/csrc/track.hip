// Per-frame bookkeeping of Tracking between the hot-path stages, kept on the
// device so a front-end step never round-trips to the host:
//   motion-model prediction  mCurrentFrame.mTcw = mVelocity * mLastFrame.mTcw
//                            (Tracking.cc:1511)
//   outlier discard after PoseOptimization (Tracking.cc:1550-1563) and the GF
//                            budget num_to_match = budget - nMatchesFound
//                            (Tracking.cc:3228)
//   matched-point gather for the FRAME_INFO_MATRIX build (Observability.cc:
//                            386-520 over mCurrentFrame.mvpMapPoints)
//   mbTrackInView = false for points already matched (Tracking.cc:3205)
// One 64-lane wave per frame; all of it is byte/index work.
#include "common.h"

namespace {

__global__ __launch_bounds__(64) void k_motion_predict(int nframes, const float* __restrict__ V,
                                                       const float* __restrict__ Tlast, float* __restrict__ Tcw) {
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= nframes) return;
    const float* a = V + 16 * f;
    const float* b = Tlast + 16 * f;
    float o[16];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = a[4 * i] * b[j];
            for (int k = 1; k < 4; k++) s = s + a[4 * i + k] * b[4 * k + j];
            o[4 * i + j] = s;
        }
    for (int i = 0; i < 16; i++) Tcw[16 * f + i] = o[i];
}

__global__ __launch_bounds__(64) void k_discard_outliers(int32_t* __restrict__ kp2mp, uint8_t* __restrict__ outl,
                                                         const int32_t* __restrict__ nkps, int stride, int budget,
                                                         int32_t* __restrict__ nmatches,
                                                         int32_t* __restrict__ num_to_match) {
    const int f = blockIdx.x, l = threadIdx.x;
    const int n = nkps[f];
    int32_t* km = kp2mp + (size_t)f * stride;
    uint8_t* ou = outl + (size_t)f * stride;
    int cnt = 0;
    for (int i = l; i < n; i += 64) {
        if (km[i] >= 0) {
            if (ou[i]) {
                km[i] = -1;
                ou[i] = 0;
            } else {
                cnt++;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (l == 0) {
        if (nmatches) nmatches[f] = cnt;
        if (num_to_match) num_to_match[f] = budget - cnt;
    }
}

struct GatherArgs {
    const gf_keypoint* kps;
    const int32_t* nkps;
    int kp_stride;
    const int32_t* kp2mp;
    const gf_map_point* map;
    int map_stride;
    float level_sigma2[16];
    int nlevels;
    float* pos;
    float* sigma2;
    int32_t* idx;
    int32_t* n;
};

// Ordered compaction of the matched keypoints: world position of the map
// point, level sigma^2 of the keypoint octave, keypoint index.
__global__ __launch_bounds__(64) void k_matched_gather(GatherArgs G) {
    const int f = blockIdx.x, l = threadIdx.x;
    const int n = G.nkps[f];
    const size_t kb = (size_t)f * G.kp_stride;
    int cnt = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + l;
        const int mp = i < n ? G.kp2mp[kb + i] : -1;
        const bool on = mp >= 0;
        const unsigned long long m = __ballot(on);
        const int pos = cnt + __popcll(m & ((1ull << l) - 1ull));
        if (on) {
            const gf_map_point& P = G.map[(size_t)f * G.map_stride + mp];
            float* o = G.pos + (kb + pos) * 3;
            o[0] = P.pos[0];
            o[1] = P.pos[1];
            o[2] = P.pos[2];
            const int oc = min(max(G.kps[kb + i].octave, 0), G.nlevels - 1);
            G.sigma2[kb + pos] = G.level_sigma2[oc];
            if (G.idx) G.idx[kb + pos] = i;
        }
        cnt += __popcll(m);
    }
    if (l == 0) G.n[f] = cnt;
}

__global__ __launch_bounds__(64) void k_views_exclude(const int32_t* __restrict__ kp2mp, const int32_t* __restrict__ nkps,
                                                      int kp_stride, gf_mp_view* __restrict__ views, int mp_stride,
                                                      const int32_t* __restrict__ nmp) {
    const int f = blockIdx.x;
    const int n = nkps[f], m = nmp[f];
    for (int i = threadIdx.x; i < n; i += 64) {
        const int mp = kp2mp[(size_t)f * kp_stride + i];
        if (mp >= 0 && mp < m) views[(size_t)f * mp_stride + mp].in_view = 0;
    }
}

}  // namespace

extern "C" {

int gf_motion_predict_dev(gf_ctx* ctx, int nframes, const float* d_velocity, const float* d_Tcw_last, float* d_Tcw,
                          void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_velocity && d_Tcw_last && d_Tcw, GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_motion_predict");
    GF_LAUNCH(k_motion_predict, (nframes + 63) / 64, 64, 0, s, nframes, d_velocity, d_Tcw_last, d_Tcw);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_discard_outliers_dev(gf_ctx* ctx, int nframes, int32_t* d_kp2mp, uint8_t* d_outlier, const int32_t* d_nkps,
                            int kp_stride, int budget, int32_t* d_nmatches, int32_t* d_num_to_match, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_kp2mp && d_outlier && d_nkps && kp_stride > 0, GF_ERR_ARG, "bad arg");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_discard_outliers");
    GF_LAUNCH(k_discard_outliers, nframes, 64, 0, s, d_kp2mp, d_outlier, d_nkps, kp_stride, budget, d_nmatches,
                                              d_num_to_match);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_matched_gather_dev(gf_ctx* ctx, int nframes, const gf_keypoint* d_kps, const int32_t* d_nkps, int kp_stride,
                          const int32_t* d_kp2mp, const gf_map_point* d_map, int map_stride,
                          const float* level_sigma2, int nlevels, float* d_pos, float* d_sigma2, int32_t* d_idx,
                          int32_t* d_n, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_kps && d_nkps && d_kp2mp && d_map && level_sigma2 && d_pos && d_sigma2 && d_n, GF_ERR_ARG, "null arg");
    GF_CHECK(nlevels >= 1 && nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    GatherArgs G{};
    G.kps = d_kps;
    G.nkps = d_nkps;
    G.kp_stride = kp_stride;
    G.kp2mp = d_kp2mp;
    G.map = d_map;
    G.map_stride = map_stride;
    for (int i = 0; i < nlevels; i++) G.level_sigma2[i] = level_sigma2[i];
    G.nlevels = nlevels;
    G.pos = d_pos;
    G.sigma2 = d_sigma2;
    G.idx = d_idx;
    G.n = d_n;
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_matched_gather");
    GF_LAUNCH(k_matched_gather, nframes, 64, 0, s, G);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_views_exclude_matched_dev(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps,
                                 int kp_stride, gf_mp_view* d_views, const int32_t* d_nmp, int mp_stride,
                                 void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_kp2mp && d_nkps && d_views && d_nmp, GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_views_exclude");
    GF_LAUNCH(k_views_exclude, nframes, 64, 0, s, d_kp2mp, d_nkps, kp_stride, d_views, mp_stride, d_nmp);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

}  // extern "C"
