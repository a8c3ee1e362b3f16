// Batched tracking front end: Tracking::GrabImage (Tracking.cc:461-917) in the
// WORKING state for B independent sequences, chained on one HIP stream with
// no host round trip (see gf_frontend_* in include/gfslam/abi.h for the
// reference call sequence). The stages are the library's device-family entry
// points; this file owns the per-stream state buffers and the small
// bookkeeping kernels between the stages:
//   k_fe_begin   frame source pointer, timestamps, motion model
//                mTcw = mVelocity * mLastFrame.mTcw (Tracking.cc:1519), the
//                fresh Frame's mvpMapPoints / mvpMatchScore / mvbOutlier
//   k_fe_branch  SearchReferencePointsInFrustum's num_to_match <= 0 exit
//                (Tracking.cc:3231-3249): mLeftMapPoints from the stale
//                mbTrackInView flags, mbNeedVizCheck
//   k_fe_decide  nToMatch after isInFrustum and the choice between
//                SearchByProjection (nToMatch < 400) and runActiveMapMatching
//                (Tracking.cc:3316-3343)
//   k_fe_post    motion-model update mVelocity = mTcw * LastTwc (:729-738)
//                and the post-publish list of SearchAdditionalMatchesInFrame
//   k_fe_end     outliers set NULL (:899-905), mLastFrame = Frame(mCurrentFrame)
//                (:907), updateAtFrameId stamps shifted to the next frame
// Branch choices are per stream, so each gated stage gets a per-stream count
// that is 0 for the streams that skip it (the kernels then do nothing for
// that stream and leave its state untouched).
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <limits>
#include <vector>

#include "common.h"
#include "reloc.h"
#include "undist.h"

namespace {

struct FeDev {
    int B, cap, M, budget, gf, src_mode, period;
    double dt;
    long long frame_stride;
    // frame source
    const uint8_t** ptrs;
    const uint8_t* const* bases;
    const int32_t* phase;
    int32_t* step;
    // current frame
    int32_t* nkp;
    float* Tcw;
    int32_t* kp2mp;
    int32_t* score;
    uint8_t* outl;
    gf_keypoint* kps;
    uint8_t* desc;
    // last frame
    gf_keypoint* last_kps;
    uint8_t* last_desc;
    int32_t* last_nkp;
    int32_t* last_kp2mp;
    uint8_t* last_outl;
    float* last_pos;
    float* Tcw_last;
    float* V;
    double* t_prev;
    double* t_cur;
    // map the tracking stages work on: the stream's map, or with a keyframe
    // graph (gf_frontend_set_covis) the local map UpdateReference assembled
    // this step, gathered from the stream's map in mvpLocalMapPoints order
    const gf_map_point* map;
    const int32_t* nmp;
    gf_mp_view* views;
    int32_t* upd;
    // the stream's map itself (GF_FE_MAP... fields) and the local-map lists
    int refmap;
    const gf_map_point* gmap;
    const int32_t* gnmp;
    int32_t* gupd;
    int32_t* lmp;  // [B][M] local map points (map indices), mvpLocalMapPoints order
    int32_t* nlm;  // [B]
    int32_t* g2l;  // [B][M] map index -> local index, -1 outside the local map
    // lists and gates
    int32_t* left;
    int32_t* left1;
    int32_t* nleft;
    int32_t* nlist;
    int32_t* nlist_viz;
    int32_t* m_frustum;
    int32_t* m_active;
    int32_t* m_m2;
    int32_t* nm2;    // matches of SearchByProjection(F, local, 1)
    int32_t* stats;  // [GF_FE_NSTAT][B]
    int32_t* hist;   // [B][8] running counters (GF_FE_HIST)
    // time budgets (gf_set_budgets; device clock ticks of 100 MHz; < 0: no budget)
    long long match_ticks, select_ticks;
    long long* clk;        // [B][ck_stride] clock record (GF_FE_CLOCK)
    long long ck_stride;
    int ck_R;              // length of the per-round array
    unsigned long long* t_frame;  // [B] timer_all: the frame's start, after the extraction gate
    unsigned long long* t_viz0;   // [B] the isInFrustum loop's timer (Tracking.cc:3252)
    unsigned long long* t_mat0;   // [B] after the loop (Tracking.cc:3311)
    unsigned long long* t_sel0;   // [B] RunMapPointsSelection / SearchAdditionalMatchesInFrame start
    long long* viz_time;   // [B] time_Viz
    long long* cap2_mi;    // [B] 2 x MAP_INFO cap of the active branch
    long long* rest2;      // [B] 2 x timeCost_rest
    long long* cap2_sel;   // [B] 2 x MAP_INFO cap of RunMapPointsSelection (-1: skip all)
    gf_mp_view* vtmp;      // [B][M] clocked isInFrustum results (kept before the cut)
    int32_t* ncut;         // [B] points the isInFrustum cap moved to mLeftMapPoints
    int32_t* nlist0;       // [B] mLeftMapPoints size before SearchAdditionalMatchesInFrame
    // the tracking state machine (GF_FE_TRACK) and the per-stream gates of its stages
    const long long* syn; // test clock [GF_CK_NSITE][2] (gf_frontend_set_test_clock); null: the device clock
    int32_t* track;        // [B][GF_TR_N]
    int32_t* m3_nlast;     // [B] last-frame points SearchByProjection(Cur, Last) projects (0 off the motion model)
    int32_t* rl_gate;      // [B] 1: Relocalisation this step
    const int32_t* kfc;    // [B] KeyFramesInMap() of the stream's keyframe graph (-1: no graph, assumed > 5)
    int32_t* nkp_tl;       // [B] keypoints TrackLocalMap sees (0: it does not run)
    int32_t* nkp_fi;       // [B] keypoints of its FRAME_INFO_MATRIX pass
    int32_t* gate_tl;      // [B] TrackLocalMap runs
    int32_t* gate_fi;      // [B] its updatePWLSVec + FRAME_INFO_MATRIX run (not within 2 frames of a relocalisation)
    int32_t* gate_post;    // [B] the frame ends WORKING: motion model, prediction, post-publish block
    int32_t* nmp_post;     // [B] RunMapPointsSelection's points (0 when the frame is lost)
    int32_t* nmp_step;     // [B] without keyframe graphs: the map's size when TrackLocalMap runs, else 0
    float* th_m2;          // [B] SearchByProjection(F, local, th): 5 within 2 frames of a relocalisation (:3318-3320)
    int max_frames;        // mMaxFrames
    // per-frame stage log (gf_frontend_set_time_log; tl_cap 0: off)
    int tl_cap;
    long long* tl_stamp;   // [tl_cap][GF_TL_NSITE] device clock at the stage boundaries
    gf_time_rec* tl_rec;   // [tl_cap][B]
};

__device__ __forceinline__ long long* ck_rec(const FeDev& D, int b) { return D.clk + (long long)b * D.ck_stride; }
__device__ __forceinline__ int ck_off_viz(const FeDev& D) { return GF_CK_OFF_VIZ(D.M, D.ck_R); }
__device__ __forceinline__ int ck_off_mi(const FeDev& D) { return GF_CK_OFF_MI(D.M, D.ck_R); }
__device__ __forceinline__ int ck_off_sel(const FeDev& D) { return GF_CK_OFF_SEL(D.M, D.ck_R); }
__device__ __forceinline__ int ck_off_sa(const FeDev& D) { return GF_CK_OFF_SA(D.M, D.ck_R); }

__device__ __forceinline__ int32_t* stat(const FeDev& D, int which) { return D.stats + (long long)which * D.B; }

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// 4x4 row-major float product, summation order of the reference's cv::Mat
// gemm restatement (oracle/chain.cpp uses the same order).
__device__ __forceinline__ void mat44(const float* a, const float* b, float* o) {
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            float s = a[4 * i] * b[j];
            for (int k = 1; k < 4; k++) s = s + a[4 * i + k] * b[4 * k + j];
            o[4 * i + j] = s;
        }
}

__global__ __launch_bounds__(256) void k_fe_begin(FeDev D) {
    const int b = blockIdx.x, t = threadIdx.x;
    if (t == 0) {
        if (D.src_mode == 1) {
            const int k = *D.step;
            const int idx = (int)(((long long)D.phase[b] + k) % D.period);
            D.ptrs[b] = D.bases[b] + (long long)idx * D.frame_stride;
        }
        D.t_cur[b] = D.t_cur[b] + D.dt;  // mCurrentFrame.mTimeStamp (mLastFrame's may be older after a loss)
        // the initial estimate's path (Tracking.cc:602-628): LOST -> Relocalisation;
        // a velocity and >= 2 frames since a relocalisation -> TrackWithMotionModel
        // (mTcw = mVelocity * mLastFrame.mTcw, :1519) unless the map holds fewer
        // than 4 keyframes (:602); else TrackPreviousFrame (mTcw = mLastFrame.mTcw,
        // :1353); a fresh Frame's mTcw is empty (zeros)
        int32_t* T = D.track + (size_t)b * GF_TR_N;
        T[GF_TR_QUERY] += 1;  // mnId
        const int since = min(T[GF_TR_SINCE] + 1, 1 << 30);
        T[GF_TR_SINCE] = since;
        const int kfc = D.kfc[b];
        const int path = T[GF_TR_STATE] == 1 ? 3 : (T[GF_TR_VEL] && since >= 2 && !(kfc >= 0 && kfc < 4)) ? 0 : 2;
        T[GF_TR_PATH] = path;
        T[GF_TR_OK] = 0;
        D.m3_nlast[b] = path == 0 ? D.last_nkp[b] : 0;
        D.rl_gate[b] = path == 3;
        float o[16];
        if (path == 0) {
            mat44(D.V + 16 * b, D.Tcw_last + 16 * b, o);
        } else {
            for (int i = 0; i < 16; i++) o[i] = path == 2 ? D.Tcw_last[16 * b + i] : 0.f;
        }
        for (int i = 0; i < 16; i++) D.Tcw[16 * b + i] = o[i];
        for (int s = 0; s < GF_FE_NSTAT; s++)
            if (s != GF_ST_FRAMES) stat(D, s)[b] = 0;
        D.ncut[b] = 0;
    }
    if (D.match_ticks >= 0 || D.select_ticks >= 0) {  // timer_all (Tracking.cc:866) and a fresh record header
        long long* r = ck_rec(D, b);
        if (t < GF_CK_HEADER) r[t] = -1;
        if (t == 0) {
            r[GF_CK_FLAGS] = (D.match_ticks >= 0 ? 1 : 0) | (D.select_ticks >= 0 ? 2 : 0);
            r[GF_CK_MATCH] = D.match_ticks;
            r[GF_CK_SELECT] = D.select_ticks;
            D.t_frame[b] = now_ticks();
        }
    }
    const long long o = (long long)b * D.cap;
    for (int i = t; i < D.cap; i += 256) {
        D.kp2mp[o + i] = -1;
        D.score[o + i] = 999;
        D.outl[o + i] = 0;
    }
}

// Ordered compaction of views[i].in_view over the stream's map (one wave).
__device__ int compact_in_view(const FeDev& D, int b, int32_t* out) {
    const int lane = threadIdx.x;
    const int m = D.nmp[b];
    int cnt = 0;
    for (int base = 0; base < m; base += 64) {
        const int i = base + lane;
        const bool on = i < m && D.views[(long long)b * D.M + i].in_view;
        const unsigned long long msk = __ballot(on);
        if (on) out[(long long)b * D.M + cnt + __popcll(msk & ((1ull << lane) - 1ull))] = i;
        cnt += __popcll(msk);
    }
    return cnt;
}

// mbTrackInView = false for the points the frame already matched (the
// mnLastFrameSeen = mnId / mbTrackInView = false loop of
// SearchReferencePointsInFrustum, Tracking.cc:3194-3208).
__device__ __forceinline__ void exclude_matched(const FeDev& D, int b) {
    const int n = D.nkp_tl[b], m = D.nmp[b];
    const long long ko = (long long)b * D.cap, o = (long long)b * D.M;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int mp = D.kp2mp[ko + i];
        if (mp >= 0 && mp < m) D.views[o + mp].in_view = 0;
    }
    __syncthreads();
}

__global__ __launch_bounds__(64) void k_fe_branch(FeDev D) {
    const int b = blockIdx.x, lane = threadIdx.x;
    exclude_matched(D, b);
    const int ntm = stat(D, GF_ST_TO_MATCH)[b];
    if (!D.gate_tl[b]) {  // no TrackLocalMap: the initial estimate failed
        if (lane == 0) {
            stat(D, GF_ST_BRANCH)[b] = 5;
            D.nlist[b] = 0;
            D.nlist_viz[b] = 0;
            D.m_frustum[b] = 0;
        }
    } else if (D.gf && ntm <= 0) {
        // mbTrackInView as left by earlier frames (matched points already false)
        const int n = compact_in_view(D, b, D.left1);
        if (lane == 0) {
            stat(D, GF_ST_BRANCH)[b] = 1;
            D.nlist[b] = n;
            D.nlist_viz[b] = n;
            D.m_frustum[b] = 0;
        }
    } else if (lane == 0) {
        stat(D, GF_ST_BRANCH)[b] = 0;
        D.nlist[b] = 0;
        D.nlist_viz[b] = 0;
        D.m_frustum[b] = D.nmp[b];
        if (D.gf && D.match_ticks >= 0) D.t_viz0[b] = now_ticks();  // timer.tic() (Tracking.cc:3252)
    }
}

// Keypoint-matched map points of a stream (mnLastFrameSeen == mnId) as a bitmap
// in LDS; M <= 4096.
__device__ void matched_bits(const FeDev& D, int b, int m, uint32_t* bits) {
    const int t = threadIdx.x;
    for (int w = t; w < 128; w += blockDim.x) bits[w] = 0u;
    __syncthreads();
    const int n = D.nkp[b];
    const long long o = (long long)b * D.cap;
    for (int i = t; i < n; i += blockDim.x) {
        const int mp = D.kp2mp[o + i];
        if (mp >= 0 && mp < m) atomicOr(&bits[mp >> 5], 1u << (mp & 31));
    }
    __syncthreads();
}

__device__ __forceinline__ bool is_matched(const uint32_t* bits, int i) { return (bits[i >> 5] >> (i & 31)) & 1u; }

// nToMatch and the search branch (Tracking.cc:3305-3343). With a match budget
// the isInFrustum results are in vtmp with each point's elapsed time in the
// clock record: the loop stops at the first point not matched this frame whose
// elapsed > time_total_match / 2 (:3262-3270); the points before it take their
// results, the rest keep their state and go to mLeftMapPoints in list order,
// and mvpLocalMapPoints (the search's list) ends at the cut.
__global__ __launch_bounds__(256) void k_fe_decide(FeDev D) {
    __shared__ int s_cnt, s_cut, s_last;
    __shared__ uint32_t bits[128];
    const int b = blockIdx.x, t = threadIdx.x;
    if (t == 0) {
        s_cnt = 0;
        s_cut = INT_MAX;
        s_last = -1;
    }
    __syncthreads();
    const int br = stat(D, GF_ST_BRANCH)[b];
    const bool clocked = D.gf && D.match_ticks >= 0 && br == 0;
    if (br == 0 && !clocked) exclude_matched(D, b);  // after the unclocked isInFrustum pass
    const int m = D.nmp[b];
    const long long o = (long long)b * D.M;
    int cut = m;
    if (clocked) {
        matched_bits(D, b, m, bits);
        const long long* el = ck_rec(D, b) + ck_off_viz(D);
        for (int i = t; i < m; i += 256) {
            if (is_matched(bits, i)) continue;  // mnLastFrameSeen == mnId: skipped before the clock
            if (2 * el[i] > D.match_ticks) atomicMin(&s_cut, i);
            atomicMax(&s_last, i);
        }
        __syncthreads();
        cut = min(s_cut, m);
        for (int i = t; i < cut; i += 256) {
            gf_mp_view v = D.vtmp[o + i];
            if (is_matched(bits, i)) v.in_view = 0;
            D.views[o + i] = v;
        }
        for (int i = cut + t; i < m; i += 256) D.left1[o + i - cut] = i;
    }
    if (br == 0) {
        int c = 0;
        for (int i = t; i < cut; i += 256) c += D.views[o + i].in_view ? 1 : 0;
        c = gfd::warp_sum(c);
        if ((t & 63) == 0) atomicAdd(&s_cnt, c);
    }
    __syncthreads();
    if (t != 0) return;
    D.m_active[b] = 0;
    D.m_m2[b] = 0;
    if (br != 0) return;
    if (clocked) {
        // time_Viz: the last value the loop compared (0 when it compared none)
        const long long* el = ck_rec(D, b) + ck_off_viz(D);
        const long long viz = cut < m ? el[cut] : (s_last >= 0 ? el[s_last] : 0);
        long long* r = ck_rec(D, b);
        r[GF_CK_VIZ_CUT] = cut;
        r[GF_CK_VIZ_TIME] = viz;
        D.viz_time[b] = viz;
        D.cap2_mi[b] = D.match_ticks - viz;  // (total - time_Viz) / 2, doubled
        D.ncut[b] = m - cut;
        stat(D, GF_ST_NCUT)[b] = m - cut;
        if (cut < m) stat(D, GF_ST_FLAGS)[b] |= 8 | 32;
    }
    const int n = s_cnt;
    stat(D, GF_ST_IN_VIEW)[b] = n;
    int nb;
    if (n == 0) {
        nb = 4;
    } else if (!D.gf || n < 400 || D.th_m2[b] != 1.f) {  // Tracking.cc:3318-3323
        nb = 2;
        D.m_m2[b] = cut;
    } else {
        nb = 3;
        D.m_active[b] = cut;
    }
    stat(D, GF_ST_BRANCH)[b] = nb;
    if (clocked) D.t_mat0[b] = now_ticks();  // timer.tic() (Tracking.cc:3311)
}

__global__ __launch_bounds__(256) void k_fe_post(FeDev D) {
    __shared__ int s_tail[4096];
    const int b = blockIdx.x, t = threadIdx.x;
    const int br = stat(D, GF_ST_BRANCH)[b];
    const long long o = (long long)b * D.M;
    const int ncut = D.ncut[b];
    int n = 0;
    if (br == 1) {
        n = D.nlist[b];
        for (int i = t; i < n; i += 256) D.left[o + i] = D.left1[o + i];
    } else {
        // mLeftMapPoints: the points the isInFrustum cap cut (Tracking.cc:3265),
        // then runActiveMapMatching's leftovers (push_back, Observability.cc:1517-1519)
        const int na = br == 3 ? D.nleft[b] : 0;
        if (ncut > 0 && na > 0) {
            for (int i = t; i < na; i += 256) s_tail[i] = D.left[o + i];
            __syncthreads();
            for (int i = t; i < na; i += 256) D.left[o + ncut + i] = s_tail[i];
        }
        for (int i = t; i < ncut; i += 256) D.left[o + i] = D.left1[o + i];
        n = ncut + na;
    }
    if (t != 0) return;
    if (br == 2) stat(D, GF_ST_LOCAL)[b] = D.nm2[b];
    // TrackLocalMap's verdict (Tracking.cc:2819-2824), mState (:713-716)
    int32_t* T = D.track + (size_t)b * GF_TR_N;
    bool ok = false;
    if (D.gate_tl[b]) {
        const int inl = stat(D, GF_ST_INL2)[b];
        ok = !(T[GF_TR_SINCE] < D.max_frames && inl < 25) && inl >= 15;
        if (!ok) stat(D, GF_ST_FLAGS)[b] |= 16384;
    }
    T[GF_TR_STATE] = ok ? 0 : 1;
    T[GF_TR_VEL] = ok ? 1 : 0;  // mVelocity = cv::Mat() when lost
    D.gate_post[b] = ok;
    D.nmp_post[b] = ok ? D.nmp[b] : 0;
    stat(D, GF_ST_NLEFT)[b] = n;
    if (!ok) {  // no post-publish block: the leftovers stay unsearched
        D.nlist[b] = 0;
        D.nlist0[b] = 0;
        D.nlist_viz[b] = 0;
        return;
    }
    // motion model (Tracking.cc:729-738): LastTwc from mLastFrame.mTcw, mVelocity = mTcw * LastTwc
    const float* L = D.Tcw_last + 16 * b;
    float Twc[16] = {0};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Twc[4 * i + j] = L[4 * j + i];
    for (int i = 0; i < 3; i++) {
        float s = Twc[4 * i] * L[3];
        s = s + Twc[4 * i + 1] * L[7];
        s = s + Twc[4 * i + 2] * L[11];
        Twc[4 * i + 3] = -s;
    }
    Twc[15] = 1.f;
    float Vn[16];
    mat44(D.Tcw + 16 * b, Twc, Vn);
    for (int i = 0; i < 16; i++) D.V[16 * b + i] = Vn[i];
    D.nlist[b] = n;
    D.nlist0[b] = n;
    const bool viz = (br == 1 || ncut > 0);  // mbNeedVizCheck
    D.nlist_viz[b] = viz ? n : 0;
    if (D.select_ticks >= 0) {
        // timeCost_rest = budget - timeCost_sofar (Tracking.cc:866), shared by
        // RunMapPointsSelection and SearchAdditionalMatchesInFrame, whose
        // timers start here
        const unsigned long long now = now_ticks();
        const long long sofar = D.syn ? D.syn[2 * GF_CK_SITE_SOFAR] : (long long)(now - D.t_frame[b]);
        const long long rest = D.select_ticks - sofar;
        ck_rec(D, b)[GF_CK_SOFAR] = sofar;
        D.rest2[b] = 2 * rest;
        D.cap2_sel[b] = rest > 0 ? 2 * rest : -1;  // <= 0: "too little budget available" (:1727-1731)
        D.t_sel0[b] = now;
        if (rest <= 0) stat(D, GF_ST_FLAGS)[b] |= 8 | 16;
    }
}

// The visibility pass of SearchAdditionalMatchesInFrame skips the points
// matched before the local-map search (mnLastFrameSeen == mnId,
// Tracking.cc:3110-3111), so they keep mbTrackInView = false: after the list
// frustum of a stream that ran the pass, matched points are out of view again.
// Only the isInFrustum-cut list (branch 5) holds such points.
// With a select budget the visibility pass is clocked (Tracking.cc:3107-3119):
// its results are in vtmp, and the pass stops at the first list point not
// matched before the local-map search whose elapsed > timeCost_rest / 2; the
// points before it take their results and mLeftMapPoints is erased from there.
__global__ __launch_bounds__(256) void k_fe_viz_exclude(FeDev D) {
    __shared__ uint32_t bits[128];
    __shared__ int s_cut;
    const int b = blockIdx.x, t = threadIdx.x;
    const int nl = D.nlist_viz[b];
    if (nl <= 0) return;
    const int n = D.nkp[b], m = D.nmp[b];
    const long long o = (long long)b * D.cap, om = (long long)b * D.M;
    if (D.select_ticks < 0) {
        for (int i = t; i < n; i += 256) {
            const int mp = D.kp2mp[o + i];
            if (mp >= 0 && mp < m) D.views[om + mp].in_view = 0;
        }
        return;
    }
    if (t == 0) s_cut = INT_MAX;
    matched_bits(D, b, m, bits);
    const long long* el = ck_rec(D, b) + ck_off_sa(D);
    const long long rest2 = D.rest2[b];
    const int32_t* L = D.left + om;
    for (int k = t; k < nl; k += 256)
        if (!is_matched(bits, L[k]) && 2 * el[k] > rest2) atomicMin(&s_cut, k);
    __syncthreads();
    const int cut = min(s_cut, nl);
    for (int k = t; k < cut; k += 256) D.views[om + L[k]] = D.vtmp[om + L[k]];
    __syncthreads();
    for (int i = t; i < n; i += 256) {  // as above: matched points end out of view
        const int mp = D.kp2mp[o + i];
        if (mp >= 0 && mp < m) D.views[om + mp].in_view = 0;
    }
    if (t == 0) {
        ck_rec(D, b)[GF_CK_SA_CUT] = cut;
        if (cut < nl) {
            D.nlist[b] = cut;  // mLeftMapPoints.erase(vit, vend)
            stat(D, GF_ST_NLEFT)[b] = cut;
            stat(D, GF_ST_FLAGS)[b] |= 8 | 512;
        }
    }
}

constexpr int END_U = 4;
__global__ __launch_bounds__(256) void k_fe_end(FeDev D) {
    const int b = blockIdx.x, t = threadIdx.x;
    const bool working = D.gate_post[b];  // mState == WORKING (Tracking.cc:854)
    const int n = working ? D.nkp[b] : 0;
    const long long o = (long long)b * D.cap;
    // each loop: END_U elements' loads (clamped, unconditional), then their
    // stores (the stores may alias the next loads, so a plain loop would wait
    // on every element)
    for (int i0 = t; i0 < n; i0 += 256 * END_U) {
        int mp[END_U];
        uint8_t ou[END_U];
        gf_keypoint kp[END_U];
        float3 pos[END_U];
#pragma unroll
        for (int u = 0; u < END_U; u++) {
            const long long i = o + min(i0 + 256 * u, n - 1);
            mp[u] = D.kp2mp[i];
            ou[u] = D.outl[i];
            kp[u] = D.kps[i];
        }
#pragma unroll
        for (int u = 0; u < END_U; u++) {
            const gf_map_point& P = D.gmap[(long long)b * D.M + max(mp[u], 0)];
            pos[u] = make_float3(P.pos[0], P.pos[1], P.pos[2]);
        }
#pragma unroll
        for (int u = 0; u < END_U; u++) {
            const int i = i0 + 256 * u;
            if (i >= n) continue;
            const int m1 = mp[u] >= 0 && ou[u] ? -1 : mp[u];  // Tracking.cc:899-905 (mvbOutlier stays set)
            D.kp2mp[o + i] = m1;
            D.last_kp2mp[o + i] = m1;
            D.last_outl[o + i] = ou[u];
            D.last_kps[o + i] = kp[u];
            float* p = D.last_pos + 3 * (o + i);
            const bool on = m1 >= 0;
            p[0] = on ? pos[u].x : 0.f;
            p[1] = on ? pos[u].y : 0.f;
            p[2] = on ? pos[u].z : 0.f;
        }
    }
    const uint4* ds = (const uint4*)(D.desc + o * 32);
    uint4* dd = (uint4*)(D.last_desc + o * 32);
    for (int i0 = t; i0 < 2 * n; i0 += 256 * END_U) {
        uint4 v[END_U];
#pragma unroll
        for (int u = 0; u < END_U; u++) v[u] = ds[min(i0 + 256 * u, 2 * n - 1)];
#pragma unroll
        for (int u = 0; u < END_U; u++)
            if (i0 + 256 * u < 2 * n) dd[i0 + 256 * u] = v[u];
    }
    const int m = D.gnmp[b];
    int32_t* gu = D.gupd + (long long)b * D.M;
    for (int i0 = t; i0 < m; i0 += 256 * END_U) {
        int v[END_U];
#pragma unroll
        for (int u = 0; u < END_U; u++) v[u] = gu[min(i0 + 256 * u, m - 1)];
#pragma unroll
        for (int u = 0; u < END_U; u++)
            if (i0 + 256 * u < m) gu[i0 + 256 * u] = v[u] - 1;
    }
    if (t == 0) {
        if (working) {  // mLastFrame = Frame(mCurrentFrame) (:910)
            D.last_nkp[b] = n;
            for (int i = 0; i < 16; i++) D.Tcw_last[16 * b + i] = D.Tcw[16 * b + i];
            D.t_prev[b] = D.t_cur[b];
        }
        int fl = stat(D, GF_ST_FLAGS)[b];
        if (D.match_ticks >= 0 || D.select_ticks >= 0) {  // the caps that fired, from the clock record
            const long long* r = ck_rec(D, b);
            if (D.match_ticks >= 0 && D.m_active[b] > 0) {
                for (int w = 0; w * 64 < D.m_active[b]; w++)
                    if (2 * r[ck_off_mi(D) + w] > D.cap2_mi[b]) fl |= 8 | 64;
                if (r[GF_CK_AM_CUT] >= 0) fl |= 8 | 128;
            }
            if (D.select_ticks >= 0 && D.gf && D.cap2_sel[b] >= 0) {
                for (int w = 0; w * 64 < D.nmp[b]; w++)
                    if (2 * r[ck_off_sel(D) + w] > D.cap2_sel[b]) fl |= 8 | 256;
                if (r[GF_CK_BUDGET_CUT] >= 0) fl |= 8 | 1024;
            }
        }
        const int32_t* T = D.track + (size_t)b * GF_TR_N;
        if (T[GF_TR_PATH] == 1) fl |= stat(D, GF_ST_M3)[b] < 20 ? 1 : 2;  // TrackWithMotionModel failed
        if (D.gate_tl[b] && stat(D, GF_ST_INL2)[b] < 15) fl |= 4;
        stat(D, GF_ST_FLAGS)[b] = fl;
        stat(D, GF_ST_FRAMES)[b] += 1;
        int32_t* h = D.hist + 8LL * b;
        const int br = stat(D, GF_ST_BRANCH)[b];
        if (br >= 0 && br < 5) h[br] += 1;
        if (fl & 8) h[5] += 1;  // a time cap fired
        h[6] += stat(D, GF_ST_LDETS)[b];
        h[7] += stat(D, GF_ST_LOCAL)[b];
        if (b == 0) *D.step += 1;
    }
}

// Stage log (logCurrentFrame, Tracking.h:254-280): one boundary of this
// step, in the ring slot of the step counter (advanced by k_fe_end).
__global__ __launch_bounds__(64) void k_fe_tstamp(FeDev D, int site) {
    if (threadIdx.x == 0) {
        const int slot = *D.step % D.tl_cap;
        long long* st = D.tl_stamp + (long long)slot * GF_TL_NSITE;
        if (site == GF_TL_BEGIN)
            for (int k = 1; k < GF_TL_NSITE; k++) st[k] = 0;  // the boundaries this step does not reach read 0
        st[site] = (long long)now_ticks();
    }
}

// After k_fe_end: the step's end stamp and each stream's counts.
__global__ __launch_bounds__(64) void k_fe_tlog(FeDev D) {
    const int step = *D.step - 1;  // k_fe_end advanced the counter
    const int slot = step % D.tl_cap;
    for (int b = blockIdx.x * 64 + threadIdx.x; b < D.B; b += gridDim.x * 64) {
        gf_time_rec r;
        r.frame_time_stamp = D.t_cur[b];
        r.path = D.track[(size_t)b * GF_TR_N + GF_TR_PATH];
        r.branch = stat(D, GF_ST_BRANCH)[b];
        r.found = stat(D, GF_ST_FOUND)[b];
        r.tpf = stat(D, GF_ST_TPF)[b];
        r.local = stat(D, GF_ST_LOCAL)[b];
        r.inliers = stat(D, GF_ST_INL2)[b];
        r.extra = stat(D, GF_ST_EXTRA)[b];
        r.track_map = D.gate_tl[b];
        r.flags = stat(D, GF_ST_FLAGS)[b];
        r.step = step;
        D.tl_rec[(long long)slot * D.B + b] = r;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) D.tl_stamp[(long long)slot * GF_TL_NSITE + GF_TL_END] = (long long)now_ticks();
}

// Bootstrap: the matched frame becomes the last frame (kp2mp as matched).
__global__ __launch_bounds__(256) void k_fe_boot_end(FeDev D) {
    const int b = blockIdx.x, t = threadIdx.x;
    const int n = D.nkp[b];
    const long long o = (long long)b * D.cap;
    for (int i = t; i < n; i += 256) {
        const int mp = D.kp2mp[o + i];
        D.last_kp2mp[o + i] = mp;
        D.last_outl[o + i] = 0;
        D.last_kps[o + i] = D.kps[o + i];
        float* p = D.last_pos + 3 * (o + i);
        if (mp >= 0) {
            const gf_map_point& P = D.gmap[(long long)b * D.M + mp];
            p[0] = P.pos[0];
            p[1] = P.pos[1];
            p[2] = P.pos[2];
        } else {
            p[0] = p[1] = p[2] = 0.f;
        }
    }
    const uint4* ds = (const uint4*)(D.desc + o * 32);
    uint4* dd = (uint4*)(D.last_desc + o * 32);
    for (int i = t; i < 2 * n; i += 256) dd[i] = ds[i];
    if (t == 0) {
        D.last_nkp[b] = n;
        for (int i = 0; i < 16; i++) D.Tcw_last[16 * b + i] = D.Tcw[16 * b + i];
        D.t_prev[b] = D.t_cur[b];
        int32_t* T = D.track + (size_t)b * GF_TR_N;  // WORKING, a velocity, no relocalisation so far
        T[GF_TR_STATE] = 0;
        T[GF_TR_VEL] = 1;
        T[GF_TR_SINCE] = 1 << 30;
        T[GF_TR_PATH] = 0;
        T[GF_TR_OK] = 1;
        if (b == 0) *D.step += 1;
    }
}

// Local-map arrays for the step (one workgroup per stream). Gather: entry k
// of the local map is the stream's map point lmp[k] (UpdateReference order);
// the frame's matches move to local indices (a match outside the local map is
// dropped; UpdateReference puts every matched point's keyframes in it).
struct MapArrays {
    const gf_map_point* map;
    const uint8_t* desc;
    const float* pos;
    gf_mp_view* views;
    double* H;
    double* info;
    float* uv;
    int32_t* upd;
};

// Per-point rows of the map arrays for the local points [k0, k0 + np) of a
// stream (np <= ROWS_PER_BLOCK): gather (dst local <- src map point lm[k]) or
// scatter (dst map point lm[k] <- src local). Every array's row block fits one
// word per thread, so a workgroup issues all its arrays' loads (clamped,
// unconditional) before the first store.
constexpr int ROWS_PER_BLOCK = 32;
constexpr int IX_U = 4;  // index conversions: loads in flight per thread

struct RowWord {
    uint32_t v;
    long long at;  // destination word, -1: none
};
template <int W, typename T>
__device__ __forceinline__ RowWord row_load(const T* src_, const int32_t* lm, long long o, int k0, int np,
                                            bool gather) {
    static_assert(W * ROWS_PER_BLOCK <= 256, "one word per thread");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(src_);
    const int nw = np * W, w0 = threadIdx.x, w = min(w0, nw - 1);
    const int p = w / W, e = w - p * W, k = k0 + p;
    const long long g = o + lm[k], l = o + k;
    return RowWord{src[(gather ? g : l) * W + e], w0 < nw ? (gather ? l : g) * W + e : -1};
}
template <typename T>
__device__ __forceinline__ void row_store(T* dst, const RowWord& r) {
    if (r.at >= 0) reinterpret_cast<uint32_t*>(dst)[r.at] = r.v;
}

// Index conversion for the step: g2l of the local points, the frame's matches
// to local indices (a match outside the local map is dropped; UpdateReference
// puts every matched point's keyframes in it).
__device__ void gather_index(const FeDev& D, int b, int32_t* lnmp) {
    const int t = threadIdx.x;
    const int n = D.nlm[b];
    const long long o = (long long)b * D.M;
    const int32_t* lm = D.lmp + o;
    // batches of IX_U independent loads, then their stores (the stores may
    // alias the next loads, so a plain loop waits on every load)
    for (int k0 = t; k0 < n; k0 += 256 * IX_U) {
        int v[IX_U];
#pragma unroll
        for (int u = 0; u < IX_U; u++) v[u] = lm[min(k0 + 256 * u, n - 1)];
#pragma unroll
        for (int u = 0; u < IX_U; u++)
            if (k0 + 256 * u < n) D.g2l[o + v[u]] = k0 + 256 * u;
    }
    if (t == 0) {
        lnmp[b] = n;
        stat(D, GF_ST_NLOCAL)[b] = n;
    }
    __syncthreads();
    const long long ko = (long long)b * D.cap;
    const int nk = D.nkp_tl[b];
    for (int i0 = t; i0 < nk; i0 += 256 * IX_U) {
        int mp[IX_U], l[IX_U];
#pragma unroll
        for (int u = 0; u < IX_U; u++) mp[u] = D.kp2mp[ko + min(i0 + 256 * u, nk - 1)];
#pragma unroll
        for (int u = 0; u < IX_U; u++) l[u] = D.g2l[o + max(mp[u], 0)];
#pragma unroll
        for (int u = 0; u < IX_U; u++) {
            const int i = i0 + 256 * u;
            if (i >= nk || mp[u] < 0) continue;
            D.kp2mp[ko + i] = l[u];
            if (l[u] < 0) D.score[ko + i] = 999;
        }
    }
}

// Matches and mLeftMapPoints back to map indices, g2l reset.
__device__ void scatter_index(const FeDev& D, int b) {
    const int t = threadIdx.x;
    const int n = D.nlm[b];
    const long long o = (long long)b * D.M;
    const int32_t* lm = D.lmp + o;
    for (int k0 = t; k0 < n; k0 += 256 * IX_U) {
        int v[IX_U];
#pragma unroll
        for (int u = 0; u < IX_U; u++) v[u] = lm[min(k0 + 256 * u, n - 1)];
#pragma unroll
        for (int u = 0; u < IX_U; u++)
            if (k0 + 256 * u < n) D.g2l[o + v[u]] = -1;
    }
    const long long ko = (long long)b * D.cap;
    const int nk = D.nkp_tl[b];
    for (int i0 = t; i0 < nk; i0 += 256 * IX_U) {
        int l[IX_U], g[IX_U];
#pragma unroll
        for (int u = 0; u < IX_U; u++) l[u] = D.kp2mp[ko + min(i0 + 256 * u, nk - 1)];
#pragma unroll
        for (int u = 0; u < IX_U; u++) g[u] = lm[max(l[u], 0)];
#pragma unroll
        for (int u = 0; u < IX_U; u++)
            if (i0 + 256 * u < nk && l[u] >= 0) D.kp2mp[ko + i0 + 256 * u] = g[u];
    }
    const int nl = stat(D, GF_ST_NLEFT)[b];
    for (int j0 = t; j0 < nl; j0 += 256 * IX_U) {
        int l[IX_U], g[IX_U];
#pragma unroll
        for (int u = 0; u < IX_U; u++) l[u] = D.left[o + min(j0 + 256 * u, nl - 1)];
#pragma unroll
        for (int u = 0; u < IX_U; u++) g[u] = lm[l[u]];
#pragma unroll
        for (int u = 0; u < IX_U; u++)
            if (j0 + 256 * u < nl) D.left[o + j0 + 256 * u] = g[u];
    }
}

// The local map (grid: 1 + point chunks x streams): workgroup 0 converts the
// indices, the others gather the local map's rows from the stream's map.
__global__ __launch_bounds__(256) void k_fe_gather(FeDev D, MapArrays G, MapArrays L, int32_t* lnmp) {
    const int b = blockIdx.y;
    if (blockIdx.x == 0) {
        gather_index(D, b, lnmp);
        return;
    }
    const int k0 = (blockIdx.x - 1) * ROWS_PER_BLOCK;
    const int n = D.nlm[b];
    if (k0 >= n) return;
    const int np = min(ROWS_PER_BLOCK, n - k0);
    const long long o = (long long)b * D.M;
    const int32_t* lm = D.lmp + o;
    const RowWord rm = row_load<sizeof(gf_map_point) / 4>(G.map, lm, o, k0, np, true);
    const RowWord rd = row_load<8>(G.desc, lm, o, k0, np, true);
    const RowWord rp = row_load<3>(G.pos, lm, o, k0, np, true);
    const RowWord rv = row_load<sizeof(gf_mp_view) / 4>(G.views, lm, o, k0, np, true);
    const RowWord ru = row_load<1>(G.upd, lm, o, k0, np, true);
    row_store((gf_map_point*)L.map, rm);
    row_store((uint8_t*)L.desc, rd);
    row_store((float*)L.pos, rp);
    row_store(L.views, rv);
    row_store(L.upd, ru);
}

// Back to the stream's map: workgroup 0 converts the indices, the others
// scatter the local map's visibility and updateAtFrameId (H / ObsMat /
// u_proj are written in map order through the remap).
__global__ __launch_bounds__(256) void k_fe_scatter(FeDev D, MapArrays G, MapArrays L) {
    const int b = blockIdx.y;
    if (blockIdx.x == 0) {
        scatter_index(D, b);
        return;
    }
    const int k0 = (blockIdx.x - 1) * ROWS_PER_BLOCK;
    const int n = D.nlm[b];
    if (k0 >= n) return;
    const int np = min(ROWS_PER_BLOCK, n - k0);
    const long long o = (long long)b * D.M;
    const int32_t* lm = D.lmp + o;
    const RowWord rv = row_load<sizeof(gf_mp_view) / 4>(L.views, lm, o, k0, np, false);
    const RowWord ru = row_load<1>(L.upd, lm, o, k0, np, false);
    row_store(G.views, rv);
    row_store(G.upd, ru);
}

__global__ void k_fe_boot_begin(FeDev D) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= D.B) return;
    if (D.src_mode == 1) {
        const int idx = (int)(((long long)D.phase[b] + *D.step) % D.period);
        D.ptrs[b] = D.bases[b] + (long long)idx * D.frame_stride;
    }
}

}  // namespace

struct gf_frontend {
    gf_ctx* ctx = nullptr;
    gf_frontend_params p{};
    gf_extractor* ex = nullptr;
    int cap = 0;
    gf_frame_info fi{};
    gf_obs_camera ocam{};
    float inv_sigma2[16] = {}, level_sigma2[16] = {};
    FeDev D{};
    // fields
    void* field_ptr[GF_FE_NFIELDS] = {};
    size_t field_bytes[GF_FE_NFIELDS] = {};
    // the stream maps (the GF_FE_MAP... fields); the working arrays below
    // (D.map, D.views, D.upd, D.nmp, mp_pos, mp_H, mp_info, mp_uv, wdesc) alias
    // them, or with keyframe graphs hold the local map of the step
    MapArrays gm{};
    int32_t* g_nmp = nullptr;
    const uint8_t* wdesc = nullptr;
    int32_t* w_nmp = nullptr;
    // keyframe graphs (gf_frontend_set_covis): per-stream slabs, device array of
    // per-stream gf_covis_map, UpdateReference outputs and scratch
    static const int KF_CAP = 64;
    int covis_set = 0;
    std::vector<int> h_nmp;
    std::vector<uint8_t> has_covis;
    gf_covis_map* d_covis = nullptr;
    uint8_t *cv_kf_bad = nullptr, *cv_mp_bad = nullptr;
    int32_t *cv_kf_mp_off = nullptr, *cv_kf_mp = nullptr, *cv_kf_cov_off = nullptr, *cv_kf_cov = nullptr;
    int32_t *cv_mp_obs_off = nullptr, *cv_mp_obs = nullptr;
    size_t slot_cap = 0;
    int32_t *lkf = nullptr, *nlkf = nullptr, *ref_kf = nullptr, *rm_first = nullptr;
    // device buffers not exported as fields
    int32_t* scratch = nullptr;
    int32_t* num_to_match = nullptr;  // = stats column
    double* Xv = nullptr;
    double* Xv_next = nullptr;
    double* base = nullptr;
    double* mp_H = nullptr;
    double* mp_info = nullptr;
    double* mp_info_lt = nullptr;  // [B][M][32]: the packed lower triangle of every mp_info block
    float* mp_uv = nullptr;
    float* mp_pos = nullptr;
    uint8_t* mp_updated = nullptr;
    int32_t* nview = nullptr;
    int32_t *qres = nullptr, *qold = nullptr, *merr = nullptr;  // SearchByProjection_Budget scratch
    uint8_t* staging = nullptr;
    const uint8_t** staging_ptrs = nullptr;
    std::vector<void*> allocs;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    bool sourced = false;
    // extraction gate (gf_frontend_set_gate): caller-owned events
    hipEvent_t gate_wait = nullptr, gate_done = nullptr;
    bool extracted = false;  // gf_frontend_step_extract ran, gf_frontend_step_track not yet
    int gate_stage = 4;
    // tracking stream (gf_frontend_set_track_priority): the kernels after
    // extraction run on ts, joined back into the context's stream at the end
    hipStream_t ts = nullptr;
    hipEvent_t ev_extracted = nullptr, ev_tracked = nullptr;
    // a captured step forks RunMapPointsSelection's prediction (updatePWLSVec,
    // MAP_INFO at kinematic[1]) from SearchAdditionalMatchesInFrame, as
    // Tracking.cc:884-891 runs them on two threads: two graph branches
    bool fork_post = false;
    hipStream_t fork_s = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // track-loss paths (reloc.hip): their arguments; relocalisation needs a
    // vocabulary and a keyframe database on some stream (rl_on)
    gf::TrackLossArgs TL{};
    gf_vocab* voc = nullptr;
    bool rl_alloc = false, rl_on = false;
    std::vector<gf::KfdbDev> h_kfdb;
    gf::KfdbDev* d_kfdb = nullptr;
    std::vector<int32_t> h_kfc;
    int32_t* d_kfc = nullptr;
    long long* d_syn = nullptr;  // gf_frontend_set_test_clock's (base, slope) pairs
    int tl_alloc = 0;            // time-log ring entries allocated
    int tl_first = 0;            // step counter when the log was switched on
    std::vector<std::vector<int32_t>> h_slots;  // per stream: the graph's slots per keyframe
    void* bow_tmp = nullptr;
};

namespace {

int fe_alloc(gf_frontend* fe, size_t bytes, void** out) {
    GF_HIP(hipMalloc(out, std::max<size_t>(bytes, 16)));
    fe->allocs.push_back(*out);
    GF_HIP(hipMemset(*out, 0, std::max<size_t>(bytes, 16)));
    return GF_OK;
}

template <typename T>
int fe_field(gf_frontend* fe, int field, size_t count, T** out) {
    void* p = nullptr;
    int rc = fe_alloc(fe, sizeof(T) * count, &p);
    if (rc) return rc;
    *out = (T*)p;
    if (field >= 0) {
        fe->field_ptr[field] = p;
        fe->field_bytes[field] = sizeof(T) * count;
    }
    return GF_OK;
}

// Drop the captured graph (if any) and release the context's scratch pin.
void fe_drop_graph(gf_frontend* fe) {
    if (fe->exec) (void)hipGraphExecDestroy(fe->exec);
    if (fe->graph) (void)hipGraphDestroy(fe->graph);
    if (fe->exec || fe->graph) fe->ctx->ws_pinned--;
    fe->exec = nullptr;
    fe->graph = nullptr;
}

void fe_free(gf_frontend* fe) {
    fe_drop_graph(fe);
    for (void* p : fe->allocs) (void)hipFree(p);
    fe->allocs.clear();
    if (fe->ex) (void)gf_extractor_destroy(fe->ex);
    fe->ex = nullptr;
}

#define FE_RC(expr)                \
    do {                           \
        int _rc = (expr);          \
        if (_rc) return _rc;       \
    } while (0)

// mvKeysUn (Frame::UndistortKeyPoints, Frame.cc:389-423): in place, the
// keypoints' other fields kept; nothing to do when k1 == 0 (a copy there).
int fe_undistort(gf_frontend* fe, hipStream_t s) {
    if (fe->p.dist[0] == 0.f) return GF_OK;
    const float K[4] = {fe->p.fx, fe->p.fy, fe->p.cx, fe->p.cy};
    return gf_undistort_keypoints_dev(fe->ctx, fe->D.B, K, fe->p.dist, fe->D.kps, fe->D.nkp, fe->D.cap, fe->D.kps, s);
}

// A stage boundary of the per-frame log (gf_frontend_set_time_log), when on.
int fe_tstamp(gf_frontend* fe, hipStream_t s, int site) {
    if (!fe->D.tl_cap) return GF_OK;
    GF_LAUNCH(k_fe_tstamp, 1, 64, 0, s, fe->D, site);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

// The step's first part: the extraction gate, Frame construction (ORB
// extraction, undistortion).
int fe_extract(gf_frontend* fe, hipStream_t s) {
    FeDev& D = fe->D;
    // the frame's clock starts after the extraction gate: waiting behind the
    // other front ends' extraction is not this frame's time
    if (fe->gate_wait) GF_HIP(hipStreamWaitEvent(s, fe->gate_wait, 0));
    FE_RC(fe_tstamp(fe, s, GF_TL_BEGIN));
    {
        GF_PROF(fe->ctx, s, "k_fe_begin");
        GF_LAUNCH(k_fe_begin, D.B, 256, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    FE_RC(gf_orb_extract_ptrs_dev(fe->ex, D.B, (const uint8_t* const*)D.ptrs, fe->p.width, D.kps, D.desc, D.nkp,
                                  D.cap, s));
    if (fe->gate_done && fe->gate_stage >= 4) GF_HIP(hipEventRecord(fe->gate_done, s));
    FE_RC(fe_undistort(fe, s));
    return fe_tstamp(fe, s, GF_TL_EXTRACTED);
}

// The step's second part: tracking on the extracted frame.
int fe_track_frame(gf_frontend* fe, hipStream_t s) {
    gf_ctx* ctx = fe->ctx;
    FeDev& D = fe->D;
    const int B = D.B, cap = D.cap, M = D.M;
    const gf_frame_info* fi = &fe->fi;
    int32_t* st = D.stats;
    auto col = [&](int c) { return st + (size_t)c * B; };
    const hipStream_t s_ctx = s;
    if (fe->ts) {  // fork: tracking on the prioritised stream
        GF_HIP(hipEventRecord(fe->ev_extracted, s));
        GF_HIP(hipStreamWaitEvent(fe->ts, fe->ev_extracted, 0));
        s = fe->ts;
    }
    // TrackWithMotionModel (the streams on the motion model; the others project
    // no last-frame point), PoseOptimization when >= 20 matches (:1559)
    {
        gf::CandidateCount cc(col(GF_ST_CAND_LAST));
        FE_RC(gf_match_lastframe_dev(ctx, fi, B, D.kps, D.desc, D.nkp, cap, D.Tcw, D.last_kps, D.last_desc,
                                     D.last_kp2mp, D.last_outl, D.last_pos, D.m3_nlast, cap, 15.f, 1, D.kp2mp,
                                     D.score, col(GF_ST_M3), fe->scratch, s));
    }
    gf::CandidateCount cc(col(GF_ST_CAND_PROJ));  // the projection searches below
    FE_RC(gf::pose_opt_frames_gated(ctx, B, D.Tcw, D.kps, D.nkp, cap, D.kp2mp, D.gmap, M, fe->inv_sigma2,
                                    fe->p.nlevels, fi->fx, fi->fy, fi->cx, fi->cy, D.outl, col(GF_ST_INL1),
                                    col(GF_ST_ITER1), col(GF_ST_EDGES1), col(GF_ST_M3), 20, s));
    FE_RC(fe_tstamp(fe, s, GF_TL_MOTION));
    // Relocalisation of the LOST streams: ComputeBoW, the keyframe database's
    // candidates, SearchByBoW per candidate (Tracking.cc:3861-3922)
    if (fe->rl_on) {
        const gf::TrackLossArgs& TL = fe->TL;
        FE_RC(gf::bow_transform_gated(fe->voc, B, D.desc, D.nkp, D.rl_gate, cap, 4, (int32_t*)TL.words,
                                      (double*)TL.values, (int32_t*)TL.nwords, (int32_t*)TL.fv_nodes,
                                      (int32_t*)TL.fv_start, (int32_t*)TL.fv_feats, (int32_t*)TL.nfv, fe->bow_tmp, s));
        FE_RC(gf::reloc_candidates(ctx, TL, s));
        FE_RC(gf::match_bow_pairs(ctx, 0, 0.75f, 1, B * TL.ncs, TL.pairs, TL.bow_nm, cap, s));  // b side: the frame
    }
    // the motion model's outlier discard and failure test, TrackPreviousFrame,
    // the relocalisation loop, and the gates of the TrackLocalMap stages below
    FE_RC(gf::track_loss(ctx, fe->TL, s));
    FE_RC(fe_tstamp(fe, s, GF_TL_INIT_POSE));
    const MapArrays WM{D.map, fe->wdesc, fe->mp_pos, D.views, fe->mp_H, fe->mp_info, fe->mp_uv, D.upd};
    // keyframe graphs: H / ObsMat / u_proj stay in map order (the local map's
    // point q is map point lmp[q]); the other per-point arrays are gathered
    const int32_t* rmp = D.refmap ? D.lmp : nullptr;
    if (D.refmap) {
        // TrackLocalMap -> UpdateReference (Tracking.cc:2745, 3689-3852): local
        // keyframes and mvpLocalMapPoints from this frame's matches
        FE_RC(gf::update_reference_frames(ctx, fe->d_covis, M, B, D.kp2mp, D.nkp_tl, cap, fe->lkf, fe->nlkf,
                                          gf_frontend::KF_CAP, D.lmp, D.nlm, M, fe->ref_kf, fe->rm_first,
                                          gf_frontend::KF_CAP, s));
        GF_PROF(ctx, s, "k_fe_gather");
        GF_LAUNCH(k_fe_gather, dim3(1 + (M + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK, B), 256, 0, s, D, fe->gm, WM,
                  fe->w_nmp);
        GF_HIP(hipGetLastError());
    }
    FE_RC(fe_tstamp(fe, s, GF_TL_REF_UPDATED));
    // TrackLocalMap -> SearchReferencePointsInFrustum
    if (D.gf) {
        FE_RC(gf::obs_update_gated(ctx, B, D.t_prev, D.Tcw_last, D.t_cur, D.Tcw, fe->Xv, nullptr, D.gate_fi, s));
        FE_RC(gf::obs_frame_info(ctx, &fe->ocam, B, fe->Xv, D.kps, D.nkp_fi, cap, D.kp2mp, D.outl, fe->mp_pos,
                                 D.nmp, M, fe->level_sigma2, fe->p.nlevels, fe->mp_H, fe->mp_info, fe->mp_uv, rmp, s,
                                 fe->mp_info_lt));
        FE_RC(gf::obs_accumulate_matched(ctx, B, D.kp2mp, D.nkp_tl, cap, fe->mp_info, D.upd, D.nmp, M, 1, 1e-5,
                                         fe->base, rmp, s, D.gate_tl));
    }
    {
        GF_PROF(ctx, s, "k_fe_branch");
        GF_LAUNCH(k_fe_branch, B, 64, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    const bool mclk = D.gf && D.match_ticks >= 0, sclk = D.gf && D.select_ticks >= 0;
    auto clock = [&](const unsigned long long* t0, int off, int site) {
        gf::StageClock c;
        c.t0 = t0;
        c.rec = D.clk;
        c.stride = D.ck_stride;
        c.off = off;
        c.syn = D.syn ? D.syn + 2 * site : nullptr;
        return c;
    };
    const int R = D.ck_R;
    if (mclk) {  // the isInFrustum loop on its clock (k_fe_decide applies the cap)
        FE_RC(gf::frustum_clocked(ctx, fi, B, D.Tcw, D.map, D.m_frustum, nullptr, nullptr, M, 0.5f, D.views,
                                  fe->nview, clock(D.t_viz0, GF_CK_OFF_VIZ(M, R), GF_CK_SITE_VIZ), D.vtmp, s));
    } else {
        FE_RC(gf_frustum_dev(ctx, fi, B, D.Tcw, D.map, D.m_frustum, M, 0.5f, D.views, fe->nview, s));
    }
    {
        GF_PROF(ctx, s, "k_fe_decide");
        GF_LAUNCH(k_fe_decide, B, 256, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    FE_RC(fe_tstamp(fe, s, GF_TL_FRUSTUM));
    if (D.gf) {
        FE_RC(gf::obs_map_info(ctx, &fe->ocam, B, fe->Xv, fe->mp_pos, D.m_active, M, 0, D.views, D.upd, 1, fe->mp_H,
                               fe->mp_info, fe->mp_uv, fe->mp_updated, rmp, s,
                               mclk ? clock(D.t_mat0, GF_CK_OFF_MI(M, R), GF_CK_SITE_MI) : gf::StageClock{}, D.cap2_mi,
                               fe->mp_info_lt));
        FE_RC(fe_tstamp(fe, s, GF_TL_MAT_ONLINE));
        gf::ActiveClock ac;
        if (mclk) {
            ac.mat_t0 = D.t_mat0;
            ac.viz = D.viz_time;
            ac.match_ticks = D.match_ticks;
            ac.rec = D.clk;
            ac.stride = D.ck_stride;
            ac.off = GF_CK_OFF_AM(M, R);
            ac.rounds = R;
            ac.syn = D.syn ? D.syn + 2 * GF_CK_SITE_AM_START : nullptr;
        }
        FE_RC(gf::obs_active_match(ctx, fi, B, D.kps, D.desc, D.nkp, cap, D.views, fe->wdesc, fe->mp_updated,
                                   fe->mp_info, fe->mp_H, D.m_active, M, fe->base, fe->level_sigma2,
                                   col(GF_ST_TO_MATCH), 1.f, 0.8f, (gf_rng*)fe->field_ptr[GF_FE_RNG], D.kp2mp, D.score,
                                   D.left, D.nleft, col(GF_ST_LOCAL), col(GF_ST_LDETS), rmp, s, ac, fe->mp_info_lt));
        FE_RC(fe_tstamp(fe, s, GF_TL_SELECTED));
    }
    FE_RC(gf::match_project_th(ctx, fi, B, D.kps, D.desc, D.nkp, cap, D.views, fe->wdesc, D.m_m2, M, D.th_m2, 0.8f,
                               D.kp2mp, D.score, D.nm2, s));
    FE_RC(fe_tstamp(fe, s, GF_TL_SEARCHED));
    FE_RC(gf::pose_opt_frames_gated(ctx, B, D.Tcw, D.kps, D.nkp, cap, D.kp2mp, D.map, M, fe->inv_sigma2,
                                    fe->p.nlevels, fi->fx, fi->fy, fi->cx, fi->cy, D.outl, col(GF_ST_INL2),
                                    col(GF_ST_ITER2), col(GF_ST_EDGES2), D.gate_tl, 1, s));
    {
        GF_PROF(ctx, s, "k_fe_post");
        GF_LAUNCH(k_fe_post, B, 256, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    FE_RC(fe_tstamp(fe, s, GF_TL_OPTIMISED));
    if (D.gf) {
        // predictPWLSVec(dt, 2) + RunMapPointsSelection (MAP_INFO_MATRIX at kinematic[1], check_viz);
        // in a captured step a branch of its own beside SearchAdditionalMatchesInFrame
        // (no shared data: the prediction writes Xv / H / ObsMat / u_proj / stamps,
        // the search reads views, descriptors and keypoints)
        hipStream_t sp = s;
        if (fe->fork_post) {
            GF_HIP(hipEventRecord(fe->ev_fork, s));
            GF_HIP(hipStreamWaitEvent(fe->fork_s, fe->ev_fork, 0));
            sp = fe->fork_s;
        }
        FE_RC(gf::obs_update_gated(ctx, B, D.t_prev, D.Tcw_last, D.t_cur, D.Tcw, fe->Xv, fe->Xv_next, D.gate_post,
                                   sp));
        FE_RC(gf::obs_map_info(ctx, &fe->ocam, B, fe->Xv_next, fe->mp_pos, D.nmp_post, M, 1, nullptr, D.upd, 2,
                               fe->mp_H, fe->mp_info, fe->mp_uv, nullptr, rmp, sp,
                               sclk ? clock(D.t_sel0, GF_CK_OFF_SEL(M, R), GF_CK_SITE_SEL) : gf::StageClock{}, D.cap2_sel,
                               fe->mp_info_lt));
        if (fe->fork_post) GF_HIP(hipEventRecord(fe->ev_join, sp));
        // SearchAdditionalMatchesInFrame
        if (sclk) {
            FE_RC(gf::frustum_clocked(ctx, fi, B, D.Tcw, D.map, nullptr, D.left, D.nlist_viz, M, 0.5f, D.views,
                                      fe->nview, clock(D.t_sel0, GF_CK_OFF_SA(M, R), GF_CK_SITE_SA), D.vtmp, s));
        } else {
            FE_RC(gf_frustum_list_dev(ctx, fi, B, D.Tcw, D.map, M, D.left, D.nlist_viz, 0.5f, D.views, fe->nview,
                                      s));
        }
        {
            GF_PROF(ctx, s, "k_fe_viz_exclude");
            GF_LAUNCH(k_fe_viz_exclude, B, 256, 0, s, D);
            GF_HIP(hipGetLastError());
        }
        FE_RC(gf::match_project_list_budget(ctx, fi, B, D.kps, D.desc, D.nkp, cap, D.views, fe->wdesc, M, D.left,
                                            D.nlist, 0.8f, 0.8f, D.kp2mp, D.score, col(GF_ST_EXTRA),
                                            sclk ? clock(D.t_sel0, GF_CK_OFF_BUD(M, R), GF_CK_SITE_SA_SOFAR) : gf::StageClock{},
                                            D.rest2, fe->qres, fe->qold, fe->merr, s));
        if (fe->fork_post) GF_HIP(hipStreamWaitEvent(s, fe->ev_join, 0));  // thread_Select.join()
    }
    if (D.refmap) {
        GF_PROF(ctx, s, "k_fe_scatter");
        GF_LAUNCH(k_fe_scatter, dim3(1 + (M + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK, B), 256, 0, s, D, fe->gm, WM);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_fe_end");
        GF_LAUNCH(k_fe_end, B, 256, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    if (D.tl_cap) {
        GF_LAUNCH(k_fe_tlog, (B + 63) / 64, 64, 0, s, D);
        GF_HIP(hipGetLastError());
    }
    if (fe->ts) {  // join: the context's stream sees the whole step
        GF_HIP(hipEventRecord(fe->ev_tracked, s));
        GF_HIP(hipStreamWaitEvent(s_ctx, fe->ev_tracked, 0));
    }
    return GF_OK;
}

// The tracking step after the frame source pointers are set.
int fe_track(gf_frontend* fe, hipStream_t s) {
    FE_RC(fe_extract(fe, s));
    return fe_track_frame(fe, s);
}

}  // namespace

extern "C" {

int gf_frontend_create(gf_ctx* ctx, const gf_frontend_params* p, gf_frontend** out) {
    GF_CHECK(ctx && p && out, GF_ERR_ARG, "null arg");
    GF_CHECK(p->batch > 0 && p->map_cap > 0 && p->map_cap <= 4096, GF_ERR_ARG, "batch / map_cap out of range");
    GF_CHECK(p->nlevels >= 1 && p->nlevels <= 16 && p->dt > 0, GF_ERR_ARG, "bad front-end parameters");
    GF_CHECK(!ctx->track_stream, GF_ERR_ARG,
             "the context's front end runs tracking on its own stream (gf_frontend_set_track_priority): "
             "use another context");
    GF_HIP(hipSetDevice(ctx->device));
    gf_frontend* fe = new gf_frontend();
    fe->ctx = ctx;
    fe->p = *p;
    int rc = gf_extractor_create(ctx, p->nfeatures, p->scale_factor, p->nlevels, p->harris_score ? 0 : 1, p->fast_th, p->width, p->height,
                                 p->batch, &fe->ex);
    if (rc) {
        delete fe;
        return rc;
    }
    gf_extractor_capacity(fe->ex, &fe->cap);
    const int B = p->batch, cap = fe->cap, M = p->map_cap;
    // Frame tables: bounds of the undistorted image (Frame::ComputeImageBounds,
    // Frame.cc:425-493), mvScaleFactors as float products, mvLevelSigma2 and
    // mvInvLevelSigma2 (ORBextractor.cc:474-478, Frame.cc:93-98).
    const float K[4] = {p->fx, p->fy, p->cx, p->cy};
    int bnd[4];
    gfu::image_bounds(K, p->dist, p->width, p->height, bnd);
    fe->fi = gf_frame_info{bnd[0], bnd[1], bnd[2], bnd[3], p->fx, p->fy, p->cx, p->cy, p->nlevels, p->scale_factor};
    float sf = 1.f;
    for (int l = 0; l < p->nlevels; l++) {
        if (l) sf = sf * p->scale_factor;
        fe->level_sigma2[l] = sf * sf;
        fe->inv_sigma2[l] = 1.0f / (sf * sf);
    }
    // Observability camera + the margins Tracking sets (Tracking.cc:875-877)
    gf_obs_camera& oc = fe->ocam;
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
    oc.bound_x = (int)((bnd[1] - bnd[0]) * 0.1);
    oc.bound_y = (int)((bnd[3] - bnd[2]) * 0.1);
    oc.bound_depth = 0.f;
    FeDev& D = fe->D;
    D.B = B;
    D.cap = cap;
    D.M = M;
    D.budget = p->gf_budget;
    D.gf = p->gf ? 1 : 0;
    D.dt = p->dt;
    D.match_ticks = -1;
    D.select_ticks = -1;
    auto bail = [&](int e) {
        fe_free(fe);
        delete fe;
        return e;
    };
#define F(field, type, count, dst)                          \
    if ((rc = fe_field<type>(fe, field, (count), &(dst)))) \
        return bail(rc);
    F(GF_FE_KPS, gf_keypoint, (size_t)B * cap, D.kps);
    F(GF_FE_DESC, uint8_t, (size_t)B * cap * 32, D.desc);
    F(GF_FE_NKP, int32_t, B, D.nkp);
    F(GF_FE_TCW, float, (size_t)B * 16, D.Tcw);
    F(GF_FE_KP2MP, int32_t, (size_t)B * cap, D.kp2mp);
    F(GF_FE_SCORE, int32_t, (size_t)B * cap, D.score);
    F(GF_FE_OUTLIER, uint8_t, (size_t)B * cap, D.outl);
    F(GF_FE_LAST_KPS, gf_keypoint, (size_t)B * cap, D.last_kps);
    F(GF_FE_LAST_DESC, uint8_t, (size_t)B * cap * 32, D.last_desc);
    F(GF_FE_LAST_NKP, int32_t, B, D.last_nkp);
    F(GF_FE_LAST_KP2MP, int32_t, (size_t)B * cap, D.last_kp2mp);
    F(GF_FE_LAST_OUTLIER, uint8_t, (size_t)B * cap, D.last_outl);
    F(GF_FE_LAST_POS, float, (size_t)B * cap * 3, D.last_pos);
    F(GF_FE_TCW_LAST, float, (size_t)B * 16, D.Tcw_last);
    F(GF_FE_VELOCITY, float, (size_t)B * 16, D.V);
    F(GF_FE_T_PREV, double, B, D.t_prev);
    F(GF_FE_T_CUR, double, B, D.t_cur);
    gf_map_point* map = nullptr;
    F(GF_FE_MAP, gf_map_point, (size_t)B * M, map);
    D.map = map;
    uint8_t* mdesc = nullptr;
    F(GF_FE_MAP_DESC, uint8_t, (size_t)B * M * 32, mdesc);
    int32_t* nmp = nullptr;
    F(GF_FE_NMP, int32_t, B, nmp);
    D.nmp = nmp;
    F(GF_FE_VIEWS, gf_mp_view, (size_t)B * M, D.views);
    F(GF_FE_XV, double, (size_t)B * 13, fe->Xv);
    F(GF_FE_XV_NEXT, double, (size_t)B * 13, fe->Xv_next);
    F(GF_FE_BASE, double, (size_t)B * 49, fe->base);
    F(GF_FE_MP_H, double, (size_t)B * M * 14, fe->mp_H);
    F(GF_FE_MP_INFO, double, (size_t)B * M * 49, fe->mp_info);
    {
        void* lt = nullptr;
        if ((rc = fe_alloc(fe, sizeof(double) * (size_t)B * M * 32, &lt))) return bail(rc);
#ifndef GF_NO_PACKED_INFO
        fe->mp_info_lt = (double*)lt;
#endif
    }
    F(GF_FE_MP_UV, float, (size_t)B * M * 2, fe->mp_uv);
    F(GF_FE_MP_UPD, int32_t, (size_t)B * M, D.upd);
    gf_rng* rng = nullptr;
    F(GF_FE_RNG, gf_rng, B, rng);
    F(GF_FE_LEFT, int32_t, (size_t)B * M, D.left);
    F(GF_FE_STATS, int32_t, (size_t)GF_FE_NSTAT * B, D.stats);
    F(GF_FE_HIST, int32_t, (size_t)8 * B, D.hist);
    F(-1, int32_t, (size_t)B * M, D.left1);
    F(-1, int32_t, B, D.nleft);
    F(-1, int32_t, B, D.nlist);
    F(-1, int32_t, B, D.nlist_viz);
    F(-1, int32_t, B, D.m_frustum);
    F(-1, int32_t, B, D.m_active);
    F(-1, int32_t, B, D.m_m2);
    F(-1, int32_t, B, D.nm2);
    F(-1, int32_t, (size_t)2 * B * cap, fe->scratch);
    F(-1, float, (size_t)B * M * 3, fe->mp_pos);
    F(-1, uint8_t, (size_t)B * M, fe->mp_updated);
    F(-1, int32_t, B, fe->nview);
    F(-1, int32_t, 1, D.step);
    // time budgets: timers, caps and the clock record
    D.ck_R = std::max(p->gf_budget, 1);
    D.ck_stride = GF_CK_WORDS((long long)M, (long long)D.ck_R);
    F(GF_FE_CLOCK, long long, (size_t)B * D.ck_stride, D.clk);
    F(-1, unsigned long long, B, D.t_frame);
    F(-1, unsigned long long, B, D.t_viz0);
    F(-1, unsigned long long, B, D.t_mat0);
    F(-1, unsigned long long, B, D.t_sel0);
    F(-1, long long, B, D.viz_time);
    F(-1, long long, B, D.cap2_mi);
    F(-1, long long, B, D.rest2);
    F(-1, long long, B, D.cap2_sel);
    F(-1, gf_mp_view, (size_t)B * M, D.vtmp);
    F(-1, int32_t, B, D.ncut);
    F(-1, int32_t, B, D.nlist0);
    F(-1, int32_t, (size_t)B * M, fe->qres);
    F(-1, int32_t, (size_t)B * M, fe->qold);
    F(-1, int32_t, B, fe->merr);
    // the tracking state machine, its gates and the track-loss scratch
    F(GF_FE_TRACK, int32_t, (size_t)B * GF_TR_N, D.track);
    gf_reloc_kf* rkf = nullptr;
    F(GF_FE_RELOC, gf_reloc_kf, (size_t)B * gf::RL_NC, rkf);
    F(-1, int32_t, B, D.m3_nlast);
    F(-1, int32_t, B, D.rl_gate);
    F(-1, int32_t, B, D.nkp_tl);
    F(-1, int32_t, B, D.nkp_fi);
    F(-1, int32_t, B, D.gate_tl);
    F(-1, int32_t, B, D.gate_fi);
    F(-1, int32_t, B, D.gate_post);
    F(-1, int32_t, B, D.nmp_post);
    F(-1, int32_t, B, D.nmp_step);
    F(-1, float, B, D.th_m2);
    F(-1, int32_t, B, fe->d_kfc);
    gf::TrackLossArgs& TL = fe->TL;
    F(-1, int32_t, (size_t)B * gf::grid_ints(cap), TL.grid);
    F(-1, int32_t, (size_t)B * cap, TL.rec);
    F(-1, gf_pose_edge, (size_t)B * cap, TL.edges);
    F(-1, int32_t, (size_t)B * cap, TL.edge_kp);
    F(-1, uint8_t, (size_t)B * cap, TL.eoutl);
    F(-1, double, (size_t)3 * B * cap, TL.pwork);
    F(-1, int32_t, (size_t)4 * B, TL.pint);
    D.max_frames = p->max_frames > 0 ? p->max_frames : (int)(18.0 / (30.0 * p->dt) + 1e-6);  // 18 * fps / 30
    // the stream maps; the working arrays alias them until a keyframe graph is set
    fe->gm = MapArrays{map, mdesc, fe->mp_pos, D.views, fe->mp_H, fe->mp_info, fe->mp_uv, D.upd};
    fe->g_nmp = nmp;
    fe->wdesc = mdesc;
    fe->w_nmp = nmp;
    D.nmp = D.nmp_step;  // TrackLocalMap sees no map on a stream whose initial estimate failed
    D.gmap = map;
    D.gnmp = nmp;
    D.gupd = D.upd;
    D.refmap = 0;
    fe->has_covis.assign(B, 0);
    const uint8_t** ptrs = nullptr;
    F(-1, const uint8_t*, B, ptrs);
    D.ptrs = ptrs;
    const uint8_t** bases = nullptr;
    F(-1, const uint8_t*, B, bases);
    D.bases = bases;
    int32_t* phase = nullptr;
    F(-1, int32_t, B, phase);
    D.phase = phase;
#undef F
    // updateAtFrameId = -1 (never): no stamp equals the current (1) or next (2) frame
    std::vector<int32_t> neg((size_t)B * M, -1000);
    if (hipMemcpy(D.upd, neg.data(), neg.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(gf::fail(GF_ERR_HIP, "upload stamps"));
    // std::srand(1) for every stream until set_rng
    std::vector<gf_rng> r(B);
    for (int b = 0; b < B; b++) gf_rng_seed(&r[b], 1);
    if (hipMemcpy(rng, r.data(), sizeof(gf_rng) * B, hipMemcpyHostToDevice) != hipSuccess)
        return bail(gf::fail(GF_ERR_HIP, "upload rng"));
    std::vector<float> I((size_t)B * 16, 0.f);
    for (int b = 0; b < B; b++)
        for (int i = 0; i < 4; i++) I[16 * b + 5 * i] = 1.f;
    if (hipMemcpy(D.Tcw_last, I.data(), I.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(D.V, I.data(), I.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bail(gf::fail(GF_ERR_HIP, "upload poses"));
    fe->h_kfc.assign(B, -1);  // no keyframe graph: the map is assumed to hold > 5 keyframes
    if (hipMemcpy(fe->d_kfc, fe->h_kfc.data(), 4 * (size_t)B, hipMemcpyHostToDevice) != hipSuccess)
        return bail(gf::fail(GF_ERR_HIP, "upload keyframe counts"));
    fe->h_kfdb.assign(B, gf::KfdbDev{});
    TL.B = B;
    TL.cap = cap;
    TL.M = M;
    TL.budget = p->gf_budget;
    TL.nlevels = p->nlevels;
    TL.fc = gf::make_frame_const(&fe->fi);
    for (int l = 0; l < 16; l++) {
        TL.inv_sigma2[l] = fe->inv_sigma2[l];
        TL.level_sigma2[l] = fe->level_sigma2[l];
    }
    TL.kps = D.kps;
    TL.desc = D.desc;
    TL.nkp = D.nkp;
    TL.kp2mp = D.kp2mp;
    TL.score = D.score;
    TL.outl = D.outl;
    TL.Tcw = D.Tcw;
    TL.last_kps = D.last_kps;
    TL.last_desc = D.last_desc;
    TL.last_nkp = D.last_nkp;
    TL.last_kp2mp = D.last_kp2mp;
    TL.last_pos = D.last_pos;
    TL.Tcw_last = D.Tcw_last;
    TL.gmap = map;
    TL.gdesc = mdesc;
    TL.track = D.track;
    TL.stats = D.stats;
    TL.rng = rng;
    TL.kf_count = fe->d_kfc;
    D.kfc = fe->d_kfc;
    TL.gnmp = nmp;
    TL.nkp_tl = D.nkp_tl;
    TL.nkp_fi = D.nkp_fi;
    TL.gate_tl = D.gate_tl;
    TL.gate_fi = D.gate_fi;
    TL.th_m2 = D.th_m2;
    TL.nmp_step = D.nmp_step;
    TL.rkf = rkf;
    TL.rl_gate = D.rl_gate;
    TL.ncs = 1;
    ctx->frontends++;
    *out = fe;
    return GF_OK;
}

int gf_frontend_destroy(gf_frontend* fe) {
    if (!fe) return GF_OK;
    (void)hipSetDevice(fe->ctx->device);
    (void)hipStreamSynchronize(fe->ctx->stream);
    fe->ctx->frontends--;
    if (fe->fork_s) {
        (void)hipStreamSynchronize(fe->fork_s);
        (void)hipEventDestroy(fe->ev_fork);
        (void)hipEventDestroy(fe->ev_join);
        (void)hipStreamDestroy(fe->fork_s);
    }
    if (fe->ts) {
        fe->ctx->track_stream = false;
        (void)hipStreamSynchronize(fe->ts);
        (void)hipEventDestroy(fe->ev_extracted);
        (void)hipEventDestroy(fe->ev_tracked);
        (void)hipStreamDestroy(fe->ts);
    }
    fe_free(fe);
    delete fe;
    return GF_OK;
}

int gf_frontend_capacity(gf_frontend* fe, int* cap) {
    GF_CHECK(fe && cap, GF_ERR_ARG, "null arg");
    *cap = fe->cap;
    return GF_OK;
}

int gf_frontend_set_source(gf_frontend* fe, const uint8_t* const* d_bases, const int32_t* phase, int period,
                           size_t frame_stride) {
    GF_CHECK(fe && d_bases && phase && period > 0, GF_ERR_ARG, "bad source");
    GF_CHECK(frame_stride >= (size_t)fe->p.width * fe->p.height, GF_ERR_ARG, "frame stride below the image size");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));  // a step in flight reads these buffers
    const int B = fe->D.B;
    for (int b = 0; b < B; b++) GF_CHECK(d_bases[b] && phase[b] >= 0, GF_ERR_ARG, "bad source entry");
    GF_HIP(hipMemcpy((void*)fe->D.bases, d_bases, sizeof(void*) * B, hipMemcpyHostToDevice));
    GF_HIP(hipMemcpy((void*)fe->D.phase, phase, sizeof(int32_t) * B, hipMemcpyHostToDevice));
    fe->D.period = period;
    fe->D.frame_stride = (long long)frame_stride;
    fe->D.src_mode = 1;
    fe->sourced = true;
    return GF_OK;
}

int gf_frontend_set_map(gf_frontend* fe, int stream, const gf_map_point* mps, const uint8_t* desc, int m) {
    GF_CHECK(fe && stream >= 0 && stream < fe->D.B, GF_ERR_ARG, "bad stream");
    GF_CHECK(m >= 0 && m <= fe->D.M && (m == 0 || (mps && desc)), GF_ERR_ARG, "bad map");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));  // a step in flight reads these buffers
    const size_t M = fe->D.M, o = (size_t)stream * M;
    std::vector<float> pos(3 * (size_t)m);
    for (int i = 0; i < m; i++)
        for (int c = 0; c < 3; c++) pos[3 * i + c] = mps[i].pos[c];
    if (m) {
        GF_HIP(hipMemcpy((gf_map_point*)fe->gm.map + o, mps, sizeof(gf_map_point) * m, hipMemcpyHostToDevice));
        GF_HIP(hipMemcpy((uint8_t*)fe->gm.desc + o * 32, desc, 32 * (size_t)m, hipMemcpyHostToDevice));
        GF_HIP(hipMemcpy((float*)fe->gm.pos + 3 * o, pos.data(), 12 * (size_t)m, hipMemcpyHostToDevice));
    }
    GF_HIP(hipMemcpy(fe->g_nmp + stream, &m, 4, hipMemcpyHostToDevice));
    std::vector<int32_t> neg(M, -1000);
    GF_HIP(hipMemcpy(fe->gm.upd + o, neg.data(), 4 * M, hipMemcpyHostToDevice));
    GF_HIP(hipMemset(fe->gm.views + o, 0, sizeof(gf_mp_view) * M));
    if (fe->covis_set) fe->has_covis[stream] = 0;  // the keyframe graph indexes the old points
    return GF_OK;
}

static int fe_enable_covis(gf_frontend* fe) {
    FeDev& D = fe->D;
    const size_t B = D.B, M = D.M;
    int rc;
    void* p;
#define A_(bytes, dst)                                 \
    if ((rc = fe_alloc(fe, (bytes), &p))) return rc; \
    dst = (decltype(dst))p;
    gf_map_point* wmap;
    uint8_t* wdesc;
    A_(sizeof(gf_map_point) * B * M, wmap);
    A_(32 * B * M, wdesc);
    A_(12 * B * M, fe->mp_pos);
    A_(sizeof(gf_mp_view) * B * M, D.views);
    A_(4 * B * M, D.upd);
    A_(4 * B, fe->w_nmp);
    A_(4 * B * M, D.lmp);
    A_(4 * B, D.nlm);
    A_(4 * B * M, D.g2l);
    A_(4 * B * gf_frontend::KF_CAP, fe->lkf);
    A_(4 * B, fe->nlkf);
    A_(4 * B, fe->ref_kf);
    A_(4 * B * M, fe->rm_first);
    fe->slot_cap = (size_t)gf_frontend::KF_CAP * (size_t)D.cap;
    A_(sizeof(gf_covis_map) * B, fe->d_covis);
    A_(B * gf_frontend::KF_CAP, fe->cv_kf_bad);
    A_(4 * B * (gf_frontend::KF_CAP + 1), fe->cv_kf_mp_off);
    A_(4 * B * fe->slot_cap, fe->cv_kf_mp);
    A_(4 * B * (gf_frontend::KF_CAP + 1), fe->cv_kf_cov_off);
    A_(4 * B * gf_frontend::KF_CAP * gf_frontend::KF_CAP, fe->cv_kf_cov);
    A_(B * M, fe->cv_mp_bad);
    A_(4 * B * (M + 1), fe->cv_mp_obs_off);
    A_(4 * B * fe->slot_cap, fe->cv_mp_obs);
#undef A_
    GF_HIP(hipMemset(D.g2l, 0xff, 4 * B * M));
    D.map = wmap;
    D.nmp = fe->w_nmp;
    fe->wdesc = wdesc;
    D.refmap = 1;
    fe->covis_set = 1;
    fe->TL.covis = fe->d_covis;
    fe->h_slots.assign(B, {});
    return GF_OK;
}

int gf_frontend_set_covis(gf_frontend* fe, int stream, const gf_covis_map* g) {
    GF_CHECK(fe && g && stream >= 0 && stream < fe->D.B, GF_ERR_ARG, "bad arguments");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "set keyframe graphs before capturing a graph");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    int32_t nmp = 0;
    GF_HIP(hipMemcpy(&nmp, fe->g_nmp + stream, 4, hipMemcpyDeviceToHost));
    const int nkf = g->nkf;
    GF_CHECK(g->nmp == nmp, GF_ERR_ARG, "the keyframe graph must index the stream's map points (gf_frontend_set_map)");
    GF_CHECK(nkf >= 0 && nkf <= gf_frontend::KF_CAP, GF_ERR_UNSUPPORTED, "at most 64 keyframes per stream graph");
    GF_CHECK(nkf == 0 || (g->kf_bad && g->kf_mp_off && g->kf_cov_off), GF_ERR_ARG, "null keyframe arrays");
    GF_CHECK(nmp == 0 || (g->mp_bad && g->mp_obs_off), GF_ERR_ARG, "null map point arrays");
    if (!fe->covis_set) FE_RC(fe_enable_covis(fe));
    // host validation: the kernels index with these
    const size_t ns = nkf ? (size_t)g->kf_mp_off[nkf] : 0, nc = nkf ? (size_t)g->kf_cov_off[nkf] : 0;
    const size_t no = nmp ? (size_t)g->mp_obs_off[nmp] : 0;
    GF_CHECK(ns <= fe->slot_cap && no <= fe->slot_cap && nc <= (size_t)nkf * nkf, GF_ERR_CAP,
             "keyframe graph larger than the per-stream capacity");
    for (int k = 0; k < nkf; k++)
        GF_CHECK(g->kf_mp_off[k] >= 0 && g->kf_mp_off[k] <= g->kf_mp_off[k + 1] && g->kf_cov_off[k] >= 0 &&
                     g->kf_cov_off[k] <= g->kf_cov_off[k + 1],
                 GF_ERR_ARG, "keyframe offsets must be ascending");
    for (size_t i = 0; i < ns; i++)
        GF_CHECK(g->kf_mp[i] >= -1 && g->kf_mp[i] < nmp, GF_ERR_ARG, "keyframe slot out of range");
    for (size_t i = 0; i < nc; i++) GF_CHECK(g->kf_cov[i] >= 0 && g->kf_cov[i] < nkf, GF_ERR_ARG, "bad covisible keyframe");
    for (int m = 0; m < nmp; m++)
        GF_CHECK(g->mp_obs_off[m] >= 0 && g->mp_obs_off[m] <= g->mp_obs_off[m + 1], GF_ERR_ARG,
                 "observation offsets must be ascending");
    for (size_t i = 0; i < no; i++) GF_CHECK(g->mp_obs[i] >= 0 && g->mp_obs[i] < nkf, GF_ERR_ARG, "bad observation");
    const size_t b = stream, M = fe->D.M, KC = gf_frontend::KF_CAP;
    gf_covis_map d{};
    d.nkf = nkf;
    d.nmp = nmp;
    d.kf_bad = fe->cv_kf_bad + b * KC;
    d.kf_mp_off = fe->cv_kf_mp_off + b * (KC + 1);
    d.kf_mp = fe->cv_kf_mp + b * fe->slot_cap;
    d.kf_cov_off = fe->cv_kf_cov_off + b * (KC + 1);
    d.kf_cov = fe->cv_kf_cov + b * KC * KC;
    d.mp_bad = fe->cv_mp_bad + b * M;
    d.mp_obs_off = fe->cv_mp_obs_off + b * (M + 1);
    d.mp_obs = fe->cv_mp_obs + b * fe->slot_cap;
    auto up = [](const void* dst, const void* src, size_t bytes) -> hipError_t {
        return bytes ? hipMemcpy((void*)dst, src, bytes, hipMemcpyHostToDevice) : hipSuccess;
    };
    if (nkf) {
        GF_HIP(up(d.kf_bad, g->kf_bad, nkf));
        GF_HIP(up(d.kf_mp_off, g->kf_mp_off, 4 * ((size_t)nkf + 1)));
        GF_HIP(up(d.kf_cov_off, g->kf_cov_off, 4 * ((size_t)nkf + 1)));
    }
    GF_HIP(up(d.kf_mp, g->kf_mp, 4 * ns));
    GF_HIP(up(d.kf_cov, g->kf_cov, 4 * nc));
    if (nmp) {
        GF_HIP(up(d.mp_bad, g->mp_bad, nmp));
        GF_HIP(up(d.mp_obs_off, g->mp_obs_off, 4 * ((size_t)nmp + 1)));
    }
    GF_HIP(up(d.mp_obs, g->mp_obs, 4 * no));
    GF_HIP(hipMemcpy(fe->d_covis + b, &d, sizeof(d), hipMemcpyHostToDevice));
    fe->has_covis[b] = 1;
    // KeyFramesInMap() for TrackPreviousFrame's octave floor; a keyframe
    // database set earlier indexed the old graph
    fe->h_kfc[b] = nkf;
    GF_HIP(hipMemcpy(fe->d_kfc + b, &fe->h_kfc[b], 4, hipMemcpyHostToDevice));
    fe->h_slots[b].resize(nkf);
    for (int k = 0; k < nkf; k++) fe->h_slots[b][k] = g->kf_mp_off[k + 1] - g->kf_mp_off[k];
    if (fe->rl_alloc && fe->h_kfdb[b].nkf) FE_RC(gf_frontend_set_kfdb(fe, stream, nullptr));
    return GF_OK;
}

static int fe_enable_reloc(gf_frontend* fe) {
    FeDev& D = fe->D;
    gf::TrackLossArgs& TL = fe->TL;
    const size_t B = D.B, cap = D.cap, NC = gf::RL_NC;
    int rc;
    void* p;
#define A_(bytes, dst)                                 \
    if ((rc = fe_alloc(fe, (bytes), &p))) return rc; \
    dst = (decltype(dst))p;
    A_(sizeof(gf::KfdbDev) * B, fe->d_kfdb);
    A_(4 * B * cap, TL.words);
    A_(8 * B * cap, TL.values);
    A_(4 * B, TL.nwords);
    A_(4 * B * cap, TL.fv_nodes);
    A_(4 * B * (cap + 1), TL.fv_start);
    A_(4 * B * cap, TL.fv_feats);
    A_(4 * B, TL.nfv);
    A_(16 * B * cap, fe->bow_tmp);
    A_(sizeof(gf::BowPairDev) * B * NC, TL.pairs);
    A_(4 * B * NC * cap, TL.bow_out);
    A_(4 * B * NC, TL.bow_nm);
    A_(4 * B * NC, TL.cands);
    A_(4 * B, TL.ncand);
    A_(sizeof(gf_pnp_state) * B * NC, TL.pst);
    A_(B * NC * cap, TL.pbest);
    A_(12 * B * cap, TL.p3d);
    A_(8 * B * cap, TL.p2d);
    A_(4 * B * cap, TL.psig);
    A_(4 * B * cap, TL.pidx);
    A_(B * cap, TL.pinl);
    A_(4 * B * gf::RL_LCAP * 8, TL.pdraws);
    A_(8 * B * gf::RL_LCAP * 12, TL.prt);
    A_(4 * B * gf::RL_LCAP, TL.pcnt);
    A_(8 * B * cap * gf::RL_WORK, TL.pwk);
    A_(4 * B * 16, TL.ptcw);
    A_(4 * B * 2, TL.pflags);
#undef A_
    TL.kfdb = fe->d_kfdb;
    fe->rl_alloc = true;
    return GF_OK;
}

int gf_frontend_set_kfdb(gf_frontend* fe, int stream, gf_kfdb* db) {
    GF_CHECK(fe && stream >= 0 && stream < fe->D.B, GF_ERR_ARG, "bad stream");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "set keyframe databases before capturing a graph");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    gf::KfdbDev v{};
    if (db) {
        v = gf::kfdb_dev(db);
        GF_CHECK(fe->covis_set && fe->has_covis[stream], GF_ERR_ARG,
                 "a keyframe database needs the stream's keyframe graph (gf_frontend_set_covis)");
        GF_CHECK(v.nkf == fe->h_kfc[stream], GF_ERR_ARG, "the database and the keyframe graph differ in keyframes");
        std::vector<int32_t> off(v.nkf + 1);
        GF_HIP(hipMemcpy(off.data(), v.kp_off, 4 * off.size(), hipMemcpyDeviceToHost));
        for (int k = 0; k < v.nkf; k++)
            GF_CHECK(off[k + 1] - off[k] == fe->h_slots[stream][k], GF_ERR_ARG,
                     "keyframe " + std::to_string(k) + ": keypoints and graph slots differ");
    }
    if (!fe->rl_alloc) FE_RC(fe_enable_reloc(fe));
    fe->h_kfdb[stream] = v;
    GF_HIP(hipMemcpy(fe->d_kfdb + stream, &v, sizeof(v), hipMemcpyHostToDevice));
    GF_HIP(hipMemset(fe->TL.rkf + (size_t)stream * gf::RL_NC, 0, sizeof(gf_reloc_kf) * gf::RL_NC));
    GF_HIP(hipMemset(fe->TL.ncand + stream, 0, 4));  // no candidates of an earlier database survive
    int ncs = 1;
    for (const gf::KfdbDev& k : fe->h_kfdb) ncs = std::max(ncs, k.nkf);
    fe->TL.ncs = ncs;
    fe->rl_on = fe->voc && ncs > 0 && std::any_of(fe->h_kfdb.begin(), fe->h_kfdb.end(),
                                                  [](const gf::KfdbDev& k) { return k.nkf > 0; });
    fe->TL.rl_on = fe->rl_on;
    return GF_OK;
}

int gf_frontend_set_vocab(gf_frontend* fe, gf_vocab* voc) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "set the vocabulary before capturing a graph");
    if (fe->rl_alloc) {  // candidates computed with another vocabulary are not this step's
        GF_HIP(hipSetDevice(fe->ctx->device));
        GF_HIP(hipStreamSynchronize(fe->ctx->stream));
        GF_HIP(hipMemset(fe->TL.ncand, 0, 4 * (size_t)fe->D.B));
    }
    fe->voc = voc;
    fe->rl_on = fe->voc && std::any_of(fe->h_kfdb.begin(), fe->h_kfdb.end(),
                                       [](const gf::KfdbDev& k) { return k.nkf > 0; });
    fe->TL.rl_on = fe->rl_on;
    return GF_OK;
}

int gf_frontend_set_rng(gf_frontend* fe, int stream, uint32_t seed) {
    GF_CHECK(fe && stream >= 0 && stream < fe->D.B, GF_ERR_ARG, "bad stream");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));  // a step in flight reads these buffers
    gf_rng r;
    gf_rng_seed(&r, seed);
    GF_HIP(hipMemcpy((gf_rng*)fe->field_ptr[GF_FE_RNG] + stream, &r, sizeof(r), hipMemcpyHostToDevice));
    return GF_OK;
}

static int fe_staging(gf_frontend* fe, const uint8_t* imgs) {
    FeDev& D = fe->D;
    const size_t fb = (size_t)fe->p.width * fe->p.height;
    if (!fe->staging) {
        void* p = nullptr;
        FE_RC(fe_alloc(fe, fb * D.B, &p));
        fe->staging = (uint8_t*)p;
        std::vector<const uint8_t*> ptr(D.B);
        for (int b = 0; b < D.B; b++) ptr[b] = fe->staging + fb * b;
        GF_HIP(hipMemcpy((void*)D.ptrs, ptr.data(), sizeof(void*) * D.B, hipMemcpyHostToDevice));
    }
    GF_HIP(hipMemcpyAsync(fe->staging, imgs, fb * D.B, hipMemcpyHostToDevice, fe->ctx->stream));
    return GF_OK;
}

static int fe_bootstrap(gf_frontend* fe, const float* Tcw, const float* V, double t0, bool host);

int gf_frontend_bootstrap(gf_frontend* fe, const float* Tcw, const float* V, double t0) {
    GF_CHECK(fe && Tcw && V, GF_ERR_ARG, "null arg");
    GF_CHECK(fe->sourced, GF_ERR_ARG, "no frame source set");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    return fe_bootstrap(fe, Tcw, V, t0, false);
}

int gf_frontend_bootstrap_host(gf_frontend* fe, const uint8_t* imgs, const float* Tcw, const float* V, double t0) {
    GF_CHECK(fe && imgs && Tcw && V, GF_ERR_ARG, "null arg");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    GF_HIP(hipSetDevice(fe->ctx->device));
    FE_RC(fe_staging(fe, imgs));
    return fe_bootstrap(fe, Tcw, V, t0, true);
}

static int fe_bootstrap(gf_frontend* fe, const float* Tcw, const float* V, double t0, bool host) {
    GF_HIP(hipSetDevice(fe->ctx->device));
    FeDev& D = fe->D;
    const int B = D.B, cap = D.cap, M = D.M;
    hipStream_t s = fe->ctx->stream;
    gf_ctx* ctx = fe->ctx;
    std::vector<double> t(B, t0);
    GF_HIP(hipMemcpyAsync(D.Tcw, Tcw, sizeof(float) * 16 * B, hipMemcpyHostToDevice, s));
    GF_HIP(hipMemcpyAsync(D.V, V, sizeof(float) * 16 * B, hipMemcpyHostToDevice, s));
    GF_HIP(hipMemcpyAsync(D.t_cur, t.data(), sizeof(double) * B, hipMemcpyHostToDevice, s));
    if (!host) {
        GF_LAUNCH(k_fe_boot_begin, (B + 63) / 64, 64, 0, s, D);
        GF_HIP(hipGetLastError());
    } else {  // the step counter still advances: a sourced step after a host bootstrap continues the loop
        FeDev Dh = D;
        Dh.src_mode = 0;
        GF_LAUNCH(k_fe_boot_begin, (B + 63) / 64, 64, 0, s, Dh);
        GF_HIP(hipGetLastError());
    }
    GF_HIP(hipMemsetAsync(D.kp2mp, 0xff, sizeof(int32_t) * B * cap, s));
    std::vector<int32_t> s999((size_t)B * cap, 999);
    GF_HIP(hipMemcpyAsync(D.score, s999.data(), 4 * s999.size(), hipMemcpyHostToDevice, s));
    FE_RC(gf_orb_extract_ptrs_dev(fe->ex, B, (const uint8_t* const*)D.ptrs, fe->p.width, D.kps, D.desc, D.nkp, cap,
                                  s));
    FE_RC(fe_undistort(fe, s));
    // the first frame is matched against the whole stream map (with keyframe
    // graphs too: a local map needs the matches of a tracked frame)
    FE_RC(gf_frustum_dev(ctx, &fe->fi, B, D.Tcw, fe->gm.map, fe->g_nmp, M, 0.5f, fe->gm.views, fe->nview, s));
    FE_RC(gf_match_project_dev(ctx, &fe->fi, B, D.kps, D.desc, D.nkp, cap, fe->gm.views, fe->gm.desc, fe->g_nmp, M,
                               1.f, 0.8f, D.kp2mp, D.score, fe->scratch, s));
    GF_LAUNCH(k_fe_boot_end, B, 256, 0, s, D);
    GF_HIP(hipGetLastError());
    GF_HIP(hipStreamSynchronize(s));
    return GF_OK;
}

int gf_event_create(gf_ctx* ctx, void** out) {
    GF_CHECK(ctx && out, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    hipEvent_t e = nullptr;
    GF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = (void*)e;
    return GF_OK;
}

int gf_event_destroy(void* ev) {
    if (ev) GF_HIP(hipEventDestroy((hipEvent_t)ev));
    return GF_OK;
}

int gf_frontend_set_gate(gf_frontend* fe, void* wait_event, void* done_event) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "a captured front end cannot be gated");
    fe->gate_wait = (hipEvent_t)wait_event;
    fe->gate_done = (hipEvent_t)done_event;
    return gf::extract_stage_event(fe->ex, fe->gate_done && fe->gate_stage < 4 ? done_event : nullptr,
                                   fe->gate_stage);
}

int gf_frontend_set_gate_stage(gf_frontend* fe, int stage) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(stage >= 0 && stage <= 4, GF_ERR_ARG, "gate stage must be 0 (resize) .. 4 (describe)");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "a captured front end cannot be gated");
    fe->gate_stage = stage;
    return gf::extract_stage_event(fe->ex, fe->gate_done && stage < 4 ? (void*)fe->gate_done : nullptr, stage);
}

int gf_frontend_set_track_priority(gf_frontend* fe, int priority) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "a captured front end cannot change streams");
    GF_CHECK(!fe->ts, GF_ERR_ARG, "the tracking stream is already set");
    // the tracking kernels use the context's scratch slots: a second front end
    // on the context would run its kernels concurrently on the same buffers
    GF_CHECK(fe->ctx->frontends == 1, GF_ERR_ARG,
             "a front end with a tracking stream needs a context of its own (another front end shares it)");
    GF_HIP(hipSetDevice(fe->ctx->device));
    int least = 0, greatest = 0;
    GF_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    const int pr = std::max(std::min(priority, least), greatest);  // lower value = higher priority
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    GF_HIP(hipStreamCreateWithPriority(&fe->ts, hipStreamNonBlocking, pr));
    GF_HIP(hipEventCreateWithFlags(&fe->ev_extracted, hipEventDisableTiming));
    GF_HIP(hipEventCreateWithFlags(&fe->ev_tracked, hipEventDisableTiming));
    fe->ctx->track_stream = true;
    return GF_OK;
}

static int fe_check_covis(gf_frontend* fe) {
    if (!fe->covis_set) return GF_OK;
    for (int b = 0; b < fe->D.B; b++)
        GF_CHECK(fe->has_covis[b], GF_ERR_ARG, "stream " + std::to_string(b) + " has no keyframe graph");
    return GF_OK;
}

int gf_frontend_step(gf_frontend* fe) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    GF_CHECK(fe->sourced || fe->D.src_mode == 2, GF_ERR_ARG, "no frame source set");
    FE_RC(fe_check_covis(fe));
    GF_HIP(hipSetDevice(fe->ctx->device));
    // budgets of the context, as device clock ticks (100 MHz)
    auto ticks = [](double s) -> long long { return std::isfinite(s) && s >= 0 ? (long long)(s * 1e8) : -1; };
    const long long mt = ticks(fe->ctx->match_budget_s), stt = ticks(fe->ctx->select_budget_s);
    if (fe->exec && mt == fe->D.match_ticks && stt == fe->D.select_ticks) {
        GF_HIP(hipGraphLaunch(fe->exec, fe->ctx->stream));
        return GF_OK;
    }
    if (fe->exec) {  // budgets changed: the tick limits are kernel arguments, so capture again
        FE_RC(gf_frontend_capture(fe));
        GF_HIP(hipGraphLaunch(fe->exec, fe->ctx->stream));
        return GF_OK;
    }
    fe->D.match_ticks = mt;
    fe->D.select_ticks = stt;
    return fe_track(fe, fe->ctx->stream);
}

int gf_frontend_step_extract(gf_frontend* fe) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(fe->sourced || fe->D.src_mode == 2, GF_ERR_ARG, "no frame source set");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "a captured front end steps as one graph (gf_frontend_step)");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    FE_RC(fe_check_covis(fe));
    GF_HIP(hipSetDevice(fe->ctx->device));
    auto ticks = [](double s) -> long long { return std::isfinite(s) && s >= 0 ? (long long)(s * 1e8) : -1; };
    fe->D.match_ticks = ticks(fe->ctx->match_budget_s);
    fe->D.select_ticks = ticks(fe->ctx->select_budget_s);
    FE_RC(fe_extract(fe, fe->ctx->stream));
    fe->extracted = true;
    return GF_OK;
}

int gf_frontend_step_track(gf_frontend* fe) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(fe->extracted, GF_ERR_ARG, "no extracted frame (gf_frontend_step_extract first)");
    GF_HIP(hipSetDevice(fe->ctx->device));
    fe->extracted = false;
    return fe_track_frame(fe, fe->ctx->stream);
}

int gf_frontend_step_host(gf_frontend* fe, const uint8_t* imgs) {
    GF_CHECK(fe && imgs, GF_ERR_ARG, "null arg");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    FE_RC(fe_check_covis(fe));
    GF_HIP(hipSetDevice(fe->ctx->device));
    FeDev& D = fe->D;
    hipStream_t s = fe->ctx->stream;
    FE_RC(fe_staging(fe, imgs));
    const int mode = D.src_mode;
    D.src_mode = 2;  // pointers stay on the staging buffer
    auto ticks = [](double v) -> long long { return std::isfinite(v) && v >= 0 ? (long long)(v * 1e8) : -1; };
    D.match_ticks = ticks(fe->ctx->match_budget_s);
    D.select_ticks = ticks(fe->ctx->select_budget_s);
    int rc = fe_track(fe, s);
    D.src_mode = mode;
    if (mode == 1) {  // the next sourced step recomputes its pointers
    }
    return rc;
}

int gf_frontend_capture(gf_frontend* fe) {
    GF_CHECK(fe && fe->sourced, GF_ERR_ARG, "capture needs a frame source");
    GF_CHECK(!fe->extracted, GF_ERR_ARG, "the extracted frame has not been tracked (gf_frontend_step_track)");
    FE_RC(fe_check_covis(fe));
    // a recorded event in a graph is not the caller's event at replay: the
    // extraction gate would silently stop gating
    GF_CHECK(!fe->gate_wait && !fe->gate_done, GF_ERR_ARG, "a gated front end cannot be captured as a graph");
    GF_CHECK(!fe->ts, GF_ERR_ARG, "a front end with a tracking stream cannot be captured as a graph");
    GF_HIP(hipSetDevice(fe->ctx->device));
    hipStream_t s = fe->ctx->stream;
    GF_HIP(hipStreamSynchronize(s));
    fe_drop_graph(fe);
    auto ticks = [](double v) -> long long { return std::isfinite(v) && v >= 0 ? (long long)(v * 1e8) : -1; };
    fe->D.match_ticks = ticks(fe->ctx->match_budget_s);
    fe->D.select_ticks = ticks(fe->ctx->select_budget_s);
    const bool prof = fe->ctx->prof;
    fe->ctx->prof = false;  // no event records inside the graph
    if (!fe->fork_s) {
        GF_HIP(hipStreamCreateWithFlags(&fe->fork_s, hipStreamNonBlocking));
        GF_HIP(hipEventCreateWithFlags(&fe->ev_fork, hipEventDisableTiming));
        GF_HIP(hipEventCreateWithFlags(&fe->ev_join, hipEventDisableTiming));
    }
    fe->fork_post = true;
    GF_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = fe_track(fe, s);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(s, &g);
    fe->fork_post = false;
    fe->ctx->prof = prof;
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) return gf::fail(GF_ERR_HIP, std::string("capture: ") + hipGetErrorString(e));
    fe->graph = g;
    fe->ctx->ws_pinned++;  // the graph's kernels hold the context's scratch pointers
    GF_HIP(hipGraphInstantiate(&fe->exec, g, nullptr, nullptr, 0));
    return GF_OK;
}

int gf_frontend_sync(gf_frontend* fe) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    return GF_OK;
}

int gf_frontend_field(gf_frontend* fe, int field, size_t* bytes, void** d_ptr) {
    GF_CHECK(fe && field >= 0 && field < GF_FE_NFIELDS, GF_ERR_ARG, "bad field");
    if (bytes) *bytes = fe->field_bytes[field];
    if (d_ptr) *d_ptr = fe->field_ptr[field];
    return GF_OK;
}

int gf_frontend_read(gf_frontend* fe, int field, void* host, size_t bytes) {
    GF_CHECK(fe && host && field >= 0 && field < GF_FE_NFIELDS, GF_ERR_ARG, "bad field");
    GF_CHECK(bytes == fe->field_bytes[field], GF_ERR_ARG,
             "field size is " + std::to_string(fe->field_bytes[field]) + " bytes");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    GF_HIP(hipMemcpy(host, fe->field_ptr[field], bytes, hipMemcpyDeviceToHost));
    return GF_OK;
}

int gf_frontend_write(gf_frontend* fe, int field, const void* host, size_t bytes) {
    GF_CHECK(fe && host && field >= 0 && field < GF_FE_NFIELDS, GF_ERR_ARG, "bad field");
    GF_CHECK(bytes == fe->field_bytes[field], GF_ERR_ARG,
             "field size is " + std::to_string(fe->field_bytes[field]) + " bytes");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    GF_HIP(hipMemcpy(fe->field_ptr[field], host, bytes, hipMemcpyHostToDevice));
    if (field == GF_FE_MP_INFO) {  // keep the packed lower triangles the active matcher reads
        const size_t n = bytes / (49 * sizeof(double));
        const double* b = (const double*)host;
        std::vector<double> lt(32 * n, 0.0);
        for (size_t q = 0; q < n; q++)
            for (int i = 0; i < 7; i++)
                for (int j = 0; j <= i; j++) lt[32 * q + i * (i + 1) / 2 + j] = b[49 * q + 7 * i + j];
        GF_HIP(hipMemcpy(fe->mp_info_lt, lt.data(), lt.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    if (field == GF_FE_MAP) {  // keep the float3 position copy the Jacobian kernels read
        const size_t n = bytes / sizeof(gf_map_point);
        const gf_map_point* m = (const gf_map_point*)host;
        std::vector<float> pos(3 * n);
        for (size_t i = 0; i < n; i++)
            for (int c = 0; c < 3; c++) pos[3 * i + c] = m[i].pos[c];
        GF_HIP(hipMemcpy((float*)fe->gm.pos, pos.data(), 12 * n, hipMemcpyHostToDevice));
    }
    return GF_OK;
}

int gf_frontend_set_test_clock(gf_frontend* fe, const long long* base_slope) {
    GF_CHECK(fe, GF_ERR_ARG, "null front end");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "set the test clock before capturing a graph");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    if (!base_slope) {
        fe->D.syn = nullptr;
        return GF_OK;
    }
    if (!fe->d_syn) {
        void* p;
        FE_RC(fe_alloc(fe, sizeof(long long) * 2 * GF_CK_NSITE, &p));
        fe->d_syn = (long long*)p;
    }
    GF_HIP(hipMemcpy(fe->d_syn, base_slope, sizeof(long long) * 2 * GF_CK_NSITE, hipMemcpyHostToDevice));
    fe->D.syn = fe->d_syn;
    return GF_OK;
}

int gf_frontend_set_time_log(gf_frontend* fe, int steps) {
    GF_CHECK(fe && steps >= 0, GF_ERR_ARG, "bad arg");
    GF_CHECK(!fe->exec, GF_ERR_ARG, "set the time log before capturing a graph");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    if (steps > fe->tl_alloc) {
        void *a, *b;
        FE_RC(fe_alloc(fe, sizeof(long long) * GF_TL_NSITE * (size_t)steps, &a));
        FE_RC(fe_alloc(fe, sizeof(gf_time_rec) * (size_t)fe->D.B * steps, &b));
        fe->D.tl_stamp = (long long*)a;
        fe->D.tl_rec = (gf_time_rec*)b;
        fe->tl_alloc = steps;
    } else if (steps) {
        GF_HIP(hipMemset(fe->D.tl_stamp, 0, sizeof(long long) * GF_TL_NSITE * (size_t)steps));
        GF_HIP(hipMemset(fe->D.tl_rec, 0, sizeof(gf_time_rec) * (size_t)fe->D.B * steps));
    }
    fe->D.tl_cap = steps;
    int32_t st = 0;
    GF_HIP(hipMemcpy(&st, fe->D.step, sizeof(int32_t), hipMemcpyDeviceToHost));
    fe->tl_first = st;  // the first step the log holds
    return GF_OK;
}

int gf_frontend_read_time_log(gf_frontend* fe, long long* stamps, gf_time_rec* recs, int* nsteps) {
    GF_CHECK(fe && stamps && recs && nsteps, GF_ERR_ARG, "null arg");
    GF_CHECK(fe->D.tl_cap > 0, GF_ERR_ARG, "the time log is off (gf_frontend_set_time_log)");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    int32_t st = 0;
    GF_HIP(hipMemcpy(&st, fe->D.step, sizeof(int32_t), hipMemcpyDeviceToHost));
    const int cap = fe->D.tl_cap, B = fe->D.B;
    const int n = std::min(cap, std::max(0, st - fe->tl_first));
    std::vector<long long> hs((size_t)cap * GF_TL_NSITE);
    std::vector<gf_time_rec> hr((size_t)cap * B);
    GF_HIP(hipMemcpy(hs.data(), fe->D.tl_stamp, sizeof(long long) * hs.size(), hipMemcpyDeviceToHost));
    GF_HIP(hipMemcpy(hr.data(), fe->D.tl_rec, sizeof(gf_time_rec) * hr.size(), hipMemcpyDeviceToHost));
    for (int k = 0; k < n; k++) {  // oldest first
        const int slot = (st - n + k) % cap;
        memcpy(stamps + (size_t)k * GF_TL_NSITE, hs.data() + (size_t)slot * GF_TL_NSITE, sizeof(long long) * GF_TL_NSITE);
        memcpy(recs + (size_t)k * B, hr.data() + (size_t)slot * B, sizeof(gf_time_rec) * B);
    }
    *nsteps = n;
    return GF_OK;
}

int gf_set_budgets(gf_ctx* ctx, double match_s, double select_s) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    GF_CHECK(!(match_s < 0) && !(select_s < 0), GF_ERR_ARG, "negative budget");
    ctx->match_budget_s = match_s;
    ctx->select_budget_s = select_s;
    return GF_OK;
}

}  // extern "C"

// Map-state broadcast: every stream's local map (points,
// descriptors, sizes) of rank `root`'s front end into the front ends of all
// ranks (same batch and map capacity), device to device; the observability
// state of the received streams starts fresh as after gf_frontend_set_map.
extern "C" int gf_dist_bcast_map(gf_dist* d, gf_frontend* fe, int root) {
    GF_CHECK(d && fe, GF_ERR_ARG, "null arg");
    GF_CHECK(gf::dist_ctx(d)->device == fe->ctx->device, GF_ERR_ARG, "communicator and front end on different devices");
    GF_HIP(hipSetDevice(fe->ctx->device));
    GF_HIP(hipStreamSynchronize(fe->ctx->stream));
    int rc;
    if ((rc = gf::dist_bcast(d, fe->field_ptr[GF_FE_MAP], fe->field_bytes[GF_FE_MAP], root)) ||
        (rc = gf::dist_bcast(d, fe->field_ptr[GF_FE_MAP_DESC], fe->field_bytes[GF_FE_MAP_DESC], root)) ||
        (rc = gf::dist_bcast(d, fe->field_ptr[GF_FE_NMP], fe->field_bytes[GF_FE_NMP], root)) ||
        (rc = gf::dist_bcast(d, (void*)fe->gm.pos, sizeof(float) * 3 * (size_t)fe->D.B * fe->D.M, root)))
        return rc;
    GF_HIP(hipStreamSynchronize(gf::dist_ctx(d)->stream));
    if (gf::dist_rank(d) != root) {
        const size_t n = (size_t)fe->D.B * fe->D.M;
        std::vector<int32_t> neg(n, -1000);
        GF_HIP(hipMemcpy(fe->gm.upd, neg.data(), 4 * n, hipMemcpyHostToDevice));
        GF_HIP(hipMemset(fe->gm.views, 0, sizeof(gf_mp_view) * n));
    }
    return GF_OK;
}

