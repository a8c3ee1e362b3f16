// Shared runtime pieces of libgfslam: error capture, context, device helpers.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/gfslam/abi.h"

namespace gf {

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

#define GF_HIP(expr)                                                                       \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return ::gf::fail(GF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define GF_CHECK(cond, code, msg)                     \
    do {                                              \
        if (!(cond)) return ::gf::fail((code), (msg)); \
    } while (0)

}  // namespace gf

namespace gf {
// Per-kernel HIP-event timing (enabled by gf_prof_enable): every launch site
// brackets its kernel with an event pair on the launch stream.
struct ProfEntry {
    std::string name;
    std::vector<hipEvent_t> start, stop;  // pairs, recorded in order
};
}  // namespace gf

struct gf_ctx {
    int device = 0;
    int num_cus = 256;  // compute units of the device (launch-shape choices)
    hipStream_t stream = nullptr;
    bool prof = false;
    // gf_set_budgets: reference time budgets in seconds (+inf = parity mode)
    double match_budget_s = __builtin_inf(), select_budget_s = __builtin_inf();
    std::vector<gf::ProfEntry> prof_entries;
    std::vector<hipEvent_t> event_pool;
    std::vector<hipEvent_t> prof_spent;  // stop events of multi-launch scopes that are not read
    // grow-only device scratch for the host-family wrappers (one slot per use)
    static const int kSlots = 64;
    void* ws[kSlots] = {};
    size_t ws_size[kSlots] = {};
    // captured graphs (gf_frontend_capture) alive on this context: their
    // kernels hold scratch pointers, so no slot may be reallocated meanwhile
    int ws_pinned = 0;
    // front ends on this context, and whether one runs its tracking kernels on
    // a stream of its own (gf_frontend_set_track_priority): its kernels take
    // the context's scratch slots, so it must be the only front end here
    int frontends = 0;
    bool track_stream = false;
};

namespace gf {
// Device scratch buffer `slot` of at least `bytes` (grow-only, owned by ctx).
int ws_get(gf_ctx* ctx, int slot, size_t bytes, void** out);
// record `ev` on the extraction stream after stage `after` (0 resize, 1 blur +
// FAST map, 2 cells, 3 select, 4 describe) of the extractor's next runs; null
// clears it (the front end's extraction gate, gf_frontend_set_gate)
int extract_stage_event(::gf_extractor* ex, void* ev, int after);
// Host-family helper: copy host -> scratch slot (returns device pointer).
int ws_upload(gf_ctx* ctx, int slot, const void* host, size_t bytes, void** out);

// UpdateReference of B frames, each against its own keyframe graph (refmap.hip).
int update_reference_frames(gf_ctx* ctx, const gf_covis_map* d_maps, int nmp_cap, int nframes, int32_t* d_frame_mps,
                            const int32_t* d_nkps, int stride, int32_t* d_local_kfs, int32_t* d_n_local_kfs,
                            int kf_cap, int32_t* d_local_mps, int32_t* d_n_local_mps, int mp_cap, int32_t* d_ref_kf,
                            int32_t* d_first, int kf_max, hipStream_t s);

// The observability passes with the map-point state (H / ObsMat / u_proj) kept
// in map order while the step runs over a local map: local point q of frame f
// reads and writes entry remap[f * map_stride + q] (null: q itself). The
// extern "C" gf_obs_*_dev entry points are these with remap = null (gf.hip).
// d_info_lt (optional, [F][map_stride][32] doubles): the writers also store
// each ObsMat's lower triangle packed there, and obs_active_match's log-dets
// read it (logdet_sum_lower_packed) instead of the 49-entry block.
int obs_frame_info(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const gf_keypoint* d_kps,
                   const int32_t* d_nkps, int kp_stride, const int32_t* d_kp2mp, const uint8_t* d_outlier,
                   const float* d_map_pos, const int32_t* d_nmp, int map_stride, const float* level_sigma2,
                   int nlevels, double* d_H, double* d_info, float* d_uv, const int32_t* d_remap, void* stream,
                   double* d_info_lt = nullptr);
// One stage's time-budget clock in the front end (gf_set_budgets): the timer
// start of every frame (s_memrealtime ticks), the clock record ([F][stride]
// int64, GF_FE_CLOCK) and the offset of the stage's elapsed-time array in it.
// t0 == null: the stage runs without a budget and reads no clock.
struct StageClock {
    const unsigned long long* t0 = nullptr;
    long long* rec = nullptr;
    long long stride = 0;
    int off = 0;
    // test clock (gf_frontend_set_test_clock): the site's (base, slope) pair
    // (for the budget matcher two pairs: its start, then its points); null:
    // the device clock
    const long long* syn = nullptr;
};

// batchInfoMat_Map with its time cap (Observability.cc:564-578) when ck.t0 is
// set: each 64-point batch reads the clock once and is skipped when 2 x its
// elapsed time > cap2[f] (2 x the cap in ticks; < 0 skips every batch).
int obs_map_info(gf_ctx* ctx, const gf_obs_camera* cam, int nframes, const double* d_Xv, const float* d_map_pos,
                 const int32_t* d_nmp, int map_stride, int check_viz, const gf_mp_view* d_views, int32_t* d_upd_id,
                 int frame_id, double* d_H, double* d_info, float* d_uv, uint8_t* d_updated, const int32_t* d_remap,
                 void* stream, const StageClock& ck = StageClock{}, const long long* d_cap2 = nullptr,
                 double* d_info_lt = nullptr);

// runActiveMapMatching's time cap (Observability.cc:1260, 1366-1370) for the
// front end: time_for_match = match_ticks - time_Mat_Online - time_Viz, with
// time_Mat_Online measured from mat_t0[f] (Tracking.cc:3311) to the kernel's
// start and time_Viz = viz[f]. ck.t0 unused (the kernel starts its own timer).
struct ActiveClock {
    const unsigned long long* mat_t0 = nullptr;  // null: no budget
    const long long* viz = nullptr;
    long long match_ticks = 0;
    long long* rec = nullptr;
    long long stride = 0;
    int off = 0;    // per-round array
    int rounds = 0; // its length
    const long long* syn = nullptr;  // test clock: (base, slope) of the start, then of the rounds
};

// Frame::isInFrustum over a map (d_list null: points < d_m[f]) or over a list,
// clocked as gf_set_budgets describes when ck.t0 is set: results go to d_alt.
int frustum_clocked(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw, const gf_map_point* d_mps,
                    const int32_t* d_m, const int32_t* d_list, const int32_t* d_nlist, int mp_cap,
                    float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview, const StageClock& ck,
                    gf_mp_view* d_alt, void* stream);
// SearchByProjection_Budget (ORBmatcher.cc:276-379) over a list with its clock:
// d_rest2[f] = 2 x timeCost_rest, ck.t0 = the visibility pass's timer start.
int match_project_list_budget(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                              const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                              const uint8_t* d_mp_desc, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                              float th, float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches,
                              const StageClock& ck, const long long* d_rest2, int32_t* d_qres, int32_t* d_old,
                              int32_t* d_err, void* stream);
int obs_accumulate_matched(gf_ctx* ctx, int nframes, const int32_t* d_kp2mp, const int32_t* d_nkps, int kp_stride,
                           const double* d_info, const int32_t* d_upd_id, const int32_t* d_nmp, int map_stride,
                           int frame_id, double diag, double* d_out, const int32_t* d_remap, void* stream,
                           const int32_t* d_gate = nullptr);
// gf_obs_update_dev for the frames with d_gate[f] != 0 (null: all)
int obs_update_gated(gf_ctx* ctx, int nframes, const double* d_t_prev, const float* d_Tcw_prev, const double* d_t_cur,
                     const float* d_Tcw_cur, double* d_Xv, double* d_Xv_next, const int32_t* d_gate, void* stream);
// gf_pose_opt_frames_dev; a frame with d_gate[f] < gate_min is not optimised
// at all (its pose, flags and counts untouched)
int pose_opt_frames_gated(gf_ctx* ctx, int nframes, float* d_Tcw, const gf_keypoint* d_kps, const int32_t* d_nkps,
                          int kp_stride, const int32_t* d_kp2mp, const gf_map_point* d_map, int map_stride,
                          const float* inv_sigma2, int nlevels, float fx, float fy, float cx, float cy,
                          uint8_t* d_outlier, int32_t* d_ninliers, int32_t* d_iterations, int32_t* d_nedges,
                          const int32_t* d_gate, int gate_min, void* stream);
// gf_match_project_dev with a window factor per frame (d_th[f], the th of
// SearchByProjection(F, vpMapPoints, th))
int match_project_th(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                     const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                     const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, const float* d_th, float nnratio,
                     int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream);
// gf_bow_transform_dev over the frames with d_gate[f] != 0 (others: empty vectors)
int bow_transform_gated(gf_vocab* voc, int nframes, const uint8_t* d_desc, const int32_t* d_n, const int32_t* d_gate,
                        int cap, int levelsup, int32_t* d_words, double* d_values, int32_t* d_nwords,
                        int32_t* d_fv_nodes, int32_t* d_fv_start, int32_t* d_fv_feats, int32_t* d_nfv, void* d_tmp,
                        void* stream);  // d_tmp: nframes x cap x 16 bytes
// One ORBmatcher::SearchByBoW pair whose description already lives in device
// memory (gf_match_bow_dev copies host-built pairs).
struct BowPairDev {
    gf_bow_side a, b;
    int32_t* out;
};
int match_bow_pairs(gf_ctx* ctx, int mode, float nnratio, int check_ori, int npairs, const BowPairDev* d_pairs,
                    int32_t* d_nmatches, int bcap, void* stream);
int obs_active_match(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                     const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                     const uint8_t* d_mp_desc, const uint8_t* d_updated, const double* d_info, const double* d_H,
                     const int32_t* d_m, int mp_cap, const double* d_base, const float* level_sigma2,
                     const int32_t* d_num_to_match, float th, float nnratio, gf_rng* d_rng, int32_t* d_kp2mp,
                     int32_t* d_score, int32_t* d_left, int32_t* d_nleft, int32_t* d_nmatched, int32_t* d_nldet,
                     const int32_t* d_remap, void* stream, const ActiveClock& ck = ActiveClock{},
                     const double* d_info_lt = nullptr);

// Candidate counting for the front end's matcher calls (SURVEY §8d B_match's
// C): while a CandidateCount lives on this thread, every projection-matcher
// launch (match.hip) adds each frame's window candidate count (the
// GetFeaturesInArea sizes) to d_counts[f].
struct CandidateCount {
    int32_t* prev;
    explicit CandidateCount(int32_t* d_counts);
    ~CandidateCount();
};
int32_t* candidate_counts();

// RCCL broadcast on the communicator's stream (dist.hip), asynchronous.
int dist_bcast(gf_dist* d, void* buf, size_t bytes, int root);
int dist_rank(gf_dist* d);
gf_ctx* dist_ctx(gf_dist* d);

// Per-kernel timing when profiling is on (gf_prof_enable): a ProfScope names
// the launches made while it is the innermost open scope on this thread
// (GF_LAUNCH). Their start / stop events are taken from the kernels' own
// dispatch timestamps (hipExtLaunchKernel), not recorded on the stream
// around them, so a kernel waiting for compute units held by another stream's
// kernels does not count that wait (the figure rocprof reports). A scope
// with several launches spans the first one's start to the last one's end.
struct ProfScope {
    gf_ctx* ctx;
    hipStream_t s;
    int idx = -1;
    ProfScope* prev = nullptr;
    hipEvent_t first = nullptr, last = nullptr;
    ProfScope(gf_ctx* c, hipStream_t st, const char* name);
    ~ProfScope();
};
// The events of the next launch in the innermost scope (false: not profiling).
bool prof_launch_events(hipEvent_t* start, hipEvent_t* stop);

template <typename... KArgs, typename... Args>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, size_t lds, hipStream_t s, Args&&... args) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof_launch_events(&e0, &e1))
        hipExtLaunchKernelGGL(k, grid, block, (std::uint32_t)lds, s, e0, e1, 0, static_cast<KArgs>(args)...);
    else
        k<<<grid, block, lds, s>>>(std::forward<Args>(args)...);
}
}  // namespace gf

#define GF_PROF(ctx, stream, name) ::gf::ProfScope _gf_prof_scope((ctx), (stream), (name))
// kernel<<<grid, block, lds, stream>>>(args...), timed by the innermost GF_PROF scope
#define GF_LAUNCH(kernel, grid, block, lds, stream, ...) ::gf::launch(kernel, grid, block, lds, stream, __VA_ARGS__)

// Device-side helpers ------------------------------------------------------
namespace gfd {

// GF_TRACK_PRIO: issue priority (s_setprio) of the tracking stages' latency
// chains (ordered matcher, pose LM, UpdateReference, one-point precompute)
// while other groups' extraction waves share their SIMDs.
#ifndef GF_TRACK_PRIO
#define GF_TRACK_PRIO 0
#endif
__device__ __forceinline__ void track_prio() {
    if (GF_TRACK_PRIO) __builtin_amdgcn_s_setprio(GF_TRACK_PRIO);
}
// GF_EXT_PRIO: the same for the extraction kernels (the groups' extraction
// stages run one at a time and pace the step; the other groups' tracking
// waves share their SIMDs)
#ifndef GF_EXT_PRIO
#define GF_EXT_PRIO 0
#endif
__device__ __forceinline__ void ext_prio() {
    if (GF_EXT_PRIO) __builtin_amdgcn_s_setprio(GF_EXT_PRIO);
}

// Elapsed ticks at a budget's clock check: the device clock (s_memrealtime,
// 100 MHz) since t0, or with a test clock (syn = the site's base and slope,
// gf_frontend_set_test_clock) base + idx * slope for the idx-th check.
__device__ __forceinline__ long long ck_elapsed(unsigned long long t0, const long long* syn, int idx) {
    return syn ? syn[0] + (long long)idx * syn[1] : (long long)(__builtin_amdgcn_s_memrealtime() - t0);
}

// XCD-aware workgroup order (cdna_hip_programming.md T1, bijective form):
// the dispatcher hands consecutive workgroups to the 8 XCDs in turn, so
// neighbouring tiles — which share halo rows and cache lines — would land in
// 8 different L2s. This maps the 2-D grid's linear id so that each group of
// workgroups sharing an XCD gets one contiguous run of the logical
// (x fastest, then y) order. Speed only: any placement is correct.
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const int nwg = (int)(gridDim.x * gridDim.y), id = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int q = nwg >> 3, r = nwg & 7, x = id & 7, slot = id >> 3;
    const int lid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
    by = lid / (int)gridDim.x;
    bx = lid - by * (int)gridDim.x;
}

// A load through the global address space: global_load_* (counted by vmcnt
// only) where a generic pointer compiles to flat_load_*, which also counts
// against lgkmcnt, so the LDS waits of the kernel wait for it too. For
// device memory only (hipMalloc'd buffers, as all of this library's inputs).
template <typename T>
__device__ __forceinline__ T ldg(const T* p) {
    return *(const __attribute__((address_space(1))) T*)p;
}

__device__ __forceinline__ int reflect101(int p, int len) {
    // BORDER_REFLECT_101 for the <= 18 px excursions the kernels make.
    if (p < 0) p = -p;
    if (p >= len) p = 2 * len - p - 2;
    return p;
}

__device__ __forceinline__ int warp_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace gfd
