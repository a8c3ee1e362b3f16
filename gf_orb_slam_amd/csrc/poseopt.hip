// Motion-only pose optimisation on gfx950.
//
// One wave (PO_T threads) per problem (frame). Per-edge work — projection,
// error, Huber weight, the 2x6 pose Jacobian and its 27 contributions to the
// lower triangle of H and to b — runs one edge per thread, PO_E edges per
// pass; the reductions over edges keep the reference's order: thread k owns
// accumulator k (21 lower H entries, 6 b entries, robust chi2) and adds the
// per-edge terms staged in LDS in edge order, exactly as g2o's sequential
// loop over _activeEdges (sparse_optimizer.cpp:100-114,
// block_solver.hpp:502-562). The scalar LM logic (lambda schedule, LDLT, exp
// update, stop rules) runs redundantly on every thread from the shared sums,
// so no broadcast is needed. The problem is latency-bound (an ordered
// double-precision sum chain per LM pass), so the footprint, not the lane
// count, sets the throughput: small enough to share CUs with the other
// stream groups' kernels.
//
// Reference: Optimizer::PoseOptimization src/Optimizer.cc:279-413,
// OptimizationAlgorithmLevenberg::solve core/optimization_algorithm_levenberg.cpp:61-189,
// EdgeSE3ProjectXYZ types/sba/types_six_dof_expmap.cpp:384-428,
// BaseBinaryEdge::constructQuadraticForm core/base_binary_edge.hpp:55-122.
#include "poseopt_core.h"

namespace {
using namespace gfpose;

// WPS waves per SIMD: 2 fits two problems per CU (256 registers a lane, some
// spilled) for large batches; 1 keeps every value in registers for the
// single-problem latency path.
template <int WPS>
__global__ __launch_bounds__(PO_T, WPS) void k_pose_opt(PoseArgs A) {
    pose_opt_problem(A, blockIdx.x);
}

struct GatherArgs {
    const gf_keypoint* kps;
    const int32_t* nkps;
    int kp_stride;
    const int32_t* kp2mp;
    const gf_map_point* map;
    int map_stride;
    float inv_sigma2[16];
    int nlevels;
    gf_pose_edge* edges;
    int32_t* edge_kp;
    int32_t* nedges;
    // optional gate: frame f is not optimised at all (nedges = 0, the
    // optimisation skipped) when gate[f] < gate_min
    const int32_t* gate;
    int gate_min;
};

#ifndef GATHER_U
#define GATHER_U 4
#endif
// Ordered compaction of the matched keypoints of frame f (one wave).
__device__ __forceinline__ void gather_frame(const GatherArgs& G, int f) {
    const int l = threadIdx.x;
    if (G.gate && G.gate[f] < G.gate_min) {
        if (l == 0) G.nedges[f] = 0;
        return;
    }
    const int n = G.nkps[f];
    const size_t kb = (size_t)f * G.kp_stride;
    int cnt = 0;
    // GATHER_U rows of 64 keypoints a pass: their loads (clamped,
    // unconditional) issue together, then the compaction and the stores
    for (int base = 0; base < n; base += 64 * GATHER_U) {
        int mp[GATHER_U];
        float kx[GATHER_U], ky[GATHER_U];
        int ko[GATHER_U];
        float X[GATHER_U][3];
#pragma unroll
        for (int u = 0; u < GATHER_U; u++) {
            const size_t i = kb + min(base + 64 * u + l, n - 1);
            mp[u] = G.kp2mp[i];
            kx[u] = G.kps[i].x;
            ky[u] = G.kps[i].y;
            ko[u] = G.kps[i].octave;
        }
#pragma unroll
        for (int u = 0; u < GATHER_U; u++) {
            const gf_map_point& P = G.map[(size_t)f * G.map_stride + max(mp[u], 0)];
            X[u][0] = P.pos[0];
            X[u][1] = P.pos[1];
            X[u][2] = P.pos[2];
        }
#pragma unroll
        for (int u = 0; u < GATHER_U; u++) {
            const int i = base + 64 * u + l;
            const bool on = i < n && mp[u] >= 0;
            const unsigned long long m = __ballot(on);
            const int pos = cnt + __popcll(m & ((1ull << l) - 1ull));
            if (on) {
                gf_pose_edge e;
                e.X[0] = X[u][0];
                e.X[1] = X[u][1];
                e.X[2] = X[u][2];
                e.z[0] = kx[u];
                e.z[1] = ky[u];
                const int oc = min(max(ko[u], 0), G.nlevels - 1);
                e.inv_sigma2 = G.inv_sigma2[oc];
                G.edges[kb + pos] = e;
                G.edge_kp[kb + pos] = i;
            }
            cnt += __popcll(m);
        }
    }
    if (l == 0) G.nedges[f] = cnt;
}

// One wave per frame: its edges in keypoint order, then PoseOptimization on
// them (the gather and the LM in one launch: no launch gap between them on a
// single sequence's chain).
template <int WPS, int NT>
__global__ __launch_bounds__(NT, WPS) void k_pose_opt_frames(GatherArgs G, PoseArgs A) {
    gfd::track_prio();
    if (threadIdx.x < 64) gather_frame(G, blockIdx.x);
    __syncthreads();  // the edges (global memory) visible to the whole workgroup
    pose_opt_problem<NT>(A, blockIdx.x);
}

// Batches up to this size run a problem per 256-thread workgroup (the LM
// trials' edge passes on four waves): the single-sequence chain is one
// wave's instruction stream, and with few problems the CUs are free.
#ifndef PO_WIDE_MAX
#define PO_WIDE_MAX 64
#endif

int launch_pose(gf_ctx* ctx, int nprob, const PoseArgs& A, hipStream_t s) {
    GF_PROF(ctx, s, "k_pose_opt");
    // the spill-free build (256 registers a lane: one wave per SIMD, four
    // problems per CU); PO_WPS=2 selects the two-per-SIMD build, which spills
#ifndef PO_WPS
#define PO_WPS 1
#endif
    (void)ctx;
    GF_LAUNCH(k_pose_opt<PO_WPS>, nprob, PO_T, 0, s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

}  // namespace

extern "C" {

int gf_pose_opt_batch_dev(gf_ctx* ctx, int nprob, float* d_Tcw, const gf_pose_edge* d_edges, const int32_t* d_nedges,
                          int edge_stride, float fx, float fy, float cx, float cy, uint8_t* d_outlier,
                          int32_t* d_ninliers, int32_t* d_iterations, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nprob <= 0) return GF_OK;
    GF_CHECK(d_Tcw && d_edges && d_nedges && d_outlier && d_ninliers, GF_ERR_ARG, "null arg");
    GF_CHECK(edge_stride > 0 && edge_stride <= PO_STRIDE_MAX, GF_ERR_UNSUPPORTED, "edge_stride out of range");
    void* work;
    int rc = gf::ws_get(ctx, 40, (size_t)nprob * edge_stride * 3 * sizeof(double), &work);
    if (rc) return rc;
    PoseArgs A{};
    A.edges = d_edges;
    A.nedges = d_nedges;
    A.stride = edge_stride;
    A.Tcw = d_Tcw;
    A.outl = d_outlier;
    A.ninl = d_ninliers;
    A.iters = d_iterations;
    A.work = (double*)work;
    A.fx = fx;
    A.fy = fy;
    A.cx = cx;
    A.cy = cy;
    return launch_pose(ctx, nprob, A, (hipStream_t)stream);
}

int gf_pose_opt_frames_dev(gf_ctx* ctx, int nframes, float* d_Tcw, const gf_keypoint* d_kps, const int32_t* d_nkps,
                           int kp_stride, const int32_t* d_kp2mp, const gf_map_point* d_map, int map_stride,
                           const float* inv_sigma2, int nlevels, float fx, float fy, float cx, float cy,
                           uint8_t* d_outlier, int32_t* d_ninliers, int32_t* d_iterations, int32_t* d_nedges,
                           void* stream) {
    return gf::pose_opt_frames_gated(ctx, nframes, d_Tcw, d_kps, d_nkps, kp_stride, d_kp2mp, d_map, map_stride,
                                     inv_sigma2, nlevels, fx, fy, cx, cy, d_outlier, d_ninliers, d_iterations,
                                     d_nedges, nullptr, 0, stream);
}

}  // extern "C"

int gf::pose_opt_frames_gated(gf_ctx* ctx, int nframes, float* d_Tcw, const gf_keypoint* d_kps,
                              const int32_t* d_nkps, int kp_stride, const int32_t* d_kp2mp, const gf_map_point* d_map,
                              int map_stride, const float* inv_sigma2, int nlevels, float fx, float fy, float cx,
                              float cy, uint8_t* d_outlier, int32_t* d_ninliers, int32_t* d_iterations,
                              int32_t* d_nedges, const int32_t* d_gate, int gate_min, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nframes <= 0) return GF_OK;
    GF_CHECK(d_Tcw && d_kps && d_nkps && d_kp2mp && d_map && inv_sigma2 && d_outlier && d_ninliers, GF_ERR_ARG,
             "null arg");
    GF_CHECK(kp_stride > 0 && kp_stride <= PO_STRIDE_MAX, GF_ERR_UNSUPPORTED, "kp_stride out of range");
    GF_CHECK(nlevels >= 1 && nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    hipStream_t s = (hipStream_t)stream;
    void *edges, *ekp, *ne = d_nedges, *eout, *work;
    int rc;
    const size_t ne_tot = (size_t)nframes * kp_stride;
    if ((rc = gf::ws_get(ctx, 41, ne_tot * sizeof(gf_pose_edge), &edges)) ||
        (rc = gf::ws_get(ctx, 42, ne_tot * sizeof(int32_t), &ekp)) ||
        (!d_nedges && (rc = gf::ws_get(ctx, 43, (size_t)nframes * sizeof(int32_t), &ne))) ||
        (rc = gf::ws_get(ctx, 44, ne_tot, &eout)) ||
        (rc = gf::ws_get(ctx, 40, ne_tot * 3 * sizeof(double), &work)))
        return rc;
    GatherArgs G{};
    G.kps = d_kps;
    G.nkps = d_nkps;
    G.kp_stride = kp_stride;
    G.kp2mp = d_kp2mp;
    G.map = d_map;
    G.map_stride = map_stride;
    for (int i = 0; i < nlevels; i++) G.inv_sigma2[i] = inv_sigma2[i];
    G.nlevels = nlevels;
    G.gate = d_gate;
    G.gate_min = gate_min;
    G.edges = (gf_pose_edge*)edges;
    G.edge_kp = (int32_t*)ekp;
    G.nedges = (int32_t*)ne;
    PoseArgs A{};
    A.edges = G.edges;
    A.nedges = G.nedges;
    A.stride = kp_stride;
    A.Tcw = d_Tcw;
    A.outl = (uint8_t*)eout;
    A.ninl = d_ninliers;
    A.iters = d_iterations;
    A.work = (double*)work;
    A.fx = fx;
    A.fy = fy;
    A.cx = cx;
    A.cy = cy;
    A.edge_kp = G.edge_kp;
    A.kp_outl = d_outlier;
    A.kp_stride = kp_stride;
    A.gate = d_gate;
    A.gate_min = gate_min;
    GF_PROF(ctx, s, "k_pose_opt");
    if (nframes <= PO_WIDE_MAX)
        GF_LAUNCH((k_pose_opt_frames<1, 256>), nframes, 256, 0, s, G, A);
    else
        GF_LAUNCH((k_pose_opt_frames<PO_WPS, PO_T>), nframes, PO_T, 0, s, G, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

extern "C" {

int gf_pose_opt(gf_ctx* ctx, const float* Tcw_in, const gf_pose_edge* edges, int n, float fx, float fy, float cx,
                float cy, float* Tcw_out, uint8_t* outlier, int32_t* ninliers, int32_t* iterations) {
    GF_CHECK(ctx && Tcw_in && Tcw_out && ninliers, GF_ERR_ARG, "null arg");
    GF_CHECK(n >= 0 && (n == 0 || (edges && outlier)), GF_ERR_ARG, "bad edge list");
    GF_CHECK(n <= PO_STRIDE_MAX, GF_ERR_UNSUPPORTED, "too many edges");
    GF_HIP(hipSetDevice(ctx->device));
    const int stride = n > 0 ? n : 1;
    void *dT, *dE, *dN, *dO, *dI, *dIt;
    int rc;
    const int32_t nn = n;
    if ((rc = gf::ws_upload(ctx, 0, Tcw_in, 64, &dT)) || (rc = gf::ws_get(ctx, 1, sizeof(gf_pose_edge) * stride, &dE)) ||
        (rc = gf::ws_upload(ctx, 2, &nn, 4, &dN)) || (rc = gf::ws_get(ctx, 3, stride, &dO)) ||
        (rc = gf::ws_get(ctx, 4, 4, &dI)) || (rc = gf::ws_get(ctx, 5, 4, &dIt)))
        return rc;
    if (n > 0) GF_HIP(hipMemcpyAsync(dE, edges, sizeof(gf_pose_edge) * n, hipMemcpyHostToDevice, ctx->stream));
    rc = gf_pose_opt_batch_dev(ctx, 1, (float*)dT, (const gf_pose_edge*)dE, (const int32_t*)dN, stride, fx, fy, cx, cy,
                               (uint8_t*)dO, (int32_t*)dI, (int32_t*)dIt, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(Tcw_out, dT, 64, hipMemcpyDeviceToHost, ctx->stream));
    if (n > 0) GF_HIP(hipMemcpyAsync(outlier, dO, n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(ninliers, dI, 4, hipMemcpyDeviceToHost, ctx->stream));
    int32_t it = 0;
    GF_HIP(hipMemcpyAsync(&it, dIt, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    if (iterations) *iterations = it;
    return GF_OK;
}

}  // extern "C"
