// Relocalisation PnP on gfx950 — SURVEY.md §8(f) rank 4: ORB_SLAM::PnPsolver
// (src/PnPsolver.cc) as three kernels per iterate() call of a batch of
// independent solvers:
//   k_pnp_draw  one lane per solver replays the solver's std::rand() stream
//               (DUtils::Random::RandomInt, :163-173, with the reference's
//               write to position idx) and stores every minimal set the call
//               can use — the draws do not depend on the hypotheses, so all of
//               them are known before any pose is computed;
//   k_pnp_hyp   one thread per hypothesis: EPnP on the minimal set
//               (compute_pose :449-497) and CheckInliers (:280-311) over the
//               solver's correspondences -> inlier count, R|t;
//   k_pnp_scan  one workgroup per solver walks the hypotheses in iteration
//               order exactly as iterate() does (:154-211): best-so-far
//               update, Refine() (:232-277) on the best inlier set (EPnP on
//               lane 0, the inlier test across the workgroup), early return,
//               bNoMore; then advances the caller's std::rand() state by the
//               draws of the iterations that ran.
// The OpenCV SVD / solve / invert calls are the scalar restatement documented
// in oracle/pnp.cpp (parity unpinned against OpenCV, bit-exact against the
// oracle). f64 throughout, no contraction (-ffp-contract=off).
#include "pnp_core.h"

namespace {
using namespace gfpnp;

__global__ void k_pnp_draw(int nprob, const gf_pnp_state* __restrict__ states, const gf_rng* __restrict__ rngs,
                           int n_iterations, int lcap, int32_t* __restrict__ draws, int cap) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nprob) return;
    pnp_draw_one(states, rngs, b, n_iterations, lcap, draws, cap);
}

__global__ void __launch_bounds__(64) k_pnp_hyp(const float* __restrict__ p3d, const float* __restrict__ p2d,
                                                const float* __restrict__ sigma2, int cap, Cam cam,
                                                const gf_pnp_state* __restrict__ states, int n_iterations, int lcap,
                                                const int32_t* __restrict__ draws, double* __restrict__ hyp_rt,
                                                int32_t* __restrict__ hyp_cnt) {
    pnp_hyp_one(p3d, p2d, sigma2, cap, cam, states, n_iterations, lcap, draws, hyp_rt, hyp_cnt, blockIdx.y,
                blockIdx.x * blockDim.x + threadIdx.x);
}

__global__ void __launch_bounds__(256) k_pnp_scan(const float* __restrict__ p3d, const float* __restrict__ p2d,
                                                  const float* __restrict__ sigma2, int cap, Cam cam,
                                                  gf_pnp_state* __restrict__ states, uint8_t* __restrict__ best_mask,
                                                  int n_iterations, int lcap, const double* __restrict__ hyp_rt,
                                                  const int32_t* __restrict__ hyp_cnt, double* __restrict__ work,
                                                  gf_rng* __restrict__ rngs, float* __restrict__ Tcw_out,
                                                  uint8_t* __restrict__ inliers, int32_t* __restrict__ ninliers,
                                                  int32_t* __restrict__ flags) {
    pnp_scan_block(p3d, p2d, sigma2, cap, cam, states, best_mask, n_iterations, lcap, hyp_rt, hyp_cnt, work, rngs,
                   Tcw_out, inliers, ninliers, flags, blockIdx.x);
}

}  // namespace

extern "C" {

int gf_pnp_init(int n, const gf_pnp_params* p, gf_pnp_state* st) {
    if (!p || !st || n < 0) return gf::fail(GF_ERR_ARG, "gf_pnp_init: null arg or n < 0");
    if (p->min_set < 1 || p->min_set > kMaxSet) return gf::fail(GF_ERR_UNSUPPORTED, "gf_pnp_init: min_set > 8");
    // SetRansacParameters :93-129 (host scalar set-up)
    *st = gf_pnp_state{};
    st->n = n;
    st->min_set = p->min_set;
    st->th2 = p->th2;
    float eps = p->epsilon;
    int nMinInliers = n * eps;
    if (nMinInliers < p->min_inliers) nMinInliers = p->min_inliers;
    if (nMinInliers < p->min_set) nMinInliers = p->min_set;
    if (n > 0 && eps < (float)nMinInliers / n) eps = (float)nMinInliers / n;
    int nIterations;
    if (nMinInliers == n) {
        nIterations = 1;
    } else {
        const double it = std::ceil(std::log(1 - p->probability) / std::log(1 - std::pow(eps, 3)));
        nIterations = (it == it && it < 2147483647.0) ? (int)it : p->max_iterations;
    }
    st->min_inliers = nMinInliers;
    st->epsilon = eps;
    st->max_iterations = std::max(1, std::min(nIterations, p->max_iterations));
    return GF_OK;
}

int gf_pnp_iterate_dev(gf_ctx* ctx, int nprob, const float* d_p3d, const float* d_p2d, const float* d_sigma2,
                       int cap, const float K[4], gf_pnp_state* d_state, uint8_t* d_best_mask, int n_iterations,
                       int max_iterations, gf_rng* d_rng, float* d_Tcw, uint8_t* d_inliers, int32_t* d_ninliers,
                       int32_t* d_flags, void* stream) {
    GF_CHECK(ctx && K, GF_ERR_ARG, "gf_pnp_iterate_dev: null arg");
    if (nprob <= 0) return GF_OK;
    GF_CHECK(d_p3d && d_p2d && d_sigma2 && d_state && d_best_mask && d_rng && d_Tcw && d_inliers && d_ninliers &&
                 d_flags && cap > 0,
             GF_ERR_ARG, "gf_pnp_iterate_dev: null buffer or cap <= 0");
    const int lcap = std::max(std::max(n_iterations, max_iterations), 1);
    hipStream_t s = (hipStream_t)stream;
    void *draws, *rt, *cnt, *work;
    int rc;
    // device-family scratch slots of their own (45-48): the host wrappers own 0-16
    if ((rc = gf::ws_get(ctx, 45, sizeof(int32_t) * kMaxSet * (size_t)lcap * nprob, &draws)) ||
        (rc = gf::ws_get(ctx, 46, sizeof(double) * 12 * (size_t)lcap * nprob, &rt)) ||
        (rc = gf::ws_get(ctx, 47, sizeof(int32_t) * (size_t)lcap * nprob, &cnt)) ||
        (rc = gf::ws_get(ctx, 48, sizeof(double) * kWork * (size_t)cap * nprob, &work)))
        return rc;
    const Cam cam{(double)K[0], (double)K[1], (double)K[2], (double)K[3]};
    {
        GF_PROF(ctx, s, "k_pnp_draw");
        GF_LAUNCH(k_pnp_draw, (nprob + 63) / 64, 64, 0, s, nprob, d_state, d_rng, n_iterations, lcap, (int32_t*)draws, cap);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_pnp_hyp");
        GF_LAUNCH(k_pnp_hyp, dim3((lcap + 63) / 64, nprob), 64, 0, s, d_p3d, d_p2d, d_sigma2, cap, cam, d_state, n_iterations,
                                                               lcap, (const int32_t*)draws, (double*)rt, (int32_t*)cnt);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_pnp_scan");
        GF_LAUNCH(k_pnp_scan, nprob, 256, 0, s, d_p3d, d_p2d, d_sigma2, cap, cam, d_state, d_best_mask, n_iterations, lcap,
                                         (const double*)rt, (const int32_t*)cnt, (double*)work, d_rng, d_Tcw, d_inliers,
                                         d_ninliers, d_flags);
        GF_HIP(hipGetLastError());
    }
    return GF_OK;
}

int gf_pnp_iterate(gf_ctx* ctx, const float* p3d, const float* p2d, const float* sigma2, const float K[4],
                   gf_pnp_state* state, uint8_t* best_mask, int n_iterations, gf_rng* rng, float Tcw[16],
                   uint8_t* inliers, int32_t* ninliers, int32_t* flags) {
    GF_CHECK(ctx && K && state && rng && Tcw && ninliers && flags, GF_ERR_ARG, "gf_pnp_iterate: null arg");
    const int n = state->n;
    GF_CHECK(n == 0 || (p3d && p2d && sigma2 && best_mask && inliers), GF_ERR_ARG, "gf_pnp_iterate: null buffer");
    GF_CHECK(state->min_set >= 1 && state->min_set <= kMaxSet, GF_ERR_ARG, "gf_pnp_iterate: state not initialised");
    GF_HIP(hipSetDevice(ctx->device));
    const int cap = std::max(n, 1);
    void *d3, *d2, *ds, *dst, *dbm, *drng, *dT, *dinl, *dn, *dfl;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, p3d, sizeof(float) * 3 * (size_t)n, &d3)) ||
        (rc = gf::ws_upload(ctx, 1, p2d, sizeof(float) * 2 * (size_t)n, &d2)) ||
        (rc = gf::ws_upload(ctx, 2, sigma2, sizeof(float) * (size_t)n, &ds)) ||
        (rc = gf::ws_upload(ctx, 3, state, sizeof(gf_pnp_state), &dst)) ||
        (rc = gf::ws_upload(ctx, 4, best_mask, (size_t)n, &dbm)) ||
        (rc = gf::ws_upload(ctx, 5, rng, sizeof(gf_rng), &drng)) || (rc = gf::ws_get(ctx, 6, sizeof(float) * 16, &dT)) ||
        (rc = gf::ws_get(ctx, 7, (size_t)cap, &dinl)) || (rc = gf::ws_get(ctx, 8, sizeof(int32_t), &dn)) ||
        (rc = gf::ws_get(ctx, 9, sizeof(int32_t), &dfl)))
        return rc;
    // the draw/hypothesis bound: this call's loop count
    const int L = std::max(n_iterations, state->max_iterations - state->iterations);
    rc = gf_pnp_iterate_dev(ctx, 1, (const float*)d3, (const float*)d2, (const float*)ds, cap, K,
                            (gf_pnp_state*)dst, (uint8_t*)dbm, n_iterations, std::max(L, 1), (gf_rng*)drng,
                            (float*)dT, (uint8_t*)dinl, (int32_t*)dn, (int32_t*)dfl, ctx->stream);
    if (rc) return rc;
    hipStream_t s = ctx->stream;
    GF_HIP(hipMemcpyAsync(state, dst, sizeof(gf_pnp_state), hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(rng, drng, sizeof(gf_rng), hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(Tcw, dT, sizeof(float) * 16, hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(ninliers, dn, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(flags, dfl, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    if (n) {
        GF_HIP(hipMemcpyAsync(best_mask, dbm, (size_t)n, hipMemcpyDeviceToHost, s));
        GF_HIP(hipMemcpyAsync(inliers, dinl, (size_t)n, hipMemcpyDeviceToHost, s));
    }
    GF_HIP(hipStreamSynchronize(s));
    return GF_OK;
}

}  // extern "C"
