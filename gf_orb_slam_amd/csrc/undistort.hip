// Keypoint undistortion on gfx950 — SURVEY.md §8(f) rank 2:
// Frame::UndistortKeyPoints (src/Frame.cc:389-423) calls
// cv::undistortPoints(pts, pts, mK, mDistCoef, Mat(), mK); with k1 == 0 the
// keypoints are copied (:391-395). OpenCV 3.4's cvUndistortPointsInternal
// (modules/imgproc/src/undistort.cpp) with the default criteria
// TermCriteria(COUNT, 5, 0.01): 5 fixed-point iterations in double on the
// normalised point, 4 or 5 coefficients (k1 k2 p1 p2 [k3]) and no tilt, then
// the projection through P = K (RR = K * I). One thread per keypoint; all of
// it f64 in OpenCV's expression order (compiled without contraction).
#include "common.h"

#include "undist.h"

namespace {

using gfu::UndistCoef;
using gfu::make_coef;
using gfu::undistort_point;

__global__ void k_undistort(UndistCoef c, int copy_only, const gf_keypoint* __restrict__ in, const int32_t* __restrict__ n,
                            int cap, gf_keypoint* __restrict__ out) {
    const int f = blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= min(n[f], cap)) return;
    gf_keypoint kp = in[(long long)f * cap + i];
    if (!copy_only) undistort_point(c, kp.x, kp.y, kp.x, kp.y);
    out[(long long)f * cap + i] = kp;
}

}  // namespace

extern "C" {

int gf_undistort_keypoints_dev(gf_ctx* ctx, int nframes, const float K[4], const float dist[5],
                               const gf_keypoint* d_in, const int32_t* d_n, int cap, gf_keypoint* d_out, void* stream) {
    GF_CHECK(ctx && K && dist, GF_ERR_ARG, "null arg");
    GF_CHECK(K[0] != 0.f && K[1] != 0.f, GF_ERR_ARG, "zero focal length");
    if (nframes <= 0 || cap <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_undistort");
    GF_LAUNCH(k_undistort, dim3((cap + 255) / 256, nframes), 256, 0, s, make_coef(K, dist), dist[0] == 0.f ? 1 : 0, d_in,
                                                                 d_n, cap, d_out);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_undistort_keypoints(gf_ctx* ctx, const float K[4], const float dist[5], const gf_keypoint* kps, int n,
                           gf_keypoint* out) {
    GF_CHECK(ctx && K && dist, GF_ERR_ARG, "null arg");
    if (n <= 0) return GF_OK;
    GF_CHECK(kps && out, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *din, *dn, *dout;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, kps, sizeof(gf_keypoint) * (size_t)n, &din)) ||
        (rc = gf::ws_upload(ctx, 1, &n, sizeof(int32_t), &dn)) ||
        (rc = gf::ws_get(ctx, 2, sizeof(gf_keypoint) * (size_t)n, &dout)))
        return rc;
    rc = gf_undistort_keypoints_dev(ctx, 1, K, dist, (const gf_keypoint*)din, (const int32_t*)dn, n,
                                    (gf_keypoint*)dout, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(out, dout, sizeof(gf_keypoint) * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

}  // extern "C"
