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

/* ------------------------------------------------------- ORB extraction (E1-E8)
 * Replaces ORB_SLAM::ORBextractor (include/ORBextractor.h:57-70,
 * src/ORBextractor.cc:464-998): ctor(nfeatures, scaleFactor, nlevels,
 * scoreType, fastTh) and operator()(image, mask=empty, keypoints, descriptors).
 * The geometry (width x height) is fixed at creation: the pyramid, cell grids
 * and per-level quotas are planned once. score_type must be FAST_SCORE (1);
 * HARRIS_SCORE (0) returns GF_ERR_UNSUPPORTED. max_batch bounds nframes of the
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

/* Debug/parity hook: copies one intermediate plane of frame f of the last
 * batch to host. which: 0 = pyramid level (unblurred, ComputePyramid
 * ORBextractor.cc:922-998), 1 = blurred level interior (GaussianBlur :842).
 * out must hold w*h bytes of that level; (w,h) returned. */
int gf_extractor_debug_level(gf_extractor* ex, int frame, int level, int which, uint8_t* out,
                             int* w, int* h);

#ifdef __cplusplus
}
#endif
#endif /* GFSLAM_ABI_H */
