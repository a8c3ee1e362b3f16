// Local-mapping Hamming kernels on gfx950 — SURVEY.md §8(f) rank 3:
//
//   MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:197-262): of the
//     N descriptors observing a map point, the one whose median Hamming
//     distance to the others (sorted row, element (int)(0.5 (N-1))) is least,
//     first index on ties. One thread per row: the row's k-th smallest
//     distance by a 9-step binary search on the value (distances are
//     0..256), the point's minimum of (median << 16 | row) by atomicMin.
//
//   ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>&, th) (src/ORBmatcher.cc:
//     1590-1707): project every candidate map point into the keyframe, keep
//     the closest keypoint of the predicted level band [l-1, l] in the radius
//     th * scale[l] (first in grid order on ties), fuse when <= TH_LOW. The
//     searches are independent; the sequential part of the reference loop is
//     only what happens at the chosen slot — an occupied slot makes the
//     candidate Replace() into its occupant, an empty slot is taken by the
//     first candidate that chose it and every later one Replace()s into that
//     first one. A per-slot atomicMin over candidate order reproduces it.
//     One 1024-thread workgroup per (keyframe, candidate list) problem; the
//     64x48 keypoint grid (KeyFrame's copy of Frame.cc:100-131) lives in LDS.
#include <climits>
#include <vector>

#include "common.h"
#include "match_common.h"

#define DD_REG 32  // rows whose distances stay in registers
#define TH_LOW 50

namespace {

// ------------------------------------------------------------ distinctive descriptors

__device__ __forceinline__ int ham(const uint4 a0, const uint4 a1, const uint4* q) {
    const uint4 b0 = q[0], b1 = q[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// One thread per observation row (the map has ~10-30 rows per point, so a
// wave per point would idle most lanes): the row's point by upper_bound over
// the offsets, its N distances kept in registers when N <= DD_REG, the k-th
// smallest by a 9-step binary search on the value, and the point's argmin as
// an atomicMin of (median << 16 | row) on the output word (pre-set to ~0).
__global__ __launch_bounds__(256) void k_distinctive_rows(const uint8_t* __restrict__ desc,
                                                         const int32_t* __restrict__ offs, int nmp, int total,
                                                         uint32_t* __restrict__ key) {
    const int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= total) return;
    int lo = 0, hi = nmp;  // first p with offs[p + 1] > r
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (offs[mid + 1] <= r) lo = mid + 1;
        else hi = mid;
    }
    const int p = lo, o = offs[p], N = offs[p + 1] - o, i = r - o;
    const uint4* rows = (const uint4*)(desc + (size_t)o * 32);
    const uint4 a0 = rows[2 * i], a1 = rows[2 * i + 1];
    const int k = (N - 1) >> 1;  // (int)(0.5 * (N - 1)) for N >= 1 (MapPoint.cc:249)
    int med;
    if (N <= DD_REG) {
        int d[DD_REG];
#pragma unroll
        for (int j = 0; j < DD_REG; j++) d[j] = j < N ? ham(a0, a1, rows + 2 * j) : 1024;
        int l = 0, h = 256;  // smallest v with #{j : d_j <= v} > k; d_ii = 0 is in the row (:233)
        while (l < h) {
            const int mid = (l + h) >> 1;
            int c = 0;
#pragma unroll
            for (int j = 0; j < DD_REG; j++) c += d[j] <= mid;
            if (c > k) h = mid;
            else l = mid + 1;
        }
        med = l;
    } else {
        int l = 0, h = 256;
        while (l < h) {
            const int mid = (l + h) >> 1;
            int c = 0;
            for (int j = 0; j < N; j++) c += ham(a0, a1, rows + 2 * j) <= mid;
            if (c > k) h = mid;
            else l = mid + 1;
        }
        med = l;
    }
    atomicMin(&key[p], ((uint32_t)med << 16) | (uint32_t)i);
}

__global__ __launch_bounds__(256) void k_distinctive_pick(const uint8_t* __restrict__ desc,
                                                         const int32_t* __restrict__ offs, int nmp,
                                                         int32_t* __restrict__ best, uint8_t* __restrict__ out_desc) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int p = t >> 1;  // two lanes per point: one 16-byte half of the descriptor each
    if (p >= nmp) return;
    const uint32_t key = (uint32_t)best[p];
    const int bi = key == 0xffffffffu ? -1 : (int)(key & 0xffffu);  // no observations: left as it was (:211, :224)
    if ((t & 1) == 0) best[p] = bi;
    if (out_desc && bi >= 0)
        ((uint4*)(out_desc + (size_t)p * 32))[t & 1] = ((const uint4*)(desc + (size_t)(offs[p] + bi) * 32))[t & 1];
}

// ------------------------------------------------------------------------ Fuse

struct FuseProb {
    float T[12];  // Rcw | tcw, row-major 3x4
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
};

__global__ __launch_bounds__(MATCH_THREADS) void k_fuse(FrameConst fc, const FuseProb* __restrict__ probs) {
    extern __shared__ int lds[];
    const FuseProb& P = probs[blockIdx.x];
    const int n = P.n, tid = threadIdx.x;
    int* cell_start = lds;                 // NCELLS + 1
    int* items = cell_start + NCELLS + 1;  // n
    int* slot = items + n;                 // n: KF map point, then the first adder of an empty slot
    int* scratch = slot + n;               // n
    __shared__ int s_nf;
    if (tid == 0) s_nf = 0;
    build_grid(fc, P.kps, n, P.kf_mp, cell_start, items, slot, scratch, MATCH_THREADS);
    // slot[k] = the first candidate (list order) that chose the empty slot k; INT_MAX = none
    for (int i = tid; i < n; i += MATCH_THREADS) slot[i] = INT_MAX;
    __syncthreads();
    const int nmax = fc.nlevels - 1;
    int nf = 0;
    // pass 1: independent searches (ORBmatcher.cc:1608-1683)
    for (int i = tid; i < P.m; i += MATCH_THREADS) {
        int bestIdx = -1, bestDist = INT_MAX;
        do {
            if (P.mp_skip && P.mp_skip[i]) break;  // NULL, isBad() or IsInKeyFrame(pKF) (:1612-1616)
            const gf_map_point mp = P.mps[i];
            float Pc[3];
            transform3(P.T, mp.pos, Pc);
            if (Pc[2] < 0.0f) break;
            const float invz = 1.f / Pc[2];
            const float x = Pc[0] * invz, y = Pc[1] * invz;
            const float u = fc.fx * x + fc.cx, v = fc.fy * y + fc.cy;
            // KeyFrame::IsInImage (KeyFrame.cc:654-657)
            if (!(u >= (float)fc.min_x && u < (float)fc.max_x && v >= (float)fc.min_y && v < (float)fc.max_y)) break;
            const float PO[3] = {mp.pos[0] - P.Ow[0], mp.pos[1] - P.Ow[1], mp.pos[2] - P.Ow[2]};
            // cv::norm / Mat::dot accumulate in double
            const float dist3D =
                (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
            if (dist3D < mp.min_dist || dist3D > mp.max_dist) break;
            const double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
            if (dot < 0.5 * (double)dist3D) break;
            const float ratio = dist3D / mp.min_dist;
            int lvl = 0;
            while (lvl < fc.nlevels && fc.scales[lvl] < ratio) lvl++;  // lower_bound
            lvl = min(lvl, nmax);
            const float r = P.th * fc.scales[lvl];
            int cx0, cx1, cy0, cy1;
            if (!grid_window(fc, u, v, r, cx0, cx1, cy0, cy1)) break;
            const uint4* dq = (const uint4*)(P.mp_desc + (size_t)i * 32);
            const uint4 a0 = dq[0], a1 = dq[1];
            for (int cx = cx0; cx <= cx1; cx++)
                for (int cy = cy0; cy <= cy1; cy++) {
                    const int c = cx * GRID_ROWS + cy;
                    for (int a = cell_start[c], e = cell_start[c + 1]; a < e; a++) {
                        const int idx = items[a];
                        const gf_keypoint kp = P.kps[idx];
                        if (fabsf(kp.x - u) > r || fabsf(kp.y - v) > r) continue;
                        if (kp.octave < lvl - 1 || kp.octave > lvl) continue;
                        const int d = ham(a0, a1, (const uint4*)(P.desc + (size_t)idx * 32));
                        if (d < bestDist) {
                            bestDist = d;
                            bestIdx = idx;
                        }
                    }
                }
        } while (false);
        const bool fused = bestDist <= TH_LOW;
        if (fused) {
            nf++;
            if (P.kf_mp[bestIdx] < 0) atomicMin(&slot[bestIdx], i);
        }
        P.res[i] = gf_fuse_result{fused ? bestIdx : -1, GF_FUSE_NONE, -1};
    }
    atomicAdd(&s_nf, nf);
    __syncthreads();
    // pass 2: the action at the chosen slot (:1686-1700)
    for (int i = tid; i < P.m; i += MATCH_THREADS) {
        gf_fuse_result rr = P.res[i];
        if (rr.kp < 0) continue;
        const int occ = P.kf_mp[rr.kp];
        if (occ >= 0) {
            if (P.kf_mp_bad && P.kf_mp_bad[rr.kp]) rr.action = GF_FUSE_KEEP;
            else {
                rr.action = GF_FUSE_REPLACE;
                rr.target = occ;
            }
        } else {
            const int first = slot[rr.kp];
            if (first == i) rr.action = GF_FUSE_ADD;
            else {
                rr.action = GF_FUSE_REPLACE;
                rr.target = P.mp_ids ? P.mp_ids[first] : first;
            }
        }
        P.res[i] = rr;
    }
    if (tid == 0) *P.nfused = s_nf;
}

size_t fuse_lds_bytes(int n) { return sizeof(int) * ((size_t)NCELLS + 1 + 3 * (size_t)n); }

}  // namespace

extern "C" {

int gf_distinctive_descriptors_dev(gf_ctx* ctx, int nmp, const uint8_t* d_desc, const int32_t* d_offsets,
                                   int32_t* d_best, uint8_t* d_out_desc, int total, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (nmp <= 0) return GF_OK;
    GF_CHECK(d_offsets && d_best && total >= 0 && (total == 0 || d_desc), GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    GF_HIP(hipMemsetAsync(d_best, 0xff, 4 * (size_t)nmp, s));
    if (total > 0) {
        GF_PROF(ctx, s, "k_distinctive_rows");
        GF_LAUNCH(k_distinctive_rows, (total + 255) / 256, 256, 0, s, d_desc, d_offsets, nmp, total, (uint32_t*)d_best);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(ctx, s, "k_distinctive_pick");
        GF_LAUNCH(k_distinctive_pick, (2 * nmp + 255) / 256, 256, 0, s, d_desc, d_offsets, nmp, d_best, d_out_desc);
        GF_HIP(hipGetLastError());
    }
    return GF_OK;
}

int gf_distinctive_descriptors(gf_ctx* ctx, int nmp, const uint8_t* desc, const int32_t* offsets, int32_t* best,
                               uint8_t* out_desc) {
    GF_CHECK(ctx && (nmp <= 0 || (offsets && best)), GF_ERR_ARG, "null arg");
    if (nmp <= 0) return GF_OK;
    GF_CHECK(offsets[0] == 0, GF_ERR_ARG, "offsets[0] must be 0");
    for (int p = 0; p < nmp; p++) {
        GF_CHECK(offsets[p + 1] >= offsets[p], GF_ERR_ARG, "offsets must be non-decreasing");
        GF_CHECK(offsets[p + 1] - offsets[p] <= 65535, GF_ERR_UNSUPPORTED, "at most 65535 observations per point");
    }
    const int total = offsets[nmp];
    GF_CHECK(total == 0 || desc, GF_ERR_ARG, "null descriptors");
    GF_HIP(hipSetDevice(ctx->device));
    void *dd = nullptr, *doff, *dbest, *dout = nullptr;
    int rc;
    if ((total && (rc = gf::ws_upload(ctx, 54, desc, 32 * (size_t)total, &dd))) ||
        (rc = gf::ws_upload(ctx, 55, offsets, 4 * (size_t)(nmp + 1), &doff)) ||
        (rc = gf::ws_get(ctx, 56, 4 * (size_t)nmp, &dbest)) ||
        (out_desc && (rc = gf::ws_upload(ctx, 57, out_desc, 32 * (size_t)nmp, &dout))))
        return rc;
    rc = gf_distinctive_descriptors_dev(ctx, nmp, (const uint8_t*)dd, (const int32_t*)doff, (int32_t*)dbest,
                                        (uint8_t*)dout, total, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(best, dbest, 4 * (size_t)nmp, hipMemcpyDeviceToHost, ctx->stream));
    if (out_desc) GF_HIP(hipMemcpyAsync(out_desc, dout, 32 * (size_t)nmp, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_fuse_dev(gf_ctx* ctx, const gf_frame_info* fi, int nprob, const gf_fuse_problem* probs, void* stream) {
    GF_CHECK(ctx && fi, GF_ERR_ARG, "null arg");
    if (nprob <= 0) return GF_OK;
    GF_CHECK(probs, GF_ERR_ARG, "null problems");
    GF_CHECK(fi->nlevels >= 1 && fi->nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    GF_CHECK(fi->max_x > fi->min_x && fi->max_y > fi->min_y, GF_ERR_ARG, "empty image bounds");
    std::vector<FuseProb> P(nprob);
    int nmax = 0;
    for (int p = 0; p < nprob; p++) {
        const gf_fuse_problem& q = probs[p];
        GF_CHECK(q.n >= 0 && q.n <= KP_MAX, GF_ERR_UNSUPPORTED, "at most 4096 keyframe keypoints");
        GF_CHECK(q.m >= 0 && q.nfused && (q.m == 0 || (q.mps && q.mp_desc && q.res)) &&
                     (q.n == 0 || (q.kps && q.desc && q.kf_mp)),
                 GF_ERR_ARG, "null problem field");
        for (int k = 0; k < 12; k++) P[p].T[k] = q.Tcw[k];
        for (int k = 0; k < 3; k++) P[p].Ow[k] = q.Ow[k];
        P[p].kps = q.kps;
        P[p].desc = q.desc;
        P[p].n = q.n;
        P[p].kf_mp = q.kf_mp;
        P[p].kf_mp_bad = q.kf_mp_bad;
        P[p].mps = q.mps;
        P[p].mp_desc = q.mp_desc;
        P[p].mp_skip = q.mp_skip;
        P[p].mp_ids = q.mp_ids;
        P[p].m = q.m;
        P[p].th = q.th;
        P[p].res = q.res;
        P[p].nfused = q.nfused;
        nmax = std::max(nmax, q.n);
    }
    hipStream_t s = (hipStream_t)stream;
    void* dp;
    int rc = gf::ws_get(ctx, 58, sizeof(FuseProb) * nprob, &dp);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(dp, P.data(), sizeof(FuseProb) * nprob, hipMemcpyHostToDevice, s));
    GF_PROF(ctx, s, "k_fuse");
    GF_LAUNCH(k_fuse, nprob, MATCH_THREADS, fuse_lds_bytes(nmax), s, gf::make_frame_const(fi), (const FuseProb*)dp);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_fuse(gf_ctx* ctx, const gf_frame_info* fi, const float* Tcw, const float* Ow, const gf_keypoint* kps,
            const uint8_t* desc, int n, const int32_t* kf_mp, const uint8_t* kf_mp_bad, const gf_map_point* mps,
            const uint8_t* mp_desc, const uint8_t* mp_skip, const int32_t* mp_ids, int m, float th,
            gf_fuse_result* res, int* nfused) {
    GF_CHECK(ctx && fi && Tcw && Ow && nfused, GF_ERR_ARG, "null arg");
    GF_CHECK(n >= 0 && n <= KP_MAX, GF_ERR_UNSUPPORTED, "at most 4096 keyframe keypoints");
    *nfused = 0;
    if (m <= 0) return GF_OK;
    GF_CHECK(mps && mp_desc && res && (n == 0 || (kps && desc && kf_mp)), GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    // one scratch block: [kps | desc | kf_mp | bad | mps | mp_desc | skip | ids | res | nfused]
    size_t off = 0;
    std::vector<std::pair<const void*, size_t>> parts;
    auto add = [&](const void* h, size_t bytes) {
        const size_t o = off;
        parts.push_back({h, bytes});
        off += (bytes + 15) & ~(size_t)15;
        return o;
    };
    const size_t o_k = add(kps, sizeof(gf_keypoint) * (size_t)n), o_d = add(desc, 32 * (size_t)n),
                 o_mp = add(kf_mp, 4 * (size_t)n), o_bad = add(kf_mp_bad, kf_mp_bad ? (size_t)n : 0),
                 o_m = add(mps, sizeof(gf_map_point) * (size_t)m), o_md = add(mp_desc, 32 * (size_t)m),
                 o_sk = add(mp_skip, mp_skip ? (size_t)m : 0), o_id = add(mp_ids, mp_ids ? 4 * (size_t)m : 0),
                 o_r = add(nullptr, sizeof(gf_fuse_result) * (size_t)m), o_nf = add(nullptr, 4);
    void* dbuf;
    int rc = gf::ws_get(ctx, 59, off, &dbuf);
    if (rc) return rc;
    uint8_t* base = (uint8_t*)dbuf;
    size_t cur = 0;
    for (auto& pr : parts) {
        if (pr.first && pr.second) GF_HIP(hipMemcpyAsync(base + cur, pr.first, pr.second, hipMemcpyHostToDevice, ctx->stream));
        cur += (pr.second + 15) & ~(size_t)15;
    }
    gf_fuse_problem q{};
    for (int k = 0; k < 12; k++) q.Tcw[k] = Tcw[k];
    for (int k = 0; k < 3; k++) q.Ow[k] = Ow[k];
    q.kps = (const gf_keypoint*)(base + o_k);
    q.desc = base + o_d;
    q.n = n;
    q.kf_mp = (const int32_t*)(base + o_mp);
    q.kf_mp_bad = kf_mp_bad ? base + o_bad : nullptr;
    q.mps = (const gf_map_point*)(base + o_m);
    q.mp_desc = base + o_md;
    q.mp_skip = mp_skip ? base + o_sk : nullptr;
    q.mp_ids = mp_ids ? (const int32_t*)(base + o_id) : nullptr;
    q.m = m;
    q.th = th;
    q.res = (gf_fuse_result*)(base + o_r);
    q.nfused = (int32_t*)(base + o_nf);
    rc = gf_fuse_dev(ctx, fi, 1, &q, ctx->stream);
    if (rc) return rc;
    int32_t nf = 0;
    GF_HIP(hipMemcpyAsync(res, base + o_r, sizeof(gf_fuse_result) * (size_t)m, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(&nf, base + o_nf, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    *nfused = nf;
    return GF_OK;
}

}  // extern "C"
