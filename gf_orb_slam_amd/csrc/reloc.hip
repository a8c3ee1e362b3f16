// Track-loss paths of the batched tracking step on gfx950: the state machine
// of Tracking::GrabImage around the steady-state path (Tracking.cc:602-644).
//
//   k_reloc_cand  one wave per stream that relocalises this step:
//                 KeyFrameDatabase::DetectRelocalisationCandidates
//                 (KeyFrameDatabase.cc:198-308) on the frame's BowVector and
//                 the stream's database, then one ORBmatcher::SearchByBoW
//                 pair per candidate (k_match_bow runs them, bow.hip);
//   k_track_loss  one wave per stream: TrackWithMotionModel's outlier
//                 discard and failure test (Tracking.cc:1550-1563, 1559,
//                 1641), TrackPreviousFrame (:1325-1404)
//                 with WindowSearch (ORBmatcher.cc:979-1086) and
//                 SearchByProjection(F1, F2, window) (:1089-1168), or the
//                 relocalisation loop (:3884-4031): EPnP RANSAC iterate(5) per
//                 candidate in rounds (pnp_core.h), PoseOptimization
//                 (poseopt_core.h) and SearchByProjection(F, KF, found, th,
//                 ORBdist) (:2204-2336).
//
// These paths run on frames that lost track: they are sequential in the
// reference (claims in query order, one std::rand() stream shared by the
// candidates' RANSAC), so a stream gets one wave that walks them in order,
// with the candidate windows split over the lanes (cells in turn) and the
// (distance, position) top-2 reduced across the wave exactly as the
// reference's first-minimum loops pick. A stream on the steady-state path
// leaves both kernels at once.
#include <climits>
#include <cmath>
#include <map>
#include <vector>

#include "pnp_core.h"
#include "poseopt_core.h"
#include "reloc.h"

struct gf_kfdb {
    int device = 0;  // the context's device (the context may go first)
    gf::KfdbDev dev{};
    std::vector<void*> allocs;
};

namespace {

constexpr int TL_T = 64;  // one wave per stream
#ifndef TL_GRID
#define TL_GRID 8  // k_track_loss workgroups
#endif

__device__ __forceinline__ int32_t* stat_of(const gf::TrackLossArgs& A, int which) {
    return A.stats + (size_t)which * A.B;
}

// ------------------------------------------------------------ window walks
struct GridView {
    const int* cs;     // cell_start [NCELLS + 1]
    const int* items;  // keypoints per cell, ascending
};

// best / second best / position / keypoint of a candidate sequence
struct Top2 {
    int d1, p1, i1, d2;
};

__device__ __forceinline__ Top2 top2_init() { return Top2{INT_MAX, INT_MAX, -1, INT_MAX}; }

// The reference's loop: dist < best -> second = best, best = dist; else dist < second -> second = dist.
__device__ __forceinline__ void top2_push(Top2& t, int d, int pos, int idx) {
    if (d < t.d1) {
        t.d2 = t.d1;
        t.d1 = d;
        t.p1 = pos;
        t.i1 = idx;
    } else if (d < t.d2) {
        t.d2 = d;
    }
}

// Lanes hold disjoint, position-ordered parts of the sequence: the merged
// best is the smaller distance (ties: earlier position) and the second best
// the smaller of the winner's second and the loser's best.
__device__ __forceinline__ Top2 top2_reduce(Top2 t) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int od1 = __shfl_xor(t.d1, o, 64), op1 = __shfl_xor(t.p1, o, 64);
        const int oi1 = __shfl_xor(t.i1, o, 64), od2 = __shfl_xor(t.d2, o, 64);
        if (od1 < t.d1 || (od1 == t.d1 && op1 < t.p1)) {
            t.d2 = min(od2, t.d1);
            t.d1 = od1;
            t.p1 = op1;
            t.i1 = oi1;
        } else {
            t.d2 = min(t.d2, od1);
        }
    }
    return t;
}

// Frame::GetFeaturesInArea(x, y, r, minL, maxL) (Frame.cc:300-365) in the
// reference's order — cells ix-major then iy, keypoints ascending — with the
// cells dealt to the lanes in turn; f(idx, pos) for every keypoint passing the
// level and distance tests, pos increasing along each lane's share.
template <typename F>
__device__ __forceinline__ void area_walk(const FrameConst& fc, const GridView& G, const gf_keypoint* K, float x,
                                          float y, float r, int minL, int maxL, F&& f) {
    int cx0, cx1, cy0, cy1;
    if (!grid_window(fc, x, y, r, cx0, cx1, cy0, cy1)) return;
    const int ncy = cy1 - cy0 + 1, nc = (cx1 - cx0 + 1) * ncy;
    for (int c = threadIdx.x; c < nc; c += TL_T) {
        const int ix = cx0 + c / ncy, iy = cy0 + c % ncy;
        const int cell = ix * GRID_ROWS + iy;
        const int s = G.cs[cell], e = G.cs[cell + 1];
        for (int j = s; j < e; j++) {
            const int idx = G.items[j];
            const gf_keypoint k = K[idx];
            if (!level_ok(k.octave, minL, maxL)) continue;
            if (fabsf(k.x - x) > r || fabsf(k.y - y) > r) continue;
            f(idx, (c << 12) | (j - s));
        }
    }
}

__device__ __forceinline__ int rot_bin(float a1, float a2) {
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * (1.0f / HISTO_LENGTH));
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

// ComputeThreeMaxima (ORBmatcher.cc:2338-2379) over the recorded claims
// (rec[r] = bin << 16 | keypoint) and removal of those outside the three
// dominant bins (kp2mp = -1, and score = 999 when given). Returns the
// removals (wave-uniform).
__device__ int rotation_filter(const int32_t* rec, int nrec, int32_t* kp2mp, int32_t* score, int* s_hist,
                               int* s_keep) {
    const int lane = threadIdx.x;
    for (int i = lane; i < HISTO_LENGTH; i += TL_T) s_hist[i] = 0;
    __syncthreads();
    for (int r = lane; r < nrec; r += TL_T) atomicAdd(&s_hist[rec[r] >> 16], 1);
    __syncthreads();
    if (lane == 0) {
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int s = s_hist[i];
            if (s > max1) {
                max3 = max2;
                max2 = max1;
                max1 = s;
                ind3 = ind2;
                ind2 = ind1;
                ind1 = i;
            } else if (s > max2) {
                max3 = max2;
                max2 = s;
                ind3 = ind2;
                ind2 = i;
            } else if (s > max3) {
                max3 = s;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        s_keep[0] = ind1;
        s_keep[1] = ind2;
        s_keep[2] = ind3;
    }
    __syncthreads();
    int drop = 0;
    for (int r = lane; r < nrec; r += TL_T) {
        const int bin = rec[r] >> 16, idx = rec[r] & 0xffff;
        if (bin == s_keep[0] || bin == s_keep[1] || bin == s_keep[2]) continue;
        kp2mp[idx] = -1;
        if (score) score[idx] = 999;
        drop++;
    }
    drop = gfd::warp_sum(drop);
    __syncthreads();
    return drop;
}

// ORBmatcher::WindowSearch(F1, F2, window, vpMapPointMatches2, minL, maxL)
// (ORBmatcher.cc:979-1086): out = F2's matches (reset here).
__device__ int window_search(const FrameConst& fc, const GridView& G, const gf_keypoint* K2, const uint8_t* D2, int n2,
                             const gf_keypoint* K1, const uint8_t* D1, const int32_t* mp1, int n1, int window,
                             int minL, int maxL, float nnratio, int check_ori, int32_t* out, int32_t* rec, int* s_hist,
                             int* s_keep) {
    const int lane = threadIdx.x;
    for (int i = lane; i < n2; i += TL_T) out[i] = -1;
    __syncthreads();
    const bool bMin = minL > 0, bMax = maxL < INT_MAX;
    int nrec = 0;
    for (int i1 = 0; i1 < n1; i1++) {
        const int mp = mp1[i1];
        if (mp < 0) continue;
        const gf_keypoint k1 = K1[i1];
        if (bMin && k1.octave < minL) continue;
        if (bMax && k1.octave > maxL) continue;
        const uint8_t* d1 = D1 + 32 * (size_t)i1;
        Top2 t = top2_init();
        area_walk(fc, G, K2, k1.x, k1.y, (float)window, k1.octave, k1.octave, [&](int idx, int pos) {
            if (out[idx] >= 0) return;
            top2_push(t, hamming32(d1, D2 + 32 * (size_t)idx), pos, idx);
        });
        t = top2_reduce(t);
        if ((float)t.d1 <= (float)t.d2 * nnratio && t.d1 <= TH_HIGH) {
            if (lane == 0) {
                out[t.i1] = mp;
                rec[nrec] = (rot_bin(k1.angle, K2[t.i1].angle) << 16) | t.i1;
            }
            nrec++;
            __syncthreads();
        }
    }
    __syncthreads();
    int nm = nrec;
    if (check_ori) nm -= rotation_filter(rec, nrec, out, nullptr, s_hist, s_keep);
    return nm;
}

// Marks the map points of kp2mp (n entries) in bits (M <= 4096).
__device__ void mark_found(const int32_t* kp2mp, int n, uint32_t* bits) {
    const int lane = threadIdx.x;
    for (int w = lane; w < 128; w += TL_T) bits[w] = 0u;
    __syncthreads();
    for (int i = lane; i < n; i += TL_T) {
        const int mp = kp2mp[i];
        if (mp >= 0 && mp < 4096) atomicOr(&bits[mp >> 5], 1u << (mp & 31));
    }
    __syncthreads();
}

__device__ __forceinline__ bool bit_of(const uint32_t* bits, int i) { return (bits[i >> 5] >> (i & 31)) & 1u; }

// ORBmatcher::SearchByProjection(F1, F2, window, vpMapPointMatches2)
// (ORBmatcher.cc:1089-1168): kp2mp / score are F2's, in and out.
__device__ int search_frames(const FrameConst& fc, const GridView& G, const gf_keypoint* K2, const uint8_t* D2, int n2,
                             const float* Tcw2, const gf_keypoint* K1, const uint8_t* D1, const int32_t* mp1,
                             const float* pos1, int n1, int window, float nnratio, int32_t* kp2mp, int32_t* score,
                             uint32_t* s_found) {
    const int lane = threadIdx.x;
    mark_found(kp2mp, n2, s_found);  // spMapPointsAlreadyFound, taken at entry
    int nm = 0;
    for (int i1 = 0; i1 < n1; i1++) {
        const int mp = mp1[i1];
        if (mp < 0 || bit_of(s_found, mp)) continue;
        const int level1 = K1[i1].octave;
        float Pc[3];
        transform3(Tcw2, pos1 + 3 * (size_t)i1, Pc);
        const float invzc2 = (float)(1.0 / (double)Pc[2]);
        const float u2 = fc.fx * Pc[0] * invzc2 + fc.cx;
        const float v2 = fc.fy * Pc[1] * invzc2 + fc.cy;
        const uint8_t* d1 = D1 + 32 * (size_t)i1;
        Top2 t = top2_init();
        area_walk(fc, G, K2, u2, v2, (float)window, level1, level1, [&](int idx, int pos) {
            if (kp2mp[idx] >= 0) return;
            top2_push(t, hamming32(d1, D2 + 32 * (size_t)idx), pos, idx);
        });
        t = top2_reduce(t);
        if ((float)t.d1 <= (float)t.d2 * nnratio && t.d1 <= TH_HIGH) {
            if (lane == 0) {
                kp2mp[t.i1] = mp;
                score[t.i1] = t.d1;
            }
            nm++;
            __syncthreads();
        }
    }
    __syncthreads();
    return nm;
}

// ORBmatcher::SearchByProjection(F, pKF, sAlreadyFound, th, ORBdist)
// (ORBmatcher.cc:2204-2336), rotation consistency on.
__device__ int search_kf(const FrameConst& fc, const GridView& G, const gf_keypoint* K, const uint8_t* D, int n,
                         const float* Tcw, const gf_keypoint* kfK, const int32_t* kf_mp, int nslots,
                         const gf_map_point* mps, const uint8_t* mdesc, const uint32_t* found, float th, int orb_dist,
                         int check_ori, int32_t* kp2mp, int32_t* score, int32_t* rec, int* s_hist, int* s_keep) {
    const int lane = threadIdx.x;
    float Ow[3];  // -Rcw^T tcw (:2210)
    for (int c = 0; c < 3; c++) {
        const float a = Tcw[0 * 4 + c] * Tcw[3], b = Tcw[1 * 4 + c] * Tcw[7], d = Tcw[2 * 4 + c] * Tcw[11];
        Ow[c] = -((a + b) + d);
    }
    int nrec = 0;
    for (int i = 0; i < nslots; i++) {
        const int mp = kf_mp[i];
        if (mp < 0 || bit_of(found, mp)) continue;
        const gf_map_point P = mps[mp];
        float Pc[3];
        transform3(Tcw, P.pos, Pc);
        const float invzc = (float)(1.0 / (double)Pc[2]);
        const float u = fc.fx * Pc[0] * invzc + fc.cx;
        const float v = fc.fy * Pc[1] * invzc + fc.cy;
        if (u < fc.min_x || u > fc.max_x) continue;
        if (v < fc.min_y || v > fc.max_y) continue;
        const float PO[3] = {P.pos[0] - Ow[0], P.pos[1] - Ow[1], P.pos[2] - Ow[2]};
        const float dist3D =
            (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);  // cv::norm
        const float ratio = dist3D / P.min_dist;
        int lb = 0;  // lower_bound(mvScaleFactors, ratio)
        while (lb < fc.nlevels && fc.scales[lb] < ratio) lb++;
        const int pred = min(lb, fc.nlevels - 1);
        const float radius = th * fc.scales[pred];
        const uint8_t* dm = mdesc + 32 * (size_t)mp;
        Top2 t = top2_init();
        area_walk(fc, G, K, u, v, radius, pred - 1, pred + 1, [&](int idx, int pos) {
            if (kp2mp[idx] >= 0) return;
            top2_push(t, hamming32(dm, D + 32 * (size_t)idx), pos, idx);
        });
        t = top2_reduce(t);
        if (t.d1 <= orb_dist) {
            if (lane == 0) {
                kp2mp[t.i1] = mp;
                score[t.i1] = t.d1;
                rec[nrec] = (rot_bin(kfK[i].angle, K[t.i1].angle) << 16) | t.i1;
            }
            nrec++;
            __syncthreads();
        }
    }
    __syncthreads();
    int nm = nrec;
    if (check_ori) nm -= rotation_filter(rec, nrec, kp2mp, score, s_hist, s_keep);
    return nm;
}

// ----------------------------------------------------------- pose and PnP
// Optimizer::PoseOptimization on the stream's current matches (edges in
// keypoint order over the stream map's positions); returns nInitial - nBad.
__device__ int pose_wave(const gf::TrackLossArgs& A, int b) {
    const int lane = threadIdx.x, cap = A.cap;
    const int n = A.nkp[b];
    const int32_t* kp2mp = A.kp2mp + (size_t)b * cap;
    const gf_keypoint* K = A.kps + (size_t)b * cap;
    gf_pose_edge* E = A.edges + (size_t)b * cap;
    int32_t* ek = A.edge_kp + (size_t)b * cap;
    int cnt = 0;
    for (int base = 0; base < n; base += TL_T) {
        const int i = base + lane;
        const int mp = i < n ? kp2mp[i] : -1;
        const bool on = mp >= 0;
        const unsigned long long m = __ballot(on);
        if (on) {
            const gf_keypoint k = K[i];
            const gf_map_point& P = A.gmap[(size_t)b * A.M + mp];
            gf_pose_edge e;
            e.X[0] = P.pos[0];
            e.X[1] = P.pos[1];
            e.X[2] = P.pos[2];
            e.z[0] = k.x;
            e.z[1] = k.y;
            e.inv_sigma2 = A.inv_sigma2[min(max((int)k.octave, 0), A.nlevels - 1)];
            const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
            E[pos] = e;
            ek[pos] = i;
        }
        cnt += __popcll(m);
    }
    int32_t* pi = A.pint + 4 * (size_t)b;
    if (lane == 0) pi[0] = cnt;
    __syncthreads();
    gfpose::PoseArgs P{};
    P.edges = E;
    P.nedges = pi;
    P.stride = cap;
    P.Tcw = A.Tcw + 16 * (size_t)b;
    P.outl = A.eoutl + (size_t)b * cap;
    P.ninl = pi + 1;
    P.iters = pi + 2;
    P.work = A.pwork + 3 * (size_t)b * cap;
    P.fx = A.fc.fx;
    P.fy = A.fc.fy;
    P.cx = A.fc.cx;
    P.cy = A.fc.cy;
    P.edge_kp = ek;
    P.kp_outl = A.outl + (size_t)b * cap;
    P.kp_stride = cap;
    gfpose::pose_opt_problem<64>(P, 0);
    __syncthreads();
    return pi[1];
}

// Matches flagged as outliers set NULL; with reset the flags too (the loops of
// TrackPreviousFrame) — Relocalisation's loops leave them. Returns the count.
__device__ int discard_outliers(const gf::TrackLossArgs& A, int b, bool reset) {
    const int lane = threadIdx.x;
    const int n = A.nkp[b];
    int32_t* kp2mp = A.kp2mp + (size_t)b * A.cap;
    uint8_t* ou = A.outl + (size_t)b * A.cap;
    int c = 0;
    for (int i = lane; i < n; i += TL_T)
        if (ou[i] && kp2mp[i] >= 0) {
            kp2mp[i] = -1;
            if (reset) ou[i] = 0;
            c++;
        }
    c = gfd::warp_sum(c);
    __syncthreads();
    return c;
}

// PnPsolver::SetRansacParameters(0.99, 10, 300, 4, 0.5, 5.991) (PnPsolver.cc:93-129)
// for N correspondences (one lane).
__device__ gf_pnp_state pnp_state_for(int N) {
    gf_pnp_state st{};
    st.n = N;
    st.min_set = 4;
    st.th2 = 5.991f;
    float eps = 0.5f;
    int nMinInliers = N * eps;
    if (nMinInliers < 10) nMinInliers = 10;
    if (nMinInliers < 4) nMinInliers = 4;
    if (N > 0 && eps < (float)nMinInliers / N) eps = (float)nMinInliers / N;
    int nIterations;
    if (nMinInliers == N) {
        nIterations = 1;
    } else {
        const double it = ceil(log(1 - 0.99) / log(1 - pow((double)eps, 3.0)));
        nIterations = (it == it && it < 2147483647.0) ? (int)it : 300;
    }
    st.min_inliers = nMinInliers;
    st.epsilon = eps;
    st.max_iterations = max(1, min(nIterations, 300));
    return st;
}

// The solver's correspondences for candidate slot k: the keypoints j (in
// order) whose SearchByBoW match is set (PnPsolver ctor :50-73). Returns N.
__device__ int pnp_corr(const gf::TrackLossArgs& A, int b, const int32_t* match) {
    const int lane = threadIdx.x, cap = A.cap;
    const int n = A.nkp[b];
    const gf_keypoint* K = A.kps + (size_t)b * cap;
    float* P3 = A.p3d + 3 * (size_t)b * cap;
    float* P2 = A.p2d + 2 * (size_t)b * cap;
    float* S2 = A.psig + (size_t)b * cap;
    int32_t* PI = A.pidx + (size_t)b * cap;
    int cnt = 0;
    for (int base = 0; base < n; base += TL_T) {
        const int j = base + lane;
        const int mp = j < n ? match[j] : -1;
        const bool on = mp >= 0;
        const unsigned long long m = __ballot(on);
        if (on) {
            const int pos = cnt + __popcll(m & ((1ull << lane) - 1ull));
            const gf_keypoint k = K[j];
            const gf_map_point& P = A.gmap[(size_t)b * A.M + mp];
            P3[3 * pos] = P.pos[0];
            P3[3 * pos + 1] = P.pos[1];
            P3[3 * pos + 2] = P.pos[2];
            P2[2 * pos] = k.x;
            P2[2 * pos + 1] = k.y;
            S2[pos] = A.level_sigma2[min(max((int)k.octave, 0), A.nlevels - 1)];
            PI[pos] = j;
        }
        cnt += __popcll(m);
    }
    __syncthreads();
    return cnt;
}

// PnPsolver::iterate(5, ...) of candidate slot k: the draws on lane 0, the
// hypotheses over the lanes, the scan by the wave. Flags / inliers in
// A.pflags[b], the pose in A.ptcw[b], the inlier mask in A.pinl[b].
__device__ int pnp_iterate_wave(const gf::TrackLossArgs& A, int b, int k) {
    const int lane = threadIdx.x, cap = A.cap;
    gf_pnp_state* st = A.pst + (size_t)b * gf::RL_NC + k;
    uint8_t* bm = A.pbest + ((size_t)b * gf::RL_NC + k) * cap;
    const float* P3 = A.p3d + 3 * (size_t)b * cap;
    const float* P2 = A.p2d + 2 * (size_t)b * cap;
    const float* S2 = A.psig + (size_t)b * cap;
    int32_t* draws = A.pdraws + (size_t)b * gf::RL_LCAP * 8;
    double* rt = A.prt + (size_t)b * gf::RL_LCAP * 12;
    int32_t* cnt = A.pcnt + (size_t)b * gf::RL_LCAP;
    const gfpnp::Cam cam{(double)A.fc.fx, (double)A.fc.fy, (double)A.fc.cx, (double)A.fc.cy};
    if (lane == 0) gfpnp::pnp_draw_one(st, A.rng + b, 0, 5, gf::RL_LCAP, draws, cap);
    __syncthreads();
    for (int h = lane; h < gf::RL_LCAP; h += TL_T)
        gfpnp::pnp_hyp_one(P3, P2, S2, cap, cam, st, 5, gf::RL_LCAP, draws, rt, cnt, 0, h);
    __syncthreads();
    int32_t* fl = A.pflags + 2 * (size_t)b;
    gfpnp::pnp_scan_block(P3, P2, S2, cap, cam, st, bm, 5, gf::RL_LCAP, rt, cnt, A.pwk + (size_t)b * cap * gf::RL_WORK,
                          A.rng + b, A.ptcw + 16 * (size_t)b, A.pinl + (size_t)b * cap, fl + 1, fl, 0);
    __syncthreads();
    return fl[0];
}

// ------------------------------------------------------------ the two paths
struct TLShared {
    uint32_t found[128];
    int hist[HISTO_LENGTH];
    int keep[3];
    uint8_t discarded[gf::RL_NC];
};

__device__ GridView frame_grid(const gf::TrackLossArgs& A, int b) {
    int32_t* g = A.grid + (size_t)b * gf::grid_ints(A.cap);
    int* cs = g;
    int* items = cs + NCELLS + 1;
    int* claim = items + A.cap;
    int* scratch = claim + A.cap;
    build_grid(A.fc, A.kps + (size_t)b * A.cap, A.nkp[b], A.kp2mp + (size_t)b * A.cap, cs, items, claim,
               scratch, TL_T);
    return GridView{cs, items};
}

// Tracking::TrackPreviousFrame (Tracking.cc:1325-1404); mTcw = mLastFrame.mTcw
// and mvpMapPoints = NULL on entry. Returns bOK.
__device__ bool track_previous_frame(const gf::TrackLossArgs& A, int b, TLShared& S) {
    const int cap = A.cap;
    const GridView G = frame_grid(A, b);
    const gf_keypoint* K2 = A.kps + (size_t)b * cap;
    const uint8_t* D2 = A.desc + (size_t)b * cap * 32;
    const int n2 = A.nkp[b];
    const gf_keypoint* K1 = A.last_kps + (size_t)b * cap;
    const uint8_t* D1 = A.last_desc + (size_t)b * cap * 32;
    const int32_t* mp1 = A.last_kp2mp + (size_t)b * cap;
    const float* pos1 = A.last_pos + 3 * (size_t)b * cap;
    const int n1 = A.last_nkp[b];
    int32_t* kp2mp = A.kp2mp + (size_t)b * cap;
    int32_t* score = A.score + (size_t)b * cap;
    int32_t* rec = A.rec + (size_t)b * cap;
    const float* Tcw = A.Tcw + 16 * (size_t)b;
    // coarse levels first when the map has more than 5 keyframes (:1335-1338)
    const int kfc = A.kf_count[b];
    const int minOctave = (kfc < 0 || kfc > 5) ? (A.nlevels - 1) / 2 + 1 : 0;
    int nm = window_search(A.fc, G, K2, D2, n2, K1, D1, mp1, n1, 200, minOctave, INT_MAX, 0.9f, 1, kp2mp, rec, S.hist,
                           S.keep);
    if (nm < 10) {
        nm = window_search(A.fc, G, K2, D2, n2, K1, D1, mp1, n1, 100, 0, INT_MAX, 0.9f, 1, kp2mp, rec, S.hist,
                           S.keep);
        if (nm < 10) {
            for (int i = threadIdx.x; i < n2; i += TL_T) kp2mp[i] = -1;
            __syncthreads();
            nm = 0;
        }
    }
    if (nm >= 10) {
        pose_wave(A, b);
        nm -= discard_outliers(A, b, true);
        nm += search_frames(A.fc, G, K2, D2, n2, Tcw, K1, D1, mp1, pos1, n1, 15, 0.9f, kp2mp, score, S.found);
    } else {  // last opportunity
        nm = search_frames(A.fc, G, K2, D2, n2, Tcw, K1, D1, mp1, pos1, n1, 50, 0.9f, kp2mp, score, S.found);
    }
    if (nm >= 10) {
        pose_wave(A, b);
        nm -= discard_outliers(A, b, true);
    }
    if (threadIdx.x == 0) stat_of(A, GF_ST_TPF)[b] = nm;
    return nm >= 10;
}

// Tracking::Relocalisation (Tracking.cc:3854-4031) after the candidates and
// their SearchByBoW matches (k_reloc_cand + k_match_bow). Returns bMatch.
__device__ bool relocalise(const gf::TrackLossArgs& A, int b, TLShared& S) {
    const int lane = threadIdx.x, cap = A.cap;
    if (!A.kfdb) return false;
    const gf::KfdbDev db = A.kfdb[b];
    if (db.nkf <= 0 || !A.rl_on) return false;  // no database, or no candidates computed this step
    const int nc = A.ncand[b];
    if (nc <= 0) return false;
    const gf_covis_map cv = A.covis[b];
    const int32_t* cand = A.cands + (size_t)b * gf::RL_NC;
    const int n = A.nkp[b];
    int32_t* kp2mp = A.kp2mp + (size_t)b * cap;
    int32_t* score = A.score + (size_t)b * cap;
    int32_t* rec = A.rec + (size_t)b * cap;
    float* Tcw = A.Tcw + 16 * (size_t)b;
    // ORBmatcher(0.75, true).SearchByBoW per candidate; >= 15 -> a PnPsolver
    int nCandidates = 0;
    for (int i = 0; i < nc; i++) {
        const int kf = cand[i];
        const int nmb = A.bow_nm[(size_t)b * A.ncs + i];
        bool disc = cv.kf_bad[kf] || nmb < 15;
        if (!disc) {
            const int N = pnp_corr(A, b, A.bow_out + ((size_t)b * A.ncs + i) * cap);
            if (lane == 0) A.pst[(size_t)b * gf::RL_NC + i] = pnp_state_for(N);
            uint8_t* bm = A.pbest + ((size_t)b * gf::RL_NC + i) * cap;
            for (int j = lane; j < N; j += TL_T) bm[j] = 0;
            nCandidates++;
        }
        if (lane == 0) S.discarded[i] = disc;
    }
    __syncthreads();
    bool bMatch = false;
    int attempts = 0, nGood = 0;
    const GridView G = frame_grid(A, b);
    const gf_keypoint* K = A.kps + (size_t)b * cap;
    const uint8_t* D = A.desc + (size_t)b * cap * 32;
    const gf_map_point* mps = A.gmap + (size_t)b * A.M;
    const uint8_t* mdesc = A.gdesc + (size_t)b * A.M * 32;
    while (nCandidates > 0 && !bMatch) {
        for (int i = 0; i < nc; i++) {
            if (S.discarded[i]) continue;
            const int32_t* match = A.bow_out + ((size_t)b * A.ncs + i) * cap;
            const int N = pnp_corr(A, b, match);
            const int fl = pnp_iterate_wave(A, b, i);
            attempts++;
            if (fl & GF_PNP_NOMORE) {
                if (lane == 0) S.discarded[i] = 1;
                nCandidates--;
            }
            __syncthreads();
            if (!(fl & GF_PNP_FOUND)) continue;
            // Tcw and the inlier matches into the frame; sFound
            if (lane < 16) Tcw[lane] = A.ptcw[16 * (size_t)b + lane];
            for (int j = lane; j < n; j += TL_T) kp2mp[j] = -1;
            __syncthreads();
            const uint8_t* inl = A.pinl + (size_t)b * cap;
            const int32_t* PI = A.pidx + (size_t)b * cap;
            for (int q = lane; q < N; q += TL_T)
                if (inl[q]) kp2mp[PI[q]] = match[PI[q]];
            __syncthreads();
            mark_found(kp2mp, n, S.found);
            nGood = pose_wave(A, b);
            if (nGood < 10) continue;
            discard_outliers(A, b, false);
            if (nGood < 50) {
                const int kf = cand[i];
                const int32_t* kmp = cv.kf_mp + cv.kf_mp_off[kf];
                const int nsl = cv.kf_mp_off[kf + 1] - cv.kf_mp_off[kf];
                const gf_keypoint* kfK = db.kps + db.kp_off[kf];
                int nadd = search_kf(A.fc, G, K, D, n, Tcw, kfK, kmp, nsl, mps, mdesc, S.found, 10.f, 100, 1, kp2mp,
                                     score, rec, S.hist, S.keep);
                if (nadd + nGood >= 50) {
                    nGood = pose_wave(A, b);
                    if (nGood > 30 && nGood < 50) {
                        mark_found(kp2mp, n, S.found);
                        nadd = search_kf(A.fc, G, K, D, n, Tcw, kfK, kmp, nsl, mps, mdesc, S.found, 3.f, 64, 1, kp2mp,
                                         score, rec, S.hist, S.keep);
                        if (nGood + nadd >= 50) {
                            nGood = pose_wave(A, b);
                            discard_outliers(A, b, false);
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
    if (lane == 0) {
        stat_of(A, GF_ST_RELOC)[b] = nGood;
        stat_of(A, GF_ST_RANSAC)[b] = attempts;
    }
    return bMatch;
}

// The TrackLocalMap stages' gates for stream b (one lane): it runs when the
// initial estimate succeeded; within 2 frames of a relocalisation
// (mnId < mnLastRelocFrameId + 2) SearchReferencePointsInFrustum skips
// updatePWLSVec / FRAME_INFO_MATRIX (Tracking.cc:3162) and searches with th 5
// (:3318-3320).
__device__ void set_gates(const gf::TrackLossArgs& A, int b, bool ok, int since) {
    const bool recent = since < 2;
    const int n = A.nkp[b];
    A.gate_tl[b] = ok;
    A.nkp_tl[b] = ok ? n : 0;
    A.gate_fi[b] = ok && !recent;
    A.nkp_fi[b] = ok && !recent ? n : 0;
    A.th_m2[b] = recent ? 5.f : 1.f;
    if (A.nmp_step) A.nmp_step[b] = ok ? A.gnmp[b] : 0;
}

// The steady-state part of the step's track-loss stage, one light wave per
// stream: TrackWithMotionModel's outlier discard and failure test. A stream
// that passes gets its TrackLocalMap gates (GF_TR_OK = 1); the others (the
// motion model failed, or the stream is on TrackPreviousFrame or LOST) are
// left to k_track_loss with GF_TR_OK = 0 and GF_TR_PATH set.
__global__ __launch_bounds__(TL_T) void k_track_gate(gf::TrackLossArgs A) {
    const int b = blockIdx.x, lane = threadIdx.x, cap = A.cap;
    int32_t* T = A.track + (size_t)b * GF_TR_N;
    const int path = T[GF_TR_PATH];
    {  // TrackWithMotionModel's outlier discard (Tracking.cc:1550-1563): nMatchesFound, num_to_match
        const int n = A.nkp[b];
        int32_t* km = A.kp2mp + (size_t)b * cap;
        uint8_t* ou = A.outl + (size_t)b * cap;
        int c = 0;
        for (int i = lane; i < n; i += TL_T)
            if (km[i] >= 0) {
                if (ou[i]) {
                    km[i] = -1;
                    ou[i] = 0;
                } else {
                    c++;
                }
            }
        c = gfd::warp_sum(c);
        if (path == 0) {  // TrackWithMotionModel: < 20 matches (:1559) or < 10 after the discard (:1641)
            const bool ok = stat_of(A, GF_ST_M3)[b] >= 20 && c >= 10;
            if (ok) {
                if (lane == 0) {
                    stat_of(A, GF_ST_FOUND)[b] = c;
                    stat_of(A, GF_ST_TO_MATCH)[b] = A.budget - c;
                    T[GF_TR_OK] = 1;
                    set_gates(A, b, true, T[GF_TR_SINCE]);
                }
                return;
            }
            // fall back to TrackPreviousFrame
            for (int i = lane; i < n; i += TL_T) km[i] = -1;
            if (lane < 16) A.Tcw[16 * (size_t)b + lane] = A.Tcw_last[16 * (size_t)b + lane];
        }
        if (lane == 0) {
            T[GF_TR_OK] = 0;
            if (path == 0) T[GF_TR_PATH] = 1;
        }
    }
}

// TrackPreviousFrame or the relocalisation loop for the streams k_track_gate
// left (GF_TR_OK = 0): a small grid of one-wave workgroups walks the streams,
// since each workgroup holds a whole SIMD's registers and most steps have no
// such stream.
#ifndef TL_WAVES_PER_EU
#define TL_WAVES_PER_EU 2
#endif
// TL_WAVES_PER_EU 2 caps the kernel at 256 registers (the rest spills to
// scratch on this rare path), so its no-op waves need half a SIMD's register
// file instead of all of it to be dispatched beside the other groups' kernels
__global__ __launch_bounds__(TL_T) __attribute__((amdgpu_waves_per_eu(TL_WAVES_PER_EU))) void k_track_loss(
    gf::TrackLossArgs A) {
    __shared__ TLShared S;
    const int lane = threadIdx.x, cap = A.cap;
    // this workgroup's streams (b = blockIdx.x mod gridDim.x): their OK flags
    // read 64 at a time by the lanes and the ones still open walked in order
    // (a stream-by-stream scan paid one dependent load per stream when none
    // is open, the common case)
    for (int b0 = 0; b0 < A.B; b0 += 64 * (int)gridDim.x) {
        const int bl = b0 + (int)gridDim.x * lane + (int)blockIdx.x;
        const bool open = bl < A.B && !A.track[(size_t)bl * GF_TR_N + GF_TR_OK];
        unsigned long long todo = __ballot(open);
        while (todo) {
            const int b = b0 + (int)gridDim.x * (__ffsll((long long)todo) - 1) + (int)blockIdx.x;
            todo &= todo - 1;
            int32_t* T = A.track + (size_t)b * GF_TR_N;
            const int path = T[GF_TR_PATH];
            const bool ok = path == 3 ? relocalise(A, b, S) : track_previous_frame(A, b, S);
            // nMatchesFound / num_to_match of the frame's matches (Tracking.cc:3195-3228)
            const int n = A.nkp[b];
            int c = 0;
            for (int i = lane; i < n; i += TL_T) c += A.kp2mp[(size_t)b * cap + i] >= 0;
            c = gfd::warp_sum(c);
            if (lane == 0) {
                stat_of(A, GF_ST_FOUND)[b] = c;
                stat_of(A, GF_ST_TO_MATCH)[b] = A.budget - c;
                T[GF_TR_OK] = ok;
                int fl = stat_of(A, GF_ST_FLAGS)[b];
                fl |= path == 3 ? 4096 : 2048;
                if (!ok) fl |= 8192;
                if (path == 3 && ok) {
                    fl |= 32768;
                    T[GF_TR_SINCE] = 0;  // mnLastRelocFrameId = mCurrentFrame.mnId
                }
                stat_of(A, GF_ST_FLAGS)[b] = fl;
                set_gates(A, b, ok, T[GF_TR_SINCE]);
            }
            __syncthreads();  // the LDS goes to the next stream
        }
    }
}

// ------------------------------------------------------------ candidates
__device__ int lower_bound_i(const int32_t* a, int lo, int hi, int key) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// L1Scoring::score (DBoW2 ScoringObject.cpp): common words in ascending order.
__device__ double l1_score(const int32_t* w1, const double* v1, int n1, const int32_t* w2, const double* v2, int n2) {
    double score = 0;
    int i = 0, j = 0;
    while (i < n1 && j < n2) {
        if (w1[i] == w2[j]) {
            const double vi = v1[i], wi = v2[j];
            score += fabs(vi - wi) - fabs(vi) - fabs(wi);
            i++;
            j++;
        } else if (w1[i] < w2[j]) {
            i = lower_bound_i(w1, i, n1, w2[j]);
        } else {
            j = lower_bound_i(w2, j, n2, w1[i]);
        }
    }
    return -score / 2.0;
}

struct CandShared {
    int share[gf::RL_NC];
    uint8_t scored[gf::RL_NC];
    float acc[gf::RL_NC];
    int best[gf::RL_NC];
    int cand[gf::RL_NC];
    int ns, nc;
};

// KeyFrameDatabase::DetectRelocalisationCandidates (KeyFrameDatabase.cc:198-308)
// by one wave: frame words W / V (nw), the keyframes' query state rkf.
__device__ int reloc_candidates_wave(const gf::KfdbDev& db, const uint8_t* kf_bad, const int32_t* cov_off,
                                     const int32_t* cov, const int32_t* W, const double* V, int nw, uint32_t query,
                                     gf_reloc_kf* rkf, int32_t* cands, CandShared& S) {
    const int lane = threadIdx.x;
    if (lane == 0) {
        int ns = 0;
        for (int i = 0; i < nw; i++) {  // lKFsSharingWords, frame words ascending
            const int w = W[i];
            const int p = lower_bound_i(db.inv_words, 0, db.nw, w);
            if (p >= db.nw || db.inv_words[p] != w) continue;
            for (int e = db.inv_off[p]; e < db.inv_off[p + 1]; e++) {
                const int k = db.inv_kf[e];
                if (kf_bad && kf_bad[k]) continue;  // erased from the database
                if (rkf[k].query != query) {
                    rkf[k].words = 0;
                    rkf[k].query = query;
                    if (ns < gf::RL_NC) S.share[ns++] = k;
                }
                rkf[k].words++;
            }
        }
        S.ns = ns;
        S.nc = 0;
    }
    __syncthreads();
    const int ns = S.ns;
    if (ns == 0) return 0;
    int maxCommon = 0;
    for (int k = 0; k < ns; k++) maxCommon = max(maxCommon, rkf[S.share[k]].words);
    const int minCommon = maxCommon * 0.8f;
    for (int k = lane; k < ns; k += TL_T) {
        const int kf = S.share[k];
        const bool sc = rkf[kf].words > minCommon;
        if (sc) {
            const float si = (float)l1_score(W, V, nw, db.bow_words + db.bow_off[kf], db.bow_values + db.bow_off[kf],
                                             db.bow_off[kf + 1] - db.bow_off[kf]);
            rkf[kf].score = si;
        }
        S.scored[k] = sc;
    }
    __syncthreads();
    if (lane == 0) {
        int na = 0;
        float bestAcc = 0;
        for (int k = 0; k < ns; k++) {
            if (!S.scored[k]) continue;
            const int kf = S.share[k];
            float bestScore = rkf[kf].score, accScore = bestScore;
            int pBest = kf;
            const int nn = min(10, cov_off[kf + 1] - cov_off[kf]);  // GetBestCovisibilityKeyFrames(10)
            for (int j = 0; j < nn; j++) {
                const int k2 = cov[cov_off[kf] + j];
                if (rkf[k2].query != query) continue;
                accScore += rkf[k2].score;
                if (rkf[k2].score > bestScore) {
                    pBest = k2;
                    bestScore = rkf[k2].score;
                }
            }
            S.acc[na] = accScore;
            S.best[na] = pBest;
            na++;
            if (accScore > bestAcc) bestAcc = accScore;
        }
        const float minScore = 0.75f * bestAcc;
        unsigned long long added = 0ull;
        int nc = 0;
        for (int a = 0; a < na; a++) {
            const int k = S.best[a];
            if (S.acc[a] > minScore && !((added >> k) & 1ull)) {
                cands[nc++] = k;
                added |= 1ull << k;
            }
        }
        S.nc = nc;
    }
    __syncthreads();
    return S.nc;
}

__global__ __launch_bounds__(TL_T) void k_reloc_cand(gf::TrackLossArgs A) {
    __shared__ CandShared S;
    const int b = blockIdx.x, lane = threadIdx.x, cap = A.cap;
    const gf::KfdbDev& db = A.kfdb[b];
    int nc = 0;
    if (A.rl_gate[b] && db.nkf > 0) {
        const gf_covis_map& cv = A.covis[b];
        nc = reloc_candidates_wave(db, cv.kf_bad, cv.kf_cov_off, cv.kf_cov, A.words + (size_t)b * cap,
                                   A.values + (size_t)b * cap, A.nwords[b],
                                   (uint32_t)A.track[(size_t)b * GF_TR_N + GF_TR_QUERY], A.rkf + (size_t)b * gf::RL_NC,
                                   A.cands + (size_t)b * gf::RL_NC, S);
    }
    if (lane == 0) {
        A.ncand[b] = nc;
        stat_of(A, GF_ST_NCAND)[b] = nc;
    }
    // SearchByBoW(pKF, mCurrentFrame) pairs; empty pairs past the candidates
    const gf_covis_map* cvp = A.covis + b;
    for (int i = lane; i < A.ncs; i += TL_T) {
        gf::BowPairDev p{};
        p.out = A.bow_out + ((size_t)b * A.ncs + i) * cap;
        if (i < nc) {
            const int kf = A.cands[(size_t)b * gf::RL_NC + i];
            p.a.fv_nodes = db.fv_nodes + db.fv_off[kf];
            p.a.fv_start = db.fv_start + db.fv_off[kf];
            p.a.fv_feats = db.fv_feats;
            p.a.nfv = db.fv_off[kf + 1] - db.fv_off[kf];
            p.a.desc = db.desc + (size_t)db.kp_off[kf] * 32;
            p.a.kps = db.kps + db.kp_off[kf];
            p.a.mp = cvp->kf_mp + cvp->kf_mp_off[kf];
            p.a.n = db.kp_off[kf + 1] - db.kp_off[kf];
            p.b.fv_nodes = A.fv_nodes + (size_t)b * cap;
            p.b.fv_start = A.fv_start + (size_t)b * (cap + 1);
            p.b.fv_feats = A.fv_feats + (size_t)b * cap;
            p.b.nfv = A.nfv[b];
            p.b.desc = A.desc + (size_t)b * cap * 32;
            p.b.kps = A.kps + (size_t)b * cap;
            p.b.mp = nullptr;
            p.b.n = A.nkp[b];
        }
        A.pairs[(size_t)b * A.ncs + i] = p;
    }
}

// ---------------------------------------------------------- unit wrappers
struct UnitArgs {
    FrameConst fc;
    const gf_keypoint* K2;
    const uint8_t* D2;
    int n2;
    const gf_keypoint* K1;
    const uint8_t* D1;
    const int32_t* mp1;
    const float* pos1;
    int n1;
    const float* Tcw;
    int window, minL, maxL, check_ori, orb_dist;
    float nnratio, th;
    const gf_map_point* mps;
    const uint8_t* mdesc;
    const uint8_t* found;
    int32_t* kp2mp;
    int32_t* score;
    int32_t* grid;
    int32_t* rec;
    int32_t* nm;
};

__device__ GridView unit_grid(const UnitArgs& U) {
    int* cs = U.grid;
    int* items = cs + NCELLS + 1;
    int* claim = items + U.n2;
    int* scratch = claim + U.n2;
    build_grid(U.fc, U.K2, U.n2, U.kp2mp, cs, items, claim, scratch, TL_T);
    return GridView{cs, items};
}

__global__ __launch_bounds__(TL_T) void k_unit_window(UnitArgs U) {
    __shared__ int hist[HISTO_LENGTH], keep[3];
    const GridView G = unit_grid(U);
    const int nm = window_search(U.fc, G, U.K2, U.D2, U.n2, U.K1, U.D1, U.mp1, U.n1, U.window, U.minL, U.maxL,
                                 U.nnratio, U.check_ori, U.kp2mp, U.rec, hist, keep);
    if (threadIdx.x == 0) *U.nm = nm;
}

__global__ __launch_bounds__(TL_T) void k_unit_frames(UnitArgs U) {
    __shared__ uint32_t found[128];
    const GridView G = unit_grid(U);
    const int nm = search_frames(U.fc, G, U.K2, U.D2, U.n2, U.Tcw, U.K1, U.D1, U.mp1, U.pos1, U.n1, U.window,
                                 U.nnratio, U.kp2mp, U.score, found);
    if (threadIdx.x == 0) *U.nm = nm;
}

__global__ __launch_bounds__(TL_T) void k_unit_kf(UnitArgs U, int nmp) {
    __shared__ uint32_t found[128];
    __shared__ int hist[HISTO_LENGTH], keep[3];
    for (int w = threadIdx.x; w < 128; w += TL_T) found[w] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < nmp; i += TL_T)
        if (U.found[i]) atomicOr(&found[i >> 5], 1u << (i & 31));
    __syncthreads();
    const GridView G = unit_grid(U);
    const int nm = search_kf(U.fc, G, U.K2, U.D2, U.n2, U.Tcw, U.K1, U.mp1, U.n1, U.mps, U.mdesc, found, U.th,
                             U.orb_dist, U.check_ori, U.kp2mp, U.score, U.rec, hist, keep);
    if (threadIdx.x == 0) *U.nm = nm;
}

__global__ __launch_bounds__(TL_T) void k_unit_cand(gf::KfdbDev db, const uint8_t* kf_bad, const int32_t* cov_off,
                                                  const int32_t* cov, const int32_t* W, const double* V, int nw,
                                                  uint32_t query, gf_reloc_kf* rkf, int32_t* cands, int32_t* nc) {
    __shared__ CandShared S;
    const int n = reloc_candidates_wave(db, kf_bad, cov_off, cov, W, V, nw, query, rkf, cands, S);
    if (threadIdx.x == 0) *nc = n;
}

}  // namespace

int gf::reloc_candidates(gf_ctx* ctx, const TrackLossArgs& A, hipStream_t s) {
    GF_PROF(ctx, s, "k_reloc_cand");
    GF_LAUNCH(k_reloc_cand, A.B, TL_T, 0, s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf::track_loss(gf_ctx* ctx, const TrackLossArgs& A, hipStream_t s) {
    {
        GF_PROF(ctx, s, "k_track_gate");
        GF_LAUNCH(k_track_gate, A.B, TL_T, 0, s, A);
        GF_HIP(hipGetLastError());
    }
    // a wave of this kernel takes a whole SIMD's registers (its calls into the
    // pose LM and the searches make it compile to the 512-register limit): a
    // small grid, since each workgroup must wait for an idle SIMD beside the
    // other front ends' extraction even when it finds no stream to track
    // (64 workgroups: 0.17 ms per launch in the r05 step; a stream that lost
    // track is walked by one of TL_GRID workgroups)
    GF_PROF(ctx, s, "k_track_loss");
    GF_LAUNCH(k_track_loss, std::min(A.B, TL_GRID), TL_T, 0, s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

// ------------------------------------------------------------ C ABI
namespace {

int unit_frame(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
               UnitArgs& U) {
    GF_CHECK(fi && fi->nlevels >= 1 && fi->nlevels <= 16 && fi->max_x > fi->min_x && fi->max_y > fi->min_y,
             GF_ERR_ARG, "bad frame info");
    GF_CHECK(n2 >= 0 && n2 <= KP_MAX && (n2 == 0 || (kps2 && desc2)), GF_ERR_ARG, "bad frame keypoints");
    U.fc = gf::make_frame_const(fi);
    void *k, *d, *g, *r, *nm;
    int rc;
    const size_t nn = std::max(n2, 1);
    if ((rc = gf::ws_upload(ctx, 0, kps2, sizeof(gf_keypoint) * n2, &k)) ||
        (rc = gf::ws_upload(ctx, 1, desc2, 32 * (size_t)n2, &d)) ||
        (rc = gf::ws_get(ctx, 2, sizeof(int32_t) * gf::grid_ints((int)nn), &g)) ||
        (rc = gf::ws_get(ctx, 3, sizeof(int32_t) * nn, &r)) || (rc = gf::ws_get(ctx, 4, sizeof(int32_t), &nm)))
        return rc;
    U.K2 = (const gf_keypoint*)k;
    U.D2 = (const uint8_t*)d;
    U.n2 = n2;
    U.grid = (int32_t*)g;
    U.rec = (int32_t*)r;
    U.nm = (int32_t*)nm;
    return GF_OK;
}

}  // namespace

extern "C" {

int gf_window_search(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                     const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1, int n1, int window,
                     int min_level, int max_level, float nnratio, int check_ori, int32_t* out, int* nmatches) {
    GF_CHECK(ctx && out && nmatches, GF_ERR_ARG, "null arg");
    GF_CHECK(n1 >= 0 && n1 <= KP_MAX && (n1 == 0 || (kps1 && desc1 && mp1)), GF_ERR_ARG, "bad last frame");
    GF_HIP(hipSetDevice(ctx->device));
    UnitArgs U{};
    int rc = unit_frame(ctx, fi, kps2, desc2, n2, U);
    if (rc) return rc;
    void *k1, *d1, *m1, *o;
    if ((rc = gf::ws_upload(ctx, 5, kps1, sizeof(gf_keypoint) * n1, &k1)) ||
        (rc = gf::ws_upload(ctx, 6, desc1, 32 * (size_t)n1, &d1)) ||
        (rc = gf::ws_upload(ctx, 7, mp1, sizeof(int32_t) * n1, &m1)) ||
        (rc = gf::ws_get(ctx, 8, sizeof(int32_t) * std::max(n2, 1), &o)))
        return rc;
    U.K1 = (const gf_keypoint*)k1;
    U.D1 = (const uint8_t*)d1;
    U.mp1 = (const int32_t*)m1;
    U.n1 = n1;
    U.window = window;
    U.minL = min_level;
    U.maxL = max_level;
    U.nnratio = nnratio;
    U.check_ori = check_ori;
    U.kp2mp = (int32_t*)o;
    hipStream_t s = ctx->stream;
    GF_HIP(hipMemsetAsync(o, 0xff, sizeof(int32_t) * std::max(n2, 1), s));  // claim init for the grid build
    GF_LAUNCH(k_unit_window, 1, TL_T, 0, s, U);
    GF_HIP(hipGetLastError());
    int32_t nm = 0;
    if (n2) GF_HIP(hipMemcpyAsync(out, o, sizeof(int32_t) * n2, hipMemcpyDeviceToHost, s));
    GF_HIP(hipMemcpyAsync(&nm, U.nm, 4, hipMemcpyDeviceToHost, s));
    GF_HIP(hipStreamSynchronize(s));
    *nmatches = nm;
    return GF_OK;
}

int gf_search_frames(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps2, const uint8_t* desc2, int n2,
                     const float* Tcw2, const gf_keypoint* kps1, const uint8_t* desc1, const int32_t* mp1,
                     const float* pos1, int n1, int window, float nnratio, int32_t* kp2mp, int32_t* score,
                     int* nmatches) {
    GF_CHECK(ctx && Tcw2 && nmatches && (n2 == 0 || (kp2mp && score)), GF_ERR_ARG, "null arg");
    GF_CHECK(n1 >= 0 && n1 <= KP_MAX && (n1 == 0 || (kps1 && desc1 && mp1 && pos1)), GF_ERR_ARG, "bad last frame");
    for (int i = 0; i < n2; i++) GF_CHECK(kp2mp[i] < 4096, GF_ERR_UNSUPPORTED, "map indices must be < 4096");
    for (int i = 0; i < n1; i++) GF_CHECK(mp1[i] < 4096, GF_ERR_UNSUPPORTED, "map indices must be < 4096");
    GF_HIP(hipSetDevice(ctx->device));
    UnitArgs U{};
    int rc = unit_frame(ctx, fi, kps2, desc2, n2, U);
    if (rc) return rc;
    void *k1, *d1, *m1, *p1, *km, *sc, *T;
    if ((rc = gf::ws_upload(ctx, 5, kps1, sizeof(gf_keypoint) * n1, &k1)) ||
        (rc = gf::ws_upload(ctx, 6, desc1, 32 * (size_t)n1, &d1)) ||
        (rc = gf::ws_upload(ctx, 7, mp1, sizeof(int32_t) * n1, &m1)) ||
        (rc = gf::ws_upload(ctx, 9, pos1, sizeof(float) * 3 * n1, &p1)) ||
        (rc = gf::ws_upload(ctx, 10, kp2mp, sizeof(int32_t) * n2, &km)) ||
        (rc = gf::ws_upload(ctx, 11, score, sizeof(int32_t) * n2, &sc)) ||
        (rc = gf::ws_upload(ctx, 12, Tcw2, sizeof(float) * 16, &T)))
        return rc;
    U.K1 = (const gf_keypoint*)k1;
    U.D1 = (const uint8_t*)d1;
    U.mp1 = (const int32_t*)m1;
    U.pos1 = (const float*)p1;
    U.n1 = n1;
    U.Tcw = (const float*)T;
    U.window = window;
    U.nnratio = nnratio;
    U.kp2mp = (int32_t*)km;
    U.score = (int32_t*)sc;
    hipStream_t s = ctx->stream;
    GF_LAUNCH(k_unit_frames, 1, TL_T, 0, s, U);
    GF_HIP(hipGetLastError());
    int32_t nm = 0;
    if (n2) {
        GF_HIP(hipMemcpyAsync(kp2mp, km, sizeof(int32_t) * n2, hipMemcpyDeviceToHost, s));
        GF_HIP(hipMemcpyAsync(score, sc, sizeof(int32_t) * n2, hipMemcpyDeviceToHost, s));
    }
    GF_HIP(hipMemcpyAsync(&nm, U.nm, 4, hipMemcpyDeviceToHost, s));
    GF_HIP(hipStreamSynchronize(s));
    *nmatches = nm;
    return GF_OK;
}

int gf_search_kf_projection(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                            const float* Tcw, const gf_keypoint* kf_kps, const int32_t* kf_mp, int nslots,
                            const gf_map_point* mps, const uint8_t* mp_desc, int nmp, const uint8_t* found, float th,
                            int orb_dist, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches) {
    GF_CHECK(ctx && Tcw && nmatches && (n == 0 || (kp2mp && score)), GF_ERR_ARG, "null arg");
    GF_CHECK(nslots >= 0 && (nslots == 0 || (kf_kps && kf_mp)), GF_ERR_ARG, "bad keyframe");
    GF_CHECK(nmp >= 0 && nmp <= 4096 && (nmp == 0 || (mps && mp_desc && found)), GF_ERR_ARG, "bad map points");
    for (int i = 0; i < nslots; i++) GF_CHECK(kf_mp[i] < nmp, GF_ERR_ARG, "keyframe slot out of range");
    for (int i = 0; i < n; i++) GF_CHECK(kp2mp[i] < nmp, GF_ERR_ARG, "frame match out of range");
    GF_HIP(hipSetDevice(ctx->device));
    UnitArgs U{};
    int rc = unit_frame(ctx, fi, kps, desc, n, U);
    if (rc) return rc;
    void *k1, *m1, *mp, *md, *fd, *km, *sc, *T;
    if ((rc = gf::ws_upload(ctx, 5, kf_kps, sizeof(gf_keypoint) * nslots, &k1)) ||
        (rc = gf::ws_upload(ctx, 7, kf_mp, sizeof(int32_t) * nslots, &m1)) ||
        (rc = gf::ws_upload(ctx, 9, mps, sizeof(gf_map_point) * nmp, &mp)) ||
        (rc = gf::ws_upload(ctx, 13, mp_desc, 32 * (size_t)nmp, &md)) ||
        (rc = gf::ws_upload(ctx, 14, found, (size_t)nmp, &fd)) ||
        (rc = gf::ws_upload(ctx, 10, kp2mp, sizeof(int32_t) * n, &km)) ||
        (rc = gf::ws_upload(ctx, 11, score, sizeof(int32_t) * n, &sc)) ||
        (rc = gf::ws_upload(ctx, 12, Tcw, sizeof(float) * 16, &T)))
        return rc;
    U.K1 = (const gf_keypoint*)k1;
    U.mp1 = (const int32_t*)m1;
    U.n1 = nslots;
    U.mps = (const gf_map_point*)mp;
    U.mdesc = (const uint8_t*)md;
    U.found = (const uint8_t*)fd;
    U.Tcw = (const float*)T;
    U.th = th;
    U.orb_dist = orb_dist;
    U.check_ori = check_ori;
    U.kp2mp = (int32_t*)km;
    U.score = (int32_t*)sc;
    hipStream_t s = ctx->stream;
    GF_LAUNCH(k_unit_kf, 1, TL_T, 0, s, U, nmp);
    GF_HIP(hipGetLastError());
    int32_t nm = 0;
    if (n) {
        GF_HIP(hipMemcpyAsync(kp2mp, km, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
        GF_HIP(hipMemcpyAsync(score, sc, sizeof(int32_t) * n, hipMemcpyDeviceToHost, s));
    }
    GF_HIP(hipMemcpyAsync(&nm, U.nm, 4, hipMemcpyDeviceToHost, s));
    GF_HIP(hipStreamSynchronize(s));
    *nmatches = nm;
    return GF_OK;
}

int gf_kfdb_create(gf_ctx* ctx, const gf_keyframe_db* db, gf_kfdb** out) {
    GF_CHECK(ctx && db && out, GF_ERR_ARG, "null arg");
    const int nkf = db->nkf;
    GF_CHECK(nkf >= 0 && nkf <= gf::RL_NC, GF_ERR_UNSUPPORTED, "at most 64 keyframes per database");
    GF_CHECK(nkf == 0 || (db->kp_off && db->bow_off && db->fv_off && db->fv_start), GF_ERR_ARG, "null offsets");
    const int nk = nkf ? db->kp_off[nkf] : 0, nb = nkf ? db->bow_off[nkf] : 0, nn = nkf ? db->fv_off[nkf] : 0;
    const int nf = nkf ? db->fv_start[nn] : 0;
    GF_CHECK(nk >= 0 && nb >= 0 && nn >= 0 && nf >= 0, GF_ERR_ARG, "negative sizes");
    GF_CHECK((nk == 0 || (db->kps && db->desc)) && (nb == 0 || (db->bow_words && db->bow_values)) &&
                 (nn == 0 || db->fv_nodes) && (nf == 0 || db->fv_feats),
             GF_ERR_ARG, "null database arrays");
    for (int k = 0; k < nkf; k++) {
        GF_CHECK(db->kp_off[k] >= 0 && db->kp_off[k] <= db->kp_off[k + 1] && db->kp_off[k + 1] - db->kp_off[k] <= KP_MAX,
                 GF_ERR_ARG, "keypoint offsets must ascend (<= 4096 a keyframe)");
        GF_CHECK(db->bow_off[k] >= 0 && db->bow_off[k] <= db->bow_off[k + 1], GF_ERR_ARG, "BowVector offsets");
        GF_CHECK(db->fv_off[k] >= 0 && db->fv_off[k] <= db->fv_off[k + 1], GF_ERR_ARG, "FeatureVector offsets");
        for (int e = db->bow_off[k] + 1; e < db->bow_off[k + 1]; e++)
            GF_CHECK(db->bow_words[e] > db->bow_words[e - 1], GF_ERR_ARG, "BowVector words must ascend");
        const int nkp = db->kp_off[k + 1] - db->kp_off[k];
        for (int g = db->fv_off[k]; g < db->fv_off[k + 1]; g++) {
            GF_CHECK(db->fv_start[g] >= 0 && db->fv_start[g] <= db->fv_start[g + 1] && db->fv_start[g + 1] <= nf,
                     GF_ERR_ARG, "FeatureVector starts must ascend");
            if (g > db->fv_off[k]) GF_CHECK(db->fv_nodes[g] > db->fv_nodes[g - 1], GF_ERR_ARG, "nodes must ascend");
            for (int x = db->fv_start[g]; x < db->fv_start[g + 1]; x++)
                GF_CHECK(db->fv_feats[x] >= 0 && db->fv_feats[x] < nkp, GF_ERR_ARG, "feature index out of range");
        }
    }
    GF_HIP(hipSetDevice(ctx->device));
    gf_kfdb* d = new gf_kfdb();
    d->device = ctx->device;
    auto up = [&](const void* src, size_t bytes) -> void* {
        void* p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) return nullptr;
        d->allocs.push_back(p);
        if (bytes && hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return p;
    };
    // mvInvertedFile: keyframes per word in insertion (index) order
    std::map<int, std::vector<int>> inv;
    for (int k = 0; k < nkf; k++)
        for (int e = db->bow_off[k]; e < db->bow_off[k + 1]; e++) inv[db->bow_words[e]].push_back(k);
    std::vector<int32_t> iw, io(1, 0), ik;
    for (auto& e : inv) {
        iw.push_back(e.first);
        for (int k : e.second) ik.push_back(k);
        io.push_back((int32_t)ik.size());
    }
    gf::KfdbDev& v = d->dev;
    v.nkf = nkf;
    v.kp_off = (const int32_t*)up(db->kp_off, 4 * (size_t)(nkf + 1));
    v.kps = (const gf_keypoint*)up(db->kps, sizeof(gf_keypoint) * nk);
    v.desc = (const uint8_t*)up(db->desc, 32 * (size_t)nk);
    v.bow_off = (const int32_t*)up(db->bow_off, 4 * (size_t)(nkf + 1));
    v.bow_words = (const int32_t*)up(db->bow_words, 4 * (size_t)nb);
    v.bow_values = (const double*)up(db->bow_values, 8 * (size_t)nb);
    v.fv_off = (const int32_t*)up(db->fv_off, 4 * (size_t)(nkf + 1));
    v.fv_nodes = (const int32_t*)up(db->fv_nodes, 4 * (size_t)nn);
    v.fv_start = (const int32_t*)up(db->fv_start, 4 * (size_t)(nn + 1));
    v.fv_feats = (const int32_t*)up(db->fv_feats, 4 * (size_t)nf);
    v.nw = (int)iw.size();
    v.inv_words = (const int32_t*)up(iw.data(), 4 * iw.size());
    v.inv_off = (const int32_t*)up(io.data(), 4 * io.size());
    v.inv_kf = (const int32_t*)up(ik.data(), 4 * ik.size());
    if (!v.kp_off || !v.kps || !v.desc || !v.bow_off || !v.bow_words || !v.bow_values || !v.fv_off || !v.fv_nodes ||
        !v.fv_start || !v.fv_feats || !v.inv_words || !v.inv_off || !v.inv_kf) {
        gf_kfdb_destroy(d);
        return gf::fail(GF_ERR_HIP, "keyframe database upload");
    }
    *out = d;
    return GF_OK;
}

int gf_kfdb_destroy(gf_kfdb* d) {
    if (!d) return GF_OK;
    (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();
    for (void* p : d->allocs) (void)hipFree(p);
    delete d;
    return GF_OK;
}

int gf_reloc_candidates(gf_ctx* ctx, const int32_t* words, const double* values, int nwords, const gf_keyframe_db* db,
                        const uint8_t* kf_bad, const int32_t* cov_off, const int32_t* cov, uint32_t query,
                        gf_reloc_kf* state, int32_t* cands, int* ncand) {
    GF_CHECK(ctx && db && state && cands && ncand && cov_off && (nwords == 0 || (words && values)), GF_ERR_ARG,
             "null arg");
    GF_CHECK(query != 0, GF_ERR_ARG, "query id 0 is every keyframe's initial mnRelocQuery");
    for (int i = 1; i < nwords; i++) GF_CHECK(words[i] > words[i - 1], GF_ERR_ARG, "frame words must ascend");
    const int nkf = db->nkf;
    const int ncov = nkf ? cov_off[nkf] : 0;
    for (int i = 0; i < ncov; i++) GF_CHECK(cov[i] >= 0 && cov[i] < nkf, GF_ERR_ARG, "bad covisible keyframe");
    gf_kfdb* d = nullptr;
    int rc = gf_kfdb_create(ctx, db, &d);
    if (rc) return rc;
    void *w, *v, *kb, *co, *cv, *st, *cd, *nc;
    std::vector<uint8_t> bad(std::max(nkf, 1), 0);
    if (kf_bad) std::copy(kf_bad, kf_bad + nkf, bad.begin());
    if ((rc = gf::ws_upload(ctx, 0, words, 4 * (size_t)nwords, &w)) ||
        (rc = gf::ws_upload(ctx, 1, values, 8 * (size_t)nwords, &v)) ||
        (rc = gf::ws_upload(ctx, 2, bad.data(), bad.size(), &kb)) ||
        (rc = gf::ws_upload(ctx, 3, cov_off, 4 * (size_t)(nkf + 1), &co)) ||
        (rc = gf::ws_upload(ctx, 4, cov, 4 * (size_t)ncov, &cv)) ||
        (rc = gf::ws_upload(ctx, 5, state, sizeof(gf_reloc_kf) * nkf, &st)) ||
        (rc = gf::ws_get(ctx, 6, 4 * (size_t)gf::RL_NC, &cd)) || (rc = gf::ws_get(ctx, 7, 4, &nc))) {
        gf_kfdb_destroy(d);
        return rc;
    }
    hipStream_t s = ctx->stream;
    GF_LAUNCH(k_unit_cand, 1, TL_T, 0, s, d->dev, (const uint8_t*)kb, (const int32_t*)co, (const int32_t*)cv,
              (const int32_t*)w, (const double*)v, nwords, query, (gf_reloc_kf*)st, (int32_t*)cd, (int32_t*)nc);
    hipError_t e = hipGetLastError();
    int32_t n = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&n, nc, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && nkf) e = hipMemcpyAsync(state, st, sizeof(gf_reloc_kf) * nkf, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(cands, cd, 4 * (size_t)gf::RL_NC, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    gf_kfdb_destroy(d);
    GF_HIP(e);
    *ncand = n;
    return GF_OK;
}

}  // extern "C"

const gf::KfdbDev& gf::kfdb_dev(const gf_kfdb* db) { return db->dev; }
