// Projection matching on gfx950 — SURVEY.md §8a rows E8, M1-M3, M7.
//
// ORBmatcher's projection searches are order dependent: map point k may only
// take keypoints that no earlier map point claimed (F.mvpMapPoints[idx] is
// tested before the distance, ORBmatcher.cc:426-427 / :2136). The kernel
// resolves that sequential semantics exactly, in parallel rounds:
//
//   round: every unresolved query k marks, for each unclaimed candidate
//          keypoint c in its window, minU[c] = min(minU[c], k);
//          a query whose unclaimed candidates all have minU == k has no
//          earlier unresolved competitor, so its sequential outcome is
//          already determined: it walks its candidates in the reference
//          order (grid cells ix-major, iy, keypoint index), takes best /
//          second best exactly as the CPU loop does, and claims.
//
// Queries resolved in the same round have disjoint unclaimed candidate sets,
// the lowest unresolved query is always resolvable, and claims are
// monotone, so the result equals the sequential loop bit for bit. One
// workgroup per frame (frames are independent streams), the 64x48 grid CSR,
// claims and the round state live in LDS.
#include <climits>
#include <cmath>
#include <vector>

#include "common.h"

#include "match_common.h"

namespace {

enum { MODE_PROJECT = 0, MODE_LAST = 1 };

struct MatchArgs {
    int mode;
    // current frame
    const gf_keypoint* kps;
    const uint8_t* desc;
    const int32_t* n;
    int kp_cap;
    // MODE_PROJECT queries
    const gf_mp_view* views;
    const uint8_t* qdesc;
    const int32_t* m;
    int q_cap;
    const int32_t* list;   // MODE_PROJECT: optional query list [F][q_cap] (map indices, in order)
    const int32_t* nlist;  // its length per frame
    // MODE_LAST queries
    const gf_keypoint* last_kps;
    const int32_t* last_kp2mp;
    const uint8_t* last_outlier;
    const float* last_pos;
    const float* Tcw;  // [F][16]
    float th, nnratio;
    const float* th_per;  // MODE_PROJECT: th per frame (null: th)
    int check_ori;
    // in/out
    int32_t* kp2mp;
    int32_t* score;
    int32_t* nmatches;
    int32_t* qres;  // [F][q_cap] scratch: matched kp per query (MODE_LAST)
    int32_t* err;   // [F] round-limit flag
    const struct SeqPre* pre;  // [F][q_cap] MODE_LAST: each query against the starting claims
    int* grid_cs;              // [F][NCELLS + 1] keypoint grid CSR (k_match_seq_pre writes, rescans read)
    int* grid_items;           // [F][kp_cap]
    // SearchByProjection_Budget's clock (list mode, gf_set_budgets; null: none):
    // the visibility pass's timer start per frame, 2 x timeCost_rest in ticks,
    // the clock record and scratch for undoing the claims after the cut
    const unsigned long long* ck_t0;
    const long long* ck_rest2;
    long long* ck_rec;
    long long ck_stride;
    int ck_off;       // offset of the per-point array in a stream's record
    const long long* ck_syn;  // test clock: (base, slope) of the start, then of the points; null: device clock
    int32_t* ck_old;  // [F][q_cap] score a query's claim overwrote
    // candidates the windows list (GetFeaturesInArea sizes), added to
    // ncand[f] (SURVEY §8d B_match's C); null: not counted
    int32_t* ncand;
};


struct Query {
    bool valid;
    float x, y, r;
    int minL, maxL;
    int cx0, cx1, cy0, cy1;  // grid window (empty if cx0 > cx1)
    const uint8_t* d;
    int id;  // value written into kp2mp
};


__device__ Query make_query(const MatchArgs& A, const FrameConst& fc, int f, int k) {
    Query q;
    q.valid = false;
    q.cx0 = 1;
    q.cx1 = 0;
    if (A.mode == MODE_PROJECT) {
        if (A.list) k = A.list[(long long)f * A.q_cap + k];
        const gf_mp_view v = A.views[(long long)f * A.q_cap + k];
        if (!v.in_view) return q;
        const int pl = min(max(v.level, 0), fc.nlevels - 1);
        float r = v.view_cos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
        const float th = A.th_per ? A.th_per[f] : A.th;
        if (th != 1.0) r *= th;
        q.r = r * fc.scales[pl];
        q.x = v.u;
        q.y = v.v;
        q.minL = pl - 1;
        q.maxL = pl;
        q.d = A.qdesc + ((long long)f * A.q_cap + k) * 32;
        q.id = k;
    } else {
        const long long li = (long long)f * A.q_cap + k;
        const int mp = A.last_kp2mp[li];
        if (mp < 0 || A.last_outlier[li]) return q;
        float Pc[3];
        transform3(A.Tcw + 16 * f, A.last_pos + 3 * li, Pc);
        const float invzc = (float)(1.0 / (double)Pc[2]);
        const float u = fc.fx * Pc[0] * invzc + fc.cx;
        const float v = fc.fy * Pc[1] * invzc + fc.cy;
        if (u < fc.min_x || u > fc.max_x) return q;
        if (v < fc.min_y || v > fc.max_y) return q;
        const int oct = A.last_kps[li].octave;
        q.r = A.th * fc.scales[oct];
        q.x = u;
        q.y = v;
        q.minL = oct - 1;
        q.maxL = oct + 1;
        q.d = A.qdesc + li * 32;
        q.id = mp;
    }
    q.valid = true;
    // Frame::GetFeaturesInArea window (Frame.cc:305-327)
    int nMinCellX = max(0, (int)floorf((q.x - fc.min_x - q.r) * fc.invW));
    int nMaxCellX = min(GRID_COLS - 1, (int)ceilf((q.x - fc.min_x + q.r) * fc.invW));
    int nMinCellY = max(0, (int)floorf((q.y - fc.min_y - q.r) * fc.invH));
    int nMaxCellY = min(GRID_ROWS - 1, (int)ceilf((q.y - fc.min_y + q.r) * fc.invH));
    if (nMinCellX >= GRID_COLS || nMaxCellX < 0 || nMinCellY >= GRID_ROWS || nMaxCellY < 0) return q;
    q.cx0 = nMinCellX;
    q.cx1 = nMaxCellX;
    q.cy0 = nMinCellY;
    q.cy1 = nMaxCellY;
    return q;
}


// Rotation-consistency histogram of SearchByProjection(Cur, Last)
// (ORBmatcher.cc:2146-2190, ComputeThreeMaxima :2338-2379) over qres.
__device__ void rotation_filter(const MatchArgs& A, int f, int nq, const gf_keypoint* K, int* claim, int32_t* score,
                                int* s_nm, int* s_hist, int* s_keep, int nthreads) {
    const int tid = threadIdx.x;
        const float factor = 1.0f / HISTO_LENGTH;
        for (int k = tid; k < nq; k += nthreads) {
            const int j = A.qres[(long long)f * A.q_cap + k];
            if (j < 0) continue;
            float rot = A.last_kps[(long long)f * A.q_cap + k].angle - K[j].angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            atomicAdd(&s_hist[bin], 1);
        }
        __syncthreads();
        if (tid == 0) {
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
        for (int k = tid; k < nq; k += nthreads) {
            const int j = A.qres[(long long)f * A.q_cap + k];
            if (j < 0) continue;
            float rot = A.last_kps[(long long)f * A.q_cap + k].angle - K[j].angle;
            if (rot < 0.0) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == HISTO_LENGTH) bin = 0;
            if (bin == s_keep[0] || bin == s_keep[1] || bin == s_keep[2]) continue;
            claim[j] = -1;
            score[j] = 999;
            atomicSub(s_nm, 1);
        }
        __syncthreads();
}

// k_match's LDS is sized by the front end's capacities (kp_cap keypoints,
// q_cap queries), not by the KP_MAX / Q_MAX maxima, so a workgroup fits
// beside other kernels' workgroups on a CU. With MATCH_STAGE it also stages
// the frame's keypoint positions / octaves (float4) and descriptors (48 B a
// keypoint; the candidate loops then read no global memory) when that stays
// within MATCH_STAGE_LDS. Off by default since r04: in the 4-group step the
// staged workgroup's extra ~60 KB of LDS keeps the other groups' extraction
// workgroups off its CU (A/B, one box: 101.2k vs 100.1k / 100.3k frames/s,
// profiles/r04/ab4_*.json).
#ifndef MATCH_STAGE
#define MATCH_STAGE 0
#endif
#define MATCH_STAGE_LDS (96 * 1024)
// candidates whose loads k_match issues together in its window walks
#ifndef MATCH_MB
#define MATCH_MB 2
#endif
// and their descriptors too (more registers a thread)
// the thread's first query kept in registers over the claim rounds
#ifndef MATCH_QCACHE
#define MATCH_QCACHE 0
#endif
#ifndef MATCH_DESC_AHEAD
#define MATCH_DESC_AHEAD 0
#endif
__host__ __device__ __forceinline__ size_t match_base_lds(int kp_cap, int q_cap) {
    const int kc = kp_cap < KP_MAX ? kp_cap : KP_MAX, qc = q_cap < Q_MAX ? q_cap : Q_MAX;
    return (sizeof(int) * (NCELLS + 1 + 3 * (size_t)kc) + (size_t)qc + 15) & ~(size_t)15;
}
__host__ __device__ __forceinline__ bool match_stage(int kp_cap, int q_cap) {
    return MATCH_STAGE && match_base_lds(kp_cap, q_cap) + 48 * (size_t)kp_cap <= MATCH_STAGE_LDS;
}

__global__ __launch_bounds__(MATCH_THREADS) void k_match(MatchArgs A, FrameConst fc) {
    gfd::track_prio();
    extern __shared__ __align__(16) int lds[];
    const int kc = min(A.kp_cap, KP_MAX);
    int* cell_start = lds;                  // NCELLS + 1
    int* items = cell_start + NCELLS + 1;   // kc
    int* claim = items + kc;                // kc
    int* minU = claim + kc;                 // kc
    uint8_t* done = (uint8_t*)(minU + kc);  // min(q_cap, Q_MAX)
    __shared__ int s_any, s_nm, s_hist[HISTO_LENGTH], s_keep[3], s_cand;

    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(A.n[f], kc);
    int nq = min(A.list ? A.nlist[f] : A.m[f], min(A.q_cap, Q_MAX));
    // SearchByProjection_Budget (ORBmatcher.cc:281-288, 366-371): the budget
    // left after the visibility pass; none left: return at once
    const bool clocked = A.ck_t0 != nullptr;
    __shared__ unsigned long long s_now0;
    __shared__ long long s_constr2;
    __shared__ int s_cut;
    long long* rec = clocked ? A.ck_rec + (long long)f * A.ck_stride : nullptr;
    if (clocked) {
        if (tid == 0) {
            const unsigned long long now0 = __builtin_amdgcn_s_memrealtime();
            const long long so_far = A.ck_syn ? A.ck_syn[0] : (long long)(now0 - A.ck_t0[f]);
            s_now0 = now0;
            s_constr2 = A.ck_rest2[f] - 2 * so_far;
            s_cut = INT_MAX;
            rec[GF_CK_SA_SOFAR] = so_far;
            rec[GF_CK_BUDGET_CUT] = -1;
        }
        __syncthreads();
        if (s_constr2 <= 0) nq = 0;
    }
    const gf_keypoint* K = A.kps + (long long)f * A.kp_cap;
    const uint8_t* D = A.desc + (long long)f * A.kp_cap * 32;
    int32_t* kp2mp = A.kp2mp + (long long)f * A.kp_cap;
    int32_t* score = A.score + (long long)f * A.kp_cap;
    const bool stg = match_stage(A.kp_cap, A.q_cap);
    float4* X = reinterpret_cast<float4*>(reinterpret_cast<uint8_t*>(lds) + match_base_lds(A.kp_cap, A.q_cap));
    uint8_t* Ds = reinterpret_cast<uint8_t*>(X + A.kp_cap);
    if (stg) {
        for (int i = tid; i < n; i += MATCH_THREADS) {
            const gf_keypoint kp = K[i];
            X[i] = make_float4(kp.x, kp.y, __int_as_float(kp.octave), 0.f);
        }
        for (int i = tid; i < 2 * n; i += MATCH_THREADS)
            reinterpret_cast<uint4*>(Ds)[i] = reinterpret_cast<const uint4*>(D)[i];
    }
    const uint8_t* DD = stg ? (const uint8_t*)Ds : D;
    auto cand = [&](int idx, float& x, float& y, int& oct) {
        if (stg) {
            const float4 v = X[idx];
            x = v.x;
            y = v.y;
            oct = __float_as_int(v.z);
        } else {
            const gf_keypoint kp = K[idx];
            x = kp.x;
            y = kp.y;
            oct = kp.octave;
        }
    };

    if (tid == 0) {
        s_nm = 0;
        s_cand = 0;
        for (int b = 0; b < HISTO_LENGTH; b++) s_hist[b] = 0;
    }
    build_grid(fc, K, n, kp2mp, cell_start, items, claim, minU, MATCH_THREADS);
    for (int k = tid; k < nq; k += MATCH_THREADS) done[k] = 0;
    __syncthreads();

    // ---- claim-resolution rounds
#if MATCH_QCACHE
    // the thread's first query, kept in registers over the rounds
    Query q0;
    q0.valid = false;
    q0.cx0 = 1;
    q0.cx1 = 0;
    if (tid < nq) q0 = make_query(A, fc, f, tid);
#define MATCH_Q(k) ((k) == tid ? q0 : make_query(A, fc, f, (k)))
#else
#define MATCH_Q(k) make_query(A, fc, f, (k))
#endif
    int rounds = 0;
    while (true) {
        for (int i = tid; i < n; i += MATCH_THREADS) minU[i] = INT_MAX;
        if (tid == 0) s_any = 0;
        __syncthreads();
        for (int k = tid; k < nq; k += MATCH_THREADS) {
            if (clocked && rounds == 0)  // per point, from the matcher's start
                rec[A.ck_off + k] = gfd::ck_elapsed(s_now0, A.ck_syn ? A.ck_syn + 2 : nullptr, k);
            if (done[k]) continue;
            const Query q = MATCH_Q(k);
            if (!q.valid) continue;
            for (int ix = q.cx0; ix <= q.cx1; ix++) {
                const int s = cell_start[ix * GRID_ROWS + q.cy0], e = cell_start[ix * GRID_ROWS + q.cy1 + 1];
                for (int t0 = s; t0 < e; t0 += MATCH_MB) {
                    // MATCH_MB candidates' loads issued together (clamped
                    // indices, unconditional), then tested in order
                    int id[MATCH_MB], ko[MATCH_MB];
                    float kx[MATCH_MB], ky[MATCH_MB];
#pragma unroll
                    for (int u = 0; u < MATCH_MB; u++) id[u] = items[min(t0 + u, e - 1)];
#pragma unroll
                    for (int u = 0; u < MATCH_MB; u++) cand(id[u], kx[u], ky[u], ko[u]);
#pragma unroll
                    for (int u = 0; u < MATCH_MB; u++) {
                        if (t0 + u >= e || claim[id[u]] >= 0) continue;
                        if (!level_ok(ko[u], q.minL, q.maxL)) continue;
                        if (fabsf(kx[u] - q.x) > q.r || fabsf(ky[u] - q.y) > q.r) continue;
                        atomicMin(&minU[id[u]], k);
                    }
                }
            }
        }
        __syncthreads();
        for (int k = tid; k < nq; k += MATCH_THREADS) {
            if (done[k]) continue;
            const Query q = MATCH_Q(k);
            int bestDist = INT_MAX, bestLevel = -1, bestDist2 = INT_MAX, bestLevel2 = -1, bestIdx = -1;
            bool ok = true, near = false;
            int ncq = 0;
            if (q.valid) {
                const uint4 qa = reinterpret_cast<const uint4*>(q.d)[0], qb = reinterpret_cast<const uint4*>(q.d)[1];
                for (int ix = q.cx0; ix <= q.cx1 && ok; ix++) {
                    const int s = cell_start[ix * GRID_ROWS + q.cy0], e = cell_start[ix * GRID_ROWS + q.cy1 + 1];
                    for (int t0 = s; t0 < e && ok; t0 += MATCH_MB) {
                        // positions and descriptors of MATCH_MB candidates
                        // loaded together, then walked in the reference order
                        int id[MATCH_MB], ko[MATCH_MB];
                        float kx[MATCH_MB], ky[MATCH_MB];
#if MATCH_DESC_AHEAD
                        uint4 da[MATCH_MB], db[MATCH_MB];
#endif
#pragma unroll
                        for (int u = 0; u < MATCH_MB; u++) id[u] = items[min(t0 + u, e - 1)];
#pragma unroll
                        for (int u = 0; u < MATCH_MB; u++) {
                            cand(id[u], kx[u], ky[u], ko[u]);
#if MATCH_DESC_AHEAD
                            const uint4* pd = reinterpret_cast<const uint4*>(DD + (long long)id[u] * 32);
                            da[u] = pd[0];
                            db[u] = pd[1];
#endif
                        }
#pragma unroll
                        for (int u = 0; u < MATCH_MB; u++) {
                            if (t0 + u >= e || !ok) continue;
                            if (!level_ok(ko[u], q.minL, q.maxL)) continue;
                            if (fabsf(kx[u] - q.x) > q.r || fabsf(ky[u] - q.y) > q.r) continue;
                            near = true;  // GetFeaturesInArea lists it (claimed or not)
                            ncq++;
                            if (__hip_atomic_load(&claim[id[u]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= 0)
                                continue;
                            if (minU[id[u]] != k) {
                                ok = false;
                                continue;
                            }
#if MATCH_DESC_AHEAD
                            const int dist = hamming_regs(qa, qb, da[u], db[u]);
#else
                            const uint4* pd = reinterpret_cast<const uint4*>(DD + (long long)id[u] * 32);
                            const int dist = hamming_regs(qa, qb, pd[0], pd[1]);
#endif
                            if (dist < bestDist) {
                                bestDist2 = bestDist;
                                bestDist = dist;
                                bestLevel2 = bestLevel;
                                bestLevel = ko[u];
                                bestIdx = id[u];
                            } else if (dist < bestDist2) {
                                bestLevel2 = ko[u];
                                bestDist2 = dist;
                            }
                        }
                    }
                }
            }
            if (!ok) {
                s_any = 1;
                continue;
            }
            if (A.ncand && ncq && !clocked) atomicAdd(&s_cand, ncq);
            done[k] = 1;
            int res = -1;
            bool reject = false;
            if (q.valid && bestDist <= TH_HIGH) {
                reject = A.mode == MODE_PROJECT && bestLevel == bestLevel2 &&
                         (float)bestDist > A.nnratio * (float)bestDist2;
                if (!reject) {
                    __hip_atomic_store(&claim[bestIdx], q.id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (clocked) A.ck_old[(long long)f * A.q_cap + k] = score[bestIdx];
                    score[bestIdx] = bestDist;
                    atomicAdd(&s_nm, 1);
                    res = bestIdx;
                }
            }
            if (A.mode == MODE_LAST || clocked) A.qres[(long long)f * A.q_cap + k] = res;
            // the points that reach SearchByProjection_Budget's clock check
            // (ORBmatcher.cc:366-371): in view, a non-empty area, not rejected
            // by the ratio test
            if (clocked && q.valid && near && !reject) done[k] = 2;
        }
        __syncthreads();
        if (!s_any) break;
        if (++rounds > nq + 2) {
            if (tid == 0) A.err[f] = 1;
            break;
        }
        __syncthreads();
    }

    if (clocked) {
        // the break: the first checked point whose elapsed >= the budget left;
        // later points' claims are undone (they never ran; claims of earlier
        // points do not depend on them)
        __syncthreads();
        for (int k = tid; k < nq; k += MATCH_THREADS)
            if (done[k] == 2 && 2 * rec[A.ck_off + k] >= s_constr2) atomicMin(&s_cut, k);
        __syncthreads();
        const int c = s_cut;
        if (c != INT_MAX) {
            for (int k = c + 1 + tid; k < nq; k += MATCH_THREADS) {
                const int r = A.qres[(long long)f * A.q_cap + k];
                if (r < 0) continue;
                claim[r] = -1;
                score[r] = A.ck_old[(long long)f * A.q_cap + k];
                atomicSub(&s_nm, 1);
            }
            if (tid == 0) rec[GF_CK_BUDGET_CUT] = c;
        }
        if (A.ncand) {  // the candidates of the points that ran (the list up to the break)
            const int nrun = c == INT_MAX ? nq : c + 1;
            for (int k = tid; k < nrun; k += MATCH_THREADS) {
                const Query q = make_query(A, fc, f, k);
                if (!q.valid) continue;
                int ncq = 0;
                for (int ix = q.cx0; ix <= q.cx1; ix++) {
                    const int s0 = cell_start[ix * GRID_ROWS + q.cy0], e0 = cell_start[ix * GRID_ROWS + q.cy1 + 1];
                    for (int t = s0; t < e0; t++) {
                        float kx, ky;
                        int ko;
                        cand(items[t], kx, ky, ko);
                        ncq += level_ok(ko, q.minL, q.maxL) && fabsf(kx - q.x) <= q.r && fabsf(ky - q.y) <= q.r;
                    }
                }
                if (ncq) atomicAdd(&s_cand, ncq);
            }
        }
        __syncthreads();
    }
    // ---- rotation consistency (ORBmatcher.cc:2146-2190)
    if (A.mode == MODE_LAST && A.check_ori) rotation_filter(A, f, nq, K, claim, score, &s_nm, s_hist, s_keep, MATCH_THREADS);
    for (int i = tid; i < n; i += MATCH_THREADS) kp2mp[i] = claim[i];
    if (tid == 0) {
        A.nmatches[f] = s_nm;
        if (A.ncand) A.ncand[f] += s_cand;  // launches on one stream: no race
    }
}

// ---- Per-query precompute for the wave-sequential matcher (SearchByProjection
// (Cur, Last), best candidate only). Every valid query runs its window scan at
// once (one thread each) against the frame's starting claims and keeps its
// four smallest (distance, candidate order) candidates. Claims only remove
// keypoints, so in the ordered pass a query's outcome is the first of its four
// still unclaimed (ties already resolved by candidate order, as the
// sequential `dist < bestDist` loop does); only a query that lost all four
// while its window holds more candidates scans again.
struct SeqPre {
    int32_t id;
    int16_t h[4];   // the four smallest (distance, candidate order) candidates, ascending; -1 = none
    int16_t d[4];   // their distances
    int16_t ncand;  // candidates in the window, capped at 5
    int16_t pad;
};

#ifndef SEQ_PRE_THREADS
#define SEQ_PRE_THREADS 1024
#endif
// descriptors staged in LDS up to this capacity; 0 since r04 (A/B in the
// 4-group step: 103.0k vs 101.8k / 101.4k frames/s with k_onepoint_pre's
// likewise: the smaller workgroups leave room for the other groups'
// extraction, the descriptor reads hit L2; profiles/r04/ab5_*.json)
#ifndef SEQ_PRE_DESC_MAX
#define SEQ_PRE_DESC_MAX 0
#endif
#define SEQ_PRE_G 4  // lanes per query
#ifndef SEQ_PRE_MB
#define SEQ_PRE_MB 1  // candidates a lane loads together (2: 81 VGPRs, no faster in the step)
#endif
__global__ __launch_bounds__(SEQ_PRE_THREADS) void k_match_seq_pre(MatchArgs A, FrameConst fc,
                                                                   SeqPre* __restrict__ out) {
    gfd::track_prio();
    extern __shared__ __align__(16) uint8_t smem[];
    const int f = blockIdx.x, tid = threadIdx.x;
    const int n = min(A.n[f], KP_MAX);
    const int nq = min(A.m[f], Q_MAX);
    float4* X = (float4*)smem;                  // kp_cap: x, y, octave
    int* cell_start = (int*)(X + A.kp_cap);     // NCELLS + 1
    int* items = cell_start + NCELLS + 1;       // kp_cap
    int* claim = items + A.kp_cap;              // kp_cap
    int* scratch = claim + A.kp_cap;            // kp_cap
    uint8_t* Ds = (uint8_t*)(scratch + A.kp_cap);  // 32 x kp_cap when kp_cap <= SEQ_PRE_DESC_MAX
    const gf_keypoint* K = A.kps + (long long)f * A.kp_cap;
    const uint8_t* D = A.desc + (long long)f * A.kp_cap * 32;
    const bool dl = A.kp_cap <= SEQ_PRE_DESC_MAX;
    for (int i = tid; i < n; i += SEQ_PRE_THREADS) {
        const gf_keypoint kp = K[i];
        X[i] = make_float4(kp.x, kp.y, __int_as_float(kp.octave), 0.f);
    }
    if (dl)
        for (int i = tid; i < 2 * n; i += SEQ_PRE_THREADS)
            reinterpret_cast<uint4*>(Ds)[i] = reinterpret_cast<const uint4*>(D)[i];
    build_grid(fc, K, n, A.kp2mp + (long long)f * A.kp_cap, cell_start, items, claim, scratch, SEQ_PRE_THREADS);
    for (int c = tid; c < NCELLS + 1; c += SEQ_PRE_THREADS) A.grid_cs[(long long)f * (NCELLS + 1) + c] = cell_start[c];
    for (int i = tid; i < n; i += SEQ_PRE_THREADS) A.grid_items[(long long)f * A.kp_cap + i] = items[i];
    const uint8_t* DD = dl ? (const uint8_t*)Ds : D;
    // SEQ_PRE_G lanes per query: lane g of the group takes candidates
    // g, g + G, ... of the window (ix-major, then the CSR: the reference's
    // order t) and keeps its four smallest (distance, t); a butterfly over the
    // group merges them, so the four smallest over the window come out with
    // the sequential loop's tie order.
    const int g = tid & (SEQ_PRE_G - 1);
    constexpr unsigned long long NONE = ~0ull;
    __shared__ int s_cand;
    if (tid == 0) s_cand = 0;
    __syncthreads();
    int na = 0;  // this lane's area candidates (GetFeaturesInArea), for B_match's C
    for (int k0 = 0; k0 < nq; k0 += SEQ_PRE_THREADS / SEQ_PRE_G) {
        const int k = k0 + tid / SEQ_PRE_G;
        const bool live = k < nq;
        Query q;
        if (live) q = make_query(A, fc, f, k);
        unsigned long long key[4] = {NONE, NONE, NONE, NONE};
        int nc = 0;
        if (live && q.valid) {
            const uint4 qa = reinterpret_cast<const uint4*>(q.d)[0], qb = reinterpret_cast<const uint4*>(q.d)[1];
            int t0 = 0;  // candidate order of the column's first item
            for (int ix = q.cx0; ix <= q.cx1; ix++) {
                const int s0 = cell_start[ix * GRID_ROWS + q.cy0], s1 = cell_start[ix * GRID_ROWS + q.cy1 + 1];
                for (int tb = s0 + g; tb < s1; tb += SEQ_PRE_G * SEQ_PRE_MB) {
                    // SEQ_PRE_MB of this lane's candidates: positions and
                    // descriptors loaded together (clamped, unconditional)
                    int id[SEQ_PRE_MB];
                    float4 kq[SEQ_PRE_MB];
                    uint4 da[SEQ_PRE_MB], db[SEQ_PRE_MB];
#pragma unroll
                    for (int u = 0; u < SEQ_PRE_MB; u++) id[u] = items[min(tb + u * SEQ_PRE_G, s1 - 1)];
#pragma unroll
                    for (int u = 0; u < SEQ_PRE_MB; u++) {
                        kq[u] = X[id[u]];
                        const uint4* pd = reinterpret_cast<const uint4*>(DD + (long long)id[u] * 32);
                        da[u] = pd[0];
                        db[u] = pd[1];
                    }
#pragma unroll
                    for (int u = 0; u < SEQ_PRE_MB; u++) {
                        const int t = tb + u * SEQ_PRE_G, idx = id[u];
                        if (t >= s1) continue;
                        const float4 kp = kq[u];
                        const int oct = __float_as_int(kp.z);
                        if (!level_ok(oct, q.minL, q.maxL) || fabsf(kp.x - q.x) > q.r || fabsf(kp.y - q.y) > q.r)
                            continue;
                        na++;
                        if (claim[idx] >= 0) continue;
                        const int dist = hamming_regs(qa, qb, da[u], db[u]);
                        nc++;
                        const unsigned long long kk = ((unsigned long long)dist << 48) |
                                                      ((unsigned long long)(t0 + t - s0) << 16) | (unsigned)idx;
                        if (kk < key[3]) {
                            key[3] = kk;
                            if (key[3] < key[2]) { const unsigned long long x = key[2]; key[2] = key[3]; key[3] = x; }
                            if (key[2] < key[1]) { const unsigned long long x = key[1]; key[1] = key[2]; key[2] = x; }
                            if (key[1] < key[0]) { const unsigned long long x = key[0]; key[0] = key[1]; key[1] = x; }
                        }
                    }
                }
                t0 += s1 - s0;
            }
        }
#pragma unroll
        for (int o = 1; o < SEQ_PRE_G; o <<= 1) {
            unsigned long long p[4];
#pragma unroll
            for (int j = 0; j < 4; j++) p[j] = __shfl_xor(key[j], o, 64);
            nc += __shfl_xor(nc, o, 64);
            // the four smallest of two ascending lists, ascending: a bitonic
            // merge with fixed indices (min of one list against the other
            // reversed, then a two-stage sort), so the lists stay in registers
            // (a data-dependent merge index put them in scratch memory). Keys
            // are distinct (they carry the candidate order), so the result is
            // the merge's.
#pragma unroll
            for (int j = 0; j < 4; j++) key[j] = key[j] < p[3 - j] ? key[j] : p[3 - j];
            auto cx = [](unsigned long long& x, unsigned long long& y) {
                const unsigned long long lo = x < y ? x : y, hi = x < y ? y : x;
                x = lo;
                y = hi;
            };
            cx(key[0], key[2]);
            cx(key[1], key[3]);
            cx(key[0], key[1]);
            cx(key[2], key[3]);
        }
        if (live && g == 0) {
            SeqPre r;
            r.id = q.id;
            r.pad = 0;
            for (int j = 0; j < 4; j++) {
                const bool on = q.valid && key[j] != NONE;
                r.h[j] = on ? (int16_t)(key[j] & 0xffff) : (int16_t)-1;
                r.d[j] = on ? (int16_t)(key[j] >> 48) : (int16_t)0;
            }
            r.ncand = q.valid ? (int16_t)min(nc, 5) : (int16_t)0;
            out[(long long)f * A.q_cap + k] = r;
        }
    }
    if (A.ncand) {
        na = gfd::warp_sum(na);
        if ((tid & 63) == 0 && na) atomicAdd(&s_cand, na);
        __syncthreads();
        if (tid == 0) A.ncand[f] += s_cand;
    }
}

size_t seq_pre_lds_bytes(int kp_cap) {
    return 16 * (size_t)kp_cap + sizeof(int) * (NCELLS + 1 + 3 * (size_t)kp_cap) +
           (kp_cap <= SEQ_PRE_DESC_MAX ? 32 * (size_t)kp_cap : 0);
}

// ---- Wave-sequential variant for few, wide queries (SearchByProjection(Cur,
// Last, th), th = 15 px x scale): the queries run in the reference order, one
// after the other, and each query's candidate window is scanned by the 64
// lanes of one wave. Each lane keeps the two smallest (distance, candidate
// order) pairs of its candidates; a butterfly merge gives the global best
// and second best, which is exactly what the sequential `dist < bestDist /
// dist < bestDist2` loop keeps (ties go to the earlier candidate).
constexpr int SEQ_THREADS = 64;

__device__ __forceinline__ void top2_insert(unsigned long long key, unsigned long long& k1, unsigned long long& k2) {
    if (key < k1) {
        k2 = k1;
        k1 = key;
    } else if (key < k2) {
        k2 = key;
    }
}

__global__ __launch_bounds__(SEQ_THREADS) void k_match_seq(MatchArgs A, FrameConst fc) {
    gfd::track_prio();
    extern __shared__ __align__(16) int lds[];
    // everything the ordered loop touches lives in LDS, so its per-query
    // barrier waits on LDS only (global stores would be drained every query)
    int* claim = lds;                            // kp_cap
    SeqPre* spre = (SeqPre*)(claim + A.kp_cap);  // q_cap: the precomputed outcomes, staged once
    int16_t* sdist = (int16_t*)(spre + A.q_cap); // kp_cap: score of each claim made here
    int16_t* sres = sdist + A.kp_cap;            // q_cap: matched keypoint per query (-1 none)
    int16_t* qidx = sres + A.q_cap;              // q_cap: query index of each staged outcome
    int* mk = (int*)(((uintptr_t)(qidx + A.q_cap) + 15) & ~(uintptr_t)15);  // kp_cap: first claiming lane of a batch
    __shared__ int s_nm, s_hist[HISTO_LENGTH], s_keep[3];

    const int f = blockIdx.x, lane = threadIdx.x;
    const int n = min(A.n[f], A.kp_cap);
    const int nq = min(A.m[f], A.q_cap);
    // the keypoint grid comes from k_match_seq_pre (HBM; only rescans read it)
    const int* cell_start = A.grid_cs + (long long)f * (NCELLS + 1);
    const int* items = A.grid_items + (long long)f * A.kp_cap;
    const gf_keypoint* K = A.kps + (long long)f * A.kp_cap;
    const uint8_t* D = A.desc + (long long)f * A.kp_cap * 32;
    int32_t* kp2mp = A.kp2mp + (long long)f * A.kp_cap;
    int32_t* score = A.score + (long long)f * A.kp_cap;
    if (lane == 0) {
        s_nm = 0;
        for (int b = 0; b < HISTO_LENGTH; b++) s_hist[b] = 0;
    }
    for (int i = lane; i < n; i += SEQ_THREADS) {
        claim[i] = kp2mp[i];
        sdist[i] = -1;
    }
    // the queries with candidates, in the reference order (the others match
    // nothing); their precomputed outcomes staged in LDS
    int nvalid = 0;
    for (int base = 0; base < nq; base += SEQ_THREADS) {
        const int k = base + lane;
        SeqPre pr;
        bool on = false;
        if (k < nq) {
            pr = A.pre[(long long)f * A.q_cap + k];
            on = pr.ncand > 0;
            sres[k] = -1;
        }
        const unsigned long long m = __ballot(on);
        if (on) {
            pr.pad = 0;
            spre[nvalid + __popcll(m & ((1ull << lane) - 1ull))] = pr;
            qidx[nvalid + __popcll(m & ((1ull << lane) - 1ull))] = (int16_t)k;
        }
        nvalid += __popcll(m);
    }
    __syncthreads();

    const unsigned long long NONE = ~0ull;
    // Queries in batches of 64, one per lane, against the claims at the
    // batch start. A query's outcome can only change when an earlier query
    // of its batch claims the keypoint it picked (claims only remove
    // candidates, and its earlier candidates were already claimed), so the
    // outcomes up to the first such collision — or the first query that must
    // rescan its window — are exactly the sequential ones and are committed
    // together; that query then runs alone (rescan) or heads the next batch.
    for (int i = lane; i < n; i += SEQ_THREADS) mk[i] = INT_MAX;
    __syncthreads();
    int qi0 = 0;
    while (qi0 < nvalid) {
        const int qi = qi0 + lane;
        const bool in = qi < nvalid;
        int k = 0, pick = -1, res = -1, id = 0;
        int16_t dres = 0;
        bool rescan = false;
        if (in) {
            const SeqPre pr = spre[qi];
            k = qidx[qi];
            id = pr.id;
            // j = the first of the four precomputed candidates that is absent or
            // still unclaimed (4: all claimed). Fixed indices throughout: a
            // data-dependent index into the record put it in scratch memory.
            const int h0 = pr.h[0], h1 = pr.h[1], h2 = pr.h[2], h3 = pr.h[3];
            const bool c0 = h0 >= 0 && claim[max(h0, 0)] >= 0, c1 = h1 >= 0 && claim[max(h1, 0)] >= 0;
            const bool c2 = h2 >= 0 && claim[max(h2, 0)] >= 0, c3 = h3 >= 0 && claim[max(h3, 0)] >= 0;
            const int j = !c0 ? 0 : !c1 ? 1 : !c2 ? 2 : !c3 ? 3 : 4;
            const int hj = j == 0 ? h0 : j == 1 ? h1 : j == 2 ? h2 : j == 3 ? h3 : -1;
            const int dj = j == 0 ? pr.d[0] : j == 1 ? pr.d[1] : j == 2 ? pr.d[2] : j == 3 ? pr.d[3] : 0;
            const bool known = (j < 4 && hj >= 0) || j >= pr.ncand;
            rescan = !known;
            if (known && j < 4 && hj >= 0) {
                pick = hj;
                if (j < pr.ncand && dj <= TH_HIGH) {
                    res = pick;
                    dres = (int16_t)dj;
                }
            }
            if (res >= 0) atomicMin(&mk[res], lane);
        }
        __syncthreads();
        const bool unsafe = in && (rescan || (pick >= 0 && mk[pick] < lane));
        const unsigned long long ub = __ballot(unsafe);
        const int stop = ub ? __ffsll((long long)ub) - 1 : SEQ_THREADS;  // first lane not committed
        const bool commit = in && lane < stop && res >= 0;
        __syncthreads();  // every lane has read mk before it is reset
        if (commit) {
            claim[res] = id;
            sdist[res] = dres;
            sres[k] = (int16_t)res;
        }
        if (res >= 0) mk[res] = INT_MAX;
        const unsigned long long cb = __ballot(commit);
        if (lane == 0) s_nm += __popcll(cb);
        __syncthreads();
        if (stop >= SEQ_THREADS || qi0 + stop >= nvalid) {
            qi0 += SEQ_THREADS;
            continue;
        }
        const bool rs = (ub >> stop) & 1ull ? __shfl(rescan ? 1 : 0, stop, 64) != 0 : false;
        if (!rs) {  // a collision: the query heads the next batch
            qi0 += stop;
            continue;
        }
        // the query at `stop` lost its four precomputed candidates: rescan its window
        k = qidx[qi0 + stop];
        qi0 += stop + 1;
        {
        const Query q = make_query(A, fc, f, k);
        unsigned long long k1 = NONE, k2 = NONE;
        // walk the window's columns; candidate order t runs ix-major, then the CSR
        int col = q.cx0, colStart = 0;
        int cs = cell_start[col * GRID_ROWS + q.cy0], ce = cell_start[col * GRID_ROWS + q.cy1 + 1];
        int t = lane;
        while (col <= q.cx1) {
            if (t - colStart >= ce - cs) {  // next column
                colStart += ce - cs;
                col++;
                if (col > q.cx1) break;
                cs = cell_start[col * GRID_ROWS + q.cy0];
                ce = cell_start[col * GRID_ROWS + q.cy1 + 1];
                continue;
            }
            const int idx = items[cs + (t - colStart)];
            const gf_keypoint kp = K[idx];
            if (level_ok(kp.octave, q.minL, q.maxL) && !(fabsf(kp.x - q.x) > q.r || fabsf(kp.y - q.y) > q.r) &&
                claim[idx] < 0) {
                const int dist = hamming32(q.d, D + (long long)idx * 32);
                top2_insert(((unsigned long long)dist << 40) | ((unsigned long long)t << 8) |
                                (unsigned long long)(kp.octave & 0xff),
                            k1, k2);
            }
            t += SEQ_THREADS;
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long o1 = __shfl_xor(k1, o, 64), o2 = __shfl_xor(k2, o, 64);
            top2_insert(o1, k1, k2);
            top2_insert(o2, k1, k2);
        }
        if (lane == 0 && k1 != NONE) {
            const int bestDist = (int)(k1 >> 40);
            const int bestLevel = (int)(k1 & 0xff);
            const int bestDist2 = k2 == NONE ? INT_MAX : (int)(k2 >> 40);
            const int bestLevel2 = k2 == NONE ? -1 : (int)(k2 & 0xff);
            if (bestDist <= TH_HIGH) {
                const bool reject = A.mode == MODE_PROJECT && bestLevel == bestLevel2 &&
                                    (float)bestDist > A.nnratio * (float)bestDist2;
                if (!reject) {
                    // candidate order -> keypoint index
                    int tt = (int)((k1 >> 8) & 0xffffffffull), c = q.cx0;
                    for (;; c++) {
                        const int len = cell_start[c * GRID_ROWS + q.cy1 + 1] - cell_start[c * GRID_ROWS + q.cy0];
                        if (tt < len) break;
                        tt -= len;
                    }
                    const int bestIdx = items[cell_start[c * GRID_ROWS + q.cy0] + tt];
                    claim[bestIdx] = q.id;
                    sdist[bestIdx] = (int16_t)bestDist;
                    s_nm++;
                    sres[k] = (int16_t)bestIdx;
                }
            }
        }
        }
        __syncthreads();
    }
    for (int i = lane; i < n; i += SEQ_THREADS)
        if (sdist[i] >= 0) score[i] = sdist[i];
    for (int k = lane; k < nq; k += SEQ_THREADS) A.qres[(long long)f * A.q_cap + k] = sres[k];
    __syncthreads();
    if (A.mode == MODE_LAST && A.check_ori) rotation_filter(A, f, nq, K, claim, score, &s_nm, s_hist, s_keep, SEQ_THREADS);
    for (int i = lane; i < n; i += SEQ_THREADS) kp2mp[i] = claim[i];
    if (lane == 0) A.nmatches[f] = s_nm;
}

size_t seq_lds_bytes(int kp_cap, int q_cap) {
    return sizeof(int) * (size_t)kp_cap + sizeof(SeqPre) * (size_t)q_cap + 2 * ((size_t)kp_cap + 2 * q_cap) + 16 +
           sizeof(int) * (size_t)kp_cap;
}

// ---- Frame::isInFrustum (Frame.cc:166-227), one thread per map point.
// Clocked form (the front end's time budgets, gf_set_budgets): each point's
// elapsed time since the loop's timer start ck_t0[f] is written to the clock
// record at its list position, and the result goes to `alt` (same indexing as
// views): the front end keeps it only for the points before the cut.
struct FrustumClock {
    const unsigned long long* t0;  // null: not clocked
    long long* rec;
    long long stride;
    int off;
    gf_mp_view* alt;
    const long long* syn;  // test clock (base, slope); null: the device clock
};

__global__ void k_frustum(FrameConst fc, const float* __restrict__ Tcw, const gf_map_point* __restrict__ mps,
                          const int32_t* __restrict__ m, int cap, float viewCosLimit, gf_mp_view* __restrict__ views,
                          int32_t* __restrict__ nview, const int32_t* __restrict__ list,
                          const int32_t* __restrict__ nlist, FrustumClock ck) {
    const int f = blockIdx.y;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    const float* T = Tcw + 16 * f;
    int in = 0;
    const bool run = list ? i < nlist[f] : i < m[f];
    if (run && ck.t0) {
        ck.rec[(long long)f * ck.stride + ck.off + i] = gfd::ck_elapsed(ck.t0[f], ck.syn, i);
        views = ck.alt;
    }
    if (run && list) i = list[(long long)f * cap + i];  // the list's map point
    if (run) {
        gf_mp_view v;
        v.in_view = 0;
        v.u = v.v = v.view_cos = 0.f;
        v.level = 0;
        const gf_map_point mp = mps[(long long)f * cap + i];
        float Ow[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            float a = T[0 * 4 + c] * T[3], b = T[1 * 4 + c] * T[7], d = T[2 * 4 + c] * T[11];
            Ow[c] = -((a + b) + d);
        }
        float Pc[3];
        transform3(T, mp.pos, Pc);
        do {
            if (Pc[2] < 0.0) break;
            const float invz = (float)(1.0 / (double)Pc[2]);
            const float u = fc.fx * Pc[0] * invz + fc.cx;
            const float vv = fc.fy * Pc[1] * invz + fc.cy;
            if (u < fc.min_x || u > fc.max_x) break;
            if (vv < fc.min_y || vv > fc.max_y) break;
            const float PO[3] = {mp.pos[0] - Ow[0], mp.pos[1] - Ow[1], mp.pos[2] - Ow[2]};
            const float dist =
                (float)sqrt((double)PO[0] * PO[0] + (double)PO[1] * PO[1] + (double)PO[2] * PO[2]);
            if (dist < mp.min_dist || dist > mp.max_dist) break;
            double dot = (double)PO[0] * mp.normal[0] + (double)PO[1] * mp.normal[1] + (double)PO[2] * mp.normal[2];
            const float viewCos = (float)(dot / dist);
            if (viewCos < viewCosLimit) break;
            const float ratio = dist / mp.min_dist;
            int lvl = 0;
            while (lvl < fc.nlevels && fc.scales[lvl] < ratio) lvl++;
            if (lvl >= fc.nlevels) lvl = fc.nlevels - 1;
            v.in_view = 1;
            v.u = u;
            v.v = vv;
            v.level = lvl;
            v.view_cos = viewCos;
            in = 1;
        } while (0);
        views[(long long)f * cap + i] = v;
    }
    // count in-view points
    int s = gfd::warp_sum(in);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(&nview[f], s);
}

__global__ void k_hamming(const uint8_t* a, const uint8_t* b, int n, int32_t* dist) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dist[i] = hamming32(a + 32LL * i, b + 32LL * i);
}

size_t match_lds_bytes(int kp_cap, int q_cap) {
    return match_base_lds(kp_cap, q_cap) + (match_stage(kp_cap, q_cap) ? 48 * (size_t)kp_cap : 0);
}

}  // namespace

namespace gf {
FrameConst make_frame_const(const gf_frame_info* fi) {
    FrameConst fc{};
    fc.min_x = fi->min_x;
    fc.max_x = fi->max_x;
    fc.min_y = fi->min_y;
    fc.max_y = fi->max_y;
    fc.fx = fi->fx;
    fc.fy = fi->fy;
    fc.cx = fi->cx;
    fc.cy = fi->cy;
    fc.nlevels = fi->nlevels;
    fc.invW = (float)GRID_COLS / (float)(fi->max_x - fi->min_x);
    fc.invH = (float)GRID_ROWS / (float)(fi->max_y - fi->min_y);
    fc.scales[0] = 1.f;
    for (int i = 1; i < fi->nlevels && i < 16; i++) fc.scales[i] = fc.scales[i - 1] * fi->scale_factor;
    return fc;
}
}  // namespace gf

static int check_fi(const gf_frame_info* fi) {
    GF_CHECK(fi, GF_ERR_ARG, "null frame info");
    GF_CHECK(fi->nlevels >= 1 && fi->nlevels <= 16, GF_ERR_ARG, "nlevels out of range");
    GF_CHECK(fi->max_x > fi->min_x && fi->max_y > fi->min_y, GF_ERR_ARG, "empty image bounds");
    return GF_OK;
}

namespace {
thread_local int32_t* tl_ncand = nullptr;
}
gf::CandidateCount::CandidateCount(int32_t* d_counts) : prev(tl_ncand) { tl_ncand = d_counts; }
gf::CandidateCount::~CandidateCount() { tl_ncand = prev; }
int32_t* gf::candidate_counts() { return tl_ncand; }

static int launch_match(gf_ctx* ctx, const MatchArgs& A0, const FrameConst& fc, int nframes, hipStream_t s) {
    MatchArgs A = A0;
    A.ncand = tl_ncand;
    static unsigned long long attr_mask = 0;
    if (!(attr_mask & (1ull << ctx->device))) {
        GF_HIP(hipFuncSetAttribute((const void*)k_match, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
        GF_HIP(hipFuncSetAttribute((const void*)k_match_seq, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   152 * 1024));
        GF_HIP(hipFuncSetAttribute((const void*)k_match_seq_pre, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)seq_pre_lds_bytes(KP_MAX)));
        attr_mask |= 1ull << ctx->device;
    }
    if (A.mode == MODE_LAST) {  // few queries, wide windows: wave-sequential in the reference order
        {
            GF_PROF(ctx, s, "k_match_seq_pre");
            GF_LAUNCH(k_match_seq_pre, nframes, SEQ_PRE_THREADS, seq_pre_lds_bytes(A.kp_cap), s, A, fc, (SeqPre*)A.pre);
            GF_HIP(hipGetLastError());
        }
        GF_PROF(ctx, s, "k_match_lastframe");
        GF_LAUNCH(k_match_seq, nframes, SEQ_THREADS, seq_lds_bytes(A.kp_cap, A.q_cap), s, A, fc);
    } else {  // many queries, narrow windows: claim-resolution rounds
        GF_PROF(ctx, s, "k_match_project");
        GF_LAUNCH(k_match, nframes, MATCH_THREADS, match_lds_bytes(A.kp_cap, A.q_cap), s, A, fc);
    }
    GF_HIP(hipGetLastError());
    return GF_OK;
}

static int project_impl(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                        const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                        const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, float th, const float* d_th,
                        float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream);

extern "C" {

int gf_frustum_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw, const gf_map_point* d_mps,
                   const int32_t* d_m, int mp_cap, float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview,
                   void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    if (nframes <= 0 || mp_cap <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    FrameConst fc = gf::make_frame_const(fi);
    GF_HIP(hipMemsetAsync(d_nview, 0, sizeof(int32_t) * nframes, s));
    GF_PROF(ctx, s, "k_frustum");
    GF_LAUNCH(k_frustum, dim3((mp_cap + 255) / 256, nframes), 256, 0, s, fc, d_Tcw, d_mps, d_m, mp_cap, view_cos_limit,
                                                                   d_views, d_nview, nullptr, nullptr,
                                                                   FrustumClock{});
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_frustum_list_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw,
                        const gf_map_point* d_mps, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                        float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    if (nframes <= 0 || mp_cap <= 0) return GF_OK;
    GF_CHECK(d_Tcw && d_mps && d_list && d_nlist && d_views && d_nview, GF_ERR_ARG, "null arg");
    hipStream_t s = (hipStream_t)stream;
    FrameConst fc = gf::make_frame_const(fi);
    GF_HIP(hipMemsetAsync(d_nview, 0, sizeof(int32_t) * nframes, s));
    GF_PROF(ctx, s, "k_frustum_list");
    GF_LAUNCH(k_frustum, dim3((mp_cap + 255) / 256, nframes), 256, 0, s, fc, d_Tcw, d_mps, nullptr, mp_cap, view_cos_limit,
                                                                   d_views, d_nview, d_list, d_nlist,
                                                                   FrustumClock{});
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_match_project_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                         const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                         const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, float th, float nnratio,
                         int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream) {
    return project_impl(ctx, fi, nframes, d_kps, d_desc, d_n, kp_cap, d_views, d_mp_desc, d_m, mp_cap, th, nullptr,
                        nnratio, d_kp2mp, d_score, d_nmatches, stream);
}

}  // extern "C"

int gf::match_project_th(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                         const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                         const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, const float* d_th, float nnratio,
                         int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream) {
    return project_impl(ctx, fi, nframes, d_kps, d_desc, d_n, kp_cap, d_views, d_mp_desc, d_m, mp_cap, 1.f, d_th,
                        nnratio, d_kp2mp, d_score, d_nmatches, stream);
}

static int project_impl(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                        const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                        const uint8_t* d_mp_desc, const int32_t* d_m, int mp_cap, float th, const float* d_th,
                        float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    GF_CHECK(kp_cap <= KP_MAX && mp_cap <= Q_MAX, GF_ERR_UNSUPPORTED, "frame exceeds matcher limits (4096 kps, 8192 mps)");
    if (nframes <= 0) return GF_OK;
    MatchArgs A{};
    A.mode = MODE_PROJECT;
    A.kps = d_kps;
    A.desc = d_desc;
    A.n = d_n;
    A.kp_cap = kp_cap;
    A.views = d_views;
    A.qdesc = d_mp_desc;
    A.m = d_m;
    A.q_cap = mp_cap;
    A.th = th;
    A.th_per = d_th;
    A.nnratio = nnratio;
    A.kp2mp = d_kp2mp;
    A.score = d_score;
    A.nmatches = d_nmatches;
    void* err;
    rc = gf::ws_get(ctx, 31, sizeof(int32_t) * nframes, &err);
    if (rc) return rc;
    A.err = (int32_t*)err;
    return launch_match(ctx, A, gf::make_frame_const(fi), nframes, (hipStream_t)stream);
}

extern "C" {

int gf_match_project_list_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                              const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                              const uint8_t* d_mp_desc, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                              float th, float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches,
                              void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    GF_CHECK(kp_cap <= KP_MAX && mp_cap <= Q_MAX, GF_ERR_UNSUPPORTED, "frame exceeds matcher limits (4096 kps, 8192 mps)");
    GF_CHECK(d_list && d_nlist, GF_ERR_ARG, "null list");
    if (nframes <= 0) return GF_OK;
    MatchArgs A{};
    A.mode = MODE_PROJECT;
    A.kps = d_kps;
    A.desc = d_desc;
    A.n = d_n;
    A.kp_cap = kp_cap;
    A.views = d_views;
    A.qdesc = d_mp_desc;
    A.m = d_nlist;
    A.q_cap = mp_cap;
    A.list = d_list;
    A.nlist = d_nlist;
    A.th = th;
    A.nnratio = nnratio;
    A.kp2mp = d_kp2mp;
    A.score = d_score;
    A.nmatches = d_nmatches;
    void* err;
    rc = gf::ws_get(ctx, 38, sizeof(int32_t) * nframes, &err);
    if (rc) return rc;
    A.err = (int32_t*)err;
    return launch_match(ctx, A, gf::make_frame_const(fi), nframes, (hipStream_t)stream);
}

int gf_match_lastframe_dev(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                           const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const float* d_Tcw,
                           const gf_keypoint* d_last_kps, const uint8_t* d_last_desc, const int32_t* d_last_kp2mp,
                           const uint8_t* d_last_outlier, const float* d_last_pos, const int32_t* d_n_last,
                           int last_cap, float th, int check_ori, int32_t* d_kp2mp, int32_t* d_score,
                           int32_t* d_nmatches, int32_t* d_scratch, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    GF_CHECK(kp_cap <= KP_MAX && last_cap <= Q_MAX, GF_ERR_UNSUPPORTED, "frame exceeds matcher limits");
    if (nframes <= 0) return GF_OK;
    MatchArgs A{};
    A.mode = MODE_LAST;
    A.kps = d_kps;
    A.desc = d_desc;
    A.n = d_n;
    A.kp_cap = kp_cap;
    A.qdesc = d_last_desc;
    A.m = d_n_last;
    A.q_cap = last_cap;
    A.last_kps = d_last_kps;
    A.last_kp2mp = d_last_kp2mp;
    A.last_outlier = d_last_outlier;
    A.last_pos = d_last_pos;
    A.Tcw = d_Tcw;
    A.th = th;
    A.check_ori = check_ori;
    A.kp2mp = d_kp2mp;
    A.score = d_score;
    A.nmatches = d_nmatches;
    A.qres = d_scratch;
    void* err;
    rc = gf::ws_get(ctx, 31, sizeof(int32_t) * nframes, &err);
    if (rc) return rc;
    A.err = (int32_t*)err;
    void* pre;
    rc = gf::ws_get(ctx, 33, sizeof(SeqPre) * (size_t)nframes * last_cap, &pre);
    if (rc) return rc;
    A.pre = (const SeqPre*)pre;
    void *gcs, *gitems;
    if ((rc = gf::ws_get(ctx, 36, sizeof(int) * (size_t)nframes * (NCELLS + 1), &gcs)) ||
        (rc = gf::ws_get(ctx, 37, sizeof(int) * (size_t)nframes * kp_cap, &gitems)))
        return rc;
    A.grid_cs = (int*)gcs;
    A.grid_items = (int*)gitems;
    GF_CHECK(seq_pre_lds_bytes(kp_cap) <= 160 * 1024 && seq_lds_bytes(kp_cap, last_cap) <= 152 * 1024,
             GF_ERR_UNSUPPORTED, "keypoint / last-frame capacity too large for LDS");
    return launch_match(ctx, A, gf::make_frame_const(fi), nframes, (hipStream_t)stream);
}

// ------------------------------------------------------------ host family
int gf_frustum(gf_ctx* ctx, const gf_frame_info* fi, const float* Tcw, const gf_map_point* mps, int m,
               float view_cos_limit, gf_mp_view* views, int* n_in_view) {
    GF_CHECK(ctx && Tcw && n_in_view, GF_ERR_ARG, "null arg");
    *n_in_view = 0;
    if (m <= 0) return GF_OK;
    GF_CHECK(mps && views, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dT, *dM, *dm, *dV, *dn;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, Tcw, 64, &dT)) || (rc = gf::ws_upload(ctx, 1, mps, sizeof(gf_map_point) * m, &dM)) ||
        (rc = gf::ws_upload(ctx, 2, &m, 4, &dm)) || (rc = gf::ws_get(ctx, 3, sizeof(gf_mp_view) * m, &dV)) ||
        (rc = gf::ws_get(ctx, 4, 4, &dn)))
        return rc;
    rc = gf_frustum_dev(ctx, fi, 1, (const float*)dT, (const gf_map_point*)dM, (const int32_t*)dm, m, view_cos_limit,
                        (gf_mp_view*)dV, (int32_t*)dn, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(views, dV, sizeof(gf_mp_view) * m, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(n_in_view, dn, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_match_project(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                     const gf_mp_view* views, const uint8_t* mp_desc, int m, float th, float nnratio, int32_t* kp2mp,
                     int32_t* score, int* nmatches) {
    GF_CHECK(ctx && nmatches, GF_ERR_ARG, "null arg");
    *nmatches = 0;
    if (n <= 0 || m <= 0) return GF_OK;
    GF_CHECK(kps && desc && views && mp_desc && kp2mp && score, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dK, *dD, *dn, *dV, *dQ, *dm, *dC, *dS, *dN;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, kps, sizeof(gf_keypoint) * n, &dK)) ||
        (rc = gf::ws_upload(ctx, 1, desc, 32 * (size_t)n, &dD)) || (rc = gf::ws_upload(ctx, 2, &n, 4, &dn)) ||
        (rc = gf::ws_upload(ctx, 3, views, sizeof(gf_mp_view) * m, &dV)) ||
        (rc = gf::ws_upload(ctx, 4, mp_desc, 32 * (size_t)m, &dQ)) || (rc = gf::ws_upload(ctx, 5, &m, 4, &dm)) ||
        (rc = gf::ws_upload(ctx, 6, kp2mp, 4 * (size_t)n, &dC)) || (rc = gf::ws_upload(ctx, 7, score, 4 * (size_t)n, &dS)) ||
        (rc = gf::ws_get(ctx, 8, 4, &dN)))
        return rc;
    rc = gf_match_project_dev(ctx, fi, 1, (const gf_keypoint*)dK, (const uint8_t*)dD, (const int32_t*)dn, n,
                              (const gf_mp_view*)dV, (const uint8_t*)dQ, (const int32_t*)dm, m, th, nnratio,
                              (int32_t*)dC, (int32_t*)dS, (int32_t*)dN, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(kp2mp, dC, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(score, dS, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(nmatches, dN, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_match_lastframe(gf_ctx* ctx, const gf_frame_info* fi, const gf_keypoint* kps, const uint8_t* desc, int n,
                       const float* Tcw, const gf_keypoint* last_kps, const uint8_t* last_desc,
                       const int32_t* last_kp2mp, const uint8_t* last_outlier, const float* last_pos, int n_last,
                       float th, int check_ori, int32_t* kp2mp, int32_t* score, int* nmatches) {
    GF_CHECK(ctx && nmatches, GF_ERR_ARG, "null arg");
    *nmatches = 0;
    if (n <= 0 || n_last <= 0) return GF_OK;
    GF_CHECK(kps && desc && Tcw && last_kps && last_desc && last_kp2mp && last_outlier && last_pos && kp2mp && score,
             GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dK, *dD, *dn, *dT, *dLK, *dLD, *dLM, *dLO, *dLP, *dnl, *dC, *dS, *dN, *dR;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, kps, sizeof(gf_keypoint) * n, &dK)) ||
        (rc = gf::ws_upload(ctx, 1, desc, 32 * (size_t)n, &dD)) || (rc = gf::ws_upload(ctx, 2, &n, 4, &dn)) ||
        (rc = gf::ws_upload(ctx, 3, Tcw, 64, &dT)) ||
        (rc = gf::ws_upload(ctx, 4, last_kps, sizeof(gf_keypoint) * n_last, &dLK)) ||
        (rc = gf::ws_upload(ctx, 5, last_desc, 32 * (size_t)n_last, &dLD)) ||
        (rc = gf::ws_upload(ctx, 6, last_kp2mp, 4 * (size_t)n_last, &dLM)) ||
        (rc = gf::ws_upload(ctx, 7, last_outlier, (size_t)n_last, &dLO)) ||
        (rc = gf::ws_upload(ctx, 8, last_pos, 12 * (size_t)n_last, &dLP)) ||
        (rc = gf::ws_upload(ctx, 9, &n_last, 4, &dnl)) || (rc = gf::ws_upload(ctx, 10, kp2mp, 4 * (size_t)n, &dC)) ||
        (rc = gf::ws_upload(ctx, 11, score, 4 * (size_t)n, &dS)) || (rc = gf::ws_get(ctx, 12, 4, &dN)) ||
        (rc = gf::ws_get(ctx, 13, 4 * (size_t)n_last, &dR)))
        return rc;
    rc = gf_match_lastframe_dev(ctx, fi, 1, (const gf_keypoint*)dK, (const uint8_t*)dD, (const int32_t*)dn, n,
                                (const float*)dT, (const gf_keypoint*)dLK, (const uint8_t*)dLD, (const int32_t*)dLM,
                                (const uint8_t*)dLO, (const float*)dLP, (const int32_t*)dnl, n_last, th, check_ori,
                                (int32_t*)dC, (int32_t*)dS, (int32_t*)dN, (int32_t*)dR, ctx->stream);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(kp2mp, dC, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(score, dS, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(nmatches, dN, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_descriptor_distance(gf_ctx* ctx, const uint8_t* a, const uint8_t* b, int n, int32_t* dist) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (n <= 0) return GF_OK;
    GF_CHECK(a && b && dist, GF_ERR_ARG, "null arg");
    GF_HIP(hipSetDevice(ctx->device));
    void *dA, *dB, *dO;
    int rc;
    if ((rc = gf::ws_upload(ctx, 0, a, 32 * (size_t)n, &dA)) || (rc = gf::ws_upload(ctx, 1, b, 32 * (size_t)n, &dB)) ||
        (rc = gf::ws_get(ctx, 2, 4 * (size_t)n, &dO)))
        return rc;
    GF_LAUNCH(k_hamming, (n + 255) / 256, 256, 0, ctx->stream, (const uint8_t*)dA, (const uint8_t*)dB, n, (int32_t*)dO);
    GF_HIP(hipGetLastError());
    GF_HIP(hipMemcpyAsync(dist, dO, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

}  // extern "C"

// Front-end forms with the time-budget clocks (frontend.hip, gf_set_budgets).
int gf::frustum_clocked(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const float* d_Tcw,
                        const gf_map_point* d_mps, const int32_t* d_m, const int32_t* d_list, const int32_t* d_nlist,
                        int mp_cap, float view_cos_limit, gf_mp_view* d_views, int32_t* d_nview,
                        const gf::StageClock& ck, gf_mp_view* d_alt, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    if (nframes <= 0 || mp_cap <= 0) return GF_OK;
    hipStream_t s = (hipStream_t)stream;
    const FrameConst fc = gf::make_frame_const(fi);
    GF_HIP(hipMemsetAsync(d_nview, 0, sizeof(int32_t) * nframes, s));
    GF_PROF(ctx, s, d_list ? "k_frustum_list" : "k_frustum");
    const FrustumClock fk{ck.t0, ck.rec, ck.stride, ck.off, d_alt, ck.syn};
    GF_LAUNCH(k_frustum, dim3((mp_cap + 255) / 256, nframes), 256, 0, s, fc, d_Tcw, d_mps, d_m, mp_cap, view_cos_limit,
                                                                   d_views, d_nview, d_list, d_nlist,
                                                                   ck.t0 ? fk : FrustumClock{});
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf::match_project_list_budget(gf_ctx* ctx, const gf_frame_info* fi, int nframes, const gf_keypoint* d_kps,
                                  const uint8_t* d_desc, const int32_t* d_n, int kp_cap, const gf_mp_view* d_views,
                                  const uint8_t* d_mp_desc, int mp_cap, const int32_t* d_list, const int32_t* d_nlist,
                                  float th, float nnratio, int32_t* d_kp2mp, int32_t* d_score, int32_t* d_nmatches,
                                  const gf::StageClock& ck, const long long* d_rest2, int32_t* d_qres,
                                  int32_t* d_old, int32_t* d_err, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    int rc = check_fi(fi);
    if (rc) return rc;
    GF_CHECK(kp_cap <= KP_MAX && mp_cap <= Q_MAX, GF_ERR_UNSUPPORTED, "frame exceeds matcher limits (4096 kps, 8192 mps)");
    if (nframes <= 0) return GF_OK;
    MatchArgs A{};
    A.mode = MODE_PROJECT;
    A.kps = d_kps;
    A.desc = d_desc;
    A.n = d_n;
    A.kp_cap = kp_cap;
    A.views = d_views;
    A.qdesc = d_mp_desc;
    A.m = d_nlist;
    A.q_cap = mp_cap;
    A.list = d_list;
    A.nlist = d_nlist;
    A.th = th;
    A.nnratio = nnratio;
    A.kp2mp = d_kp2mp;
    A.score = d_score;
    A.nmatches = d_nmatches;
    A.err = d_err;
    if (ck.t0) {
        GF_CHECK(d_rest2 && d_qres && d_old && ck.rec, GF_ERR_ARG, "null clock arg");
        A.ck_t0 = ck.t0;
        A.ck_rest2 = d_rest2;
        A.ck_rec = ck.rec;
        A.ck_stride = ck.stride;
        A.ck_off = ck.off;
        A.ck_syn = ck.syn;
        A.ck_old = d_old;
        A.qres = d_qres;
    }
    return launch_match(ctx, A, gf::make_frame_const(fi), nframes, (hipStream_t)stream);
}
