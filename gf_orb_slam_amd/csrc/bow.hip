// Bag of words on gfx950 — SURVEY.md §8a rows D1 (DBoW2 transform) and M6
// (ORBmatcher::SearchByBoW).
//
//   k_bow_descend  one thread per descriptor: descent of the vocabulary tree,
//                  first-minimum Hamming child per level
//                  (TemplatedVocabulary.h:1232-1273) -> word, weight, node at
//                  level L - levelsup
//   k_bow_build    one workgroup per frame: BowVector (words ascending,
//                  addWeight / addIfNotExist in feature order, L1/L2/size
//                  normalisation in word order, BowVector.cpp:34-84) and
//                  FeatureVector (nodes ascending, features in order,
//                  FeatureVector.cpp:31-45) from two bitonic sorts in LDS
//   k_match_bow    one workgroup per (a, b) pair: the nodes both
//                  FeatureVectors share are independent (a b feature belongs
//                  to one node, so claims never cross nodes); a wave walks one
//                  node's a features in order, 64 b features per step, and
//                  keeps the sequential best / second-best / claim semantics
//                  exactly (ORBmatcher.cc:745-829, 1317-1399); then the
//                  rotation histogram (:832-850, :1401-1421)
//
// The tree (descriptors, children CSR, weights, word ids) is device resident
// for the context; ORBvoc-size trees (k = 10, L = 6: ~1.1 M nodes, ~45 MB)
// stay in HBM, their top levels in L2.
#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "match_common.h"

struct gf_vocab {
    gf_ctx* ctx = nullptr;
    int k = 0, L = 0, scoring = 0, weighting = 0, nnodes = 0, nwords = 0;
    uint8_t* d_desc = nullptr;
    int32_t *d_cstart = nullptr, *d_child = nullptr, *d_word = nullptr;
    double* d_weight = nullptr;
    // host-family staging
    size_t stage_cap = 0;
    uint8_t* d_in = nullptr;
    void* d_stage = nullptr;
};

namespace {

constexpr int BOW_MAX = 4096;
// dynamic LDS of k_bow_build (bitonic keys and values over pow2(cap)) and
// k_match_bow (per b-side feature: common node pair, match record, claim, bin)
static size_t bow_build_lds(int cap) {
    size_t p2 = 1;
    while ((int)p2 < cap) p2 <<= 1;
    return 24 * p2;
}
static size_t match_bow_lds(int bcap) { return (8 + 4 + 1 + 1) * (size_t)bcap + 16; }

struct VocabDev {
    const uint8_t* desc;
    const int32_t* cstart;
    const int32_t* child;
    const int32_t* word;
    const double* weight;
    int L, scoring, weighting;
};

__device__ __forceinline__ int ham_regs(const uint32_t* f, const uint8_t* nd) {
    const uint4* p = (const uint4*)nd;
    const uint4 a = p[0], b = p[1];
    return __popc(f[0] ^ a.x) + __popc(f[1] ^ a.y) + __popc(f[2] ^ a.z) + __popc(f[3] ^ a.w) + __popc(f[4] ^ b.x) +
           __popc(f[5] ^ b.y) + __popc(f[6] ^ b.z) + __popc(f[7] ^ b.w);
}

__global__ __launch_bounds__(256) void k_bow_descend(VocabDev V, const uint8_t* __restrict__ desc,
                                                     const int32_t* __restrict__ nfeat, int cap, int levelsup,
                                                     int32_t* __restrict__ wid, double* __restrict__ wval,
                                                     int32_t* __restrict__ nid, const int32_t* __restrict__ gate) {
    const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (gate && !gate[f]) return;
    if (i >= min(nfeat[f], cap)) return;
    const size_t g = (size_t)f * cap + i;
    uint32_t x[8];
    {
        const uint4* p = (const uint4*)(desc + g * 32);
        const uint4 a = p[0], b = p[1];
        x[0] = a.x, x[1] = a.y, x[2] = a.z, x[3] = a.w, x[4] = b.x, x[5] = b.y, x[6] = b.z, x[7] = b.w;
    }
    const int nid_level = V.L - levelsup;
    int node = 0, level = 0, at = 0;  // node at nid_level; root when the branch ends above it
    int cs = V.cstart[0], ce = V.cstart[1];
    while (ce > cs) {
        ++level;
        int fin = V.child[cs];
        int best = ham_regs(x, V.desc + (size_t)fin * 32);
        for (int c = cs + 1; c < ce; c++) {
            const int id = V.child[c];
            const int d = ham_regs(x, V.desc + (size_t)id * 32);
            if (d < best) {
                best = d;
                fin = id;
            }
        }
        if (level == nid_level) at = fin;
        node = fin;
        cs = V.cstart[node];
        ce = V.cstart[node + 1];
    }
    wid[g] = V.word[node];
    wval[g] = V.weight[node];
    nid[g] = nid_level <= 0 ? 0 : at;
}

// in-place ascending bitonic sort of n2 (power of two) keys by the workgroup
__device__ void bitonic(unsigned long long* a, int n2) {
    for (int k = 2; k <= n2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < n2; i += blockDim.x) {
                const int l = i ^ j;
                if (l > i) {
                    const unsigned long long x = a[i], y = a[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        a[i] = y;
                        a[l] = x;
                    }
                }
            }
            __syncthreads();
        }
}

__device__ int block_excl_scan(int v, int* tmp, int& total) {  // 256 threads
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[w] = x;
    __syncthreads();
    int base = 0;
    for (int i = 0; i < w; i++) base += tmp[i];
    total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    __syncthreads();
    return base + x - v;
}

__global__ __launch_bounds__(256) void k_bow_build(VocabDev V, int nframes, const int32_t* __restrict__ nfeat, int cap,
                                                   const int32_t* __restrict__ wid, const double* __restrict__ wval,
                                                   const int32_t* __restrict__ nid, int32_t* __restrict__ words,
                                                   double* __restrict__ values, int32_t* __restrict__ nwords,
                                                   int32_t* __restrict__ fv_nodes, int32_t* __restrict__ fv_start,
                                                   int32_t* __restrict__ fv_feats, int32_t* __restrict__ nfv,
                                                   const int32_t* __restrict__ gate) {
    // sized by the launch to the next power of two of cap (bitonic length):
    // kw, kn (8 B), vals (8 B) per entry. A BOW_MAX-sized static array held
    // 96 KB per workgroup, so the launch waited for nearly empty CUs beside
    // the other front ends' extraction even when no stream relocalised
    extern __shared__ __align__(16) unsigned long long bow_lds[];
    int p2 = 1;
    while (p2 < cap) p2 <<= 1;
    unsigned long long* kw = bow_lds;
    unsigned long long* kn = kw + p2;
    double* vals = reinterpret_cast<double*>(kn + p2);
    __shared__ int tmp[4], s_m;
    __shared__ double s_norm;
    const int tid = threadIdx.x;
    // a small grid walks the frames: with a gate most frames are off, and a
    // workgroup per frame would hold this kernel's LDS across the whole chip
    for (int f = blockIdx.x; f < nframes; f += gridDim.x) {
    if (gate && !gate[f]) {  // empty vectors
        if (tid == 0) {
            nwords[f] = 0;
            nfv[f] = 0;
            fv_start[(size_t)f * (cap + 1)] = 0;
        }
        continue;
    }
    const int n = min(nfeat[f], cap);
    const size_t g0 = (size_t)f * cap;
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    if (tid == 0) s_m = 0;
    __syncthreads();
    int cnt = 0;
    for (int i = tid; i < n2; i += 256) {
        const bool ok = i < n && wval[g0 + i] > 0;  // stopped words (weight 0) are left out of both vectors
        kw[i] = ok ? ((unsigned long long)(uint32_t)wid[g0 + i] << 32) | (uint32_t)i : ~0ull;
        kn[i] = ok ? ((unsigned long long)(uint32_t)nid[g0 + i] << 32) | (uint32_t)i : ~0ull;
        cnt += ok;
    }
    atomicAdd(&s_m, cnt);
    __syncthreads();
    bitonic(kw, n2);
    bitonic(kn, n2);
    const int m = s_m;
    // ---- BowVector: one head per word; value accumulated in feature order
    int total = 0, base = 0;
    for (int c0 = 0; c0 < m; c0 += 256) {
        const int i = c0 + tid;
        const bool head = i < m && (i == 0 || (kw[i] >> 32) != (kw[i - 1] >> 32));
        int tot;
        const int pos = base + block_excl_scan(head ? 1 : 0, tmp, tot);
        if (head) {
            const uint32_t w = (uint32_t)(kw[i] >> 32);
            double v = wval[g0 + (uint32_t)kw[i]];
            if (V.weighting == 0 || V.weighting == 1)  // TF_IDF, TF: addWeight
                for (int j = i + 1; j < m && (uint32_t)(kw[j] >> 32) == w; j++) v += wval[g0 + (uint32_t)kw[j]];
            vals[pos] = v;                               // IDF, BINARY: addIfNotExist keeps the first
            words[g0 + pos] = (int32_t)w;
        }
        base += tot;
    }
    total = base;
    __syncthreads();
    if (tid == 0) {
        double norm = 0.0;
        if (V.scoring == 5) {  // DOT_PRODUCT: no normalisation; TF / TF_IDF divide by the size
            norm = (V.weighting == 0 || V.weighting == 1) && total > 0 ? (double)total : 0.0;
        } else if (V.scoring == 1) {  // L2_NORM
            for (int i = 0; i < total; i++) norm += vals[i] * vals[i];
            norm = sqrt(norm);
        } else {  // L1
            for (int i = 0; i < total; i++) norm += fabs(vals[i]);
        }
        s_norm = norm;
    }
    __syncthreads();
    const double norm = s_norm;
    for (int i = tid; i < total; i += 256) values[g0 + i] = norm > 0.0 ? vals[i] / norm : vals[i];
    if (tid == 0) nwords[f] = total;
    // ---- FeatureVector: one head per node, features in order
    base = 0;
    for (int c0 = 0; c0 < m; c0 += 256) {
        const int i = c0 + tid;
        const bool head = i < m && (i == 0 || (kn[i] >> 32) != (kn[i - 1] >> 32));
        int tot;
        const int pos = base + block_excl_scan(head ? 1 : 0, tmp, tot);
        if (head) {
            fv_nodes[g0 + pos] = (int32_t)(kn[i] >> 32);
            fv_start[(size_t)f * (cap + 1) + pos] = i;
        }
        if (i < m) fv_feats[g0 + i] = (int32_t)(uint32_t)kn[i];
        base += tot;
    }
    if (tid == 0) {
        nfv[f] = base;
        fv_start[(size_t)f * (cap + 1) + base] = m;
    }
    __syncthreads();  // the LDS goes to the next frame
    }
}

// ComputeThreeMaxima (ORBmatcher.cc:2338-2379) over the recorded matches' bins;
// drops the matches outside the three dominant bins. All threads of the block.
__device__ void rotation_filter(int nm, const uint8_t* rbin, const int* rec, int32_t* out, int* s_hist,
                                int* s_keep, int* s_nm) {
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int r = tid; r < nm; r += nt) atomicAdd(&s_hist[rbin[r]], 1);
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
    int drop = 0;
    for (int r = tid; r < nm; r += nt) {
        const int b = rbin[r];
        if (b == s_keep[0] || b == s_keep[1] || b == s_keep[2]) continue;
        out[rec[r]] = -1;
        drop++;
    }
    atomicSub(s_nm, drop);
    __syncthreads();
}

using BowPair = gf::BowPairDev;

// (d1, position of d1, d2) of a stream, reduced across the wave: the winner
// has the smaller d1 (ties: earlier position); second = min(winner d2, loser d1)
__device__ __forceinline__ void top2_merge(int& d1, int& p1, int& d2, int od1, int op1, int od2) {
    if (od1 < d1 || (od1 == d1 && op1 < p1)) {
        d2 = min(od2, d1);
        d1 = od1;
        p1 = op1;
    } else {
        d2 = min(d2, od1);
    }
}

__global__ __launch_bounds__(256) void k_match_bow(const BowPair* __restrict__ pairs, int npairs, int mode,
                                                   float nnratio, int check_ori, int32_t* __restrict__ nmatches,
                                                   int bcap) {
    // sized by the launch for bcap b-side features (every array's index is
    // below B.n: common nodes <= B.nfv, matches <= claimed b features):
    // common (8 B), rec (4 B), claimed, rbin (1 B) per entry
    extern __shared__ __align__(16) int2 mb_lds[];
    int2* common = mb_lds;
    int* rec = reinterpret_cast<int*>(common + bcap);
    uint8_t* claimed = reinterpret_cast<uint8_t*>(rec + bcap);
    uint8_t* rbin = claimed + bcap;
    __shared__ int s_nc, s_nm, s_hist[HISTO_LENGTH], s_keep[3];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    // a small grid walks the pairs (the step's pair list is mostly the empty
    // pairs of streams that do not relocalise)
    for (int pi = blockIdx.x; pi < npairs; pi += gridDim.x) {
    const BowPair P = pairs[pi];
    const gf_bow_side& A = P.a;
    const gf_bow_side& B = P.b;
    if (B.n > bcap) {  // the launch's LDS does not hold this pair (the hosts size it: not reached)
        if (tid == 0) nmatches[pi] = -1;
        continue;
    }
    const int nout = mode == 0 ? B.n : A.n;
    for (int i = tid; i < nout; i += 256) P.out[i] = -1;
    if (A.nfv == 0 || B.nfv == 0) {  // no common node: no match
        if (tid == 0) nmatches[pi] = 0;
        continue;
    }
    for (int i = tid; i < B.n; i += 256) claimed[i] = 0;
    if (tid == 0) s_nc = s_nm = 0;
    if (tid < HISTO_LENGTH) s_hist[tid] = 0;
    __syncthreads();
    // nodes present in both FeatureVectors (the reference's merge walk visits exactly these)
    for (int ib = tid; ib < B.nfv; ib += 256) {
        const int key = B.fv_nodes[ib];
        int lo = 0, hi = A.nfv;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (A.fv_nodes[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        if (lo < A.nfv && A.fv_nodes[lo] == key) common[atomicAdd(&s_nc, 1)] = make_int2(lo, ib);
    }
    __syncthreads();
    const int nc = s_nc;
    const float factor = 1.0f / HISTO_LENGTH;
    for (int c = w; c < nc; c += 4) {
        const int ia = common[c].x, ib = common[c].y;
        const int as = A.fv_start[ia], ae = A.fv_start[ia + 1], bs = B.fv_start[ib], be = B.fv_start[ib + 1];
        for (int x = as; x < ae; x++) {  // a features of the node, in order (sequential claims)
            const int idxA = A.fv_feats[x];
            if (A.mp[idxA] < 0) continue;
            const uint8_t* da = A.desc + (size_t)idxA * 32;
            int d1 = INT_MAX, p1 = INT_MAX, d2 = INT_MAX;
            for (int y = bs + lane; y < be; y += 64) {  // lane-local stream in position order
                const int idxB = B.fv_feats[y];
                const bool skip = mode == 0 ? claimed[idxB] : (claimed[idxB] || B.mp[idxB] < 0);
                if (skip) continue;
                const int d = hamming32(da, B.desc + (size_t)idxB * 32);
                if (d < d1) {
                    d2 = d1;
                    d1 = d;
                    p1 = y;
                } else if (d < d2) {
                    d2 = d;
                }
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int od1 = __shfl_xor(d1, o, 64), op1 = __shfl_xor(p1, o, 64), od2 = __shfl_xor(d2, o, 64);
                top2_merge(d1, p1, d2, od1, op1, od2);
            }
            const bool ok = mode == 0 ? d1 <= 50 : d1 < 50;  // TH_LOW
            if (!ok || !(static_cast<float>(d1) < nnratio * static_cast<float>(d2))) continue;
            const int bestB = B.fv_feats[p1];
            if (lane == 0) {
                claimed[bestB] = 1;
                const int o = mode == 0 ? bestB : idxA;
                P.out[o] = mode == 0 ? A.mp[idxA] : B.mp[bestB];
                const int r = atomicAdd(&s_nm, 1);
                rec[r] = o;
                float rot = A.kps[idxA].angle - B.kps[bestB].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rbin[r] = (uint8_t)bin;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();
    const int nm = s_nm;
    if (check_ori) rotation_filter(nm, rbin, rec, P.out, s_hist, s_keep, &s_nm);
    if (tid == 0) nmatches[pi] = s_nm;
    __syncthreads();  // the LDS goes to the next pair
    }
}

// SearchForTriangulation (ORBmatcher.cc:1426-1588): same node walk as
// SearchByBoW, but over keypoints WITHOUT a map point. Per a feature: best =
// min distance over unclaimed b candidates with d <= TH_LOW; the reference
// sorts (dist, idx2) and takes the first within round(2 best) passing the
// epipolar test, i.e. the (dist, idx2)-least passing candidate with
// d <= min(TH_LOW, 2 best): two wave reductions.
struct TriPair {
    gf_bow_side a, b;
    float F[9];
    float sigma2[16];
    int32_t nlevels;
    int32_t* out;
};

__device__ __forceinline__ bool epipolar_ok(float a, float b, float c, const gf_keypoint& kp2, const TriPair& P) {
    // CheckDistEpipolarLine (ORBmatcher.cc:705-722)
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    const int o = min(max(kp2.octave, 0), P.nlevels - 1);
    return (double)dsqr < 3.84 * (double)P.sigma2[o];
}

#define TRI_THREADS 1024
#define TRI_CT 4  // b candidates per lane held in registers (nodes of <= 256 b features)

__device__ __forceinline__ int hamming_r(const uint4 a0, const uint4 a1, const uint8_t* b) {
    const uint4 b0 = ((const uint4*)b)[0], b1 = ((const uint4*)b)[1];
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Match step of one a feature against the node's b candidates: best over the
// unclaimed (d <= TH_LOW), then the (d, idx)-least epipolar-passing one with
// d <= 2 best. Returns the b index or -1 (wave-uniform).
__device__ __forceinline__ int tri_pick(const int* d, const int* idx, const bool* ok, int n, float la, float lb,
                                        float lc, const gf_keypoint* kps, const TriPair& P) {
    int best = INT_MAX;
    for (int t = 0; t < n; t++)
        if (ok[t] && d[t] <= 50) best = min(best, d[t]);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) best = min(best, __shfl_xor(best, o, 64));
    if (best == INT_MAX) return -1;
    const int dth = min(2 * best, 50);  // round(2 * BestDist) is exact
    unsigned key = 0xffffffffu;
    for (int t = 0; t < n; t++) {
        if (!ok[t] || d[t] > dth) continue;
        const unsigned k = ((unsigned)d[t] << 16) | (unsigned)idx[t];
        if (k < key && epipolar_ok(la, lb, lc, kps[idx[t]], P)) key = k;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) key = min(key, (unsigned)__shfl_xor((int)key, o, 64));
    return key == 0xffffffffu ? -1 : (int)(key & 0xffffu);
}

__global__ __launch_bounds__(TRI_THREADS) void k_search_tri(const TriPair* __restrict__ pairs, int check_ori,
                                                            int32_t* __restrict__ nmatches) {
    __shared__ uint8_t claimed[BOW_MAX];
    __shared__ int2 common[BOW_MAX];
    __shared__ int rec[BOW_MAX];
    __shared__ uint8_t rbin[BOW_MAX];
    __shared__ int s_nc, s_nm, s_hist[HISTO_LENGTH], s_keep[3];
    __shared__ int st_idx[TRI_THREADS / 64][64];
    __shared__ uint4 st_desc[TRI_THREADS / 64][64][2];
    __shared__ float3 st_kp[TRI_THREADS / 64][64];
    const TriPair& P = pairs[blockIdx.x];
    const gf_bow_side& A = P.a;
    const gf_bow_side& B = P.b;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, nw = TRI_THREADS / 64;
    for (int i = tid; i < A.n; i += TRI_THREADS) P.out[i] = -1;
    for (int i = tid; i < B.n; i += TRI_THREADS) claimed[i] = 0;
    if (tid == 0) s_nc = s_nm = 0;
    if (tid < HISTO_LENGTH) s_hist[tid] = 0;
    __syncthreads();
    for (int ib = tid; ib < B.nfv; ib += TRI_THREADS) {
        const int key = B.fv_nodes[ib];
        int lo = 0, hi = A.nfv;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (A.fv_nodes[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        if (lo < A.nfv && A.fv_nodes[lo] == key) common[atomicAdd(&s_nc, 1)] = make_int2(lo, ib);
    }
    __syncthreads();
    const int nc = s_nc;
    const float factor = 1.0f / HISTO_LENGTH;
    const float* F = P.F;
    for (int c = w; c < nc; c += nw) {
        const int ia = common[c].x, ib = common[c].y;
        const int as = A.fv_start[ia], ae = A.fv_start[ia + 1], bs = B.fv_start[ib], be = B.fv_start[ib + 1];
        // a b feature sits in exactly one node, so only this wave claims it:
        // for nodes of <= 64 TRI_CT b features the candidates and their claim
        // flags stay in registers for the whole walk
        const bool regs = be - bs <= 64 * TRI_CT;
        uint4 cd[TRI_CT][2];
        int cidx[TRI_CT];
        bool cok[TRI_CT];
        if (regs) {
#pragma unroll
            for (int t = 0; t < TRI_CT; t++) {
                const int y = bs + lane + 64 * t;
                cok[t] = false;
                cidx[t] = 0;
                if (y < be) {
                    cidx[t] = B.fv_feats[y];
                    cok[t] = B.mp[cidx[t]] < 0;  // no MapPoint yet (:1484-1486)
                    const uint4* q = (const uint4*)(B.desc + (size_t)cidx[t] * 32);
                    cd[t][0] = q[0];
                    cd[t][1] = q[1];
                }
            }
        }
        // the node's a features are staged into LDS 64 at a time (one parallel
        // load), so the sequential walk reads LDS instead of chained global loads
        for (int x0 = as; x0 < ae; x0 += 64) {
        {
            const int x = x0 + lane;
            int idx = -1;
            if (x < ae) {
                idx = A.fv_feats[x];
                if (A.mp[idx] >= 0) idx = -1;  // already has a MapPoint (:1466-1468)
            }
            st_idx[w][lane] = idx;
            if (idx >= 0) {
                const uint4* q = (const uint4*)(A.desc + (size_t)idx * 32);
                st_desc[w][lane][0] = q[0];
                st_desc[w][lane][1] = q[1];
                const gf_keypoint k = A.kps[idx];
                st_kp[w][lane] = make_float3(k.x, k.y, k.angle);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        const int xn = min(64, ae - x0);
        for (int xi = 0; xi < xn; xi++) {
            const int idxA = st_idx[w][xi];
            if (idxA < 0) continue;
            const uint4 a0 = st_desc[w][xi][0], a1 = st_desc[w][xi][1];
            const float3 kp1 = st_kp[w][xi];
            // epipolar line l = x1' F12 (:708-710)
            const float la = kp1.x * F[0] + kp1.y * F[3] + F[6];
            const float lb = kp1.x * F[1] + kp1.y * F[4] + F[7];
            const float lc = kp1.x * F[2] + kp1.y * F[5] + F[8];
            int bestB;
            if (regs) {
                int d[TRI_CT];
#pragma unroll
                for (int t = 0; t < TRI_CT; t++)
                    d[t] = __popc(a0.x ^ cd[t][0].x) + __popc(a0.y ^ cd[t][0].y) + __popc(a0.z ^ cd[t][0].z) +
                           __popc(a0.w ^ cd[t][0].w) + __popc(a1.x ^ cd[t][1].x) + __popc(a1.y ^ cd[t][1].y) +
                           __popc(a1.z ^ cd[t][1].z) + __popc(a1.w ^ cd[t][1].w);
                bestB = tri_pick(d, cidx, cok, TRI_CT, la, lb, lc, B.kps, P);
                if (bestB < 0) continue;
#pragma unroll
                for (int t = 0; t < TRI_CT; t++)
                    if (cidx[t] == bestB) cok[t] = false;
            } else {  // large node: stream the candidates from memory, claims in LDS
                int best = INT_MAX;
                for (int y = bs + lane; y < be; y += 64) {
                    const int idxB = B.fv_feats[y];
                    if (claimed[idxB] || B.mp[idxB] >= 0) continue;
                    const int dd = hamming_r(a0, a1, B.desc + (size_t)idxB * 32);
                    if (dd <= 50) best = min(best, dd);
                }
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) best = min(best, __shfl_xor(best, o, 64));
                if (best == INT_MAX) continue;
                const int dth = min(2 * best, 50);
                unsigned key = 0xffffffffu;
                for (int y = bs + lane; y < be; y += 64) {
                    const int idxB = B.fv_feats[y];
                    if (claimed[idxB] || B.mp[idxB] >= 0) continue;
                    const int dd = hamming_r(a0, a1, B.desc + (size_t)idxB * 32);
                    if (dd > dth) continue;
                    const unsigned k = ((unsigned)dd << 16) | (unsigned)idxB;
                    if (k < key && epipolar_ok(la, lb, lc, B.kps[idxB], P)) key = k;
                }
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) key = min(key, (unsigned)__shfl_xor((int)key, o, 64));
                if (key == 0xffffffffu) continue;
                bestB = (int)(key & 0xffffu);
                if (lane == 0) claimed[bestB] = 1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (lane == 0) {
                P.out[idxA] = bestB;
                const int r = atomicAdd(&s_nm, 1);
                rec[r] = idxA;
                float rot = kp1.z - B.kps[bestB].angle;  // kp1.angle - kp2.angle
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)roundf(rot * factor);
                if (bin == HISTO_LENGTH) bin = 0;
                rbin[r] = (uint8_t)bin;
            }
        }
        }
    }
    __syncthreads();
    const int nm = s_nm;
    if (check_ori) rotation_filter(nm, rbin, rec, P.out, s_hist, s_keep, &s_nm);
    if (tid == 0) nmatches[blockIdx.x] = s_nm;
}

VocabDev vdev(const gf_vocab* v) {
    return VocabDev{v->d_desc, v->d_cstart, v->d_child, v->d_word, v->d_weight, v->L, v->scoring, v->weighting};
}

}  // namespace

static int bow_transform_impl(gf_vocab* v, int nframes, const uint8_t* d_desc, const int32_t* d_n,
                              const int32_t* d_gate, int cap, int levelsup, int32_t* d_words, double* d_values,
                              int32_t* d_nwords, int32_t* d_fv_nodes, int32_t* d_fv_start, int32_t* d_fv_feats,
                              int32_t* d_nfv, void* tmp, void* stream);

extern "C" {

int gf_vocab_destroy(gf_vocab* v) {
    if (!v) return GF_OK;
    if (v->ctx) (void)hipSetDevice(v->ctx->device);
    void* ps[] = {v->d_desc, v->d_cstart, v->d_child, v->d_word, v->d_weight, v->d_in, v->d_stage};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete v;
    return GF_OK;
}

int gf_vocab_create(gf_ctx* ctx, const gf_vocab_arrays* T, gf_vocab** out) {
    GF_CHECK(ctx && T && out, GF_ERR_ARG, "null arg");
    GF_CHECK(T->nnodes >= 1 && T->parent && T->desc && T->weight && T->is_leaf, GF_ERR_ARG, "empty tree");
    GF_CHECK(T->scoring >= 0 && T->scoring <= 5 && T->weighting >= 0 && T->weighting <= 3, GF_ERR_ARG,
             "bad scoring / weighting");
    const int n = T->nnodes;
    // children in record order (CSR), word ids in record order of the leaves
    std::vector<int32_t> cnt(n + 1, 0), cstart(n + 1, 0), child(std::max(n - 1, 1)), word(n, 0);  // Node::word_id defaults to 0
    int nw = 0;
    for (int i = 1; i < n; i++) {
        GF_CHECK(T->parent[i] >= 0 && T->parent[i] < i, GF_ERR_ARG, "parent must precede its child");
        cnt[T->parent[i]]++;
        if (T->is_leaf[i]) word[i] = nw++;
    }
    for (int i = 0; i < n; i++) cstart[i + 1] = cstart[i] + cnt[i];
    std::vector<int32_t> cur(cstart.begin(), cstart.end() - 1);
    for (int i = 1; i < n; i++) child[cur[T->parent[i]]++] = i;
    GF_HIP(hipSetDevice(ctx->device));
    gf_vocab* v = new gf_vocab();
    v->ctx = ctx;
    v->k = T->k;
    v->L = T->L;
    v->scoring = T->scoring;
    v->weighting = T->weighting;
    v->nnodes = n;
    v->nwords = nw;
    hipError_t e;
    if ((e = hipMalloc((void**)&v->d_desc, 32 * (size_t)n)) || (e = hipMalloc((void**)&v->d_cstart, 4 * (size_t)(n + 1))) ||
        (e = hipMalloc((void**)&v->d_child, 4 * child.size())) || (e = hipMalloc((void**)&v->d_word, 4 * (size_t)n)) ||
        (e = hipMalloc((void**)&v->d_weight, 8 * (size_t)n)) ||
        (e = hipMemcpy(v->d_desc, T->desc, 32 * (size_t)n, hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(v->d_cstart, cstart.data(), 4 * (size_t)(n + 1), hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(v->d_child, child.data(), 4 * child.size(), hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(v->d_word, word.data(), 4 * (size_t)n, hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(v->d_weight, T->weight, 8 * (size_t)n, hipMemcpyHostToDevice))) {
        gf_vocab_destroy(v);
        return gf::fail(GF_ERR_HIP, hipGetErrorString(e));
    }
    *out = v;
    return GF_OK;
}

int gf_vocab_load(gf_ctx* ctx, const char* path, gf_vocab** out) {
    GF_CHECK(ctx && path && out, GF_ERR_ARG, "null arg");
    gf_vocab_arrays T{};
    int rc = gf_vocab_read(path, &T);
    if (rc) return gf::fail(rc, std::string("cannot read vocabulary ") + path);
    std::vector<int32_t> parent(T.nnodes);
    std::vector<uint8_t> desc(32 * (size_t)T.nnodes), leaf(T.nnodes);
    std::vector<double> weight(T.nnodes);
    T.parent = parent.data();
    T.desc = desc.data();
    T.weight = weight.data();
    T.is_leaf = leaf.data();
    rc = gf_vocab_read(path, &T);
    if (rc) return gf::fail(rc, std::string("cannot read vocabulary ") + path);
    return gf_vocab_create(ctx, &T, out);
}

int gf_vocab_info(gf_vocab* v, int* k, int* L, int* nnodes, int* nwords) {
    GF_CHECK(v, GF_ERR_ARG, "null vocab");
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (nnodes) *nnodes = v->nnodes;
    if (nwords) *nwords = v->nwords;
    return GF_OK;
}

int gf_bow_transform_dev(gf_vocab* v, int nframes, const uint8_t* d_desc, const int32_t* d_n, int cap, int levelsup,
                         int32_t* d_words, double* d_values, int32_t* d_nwords, int32_t* d_fv_nodes,
                         int32_t* d_fv_start, int32_t* d_fv_feats, int32_t* d_nfv, void* stream) {
    GF_CHECK(v, GF_ERR_ARG, "null vocab");
    if (nframes <= 0) return GF_OK;
    void* tmp;
    int rc = gf::ws_get(v->ctx, 48, (size_t)nframes * std::max(cap, 1) * 16, &tmp);
    if (rc) return rc;
    return bow_transform_impl(v, nframes, d_desc, d_n, nullptr, cap, levelsup, d_words, d_values, d_nwords, d_fv_nodes,
                              d_fv_start, d_fv_feats, d_nfv, tmp, stream);
}

}  // extern "C"

// Scratch of nframes x cap x 16 bytes: the caller's (a front end's own
// buffer: the context's slot 48 is also the batched PnP's work buffer).
static int bow_transform_impl(gf_vocab* v, int nframes, const uint8_t* d_desc, const int32_t* d_n,
                              const int32_t* d_gate, int cap, int levelsup, int32_t* d_words, double* d_values,
                              int32_t* d_nwords, int32_t* d_fv_nodes, int32_t* d_fv_start, int32_t* d_fv_feats,
                              int32_t* d_nfv, void* tmp, void* stream) {
    GF_CHECK(d_desc && d_n && d_words && d_values && d_nwords && d_fv_nodes && d_fv_start && d_fv_feats && d_nfv,
             GF_ERR_ARG, "null arg");
    GF_CHECK(cap > 0 && cap <= BOW_MAX, GF_ERR_UNSUPPORTED, "cap must be in 1..4096");
    GF_CHECK(v->nnodes > 1, GF_ERR_ARG, "empty vocabulary");
    hipStream_t s = (hipStream_t)stream;
    int32_t* wid = (int32_t*)tmp;
    int32_t* nid = wid + (size_t)nframes * cap;
    double* wv = (double*)(nid + (size_t)nframes * cap);
    const VocabDev V = vdev(v);
    static bool lds_attr = false;  // k_bow_build may take up to 96 KB of dynamic LDS (cap 4096)
    if (!lds_attr) {
        GF_HIP(hipFuncSetAttribute((const void*)k_bow_build, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)bow_build_lds(BOW_MAX)));
        lds_attr = true;
    }
    {
        GF_PROF(v->ctx, s, "k_bow_descend");
        GF_LAUNCH(k_bow_descend, dim3((cap + 255) / 256, nframes), 256, 0, s, V, d_desc, d_n, cap, levelsup, wid, wv, nid,
                  d_gate);
        GF_HIP(hipGetLastError());
    }
    {
        GF_PROF(v->ctx, s, "k_bow_build");
        GF_LAUNCH(k_bow_build, std::min(nframes, d_gate ? 32 : nframes), 256, bow_build_lds(cap), s, V, nframes, d_n, cap,
                  wid, wv, nid,
                  d_words, d_values, d_nwords, d_fv_nodes, d_fv_start, d_fv_feats, d_nfv, d_gate);
        GF_HIP(hipGetLastError());
    }
    return GF_OK;
}

int gf::bow_transform_gated(gf_vocab* voc, int nframes, const uint8_t* d_desc, const int32_t* d_n,
                            const int32_t* d_gate, int cap, int levelsup, int32_t* d_words, double* d_values,
                            int32_t* d_nwords, int32_t* d_fv_nodes, int32_t* d_fv_start, int32_t* d_fv_feats,
                            int32_t* d_nfv, void* tmp, void* stream) {
    GF_CHECK(voc, GF_ERR_ARG, "null vocab");
    if (nframes <= 0) return GF_OK;
    return bow_transform_impl(voc, nframes, d_desc, d_n, d_gate, cap, levelsup, d_words, d_values, d_nwords,
                              d_fv_nodes, d_fv_start, d_fv_feats, d_nfv, tmp, stream);
}

int gf::match_bow_pairs(gf_ctx* ctx, int mode, float nnratio, int check_ori, int npairs, const gf::BowPairDev* d_pairs,
                        int32_t* d_nmatches, int bcap, void* stream) {
    if (npairs <= 0) return GF_OK;
    GF_CHECK(bcap > 0 && bcap <= BOW_MAX, GF_ERR_UNSUPPORTED, "b side: at most 4096 features");
    hipStream_t s = (hipStream_t)stream;
    GF_PROF(ctx, s, "k_match_bow");
    GF_LAUNCH(k_match_bow, std::min(npairs, 256), 256, match_bow_lds(bcap), s, d_pairs, npairs, mode, nnratio,
              check_ori, d_nmatches, bcap);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

extern "C" {

int gf_bow_transform(gf_vocab* v, const uint8_t* desc, int n, int levelsup, int32_t* words, double* values,
                     int* nwords, int32_t* fv_nodes, int32_t* fv_start, int32_t* fv_feats, int* nfv) {
    GF_CHECK(v && nwords && nfv && (n == 0 || (desc && words && values && fv_nodes && fv_feats)) && fv_start,
             GF_ERR_ARG, "null arg");
    GF_CHECK(n >= 0 && n <= BOW_MAX, GF_ERR_UNSUPPORTED, "at most 4096 descriptors");
    if (n == 0 || v->nnodes <= 1) {  // transform() of an empty vocabulary / no features: empty vectors
        *nwords = 0;
        *nfv = 0;
        fv_start[0] = 0;
        return GF_OK;
    }
    gf_ctx* ctx = v->ctx;
    GF_HIP(hipSetDevice(ctx->device));
    const int cap = n;
    void *dd, *dn, *dout;
    const int32_t nn = n;
    int rc;
    const size_t out_bytes = (size_t)cap * (4 + 8 + 4 + 4 + 4) + 4 + 4 * 3;
    if ((rc = gf::ws_upload(ctx, 49, desc, 32 * (size_t)n, &dd)) || (rc = gf::ws_upload(ctx, 50, &nn, 4, &dn)) ||
        (rc = gf::ws_get(ctx, 51, out_bytes, &dout)))
        return rc;
    double* dv = (double*)dout;
    int32_t* dw = (int32_t*)(dv + cap);
    int32_t* dnode = dw + cap;
    int32_t* dfeat = dnode + cap;
    int32_t* dstart = dfeat + cap;  // cap + 1
    int32_t* dcounts = dstart + cap + 1;
    rc = gf_bow_transform_dev(v, 1, (const uint8_t*)dd, (const int32_t*)dn, cap, levelsup, dw, dv, dcounts, dnode,
                              dstart, dfeat, dcounts + 1, ctx->stream);
    if (rc) return rc;
    int32_t counts[2];
    GF_HIP(hipMemcpyAsync(counts, dcounts, 8, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    *nwords = counts[0];
    *nfv = counts[1];
    GF_HIP(hipMemcpyAsync(words, dw, 4 * (size_t)counts[0], hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(values, dv, 8 * (size_t)counts[0], hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(fv_nodes, dnode, 4 * (size_t)counts[1], hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(fv_start, dstart, 4 * (size_t)(counts[1] + 1), hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(fv_feats, dfeat, 4 * (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    return GF_OK;
}

int gf_match_bow_dev(gf_ctx* ctx, int mode, float nnratio, int check_ori, int npairs, const gf_bow_side* a,
                     const gf_bow_side* b, int32_t* const* outs, int32_t* d_nmatches, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (npairs <= 0) return GF_OK;
    GF_CHECK(a && b && outs && d_nmatches, GF_ERR_ARG, "null arg");
    GF_CHECK(mode == 0 || mode == 1, GF_ERR_ARG, "mode must be 0 (KeyFrame, Frame) or 1 (KeyFrame, KeyFrame)");
    std::vector<BowPair> P(npairs);
    for (int p = 0; p < npairs; p++) {
        GF_CHECK(a[p].n >= 0 && a[p].n <= BOW_MAX && b[p].n >= 0 && b[p].n <= BOW_MAX && a[p].nfv <= a[p].n &&
                     b[p].nfv <= b[p].n,
                 GF_ERR_UNSUPPORTED, "at most 4096 features per side");
        P[p].a = a[p];
        P[p].b = b[p];
        P[p].out = outs[p];
    }
    hipStream_t s = (hipStream_t)stream;
    void* dp;
    int rc = gf::ws_get(ctx, 52, sizeof(BowPair) * npairs, &dp);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(dp, P.data(), sizeof(BowPair) * npairs, hipMemcpyHostToDevice, s));
    int bcap = 1;
    for (int p = 0; p < npairs; p++) bcap = std::max(bcap, b[p].n);
    GF_PROF(ctx, s, "k_match_bow");
    GF_LAUNCH(k_match_bow, std::min(npairs, 256), 256, match_bow_lds(bcap), s, (const BowPair*)dp, npairs, mode,
              nnratio, check_ori, d_nmatches, bcap);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

// Copies both sides of a host pair into one scratch block (slot 53); sd
// receives the device views, dout / dnm the output vector and count.
static int stage_bow_pair(gf_ctx* ctx, const gf_bow_side* a, const gf_bow_side* b, int nout, gf_bow_side sd[2],
                          int32_t** dout, int32_t** dnm) {
    sd[0] = *a;
    sd[1] = *b;
    size_t off = 0;
    std::vector<std::pair<const void*, size_t>> parts;
    auto add = [&](const void* h, size_t bytes) {
        const size_t o = off;
        parts.push_back({h, bytes});
        off += (bytes + 15) & ~(size_t)15;
        return o;
    };
    size_t o_an = add(a->fv_nodes, 4 * (size_t)a->nfv), o_as = add(a->fv_start, 4 * (size_t)(a->nfv + 1)),
           o_af = add(a->fv_feats, 4 * (size_t)a->n), o_ad = add(a->desc, 32 * (size_t)a->n),
           o_ak = add(a->kps, sizeof(gf_keypoint) * (size_t)a->n), o_am = add(a->mp, 4 * (size_t)a->n);
    size_t o_bn = add(b->fv_nodes, 4 * (size_t)b->nfv), o_bs = add(b->fv_start, 4 * (size_t)(b->nfv + 1)),
           o_bf = add(b->fv_feats, 4 * (size_t)b->n), o_bd = add(b->desc, 32 * (size_t)b->n),
           o_bk = add(b->kps, sizeof(gf_keypoint) * (size_t)b->n), o_bm = add(b->mp, 4 * (size_t)b->n);
    const size_t o_out = add(nullptr, 4 * (size_t)std::max(nout, 1)), o_nm = add(nullptr, 4);
    void* dbuf;
    int rc = gf::ws_get(ctx, 53, off, &dbuf);
    if (rc) return rc;
    uint8_t* base = (uint8_t*)dbuf;
    size_t cur = 0;
    for (auto& pr : parts) {
        if (pr.first && pr.second) GF_HIP(hipMemcpyAsync(base + cur, pr.first, pr.second, hipMemcpyHostToDevice, ctx->stream));
        cur += (pr.second + 15) & ~(size_t)15;
    }
    sd[0].fv_nodes = (const int32_t*)(base + o_an);
    sd[0].fv_start = (const int32_t*)(base + o_as);
    sd[0].fv_feats = (const int32_t*)(base + o_af);
    sd[0].desc = base + o_ad;
    sd[0].kps = (const gf_keypoint*)(base + o_ak);
    sd[0].mp = (const int32_t*)(base + o_am);
    sd[1].fv_nodes = (const int32_t*)(base + o_bn);
    sd[1].fv_start = (const int32_t*)(base + o_bs);
    sd[1].fv_feats = (const int32_t*)(base + o_bf);
    sd[1].desc = base + o_bd;
    sd[1].kps = (const gf_keypoint*)(base + o_bk);
    sd[1].mp = (const int32_t*)(base + o_bm);
    *dout = (int32_t*)(base + o_out);
    *dnm = (int32_t*)(base + o_nm);
    return GF_OK;
}

static int fetch_bow_result(gf_ctx* ctx, int nout, const int32_t* dout, const int32_t* dnm, int32_t* out,
                            int* nmatches) {
    int32_t nm = 0;
    if (nout) GF_HIP(hipMemcpyAsync(out, dout, 4 * (size_t)nout, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipMemcpyAsync(&nm, dnm, 4, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    *nmatches = nm;
    return GF_OK;
}

int gf_match_bow(gf_ctx* ctx, int mode, float nnratio, int check_ori, const gf_bow_side* a, const gf_bow_side* b,
                 int32_t* out, int* nmatches) {
    GF_CHECK(ctx && a && b && out && nmatches, GF_ERR_ARG, "null arg");
    GF_CHECK(a->n <= BOW_MAX && b->n <= BOW_MAX, GF_ERR_UNSUPPORTED, "at most 4096 features per side");
    GF_HIP(hipSetDevice(ctx->device));
    const int nout = mode == 0 ? b->n : a->n;
    gf_bow_side sd[2];
    int32_t *dout, *dnm;
    int rc = stage_bow_pair(ctx, a, b, nout, sd, &dout, &dnm);
    if (rc) return rc;
    rc = gf_match_bow_dev(ctx, mode, nnratio, check_ori, 1, &sd[0], &sd[1], &dout, dnm, ctx->stream);
    if (rc) return rc;
    return fetch_bow_result(ctx, nout, dout, dnm, out, nmatches);
}

int gf_search_for_triangulation_dev(gf_ctx* ctx, int check_ori, int npairs, const gf_bow_side* a,
                                    const gf_bow_side* b, const float* F12, const float* sigma2_b, int nlevels,
                                    int32_t* const* outs, int32_t* d_nmatches, void* stream) {
    GF_CHECK(ctx, GF_ERR_ARG, "null ctx");
    if (npairs <= 0) return GF_OK;
    GF_CHECK(a && b && F12 && sigma2_b && outs && d_nmatches, GF_ERR_ARG, "null arg");
    GF_CHECK(nlevels >= 1 && nlevels <= 16, GF_ERR_ARG, "nlevels must be in 1..16");
    std::vector<TriPair> T(npairs);
    for (int p = 0; p < npairs; p++) {
        GF_CHECK(a[p].n >= 0 && b[p].n >= 0 && a[p].n <= BOW_MAX && b[p].n <= BOW_MAX && a[p].nfv <= a[p].n &&
                     b[p].nfv <= b[p].n,
                 GF_ERR_UNSUPPORTED, "at most 4096 features per side");
        T[p] = TriPair{};
        T[p].a = a[p];
        T[p].b = b[p];
        for (int i = 0; i < 9; i++) T[p].F[i] = F12[9 * p + i];
        for (int i = 0; i < nlevels; i++) T[p].sigma2[i] = sigma2_b[i];
        T[p].nlevels = nlevels;
        T[p].out = outs[p];
    }
    hipStream_t s = (hipStream_t)stream;
    void* dp;
    int rc = gf::ws_get(ctx, 60, sizeof(TriPair) * npairs, &dp);
    if (rc) return rc;
    GF_HIP(hipMemcpyAsync(dp, T.data(), sizeof(TriPair) * npairs, hipMemcpyHostToDevice, s));
    GF_PROF(ctx, s, "k_search_tri");
    GF_LAUNCH(k_search_tri, npairs, TRI_THREADS, 0, s, (const TriPair*)dp, check_ori, d_nmatches);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

int gf_search_for_triangulation(gf_ctx* ctx, int check_ori, const gf_bow_side* a, const gf_bow_side* b,
                                const float* F12, const float* sigma2_b, int nlevels, int32_t* out, int* nmatches) {
    GF_CHECK(ctx && a && b && F12 && sigma2_b && nmatches && (a->n == 0 || out), GF_ERR_ARG, "null arg");
    GF_CHECK(a->n >= 0 && b->n >= 0 && a->n <= BOW_MAX && b->n <= BOW_MAX, GF_ERR_UNSUPPORTED,
             "at most 4096 features per side");
    GF_HIP(hipSetDevice(ctx->device));
    gf_bow_side sd[2];
    int32_t *dout, *dnm;
    int rc = stage_bow_pair(ctx, a, b, a->n, sd, &dout, &dnm);
    if (rc) return rc;
    rc = gf_search_for_triangulation_dev(ctx, check_ori, 1, &sd[0], &sd[1], F12, sigma2_b, nlevels, &dout, dnm,
                                         ctx->stream);
    if (rc) return rc;
    return fetch_bow_result(ctx, a->n, dout, dnm, out, nmatches);
}

}  // extern "C"

// Vocabulary broadcast: rank `root` holds *voc; every other
// rank receives the tree into a vocabulary of its own on the communicator's
// device (*voc created here; pass *voc == NULL). Device to device: the
// header first, then the node arrays in place.
extern "C" int gf_dist_bcast_vocab(gf_dist* d, gf_vocab** voc, int root) {
    GF_CHECK(d && voc, GF_ERR_ARG, "null arg");
    gf_ctx* ctx = gf::dist_ctx(d);
    const bool is_root = gf::dist_rank(d) == root;
    GF_CHECK(!is_root || *voc, GF_ERR_ARG, "root has no vocabulary");
    GF_HIP(hipSetDevice(ctx->device));
    int32_t hdr[8] = {0};
    if (is_root) {
        gf_vocab* v = *voc;
        int32_t h[8] = {v->k, v->L, v->scoring, v->weighting, v->nnodes, v->nwords, 0, 0};
        memcpy(hdr, h, sizeof(h));
    }
    int32_t* dh = nullptr;
    GF_HIP(hipMalloc(&dh, sizeof(hdr)));
    hipError_t e = hipMemcpy(dh, hdr, sizeof(hdr), hipMemcpyHostToDevice);
    int rc = e == hipSuccess ? gf::dist_bcast(d, dh, sizeof(hdr), root) : GF_ERR_HIP;
    if (!rc) e = hipMemcpyAsync(hdr, dh, sizeof(hdr), hipMemcpyDeviceToHost, ctx->stream);
    if (!rc && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(dh);
    if (rc) return rc;
    GF_HIP(e);
    const int n = hdr[4];
    GF_CHECK(n >= 1, GF_ERR_ARG, "empty vocabulary");
    gf_vocab* v = *voc;
    if (!is_root) {
        v = new gf_vocab();
        v->ctx = ctx;
        v->k = hdr[0];
        v->L = hdr[1];
        v->scoring = hdr[2];
        v->weighting = hdr[3];
        v->nnodes = n;
        v->nwords = hdr[5];
        if ((e = hipMalloc((void**)&v->d_desc, 32 * (size_t)n)) ||
            (e = hipMalloc((void**)&v->d_cstart, 4 * (size_t)(n + 1))) ||
            (e = hipMalloc((void**)&v->d_child, 4 * (size_t)std::max(n - 1, 1))) ||
            (e = hipMalloc((void**)&v->d_word, 4 * (size_t)n)) || (e = hipMalloc((void**)&v->d_weight, 8 * (size_t)n))) {
            gf_vocab_destroy(v);
            return gf::fail(GF_ERR_HIP, hipGetErrorString(e));
        }
    }
    if ((rc = gf::dist_bcast(d, v->d_desc, 32 * (size_t)n, root)) ||
        (rc = gf::dist_bcast(d, v->d_cstart, 4 * (size_t)(n + 1), root)) ||
        (rc = gf::dist_bcast(d, v->d_child, 4 * (size_t)std::max(n - 1, 1), root)) ||
        (rc = gf::dist_bcast(d, v->d_word, 4 * (size_t)n, root)) ||
        (rc = gf::dist_bcast(d, v->d_weight, 8 * (size_t)n, root))) {
        if (!is_root) gf_vocab_destroy(v);
        return rc;
    }
    GF_HIP(hipStreamSynchronize(ctx->stream));
    *voc = v;
    return GF_OK;
}

// Host copy of a device vocabulary's node arrays (for checksums across ranks):
// desc (nnodes x 32), weight (nnodes), word (nnodes), cstart (nnodes + 1).
extern "C" int gf_vocab_download(gf_vocab* v, uint8_t* desc, double* weight, int32_t* word, int32_t* cstart) {
    GF_CHECK(v, GF_ERR_ARG, "null vocabulary");
    GF_HIP(hipSetDevice(v->ctx->device));
    const size_t n = v->nnodes;
    if (desc) GF_HIP(hipMemcpy(desc, v->d_desc, 32 * n, hipMemcpyDeviceToHost));
    if (weight) GF_HIP(hipMemcpy(weight, v->d_weight, 8 * n, hipMemcpyDeviceToHost));
    if (word) GF_HIP(hipMemcpy(word, v->d_word, 4 * n, hipMemcpyDeviceToHost));
    if (cstart) GF_HIP(hipMemcpy(cstart, v->d_cstart, 4 * (n + 1), hipMemcpyDeviceToHost));
    return GF_OK;
}
