// Local-map assembly: Tracking::UpdateReference
// (src/Tracking.cc:3689-3852) for a batch of frames tracking one map.
//
// One 1024-thread workgroup per frame:
//   1. votes: every non-bad map point of the frame adds one to each observing
//      keyframe's LDS counter (integer atomics: order-free); bad ones are set
//      to -1 in the frame (:3778-3793);
//   2. the voted, non-bad keyframes in index order (= ascending KeyFrame*, the
//      std::map order) by a workgroup scan; pKFmax = the first with the
//      largest count, by a (count, -index) max-reduction (:3798-3817);
//   3. neighbours: one wave replays the sequential loop — while the list holds
//      <= 80, keyframe p of the original list adds the first of its best 10
//      covisible keyframes that is neither bad nor listed; the 10 candidates
//      are tested on 10 lanes and the first by a ballot (:3820-3848);
//   4. map points: the local keyframes' slots form one sequence (keyframe
//      order, then slot order); each point's first position comes from an
//      atomicMin over the sequence, then the points at their first position
//      are compacted in sequence order by workgroup scans (:3737-3763).
// Scratch: the first-position array (one int per map point per frame, global
// memory) is reset by the same kernel for exactly the points it touched.
#include <algorithm>
#include <climits>

#include "common.h"

namespace {

#ifndef RM_THREADS
#define RM_THREADS 1024
#endif
constexpr int RM_T = RM_THREADS;
constexpr int RM_MAXKF = 8192;

struct RefArgs {
    gf_covis_map m;
    const gf_covis_map* maps;  // per-frame maps (device array), else m for every frame
    int first_stride;          // map points per frame in `first`
    int32_t* frame_mps;
    const int32_t* nkps;
    int stride;
    int32_t* local_kfs;
    int32_t* n_local_kfs;
    int kf_cap;
    int32_t* local_mps;
    int32_t* n_local_mps;
    int mp_cap;
    int32_t* ref_kf;
    int32_t* first;  // [nframes][nmp] scratch
    int kfc;         // keyframe capacity of the launch's maps (sizes the LDS)
};

// LDS of k_update_reference for maps of at most kfc keyframes: votes / slot
// offsets [kfc + 1], local keyframes [kfc], marks [kfc]. (Sized per launch:
// the front end's graphs hold at most 64 keyframes, and a fixed 8192-keyframe
// footprint, 74 KB, kept the other stream groups' workgroups off the CU.)
// voted keyframes whose first 10 covisible neighbours are staged in LDS for
// the neighbour replay (more voted keyframes: the replay reads them from HBM)
constexpr int RM_NBMAX = 256;
size_t rm_lds_bytes(int kfc) {
    const size_t a = ((size_t)(kfc + 1) * 4 + 15) & ~(size_t)15, b = ((size_t)kfc * 4 + 15) & ~(size_t)15;
    // + the local keyframes' first map-point slots, + the staged neighbours
    return a + b + (((size_t)kfc + 15) & ~(size_t)15) + b + 40 * (size_t)std::min(kfc, RM_NBMAX);
}

// map-point slots per thread kept in registers across the three slot passes
constexpr int RM_SC = 8;

// exclusive scan over the workgroup (16 waves); total returned in `total`
__device__ int scan_1024(int v, int* tmp, int& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < RM_T / 64; i++) {
        const int t = tmp[i];
        base += i < wid ? t : 0;
        tot += t;
    }
    total = tot;
    __syncthreads();
    return base + x - v;
}

#ifndef RM_OB
#define RM_OB 4  // a point's observations loaded together in the votes
#endif
__global__ __launch_bounds__(RM_T) void k_update_reference(RefArgs A) {
    gfd::track_prio();
    extern __shared__ __align__(16) uint8_t rm_lds[];
    int* cnt = reinterpret_cast<int*>(rm_lds);  // votes, then the slot offsets of the local keyframes
    int* lkf = reinterpret_cast<int*>(rm_lds + (((size_t)(A.kfc + 1) * 4 + 15) & ~(size_t)15));  // local keyframes
    uint8_t* mark = reinterpret_cast<uint8_t*>(lkf) + (((size_t)A.kfc * 4 + 15) & ~(size_t)15);
    int* kb = reinterpret_cast<int*>(mark + (((size_t)A.kfc + 15) & ~(size_t)15));  // kf_mp_off of local keyframe p
    int* snb = kb + ((A.kfc + 3) & ~3);  // [min(kfc, RM_NBMAX)][10]: neighbour index, -1 none, -2 bad
    __shared__ int tmp[RM_T / 64];
    __shared__ unsigned long long s_best;
    __shared__ int s_nl;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const gf_covis_map M = A.maps ? A.maps[f] : A.m;
    const int nkf = M.nkf;
    int32_t* fm = A.frame_mps + (size_t)f * A.stride;
    const int nkp = min(max(A.nkps[f], 0), A.stride);
    for (int k = tid; k < nkf; k += RM_T) {
        cnt[k] = 0;
        mark[k] = 0;
    }
    if (tid == 0) s_best = 0ull;
    __syncthreads();
    // 1. votes
    // the point's flag and observation range loaded together (clamped,
    // unconditional), its observations RM_OB at a time
    for (int i = tid; i < nkp; i += RM_T) {
        const int m = fm[i];
        if (M.nmp <= 0) continue;  // no points: no matches either
        const int mc = min(max(m, 0), M.nmp - 1);
        const bool bad = M.mp_bad[mc] != 0;
        const int o0 = M.mp_obs_off[mc], o1 = M.mp_obs_off[mc + 1];
        if (m < 0) continue;
        if (bad) {
            fm[i] = -1;
            continue;
        }
        for (int o = o0; o < o1; o += RM_OB) {
            int kq[RM_OB];
#pragma unroll
            for (int u = 0; u < RM_OB; u++) kq[u] = M.mp_obs[min(o + u, o1 - 1)];
#pragma unroll
            for (int u = 0; u < RM_OB; u++)
                if (o + u < o1) atomicAdd(&cnt[kq[u]], 1);
        }
    }
    __syncthreads();
    // 2. voted, non-bad keyframes in index order; pKFmax
    int nl = 0;
    for (int k0 = 0; k0 < nkf; k0 += RM_T) {
        const int k = k0 + tid;
        const int c = k < nkf ? cnt[k] : 0;
        const bool in = k < nkf && c > 0 && !M.kf_bad[k];
        int tot;
        const int pos = nl + scan_1024(in ? 1 : 0, tmp, tot);
        if (in) {
            lkf[pos] = k;
            mark[k] = 1;
            // larger count first, then smaller index: (count << 32) | ~index
            atomicMax(&s_best, ((unsigned long long)(unsigned)c << 32) | (unsigned)(0x7fffffff - k));
        }
        nl += tot;
    }
    __syncthreads();
    const int nk0 = nl;
    // 3. neighbours (sequential replay on wave 0). The voted keyframes' first
    // 10 covisible neighbours and their bad flags are loaded by every thread
    // at once into LDS first, so the replay's steps wait on LDS, not on three
    // dependent HBM loads each
    const bool staged = nk0 <= min(A.kfc, RM_NBMAX);
    if (staged) {
        for (int e = tid; e < 10 * nk0; e += RM_T) {
            const int p = e / 10, j = e - 10 * p, kf = lkf[p];
            const int o0 = M.kf_cov_off[kf], deg = min(10, M.kf_cov_off[kf + 1] - o0);
            int nb = -1;
            if (j < deg) {
                nb = M.kf_cov[o0 + j];
                if (M.kf_bad[nb]) nb = -2;
            }
            snb[e] = nb;
        }
        __syncthreads();
    }
    if (tid < 64) {
        int n = nk0;
        for (int p = 0; p < nk0; p++) {
            if (n > 80) break;
            int nb = -1;
            bool ok = false;
            if (staged) {
                if (lane < 10) {
                    nb = snb[10 * p + lane];
                    ok = nb >= 0 && !mark[nb];
                }
            } else {
                const int kf = lkf[p];
                const int o0 = M.kf_cov_off[kf], deg = min(10, M.kf_cov_off[kf + 1] - o0);
                if (lane < deg) {
                    nb = M.kf_cov[o0 + lane];
                    ok = !M.kf_bad[nb] && !mark[nb];
                }
            }
            const unsigned long long b = __ballot(ok);
            if (b) {
                const int first = __ffsll((long long)b) - 1;
                const int pick = __shfl(nb, first, 64);
                if (lane == 0) {
                    lkf[n] = pick;
                    mark[pick] = 1;
                }
                n++;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        if (lane == 0) s_nl = n;
    }
    __syncthreads();
    nl = s_nl;
    // outputs: keyframes, reference keyframe
    int32_t* okf = A.local_kfs + (size_t)f * A.kf_cap;
    for (int p = tid; p < nl && p < A.kf_cap; p += RM_T) okf[p] = lkf[p];
    if (tid == 0) {
        A.n_local_kfs[f] = nl;
        A.ref_kf[f] = s_best ? 0x7fffffff - (int)(unsigned)(s_best & 0xffffffffu) : -1;
    }
    // 4. map points: slot offsets of the local keyframes (cnt reused), their
    // first kf_mp index in kb
    int total = 0;
    for (int p0 = 0; p0 < nl; p0 += RM_T) {
        const int p = p0 + tid;
        int len = 0;
        if (p < nl) {
            const int o0 = M.kf_mp_off[lkf[p]];
            len = M.kf_mp_off[lkf[p] + 1] - o0;
            kb[p] = o0;
        }
        int tot;
        const int off = total + scan_1024(len, tmp, tot);
        if (p < nl) cnt[p] = off;
        total += tot;
    }
    if (tid == 0) cnt[nl] = total;
    __syncthreads();
    int32_t* first = A.first + (size_t)f * A.first_stride;
    auto slot_idx = [&](int q) -> int {  // kf_mp index of sequence position q
        int lo = 0, hi = nl - 1;          // last p with cnt[p] <= q
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cnt[mid] <= q)
                lo = mid;
            else
                hi = mid - 1;
        }
        return kb[lo] + (q - cnt[lo]);
    };
    auto slot_mp = [&](int q) -> int { return M.kf_mp[slot_idx(q)]; };
    // the thread's slots q = tid + RM_T k: map point and bad flag loaded once,
    // all in flight together (the passes below were each a chain of
    // dependent loads per slot); past RM_SC slots per thread, looked up per pass
    const int nch = (total + RM_T - 1) / RM_T;
    int mq[RM_SC];
    bool bq[RM_SC];
    if (total > 0) {  // loads at clamped indices, unconditional (a load behind a branch waits before the next)
        int ix[RM_SC];
#pragma unroll
        for (int k = 0; k < RM_SC; k++) ix[k] = slot_idx(min(tid + RM_T * k, total - 1));
#pragma unroll
        for (int k = 0; k < RM_SC; k++) mq[k] = M.kf_mp[ix[k]];
#pragma unroll
        for (int k = 0; k < RM_SC; k++) bq[k] = M.nmp > 0 ? M.mp_bad[min(max(mq[k], 0), M.nmp - 1)] != 0 : true;
#pragma unroll
        for (int k = 0; k < RM_SC; k++)
            if (tid + RM_T * k >= total) mq[k] = -1;
    } else {
#pragma unroll
        for (int k = 0; k < RM_SC; k++) {
            mq[k] = -1;
            bq[k] = true;
        }
    }
    auto slot = [&](int k, int q, int& m, bool& bad) {
        if (k < RM_SC) {
#pragma unroll
            for (int u = 0; u < RM_SC; u++)
                if (u == k) {
                    m = mq[u];
                    bad = bq[u];
                }
        } else {
            m = q < total ? slot_mp(q) : -1;
            bad = m < 0 || M.mp_bad[m];
        }
    };
    for (int k = 0; k < nch; k++) {
        int m;
        bool bad;
        slot(k, tid + RM_T * k, m, bad);
        if (m >= 0) first[m] = INT_MAX;
    }
    __syncthreads();
    for (int k = 0; k < nch; k++) {
        const int q = tid + RM_T * k;
        int m;
        bool bad;
        slot(k, q, m, bad);
        if (m >= 0 && !bad) atomicMin(&first[m], q);
    }
    __syncthreads();
    int32_t* omp = A.local_mps + (size_t)f * A.mp_cap;
    int nm = 0;
    for (int k = 0; k < nch; k++) {
        const int q = tid + RM_T * k;
        int m;
        bool bad;
        slot(k, q, m, bad);
        // (an L2-coherent read: the atomics above executed there)
        const bool keep = m >= 0 && !bad && __hip_atomic_load(&first[m], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == q;
        int tot;
        const int pos = nm + scan_1024(keep ? 1 : 0, tmp, tot);
        if (keep && pos < A.mp_cap) omp[pos] = m;
        nm += tot;
    }
    if (tid == 0) A.n_local_mps[f] = nm;
}

// dynamic LDS above 64 KB (maps of more than ~5400 keyframes) needs the attribute
int rm_lds_attr(gf_ctx* ctx) {
    static unsigned long long mask = 0;
    if (!(mask & (1ull << ctx->device))) {
        GF_HIP(hipFuncSetAttribute((const void*)k_update_reference, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)rm_lds_bytes(RM_MAXKF)));
        mask |= 1ull << ctx->device;
    }
    return GF_OK;
}

}  // namespace

extern "C" {

int gf_update_reference_dev(gf_ctx* ctx, const gf_covis_map* d_map, int nframes, int32_t* d_frame_mps,
                            const int32_t* d_nkps, int stride, int32_t* d_local_kfs, int32_t* d_n_local_kfs,
                            int kf_cap, int32_t* d_local_mps, int32_t* d_n_local_mps, int mp_cap, int32_t* d_ref_kf,
                            void* stream) {
    GF_CHECK(ctx && d_map, GF_ERR_ARG, "null arg");
    if (nframes <= 0) return GF_OK;
    const gf_covis_map& m = *d_map;
    GF_CHECK(m.nkf >= 0 && m.nkf <= RM_MAXKF, GF_ERR_UNSUPPORTED, "more than 8192 keyframes");
    GF_CHECK(m.nmp >= 0, GF_ERR_ARG, "negative map size");
    GF_CHECK(d_frame_mps && d_nkps && d_local_kfs && d_n_local_kfs && d_local_mps && d_n_local_mps && d_ref_kf,
             GF_ERR_ARG, "null output");
    GF_CHECK(stride > 0 && kf_cap >= 0 && mp_cap >= 0, GF_ERR_ARG, "bad stride or caps");
    GF_CHECK(m.nkf == 0 || (m.kf_bad && m.kf_mp_off && m.kf_cov_off), GF_ERR_ARG, "null keyframe arrays");
    GF_CHECK(m.nmp == 0 || (m.mp_bad && m.mp_obs_off), GF_ERR_ARG, "null map point arrays");
    void* first = nullptr;
    int rc = gf::ws_get(ctx, 61, (size_t)nframes * std::max(m.nmp, 1) * sizeof(int32_t), &first);
    if (rc) return rc;
    RefArgs A{};
    A.m = m;
    A.frame_mps = d_frame_mps;
    A.nkps = d_nkps;
    A.stride = stride;
    A.local_kfs = d_local_kfs;
    A.n_local_kfs = d_n_local_kfs;
    A.kf_cap = kf_cap;
    A.local_mps = d_local_mps;
    A.n_local_mps = d_n_local_mps;
    A.mp_cap = mp_cap;
    A.ref_kf = d_ref_kf;
    A.first = (int32_t*)first;
    A.first_stride = m.nmp;
    A.kfc = std::max(m.nkf, 1);
    hipStream_t s = (hipStream_t)stream;
    if ((rc = rm_lds_attr(ctx))) return rc;
    GF_PROF(ctx, s, "k_update_reference");
    GF_LAUNCH(k_update_reference, nframes, RM_T, rm_lds_bytes(A.kfc), s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}

}  // extern "C"

namespace gf {
// UpdateReference for B frames each against its own map: d_maps is a device
// array of B gf_covis_map whose arrays are device pointers, every map with at
// most nmp_cap points and kf_max keyframes (the front end's per-stream
// keyframe graphs); d_first is scratch of B * nmp_cap ints.
int update_reference_frames(gf_ctx* ctx, const gf_covis_map* d_maps, int nmp_cap, int nframes, int32_t* d_frame_mps,
                            const int32_t* d_nkps, int stride, int32_t* d_local_kfs, int32_t* d_n_local_kfs,
                            int kf_cap, int32_t* d_local_mps, int32_t* d_n_local_mps, int mp_cap, int32_t* d_ref_kf,
                            int32_t* d_first, int kf_max, hipStream_t s) {
    if (nframes <= 0) return GF_OK;
    GF_CHECK(kf_max >= 0 && kf_max <= RM_MAXKF, GF_ERR_UNSUPPORTED, "more than 8192 keyframes");
    if (int rc = rm_lds_attr(ctx)) return rc;
    RefArgs A{};
    A.kfc = std::max(kf_max, 1);
    A.maps = d_maps;
    A.first_stride = nmp_cap;
    A.frame_mps = d_frame_mps;
    A.nkps = d_nkps;
    A.stride = stride;
    A.local_kfs = d_local_kfs;
    A.n_local_kfs = d_n_local_kfs;
    A.kf_cap = kf_cap;
    A.local_mps = d_local_mps;
    A.n_local_mps = d_n_local_mps;
    A.mp_cap = mp_cap;
    A.ref_kf = d_ref_kf;
    A.first = d_first;
    GF_PROF(ctx, s, "k_update_reference");
    GF_LAUNCH(k_update_reference, nframes, RM_T, rm_lds_bytes(A.kfc), s, A);
    GF_HIP(hipGetLastError());
    return GF_OK;
}
}  // namespace gf

extern "C" {

int gf_update_reference(gf_ctx* ctx, const gf_covis_map* map, int32_t* frame_mps, int nkp, int32_t* local_kfs,
                        int* n_local_kfs, int kf_cap, int32_t* local_mps, int* n_local_mps, int mp_cap,
                        int32_t* ref_kf) {
    GF_CHECK(ctx && map && n_local_kfs && n_local_mps && ref_kf, GF_ERR_ARG, "null arg");
    GF_CHECK(nkp >= 0 && (nkp == 0 || frame_mps), GF_ERR_ARG, "bad frame");
    GF_CHECK(kf_cap >= 0 && mp_cap >= 0 && (kf_cap == 0 || local_kfs) && (mp_cap == 0 || local_mps), GF_ERR_ARG,
             "bad outputs");
    const gf_covis_map& h = *map;
    GF_CHECK(h.nkf >= 0 && h.nkf <= RM_MAXKF && h.nmp >= 0, GF_ERR_UNSUPPORTED, "map size out of range");
    GF_HIP(hipSetDevice(ctx->device));
    const int nkf = h.nkf, nmp = h.nmp;
    const size_t nkm = nkf ? (size_t)h.kf_mp_off[nkf] : 0, nkc = nkf ? (size_t)h.kf_cov_off[nkf] : 0;
    const size_t nob = nmp ? (size_t)h.mp_obs_off[nmp] : 0;
    gf_covis_map d{};
    d.nkf = nkf;
    d.nmp = nmp;
    void* p;
    int rc;
    auto up = [&](int slot, const void* src, size_t bytes) -> void* {
        if (rc) return nullptr;
        rc = gf::ws_upload(ctx, slot, src, std::max<size_t>(bytes, 4), &p);
        return rc ? nullptr : p;
    };
    rc = 0;
    static const int32_t zero = 0;
    d.kf_bad = (const uint8_t*)up(16, nkf ? (const void*)h.kf_bad : &zero, nkf);
    d.kf_mp_off = (const int32_t*)up(17, nkf ? (const void*)h.kf_mp_off : &zero, 4 * ((size_t)nkf + 1));
    d.kf_mp = (const int32_t*)up(18, nkm ? (const void*)h.kf_mp : &zero, 4 * nkm);
    d.kf_cov_off = (const int32_t*)up(19, nkf ? (const void*)h.kf_cov_off : &zero, 4 * ((size_t)nkf + 1));
    d.kf_cov = (const int32_t*)up(20, nkc ? (const void*)h.kf_cov : &zero, 4 * nkc);
    d.mp_bad = (const uint8_t*)up(21, nmp ? (const void*)h.mp_bad : &zero, nmp);
    d.mp_obs_off = (const int32_t*)up(22, nmp ? (const void*)h.mp_obs_off : &zero, 4 * ((size_t)nmp + 1));
    d.mp_obs = (const int32_t*)up(23, nob ? (const void*)h.mp_obs : &zero, 4 * nob);
    const int32_t nk = nkp;
    void* dfm = up(24, nkp ? (const void*)frame_mps : &zero, 4 * (size_t)std::max(nkp, 1));
    void* dnk = up(25, &nk, 4);
    if (rc) return rc;
    void *dkf, *dnkf, *dmp, *dnmp, *dref;
    if ((rc = gf::ws_get(ctx, 26, 4 * (size_t)std::max(kf_cap, 1), &dkf)) ||
        (rc = gf::ws_get(ctx, 27, 4 * (size_t)std::max(mp_cap, 1), &dmp)) || (rc = gf::ws_get(ctx, 28, 16, &dnkf)))
        return rc;
    dnmp = (int32_t*)dnkf + 1;
    dref = (int32_t*)dnkf + 2;
    rc = gf_update_reference_dev(ctx, &d, 1, (int32_t*)dfm, (const int32_t*)dnk, std::max(nkp, 1), (int32_t*)dkf,
                                 (int32_t*)dnkf, kf_cap, (int32_t*)dmp, (int32_t*)dnmp, mp_cap, (int32_t*)dref,
                                 ctx->stream);
    if (rc) return rc;
    int32_t cnts[3];
    GF_HIP(hipMemcpyAsync(cnts, dnkf, 12, hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    *n_local_kfs = cnts[0];
    *n_local_mps = cnts[1];
    *ref_kf = cnts[2];
    if (nkp) GF_HIP(hipMemcpyAsync(frame_mps, dfm, 4 * (size_t)nkp, hipMemcpyDeviceToHost, ctx->stream));
    if (kf_cap && cnts[0]) GF_HIP(hipMemcpyAsync(local_kfs, dkf, 4 * (size_t)std::min(cnts[0], kf_cap),
                                                 hipMemcpyDeviceToHost, ctx->stream));
    if (mp_cap && cnts[1]) GF_HIP(hipMemcpyAsync(local_mps, dmp, 4 * (size_t)std::min(cnts[1], mp_cap),
                                                 hipMemcpyDeviceToHost, ctx->stream));
    GF_HIP(hipStreamSynchronize(ctx->stream));
    GF_CHECK(cnts[0] <= kf_cap && cnts[1] <= mp_cap, GF_ERR_CAP, "local map larger than the output capacity");
    return GF_OK;
}

}  // extern "C"
